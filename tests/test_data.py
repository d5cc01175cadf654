"""SRN loader (codenerf_amd.data) against the reference's own parsing
(golden: tools/gen_golden_data.py ran src/data.py's load_poses /
load_intrinsic on the same synthetic split) and the src/data.py semantics."""
import os

import numpy as np
import torch

from golden_util import load


def _split(tmp_path, spec):
    from codenerf_amd.data import make_synthetic_srn
    return make_synthetic_srn(str(tmp_path), "srn_cars", "cars_train", n_obj=int(spec[0]), n_views=int(spec[1]),
                              H=int(spec[2]), W=int(spec[3]), focal=float(spec[4]), radius=float(spec[5]),
                              seed=int(spec[6]))


def test_loader_matches_reference_parsing(tmp_path):
    from codenerf_amd.data import load_poses, load_intrinsic
    g = load("srn_loader")
    base = _split(tmp_path, g["spec"])
    for k, oid in enumerate(sorted(os.listdir(base))):
        poses = load_poses(os.path.join(base, oid, "pose"), [2, 0, 1])
        np.testing.assert_array_equal(poses.numpy(), g[f"poses_{k}"])
        focal, H, W = load_intrinsic(os.path.join(base, oid, "intrinsics.txt"))
        np.testing.assert_array_equal(np.array([focal, H, W], dtype=np.float64), g[f"intr_{k}"])


def test_srn_dataset_train_and_test_items(tmp_path):
    from codenerf_amd.data import SRN, collate_one, make_synthetic_srn
    make_synthetic_srn(str(tmp_path), "srn_cars", "cars_train", n_obj=2, n_views=4, H=128, W=128, seed=3)
    ds = SRN("srn_cars", "cars_train", str(tmp_path), num_instances_per_obj=2, crop_img=True, n_train_views=4)
    assert len(ds) == 2 and ds.train
    np.random.seed(0)
    focal, H, W, imgs, poses, inst, idx = ds[1]
    assert (H, W) == (64, 64) and focal == 131.25 and idx == 1
    assert imgs.shape == (2, 64 * 64, 3) and imgs.dtype == torch.float32
    assert float(imgs.min()) >= 0 and float(imgs.max()) <= 1
    assert poses.shape == (2, 4, 4)
    # camera centre on the radius-1.3 sphere, OpenGL axes: -z looks at the origin
    c = poses[0, :3, 3]
    assert abs(float(c.norm()) - 1.3) < 1e-5
    fwd = -poses[0, :3, 2]
    assert float(torch.dot(fwd, -c / c.norm())) > 0.9999
    b = collate_one(ds[0])
    assert b[0].dtype == torch.float64 and b[3].shape[0] == 1
    # test split: all views, no crop
    make_synthetic_srn(str(tmp_path), "srn_cars", "cars_test", n_obj=1, n_views=3, H=32, W=32, seed=4)
    dt = SRN("srn_cars", "cars_test", str(tmp_path), crop_img=False)
    assert not dt.train
    focal, H, W, imgs, poses, idx = dt[0]
    assert imgs.shape == (3, 32, 32, 3) and poses.shape == (3, 4, 4)


def test_chairs_split_name_is_train(tmp_path):
    # reference: 'chairs_2.0_train'.split('_')[1] == '2.0' -> test mode (crash); fixed here
    from codenerf_amd.data import SRN, make_synthetic_srn
    make_synthetic_srn(str(tmp_path), "srn_chairs", "chairs_train/chairs_2.0_train", n_obj=1, n_views=2, H=32,
                       W=32, radius=2.0, seed=5)
    ds = SRN("srn_chairs", "chairs_train/chairs_2.0_train", str(tmp_path), crop_img=False, n_train_views=2)
    assert ds.train


def test_synthetic_views_render_the_object():
    # every synthetic view shows the object (non-white pixels) and white background
    from codenerf_amd.data import _object_spec, _render_object, look_at_srn, SRN_TO_GL
    rng = np.random.Generator(np.random.PCG64(9))
    spec = _object_spec(rng)
    for az in (0.0, 90.0, 200.0):
        img = _render_object(spec, look_at_srn(1.3, az, 20.0) @ SRN_TO_GL, 64, 64, 65.6)
        obj = (img < 0.99).any(-1)
        assert 0.05 < obj.mean() < 0.9
        assert np.allclose(img[0, 0], 1.0)
