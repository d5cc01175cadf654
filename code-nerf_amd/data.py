"""SRN-format data: the reference loader (src/data.py) and a synthetic
SRN-format dataset generator (no ShapeNet-SRN data is available offline).

Loader semantics follow src/data.py:10-89:
  * poses: ``pose/*.txt`` (4x4, sorted by file name) right-multiplied by
    diag(1, -1, -1, 1) (SRN/OpenCV -> OpenGL camera axes), float32;
  * images: ``rgb/*.png`` as float32 RGB in [0, 1];
  * intrinsics: focal = first number of the first line of intrinsics.txt,
    H W = the last line;
  * train split: 1 randomly chosen view per object (np.random.choice(50, k)),
    with the optional central crop [32:-32, 32:-32] and H, W halved (focal
    unchanged); test / val split: the first 250 views.
One deliberate fix: the reference decides "train" with
``splits.split('_')[1] == 'train'``, which is False for the chairs split
``chairs_2.0_train`` and then crashes the trainer; here the LAST '_' field of
the split name decides.

Images are read with PIL (imageio, which the reference uses, is not
installed); PNG decoding is lossless either way.
"""
import math
import os

import numpy as np
import torch

SRN_TO_GL = np.diag(np.array([1.0, -1.0, -1.0, 1.0]))


def _sorted_files(d):
    return np.sort([os.path.join(d, f.name) for f in os.scandir(d)])


def load_poses(pose_dir, idxs=()):
    files = np.array(_sorted_files(pose_dir))[np.asarray(idxs, dtype=np.int64)]
    poses = [np.loadtxt(f).reshape(4, 4) @ SRN_TO_GL for f in files]
    return torch.from_numpy(np.array(poses)).float()


def load_imgs(img_dir, idxs=()):
    from PIL import Image
    files = np.array(_sorted_files(img_dir))[np.asarray(idxs, dtype=np.int64)]
    imgs = []
    for f in files:
        with Image.open(f) as im:
            imgs.append(np.asarray(im.convert("RGB"), dtype=np.float32) / 255.0)
    return torch.from_numpy(np.array(imgs))


def load_intrinsic(path):
    with open(path) as f:
        lines = f.readlines()
    focal = float(lines[0].split()[0])
    H, W = lines[-1].split()
    return focal, int(H), int(W)


class SRN:
    """Map-style dataset over the objects of one SRN category split."""

    def __init__(self, cat="srn_cars", splits="cars_train", data_dir="../data/ShapeNet_SRN/",
                 num_instances_per_obj=1, crop_img=True, n_train_views=50, n_test_views=250):
        self.data_dir = os.path.join(data_dir, cat, splits)
        self.ids = np.sort([f.name for f in os.scandir(self.data_dir)])
        self.lenids = len(self.ids)
        self.num_instances_per_obj = num_instances_per_obj
        self.train = os.path.basename(os.path.normpath(splits)).split("_")[-1] == "train"
        self.crop_img = crop_img
        self.n_train_views = n_train_views
        self.n_test_views = n_test_views

    def __len__(self):
        return self.lenids

    def __getitem__(self, idx):
        obj_id = self.ids[idx]
        if self.train:
            focal, H, W, imgs, poses, instances = self.return_train_data(obj_id)
            return focal, H, W, imgs, poses, instances, idx
        focal, H, W, imgs, poses = self.return_test_val_data(obj_id)
        return focal, H, W, imgs, poses, idx

    def _paths(self, obj_id):
        base = os.path.join(self.data_dir, obj_id)
        return os.path.join(base, "pose"), os.path.join(base, "rgb"), os.path.join(base, "intrinsics.txt")

    def return_train_data(self, obj_id):
        pose_dir, img_dir, intr = self._paths(obj_id)
        instances = np.random.choice(self.n_train_views, self.num_instances_per_obj)
        poses = load_poses(pose_dir, instances)
        imgs = load_imgs(img_dir, instances)
        focal, H, W = load_intrinsic(intr)
        if self.crop_img:
            imgs = imgs[:, 32:-32, 32:-32, :]
            H, W = H // 2, W // 2
        return focal, H, W, imgs.reshape(self.num_instances_per_obj, -1, 3), poses, instances

    def return_test_val_data(self, obj_id):
        pose_dir, img_dir, intr = self._paths(obj_id)
        n = min(self.n_test_views, len(os.listdir(img_dir)))
        instances = np.arange(n)
        poses = load_poses(pose_dir, instances)
        imgs = load_imgs(img_dir, instances)
        focal, H, W = load_intrinsic(intr)
        return focal, H, W, imgs, poses


def collate_one(item):
    """What torch's default_collate with batch_size=1 hands the reference loop:
    a leading batch dim, python ints -> int64 tensors, float focal -> float64
    tensor (which is why get_rays computes directions in float64)."""
    out = []
    for v in item:
        if isinstance(v, torch.Tensor):
            out.append(v[None])
        elif isinstance(v, float):
            out.append(torch.tensor([v], dtype=torch.float64))
        elif isinstance(v, (int, np.integer)):
            out.append(torch.tensor([int(v)]))
        elif isinstance(v, np.ndarray):
            out.append(torch.from_numpy(v)[None])
        else:
            out.append(v)
    return out


# ---------------------------------------------------------------- synthetic data
def look_at_srn(radius, az_deg, el_deg):
    """Camera-to-world in the SRN file convention (OpenCV axes: x right,
    y down, z forward), camera on a sphere looking at the origin."""
    az, el = math.radians(az_deg), math.radians(el_deg)
    eye = np.array([radius * math.cos(el) * math.sin(az), radius * math.sin(el),
                    radius * math.cos(el) * math.cos(az)])
    fwd = -eye / np.linalg.norm(eye)
    up = np.array([0.0, 1.0, 0.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    tup = np.cross(right, fwd)
    c2w_gl = np.eye(4)
    c2w_gl[:3, 0], c2w_gl[:3, 1], c2w_gl[:3, 2], c2w_gl[:3, 3] = right, tup, -fwd, eye
    return c2w_gl @ SRN_TO_GL          # diag is its own inverse


def _render_object(spec, c2w_gl, H, W, focal):
    """Ray-cast an object made of axis-aligned ellipsoids (Lambert shading,
    white background) with the reference's camera model (src/utils.py:10-19)."""
    i, j = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64), indexing="xy")
    dirs = np.stack([(i - W * 0.5) / focal, -(j - H * 0.5) / focal, -np.ones_like(i)], -1)
    d = dirs @ c2w_gl[:3, :3].T
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    o = np.broadcast_to(c2w_gl[:3, 3], d.shape)
    best_t = np.full((H, W), np.inf)
    color = np.ones((H, W, 3))
    light = np.array([0.4, 0.8, 0.45])
    light /= np.linalg.norm(light)
    for center, radii, rgb in spec:
        c, r = np.asarray(center), np.asarray(radii)
        oc = (o - c) / r
        dd = d / r
        a = (dd * dd).sum(-1)
        b = 2 * (oc * dd).sum(-1)
        cc = (oc * oc).sum(-1) - 1
        disc = b * b - 4 * a * cc
        hit = disc > 0
        t = np.where(hit, (-b - np.sqrt(np.maximum(disc, 0))) / (2 * a), np.inf)
        t = np.where(t > 1e-4, t, np.inf)
        closer = t < best_t
        if not closer.any():
            continue
        p = o + d * np.where(closer, t, 0.0)[..., None]
        n = (p - c) / (r * r)
        n /= np.linalg.norm(n, axis=-1, keepdims=True) + 1e-12
        shade = 0.35 + 0.65 * np.clip((n * light).sum(-1), 0, 1)
        col = np.asarray(rgb)[None, None, :] * shade[..., None]
        color = np.where(closer[..., None], col, color)
        best_t = np.where(closer, t, best_t)
    return np.clip(color, 0, 1)


def _object_spec(rng):
    """A car-like compound of 2-4 ellipsoids inside the unit sphere."""
    body = rng.uniform(0.2, 0.9, 3)
    spec = [((0, rng.uniform(-0.1, 0.05), 0), (rng.uniform(0.35, 0.5), rng.uniform(0.12, 0.2),
                                              rng.uniform(0.2, 0.3)), body)]
    spec.append(((rng.uniform(-0.1, 0.1), rng.uniform(0.08, 0.18), 0),
                 (rng.uniform(0.15, 0.3), rng.uniform(0.08, 0.14), rng.uniform(0.15, 0.22)),
                 np.clip(body * rng.uniform(0.5, 1.2), 0, 1)))
    for _ in range(int(rng.integers(0, 3))):
        spec.append(((rng.uniform(-0.35, 0.35), rng.uniform(-0.2, -0.1), rng.choice([-0.22, 0.22])),
                     (0.08, 0.08, 0.04), (0.1, 0.1, 0.1)))
    return spec


def make_synthetic_srn(root, cat="srn_cars", splits="cars_train", n_obj=4, n_views=50, H=128, W=128,
                       focal=131.25, radius=1.3, seed=0):
    """Write an SRN-format split under ``root/cat/splits``: per object
    ``rgb/%06d.png``, ``pose/%06d.txt`` (SRN convention) and
    ``intrinsics.txt``; views on the radius-``radius`` sphere."""
    from PIL import Image
    rng = np.random.Generator(np.random.PCG64(seed))
    base = os.path.join(root, cat, splits)
    for k in range(n_obj):
        obj = os.path.join(base, f"synth{seed:03d}_{k:05d}")
        os.makedirs(os.path.join(obj, "rgb"), exist_ok=True)
        os.makedirs(os.path.join(obj, "pose"), exist_ok=True)
        spec = _object_spec(rng)
        with open(os.path.join(obj, "intrinsics.txt"), "w") as f:
            f.write(f"{focal} {W / 2} {H / 2} 0.\n0. 0. 0.\n1.\n{H} {W}\n")
        for v in range(n_views):
            az, el = rng.uniform(-180, 180), rng.uniform(-5, 50)
            c2w_srn = look_at_srn(radius, az, el)
            img = _render_object(spec, c2w_srn @ SRN_TO_GL, H, W, focal)
            Image.fromarray((img * 255 + 0.5).astype(np.uint8)).save(os.path.join(obj, "rgb", f"{v:06d}.png"))
            np.savetxt(os.path.join(obj, "pose", f"{v:06d}.txt"), c2w_srn.reshape(1, 16))
    return base
