"""GPU: object-sharded data parallelism on the HIP kernels.

Two ranks share cuda:0 over gloo (the 8-GPU run uses RCCL with the same
code); each runs ``TrainCore.train_step`` on its own object -- the fused HIP
image step, the async model-bucket all-reduce, the all_gather of the touched
code rows, AdamW.  Checked over two steps: the replicas are bit-identical, the
exchanged gradients equal one process that accumulates both objects'
gradients before its step (rtol 1e-5: the sum order differs), and so do the
parameters (AdamW moves an element by ~lr whatever its gradient's size, so
near-zero gradients may step apart: bounded by the step size, 99% close).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, NC, NF, N_OBJ, STEPS = 32, 16, 16, 4, 2


def _scene(rank):
    from oracle.params import look_at_pose
    from codenerf_amd.data import _object_spec, _render_object
    c2w = look_at_pose(1.3, 40.0 * rank - 20, 15.0 + 10 * rank)
    spec = _object_spec(np.random.Generator(np.random.PCG64(60 + rank)))
    img = _render_object(spec, c2w.astype(np.float64), H, H, 32.8)
    return torch.tensor(c2w), torch.tensor(img.reshape(-1, 3), dtype=torch.float32)


def _core(dist=None):
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.trainer_core import TrainCore
    from oracle.params import make_codes, make_params
    dev = torch.device("cuda", 0)
    m = CodeNeRF(3, 1, precision="fp32")
    m.load_state_dict({k: torch.tensor(v) for k, v in make_params(61).items()})
    m = m.to(dev)
    s0, t0 = make_codes(61, N_OBJ)
    st = torch.nn.Parameter(torch.tensor(s0, device=dev))
    tt = torch.nn.Parameter(torch.tensor(t0, device=dev))
    return TrainCore(m, st, tt, near=0.8, far=1.8, n_coarse=NC, n_fine=NF, chunk=256, dist=dist)


def _flat(core):
    return torch.cat([p.detach().reshape(-1) for p in core.model.parameters()] +
                     [core.shape_codes.detach().reshape(-1), core.texture_codes.detach().reshape(-1)]).cpu()


def _grads(core):
    return torch.cat([core.bucket.flat, core.shape_codes.grad.reshape(-1), core.texture_codes.grad.reshape(-1)]).cpu()


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from codenerf_amd.dp import object_for
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    core = _core(dist)
    c2w, gt = _scene(rank)
    grads = []
    for step in range(STEPS):
        torch.manual_seed(100 + 10 * step + rank)
        core.train_step(H, H, 32.8, c2w.cuda(), gt.cuda(), object_for(step, rank, world, N_OBJ))
        torch.cuda.synchronize()
        grads.append(_grads(core).numpy())
    q.put((rank, _flat(core).numpy(), grads))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(300)
def test_two_ranks_on_hip_match_summed_single_process():
    import torch.multiprocessing as mp
    from codenerf_amd import engine as _eng
    from codenerf_amd.dp import object_for
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (f, g)) for r, f, g in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][0], res[1][0])          # replicas bit-identical
    for s in range(STEPS):
        np.testing.assert_array_equal(res[0][1][s], res[1][1][s])
    # one process: both objects' gradients accumulated, then the same step
    core = _core()
    dev = torch.device("cuda", 0)
    scenes = [_scene(r) for r in range(world)]
    for step in range(STEPS):
        core.exchange.zero()
        objs = [object_for(step, r, world, N_OBJ) for r in range(world)]
        for r in range(world):
            torch.manual_seed(100 + 10 * step + r)
            c2w, gt = scenes[r]
            ro, vd = _eng.get_rays_dev(H, H, 32.8, True, c2w.to(dev))
            z = core.stratified_z(dev)
            rnd = torch.rand(H * H, NF, device=dev)
            core.step_impl.forward_backward_fine(ro, vd, z, rnd, gt.to(dev), core.shape_codes, core.texture_codes,
                                                 objs[r])
        core.step_grads(objs)
        torch.cuda.synchronize()
        g = _grads(core).numpy()
        np.testing.assert_allclose(res[0][1][step], g, rtol=1e-5, atol=1e-6 * np.abs(g).max())
    flat = _flat(core).numpy()
    d = np.abs(res[0][0] - flat)
    assert d.max() <= 2 * STEPS * 1e-3 + 1e-6
    assert np.mean(d <= 1e-6 + 1e-4 * np.abs(flat)) > 0.99


# ---------------------------------------------------------------- evaluation / inference sharding
def _hp(root):
    return {"net_hyperparams": {"shape_blocks": 3, "texture_blocks": 1, "W": 256, "num_xyz_freq": 10,
                                "num_dir_freq": 4, "latent_dim": 256},
            "data": {"cat": "srn_cars", "splits": "cars_train", "data_dir": root, "n_train_views": 4,
                     "n_test_views": 7},
            "N_samples": 16, "near": 0.8, "far": 1.8, "loss_reg_coef": 1e-4,
            "lr_schedule": [{"type": "step", "lr": 1e-4, "interval": 3}, {"type": "step", "lr": 1e-3, "interval": 3}],
            "check_points": 1000, "N_importance": 0, "precision": "fp32"}


def _optimize(root, exps, dist=None):
    from codenerf_amd.optimizer import Optimizer
    opt = Optimizer("t", 0, [0], "test", hpams=_hp(root), batch_size=512, num_opts=2, exp_root=exps, dist=dist)
    torch.manual_seed(7)
    np.random.seed(7)
    opt.optimize_objs([0], lr=1e-2, lr_half_interval=2, save_img=False)
    return opt.psnr_eval, opt.ssim_eval


def _shard_worker(rank, world, port, root, exps, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    from codenerf_amd import engine as _eng
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.render import ImageStep
    from oracle.params import make_codes, make_params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    psnr, ssim = _optimize(root, exps, dist)
    # one 64x64 image rendered as two ray blocks
    m = CodeNeRF(3, 1, precision="fp32")
    m.load_state_dict({k: torch.tensor(v) for k, v in make_params(71).items()})
    m = m.cuda()
    c2w, _ = _scene(0)
    ro, vd = _eng.get_rays_dev(64, 64, 65.6, True, c2w.cuda())
    s, t = (torch.tensor(c[0], device="cuda") for c in make_codes(71, 1))
    z = torch.linspace(0.8, 1.8, 32, device="cuda")
    rgb, depth = ImageStep(m).render_sharded(ro, vd, z, s, t, dist)
    q.put((rank, psnr, ssim, rgb.cpu().numpy(), depth.cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_shard_eval_views_and_ray_blocks(tmp_path):
    """Optimizer evaluation views split across two ranks (src/optimizer.py:108-130)
    give the single-process metrics; an image rendered as two ray blocks and
    all-gathered equals the one-rank render bit for bit."""
    import torch.multiprocessing as mp
    from codenerf_amd import engine as _eng
    from codenerf_amd.data import make_synthetic_srn
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.render import ImageStep
    from codenerf_amd.trainer import Trainer
    from oracle.params import make_codes, make_params
    root, exps = str(tmp_path / "data"), str(tmp_path / "exps")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=2, n_views=4, H=32, W=32, focal=32.8, seed=3)
    make_synthetic_srn(root, "srn_cars", "cars_test", n_obj=1, n_views=7, H=32, W=32, focal=32.8, seed=4)
    Trainer("t", 0, hpams=_hp(root), batch_size=512, check_iter=0, exp_root=exps).training(0, 2, 1)
    psnr1, ssim1 = _optimize(root, exps)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, root, exps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(psnr1[0]) == 6                          # 7 views minus the target
    for r in range(world):
        assert res[r][0] == psnr1 and res[r][1] == ssim1
    m = CodeNeRF(3, 1, precision="fp32")
    m.load_state_dict({k: torch.tensor(v) for k, v in make_params(71).items()})
    m = m.cuda()
    c2w, _ = _scene(0)
    ro, vd = _eng.get_rays_dev(64, 64, 65.6, True, c2w.cuda())
    s, t = (torch.tensor(c[0], device="cuda") for c in make_codes(71, 1))
    rgb, depth = ImageStep(m).render(ro, vd, torch.linspace(0.8, 1.8, 32, device="cuda"), s, t)
    for r in range(world):
        np.testing.assert_array_equal(res[r][2], rgb.cpu().numpy())
        np.testing.assert_array_equal(res[r][3], depth.cpu().numpy())
