"""Data-parallel semantics on CPU: world_size-2 gloo (the GPU path runs the
same code over RCCL).  Each rank renders its own object with the oracle's
image step; the model gradient bucket is summed by one async all-reduce and
the touched code-table rows are all-gathered (codenerf_amd.dp.GradExchange);
every rank applies AdamW.  Checked: replicas identical
after the step, and equal to one process that accumulates both objects'
gradients before the same AdamW step (1 GPU with 1 object
per step is the reference; N ranks sum N objects' gradients)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_cpu
from oracle.params import make_params, make_codes

N_OBJ, H, NS = 4, 6, 12


def _setup(seed=3):
    p = ref_cpu.param_tensors(make_params(seed))
    st, tt = (torch.tensor(a, requires_grad=True) for a in make_codes(seed, N_OBJ))
    g = torch.Generator().manual_seed(seed)
    ro = torch.zeros(H * H, 3) + torch.tensor([0.1, 0.3, 1.3])
    vd = torch.nn.functional.normalize(torch.randn(H * H, 3, generator=g) * 0.2 + torch.tensor([0., -.2, -1.]),
                                       dim=-1)
    z = torch.linspace(0.8, 1.8, NS)
    gts = [torch.rand(H * H, 3, generator=g) for _ in range(N_OBJ)]
    return p, st, tt, ro, vd, z, gts


def _opt(p, st, tt):
    return ref_cpu.AdamWRef([(list(p.values()), 1e-4), ([st], 1e-3), ([tt], 1e-3)])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from codenerf_amd.dp import GradExchange, object_for
    torch.set_num_threads(1)
    p, st, tt, ro, vd, z, gts = _setup()
    ex = GradExchange(list(p.values()), [st, tt], dist)
    opt = _opt(p, st, tt)
    for step in range(2):
        ex.zero()
        obj = object_for(step, rank, world, N_OBJ)
        ref_cpu.image_step(p, st, tt, obj, ro, vd, z, gts[obj], chunk=16)
        ex.exchange_rows([obj])          # all_gather of the touched code rows
        work = ex.start_model()          # async model all-reduce
        ex.finish(work)
        opt.step()
    flat = torch.cat([t.detach().reshape(-1) for t in list(p.values()) + [st, tt]])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        out.put([g.numpy() for g in gathered])
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(300)
def test_two_rank_step_matches_summed_single_process():
    from codenerf_amd.dp import GradExchange, object_for
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    np.testing.assert_array_equal(res[0], res[1])          # replicas bit-identical
    # single process: both ranks' objects accumulated, then the same AdamW step
    p, st, tt, ro, vd, z, gts = _setup()
    ex = GradExchange(list(p.values()), [st, tt])
    opt = _opt(p, st, tt)
    for step in range(2):
        ex.zero()
        for rank in range(world):
            obj = object_for(step, rank, world, N_OBJ)
            ref_cpu.image_step(p, st, tt, obj, ro, vd, z, gts[obj], chunk=16)
        opt.step()
    flat = torch.cat([t.detach().reshape(-1) for t in list(p.values()) + [st, tt]]).numpy()
    np.testing.assert_allclose(res[0], flat, rtol=1e-6, atol=1e-8)


def test_object_assignment_covers_distinct_objects():
    from codenerf_amd.dp import object_for
    for world in (1, 2, 4, 8):
        for step in range(5):
            objs = [object_for(step, r, world, 64) for r in range(world)]
            assert len(set(objs)) == world


# ---------------------------------------------------------------- evaluation / inference sharding
def _eval_worker(rank, world, port, out):
    """Evaluation views split across ranks (src/optimizer.py:108-130) and one
    image rendered as contiguous ray blocks (C5 inference), with the oracle's
    renderer standing in for the HIP one."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from codenerf_amd import dp
    torch.set_num_threads(1)
    p, st, tt, ro, vd, z, gts = _setup()
    views = [0, 2, 3, 5, 6]

    def view_metric(v):
        with torch.no_grad():
            xyz = ro[:, None, :] + vd[:, None, :] * (z + 0.01 * v)[:, None]
            sig, rgb = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, NS, -1), st[v % N_OBJ][None],
                                                tt[v % N_OBJ][None])
            col, _ = ref_cpu.volume_rendering(sig, rgb, z)
        return float(((col - gts[v % N_OBJ]) ** 2).mean())

    local = {v: view_metric(v) for v in dp.shard(views, dist)}
    merged = dp.gather_by_key(local, dist)
    R = ro.shape[0]
    a, b = dp.ray_block(R, dist, align=4)
    with torch.no_grad():
        xyz = ro[a:b, None, :] + vd[a:b, None, :] * z[:, None]
        sig, rgb = ref_cpu.codenerf_forward(p, xyz, vd[a:b, None, :].expand(-1, NS, -1), st[1][None], tt[1][None])
        col, _ = ref_cpu.volume_rendering(sig, rgb, z)
    img = dp.gather_ray_blocks(col, R, dist, align=4)
    if rank == 0:
        out.put((merged, img.numpy(), sorted(local)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_eval_views_and_ray_blocks_sharded_match_single_process():
    from codenerf_amd import dp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_eval_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    merged, img, mine = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert mine == [0, 3, 6]                       # round-robin share of rank 0
    p, st, tt, ro, vd, z, gts = _setup()
    views = [0, 2, 3, 5, 6]
    ref = {}
    for v in views:
        with torch.no_grad():
            xyz = ro[:, None, :] + vd[:, None, :] * (z + 0.01 * v)[:, None]
            sig, rgb = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, NS, -1), st[v % N_OBJ][None],
                                                tt[v % N_OBJ][None])
            col, _ = ref_cpu.volume_rendering(sig, rgb, z)
        ref[v] = float(((col - gts[v % N_OBJ]) ** 2).mean())
    assert list(merged) == views and merged == ref
    with torch.no_grad():
        xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
        sig, rgb = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, NS, -1), st[1][None], tt[1][None])
        col, _ = ref_cpu.volume_rendering(sig, rgb, z)
    np.testing.assert_allclose(img, col.numpy(), rtol=1e-6, atol=1e-7)


def test_ray_blocks_cover_the_image():
    from codenerf_amd import dp

    class FakeDist:
        def __init__(self, world, rank):
            self.w, self.r = world, rank

        def is_initialized(self):
            return True

        def get_world_size(self, group=None):
            return self.w

        def get_rank(self, group=None):
            return self.r

    for R in (1, 7, 36, 65536):
        for world in (1, 2, 3, 8):
            for align in (1, 4, 2048):
                blocks = [dp.ray_block(R, FakeDist(world, r), align=align) for r in range(world)]
                covered = [i for a, b in blocks for i in range(a, b)]
                assert covered == list(range(R)), (R, world, align)


# ---------------------------------------------------------------- code-row exchange edge cases
def _rows_worker(rank, world, port, out):
    """Duplicated rows on one rank and unequal row counts across ranks: every
    rank's distinct rows are summed once into the dense tables."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from codenerf_amd.dp import GradExchange
    w = torch.zeros(4, 3, requires_grad=True)
    st = torch.zeros(6, 5, requires_grad=True)
    tt = torch.zeros(6, 5, requires_grad=True)
    ex = GradExchange([w], [st, tt], dist)
    rows = [1, 1, 2] if rank == 0 else [3]
    for t in (st, tt):
        t.grad.copy_(torch.arange(30, dtype=torch.float32).reshape(6, 5) * (rank + 1))
    ex.exchange_rows(rows)
    if rank == 0:
        out.put((st.grad.numpy().copy(), tt.grad.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_exchange_rows_dedups_and_pads_unequal_counts():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    sg, tg = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    base = np.arange(30, dtype=np.float32).reshape(6, 5)
    want = np.zeros((6, 5), np.float32)
    want[1] = base[1]            # rank 0's rows 1 (once) and 2
    want[2] = base[2]
    want[3] = 2 * base[3]        # rank 1's row 3 (its grads are 2x)
    np.testing.assert_array_equal(sg, want)
    np.testing.assert_array_equal(tg, want)


def test_zero_after_fused_zero_grad_step_clears_direct_backward_writes():
    """a fused zero-grad AdamW step sets GradExchange.clean so the
    next zero() skips its launch; a backward that writes .grad WITHOUT going
    through TrainCore.step_grads (ImageStep.forward_backward called
    directly) must re-arm it -- ImageStep notifies its grad_listeners."""
    from codenerf_amd.dp import GradExchange
    from codenerf_amd.render import ImageStep
    params = [torch.zeros(4, 3), torch.zeros(5)]
    table = torch.zeros(6, 2)
    ex = GradExchange(params, [table])
    step = ImageStep(model=None)
    step.grad_listeners.append(ex.mark_dirty)
    ex.clean = True                     # as after a zero_grad AdamW step
    step._writing_grads()               # what _coarse_part / _fine_part do before writing
    params[0].grad.fill_(1.0)
    table.grad.fill_(2.0)
    ex.zero()
    assert float(params[0].grad.abs().sum()) == 0.0 and float(table.grad.abs().sum()) == 0.0
    # without a write in between, the clean flag still saves the launch once
    ex.clean = True
    ex.zero()
    assert ex.clean is False
