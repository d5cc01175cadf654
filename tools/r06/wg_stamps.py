"""Workgroup timeline of the bf16x3 training forward (TRAIN_HI, the bf16x3f
plan's) from the stamps of variants/stamps (tools/r06/patch_stamps.py):
per workgroup entry / first block / last block (s_memtime, shader cycles),
per CU the workgroups in order, and so the share of a CU's time spent in
workgroup prologues and between workgroups -- the edges a persistent chain
would cover.  Timing only: the variant overwrites sigma.

  CODENERF_MEASURE=1 CODENERF_LIB=variants/stamps/libcodenerf_hip.so python tools/r06/wg_stamps.py
"""
import collections
import json
import math
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.trainer_core import TrainCore
    from bench import make_pose
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = CodeNeRF(3, 1, precision="bf16x3f").to(dev)
    sc = torch.nn.Parameter(torch.randn(4, 256, device=dev) / math.sqrt(128))
    tc = torch.nn.Parameter(torch.randn(4, 256, device=dev) / math.sqrt(128))
    core = TrainCore(model, sc, tc, near=0.8, far=1.8, n_coarse=64, n_fine=64)
    H = W = 128
    R = H * W
    gt = torch.rand(R, 3, device=dev)
    pose = make_pose(1.3, 30.0, 20.0).to(dev)
    saved = [p.detach().clone() for p in model.param_list() + [sc, tc]]
    core.train_step(H, W, 131.25, pose, gt, 0)
    torch.cuda.synchronize()
    with torch.no_grad():
        for p, q in zip(model.param_list() + [sc, tc], saved):
            p.copy_(q)
    eng = model.engine()
    params = model.param_list()
    eng.ensure_packed(params)
    buf = core.step_impl._ws[eng.device]
    Mc = R * 64
    blob, _ = eng.latent_fwd(params, sc.detach()[0], tc.detach()[0])
    ro = torch.rand(R, 3, device=dev) * 0.1 + torch.tensor([0.0, 0.4, 1.2], device=dev)
    vd = torch.nn.functional.normalize(torch.randn(R, 3, device=dev), dim=-1)
    z = torch.linspace(0.8, 1.8, 64, device=dev)
    sig = buf["sig"][:eng.pad(Mc)]
    for _ in range(5):                      # warm: clocks settle
        eng.mlp_fwd(blob, Mc, rays_o=ro, rays_d=vd, z=z, n_samples=64, act=buf["act"], act_M=buf["cap"],
                    act_row0=0, sigma=sig, rgb=buf["rgb"][:eng.pad(Mc)])
    torch.cuda.synchronize()
    st = sig.view(torch.int32).view(-1, 128)[:, :9].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    assert (st[:, 5] == 0x57A3).all(), "not the stamps variant"
    t0, t1, t2 = st[:, 0], st[:, 1], st[:, 2]
    base = t0.min()
    t0, t1, t2 = (t0 - base) % 2**32, (t1 - base) % 2**32, (t2 - base) % 2**32
    ta, tb, tc = ((st[:, k] - base) % 2**32 for k in (6, 7, 8))
    phases = {"entry_to_blob_in_lds": float(np.mean(ta - t0)), "prologue_pe_and_stores": float(np.mean(tb - ta)),
              "barrier": float(np.mean(tc - tb)), "to_first_block": float(np.mean(t1 - tc))}
    hw, xcc = st[:, 3], st[:, 4]
    # CU identity: XCC id, and HW_ID's SE (bits 13-15), SH (12), CU (8-11)
    cu = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 20 + ((hw >> 8) & 15)
    per = collections.defaultdict(list)
    for i in range(len(t0)):
        per[int(cu[i])].append((int(t0[i]), int(t1[i]), int(t2[i])))
    span = pro = gap = body = 0
    nwg = []
    for c, v in per.items():
        v.sort()
        nwg.append(len(v))
        span += v[-1][2] - v[0][0]
        for k, (a, b, e) in enumerate(v):
            pro += b - a
            body += e - b
            if k:
                gap += a - v[k - 1][2]
    out = {"workgroups": int(len(t0)), "cus": len(per), "wg_per_cu": [int(min(nwg)), int(max(nwg))],
           "wg_cycles_mean": float(np.mean(t2 - t0)), "prologue_cycles_mean": float(np.mean(t1 - t0)),
           "body_cycles_mean": float(np.mean(t2 - t1)), "prologue_phases_cycles": phases,
           "share_of_cu_span": {"prologue": round(pro / span, 4), "between_workgroups": round(gap / span, 4),
                                "blocks": round(body / span, 4)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
