"""Diagnostics (GPU): per-tensor gradient error of the fused step vs the CPU
oracle, and xyz / PE input comparisons.  Not a test; prints a table."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
from golden_util import TRAIN_CASES, load, case_params, oracle_image_step  # noqa: E402


def oracle64(g):
    """The oracle replayed in float64 (ground truth for error budgets)."""
    from oracle import ref_cpu
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in case_params(g).items()}
    st = torch.tensor(g["shape_table"], dtype=torch.float64, requires_grad=True)
    tt = torch.tensor(g["texture_table"], dtype=torch.float64, requires_grad=True)
    f = lambda k: torch.tensor(g[k], dtype=torch.float64)
    losses, rgb = ref_cpu.image_step(p, st, tt, int(g["obj_idx"]), f("rays_o"), f("viewdir"), f("z_vals"),
                                     f("gt"), chunk=int(g["chunk"]))
    return dict(params=p, losses=losses, rgb=rgb)


def main():
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.render import ImageStep
    from codenerf_amd import engine as E
    dev = torch.device("cuda", 0)
    for case in TRAIN_CASES:
        g = load(case)
        for prec in ("fp32", "bf16"):
            m = CodeNeRF(3, 1, precision=prec)
            m.load_state_dict({k: torch.tensor(v) for k, v in case_params(g).items()})
            m = m.to(dev)
            st = torch.nn.Parameter(torch.tensor(g["shape_table"], device=dev))
            tt = torch.nn.Parameter(torch.tensor(g["texture_table"], device=dev))
            step = ImageStep(m, chunk=int(g["chunk"]))
            losses, rgb, _ = step.forward_backward(torch.tensor(g["rays_o"], device=dev),
                                                   torch.tensor(g["viewdir"], device=dev),
                                                   torch.tensor(g["z_vals"], device=dev),
                                                   torch.tensor(g["gt"], device=dev), st, tt, int(g["obj_idx"]))
            torch.cuda.synchronize()
            r = oracle_image_step(g)
            r64 = oracle64(g)
            worst = []
            for (k, p) in m.named_parameters():
                a = p.grad.cpu().double().numpy()
                b = r["params"][k].grad.double().numpy()
                c = r64["params"][k].grad.numpy()
                scale = np.abs(c).max() + 1e-30
                worst.append((np.abs(a - c).max() / scale, k, np.abs(b - c).max() / scale))
            worst.sort(reverse=True)
            rgb_err = np.abs(rgb.cpu().numpy() - r["rgb"].numpy()).max()
            ca = st.grad.cpu().numpy()
            cb = r["shape_table"].grad.numpy()
            print(f"{case:22s} {prec}: rgb {rgb_err:.2e}  loss rel "
                  f"{np.abs(losses.cpu().numpy() / np.array(r['losses']) - 1).max():.2e}  "
                  f"code {np.abs(ca - cb).max() / (np.abs(cb).max() + 1e-30):.2e}  worst grads "
                  + ", ".join(f"{k}: ours {e:.1e} ref {e2:.1e}" for e, k, e2 in worst[:3]))
    # xyz: torch expression vs kernel
    R, N = 4096, 64
    ro = torch.randn(R, 3, device=dev)
    vd = torch.nn.functional.normalize(torch.randn(R, 3, device=dev), dim=-1)
    z = torch.linspace(0.8, 1.8, N, device=dev)
    x_t = ro[:, None, :] + vd[:, None, :] * z[:, None]
    x_k, _ = E.sample_points(ro, vd, z, R, N)
    torch.cuda.synchronize()
    x_c = ro.cpu()[:, None, :] + vd.cpu()[:, None, :] * z.cpu()[:, None]
    print("xyz torch-gpu vs kernel mismatches:", int((x_t != x_k).sum()), "of", x_t.numel())
    print("xyz torch-cpu vs kernel mismatches:", int((x_c != x_k.cpu()).sum()))
    print("xyz torch-cpu vs torch-gpu mismatches:", int((x_c != x_t.cpu()).sum()))


if __name__ == "__main__":
    main()
