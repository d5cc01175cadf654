"""CPU: the kernel-arithmetic emulation of the oracle (oracle/ref_cpu.py
``bf16_operands``) -- test infrastructure for tests/test_gpu_x3_trace.py and
the bf16x3 trajectory tests.

* ``fold`` (_FoldBlock: encoding_shape / sigma / encoding_viewdir through the
  encoding_shape fold, as the dW pass forms their gradients) with every
  operand in fp32 reproduces the plain fp32 oracle's gradients; with the
  kernels' per-layer exception (X3_LAYER_OPS) the dir-PE columns of
  encoding_viewdir's weight come from the bf16-rounded dir PE;
* ``x3`` (three products, lo*lo dropped) stays within 2^-14 of the exact
  split product;
* OPS_BF16X3_K (the kernels' arithmetic op for op) is as close to float64 as
  the round-4 emulation OPS_BF16X3_DB on every tensor (within 2x)."""
import numpy as np
import torch

from golden_util import load
from oracle import ref_cpu
from oracle.params import make_params


def _grads(g, dtype=torch.float32, **kw):
    p = {k: torch.tensor(v, dtype=dtype).requires_grad_() for k, v in make_params(int(g["seed"])).items()}
    st = torch.tensor(g["shape_table"], dtype=dtype).requires_grad_()
    tt = torch.tensor(g["texture_table"], dtype=dtype).requires_grad_()
    f = lambda k: torch.tensor(g[k], dtype=dtype)
    args = (p, st, tt, int(g["obj_idx"]), f("rays_o"), f("viewdir"), f("z_vals"), f("gt"))
    if kw:
        with ref_cpu.bf16_operands(**kw):
            ref_cpu.image_step(*args, chunk=int(g["chunk"]))
    else:
        ref_cpu.image_step(*args, chunk=int(g["chunk"]))
    out = {k: v.grad.double() for k, v in p.items()}
    out["shape_code"], out["texture_code"] = st.grad.double(), tt.grad.double()
    return out


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-300))


F = "f"
FP32_OPS = dict(fw_w=F, fw_x=F, bw_w=F, bw_dy=F, dw_x=F, dw_dy=F)


def test_fold_in_fp32_reproduces_the_oracle():
    g = load("c1_32x32_n32")
    plain = _grads(g, ops=FP32_OPS)                      # the emulation's own matmul path, no fold
    fold = _grads(g, ops=dict(FP32_OPS, fold=True))
    for k, ref in plain.items():
        assert _rel(fold[k], ref) < 1e-5, (k, _rel(fold[k], ref))
    # with the kernels' per-layer exception the dir-PE columns of
    # encoding_viewdir's weight gradient come from the bf16-rounded PE
    hi = _grads(g, ops=dict(FP32_OPS, fold=True), layer_ops=ref_cpu.X3_LAYER_OPS)
    k = "encoding_viewdir.0.weight"
    assert _rel(hi[k][:, :256], plain[k][:, :256]) < 1e-5
    assert 1e-5 < _rel(hi[k][:, 256:], plain[k][:, 256:]) < 2 ** -7


def test_three_product_split_drops_only_lo_lo():
    torch.manual_seed(0)
    a, b = torch.randn(64, 96), torch.randn(96, 48)
    o = {"x3": True}
    exact = ref_cpu._q(a, "s") @ ref_cpu._q(b, "s")
    three = ref_cpu._mm(a, "s", b, "s", o)
    assert _rel(three.double(), exact.double()) < 2 ** -14
    assert _rel(three.double(), (a.double() @ b.double())) < 2 ** -13


def test_kernel_emulation_as_close_to_float64_as_round4():
    g = load("c1_32x32_n32")
    f64 = _grads(g, torch.float64)
    k = _grads(g, ops=ref_cpu.OPS_BF16X3_K, layer_ops=ref_cpu.X3_LAYER_OPS)
    d = _grads(g, ops=ref_cpu.OPS_BF16X3_DB, layer_ops=ref_cpu.X3_LAYER_OPS)
    for name in f64:
        ek, ed = _rel(k[name], f64[name]), _rel(d[name], f64[name])
        assert ek < 2 * ed + 1e-5, (name, ek, ed)
        assert ek < 2e-3, (name, ek)
