"""Pin the CPU oracle (oracle/ref_cpu.py) to the reference's golden vectors.

The vectors were produced by importing the reference's src/model.py and
src/utils.py (tools/gen_golden.py).  CPU only.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu
from oracle.params import make_params, param_specs
from golden_util import TRAIN_CASES, load, case_params, digest_matches, oracle_image_step


def test_param_specs_match_reference_names():
    g = load("c1_32x32_n32")
    names = [str(n) for n in g["param_names"]]
    assert names == [n for n, _ in param_specs()]
    p = make_params(0)
    assert sum(v.size for v in p.values()) == 714756


def test_positional_encoding():
    g = load("pe_render")
    x, d = torch.tensor(g["x"]), torch.tensor(g["d"])
    np.testing.assert_array_equal(ref_cpu.positional_encoding(x, 10).numpy(), g["pe10"])
    np.testing.assert_array_equal(ref_cpu.positional_encoding(d, 4).numpy(), g["pe4"])


def test_volume_rendering_fwd_bwd():
    g = load("pe_render")
    sig = torch.tensor(g["sig"], requires_grad=True)
    rgbs = torch.tensor(g["rgbs"], requires_grad=True)
    rgb, depth = ref_cpu.volume_rendering(sig, rgbs, torch.tensor(g["z"]))
    np.testing.assert_array_equal(rgb.detach().numpy(), g["rgb"])
    np.testing.assert_array_equal(depth.detach().numpy(), g["depth"])
    ((rgb * torch.tensor(g["drgb"])).sum() + (depth * torch.tensor(g["ddepth"])).sum()).backward()
    np.testing.assert_array_equal(sig.grad.numpy(), g["dsig"])
    np.testing.assert_array_equal(rgbs.grad.numpy(), g["drgbs"])


@pytest.mark.parametrize("case", TRAIN_CASES)
def test_rays_and_samples(case):
    g = load(case)
    H, W = int(g["H"]), int(g["W"])
    focal = torch.tensor([float(g["focal"])], dtype=torch.float64)
    ro, vd = ref_cpu.get_rays(H, W, focal, torch.tensor(g["c2w"]))
    np.testing.assert_array_equal(ro.numpy(), g["rays_o"])
    np.testing.assert_array_equal(vd.numpy(), g["viewdir"])
    z = ref_cpu.stratified_z(float(g["near"]), float(g["far"]), int(g["N"]), torch.tensor(g["jitter"]))
    np.testing.assert_array_equal(z.numpy(), g["z_vals"])


@pytest.mark.parametrize("case", TRAIN_CASES)
def test_forward_render(case):
    g = load(case)
    p = ref_cpu.param_tensors(case_params(g), requires_grad=False)
    oi = int(g["obj_idx"])
    s = torch.tensor(g["shape_table"][oi:oi + 1])
    t = torch.tensor(g["texture_table"][oi:oi + 1])
    xyz, vd, z = ref_cpu.sample_from_rays(torch.tensor(g["rays_o"]), torch.tensor(g["viewdir"]),
                                          float(g["near"]), float(g["far"]), int(g["N"]),
                                          torch.tensor(g["jitter"]))
    sig, rgbs = ref_cpu.codenerf_forward(p, xyz, vd, s, t)
    if "sigmas" in g:
        np.testing.assert_allclose(sig.numpy(), g["sigmas"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rgbs.numpy(), g["rgbs"], rtol=1e-5, atol=1e-6)
    rgb, depth = ref_cpu.volume_rendering(sig, rgbs, z)
    np.testing.assert_allclose(rgb.numpy(), g["rgb"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(depth.numpy(), g["depth"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", TRAIN_CASES)
def test_train_step_grads_and_adamw(case):
    g = load(case)
    r = oracle_image_step(g)
    np.testing.assert_allclose(r["losses"], g["chunk_losses"], rtol=1e-5)
    for k, prm in r["params"].items():
        ok, err = digest_matches(g, k, prm.grad.numpy())
        assert ok, (k, err)
    np.testing.assert_allclose(r["shape_table"].grad.numpy(), g["grad/shape_table"], rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(r["texture_table"].grad.numpy(), g["grad/texture_table"], rtol=1e-4, atol=1e-9)
    # one AdamW step, groups as src/trainer.py:116-120
    opt = ref_cpu.AdamWRef([(list(r["params"].values()), 1e-4), ([r["shape_table"]], 1e-3),
                            ([r["texture_table"]], 1e-3)])
    opt.step()
    for k, prm in r["params"].items():
        idx = g[f"adamw/{k}/idx"]
        np.testing.assert_allclose(prm.detach().numpy().reshape(-1)[idx], g[f"adamw/{k}/vals"],
                                   rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(r["shape_table"].detach().numpy(), g["adamw/shape_table"], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(r["texture_table"].detach().numpy(), g["adamw/texture_table"], rtol=1e-6, atol=1e-8)


def test_bf16_operand_mode_is_scoped_and_close():
    """ref_cpu.bf16_operands() restates the bf16 kernels' operand rounding;
    outside the block the oracle is the fp32 reference again."""
    import torch
    from oracle import ref_cpu
    from oracle.params import make_params, make_codes
    p = ref_cpu.param_tensors(make_params(2), requires_grad=False)
    s, t = (torch.tensor(c) for c in make_codes(2, 1))
    g = torch.Generator().manual_seed(0)
    x = torch.rand(64, 8, 3, generator=g) * 2 - 1
    v = torch.nn.functional.normalize(torch.randn(64, 8, 3, generator=g), dim=-1)
    s32, r32 = ref_cpu.codenerf_forward(p, x, v, s, t)
    with ref_cpu.bf16_operands():
        s16, r16 = ref_cpu.codenerf_forward(p, x, v, s, t)
    s32b, r32b = ref_cpu.codenerf_forward(p, x, v, s, t)
    assert torch.equal(s32, s32b) and torch.equal(r32, r32b)
    assert not torch.equal(r16, r32)
    assert float((r16 - r32).abs().max()) < 5e-3
