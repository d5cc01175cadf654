import sys, os, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import test_gpu_dw as T
from codenerf_amd.model import CodeNeRF
dev = torch.device("cuda", 0)
torch.manual_seed(3)
m = CodeNeRF(3, 1, precision="bf16").to(dev)
eng = m.engine(); params = m.param_list()
R, N = 3000 - 7, 64; M = R * N
ro = torch.zeros(R, 3, device=dev) + torch.tensor([0.0, 0.4, 1.2], device=dev)
vd = torch.nn.functional.normalize(torch.randn(R, 3, device=dev) * 0.2 + torch.tensor([0., -0.3, -1.], device=dev), dim=-1)
z = torch.linspace(0.8, 1.8, N, device=dev)
s = torch.randn(256, device=dev) / 11.3; t = torch.randn(256, device=dev) / 11.3
eng.ensure_packed(params, bwd=True)
blob, zvec = eng.latent_fwd(params, s, t)
act = eng.new_act(M); act.fill_(0x7f)
eng.mlp_fwd(blob, M, rays_o=ro, rays_d=vd, z=z, n_samples=N, act=act)
Mp = eng.pad(M)
dsig = torch.zeros(Mp, device=dev); drgb = torch.zeros(Mp, 3, device=dev)
dsig[:M] = torch.randn(M, device=dev) * 1e-3; drgb[:M] = torch.randn(M, 3, device=dev) * 1e-3
eng.mlp_bwd(blob, M, dsig, drgb, act)
torch.cuda.synchronize()
off = T.act_offsets(Mp, 2)
for name, F in [("pe", 64), ("dir", 32)] + [(f"Y{p}", T.plane_width(p)) for p in range(8)] + [(f"dA{p}", T.dplane_width(p)) for p in range(8)] + [("d8", 32)]:
    a = T.decode(act, off[name], F, Mp, torch.bfloat16)
    bad = (a == T.decode(torch.full_like(act, 0x7f), 0, F, Mp, torch.bfloat16)[0, 0]).nonzero()
    pad_nz = (a[M:] != 0).nonzero()
    print(name, "unwritten(0x7f7f):", bad.shape[0], bad[:4].tolist(), "pad nonzero:", pad_nz.shape[0], pad_nz[:6].tolist())
a = T.decode(act, off["dA0"], 256, Mp, torch.bfloat16)
nz = (a[M:] != 0).nonzero()
print("dA0 pad values", [(int(i), int(j), float(a[M + i, j])) for i, j in nz[:12].tolist()])
print("isnan any dA0", torch.isnan(a).any().item(), "valid nan", torch.isnan(a[:M]).any().item())
# zero upstream -> all dA must be zero
dsig.zero_(); drgb.zero_(); act2 = act.clone()
eng.mlp_bwd(blob, M, dsig, drgb, act2); torch.cuda.synchronize()
for p in range(8):
    a = T.decode(act2, off[f"dA{p}"], T.dplane_width(p), Mp, torch.bfloat16)
    print("zero-upstream dA", p, "nonzero", (a != 0).sum().item())
