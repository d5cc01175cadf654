"""CPU emulation of the bf16 chain path's operand roundings (weights, layer inputs,
upstream gradients) on the oracle's image step: which rounding moves the
gradients most (relative L2 error, fraction of sign flips vs pure fp32).
Result quoted in DESIGN.md section 4 / tests/test_gpu_converge.py."""
import sys, torch, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
from oracle import ref_cpu
from oracle.params import make_params, make_codes, look_at_pose
import torch.nn.functional as F
torch.set_num_threads(8)
def rb(t): return t.to(torch.bfloat16).to(torch.float32)
FLAGS = dict(w=False, x=False, dy=False)
class Lin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        xx = rb(x) if FLAGS['x'] else x
        ww = rb(w) if FLAGS['w'] else w
        ctx.save_for_backward(xx, ww)
        return xx @ ww.t() + b
    @staticmethod
    def backward(ctx, dy):
        xx, ww = ctx.saved_tensors
        d = rb(dy) if FLAGS['dy'] else dy
        return d @ ww, d.reshape(-1, d.shape[-1]).t() @ xx.reshape(-1, xx.shape[-1]), d.reshape(-1, d.shape[-1]).sum(0)
ref_cpu._lin = lambda p, name, x: Lin.apply(x, p[name + ".weight"], p[name + ".bias"])
from codenerf_amd.data import _object_spec, _render_object
H=32; focal=32.8
c2w = look_at_pose(1.3, 30., 20.)
spec=_object_spec(np.random.Generator(np.random.PCG64(5)))
gt = torch.tensor(_render_object(spec, c2w.astype(np.float64), H, H, focal).reshape(-1,3), dtype=torch.float32)
ro, vd = ref_cpu.get_rays(H, H, torch.tensor([focal],dtype=torch.float64), torch.tensor(c2w))
z = ref_cpu.stratified_z(0.8,1.8,32, jitter=torch.rand(32, generator=torch.Generator().manual_seed(1)))
params = make_params(3); s0,t0 = make_codes(3,1)
def run():
    p = ref_cpu.param_tensors(params)
    st = torch.tensor(s0, requires_grad=True); tt = torch.tensor(t0, requires_grad=True)
    ref_cpu.image_step(p, st, tt, 0, ro, vd, z, gt, chunk=256)
    return {k: v.grad.clone() for k,v in p.items()}
base = run()
for cfg in [dict(w=True), dict(x=True), dict(dy=True), dict(w=True,x=True,dy=True)]:
    FLAGS.update(w=False,x=False,dy=False); FLAGS.update(cfg)
    g = run()
    errs = {k: float((g[k]-base[k]).norm()/base[k].norm()) for k in base}
    # fraction of sign flips weighted
    flips = np.mean([float(((g[k]*base[k])<0).float().mean()) for k in base if base[k].numel()>300])
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
    print(cfg, "mean relL2 %.2e"%np.mean(list(errs.values())), "sign flips %.4f"%flips, [(k, "%.1e"%e) for k,e in worst])
