"""Fused AdamW: torch.optim.AdamW semantics (as used at src/trainer.py:116-120
and src/optimizer.py:195-198) with the update of every parameter of every
group done by one HIP launch (optim.hip)."""
import torch

from . import engine as _eng


class FusedAdamW:
    def __init__(self, param_groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if isinstance(param_groups, torch.Tensor):
            raise TypeError("params must be an iterable of tensors or of dicts")
        groups = list(param_groups)
        if groups and not isinstance(groups[0], dict):
            groups = [{"params": groups}]
        self.param_groups = []
        for g in groups:
            ps = g["params"]
            ps = [ps] if isinstance(ps, torch.Tensor) else list(ps)
            self.param_groups.append(dict(params=ps, lr=g.get("lr", lr), betas=g.get("betas", betas),
                                          eps=g.get("eps", eps), weight_decay=g.get("weight_decay", weight_decay)))
        self.state = {}

    def zero_grad(self, set_to_none=False):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()

    @torch.no_grad()
    def step(self, groups=None, zero_grad=False):
        """groups: indices of the param groups to update (default all) -- a
        step split over two calls (codes while the model gradients are still
        being all-reduced, then the model) is the same update as one call.
        zero_grad: the update kernel leaves every gradient it read at 0 (the
        next zero_grad() for free)."""
        # one launch per (betas, eps, weight_decay) combination; lr is per tensor
        buckets = {}
        sel = self.param_groups if groups is None else [self.param_groups[i] for i in groups]
        for g in sel:
            key = (tuple(g["betas"]), g["eps"], g["weight_decay"])
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state.get(p)
                if st is None:
                    st = self.state[p] = dict(step=0, exp_avg=torch.zeros_like(p), exp_avg_sq=torch.zeros_like(p))
                st["step"] += 1
                buckets.setdefault((key, st["step"]), []).append((p, st, g["lr"]))
        for ((betas, eps, wd), step), items in buckets.items():
            _eng.adamw_step([p for p, _, _ in items], [p.grad for p, _, _ in items],
                            [s["exp_avg"] for _, s, _ in items], [s["exp_avg_sq"] for _, s, _ in items],
                            [lr for _, _, lr in items], wd, betas[0], betas[1], eps, step, zero_grad=zero_grad)
