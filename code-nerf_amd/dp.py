"""Data-parallel plumbing of the training step.

One process per GPU; each rank renders its own object(s) (weak scaling: the
per-rank work is fixed as ranks are added).  The only exchange per optimiser
step is one SUM all-reduce of the flat fp32 gradient bucket (RCCL over xGMI
on MI355X; gloo in the CPU tests) -- model gradients (714,756 floats, 2.9 MB)
followed by the two code tables, whose rows are touched only by the objects
rendered this step.  Every rank then runs the same dense AdamW on identical
data, so replicas stay bit-identical without a parameter broadcast.

The reference has no distributed path (one device, src/trainer.py:25); with
one rank this reduces exactly to its loop.
"""
import torch


class GradBucket:
    """One flat fp32 buffer holding the gradient of every tensor; each
    tensor's ``.grad`` is a view into it, so zeroing is one memset and the
    data-parallel exchange is one collective."""

    def __init__(self, tensors):
        self.tensors = list(tensors)
        total = sum(t.numel() for t in self.tensors)
        dev = self.tensors[0].device
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for t in self.tensors:
            if t.dtype != torch.float32:
                raise TypeError("GradBucket: fp32 tensors only")
            t.grad = self.flat[off:off + t.numel()].view_as(t)
            off += t.numel()

    def zero(self):
        self.flat.zero_()

    def all_reduce(self, dist, group=None):
        """Sum the gradients of all ranks (in place)."""
        if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)


def object_for(step, rank, world, n_objects):
    """Object rendered by ``rank`` at global step ``step``: consecutive ranks
    take consecutive objects, so one step covers ``world`` distinct objects
    (the reference iterates one object per step, src/trainer.py:56-58)."""
    return (step * world + rank) % n_objects


def broadcast_from(tensors, dist, src=0):
    """Make every rank start from rank ``src``'s values (weights, codes)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        for t in tensors:
            dist.broadcast(t.data, src)
