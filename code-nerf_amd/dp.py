"""Data-parallel plumbing of the training step.

One process per GPU; each rank renders its own object(s) (weak scaling: the
per-rank work is fixed as ranks are added).  Per optimiser step the ranks
exchange

  * the model gradients: one SUM all-reduce of a flat fp32 bucket (714,756
    floats = 2.86 MB at the srncar net; RCCL over xGMI on MI355X, gloo in the
    CPU tests), issued asynchronously AFTER the small code-row exchange below
    (on one communicator, a collective queued behind it would wait for it),
    so the code tables' AdamW runs while it is in flight;
  * the code-table gradients, which are row-sparse (a rank touches only the
    rows of the objects it rendered): an all_gather of (row index, shape row,
    texture row) = 513 floats per rendered object, scattered back into the
    dense gradient tables in rank order on every rank.

Every rank then runs the same dense AdamW over the model and both code tables
(the reference's dense-embedding AdamW moves every row every step,
src/trainer.py:116-120), so replicas stay bit-identical without a parameter
broadcast.  The reference has no distributed path (one device,
src/trainer.py:25); with one rank every exchange is skipped and the step is
exactly its loop.
"""
import torch


def _active(dist, group=None):
    return dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1


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

    def all_reduce(self, dist, group=None, async_op=False):
        """Sum the gradients of all ranks (in place).  async_op: returns the
        collective's work handle (None when there is nothing to exchange)."""
        if _active(dist, group):
            return dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        return None


class GradExchange:
    """The per-step gradient exchange of object-sharded data parallelism:
    model bucket all-reduce (async) + touched code-row all_gather."""

    def __init__(self, model_params, code_tables, dist=None, group=None):
        self.bucket = GradBucket(model_params)
        self.tables = list(code_tables)
        for t in self.tables:
            t.grad = torch.zeros_like(t)
        self.dist, self.group = dist, group
        # set by a fused AdamW step that left every gradient at 0: the next
        # zero() then needs no launch (and consumes the flag)
        self.clean = False

    @property
    def active(self):
        return _active(self.dist, self.group)

    def zero(self):
        if self.clean:
            self.clean = False
            return
        self.bucket.zero()
        for t in self.tables:
            t.grad.zero_()

    def mark_dirty(self):
        """A backward wrote into the gradients: the next zero() must clear them."""
        self.clean = False

    def start_model(self):
        """Launch the model-gradient all-reduce; returns a handle for finish()."""
        return self.bucket.all_reduce(self.dist, self.group, async_op=True)

    @staticmethod
    def finish(handle):
        if handle is not None:
            handle.wait()

    def exchange_rows(self, rows, max_rows=None):
        """All-gather the gradient rows ``rows`` (object indices this rank
        rendered; duplicates are taken once) of every code table and rebuild
        the dense gradient tables from them, identically on every rank.
        Payload per object: 1 + 256 x n_tables floats.  Ranks may pass
        different counts: every rank pads to ``max_rows`` (default: the
        largest count, agreed by one small all_gather first) with index -1
        rows, which are dropped."""
        if not self.active:
            return
        dist, group = self.dist, self.group
        world = dist.get_world_size(group)
        t0 = self.tables[0]
        dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else t0.device
        uniq = sorted(set(int(r) for r in rows))
        k = len(uniq)
        if max_rows is None:
            cnt = torch.tensor([k], dtype=torch.int64, device=dev)
            cnts = [torch.empty_like(cnt) for _ in range(world)]
            dist.all_gather(cnts, cnt, group=group)
            max_rows = int(max(int(c) for c in cnts))
        if k > max_rows:
            raise ValueError(f"exchange_rows: {k} rows exceed max_rows={max_rows}")
        idx = torch.as_tensor(uniq, dtype=torch.long, device=t0.device)
        width = sum(t.shape[1] for t in self.tables)
        mine = torch.zeros(max_rows, 1 + width, dtype=torch.float32, device=t0.device)
        mine[:, 0] = -1.0
        mine[:k, 0] = idx.to(torch.float32)             # exact: object counts are far below 2^24
        off = 1
        for t in self.tables:
            mine[:k, off:off + t.shape[1]] = t.grad[idx]
            off += t.shape[1]
        mine = mine.to(dev)
        got = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(got, mine, group=group)
        allrows = torch.cat(got).to(t0.device)          # rank order: identical on every rank
        allrows = allrows[allrows[:, 0] >= 0]
        rid = allrows[:, 0].long()
        off = 1
        for t in self.tables:
            t.grad.zero_()
            t.grad.index_add_(0, rid, allrows[:, off:off + t.shape[1]])
            off += t.shape[1]

    def bytes_per_step(self, rows_per_rank=1):
        """Bytes each rank contributes to the exchange (fp32)."""
        width = sum(t.shape[1] for t in self.tables)
        return {"model_all_reduce": self.bucket.flat.numel() * 4, "code_rows_all_gather": rows_per_rank * (1 + width) * 4}


def world_rank(dist, group=None):
    """(world, rank) of this process; (1, 0) without an initialised group."""
    if dist is not None and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def shard(items, dist, group=None):
    """This rank's share of ``items`` (round-robin, order kept): evaluation
    views of src/optimizer.py:108-130 split across ranks."""
    world, rank = world_rank(dist, group)
    return list(items)[rank::world]


def gather_by_key(local, dist, group=None):
    """Merge every rank's {key: value} into one dict ordered by key, on every
    rank (all_gather_object; no-op with one rank)."""
    world, _ = world_rank(dist, group)
    if world == 1:
        return dict(sorted(local.items()))
    parts = [None] * world
    dist.all_gather_object(parts, dict(local), group=group)
    merged = {}
    for p in parts:
        merged.update(p)
    return dict(sorted(merged.items()))


def ray_block(R, dist, group=None, align=1):
    """Contiguous ray range [a, b) of this rank when one image is split into
    row blocks (C5 inference); blocks are multiples of
    ``align`` rays except the last."""
    world, rank = world_rank(dist, group)
    per = -(-R // world)
    per = -(-per // align) * align
    a = min(R, rank * per)
    return a, min(R, a + per)


def gather_ray_blocks(block, R, dist, group=None, align=1):
    """Reassemble an image of R rays from every rank's ``block`` (rows
    [a, b) of ray_block), on every rank."""
    world, _ = world_rank(dist, group)
    if world == 1:
        return block
    per = -(-R // world)
    per = -(-per // align) * align
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else block.device
    pad = torch.zeros((per,) + tuple(block.shape[1:]), dtype=block.dtype, device=dev)
    pad[:block.shape[0]] = block.to(dev)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat(parts)[:R].to(block.device)


def object_for(step, rank, world, n_objects):
    """Object rendered by ``rank`` at global step ``step``: consecutive ranks
    take consecutive objects, so one step covers ``world`` distinct objects
    (the reference iterates one object per step, src/trainer.py:56-58)."""
    return (step * world + rank) % n_objects


def broadcast_from(tensors, dist, src=0):
    """Make every rank start from rank ``src``'s values (weights, codes)."""
    if _active(dist):
        for t in tensors:
            dist.broadcast(t.data, src)
