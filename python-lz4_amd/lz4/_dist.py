"""Multi-GPU sharding of a block batch.

Blocks are independent, so a batch shards across ranks with no exchange:
rank r owns the contiguous range shard_range(n, r, world).  The one real
exchange is collecting per-shard *compressed* output at a root (config 5):

  1. all_gather of per-rank (block count, compressed byte total) -- tiny;
  2. the root sizes one output buffer and receives every rank's compacted
     shard at its prefix offset (point-to-point, one stream per peer; over
     xGMI each sender uses its own link into the root);
  3. all_gather of per-block compressed lengths, so every rank (or just the
     root) can rebuild the block index.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm, device
tensors) on the GPU box, "gloo" (CPU tensors) in the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block range [lo, hi) of `rank`; sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world or n < 0:
        raise ValueError("bad shard arguments")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def gather_compressed(comp: torch.Tensor, block_len: torch.Tensor, root: int = 0, group=None):
    """Collect every rank's compacted compressed shard at `root`.

    comp      -- this rank's compressed blocks, back to back (uint8, 1-D)
    block_len -- their sizes (int32, 1-D); sum == comp.numel()

    Returns (buf, offsets, lengths) on the root: all shards concatenated in
    rank order, the int64 start of every block in buf, and the int32 block
    sizes (global block order == rank order).  Other ranks get
    (None, None, lengths).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = comp.device
    if comp.dtype != torch.uint8 or comp.dim() != 1 or block_len.dim() != 1:
        raise ValueError("comp must be 1-D uint8 and block_len 1-D")
    meta = torch.tensor([block_len.numel(), comp.numel()], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    counts = [int(m[0]) for m in metas]
    totals = [int(m[1]) for m in metas]

    # per-block lengths, padded to the largest shard for all_gather
    mx = max(counts) if counts else 0
    padded = torch.zeros(mx, dtype=torch.int32, device=dev)
    padded[: block_len.numel()] = block_len.to(torch.int32)
    lens_all = [torch.empty(mx, dtype=torch.int32, device=dev) for _ in range(world)]
    dist.all_gather(lens_all, padded, group=group)
    lengths = torch.cat([lens_all[r][: counts[r]] for r in range(world)])

    if rank == root:
        starts = [0]
        for t in totals[:-1]:
            starts.append(starts[-1] + t)
        buf = torch.empty(sum(totals), dtype=torch.uint8, device=dev)
        buf[starts[rank]: starts[rank] + totals[rank]].copy_(comp)
        reqs = []
        for r in range(world):
            if r != rank and totals[r] > 0:
                reqs.append(dist.irecv(buf[starts[r]: starts[r] + totals[r]], src=_global(r, group), group=group))
        for q in reqs:
            q.wait()
        offsets = torch.zeros(lengths.numel(), dtype=torch.int64, device=dev)
        if lengths.numel() > 1:
            offsets[1:] = torch.cumsum(lengths[:-1].to(torch.int64), 0)
        return buf, offsets, lengths
    if totals[rank] > 0:
        dist.send(comp, dst=_global(root, group), group=group)
    return None, None, lengths


def _global(r: int, group) -> int:
    return r if group is None else dist.get_global_rank(group, r)
