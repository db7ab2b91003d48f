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


class GatherHandle:
    """An in-flight gather_compressed (gather_start -> gather_finish)."""

    def __init__(self, reqs, result):
        self.reqs = reqs
        self.result = result


def gather_start(comp: torch.Tensor, block_len: torch.Tensor, root: int = 0, group=None,
                 out: torch.Tensor | None = None) -> GatherHandle:
    """Start collecting every rank's compacted compressed shard at `root`.

    comp      -- this rank's compressed blocks, back to back (uint8, 1-D)
    block_len -- their sizes (int32, 1-D); sum == comp.numel()
    out       -- (root, optional) a uint8 buffer to receive into, reused
                 across calls when large enough

    The two metadata all_gathers (counts and totals, then per-block lengths)
    complete here; the bulk point-to-point transfers are only posted
    (isend / irecv), so the caller can enqueue more work -- e.g. compress
    the next wave -- while they run.  gather_finish waits for them.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = comp.device
    if comp.dtype != torch.uint8 or comp.dim() != 1 or block_len.dim() != 1:
        raise ValueError("comp must be 1-D uint8 and block_len 1-D")
    meta = torch.tensor([block_len.numel(), comp.numel()], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    mm = torch.stack(metas).cpu()
    counts = [int(x) for x in mm[:, 0]]
    totals = [int(x) for x in mm[:, 1]]

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
        need = sum(totals)
        buf = out[:need] if out is not None and out.numel() >= need else torch.empty(need, dtype=torch.uint8,
                                                                                    device=dev)
        buf[starts[rank]: starts[rank] + totals[rank]].copy_(comp)
        reqs = []
        for r in range(world):
            if r != rank and totals[r] > 0:
                reqs.append(dist.irecv(buf[starts[r]: starts[r] + totals[r]], src=_global(r, group), group=group))
        offsets = torch.zeros(lengths.numel(), dtype=torch.int64, device=dev)
        if lengths.numel() > 1:
            offsets[1:] = torch.cumsum(lengths[:-1].to(torch.int64), 0)
        return GatherHandle(reqs, (buf, offsets, lengths))
    reqs = [dist.isend(comp, dst=_global(root, group), group=group)] if totals[rank] > 0 else []
    return GatherHandle(reqs, (None, None, lengths))


def gather_finish(h: GatherHandle):
    """Wait for a gather_start; returns (buf, offsets, lengths) on the root:
    all shards concatenated in rank order, the int64 start of every block
    in buf, and the int32 block sizes (global block order == rank order).
    Other ranks get (None, None, lengths)."""
    for q in h.reqs:
        q.wait()
    h.reqs = []
    return h.result


def gather_compressed(comp: torch.Tensor, block_len: torch.Tensor, root: int = 0, group=None):
    """Collect every rank's compacted compressed shard at `root` (blocking
    gather_start + gather_finish)."""
    return gather_finish(gather_start(comp, block_len, root, group))


def compress_gather_waves(compress_wave, waves: int, root: int = 0, group=None, overlap: bool = True,
                          consume=None) -> dict:
    """Config 5's wave driver: a shard larger
    than HBM is compressed in `waves` waves over a resident working set, and
    every wave's compressed output is gathered at `root`.

    compress_wave(w) -> (comp uint8 1-D, block_len int32 1-D): enqueues wave
    w's compression + compaction on the current stream and returns its
    compacted output (the buffers must stay valid until the wave after next
    is requested: double-buffer them).  With `overlap`, the gather of wave w
    runs while wave w + 1 compresses (the bulk transfers are posted before
    the next wave is enqueued).  consume(w, buf, offsets, lengths) is called
    on the root with each gathered wave.  Returns byte counts for rates.
    """
    rank = dist.get_rank(group)
    bufs = [None, None]
    stats = {"waves": waves, "comp_bytes": 0, "gathered_bytes": 0, "blocks": 0}
    pending = None

    def done(w, h):
        buf, off, lens = gather_finish(h)
        if rank == root:
            stats["gathered_bytes"] += buf.numel()
            if consume is not None:
                consume(w, buf, off, lens)
            bufs[w & 1] = buf

    for w in range(waves):
        comp, lens = compress_wave(w)
        stats["comp_bytes"] += comp.numel()
        stats["blocks"] += lens.numel()
        if pending is not None and not overlap:
            done(*pending)
            pending = None
        h = gather_start(comp, lens, root, group, out=bufs[w & 1] if rank == root else None)
        if pending is not None:
            done(*pending)
        pending = (w, h)
        if not overlap:
            done(*pending)
            pending = None
    if pending is not None:
        done(*pending)
    return stats


def _global(r: int, group) -> int:
    return r if group is None else dist.get_global_rank(group, r)
