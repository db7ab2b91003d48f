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


class _Side:
    """The side stream the gather runs on (GPU tensors): high priority, so its
    copies and the RCCL launches it orders are not queued behind compression
    kernels.  Collectives posted under it make RCCL's stream wait only for
    what was recorded here (torch's ProcessGroupNCCL syncs with the *current*
    stream), i.e. for the wave being gathered, not for the next wave's
    compression enqueued after it.  With CPU tensors (gloo) it is a no-op."""

    def __init__(self, dev: torch.device):
        self.gpu = dev.type == "cuda"
        self.stream = torch.cuda.Stream(device=dev, priority=-1) if self.gpu else None

    def ctx(self):
        return torch.cuda.stream(self.stream) if self.gpu else _Null()

    def mark(self):
        """An event after everything enqueued on the current stream so far (None on CPU)."""
        if not self.gpu:
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.stream.device))
        return ev

    def wait(self, ev):
        """Order the side stream after `ev`."""
        if ev is not None:
            self.stream.wait_event(ev)

    def before_current(self):
        """Order the current stream after everything enqueued on the side stream so far."""
        if self.gpu:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _page_bounds(lens: torch.Tensor, page_blocks: int) -> torch.Tensor:
    """Byte offsets of the page cuts of one shard: page k = blocks
    [k * page_blocks, (k + 1) * page_blocks); returns int64 [pages + 1].
    Per-page sums (a plain reduction) and a scan over the few page sums: a
    device-wide scan of every block length is a look-back scan whose waiting
    workgroups would sit on CUs beside the next wave's compression."""
    n = lens.numel()
    pages = (n + page_blocks - 1) // page_blocks
    out = torch.zeros(pages + 1, dtype=torch.int64, device=lens.device)
    if n:
        full = n // page_blocks
        sums = torch.zeros(pages, dtype=torch.int64, device=lens.device)
        if full:
            sums[:full] = lens[: full * page_blocks].view(full, page_blocks).to(torch.int64).sum(1)
        if n > full * page_blocks:
            sums[full] = lens[full * page_blocks:].to(torch.int64).sum()
        torch.cumsum(sums, 0, out=out[1:])
    return out


def compress_gather_waves(compress_wave, waves: int, root: int = 0, group=None, overlap: bool = True,
                          consume=None, page_blocks: int = 4096, ring: int = 4) -> dict:
    """Config 5's wave driver: a shard larger
    than HBM is compressed in `waves` waves over a resident working set, and
    every wave's compressed output is gathered at `root`, which consumes it
    page by page (a root cannot hold 8 ranks' waves: at 1 M x 64 KiB blocks
    a wave is ~34 GiB compressed per rank).

    compress_wave(w) -> (comp uint8 1-D, block_len int32 1-D): enqueues wave
    w's compression + compaction on the current stream and returns the
    compacted blocks, back to back (comp may be longer than the blocks).
    The driver calls compress_wave(w + 2) only after wave w's transfers out
    of its buffers are ordered before the current stream, so two buffers
    alternated by w & 1 are enough.

    consume(w, src_rank, first_block, buf, lens) is called on the root for
    every page: `lens` (int32, device) are the sizes of blocks
    first_block .. first_block + len(lens) of rank src_rank's wave w, back to
    back in `buf`.  On GPU tensors it is called under the gather's side
    stream and must only enqueue work there; `buf` is valid only during the
    call's stream work (the memory is reused for a later page), so clone it
    to keep it.

    Per wave: the root learns every rank's page sizes from two small
    all_gathers (block counts, then block sizes) -- the one host wait per
    wave, needed because point-to-point sizes must be known on the host.
    With `overlap` (default) wave w's gather is posted only after wave w + 1's
    compression is enqueued, so that wait lands while the GPU compresses and
    the transfers run beside the next wave; without it each wave's gather
    completes before the next wave starts.  Peers send their pages with
    isend; the root receives them into a ring of `ring` page buffers per peer
    and consumes its own shard in place.  Returns byte counts for rates.
    """
    # one process and no process group (bench.py at N = 1): rank 0 of 1,
    # nothing to exchange
    grouped = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if grouped else 0
    world = dist.get_world_size(group) if grouped else 1
    stats = {"waves": waves, "comp_bytes": 0, "gathered_bytes": 0, "blocks": 0, "pages": 0, "host_waits": 0}
    side = None
    sends = {}            # wave -> outstanding send works (buffers of that wave in use)
    slots = {}            # (peer, ring index) -> receive buffer
    pending = None

    def post(w, comp, lens, ev):
        dev = comp.device
        side.wait(ev)                 # wave w's compression, not the next wave's
        with side.ctx():
            meta = torch.tensor([lens.numel()], dtype=torch.int64, device=dev)
            if world > 1:
                metas = [torch.empty_like(meta) for _ in range(world)]
                dist.all_gather(metas, meta, group=group)
                counts = [int(x) for x in torch.cat(metas).cpu()]          # host wait (1)
                mx = max(counts)
                padded = torch.zeros(mx, dtype=torch.int32, device=dev)
                padded[: lens.numel()] = lens
                lens_all = [torch.empty(mx, dtype=torch.int32, device=dev) for _ in range(world)]
                dist.all_gather(lens_all, padded, group=group)
                lens_all = [lens_all[r][: counts[r]] for r in range(world)]
            else:
                lens_all = [lens]
            need = range(world) if rank == root else [rank]
            bounds = {r: _page_bounds(lens_all[r], page_blocks) for r in need}
            hb = torch.cat([bounds[r] for r in need]).cpu().tolist()    # host wait (2), same sync point
            stats["host_waits"] += 2
            pos = 0
            host_bounds = {}
            for r in need:
                k = bounds[r].numel()
                host_bounds[r] = hb[pos: pos + k]
                pos += k
            mine = host_bounds[rank]
            stats["comp_bytes"] += mine[-1]
            stats["blocks"] += lens.numel()
            if rank != root:
                works = []
                for k in range(len(mine) - 1):
                    a, b = mine[k], mine[k + 1]
                    if b > a:
                        works.append(dist.isend(comp[a:b], dst=_global(root, group), group=group))
                        stats["pages"] += 1
                sends[w] = works
                return
            # root: own shard in place, then every peer's pages through the ring
            for k in range(len(mine) - 1):
                if consume is not None:
                    consume(w, rank, k * page_blocks, comp[mine[k]: mine[k + 1]],
                            lens_all[rank][k * page_blocks: (k + 1) * page_blocks])
            stats["gathered_bytes"] += mine[-1]
            live = {}         # (peer, ring index) -> (work, page, lo, hi)

            def finish(key):
                q, k, lo, hi = live.pop(key)
                q.wait()      # GPU: the side stream waits for the receive (no host wait)
                if consume is not None:
                    consume(w, key[0], k * page_blocks, slots[key][: hi - lo],
                            lens_all[key[0]][k * page_blocks: (k + 1) * page_blocks])

            npages = max((len(host_bounds[r]) - 1 for r in range(world) if r != rank), default=0)
            for k in range(npages):
                for r in range(world):
                    if r == rank or k >= len(host_bounds[r]) - 1:
                        continue
                    lo, hi = host_bounds[r][k], host_bounds[r][k + 1]
                    if hi == lo:
                        continue
                    key = (r, k % ring)
                    if key in live:
                        finish(key)   # its consume is ordered before the next receive into the slot
                    buf = slots.get(key)
                    if buf is None or buf.numel() < hi - lo:
                        slots[key] = buf = torch.empty(max(hi - lo, 1 << 20), dtype=torch.uint8, device=dev)
                    live[key] = (dist.irecv(buf[: hi - lo], src=_global(r, group), group=group), k, lo, hi)
                    stats["gathered_bytes"] += hi - lo
                    stats["pages"] += 1
            for key in list(live):
                finish(key)

    def release(w):
        """Order the current stream after wave w's transfers (its buffers are reused)."""
        for q in sends.pop(w, []):
            q.wait()
        if side is not None:
            side.before_current()

    for w in range(waves):
        if w >= 2:
            release(w - 2)
        comp, lens = compress_wave(w)
        if side is None:
            side = _Side(comp.device)
        ev = side.mark()
        if not overlap:
            post(w, comp, lens, ev)
            release(w)
            continue
        if pending is not None:
            post(*pending)          # wave w - 1, while wave w compresses
        pending = (w, comp, lens, ev)
    if pending is not None:
        post(*pending)
    for w in list(sends):
        release(w)
    if side is not None:
        side.before_current()
    return stats


def _global(r: int, group) -> int:
    return r if group is None else dist.get_global_rank(group, r)
