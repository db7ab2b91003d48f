"""Benchmark: batched LZ4 block codec on MI355X (BASELINE.json configs 2 and 3).

One "step" = one pass of the hot path over one batch: decompress of
1,048,576 x 64 KiB device-resident blocks (config 2, the headline `value`),
plus the compress pass of the same batch (config 3) reported beside it.

Data: the Silesia corpus is not available offline, so a seeded synthetic
"silesia-like" mix (lz4/_synth.py) stands in.  A pool of unique blocks is
generated on the host and tiled on the device with a per-tile XOR key (so
every block is distinct in memory and no tile is served from cache), then
compressed by our own compressor, which is byte-identical to
LZ4_compress_default (tests/test_gpu_codec.py) -- i.e. the decompress input
is exactly what lz4libs would produce.  Output is verified bit-exact against
the original blocks at full size.

Multi-GPU (one process per GPU; `--gpus N` without a launcher starts
torch.distributed.run itself): every rank decodes its own 1 M-block shard
(weak scaling, no data-path collective); timing is the max over ranks between
barriers.  value = all ranks' bytes / that time.  Config 5 (compress a shard
larger than HBM in waves, gather every wave's compressed output at rank 0
over RCCL, the gather of wave k overlapped with the compression of wave k+1)
is reported beside it, weak and strong scaling.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))

from lz4 import _native as N  # noqa: E402
from lz4 import _synth  # noqa: E402

BLOCK = 65536
GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_batch(n_blocks: int, pool: int, kind: str, seed: int, dev) -> torch.Tensor:
    """n_blocks x 64 KiB on the device: a host-generated pool tiled with a
    per-tile XOR key."""
    host = _synth.blocks(pool, kind, seed=seed)
    d_pool = torch.from_numpy(host).to(dev)
    out = torch.empty((n_blocks, BLOCK), dtype=torch.uint8, device=dev)
    tiles = (n_blocks + pool - 1) // pool
    for t in range(tiles):
        lo, hi = t * pool, min(n_blocks, (t + 1) * pool)
        key = (t * 151 + 7) & 0xFF if t else 0
        if key:
            torch.bitwise_xor(d_pool[: hi - lo], key, out=out[lo:hi])
        else:
            out[lo:hi].copy_(d_pool[: hi - lo])
    del d_pool
    return out.view(-1)


def compress_all(src: torch.Tensor, n: int, table: int, dev, events=None):
    """Compress n blocks into bound-sized slots; returns slots, offsets, lengths."""
    cap = N.compress_bound(BLOCK)
    cap16 = (cap + 15) // 16 * 16
    src_off = torch.arange(n, dtype=torch.int64, device=dev) * BLOCK
    src_len = torch.full((n,), BLOCK, dtype=torch.int32, device=dev)
    dst = torch.empty(n * cap16, dtype=torch.uint8, device=dev)
    dst_off = torch.arange(n, dtype=torch.int64, device=dev) * cap16
    dst_cap = torch.full((n,), cap, dtype=torch.int32, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    return (src_off, src_len, dst, dst_off, dst_cap, out_len)


class _HostEvent:
    """torch.cuda.Event's timing interface on the host clock (CPU runs of the
    timing helpers: tests/test_bench_dist.py)."""

    def __init__(self):
        self.t = 0.0

    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, end) -> float:
        return (end.t - self.t) * 1e3


def time_median(fn, reps: int, warmup: int, world: int):
    """`warmup` untimed calls, then `reps` calls each timed alone (barrier +
    sync around it, max over ranks): (median wall seconds, the samples).  For
    one-shot calls whose first run pays allocations or whose time moves from
    call to call (a single sample of the frame decode read 47 vs
    87-93 GiB/s)."""
    for _ in range(warmup):
        fn()
    ws = [time_kernel(fn, 1, 0, world)[0] for _ in range(reps)]
    return float(np.median(ws)), ws


def time_kernel(fn, steps: int, warmup: int, world: int, device: str = "cuda"):
    """Warmup, then time exactly `steps` calls bracketed by barrier+sync;
    returns (wall seconds, mean per-launch seconds from HIP events recorded on
    the launch stream), each the MAX over ranks.  device="cpu" runs the same
    protocol on the host clock (gloo process groups, CPU tests)."""
    cuda = device == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()

    for _ in range(warmup):
        fn()
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    ev = (lambda: torch.cuda.Event(enable_timing=True)) if cuda else _HostEvent
    evs = [(ev(), ev()) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in evs:
        a.record()
        fn()
        b.record()
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    wall = time.perf_counter() - t0
    ev_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    if world > 1:
        t = torch.tensor([wall, ev_ms], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        wall, ev_ms = float(t[0]), float(t[1])
    return wall, ev_ms / 1e3


def aggregate_gib_s(world: int, units_per_rank: int, unit_bytes: int, wall_s: float, steps: int) -> float:
    """Whole-job rate: the bytes ALL ranks processed (weak scaling: every
    rank the same units) over the max-over-ranks time of one step."""
    return world * units_per_rank * unit_bytes / (wall_s / steps) / GIB


def runs_cpu_baseline(rank: int, no_cpu: bool) -> bool:
    """The CPU baseline is timed on rank 0 only (its host cores), once."""
    return rank == 0 and not no_cpu


def host_threads() -> int:
    """Host threads for the CPU baselines: this process's CPU share.  The GPU
    box gives one GPU's job 16 cores (OMP_NUM_THREADS) while nproc shows the
    whole machine, so the share is min(affinity, OMP_NUM_THREADS or 16)."""
    try:
        vis = len(os.sched_getaffinity(0))
    except AttributeError:
        vis = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(vis, share))


def cpu_baseline(host_blocks: np.ndarray, comp_host: list, seconds: float = 10.0) -> dict:
    """Reference lz4libs (oracle/_ref, compiled from /root/reference) on the
    host cores: LZ4_decompress_safe over a bounded sample of the same
    workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O   # test/bench infrastructure only
    cb = O.CpuBench()
    cores = host_threads()
    n = len(comp_host)
    lens = np.array([len(c) for c in comp_host], dtype=np.int32)
    src = np.frombuffer(b"".join(comp_host), dtype=np.uint8)
    src_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    dst = np.empty(n * BLOCK, dtype=np.uint8)
    dst_off = (np.arange(n, dtype=np.int64) * BLOCK)
    dst_cap = np.full(n, BLOCK, dtype=np.int32)
    secs, out = cb.run("decompress", cores, 1, src, src_off, lens, dst, dst_off, dst_cap)
    reps = max(1, int(seconds / max(secs, 1e-3)))
    secs, out = cb.run("decompress", cores, reps, src, src_off, lens, dst, dst_off, dst_cap)
    assert (out == BLOCK).all(), "CPU baseline decode failed"
    assert np.array_equal(dst.reshape(n, BLOCK), host_blocks[:n]), "CPU baseline output mismatch"
    val = n * reps * BLOCK / secs / GIB
    res = {"value": round(val, 3), "unit": "GiB/s", "cores": cores, "kind": cb.kind,
           "cores_note": "this process's CPU share (min of its affinity and OMP_NUM_THREADS, 16 on the GPU box)",
           "sample": f"LZ4_decompress_safe, {n} x 64 KiB silesia-like blocks x {reps} reps "
                     f"({secs:.1f} s, {cores} pthreads, one contiguous slice each)"}
    # the same decode on one core (all cores and 1 core), ~3 s
    n1 = max(1, n // 8)
    s1, _ = cb.run("decompress", 1, 1, src, src_off[:n1], lens[:n1], dst, dst_off[:n1], dst_cap[:n1])
    r1 = max(1, int(3.0 / max(s1, 1e-3)))
    s1, _ = cb.run("decompress", 1, r1, src, src_off[:n1], lens[:n1], dst, dst_off[:n1], dst_cap[:n1])
    res["single_core_value"] = round(n1 * r1 * BLOCK / s1 / GIB, 3)
    # LZ4_compress_default (the config-3 parse the GPU's ratio is compared to), all cores, ~5 s
    raw = np.ascontiguousarray(host_blocks[:n]).reshape(-1)
    r_off = np.arange(n, dtype=np.int64) * BLOCK
    r_len = np.full(n, BLOCK, dtype=np.int32)
    cstride = 65824
    cdst = np.empty(n * cstride, dtype=np.uint8)
    c_off = np.arange(n, dtype=np.int64) * cstride
    c_cap = np.full(n, cstride, dtype=np.int32)
    sc, outc = cb.run("compress", cores, 1, raw, r_off, r_len, cdst, c_off, c_cap)
    rc = max(1, int(5.0 / max(sc, 1e-3)))
    sc, outc = cb.run("compress", cores, rc, raw, r_off, r_len, cdst, c_off, c_cap)
    assert (outc > 0).all(), "CPU baseline compress failed"
    res["compress_value"] = round(n * rc * BLOCK / sc / GIB, 3)
    res["compress_sample"] = f"LZ4_compress_default, same {n} blocks x {rc} reps ({sc:.1f} s, {cores} pthreads)"
    return res


def frame_cpu_reference(sample: bytes) -> dict | None:
    """The reference's own LZ4F_compressFrame / LZ4F_decompress (oracle/_ref,
    compiled from /root/reference/lz4libs) on ONE host thread over a sample of
    config 4's input: 4 MiB independent blocks, content checksum, level 0 --
    the rate the drop-in lz4.frame calls replace.  None when
    the reference build is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O   # test/bench infrastructure only
    if not os.path.exists(O.REF_SO):
        return None
    ref = O.Reference()
    t = time.perf_counter()
    fr = ref.compress_frame(sample, block_size_id=7, linked=False, content_checksum=True)
    tc = time.perf_counter() - t
    dst = np.empty(len(sample) + 64, dtype=np.uint8)
    t = time.perf_counter()
    got = ref.decompress_frame_into(fr, dst)
    td = time.perf_counter() - t
    assert got == len(sample) and dst[:got].tobytes() == sample, "reference frame round trip failed"
    return {"compress_gib_s": round(len(sample) / tc / GIB, 3), "decompress_gib_s": round(len(sample) / td / GIB, 3),
            "threads": 1, "kind": "reference", "ratio": round(len(sample) / len(fr), 4),
            "sample": f"LZ4F_compressFrame / LZ4F_decompress, first {len(sample) >> 20} MiB of the config-4 input, "
                      "4 MiB independent blocks, content checksum, one call each on one thread"}


def config5(src, n, world, rank, dev, wave_blocks, waves, strong_total):
    """BASELINE config 5: 256 M x 64 KiB = 16 TiB cannot be
    device-resident, so every rank compresses its share in waves of
    `wave_blocks` over a resident working set (the rank's generated blocks,
    a different window of them each wave when the wave is smaller), each
    wave compacted and gathered at rank 0 over RCCL (lz4._dist), which
    consumes every page (XXH32 of every block, LZ4F's block checksum) -- the
    gather of wave k runs beside the compression of wave k+1.  Weak scaling:
    `waves` waves per rank (32 x 1 M at 8 ranks = the stated 256 M job);
    strong scaling: `strong_total` blocks over all ranks.  Parallel-parse
    compressor (config 3's kernel)."""
    from lz4._dist import compress_gather_waves
    bw = min(wave_blocks, n)
    cap = N.compress_bound(BLOCK)
    cap16 = (cap + 15) // 16 * 16
    base_off = torch.arange(bw, dtype=torch.int64, device=dev) * BLOCK
    src_len = torch.full((bw,), BLOCK, dtype=torch.int32, device=dev)
    slots = torch.empty(bw * cap16, dtype=torch.uint8, device=dev)
    slot_off = torch.arange(bw, dtype=torch.int64, device=dev) * cap16
    slot_cap = torch.full((bw,), cap, dtype=torch.int32, device=dev)
    lens = [torch.empty(bw, dtype=torch.int32, device=dev) for _ in range(2)]
    # compacted waves: sized for a ratio >= 1.5 (silesia-like is ~1.9); a wave
    # that does not fit fails the run below instead of overflowing
    comp_cap = bw * BLOCK * 2 // 3
    comp = [torch.empty(comp_cap, dtype=torch.uint8, device=dev) for _ in range(2)]
    windows = max(1, n // bw)
    digest = torch.zeros(1, dtype=torch.int64, device=dev)
    overflow = torch.zeros(1, dtype=torch.int64, device=dev)
    sums = torch.empty(8192, dtype=torch.int32, device=dev)
    page_blocks = 4096

    def compress_wave(w):
        so = base_off + ((w % windows) * bw) * BLOCK
        ln = lens[w & 1]
        N.launch_compress(src, so, src_len, slots, slot_off, slot_cap, ln, bw, N.PARSE_PARALLEL, 1)
        offs = N.exclusive_scan(ln)
        # capacity check on the device: a too-large wave is compacted to zero
        # blocks (its lengths zeroed) and counted, never written past comp
        over = offs[bw] > comp_cap
        ln.masked_fill_(over, 0)
        offs.masked_fill_(over, 0)
        overflow.add_(over)
        N.gather(slots, slot_off, ln, comp[w & 1], offs, bw)
        return comp[w & 1], ln

    def consume(w, r, first, buf, blens):
        k = blens.numel()
        offs = N.exclusive_scan(blens)
        N.launch_xxh32_batch(buf, offs, blens.to(torch.int64), 0, sums, k)
        digest.add_(sums[:k].to(torch.int64).sum())

    def run(nw):
        box = {}

        def go():
            box["st"] = compress_gather_waves(compress_wave, nw, root=0, consume=consume, page_blocks=page_blocks)

        wall, _ = time_kernel(go, 1, 0, world)
        st = box["st"]
        if int(overflow.item()):
            raise SystemExit("config 5: a wave did not fit its compaction buffer")
        res = {"waves_per_rank": nw, "blocks_per_rank": nw * bw, "total_blocks": world * nw * bw,
               "seconds": round(wall, 3), "aggregate_gib_s": round(world * nw * bw * BLOCK / wall / GIB, 2),
               "ratio": round(nw * bw * BLOCK / max(st["comp_bytes"], 1), 4),
               "host_waits_per_wave": st["host_waits"] // max(1, nw)}
        g = torch.tensor([st["gathered_bytes"]], dtype=torch.int64, device=dev)
        if world > 1:
            torch.distributed.all_reduce(g)
        res["root_consumed_gb_s"] = round(int(g) / wall / 1e9, 2)
        res["pages_at_root"] = st["pages"] if rank == 0 else None
        return res

    # warm the path (allocations, RCCL peer connections) with one wave
    run(1)
    out = {"wave_blocks_per_rank": bw, "block_size": BLOCK, "parse": "parallel (LZ4M_PARSE_PARALLEL)",
           "gather": ("rank 0 over RCCL (isend/irecv pages of %d blocks), overlapped with the next wave"
                      % page_blocks) if world > 1 else "none (1 rank); rank 0 consumes its own pages",
           "root_consumer": "XXH32 of every gathered block (lz4m_xxh32_batch), one page at a time",
           "weak": run(waves)}
    sw = max(1, strong_total // (world * bw))
    out["strong"] = dict(out["weak"], same_run_as_weak=True) if sw == waves else run(sw)
    out["strong"]["total_blocks_fixed"] = strong_total
    out["stated_config_fraction"] = round(world * waves * bw / float(1 << 28), 4)
    del slots, comp
    return out


def config1(n_blocks: int, dev) -> dict:
    """BASELINE config 1: the lz4.block.compress / decompress round trip on
    n x 64 KiB random blocks (random.Random(12345)), through
    the per-call drop-in API and through the batched host API, beside the
    reference lz4libs (oracle/_ref) on 1 host thread and on all of them."""
    import random
    import lz4.block as LB
    rnd = random.Random(12345)
    blocks = [rnd.randbytes(BLOCK) for _ in range(n_blocks)]
    tot = n_blocks * BLOCK
    LB.decompress(LB.compress(blocks[0]))   # warm the staging buffers
    t0 = time.perf_counter()
    comp = [LB.compress(b) for b in blocks]
    t1 = time.perf_counter()
    back = [LB.decompress(c) for c in comp]
    t2 = time.perf_counter()
    assert back == blocks, "config 1 round trip failed"
    # batched: one untimed call of each (the first grows the pinned and
    # device staging buffers to the batch), then the median of three
    LB.decompress_many(LB.compress_many(blocks))
    tc, td = [], []
    for _ in range(3):
        ta = time.perf_counter()
        cm = LB.compress_many(blocks)
        tb = time.perf_counter()
        bm = LB.decompress_many(cm)
        tc.append(tb - ta)
        td.append(time.perf_counter() - tb)
        assert bm == blocks and cm == comp, "config 1 batched round trip failed"
        del cm, bm
    t3, t4 = 0.0, sorted(tc)[1]
    t5 = t4 + sorted(td)[1]
    res = {"blocks": n_blocks, "data": "random.Random(12345).randbytes(65536) per block",
           "per_call_compress_us": round((t1 - t0) / n_blocks * 1e6, 1),
           "per_call_decompress_us": round((t2 - t1) / n_blocks * 1e6, 1),
           "per_call_roundtrip_gib_s": round(tot / (t2 - t0) / GIB, 3),
           "batched_compress_gib_s": round(tot / (t4 - t3) / GIB, 3),
           "batched_decompress_gib_s": round(tot / (t5 - t4) / GIB, 3),
           "batched_roundtrip_gib_s": round(tot / (t5 - t3) / GIB, 3),
           "batched_note": "compress_many / decompress_many of the whole list, median of 3 after one untimed call"}
    # reference lz4libs on the host cores (LZ4_compress_default is byte-identical
    # to lz4.block.compress on random data)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O   # test/bench infrastructure only
    cb = O.CpuBench()
    raw = np.frombuffer(b"".join(blocks), dtype=np.uint8)
    r_off = np.arange(n_blocks, dtype=np.int64) * BLOCK
    r_len = np.full(n_blocks, BLOCK, dtype=np.int32)
    cstride = 65824
    cdst = np.empty(n_blocks * cstride, dtype=np.uint8)
    c_off = np.arange(n_blocks, dtype=np.int64) * cstride
    c_cap = np.full(n_blocks, cstride, dtype=np.int32)
    dst = np.empty(n_blocks * BLOCK, dtype=np.uint8)
    cores = host_threads()
    for th in sorted({1, cores}):
        sc, outc = cb.run("compress", th, 3, raw, r_off, r_len, cdst, c_off, c_cap)
        sd, outd = cb.run("decompress", th, 3, cdst, c_off, outc.astype(np.int32), dst, r_off, r_len)
        assert (outd == BLOCK).all()
        key = "ref_1thread" if th == 1 else f"ref_{th}threads"
        res[key] = {"compress_gib_s": round(3 * tot / sc / GIB, 3), "decompress_gib_s": round(3 * tot / sd / GIB, 3),
                    "roundtrip_gib_s": round(3 * tot / (sc + sd) / GIB, 3), "kind": cb.kind}
    return res


def decoder_src_sha() -> str:
    """Identity of the decoder kernels that profiles/pmc_decompress.json
    must have been measured on (roofline.traffic is reported only on a match)."""
    h = hashlib.sha256()
    for f in ("lz4m_rows.hip", "lz4m_rows.h", "lz4m_decompress.hip", "lz4m_common.h"):
        with open(os.path.join(ROOT, "python-lz4_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--blocks", type=int, default=1 << 20, help="64 KiB blocks per GPU (config 2: 1M)")
    ap.add_argument("--pool", type=int, default=4096, help="unique host-generated blocks per rank")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-compress", action="store_true")
    ap.add_argument("--random-blocks", type=int, default=1 << 17, help="blocks of the random-data extra line")
    ap.add_argument("--frame-gib", type=int, default=8,
                    help="config 4: GiB of input in one LZ4 frame of 4 MiB independent blocks + content checksum; 0 = skip")
    ap.add_argument("--e2e-blocks", type=int, default=1 << 18,
                    help="blocks of the host-to-host (PCIe-inclusive) extra line; 0 = skip")
    ap.add_argument("--c5-wave-blocks", type=int, default=1 << 20,
                    help="config 5: 64 KiB blocks per rank per wave (compressed, compacted, gathered at rank 0)")
    ap.add_argument("--c5-waves", type=int, default=32,
                    help="config 5 weak scaling: waves per rank (32 x 1 M at 8 GPUs = the stated 256 M blocks)")
    ap.add_argument("--c5-total", type=int, default=1 << 25,
                    help="config 5 strong scaling: blocks in total over all ranks (32 M); 0 = skip config 5")
    ap.add_argument("--c1-blocks", type=int, default=1000,
                    help="config 1: random 64 KiB blocks through the per-call lz4.block API; 0 = skip")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # one process per GPU: start the launcher as a child (nothing has
        # touched the GPU in this process) and exit with its status
        s0 = socket.socket()
        s0.bind(("127.0.0.1", 0))
        port = s0.getsockname()[1]
        s0.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        raise SystemExit(subprocess.call(cmd))
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one process per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # RCCL on high-priority streams: config 5's gather shares the GPU with
        # compression kernels
        opts = torch.distributed.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        torch.distributed.init_process_group("nccl", device_id=dev, pg_options=opts)
    N.lib()

    n = args.blocks
    log(f"[bench] rank {rank}/{world}: generating {n} x 64 KiB silesia-like blocks (pool {args.pool})")
    t_gen = time.perf_counter()
    src = make_batch(n, args.pool, "silesia", seed=2026 + rank, dev=dev)
    log(f"[bench] data ready in {time.perf_counter() - t_gen:.1f}s")

    # ---- compress (config 3): parallel-parse compressor, ratio vs LZ4_compress_default ----
    src_off, src_len, slots, slot_off, slot_cap, out_len = compress_all(src, n, N.PARSE_PARALLEL, dev)
    dst = torch.empty(n * BLOCK, dtype=torch.uint8, device=dev)
    dst_off = torch.arange(n, dtype=torch.int64, device=dev) * BLOCK
    dst_cap = torch.full((n,), BLOCK, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)

    def do_pcompress():
        N.launch_compress(src, src_off, src_len, slots, slot_off, slot_cap, out_len, n, N.PARSE_PARALLEL, 1)

    c3 = {}
    if not args.no_compress:
        c_wall, c_ev = time_kernel(do_pcompress, max(1, args.steps // 2), 1, world)
        assert int((out_len <= 0).sum()) == 0, "parallel compress failed on some block"
        par_total = int(out_len.to(torch.int64).sum())
        # validity at full size: our decoder (bit-exact to LZ4_decompress_safe)
        # must restore every block
        N.launch_decompress(slots, slot_off, out_len, dst, dst_off, dst_cap, status, n, src_bytes=par_total)
        assert bool((status == BLOCK).all()) and torch.equal(dst, src), "parallel-parse blocks do not round-trip"
        c3 = {"compress_gib_s": round(world * n * BLOCK / (c_wall / max(1, args.steps // 2)) / GIB, 2),
              "compress_kernel_ms": round(c_ev * 1e3, 3),
              "compress_ratio": round(n * BLOCK / par_total, 4),
              "compress_algo_gbs": round((n * BLOCK + par_total) / c_ev / 1e9, 1),
              "compress_parse": "parallel, 12-bit hash table (LZ4M_PARSE_PARALLEL)"}
        # the same parse with the reference's 13-bit table (LZ4M_PARSE_PARALLEL_HQ)
        h_wall, h_ev = time_kernel(lambda: N.launch_compress(src, src_off, src_len, slots, slot_off, slot_cap,
                                                             out_len, n, N.PARSE_PARALLEL_HQ, 1), 1, 0, world)
        assert int((out_len <= 0).sum()) == 0, "parallel (HQ) compress failed on some block"
        c3["compress_hq_gib_s"] = round(world * n * BLOCK / h_wall / GIB, 2)
        c3["compress_hq_ratio"] = round(n * BLOCK / int(out_len.to(torch.int64).sum()), 4)

    log("[bench] parallel compress done")
    # ---- decode input: the exact LZ4_compress_default parse (byU16/hash4) ----
    def do_compress_exact():
        N.launch_compress(src, src_off, src_len, slots, slot_off, slot_cap, out_len, n, N.TABLE_U16_HASH4, 1)

    x_wall, x_ev = time_kernel(do_compress_exact, 1, 0, world)
    assert int((out_len <= 0).sum()) == 0, "compress failed on some block"
    comp_total = int(out_len.to(torch.int64).sum())
    ratio = n * BLOCK / comp_total
    if c3:
        c3["compress_ratio_vs_default"] = round(c3["compress_ratio"] / ratio, 4)
        c3["compress_hq_ratio_vs_default"] = round(c3["compress_hq_ratio"] / ratio, 4)
    c3["compress_exact_gib_s"] = round(world * n * BLOCK / x_wall / GIB, 2)

    # compact into one contiguous compressed buffer (what a file/socket holds)
    offs = N.exclusive_scan(out_len)
    comp = torch.empty(comp_total, dtype=torch.uint8, device=dev)
    N.gather(slots, slot_off, out_len, comp, offs, n)
    c_off = offs[:n].clone()
    c_len = out_len.clone()
    comp_sample = None
    if runs_cpu_baseline(rank, args.no_cpu):   # cpu_baseline at every N (rank 0, after the timed regions)
        k = min(n, 16384)
        comp_host_np = comp[: int(offs[k])].cpu().numpy()
        oh = offs[: k + 1].cpu().numpy()
        comp_sample = [comp_host_np[oh[i]:oh[i + 1]].tobytes() for i in range(k)]
    del slots, slot_off, slot_cap
    torch.cuda.empty_cache()

    log("[bench] exact compress done")
    # ---- decompress (config 2, headline) ----
    def do_decompress():
        N.launch_decompress(comp, c_off, c_len, dst, dst_off, dst_cap, status, n)

    d_wall, d_ev = time_kernel(do_decompress, args.steps, args.warmup, world)
    ok_status = bool((status == BLOCK).all())
    ok_bytes = bool(torch.equal(dst, src))
    if not (ok_status and ok_bytes):
        raise SystemExit(f"decompress verification failed: status_ok={ok_status} bytes_ok={ok_bytes}")

    extra = {}
    # ---- extra: a mid-size batch of the same blocks (65 536), which goes to the
    # a mid-size batch through the default dispatch (the row decoder from 32 768 blocks)
    nm = min(65536, n)
    dst[: nm * BLOCK].zero_()

    def do_mid():
        N.launch_decompress(comp, c_off[:nm], c_len[:nm], dst, dst_off[:nm], dst_cap[:nm], status[:nm], nm)

    m_wall, m_ev = time_kernel(do_mid, args.steps, 1, world)
    if not (bool((status[:nm] == BLOCK).all()) and torch.equal(dst[: nm * BLOCK], src[: nm * BLOCK])):
        raise SystemExit("mid-size batch decompress verification failed")
    extra["decompress_mid_batch"] = {"blocks": nm, "gib_s": round(world * nm * BLOCK / (m_wall / args.steps) / GIB, 2),
                                     "kernel_ms": round(m_ev * 1e3, 3),
                                     "kernel": "default dispatch: row decoder (>= 32 768 blocks)"}

    # ---- extra: end to end from pinned host memory (PCIe-inclusive) ----
    # lz4.block.decompress_host: chunks of 16 384 blocks pipelined over three
    # streams (copy in || decode || copy out)
    if args.e2e_blocks > 0:
        import lz4.block as LB
        # every rank pins its own host buffers (24 GiB at 256 K blocks): at
        # N > 1 a quarter of that per rank keeps a node's pinned memory modest
        ne = min(args.e2e_blocks if world == 1 else args.e2e_blocks // 4, n)
        e_comp_bytes = int(c_off[ne - 1]) + int(c_len[ne - 1]) if ne < n else comp_total
        h_comp = torch.empty(e_comp_bytes, dtype=torch.uint8, pin_memory=True)
        h_comp.copy_(comp[:e_comp_bytes])
        h_out = torch.empty(ne * BLOCK, dtype=torch.uint8, pin_memory=True)
        h_coff, h_clen = c_off[:ne].cpu(), c_len[:ne].cpu()
        h_ooff = torch.arange(ne, dtype=torch.int64) * BLOCK
        h_ocap = torch.full((ne,), BLOCK, dtype=torch.int32)
        box = {}

        def do_e2e():
            box["st"] = LB.decompress_host(h_comp, h_coff, h_clen, h_out, h_ooff, h_ocap, chunk_blocks=16384)

        e_wall, _ = time_kernel(do_e2e, max(1, args.steps // 2), 1, world)
        assert bool((box.pop("st") == BLOCK).all()), "end-to-end decode failed"
        assert torch.equal(h_out[: 4 * BLOCK], src[: 4 * BLOCK].cpu()) and \
            torch.equal(h_out[-4 * BLOCK:], src[(ne - 4) * BLOCK: ne * BLOCK].cpu())
        extra["end_to_end_host_gib_s"] = round(world * ne * BLOCK / (e_wall / max(1, args.steps // 2)) / GIB, 2)
        extra["end_to_end_blocks"] = ne
        extra["end_to_end_note"] = "pinned host bytes -> H2D -> decode -> D2H, 16 384-block chunks pipelined"
        del h_comp, h_out

    # ---- extra: incompressible (random) blocks ----
    if args.random_blocks > 0:
        del dst
        torch.cuda.empty_cache()
        nr = min(args.random_blocks, n)
        rsrc = make_batch(nr, min(args.pool, nr), "random", seed=99 + rank, dev=dev)
        r_off, r_len, r_slots, r_soff, r_scap, r_olen = compress_all(rsrc, nr, N.TABLE_U16_HASH4, dev)
        N.launch_compress(rsrc, r_off, r_len, r_slots, r_soff, r_scap, r_olen, nr, N.TABLE_U16_HASH4, 1)
        rdst = torch.empty(nr * BLOCK, dtype=torch.uint8, device=dev)
        rst = torch.empty(nr, dtype=torch.int32, device=dev)

        def do_rand():
            N.launch_decompress(r_slots, r_soff, r_olen, rdst, dst_off[:nr], dst_cap[:nr], rst, nr)

        r_wall, r_ev = time_kernel(do_rand, args.steps, 1, world)
        assert bool(torch.equal(rdst, rsrc)), "random-data round trip failed"
        r_cbytes = int(r_olen.to(torch.int64).sum())
        extra["decompress_random_gib_s"] = round(world * nr * BLOCK / (r_wall / args.steps) / GIB, 2)
        extra["decompress_random_kernel_gbs"] = round((r_cbytes + nr * BLOCK) / r_ev / 1e9, 1)
        del rsrc, rdst, r_slots, rst

    # ---- extra: measured HBM copy bandwidth (report the spec and a copy) ----
    cb = 8 << 30
    ca = torch.empty(cb, dtype=torch.uint8, device=dev)
    cbuf = torch.empty(cb, dtype=torch.uint8, device=dev)
    c_wall, c_ev = time_kernel(lambda: cbuf.copy_(ca), 3, 1, world)
    extra["hbm_copy_gb_s"] = round(2 * cb / c_ev / 1e9, 1)
    extra["hbm_copy_note"] = "device-to-device copy of 8 GiB (read + write bytes / time), torch copy_"
    del ca, cbuf
    torch.cuda.empty_cache()

    log("[bench] decode done")
    # ---- config 5: compress in waves, gather every wave at rank 0 (RCCL) ----
    # (after config 2's buffers are gone: a 1 M-block wave needs its bound-sized
    # slots and two compaction buffers beside the 64 GiB working set)
    del comp
    dst = None
    torch.cuda.empty_cache()
    if args.c5_total > 0:
        extra["config5"] = config5(src, n, world, rank, dev, args.c5_wave_blocks, args.c5_waves, args.c5_total)
        torch.cuda.empty_cache()
        log("[bench] config 5 done")
    # ---- extra: config 4, one frame of 4 MiB independent blocks + XXH32 content checksum ----
    if args.frame_gib > 0:
        from lz4.frame._frame import _compress_frame
        dst = dst_off = dst_cap = None
        torch.cuda.empty_cache()
        FB = 4 << 20
        L = args.frame_gib << 30
        fsrc = make_batch(L // BLOCK, min(args.pool, L // BLOCK), "silesia", seed=77 + rank, dev=dev)
        kw = dict(block_size=7, block_linked=False, parse="parallel")
        box = {}

        def do_frame():
            box["f"] = _compress_frame(fsrc, L, content_checksum=True, **kw)

        def do_frame_nochk():
            box["g"] = _compress_frame(fsrc, L, content_checksum=False, **kw)

        hsum = torch.empty(1, dtype=torch.int32, device=dev)
        f_wall, _ = time_kernel(do_frame, 1, 1, world)
        g_wall, _ = time_kernel(do_frame_nochk, 1, 0, world)
        h_wall, h_ev = time_kernel(lambda: N.launch_xxh32_long(fsrc, L, 0, hsum), 1, 0, world)
        # the content checksum as lz4.frame runs it: a host core over pipelined PCIe copies
        hb = {}
        hh_wall, _ = time_kernel(lambda: hb.__setitem__("h", N.xxh32_of_device(fsrc, L)), 1, 0, world)
        assert hb["h"] == int(hsum.item()) & 0xFFFFFFFF, "host and device content XXH32 differ"
        # the same 8 GiB framed with the exact parse (LZ4F_compressFrame's blocks): the ratio reference
        ex_frame, _ = _compress_frame(fsrc, L, content_checksum=False, block_size=7, block_linked=False,
                                      parse="exact")
        ex_len = int(ex_frame.numel())
        del ex_frame
        frame, meta = box.pop("f")
        frame_nc, _ = box.pop("g")
        box.clear()
        # validate: decode the frame on the device (record walk, batched block
        # decode, content checksum check), compare with the input
        import lz4.frame as F
        assert not bool(meta["raw"].any()), "unexpected stored-raw block"
        nbk = L // FB
        # one untimed call first, as for the compress side: the first call also
        # allocates the output slots and pinned staging
        # (median of three timed calls after the untimed one)
        fd_wall, fd_all = time_median(lambda: box.__setitem__("d", F.decompress_device(frame)), 3, 1, world)
        fd_s = fd_wall
        assert torch.equal(box.pop("d"), fsrc), "config-4 frame does not round-trip"
        fn_wall, fn_all = time_median(lambda: box.__setitem__("d", F.decompress_device(frame_nc)), 3, 1, world)
        assert torch.equal(box.pop("d"), fsrc), "config-4 frame (no content checksum) does not round-trip"
        del frame_nc
        assert int(frame[-4:].view(torch.int32).item()) == int(hsum.item()), "content checksum field mismatch"
        extra["frame4m"] = {
            "input_gib": args.frame_gib, "blocks": nbk, "ratio": round(L / frame.numel(), 4),
            "compress_frame_gib_s": round(world * L / f_wall / GIB, 2),
            "compress_frame_no_content_checksum_gib_s": round(world * L / g_wall / GIB, 2),
            "ratio_exact_parse": round(L / ex_len, 4),
            "ratio_vs_exact_parse": round((L / frame.numel()) / (L / ex_len), 4),
            "content_xxh32_host_gb_s": round(L / hh_wall / 1e9, 3),
            "content_xxh32_gpu_gb_s": round(L / h_ev / 1e9, 3),
            "decompress_frame_gib_s": round(world * L / fd_s / GIB, 2),
            "decompress_frame_no_content_checksum_gib_s": round(world * L / fn_wall / GIB, 2),
            "decompress_frame_samples_s": [round(x, 4) for x in fd_all],
            "decompress_frame_no_content_checksum_samples_s": [round(x, 4) for x in fn_all],
            "note": "content XXH32 is one serial stream (SURVEY 0.5): a host core hashes the bytes streamed back "
                    "over PCIe while the device compresses / decodes (lz4m_xxh32_host_*)"}
        # the drop-in call itself: lz4.frame.compress / decompress on the caller's
        # host bytes -- the exact parse (blocks byte-identical to LZ4F_compressFrame's), 4 MiB
        # independent blocks, content checksum (_frame.c:226-228 -> lz4frame.c:475-515; decode
        # lz4frame.c:1556-2058) -- host bytes in, host bytes out, PCIe included
        if world == 1:
            hb = fsrc.cpu().numpy().tobytes()
            kw4 = dict(block_size=F.BLOCKSIZE_MAX4MB, block_linked=False, content_checksum=True)
            F.decompress(F.compress(hb[: 64 << 20], **kw4))   # warm-up: kernels, pinned staging
            dbox = {}
            di_wall, _ = time_kernel(lambda: dbox.__setitem__("f", F.compress(hb, **kw4)), 1, 0, world)
            fr_h = dbox.pop("f")
            do_wall, _ = time_kernel(lambda: dbox.__setitem__("d", F.decompress(fr_h)), 1, 0, world)
            assert dbox.pop("d") == hb, "drop-in config-4 frame does not round-trip"
            assert len(fr_h) == ex_len + 4, "drop-in frame size differs from the exact-parse frame (+ content checksum)"
            extra["frame4m"]["dropin_compress_gib_s"] = round(L / di_wall / GIB, 2)
            extra["frame4m"]["dropin_decompress_gib_s"] = round(L / do_wall / GIB, 2)
            extra["frame4m"]["dropin_note"] = ("lz4.frame.compress(bytes, block_size=BLOCKSIZE_MAX4MB, block_linked=False, "
                                               "content_checksum=True) and lz4.frame.decompress of its result: host bytes "
                                               "in and out, exact parse, PCIe and the serial content XXH32 included")
            if runs_cpu_baseline(rank, args.no_cpu):
                extra["frame4m"]["cpu_reference"] = frame_cpu_reference(hb[: 1 << 30])
            del hb, fr_h
        # lz4.frame.compress's defaults (64 KiB linked blocks, the exact parse, byte-identical to the
        # reference): speculative-parallel linked compression on a 256 MiB sample of the same input
        LS = min(L, 256 << 20)
        dl = {}
        dl_wall, _ = time_kernel(lambda: dl.__setitem__("f", _compress_frame(fsrc, LS)), 3, 1, world)
        dl_wall /= 3
        dfr = dl.pop("f")[0]
        assert torch.equal(F.decompress_device(dfr), fsrc[:LS]), "default linked frame does not round-trip"
        extra["frame4m"]["compress_frame_default_linked_gib_s"] = round(world * LS / dl_wall / GIB, 3)
        extra["frame4m"]["compress_frame_default_linked_sample_mib"] = LS >> 20
        extra["frame4m"]["compress_frame_default_linked_passes"] = int(N.lib().lz4m_compress_linked_passes())
        extra["frame4m"]["compress_frame_default_linked_ratio"] = round(LS / dfr.numel(), 4)
        del dfr, fsrc, frame, meta
        torch.cuda.empty_cache()

    # ---- config 1: the per-call drop-in path (host bytes in, host bytes out) ----
    if args.c1_blocks > 0 and world == 1 and not args.no_cpu:
        extra["config1"] = config1(args.c1_blocks, dev)
        log("[bench] config 1 done")

    # ---- report ----
    d_step = d_wall / args.steps
    value = aggregate_gib_s(world, n, BLOCK, d_wall, args.steps)
    algo_bytes = comp_total + n * BLOCK          # per launch: read compressed + write decoded
    achieved = algo_bytes / d_ev / 1e9           # GB/s, from HIP events on the launch stream
    # HBM bytes per launch of the decoder from the committed PMC summary of
    # this same command (tools/pmc_bench.sh -> profiles/pmc_decompress.json),
    # used only when it was measured on this configuration
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_decompress.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if (pmc.get("blocks") == n and pmc.get("pool") == args.pool
                    and pmc.get("decoder_src_sha") == decoder_src_sha()):
                traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    res = {
        "metric": "GiB/s uncompressed, device-resident, 64 KiB blocks (decompress; compress)",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(d_step * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (silesia-like mix, lz4/_synth.py; Silesia unavailable offline)",
        "config": {"workload": "config 2: decompress 1M x 64 KiB blocks, device-resident, LZ4_compress_default input",
                   "blocks_per_gpu": n, "block_size": BLOCK, "ratio": round(ratio, 4),
                   "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic},
        "decompress_kernel_ms": round(d_ev * 1e3, 3),
        "decompress_read_gbs": round(comp_total / d_ev / 1e9, 1),
        "compress": c3,
        "extra": extra,
    }
    if comp_sample is not None:
        host_blocks = src[: len(comp_sample) * BLOCK].view(-1, BLOCK).cpu().numpy()
        res["cpu_baseline"] = cpu_baseline(host_blocks, comp_sample)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
