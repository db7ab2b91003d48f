"""The config-5 wave driver (lz4/_dist.py compress_gather_waves) on the GPU:
world size 1 over the NCCL (= RCCL) backend, the real parallel-parse
compressor and compaction kernels, and the root consuming every page by
decoding it -- the decoded bytes must equal the wave's input bit for bit.
The multi-rank exchange itself is covered over gloo in tests/test_dist.py
(two ranks cannot share one GPU under RCCL)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

from lz4 import _native as N  # noqa: E402
from lz4 import _synth  # noqa: E402

BLOCK = 65536


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("overlap", [True, False])
def test_compress_gather_waves_nccl_world1(gpu, overlap):
    import torch.distributed as dist
    from lz4._dist import compress_gather_waves
    dev = torch.device("cuda", 0)
    kinds = ("silesia", "text", "records", "runs", "random", "markup")
    host = [_synth.blocks(48, k, seed=40 + i) for i, k in enumerate(kinds)]
    src = torch.from_numpy(__import__("numpy").concatenate(host)).to(dev).view(-1)
    nblk = src.numel() // BLOCK                 # 288 blocks, 96 per wave
    bw, waves = 96, 3
    cap = N.compress_bound(BLOCK)
    cap16 = (cap + 15) // 16 * 16
    slots = torch.empty(bw * cap16, dtype=torch.uint8, device=dev)
    slot_off = torch.arange(bw, dtype=torch.int64, device=dev) * cap16
    slot_cap = torch.full((bw,), cap, dtype=torch.int32, device=dev)
    src_len = torch.full((bw,), BLOCK, dtype=torch.int32, device=dev)
    lens = [torch.empty(bw, dtype=torch.int32, device=dev) for _ in range(2)]
    comp = [torch.empty(bw * cap16, dtype=torch.uint8, device=dev) for _ in range(2)]
    assert waves * bw == nblk

    def compress_wave(w):
        so = torch.arange(bw, dtype=torch.int64, device=dev) * BLOCK + w * bw * BLOCK
        N.launch_compress(src, so, src_len, slots, slot_off, slot_cap, lens[w & 1], bw, N.PARSE_PARALLEL, 1)
        offs = N.exclusive_scan(lens[w & 1])
        N.gather(slots, slot_off, lens[w & 1], comp[w & 1], offs, bw)
        return comp[w & 1], lens[w & 1]

    checks, seen = [], []

    def consume(w, r, first, buf, blens):
        # on the gather's side stream: decode the page now, before its memory is reused
        k = blens.numel()
        offs = N.exclusive_scan(blens)
        out = torch.empty(k * BLOCK, dtype=torch.uint8, device=dev)
        st = torch.empty(k, dtype=torch.int32, device=dev)
        N.launch_decompress(buf, offs[:k], blens, out, torch.arange(k, dtype=torch.int64, device=dev) * BLOCK,
                            torch.full((k,), BLOCK, dtype=torch.int32, device=dev), st, k)
        lo = (w * bw + first) * BLOCK
        checks.append(bool((st == BLOCK).all()) and torch.equal(out, src[lo: lo + k * BLOCK]))
        seen.append((w, r, first, k))

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, pg_options=opts)
    try:
        st = compress_gather_waves(compress_wave, waves, root=0, overlap=overlap, consume=consume, page_blocks=40)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert seen == [(w, 0, f, min(40, bw - f)) for w in range(waves) for f in range(0, bw, 40)]
    assert checks and all(checks)
    assert st["blocks"] == nblk and st["gathered_bytes"] == st["comp_bytes"] > 0


def _nccl_world2_worker(rank, port, ring, q):
    """One rank of the world-2 RCCL exchange: rank r compresses its own shard
    (seeded by rank), the root (rank 0) decodes every page it receives and
    checks it against that rank's shard."""
    import numpy as np
    import torch.distributed as dist
    from lz4._dist import compress_gather_waves
    try:
        dev = torch.device("cuda", rank)
        torch.cuda.set_device(dev)
        bw, waves = 24, 3
        shards = [torch.from_numpy(np.concatenate([_synth.blocks(bw * waves // 3, k, seed=60 + 7 * r + i)
                                                   for i, k in enumerate(("silesia", "text", "random"))]))
                  for r in range(2)]
        src = shards[rank].to(dev).view(-1)
        cap = N.compress_bound(BLOCK)
        cap16 = (cap + 15) // 16 * 16
        slots = torch.empty(bw * cap16, dtype=torch.uint8, device=dev)
        slot_off = torch.arange(bw, dtype=torch.int64, device=dev) * cap16
        slot_cap = torch.full((bw,), cap, dtype=torch.int32, device=dev)
        src_len = torch.full((bw,), BLOCK, dtype=torch.int32, device=dev)
        lens = [torch.empty(bw, dtype=torch.int32, device=dev) for _ in range(2)]
        comp = [torch.empty(bw * cap16, dtype=torch.uint8, device=dev) for _ in range(2)]

        def compress_wave(w):
            so = torch.arange(bw, dtype=torch.int64, device=dev) * BLOCK + w * bw * BLOCK
            N.launch_compress(src, so, src_len, slots, slot_off, slot_cap, lens[w & 1], bw, N.PARSE_PARALLEL, 1)
            offs = N.exclusive_scan(lens[w & 1])
            N.gather(slots, slot_off, lens[w & 1], comp[w & 1], offs, bw)
            return comp[w & 1], lens[w & 1]

        want = [s.to(dev).view(-1) for s in shards]
        checks, seen = [], []

        def consume(w, r, first, buf, blens):
            k = blens.numel()
            offs = N.exclusive_scan(blens)
            out = torch.empty(k * BLOCK, dtype=torch.uint8, device=dev)
            st = torch.empty(k, dtype=torch.int32, device=dev)
            N.launch_decompress(buf, offs[:k], blens, out, torch.arange(k, dtype=torch.int64, device=dev) * BLOCK,
                                torch.full((k,), BLOCK, dtype=torch.int32, device=dev), st, k)
            lo = (w * bw + first) * BLOCK
            checks.append(bool((st == BLOCK).all()) and torch.equal(out, want[r][lo: lo + k * BLOCK]))
            seen.append((w, r, first, k))

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
        try:
            compress_gather_waves(compress_wave, waves, root=0, overlap=True, consume=consume, page_blocks=7,
                                  ring=ring)
            torch.cuda.synchronize()
        finally:
            dist.destroy_process_group()
        if rank == 0:
            exp = sorted((w, r, f, min(7, bw - f)) for w in range(waves) for r in range(2) for f in range(0, bw, 7))
            q.put((rank, sorted(seen) == exp and bool(checks) and all(checks), None))
        else:
            q.put((rank, not seen, None))
    except Exception as e:   # reported to the parent, which fails the test
        q.put((rank, False, repr(e)))


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (two ranks cannot share one under RCCL)")
@pytest.mark.parametrize("ring", [1, 2])
def test_compress_gather_waves_nccl_world2(ring):
    """The config-5 exchange over RCCL at world size 2: peers'
    isend of pages into the root's ring of `ring` receive slots per peer, the
    two all_gathers of sizes per wave, and the side-stream ordering, with the
    root decoding every page (3 waves x 24 blocks per rank, pages of 7)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_nccl_world2_worker, args=(r, port, ring, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=120) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(ok for _, ok, _ in res), res
