"""Multi-rank path on CPU (gloo, world size 2 and 3): contiguous sharding and
the gather of compressed shards at a root (lz4/_dist.py).
The GPU run uses the same code over RCCL (backend "nccl")."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lz4._dist import gather_compressed, shard_range


def test_shard_range_partitions():
    for n in [0, 1, 7, 64, 1000, 1 << 20]:
        for world in [1, 2, 3, 8]:
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_blocks(rank, nblocks):
    g = torch.Generator().manual_seed(100 + rank)
    lens = torch.randint(1, 300, (nblocks,), generator=g, dtype=torch.int32)
    data = torch.randint(0, 256, (int(lens.sum()),), generator=g, dtype=torch.uint8)
    return data, lens


def _worker(rank, world, port, counts, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data, lens = _shard_blocks(rank, counts[rank])
        buf, off, got_lens = gather_compressed(data, lens, root=root)
        if rank == root:
            parts = [_shard_blocks(r, counts[r]) for r in range(world)]
            exp = torch.cat([p[0] for p in parts])
            exp_lens = torch.cat([p[1] for p in parts])
            ok = torch.equal(buf, exp) and torch.equal(got_lens, exp_lens)
            # offsets index every block
            ok = ok and int(off[-1]) + int(got_lens[-1]) == buf.numel() if got_lens.numel() else ok
            q.put(("root", bool(ok)))
        else:
            q.put(("peer", buf is None and got_lens.numel() == sum(counts)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,counts,root", [(2, [5, 9], 0), (2, [0, 4], 1), (3, [3, 0, 6], 0)])
def test_gather_compressed_gloo(world, counts, root):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = [q.get(timeout=10) for _ in range(world)]
    assert all(ok for _, ok in res), res


def _wave_worker(rank, world, port, waves, q):
    """The config-5 wave driver with a CPU stand-in for the compressor: each
    wave yields this rank's chunk of seeded variable-length 'blocks'."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lz4._dist import compress_gather_waves
    try:
        def wave(w):
            return _shard_blocks(rank * 100 + w, 3 + (w + rank) % 4)

        got = {}

        def consume(w, buf, off, lens):
            got[w] = (buf.clone(), off.clone(), lens.clone())

        for overlap in (True, False):
            got.clear()
            st = compress_gather_waves(wave, waves, root=0, overlap=overlap, consume=consume)
            if rank == 0:
                ok = sorted(got) == list(range(waves))
                for w in range(waves):
                    parts = [_shard_blocks(r * 100 + w, 3 + (w + r) % 4) for r in range(world)]
                    buf, off, lens = got[w]
                    ok = ok and torch.equal(buf, torch.cat([p[0] for p in parts]))
                    ok = ok and torch.equal(lens, torch.cat([p[1] for p in parts]))
                    ok = ok and torch.equal(off[1:], torch.cumsum(lens[:-1].to(torch.int64), 0))
                ok = ok and st["gathered_bytes"] == sum(int(got[w][0].numel()) for w in range(waves))
                q.put(("root", bool(ok)))
            else:
                q.put(("peer", st["waves"] == waves and not got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,waves", [(2, 3), (3, 2)])
def test_wave_driver_gloo(world, waves):
    """compress -> compact -> gather per wave, gathers overlapped with the next
    wave (and not), world size 2 and 3 over gloo: the root receives every
    wave's blocks in rank order with the right index."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wave_worker, args=(r, world, port, waves, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = [q.get(timeout=10) for _ in range(2 * world)]
    assert all(ok for _, ok in res), res
