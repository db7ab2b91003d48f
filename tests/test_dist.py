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
    wave yields this rank's chunk of seeded variable-length 'blocks', padded
    past the blocks' end like a compaction buffer."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lz4._dist import compress_gather_waves
    try:
        def blocks(r, w):
            return _shard_blocks(r * 100 + w, 3 + 2 * ((w + r) % 4))

        def wave(w):
            data, lens = blocks(rank, w)
            return torch.cat([data, torch.full((17,), 0xEE, dtype=torch.uint8)]), lens

        got = {}

        def consume(w, r, first, buf, lens):
            got.setdefault((w, r), []).append((first, buf.clone(), lens.clone()))

        oks = []
        for overlap, page_blocks, ring in ((True, 2, 2), (False, 3, 1), (True, 4096, 4)):
            got.clear()
            st = compress_gather_waves(wave, waves, root=0, overlap=overlap, consume=consume,
                                       page_blocks=page_blocks, ring=ring)
            ok = st["waves"] == waves
            if rank == 0:
                ok = ok and sorted(got) == [(w, r) for w in range(waves) for r in range(world)]
                total = 0
                for (w, r), pages in got.items():
                    data, lens = blocks(r, w)
                    firsts = [f for f, _, _ in pages]
                    ok = ok and firsts == list(range(0, lens.numel(), page_blocks))
                    ok = ok and torch.equal(torch.cat([b for _, b, _ in pages]), data)
                    ok = ok and torch.equal(torch.cat([x for _, _, x in pages]), lens)
                    ok = ok and all(int(x.to(torch.int64).sum()) == b.numel() for _, b, x in pages)
                    total += data.numel()
                ok = ok and st["gathered_bytes"] == total
            else:
                ok = ok and not got and st["comp_bytes"] == sum(int(blocks(rank, w)[1].sum()) for w in range(waves))
            oks.append(bool(ok))
        q.put(("root" if rank == 0 else "peer", all(oks), oks))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,waves", [(2, 3), (3, 2)])
def test_wave_driver_gloo(world, waves):
    """compress -> compact -> paged gather per wave, gathers overlapped with
    the next wave (and not), world size 2 and 3 over gloo, pages of 2, 3 and
    4096 blocks through a ring of 2, 1 and 4 receive buffers: the root
    consumes every rank's blocks of every wave, page by page, with their
    sizes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wave_worker, args=(r, world, port, waves, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = [q.get(timeout=10) for _ in range(world)]
    assert all(r[1] for r in res), res


def test_wave_driver_without_process_group():
    """bench.py at N = 1 starts no process group: the wave driver then runs as
    rank 0 of 1 (no exchange) and the root consumes its own pages."""
    from lz4._dist import compress_gather_waves
    assert not dist.is_initialized()
    waves, page_blocks = 3, 2

    def wave(w):
        data, lens = _shard_blocks(w, 5)
        return torch.cat([data, torch.full((9,), 0xEE, dtype=torch.uint8)]), lens

    got = {}

    def consume(w, r, first, buf, lens):
        got.setdefault(w, []).append((r, first, buf.clone(), lens.clone()))

    for overlap in (True, False):
        got.clear()
        st = compress_gather_waves(wave, waves, root=0, overlap=overlap, consume=consume, page_blocks=page_blocks)
        assert st["waves"] == waves and st["host_waits"] == 2 * waves
        for w in range(waves):
            data, lens = _shard_blocks(w, 5)
            pages = got[w]
            assert [p[1] for p in pages] == list(range(0, lens.numel(), page_blocks))
            assert all(p[0] == 0 for p in pages)
            assert torch.equal(torch.cat([p[2] for p in pages]), data)
            assert torch.equal(torch.cat([p[3] for p in pages]), lens)
        assert st["gathered_bytes"] == st["comp_bytes"] == sum(int(_shard_blocks(w, 5)[1].sum()) for w in range(waves))
