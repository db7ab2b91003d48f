"""CPU tests of lz4m_host_copy (the drop-in frame calls' staging copies,
python-lz4_amd/csrc/lz4m_host_copy.c): bytes and the streamed XXH32 equal a
plain copy and the oracle's hash, for every thread count, from several host
threads at once, and in a forked child after the pool has started."""
import ctypes as C
import os
import threading

import numpy as np
import pytest


def _copy(lib, src, threads, seed=None):
    import lz4._native as N
    dst = np.empty_like(src)
    st = None
    if seed is not None:
        st = N.HostXXH32(seed)
    lib.lz4m_host_copy(dst.ctypes.data_as(C.c_void_p), src.ctypes.data_as(C.c_void_p), src.size, threads,
                       None if st is None else st._st)
    return dst, (st.digest() if st is not None else None)


@pytest.mark.parametrize("n", [0, 1, 4 << 20, (17 << 20) + 3])
@pytest.mark.parametrize("threads", [1, 4, 16])
def test_host_copy_bytes_and_hash(oracle, n, threads):
    import lz4._native as N
    lib = N.lib()
    src = np.random.default_rng(n + threads).integers(0, 256, n, dtype=np.uint8)
    dst, h = _copy(lib, src, threads, seed=7)
    assert np.array_equal(dst, src)
    assert h == oracle.xxh32(src.tobytes(), 7)


def test_host_copy_from_many_threads(oracle):
    import lz4._native as N
    lib = N.lib()
    srcs = [np.random.default_rng(k).integers(0, 256, (6 << 20) + k, dtype=np.uint8) for k in range(6)]
    bad = []

    def work(k):
        for _ in range(3):
            dst, h = _copy(lib, srcs[k], 8, seed=k)
            if not np.array_equal(dst, srcs[k]) or h != oracle.xxh32(srcs[k].tobytes(), k):
                bad.append(k)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not bad


def test_host_copy_in_forked_child():
    import lz4._native as N
    lib = N.lib()
    src = np.random.default_rng(3).integers(0, 256, 8 << 20, dtype=np.uint8)
    dst, _ = _copy(lib, src, 8)   # the pool is running in this process
    assert np.array_equal(dst, src)
    pid = os.fork()
    if pid == 0:   # the child starts its own workers
        d2, _ = _copy(lib, src, 8)
        os._exit(0 if np.array_equal(d2, src) else 1)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0


def _copy_many(lib, srcs, threads, null_empty=True):
    """lz4m_host_copy_many over numpy sources; empty items get NULL pointers
    (as lz4.block.compress_many passes for empty bytes)."""
    dsts = [np.full(len(s), 0xA5, dtype=np.uint8) for s in srcs]
    n = len(srcs)
    D = (C.c_void_p * max(n, 1))()
    S = (C.c_void_p * max(n, 1))()
    L = (C.c_size_t * max(n, 1))()
    for i, (d, s) in enumerate(zip(dsts, srcs)):
        empty = len(s) == 0 and null_empty
        D[i] = None if empty else d.ctypes.data
        S[i] = None if empty else s.ctypes.data
        L[i] = len(s)
    lib.lz4m_host_copy_many(D, S, L, n, threads)
    return dsts


def _rand_items(rng, sizes):
    return [rng.integers(0, 256, int(k), dtype=np.uint8) for k in sizes]


@pytest.mark.parametrize("threads", [1, 2, 3, 16])
@pytest.mark.parametrize("case", ["empty_null", "fewer_than_threads", "skewed", "just_below_4mib",
                                  "just_above_4mib", "one_huge", "zero_items"])
def test_host_copy_many_matches_per_item_copy(case, threads):
    """lz4m_host_copy_many (the packing and unpacking of compress_many /
    decompress_many, lz4m_host_copy.c) equals a per-item copy: empty items
    with NULL pointers, fewer items than threads, heavily skewed sizes, totals
    on both sides of the 4 MiB threading threshold, one item larger than
    total / threads."""
    import lz4._native as N
    lib = N.lib()
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    sizes = {
        "empty_null": [0, 5, 0, 0, 70000, 0, 1, 0] * 40,
        "fewer_than_threads": [3 << 20, 2 << 20],
        "skewed": [1, 2, 3, 9 << 20, 4, 0, 5, 1 << 20, 7, 11],
        "just_below_4mib": [(1 << 20) - 1, 1 << 20, 1 << 20, (1 << 20) - 2],
        "just_above_4mib": [(1 << 20) + 1, 1 << 20, 1 << 20, (1 << 20) + 2],
        "one_huge": [12 << 20] + [100] * 50,
        "zero_items": [],
    }[case]
    srcs = _rand_items(rng, sizes)
    dsts = _copy_many(lib, srcs, threads)
    for s, d in zip(srcs, dsts):
        assert np.array_equal(s, d)


def test_host_copy_many_from_many_threads():
    """Concurrent lz4m_host_copy_many calls from several host threads share
    one pool (calls are serialised inside it) and all copy exactly."""
    import lz4._native as N
    lib = N.lib()
    bad = []

    def work(k):
        rng = np.random.default_rng(100 + k)
        for _ in range(3):
            sizes = rng.integers(0, 1 << 20, 12)
            sizes[rng.integers(0, 12, 3)] = 0
            srcs = _rand_items(rng, sizes)
            for s, d in zip(srcs, _copy_many(lib, srcs, 8)):
                if not np.array_equal(s, d):
                    bad.append(k)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not bad


@pytest.mark.parametrize("as_bytearray", [False, True])
@pytest.mark.parametrize("huge", ["1", "0"])
def test_new_host_buffer_filled_by_copy(monkeypatch, as_bytearray, huge):
    """_new_host_buffer (the drop-in results: uninitialised bytes / bytearray,
    transparent huge pages asked for on its aligned interior unless
    LZ4M_HUGEPAGES=0): the right type and size, and a pool copy into its
    address lands in the object."""
    import lz4._native as N
    monkeypatch.setenv("LZ4M_HUGEPAGES", huge)
    n = (9 << 20) + 5
    src = np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8)
    obj, addr = N._new_host_buffer(n, as_bytearray)
    assert isinstance(obj, bytearray if as_bytearray else bytes) and len(obj) == n
    N.lib().lz4m_host_copy(addr, src.ctypes.data_as(C.c_void_p), n, 4, None)
    assert obj == src.tobytes()


def test_feed_hash_in_order(oracle):
    """The pipelined frame decode's hash thread (_FeedHash): ranges handed to
    it in order hash to the one-shot XXH32 of their concatenation."""
    from lz4.frame._frame import _FeedHash
    data = np.random.default_rng(5).integers(0, 256, (3 << 20) + 77, dtype=np.uint8)
    h = _FeedHash()
    h.start()
    cuts = [0, 1, 4096, 70000, 1 << 20, (2 << 20) + 3, data.size]
    base = data.ctypes.data
    for a, b in zip(cuts, cuts[1:]):
        h.put(base + a, b - a)
    assert h.digest() == oracle.xxh32(data.tobytes(), 0)
