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
