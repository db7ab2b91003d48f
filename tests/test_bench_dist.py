"""bench.py's multi-rank reporting path on CPU (gloo, world size 2): the
timing protocol (warmup, barrier + sync around exactly `steps` calls) takes
the MAX over ranks, `value` counts every rank's bytes over that max time
(weak scaling), and the CPU baseline runs on rank 0 only.  The GPU run uses
the same helpers over RCCL with HIP events."""
import os
import socket
import sys
import time

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []
        delay = 0.02 * (rank + 1)   # rank 1 is the slow one

        def step():
            calls.append(1)
            time.sleep(delay)

        wall, ev = B.time_kernel(step, steps=3, warmup=2, world=world, device="cpu")
        q.put((rank, len(calls), wall, ev, B.runs_cpu_baseline(rank, False)))
    finally:
        dist.destroy_process_group()


def test_time_kernel_max_over_ranks_and_aggregate():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # exactly warmup + steps calls on every rank
    assert all(o[1] == 5 for o in out)
    # every rank reports the same (max) wall and per-step time: the slow rank's
    walls = {round(o[2], 9) for o in out}
    evs = {round(o[3], 9) for o in out}
    assert len(walls) == 1 and len(evs) == 1
    wall, ev = out[0][2], out[0][3]
    assert ev >= 0.04 * 0.95 and wall >= 3 * 0.04 * 0.95
    # the CPU baseline on rank 0 only
    assert [o[4] for o in out] == [True, False]
    # value = all ranks' bytes / the max-over-ranks time per step
    v = B.aggregate_gib_s(world, 1 << 20, 65536, wall, 3)
    assert abs(v - world * (1 << 20) * 65536 / (wall / 3) / (1 << 30)) < 1e-9
    assert B.aggregate_gib_s(1, 1 << 20, 65536, wall, 3) * 2 == v


def test_runs_cpu_baseline_flag():
    assert B.runs_cpu_baseline(0, False)
    assert not B.runs_cpu_baseline(0, True)
    assert not B.runs_cpu_baseline(3, False)
