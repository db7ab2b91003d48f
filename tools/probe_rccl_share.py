"""Dev probe: can two ranks share one GPU under RCCL (world size 2 on a
one-GPU box)?  Each rank inits "nccl" on cuda:0, all_gathers a tensor and
sends one to the other; prints what happened.  (test_gpu_dist's world-2
RCCL test skips on one GPU; this decides whether it can run there.)"""
import os
import sys
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
        x = torch.full((4,), rank + 1, dtype=torch.int32, device=dev)
        out = [torch.empty_like(x) for _ in range(2)]
        dist.all_gather(out, x)
        if rank == 0:
            dist.send(x + 10, 1)
        else:
            y = torch.empty_like(x)
            dist.recv(y, 0)
            out.append(y)
        torch.cuda.synchronize()
        print(f"rank {rank}: ok {[t.tolist() for t in out]}", flush=True)
        dist.destroy_process_group()
    except Exception as e:
        print(f"rank {rank}: {type(e).__name__}: {str(e)[:400]}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    mp.spawn(worker, args=(29577,), nprocs=2, join=True)
