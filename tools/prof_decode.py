"""Decoder profiling driver: per-kind timing of the batched decode kernel."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import torch
from lz4 import _native as N, _synth
sys.path.insert(0, ROOT)
import bench

dev = torch.device("cuda", 0)
n = int(os.environ.get("NBLK", 65536))
kinds = os.environ.get("KINDS", "silesia,text,source,records,markup,random,runs").split(",")
reps = int(os.environ.get("REPS", 3))
out = {}
for kind in kinds:
    src = bench.make_batch(n, min(2048, n), kind, 7, dev)
    so, sl, slots, soff, scap, olen = bench.compress_all(src, n, 0, dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
    torch.cuda.synchronize()
    cbytes = int(olen.to(torch.int64).sum())
    dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
    doff = torch.arange(n, dtype=torch.int64, device=dev) * 65536
    dcap = torch.full((n,), 65536, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, n)
    torch.cuda.synchronize()
    if not os.environ.get("PROF_NOCHECK"):
        assert torch.equal(dst, src)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, n); b.record()
        torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    ms = min(ts)
    if os.environ.get("LZ4M_STATS"):
        w = list(N._WORK.values())[0].view(torch.int64).cpu().tolist()
        it, live, fast, slow, slanes, coop, refill = w[1:8]
        if os.environ.get("LZ4M_STATS") == "2":
            tot = sum(w[8:13])
            print(kind, "cycle shares: exec %.2f room+window %.2f parse %.2f slow %.2f refill %.2f; cycles/round %.0f" %
                  tuple([x / tot for x in w[8:13]] + [tot / max(1, it)]), flush=True)
            print(kind, "slow-step split: decode_step %.2f final-wait %.2f (of all cycles); cycles per slow step %.0f" %
                  (w[13] / tot, w[14] / tot, w[11] / max(1, slow)), flush=True)
        print(kind, f"waves-iter {it} live/iter {live/it:.1f} fast/iter {fast/it:.1f} slow-steps {slow} "
              f"({slow/it:.3f}/iter, {slanes/max(1,slow):.1f} lanes) coop {coop} refills {refill} "
              f"fast-lane-seqs/block {fast/n:.0f} iters/block-lane {it*64/n:.0f}", flush=True)
    out[kind] = {"ms": round(ms, 3), "ratio": round(n * 65536 / cbytes, 3), "GiB_s": round(n * 65536 / ms / 1e-3 / 2**30, 1),
                 "algo_GB_s": round((cbytes + n * 65536) / ms / 1e6, 1)}
    print(kind, out[kind], flush=True)
    del src, slots, dst
    torch.cuda.empty_cache()
print(json.dumps(out))
