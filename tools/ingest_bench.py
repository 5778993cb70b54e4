"""End-to-end (PCIe-inclusive) rate of dgrep_scan from a HOST buffer — the
worker's split ingest + scan + result readback, for the
ingest configurations of dgrep_set_ingest. Not the bench metric (that one is
HBM-resident, bench.py); run on the GPU box:

    python tools/ingest_bench.py [--gib 4] [--workload c2]

Prints one JSON line per configuration.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-grep_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import numpy as np
    import torch

    import bench
    import dgrep

    wl = bench.WORKLOADS[args.workload]
    pattern = bench.workload_pattern(wl)
    n = int(args.gib * (1 << 30))
    ctx = dgrep.Context(0)
    ctx.load(pattern)
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.synth(d.data_ptr(), n, wl["seed"], wl["kind"])
    host = d[:n].cpu().numpy()  # pageable host split, as Go's os.ReadFile leaves it
    del d
    torch.cuda.empty_cache()
    data = host.tobytes()
    configs = [("direct pageable hipMemcpyAsync", 0, 0, 0), ("pinned 64MiB x4, 4 threads", 64 << 20, 4, 4),
               ("pinned 64MiB x4, 8 threads", 64 << 20, 4, 8), ("pinned 256MiB x3, 8 threads", 256 << 20, 3, 8)]
    ref = None
    for name, chunk, bufs, threads in configs:
        ctx.set_ingest(chunk, bufs, threads)
        best, ingest_ms, count = None, None, None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            ln, st, le = ctx.scan(data)
            dt = time.perf_counter() - t0
            if best is None or dt < best:
                best, ingest_ms, count = dt, ctx.last_ingest_ms(), len(ln)
        if ref is None:
            ref = (ln, st, le)
        else:
            for a, b in zip((ln, st, le), ref):
                np.testing.assert_array_equal(a, b)
        print(json.dumps({"ingest": name, "split_bytes": n, "matching_lines": count,
                          "end_to_end_gbs": round(n / best / 1e9, 2), "end_to_end_s": round(best, 4),
                          "ingest_ms": round(ingest_ms, 2), "scan_kernel_ms": round(ctx.last_kernel_ms(), 3),
                          "host_threads_available": os.cpu_count()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
