"""Throughput of the GPU partition + intermediate writer (dgrep_encode_device)
over the Map output of an HBM-resident split, next to
the oracle's CPU restatement of writeMapOutput on a sample, then the reduce
(dgrep_reduce) over all the encoded lines. Run on the GPU box:

    python tools/encode_bench.py [--workload c2] [--gib 16] [--nreduce 10]

Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-grep_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--nreduce", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()

    import torch

    import bench
    import dgrep
    import oracle_lib as O

    wl = bench.WORKLOADS[args.workload]
    pattern = bench.workload_pattern(wl)
    n = int(args.gib * (1 << 30))
    ctx = dgrep.Context(0)
    ctx.load(pattern)
    buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.synth(buf.data_ptr(), n, wl["seed"], wl["kind"])
    cap = max(1 << 16, n // 2048)
    ln = torch.empty(cap, dtype=torch.int64, device="cuda")
    st = torch.empty(cap, dtype=torch.int64, device="cuda")
    le = torch.empty(cap, dtype=torch.int64, device="cuda")
    cnt = ctx.scan_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cap)
    assert cnt <= cap
    fname = "split-%s.log" % args.workload
    b, e, total = ctx.encode_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, fname,
                                    args.nreduce, 0, 0)
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    ms = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        b, e, total = ctx.encode_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, fname,
                                        args.nreduce, out.data_ptr(), total)
        ms.append(ctx.last_encode_ms())
    value_bytes = int(le[:cnt].to(torch.int64).sum().item())
    # spot check: the first 2,000 records of partition 0..nreduce-1 vs the oracle
    lnh, sth, leh = ln[:2000].cpu().numpy(), st[:2000].cpu().numpy(), le[:2000].cpu().numpy()
    host = buf[: int(sth[-1] + leh[-1]) + 1].cpu().numpy().tobytes()
    raw = out.cpu().numpy().tobytes()
    parts = [bytearray() for _ in range(args.nreduce)]
    t0 = time.perf_counter()
    for a, s_, l_ in zip(lnh.tolist(), sth.tolist(), leh.tolist()):
        key = O.format_key(fname.encode(), a)
        parts[O.ihash(key) % args.nreduce] += O.json_kv(key, host[s_:s_ + l_])
    cpu_s = time.perf_counter() - t0
    for p in range(args.nreduce):
        assert raw[b[p]:b[p] + len(parts[p])] == bytes(parts[p]), p
    best = min(ms)
    # the reduce side: every partition's lines through dgrep_reduce (all keys distinct)
    red_ms, red_out = [], b""
    for _ in range(3):
        red_out = ctx.reduce(raw[: total])
        red_ms.append(ctx.last_kernel_ms())
    assert red_out.count(b"\n") == cnt
    print(json.dumps({
        "what": "GPU partition + intermediate writer (ihash %% nReduce, json.Encoder lines), map_reduce/worker.go:78-109",
        "workload": wl["desc"], "records": cnt, "nreduce": args.nreduce, "value_bytes": value_bytes,
        "output_bytes": total, "encode_ms_best": round(best, 3), "encode_ms_all": [round(x, 3) for x in ms],
        "records_per_s": round(cnt / (best * 1e-3)), "output_gbs": round(total / (best * 1e-3) / 1e9, 2),
        "cpu_oracle_records_per_s_1core": round(2000 / cpu_s),
        "checked": "first 2,000 records bit-exact vs oracle per partition prefix",
        "reduce_ms_best": round(min(red_ms), 3), "reduce_lines_per_s": round(cnt / (min(red_ms) * 1e-3)),
        "reduce_output_bytes": len(red_out)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
