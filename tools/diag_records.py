#!/usr/bin/env python3
"""Run ON THE GPU BOX: scan one synthetic split and, for every record that is
not a whole line (bench.check_records' start / end tests), print where it came
from -- its start and length, the lane chunk it lies in (start % chunk), tile,
lane, and the bytes around it -- together with the oracle's record for the
line the GPU should have reported. Test tooling, not product.

  python tools/diag_records.py [--gib 32] [--seed 100] [--pattern error] [--chunk 0] [--max 8]
  (DGREP_LIB=... selects a variant library)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-grep_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=32.0)
    ap.add_argument("--seed", type=int, default=100)
    ap.add_argument("--kind", type=int, default=0)
    ap.add_argument("--pattern", default="error")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--max", type=int, default=8)
    args = ap.parse_args()

    import torch

    import dgrep
    import oracle_lib as O

    n = int(args.gib * (1 << 30))
    n -= n % 64
    dev = torch.device("cuda", 0)
    ctx = dgrep.Context(0)
    print("library:", dgrep.LIB_PATH, dgrep.build_info(), flush=True)
    if args.chunk:
        ctx.set_lane_chunk(args.chunk)
    ctx.load(args.pattern)
    buf = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    ctx.synth(buf.data_ptr(), n, args.seed, args.kind)
    cap = max(1 << 16, n // 2048)
    line_t = torch.empty(cap, dtype=torch.int64, device=dev)
    start_t = torch.empty(cap, dtype=torch.int64, device=dev)
    len_t = torch.empty(cap, dtype=torch.int64, device=dev)
    cnt = ctx.scan_device(buf.data_ptr(), n, line_t.data_ptr(), start_t.data_ptr(), len_t.data_ptr(), cap)
    st_ = ctx.scan_stats()
    C = int(st_["lane_chunk"])
    print("records %d, stepper %s, lane chunk %d, overflow lanes %d, pending %d" % (
        cnt, st_["stepper"], C, st_["overflow_lanes"], st_["pending"]), flush=True)
    st = start_t[:cnt]
    en = st + len_t[:cnt]
    prev_ok = (st == 0) | (buf[(st - 1).clamp(min=0)] == 10)
    end_ok = (en == n) | (buf[en.clamp(max=n - 1)] == 10)
    bad = torch.nonzero(~(prev_ok & end_ok)).flatten()
    print("records failing the start test: %d, the end test: %d, either: %d" % (
        int((~prev_ok).sum()), int((~end_ok).sum()), bad.numel()), flush=True)
    tile = 64 * C
    for i in bad[: args.max].tolist():
        s, L, ln = int(start_t[i]), int(len_t[i]), int(line_t[i])
        lo = max(0, s - 300)
        win = buf[lo:min(n, s + L + 300)].cpu().numpy().tobytes()
        # the oracle's records over the window (whole lines around the record)
        a = win.find(b"\n") + 1 if lo else 0
        b = win.rfind(b"\n")
        oln, ost, ole = O.grep_map(args.pattern.encode(), win[a:b], threads=1)
        near = [(int(x) + lo + a, int(y)) for x, y in zip(ost, ole)]
        print("--- record %d: start %d len %d line %d | start %% C = %d (C = %d), tile %d, lane %d, "
              "chunk end at %d; prev byte %r, byte after %r" % (
                  i, s, L, ln, s % C, C, s // tile, (s % tile) // C, (s // C + 1) * C,
                  win[s - lo - 1:s - lo] if s else b"", win[s - lo + L:s - lo + L + 1]), flush=True)
        print("    neighbours (GPU):", [(int(start_t[j]), int(len_t[j])) for j in range(max(0, i - 2), min(cnt, i + 3))])
        print("    oracle lines in +-300 B:", near)
    if bad.numel() == 0:
        print("every record is a whole line", flush=True)


if __name__ == "__main__":
    main()
