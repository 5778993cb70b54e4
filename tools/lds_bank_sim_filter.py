"""LDS bank-conflict model of the filter stepper's chain reads (CPU only).

Replays the dependent ds_read_u16 of StepFilter (csrc/kernels/scan_dfa.hip)
for a wave's 64 lanes stepping config 4's corpus (synth kind 1, seed 4) with
its 1,000-keyword (?i) DFA, the filter image of build_filter_image
(csrc/runtime/dgrep_runtime.hip: breadth-first rows from start, CAND for the
rest), and scores row layouts the same way tools/lds_bank_sim.py does for the
pair stepper: a wave64 u16 read is two 32-lane groups, each taking as many LDS
cycles as the most distinct dwords one bank ((a/4) mod 32) holds
(MI355X_MICROARCH.md, LDS). Layouts:
  row:   [state][class] rows at a pitch of P entries (the shipped image, P/2 odd)
  colT:  [class][state] columns of R entries (R/2 odd): lanes in different
         states reading one class hit consecutive dwords
usage: python tools/lds_bank_sim_filter.py [--waves 8] [--words 256]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-grep_amd"))
import dgrep  # noqa: E402


def group_cycles(dw):
    """dw: [n, 64] dword addresses -> [n] LDS cycles of two 32-lane groups."""
    tot = np.zeros(len(dw), np.int64)
    for g in (slice(0, 32), slice(32, 64)):
        d = dw[:, g]
        for i in range(len(d)):
            u = np.unique(d[i])
            tot[i] += max(1, np.bincount(u % 32, minlength=32).max())
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--words", type=int, default=256)
    ap.add_argument("--chunk", type=int, default=32768)
    a = ap.parse_args()
    kws = dgrep.synth_keywords(4, 1000)
    cp = dgrep.CompiledPattern("(?i)(" + "|".join(k.decode() for k in kws) + ")")
    bc, T = cp.tables()
    T = T.astype(np.int64)
    S, K = cp.nstates, cp.nclasses
    # breadth-first ids from start (start, start_m first), as build_filter_image
    order, seen = [cp.start, cp.start_m], {cp.start, cp.start_m}
    q = 0
    while q < len(order):
        for k in range(K):
            x = int(T[order[q], k])
            if x not in seen:
                seen.add(x)
                order.append(x)
        q += 1
    P = ((K + 1) & ~1) + (0 if ((K + 1) & 2) else 2)
    R = min(S, (124 * 1024 - 256) // (2 * P)) - 2
    bid = np.full(S, R, np.int64)  # non-resident -> CAND (row R)
    for i, x in enumerate(order[:R]):
        bid[x] = i
    lanes = 64 * a.waves
    data = np.frombuffer(dgrep.synth_corpus_host(lanes * a.chunk, 4, 1), np.uint8)
    # each lane from a point well inside its chunk (past the first lines)
    lane_data = data.reshape(lanes, a.chunk)[:, 4096: 4096 + 4 * a.words].astype(np.int64)
    cls = bc.astype(np.int64)[lane_data]
    s = np.full(lanes, cp.start, np.int64)
    cand = np.zeros(lanes, bool)
    rows, cols = [], []
    nl = bc[ord("\n")]
    for j in range(4 * a.words):
        c = cls[:, j]
        r = np.where(cand, R, bid[s])
        rows.append(r)
        cols.append(c)
        nxt = T[s, c]
        # CAND until '\n', then start (CAND_END behaves like start)
        cand = np.where(c == nl, False, cand | (bid[nxt] >= R))
        s = np.where(c == nl, cp.start, nxt)
    rows, cols = np.stack(rows), np.stack(cols)
    Rp = R + 1 + 2  # rows incl. CAND, start_m, CAND_END
    Rt = ((Rp + 1) & ~1) + (0 if ((Rp + 1) & 2) else 2)  # R/2 odd

    def score(dw):
        cyc = []
        for w in range(a.waves):
            cyc.append(group_cycles(dw[:, 64 * w: 64 * w + 64]))
        return float(np.mean(np.concatenate(cyc)))

    layouts = {
        "row (shipped, P=%d)" % P: 64 + (rows * P + cols) // 2,
        "row P=%d (even dwords)" % (P + 2 if (P // 2) % 2 else P): 64 + (rows * (P + 2 if (P // 2) % 2 else P) + cols) // 2,
        "colT (R=%d)" % Rt: 128 + (cols * Rt + rows) // 2,
    }
    print(f"C4 filter: S={S} K={K} resident rows {R}; {a.waves} waves x {4 * a.words} bytes from 4 KiB into 32 KiB chunks")
    print(f"  lanes in CAND: {float(np.mean(rows == R)):.3f}; distinct rows per 32-lane group: "
          f"{float(np.mean([len(np.unique(rows[i, g:g + 32])) for i in range(0, len(rows), 7) for g in (0, 32)])):.1f}")
    for name, dw in layouts.items():
        print(f"  {name:28s}: {score(dw):.2f} LDS cycles per chain read (2 = conflict-free)")


if __name__ == "__main__":
    main()
