"""LDS bank-conflict model of the pair stepper's reads (CPU only).

Replays what a wave's 64 lanes read from LDS while stepping a corpus with the
pair stepper (StepPair in csrc/kernels/scan_dfa.hip, image of build_pair_image
in csrc/runtime/dgrep_runtime.hip): per word the four byte-table reads
(UA[b0], UB[b1], UA[b2], UB[b3]) and the two dependent T2 reads. A wave64
ds_read_b32 / ds_read_u16 is served as two 32-lane groups; a group takes as
many LDS cycles as the most distinct dwords any one bank ((a/4) mod 32) holds
(MI355X_MICROARCH.md, LDS). Prints the modelled cycles per instruction for
each kind of read and each byte-table layout given, so a layout can be judged
before it is built (shadow states are left out: they are rare).

usage: python tools/lds_bank_sim.py [--workload c3] [--waves 8] [--words 512]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-grep_amd"))
import dgrep  # noqa: E402

PATTERNS = {"c3": (b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", 3, 8192),
            "c4": (b"timeout while waiting for lock|connection reset by peer|(WARN|ERROR) [a-z_]+", 4, 8192)}


def group_cycles(addr):
    """addr: [n_instr, 64] byte addresses -> [n_instr] LDS cycles (two 32-lane groups)."""
    dw = addr // 4
    total = np.zeros(len(addr), np.int64)
    for g in (slice(0, 32), slice(32, 64)):
        d = dw[:, g]
        bank = d % 32
        cyc = np.ones(len(addr), np.int64)
        for i in range(len(addr)):
            u = np.unique(d[i])
            cyc[i] = max(1, np.bincount(u % 32, minlength=32).max())
        total += cyc
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--words", type=int, default=512)
    a = ap.parse_args()
    pat, seed, chunk = PATTERNS[a.workload]
    cp = dgrep.CompiledPattern(pat)
    bc, T = cp.tables()
    T = T.astype(np.int64)
    S, K = cp.nstates, cp.nclasses
    row = ((2 * K * K + 3) & ~3) | 4
    lanes = 64 * a.waves
    data = np.frombuffer(dgrep.synth_corpus_host(lanes * chunk, seed, 0), np.uint8)
    lane_data = data.reshape(lanes, chunk)[:, : 4 * a.words].astype(np.int64)
    words = lane_data.reshape(lanes, a.words, 4)
    cls = bc.astype(np.int64)[words]
    # states: lanes start at the DFA start state at their chunk start
    s = np.full(lanes, cp.start, np.int64)
    prep = {"u32 [256] (now)": [], "u32 [256] x2 (lane half)": [], "per-bank copies": []}
    chain = []
    lane = np.arange(lanes) % 64
    for j in range(a.words):
        b = words[:, j, :]
        for k in range(4):
            base = 0 if k % 2 == 0 else 1024
            prep["u32 [256] (now)"].append(base + 4 * b[:, k])
            prep["u32 [256] x2 (lane half)"].append(base * 2 + 4 * b[:, k] + 1024 * ((lane // 16) % 2))
            prep["per-bank copies"].append(128 * b[:, k] + 4 * (lane % 32) + (2 if k % 2 else 0))
        c = cls[:, j, :]
        col1 = 2 * (c[:, 0] * K + c[:, 1])
        chain.append(2048 + s * row + col1)
        s = T[T[s, c[:, 0]], c[:, 1]]
        col2 = 2 * (c[:, 2] * K + c[:, 3])
        chain.append(2048 + s * row + col2)
        s = T[T[s, c[:, 2]], c[:, 3]]

    def per_wave(lst):
        arr = np.stack(lst)  # [n, lanes]
        cyc = []
        for w in range(a.waves):
            cyc.append(group_cycles(arr[:, 64 * w: 64 * w + 64]))
        return float(np.mean(np.concatenate(cyc)))

    ch = per_wave(chain)
    print(f"{a.workload}: {a.waves} waves x {a.words} words; LDS cycles per wave-instruction (2 = conflict-free)")
    print(f"  chain T2 reads (2/word): {ch:.2f}")
    for name, lst in prep.items():
        p = per_wave(lst)
        print(f"  byte tables {name:28s} (4/word): {p:.2f}  -> per word {4 * p + 2 * ch:.1f} cycles")


if __name__ == "__main__":
    main()
