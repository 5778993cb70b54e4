"""CPU emulation of the default-row records of long_dfa_seg_kernel (DfaXRec in
csrc/kernels/scan_common.h, built by build_ximg in
csrc/runtime/dgrep_runtime.hip, read by FullDfa::next in
csrc/kernels/scan_dfa.hip).

A u16 DFA's first H breadth-first rows sit in LDS whole; each further state
gets an 8-byte record: the resident row that differs from its own in the
fewest classes (its DEFAULT), plus at most two (class, next state)
exceptions; a state no resident row comes within two classes of gets an extra
row of its own as default (build_ximg). The emulation restates the construction in numpy and checks that
the record lookup reproduces every entry of the table, for the configs'
keyword automaton and a few other filter-sized patterns. The GPU long-line
tests (tests/test_gpu_long_lines.py) check the C++ builder and the kernel."""
import collections

import numpy as np
import pytest

import dgrep

NONE = 0xFF
BUDGET = 158 * 1024


def bfs_table(cp):
    _, T = cp.tables()
    T = T.astype(np.int64)
    S, K = cp.nstates, cp.nclasses
    order, bid = [], -np.ones(S, np.int64)

    def visit(x):
        if bid[x] < 0:
            bid[x] = len(order)
            order.append(x)

    visit(cp.start)
    visit(cp.start_m)
    q = 0
    while q < len(order):
        for c in range(K):
            visit(int(T[order[q], c]))
        q += 1
    for x in range(S):
        visit(x)
    return bid[T[np.array(order)]]


def build_ximg(F, budget=BUDGET):
    """(H, extra rows, records): rows [0, H) resident, records for [H, S);
    a state no resident row comes within two classes of gets an extra row."""
    S, K = F.shape
    row = 2 * K
    H = min(S, (budget - 8 - 8 * S) // (row - 8))
    while H >= 64:
        recs, extra = [], []
        for j in range(S - H):
            f = F[H + j]
            diff = (F[:H] != f).sum(1)
            d = int(np.argmin(diff))
            if diff[d] > 2:
                recs.append((H + len(extra), NONE, NONE, 0, 0))
                extra.append(H + j)
                continue
            ex = [(int(k), int(f[k])) for k in np.flatnonzero(F[d] != f)] + [(NONE, 0), (NONE, 0)]
            recs.append((d, ex[0][0], ex[1][0], ex[0][1], ex[1][1]))
        off = ((H + len(extra)) * row + 7) & ~7
        size = (off + 8 * len(recs) + 15) & ~15
        if size <= budget:
            return H, extra, recs, size
        H -= (size - budget) // (row - 8) + 1 + len(extra)
    return None


def lookup(F, H, extra, recs, s, c):
    if s < H:
        return int(F[s, c])
    d, c1, c2, n1, n2 = recs[s - H]
    t = int(F[d, c]) if d < H else int(F[extra[d - H], c])
    t = n2 if c == c2 else t
    t = n1 if c == c1 else t
    return t


def patterns():
    kws = dgrep.synth_keywords(4, 1000)
    return [b"(?i)(" + b"|".join(kws) + b")",
            b"(?i)(" + b"|".join(kws[:300]) + b")",
            b"[a-z]{3}[0-9]{3}x[a-f]+z"]


@pytest.mark.parametrize("pattern", patterns(), ids=["c4", "c4_300", "classes"])
def test_xrec_lookup_reproduces_the_table(pattern):
    cp = dgrep.CompiledPattern(pattern)
    F = bfs_table(cp)
    S, K = F.shape
    if S <= 256:
        pytest.skip("not a filter-sized DFA")
    H, extra, recs, _ = build_ximg(F)
    assert H >= 64 and H + len(recs) == S
    for s in range(S):
        for c in range(K):
            assert lookup(F, H, extra, recs, s, c) == F[s, c], (s, c)


def test_xrec_covers_config4():
    """Config 4's keyword automaton: every state past the rows gets a record,
    all but a handful with a default."""
    F = bfs_table(dgrep.CompiledPattern(patterns()[0]))
    S, K = F.shape
    H, extra, recs, size = build_ximg(F)
    assert H + len(recs) == S and size <= BUDGET
    assert len(extra) <= 8, len(extra)
    ex = collections.Counter((r[1] != NONE) + (r[2] != NONE) for r in recs if r[0] < H)
    assert ex[1] > 10 * ex[2]
