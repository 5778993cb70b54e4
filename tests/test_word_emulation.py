"""CPU emulation of the word stepper's algorithm (StepWord in
csrc/kernels/scan_dfa.hip, image built by build_word_image in
csrc/runtime/dgrep_runtime.hip): ONE table lookup per 4-byte word, the word's
class found in two table levels (pair classes, then word classes), EVENT
shadows for a word whose single '\\n' ends a matching line before its last
byte, RECHECK shadows for a word with two or more '\\n' (its events recomputed
byte by byte from the state before it).

The emulation restates the construction in numpy (word functions over every
quad of byte classes, pair classes as equivalence in either half, ids, the
>= thr_e / >= thr_r rules) and steps whole splits word by word from offset 0,
then compares the matching line numbers with the oracle's restatement of
grep.go Map. The GPU parity tests check the C++ builder and the kernel; this
pins the algorithm itself, CPU only."""
import random

import numpy as np
import pytest

import dgrep
import oracle_lib as O


def build_word(cp):
    bc, T = cp.tables()
    T = T.astype(np.int64)
    S, K, M = cp.nstates, cp.nclasses, cp.start_m
    cn = int(bc[10])
    # every quad of classes, every start state: code x / S + x (event) / 2S + x (recheck)
    q = np.arange(K ** 4)
    cs = [q // K ** 3, q // K ** 2 % K, q // K % K, q % K]
    nl = sum((c == cn).astype(np.int64) for c in cs)
    x = np.broadcast_to(np.arange(S), (K ** 4, S)).copy()
    ev = np.zeros((K ** 4, S), bool)
    for k, c in enumerate(cs):
        y = T[x, c[:, None]]
        if k < 3:
            ev |= (c[:, None] == cn) & (y == M)
        x = y
    F = np.where(nl[:, None] >= 2, 2 * S + x, np.where((nl[:, None] == 1) & ev, S + x, x))
    _, wq, = np.unique(F, axis=0, return_inverse=True)[:2]
    wq = wq.reshape(-1)
    W = int(wq.max()) + 1
    wrep = np.zeros(W, np.int64)
    wrep[wq] = q
    K2 = K * K
    wq2 = wq.reshape(K2, K2)
    sig = np.concatenate([wq2, wq2.T], axis=1)
    _, pc = np.unique(sig, axis=0, return_inverse=True)[:2]
    pc = pc.reshape(-1)
    P = int(pc.max()) + 1
    WC = np.zeros((P, P), np.int64)
    for a in range(K2):
        WC[pc[a], pc] = wq2[a]
    # every pair of pairs is consistent with WC (the pair classes' meaning)
    assert (WC[pc[:, None], pc[None, :]] == wq2).all()
    is_e = np.zeros(S, bool)
    is_r = np.zeros(S, bool)
    is_e[(F[(F >= S) & (F < 2 * S)] - S)] = True
    is_r[(F[F >= 2 * S] - 2 * S)] = True
    ids, orig = {}, []
    for s in range(S):
        if s != M:
            ids[s] = len(orig)
            orig.append(s)
    first_e = len(orig)
    eid = {}
    for s in np.flatnonzero(is_e):
        eid[int(s)] = len(orig)
        orig.append(int(s))
    ids[M] = len(orig)
    orig.append(M)
    first_r = len(orig)
    rid = {}
    for s in np.flatnonzero(is_r):
        rid[int(s)] = len(orig)
        orig.append(int(s))
    Sp = len(orig)

    def cid(v):
        v = int(v)
        return rid[v - 2 * S] if v >= 2 * S else eid[v - S] if v >= S else ids[v]

    TW = np.array([[cid(F[wrep[w], orig[i]]) for w in range(W)] for i in range(Sp)], np.int64)
    T1 = np.array([[ids[int(T[orig[i], c])] for c in range(K)] for i in range(Sp)], np.int64)
    return dict(TW=TW, T1=T1, bc=bc.astype(np.int64), pc=pc, WC=WC, K=K, P=P, W=W, Sp=Sp, start=ids[cp.start],
                M=ids[M], thr_e=first_e, thr_r=first_r)


def emulate(d, data: bytes):
    """Matching line numbers (1-based) by word-wise stepping from offset 0."""
    bc, K, M = d["bc"], d["K"], d["M"]
    out = []
    s, line = d["start"], 1
    n4 = len(data) - len(data) % 4
    arr = np.frombuffer(data[:n4], np.uint8).reshape(-1, 4).astype(np.int64) if n4 else np.zeros((0, 4), np.int64)
    c = bc[arr]
    p01 = d["pc"][c[:, 0] * K + c[:, 1]]
    p23 = d["pc"][c[:, 2] * K + c[:, 3]]
    wcls = d["WC"][p01, p23]
    for i in range(len(arr)):
        sp = s
        s = int(d["TW"][sp, wcls[i]])
        nls = [k for k in range(4) if arr[i, k] == 10]
        if s >= d["thr_e"]:
            if len(nls) == 1:
                assert s < d["thr_r"]
                out.append(line)  # the event: this '\n' ends a matching line
            else:
                assert s >= d["thr_r"] and len(nls) >= 2
                x = sp
                for k in range(4):
                    x = int(d["T1"][x, c[i, k]])
                    if arr[i, k] == 10 and x == M:
                        out.append(line + sum(1 for j in nls if j < k))
        line += len(nls)
    for b in data[n4:]:
        s = int(d["T1"][s, bc[b]])
        if b == 10:
            if s == M:
                out.append(line)
            line += 1
    if int(d["T1"][s, bc[10]]) == M:  # the final piece of strings.Split
        out.append(line)
    return out


PATTERNS = [b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"(WARN|ERROR) [a-z_]+", b"timeout while waiting for lock",
            b"\\bkey\\b", b"^[ -~]{45}$", b"e(r|x)+o", b"a|^$", b"^$|error", b"x*$|WARN", b"error", b"^$", b""]


@pytest.mark.parametrize("pattern", PATTERNS)
def test_word_emulation_matches_oracle(pattern):
    cp = dgrep.CompiledPattern(pattern)
    d = build_word(cp)
    rnd = random.Random(hash(pattern) & 0xffff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\n\n", b"\n\n\n", b"\r",
             b"\xe2\x82\xac", b"\xff", b"WARN ab", b"ERROR x", b"error", b"2024-01-02", b"key ", b"timeout while waiting for lock"]
    cases = [b"", b"\n", b"\n\n", b"x\n", b"error", b"error\n", b"\nerror\n\n", dgrep.synth_corpus_host(20000, 3, 0)]
    cases += [b"".join(rnd.choice(alpha) for _ in range(rnd.choice([3, 50, 700, 3000]))) for _ in range(12)]
    for data in cases:
        ln, _, _ = O.grep_map(pattern, data)
        assert emulate(d, data) == [int(x) for x in ln], (pattern, data[:80])


def test_word_tables_small_for_the_configs():
    """C3's regex: 20 states x 12 classes -> 69 word classes, 27 pair classes,
    4 event and 4 recheck shadows: the tables fit the 16 KiB image with room."""
    cp = dgrep.CompiledPattern(PATTERNS[0])
    d = build_word(cp)
    assert (cp.nstates, cp.nclasses) == (20, 12)
    assert d["W"] == 69 and d["P"] == 27 and d["Sp"] == 28
