"""CPU emulation of the pair stepper's algorithm (StepPair in
csrc/kernels/scan_dfa.hip, image built by build_pair_image in
csrc/runtime/dgrep_runtime.hip): two input bytes per table lookup, with
SHADOW states carrying the event of a '\\n' that is the first byte of a pair.

The emulation restates the construction (ids, premultiplied rows, shadow
targets, the >= thr / >= M event rule) in numpy and steps whole splits pair by
pair from offset 0, then compares the matching line numbers with the oracle's
restatement of grep.go Map. The GPU parity tests check the C++ builder and the
kernel; this pins the algorithm itself, CPU only."""
import random
import zlib

import numpy as np
import pytest

import dgrep
import oracle_lib as O


def build_pair(cp):
    bc, T = cp.tables()
    S, K, M = cp.nstates, cp.nclasses, cp.start_m
    cn = int(bc[10])
    any_flag = bool((T[:, cn] == M).any())
    targets = []
    if any_flag:
        for c in range(K):
            y = int(T[M, c])
            if y not in targets:
                targets.append(y)
    ids, orig = {}, []
    for s in range(S):
        if s != M:
            ids[s] = len(orig)
            orig.append(s)
    shadow = {}
    for y in targets:
        if y != M:
            shadow[y] = len(orig)
            orig.append(y)
    ids[M] = len(orig)
    orig.append(M)
    if M in targets:
        shadow[M] = len(orig)
        orig.append(M)
    Sp = len(orig)
    assert Sp == S + len(targets)
    T2 = np.zeros((Sp, K, K), np.int64)
    T1 = np.zeros((Sp, K), np.int64)
    for i, x in enumerate(orig):
        for c1 in range(K):
            a = int(T[x, c1])
            T1[i, c1] = ids[a]
            flagged = c1 == cn and a == M
            for c2 in range(K):
                y = int(T[a, c2])
                T2[i, c1, c2] = shadow[y] if flagged else ids[y]
    return dict(T2=T2, T1=T1, bc=bc, start=ids[cp.start], M=ids[M], thr=S - 1, cn=cn, Sp=Sp, K=K)


def run_pair(P, data: bytes):
    """Matching line numbers, stepping pairs from offset 0 (one lane)."""
    cls = P["bc"][np.frombuffer(data, np.uint8)] if data else np.zeros(0, np.int64)
    v, M, thr = P["start"], P["M"], P["thr"]
    out = []
    line = 1
    n2 = len(data) - len(data) % 2
    for i in range(0, n2, 2):
        v = int(P["T2"][v, cls[i], cls[i + 1]])
        e1 = v >= thr and v != M
        e2 = v >= M
        if e1:
            assert data[i] == 10
            out.append(line)
        if data[i] == 10:
            line += 1
        if e2:
            assert data[i + 1] == 10
            out.append(line)
        if data[i + 1] == 10:
            line += 1
    for i in range(n2, len(data)):
        v = int(P["T1"][v, cls[i]])
        if data[i] == 10:
            if v == M:
                out.append(line)
            line += 1
    if int(P["T1"][v, P["cn"]]) == M:
        out.append(line)  # strings.Split's final piece
    return out


PATTERNS = [b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"(WARN|ERROR) [a-z_]+", b"timeout while waiting for lock",
            b"^$", b"", b"^", b"x*$", b"\\bkey\\b", b"(?i)k", b"e(r|x)+o", b"^[ -~]{5}$", b"\\x{FFFD}", b"a|^$",
            b"[^a-z ]{3}", b"(alpha|bravo|charlie)[0-9]+"]


@pytest.mark.parametrize("pattern", PATTERNS)
def test_pair_algorithm_matches_oracle(pattern):
    cp = dgrep.CompiledPattern(pattern)
    P = build_pair(cp)
    rnd = random.Random(zlib.crc32(pattern) & 0xffff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b"K", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\n\n", b"\r",
             b"\xe2\x82\xac", b"\xe2\x82", b"\xff", b"\xc5\xbf", b"WARN ab", b"ERROR x", b"error", b"2024-01",
             b"key ", b"timeout while waiting for lock", b"alpha7"]
    cases = [b"", b"\n", b"\n\n", b"\n\n\n", b"x", b"x\n", b"\nx", b"2024-01-02 WARN ab\n\n2024-01-02 WARN ab"]
    for _ in range(30):
        cases.append(b"".join(rnd.choice(alpha) for _ in range(rnd.choice([3, 30, 300]))))
    cases.append(dgrep.synth_corpus_host(20000, 3, 0))
    for data in cases:
        want = O.grep_map(pattern, data)[0].tolist()
        assert run_pair(P, data) == want, (pattern, data[:80])


def test_pair_image_sizes():
    """C3's regex fits the pair stepper's LDS budget (kPairMaxT2 = 32 KiB of
    T2); 1,000 keywords do not (they stay on the wide stepper)."""
    c3 = dgrep.CompiledPattern(b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+")
    P = build_pair(c3)
    assert 2 * P["Sp"] * P["K"] ** 2 <= 32768
    kws = dgrep.synth_keywords(4, 1000)
    c4 = dgrep.CompiledPattern(b"(?i)(" + b"|".join(kws) + b")")
    assert 2 * c4.nstates * c4.nclasses ** 2 > 32768
