"""GPU parity for patterns over the compiler's DFA budget (DGREP_DFA_PARTIAL):
the filter stepper runs the blob's first DFA states and verify_nfa_kernel
decides every line that leaves them with the blob's NFA program. Compared
bit-exactly with the oracle (grep.go:17-29 restated), through the C ABI."""
import random
import zlib

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_parity import PATTERNS, _check

pytestmark = pytest.mark.gpu


def _ab_lines(rnd, n):
    out = []
    for _ in range(n):
        k = rnd.random()
        if k < 0.6:
            out.append(bytes(rnd.choice(b"ab") for _ in range(rnd.randint(0, 60))))
        elif k < 0.8:
            out.append(bytes(rnd.choice(b"abc") for _ in range(rnd.randint(15, 40))))
        else:
            out.append(rnd.choice([b"", "é".encode() * 30, b"a" * 21, b"\xff" * 25, b"x" + b"a" * 22]))
    return b"\n".join(out)


HUGE = [b"[ab]*a[ab]{21}", b"a.{20}$", b"(?i)\\bk.{19}s",
        # more than 256 NFA positions: verify_nfa_kernel's 32-word instance
        b"[ab]*a[ab]{300}", b"x\\pL{280}y"]


@pytest.mark.parametrize("pattern", HUGE)
def test_budget_exceeding_patterns_on_gpu(gpu_ctx, pattern):
    import dgrep

    cp = gpu_ctx.load(pattern)
    assert cp.partial, cp.flags
    rnd = random.Random(len(pattern))
    data = _ab_lines(rnd, 40000) + b"\n" + dgrep.synth_corpus_host(1 << 20, 5, 0)
    # lines long enough for the > 256-position patterns to match
    data += b"\n" + b"ab" * 200 + b"\n" + b"b" * 299 + b"\nx" + b"q" * 280 + b"y\nx" + "é".encode() * 280 + b"y"
    n = _check(gpu_ctx, cp, data, threads=16)
    st = gpu_ctx.scan_stats()
    assert st["stepper"] == "filter", st
    assert n > 0 or pattern.startswith(b"(?i)")


@pytest.mark.parametrize("pattern", PATTERNS)
def test_forced_partial_every_pattern(gpu_ctx, pattern):
    """State budget 3 (dgrep_compile_budget): almost every line becomes a candidate and is
    decided by the NFA program on the GPU (edges: empty split, no trailing
    '\\n', invalid UTF-8, lines across chunk and tile edges)."""
    import dgrep

    cp = gpu_ctx.load(dgrep.CompiledPattern(pattern, state_budget=3))
    if cp.go_syntax_error:
        return
    assert cp.partial, (pattern, cp.nstates)
    rnd = random.Random(zlib.crc32(pattern) & 0xffff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\xe2\x82\xac", b"\xff",
             b"WARN", b"ERROR", b"error", b"2024-01", b"key ", b"\xe2\x82"]
    for size in (0, 1, 777, 70000):
        data = b"".join(rnd.choice(alpha) for _ in range(size // 3 + 1))[:size]
        _check(gpu_ctx, cp, data)
    data = bytearray(dgrep.synth_corpus_host(3 << 20, 9, 0))
    for edge in (4095, 4096, 65535, 65536, 262143, 262144):
        data[edge] = 0x0A
    _check(gpu_ctx, cp, bytes(data), threads=16)


def test_partial_pattern_rejects_other_steppers(gpu_ctx):
    import dgrep

    try:
        for mode in ("table", "pair"):
            gpu_ctx.set_stepper(mode, 0)
            with pytest.raises(dgrep.DgrepError):
                gpu_ctx.load(b"[ab]*a[ab]{21}")
    finally:
        gpu_ctx.set_stepper("auto", 0)
    cp = gpu_ctx.load(b"[ab]*a[ab]{21}")
    got = gpu_ctx.scan(b"a" + b"b" * 21 + b"\nab\n" + b"a" * 30)
    want = O.grep_map(cp.pattern, b"a" + b"b" * 21 + b"\nab\n" + b"a" * 30)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
