"""Patterns whose DFA exceeds the compiler's state budget (DGREP_DFA_PARTIAL,
include/dgrep_blob.h): the blob keeps the first DFA states as a filter and an
NFA program decides the lines that leave them. On the CPU, both halves are
interpreted by tests/nfa_runner.py and must reproduce the oracle's Map output
(grep.go:17-29) bit-exactly. dgrep_compile_budget (a test entry point of the
compiler) forces the partial form on small patterns, so the NFA program is
checked on the same random patterns as the DFA (test_compiler.py)."""
import ctypes
import random

import numpy as np
import pytest

import dgrep
import oracle_lib as O
from nfa_runner import NfaProgram, nfa_only, run_partial
from test_compiler import ALPHA, _rand_pattern


def _eq(got, want, what):
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g.astype(np.int64), w.astype(np.int64), err_msg=str(what))


@pytest.mark.parametrize("budget", ["3", "12"])
def test_partial_program_vs_oracle_random(budget):
    rnd = random.Random(1000 + int(budget))
    checked = 0
    for _ in range(300):
        pat = _rand_pattern(rnd).encode()
        if O.compile_status(pat) != O.ORC_OK:
            continue
        try:
            cp = dgrep.CompiledPattern(pat, state_budget=int(budget))
        except dgrep.UnsupportedPattern:
            continue
        if not cp.partial:
            continue  # the whole DFA fits even the lowered budget
        data = b"".join(rnd.choice(ALPHA) for _ in range(rnd.randint(0, 240)))
        want = O.grep_map(pat, data)
        _eq(run_partial(cp, data), want, (pat, data))
        _eq(nfa_only(cp, data), want, (pat, data))
        checked += 1
    assert checked > 150, checked


KNOWN = [
    # pattern, lines (no '\n'); the DFA of each exceeds 2**21 states
    (b"[ab]*a[ab]{21}", [b"", b"a" * 22, b"b" * 40, b"a" + b"b" * 21, b"a" + b"b" * 20, b"xa" + b"ab" * 11,
                         b"ab" * 30 + b"c", b"\xffa" + b"b" * 21]),
    (b"a.{20}$", [b"a" * 21, b"a" * 20, b"xa" + "é".encode() * 20, b"a" + b"\xff" * 20, b"a" + b"\xe2\x82" * 10,
                  b"za" + "€".encode() * 19 + b"q", b"a" + "€".encode() * 21]),
    # more than 256 NFA positions (round 2 refused these with DGREP_E_TOO_LARGE)
    (b"[ab]*a[ab]{300}", [b"a" * 301, b"a" * 300, b"b" * 400, b"a" + b"b" * 300, b"ab" * 151, b"ba" * 150 + b"c"]),
    (b"x\\pL{280}y", [b"x" + b"q" * 280 + b"y", b"x" + "é".encode() * 280 + b"y", b"x" + b"q" * 279 + b"y",
                       b"zx" + b"\xff" * 280 + b"y", b"x" + "中".encode() * 280 + b"yz"]),
]


@pytest.mark.parametrize("pattern,lines", KNOWN)
def test_budget_exceeding_patterns_compile_partial(pattern, lines):
    cp = dgrep.CompiledPattern(pattern)
    assert cp.partial and cp.nstates == 65535, (cp.flags, cp.nstates)
    prog = NfaProgram(cp.nfa_program())
    assert prog.npos <= 1024
    data = b"\n".join(lines)
    _eq(run_partial(cp, data), O.grep_map(pattern, data), pattern)
    for line in lines:
        assert prog.match(line) == bool(O.Regexp(pattern).match(line)), (pattern, line)


def test_blob_info_checks_the_program():
    cp = dgrep.CompiledPattern(b"[ab]*a[ab]{21}")
    L = dgrep.lib()
    info = dgrep._BlobInfo()
    assert L.dgrep_blob_info_get(cp.blob, len(cp.blob), ctypes.byref(info)) == dgrep.DGREP_OK
    assert info.flags & dgrep.DFA_PARTIAL
    # the flag without the program, and the program without the flag, are malformed
    ne = cp.nstates * cp.nclasses
    cut = bytearray(cp.blob[:288 + 4 * ne])
    cut[28:32] = (0).to_bytes(4, "little")
    assert L.dgrep_blob_info_get(bytes(cut), len(cut), ctypes.byref(info)) == dgrep.DGREP_E_INVALID
    noflag = bytearray(cp.blob)
    noflag[8:12] = (0).to_bytes(4, "little")
    assert L.dgrep_blob_info_get(bytes(noflag), len(noflag), ctypes.byref(info)) == dgrep.DGREP_E_INVALID


def _bad(blob: bytes) -> bool:
    info = dgrep._BlobInfo()
    return dgrep.lib().dgrep_blob_info_get(blob, len(blob), ctypes.byref(info)) == dgrep.DGREP_E_INVALID


@pytest.mark.parametrize("pattern", [b"[ab]*a[ab]{21}", b"a.{20}$", b"\\bx[ab]*a[ab]{21}"])
def test_blob_info_rejects_malformed_programs(pattern):
    """Every field verify_nfa_kernel indexes with is checked on the host
    (dgrep_blob_info_get, which dgrep_load_dfa calls first): header sizes,
    decoder children, leaf classes, U+FFFD's class, depths, word flags and
    position bits beyond npos. A program that fails any of them never reaches
    the device."""
    cp = dgrep.CompiledPattern(pattern)
    assert cp.partial
    ne = cp.nstates * cp.nclasses
    off = 288 + 4 * ne  # the program's first word
    prog = np.frombuffer(cp.blob[off:], dtype=np.uint32).copy()
    assert not _bad(cp.blob)
    npos, nw, nrc, nnodes, nctx = (int(x) for x in prog[1:6])

    def with_word(i, v):
        p = prog.copy()
        p[i] = np.uint32(v & 0xffffffff)
        return cp.blob[:off] + p.tobytes()

    assert _bad(with_word(0, 0x12345678))          # magic
    assert _bad(with_word(1, 257))                 # npos above the maximum
    assert _bad(with_word(2, nw + 1))              # nw != ceil(npos / 32)
    assert _bad(with_word(3, nrc + 1))             # size no longer matches the layout
    assert _bad(with_word(4, nnodes + 1))
    assert _bad(with_word(5, 2))                   # nctx neither 1 nor 4
    assert _bad(with_word(6, nrc))                 # U+FFFD's class out of range
    assert _bad(with_word(7, 2))                   # has_word not a flag
    child0 = 8
    assert _bad(with_word(child0 + ord("a"), nnodes))          # interior child beyond the trie
    assert _bad(with_word(child0 + ord("a"), 0))               # a child back to the root
    assert _bad(with_word(child0 + ord("a"), (-2 - nrc)))      # leaf class beyond nrc
    depth0 = child0 + nnodes * 256
    assert _bad(with_word(depth0, 1))                          # the root holds no pending byte
    word0 = depth0 + nnodes
    assert _bad(with_word(word0, 7))
    has0 = word0 + nrc
    if npos % 32:
        assert _bad(with_word(has0 + nw - 1, 1 << 31))         # a position bit beyond npos
    # truncated, and a DFA byte class / transition out of range
    assert _bad(cp.blob[:-4])
    bc = bytearray(cp.blob)
    bc[32 + ord("a")] = cp.nclasses
    assert _bad(bytes(bc))
    tr = bytearray(cp.blob)
    tr[288:292] = (cp.nstates).to_bytes(4, "little")
    assert _bad(bytes(tr))
