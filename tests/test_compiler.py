"""The product's pattern compiler (libdgrep.so: dgrep_compile, host-only)
against the oracle, on the CPU: every DFA it emits is interpreted by
tests/dfa_runner.py and must reproduce the oracle's Map output bit-exactly.
"""
import random

import numpy as np
import pytest

import dgrep
import oracle_lib as O
from dfa_runner import match_line, run_blob
from go_cases import CASES


def _compile(pattern):
    try:
        return dgrep.CompiledPattern(pattern)
    except dgrep.UnsupportedPattern:
        return "UNSUP"


@pytest.mark.parametrize("pattern,line,expected", CASES)
def test_go_known_answers_compiler(pattern, line, expected):
    cp = _compile(pattern)
    if expected == "UNSUP":
        assert cp == "UNSUP"
        return
    assert cp != "UNSUP", pattern
    if expected == "ERR":
        assert cp.go_syntax_error
        assert cp.flags & dgrep.DFA_MATCH_NONE
        return
    assert not cp.go_syntax_error
    if b"\n" in line:
        pytest.skip("line contains '\\n' (never happens after strings.Split)")
    assert match_line(cp, line) == expected


def _rand_pattern(rnd, depth=0):
    atoms = ["a", "b", "e", "r", "k", "s", "1", "_", " ", ".", "\\.", "[ab]", "[^ab]", "[a-e]", "[^\\x00-\\x7f]",
             "\\d", "\\w", "\\W", "\\s", "\\S", "\\pL", "\\PL", "\\p{Nd}", "é", "€", "\\x{FFFD}", "[é-ü]",
             "[[:alpha:]]", "[[:^space:]]", "\\b", "\\B", "^", "$", "\\A", "\\z", "(?i)k", "(?i:s)", "(?i)[a-c]",
             "\\Qa.b\\E", "x{2}"]
    if depth > 2 or rnd.random() < 0.4:
        s = rnd.choice(atoms)
    else:
        k = rnd.random()
        if k < 0.45:
            s = "".join(_rand_pattern(rnd, depth + 1) for _ in range(rnd.randint(2, 4)))
        elif k < 0.75:
            s = "(%s)" % "|".join(_rand_pattern(rnd, depth + 1) for _ in range(rnd.randint(2, 3)))
        else:
            s = "(?:%s)" % _rand_pattern(rnd, depth + 1)
    if rnd.random() < 0.3 and s not in ("^", "$", "\\b", "\\B", "\\A", "\\z"):
        s = "(?:%s)" % s + rnd.choice(["*", "+", "?", "{2}", "{0,2}", "{1,}", "*?"])
    return s


ALPHA = [b"a", b"b", b"e", b"r", b"k", b"K", b"s", b"S", b"1", b"_", b" ", b".", b"\n", b"\r", b"\t",
         "é".encode(), "€".encode(), "ü".encode(), b"\xe2\x84\xaa", b"\xc5\xbf", b"\xef\xbf\xbd",
         b"\xff", b"\x80", b"\xe2\x82", b"\xc3", b"\xf0\x9f\x98\x80", b"\xf0\x9f", b"\xed\xa0\x80", b"error"]


def test_compiler_vs_oracle_random():
    rnd = random.Random(99)
    checked = 0
    for it in range(700):
        pat = _rand_pattern(rnd).encode()
        ost = O.compile_status(pat)
        cp = _compile(pat)
        if ost == O.ORC_EUNSUPPORTED:
            assert cp == "UNSUP", pat
            continue
        assert cp != "UNSUP", (pat, ost)
        assert cp.go_syntax_error == (ost == O.ORC_ESYNTAX), pat
        for _ in range(12):
            data = b"".join(rnd.choice(ALPHA) for _ in range(rnd.randint(0, 24)))
            got = run_blob(cp, data)
            want = O.grep_map(pat, data)
            for g, w in zip(got, want):
                np.testing.assert_array_equal(g, w, err_msg=repr((pat, data)))
            checked += 1
    assert checked > 5000


CONFIG_PATTERNS = [
    (b"error", 7),
    (b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", None),
    (b"timeout while waiting for lock", None),
    (b"", 2),
]


@pytest.mark.parametrize("pattern,states", CONFIG_PATTERNS)
def test_config_patterns_on_synthetic_corpus(pattern, states):
    cp = dgrep.CompiledPattern(pattern)
    if states is not None:
        assert cp.nstates == states
    assert cp.nstates <= 256  # LDS-resident u8 path
    data = dgrep.synth_corpus_host(1 << 20, 3, 0)
    got = run_blob(cp, data)
    want = O.grep_map(pattern, data)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def test_blob_flags():
    assert dgrep.CompiledPattern("").flags & dgrep.DFA_MATCH_ALL
    assert dgrep.CompiledPattern("x*").flags & dgrep.DFA_MATCH_ALL
    assert dgrep.CompiledPattern("a**").flags == dgrep.DFA_GO_SYNTAX_ERROR | dgrep.DFA_MATCH_NONE
    assert dgrep.CompiledPattern("^\\b$").flags & dgrep.DFA_MATCH_NONE
    assert dgrep.CompiledPattern("[^\\x00-\\x{10FFFF}]").flags & dgrep.DFA_MATCH_NONE
    cp = dgrep.CompiledPattern("error")
    assert cp.start == 0 and cp.start_m == 1


def test_keyword_alternation_compiles():
    kws = dgrep.synth_keywords(4, 200)
    pat = b"(?i)(" + b"|".join(kws) + b")"
    cp = dgrep.CompiledPattern(pat)
    assert cp.nstates > 256  # config 4 needs the large-table path
    data = dgrep.synth_corpus_host(256 << 10, 4, 1)
    got = run_blob(cp, data)
    want = O.grep_map(pat, data)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


FOLD_ATOMS = ["(?i)é", "(?i)σ", "(?i)ς", "(?i)ß", "(?i)ẞ", "(?i)µ", "(?i)θ", "(?i)i", "(?i)İ", "(?i)ı", "(?i)д",
              "(?i)[α-ω]", "(?i)[^é]", "(?i)\\pL", "(?i)\\p{Lu}", "(?i)\\P{Ll}", "(?i)\\p{Mn}", "(?i)[\\x{100}-\\x{17f}]",
              "(?i)Å", "(?i)k", "(?i)[ǅ]", "é", "σ", "\\pL", "."]
FOLD_ALPHA = [s.encode() for s in ["é", "É", "e", "σ", "ς", "Σ", "ß", "ẞ", "ss", "µ", "μ", "Μ", "θ", "ϑ", "ϴ", "Θ", "i", "I",
                                   "İ", "ı", "д", "Д", "Å", "å", "Å", "k", "K", "K", "ǅ", "Ǆ", "ǆ", "ͅ", "ι", "ι", "ā", "Ā",
                                   "ſ", "x", " ", "1", "\n"]] + [b"\xff", b"\xce"]


def test_compiler_vs_oracle_unicode_folding():
    """(?i) over non-ASCII runes and folding categories (unicode.SimpleFold
    orbits, unicode.FoldCategory): the product's DFA and the oracle's Pike VM,
    both built from the generated Unicode 13.0 orbit table, agree on random
    patterns and lines (parity of the orbit table itself is unpinned)."""
    rnd = random.Random(7)
    checked = 0
    for it in range(250):
        pat = "".join(rnd.choice(FOLD_ATOMS) for _ in range(rnd.randint(1, 3)))
        if rnd.random() < 0.3:
            pat = "(%s)|%s" % (pat, rnd.choice(FOLD_ATOMS))
        pat = pat.encode()
        assert O.compile_status(pat) == O.ORC_OK, pat
        cp = _compile(pat)
        assert cp != "UNSUP", pat
        for _ in range(16):
            data = b"".join(rnd.choice(FOLD_ALPHA) for _ in range(rnd.randint(0, 10)))
            got = run_blob(cp, data)
            want = O.grep_map(pat, data)
            for g, w in zip(got, want):
                np.testing.assert_array_equal(g, w, err_msg=repr((pat, data)))
            checked += 1
    assert checked == 4000


def test_fold_orbit_table_shape():
    """The generated orbit table (tools/gen_unicode_tables.py): cyclic, closed,
    at most 4 runes per orbit, and the orbits Go documents."""
    import re as _re

    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "distributed-grep_amd", "csrc", "compiler", "unicode_tables.inc")).read()
    m = _re.search(r"dg_fold\[\] = \{([^}]*)\}", src)
    vals = [int(x, 16) for x in m.group(1).split(",")]
    nxt = dict(zip(vals[0::2], vals[1::2]))

    def orbit(r):
        out, x = {r}, nxt.get(r)
        while x is not None and x != r:
            out.add(x)
            x = nxt[x]
        return out

    for r in nxt:
        assert nxt[r] in nxt and r in orbit(nxt[r]) and len(orbit(r)) <= 4
    assert orbit(ord("k")) == {ord("k"), ord("K"), 0x212A}
    assert orbit(ord("s")) == {ord("s"), ord("S"), 0x17F}
    assert orbit(0x3C3) == {0x3A3, 0x3C3, 0x3C2}
    assert orbit(0xDF) == {0xDF, 0x1E9E}
    assert orbit(0x3B8) == {0x398, 0x3B8, 0x3D1, 0x3F4}
    assert orbit(0x345) == {0x345, 0x399, 0x3B9, 0x1FBE}
    assert 0x130 not in nxt and 0x131 not in nxt and orbit(ord("i")) == {ord("i"), ord("I")}
