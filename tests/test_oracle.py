"""The oracle (CPU restatement of grep.go Map + Go regexp) checked against
everything that can pin it offline (the reference ships no
tests or vectors, and no Go toolchain exists here):

* Go-documented known answers (tests/go_cases.py);
* Python `re` (bytes mode) on randomly generated patterns and lines restricted
  to the dialect subset where Go and Python agree (ASCII inputs, no `{,n}`,
  no `\\s`, no `(?i)`+non-ASCII);
* the third-party `regex` module on Go-decoded pieces, for the Unicode
  patterns `re` cannot read (categories, (?i) orbits, invalid UTF-8);
* the SURVEY's ihash known answers and Go's JSON/Sprintf formats.
"""
import random
import re

import pytest

import oracle_lib as O
from go_cases import CASES


@pytest.mark.parametrize("pattern,line,expected", CASES)
def test_go_known_answers(pattern, line, expected):
    r = O.Regexp(pattern)
    if expected == "ERR":
        assert r.status == O.ORC_ESYNTAX, r.error
    elif expected == "UNSUP":
        assert r.status == O.ORC_EUNSUPPORTED, (r.status, r.error)
    else:
        assert r.status == O.ORC_OK, r.error
        assert r.match(line) == expected


def _rand_pattern(rnd, depth=0):
    atoms = ["a", "b", "c", "1", "_", ".", "\\.", "[ab]", "[^ab]", "[a-c]", "\\d", "\\D", "\\w", "\\W", "x",
             "^", "$", "\\b", "\\B", " "]
    if depth > 2 or rnd.random() < 0.45:
        s = rnd.choice(atoms)
    else:
        k = rnd.random()
        if k < 0.4:
            s = "".join(_rand_pattern(rnd, depth + 1) for _ in range(rnd.randint(2, 4)))
        elif k < 0.7:
            s = "|".join(_rand_pattern(rnd, depth + 1) for _ in range(rnd.randint(2, 3)))
            s = rnd.choice(["(%s)", "(?:%s)"]) % s
        else:
            s = "(%s)" % _rand_pattern(rnd, depth + 1)
    if s not in ("^", "$", "\\b", "\\B") and rnd.random() < 0.3:
        s += rnd.choice(["*", "+", "?", "{2}", "{1,3}", "{0,2}", "{2,}", "*?", "+?"])
    return s


def test_oracle_vs_python_re_random():
    rnd = random.Random(1234)
    alphabet = "abc1_ .-x"
    checked = 0
    for _ in range(1500):
        pat = _rand_pattern(rnd)
        if rnd.random() < 0.2:
            pat = "(?i)" + pat.upper()
        try:
            py = re.compile(pat.encode())
        except re.error:
            continue
        go = O.Regexp(pat.encode())
        assert go.status == O.ORC_OK, (pat, go.error)
        for _ in range(25):
            line = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(0, 12))).encode()
            if not line and "\\B" in pat:
                continue  # Python's \B never matches an empty string; Go's does (^\B$ matches "")
            assert go.match(line) == (py.search(line) is not None), (pat, line)
            checked += 1
    assert checked > 10000


def test_map_split_semantics():
    # strings.Split: k newlines -> k+1 lines; trailing '\n' gives an empty last line
    ln, st, le = O.grep_map(b"", b"")
    assert list(ln) == [1] and list(st) == [0] and list(le) == [0]
    ln, st, le = O.grep_map(b"", b"a\nb\n")
    assert list(ln) == [1, 2, 3] and list(st) == [0, 2, 4] and list(le) == [1, 1, 0]
    ln, st, le = O.grep_map(b"x", b"x\r\n\nyx")
    assert list(ln) == [1, 3] and list(le) == [2, 2]
    ln, _, _ = O.grep_map(b"a**", b"a\na\n")  # Go syntax error: no match on any line
    assert len(ln) == 0
    # recompile-per-line mode (grep.go:21 exactly) agrees with compile-once
    data = b"error\nok\nan error x\n\nerror"
    a = O.grep_map(b"error", data)
    b = O.grep_map(b"error", data, recompile_per_line=True)
    c = O.grep_map(b"error", data, threads=3)
    for x, y, z in zip(a, b, c):
        assert list(x) == list(y) == list(z)


def test_multithreaded_map_equals_single():
    rnd = random.Random(5)
    data = b"".join(rnd.choice([b"error", b"x", b"\n", b"ok", b" "]) for _ in range(20000))
    for threads in (2, 7, 16):
        for pat in (b"error", b"", b"^ok", b"x$"):
            a = O.grep_map(pat, data)
            b = O.grep_map(pat, data, threads=threads)
            for x, y in zip(a, b):
                assert list(x) == list(y)


def test_ihash_known_answers():
    # ihash("log.txt (line number #1)") = 228607205 -> partition 5
    assert O.ihash(b"log.txt (line number #1)") == 228607205
    assert O.ihash(b"log.txt (line number #1)") % 10 == 5
    assert O.ihash(b"log.txt (line number #2)") == 631071382
    assert O.ihash(b"log.txt (line number #2)") % 10 == 2


def test_key_and_json_format():
    assert O.format_key(b"log.txt", 12) == b"log.txt (line number #12)"
    assert O.json_kv(b"k", b"v") == b'{"Key":"k","Value":"v"}\n'
    # HTML escaping, control characters, invalid UTF-8 and U+2028 as encoding/json does
    assert O.json_kv(b"<&>", b"\t\"\\\x01\xff\xe2\x80\xa8") == \
        b'{"Key":"\\u003c\\u0026\\u003e","Value":"\\t\\"\\\\\\u0001\\ufffd\\u2028"}\n'


def test_memoized_matcher_equals_pike_vm_random():
    """orc_map_mt decides lines with the memoized Pike VM (a lazy DFA over the
    same program, oracle/goregexp.c orc_matcher_*); it must give exactly the
    plain Pike VM's verdicts (orc_map): random patterns from the compiler
    tests (Unicode classes, (?i), \\b, anchors, repeats) over random lines with
    invalid UTF-8, many lines per split so the cached transitions are reused."""
    from test_compiler import ALPHA, _rand_pattern

    rnd = random.Random(4242)
    checked = 0
    for _ in range(400):
        pat = _rand_pattern(rnd).encode()
        if O.compile_status(pat) == O.ORC_EUNSUPPORTED:
            continue
        data = b"".join(rnd.choice(ALPHA) for _ in range(rnd.randint(0, 600)))
        a = O.grep_map(pat, data)
        b = O.grep_map(pat, data, threads=2)
        for x, y in zip(a, b):
            assert list(x) == list(y), pat
        checked += 1
    assert checked > 300


def test_memoized_matcher_cache_flush():
    """A pattern whose lazy DFA outgrows the matcher's cache (2^15 states for
    [ab]*a[ab]{14}): the cache is flushed mid-line and rebuilt, verdicts equal
    the plain Pike VM's."""
    rnd = random.Random(7)
    lines = [bytes(rnd.choice(b"ab") for _ in range(rnd.randint(0, 300))) for _ in range(300)]
    data = b"\n".join(lines)
    for pat in (b"[ab]*a[ab]{14}", b"a[ab]{12}b$"):
        a = O.grep_map(pat, data)
        b = O.grep_map(pat, data, threads=2)
        assert len(a[0]) > 10
        for x, y in zip(a, b):
            assert list(x) == list(y), pat


def test_oracle_vs_regex_module_random():
    """A second, third-party engine on the patterns Python `re` cannot read:
    the `regex` module (VERSION0: simple case folding, like Go's (?i)) on each
    strings.Split piece decoded as Go decodes it (an invalid byte is U+FFFD),
    over random patterns from the compiler tests -- Unicode categories, (?i)
    over the k/K/U+212A and s/S/U+017F orbits, \\b, anchors, \\x{FFFD},
    repeats -- and random lines with invalid UTF-8. The pattern translation
    (Go's ASCII \\s \\d \\w \\b and POSIX classes spelled out; skipped: Unicode
    classes under (?i), where Go widens by FoldCategory) is the golden
    generator's (tests/golden/make_golden.py)."""
    import importlib.util
    import os
    import sys

    pytest.importorskip("regex")
    from test_compiler import ALPHA, _rand_pattern

    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(here, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    sys.modules.setdefault("make_golden", mg)
    spec.loader.exec_module(mg)
    rnd = random.Random(2718)
    checked = patterns = 0
    for _ in range(1500):
        pat = _rand_pattern(rnd).encode()
        if mg._pyregex_pattern(pat) is None:
            continue
        patterns += 1
        for _ in range(6):
            data = b"".join(rnd.choice(ALPHA) for _ in range(rnd.randint(0, 40)))
            got = mg._pyregex_lines(pat, data)
            if got is None:
                break
            want = [int(x) for x in O.grep_map(pat, data)[0]]
            assert got == want, (pat, data)
            checked += 1
    assert patterns > 500 and checked > 3000, (patterns, checked)
