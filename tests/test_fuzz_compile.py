"""ASan/UBSan fuzz of the product's pattern compiler (csrc/compiler, the code
dgrep_compile runs on the untrusted pattern string inside the worker; the
reference compiles the same user string with regexp.Compile at
application/grep.go:21). tests/fuzz/compile_fuzz is the compiler built with
-fsanitize=address,undefined; it must compile every input to a documented
status (OK with a well-formed blob, UNSUPPORTED, TOO_LARGE) and exit cleanly.
Inputs: random bytes, regex-shaped token soups (hypothesis, derandomized),
and the Go-documented cases of tests/go_cases.py."""
import os
import random
import struct
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as hs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIR = os.path.join(ROOT, "tests", "fuzz")
EXE = os.path.join(DIR, "compile_fuzz")

TOKENS = [b"a", b"b", b"x", b"K", b"\xc5\xbf", b"\xe2\x84\xaa", b"\xff", b"\xe2\x82", b".", b"^", b"$", b"\\A", b"\\z",
          b"\\b", b"\\B", b"\\d", b"\\w", b"\\s", b"\\D", b"\\W", b"\\S", b"\\pL", b"\\p{Greek}", b"\\PN", b"\\x{FFFD}",
          b"\\x41", b"\\Q.*\\E", b"[a-z]", b"[^a-c]", b"[[:alpha:]]", b"[\\d_-]", b"[]a]", b"[a-]", b"(", b")", b"(?:",
          b"(?i)", b"(?s)", b"(?m)", b"(?U)", b"(?i:", b"(?P<n>", b"|", b"*", b"+", b"?", b"*?", b"+?", b"{2}", b"{1,3}",
          b"{0,}", b"{1001}", b"{2,1}", b"\\", b"\\n", b"\\t", b"\\1", b"{", b"}", b"[", b"]", b"\\C", b"\\pZ", b"\\p{^L}"]


def _build():
    subprocess.run(["make", "-s", "-C", DIR], check=True, capture_output=True)


def _feed(patterns):
    payload = b"".join(struct.pack("<I", len(p)) + p for p in patterns)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([EXE], input=payload, capture_output=True, timeout=600, env=env)
    return p


def _soup(rnd, n):
    return b"".join(rnd.choice(TOKENS) for _ in range(n))


def test_fuzz_random_bytes_and_token_soups():
    _build()
    rnd = random.Random(20261016)
    pats = [bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 24))) for _ in range(800)]
    pats += [_soup(rnd, rnd.randrange(1, 12)) for _ in range(1500)]
    import go_cases

    pats += [c[0] if isinstance(c[0], bytes) else str(c[0]).encode() for c in getattr(go_cases, "CASES", [])]
    p = _feed(pats)
    assert p.returncode == 0, (p.returncode, p.stderr.decode(errors="replace")[-3000:])
    assert b"ERROR: AddressSanitizer" not in p.stderr and b"runtime error" not in p.stderr
    assert p.stdout.startswith(b"%d patterns" % len(pats)), p.stdout


@settings(max_examples=12, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
@given(hs.lists(hs.lists(hs.sampled_from(TOKENS), min_size=1, max_size=10).map(b"".join), min_size=20, max_size=40))
def test_fuzz_hypothesis_batches(batch):
    _build()
    p = _feed(batch)
    assert p.returncode == 0, (batch, p.stderr.decode(errors="replace")[-2000:])
    assert b"AddressSanitizer" not in p.stderr and b"runtime error" not in p.stderr
