#!/usr/bin/env python3
"""Generate tests/golden/vectors.json — the committed golden vectors of the
Map hot path (application/grep.go:13-36) and of its after-Map parity sink.

The reference ships no tests, fixtures or golden vectors, and its algorithm
lives in the Go standard library (regexp, strings.Split, fmt, hash/fnv), which
is not in this image. So each vector's expected output comes
from the oracle's restatement (oracle/, the CPU checker), and the script only
writes a vector after pinning it against every independent witness that is
present here and agrees with Go on that case:

* ``python-re``: Python 3 ``re`` in bytes mode, per piece of
  ``data.split(b"\\n")`` (the pieces strings.Split gives), on the dialect
  subset where Go RE2 and Python agree (ASCII data, no ``\\s`` (Python adds
  ``\\v``), no ``{,n}``, no Unicode classes);
* ``gnu-grep``: ``LC_ALL=C grep -a -n -E`` for ERE-compatible patterns (grep
  never reports the empty piece after a trailing '\\n'; that piece is checked
  against the oracle alone);
* ``perl-re``: perl 5.34's regex engine (Unicode 13.0, like Go 1.18) for
  patterns built only from Unicode script / category classes, literals and
  ``+ * ?``, without (?i) (perl folds fully, Go simply): each piece decoded as
  Go decodes it (an invalid byte is U+FFFD), ``\\p{Name}`` of a script given to
  perl as ``\\p{Script=Name}`` (perl's bare ``\\p{Greek}`` means
  Script_Extensions).

* ``py-regex``: the ``regex`` module (a third-party engine, VERSION0 = simple
  case folding like Go's ``(?i)``) on each piece decoded as Go decodes it, for
  patterns it reads as Go does once Go's ASCII ``\\s \\d \\w \\b`` and
  ``\\x{...}`` are spelled out (``_pyregex_pattern``): Unicode classes,
  scripts, folding and invalid UTF-8 data (not a Unicode class under ``(?i)``:
  Go widens it by FoldCategory / FoldScript, regex does not).

A vector with no applicable witness (Go syntax errors, Unicode classes under (?i)) is still written, marked ``"witnesses": []`` — parity
unpinned for that case.

Run from the repo root after `make` (needs oracle/liboracle.so, and
libdgrep.so for the host twin of the synthetic corpus generator):
    python tests/golden/make_golden.py
"""
import base64
import json
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "distributed-grep_amd"))

import oracle_lib as O  # noqa: E402
import dgrep  # noqa: E402  (host-only calls: corpus + keyword generator)

N_REDUCE = 10  # main/coordinator_launch.go:17


def _py_ok(pattern: bytes, data: bytes) -> bool:
    if any(b >= 0x80 for b in data) or any(b >= 0x80 for b in pattern):
        return False
    if re.search(rb"\\[sSpPzQEx]|\{,|\(\?[a-zA-Z]*U|\[\[:", pattern):
        return False
    try:
        re.compile(pattern)
    except re.error:
        return False
    return O.compile_status(pattern) == O.ORC_OK


def _grep_ok(pattern: bytes, data: bytes) -> bool:
    if shutil.which("grep") is None:
        return False
    if any(b >= 0x80 for b in data) or any(b >= 0x80 for b in pattern):
        return False
    # the ERE subset shared with RE2: no Perl escapes, flags, lazy operators
    if re.search(rb"\\[dDwWsSbBAzpPQExr]|\(\?|\*\?|\+\?|\?\?|\{,", pattern):
        return False
    if b"\x00" in data or O.compile_status(pattern) != O.ORC_OK:
        return False
    return True


def _python_lines(pattern: bytes, data: bytes):
    rx = re.compile(pattern)
    return [i + 1 for i, line in enumerate(data.split(b"\n")) if rx.search(line)]


def _grep_lines(pattern: bytes, data: bytes):
    p = subprocess.run(["grep", "-a", "-n", "-E", "-e", pattern.decode("ascii"), "-"], input=data,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=dict(os.environ, LC_ALL="C"))
    if p.returncode not in (0, 1):
        return None
    return [int(ln.split(b":", 1)[0]) for ln in p.stdout.split(b"\n") if ln]


_SCRIPT_CLASS = re.compile(rb"\\[pP]\{(\^?)([A-Za-z_]+)\}")


def _perl_ok(pattern: bytes, data: bytes) -> bool:
    if shutil.which("perl") is None or O.compile_status(pattern) != O.ORC_OK:
        return False
    if not _SCRIPT_CLASS.search(pattern):
        return False
    rest = _SCRIPT_CLASS.sub(b"", pattern)
    return re.fullmatch(rb"[A-Za-z0-9 +*?^$]*", rest) is not None


def _go_decode(line: bytes) -> str:
    """Go's utf8.DecodeRune walk: a byte that does not start a valid sequence is U+FFFD, width 1."""
    out, i = [], 0
    while i < len(line):
        for w in (1, 2, 3, 4):
            try:
                ch = line[i:i + w].decode("utf-8")
            except UnicodeDecodeError:
                continue
            if len(ch) == 1:
                out.append(ch)
                i += w
                break
        else:
            out.append("\ufffd")
            i += 1
    return "".join(out)


def _perl_lines(pattern: bytes, data: bytes):
    categories = {"L", "Lu", "Ll", "Lt", "Lm", "Lo", "M", "Mn", "Mc", "Me", "N", "Nd", "Nl", "No", "P", "S", "Z",
                  "C", "Cc", "Cf", "Co", "Cs", "Any"}

    def conv(m):
        neg, name = m.group(1), m.group(2)
        if name.decode() in categories:
            return m.group(0)
        return b"\\" + m.group(0)[1:2] + b"{" + neg + b"Script=" + name + b"}"

    pp = _SCRIPT_CLASS.sub(conv, pattern).decode()
    lines = [_go_decode(x) for x in data.split(b"\n")]
    prog = 'binmode STDIN, ":encoding(UTF-8)"; my $re = qr/$ARGV[0]/; my $n = 0; ' \
           'while (my $l = <STDIN>) { chomp $l; $n++; print "$n\\n" if $l =~ $re; }'
    inp = "\n".join(lines) + "\n"
    p = subprocess.run(["perl", "-e", prog, pp], input=inp.encode("utf-8", "surrogatepass"), stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE)
    if p.returncode != 0:
        return None
    return [int(x) for x in p.stdout.split()]


# ``py-regex``: the third-party ``regex`` module (VERSION0: simple case
# folding, as Go's (?i)) in str mode on each piece decoded as Go decodes it,
# for patterns it reads as Go does once Go's ASCII-only Perl and POSIX classes
# and \x{...} are spelled out; skipped: those Perl escapes inside a bracket
# class, Unicode classes under (?i), Go syntax errors (a parse result, not a
# match).
_ASCII_ESC = {
    "s": r"[\t\n\f\r ]", "S": r"[^\t\n\f\r ]", "d": r"[0-9]", "D": r"[^0-9]",
    "w": r"[0-9A-Za-z_]", "W": r"[^0-9A-Za-z_]",
    "b": r"(?:(?<=[0-9A-Za-z_])(?![0-9A-Za-z_])|(?<![0-9A-Za-z_])(?=[0-9A-Za-z_]))",
    "B": r"(?:(?<=[0-9A-Za-z_])(?=[0-9A-Za-z_])|(?<![0-9A-Za-z_])(?![0-9A-Za-z_]))",
    "z": r"\Z",
}


_POSIX = {"upper": "A-Z", "lower": "a-z", "digit": "0-9", "alpha": "A-Za-z", "alnum": "0-9A-Za-z",
          "xdigit": "0-9A-Fa-f", "space": "\\t\\n\\v\\f\\r ", "blank": "\\t ", "word": "0-9A-Za-z_"}


def _pyregex_pattern(pattern: bytes):
    """Go pattern -> an equivalent pattern for the regex module, or None."""
    try:
        import regex  # noqa: F401
        p = pattern.decode("utf-8")
    except (ImportError, UnicodeDecodeError):
        return None
    if O.compile_status(pattern) != O.ORC_OK or "\\Q" in p:
        return None
    # Go's POSIX classes are ASCII (regex reads them as Unicode properties)
    for name, rng in _POSIX.items():
        p = p.replace("[:%s:]" % name, rng)
    if "[:" in p:
        return None
    # Go folds a class under (?i) through unicode.FoldCategory / FoldScript
    # ((?i)\p{Greek} also matches U+00B5 and U+0345); regex does not
    if "(?i" in p and ("\\p" in p or "\\P" in p):
        return None
    out, i, in_class = [], 0, False
    while i < len(p):
        c = p[i]
        if c == "\\" and i + 1 < len(p):
            e = p[i + 1]
            if e == "x" and i + 2 < len(p) and p[i + 2] == "{":
                j = p.index("}", i + 3)
                out.append("\\U%08x" % int(p[i + 3:j], 16))
                i = j + 1
                continue
            if e in _ASCII_ESC:
                if in_class:
                    return None
                out.append(_ASCII_ESC[e])
            else:
                out.append(p[i:i + 2])
            i += 2
            continue
        if c == "[" and not in_class:
            in_class = True
            out.append(c)
            i += 1
            # a leading ']' (or '^]') is a literal
            if p[i:i + 1] == "^":
                out.append("^")
                i += 1
            if p[i:i + 1] == "]":
                out.append("\\]")
                i += 1
            continue
        if c == "]" and in_class:
            in_class = False
        out.append(c)
        i += 1
    return "".join(out)


def _pyregex_lines(pattern: bytes, data: bytes):
    import regex

    rp = _pyregex_pattern(pattern)
    try:
        rx = regex.compile(rp, flags=regex.VERSION0)
    except regex.error:
        return None
    return [i + 1 for i, line in enumerate(data.split(b"\n")) if rx.search(_go_decode(line))]


_INPUTS = []


def _input_index(data: bytes) -> int:
    """Inputs are stored once (vectors reference them by index)."""
    for i, d in enumerate(_INPUTS):
        if d == data:
            return i
    _INPUTS.append(data)
    return len(_INPUTS) - 1


def vector(name: str, filename: str, pattern: bytes, data: bytes):
    ln, st, le = O.grep_map(pattern, data)
    ln, st, le = [int(x) for x in ln], [int(x) for x in st], [int(x) for x in le]
    witnesses = []
    if _py_ok(pattern, data):
        assert _python_lines(pattern, data) == ln, (name, "python-re disagrees with the oracle")
        witnesses.append("python-re")
    if _grep_ok(pattern, data):
        g = _grep_lines(pattern, data)
        if g is not None:
            last = data.count(b"\n") + 1
            want = [x for x in ln if not (x == last and (data.endswith(b"\n") or not data))]
            assert g == want, (name, "gnu-grep disagrees with the oracle", g[:10], want[:10])
            witnesses.append("gnu-grep")
    if _pyregex_pattern(pattern) is not None:
        g = _pyregex_lines(pattern, data)
        if g is not None:
            assert g == ln, (name, "py-regex disagrees with the oracle", g[:10], ln[:10])
            witnesses.append("py-regex")
    if _perl_ok(pattern, data):
        g = _perl_lines(pattern, data)
        if g is not None:
            assert g == ln, (name, "perl-re disagrees with the oracle", g[:10], ln[:10])
            witnesses.append("perl-re")
    fn = filename.encode()
    keys = [O.format_key(fn, x) for x in ln]
    values = [data[s:s + n] for s, n in zip(st, le)]
    # after Reduce (grep.go:38-40 returns values[0]; keys are unique per file):
    # each KeyValue crosses the shuffle as a json.Encoder line (worker.go:92-93:
    # an invalid UTF-8 byte becomes �) read back by json.Decoder
    # (worker.go:53-56), then one "%v %v\n" line per key (worker.go:111-124,
    # 163-165), compared key-sorted because the reference writes them in Go map
    # order (worker.go:163)
    reduce_out = O.reduce_lines(keys, values)
    return {
        "name": name,
        "filename": filename,
        "pattern_b64": base64.b64encode(pattern).decode(),
        "input": _input_index(data),
        "go_syntax_error": O.compile_status(pattern) == O.ORC_ESYNTAX,
        "line_no": ln,
        "start": st,
        "len": le,
        "keys_b64": [base64.b64encode(k).decode() for k in keys],
        "reduce_b64": base64.b64encode(reduce_out).decode(),
        "partition": [O.ihash(k) % N_REDUCE for k in keys],  # map_reduce/worker.go:13-17,84
        "witnesses": witnesses,
    }


EDGE_DATA = [
    b"", b"\n", b"\n\n", b"error", b"error\n", b"x\nerror", b"\nerror\n\n", b"ERROR\nError\nerror\n",
    b"a\r\nerror\r\n", b"key\nk\n", b"an error\n" * 3 + b"no", b"2024-01-02T03:04:05.678 WARN auth_svc: x\n",
    b"\xff\xfe\n\xe2\x82\xac\n\xe2\x82\n\xef\xbf\xbd\n", b"\xe2\x84\xaaey\n\xc5\xbftop\nKEY\nstop\n",
    b"a" * 3000 + b"error" + b"b" * 3000 + b"\nerror", b"tab\there\nvt\x0bhere\n", b"\x00error\x00\n",
    "Αθήνα error\nµ micro\nͅ ypogegrammeni\nι iota\n中文 log\nМосква\nK kelvin\n123\n\n".encode() + b"\xce\xff\n",
]

EDGE_PATTERNS = [
    b"", b"error", b"^$", b"^", b"$", b"(?i)error", b"(?i)key", b"(?i)stop", b"^error$", b"error$", b"^e",
    b"\\berror\\b", b"\\Berr", b"e(r|x)+o", b"[^a-z ]{3}", b"\\x{FFFD}", b"\\x{20AC}", b"\\s", b"\\d+",
    b"\\w{4}", b"(WARN|ERROR) [a-z_]+", b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"a**", b"(", b"x{1001}",
    b"\\r$", b"(?s).", b"[[:upper:]]", b"\\pL", b"[a-c]+r",
    b"\\p{Greek}", b"(?i)\\p{Greek}", b"\\P{Latin}", b"^\\p{Han}+", b"\\p{Cyrillic}+$", b"(?i)\\p{Common}",
    b"\\p{Greek} \\p{Latin}+", b"\\p{Bogus}",
]


def main():
    vecs = []
    for i, d in enumerate(EDGE_DATA):
        for p in EDGE_PATTERNS:
            if O.compile_status(p) == O.ORC_EUNSUPPORTED:
                continue
            vecs.append(vector("edge%02d/%s" % (i, p.decode("latin-1")), "f.log", p, d))
    # windows of the synthetic corpus (SURVEY §8d generator, the seeds of C1-C4)
    for tag, seed, pats in (("c1", 1, [b"error"]), ("c2", 2, [b"error", b"timeout while waiting for lock"]),
                            ("c3", 3, [b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"(WARN|ERROR) [a-z_]+"])):
        data = dgrep.synth_corpus_host(48 << 10, seed, 0)
        for p in pats:
            vecs.append(vector("synth-%s/%s" % (tag, p.decode()), "log.txt", p, data))
    kws = dgrep.synth_keywords(4, 40)
    p4 = b"(?i)(" + b"|".join(kws) + b")"
    vecs.append(vector("synth-c4/40-keyword (?i) alternation", "log.txt", p4,
                       dgrep.synth_corpus_host(64 << 10, 4, 1)))
    out = os.path.join(HERE, "vectors.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "n_reduce": N_REDUCE,
                   "inputs_b64": [base64.b64encode(d).decode() for d in _INPUTS], "vectors": vecs}, f,
                  separators=(",", ":"))
        f.write("\n")
    pinned = sum(1 for v in vecs if v["witnesses"])
    print("wrote %d vectors (%d pinned by an independent witness) to %s" % (len(vecs), pinned, out))


if __name__ == "__main__":
    main()
