"""The grep reduce task on the GPU (dgrep_reduce) vs a restatement of
map_reduce/worker.go:22-68,161-165 with grep.go:38-40's Reduce: decode every
json.Encoder KeyValue line, keep one value per distinct key (any of its values:
sort.Sort is unstable), write "key value\\n" (Go map order = unordered, so the
comparison is on key-sorted lines). End-to-end: Map + writeMapOutput
(dgrep_map_partitions) of several map tasks, then each partition's reduce."""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu


def go_decode_str(s: str) -> bytes:
    # json.loads keeps lone surrogates; Go's decoder turns each into U+FFFD
    out = []
    for ch in s:
        o = ord(ch)
        out.append("�" if 0xD800 <= o < 0xE000 else ch)
    return "".join(out).encode("utf-8")


def expected_reduce(data: bytes):
    """{raw key: set of raw values} of the input's KeyValue lines."""
    kv = {}
    for line in data.split(b"\n")[:-1]:
        d = json.loads(line)
        kv.setdefault(go_decode_str(d["Key"]), set()).add(go_decode_str(d["Value"]))
    return kv


def check_reduce(got: bytes, data: bytes):
    want = expected_reduce(data)
    lines = got.split(b"\n")
    assert lines[-1] == b""
    seen = set()
    for ln in lines[:-1]:
        # keys of the grep plugin never contain " ) " followed by a space-free
        # tail; split after the key, which ends with ')' + ' '
        k, sep, v = ln.partition(b") ")
        k += b")"
        assert sep, ln
        assert k in want, k
        assert v in want[k], (k, v)
        assert k not in seen, k
        seen.add(k)
    assert seen == set(want)


@pytest.fixture
def ctx(gpu_ctx):
    return gpu_ctx


def test_reduce_after_map_partitions(ctx):
    import dgrep

    files = {
        b"split-0.log": dgrep.synth_corpus_host(3 << 20, 21, 0),
        b"split-1.log": dgrep.synth_corpus_host(5 << 20, 22, 1) + b"\nerror <&> \"q\" \xff\xe2\x80\xa8 tail",
        "ünï-2.log".encode(): b"error one\nnothing\nerror \x01\x7f\n\nerror",
    }
    nreduce = 5
    ctx.load(b"error")
    parts = {f: ctx.map_partitions(f, d, nreduce) for f, d in files.items()}
    for r in range(nreduce):
        data = b"".join(parts[f][r] for f in files)
        got = ctx.reduce(data)
        check_reduce(got, data)
        # and against the Map output itself: every record of partition r, once
        want = set()
        for f, d in files.items():
            ln, st, le = O.grep_map(b"error", d, threads=8)
            for a, b, c in zip(ln.tolist(), st.tolist(), le.tolist()):
                key = O.format_key(f, a)
                if O.ihash(key) % nreduce == r:
                    want.add(go_decode_str(json.loads(O.json_kv(key, d[b:b + c]))["Key"]) + b" " +
                             go_decode_str(json.loads(O.json_kv(key, d[b:b + c]))["Value"]))
        assert set(got.split(b"\n")[:-1]) == want


def test_reduce_duplicate_keys(ctx):
    import dgrep

    ctx.load(b"error")
    d = dgrep.synth_corpus_host(1 << 20, 5, 0)
    p = ctx.map_partitions(b"same.log", d, 3)
    for r in range(3):
        data = p[r] + p[r] + p[r]  # the same map task's output three times
        got = ctx.reduce(data)
        assert got.count(b"\n") == p[r].count(b"\n")
        check_reduce(got, data)
    long_key = "k" * 100 + " (line number #7)"
    rows = [("a (line number #1)", "v1"), ("a (line number #1)", "v2"), (long_key, "x"), (long_key, "y"),
            ("b<&> (line number #2)", " �\U0001F600"), ("a (line number #1)", "v3")]
    data = b"".join(json.dumps({"Key": k, "Value": v}, separators=(",", ":"), ensure_ascii=True).encode() + b"\n"
                    for k, v in rows)
    got = ctx.reduce(data)
    assert got.count(b"\n") == 3
    check_reduce(got, data)


def test_reduce_escapes_and_surrogates(ctx):
    data = (b'{"Key":"\\u003cx\\u003e (line number #1)","Value":"\\ud83d\\ude00 \\ud800 \\udc00 \\/ \\b\\f\\n\\r\\t"}\n'
            b'{"Key":"y (line number #2)","Value":""}\n')
    got = ctx.reduce(data)
    # (a decoded value may hold '\n', so no line-wise check here)
    assert got.count(b"y (line number #2) \n") == 1
    assert b"<x> (line number #1) \xf0\x9f\x98\x80 \xef\xbf\xbd \xef\xbf\xbd / \x08\x0c\n\r\t\n" in got


def test_reduce_rejects_malformed(ctx):
    import dgrep

    for bad in (b'{"Key":"a","Value":"b"}\nnot json\n', b'{"Key":"a","Value":"b"}', b'{"Key":"a\x01","Value":"b"}\n',
                b'{"Value":"b","Key":"a"}\n'):
        with pytest.raises(dgrep.DgrepError):
            ctx.reduce(bad)
    assert ctx.reduce(b"") == b""


def test_reduce_newline_segments_and_short_lines(ctx):
    """Newline positions come from per-256-KiB-segment passes: inputs of
    0.5-3 MiB put lines across segment edges; keys and values of every
    length 0..9 put line edges at every dword phase of the output; escaped
    lines sit between plain ones."""
    rows = []
    for k in range(60000):
        key = "f%d (line number #%d)" % (k % 7, k)
        val = "v" * (k % 10) if k % 13 else "eé<%d>\"" % k
        rows.append((key if k % 11 else key.replace("f", "g "), val))
    data = b"".join(json.dumps({"Key": kk, "Value": v}, separators=(",", ":"), ensure_ascii=False).encode() + b"\n"
                    for kk, v in rows)
    for cut in (len(data), data.rfind(b"\n", 0, 600000) + 1):
        got = ctx.reduce(data[:cut])
        check_reduce(got, data[:cut])
