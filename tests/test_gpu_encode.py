"""Partition + intermediate writer on the GPU (dgrep_map_partitions /
dgrep_encode_device) vs the oracle's restatement of map_reduce/worker.go:78-109:
partition p of a map task = the json.Encoder lines of its KeyValues with
ihash(Key) % nReduce == p, in Map output order. Bit-exact.

The CPU-only test pins the oracle's ihash with an independent FNV-1a and the
known answers recorded in SURVEY.md §8a."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_lib as O  # noqa: E402

FNAMES = [b"log.txt", b"a<b>&\"q\\.log", "ünï€.log".encode(), b"bad\xff\xfe.log", b"",
          b"tab\there\n.log"]

SPECIAL = b"\n".join([
    b"error <tag> & \"quoted\" \\ back\tslash\r\x01\x1f\x7f end",
    b"error \xff\xc3(\xe2\x28\xa1 invalid utf-8",
    b"\xe2\x80\xa8 error \xe2\x80\xa9 separators",
    b"error emoji \xf0\x9f\x98\x80 overlong \xc0\xaf surrogate \xed\xa0\x80",
    b"no match here",
    b"",
    b"error",
    b"error at the end, truncated rune \xe2\x82",
])


def _fnv1a_ihash(key: bytes) -> int:
    h = 2166136261
    for b in key:
        h = ((h ^ b) * 16777619) & 0xFFFFFFFF
    return h & 0x7FFFFFFF


def test_oracle_ihash_pinned():
    # SURVEY.md §8a known answers; an independent FNV-1a restatement agrees
    assert O.ihash(b"log.txt (line number #1)") == 228607205
    assert O.ihash(b"log.txt (line number #2)") == 631071382
    assert 228607205 % 10 == 5 and 631071382 % 10 == 2
    for k in (b"", b"x", "ü".encode(), bytes(range(256))):
        assert O.ihash(k) == _fnv1a_ihash(k)
    assert O.format_key(b"f.log", 12) == b"f.log (line number #12)"


def _go_json_str_witness(b: bytes) -> bytes:
    """Go encoding/json string encoding (HTML escaping on) derived from Python's
    json module for VALID UTF-8: Python leaves <>& and U+2028/9 alone and uses
    \\b \\f short forms, Go 1.18 does not."""
    import json as J

    s = J.dumps(b.decode("utf-8"), ensure_ascii=False)
    s = s.replace("\\b", "\\u0008").replace("\\f", "\\u000c")
    s = s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
    s = s.replace("\u2028", "\\u2028").replace("\u2029", "\\u2029")
    return s.encode("utf-8")


def test_oracle_json_kv_vs_python_json():
    """The oracle's json.Encoder restatement against an independent witness on
    valid UTF-8 (invalid UTF-8 -> \\ufffd per byte stays pinned only by the
    restatement of utf8.DecodeRune)."""
    import random

    rnd = random.Random(5)
    pool = ["a", "Z", " ", "<", ">", "&", '"', "\\", "/", "\n", "\r", "\t", "\b", "\f", "\x00", "\x1f", "\x7f",
            "é", "€", "\u2028", "\u2029", "\U0001F600", "#", "(", ")"]
    for _ in range(400):
        k = "".join(rnd.choice(pool) for _ in range(rnd.randrange(0, 12))).encode()
        v = "".join(rnd.choice(pool) for _ in range(rnd.randrange(0, 40))).encode()
        want = b'{"Key":' + _go_json_str_witness(k) + b',"Value":' + _go_json_str_witness(v) + b"}\n"
        assert O.json_kv(k, v) == want, (k, v)


def expected_partitions(pattern: bytes, filename: bytes, data: bytes, nreduce: int):
    ln, st, le = O.grep_map(pattern, data, threads=16)
    parts = [bytearray() for _ in range(nreduce)]
    for a, b, c in zip(ln.tolist(), st.tolist(), le.tolist()):
        key = O.format_key(filename, a)
        parts[O.ihash(key) % nreduce] += O.json_kv(key, data[b:b + c])
    return [bytes(p) for p in parts]


@pytest.fixture
def ctx(gpu_ctx):
    # the session context (conftest): torch initialises the GPU before libdgrep
    return gpu_ctx


@pytest.mark.gpu
@pytest.mark.parametrize("nreduce", [1, 7, 10, 256])
@pytest.mark.parametrize("filename", FNAMES)
def test_partitions_special_bytes(ctx, filename, nreduce):
    for pattern in (b"error", b"", b"^$", b"zzz_never"):
        ctx.load(pattern)
        got = ctx.map_partitions(filename, SPECIAL, nreduce)
        assert got == expected_partitions(pattern, filename, SPECIAL, nreduce), (pattern, filename, nreduce)


@pytest.mark.gpu
@pytest.mark.parametrize("size", [0, 1, 4 << 20, 12 << 20])
def test_partitions_synth_corpus(ctx, size):
    import dgrep

    data = dgrep.synth_corpus_host(size, 9, 1) if size else b""
    for pattern in (b"error", b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b""):
        ctx.load(pattern)
        got = ctx.map_partitions(b"split-0003.log", data, 10)
        want = expected_partitions(pattern, b"split-0003.log", data, 10)
        assert len(got) == len(want)
        for p, (g, w) in enumerate(zip(got, want)):
            assert g == w, (pattern, size, p, len(g), len(w))


@pytest.mark.gpu
def test_encode_device_capacity_retry(ctx):
    import torch
    import dgrep

    n = 8 << 20
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.synth(buf.data_ptr(), n, 3, 0)
    ctx.load(b"error")
    cap = 1 << 20
    ln = torch.empty(cap, dtype=torch.int64, device="cuda")
    st = torch.empty(cap, dtype=torch.int64, device="cuda")
    le = torch.empty(cap, dtype=torch.int64, device="cuda")
    cnt = ctx.scan_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cap)
    assert 0 < cnt <= cap
    small = torch.empty(1000, dtype=torch.uint8, device="cuda")
    b, e, total = ctx.encode_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, "x.log", 10,
                                    small.data_ptr(), small.numel())
    assert total > small.numel()
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    b, e, total2 = ctx.encode_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, "x.log", 10,
                                     out.data_ptr(), total)
    assert total2 == total
    raw = out.cpu().numpy().tobytes()
    want = expected_partitions(b"error", b"x.log", buf.cpu().numpy().tobytes(), 10)
    assert [raw[x:y] for x, y in zip(b, e)] == want
    assert ctx.last_encode_ms() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("filename", [b"f" * 2100, b"dir/" + b"<&>" * 700, b"a"])
def test_partitions_head_sizes(ctx, filename):
    """The wave writer keeps the line head `{"Key":"<file> (line number #` in
    LDS (2 KiB); longer file names take the per-thread writer. Short and empty
    lines put line edges at every dword phase of the output."""
    import dgrep

    lines = [b"error" + b"x" * (k % 9) for k in range(3000)] + [b"error", b"", b"error\xff\"<"]
    data = b"\n".join(lines) + b"\n" + dgrep.synth_corpus_host(1 << 20, 4, 0)
    ctx.load(b"error|^$")
    got = ctx.map_partitions(filename, data, 7)
    assert got == expected_partitions(b"error|^$", filename, data, 7)
