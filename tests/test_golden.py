"""The committed golden vectors (tests/golden/vectors.json, made by
tests/golden/make_golden.py) against the oracle, the product's pattern
compiler and — on the GPU box — the HIP scan through the C ABI.

Each vector holds an input split, a pattern and the Map output of
application/grep.go:13-36 (1-based line numbers, byte starts and lengths of
the matching lines), the keys grep.go:25 builds, the key-sorted Reduce output
lines (map_reduce/worker.go:111-124,163-165) and the ihash partitions
(worker.go:13-17). Vectors whose "witnesses" list is non-empty were checked,
when generated, against Python `re`, GNU grep, perl's regex engine and/or the
`regex` module (test_witnesses_still_agree re-runs the Python ones); the rest
are parity unpinned.
"""
import base64
import json
import os

import numpy as np
import pytest

import dgrep
import oracle_lib as O
from dfa_runner import run_blob

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "vectors.json")) as _f:
    GOLDEN = json.load(_f)
INPUTS = [base64.b64decode(x) for x in GOLDEN["inputs_b64"]]
VECTORS = GOLDEN["vectors"]


def _unpack(v):
    return base64.b64decode(v["pattern_b64"]), INPUTS[v["input"]]


def _want(v):
    return (np.array(v["line_no"], np.uint64), np.array(v["start"], np.uint64), np.array(v["len"], np.uint64))


def _eq(got, want, name):
    for g, w in zip(got, want):
        np.testing.assert_array_equal(np.asarray(g).astype(np.uint64), w.astype(np.uint64), err_msg=name)


def test_golden_shape():
    assert len(VECTORS) > 400
    pinned = [v for v in VECTORS if v["witnesses"]]
    assert len(pinned) > 550
    assert any(v["go_syntax_error"] for v in VECTORS)
    assert any(v["name"].startswith("synth-c3") and v["line_no"] for v in VECTORS)


def test_witnesses_still_agree():
    """The Python witnesses re-run on every vector they pinned: Python `re` per
    strings.Split piece, and the `regex` module on Go-decoded pieces."""
    import importlib.util
    import re
    import sys

    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    sys.modules.setdefault("make_golden", mg)
    spec.loader.exec_module(mg)
    n = {"python-re": 0, "py-regex": 0}
    for v in VECTORS:
        p, d = _unpack(v)
        if "python-re" in v["witnesses"]:
            rx = re.compile(p)
            got = [i + 1 for i, line in enumerate(d.split(b"\n")) if rx.search(line)]
            assert got == v["line_no"], v["name"]
            n["python-re"] += 1
        if "py-regex" in v["witnesses"]:
            assert mg._pyregex_lines(p, d) == v["line_no"], v["name"]
            n["py-regex"] += 1
    assert n["python-re"] > 300 and n["py-regex"] > 500, n


def test_oracle_reproduces_golden():
    for v in VECTORS:
        p, d = _unpack(v)
        _eq(O.grep_map(p, d), _want(v), v["name"])


def test_compiler_dfa_reproduces_golden():
    for v in VECTORS:
        p, d = _unpack(v)
        cp = dgrep.CompiledPattern(p)
        assert cp.go_syntax_error == v["go_syntax_error"], v["name"]
        _eq(run_blob(cp, d), _want(v), v["name"])


def test_keys_partitions_and_reduce_lines():
    for v in VECTORS:
        p, d = _unpack(v)
        fn = v["filename"]
        keys = [dgrep.format_key(fn, n).encode() for n in v["line_no"]]
        assert keys == [base64.b64decode(k) for k in v["keys_b64"]], v["name"]
        assert [O.ihash(k) % GOLDEN["n_reduce"] for k in keys] == v["partition"], v["name"]
        vals = [d[s:s + n] for s, n in zip(v["start"], v["len"])]
        assert O.reduce_lines(keys, vals) == base64.b64decode(v["reduce_b64"]), v["name"]


def test_reduce_lines_carry_the_json_roundtrip():
    """The after-Reduce lines are what json.Encoder -> json.Decoder leave of a
    value (map_reduce/worker.go:92-93, 53-56): every invalid UTF-8 byte is one
    U+FFFD, so the reduce output is valid UTF-8 even where the line was not."""
    bad = [v for v in VECTORS if any(b >= 0x80 for b in INPUTS[v["input"]]) and v["line_no"]]
    assert bad
    for v in VECTORS:
        red = base64.b64decode(v["reduce_b64"])
        red.decode("utf-8")  # strict: raises on raw invalid bytes
    # edge12 = b"\xff\xfe\n\xe2\x82\xac\n\xe2\x82\n\xef\xbf\xbd\n": "" matches every line
    v = next(v for v in VECTORS if v["name"] == "edge12/")
    want = [b"f.log (line number #1) \xef\xbf\xbd\xef\xbf\xbd\n", b"f.log (line number #2) \xe2\x82\xac\n",
            b"f.log (line number #3) \xef\xbf\xbd\xef\xbf\xbd\n", b"f.log (line number #4) \xef\xbf\xbd\n",
            b"f.log (line number #5) \n"]
    assert base64.b64decode(v["reduce_b64"]) == b"".join(sorted(want))


@pytest.mark.gpu
def test_gpu_map_partitions_reduce_reproduces_golden(gpu_ctx):
    """End to end after Reduce, on the GPU: Map + writeMapOutput
    (dgrep_map_partitions, nReduce 10 as main/coordinator_launch.go:17) then one
    reduce task per partition (dgrep_reduce); the union of the mr-out-<r> lines,
    key-sorted, must equal the vector's reduce lines."""
    nred = GOLDEN["n_reduce"]
    for v in VECTORS:
        p, d = _unpack(v)
        gpu_ctx.load(p)
        parts = gpu_ctx.map_partitions(v["filename"], d, nred)
        lines = []
        for r, part in enumerate(parts):
            out = gpu_ctx.reduce(part)
            assert out == b"" or out.endswith(b"\n"), (v["name"], r)
            lines += [x + b"\n" for x in out.split(b"\n")[:-1]]
        assert b"".join(sorted(lines)) == base64.b64decode(v["reduce_b64"]), v["name"]


@pytest.mark.gpu
def test_gpu_scan_reproduces_golden(gpu_ctx):
    for v in VECTORS:
        p, d = _unpack(v)
        gpu_ctx.load(p)
        _eq(gpu_ctx.scan(d), _want(v), v["name"])


@pytest.mark.gpu
def test_gpu_map_keys_match_golden(gpu_ctx):
    for v in VECTORS:
        if not v["name"].startswith("synth"):
            continue
        p, d = _unpack(v)
        dgrep.set_pattern(p.decode())
        kva = dgrep.Map(v["filename"], d)
        assert [kv.Key.encode() for kv in kva] == [base64.b64decode(k) for k in v["keys_b64"]], v["name"]
        assert [kv.Value for kv in kva] == [d[s:s + n] for s, n in zip(v["start"], v["len"])]
