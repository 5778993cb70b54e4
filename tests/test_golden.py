"""The committed golden vectors (tests/golden/vectors.json, made by
tests/golden/make_golden.py) against the oracle, the product's pattern
compiler and — on the GPU box — the HIP scan through the C ABI.

Each vector holds an input split, a pattern and the Map output of
application/grep.go:13-36 (1-based line numbers, byte starts and lengths of
the matching lines), the keys grep.go:25 builds, the key-sorted Reduce output
lines (map_reduce/worker.go:111-124,163-165) and the ihash partitions
(worker.go:13-17). Vectors whose "witnesses" list is non-empty were checked,
when generated, against Python `re` and/or GNU grep; the rest are parity
unpinned.
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
    return (np.array(v["line_no"], np.uint64), np.array(v["start"], np.uint64), np.array(v["len"], np.uint32))


def _eq(got, want, name):
    for g, w in zip(got, want):
        np.testing.assert_array_equal(np.asarray(g).astype(np.uint64), w.astype(np.uint64), err_msg=name)


def test_golden_shape():
    assert len(VECTORS) > 400
    pinned = [v for v in VECTORS if v["witnesses"]]
    assert len(pinned) > 300
    assert any(v["go_syntax_error"] for v in VECTORS)
    assert any(v["name"].startswith("synth-c3") and v["line_no"] for v in VECTORS)


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
        red = b"".join(sorted(k + b" " + x + b"\n" for k, x in zip(keys, vals)))
        assert red == base64.b64decode(v["reduce_b64"]), v["name"]


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
