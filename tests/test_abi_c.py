"""The boundary from C: tests/abi_c/plugin_sequence.c, built with gcc against
include/dgrep.h and linked to libdgrep.so, runs the cgo plugin's call sequence
(main/worker_launch.go:21-34 loads the plugin, whose Map calls
dgrep_compile -> dgrep_open -> dgrep_load_dfa -> dgrep_scan ->
dgrep_result_free -> dgrep_close), the error paths (dgrep_last_error after a
malformed blob, DGREP_E_NO_DFA) and a scan from a second pthread. On the GPU
box its records must equal the oracle's; here (no GPU) it must fail loudly at
dgrep_open -- there is no CPU fallback."""
import os
import subprocess

import numpy as np
import pytest

import dgrep
import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIR = os.path.join(ROOT, "tests", "abi_c")
EXE = os.path.join(DIR, "plugin_sequence")


def _build():
    subprocess.run(["make", "-s", "-C", DIR], check=True, capture_output=True)
    assert os.access(EXE, os.X_OK)


def _run(tmp_path, pattern: bytes, data: bytes, env=None):
    (tmp_path / "p").write_bytes(pattern)
    (tmp_path / "d").write_bytes(data)
    out = tmp_path / "o"
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run([EXE, str(tmp_path / "p"), str(tmp_path / "d"), str(out)], capture_output=True, text=True,
                       timeout=120, env=e)
    return p, out


def _parse(path):
    blocks, cur = [], None
    for line in open(path):
        if line.startswith("#"):
            cur = []
            blocks.append((int(line[1:]), cur))
        else:
            cur.append(tuple(int(x) for x in line.split()))
    return blocks


def test_c_caller_builds_and_fails_loudly_without_gpu(tmp_path):
    import torch

    _build()
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    p, _ = _run(tmp_path, b"error", b"an error\n")
    assert p.returncode != 0
    assert "dgrep_pick_device rc=4" in p.stderr, p.stderr  # DGREP_E_HIP: no device at all


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", [b"error", b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"", b"a**"])
def test_c_caller_plugin_sequence(tmp_path, pattern):
    _build()
    data = dgrep.synth_corpus_host(3 << 20, 31, 0) + b"\nan error at the end"
    p, out = _run(tmp_path, pattern, data, {"DGREP_DEVICE": "0"})
    assert p.returncode == 0, p.stderr
    assert "plugin sequence OK" in p.stdout
    ln, st, le = O.grep_map(pattern, data, threads=16)
    want = list(zip(ln.tolist(), st.tolist(), le.tolist()))
    blocks = _parse(out)
    assert len(blocks) == 3
    for count, recs in blocks:  # main thread, the second pthread, a second context
        assert count == len(want)
        assert recs == want


@pytest.mark.gpu
@pytest.mark.parametrize("env,code", [({"DGREP_DEVICE": "99"}, 4), ({"DGREP_DEVICE": "x"}, 1),
                                      ({"DGREP_WORKER_ID": "7"}, 0)])
def test_c_caller_device_selection(tmp_path, env, code):
    """The worker's device (dgrep_pick_device): DGREP_DEVICE=99 is a device
    that is not present (DGREP_E_HIP = 4), a non-number is DGREP_E_INVALID; a
    worker id maps to worker_id % device_count."""
    _build()
    env = dict(env)
    env.setdefault("DGREP_DEVICE", None)
    e = {k: v for k, v in env.items() if v is not None}
    base = {k: v for k, v in os.environ.items() if k not in ("DGREP_DEVICE", "DGREP_WORKER_ID")}
    base.update(e)
    (tmp_path / "p").write_bytes(b"error")
    (tmp_path / "d").write_bytes(b"an error\nno\n")
    p = subprocess.run([EXE, str(tmp_path / "p"), str(tmp_path / "d"), str(tmp_path / "o")], capture_output=True,
                       text=True, timeout=120, env=base)
    if code == 0:
        assert p.returncode == 0, p.stderr
    else:
        assert p.returncode != 0 and ("dgrep_pick_device rc=%d" % code) in p.stderr, p.stderr
