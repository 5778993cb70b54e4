"""C ABI checks that need no GPU: libdgrep.so loads, exports every function
include/*.h declares, validates blobs, and fails loudly (no CPU fallback) when
no GPU is present."""
import ctypes
import os
import re

import pytest

import dgrep

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("dgrep.h",):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(?:int|void|const char\*)\s+(dgrep_\w+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_exports_every_declared_symbol():
    L = dgrep.lib()
    declared = _declared()
    assert len(declared) >= 15
    missing = [n for n in declared if not hasattr(L, n)]
    assert not missing, missing
    assert set(dgrep.EXPORTS) <= declared


def test_compile_errors_and_unsupported():
    with pytest.raises(dgrep.UnsupportedPattern):
        dgrep.CompiledPattern("(" * 1001 + "a" + ")" * 1001)  # nesting beyond 1000: refused, never guessed
    assert dgrep.CompiledPattern("\\p{Greek}").nstates > 1
    cp = dgrep.CompiledPattern("(")
    assert cp.go_syntax_error
    assert "syntax" in cp.message


def test_blob_validation():
    L = dgrep.lib()
    cp = dgrep.CompiledPattern("error")
    info = dgrep._BlobInfo()
    assert L.dgrep_blob_info_get(cp.blob, len(cp.blob), ctypes.byref(info)) == dgrep.DGREP_OK
    assert (info.nstates, info.start, info.start_m) == (cp.nstates, 0, 1)
    bad = bytearray(cp.blob)
    bad[0] ^= 0xFF
    assert L.dgrep_blob_info_get(bytes(bad), len(bad), ctypes.byref(info)) == dgrep.DGREP_E_INVALID
    assert L.dgrep_blob_info_get(cp.blob, len(cp.blob) - 4, ctypes.byref(info)) == dgrep.DGREP_E_INVALID


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(dgrep.DgrepError):
        dgrep.Context(0)
    dgrep.set_pattern("error")
    with pytest.raises(dgrep.DgrepError):
        dgrep.Map("f", "an error\n")


def test_synth_host_deterministic_and_shaped():
    a = dgrep.synth_corpus_host(1 << 16, 5, 0)
    b = dgrep.synth_corpus_host(1 << 16, 5, 0)
    assert a == b and len(a) == 1 << 16
    assert a.endswith(b"\n")
    lines = a.split(b"\n")[:-1]
    assert all(40 <= len(x) + 1 <= 200 for x in lines)
    assert all(32 <= c < 127 for x in lines for c in x)
    assert dgrep.synth_corpus_host(1 << 16, 6, 0) != a
    kws = dgrep.synth_keywords(4, 1000)
    assert len(set(kws)) > 990 and all(5 <= len(k) <= 12 and k.isalpha() and k.islower() for k in kws)


def test_build_info_names_commit_and_arch():
    """dgrep_build_info() stamps the commit the library was built from (the
    bench reports it as config.build) and the tuning knobs compiled in."""
    info = dgrep.build_info()
    head = info.split()[0]
    assert re.fullmatch(r"head=([0-9a-f]{40}(-dirty)?|unknown)", head), info
    assert "arch=gfx950" in info and "hipflags=" in info


def test_synth_long_line_kinds():
    """kinds 2/3 of the corpus generator (bench workloads `long`, `long1g`):
    printable ASCII and '\\n' only; kind 2's lines average megabytes (a page
    of short log lines now and then); kind 3's first 1 GiB holds no '\\n'
    (checked on its first 64 MiB here)."""
    import numpy as np

    d = np.frombuffer(dgrep.synth_corpus_host(64 << 20, 3, 2), np.uint8)
    assert bool(((d == 10) | ((d >= 0x20) & (d < 0x7f))).all())
    nl = np.flatnonzero(d == 10)
    gaps = np.diff(nl)
    assert gaps.max() > (2 << 20)            # long lines
    assert (gaps < 300).sum() > 100          # and pages of log lines
    d3 = np.frombuffer(dgrep.synth_corpus_host(64 << 20, 3, 3), np.uint8)
    assert not (d3 == 10).any()


def test_synth_kind4_plants_keywords_in_long_lines():
    """kind 4 (bench workload long_c4): kind 2's long lines with config 4's
    keywords planted (random case) in filler pages, and kind-1 boundary lines;
    kind 2 itself is unchanged by it (same bytes as before the kind existed is
    not checkable here, but kind 2 and 4 share every '\\n')."""
    import numpy as np

    n = 64 << 20
    d4 = dgrep.synth_corpus_host(n, 4, 4)
    d2 = dgrep.synth_corpus_host(n, 4, 2)
    a4, a2 = np.frombuffer(d4, np.uint8), np.frombuffer(d2, np.uint8)
    np.testing.assert_array_equal(np.flatnonzero(a4 == 10), np.flatnonzero(a2 == 10))
    kws = dgrep.synth_keywords(4, 1000)
    low = d4.lower()
    found = sum(1 for k in kws if k in low)
    assert found >= 3, found
    assert bool(((a4 == 10) | ((a4 >= 0x20) & (a4 < 0x7f))).all())


def _cpu_ctx():
    """A context from dgrep_open on a machine without a GPU: the call fails
    (DGREP_E_HIP) but hands back the context so the caller can read the message;
    the setters below touch only host state."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: the GPU suite covers the setters through real scans")
    L = dgrep.lib()
    h = ctypes.c_void_p()
    assert L.dgrep_open(0, ctypes.byref(h)) == dgrep.DGREP_E_HIP
    assert h.value
    return L, h


def test_set_lane_chunk_accepts_exactly_the_documented_range():
    """include/dgrep.h: 0 (adaptive) or a multiple of 128 in [4096, 65536];
    anything else is DGREP_E_INVALID."""
    L, h = _cpu_ctx()
    try:
        ok = [0, 4096, 4224, 8192, 12416, 32768, 32896, 65408, 65536]
        bad = [1, 127, 128, 4000, 4095, 4097, 4160, 8193, 65537, 65664, 131072, 1 << 20, 0xFFFFFFFF]
        for v in ok:
            assert L.dgrep_set_lane_chunk(h, v) == dgrep.DGREP_OK, v
        for v in bad:
            assert L.dgrep_set_lane_chunk(h, v) == dgrep.DGREP_E_INVALID, v
        # every multiple of 128 in range, and every non-multiple near the ends
        for v in range(4096, 65536 + 1, 128):
            assert L.dgrep_set_lane_chunk(h, v) == dgrep.DGREP_OK, v
        for v in list(range(3968, 4096)) + list(range(65537, 65700)):
            assert L.dgrep_set_lane_chunk(h, v) == dgrep.DGREP_E_INVALID, v
    finally:
        L.dgrep_close(h)


def test_set_stepper_rejects_removed_steppers():
    """dgrep_set_stepper: 0 auto, 2 table, 3 pair, 4 filter; 1 (wide) and 5
    (word) were removed in round 6 and are DGREP_E_INVALID, as is anything else."""
    L, h = _cpu_ctx()
    try:
        for f in (0, 2, 3, 4):
            assert L.dgrep_set_stepper(h, f, 0) == dgrep.DGREP_OK, f
        for f in (-1, 1, 5, 6, 100):
            assert L.dgrep_set_stepper(h, f, 0) == dgrep.DGREP_E_INVALID, f
    finally:
        L.dgrep_close(h)


def test_scan_stats_sized_getter():
    """dgrep_last_scan_stats(ctx, out, out_size) never writes past out_size (a
    binding built against a shorter layout) and zeroes a longer caller's tail."""
    L, h = _cpu_ctx()
    try:
        full = ctypes.sizeof(dgrep._ScanStats)
        assert full == 80
        buf = (ctypes.c_uint8 * (full + 32))(*([0xAB] * (full + 32)))
        assert L.dgrep_last_scan_stats(h, ctypes.cast(buf, ctypes.POINTER(dgrep._ScanStats)), 8) == dgrep.DGREP_OK
        assert list(buf[8:]) == [0xAB] * (full + 24)   # nothing past the 8 bytes asked for
        assert L.dgrep_last_scan_stats(h, ctypes.cast(buf, ctypes.POINTER(dgrep._ScanStats)), full + 16) == dgrep.DGREP_OK
        assert list(buf[full:full + 16]) == [0] * 16    # a longer caller struct: zeroed tail
        assert list(buf[full + 16:]) == [0xAB] * 16
        assert L.dgrep_last_scan_stats(h, ctypes.cast(buf, ctypes.POINTER(dgrep._ScanStats)), 0) == dgrep.DGREP_E_INVALID
    finally:
        L.dgrep_close(h)
