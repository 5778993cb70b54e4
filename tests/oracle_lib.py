"""ctypes binding of the ORACLE (oracle/liboracle.so) — test infrastructure only.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker; the product path (libdgrep.so) never loads it.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

ORC_OK, ORC_ESYNTAX, ORC_EUNSUPPORTED = 0, 1, 2

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.orc_compile.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                  ctypes.c_char_p, ctypes.c_size_t]
        L.orc_compile.restype = ctypes.c_int
        L.orc_match.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.orc_match.restype = ctypes.c_int
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_free.restype = None
        for fn in (L.orc_map,):
            fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
            fn.restype = ctypes.c_int64
        L.orc_map_mt.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_map_mt.restype = ctypes.c_int64
        L.orc_ihash.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.orc_ihash.restype = ctypes.c_uint32
        L.orc_format_key.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_char_p,
                                     ctypes.c_size_t]
        L.orc_format_key.restype = ctypes.c_size_t
        L.orc_json_kv.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                  ctypes.c_char_p, ctypes.c_size_t]
        L.orc_json_kv.restype = ctypes.c_size_t
        _lib = L
    return _lib


class Regexp:
    """Go regexp.Compile(pattern) restated; .match(line) = regexp.Match."""

    def __init__(self, pattern: bytes):
        if isinstance(pattern, str):
            pattern = pattern.encode()
        self.pattern = pattern
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(256)
        self.status = lib().orc_compile(pattern, len(pattern), ctypes.byref(h), err, 256)
        self.error = err.value.decode(errors="replace")
        self._h = h

    def match(self, line: bytes) -> bool:
        if isinstance(line, str):
            line = line.encode()
        return bool(lib().orc_match(self._h, line, len(line)))

    def __del__(self):
        try:
            lib().orc_free(self._h)
        except Exception:
            pass


def compile_status(pattern: bytes) -> int:
    return Regexp(pattern).status


def grep_map(pattern: bytes, contents: bytes, recompile_per_line=False, threads=0):
    """grep.go Map restated: returns (line_no u64[], start u64[], len u64[])."""
    if isinstance(pattern, str):
        pattern = pattern.encode()
    buf = np.frombuffer(contents, dtype=np.uint8) if len(contents) else np.zeros(1, np.uint8)
    ptr = buf.ctypes.data
    L = lib()
    # at most one record per line: one pass fills the arrays
    cap = int(np.count_nonzero(buf[:len(contents)] == 10)) + 1
    for _ in range(2):
        ln = np.zeros(max(cap, 1), np.uint64)
        st = np.zeros(max(cap, 1), np.uint64)
        lens = np.zeros(max(cap, 1), np.uint64)
        if threads and threads > 1:
            cnt = L.orc_map_mt(pattern, len(pattern), ptr, len(contents), threads, ln.ctypes.data,
                               st.ctypes.data, lens.ctypes.data, cap)
        else:
            cnt = L.orc_map(pattern, len(pattern), ptr, len(contents), int(recompile_per_line), ln.ctypes.data,
                            st.ctypes.data, lens.ctypes.data, cap)
        if cnt < 0:
            raise NotImplementedError("pattern unsupported by the oracle: %r" % pattern)
        if cnt <= cap:
            return ln[:cnt], st[:cnt], lens[:cnt]
        cap = cnt
    raise AssertionError("unreachable")


def ihash(key: bytes) -> int:
    return lib().orc_ihash(key, len(key))


def format_key(filename: bytes, line: int) -> bytes:
    n = lib().orc_format_key(filename, len(filename), line, None, 0)
    out = ctypes.create_string_buffer(n)
    lib().orc_format_key(filename, len(filename), line, out, n)
    return out.raw[:n]


def json_kv(key: bytes, value: bytes) -> bytes:
    n = lib().orc_json_kv(key, len(key), value, len(value), None, 0)
    out = ctypes.create_string_buffer(n)
    lib().orc_json_kv(key, len(key), value, len(value), out, n)
    return out.raw[:n]


def _go_json_str(s: str) -> bytes:
    # Go's json.Decoder turns a lone surrogate escape into U+FFFD; Python keeps it
    return "".join("�" if 0xD800 <= ord(ch) < 0xE000 else ch for ch in s).encode("utf-8")


def json_roundtrip_kv(key: bytes, value: bytes):
    """(Key, Value) as the reduce task sees them: json.Encoder (the oracle's
    restatement of map_reduce/worker.go:92-93, invalid UTF-8 byte -> \\ufffd)
    then json.Decoder (worker.go:53-56). Python's json parses the encoder's
    output (standard escapes only); the decode side maps lone surrogates to
    U+FFFD as Go does."""
    import json

    line = json_kv(key, value)
    assert line.endswith(b"\n"), line
    d = json.loads(line)
    return _go_json_str(d["Key"]), _go_json_str(d["Value"])


def reduce_lines(keys, values) -> bytes:
    """The grep reduce output (Reduce = values[0], grep.go:38-40) of one map
    task's KeyValues, written "%v %v\\n" per key (map_reduce/worker.go:163-165),
    key-sorted because the reference writes them in Go map order
    (worker.go:163). Keys of one file are distinct."""
    lines = []
    for k, v in zip(keys, values):
        k2, v2 = json_roundtrip_kv(k, v)
        lines.append(k2 + b" " + v2 + b"\n")
    return b"".join(sorted(lines))
