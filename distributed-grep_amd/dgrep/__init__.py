"""dgrep — host-side mirror of distributed-grep's grep plugin over libdgrep.so.

The reference plugin (application/grep.go) exports

    func Map(filename string, contents string) []mapreduce.KeyValue   // grep.go:13-36
    func Reduce(key string, values []string) string                   // grep.go:38-40

with the pattern held in the package variable `pattern` (grep.go:11, default
""). This module keeps those names, argument meanings and error behaviour:

* ``Map(filename, contents)`` returns ``[KeyValue(Key, Value), ...]`` in line
  order, Key = ``"%s (line number #%d)" % (filename, n)`` (grep.go:25), Value =
  the line without its '\\n'. A pattern that Go's regexp.Compile rejects gives
  an empty list (grep.go:21 discards the error). Any device failure raises
  (the Go plugin would panic, and the coordinator re-assigns the task after
  its 10 s timeout, map_reduce/coordinator.go:105).
* ``Reduce(key, values)`` returns ``values[0]``.
* ``pattern`` defaults to "" (every line matches) and can be overridden with
  the DGREP_PATTERN environment variable or :func:`set_pattern`.

The matching itself runs on the GPU through the C ABI in include/dgrep.h; there
is no CPU fallback: if libdgrep.so or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import threading
from collections import namedtuple
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DGREP_LIB") or os.path.join(os.path.dirname(_HERE), "libdgrep.so")

DGREP_OK = 0
DGREP_E_INVALID = 1
DGREP_E_UNSUPPORTED = 2
DGREP_E_TOO_LARGE = 3
DGREP_E_HIP = 4
DGREP_E_NOMEM = 5
DGREP_E_NO_DFA = 6

DFA_GO_SYNTAX_ERROR = 1
DFA_MATCH_NONE = 2
DFA_MATCH_ALL = 4
DFA_PARTIAL = 8

# Symbols declared in include/dgrep.h (tests check the library exports all).
EXPORTS = (
    "dgrep_compile", "dgrep_compile_budget", "dgrep_blob_free", "dgrep_blob_info_get", "dgrep_open", "dgrep_close",
    "dgrep_last_error", "dgrep_pick_device", "dgrep_set_stream", "dgrep_load_dfa", "dgrep_scan", "dgrep_result_free",
    "dgrep_scan_device", "dgrep_synth_corpus", "dgrep_synth_corpus_host", "dgrep_synth_keyword",
    "dgrep_last_kernel_ms", "dgrep_take_kernel_ms", "dgrep_set_stepper", "dgrep_set_lane_chunk", "dgrep_set_ingest", "dgrep_last_ingest_ms",
    "dgrep_map_partitions", "dgrep_partitions_free", "dgrep_encode_device", "dgrep_last_encode_ms",
    "dgrep_reduce", "dgrep_reduce_free", "dgrep_last_scan_stats", "dgrep_build_info",
    "dgrep_comm_unique_id", "dgrep_comm_open", "dgrep_comm_close", "dgrep_gather_records_device",
    "dgrep_gather_records", "dgrep_gathered_free", "dgrep_comm_last_error",
)
COMM_ID_BYTES = 128

STEPPERS = {0: "table", 1: "sheng", 3: "pair", 4: "filter"}

KeyValue = namedtuple("KeyValue", ["Key", "Value"])  # map_reduce/helper_types.go:8-11


class DgrepError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("dgrep error %d: %s" % (code, msg))
        self.code = code


class UnsupportedPattern(DgrepError):
    pass


class _Result(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("line_no", ctypes.POINTER(ctypes.c_uint64)),
                ("start", ctypes.POINTER(ctypes.c_uint64)), ("len", ctypes.POINTER(ctypes.c_uint64))]


class _Partitions(ctypes.Structure):
    _fields_ = [("nreduce", ctypes.c_uint32), ("total", ctypes.c_uint64), ("begin", ctypes.POINTER(ctypes.c_uint64)),
                ("end", ctypes.POINTER(ctypes.c_uint64)), ("bytes", ctypes.c_void_p)]


class _ReduceOut(ctypes.Structure):
    _fields_ = [("lines_in", ctypes.c_uint64), ("total", ctypes.c_uint64), ("bytes", ctypes.c_void_p)]


class _ScanStats(ctypes.Structure):
    _fields_ = [("stepper", ctypes.c_uint32), ("lane_chunk", ctypes.c_uint32), ("lane_slots", ctypes.c_uint32),
                ("scan_attempts", ctypes.c_uint32), ("tiles", ctypes.c_uint64), ("overflow_lanes", ctypes.c_uint64),
                ("matches", ctypes.c_uint64), ("scan_ms", ctypes.c_float), ("overflow_ms", ctypes.c_float),
                ("verify_ms", ctypes.c_float), ("candidates", ctypes.c_uint64), ("pending", ctypes.c_uint64),
                ("reserved0", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class _Gathered(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("line_no", ctypes.POINTER(ctypes.c_uint64)),
                ("start", ctypes.POINTER(ctypes.c_uint64)), ("len", ctypes.POINTER(ctypes.c_uint64)),
                ("split", ctypes.POINTER(ctypes.c_uint32))]


class _BlobInfo(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32), ("nstates", ctypes.c_uint32), ("nclasses", ctypes.c_uint32),
                ("start", ctypes.c_uint32), ("start_m", ctypes.c_uint32)]


_lib = None
_lib_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    """Load libdgrep.so (fails loudly if it was not built)."""
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError("libdgrep.so not built (run __graft_entry__.build() or `make`): " + LIB_PATH)
            L = ctypes.CDLL(LIB_PATH)
            vp, sz, u64, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int
            L.dgrep_compile.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.c_char_p, sz]
            L.dgrep_compile.restype = i
            L.dgrep_compile_budget.argtypes = [ctypes.c_char_p, sz, ctypes.c_uint32, ctypes.POINTER(vp),
                                               ctypes.POINTER(sz), ctypes.c_char_p, sz]
            L.dgrep_compile_budget.restype = i
            L.dgrep_blob_free.argtypes = [vp]
            L.dgrep_blob_free.restype = None
            L.dgrep_blob_info_get.argtypes = [vp, sz, ctypes.POINTER(_BlobInfo)]
            L.dgrep_blob_info_get.restype = i
            L.dgrep_pick_device.argtypes = [i, ctypes.POINTER(i)]
            L.dgrep_pick_device.restype = i
            L.dgrep_open.argtypes = [i, ctypes.POINTER(vp)]
            L.dgrep_open.restype = i
            L.dgrep_close.argtypes = [vp]
            L.dgrep_close.restype = None
            L.dgrep_last_error.argtypes = [vp]
            L.dgrep_last_error.restype = ctypes.c_char_p
            L.dgrep_set_stream.argtypes = [vp, vp]
            L.dgrep_set_stream.restype = i
            L.dgrep_load_dfa.argtypes = [vp, vp, sz]
            L.dgrep_load_dfa.restype = i
            L.dgrep_set_stepper.argtypes = [vp, i, ctypes.c_uint32]
            L.dgrep_set_stepper.restype = i
            L.dgrep_set_lane_chunk.argtypes = [vp, ctypes.c_uint32]
            L.dgrep_set_lane_chunk.restype = i
            L.dgrep_scan.argtypes = [vp, vp, sz, ctypes.POINTER(_Result)]
            L.dgrep_scan.restype = i
            L.dgrep_result_free.argtypes = [ctypes.POINTER(_Result)]
            L.dgrep_result_free.restype = None
            L.dgrep_scan_device.argtypes = [vp, vp, sz, vp, vp, vp, u64, ctypes.POINTER(u64)]
            L.dgrep_scan_device.restype = i
            L.dgrep_synth_corpus.argtypes = [vp, vp, sz, u64, i]
            L.dgrep_synth_corpus.restype = i
            L.dgrep_synth_corpus_host.argtypes = [vp, sz, u64, i]
            L.dgrep_synth_corpus_host.restype = i
            L.dgrep_synth_keyword.argtypes = [u64, i, ctypes.c_char_p]
            L.dgrep_synth_keyword.restype = i
            L.dgrep_last_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
            L.dgrep_last_kernel_ms.restype = i
            L.dgrep_take_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
            L.dgrep_take_kernel_ms.restype = i
            L.dgrep_set_ingest.argtypes = [vp, sz, i, i]
            L.dgrep_set_ingest.restype = i
            L.dgrep_last_ingest_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
            L.dgrep_last_ingest_ms.restype = i
            L.dgrep_map_partitions.argtypes = [vp, vp, sz, ctypes.c_char_p, sz, ctypes.c_uint32,
                                               ctypes.POINTER(_Partitions)]
            L.dgrep_map_partitions.restype = i
            L.dgrep_partitions_free.argtypes = [ctypes.POINTER(_Partitions)]
            L.dgrep_partitions_free.restype = None
            L.dgrep_encode_device.argtypes = [vp, vp, sz, vp, vp, vp, u64, ctypes.c_char_p, sz, ctypes.c_uint32, vp,
                                              u64, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]
            L.dgrep_encode_device.restype = i
            L.dgrep_last_encode_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
            L.dgrep_last_encode_ms.restype = i
            L.dgrep_reduce.argtypes = [vp, vp, sz, ctypes.POINTER(_ReduceOut)]
            L.dgrep_reduce.restype = i
            L.dgrep_reduce_free.argtypes = [ctypes.POINTER(_ReduceOut)]
            L.dgrep_reduce_free.restype = None
            L.dgrep_last_scan_stats.argtypes = [vp, ctypes.POINTER(_ScanStats), sz]
            L.dgrep_last_scan_stats.restype = i
            L.dgrep_build_info.argtypes = []
            L.dgrep_build_info.restype = ctypes.c_char_p
            L.dgrep_comm_unique_id.argtypes = [vp]
            L.dgrep_comm_unique_id.restype = i
            L.dgrep_comm_open.argtypes = [vp, vp, i, i, ctypes.POINTER(vp)]
            L.dgrep_comm_open.restype = i
            L.dgrep_comm_close.argtypes = [vp]
            L.dgrep_comm_close.restype = None
            L.dgrep_gather_records_device.argtypes = [vp, vp, vp, vp, u64, ctypes.c_uint32, i, ctypes.POINTER(vp),
                                                      ctypes.POINTER(u64), vp]
            L.dgrep_gather_records_device.restype = i
            L.dgrep_gather_records.argtypes = [vp, vp, vp, vp, u64, ctypes.c_uint32, i, ctypes.POINTER(_Gathered)]
            L.dgrep_gather_records.restype = i
            L.dgrep_gathered_free.argtypes = [ctypes.POINTER(_Gathered)]
            L.dgrep_gathered_free.restype = None
            L.dgrep_comm_last_error.argtypes = [vp]
            L.dgrep_comm_last_error.restype = ctypes.c_char_p
            _lib = L
    return _lib


class CompiledPattern:
    """A pattern compiled by dgrep_compile (Go regexp/syntax semantics)."""

    def __init__(self, pattern, state_budget: int = 0):
        """state_budget (tests only): a lowered DFA state budget, so that small
        patterns compile to partial blobs (dgrep_compile_budget)."""
        if isinstance(pattern, str):
            pattern = pattern.encode("utf-8", "surrogateescape")
        self.pattern = bytes(pattern)
        L = lib()
        blob = ctypes.c_void_p()
        n = ctypes.c_size_t()
        err = ctypes.create_string_buffer(512)
        rc = L.dgrep_compile_budget(self.pattern, len(self.pattern), state_budget, ctypes.byref(blob),
                                    ctypes.byref(n), err, 512)
        msg = err.value.decode(errors="replace")
        if rc == DGREP_E_UNSUPPORTED:
            raise UnsupportedPattern(rc, msg)
        if rc != DGREP_OK:
            raise DgrepError(rc, msg)
        self.blob = ctypes.string_at(blob, n.value)
        L.dgrep_blob_free(blob)
        info = _BlobInfo()
        rc = L.dgrep_blob_info_get(self.blob, len(self.blob), ctypes.byref(info))
        if rc != DGREP_OK:
            raise DgrepError(rc, "malformed blob")
        self.flags = info.flags
        self.nstates = info.nstates
        self.nclasses = info.nclasses
        self.start = info.start
        self.start_m = info.start_m
        self.message = msg

    @property
    def partial(self) -> bool:
        """DFA over the state budget: first states + CAND, lines that reach CAND
        are decided by the blob's NFA program (dgrep_blob.h)."""
        return bool(self.flags & DFA_PARTIAL)

    def nfa_program(self) -> np.ndarray:
        """The NFA program (u32 words) of a partial blob -- for tests."""
        ne = self.nstates * self.nclasses
        return np.frombuffer(self.blob[288 + 4 * ne:], dtype=np.uint32)

    @property
    def go_syntax_error(self) -> bool:
        return bool(self.flags & DFA_GO_SYNTAX_ERROR)

    def tables(self) -> Tuple[np.ndarray, np.ndarray]:
        """(byte_class[256] u8, trans[nstates, nclasses] u32) — for tests/inspection."""
        bc = np.frombuffer(self.blob[32:288], dtype=np.uint8)
        ne = self.nstates * self.nclasses
        tr = np.frombuffer(self.blob[288:288 + 4 * ne], dtype=np.uint32).reshape(self.nstates, self.nclasses)
        return bc, tr


class Context:
    """One device context (a HIP device + stream) — dgrep_open/close."""

    def __init__(self, device: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        rc = self._L.dgrep_open(device, ctypes.byref(h))
        self._h = h
        if rc != DGREP_OK:
            msg = self._err()
            self.close()
            raise DgrepError(rc, msg)
        self.device = device
        self.pattern: Optional[CompiledPattern] = None

    def _err(self) -> str:
        m = self._L.dgrep_last_error(self._h)
        return m.decode(errors="replace") if m else ""

    def _check(self, rc: int):
        if rc != DGREP_OK:
            if rc == DGREP_E_UNSUPPORTED:
                raise UnsupportedPattern(rc, self._err())
            raise DgrepError(rc, self._err())

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.dgrep_close(self._h)
        self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream: int):
        self._check(self._L.dgrep_set_stream(self._h, ctypes.c_void_p(hip_stream or None)))

    def set_lane_chunk(self, chunk_bytes: int = 0):
        """Testing/tuning: the Sheng / pair / filter lane chunk for later scans
        (dgrep_set_lane_chunk; 0 = adaptive, else a multiple of 128 in [4096, 65536])."""
        self._check(self._L.dgrep_set_lane_chunk(self._h, chunk_bytes))

    _FORCE = {"auto": 0, "table": 2, "pair": 3, "filter": 4}

    def set_stepper(self, force="auto", filter_rows: int = 0):
        """Testing/tuning: the stepper the next load() uses (dgrep_set_stepper):
        "auto" (default: by DFA size), "table" (u8, <= 256 states), "pair" (fails
        at load if its two-byte table does not fit) or "filter"; filter_rows caps
        the filter's LDS rows (nearly every line then becomes a candidate)."""
        self._check(self._L.dgrep_set_stepper(self._h, self._FORCE[force], filter_rows))

    def load(self, pattern) -> CompiledPattern:
        cp = pattern if isinstance(pattern, CompiledPattern) else CompiledPattern(pattern)
        self._check(self._L.dgrep_load_dfa(self._h, cp.blob, len(cp.blob)))
        self.pattern = cp
        return cp

    def scan(self, contents) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Host split -> (line_no u64[], start u64[], len u64[]) of matching lines."""
        if isinstance(contents, str):
            contents = contents.encode("utf-8", "surrogateescape")
        buf = np.frombuffer(contents, dtype=np.uint8) if len(contents) else np.zeros(1, np.uint8)
        res = _Result()
        self._check(self._L.dgrep_scan(self._h, ctypes.c_void_p(buf.ctypes.data), len(contents), ctypes.byref(res)))
        try:
            n = int(res.count)
            if n == 0:
                return np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint64)
            ln = np.ctypeslib.as_array(res.line_no, shape=(n,)).copy()
            st = np.ctypeslib.as_array(res.start, shape=(n,)).copy()
            le = np.ctypeslib.as_array(res.len, shape=(n,)).copy()
            return ln, st, le
        finally:
            self._L.dgrep_result_free(ctypes.byref(res))

    def scan_device(self, d_data: int, n: int, d_line: int, d_start: int, d_len: int, capacity: int) -> int:
        """HBM-resident split at device pointer d_data; returns the match count."""
        cnt = ctypes.c_uint64()
        self._check(self._L.dgrep_scan_device(self._h, ctypes.c_void_p(d_data), n, ctypes.c_void_p(d_line),
                                              ctypes.c_void_p(d_start), ctypes.c_void_p(d_len), capacity,
                                              ctypes.byref(cnt)))
        return int(cnt.value)

    def synth(self, d_out: int, n: int, seed: int, kind: int = 0):
        self._check(self._L.dgrep_synth_corpus(self._h, ctypes.c_void_p(d_out), n, seed, kind))

    def set_ingest(self, chunk_bytes: int, nbufs: int = 0, threads: int = 0):
        """Ingest pipeline of scan(): pinned staging pieces of chunk_bytes (0 =
        one direct pageable copy), nbufs buffers, threads host-copy threads
        (dgrep_set_ingest; 0 keeps the current value)."""
        self._check(self._L.dgrep_set_ingest(self._h, chunk_bytes, nbufs, threads))

    def last_ingest_ms(self) -> float:
        ms = ctypes.c_float()
        self._check(self._L.dgrep_last_ingest_ms(self._h, ctypes.byref(ms)))
        return float(ms.value)

    def map_partitions(self, filename, contents, nreduce: int) -> List[bytes]:
        """Map + writeMapOutput of one split on the GPU (dgrep_map_partitions):
        element p is the byte content of mr-<task>-<p> (map_reduce/worker.go:78-109)."""
        if isinstance(contents, str):
            contents = contents.encode("utf-8", "surrogateescape")
        fname = filename.encode("utf-8", "surrogateescape") if isinstance(filename, str) else bytes(filename)
        buf = np.frombuffer(contents, dtype=np.uint8) if len(contents) else np.zeros(1, np.uint8)
        res = _Partitions()
        self._check(self._L.dgrep_map_partitions(self._h, ctypes.c_void_p(buf.ctypes.data), len(contents), fname,
                                                 len(fname), nreduce, ctypes.byref(res)))
        try:
            raw = ctypes.string_at(res.bytes, res.total) if res.total else b""
            return [raw[res.begin[p]:res.end[p]] for p in range(nreduce)]
        finally:
            self._L.dgrep_partitions_free(ctypes.byref(res))

    def encode_device(self, d_data: int, n: int, d_line: int, d_start: int, d_len: int, count: int, filename,
                      nreduce: int, d_out: int, out_cap: int):
        """dgrep_encode_device: returns (begin[], end[], total)."""
        fname = filename.encode("utf-8", "surrogateescape") if isinstance(filename, str) else bytes(filename)
        b = (ctypes.c_uint64 * nreduce)()
        e = (ctypes.c_uint64 * nreduce)()
        tot = ctypes.c_uint64()
        self._check(self._L.dgrep_encode_device(self._h, ctypes.c_void_p(d_data), n, ctypes.c_void_p(d_line),
                                                ctypes.c_void_p(d_start), ctypes.c_void_p(d_len), count, fname,
                                                len(fname), nreduce, ctypes.c_void_p(d_out), out_cap, b, e,
                                                ctypes.byref(tot)))
        return list(b), list(e), int(tot.value)

    def reduce(self, data: bytes) -> bytes:
        """One grep reduce task on the GPU (dgrep_reduce): data = the
        concatenated mr-<map>-<r> files; returns the content of mr-out-<r>."""
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        res = _ReduceOut()
        self._check(self._L.dgrep_reduce(self._h, ctypes.c_void_p(buf.ctypes.data), len(data), ctypes.byref(res)))
        try:
            return ctypes.string_at(res.bytes, res.total) if res.total else b""
        finally:
            self._L.dgrep_reduce_free(ctypes.byref(res))

    def last_encode_ms(self) -> float:
        ms = ctypes.c_float()
        self._check(self._L.dgrep_last_encode_ms(self._h, ctypes.byref(ms)))
        return float(ms.value)

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        self._check(self._L.dgrep_last_kernel_ms(self._h, ctypes.byref(ms)))
        return float(ms.value)

    def take_kernel_ms(self):
        """(sum of the scans' device ms, number of scans) since the previous take (dgrep_take_kernel_ms)."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        self._check(self._L.dgrep_take_kernel_ms(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return float(ms.value), int(n.value)

    def scan_stats(self) -> dict:
        """dgrep_last_scan_stats of the last scan (stepper, lane chunk, overflow lanes, times)."""
        st = _ScanStats()
        self._check(self._L.dgrep_last_scan_stats(self._h, ctypes.byref(st), ctypes.sizeof(st)))
        d = {f: getattr(st, f) for f, _ in _ScanStats._fields_}
        d["stepper"] = STEPPERS.get(d["stepper"], d["stepper"])
        return d


def build_info() -> str:
    """dgrep_build_info(): "head=<commit>[-dirty] arch=gfx950 hipflags=..."."""
    return lib().dgrep_build_info().decode()


def synth_corpus_host(n: int, seed: int, kind: int = 0) -> bytes:
    """CPU twin of dgrep_synth_corpus (same generator code, synth.h)."""
    out = ctypes.create_string_buffer(max(n, 1))
    rc = lib().dgrep_synth_corpus_host(out, n, seed, kind)
    if rc != DGREP_OK:
        raise DgrepError(rc, "synth")
    return out.raw[:n]


def synth_keywords(seed: int, count: int = 1000) -> List[bytes]:
    out = []
    buf = ctypes.create_string_buffer(16)
    for i in range(count):
        k = lib().dgrep_synth_keyword(seed, i, buf)
        out.append(buf.raw[:k])
    return out


# ---- the plugin surface (application/grep.go) --------------------------------

pattern: str = os.environ.get("DGREP_PATTERN", "")  # grep.go:11 `var pattern string = ""`

class Comm:
    """The C ABI's multi-GPU exchange (include/dgrep.h, dgrep_comm_*): an RCCL
    communicator on a Context's device and stream. Rank 0 (or any one rank)
    makes the id with :meth:`unique_id` and hands the 128 bytes to the others;
    every rank then constructs a Comm (collective)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        rc = lib().dgrep_comm_unique_id(buf)
        if rc != DGREP_OK:
            raise DgrepError(rc, "dgrep_comm_unique_id failed")
        return buf.raw

    def __init__(self, ctx: "Context", uid: bytes, nranks: int, rank: int):
        self._L = lib()
        self.ctx, self.nranks, self.rank = ctx, nranks, rank
        h = ctypes.c_void_p()
        rc = self._L.dgrep_comm_open(ctx._h, ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES), nranks, rank,
                                     ctypes.byref(h))
        self._h = h
        if rc != DGREP_OK:
            msg = self._err()
            self.close()
            raise DgrepError(rc, msg)

    def _err(self) -> str:
        m = self._L.dgrep_comm_last_error(self._h) if self._h else None
        return m.decode(errors="replace") if m else ""

    def gather_device(self, d_line: int, d_start: int, d_len: int, count: int, split: int = 0, root: int = 0):
        """dgrep_gather_records_device: (device pointer of the packed 28-B
        records, total, per-rank counts) on the root; (None, count, None) elsewhere."""
        ptr = ctypes.c_void_p()
        total = ctypes.c_uint64()
        counts = (ctypes.c_uint64 * self.nranks)()
        rc = self._L.dgrep_gather_records_device(self._h, d_line, d_start, d_len, count, split & 0xFFFFFFFF, root,
                                                 ctypes.byref(ptr), ctypes.byref(total), counts)
        if rc != DGREP_OK:
            raise DgrepError(rc, self._err())
        if self.rank != root:
            return None, total.value, None
        return ptr.value, total.value, list(counts)

    def gather(self, d_line: int, d_start: int, d_len: int, count: int, split: int = 0, root: int = 0):
        """dgrep_gather_records: (line_no, start, len, split) numpy arrays on the
        root (rank order), None elsewhere."""
        g = _Gathered()
        rc = self._L.dgrep_gather_records(self._h, d_line, d_start, d_len, count, split & 0xFFFFFFFF, root,
                                          ctypes.byref(g))
        if rc != DGREP_OK:
            raise DgrepError(rc, self._err())
        try:
            if self.rank != root:
                return None
            n = g.count
            arr = lambda p, t: np.ctypeslib.as_array(p, shape=(n,)).astype(t) if n else np.zeros(0, t)
            return (arr(g.line_no, np.uint64), arr(g.start, np.uint64), arr(g.len, np.uint64),
                    arr(g.split, np.uint32))
        finally:
            self._L.dgrep_gathered_free(ctypes.byref(g))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.dgrep_comm_close(self._h)
        self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_ctx_local = threading.local()


def set_pattern(p: str):
    global pattern
    pattern = p


def pick_device(worker_id: int = -1) -> int:
    """dgrep_pick_device: DGREP_DEVICE, else worker_id % device count (worker_id
    < 0: DGREP_WORKER_ID, else the process id). Raises if the device is absent."""
    d = ctypes.c_int()
    rc = lib().dgrep_pick_device(worker_id, ctypes.byref(d))
    if rc != DGREP_OK:
        raise DgrepError(rc, "no such device (DGREP_DEVICE=%r, worker %d)" % (os.environ.get("DGREP_DEVICE"), worker_id))
    return d.value


def _default_device() -> int:
    """The module-level Map's device: the worker rule (pick_device) only when
    DGREP_DEVICE or DGREP_WORKER_ID says which worker this is; otherwise device
    0, as before round 3 (never a device that depends on the process id, which
    could differ from the caller's torch device)."""
    if os.environ.get("DGREP_DEVICE") or os.environ.get("DGREP_WORKER_ID"):
        return pick_device()
    return 0


def _context() -> Context:
    ctx = getattr(_ctx_local, "ctx", None)
    if ctx is None:
        ctx = Context(_default_device())
        _ctx_local.ctx = ctx
        _ctx_local.loaded = None
    if _ctx_local.loaded != pattern:
        ctx.load(pattern)
        _ctx_local.loaded = pattern
    return ctx


def format_key(filename: str, line_no: int) -> str:
    """fmt.Sprintf("%s (line number #%v)", filename, line_number+1) (grep.go:25)."""
    return "%s (line number #%d)" % (filename, line_no)


def Map(filename: str, contents) -> List[KeyValue]:
    """grep.go:13-36 on the GPU: matching lines of `contents`, in line order."""
    raw = contents.encode("utf-8", "surrogateescape") if isinstance(contents, str) else bytes(contents)
    ln, st, le = _context().scan(raw)
    kva = []
    for n, s, l in zip(ln.tolist(), st.tolist(), le.tolist()):
        v = raw[s:s + l]
        kva.append(KeyValue(format_key(filename, n), v.decode("utf-8", "surrogateescape")
                            if isinstance(contents, str) else v))
    return kva


def Reduce(key: str, values: Sequence[str]) -> str:
    """grep.go:38-40."""
    return values[0]
