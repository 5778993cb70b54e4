"""Long lines on the GPU (application/grep.go:17 splits a file of any shape;
map_reduce/worker.go:72-76 reads whole files). A lane whose chunk holds no
'\\n' owns no line and stops at its chunk end; on the <= 256-state steppers a
line still open two chunks past its owner's chunk is parked and finished by the
long-line kernels (end from the per-chunk '\\n' counts, per-segment transition
maps composed in order) -- checked bit-exactly against the oracle for every
such stepper, with matches at a line's start, middle and far end, lines ending
exactly at chunk edges, newline-free and unterminated splits. A line over
4 GiB is reported with its 64-bit length, checked against the oracle."""
import random

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _check(ctx, pattern, data, threads=16):
    ctx.load(pattern)
    ln, st, le = ctx.scan(data)
    oln, ost, ole = O.grep_map(pattern, data, threads=threads)
    assert len(ln) == len(oln), (pattern, len(ln), len(oln))
    np.testing.assert_array_equal(ln, oln)
    np.testing.assert_array_equal(st, ost)
    np.testing.assert_array_equal(le.astype(np.uint64), ole.astype(np.uint64))
    return ctx.scan_stats()


def _long_split(seed, sizes, plant=b"error"):
    rnd = random.Random(seed)
    parts = []
    for L in sizes:
        body = bytearray(rnd.choice(b"abcdfghij ") for _ in range(L))
        where = rnd.random()
        if where < 0.25 and L > 10:
            body[:5] = plant
        elif where < 0.5 and L > 10:
            body[-5:] = plant
        elif where < 0.75 and L > 10:
            q = rnd.randrange(L - 5)
            body[q:q + 5] = plant
        parts.append(bytes(body))
    return b"\n".join(parts)


STEPPER_PATTERNS = [
    ("auto", b"error"),                                   # Sheng (<= 8 states)
    ("auto", b""),                                        # every line
    ("auto", b"^[a-j ]*error[a-j ]*$"),                   # pair stepper (the default above 8 states)
    ("pair", b"(WARN|ERROR) [a-z_]+"),                    # pair stepper, C3's event pattern
    ("table", b"error$"),                                 # u8 table, two chunks per lane
    ("auto", b"(?i)e[r]+or"),
]


@pytest.mark.parametrize("force,pattern", STEPPER_PATTERNS)
def test_long_lines_parked_and_resolved(gpu_ctx, force, pattern):
    sizes = [10, 300, 70000, 5, 1 << 20, 3 << 20, 40000, 9000, 100, (1 << 22) + 7, 2]
    data = _long_split(5, sizes)
    try:
        gpu_ctx.set_stepper(force)
        st = _check(gpu_ctx, pattern, data)
        assert st["pending"] > 0, st  # some lines were parked and resolved
        # unterminated last line that is long, and a newline-free split
        _check(gpu_ctx, pattern, data + b"\n" + b"x" * 200000 + b"error")
        _check(gpu_ctx, pattern, b"y" * (3 << 20) + b"error" + b"z" * 100000)
        _check(gpu_ctx, pattern, b"error" + b"y" * (3 << 20))
    finally:
        gpu_ctx.set_stepper("auto")


@pytest.mark.parametrize("chunk", [4096, 8192, 32768])
def test_long_lines_at_chunk_edges(gpu_ctx, chunk):
    """Lines ending exactly at chunk boundaries and at 2 C (the parking point)."""
    gpu_ctx.set_lane_chunk(chunk)
    try:
        for extra in (-1, 0, 1):
            sizes = [chunk - 1, 2 * chunk + extra, 3 * chunk - 1, 5 * chunk + extra, chunk * 64 + extra, 7]
            data = _long_split(11 + extra, sizes)
            _check(gpu_ctx, b"error", data)
            _check(gpu_ctx, b"", data)
    finally:
        gpu_ctx.set_lane_chunk(0)


def test_long_lines_workload_scale(gpu_ctx):
    """Hundreds of 64 KiB-8 MiB lines mixed with normal log lines."""
    import dgrep

    rnd = random.Random(21)
    parts = []
    for i in range(120):
        if rnd.random() < 0.5:
            parts.append(dgrep.synth_corpus_host(rnd.randrange(1, 200000), 100 + i, 0).rstrip(b"\n"))
        else:
            L = rnd.randrange(64 << 10, 8 << 20)
            b = bytearray(b"q" * L)
            if rnd.random() < 0.5:
                q = rnd.randrange(L - 5)
                b[q:q + 5] = b"error"
            parts.append(bytes(b))
    data = b"\n".join(parts)
    st = _check(gpu_ctx, b"error", data)
    assert st["pending"] > 10


def test_line_over_4gib(gpu_ctx):
    """One 4.5 GiB line (no '\\n') then a short one: the "" pattern (the
    reference's shipped grep.go:11) matches both; `error` planted 3 bytes
    before the long line's end matches only it. Checked against the expected
    records AND the oracle's Map over the same 4.5 GiB (64-bit lengths on
    both sides since round 4)."""
    import torch

    n_long = (9 << 29) + 3  # 4.5 GiB + 3
    tail = b"\nabc"
    n = n_long + len(tail)
    buf = torch.full((n + 64,), ord("x"), dtype=torch.uint8, device="cuda")
    buf[n_long - 8:n_long - 3] = torch.tensor(list(b"error"), dtype=torch.uint8, device="cuda")
    buf[n_long:n] = torch.tensor(list(tail), dtype=torch.uint8, device="cuda")
    host = buf[:n].cpu().numpy()
    cap = 16
    line_t = torch.zeros(cap, dtype=torch.int64, device="cuda")
    start_t = torch.zeros(cap, dtype=torch.int64, device="cuda")
    len_t = torch.zeros(cap, dtype=torch.int64, device="cuda")
    for pattern, want in ((b"", [(1, 0, n_long), (2, n_long + 1, 3)]), (b"error", [(1, 0, n_long)]),
                          (b"^x*$", [])):
        gpu_ctx.load(pattern)
        cnt = gpu_ctx.scan_device(buf.data_ptr(), n, line_t.data_ptr(), start_t.data_ptr(), len_t.data_ptr(), cap)
        got = list(zip(line_t[:cnt].tolist(), start_t[:cnt].tolist(), len_t[:cnt].tolist()))
        assert got == want, (pattern, got)
        assert gpu_ctx.scan_stats()["pending"] >= 1
        oln, ost, ole = O.grep_map(pattern, host, threads=16)
        assert list(zip(oln.tolist(), ost.tolist(), ole.tolist())) == want, pattern
    del buf, host
    torch.cuda.empty_cache()


def _dense_then_long(chunk, long_len, long_matches, dense=b"error", seed=3):
    """Normal lines, then dense matching lines up to 64 bytes before a lane
    chunk's end, then one line of long_len bytes (so the lane owning it also
    owns hundreds of matching lines: it overflows AND parks), then normal lines."""
    rnd = random.Random(seed)
    head = b"".join(b"abc def %d\n" % rnd.randrange(1000) for _ in range(50))
    target = ((len(head) // chunk) + 3) * chunk - 64  # the long line starts here
    body = bytearray(head)
    while len(body) + len(dense) + 1 <= target - 8:
        body += dense + b"\n"
    body += b"f" * (target - len(body) - 1) + b"\n"
    assert len(body) == target
    line = bytearray(b"q" * long_len)
    if long_matches:
        line[-5:] = b"error"
    return bytes(body) + bytes(line) + b"\n" + b"tail line error\nlast\n"


@pytest.mark.parametrize("force,pattern,chunk", [
    ("auto", b"error", 4096),                      # Sheng (chunk maps: parked at C + 4 KiB)
    ("auto", b"error", 32768),
    ("auto", b"^[a-j ]*error[a-j ]*$", 4096),      # pair (parked at 2 C)
    ("table", b"error$", 0),                       # u8 table, two 2 KiB chunks per lane
])
@pytest.mark.parametrize("long_matches", [False, True])
def test_overflowing_lane_with_parked_line(gpu_ctx, force, pattern, chunk, long_matches):
    """A lane that owns more matching lines than its slots + spill area AND
    parks its last (long) line: the overflow pass re-runs it and must stop at
    the same park point, staging the same pending record (a non-matching long
    line left an unfilled record before round 4)."""
    c = chunk or 2048
    data = _dense_then_long(c, 6 * max(c, 4096) + 123, long_matches)
    try:
        gpu_ctx.set_stepper(force)
        gpu_ctx.set_lane_chunk(chunk)
        st = _check(gpu_ctx, pattern, data)
        assert st["overflow_lanes"] > 0 and st["pending"] > 0, st
    finally:
        gpu_ctx.set_stepper("auto")
        gpu_ctx.set_lane_chunk(0)


@pytest.mark.parametrize("force,pattern", [("auto", b"error"), ("auto", b"^[a-j ]*error[a-j ]*$"),
                                           ("table", b"error$"), ("filter", b"error"),
                                           ("filter", b"(WARN|ERROR) [a-z_]+|x error 4")])
def test_count_exact_when_capacity_too_small_with_parked_lines(gpu_ctx, force, pattern):
    """dgrep_scan_device with a capacity below the match count (a size query:
    0, or 1) must still return the exact number of matching lines when some
    parked long lines do not match (dgrep.h: the count is exact)."""
    import torch

    sizes = [10, 300, 70000, 5, 1 << 20, 3 << 20, 40000, 9000, 100, (1 << 22) + 7, 2]
    data = _long_split(9, sizes)
    data = data + b"\n" + b"\n".join(b"x error %d" % i for i in range(500))
    oln, _, _ = O.grep_map(pattern, data, threads=16)
    n = len(data)
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    out = [torch.zeros(4, dtype=torch.int64, device="cuda") for _ in range(3)]
    try:
        # the filter with 4 LDS rows: nearly every line a candidate, so the
        # first scan outgrows its staging buffer and must re-scan before counting
        gpu_ctx.set_stepper(force, 4 if force == "filter" else 0)
        gpu_ctx.load(pattern)
        for cap in (0, 1, 4):
            cnt = gpu_ctx.scan_device(buf.data_ptr(), n, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), cap)
            assert cnt == len(oln), (cap, cnt, len(oln))
            assert gpu_ctx.scan_stats()["pending"] > 0
    finally:
        gpu_ctx.set_stepper("auto")


def _c4_pattern(seed=4, nkw=1000):
    import dgrep

    return b"(?i)(" + b"|".join(dgrep.synth_keywords(seed, nkw)) + b")"


def test_filter_long_lines_c4_keywords(gpu_ctx):
    """Config 4's 1,000-keyword pattern (the filter stepper: > 256 DFA states)
    over lines of 1-8 MiB, keywords planted in some (start, middle, end, mixed
    case), between short log lines: bit-exact vs the oracle."""
    import dgrep

    kws = dgrep.synth_keywords(4, 1000)
    rnd = random.Random(41)
    words = [b"request", b"user", b"cache", b"latency", b"retry", b"shard", b"value", b"node"]
    parts = []
    for i in range(9):
        L = rnd.randrange(1 << 20, 8 << 20)
        body = bytearray(b" ".join(rnd.choice(words) for _ in range(L // 5))[:L])
        where = i % 4
        if where:
            kw = bytearray(rnd.choice(kws))
            for k in range(len(kw)):
                if rnd.random() < 0.5:
                    kw[k] -= 32
            q = {1: 0, 2: L // 2, 3: L - len(kw)}[where]
            body[q:q + len(kw)] = kw
        parts.append(bytes(body))
        parts.append(dgrep.synth_corpus_host(rnd.randrange(100, 20000), 300 + i, 1).rstrip(b"\n"))
    data = b"\n".join(parts)
    pattern = _c4_pattern()
    st = _check(gpu_ctx, pattern, data)
    assert st["stepper"] == "filter", st


def test_filter_long_lines_synth_kind4(gpu_ctx):
    """The long_c4 bench workload's corpus (synth kind 4) on the filter stepper,
    24 MiB generated on the host, vs the oracle."""
    import dgrep

    data = dgrep.synth_corpus_host(24 << 20, 4, 4)
    assert data.count(b"\n") < 10000  # mostly long lines
    st = _check(gpu_ctx, _c4_pattern(), data)
    assert st["stepper"] == "filter", st


def test_filter_long_lines_large_keyword_dfa(gpu_ctx):
    """3,000 (?i) keywords (18,584 DFA states): the whole-DFA LDS image of the
    long-line and verification kernels holds ~230 whole rows and a default-row
    record for every other state (csrc/runtime build_ximg), so most cold steps
    go through records; long lines with planted keywords and log lines between,
    bit-exact vs the oracle."""
    import dgrep

    kws = [k for s in (4, 5, 6) for k in dgrep.synth_keywords(s, 1000)]
    rnd = random.Random(4242)
    words = [b"request", b"user", b"cache", b"latency", b"retry", b"shard", b"value", b"node"]
    parts = []
    for i in range(8):
        L = rnd.randrange(256 << 10, 2 << 20)
        body = bytearray(b" ".join(rnd.choice(words) for _ in range(L // 5))[:L])
        for _ in range(i % 3):
            kw = rnd.choice(kws)
            q = rnd.randrange(L - len(kw))
            body[q:q + len(kw)] = kw
        parts.append(bytes(body))
        parts.append(dgrep.synth_corpus_host(rnd.randrange(100, 20000), 500 + i, 1).rstrip(b"\n"))
    data = b"\n".join(parts)
    st = _check(gpu_ctx, b"(?i)(" + b"|".join(kws) + b")", data)
    assert st["stepper"] == "filter" and st["pending"] > 0, st


@pytest.mark.parametrize("extra", [b"|^([^k]*k[^k]*k)*[^k]*$",     # an even number of k (parity: never forgets)
                                   b"|^([^k]*k[^k]*k[^k]*k)*[^k]*$",  # k count divisible by 3
                                   b"|k[^z]*y"])                     # a k since the last z, then y
def test_filter_long_lines_unbounded_memory(gpu_ctx, extra):
    """Parked filter lines whose DFA keeps a finite memory of the WHOLE line
    (config 4's keywords OR a k-parity / k-count-mod-3 / k-then-y branch):
    a segment's entry state is not the state its 256-byte lookback reaches from
    start, so the seg kernel's extra lookback seeds must supply the right guess
    (or the fix kernel re-runs the segment from the true state). Lines of
    0.3-3 MiB whose k count / z placement is chosen so that both verdicts
    occur, the bench workload long_c4p's corpus (synth kind 4), bit-exact vs
    the oracle."""
    import dgrep

    rnd = random.Random(zlib_crc(extra))
    words = [b"request", b"user", b"cache", b"latency", b"retry", b"shard", b"value", b"node", b"kind", b"yes",
             b"zone"]
    parts = []
    for i in range(10):
        L = rnd.randrange(300 << 10, 3 << 20)
        body = bytearray(b" ".join(rnd.choice(words) for _ in range(L // 5))[:L])
        if i % 2:  # flip the k parity of the line at a random place
            q = rnd.randrange(L)
            body[q] = ord("k") if body[q] != ord("k") else ord("x")
        parts.append(bytes(body))
        parts.append(dgrep.synth_corpus_host(rnd.randrange(100, 20000), 700 + i, 1).rstrip(b"\n"))
    data = b"\n".join(parts) + b"\n" + dgrep.synth_corpus_host(20 << 20, 4, 4)
    st = _check(gpu_ctx, _c4_pattern() + extra, data)
    assert st["stepper"] == "filter" and st["pending"] > 0, st


def zlib_crc(b):
    import zlib

    return zlib.crc32(b)
