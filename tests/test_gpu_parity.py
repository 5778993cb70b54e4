"""GPU parity: libdgrep.so (HIP, gfx950) against the CPU oracle.

Every test calls the product through its C ABI (dgrep_scan / dgrep_scan_device)
and compares bit-exactly with the oracle's restatement of grep.go Map
(oracle/, parity unpinned — see oracle/oracle.h). Sizes are chosen so the
oracle finishes in seconds; full-size runs are covered by bench.py's
size-independent checks.
"""
import random
import zlib

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

PATTERNS = [
    b"error",
    b"",
    b"^$",
    b"(?i)ERROR",
    b"timeout while waiting for lock",
    b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+",
    b"\\bkey\\b",
    b"k$",
    b"^2024-0[1-3]",
    b"[^a-z ]{3}",
    b"\\x{FFFD}",
    b"^[ -~]{45}$",
    b"(?i)k",
    b"a**",  # Go syntax error: nothing matches
    b"e(r|x)+o",
]


def _oracle(pattern, data, threads=1):
    ln, st, le = O.grep_map(pattern, data, threads=threads)
    return ln, st, le


def _check(ctx, pattern, data, threads=1):
    import dgrep

    if isinstance(pattern, dgrep.CompiledPattern):
        pattern = pattern.pattern
    else:
        ctx.load(pattern)
    ln, st, le = ctx.scan(data)
    oln, ost, ole = _oracle(pattern, data, threads)
    assert len(ln) == len(oln), (pattern, len(ln), len(oln))
    np.testing.assert_array_equal(ln, oln)
    np.testing.assert_array_equal(st, ost)
    np.testing.assert_array_equal(le, ole)
    return len(ln)


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_synth_device_matches_host(gpu_ctx, kind):
    import torch
    import dgrep

    n = (1 << 22) + 12345
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu_ctx.synth(buf.data_ptr(), n, 7, kind)
    torch.cuda.synchronize()
    host = dgrep.synth_corpus_host(n, 7, kind)
    assert buf.cpu().numpy().tobytes() == host


@pytest.mark.parametrize("pattern", PATTERNS)
def test_edge_inputs(gpu_ctx, pattern):
    cases = [b"", b"\n", b"\n\n", b"error", b"error\n", b"x\nerror", b"\nerror\n\n", b"key\nk\n",
             b"\xff\xfe\n\xe2\x82\xac\n\xe2\x82\n", b"a" * 5000 + b"error" + b"b" * 5000 + b"\nerror"]
    for data in cases:
        _check(gpu_ctx, pattern, data)


@pytest.mark.parametrize("pattern", PATTERNS)
def test_random_small(gpu_ctx, pattern):
    rnd = random.Random(zlib.crc32(pattern) & 0xffff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b"K", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\r", b"\xe2\x82\xac",
             b"\xe2\x82", b"\xff", b"\xc5\xbf", b"WARN", b"ERROR", b"error", b"2024-01", b"key "]
    for _ in range(20):
        n = rnd.choice([10, 100, 1000, 70000, 300000])
        data = b"".join(rnd.choice(alpha) for _ in range(n // 3))
        _check(gpu_ctx, pattern, data)


# chunk edges: 1 KiB (table stepper) / 4 KiB (Sheng); tile edges: 64 KiB / 256 KiB
@pytest.mark.parametrize("size", [1, 63, 64, 127, 128, 129, 1023, 1024, 1025, 2048, 2049, 4095, 4096, 4097, 65535,
                                  65536, 65537, 131071, 131072, 131073, 262143, 262144, 262145, 3 * 262144 + 17])
def test_tile_and_chunk_boundaries(gpu_ctx, size):
    import dgrep

    data = bytearray(dgrep.synth_corpus_host(size, 11, 0))
    # force lines that end / start exactly at chunk and tile edges
    for edge in (1023, 1024, 2047, 2048, 4095, 4096, 65535, 65536, 131071, 131072, 262143, 262144):
        if edge < size:
            data[edge] = 0x0A
    data = bytes(data)
    for pattern in (b"error", b"", b"^2024", b"ok$", b"(WARN|ERROR) [a-z_]+"):
        _check(gpu_ctx, pattern, data)


# Sheng stepper with the lane chunks the adaptive choice produces on large
# splits (dgrep_set_lane_chunk forces them at oracle-friendly sizes): chunk and
# tile edges, lines longer than a chunk, and more matching lines per lane than
# LDS slots (pattern "" matches every line: the overflow kernel)
@pytest.mark.parametrize("chunk", [4224, 8192, 14592, 16384, 32768, 65536])
def test_sheng_adaptive_chunks(gpu_ctx, chunk):
    import dgrep

    tile = 64 * chunk
    try:
        gpu_ctx.set_lane_chunk(chunk)
        for size in (chunk - 1, chunk + 1, tile - 1, tile, tile + 1, 2 * tile + 777):
            data = bytearray(dgrep.synth_corpus_host(size, 13, 0))
            for edge in (chunk - 1, chunk, 2 * chunk, tile - 1, tile, tile + chunk):
                if edge < size:
                    data[edge] = 0x0A
            if size > 3 * chunk:
                data[chunk + 5:3 * chunk] = b"x" * (2 * chunk - 5)  # a line over two chunk edges
                data[2 * chunk:2 * chunk + 5] = b"error"
            data = bytes(data)
            for pattern in (b"error", b"", b"^2024", b"ok$"):
                cp = gpu_ctx.load(pattern)
                assert cp.nstates <= 8, (pattern, cp.nstates)
                _check(gpu_ctx, cp, data)
    finally:
        gpu_ctx.set_lane_chunk(0)


def test_lane_chunk_validation(gpu_ctx):
    import dgrep

    for bad in (100, 4000, 4097, 32900, 65664, 131072, 1 << 20):
        with pytest.raises(dgrep.DgrepError):
            gpu_ctx.set_lane_chunk(bad)
    gpu_ctx.set_lane_chunk(0)


@pytest.mark.parametrize("stepper", ["auto", "pair", "filter"])
@pytest.mark.parametrize("chunk", [32768, 65536])
def test_lines_starting_at_chunk_end(gpu_ctx, stepper, chunk):
    """A lane's last owned line can start exactly AT its chunk end (the chunk's
    last byte is '\\n'): at 64 KiB chunks that start (65,536) does not fit the
    LDS slot's 16 bits -- round 4's 64 KiB build stored it as 0 and failed the
    32 GiB C5 parity. Short and parked (pending) lines there, on every lane of
    a tile; and a tile of nothing but '\\n' before a matching line, whose
    tile-relative line index (64 C newlines = 2^22 at 64 KiB) needs 23 bits."""
    import dgrep

    tile = 64 * chunk
    rnd = random.Random(chunk + len(stepper))
    data = bytearray(dgrep.synth_corpus_host(3 * tile + 999, 21, 0))
    for lane in range(3 * 64):
        e = (lane + 1) * chunk - 1
        data[e] = 0x0A
        kind = rnd.randrange(4)
        if kind == 0:  # a short matching line right at the chunk end
            data[e + 1:e + 12] = b"error here\n"
        elif kind == 1 and lane % 7 == 0:  # a long line from the chunk end (parked), matching at its far end
            L = chunk + 4096 + 700 if rnd.random() < 0.5 else 2 * chunk + 300
            L = min(L, len(data) - e - 40)
            data[e + 1:e + 1 + L] = b"y" * (L - 8) + b"error!!\n"
    data = bytes(data)
    newline_tile = b"\n" * tile + b"x error\n" + b"ok\n" * 100 + b"\n" * (chunk - 1) + b"error tail"
    try:
        gpu_ctx.set_stepper(stepper)
        gpu_ctx.set_lane_chunk(chunk)
        for pattern in (b"error", b"^$|error", b"!!$", b"x error"):
            cp = gpu_ctx.load(pattern)
            _check(gpu_ctx, cp, data, threads=16)
            st = gpu_ctx.scan_stats()
            assert st["lane_chunk"] == chunk, st
            # auto: Sheng for <= 8 states ("error"), else the pair stepper
            assert st["stepper"] == stepper or (stepper == "auto" and st["stepper"] in ("sheng", "pair")), st
            _check(gpu_ctx, cp, newline_tile, threads=16)
    finally:
        gpu_ctx.set_lane_chunk(0)
        gpu_ctx.set_stepper("auto")


# table-stepper instantiations: <= 64 states run two chunks per lane (tile 256
# KiB), 65-256 states one (tile 128 KiB); both at their chunk and tile edges
@pytest.mark.parametrize("pattern", [b"(alpha|bravo|charlie|delta|echo|foxtrot|golf|hotel|india|juliet)[0-9]+",
                                     b"(alpha|bravo|charlie|delta|echo|foxtrot|golf|hotel|india|juliet|kilo|lima|"
                                     b"mike|november|oscar|papa|quebec|romeo)"])
def test_table_stream_configs_at_edges(gpu_ctx, pattern):
    import dgrep

    rnd = random.Random(7)
    words = [b"alpha", b"bravo7", b"romeo", b"x", b"juliet12", b"error", b" ", b"  ", b"quebec", b"kilo9"]
    for size in (2047, 2048, 2049, 131071, 131072, 131073, 262143, 262144, 262145, 5 * 131072 + 33):
        data = bytearray(b"".join(rnd.choice(words) for _ in range(size // 3))[:size])
        for edge in (2047, 2048, 4095, 4096, 131071, 131072, 262143, 262144):
            if edge < len(data):
                data[edge] = 0x0A
        try:
            gpu_ctx.set_stepper("table")
            cp = gpu_ctx.load(pattern)
            assert 8 < cp.nstates <= 256
            _check(gpu_ctx, cp, bytes(data))
            assert gpu_ctx.scan_stats()["stepper"] == "table"
        finally:
            gpu_ctx.set_stepper("auto")


def test_long_lines_cross_many_chunks(gpu_ctx):
    rnd = random.Random(3)
    parts = []
    for i in range(40):
        L = rnd.choice([10, 5000, 300000, 70000])
        body = bytes(rnd.choice(b"abcdefghij ") for _ in range(L))
        if rnd.random() < 0.5:
            p = rnd.randrange(L)
            body = body[:p] + b"error" + body[p:]
        parts.append(body)
    data = b"\n".join(parts)
    for pattern in (b"error", b"^[a-j ]*$", b"error$", b""):
        _check(gpu_ctx, pattern, data)


def test_dense_matches_overflow_slots(gpu_ctx):
    # every line matches and lines are short: lanes own far more matching lines
    # than their LDS slots and take the direct-write path
    data = b"\n".join(b"error %d" % i for i in range(200000))
    _check(gpu_ctx, b"error", data)
    _check(gpu_ctx, b"", data)
    data2 = b"\n" * 100000
    _check(gpu_ctx, b"", data2)
    _check(gpu_ctx, b"^$", data2)


def _dense_lines(seed, count, maxlen):
    rnd = random.Random(seed)
    return b"\n".join(b"error WARN ab " + b"x" * rnd.randrange(maxlen) for _ in range(count))


@pytest.mark.parametrize("chunk", [4096, 8192, 32768, 65536])
def test_overflow_pass_dense_every_chunk(gpu_ctx, chunk):
    """More matching lines per lane chunk than LDS slots at every Sheng chunk
    shipped: the wave-parallel overflow pass (one wave per lane chunk, 64
    sub-chunks, count pass + write pass) must give the oracle's records,
    including lines that cross sub-chunk and chunk edges."""
    try:
        gpu_ctx.set_lane_chunk(chunk)
        for maxlen in (4, 40, 700, 0):
            # maxlen 0: 2-byte lines, more matching lines per lane than its LDS
            # slots plus its HBM spill area hold -> the overflow pass
            data = (_dense_lines(chunk + maxlen, 40000 if maxlen < 100 else 8000, maxlen) if maxlen else
                    b"e\n" * 300000)
            for pattern in (b"error", b"", b"b x", b"e"):
                cp = gpu_ctx.load(pattern)
                assert cp.nstates <= 8
                n = _check(gpu_ctx, cp, data)
                st = gpu_ctx.scan_stats()
                assert st["stepper"] == "sheng" and st["lane_chunk"] == chunk
                if maxlen == 0 and n:
                    assert st["overflow_lanes"] > 0, st
    finally:
        gpu_ctx.set_lane_chunk(0)


@pytest.mark.parametrize("pattern", [b"(WARN|ERROR) [a-z_]+", b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+|error"])
def test_overflow_pass_dense_table(gpu_ctx, pattern):
    try:
        gpu_ctx.set_stepper("table")
        for maxlen in (4, 40, 700):
            data = _dense_lines(maxlen, 30000 if maxlen < 100 else 6000, maxlen)
            cp = gpu_ctx.load(pattern)
            assert 8 < cp.nstates <= 256
            _check(gpu_ctx, cp, data)
            st = gpu_ctx.scan_stats()
            assert st["stepper"] == "table"
            if maxlen < 100:
                assert st["overflow_lanes"] > 0
    finally:
        gpu_ctx.set_stepper("auto")


def test_adaptive_chunk_on_large_split_and_density_cap(gpu_ctx):
    """The adaptive Sheng chunk on a 6 GiB HBM-resident split (large enough to
    select more than the compiled 4 KiB at >= 2.5 tiles per resident wave:
    dgrep_last_scan_stats reports it),
    then a dense pattern: after its first scan the match density caps the
    chunk. Every record is checked structurally and evenly spaced windows
    (split start and end included) against the oracle (bench.verify_windows)."""
    import torch
    import bench

    n = 6 << 30
    buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    gpu_ctx.synth(buf.data_ptr(), n, 21, 0)
    cap = 100 << 20
    ln = torch.empty(cap, dtype=torch.int64, device="cuda")
    st = torch.empty(cap, dtype=torch.int64, device="cuda")
    le = torch.empty(cap, dtype=torch.int64, device="cuda")
    chunks = {}
    for pattern in ("error", "r"):
        gpu_ctx.load(pattern)
        for rep in range(2):
            cnt = gpu_ctx.scan_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cap)
            assert 0 < cnt <= cap
            s = gpu_ctx.scan_stats()
            chunks[(pattern, rep)] = s["lane_chunk"]
            assert bench.verify_windows(buf, n, ln[:cnt], st[:cnt], le[:cnt], pattern, 3, 1 << 20) == 3
    assert chunks[("error", 0)] >= 8192 and chunks[("error", 1)] == chunks[("error", 0)], chunks
    # "r" matches nearly every ~120-B line: 24 slots cap the chunk at the 4 KiB floor
    assert chunks[("r", 0)] >= 8192 and chunks[("r", 1)] == 4096, chunks
    # the pair stepper (config 3's pattern): 4.5 KiB doubled once, to its 9 KiB cap
    c3 = "^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+"
    gpu_ctx.load(c3)
    cnt = gpu_ctx.scan_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cap)
    assert 0 <= cnt <= cap
    s = gpu_ctx.scan_stats()
    assert s["stepper"] == "pair" and s["lane_chunk"] == 9216, s
    assert bench.verify_windows(buf, n, ln[:cnt], st[:cnt], le[:cnt], c3, 3, 1 << 20) == 3
    del buf, ln, st, le
    torch.cuda.empty_cache()


@pytest.mark.parametrize("seed,pattern", [(1, b"error"), (2, b"timeout while waiting for lock"),
                                          (3, b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+")])
def test_synth_corpus_vs_oracle(gpu_ctx, seed, pattern):
    import dgrep

    data = dgrep.synth_corpus_host(24 << 20, seed, 0)
    n = _check(gpu_ctx, pattern, data, threads=16)
    assert n > 0


def test_scan_device_resident(gpu_ctx):
    import torch
    import dgrep

    n = 32 << 20
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu_ctx.synth(buf.data_ptr(), n, 1, 0)
    gpu_ctx.load(b"error")
    cap = 1 << 20
    ln = torch.empty(cap, dtype=torch.int64, device="cuda")
    st = torch.empty(cap, dtype=torch.int64, device="cuda")
    le = torch.empty(cap, dtype=torch.int64, device="cuda")
    cnt = gpu_ctx.scan_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), cap)
    host = buf.cpu().numpy().tobytes()
    oln, ost, ole = O.grep_map(b"error", host, threads=16)
    assert cnt == len(oln)
    np.testing.assert_array_equal(ln[:cnt].cpu().numpy().astype(np.uint64), oln)
    np.testing.assert_array_equal(st[:cnt].cpu().numpy().astype(np.uint64), ost)
    np.testing.assert_array_equal(le[:cnt].cpu().numpy().astype(np.uint64), ole)
    # capacity too small: count reported, caller retries
    cnt2 = gpu_ctx.scan_device(buf.data_ptr(), n, ln.data_ptr(), st.data_ptr(), le.data_ptr(), 10)
    assert cnt2 == cnt


@pytest.mark.parametrize("chunk,bufs,threads", [(1 << 20, 2, 1), ((1 << 20) + 4097, 3, 4), (8 << 20, 4, 8)])
def test_ingest_pipeline_bit_exact(chunk, bufs, threads):
    """dgrep_scan's pinned-staging ingest (pieces of `chunk` bytes through
    `bufs` rotating buffers) lands the split in HBM byte for byte: same
    records as the direct copy and as the oracle, across piece boundaries."""
    import dgrep

    data = bytearray(dgrep.synth_corpus_host(20 << 20, 5, 0))
    for k in range(1, 20):  # lines ending exactly at piece edges
        e = k * chunk
        if e < len(data):
            data[e - 1] = 0x0A
    data = bytes(data)
    ctx = dgrep.Context(0)
    try:
        for pattern in (b"error", b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+"):
            ctx.load(pattern)
            ctx.set_ingest(0)
            want = ctx.scan(data)
            ctx.set_ingest(chunk, bufs, threads)
            got = ctx.scan(data)
            assert ctx.last_ingest_ms() > 0
            for g, w in zip(got, want):
                np.testing.assert_array_equal(g, w)
            oln, ost, ole = _oracle(pattern, data, 16)
            np.testing.assert_array_equal(got[0], oln)
            np.testing.assert_array_equal(got[1], ost)
            np.testing.assert_array_equal(got[2], ole)
            # a second, shorter split reuses the staging buffers
            short = data[: (5 << 20) + 3]
            got2 = ctx.scan(short)
            o2 = _oracle(pattern, short, 16)
            np.testing.assert_array_equal(got2[0], o2[0])
            np.testing.assert_array_equal(got2[1], o2[1])
    finally:
        ctx.close()


def test_map_reduce_surface(gpu_ctx):
    import dgrep

    dgrep.set_pattern("error")
    kva = dgrep.Map("log.txt", "ok\nan error\nerror\n")
    assert kva == [dgrep.KeyValue("log.txt (line number #2)", "an error"),
                   dgrep.KeyValue("log.txt (line number #3)", "error")]
    assert dgrep.Reduce(kva[0].Key, [kva[0].Value, "x"]) == "an error"
    dgrep.set_pattern("")
    assert len(dgrep.Map("f", "a\nb\n")) == 3  # trailing empty line matches ""
    dgrep.set_pattern("a**")
    assert dgrep.Map("f", "a\n") == []


# ---- the filter stepper forced on small DFAs (few LDS rows: nearly every line a candidate)
@pytest.fixture
def few_rows_ctx(gpu_ctx):
    yield gpu_ctx
    gpu_ctx.set_stepper("auto", 0)


@pytest.mark.parametrize("rows", [0, 4])  # 0: as many LDS rows as fit; 4: nearly every line verified
@pytest.mark.parametrize("pattern", PATTERNS)
def test_filter_stepper_forced(few_rows_ctx, pattern, rows):
    few_rows_ctx.set_stepper("filter", rows)
    wide_ctx = few_rows_ctx
    rnd = random.Random(zlib.crc32(pattern) & 0xfff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\xe2\x82\xac", b"\xff",
             b"WARN", b"ERROR", b"error", b"2024-01", b"key "]
    for n in (0, 1, 100, 5000, 70000, 300000):
        data = b"".join(rnd.choice(alpha) for _ in range(n // 3))
        _check(wide_ctx, pattern, data)


def test_filter_stepper_boundaries_and_overflow(few_rows_ctx):
    import dgrep

    wide_ctx = few_rows_ctx
    wide_ctx.set_stepper("filter", 4)
    for size in (1023, 1024, 1025, 65535, 65536, 65537, 3 * 65536 + 17):
        data = bytearray(dgrep.synth_corpus_host(size, 11, 0))
        for edge in (1023, 1024, 65535, 65536):
            if edge < size:
                data[edge] = 0x0A
        for pattern in (b"error", b"", b"^2024", b"(WARN|ERROR) [a-z_]+"):
            _check(wide_ctx, pattern, bytes(data))
    data = b"\n".join(b"error %d" % i for i in range(100000))
    _check(wide_ctx, b"error", data)


@pytest.mark.parametrize("nkw,size", [(200, 4 << 20), (1000, 1 << 20), (1000, 12 << 20)])
def test_keyword_alternation_c4(gpu_ctx, nkw, size):
    """SURVEY config 4: (?i) alternation of seeded keywords (> 256 DFA states):
    the filter stepper, whose candidates are verified on the whole DFA."""
    import dgrep

    kws = dgrep.synth_keywords(4, nkw)
    pattern = b"(?i)(" + b"|".join(kws) + b")"
    cp = gpu_ctx.load(pattern)
    assert cp.nstates > 256
    data = dgrep.synth_corpus_host(size, 4, 1)
    n = _check(gpu_ctx, cp, data, threads=16)
    assert n > 0
    st = gpu_ctx.scan_stats()
    assert st["stepper"] == ("filter" if nkw == 1000 else "filter"), st
    if nkw == 1000:
        assert st["candidates"] > 0, st  # lines that left the LDS states and did not match


@pytest.fixture
def filter_ctx(gpu_ctx):
    yield gpu_ctx
    gpu_ctx.set_stepper("auto")


@pytest.mark.parametrize("rows", [0, 3, 6])  # 0: as many LDS rows as fit; 3/6: nearly every line a candidate
@pytest.mark.parametrize("pattern", PATTERNS)
def test_filter_stepper_forced(filter_ctx, pattern, rows):
    filter_ctx.set_stepper("filter", rows)
    rnd = random.Random(zlib.crc32(pattern) & 0xfff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\xe2\x82\xac", b"\xff",
             b"WARN", b"ERROR", b"error", b"2024-01", b"key "]
    for n in (0, 1, 100, 5000, 70000, 300000):
        data = b"".join(rnd.choice(alpha) for _ in range(n // 3))
        try:
            _check(filter_ctx, pattern, data)
        except dgrep_unsupported():
            assert rows in (3, 6)  # too few rows for start, start_m and CAND
            return
        if n:
            assert filter_ctx.scan_stats()["stepper"] == "filter"


def dgrep_unsupported():
    import dgrep

    return dgrep.UnsupportedPattern


@pytest.mark.parametrize("chunk", [0, 65536])  # 65536: the adaptive filter cap on 16 GiB splits
def test_filter_candidates_dense_and_long(filter_ctx, chunk):
    """Every line a candidate (3 LDS rows): staging grows past the caller's
    capacity, verification keeps exactly the matching lines, at chunk, tile
    and overflow edges; lines longer than a chunk."""
    import dgrep

    filter_ctx.set_stepper("filter", 4)
    big = (9 << 20) + 12345 if chunk else 3 << 20  # > 2 tiles at 64 KiB chunks
    try:
        filter_ctx.set_lane_chunk(chunk)
        for pattern in (b"error", b"(WARN|ERROR) [a-z_]+", b"^$|ab x"):
            for data in (_dense_lines(5, 60000, 6), _dense_lines(6, 3000, 3000),
                         dgrep.synth_corpus_host(big, 9, 0)):
                _check(filter_ctx, pattern, data, threads=16)
                st = filter_ctx.scan_stats()
                assert st["stepper"] == "filter", st
                if chunk:
                    assert st["lane_chunk"] == chunk, st
    finally:
        filter_ctx.set_lane_chunk(0)


def test_filter_long_candidates_wave_verified(filter_ctx):
    """Candidate lines above verify_kernel's wave threshold (16 KiB) are decided
    by the whole wave from guessed segment entry states: keyword-style
    patterns (the guess is exact), an anchored one and one whose state remembers
    an unbounded past (guesses wrong, segments re-run in order), matches at the start, middle, end or not
    at all, lines up to past the filter's park point; every line a candidate
    (4 LDS rows) and the shipped LDS image."""
    import dgrep

    rnd = random.Random(1616)
    alpha = [b"a", b"b", b"e", b"r", b"o", b"x", b"y", b"k", b" ", b"_", b"1", b"z"]
    kws = dgrep.synth_keywords(4, 200)
    lines = []
    for i in range(40):
        n = rnd.randrange(16500, 90000)
        body = bytearray(b"".join(rnd.choice(alpha) for _ in range(n)))
        where = rnd.choice(["none", "start", "mid", "end"])
        tok = rnd.choice([b"error", b"ERROR abc", rnd.choice(kws).upper(), b"ab"])
        if where == "start":
            body[0:len(tok)] = tok
        elif where == "mid":
            m = rnd.randrange(len(body) - len(tok))
            body[m:m + len(tok)] = tok
        elif where == "end":
            body[-len(tok):] = tok
        lines.append(bytes(body))
        lines.append(b"short line %d" % i)
    data = b"\n".join(lines) + b"\n"
    # only lines of 16.5-30 KiB, each right after a '\n' at a 32 KiB chunk's
    # first byte (filler lines between): at 32 KiB chunks none is parked (the
    # filter parks a line still open 4 KiB past its owner's chunk end), so
    # every dropped candidate went through the wave verifier
    mid = bytearray()
    for l in lines:
        if 16500 <= len(l) < 30000:
            mid += b"z" * ((-len(mid)) % 32768) + b"\n" + l + b"\n"
    mid = bytes(mid)
    patterns = [b"error", b"(WARN|ERROR) [a-z_]+", b"^ab.*x", b"k[^z]*y",
                b"(?i)(" + b"|".join(kws) + b")"]
    try:
        # 32 KiB chunks: lines of 16-64 KiB stay candidates (wave-verified),
        # longer ones are parked; 0 = adaptive (4 KiB here): lines over 8 KiB parked
        for chunk in (32768, 0):
            filter_ctx.set_lane_chunk(chunk)
            for rows in (4, 0):
                for pattern in patterns:
                    filter_ctx.set_stepper("filter", rows)
                    _check(filter_ctx, pattern, data, threads=16)
                    st = filter_ctx.scan_stats()
                    assert st["stepper"] == "filter"
                    assert st["pending"] > 0, st
                    if chunk and rows == 4:
                        _check(filter_ctx, pattern, mid, threads=16)
                        st = filter_ctx.scan_stats()
                        assert st["pending"] == 0 and st["lane_chunk"] == chunk, st
                        # 4 LDS rows: every line is a candidate; those not matching are dropped
                        if pattern in (b"error", b"(WARN|ERROR) [a-z_]+", b"^ab.*x"):
                            assert st["candidates"] > 0, st
    finally:
        filter_ctx.set_lane_chunk(0)


def test_filter_verification_with_overflow(filter_ctx):
    """Filter with 4 LDS rows (nearly every line a candidate) and lanes whose
    records overflow their slots + spill: candidates staged by the scan AND by
    the overflow pass are decided by verify_kernel in one call, bit-exact vs
    the oracle."""
    filter_ctx.set_stepper("filter", 4)
    try:
        filter_ctx.set_lane_chunk(4096)
        # 4-7 B lines: ~750 per 4 KiB lane chunk (> 4 slots + 240 spill records)
        # in the dense part, longer lines after it (lanes that verify in-kernel)
        rnd = random.Random(7)
        data = b"\n".join(b"ab " + b"x" * rnd.randrange(4) for _ in range(60000)) + b"\n" + b"\n".join(
            b"noise line %d: a b, ab xx, the pattern or not" % i for i in range(20000))
        for pattern in (b"ab x{3}", b"^ab x?$", b"b xx"):
            _check(filter_ctx, pattern, data, threads=16)
            st = filter_ctx.scan_stats()
            assert st["stepper"] == "filter", st
            assert st["overflow_lanes"] > 0, st
            assert st["candidates"] > 0, st  # dropped, in the kernel or by verify_kernel
    finally:
        filter_ctx.set_lane_chunk(0)


# ---- the pair stepper (two bytes per LDS lookup, shadow states) -------------
PAIR_PATTERNS = [b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"(WARN|ERROR) [a-z_]+",
                 b"timeout while waiting for lock", b"\\bkey\\b", b"^[ -~]{45}$", b"e(r|x)+o", b"a|^$",
                 b"[^a-z ]{3}", b"^$|error", b"x*$|WARN"]


@pytest.fixture
def pair_ctx(gpu_ctx):
    # the pair stepper (two bytes per lookup), also for DFAs the default gives
    # to Sheng (<= 8 states)
    gpu_ctx.set_stepper("pair")
    gpu_ctx.test_mode = "pair"
    yield gpu_ctx
    gpu_ctx.set_stepper("auto")


def _load_mode(ctx, pattern):
    return ctx.load(pattern)


@pytest.mark.parametrize("pattern", PAIR_PATTERNS + [b"error", b"", b"^$", b"(?i)k", b"\\x{FFFD}"])
def test_pair_stepper_edges_and_random(pair_ctx, pattern):
    gpu_ctx = pair_ctx
    cp = _load_mode(gpu_ctx, pattern)
    for data in [b"", b"\n", b"\n\n", b"\n\n\n", b"x", b"x\n", b"\nx", b"error\n\nerror", b"key\nk\n",
                 b"\xff\xfe\n\xe2\x82\xac\n\xe2\x82\n", b"a" * 5000 + b"WARN ab" + b"b" * 5000 + b"\nerror"]:
        _check(gpu_ctx, cp, data)
        assert gpu_ctx.scan_stats()["stepper"] == gpu_ctx.test_mode, pattern
    rnd = random.Random(zlib.crc32(pattern) & 0xffff)
    alpha = [b"a", b"e", b"r", b"o", b"x", b"k", b" ", b"_", b"1", b"-", b"\n", b"\n", b"\n\n", b"\r",
             b"\xe2\x82\xac", b"\xff", b"WARN ab", b"ERROR x", b"error", b"2024-01-02", b"key "]
    for _ in range(12):
        n = rnd.choice([10, 1000, 70000, 300000])
        _check(gpu_ctx, cp, b"".join(rnd.choice(alpha) for _ in range(n // 3)))


@pytest.mark.parametrize("chunk", [4096, 4224, 8192, 12416, 32768, 65536])
def test_pair_stepper_chunk_and_tile_edges(pair_ctx, chunk):
    """Chunk and tile edges at forced lane chunks, including odd multiples of
    the 128-B block (4224 = 33 blocks, 12416 = 97): the wave-uniform in-chunk
    loop steps two blocks per iteration and must stop exactly at C."""
    import dgrep

    gpu_ctx = pair_ctx
    tile = 64 * chunk
    try:
        gpu_ctx.set_lane_chunk(chunk)
        for size in (chunk - 1, chunk, chunk + 1, tile - 1, tile, tile + 1, 2 * tile + 777):
            data = bytearray(dgrep.synth_corpus_host(size, 17, 0))
            # '\n' first and second in a pair at chunk / tile edges and beside them
            for edge in (chunk - 2, chunk - 1, chunk, chunk + 1, 2 * chunk, tile - 1, tile, tile + chunk):
                if edge < size:
                    data[edge] = 0x0A
            if size > 3 * chunk:
                data[chunk + 5:3 * chunk] = b"x" * (2 * chunk - 5)  # a line over two chunk edges
                data[2 * chunk:2 * chunk + 8] = b" WARN ab"
            data = bytes(data)
            for pattern in (b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", b"^$|ok$", b"(WARN|ERROR) [a-z_]+"):
                cp = _load_mode(gpu_ctx, pattern)
                _check(gpu_ctx, cp, data)
                st = gpu_ctx.scan_stats()
                assert st["stepper"] == gpu_ctx.test_mode and st["lane_chunk"] == chunk, st
    finally:
        gpu_ctx.set_lane_chunk(0)


def test_pair_stepper_dense_overflow(pair_ctx):
    gpu_ctx = pair_ctx
    for maxlen in (2, 5, 40, 700):
        data = _dense_lines(maxlen + 1, 40000 if maxlen < 100 else 6000, maxlen)
        for pattern in (b"(WARN|ERROR) [a-z_]+", b"^$|error", b"b x*$"):
            cp = _load_mode(gpu_ctx, pattern)
            _check(gpu_ctx, cp, data)
            assert gpu_ctx.scan_stats()["stepper"] == gpu_ctx.test_mode
    data2 = b"\n" * 100001
    for pattern in (b"^$|error", b"a|^$"):
        _check(gpu_ctx, _load_mode(gpu_ctx, pattern), data2)


@pytest.mark.parametrize("chunk", [4096, 32768])
def test_pair_deferred_events_line_shapes(pair_ctx, chunk):
    """The pair stepper's event path: matching and non-matching lines of
    every length 1..260 B in a rotating order, so every 128-B block position
    holds an event word, a previous '\\n' in the same word / an earlier word /
    an earlier block, and blocks with several '\\n' in one word next to events
    (the general per-word loop)."""
    gpu_ctx = pair_ctx
    rnd = random.Random(chunk)
    lines = []
    for i in range(60000):
        n = rnd.choice([1, 2, 3, 4, 5, 7, 8, 13, 40, 64, 127, 128, 129, 260]) if i % 3 else rnd.randint(1, 260)
        body = bytes(rnd.choice(b"abxy _-") for _ in range(n - 1))
        if rnd.random() < 0.3 and n > 8:
            k = rnd.randint(0, n - 9)
            body = body[:k] + b"WARN ab" + body[k + 7:]
        lines.append(body[: n - 1] + b"\n")
    data = b"".join(lines)
    try:
        gpu_ctx.set_lane_chunk(chunk)
        for pattern in (b"(WARN|ERROR) [a-z_]+", b"^$|b$", b"WARN ab"):
            cp = _load_mode(gpu_ctx, pattern)
            _check(gpu_ctx, cp, data)
            _check(gpu_ctx, cp, data[: len(data) // 2 + 13])
            assert gpu_ctx.scan_stats()["stepper"] == gpu_ctx.test_mode
    finally:
        gpu_ctx.set_lane_chunk(0)


@pytest.mark.parametrize("mode", ["table", "pair", "filter"])
def test_forced_steppers_agree_on_c3(gpu_ctx, mode):
    """C3's regex through each stepper that can hold it (dgrep_set_stepper)."""
    import dgrep

    data = dgrep.synth_corpus_host(6 << 20, 3, 0)
    try:
        gpu_ctx.set_stepper(mode)
        cp = gpu_ctx.load(b"^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+")
        _check(gpu_ctx, cp, data, threads=16)
        assert gpu_ctx.scan_stats()["stepper"] == mode
    finally:
        gpu_ctx.set_stepper("auto")


@pytest.mark.parametrize("pattern", [b"a[ab]{15}$", b"a[ab]{16}$", b"(?i)b[ab]{15}[^b]$"])
def test_dfa_beyond_65535_states(gpu_ctx, pattern):
    """DFAs of 65,536 .. 2^21 states (the compiler's budget): the filter keeps
    the shallowest rows in LDS and verifies candidate lines on the whole DFA,
    read with u32 ids from HBM (no u16 limit)."""
    cp = gpu_ctx.load(pattern)
    assert cp.nstates > 65535, cp.nstates
    rnd = random.Random(len(pattern))
    lines = []
    for _ in range(30000):
        L = rnd.choice([3, 10, 17, 18, 25, 60])
        lines.append(bytes(rnd.choice(b"ababababAB") if rnd.random() < 0.98 else rnd.choice(b"x \xc5") for _ in range(L)))
    data = b"\n".join(lines)
    n = _check(gpu_ctx, cp, data, threads=16)
    assert n > 0
    st = gpu_ctx.scan_stats()
    assert st["stepper"] == "filter" and st["candidates"] > 0, st


@pytest.mark.parametrize("pattern", ["(?i)é", "(?i)σ+", "(?i)straße", "(?i)\\p{Lu}x", "(?i)[α-ω]{2}", "(?i)\\P{Ll}k",
                                     "(?i)(kelvin|ſ|µ)"])
def test_unicode_case_folding(gpu_ctx, pattern):
    """(?i) over non-ASCII runes: unicode.SimpleFold orbits and FoldCategory
    (generated from Unicode 13.0; parity of the table is unpinned)."""
    rnd = random.Random(pattern)
    alpha = [s.encode() for s in ["é", "É", "e", "σ", "ς", "Σ", "ß", "ẞ", "ss", "STRASSE", "straße", "STRAẞE", "µ",
                                  "Μ", "K", "kelvin", "ſ", "α", "Ω", "x", "X", " ", "\n", "\n"]] + [b"\xff"]
    data = b"".join(rnd.choice(alpha) for _ in range(60000))
    pattern = pattern.encode()
    n = _check(gpu_ctx, pattern, data, threads=16)
    assert n > 0


SCRIPT_PATTERNS = [b"(?i)\\p{Greek}+", b"\\P{Latin}", b"\\p{Han}", b"\\p{Cyrillic}[a-z]", b"(?i)\\p{Common}{3}$",
                   b"\\p{Greek}\\P{Greek}", b"(?i)\\P{Inherited}\\p{Inherited}"]


def _multiscript_split(seed, n_lines):
    rnd = random.Random(seed)
    words = ["error", "Αθήνα", "αβγ", "ΣΟΦΙΑ", "µ", "ͅ", "ι", "ι", "中文", "日本語", "Москва", "дом",
             "K", "K", "ß", "ẞ", "123", "é", "́", "၀0", "\U00010300", " ", "-", ":"]
    lines = []
    for _ in range(n_lines):
        lines.append("".join(rnd.choice(words) for _ in range(rnd.randint(0, 12))).encode() +
                     (b"\xff" if rnd.random() < 0.05 else b""))
    return b"\n".join(lines)


@pytest.mark.parametrize("pattern", SCRIPT_PATTERNS)
def test_unicode_script_classes(gpu_ctx, pattern):
    """\\p{Script} / \\P{Script} (unicode.Scripts, Unicode 13.0) and (?i) with
    unicode.FoldScript, over lines mixing Greek, Latin, Cyrillic, Han, combining
    marks and invalid UTF-8, at small size and across chunk/tile edges."""
    import dgrep

    for size in (0, 2000, 40000):
        _check(gpu_ctx, pattern, _multiscript_split(size, size // 10 + 1), threads=8)
    data = bytearray(dgrep.synth_corpus_host(2 << 20, 13, 0))
    data += _multiscript_split(1, 5000)
    _check(gpu_ctx, pattern, bytes(data), threads=16)
