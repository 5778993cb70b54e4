#!/usr/bin/env python3
"""bench.py — the distributed-grep Map hot path on MI355X.

One *step* = one pass of the Map hot path (application/grep.go:17-29: split on
'\\n' + regexp.Match per line) over one HBM-resident synthetic split, producing
the matching lines' (line_no, start, len) records in HBM (dgrep_scan_device).
With N > 1 ranks (one process per GPU, torch.distributed over RCCL), every rank
scans its own split (Map tasks shard per split, map_reduce/coordinator.go:312)
and the compacted match records are gathered to rank 0 over xGMI in the same
step — the only exchange the path has.

Default workload: at N=1 BASELINE.json configs[1] = SURVEY §8d C2 (a 16 GiB
seeded synthetic log split, literal pattern `error`, LDS-resident DFA); at
N>1 configs[4] = C5 (one 32 GiB split per GPU, seed 100 + rank, `error`, and
the RCCL gather of the match records to rank 0 inside every step).
`value` = whole-job GB/s of text scanned (sum over ranks / max-over-ranks
time); `roofline` = the scan kernel's algorithmic bytes (split bytes read +
16 B per staged match) / its HIP-event time against the 8 TB/s HBM peak;
`cpu_baseline` = the oracle's restatement of grep.go Map (per-line
regexp compile, as grep.go:21 does) on one host core, on a bounded prefix
sample of the same split.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-grep_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
STAGED_LINE_BYTES = 16  # StagedLine written by the scan kernel per match


def kernels_timed(stepper):
    """The kernels dgrep_last_kernel_ms covers for this stepper (roofline.kernel)."""
    step = {"sheng": "StepSheng8", "pair": "StepPair", "table": "StepTable", "filter": "StepFilter"}.get(
        stepper, str(stepper))
    ks = ["dgrep::scan_dfa8_kernel<dgrep::%s>" % step]
    if stepper == "filter":
        ks.append("dgrep::verify_kernel (candidate lines on the whole DFA)")
    ks.append("dgrep::scan_overflow_kernel / long-line kernels when a scan needs them")
    return ks
LEN_DTYPE = "int64"  # torch dtype of the length array dgrep_scan_device writes (uint64 in dgrep.h)

WORKLOADS = {
    # BASELINE.json configs[0] / SURVEY §8d C1: the reference's CPU-runnable case
    # (64 MiB, seed 1, 'error'); its cpu_baseline sample covers the whole split
    "c1": dict(pattern="error", seed=1, kind=0, gib=1 / 16,
               desc="C1: 64 MiB synthetic log split (seed 1), literal 'error' (the reference's CPU case)"),
    "c2": dict(pattern="error", seed=2, kind=0, gib=16.0,
               desc="C2: 16 GiB synthetic log split (seed 2), literal 'error', LDS-resident DFA"),
    "c2b": dict(pattern="timeout while waiting for lock", seed=2, kind=0, gib=16.0,
                desc="C2 (long planted literal): 16 GiB split (seed 2)"),
    "c3": dict(pattern="^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", seed=3, kind=0, gib=16.0,
               desc="C3: 16 GiB split (seed 3), anchored regex with classes/alternation"),
    "c4": dict(pattern=None, seed=4, kind=1, gib=16.0, verify_window=256 << 10,
               desc="C4: 16 GiB split (seed 4, keywords planted), (?i) alternation of 1,000 seeded keywords, "
                    "filter stepper (the DFA's shallow states in LDS, candidate lines verified on the whole DFA)"),
    # SURVEY §8d C5 / BASELINE.json configs[4]: 8 splits x 32 GiB, seeds 100-107
    "c5": dict(pattern="error", seed=100, rank_seed_step=1, kind=0, gib=32.0,
               desc="C5: one 32 GiB synthetic log split per GPU (seed 100 + rank), literal 'error'"),
    # long lines (kind 2: geometric, 4 MiB mean, each followed by a page of log
    # lines; kind 3: the same after one newline-free 1 GiB line): lanes park a
    # line that runs past the next chunk, the long-line kernels finish it
    "long": dict(pattern="error", seed=7, kind=2, gib=16.0,
                 desc="long lines: 16 GiB split (seed 7) of 4 MiB-mean lines (no line limit) between pages of log "
                      "lines, literal 'error'"),
    "long1g": dict(pattern="error", seed=8, kind=3, gib=16.0,
                   desc="long lines + one newline-free 1 GiB line: 16 GiB split (seed 8), literal 'error'"),
    # config 4's 1,000-keyword pattern over long lines (kind 4: kind 2 with the
    # keywords planted in filler pages and boundary lines): the filter stepper
    "long_c4": dict(pattern=None, seed=4, kind=4, gib=16.0, verify_window=256 << 10,
                    desc="long lines + C4 keywords: 16 GiB split (seed 4) of 4 MiB-mean lines between pages of log "
                         "lines, (?i) alternation of 1,000 seeded keywords (filter stepper)"),
    # config 4's keywords OR "an even number of k" over the same long lines: a
    # DFA (13,354 states) whose state depends on the whole line so far (the k
    # parity), so about half of a parked line's segment guesses (the state after
    # a 256-byte lookback) fail and those segments are re-run from the true state
    # (long_dfa_fix_kernel). (k[^z]*y, the other unbounded-memory example, never
    # fails a guess on this corpus: it holds no 'z' and a 'k' every ~40 bytes.)
    "long_c4p": dict(pattern=None, extra="|^([^k]*k[^k]*k)*[^k]*$", seed=4, kind=4, gib=16.0, verify_window=256 << 10,
                     desc="long lines + C4 keywords | even number of k: 16 GiB split (seed 4) of 4 MiB-mean lines, the "
                          "filter stepper on an automaton with unbounded memory (segment guesses fail)"),
    # a dense Sheng line (~60 % of lines match): the lane chunk adapts to the match density
    "dense": dict(pattern="e", seed=2, kind=0, gib=16.0,
                  desc="dense: 16 GiB split (seed 2), literal 'e' (most lines match)"),
}


def workload_pattern(wl):
    """C4's pattern is (?i)(kw_0|...|kw_999) over the corpus generator's seeded
    keyword set; the others are literal strings."""
    if wl["pattern"] is not None:
        return wl["pattern"]
    import dgrep
    return "(?i)(" + "|".join(k.decode() for k in dgrep.synth_keywords(wl["seed"], 1000)) + ")" + wl.get("extra", "")



def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU). Without WORLD_SIZE in the environment, N > 1 starts N "
                         "fresh rank processes under torch.distributed.run; under a launcher it must equal "
                         "WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: c2 on one GPU, c5 on more")
    ap.add_argument("--split-gib", type=float, default=None, help="per-GPU split size (default: workload's)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU baseline budget: whole 1 MiB pieces of the split until this much time is spent")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", choices=["full", "windows", "none"], default="full",
                    help="after the timed steps: every record of the split against the oracle over the whole split "
                         "(full; each rank its own split), or --verify-windows whole-line windows")
    ap.add_argument("--verify-seconds", type=float, default=240.0,
                    help="full verification stops (and says how far it got) after this much wall time")
    ap.add_argument("--verify-windows", type=int, default=6)
    ap.add_argument("--lane-chunk", type=int, default=0, help="tuning: force the Sheng/pair/filter lane chunk (0 = adaptive)")
    ap.add_argument("--base-offset", type=int, default=0,
                    help="ablation: place the split this many bytes (a multiple of 64) into its HBM allocation")
    ap.add_argument("--alloc-gib", type=float, default=0.0,
                    help="ablation: allocate at least this many GiB for the split's buffer")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the N-rank report (gloo, oracle instead of the GPU scan; value null)")
    ap.add_argument("--exchange", choices=["auto", "capi", "torch"], default="auto",
                    help="the N > 1 record gather inside each step: the C ABI's RCCL gather (capi, the default at "
                         "N > 1) or dgrep/dist.py over torch.distributed (torch); capi at N = 1 rehearses the "
                         "self-copy path and the gather check")
    ap.add_argument("--pattern", default=None,
                    help="ablation only: scan the workload's split with this pattern instead (not a BASELINE config)")
    return ap.parse_args()


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """`--gpus N` (N > 1) without a launcher: start N rank processes under
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) as a CHILD
    process and return its exit code. Nothing here touches the GPU: counting
    devices does not initialise HIP on this image, and the ranks are fresh
    processes (never an exec from a process that holds the GPU)."""
    import subprocess

    import torch

    have = torch.cuda.device_count()
    if have < args.gpus and not args.dry_run:
        log("bench.py --gpus %d: only %d GPU(s) visible; refusing to report an N=%d line" % (args.gpus, have, have))
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        log("bench.py --gpus %d disagrees with WORLD_SIZE=%d" % (args.gpus, world))
        sys.exit(2)
    if args.gpus is not None and args.gpus < 1:
        log("bench.py --gpus must be >= 1")
        sys.exit(2)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        # CPU rehearsal of the N-rank line (gloo): no GPU is touched
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    if args.workload is None:
        args.workload = "c2" if world == 1 else "c5"
    wl = WORKLOADS[args.workload]
    gib = args.split_gib if args.split_gib is not None else wl["gib"]
    n = int(gib * (1 << 30))
    n -= n % 64
    pattern = args.pattern if args.pattern is not None else workload_pattern(wl)
    seed = wl["seed"] + wl.get("rank_seed_step", 1000) * rank

    m = (measure_dry if args.dry_run else measure_gpu)(args, wl, world, rank, local, dev, n, pattern, seed)
    count = m["count"]

    # ---- parity on the full split: every rank checks its own ----------------
    verified = None
    if args.dry_run:
        verified = {"mode": "none (dry run: the records are the oracle's own)"}
    elif args.verify == "full":
        threads = verify_threads(world)
        verified = verify_full(m["buf"], n, m["line"][:count], m["start"][:count], m["len"][:count], pattern,
                               threads, args.verify_seconds)
        if world > 1:
            ok = torch.tensor([verified["records_checked"], int(verified["complete"])], dtype=torch.int64, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            verified["all_ranks_complete"] = bool(ok[1].item())
    elif args.verify == "windows" and rank == 0 and args.verify_windows > 0:
        verified = {"mode": "windows", "windows": verify_windows(m["buf"], n, m["line"][:count], m["start"][:count],
                                                                 m["len"][:count], pattern, args.verify_windows,
                                                                 wl.get("verify_window", 2 << 20))}

    # ---- the exchange: what rank 0 received in the last timed step ----------
    gather = None
    if world > 1 or m["comm"] is not None:
        gather = check_gather(m, world, rank, dev, seed)
        if m["comm"] is not None:
            m["comm"].close()

    # ---- CPU comparators, on rank 0 while the other ranks wait ---------------
    cpu = cpu_mt = cpu_workers = None
    if world > 1:
        dist.barrier()
    if rank == 0 and not args.no_cpu_baseline:
        if world == 1:
            cpu = cpu_baseline(m["buf"], n, pattern, args.cpu_seconds)
            cpu_mt = cpu_baseline_mt(m["buf"], n, pattern, args.cpu_seconds / 2)
        else:
            # the reference at N: coordinator + N Go workers, one file each on
            # one core (map_reduce/worker.go:126-145, coordinator.go:312,329-333):
            # N threads of the per-line-compile restatement, each on its own part
            # of the split; and the compiled-once oracle on the node's CPU share
            cpu_workers = cpu_baseline_workers(m["buf"], n, pattern, args.cpu_seconds, world)
            cpu_mt = cpu_baseline_mt(m["buf"], n, pattern, args.cpu_seconds / 2, threads=node_threads(world))
    if world > 1:
        dist.barrier()

    line = build_line(args, wl, world, rank, dev, n, pattern, seed, m, verified, cpu, cpu_mt, cpu_workers, gather)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure_gpu(args, wl, world, rank, local, dev, n, pattern, seed):
    """Generate the rank's split in HBM, then W untimed and K timed steps of
    dgrep_scan_device (+ the record gather at N > 1), bracketed by a barrier and
    a device synchronisation."""
    import torch
    import torch.distributed as dist

    import dgrep

    ctx = dgrep.Context(local)
    if args.lane_chunk:
        ctx.set_lane_chunk(args.lane_chunk)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    cp = ctx.load(pattern)

    t = time.time()
    off = args.base_offset - args.base_offset % 64
    alloc = torch.empty(max(n + 64 + off, int(args.alloc_gib * (1 << 30))), dtype=torch.uint8, device=dev)
    buf = alloc[off:]
    ctx.synth(buf.data_ptr(), n, seed, wl["kind"])
    torch.cuda.synchronize(dev)
    log("rank %d: generated %.1f GiB split in %.1fs; DFA %d states x %d classes" %
        (rank, n / 2**30, time.time() - t, cp.nstates, cp.nclasses))

    # size the result arrays from a first scan (capacity-retry protocol of the ABI)
    cap = max(1 << 16, n // 4096)
    res = None
    for _ in range(3):
        res = (torch.empty(cap, dtype=torch.int64, device=dev), torch.empty(cap, dtype=torch.int64, device=dev),
               torch.empty(cap, dtype=getattr(torch, LEN_DTYPE), device=dev))
        cnt = ctx.scan_device(buf.data_ptr(), n, res[0].data_ptr(), res[1].data_ptr(), res[2].data_ptr(), cap)
        if cnt <= cap:
            break
        cap = int(cnt * 1.05) + 1024
    line_t, start_t, len_t = res

    # N > 1: the path's only exchange -- compacted records -> rank 0 over
    # RCCL/xGMI -- through the C ABI a Go worker binds (dgrep_gather_records_device,
    # csrc/runtime/exchange.hip), on the scan's stream; checked after the timed
    # steps against the torch path (check_gather)
    from dgrep.dist import gather_records

    use_capi = args.exchange == "capi" or (args.exchange == "auto" and world > 1)
    comm = open_comm(ctx, world, rank, dev) if use_capi else None
    last = {}

    def step():
        c = ctx.scan_device(buf.data_ptr(), n, line_t.data_ptr(), start_t.data_ptr(), len_t.data_ptr(), cap)
        if comm is not None:
            last["gather"] = comm.gather_device(line_t.data_ptr(), start_t.data_ptr(), len_t.data_ptr(), c,
                                                split=seed, root=0)
        elif world > 1:
            gather_records(line_t, start_t, len_t, c, dst=0, split=seed)
        return c

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.take_kernel_ms()  # reset: the timed steps' device time is read once, after them
    t0 = time.perf_counter()
    count = 0
    for _ in range(args.steps):
        count = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # scan kernel + overflow pass + verification, HIP events on the launch
    # stream, summed by the library over the timed steps (no host call between
    # two steps but the scan itself)
    kms_sum, kms_n = ctx.take_kernel_ms()
    assert kms_n == args.steps, (kms_n, args.steps)
    kms = [kms_sum / kms_n] * kms_n
    stats = [ctx.scan_stats()]
    return dict(buf=buf, line=line_t, start=start_t, len=len_t, count=count, kms=kms, stats=stats, elapsed=elapsed,
                nstates=cp.nstates, nclasses=cp.nclasses, build=dgrep.build_info(), comm=comm,
                gather=last.get("gather"), exchange="capi" if comm is not None else ("torch" if world > 1 else None))


def open_comm(ctx, world, rank, dev):
    """The C ABI's RCCL communicator (dgrep_comm_open) on the scan context's
    device and stream: rank 0 makes the 128-byte id, torch.distributed hands it
    to the others (a Go worker would use its own channel)."""
    import torch
    import torch.distributed as dist

    import dgrep

    if world == 1:  # --exchange capi at N = 1: the self-copy path (a rehearsal of the line's fields)
        return dgrep.Comm(ctx, dgrep.Comm.unique_id(), 1, 0)
    uid = torch.zeros(dgrep.COMM_ID_BYTES, dtype=torch.uint8, device=dev)
    if rank == 0:
        uid.copy_(torch.frombuffer(bytearray(dgrep.Comm.unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, 0)
    return dgrep.Comm(ctx, bytes(uid.cpu().numpy().tobytes()), world, rank)


def record_checksum(line_t, start_t, len_t, count, split, dev):
    """(count, split, sums of line / start / len, and a position-weighted sum
    of all three) as int64 (sums wrap alike on every rank)."""
    import torch

    ln, st, le = (x[:count].to(torch.int64) for x in (line_t, start_t, len_t))
    w = torch.arange(1, count + 1, dtype=torch.int64, device=ln.device)
    v = [count, split, int(ln.sum()), int(st.sum()), int(le.sum()), int(((ln * 3 + st * 5 + le * 7) * w).sum())]
    return torch.tensor(v, dtype=torch.int64, device=dev)


def copy_device_records(ptr, total, dev):
    """The comm-owned packed records (device pointer from
    dgrep_gather_records_device) into a torch int32 tensor (hipMemcpy D2D)."""
    import ctypes

    import torch

    from dgrep.dist import REC_WORDS

    out = torch.empty(total * REC_WORDS, dtype=torch.int32, device=dev)
    if total:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        rc = hip.hipMemcpy(out.data_ptr(), ptr, out.numel() * 4, 3)  # hipMemcpyDeviceToDevice
        if rc != 0:
            raise RuntimeError("hipMemcpy of the gathered records failed: %d" % rc)
    return out


def check_gather(m, world, rank, dev, seed):
    """After the timed steps: the records rank 0 received in the LAST timed
    step must be every rank's own records, in rank order, with its split id.
    Checked two ways: per-rank checksums all-gathered from the ranks
    themselves, and (C ABI exchange) record-by-record against the torch path
    (dgrep/dist.py gather_records) run once more over the same arrays."""
    import torch
    import torch.distributed as dist

    from dgrep.dist import gather_records, unpack_records

    count = m["count"]
    mine = record_checksum(m["line"], m["start"], m["len"], count, seed, dev)
    if world > 1:
        allc = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        ref = gather_records(m["line"], m["start"], m["len"], count, dst=0, split=seed)
    else:
        allc = [mine]
        ref = [tuple(x[:count].to(torch.int64) for x in (m["line"], m["start"], m["len"])) +
               (torch.full((count,), seed & 0xFFFFFFFF, dtype=torch.int64, device=dev),)]
    if rank != 0:
        return None
    want = [c.cpu().tolist() for c in allc]
    ok = True
    for r, (ln, st, le, sp) in enumerate(ref):
        got = record_checksum(ln, st, le, ln.numel(), want[r][1], dev).cpu().tolist()
        ok = ok and got == want[r] and bool((sp == want[r][1]).all())
    out = {"exchange": m["exchange"] or "torch", "records": sum(w[0] for w in want),
           "per_rank_counts": [w[0] for w in want], "checksums_match": bool(ok)}
    if m["exchange"] == "capi":
        ptr, total, counts = m["gather"]
        same = total == out["records"] and counts == out["per_rank_counts"]
        if same:
            packed = copy_device_records(ptr, total, dev)
            off = 0
            for r, (ln, st, le, sp) in enumerate(ref):
                c = ln.numel()
                g = unpack_records(packed[off * 7:(off + c) * 7], c)
                same = same and all(torch.equal(a, b) for a, b in zip(g, (ln, st, le, sp)))
                off += c
        out["capi_equals_torch_path"] = bool(same)
        ok = ok and same
    out["gather_verified"] = bool(ok)
    log("gather check: %s" % json.dumps(out))
    return out


def measure_dry(args, wl, world, rank, local, dev, n, pattern, seed):
    """--dry-run: the same line on the CPU (gloo), for rehearsing the N-rank
    report without a GPU. The split comes from the generator's host twin and
    the "scan" is the oracle's Map (kernel times = its wall time): the numbers
    are NOT a measurement of this framework and the line says so."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import dgrep

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    from dgrep.dist import gather_records

    buf = torch.frombuffer(bytearray(dgrep.synth_corpus_host(n, seed, wl["kind"]) + bytes(64)), dtype=torch.uint8)
    host = buf[:n].numpy()
    kms, stats, count, res = [], [], 0, None
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t = time.perf_counter()
        ln, st, le = O.grep_map(pattern.encode(), host, threads=2)
        kms.append((time.perf_counter() - t) * 1e3)
        count = len(ln)
        res = (torch.from_numpy(ln.astype(np.int64)), torch.from_numpy(st.astype(np.int64)),
               torch.from_numpy(le.astype(np.int64)))
        if world > 1:
            # the CPU rehearsal exchanges over gloo with the torch path
            gather_records(res[0], res[1], res[2], count, dst=0, split=seed)
        stats.append(dict(stepper="oracle (dry run)", lane_chunk=0, overflow_ms=0.0, verify_ms=0.0,
                          scan_ms=kms[-1], candidates=0, overflow_lanes=0, pending=0))
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return dict(buf=buf, line=res[0], start=res[1], len=res[2], count=count, kms=kms, stats=stats, elapsed=elapsed,
                nstates=0, nclasses=0, build=dgrep.build_info(), comm=None, gather=None,
                exchange="torch (gloo, dry run)")


def build_line(args, wl, world, rank, dev, n, pattern, seed, m, verified, cpu, cpu_mt, cpu_workers, gather=None):
    """The JSON line (rank 0 prints it). Every rank takes part in the
    reductions: wall time = max over ranks; the roofline comes from the SLOWEST
    rank's kernel time (max over ranks of its mean), per GPU and for the node."""
    import numpy as np
    import torch
    import torch.distributed as dist

    count, kms, stats = m["count"], m["kms"], m["stats"]
    # algorithmic bytes of the timed kernels: the split read once, plus per
    # matching line the 16-byte staged record the ordering passes (not timed)
    # read back
    alg = n + STAGED_LINE_BYTES * count
    kern_ms, kern_med = float(np.mean(kms)), float(np.median(kms))
    mine = torch.tensor([m["elapsed"], kern_ms, kern_med, float(alg), float(count)], dtype=torch.float64, device=dev)
    if world > 1:
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per = torch.stack(allr).cpu().numpy()
    else:
        per = mine.cpu().numpy()[None, :]
    elapsed = float(per[:, 0].max())
    ms_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed / 1e9
    slow = int(per[:, 1].argmax())
    kern_max = float(per[slow, 1])
    achieved = float(per[slow, 3]) / (kern_max * 1e-3) / 1e9       # the slowest rank's own bytes / its time
    agg = float(per[:, 3].sum()) / (kern_max * 1e-3) / 1e9          # all ranks' bytes / the slowest time
    st = stats[-1]

    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath) and not args.dry_run:
        try:
            with open(tpath) as f:
                tr = json.load(f).get(args.workload)
            if tr and abs(tr.get("split_bytes", 0) - n) < 1024:
                traffic = tr.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if rank != 0:
        return None
    counts = [int(c) for c in per[:, 4]]
    out = {
        "metric": "GB/s text scanned per GPU and whole node (1/2/4/8×MI355X), % of HBM peak",
        "value": round(value, 2) if not args.dry_run else None,
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded log corpus generated in HBM, SURVEY.md §8d)",
        "config": {
            "workload": (wl["desc"] if world == 1 else wl["desc"] + "; one split per GPU + RCCL gather of match records to rank 0")
                        + ("" if args.pattern is None else "; ABLATION: pattern overridden"),
            "pattern": pattern if len(pattern) < 200 else pattern[:120] + "...(%d bytes)" % len(pattern),
            "split_bytes_per_gpu": n,
            "total_bytes": n * world,
            "matching_lines_per_split": counts[0] if world == 1 else counts,
            "dfa_states": m["nstates"],
            "dfa_byte_classes": m["nclasses"],
            "parallelism": "1 split per GPU x %d" % world,
            "per_gpu_gbs": round(value / world, 2),
            "hbm_frac_whole_node": round(value / (HBM_PEAK_GBS * world), 4),
            "verified": verified,
            "seed": seed,
            "stepper": st["stepper"],
            "lane_chunk": st["lane_chunk"],
            "build": m["build"].split()[0][len("head="):],
            "build_info": m["build"],
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kernels_timed(st["stepper"])[0],
            "kernels_timed": kernels_timed(st["stepper"]),
            "record_bytes": STAGED_LINE_BYTES,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel_ms_avg": round(kern_max, 4),
            "per_rank_kernel_ms_avg": [round(float(x), 4) for x in per[:, 1]],
            "slowest_rank": slow,
            "aggregate": {"achieved": round(agg, 2), "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                          "frac": round(agg / (HBM_PEAK_GBS * world), 4),
                          "note": "all ranks' algorithmic bytes / the slowest rank's mean kernel time"},
            # the last timed step's split of the kernel time (dgrep_last_scan_stats)
            "overflow_ms_last": round(float(st["overflow_ms"]), 4),
            "verify_ms_last": round(float(st["verify_ms"]), 4),
            "scan_ms_last": round(float(st["scan_ms"]), 4),
            "candidates_dropped": int(st["candidates"]),
            "overflow_lanes": int(st["overflow_lanes"]),
            "pending_lines": int(st["pending"]),
            "timing": "HIP events on the launch stream around the scan kernel, the overflow pass and the "
                      "verification / long-line resolution (dgrep_take_kernel_ms: summed by the library over the timed steps, read once after them), averaged; "
                      "at N > 1 the slowest rank's average (kernel_ms_avg) prices `achieved`",
            "algorithmic_bytes_per_launch": int(per[slow, 3]),
        },
        "cpu_baseline": cpu,
        "cpu_baseline_mt": cpu_mt,
    }
    if world > 1:
        out["cpu_baseline_workers"] = cpu_workers
    if gather is not None:
        out["exchange"] = gather["exchange"] if gather else m["exchange"]
        out["gather_verified"] = bool(gather and gather["gather_verified"])
        out["gather"] = gather
    if args.dry_run:
        out["dry_run"] = ("CPU rehearsal (gloo): the split is scanned by the oracle, not by the GPU; "
                          "value is null and no number here measures this framework")
    return out


def last_newline(host):
    """Index of the last '\n' in a host uint8 array (-1: none), searching the
    tail first."""
    import numpy as np

    span = 1 << 20
    end = len(host)
    while end > 0:
        lo = max(0, end - span)
        nl = np.flatnonzero(host[lo:end] == 10)
        if nl.size:
            return lo + int(nl[-1])
        end = lo
        span *= 4
    return -1


def verify_threads(world):
    """Host threads for the oracle: the process's CPU share split over the ranks
    of this node, 16 at most (the GPU box grants 16 CPUs per GPU)."""
    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(16, cpus // max(1, world)))


def verify_full(buf, n, line_t, start_t, len_t, pattern, threads, seconds, piece=1 << 30):
    """Parity at full size: the oracle's Map (orc_map_mt, the memoized Pike VM
    restatement of grep.go:17-29) over the WHOLE split, in ~1 GiB pieces cut
    after a '\n', must equal every GPU record -- line number (offset by the
    '\n' count before the piece), start and length. Also the structural check
    of every record (check_records). Stops after `seconds` of wall time and
    reports how far it got (`complete` false)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    t0 = time.time()
    check_records(buf, n, line_t, start_t, len_t)
    gl = line_t.cpu().numpy().astype(np.uint64)
    gs = start_t.cpu().numpy().astype(np.uint64)
    ge = len_t.cpu().numpy().astype(np.uint64)
    a, lines_before, checked, pieces = 0, 0, 0, 0
    while a < n:
        if time.time() - t0 > seconds:
            break
        host = buf[a:min(n, a + piece)].cpu().numpy()
        last = a + len(host) >= n
        if not last:
            cut = last_newline(host)
            if cut < 0:  # no '\n' in the whole piece (a line over 1 GiB): take the rest of the split
                host = buf[a:n].cpu().numpy()
                last = True
            else:
                host = host[:cut + 1]
        b = a + len(host)
        ln, st, le = O.grep_map(pattern.encode(), memoryview(host), threads=threads)
        if not last and len(st) and int(st[-1]) == len(host):
            ln, st, le = ln[:-1], st[:-1], le[:-1]  # the empty piece after the cut's '\n' is not a line
        i, j = np.searchsorted(gs, a), np.searchsorted(gs, b if not last else n + 1)
        np.testing.assert_array_equal(gl[i:j], ln.astype(np.uint64) + np.uint64(lines_before),
                                      err_msg="line numbers in piece at %d" % a)
        np.testing.assert_array_equal(gs[i:j], st.astype(np.uint64) + np.uint64(a), err_msg="starts at %d" % a)
        np.testing.assert_array_equal(ge[i:j], le.astype(np.uint64), err_msg="lengths at %d" % a)
        lines_before += int(np.count_nonzero(host == 10))
        checked += j - i
        pieces += 1
        a = b
    complete = a >= n and checked == len(gs)
    log("full-split parity: %s records equal the oracle over %.2f GiB (%d pieces, %d threads, %.1f s)%s" % (
        checked, a / 2**30, pieces, threads, time.time() - t0, "" if complete else " -- INCOMPLETE (time budget)"))
    if complete:
        log("all %d records equal the oracle" % checked)
    return {"mode": "full", "complete": bool(complete), "records_checked": int(checked), "bytes_checked": int(a),
            "oracle_threads": threads, "seconds": round(time.time() - t0, 1)}


def verify_windows(buf, n, line_t, start_t, len_t, pattern, k, win):
    """Parity at full size: k whole-line windows, evenly spaced so that the
    first and the last always sit at the split's start and end, re-run on the
    oracle (lines renumbered by the '\\n' count before the window, counted on the
    GPU) must equal the GPU records inside the window. Every record (not only
    those in windows) must be a whole line -- preceded by '\\n' or the split
    start, followed by '\\n' or the split end -- whose line number is 1 + the
    number of '\\n' before it (searchsorted over the GPU's newline positions),
    and records must be strictly ascending."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    if line_t.numel() > 1:
        assert bool((line_t[1:] > line_t[:-1]).all()), "line numbers not strictly ascending"
    check_records(buf, n, line_t, start_t, len_t)
    ok = 0
    span = max(0, n - win)
    for w in range(k):
        a0 = (span * w) // max(1, k - 1) if k > 1 else 0
        chunk = buf[a0:min(n, a0 + win)].cpu().numpy().tobytes()
        i = chunk.find(b"\n")
        j = chunk.rfind(b"\n")
        if i < 0 or j <= i:
            continue
        a, b = a0 + i + 1, a0 + j  # whole lines [a, b), b = a '\n'
        text = chunk[i + 1:j]
        # 1 GiB pieces: a whole-prefix compare + sum needs ~9 bytes of HBM per
        # split byte (a 32 GiB C5 split asked for 205 GiB)
        step = 1 << 30
        nl_before = sum(int((buf[o:min(a, o + step)] == 10).sum().item()) for o in range(0, a, step))
        oln, ost, ole = O.grep_map(pattern.encode(), text, threads=min(16, os.cpu_count() or 1))
        sel = (start_t >= a) & (start_t < b)
        gl = line_t[sel].cpu().numpy().astype(np.int64)
        gs = start_t[sel].cpu().numpy().astype(np.int64)
        ge = len_t[sel].cpu().numpy().astype(np.int64)
        np.testing.assert_array_equal(gl, oln.astype(np.int64) + nl_before)
        np.testing.assert_array_equal(gs, ost.astype(np.int64) + a)
        np.testing.assert_array_equal(ge, ole.astype(np.int64))
        ok += 1
        log("verified window %d/%d at byte %d (%d matching lines)" % (ok, k, a, len(oln)))
    return ok


def check_records(buf, n, line_t, start_t, len_t):
    """Structural check of every GPU record on the GPU (see verify_windows)."""
    import torch

    if line_t.numel() == 0:
        return
    st = start_t.to(torch.int64)
    en = st + len_t.to(torch.int64)
    assert bool((st >= 0).all()) and bool((en <= n).all()), "record outside the split"
    step = 1 << 30  # torch.nonzero mis-sizes its output past 2**31 elements: 1 GiB pieces
    nlpos = torch.cat([torch.nonzero(buf[o:min(n, o + step)] == 10).flatten() + o for o in range(0, n, step)])
    prev_ok = (st == 0) | (buf[(st - 1).clamp(min=0)] == 10)
    end_ok = (en == n) | (buf[en.clamp(max=n - 1)] == 10)
    assert bool(prev_ok.all()), "a record does not start at a line start"
    assert bool(end_ok.all()), "a record does not end at a line end"
    nl_in = torch.searchsorted(nlpos, en) - torch.searchsorted(nlpos, st)
    assert bool((nl_in == 0).all()), "a record spans a newline"
    want = torch.searchsorted(nlpos, st) + 1
    assert bool((line_t.to(torch.int64) == want).all()), "line numbers disagree with the newline count"
    del nlpos
    log("checked %d records: whole lines, numbering consistent" % line_t.numel())


def cpu_baseline(buf, n, pattern, seconds):
    """The oracle's restatement of grep.go Map on one host core: per line,
    regexp.Match(pattern, line) recompiles the pattern (grep.go:21) — the
    reference's own algorithm, not a tuned CPU grep. Bounded: successive
    whole-line pieces from the start of the split (64 KiB, doubling up to
    1 MiB) until `seconds` of CPU time are spent."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    piece, done, matches, dt = 64 << 10, 0, 0, 0.0
    while dt < seconds and done < n:
        data = buf[done:min(n, done + piece)].cpu().numpy().tobytes()
        j = data.rfind(b"\n")
        data = data[: j + 1] if j >= 0 else data
        t = time.perf_counter()
        ln, _, _ = O.grep_map(pattern.encode(), data, recompile_per_line=True)
        dt += time.perf_counter() - t
        done += len(data)
        matches += len(ln)
        piece = min(piece * 2, 1 << 20)
    return {
        "value": round(done / dt / 1e9, 6),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": "first %.2f MiB of the same split (%d matching lines), oracle/ grep.go Map restatement with "
                  "per-line pattern compile (as grep.go:21), 1 thread, %.1f s" % (done / 2**20, matches, dt),
    }


def node_threads(world):
    """Host threads for a node-wide CPU comparator: the process's CPU share,
    at most 16 per GPU of the job (the GPU box grants 16 CPUs per GPU)."""
    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(16 * max(1, world), cpus))


def cpu_baseline_workers(buf, n, pattern, seconds, workers):
    """The reference at N GPUs' worth of work: its coordinator hands one file to
    each of N workers, and each worker's Map runs on ONE core
    (map_reduce/worker.go:126-145; coordinator.go:312,329-333), re-compiling the
    pattern per line (grep.go:21). Restated with the oracle: N threads, each
    scanning its own part of the split (successive whole-line pieces from
    offset i*n/N) with per-line compile, until `seconds` of wall time; value =
    all threads' bytes / wall time (ctypes releases the GIL in the oracle)."""
    import threading

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    done = [0] * workers
    matches = [0] * workers
    t0 = time.perf_counter()

    def work(i):
        pos = (n * i // workers)
        end = n * (i + 1) // workers
        host = buf[pos:min(end, pos + (64 << 20))].cpu().numpy().tobytes()  # this worker's part (<= 64 MiB)
        a = host.find(b"\n") + 1 if i else 0  # start at a line start
        piece = 64 << 10
        while time.perf_counter() - t0 < seconds and a < len(host):
            data = host[a:a + piece]
            j = data.rfind(b"\n")
            data = data[: j + 1] if j >= 0 else data
            ln, _, _ = O.grep_map(pattern.encode(), data, recompile_per_line=True)
            done[i] += len(data)
            matches[i] += len(ln)
            a += len(data)
            piece = min(piece * 2, 1 << 20)

    th = [threading.Thread(target=work, args=(i,)) for i in range(workers)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    return {
        "value": round(sum(done) / dt / 1e9, 6),
        "unit": "GB/s",
        "cores": workers,
        "workers": workers,
        "kind": "port",
        "sample": "%d worker threads (the reference's N workers, one file each on one core), each on its own part of "
                  "rank 0's split: %.2f MiB in all (%d matching lines), oracle/ grep.go Map restatement with "
                  "per-line pattern compile (as grep.go:21), %.1f s wall" % (workers, sum(done) / 2**20,
                                                                            sum(matches), dt),
    }


def cpu_baseline_mt(buf, n, pattern, seconds, threads=None):
    """SURVEY.md §8d comparator (3): the oracle's Map with the pattern compiled
    once per call, lines split over T host threads (default T = the box's CPU
    share, at most 16; at N > 1 the node's share, node_threads). Bounded like
    cpu_baseline: doubling whole-line pieces from the split's start (256 KiB up
    to 64 MiB, sized to the time left) until `seconds` of wall time are spent."""
    import ctypes

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    T = threads or max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)))
    L = O.lib()
    pat = pattern.encode()
    piece, done, matches, dt = 256 << 10, 0, 0, 0.0
    while dt < seconds and done < n:
        data = buf[done:min(n, done + piece)].cpu().numpy()
        nl = np.flatnonzero(data == 10)
        data = data[: int(nl[-1]) + 1] if nl.size else data
        cap = int(nl.size) + 1
        ln = np.zeros(cap, np.uint64)
        st = np.zeros(cap, np.uint64)
        le = np.zeros(cap, np.uint64)
        t = time.perf_counter()
        cnt = L.orc_map_mt(pat, len(pat), data.ctypes.data, len(data), T, ln.ctypes.data, st.ctypes.data,
                           le.ctypes.data, cap)
        dt += time.perf_counter() - t
        if cnt < 0 or cnt > cap:
            return None
        done += len(data)
        matches += int(cnt)
        # next piece: double, but no more than the remaining time allows
        piece = int(max(64 << 10, min(piece * 2, 64 << 20, done / dt * (seconds - dt))))
    return {
        "value": round(done / dt / 1e9, 6),
        "unit": "GB/s",
        "cores": T,
        "kind": "port",
        "sample": "first %.2f MiB of the same split (%d matching lines), oracle/ Map restatement with the pattern "
                  "compiled once per call, lines split over %d threads, %.1f s" % (done / 2**20, matches, T, dt),
    }


if __name__ == "__main__":
    main()
