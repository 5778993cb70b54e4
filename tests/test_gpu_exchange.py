"""The C ABI's multi-GPU exchange (include/dgrep.h dgrep_comm_* /
dgrep_gather_records*, csrc/runtime/exchange.hip): the RCCL gather a Go worker
can call through cgo, replacing the SFTP shipping of map output
(map_reduce/coordinator.go:136-142) for workers on one node.

On the one-GPU box: world 1 through the C ABI (records, split ids, counts equal
the scan's), the same records as the torch path (dgrep/dist.py) packs, and --
if RCCL accepts two ranks on one device -- world 2 from two processes, each
scanning its own split, the root receiving both in rank order. The 8-rank case
runs only on an 8-GPU node."""
import multiprocessing as mp
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scan(ctx, n, seed, pattern="error"):
    import torch

    buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.load(pattern)
    ctx.synth(buf.data_ptr(), n, seed, 0)
    cap = max(1 << 12, n // 1024)
    out = [torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(3)]
    cnt = ctx.scan_device(buf.data_ptr(), n, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), cap)
    assert 0 < cnt <= cap
    return buf, out, cnt


def test_capi_gather_world1(gpu_ctx):
    import torch

    import dgrep

    n = 64 << 20
    buf, (ln, st, le), cnt = _scan(gpu_ctx, n, 5)
    comm = dgrep.Comm(gpu_ctx, dgrep.Comm.unique_id(), 1, 0)
    try:
        got = comm.gather(ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, split=0xDEADBEEF, root=0)
        assert got is not None
        gl, gs, ge, gp = got
        np.testing.assert_array_equal(gl, ln[:cnt].cpu().numpy().astype(np.uint64))
        np.testing.assert_array_equal(gs, st[:cnt].cpu().numpy().astype(np.uint64))
        np.testing.assert_array_equal(ge, le[:cnt].cpu().numpy().astype(np.uint64))
        assert (gp == 0xDEADBEEF).all()
        # device variant: root gets the comm-owned packed buffer and the counts
        ptr, total, counts = comm.gather_device(ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, split=7, root=0)
        assert total == cnt and counts == [cnt] and ptr
        # an empty rank
        assert comm.gather(ln.data_ptr(), st.data_ptr(), le.data_ptr(), 0, split=1, root=0)[0].size == 0
    finally:
        comm.close()
    del buf
    torch.cuda.empty_cache()


def _rank2(rank, uid_q, res_q, n):
    try:
        import torch

        import dgrep

        ctx = dgrep.Context(0)
        if rank == 0:
            uid = dgrep.Comm.unique_id()
            uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        try:
            comm = dgrep.Comm(ctx, uid, 2, rank)
        except dgrep.DgrepError as e:
            res_q.put(("init_failed", rank, str(e)))
            return
        buf, (ln, st, le), cnt = _scan(ctx, n, 40 + rank)
        mine = (ln[:cnt].cpu().numpy(), st[:cnt].cpu().numpy(), le[:cnt].cpu().numpy())
        got = comm.gather(ln.data_ptr(), st.data_ptr(), le.data_ptr(), cnt, split=100 + rank, root=0)
        res_q.put(("ok", rank, mine, got))
        comm.close()
        ctx.close()
    except Exception as e:  # reported to the parent
        res_q.put(("error", rank, repr(e)))


def test_capi_gather_two_ranks_one_gpu():
    import torch

    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    uid_q, res_q = ctx.Queue(), ctx.Queue()
    n = 48 << 20
    ps = [ctx.Process(target=_rank2, args=(r, uid_q, res_q, n)) for r in (0, 1)]
    for p in ps:
        p.start()
    import queue

    out = []
    try:
        for _ in range(2):
            try:
                out.append(res_q.get(timeout=150))
            except queue.Empty:
                break  # a rank is stuck (e.g. its peer's init failed): killed below
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    fails = [o for o in out if o[0] == "init_failed"]
    if fails:
        pytest.skip("RCCL refuses two ranks on one GPU here: %s" % fails[0][2][:200])
    errs = [o for o in out if o[0] == "error"]
    assert not errs, errs
    assert len(out) == 2, out
    by = {o[1]: o for o in out}
    got = by[0][3]
    want = [by[r][2] for r in (0, 1)]
    gl, gs, ge, gp = got
    c0 = len(want[0][0])
    for r, (a, b) in enumerate(((0, c0), (c0, len(gl)))):
        np.testing.assert_array_equal(gl[a:b], want[r][0].astype(np.uint64))
        np.testing.assert_array_equal(gs[a:b], want[r][1].astype(np.uint64))
        np.testing.assert_array_equal(ge[a:b], want[r][2].astype(np.uint64))
        assert (gp[a:b] == 100 + r).all()
    assert by[1][3] is None
