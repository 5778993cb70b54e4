"""BASELINE.json configs[4] / SURVEY §8d C5 on one GPU: a 32 GiB synthetic
split (seed 100, literal `error`) scanned in HBM, EVERY record checked against
the oracle over the whole split (bench.verify_full: the memoized Pike VM
restatement of grep.go:17-29 in 1 GiB pieces), and the records gathered to
rank 0 over the `nccl` backend (RCCL) at world size 1 -- the exchange step of
bench.py --gpus N (dgrep/dist.py) on the real backend. The N > 1 exchange is
covered by tests/test_dist.py (gloo, world 2/4) and by the driver's 8-GPU run."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_c5_split_full_parity_and_nccl_gather(gpu_ctx):
    import torch
    import torch.distributed as dist

    import bench
    from dgrep.dist import gather_records

    n = 32 << 30
    dev = torch.device("cuda", 0)
    buf = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    gpu_ctx.load("error")
    gpu_ctx.synth(buf.data_ptr(), n, 100, 0)
    cap = n // 2048
    line_t = torch.empty(cap, dtype=torch.int64, device=dev)
    start_t = torch.empty(cap, dtype=torch.int64, device=dev)
    len_t = torch.empty(cap, dtype=getattr(torch, bench.LEN_DTYPE), device=dev)
    cnt = gpu_ctx.scan_device(buf.data_ptr(), n, line_t.data_ptr(), start_t.data_ptr(), len_t.data_ptr(), cap)
    assert 0 < cnt <= cap
    v = bench.verify_full(buf, n, line_t[:cnt], start_t[:cnt], len_t[:cnt], "error", bench.verify_threads(1), 90.0)
    assert v["complete"] and v["records_checked"] == cnt, v

    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1,
                                device_id=dev)
    try:
        out = gather_records(line_t, start_t, len_t, cnt, dst=0, split=100)
        assert len(out) == 1
        ln, st, le, sp = out[0]
        assert ln.numel() == cnt
        assert torch.equal(ln, line_t[:cnt]) and torch.equal(st, start_t[:cnt])
        assert torch.equal(le, len_t[:cnt].to(torch.int64))
        assert bool((sp == 100).all())
    finally:
        dist.destroy_process_group()
    del buf
    torch.cuda.empty_cache()
    assert np.isfinite(v["seconds"])
