"""bench.py's rank launch contract on a machine without GPUs: `--gpus N`
(N > 1) without a launcher must start N rank processes or fail fast -- never
print an N=1 line -- and `--gpus` must agree with WORLD_SIZE under a launcher."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus_without_devices_fails_fast():
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible: the launch path would really start ranks")
    p = _run(["--gpus", "2", "--steps", "2"])
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert p.stdout.strip() == "", "no JSON line may be printed"
    assert "GPU(s) visible" in p.stderr


def test_gpus_disagrees_with_world_size():
    p = _run(["--gpus", "4", "--steps", "2"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert p.stdout.strip() == ""
    assert "disagrees with WORLD_SIZE" in p.stderr


def test_dry_run_world2_line():
    """`bench.py --gpus 2 --dry-run` (CPU, gloo, the oracle standing in for the
    scan): the N > 1 line carries the node-wide CPU comparators and prices the
    roofline with the SLOWEST rank's kernel time, per GPU and for the node."""
    import json

    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--split-gib",
                        "0.01", "--steps", "2", "--warmup", "0", "--cpu-seconds", "1"],
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")},
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] is None and "dry_run" in d
    r = d["roofline"]
    per = r["per_rank_kernel_ms_avg"]
    assert len(per) == 2 and r["kernel_ms_avg"] == max(per) and r["slowest_rank"] == per.index(max(per))
    assert r["aggregate"]["peak"] == 2 * r["peak"] and r["aggregate"]["achieved"] >= r["achieved"]
    assert d["cpu_baseline_mt"] and d["cpu_baseline_mt"]["cores"] >= 1 and d["cpu_baseline_mt"]["value"] > 0
    w = d["cpu_baseline_workers"]
    assert w and w["cores"] == 2 and w["workers"] == 2 and w["value"] > 0
    assert len(d["config"]["matching_lines_per_split"]) == 2
    # the exchange: rank 0's gathered records checked against every rank's own
    assert d["exchange"].startswith("torch") and d["gather_verified"] is True
    g = d["gather"]
    assert g["per_rank_counts"] == d["config"]["matching_lines_per_split"] and g["checksums_match"]
