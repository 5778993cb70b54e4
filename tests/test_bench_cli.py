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
