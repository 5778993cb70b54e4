"""bench.py's full-split parity check (verify_full) on CPU tensors: pieces cut
after a '\\n' must reproduce the oracle's whole-split records exactly, line
numbers carried across pieces; a piece with no '\\n' (a line longer than the
piece) extends to the split's end; a single wrong record is caught."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import dgrep  # noqa: E402
import oracle_lib as O  # noqa: E402


def _split():
    data = bytearray(dgrep.synth_corpus_host(3 << 20, 5, 0))
    data += b"x" * (2 << 20) + b" an error in a long line"  # no '\n': longer than a piece
    data += b"\nlast error"
    return bytes(data)


@pytest.mark.parametrize("pattern", ["error", "^[0-9]{4}-[0-9]{2}.*(WARN|ERROR) [a-z_]+", ""])
def test_verify_full_matches_and_catches(pattern):
    data = _split()
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ln, st, le = O.grep_map(pattern.encode(), data, threads=2)
    t = [torch.from_numpy(x.astype(np.int64)) for x in (ln, st, le)]
    v = bench.verify_full(buf, len(data), t[0], t[1], t[2], pattern, 2, 60.0, piece=1 << 20)
    assert v["complete"] and v["records_checked"] == len(ln)
    bad = t[2].clone()
    bad[len(bad) // 2] += 1
    with pytest.raises(AssertionError):
        bench.verify_full(buf, len(data), t[0], t[1], bad, pattern, 2, 60.0, piece=1 << 20)
