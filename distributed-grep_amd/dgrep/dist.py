"""Multi-GPU exchange for the Map hot path: one split per GPU, match records
gathered to the reducing rank.

In the reference, each map task (one input file, map_reduce/coordinator.go:312,
329-333) is scanned independently and its output travels to the reducers by
SFTP (map_reduce/coordinator.go:136-142). Here one process per GPU scans its
split in HBM and the compacted records — (line_no, start, len) per matching
line, never the line bytes — are gathered to rank `dst` with torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests). RCCL has no
gatherv: counts are all-gathered first, records are padded to the largest
count and gathered in one collective.
"""
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def pack_records(line_no: torch.Tensor, start: torch.Tensor, length: torch.Tensor, count: int,
                 width: int) -> torch.Tensor:
    """[3, width] int64: rows line_no / start / len, zero-padded past `count`."""
    rec = torch.zeros((3, max(width, 1)), dtype=torch.int64, device=line_no.device)
    if count:
        rec[0, :count] = line_no[:count].to(torch.int64)
        rec[1, :count] = start[:count].to(torch.int64)
        rec[2, :count] = length[:count].to(torch.int64)
    return rec


def gather_records(line_no: torch.Tensor, start: torch.Tensor, length: torch.Tensor, count: int,
                   dst: int = 0, group=None) -> Optional[List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]]:
    """Gather every rank's match records to `dst`. Returns, on `dst`, one
    (line_no, start, len) triple per rank in rank order (each trimmed to that
    rank's count); None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = line_no.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    width = max(counts)
    rec = pack_records(line_no, start, length, count, width)
    if rank == dst:
        bufs = [torch.empty_like(rec) for _ in range(world)]
        dist.gather(rec, gather_list=bufs, dst=dst, group=group)
        return [(b[0, :c], b[1, :c], b[2, :c]) for b, c in zip(bufs, counts)]
    dist.gather(rec, dst=dst, group=group)
    return None
