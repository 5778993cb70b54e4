"""Multi-GPU exchange for the Map hot path: one split per GPU, match records
gathered to the reducing rank.

In the reference, each map task (one input file, map_reduce/coordinator.go:312,
329-333) is scanned independently and its output travels to the reducers by
SFTP (map_reduce/coordinator.go:136-142). Here one process per GPU scans its
split in HBM and the compacted records -- never the line bytes -- go to rank
`dst` with torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo"
in the CPU tests).

The exchange: RCCL has no gatherv, so
  1. the per-rank record counts are all-gathered (one 8-byte element per rank);
  2. every rank packs its records into 28-byte records {u64 line_no, u64 start,
     u64 len, u32 split} (7 int32 words, on the device) -- `split` names the map
     task the record came from (the coordinator's task id for the file,
     map_reduce/coordinator.go:329-333), so the reducing rank can rebuild each
     Key = Sprintf("%s (line number #%v)", filename[split], line_no)
     (grep.go:25) without a side channel -- and the senders' records move with
     grouped point-to-point send/recv (batch_isend_irecv) straight into one
     buffer on `dst`, in rank order: exactly sum(counts) x 28 bytes cross xGMI,
     each sender on its own link; nothing is padded to the largest count.
Only `dst` turns the gathered counts into host integers (it must size its
receive buffers); the senders already hold their own count, which
dgrep_scan_device returns.
"""
from typing import Optional

import torch
import torch.distributed as dist

REC_WORDS = 7  # int32 words per record: line_no (2), start (2), len (2), split (1) = 28 B
REC_BYTES = 4 * REC_WORDS


def pack_records(line_no: torch.Tensor, start: torch.Tensor, length: torch.Tensor, count: int,
                 split: int = 0) -> torch.Tensor:
    """[count * 7] int32 on the records' device: per record the little-endian
    words of (u64 line_no, u64 start, u64 len, u32 split)."""
    dev = line_no.device
    if count == 0:
        return torch.empty(0, dtype=torch.int32, device=dev)
    ln = line_no[:count].to(torch.int64).contiguous().view(torch.int32).view(count, 2)
    st = start[:count].to(torch.int64).contiguous().view(torch.int32).view(count, 2)
    le = length[:count].to(torch.int64).contiguous().view(torch.int32).view(count, 2)
    sp = torch.full((count, 1), int(split) & 0xFFFFFFFF, dtype=torch.int64, device=dev).to(torch.int32)
    return torch.cat([ln, st, le, sp], dim=1).reshape(-1)


def unpack_records(buf: torch.Tensor, count: int):
    """Inverse of pack_records: (line_no int64, start int64, len int64, split int64)."""
    r = buf[: count * REC_WORDS].view(count, REC_WORDS)
    def words(lo, hi):
        # a fresh dense copy: 8-byte aligned and contiguous whatever the slice was
        t = torch.empty((count, hi - lo), dtype=torch.int32, device=buf.device)
        t.copy_(r[:, lo:hi])
        return t

    ln = words(0, 2).view(torch.int64).reshape(-1)
    st = words(2, 4).view(torch.int64).reshape(-1)
    le = words(4, 6).view(torch.int64).reshape(-1)
    sp = words(6, 7).reshape(-1).to(torch.int64) & 0xFFFFFFFF
    return ln, st, le, sp


def gather_records(line_no: torch.Tensor, start: torch.Tensor, length: torch.Tensor, count: int,
                   dst: int = 0, group=None, split: Optional[int] = None):
    """Gather every rank's match records to `dst`. `split` is this rank's map
    task id (default: its rank). Returns, on `dst`, one (line_no, start, len,
    split) tuple per rank in rank order (each exactly that rank's count long);
    None elsewhere. `dst` and the peers are global ranks."""
    world = dist.get_world_size(group)
    rank = dist.get_rank()
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(world))
    dev = line_no.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.empty(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    packed = pack_records(line_no, start, length, count, rank if split is None else split)
    if rank != dst:
        if count:
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, packed, dst, group)]):
                req.wait()
        return None
    cl = torch.cat(counts).tolist()  # the root sizes its receive buffer: its one host sync
    total = sum(cl)
    out = torch.empty(total * REC_WORDS, dtype=torch.int32, device=dev)
    ops, off, views = [], 0, []
    for peer, c in zip(ranks, cl):
        seg = out[off * REC_WORDS:(off + c) * REC_WORDS]
        views.append((seg, c))
        if peer == dst:
            if c:
                seg.copy_(packed)
        elif c:
            ops.append(dist.P2POp(dist.irecv, seg, peer, group))
        off += c
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return [unpack_records(seg, c) for seg, c in views]
