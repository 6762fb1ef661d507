"""Recording sharding and the per-file result gather.

Recordings are independent: rank r of a world of N processes (one per GPU)
takes files r, r+N, r+2N, ... and classifies them on its own GPU with no
data-path collective.  The only exchange is at the end: every rank's
per-track score records are gathered to every rank (RCCL all-gather over xGMI
with the "nccl" backend; gloo on CPU in the tests), and rank 0 renders the
results in file order, so the output is identical to a 1-GPU run.

Record layout (float32 row, fixed width 3 + L):
    [file_idx, track_idx, n_labels_valid, p_0 .. p_{L-1}]
Rows are padded to the largest per-rank count before the all-gather (the
collective needs equal sizes); padding rows carry file_idx = -1.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard(items, rank: int, world: int):
    """Static round-robin split of a file list: file i goes to rank i % world."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return [(i, x) for i, x in enumerate(items) if i % world == rank]


def pack_records(file_idx, track_idx, scores, width):
    """Rows [file_idx, track_idx, L, scores...] padded to ``width`` labels."""
    scores = np.asarray(scores, np.float32)
    n, L = scores.shape if scores.ndim == 2 else (0, 0)
    if L > width:
        raise ValueError(f"{L} labels > record width {width}")
    rec = np.zeros((n, 3 + width), np.float32)
    rec[:, 0] = file_idx
    rec[:, 1] = track_idx
    rec[:, 2] = L
    if n:
        rec[:, 3:3 + L] = scores
    return rec


def gather_records(rec: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather variable-length record blocks; returns every valid row of
    every rank sorted by (file_idx, track_idx).  ``rec`` lives on the device
    the process group's backend uses (cuda for nccl, cpu for gloo)."""
    if not dist.is_initialized():
        out = rec
    else:
        world = dist.get_world_size(group)
        n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=rec.device)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n, group=group)
        m = int(max(int(c.item()) for c in counts))
        pad = torch.full((m, rec.shape[1]), -1.0, dtype=rec.dtype, device=rec.device)
        pad[:rec.shape[0]] = rec
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out = torch.cat(parts)
    out = out[out[:, 0] >= 0]
    if out.shape[0] == 0:
        return out
    key = out[:, 0].double() * 1e6 + out[:, 1].double()
    return out[torch.argsort(key)]


def unpack_records(rec: torch.Tensor):
    """{file_idx: {track_idx: np.float32[L]}} from gathered rows."""
    res = {}
    for row in rec.cpu().numpy():
        f, t, L = int(row[0]), int(row[1]), int(row[2])
        res.setdefault(f, {})[t] = row[3:3 + L].copy()
    return res
