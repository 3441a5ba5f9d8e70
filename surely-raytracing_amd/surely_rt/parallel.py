"""Row tiling of the framebuffer across ranks + gather to rank 0.

The reference parallelises only inside one process (rayon over 3-row chunks,
/root/reference/src/render.rs:171-197). Pixels are independent, so across GPUs the image is
split by rows with NO data-path collective; the only exchange is the final framebuffer gather
to rank 0 (torch.distributed: RCCL over xGMI with the "nccl" backend, gloo on CPU).

Rows are dealt cyclically (row r -> rank r % world): light, glass-caustic and wall rows have
very different costs, and interleaving balances them. The RNG is keyed by the global
(pixel, sample) pair, so the gathered image is bitwise identical for any world size.
"""
from __future__ import annotations

import numpy as np


def cyclic_rows(height: int, rank: int, world: int):
    """(row_begin, row_step, n_rows) of `rank`'s rows under cyclic tiling."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank, world, len(range(rank, height, world))


def max_rows(height: int, world: int) -> int:
    """Rows per rank after padding to an equal gather count."""
    return -(-height // world)


def deinterleave(gathered, height: int, world: int):
    """gathered: [world, max_rows, W, 3] (numpy or torch) -> [height, W, 3] in image order."""
    W = gathered.shape[2]
    if isinstance(gathered, np.ndarray):
        out = np.empty((height, W, 3), gathered.dtype)
    else:
        import torch

        out = torch.empty((height, W, 3), dtype=gathered.dtype, device=gathered.device)
    for r in range(world):
        n = len(range(r, height, world))
        out[r::world] = gathered[r, :n]
    return out


def gather_frame(local, height: int, rank: int, world: int, dst: int = 0):
    """Gather every rank's padded row block to `dst` and de-interleave there.

    local: torch tensor [max_rows(height, world), W, 3] on this rank's device.
    Returns the full [height, W, 3] tensor on dst, None elsewhere.
    """
    import torch
    import torch.distributed as dist

    if world == 1:
        n = len(range(0, height, 1))
        return local[:n]
    bufs = [torch.empty_like(local) for _ in range(world)] if rank == dst else None
    dist.gather(local, gather_list=bufs, dst=dst)
    if rank != dst:
        return None
    return deinterleave(torch.stack(bufs), height, world)


def rank_report(local: dict, rank: int, world: int, dst: int = 0):
    """Every rank's timings (a dict of floats: rt_trace ms, render ms, gather ms, ...) gathered
    to `dst` (torch.distributed.gather_object; outside any timed region). On dst: each key as a
    per-rank list, plus the slowest / fastest rank ratio of the render and kernel times (the
    share imbalance a strong-scaling step pays). None elsewhere."""
    import torch.distributed as dist

    objs = [None] * world if rank == dst else None
    dist.gather_object(local, objs, dst=dst)
    if rank != dst:
        return None
    rep = {f"{k}_per_rank": [round(float(o[k]), 3) for o in objs] for k in sorted(local)}
    for k in ("trace_ms", "render_ms", "gather_ms"):
        if k in local:
            v = [float(o[k]) for o in objs]
            rep[f"{k}_slowest"] = round(max(v), 3)
            if k != "gather_ms" and min(v) > 0:
                rep[f"{k}_slowest_fastest_ratio"] = round(max(v) / min(v), 4)
    return rep
