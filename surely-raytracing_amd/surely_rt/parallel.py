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

import ctypes as C
from pathlib import Path

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


GATHER_RCCL = "rt_gather_frame (ncclGather, librtgather.so, include/rt_gather.h)"
GATHER_TORCH = "torch.distributed.gather"


def gather_choice(world: int, rehearse: bool) -> str:
    """Which frame gather bench.py times at `world` ranks: the product's own C-ABI gather
    (rt_gather_frame: one ncclGather over RCCL/xGMI + the de-interleave kernel on rank 0) when
    every rank has its own GPU; torch.distributed.gather over gloo through host memory in the
    one-GPU rehearsal (RT_BENCH_REHEARSAL=1: RCCL refuses two ranks on one device); none at
    one rank (the rows are the frame)."""
    if world <= 1:
        return "none (one rank renders every row)"
    if rehearse:
        return GATHER_TORCH + " (gloo rehearsal on one GPU, through host memory)"
    return GATHER_RCCL


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


# ---------------------------------------------------------------- the C-ABI RCCL gather
_gather = None


def gather_lib():
    """librtgather.so (include/rt_gather.h): the framebuffer gather over RCCL for a host that runs
    one process per GPU without torch.distributed. Raises if it is not built."""
    global _gather
    if _gather is None:
        path = Path(__file__).resolve().parent.parent.parent / "build" / "librtgather.so"
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make gather`")
        lib = C.CDLL(str(path))
        p = C.c_void_p
        sig = {
            "rt_gather_last_error": (C.c_char_p, []),
            "rt_gather_unique_id": (C.c_int, [C.c_char_p]),
            "rt_gather_comm_create": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int,
                                                C.POINTER(p)]),
            "rt_gather_comm_destroy": (None, [p]),
            "rt_gather_rows": (C.c_int, [C.c_int, C.c_int, C.c_int]),
            "rt_gather_max_rows": (C.c_int, [C.c_int, C.c_int]),
            "rt_gather_frame": (C.c_int, [p, p, C.c_int, C.c_int, p, p, p]),
            "rt_gather_deinterleave": (C.c_int, [p, C.c_int, C.c_int, C.c_int, p, p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _gather = lib
    return _gather


class RcclFrameGather:
    """One rank's member of an RCCL communicator for the frame gather (rt_gather_comm)."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int = 0):
        self._lib = gather_lib()
        h = C.c_void_p()
        rc = self._lib.rt_gather_comm_create(uid, world, rank, device, C.byref(h))
        if rc != 0:
            raise RuntimeError(self._lib.rt_gather_last_error().decode())
        self._h, self.world, self.rank = h, world, rank

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        lib = gather_lib()
        if lib.rt_gather_unique_id(buf) != 0:
            raise RuntimeError(lib.rt_gather_last_error().decode())
        return buf.raw

    def gather(self, local_ptr: int, width: int, height: int, scratch_ptr: int, frame_ptr: int,
               stream: int = 0):
        rc = self._lib.rt_gather_frame(self._h, C.c_void_p(local_ptr), width, height,
                                       C.c_void_p(scratch_ptr or None),
                                       C.c_void_p(frame_ptr or None), C.c_void_p(stream or None))
        if rc != 0:
            raise RuntimeError(self._lib.rt_gather_last_error().decode())

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt_gather_comm_destroy(self._h)
            self._h = None
