"""Multi-GPU: frames shard across ranks, one process per GPU, no collective on the data path.

LoRa frames (and channels) are independent: rank r demodulates a
contiguous block of frames on its own GPU.  Collectives appear only around the
measurement (max-over-ranks time, summed units) and, optionally, to gather results
to one rank for checking - never inside the demodulation itself.
The helpers use whichever torch.distributed backend the caller initialised (bench.py
uses gloo over host TCP, for the timing barrier and the max/sum of the timings only; the
tests use gloo on CPU); nothing here runs on the demodulation path, so no RCCL is needed.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n_frames: int, rank: int, world: int) -> Tuple[int, int]:
    """Balanced contiguous [start, stop) block of frames owned by `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(int(n_frames), world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def _active(group) -> bool:
    return dist.is_available() and dist.is_initialized()


def _coll_device(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def aggregate_throughput(local_units: float, local_seconds: float,
                         group: Optional[object] = None) -> Tuple[float, float, float]:
    """Whole-job throughput for weak scaling: (sum of units over ranks,
    max of seconds over ranks, units / seconds).  Single process: the local values."""
    if not _active(group):
        return float(local_units), float(local_seconds), float(local_units) / float(local_seconds)
    dev = _coll_device(group)
    t = torch.tensor([float(local_seconds)], dtype=torch.float64, device=dev)
    u = torch.tensor([float(local_units)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(u, op=dist.ReduceOp.SUM, group=group)
    units, secs = float(u.item()), float(t.item())
    return units, secs, units / secs


def gather_frames(local: torch.Tensor, n_frames: int, group: Optional[object] = None) -> torch.Tensor:
    """Reassemble per-rank [F_r, ...] results (blocks from shard_range) into the global
    [n_frames, ...] tensor on every rank.  Checking/reporting only."""
    if not _active(group):
        return local
    world = dist.get_world_size(group)
    dev = _coll_device(group)
    biggest = max(b - a for a, b in (shard_range(n_frames, r, world) for r in range(world)))
    pad = torch.zeros((biggest,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[: local.shape[0]] = local.to(dev)
    # gloo/nccl all_gather need a wire dtype they know; uint16/uint8 travel as int32
    wire = pad.to(torch.int32) if pad.dtype in (torch.uint16, torch.uint8, torch.bool) else pad
    parts = [torch.empty_like(wire) for _ in range(world)]
    dist.all_gather(parts, wire, group=group)
    out = [p[: b - a] for p, (a, b) in zip(parts, (shard_range(n_frames, r, world) for r in range(world)))]
    return torch.cat(out).to(local.dtype).to(local.device)
