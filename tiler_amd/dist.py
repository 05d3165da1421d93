"""Multi-GPU sharding of the hot path: one process per GPU, torch.distributed
(RCCL over xGMI on MI355X, gloo on CPU for tests).

The work units are independent, so there is no data-path collective:
  * FrameTiling and Smooth: keyframes (PrepareFrameTiling / DoTemporalSmoothing are keyframe-local,
    main.pas:4005-4011, 4081-4082) -> longest-processing-time assignment by frames x tiles;
  * GlobalTiling K-Modes: palette bins (DoKModes per bin, main.pas:4339) -> LPT by n_bin x k_bin.
The exchanges are the pipeline's own: the global tileset broadcast before FrameTiling, the tilemap
gather after it, the UseCount all-reduce for ReindexTiles (main.pas:1208-1221) and the all-gather of
per-bin merge results after K-Modes.
"""
from __future__ import annotations

import heapq
from typing import Callable, Sequence

import numpy as np


def lpt_assign(costs: Sequence[float], world: int) -> list[list[int]]:
    """Longest-processing-time-first: unit i -> rank; deterministic (ties by unit then rank index)."""
    order = sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i))
    heap = [(0.0, r) for r in range(world)]
    out: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + float(costs[i]), r))
    return [sorted(o) for o in out]


def plan_keyframes(kf_frames: Sequence[int], tiles_per_frame: int, world: int) -> list[list[int]]:
    return lpt_assign([f * tiles_per_frame for f in kf_frames], world)


def plan_bins(bin_sizes: Sequence[int], k_per_bin: Sequence[int], world: int) -> list[list[int]]:
    return lpt_assign([max(1, n) * max(1, k) for n, k in zip(bin_sizes, k_per_bin)], world)


def broadcast_array(a: np.ndarray | None, shape, dtype, src: int = 0, device=None) -> np.ndarray:
    """Rank `src` sends `a`; every rank returns it (the tileset 'all-gather' of the north star)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(a)).to(device) if dist.get_rank() == src else \
        torch.empty(shape, dtype=getattr(torch, np.dtype(dtype).name), device=device)
    dist.broadcast(t, src)
    return t.cpu().numpy()


def allreduce_sum(a: np.ndarray, device=None) -> np.ndarray:
    """UseCount histogram for ReindexTiles (main.pas:1208-1221)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(a)).to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def run_sharded(n_units: int, costs: Sequence[float], fn: Callable[[int], dict], device=None) -> dict[int, dict]:
    """Run fn(unit) for this rank's units (LPT plan) and all-gather every unit's result dict of numpy arrays.
    Returns {unit: result} on every rank."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    plan = lpt_assign(costs, world)
    mine = {u: fn(u) for u in plan[rank]}
    gathered: list = [None] * world
    dist.all_gather_object(gathered, mine)
    out: dict[int, dict] = {}
    for g in gathered:
        out.update(g)
    assert sorted(out) == list(range(n_units))
    return out
