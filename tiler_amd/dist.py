"""Multi-GPU sharding of the hot path: one process per GPU, torch.distributed (RCCL over xGMI
on MI355X with backend "nccl"; gloo on CPU for tests).

The work units are independent, so the data path has no collective of its own:
  * FrameTiling and Smooth: keyframes (PrepareFrameTiling / DoTemporalSmoothing are keyframe-local,
    main.pas:4005-4011, 4081-4082) -> longest-processing-time assignment by frames x tiles;
  * GlobalTiling K-Modes: palette bins (DoKModes per bin, main.pas:4339) -> LPT by n_bin x k_bin.
The exchanges are the pipeline's own, each ONE fixed-layout tensor collective (no pickled objects):
  * after K-Modes: the merge map, int32 [T] (-1 = kept), all-reduced with MAX -- every tile belongs to exactly
    one bin, so exactly one rank writes its entry; every rank then applies MergeTiles identically and holds the
    reduced tileset (the north star's tileset all-gather);
  * before ReindexTiles: the UseCount histogram, int64 [T], all-reduced with SUM (main.pas:1208-1221);
  * for SaveStream: each rank writes AND compresses its own keyframes' streams (LZCompress per keyframe is
    independent); the stream lengths, int64 [KF], are all-reduced with SUM and each rank sends its streams to the
    saving rank as one uint8 buffer (point-to-point, gather_units), which assembles the file.  No rank holds
    another rank's frames or tilemaps at any point: per-rank memory is O(its keyframes) plus the tileset.
Tensors live on the rank's GPU under nccl (RCCL reads HBM directly) and on the CPU under gloo.
"""
from __future__ import annotations

import heapq
from typing import Sequence

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


def comm_device():
    """Where collective tensors live: this rank's GPU under nccl (RCCL), the CPU under gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _to_tensor(a: np.ndarray, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def broadcast_array(a: np.ndarray | None, shape, dtype, src: int = 0, device=None) -> np.ndarray:
    """Rank `src` sends `a`; every rank returns it."""
    import torch
    import torch.distributed as dist
    device = comm_device() if device is None else device
    t = _to_tensor(a, device) if dist.get_rank() == src else \
        torch.empty(shape, dtype=getattr(torch, np.dtype(dtype).name), device=device)
    dist.broadcast(t, src)
    return t.cpu().numpy()


def allreduce(a: np.ndarray, op: str = "sum", device=None) -> np.ndarray:
    """Element-wise SUM / MAX over ranks of a fixed-layout array (UseCount histogram, merge map)."""
    import torch.distributed as dist
    t = _to_tensor(a, comm_device() if device is None else device)
    dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op])
    return t.cpu().numpy()


def allreduce_sum(a: np.ndarray, device=None) -> np.ndarray:
    """UseCount histogram for ReindexTiles (main.pas:1208-1221)."""
    return allreduce(a, "sum", device)


def gather_units(parts: dict, owner_of, dst: int = 0, device=None) -> list | None:
    """Variable-size byte units (e.g. compressed keyframe streams) onto rank `dst`, in unit order.  parts maps
    unit -> bytes for the units this rank owns (owner_of[u] == rank); the lengths, int64 [n_units], are all-reduced
    (SUM: one owner per unit), then every other rank sends its units concatenated in unit order as ONE uint8 tensor.
    Returns the list of all units' bytes on dst, None elsewhere."""
    import torch
    import torch.distributed as dist
    device = comm_device() if device is None else device
    rank, world = dist.get_rank(), dist.get_world_size()
    n = len(owner_of)
    lens = np.zeros(n, np.int64)
    for u, b in parts.items():
        assert owner_of[u] == rank, (u, owner_of[u], rank)
        lens[u] = len(b)
    lens = allreduce(lens, "sum", device)
    if rank != dst:
        mine = [u for u in range(n) if owner_of[u] == rank]
        total = int(sum(lens[u] for u in mine))
        if total:
            buf = np.frombuffer(b"".join(parts[u] for u in mine), np.uint8)
            dist.send(torch.from_numpy(buf.copy()).to(device), dst)
        return None
    out = [parts.get(u) for u in range(n)]
    for r in range(world):
        if r == dst:
            continue
        units = [u for u in range(n) if owner_of[u] == r]
        total = int(sum(lens[u] for u in units))
        if not total:
            for u in units:
                out[u] = b""
            continue
        t = torch.empty(total, dtype=torch.uint8, device=device)
        dist.recv(t, r)
        buf = t.cpu().numpy().tobytes()
        o = 0
        for u in units:
            out[u] = buf[o:o + int(lens[u])]
            o += int(lens[u])
    return out
