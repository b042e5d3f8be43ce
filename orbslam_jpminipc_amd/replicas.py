"""Multi-GPU plumbing: one process per GPU, independent frame streams, no data-path collectives.

Frames of different streams are independent and SearchForInitialization pairs frames of
the same stream, so the front end shards as replicas: stream s runs on
rank s mod world.  The only cross-rank traffic is the benchmark's barrier and the max over
ranks of the timed region (a 1-element all-reduce) and a gather of the per-rank seconds.  These
scalars go over "gloo" by default, on GPUs too: nothing on the data path is exchanged, so
RCCL ("nccl") would add only its per-rank init; it stays selectable.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int
    local_rank: int
    world: int


def init_from_env(backend: str | None = None) -> DistInfo:
    """Read RANK / LOCAL_RANK / WORLD_SIZE (torch.distributed.run); init a group if world > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return DistInfo(rank, local, world)


def streams_of_rank(n_streams: int, rank: int, world: int) -> list[int]:
    """Stream s -> rank s mod world (SURVEY.md §8e partitioning)."""
    return [s for s in range(n_streams) if s % world == rank]


def barrier(info: DistInfo) -> None:
    if info.world > 1:
        dist.barrier()


def max_over_ranks(value: float, info: DistInfo) -> float:
    """Max of a per-rank scalar (the timed region); identity when world == 1."""
    if info.world == 1:
        return float(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, info: DistInfo) -> float:
    if info.world == 1:
        return float(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_over_ranks(value: float, info: DistInfo) -> list[float]:
    """Every rank's scalar, in rank order (the per-rank timed regions of the benchmark)."""
    if info.world == 1:
        return [float(value)]
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(info.world)]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def whole_job_rate(units_per_rank: int, world: int, seconds_max: float) -> float:
    """Whole-job throughput: all ranks' units over the slowest rank's time (weak scaling)."""
    return units_per_rank * world / seconds_max


def shutdown(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
