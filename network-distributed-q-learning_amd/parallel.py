"""Multi-GPU env sharding: one process per GPU, each owning a disjoint block of envs.

The reference parallelises by launching independent ``main.py`` processes per seed /
hyper-parameter (hyperparam_tuning.py:85-91) with no communication; the MI355X build
does the same inside one job: rank r owns envs [r*E, (r+1)*E) (seeds base + global env
index), runs them with no collective on the data path (weak scaling), and only the
run's summary numbers are reduced (timing max, decision count sum) or gathered (per-env
episode statistics, a few bytes per env) at the end.  ``torch.distributed`` with backend
"nccl" is RCCL over xGMI on the GPU box; tests use "gloo" on the CPU.
"""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np


def world() -> Tuple[int, int, int]:
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl"):
    """Initialise torch.distributed from the torchrun environment; returns the module or None."""
    ws, rank, local = world()
    if ws <= 1:
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend)
    return dist


def shard_seeds(base_seed: int, envs_per_rank: int, rank: int) -> List[int]:
    return [int(base_seed) + rank * envs_per_rank + i for i in range(envs_per_rank)]


def reduce_timing(dist, seconds: float, count: float, device=None) -> Tuple[float, float]:
    """(max seconds over ranks, sum of counts over ranks)."""
    if dist is None:
        return float(seconds), float(count)
    import torch
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    n = torch.tensor([count], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), float(n.item())


def gather_env_stats(dist, arr: np.ndarray, device=None) -> np.ndarray:
    """Concatenate per-env arrays (env axis last) from all ranks, in rank order."""
    if dist is None:
        return arr
    import torch
    t = torch.from_numpy(np.ascontiguousarray(arr)).to(device) if device is not None else torch.from_numpy(
        np.ascontiguousarray(arr))
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return np.concatenate([p.cpu().numpy() for p in parts], axis=-1)
