"""Multi-GPU execution: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm) / xGMI.

* :func:`init_distributed` -- env:// rendezvous (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*), one
  device per local rank, RCCL on GPUs and gloo on CPU (tests).
* :func:`make_groups` -- TP groups of ``tp`` consecutive ranks (the 8 GPUs of a node are fully
  xGMI-connected, so any grouping is one hop), DP groups across them.
* :mod:`.tp` -- Megatron column/row sharding of the decoder (one all-reduce after o_proj and after
  down_proj, vocab-parallel lm_head).
* :mod:`.dp` -- data-parallel thread sharding for the orchestrator (stable hash of thread ids).
* :mod:`.knn` -- vector index sharded over ranks: local top-k on every shard, all-gather of the
  k candidates, exact merge.
"""
from __future__ import annotations

import dataclasses
import datetime
import os

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = dataclasses.field(default_factory=lambda: torch.device("cpu"))
    backend: str | None = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: str | None = None, timeout_s: int = 600) -> DistEnv:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or os.environ.get("CFC_DIST_BACKEND") or None
    use_gpu = torch.cuda.is_available() and (backend != "gloo" or os.environ.get("CFC_DIST_BACKEND") == "gloo")
    if use_gpu:
        # ranks beyond the visible GPUs share them (rehearsing N ranks on fewer GPUs with gloo)
        dev_idx = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    be = backend or ("nccl" if use_gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        if be == "nccl":
            from .resilience import configure_collective_timeouts
            configure_collective_timeouts(timeout_s)
        kw = {"device_id": device} if be == "nccl" else {}
        dist.init_process_group(be, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistEnv(rank, world, local, device, be if world > 1 else None)


@dataclasses.dataclass
class Groups:
    tp_group: object
    dp_group: object
    tp_rank: int
    tp_size: int
    dp_rank: int
    dp_size: int
    tp_cpu_group: object = None   # gloo twin of tp_group for host objects (prompts) off the main thread
    tp_src: int = 0               # global rank of this TP group's leader

    @property
    def is_tp_leader(self) -> bool:
        return self.tp_rank == 0


def make_groups(env: DistEnv, tp: int) -> Groups:
    if env.world % tp:
        raise ValueError(f"world size {env.world} not divisible by tp={tp}")
    if env.world == 1:
        return Groups(None, None, 0, 1, 0, 1)
    tp_groups, tp_cpu, dp_groups = [], [], []
    for s in range(0, env.world, tp):  # every rank must create every group, in the same order
        ranks = list(range(s, s + tp))
        tp_groups.append(dist.new_group(ranks))
        # a SEPARATE gloo group even when the job runs on gloo: host objects (prompts, engine steps)
        # are broadcast from another thread than the TP all-reduces, and two threads issuing
        # collectives on one group can order them differently on different ranks (deadlock)
        tp_cpu.append(dist.new_group(ranks, backend="gloo"))
    for i in range(tp):
        dp_groups.append(dist.new_group(list(range(i, env.world, tp))))
    g = env.rank // tp
    return Groups(tp_groups[g], dp_groups[env.rank % tp], env.rank % tp, tp, g, env.world // tp,
                  tp_cpu_group=tp_cpu[g], tp_src=g * tp)
