"""Data parallelism for the summarization pipeline.

The reference scales horizontally by running more service replicas behind RabbitMQ competing
consumers (orchestrator and summarization are stateless per thread).  On a node of
8 MI355X the equivalent is one engine per GPU (or per TP group) and a deterministic split of the
threads across them:

* :func:`owner_of` -- stable owner rank of a key (sha1, independent of PYTHONHASHSEED) so every
  rank computes the same split without communication;
* :func:`balanced_shard` -- longest-processing-time-first assignment by cost (prompt tokens), so
  ranks finish together instead of waiting on the one that drew the 10k-token threads;
* :func:`gather_objects` -- results back to every rank (all_gather_object; small payloads).

Reference scaling it replaces: competing consumers per queue, Container Apps replicas on queue
length (infra/azure/modules/containerapps.bicep:262-263,711-730).
"""
from __future__ import annotations

import hashlib
import heapq
from typing import Callable, Sequence, TypeVar

import torch.distributed as dist

T = TypeVar("T")


def owner_of(key: str, world: int) -> int:
    if world <= 1:
        return 0
    return int.from_bytes(hashlib.sha1(key.encode("utf-8")).digest()[:8], "big") % world


def hash_shard(items: Sequence[T], rank: int, world: int, key: Callable[[T], str] = str) -> list[T]:
    return [x for x in items if owner_of(key(x), world) == rank]


def balanced_shard(costs: Sequence[float], world: int) -> list[list[int]]:
    """Indices per rank; LPT greedy (<= 4/3 of the optimal makespan), ties broken by index."""
    bins: list[list[int]] = [[] for _ in range(world)]
    heap = [(0.0, r) for r in range(world)]
    for i in sorted(range(len(costs)), key=lambda j: (-costs[j], j)):
        load, r = heapq.heappop(heap)
        bins[r].append(i)
        heapq.heappush(heap, (load + float(costs[i]), r))
    return [sorted(b) for b in bins]


def gather_objects(obj, group=None) -> list:
    """List of every rank's ``obj`` (rank order); ``[obj]`` when not distributed."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out
