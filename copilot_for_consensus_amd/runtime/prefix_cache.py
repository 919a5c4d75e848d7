"""Prefix cache over the paged KV cache: full 32-token blocks shared across sequences.

Every summarization prompt starts with the same system prompt and template head (SURVEY §3.3,
orchestrator prompts), so the KV of those leading blocks is identical for every thread.  The
engine looks each prompt's leading full blocks up by a hash chain (block j's key covers tokens
[0, 32(j+1))), points the sequence's block table at the cached physical blocks and starts its
prefill after them -- the prefill kernel already reads keys [0, ctx) from the cache, so no kernel
change is needed.

Ownership: a block's refcount = sequences using it (+ nothing for the cache itself); blocks whose
refcount drops to 0 stay cached in LRU order and go back to the pool only when an allocation
needs room (``alloc`` evicts).  Entries inserted for a batch are visible to later prompts of the
SAME batch: the prefill writes a layer's K/V for every token of a chunk before that layer's
attention runs, and an owning prompt is always prefilled in the same or an earlier chunk than the
prompts that reuse its blocks.

Reference counterpart: llama.cpp's prompt cache behind llamacpp_summarizer.py:108 (the server
reuses a matching prompt prefix).
"""
from __future__ import annotations

import collections
import hashlib

import numpy as np

from ..ops.reference import KV_BLOCK


def block_keys(tokens: list[int], n_blocks: int) -> list[bytes]:
    """Hash-chain keys of the first ``n_blocks`` full blocks."""
    keys, h = [], b""
    arr = np.asarray(tokens[:n_blocks * KV_BLOCK], dtype=np.int64)
    for j in range(n_blocks):
        h = hashlib.blake2b(h + arr[j * KV_BLOCK:(j + 1) * KV_BLOCK].tobytes(), digest_size=16).digest()
        keys.append(h)
    return keys


class PrefixCache:
    def __init__(self, pool, max_cached_blocks: int | None = None):
        self.pool = pool
        self.max_cached = max_cached_blocks
        self._block: dict[bytes, int] = {}                       # key -> physical block
        self._key: dict[int, bytes] = {}                          # physical block -> key
        self._ref: collections.Counter = collections.Counter()    # physical block -> users
        self._lru: collections.OrderedDict = collections.OrderedDict()  # unreferenced cached blocks
        self.hits = 0        # blocks served from the cache
        self.lookups = 0     # shareable blocks looked up

    # ------------------------------------------------------------------ allocation
    def alloc(self, n: int) -> list[int]:
        """Fresh blocks from the pool, evicting unreferenced cached blocks if the pool is short."""
        short = n - self.pool.num_free()
        if short > 0:
            self.evict(short)
        out = self.pool.alloc(n)
        for b in out:
            self._ref[b] += 1
        return out

    def evict(self, n: int) -> int:
        freed = []
        while self._lru and len(freed) < n:
            b, _ = self._lru.popitem(last=False)
            del self._block[self._key.pop(b)]
            freed.append(b)
        self.pool.free(freed)
        return len(freed)

    # ------------------------------------------------------------------ sharing
    def acquire(self, tokens: list[int]) -> list[int]:
        """Longest cached prefix of whole blocks (always leaving >= 1 token to prefill)."""
        n = (len(tokens) - 1) // KV_BLOCK
        self.lookups += n
        out = []
        for k in block_keys(tokens, n):
            b = self._block.get(k)
            if b is None:
                break
            if self._ref[b] == 0:
                self._lru.pop(b, None)
            self._ref[b] += 1
            out.append(b)
        self.hits += len(out)
        return out

    def insert(self, tokens: list[int], table: list[int]) -> None:
        """Publish the full prompt blocks of a sequence (its table must already hold them)."""
        n = (len(tokens) - 1) // KV_BLOCK
        for k, b in zip(block_keys(tokens, n), table):
            if k in self._block or b in self._key:
                continue
            self._block[k] = b
            self._key[b] = k
        if self.max_cached is not None and len(self._block) > self.max_cached:
            self.evict(len(self._block) - self.max_cached)

    def invalidate(self, table: list[int]) -> None:
        """Drop cache entries pointing at these blocks (their contents were never computed)."""
        for b in table:
            k = self._key.pop(b, None)
            if k is not None:
                del self._block[k]
                self._lru.pop(b, None)

    def release(self, table: list[int]) -> None:
        to_pool = []
        for b in table:
            self._ref[b] -= 1
            if self._ref[b] <= 0:
                del self._ref[b]
                if b in self._key:
                    self._lru[b] = None          # stays cached, evictable
                else:
                    to_pool.append(b)
        self.pool.free(to_pool)

    def cached_blocks(self) -> int:
        return len(self._block)

    def clear(self) -> None:
        self.evict(len(self._lru))
