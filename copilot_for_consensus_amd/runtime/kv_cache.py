"""Paged KV cache sized for one MI355X (288 GB HBM3E).

Layout per layer (see csrc/kernels/attention.hip for why):
  K: [num_blocks, kv_heads, 32, head_dim]        (row = key)
  V: [num_blocks, kv_heads, head_dim, 32]        (transposed, keys slot-permuted per block)
Both live in ONE allocation per tensor kind ([layers, ...]) so the cache is a single HBM
region; blocks are handed out by :class:`BlockPool` (the C++ free list in
csrc/runtime/blockpool.cpp when the runtime library is available).

Sized for the reference's LLM context (LLAMA_ARG_CTX_SIZE 4096, docker-compose.infra.yml:297) and
beyond.
"""
from __future__ import annotations

import math

import torch

from ..ops.reference import KV_BLOCK


class BlockPool:
    """LIFO free list of KV blocks (native C++ implementation with a Python fallback on CPU)."""

    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._native = None
        try:
            from ..ops._native import runtime
            lib = runtime()
            if hasattr(lib, "cfc_blockpool_create"):
                self._lib = lib
                self._native = lib.cfc_blockpool_create(num_blocks)
        except Exception:  # runtime lib not built (pure-CPU CI before build) -> python list
            self._native = None
        if self._native is None:
            self._free = list(range(num_blocks - 1, -1, -1))

    def __del__(self):
        if getattr(self, "_native", None):
            self._lib.cfc_blockpool_destroy(self._native)
            self._native = None

    def num_free(self) -> int:
        if self._native:
            return int(self._lib.cfc_blockpool_num_free(self._native))
        return len(self._free)

    def alloc(self, n: int) -> list[int]:
        if n == 0:
            return []
        if self._native:
            import numpy as np
            out = np.empty(n, dtype=np.int32)
            rc = self._lib.cfc_blockpool_alloc(self._native, n, out.ctypes.data)
            if rc != 0:
                raise MemoryError(f"KV cache exhausted: need {n} blocks, {self.num_free()} free")
            return out.tolist()
        if n > len(self._free):
            raise MemoryError(f"KV cache exhausted: need {n} blocks, {len(self._free)} free")
        out = self._free[-n:][::-1]
        del self._free[-n:]
        return out

    def free(self, blocks: list[int]) -> None:
        if not blocks:
            return
        if self._native:
            import numpy as np
            arr = np.asarray(blocks, dtype=np.int32)
            self._lib.cfc_blockpool_free(self._native, arr.ctypes.data, len(blocks))
            return
        self._free.extend(reversed(blocks))


class PagedKVCache:
    """K [layers][blocks, kv_heads, 32, D] and V^T [layers][blocks, kv_heads, D, 32] (slot-permuted,
    stored as [4 slot groups][D][8] per block and head: ops.reference.v_groups).

    ``dtype`` bf16 (default) or ``torch.float8_e4m3fn``: the FP8 cache halves the bytes the decode
    attention streams; it holds K / ``k_scale`` and V / ``v_scale`` (clamped to +-448) and the
    kernels scale back.  Opt-in: it is a precision trade-off, not the default."""

    def __init__(self, layers: int, num_blocks: int, kv_heads: int, head_dim: int, device, dtype=torch.bfloat16,
                 k_scale: float = 1.0, v_scale: float = 1.0):
        if dtype not in (torch.bfloat16, torch.float8_e4m3fn):
            raise ValueError(f"KV cache dtype {dtype} not supported (bfloat16 or float8_e4m3fn)")
        self.layers, self.num_blocks, self.kv_heads, self.head_dim = layers, num_blocks, kv_heads, head_dim
        self.dtype, self.k_scale, self.v_scale = dtype, float(k_scale), float(v_scale)
        self.device = torch.device(device)
        # zero-initialised: slots of a partially filled block are read (then masked) by the kernels
        self._k = torch.zeros(layers, num_blocks, kv_heads, KV_BLOCK, head_dim, dtype=dtype, device=self.device)
        self._v = torch.zeros(layers, num_blocks, kv_heads, head_dim, KV_BLOCK, dtype=dtype, device=self.device)
        self.k = [self._k[i] for i in range(layers)]
        self.v = [self._v[i] for i in range(layers)]
        self.pool = BlockPool(num_blocks)

    @staticmethod
    def bytes_per_block(layers: int, kv_heads: int, head_dim: int, dtype_bytes: int = 2) -> int:
        return 2 * layers * kv_heads * KV_BLOCK * head_dim * dtype_bytes

    @classmethod
    def for_budget(cls, layers, kv_heads, head_dim, device, max_tokens: int, dtype=torch.bfloat16):
        nb = math.ceil(max_tokens / KV_BLOCK) + 1
        return cls(layers, nb, kv_heads, head_dim, device, dtype)

    def nbytes(self) -> int:
        return self._k.numel() * self._k.element_size() * 2


def blocks_needed(n_tokens: int) -> int:
    return math.ceil(n_tokens / KV_BLOCK)
