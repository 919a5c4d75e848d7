"""One-shot all-reduce over IPC-mapped peer buffers for tensor-parallel decode (csrc/kernels/comm.hip).

Why: TP decode issues two all-reduces per layer (after o_proj and down_proj) of B x hidden bf16 --
64 collectives per token for a 32-layer model, each 8 KiB-1 MiB.  At these sizes RCCL's ring
pays per-hop latency on every one of them; the xGMI mesh of an MI355X node is point-to-point
(every GPU pair one hop, 7 links per GPU), so each rank can simply READ all peers' contributions
directly: one barrier + one pass, every link used in parallel.  ("custom one-shot
all-reduce via IPC peer pointers, captured in the hipGraph with the decode step".)

Setup (collective over the TP group, once): every rank allocates an uncached region
(signals + 2 staging buffers), exports its IPC handle, all-gathers the handles (over a CPU/gloo
twin group or the RCCL group itself) and opens the peers' regions.  ``validate()`` compares one
call against ``torch.distributed.all_reduce``; the decoder uses this path only after validation
passed on every rank (agreed through an all-reduce of the verdict), else it keeps RCCL.
Tensors larger than the staging buffer or not a multiple of 8 elements also fall back to RCCL.
"""
from __future__ import annotations

import ctypes
import logging

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

DEFAULT_STAGING_BYTES = 8 << 20   # covers B x hidden bf16 up to B=512 at hidden 8192
DEFAULT_BLOCKS = 32


def _lib():
    from ..ops._native import kernels
    return kernels()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


class OneShotAllReduce:
    def __init__(self, group=None, device=None, staging_bytes: int = DEFAULT_STAGING_BYTES,
                 blocks: int = DEFAULT_BLOCKS, exchange_group=None):
        lib = _lib()
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > 8:
            raise ValueError("one-shot all-reduce supports up to 8 ranks (one xGMI hop)")
        self.device = torch.device(device or "cuda")
        self.staging_bytes = int(staging_bytes)
        self.blocks = min(int(blocks), lib.cfc_ar_max_blocks() - 1)   # the last signal block: keymax
        self.key_rows = lib.cfc_ar_key_rows()
        region = ctypes.c_int64()
        _check(lib.cfc_ar_region_bytes(self.staging_bytes, ctypes.byref(region)), "cfc_ar_region_bytes")
        self.region_bytes = region.value
        hsize = lib.cfc_ar_ipc_handle_size()
        # every step below is collective: a local failure is carried to the peers (None handle /
        # failed open) instead of raised before the exchange, so no rank is left waiting
        self._own, self._opened, self.broken = 0, [], False
        mine = None
        try:
            base = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                _check(lib.cfc_ar_alloc(self.region_bytes, ctypes.byref(base)), "cfc_ar_alloc")
            self._own = base.value
            handle = (ctypes.c_char * hsize)()
            _check(lib.cfc_ar_ipc_handle(ctypes.c_void_p(self._own), handle), "cfc_ar_ipc_handle")
            mine = bytes(handle)
        except RuntimeError as e:
            log.warning("one-shot all-reduce: %s", e)
        handles = [mine]
        if self.world > 1:
            handles = [None] * self.world
            dist.all_gather_object(handles, mine, group=exchange_group or group)
        bases = []
        if any(h is None for h in handles):
            self.broken = True
        else:
            with torch.cuda.device(self.device):
                for r, h in enumerate(handles):
                    if r == self.rank:
                        bases.append(self._own)
                        continue
                    p = ctypes.c_void_p()
                    if lib.cfc_ar_ipc_open(ctypes.create_string_buffer(h, hsize), ctypes.byref(p)) != 0:
                        log.warning("one-shot all-reduce: cannot map rank %d's region", r)
                        self.broken = True
                        break
                    self._opened.append(p.value)
                    bases.append(p.value)
        self._bases = (ctypes.c_void_p * self.world)(*(bases if not self.broken else [0] * self.world))
        self.epochs = torch.zeros(lib.cfc_ar_max_blocks(), dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.enabled = False   # set by validate()

    def supports(self, x: torch.Tensor) -> bool:
        return (self.enabled and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.staging_bytes and x.data_ptr() % 16 == 0)

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        out = torch.empty_like(x) if out is None else out
        rc = _lib().cfc_oneshot_allreduce(x.data_ptr(), out.data_ptr(), x.numel(), self._bases, self.world,
                                          self.rank, self.staging_bytes, self.blocks, self.epochs.data_ptr(),
                                          self.err.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)
        _check(rc, "cfc_oneshot_allreduce")
        return out

    def supports_slabs(self, part: torch.Tensor) -> bool:
        """fp32 split-K slabs [split, M, N] the fused all-reduce + residual + RMSNorm takes."""
        if not self.enabled or part.dim() != 3 or part.dtype != torch.float32 or not part.is_contiguous():
            return False
        _, M, N = part.shape
        return N % 8 == 0 and N <= 8192 and M * N * 4 <= self.staging_bytes and part.data_ptr() % 16 == 0

    def residual_rmsnorm(self, part: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                         out: torch.Tensor | None = None) -> torch.Tensor:
        """The row-parallel projection's epilogue over the TP group in ONE kernel: this rank's fp32
        k-slice slabs are summed, exchanged and added over the ranks in fp32, then residual +=
        bf16(sum) and out = RMSNorm(residual) * norm_w -- the TP = 1 reduce kernel's arithmetic
        (cfc_splitk_residual_rmsnorm) with the projection summed over every rank before its one
        bf16 rounding (comm.hip: oneshot_ar_residual_rmsnorm_kernel)."""
        split, M, N = part.shape
        out = torch.empty(M, N, dtype=torch.bfloat16, device=part.device) if out is None else out
        rc = _lib().cfc_oneshot_ar_residual_rmsnorm(
            part.data_ptr(), split, M, N, residual.data_ptr(), norm_w.data_ptr(), float(eps), out.data_ptr(),
            self._bases, self.world, self.rank, self.staging_bytes, self.blocks, self.epochs.data_ptr(),
            self.err.data_ptr(), torch.cuda.current_stream(part.device).cuda_stream)
        _check(rc, "cfc_oneshot_ar_residual_rmsnorm")
        return out

    def supports_keys(self, n: int) -> bool:
        return self.enabled and 0 < n <= self.key_rows

    def keymax(self, keys: torch.Tensor, out_ids: torch.Tensor) -> torch.Tensor:
        """out_ids[i] = 0xffffffff - low word of max over ranks of keys[i] (int64 keys, int32 out):
        the TP greedy lm_head's (max logit, argmax) reduce (see models.decoder.argmax_keys)."""
        if keys.dtype != torch.int64 or out_ids.dtype != torch.int32 or not keys.is_contiguous():
            raise ValueError("keymax: int64 contiguous keys -> int32 ids")
        rc = _lib().cfc_oneshot_keymax(keys.data_ptr(), out_ids.data_ptr(), keys.numel(), self._bases, self.world,
                                       self.rank, self.staging_bytes, self.epochs.data_ptr(), self.err.data_ptr(),
                                       torch.cuda.current_stream(keys.device).cuda_stream)
        _check(rc, "cfc_oneshot_keymax")
        return out_ids

    def errors(self) -> int:
        return int(self.err.item())

    def validate(self, numels=(8, 4096 * 8, 4096 * 128), seed: int = 0) -> bool:
        """Run the kernel against RCCL on a few sizes; enable only if every rank agrees it matched."""
        ok = not self.broken
        self.enabled = ok
        try:
            for n in numels:
                if not ok or n * 2 > self.staging_bytes:
                    continue
                g = torch.Generator(device=self.device).manual_seed(seed + 7 * self.rank + n)
                x = torch.randn(n, generator=g, device=self.device).to(torch.bfloat16)
                want = x.float()
                if self.world > 1:
                    dist.all_reduce(want, group=self.group)
                got = self(x).float()
                torch.cuda.synchronize(self.device)
                # fp32 sum of bf16 inputs rounded once: within one bf16 ulp of the exact sum
                tol = 2 ** -7 * want.abs().clamp_min(1e-3) + 1e-3
                if self.errors() or not bool(((got - want).abs() <= tol).all()):
                    ok = False
                    break
        except RuntimeError as e:
            log.warning("one-shot all-reduce validation failed: %s", e)
            ok = False
        if self.world > 1:
            flag = torch.tensor([0 if ok else 1], device=self.device, dtype=torch.int32)
            dist.all_reduce(flag, group=self.group)
            ok = int(flag.item()) == 0
        self.enabled = ok
        return ok

    def close(self) -> None:
        lib = _lib()
        for p in self._opened:
            lib.cfc_ar_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        if self._own:
            lib.cfc_ar_free(ctypes.c_void_p(self._own))
            self._own = 0
        self.enabled = False


def maybe_create(group, device, exchange_group=None, **kw) -> OneShotAllReduce | None:
    """Build + validate the one-shot all-reduce for a TP group; None (use RCCL) on any failure.
    ``CFC_CUSTOM_AR=0`` disables it."""
    import os
    if os.environ.get("CFC_CUSTOM_AR", "1") == "0" or group is None or not torch.cuda.is_available():
        return None
    try:
        ar = OneShotAllReduce(group, device, exchange_group=exchange_group, **kw)
    except Exception as e:  # noqa: BLE001 -- IPC unavailable: RCCL path
        log.warning("one-shot all-reduce unavailable (%s); using RCCL", e)
        return None
    if not ar.validate():
        log.warning("one-shot all-reduce failed validation; using RCCL")
        ar.close()
        return None
    return ar
