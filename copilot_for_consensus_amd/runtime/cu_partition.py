"""Disjoint CU partitions for running one batch's prefill beside another batch's decode.

Decode is HBM-bound (paged attention, weight-streaming GEMMs) and prefill MFMA-bound, but on two
plain streams the prefill GEMMs' workgroups take the CUs the decode kernels stream through and the
pair runs slower than back to back (profiles/overlap_two_streams_r02.log).  On disjoint CU sets
(hipExtStreamCreateWithCUMask, masks in 8-CU blocks -- single-CU interleaves are not honoured,
profiles/cu_mask_overlap_probe_r02.log) decode on half the chip runs 1.41x slower and prefill 1.55x,
so a decode that gives half the CUs to the next batch's prefill and takes the whole chip back
when that prefill is done finishes both sooner than the sequential pair.
"""
from __future__ import annotations

import ctypes

import torch

_hip = None


def _lib():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
    return _hip


def masked_stream(cus: list[int], n_cu: int, device=None) -> torch.cuda.ExternalStream:
    """A HIP stream whose kernels run only on the listed CUs."""
    words = (n_cu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
        err = _lib().hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if err != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {err}")
    return torch.cuda.ExternalStream(s.value, device=device)


def partition_streams(device=None, block: int = 8):
    """(prefill stream, decode stream) on alternating ``block``-CU blocks: half the chip each."""
    n_cu = torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device()
                                            ).multi_processor_count
    pre = [c for c in range(n_cu) if (c // block) % 2 == 0]
    dec = [c for c in range(n_cu) if (c // block) % 2 == 1]
    return masked_stream(pre, n_cu, device), masked_stream(dec, n_cu, device)


def priority_streams(device=None):
    """(prefill stream, decode stream) on the whole chip, the decode stream at the highest
    priority: the dispatcher serves the decode kernels' workgroups first and the prefill GEMMs
    fill what is left (the alternative to disjoint CU sets)."""
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    return torch.cuda.Stream(device=device, priority=lo), torch.cuda.Stream(device=device, priority=hi)
