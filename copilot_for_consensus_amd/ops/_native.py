"""ctypes bindings for the in-tree native libraries.

``libcfc_kernels.so`` (HIP, gfx950) and ``libcfc_runtime.so`` (host C++) are loaded from
``copilot_for_consensus_amd/_lib``.  On a machine with a GPU the kernels library is REQUIRED:
``kernels()`` raises if it is missing or fails to load, so no GPU path can silently run on a
PyTorch fallback.  ``build()`` in ``__graft_entry__`` produces both libraries.
"""
from __future__ import annotations

import ctypes
from pathlib import Path
import os
import threading
from ctypes import c_float, c_int, c_int64, c_uint32, c_void_p

from .._build import KERNELS_LIB, RUNTIME_LIB

_lock = threading.Lock()
_kernels = None
_runtime = None

P = c_void_p
I = c_int
F = c_float

# name -> argtypes (every kernel launcher returns int: 0 = ok, <0 = bad arguments, >0 = hipError)
_KERNEL_SIGS = {
    "cfc_rmsnorm": [P, P, P, P, I, I, F, I, P],
    "cfc_layernorm": [P, P, P, P, P, P, P, P, P, P, I, I, F, I, P],
    "cfc_paged_decode_attention": [P, P, P, P, P, I, I, I, I, I, I, I, F, I, P, P, P, P, P],
    "cfc_prefill_attention": [P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, I, P, P],
    "cfc_prefill_rows": [I, I],
    "cfc_encoder_rows": [],
    "cfc_encoder_attention": [P, P, P, P, I, I, I, I, I, F, P, P],
    "cfc_rope_kv_write_part": [P, I, P, P, P, P, P, P, I, I, I, I, I, ctypes.c_float, ctypes.c_float, P],
    "cfc_rope_kv_write": [P, P, P, P, P, P, P, I, I, I, I, I, P],
    "cfc_set_kv_vstore_mode": [I],
    "cfc_set_decode_rope_probe": [I],
    "cfc_v_cache_write_runs": [P, P, I, P, I, I, I, P],
    "cfc_decode_advance_cb": [P, P, I, P, P, P, P, P, P, P, I, P, P, I, I] + [P] * 6 + [I] * 4 + [P] * 4,
    "cfc_rope_kv_write_fp8": [P, P, P, P, P, P, P, I, I, I, I, I, F, F, P],
    "cfc_v_cache_write_runs_fp8": [P, P, I, P, I, I, I, F, P],
    "cfc_paged_decode_attention_fp8": [P, P, P, P, P, I, I, I, I, I, I, I, F, I, F, F, P, P, P, P, P],
    "cfc_paged_decode_rope_attention": [P, P, I, P, P, P, P, P, P, P, I, I, I, I, I, I, I, F, I, I, F, F, P, P, P, P,
                                        P],
    "cfc_prefill_attention_fp8": [P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, I, F, F, P, P],
    "cfc_silu_mul": [P, P, I, I, I, P],
    "cfc_quant_fp8_rows": [P, P, P, I, I, P],
    "cfc_rmsnorm_fp8": [P, P, P, P, P, I, I, F, I, P],
    "cfc_silu_mul_fp8": [P, P, P, I, I, I, P],
    "cfc_bias_gelu": [P, P, P, I, I, P],
    "cfc_embedding": [P, P, P, I, I, P],
    "cfc_sample": [P, I, I, F, c_uint32, P, P, P],
    "cfc_sample_truncated": [P, I, I, F, I, F, F, c_uint32, P, P, P],
    "cfc_decode_advance": [P, P, I, P, P, P, P, P, P, I, P, P, I, I] + [P] * 6 + [I] * 4 + [P] * 4,
    "cfc_knn_scores": [P, P, I, I, I, P, P, P, P],
    "cfc_topk_pass": [P, P, I, I, I, I, P, P, P],
    "cfc_knn_topk": [P, P, I, I, I, I, P, P, P, I, P, P, P],
    "cfc_knn_topk_rows": [],
    "cfc_knn_flat_rows": [I, I],
    "cfc_ivf_topk": [P, P, I, I, I, P, P, P, P, I, P, I, I, P, P, P],
    "cfc_topk_chunk_size": [],
    "cfc_l2_normalize": [P, P, P, I, I, P],
    "cfc_pool": [P, P, P, P, I, I, I, I, P],
    "cfc_splitk_reduce": [P, I, I, I, I, P, I, P],
    "cfc_dgemm": [P, P, I, I, I, I, I, I, I, P, P, I, P],
    "cfc_pgemm": [P, P, P, P, I, I, I, I, I, I, P],
    "cfc_pgemm_ln": [P, P, P, P, P, P, P, I, I, I, F, P],
    "cfc_pgemm_probe": [P, P, P, I, I, I, I, I, I, P],
    "cfc_pgemm_ppp_probe": [P, P, P, I, I, I, I, I, I, I, P],
    "cfc_dgemm_bm": [I],
    "cfc_dgemm_pack": [P, P, I, I, I, P],
    "cfc_dgemm_ablate": [P, P, I, I, I, I, I, I, P, P],
    "cfc_gemv": [P, P, I, I, I, I, P, P, I, P],
    "cfc_gemv_packed": [P, P, I, I, I, I, I, P, P, I, I, I, P, I, P, P, P, F, P],
    "cfc_qgemv": [P, I, I, I, I, P, P, c_int64, c_int64, c_int64, I, P, P, I, P],
    "cfc_dequant_bf16": [P, I, c_int64, P, P],
    "cfc_splitk_residual_rmsnorm": [P, I, I, I, P, P, F, P, P],
    "cfc_ar_region_bytes": [c_int64, P],
    "cfc_ar_alloc": [c_int64, P],
    "cfc_ar_free": [P],
    "cfc_ar_ipc_handle_size": [],
    "cfc_ar_ipc_handle": [P, P],
    "cfc_ar_ipc_open": [P, P],
    "cfc_ar_ipc_close": [P],
    "cfc_ar_max_blocks": [],
    "cfc_oneshot_allreduce": [P, P, c_int64, P, I, I, c_int64, I, P, P, P],
    "cfc_oneshot_keymax": [P, P, I, P, I, I, c_int64, P, P, P],
    "cfc_oneshot_ar_residual_rmsnorm": [P, I, I, I, P, P, F, P, P, I, I, c_int64, I, P, P, P],
    "cfc_ar_key_rows": [],
}

_RUNTIME_SIGS = {
    "cfc_bpe_create": [],
    "cfc_bpe_destroy": [P],
    "cfc_bpe_add_token": [P, ctypes.c_char_p, I, I],
    "cfc_bpe_add_merge": [P, I, I, I, I],
    "cfc_bpe_finalize": [P],
    "cfc_bpe_set_mode": [P, I, I],
    "cfc_bpe_encode_pieces": [P, ctypes.c_char_p, P, I, P, I],
    "cfc_bpe_encode": [P, ctypes.c_char_p, I, P, I],
    "cfc_bpe_decode": [P, P, I, ctypes.c_char_p, I],
    "cfc_bpe_train": [ctypes.c_char_p, I, I, P, P, I],
    "cfc_bpe_encode_batch": [P, ctypes.c_char_p, P, I, I, P, P, I],
    "cfc_wp_encode_batch": [P, ctypes.c_char_p, P, I, I, P, P, I],
    "cfc_wp_create": [I, I, I, I],
    "cfc_wp_destroy": [P],
    "cfc_wp_add_token": [P, ctypes.c_char_p, I, I],
    "cfc_wp_finalize": [P],
    "cfc_wp_encode": [P, ctypes.c_char_p, I, P, I],
    "cfc_blockpool_create": [I],
    "cfc_blockpool_destroy": [P],
    "cfc_blockpool_alloc": [P, I, P],
    "cfc_blockpool_free": [P, P, I],
    "cfc_blockpool_num_free": [P],
    "cfc_mbox_split": [ctypes.c_char_p, c_int64, P, I],
}

_RESTYPES = {
    "cfc_bpe_create": c_void_p, "cfc_wp_create": c_void_p, "cfc_blockpool_create": c_void_p,
    "cfc_mbox_split": c_int64,
}


def _bind(lib, sigs):
    for name, args in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, c_int)
    return lib


def kernels_available() -> bool:
    return KERNELS_LIB.exists()


def kernels():
    """Load libcfc_kernels.so (raises with a build hint if it is missing)."""
    global _kernels
    if _kernels is None:
        with _lock:
            if _kernels is None:
                # CFC_KERNELS_LIB: another build of the library (A/B of two kernel versions on one box)
                lib = Path(os.environ.get("CFC_KERNELS_LIB") or KERNELS_LIB)
                if not lib.exists():
                    raise RuntimeError(
                        f"native HIP kernels not built: {lib} is missing. Run "
                        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950).")
                _kernels = _bind(ctypes.CDLL(str(lib), mode=os.RTLD_LOCAL), _KERNEL_SIGS)
    return _kernels


def runtime():
    """Load libcfc_runtime.so (host C++ runtime: tokenizers, block pool, mbox splitter)."""
    global _runtime
    if _runtime is None:
        with _lock:
            if _runtime is None:
                if not RUNTIME_LIB.exists():
                    from .._build import build_runtime
                    build_runtime(verbose=False)
                _runtime = _bind(ctypes.CDLL(str(RUNTIME_LIB), mode=os.RTLD_LOCAL), _RUNTIME_SIGS)
    return _runtime


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc} ({'bad arguments' if rc < 0 else 'hipError'})")
