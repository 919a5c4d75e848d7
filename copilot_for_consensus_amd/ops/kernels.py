"""Python entry points of the native HIP kernels.

Every function takes torch tensors.  CUDA (= HIP on ROCm) tensors go to ``libcfc_kernels.so`` on
PyTorch's current stream (so the calls are hipGraph-capturable); CPU tensors run the fp32
reference in :mod:`.reference` (CI / BASELINE config 1 have no GPU).  There is no silent
fallback for GPU tensors: a missing native library raises.

Reference call sites these ops replace: SentenceTransformer.encode
(sentence_transformer_provider.py:93), the LLM servers' generation (local_llm_summarizer.py:107,
llamacpp_summarizer.py:108-113) and the vector stores' scans (inmemory.py:106-119,
faiss_store.py:214).
"""
from __future__ import annotations

import dataclasses
import math
import os

import torch

from . import reference as ref
from ._native import check, kernels

KV_BLOCK = ref.KV_BLOCK


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _req(t: torch.Tensor, dtype, name: str):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


# ----------------------------------------------------------------------------- norms

def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """out = RMSNorm(x [+ residual]) * w; with ``residual`` it is updated in place to x + residual."""
    if not x.is_cuda:
        o, r = ref.rmsnorm(x, w, eps, residual)
        if residual is not None:
            residual.copy_(r)
        if out is not None:
            out.copy_(o)
            return out
        return o
    _req(x, torch.bfloat16, "x")
    dim = x.shape[-1]
    rows = x.numel() // dim
    out = torch.empty_like(x) if out is None else out
    check(kernels().cfc_rmsnorm(out.data_ptr(), _p(residual), x.data_ptr(), w.data_ptr(), rows, dim, float(eps),
                                1 if residual is not None else 0, _stream(x)), "cfc_rmsnorm")
    return out


def layernorm(x, gamma, beta, eps, bias=None, residual=None, out=None):
    """LN(x [+ bias + residual]) (post-LN BERT sub-layer epilogue)."""
    if not x.is_cuda:
        return ref.layernorm(x, gamma, beta, eps, bias, residual)
    _req(x, torch.bfloat16, "x")
    dim = x.shape[-1]
    rows = x.numel() // dim
    out = torch.empty_like(x) if out is None else out
    mode = 1 if (bias is not None or residual is not None) else 0
    if mode == 1 and (bias is None or residual is None):
        raise ValueError("layernorm: bias and residual must be given together")
    check(kernels().cfc_layernorm(out.data_ptr(), x.data_ptr(), _p(bias), _p(residual), gamma.data_ptr(),
                                  beta.data_ptr(), None, None, None, None, rows, dim, float(eps), mode, _stream(x)),
          "cfc_layernorm")
    return out


def embed_layernorm(ids, positions, word_emb, pos_emb, type_emb, gamma, beta, eps):
    if not word_emb.is_cuda:
        return ref.embed_layernorm(ids, positions, word_emb, pos_emb, type_emb, gamma, beta, eps)
    _req(ids, torch.int32, "ids")
    _req(positions, torch.int32, "positions")
    T, dim = ids.numel(), word_emb.shape[1]
    out = torch.empty(T, dim, dtype=word_emb.dtype, device=word_emb.device)
    check(kernels().cfc_layernorm(out.data_ptr(), word_emb.data_ptr(), None, None, gamma.data_ptr(), beta.data_ptr(),
                                  ids.data_ptr(), positions.data_ptr(), pos_emb.data_ptr(), type_emb.data_ptr(), T,
                                  dim, float(eps), 2, _stream(word_emb)), "cfc_layernorm(embed)")
    return out


# ----------------------------------------------------------------------------- decoder ops

def v_runs(slots) -> "np.ndarray":
    """Host-side run list for :func:`rope_kv_write`'s prefill V path: maximal groups of consecutive
    tokens whose slots fall in one cache block at consecutive offsets -> int32 [R, 4]
    {first token, count, block, first offset}."""
    import numpy as np
    s = np.asarray(slots, dtype=np.int64)
    if s.size == 0:
        return np.zeros((0, 4), np.int32)
    blk, off = s // KV_BLOCK, s % KV_BLOCK
    brk = np.flatnonzero((np.diff(blk) != 0) | (np.diff(off) != 1)) + 1
    starts = np.concatenate([[0], brk])
    ends = np.concatenate([brk, [s.size]])
    return np.stack([starts, ends - starts, blk[starts], off[starts]], 1).astype(np.int32)


def _fp8(cache) -> bool:
    return cache.dtype == torch.float8_e4m3fn


# decode V stores write-through by default: the partial V lines leave L2 during rope_kv, not at its
# end (8.7 -> 7.7 us per decode call in place, bit-identical; profiles/r05_rope_kv_step_prof.txt)
_KV_VSTORE = {"mode": int(os.environ.get("CFC_KV_VSTORE", "1")), "applied": None}


def set_kv_vstore_mode(mode: int) -> None:
    """Decode V-cache store mode of the rope_kv kernels: 0 plain, 1 write-through, 2 nontemporal
    (elementwise.hip cfc_set_kv_vstore_mode).  Applies to launches (and graph captures) after it."""
    check(kernels().cfc_set_kv_vstore_mode(int(mode)), "cfc_set_kv_vstore_mode")
    _KV_VSTORE.update(mode=int(mode), applied=int(mode))


def _apply_vstore():
    if _KV_VSTORE["applied"] != _KV_VSTORE["mode"]:
        set_kv_vstore_mode(_KV_VSTORE["mode"])


def rope_kv_write_part(part, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D, k_scale=1.0, v_scale=1.0):
    """Decode RoPE + K/V write reading the qkv projection's fp32 split-K slabs ``part``
    [split, T, (Hq + 2 Hkv) D] directly (the split-K reduce folded in; same bf16 values)."""
    split, T, N = part.shape
    if not part.is_cuda:
        qkv = part.sum(0).to(torch.bfloat16)
        return rope_kv_write(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D, k_scale=k_scale,
                             v_scale=v_scale)
    if N != (Hq + 2 * Hkv) * D or part.dtype != torch.float32 or not part.is_contiguous():
        raise ValueError(f"rope_kv_write_part: part {tuple(part.shape)} {part.dtype}")
    _req(positions, torch.int32, "positions")
    _req(slots, torch.int32, "slots")
    _apply_vstore()
    q_out = torch.empty(T, Hq, D, dtype=torch.bfloat16, device=part.device)
    check(kernels().cfc_rope_kv_write_part(part.data_ptr(), split, positions.data_ptr(), slots.data_ptr(),
                                           cos_sin.data_ptr(), q_out.data_ptr(), k_cache.data_ptr(),
                                           v_cache.data_ptr(), T, Hq, Hkv, D, int(_fp8(k_cache)), 1.0 / k_scale,
                                           1.0 / v_scale, _stream(part)), "cfc_rope_kv_write_part")
    return q_out


def rope_kv_write(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D, q_out=None, runs=None,
                  k_scale=1.0, v_scale=1.0):
    """RoPE on q/k + paged K/V cache write.  ``runs`` (device int32 [R, 4] from :func:`v_runs`):
    write V per whole cache block (prefill); without it V is written per token (decode).
    float8_e4m3fn caches store K / k_scale and V / v_scale."""
    if not qkv.is_cuda:
        q = ref.rope_kv_write(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D, k_scale, v_scale)
        if q_out is not None:
            q_out.view_as(q).copy_(q)
            return q_out
        return q
    _req(qkv, torch.bfloat16, "qkv")
    _req(positions, torch.int32, "positions")
    _req(slots, torch.int32, "slots")
    T = qkv.shape[0]
    if qkv.shape[1] != (Hq + 2 * Hkv) * D:
        raise ValueError("rope_kv_write: qkv width mismatch")
    if runs is not None:
        _req(runs, torch.int32, "runs")
    q_out = torch.empty(T, Hq, D, dtype=qkv.dtype, device=qkv.device) if q_out is None else q_out
    write_v = 0 if runs is not None else 1
    _apply_vstore()
    if _fp8(k_cache):
        check(kernels().cfc_rope_kv_write_fp8(qkv.data_ptr(), positions.data_ptr(), slots.data_ptr(),
                                              cos_sin.data_ptr(), q_out.data_ptr(), k_cache.data_ptr(),
                                              v_cache.data_ptr(), T, Hq, Hkv, D, write_v, 1.0 / k_scale,
                                              1.0 / v_scale, _stream(qkv)), "cfc_rope_kv_write_fp8")
        if runs is not None:
            check(kernels().cfc_v_cache_write_runs_fp8(qkv.data_ptr(), runs.data_ptr(), runs.shape[0],
                                                       v_cache.data_ptr(), Hq, Hkv, D, 1.0 / v_scale, _stream(qkv)),
                  "cfc_v_cache_write_runs_fp8")
        return q_out
    check(kernels().cfc_rope_kv_write(qkv.data_ptr(), positions.data_ptr(), slots.data_ptr(), cos_sin.data_ptr(),
                                      q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), T, Hq, Hkv, D,
                                      write_v, _stream(qkv)), "cfc_rope_kv_write")
    if runs is not None:
        check(kernels().cfc_v_cache_write_runs(qkv.data_ptr(), runs.data_ptr(), runs.shape[0], v_cache.data_ptr(),
                                               Hq, Hkv, D, _stream(qkv)), "cfc_v_cache_write_runs")
    return q_out


def decode_partitions(max_ctx: int, part_blocks: int) -> int:
    return max(1, math.ceil(math.ceil(max_ctx / KV_BLOCK) / part_blocks))


def paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale, out=None, part_blocks=16,
                           num_partitions=None, workspace=None, window=0, k_scale=1.0, v_scale=1.0, shared_blocks=None):
    """q [B, Hq, D]; caches [nblk, Hkv, 32, D] / [nblk, Hkv, D, 32]; returns [B, Hq, D].

    ``part_blocks`` > 0: split-KV partitions of that many blocks; ``part_blocks`` = -P: P balanced
    partitions of each sequence's own context (what the engine uses).  ``window`` > 0: sliding-window
    attention over the last ``window`` keys (Mistral v0.1).  ``shared_blocks`` (device int32 [1]):
    every sequence's first that-many blocks are read through the caches (the batch's shared prefix
    blocks), the rest nontemporal."""
    if not q.is_cuda:
        return ref.paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale, window=window,
                                          k_scale=k_scale, v_scale=v_scale)
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    _req(block_tables, torch.int32, "block_tables")
    _req(ctx_lens, torch.int32, "ctx_lens")
    max_blocks = block_tables.shape[1]
    if part_blocks < 0:          # -P: every sequence's own blocks split into P balanced ranges
        num_partitions, part_blocks = -part_blocks, 0
    if part_blocks == 0 and not num_partitions:
        raise ValueError("balanced partitioning needs num_partitions (or part_blocks=-P)")
    Pn = num_partitions or math.ceil(max_blocks / part_blocks)
    out = torch.empty_like(q) if out is None else out
    if Pn > 1:
        if workspace is None:
            workspace = torch.empty(B * Hq * Pn * (D + 2), dtype=torch.float32, device=q.device)
        part_o = workspace
        part_ml = workspace[B * Hq * Pn * D:]
    else:
        part_o = part_ml = None
    if _fp8(k_cache):
        check(kernels().cfc_paged_decode_attention_fp8(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                                       block_tables.data_ptr(), ctx_lens.data_ptr(), B, Hq, Hkv, D,
                                                       max_blocks, part_blocks, Pn, float(scale), int(window or 0),
                                                       float(k_scale), float(v_scale), _p(part_o), _p(part_ml),
                                                       out.data_ptr(), _p(shared_blocks), _stream(q)),
              "cfc_paged_decode_attention_fp8")
        return out
    check(kernels().cfc_paged_decode_attention(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                               block_tables.data_ptr(), ctx_lens.data_ptr(), B, Hq, Hkv, D,
                                               max_blocks, part_blocks, Pn, float(scale), int(window or 0), _p(part_o),
                                               _p(part_ml), out.data_ptr(), _p(shared_blocks), _stream(q)),
          "cfc_paged_decode_attention")
    return out


def paged_decode_rope_attention(qkv, positions, slots, cos_sin, k_cache, v_cache, block_tables, ctx_lens, scale,
                                Hq, Hkv, D, part_blocks=-1, workspace=None, window=0, k_scale=1.0, v_scale=1.0,
                                out=None, shared_blocks=None):
    """One decode step's RoPE + K/V cache write + paged attention in ONE kernel
    (attention.hip ``DecRope``): ``qkv`` is the qkv projection output, bf16 [B, (Hq + 2 Hkv) D] or the
    decode GEMM's fp32 split-K slabs [split, B, (Hq + 2 Hkv) D].  Same cache bytes and output as
    :func:`rope_kv_write` (/ ``_part``) followed by :func:`paged_decode_attention`."""
    if not qkv.is_cuda:
        qb = qkv.sum(0).to(torch.bfloat16) if qkv.dim() == 3 else qkv
        q = rope_kv_write(qb, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D, k_scale=k_scale,
                          v_scale=v_scale)
        return paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale, out=out,
                                      part_blocks=part_blocks, workspace=workspace, window=window, k_scale=k_scale,
                                      v_scale=v_scale, shared_blocks=shared_blocks)
    if qkv.dim() == 3:
        split, B, N = qkv.shape
        if qkv.dtype != torch.float32:
            raise ValueError(f"paged_decode_rope_attention: split-K slabs must be fp32, got {qkv.dtype}")
        qkv_p, part_p = None, qkv.data_ptr()
    else:
        (B, N), split = qkv.shape, 0
        _req(qkv, torch.bfloat16, "qkv")
        qkv_p, part_p = qkv.data_ptr(), None
    if not qkv.is_contiguous() or N != (Hq + 2 * Hkv) * D:
        raise ValueError(f"paged_decode_rope_attention: qkv {tuple(qkv.shape)} for Hq={Hq} Hkv={Hkv} D={D}")
    if k_cache.shape[1] != Hkv or k_cache.shape[-1] != D or v_cache.shape[-2] != D:
        raise ValueError("paged_decode_rope_attention: cache shape mismatch")
    _req(positions, torch.int32, "positions")
    _req(slots, torch.int32, "slots")
    _req(block_tables, torch.int32, "block_tables")
    _req(ctx_lens, torch.int32, "ctx_lens")
    if positions.numel() != B or slots.numel() != B or ctx_lens.numel() != B or block_tables.shape[0] != B:
        raise ValueError("paged_decode_rope_attention: per-row tensors must have B entries")
    if cos_sin.dtype != torch.float32 or tuple(cos_sin.shape[1:]) != (D // 2, 2) or not cos_sin.is_contiguous():
        raise ValueError("paged_decode_rope_attention: cos_sin must be fp32 [max_pos, D/2, 2]")
    max_blocks = block_tables.shape[1]
    if part_blocks < 0:
        Pn, part_blocks = -part_blocks, 0
    else:
        Pn = math.ceil(max_blocks / part_blocks)
    out = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=qkv.device) if out is None else out
    if Pn > 1:
        if workspace is None:
            workspace = torch.empty(B * Hq * Pn * (D + 2), dtype=torch.float32, device=qkv.device)
        part_o, part_ml = workspace, workspace[B * Hq * Pn * D:]
    else:
        part_o = part_ml = None
    check(kernels().cfc_paged_decode_rope_attention(
        qkv_p, part_p, split, positions.data_ptr(), slots.data_ptr(), cos_sin.data_ptr(), k_cache.data_ptr(),
        v_cache.data_ptr(), block_tables.data_ptr(), ctx_lens.data_ptr(), B, Hq, Hkv, D, max_blocks, part_blocks, Pn,
        float(scale), int(window or 0), int(_fp8(k_cache)), float(k_scale), float(v_scale), _p(part_o), _p(part_ml),
        out.data_ptr(), _p(shared_blocks), _stream(qkv)), "cfc_paged_decode_rope_attention")
    return out


PREFILL_TILE_ROWS = 128   # query rows per workgroup of the legacy single-head prefill kernels
ENCODER_TILE_ROWS = 256   # query rows per workgroup of the encoder attention kernel (attention.hip ENC_ROWS)


def prefill_rows(Hq: int, Hkv: int) -> int:
    """Query rows per tile the decoder prefill kernel expects: the default GQA-packed kernel takes
    256 / G rows of all G = Hq / Hkv heads of one kv-head per workgroup (attention.hip:
    prefill_gqa_kernel), the legacy kernels 128 rows of one head."""
    lib = kernels() if torch.cuda.is_available() else None
    if lib is None:
        return PREFILL_TILE_ROWS
    return int(lib.cfc_prefill_rows(int(Hq), int(Hkv)))


# context tokens of one group of sequences in the prefill attention's tile order: the grid gives each
# XCD whole kv-heads, and a group's K / V for one kv-head (512 B per token) then stays inside that
# XCD's 4-MB L2 while its tiles run (~3 MB)
PREFILL_GROUP_CTX = int(os.environ.get("CFC_PREFILL_GROUP_CTX", "6144"))


def prefill_tiles(cu_q: list[int], tile: int = PREFILL_TILE_ROWS, ctx_lens: list[int] | None = None):
    """(tile_seq, tile_q0) lists.  With ``ctx_lens``: consecutive sequences in groups of at most
    PREFILL_GROUP_CTX context tokens, the groups in order, each group's tiles heaviest-first (most
    keys to visit under the causal mask) so its long diagonal tiles start first and the grid drains
    evenly.  Against one global heaviest-first order, which interleaves every sequence's K / V in L2
    (scripts/probe_prefill_attn_order.py, profiles/r06_prefill_attn_order*.log): 24 x 700 tokens
    208-213 -> 159-168 us, 6 x 2800 437 -> 415 us on one box and level on another, one 16.8k
    sequence unchanged."""
    tiles = []
    group, acc = 0, 0
    for s in range(len(cu_q) - 1):
        n = cu_q[s + 1] - cu_q[s]
        base = (ctx_lens[s] - n) if ctx_lens is not None else 0
        if ctx_lens is not None:
            if acc and acc + ctx_lens[s] > PREFILL_GROUP_CTX:
                group, acc = group + 1, 0
            acc += ctx_lens[s]
        for r in range(0, n, tile):
            tiles.append((group, base + min(r + tile, n), s, r))
    if ctx_lens is not None:
        tiles.sort(key=lambda x: (x[0], -x[1]))
    return [t[2] for t in tiles], [t[3] for t in tiles]


def prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, tiles=None, out=None, window=0,
                      k_scale=1.0, v_scale=1.0):
    """q [T, Hq, D] (packed varlen); cu_q [S+1] int32; ctx_lens [S] int32 (cached + new);
    ``window`` > 0: sliding-window attention (needs the GQA-packed kernel's G in {1, 2, 4, 8})."""
    if not q.is_cuda:
        return ref.prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, window=window,
                                     k_scale=k_scale, v_scale=v_scale)
    T, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    rows = prefill_rows(Hq, Hkv)
    if tiles is None:
        seqs, q0 = prefill_tiles(cu_q.tolist(), rows, ctx_lens.tolist())
        tiles = (torch.tensor(seqs, dtype=torch.int32, device=q.device),
                 torch.tensor(q0, dtype=torch.int32, device=q.device))
    tile_seq, tile_q0 = tiles
    out = torch.empty_like(q) if out is None else out
    if _fp8(k_cache):
        check(kernels().cfc_prefill_attention_fp8(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                                  block_tables.data_ptr(), cu_q.data_ptr(), ctx_lens.data_ptr(),
                                                  tile_seq.data_ptr(), tile_q0.data_ptr(), tile_seq.numel(), rows, Hq,
                                                  Hkv, D, block_tables.shape[1], float(scale), int(window or 0),
                                                  float(k_scale), float(v_scale), out.data_ptr(), _stream(q)),
              "cfc_prefill_attention_fp8")
        return out
    check(kernels().cfc_prefill_attention(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                          block_tables.data_ptr(), cu_q.data_ptr(), ctx_lens.data_ptr(),
                                          tile_seq.data_ptr(), tile_q0.data_ptr(), tile_seq.numel(), rows, Hq, Hkv, D,
                                          block_tables.shape[1], float(scale), int(window or 0), out.data_ptr(),
                                          _stream(q)),
          "cfc_prefill_attention")
    return out


def encoder_attention(qkv, cu_seqlens, H, D, scale, max_seqlen, tiles=None, out=None):
    if not qkv.is_cuda:
        return ref.encoder_attention(qkv, cu_seqlens, H, D, scale)
    T = qkv.shape[0]
    if tiles is None:
        seqs, q0 = prefill_tiles(cu_seqlens.tolist(), ENCODER_TILE_ROWS)
        tiles = (torch.tensor(seqs, dtype=torch.int32, device=qkv.device),
                 torch.tensor(q0, dtype=torch.int32, device=qkv.device))
    out = torch.empty(T, H, D, dtype=qkv.dtype, device=qkv.device) if out is None else out
    check(kernels().cfc_encoder_attention(qkv.data_ptr(), cu_seqlens.data_ptr(), tiles[0].data_ptr(),
                                          tiles[1].data_ptr(), tiles[0].numel(), ENCODER_TILE_ROWS, H, D,
                                          int(max_seqlen), float(scale), out.data_ptr(), _stream(qkv)),
          "cfc_encoder_attention")
    return out


# ----------------------------------------------------------------------------- decode GEMM helpers

_workspaces: dict = {}
# Superseded workspaces are never freed: a hipGraph captured while one of them was current keeps
# its raw pointer and writes fp32 partials through it on every replay.  Growth at least doubles,
# so the retired buffers add up to less than the live one.
_retired_workspaces: list = []


def _workspace(device, numel: int) -> torch.Tensor:
    """Grow-only fp32 split-K workspace per device (sized during the eager warm-up, so hipGraph
    capture sees a fixed pointer; see _retired_workspaces for why old ones stay allocated)."""
    device = torch.device(device)
    # one per (device, stream): two streams' kernels in flight at once (a prefill beside a decode,
    # the node's consumer threads) must not share their split-K slabs
    key = (device, torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() < numel:
        size = max(numel, 1 << 20, 2 * ws.numel() if ws is not None else 0)
        if ws is not None:
            _retired_workspaces.append(ws)
        ws = torch.empty(size, dtype=torch.float32, device=device)
        _workspaces[key] = ws
    return ws


def _linear_residual_rmsnorm_ref(x, w, residual, norm_w, eps):
    """CPU path: residual += bf16(x @ w^T); returns RMSNorm(residual) * norm_w."""
    y = torch.nn.functional.linear(x, w)
    o, r = ref.rmsnorm(y, norm_w, eps, residual)
    residual.copy_(r)
    return o


def lib_splitk_linear_residual_rmsnorm(x: torch.Tensor, w: torch.Tensor, split: int, residual: torch.Tensor,
                                       norm_w: torch.Tensor, eps: float) -> torch.Tensor:
    """Decode projection as a strided-batched library GEMM over ``split`` K slices (fp32 partials:
    ``split`` x more output tiles for the small-N shapes that leave most CUs idle as one GEMM), then
    one kernel that sums the partials, adds the residual and applies the next RMSNorm:
    residual += bf16(x @ w^T); returns RMSNorm(residual) * norm_w."""
    if not x.is_cuda:
        return _linear_residual_rmsnorm_ref(x, w, residual, norm_w, eps)
    M, Kd = x.shape
    N = w.shape[0]
    if Kd % split:
        raise ValueError(f"K={Kd} not divisible by split={split}")
    Ks = Kd // split
    part = _workspace(x.device, split * M * N)[:split * M * N].view(split, M, N)
    torch.bmm(x.view(M, split, Ks).permute(1, 0, 2), w.view(N, split, Ks).permute(1, 2, 0),
              out_dtype=torch.float32, out=part)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    check(kernels().cfc_splitk_residual_rmsnorm(part.data_ptr(), split, M, N, residual.data_ptr(), norm_w.data_ptr(),
                                                float(eps), out.data_ptr(), _stream(x)), "cfc_splitk_residual_rmsnorm")
    return out


# ----------------------------------------------------------------------------- decode GEMM (dgemm.hip)

DGEMM_BNS = (128, 112, 96, 64)   # W rows per workgroup the kernel is built for
DGEMM_CUS = 256                  # one workgroup per CU
DGEMM_CU_RATE = 25e9             # W bytes/s one workgroup streams (6.4 TB/s over 256 CUs)
DGEMM_PART_RATE = 6e12           # fp32 partial slab traffic, bytes/s
DGEMM_X_RATE = 90e9              # per-CU L2 -> LDS rate of the X re-reads (ablation: X costs ~12 us of gate/up)
# split-K slabs stored write-through (dgemm.hip DG_PART_WT; CFC_DGEMM_SLAB_WT=0 for plain stores): the
# kernel boundary no longer writes back 8-17 MB of dirty partials before the reduce / rope_kv may
# start -- decode 6.48 -> 6.42 s per 128-thread batch, bit-identical (profiles/r05_ab_slab_wt.log)
DGEMM_PART_MODE = 0 if os.environ.get("CFC_DGEMM_SLAB_WT", "1") == "0" else 3


class PackedWeight:
    """A projection weight in the decode GEMM's fragment-packed layout for bn-row workgroups
    (cfc_dgemm_pack): [N/bn][K/32][bn/16][64 lanes][8] bf16 -- every 16-row x 32-k MFMA B fragment
    1 KB contiguous in lane order, each workgroup's W slice one contiguous span.  The prefill GEMM
    (pgemm ping-pong) and the B <= 4 GEMV read it too, so by default it is the ONLY copy
    (DecoderWeights.pack_decode(drop_rowmajor=True))."""

    __slots__ = ("data", "N", "K", "bn")

    def __init__(self, data: torch.Tensor, N: int, K: int, bn: int):
        self.data, self.N, self.K, self.bn = data, N, K, bn

    @property
    def shape(self):
        return (self.N, self.K)

    def nbytes(self) -> int:
        return self.data.numel() * self.data.element_size()


def pack_dgemm_weight(w: torch.Tensor, bn: int | None = None, swiglu: bool = False, m: int = 128) -> PackedWeight:
    """Row-major bf16 W[N, K] -> PackedWeight for bn-row workgroups (default: the tile width the
    decode GEMM picks for an m-row batch of this shape)."""
    N, Kd = w.shape
    bn = bn or dgemm_config(m, N, Kd, swiglu=swiglu)[0]
    if w.is_cuda:
        _req(w, torch.bfloat16, "w")
        out = torch.empty(N * Kd, dtype=torch.bfloat16, device=w.device)
        check(kernels().cfc_dgemm_pack(w.data_ptr(), out.data_ptr(), N, Kd, bn, _stream(w)), "cfc_dgemm_pack")
    else:
        out = ref.pack_dgemm_weight(w, bn).reshape(-1)
    return PackedWeight(out, N, Kd, bn)


def _rowmajor(w):
    if isinstance(w, PackedWeight):
        return ref.unpack_dgemm_weight(w.data.view(w.N // w.bn, w.K // 32, w.bn // 16, 64, 8))
    return w


def dgemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the decode GEMM takes: bf16, contiguous, N % 64 == 0, K % 64 == 0."""
    if isinstance(w, PackedWeight):
        return (x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16 and x.is_contiguous()
                and w.K == x.shape[1] and w.N % 64 == 0 and w.K % 64 == 0 and x.shape[0] >= 1)
    return (x.is_cuda and x.dim() == 2 and w.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.is_contiguous() and w.is_contiguous() and w.shape[1] == x.shape[1]
            and w.shape[0] % 64 == 0 and x.shape[1] % 64 == 0 and x.shape[0] >= 1)


def dgemm_config(M: int, N: int, K: int, swiglu: bool = False, bn: int | None = None) -> tuple[int, int]:
    """(W rows per workgroup, split-K) for one decode projection, from a three-term cost model:
    each workgroup streams its W slice from HBM at a per-CU rate and re-reads its X slice (every
    workgroup reads all BM rows of its K range: X traffic / W traffic = BM / BN) from L2 at a
    per-CU rate, in ceil(blocks / CUs) rounds (a partial second round doubles the time of the CUs
    that run it), plus the fp32 partial slabs written and read back once.  A fused SwiGLU epilogue
    needs split 1.  Rates fitted to bench_dgemm.py sweeps on one MI355X (profiles/dgemm_*.txt)."""
    bm = 64 if M <= 64 else (128 if M <= 128 else 256)
    mt = (M + bm - 1) // bm
    best = None
    for cand in (bn,) if bn else DGEMM_BNS:
        if N % cand:
            continue
        tiles = (N // cand) * mt
        for split in ([1] if swiglu else range(1, K // 64 + 1)):
            blocks = tiles * split
            rounds = -(-blocks // DGEMM_CUS)
            t = rounds * (cand * K * 2 / split / DGEMM_CU_RATE + bm * K * 2 / split / DGEMM_X_RATE)
            if split > 1:
                t += 2 * split * M * N * 4 / DGEMM_PART_RATE
            if best is None or t < best[0] - 1e-12:
                best = (t, cand, split)
    return best[1], best[2]


def dgemm(x: torch.Tensor, w: torch.Tensor, epi: str = "bf16", split: int = 1, bn: int | None = None,
          out: torch.Tensor | None = None, part: torch.Tensor | None = None) -> torch.Tensor:
    """One launch of the decode GEMM.  ``epi``: "bf16" -> out [M, N]; "swiglu" -> out [M, N/2]
    (8-row interleaved gate/up weights); "part" -> fp32 split-K slabs part [split, M, N].
    ``w``: row-major bf16 [N, K] or a PackedWeight (the fast, contiguous-stream layout)."""
    M, Kd = x.shape
    N = w.shape[0]
    if not dgemm_ok(x, w):
        raise ValueError(f"dgemm: x {tuple(x.shape)} {x.dtype} w {tuple(w.shape)} {getattr(w, 'dtype', 'packed')}")
    packed = isinstance(w, PackedWeight)
    wptr = w.data.data_ptr() if packed else w.data_ptr()
    mode = {"part": DGEMM_PART_MODE, "bf16": 1, "swiglu": 2}[epi]
    if packed:
        if bn not in (None, w.bn):
            raise ValueError(f"dgemm: weight packed for bn={w.bn}, asked for bn={bn}")
        bn = w.bn
    bn = bn or dgemm_config(M, N, Kd, swiglu=mode == 2)[0]
    st = _stream(x)
    if mode in (0, 3):
        part = _workspace(x.device, split * M * N)[:split * M * N].view(split, M, N) if part is None else part
        check(kernels().cfc_dgemm(x.data_ptr(), wptr, M, N, Kd, split, mode, bn, int(packed), part.data_ptr(), None,
                                  0, st), "cfc_dgemm")
        return part
    if out is None:
        out = torch.empty(M, N // 2 if mode == 2 else N, dtype=torch.bfloat16, device=x.device)
    check(kernels().cfc_dgemm(x.data_ptr(), wptr, M, N, Kd, 1, mode, bn, int(packed), None, out.data_ptr(),
                              out.stride(0), st), "cfc_dgemm")
    return out


def dgemm_linear(x: torch.Tensor, w: torch.Tensor, split: int | None = None, bn: int | None = None) -> torch.Tensor:
    """bf16 x [M, K] @ w[N, K]^T on the decode GEMM (split-K slabs + reduce when N is small)."""
    if not x.is_cuda:
        return torch.nn.functional.linear(x, _rowmajor(w))
    M, Kd = x.shape
    cbn, csplit = dgemm_config(M, w.shape[0], Kd, bn=getattr(w, "bn", None) or bn)
    bn, split = bn or cbn, split or csplit
    if split == 1:
        return dgemm(x, w, "bf16", bn=bn)
    return splitk_reduce(dgemm(x, w, "part", split, bn=bn))


def dgemm_swiglu(x: torch.Tensor, w_gu_interleaved: torch.Tensor, split: int | None = None,
                 bn: int | None = None) -> torch.Tensor:
    """silu(x @ gate^T) * (x @ up^T) for 8-row interleaved gate/up weights (SwiGLU in the GEMM's
    epilogue; split-K slabs + the SwiGLU reduce when asked for a split, e.g. TP-sharded N)."""
    if not x.is_cuda:
        return ref.silu_mul_interleaved(torch.nn.functional.linear(x, _rowmajor(w_gu_interleaved)))
    M, Kd = x.shape
    N = w_gu_interleaved.shape[0]
    wbn = getattr(w_gu_interleaved, "bn", None) or bn
    if split is None:
        fbn, _ = dgemm_config(M, N, Kd, swiglu=True, bn=wbn)
        pbn, psplit = dgemm_config(M, N, Kd, bn=wbn)
        # split-K + reduce only when the fused grid would leave most CUs idle
        use_split = (N // fbn) * ((M + 255) // 256) < DGEMM_CUS // 2 and psplit > 1
        bn, split = (bn or pbn, psplit) if use_split else (bn or fbn, 1)
    if split == 1:
        return dgemm(x, w_gu_interleaved, "swiglu", bn=bn)
    return splitk_reduce(dgemm(x, w_gu_interleaved, "part", split, bn=bn), swiglu=True)


def dgemm_residual_rmsnorm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor,
                           eps: float, split: int | None = None, bn: int | None = None) -> torch.Tensor:
    """residual += bf16(x @ w^T); returns RMSNorm(residual) * norm_w.  The split-K slabs go straight
    into the residual + RMSNorm reduce (same rounding points as the library split-K path)."""
    if not x.is_cuda:
        return _linear_residual_rmsnorm_ref(x, _rowmajor(w), residual, norm_w, eps)
    M, Kd = x.shape
    cbn, csplit = dgemm_config(M, w.shape[0], Kd, bn=getattr(w, "bn", None) or bn)
    bn, split = bn or cbn, split or csplit
    return splitk_residual_rmsnorm(dgemm(x, w, "part", split, bn=bn), residual, norm_w, eps)


# ------------------------------------------------------------------ prefill / encoder GEMM
PGEMM_EPI = {"bf16": 0, "bias": 1, "bias_gelu": 2, "swiglu": 3, "f32": 4}


def pgemm_ok(x: torch.Tensor, w) -> bool:
    """Shapes the prefill GEMM (pgemm.hip) takes: bf16 contiguous, K % 64 == 0, N % 64 == 0, byte
    spans < 4 GiB (32-bit DMA offsets); ``w`` row-major [N, K] or a PackedWeight."""
    if isinstance(w, PackedWeight):
        return (x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16 and x.is_contiguous() and x.shape[1] == w.K
                and w.K % 64 == 0 and w.N % 64 == 0 and x.shape[0] >= 1 and x.numel() * 2 < 2 ** 32
                and w.N * w.K * 2 < 2 ** 32)
    return (x.is_cuda and x.dim() == 2 and w.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.is_contiguous() and w.is_contiguous() and x.shape[1] == w.shape[1] and x.shape[1] % 64 == 0
            and w.shape[0] % 64 == 0 and x.shape[0] >= 1 and x.numel() * 2 < 2 ** 32 and w.numel() * 2 < 2 ** 32)


PGEMM_VARIANTS = {"ring5": 0, "stage2": 1, "ring4": 2, "pp": 3, "w4": 4, "pps": 5, "ppp": 6}
# row-major W default K loop (a PackedWeight always runs the ping-pong kernel "pp")
PGEMM_VARIANT = os.environ.get("CFC_PGEMM_VARIANT", "stage2")


def pgemm(x: torch.Tensor, w, epi: str = "bf16", bias: torch.Tensor | None = None,
          out: torch.Tensor | None = None, variant: str | None = None) -> torch.Tensor:
    """Hand-written MFMA GEMM for prefill / encoder shapes: x [M, K] @ w[N, K]^T with the following
    elementwise op fused into the epilogue.  ``epi``: "bf16"; "bias" (+ bias[N]); "bias_gelu"
    (gelu_erf(y + bias)); "swiglu" (8-row interleaved gate/up weights -> [M, N/2] =
    silu(gate) * up with the unfused path's bf16 rounding of gate and up).  ``w``: row-major bf16
    [N, K], or the decode GEMM's PackedWeight (one weight copy for prefill and decode: the "w4",
    "pps", "ppp" or, for any other variant, the "pp" kernel).  ``variant``: the K loop ("stage2": 2 LDS
    stages of BK=64; "ring5" / "ring4": BK=32 rings of 5 / 4 LDS slots; "pp": two wave groups
    ping-ponging over half-tile stages; "pps": "pp" with the LDS-staged 16-byte-store epilogue;
    "ppp": "pp" made persistent (one workgroup per CU walking the tiles, the DMA stream running on
    across tile boundaries; packed W, bf16 / SwiGLU epilogues, "pp" otherwise); "w4": four 128x128 waves software-pipelined over a 4-stage ring),
    $CFC_PGEMM_VARIANT when None."""
    mode = PGEMM_EPI[epi]
    packed = isinstance(w, PackedWeight)
    if not x.is_cuda:
        y = torch.nn.functional.linear(x.float(), _rowmajor(w).float())
        if mode in (1, 2):
            y = y + bias.float()
        if mode == 2:
            y = torch.nn.functional.gelu(y)
        if mode == 3:
            return ref.silu_mul_interleaved(y.to(x.dtype))
        if mode == 4:
            return y
        return y.to(x.dtype)
    if not pgemm_ok(x, w):
        raise ValueError(f"pgemm: x {tuple(x.shape)} {x.dtype} w {tuple(w.shape)} {getattr(w, 'dtype', 'packed')}")
    M, Kd = x.shape
    N = w.shape[0]
    if mode in (1, 2):
        _req(bias, torch.bfloat16, "bias")
        if bias.numel() != N:
            raise ValueError(f"pgemm: bias of {bias.numel()} for N = {N}")
    if mode == 4 and (variant or PGEMM_VARIANT) not in ("pp", "pps", "ppp") and not packed:
        variant = "pp"              # the fp32 epilogue is built for the ping-pong kernel only
    if out is None:
        out = torch.empty(M, N // 2 if mode == 3 else N, dtype=torch.float32 if mode == 4 else torch.bfloat16,
                          device=x.device)
    wptr = w.data.data_ptr() if packed else w.data_ptr()
    check(kernels().cfc_pgemm(x.data_ptr(), wptr, bias.data_ptr() if bias is not None else None,
                              out.data_ptr(), M, N, Kd, mode | (PGEMM_VARIANTS[variant or PGEMM_VARIANT] << 4),
                              out.stride(0), w.bn // 16 if packed else 0, _stream(x)), "cfc_pgemm")
    return out


PGEMM_LN_N = (384,)     # output widths the fused GEMM + LayerNorm kernel is built for


def pgemm_ln_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return pgemm_ok(x, w) and w.shape[0] in PGEMM_LN_N


def pgemm_ln(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: torch.Tensor, gamma: torch.Tensor,
             beta: torch.Tensor, eps: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """LayerNorm(x @ w^T + bias + residual) * gamma + beta in one kernel (the post-LN encoder
    sub-layer: attention o-proj and FFN down with their residual and LayerNorm).
    Numerics as the unfused path: projection rounded to bf16, the rest in fp32."""
    if not x.is_cuda:
        y = torch.nn.functional.linear(x.float(), w.float()).to(x.dtype)
        return ref.layernorm(y, gamma, beta, eps, bias, residual)
    if not pgemm_ln_ok(x, w):
        raise ValueError(f"pgemm_ln: x {tuple(x.shape)} w {tuple(w.shape)}")
    M, Kd = x.shape
    N = w.shape[0]
    for t, name in ((bias, "bias"), (gamma, "gamma"), (beta, "beta")):
        _req(t, torch.bfloat16, name)
        if t.numel() != N:
            raise ValueError(f"pgemm_ln: {name} of {t.numel()} for N = {N}")
    _req(residual, torch.bfloat16, "residual")
    if residual.shape != (M, N) or not residual.is_contiguous():
        raise ValueError(f"pgemm_ln: residual {tuple(residual.shape)} for [{M}, {N}]")
    out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device) if out is None else out
    check(kernels().cfc_pgemm_ln(x.data_ptr(), w.data_ptr(), bias.data_ptr(), residual.data_ptr(), gamma.data_ptr(),
                                 beta.data_ptr(), out.data_ptr(), M, N, Kd, float(eps), _stream(x)), "cfc_pgemm_ln")
    return out


GEMV_MAX_M = 4   # decode batches up to this size take the weight-streaming GEMV (gemm.hip: gemv_kernel)


GEMV_TILE_CUS = 256      # the packed GEMV's slab form aims at one workgroup per CU


def gemv_packed_config(N: int, K: int, nw: int, M: int = 1, slab: bool = True) -> tuple[int, int]:
    """(k-slices, waves per workgroup) of the packed GEMV (gemm.hip: gemv_tile_kernel).  Fitted to a
    (split x waves) sweep on the 7B / 13B decode projections (profiles/r04_gemv_grid.jsonl): the
    fastest points put ONE 8-wave workgroup on each CU -- split = the largest with tiles x split
    <= 256 (qkv 7B: 4, down: 8, 13B down: 6) -- within 3% of the best of the grid; a partial
    second round (tiles x split just over 256, e.g. 13B down at 7) costs up to 30%, and fewer
    slabs also keep the consumer's one-workgroup-per-row reduce short.  Each wave keeps >= one
    step of U kg.  In-kernel epilogues (slab=False) take split 1, 16 waves at M = 1 (VGPRs)."""
    u = 2 if M > 2 else (3 if nw >= 7 else 4)
    tiles, kg = N // (16 * nw), K // 32
    if not slab:
        return 1, (16 if M == 1 and kg >= 16 * u else 8 if kg >= 8 * u else 4)
    split = max(1, min(GEMV_TILE_CUS // tiles, kg // (8 * u)))
    return split, (8 if kg // split >= 8 * u else 4)


def gemv_part(x: torch.Tensor, w: "PackedWeight", split: int | None = None, waves: int | None = None,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """x [M <= 4, K] @ W^T over a PackedWeight as fp32 k-slice slabs [split, M, N] (sum over dim 0 =
    the product) in the split-K workspace: the packed GEMV's full-chip form, consumed by the
    slab-reading RoPE / KV write and residual + RMSNorm reduce."""
    M, Kd = x.shape
    N = w.N
    if not isinstance(w, PackedWeight) or w.K != Kd or not (1 <= M <= GEMV_MAX_M) or not x.is_contiguous():
        raise ValueError(f"gemv_part: x {tuple(x.shape)}, packed W [{N}, {w.K}] needed (M <= {GEMV_MAX_M}, contiguous x)")
    cs, cw = gemv_packed_config(N, Kd, w.bn // 16, M)
    split, waves = split or cs, waves or cw
    if not x.is_cuda:
        y = torch.nn.functional.linear(x.float(), _rowmajor(w).float())
        return torch.cat([y[None], torch.zeros(split - 1, M, N)]) if split > 1 else y[None]
    _req(x, torch.bfloat16, "x")
    part = out if out is not None else _workspace(x.device, split * M * N)[:split * M * N].view(split, M, N)
    if part.shape != (split, M, N) or part.dtype != torch.float32 or not part.is_contiguous():
        raise ValueError(f"gemv_part: out {tuple(part.shape)} {part.dtype}, fp32 [{split}, {M}, {N}] needed")
    check(kernels().cfc_gemv_packed(x.data_ptr(), w.data.data_ptr(), M, N, Kd, w.bn // 16, 0, part.data_ptr(), None,
                                    N, split, waves, None, 0, None, None, None, 0.0, _stream(x)), "cfc_gemv_packed")
    return part


def gemv_norm(part: torch.Tensor, res_in: torch.Tensor, res_out: torch.Tensor, norm_w: torch.Tensor, eps: float,
              w: "PackedWeight", epi: str = "slabs", split: int | None = None, waves: int | None = None,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """The packed GEMV with the residual + RMSNorm that produces its input folded into its prologue:
    x = RMSNorm(res_in + sum(part)) * norm_w, exactly as splitk_residual_rmsnorm computes it, then
    x @ W^T.  res_out <- res_in + sum(part) (bf16); res_in is left unchanged (it must be a different
    buffer: the other workgroups still read it).  ``epi``: "slabs" -> fp32 k-slice slabs
    [split, M, N] (in ``out`` or the split-K workspace); "bf16" / "swiglu" -> split 1, in-kernel
    epilogue.  One launch instead of the reduce kernel plus the GEMV (gemm.hip: gemv_tile_kernel)."""
    S_in, M, Kd = part.shape
    N = w.N
    if (not isinstance(w, PackedWeight) or w.K != Kd or not (1 <= M <= GEMV_MAX_M) or part.dtype != torch.float32
            or not (part.is_contiguous() and res_in.is_contiguous() and res_out.is_contiguous())
            or res_in.shape != (M, Kd) or res_out.shape != (M, Kd) or norm_w.numel() != Kd):
        raise ValueError(f"gemv_norm: fp32 slabs {tuple(part.shape)}, residuals [{M}, {Kd}], packed W [{N}, {w.K}] "
                         f"needed (M <= {GEMV_MAX_M}, contiguous)")
    slab = epi == "slabs"
    cs, cw = gemv_packed_config(N, Kd, w.bn // 16, M, slab=slab)
    split = (split or cs) if slab else 1
    # the prologue's registers: 16-wave groups spill (<= 8 waves); otherwise the unfused GEMV's own
    # wave count, so the slabs (and a split-1 epilogue at M > 1) match the unfused path bit for bit
    waves = waves or min(cw, 8)
    if not part.is_cuda:      # splitk_residual_rmsnorm's CPU arithmetic
        x, r = ref.rmsnorm(part.sum(0).to(res_in.dtype), norm_w, eps, res_in)
        res_out.copy_(r)
        if slab:
            return gemv_part(x, w, split)
        return gemv(x, w, epi)
    for t, nm in ((res_in, "res_in"), (res_out, "res_out"), (norm_w, "norm_w")):
        _req(t, torch.bfloat16, nm)
    if res_in.data_ptr() == res_out.data_ptr():
        raise ValueError("gemv_norm: res_out must be a different buffer from res_in")
    if slab:
        if out is None:
            out = _workspace(part.device, split * M * N)[:split * M * N].view(split, M, N)
        yf, yb, mode, ldo = out.data_ptr(), None, 0, N
    else:
        mode = {"bf16": 1, "swiglu": 2}[epi]
        if out is None:
            out = torch.empty(M, N // 2 if epi == "swiglu" else N, dtype=torch.bfloat16, device=part.device)
        yf, yb, ldo = None, out.data_ptr(), out.shape[1]
    check(kernels().cfc_gemv_packed(None, w.data.data_ptr(), M, N, Kd, w.bn // 16, mode, yf, yb, ldo, split, waves,
                                    part.data_ptr(), S_in, res_in.data_ptr(), res_out.data_ptr(), norm_w.data_ptr(),
                                    float(eps), _stream(part)), "cfc_gemv_packed")
    return out


def gemv(x: torch.Tensor, w, epi: str = "bf16", out: torch.Tensor | None = None, waves: int | None = None) -> torch.Tensor:
    """x [M <= 4, K] @ w[N, K]^T on the GEMV kernel.  ``epi``: "bf16" -> bf16 [M, N]; "f32" -> fp32
    [M, N]; "swiglu" -> bf16 [M, N/2] = silu(gate) * up for 8-row interleaved gate/up weights.
    ``w``: row-major bf16 or a PackedWeight (the packed-weight GEMV: one weight copy)."""
    packed = isinstance(w, PackedWeight)
    if not x.is_cuda:
        y = torch.nn.functional.linear(x.float(), _rowmajor(w).float())
        if epi == "swiglu":
            return ref.silu_mul_interleaved(y.to(x.dtype))
        return y if epi == "f32" else y.to(x.dtype)
    _req(x, torch.bfloat16, "x")
    if not packed:
        _req(w, torch.bfloat16, "w")
    M, Kd = x.shape
    N = w.shape[0]
    if w.shape[1] != Kd or not (1 <= M <= GEMV_MAX_M) or not x.is_contiguous() or not (packed or w.is_contiguous()):
        raise ValueError(f"gemv: x {tuple(x.shape)} w {tuple(w.shape)} (M <= {GEMV_MAX_M}, contiguous)")
    mode = {"f32": 0, "bf16": 1, "swiglu": 2}[epi]
    if out is None:
        shape = (M, N // 2) if epi == "swiglu" else (M, N)
        out = torch.empty(shape, dtype=torch.float32 if epi == "f32" else torch.bfloat16, device=x.device)
    yf, yb = (out.data_ptr(), None) if epi == "f32" else (None, out.data_ptr())
    if packed:
        waves = waves or gemv_packed_config(N, Kd, w.bn // 16, M, slab=False)[1]
        check(kernels().cfc_gemv_packed(x.data_ptr(), w.data.data_ptr(), M, N, Kd, w.bn // 16, mode, yf, yb,
                                        out.shape[1], 1, waves, None, 0, None, None, None, 0.0, _stream(x)),
              "cfc_gemv_packed")
    else:
        check(kernels().cfc_gemv(x.data_ptr(), w.data_ptr(), M, N, Kd, mode, yf, yb, out.shape[1], _stream(x)),
              "cfc_gemv")
    return out


def gemv_residual_rmsnorm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor,
                          eps: float) -> torch.Tensor:
    """residual += bf16(x @ w^T) via the GEMV (fp32 out) and the split = 1 residual + RMSNorm reduce;
    returns RMSNorm(residual) * norm_w (same rounding points as lib_splitk_linear_residual_rmsnorm)."""
    if not x.is_cuda:
        return _linear_residual_rmsnorm_ref(x, _rowmajor(w), residual, norm_w, eps)
    M, N = x.shape[0], w.shape[0]
    if isinstance(w, PackedWeight):
        part = gemv_part(x, w)                      # [split, M, N] slabs, summed by the reduce below
    else:
        part = _workspace(x.device, M * N)[:M * N].view(1, M, N)
        gemv(x, w, "f32", out=part[0])
    out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    check(kernels().cfc_splitk_residual_rmsnorm(part.data_ptr(), part.shape[0], M, N, residual.data_ptr(), norm_w.data_ptr(),
                                                float(eps), out.data_ptr(), _stream(x)), "cfc_splitk_residual_rmsnorm")
    return out


def splitk_reduce(part: torch.Tensor, out: torch.Tensor | None = None, swiglu: bool = False) -> torch.Tensor:
    """Sum fp32 slabs [split, M, N] -> bf16 [M, N] (or silu(gate) * up [M, N/2] for interleaved gate/up)."""
    split, M, N = part.shape
    if not part.is_cuda:
        y = part.sum(0).to(torch.bfloat16)
        return ref.silu_mul_interleaved(y) if swiglu else y
    cols = N // 2 if swiglu else N
    out = torch.empty(M, cols, dtype=torch.bfloat16, device=part.device) if out is None else out
    check(kernels().cfc_splitk_reduce(part.data_ptr(), split, M, N, 1 if swiglu else 0, out.data_ptr(), out.shape[1],
                                      _stream(part)), "cfc_splitk_reduce")
    return out


def splitk_residual_rmsnorm(part: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor, eps: float) -> torch.Tensor:
    """residual += bf16(sum of fp32 slabs [split, M, N]); returns RMSNorm(residual) * norm_w."""
    split, M, N = part.shape
    if not part.is_cuda:
        y = part.sum(0).to(residual.dtype)
        o, r = ref.rmsnorm(y, norm_w, eps, residual)
        residual.copy_(r)
        return o
    out = torch.empty(M, N, dtype=torch.bfloat16, device=part.device)
    check(kernels().cfc_splitk_residual_rmsnorm(part.data_ptr(), split, M, N, residual.data_ptr(), norm_w.data_ptr(),
                                                float(eps), out.data_ptr(), _stream(part)), "cfc_splitk_residual_rmsnorm")
    return out


# ----------------------------------------------------------------------------- ggml-quantized weights

QGEMV_TYPES = (8, 12, 14)    # Q8_0, Q4_K, Q6_K: the types the quantized GEMV streams (quant.hip)


def _planar(qtype: int, blocks):
    """ggml blocks [N, nb, size] (numpy uint8) -> the planes of the GPU layout (quant.hip header):
    every plane is row-major [N, ...] so a wave's 16-B loads of one plane are contiguous.
      Q4_K: NIB [N, K/2] (32-weight chunk c, byte i = q[32c+i] | q[32c+16+i] << 4), HDR [N, nb, 16]
            (the ggml fp16 d, fp16 dmin, 12 scale bytes);
      Q6_K: NIB [N, K/2] (low 4 bits, same order), HI [N, K/4] (chunk c: dword h, byte b, bits
            2f..2f+1 = the top 2 bits of weight 16h + 4f + b), SC [N, K/16] int8, D [N, nb] fp16;
      Q8_0: Q [N, K] int8, D [N, K/32] fp16."""
    import numpy as np
    N, nb, _ = blocks.shape
    if qtype == 8:
        return [np.ascontiguousarray(blocks[:, :, 2:34]).reshape(N, -1),
                np.ascontiguousarray(blocks[:, :, 0:2]).reshape(N, -1)]
    if qtype == 12:
        qs = blocks[:, :, 16:144]                                   # ggml: qs[32j + l] = q[64j+l] | q[64j+32+l] << 4
        lo, hi = qs & 0xF, qs >> 4
        q = np.empty((N, nb, 256), np.uint8)
        for j in range(4):
            q[:, :, 64 * j:64 * j + 32] = lo[:, :, 32 * j:32 * j + 32]
            q[:, :, 64 * j + 32:64 * j + 64] = hi[:, :, 32 * j:32 * j + 32]
        q = q.reshape(N, -1, 32)
        nib = (q[:, :, :16] | (q[:, :, 16:] << 4)).reshape(N, -1)
        return [np.ascontiguousarray(nib), np.ascontiguousarray(blocks[:, :, 0:16]).reshape(N, -1)]
    if qtype == 14:
        ql, qh = blocks[:, :, 0:128], blocks[:, :, 128:192]
        q6 = np.empty((N, nb, 256), np.uint8)
        for h in range(2):
            L, H = ql[:, :, 64 * h:64 * h + 64], qh[:, :, 32 * h:32 * h + 32]
            q6[:, :, 128 * h:128 * h + 32] = (L[:, :, :32] & 0xF) | ((H & 3) << 4)
            q6[:, :, 128 * h + 32:128 * h + 64] = (L[:, :, 32:] & 0xF) | (((H >> 2) & 3) << 4)
            q6[:, :, 128 * h + 64:128 * h + 96] = (L[:, :, :32] >> 4) | (((H >> 4) & 3) << 4)
            q6[:, :, 128 * h + 96:128 * h + 128] = (L[:, :, 32:] >> 4) | (((H >> 6) & 3) << 4)
        c = q6.reshape(N, -1, 32)                                   # 32-weight chunks
        nib = ((c[:, :, :16] & 0xF) | ((c[:, :, 16:] & 0xF) << 4)).reshape(N, -1)
        top = (c >> 4).reshape(N, -1, 2, 4, 4)                       # [chunk, half h, f, b]
        hi = (top[:, :, :, 0] | (top[:, :, :, 1] << 2) | (top[:, :, :, 2] << 4) | (top[:, :, :, 3] << 6))
        return [np.ascontiguousarray(nib), np.ascontiguousarray(hi.reshape(N, -1)),
                np.ascontiguousarray(blocks[:, :, 192:208]).reshape(N, -1),
                np.ascontiguousarray(blocks[:, :, 208:210]).reshape(N, -1)]
    raise ValueError(f"ggml type {qtype} has no quantized GEMV layout")


@dataclasses.dataclass
class QWeight:
    """One ggml-quantized weight [N, K] in the planar GPU layout of csrc/kernels/quant.hip (see
    :func:`_planar`): all planes in ONE device buffer ``buf``, plane p at byte ``offs[p]``."""
    qtype: int
    N: int
    K: int
    buf: torch.Tensor
    offs: tuple

    @classmethod
    def _from_planes(cls, qtype, N, K, planes, device) -> "QWeight":
        import numpy as np
        offs, pos = [], 0
        for pl in planes:
            offs.append(pos)
            pos += (pl.nbytes + 255) // 256 * 256                      # every plane 256-B aligned
        host = np.zeros(pos, np.uint8)
        for o, pl in zip(offs, planes):
            host[o:o + pl.nbytes] = np.ascontiguousarray(pl).view(np.uint8).reshape(-1)
        offs += [0] * (3 - len(offs))
        return cls(qtype, N, K, torch.from_numpy(host).to(device), tuple(offs[:4]))

    @classmethod
    def from_raw(cls, raw, qtype: int, N: int, K: int, device, rows=None) -> "QWeight":
        """``raw``: the tensor's ggml blocks (numpy uint8, file layout); ``rows``: optional row
        permutation applied to whole block rows (llama q/k un-permute)."""
        import numpy as np
        from ..runtime import gguf as G
        per, size = G.BLOCK[qtype]
        blocks = np.asarray(raw, dtype=np.uint8).reshape(N, K // per, size)
        if rows is not None:
            blocks = blocks[np.asarray(rows)]
        return cls._from_planes(qtype, N, K, _planar(qtype, blocks), device)

    @classmethod
    def random(cls, qtype: int, N: int, K: int, device, generator=None) -> "QWeight":
        """Random planes with small fixed scales (benchmarks: the bytes, not the values, matter)."""
        import numpy as np
        rng = np.random.default_rng(int(torch.randint(0, 2 ** 31, (1,), generator=generator).item())
                                    if generator is not None and generator.device.type == "cpu" else None)
        nb = K // 256
        half = np.frombuffer(np.float16(0.001).tobytes(), np.uint8)
        if qtype == 8:
            planes = [rng.integers(0, 256, (N, K), dtype=np.uint8), np.tile(half, (N, K // 32))]
        elif qtype == 12:
            hdr = rng.integers(0, 256, (N, nb, 16), dtype=np.uint8)
            hdr[:, :, 0:2] = half
            hdr[:, :, 2:4] = half
            planes = [rng.integers(0, 256, (N, K // 2), dtype=np.uint8), hdr.reshape(N, -1)]
        elif qtype == 14:
            planes = [rng.integers(0, 256, (N, K // 2), dtype=np.uint8),
                      rng.integers(0, 256, (N, K // 4), dtype=np.uint8),
                      rng.integers(0, 256, (N, K // 16), dtype=np.uint8), np.tile(half, (N, nb))]
        else:
            raise ValueError(f"ggml type {qtype} has no quantized GEMV layout")
        return cls._from_planes(qtype, N, K, planes, device)

    @property
    def nbytes(self) -> int:
        from ..runtime import gguf as G
        per, size = G.BLOCK[self.qtype]
        return self.N * self.K // per * size


def llama_cpp_q4km_types(layers: int) -> list[dict]:
    """Per-layer ggml types of llama.cpp's Q4_K_M recipe: Q4_K everywhere except attn_v and
    ffn_down in the "more bits" layers (first and last eighth, every third in between), which
    are Q6_K; the output projection is Q6_K."""
    def more_bits(i):
        return i < layers // 8 or i >= 7 * layers // 8 or (i - layers // 8) % 3 == 2
    out = []
    for i in range(layers):
        t6 = 14 if more_bits(i) else 12
        out.append({"q": 12, "k": 12, "v": t6, "o": 12, "gate": 12, "up": 12, "down": t6})
    return out


def attach_random_quant(weights, recipe: str = "q4_k_m", seed: int = 0):
    """Give random-init DecoderWeights ggml-quantized projection copies (random blocks) so the
    quantized decode path can be benchmarked on a model of the right shape without a file."""
    cfg = weights.cfg
    dev = weights.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    D = cfg.head_dim
    shapes = {"q": (weights.heads * D, cfg.hidden), "k": (weights.kv_heads * D, cfg.hidden),
              "v": (weights.kv_heads * D, cfg.hidden), "o": (cfg.hidden, weights.heads * D),
              "gate": (weights.ffn, cfg.hidden), "up": (weights.ffn, cfg.hidden), "down": (cfg.hidden, weights.ffn)}
    if recipe == "q4_k_m":
        types, head_t = llama_cpp_q4km_types(cfg.layers), 14
    elif recipe == "q8_0":
        types, head_t = [{k: 8 for k in shapes} for _ in range(cfg.layers)], 8
    else:
        raise ValueError(f"unknown quantization recipe {recipe!r}")
    weights.qlayers = [{k: QWeight.random(t[k], *shapes[k], dev, g) for k in shapes} for t in types]
    weights.q_lm_head = QWeight.random(head_t, weights.vocab_shard, cfg.hidden, dev, g)
    return weights


QGEMV_LDS_BYTES = 160 * 1024   # the quantized GEMV stages all of X in LDS (quant.hip: qgemv_launch_rk)


def qgemv_fits(M: int, K: int) -> bool:
    """Whether an M-row X of K columns fits the quantized GEMV's LDS stage (M*K*2 + 16 bytes):
    a 70B-class ffn_down (K = 28672) fits 2 rows, not 3 -- those batches take the bf16 GEMV."""
    return M * K * 2 + 16 <= QGEMV_LDS_BYTES


def qgemv(x: torch.Tensor, qw: QWeight, epi: str = "bf16", qw2: QWeight | None = None,
          out: torch.Tensor | None = None, ldo: int | None = None) -> torch.Tensor:
    """x [M <= 4, K] bf16 @ dequant(qw)^T on the quantized GEMV (quant.hip).  ``epi``: "bf16" ->
    [M, N] bf16; "f32" -> [M, N] fp32; "swiglu" -> bf16 [M, N] = silu(x @ qw^T) * (x @ qw2^T).
    ``out`` may be a column slice of a wider buffer (row stride ``ldo``)."""
    M, Kd = x.shape
    if Kd != qw.K or not (1 <= M <= GEMV_MAX_M):
        raise ValueError(f"qgemv: x {tuple(x.shape)} vs weight K={qw.K} (M <= {GEMV_MAX_M})")
    if epi == "swiglu" and (qw2 is None or qw2.qtype != qw.qtype or qw2.N != qw.N or qw2.K != qw.K):
        raise ValueError("qgemv swiglu: gate and up weights must share type and shape")
    _req(x, torch.bfloat16, "x")
    mode = {"f32": 0, "bf16": 1, "swiglu": 2}[epi]
    if out is None:
        out = torch.empty(M, qw.N, dtype=torch.float32 if epi == "f32" else torch.bfloat16, device=x.device)
        ldo = qw.N
    elif ldo is None:
        ldo = out.stride(0)
    yf, yb = (out.data_ptr(), None) if epi == "f32" else (None, out.data_ptr())
    o = tuple(qw.offs) + (0,) * (4 - len(qw.offs))
    check(kernels().cfc_qgemv(x.data_ptr(), M, qw.N, Kd, qw.qtype, qw.buf.data_ptr(),
                              qw2.buf.data_ptr() if qw2 is not None else None, o[1], o[2], o[3],
                              mode, yf, yb, int(ldo), _stream(x)), "cfc_qgemv")
    return out


def dequant_bf16(raw, qtype: int, shape, device) -> torch.Tensor:
    """ggml blocks (numpy uint8, file layout) -> bf16 tensor of ``shape`` on ``device`` (GPU
    kernel for CUDA devices, numpy reference otherwise)."""
    import numpy as np
    from ..runtime import gguf as G
    device = torch.device(device)
    if device.type != "cuda":
        return torch.from_numpy(G.dequantize(raw, qtype, tuple(shape))).to(torch.bfloat16)
    n = int(np.prod(shape))
    src = torch.from_numpy(np.array(raw, dtype=np.uint8, copy=True).reshape(-1)).to(device)
    out = torch.empty(tuple(shape), dtype=torch.bfloat16, device=device)
    check(kernels().cfc_dequant_bf16(src.data_ptr(), int(qtype), n, out.data_ptr(), _stream(out)),
          "cfc_dequant_bf16")
    return out


def lib_split_for(K: int, N: int) -> int:
    """Split factor for the batched split-K decode GEMM (measured on MI355X at M=128:
    down 4096x14336 -> 8 (29 vs 42 us), o 4096x4096 -> 4); 1 = not worth splitting."""
    if N > 8192:
        return 1
    for s in ((8, 4, 2) if K >= 8192 else (4, 2)):
        if K % s == 0 and K // s >= 512:
            return s
    return 1


def silu_mul(gu, out=None, interleaved: bool = False):
    """silu(gate) * up; ``interleaved``: gate/up in 8-column groups (see ref.interleave_gate_up)."""
    if not gu.is_cuda:
        return ref.silu_mul_interleaved(gu) if interleaved else ref.silu_mul(gu)
    _req(gu, torch.bfloat16, "gu")
    T, F2 = gu.shape
    out = torch.empty(T, F2 // 2, dtype=gu.dtype, device=gu.device) if out is None else out
    for t0 in range(0, T, 65535):
        t1 = min(T, t0 + 65535)
        check(kernels().cfc_silu_mul(out[t0:t1].data_ptr(), gu[t0:t1].data_ptr(), t1 - t0, F2 // 2,
                                     1 if interleaved else 0, _stream(gu)), "cfc_silu_mul")
    return out


FP8_MAX = 448.0   # OCP e4m3fn


def quant_fp8_rows(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-row FP8 (e4m3fn) quantisation: (x8 [M, K], scale [M, 1] f32) with x ~= x8 * scale."""
    if not x.is_cuda:
        return ref.quant_fp8_rows(x)
    _req(x, torch.bfloat16, "x")
    M, Kd = x.shape
    out = torch.empty(M, Kd, dtype=torch.float8_e4m3fn, device=x.device)
    scale = torch.empty(M, 1, dtype=torch.float32, device=x.device)
    check(kernels().cfc_quant_fp8_rows(out.data_ptr(), scale.data_ptr(), x.data_ptr(), M, Kd, _stream(x)),
          "cfc_quant_fp8_rows")
    return out, scale


def quant_fp8_weight(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-output-channel FP8 weight: (w8 [N, K] e4m3fn, scale [1, N] f32), done once at load."""
    s = (w.float().abs().amax(1, keepdim=True) / FP8_MAX).clamp_min(1e-12)
    return (w.float() / s).to(torch.float8_e4m3fn), s.t().contiguous()


def rmsnorm_fp8(x: torch.Tensor, w: torch.Tensor, eps: float,
                residual: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """quant_fp8_rows(rmsnorm(x, w, eps, residual)) in one kernel: (x8 [M, K] e4m3fn, scale [M, 1])."""
    if not x.is_cuda:
        return ref.quant_fp8_rows(rmsnorm(x, w, eps, residual))
    _req(x, torch.bfloat16, "x")
    dim = x.shape[-1]
    rows = x.numel() // dim
    out = torch.empty(rows, dim, dtype=torch.float8_e4m3fn, device=x.device)
    scale = torch.empty(rows, 1, dtype=torch.float32, device=x.device)
    check(kernels().cfc_rmsnorm_fp8(out.data_ptr(), scale.data_ptr(), _p(residual), x.data_ptr(), w.data_ptr(), rows,
                                    dim, float(eps), 1 if residual is not None else 0, _stream(x)), "cfc_rmsnorm_fp8")
    return out, scale


def silu_mul_fp8(gu: torch.Tensor, interleaved: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """quant_fp8_rows(silu_mul(gu)) in one kernel: (a8 [T, F] e4m3fn, scale [T, 1])."""
    if not gu.is_cuda or gu.shape[1] // 2 > 32768:
        return quant_fp8_rows(silu_mul(gu, interleaved=interleaved))
    _req(gu, torch.bfloat16, "gu")
    T, F2 = gu.shape
    out = torch.empty(T, F2 // 2, dtype=torch.float8_e4m3fn, device=gu.device)
    scale = torch.empty(T, 1, dtype=torch.float32, device=gu.device)
    check(kernels().cfc_silu_mul_fp8(out.data_ptr(), scale.data_ptr(), gu.data_ptr(), T, F2 // 2,
                                     1 if interleaved else 0, _stream(gu)), "cfc_silu_mul_fp8")
    return out, scale


def linear_fp8(x, w8: torch.Tensor, w_scale: torch.Tensor) -> torch.Tensor:
    """W8A8 FP8 linear on the MFMA FP8 path (hipBLASLt through torch._scaled_mm): per-token
    activation scales x per-output-channel weight scales, bf16 out.  ~1.8-1.9x the bf16 GEMM rate
    at prefill shapes on gfx950 (profiles/fp8_gemm_probe_r02.log).  ``x`` is a bf16 activation
    (quantised here) or an already-quantised (x8, scale) pair from rmsnorm_fp8 / silu_mul_fp8."""
    x8, sx = x if isinstance(x, tuple) else (ref.quant_fp8_rows(x) if not x.is_cuda else quant_fp8_rows(x))
    if not x8.is_cuda:
        return ((x8.float() * sx) @ (w8.float() * w_scale.t()).T).to(torch.bfloat16)
    return torch._scaled_mm(x8, w8.t(), scale_a=sx, scale_b=w_scale, out_dtype=torch.bfloat16)


def bias_gelu(x, bias, out=None):
    if not x.is_cuda:
        return ref.bias_gelu(x, bias)
    _req(x, torch.bfloat16, "x")
    T, F = x.shape
    out = torch.empty_like(x) if out is None else out
    check(kernels().cfc_bias_gelu(out.data_ptr(), x.data_ptr(), _p(bias), T, F, _stream(x)), "cfc_bias_gelu")
    return out


def embedding(table, ids, out=None):
    if not table.is_cuda:
        return table[ids.long()]
    _req(ids, torch.int32, "ids")
    T, dim = ids.numel(), table.shape[1]
    out = torch.empty(T, dim, dtype=table.dtype, device=table.device) if out is None else out
    check(kernels().cfc_embedding(out.data_ptr(), table.data_ptr(), ids.data_ptr(), T, dim, _stream(table)),
          "cfc_embedding")
    return out


@dataclasses.dataclass(frozen=True)
class SamplingParams:
    """Decoding controls.  ``temperature <= 0`` is greedy (the truncation knobs are then moot);
    otherwise top-k -> top-p -> min-p cut on the raw logits, then temperature, as llama.cpp's
    default sampler chain (the reference's /completion call sets only temperature 0.7 and runs
    with the server defaults top_k 40, top_p 0.95, min_p 0.05)."""
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    min_p: float = 0.0

    @classmethod
    def of(cls, t) -> "SamplingParams":
        return t if isinstance(t, SamplingParams) else cls(float(t))

    @property
    def truncated(self) -> bool:
        return self.temperature > 0 and (self.top_k > 0 or self.top_p < 1.0 or self.min_p > 0.0)


def sample(logits, out_ids, temperature=0.0, seed=0, step=None):
    """One token per row into out_ids (int32): greedy, Gumbel-max over the full softmax, or the
    truncated chain of :class:`SamplingParams` (``temperature`` may be a float or SamplingParams)."""
    sp = SamplingParams.of(temperature)
    if not logits.is_cuda:
        if sp.temperature <= 0:
            out_ids.copy_(ref.sample_greedy(logits))
        else:
            g = torch.Generator().manual_seed(int(seed) + int(step[0]) if step is not None else int(seed))
            if sp.truncated:
                out_ids.copy_(ref.sample_truncated(logits, sp.temperature, sp.top_k, sp.top_p, sp.min_p, g))
            else:
                p = torch.softmax(logits.float() / sp.temperature, -1)
                out_ids.copy_(torch.multinomial(p, 1, generator=g)[:, 0].to(torch.int32))
        return out_ids
    _req(logits, torch.bfloat16, "logits")
    B, V = logits.shape
    if sp.truncated:
        check(kernels().cfc_sample_truncated(logits.data_ptr(), B, V, sp.temperature, int(sp.top_k), float(sp.top_p),
                                             float(sp.min_p), int(seed) & 0xFFFFFFFF, _p(step), out_ids.data_ptr(),
                                             _stream(logits)), "cfc_sample_truncated")
        return out_ids
    check(kernels().cfc_sample(logits.data_ptr(), B, V, float(sp.temperature), int(seed) & 0xFFFFFFFF, _p(step),
                               out_ids.data_ptr(), _stream(logits)), "cfc_sample")
    return out_ids


def _stop_args(stop_state):
    """ctypes tail of the decode-advance calls: the stop-string tables (runtime/stops.py) or nulls."""
    if stop_state is None:
        return [None] * 6 + [0, 0, 0, 0] + [None] * 3
    a = stop_state.kernel_args()
    return [a["head"].data_ptr(), a["tail"].data_ptr(), a["tlen"].data_ptr(), a["contains"].data_ptr(),
            a["stops"].data_ptr(), a["stop_lens"].data_ptr(), a["n_str"], a["L"], a["H"], a["strip"],
            a["win"].data_ptr(), a["wlen"].data_ptr(), a["keep"].data_ptr()]


def decode_advance_cb(next_ids, tokens, gen, limit, input_ids, positions, ctx_lens, slots, block_tables, done,
                      stop_ids, stop_state=None):
    """Continuous-batching bookkeeping after a decode step: per-slot token count / limit; finished
    and empty slots (done = 1) are frozen (graph-capturable, no host sync).  ``stop_state``
    (runtime.stops.StopState): slots also finish when their text reaches a stop string."""
    B = next_ids.numel()
    cap = tokens.shape[1]
    if not next_ids.is_cuda:
        act = done == 0
        if not bool(act.any()):
            return
        idx = act.nonzero().flatten()
        g = gen[idx].long()
        rec = g < cap
        tokens[idx[rec], g[rec]] = next_ids[idx[rec]].to(tokens.dtype)
        gen[idx] += 1
        fin = gen[idx] >= limit[idx]
        if stop_ids.numel():
            fin |= torch.isin(next_ids[idx], stop_ids)
        if stop_state is not None:
            for k, b in enumerate(idx.tolist()):
                if stop_state.host_feed(b, int(next_ids[b])):
                    fin[k] = True
                    stop_state.keep[b] = int(gen[b])
        done[idx] = fin.to(done.dtype)
        go = idx[~fin]
        input_ids[go] = next_ids[go]
        positions[go] += 1
        ctx_lens[go] = positions[go] + 1
        pos = positions[go].long()
        slots[go] = (block_tables[go, pos // KV_BLOCK] * KV_BLOCK + pos % KV_BLOCK).to(slots.dtype)
        return
    check(kernels().cfc_decode_advance_cb(next_ids.data_ptr(), tokens.data_ptr(), cap, gen.data_ptr(),
                                          limit.data_ptr(), input_ids.data_ptr(), positions.data_ptr(),
                                          ctx_lens.data_ptr(), slots.data_ptr(), block_tables.data_ptr(),
                                          block_tables.shape[1], done.data_ptr(),
                                          _p(stop_ids) if stop_ids.numel() else None, stop_ids.numel(), B,
                                          *_stop_args(stop_state), _stream(next_ids)), "cfc_decode_advance_cb")


def decode_advance(next_ids, tokens, step, input_ids, positions, ctx_lens, slots, block_tables, done, stop_ids,
                   stop_state=None):
    """Device-side bookkeeping after each decode step (graph-capturable, no host sync).
    ``stop_state``: a slot whose text reaches a stop string is marked done and keeps
    ``stop_state.keep[b]`` tokens."""
    B = next_ids.numel()
    max_new = tokens.shape[1]
    if not next_ids.is_cuda:
        st = int(step[0])
        if stop_state is not None:
            for b in range(B):
                if not int(done[b]) and stop_state.host_feed(b, int(next_ids[b])):
                    done[b] = 1
                    stop_state.keep[b] = st + 1
        if st < max_new:
            tokens[:, st] = next_ids
        input_ids.copy_(next_ids)
        positions += 1
        ctx_lens.copy_(positions + 1)
        pos = positions.long()
        slots.copy_(block_tables[torch.arange(B), pos // KV_BLOCK] * KV_BLOCK + pos % KV_BLOCK)
        if stop_ids.numel():
            done |= torch.isin(next_ids, stop_ids).to(done.dtype)
        step += 1
        return
    check(kernels().cfc_decode_advance(next_ids.data_ptr(), tokens.data_ptr(), max_new, step.data_ptr(),
                                       input_ids.data_ptr(), positions.data_ptr(), ctx_lens.data_ptr(),
                                       slots.data_ptr(), block_tables.data_ptr(), block_tables.shape[1],
                                       done.data_ptr(), _p(stop_ids) if stop_ids.numel() else None,
                                       stop_ids.numel(), B, *_stop_args(stop_state), _stream(next_ids)),
          "cfc_decode_advance")


# ----------------------------------------------------------------------------- vector search

def knn_scores(X, Q, xnorm2=None, qnorm2=None, out=None):
    """scores [nq, N] fp32 for nq <= 16 queries (dot, or -squared-L2 when norms are given)."""
    if not X.is_cuda:
        return ref.knn_scores(X, Q, xnorm2, qnorm2)
    N, dim = X.shape
    nq = Q.shape[0]
    out = torch.empty(nq, N, dtype=torch.float32, device=X.device) if out is None else out
    check(kernels().cfc_knn_scores(X.data_ptr(), Q.data_ptr(), N, nq, dim, _p(xnorm2), _p(qnorm2), out.data_ptr(),
                                   _stream(X)), "cfc_knn_scores")
    return out


def topk(scores: torch.Tensor, k: int, ids: torch.Tensor | None = None):
    """Exact top-k per row of ``scores`` [nq, n]; returns (values, ids) sorted descending."""
    nq, n = scores.shape
    k_eff = min(k, n)
    if not scores.is_cuda:
        v, i = torch.topk(scores.float(), k_eff, dim=1)
        if ids is not None:
            i = torch.gather(ids, 1, i)
        return v, i
    lib = kernels()
    chunk = lib.cfc_topk_chunk_size()
    cur_v, cur_i, cur_n = scores.contiguous(), ids, n
    while True:
        nch = math.ceil(cur_n / chunk)
        ov = torch.empty(nq, nch * k_eff, dtype=torch.float32, device=scores.device)
        oi = torch.empty(nq, nch * k_eff, dtype=torch.int64, device=scores.device)
        check(lib.cfc_topk_pass(cur_v.data_ptr(), _p(cur_i), nq, cur_n, cur_v.shape[1], k_eff, ov.data_ptr(),
                                oi.data_ptr(), _stream(scores)), "cfc_topk_pass")
        cur_v, cur_i, cur_n = ov, oi, nch * k_eff
        if nch == 1:
            break
    order = torch.argsort(cur_v, dim=1, descending=True, stable=True)
    return torch.gather(cur_v, 1, order), torch.gather(cur_i, 1, order)


def _merge_candidates(cv: torch.Tensor, ci: torch.Tensor, k: int):
    """Exact top-k of per-chunk candidates [nq, m] (values, row ids) -> sorted [nq, k]."""
    return topk(cv, k, ci)


def knn_topk(X, Q, k: int, xnorm2=None, qnorm2=None, alive=None, row_lo: int = 0, N: int | None = None):
    """Fused flat scan + top-k (knn.hip knn_topk_kernel) over rows [row_lo, N) of X for <= 16
    queries: (scores [nq, k] descending, row indices [nq, k]); the [nq, N] scores never reach HBM."""
    N = X.shape[0] if N is None else N
    nq = Q.shape[0]
    if not X.is_cuda:
        sc = ref.knn_scores(X[row_lo:N], Q, None if xnorm2 is None else xnorm2[row_lo:N], qnorm2)
        if alive is not None:
            sc = sc.masked_fill(~alive[row_lo:N].bool()[None], float("-inf"))
        v, i = torch.topk(sc.float(), min(k, N - row_lo), dim=1)
        return v, i + row_lo
    R = kernels().cfc_knn_flat_rows(nq, k)
    nch = -(-(N - row_lo) // R)
    cv = torch.empty(nq, nch * k, dtype=torch.float32, device=X.device)
    ci = torch.empty(nq, nch * k, dtype=torch.int64, device=X.device)
    check(kernels().cfc_knn_topk(X.data_ptr(), Q.data_ptr(), N, row_lo, nq, X.shape[1], _p(xnorm2), _p(qnorm2),
                                 _p(alive), k, cv.data_ptr(), ci.data_ptr(), _stream(X)), "cfc_knn_topk")
    return _merge_candidates(cv, ci, min(k, N - row_lo))


def ivf_topk(X, Q, probe: torch.Tensor, list_off: torch.Tensor, maxc: int, k: int, xnorm2=None, qnorm2=None,
             alive=None):
    """IVF scan of the probed lists, one launch for every (query, probe, chunk): candidates
    [nq, nprobe * maxc * k] (values, row indices; -inf / -1 padding).  ``probe`` int32 [nq, nprobe]
    list ids, ``list_off`` int64 [nlist + 1] row offsets on the device."""
    nq, nprobe = probe.shape
    cv = torch.empty(nq, nprobe * maxc * k, dtype=torch.float32, device=X.device)
    ci = torch.empty(nq, nprobe * maxc * k, dtype=torch.int64, device=X.device)
    check(kernels().cfc_ivf_topk(X.data_ptr(), Q.data_ptr(), X.shape[0], nq, X.shape[1], _p(xnorm2), _p(qnorm2),
                                 _p(alive), probe.data_ptr(), nprobe, list_off.data_ptr(), maxc, k, cv.data_ptr(),
                                 ci.data_ptr(), _stream(X)), "cfc_ivf_topk")
    return cv, ci


def l2_normalize(x, out=None, norms2=None):
    if not x.is_cuda:
        o, n2 = ref.l2_normalize(x)
        if norms2 is not None:
            norms2.copy_(n2)
        return o
    rows, dim = x.shape
    out = torch.empty_like(x) if out is None else out
    check(kernels().cfc_l2_normalize(out.data_ptr(), x.data_ptr(), _p(norms2), rows, dim, _stream(x)),
          "cfc_l2_normalize")
    return out


def pool(hidden, cu_seqlens, mode="mean", normalize=True):
    """[nseq, dim] fp32 sentence embeddings from packed token states."""
    if not hidden.is_cuda:
        return ref.pool(hidden, cu_seqlens, mode, normalize)
    nseq = cu_seqlens.numel() - 1
    dim = hidden.shape[-1]
    out = torch.empty(nseq, dim, dtype=torch.float32, device=hidden.device)
    check(kernels().cfc_pool(out.data_ptr(), None, hidden.data_ptr(), cu_seqlens.data_ptr(), nseq, dim,
                             1 if mode == "cls" else 0, 1 if normalize else 0, _stream(hidden)), "cfc_pool")
    return out
