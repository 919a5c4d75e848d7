"""Plain-PyTorch fp32 reference implementations of every native op.

They define the exact semantics (including the paged KV-cache layouts) that the HIP kernels in
``csrc/kernels`` must reproduce; the numerics tests compare the two, and CPU-only runs (CI,
BASELINE config 1) execute these.  Inputs/outputs use the same dtypes as the kernels (bf16
activations), the math runs in fp32.

These define the semantics the HIP kernels are tested against -- the attention/sampling the
reference's engines run behind local_llm_summarizer.py:107 and llamacpp_summarizer.py:108-113.
"""
from __future__ import annotations

import math

import torch

KV_BLOCK = 32


def v_slot_perm(device=None) -> torch.Tensor:
    """slot index (0..31) of every key inside a KV block in the transposed V cache."""
    k = torch.arange(KV_BLOCK, device=device)
    hi, g, j = k >> 4, (k >> 2) & 3, (k & 3) + 4 * (k >> 4)
    del hi
    return 8 * g + j


def v_groups(v_cache: torch.Tensor) -> torch.Tensor:
    """View of a V cache [nblk, Hkv, D, 32] as its storage order [nblk, Hkv, 4, D, 8]: slot position
    p of row d lives at [..., p // 8, d, p % 8] (common.h kv_v_off) -- the 8 positions of one P.V
    fragment stay 16 contiguous bytes, and one token's column spans 16 cache lines instead of 64."""
    nb, h, d, s = v_cache.shape
    return v_cache.view(nb, h, s // 8, d, 8)


def rmsnorm(x, w, eps, residual=None):
    """Returns (out, new_residual).  With residual: residual <- x + residual; out = norm(residual)."""
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        base = r
    else:
        r = None
        base = x
    xf = base.float()
    out = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return out.to(x.dtype), r


def layernorm(x, gamma, beta, eps, bias=None, residual=None):
    xf = x.float()
    if bias is not None:
        xf = xf + bias.float()
    if residual is not None:
        xf = xf + residual.float()
    out = torch.nn.functional.layer_norm(xf, (xf.shape[-1],), gamma.float(), beta.float(), eps)
    return out.to(x.dtype)


def embed_layernorm(ids, positions, word_emb, pos_emb, type_emb, gamma, beta, eps):
    x = word_emb[ids.long()].float() + pos_emb[positions.long()].float() + type_emb[0].float()
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), gamma.float(), beta.float(), eps).to(word_emb.dtype)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None, llama3_scaling=None) -> torch.Tensor:
    """[max_pos, D/2, 2] fp32 table of (cos, sin) for rotate-half RoPE.

    ``llama3_scaling`` = (factor, low_freq_factor, high_freq_factor, original_max_positions): the
    Llama-3.1 frequency rescaling (long wavelengths divided by ``factor``, short ones kept, a
    smooth blend in between)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if llama3_scaling is not None:
        factor, low, high, orig = llama3_scaling
        wavelen = 2 * math.pi / inv
        scaled = torch.where(wavelen > orig / low, inv / factor, inv)
        smooth = (orig / wavelen - low) / (high - low)
        blend = (1 - smooth) * scaled / factor + smooth * scaled
        medium = ~(wavelen < orig / high) & ~(wavelen > orig / low)
        inv = torch.where(medium, blend, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.stack([ang.cos(), ang.sin()], -1).float().to(device)


def _to_cache(x, cache, scale):
    """Value as stored in a cache of ``cache.dtype`` (fp8 e4m3fn caches hold x / scale, clamped)."""
    if cache.dtype == torch.float8_e4m3fn:
        return (x.float() / scale).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    return x.to(cache.dtype)


def rope_kv_write(qkv, positions, slots, cos_sin, k_cache, v_cache, Hq, Hkv, D, k_scale=1.0, v_scale=1.0):
    """Apply RoPE to q/k of the fused projection, write k/v into the paged cache. Returns q."""
    T = qkv.shape[0]
    x = qkv.float().view(T, Hq + 2 * Hkv, D)
    cs = cos_sin[positions.long()]  # [T, D/2, 2]
    cos, sin = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    half = D // 2

    def rot(t):
        a, b = t[..., :half], t[..., half:]
        return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

    q = rot(x[:, :Hq]).to(qkv.dtype)
    k = rot(x[:, Hq:Hq + Hkv]).to(qkv.dtype)
    v = x[:, Hq + Hkv:].to(qkv.dtype)
    perm = v_slot_perm(qkv.device)
    for t in range(T):
        s = int(slots[t])
        if s < 0:
            continue
        blk, off = divmod(s, KV_BLOCK)
        k_cache[blk, :, off, :] = _to_cache(k[t], k_cache, k_scale)
        p = int(perm[off])
        v_groups(v_cache)[blk, :, p >> 3, :, p & 7] = _to_cache(v[t], v_cache, v_scale)
    return q


def gather_kv(k_cache, v_cache, block_table, n, k_scale=1.0, v_scale=1.0):
    """Contiguous K, V [n, Hkv, D] of one sequence from the paged caches (fp8 caches dequantized
    to fp32 with their scales)."""
    perm = v_slot_perm(k_cache.device)
    nb = (n + KV_BLOCK - 1) // KV_BLOCK
    blocks = block_table[:nb].long()
    k = k_cache[blocks].permute(0, 2, 1, 3).reshape(nb * KV_BLOCK, k_cache.shape[1], k_cache.shape[3])
    vt = v_groups(v_cache)[blocks].permute(0, 1, 3, 2, 4).reshape(nb, v_cache.shape[1], v_cache.shape[2], KV_BLOCK)
    v = vt[..., perm].permute(0, 3, 1, 2).reshape(nb * KV_BLOCK, v_cache.shape[1], v_cache.shape[2])
    if k_cache.dtype == torch.float8_e4m3fn:
        k, v = k.float() * k_scale, v.float() * v_scale
    return k[:n], v[:n]


def _attend(q, k, v, scale, causal_offset=None, window=0):
    """q [m, Hq, D], k/v [n, Hkv, D] -> [m, Hq, D] fp32 (GQA).  ``window`` > 0: sliding-window
    attention as HF Mistral masks it -- a query at position p sees keys k with p - window < k <= p."""
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    kk = k.float().repeat_interleave(G, 1)
    vv = v.float().repeat_interleave(G, 1)
    s = torch.einsum("mhd,nhd->hmn", q.float(), kk) * scale
    m, n = q.shape[0], k.shape[0]
    if causal_offset is not None or window:
        off = causal_offset if causal_offset is not None else n - m
        pos = torch.arange(m, device=q.device)[:, None] + off
        keys = torch.arange(n, device=q.device)[None, :]
        mask = keys > pos
        if window:
            mask = mask | (keys <= pos - window)
        s = s.masked_fill(mask[None], float("-inf"))
    p = torch.softmax(s, -1)
    return torch.einsum("hmn,nhd->mhd", p, vv)


def paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale, window=0, k_scale=1.0, v_scale=1.0):
    out = torch.empty_like(q)
    for b in range(q.shape[0]):
        n = int(ctx_lens[b])
        k, v = gather_kv(k_cache, v_cache, block_tables[b], n, k_scale, v_scale)
        out[b] = _attend(q[b:b + 1], k, v, scale, window=window)[0].to(q.dtype)
    return out


def prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, window=0, k_scale=1.0, v_scale=1.0):
    out = torch.empty_like(q)
    for s in range(len(cu_q) - 1):
        a, b = int(cu_q[s]), int(cu_q[s + 1])
        if b == a:
            continue
        n = int(ctx_lens[s])
        k, v = gather_kv(k_cache, v_cache, block_tables[s], n, k_scale, v_scale)
        out[a:b] = _attend(q[a:b], k, v, scale, causal_offset=n - (b - a), window=window).to(q.dtype)
    return out


def encoder_attention(qkv, cu_seqlens, H, D, scale):
    T = qkv.shape[0]
    x = qkv.view(T, 3, H, D)
    out = torch.empty(T, H, D, dtype=qkv.dtype, device=qkv.device)
    for s in range(len(cu_seqlens) - 1):
        a, b = int(cu_seqlens[s]), int(cu_seqlens[s + 1])
        if b == a:
            continue
        out[a:b] = _attend(x[a:b, 0], x[a:b, 1], x[a:b, 2], scale).to(qkv.dtype)
    return out


def silu_mul(gu):
    F = gu.shape[-1] // 2
    g, u = gu[..., :F].float(), gu[..., F:].float()
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


# gate/up rows of the fused MLP projection are stored interleaved in groups of GU_GROUP rows, so a
# 16-row MFMA n-tile of the decode GEMM holds 8 gate rows and the 8 matching up rows
# (csrc/kernels/dgemm.hip SwiGLU epilogue; the prefill silu_mul and the GEMV read the same layout)
GU_GROUP = 8


def interleave_gate_up(gu_w: torch.Tensor) -> torch.Tensor:
    """[gate; up] rows (2F, H) -> 8-row groups [gate 8t..8t+7; up 8t..8t+7] (F % 8 == 0)."""
    F, G = gu_w.shape[0] // 2, GU_GROUP
    g, u = gu_w[:F].reshape(F // G, G, -1), gu_w[F:].reshape(F // G, G, -1)
    return torch.stack([g, u], 1).reshape(2 * F, -1).contiguous()


def deinterleave_gate_up(w: torch.Tensor) -> torch.Tensor:
    F, G = w.shape[0] // 2, GU_GROUP
    v = w.reshape(F // G, 2, G, -1)
    return torch.cat([v[:, 0].reshape(F, -1), v[:, 1].reshape(F, -1)]).contiguous()


def pack_dgemm_weight(w: torch.Tensor, bn: int) -> torch.Tensor:
    """Row-major W[N, K] -> the decode GEMM's fragment-packed layout for bn-row workgroups,
    [N/bn, K/32, bn/16, 64, 8]: packed[t, kg, w, 16 q + r, j] = W[bn t + 16 w + r, 32 kg + 8 q + j]
    (lane 16q + r of a 16x16x32 MFMA holds B[k = 8q + j][n = r]; one workgroup's slice is contiguous)."""
    N, K = w.shape
    v = w.reshape(N // bn, bn // 16, 16, K // 32, 4, 8)          # t, w, r, kg, q, j
    return v.permute(0, 3, 1, 4, 2, 5).reshape(N // bn, K // 32, bn // 16, 64, 8).contiguous()


def unpack_dgemm_weight(p: torch.Tensor) -> torch.Tensor:
    T, G, NW = p.shape[0], p.shape[1], p.shape[2]
    v = p.reshape(T, G, NW, 4, 16, 8)                              # t, kg, w, q, r, j
    return v.permute(0, 2, 4, 1, 3, 5).reshape(T * NW * 16, G * 32).contiguous()


def silu_mul_interleaved(gu):
    F, G = gu.shape[-1] // 2, GU_GROUP
    v = gu.reshape(*gu.shape[:-1], F // G, 2, G).float()
    return (torch.nn.functional.silu(v[..., 0, :]) * v[..., 1, :]).reshape(*gu.shape[:-1], F).to(gu.dtype)


def bias_gelu(x, bias):
    xf = x.float() + (bias.float() if bias is not None else 0.0)
    return torch.nn.functional.gelu(xf).to(x.dtype)


def sample_greedy(logits):
    """argmax, NaN ranked as -inf (as the HIP sampler): an all-NaN row gives token 0."""
    x = logits.float()
    return torch.argmax(torch.nan_to_num(x, nan=-math.inf, posinf=math.inf, neginf=-math.inf), -1).to(torch.int32)


def truncation_keep(sorted_logits: torch.Tensor, top_p: float, min_p: float) -> int:
    """How many of the (descending) top-k logits survive top-p then min-p (at least one)."""
    v = sorted_logits.float()
    p = torch.softmax(v, -1)
    minp_logit = float(v[0]) + math.log(min_p) if min_p > 0 else -math.inf
    cum, keep = 0.0, 0
    while keep < v.numel():
        if keep > 0 and float(v[keep]) < minp_logit:
            break
        cum += float(p[keep])
        keep += 1
        if cum >= top_p:
            break
    return max(1, keep)


def sample_truncated(logits, temperature, top_k, top_p, min_p, generator=None, cap: int = 256):
    """top-k -> top-p -> min-p -> temperature -> draw (ties ordered by index), one id per row."""
    out = []
    for row in logits.float():
        row = torch.nan_to_num(row, nan=-math.inf, posinf=math.inf, neginf=-math.inf)
        k = min(top_k if top_k > 0 else cap, cap, row.numel())
        vals, idx = torch.sort(row, descending=True, stable=True)
        vals, idx = vals[:k], idx[:k]
        keep = truncation_keep(vals, top_p, min_p)
        if temperature <= 0:
            out.append(int(idx[0]))
            continue
        p = torch.softmax(vals[:keep] / temperature, -1)
        out.append(int(idx[torch.multinomial(p, 1, generator=generator)[0]]))
    return torch.tensor(out, dtype=torch.int32)


def knn_scores(X, Q, xnorm2=None, qnorm2=None):
    dots = Q.float() @ X.float().T
    if xnorm2 is None:
        return dots
    return -(xnorm2.float()[None, :] + qnorm2.float()[:, None] - 2 * dots)


def l2_normalize(x):
    xf = x.float()
    n2 = xf.pow(2).sum(-1)
    inv = torch.where(n2 > 0, torch.rsqrt(n2), torch.zeros_like(n2))
    return (xf * inv[:, None]).to(x.dtype), n2


def pool(hidden, cu_seqlens, mode="mean", normalize=True):
    outs = []
    for s in range(len(cu_seqlens) - 1):
        a, b = int(cu_seqlens[s]), int(cu_seqlens[s + 1])
        h = hidden[a:b].float()
        if b == a:
            v = torch.zeros(hidden.shape[-1], device=hidden.device)
        elif mode == "cls":
            v = h[0]
        else:
            v = h.mean(0)
        if normalize:
            n = v.norm()
            v = v / n if n > 0 else v
        outs.append(v)
    return torch.stack(outs) if outs else torch.empty(0, hidden.shape[-1])


def softmax_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)


def quant_fp8_rows(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 reference of the per-row FP8 quantisation kernel."""
    xf = x.float()
    amax = xf.abs().amax(1, keepdim=True)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    return (xf / s).clamp(-448.0, 448.0).to(torch.float8_e4m3fn), s
