"""Tensor parallelism for the decoder (Megatron-style), RCCL all-reduce over xGMI.

Sharding (per rank r of T):
  * fused QKV [(Hq+2Hkv)*D, H]: rows of q heads [r*Hq/T, ...), k heads and v heads likewise, each
    rank's three slices re-fused -> the RoPE/KV-write kernel and the KV cache hold only local
    kv heads (KV cache memory / T);
  * O [H, Hq*D]: column slice of the local heads -> partial sums, one all-reduce;
  * gate|up [2F, H]: gate rows and up rows of the local F/T slice, re-fused;
  * down [H, F]: column slice -> partial sums, one all-reduce;
  * lm_head [V, H]: vocab rows [r*V/T, ...) -> all-gather of logits;
  * embeddings / norms replicated.
Two all-reduces of B x H x 2 bytes per layer at decode (64 KiB at B=8) are latency-bound; the
collectives run inside the captured decode hipGraph so there is no host launch per call.
"""
from __future__ import annotations

import torch

from ..models.decoder import DecoderConfig, DecoderWeights


def shard_weights(full: DecoderWeights, tp_rank: int, tp_size: int, device=None) -> DecoderWeights:
    """Slice an unsharded model into rank ``tp_rank``'s TP shard."""
    cfg: DecoderConfig = full.cfg
    dev = device or full.device
    w = DecoderWeights(cfg, dev, tp_rank, tp_size)
    D, Hq, Hkv, F = cfg.head_dim, cfg.heads, cfg.kv_heads, cfg.ffn
    hq, hk, f = Hq // tp_size, Hkv // tp_size, F // tp_size

    def rows(t, start, n):
        return t[start:start + n]

    from ..ops.reference import deinterleave_gate_up
    for layer in full.layers:
        qkv = layer["qkv"]
        q = rows(qkv, tp_rank * hq * D, hq * D)
        k = rows(qkv, Hq * D + tp_rank * hk * D, hk * D)
        v = rows(qkv, (Hq + Hkv) * D + tp_rank * hk * D, hk * D)
        gu = deinterleave_gate_up(layer["gate_up"]) if full.gate_up_interleaved else layer["gate_up"]
        g = rows(gu, tp_rank * f, f)
        u = rows(gu, F + tp_rank * f, f)
        w.layers.append({
            "attn_norm": layer["attn_norm"].to(dev),
            "qkv": torch.cat([q, k, v]).contiguous().to(dev),
            "o": layer["o"][:, tp_rank * hq * D:(tp_rank + 1) * hq * D].contiguous().to(dev),
            "mlp_norm": layer["mlp_norm"].to(dev),
            "gate_up": torch.cat([g, u]).contiguous().to(dev),
            "down": layer["down"][:, tp_rank * f:(tp_rank + 1) * f].contiguous().to(dev),
        })
    w.embed = full.embed.to(dev)
    w.final_norm = full.final_norm.to(dev)
    vs = cfg.vocab_size // tp_size
    w.lm_head = full.lm_head[tp_rank * vs:(tp_rank + 1) * vs].contiguous().to(dev)
    return w.finalize()


def unshard_weights(shards: list[DecoderWeights], device=None) -> DecoderWeights:
    """The inverse of :func:`shard_weights`: one unsharded model from the TP shards of ranks 0..T-1
    (e.g. the reference of a TP run whose shards were generated per rank by random_sharded).  Each
    shard's layer tensors are released as they are consumed, so peak memory is the full model plus
    one layer."""
    from ..ops.reference import deinterleave_gate_up
    s0 = shards[0]
    cfg: DecoderConfig = s0.cfg
    dev = device or s0.device
    T, D = len(shards), cfg.head_dim
    w = DecoderWeights(cfg, dev)
    for i in range(cfg.layers):
        parts = [sh.rowmajor_layer(i) for sh in shards]
        hq, hk = shards[0].heads, shards[0].kv_heads
        qkv = [p["qkv"].to(dev) for p in parts]
        gus = [deinterleave_gate_up(p["gate_up"].to(dev)) if sh.gate_up_interleaved else p["gate_up"].to(dev)
               for p, sh in zip(parts, shards)]
        f = gus[0].shape[0] // 2
        w.layers.append({
            "attn_norm": parts[0]["attn_norm"].to(dev),
            "qkv": torch.cat([t[:hq * D] for t in qkv] + [t[hq * D:(hq + hk) * D] for t in qkv]
                             + [t[(hq + hk) * D:] for t in qkv]).contiguous(),
            "o": torch.cat([p["o"].to(dev) for p in parts], 1).contiguous(),
            "mlp_norm": parts[0]["mlp_norm"].to(dev),
            "gate_up": torch.cat([g[:f] for g in gus] + [g[f:] for g in gus]).contiguous(),
            "down": torch.cat([p["down"].to(dev) for p in parts], 1).contiguous(),
        })
        del parts, qkv, gus
        for sh in shards:                      # free the consumed layer of every shard
            sh.layers[i] = {}
            if sh.packed is not None:
                sh.packed[i] = {}
    w.embed = s0.embed.to(dev)
    w.final_norm = s0.final_norm.to(dev)
    w.lm_head = torch.cat([sh.lm_head.to(dev) for sh in shards]).contiguous()
    return w.finalize()


def random_sharded(cfg: DecoderConfig, device, seed: int, tp_rank: int, tp_size: int) -> DecoderWeights:
    """Random-init weights of a TP shard without materialising the full model on any rank.

    Replicated tensors (embeddings, norms) use the same generator on every rank; sharded tensors
    use a per-rank stream, so the implied full model is the concatenation of the shards."""
    return DecoderWeights.random(cfg, device, seed=seed, tp_rank=tp_rank, tp_size=tp_size)
