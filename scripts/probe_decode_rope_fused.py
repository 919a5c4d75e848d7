#!/usr/bin/env python3
"""Decode RoPE + KV write fused into the attention prologue vs rope_kv -> attention, at the headline
shape (B = 128 sequences of ~2.9k context, Mistral-7B heads, qkv from the decode GEMM's split-K slabs).

Each arm is a hipGraph of REPS repetitions of [qkv decode GEMM -> RoPE / KV write / attention]; the
KV cache (~0.75 GB) is larger than the Infinity Cache, so every repetition streams it from HBM as a
decode layer does.  Arms alternate (A/B/A/B) in one process.  Also checks that both arms write the same
cache bytes and return the same output.  Prints one JSON line per arm and round."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.ops import reference as R  # noqa: E402

REPS = 16


def graph_us(body, reps=5):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            body()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) / REPS)
    return sorted(ts)[len(ts) // 2] * 1e6


def main():
    torch.manual_seed(0)
    B, Hq, Hkv, D, Kd = 128, 32, 8, 128, 4096
    N = (Hq + 2 * Hkv) * D
    bs = R.KV_BLOCK
    ctx = torch.randint(2700, 3100, (B,), dtype=torch.int32)
    nb = [(int(c) + bs - 1) // bs for c in ctx]
    max_blocks = 8 * ((max(nb) + 7) // 8)
    nblk = sum(nb) + 8
    perm = torch.randperm(nblk)[:sum(nb)].int()
    bt = torch.zeros(B, max_blocks, dtype=torch.int32)
    o = 0
    for b in range(B):
        bt[b, :nb[b]] = perm[o:o + nb[b]]
        o += nb[b]
    kc = (torch.randn(nblk, Hkv, bs, D, device="cuda") * 0.5).bfloat16()
    vc = (torch.randn(nblk, Hkv, D, bs, device="cuda") * 0.5).bfloat16()
    pos = (ctx - 1).cuda()
    slots = (bt[torch.arange(B), (ctx - 1).long() // bs] * bs + (ctx - 1) % bs).int().cuda()
    ctx_d, bt_d = ctx.cuda(), bt.cuda()
    cs = R.rope_cos_sin(8192, D, 1e6).cuda()
    x = (torch.randn(B, Kd, device="cuda") * 0.05).bfloat16()
    w = K.pack_dgemm_weight((torch.randn(N, Kd, device="cuda") * 0.02).bfloat16())
    bn, split = K.dgemm_config(B, N, Kd, bn=w.bn)
    part = torch.empty(split, B, N, device="cuda")
    scale = D ** -0.5
    out_f = torch.empty(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    out_u = torch.empty_like(out_f)

    def gemm():
        K.dgemm(x, w, "part", split, part=part)

    def fused():
        K.paged_decode_rope_attention(part, pos, slots, cs, kc, vc, bt_d, ctx_d, scale, Hq, Hkv, D,
                                      part_blocks=-1, out=out_f)

    def unfused():
        q = K.rope_kv_write_part(part, pos, slots, cs, kc, vc, Hq, Hkv, D)
        K.paged_decode_attention(q, kc, vc, bt_d, ctx_d, scale, out=out_u, part_blocks=-1)

    noslots = torch.full_like(slots, -1)

    def fused_nokv():      # slots = -1: RoPE of q only, no cache write
        K.paged_decode_rope_attention(part, pos, noslots, cs, kc, vc, bt_d, ctx_d, scale, Hq, Hkv, D,
                                      part_blocks=-1, out=out_f)

    def unfused_nokv():
        q = K.rope_kv_write_part(part, pos, noslots, cs, kc, vc, Hq, Hkv, D)
        K.paged_decode_attention(q, kc, vc, bt_d, ctx_d, scale, out=out_u, part_blocks=-1)

    q_fixed = K.rope_kv_write_part(part, pos, noslots, cs, kc, vc, Hq, Hkv, D)

    qkv_b = torch.empty(B, N, device="cuda", dtype=torch.bfloat16)
    q_b = torch.empty(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    no_runs = torch.zeros(0, 4, dtype=torch.int32, device="cuda")

    def gemm_b():
        K.dgemm(x, w, "bf16", out=qkv_b)

    def unfused_bf16():     # bf16 qkv in, K and V written
        K.rope_kv_write(qkv_b, pos, slots, cs, kc, vc, Hq, Hkv, D, q_out=q_b)
        K.paged_decode_attention(q_b, kc, vc, bt_d, ctx_d, scale, out=out_u, part_blocks=-1)

    def unfused_bf16_noV():  # bf16 qkv in, K written, V skipped (no partial-line stores)
        K.rope_kv_write(qkv_b, pos, slots, cs, kc, vc, Hq, Hkv, D, q_out=q_b, runs=no_runs)
        K.paged_decode_attention(q_b, kc, vc, bt_d, ctx_d, scale, out=out_u, part_blocks=-1)

    def probe_arm(bits):
        def run():
            K.kernels().cfc_set_decode_rope_probe(bits)
            fused()
            K.kernels().cfc_set_decode_rope_probe(0)
        return run

    def attn_only():
        K.paged_decode_attention(q_fixed, kc, vc, bt_d, ctx_d, scale, out=out_u, part_blocks=-1)

    # same bytes: run each once from the same cache state
    gemm()
    k0, v0 = kc.clone(), vc.clone()
    fused()
    kf, vf = kc.clone(), vc.clone()
    kc.copy_(k0)
    vc.copy_(v0)
    unfused()
    torch.cuda.synchronize()
    same = bool(torch.equal(out_f, out_u) and torch.equal(kf, kc) and torch.equal(vf, vc))
    del k0, v0, kf, vf
    kv_bytes = sum(nb) * Hkv * bs * D * 2 * 2
    print(json.dumps({"B": B, "split": split, "bn": bn, "mean_ctx": float(ctx.float().mean()),
                      "kv_mb": round(kv_bytes / 2**20, 1), "bit_identical": same}), flush=True)
    base = graph_us(gemm)
    base_b = graph_us(gemm_b)
    arms = [("unfused", unfused), ("fused", fused), ("unfused_noKV", unfused_nokv), ("fused_noKV", fused_nokv),
            ("attention_only", attn_only), ("unfused_bf16", unfused_bf16), ("unfused_bf16_noV", unfused_bf16_noV),
            ("fused_noKrow", probe_arm(1)), ("fused_noVtile", probe_arm(2)), ("fused_noKrow_noVtile", probe_arm(3)),
            ("fused_ntVtile", probe_arm(4))]
    only = sys.argv[1:]
    for rnd in range(2):
        for name, fn in arms:
            if only and name not in only:
                continue
            g = gemm_b if "bf16" in name else gemm
            t = graph_us(lambda: (g(), fn()))
            b0 = base_b if "bf16" in name else base
            print(json.dumps({"round": rnd, "arm": name, "gemm_us": round(b0, 2), "step_us": round(t, 2),
                              "rope_attn_us": round(t - b0, 2),
                              "kv_tb_s": round(kv_bytes / ((t - b0) * 1e-6) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
