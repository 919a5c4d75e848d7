"""Prefill attention tile orders (ops.kernels.prefill_tiles) at a fixed token count: global heaviest-first,
natural, per-sequence heaviest-first, pairs of sequences heaviest-first -- hipGraph timing, causal TF/s
(profiles/r06_prefill_attn_order.log)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from bench_pgemm import timed  # noqa: E402


def main():
    Hq, Hkv, D = 32, 8, 128
    for nseq, L in ((24, 700), (6, 2800), (1, 16800)):
        nb_per = math.ceil(L / 32)
        nblk = nseq * nb_per + 4
        kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
        vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
        bt = torch.randperm(nblk - 4, device="cuda").int().view(nseq, nb_per)
        cu = torch.arange(0, nseq + 1, device="cuda", dtype=torch.int32) * L
        ctx = torch.full((nseq,), L, device="cuda", dtype=torch.int32)
        q = torch.randn(nseq * L, Hq, D, device="cuda").bfloat16()
        out = torch.empty_like(q)
        rows = K.prefill_rows(Hq, Hkv)
        default_group = K.PREFILL_GROUP_CTX
        for name in ("heavy-first", "natural", "grouped", "grouped2", "production"):
            # heavy-first: one global heaviest-first order (round 5); production: the engine's groups
            K.PREFILL_GROUP_CTX = (1 << 40) if name == "heavy-first" else default_group
            seqs, q0 = K.prefill_tiles(cu.tolist(), rows, ctx.tolist() if name in ("heavy-first", "production") else None)
            K.PREFILL_GROUP_CTX = default_group
            if name.startswith("grouped"):
                # sequence by sequence (K/V locality), heaviest tile first within each sequence;
                # grouped2: sequences in pairs, the pair's tiles heavy-first
                g = 2 if name == "grouped2" else 1
                pairs = sorted(zip(seqs, q0), key=lambda t: (t[0] // g, -t[1]))
                seqs, q0 = [a for a, _ in pairs], [b for _, b in pairs]
            tiles = (torch.tensor(seqs, dtype=torch.int32, device="cuda"), torch.tensor(q0, dtype=torch.int32, device="cuda"))
            t = timed(lambda: K.prefill_attention(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), tiles=tiles, out=out))
            print(f"nseq={nseq} L={L} {name}: {t*1e6:.1f} us  {2.0*nseq*L*L*D*Hq/t/1e12:.0f} TF/s", flush=True)



if __name__ == "__main__":
    main()
