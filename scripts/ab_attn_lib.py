#!/usr/bin/env python3
"""A/B of the prefill attention kernel against another build of attention.hip in ONE process:
the in-tree library (ops.kernels) vs a library given on the command line (same C API), identical
inputs, interleaved hipGraph timing, and a bit-identity check of the two outputs.
Usage: ab_attn_lib.py OTHER.so [rounds]"""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from copilot_for_consensus_amd.ops import _native, kernels as K  # noqa: E402
from bench_pgemm import timed  # noqa: E402


def case(other, nseq, L, Hq=32, Hkv=8, D=128, rounds=3):
    nb_per = math.ceil(L / 32)
    nblk = nseq * nb_per + 4
    kc = torch.randn(nblk, Hkv, 32, D, device="cuda").bfloat16()
    vc = torch.randn(nblk, Hkv, D, 32, device="cuda").bfloat16()
    bt = torch.randperm(nblk - 4, device="cuda").int().view(nseq, nb_per)
    cu = torch.arange(0, nseq + 1, device="cuda", dtype=torch.int32) * L
    ctx = torch.full((nseq,), L, device="cuda", dtype=torch.int32)
    q = torch.randn(nseq * L, Hq, D, device="cuda").bfloat16()
    rows = K.prefill_rows(Hq, Hkv)
    seqs, q0 = K.prefill_tiles(cu.tolist(), rows, ctx.tolist())
    ts_, tq = (torch.tensor(seqs, dtype=torch.int32, device="cuda"), torch.tensor(q0, dtype=torch.int32, device="cuda"))
    outs = {"new": torch.empty_like(q), "old": torch.empty_like(q)}
    libs = {"new": K.kernels(), "old": other}

    def run(tag):
        K.check(libs[tag].cfc_prefill_attention(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), cu.data_ptr(),
                                                ctx.data_ptr(), ts_.data_ptr(), tq.data_ptr(), ts_.numel(), rows, Hq,
                                                Hkv, D, bt.shape[1], 1 / math.sqrt(D), 0, outs[tag].data_ptr(),
                                                K._stream(q)), tag)
    run("new")
    run("old")
    torch.cuda.synchronize()
    same = torch.equal(outs["new"], outs["old"])
    t = {"new": [], "old": []}
    for _ in range(rounds):
        for tag in ("old", "new"):
            t[tag].append(timed(lambda tag=tag: run(tag)))
    flops = 2.0 * nseq * L * L * D * Hq
    res = {k: round(sorted(v)[len(v) // 2] * 1e3, 4) for k, v in t.items()}
    print(f"prefill nseq={nseq} L={L}: old {res['old']} ms  new {res['new']} ms  "
          f"({flops / res['new'] / 1e9:.0f} TF/s new)  bit-identical={same}", flush=True)


if __name__ == "__main__":
    other = _native._bind(ctypes.CDLL(sys.argv[1], mode=os.RTLD_LOCAL),
                          {"cfc_prefill_attention": _native._KERNEL_SIGS["cfc_prefill_attention"]})
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.manual_seed(0)
    for _ in range(2):
        case(other, 6, 2800, rounds=rounds)
        case(other, 1, 16384, rounds=rounds)
