#!/usr/bin/env python3
"""Single-stream latency benchmark: one request at a time, the operating point of every decode speed
the reference publishes (Ollama / llama.cpp, BASELINE.md: Mistral 150-200 tok/s on an RTX 4090,
Llama 2 13B 20-25 tok/s and TTFT ~2 s on an RX 6700 XT, ...).

For each model: random-init bf16 weights of that architecture, a synthetic prompt of ``--prompt``
tokens, greedy decode of ``--new`` tokens with the hipGraph decode step.  Reports TTFT (prefill of
the prompt + first token) and decode tokens/s (tokens after the first / decode wall time), median
over ``--reps`` runs.  The prefix cache is off so every run prefills the whole prompt.

    python scripts/bench_latency.py --models mistral-7b llama-2-7b llama-2-13b --prompt 512 2500
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config  # noqa: E402
from copilot_for_consensus_amd.runtime.engine import LLMEngine  # noqa: E402
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache, blocks_needed  # noqa: E402

# Published single-stream decode speeds (tok/s) for the same architecture, best hardware quoted
# (BASELINE.md).  Quantised (Q4_K_M / Q8_0) on the reference side; bf16 here.
PUBLISHED = {
    "mistral-7b": {"tok_s": 200.0, "hw": "RTX 4090, Ollama (docs/operations/ollama-gpu-setup.md:150)"},
    "llama-2-7b": {"tok_s": 80.0, "hw": "RTX 3060, Ollama (docs/operations/ollama-gpu-setup.md:152)"},
    "llama-2-13b": {"tok_s": 25.0, "ttft_s": 2.0, "hw": "RX 6700 XT, llama.cpp Q4_K_M (docs/operations/llm-gpu-setup.md:476)"},
}


def run_model(name, prompt_lens, new, reps, seed, weights="bf16"):
    cfg = get_config(name)
    dev = torch.device("cuda")
    w = DecoderWeights.random(cfg, dev, seed=seed)
    wbytes = cfg.num_params() * 2
    if weights != "bf16":
        # ggml-quantized projections (llama.cpp's Q4_K_M type recipe, or all Q8_0), random blocks:
        # decode streams them (csrc/kernels/quant.hip); prefill keeps the bf16 copies
        from copilot_for_consensus_amd.ops.kernels import attach_random_quant
        attach_random_quant(w, weights, seed)
        wbytes = sum(q.nbytes for layer in w.qlayers for q in layer.values()) + w.q_lm_head.nbytes
    model = DecoderModel(w)
    if weights != "bf16":
        assert model.decode_qgemv
    kv = PagedKVCache(cfg.layers, blocks_needed(max(prompt_lens) + new) + 8, cfg.kv_heads, cfg.head_dim, dev)
    eng = LLMEngine(model, kv, max_prefill_tokens=16384, prefix_cache=False)
    g = torch.Generator().manual_seed(seed)
    rows = []
    for plen in prompt_lens:
        prompt = [cfg.bos_id] + torch.randint(3, cfg.vocab_size, (plen - 1,), generator=g).tolist()
        eng.generate([prompt], max_new_tokens=new, ignore_eos=True)      # capture the graph, warm GEMMs
        ttft, tps = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = eng.generate([prompt], max_new_tokens=new, ignore_eos=True)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            ttft.append(res.ttft_s)
            tps.append((len(res.tokens[0]) - 1) / max(wall - res.ttft_s, 1e-9))
        row = {"model": name, "prompt_tokens": plen, "new_tokens": new, "ttft_s": round(statistics.median(ttft), 4),
               "decode_tok_s": round(statistics.median(tps), 1),
               "ms_per_token": round(1000.0 / statistics.median(tps), 3),
               "weights": weights, "weight_gb": round(wbytes / 1e9, 2)}
        # HBM bytes one decode step must read: all weights + the KV of the context so far
        kv_bytes = 2 * cfg.layers * cfg.kv_heads * cfg.head_dim * 2 * (plen + new / 2)
        row["achieved_TB_s"] = round((wbytes + kv_bytes) * statistics.median(tps) / 1e12, 2)
        pub = PUBLISHED.get(name)
        if pub:
            row["published_tok_s"] = pub["tok_s"]
            row["published_hw"] = pub["hw"]
            row["vs_published"] = round(row["decode_tok_s"] / pub["tok_s"], 2)
        print(json.dumps(row), flush=True)
        rows.append(row)
    del eng, kv, model
    torch.cuda.empty_cache()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["mistral-7b", "llama-2-7b", "llama-2-13b"])
    ap.add_argument("--prompt", nargs="+", type=int, default=[512, 2500])
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--weights", choices=["bf16", "q4_k_m", "q8_0"], default="bf16",
                    help="decode weight format (q4_k_m / q8_0: ggml blocks streamed by the quantized GEMV)")
    a = ap.parse_args()
    for name in a.models:
        run_model(name, a.prompt, a.new, a.reps, a.seed, a.weights)


if __name__ == "__main__":
    main()
