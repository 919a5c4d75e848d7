#!/usr/bin/env python3
"""Serving benchmark for the continuous-batching engine (runtime/continuous.py) on one MI355X:
Mistral-7B bf16 (random weights), requests with RAG-sized prompts (~2.5k tokens) arriving as a
Poisson process, 512 generated tokens each.  Reports completed threads/s and p50/p95 latency from
arrival to the last token -- the serving-side view of the BASELINE metric (bench.py measures the
batch pipeline)."""
import argparse
import json
import os
import random
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, get_config  # noqa: E402
from copilot_for_consensus_amd.runtime.continuous import ContinuousEngine  # noqa: E402
from copilot_for_consensus_amd.runtime.engine import LLMEngine  # noqa: E402
from copilot_for_consensus_amd.runtime.kv_cache import PagedKVCache, blocks_needed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--rate", type=float, default=12.0, help="arrivals per second")
    ap.add_argument("--requests", type=int, default=384)
    ap.add_argument("--slots", type=int, default=128)
    ap.add_argument("--max-new", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=2500)
    ap.add_argument("--steps-per-sync", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--min-admit", type=int, default=1)
    ap.add_argument("--max-wait", type=float, default=0.5)
    a = ap.parse_args()
    cfg = get_config(a.model)
    dev = torch.device("cuda")
    model = DecoderModel(DecoderWeights.random(cfg, dev, seed=1234))
    nblk = int(1.2 * a.slots * blocks_needed(int(a.prompt * 1.3) + 200 + a.max_new)) + 64
    kv = PagedKVCache(cfg.layers, nblk, cfg.kv_heads, cfg.head_dim, dev)
    eng = LLMEngine(model, kv, max_prefill_tokens=16384)
    ce = ContinuousEngine(eng, max_slots=a.slots, max_new_cap=a.max_new, max_prompt=int(a.prompt * 1.3) + 200,
                          steps_per_sync=a.steps_per_sync, min_admit=a.min_admit, max_wait_s=a.max_wait)
    rng = random.Random(a.seed)
    system = [rng.randrange(3, cfg.vocab_size) for _ in range(170)]      # shared system prompt (prefix cache)
    prompts = [[1] + system + [rng.randrange(3, cfg.vocab_size) for _ in range(int(rng.uniform(0.7, 1.3) * a.prompt))]
               for _ in range(a.requests)]
    # warm-up: capture the graph, tune nothing at run time
    ce.submit(prompts[0][:300], 8)
    ce.run()
    t, arrivals = 0.0, []
    for _ in range(a.requests):
        t += rng.expovariate(a.rate)
        arrivals.append(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    handles, i, done = [], 0, []
    while len(done) < a.requests:
        now = time.perf_counter() - t0
        while i < a.requests and arrivals[i] <= now:
            h = ce.submit(prompts[i], a.max_new)
            h.submitted_s = t0 + arrivals[i]          # latency from the scheduled arrival
            handles.append(h)
            i += 1
        if ce.pending() == 0:
            time.sleep(max(0.0, min(0.01, arrivals[i] - now)))
            continue
        done += ce.step()
    elapsed = time.perf_counter() - t0
    lat = sorted(h.latency_s for h in handles)
    ttft = sorted(h.first_token_s - h.submitted_s for h in handles)
    out = {"metric": "continuous-batching serving: threads/s and latency (arrival -> last token)",
           "model": a.model, "dtype": "bf16", "data": "synthetic prompts, random-init weights",
           "arrival_rate": a.rate, "requests": a.requests, "slots": a.slots, "prompt_tokens": a.prompt,
           "max_new_tokens": a.max_new, "threads_per_s": round(a.requests / elapsed, 3),
           "p50_latency_s": round(statistics.median(lat), 3), "p95_latency_s": round(lat[int(0.95 * len(lat)) - 1], 3),
           "p50_ttft_s": round(statistics.median(ttft), 3),
           "generated_tokens_per_s": round(sum(len(h.tokens) for h in handles) / elapsed, 1),
           "decode_steps": ce.stats["steps"], "prefill_s": round(ce.stats["prefill_s"], 2),
           "min_admit": a.min_admit, "max_wait_s": a.max_wait}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
