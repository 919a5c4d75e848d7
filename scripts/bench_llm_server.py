#!/usr/bin/env python3
"""HTTP serving throughput of the HIP LLM server (serving/llm_server.py) under concurrent clients.

The reference sends one ``POST /completion`` (llama.cpp) or ``/api/generate`` (Ollama) per thread
summary.  Here ``--clients`` concurrent clients each send ``--requests-per-client`` llama.cpp
``/completion`` requests (token-id prompts of ~2.5k tokens, ``n_predict`` 512, greedy, EOS ignored
so every request generates the full budget) to one server process on one GPU; prints one JSON line
with completed requests/s, generated tokens/s and latency percentiles.
"""
import argparse
import concurrent.futures as cf
import json
import os
import random
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--requests-per-client", type=int, default=2)
    ap.add_argument("--prompt", type=int, default=2560)
    ap.add_argument("--new", type=int, default=512)
    ap.add_argument("--max-batch", type=int, default=128)
    a = ap.parse_args()
    import requests
    import uvicorn

    from copilot_for_consensus_amd.serving import build_from_config
    app, s = build_from_config({"model": a.model, "device": "cuda", "max_new_tokens": a.new, "max_batch": a.max_batch,
                                "kv_cache_tokens": a.max_batch * (a.prompt + 600 + a.new) + 65536},
                               max_prompt=a.prompt + 600, max_new_cap=a.new)
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error", limit_concurrency=4096))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    while not server.started:
        time.sleep(0.05)
    base = f"http://127.0.0.1:{server.servers[0].sockets[0].getsockname()[1]}"
    rng = random.Random(0)
    V = s.cfg.vocab_size

    def prompt():
        n = rng.randint(a.prompt - 256, a.prompt + 256)
        return [s.cfg.bos_id] + [rng.randrange(3, V) for _ in range(n - 1)]

    def one(p):
        t = time.perf_counter()
        r = requests.post(f"{base}/completion", json={"prompt": p, "n_predict": a.new, "temperature": 0,
                                                      "ignore_eos": True}, timeout=1200).json()
        return time.perf_counter() - t, r["tokens_predicted"], r["tokens_evaluated"]

    # warm-up: graph capture + library handles
    one(prompt())
    work = [prompt() for _ in range(a.clients * a.requests_per_client)]
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(a.clients) as pool:
        res = list(pool.map(one, work))
    wall = time.perf_counter() - t0
    lat = sorted(x[0] for x in res)
    gen = sum(x[1] for x in res)
    out = {"metric": "llm-server requests/s (llama.cpp /completion, concurrent clients)", "model": a.model,
           "clients": a.clients, "requests": len(res), "wall_s": round(wall, 2),
           "requests_per_s": round(len(res) / wall, 3), "generated_tokens_per_s": round(gen / wall, 1),
           "prompt_tokens_per_s": round(sum(x[2] for x in res) / wall, 1),
           "latency_p50_s": round(statistics.median(lat), 2), "latency_p95_s": round(lat[int(0.95 * (len(lat) - 1))], 2),
           "max_batch_seen": app.state.scheduler.max_seen_batch}
    print(json.dumps(out), flush=True)
    server.should_exit = True
    th.join(10)


if __name__ == "__main__":
    main()
