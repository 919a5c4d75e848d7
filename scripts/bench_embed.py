#!/usr/bin/env python3
"""BASELINE config 2: copilot_embedding encoder (all-MiniLM-L6 / bge-small) bf16, batch 256, 1 GPU.

Chunks are synthetic mailing-list text of the reference chunker's size (384 words, chunkers.py:114),
tokenized by the C++ WordPiece tokenizer and truncated to the model's max length (256 for MiniLM,
512 for BGE).  Reports chunks/s (tokenizer included and excluded) and encoder tokens/s.  The
reference embeds one chunk per call (embedding/app/service.py:393)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from copilot_for_consensus_amd.embedding import HipEncoderProvider  # noqa: E402
from copilot_for_consensus_amd.utils.synthetic import SyntheticArchive  # noqa: E402


def run(model, batch=256, iters=10):
    prov = HipEncoderProvider(model_name=model, device="cuda")
    words = SyntheticArchive(seed=3).corpus(384 * batch * 2).split()
    texts = [" ".join(words[i * 384:(i + 1) * 384]) for i in range(batch)]
    ids, cu = prov.tokenizer.encode_packed(texts)          # packed once: the encoder-only timing
    ntok = int(cu[-1])
    for _ in range(3):
        prov.model.encode_packed(ids, cu)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        prov.model.encode_packed(ids, cu)
    torch.cuda.synchronize()
    enc = (time.perf_counter() - t) / iters
    prov.embed_tensor(texts)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        prov.embed_tensor(texts)
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t) / iters
    r = {"model": prov.model_name, "batch": batch, "tokens_per_chunk": round(ntok / batch, 1),
         "encoder_ms_per_batch": round(enc * 1e3, 2), "chunks_per_s_encoder": round(batch / enc, 1),
         "encoder_tokens_per_s": round(ntok / enc, 1), "chunks_per_s_with_tokenizer": round(batch / e2e, 1)}
    print(json.dumps(r), flush=True)
    return r


if __name__ == "__main__":
    out = [run(m) for m in (sys.argv[1:] or ["minilm-l6", "bge-small"])]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bench_embed.json", "w") as fh:
        json.dump(out, fh, indent=1)
