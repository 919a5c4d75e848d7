"""Embedding server: the HIP encoder behind the OpenAI, Ollama and HF text-embeddings-inference APIs.

The reference embeds through SentenceTransformers in-process (sentence_transformer_provider.py:93),
HF transformers (huggingface_provider.py:98) or the OpenAI embeddings API (openai_provider.py:
124-126), and its config schemas carry an Ollama embedding driver (embedding_ollama.json).  This
server puts the batched varlen HIP encoder (MiniLM / BGE, csrc/kernels) behind those HTTP APIs so a
remote client -- or the reference's OpenAI driver with ``base_url`` pointed here -- embeds on the
MI355X.  Concurrent requests are coalesced: a scheduler thread gathers the texts of every request
that arrives within ``batch_wait_ms`` and runs them as one packed encoder forward.

Routes: POST /v1/embeddings, GET /v1/models (OpenAI); POST /api/embed, POST /api/embeddings
(Ollama, new and legacy); POST /embed, GET /info (text-embeddings-inference); GET /health.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Any

from fastapi import Body, FastAPI, HTTPException


class _Job:
    __slots__ = ("texts", "vectors", "error", "loop", "event", "n_tokens")

    def __init__(self, texts: list[str]):
        self.texts, self.vectors, self.error, self.loop, self.event, self.n_tokens = texts, None, None, None, None, 0


class EmbedBatcher:
    def __init__(self, provider, max_batch_texts: int = 256, batch_wait_ms: float = 2.0):
        self.p, self.max_texts, self.wait_s = provider, int(max_batch_texts), batch_wait_ms / 1000.0
        self.q: queue.Queue[_Job] = queue.Queue()
        self.forwards = 0
        self.texts_embedded = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, name="embed-batcher", daemon=True)
        self._t.start()

    async def embed(self, texts: list[str]) -> list[list[float]]:
        import asyncio
        j = _Job(texts)
        j.loop, j.event = asyncio.get_running_loop(), asyncio.Event()
        self.q.put(j)
        await asyncio.wait_for(j.event.wait(), 300)
        if j.error:
            raise RuntimeError(j.error)
        return j.vectors

    def _loop(self) -> None:
        while not self._stop.is_set():
            try:
                jobs = [self.q.get(timeout=0.1)]
            except queue.Empty:
                continue
            n = len(jobs[0].texts)
            deadline = time.perf_counter() + self.wait_s
            while n < self.max_texts:
                left = deadline - time.perf_counter()
                try:
                    j = self.q.get(timeout=left) if left > 0 else self.q.get_nowait()
                except queue.Empty:
                    break
                jobs.append(j)
                n += len(j.texts)
            texts = [t for j in jobs for t in j.texts]
            try:
                vecs = self.p.embed_tensor(texts).float().cpu().tolist() if hasattr(self.p, "embed_tensor") \
                    else [self.p.embed(t) for t in texts]
                self.forwards += 1
                self.texts_embedded += len(texts)
                o = 0
                for j in jobs:
                    j.vectors = vecs[o:o + len(j.texts)]
                    o += len(j.texts)
            except Exception as e:  # noqa: BLE001 -- every waiter gets the failure
                for j in jobs:
                    j.error = f"{type(e).__name__}: {e}"
            for j in jobs:
                j.loop.call_soon_threadsafe(j.event.set)

    def close(self) -> None:
        self._stop.set()
        self._t.join(5)


def _texts(x: Any, field: str) -> list[str]:
    if isinstance(x, str):
        return [x]
    if isinstance(x, list) and x and all(isinstance(t, str) for t in x):
        return list(x)
    raise HTTPException(400, f"'{field}' must be a string or a non-empty list of strings")


def create_embedding_app(provider, max_batch_texts: int = 256, batch_wait_ms: float = 2.0) -> FastAPI:
    b = EmbedBatcher(provider, max_batch_texts, batch_wait_ms)
    app = FastAPI(title=f"copilot-for-consensus HIP embedding server ({provider.model_name})")
    app.state.batcher = b
    name, dim = provider.model_name, int(provider.dimension)

    def usage(texts):
        n = sum(len(t.split()) for t in texts)     # word counts, as the reference's local backends report
        return {"prompt_tokens": n, "total_tokens": n}

    @app.get("/health")
    def health():
        return {"status": "ok", "model": name, "dimension": dim}

    @app.post("/v1/embeddings")
    async def openai_embeddings(body: dict = Body(...)):
        texts = _texts(body.get("input"), "input")
        vecs = await b.embed(texts)
        return {"object": "list", "model": name, "usage": usage(texts),
                "data": [{"object": "embedding", "index": i, "embedding": v} for i, v in enumerate(vecs)]}

    @app.get("/v1/models")
    def models():
        return {"object": "list", "data": [{"id": name, "object": "model", "owned_by": "copilot-for-consensus-amd"}]}

    @app.post("/api/embed")
    async def ollama_embed(body: dict = Body(...)):
        texts = _texts(body.get("input"), "input")
        return {"model": name, "embeddings": await b.embed(texts), "prompt_eval_count": usage(texts)["total_tokens"]}

    @app.post("/api/embeddings")
    async def ollama_embeddings_legacy(body: dict = Body(...)):
        return {"embedding": (await b.embed(_texts(body.get("prompt"), "prompt")))[0]}

    @app.post("/embed")
    async def tei_embed(body: dict = Body(...)):
        return await b.embed(_texts(body.get("inputs"), "inputs"))

    @app.get("/info")
    def tei_info():
        return {"model_id": name, "model_dtype": "bfloat16", "max_client_batch_size": max_batch_texts,
                "dimension": dim}

    return app
