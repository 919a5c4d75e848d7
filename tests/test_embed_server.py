"""The HIP encoder behind the OpenAI / Ollama / TEI embedding APIs (serving/embed_server.py):
vectors equal the provider's own batch output, concurrent requests coalesce into shared encoder
forwards (CPU: tiny encoder on the reference path; GPU: MiniLM through the HIP kernels)."""
from __future__ import annotations

import concurrent.futures as cf
import threading
import time

import numpy as np
import pytest
import requests
import uvicorn

from copilot_for_consensus_amd.embedding import HipEncoderProvider
from copilot_for_consensus_amd.serving import create_embedding_app


def _serve(provider):
    app = create_embedding_app(provider, batch_wait_ms=20.0)
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error"))
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    while not server.started:
        time.sleep(0.02)
    return app, server, t, f"http://127.0.0.1:{server.servers[0].sockets[0].getsockname()[1]}"


def _check(provider, base, app, atol):
    texts = [f"message {i} about draft-ietf-quic-{i} and consensus" for i in range(24)]
    want = np.asarray(provider.embed_batch(texts))
    r = requests.post(f"{base}/v1/embeddings", json={"input": texts[:3], "model": "x"}).json()
    got = np.asarray([d["embedding"] for d in sorted(r["data"], key=lambda d: d["index"])])
    np.testing.assert_allclose(got, want[:3], atol=atol)
    assert r["usage"]["prompt_tokens"] == sum(len(t.split()) for t in texts[:3])
    e = requests.post(f"{base}/api/embed", json={"model": "x", "input": texts[3]}).json()["embeddings"]
    np.testing.assert_allclose(e[0], want[3], atol=atol)
    leg = requests.post(f"{base}/api/embeddings", json={"model": "x", "prompt": texts[4]}).json()["embedding"]
    np.testing.assert_allclose(leg, want[4], atol=atol)
    tei = requests.post(f"{base}/embed", json={"inputs": texts[5:7]}).json()
    np.testing.assert_allclose(tei, want[5:7], atol=atol)
    assert requests.post(f"{base}/v1/embeddings", json={"input": 5}).status_code == 400
    assert requests.get(f"{base}/info").json()["dimension"] == provider.dimension
    b = app.state.batcher
    f0 = b.forwards
    with cf.ThreadPoolExecutor(16) as pool:
        outs = list(pool.map(lambda t: requests.post(f"{base}/v1/embeddings", json={"input": t}).json(), texts[8:24]))
    np.testing.assert_allclose([o["data"][0]["embedding"] for o in outs], want[8:24], atol=atol)
    assert b.forwards - f0 < 16                      # coalesced into shared forwards


def test_embedding_server_cpu():
    p = HipEncoderProvider(model_name="tiny", device="cpu")
    app, server, t, base = _serve(p)
    try:
        _check(p, base, app, atol=1e-5)
    finally:
        server.should_exit = True
        t.join(10)


@pytest.mark.gpu
def test_embedding_server_gpu():
    p = HipEncoderProvider(model_name="all-MiniLM-L6-v2", device="cuda")
    app, server, t, base = _serve(p)
    try:
        # batched varlen forwards group different texts: bf16 rounding differs slightly by batch
        _check(p, base, app, atol=2e-2)
    finally:
        server.should_exit = True
        t.join(10)
