"""The OpenAI / Azure OpenAI drivers over REST (no SDK): against this framework's own LLM and
embedding servers, and against a rate-limiting stub for the reference's 429 handling
(openai_summarizer.py:189-286: full jitter, retry-after(-ms) honoured, max_retries)."""
from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np
import pytest
import uvicorn

from copilot_for_consensus_amd.embedding import HipEncoderProvider, create_embedding_provider
from copilot_for_consensus_amd.serving import build_from_config, create_embedding_app
from copilot_for_consensus_amd.summarization import Thread, create_llm_backend
from copilot_for_consensus_amd.utils.openai_rest import OpenAIHTTPError, OpenAIRestClient


def _serve(app):
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error"))
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    while not server.started:
        time.sleep(0.02)
    return server, t, f"http://127.0.0.1:{server.servers[0].sockets[0].getsockname()[1]}"


class _Cfg:
    def __init__(self, name, **kw):
        self.driver_name, self.driver_config = name, kw


def test_openai_drivers_against_own_servers():
    llm_app, s = build_from_config({"model": "tiny", "device": "cpu", "max_new_tokens": 16, "max_batch": 4,
                                    "kv_cache_tokens": 1 << 15}, max_prompt=512, max_new_cap=64)
    prov = HipEncoderProvider(model_name="tiny", device="cpu")
    srv1, t1, llm = _serve(llm_app)
    srv2, t2, emb = _serve(create_embedding_app(prov))
    try:
        summ = create_llm_backend(_Cfg("openai", openai_base_url=f"{llm}/v1", openai_model="tiny", openai_api_key="k"))
        out = summ.summarize(Thread("t1", [], prompt="Summarize: the group agreed.", context_window_tokens=12))
        assert out.thread_id == "t1" and out.llm_backend == "openai" and 0 < out.tokens_completion <= 12
        e = create_embedding_provider(_Cfg("openai", base_url=f"{emb}/v1", model="tiny", api_key="k"))
        assert e.dimension == prov.dimension
        np.testing.assert_allclose(e.embed_batch(["a b", "c d e"]), prov.embed_batch(["a b", "c d e"]), atol=1e-5)
    finally:
        for srv, t in ((srv1, t1), (srv2, t2)):
            srv.should_exit = True
            t.join(10)


class _RateLimited(BaseHTTPRequestHandler):
    fails = 2
    calls: list = []

    def do_POST(self):
        n = int(self.headers.get("Content-Length", 0))
        body = json.loads(self.rfile.read(n))
        type(self).calls.append((self.path, dict(self.headers), body))
        if len(type(self).calls) <= type(self).fails:
            self.send_response(429)
            self.send_header("retry-after-ms", "10")
            self.end_headers()
            self.wfile.write(b'{"error": "rate limit"}')
            return
        out = json.dumps({"choices": [{"message": {"role": "assistant", "content": "ok"}}],
                          "usage": {"prompt_tokens": 3, "completion_tokens": 1}}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(out)))
        self.end_headers()
        self.wfile.write(out)

    def log_message(self, *a):
        pass


@pytest.fixture
def stub():
    _RateLimited.calls = []
    _RateLimited.fails = 2
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _RateLimited)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield srv, f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


def test_rate_limit_backoff_and_azure_routing(stub):
    _, base = stub
    slept = []
    c = OpenAIRestClient(azure_endpoint=base, deployment="gpt4", api_key="secret", api_version="2024-01-01",
                         max_retries=3, sleep=slept.append)
    r = c.chat("ignored", [{"role": "user", "content": "x"}], max_tokens=5)
    assert r["choices"][0]["message"]["content"] == "ok" and c.retries == 2
    assert all(0 <= d <= 0.015 for d in slept)                      # retry-after-ms 10 x 1.5 jitter cap
    path, headers, body = _RateLimited.calls[-1]
    assert path == "/openai/deployments/gpt4/chat/completions?api-version=2024-01-01"
    hl = {k.lower(): v for k, v in headers.items()}
    assert hl.get("api-key") == "secret" and "model" not in body and body["max_tokens"] == 5
    _RateLimited.calls, _RateLimited.fails = [], 10
    c2 = OpenAIRestClient(base_url=base, api_key="k", max_retries=2, sleep=lambda _: None)
    with pytest.raises(OpenAIHTTPError) as ei:
        c2.chat("m", [{"role": "user", "content": "x"}])
    assert ei.value.status_code == 429 and len(_RateLimited.calls) == 3     # first try + 2 retries
    assert _RateLimited.calls[0][1].get("Authorization") == "Bearer k"


def test_backoff_formula():
    c = OpenAIRestClient(base_backoff_seconds=5)
    assert all(0 <= c.backoff(1, None) <= 5 for _ in range(50))
    assert all(0 <= c.backoff(3, None) <= 20 for _ in range(50))
    assert all(0 <= c.backoff(10, None) <= 120 for _ in range(50))        # capped at 2 minutes
    assert all(0 <= c.backoff(1, 100.0) <= 120 for _ in range(50))
