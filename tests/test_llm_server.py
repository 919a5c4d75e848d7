"""The HIP LLM engine behind the llama.cpp / Ollama / OpenAI HTTP APIs (serving/llm_server.py),
driven by this framework's copies of the reference's own HTTP summarizer drivers
(LlamaCppSummarizer = llamacpp_summarizer.py:108-113, LocalLLMSummarizer = local_llm_summarizer.py:107)
and by raw requests.  CPU: tiny random-init decoder; GPU: same through the HIP kernels, with
concurrent requests batched into one generation."""
from __future__ import annotations

import concurrent.futures as cf
import json
import threading
import time

import pytest
import requests
import torch
import uvicorn

from copilot_for_consensus_amd.serving import build_from_config, chat_prompt
from copilot_for_consensus_amd.summarization import LlamaCppSummarizer, LocalLLMSummarizer, Thread


def _serve(app):
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error"))
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    deadline = time.time() + 30
    while not server.started and time.time() < deadline:
        time.sleep(0.02)
    return server, t, server.servers[0].sockets[0].getsockname()[1]


def _stack(device):
    app, s = build_from_config({"model": "tiny", "device": device, "max_new_tokens": 16, "kv_cache_tokens": 1 << 15,
                                "max_batch": 16}, max_prompt=256, max_new_cap=64)
    server, t, port = _serve(app)
    return app, s, server, t, f"http://127.0.0.1:{port}"


@pytest.fixture(scope="module")
def cpu_stack():
    app, s, server, t, base = _stack("cpu")
    yield app, s, base
    server.should_exit = True
    t.join(10)


def _check_apis(app, s, base):
    prompt = "Summarize this email thread: the working group agreed on the draft."
    ids = s.tokenizer.encode(prompt)
    # greedy reference: the engine alone
    want = s.engine.generate([ids], 12, temperature=0.0).tokens[0]
    r = requests.post(f"{base}/completion", json={"prompt": prompt, "n_predict": 12, "temperature": 0.0}).json()
    assert r["tokens_predicted"] == len(want) and r["content"] == s.tokenizer.decode(want)
    assert r["tokens_evaluated"] == len(ids) and "predicted_per_second" in r["timings"]
    assert requests.get(f"{base}/health").json()["status"] == "ok"
    toks = requests.post(f"{base}/tokenize", json={"content": prompt}).json()["tokens"]
    assert requests.post(f"{base}/detokenize", json={"tokens": toks}).json()["content"].strip() == prompt
    # Ollama, non-streaming (the reference's call) and streaming NDJSON
    o = requests.post(f"{base}/api/generate", json={"model": "x", "prompt": prompt, "stream": False,
                                                    "options": {"num_predict": 12, "temperature": 0}}).json()
    assert o["done"] is True and o["response"] == r["content"] and o["eval_count"] == len(want)
    lines = [json.loads(x) for x in requests.post(f"{base}/api/generate", json={
        "prompt": prompt, "options": {"num_predict": 12, "temperature": 0}}).text.splitlines()]
    assert lines[0]["done"] is False and lines[-1]["done"] is True and len(lines) >= 2
    assert "".join(x["response"] for x in lines) == r["content"]           # deltas add up to the text
    assert requests.get(f"{base}/api/tags").json()["models"][0]["name"] == s.cfg.name
    # OpenAI completions + chat (+ SSE framing)
    c = requests.post(f"{base}/v1/completions", json={"prompt": prompt, "max_tokens": 12, "temperature": 0}).json()
    assert c["choices"][0]["text"] == r["content"] and c["usage"]["completion_tokens"] == len(want)
    ch = requests.post(f"{base}/v1/chat/completions", json={
        "messages": [{"role": "system", "content": "be brief"}, {"role": "user", "content": prompt}],
        "max_tokens": 8, "temperature": 0}).json()
    assert ch["object"] == "chat.completion" and ch["choices"][0]["message"]["role"] == "assistant"
    ev = [x for x in requests.post(f"{base}/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "hi"}], "max_tokens": 4, "stream": True}).text.split("\n\n") if x]
    assert ev[-1] == "data: [DONE]" and json.loads(ev[0][6:])["object"] == "chat.completion.chunk"
    chunks = [json.loads(x[6:]) for x in ev[:-1]]
    assert chunks[0]["choices"][0]["delta"]["role"] == "assistant" and chunks[-1]["choices"][0]["finish_reason"]
    # llama.cpp SSE stream: several deltas while generating, then the final record
    sse = [json.loads(x[6:]) for x in requests.post(f"{base}/completion", json={
        "prompt": prompt, "n_predict": 12, "temperature": 0, "stream": True}).text.split("\n\n") if x]
    assert sse[-1]["stop"] is True and "".join(x["content"] for x in sse) == r["content"]
    # errors
    assert requests.post(f"{base}/completion", json={"prompt": 42}).status_code == 400
    long = requests.post(f"{base}/completion", json={"prompt": "x " * 5000, "n_predict": 4, "temperature": 0}).json()
    assert long["truncated"] and long["tokens_evaluated"] <= s.cfg.max_positions - 4    # cut, like llama.cpp
    assert requests.post(f"{base}/v1/chat/completions", json={"messages": []}).status_code == 400
    return prompt, want


def test_apis_on_cpu(cpu_stack):
    _check_apis(*cpu_stack)


def test_reference_drivers_against_server(cpu_stack):
    _, s, base = cpu_stack
    th = Thread(thread_id="t1", messages=[], top_k=5, context_window_tokens=4096,
                prompt="Summarize: consensus reached on draft-ietf-quic-http.")
    out = LlamaCppSummarizer(llamacpp_endpoint=base, llamacpp_model="tiny").summarize(th)
    assert out.thread_id == "t1" and isinstance(out.summary_markdown, str)
    out2 = LocalLLMSummarizer(local_llm_endpoint=base, local_llm_model="tiny").summarize(th)
    assert out2.thread_id == "t1" and isinstance(out2.summary_markdown, str)


def test_stop_strings_and_limits(cpu_stack):
    _, s, base = cpu_stack
    prompt = "The quick brown fox"
    full = requests.post(f"{base}/completion", json={"prompt": prompt, "n_predict": 16, "temperature": 0}).json()
    text = full["content"]
    if len(text) > 4:
        word = text[2:4]
        cut = requests.post(f"{base}/completion", json={"prompt": prompt, "n_predict": 16, "temperature": 0,
                                                        "stop": [word]}).json()
        assert cut["content"] == text[:text.find(word)] and cut["stopped_word"] and cut["stopping_word"] == word
    lim = requests.post(f"{base}/completion", json={"prompt": prompt, "n_predict": 3, "temperature": 0,
                                                    "ignore_eos": True}).json()
    assert lim["tokens_predicted"] == 3 and lim["stopped_limit"]


def test_chat_templates():
    msgs = [{"role": "system", "content": "S"}, {"role": "user", "content": "U1"},
            {"role": "assistant", "content": "A1"}, {"role": "user", "content": "U2"}]
    assert chat_prompt(msgs, "mistral") == "[INST] S\n\nU1 [/INST] A1</s>[INST] U2 [/INST]"
    l3 = chat_prompt(msgs[:2], "llama3")
    assert l3.endswith("<|start_header_id|>assistant<|end_header_id|>\n\n") and "<|eot_id|>" in l3


@pytest.mark.gpu
def test_server_on_gpu_batches_concurrent_requests():
    app, s, server, t, base = _stack("cuda")
    try:
        _check_apis(app, s, base)
        sched = app.state.scheduler
        before = sched.batches
        prompts = [f"thread {i}: please summarize the discussion about draft {i}" for i in range(12)]
        with cf.ThreadPoolExecutor(12) as pool:
            outs = list(pool.map(lambda p: requests.post(f"{base}/completion", json={
                "prompt": p, "n_predict": 10, "temperature": 0}).json(), prompts))
        assert all(o["tokens_predicted"] <= 10 for o in outs)
        assert sched.batches - before < len(prompts) and sched.max_seen_batch > 1     # batched on the GPU
        # each batched answer equals the request run alone (greedy)
        for p, o in zip(prompts[:3], outs[:3]):
            alone = s.engine.generate([s.tokenizer.encode(p)], 10, temperature=0.0).tokens[0]
            assert o["content"] == s.tokenizer.decode(alone)
        assert torch.cuda.is_available()
    finally:
        server.should_exit = True
        t.join(10)


def test_stream_cancel_on_disconnect(cpu_stack):
    """A streaming client that goes away mid-generation frees its slot (the request is cancelled)."""
    app, s, base = cpu_stack
    sched = app.state.scheduler
    with requests.post(f"{base}/completion", json={"prompt": "tell a long story", "n_predict": 60,
                                                   "temperature": 0, "ignore_eos": True, "stream": True},
                       stream=True) as resp:
        for line in resp.iter_lines():
            if line:
                break                      # first delta arrived; drop the connection
    deadline = time.time() + 20
    while time.time() < deadline and any(ce.pending() for ce in sched.engines.values()):
        time.sleep(0.05)
    assert not any(ce.pending() for ce in sched.engines.values())
    # the server still answers normally afterwards
    assert requests.post(f"{base}/completion", json={"prompt": "x", "n_predict": 2, "temperature": 0}).status_code == 200
