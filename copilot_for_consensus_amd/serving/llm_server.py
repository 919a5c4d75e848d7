"""LLM inference server: the HIP decoder behind the HTTP APIs of the engines the reference calls.

The reference's summarizers reach an LLM over HTTP: Ollama ``POST /api/generate``
(local_llm_summarizer.py:107, ``stream: false``), the llama.cpp server ``POST /completion``
(llamacpp_summarizer.py:108-113: ``n_predict`` 512, ``temperature`` 0.7, stops ``</s>`` /
``\\n\\n\\n``) and OpenAI chat completions (openai_summarizer.py:313-317).  Its compose file runs
those servers as containers (docker-compose.infra.yml: ``ollama``, ``llama-cpp``).  This module is
the MI355X replacement for those containers: the same routes and JSON, served by this framework's
engine (paged KV, GQA flash prefill, hipGraph decode, on-device sampling; GGUF or safetensors
weights), so ``LLM_BACKEND_TYPE=local`` / ``llamacpp`` / ``openai`` deployments -- the reference's
own drivers included -- run on the GPU without code changes.

Concurrent requests share the GPU through continuous batching: each distinct sampling
configuration gets a slot-based engine (runtime/continuous.py) whose hipGraph-captured decode step
runs over every in-flight request, and new requests are admitted between bursts; per-request token
limits, EOS and stop strings are applied per row.  Requests beyond the slot engine's caps fall back
to grouped batched ``LLMEngine.generate`` calls.

Routes:
  llama.cpp  POST /completion, POST /tokenize, POST /detokenize, GET /health, GET /props
  Ollama     POST /api/generate, POST /api/chat, GET /api/tags, GET /api/version
  OpenAI     POST /v1/completions, POST /v1/chat/completions, GET /v1/models
``stream: true`` streams text deltas as the slot engine produces them (read after every burst of
decode steps), in each API's framing (SSE for llama.cpp / OpenAI, NDJSON for Ollama), then the
API's final record; a client that disconnects cancels its generation.
"""
from __future__ import annotations

import dataclasses
import json
import queue
import threading
import time
import uuid
from typing import Any

from fastapi import Body, FastAPI, HTTPException
from fastapi.responses import JSONResponse, StreamingResponse


@dataclasses.dataclass
class GenRequest:
    prompt_ids: list[int]
    max_new: int
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    min_p: float = 0.0
    seed: int = 0
    stop: tuple[str, ...] = ()
    ignore_eos: bool = False
    submitted: float = dataclasses.field(default_factory=time.perf_counter)
    done: threading.Event = dataclasses.field(default_factory=threading.Event)
    text: str = ""
    tokens: list[int] = dataclasses.field(default_factory=list)
    finish: str = "stop"                 # stop | length
    stopping_word: str = ""
    prompt_s: float = 0.0
    gen_s: float = 0.0
    error: str | None = None
    truncated: bool = False              # the prompt was cut to fit the context
    stream: bool = False                 # push text deltas through on_delta while generating
    on_delta: Any = None
    emitted: int = 0                     # characters already pushed
    handle: Any = None                   # (engine key, continuous Request) while on a slot engine
    loop: Any = None                     # asyncio loop + event of an async waiter (the HTTP handlers)
    aevent: Any = None

    def complete(self) -> None:
        if self.stream and self.on_delta is not None and not self.error:
            if len(self.text) > self.emitted:
                self.on_delta(self.text[self.emitted:])
                self.emitted = len(self.text)
        self.done.set()
        if self.aevent is not None:
            self.loop.call_soon_threadsafe(self.aevent.set)

    def key(self):
        sampled = self.temperature > 0
        return (round(self.temperature, 6), self.top_k if sampled else 0, round(self.top_p, 6) if sampled else 1.0,
                round(self.min_p, 6) if sampled else 0.0, self.seed if sampled else 0, self.ignore_eos)


class BatchScheduler:
    """Runs requests on the engine: continuous batching (runtime/continuous.py: one hipGraph-captured
    decode step over a fixed set of slots, requests admitted between bursts) for each distinct
    sampling configuration, up to ``max_engines`` of them; requests beyond a continuous engine's
    prompt / token caps, or past that many configurations, run as grouped batched ``generate``
    calls (micro-batching)."""

    def __init__(self, engine, tokenizer, max_batch: int = 64, batch_wait_ms: float = 5.0, continuous: bool = True,
                 max_engines: int = 4, max_prompt: int = 4096, max_new_cap: int = 512, steps_per_sync: int = 8):
        self.engine, self.tok = engine, tokenizer
        self.max_batch, self.wait_s = int(max_batch), batch_wait_ms / 1000.0
        self.continuous, self.max_engines = continuous, int(max_engines)
        self.max_prompt, self.cap, self.steps_per_sync = int(max_prompt), int(max_new_cap), int(steps_per_sync)
        self.q: queue.Queue[GenRequest] = queue.Queue()
        self._stop = threading.Event()
        self.batches = 0
        self.served = 0
        self.max_seen_batch = 0
        self.engines: dict[tuple, Any] = {}        # sampling key -> ContinuousEngine
        self._inflight: dict[tuple, dict[int, GenRequest]] = {}
        self._t = threading.Thread(target=self._loop, name="llm-scheduler", daemon=True)
        self._t.start()

    def submit(self, r: GenRequest, timeout: float = 600.0) -> GenRequest:
        self.q.put(r)
        if not r.done.wait(timeout):
            raise TimeoutError("generation timed out")
        if r.error:
            raise RuntimeError(r.error)
        return r

    def cancel(self, r: GenRequest) -> None:
        """Thread-safe: stop a request whose client went away."""
        self.q.put(("cancel", r))

    async def asubmit(self, r: GenRequest, timeout: float = 600.0) -> GenRequest:
        """Non-blocking wait for the HTTP handlers: no worker thread is held per in-flight request."""
        import asyncio
        r.loop, r.aevent = asyncio.get_running_loop(), asyncio.Event()
        self.q.put(r)
        await asyncio.wait_for(r.aevent.wait(), timeout)
        if r.error:
            raise RuntimeError(r.error)
        return r

    def close(self) -> None:
        self._stop.set()
        self._t.join(5)

    # ------------------------------------------------------------------ scheduling
    def _continuous_for(self, r: GenRequest):
        if not self.continuous or len(r.prompt_ids) > self.max_prompt or r.max_new > self.cap:
            return None
        key = r.key()
        ce = self.engines.get(key)
        if ce is None:
            if len(self.engines) >= self.max_engines:
                return None
            from ..ops import kernels as K
            from ..runtime.continuous import ContinuousEngine
            stops = () if r.ignore_eos else (self.engine.cfg.eos_id,)
            ce = ContinuousEngine(self.engine, max_slots=self.max_batch, max_new_cap=self.cap,
                                  max_prompt=self.max_prompt, steps_per_sync=self.steps_per_sync, stop_ids=stops,
                                  seed=r.seed, max_wait_s=self.wait_s)
            ce.sampling = K.SamplingParams(r.temperature, r.top_k, r.top_p, r.min_p) if r.temperature > 0 \
                else K.SamplingParams.of(0.0)
            self.engines[key] = ce
            self._inflight[key] = {}
        return ce

    def _loop(self) -> None:
        while not self._stop.is_set():
            busy = any(ce.pending() for ce in self.engines.values())
            batch: list[GenRequest] = []
            try:
                batch.append(self.q.get(timeout=0.0 if busy else 0.1) if busy else self.q.get(timeout=0.1))
            except queue.Empty:
                pass
            if batch and not busy:       # an idle engine waits a moment so a burst of arrivals shares a prefill
                deadline = time.perf_counter() + self.wait_s
                while len(batch) < self.max_batch:
                    left = deadline - time.perf_counter()
                    try:
                        batch.append(self.q.get(timeout=left) if left > 0 else self.q.get_nowait())
                    except queue.Empty:
                        break
            while True:                  # everything else already queued
                try:
                    batch.append(self.q.get_nowait())
                except queue.Empty:
                    break
            legacy: dict[tuple, list[GenRequest]] = {}
            for r in batch:
                if isinstance(r, tuple):          # ("cancel", request)
                    h = r[1].handle
                    if h is not None and h[0] in self.engines:
                        self.engines[h[0]].cancel(h[1])
                    continue
                ce = self._continuous_for(r)
                if ce is None:
                    legacy.setdefault(r.key(), []).append(r)
                else:
                    cr = ce.submit(r.prompt_ids, r.max_new)
                    r.handle = (r.key(), cr)
                    self._inflight[r.key()][cr.rid] = r
            for g in legacy.values():
                for s in range(0, len(g), self.max_batch):
                    self._run(g[s:s + self.max_batch])
            for key, ce in list(self.engines.items()):
                if not ce.pending():
                    continue
                try:
                    active = sum(x is not None for x in ce.slot_req)
                    finished = ce.step()
                    self.max_seen_batch = max(self.max_seen_batch, active,
                                              sum(x is not None for x in ce.slot_req))
                except Exception as e:  # noqa: BLE001 -- fail every request of this engine, drop it
                    for r in self._inflight.pop(key, {}).values():
                        r.error = f"{type(e).__name__}: {e}"
                        r.complete()
                    self.engines.pop(key, None)
                    continue
                if finished:
                    self.batches += 1
                self._stream_partials(key, ce, {cr.rid for cr in finished})
                for cr in finished:
                    r = self._inflight[key].pop(cr.rid)
                    self._finish(r, cr.tokens, cr.tokens is not None and len(cr.tokens) >= r.max_new,
                                 (cr.first_token_s or cr.submitted_s) - cr.submitted_s,
                                 cr.finished_s - (cr.first_token_s or cr.submitted_s))
                    r.complete()

    def _stream_partials(self, key, ce, finishing: set[int]) -> None:
        """Push the new text of streaming requests still running; a stop string seen mid-stream
        cancels the slot (the text up to it is what the client gets)."""
        live = {rid: r for rid, r in self._inflight.get(key, {}).items() if r.stream and rid not in finishing}
        if not live:
            return
        parts = ce.partial([r.handle[1] for r in live.values()])
        for rid, toks in parts.items():
            r = live[rid]
            text = self.tok.decode(toks[:r.max_new])
            cut = min((i for i in (text.find(s) for s in r.stop) if i >= 0), default=-1)
            if cut >= 0:
                ce.cancel(r.handle[1])
                text = text[:cut]
            hold = max((len(s) for s in r.stop), default=1) - 1     # a stop string may be forming
            upto = len(text) if cut >= 0 else max(r.emitted, len(text) - hold)
            # a multi-byte character still being generated decodes as U+FFFD: wait for it
            while upto > r.emitted and text[upto - 1] == "\ufffd":
                upto -= 1
            if upto > r.emitted:
                r.on_delta(text[r.emitted:upto])
                r.emitted = upto

    def _finish(self, r: GenRequest, toks: list[int], hit_limit: bool, prompt_s: float, gen_s: float) -> None:
        toks = list(toks[:r.max_new])
        text = self.tok.decode(toks)
        cut, word = -1, ""
        for s in r.stop:
            i = text.find(s)
            if i >= 0 and (cut < 0 or i < cut):
                cut, word = i, s
        if cut >= 0:
            text, r.stopping_word, r.finish = text[:cut], word, "stop"
        else:
            r.finish = "length" if hit_limit else "stop"
        r.text, r.tokens = text, toks
        r.prompt_s, r.gen_s = prompt_s, gen_s
        self.served += 1

    def _run(self, group: list[GenRequest]) -> None:
        r0 = group[0]
        limit = self.engine.cfg.max_positions
        if len(group) > 1 and max(len(r.prompt_ids) for r in group) + max(r.max_new for r in group) > limit:
            for r in group:               # each fits alone; together the longest prompt + largest budget do not
                self._run([r])
            return
        try:
            t0 = time.perf_counter()
            res = self.engine.generate([r.prompt_ids for r in group], max(r.max_new for r in group),
                                       temperature=r0.temperature, seed=r0.seed, ignore_eos=r0.ignore_eos,
                                       top_k=r0.top_k, top_p=r0.top_p, min_p=r0.min_p)
            dt = time.perf_counter() - t0
            self.batches += 1
            self.max_seen_batch = max(self.max_seen_batch, len(group))
            for r, toks in zip(group, res.tokens):
                self._finish(r, toks, len(toks) >= r.max_new, res.prefill_s, max(dt - res.prefill_s, 0.0))
        except Exception as e:  # noqa: BLE001 -- every waiter must be released with the failure
            for r in group:
                r.error = f"{type(e).__name__}: {e}"
        finally:
            for r in group:
                r.complete()


def chat_prompt(messages: list[dict], family: str) -> str:
    """Instruction templates of the model families this framework serves."""
    msgs = [m for m in messages if isinstance(m, dict)]
    if family == "llama3":
        out = []
        for m in msgs:
            out.append(f"<|start_header_id|>{m.get('role', 'user')}<|end_header_id|>\n\n{m.get('content', '')}<|eot_id|>")
        return "".join(out) + "<|start_header_id|>assistant<|end_header_id|>\n\n"
    # Mistral / Llama-2 [INST] format; a system message is folded into the first user turn
    system = "\n\n".join(m.get("content", "") for m in msgs if m.get("role") == "system")
    out, pending_sys = [], system
    for m in msgs:
        role, content = m.get("role"), m.get("content", "")
        if role == "user":
            if pending_sys:
                content, pending_sys = f"{pending_sys}\n\n{content}", ""
            out.append(f"[INST] {content} [/INST]")
        elif role == "assistant":
            out.append(f" {content}</s>")
    return "".join(out)


def create_llm_app(engine, tokenizer, model_name: str, context_limit: int, family: str = "mistral",
                   max_batch: int = 64, batch_wait_ms: float = 5.0, default_n_predict: int = 512,
                   continuous: bool = True, max_prompt: int = 4096, max_new_cap: int = 512) -> FastAPI:
    sched = BatchScheduler(engine, tokenizer, max_batch=max_batch, batch_wait_ms=batch_wait_ms, continuous=continuous,
                           max_prompt=min(max_prompt, context_limit - 1),
                           max_new_cap=max(1, min(max_new_cap, context_limit - 1)))
    app = FastAPI(title=f"copilot-for-consensus HIP LLM server ({model_name})")
    app.state.scheduler = sched
    started = time.time()

    def encode(prompt) -> list[int]:
        if isinstance(prompt, list) and all(isinstance(x, int) for x in prompt):
            ids = list(prompt)
        elif isinstance(prompt, str):
            ids = tokenizer.encode(prompt)
        else:
            raise HTTPException(400, "prompt must be a string or a list of token ids")
        if not ids:
            raise HTTPException(400, "empty prompt")
        return ids

    def prepare(prompt, n_predict, temperature, top_k, top_p, min_p, seed, stop, ignore_eos=False) -> GenRequest:
        ids = encode(prompt)
        want = None if n_predict is None or int(n_predict) < 0 else int(n_predict)
        if want == 0:
            raise HTTPException(400, "n_predict must be positive")
        truncated = False
        budget = context_limit - min(want or 1, context_limit // 2)
        if len(ids) > budget:
            # like the llama.cpp / Ollama servers: an over-long prompt is truncated, not refused --
            # keep the head (instructions) and the newest tail, reserve room for the generation
            half = budget // 2
            ids, truncated = ids[:half] + ids[len(ids) - (budget - half):], True
        room = context_limit - len(ids)
        n = room if want is None else min(want, room)
        if isinstance(stop, str):
            stop = [stop]
        r = GenRequest(ids, n, float(temperature or 0.0), int(top_k or 0), float(1.0 if top_p is None else top_p),
                       float(min_p or 0.0), int(seed or 0), tuple(s for s in (stop or []) if s), bool(ignore_eos))
        r.truncated = truncated
        return r

    async def run(*args, **kw) -> GenRequest:
        try:
            return await sched.asubmit(prepare(*args, **kw))
        except RuntimeError as e:
            raise HTTPException(500, str(e))

    def streamed(r: GenRequest, frame_delta, frame_final, media_type: str, tail: str | None = None):
        """Incremental response: one frame per text delta while the slot engine generates, then the
        API's final record; a client that disconnects cancels the generation."""
        import asyncio
        loop = asyncio.get_event_loop()
        q: asyncio.Queue = asyncio.Queue()
        r.stream, r.loop, r.aevent = True, loop, asyncio.Event()
        r.on_delta = lambda text: loop.call_soon_threadsafe(q.put_nowait, text)
        sched.q.put(r)

        async def gen():
            done_wait = asyncio.ensure_future(r.aevent.wait())
            try:
                while True:
                    get = asyncio.ensure_future(q.get())
                    finished, _ = await asyncio.wait({get, done_wait}, return_when=asyncio.FIRST_COMPLETED)
                    if get in finished:
                        yield frame_delta(get.result())
                        continue
                    get.cancel()
                    while not q.empty():
                        yield frame_delta(q.get_nowait())
                    break
                yield frame_final(None if r.error else r)
                if tail:
                    yield tail
            finally:
                if not r.done.is_set():
                    sched.cancel(r)
                done_wait.cancel()
        return StreamingResponse(gen(), media_type=media_type)

    # ------------------------------------------------------------------ llama.cpp server
    @app.get("/health")
    def health():
        return {"status": "ok", "slots_idle": 1, "slots_processing": 0}

    @app.get("/props")
    def props():
        return {"default_generation_settings": {"n_ctx": context_limit, "model": model_name,
                                                "n_predict": default_n_predict},
                "total_slots": max_batch}

    @app.post("/tokenize")
    def tokenize(body: dict = Body(...)):
        return {"tokens": tokenizer.encode(body.get("content", ""), add_bos=bool(body.get("add_special", False)))}

    @app.post("/detokenize")
    def detokenize(body: dict = Body(...)):
        return {"content": tokenizer.decode(list(body.get("tokens") or []))}

    @app.post("/completion")
    async def completion(body: dict = Body(...)):
        # llama.cpp defaults: temperature 0.8, top_k 40, top_p 0.95, min_p 0.05
        args = (body.get("prompt"), body.get("n_predict", default_n_predict), body.get("temperature", 0.8),
                body.get("top_k", 40), body.get("top_p", 0.95), body.get("min_p", 0.05), body.get("seed"),
                body.get("stop"), body.get("ignore_eos", False))
        if body.get("stream"):
            return streamed(prepare(*args), lambda d: "data: " + json.dumps({"content": d, "stop": False}) + "\n\n",
                            lambda r: "data: " + json.dumps({**llama_record(r), "content": ""} if r else
                                                            {"error": "generation failed", "stop": True}) + "\n\n",
                            "text/event-stream")
        return llama_record(await run(*args))

    def llama_record(r: GenRequest) -> dict:
        return {"content": r.text, "model": model_name, "stop": True, "tokens_predicted": len(r.tokens),
               "tokens_evaluated": len(r.prompt_ids), "stopped_eos": r.finish == "stop" and not r.stopping_word,
               "stopped_word": bool(r.stopping_word), "stopped_limit": r.finish == "length",
               "stopping_word": r.stopping_word, "truncated": r.truncated,
               "timings": {"prompt_n": len(r.prompt_ids), "prompt_ms": 1000 * r.prompt_s,
                           "predicted_n": len(r.tokens), "predicted_ms": 1000 * r.gen_s,
                           "predicted_per_second": len(r.tokens) / r.gen_s if r.gen_s > 0 else 0.0}}

    # ------------------------------------------------------------------ Ollama
    def ollama_opts(body):
        o = dict(body.get("options") or {})
        return (o.get("num_predict", default_n_predict), o.get("temperature", 0.8), o.get("top_k", 40),
                o.get("top_p", 0.9), o.get("min_p", 0.0), o.get("seed"), o.get("stop"))

    def ollama_record(r: GenRequest, extra: dict) -> dict:
        return {"model": model_name, "created_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), **extra,
                "done": True, "done_reason": r.finish, "total_duration": int(1e9 * (r.prompt_s + r.gen_s)),
                "load_duration": 0, "prompt_eval_count": len(r.prompt_ids),
                "prompt_eval_duration": int(1e9 * r.prompt_s), "eval_count": len(r.tokens),
                "eval_duration": int(1e9 * r.gen_s)}

    def now_iso() -> str:
        return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())

    @app.post("/api/generate")
    async def ollama_generate(body: dict = Body(...)):
        prompt = body.get("prompt", "")
        if body.get("system") and not body.get("raw"):
            prompt = chat_prompt([{"role": "system", "content": body["system"]}, {"role": "user", "content": prompt}],
                                 family)
        n, temp, k, p, mp, seed, stop = ollama_opts(body)
        if body.get("stream", True):                 # Ollama streams unless told not to
            return streamed(prepare(prompt, n, temp, k, p, mp, seed, stop),
                            lambda d: json.dumps({"model": model_name, "created_at": now_iso(), "response": d,
                                                  "done": False}) + "\n",
                            lambda r: json.dumps(ollama_record(r, {"response": "", "context": []}) if r else
                                                 {"error": "generation failed"}) + "\n",
                            "application/x-ndjson")
        r = await run(prompt, n, temp, k, p, mp, seed, stop)
        return ollama_record(r, {"response": r.text, "context": []})

    @app.post("/api/chat")
    async def ollama_chat(body: dict = Body(...)):
        n, temp, k, p, mp, seed, stop = ollama_opts(body)
        prompt = chat_prompt(body.get("messages") or [], family)
        if body.get("stream", True):
            return streamed(prepare(prompt, n, temp, k, p, mp, seed, stop),
                            lambda d: json.dumps({"model": model_name, "created_at": now_iso(),
                                                  "message": {"role": "assistant", "content": d},
                                                  "done": False}) + "\n",
                            lambda r: json.dumps(ollama_record(r, {"message": {"role": "assistant", "content": ""}})
                                                 if r else {"error": "generation failed"}) + "\n",
                            "application/x-ndjson")
        r = await run(prompt, n, temp, k, p, mp, seed, stop)
        return ollama_record(r, {"message": {"role": "assistant", "content": r.text}})

    @app.get("/api/tags")
    def ollama_tags():
        return {"models": [{"name": model_name, "model": model_name, "modified_at": "", "size": 0,
                            "details": {"family": family, "format": "hip"}}]}

    @app.get("/api/version")
    def ollama_version():
        return {"version": "0.0.0-cfc-hip"}

    # ------------------------------------------------------------------ OpenAI
    def oai_usage(r: GenRequest) -> dict:
        return {"prompt_tokens": len(r.prompt_ids), "completion_tokens": len(r.tokens),
                "total_tokens": len(r.prompt_ids) + len(r.tokens)}

    def sse(obj: dict) -> str:
        return "data: " + json.dumps(obj) + "\n\n"

    @app.post("/v1/completions")
    async def oai_completions(body: dict = Body(...)):
        if int(body.get("n", 1)) != 1:
            raise HTTPException(400, "only n=1 is supported")
        prompt = body.get("prompt", "")
        if isinstance(prompt, list) and prompt and isinstance(prompt[0], str):
            if len(prompt) != 1:
                raise HTTPException(400, "one prompt per request")
            prompt = prompt[0]
        args = (prompt, body.get("max_tokens", 16), body.get("temperature", 1.0), 0, body.get("top_p", 1.0), 0.0,
                body.get("seed"), body.get("stop"))
        cid, created = f"cmpl-{uuid.uuid4().hex[:24]}", int(time.time())
        head = {"id": cid, "object": "text_completion", "created": created, "model": model_name}
        if body.get("stream"):
            return streamed(prepare(*args),
                            lambda d: sse({**head, "choices": [{"text": d, "index": 0, "logprobs": None,
                                                                "finish_reason": None}]}),
                            lambda r: sse({**head, "choices": [{"text": "", "index": 0, "logprobs": None,
                                                                "finish_reason": r.finish if r else "error"}]}),
                            "text/event-stream", tail="data: [DONE]\n\n")
        r = await run(*args)
        choice = {"text": r.text, "index": 0, "logprobs": None, "finish_reason": r.finish}
        return {"id": cid, "object": "text_completion", "created": created, "model": model_name,
                "choices": [choice], "usage": oai_usage(r)}

    @app.post("/v1/chat/completions")
    async def oai_chat(body: dict = Body(...)):
        if int(body.get("n", 1)) != 1:
            raise HTTPException(400, "only n=1 is supported")
        msgs = body.get("messages")
        if not isinstance(msgs, list) or not msgs:
            raise HTTPException(400, "messages must be a non-empty list")
        args = (chat_prompt(msgs, family), body.get("max_tokens", body.get("max_completion_tokens")),
                body.get("temperature", 1.0), 0, body.get("top_p", 1.0), 0.0, body.get("seed"), body.get("stop"))
        cid, created = f"chatcmpl-{uuid.uuid4().hex[:24]}", int(time.time())
        head = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model_name}
        if body.get("stream"):
            first = {"sent": False}

            def delta(d):
                dd = {"content": d} if first["sent"] else {"role": "assistant", "content": d}
                first["sent"] = True
                return sse({**head, "choices": [{"index": 0, "delta": dd, "finish_reason": None}]})
            return streamed(prepare(*args), delta,
                            lambda r: sse({**head, "choices": [{"index": 0, "delta": {},
                                                                "finish_reason": r.finish if r else "error"}]}),
                            "text/event-stream", tail="data: [DONE]\n\n")
        r = await run(*args)
        return {"id": cid, "object": "chat.completion", "created": created, "model": model_name,
                "choices": [{"index": 0, "message": {"role": "assistant", "content": r.text},
                             "finish_reason": r.finish}], "usage": oai_usage(r)}

    @app.get("/v1/models")
    def oai_models():
        return {"object": "list", "data": [{"id": model_name, "object": "model", "created": int(started),
                                            "owned_by": "copilot-for-consensus-amd"}]}

    @app.get("/metrics")
    def metrics():
        return JSONResponse({"requests_served": sched.served, "batches": sched.batches,
                             "max_batch_seen": sched.max_seen_batch, "queue_depth": sched.q.qsize()})

    return app


def build_from_config(cfg: dict[str, Any], **server_kw):
    """(app, summarizer) from the ``llm_backend`` hip driver settings (LLM_MODEL_PRESET / LLM_GGUF_PATH /
    LLM_CHECKPOINT_DIR / LLM_KV_CACHE_TOKENS / LLM_MAX_BATCH ...)."""
    from ..summarization import HipLLMSummarizer
    s = HipLLMSummarizer(**{k: v for k, v in cfg.items() if v is not None})
    name = s.cfg.name
    family = "llama3" if "llama-3" in name or "llama3" in name or s.cfg.vocab_size > 100000 else "mistral"
    app = create_llm_app(s.engine, s.tokenizer, name, s.cfg.max_positions, family=family,
                         max_batch=s.max_batch, default_n_predict=s.max_new_tokens, **server_kw)
    return app, s
