"""Summarizers (API of adapters/copilot_summarization: Summarizer.summarize(Thread) -> Summary,
summarizer.py:20; models Thread / Summary / Citation, models.py).

* :class:`HipLLMSummarizer` (driver ``hip``) -- the MI355X decoder engine (runtime/engine.py):
  ``summarize_batch`` generates many threads at once (continuous prefill + hipGraph decode), and
  token counts are real tokenizer counts (the local reference backends report word counts,
  local_llm_summarizer.py:101,129).
* :class:`MockSummarizer` -- deterministic canned summary with optional latency.
* :class:`LocalLLMSummarizer` (Ollama ``/api/generate``), :class:`LlamaCppSummarizer`
  (``/completion``), :class:`OpenAISummarizer` -- HTTP drivers kept for deployment parity.
"""
from __future__ import annotations

import dataclasses
import json
import time
from abc import ABC, abstractmethod

import torch


@dataclasses.dataclass
class Citation:
    message_id: str
    chunk_id: str
    offset: int = 0


@dataclasses.dataclass
class Thread:
    thread_id: str
    messages: list[str]
    top_k: int = 10
    context_window_tokens: int = 4096
    prompt: str = "Summarize the following discussion thread:"


@dataclasses.dataclass
class Summary:
    thread_id: str
    summary_markdown: str
    citations: list[Citation] = dataclasses.field(default_factory=list)
    llm_backend: str = "unknown"
    llm_model: str = "unknown"
    tokens_prompt: int = 0
    tokens_completion: int = 0
    latency_ms: int = 0


class Summarizer(ABC):
    backend = "unknown"
    model = "unknown"

    @abstractmethod
    def summarize(self, thread: Thread) -> Summary: ...

    def summarize_batch(self, threads: list[Thread]) -> list[Summary]:
        return [self.summarize(t) for t in threads]


class MockSummarizer(Summarizer):
    backend, model = "mock", "mock"

    def __init__(self, mock_latency_ms: int = 100, **_):
        self.latency_ms = int(mock_latency_ms or 0)

    def summarize(self, thread: Thread) -> Summary:
        if self.latency_ms:
            time.sleep(self.latency_ms / 1000)
        body = "\n".join(f"- {m[:80]}" for m in thread.messages[:5])
        md = f"# Summary of thread {thread.thread_id}\n\n{len(thread.messages)} excerpts reviewed.\n\n{body}\n"
        return Summary(thread.thread_id, md, [], self.backend, self.model, len(thread.prompt.split()),
                       len(md.split()), self.latency_ms)


class HipLLMSummarizer(Summarizer):
    backend = "hip"

    def __init__(self, model: str = "mistral-7b", checkpoint_dir: str | None = None, gguf_path: str | None = None,
                 tensor_parallel: int = 1,
                 max_new_tokens: int = 512, temperature: float = 0.0, max_batch: int = 128,
                 kv_cache_tokens: int = 524288, device: str = "cuda", seed: int = 1234, tp_group=None,
                 tp_rank: int = 0, ignore_eos: bool = False, top_k: int = 40, top_p: float = 0.95,
                 min_p: float = 0.05, stop_sequences=("</s>", "\n\n\n"), weight_dtype: str = "bf16",
                 kv_cache_dtype: str = "bf16", **_):
        from ..models.decoder import DecoderModel, DecoderWeights, get_config, load_config_json
        from ..runtime.engine import LLMEngine
        from ..runtime.kv_cache import PagedKVCache
        from ..runtime.tokenizer import load_hf_tokenizer, synthetic_bpe
        dev = torch.device(device if (not str(device).startswith("cuda") or torch.cuda.is_available()) else "cpu")
        if gguf_path is None and checkpoint_dir and str(checkpoint_dir).endswith(".gguf"):
            gguf_path, checkpoint_dir = checkpoint_dir, None
        if gguf_path:
            # llama.cpp / Ollama weights: bf16 copies for prefill and batches, the ggml blocks kept
            # for the quantized B <= 4 decode GEMV (runtime/gguf.py, csrc/kernels/quant.hip)
            from ..runtime import gguf as G
            if tensor_parallel > 1:
                raise ValueError("GGUF checkpoints run on one GPU (tensor_parallel must be 1)")
            w = DecoderWeights.from_gguf(gguf_path, dev)
            cfg = w.cfg
            self.tokenizer = G.tokenizer_from_gguf(G.GGUFReader(gguf_path).metadata)
        elif checkpoint_dir:
            from pathlib import Path
            cfg = load_config_json(Path(checkpoint_dir) / "config.json")
            w = DecoderWeights.from_safetensors(cfg, checkpoint_dir, dev, tp_rank, tensor_parallel)
            self.tokenizer = load_hf_tokenizer(Path(checkpoint_dir) / "tokenizer.json")
        else:
            cfg = get_config(model)
            w = DecoderWeights.random(cfg, dev, seed=seed, tp_rank=tp_rank, tp_size=tensor_parallel)
            self.tokenizer = synthetic_bpe(cfg.vocab_size)
        if weight_dtype == "fp8":
            w.to_fp8()           # opt-in W8A8 FP8 projections (LLM_WEIGHT_DTYPE=fp8)
        self.cfg = cfg
        self.model = cfg.name
        custom_ar = None
        if tp_group is not None and tensor_parallel > 1:
            from ..parallel.custom_ar import maybe_create
            custom_ar = maybe_create(tp_group, dev)
        self.decoder = DecoderModel(w, tp_group=tp_group, custom_ar=custom_ar)
        kvd = torch.float8_e4m3fn if kv_cache_dtype == "fp8" else torch.bfloat16
        self.kv = PagedKVCache.for_budget(cfg.layers, w.kv_heads, cfg.head_dim, dev, kv_cache_tokens, dtype=kvd)
        self.engine = LLMEngine(self.decoder, self.kv)
        self.max_new_tokens, self.temperature = int(max_new_tokens), float(temperature)
        # llama.cpp server sampling defaults + the reference's stop sequences (llamacpp_summarizer.py:111-113)
        from ..ops.kernels import SamplingParams
        self.sampling = SamplingParams(float(temperature), int(top_k), float(top_p), float(min_p))
        if isinstance(stop_sequences, str):
            stop_sequences = json.loads(stop_sequences)
        self.stop_sequences = tuple(s for s in (stop_sequences or ()) if s)
        # the stops are matched on the device as tokens arrive (runtime/stops.py): a thread stops
        # decoding at "\n\n\n" even when it spans several tokens, not after max_new_tokens
        from ..runtime.stops import StopStringMatcher
        self.stop_matcher = StopStringMatcher.for_tokenizer(self.tokenizer, self.stop_sequences)
        self.max_batch = int(max_batch)
        self.ignore_eos = ignore_eos
        self.context_limit = cfg.max_positions - self.max_new_tokens
        self.last_stats: dict = {}

    def gpu_stats(self, res) -> dict:
        """Engine/GPU figures of the last batch (tokens/s, TTFT, HBM use)."""
        gen = sum(len(t) for t in res.tokens)
        st = {"ttft_seconds": res.ttft_s, "prefill_seconds": res.prefill_s, "decode_seconds": res.decode_s,
              "decode_tokens_per_second": gen / res.decode_s if res.decode_s > 0 else 0.0,
              "prefill_tokens_per_second": sum(res.prompt_lens) / res.prefill_s if res.prefill_s > 0 else 0.0,
              "prefix_cached_tokens": res.cached_prompt_tokens, "batch_threads": len(res.tokens)}
        if torch.cuda.is_available() and self.kv.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.kv.device)
            st["hbm_used_bytes"] = total - free
            st["hbm_total_bytes"] = total
            st["kv_cache_bytes"] = self.kv.nbytes()
        return st

    def _tokens(self, prompt: str) -> list[int]:
        ids = self.tokenizer.encode(prompt)
        if len(ids) > self.context_limit:  # keep the head (instructions) and the tail (latest excerpts)
            half = self.context_limit // 2
            ids = ids[:half] + ids[-(self.context_limit - half):]
        return ids

    def summarize_batch(self, threads: list[Thread], token_ids: list[list[int]] | None = None) -> list[Summary]:
        out: list[Summary] = []
        for s in range(0, len(threads), self.max_batch):
            part = threads[s:s + self.max_batch]
            ids = token_ids[s:s + self.max_batch] if token_ids is not None else [self._tokens(t.prompt) for t in part]
            t0 = time.perf_counter()
            res = self.generate_ids(ids)
            ms = int(1000 * (time.perf_counter() - t0))
            self.last_stats = self.gpu_stats(res)
            for t, p, g in zip(part, ids, res.tokens):
                text = self.apply_stops(self.tokenizer.decode(g)).strip() or "(empty summary)"
                out.append(Summary(t.thread_id, text, [], self.backend, self.model, len(p), len(g), ms))
        return out

    # TP leader: called with every engine call's control message before it runs, so the followers
    # (parallel/dp_service.tp_follow -> tp_serve) make the same device calls in lockstep:
    # ("gen", ids) for a static batch, ("cstart", params) / ("cstep", ...) / ("creset",) / ("cstop",)
    # for the continuous engine
    tp_hook = None

    def generate_ids(self, ids: list[list[int]]):
        if self.tp_hook is not None:
            self.tp_hook(("gen", ids))
        return self.engine.generate(ids, self.max_new_tokens, temperature=self.sampling, ignore_eos=self.ignore_eos,
                                    stop_strings=None if self.ignore_eos else self.stop_matcher)

    def tp_serve(self, msg) -> None:
        """TP follower side of one leader message (see ``tp_hook``)."""
        kind = msg[0]
        if kind == "gen":
            self.generate_ids(msg[1])
        elif kind == "cstart":
            self._ce = self._new_continuous(**msg[1])
        elif kind == "cstep":
            self._ce.follow(msg)
        elif kind == "creset":
            self._ce = self._reset_continuous(self._ce)
        elif kind == "cstop":
            if getattr(self, "_ce", None) is not None:
                self._ce.close()
                self._ce = None
        else:
            raise ValueError(f"unknown TP control message {kind!r}")

    def progress(self) -> int:
        """Forward-progress counter for liveness checks (parallel/dp_node.py heartbeat): prefill
        chunks and decode steps of the engine, plus the continuous engine's decode steps.  A host
        counter -- it stops moving when a GPU call hangs."""
        ce = getattr(self, "_ce", None)
        return int(self.engine.progress) + (int(ce.stats.get("steps", 0)) if ce is not None else 0)

    def apply_stops(self, text: str) -> str:
        """Cut at the first stop sequence (string-level stops, as the llama.cpp server applies them)."""
        cut = min((i for i in (text.find(s) for s in self.stop_sequences) if i >= 0), default=-1)
        return text if cut < 0 else text[:cut]

    def summarize(self, thread: Thread) -> Summary:
        return self.summarize_batch([thread])[0]

    # ------------------------------------------------------------ continuous (service) mode
    def _new_continuous(self, steps_per_sync: int, min_admit: int, max_wait_s: float):
        from ..runtime.continuous import ContinuousEngine
        eos = () if self.ignore_eos else (self.cfg.eos_id,)
        return ContinuousEngine(self.engine, max_slots=self.max_batch, max_new_cap=self.max_new_tokens,
                                max_prompt=self.context_limit, steps_per_sync=steps_per_sync, stop_ids=eos,
                                temperature=self.sampling, min_admit=min_admit, max_wait_s=max_wait_s,
                                stop_strings=None if self.ignore_eos else self.stop_matcher, sync=self.tp_hook)

    def start_continuous(self, steps_per_sync: int = 16, min_admit: int = 1, max_wait_s: float = 0.05) -> None:
        """Serve :meth:`submit` ted threads through a ContinuousEngine on a background thread: a
        thread joins the running decode batch at the next burst boundary and leaves it at its stop
        (EOS, a stop string on the device, or max_new_tokens), its slot refilled from the queue --
        no batch-of-N latency for a bursty bus load.  Under tensor
        parallelism the followers build the same engine and replay every step (``tp_hook``)."""
        import collections
        import threading

        if getattr(self, "_ce", None) is not None:
            return
        params = dict(steps_per_sync=steps_per_sync, min_admit=min_admit, max_wait_s=max_wait_s)
        if self.tp_hook is not None:
            self.tp_hook(("cstart", params))
        self._ce = self._new_continuous(**params)
        self._inbox: collections.deque = collections.deque()
        self._cv = threading.Condition()
        self._live: dict = {}
        self._ce_stop = False
        self._ce_thread = threading.Thread(target=self._serve, name="llm-continuous", daemon=True)
        self._ce_thread.start()

    def submit(self, thread: Thread, done) -> None:
        """Queue one thread; ``done(summary, error)`` is called exactly once, from the engine thread
        (with an error when the engine fails or is stopped before the thread finished)."""
        ids = self._tokens(thread.prompt)
        with self._cv:
            if self._ce_stop:
                raise RuntimeError("summarizer is stopping")
            self._inbox.append((thread, ids, time.perf_counter(), done))
            self._cv.notify()

    @staticmethod
    def _deliver(done, summary, error) -> None:
        """One call of a request's callback; a callback that raises is logged, never re-invoked
        (it may already have published its SummaryComplete)."""
        try:
            done(summary, error)
        except Exception as e:  # noqa: BLE001 -- the engine thread must keep serving
            import sys
            print(f"[summarizer] done callback failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)

    def _finish(self, thread, ids, t0, done, toks) -> None:
        try:
            text = self.apply_stops(self.tokenizer.decode(toks)).strip() or "(empty summary)"
            s = Summary(thread.thread_id, text, [], self.backend, self.model, len(ids), len(toks),
                        int(1000 * (time.perf_counter() - t0)))
        except Exception as e:  # noqa: BLE001 -- a decode failure fails this thread alone
            self._deliver(done, None, e)
            return
        self._deliver(done, s, None)

    def _serve(self) -> None:
        from ..services.base import own_gpu_stream
        own_gpu_stream()
        ce = self._ce
        try:
            while True:
                t_idle = time.perf_counter()
                with self._cv:
                    while not self._ce_stop and not self._inbox and not ce.pending():
                        self._cv.wait(0.5)
                    ce.stats["idle_s"] = ce.stats.get("idle_s", 0.0) + time.perf_counter() - t_idle
                    if self._ce_stop:
                        break
                    new = list(self._inbox)
                    self._inbox.clear()
                for item in new:
                    thread, ids, t0, done = item
                    try:
                        r = ce.submit(ids, self.max_new_tokens)
                    except ValueError as e:
                        self._deliver(done, None, e)
                        continue
                    self._live[r.rid] = item
                try:
                    finished = ce.step()
                except Exception as e:  # noqa: BLE001 -- engine failure: every queued / running thread fails
                    live, self._live = list(self._live.values()), {}
                    for item in live:
                        self._deliver(item[3], None, e)
                    self._ce = ce = self._reset_continuous(ce, leader=True)
                    continue
                if not finished and all(x is None for x in ce.slot_req):
                    t_idle = time.perf_counter()
                    with self._cv:      # admission is waiting for more requests: do not spin on the GIL
                        self._cv.wait(0.005)
                    ce.stats["idle_s"] = ce.stats.get("idle_s", 0.0) + time.perf_counter() - t_idle
                t_del = time.perf_counter()
                for r in finished:
                    item = self._live.pop(r.rid, None)
                    if item is not None:
                        self._finish(*item, r.tokens or [])
                if finished:    # detokenize + the service's callback (SummaryComplete publish) per thread
                    ce.stats["deliver_s"] = ce.stats.get("deliver_s", 0.0) + time.perf_counter() - t_del
        finally:
            # stopped (or the thread died): every thread still queued or running gets its failure, so
            # the service publishes SummarizationFailed and releases its in-flight key -- none is
            # dropped silently (the bus message was acked when the request was queued)
            with self._cv:
                left = list(self._inbox) + list(self._live.values())
                self._inbox.clear()
                self._live = {}
            err = RuntimeError("summarizer stopped before the thread finished")
            for item in left:
                self._deliver(item[3], None, err)

    def _reset_continuous(self, ce, leader: bool = False):
        if leader and self.tp_hook is not None:
            self.tp_hook(("creset",))
        try:
            ce.close()
        except Exception:  # noqa: BLE001 -- best effort: the old slots' blocks may be gone with the error
            pass
        return self._new_continuous(ce.steps_per_sync, ce.min_admit, ce.max_wait_s)

    def stop_continuous(self) -> None:
        if getattr(self, "_ce", None) is None:
            return
        with self._cv:
            self._ce_stop = True
            self._cv.notify()
        self._ce_thread.join(timeout=30)
        if self._ce_thread.is_alive():
            return             # a step is still running on the device: leave the engine to it
        if self.tp_hook is not None:
            self.tp_hook(("cstop",))
        self._ce.close()
        self._ce = None


class _HTTPSummarizer(Summarizer):
    """Shared HTTP behaviour of the Ollama / llama.cpp drivers (reference local_llm_summarizer.py,
    llamacpp_summarizer.py): timeouts, connection and HTTP errors raise (infrastructure failures
    the service retries); an empty completion degrades to a fallback text with 0 completion tokens."""

    @staticmethod
    def _check_timeout(timeout):
        if timeout is None or float(timeout) <= 0:
            raise ValueError(f"timeout must be a positive number of seconds, got {timeout!r}")
        return float(timeout)

    def _post(self, url, payload, timeout):
        import requests
        r = requests.post(url, json=payload, timeout=timeout, headers={"Content-Type": "application/json"})
        r.raise_for_status()
        return r.json()

    def _summary(self, thread, text, t0):
        if not text:
            return Summary(thread.thread_id, f"Unable to generate summary for thread {thread.thread_id}", [],
                           self.backend, self.model, len(thread.prompt.split()), 0,
                           int(1000 * (time.perf_counter() - t0)))
        return Summary(thread.thread_id, text, [], self.backend, self.model, len(thread.prompt.split()),
                       len(text.split()), int(1000 * (time.perf_counter() - t0)))


class LocalLLMSummarizer(_HTTPSummarizer):
    """Ollama ``/api/generate`` (reference local_llm_summarizer.py:67,107)."""
    backend = "local"

    def __init__(self, local_llm_model="mistral", local_llm_endpoint="http://ollama:11434",
                 local_llm_timeout_seconds=300, **_):
        if not local_llm_model or not local_llm_endpoint:
            raise ValueError("local LLM driver needs local_llm_model and local_llm_endpoint")
        self.model, self.endpoint = local_llm_model, str(local_llm_endpoint).rstrip("/")
        self.timeout = self._check_timeout(local_llm_timeout_seconds)

    def summarize(self, thread):
        t0 = time.perf_counter()
        d = self._post(f"{self.endpoint}/api/generate", {"model": self.model, "prompt": thread.prompt,
                                                          "stream": False}, self.timeout)
        return self._summary(thread, d.get("response", ""), t0)


class LlamaCppSummarizer(_HTTPSummarizer):
    """llama.cpp server ``/completion`` (reference llamacpp_summarizer.py:68,108-113)."""
    backend = "llamacpp"

    def __init__(self, llamacpp_model="mistral", llamacpp_endpoint="http://llama-cpp:8081",
                 llamacpp_timeout_seconds=300, **_):
        if not llamacpp_model or not llamacpp_endpoint:
            raise ValueError("llama.cpp driver needs llamacpp_model and llamacpp_endpoint")
        self.model, self.endpoint = llamacpp_model, str(llamacpp_endpoint).rstrip("/")
        self.timeout = self._check_timeout(llamacpp_timeout_seconds)

    def summarize(self, thread):
        t0 = time.perf_counter()
        d = self._post(f"{self.endpoint}/completion", {"prompt": thread.prompt, "n_predict": 512, "temperature": 0.7,
                                                        "stop": ["</s>", "\n\n\n"]}, self.timeout)
        return self._summary(thread, d.get("content", ""), t0)


class OpenAISummarizer(Summarizer):
    """OpenAI / Azure OpenAI chat completions over REST (reference openai_summarizer.py:46; no SDK
    needed): one user message with the prompt, ``max_tokens`` = the thread's context window
    (:313-317), 429s retried with full-jitter backoff honouring retry-after (:189-286).  Any
    OpenAI-compatible server works, including this framework's LLM server (serving/llm_server.py)."""
    backend = "openai"

    def __init__(self, openai_api_key=None, openai_model=None, openai_base_url=None, azure_openai_api_key=None,
                 azure_openai_endpoint=None, azure_openai_deployment=None, azure_openai_model=None,
                 azure_openai_api_version=None, max_retries: int = 3, base_backoff_seconds: float = 5.0, **_):
        from ..utils.openai_rest import OpenAIRestClient
        self.is_azure = bool(azure_openai_endpoint and azure_openai_deployment)
        self.client = OpenAIRestClient(
            api_key=azure_openai_api_key if self.is_azure else openai_api_key, base_url=openai_base_url,
            azure_endpoint=azure_openai_endpoint if self.is_azure else None, api_version=azure_openai_api_version,
            deployment=azure_openai_deployment, max_retries=max_retries, base_backoff_seconds=base_backoff_seconds)
        self.model = (azure_openai_deployment if self.is_azure else openai_model) or "gpt-4o-mini"
        self.backend = "azure" if self.is_azure else "openai"

    def summarize(self, thread):
        t0 = time.perf_counter()
        r = self.client.chat(self.model, [{"role": "user", "content": thread.prompt}],
                             max_tokens=thread.context_window_tokens)
        text = r["choices"][0]["message"].get("content")
        if text is None:
            raise AttributeError("OpenAI response message content was None")
        usage = r.get("usage") or {}
        return Summary(thread.thread_id, text, [], self.backend, self.model, int(usage.get("prompt_tokens", 0)),
                       int(usage.get("completion_tokens", 0)), int(1000 * (time.perf_counter() - t0)))


def create_llm_backend(cfg=None, **overrides) -> Summarizer:
    name = str(getattr(cfg, "driver_name", cfg) or "hip").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "hip":
        return HipLLMSummarizer(**kw)
    if name == "mock":
        return MockSummarizer(**kw)
    if name == "local":
        return LocalLLMSummarizer(**kw)
    if name == "llamacpp":
        return LlamaCppSummarizer(**kw)
    if name in ("openai", "azure_openai_gpt"):
        return OpenAISummarizer(**kw)
    raise ValueError(f"unknown llm backend {name!r}")
