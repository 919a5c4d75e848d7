"""The benchmark's unit of work: one batch of threads summarized end to end on one GPU.

The reference's per-thread path it batches: summarization/app/service.py:289 ->
local_llm_summarizer.py:107 (one thread per call); embedding one chunk per call
(embedding/app/service.py:384-393).
"""
from __future__ import annotations

import dataclasses
import os
import random
import time

import torch

from ..observability import span


@dataclasses.dataclass
class StepResult:
    threads: int
    latencies_s: list[float]
    generated_tokens: int
    prompt_tokens: int
    stage_s: dict[str, float]

    def summary(self) -> str:
        st = " ".join(f"{k}={v:.2f}s" for k, v in self.stage_s.items())
        return (f"threads={self.threads} prompt_tok={self.prompt_tokens} gen_tok={self.generated_tokens} "
                f"p50={sorted(self.latencies_s)[len(self.latencies_s) // 2]:.2f}s {st}")


class BenchPipeline:
    def __init__(self, model="mistral-7b", encoder="minilm-l6", device="cuda", threads_per_step=128,
                 max_new_tokens=512, tp=1, prefill_tokens=16384, llm_only=False, use_graph=True, seed=0,
                 index_prefill=1_000_000, groups=None, kv_dtype="bf16", weight_dtype="bf16", kv_max_prompt=4096,
                 index_group=None, overlap_prefill=False):
        from ..models.decoder import DecoderModel, DecoderWeights, get_config
        from ..runtime.engine import LLMEngine
        from ..runtime.kv_cache import PagedKVCache, blocks_needed

        self.groups = groups
        tp_rank = groups.tp_rank if groups is not None else 0
        if groups is not None and groups.tp_size != tp:
            raise ValueError("groups.tp_size != tp")
        if tp > 1 and groups is None:
            raise ValueError("tp > 1 needs process groups (parallel.make_groups)")
        # TP followers run the LLM only; the leader prepares the batch and broadcasts the prompts
        self.follower = tp > 1 and tp_rank != 0
        self.device = torch.device(device)
        self.cfg = get_config(model)
        self.threads_per_step = threads_per_step
        self.max_new = max_new_tokens
        self.llm_only = llm_only
        self.rng = random.Random(seed)
        self.seed = seed
        w = DecoderWeights.random(self.cfg, self.device, seed=1234, tp_rank=tp_rank, tp_size=tp)
        if weight_dtype == "fp8":
            w.to_fp8()           # opt-in W8A8 FP8 projections (precision trade-off, not the headline)
        custom_ar = None
        if tp > 1:
            from ..parallel.custom_ar import maybe_create
            custom_ar = maybe_create(groups.tp_group, self.device, exchange_group=groups.tp_cpu_group)
        self.model = DecoderModel(w, tp_group=groups.tp_group if tp > 1 else None, custom_ar=custom_ar)
        # KV budget: every thread of a step at ``kv_max_prompt`` prompt tokens + max_new, x1.1 (the
        # prompts this pipeline builds stay near 2.6k; a 70B model on one GPU needs the tighter bound)
        max_prompt = int(kv_max_prompt)
        # prefill of batch i+1 beside the decode of batch i (run_steps_overlapped): two batches' KV
        self.overlap_prefill = bool(overlap_prefill) and tp == 1 and self.device.type == "cuda"
        nblk = int(1.1 * threads_per_step * blocks_needed(max_prompt + max_new_tokens)) + 64
        if self.overlap_prefill:
            nblk *= 2
        kvd = {"bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn}[kv_dtype]
        self.kv = PagedKVCache(self.cfg.layers, nblk, w.kv_heads, self.cfg.head_dim, self.device, dtype=kvd)
        self.engine = LLMEngine(self.model, self.kv, max_prefill_tokens=prefill_tokens, use_graph=use_graph)
        self.rag = None
        # the next batch's encoder / kNN work runs on this stream beside the decode graph.  Its kernels
        # only get CUs the decode's workgroups leave free, so alone 0.15 s of encoder work stretches to
        # ~0.9 s of wall time (BENCH_r03 embed stage); CFC_PREP_STREAM_PRIORITY=high dispatches them
        # ahead of the decode's queued workgroups instead (shorter embed stage, decode pays its GPU time)
        prio = -1 if os.environ.get("CFC_PREP_STREAM_PRIORITY", "normal") == "high" else 0
        self.side_stream = torch.cuda.Stream(self.device, priority=prio) if self.device.type == "cuda" else None
        self._last_gen_s: float | None = None
        self._last_prep_s = 0.0
        # just-in-time preparation: batch i+1's CPU + encoder stages start so they end
        # ``margin`` x (the slowest of the last 4 preparations) + ``slack`` s before batch i's LLM
        # work does -- a thread's latency counts from its preparation's start, so an early start is
        # latency with no throughput in it (wait_prep in the step summary shows a late one).
        # 2.0 / 0.25 -> 1.25 / 0.1: saturated p50 10.8-11.0 -> 10.3 s at unchanged throughput, 0.01-0.09 s
        # of wait_prep over 20 steps (profiles/r05_ab_prep_margin.log)
        self._prep_hist: list[float] = []
        self.prep_margin = float(os.environ.get("CFC_PREP_MARGIN", "1.25"))
        self.prep_slack_s = float(os.environ.get("CFC_PREP_SLACK_S", "0.1"))
        if not llm_only and not self.follower:
            from ..bus import CountingPublisher
            from .rag import RagPipeline
            self.events = CountingPublisher()
            self.rag = RagPipeline(encoder=encoder, device=self.device, decoder_vocab=self.cfg.vocab_size,
                                   bos_id=self.cfg.bos_id, seed=seed, publisher=self.events, llm_model=model,
                                   max_prompt_tokens=self.cfg.max_positions - max_new_tokens,
                                   index_prefill=index_prefill, index_group=index_group)

    def prepare_sources(self, steps: list[int]) -> None:
        """Generate the synthetic archives of the given steps up front (outside the timed region)."""
        if self.rag is not None and not self.follower:
            self.rag.prepare_sources(self.threads_per_step, steps)

    def _synthetic_prompts(self, n):
        # ~2.5-3k prompt tokens: BASELINE.md "prefill of about 2.5k-3k tokens"
        out = []
        for _ in range(n):
            L = self.rng.randint(2560, 3072)
            out.append([self.cfg.bos_id] + [self.rng.randrange(3, self.cfg.vocab_size) for _ in range(L - 1)])
        return out

    def _prepare(self, step: int, not_before: float | None = None):
        if not_before is not None:
            # just-in-time: start this batch's CPU/encoder work so it completes as the running
            # LLM batch drains -- overlapped, but the threads do not queue behind a whole batch
            delay = not_before - time.perf_counter()
            if delay > 0:
                time.sleep(delay)
        t0 = time.perf_counter()
        if self.groups is not None and self.groups.tp_size > 1:
            return self._prepare_tp(t0, step)
        if self.rag is None:
            return t0, None, self._synthetic_prompts(self.threads_per_step), {}
        with span(f"bench.prepare.step{step}"):
            return self._prepare_rag(t0, step)

    def _prepare_tp(self, t0, step):
        import torch.distributed as dist
        g = self.groups
        if self.follower:
            box = [None]
            dist.broadcast_object_list(box, src=g.tp_src, group=g.tp_cpu_group)
            return t0, None, box[0], {}
        if self.rag is None:
            t0, ctx, prompts, stages = t0, None, self._synthetic_prompts(self.threads_per_step), {}
        else:
            t0, ctx, prompts, stages = self._prepare_rag(t0, step)
        dist.broadcast_object_list([prompts], src=g.tp_src, group=g.tp_cpu_group)
        return t0, ctx, prompts, stages

    def _prepare_rag(self, t0, step):
        if self.device.type == "cuda":
            # the encoder / kNN work of this batch runs on its own stream, beside the decode graph
            with torch.cuda.stream(self.side_stream):
                ctx = self.rag.prepare(self.threads_per_step, step)
                self.side_stream.synchronize()
        else:
            ctx = self.rag.prepare(self.threads_per_step, step)
        return t0, ctx, ctx.prompts, dict(ctx.stage_s)

    def run_steps(self, steps: list[int], overlap: bool = True, on_step=None) -> list[StepResult]:
        """Run batches back to back.  With ``overlap`` the CPU + encoder stages of batch i+1 run on
        a worker thread (and a side HIP stream) while batch i is in the LLM; batch 0 is prepared
        inline so exactly the listed batches' work happens inside the caller's timing window."""
        import concurrent.futures as cf
        results = []
        if not steps:
            return results
        pool = cf.ThreadPoolExecutor(1) if overlap else None
        pending = self._prepare(steps[0])
        try:
            for n, step in enumerate(steps):
                t0, ctx, prompts, stages = pending
                fut = None
                if pool and n + 1 < len(steps):
                    start_at = None
                    if self._last_gen_s is not None:
                        lead = self.prep_margin * max(self._prep_hist) + self.prep_slack_s
                        start_at = time.perf_counter() + max(0.0, self._last_gen_s - lead)
                    fut = pool.submit(self._prepare, steps[n + 1], start_at)
                tg = time.perf_counter()
                with span(f"bench.llm.step{step}"):
                    res = self.engine.generate(prompts, self.max_new, temperature=0.0, ignore_eos=True)
                self._last_gen_s = time.perf_counter() - tg
                self._last_prep_s = sum(v for k, v in stages.items() if k != "wait_prep")
                self._prep_hist = (self._prep_hist + [self._last_prep_s])[-4:]
                stages["prefill"] = res.prefill_s
                stages["decode"] = res.decode_s
                # engine time outside its prefill / decode windows (setup, first-token sync, harvest)
                stages["llm_other"] = self._last_gen_s - res.prefill_s - res.decode_s
                t2 = time.perf_counter()
                if ctx is not None:
                    self.rag.finish(ctx, res)
                    stages["report"] = time.perf_counter() - t2
                t3 = time.perf_counter()
                stages["total"] = t3 - t0
                n_thr = 0 if self.follower else len(prompts)  # a TP group counts its threads once
                results.append(StepResult(n_thr, [t3 - t0] * n_thr, sum(len(t) for t in res.tokens),
                                          sum(res.prompt_lens), stages))
                if on_step is not None:   # progress report (host-side print, no device sync)
                    on_step(n, results[-1])
                tw = time.perf_counter()
                if fut is not None:
                    pending = fut.result()
                elif n + 1 < len(steps):
                    pending = self._prepare(steps[n + 1])
                if n + 1 < len(steps):       # the next batch's preparation not hidden behind this one
                    pending[3]["wait_prep"] = time.perf_counter() - tw
        finally:
            if pool:
                pool.shutdown(wait=True)
        return results

    def run_steps_overlapped(self, steps: list[int], on_step=None) -> list[StepResult]:
        """Batch i+1's preparation AND prefill run on a worker thread while batch i decodes: the
        prefill on one half of the CUs, the decode on the other half until that prefill is done,
        then on the whole GPU (runtime/cu_partition.py).  Batch 0 is prepared and prefilled inline
        on the whole GPU, so exactly the listed batches' work happens inside the caller's window.
        Two decode states (slots 0 / 1) and two batches of KV blocks are live at a time."""
        import concurrent.futures as cf

        import os

        from ..runtime.cu_partition import partition_streams, priority_streams
        results = []
        if not steps:
            return results
        full = torch.cuda.current_stream(self.device)
        if getattr(self, "_partitions", None) is None:
            # CFC_OVERLAP_MODE: cumask = disjoint CU halves; priority = whole chip, decode stream first
            mode = os.environ.get("CFC_OVERLAP_MODE", "cumask")
            self._partitions = priority_streams(self.device) if mode == "priority" else partition_streams(self.device)
        sp, sd = self._partitions

        def prep_and_start(step, slot, stream):
            t0, ctx, prompts, stages = self._prepare(step)
            with torch.cuda.stream(stream):
                job = self.engine.start(prompts, self.max_new, temperature=0.0, ignore_eos=True, slot=slot,
                                        stream_sync=True)
            return t0, ctx, prompts, stages, job

        pool = cf.ThreadPoolExecutor(1)
        pending = prep_and_start(steps[0], steps[0] % 2, full)
        try:
            for n, step in enumerate(steps):
                t0, ctx, prompts, stages, job = pending
                fut = None
                if n + 1 < len(steps):
                    fut = pool.submit(prep_and_start, steps[n + 1], steps[n + 1] % 2, sp)
                with span(f"bench.llm.step{step}"):
                    if fut is not None:
                        with torch.cuda.stream(sd):
                            res = self.engine.finish(job, switch=lambda f=fut: full if f.done() else None)
                    else:
                        res = self.engine.finish(job)
                stages["prefill"] = res.prefill_s
                stages["decode"] = res.decode_s
                t2 = time.perf_counter()
                if ctx is not None:
                    self.rag.finish(ctx, res)
                    stages["report"] = time.perf_counter() - t2
                t3 = time.perf_counter()
                stages["total"] = t3 - t0
                results.append(StepResult(len(prompts), [t3 - t0] * len(prompts), sum(len(t) for t in res.tokens),
                                          sum(res.prompt_lens), stages))
                if on_step is not None:
                    on_step(n, results[-1])
                if fut is not None:
                    pending = fut.result()
        finally:
            pool.shutdown(wait=True)
        return results

    def run_step(self, step: int) -> StepResult:
        return self.run_steps([step], overlap=False)[0]

    def search_probe(self, n_queries: int = 64, limit: int = 50, seed: int = 0) -> dict | None:
        """Topic-search latency through the reporting service (RagPipeline.search_probe); None on
        ranks without the RAG stages (TP followers, --llm-only)."""
        if self.rag is None:
            return None
        if self.device.type == "cuda":
            with torch.cuda.stream(self.side_stream):
                return self.rag.search_probe(n_queries, limit, seed)
        return self.rag.search_probe(n_queries, limit, seed)

    def latency_probe(self, steps: list[int], rate_per_s: float, seed: int = 0, steps_per_sync: int = 16,
                      max_threads: int | None = None) -> dict:
        """The latency half of the metric under load below saturation: the threads of ``steps``
        (prepared by the same RAG path as the throughput steps) arrive as a Poisson process of
        ``rate_per_s`` and are served by the continuous engine (runtime/continuous.py -- the
        summarization service's engine): a thread joins the running decode batch at the next burst
        boundary and leaves it after its 512 tokens.  Latency = its batch's whole preparation time
        (parse / chunk / embed / select of the step it came from: the thread could not be submitted
        before that batch was prepared) + arrival -> last token.  Not in the timed throughput window.
        Under tensor parallelism the TP followers replay every engine step the leader takes (the
        leader's ``sync`` messages over the TP group's CPU twin, as the summarization service's
        followers do) and return {}."""
        import numpy as np

        from ..runtime.continuous import ContinuousEngine
        prompts, prep_of = [], []
        for st in steps:
            _, ctx, p, stages = self._prepare(st)
            prep = sum(v for k, v in stages.items() if k != "wait_prep")
            prompts.extend(p)
            prep_of.extend([prep] * len(p))
        if not prompts:
            return {}
        if max_threads is not None:
            prompts, prep_of = prompts[:max_threads], prep_of[:max_threads]
        params = dict(max_slots=self.threads_per_step, max_new_cap=self.max_new, max_prompt=max(len(x) for x in prompts),
                      steps_per_sync=steps_per_sync, stop_ids=(), min_admit=1, max_wait_s=0.05)
        tp = self.groups is not None and self.groups.tp_size > 1
        if tp:
            import torch.distributed as dist
            g = self.groups

            def bcast(msg):
                box = [msg]
                dist.broadcast_object_list(box, src=g.tp_src, group=g.tp_cpu_group)
                return box[0]
            if self.follower:
                ce = ContinuousEngine(self.engine, **params)
                try:
                    while (msg := bcast(None)) is not None:
                        ce.follow(msg)
                finally:
                    ce.close()
                return {}
            ce = ContinuousEngine(self.engine, **params, sync=bcast)
        else:
            ce = ContinuousEngine(self.engine, **params)
        rng = np.random.default_rng(seed)
        arrive = np.cumsum(rng.exponential(1.0 / float(rate_per_s), len(prompts)))
        t0 = time.perf_counter()
        nxt, lat, arrival_of = 0, [], {}
        try:
            while nxt < len(prompts) or ce.pending():
                now = time.perf_counter() - t0
                while nxt < len(prompts) and arrive[nxt] <= now:
                    r = ce.submit(prompts[nxt], self.max_new)
                    arrival_of[r.rid] = (t0 + float(arrive[nxt]), prep_of[nxt])
                    nxt += 1
                if ce.pending():
                    for r in ce.step():
                        at, prep = arrival_of.pop(r.rid)
                        lat.append(r.finished_s - at + prep)
                elif nxt < len(prompts):
                    time.sleep(max(0.0, float(arrive[nxt]) - (time.perf_counter() - t0)))
        finally:
            if tp:
                bcast(None)               # the followers leave their replay loop
            ce.close()
        wall = time.perf_counter() - t0
        lat = np.asarray(lat)
        return {"arrival_rate_per_gpu": float(rate_per_s), "threads": int(len(lat)),
                "p50_s": round(float(np.percentile(lat, 50)), 3), "p95_s": round(float(np.percentile(lat, 95)), 3),
                "throughput_threads_per_s": round(len(lat) / wall, 3),
                "prep_per_thread_s": round(float(np.mean(prep_of)), 4),
                "prep_charged": "the thread's whole batch preparation",
                "engine": f"continuous ({self.threads_per_step} slots, {steps_per_sync} decode steps per admission)"
                          + (f", TP={self.groups.tp_size}" if tp else "")}
