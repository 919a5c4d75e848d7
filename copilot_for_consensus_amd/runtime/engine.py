"""Batched LLM generation engine (prefill + hipGraph-captured decode) over the paged KV cache.

The reference summarizes one thread at a time per replica with a blocking HTTP call to
Ollama/llama.cpp (summarization/app/service.py:289; local_llm_summarizer.py:107).  Here a
batch of threads is generated together:

  1. packed varlen prefill in chunks of ``max_prefill_tokens`` (large GEMMs for the ping-pong MFMA GEMM, our
     flash prefill kernel over the paged cache; long prompts are split = chunked prefill);
  2. one decode step = embedding -> 32 x (RMSNorm, QKV GEMM, RoPE+KV write, paged decode
     attention, O GEMM, RMSNorm, gate|up GEMM, SwiGLU, down GEMM) -> lm_head -> sampler ->
     on-device state advance.  The whole step is captured once in a hipGraph and replayed
     ``max_new_tokens-1`` times with NO host work or sync in between (EOS/stop flags live on the
     device and are polled every ``stop_check_interval`` steps).
"""
from __future__ import annotations

import dataclasses
import math
import os
import threading
import time

import numpy as np
import torch

from ..observability import span
from ..ops import kernels as K
from ..ops.reference import KV_BLOCK
from .kv_cache import PagedKVCache, blocks_needed
from .prefix_cache import PrefixCache


@dataclasses.dataclass
class GenerationResult:
    tokens: list[list[int]]          # generated ids per prompt (stop token excluded)
    prompt_lens: list[int]
    prefill_s: float = 0.0
    decode_s: float = 0.0
    ttft_s: float = 0.0
    decode_steps: int = 0
    cached_prompt_tokens: int = 0    # prompt tokens served from the prefix cache

    @property
    def total_s(self) -> float:
        return self.prefill_s + self.decode_s


@dataclasses.dataclass
class _Job:
    """A prefilled batch waiting for (or in) its decode: LLMEngine.start -> LLMEngine.finish."""
    st: object
    tables: list
    fresh: list
    lens: list
    start: list
    B: int
    max_new: int
    stop_ids: tuple
    stop_strings: object
    part_blocks: int
    temperature: object
    seed: int
    prefill_s: float
    ready: object = None          # event recorded after the state setup (stream handoff)
    order: list | None = None     # slot s holds caller prompt order[s] (longest-first slots)


class _DecodeState:
    """Static device buffers a captured decode graph reads and writes."""

    def __init__(self, B, max_blocks, max_new, device, n_part_ws):
        i32 = dict(dtype=torch.int32, device=device)
        self.ids = torch.zeros(B, **i32)
        self.positions = torch.zeros(B, **i32)
        self.ctx_lens = torch.ones(B, **i32)
        self.slots = torch.zeros(B, **i32)
        self.block_tables = torch.zeros(B, max_blocks, **i32)
        self.step = torch.zeros(1, **i32)
        self.shared = torch.zeros(1, **i32)     # leading KV blocks all rows share (read cached)
        self.tokens = torch.zeros(B, max_new, **i32)
        self.done = torch.zeros(B, **i32)
        self.next_ids = torch.zeros(B, **i32)
        self.stop_ids = torch.zeros(0, **i32)
        self.stop_state = None     # runtime.stops.StopState when the request has stop strings
        self.workspace = torch.empty(max(1, n_part_ws), dtype=torch.float32, device=device)
        self.graph = None

    def tensors(self):
        extra = [self.stop_state.win, self.stop_state.wlen, self.stop_state.keep] if self.stop_state else []
        return [self.ids, self.positions, self.ctx_lens, self.slots, self.block_tables, self.step, self.tokens,
                self.done, self.next_ids] + extra


class LLMEngine:
    def __init__(self, model, kv: PagedKVCache, max_prefill_tokens: int = 16384, use_graph: bool = True,
                 stop_check_interval: int = 64, prefix_cache: bool | None = None):
        self.model = model
        self.cfg = model.cfg
        self.kv = kv
        self.device = kv.device
        self.max_prefill_tokens = max_prefill_tokens
        self.use_graph = use_graph and kv.device.type == "cuda"
        tp_group = getattr(model, "tp_group", None)
        # gloo collectives cannot be captured in a hipGraph (RCCL's can): with a gloo TP group a
        # step is captured only when every collective in it runs on the one-shot IPC kernels
        # (greedy decode: o/down all-reduces + the argmax key reduce; see _graph_for)
        self._gloo_tp = False
        if tp_group is not None and getattr(model.w, "tp_size", 1) > 1:
            import torch.distributed as dist
            self._gloo_tp = dist.get_backend(tp_group) == "gloo"
        self.last_used_graph = False
        # query rows per prefill attention tile (the GQA-packed kernel takes 256 / G)
        self._prefill_rows = (K.prefill_rows(model.w.heads, model.w.kv_heads) if kv.device.type == "cuda"
                              else K.PREFILL_TILE_ROWS)
        self.stop_check_interval = stop_check_interval
        # host-side forward-progress counter (prefill chunks + decode steps issued): read by the DP
        # heartbeat (parallel/dp_node.py), it freezes when a GPU call hangs and the host blocks
        self.progress = 0
        self._states: dict[tuple, _DecodeState] = {}
        self._alloc_lock = threading.RLock()     # KV / prefix-cache bookkeeping of start / finish
        # shared-prefix reuse of whole KV blocks (system prompt + template head of every thread)
        if prefix_cache is None:
            prefix_cache = os.environ.get("CFC_PREFIX_CACHE", "1") != "0"
        self.prefix_cache = PrefixCache(kv.pool) if prefix_cache else None
        # CFC_DECODE_SHARED_CACHED=0: every KV block nontemporal, shared prefix included
        self.shared_cached = os.environ.get("CFC_DECODE_SHARED_CACHED", "1") != "0"
        # slots filled longest prompt first (CFC_DECODE_LPT=0: caller order).  The decode attention
        # grid walks the slots in order (blockIdx.z = slot), so the longest sequences' workgroups are
        # dispatched first and the short ones fill the CUs that free up (longest-processing-time-
        # first list scheduling) instead of a random long one ending the kernel alone: decode 6.03 ->
        # 5.88 s per 128-thread batch (profiles/r05_ab_decode_lpt.log)
        self.lpt = os.environ.get("CFC_DECODE_LPT", "1") != "0"
        # TP > 1, opt-in (CFC_TP_PREFILL_OVERLAP=1): prefill chunks as two interleaved halves, each
        # half's all-reduces (async, on the process group) under the other half's GEMMs.  Numerics
        # and the one-shot all-reduce's epoch bookkeeping checked on the CPU
        # (tests/test_parallel_cpu.py); the TP=2 rehearsal on one GPU (gloo) runs it to completion
        # with the one-shot all-reduce's error counter at 0 and identical per-block epochs on both
        # ranks after every batch (profiles/r06_tp2_overlap_gloo_1gpu.log).  The round-5 rehearsal
        # that stopped at its 150 s limit inside the second batch's decode graph was rerun this way
        # and completed: no all-reduce timed out and no epoch desync -- not reproduced.
        # Not measured on a multi-GPU node (RCCL), so it stays opt-in.
        self.tp_overlap = os.environ.get("CFC_TP_PREFILL_OVERLAP", "0") in ("1", "force")
        # CFC_AR_DEBUG=1: print the one-shot all-reduce's error counter and epochs per batch
        self._ar_debug = os.environ.get("CFC_AR_DEBUG", "0") == "1"
        if self.device.type == "cuda":
            from .gemm_tuning import enable_tuned_gemms
            self.tuned_gemms = enable_tuned_gemms()

    # ------------------------------------------------------------------ helpers
    def _part_blocks(self, B, max_blocks):
        """Split-KV partitioning of the decode attention, as ``-P``: each sequence's own blocks in
        P balanced ranges, P the smallest giving >= CFC_DECODE_WGS workgroups (default 512, two per
        CU).  Long KV runs per workgroup win: at B=128 P=1 streams 6.5 TB/s vs 5.0-5.4 for fixed
        26-block partitions (scripts/bench_decode_attn.py, profiles/decode_attn_partitions_r01.log)."""
        target = int(os.environ.get("CFC_DECODE_WGS", "512"))
        P = max(1, math.ceil(target / max(1, B * self.model.w.kv_heads)))
        return -min(P, max(1, max_blocks // 2))

    def _i32(self, x):
        return torch.tensor(x, dtype=torch.int32, device=self.device)

    def _ar_trace(self, tag):
        """CFC_AR_DEBUG=1: this rank's one-shot all-reduce error count and per-block epochs."""
        ar = getattr(self.model, "custom_ar", None)
        if self._ar_debug and ar is not None:
            torch.cuda.synchronize(self.device)
            ep = ar.epochs.tolist()
            print(f"[ar-debug] rank {ar.rank} {tag}: errors={ar.errors()} epochs[0:4]={ep[:4]} "
                  f"epochs[32]={ep[32]} key={ep[-1]} distinct={sorted(set(ep))[:6]}", flush=True)

    def _prefill(self, prompts, tables, temperature, seed, start=None):
        """Chunked packed prefill; returns first sampled token per prompt.  ``start[s]`` tokens of
        prompt s are already in the cache (shared prefix blocks)."""
        n = len(prompts)
        first_dev = torch.zeros(n, dtype=torch.int32, device=self.device)
        pos = list(start) if start is not None else [0] * n  # tokens of each prompt already in the cache
        order = list(range(n))
        while order:
            chunk, budget = [], self.max_prefill_tokens
            for s in list(order):
                if budget <= 0:
                    break
                take = min(len(prompts[s]) - pos[s], budget)
                chunk.append((s, pos[s], pos[s] + take))
                budget -= take
                if pos[s] + take == len(prompts[s]):
                    order.remove(s)
                else:
                    break  # a split sequence ends the chunk
            halves = self._overlap_split(chunk)
            metas = [self._chunk_meta(prompts, tables, part) for part in halves]
            if len(metas) == 2:
                hiddens = self.model.forward_prefill_overlap([m[0] for m in metas], self.kv)
            else:
                hiddens = [self.model.forward_prefill(**metas[0][0], kv=self.kv)]
            for (_, finishing, d_fin), hidden in zip(metas, hiddens):
                if finishing:
                    out = torch.empty(len(finishing), dtype=torch.int32, device=self.device)
                    self._next_tokens(hidden, out, temperature, seed,
                                      torch.zeros(1, dtype=torch.int32, device=self.device))
                    first_dev.index_copy_(0, d_fin.long(), out)
            for (s, _, b) in chunk:
                pos[s] = b
            self.progress += 1
        return first_dev.tolist()      # the one host sync of the prefill

    def _overlap_split(self, chunk):
        """TP > 1: a prefill chunk of >= 2 sequences as two halves of whole sequences (token counts
        balanced), run interleaved so each half's row-parallel all-reduces hide under the other
        half's GEMMs (DecoderModel.forward_prefill_overlap); opt-in, CFC_TP_PREFILL_OVERLAP=1."""
        if (len(chunk) < 2 or not self.tp_overlap
                or not getattr(self.model, "supports_prefill_overlap", lambda: False)()):
            return [chunk]
        sizes = [b - a for (_, a, b) in chunk]
        total, acc, best = sum(sizes), 0, (None, 1)
        for k in range(1, len(chunk)):
            acc += sizes[k - 1]
            d = abs(2 * acc - total)
            if best[0] is None or d < best[0]:
                best = (d, k)
        k = best[1]
        return [chunk[:k], chunk[k:]]

    def _chunk_meta(self, prompts, tables, chunk):
        """Device metadata of one packed prefill pass over ``chunk`` [(seq, first, end)]: the
        forward_prefill keyword arguments, the sequences finishing in it, and their ids on device."""
        cu, ctx, rows, last_rows, finishing = [0], [], [], [], []
        ids_np, pos_np, slot_np = [], [], []
        for (s, a, b) in chunk:
            ids_np.append(np.asarray(prompts[s][a:b], dtype=np.int32))
            p = np.arange(a, b, dtype=np.int32)
            pos_np.append(p)
            slot_np.append(np.asarray(tables[s], dtype=np.int32)[p // KV_BLOCK] * KV_BLOCK + p % KV_BLOCK)
            cu.append(cu[-1] + (b - a))
            ctx.append(b)
            rows.append(s)
            if b == len(prompts[s]):
                last_rows.append(cu[-1] - 1)
                finishing.append(s)
        maxb = max(len(tables[s]) for s in rows)
        bt = np.zeros((len(rows), maxb), dtype=np.int32)
        for r, s in enumerate(rows):
            bt[r, :len(tables[s])] = tables[s]
        tseq, tq0 = K.prefill_tiles(cu, self._prefill_rows, ctx)
        # everything the pass needs in ONE pinned host buffer and one non-blocking copy: a
        # pageable torch.tensor(..., device=cuda) synchronises the stream, so the GPU would idle
        # while the host builds the next chunk
        slots_np = np.concatenate(slot_np)
        runs = K.v_runs(slots_np)
        parts = [np.concatenate(ids_np), np.concatenate(pos_np), slots_np,
                 np.asarray(cu, np.int32), np.asarray(ctx, np.int32), np.asarray(tseq, np.int32),
                 np.asarray(tq0, np.int32), np.asarray(last_rows, np.int32),
                 np.asarray(finishing, np.int32), bt.reshape(-1), runs.reshape(-1)]
        dev = self._h2d(np.concatenate(parts))
        offs = np.cumsum([0] + [len(x) for x in parts]).tolist()
        d_ids, d_pos, d_slots, d_cu, d_ctx, d_tseq, d_tq0, d_last, d_fin, d_bt, d_runs = (
            dev[offs[i]:offs[i + 1]] for i in range(len(parts)))
        kw = dict(ids=d_ids, positions=d_pos, slots=d_slots, cu_q=d_cu, ctx_lens=d_ctx,
                  block_tables=d_bt.view(len(rows), maxb), tiles=(d_tseq, d_tq0),
                  last_idx=d_last.long() if last_rows else None, v_runs=d_runs.view(-1, 4))
        return kw, finishing, d_fin

    def _h2d(self, a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(a)
        if self.device.type != "cuda":
            return t.clone()
        return t.pin_memory().to(self.device, non_blocking=True)

    def _tp_greedy(self, temperature) -> bool:
        return getattr(self.model.w, "tp_size", 1) > 1 and K.SamplingParams.of(temperature).temperature <= 0

    def _graph_for(self, B, temperature) -> bool:
        if not self.use_graph:
            return False
        if self._gloo_tp:
            return self._tp_greedy(temperature) and self.model.graph_collectives_ok(B)
        return True

    def _next_tokens(self, hidden, out, temperature, seed, step):
        """Sample the next token of every row; TP greedy reduces (max, argmax) keys instead of
        all-gathering the logits (DecoderModel.greedy_ids)."""
        if self._tp_greedy(temperature):
            return self.model.greedy_ids(hidden, out)
        return K.sample(self.model.logits(hidden), out, temperature, seed, step)

    def _decode_step(self, st: _DecodeState, part_blocks, temperature, seed):
        hidden = self.model.forward_decode(st.ids, st.positions, st.slots, st.ctx_lens, st.block_tables, self.kv,
                                           attn_workspace=st.workspace, part_blocks=part_blocks,
                                           shared_blocks=st.shared)
        self._next_tokens(hidden, st.next_ids, temperature, seed, st.step)
        K.decode_advance(st.next_ids, st.tokens, st.step, st.ids, st.positions, st.ctx_lens, st.slots,
                         st.block_tables, st.done, st.stop_ids, st.stop_state)

    def _state(self, B, max_blocks, max_new, part_blocks, stop_ids, stop_strings=None, slot=0):
        key = (B, max_blocks, max_new, tuple(stop_ids), id(stop_strings) if stop_strings is not None else None, slot)
        st = self._states.get(key)
        if st is None:
            P = -part_blocks if part_blocks < 0 else math.ceil(max_blocks / part_blocks)
            ws = B * self.model.w.heads * P * (self.cfg.head_dim + 2) if P > 1 else 1
            st = _DecodeState(B, max_blocks, max_new, self.device, ws)
            # persistent: a captured graph holds these pointers
            st.stop_ids = torch.tensor(list(stop_ids), dtype=torch.int32, device=self.device)
            if stop_strings is not None:
                st.stop_state = stop_strings.new_state(B, self.device)
                st.stop_matcher = stop_strings      # keeps id(stop_strings) in the key valid
            self._states[key] = st
        return st

    def capture_stream(self):
        """One side stream per engine for every decode-graph warm-up AND capture: the split-K
        workspaces are per stream (ops.kernels._workspace), so the warm-up sizes exactly the
        buffers the capture then records, and captures do not mint a workspace per stream."""
        if getattr(self, "_capture_s", None) is None:
            self._capture_s = torch.cuda.Stream(device=self.device)
        return self._capture_s

    def _capture(self, st, part_blocks, temperature, seed):
        saved = [t.clone() for t in st.tensors()]
        s = self.capture_stream()
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._decode_step(st, part_blocks, temperature, seed)
        torch.cuda.current_stream(self.device).wait_stream(s)
        for t, v in zip(st.tensors(), saved):
            t.copy_(v)
        g = torch.cuda.CUDAGraph()
        # other threads may use the GPU (thread_local); captured on the warm-up's stream
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            self._decode_step(st, part_blocks, temperature, seed)
        for t, v in zip(st.tensors(), saved):
            t.copy_(v)
        st.graph = (g, part_blocks, temperature, seed)

    # ------------------------------------------------------------------ API
    @torch.inference_mode()
    def generate(self, prompts: list[list[int]], max_new_tokens: int, temperature: float = 0.0, seed: int = 0,
                 stop_ids: tuple[int, ...] = (), ignore_eos: bool = False, top_k: int = 0, top_p: float = 1.0,
                 min_p: float = 0.0, stop_strings=None) -> GenerationResult:
        """``temperature`` (or a :class:`ops.kernels.SamplingParams`) with optional top-k / top-p /
        min-p truncation -- all applied on device inside the captured decode step.
        ``stop_strings`` (runtime.stops.StopStringMatcher): a sequence finishes, on the device, at
        the token whose text completes a stop string; its tokens end with that token (the caller
        cuts the text at the stop, as llama.cpp's server does)."""
        if top_k or top_p < 1.0 or min_p > 0.0:
            temperature = K.SamplingParams(float(temperature), int(top_k), float(top_p), float(min_p))
        else:
            temperature = K.SamplingParams.of(temperature)
        B = len(prompts)
        if B == 0:
            return GenerationResult([], [])
        if any(len(p) == 0 for p in prompts):
            raise ValueError("empty prompt")
        if not ignore_eos and self.cfg.eos_id not in stop_ids:
            stop_ids = tuple(stop_ids) + (self.cfg.eos_id,)
        if ignore_eos:
            stop_ids = ()
        job = self.start(prompts, max_new_tokens, temperature, seed, stop_ids, stop_strings=stop_strings,
                         _resolved=True)
        return self.finish(job)

    @torch.inference_mode()
    def start(self, prompts: list[list[int]], max_new_tokens: int, temperature=0.0, seed: int = 0,
              stop_ids: tuple[int, ...] = (), ignore_eos: bool = False, stop_strings=None, slot: int = 0,
              stream_sync: bool = False, _resolved: bool = False) -> _Job:
        """First half of :meth:`generate`: KV allocation, the chunked prefill and the decode state
        of the batch.  ``slot`` picks one of several decode states (and captured graphs) of the same
        shape, so a batch can be prefilled while another one decodes; ``stream_sync`` waits on the
        current stream only (not the device) -- the other batch's decode keeps running.  A
        thread-safe pair with :meth:`finish` (allocation and release are serialised)."""
        if not _resolved:
            temperature = K.SamplingParams.of(temperature)
            if not ignore_eos and self.cfg.eos_id not in stop_ids:
                stop_ids = tuple(stop_ids) + (self.cfg.eos_id,)
            if ignore_eos:
                stop_ids = ()
        B = len(prompts)
        order = None
        if self.lpt and B > 1:
            order = sorted(range(B), key=lambda i: -len(prompts[i]))
            prompts = [prompts[i] for i in order]
        lens = [len(p) for p in prompts]
        if max(lens) + max_new_tokens > self.cfg.max_positions:
            raise ValueError("prompt + max_new_tokens exceeds max_positions")
        # round the block-table width up so graphs are reused across batches of similar length
        need = [blocks_needed(n + max_new_tokens) for n in lens]
        max_blocks = 8 * math.ceil(max(need) / 8)
        pc = self.prefix_cache
        tables, start, fresh = [], [], []
        with self._alloc_lock:
            try:
                for p, n in zip(prompts, need):
                    shared = pc.acquire(p) if pc is not None else []
                    tables.append(shared)       # registered before alloc so a failure releases it
                    new = pc.alloc(n - len(shared)) if pc is not None else self.kv.pool.alloc(n)
                    fresh.append(new)
                    tables[-1] = shared + new
                    start.append(len(shared) * KV_BLOCK)
                    if pc is not None:
                        pc.insert(p, tables[-1])
            except BaseException:
                self._release(tables, fresh, failed=True)
                raise
        sync = self.device.type == "cuda"

        def barrier():
            if sync:
                if stream_sync:
                    torch.cuda.current_stream(self.device).synchronize()
                else:
                    torch.cuda.synchronize(self.device)
        try:
            barrier()
            t0 = time.perf_counter()
            with span("llm.prefill"):
                first = self._prefill(prompts, tables, temperature, seed, start)
            barrier()
            t1 = time.perf_counter()
            self._ar_trace(f"after prefill of {B} x {sum(lens)} tokens")

            part_blocks = self._part_blocks(B, max_blocks)
            st = self._state(B, max_blocks, max_new_tokens, part_blocks, stop_ids, stop_strings, slot)
            st.block_tables.zero_()
            bt = torch.zeros(B, max_blocks, dtype=torch.int32)
            for b, t in enumerate(tables):
                bt[b, :len(t)] = torch.tensor(t, dtype=torch.int32)
            st.block_tables.copy_(bt)
            f = torch.tensor(first, dtype=torch.int32)
            lens_t = torch.tensor(lens, dtype=torch.int32)
            st.ids.copy_(f)
            st.positions.copy_(lens_t)
            st.ctx_lens.copy_(lens_t + 1)
            pos = lens_t.long()
            st.slots.copy_(bt[torch.arange(B), pos // KV_BLOCK] * KV_BLOCK + pos % KV_BLOCK)
            st.tokens.zero_()
            st.tokens[:, 0].copy_(f)
            st.step.fill_(1)
            # the prefix blocks every sequence maps to the same physical blocks: the decode attention
            # reads them through L2 / MALL (once for the batch) instead of nontemporal per sequence
            st.shared.fill_(min(start) // KV_BLOCK if start and self.shared_cached else 0)
            done0 = torch.isin(f, st.stop_ids.cpu()).to(torch.int32) if stop_ids else torch.zeros(B, dtype=torch.int32)
            if stop_strings is not None:
                # the prefill's token is the first of every sequence: fed on the host
                states, keep = [], []
                for b in range(B):
                    s0, hit = stop_strings.feed(stop_strings.initial(), int(first[b]))
                    states.append(s0)
                    keep.append(1 if hit else st.stop_state.cap)
                    if hit:
                        done0[b] = 1
                st.stop_state.set_slots(range(B), states, keep)
            st.done.copy_(done0)
            ready = None
            if sync:
                ready = torch.cuda.Event()
                ready.record(torch.cuda.current_stream(self.device))
        except BaseException:
            with self._alloc_lock:
                self._release(tables, fresh, failed=True)
            raise
        return _Job(st, tables, fresh, lens, start, B, max_new_tokens, tuple(stop_ids), stop_strings, part_blocks,
                    temperature, seed, t1 - t0, ready, order)

    @torch.inference_mode()
    def finish(self, job: _Job, switch=None) -> GenerationResult:
        """Second half of :meth:`generate`: the decode of a started batch, on the current stream.
        ``switch``: called between decode steps; a stream it returns takes the remaining steps
        (ordered behind the steps already issued) -- a decode that started on a partition of the
        CUs beside another batch's prefill widens to the whole GPU once that prefill is done."""
        st, B, max_new_tokens = job.st, job.B, job.max_new
        stop_ids, stop_strings, part_blocks = job.stop_ids, job.stop_strings, job.part_blocks
        temperature, seed = job.temperature, job.seed
        sync = self.device.type == "cuda"
        ok = False
        try:
            if job.ready is not None:
                torch.cuda.current_stream(self.device).wait_event(job.ready)
            t1 = time.perf_counter()
            steps = 0
            rng = span("llm.decode")
            rng.__enter__()
            use_graph = self._graph_for(B, temperature)
            self.last_used_graph = use_graph
            if use_graph and (st.graph is None or st.graph[1:] != (part_blocks, temperature, seed)):
                self._capture(st, part_blocks, temperature, seed)
                self._ar_trace("after capture")
            cur = torch.cuda.current_stream(self.device) if sync else None
            for i in range(1, max_new_tokens):
                if switch is not None and cur is not None:
                    nxt = switch()
                    if nxt is not None and nxt != cur:
                        nxt.wait_stream(cur)
                        cur, switch = nxt, None
                if cur is not None:
                    with torch.cuda.stream(cur):
                        if use_graph:
                            st.graph[0].replay()
                        else:
                            self._decode_step(st, part_blocks, temperature, seed)
                elif use_graph:
                    st.graph[0].replay()
                else:
                    self._decode_step(st, part_blocks, temperature, seed)
                steps += 1
                self.progress += 1
                if (stop_ids or stop_strings is not None) and (i % self.stop_check_interval == 0) \
                        and bool(st.done.all()):
                    break
            if cur is not None:
                torch.cuda.current_stream(self.device).wait_stream(cur)
            tokens = st.tokens.cpu()
            keep = st.stop_state.keep.cpu().tolist() if stop_strings is not None else [steps + 1] * B
            if sync:
                torch.cuda.current_stream(self.device).synchronize()
            self._ar_trace(f"after {steps} decode steps")
            rng.__exit__(None, None, None)
            t2 = time.perf_counter()
            ok = True
        finally:
            with self._alloc_lock:
                self._release(job.tables, job.fresh, failed=not ok)
        out = []
        stop = set(stop_ids)
        for b in range(B):
            row = tokens[b, :min(steps + 1, keep[b])].tolist()
            for j, t in enumerate(row):
                if t in stop:
                    row = row[:j]
                    break
            out.append(row)
        lens = job.lens
        if job.order is not None:            # back to the caller's prompt order
            inv = [0] * B
            for slot, i in enumerate(job.order):
                inv[i] = slot
            out, lens = [out[inv[i]] for i in range(B)], [lens[inv[i]] for i in range(B)]
        return GenerationResult(out, lens, prefill_s=job.prefill_s, decode_s=t2 - t1, ttft_s=job.prefill_s,
                                decode_steps=steps, cached_prompt_tokens=sum(job.start))

    def _release(self, tables, fresh, failed: bool = False):
        if self.prefix_cache is None:
            for t in tables:
                self.kv.pool.free(t)
            return
        if failed:  # this call's own blocks may have been published before their prefill ran
            for t in fresh:
                self.prefix_cache.invalidate(t)
        for t in tables:
            self.prefix_cache.release(t)
