"""Continuous batching over the paged KV cache ("continuous batching of
threads"; the reference's llama.cpp / Ollama servers interleave concurrent requests the same way,
llamacpp_summarizer.py:108 -> llama-server slots, docker-compose.infra.yml:296-298).

:class:`LLMEngine.generate` runs a batch to completion; a thread that finishes early leaves its row
idle until the slowest one is done, and a thread that arrives mid-batch waits for the whole batch.
Here the decode batch is a fixed set of ``max_slots`` slots:

* one decode step over all slots is captured ONCE in a hipGraph (fixed shapes: slots x the
  block-table width) and replayed ``steps_per_sync`` times between host visits;
* every slot carries its own generated-token count and limit on the device
  (``decode_advance_cb_kernel``); a finished or empty slot is frozen -- it keeps pointing at its
  own last KV slot, or at a scratch block when empty -- so the captured step runs over it harmlessly;
* between bursts the host harvests finished slots (one device->host copy of their rows), returns
  their KV blocks, and admits queued requests into the free slots: their prompts go through the
  engine's chunked packed prefill (prefix-cache aware) and their first token, position, block table
  and limit are written into the slot rows.

Greedy outputs equal :meth:`LLMEngine.generate` on each request alone (tests/test_continuous.py).

Tensor parallel: every rank of a TP group holds a ContinuousEngine over its weight shard, and all
of them must make the same device calls in the same order (prefills, decode bursts: their
all-reduces pair up).  The leader alone decides admissions (they depend on its clock and its
queue) and hands each step's decision to the followers through ``sync`` -- a ("cstep", admitted
requests, slots to cancel, burst length) message; a follower replays it with :meth:`follow`.  The
rest is deterministic on every rank: the block allocator and the prefix cache see the same calls,
greedy tokens are all-reduced, so slots finish and free together.
"""
from __future__ import annotations

import collections
import dataclasses
import math
import time

import numpy as np
import torch

from ..ops import kernels as K
from ..ops.reference import KV_BLOCK
from .kv_cache import blocks_needed


@dataclasses.dataclass
class Request:
    rid: int
    prompt: list[int]
    max_new: int
    submitted_s: float
    first_token_s: float | None = None
    finished_s: float | None = None
    tokens: list[int] | None = None
    slot: int | None = None              # decode slot while running
    cancelled: bool = False

    @property
    def latency_s(self) -> float | None:
        return None if self.finished_s is None else self.finished_s - self.submitted_s


class ContinuousEngine:
    def __init__(self, engine, max_slots: int = 128, max_new_cap: int = 512, max_prompt: int = 4096,
                 steps_per_sync: int = 16, stop_ids: tuple[int, ...] = (), temperature: float = 0.0, seed: int = 0,
                 max_admit_tokens: int | None = None, min_admit: int = 1, max_wait_s: float = 0.5,
                 stop_strings=None, bulk_admit_frac: float = 0.5, sync=None):
        self.engine = engine
        # TP leader: called with each step's decision before any device work (see the module doc)
        self.sync = sync
        self.model = engine.model
        self.kv = engine.kv
        self.device = self.kv.device
        self.B = int(max_slots)
        self.cap = int(max_new_cap)
        self.max_prompt = int(max_prompt)
        self.steps_per_sync = max(1, int(steps_per_sync))
        self.stop_ids = tuple(int(s) for s in stop_ids)
        self.sampling = K.SamplingParams.of(temperature)
        self.seed = int(seed)
        self.max_admit_tokens = max_admit_tokens or engine.max_prefill_tokens * 4
        # admission batching: prefill waits for `min_admit` queued threads (or the oldest waiting
        # `max_wait_s`, or an idle engine) -- fewer, larger prefills interrupt the decode less
        self.min_admit, self.max_wait_s = max(1, int(min_admit)), float(max_wait_s)
        # bulk admission: with at least this fraction of the slots free, the token budget is lifted
        # and every free slot is filled in one (chunked) prefill.  Pausing a mostly empty decode
        # batch costs little, while admitting a backlog ~24 prompts at a time with a 16-step burst
        # between groups staggers the slots' finish times for good: every later refill is then a
        # small group and the decode batch never runs full (the static batch's throughput).
        self.bulk_free = max(1, math.ceil(float(bulk_admit_frac) * self.B)) if bulk_admit_frac > 0 else self.B + 1
        self.max_blocks = 8 * math.ceil(blocks_needed(self.max_prompt + self.cap) / 8)
        # empty slots read and write this block only
        self.scratch = self.kv.pool.alloc(1)[0]
        B, dev = self.B, self.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.ids = torch.zeros(B, **i32)
        self.positions = torch.zeros(B, **i32)
        self.ctx_lens = torch.ones(B, **i32)
        self.slots = torch.full((B,), self.scratch * KV_BLOCK, **i32)
        self.block_tables = torch.full((B, self.max_blocks), self.scratch, **i32)
        self.tokens = torch.zeros(B, self.cap, **i32)
        self.gen = torch.zeros(B, **i32)
        self.limit = torch.ones(B, **i32)
        self.done = torch.ones(B, **i32)
        self.next_ids = torch.zeros(B, **i32)
        self.step_t = torch.zeros(1, **i32)     # sampler RNG salt
        # leading KV blocks every occupied slot shares (prefix cache): read through the caches
        self.shared = torch.zeros(1, **i32)
        self._slot_shared = [0] * B
        self.stop_t = torch.tensor(self.stop_ids, **i32)
        # stop strings matched on the device (runtime/stops.py): a slot finishes at the token that
        # completes one, so the slot is freed and refilled instead of decoding to its limit
        self.stop_strings = stop_strings
        self.stop_state = stop_strings.new_state(B, dev) if stop_strings is not None else None
        # decode width: a burst runs the captured step over the first W slots only (admission takes
        # the lowest free slot), W the smallest bucket holding every occupied slot -- one request
        # alone decodes at B = 1 on the GEMV path, not as 1 live row of a 128-row batched GEMM
        # (light load: 6.5 -> ~3.3 ms per token).  One graph, split-KV partitioning and attention
        # workspace per width.
        self.widths = sorted({w for w in (1, 2, 4, 8, 16, 32, 64) if w < B} | {B})
        self._pb = {w: engine._part_blocks(w, self.max_blocks) for w in self.widths}
        ws = max(w * self.model.w.heads * -pb * (self.model.cfg.head_dim + 2) if -pb > 1 else 1
                 for w, pb in self._pb.items())
        self.workspace = torch.empty(max(1, ws), dtype=torch.float32, device=dev)
        self.part_blocks = self._pb[B]
        self.use_graph = engine._graph_for(B, self.sampling)
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.queue: collections.deque[Request] = collections.deque()
        self.slot_req: list[Request | None] = [None] * B
        self.slot_tables: list[tuple[list[int], list[int]] | None] = [None] * B
        self.free = list(range(B - 1, -1, -1))
        self._cancelled: list[Request] = []
        self._cancel_slots: list[int] = []     # running requests to stop at the next step
        self._rid = 0
        self.stats = {"steps": 0, "admitted": 0, "finished": 0, "prefill_s": 0.0, "decode_s": 0.0}
        self.admit_log: list[tuple] = []     # (admit time, requests, first arrival, last arrival), epoch s

    # ------------------------------------------------------------------ API
    def submit(self, prompt: list[int], max_new: int) -> Request:
        if not prompt:
            raise ValueError("empty prompt")
        if len(prompt) > self.max_prompt or max_new > self.cap or max_new < 1:
            raise ValueError(f"prompt {len(prompt)} > {self.max_prompt} or max_new {max_new} outside [1, {self.cap}]")
        r = Request(self._rid, list(prompt), int(max_new), time.perf_counter())
        self._rid += 1
        self.queue.append(r)
        return r

    def pending(self) -> int:
        return len(self.queue) + sum(r is not None for r in self.slot_req) + len(self._cancelled)

    def cancel(self, r: Request) -> None:
        """Stop a request early (client gone, stop string seen): a queued one is dropped, a running
        one has its slot marked done on the device at the next step, so that step's harvest returns
        its tokens so far."""
        if r.finished_s is not None or r.cancelled:
            return
        r.cancelled = True
        if r in self.queue:
            self.queue.remove(r)
            r.tokens, r.finished_s = [], time.perf_counter()
            self._cancelled.append(r)
        elif r.slot is not None and self.slot_req[r.slot] is r:
            self._cancel_slots.append(r.slot)

    def partial(self, reqs: list[Request]) -> dict[int, list[int]]:
        """Tokens generated so far by running requests (one device->host copy): rid -> tokens."""
        live = [r for r in reqs if r.slot is not None and self.slot_req[r.slot] is r]
        if not live:
            return {}
        idx = torch.tensor([r.slot for r in live], dtype=torch.long, device=self.device)
        gen = self.gen.index_select(0, idx).cpu().tolist()
        toks = self.tokens.index_select(0, idx).cpu()
        stop = set(self.stop_ids)
        out = {}
        for i, r in enumerate(live):
            row = toks[i, :min(gen[i], self.cap)].tolist()
            for j, t in enumerate(row):
                if t in stop:
                    row = row[:j]
                    break
            out[r.rid] = row
        return out

    @torch.inference_mode()
    def step(self) -> list[Request]:
        """Admit what fits, run one burst of decode steps, harvest; returns requests finished now."""
        take = self._select()
        cancels, self._cancel_slots = self._cancel_slots, []
        if self.sync is not None:
            self.sync(("cstep", [(r.rid, r.prompt, r.max_new) for r in take], cancels, self.steps_per_sync))
        early, self._cancelled = self._cancelled, []
        return early + self._run_step(take, cancels, self.steps_per_sync)

    @torch.inference_mode()
    def follow(self, msg) -> int:
        """TP follower: replay one leader step (the ``sync`` message) on this rank's shard.  Returns
        how many requests finished (the leader reports them; followers only free their slots)."""
        _, admitted, cancels, n = msg
        now = time.perf_counter()
        take = [Request(int(rid), list(p), int(mx), now) for rid, p, mx in admitted]
        fin = self._run_step(take, list(cancels), int(n))
        self.queue.clear()       # held back for lack of KV blocks: the leader sends them again
        return len(fin)

    def _run_step(self, take: list[Request], cancels: list[int], n: int) -> list[Request]:
        for s in cancels:
            if self.slot_req[s] is not None:
                self.done[s] = 1
        self._admit(take)
        if all(r is None for r in self.slot_req):
            return []
        t = time.perf_counter()
        self._burst(n)
        out = self._harvest()
        self.stats["decode_s"] += time.perf_counter() - t
        return out

    def run(self) -> list[Request]:
        done: list[Request] = []
        while self.pending():
            done.extend(self.step())
        return done

    def close(self) -> None:
        for s in range(self.B):
            if self.slot_tables[s] is not None:
                self._release_slot(s)
        self.kv.pool.free([self.scratch])

    # ------------------------------------------------------------------ internals
    def _select(self) -> list[Request]:
        """The admission decision (leader side): queued requests to prefill into free slots now."""
        if not self.queue or not self.free:
            return []
        waited = time.perf_counter() - self.queue[0].submitted_s
        # an idle engine waits too (up to max_wait_s for min_admit requests): admitting the first
        # arrival alone would stagger every later admission into small prefills
        if len(self.queue) < min(self.min_admit, len(self.free)) and waited < self.max_wait_s:
            return []
        take: list[Request] = []
        budget = self.max_admit_tokens if len(self.free) < self.bulk_free else float("inf")
        while self.queue and len(take) < len(self.free) and (not take or budget >= len(self.queue[0].prompt)):
            r = self.queue.popleft()
            take.append(r)
            budget -= len(r.prompt)
        return take

    def _admit(self, take: list[Request]) -> None:
        """Prefill ``take`` into free slots; what the KV pool cannot hold goes back to the queue front."""
        if not take:
            return
        idle = all(r is None for r in self.slot_req)
        pc = self.engine.prefix_cache
        tables, fresh, start = [], [], []
        try:
            for i, r in enumerate(take):
                n = blocks_needed(len(r.prompt) + r.max_new)
                shared = pc.acquire(r.prompt) if pc is not None else []
                try:
                    new = pc.alloc(n - len(shared)) if pc is not None else self.kv.pool.alloc(n)
                except MemoryError:
                    # KV cache full: admit what fits, the rest waits in the queue for running slots to
                    # finish and return their blocks (only a request that can never fit is an error)
                    self.engine._release([shared], [[]])
                    if i == 0 and idle:
                        raise
                    self.queue.extendleft(reversed(take[i:]))
                    take = take[:i]
                    break
                tables.append(shared + new)
                fresh.append(new)
                start.append(len(shared) * KV_BLOCK)
                if pc is not None:
                    pc.insert(r.prompt, tables[-1])
        except BaseException:
            self.engine._release(tables, fresh, failed=True)
            self.queue.extendleft(reversed(take))
            raise
        if not take:
            return
        if self.engine.lpt and len(take) > 1:
            # longest prompt into the lowest free slot: the decode attention grid walks slots in
            # order, so long contexts start first (list scheduling; engine.py's CFC_DECODE_LPT).
            # A stable sort on the admitted list, so TP followers replaying it place the same slots.
            order = sorted(range(len(take)), key=lambda i: -len(take[i].prompt))
            take, tables, fresh, start = ([v[i] for i in order] for v in (take, tables, fresh, start))
        t = time.perf_counter()
        try:
            first = self.engine._prefill([r.prompt for r in take], tables, self.sampling, self.seed, start)
        except BaseException:
            # nothing was installed in a slot yet: return the blocks, put the requests back in front
            self.engine._release(tables, fresh, failed=True)
            self.queue.extendleft(reversed(take))
            raise
        now = time.perf_counter()
        self.stats["prefill_s"] += now - t
        slots = [self.free.pop() for _ in take]
        bt = np.full((len(take), self.max_blocks), self.scratch, np.int32)
        rows = np.zeros((len(take), 6), np.int32)       # ids, positions, ctx, slot, limit, done
        sstates = []
        for i, (r, s, tbl, f) in enumerate(zip(take, slots, tables, first)):
            bt[i, :len(tbl)] = tbl
            n = len(r.prompt)
            hit = False
            if self.stop_strings is not None:    # the prefill's token is every request's first
                st0, hit = self.stop_strings.feed(self.stop_strings.initial(), int(f))
                sstates.append(st0)
            rows[i] = (f, n, n + 1, tbl[n // KV_BLOCK] * KV_BLOCK + n % KV_BLOCK, r.max_new,
                       int(r.max_new <= 1 or f in self.stop_ids or hit))
            r.first_token_s = now
            self.slot_req[s] = r
            r.slot = s
            self.slot_tables[s] = (tbl, fresh[i])
            self._slot_shared[s] = start[i] // KV_BLOCK
        occupied = [self._slot_shared[q] for q in range(self.B) if self.slot_req[q] is not None]
        self.shared.fill_(min(occupied) if occupied and self.engine.shared_cached else 0)
        idx = torch.tensor(slots, dtype=torch.long, device=self.device)
        rows_t = torch.from_numpy(rows).to(self.device)
        self.block_tables.index_copy_(0, idx, torch.from_numpy(bt).to(self.device))
        for j, dst in enumerate((self.ids, self.positions, self.ctx_lens, self.slots, self.limit, self.done)):
            dst.index_copy_(0, idx, rows_t[:, j].contiguous())
        self.gen.index_fill_(0, idx, 1)
        if self.stop_state is not None:
            self.stop_state.set_slots(slots, sstates)
        self.tokens.index_copy_(0, idx, torch.nn.functional.pad(rows_t[:, :1], (0, self.cap - 1)))
        self.stats["admitted"] += len(take)
        # admission timeline (wall clock): when, how many, first / last arrival of the admitted requests
        sub = [r.submitted_s for r in take]
        off = time.time() - time.perf_counter()
        self.admit_log.append((round(t + off, 3), len(take), round(min(sub) + off, 3), round(max(sub) + off, 3)))
        self.stats["admissions"] = self.stats.get("admissions", 0) + 1

    def _width(self) -> int:
        hi = max((s for s in range(self.B) if self.slot_req[s] is not None), default=0) + 1
        return next(w for w in self.widths if w >= hi)

    def _decode_step(self, W: int) -> None:
        ss = self.stop_state.view(W) if self.stop_state is not None else None
        hidden = self.model.forward_decode(self.ids[:W], self.positions[:W], self.slots[:W], self.ctx_lens[:W],
                                           self.block_tables[:W], self.kv, attn_workspace=self.workspace,
                                           part_blocks=self._pb[W], shared_blocks=self.shared)
        self.engine._next_tokens(hidden, self.next_ids[:W], self.sampling, self.seed, self.step_t)
        K.decode_advance_cb(self.next_ids[:W], self.tokens[:W], self.gen[:W], self.limit[:W], self.ids[:W],
                            self.positions[:W], self.ctx_lens[:W], self.slots[:W], self.block_tables[:W],
                            self.done[:W], self.stop_t, ss)
        self.step_t.add_(1)

    def _state(self):
        extra = [self.stop_state.win, self.stop_state.wlen, self.stop_state.keep] if self.stop_state else []
        return [self.ids, self.positions, self.ctx_lens, self.slots, self.tokens, self.gen, self.done,
                self.next_ids, self.step_t] + extra

    def _burst(self, n: int) -> None:
        W = self._width()          # no admission inside a burst: the occupied slots only shrink
        if self.use_graph and W not in self.graphs:
            saved = [t.clone() for t in self._state()]
            s = self.engine.capture_stream()
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._decode_step(W)       # warm-up (workspaces, library handles) outside capture
            torch.cuda.current_stream(self.device).wait_stream(s)
            for t, v in zip(self._state(), saved):
                t.copy_(v)
            g = torch.cuda.CUDAGraph()
            # thread_local: other service threads keep launching / syncing their own streams while
            # this step is captured (global mode would invalidate the capture)
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                self._decode_step(W)
            for t, v in zip(self._state(), saved):
                t.copy_(v)
            self.graphs[W] = g
        g = self.graphs.get(W)
        for _ in range(n):
            if g is not None:
                g.replay()
            else:
                self._decode_step(W)
        self.stats["steps"] += n
        self.stats["width_steps"] = self.stats.get("width_steps", 0) + n * W

    def _harvest(self) -> list[Request]:
        done = self.done.cpu().numpy()
        fin = [s for s in range(self.B) if self.slot_req[s] is not None and done[s]]
        if not fin:
            return []
        idx = torch.tensor(fin, dtype=torch.long, device=self.device)
        gen = self.gen.index_select(0, idx).cpu().tolist()
        toks = self.tokens.index_select(0, idx).cpu()
        now = time.perf_counter()
        stop = set(self.stop_ids)
        out = []
        for i, s in enumerate(fin):
            row = toks[i, :min(gen[i], self.cap)].tolist()
            for j, t in enumerate(row):
                if t in stop:
                    row = row[:j]
                    break
            r = self.slot_req[s]
            r.tokens, r.finished_s, r.slot = row, now, None
            out.append(r)
            self._release_slot(s)
        # freeze the freed rows on the scratch block before their KV blocks can be reused
        self.block_tables.index_fill_(0, idx, self.scratch)
        self.slots.index_fill_(0, idx, self.scratch * KV_BLOCK)
        self.positions.index_fill_(0, idx, 0)
        self.ctx_lens.index_fill_(0, idx, 1)
        self.stats["finished"] += len(out)
        return out

    def _release_slot(self, s: int) -> None:
        tbl, fresh = self.slot_tables[s]
        self.engine._release([tbl], [fresh])
        self.slot_tables[s] = None
        self.slot_req[s] = None
        self.free.append(s)
        self.free.sort(reverse=True)     # pop() takes the lowest free slot: the decode width stays small
