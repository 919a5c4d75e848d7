"""``bench.py --pipeline node``: the headline workload through the REAL services.

The default bench pipeline (pipeline/bench_pipeline.py) calls the stage code directly with a
static 128-thread LLM batch.  This one runs the deployment itself: a :class:`~..services.node.Node`
(ingestion, parsing, chunking, embedding, orchestrator, summarization, reporting on the in-process
bus, document store in memory, HIP encoder + HBM vector index + HIP decoder on the GPU) with the
summarization service on its continuous engine.  Each step's synthetic mailing-list archive enters
through the ingestion service (a local source: fetch -> archive store -> ``ArchiveIngested``) and
the step is done when every one of its threads has a report in the store.  Archives are submitted
paced: at most two steps in flight (``CFC_NODE_MAX_INFLIGHT``; 0 queues every step at once, a
backfill's backlog), so stages overlap the way the event-driven services overlap them and the
reported latency is a step's own.

Under torchrun (``world > 1``) the bench runs the topology ``services.main node`` deploys
(services/main.py ``_distributed``): global rank 0 runs the services with the DP facades over the
ranks (parallel/dp_node.py), EVERY rank runs a :class:`~..parallel.dp_node.DPNodeWorker` with its
own HIP encoder, HBM index shard (1M resident vectors each) and continuous LLM engine; a step is
one archive of ``threads_per_step x world`` threads (weak scaling), its threads embedded, indexed
and summarized on their owner GPUs through the node's control plane.

Same model, encoder, threads per step, generated tokens (``LLM_IGNORE_EOS`` as the bench
pipeline's ``ignore_eos``: random-init weights would otherwise stop at arbitrary points) and
selection settings (top-5 chunks, 2048-token context) as the bench pipeline.
"""
from __future__ import annotations

import dataclasses
import os
import statistics
import sys
import tempfile
import time
from datetime import datetime
from pathlib import Path

import torch


@dataclasses.dataclass
class NodeStepResult:
    threads: int
    generated_tokens: int
    prompt_tokens: int
    latencies_s: list
    wall_s: float

    def summary(self) -> str:
        p50 = statistics.median(self.latencies_s) if self.latencies_s else float("nan")
        return (f"threads={self.threads} prompt_tok={self.prompt_tokens} gen_tok={self.generated_tokens} "
                f"p50={p50:.2f}s wall={self.wall_s:.2f}s")


class NodeBench:
    def __init__(self, model: str = "mistral-7b", encoder: str = "minilm-l6", device="cuda",
                 threads_per_step: int = 128, max_new_tokens: int = 512, seed: int = 0,
                 index_prefill: int = 1_000_000, continuous: bool = True, dp: dict | None = None,
                 min_admit: int | None = None, admit_wait_ms: int | None = None):
        """``dp`` (torchrun): {"store": the job's TCPStore, "rank": DP rank, "world": DP size} -- the
        services.main DP topology (rank 0 services + a DPNodeWorker on every rank)."""
        from ..services.node import Node
        from ..utils.synthetic import SyntheticArchive
        dev = str(device)
        self.dp = dp
        world = int(dp["world"]) if dp else 1
        self.rank = int(dp["rank"]) if dp else 0
        self.tmp = Path(tempfile.mkdtemp(prefix="cfc-node-bench-"))
        enc_name = {"minilm-l6": "all-MiniLM-L6-v2"}.get(encoder, encoder)
        self.env = {
            "EMBEDDING_BACKEND_TYPE": "hip", "EMBEDDING_MODEL_NAME": enc_name, "EMBEDDING_DEVICE": dev,
            "EMBEDDING_RANDOM_SEED": str(seed),
            "VECTOR_STORE_TYPE": "hip", "VECTOR_STORE_DEVICE": dev,
            "VECTOR_STORE_CAPACITY": str(index_prefill + (1 << 20)),
            "LLM_BACKEND_TYPE": "hip", "LLM_MODEL_PRESET": model, "LLM_DEVICE": dev,
            "LLM_MAX_NEW_TOKENS": str(max_new_tokens), "LLM_MAX_BATCH": str(threads_per_step),
            "LLM_TEMPERATURE": "0", "LLM_IGNORE_EOS": "true", "LLM_RANDOM_SEED": "1234",
            "LLM_KV_CACHE_TOKENS": str(max(65536, threads_per_step * (4096 + max_new_tokens))),
            "SUMMARIZATION_CONTINUOUS_BATCHING": "true" if continuous else "false",
            "SUMMARIZATION_MAX_BATCH_THREADS": str(threads_per_step),
            # admission: wait for a full batch (or 3 s) -- overridable for A/B runs.  Under DP a rank
            # receives ~threads_per_step of a step's threads (hash ownership), not exactly that many
            "SUMMARIZATION_MIN_ADMIT": str(min_admit) if min_admit is not None else os.environ.get(
                "CFC_NODE_MIN_ADMIT", str(threads_per_step if world == 1 else max(1, (9 * threads_per_step) // 10))),
            "SUMMARIZATION_ADMIT_WAIT_MS": str(admit_wait_ms) if admit_wait_ms is not None else os.environ.get(
                "CFC_NODE_ADMIT_WAIT_MS", "3000"),
            "ORCHESTRATOR_TOP_K": "5", "ORCHESTRATOR_CONTEXT_WINDOW_TOKENS": "2048",
            "INGESTION_STORAGE_PATH": str(self.tmp / "ingest"), "INGESTION_SCHEDULE_INTERVAL_SECONDS": "0",
            "ARCHIVE_STORE_TYPE": "local", "ARCHIVE_BASE_PATH": str(self.tmp / "archives"),
            "DOCUMENT_STORE_TYPE": "inmemory", "MESSAGE_BUS_TYPE": "inproc",
        }
        t0 = time.time()
        self.node, self.worker = None, None
        if dp:
            self._build_dp(dev, seed, index_prefill, threads_per_step)
        else:
            self.node = Node(env=self.env)
            if index_prefill and hasattr(self.node.vectors, "add_embeddings"):
                self._prefill_index(self.node.vectors, int(self.node.embedder.dimension), dev, seed, index_prefill)
        print(f"[bench-node] rank {self.rank}: services and models built in {time.time() - t0:.1f}s",
              file=sys.stderr, flush=True)
        self.threads_per_step = threads_per_step
        self.step_threads = threads_per_step * world     # one archive per step for the whole node
        self.generator = SyntheticArchive(seed=seed)
        self.sources: dict[int, Path] = {}
        self.submitted: dict[int, float] = {}
        if self.node is not None:
            self.node.start(threaded=True)
            print(f"[bench-node] node running ({time.time() - t0:.1f}s)", file=sys.stderr, flush=True)
            self.ingestion = self.node.services["ingestion"]
            self.store = self.node.store

    @staticmethod
    def _prefill_index(index, dim, dev, seed, n_rows):
        """The same 1M-vector resident index the bench pipeline searches next to (rows of other lists)."""
        g = torch.Generator(device=dev).manual_seed(seed + 99)
        for s in range(0, n_rows, 1 << 18):
            n = min(1 << 18, n_rows - s)
            v = torch.randn(n, dim, device=dev, generator=g)
            index.add_embeddings([f"prefill-{s + i}" for i in range(n)], v, [{} for _ in range(n)])

    def _build_dp(self, dev, seed, index_prefill, threads_per_step):
        """services.main's DP roles on this rank (see the module doc)."""
        from ..config.loader import get_config
        from ..embedding import create_embedding_provider
        from ..parallel.dp_node import DPNodeWorker, build_rank0
        from ..services.node import Node
        from ..summarization import create_llm_backend
        from ..vectorstore import create_vector_store
        env, dp = self.env, self.dp
        ecfg, scfg = get_config("embedding", env=env), get_config("summarization", env=env)
        embedder = create_embedding_provider(ecfg.embedding_backend)
        index = create_vector_store(ecfg.vector_store, dimension=int(embedder.dimension))
        if index_prefill:
            self._prefill_index(index, int(embedder.dimension), dev, seed + 7919 * self.rank, index_prefill)
        local = create_llm_backend(scfg.llm_backend)
        self.worker = DPNodeWorker(dp["store"], self.rank, int(dp["world"]), embedder, index, local,
                                   continuous=dict(min_admit=int(scfg.min_admit),
                                                   max_wait_s=scfg.admit_wait_ms / 1000.0))
        if self.rank == 0:
            vs, summ = build_rank0(dp["store"], int(dp["world"]), self.worker,
                                   heartbeat_timeout=float(os.environ.get("CFC_DP_HEARTBEAT_TIMEOUT", "60")))
            self.dp_facades = (vs, summ)
            self.node = Node(env=env, summarizer=summ, vector_store=vs, embedding_provider=embedder)
            self.worker.start(serve=False)
        else:
            self.worker.start(serve=True)

    def prepare_sources(self, steps) -> None:
        """The steps' archives as local mailing-list sources (outside the timed region)."""
        for s in steps:
            d = self.tmp / f"src{s}"
            d.mkdir(parents=True, exist_ok=True)
            (d / f"step{s}.mbox").write_bytes(self.generator.mbox(self.step_threads))
            self.sources[s] = d

    def _submit(self, step: int) -> tuple[list[str], float]:
        t0 = time.time()
        self.submitted[step] = t0
        ids = self.ingestion.ingest_archive({"name": f"bench-{step}", "source_type": "local",
                                            "url": str(self.sources[step]), "enabled": True})
        return ids, t0

    def _thread_ids(self, archive_ids: list[str]) -> list[str]:
        return [t["_id"] for t in self.store.query_documents("threads", {"archive_id": {"$in": archive_ids}},
                                                             limit=1 << 20)]

    def run_steps(self, steps, on_step=None, timeout_s: float = 3600.0, max_inflight: int | None = None
                  ) -> list[NodeStepResult]:
        """Submit the steps' archives through the ingestion service and wait until each step's
        threads all have reports.  ``max_inflight`` (default $CFC_NODE_MAX_INFLIGHT, 0 = all at
        once): at most that many steps submitted and unfinished -- a paced source, so a step's
        latency is its own (queue + upstream + summarization), not the position in a whole backlog;
        2 keeps the next batch's upstream work overlapped with the running decode."""
        if max_inflight is None:
            max_inflight = int(os.environ.get("CFC_NODE_MAX_INFLIGHT", "2"))
        todo = list(steps)
        subs = {}
        ce = self._engine()
        base = ce.stats["admitted"] if ce is not None else 0

        def upstream_done() -> bool:
            # with the continuous engine: every thread submitted so far has been admitted, i.e. at
            # most one step is upstream (ingest..orchestrate) at a time.  Submitting two at once made
            # their threads interleave into both engine batches, so the pair finished together and
            # the next pair's upstream ran with the GPU idle (profiles/r04_bench_node_*timeline*)
            if ce is None or ce.stats["admitted"] - base >= self.step_threads * len(subs):
                return True
            # a step whose threads cannot all reach the engine must not stall the source for good
            return bool(subs) and time.time() - max(t0 for _, t0 in subs.values()) > 30.0

        def just_in_time() -> bool:
            # the next step enters the source so its upstream (ingest .. orchestrate, measured on the
            # previous step) completes as the running batch drains -- the bench pipeline's policy:
            # its threads do not wait in the engine queue for a whole batch (p50), and the engine
            # is never idle for lack of them (throughput)
            log = ce.admit_log if ce is not None else []
            if len(log) < 2 or not self.submitted:
                return True
            batch_s = log[-1][0] - log[-2][0]
            last_sub = max(self.submitted.values())
            upstream_s = max(0.5, log[-1][3] - last_sub) if log[-1][3] >= last_sub else 1.0
            return time.time() >= log[-1][0] + batch_s - (2.0 * upstream_s + 0.5)

        def refill():
            while todo and (max_inflight <= 0 or (len(subs) - len(out) < max_inflight and upstream_done()
                                                  and just_in_time())):
                s = todo.pop(0)
                subs[s] = self._submit(s)
        out: list[NodeStepResult] = []
        refill()
        deadline = time.time() + timeout_s
        pending = list(steps)
        last_note = time.time()
        tids_of: dict = {}
        # the poll runs on the main thread beside the services' threads and the engine thread: it
        # counts (no document copies) and sleeps 0.1 s, so it never competes for the GIL noticeably
        while pending:
            refill()                              # the next step once the last one was admitted
            if time.time() - last_note > 15:      # a visible heartbeat of the pipeline's progress
                last_note = time.time()
                c = {k: self.store.count_documents(k, {}) for k in ("messages", "threads", "chunks", "summaries")}
                c["embedded"] = self.store.count_documents("chunks", {"embedding_generated": True})
                print(f"[bench-node] waiting on step {pending[0]}: {c}", file=sys.stderr, flush=True)
            if time.time() > deadline:
                raise TimeoutError(f"node bench: steps {pending} unfinished after {timeout_s}s")
            s = pending[0]
            if s not in subs:                     # paced: not submitted yet (the running step drains first)
                time.sleep(0.05)
                continue
            aids, t0 = subs[s]
            tids = tids_of.get(s)
            if tids is None:
                if self.store.count_documents("threads", {"archive_id": {"$in": aids}}) < self.step_threads:
                    time.sleep(0.1)
                    continue
                tids = tids_of[s] = self._thread_ids(aids)
            if self.store.count_documents("summaries", {"thread_id": {"$in": tids}}) < len(tids):
                time.sleep(0.1)
                continue
            reports = self.store.query_documents("summaries", {"thread_id": {"$in": tids}}, limit=1 << 20)
            if len({r["thread_id"] for r in reports}) < len(tids):
                time.sleep(0.1)
                continue
            lat = [max(0.0, datetime.fromisoformat(r["generated_at"].replace("Z", "+00:00")).timestamp() - t0)
                   for r in reports]
            meta = [r.get("metadata") or {} for r in reports]
            res = NodeStepResult(len(tids), sum(int(m.get("tokens_completion", 0)) for m in meta),
                                 sum(int(m.get("tokens_prompt", 0)) for m in meta), lat, time.time() - t0)
            out.append(res)
            if on_step is not None:
                on_step(s, res)
            pending.pop(0)
            refill()
        return out

    def light_load_probe(self, rate_per_s: float, n_threads: int, seed: int = 0, timeout_s: float = 600.0) -> dict:
        """The latency half through the services at a light load: ``n_threads`` one-thread archives
        enter the ingestion service as a Poisson process of ``rate_per_s`` (each a local source, as a
        mailing list delivering one new thread); a thread's latency is archive submit -> its report
        stored by the reporting service (ingest, parse, chunk, embed, index, select, prefill +
        decode, report: every hop on the in-process bus).  The reference's figure of merit at one
        thread at a time (summarization/app/service.py:329-345 summarization_latency_seconds covers
        the LLM call only; this covers the whole path)."""
        import numpy as np
        from ..utils.synthetic import SyntheticArchive
        gen = SyntheticArchive(seed=seed + 31337)
        srcs = []
        for i in range(n_threads):
            d = self.tmp / f"light{seed}-{i}"
            d.mkdir(parents=True, exist_ok=True)
            (d / "one.mbox").write_bytes(gen.mbox(1))
            srcs.append(d)
        rng = np.random.default_rng(seed)
        arrive = np.cumsum(rng.exponential(1.0 / float(rate_per_s), n_threads))
        t0 = time.time()
        sub: dict[int, tuple[list[str], float]] = {}
        lat: dict[int, float] = {}
        nxt = 0
        deadline = t0 + float(arrive[-1]) + timeout_s
        while len(lat) < n_threads:
            now = time.time()
            if now > deadline:
                raise TimeoutError(f"light-load probe: {n_threads - len(lat)} threads unfinished")
            while nxt < n_threads and t0 + arrive[nxt] <= now:
                ts = time.time()
                ids = self.ingestion.ingest_archive({"name": f"light-{seed}-{nxt}", "source_type": "local",
                                                    "url": str(srcs[nxt]), "enabled": True})
                sub[nxt] = (ids, ts)
                nxt += 1
            for i, (aids, ts) in list(sub.items()):
                if i in lat:
                    continue
                tids = self._thread_ids(aids)
                if not tids:
                    continue
                reps = self.store.query_documents("summaries", {"thread_id": {"$in": tids}}, limit=len(tids) + 4)
                if len({r["thread_id"] for r in reps}) < len(tids):
                    continue
                done = max(datetime.fromisoformat(r["generated_at"].replace("Z", "+00:00")).timestamp() for r in reps)
                lat[i] = max(0.0, done - ts)
            time.sleep(0.02)
        v = np.asarray([lat[i] for i in range(n_threads)])
        return {"arrival_rate_per_gpu": float(rate_per_s), "threads": int(n_threads),
                "p50_s": round(float(np.percentile(v, 50)), 3), "p95_s": round(float(np.percentile(v, 95)), 3),
                "path": "services: archive submit (ingestion) -> report stored (reporting), in-proc bus, "
                        "continuous engine admitting each thread on arrival"}

    def _engine(self):
        if self.node is None:
            return None
        llm = getattr(self.node.services.get("summarization"), "summarizer", None)
        return getattr(llm, "_ce", None)

    def engine_stats(self) -> dict:
        """The summarizer's continuous-engine counters (admissions, decode steps, prefill / decode s)."""
        # DP: every rank's engine sits in its worker (rank 0's node summarizer is the DP router)
        ce = getattr(getattr(self.worker, "summarizer", None), "_ce", None) if self.worker is not None \
            else self._engine()
        return dict(ce.stats) if ce is not None else {}

    def dp_stats(self) -> dict:
        """This rank's DP worker counters (embedded chunks, summaries, topic queries) + its engine's."""
        if self.worker is None:
            return {}
        eng = getattr(getattr(self.worker, "summarizer", None), "_ce", None)
        out = {"rank": self.rank, **dict(self.worker.stats)}
        if eng is not None:
            out.update(admitted=eng.stats.get("admitted"), finished=eng.stats.get("finished"))
        return out

    def close(self) -> None:
        print(f"[bench-node] rank {self.rank} continuous engine: {self.engine_stats()}", file=sys.stderr, flush=True)
        if self.node is not None:
            ce = self._engine()
            if ce is not None:
                subs = {s: round(t0, 3) for s, t0 in self.submitted.items()}
                print(f"[bench-node] step submit times: {subs}", file=sys.stderr, flush=True)
                print(f"[bench-node] admissions (t, n, first arrival, last arrival): {ce.admit_log}",
                      file=sys.stderr, flush=True)
            self.node.stop()
        if self.worker is not None:
            if self.rank == 0:
                from ..parallel.dp_node import shutdown_workers
                shutdown_workers(self.dp["store"])
                self.dp_facades[0].close()
            self.worker.stop()
        import shutil
        shutil.rmtree(self.tmp, ignore_errors=True)
