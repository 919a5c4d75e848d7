"""In-process, batched driver of the services' own stage methods: ingest -> parse -> chunk -> embed ->
index -> select -> prompt (-> summarize, done by the caller's LLM engine) -> summaries / reports.

There is ONE implementation of every stage: the service classes the deployed node runs
(services/ingestion.py, services/processing.py, services/reporting.py).  This driver calls their
batch entry points directly, in order, once per batch of threads, instead of letting each
service's consumer loop receive the previous stage's event from the bus:

  IngestionService.record_archive -> ParsingService.process_archive -> ChunkingService.process_messages ->
  EmbeddingService.process_chunks -> OrchestratorService.orchestrate_threads ->
  SummarizationService.prepare -> (LLM engine) -> SummarizationService.publish_summary ->
  ReportingService.process_summary

so documents, ids, events (every one schema-validated on publish) and the store layout are exactly
the node's.  What the batch form saves is the per-item transport: the encoder embeds the whole
batch's chunks in a few packed forwards, the vectors go from the encoder to the HBM index without
leaving the GPU, and the orchestrator scores all threads' candidates in one index pass
(centroid_scores_many).

Reference: the six-service event flow; orchestrator context selection
(orchestrator/app/context_selectors.py:17,95-107; context_sources.py:21,57-64) and the
summarization request path (summarization/app/service.py:289).
"""
from __future__ import annotations

import dataclasses
import random
import time

import torch

from ..archive import InMemoryArchiveStore
from ..bus import NoopPublisher, ValidatingEventPublisher
from ..storage.document_store import InMemoryDocumentStore
from ..utils.synthetic import SyntheticArchive


@dataclasses.dataclass
class PreparedBatch:
    threads: list[dict]
    prompts: list[list[int]]
    prompt_texts: list[str]
    selections: list          # the SummarizationRequested events (selected chunks + selection metadata)
    contexts: list[dict]
    stage_s: dict[str, float]
    archive_id: str


class _ShardedRows:
    """The EmbeddingService / OrchestratorService face of the DP-sharded HBM index (parallel/knn.py):
    ``add_embeddings`` is the collective ``add_thread_rows`` (every DP rank calls it once per batch
    with its own threads' rows, each thread's rows consecutive -- EmbeddingService orders them so);
    the owners' thread-restricted relevance it returns answers ``centroid_scores`` for those rows."""

    def __init__(self, sharded):
        self.sharded = sharded
        self._scores: dict[str, float] = {}

    def add_embeddings(self, ids, vectors, metadatas):
        ids = list(ids)
        s = self.sharded.add_thread_rows([m["thread_id"] for m in metadatas], ids, vectors)
        self._scores = dict(zip(ids, s.cpu().tolist()))

    def centroid_scores(self, ids):
        return {i: self._scores[i] for i in ids if i in self._scores}

    def centroid_scores_many(self, groups):
        return [self.centroid_scores(g) for g in groups]


class RagPipeline:
    def __init__(self, encoder: str = "minilm-l6", device="cuda", decoder_vocab: int = 32000, bos_id: int = 1,
                 seed: int = 0, top_k: int = 5, context_window_tokens: int = 2048, index_prefill: int = 1_000_000,
                 publisher=None, validate_events: bool = True, llm_model: str = "mistral-7b",
                 max_prompt_tokens: int | None = None, index_group=None):
        from ..archive import SourceConfig
        from ..embedding import HipEncoderProvider
        from ..runtime.tokenizer import synthetic_bpe
        from ..services.ingestion import IngestionService
        from ..services.processing import (ChunkingService, EmbeddingService, OrchestratorService, ParsingService,
                                           SummarizationService)
        from ..services.reporting import ReportingService
        from ..vectorstore import HipFlatIndex
        self.device = torch.device(device)
        self.embedder = HipEncoderProvider(model_name=encoder, device=str(self.device), seed=seed)
        self.bpe = synthetic_bpe(decoder_vocab)
        self.bos_id = bos_id
        self.docs = InMemoryDocumentStore()
        self.archives = InMemoryArchiveStore()
        self.local_index = HipFlatIndex(dimension=self.embedder.dimension, distance="cosine",
                                        capacity=index_prefill + (1 << 18), device=str(self.device))
        # DP ranks (index_group): one logical index sharded over the GPUs -- each rank's shard holds
        # its 1M prefill rows and the chunk vectors of the threads it owns
        self.sharded = None
        vectors = self.local_index
        if index_group is not None:
            from ..parallel.knn import ShardedVectorIndex
            self.sharded = ShardedVectorIndex(self.local_index, group=index_group)
            vectors = _ShardedRows(self.sharded)
        self.index = self.local_index
        if index_prefill:
            # in 16M-row pieces: a 100M-row index (BASELINE config 5) would need 154 GB of fp32 noise
            # at once next to its own 77 GB
            g = torch.Generator(device=self.device).manual_seed(seed + 99)
            for s in range(0, index_prefill, 1 << 24):
                n = min(1 << 24, index_prefill - s)
                noise = torch.randn(n, self.embedder.dimension, device=self.device, generator=g)
                self.index.add_bulk([f"prefill-{i}" for i in range(s, s + n)], noise)
                del noise
        pub = publisher or NoopPublisher()
        self.pub = ValidatingEventPublisher(pub) if validate_events else pub
        # the node's services over one store; no subscriber: this driver hands each stage its input
        self.ingestion = IngestionService(self.pub, self.docs, self.archives)
        self.parsing = ParsingService(self.pub, None, self.docs, self.archives)
        self.chunking = ChunkingService(self.pub, None, self.docs)
        self.embedding = EmbeddingService(self.pub, None, self.docs, self.embedder, vectors)
        self.orchestrator = OrchestratorService(self.pub, None, self.docs, vector_store=vectors, top_k=top_k,
                                                context_window_tokens=context_window_tokens)
        self.summarization = SummarizationService(self.pub, None, self.docs, summarizer=None, continuous=False)
        self.reporting = ReportingService(self.pub, None, self.docs)
        self.source = SourceConfig.from_mapping({"name": "bench", "source_type": "local", "url": "file:///bench"})
        self.top_k, self.budget = top_k, context_window_tokens
        self.template = self.orchestrator.template
        self.generator = SyntheticArchive(seed=seed)
        self.sources: dict[int, bytes] = {}
        self.llm_model = llm_model
        self.max_prompt_tokens = max_prompt_tokens

    # ------------------------------------------------------------------ data source
    def prepare_sources(self, n_threads: int, steps: list[int]) -> None:
        """Pre-generate the step archives (the remote mailing list; not part of the timed work)."""
        for s in steps:
            if s not in self.sources:
                self.sources[s] = self.generator.mbox(n_threads)

    # ------------------------------------------------------------------ stages
    def prepare(self, n_threads: int, step: int) -> PreparedBatch:
        st: dict[str, float] = {}
        t = time.perf_counter()
        raw = self.sources.pop(step, None) or self.generator.mbox(n_threads)
        aid = self.ingestion.record_archive(self.source, raw, f"/bench/step{step}.mbox")
        if aid is None:   # identical content already ingested (IngestionService dedupes by hash)
            raise ValueError(f"step {step}: archive already ingested")
        st["ingest"] = time.perf_counter() - t

        t = time.perf_counter()
        parsed = self.parsing.process_archive(aid)
        st["parse"] = time.perf_counter() - t

        t = time.perf_counter()
        chunk_ids = self.chunking.process_messages(parsed["message_doc_ids"])
        st["chunk"] = time.perf_counter() - t

        # embed (packed varlen encoder on the GPU) -> HBM index, each thread's rows adjacent
        t = time.perf_counter()
        self.embedding.process_chunks(chunk_ids)
        st["embed"] = time.perf_counter() - t

        # orchestrate: every thread's candidates scored in one index pass, then the service's own
        # selection / dedupe / SummarizationRequested; the prompt as the summarization service builds it
        t = time.perf_counter()
        requests = [ev for ev in self.orchestrator.orchestrate_threads(parsed["thread_ids"]) if ev is not None]
        threads, texts, ctxs = [], [], []
        for ev in requests:
            tid, ctx, prompt = self.summarization.prepare(ev)
            threads.append(self.docs.get_document("threads", tid))
            texts.append(prompt)
            ctxs.append(ctx)
        st["select"] = time.perf_counter() - t

        t = time.perf_counter()
        prompts = [self._clip(ids) for ids in self.bpe.encode_batch(texts)]
        st["tokenize"] = time.perf_counter() - t
        return PreparedBatch(threads, prompts, texts, requests, ctxs, st, aid)

    def search_probe(self, n_queries: int = 64, limit: int = 50, seed: int = 0) -> dict:
        """The reference's one live vector-query path, timed: ``GET /api/reports/search`` ->
        ReportingService.search_reports_by_topic (reporting/app/service.py:797-828): embed the topic
        on the HIP encoder, HIP kNN top-(limit x 3) over the whole resident index (the prefill rows +
        every chunk the run embedded), group by thread, enrich from the document store.  Topics
        are thread subjects of the run; ``min_score`` 0 so every hit thread is enriched (the most
        work per query).  Against the reporting P95 SLO of 0.5 s
        (infra/prometheus/alerts/slo_latency.yml:249).  With a DP-sharded index the query is the
        global exact top-k over every rank's shard (parallel/knn.py ShardedVectorIndex.query: local
        HIP scan + all-gather of the candidates + merge), a collective every DP rank runs in step
        with the same query count; enrichment finds the summaries this rank's store holds."""
        from ..services.reporting import ReportingService
        rep = ReportingService(self.pub, None, self.docs,
                               vector_store=self.sharded if self.sharded is not None else self.local_index,
                               embedding_provider=self.embedder)
        subjects = sorted({t["subject"] for t in self.docs.query_documents("threads", {}, limit=1 << 30)
                           if t.get("subject")})
        if not subjects:
            return {}
        rng = random.Random(seed)
        rep.search_reports_by_topic(subjects[0], limit=limit, min_score=0.0)     # warm-up
        lat, found = [], 0
        for _ in range(n_queries):
            topic = rng.choice(subjects)
            t = time.perf_counter()
            res = rep.search_reports_by_topic(topic, limit=limit, min_score=0.0)
            lat.append(time.perf_counter() - t)
            found += len(res)
        lat.sort()
        rows = int(self.local_index.count())
        if self.sharded is not None:
            rows = int(self.sharded.count())
        return {"queries": n_queries, "limit": limit, "top_k": 3 * limit, "index_rows": rows,
                "p50_ms": round(1e3 * lat[len(lat) // 2], 2), "p95_ms": round(1e3 * lat[int(0.95 * (len(lat) - 1))], 2),
                "max_ms": round(1e3 * lat[-1], 2), "reports_per_query": round(found / n_queries, 1),
                "path": "ReportingService.search_reports_by_topic: HIP encoder embed -> HIP kNN (flat cosine, "
                        "fused top-k) over the HBM index -> group by thread -> document-store enrichment",
                "slo_p95_ms": 500}

    def _clip(self, ids: list[int]) -> list[int]:
        """Keep the instructions (head) and the latest excerpts (tail) if a prompt exceeds the context."""
        L = self.max_prompt_tokens
        if L is None or len(ids) <= L:
            return ids
        half = L // 2
        return ids[:half] + ids[-(L - half):]

    def finish(self, batch: PreparedBatch, gen) -> list[dict]:
        """Detokenise; SummaryComplete through the summarization service, the summaries document +
        thread link + ReportPublished through the reporting service."""
        from ..summarization import Summary
        reports = []
        for th, ctx, toks, p in zip(batch.threads, batch.contexts, gen.tokens, batch.prompts):
            text = self.bpe.decode(toks).strip() or "(empty summary)"
            s = Summary(th["_id"], text, llm_backend="hip", llm_model=self.llm_model, tokens_prompt=len(p),
                        tokens_completion=len(toks), latency_ms=int(1000 * gen.total_s))
            ev = self.summarization.publish_summary(th["_id"], ctx, s)
            rid = self.reporting.process_summary(ev["data"], ev)
            reports.append(self.docs.get_document("summaries", rid))
        return reports
