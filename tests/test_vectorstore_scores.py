"""Thread-restricted relevance (VectorStore.centroid_scores / HipFlatIndex.span_centroid_scores):
the orchestrator scores every chunk of a thread by cosine to the thread's centroid on one scale."""
import numpy as np
import torch

from copilot_for_consensus_amd.vectorstore import HipFlatIndex, InMemoryVectorStore


def _ref(X):
    Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
    c = Xn.mean(0)
    return Xn @ (c / np.linalg.norm(c))


def test_centroid_scores_generic_and_flat_agree():
    rng = np.random.default_rng(0)
    X = rng.standard_normal((12, 32)).astype(np.float32)
    ids = [f"c{i}" for i in range(12)]
    mem = InMemoryVectorStore(32)
    mem.add_embeddings(ids, X)
    flat = HipFlatIndex(32, device="cpu")
    flat.add_embeddings(ids + ["other"], np.vstack([X, rng.standard_normal((1, 32))]))
    want = _ref(X[:5])
    for store in (mem, flat):
        got = store.centroid_scores(ids[:5] + ["missing"])
        assert list(got) == ids[:5]
        np.testing.assert_allclose([got[i] for i in ids[:5]], want, atol=2e-2)   # bf16 rows in the flat index


def test_span_centroid_scores_segments():
    rng = np.random.default_rng(1)
    X = torch.tensor(rng.standard_normal((10, 16)).astype(np.float32))
    spans = [(2, 5), (5, 6), (6, 10)]
    got = HipFlatIndex.span_centroid_scores(X, spans)
    want = np.concatenate([_ref(X[a:b].numpy()) for a, b in spans])
    np.testing.assert_allclose(got.numpy(), want, atol=1e-5)


def test_orchestrator_candidates_one_scale():
    from copilot_for_consensus_amd.services.processing import OrchestratorService
    from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore

    store = InMemoryDocumentStore()
    for i in range(4):
        store.insert_document("chunks", {"_id": f"k{i}", "thread_id": "t", "embedding_generated": True, "text": "x"})
    mem = InMemoryVectorStore(8)
    mem.add_embeddings(["k0", "k1", "k2"], np.eye(8, dtype=np.float32)[:3] + 0.1)

    class Svc(OrchestratorService):
        def __init__(self):   # only what candidates() needs
            from copilot_for_consensus_amd.observability import SilentLogger
            self.store, self.vectors, self.log = store, mem, SilentLogger()

    c = {x["_id"]: x for x in Svc().candidates("t")}
    assert c["k3"]["similarity_score"] == 0.0 and c["k3"]["source_type"] == "thread_chunks"
    assert all(0.0 < c[k]["similarity_score"] <= 1.0 and c[k]["source_type"] == "vector_store" for k in ("k0", "k1", "k2"))
    Svc.__init__ = lambda self: setattr(self, "store", store) or setattr(self, "vectors", None)
    assert {x["similarity_score"] for x in Svc().candidates("t")} == {0.5}
