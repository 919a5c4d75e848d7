"""Vector-store contract over every local driver (numpy reference, HIP flat index, HIP IVF index,
FAISS-semantics mode), run on the CPU device.  Mirrors the behaviours the reference checks in
adapters/copilot_vectorstore/tests/test_inmemory.py and test_faiss.py (initialisation, single and
batch adds, length / dimension mismatches, empty-store queries, similarity order, top_k, delete /
get of missing ids, clear, metadata copies, cosine values, L2 -> 1/(1+d) conversion, IVF, save /
load) with one deliberate difference: a repeated id is an upsert (the interface's documented
contract, interface.py:54), where the reference's in-memory and FAISS stores raise."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from copilot_for_consensus_amd.vectorstore import (HipFlatIndex, HipIVFIndex, InMemoryVectorStore, SearchResult,
                                                  create_vector_store)

DIM = 8


def _make(kind):
    if kind == "inmemory":
        return InMemoryVectorStore(dimension=DIM)
    if kind == "flat":
        return HipFlatIndex(DIM, "cosine", capacity=16, device="cpu")
    if kind == "ivf":
        return HipIVFIndex(DIM, "cosine", nlist=2, nprobe=2, capacity=16, device="cpu")
    if kind == "faiss":
        return create_vector_store("faiss", dimension=DIM, capacity=16, device="cpu")
    raise AssertionError(kind)


KINDS = ["inmemory", "flat", "ivf", "faiss"]
COSINE_KINDS = ["inmemory", "flat", "ivf"]


@pytest.fixture(params=KINDS)
def store(request):
    return _make(request.param)


def _e(i, dim=DIM):
    v = np.zeros(dim, np.float32)
    v[i % dim] = 1.0
    return v


def test_initialization_is_empty(store):
    assert store.count() == 0 and len(store) == 0
    assert store.query(_e(0), top_k=5) == []


@pytest.mark.parametrize("bad", [0, -4])
def test_invalid_dimension_rejected(bad):
    with pytest.raises(ValueError):
        HipFlatIndex(bad, device="cpu")
    with pytest.raises(ValueError):
        InMemoryVectorStore(dimension=bad)


def test_invalid_distance_and_index_type_rejected():
    with pytest.raises(ValueError):
        HipFlatIndex(DIM, "manhattan", device="cpu")
    with pytest.raises(ValueError):
        create_vector_store("hip", dimension=DIM, index_type="hnsw", device="cpu")
    with pytest.raises(ValueError):
        create_vector_store("faiss", dimension=DIM, index_type="pq", device="cpu")
    with pytest.raises(ValueError):
        create_vector_store("pinecone")


def test_add_single_and_get(store):
    store.add_embedding("a", _e(1), {"thread_id": "t1"})
    assert store.count() == 1
    got = store.get("a")
    assert isinstance(got, SearchResult) and got.id == "a"
    assert got.metadata == {"thread_id": "t1"}
    assert np.allclose(np.asarray(got.vector) / np.linalg.norm(got.vector), _e(1), atol=1e-2)


def test_add_batch(store):
    store.add_embeddings(["a", "b", "c"], np.stack([_e(0), _e(1), _e(2)]), [{"k": 0}, {"k": 1}, {"k": 2}])
    assert store.count() == 3
    assert [store.get(i).metadata["k"] for i in "abc"] == [0, 1, 2]


def test_batch_without_metadata_gives_empty_dicts(store):
    store.add_embeddings(["a", "b"], [_e(0), _e(1)])
    assert store.get("a").metadata == {} and store.get("b").metadata == {}


def test_mismatched_lengths_raise(store):
    with pytest.raises(ValueError):
        store.add_embeddings(["a", "b"], [_e(0)])


@pytest.mark.parametrize("bad", [np.zeros(DIM + 1, np.float32), np.zeros(3, np.float32)])
def test_wrong_dimension_rejected_on_add_and_query(store, bad):
    store.add_embedding("a", _e(0))
    with pytest.raises(ValueError):
        store.add_embedding("b", bad)
    with pytest.raises(ValueError):
        store.query(bad)


def test_empty_vector_rejected(store):
    with pytest.raises(ValueError):
        store.add_embedding("a", [])


def test_empty_vector_rejected_before_dimension_is_known():
    s = InMemoryVectorStore()
    with pytest.raises(ValueError):
        s.add_embedding("a", [])
    s.add_embedding("a", [1.0, 0.0])      # the first real vector fixes the dimension
    assert s.dim == 2


def test_repeated_id_is_an_upsert(store):
    store.add_embedding("a", _e(0), {"v": 1})
    store.add_embedding("a", _e(3), {"v": 2})
    assert store.count() == 1
    assert store.get("a").metadata == {"v": 2}
    top = store.query(_e(3), top_k=1)
    assert top[0].id == "a" and top[0].score > 0.99 - (0 if top[0].score <= 1 else 1)


def test_query_returns_most_similar_first(store):
    rng = np.random.default_rng(0)
    base = rng.standard_normal((20, DIM)).astype(np.float32)
    store.add_embeddings([f"v{i}" for i in range(20)], base)
    q = base[7] + 0.01 * rng.standard_normal(DIM).astype(np.float32)
    res = store.query(q, top_k=5)
    assert res[0].id == "v7"
    scores = [r.score for r in res]
    assert scores == sorted(scores, reverse=True)


def test_top_k_respected_and_clamped(store):
    store.add_embeddings([f"v{i}" for i in range(6)], [_e(i) + 0.1 for i in range(6)])
    assert len(store.query(_e(0), top_k=3)) == 3
    assert len(store.query(_e(0), top_k=1)) == 1
    assert len(store.query(_e(0), top_k=100)) == 6


def test_delete_and_missing_ids(store):
    store.add_embeddings(["a", "b"], [_e(0), _e(1)])
    store.delete("a")
    assert store.count() == 1
    assert [r.id for r in store.query(_e(0), top_k=5)] == ["b"]
    with pytest.raises(KeyError):
        store.delete("a")
    with pytest.raises(KeyError):
        store.get("a")
    with pytest.raises(KeyError):
        store.delete("never-added")


def test_clear(store):
    store.add_embeddings(["a", "b"], [_e(0), _e(1)])
    store.clear()
    assert store.count() == 0
    assert store.query(_e(0)) == []
    store.add_embedding("c", _e(2))        # usable after clear
    assert [r.id for r in store.query(_e(2), top_k=2)] == ["c"]


def test_metadata_is_copied(store):
    meta = {"tags": ["x"]}
    store.add_embedding("a", _e(0), meta)
    meta["tags"].append("mutated")
    meta["new"] = 1
    got = store.get("a").metadata
    assert "new" not in got
    got["extra"] = True
    assert "extra" not in store.get("a").metadata
    res = store.query(_e(0), top_k=1)[0]
    res.metadata["extra"] = True
    assert "extra" not in store.query(_e(0), top_k=1)[0].metadata


@pytest.mark.parametrize("kind", COSINE_KINDS)
def test_cosine_similarity_values(kind):
    s = _make(kind)
    a = np.array([1, 0, 0, 0, 0, 0, 0, 0], np.float32)
    b = np.array([1, 1, 0, 0, 0, 0, 0, 0], np.float32)
    c = np.array([-1, 0, 0, 0, 0, 0, 0, 0], np.float32)
    s.add_embeddings(["a", "b", "c"], [a, 3 * b, c])   # scale must not matter for cosine
    res = {r.id: r.score for r in s.query(2 * a, top_k=3)}
    assert res["a"] == pytest.approx(1.0, abs=1e-2)
    assert res["b"] == pytest.approx(1 / math.sqrt(2), abs=1e-2)
    assert res["c"] == pytest.approx(-1.0, abs=1e-2)


def test_faiss_l2_distance_to_similarity():
    s = create_vector_store("faiss", dimension=DIM, device="cpu")
    s.add_embeddings(["same", "near", "far"], [_e(0), _e(0) + 0.5 * _e(1), 3 * _e(2)])
    res = {r.id: r.score for r in s.query(_e(0), top_k=3)}
    # IndexFlatL2 returns squared L2 d; the reference reports 1 / (1 + d) (faiss_store.py:224)
    assert res["same"] == pytest.approx(1.0, abs=1e-3)
    assert res["near"] == pytest.approx(1 / (1 + 0.25), abs=1e-2)
    assert res["far"] == pytest.approx(1 / (1 + 1 + 9), abs=1e-2)
    assert res["same"] > res["near"] > res["far"]


def test_query_batch_equals_single_queries(store):
    rng = np.random.default_rng(1)
    base = rng.standard_normal((30, DIM)).astype(np.float32)
    store.add_embeddings([f"v{i}" for i in range(30)], base)
    qs = rng.standard_normal((5, DIM)).astype(np.float32)
    batch = store.query_batch(qs, top_k=4)
    for q, got in zip(qs, batch):
        assert [r.id for r in got] == [r.id for r in store.query(q, top_k=4)]


@pytest.mark.parametrize("kind", ["flat", "ivf"])
def test_save_and_load_round_trip(kind, tmp_path):
    s = _make(kind)
    rng = np.random.default_rng(2)
    base = rng.standard_normal((40, DIM)).astype(np.float32)
    s.add_embeddings([f"v{i}" for i in range(40)], base, [{"i": i} for i in range(40)])
    s.delete("v3")
    s.save(tmp_path / "idx")
    t = HipFlatIndex.load(tmp_path / "idx", device="cpu")
    assert t.count() == 39
    assert t.get("v5").metadata == {"i": 5}
    with pytest.raises(KeyError):
        t.get("v3")
    q = base[11]
    assert [r.id for r in t.query(q, top_k=5)] == [r.id for r in s.query(q, top_k=5)]


def test_ivf_matches_flat_with_all_lists_probed():
    rng = np.random.default_rng(3)
    base = rng.standard_normal((200, DIM)).astype(np.float32)
    ids = [f"v{i}" for i in range(200)]
    flat = HipFlatIndex(DIM, "cosine", device="cpu")
    ivf = HipIVFIndex(DIM, "cosine", nlist=8, nprobe=8, device="cpu")
    flat.add_embeddings(ids, base)
    ivf.add_embeddings(ids, base)
    ivf.train(iters=5)
    assert ivf._list_off[-1] == 200 and len(ivf._list_off) == 9
    for q in rng.standard_normal((6, DIM)).astype(np.float32):
        assert [r.id for r in ivf.query(q, top_k=10)] == [r.id for r in flat.query(q, top_k=10)]
    # rows added after training form a tail that is still searched
    ivf.add_embedding("late", base[0] * 5)
    assert ivf.query(base[0], top_k=2)[0].id in ("v0", "late")
    assert {r.id for r in ivf.query(base[0], top_k=2)} == {"v0", "late"}


def test_compaction_after_many_deletes_keeps_answers():
    s = HipFlatIndex(DIM, "cosine", capacity=16, device="cpu")
    rng = np.random.default_rng(4)
    base = rng.standard_normal((3000, DIM)).astype(np.float32)
    s.add_embeddings([f"v{i}" for i in range(3000)], base)
    for i in range(0, 3000, 2):
        s.delete(f"v{i}")
    assert s.count() == 1500
    assert s._dead < 1500          # compaction ran at least once
    ref = InMemoryVectorStore(dimension=DIM)
    ref.add_embeddings([f"v{i}" for i in range(1, 3000, 2)], base[1::2])
    q = base[101]
    assert [r.id for r in s.query(q, top_k=5)] == [r.id for r in ref.query(q, top_k=5)]


def test_gpu_produced_tensors_accepted(store):
    t = torch.randn(4, DIM)
    store.add_embeddings(["a", "b", "c", "d"], t)
    assert store.query(t[2], top_k=1)[0].id == "c"


def _blob(n, dim, clusters, rng, spread=0.15):
    """Embedding-like data: one dominant common direction (rows ~0.95 cosine to each other) plus
    cluster structure around it -- the shape random-init / real encoders produce."""
    mu = rng.standard_normal(dim).astype(np.float32)
    mu /= np.linalg.norm(mu)
    cent = rng.standard_normal((clusters, dim)).astype(np.float32) * spread
    lab = rng.integers(0, clusters, n)
    X = 4 * mu + cent[lab] + 0.02 * rng.standard_normal((n, dim)).astype(np.float32)
    return X / np.linalg.norm(X, axis=1, keepdims=True)


def test_ivf_centered_kmeans_spreads_a_dominant_direction_over_the_lists():
    rng = np.random.default_rng(7)
    X = _blob(4000, DIM, 40, rng)
    ivf = HipIVFIndex(DIM, "cosine", nlist=32, nprobe=4, device="cpu")
    ivf.add_embeddings([f"r{i}" for i in range(4000)], X)
    ivf.train(iters=6)
    sizes = np.diff(np.asarray(ivf._list_off))
    assert ivf.center is not None
    assert sizes.max() < 0.25 * 4000, sizes          # no list swallows the blob
    flat = HipFlatIndex(DIM, "cosine", device="cpu")
    flat.add_embeddings([f"r{i}" for i in range(4000)], X)
    Q = _blob(16, DIM, 40, np.random.default_rng(7))  # same direction / clusters as the rows
    hit = sum(len({r.id for r in a} & {r.id for r in b})
              for a, b in zip(ivf.query_batch(Q, top_k=10), flat.query_batch(Q, top_k=10)))
    assert hit / 160 >= 0.8, hit


def test_ivf_compaction_keeps_lists_contiguous_and_answers_exact():
    rng = np.random.default_rng(8)
    X = rng.standard_normal((1200, DIM)).astype(np.float32)
    ids = [f"v{i}" for i in range(1200)]
    ivf = HipIVFIndex(DIM, "cosine", nlist=12, nprobe=12, device="cpu")
    ivf.add_embeddings(ids, X)
    ivf.train(iters=4)
    for i in range(0, 1200, 3):
        ivf.delete(f"v{i}")
    ivf.compact()
    flat = HipFlatIndex(DIM, "cosine", device="cpu")
    live = [i for i in range(1200) if i % 3]
    flat.add_embeddings([ids[i] for i in live], X[live])
    assert ivf._list_off[-1] == ivf._trained_n == len(live) == ivf.count()
    for q in rng.standard_normal((5, DIM)).astype(np.float32):
        assert [r.id for r in ivf.query(q, top_k=8)] == [r.id for r in flat.query(q, top_k=8)]


def test_ivf_save_load_keeps_the_trained_lists(tmp_path):
    rng = np.random.default_rng(9)
    X = _blob(2000, DIM, 20, rng)
    ivf = HipIVFIndex(DIM, "cosine", nlist=16, nprobe=3, device="cpu")
    ivf.add_embeddings([f"r{i}" for i in range(2000)], X)
    ivf.train(iters=4)
    ivf.save(tmp_path)
    back = HipIVFIndex.load(tmp_path, device="cpu")
    assert back.centroids is not None and back._list_off == ivf._list_off and back.nprobe == 3
    assert torch.allclose(back.center, ivf.center)
    for q in X[:6]:
        assert [r.id for r in back.query(q, top_k=5)] == [r.id for r in ivf.query(q, top_k=5)]
