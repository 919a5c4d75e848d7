"""Document store: Mongo operator semantics, hash-index consistency, updates, aggregation,
validation decorator.  Mirrors adapters/copilot_storage/tests/test_inmemory_document_store.py and
test_validating_document_store.py of the reference, plus the ``$in`` / ``$or`` / dotted-path
operators its services shim in their own tests."""
from __future__ import annotations

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from copilot_for_consensus_amd.storage import query
from copilot_for_consensus_amd.storage.document_store import (DocumentAlreadyExistsError, DocumentNotFoundError,
                                                               DocumentStoreError, InMemoryDocumentStore,
                                                               ValidatingDocumentStore, create_document_store)


@pytest.fixture
def store():
    s = InMemoryDocumentStore()
    s.connect()
    return s


def _seed(store):
    docs = [
        {"_id": "a", "thread_id": "t1", "n": 1, "tags": ["x", "y"], "meta": {"lang": "en"}, "embedding_generated": False},
        {"_id": "b", "thread_id": "t1", "n": 5, "tags": ["y"], "meta": {"lang": "fr"}, "embedding_generated": True},
        {"_id": "c", "thread_id": "t2", "n": 9, "tags": [], "meta": {"lang": "en"}, "embedding_generated": False},
        {"_id": "d", "thread_id": None, "n": None},
    ]
    for d in docs:
        store.insert_document("chunks", d)
    return docs


def ids(docs):
    return sorted(d["_id"] for d in docs)


def test_insert_get_roundtrip_is_a_copy(store):
    doc = {"_id": "x1", "body": {"k": [1, 2]}}
    assert store.insert_document("messages", doc) == "x1"
    got = store.get_document("messages", "x1")
    assert got == doc
    got["body"]["k"].append(3)  # mutating the returned copy must not leak into the store
    assert store.get_document("messages", "x1")["body"]["k"] == [1, 2]
    doc["body"]["k"].append(9)  # nor mutating the caller's dict after insert
    assert store.get_document("messages", "x1")["body"]["k"] == [1, 2]


def test_insert_generates_id_and_rejects_duplicates(store):
    new_id = store.insert_document("messages", {"a": 1})
    assert isinstance(new_id, str) and len(new_id) >= 16
    with pytest.raises(DocumentAlreadyExistsError):
        store.insert_document("messages", {"_id": new_id, "a": 2})


def test_insert_many_ignores_duplicates(store):
    store.insert_document("chunks", {"_id": "a"})
    out = store.insert_many("chunks", [{"_id": "a"}, {"_id": "b"}, {"_id": "c"}])
    assert sorted(out) == ["b", "c"]
    assert store.count_documents("chunks") == 3


def test_missing_document(store):
    assert store.get_document("threads", "nope") is None
    with pytest.raises(DocumentNotFoundError):
        store.update_document("threads", "nope", {"a": 1})
    with pytest.raises(DocumentNotFoundError):
        store.delete_document("threads", "nope")


@pytest.mark.parametrize("flt,expect", [
    ({"thread_id": "t1"}, ["a", "b"]),
    ({"thread_id": {"$in": ["t1", "t2"]}}, ["a", "b", "c"]),
    ({"thread_id": {"$nin": ["t1"]}}, ["c", "d"]),
    ({"n": {"$gt": 1}}, ["b", "c"]),
    ({"n": {"$gte": 1, "$lt": 9}}, ["a", "b"]),
    ({"n": {"$lte": 5}}, ["a", "b"]),
    ({"n": {"$ne": 5}}, ["a", "c", "d"]),
    ({"tags": "y"}, ["a", "b"]),                       # scalar condition on an array: any element
    ({"tags": {"$all": ["x", "y"]}}, ["a"]),
    ({"tags": {"$size": 0}}, ["c"]),
    ({"meta.lang": "en"}, ["a", "c"]),                 # dotted path
    ({"meta": {"$exists": False}}, ["d"]),
    ({"thread_id": None}, ["d"]),
    ({"$or": [{"n": 1}, {"n": 9}]}, ["a", "c"]),
    ({"$and": [{"thread_id": "t1"}, {"embedding_generated": False}]}, ["a"]),
    ({"$nor": [{"thread_id": "t1"}]}, ["c", "d"]),
    ({"n": {"$not": {"$gt": 4}}}, ["a", "d"]),
    ({"meta.lang": {"$regex": "^E", "$options": "i"}}, ["a", "c"]),
    ({"tags": {"$elemMatch": {"$eq": "x"}}}, ["a"]),
    ({"_id": {"$in": ["a", "c", "zz"]}}, ["a", "c"]),
])
def test_query_operators(store, flt, expect):
    _seed(store)
    assert ids(store.query_documents("chunks", flt)) == expect
    assert store.count_documents("chunks", flt) == len(expect)


def test_unsupported_operator_raises(store):
    _seed(store)
    with pytest.raises(ValueError):
        store.query_documents("chunks", {"n": {"$near": 3}})


def test_sort_skip_limit(store):
    _seed(store)
    got = store.query_documents("chunks", {}, sort_by="n", sort_order="asc")
    assert [d["_id"] for d in got] == ["d", "a", "b", "c"]  # None sorts first ascending
    got = store.query_documents("chunks", {}, sort_by="n", sort_order="desc", limit=2)
    assert [d["_id"] for d in got] == ["c", "b"]
    got = store.query_documents("chunks", {}, sort_by="n", sort_order="asc", skip=1, limit=2)
    assert [d["_id"] for d in got] == ["a", "b"]
    with pytest.raises(DocumentStoreError):
        store.query_documents("chunks", {}, sort_order="sideways")


def test_update_operators_and_index_maintenance(store):
    _seed(store)
    store.update_document("chunks", "a", {"$set": {"embedding_generated": True, "meta.lang": "de"},
                                          "$inc": {"attemptCount": 1}, "$push": {"tags": "z"}})
    a = store.get_document("chunks", "a")
    assert a["embedding_generated"] is True and a["meta"]["lang"] == "de" and a["attemptCount"] == 1
    assert a["tags"] == ["x", "y", "z"]
    store.update_document("chunks", "a", {"$addToSet": {"tags": "z"}, "$unset": {"meta": ""}})
    a = store.get_document("chunks", "a")
    assert a["tags"] == ["x", "y", "z"] and "meta" not in a
    # the hash index on embedding_generated must follow the update
    assert ids(store.query_documents("chunks", {"embedding_generated": False})) == ["c"]
    # a plain patch replaces fields; the id is immutable
    store.update_document("chunks", "c", {"thread_id": "t9", "_id": "hijack"})
    assert store.get_document("chunks", "c")["thread_id"] == "t9"
    assert ids(store.query_documents("chunks", {"thread_id": "t9"})) == ["c"]
    assert store.query_documents("chunks", {"thread_id": "t2"}) == []


def test_update_many_delete_many(store):
    _seed(store)
    assert store.update_many("chunks", {"thread_id": "t1"}, {"$set": {"embedding_generated": True}}) == 2
    assert ids(store.query_documents("chunks", {"embedding_generated": True})) == ["a", "b"]
    assert store.delete_many("chunks", {"thread_id": {"$in": ["t1"]}}) == 2
    assert ids(store.query_documents("chunks", {})) == ["c", "d"]
    store.delete_document("chunks", "c")
    assert store.query_documents("chunks", {"thread_id": "t2"}) == []
    store.clear_collection("chunks")
    assert store.count_documents("chunks") == 0


def test_aggregate_pipeline(store):
    _seed(store)
    for t in ("t1", "t2"):
        store.insert_document("threads", {"_id": t, "subject": f"s-{t}"})
    out = store.aggregate_documents("chunks", [
        {"$match": {"thread_id": {"$in": ["t1", "t2"]}}},
        {"$group": {"_id": "$thread_id", "count": {"$sum": 1}, "total": {"$sum": "$n"}, "hi": {"$max": "$n"}}},
        {"$sort": {"_id": 1}},
    ])
    assert out == [{"_id": "t1", "count": 2, "total": 6, "hi": 5}, {"_id": "t2", "count": 1, "total": 9, "hi": 9}]
    out = store.aggregate_documents("chunks", [
        {"$match": {"_id": "a"}},
        {"$lookup": {"from": "threads", "localField": "thread_id", "foreignField": "_id", "as": "thread"}},
        {"$project": {"thread": 1}},
    ])
    assert out == [{"_id": "a", "thread": [{"_id": "t1", "subject": "s-t1"}]}]
    assert store.aggregate_documents("chunks", [{"$match": {"n": {"$gt": 0}}}, {"$count": "c"}]) == [{"c": 3}]
    assert len(store.aggregate_documents("chunks", [{"$skip": 1}, {"$limit": 2}])) == 2
    with pytest.raises(DocumentStoreError):
        store.aggregate_documents("chunks", [{"$bucket": {}}])


def test_threadsafe_concurrent_inserts(store):
    import threading

    def worker(k):
        for i in range(200):
            store.insert_document("messages", {"_id": f"{k}-{i}", "archive_id": f"arc{k % 3}"})

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert store.count_documents("messages") == 1600
    assert sum(store.count_documents("messages", {"archive_id": f"arc{j}"}) for j in range(3)) == 1600


def test_validating_store_rejects_bad_documents():
    vs = ValidatingDocumentStore(InMemoryDocumentStore())
    vs.connect()
    with pytest.raises(Exception):
        vs.insert_document("archives", {"_id": "not-hex", "status": "weird-status"})
    lenient = ValidatingDocumentStore(InMemoryDocumentStore(), strict=False)
    lenient.insert_document("archives", {"_id": "not-hex", "status": "weird-status"})
    assert lenient.get_document("archives", "not-hex") is not None


def test_factory_drivers():
    s = create_document_store("inmemory")
    assert isinstance(s, InMemoryDocumentStore)
    v = create_document_store("inmemory", enable_validation=True)
    assert isinstance(v, ValidatingDocumentStore)
    with pytest.raises(ValueError):
        create_document_store("cassandra")


# ------------------------------------------------------------------ property tests
_vals = st.one_of(st.none(), st.integers(-3, 3), st.sampled_from(["p", "q", "r"]))
_docs = st.lists(st.fixed_dictionaries({}, optional={
    "thread_id": _vals, "archive_id": _vals, "n": st.integers(-5, 5), "tags": st.lists(st.sampled_from(["p", "q"]), max_size=3),
}), max_size=12)
_filters = st.one_of(
    st.builds(lambda v: {"thread_id": v}, _vals),
    st.builds(lambda vs: {"thread_id": {"$in": vs}}, st.lists(_vals, max_size=3)),
    st.builds(lambda v, n: {"archive_id": v, "n": {"$gte": n}}, _vals, st.integers(-5, 5)),
    st.builds(lambda v: {"tags": v}, st.sampled_from(["p", "q"])),
    st.builds(lambda a, b: {"$or": [{"thread_id": a}, {"archive_id": b}]}, _vals, _vals),
    # pre-hashed $in / $nin sets (query.prepare_filter) against the linear matcher: array fields,
    # missing fields (None in the set), $nin, nested under $or / $and
    st.builds(lambda vs: {"tags": {"$in": vs}}, st.lists(st.sampled_from(["p", "q", "r"]), max_size=3)),
    st.builds(lambda vs: {"archive_id": {"$nin": vs}}, st.lists(_vals, max_size=3)),
    st.builds(lambda vs: {"absent": {"$in": vs}}, st.lists(_vals, max_size=2)),
    st.builds(lambda a, vs: {"$and": [{"thread_id": {"$in": vs}}, {"n": {"$gte": a}}]}, st.integers(-5, 5),
              st.lists(_vals, max_size=3)),
)


@settings(max_examples=150, deadline=None)
@given(_docs, _filters)
def test_indexed_lookup_equals_full_scan(docs, flt):
    """The hash-index fast path must never change a query's answer."""
    indexed = InMemoryDocumentStore(indexes={"c": ("thread_id", "archive_id", "tags")})
    plain = InMemoryDocumentStore(indexes={})
    for i, d in enumerate(docs):
        d = {"_id": f"d{i}", **d}
        indexed.insert_document("c", d)
        plain.insert_document("c", d)
    want = sorted(d["_id"] for d in plain.collections["c"].values() if query.matches(d, flt))
    assert ids(plain.query_documents("c", flt, limit=None)) == want
    assert ids(indexed.query_documents("c", flt, limit=None)) == want


def test_validating_store_batch_skips_invalid_and_keeps_the_rest():
    """One malformed message must not fail a whole archive (reference parsing service: log the
    validation error, skip, continue)."""
    inner = InMemoryDocumentStore()
    vs = ValidatingDocumentStore(inner)
    good = {"_id": "0123456789abcdef", "file_hash": "a" * 64, "file_size_bytes": 1, "source": "s",
            "ingestion_date": "2025-01-01T00:00:00Z", "status": "pending"}
    bad = {"_id": "fedcba9876543210", "status": "weird-status"}
    ids = vs.insert_many("archives", [good, bad])
    assert ids == ["0123456789abcdef"] and vs.skipped == 1 and len(vs.validation_errors) == 1
    assert inner.get_document("archives", "fedcba9876543210") is None
    lenient = ValidatingDocumentStore(InMemoryDocumentStore(), strict=False)
    assert len(lenient.insert_many("archives", [good, bad])) == 2      # lenient: recorded, stored


def test_validating_store_checks_updates_against_the_result():
    vs = ValidatingDocumentStore(InMemoryDocumentStore())
    vs.insert_document("archives", {"_id": "0123456789abcdef", "file_hash": "a" * 64, "file_size_bytes": 1,
                                    "source": "s", "ingestion_date": "2025-01-01T00:00:00Z", "status": "pending"})
    vs.update_document("archives", "0123456789abcdef", {"$set": {"status": "completed"}})
    with pytest.raises(DocumentStoreError):
        vs.update_document("archives", "0123456789abcdef", {"$set": {"status": "exploded"}})
    assert vs.get_document("archives", "0123456789abcdef")["status"] == "completed"
    with pytest.raises(DocumentNotFoundError):
        vs.update_document("archives", "ffffffffffffffff", {"status": "completed"})
