"""The MongoDB document-store driver (storage/document_store.py: MongoDocumentStore) against a
stand-in pymongo client (tests/fake_pymongo.py): the image has the pymongo package but no MongoDB
server, so the client API is faked in-process (wire-level parity with a live mongod stays unpinned).

Checks the reference driver's contract (mongo_document_store.py:103-452): ping on connect, admin
authSource by default, typed connection errors; ObjectId ids round-trip as strings (nested ids in
aggregation results too); sanitised results; sort_order validation; duplicate keys ->
DocumentAlreadyExistsError; the collections.config.json indexes created on connect; and the whole
service pipeline running on DOCUMENT_STORE_TYPE=mongodb.
"""
from __future__ import annotations

import os
import shutil

import pytest

import fake_pymongo
from copilot_for_consensus_amd.storage.document_store import (DocumentAlreadyExistsError, DocumentNotFoundError,
                                                              DocumentStoreConnectionError, DocumentStoreError,
                                                              DocumentStoreNotConnectedError, MongoDocumentStore,
                                                              create_document_store)


@pytest.fixture
def server(monkeypatch):
    return fake_pymongo.install(monkeypatch)


def _store(**kw):
    s = MongoDocumentStore(host="127.0.0.1", port=27017, database="copilot", **kw)
    s.connect()
    return s


def test_connect_auth_and_failures(server):
    with pytest.raises(DocumentStoreNotConnectedError):
        MongoDocumentStore(host="h").get_document("archives", "x")
    server.up = False
    with pytest.raises(DocumentStoreConnectionError):
        _store()
    server.up = True
    server.users = {("svc", "pw"): "admin"}
    with pytest.raises(DocumentStoreConnectionError):
        _store(username="svc", password="wrong")
    s = _store(username="svc", password="pw")
    assert server.clients[-1]["authSource"] == "admin"          # reference default
    s.disconnect()
    with pytest.raises(ValueError):
        MongoDocumentStore(host="")


def test_collections_and_indexes_created_on_connect(server):
    from copilot_for_consensus_amd.contracts.documents import collections_config
    _store()
    names = set(server.dbs["copilot"])
    assert {c["name"] for c in collections_config()["collections"]} <= names
    # a unique index from the config is enforced by the server
    s = _store()
    s.insert_document("sources", {"name": "wg", "source_type": "local", "url": "/x"})
    with pytest.raises(DocumentAlreadyExistsError):
        s.insert_document("sources", {"name": "wg", "source_type": "local", "url": "/y"})


def test_crud_objectid_roundtrip_and_errors(server):
    s = _store()
    oid = s.insert_document("archives", {"source": "wg", "status": "pending", "file_size_bytes": 3})
    assert fake_pymongo.ObjectId.is_valid(oid)                     # server-assigned, returned as str
    got = s.get_document("archives", oid)
    assert got["_id"] == oid and got["status"] == "pending"
    s.update_document("archives", oid, {"status": "processed"})
    s.update_document("archives", oid, {"$inc": {"file_size_bytes": 2}})
    assert s.get_document("archives", oid)["file_size_bytes"] == 5
    sid = s.insert_document("archives", {"_id": "abcdef0123456789", "source": "wg", "status": "pending"})
    assert sid == "abcdef0123456789" and s.get_document("archives", sid)["source"] == "wg"
    with pytest.raises(DocumentAlreadyExistsError):
        s.insert_document("archives", {"_id": sid})
    with pytest.raises(DocumentNotFoundError):
        s.update_document("archives", "f" * 24, {"status": "x"})
    s.delete_document("archives", oid)
    assert s.get_document("archives", oid) is None
    with pytest.raises(DocumentNotFoundError):
        s.delete_document("archives", oid)


def test_query_sort_skip_limit_and_batched_ops(server):
    s = _store()
    for i in range(10):
        s.insert_document("messages", {"_id": f"{i:016x}", "thread_id": "t1" if i < 6 else "t2", "n": i,
                                       **({"date": f"2025-01-{i + 1:02d}"} if i % 3 else {})})
    q = s.query_documents("messages", {"thread_id": {"$in": ["t1"]}, "n": {"$gte": 2}}, sort_by="n",
                          sort_order="asc", limit=2, skip=1)
    assert [d["n"] for d in q] == [3, 4]
    desc = s.query_documents("messages", {}, sort_by="date", sort_order="desc", limit=0)
    assert [d.get("date") for d in desc[-4:]] == [None] * 4          # missing dates sort lowest
    with pytest.raises(DocumentStoreError):
        s.query_documents("messages", {}, sort_by="n", sort_order="sideways")
    assert s.count_documents("messages", {"thread_id": "t2"}) == 4
    assert s.update_many("messages", {"thread_id": "t2"}, {"status": "done"}) == 4
    assert s.delete_many("messages", {"status": "done"}) == 4
    ids = s.insert_many("messages", [{"_id": "0" * 16, "n": 0}, {"_id": "f" * 16, "n": 99}])
    assert ids == ["f" * 16]                                         # duplicate skipped
    with pytest.raises(DocumentAlreadyExistsError):
        s.insert_many("messages", [{"_id": "0" * 16}], ignore_duplicates=False)


def test_aggregate_lookup_stringifies_nested_ids(server):
    s = _store()
    t = s.insert_document("threads", {"subject": "s"})             # ObjectId thread id
    s.insert_document("summaries", {"_id": "1" * 16, "thread_id": fake_pymongo.ObjectId(t), "summary_type": "x"})
    out = s.aggregate_documents("summaries", [{"$lookup": {"from": "threads", "localField": "thread_id",
                                                           "foreignField": "_id", "as": "thread"}}])
    assert out[0]["thread_id"] == t and out[0]["thread"][0]["_id"] == t
    assert isinstance(out[0]["thread"][0]["_id"], str)


def test_services_pipeline_on_mongodb(server, tmp_path):
    """The whole pipeline with the reference's default store driver (DOCUMENT_STORE_TYPE=mongodb)."""
    from copilot_for_consensus_amd.embedding import HipEncoderProvider
    from copilot_for_consensus_amd.services.node import Node
    from copilot_for_consensus_amd.summarization import MockSummarizer
    from copilot_for_consensus_amd.vectorstore import HipFlatIndex
    env = {"DOCUMENT_STORE_TYPE": "mongodb", "MONGODB_HOST": "127.0.0.1", "MESSAGE_BUS_TYPE": "inproc",
           "METRICS_TYPE": "noop", "LOG_TYPE": "silent", "ERROR_REPORTER_TYPE": "silent",
           "EMBEDDING_BACKEND_TYPE": "mock", "VECTOR_STORE_TYPE": "inmemory", "LLM_BACKEND_TYPE": "mock",
           "ARCHIVE_STORE_TYPE": "inmemory", "SECRET_PROVIDER_TYPE": "env"}
    emb = HipEncoderProvider(model_name="tiny", device="cpu")
    node = Node(env=env, embedding_provider=emb, vector_store=HipFlatIndex(emb.dimension, device="cpu"),
                summarizer=MockSummarizer(mock_latency_ms=0))
    assert isinstance(node.store, MongoDocumentStore)
    node.start(threaded=False)
    src = tmp_path / "src"
    src.mkdir()
    shutil.copy(os.path.join(os.path.dirname(__file__), "fixtures", "sample.mbox"), src / "list.mbox")
    ing = node.services["ingestion"]
    ing.create_source({"name": "wg", "source_type": "local", "url": str(src)})
    ing.trigger_ingestion("wg")
    node.drain()
    db = server.dbs["copilot"]
    assert len(db["summaries"].docs) == 2 and len(db["threads"].docs) == 2
    assert all(d.get("summary_id") for d in db["threads"].docs.values())
    assert create_document_store("mongodb").__class__ is MongoDocumentStore


def test_real_bson_object_ids_round_trip():
    """With the real pymongo package present, ids use bson.ObjectId: a 24-hex id is queried as an
    ObjectId, anything else (the framework's 16-hex content ids) as the raw string, and nested
    ObjectIds in results come back as strings."""
    bson = pytest.importorskip("bson")
    oid = bson.ObjectId()
    s = MongoDocumentStore(host="127.0.0.1", port=27017, database="copilot")
    q = s._oid_query(str(oid))
    assert isinstance(q["_id"], bson.ObjectId) and q["_id"] == oid
    assert s._oid_query("0123456789abcdef") == {"_id": "0123456789abcdef"}
    doc = {"_id": oid, "thread": {"ids": [bson.ObjectId(), "x"]}}
    out = MongoDocumentStore._stringify_ids(doc)
    assert out["_id"] == str(oid) and isinstance(out["thread"]["ids"][0], str) and out["thread"]["ids"][1] == "x"
