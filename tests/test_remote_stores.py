"""Networked stores for one-process-per-service deployments: the document store server (MongoDB's
role; WAL + snapshot durability, typed errors over the wire) and the Qdrant-REST front of the HIP
index, driven by this framework's own Qdrant driver (vectorstore/remote.py) exactly as the
reference's qdrant_store.py would drive a Qdrant server."""
from __future__ import annotations

import threading

import numpy as np
import pytest
import uvicorn

from copilot_for_consensus_amd.storage.document_store import (DocumentAlreadyExistsError, DocumentNotFoundError,
                                                              create_document_store)
from copilot_for_consensus_amd.storage.server import DocumentStoreServer, RemoteDocumentStore


def test_docstore_roundtrip_and_errors(tmp_path):
    srv = DocumentStoreServer(host="127.0.0.1", port=0, data_dir=tmp_path / "ds").start()
    try:
        class Cfg:
            driver_name = "cfcstore"
            driver_config = {"host": "127.0.0.1", "port": srv.port}
        st = create_document_store(Cfg())
        st.connect()
        st.insert_document("messages", {"_id": "m1", "thread_id": "t1", "n": 3})
        assert st.insert_many("messages", [{"_id": "m1"}, {"_id": "m2", "thread_id": "t1", "n": 5},
                                            {"_id": "m3", "thread_id": "t2", "n": 7}]) == ["m2", "m3"]
        with pytest.raises(DocumentAlreadyExistsError):
            st.insert_document("messages", {"_id": "m1"})
        with pytest.raises(DocumentNotFoundError):
            st.update_document("messages", "nope", {"x": 1})
        assert [d["_id"] for d in st.query_documents("messages", {"_id": {"$in": ["m1", "m3"]}}, sort_by="n",
                                                      sort_order="asc")] == ["m1", "m3"]
        assert st.update_many("messages", {"thread_id": "t1"}, {"seen": True}) == 2
        assert st.count_documents("messages", {"seen": True}) == 2
        agg = st.aggregate_documents("messages", [{"$group": {"_id": "$thread_id", "total": {"$sum": "$n"}}}])
        assert {g["_id"]: g["total"] for g in agg} == {"t1": 8, "t2": 7}
        auto = st.insert_document("sources", {"name": "ietf"})      # id assigned server side (logged)
        st.delete_document("messages", "m3")
        assert st.get_document("messages", "m3") is None
    finally:
        srv.close()
    # restart from snapshot + WAL: same documents
    srv2 = DocumentStoreServer(host="127.0.0.1", port=0, data_dir=tmp_path / "ds").start()
    try:
        st2 = RemoteDocumentStore(host="127.0.0.1", port=srv2.port)
        st2.connect()
        assert st2.collection_counts() == {"messages": 2, "sources": 1}
        assert st2.get_document("sources", auto)["name"] == "ietf"
        assert st2.get_document("messages", "m2")["seen"] is True
    finally:
        srv2.close()


def test_docstore_wal_replay_after_crash(tmp_path):
    """No clean shutdown (no snapshot): the write-ahead log alone restores every acknowledged write;
    a torn last record is dropped."""
    srv = DocumentStoreServer(host="127.0.0.1", port=0, data_dir=tmp_path / "ds").start()
    st = RemoteDocumentStore(host="127.0.0.1", port=srv.port)
    st.connect()
    for i in range(50):
        st.insert_document("chunks", {"_id": f"c{i}", "embedding_generated": False})
    st.update_many("chunks", {"_id": {"$in": [f"c{i}" for i in range(10)]}}, {"embedding_generated": True})
    srv.server.shutdown()
    srv.server.server_close()
    srv._wal.close()                      # simulate a crash: no snapshot
    with open(tmp_path / "ds" / "wal.jsonl", "a") as fh:
        fh.write('{"op": "insert_document", "args": ["chunks", {"_id": "tor')
    srv2 = DocumentStoreServer(host="127.0.0.1", port=0, data_dir=tmp_path / "ds").start()
    try:
        assert srv2.replayed == 51
        st2 = RemoteDocumentStore(host="127.0.0.1", port=srv2.port)
        assert st2.count_documents("chunks") == 50
        assert st2.count_documents("chunks", {"embedding_generated": True}) == 10
    finally:
        srv2.close()


def test_docstore_client_reconnects_after_restart(tmp_path):
    srv = DocumentStoreServer(host="127.0.0.1", port=0, data_dir=tmp_path / "ds").start()
    port = srv.port
    st = RemoteDocumentStore(host="127.0.0.1", port=port)
    st.connect()
    st.insert_document("threads", {"_id": "t"})
    srv.close()
    srv2 = DocumentStoreServer(host="127.0.0.1", port=port, data_dir=tmp_path / "ds").start()
    try:
        assert st.get_document("threads", "t") == {"_id": "t"}     # stale socket detected, reconnected
        st.insert_document("threads", {"_id": "u"})
    finally:
        srv2.close()


@pytest.fixture
def qdrant_server(tmp_path):
    from copilot_for_consensus_amd.vectorstore.server import create_vector_app
    app = create_vector_app(device="cpu", capacity=4096, persist_dir=str(tmp_path / "vs"))
    cfg = uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error")
    server = uvicorn.Server(cfg)
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    import time
    while not server.started:
        time.sleep(0.02)
    port = server.servers[0].sockets[0].getsockname()[1]
    yield app, port
    server.should_exit = True
    t.join(10)


def test_qdrant_rest_front_with_reference_driver(qdrant_server):
    from copilot_for_consensus_amd.vectorstore import InMemoryVectorStore, create_vector_store
    app, port = qdrant_server

    class Cfg:
        driver_name = "qdrant"
        driver_config = {"host": "127.0.0.1", "port": port, "collection_name": "embeddings", "vector_size": 16,
                         "distance": "cosine", "upsert_batch_size": 7}
    vs = create_vector_store(Cfg())
    ref = InMemoryVectorStore(16)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((40, 16)).astype(np.float32)
    ids = [f"chunk-{i}" for i in range(40)]
    meta = [{"thread_id": f"t{i % 5}"} for i in range(40)]
    vs.add_embeddings(ids, X, meta)
    ref.add_embeddings(ids, X, meta)
    vs.add_embeddings(["chunk-3"], X[7:8], [{"thread_id": "moved"}])      # upsert overwrites
    ref.add_embeddings(["chunk-3"], X[7:8], [{"thread_id": "moved"}])
    assert vs.count() == 40
    q = rng.standard_normal(16).astype(np.float32)
    got, want = vs.query(q, top_k=5), ref.query(q, top_k=5)
    assert [r.id for r in got] == [r.id for r in want]
    np.testing.assert_allclose([r.score for r in got], [r.score for r in want], atol=2e-2)   # bf16 storage
    assert got[0].metadata["thread_id"] == want[0].metadata["thread_id"]
    assert vs.get("chunk-3").metadata == {"thread_id": "moved"}
    vs.delete("chunk-0")
    assert vs.count() == 39
    with pytest.raises(KeyError):
        vs.get("chunk-0")
    # a second client sees the same collection (dimension checked); persistence snapshot works
    vs2 = create_vector_store(Cfg())
    assert vs2.count() == 39
    app.state.save_all()


def test_qdrant_rest_query_points_and_errors(qdrant_server):
    import json
    import urllib.request
    _, port = qdrant_server
    base = f"http://127.0.0.1:{port}"

    def call(method, path, body=None):
        req = urllib.request.Request(base + path, method=method, data=None if body is None else json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req) as r:
                return r.status, json.loads(r.read())
        except urllib.error.HTTPError as e:
            return e.code, json.loads(e.read())

    assert call("GET", "/collections/x")[0] == 404
    assert call("PUT", "/collections/x", {"vectors": {"size": 3, "distance": "Euclid"}})[0] == 200
    assert call("PUT", "/collections/x", {"vectors": {"size": 3, "distance": "Euclid"}})[0] == 409
    assert call("PUT", "/collections/x/points", {"points": [{"id": 1, "vector": [0, 0, 0]},
                                                            {"id": 2, "vector": [3, 4, 0], "payload": {"a": 1}}]})[0] == 200
    code, data = call("POST", "/collections/x/points/query", {"query": [3, 4, 0], "limit": 2, "with_payload": True})
    pts = data["result"]["points"]
    assert code == 200 and [p["id"] for p in pts] == [2, 1]
    assert pts[0]["score"] == pytest.approx(0.0, abs=1e-3) and pts[1]["score"] == pytest.approx(5.0, rel=1e-2)
    code, data = call("POST", "/collections/x/points/search", {"vector": [1, 1], "limit": 1})
    assert code == 400
    code, data = call("POST", "/collections/x/points/search/batch",
                      {"searches": [{"vector": [0, 0, 0], "limit": 1}, {"vector": [3, 4, 0], "limit": 1}]})
    assert [[p["id"] for p in r] for r in data["result"]] == [[1], [2]]


def test_qdrant_rest_rejects_path_traversal_names(qdrant_server, tmp_path):
    """a collection named '..' (or with a slash) must never reach save() / rmtree()."""
    import json
    import urllib.request
    app, port = qdrant_server
    base = f"http://127.0.0.1:{port}"
    marker = tmp_path / "keep.txt"
    marker.write_text("x")

    def call(method, path, body=None):
        req = urllib.request.Request(base + path, method=method, data=None if body is None else json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req) as r:
                return r.status
        except urllib.error.HTTPError as e:
            return e.code

    for bad in ("%2E%2E", "a%2Fb", "..", "x%00y", "a.b"):
        assert call("PUT", f"/collections/{bad}", {"vectors": {"size": 3}}) in (400, 404), bad
        assert call("DELETE", f"/collections/{bad}") in (400, 404), bad
        assert call("PUT", f"/collections/{bad}/points", {"points": []}) in (400, 404), bad
    assert call("PUT", "/collections/ok_name-1", {"vectors": {"size": 3}}) == 200
    app.state.save_all()
    assert marker.exists() and (tmp_path / "vs" / "ok_name-1" / "collection.json").exists()
    assert call("DELETE", "/collections/ok_name-1") == 200
    assert marker.exists() and not (tmp_path / "vs" / "ok_name-1").exists()
    assert sorted(app.state.collections) == []


def test_docstore_client_retries_only_idempotent_writes():
    """After a lost reply a plain field update is re-sent, a counter / array operator update is
    not (it may already have been applied)."""
    from copilot_for_consensus_amd.storage.server import _idempotent
    assert _idempotent("update_document", ("c", "id", {"status": "done"}))
    assert _idempotent("update_many", ("c", {"a": 1}, {"$set": {"b": 2}}))
    assert _idempotent("clear_collection", ("c",))
    assert not _idempotent("update_document", ("c", "id", {"$inc": {"attemptCount": 1}}))
    assert not _idempotent("update_many", ("c", {}, {"$push": {"log": "x"}}))
    assert not _idempotent("insert_document", ("c", {"_id": "x"}))
