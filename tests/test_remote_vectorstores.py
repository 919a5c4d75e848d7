"""REST vector-store drivers (Qdrant, Azure AI Search) against in-process fakes of the services'
HTTP APIs (no network): upsert semantics, uuid5 id mapping, search ordering, delete/count/get."""
import json
import math
import re

import pytest

from copilot_for_consensus_amd.vectorstore import create_vector_store
from copilot_for_consensus_amd.vectorstore.remote import AzureAISearchVectorStore, QdrantVectorStore, string_to_uuid


def _cos(a, b):
    na = math.sqrt(sum(x * x for x in a)) or 1.0
    nb = math.sqrt(sum(x * x for x in b)) or 1.0
    return sum(x * y for x, y in zip(a, b)) / (na * nb)


class FakeQdrant:
    def __init__(self):
        self.cols = {}

    def __call__(self, method, url, body, headers):
        path = re.sub(r"^http://[^/]+", "", url).split("?")[0]
        req = json.loads(body) if body else None
        m = re.match(r"^/collections/([^/]+)(/.*)?$", path)
        name, rest = m.group(1), m.group(2) or ""
        col = self.cols.get(name)
        if rest == "" and method == "GET":
            if col is None:
                return 404, b'{"status":"not found"}'
            return 200, json.dumps({"result": {"config": {"params": {"vectors": col["cfg"]}}}}).encode()
        if rest == "" and method == "PUT":
            self.cols[name] = {"cfg": req["vectors"], "pts": {}}
            return 200, b'{"result":true}'
        if rest == "" and method == "DELETE":
            self.cols.pop(name, None)
            return 200, b'{"result":true}'
        if rest == "/points" and method == "PUT":
            for p in req["points"]:
                col["pts"][p["id"]] = p
            return 200, b'{"result":{}}'
        if rest == "/points/search":
            sc = sorted(((_cos(req["vector"], p["vector"]), p) for p in col["pts"].values()), key=lambda t: -t[0])
            return 200, json.dumps({"result": [{**p, "score": s} for s, p in sc[:req["limit"]]]}).encode()
        if rest == "/points/delete":
            for i in req["points"]:
                col["pts"].pop(i, None)
            return 200, b'{"result":{}}'
        if rest == "/points/count":
            return 200, json.dumps({"result": {"count": len(col["pts"])}}).encode()
        if rest.startswith("/points/") and method == "GET":
            p = col["pts"].get(rest.split("/")[-1])
            return (404, b'{"result":null}') if p is None else (200, json.dumps({"result": p}).encode())
        return 400, b'{}'


def test_qdrant_rest_driver():
    fake = FakeQdrant()
    vs = QdrantVectorStore(collection_name="c", vector_size=3, transport=fake, upsert_batch_size=2)
    vs.add_embeddings(["a", "b", "c"], [[1, 0, 0], [0, 1, 0], [0.9, 0.1, 0]], [{"k": 1}, {"k": 2}, {"k": 3}])
    assert vs.count() == 3 and string_to_uuid("a") in fake.cols["c"]["pts"]
    res = vs.query([1, 0, 0], top_k=2)
    assert [r.id for r in res] == ["a", "c"] and res[0].metadata == {"k": 1}
    vs.add_embedding("a", [0, 0, 1], {"k": 9})     # upsert, not duplicate
    assert vs.count() == 3 and vs.get("a").metadata == {"k": 9}
    vs.delete("b")
    with pytest.raises(KeyError):
        vs.get("b")
    vs.clear()
    assert vs.count() == 0
    with pytest.raises(ValueError):
        QdrantVectorStore(collection_name="c", vector_size=4, transport=fake)


class FakeSearch:
    def __init__(self):
        self.indexes = {}

    def __call__(self, method, url, body, headers):
        assert headers["api-key"] == "k"
        path = re.sub(r"^https://[^/]+", "", url).split("?")[0]
        req = json.loads(body) if body else None
        m = re.match(r"^/indexes/([^/]+)(/.*)?$", path)
        name, rest = m.group(1), m.group(2) or ""
        idx = self.indexes.get(name)
        if rest == "":
            if method == "GET":
                return (404, b"{}") if idx is None else (200, b"{}")
            if method == "PUT":
                self.indexes[name] = {}
                return 201, b"{}"
            if method == "DELETE":
                self.indexes.pop(name, None)
                return 204, b""
        if rest == "/docs/index":
            for d in req["value"]:
                if d["@search.action"] == "delete":
                    idx.pop(d["id"], None)
                else:
                    idx[d["id"]] = {k: v for k, v in d.items() if not k.startswith("@")}
            return 200, b'{"value":[]}'
        if rest == "/docs/search":
            q = req["vectorQueries"][0]
            sc = sorted(((_cos(q["vector"], d["embedding"]), d) for d in idx.values()), key=lambda t: -t[0])
            return 200, json.dumps({"value": [{**d, "@search.score": s} for s, d in sc[:q["k"]]]}).encode()
        if rest == "/docs/$count":
            return 200, str(len(idx)).encode()
        if rest.startswith("/docs/"):
            d = idx.get(rest.split("/")[-1])
            return (404, b"{}") if d is None else (200, json.dumps(d).encode())
        return 400, b"{}"


def test_azure_ai_search_rest_driver():
    vs = create_vector_store("azure_ai_search", endpoint="https://x.search.windows.net", api_key="k",
                             vector_size=2, transport=FakeSearch())
    assert isinstance(vs, AzureAISearchVectorStore)
    vs.add_embeddings(["m1", "m2"], [[1, 0], [0, 1]], [{"t": "a"}, {"t": "b"}])
    r = vs.query([0.1, 1.0], top_k=1)
    assert r[0].id == "m2" and r[0].metadata == {"t": "b"} and vs.count() == 2
    vs.delete("m1")
    assert vs.count() == 1
