"""Vector stores backed by external services, spoken to over their REST APIs (no SDK needed).

These are the reference's off-GPU drivers (qdrant_store.py:78, azure_ai_search_store.py:32),
kept so a deployment that already runs Qdrant / Azure AI Search can point this framework at it.
The MI355X hot path is the HBM-resident :class:`~copilot_for_consensus_amd.vectorstore.HipFlatIndex`.

* :class:`QdrantVectorStore` -- collection created on demand (size, Cosine/Euclid), string ids
  mapped to uuid5 (DNS namespace, reference qdrant_store.py:18-25) with the original id kept in the
  payload as ``_original_id``, batched upserts (100), ``/points/search`` with payload + vectors.
* :class:`AzureAISearchVectorStore` -- index with an HNSW cosine vector field, ``mergeOrUpload``
  batches, ``vectorQueries`` kNN search; metadata stored as a JSON string field.
"""
from __future__ import annotations

import json
import urllib.error
import urllib.request
import uuid
from typing import Any, Callable

import numpy as np

from . import SearchResult, VectorStore, _as_matrix

_NS = uuid.UUID("6ba7b810-9dad-11d1-80b4-00c04fd430c8")


def string_to_uuid(s: str) -> str:
    return str(uuid.uuid5(_NS, s))


class _Http:
    def __init__(self, base: str, headers: dict[str, str], timeout: float = 30.0,
                 transport: Callable | None = None):
        self.base, self.headers, self.timeout = base.rstrip("/"), headers, timeout
        self.transport = transport or self._urllib

    def _urllib(self, method: str, url: str, body: bytes | None, headers: dict) -> tuple[int, bytes]:
        req = urllib.request.Request(url, data=body, method=method, headers=headers)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read()
        except (urllib.error.URLError, OSError) as e:
            raise ConnectionError(f"{method} {url}: {e}") from e

    def __call__(self, method: str, path: str, payload: Any = None, ok=(200, 201, 202, 204)) -> tuple[int, Any]:
        body = None if payload is None else json.dumps(payload).encode()
        h = dict(self.headers)
        if body is not None:
            h["Content-Type"] = "application/json"
        code, raw = self.transport(method, self.base + path, body, h)
        data = json.loads(raw) if raw else None
        if code not in ok:
            raise RuntimeError(f"{method} {path}: HTTP {code}: {str(data)[:300]}")
        return code, data


class QdrantVectorStore(VectorStore):
    def __init__(self, host: str = "localhost", port: int = 6333, collection_name: str = "embeddings",
                 vector_size: int = 384, distance: str = "cosine", upsert_batch_size: int = 100,
                 api_key: str | None = None, url: str | None = None, transport: Callable | None = None, **_):
        if distance not in ("cosine", "euclid", "euclidean"):
            raise ValueError(f"distance must be cosine or euclid, got {distance!r}")
        self.collection, self.dim, self.batch = collection_name, int(vector_size), int(upsert_batch_size)
        self.distance = "Cosine" if distance == "cosine" else "Euclid"
        hdr = {"api-key": api_key} if api_key else {}
        self.http = _Http(url or f"http://{host}:{port}", hdr, transport=transport)
        self._ensure_collection()

    def _ensure_collection(self):
        code, data = self.http("GET", f"/collections/{self.collection}", ok=(200, 404))
        if code == 404:
            # several services start at once: another one may create it between our GET and PUT
            code, _ = self.http("PUT", f"/collections/{self.collection}",
                                {"vectors": {"size": self.dim, "distance": self.distance}}, ok=(200, 400, 409))
            if code == 200:
                return
            code, data = self.http("GET", f"/collections/{self.collection}")
        vec = data["result"]["config"]["params"]["vectors"]
        if int(vec["size"]) != self.dim:
            raise ValueError(f"collection {self.collection} has vector size {vec['size']}, expected {self.dim}")

    def add_embeddings(self, ids, vectors, metadatas=None):
        X = _as_matrix(vectors, self.dim)
        if len(ids) != X.shape[0]:
            raise ValueError("ids and vectors length mismatch")
        metadatas = list(metadatas) if metadatas is not None else [{} for _ in ids]
        pts = [{"id": string_to_uuid(i), "vector": X[j].tolist(), "payload": {**(metadatas[j] or {}),
                                                                              "_original_id": i}}
               for j, i in enumerate(ids)]
        for s in range(0, len(pts), self.batch):
            self.http("PUT", f"/collections/{self.collection}/points?wait=true", {"points": pts[s:s + self.batch]})

    def _result(self, p, score) -> SearchResult:
        payload = dict(p.get("payload") or {})
        oid = payload.pop("_original_id", str(p["id"]))
        vec = p.get("vector") or []
        if isinstance(vec, dict):
            vec = vec.get("default") or next(iter(vec.values()), [])
        return SearchResult(oid, float(score), list(vec), payload)

    def query(self, query_vector, top_k: int = 10):
        q = _as_matrix(query_vector, self.dim)[0].tolist()
        _, data = self.http("POST", f"/collections/{self.collection}/points/search",
                            {"vector": q, "limit": int(top_k), "with_payload": True, "with_vector": True})
        return [self._result(p, p["score"]) for p in data["result"]]

    def delete(self, id):
        self.get(id)  # KeyError if absent (interface contract)
        self.http("POST", f"/collections/{self.collection}/points/delete?wait=true",
                  {"points": [string_to_uuid(id)]})

    def clear(self):
        self.http("DELETE", f"/collections/{self.collection}")
        self._ensure_collection()

    def count(self):
        _, data = self.http("POST", f"/collections/{self.collection}/points/count", {"exact": True})
        return int(data["result"]["count"])

    def get(self, id):
        code, data = self.http("GET", f"/collections/{self.collection}/points/{string_to_uuid(id)}", ok=(200, 404))
        if code == 404 or not data or not data.get("result"):
            raise KeyError(id)
        return self._result(data["result"], 1.0)

    def centroid_scores(self, ids):
        """One retrieve call for the thread's points (Qdrant POST /points), scored locally."""
        ids = list(ids)
        if not ids:
            return {}
        _, data = self.http("POST", f"/collections/{self.collection}/points",
                            {"ids": [string_to_uuid(i) for i in ids], "with_vector": True, "with_payload": True})
        got = {r.id: r.vector for r in (self._result(p, 1.0) for p in data.get("result") or [])}
        have = [i for i in ids if i in got and got[i]]
        if not have:
            return {}
        X = np.asarray([got[i] for i in have], dtype=np.float32)
        X = X / np.maximum(np.linalg.norm(X, axis=1, keepdims=True), 1e-12)
        c = X.mean(0)
        c = c / max(float(np.linalg.norm(c)), 1e-12)
        return dict(zip(have, (X @ c).astype(float).tolist()))


class AzureAISearchVectorStore(VectorStore):
    API = "2023-11-01"

    def __init__(self, endpoint: str | None = None, api_key: str | None = None, index_name: str = "embeddings",
                 vector_size: int = 384, transport: Callable | None = None, batch: int = 1000, **_):
        if not endpoint or not api_key:
            raise ValueError("azure_ai_search vector store: endpoint (AZURE_SEARCH_ENDPOINT) and api_key are required")
        self.index, self.dim, self.batch = index_name, int(vector_size), batch
        self.http = _Http(endpoint, {"api-key": api_key}, transport=transport)
        self._ensure_index()

    def _p(self, path: str) -> str:
        return f"{path}{'&' if '?' in path else '?'}api-version={self.API}"

    def _ensure_index(self):
        code, _ = self.http("GET", self._p(f"/indexes/{self.index}"), ok=(200, 404))
        if code == 200:
            return
        self.http("PUT", self._p(f"/indexes/{self.index}"), {
            "name": self.index,
            "fields": [{"name": "id", "type": "Edm.String", "key": True, "filterable": True},
                       {"name": "original_id", "type": "Edm.String", "filterable": True},
                       {"name": "metadata", "type": "Edm.String"},
                       {"name": "embedding", "type": "Collection(Edm.Single)", "searchable": True,
                        "dimensions": self.dim, "vectorSearchProfile": "hnsw-cosine"}],
            "vectorSearch": {"algorithms": [{"name": "hnsw", "kind": "hnsw",
                                             "hnswParameters": {"metric": "cosine"}}],
                             "profiles": [{"name": "hnsw-cosine", "algorithm": "hnsw"}]}})

    @staticmethod
    def _key(i: str) -> str:
        # document keys allow [A-Za-z0-9_-=]; encode arbitrary ids reversibly-enough via uuid5
        return string_to_uuid(i)

    def add_embeddings(self, ids, vectors, metadatas=None):
        X = _as_matrix(vectors, self.dim)
        metadatas = list(metadatas) if metadatas is not None else [{} for _ in ids]
        docs = [{"@search.action": "mergeOrUpload", "id": self._key(i), "original_id": i,
                 "metadata": json.dumps(metadatas[j] or {}), "embedding": X[j].tolist()} for j, i in enumerate(ids)]
        for s in range(0, len(docs), self.batch):
            self.http("POST", self._p(f"/indexes/{self.index}/docs/index"), {"value": docs[s:s + self.batch]})

    def _result(self, d) -> SearchResult:
        return SearchResult(d.get("original_id") or d["id"], float(d.get("@search.score", 1.0)),
                            list(d.get("embedding") or []), json.loads(d.get("metadata") or "{}"))

    def query(self, query_vector, top_k: int = 10):
        q = _as_matrix(query_vector, self.dim)[0].tolist()
        _, data = self.http("POST", self._p(f"/indexes/{self.index}/docs/search"), {
            "vectorQueries": [{"kind": "vector", "vector": q, "fields": "embedding", "k": int(top_k)}],
            "select": "id,original_id,metadata,embedding", "top": int(top_k)})
        return [self._result(d) for d in data.get("value", [])]

    def delete(self, id):
        self.get(id)
        self.http("POST", self._p(f"/indexes/{self.index}/docs/index"),
                  {"value": [{"@search.action": "delete", "id": self._key(id)}]})

    def clear(self):
        self.http("DELETE", self._p(f"/indexes/{self.index}"), ok=(200, 204, 404))
        self._ensure_index()

    def count(self):
        _, data = self.http("GET", self._p(f"/indexes/{self.index}/docs/$count"))
        return int(data)

    def get(self, id):
        code, data = self.http("GET", self._p(f"/indexes/{self.index}/docs/{self._key(id)}"), ok=(200, 404))
        if code == 404:
            raise KeyError(id)
        return self._result(data)
