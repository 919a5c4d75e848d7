"""Qdrant-compatible REST front for the HBM-resident HIP index.

The reference's embedding, orchestrator and reporting services share a Qdrant server
(qdrant_store.py:78; docker-compose ``vectorstore``).  A GPU index lives inside one process, so
when the services run as separate processes ``python -m copilot_for_consensus_amd.services.main
vectorstore`` owns the :class:`~copilot_for_consensus_amd.vectorstore.HipFlatIndex` (or IVF) and
serves the subset of Qdrant's REST API the reference's driver uses -- the same URLs and JSON, so
``VECTOR_STORE_TYPE=qdrant`` (vectorstore/remote.py, or the reference's qdrant-client) pointed at
this server runs its searches on the MI355X:

  GET/PUT/DELETE /collections/{name}            (vectors.size, vectors.distance Cosine | Euclid | Dot)
  PUT  /collections/{name}/points               upsert {"points": [{"id", "vector", "payload"}]}
  POST /collections/{name}/points/search        {"vector", "limit", "with_payload", "with_vector", "score_threshold"}
  POST /collections/{name}/points/search/batch  {"searches": [...]}   (one fused kNN launch per 16 queries)
  POST /collections/{name}/points/query         {"query", "limit", ...} -> {"points": [...]}  (query_points :371)
  POST /collections/{name}/points/delete        {"points": [ids]}
  POST /collections/{name}/points/count         -> {"count"}
  GET  /collections/{name}/points/{id}
  POST /collections/{name}/points               retrieve {"ids", "with_vector", "with_payload"} (missing ids skipped)
  GET  /collections, /healthz, /readyz

Scores follow Qdrant: cosine similarity / dot product (descending), Euclid = distance (ascending).
Collections persist as the index's safetensors + JSON sidecar (``--persist-dir``) at shutdown and
on ``POST /collections/{name}/snapshots``.
"""
from __future__ import annotations

import contextlib
import math
import re
import threading
import time
from pathlib import Path
from typing import Any

from fastapi import Body, FastAPI
from fastapi.responses import JSONResponse

_DIST = {"cosine": "cosine", "euclid": "l2", "dot": "dot"}


# Qdrant's own rule for collection names; anything else (e.g. "..", "a/b", "%2E%2E") would name a
# directory outside the persist root once it reaches save() / rmtree()
_VALID_NAME = re.compile(r"^[A-Za-z0-9_-]{1,255}$")


def _ok(result: Any, t0: float) -> dict:
    return {"result": result, "status": "ok", "time": time.perf_counter() - t0}


def _err(code: int, msg: str) -> JSONResponse:
    return JSONResponse({"status": {"error": msg}, "result": None}, status_code=code)


class _Collection:
    def __init__(self, name: str, size: int, distance: str, device: str, capacity: int, index_type: str,
                 nlist: int, nprobe: int):
        from . import HipFlatIndex, HipIVFIndex
        self.name, self.size, self.distance = name, int(size), distance
        metric = _DIST[distance.lower()]
        if index_type == "ivf":
            self.index = HipIVFIndex(self.size, metric, nlist=nlist, nprobe=nprobe, capacity=capacity, device=device)
        else:
            self.index = HipFlatIndex(self.size, metric, capacity=capacity, device=device)

    def info(self) -> dict:
        return {"status": "green", "points_count": self.index.count(), "vectors_count": self.index.count(),
                "indexed_vectors_count": self.index.count(),
                "config": {"params": {"vectors": {"size": self.size, "distance": self.distance}}}}

    def score(self, s: float) -> float:
        return math.sqrt(max(0.0, s)) if self.distance.lower() == "euclid" else s


def create_vector_app(device: str = "cuda", capacity: int = 1 << 20, index_type: str = "flat", nlist: int = 0,
                      nprobe: int = 8, persist_dir: str | None = None) -> FastAPI:
    @contextlib.asynccontextmanager
    async def lifespan(_app):
        yield
        _app.state.save_all()      # persist every collection at shutdown

    app = FastAPI(title="copilot-for-consensus HIP vector store (Qdrant REST subset)", lifespan=lifespan)
    cols: dict[str, _Collection] = {}
    lock = threading.RLock()
    persist = Path(persist_dir) if persist_dir else None
    app.state.collections = cols

    def load_persisted() -> None:
        if not persist or not persist.exists():
            return
        import json

        from . import HipFlatIndex
        for d in sorted(p for p in persist.iterdir() if (p / "collection.json").exists()):
            meta = json.loads((d / "collection.json").read_text())
            if not _VALID_NAME.match(str(meta.get("name", ""))) or meta["name"] != d.name:
                continue   # a hand-edited or foreign directory: never let it name a path
            c = _Collection(meta["name"], meta["size"], meta["distance"], device, 1024, "flat", 0, 8)
            if (d / "index.json").exists():
                c.index = HipFlatIndex.load(d, device=device)
            cols[meta["name"]] = c

    def save(c: _Collection) -> None:
        if not persist:
            return
        import json
        d = coll_dir(c.name)
        c.index.save(d)
        (d / "collection.json").write_text(json.dumps({"name": c.name, "size": c.size, "distance": c.distance}))

    load_persisted()
    app.state.save_all = lambda: [save(c) for c in list(cols.values())]

    def coll_dir(name: str) -> Path:
        """persist/<name>, refused unless it resolves to a direct child of the persist root."""
        d = (persist / name).resolve()
        if not _VALID_NAME.match(name) or d.parent != persist.resolve():
            raise ValueError(f"invalid collection name {name!r}")
        return d

    @app.middleware("http")
    async def reject_bad_names(request, call_next):
        parts = request.url.path.split("/")
        if len(parts) >= 3 and parts[1] == "collections" and parts[2] and not _VALID_NAME.match(parts[2]):
            return _err(400, f"invalid collection name {parts[2]!r}: expected [A-Za-z0-9_-]{{1,255}}")
        return await call_next(request)

    def get(name: str) -> _Collection | None:
        with lock:
            return cols.get(name)

    def point(c: _Collection, r, with_payload=True, with_vector=False) -> dict:
        payload = dict(r.metadata) if with_payload else None
        pid = payload.pop("_qdrant_id", r.id) if payload is not None else r.metadata.get("_qdrant_id", r.id)
        out = {"id": pid, "version": 0, "score": c.score(r.score), "payload": payload}
        out["vector"] = list(r.vector) if with_vector else None
        return out

    def search(c: _Collection, queries: list[dict]) -> list[list[dict]]:
        vecs = [q.get("vector") if isinstance(q.get("vector"), list) else (q.get("vector") or {}).get("vector")
                for q in queries]
        if any(v is None or len(v) != c.size for v in vecs):
            raise ValueError(f"query vectors must have dimension {c.size}")
        k = max(int(q.get("limit", 10)) + int(q.get("offset", 0)) for q in queries)
        need_vec = any(q.get("with_vector") for q in queries)
        res = c.index.query_batch(vecs, k, with_vectors=need_vec) if hasattr(c.index, "query_batch") else \
            [c.index.query(v, k) for v in vecs]
        out = []
        for q, rs in zip(queries, res):
            rs = rs[int(q.get("offset", 0)):int(q.get("offset", 0)) + int(q.get("limit", 10))]
            pts = [point(c, r, q.get("with_payload", False) is not False, bool(q.get("with_vector"))) for r in rs]
            thr = q.get("score_threshold")
            if thr is not None:
                asc = c.distance.lower() == "euclid"
                pts = [p for p in pts if (p["score"] <= thr if asc else p["score"] >= thr)]
            out.append(pts)
        return out

    @app.get("/healthz")
    @app.get("/readyz")
    def health():
        return {"title": "cfc-vectorstore", "status": "ok"}

    @app.get("/collections")
    def list_collections():
        t0 = time.perf_counter()
        with lock:
            return _ok({"collections": [{"name": n} for n in cols]}, t0)

    @app.get("/collections/{name}")
    def collection_info(name: str):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        return _ok(c.info(), t0)

    @app.put("/collections/{name}")
    def create_collection(name: str, body: dict = Body(...)):
        t0 = time.perf_counter()
        vec = body.get("vectors") or {}
        size, dist = vec.get("size"), str(vec.get("distance", "Cosine"))
        if not isinstance(size, int) or size <= 0 or dist.lower() not in _DIST:
            return _err(400, "vectors.size must be a positive int and distance one of Cosine, Euclid, Dot")
        if not _VALID_NAME.match(name):
            return _err(400, f"invalid collection name {name!r}: expected [A-Za-z0-9_-]{{1,255}}")
        with lock:
            if name in cols:
                return _err(409, f"Collection `{name}` already exists!")
            cols[name] = _Collection(name, size, dist.capitalize(), device, capacity, index_type, nlist, nprobe)
        return _ok(True, t0)

    @app.delete("/collections/{name}")
    def delete_collection(name: str):
        t0 = time.perf_counter()
        with lock:
            found = cols.pop(name, None) is not None
        if found and persist and coll_dir(name).exists():
            import shutil
            shutil.rmtree(coll_dir(name), ignore_errors=True)
        return _ok(found, t0)

    @app.put("/collections/{name}/points")
    def upsert(name: str, body: dict = Body(...), wait: bool = True):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        pts = body.get("points")
        if isinstance(pts, dict):                       # batch form {"ids", "vectors", "payloads"}
            pts = [{"id": i, "vector": v, "payload": p} for i, v, p in
                   zip(pts["ids"], pts["vectors"], pts.get("payloads") or [{}] * len(pts["ids"]))]
        if not isinstance(pts, list) or any(len(p.get("vector") or []) != c.size for p in pts):
            return _err(400, f"every point needs a vector of dimension {c.size}")
        ids = [str(p["id"]) for p in pts]
        metas = [{**(p.get("payload") or {}), "_qdrant_id": p["id"]} for p in pts]
        c.index.add_embeddings(ids, [p["vector"] for p in pts], metas)
        return _ok({"operation_id": 0, "status": "completed"}, t0)

    @app.post("/collections/{name}/points")
    def retrieve_points(name: str, body: dict = Body(...)):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        out = []
        for pid in body.get("ids") or []:
            try:
                r = c.index.get(str(pid))
            except KeyError:
                continue
            out.append(point(c, r, bool(body.get("with_payload", True)), bool(body.get("with_vector", False))))
        return _ok(out, t0)

    @app.post("/collections/{name}/points/search")
    def search_points(name: str, body: dict = Body(...)):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        try:
            return _ok(search(c, [body])[0], t0)
        except ValueError as e:
            return _err(400, str(e))

    @app.post("/collections/{name}/points/search/batch")
    def search_batch(name: str, body: dict = Body(...)):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        try:
            return _ok(search(c, list(body.get("searches") or [])), t0)
        except ValueError as e:
            return _err(400, str(e))

    @app.post("/collections/{name}/points/query")
    def query_points(name: str, body: dict = Body(...)):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        q = dict(body)
        q["vector"] = q.pop("query", None)
        try:
            return _ok({"points": search(c, [q])[0]}, t0)
        except ValueError as e:
            return _err(400, str(e))

    @app.post("/collections/{name}/points/delete")
    def delete_points(name: str, body: dict = Body(...), wait: bool = True):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        for pid in body.get("points") or []:
            try:
                c.index.delete(str(pid))
            except KeyError:
                pass                                    # Qdrant: deleting an absent point is not an error
        return _ok({"operation_id": 0, "status": "completed"}, t0)

    @app.post("/collections/{name}/points/count")
    def count_points(name: str, body: dict = Body(default={})):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        return _ok({"count": c.index.count()}, t0)

    @app.get("/collections/{name}/points/{pid}")
    def get_point(name: str, pid: str):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        try:
            r = c.index.get(pid)
        except KeyError:
            return _err(404, f"No point with id {pid} found")
        return _ok(point(c, r, True, True), t0)

    @app.post("/collections/{name}/snapshots")
    def snapshot(name: str):
        t0 = time.perf_counter()
        c = get(name)
        if c is None:
            return _err(404, f"Collection `{name}` doesn't exist!")
        save(c)
        return _ok({"name": name, "persisted": bool(persist)}, t0)

    return app
