"""Document storage: interface, in-memory store with indexes + Mongo operators, validating
decorator, MongoDB driver (optional, needs pymongo) and factory.

Interface = adapters/copilot_storage/copilot_storage/document_store.py:40-138 of the reference
(insert_document / get_document / query_documents(filter, limit, sort_by, sort_order) /
update_document / delete_document / aggregate_documents) plus batched ``insert_many`` /
``update_many`` so the pipeline's per-document hot loops become one call.
"""
from __future__ import annotations

import copy
import threading
import uuid
from abc import ABC, abstractmethod
from collections import defaultdict
from typing import Any

from .query import apply_update, get_path, matches, prepare_filter, simple_equality_keys

SYSTEM_FIELDS = ("_rid", "_self", "_etag", "_attachments", "_ts")


class DocumentStoreError(Exception):
    pass


class DocumentStoreNotConnectedError(DocumentStoreError):
    pass


class DocumentStoreConnectionError(DocumentStoreError):
    pass


class DocumentNotFoundError(DocumentStoreError):
    pass


class DocumentAlreadyExistsError(DocumentStoreError):
    pass


_ATOMS = (str, int, float, bool, type(None))


def _jcopy(o):
    """Deep copy of a JSON-like document (dicts, lists, scalars): ~6x faster than copy.deepcopy, which
    the in-memory store runs on every read and write (the node's services read thousands of chunk /
    message documents per batch).  Anything else (datetime, bytes, ObjectId-likes) falls back to
    copy.deepcopy."""
    t = type(o)
    if t is dict:
        return {k: (v if type(v) in _ATOMS else _jcopy(v)) for k, v in o.items()}
    if t is list:
        return [v if type(v) in _ATOMS else _jcopy(v) for v in o]
    if t in _ATOMS:
        return o
    return copy.deepcopy(o)


def sanitize_document(doc: dict) -> dict:
    for f in SYSTEM_FIELDS:
        doc.pop(f, None)
    return doc


class DocumentStore(ABC):
    def connect(self) -> None:
        pass

    def disconnect(self) -> None:
        pass

    @abstractmethod
    def insert_document(self, collection: str, doc: dict[str, Any]) -> str: ...

    @abstractmethod
    def get_document(self, collection: str, doc_id: str) -> dict[str, Any] | None: ...

    @abstractmethod
    def query_documents(self, collection: str, filter_dict: dict[str, Any], limit: int = 100,
                        sort_by: str | None = None, sort_order: str = "desc", skip: int = 0) -> list[dict]: ...

    @abstractmethod
    def update_document(self, collection: str, doc_id: str, patch: dict[str, Any]) -> None: ...

    @abstractmethod
    def delete_document(self, collection: str, doc_id: str) -> None: ...

    # ---- batched helpers (default: loop) ----
    def insert_many(self, collection: str, docs: list[dict], ignore_duplicates: bool = True) -> list[str]:
        ids = []
        for d in docs:
            try:
                ids.append(self.insert_document(collection, d))
            except DocumentAlreadyExistsError:
                if not ignore_duplicates:
                    raise
        return ids

    def update_many(self, collection: str, filter_dict: dict, patch: dict) -> int:
        n = 0
        for d in self.query_documents(collection, filter_dict, limit=1 << 62):
            self.update_document(collection, d["_id"], patch)
            n += 1
        return n

    def delete_many(self, collection: str, filter_dict: dict) -> int:
        n = 0
        for d in self.query_documents(collection, filter_dict, limit=1 << 62):
            self.delete_document(collection, d["_id"])
            n += 1
        return n

    def count_documents(self, collection: str, filter_dict: dict | None = None) -> int:
        return len(self.query_documents(collection, filter_dict or {}, limit=1 << 62))

    def aggregate_documents(self, collection: str, pipeline: list[dict]) -> list[dict]:
        raise NotImplementedError


# Fields indexed in every collection (hash index: value -> set(ids)); mirrors the reference's
# collections.config.json indexes that the pipeline actually filters on.
DEFAULT_INDEXES = {
    "messages": ("archive_id", "thread_id", "message_id"),
    "chunks": ("thread_id", "message_doc_id", "embedding_generated", "archive_id"),
    "threads": ("archive_id", "summary_id"),
    "archives": ("source", "status", "file_hash"),
    "summaries": ("thread_id",),
    "sources": ("name",),
}


_ABSENT = ("__absent__",)


def _hashable(v):
    if isinstance(v, list):
        return None
    try:
        hash(v)
        return v
    except TypeError:
        return None


class InMemoryDocumentStore(DocumentStore):
    """Thread-safe in-memory store with hash indexes and Mongo query operators."""

    def __init__(self, indexes: dict[str, tuple[str, ...]] | None = None, **_):
        self._lock = threading.RLock()
        self.collections: dict[str, dict[str, dict]] = defaultdict(dict)
        self._index_fields = dict(DEFAULT_INDEXES if indexes is None else indexes)
        self._idx: dict[tuple[str, str], dict[Any, set]] = defaultdict(lambda: defaultdict(set))
        self._overflow: dict[tuple[str, str], set] = defaultdict(set)
        # insertion sequence per document: index-narrowed scans return documents in insertion
        # ("natural") order, as a full scan and MongoDB do
        self._seq: dict[tuple[str, str], int] = {}
        self._next_seq = 0
        self.connected = False

    @classmethod
    def from_config(cls, _cfg=None):
        return cls()

    def connect(self) -> None:
        self.connected = True

    def disconnect(self) -> None:
        self.connected = False

    # ---------------------------------------------------------------- index maintenance
    # Multikey hash index like Mongo's: a scalar is indexed under itself, an array under each of
    # its elements, an absent field under ``_ABSENT`` (an equality-to-None query matches both null
    # and absent).  Values that cannot be hashed go to a per-field overflow set that every lookup
    # on that field includes, so the index only ever narrows the scan, never changes its result.
    def _index_keys(self, doc, f):
        if f not in doc:
            return [_ABSENT], True
        v = doc[f]
        vals = v if isinstance(v, list) else [v]
        keys = [_hashable(x) for x in vals]
        ok = all(k is not None or x is None for k, x in zip(keys, vals))
        return keys, ok

    def _index_add(self, coll, doc):
        for f in self._index_fields.get(coll, ()):
            keys, ok = self._index_keys(doc, f)
            idx = self._idx[(coll, f)]
            for k in keys:
                idx[k].add(doc["_id"])
            if not ok or isinstance(doc.get(f), list):
                self._overflow[(coll, f)].add(doc["_id"])

    def _index_remove(self, coll, doc):
        for f in self._index_fields.get(coll, ()):
            keys, _ = self._index_keys(doc, f)
            idx = self._idx[(coll, f)]
            for k in keys:
                idx.get(k, set()).discard(doc["_id"])
            self._overflow[(coll, f)].discard(doc["_id"])

    def _lookup(self, coll, f, val):
        idx = self._idx[(coll, f)]
        hv = _hashable(val)
        if hv is None and val is not None:
            return None  # unhashable query value: no index answer, scan
        ids = set(idx.get(hv, ()))
        if val is None:
            ids |= idx.get(_ABSENT, set())
        return ids

    def _candidates(self, coll, flt):
        best = None
        for f, (kind, val) in simple_equality_keys(flt).items():
            if f == "_id":
                try:
                    ids = set(val) if kind == "in" else {val}
                except TypeError:
                    continue
            elif f in self._index_fields.get(coll, ()):
                ids = set()
                for v in (val if kind == "in" else [val]):
                    got = self._lookup(coll, f, v)
                    if got is None:
                        ids = None
                        break
                    ids |= got
                if ids is None:
                    continue
                # arrays / unhashable values may match in ways a hash lookup cannot see
                # (element of a list-valued query, nested dicts): always re-check those docs
                ids |= self._overflow[(coll, f)]
            else:
                continue
            if best is None or len(ids) < len(best):
                best = ids
        return best

    # ---------------------------------------------------------------- API
    def insert_document(self, collection: str, doc: dict[str, Any]) -> str:
        with self._lock:
            doc_id = doc.get("_id") or str(uuid.uuid4())
            coll = self.collections[collection]
            if doc_id in coll:
                raise DocumentAlreadyExistsError(f"Document with id {doc_id} already exists in {collection}")
            d = _jcopy(doc)
            d["_id"] = doc_id
            coll[doc_id] = d
            self._seq[(collection, doc_id)] = self._next_seq
            self._next_seq += 1
            self._index_add(collection, d)
            return doc_id

    def get_document(self, collection: str, doc_id: str) -> dict[str, Any] | None:
        with self._lock:
            d = self.collections[collection].get(doc_id)
            return sanitize_document(_jcopy(d)) if d is not None else None

    def _select(self, collection, filter_dict):
        filter_dict = prepare_filter(filter_dict)
        coll = self.collections[collection]
        cand = self._candidates(collection, filter_dict)
        if cand is not None:
            seq = self._seq
            it = (coll[i] for i in sorted((i for i in cand if i in coll), key=lambda i: seq.get((collection, i), 0)))
        else:
            it = coll.values()
        return [d for d in it if matches(d, filter_dict)]

    def query_documents(self, collection: str, filter_dict: dict[str, Any] | None = None, limit: int = 100,
                        sort_by: str | None = None, sort_order: str = "desc", skip: int = 0) -> list[dict]:
        if sort_order not in ("asc", "desc"):
            raise DocumentStoreError(f"Invalid sort_order {sort_order!r}")
        with self._lock:
            res = self._select(collection, filter_dict or {})
            if sort_by:
                # None sorts first in asc / last in desc (Cosmos/Mongo behaviour)
                def key(d):
                    v = get_path(d, sort_by)
                    return (0, "") if v is None or v is get_path({}, "x") else (1, v if isinstance(v, (int, float)) else str(v))
                try:
                    res.sort(key=key, reverse=sort_order == "desc")
                except TypeError:
                    res.sort(key=lambda d: str(get_path(d, sort_by)), reverse=sort_order == "desc")
            res = res[skip:skip + limit] if limit is not None else res[skip:]
            return [sanitize_document(_jcopy(d)) for d in res]

    def count_documents(self, collection: str, filter_dict: dict | None = None) -> int:
        with self._lock:
            return len(self._select(collection, filter_dict or {}))

    def update_document(self, collection: str, doc_id: str, patch: dict[str, Any]) -> None:
        with self._lock:
            d = self.collections[collection].get(doc_id)
            if d is None:
                raise DocumentNotFoundError(f"Document {doc_id} not found in collection {collection}")
            self._index_remove(collection, d)
            apply_update(d, _jcopy(patch))
            d["_id"] = doc_id
            self._index_add(collection, d)

    def update_many(self, collection: str, filter_dict: dict, patch: dict) -> int:
        with self._lock:
            docs = self._select(collection, filter_dict)
            for d in docs:
                self._index_remove(collection, d)
                apply_update(d, _jcopy(patch))
                self._index_add(collection, d)
            return len(docs)

    def delete_document(self, collection: str, doc_id: str) -> None:
        with self._lock:
            d = self.collections[collection].pop(doc_id, None)
            if d is None:
                raise DocumentNotFoundError(f"Document {doc_id} not found in collection {collection}")
            self._index_remove(collection, d)
            self._seq.pop((collection, doc_id), None)

    def delete_many(self, collection: str, filter_dict: dict) -> int:
        with self._lock:
            docs = self._select(collection, filter_dict)
            for d in docs:
                self.collections[collection].pop(d["_id"], None)
                self._index_remove(collection, d)
                self._seq.pop((collection, d["_id"]), None)
            return len(docs)

    def clear_collection(self, collection: str) -> None:
        with self._lock:
            self.collections[collection].clear()
            self._seq = {k: v for k, v in self._seq.items() if k[0] != collection}
            for k in [k for k in self._idx if k[0] == collection]:
                del self._idx[k]
            for k in [k for k in self._overflow if k[0] == collection]:
                del self._overflow[k]

    def clear_all(self) -> None:
        with self._lock:
            self.collections.clear()
            self._seq.clear()
            self._idx.clear()
            self._overflow.clear()

    def aggregate_documents(self, collection: str, pipeline: list[dict]) -> list[dict]:
        """$match / $lookup / $project / $sort / $limit / $skip / $count / $group(count|sum)."""
        with self._lock:
            docs = [_jcopy(d) for d in self.collections[collection].values()]
            for stage in pipeline:
                (op, spec), = stage.items()
                if op == "$match":
                    docs = [d for d in docs if matches(d, spec)]
                elif op == "$lookup":
                    other = self.collections[spec["from"]].values()
                    for d in docs:
                        lv = get_path(d, spec["localField"])
                        d[spec["as"]] = [_jcopy(o) for o in other
                                         if (get_path(o, spec["foreignField"]) == lv) or
                                         (isinstance(lv, list) and get_path(o, spec["foreignField"]) in lv)]
                elif op == "$project":
                    inc = {k for k, v in spec.items() if v}
                    docs = [{k: d[k] for k in d if k in inc or (k == "_id" and spec.get("_id", 1))} for d in docs]
                elif op == "$sort":
                    for k, direction in reversed(list(spec.items())):
                        docs.sort(key=lambda d: (get_path(d, k) is None, str(get_path(d, k))), reverse=direction < 0)
                elif op == "$limit":
                    docs = docs[:spec]
                elif op == "$skip":
                    docs = docs[spec:]
                elif op == "$count":
                    docs = [{spec: len(docs)}]
                elif op == "$group":
                    key = spec["_id"]
                    groups: dict = {}
                    for d in docs:
                        gk = get_path(d, key[1:]) if isinstance(key, str) and key.startswith("$") else key
                        g = groups.setdefault(_hashable(gk), {"_id": gk})
                        for name, acc in spec.items():
                            if name == "_id":
                                continue
                            (aop, aarg), = acc.items()
                            if aop == "$sum":
                                inc = aarg if isinstance(aarg, (int, float)) else (get_path(d, aarg[1:]) or 0)
                                g[name] = g.get(name, 0) + inc
                            elif aop == "$max":
                                v = get_path(d, aarg[1:])
                                g[name] = v if name not in g else max(g[name], v)
                            elif aop == "$min":
                                v = get_path(d, aarg[1:])
                                g[name] = v if name not in g else min(g[name], v)
                    docs = list(groups.values())
                else:
                    raise DocumentStoreError(f"unsupported aggregation stage {op}")
            return [sanitize_document(d) for d in docs]


class ValidatingDocumentStore(DocumentStore):
    """Validates inserted documents against the collection schema (reference
    validating_document_store.py:35); strict mode raises, lenient mode records errors."""

    def __init__(self, store: DocumentStore, schema_provider=None, strict: bool = True):
        from ..contracts.registry import default_provider
        self._inner = store
        self._schemas = schema_provider or default_provider()
        self.strict = strict
        self.validation_errors: list[tuple[str, list[str]]] = []
        self.skipped = 0

    def _check(self, collection, doc):
        errs = self._schemas.validate_document(collection, doc)
        if errs:
            self.validation_errors.append((collection, errs))
            if self.strict:
                raise DocumentStoreError(f"{collection} document failed validation: {'; '.join(errs[:5])}")

    def insert_document(self, collection, doc):
        self._check(collection, doc)
        return self._inner.insert_document(collection, doc)

    def insert_many(self, collection, docs, ignore_duplicates=True):
        """Batch insert.  In strict mode an invalid document is skipped (and recorded in
        ``validation_errors`` / counted in ``skipped``) while the rest of the batch is stored --
        the reference's per-message loop that logs a validation error and continues
        (parsing/app/service.py _store_messages); one malformed message must not fail the archive."""
        ok = []
        for d in docs:
            errs = self._schemas.validate_document(collection, d)
            if errs:
                self.validation_errors.append((collection, errs))
                if self.strict:
                    self.skipped += 1
                    continue
            ok.append(d)
        return self._inner.insert_many(collection, ok, ignore_duplicates)

    def get_document(self, collection, doc_id):
        return self._inner.get_document(collection, doc_id)

    def query_documents(self, collection, filter_dict=None, limit=100, sort_by=None, sort_order="desc", skip=0):
        return self._inner.query_documents(collection, filter_dict or {}, limit, sort_by, sort_order, skip)

    def update_document(self, collection, doc_id, patch):
        """Strict mode validates the document as it WILL be after the update (store metadata
        fields such as Cosmos' ``_etag`` / ``_ts`` ignored), reference validating_document_store.py."""
        if self.strict:
            cur = self._inner.get_document(collection, doc_id)
            if cur is None:
                raise DocumentNotFoundError(f"Document {doc_id} not found in collection {collection}")
            after = sanitize_document(_jcopy(cur))
            apply_update(after, _jcopy(patch))
            after["_id"] = doc_id
            self._check(collection, after)
        return self._inner.update_document(collection, doc_id, patch)

    def update_many(self, collection, filter_dict, patch):
        return self._inner.update_many(collection, filter_dict, patch)

    def delete_document(self, collection, doc_id):
        return self._inner.delete_document(collection, doc_id)

    def delete_many(self, collection, filter_dict):
        return self._inner.delete_many(collection, filter_dict)

    def count_documents(self, collection, filter_dict=None):
        return self._inner.count_documents(collection, filter_dict)

    def aggregate_documents(self, collection, pipeline):
        return self._inner.aggregate_documents(collection, pipeline)

    def connect(self):
        self._inner.connect()

    def disconnect(self):
        self._inner.disconnect()

    def __getattr__(self, name):
        return getattr(self._inner, name)


class MongoDocumentStore(DocumentStore):
    """MongoDB driver (reference mongo_document_store.py:33-452); needs ``pymongo``.

    Same contract as the reference's driver: ``connect`` pings the server and authenticates
    against ``admin`` unless ``authSource`` is given, failures raise DocumentStoreConnectionError;
    ids that parse as ObjectIds are matched as ObjectIds and every ``_id`` (nested ones in
    aggregation results too) comes back as a string; results are sanitised of backend fields;
    ``sort_order`` must be asc / desc; driver errors surface as DocumentStoreError.  The batched
    helpers run as single server-side operations (insert_many unordered, update_many, delete_many,
    count_documents) instead of the base class's per-document loops."""

    def __init__(self, host="documentdb", port=27017, database="copilot", username=None, password=None,
                 ensure_indexes=True, client_options: dict | None = None, **_):
        if not host:
            raise ValueError("MongoDB host is required")
        if not port:
            raise ValueError("MongoDB port is required")
        if not database:
            raise ValueError("MongoDB database is required")
        try:
            import pymongo  # type: ignore
        except ImportError as e:  # pragma: no cover
            raise ImportError("DOCUMENT_STORE_TYPE=mongodb needs 'pymongo'; use 'cfcstore' (native store server) "
                              "or 'inmemory'") from e
        self._pymongo = pymongo
        self.host, self.port, self.username, self.password = host, int(port), username, password
        self.client_options = dict(client_options or {})
        self._dbname = database
        self.ensure_indexes = ensure_indexes
        self.client = self.db = None

    def connect(self):
        params: dict[str, Any] = {"host": self.host, "port": self.port}
        if self.username and self.password:
            params.update(username=self.username, password=self.password)
            params.setdefault("authSource", self.client_options.get("authSource", "admin"))
        params.update(self.client_options)
        try:
            self.client = self._pymongo.MongoClient(**params)
            self.client.admin.command("ping")
            self.db = self.client[self._dbname]
        except Exception as e:  # noqa: BLE001 -- ConnectionFailure, auth errors, DNS: one typed error
            self.client = self.db = None
            raise DocumentStoreConnectionError(f"cannot connect to MongoDB at {self.host}:{self.port}: {e}") from e
        if self.ensure_indexes:
            self.ensure_collections()

    def disconnect(self):
        if self.client is not None:
            self.client.close()
        self.client = self.db = None

    def ensure_collections(self, config: dict | None = None) -> int:
        """Create the collections and indexes of collections.config.json (what the reference's
        infra/init/mongo-init.js does at container start); idempotent.  Returns indexes ensured."""
        from ..contracts.documents import collections_config
        cfg = config or collections_config()
        existing = set(self.db.list_collection_names())
        n = 0
        for d in cfg.get("collections", []):
            if d["name"] not in existing:
                self.db.create_collection(d["name"])
            for spec in d.get("indexes", []):
                self.db[d["name"]].create_index(list(spec["keys"].items()), **spec.get("options", {}))
                n += 1
        return n

    # -- helpers ---------------------------------------------------------------------------------
    def _c(self, collection):
        if self.db is None:
            raise DocumentStoreNotConnectedError("not connected to MongoDB: call connect() first")
        return self.db[collection]

    def _oid_query(self, doc_id) -> dict:
        """{"_id": ObjectId(doc_id)} when doc_id is a valid ObjectId string, else the raw id."""
        try:
            from bson import ObjectId  # type: ignore  (ships with pymongo)
            if isinstance(doc_id, str) and ObjectId.is_valid(doc_id):
                return {"_id": ObjectId(doc_id)}
        except ImportError:
            pass
        return {"_id": doc_id}

    @classmethod
    def _stringify_ids(cls, obj):
        """ObjectId -> str, recursively (aggregation results carry nested ids from $lookup)."""
        if isinstance(obj, dict):
            for k, v in obj.items():
                obj[k] = cls._stringify_ids(v)
            return obj
        if isinstance(obj, list):
            return [cls._stringify_ids(v) for v in obj]
        if type(obj).__name__ == "ObjectId":
            return str(obj)
        return obj

    def _out(self, doc):
        if doc is None:
            return None
        if "_id" in doc:
            doc["_id"] = str(doc["_id"])
        return sanitize_document(doc)

    def _run(self, what: str, fn):
        try:
            return fn()
        except (DocumentStoreError, ValueError):
            raise
        except Exception as e:  # noqa: BLE001 -- pymongo OperationFailure / AutoReconnect / ...
            if isinstance(e, self._pymongo.errors.DuplicateKeyError):
                raise DocumentAlreadyExistsError(str(e)) from e
            raise DocumentStoreError(f"MongoDB {what} failed: {e}") from e

    # -- DocumentStore ---------------------------------------------------------------------------
    def insert_document(self, collection, doc):
        c = self._c(collection)
        return self._run("insert", lambda: str(c.insert_one(dict(doc)).inserted_id))

    def insert_many(self, collection, docs, ignore_duplicates: bool = True):
        c, docs = self._c(collection), [dict(d) for d in docs]
        if not docs:
            return []
        try:
            res = c.insert_many(docs, ordered=False)
            return [str(i) for i in res.inserted_ids]
        except self._pymongo.errors.BulkWriteError as e:
            errs = e.details.get("writeErrors", [])
            if any(w.get("code") != 11000 for w in errs):       # 11000 = duplicate key
                raise DocumentStoreError(f"MongoDB insert_many failed: {e}") from e
            if not ignore_duplicates:
                raise DocumentAlreadyExistsError(str(e)) from e
            failed = {w["index"] for w in errs}
            return [str(d["_id"]) for i, d in enumerate(docs) if i not in failed]

    def get_document(self, collection, doc_id):
        c = self._c(collection)
        return self._out(self._run("get", lambda: c.find_one(self._oid_query(doc_id))))

    def query_documents(self, collection, filter_dict=None, limit=100, sort_by=None, sort_order="desc", skip=0):
        if sort_order not in ("asc", "desc"):
            raise DocumentStoreError(f"Invalid sort_order {sort_order!r}: must be 'asc' or 'desc'")
        c = self._c(collection)

        def run():
            cur = c.find(filter_dict or {})
            if sort_by:
                cur = cur.sort(sort_by, self._pymongo.DESCENDING if sort_order == "desc" else self._pymongo.ASCENDING)
            if skip:
                cur = cur.skip(int(skip))
            if limit:
                cur = cur.limit(int(limit))
            return [self._out(d) for d in cur]
        return self._run("query", run)

    def count_documents(self, collection, filter_dict=None):
        c = self._c(collection)
        return int(self._run("count", lambda: c.count_documents(filter_dict or {})))

    def update_document(self, collection, doc_id, patch):
        c = self._c(collection)
        upd = patch if any(k.startswith("$") for k in patch) else {"$set": patch}
        if self._run("update", lambda: c.update_one(self._oid_query(doc_id), upd)).matched_count == 0:
            raise DocumentNotFoundError(f"document {doc_id} not found in {collection}")

    def update_many(self, collection, filter_dict, patch):
        c = self._c(collection)
        upd = patch if any(k.startswith("$") for k in patch) else {"$set": patch}
        return int(self._run("update_many", lambda: c.update_many(filter_dict, upd)).modified_count)

    def delete_document(self, collection, doc_id):
        c = self._c(collection)
        if self._run("delete", lambda: c.delete_one(self._oid_query(doc_id))).deleted_count == 0:
            raise DocumentNotFoundError(f"document {doc_id} not found in {collection}")

    def delete_many(self, collection, filter_dict):
        c = self._c(collection)
        return int(self._run("delete_many", lambda: c.delete_many(filter_dict)).deleted_count)

    def aggregate_documents(self, collection, pipeline):
        c = self._c(collection)
        docs = self._run("aggregate", lambda: list(c.aggregate(pipeline)))
        return [sanitize_document(self._stringify_ids(d)) for d in docs]


def create_document_store(cfg=None, enable_validation: bool = False, strict: bool = True) -> DocumentStore:
    name = str(getattr(cfg, "driver_name", cfg) or "inmemory").strip().lower()
    kw = dict(getattr(cfg, "driver_config", {}) or {})
    if name == "inmemory":
        store: DocumentStore = InMemoryDocumentStore()
    elif name == "mongodb":
        store = MongoDocumentStore(**kw)
    elif name == "cfcstore":
        from .server import RemoteDocumentStore
        store = RemoteDocumentStore(**{k: v for k, v in kw.items() if v is not None})
    elif name in ("azure_cosmosdb", "azurecosmos"):
        from ..cloud.azure import AzureCosmosDocumentStore
        store = AzureCosmosDocumentStore(**{k: v for k, v in kw.items() if v is not None})
    else:
        raise ValueError(f"unknown document_store driver {name!r}")
    return ValidatingDocumentStore(store, strict=strict) if enable_validation else store
