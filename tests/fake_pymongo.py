"""A stand-in for ``pymongo`` + ``bson`` (absent from this image): an in-memory MongoDB server.

Covers the API surface the MongoDB document-store driver uses with MongoDB's semantics where the
driver depends on them: ObjectId ``_id`` assignment (written back into the caller's dict, as
pymongo does), unique indexes -> DuplicateKeyError (code 11000), unordered ``insert_many`` ->
BulkWriteError with per-index write errors, find / sort (missing and null lowest) / skip / limit
cursors, update / delete results with matched / modified / deleted counts, aggregation (delegated
to the framework's in-memory aggregation engine), ``ping``, authentication against a user table
and a server that can be taken down (``SERVER.up = False``: ConnectionFailure).
Filters and update operators use storage/query.py, the matcher the in-memory store runs.
"""
from __future__ import annotations

import copy
import itertools
import os
import threading
import types

from copilot_for_consensus_amd.storage.query import _MISSING, apply_update, get_path, matches

ASCENDING, DESCENDING = 1, -1


class _Errors:
    class PyMongoError(Exception):
        pass

    class ConnectionFailure(PyMongoError):
        pass

    class ServerSelectionTimeoutError(ConnectionFailure):
        pass

    class OperationFailure(PyMongoError):
        def __init__(self, msg, code=None, details=None):
            super().__init__(msg)
            self.code, self.details = code, details or {}

    class DuplicateKeyError(OperationFailure):
        pass

    class BulkWriteError(OperationFailure):
        pass


errors = types.SimpleNamespace(**{k: v for k, v in vars(_Errors).items() if not k.startswith("_")})

_counter = itertools.count(int.from_bytes(os.urandom(3), "big"))


class ObjectId:
    def __init__(self, oid=None):
        if oid is None:
            self._h = os.urandom(8).hex() + f"{next(_counter) & 0xFFFFFFFF:08x}"
        elif isinstance(oid, ObjectId):
            self._h = oid._h
        elif ObjectId.is_valid(oid):
            self._h = oid.lower()
        else:
            raise TypeError(f"{oid!r} is not a valid ObjectId")

    @staticmethod
    def is_valid(oid) -> bool:
        if isinstance(oid, ObjectId):
            return True
        return isinstance(oid, str) and len(oid) == 24 and all(c in "0123456789abcdefABCDEF" for c in oid)

    def __str__(self):
        return self._h

    def __repr__(self):
        return f"ObjectId('{self._h}')"

    def __eq__(self, other):
        return isinstance(other, ObjectId) and other._h == self._h

    def __lt__(self, other):
        return self._h < other._h

    def __hash__(self):
        return hash(("oid", self._h))


bson = types.ModuleType("bson")
bson.ObjectId = ObjectId


class _Server:
    def __init__(self):
        self.lock = threading.RLock()
        self.reset()

    def reset(self):
        with self.lock:
            self.dbs: dict[str, dict[str, _CollData]] = {}
            self.up = True
            self.users: dict[tuple[str, str], str] | None = None     # (user, password) -> authSource
            self.clients: list[dict] = []


class _CollData:
    def __init__(self):
        self.docs: dict = {}                       # _id -> doc, insertion ordered
        self.unique: list[str] = []


SERVER = _Server()


def _sort_key(v):
    """MongoDB order for the types the pipeline stores: missing/null < numbers < strings < others."""
    if v is _MISSING or v is None:
        return (0, 0)
    if isinstance(v, bool):
        return (3, v)
    if isinstance(v, (int, float)):
        return (1, v)
    if isinstance(v, str):
        return (2, v)
    return (4, str(v))


class Cursor:
    def __init__(self, docs):
        self._docs, self._skip, self._limit = docs, 0, 0

    def sort(self, key, direction=ASCENDING):
        self._docs.sort(key=lambda d: _sort_key(get_path(d, key)), reverse=direction == DESCENDING)
        return self

    def skip(self, n):
        self._skip = int(n)
        return self

    def limit(self, n):
        self._limit = int(n)
        return self

    def __iter__(self):
        out = self._docs[self._skip:]
        return iter(out[:self._limit] if self._limit else out)


class Collection:
    def __init__(self, db, name):
        self.db, self.name = db, name

    @property
    def _d(self) -> _CollData:
        with SERVER.lock:
            return self.db._data.setdefault(self.name, _CollData())

    def _check_unique(self, d: _CollData, doc, ignore_id=None):
        if doc["_id"] in d.docs and doc["_id"] != ignore_id:
            raise errors.DuplicateKeyError(f"E11000 duplicate key error collection: {self.name} _id", 11000)
        for f in d.unique:
            v = get_path(doc, f)
            if v is _MISSING:
                continue
            for other in d.docs.values():
                if other["_id"] != doc["_id"] and get_path(other, f) == v:
                    raise errors.DuplicateKeyError(f"E11000 duplicate key error collection: {self.name} {f}", 11000)

    def create_index(self, keys, unique=False, name=None, **_):
        with SERVER.lock:
            if unique:
                for f, _dir in keys:
                    if f not in self._d.unique:
                        self._d.unique.append(f)
        return name or "_".join(f"{f}_{d}" for f, d in keys)

    def insert_one(self, doc):
        with SERVER.lock:
            doc.setdefault("_id", ObjectId())
            d = self._d
            self._check_unique(d, doc)
            d.docs[doc["_id"]] = copy.deepcopy(doc)
        return types.SimpleNamespace(inserted_id=doc["_id"], acknowledged=True)

    def insert_many(self, docs, ordered=True):
        ids, errs = [], []
        for i, doc in enumerate(docs):
            try:
                ids.append(self.insert_one(doc).inserted_id)
            except errors.DuplicateKeyError as e:
                errs.append({"index": i, "code": 11000, "errmsg": str(e)})
                if ordered:
                    break
        if errs:
            raise errors.BulkWriteError("batch op errors occurred", 65,
                                        {"writeErrors": errs, "nInserted": len(ids)})
        return types.SimpleNamespace(inserted_ids=ids, acknowledged=True)

    def _select(self, flt):
        with SERVER.lock:
            return [d for d in self._d.docs.values() if matches(d, flt or {})]

    def find(self, filter=None, projection=None):                 # noqa: A002 -- pymongo's name
        return Cursor([copy.deepcopy(d) for d in self._select(filter)])

    def find_one(self, filter=None):                              # noqa: A002
        got = self._select(filter)
        return copy.deepcopy(got[0]) if got else None

    def count_documents(self, filter):                            # noqa: A002
        return len(self._select(filter))

    def _update(self, flt, upd, many):
        matched = modified = 0
        with SERVER.lock:
            d = self._d
            for doc in self._select(flt):
                matched += 1
                new = apply_update(copy.deepcopy(doc), upd)
                self._check_unique(d, new, ignore_id=doc["_id"])
                if new != doc:
                    d.docs[doc["_id"]] = new
                    modified += 1
                if not many:
                    break
        return types.SimpleNamespace(matched_count=matched, modified_count=modified, acknowledged=True)

    def update_one(self, filter, update):                         # noqa: A002
        return self._update(filter, update, False)

    def update_many(self, filter, update):                        # noqa: A002
        return self._update(filter, update, True)

    def _delete(self, flt, many):
        n = 0
        with SERVER.lock:
            for doc in self._select(flt):
                del self._d.docs[doc["_id"]]
                n += 1
                if not many:
                    break
        return types.SimpleNamespace(deleted_count=n, acknowledged=True)

    def delete_one(self, filter):                                 # noqa: A002
        return self._delete(filter, False)

    def delete_many(self, filter):                                # noqa: A002
        return self._delete(filter, True)

    def aggregate(self, pipeline):
        from copilot_for_consensus_amd.storage.document_store import InMemoryDocumentStore
        tmp = InMemoryDocumentStore()
        with SERVER.lock:
            for cname, cd in self.db._data.items():
                for doc in cd.docs.values():
                    tmp.insert_document(cname, copy.deepcopy(doc))
        return iter(tmp.aggregate_documents(self.name, pipeline))


class Database:
    def __init__(self, client, name):
        self.client, self.name = client, name
        with SERVER.lock:
            self._data = SERVER.dbs.setdefault(name, {})

    def __getitem__(self, name):
        return Collection(self, name)

    def list_collection_names(self):
        with SERVER.lock:
            return list(self._data)

    def create_collection(self, name):
        with SERVER.lock:
            if name in self._data:
                raise errors.OperationFailure(f"collection {name} already exists", 48)
            self._data[name] = _CollData()
        return Collection(self, name)

    def command(self, cmd):
        if not SERVER.up:
            raise errors.ServerSelectionTimeoutError("No servers found yet")
        if self.client._auth_error:
            raise errors.OperationFailure("Authentication failed.", 18)
        if cmd == "ping":
            return {"ok": 1.0}
        raise errors.OperationFailure(f"no such command: {cmd}", 59)


class MongoClient:
    def __init__(self, host="localhost", port=27017, username=None, password=None, authSource=None, **kw):
        self.kwargs = dict(host=host, port=port, username=username, password=password, authSource=authSource, **kw)
        SERVER.clients.append(self.kwargs)
        users = SERVER.users
        self._auth_error = users is not None and users.get((username, password)) != (authSource or "admin")
        self.closed = False

    @property
    def admin(self):
        return Database(self, "admin")

    def __getitem__(self, name):
        if not SERVER.up:
            raise errors.ServerSelectionTimeoutError("No servers found yet")
        return Database(self, name)

    def close(self):
        self.closed = True


def install(monkeypatch):
    """Make ``import pymongo`` / ``import bson`` resolve to this stand-in (fresh server)."""
    import sys
    SERVER.reset()
    mod = sys.modules[__name__]
    monkeypatch.setitem(sys.modules, "pymongo", mod)
    monkeypatch.setitem(sys.modules, "pymongo.errors", errors)
    monkeypatch.setitem(sys.modules, "bson", bson)
    return SERVER
