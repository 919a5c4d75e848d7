"""Networked document store: the MongoDB role for one-process-per-service deployments.

The reference's services share MongoDB (mongo_document_store.py:33; docker-compose.infra.yml
``documentdb``).  When the services of this framework run as separate processes on a node without
MongoDB, ``python -m copilot_for_consensus_amd.services.main docstore`` serves the in-memory store
(Mongo query operators, hash indexes, $lookup / $group aggregation -- storage/document_store.py)
over TCP, and :class:`RemoteDocumentStore` (``DOCUMENT_STORE_TYPE=cfcstore``) is the client.

Durability: every mutating call is appended to a write-ahead log (JSON lines, optional fsync)
after it is applied and before it is acknowledged; a snapshot of all collections replaces the log
every ``snapshot_every`` writes and at shutdown.  Start-up = snapshot + log replay, so the
pipeline's status fields and deterministic ids survive a restart of the store.

Wire format: u32 big-endian length + UTF-8 JSON, request ``{"id", "op", "args", "kwargs"}``,
reply ``{"id", "ok", "result"}`` or ``{"id", "ok": false, "error": <class>, "message"}``.
"""
from __future__ import annotations

import json
import os
import select
import socket
import socketserver
import struct
import threading
import uuid
from pathlib import Path
from typing import Any

from .document_store import (DocumentAlreadyExistsError, DocumentNotFoundError, DocumentStore,
                             DocumentStoreConnectionError, DocumentStoreError, DocumentStoreNotConnectedError,
                             InMemoryDocumentStore)

READ_OPS = {"get_document", "query_documents", "count_documents", "aggregate_documents", "ping", "collections"}
WRITE_OPS = {"insert_document", "insert_many", "update_document", "update_many", "delete_document", "delete_many",
             "clear_collection"}
_ERRORS = {c.__name__: c for c in (DocumentAlreadyExistsError, DocumentNotFoundError, DocumentStoreError,
                                    DocumentStoreConnectionError, DocumentStoreNotConnectedError)}
MAX_FRAME = 256 << 20


def _send(sock: socket.socket, obj: Any) -> None:
    b = json.dumps(obj, default=str).encode()
    sock.sendall(struct.pack(">I", len(b)) + b)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket) -> Any:
    (n,) = struct.unpack(">I", _recv_exact(sock, 4))
    if n > MAX_FRAME:
        raise ConnectionError(f"frame of {n} bytes exceeds the limit")
    return json.loads(_recv_exact(sock, n))


class DocumentStoreServer:
    def __init__(self, store: InMemoryDocumentStore | None = None, host: str = "0.0.0.0", port: int = 27027,
                 data_dir: str | os.PathLike | None = None, fsync: bool = False, snapshot_every: int = 50_000,
                 read_only: bool = False):
        """``read_only``: refuse every write (a view of another component's store, e.g. the chunk
        texts the DP node's owner ranks read: parallel/dp_node.py)."""
        self.read_only = bool(read_only)
        self.store = store or InMemoryDocumentStore()
        self.store.connect()
        self.data_dir = Path(data_dir) if data_dir else None
        self.fsync, self.snapshot_every = fsync, int(snapshot_every)
        self._wlock = threading.Lock()           # orders applied writes == log order
        self._wal = None
        self._writes_since_snapshot = 0
        self.replayed = 0
        if self.data_dir:
            self.data_dir.mkdir(parents=True, exist_ok=True)
            self._load()
            self._wal = open(self.data_dir / "wal.jsonl", "a", encoding="utf-8")
        outer = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                sock = self.request
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                while True:
                    try:
                        req = _recv(sock)
                    except (ConnectionError, OSError, ValueError):
                        return
                    _send(sock, outer.dispatch(req))

        class Server(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self.server = Server((host, port), Handler)
        self.port = self.server.server_address[1]
        self._thread: threading.Thread | None = None

    # ------------------------------------------------------------------ persistence
    def _load(self) -> None:
        snap = self.data_dir / "snapshot.json"
        if snap.exists():
            data = json.loads(snap.read_text(encoding="utf-8"))
            for coll, docs in data.get("collections", {}).items():
                for d in docs:
                    self.store.insert_document(coll, d)
        wal = self.data_dir / "wal.jsonl"
        if wal.exists():
            good = 0
            with open(wal, "rb") as fh:
                for line in fh:
                    try:
                        rec = json.loads(line)
                    except ValueError:
                        break                          # torn last line from a crash: drop it
                    try:
                        getattr(self.store, rec["op"])(*rec.get("args", []), **rec.get("kwargs", {}))
                    except DocumentStoreError:
                        pass                           # replayed exactly as it failed the first time
                    good += len(line)
                    self.replayed += 1
            if good < wal.stat().st_size:
                with open(wal, "r+b") as fh:
                    fh.truncate(good)

    def snapshot(self) -> None:
        if not self.data_dir:
            return
        with self._wlock:
            with self.store._lock:
                data = {"collections": {c: list(docs.values()) for c, docs in self.store.collections.items()}}
            tmp = self.data_dir / "snapshot.json.tmp"
            with open(tmp, "w", encoding="utf-8") as fh:
                json.dump(data, fh, default=str)
                fh.flush()
                os.fsync(fh.fileno())
            os.replace(tmp, self.data_dir / "snapshot.json")
            self._wal.close()
            self._wal = open(self.data_dir / "wal.jsonl", "w", encoding="utf-8")
            self._writes_since_snapshot = 0

    # ------------------------------------------------------------------ requests
    def dispatch(self, req: dict) -> dict:
        rid, op = req.get("id"), req.get("op")
        args, kwargs = list(req.get("args") or []), dict(req.get("kwargs") or {})
        try:
            if op == "ping":
                return {"id": rid, "ok": True, "result": "pong"}
            if op == "collections":
                with self.store._lock:
                    return {"id": rid, "ok": True,
                            "result": {c: len(d) for c, d in self.store.collections.items()}}
            if op in READ_OPS:
                return {"id": rid, "ok": True, "result": getattr(self.store, op)(*args, **kwargs)}
            if op not in WRITE_OPS:
                raise DocumentStoreError(f"unknown operation {op!r}")
            if self.read_only:
                raise DocumentStoreError(f"{op}: this document store is served read-only")
            # ids are fixed here so the log replays to the same documents
            if op == "insert_document" and not args[1].get("_id"):
                args[1] = {**args[1], "_id": str(uuid.uuid4())}
            if op == "insert_many":
                args[1] = [d if d.get("_id") else {**d, "_id": str(uuid.uuid4())} for d in args[1]]
            with self._wlock:
                result = getattr(self.store, op)(*args, **kwargs)
                if self._wal is not None:
                    self._wal.write(json.dumps({"op": op, "args": args, "kwargs": kwargs}, default=str) + "\n")
                    self._wal.flush()
                    if self.fsync:
                        os.fsync(self._wal.fileno())
                    self._writes_since_snapshot += 1
            if self._wal is not None and self._writes_since_snapshot >= self.snapshot_every:
                self.snapshot()
            return {"id": rid, "ok": True, "result": result}
        except Exception as e:  # noqa: BLE001 -- every failure goes back to the caller as a typed error
            return {"id": rid, "ok": False, "error": type(e).__name__, "message": str(e)}

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "DocumentStoreServer":
        self._thread = threading.Thread(target=self.server.serve_forever, name="docstore-server", daemon=True)
        self._thread.start()
        return self

    def serve_forever(self) -> None:
        try:
            self.server.serve_forever()
        finally:
            self.close()

    def close(self) -> None:
        self.server.shutdown() if self._thread else None
        self.server.server_close()
        if self._wal is not None:
            self.snapshot()
            self._wal.close()
            self._wal = None


_NON_IDEMPOTENT_OPERATORS = ("$inc", "$push", "$addToSet", "$pop", "$pull", "$mul")


def _idempotent(op: str, args) -> bool:
    """A write that is safe to re-send after a lost reply: clear_collection, and updates whose
    patch only sets fields (plain values or $set / $unset) -- never $inc / $push & co."""
    if op == "clear_collection":
        return True
    if op not in ("update_document", "update_many"):
        return False
    patch = args[-1] if args else None
    return isinstance(patch, dict) and not any(k in _NON_IDEMPOTENT_OPERATORS for k in patch)


class RemoteDocumentStore(DocumentStore):
    """Client of :class:`DocumentStoreServer` (``DOCUMENT_STORE_TYPE=cfcstore``)."""

    def __init__(self, host: str = "documentdb", port: int = 27027, timeout: float = 30.0, **_):
        self.host, self.port, self.timeout = host, int(port), timeout
        self._sock: socket.socket | None = None
        self._lock = threading.Lock()
        self._ids = 0

    def connect(self) -> None:
        try:
            s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        except OSError as e:
            raise DocumentStoreConnectionError(f"cannot reach document store {self.host}:{self.port}: {e}") from e
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock = s
        self._call("ping")

    def disconnect(self) -> None:
        if self._sock is not None:
            self._sock.close()
            self._sock = None

    def _call(self, op: str, *args, **kwargs):
        with self._lock:
            for attempt in range(2):   # reconnect and retry once (a restarted store)
                try:
                    if self._sock is not None and select.select([self._sock], [], [], 0)[0]:
                        # readable while idle = the peer closed (restarted store): start over
                        self._sock.close()
                        self._sock = None
                    if self._sock is None:
                        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
                        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                        self._sock = s
                    self._ids += 1
                    _send(self._sock, {"id": self._ids, "op": op, "args": list(args), "kwargs": kwargs})
                    rep = _recv(self._sock)
                    break
                except (OSError, ConnectionError) as e:
                    if self._sock is not None:
                        self._sock.close()
                    self._sock = None
                    if attempt or (op in WRITE_OPS and not _idempotent(op, args)):
                        # an insert / delete / counter update may have been applied before the
                        # connection broke: surface the failure instead of applying it twice
                        raise DocumentStoreConnectionError(f"{op}: {e}") from e
        if not rep.get("ok"):
            raise _ERRORS.get(rep.get("error"), DocumentStoreError)(rep.get("message", "document store error"))
        return rep.get("result")

    def insert_document(self, collection, doc):
        return self._call("insert_document", collection, doc)

    def get_document(self, collection, doc_id):
        return self._call("get_document", collection, doc_id)

    def query_documents(self, collection, filter_dict=None, limit=100, sort_by=None, sort_order="desc", skip=0):
        return self._call("query_documents", collection, filter_dict or {}, limit=limit, sort_by=sort_by,
                          sort_order=sort_order, skip=skip)

    def update_document(self, collection, doc_id, patch):
        self._call("update_document", collection, doc_id, patch)

    def delete_document(self, collection, doc_id):
        self._call("delete_document", collection, doc_id)

    def insert_many(self, collection, docs, ignore_duplicates=True):
        return self._call("insert_many", collection, list(docs), ignore_duplicates=ignore_duplicates)

    def update_many(self, collection, filter_dict, patch):
        return self._call("update_many", collection, filter_dict, patch)

    def delete_many(self, collection, filter_dict):
        return self._call("delete_many", collection, filter_dict)

    def count_documents(self, collection, filter_dict=None):
        return self._call("count_documents", collection, filter_dict or {})

    def aggregate_documents(self, collection, pipeline):
        return self._call("aggregate_documents", collection, pipeline)

    def clear_collection(self, collection):
        self._call("clear_collection", collection)

    def collection_counts(self) -> dict[str, int]:
        return self._call("collections")
