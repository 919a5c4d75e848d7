"""Host-side row table of an HBM vector index: ids and metadata without a Python object per row.

The reference keeps ids in Python / FAISS side maps (faiss_store.py:303-345: ``index.add`` plus an
``id_map`` dict and a ``metadata`` dict per vector).  At the scale the MI355X index holds (100M+
rows per GPU) per-row Python strings and dicts cost tens of GB of host memory and minutes to
permute.  Here every per-row field is a numpy column:

* ids and metadata are UTF-8 bytes in two append-only heaps; a row holds (offset, length) into
  each -- a regroup / compaction permutes 4 small integer columns, never the bytes;
* lookup id -> row is a 64-bit xxh3 hash: a sorted (hash, row) array searched with
  ``np.searchsorted`` plus a dict of the rows added since the last sort (re-merged when it grows);
  the stored id bytes are compared on every hit, so a hash collision can never return a wrong row;
* metadata is compact JSON per row (empty = no bytes at all), decoded only for rows a query returns;
* save / load are plain ``.npy`` files (no pickle).
"""
from __future__ import annotations

import json
from pathlib import Path

import hashlib

import numpy as np

try:
    import xxhash
except ImportError:  # optional: the standard library's blake2b gives the same 64-bit lookup key
    xxhash = None

_EMPTY = np.zeros(0, np.uint8)
# which 64-bit hash the "hash" column holds (saved with the table; a load under the other one rehashes)
HASH_NAME = "xxh3_64" if xxhash is not None else "blake2b_64"


def _hash(b: bytes) -> int:
    if xxhash is not None:
        return xxhash.xxh3_64_intdigest(b)
    return int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little")


class _Heap:
    """Append-only byte heap (amortised doubling)."""

    def __init__(self, cap: int = 1 << 16):
        self.buf = np.zeros(cap, np.uint8)
        self.n = 0

    def append(self, data: bytes) -> int:
        off = self.n
        need = off + len(data)
        if need > self.buf.size:
            nb = np.zeros(max(need, 2 * self.buf.size), np.uint8)
            nb[:off] = self.buf[:off]
            self.buf = nb
        self.buf[off:need] = np.frombuffer(data, np.uint8)
        self.n = need
        return off

    def get(self, off: int, ln: int) -> bytes:
        return self.buf[off:off + ln].tobytes()


class RowTable:
    MERGE_MIN = 1 << 16

    def __init__(self, capacity: int = 1024):
        self.n = 0
        self._ids, self._meta = _Heap(), _Heap()
        self._cols = {}
        self._grow(max(1, capacity))
        self._sorted_h = np.zeros(0, np.uint64)
        self._sorted_r = np.zeros(0, np.int64)
        self._recent: dict[int, list[int]] = {}
        self._nrecent = 0

    # ------------------------------------------------------------ columns
    def _grow(self, cap: int) -> None:
        spec = {"hash": np.uint64, "ioff": np.int64, "ilen": np.int32, "moff": np.int64, "mlen": np.int32,
                "live": np.bool_}
        old = self._cols
        self._cols = {}
        for k, dt in spec.items():
            a = np.zeros(cap, dt)
            if k in old:
                a[:self.n] = old[k][:self.n]
            self._cols[k] = a
        self.cap = cap

    def _reserve(self, n: int) -> None:
        if n > self.cap:
            self._grow(max(n, 2 * self.cap))

    @property
    def live(self) -> np.ndarray:
        return self._cols["live"][:self.n]

    # ------------------------------------------------------------ lookup
    def _candidates(self, h: int):
        i = int(np.searchsorted(self._sorted_h, np.uint64(h), side="left"))
        while i < self._sorted_h.size and int(self._sorted_h[i]) == h:
            yield int(self._sorted_r[i])
            i += 1
        yield from self._recent.get(h, ())

    def find(self, key: str) -> int:
        """Row of a live id, or -1."""
        b = key.encode("utf-8")
        c = self._cols
        for r in self._candidates(_hash(b)):
            if c["live"][r] and c["ilen"][r] == len(b) and self._ids.get(int(c["ioff"][r]), len(b)) == b:
                return r
        return -1

    def find_many(self, keys) -> np.ndarray:
        return np.fromiter((self.find(k) for k in keys), np.int64, len(keys))

    def _index(self, r: int, h: int) -> None:
        self._recent.setdefault(h, []).append(r)
        self._nrecent += 1

    def _maybe_merge(self) -> None:
        if self._nrecent > max(self.MERGE_MIN, self._sorted_h.size // 8):
            self.rebuild()

    def rebuild(self) -> None:
        """Re-sort the (hash, row) lookup over the live rows (after a permutation or many inserts)."""
        live = np.nonzero(self.live)[0]
        h = self._cols["hash"][live]
        o = np.argsort(h, kind="stable")
        self._sorted_h, self._sorted_r = h[o], live[o].astype(np.int64)
        self._recent = {}
        self._nrecent = 0

    # ------------------------------------------------------------ writes
    def upsert(self, keys, metas=None) -> np.ndarray:
        """Rows of ``keys``: existing live rows are reused (metadata replaced), new ids appended."""
        keys = list(keys)
        metas = list(metas) if metas is not None else [None] * len(keys)
        rows = np.empty(len(keys), np.int64)
        self._reserve(self.n + len(keys))
        c = self._cols
        for j, (k, m) in enumerate(zip(keys, metas)):
            r = self.find(k)
            if r < 0:
                b = k.encode("utf-8")
                r = self.n
                self.n += 1
                h = _hash(b)
                c["hash"][r] = h
                c["ioff"][r], c["ilen"][r] = self._ids.append(b), len(b)
                c["live"][r] = True
                self._index(r, h)
            self._set_meta(r, m)
            rows[j] = r
        self._maybe_merge()
        return rows

    def append_bulk(self, keys, metas=None) -> np.ndarray:
        """Fast path for a bulk build of NEW ids (no duplicate check against the table): one heap
        append and vectorised hashing bookkeeping.  Returns the new rows."""
        keys = list(keys)
        n0, k = self.n, len(keys)
        self._reserve(n0 + k)
        enc = [s.encode("utf-8") for s in keys]
        lens = np.fromiter((len(b) for b in enc), np.int32, k)
        base = self._ids.append(b"".join(enc))
        c = self._cols
        c["ioff"][n0:n0 + k] = base + np.concatenate(([0], np.cumsum(lens[:-1], dtype=np.int64))) if k else 0
        c["ilen"][n0:n0 + k] = lens
        c["hash"][n0:n0 + k] = np.fromiter((_hash(b) for b in enc), np.uint64, k)
        c["live"][n0:n0 + k] = True
        c["moff"][n0:n0 + k] = 0
        c["mlen"][n0:n0 + k] = 0
        self.n = n0 + k
        if metas is not None:
            for j, m in enumerate(metas):
                self._set_meta(n0 + j, m)
        self.rebuild()
        return np.arange(n0, n0 + k, dtype=np.int64)

    def _set_meta(self, r: int, m) -> None:
        c = self._cols
        if not m:
            c["moff"][r], c["mlen"][r] = 0, 0
            return
        b = json.dumps(m, separators=(",", ":"), sort_keys=True).encode("utf-8")
        c["moff"][r], c["mlen"][r] = self._meta.append(b), len(b)

    def kill(self, r: int) -> None:
        self._cols["live"][r] = False

    def permute(self, order: np.ndarray) -> None:
        """Row i becomes old row order[i] (a regroup); rows not in ``order`` are dropped."""
        order = np.asarray(order, np.int64)
        for k, a in self._cols.items():
            a[:order.size] = a[order]
        self.n = order.size
        self.rebuild()

    def clear(self) -> None:
        self.__init__(self.cap)

    # ------------------------------------------------------------ reads
    def id_at(self, r: int) -> str | None:
        c = self._cols
        if r < 0 or r >= self.n or not c["live"][r]:
            return None
        return self._ids.get(int(c["ioff"][r]), int(c["ilen"][r])).decode("utf-8")

    def meta_at(self, r: int) -> dict:
        c = self._cols
        ln = int(c["mlen"][r])
        return json.loads(self._meta.get(int(c["moff"][r]), ln)) if ln else {}

    def ids(self) -> list[str]:
        return [self.id_at(r) for r in range(self.n) if self._cols["live"][r]]

    # ------------------------------------------------------------ persistence
    def save(self, path) -> None:
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        for k, a in self._cols.items():
            np.save(p / f"rows_{k}.npy", a[:self.n])
        np.save(p / "rows_idheap.npy", self._ids.buf[:self._ids.n])
        np.save(p / "rows_metaheap.npy", self._meta.buf[:self._meta.n])
        (p / "rows_hash.txt").write_text(HASH_NAME)

    @classmethod
    def load(cls, path) -> "RowTable":
        p = Path(path)
        live = np.load(p / "rows_live.npy")
        t = cls(max(1, live.size))
        for k in t._cols:
            a = np.load(p / f"rows_{k}.npy")
            t._cols[k][:a.size] = a
        t.n = live.size
        for name, heap in (("idheap", t._ids), ("metaheap", t._meta)):
            b = np.load(p / f"rows_{name}.npy")
            heap.buf = np.concatenate([b, np.zeros(max(1024, b.size), np.uint8)])
            heap.n = b.size
        saved = (p / "rows_hash.txt").read_text().strip() if (p / "rows_hash.txt").exists() else "xxh3_64"
        if saved != HASH_NAME:
            # written under the other hash function (xxhash present there, absent here or vice versa)
            c = t._cols
            c["hash"][:t.n] = np.fromiter(
                (_hash(t._ids.get(int(c["ioff"][r]), int(c["ilen"][r]))) for r in range(t.n)), np.uint64, t.n)
        t.rebuild()
        return t
