"""Mongo-style filter matching and update operators for the in-memory document store.

The reference's InMemoryDocumentStore supports only equality filters
(adapters/copilot_storage/copilot_storage/inmemory_document_store.py:132), so its services ship
shims for ``$in`` in tests.  This matcher implements the operators the pipeline and
the REST queries use: $eq $ne $gt $gte $lt $lte $in $nin $exists $regex $size $all $elemMatch
$not $and $or $nor, dotted paths, and Mongo's array semantics (a scalar condition on an array
field matches if ANY element matches).
"""
from __future__ import annotations

import re
from typing import Any

_MISSING = object()


def get_path(doc: Any, path: str) -> Any:
    cur = doc
    for part in path.split("."):
        if isinstance(cur, dict):
            cur = cur.get(part, _MISSING)
        elif isinstance(cur, list) and part.isdigit():
            i = int(part)
            cur = cur[i] if i < len(cur) else _MISSING
        else:
            return _MISSING
        if cur is _MISSING:
            return _MISSING
    return cur


def _cmp(a, b, op) -> bool:
    if a is _MISSING or a is None or b is None:
        return False
    try:
        if op == "$gt":
            return a > b
        if op == "$gte":
            return a >= b
        if op == "$lt":
            return a < b
        if op == "$lte":
            return a <= b
    except TypeError:
        return str(a) > str(b) if op == "$gt" else (str(a) >= str(b) if op == "$gte" else
                                                      (str(a) < str(b) if op == "$lt" else str(a) <= str(b)))
    raise ValueError(op)


_SCALARS = (str, int, float, bool, type(None))


class _InSet(frozenset):
    """A ``$in`` list of hashable scalars, pre-hashed once per query (prepare_filter): membership
    instead of a linear scan per document (an $in over 1,700 chunk ids against 1,700 candidates was
    millions of comparisons under the store lock)."""


def _in_set(v, arg: _InSet) -> bool:
    if v is _MISSING:
        return None in arg
    if isinstance(v, list):
        return any(type(x) in _SCALARS and x in arg for x in v)
    return type(v) in _SCALARS and v in arg


def prepare_filter(flt):
    """Same filter with every ``$in`` / ``$nin`` list of hashable scalars as a pre-hashed set; the
    result matches exactly the same documents (Mongo equality of scalars == Python hash equality)."""
    if isinstance(flt, dict):
        out = {}
        for k, v in flt.items():
            if k in ("$in", "$nin") and isinstance(v, (list, tuple)) and all(type(a) in _SCALARS for a in v):
                out[k] = _InSet(v)
            elif k in ("$and", "$or", "$nor") and isinstance(v, list):
                out[k] = [prepare_filter(c) for c in v]
            elif isinstance(v, dict):
                out[k] = prepare_filter(v)
            else:
                out[k] = v
        return out
    return flt


def _eq(v, target) -> bool:
    if v is _MISSING:
        return target is None
    if isinstance(v, list) and not isinstance(target, list):
        return target in v
    return v == target


def _match_ops(v, cond: dict) -> bool:
    for op, arg in cond.items():
        if op == "$eq":
            ok = _eq(v, arg)
        elif op == "$ne":
            ok = not _eq(v, arg)
        elif op in ("$gt", "$gte", "$lt", "$lte"):
            ok = any(_cmp(x, arg, op) for x in v) if isinstance(v, list) else _cmp(v, arg, op)
        elif op == "$in":
            ok = _in_set(v, arg) if isinstance(arg, _InSet) else any(_eq(v, a) for a in arg)
        elif op == "$nin":
            ok = not (_in_set(v, arg) if isinstance(arg, _InSet) else any(_eq(v, a) for a in arg))
        elif op == "$exists":
            ok = (v is not _MISSING) == bool(arg)
        elif op == "$regex":
            flags = re.IGNORECASE if "i" in cond.get("$options", "") else 0
            pat = re.compile(arg, flags)
            ok = (isinstance(v, str) and bool(pat.search(v))) or (
                isinstance(v, list) and any(isinstance(x, str) and pat.search(x) for x in v))
        elif op == "$options":
            ok = True
        elif op == "$size":
            ok = isinstance(v, list) and len(v) == arg
        elif op == "$all":
            ok = isinstance(v, list) and all(a in v for a in arg)
        elif op == "$elemMatch":
            ok = isinstance(v, list) and any(
                matches(x, arg) if isinstance(x, dict) else _match_ops(x, arg) for x in v)
        elif op == "$not":
            ok = not (_match_ops(v, arg) if isinstance(arg, dict) else _eq(v, arg))
        else:
            raise ValueError(f"unsupported query operator {op}")
        if not ok:
            return False
    return True


def matches(doc: dict, flt: dict | None) -> bool:
    if not flt:
        return True
    for key, cond in flt.items():
        if key == "$and":
            if not all(matches(doc, c) for c in cond):
                return False
        elif key == "$or":
            if not any(matches(doc, c) for c in cond):
                return False
        elif key == "$nor":
            if any(matches(doc, c) for c in cond):
                return False
        else:
            v = get_path(doc, key)
            if isinstance(cond, dict) and cond and all(k.startswith("$") for k in cond):
                if not _match_ops(v, cond):
                    return False
            elif not _eq(v, cond):
                return False
    return True


def apply_update(doc: dict, patch: dict) -> dict:
    """Apply a plain patch (field replace) or operator update ($set $unset $inc $push $addToSet)."""
    if not any(k.startswith("$") for k in patch):
        doc.update(patch)
        return doc
    for op, fields in patch.items():
        for path, val in fields.items():
            parts = path.split(".")
            tgt = doc
            for p in parts[:-1]:
                tgt = tgt.setdefault(p, {})
            last = parts[-1]
            if op == "$set":
                tgt[last] = val
            elif op == "$unset":
                tgt.pop(last, None)
            elif op == "$inc":
                tgt[last] = (tgt.get(last) or 0) + val
            elif op == "$push":
                tgt.setdefault(last, []).append(val)
            elif op == "$addToSet":
                lst = tgt.setdefault(last, [])
                if val not in lst:
                    lst.append(val)
            else:
                raise ValueError(f"unsupported update operator {op}")
    return doc


def simple_equality_keys(flt: dict) -> dict:
    """The top-level plain-equality / $in terms usable for an index lookup."""
    out = {}
    for k, v in (flt or {}).items():
        if k.startswith("$") or "." in k:
            continue
        if isinstance(v, dict):
            if set(v) == {"$in"}:
                out[k] = ("in", v["$in"])
            elif set(v) == {"$eq"}:
                out[k] = ("eq", v["$eq"])
        elif not isinstance(v, list):
            out[k] = ("eq", v)
    return out
