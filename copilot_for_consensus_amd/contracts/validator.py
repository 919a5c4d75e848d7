"""Self-contained JSON Schema (Draft 2020-12 subset) validator.

The reference validates every event and document with ``jsonschema`` + a ``referencing``
registry (adapters/copilot_schema_validation/copilot_schema_validation/schema_validator.py:18,91).
``jsonschema`` is not part of this image, and the schemas this package emits use a small,
well-defined subset, so validation is implemented here: type (incl. type lists / null),
properties, required, additionalProperties (bool or schema), enum, const, pattern,
min/maxLength, minimum/maximum, items, min/maxItems, uniqueItems, format (date-time, uuid,
email), allOf / anyOf / oneOf / not, and ``$ref`` resolved against a registry by ``$id``
(absolute or relative file name) or a local ``#/$defs/...`` pointer.
"""
from __future__ import annotations

import re
import uuid
from datetime import datetime
from typing import Any, Callable

_TYPES: dict[str, Callable[[Any], bool]] = {
    "object": lambda v: isinstance(v, dict),
    "array": lambda v: isinstance(v, list),
    "string": lambda v: isinstance(v, str),
    "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
    "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
    "boolean": lambda v: isinstance(v, bool),
    "null": lambda v: v is None,
}

_EMAIL = re.compile(r"^[^@\s]+@[^@\s]+$")


def _check_format(fmt: str, v: str) -> bool:
    if fmt == "date-time":
        try:
            datetime.fromisoformat(v.replace("Z", "+00:00"))
            return "T" in v or " " in v
        except ValueError:
            return False
    if fmt == "uuid":
        try:
            uuid.UUID(v)
            return True
        except ValueError:
            return False
    if fmt == "email":
        return bool(_EMAIL.match(v))
    return True  # unknown formats are annotations only (Draft 2020-12 default)


class ValidationError(ValueError):
    def __init__(self, errors: list[str]):
        super().__init__("; ".join(errors[:10]))
        self.errors = errors


class SchemaRegistry:
    """Maps schema ids / file names to schema documents for ``$ref`` resolution."""

    def __init__(self):
        self._by_key: dict[str, dict] = {}

    def add(self, schema: dict, *aliases: str) -> None:
        keys = list(aliases)
        sid = schema.get("$id")
        if sid:
            keys += [sid, sid.rsplit("/", 1)[-1]]
        for k in keys:
            self._by_key[k] = schema
            self._by_key[k.rsplit("/", 1)[-1]] = schema

    def resolve(self, ref: str, root: dict) -> dict:
        base, _, frag = ref.partition("#")
        doc = root if not base else self._by_key.get(base) or self._by_key.get(base.rsplit("/", 1)[-1])
        if doc is None:
            raise KeyError(f"unresolvable $ref {ref!r}")
        node: Any = doc
        for part in [p for p in frag.split("/") if p]:
            node = node[part.replace("~1", "/").replace("~0", "~")]
        return node


_PATTERN_CACHE: dict[str, re.Pattern] = {}
_ANNOTATIONS = {"type", "description", "title", "$comment", "examples"}


def _simple_type(s: Any) -> str | None:
    """The type name of an items schema that only constrains the JSON type (else None)."""
    if isinstance(s, dict) and isinstance(s.get("type"), str) and s["type"] in _TYPES and s.keys() <= _ANNOTATIONS:
        return s["type"]
    return None


def _validate(v: Any, s: Any, path: str, errs: list[str], reg: SchemaRegistry | None, root: dict) -> None:
    if s is True or s is None:
        return
    if s is False:
        errs.append(f"{path}: not allowed")
        return
    if "$ref" in s:
        if reg is None and not s["$ref"].startswith("#"):
            raise KeyError(f"$ref {s['$ref']!r} needs a registry")
        target = (reg or SchemaRegistry()).resolve(s["$ref"], root)
        _validate(v, target, path, errs, reg, target if not s["$ref"].startswith("#") else root)
    t = s.get("type")
    if t is not None:
        types = t if isinstance(t, list) else [t]
        if not any(_TYPES[x](v) for x in types):
            errs.append(f"{path}: expected {t}, got {type(v).__name__}")
            return
    if "const" in s and v != s["const"]:
        errs.append(f"{path}: must equal {s['const']!r}")
    if "enum" in s and v not in s["enum"]:
        errs.append(f"{path}: {v!r} not in {s['enum']}")
    if isinstance(v, str):
        if "minLength" in s and len(v) < s["minLength"]:
            errs.append(f"{path}: shorter than {s['minLength']}")
        if "maxLength" in s and len(v) > s["maxLength"]:
            errs.append(f"{path}: longer than {s['maxLength']}")
        if "pattern" in s:
            pat = _PATTERN_CACHE.get(s["pattern"])
            if pat is None:
                pat = _PATTERN_CACHE[s["pattern"]] = re.compile(s["pattern"])
            if not pat.search(v):
                errs.append(f"{path}: {v!r} does not match {s['pattern']}")
        if "format" in s and not _check_format(s["format"], v):
            errs.append(f"{path}: not a valid {s['format']}")
    if _TYPES["number"](v):
        if "minimum" in s and v < s["minimum"]:
            errs.append(f"{path}: {v} < minimum {s['minimum']}")
        if "maximum" in s and v > s["maximum"]:
            errs.append(f"{path}: {v} > maximum {s['maximum']}")
    if isinstance(v, list):
        if "minItems" in s and len(v) < s["minItems"]:
            errs.append(f"{path}: fewer than {s['minItems']} items")
        if "maxItems" in s and len(v) > s["maxItems"]:
            errs.append(f"{path}: more than {s['maxItems']} items")
        if s.get("uniqueItems") and len({repr(x) for x in v}) != len(v):
            errs.append(f"{path}: items not unique")
        if "items" in s:
            it = s["items"]
            simple = _simple_type(it)
            if simple is not None:
                # fast path for id lists ({"type": "string"} items): one type check per item, no
                # recursion or path formatting unless an item fails
                ok = _TYPES[simple]
                for i, x in enumerate(v):
                    if not ok(x):
                        errs.append(f"{path}[{i}]: expected {simple}, got {type(x).__name__}")
            else:
                for i, x in enumerate(v):
                    _validate(x, it, f"{path}[{i}]", errs, reg, root)
    if isinstance(v, dict):
        props = s.get("properties", {})
        for k in s.get("required", []):
            if k not in v:
                errs.append(f"{path}: missing required '{k}'")
        for k, x in v.items():
            if k in props:
                _validate(x, props[k], f"{path}.{k}", errs, reg, root)
            elif "additionalProperties" in s:
                ap = s["additionalProperties"]
                if ap is False:
                    errs.append(f"{path}: unexpected property '{k}'")
                elif isinstance(ap, dict):
                    _validate(x, ap, f"{path}.{k}", errs, reg, root)
    for sub in s.get("allOf", []):
        _validate(v, sub, path, errs, reg, root)
    if "anyOf" in s:
        if not any(not _collect(v, sub, path, reg, root) for sub in s["anyOf"]):
            errs.append(f"{path}: matches none of anyOf")
    if "oneOf" in s:
        n = sum(1 for sub in s["oneOf"] if not _collect(v, sub, path, reg, root))
        if n != 1:
            errs.append(f"{path}: matches {n} of oneOf (need exactly 1)")
    if "not" in s and not _collect(v, s["not"], path, reg, root):
        errs.append(f"{path}: matches 'not' schema")


def _collect(v, s, path, reg, root) -> list[str]:
    e: list[str] = []
    _validate(v, s, path, e, reg, root)
    return e


def iter_errors(instance: Any, schema: dict, registry: SchemaRegistry | None = None) -> list[str]:
    return _collect(instance, schema, "$", registry, schema)


def validate_json(instance: Any, schema: dict, registry: SchemaRegistry | None = None) -> tuple[bool, list[str]]:
    """(is_valid, errors) -- the reference's validate_json contract (schema_validator.py:91)."""
    errs = iter_errors(instance, schema, registry)
    return (not errs, errs)


def validate_or_raise(instance: Any, schema: dict, registry: SchemaRegistry | None = None) -> None:
    errs = iter_errors(instance, schema, registry)
    if errs:
        raise ValidationError(errs)
