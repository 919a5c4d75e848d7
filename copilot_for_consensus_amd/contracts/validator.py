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


# ---------------------------------------------------------------------------------------------
# Schemas are compiled once into closures (one per schema node): validating an event then costs a
# few attribute-free checks per field instead of re-reading every keyword of the schema dict on
# every value (~30 dict lookups per node; thousands of events per batch go through this).  The
# error messages and the keyword semantics are those of the original interpreter.
_COMPILED: dict[tuple[int, int, int], tuple] = {}


def _compiled(s: Any, reg: SchemaRegistry | None, root: Any) -> Callable:
    key = (id(s), id(reg), id(root))
    hit = _COMPILED.get(key)
    if hit is None or hit[1] is not s or hit[3] is not root:
        # the schema / root objects are kept alive with the entry, so their ids cannot be reused
        hit = _COMPILED[key] = (_build(s, reg, root), s, reg, root)
    return hit[0]


def _noop(v, path, errs):
    return None


def _build(s: Any, reg: SchemaRegistry | None, root: Any) -> Callable:
    if s is True or s is None:
        return _noop
    if s is False:
        return lambda v, path, errs: errs.append(f"{path}: not allowed")
    ref_fn = None
    if "$ref" in s:
        ref = s["$ref"]
        if reg is None and not ref.startswith("#"):
            raise KeyError(f"$ref {ref!r} needs a registry")
        target = (reg or SchemaRegistry()).resolve(ref, root)
        troot = target if not ref.startswith("#") else root

        def ref_fn(v, path, errs, target=target, troot=troot):     # lazy: schemas may recurse
            _compiled(target, reg, troot)(v, path, errs)
    t = s.get("type")
    types = tuple(_TYPES[x] for x in (t if isinstance(t, list) else [t])) if t is not None else None
    has_const, const = "const" in s, s.get("const")
    enum = s.get("enum")
    min_len, max_len = s.get("minLength"), s.get("maxLength")
    pat = re.compile(s["pattern"]) if "pattern" in s else None
    fmt = s.get("format")
    str_checks = min_len is not None or max_len is not None or pat is not None or fmt is not None
    minimum, maximum = s.get("minimum"), s.get("maximum")
    num_checks = minimum is not None or maximum is not None
    min_items, max_items, unique = s.get("minItems"), s.get("maxItems"), bool(s.get("uniqueItems"))
    items = s.get("items")
    has_items = "items" in s
    simple = _simple_type(items) if has_items else None
    items_fn = _compiled(items, reg, root) if has_items and simple is None and items is not True else None
    list_checks = min_items is not None or max_items is not None or unique or has_items
    props = {k: _compiled(sub, reg, root) for k, sub in s.get("properties", {}).items()}
    required = tuple(s.get("required", ()))
    has_ap = "additionalProperties" in s
    ap = s.get("additionalProperties")
    ap_fn = _compiled(ap, reg, root) if isinstance(ap, dict) else None
    dict_checks = bool(props) or bool(required) or has_ap
    all_of = tuple(_compiled(x, reg, root) for x in s.get("allOf", ()))
    any_of = tuple(_compiled(x, reg, root) for x in s["anyOf"]) if "anyOf" in s else None
    one_of = tuple(_compiled(x, reg, root) for x in s["oneOf"]) if "oneOf" in s else None
    not_fn = _compiled(s["not"], reg, root) if "not" in s else None
    is_num = _TYPES["number"]

    def fails(fn, v, path):
        e: list[str] = []
        fn(v, path, e)
        return bool(e)

    def f(v, path, errs):
        if ref_fn is not None:
            ref_fn(v, path, errs)
        if types is not None and not any(tf(v) for tf in types):
            errs.append(f"{path}: expected {t}, got {type(v).__name__}")
            return
        if has_const and v != const:
            errs.append(f"{path}: must equal {const!r}")
        if enum is not None and v not in enum:
            errs.append(f"{path}: {v!r} not in {enum}")
        if str_checks and isinstance(v, str):
            if min_len is not None and len(v) < min_len:
                errs.append(f"{path}: shorter than {min_len}")
            if max_len is not None and len(v) > max_len:
                errs.append(f"{path}: longer than {max_len}")
            if pat is not None and not pat.search(v):
                errs.append(f"{path}: {v!r} does not match {pat.pattern}")
            if fmt is not None and not _check_format(fmt, v):
                errs.append(f"{path}: not a valid {fmt}")
        if num_checks and is_num(v):
            if minimum is not None and v < minimum:
                errs.append(f"{path}: {v} < minimum {minimum}")
            if maximum is not None and v > maximum:
                errs.append(f"{path}: {v} > maximum {maximum}")
        if list_checks and isinstance(v, list):
            if min_items is not None and len(v) < min_items:
                errs.append(f"{path}: fewer than {min_items} items")
            if max_items is not None and len(v) > max_items:
                errs.append(f"{path}: more than {max_items} items")
            if unique and len({repr(x) for x in v}) != len(v):
                errs.append(f"{path}: items not unique")
            if simple is not None:
                ok = _TYPES[simple]
                for i, x in enumerate(v):
                    if not ok(x):
                        errs.append(f"{path}[{i}]: expected {simple}, got {type(x).__name__}")
            elif items_fn is not None:
                for i, x in enumerate(v):
                    items_fn(x, f"{path}[{i}]", errs)
        if dict_checks and isinstance(v, dict):
            for k in required:
                if k not in v:
                    errs.append(f"{path}: missing required '{k}'")
            for k, x in v.items():
                pf = props.get(k)
                if pf is not None:
                    pf(x, f"{path}.{k}", errs)
                elif has_ap:
                    if ap is False:
                        errs.append(f"{path}: unexpected property '{k}'")
                    elif ap_fn is not None:
                        ap_fn(x, f"{path}.{k}", errs)
        for sub in all_of:
            sub(v, path, errs)
        if any_of is not None and not any(not fails(sub, v, path) for sub in any_of):
            errs.append(f"{path}: matches none of anyOf")
        if one_of is not None:
            n = sum(1 for sub in one_of if not fails(sub, v, path))
            if n != 1:
                errs.append(f"{path}: matches {n} of oneOf (need exactly 1)")
        if not_fn is not None and not fails(not_fn, v, path):
            errs.append(f"{path}: matches 'not' schema")
    return f


def _validate(v: Any, s: Any, path: str, errs: list[str], reg: SchemaRegistry | None, root: dict) -> None:
    _compiled(s, reg, root)(v, path, errs)


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
