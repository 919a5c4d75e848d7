"""Export and self-check the contracts (events, documents, service configs).

Parity target: scripts/validate_schema_registry.py and the schema files under docs/schemas/ of the
reference (plus generate_typed_configs.py's role of keeping config schemas and code in sync --
here the config schemas are generated from config/specs.py, so only export is needed).

    python -m copilot_for_consensus_amd.tools.schemas export docs/schemas
    python -m copilot_for_consensus_amd.tools.schemas check

Reference: scripts/generate_typed_configs.py:1-14 and scripts/generate_service_openapi.py.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path


def driver_json_schema(adapter: str, driver: str) -> dict:
    """One driver's schema in the reference's layout (docs/schemas/configs/adapters/drivers/
    <adapter>/<driver>.json): properties with source/env_var/default plus the validation keywords
    and x-* extensions of config/specs.py CONSTRAINTS."""
    from ..config.loader import _field_schema
    from ..config.specs import ADAPTERS, CONSTRAINTS, SECRET_FIELDS
    fields = ADAPTERS[adapter][3][driver]
    c = CONSTRAINTS.get((adapter, driver), {})
    props = {}
    for name, spec in fields.items():
        p = _field_schema(spec)
        secret = SECRET_FIELDS.get((adapter, driver, name))
        if secret:
            p.update(source="secret", secret_name=secret)
        p.update({k: v for k, v in c.get("fields", {}).get(name, {}).items() if k != "case_insensitive"})
        props[name] = p
    out = {"$schema": "https://json-schema.org/draft/2020-12/schema", "title": f"{adapter} driver {driver}",
           "type": "object", "properties": props}
    if c.get("required"):
        out["required"] = list(c["required"])
    if c.get("conditional_required"):
        out["x-conditional_required"] = [dict(r) for r in c["conditional_required"]]
    if c.get("required_one_of"):
        out["x-required_one_of"] = [list(g) for g in c["required_one_of"]]
    return out


def adapter_json_schema(adapter: str) -> dict:
    """The adapter schema (reference docs/schemas/configs/adapters/<adapter>.json): discriminant
    env var and the driver schema references."""
    from ..config.specs import ADAPTERS
    field, env, default, drivers = ADAPTERS[adapter]
    return {"$schema": "https://json-schema.org/draft/2020-12/schema", "title": f"{adapter} adapter",
            "type": "object",
            "discriminant": {"field": field, "env_var": env, "enum": sorted(drivers), "default": default},
            "drivers": {d: {"$ref": f"drivers/{adapter}/{d}.json"} for d in drivers}}


def export_all(root: str | Path) -> list[Path]:
    from ..config.loader import config_json_schema
    from ..config.specs import ADAPTERS, SERVICES
    from ..contracts.registry import default_provider
    root = Path(root)
    out = default_provider().export(root)
    cd = root / "configs" / "services"
    cd.mkdir(parents=True, exist_ok=True)
    for svc in SERVICES:
        p = cd / f"{svc}.json"
        p.write_text(json.dumps(config_json_schema(svc), indent=2) + "\n", encoding="utf-8")
        out.append(p)
    ad = root / "configs" / "adapters"
    for adapter, (_f, _e, _d, drivers) in ADAPTERS.items():
        (ad / "drivers" / adapter).mkdir(parents=True, exist_ok=True)
        p = ad / f"{adapter}.json"
        p.write_text(json.dumps(adapter_json_schema(adapter), indent=2) + "\n", encoding="utf-8")
        out.append(p)
        for d in drivers:
            p = ad / "drivers" / adapter / f"{d}.json"
            p.write_text(json.dumps(driver_json_schema(adapter, d), indent=2) + "\n", encoding="utf-8")
            out.append(p)
    return out


def check() -> list[str]:
    """Structural checks: every event type routable and its schema self-consistent; document
    schemas accept a minimal example; config schemas build for every service; env vars unique
    per service."""
    from ..config.loader import config_json_schema
    from ..config.specs import ADAPTERS, SERVICES
    from ..contracts.events import EVENT_SPECS, Event, routing_key_for
    from ..contracts.registry import default_provider
    prov = default_provider()
    problems = []
    keys = {}
    for t in EVENT_SPECS:
        rk = routing_key_for(t)
        if rk in keys:
            problems.append(f"routing key {rk} shared by {keys[rk]} and {t}")
        keys[rk] = t
        if prov.get_event_schema(t) is None:
            problems.append(f"no schema for event {t}")
        errs = prov.validate_event(Event.create(t).to_dict())
        if not errs:
            problems.append(f"{t}: empty payload unexpectedly valid (required fields missing from schema?)")
    for svc in SERVICES:
        try:
            sch = config_json_schema(svc)
        except Exception as e:  # pragma: no cover - surfaced as a problem
            problems.append(f"config schema for {svc}: {e!r}")
            continue
        if not isinstance(sch.get("service_settings"), dict) or sch.get("service_name") != svc:
            problems.append(f"config schema for {svc} lacks service_name/service_settings")
        envs = [v.get("env_var") for v in sch["service_settings"].values() if isinstance(v, dict)]
        flat = [e for x in envs for e in (x if isinstance(x, list) else [x]) if e]
        dup = {e for e in flat if flat.count(e) > 1}
        if dup:
            problems.append(f"{svc}: env vars bound to several settings: {sorted(dup)}")
    for adapter, (field, env, default, drivers) in ADAPTERS.items():
        if default is not None and default not in drivers:
            problems.append(f"adapter {adapter}: default driver {default!r} not among {sorted(drivers)}")
    return problems


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    e = sub.add_parser("export")
    e.add_argument("root")
    sub.add_parser("check")
    a = ap.parse_args(argv)
    if a.cmd == "export":
        print(f"wrote {len(export_all(a.root))} schema files under {a.root}")
        return 0
    probs = check()
    for p in probs:
        print(p, file=sys.stderr)
    print("schema registry OK" if not probs else f"{len(probs)} problem(s)")
    return 1 if probs else 0


if __name__ == "__main__":
    sys.exit(main())
