"""Typed configuration loading: ``get_config(service)`` -> ServiceConfig.

Mirrors the reference's runtime loader (adapters/copilot_config/copilot_config/runtime_loader.py:423
``get_config``; adapter_factory.py:26 ``create_adapter``): service settings come from env vars
(with aliases) and defaults, each adapter's driver is chosen by its discriminant env var, driver
fields are read from env / secrets, coerced to their types and validated against the driver's
constraints (specs.CONSTRAINTS: required, minLength, pattern, enum, minimum / maximum, format: uri,
conditional and one-of requirements -- the reference's schema_validation.py:279-372, applied at
load time as runtime_loader.py:217 does).  Instead of
code-generated dataclasses (scripts/generate_typed_configs.py) the typed objects are built from
the spec tables at import time, and ``config_json_schema`` emits the JSON Schema served at
``/.well-known/configuration-schema``.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Any, Mapping

from . import specs


class ConfigError(ValueError):
    pass


def _coerce(kind: str, raw: Any, name: str):
    if raw is None:
        return None
    if kind == specs.B:
        if isinstance(raw, bool):
            return raw
        v = str(raw).strip().lower()
        if v in ("1", "true", "yes", "on"):
            return True
        if v in ("0", "false", "no", "off", ""):
            return False
        raise ConfigError(f"{name}: cannot parse bool from {raw!r}")
    if kind == specs.I:
        try:
            return int(raw)
        except (TypeError, ValueError):
            raise ConfigError(f"{name}: cannot parse int from {raw!r}") from None
    if kind == specs.F:
        try:
            return float(raw)
        except (TypeError, ValueError):
            raise ConfigError(f"{name}: cannot parse float from {raw!r}") from None
    return str(raw)


def _read(spec: tuple, name: str, env: Mapping[str, str], overrides: Mapping[str, Any] | None = None):
    kind, env_var, default = spec[0], spec[1], spec[2]
    if overrides and name in overrides:
        return _coerce(kind, overrides[name], name)
    names = env_var if isinstance(env_var, list) else ([env_var] if env_var else [])
    for n in names:
        if n in env:
            return _coerce(kind, env[n], n)
    return default


@dataclasses.dataclass
class AdapterConfig:
    adapter: str
    driver_name: str | None
    driver_config: dict[str, Any]

    def __getattr__(self, item):
        try:
            return self.__dict__["driver_config"][item]
        except KeyError:
            raise AttributeError(item) from None


@dataclasses.dataclass
class ServiceConfig:
    service_name: str
    service_settings: dict[str, Any]
    adapters: dict[str, AdapterConfig]

    def __getattr__(self, item):
        d = self.__dict__
        if item in d.get("service_settings", {}):
            return d["service_settings"][item]
        if item in d.get("adapters", {}):
            return d["adapters"][item]
        raise AttributeError(item)


class EnvConfigProvider:
    """Reads configuration values from a mapping (os.environ by default)."""

    def __init__(self, env: Mapping[str, str] | None = None):
        self.env = os.environ if env is None else env

    def get(self, key: str, default=None):
        return self.env.get(key, default)


class StaticConfigProvider(EnvConfigProvider):
    def __init__(self, values: Mapping[str, Any]):
        super().__init__({k: str(v) for k, v in values.items()})


def env_is_set(name: str, env: Mapping[str, str] | None = None) -> bool:
    """True when the variable is explicitly set (to tell a deployment's choice from a spec default)."""
    return bool((os.environ if env is None else env).get(name))


def _missing(value: Any, rules: Mapping[str, Any]) -> bool:
    if value is None:
        return True
    return isinstance(value, str) and int(rules.get("minLength", 0) or 0) >= 1 and len(value.strip()) < rules["minLength"]


def _is_uri(value: str) -> bool:
    from urllib.parse import urlparse
    p = urlparse(value)
    return bool(p.scheme and p.netloc)


def validate_driver_config(adapter: str, driver: str, config: Mapping[str, Any]) -> None:
    """Raise ConfigError when ``config`` breaks a rule of (adapter, driver) in specs.CONSTRAINTS.
    Messages follow the reference: "<field> parameter is required" / "... is invalid"."""
    import re

    c = specs.CONSTRAINTS.get((adapter, driver))
    if not c:
        return
    fields = c.get("fields", {})
    where = f"{adapter}/{driver}"
    for name in c.get("required", []):
        if _missing(config.get(name), fields.get(name, {})):
            raise ConfigError(f"{where}: {name} parameter is required")
    for name, rules in fields.items():
        v = config.get(name)
        if v is None:
            continue
        if isinstance(v, str):
            if _missing(v, rules):
                raise ConfigError(f"{where}: {name} parameter is required")
            if "pattern" in rules and re.match(rules["pattern"], v) is None:
                raise ConfigError(f"{where}: {name} parameter is invalid ({v!r} !~ {rules['pattern']})")
            if "enum" in rules:
                vals = rules["enum"]
                ok = (v.upper() in [str(e).upper() for e in vals]) if rules.get("case_insensitive") else v in vals
                if not ok:
                    raise ConfigError(f"{where}: {name} parameter is invalid ({v!r} not in {vals})")
            if rules.get("format") == "uri" and not _is_uri(v):
                raise ConfigError(f"{where}: {name} parameter is invalid (not a URI: {v!r})")
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            if "minimum" in rules and v < rules["minimum"]:
                raise ConfigError(f"{where}: {name} parameter is invalid ({v} < {rules['minimum']})")
            if "maximum" in rules and v > rules["maximum"]:
                raise ConfigError(f"{where}: {name} parameter is invalid ({v} > {rules['maximum']})")
    for rule in c.get("conditional_required", []):
        cond = rule["if"]
        actual = config.get(cond["field"])
        if isinstance(actual, str) and isinstance(cond["equals"], str):
            hit = actual.upper() == cond["equals"].upper()
        else:
            hit = actual == cond["equals"]
        for name in rule.get("then_required" if hit else "else_required", []):
            if _missing(config.get(name), fields.get(name, {})):
                raise ConfigError(f"{where}: {name} parameter is required when {cond['field']}={actual!r}")
    for group in c.get("required_one_of", []):
        if all(_missing(config.get(n), fields.get(n, {})) for n in group):
            raise ConfigError(f"{where}: Either {' or '.join(group)} parameter is required")


def load_adapter_config(adapter: str, env: Mapping[str, str] | None = None, driver: str | None = None,
                        secrets=None, overrides: Mapping[str, Any] | None = None,
                        validate: bool = True) -> AdapterConfig:
    env = os.environ if env is None else env
    field, disc_env, default_driver, drivers = specs.ADAPTERS[adapter]
    if driver is None:
        driver = env.get(disc_env, default_driver) if disc_env else default_driver
    if isinstance(driver, str):
        driver = driver.strip().lower()      # VECTOR_STORE_TYPE=Qdrant selects the qdrant driver
    if driver is not None and driver not in drivers:
        raise ConfigError(f"{adapter}: unknown driver {driver!r} ({disc_env}); choose one of {sorted(drivers)}")
    cfg: dict[str, Any] = {}
    if driver is not None:
        for name, spec in drivers[driver].items():
            val = _read(spec, name, env, overrides)
            if val is None and secrets is not None:
                secret_name = specs.SECRET_FIELDS.get((adapter, driver, name))
                if secret_name:
                    try:
                        if secrets.secret_exists(secret_name):
                            val = secrets.get_secret(secret_name)
                    except Exception:  # secret backends are best effort at config time
                        val = None
            cfg[name] = val
        if validate:
            validate_driver_config(adapter, driver, cfg)
    return AdapterConfig(adapter, driver, cfg)


def get_config(service: str, env: Mapping[str, str] | None = None, secrets=None,
               overrides: Mapping[str, Any] | None = None) -> ServiceConfig:
    if service not in specs.SERVICES:
        raise ConfigError(f"unknown service {service!r}; known: {sorted(specs.SERVICES)}")
    env = os.environ if env is None else env
    sspec = specs.SERVICES[service]
    settings = {n: _read(sp, n, env, overrides) for n, sp in sspec["settings"].items()}
    if secrets is None and "secret_provider" in sspec["adapters"]:
        try:
            from ..security.secrets import create_secret_provider
            sp = load_adapter_config("secret_provider", env)
            # the env driver reads the same mapping the rest of the config comes from
            secrets = create_secret_provider(sp, **({"env": env} if sp.driver_name == "env" else {}))
        except Exception:
            secrets = None
    adapters = {}
    for a in sspec["adapters"]:
        if a == "oidc_providers":
            adapters[a] = AdapterConfig(a, None, {d: load_adapter_config(a, env, driver=d, secrets=secrets).driver_config
                                                  for d in specs.ADAPTERS[a][3]})
        else:
            adapters[a] = load_adapter_config(a, env, secrets=secrets)
    return ServiceConfig(service, settings, adapters)


_JSON_TYPES = {specs.S: "string", specs.I: "integer", specs.F: "number", specs.B: "boolean"}


def _field_schema(spec: tuple) -> dict:
    kind, env_var, default = spec[0], spec[1], spec[2]
    d: dict[str, Any] = {"type": [_JSON_TYPES[kind], "null"] if default is None else _JSON_TYPES[kind]}
    if env_var:
        d["source"] = "env"
        d["env_var"] = env_var
    if default is not None:
        d["default"] = default
    return d


def config_json_schema(service: str) -> dict:
    sspec = specs.SERVICES[service]
    adapters = {}
    for a in sspec["adapters"]:
        field, disc_env, default_driver, drivers = specs.ADAPTERS[a]
        adapters[a] = {
            "type": "object",
            "discriminant": {"field": field, "env_var": disc_env, "enum": sorted(drivers), "default": default_driver},
            "drivers": {d: {"type": "object", "properties": {n: _field_schema(sp) for n, sp in f.items()}}
                        for d, f in drivers.items()},
        }
    return {
        "$schema": "https://json-schema.org/draft/2020-12/schema",
        "service_name": service,
        "schema_version": "1.0.0",
        "service_settings": {n: _field_schema(sp) for n, sp in sspec["settings"].items()},
        "adapters": adapters,
    }
