"""Schema-first configuration: env parsing and coercion, aliases, discriminant driver selection,
secret-backed fields, the exported JSON schema -- and, when the reference checkout is mounted, a
sweep asserting every service setting and driver field the reference declares
(docs/schemas/configs/services/*.json, adapters/*.json, adapters/drivers/*/*.json) exists here
with the same env var(s) and default, so an existing deployment's environment keeps working.
Mirrors adapters/copilot_config/tests (test_runtime_loader.py, test_schema_validation.py)."""
from __future__ import annotations

import json
from pathlib import Path

import pytest

from copilot_for_consensus_amd.config import specs
from copilot_for_consensus_amd.config.loader import (ConfigError, config_json_schema, get_config,
                                                     load_adapter_config)
from copilot_for_consensus_amd.security.secrets import EnvSecretProvider

REF = Path("/root/reference/docs/schemas/configs")
needs_ref = pytest.mark.skipif(not REF.exists(), reason="reference checkout not mounted")


def test_defaults_without_env():
    cfg = get_config("embedding", env={})
    assert cfg.batch_size == 32 and cfg.http_port == 8000 and cfg.jwt_auth_enabled is True
    assert cfg.vector_store.driver_name == "hip" and cfg.embedding_backend.driver_name == "hip"
    assert cfg.message_bus.driver_name == "inproc"


def test_env_coercion_and_aliases():
    env = {"EMBEDDING_BATCH_SIZE": "256", "JWT_AUTH_ENABLED": "false", "EMBEDDING_HTTP_PORT": "9000",
           "VECTOR_STORE_TYPE": "qdrant", "QDRANT_HOST": "qd", "QDRANT_PORT": "7000"}
    cfg = get_config("embedding", env=env)
    assert cfg.batch_size == 256 and cfg.jwt_auth_enabled is False and cfg.http_port == 9000
    vs = cfg.vector_store
    assert vs.driver_name == "qdrant" and vs.driver_config["host"] == "qd" and vs.driver_config["port"] == 7000
    # the service-specific name wins over the global alias
    cfg = get_config("embedding", env={"EMBEDDING_JWT_AUTH_ENABLED": "1", "JWT_AUTH_ENABLED": "0"})
    assert cfg.jwt_auth_enabled is True


@pytest.mark.parametrize("raw,ok", [("yes", True), ("on", True), ("TRUE", True), ("0", False), ("no", False)])
def test_bool_spellings(raw, ok):
    assert get_config("embedding", env={"JWT_AUTH_ENABLED": raw}).jwt_auth_enabled is ok


def test_bad_values_raise():
    with pytest.raises(ConfigError):
        get_config("embedding", env={"EMBEDDING_BATCH_SIZE": "many"})
    with pytest.raises(ConfigError):
        get_config("embedding", env={"VECTOR_STORE_TYPE": "pinecone"})
    with pytest.raises(ConfigError):
        get_config("billing")


def test_secret_backed_driver_fields():
    secrets = EnvSecretProvider(env={"RABBITMQ_USERNAME": "guest", "RABBITMQ_PASSWORD": "pw"})
    bus = load_adapter_config("message_bus", env={"MESSAGE_BUS_TYPE": "rabbitmq"}, secrets=secrets)
    assert bus.driver_config["rabbitmq_username"] == "guest" and bus.driver_config["rabbitmq_password"] == "pw"
    assert bus.driver_config["rabbitmq_host"] == "messagebus"


def test_overrides_beat_env():
    cfg = load_adapter_config("chunker", env={"CHUNK_SIZE_TOKENS": "300"}, overrides={"overlap": 7})
    assert cfg.driver_config["chunk_size"] == 300 and cfg.driver_config["overlap"] == 7


def test_every_service_loads_and_exports_schema():
    from copilot_for_consensus_amd.security.jwt import RSAKey, rsa_private_pem, rsa_public_pem
    k = RSAKey.generate(1024)
    # the auth service's default local RS256 signer needs its key pair (reference
    # drivers/jwt_signer/local.json x-conditional_required), here as env secrets
    keys = {"JWT_PRIVATE_KEY": rsa_private_pem(k), "JWT_PUBLIC_KEY": rsa_public_pem(k), "SECRET_PROVIDER_TYPE": "env"}
    for svc in specs.SERVICES:
        cfg = get_config(svc, env=keys if svc == "auth" else {})
        sch = config_json_schema(svc)
        assert sch["service_name"] == svc
        for a in specs.SERVICES[svc]["adapters"]:
            assert a in sch["adapters"]
            assert getattr(cfg, a) is not None
        json.dumps(sch)


# ------------------------------------------------------------------ reference parity sweep
def _envs(e):
    return set(e) if isinstance(e, list) else {e}


@needs_ref
@pytest.mark.parametrize("path", sorted(p.name for p in (REF / "services").glob("*.json")) if REF.exists() else [])
def test_service_settings_match_reference(path):
    ref = json.loads((REF / "services" / path).read_text())
    svc = ref["service_name"]
    mine = specs.SERVICES[svc]
    diffs = []
    for name, s in ref.get("service_settings", {}).items():
        m = mine["settings"].get(name)
        if m is None:
            diffs.append(("missing", name))
            continue
        if s.get("source") == "env" and not (_envs(s["env_var"]) & _envs(m[1])):
            diffs.append(("env", name, m[1], s["env_var"]))
        if "default" in s and m[2] != s["default"]:
            diffs.append(("default", name, m[2], s["default"]))
    missing_adapters = set(ref.get("adapters", {})) - set(mine["adapters"])
    assert diffs == [] and not missing_adapters, (diffs, missing_adapters)


@needs_ref
@pytest.mark.parametrize("path", sorted(p.name for p in (REF / "adapters").glob("*.json")) if REF.exists() else [])
def test_adapter_drivers_match_reference(path):
    ref = json.loads((REF / "adapters" / path).read_text())
    adapter = path[:-5]
    field, disc_env, _, drivers = specs.ADAPTERS[adapter]
    disc = ref["properties"].get("discriminant", {})
    diffs = []
    if disc and disc.get("env_var") != disc_env:
        diffs.append(("discriminant", disc_env, disc.get("env_var")))
    for dname, refd in ref["properties"].get("drivers", {}).get("properties", {}).items():
        if dname not in drivers:
            diffs.append(("driver missing", dname))
            continue
        dspec = json.loads((REF / "adapters" / refd["$ref"]).resolve().read_text())
        for fname, fs in dspec.get("properties", {}).items():
            m = drivers[dname].get(fname)
            if m is None:
                diffs.append(("field missing", dname, fname))
                continue
            if fs.get("source") == "env" and fs.get("env_var") and not (_envs(fs["env_var"]) & _envs(m[1])):
                diffs.append(("env", dname, fname, m[1], fs["env_var"]))
            if "default" in fs and m[2] != fs["default"]:
                diffs.append(("default", dname, fname, m[2], fs["default"]))
    assert diffs == [], diffs
