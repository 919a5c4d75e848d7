"""Load-time driver-config validation (config/specs.py CONSTRAINTS, config/loader.py
validate_driver_config): one case per constraint class of the reference's driver schemas
(docs/schemas/configs/adapters/drivers/*/*.json, enforced by copilot_config/schema_validation.py:279-372)."""
from __future__ import annotations

import json

import pytest

from copilot_for_consensus_amd.config import specs
from copilot_for_consensus_amd.config.loader import ConfigError, get_config, load_adapter_config


def test_required_field_missing():
    # embedding_openai.json: "required": ["api_key", "model"]
    with pytest.raises(ConfigError, match="api_key parameter is required"):
        load_adapter_config("embedding_backend", env={"EMBEDDING_BACKEND_TYPE": "openai", "EMBEDDING_MODEL": "m"})


def test_min_length_counts_as_missing():
    # pushgateway "gateway": required + minLength 1 -- a blank value is missing, not valid
    with pytest.raises(ConfigError, match="gateway parameter is required"):
        load_adapter_config("metrics", env={"METRICS_TYPE": "pushgateway", "PUSHGATEWAY_GATEWAY": "   "})


@pytest.mark.parametrize("dev,ok", [("cpu", True), ("cuda", True), ("cuda:3", True), ("mps", True),
                                    ("gpu0", False), ("cuda:", False), ("CUDA", False)])
def test_pattern(dev, ok):
    # embedding_sentencetransformers.json device pattern ^(cpu|mps|cuda(:\d+)?)$
    env = {"EMBEDDING_BACKEND_TYPE": "sentencetransformers", "SENTENCETRANSFORMERS_DEVICE": dev}
    if ok:
        assert load_adapter_config("embedding_backend", env=env).device == dev
    else:
        with pytest.raises(ConfigError, match="device parameter is invalid"):
            load_adapter_config("embedding_backend", env=env)


def test_enum():
    with pytest.raises(ConfigError, match="algorithm parameter is invalid"):
        load_adapter_config("jwt_signer", env={"AUTH_JWT_ALGORITHM": "none", "JWT_SECRET_KEY": "x"})
    env = {"MESSAGE_BUS_TYPE": "rabbitmq", "RABBITMQ_USERNAME": "u", "RABBITMQ_PASSWORD": "p"}
    cfg = load_adapter_config("message_bus", env=env, overrides={"rabbitmq_username": "u", "rabbitmq_password": "p"})
    assert cfg.exchange_type == "topic"
    with pytest.raises(ConfigError, match="exchange_type parameter is invalid"):
        load_adapter_config("message_bus", env=env, overrides={"rabbitmq_username": "u", "rabbitmq_password": "p",
                                                                "exchange_type": "broadcast"})


def test_enum_case_insensitive_where_the_driver_is():
    assert load_adapter_config("logger", env={"LOG_LEVEL": "info"}).level == "info"
    with pytest.raises(ConfigError, match="level parameter is invalid"):
        load_adapter_config("logger", env={"LOG_LEVEL": "verbose"})


@pytest.mark.parametrize("port,ok", [("1", True), ("65535", True), ("0", False), ("70000", False)])
def test_minimum_maximum(port, ok):
    env = {"DOCUMENT_STORE_TYPE": "mongodb", "MONGODB_PORT": port}
    if ok:
        assert load_adapter_config("document_store", env=env).port == int(port)
    else:
        with pytest.raises(ConfigError, match="port parameter is invalid"):
            load_adapter_config("document_store", env=env)


def test_float_bounds():
    env = {"MESSAGE_BUS_TYPE": "azure_service_bus", "SERVICEBUS_CONNECTION_STRING": "Endpoint=sb://x/"}
    assert load_adapter_config("message_bus", env=env, overrides={"retry_backoff_seconds": 0.1})
    with pytest.raises(ConfigError, match="retry_backoff_seconds parameter is invalid"):
        load_adapter_config("message_bus", env=env, overrides={"retry_backoff_seconds": 0.05})


def test_format_uri():
    with pytest.raises(ConfigError, match="llamacpp_endpoint parameter is invalid"):
        load_adapter_config("llm_backend", env={"LLM_BACKEND_TYPE": "llamacpp", "LLAMACPP_ENDPOINT": "llama-cpp:8081"})
    assert load_adapter_config("llm_backend", env={"LLM_BACKEND_TYPE": "llamacpp"}).llamacpp_endpoint.startswith("http")


def test_conditional_required_hs256_needs_secret():
    # jwt_signer/local.json x-conditional_required: HS* -> secret_key, RS* / ES* -> the key pair
    with pytest.raises(ConfigError, match="secret_key parameter is required"):
        load_adapter_config("jwt_signer", env={"AUTH_JWT_ALGORITHM": "HS256"})
    ok = load_adapter_config("jwt_signer", env={"AUTH_JWT_ALGORITHM": "HS256"}, overrides={"secret_key": "s"})
    assert ok.secret_key == "s"
    with pytest.raises(ConfigError, match="private_key parameter is required"):
        load_adapter_config("jwt_signer", env={"AUTH_JWT_ALGORITHM": "RS256"})
    with pytest.raises(ConfigError, match="private_key parameter is required"):
        get_config("auth", env={})         # the auth service refuses to start without its key


def test_conditional_required_else_branch():
    # azure_service_bus: managed identity -> namespace, otherwise -> connection string
    with pytest.raises(ConfigError, match="connection_string parameter is required"):
        load_adapter_config("message_bus", env={"MESSAGE_BUS_TYPE": "azure_service_bus"})
    with pytest.raises(ConfigError, match="servicebus_fully_qualified_namespace parameter is required"):
        load_adapter_config("message_bus", env={"MESSAGE_BUS_TYPE": "azure_service_bus",
                                                "SERVICEBUS_USE_MANAGED_IDENTITY": "true"})
    assert load_adapter_config("message_bus", env={"MESSAGE_BUS_TYPE": "azure_service_bus",
                                                   "SERVICEBUS_USE_MANAGED_IDENTITY": "true",
                                                   "SERVICEBUS_FULLY_QUALIFIED_NAMESPACE": "ns.servicebus"})


def test_required_one_of():
    with pytest.raises(ConfigError, match="Either vault_url or vault_name parameter is required"):
        load_adapter_config("secret_provider", env={"SECRET_PROVIDER_TYPE": "azure_key_vault"})
    assert load_adapter_config("secret_provider", env={"SECRET_PROVIDER_TYPE": "azure_key_vault",
                                                       "AZURE_KEY_VAULT_NAME": "kv"}).vault_name == "kv"


def test_secret_backed_key_pair_satisfies_the_rule(tmp_path):
    from copilot_for_consensus_amd.security.jwt import RSASigner, create_jwt_signer, generate_keys
    generate_keys(tmp_path)
    cfg = get_config("auth", env={"SECRET_PROVIDER_TYPE": "local", "SECRETS_BASE_PATH": str(tmp_path)})
    signer = create_jwt_signer(cfg.jwt_signer)
    assert isinstance(signer, RSASigner) and signer.verify(b"m", signer.sign(b"m"))


def test_every_constraint_names_real_fields():
    for (adapter, driver), c in specs.CONSTRAINTS.items():
        fields = specs.ADAPTERS[adapter][3][driver]
        names = set(c.get("required", [])) | set(c.get("fields", {}))
        for r in c.get("conditional_required", []):
            names |= {r["if"]["field"], *r.get("then_required", []), *r.get("else_required", [])}
        for g in c.get("required_one_of", []):
            names |= set(g)
        assert names <= set(fields), (adapter, driver, names - set(fields))


def test_exported_driver_schemas_carry_the_rules(tmp_path):
    from copilot_for_consensus_amd.tools.schemas import export_all
    export_all(tmp_path)
    local = json.loads((tmp_path / "configs" / "adapters" / "drivers" / "jwt_signer" / "local.json").read_text())
    assert local["required"] == ["algorithm", "key_id"]
    assert {"if": {"field": "algorithm", "equals": "HS256"}, "then_required": ["secret_key"]} \
        in local["x-conditional_required"]
    st = json.loads((tmp_path / "configs" / "adapters" / "drivers" / "embedding_backend"
                     / "sentencetransformers.json").read_text())
    assert st["properties"]["device"]["pattern"] == r"^(cpu|mps|cuda(:\d+)?)$"
    adapter = json.loads((tmp_path / "configs" / "adapters" / "embedding_backend.json").read_text())
    assert adapter["discriminant"]["env_var"] == "EMBEDDING_BACKEND_TYPE"
    assert "sentencetransformers" in adapter["drivers"]
