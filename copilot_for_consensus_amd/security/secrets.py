"""Secret providers (adapters/copilot_secrets: get_secret / get_secret_bytes / secret_exists).

* LocalFileSecretProvider -- one file per secret under ``base_path`` (``/run/secrets`` in compose,
  local_provider.py:17); names are sanitised so a secret name cannot escape the directory.
* EnvSecretProvider -- ``<PREFIX><NAME>`` environment variables (upper-cased).
* AzureKeyVaultSecretProvider -- cloud/azure.py (imports azure-keyvault-secrets on construction).
"""
from __future__ import annotations

import os
import re
from abc import ABC, abstractmethod
from pathlib import Path


class SecretNotFoundError(KeyError):
    pass


class SecretProvider(ABC):
    @abstractmethod
    def get_secret(self, name: str) -> str: ...

    def get_secret_bytes(self, name: str) -> bytes:
        return self.get_secret(name).encode()

    @abstractmethod
    def secret_exists(self, name: str) -> bool: ...


_SAFE = re.compile(r"^[A-Za-z0-9_.-]+$")


class LocalFileSecretProvider(SecretProvider):
    def __init__(self, base_path: str = "/run/secrets", **_):
        self.base = Path(base_path)

    def _path(self, name: str) -> Path:
        if not _SAFE.match(name) or name in (".", ".."):
            raise ValueError(f"invalid secret name {name!r}")
        return self.base / name

    def get_secret(self, name):
        p = self._path(name)
        if not p.is_file():
            raise SecretNotFoundError(name)
        return p.read_text(encoding="utf-8").strip()

    def get_secret_bytes(self, name):
        p = self._path(name)
        if not p.is_file():
            raise SecretNotFoundError(name)
        return p.read_bytes()

    def secret_exists(self, name):
        try:
            return self._path(name).is_file()
        except ValueError:
            return False


class EnvSecretProvider(SecretProvider):
    def __init__(self, prefix: str = "", env=None, **_):
        self.prefix = prefix or ""
        self.env = os.environ if env is None else env

    def _k(self, name):
        return (self.prefix + name).upper().replace("-", "_").replace(".", "_")

    def get_secret(self, name):
        k = self._k(name)
        if k not in self.env:
            raise SecretNotFoundError(name)
        return self.env[k]

    def secret_exists(self, name):
        return self._k(name) in self.env


def create_secret_provider(cfg=None, **overrides) -> SecretProvider:
    name = str(getattr(cfg, "driver_name", cfg) or "local").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "local":
        return LocalFileSecretProvider(**kw)
    if name == "env":
        return EnvSecretProvider(**kw)
    if name in ("azure_key_vault", "azurekeyvault"):
        from ..cloud.azure import AzureKeyVaultSecretProvider
        return AzureKeyVaultSecretProvider(**kw)
    raise ValueError(f"unknown secret provider {name!r}")
