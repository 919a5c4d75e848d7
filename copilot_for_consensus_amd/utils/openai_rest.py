"""Minimal OpenAI / Azure OpenAI REST client (no SDK) with the reference's rate-limit handling.

The reference's OpenAI drivers use the ``openai`` SDK (openai_summarizer.py:46, openai_provider.py:
20), which this image does not ship.  This client speaks the same two endpoints over plain HTTP --
``POST {base}/chat/completions`` and ``POST {base}/embeddings``; Azure:
``{endpoint}/openai/deployments/{deployment}/...?api-version=`` with an ``api-key`` header -- and
retries 429s the way openai_summarizer.py:189-286 does: full jitter over an exponential backoff
(``base_backoff_seconds * 2^(attempt-1)``, capped at 120 s), or over ``retry-after(-ms)`` x 1.5 when
the server sends one, at most ``max_retries`` times.  Any OpenAI-compatible server works,
including this framework's own LLM and embedding servers (serving/).
"""
from __future__ import annotations

import json
import random
import time
import urllib.error
import urllib.request
from typing import Any, Callable


class OpenAIHTTPError(RuntimeError):
    def __init__(self, status: int, body: str):
        super().__init__(f"HTTP {status}: {body[:300]}")
        self.status_code = status


class OpenAIRestClient:
    RETRY_AFTER_JITTER = 1.5

    def __init__(self, api_key: str | None = None, base_url: str | None = None, azure_endpoint: str | None = None,
                 api_version: str | None = None, deployment: str | None = None, max_retries: int = 3,
                 base_backoff_seconds: float = 5.0, timeout: float = 300.0, sleep: Callable[[float], None] = time.sleep,
                 organization: str | None = None):
        self.key, self.azure = api_key, bool(azure_endpoint)
        self.base = (azure_endpoint or base_url or "https://api.openai.com/v1").rstrip("/")
        self.api_version, self.deployment = api_version or "2024-02-15-preview", deployment
        self.max_retries, self.base_backoff = int(max_retries), float(base_backoff_seconds)
        self.timeout, self.sleep, self.org = timeout, sleep, organization
        self.retries = 0

    def _url(self, op: str) -> str:
        if self.azure:
            return f"{self.base}/openai/deployments/{self.deployment}/{op}?api-version={self.api_version}"
        return f"{self.base}/{op}"

    def _headers(self) -> dict[str, str]:
        h = {"Content-Type": "application/json"}
        if self.key:
            h["api-key" if self.azure else "Authorization"] = self.key if self.azure else f"Bearer {self.key}"
        if self.org and not self.azure:
            h["OpenAI-Organization"] = self.org
        return h

    def backoff(self, attempt: int, retry_after: float | None) -> float:
        """Full-jitter delay (openai_summarizer.py:256-285)."""
        if retry_after is not None and retry_after > 0:
            cap = min(retry_after * self.RETRY_AFTER_JITTER, 120.0)
        else:
            cap = min(self.base_backoff * (2 ** (attempt - 1)), 120.0)
        return random.uniform(0, cap)

    @staticmethod
    def _retry_after(headers) -> float | None:
        try:
            if headers.get("retry-after-ms"):
                return int(headers["retry-after-ms"]) / 1000.0
            if headers.get("retry-after"):
                return float(headers["retry-after"])
        except (TypeError, ValueError):
            return None
        return None

    def post(self, op: str, payload: dict) -> dict:
        body = json.dumps(payload).encode()
        attempt = 0
        while True:
            req = urllib.request.Request(self._url(op), data=body, method="POST", headers=self._headers())
            try:
                with urllib.request.urlopen(req, timeout=self.timeout) as r:
                    return json.loads(r.read())
            except urllib.error.HTTPError as e:
                text = e.read().decode(errors="replace")
                if e.code != 429 or attempt >= self.max_retries:
                    raise OpenAIHTTPError(e.code, text) from None
                attempt += 1
                self.retries += 1
                self.sleep(self.backoff(attempt, self._retry_after(e.headers)))

    def chat(self, model: str, messages: list[dict], max_tokens: int | None = None, **kw) -> dict:
        payload: dict[str, Any] = {"messages": messages, **kw}
        if not self.azure:
            payload["model"] = model
        if max_tokens is not None:
            payload["max_tokens"] = int(max_tokens)
        return self.post("chat/completions", payload)

    def embeddings(self, model: str, inputs: str | list[str]) -> list[list[float]]:
        payload: dict[str, Any] = {"input": inputs}
        if not self.azure:
            payload["model"] = model
        data = self.post("embeddings", payload)["data"]
        return [d["embedding"] for d in sorted(data, key=lambda d: d.get("index", 0))]
