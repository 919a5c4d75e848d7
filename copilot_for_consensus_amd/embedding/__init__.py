"""Embedding providers (API of adapters/copilot_embedding: EmbeddingProvider.embed(text), base.py:12).

* :class:`HipEncoderProvider` (driver ``hip``) -- the MI355X encoder (models/encoder.py) behind the
  reference's single-text API, plus ``embed_batch`` / ``embed_tensor`` which the embedding
  service uses: hundreds of chunks per forward, varlen-packed, vectors left in HBM for the
  HIP index (the reference calls ``embed`` once per chunk, embedding/app/service.py:384-393).
* :class:`MockEmbeddingProvider` (driver ``mock``) -- deterministic vectors from SHA-256 of the
  text (the reference uses Python's per-process-salted ``hash``, mock_provider.py:75; SHA-256
  keeps test vectors stable across processes).
* ``sentencetransformers`` / ``huggingface`` / ``openai`` drivers load their external libraries
  lazily and fail with an explanation when absent.
"""
from __future__ import annotations

import hashlib
import struct
from abc import ABC, abstractmethod

import numpy as np
import torch


class EmbeddingProvider(ABC):
    model_name: str = "unknown"
    backend: str = "unknown"
    dimension: int = 0

    @abstractmethod
    def embed(self, text: str) -> list[float]: ...

    def embed_batch(self, texts: list[str]) -> list[list[float]]:
        return [self.embed(t) for t in texts]

    def embed_tensor(self, texts: list[str]) -> torch.Tensor:
        return torch.tensor(self.embed_batch(texts), dtype=torch.float32)


def _check_text(text):
    if text is None:
        raise ValueError("Text cannot be None")
    if not isinstance(text, str):
        raise ValueError(f"Text must be a string, got {type(text).__name__}")
    if not text.strip():
        raise ValueError("Text cannot be empty or whitespace-only")


class MockEmbeddingProvider(EmbeddingProvider):
    backend = "mock"

    def __init__(self, dimension: int = 384, **_):
        self.dimension = int(dimension)
        self.model_name = f"mock-{self.dimension}"

    def embed(self, text: str) -> list[float]:
        _check_text(text)
        out = []
        counter = 0
        while len(out) < self.dimension:
            h = hashlib.sha256(f"{counter}:{text}".encode()).digest()
            out.extend(x / 4294967295.0 for x in struct.unpack("<8I", h))
            counter += 1
        return out[:self.dimension]


class HipEncoderProvider(EmbeddingProvider):
    backend = "hip"

    def __init__(self, model_name: str = "all-MiniLM-L6-v2", checkpoint_dir: str | None = None, device: str = "cuda",
                 seed: int = 0, max_tokens_per_forward: int = 65536, **_):
        from ..models.encoder import EncoderModel, get_encoder_config
        from ..runtime.tokenizer import WordPieceTokenizer, synthetic_wordpiece
        cfg = get_encoder_config(model_name)
        dev = device if (not str(device).startswith("cuda") or torch.cuda.is_available()) else "cpu"
        if checkpoint_dir:
            from pathlib import Path
            self.model = EncoderModel.from_safetensors(cfg, checkpoint_dir, dev)
            self.tokenizer = WordPieceTokenizer.from_vocab_txt(Path(checkpoint_dir) / "vocab.txt",
                                                               max_length=cfg.max_seq_length)
        else:
            self.model = EncoderModel.random(cfg, dev, seed=seed)
            self.tokenizer = synthetic_wordpiece(cfg.vocab_size, cfg.max_seq_length)
        self.model_name = cfg.name
        self.dimension = cfg.hidden
        self.max_tokens_per_forward = max_tokens_per_forward

    def embed_tensor(self, texts: list[str]) -> torch.Tensor:
        """[n, dim] fp32 L2-normalised embeddings, on the encoder's device."""
        for t in texts:
            _check_text(t)
        ids = self.tokenizer.encode_batch(texts)
        return self.model.encode_ids(ids, max_tokens_per_forward=self.max_tokens_per_forward)

    def embed_batch(self, texts: list[str]) -> list[list[float]]:
        return self.embed_tensor(texts).cpu().tolist()

    def embed(self, text: str) -> list[float]:
        return self.embed_batch([text])[0]


class SentenceTransformerProvider(EmbeddingProvider):  # pragma: no cover - optional dependency
    backend = "sentencetransformers"

    def __init__(self, model_name="all-MiniLM-L6-v2", device="cpu", cache_dir=None, **_):
        try:
            from sentence_transformers import SentenceTransformer
        except ImportError as e:
            raise ImportError("sentence-transformers is not installed; use EMBEDDING_BACKEND_TYPE=hip") from e
        self.model = SentenceTransformer(model_name, device=device, cache_folder=cache_dir)
        self.model_name = model_name
        self.dimension = self.model.get_sentence_embedding_dimension()

    def embed(self, text):
        _check_text(text)
        return self.model.encode(text).tolist()


class OpenAIEmbeddingProvider(EmbeddingProvider):
    """OpenAI / Azure OpenAI embeddings over REST (reference openai_provider.py:20,124-126; no SDK
    needed): ``POST {base}/embeddings`` with 429 backoff -- works against any OpenAI-compatible
    endpoint, including this framework's HIP embedding server (serving/embed_server.py)."""
    backend = "openai"

    def __init__(self, api_key=None, model=None, organization=None, base_url=None, api_base=None, api_version=None,
                 deployment_name=None, **_):
        from ..utils.openai_rest import OpenAIRestClient
        azure = bool(api_base and deployment_name)
        self.client = OpenAIRestClient(api_key=api_key, base_url=base_url, azure_endpoint=api_base if azure else None,
                                       api_version=api_version, deployment=deployment_name, organization=organization)
        self.model_name = model or deployment_name or "text-embedding-3-small"
        self._dim = None

    @property
    def dimension(self) -> int:
        if self._dim is None:            # probe once, as the reference's embedding main does (main.py:295)
            self._dim = len(self.embed("test"))
        return self._dim

    def embed(self, text):
        _check_text(text)
        return self.client.embeddings(self.model_name, text)[0]

    def embed_batch(self, texts: list[str]) -> list[list[float]]:
        for t in texts:
            _check_text(t)
        return self.client.embeddings(self.model_name, list(texts)) if texts else []


def create_embedding_provider(cfg=None, **overrides) -> EmbeddingProvider:
    name = getattr(cfg, "driver_name", cfg) or "hip"
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "hip":
        return HipEncoderProvider(**kw)
    if name == "mock":
        return MockEmbeddingProvider(**kw)
    if name == "sentencetransformers":
        return SentenceTransformerProvider(**kw)
    if name == "huggingface":
        # the HIP encoder loads HF BERT safetensors directly (same math, unmasked-mean quirk aside)
        return HipEncoderProvider(model_name=kw.get("model_name") or "all-MiniLM-L6-v2",
                                  device=kw.get("device") or "cuda")
    if name in ("openai", "azure_openai"):
        return OpenAIEmbeddingProvider(**kw)
    raise ValueError(f"unknown embedding backend {name!r}")


__all__ = ["EmbeddingProvider", "MockEmbeddingProvider", "HipEncoderProvider", "create_embedding_provider"]
del np
