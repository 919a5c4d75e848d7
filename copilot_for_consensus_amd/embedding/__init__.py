"""Embedding providers (API of adapters/copilot_embedding: EmbeddingProvider.embed(text), base.py:12).

* :class:`HipEncoderProvider` (driver ``hip``) -- the MI355X encoder (models/encoder.py) behind the
  reference's single-text API, plus ``embed_batch`` / ``embed_tensor`` which the embedding
  service uses: hundreds of chunks per forward, varlen-packed, vectors left in HBM for the
  HIP index (the reference calls ``embed`` once per chunk, embedding/app/service.py:384-393).
* :class:`MockEmbeddingProvider` (driver ``mock``) -- deterministic vectors from SHA-256 of the
  text (the reference uses Python's per-process-salted ``hash``, mock_provider.py:75; SHA-256
  keeps test vectors stable across processes).
* ``sentencetransformers`` / ``huggingface`` read the model directory (HF BERT safetensors, the
  sentence-transformers module configs) and run it on the HIP encoder with the reference driver's
  pooling / normalisation / truncation; ``openai`` speaks the REST API.
"""
from __future__ import annotations

import hashlib
import json
import struct
from abc import ABC, abstractmethod
from pathlib import Path

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
                 seed: int = 0, max_tokens_per_forward: int = 65536, pooling: str | None = None,
                 normalize: bool | None = None, max_length: int | None = None, **_):
        """``checkpoint_dir``: an HF BERT directory (config.json, *.safetensors, vocab.txt); its
        config.json sets the architecture, otherwise ``model_name`` names a preset.  ``pooling`` /
        ``normalize`` / ``max_length`` override the preset's (mean / CLS, L2, truncation length)."""
        import dataclasses

        from ..models.encoder import EncoderModel, encoder_config_from_hf, get_encoder_config
        from ..runtime.tokenizer import WordPieceTokenizer, synthetic_wordpiece
        over = {k: v for k, v in (("pooling", pooling), ("normalize", normalize)) if v is not None}
        if checkpoint_dir and (Path(checkpoint_dir) / "config.json").exists():
            cfg = encoder_config_from_hf(Path(checkpoint_dir) / "config.json", name=Path(model_name).name, **over)
        else:
            cfg = dataclasses.replace(get_encoder_config(model_name), **over)
        if max_length:
            cfg = dataclasses.replace(cfg, max_seq_length=min(int(max_length), cfg.max_positions))
        dev = device if (not str(device).startswith("cuda") or torch.cuda.is_available()) else "cpu"
        if checkpoint_dir:
            self.model = EncoderModel.from_safetensors(cfg, checkpoint_dir, dev)
            self.tokenizer = WordPieceTokenizer.from_vocab_txt(Path(checkpoint_dir) / "vocab.txt",
                                                               lowercase=_tokenizer_lowercase(Path(checkpoint_dir)),
                                                               max_length=cfg.max_seq_length)
        else:
            self.model = EncoderModel.random(cfg, dev, seed=seed)
            self.tokenizer = synthetic_wordpiece(cfg.vocab_size, cfg.max_seq_length)
        self.model_name = cfg.name
        self.dimension = cfg.hidden
        self.max_tokens_per_forward = max_tokens_per_forward

    def embed_tensor(self, texts: list[str]) -> torch.Tensor:
        """[n, dim] fp32 embeddings (L2-normalised unless configured otherwise), on the encoder's device."""
        for t in texts:
            _check_text(t)
        ids, cu = self.tokenizer.encode_packed(texts)
        return self.model.encode_packed(ids, cu, max_tokens_per_forward=self.max_tokens_per_forward)

    def embed_batch(self, texts: list[str]) -> list[list[float]]:
        return self.embed_tensor(texts).cpu().tolist()

    def embed(self, text: str) -> list[float]:
        return self.embed_batch([text])[0]


def _tokenizer_lowercase(d: Path) -> bool:
    f = d / "tokenizer_config.json"
    if f.exists():
        return bool(json.loads(f.read_text()).get("do_lower_case", True))
    return True


def resolve_model_dir(model_name: str, cache_dir: str | None = None) -> Path:
    """Local directory of an HF / sentence-transformers model: ``model_name`` itself, or under
    ``cache_dir`` (plain ``<cache>/<name>``, the hub layout ``<cache>/models--org--name/snapshots/*``,
    sentence-transformers' ``<cache>/sentence-transformers_<name>``), or the default hub cache.
    There is no download path: a model that is not on disk is an error."""
    cands = [Path(model_name)]
    roots = [Path(cache_dir)] if cache_dir else []
    roots.append(Path.home() / ".cache" / "huggingface" / "hub")
    for r in roots:
        cands += [r / model_name, r / Path(model_name).name]
        hub = r / ("models--" + model_name.replace("/", "--")) / "snapshots"
        if hub.is_dir():
            cands += sorted(hub.iterdir(), reverse=True)
        cands.append(r / ("sentence-transformers_" + Path(model_name).name))
    for c in cands:
        if (c / "config.json").exists() and any(c.glob("*.safetensors")):
            return c
    raise FileNotFoundError(f"model {model_name!r} not found locally (looked in {[str(c) for c in cands[:6]]}); "
                            "place the safetensors checkpoint there -- this deployment does not download models")


class HuggingFaceEmbeddingProvider(HipEncoderProvider):
    """The reference's ``huggingface`` backend (huggingface_provider.py:15-101: AutoModel, truncation
    to ``max_length`` 512, mean of the last hidden state, no normalisation) with the checkpoint run
    on the HIP encoder.  Sequences are varlen-packed, so the mean covers exactly each text's tokens:
    the reference's per-text (unpadded) result."""
    backend = "huggingface"

    def __init__(self, model_name="sentence-transformers/all-MiniLM-L6-v2", device="cuda", max_length=512,
                 cache_dir=None, **kw):
        d = resolve_model_dir(model_name, cache_dir)
        super().__init__(model_name=model_name, checkpoint_dir=str(d), device=device, pooling="mean",
                         normalize=False, max_length=max_length, **kw)


class SentenceTransformerProvider(EmbeddingProvider):
    """The reference's default ``sentencetransformers`` backend (sentence_transformer_provider.py:
    15-93).  With the sentence-transformers package installed it is used as is; without it (this
    image) the model directory is read natively -- modules.json (Transformer -> Pooling [->
    Normalize]), 1_Pooling/config.json (mean / CLS) and sentence_bert_config.json (max_seq_length)
    -- and served by the HIP encoder."""
    backend = "sentencetransformers"

    def __init__(self, model_name="all-MiniLM-L6-v2", device="cuda", cache_dir=None, **kw):
        try:
            from sentence_transformers import SentenceTransformer  # type: ignore
        except ImportError:
            SentenceTransformer = None
        self.model_name = model_name
        self.st = self.hip = None
        if SentenceTransformer is not None:  # pragma: no cover - package absent in this image
            self.st = SentenceTransformer(model_name, device=device, cache_folder=cache_dir)
            self.dimension = self.st.get_sentence_embedding_dimension()
            return
        name = model_name if "/" in model_name or Path(model_name).is_dir() else f"sentence-transformers/{model_name}"
        d = resolve_model_dir(name, cache_dir)
        pooling, normalize, max_len = "mean", False, None
        mods = json.loads((d / "modules.json").read_text()) if (d / "modules.json").exists() else []
        for m in mods:
            kind = m.get("type", "")
            if kind.endswith("Pooling"):
                pc = json.loads((d / m["path"] / "config.json").read_text())
                if pc.get("pooling_mode_cls_token"):
                    pooling = "cls"
                elif not pc.get("pooling_mode_mean_tokens", True):
                    raise ValueError(f"{d}: only mean / CLS pooling are supported")
            elif kind.endswith("Normalize"):
                normalize = True
        if (d / "sentence_bert_config.json").exists():
            max_len = json.loads((d / "sentence_bert_config.json").read_text()).get("max_seq_length")
        self.hip = HipEncoderProvider(model_name=model_name, checkpoint_dir=str(d), device=device, pooling=pooling,
                                      normalize=normalize, max_length=max_len, **kw)
        self.dimension = self.hip.dimension

    def embed(self, text):
        _check_text(text)
        if self.st is not None:  # pragma: no cover
            return self.st.encode(text).tolist()
        return self.hip.embed(text)

    def embed_batch(self, texts):
        return self.hip.embed_batch(texts) if self.hip is not None else [self.embed(t) for t in texts]

    def embed_tensor(self, texts):
        return self.hip.embed_tensor(texts) if self.hip is not None else super().embed_tensor(texts)


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
    name = str(getattr(cfg, "driver_name", cfg) or "hip").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name == "hip":
        return HipEncoderProvider(**kw)
    if name == "mock":
        return MockEmbeddingProvider(**kw)
    if name == "sentencetransformers":
        return SentenceTransformerProvider(**kw)
    if name == "huggingface":
        return HuggingFaceEmbeddingProvider(**kw)
    if name in ("openai", "azure_openai"):
        return OpenAIEmbeddingProvider(**kw)
    raise ValueError(f"unknown embedding backend {name!r}")


__all__ = ["EmbeddingProvider", "MockEmbeddingProvider", "HipEncoderProvider", "HuggingFaceEmbeddingProvider",
           "SentenceTransformerProvider", "OpenAIEmbeddingProvider", "resolve_model_dir", "create_embedding_provider"]
