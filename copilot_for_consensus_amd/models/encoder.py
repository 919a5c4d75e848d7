"""BERT-family sentence encoder (all-MiniLM-L6-v2, bge-small/base) for the embedding service.

Replaces ``SentenceTransformer(model).encode(text)`` (adapters/copilot_embedding/copilot_embedding/
sentence_transformer_provider.py:50,93) and the HF ``AutoModel`` mean-pool provider
(huggingface_provider.py:44,98-101).  The reference embeds ONE chunk per call
(embedding/app/service.py:384-393); this encoder runs packed varlen batches (no padding) of
hundreds of chunks per forward:

    embed gather + pos + type + LayerNorm       (1 HIP kernel)
    per layer: QKV GEMM(+bias)  -> varlen bidirectional MFMA attention (HIP)
               O GEMM -> bias + residual + LayerNorm (HIP)
               FFN-up GEMM -> bias + GELU (HIP) -> FFN-down GEMM -> bias + residual + LN (HIP)
    masked mean / CLS pooling + L2 normalise    (1 HIP kernel)
"""
from __future__ import annotations

import dataclasses
import math
import os
from pathlib import Path

import torch
import torch.nn.functional as F

from ..ops import kernels as K


@dataclasses.dataclass(frozen=True)
class EncoderConfig:
    name: str
    vocab_size: int = 30522
    hidden: int = 384
    layers: int = 6
    heads: int = 12
    ffn: int = 1536
    max_positions: int = 512
    max_seq_length: int = 256     # sentence-transformers truncation length
    ln_eps: float = 1e-12
    pooling: str = "mean"         # "mean" (MiniLM) or "cls" (BGE)
    normalize: bool = True

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


ENCODER_PRESETS = {
    "minilm-l6": EncoderConfig("all-MiniLM-L6-v2"),
    "all-MiniLM-L6-v2": EncoderConfig("all-MiniLM-L6-v2"),
    "bge-small": EncoderConfig("bge-small-en-v1.5", layers=12, max_seq_length=512, pooling="cls"),
    "bge-base": EncoderConfig("bge-base-en-v1.5", hidden=768, layers=12, heads=12, ffn=3072, max_seq_length=512,
                              pooling="cls"),
    "tiny": EncoderConfig("tiny", vocab_size=1000, hidden=64, layers=2, heads=2, ffn=128, max_positions=512,
                          max_seq_length=128),
}


def encoder_config_from_hf(config_json, name: str | None = None, **over) -> EncoderConfig:
    """EncoderConfig from an HF BertConfig ``config.json`` (BERT / MiniLM / BGE checkpoints)."""
    import json
    c = json.loads(Path(config_json).read_text())
    if c.get("model_type", "bert") not in ("bert", "xlm-roberta", "roberta") and "hidden_size" not in c:
        raise ValueError(f"{config_json}: not a BERT-family config")
    kw = dict(vocab_size=int(c["vocab_size"]), hidden=int(c["hidden_size"]), layers=int(c["num_hidden_layers"]),
              heads=int(c["num_attention_heads"]), ffn=int(c["intermediate_size"]),
              max_positions=int(c.get("max_position_embeddings", 512)), ln_eps=float(c.get("layer_norm_eps", 1e-12)),
              max_seq_length=min(512, int(c.get("max_position_embeddings", 512))))
    kw.update(over)
    return EncoderConfig(name or Path(config_json).parent.name, **kw)


def get_encoder_config(name) -> EncoderConfig:
    if isinstance(name, EncoderConfig):
        return name
    key = name.split("/")[-1]
    if key not in ENCODER_PRESETS:
        raise KeyError(f"unknown encoder {name!r}; known: {sorted(ENCODER_PRESETS)}")
    return ENCODER_PRESETS[key]


class EncoderModel:
    def __init__(self, cfg: EncoderConfig, device, dtype=torch.bfloat16):
        self.cfg, self.device, self.dtype = get_encoder_config(cfg), torch.device(device), dtype
        self.p: dict[str, torch.Tensor] = {}
        self.layers: list[dict[str, torch.Tensor]] = []
        self.scale = 1.0 / math.sqrt(self.cfg.head_dim)

    @classmethod
    def random(cls, cfg, device, seed: int = 0, std: float = 0.02):
        m = cls(get_encoder_config(cfg), device)
        c = m.cfg
        gen = torch.Generator(device=m.device)
        gen.manual_seed(seed)

        def rnd(*shape):
            t = torch.empty(*shape, dtype=m.dtype, device=m.device)
            return t.normal_(0.0, std, generator=gen)

        def ones(n):
            return torch.ones(n, dtype=m.dtype, device=m.device)

        def zeros(n):
            return torch.zeros(n, dtype=m.dtype, device=m.device)

        h, f = c.hidden, c.ffn
        m.p = {"word": rnd(c.vocab_size, h), "pos": rnd(c.max_positions, h), "type": rnd(2, h),
               "emb_g": ones(h), "emb_b": zeros(h)}
        for _ in range(c.layers):
            m.layers.append({"qkv": rnd(3 * h, h), "qkv_b": zeros(3 * h), "o": rnd(h, h), "o_b": zeros(h),
                             "ln1_g": ones(h), "ln1_b": zeros(h), "up": rnd(f, h), "up_b": zeros(f),
                             "down": rnd(h, f), "down_b": zeros(h), "ln2_g": ones(h), "ln2_b": zeros(h)})
        return m

    @classmethod
    def from_safetensors(cls, cfg, ckpt_dir, device):
        """Load an HF BertModel checkpoint (``model.safetensors``)."""
        from safetensors import safe_open

        m = cls(get_encoder_config(cfg), device)
        files = sorted(Path(ckpt_dir).glob("*.safetensors"))
        t = {}
        for fpath in files:
            with safe_open(str(fpath), framework="pt", device="cpu") as fh:
                for k in fh.keys():
                    t[k.removeprefix("bert.")] = fh.get_tensor(k)

        def d(x):
            return x.to(device=m.device, dtype=m.dtype).contiguous()

        m.p = {"word": d(t["embeddings.word_embeddings.weight"]), "pos": d(t["embeddings.position_embeddings.weight"]),
               "type": d(t["embeddings.token_type_embeddings.weight"]), "emb_g": d(t["embeddings.LayerNorm.weight"]),
               "emb_b": d(t["embeddings.LayerNorm.bias"])}
        for i in range(m.cfg.layers):
            p = f"encoder.layer.{i}."
            a = p + "attention."
            m.layers.append({
                "qkv": d(torch.cat([t[a + "self.query.weight"], t[a + "self.key.weight"], t[a + "self.value.weight"]])),
                "qkv_b": d(torch.cat([t[a + "self.query.bias"], t[a + "self.key.bias"], t[a + "self.value.bias"]])),
                "o": d(t[a + "output.dense.weight"]), "o_b": d(t[a + "output.dense.bias"]),
                "ln1_g": d(t[a + "output.LayerNorm.weight"]), "ln1_b": d(t[a + "output.LayerNorm.bias"]),
                "up": d(t[p + "intermediate.dense.weight"]), "up_b": d(t[p + "intermediate.dense.bias"]),
                "down": d(t[p + "output.dense.weight"]), "down_b": d(t[p + "output.dense.bias"]),
                "ln2_g": d(t[p + "output.LayerNorm.weight"]), "ln2_b": d(t[p + "output.LayerNorm.bias"]),
            })
        return m

    # ------------------------------------------------------------------ forward
    def forward_packed(self, ids: torch.Tensor, positions: torch.Tensor, cu_seqlens: torch.Tensor, max_seqlen: int,
                       tiles=None) -> torch.Tensor:
        """Token states [T, H] for packed varlen input."""
        c = self.cfg
        x = K.embed_layernorm(ids, positions, self.p["word"], self.p["pos"], self.p["type"], self.p["emb_g"],
                              self.p["emb_b"], c.ln_eps)
        lin = self._linear
        for lw in self.layers:
            qkv = lin(x, lw["qkv"], "bias", lw["qkv_b"])
            a = K.encoder_attention(qkv, cu_seqlens, c.heads, c.head_dim, self.scale, max_seqlen, tiles=tiles)
            x = self._linear_ln(a.view(a.shape[0], -1), lw["o"], lw["o_b"], x, lw["ln1_g"], lw["ln1_b"])
            h = lin(x, lw["up"], "bias_gelu", lw["up_b"])
            x = self._linear_ln(h, lw["down"], lw["down_b"], x, lw["ln2_g"], lw["ln2_b"])
        return x

    # projection GEMMs: the hand-written pgemm (csrc/kernels/pgemm.hip, bias / bias+GELU fused in
    # its epilogue) where it measured at or above hipBLASLt -- the small-K (K <= 512) shapes of the
    # MiniLM-class encoders (profiles/r03_pgemm_v1_vs_hipblaslt.log); the library GEMM for K >= 768
    # (BGE-base).  Re-measured in round 5 with the decoder's ping-pong kernels in the race
    # (profiles/r05_pgemm_encoder_variants.jsonl, 32k rows): MiniLM qkv+bias 442 TF/s (2-stage) vs
    # 433 library, up+GELU 426 vs 407 -- the ping-pong variants lose there (313 / 287: K = 384 is six
    # K-tiles, too short for their pipeline); BGE-base qkv+bias 746 vs 938 library, up+GELU 668 vs
    # 675, down 1166 (pps) vs 1195 -- so the K <= 512 threshold stands.
    # CFC_ENCODER_GEMM = auto | hip | lib.
    PGEMM_MAX_K = 512

    def _linear(self, x, w, epi: str = "bf16", bias=None):
        mode = os.environ.get("CFC_ENCODER_GEMM", "auto")
        use = x.is_cuda and K.pgemm_ok(x, w) and (mode == "hip" or (mode == "auto" and w.shape[1] <= self.PGEMM_MAX_K))
        if use:
            return K.pgemm(x, w, epi, bias=bias)
        y = F.linear(x, w, bias if epi == "bias" else None)
        return K.bias_gelu(y, bias) if epi == "bias_gelu" else y

    def _linear_ln(self, x, w, bias, residual, gamma, beta):
        """LayerNorm(x @ w^T + bias + residual): one fused kernel (pgemm_ln: the row statistics
        reduced inside the workgroup that owns the whole row) for the hidden sizes it is built for
        (384), else the projection then the residual + LayerNorm kernel.  CFC_ENCODER_LN_FUSED=0
        forces the unfused path."""
        eps = self.cfg.ln_eps
        if (x.is_cuda and os.environ.get("CFC_ENCODER_LN_FUSED", "1") != "0"
                and os.environ.get("CFC_ENCODER_GEMM", "auto") != "lib" and K.pgemm_ln_ok(x, w)):
            return K.pgemm_ln(x, w, bias, residual, gamma, beta, eps)
        return K.layernorm(self._linear(x, w), gamma, beta, eps, bias=bias, residual=residual)

    @torch.inference_mode()
    def encode_ids(self, batch: list[list[int]], pooling: str | None = None, normalize: bool | None = None,
                   max_tokens_per_forward: int = 65536) -> torch.Tensor:
        """Sentence embeddings [n, H] fp32 for pre-tokenised sequences (truncated to max_seq_length)."""
        import numpy as np
        seqs = [s[:self.cfg.max_seq_length] for s in batch]
        cu = np.zeros(len(seqs) + 1, dtype=np.int32)
        np.cumsum([len(s) for s in seqs], out=cu[1:])
        ids = np.fromiter((t for s in seqs for t in s), dtype=np.int32, count=int(cu[-1]))
        return self.encode_packed(ids, cu, pooling, normalize, max_tokens_per_forward)

    @torch.inference_mode()
    def encode_packed(self, ids, cu_seqlens, pooling: str | None = None, normalize: bool | None = None,
                      max_tokens_per_forward: int = 65536) -> torch.Tensor:
        """Sentence embeddings [n, H] fp32 for sequences already packed (numpy int32 ``ids`` [T],
        ``cu_seqlens`` [n+1], each at most max_seq_length long): positions, forward groups and the
        device copies are built with array operations, no per-token Python."""
        import numpy as np
        c = self.cfg
        pooling = pooling or c.pooling
        normalize = c.normalize if normalize is None else normalize
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        cu = np.ascontiguousarray(cu_seqlens, dtype=np.int64)
        lens = np.diff(cu)
        if len(lens) and int(lens.max()) > c.max_seq_length:
            raise ValueError(f"sequence of {int(lens.max())} tokens > max_seq_length {c.max_seq_length}")
        pos_all = (np.arange(int(cu[-1]), dtype=np.int64) - np.repeat(cu[:-1], lens)).astype(np.int32)
        dev = self.device
        outs = []
        i, n = 0, len(lens)
        while i < n:
            # as many whole sequences as fit in max_tokens_per_forward (at least one)
            j = int(np.searchsorted(cu, cu[i] + max_tokens_per_forward, side="right")) - 1
            j = min(max(j, i + 1), n)
            t0, t1 = int(cu[i]), int(cu[j])
            cu_part = (cu[i:j + 1] - t0).astype(np.int32)
            seq_t, q0_t = K.prefill_tiles(cu_part.tolist(), K.ENCODER_TILE_ROWS)
            tiles = (torch.tensor(seq_t, dtype=torch.int32, device=dev), torch.tensor(q0_t, dtype=torch.int32, device=dev))
            cu_t = torch.from_numpy(cu_part).to(dev)
            h = self.forward_packed(torch.from_numpy(ids[t0:t1]).to(dev), torch.from_numpy(pos_all[t0:t1]).to(dev),
                                    cu_t, int(lens[i:j].max()), tiles=tiles)
            outs.append(K.pool(h, cu_t, pooling, normalize))
            i = j
        return torch.cat(outs, 0)
