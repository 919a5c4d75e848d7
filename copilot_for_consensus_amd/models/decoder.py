"""Mistral / Llama decoder (the summarization LLM).

Replaces the LLM the reference reaches over HTTP (Ollama ``/api/generate``,
adapters/copilot_summarization/copilot_summarization/local_llm_summarizer.py:107; llama.cpp
``/completion``, llamacpp_summarizer.py:108; model ``mistral-7b-instruct-v0.2``,
docker-compose.infra.yml:296-298).  Inference only.

MI355X layout choices:
  * fused weights: one QKV projection [(Hq+2Hkv)*D, H], one gate|up projection [2F, H] (gate and
    up rows interleaved in 8-row groups), so a layer is 4 GEMMs + RoPE/paged-KV write + attention
    + 2 fused split-K-reduce/residual/RMSNorm kernels;
  * decode (B > 4) projections on the hand-written weight-streaming MFMA GEMM (csrc/kernels/
    dgemm.hip) with SwiGLU in the gate/up epilogue; B <= 4 on the GEMV; prefill on the hand-written
    ping-pong MFMA GEMM (pgemm.hip) reading the same fragment-packed weights (one copy);
  * tensor parallel (Megatron column/row split) with one all-reduce after o_proj and one after
    down_proj, vocab-parallel lm_head + all-gather of logits -- see :mod:`..parallel.tp`;
  * weights random-initialised directly on the device (no network: BASELINE "random-init
    weights"), or loaded from HF-style safetensors when a checkpoint directory is given.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from pathlib import Path

import torch
import torch.nn.functional as F

from ..ops import kernels as K
from ..ops.reference import interleave_gate_up, rope_cos_sin


@dataclasses.dataclass(frozen=True)
class DecoderConfig:
    name: str
    vocab_size: int
    hidden: int
    layers: int
    heads: int
    kv_heads: int
    head_dim: int
    ffn: int
    rope_theta: float = 10000.0
    rms_eps: float = 1e-5
    max_positions: int = 32768
    tie_embeddings: bool = False
    bos_id: int = 1
    eos_id: int = 2
    # Llama-3.1 RoPE frequency scaling: (factor, low_freq_factor, high_freq_factor, original_max_positions)
    rope_llama3: tuple | None = None
    # sliding-window attention (Mistral v0.1: 4096): a token sees the previous `sliding_window` positions
    sliding_window: int | None = None

    @property
    def q_size(self) -> int:
        return self.heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.kv_heads * self.head_dim

    def num_params(self) -> int:
        h, f, v = self.hidden, self.ffn, self.vocab_size
        per_layer = h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * f + 2 * h
        return self.layers * per_layer + v * h * (1 if self.tie_embeddings else 2) + h

    def flops_per_token(self, ctx: int = 0) -> float:
        """Dense GEMM flops per token (+ attention over ``ctx`` keys)."""
        h, f = self.hidden, self.ffn
        gemm = 2 * (h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * f)
        attn = 4 * self.heads * self.head_dim * ctx
        return self.layers * (gemm + attn) + 2 * h * self.vocab_size


PRESETS: dict[str, DecoderConfig] = {
    # mistral-7b-instruct-v0.2 (what docker-compose.infra.yml:296 serves): no sliding window, theta 1e6
    "mistral-7b": DecoderConfig("mistral-7b", 32000, 4096, 32, 32, 8, 128, 14336, rope_theta=1e6,
                                max_positions=32768),
    # mistral-7b v0.1: sliding-window attention over 4096 positions, theta 1e4
    "mistral-7b-v0.1": DecoderConfig("mistral-7b-v0.1", 32000, 4096, 32, 32, 8, 128, 14336, rope_theta=1e4,
                                     max_positions=32768, sliding_window=4096),
    "llama-3-8b": DecoderConfig("llama-3-8b", 128256, 4096, 32, 32, 8, 128, 14336, rope_theta=5e5,
                                max_positions=8192, bos_id=128000, eos_id=128009),
    "llama-3-70b": DecoderConfig("llama-3-70b", 128256, 8192, 80, 64, 8, 128, 28672, rope_theta=5e5,
                                 max_positions=8192, bos_id=128000, eos_id=128009),
    # Llama-2 7B / 13B (the reference's Ollama / llama.cpp docs quote decode speeds for both:
    # docs/operations/ollama-gpu-setup.md:151-152, docs/operations/llm-gpu-setup.md:467,476).
    # Plain multi-head attention: kv_heads == heads, i.e. G = 1 in the GQA-packed prefill kernel.
    "llama-2-7b": DecoderConfig("llama-2-7b", 32000, 4096, 32, 32, 32, 128, 11008, rope_theta=1e4,
                                max_positions=4096),
    "llama-2-13b": DecoderConfig("llama-2-13b", 32000, 5120, 40, 40, 40, 128, 13824, rope_theta=1e4,
                                 max_positions=4096),
    # small configs for tests / smoke runs
    "tiny-mha": DecoderConfig("tiny-mha", 512, 256, 2, 2, 2, 128, 512, rope_theta=1e4, max_positions=4096),
    "tiny": DecoderConfig("tiny", 512, 256, 2, 4, 2, 128, 512, rope_theta=1e4, max_positions=4096),
    "small": DecoderConfig("small", 32000, 1024, 4, 8, 2, 128, 2816, rope_theta=1e6, max_positions=8192),
    # Mistral / Llama-3-8B's head layout (32 q / 8 kv, head_dim 128) at GPU-test size: TP=8 leaves one
    # kv head per rank and every per-rank projection still fits the decode / prefill GEMMs (N, K % 64)
    "tiny-gqa8": DecoderConfig("tiny-gqa8", 32768, 1024, 2, 32, 8, 128, 2048, rope_theta=1e6,
                               max_positions=4096),
    # Llama-3-70B's head layout (64 q / 8 kv heads: TP=8 leaves ONE kv head per rank) at CPU-test
    # size, for the TP=4 / TP=8 shard paths on gloo (tests/test_tp_wide_cpu.py)
    "tiny-70b-heads": DecoderConfig("tiny-70b-heads", 512, 512, 2, 64, 8, 32, 1024, rope_theta=5e5,
                                    max_positions=4096),
}


def get_config(name_or_cfg) -> DecoderConfig:
    if isinstance(name_or_cfg, DecoderConfig):
        return name_or_cfg
    if name_or_cfg not in PRESETS:
        raise KeyError(f"unknown decoder preset {name_or_cfg!r}; known: {sorted(PRESETS)}")
    return PRESETS[name_or_cfg]


class DecoderWeights:
    """Per-rank (TP-sharded) weights, all bf16 on one device."""

    def __init__(self, cfg: DecoderConfig, device, tp_rank: int = 0, tp_size: int = 1, dtype=torch.bfloat16):
        if cfg.heads % tp_size or cfg.kv_heads % tp_size or cfg.ffn % tp_size or cfg.vocab_size % tp_size:
            raise ValueError(f"{cfg.name}: heads/kv_heads/ffn/vocab must divide tp_size={tp_size}")
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.heads = cfg.heads // tp_size
        self.kv_heads = cfg.kv_heads // tp_size
        self.ffn = cfg.ffn // tp_size
        self.vocab_shard = cfg.vocab_size // tp_size
        self.layers: list[dict[str, torch.Tensor]] = []
        # gate_up rows: [gate; up] (False) or 8-row interleaved groups (True, see interleave_gate_up)
        self.gate_up_interleaved = False
        self.embed: torch.Tensor | None = None
        self.final_norm: torch.Tensor | None = None
        self.lm_head: torch.Tensor | None = None
        # ggml-quantized copies of the projections for the B <= 4 decode GEMV (GGUF checkpoints)
        self.qlayers: list[dict] | None = None
        self.q_lm_head = None
        # opt-in W8A8 FP8 projections (e4m3fn + per-output-channel scales): to_fp8()
        self.fp8_layers: list[dict] | None = None
        # second copies of the decode projections in the decode GEMM's fragment-packed layout
        # (K.PackedWeight): pack_decode()
        self.packed: list[dict] | None = None
        self.packed_lm_head = None
        self.packed_only = False      # row-major projections dropped after packing
        self.cos_sin = rope_cos_sin(cfg.max_positions, cfg.head_dim, cfg.rope_theta, device=self.device,
                                    llama3_scaling=cfg.rope_llama3)

    # ---------------------------------------------------------------- init
    @classmethod
    def random(cls, cfg, device, seed: int = 0, tp_rank: int = 0, tp_size: int = 1, std: float = 0.02):
        w = cls(cfg, device, tp_rank, tp_size)
        gen = torch.Generator(device=w.device)
        gen.manual_seed(seed * 1000003 + tp_rank)
        D = cfg.head_dim

        # replicated tensors come from a rank-independent stream so every TP rank holds the same copy
        gen_rep = torch.Generator(device=w.device)
        gen_rep.manual_seed(seed * 1000003 + 999983)

        def rnd(*shape, scale=std, g=gen):
            t = torch.empty(*shape, dtype=w.dtype, device=w.device)
            t.normal_(0.0, scale, generator=g)
            return t

        h = cfg.hidden
        out_std = std / math.sqrt(2 * cfg.layers)
        for _ in range(cfg.layers):
            w.layers.append({
                "attn_norm": torch.ones(h, dtype=w.dtype, device=w.device),
                "qkv": rnd((w.heads + 2 * w.kv_heads) * D, h),
                "o": rnd(h, w.heads * D, scale=out_std),
                "mlp_norm": torch.ones(h, dtype=w.dtype, device=w.device),
                "gate_up": rnd(2 * w.ffn, h),
                "down": rnd(h, w.ffn, scale=out_std),
            })
        w.embed = rnd(cfg.vocab_size, h, scale=1.0, g=gen_rep)  # embeddings replicated (gather is cheap)
        w.final_norm = torch.ones(h, dtype=w.dtype, device=w.device)
        w.lm_head = rnd(w.vocab_shard, h)
        return w.finalize()

    @classmethod
    def from_safetensors(cls, cfg, ckpt_dir, device, tp_rank: int = 0, tp_size: int = 1):
        """Load HF Llama/Mistral safetensors (``model.layers.N.self_attn.q_proj.weight`` names)."""
        from safetensors import safe_open

        w = cls(cfg, device, tp_rank, tp_size)
        files = sorted(Path(ckpt_dir).glob("*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no *.safetensors in {ckpt_dir}")
        tensors = {}
        for f in files:
            with safe_open(str(f), framework="pt", device="cpu") as fh:
                for k in fh.keys():
                    tensors[k] = fh.get_tensor(k)
        D = cfg.head_dim

        def shard_rows(t, n):
            return t.view(tp_size, n, *t.shape[1:])[tp_rank] if tp_size > 1 else t

        def shard_cols(t, n):
            return t.view(t.shape[0], tp_size, n)[:, tp_rank].contiguous() if tp_size > 1 else t

        def dev(t):
            return t.to(device=w.device, dtype=w.dtype).contiguous()

        for i in range(cfg.layers):
            p = f"model.layers.{i}."
            q = shard_rows(tensors[p + "self_attn.q_proj.weight"], w.heads * D)
            k = shard_rows(tensors[p + "self_attn.k_proj.weight"], w.kv_heads * D)
            v = shard_rows(tensors[p + "self_attn.v_proj.weight"], w.kv_heads * D)
            g = shard_rows(tensors[p + "mlp.gate_proj.weight"], w.ffn)
            u = shard_rows(tensors[p + "mlp.up_proj.weight"], w.ffn)
            w.layers.append({
                "attn_norm": dev(tensors[p + "input_layernorm.weight"]),
                "qkv": dev(torch.cat([q, k, v], 0)),
                "o": dev(shard_cols(tensors[p + "self_attn.o_proj.weight"], w.heads * D)),
                "mlp_norm": dev(tensors[p + "post_attention_layernorm.weight"]),
                "gate_up": dev(torch.cat([g, u], 0)),
                "down": dev(shard_cols(tensors[p + "mlp.down_proj.weight"], w.ffn)),
            })
        w.embed = dev(tensors["model.embed_tokens.weight"])
        w.final_norm = dev(tensors["model.norm.weight"])
        head = tensors.get("lm_head.weight", tensors["model.embed_tokens.weight"])
        w.lm_head = dev(shard_rows(head, w.vocab_shard))
        return w.finalize()

    @classmethod
    def from_gguf(cls, path, device, cfg=None, quantized_decode: bool = True):
        """Load a llama-architecture GGUF (llama.cpp / Ollama files: Mistral, Llama).  Every tensor
        is dequantized to bf16 (GPU kernel on CUDA devices) for the batched paths; with
        ``quantized_decode`` the Q4_K / Q6_K / Q8_0 projection weights are ALSO kept in their
        block format for the B <= 4 decode GEMV (``qlayers`` / ``q_lm_head``).  q/k rows are
        un-permuted from llama.cpp's interleaved-RoPE order to this framework's rotate-half order.
        TP is not supported for GGUF checkpoints (one GPU holds any GGUF model)."""
        from ..ops.kernels import QGEMV_TYPES, QWeight, dequant_bf16
        from ..runtime import gguf as G

        r = G.GGUFReader(path)
        cfg = cfg or G.config_from_gguf(r.metadata, tensor_names=r.tensors.keys(), name=Path(path).stem)
        w = cls(cfg, device)
        D = cfg.head_dim
        qrows = G.unpermute_qk_rows(cfg.heads * D, cfg.heads)
        krows = G.unpermute_qk_rows(cfg.kv_heads * D, cfg.kv_heads)

        def info(name):
            if name not in r.tensors:
                raise KeyError(f"{path}: tensor {name} missing")
            return r.tensors[name]

        def bf16(name, rows=None):
            ti = info(name)
            t = dequant_bf16(ti.data, ti.ggml_type, ti.shape, w.device)
            if rows is not None:
                t = t.index_select(0, torch.as_tensor(rows, device=t.device))
            return t.contiguous()

        def quant(name, rows=None):
            ti = info(name)
            if not quantized_decode or ti.ggml_type not in QGEMV_TYPES or len(ti.shape) != 2:
                return None
            N, Kd = ti.shape
            return QWeight.from_raw(ti.data, ti.ggml_type, N, Kd, w.device, rows=rows)

        qlayers = []
        for i in range(cfg.layers):
            p = f"blk.{i}."
            q, k, v = bf16(p + "attn_q.weight", qrows), bf16(p + "attn_k.weight", krows), bf16(p + "attn_v.weight")
            w.layers.append({
                "attn_norm": bf16(p + "attn_norm.weight"),
                "qkv": torch.cat([q, k, v], 0).contiguous(),
                "o": bf16(p + "attn_output.weight"),
                "mlp_norm": bf16(p + "ffn_norm.weight"),
                "gate_up": torch.cat([bf16(p + "ffn_gate.weight"), bf16(p + "ffn_up.weight")], 0).contiguous(),
                "down": bf16(p + "ffn_down.weight"),
            })
            qlayers.append({"q": quant(p + "attn_q.weight", qrows), "k": quant(p + "attn_k.weight", krows),
                            "v": quant(p + "attn_v.weight"), "o": quant(p + "attn_output.weight"),
                            "gate": quant(p + "ffn_gate.weight"), "up": quant(p + "ffn_up.weight"),
                            "down": quant(p + "ffn_down.weight")})
        w.embed = bf16("token_embd.weight")
        w.final_norm = bf16("output_norm.weight")
        head = "output.weight" if "output.weight" in r.tensors else "token_embd.weight"
        w.lm_head = w.embed if head == "token_embd.weight" else bf16(head)
        if quantized_decode:
            w.qlayers = qlayers
            w.q_lm_head = quant(head)
        w.gguf_types = sorted({t.type_name for t in r.tensors.values()})
        return w.finalize()

    def finalize(self) -> "DecoderWeights":
        """Put gate/up rows in the 8-row interleaved order the fused decode SwiGLU GEMM reads (the
        prefill path's silu_mul reads the same layout, so one copy of the weights serves both)."""
        if not self.gate_up_interleaved and self.ffn % 8 == 0:
            for layer in self.layers:
                layer["gate_up"] = interleave_gate_up(layer["gate_up"])
            self.gate_up_interleaved = True
        return self

    FP8_PROJECTIONS = ("qkv", "o", "gate_up", "down")

    def to_fp8(self, keep_bf16: bool = False) -> "DecoderWeights":
        """Opt-in W8A8 FP8 (OCP e4m3fn, gfx950 MFMA FP8): every projection quantised once with
        per-output-channel scales; activations are quantised per token at run time
        (ops.kernels.linear_fp8).  A precision trade-off like llama.cpp's Q8_0 / the reference's
        Q4_K_M deployment -- not the bf16 headline.  The bf16 copies are dropped unless ``keep_bf16``;
        norms, embeddings and the lm_head stay bf16."""
        self.fp8_layers = []
        for layer in self.layers:
            q = {}
            for name in self.FP8_PROJECTIONS:
                q[name] = K.quant_fp8_weight(layer[name])
                if not keep_bf16:
                    layer[name] = None
            self.fp8_layers.append(q)
        if not keep_bf16 and self.device.type == "cuda":
            torch.cuda.empty_cache()
        return self

    DECODE_PACKED = ("qkv", "o", "gate_up", "down")

    def packed_bytes(self) -> int:
        """HBM a pack_decode() adds (the projections + the lm_head, bf16)."""
        n = sum(layer[k].numel() * 2 for layer in self.layers for k in self.DECODE_PACKED if layer.get(k) is not None)
        return n + (self.lm_head.numel() * 2 if self.lm_head is not None else 0)

    def pack_decode(self, m: int = 128, drop_rowmajor: bool = False) -> "DecoderWeights":
        """Copy every projection (and the lm_head) into the decode GEMM's fragment-packed layout,
        tiled for an m-row batch (K.pack_dgemm_weight: each 16-row x 32-k MFMA fragment 1 KB
        contiguous, each workgroup's slice one contiguous span -- the flat stream runs at ~5.8 TB/s
        where row-major fragments read at 4-5).  The prefill GEMM (pgemm.hip) reads the same packed
        copy.  ``drop_rowmajor``: free each row-major projection as soon as its packed copy exists
        (one weight copy; peak HBM = the weights + one layer), otherwise both stay (the row-major
        one for the B <= 4 GEMV and the library paths; packed_bytes() more HBM)."""
        if self.packed is not None:
            return self
        self.packed = []
        for layer in self.layers:
            self.packed.append({k: K.pack_dgemm_weight(layer[k], swiglu=k == "gate_up", m=m)
                                for k in self.DECODE_PACKED})
            if drop_rowmajor:
                for k in self.DECODE_PACKED:
                    layer[k] = None
        self.packed_only = bool(drop_rowmajor)
        head = self.lm_head
        if head is not None and head.shape[0] % 64 == 0 and head.shape[1] % 64 == 0:
            self.packed_lm_head = K.pack_dgemm_weight(head, m=m)
        if drop_rowmajor and self.device.type == "cuda":
            torch.cuda.empty_cache()
        return self

    def rowmajor_layer(self, i: int) -> dict[str, torch.Tensor]:
        """Layer i's tensors with every projection row-major (unpacked from the packed copy when the
        row-major one was dropped) -- for reference models and checkpoint export."""
        out = dict(self.layers[i])
        for k in self.DECODE_PACKED:
            if out.get(k) is None and self.packed is not None:
                out[k] = K._rowmajor(self.packed[i][k])
        return out

    def nbytes(self) -> int:
        n = sum(t.numel() * t.element_size() for layer in self.layers for t in layer.values() if t is not None)
        n += sum(p.nbytes() for layer in self.packed or [] for p in layer.values())
        n += self.packed_lm_head.nbytes() if self.packed_lm_head is not None else 0
        for q in self.fp8_layers or []:
            n += sum(a.numel() * a.element_size() + b.numel() * b.element_size() for a, b in q.values())
        return n + sum(t.numel() * t.element_size() for t in (self.embed, self.final_norm, self.lm_head))


def load_config_json(path) -> DecoderConfig:
    """DecoderConfig from an HF ``config.json`` (transformers 4.x ``rope_theta`` / ``rope_scaling``
    and 5.x ``rope_parameters`` spellings)."""
    c = json.loads(Path(path).read_text())
    rope = dict(c.get("rope_parameters") or {})
    scaling = c.get("rope_scaling") or (rope if rope.get("rope_type") not in (None, "default") else None)
    theta = c.get("rope_theta") or rope.get("rope_theta") or 10000.0
    llama3 = None
    if scaling:
        kind = scaling.get("rope_type") or scaling.get("type")
        if kind == "llama3":
            llama3 = (float(scaling["factor"]), float(scaling["low_freq_factor"]), float(scaling["high_freq_factor"]),
                      int(scaling["original_max_position_embeddings"]))
        elif kind not in (None, "default"):
            raise NotImplementedError(f"RoPE scaling {kind!r} is not supported")
    eos = c.get("eos_token_id", 2)
    window = c.get("sliding_window") if c.get("use_sliding_window", True) else None
    return DecoderConfig(
        name=c.get("_name_or_path", "hf"), vocab_size=c["vocab_size"], hidden=c["hidden_size"],
        layers=c["num_hidden_layers"], heads=c["num_attention_heads"],
        kv_heads=c.get("num_key_value_heads", c["num_attention_heads"]),
        head_dim=c.get("head_dim") or c["hidden_size"] // c["num_attention_heads"], ffn=c["intermediate_size"],
        rope_theta=float(theta), rms_eps=c.get("rms_norm_eps", 1e-5),
        max_positions=c.get("max_position_embeddings", 4096), tie_embeddings=c.get("tie_word_embeddings", False),
        bos_id=c.get("bos_token_id", 1) or 1, eos_id=eos if isinstance(eos, int) else eos[0], rope_llama3=llama3,
        sliding_window=int(window) if window else None)


DGEMM_MAX_ROWS = 256   # decode batches above this run the library GEMM (one 256-row tile per W pass)


def argmax_keys(local: torch.Tensor, offset: int) -> torch.Tensor:
    """Per row of a vocab shard's logits, (max logit, argmax) packed into ONE int64 whose signed
    order is (logit, -global index): the high word an order-preserving image of the fp32 maximum,
    the low word 0xffffffff - (offset + argmax).  The MAX over shards is then the global greedy
    token (smallest index on exact ties), so TP greedy decode reduces B int64 instead of
    all-gathering B x V logits."""
    v, i = local.float().max(dim=1)
    b = v.view(torch.int32).to(torch.int64)
    ku = torch.where(b >= 0, b + 2 ** 31, 2 ** 31 - 1 - (b & 0x7FFFFFFF))
    return ((ku - 2 ** 31) << 32) | (0xFFFFFFFF - (i.to(torch.int64) + offset))


class DecoderModel:
    """Stateless forward functions over :class:`DecoderWeights` + a paged KV cache."""

    def __init__(self, weights: DecoderWeights, tp_group=None, fused_decode: bool | None = None, custom_ar=None):
        self.w = weights
        self.cfg = weights.cfg
        self.tp_group = tp_group
        # validated one-shot IPC all-reduce (parallel/custom_ar.py) for decode-size tensors; RCCL otherwise
        self.custom_ar = custom_ar
        self.scale = 1.0 / math.sqrt(self.cfg.head_dim)
        self.window = int(self.cfg.sliding_window or 0)
        # decode GEMM mode (B > 4): "dgemm" = the hand-written weight-streaming MFMA GEMM with
        # SwiGLU fused into gate/up and split-K slabs reduced with residual + RMSNorm (default);
        # "splitk" = library GEMMs with o/down as batched split-K into the same reduce; "lib" =
        # plain library GEMMs + separate norm kernels
        mode = os.environ.get("CFC_DECODE_GEMM", "dgemm")
        if fused_decode is not None:
            mode = "dgemm" if fused_decode else "lib"
        if mode not in ("dgemm", "splitk", "lib"):
            raise ValueError(f"CFC_DECODE_GEMM={mode!r}: expected dgemm, splitk or lib")
        if mode == "dgemm" and not (weights.gate_up_interleaved and self._dgemm_shapes()):
            mode = "splitk"
        if weights.tp_size != 1 and mode == "splitk":
            mode = "lib"
        self.fp8 = weights.fp8_layers is not None
        if self.fp8:
            mode = "lib"          # W8A8: every projection through linear_fp8 (bf16 fused paths need bf16 weights)
        self.decode_gemm = mode
        # prefill GEMM (packed prompt rows): "hip" = the hand-written MFMA GEMM (csrc/kernels/pgemm.hip,
        # SwiGLU fused into gate/up, reading the packed weights), "lib" = the library GEMM + silu_mul
        # (CFC_PREFILL_GEMM); CFC_PGEMM_VARIANT picks pgemm's K loop (CFC_PGEMM_VARIANT_SWIGLU the
        # gate/up projection's, CFC_PGEMM_VARIANT when unset)
        pm = os.environ.get("CFC_PREFILL_GEMM", self.PREFILL_GEMM_DEFAULT)
        if pm not in ("hip", "lib"):
            raise ValueError(f"CFC_PREFILL_GEMM={pm!r}: expected hip or lib")
        self.prefill_gemm = "lib" if self.fp8 else pm
        self.pgemm_variant = os.environ.get("CFC_PGEMM_VARIANT", self.PGEMM_VARIANT_DEFAULT)
        self.pgemm_variant_swiglu = os.environ.get("CFC_PGEMM_VARIANT_SWIGLU", os.environ.get(
            "CFC_PGEMM_VARIANT", self.PGEMM_VARIANT_SWIGLU_DEFAULT))
        for var, v in (("CFC_PGEMM_VARIANT", self.pgemm_variant), ("CFC_PGEMM_VARIANT_SWIGLU", self.pgemm_variant_swiglu)):
            if v not in K.PGEMM_VARIANTS:
                raise ValueError(f"{var}={v!r}: expected one of {sorted(K.PGEMM_VARIANTS)}")
        # B <= 4 decode steps on the GEMV kernel (needs the interleaved gate/up layout for SwiGLU)
        gemv_shapes = (self.cfg.hidden % 8 == 0 and (weights.heads * self.cfg.head_dim) % 8 == 0
                       and weights.ffn % 8 == 0 and self.cfg.head_dim % 2 == 0)
        self.decode_gemv = (os.environ.get("CFC_DECODE_GEMV", "1") != "0" and weights.gate_up_interleaved
                            and mode in ("splitk", "dgemm") and weights.tp_size == 1 and gemv_shapes
                            and not self.fp8)
        self.fused_decode = mode == "dgemm"
        # decode RoPE + KV write inside the attention kernel's prologue: CFC_DECODE_ROPE_FUSED "1"
        # always, "0" never, unset: for B <= 4.  Measured in the headline (profiles/r04_ab_*.log) the
        # fused BATCHED step decodes slower (6.30 vs 6.09 s per batch): every attention workgroup
        # waits ~5 us for its q slabs, the RoPE and the K/V store before its first KV load, twice
        # per CU, which costs more than the 10.6-us rope_kv launch it removes.  At B = 1 the launch
        # is the larger cost: 296.5 -> 299.9 tok/s Mistral-7B (profiles/r04_latprof_*).
        self.rope_fused = os.environ.get("CFC_DECODE_ROPE_FUSED", "")
        # B <= 4 over packed weights: residual + RMSNorm folded into the next GEMV (K.gemv_norm).
        # Opt-in: bit-identical, two launches fewer per layer, but slower -- the prologue's slab reads
        # (written by another XCD, served from the MALL) stall the weight stream behind them:
        # Mistral-7B 307.7 vs 313.5 tok/s, Llama-2-13B 177.1 vs 190.9 (profiles/r04_gemv_norm_ab.log)
        self.gemv_norm_fused = os.environ.get("CFC_DECODE_GEMV_NORM", "0") == "1"
        # TP > 1: the row-parallel (o / down) partials are all-reduced in fp32 and rounded to bf16
        # ONCE, as TP = 1 rounds the full sum (CFC_TP_AR_DTYPE=fp32, default); "bf16" rounds each
        # rank's partial first and halves the prefill all-reduce bytes (round 5's behaviour).  The
        # batched decode always sums fp32 (one-shot kernel: latency-bound, bytes do not matter)
        ard = os.environ.get("CFC_TP_AR_DTYPE", "fp32")
        if ard not in ("fp32", "bf16"):
            raise ValueError(f"CFC_TP_AR_DTYPE={ard!r}: expected fp32 or bf16")
        self.tp_fp32 = weights.tp_size > 1 and ard == "fp32" and not (weights.fp8_layers is not None)
        # split-K of the batched qkv decode GEMM (its slabs feed rope_kv): 0 = the cost model's pick
        self.qkv_split = int(os.environ.get("CFC_DECODE_QKV_SPLIT", "0"))
        # B <= 4 decode on the ggml-quantized weights (GGUF checkpoints; csrc/kernels/quant.hip)
        self.decode_qgemv = (weights.qlayers is not None and os.environ.get("CFC_DECODE_QGEMV", "1") != "0"
                             and weights.tp_size == 1 and weights.gate_up_interleaved and not self.fp8)
        # packed weights (CFC_DECODE_PACKED: auto / 1 = pack, 0 = never): one fragment-packed copy read by
        # the decode GEMM and the prefill GEMM.  The row-major copies are dropped (CFC_WEIGHTS_PACKED_ONLY:
        # auto = when the decode and prefill both run on the packed copy, 1 = always, 0 = keep both)
        if (self.fused_decode or self.prefill_gemm == "hip") and weights.device.type == "cuda":
            pk = self._packing()
            if pk is not None:
                weights.pack_decode(drop_rowmajor=pk == "only")
        if weights.packed_only:
            # nothing may read the row-major projections any more (the B <= 4 GEMV reads the packed ones)
            self.decode_gemm = "dgemm"
            self.fused_decode = True
            self.prefill_gemm = "hip"

    PACKED_FREE_FRACTION = 0.3   # HBM left free after packing when both copies are kept
    PREFILL_GEMM_DEFAULT = "hip"
    # "ppp": the persistent ping-pong kernel (one workgroup per CU walking the tiles, the DMA
    # stream running on across tile boundaries, LDS-staged 16-byte stores for bf16) --
    # bit-identical to "pp" / "pps"; against "pps" (the ping-pong K loop with the LDS-staged
    # epilogue, round 4's default) on the 16k-row chunk: qkv -3.3 %, o -2.3 %, gate_up + SwiGLU
    # -3.9 %, down -1.0 % (profiles/r06_pgemm_ppp_v2.jsonl, r06_pgemm_k3.jsonl)
    PGEMM_VARIANT_DEFAULT = "ppp"
    PGEMM_VARIANT_SWIGLU_DEFAULT = "ppp"
    PGEMM_MIN_ROWS = 256         # fewer prompt rows than one 256-row tile: the decode GEMM (packed) or the library

    def _packing(self) -> str | None:
        """None (row-major only), "both" (packed + row-major) or "only" (packed only)."""
        pk = os.environ.get("CFC_DECODE_PACKED", "auto")
        if pk not in ("auto", "0", "1"):
            raise ValueError(f"CFC_DECODE_PACKED={pk!r}: expected auto, 0 or 1")
        po = os.environ.get("CFC_WEIGHTS_PACKED_ONLY", "auto")
        if po not in ("auto", "0", "1"):
            raise ValueError(f"CFC_WEIGHTS_PACKED_ONLY={po!r}: expected auto, 0 or 1")
        if pk == "0" or not self.w.layers or self.w.layers[0].get("qkv") is None or not self._dgemm_shapes():
            return None
        if not self.w.gate_up_interleaved:
            return None
        # packed-only needs every consumer of the projections on the packed copy: the fused decode
        # GEMM (not fp8 / a small-batch GEMV with quantized weights) and the hand-written prefill
        only_ok = self.decode_gemm == "dgemm" and self.prefill_gemm == "hip" and not self.fp8 \
            and self.w.qlayers is None
        if po == "1" or (po == "auto" and only_ok):
            if not only_ok:
                raise ValueError("CFC_WEIGHTS_PACKED_ONLY=1 needs CFC_DECODE_GEMM=dgemm and CFC_PREFILL_GEMM=hip")
            return "only"
        if pk == "1":
            return "both"
        free, total = torch.cuda.mem_get_info(self.w.device)
        return "both" if free - self.w.packed_bytes() > self.PACKED_FREE_FRACTION * total else None

    def _dgemm_shapes(self) -> bool:
        """Every decode projection of this rank fits the decode GEMM (N % 64, K % 64)."""
        w, D = self.w, self.cfg.head_dim
        qkv_n, q_k = (w.heads + 2 * w.kv_heads) * D, w.heads * D
        return all(n % 64 == 0 for n in (qkv_n, self.cfg.hidden, 2 * w.ffn)) and all(
            k % 64 == 0 for k in (self.cfg.hidden, q_k, w.ffn))

    def _lin(self, i: int, name: str, x: torch.Tensor) -> torch.Tensor:
        """Projection ``name`` of layer ``i``: bf16 library GEMM, or W8A8 FP8 in fp8 mode."""
        if self.fp8:
            w8, s = self.w.fp8_layers[i][name]
            return K.linear_fp8(x, w8, s)
        return F.linear(x, self.w.layers[i][name])

    def _lin32(self, i: int, name: str, x: torch.Tensor) -> torch.Tensor:
        """Projection ``name`` of layer ``i`` as an fp32 [M, N] (library / CPU path): a row-parallel
        partial that is all-reduced before its one bf16 rounding.  GPU: the library GEMM with an
        fp32 output (bf16 operands, fp32 accumulate) or the decode GEMM's fp32 split-1 output."""
        w = self.w.layers[i].get(name)
        if x.is_cuda:
            if w is not None:
                return torch.mm(x, w.t(), out_dtype=torch.float32)
            pw = self.w.packed[i][name] if self.w.packed is not None else None
            if pw is not None and K.dgemm_ok(x, pw):
                return K.dgemm(x, pw, "part", 1)[0].clone()
        return F.linear(x.float(), K._rowmajor(w if w is not None else self.w.packed[i][name]).float())

    def _plin(self, i: int, name: str, x: torch.Tensor, epi: str = "bf16") -> torch.Tensor:
        """Prefill projection (``epi`` "swiglu" returns silu(gate) * up of the interleaved gate/up
        weights): the hand-written pgemm on the packed weight when selected and the shape fits;
        fewer rows than one pgemm tile on the decode GEMM (same packed weight); else the library."""
        pw = self.w.packed[i][name] if self.w.packed is not None else None
        wt = pw if pw is not None else self.w.layers[i][name]
        if self.prefill_gemm == "hip" and x.is_cuda and x.is_contiguous() and (
                epi != "swiglu" or self.w.gate_up_interleaved):
            dg = pw is not None and K.dgemm_ok(x, pw)
            if (x.shape[0] >= self.PGEMM_MIN_ROWS and K.pgemm_ok(x, wt)
                    and not (dg and self._dgemm_faster(x.shape[0], wt.shape[0], x.shape[1]))):
                return K.pgemm(x, wt, epi, variant=self.pgemm_variant_swiglu if epi == "swiglu" else self.pgemm_variant)
            if dg:
                return K.dgemm_swiglu(x, pw) if epi == "swiglu" else K.dgemm_linear(x, pw)
        y = self._lin(i, name, x)
        return K.silu_mul(y, interleaved=self.w.gate_up_interleaved) if epi == "swiglu" else y

    def _plin32(self, i: int, name: str, x: torch.Tensor) -> torch.Tensor:
        """A row-parallel projection's fp32 partial [M, N] (TP > 1, CFC_TP_AR_DTYPE=fp32): pgemm's fp32
        epilogue on the packed weight, the decode GEMM's split-1 fp32 output for short chunks, else an
        fp32 GEMM.  A fresh tensor (the decode GEMM's output lives in a per-stream workspace that the
        next call would reuse under an asynchronous all-reduce)."""
        pw = self.w.packed[i][name] if self.w.packed is not None else None
        wt = pw if pw is not None else self.w.layers[i][name]
        if self.prefill_gemm == "hip" and x.is_cuda and x.is_contiguous():
            dg = pw is not None and K.dgemm_ok(x, pw)
            if (x.shape[0] >= self.PGEMM_MIN_ROWS and K.pgemm_ok(x, wt)
                    and not (dg and self._dgemm_faster(x.shape[0], wt.shape[0], x.shape[1]))):
                return K.pgemm(x, wt, "f32", variant=self.pgemm_variant)
            if dg:
                return K.dgemm(x, pw, "part", 1)[0].clone()
        if x.is_cuda and not isinstance(wt, K.PackedWeight):
            return torch.mm(x, wt.t(), out_dtype=torch.float32)
        return F.linear(x.float(), K._rowmajor(wt).float())

    def _tp_norm(self, part: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor) -> torch.Tensor:
        """residual += bf16(sum over the TP group of this rank's fp32 partial(s)); returns
        RMSNorm(residual) * norm_w -- TP = 1's split-K reduce arithmetic, the projection rounded to
        bf16 once.  ``part``: [M, N] or k-slice slabs [S, M, N].  One launch on the one-shot IPC
        kernel when the rows fit its staging (decode; short prefill chunks), else an fp32
        all-reduce of the row sums + the reduce kernel."""
        p3 = part if part.dim() == 3 else part[None]
        ar = self.custom_ar
        if ar is not None and ar.supports_slabs(p3):
            return ar.residual_rmsnorm(p3, residual, norm_w, self.cfg.rms_eps)
        t = p3.sum(0, keepdim=True) if p3.shape[0] > 1 else p3.contiguous()
        torch.distributed.all_reduce(t, group=self.tp_group)
        return K.splitk_residual_rmsnorm(t, residual, norm_w, self.cfg.rms_eps)

    PGEMM_MIN_TILES = 96   # fewer 256 x 256 output tiles than this: the decode GEMM is as fast or faster

    def _dgemm_faster(self, M: int, N: int, Kd: int) -> bool:
        """A prompt chunk too short to fill the chip with pgemm's 256 x 256 tiles runs on the decode
        GEMM (one W pass per 256-row tile, ~450-870 TF/s): measured crossover at ~96 tiles
        (profiles/r04_prefill_small_m.jsonl, Mistral-7B packed weights): qkv at 1024 rows (96
        tiles) 76 vs 79 us, o at 1024 (64) 71 vs 72, down at 1024 (64) 220 vs 150 and at 2048
        (128) 244 vs 298.  A 512-token prompt: 70 -> 40 (qkv), 68 -> 33 (o), 211 -> 83 us (down)."""
        return -(-M // 256) * -(-N // 256) < self.PGEMM_MIN_TILES

    def _all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.w.tp_size > 1:
            if self.custom_ar is not None and self.custom_ar.supports(x):
                return self.custom_ar(x)
            torch.distributed.all_reduce(x, group=self.tp_group)
        return x

    def _layer_pre(self, i, x, residual):
        """Returns normed input of layer i and the residual stream."""
        lw = self.w.layers[i]
        # fp8 mode: the norm emits the qkv projection's quantised input directly (K.rmsnorm_fp8)
        norm = K.rmsnorm_fp8 if self.fp8 else K.rmsnorm
        if residual is None:
            residual = x.clone()
            h = norm(x, lw["attn_norm"], self.cfg.rms_eps)
        else:
            h = norm(x, lw["attn_norm"], self.cfg.rms_eps, residual=residual)
        return h, residual

    def _mlp(self, i, attn_out, residual):
        lw = self.w.layers[i]
        if self.fp8:
            h = K.rmsnorm_fp8(attn_out, lw["mlp_norm"], self.cfg.rms_eps, residual=residual)
            a = K.silu_mul_fp8(self._lin(i, "gate_up", h), interleaved=self.w.gate_up_interleaved)
            return self._all_reduce(self._lin(i, "down", a))
        h = K.rmsnorm(attn_out, lw["mlp_norm"], self.cfg.rms_eps, residual=residual)
        a = self._plin(i, "gate_up", h, "swiglu")
        return self._all_reduce(self._plin(i, "down", a))

    def forward_prefill(self, ids, positions, slots, cu_q, ctx_lens, block_tables, kv, tiles=None,
                        last_idx=None, v_runs=None) -> torch.Tensor:
        """Packed varlen prefill. Returns hidden states of rows ``last_idx`` (or all rows).
        ``v_runs`` (ops.kernels.v_runs of the slots, on device): V written per cache block."""
        cfg, w = self.cfg, self.w
        x = K.embedding(w.embed, ids)
        residual = None
        x32 = None                     # TP fp32: this rank's fp32 partial of the previous layer's down
        eps = cfg.rms_eps
        for i in range(cfg.layers):
            lw = w.layers[i]
            if x32 is not None:
                h = self._tp_norm(x32, residual, lw["attn_norm"])
            else:
                h, residual = self._layer_pre(i, x, residual)
            qkv = self._plin(i, "qkv", h)
            q = K.rope_kv_write(qkv, positions, slots, w.cos_sin, kv.k[i], kv.v[i], w.heads, w.kv_heads,
                                cfg.head_dim, runs=v_runs, k_scale=kv.k_scale, v_scale=kv.v_scale)
            attn = K.prefill_attention(q, kv.k[i], kv.v[i], block_tables, cu_q, ctx_lens, self.scale, tiles=tiles,
                                       window=self.window, k_scale=kv.k_scale, v_scale=kv.v_scale)
            a2 = attn.view(attn.shape[0], -1)
            if self.tp_fp32:
                # row-parallel o / down: fp32 partials summed over the ranks, rounded once in the reduce
                h = self._tp_norm(self._plin32(i, "o", a2), residual, lw["mlp_norm"])
                x32 = self._plin32(i, "down", self._plin(i, "gate_up", h, "swiglu"))
                continue
            o = self._all_reduce(self._plin(i, "o", a2))
            x = self._mlp(i, o, residual)
        if x32 is not None:
            if last_idx is not None:
                x32, residual = x32.index_select(0, last_idx), residual.index_select(0, last_idx)
            return self._tp_norm(x32.contiguous(), residual, w.final_norm)
        if last_idx is not None:
            x = x.index_select(0, last_idx)
            residual = residual.index_select(0, last_idx)
        return K.rmsnorm(x, w.final_norm, cfg.rms_eps, residual=residual)

    def supports_prefill_overlap(self) -> bool:
        """Two-half overlapped prefill: TP > 1 on the bf16 path (the fp8 path keeps one pass)."""
        return self.w.tp_size > 1 and not self.fp8 and self.tp_group is not None

    def forward_prefill_overlap(self, halves: list[dict], kv) -> list[torch.Tensor]:
        """TP prefill of two independent halves of a chunk (whole sequences each; ``halves`` are
        :meth:`forward_prefill` keyword sets), interleaved layer by layer so that every row-parallel
        all-reduce of one half runs asynchronously (RCCL on its own stream; ``async_op``) while the
        other half's GEMMs and attention run: per layer A.attn -> AR(A.o) | B.attn -> AR(B.o) |
        A.mlp -> AR(A.down) | B.mlp -> AR(B.down), the same collective order on every rank.  Each
        half computes exactly what :meth:`forward_prefill` computes for its rows.  A prefill
        all-reduce is B x hidden x 2 bytes (128 MB at 16k rows of Mistral-7B): at TP = 8 over xGMI
        about as long as the rank's GEMMs, which would otherwise wait for it."""
        cfg, w = self.cfg, self.w
        dist = torch.distributed
        st = [{"m": m, "x": K.embedding(w.embed, m["ids"]), "res": None, "work": None} for m in halves]
        f32 = self.tp_fp32
        eps = cfg.rms_eps

        def start(s, t):
            s["work"] = dist.all_reduce(t, group=self.tp_group, async_op=True)

        def wait(s):
            if s["work"] is not None:
                s["work"].wait()          # NCCL: a stream dependency, the host keeps enqueueing
                s["work"] = None

        for i in range(cfg.layers):
            lw = w.layers[i]
            for s in st:
                m = s["m"]
                wait(s)                                          # x: the previous layer's reduced down
                if f32 and i > 0:
                    h = K.splitk_residual_rmsnorm(s["x"][None], s["res"], lw["attn_norm"], eps)
                else:
                    h, s["res"] = self._layer_pre(i, s["x"], s["res"])
                qkv = self._plin(i, "qkv", h)
                q = K.rope_kv_write(qkv, m["positions"], m["slots"], w.cos_sin, kv.k[i], kv.v[i], w.heads,
                                    w.kv_heads, cfg.head_dim, runs=m["v_runs"], k_scale=kv.k_scale,
                                    v_scale=kv.v_scale)
                attn = K.prefill_attention(q, kv.k[i], kv.v[i], m["block_tables"], m["cu_q"], m["ctx_lens"],
                                           self.scale, tiles=m["tiles"], window=self.window, k_scale=kv.k_scale,
                                           v_scale=kv.v_scale)
                a2 = attn.view(attn.shape[0], -1)
                s["o"] = self._plin32(i, "o", a2) if f32 else self._plin(i, "o", a2)
                start(s, s["o"])
            for s in st:
                wait(s)
                if f32:
                    h = K.splitk_residual_rmsnorm(s["o"][None], s["res"], lw["mlp_norm"], eps)
                else:
                    h = K.rmsnorm(s["o"], lw["mlp_norm"], eps, residual=s["res"])
                a = self._plin(i, "gate_up", h, "swiglu")
                s["x"] = self._plin32(i, "down", a) if f32 else self._plin(i, "down", a)
                s["o"] = None
                start(s, s["x"])
        out = []
        for s in st:
            wait(s)
            x, res, last = s["x"], s["res"], s["m"]["last_idx"]
            if last is not None:
                x, res = x.index_select(0, last), res.index_select(0, last)
            if f32:
                out.append(K.splitk_residual_rmsnorm(x[None].contiguous(), res, w.final_norm, eps))
            else:
                out.append(K.rmsnorm(x, w.final_norm, eps, residual=res))
        return out

    def forward_decode(self, ids, positions, slots, ctx_lens, block_tables, kv, attn_workspace=None,
                       part_blocks=16, shared_blocks=None) -> torch.Tensor:
        """One token per sequence. Returns final-normed hidden [B, H].  ``shared_blocks`` (device int32
        [1]): leading KV blocks every sequence shares (prefix cache) -- the attention reads them through
        the caches instead of nontemporal."""
        self._shared_blocks = shared_blocks
        cfg, w = self.cfg, self.w
        x = K.embedding(w.embed, ids)
        B = ids.shape[0]
        if (self.fused_decode and x.is_cuda and (B <= DGEMM_MAX_ROWS or self.w.packed_only)
                and not (B <= K.GEMV_MAX_M and (self.decode_gemv or self.decode_qgemv))):
            return self._forward_decode_fused(x, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                              part_blocks)
        if self.decode_gemm in ("splitk", "dgemm") and x.is_cuda and self.w.tp_size == 1:
            return self._forward_decode_splitk(x, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                               part_blocks)
        residual = None
        x32 = None
        for i in range(cfg.layers):
            lw = w.layers[i]
            if x32 is not None:
                h = self._tp_norm(x32, residual, lw["attn_norm"])
            else:
                h, residual = self._layer_pre(i, x, residual)
            qkv = self._lin(i, "qkv", h)
            attn = self._rope_attention(i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                        part_blocks)
            if self.tp_fp32:
                h = self._tp_norm(self._lin32(i, "o", attn.view(B, -1)), residual, lw["mlp_norm"])
                gu = self._lin(i, "gate_up", h)
                x32 = self._lin32(i, "down", K.silu_mul(gu, interleaved=w.gate_up_interleaved))
                continue
            o = self._all_reduce(self._lin(i, "o", attn.view(B, -1)))
            x = self._mlp(i, o, residual)
        if x32 is not None:
            return self._tp_norm(x32, residual, w.final_norm)
        return K.rmsnorm(x, w.final_norm, cfg.rms_eps, residual=residual)

    def _rope_attention(self, i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace, part_blocks):
        """RoPE + K/V cache write + paged decode attention of layer ``i`` from the qkv projection output
        (bf16 [B, N], or fp32 split-K slabs [split, B, N]).  Default: ONE kernel (the attention's
        prologue does the RoPE / KV write, ``CFC_DECODE_ROPE_FUSED=1``); else rope_kv then attention.
        Both write the same cache bytes and return the same output."""
        cfg, w = self.cfg, self.w
        sb = getattr(self, "_shared_blocks", None)
        B = qkv.shape[-2]
        fused = self.rope_fused == "1" or (self.rope_fused == "" and B <= K.GEMV_MAX_M)
        if fused and qkv.is_cuda:
            return K.paged_decode_rope_attention(qkv, positions, slots, w.cos_sin, kv.k[i], kv.v[i], block_tables,
                                                 ctx_lens, self.scale, w.heads, w.kv_heads, cfg.head_dim,
                                                 part_blocks=part_blocks, workspace=attn_workspace,
                                                 window=self.window, k_scale=kv.k_scale, v_scale=kv.v_scale,
                                                 shared_blocks=sb)
        if qkv.dim() == 3:
            q = K.rope_kv_write_part(qkv, positions, slots, w.cos_sin, kv.k[i], kv.v[i], w.heads, w.kv_heads,
                                     cfg.head_dim, k_scale=kv.k_scale, v_scale=kv.v_scale)
        else:
            q = K.rope_kv_write(qkv, positions, slots, w.cos_sin, kv.k[i], kv.v[i], w.heads, w.kv_heads,
                                cfg.head_dim, k_scale=kv.k_scale, v_scale=kv.v_scale)
        return K.paged_decode_attention(q, kv.k[i], kv.v[i], block_tables, ctx_lens, self.scale,
                                        part_blocks=part_blocks, workspace=attn_workspace, window=self.window,
                                        k_scale=kv.k_scale, v_scale=kv.v_scale, shared_blocks=sb)

    def _forward_decode_fused(self, x, positions, slots, ctx_lens, block_tables, kv, attn_workspace, part_blocks):
        """Decode layer on the hand-written decode GEMM (dgemm.hip), elementwise work in epilogues:
        qkv -> RoPE/KV write -> attention -> [o + residual + mlp RMSNorm] -> [gate_up + SwiGLU] ->
        [down + residual + next layer's RMSNorm].  Same rounding points as the library path.
        With TP the row-parallel o/down outputs are all-reduced (one-shot IPC all-reduce inside the
        decode graph when available) before the residual + RMSNorm."""
        cfg, w = self.cfg, self.w
        B = x.shape[0]
        eps = cfg.rms_eps
        residual = x.clone()
        h = K.rmsnorm(x, w.layers[0]["attn_norm"], eps)
        tp = w.tp_size > 1
        for i in range(cfg.layers):
            lw = w.layers[i]
            pw = w.packed[i] if w.packed is not None else lw    # fragment-packed copies when present
            wq = pw["qkv"]
            qbn, qsplit = K.dgemm_config(B, wq.shape[0], h.shape[1], bn=getattr(wq, "bn", None))
            qsplit = self.qkv_split or qsplit
            # split-K slabs go straight into RoPE / KV write (the reduce folded in)
            qkv = K.dgemm(h, wq, "part", qsplit, bn=qbn) if qsplit > 1 else K.dgemm_linear(h, wq)
            attn = self._rope_attention(i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                        part_blocks)
            if tp:
                h = self._tp_residual_rmsnorm(attn.view(B, -1), pw["o"], residual, lw["mlp_norm"], eps)
            else:
                h = K.dgemm_residual_rmsnorm(attn.view(B, -1), pw["o"], residual, lw["mlp_norm"], eps)
            a = K.dgemm_swiglu(h, pw["gate_up"])
            nxt = w.layers[i + 1]["attn_norm"] if i + 1 < cfg.layers else w.final_norm
            if tp:
                h = self._tp_residual_rmsnorm(a, pw["down"], residual, nxt, eps)
            else:
                h = K.dgemm_residual_rmsnorm(a, pw["down"], residual, nxt, eps)
        return h

    def _tp_residual_rmsnorm(self, x, w, residual, norm_w, eps):
        """Row-parallel projection + all-reduce + residual + RMSNorm at TP > 1 with TP = 1's
        rounding points: the decode GEMM's fp32 k-slice slabs of this rank's K shard are summed over
        the TP group in fp32 and rounded to bf16 once (as TP = 1's split-K reduce does), never per
        rank.  On the one-shot IPC kernel: ONE launch after the GEMM (comm.hip:
        oneshot_ar_residual_rmsnorm_kernel); else an fp32 all-reduce of the rank's row sums (RCCL /
        gloo) and the split = 1 reduce kernel."""
        B, Kd = x.shape
        bn, split = K.dgemm_config(B, w.shape[0], Kd, bn=getattr(w, "bn", None))
        return self._tp_norm(K.dgemm(x, w, "part", split, bn=bn), residual, norm_w)

    def _forward_decode_splitk(self, x, positions, slots, ctx_lens, block_tables, kv, attn_workspace, part_blocks):
        """Library GEMMs; o and down as batched split-K with residual + next RMSNorm in the reduce."""
        cfg, w = self.cfg, self.w
        B = x.shape[0]
        eps = cfg.rms_eps
        residual = x.clone()
        h = K.rmsnorm(x, w.layers[0]["attn_norm"], eps)
        s_o = K.lib_split_for(w.heads * cfg.head_dim, cfg.hidden)
        s_d = K.lib_split_for(w.ffn, cfg.hidden)
        if self.decode_qgemv and B <= K.GEMV_MAX_M:
            return self._forward_decode_qgemv(h, residual, positions, slots, ctx_lens, block_tables, kv,
                                              attn_workspace, part_blocks)
        if self.decode_gemv and B <= K.GEMV_MAX_M:
            return self._forward_decode_gemv(h, residual, positions, slots, ctx_lens, block_tables, kv,
                                             attn_workspace, part_blocks)
        for i in range(cfg.layers):
            lw = w.layers[i]
            qkv = F.linear(h, lw["qkv"])
            attn = self._rope_attention(i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                        part_blocks)
            h = K.lib_splitk_linear_residual_rmsnorm(attn.view(B, -1), lw["o"], s_o, residual, lw["mlp_norm"], eps)
            a = K.silu_mul(F.linear(h, lw["gate_up"]), interleaved=w.gate_up_interleaved)
            nxt = w.layers[i + 1]["attn_norm"] if i + 1 < cfg.layers else w.final_norm
            h = K.lib_splitk_linear_residual_rmsnorm(a, lw["down"], s_d, residual, nxt, eps)
        return h

    def _forward_decode_gemv(self, h, residual, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                             part_blocks):
        """Single-stream / small-batch decode (B <= 4): every projection on the weight-streaming GEMV
        kernel (gemm.hip: gemv_kernel), SwiGLU in the gate/up GEMV's epilogue, o and down feeding the
        residual + next-RMSNorm reduce.  Same rounding points as _forward_decode_splitk."""
        cfg, w = self.cfg, self.w
        B, eps = h.shape[0], cfg.rms_eps
        if w.packed_only and h.is_cuda and self.gemv_norm_fused and cfg.hidden <= 8192:
            return self._forward_decode_gemv_fused(h, residual, positions, slots, ctx_lens, block_tables, kv,
                                                   attn_workspace, part_blocks)
        for i in range(cfg.layers):
            # packed-only weights: the packed-weight GEMV reads the packed copies
            lw = w.layers[i]
            if w.packed_only:
                lw = dict(lw, **w.packed[i])
            # packed qkv: k-slice slabs straight into the slab-reading RoPE / KV write
            qkv = K.gemv_part(h, lw["qkv"]) if isinstance(lw["qkv"], K.PackedWeight) else K.gemv(h, lw["qkv"])
            attn = self._rope_attention(i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                        part_blocks)
            h = K.gemv_residual_rmsnorm(attn.view(B, -1), lw["o"], residual, lw["mlp_norm"], eps)
            a = K.gemv(h, lw["gate_up"], "swiglu")
            nxt = w.layers[i + 1]["attn_norm"] if i + 1 < cfg.layers else w.final_norm
            h = K.gemv_residual_rmsnorm(a, lw["down"], residual, nxt, eps)
        return h

    def _forward_decode_gemv_fused(self, h, residual, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                   part_blocks):
        """B <= 4 decode over the packed weights with the residual + RMSNorm reduces folded into the
        next GEMV's prologue (K.gemv_norm): per layer qkv (slabs, its input norm fused from the
        previous down's slabs) -> RoPE / attention -> o (slabs) -> gate_up + SwiGLU (its input norm
        fused from o's slabs) -> down (slabs).  Two launches fewer per layer than
        _forward_decode_gemv, bit-identical to it: the prologue repeats the reduce kernel's
        arithmetic.  The residual alternates between two buffers (a fused norm reads one while its
        workgroup 0 writes the other); consecutive slab producers alternate two halves of the
        split-K workspace (a producer's input slabs are still being read while it writes)."""
        cfg, w = self.cfg, self.w
        B, eps = h.shape[0], cfg.rms_eps
        P = [w.packed[i] for i in range(cfg.layers)]

        def nslab(W):
            return K.gemv_packed_config(W.N, W.K, W.bn // 16, B)[0] * B * W.N
        size = max(nslab(P[0][k]) for k in ("qkv", "o", "down"))
        ws = K._workspace(h.device, 2 * size)
        bufs, nb = (ws[:size], ws[size:2 * size]), 0
        res, cur = (residual, torch.empty_like(residual)), 0
        pend = None
        for i in range(cfg.layers):
            lw, pw = w.layers[i], P[i]

            def out(W):
                sp = K.gemv_packed_config(W.N, W.K, W.bn // 16, B)[0]
                return bufs[nb][:sp * B * W.N].view(sp, B, W.N)
            if pend is None:
                qkv = K.gemv_part(h, pw["qkv"], out=out(pw["qkv"]))
            else:
                qkv = K.gemv_norm(pend, res[cur], res[1 - cur], lw["attn_norm"], eps, pw["qkv"], out=out(pw["qkv"]))
                cur ^= 1
            nb ^= 1
            attn = self._rope_attention(i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                        part_blocks)
            o = K.gemv_part(attn.view(B, -1), pw["o"], out=out(pw["o"]))
            nb ^= 1
            a = K.gemv_norm(o, res[cur], res[1 - cur], lw["mlp_norm"], eps, pw["gate_up"], "swiglu")
            cur ^= 1
            pend = K.gemv_part(a, pw["down"], out=out(pw["down"]))
            nb ^= 1
        return K.splitk_residual_rmsnorm(pend, res[cur], w.final_norm, eps)

    def _forward_decode_qgemv(self, h, residual, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                              part_blocks):
        """B <= 4 decode straight from the GGUF blocks (Q4_K / Q6_K / Q8_0 weight stream, 3.6x fewer
        bytes than bf16 at Q4_K).  Projections without a quantized copy use the bf16 GEMV.  Same
        rounding points as _forward_decode_gemv."""
        cfg, w = self.cfg, self.w
        B, eps = h.shape[0], cfg.rms_eps
        qs, ks = w.heads * cfg.head_dim, w.kv_heads * cfg.head_dim
        for i in range(cfg.layers):
            lw, ql = w.layers[i], w.qlayers[i]
            # a projection takes its quantized copy only when B rows of its input fit the qgemv's
            # LDS stage (K.qgemv_fits); otherwise the bf16 GEMV of the same layer
            fit_h, fit_o, fit_d = K.qgemv_fits(B, cfg.hidden), K.qgemv_fits(B, qs), K.qgemv_fits(B, w.ffn)
            if ql["q"] is not None and ql["k"] is not None and ql["v"] is not None and fit_h:
                qkv = torch.empty(B, qs + 2 * ks, dtype=torch.bfloat16, device=h.device)
                ld = qkv.shape[1]   # q, k, v write their column slices (types may differ: Q4_K_M's v is often Q6_K)
                K.qgemv(h, ql["q"], out=qkv, ldo=ld)
                K.qgemv(h, ql["k"], out=qkv[:, qs:], ldo=ld)
                K.qgemv(h, ql["v"], out=qkv[:, qs + ks:], ldo=ld)
            else:
                qkv = K.gemv(h, lw["qkv"])
            attn = self._rope_attention(i, qkv, positions, slots, ctx_lens, block_tables, kv, attn_workspace,
                                        part_blocks)
            a2 = attn.view(B, -1)
            if ql["o"] is not None and fit_o:
                part = K._workspace(h.device, B * cfg.hidden)[:B * cfg.hidden].view(1, B, cfg.hidden)
                K.qgemv(a2, ql["o"], "f32", out=part[0])
                h = K.splitk_residual_rmsnorm(part, residual, lw["mlp_norm"], eps)
            else:
                h = K.gemv_residual_rmsnorm(a2, lw["o"], residual, lw["mlp_norm"], eps)
            g, u = ql["gate"], ql["up"]
            if g is not None and u is not None and g.qtype == u.qtype and fit_h:
                a = K.qgemv(h, g, "swiglu", qw2=u)
            else:
                a = K.gemv(h, lw["gate_up"], "swiglu")
            nxt = w.layers[i + 1]["attn_norm"] if i + 1 < cfg.layers else w.final_norm
            if ql["down"] is not None and fit_d:
                part = K._workspace(h.device, B * cfg.hidden)[:B * cfg.hidden].view(1, B, cfg.hidden)
                K.qgemv(a, ql["down"], "f32", out=part[0])
                h = K.splitk_residual_rmsnorm(part, residual, nxt, eps)
            else:
                h = K.gemv_residual_rmsnorm(a, lw["down"], residual, nxt, eps)
        return h

    def greedy_ids(self, hidden: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Greedy next tokens into ``out`` [B] int32 without gathering the logits: each vocab
        shard's argmax_keys, MAX-reduced over the TP group -- on the one-shot IPC kernel when it is
        up (then a TP decode step holds no RCCL call and is captured whole), else one RCCL / gloo
        all-reduce of B int64."""
        local = self._local_logits(hidden)
        if self.w.tp_size == 1:
            return K.sample(local, out, 0.0)
        keys = argmax_keys(local, self.w.tp_rank * self.w.vocab_shard)
        ar = self.custom_ar
        if ar is not None and ar.supports_keys(keys.numel()):
            return ar.keymax(keys, out)
        torch.distributed.all_reduce(keys, op=torch.distributed.ReduceOp.MAX, group=self.tp_group)
        out.copy_((0xFFFFFFFF - (keys & 0xFFFFFFFF)).to(torch.int32))
        return out

    def graph_collectives_ok(self, B: int) -> bool:
        """Every collective of a greedy decode step at batch B runs on the one-shot IPC kernels (so
        the step can be captured even when the process group's backend cannot be, e.g. gloo)."""
        ar = self.custom_ar
        if self.w.tp_size == 1:
            return True
        n = B * self.cfg.hidden       # the o / down all-reduces: B x hidden fp32 row sums
        return (ar is not None and ar.enabled and ar.supports_keys(B) and n % 8 == 0
                and n * 4 <= ar.staging_bytes and self.cfg.hidden <= 8192)

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """[B, V] logits (all-gathered over the vocab-parallel shards)."""
        local = self._local_logits(hidden)
        if self.w.tp_size == 1:
            return local
        parts = [torch.empty_like(local) for _ in range(self.w.tp_size)]
        torch.distributed.all_gather(parts, local, group=self.tp_group)
        return torch.cat(parts, -1)

    def _local_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """This rank's vocab shard of the logits [B, V / tp]."""
        head = self.w.lm_head
        if (self.decode_qgemv and self.w.q_lm_head is not None and hidden.is_cuda
                and hidden.shape[0] <= K.GEMV_MAX_M and hidden.is_contiguous() and self.w.q_lm_head.N % 4 == 0
                and K.qgemv_fits(hidden.shape[0], hidden.shape[1])):
            local = K.qgemv(hidden, self.w.q_lm_head)
        elif (self.decode_gemv and hidden.is_cuda and hidden.shape[0] <= K.GEMV_MAX_M
                and hidden.is_contiguous() and head.shape[0] % 2 == 0 and head.shape[1] % 8 == 0):
            # (the GEMV takes row pairs and 16-byte K slices: odd vocabularies, e.g. 32001-token
            # fine-tunes, stay on the library GEMM)
            local = K.gemv(hidden, self.w.lm_head)   # 262 MB weight stream: 4.6 -> ~6 TB/s at B=1
        elif (self.fused_decode and hidden.is_cuda and hidden.shape[0] > K.GEMV_MAX_M
                and hidden.shape[0] <= DGEMM_MAX_ROWS and K.dgemm_ok(hidden, head)):
            # the 262 MB (Mistral) / 1 GB (Llama-3) vocab stream
            ph = self.w.packed_lm_head
            local = K.dgemm_linear(hidden, ph if ph is not None else head)
        else:
            local = F.linear(hidden, self.w.lm_head)
        return local
