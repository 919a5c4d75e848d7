"""GGUF checkpoints (runtime/gguf.py) and the ggml-quantized decode path (csrc/kernels/quant.hip).

The reference serves a Q4_K_M GGUF through llama.cpp (docker-compose.infra.yml:296-298).  llama.cpp
and the ``gguf`` package are not in this image, so the block formats are pinned by hand-built
blocks whose values are computed independently from the ggml layout descriptions (parity with
llama.cpp's own dequantizer is otherwise unpinned); the container format by a writer/reader round
trip; the llama conventions by an HF model written as GGUF (q/k permuted as llama.cpp's converter
does, cross-checked against transformers' own inverse) and loaded back to the same logits."""
from __future__ import annotations

import json
import struct

import numpy as np
import pytest
import torch

from copilot_for_consensus_amd.models.decoder import DecoderConfig, DecoderModel, DecoderWeights
from copilot_for_consensus_amd.runtime import gguf as G
from copilot_for_consensus_amd.runtime.kv_cache import KV_BLOCK, PagedKVCache


def _f16b(x: float) -> bytes:
    return np.float16(x).tobytes()


def test_q4k_block_dequant_matches_layout():
    """One hand-built block_q4_K: d = 0.5, dmin = 0.25, sub-block scales 1..8 and mins 8..1 (6-bit,
    the upper four pairs split over the high bits as ggml packs them), nibble q = w % 16."""
    sc = list(range(1, 9))
    mn = list(range(8, 0, -1))
    sc[5], mn[6] = 45, 60                       # values >= 16 exercise the 2 high bits
    scales = G._pack_scale_min_k4(np.array([sc]), np.array([mn]))[0]
    q = np.arange(256) % 16
    qs = np.zeros(128, np.uint8)
    for j in range(4):
        qs[32 * j:32 * j + 32] = q[64 * j:64 * j + 32] | (q[64 * j + 32:64 * j + 64] << 4)
    raw = np.frombuffer(_f16b(0.5) + _f16b(0.25) + scales.tobytes() + qs.tobytes(), np.uint8)
    assert raw.size == 144
    got = G.dequantize(raw, G.Q4_K, (256,))
    want = np.array([0.5 * sc[w // 32] * q[w] - 0.25 * mn[w // 32] for w in range(256)], np.float32)
    np.testing.assert_array_equal(got, want)


def test_q6k_block_dequant_matches_layout():
    """block_q6_K: 6-bit q (low nibble in ql, high 2 bits in qh), int8 scale per 16 weights."""
    rng = np.random.default_rng(0)
    q = rng.integers(0, 64, 256)
    scales = rng.integers(-128, 128, 16).astype(np.int8)
    ql = np.zeros(128, np.uint8)
    qh = np.zeros(64, np.uint8)
    for h in range(2):
        Q = q[128 * h:128 * h + 128]
        for l in range(32):
            q1, q2, q3, q4 = Q[l], Q[32 + l], Q[64 + l], Q[96 + l]
            ql[64 * h + l] = (q1 & 15) | ((q3 & 15) << 4)
            ql[64 * h + 32 + l] = (q2 & 15) | ((q4 & 15) << 4)
            qh[32 * h + l] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
    raw = np.frombuffer(ql.tobytes() + qh.tobytes() + scales.tobytes() + _f16b(0.125), np.uint8)
    assert raw.size == 210
    got = G.dequantize(raw, G.Q6_K, (256,))
    want = np.array([0.125 * float(scales[w // 16]) * (int(q[w]) - 32) for w in range(256)], np.float32)
    np.testing.assert_allclose(got, want, rtol=0, atol=0)


def test_legacy_blocks_dequant_match_layout():
    rng = np.random.default_rng(1)
    qs = rng.integers(0, 256, 16, dtype=np.uint8)
    lo, hi = (qs & 15).astype(int), (qs >> 4).astype(int)
    q4 = np.concatenate([lo, hi])
    np.testing.assert_array_equal(G.dequantize(np.frombuffer(_f16b(2.0) + qs.tobytes(), np.uint8), G.Q4_0, (32,)),
                                  2.0 * (q4 - 8))
    np.testing.assert_array_equal(
        G.dequantize(np.frombuffer(_f16b(2.0) + _f16b(-1.0) + qs.tobytes(), np.uint8), G.Q4_1, (32,)), 2.0 * q4 - 1.0)
    qh = 0xA5C3F00F
    hb = np.array([(qh >> j) & 1 for j in range(32)])
    q5 = q4 | (hb << 4)
    raw5 = _f16b(0.5) + struct.pack("<I", qh) + qs.tobytes()
    np.testing.assert_array_equal(G.dequantize(np.frombuffer(raw5, np.uint8), G.Q5_0, (32,)), 0.5 * (q5 - 16))
    raw51 = _f16b(0.5) + _f16b(3.0) + struct.pack("<I", qh) + qs.tobytes()
    np.testing.assert_array_equal(G.dequantize(np.frombuffer(raw51, np.uint8), G.Q5_1, (32,)), 0.5 * q5 + 3.0)
    q8 = rng.integers(-128, 128, 32).astype(np.int8)
    np.testing.assert_array_equal(G.dequantize(np.frombuffer(_f16b(0.25) + q8.tobytes(), np.uint8), G.Q8_0, (32,)),
                                  0.25 * q8)


def test_q5k_dequant_is_q4k_plus_high_bit():
    """Q5_K = Q4_K's scales/mins + one extra bit per weight from qh (bit 2j / 2j+1 of qh[l])."""
    rng = np.random.default_rng(2)
    scales = rng.integers(0, 256, 12, dtype=np.uint8)
    qs = rng.integers(0, 256, 128, dtype=np.uint8)
    qh = rng.integers(0, 256, 32, dtype=np.uint8)
    head = _f16b(0.5) + _f16b(0.25) + scales.tobytes()
    y4 = G.dequantize(np.frombuffer(head + qs.tobytes(), np.uint8), G.Q4_K, (256,))
    y5 = G.dequantize(np.frombuffer(head + qh.tobytes() + qs.tobytes(), np.uint8), G.Q5_K, (256,))
    d, _ = G._scale_min_k4(scales[None])
    extra = np.array([16 * ((qh[w % 32] >> (2 * (w // 64) + (w // 32) % 2)) & 1) for w in range(256)])
    np.testing.assert_allclose(y5 - y4, 0.5 * d[0][np.arange(256) // 32] * extra, atol=1e-6)


@pytest.mark.parametrize("qtype,tol", [(G.Q8_0, 0.01), (G.Q4_0, 0.15), (G.Q4_K, 0.12), (G.Q6_K, 0.04),
                                       (G.F16, 1e-3), (G.BF16, 8e-3), (G.F32, 0)])
def test_quantize_roundtrip_error(qtype, tol):
    rng = np.random.default_rng(3)
    x = rng.standard_normal((8, 512)).astype(np.float32)
    y = G.dequantize(G.quantize(x, qtype), qtype, x.shape)
    rel = np.abs(y - x).max() / np.abs(x).max()
    assert rel <= tol + 1e-9, (G.TYPE_NAMES[qtype], rel)


def test_writer_reader_roundtrip(tmp_path):
    rng = np.random.default_rng(4)
    w = G.GGUFWriter("llama", alignment=64)
    w.add("general.name", "tiny")
    w.add("llama.block_count", 3)
    w.add("llama.rope.freq_base", 1e6)
    w.add("flag", True)
    w.add("big", 2 ** 40)
    w.add("tokenizer.ggml.tokens", ["<unk>", "a", "é", "東京"], G._ARR, G._STR)
    w.add("tokenizer.ggml.scores", np.array([0.0, -1.0, -2.5, -3.0], np.float32), G._ARR, G._F32)
    tens = {"a": (rng.standard_normal((4, 256)), G.Q4_K), "b": (rng.standard_normal((3, 64)), G.Q8_0),
            "c": (rng.standard_normal(7), G.F32), "d": (rng.standard_normal((2, 256)), G.Q6_K),
            "e": (rng.standard_normal((5, 32)), G.F16)}
    for name, (a, t) in tens.items():
        w.add_tensor(name, a, t)
    p = tmp_path / "t.gguf"
    w.write(p)
    r = G.GGUFReader(p)
    assert r.version == 3 and r.metadata["general.architecture"] == "llama"
    assert r.metadata["llama.block_count"] == 3 and r.metadata["flag"] is True and r.metadata["big"] == 2 ** 40
    assert abs(r.metadata["llama.rope.freq_base"] - 1e6) < 1
    assert r.metadata["tokenizer.ggml.tokens"] == ["<unk>", "a", "é", "東京"]
    np.testing.assert_array_equal(r.metadata["tokenizer.ggml.scores"], [0.0, -1.0, -2.5, -3.0])
    assert r.data_offset % 64 == 0
    for name, (a, t) in tens.items():
        ti = r.tensors[name]
        assert ti.shape == a.shape and ti.ggml_type == t
        np.testing.assert_array_equal(r.tensor(name), G.dequantize(G.quantize(a, t), t, a.shape))
    assert G.summary(p)["tensors"] == 5
    bad = tmp_path / "bad.gguf"
    bad.write_bytes(b"GGML" + bytes(40))
    with pytest.raises(G.GGUFError):
        G.GGUFReader(bad)


def test_qk_permutation_inverse_and_matches_transformers():
    rng = np.random.default_rng(5)
    w = rng.standard_normal((8 * 16, 24)).astype(np.float32)   # 8 heads of 16 rows
    p = G.permute_qk(w, 8)
    np.testing.assert_array_equal(G.unpermute_qk(p, 8), w)
    np.testing.assert_array_equal(p[G.unpermute_qk_rows(128, 8)], w)
    mg = pytest.importorskip("transformers.modeling_gguf_pytorch_utils")
    proc = mg.LlamaTensorProcessor(config={"num_attention_heads": 8, "num_key_value_heads": 8})
    np.testing.assert_array_equal(proc._reverse_permute_weights(p, 8, 8), w)


def _hf_llama(tmp_path):
    transformers = pytest.importorskip("transformers")
    torch.manual_seed(0)
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=2, num_key_value_heads=1, head_dim=128,
                                   max_position_embeddings=4096, rms_norm_eps=1e-5, rope_theta=1e6,
                                   tie_word_embeddings=False, bos_token_id=1, eos_token_id=2)
    model = transformers.LlamaForCausalLM(cfg).eval()
    d = tmp_path / "hf"
    model.save_pretrained(d, safe_serialization=True)
    return model, d


def _gguf_from_hf(model, hf_dir, path, qtypes=None, default=G.F32):
    from copilot_for_consensus_amd.models.decoder import load_config_json
    sd = {k: v.float().numpy() for k, v in model.state_dict().items()}
    cfg = load_config_json(hf_dir / "config.json")
    G.write_llama_gguf(path, cfg, sd, qtypes=qtypes, default_qtype=default)
    return cfg


def _prefill_logits(model, prompt, device):
    kv = PagedKVCache(model.cfg.layers, 16, model.w.kv_heads, model.cfg.head_dim, device)
    n = len(prompt)
    nb = -(-n // KV_BLOCK)
    blocks = list(range(nb))
    i32 = dict(dtype=torch.int32, device=device)
    ids = torch.tensor(prompt, **i32)
    pos = torch.arange(n, **i32)
    slots = torch.tensor([blocks[p // KV_BLOCK] * KV_BLOCK + p % KV_BLOCK for p in range(n)], **i32)
    hidden = model.forward_prefill(ids, pos, slots, torch.tensor([0, n], **i32), torch.tensor([n], **i32),
                                   torch.tensor([blocks], **i32), kv)
    return model.logits(hidden).float().cpu()


def test_gguf_f32_llama_loads_to_hf_logits(tmp_path):
    """HF Llama -> GGUF (F32, q/k permuted as llama.cpp does) -> from_gguf: same tensors as the
    safetensors loader and HF's logits (CPU reference ops)."""
    hf, d = _hf_llama(tmp_path)
    cfg = _gguf_from_hf(hf, d, tmp_path / "m.gguf")
    wg = DecoderWeights.from_gguf(tmp_path / "m.gguf", "cpu", quantized_decode=False)
    assert wg.cfg.layers == 2 and wg.cfg.kv_heads == 1 and wg.cfg.head_dim == 128 and not wg.cfg.tie_embeddings
    ws = DecoderWeights.from_safetensors(cfg, d, "cpu")
    for a, b in zip(wg.layers, ws.layers):
        for k in a:
            torch.testing.assert_close(a[k].float(), b[k].float(), rtol=0, atol=0)
    prompt = [1, 7, 99, 23, 5, 300, 42, 17, 8]
    got = _prefill_logits(DecoderModel(wg), prompt, "cpu")
    with torch.no_grad():
        want = hf(torch.tensor([prompt])).logits[0].float()
    assert torch.nn.functional.cosine_similarity(got, want, dim=-1).min() > 0.999
    assert (got.argmax(-1) == want.argmax(-1)).float().mean() >= 0.8


def test_gguf_config_and_tokenizer_metadata(tmp_path):
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)] + ["▁", "a", "b", "ab", "▁ab", "▁a"]
    types = [2, 3, 3] + [6] * 256 + [1] * 6
    scores = [0.0] * 259 + [-1.0, -2.0, -3.0, -4.0, -5.0, -6.0]
    cfg = DecoderConfig("t", len(toks), 256, 1, 2, 1, 128, 512)
    G.write_llama_gguf(tmp_path / "t.gguf", cfg, {}, tokens=toks, scores=scores, token_types=types)
    r = G.GGUFReader(tmp_path / "t.gguf")
    c2 = G.config_from_gguf(r.metadata, r.tensors.keys())
    assert (c2.vocab_size, c2.hidden, c2.layers, c2.heads, c2.kv_heads, c2.head_dim, c2.ffn) == \
        (len(toks), 256, 1, 2, 1, 128, 512)
    tok = G.tokenizer_from_gguf(r.metadata)
    ids = tok.encode("ab ab a", add_bos=True)
    assert [toks[i] for i in ids] == ["<s>", "▁ab", "▁ab", "▁a"]
    # an unknown character falls back to its UTF-8 bytes
    assert [toks[i] for i in tok.encode("ç", add_bos=False)] == ["▁", "<0xC3>", "<0xA7>"]


def test_gguf_tokenizer_matches_hf_sentencepiece(tmp_path):
    """A SentencePiece-BPE vocabulary trained with HF ``tokenizers`` exported as GGUF metadata
    (pieces, scores = -rank, token types) encodes like HF's tokenizer.json built from the same
    pieces with every two-piece split ranked by score (what HF's SentencePiece converter emits)."""
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers

    from copilot_for_consensus_amd.parsing import MessageParser

    msgs, _ = MessageParser().parse_mbox_bytes(open("tests/fixtures/sample.mbox", "rb").read(), "0" * 16)
    corpus = [m["body_normalized"] for m in msgs] * 3
    ref = Tokenizer(models.BPE(byte_fallback=True, unk_token="<unk>", fuse_unk=True))
    # pieces never span a word boundary (SentencePiece's split_by_whitespace): train with the
    # Metaspace pre-tokenizer, then run the Llama-2 / Mistral tokenizer.json pipeline
    ref.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="always", split=True)
    ref.train_from_iterator(corpus, trainers.BpeTrainer(
        vocab_size=1500, special_tokens=["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)]))
    d = json.loads(ref.to_str())
    d["pre_tokenizer"] = None
    d["normalizer"] = {"type": "Sequence", "normalizers": [{"type": "Prepend", "prepend": "▁"},
                                                           {"type": "Replace", "pattern": {"String": " "},
                                                            "content": "▁"}]}
    vocab = d["model"]["vocab"]
    toks = [None] * len(vocab)
    for t, i in vocab.items():
        toks[i] = t
    types = [2 if t == "<unk>" else 3 if t in ("<s>", "</s>") else 6 if (t.startswith("<0x") and len(t) == 6)
             else 1 for t in toks]
    scores = [-float(i) for i in range(len(toks))]
    # HF reference with the all-splits merge list (ranked by the merged piece's score)
    normal = sorted((i for i in range(len(toks)) if types[i] == 1 and len(toks[i]) > 1), key=lambda i: -scores[i])
    merges = []
    for i in normal:
        t = toks[i]
        for k in range(1, len(t)):
            a, b = t[:k], t[k:]
            if a in vocab and b in vocab and types[vocab[a]] == 1 and types[vocab[b]] == 1:
                merges.append([a, b])
    d["model"]["merges"] = merges
    ref = Tokenizer.from_str(json.dumps(d))
    cfg = DecoderConfig("t", len(toks), 256, 1, 2, 1, 128, 512)
    G.write_llama_gguf(tmp_path / "t.gguf", cfg, {}, tokens=toks, scores=scores, token_types=types)
    mine = G.tokenizer_from_gguf(G.GGUFReader(tmp_path / "t.gguf").metadata)
    for text in corpus[:8] + ["Hello, World! Café déjà-vu 東京 😀", "  two  spaces", "a\nb", ""]:
        assert mine.encode(text, add_bos=False) == ref.encode(text).ids, text


# ------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("qtype", [G.Q4_0, G.Q4_1, G.Q5_0, G.Q5_1, G.Q8_0, G.Q4_K, G.Q5_K, G.Q6_K, G.F16, G.BF16,
                                   G.F32])
def test_gpu_dequant_matches_numpy(qtype):
    from copilot_for_consensus_amd.ops.kernels import dequant_bf16
    rng = np.random.default_rng(6)
    shape = (6, 512)
    if qtype in (G.Q4_1, G.Q5_0, G.Q5_1, G.Q5_K):    # no quantizer here: random valid blocks
        per, size = G.BLOCK[qtype]
        raw = rng.integers(0, 256, (np.prod(shape) // per, size), dtype=np.uint8)
        raw[:, 0:2] = np.frombuffer(np.float16(0.01).tobytes(), np.uint8)
        if qtype != G.Q5_0:
            raw[:, 2:4] = np.frombuffer(np.float16(0.02).tobytes(), np.uint8)
        raw = raw.reshape(-1)
    else:
        raw = G.quantize(rng.standard_normal(shape).astype(np.float32), qtype)
    want = torch.from_numpy(G.dequantize(raw, qtype, shape)).bfloat16().float()
    got = dequant_bf16(raw, qtype, shape, "cuda").float().cpu()
    torch.testing.assert_close(got, want, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("qtype", [G.Q4_K, G.Q6_K, G.Q8_0])
@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("K", [512, 4096, 14336])
def test_gpu_qgemv_matches_dequantized_linear(qtype, M, K):
    from copilot_for_consensus_amd.ops import kernels as KK
    rng = np.random.default_rng(7)
    N = 96
    raw = G.quantize(rng.standard_normal((N, K)).astype(np.float32) * 0.05, qtype)
    wq = KK.QWeight.from_raw(raw, qtype, N, K, "cuda")
    wf = torch.from_numpy(G.dequantize(raw, qtype, (N, K)))
    x = torch.randn(M, K).bfloat16()
    want = x.float() @ wf.t()
    got = KK.qgemv(x.cuda(), wq, "f32").cpu()
    torch.testing.assert_close(got, want, rtol=2e-3, atol=2e-3 * float(want.abs().max()))
    gotb = KK.qgemv(x.cuda(), wq, "bf16").float().cpu()
    torch.testing.assert_close(gotb, want, rtol=1e-2, atol=1e-2 * float(want.abs().max()))
    # SwiGLU over a (gate, up) pair, and a column slice of a wider output buffer
    raw2 = G.quantize(rng.standard_normal((N, K)).astype(np.float32) * 0.05, qtype)
    wu = KK.QWeight.from_raw(raw2, qtype, N, K, "cuda")
    up = x.float() @ torch.from_numpy(G.dequantize(raw2, qtype, (N, K))).t()
    g = want.bfloat16().float()
    ref = (torch.nn.functional.silu(g) * up.bfloat16().float())
    sw = KK.qgemv(x.cuda(), wq, "swiglu", qw2=wu).float().cpu()
    torch.testing.assert_close(sw, ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
    wide = torch.zeros(M, 3 * N, dtype=torch.bfloat16, device="cuda")
    KK.qgemv(x.cuda(), wq, out=wide[:, N:], ldo=3 * N)
    assert float(wide[:, :N].abs().max()) == 0 and float(wide[:, 2 * N:].abs().max()) == 0
    torch.testing.assert_close(wide[:, N:2 * N].float().cpu(), gotb, rtol=0, atol=0)


@pytest.mark.gpu
def test_gpu_gguf_q4km_model_quantized_decode_matches_dequantized(tmp_path):
    """A Q4_K_M-style GGUF (Q4_K projections, Q6_K v/down/output, F32 norms): decode on the
    quantized GEMV vs the same weights dequantized to bf16 on the bf16 GEMV."""
    from copilot_for_consensus_amd.models.decoder import get_config

    cfg = get_config("small")
    torch.manual_seed(0)
    sd = {}
    h, f = cfg.hidden, cfg.ffn
    sd["model.embed_tokens.weight"] = torch.randn(cfg.vocab_size, h).numpy()
    # a peaked lm_head (logit std ~6): the two paths' weights differ by bf16 rounding of the
    # dequantized values, which must not flip near-tie greedy picks of a random model
    sd["lm_head.weight"] = (torch.randn(cfg.vocab_size, h) * 0.2).numpy()
    sd["model.norm.weight"] = np.ones(h, np.float32)
    for i in range(cfg.layers):
        p = f"model.layers.{i}."
        sd[p + "input_layernorm.weight"] = np.ones(h, np.float32)
        sd[p + "post_attention_layernorm.weight"] = np.ones(h, np.float32)
        sd[p + "self_attn.q_proj.weight"] = (torch.randn(cfg.heads * cfg.head_dim, h) * 0.02).numpy()
        sd[p + "self_attn.k_proj.weight"] = (torch.randn(cfg.kv_heads * cfg.head_dim, h) * 0.02).numpy()
        sd[p + "self_attn.v_proj.weight"] = (torch.randn(cfg.kv_heads * cfg.head_dim, h) * 0.02).numpy()
        sd[p + "self_attn.o_proj.weight"] = (torch.randn(h, cfg.heads * cfg.head_dim) * 0.005).numpy()
        sd[p + "mlp.gate_proj.weight"] = (torch.randn(f, h) * 0.02).numpy()
        sd[p + "mlp.up_proj.weight"] = (torch.randn(f, h) * 0.02).numpy()
        sd[p + "mlp.down_proj.weight"] = (torch.randn(h, f) * 0.005).numpy()
    qt = {"output.weight": G.Q6_K, "token_embd.weight": G.Q4_K}
    for i in range(cfg.layers):
        qt[f"blk.{i}.attn_v.weight"] = G.Q6_K
        qt[f"blk.{i}.ffn_down.weight"] = G.Q6_K if i % 2 == 0 else G.Q4_K
    path = tmp_path / "q4km.gguf"
    G.write_llama_gguf(path, cfg, sd, qtypes=qt, default_qtype=G.Q4_K)
    wq = DecoderWeights.from_gguf(path, "cuda")
    assert wq.qlayers is not None and wq.q_lm_head is not None and "Q6_K" in wq.gguf_types
    import os
    logits, models = [], []
    for flag in ("1", "0"):
        os.environ["CFC_DECODE_QGEMV"] = flag
        try:
            models.append(DecoderModel(wq))
        finally:
            os.environ.pop("CFC_DECODE_QGEMV", None)
    assert models[0].decode_qgemv and not models[1].decode_qgemv
    # prefill two prompts once, then ONE decode step through each path on the same cache (the
    # step rewrites the same slot): logits agree to the bf16 rounding of the dequantized weights
    lens = [300, 45]
    i32 = dict(dtype=torch.int32, device="cuda")
    kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, "cuda")
    tables = [list(range(0, 12)), list(range(12, 16))]
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist() for n in lens]
    ids = torch.tensor(prompts[0] + prompts[1], **i32)
    pos = torch.tensor(list(range(lens[0])) + list(range(lens[1])), **i32)
    slots = torch.tensor([tables[s][p // KV_BLOCK] * KV_BLOCK + p % KV_BLOCK for s in (0, 1) for p in range(lens[s])],
                         **i32)
    bt = torch.tensor([tables[0], tables[1] + [0] * 8], **i32)
    models[1].forward_prefill(ids, pos, slots, torch.tensor([0, lens[0], sum(lens)], **i32),
                              torch.tensor(lens, **i32), bt, kv)
    nxt = torch.tensor([5, 9], **i32)
    dpos = torch.tensor(lens, **i32)
    dslots = torch.tensor([tables[s][n // KV_BLOCK] * KV_BLOCK + n % KV_BLOCK for s, n in enumerate(lens)], **i32)
    for m in models:
        hidden = m.forward_decode(nxt, dpos, dslots, dpos + 1, bt, kv, part_blocks=4)
        logits.append(m.logits(hidden).float().cpu())
    a, b = logits
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert float(cos.min()) > 0.999, cos
    assert float((a - b).abs().max()) < 0.05 * float(b.std()) * 10, (a - b).abs().max()


def test_hip_summarizer_loads_gguf(tmp_path, monkeypatch):
    """LLM_BACKEND_TYPE=hip with LLAMA_ARG_MODEL pointing at a GGUF (the reference compose's
    variable): weights and tokenizer come from the file; summaries decode through the engine."""
    from copilot_for_consensus_amd.config import loader
    from copilot_for_consensus_amd.summarization import Thread, create_llm_backend

    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)]
    chars = sorted(set("abcdefghijklmnopqrstuvwxyz:.,"))
    toks += ["▁"] + chars + ["▁" + c for c in chars]
    types = [2, 3, 3] + [6] * 256 + [1] * (len(toks) - 259)
    cfg = DecoderConfig("tiny-gguf", len(toks), 128, 2, 2, 1, 64, 256, max_positions=1024)
    rng = np.random.default_rng(0)
    sd = {"model.embed_tokens.weight": rng.standard_normal((cfg.vocab_size, 128)).astype(np.float32),
          "lm_head.weight": rng.standard_normal((cfg.vocab_size, 128)).astype(np.float32) * 0.05,
          "model.norm.weight": np.ones(128, np.float32)}
    for i in range(2):
        p = f"model.layers.{i}."
        for n, shape in (("self_attn.q_proj", (128, 128)), ("self_attn.k_proj", (64, 128)),
                         ("self_attn.v_proj", (64, 128)), ("self_attn.o_proj", (128, 128)),
                         ("mlp.gate_proj", (256, 128)), ("mlp.up_proj", (256, 128)), ("mlp.down_proj", (128, 256))):
            sd[p + n + ".weight"] = rng.standard_normal(shape).astype(np.float32) * 0.05
        sd[p + "input_layernorm.weight"] = np.ones(128, np.float32)
        sd[p + "post_attention_layernorm.weight"] = np.ones(128, np.float32)
    path = tmp_path / "tiny.gguf"
    G.write_llama_gguf(path, cfg, sd, tokens=toks, token_types=types, default_qtype=G.F32)
    monkeypatch.setenv("LLAMA_ARG_MODEL", str(path))
    monkeypatch.setenv("LLM_DEVICE", "cpu")
    monkeypatch.setenv("LLM_MAX_NEW_TOKENS", "6")
    adapter = loader.load_adapter_config("llm_backend")
    assert adapter.driver_config["gguf_path"] == str(path)   # LLAMA_ARG_MODEL maps onto the hip driver
    s = create_llm_backend(adapter, kv_cache_tokens=4096)
    assert s.cfg.name == "tiny-gguf" and s.tokenizer.vocab_size == len(toks)
    out = s.summarize(Thread("t1", ["alpha beta"], prompt="summarize: the thread."))
    assert out.tokens_prompt > 3 and 1 <= out.tokens_completion <= 6 and out.llm_backend == "hip"
