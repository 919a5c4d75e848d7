"""Numerics parity with the engines the reference runs: HF ``transformers`` BertModel (what
SentenceTransformers wraps for all-MiniLM / BGE) and MistralForCausalLM / LlamaForCausalLM (what
Ollama / llama.cpp serve).  Tiny random-init HF models are saved with ``save_pretrained`` as
safetensors, loaded through this framework's checkpoint loaders, and compared with the HF fp32
forward: sentence embeddings (mean pooling + L2) and full-sequence logits through the paged-KV
prefill.  The CPU runs exercise the reference-op path; the ``gpu``-marked runs exercise the HIP
kernels (bf16 weights, so tolerances are bf16-level)."""
from __future__ import annotations

import pytest
import torch

transformers = pytest.importorskip("transformers")

from copilot_for_consensus_amd.models.decoder import DecoderModel, DecoderWeights, load_config_json  # noqa: E402
from copilot_for_consensus_amd.models.encoder import EncoderConfig, EncoderModel  # noqa: E402
from copilot_for_consensus_amd.ops import kernels as K  # noqa: E402
from copilot_for_consensus_amd.runtime.kv_cache import KV_BLOCK, PagedKVCache  # noqa: E402

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.fixture(scope="module")
def bert_dir(tmp_path_factory):
    torch.manual_seed(0)
    cfg = transformers.BertConfig(vocab_size=1000, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=512, max_position_embeddings=512, layer_norm_eps=1e-12)
    model = transformers.BertModel(cfg, add_pooling_layer=False).eval()
    d = tmp_path_factory.mktemp("bert")
    model.save_pretrained(d, safe_serialization=True)
    return d, model


@pytest.mark.parametrize("device", DEVICES)
def test_encoder_matches_hf_bert(bert_dir, device):
    d, hf = bert_dir
    ecfg = EncoderConfig("tiny-bert", vocab_size=1000, hidden=128, layers=2, heads=2, ffn=512, max_positions=512,
                         max_seq_length=512)
    mine = EncoderModel.from_safetensors(ecfg, d, device)
    g = torch.Generator().manual_seed(1)
    seqs = [torch.randint(1, 1000, (n,), generator=g).tolist() for n in (5, 17, 64, 130)]
    got = mine.encode_ids(seqs).float().cpu()
    want = []
    with torch.no_grad():
        for s in seqs:
            h = hf(input_ids=torch.tensor([s])).last_hidden_state[0]   # [n, H] fp32, no padding
            e = h.mean(0)
            want.append(e / e.norm())
    want = torch.stack(want)
    cos = (got * want).sum(1) / (got.norm(dim=1) * want.norm(dim=1))
    assert float(cos.min()) > 0.999, cos


def _hf_decoder(kind, tmp_path_factory):
    torch.manual_seed(0)
    common = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                  num_attention_heads=2, num_key_value_heads=1, head_dim=128, max_position_embeddings=4096,
                  rms_norm_eps=1e-5, tie_word_embeddings=False, bos_token_id=1, eos_token_id=2)
    if kind == "mistral":
        cfg = transformers.MistralConfig(rope_theta=1e6, sliding_window=None, **common)
        model = transformers.MistralForCausalLM(cfg)
    elif kind == "mistral_swa":    # Mistral v0.1-style sliding-window attention (window << prompt)
        cfg = transformers.MistralConfig(rope_theta=1e4, sliding_window=24, **common)
        model = transformers.MistralForCausalLM(cfg)
    elif kind == "llama":
        cfg = transformers.LlamaConfig(rope_theta=5e5, **common)
        model = transformers.LlamaForCausalLM(cfg)
    else:  # Llama-3.1 long-context RoPE frequency scaling
        scaling = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                   "original_max_position_embeddings": 64}
        cfg = transformers.LlamaConfig(rope_theta=5e5, rope_scaling=scaling, **common)
        model = transformers.LlamaForCausalLM(cfg)
    model = model.eval()
    d = tmp_path_factory.mktemp(kind)
    model.save_pretrained(d, safe_serialization=True)
    return d, model


@pytest.fixture(scope="module", params=["mistral", "mistral_swa", "llama", "llama31"])
def decoder_dir(request, tmp_path_factory):
    return _hf_decoder(request.param, tmp_path_factory)


def _our_logits(ckpt, device, ids):
    cfg = load_config_json(ckpt / "config.json")
    w = DecoderWeights.from_safetensors(cfg, ckpt, device)
    model = DecoderModel(w)
    n = len(ids)
    nblk = (n + KV_BLOCK - 1) // KV_BLOCK + 1
    kv = PagedKVCache(cfg.layers, nblk + 2, w.kv_heads, cfg.head_dim, device)
    table = list(range(1, nblk + 1))  # block 0 unused: exercises the table indirection
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device=device)  # noqa: E731
    slots = [table[p // KV_BLOCK] * KV_BLOCK + p % KV_BLOCK for p in range(n)]
    cu, ctx = [0, n], [n]
    tseq, tq0 = K.prefill_tiles(cu, K.prefill_rows(w.heads, w.kv_heads), ctx)
    hidden = model.forward_prefill(i32(ids), i32(list(range(n))), i32(slots), i32(cu), i32(ctx),
                                   i32([table]), kv, tiles=(i32(tseq), i32(tq0)))
    return model.logits(hidden).float().cpu()


@pytest.mark.parametrize("device", DEVICES)
def test_decoder_prefill_matches_hf(decoder_dir, device):
    ckpt, hf = decoder_dir
    ids = torch.randint(3, 512, (77,), generator=torch.Generator().manual_seed(5)).tolist()
    got = _our_logits(ckpt, device, ids)
    with torch.no_grad():
        want = hf(input_ids=torch.tensor([ids])).logits[0].float()
    assert got.shape == want.shape
    cos = torch.nn.functional.cosine_similarity(got, want, dim=1)
    assert float(cos.min()) > 0.9995, cos.min()
    # greedy choice agrees wherever HF's top-2 margin is clear of bf16 noise
    top2 = want.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.05 * want.std()
    assert bool((got.argmax(1) == want.argmax(1))[clear].all())
