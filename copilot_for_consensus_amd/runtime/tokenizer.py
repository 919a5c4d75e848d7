"""Python front-ends of the C++ tokenizers (csrc/runtime/tokenizer.cpp).

* :class:`BPETokenizer` -- SentencePiece-style BPE for the Mistral/Llama decoder.  Loads an HF
  ``tokenizer.json`` (BPE model) when a checkpoint is available; otherwise trains a 32000-entry
  vocabulary with the native trainer on the synthetic corpus (random-init weights need a
  tokenizer of the right vocabulary size, not a specific one).
* :class:`WordPieceTokenizer` -- BERT uncased WordPiece for the encoder.  Loads ``vocab.txt`` or
  derives a 30522-entry vocabulary from the trained BPE pieces (word-initial pieces, ``##``
  continuations), with BERT's special-token ids ([PAD]=0 [UNK]=100 [CLS]=101 [SEP]=102).
Trained vocabularies are cached as JSON under ``_lib/tokenizers`` (deterministic, git-ignored).

Replaces the HF tokenizers that run inside SentenceTransformer.encode / AutoTokenizer
(sentence_transformer_provider.py:93, huggingface_provider.py:92-101) and inside the llama.cpp /
Ollama servers (llamacpp_summarizer.py:108).
"""
from __future__ import annotations

import ctypes
import json
import os
import re
import threading
import unicodedata
from pathlib import Path

import numpy as np

from ..ops._native import runtime

CACHE_DIR = Path(__file__).resolve().parent.parent / "_lib" / "tokenizers"
_lock = threading.Lock()


def _c(s: str) -> tuple[bytes, int]:
    b = s.encode("utf-8")
    return b, len(b)


ENCODE_THREADS = max(1, min(16, int(os.environ.get("CFC_TOKENIZER_THREADS", "0")) or (os.cpu_count() or 1)))


def _batch_raw(fn, handle, texts: list[str], cap: int) -> tuple[np.ndarray, np.ndarray]:
    """Thread-parallel C++ encode of many texts: (ids [n, cap] int32, lengths [n] int32).  The BPE
    encoders report each text's full length (> cap = overflow); the WordPiece encoder stops at cap,
    so its lengths are capped (== cap may mean longer) -- it can only be used truncating."""
    bs = [t.encode("utf-8") for t in texts]
    offs = np.zeros(len(bs) + 1, dtype=np.int64)
    np.cumsum([len(b) for b in bs], out=offs[1:])
    buf = b"".join(bs)
    out = np.empty((len(bs), cap), dtype=np.int32)
    lens = np.empty(len(bs), dtype=np.int32)
    fn(handle, buf, offs.ctypes.data, len(bs), cap, out.ctypes.data, lens.ctypes.data,
       min(ENCODE_THREADS, max(1, len(bs) // 4)))
    return out, lens


def _batch(fn, handle, texts: list[str], cap: int, truncate: bool = False,
           capped_lengths: bool = False) -> list[list[int] | None]:
    """As _batch_raw, as lists.  Results longer than ``cap`` come back as None (caller re-encodes
    them singly) unless ``truncate``, which keeps their first ``cap`` ids.  ``capped_lengths``: the
    encoder stops at cap (WordPiece), so overflow is undetectable and only ``truncate`` is valid."""
    if capped_lengths and not truncate:
        raise ValueError("an encoder that stops at cap reports capped lengths: truncate=True required")
    out, lens = _batch_raw(fn, handle, texts, cap)
    return [out[i, :min(lens[i], cap)].tolist() if (truncate or lens[i] <= cap) else None for i in range(len(texts))]


class BPETokenizer:
    SPLIT_EVERY_MARK, SPLIT_SENTENCEPIECE = 0, 1
    PREPEND_UNLESS_PRESENT, PREPEND_ALWAYS, PREPEND_NEVER = 0, 1, 2

    def __init__(self, vocab: list[str], merges: list[tuple[int, int]], bos_id: int = 1, eos_id: int = 2,
                 split_mode: int = 0, prepend_mode: int = 0):
        """``split_mode`` / ``prepend_mode``: see csrc/runtime/tokenizer.cpp (HF Metaspace(split) =
        0/0, HF Llama-2/Mistral files with Prepend+Replace normalizers and no pre-tokenizer = 1/1)."""
        self.vocab = vocab
        self.bos_id, self.eos_id = bos_id, eos_id
        self._lib = runtime()
        self._h = self._lib.cfc_bpe_create()
        if self._lib.cfc_bpe_set_mode(self._h, int(split_mode), int(prepend_mode)) != 0:
            raise ValueError(f"bad BPE modes split={split_mode} prepend={prepend_mode}")
        for i, t in enumerate(vocab):
            b, n = _c(t)
            self._lib.cfc_bpe_add_token(self._h, b, n, i)
        tok2id = {t: i for i, t in enumerate(vocab)}
        for rank, (a, b) in enumerate(merges):
            merged = tok2id.get(vocab[a] + vocab[b])
            if merged is not None:
                self._lib.cfc_bpe_add_merge(self._h, a, b, rank, merged)
        self._lib.cfc_bpe_finalize(self._h)
        self._buf = np.empty(1 << 16, dtype=np.int32)
        self._enc_lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.cfc_bpe_destroy(h)
            self._h = None

    @property
    def vocab_size(self) -> int:
        return len(self.vocab)

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        b, n = _c(text)
        with self._enc_lock:
            cap = len(self._buf)
            k = self._lib.cfc_bpe_encode(self._h, b, n, self._buf.ctypes.data, cap)
            if k > cap:
                self._buf = np.empty(k * 2, dtype=np.int32)
                k = self._lib.cfc_bpe_encode(self._h, b, n, self._buf.ctypes.data, len(self._buf))
            ids = self._buf[:k].tolist()
        return ([self.bos_id] + ids) if add_bos else ids

    def encode_batch(self, texts: list[str], add_bos: bool = True, cap: int = 16384) -> list[list[int]]:
        res = _batch(self._lib.cfc_bpe_encode_batch, self._h, texts, cap)
        out = []
        for t, ids in zip(texts, res):
            if ids is None:
                out.append(self.encode(t, add_bos))
            else:
                out.append(([self.bos_id] + ids) if add_bos else ids)
        return out

    # decode() drops a leading space of the whole text (SentencePiece "▁" prefix)
    strips_leading_space = True

    def token_bytes(self, i: int) -> bytes:
        """Bytes token ``i`` contributes to decode() output (byte tokens <0xNN>, "▁" -> space;
        BOS / EOS contribute nothing) -- the stop-string matcher's view of the text."""
        if i in (self.bos_id, self.eos_id) or not 0 <= i < len(self.vocab):
            return b""
        t = self.vocab[i]
        if len(t) == 6 and t.startswith("<0x") and t.endswith(">"):
            return bytes([int(t[3:5], 16)])
        return t.replace("\u2581", " ").encode("utf-8")

    def decode(self, ids: list[int]) -> str:
        arr = np.asarray([i for i in ids if i not in (self.bos_id, self.eos_id)], dtype=np.int32)
        cap = max(64, 16 * len(arr))
        out = ctypes.create_string_buffer(cap)
        n = self._lib.cfc_bpe_decode(self._h, arr.ctypes.data, len(arr), out, cap)
        return out.raw[:min(n, cap)].decode("utf-8", errors="replace")

    # ---------------------------------------------------------------- constructors
    @classmethod
    def from_hf_json(cls, path) -> "BPETokenizer":
        d = json.loads(Path(path).read_text())
        model = d["model"]
        if model.get("type") != "BPE":
            raise ValueError("tokenizer.json is not a BPE model")
        v = model["vocab"]
        vocab = [None] * (max(v.values()) + 1)
        for t, i in v.items():
            vocab[i] = t
        for at in d.get("added_tokens", []):
            if at["id"] < len(vocab):
                vocab[at["id"]] = at["content"]
        vocab = [t if t is not None else f"<unused{i}>" for i, t in enumerate(vocab)]
        merges = []
        for m in model["merges"]:
            a, b = m.split(" ", 1) if isinstance(m, str) else m
            if a in v and b in v:
                merges.append((v[a], v[b]))
        specials = {at["content"]: at["id"] for at in d.get("added_tokens", [])}
        split_mode, prepend_mode = _sentencepiece_modes(d)
        return cls(vocab, merges, specials.get("<s>", 1), specials.get("</s>", 2), split_mode, prepend_mode)

    @classmethod
    def train(cls, corpus: str, vocab_size: int = 32000) -> "BPETokenizer":
        vocab, pairs = train_bpe(corpus, vocab_size)
        return cls(vocab, pairs)


def _flatten_steps(node: dict | None, key: str) -> list[dict]:
    if not node:
        return []
    if node.get("type") == "Sequence":
        return [x for sub in node.get(key, []) for x in _flatten_steps(sub, key)]
    return [node]


def _sentencepiece_modes(d: dict) -> tuple[int, int]:
    """(split_mode, prepend_mode) of an HF tokenizer.json's SentencePiece-style pipeline."""
    pre = _flatten_steps(d.get("pre_tokenizer"), "pretokenizers")
    norm = _flatten_steps(d.get("normalizer"), "normalizers")
    kinds = {p.get("type") for p in pre}
    if kinds - {"Metaspace"}:
        raise NotImplementedError(f"pre-tokenizers {sorted(kinds)} are not SentencePiece-style (byte-level BPE "
                                  "tokenizer.json files are not supported by BPETokenizer)")
    if pre:
        m = pre[0]
        scheme = m.get("prepend_scheme") or ("always" if m.get("add_prefix_space", True) else "never")
        prepend = BPETokenizer.PREPEND_NEVER if scheme == "never" else BPETokenizer.PREPEND_UNLESS_PRESENT
        split = BPETokenizer.SPLIT_EVERY_MARK if m.get("split", True) else BPETokenizer.SPLIT_SENTENCEPIECE
        return split, prepend
    prepends = [n for n in norm if n.get("type") == "Prepend"]
    return BPETokenizer.SPLIT_SENTENCEPIECE, (BPETokenizer.PREPEND_ALWAYS if prepends else BPETokenizer.PREPEND_NEVER)


def train_bpe(corpus: str, vocab_size: int) -> tuple[list[str], list[tuple[int, int]]]:
    """Native BPE training -> (vocab, merges).  Layout: <unk> <s> </s>, 256 byte tokens, the
    corpus' base characters, then one token per merge in rank order."""
    lib = runtime()
    b, n = _c(corpus)
    base_buf = ctypes.create_string_buffer(4 << 20)
    merges = np.empty(2 * vocab_size, dtype=np.int32)
    nm = lib.cfc_bpe_train(b, n, vocab_size, base_buf, merges.ctypes.data, vocab_size)
    base = [x.decode("utf-8", errors="replace") for x in base_buf.raw.split(b"\0\0", 1)[0].split(b"\0") if x]
    vocab = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)] + base
    pairs = [(int(merges[2 * i]), int(merges[2 * i + 1])) for i in range(nm)]
    for a, bb in pairs:
        vocab.append(vocab[a] + vocab[bb])
    while len(vocab) < vocab_size:
        vocab.append(f"<unused{len(vocab)}>")
    vocab = vocab[:vocab_size]
    return vocab, [p for p in pairs if max(p) < vocab_size]


_SYNTH_TOKENIZERS: dict = {}


# ------------------------------------------------------------------------------ byte-level BPE

# Llama-3's pre-tokenisation regex (tiktoken cl100k-style, digits in groups of up to 3)
LLAMA3_PATTERN = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                  r"|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2_PATTERN = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


def bytes_to_unicode() -> dict[int, str]:
    """GPT-2's reversible byte -> printable character map used by ByteLevel BPE vocabularies."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


class ByteLevelBPETokenizer:
    """Byte-level BPE (Llama-3 / GPT-style tokenizer.json): regex pre-tokenisation (``regex``
    module, Unicode classes), bytes mapped to printable stand-ins, then the native merge loop
    (csrc/runtime/tokenizer.cpp ``cfc_bpe_encode_pieces``).  Added/special tokens are matched
    verbatim before pre-tokenisation, as HF does."""

    def __init__(self, vocab: list[str], merges: list[tuple[int, int]], pattern: str = LLAMA3_PATTERN,
                 special_tokens: dict[str, int] | None = None, bos_id: int | None = None, eos_id: int | None = None,
                 add_prefix_space: bool = False):
        import regex
        self.vocab = vocab
        self._pat = regex.compile(pattern)
        self.special = dict(special_tokens or {})
        self._special_re = (regex.compile("|".join(regex.escape(t) for t in sorted(self.special, key=len, reverse=True)))
                            if self.special else None)
        self.bos_id, self.eos_id = bos_id, eos_id
        self.add_prefix_space = add_prefix_space
        self._b2u = bytes_to_unicode()
        self._u2b = {c: b for b, c in self._b2u.items()}
        self._lib = runtime()
        self._h = self._lib.cfc_bpe_create()
        for i, t in enumerate(vocab):
            b, n = _c(t)
            self._lib.cfc_bpe_add_token(self._h, b, n, i)
        tok2id = {t: i for i, t in enumerate(vocab)}
        for rank, (a, b) in enumerate(merges):
            merged = tok2id.get(vocab[a] + vocab[b])
            if merged is not None:
                self._lib.cfc_bpe_add_merge(self._h, a, b, rank, merged)
        self._lib.cfc_bpe_finalize(self._h)
        self._buf = np.empty(1 << 16, dtype=np.int32)
        self._enc_lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.cfc_bpe_destroy(h)
            self._h = None

    @property
    def vocab_size(self) -> int:
        return len(self.vocab)

    def _pieces(self, text: str) -> list[str]:
        if self.add_prefix_space and text and not text.startswith(" "):
            text = " " + text
        b2u = self._b2u
        return ["".join(b2u[x] for x in m.encode("utf-8")) for m in self._pat.findall(text)]

    def _encode_plain(self, text: str) -> list[int]:
        pieces = self._pieces(text)
        if not pieces:
            return []
        bs = [p.encode("utf-8") for p in pieces]
        offs = np.zeros(len(bs) + 1, dtype=np.int64)
        np.cumsum([len(b) for b in bs], out=offs[1:])
        with self._enc_lock:
            k = self._lib.cfc_bpe_encode_pieces(self._h, b"".join(bs), offs.ctypes.data, len(bs),
                                                self._buf.ctypes.data, len(self._buf))
            if k > len(self._buf):
                self._buf = np.empty(2 * k, dtype=np.int32)
                k = self._lib.cfc_bpe_encode_pieces(self._h, b"".join(bs), offs.ctypes.data, len(bs),
                                                    self._buf.ctypes.data, len(self._buf))
            return self._buf[:k].tolist()

    def encode(self, text: str, add_bos: bool = True) -> list[int]:
        ids: list[int] = [self.bos_id] if (add_bos and self.bos_id is not None) else []
        if self._special_re is None:
            return ids + self._encode_plain(text)
        pos = 0
        for m in self._special_re.finditer(text):
            ids += self._encode_plain(text[pos:m.start()])
            ids.append(self.special[m.group()])
            pos = m.end()
        return ids + self._encode_plain(text[pos:])

    def encode_batch(self, texts: list[str], add_bos: bool = True, cap: int = 16384) -> list[list[int]]:
        return [self.encode(t, add_bos) for t in texts]

    strips_leading_space = False

    def token_bytes(self, i: int) -> bytes:
        """Bytes token ``i`` contributes to decode() output (specials verbatim, BOS / EOS nothing)."""
        if i in (self.bos_id, self.eos_id) or not 0 <= i < len(self.vocab):
            return b""
        inv = getattr(self, "_inv_special", None)
        if inv is None:
            inv = self._inv_special = {v: k for k, v in self.special.items()}
        if i in inv:
            return inv[i].encode("utf-8")
        return bytes(self._u2b[c] for c in self.vocab[i] if c in self._u2b)

    def decode(self, ids: list[int]) -> str:
        skip = {i for i in (self.bos_id, self.eos_id) if i is not None}
        inv_special = {v: k for k, v in self.special.items()}
        out = bytearray()
        for i in ids:
            if i in skip:
                continue
            if i in inv_special:
                out += inv_special[i].encode("utf-8")
                continue
            out += bytes(self._u2b[c] for c in self.vocab[i] if c in self._u2b)
        return out.decode("utf-8", errors="replace")

    @classmethod
    def from_hf_json(cls, path) -> "ByteLevelBPETokenizer":
        d = json.loads(Path(path).read_text())
        model = d["model"]
        if model.get("type") != "BPE":
            raise ValueError("tokenizer.json is not a BPE model")
        pre = _flatten_steps(d.get("pre_tokenizer"), "pretokenizers")
        kinds = [p.get("type") for p in pre]
        if "ByteLevel" not in kinds:
            raise NotImplementedError("not a byte-level BPE tokenizer.json (use BPETokenizer)")
        pattern, add_prefix = GPT2_PATTERN, False
        for p in pre:
            if p.get("type") == "Split":
                pat = p.get("pattern", {})
                pattern = pat.get("Regex") or __import__("regex").escape(pat.get("String", ""))
            elif p.get("type") == "ByteLevel":
                add_prefix = bool(p.get("add_prefix_space", False))
                if p.get("use_regex", True) and "Split" not in kinds:
                    pattern = GPT2_PATTERN
        v = model["vocab"]
        added = {at["content"]: at["id"] for at in d.get("added_tokens", [])}
        size = max(list(v.values()) + list(added.values())) + 1
        vocab = [f"<unused{i}>" for i in range(size)]
        for t, i in v.items():
            vocab[i] = t
        for t, i in added.items():
            vocab[i] = t
        merges = []
        for m in model["merges"]:
            a, b = m.split(" ", 1) if isinstance(m, str) else m
            if a in v and b in v:
                merges.append((v[a], v[b]))
        bos = added.get("<|begin_of_text|>", added.get("<s>"))
        eos = added.get("<|end_of_text|>", added.get("</s>", added.get("<|endoftext|>")))
        return cls(vocab, merges, pattern, added, bos, eos, add_prefix)


def load_hf_tokenizer(path):
    """BPETokenizer (SentencePiece-style) or ByteLevelBPETokenizer, from the tokenizer.json's pipeline."""
    d = json.loads(Path(path).read_text())
    kinds = {p.get("type") for p in _flatten_steps(d.get("pre_tokenizer"), "pretokenizers")}
    return ByteLevelBPETokenizer.from_hf_json(path) if "ByteLevel" in kinds else BPETokenizer.from_hf_json(path)


def synthetic_bpe(vocab_size: int = 32000, corpus_words: int = 800_000) -> BPETokenizer:
    """Deterministic BPE trained on the synthetic mailing-list distribution (cached on disk)."""
    key = ("bpe", vocab_size)
    with _lock:
        if key in _SYNTH_TOKENIZERS:
            return _SYNTH_TOKENIZERS[key]
        path = CACHE_DIR / f"synthetic_bpe_{vocab_size}.json"
        if path.exists():
            d = json.loads(path.read_text())
            tok = BPETokenizer(d["vocab"], [tuple(m) for m in d["merges"]])
        else:
            from ..utils.synthetic import SyntheticArchive
            vocab, pairs = train_bpe(SyntheticArchive(seed=777).corpus(corpus_words), vocab_size)
            CACHE_DIR.mkdir(parents=True, exist_ok=True)
            tmp = path.with_suffix(f".{os.getpid()}.tmp")  # per-process: ranks may build it together
            tmp.write_text(json.dumps({"vocab": vocab, "merges": pairs}))
            tmp.replace(path)
            tok = BPETokenizer(vocab, pairs)
        _SYNTH_TOKENIZERS[key] = tok
        return tok




def bert_normalize(text: str, lowercase: bool = True) -> str:
    """HF BertNormalizer + the Unicode part of BertPreTokenizer, for non-ASCII text: drop control
    characters, map Unicode spaces to ' ', strip accents (NFD, drop Mn) and lower-case (uncased
    models), and space-pad Unicode punctuation so the C++ splitter isolates it.  Pure-ASCII text
    is returned unchanged: the C++ splitter treats \t \n \r as spaces and drops the other ASCII
    control characters (and DEL) itself, as HF does -- no per-text regex scan."""
    if text.isascii():
        return text
    out = []
    for c in text:
        cp = ord(c)
        if cp == 0 or cp == 0xFFFD:
            continue
        cat = unicodedata.category(c)
        if c in "\t\n\r" or cat == "Zs":
            out.append(" ")
        elif cat in ("Cc", "Cf"):
            continue
        else:
            out.append(c)
    t = "".join(out)
    if lowercase:
        t = "".join(c for c in unicodedata.normalize("NFD", t) if unicodedata.category(c) != "Mn").lower()
    return "".join(f" {c} " if ord(c) > 127 and unicodedata.category(c).startswith("P") else c for c in t)


class WordPieceTokenizer:
    PAD, UNK, CLS, SEP, MASK = 0, 100, 101, 102, 103

    def __init__(self, vocab: list[str], lowercase: bool = True, max_length: int = 512):
        self.vocab = vocab
        self.max_length = max_length
        self.lowercase = lowercase
        self._lib = runtime()
        tok2id = {t: i for i, t in enumerate(vocab)}
        self.unk_id = tok2id.get("[UNK]", self.UNK)
        self.cls_id = tok2id.get("[CLS]", self.CLS)
        self.sep_id = tok2id.get("[SEP]", self.SEP)
        self._h = self._lib.cfc_wp_create(self.unk_id, self.cls_id, self.sep_id, 1 if lowercase else 0)
        for i, t in enumerate(vocab):
            b, n = _c(t)
            self._lib.cfc_wp_add_token(self._h, b, n, i)
        self._buf = np.empty(1 << 16, dtype=np.int32)
        self._enc_lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.cfc_wp_destroy(h)
            self._h = None

    def encode(self, text: str, max_length: int | None = None) -> list[int]:
        """[CLS] pieces [SEP], truncated to max_length (sentence-transformers behaviour)."""
        L = max_length or self.max_length
        b, n = _c(bert_normalize(text, self.lowercase))
        with self._enc_lock:
            k = self._lib.cfc_wp_encode(self._h, b, n, self._buf.ctypes.data, len(self._buf))
            if k > len(self._buf):
                self._buf = np.empty(2 * k, dtype=np.int32)
                k = self._lib.cfc_wp_encode(self._h, b, n, self._buf.ctypes.data, len(self._buf))
            ids = self._buf[:min(k, L - 2)].tolist()
        return [self.cls_id] + ids + [self.sep_id]

    def encode_batch(self, texts: list[str], max_length: int | None = None) -> list[list[int]]:
        L = max_length or self.max_length
        # truncation makes every result fit: ask for L-2 pieces, longer texts are simply cut
        texts = [bert_normalize(t, self.lowercase) for t in texts]
        res = _batch(self._lib.cfc_wp_encode_batch, self._h, texts, max(1, L - 2), truncate=True,
                     capped_lengths=True)
        return [[self.cls_id] + ids + [self.sep_id] for ids in res]

    def encode_packed(self, texts: list[str], max_length: int | None = None) -> tuple[np.ndarray, np.ndarray]:
        """encode_batch as the encoder consumes it, with no per-token Python work: every text's
        [CLS] pieces [SEP] concatenated (ids int32 [T]) and the boundaries (cu_seqlens int32 [n+1])."""
        L = max_length or self.max_length
        cap = max(1, L - 2)
        texts = [bert_normalize(t, self.lowercase) for t in texts]
        out, lens = _batch_raw(self._lib.cfc_wp_encode_batch, self._h, texts, cap)
        lens = np.minimum(lens, cap)
        cu = np.zeros(len(texts) + 1, dtype=np.int32)
        np.cumsum(lens + 2, out=cu[1:])
        ids = np.empty(int(cu[-1]), dtype=np.int32)
        ids[cu[:-1]] = self.cls_id
        ids[cu[1:] - 1] = self.sep_id
        body = np.arange(cap, dtype=np.int32)[None, :]
        mask = body < lens[:, None]
        ids[((cu[:-1] + 1)[:, None] + body)[mask]] = out[mask]
        return ids, cu

    @classmethod
    def from_vocab_txt(cls, path, **kw) -> "WordPieceTokenizer":
        return cls(Path(path).read_text(encoding="utf-8").splitlines(), **kw)


def synthetic_wordpiece(vocab_size: int = 30522, max_length: int = 256) -> WordPieceTokenizer:
    key = ("wp", vocab_size, max_length)
    with _lock:
        if key in _SYNTH_TOKENIZERS:
            return _SYNTH_TOKENIZERS[key]
    bpe = synthetic_bpe()
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    seen = set(vocab)
    for c in "abcdefghijklmnopqrstuvwxyz0123456789.,!?;:'\"()-_/<>@[]{}#$%&*+=|~^`\\":
        for t in (c, "##" + c):
            if t not in seen:
                seen.add(t)
                vocab.append(t)
    for t in bpe.vocab[259:]:
        if t.startswith("<unused"):
            continue
        piece = t[1:] if t.startswith("▁") else "##" + t
        piece = piece.lower()
        if piece and piece != "##" and piece not in seen:
            seen.add(piece)
            vocab.append(piece)
        if len(vocab) >= vocab_size:
            break
    while len(vocab) < vocab_size:
        vocab.append(f"[unused{len(vocab)}]")
    tok = WordPieceTokenizer(vocab[:vocab_size], max_length=max_length)
    with _lock:
        _SYNTH_TOKENIZERS[key] = tok
    return tok
