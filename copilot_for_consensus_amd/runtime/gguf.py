"""GGUF checkpoints: reader, writer, ggml block quantization formats.

The reference serves its summarizer from a GGUF file through llama.cpp
(docker-compose.infra.yml:296-298: ``mistral-7b-instruct-v0.2.Q4_K_M.gguf``; Ollama pulls the same
kind of file, docker-compose.infra.yml:276-281), so a user switching over arrives with GGUF
weights.  This module reads them without llama.cpp or the ``gguf`` Python package:

* the container format (GGUF v2/v3: header, typed metadata key/values, tensor infos, aligned
  data section) -- tensors are numpy views of one read-only memory map, nothing is unpickled;
* the ggml block formats F32, F16, BF16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0 and the k-quants Q4_K,
  Q5_K, Q6_K: numpy dequantizers written from the ggml block layouts (``block_q4_K``: fp16 d,
  fp16 dmin, 12 bytes of 6-bit scales/mins, 128 bytes of nibbles per 256 weights; ``block_q6_K``:
  128 bytes low nibbles, 64 bytes high 2-bit pairs, 16 int8 scales, fp16 d), plus quantizers for
  Q8_0 / Q4_0 / Q4_K / Q6_K so tests can write files (any valid block encoding is a valid file;
  the dequantizer is what must match ggml);
* the llama-architecture conventions: tensor names (``blk.N.attn_q.weight`` ...), the q/k row
  permutation llama.cpp's converter applies for its interleaved RoPE (undone here: this
  framework's RoPE is rotate-half, as HF), and the SentencePiece vocabulary with scores
  (``tokenizer.ggml.*``) turned into ranked merges for the C++ BPE tokenizer.

The GPU side (dequant-to-bf16 kernels for loading, and the quantized GEMV that streams Q4_K / Q6_K
/ Q8_0 blocks straight from HBM at single-stream decode) lives in csrc/kernels/quant.hip.
"""
from __future__ import annotations

import dataclasses
import json
import struct
from pathlib import Path

import numpy as np

GGUF_MAGIC = 0x46554747   # "GGUF" little-endian
DEFAULT_ALIGNMENT = 32
QK_K = 256

# ggml_type ids (ggml.h)
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 0, 1, 2, 3, 6, 7, 8, 9
Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 10, 11, 12, 13, 14, 15
BF16 = 30
TYPE_NAMES = {F32: "F32", F16: "F16", Q4_0: "Q4_0", Q4_1: "Q4_1", Q5_0: "Q5_0", Q5_1: "Q5_1", Q8_0: "Q8_0",
              Q8_1: "Q8_1", Q2_K: "Q2_K", Q3_K: "Q3_K", Q4_K: "Q4_K", Q5_K: "Q5_K", Q6_K: "Q6_K", Q8_K: "Q8_K",
              BF16: "BF16"}
# (weights per block, bytes per block)
BLOCK = {F32: (1, 4), F16: (1, 2), BF16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q5_0: (32, 22), Q5_1: (32, 24),
         Q8_0: (32, 34), Q2_K: (256, 84), Q3_K: (256, 110), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210)}

# metadata value types
_U8, _I8, _U16, _I16, _U32, _I32, _F32, _BOOL, _STR, _ARR, _U64, _I64, _F64 = range(13)
_SCALAR = {_U8: "<B", _I8: "<b", _U16: "<H", _I16: "<h", _U32: "<I", _I32: "<i", _F32: "<f", _BOOL: "<?",
           _U64: "<Q", _I64: "<q", _F64: "<d"}
_NP = {_U8: np.uint8, _I8: np.int8, _U16: np.uint16, _I16: np.int16, _U32: np.uint32, _I32: np.int32,
       _F32: np.float32, _BOOL: np.bool_, _U64: np.uint64, _I64: np.int64, _F64: np.float64}


class GGUFError(ValueError):
    pass


@dataclasses.dataclass
class TensorInfo:
    name: str
    shape: tuple[int, ...]          # numpy order: (ne[n-1], ..., ne[0]); ne[0] is contiguous
    ggml_type: int
    offset: int                     # from the start of the data section
    data: np.ndarray | None = None  # raw bytes (uint8 view of the memory map)

    @property
    def type_name(self) -> str:
        return TYPE_NAMES.get(self.ggml_type, str(self.ggml_type))

    @property
    def n_elements(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1

    @property
    def nbytes(self) -> int:
        per, size = BLOCK[self.ggml_type]
        return self.n_elements // per * size


class GGUFReader:
    """Memory-mapped GGUF file: ``metadata`` dict and ``tensors`` (name -> TensorInfo with a raw
    uint8 view).  :meth:`tensor` returns float32 numpy, dequantized."""

    def __init__(self, path):
        self.path = Path(path)
        self._mm = np.memmap(self.path, dtype=np.uint8, mode="r")
        buf = self._mm
        self._pos = 0
        magic, self.version = struct.unpack_from("<II", buf, 0)
        if magic != GGUF_MAGIC:
            raise GGUFError(f"{path}: not a GGUF file")
        if self.version not in (2, 3):
            raise GGUFError(f"{path}: GGUF version {self.version} not supported")
        n_tensors, n_kv = struct.unpack_from("<QQ", buf, 8)
        self._pos = 24
        self.metadata: dict = {}
        for _ in range(n_kv):
            key = self._str()
            vtype = self._u32()
            self.metadata[key] = self._value(vtype)
        infos = []
        for _ in range(n_tensors):
            name = self._str()
            nd = self._u32()
            ne = struct.unpack_from(f"<{nd}Q", buf, self._pos)
            self._pos += 8 * nd
            t = self._u32()
            off = struct.unpack_from("<Q", buf, self._pos)[0]
            self._pos += 8
            if t not in BLOCK:
                raise GGUFError(f"tensor {name}: ggml type {t} not supported")
            infos.append(TensorInfo(name, tuple(int(x) for x in reversed(ne)), t, int(off)))
        align = int(self.metadata.get("general.alignment", DEFAULT_ALIGNMENT))
        self.data_offset = (self._pos + align - 1) // align * align
        self.tensors: dict[str, TensorInfo] = {}
        for ti in infos:
            a = self.data_offset + ti.offset
            if a + ti.nbytes > len(buf):
                raise GGUFError(f"tensor {ti.name} runs past the end of the file")
            ti.data = buf[a:a + ti.nbytes]
            self.tensors[ti.name] = ti

    # -- primitive readers
    def _u32(self) -> int:
        v = struct.unpack_from("<I", self._mm, self._pos)[0]
        self._pos += 4
        return v

    def _str(self) -> str:
        n = struct.unpack_from("<Q", self._mm, self._pos)[0]
        self._pos += 8
        s = bytes(self._mm[self._pos:self._pos + n]).decode("utf-8", errors="replace")
        self._pos += n
        return s

    def _value(self, vtype):
        if vtype in _SCALAR:
            fmt = _SCALAR[vtype]
            v = struct.unpack_from(fmt, self._mm, self._pos)[0]
            self._pos += struct.calcsize(fmt)
            return v
        if vtype == _STR:
            return self._str()
        if vtype == _ARR:
            et = self._u32()
            n = struct.unpack_from("<Q", self._mm, self._pos)[0]
            self._pos += 8
            if et in _NP:
                a = np.frombuffer(self._mm, dtype=_NP[et], count=n, offset=self._pos).copy()
                self._pos += a.nbytes
                return a
            return [self._value(et) for _ in range(n)]
        raise GGUFError(f"metadata value type {vtype} not supported")

    def tensor(self, name: str) -> np.ndarray:
        ti = self.tensors[name]
        return dequantize(ti.data, ti.ggml_type, ti.shape)


# ------------------------------------------------------------------------------- writer

class GGUFWriter:
    """Minimal GGUF v3 writer (tests, exporting checkpoints).  ``add_tensor`` takes float arrays
    (quantized here) or pre-quantized raw bytes with ``raw_type``."""

    def __init__(self, arch: str = "llama", alignment: int = DEFAULT_ALIGNMENT):
        self.kv: list[tuple[str, int, object]] = []
        self.tensors: list[tuple[str, tuple[int, ...], int, bytes]] = []
        self.alignment = alignment
        self.add("general.architecture", arch)
        if alignment != DEFAULT_ALIGNMENT:
            self.add("general.alignment", alignment, _U32)

    def add(self, key: str, value, vtype: int | None = None, elem_type: int | None = None):
        if vtype is None:
            if isinstance(value, bool):
                vtype = _BOOL
            elif isinstance(value, int):
                vtype = _U32 if 0 <= value < 2 ** 32 else _I64
            elif isinstance(value, float):
                vtype = _F32
            elif isinstance(value, str):
                vtype = _STR
            elif isinstance(value, (list, tuple, np.ndarray)):
                vtype = _ARR
            else:
                raise TypeError(f"{key}: {type(value)}")
        if vtype == _ARR and elem_type is None:
            v0 = value[0] if len(value) else ""
            elem_type = _STR if isinstance(v0, str) else (_F32 if isinstance(v0, (float, np.floating)) else _I32)
        self.kv.append((key, vtype, (value, elem_type)))

    def add_tensor(self, name: str, arr: np.ndarray | None, qtype: int = F32, raw: bytes | None = None,
                   shape: tuple[int, ...] | None = None):
        if raw is None:
            arr = np.ascontiguousarray(arr, dtype=np.float32)
            shape = arr.shape
            raw = quantize(arr, qtype).tobytes()
        self.tensors.append((name, tuple(shape), qtype, raw))

    @staticmethod
    def _enc_str(s: str) -> bytes:
        b = s.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    def _enc_value(self, vtype, payload) -> bytes:
        value, et = payload
        if vtype in _SCALAR:
            return struct.pack(_SCALAR[vtype], value)
        if vtype == _STR:
            return self._enc_str(value)
        if vtype == _ARR:
            out = struct.pack("<IQ", et, len(value))
            if et in _NP:
                return out + np.asarray(value, dtype=_NP[et]).tobytes()
            return out + b"".join(self._enc_value(et, (v, None)) for v in value)
        raise TypeError(vtype)

    def write(self, path):
        head = struct.pack("<IIQQ", GGUF_MAGIC, 3, len(self.tensors), len(self.kv))
        parts = [head]
        for key, vtype, payload in self.kv:
            parts += [self._enc_str(key), struct.pack("<I", vtype), self._enc_value(vtype, payload)]
        off = 0
        offsets = []
        for name, shape, qtype, raw in self.tensors:
            offsets.append(off)
            ne = tuple(reversed(shape))
            parts += [self._enc_str(name), struct.pack(f"<I{len(ne)}Q", len(ne), *ne), struct.pack("<IQ", qtype, off)]
            off += (len(raw) + self.alignment - 1) // self.alignment * self.alignment
        header = b"".join(parts)
        pad = (-len(header)) % self.alignment
        with open(path, "wb") as fh:
            fh.write(header + b"\0" * pad)
            for (name, shape, qtype, raw), o in zip(self.tensors, offsets):
                fh.write(raw)
                fh.write(b"\0" * ((-len(raw)) % self.alignment))


# ------------------------------------------------------------------------------- block formats

def _f16(b: np.ndarray) -> np.ndarray:
    return b.view(np.float16).astype(np.float32)


def _blocks(raw: np.ndarray, qtype: int) -> np.ndarray:
    per, size = BLOCK[qtype]
    raw = np.asarray(raw, dtype=np.uint8).reshape(-1)
    if raw.size % size:
        raise GGUFError(f"{TYPE_NAMES[qtype]}: {raw.size} bytes is not a whole number of blocks")
    return raw.reshape(-1, size)


def _scale_min_k4(sc: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """The 8 (scale, min) 6-bit pairs of a Q4_K / Q5_K block from its 12 scale bytes (ggml
    get_scale_min_k4).  sc: [nb, 12] uint8 -> two [nb, 8] float arrays."""
    sc = sc.astype(np.uint8)
    d = np.empty((sc.shape[0], 8), np.uint8)
    m = np.empty((sc.shape[0], 8), np.uint8)
    d[:, :4] = sc[:, 0:4] & 63
    m[:, :4] = sc[:, 4:8] & 63
    d[:, 4:] = (sc[:, 8:12] & 0xF) | ((sc[:, 0:4] >> 6) << 4)
    m[:, 4:] = (sc[:, 8:12] >> 4) | ((sc[:, 4:8] >> 6) << 4)
    return d.astype(np.float32), m.astype(np.float32)


def _pack_scale_min_k4(d: np.ndarray, m: np.ndarray) -> np.ndarray:
    """Inverse of :func:`_scale_min_k4` for 6-bit ints d, m [nb, 8] -> [nb, 12] uint8."""
    d = d.astype(np.uint8)
    m = m.astype(np.uint8)
    out = np.zeros((d.shape[0], 12), np.uint8)
    out[:, 0:4] = (d[:, :4] & 63) | ((d[:, 4:] >> 4) << 6)
    out[:, 4:8] = (m[:, :4] & 63) | ((m[:, 4:] >> 4) << 6)
    out[:, 8:12] = (d[:, 4:] & 0xF) | ((m[:, 4:] & 0xF) << 4)
    return out


def dequantize(raw: np.ndarray, qtype: int, shape) -> np.ndarray:
    """ggml blocks -> float32 array of ``shape`` (numpy order, last dim contiguous)."""
    n = int(np.prod(shape)) if len(shape) else 1
    raw = np.asarray(raw, dtype=np.uint8).reshape(-1)
    if qtype == F32:
        return raw.view(np.float32)[:n].reshape(shape).copy()
    if qtype == F16:
        return raw.view(np.float16)[:n].astype(np.float32).reshape(shape)
    if qtype == BF16:
        return (raw.view(np.uint16)[:n].astype(np.uint32) << 16).view(np.float32).reshape(shape)
    b = _blocks(raw, qtype)
    nb = b.shape[0]
    if qtype == Q8_0:
        d = _f16(b[:, 0:2].copy())
        q = b[:, 2:34].view(np.int8).astype(np.float32)
        y = d * q
    elif qtype in (Q4_0, Q4_1):
        d = _f16(b[:, 0:2].copy())
        o = 4 if qtype == Q4_1 else 2
        qs = b[:, o:o + 16]
        q = np.concatenate([qs & 0xF, qs >> 4], 1).astype(np.float32)
        y = d * (q - 8.0) if qtype == Q4_0 else d * q + _f16(b[:, 2:4].copy())
    elif qtype in (Q5_0, Q5_1):
        d = _f16(b[:, 0:2].copy())
        o = 4 if qtype == Q5_1 else 2
        qh = b[:, o:o + 4].copy().view(np.uint32)[:, 0]
        qs = b[:, o + 4:o + 20]
        j = np.arange(16, dtype=np.uint32)
        hi0 = ((qh[:, None] >> j) << 4) & 0x10
        hi1 = (qh[:, None] >> (j + 12)) & 0x10
        q = np.concatenate([(qs & 0xF) | hi0, (qs >> 4) | hi1], 1).astype(np.float32)
        y = d * (q - 16.0) if qtype == Q5_0 else d * q + _f16(b[:, 2:4].copy())
    elif qtype in (Q4_K, Q5_K):
        d = _f16(b[:, 0:2].copy())
        dmin = _f16(b[:, 2:4].copy())
        sc, mn = _scale_min_k4(b[:, 4:16])
        if qtype == Q4_K:
            qs, qh = b[:, 16:144], None
        else:
            qh, qs = b[:, 16:48], b[:, 48:176]
        y = np.empty((nb, QK_K), np.float32)
        for j in range(4):                      # 64-weight groups
            ql = qs[:, 32 * j:32 * j + 32]
            lo = (ql & 0xF).astype(np.float32)
            hi = (ql >> 4).astype(np.float32)
            if qh is not None:
                lo += ((qh >> (2 * j)) & 1).astype(np.float32) * 16
                hi += ((qh >> (2 * j + 1)) & 1).astype(np.float32) * 16
            y[:, 64 * j:64 * j + 32] = d * sc[:, 2 * j:2 * j + 1] * lo - dmin * mn[:, 2 * j:2 * j + 1]
            y[:, 64 * j + 32:64 * j + 64] = d * sc[:, 2 * j + 1:2 * j + 2] * hi - dmin * mn[:, 2 * j + 1:2 * j + 2]
    elif qtype == Q6_K:
        ql, qh = b[:, 0:128], b[:, 128:192]
        sc = b[:, 192:208].view(np.int8).astype(np.float32)
        d = _f16(b[:, 208:210].copy())
        y = np.empty((nb, QK_K), np.float32)
        for h in range(2):                      # 128-weight halves
            L, H = ql[:, 64 * h:64 * h + 64], qh[:, 32 * h:32 * h + 32]
            q1 = ((L[:, :32] & 0xF) | ((H & 3) << 4)).astype(np.float32) - 32
            q2 = ((L[:, 32:] & 0xF) | (((H >> 2) & 3) << 4)).astype(np.float32) - 32
            q3 = ((L[:, :32] >> 4) | (((H >> 4) & 3) << 4)).astype(np.float32) - 32
            q4 = ((L[:, 32:] >> 4) | (((H >> 6) & 3) << 4)).astype(np.float32) - 32
            s = sc[:, 8 * h:8 * h + 8]
            for k, q in enumerate((q1, q2, q3, q4)):
                # weights l (0..31) of this quarter: scale index 2k + l // 16
                y[:, 128 * h + 32 * k:128 * h + 32 * k + 16] = d * s[:, 2 * k:2 * k + 1] * q[:, :16]
                y[:, 128 * h + 32 * k + 16:128 * h + 32 * k + 32] = d * s[:, 2 * k + 1:2 * k + 2] * q[:, 16:]
    else:
        raise GGUFError(f"dequantize: {TYPE_NAMES.get(qtype, qtype)} not supported")
    return y.reshape(-1)[:n].reshape(shape)


def quantize(x: np.ndarray, qtype: int) -> np.ndarray:
    """float32 -> raw ggml block bytes (uint8).  Straightforward (min/max, round-to-nearest)
    encoders: enough to write valid files; llama.cpp's quantizers search scales more carefully."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    if qtype == F32:
        return x.view(np.uint8).copy()
    if qtype == F16:
        return x.astype(np.float16).view(np.uint8).copy()
    if qtype == BF16:
        u = x.view(np.uint32)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        return r.view(np.uint8).copy()
    per, size = BLOCK[qtype]
    if x.size % per:
        raise GGUFError(f"{TYPE_NAMES[qtype]}: {x.size} values is not a whole number of {per}-blocks")
    xb = x.reshape(-1, per)
    nb = xb.shape[0]
    out = np.zeros((nb, size), np.uint8)
    if qtype == Q8_0:
        amax = np.abs(xb).max(1)
        d = (amax / 127.0).astype(np.float16)
        inv = np.where(d.astype(np.float32) > 0, 1.0 / np.maximum(d.astype(np.float32), 1e-30), 0.0)
        q = np.clip(np.rint(xb * inv[:, None]), -127, 127).astype(np.int8)
        out[:, 0:2] = d.reshape(-1, 1).view(np.uint8)
        out[:, 2:34] = q.view(np.uint8)
    elif qtype == Q4_0:
        idx = np.abs(xb).argmax(1)
        mx = xb[np.arange(nb), idx]
        d = (mx / -8.0).astype(np.float16)
        df = d.astype(np.float32)
        inv = np.where(df != 0, 1.0 / np.where(df != 0, df, 1.0), 0.0)
        q = np.clip(np.floor(xb * inv[:, None] + 8.5), 0, 15).astype(np.uint8)
        out[:, 0:2] = d.reshape(-1, 1).view(np.uint8)
        out[:, 2:18] = q[:, :16] | (q[:, 16:] << 4)
    elif qtype == Q4_K:
        sub = xb.reshape(nb, 8, 32)
        mn = np.minimum(sub.min(2), 0.0)
        mx = sub.max(2)
        scale = (mx - mn) / 15.0
        d = (scale.max(1) / 63.0).astype(np.float16)
        dmin = ((-mn).max(1) / 63.0).astype(np.float16)
        df, dmf = d.astype(np.float32), dmin.astype(np.float32)
        sq = np.clip(np.rint(scale / np.where(df > 0, df, 1.0)[:, None]), 0, 63)
        mq = np.clip(np.rint(-mn / np.where(dmf > 0, dmf, 1.0)[:, None]), 0, 63)
        eff_s = df[:, None] * sq
        eff_m = dmf[:, None] * mq
        q = np.clip(np.rint((sub + eff_m[:, :, None]) / np.where(eff_s > 0, eff_s, 1.0)[:, :, None]), 0, 15)
        q = np.where(eff_s[:, :, None] > 0, q, 0).astype(np.uint8).reshape(nb, 256)
        out[:, 0:2] = d.reshape(-1, 1).view(np.uint8)
        out[:, 2:4] = dmin.reshape(-1, 1).view(np.uint8)
        out[:, 4:16] = _pack_scale_min_k4(sq, mq)
        for j in range(4):
            out[:, 16 + 32 * j:16 + 32 * j + 32] = q[:, 64 * j:64 * j + 32] | (q[:, 64 * j + 32:64 * j + 64] << 4)
    elif qtype == Q6_K:
        sub = xb.reshape(nb, 16, 16)
        amax = np.abs(sub).max(2)
        scale = amax / 31.0
        d = (scale.max(1) / 127.0).astype(np.float16)
        df = d.astype(np.float32)
        sq = np.clip(np.rint(scale / np.where(df > 0, df, 1.0)[:, None]), -127, 127)
        eff = df[:, None] * sq
        q = np.clip(np.rint(sub / np.where(eff > 0, eff, 1.0)[:, :, None]), -32, 31)
        q = (np.where(eff[:, :, None] > 0, q, 0) + 32).astype(np.uint8).reshape(nb, 256)
        ql = np.zeros((nb, 128), np.uint8)
        qh = np.zeros((nb, 64), np.uint8)
        for h in range(2):
            Q = q[:, 128 * h:128 * h + 128]
            q1, q2, q3, q4 = Q[:, 0:32], Q[:, 32:64], Q[:, 64:96], Q[:, 96:128]
            ql[:, 64 * h:64 * h + 32] = (q1 & 0xF) | ((q3 & 0xF) << 4)
            ql[:, 64 * h + 32:64 * h + 64] = (q2 & 0xF) | ((q4 & 0xF) << 4)
            qh[:, 32 * h:32 * h + 32] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
        out[:, 0:128] = ql
        out[:, 128:192] = qh
        out[:, 192:208] = sq.astype(np.int8).view(np.uint8)
        out[:, 208:210] = d.reshape(-1, 1).view(np.uint8)
    else:
        raise GGUFError(f"quantize: {TYPE_NAMES.get(qtype, qtype)} not supported")
    return out.reshape(-1)


# ------------------------------------------------------------------------------- llama conventions

def permute_qk(w: np.ndarray, n_head: int) -> np.ndarray:
    """HF rotate-half q/k rows -> llama.cpp's interleaved-pair order (its converter's permute)."""
    return w.reshape(n_head, 2, w.shape[0] // n_head // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def unpermute_qk(w: np.ndarray, n_head: int) -> np.ndarray:
    """Inverse of :func:`permute_qk` (GGUF llama q/k rows -> HF rotate-half order)."""
    return w.reshape(n_head, w.shape[0] // n_head // 2, 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def unpermute_qk_rows(n_rows: int, n_head: int) -> np.ndarray:
    """Row index map r_hf -> r_gguf, so that hf_rows = gguf_rows[map] (applies to quantized rows
    too: the permutation moves whole rows)."""
    return unpermute_qk(np.arange(n_rows), n_head)


def config_from_gguf(md: dict, tensor_names=None, name: str = "gguf"):
    """DecoderConfig from GGUF metadata (architectures llama / mistral); ``tensor_names`` tells
    whether the file has its own ``output.weight`` (else the embeddings are tied)."""
    from ..models.decoder import DecoderConfig

    arch = md.get("general.architecture", "llama")
    if arch not in ("llama", "mistral"):
        raise GGUFError(f"architecture {arch!r} is not supported (llama / mistral)")

    def g(key, default=None):
        v = md.get(f"{arch}.{key}", default)
        if v is None:
            raise GGUFError(f"metadata {arch}.{key} missing")
        return v

    hidden = int(g("embedding_length"))
    heads = int(g("attention.head_count"))
    vocab = md.get(f"{arch}.vocab_size")
    if vocab is None:
        toks = md.get("tokenizer.ggml.tokens")
        vocab = len(toks) if toks is not None else None
    if vocab is None:
        raise GGUFError("vocabulary size unknown (no vocab_size and no tokenizer.ggml.tokens)")
    window = md.get(f"{arch}.attention.sliding_window")
    return DecoderConfig(
        name=str(md.get("general.name", name)), vocab_size=int(vocab), hidden=hidden, layers=int(g("block_count")),
        heads=heads, kv_heads=int(g("attention.head_count_kv", heads)),
        head_dim=int(md.get(f"{arch}.attention.key_length", md.get(f"{arch}.rope.dimension_count", hidden // heads))),
        ffn=int(g("feed_forward_length")), rope_theta=float(md.get(f"{arch}.rope.freq_base", 10000.0)),
        rms_eps=float(md.get(f"{arch}.attention.layer_norm_rms_epsilon", 1e-5)),
        max_positions=int(md.get(f"{arch}.context_length", 4096)),
        tie_embeddings=tensor_names is not None and "output.weight" not in tensor_names,
        bos_id=int(md.get("tokenizer.ggml.bos_token_id", 1)), eos_id=int(md.get("tokenizer.ggml.eos_token_id", 2)),
        sliding_window=int(window) if window else None)


def tokenizer_from_gguf(md: dict):
    """C++ BPE tokenizer from ``tokenizer.ggml.*`` metadata.

    * ``llama`` (SentencePiece): llama.cpp merges the adjacent pair whose concatenation is the
      highest-scoring vocabulary piece; the equivalent ranked merge list is every split (a, b) of
      every normal piece, ranked by the piece's score.  Byte fallback uses the <0xXX> pieces.
    * ``gpt2`` (byte-level BPE, Llama-3): the file carries its merges."""
    from .tokenizer import BPETokenizer, ByteLevelBPETokenizer

    model = md.get("tokenizer.ggml.model", "llama")
    tokens = [str(t) for t in md["tokenizer.ggml.tokens"]]
    bos, eos = int(md.get("tokenizer.ggml.bos_token_id", 1)), int(md.get("tokenizer.ggml.eos_token_id", 2))
    tok2id = {t: i for i, t in enumerate(tokens)}
    if model == "gpt2":
        merges = []
        for m in md.get("tokenizer.ggml.merges", []):
            a, b = str(m).split(" ", 1)
            if a in tok2id and b in tok2id:
                merges.append((tok2id[a], tok2id[b]))
        t = ByteLevelBPETokenizer(tokens, merges)
        t.bos_id, t.eos_id = bos, eos
        return t
    if model != "llama":
        raise GGUFError(f"tokenizer model {model!r} is not supported")
    scores = np.asarray(md.get("tokenizer.ggml.scores", np.zeros(len(tokens))), dtype=np.float64)
    ttype = np.asarray(md.get("tokenizer.ggml.token_type", np.ones(len(tokens))), dtype=np.int64)
    normal = [i for i in range(len(tokens)) if ttype[i] == 1 and len(tokens[i]) > 1]
    normal.sort(key=lambda i: (-scores[i], i))
    merges = []
    for i in normal:
        t = tokens[i]
        for k in range(1, len(t)):
            a, b = tok2id.get(t[:k]), tok2id.get(t[k:])
            if a is not None and b is not None and ttype[a] == 1 and ttype[b] == 1:
                merges.append((a, b))
    return BPETokenizer(tokens, merges, bos, eos, BPETokenizer.SPLIT_SENTENCEPIECE,
                        BPETokenizer.PREPEND_ALWAYS if md.get("tokenizer.ggml.add_space_prefix", True)
                        else BPETokenizer.PREPEND_NEVER)


def llama_tensor_names(layers: int) -> dict[str, str]:
    """GGUF llama tensor names -> the HF names they correspond to."""
    m = {"token_embd.weight": "model.embed_tokens.weight", "output_norm.weight": "model.norm.weight",
         "output.weight": "lm_head.weight"}
    for i in range(layers):
        for g, h in (("attn_norm", "input_layernorm"), ("ffn_norm", "post_attention_layernorm"),
                     ("attn_q", "self_attn.q_proj"), ("attn_k", "self_attn.k_proj"), ("attn_v", "self_attn.v_proj"),
                     ("attn_output", "self_attn.o_proj"), ("ffn_gate", "mlp.gate_proj"), ("ffn_up", "mlp.up_proj"),
                     ("ffn_down", "mlp.down_proj")):
            m[f"blk.{i}.{g}.weight"] = f"model.layers.{i}.{h}.weight"
    return m


def write_llama_gguf(path, cfg, tensors: dict[str, np.ndarray], qtypes: dict[str, int] | None = None,
                     default_qtype: int = F32, tokens: list[str] | None = None, scores=None, token_types=None):
    """Write an HF-named llama/mistral state dict as a llama-architecture GGUF (q/k rows permuted
    the way llama.cpp's converter does).  ``qtypes``: per-GGUF-name quantization; 1-D tensors are
    always F32, as llama.cpp stores norms."""
    w = GGUFWriter("llama")
    w.add("general.name", cfg.name)
    w.add("llama.context_length", int(cfg.max_positions))
    w.add("llama.embedding_length", int(cfg.hidden))
    w.add("llama.block_count", int(cfg.layers))
    w.add("llama.feed_forward_length", int(cfg.ffn))
    w.add("llama.attention.head_count", int(cfg.heads))
    w.add("llama.attention.head_count_kv", int(cfg.kv_heads))
    w.add("llama.rope.dimension_count", int(cfg.head_dim))
    w.add("llama.attention.key_length", int(cfg.head_dim))
    w.add("llama.rope.freq_base", float(cfg.rope_theta))
    w.add("llama.attention.layer_norm_rms_epsilon", float(cfg.rms_eps))
    w.add("llama.vocab_size", int(cfg.vocab_size))
    if cfg.sliding_window:
        w.add("llama.attention.sliding_window", int(cfg.sliding_window))
    w.add("tokenizer.ggml.model", "llama")
    w.add("tokenizer.ggml.bos_token_id", int(cfg.bos_id))
    w.add("tokenizer.ggml.eos_token_id", int(cfg.eos_id))
    if tokens is not None:
        w.add("tokenizer.ggml.tokens", list(tokens), _ARR, _STR)
        w.add("tokenizer.ggml.scores", np.asarray(scores if scores is not None else -np.arange(len(tokens)),
                                                  dtype=np.float32), _ARR, _F32)
        w.add("tokenizer.ggml.token_type", np.asarray(token_types if token_types is not None
                                                      else np.ones(len(tokens)), dtype=np.int32), _ARR, _I32)
    names = llama_tensor_names(cfg.layers)
    qtypes = qtypes or {}
    for g, h in names.items():
        if h not in tensors:
            continue
        a = np.asarray(tensors[h], dtype=np.float32)
        if g.endswith("attn_q.weight"):
            a = permute_qk(a, cfg.heads)
        elif g.endswith("attn_k.weight"):
            a = permute_qk(a, cfg.kv_heads)
        qt = F32 if a.ndim == 1 else qtypes.get(g, default_qtype)
        w.add_tensor(g, a, qt)
    w.write(path)


def summary(path) -> dict:
    r = GGUFReader(path)
    types: dict[str, int] = {}
    for t in r.tensors.values():
        types[t.type_name] = types.get(t.type_name, 0) + t.n_elements
    return {"version": r.version, "tensors": len(r.tensors), "architecture": r.metadata.get("general.architecture"),
            "weights_by_type": types, "bytes": sum(t.nbytes for t in r.tensors.values())}


if __name__ == "__main__":   # python -m copilot_for_consensus_amd.runtime.gguf FILE
    import sys
    print(json.dumps(summary(sys.argv[1]), indent=1))
