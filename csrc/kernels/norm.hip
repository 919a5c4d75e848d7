// Normalisation kernels (decoder RMSNorm, encoder LayerNorm) with fused residual / bias /
// embedding-gather prologues.  Memory-bound: one workgroup per row, 16-byte vector access,
// the row is held in registers between the statistics pass and the normalise pass so each
// element is read from HBM exactly once.
//
// Reference parity: these replace the normalisation inside the engines the reference calls
// (llama.cpp RMSNorm behind llamacpp_summarizer.py:108; BERT LayerNorm inside
// SentenceTransformer.encode, sentence_transformer_provider.py:93).
#include "common.h"

namespace {

// F8: out is e4m3fn of the bf16-rounded normalised row divided by a per-row scale
// (scale[row] = amax / 448) -- the W8A8 projection's activation quantisation fused into the norm
// that produces it, so the row makes no extra HBM round trip through a bf16 tensor.
template <int VPT, bool F8>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(void* __restrict__ out, float* __restrict__ scale,
                                                      uint16_t* __restrict__ residual,
                                                      const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                      int dim, float eps, int add_residual) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = dim >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * dim);
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * dim);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      unpack8(xr[c], v[i]);
      if (add_residual) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        // residual <- x + residual (rounded to bf16 exactly like the stored stream)
        uint4 p = pack8(v[i]);
        rr[c] = p;
        unpack8(p, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)dim + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  if constexpr (!F8) {
    uint4* orow = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + (size_t)row * dim);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
        float g[8], o[8];
        unpack8(wr[c], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * g[j];
        orow[c] = pack8(o);
      }
    }
  } else {
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
        float g[8];
        unpack8(wr[c], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[i][j] = bf2f(f2bf(v[i][j] * inv * g[j]));   // the bf16 value the unfused norm would store
          amax = fmaxf(amax, fabsf(v[i][j]));
        }
      }
    }
    amax = block_max(amax, red);
    const float s = amax > 0.f ? amax / 448.f : 1.f, rs = 1.f / s;
    if (threadIdx.x == 0) scale[row] = s;
    uint2* orow = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(out) + (size_t)row * dim);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] *= rs;
        orow[c] = pack8_fp8(v[i]);
      }
    }
  }
}

// LayerNorm with optional fused prologue:
//   mode 0: y = LN(x)
//   mode 1: y = LN(x + bias + residual)          (post-LN BERT block: dense out + residual)
//   mode 2: y = LN(word_emb[ids] + pos_emb[pos] + type_emb[0])   (BERT embedding layer)
template <int VPT>
__global__ void __launch_bounds__(1024) layernorm_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ x,
                                                        const uint16_t* __restrict__ bias, const uint16_t* __restrict__ residual,
                                                        const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta,
                                                        const int32_t* __restrict__ ids, const int32_t* __restrict__ pos,
                                                        const uint16_t* __restrict__ pos_emb, const uint16_t* __restrict__ type_emb,
                                                        int dim, float eps, int mode) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = dim >> 3;
  const uint4* xr;
  if (mode == 2) xr = reinterpret_cast<const uint4*>(x + (size_t)ids[row] * dim);
  else xr = reinterpret_cast<const uint4*>(x + (size_t)row * dim);
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      unpack8(xr[c], v[i]);
      if (mode == 1) {
        float b[8], r[8];
        unpack8(reinterpret_cast<const uint4*>(bias)[c], b);
        unpack8(reinterpret_cast<const uint4*>(residual + (size_t)row * dim)[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += b[j] + r[j];
      } else if (mode == 2) {
        float p[8], t[8];
        unpack8(reinterpret_cast<const uint4*>(pos_emb + (size_t)pos[row] * dim)[c], p);
        unpack8(reinterpret_cast<const uint4*>(type_emb)[c], t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += p[j] + t[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = block_sum(s, red) / (float)dim;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; sq += d * d; }
    }
  }
  const float inv = rsqrtf(block_sum(sq, red) / (float)dim + eps);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * dim);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float g[8], b[8], o[8];
      unpack8(reinterpret_cast<const uint4*>(gamma)[c], g);
      unpack8(reinterpret_cast<const uint4*>(beta)[c], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * g[j] + b[j];
      orow[c] = pack8(o);
    }
  }
}

// One 16-B vector per thread whenever the row fits in a 1024-thread block: at decode (128 rows)
// a row is a single load round trip instead of VPT dependent ones (10 us -> ~3 us per call).
inline int pick_block(int nvec) { return nvec >= 1024 ? 1024 : ((nvec + 63) / 64) * 64; }

template <bool F8>
int launch_rmsnorm(void* out, float* scale, void* residual, const void* x, const void* w, int rows, int dim, float eps,
                   int add_residual, hipStream_t stream) {
  const int nvec = dim / 8, block = pick_block(nvec);
  const int vpt = (nvec + block - 1) / block;
  auto r = (uint16_t*)residual;
  auto xi = (const uint16_t*)x; auto wi = (const uint16_t*)w;
  switch (vpt) {
    case 1: rmsnorm_kernel<1, F8><<<rows, block, 0, stream>>>(out, scale, r, xi, wi, dim, eps, add_residual); break;
    case 2: rmsnorm_kernel<2, F8><<<rows, block, 0, stream>>>(out, scale, r, xi, wi, dim, eps, add_residual); break;
    case 3: case 4: rmsnorm_kernel<4, F8><<<rows, block, 0, stream>>>(out, scale, r, xi, wi, dim, eps, add_residual); break;
    case 5: case 6: case 7: case 8:
      rmsnorm_kernel<8, F8><<<rows, block, 0, stream>>>(out, scale, r, xi, wi, dim, eps, add_residual); break;
    default: return -2;
  }
  return CFC_CHECK_LAUNCH();
}

}  // namespace

// out = RMSNorm(x [+ residual]) * w.  When add_residual != 0, residual is updated in place to
// x + residual (the pre-norm residual stream of a Llama/Mistral block).
CFC_API int cfc_rmsnorm(void* out, void* residual, const void* x, const void* w, int rows, int dim, float eps,
                        int add_residual, hipStream_t stream) {
  if (dim % 8 != 0 || rows <= 0) return -1;
  return launch_rmsnorm<false>(out, nullptr, residual, x, w, rows, dim, eps, add_residual, stream);
}

// FP8 output: out [rows, dim] e4m3fn, scale [rows] f32 with RMSNorm(...) ~= out * scale.
CFC_API int cfc_rmsnorm_fp8(void* out, float* scale, void* residual, const void* x, const void* w, int rows, int dim,
                            float eps, int add_residual, hipStream_t stream) {
  if (dim % 8 != 0 || rows <= 0) return -1;
  return launch_rmsnorm<true>(out, scale, residual, x, w, rows, dim, eps, add_residual, stream);
}

CFC_API int cfc_layernorm(void* out, const void* x, const void* bias, const void* residual, const void* gamma,
                          const void* beta, const int32_t* ids, const int32_t* pos, const void* pos_emb,
                          const void* type_emb, int rows, int dim, float eps, int mode, hipStream_t stream) {
  if (dim % 8 != 0 || rows <= 0) return -1;
  const int nvec = dim / 8, block = pick_block(nvec);
  const int vpt = (nvec + block - 1) / block;
#define LN_ARGS (uint16_t*)out, (const uint16_t*)x, (const uint16_t*)bias, (const uint16_t*)residual, \
    (const uint16_t*)gamma, (const uint16_t*)beta, ids, pos, (const uint16_t*)pos_emb, (const uint16_t*)type_emb, dim, eps, mode
  switch (vpt) {
    case 1: layernorm_kernel<1><<<rows, block, 0, stream>>>(LN_ARGS); break;
    case 2: layernorm_kernel<2><<<rows, block, 0, stream>>>(LN_ARGS); break;
    case 3: case 4: layernorm_kernel<4><<<rows, block, 0, stream>>>(LN_ARGS); break;
    case 5: case 6: case 7: case 8: layernorm_kernel<8><<<rows, block, 0, stream>>>(LN_ARGS); break;
    default: return -2;
  }
#undef LN_ARGS
  return CFC_CHECK_LAUNCH();
}
