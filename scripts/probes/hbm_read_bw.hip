// HBM read-bandwidth roofline probe for MI355X: streams a buffer with 16-byte loads (optionally
// nontemporal), several loads in flight per lane, and reports GB/s.  Used to bound what the
// KV-bandwidth-bound paged decode attention can reach (scripts/bench_attn.py).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
#define CK(x) (void)(x)

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) read_kernel(const uint4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT) {
        const u32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p + i + u * stride));
        v[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = p[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n; i += stride) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

template <int U, bool NT>
static float run(const uint4* d, size_t n, uint32_t* out, int blocks) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) read_kernel<U, NT><<<blocks, 256>>>(d, n, out);
  CK(hipEventRecord(a));
  const int iters = 20;
  for (int it = 0; it < iters; ++it) read_kernel<U, NT><<<blocks, 256>>>(d, n, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return (float)(n * 16.0 * iters / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atoll(argv[1]) : 4096ll) << 20;  // MiB
  const size_t n = bytes / 16;
  uint4* d;
  uint32_t* out;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  CK(hipMemset(d, 1, bytes));
  CK(hipDeviceSynchronize());
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("buffer %zu MiB, %d CUs\n", bytes >> 20, cus);
  for (int per_cu : {2, 4, 8, 16}) {
    const int blocks = cus * per_cu;
    printf("blocks/CU=%2d  u1 %7.0f  u4 %7.0f  u8 %7.0f  u8-nt %7.0f GB/s\n", per_cu, run<1, false>(d, n, out, blocks),
           run<4, false>(d, n, out, blocks), run<8, false>(d, n, out, blocks), run<8, true>(d, n, out, blocks));
  }
  CK(hipFree(d));
  CK(hipFree(out));
  return 0;
}
