// Probe: does v_mfma_f32_32x32x16_bf16 round C + sum_k a_k b_k ONCE when the
// products' sum is exactly representable?  (Decides whether the KDE pass may
// fold its hi + lo add into the MFMA: DESIGN.md §4.)  For every element it
// compares D = mfma(A, B, C) with RNE(mfma(A, B, 0) + C) bit for bit.
//   hipcc --offload-arch=gfx950 -O3 mfma_chain.hip -o mfma_chain && ./mfma_chain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ inline uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ inline short bf16_of_int(int q, int e) {  // q * 2^e, |q| <= 256
  float v = ldexpf(static_cast<float>(q), e);
  return static_cast<short>(__float_as_uint(v) >> 16);
}

__global__ void probe(int iters, int mode, unsigned long long* mism,
                      unsigned long long* total) {
  const int lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  unsigned long long bad = 0, cnt = 0;
  for (int it = 0; it < iters; ++it) {
    bf16x8 a, b;
    const uint32_t base = hash(wid * 1000003u + it * 7919u);
    for (int e = 0; e < 8; ++e) {
      const uint32_t h1 = hash(base ^ (lane * 8 + e) * 2654435761u);
      const uint32_t h2 = hash(h1 + 0x9e3779b9u);
      int qa = static_cast<int>(h1 % 513) - 256;
      int qb = static_cast<int>(h2 % 513) - 256;
      if (mode == 1 && (e & 1)) {  // cancelling pairs: k odd ~ -(k even)
        const uint32_t h0 = hash(base ^ (lane * 8 + e - 1) * 2654435761u);
        qa = -(static_cast<int>(h0 % 513) - 256);
        qb = static_cast<int>(hash(h0 + 0x9e3779b9u) % 513) - 256 + (h2 & 3) - 1;
      }
      a[e] = bf16_of_int(qa, -3);
      b[e] = bf16_of_int(qb, -3);
    }
    f32x16 c;
    for (int v = 0; v < 16; ++v) {
      const uint32_t h = hash(base + lane * 16 + v + 12345u);
      // lo-like: |c| < 4 with arbitrary mantissa bits
      c[v] = (static_cast<float>(h) * 2.3283064e-10f - 0.5f) * 8.0f;
    }
    f32x16 zero = {};
    const f32x16 s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, zero, 0, 0, 0);
    const f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int v = 0; v < 16; ++v) {
      const float ref = s[v] + c[v];
      bad += (__float_as_uint(ref) != __float_as_uint(d[v]));
      ++cnt;
    }
  }
  atomicAdd(mism, bad);
  atomicAdd(total, cnt);
}

int main() {
  unsigned long long *m, *t;
  hipMalloc(&m, 8);
  hipMalloc(&t, 8);
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(m, 0, 8);
    hipMemset(t, 0, 8);
    hipLaunchKernelGGL(probe, dim3(2048), dim3(256), 0, 0, 256, mode, m, t);
    unsigned long long hm = 0, ht = 0;
    hipMemcpy(&hm, m, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    printf("mode %d (%s): %llu mismatches of %llu elements\n", mode,
           mode ? "cancelling products" : "random products", hm, ht);
  }
  return 0;
}
