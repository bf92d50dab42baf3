// Probe: does v_exp_f32 (transcendental) share the SIMD's VALU issue with
// plain fp32 VALU, and how much VALU hides beside bf16 MFMAs?  Cycles per
// SIMD at 2.4 GHz for: exp only, add only, exp and add in one wave (1:1,
// 1:2), exp waves beside add waves (half the blocks each), and an MFMA
// chain interleaved with a fixed exp/add mix (the KDE pass's per-tile work:
// 5 MFMA : 16 exp : 32 add).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/issue_mix.hip -o /tmp/issue_mix
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define R8(X) X X X X X X X X
#define EXP(a) asm volatile("v_exp_f32 %0, %0" : "+v"(a));
#define ADD(a) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(s));

__global__ __launch_bounds__(256) void k_exp(float* out, int iters, float s) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  for (int i = 0; i < iters; ++i) { R8(EXP(a0) EXP(a1) EXP(a2) EXP(a3)) }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}
__global__ __launch_bounds__(256) void k_add(float* out, int iters, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  for (int i = 0; i < iters; ++i) { R8(ADD(a0) ADD(a1) ADD(a2) ADD(a3)) }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}
// 1 exp : 1 add, same wave
__global__ __launch_bounds__(256) void k_mix11(float* out, int iters, float s) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, b0 = a0 + 2, b1 = a0 + 3;
  for (int i = 0; i < iters; ++i) { R8(EXP(a0) ADD(b0) EXP(a1) ADD(b1)) }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + b0 + b1;
}
// 1 exp : 2 add, same wave
__global__ __launch_bounds__(256) void k_mix12(float* out, int iters, float s) {
  float a0 = threadIdx.x * 1e-3f, b0 = a0 + 2, b1 = a0 + 3, a1 = a0 + 4;
  for (int i = 0; i < iters; ++i) { R8(EXP(a0) ADD(b0) ADD(b1) EXP(a1) ADD(b0) ADD(b1)) }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + b0 + b1;
}
// even blocks exp only, odd blocks add only (co-resident on every SIMD)
__global__ __launch_bounds__(256) void k_split(float* out, int iters, float s) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  if (blockIdx.x & 1) {
    for (int i = 0; i < iters; ++i) { R8(ADD(a0) ADD(a1) ADD(a2) ADD(a3)) }
  } else {
    for (int i = 0; i < iters; ++i) { R8(EXP(a0) EXP(a1) EXP(a2) EXP(a3)) }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

// MFMA chain (5 per step) with a VALU mix per step: NE exps and NA adds,
// issued in program order MFMA, valu..., MFMA, valu... (PLACE = 1) or
// MFMAs first then all VALU (PLACE = 0).
template <int NM, int NE, int NA, int PLACE>
__global__ __launch_bounds__(256) void k_mfma_mix(float* out, int iters, float s) {
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (short)(0x3F80 + threadIdx.x % 7); b[e] = (short)(0x3F00 + e); }
  f32x16 acc = {};
  float v[16];
  for (int k = 0; k < 16; ++k) v[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
    if (PLACE == 1) {
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        if (NM) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
        for (int k = m * NE / 5; k < (m + 1) * NE / 5; ++k) EXP(v[k & 15])
#pragma unroll
        for (int k = m * NA / 5; k < (m + 1) * NA / 5; ++k) ADD(v[(k + 3) & 15])
      }
    } else {
#pragma unroll
      for (int m = 0; m < NM; ++m)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < NE; ++k) EXP(v[k & 15])
#pragma unroll
      for (int k = 0; k < NA; ++k) ADD(v[(k + 3) & 15])
    }
  }
  float t = 0;
  for (int k = 0; k < 16; ++k) t += v[k] + acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main() {
  float* out;
  hipMalloc(&out, 8192 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms;
  // per-instruction kernels: blocks = 256 CUs * 8 (8 waves per SIMD)
  auto run = [&](const char* name, void (*k)(float*, int, float), int blocks,
                 int iters, double winstr_per_iter) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    const double waves = blocks * 4.0;
    const double per_simd = waves / 1024.0;  // waves per SIMD (sequential work)
    const double cyc = ms * 1e-3 * 2.4e9 / (per_simd * iters * winstr_per_iter);
    printf("%-26s blocks %5d  %.3f ms  %.2f cyc per step per wave-slot\n", name,
           blocks, ms, cyc);
  };
  const int it = 4096;
  for (int bpc : {1, 2, 8}) {
    const int B = 256 * bpc;
    printf("-- %d waves per SIMD\n", bpc);
    run("exp (1 instr)", k_exp, B, it, 32);
    run("add (1 instr)", k_add, B, it, 32);
    run("mix 1e:1a (per pair)", k_mix11, B, it, 16);
    run("mix 1e:2a (per e+2a)", k_mix12, B, it, 16);
    run("split exp|add blocks (per instr)", k_split, B, it, 32);
    run("mfma5 e16 a32 interleaved", k_mfma_mix<5, 16, 32, 1>, B, it / 4, 1);
    run("mfma5 e16 a32 clustered", k_mfma_mix<5, 16, 32, 0>, B, it / 4, 1);
    run("mfma5 only", k_mfma_mix<5, 0, 0, 1>, B, it / 4, 1);
    run("e16 a32 only (no mfma)", k_mfma_mix<0, 16, 32, 1>, B, it / 4, 1);
    run("mfma5 e16 interleaved", k_mfma_mix<5, 16, 0, 1>, B, it / 4, 1);
    run("mfma5 a32 interleaved", k_mfma_mix<5, 0, 32, 1>, B, it / 4, 1);
  }
  return 0;
}
