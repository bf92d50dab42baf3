// Issue-ceiling probe for the MFMA KDE pass (measurement infrastructure,
// not part of libabc_hip.so; bench.py loads it to price its roofline).
//
// One "step" is the per-(32x32 tile, i-tile) instruction mix of the KDE
// kernels with NO memory traffic: NM v_mfma_f32_32x32x16_bf16 on one
// accumulator (random bf16 operands), NE v_exp_f32 and NA v_add_f32 on
// independent registers, the VALU spread evenly over the MFMA gaps in
// program order (the best placement a schedule can reach).  The kernel is
// launched with WPS waves per SIMD (the KDE kernels' occupancy) on every
// SIMD of the chip, so the measured time per step and SIMD is the
// throughput ceiling of that mix at the clock the chip holds under it:
//
//   t_ceiling(launch) = tiles / 1024 SIMDs * ns_per_step
//
// Mixes (PMC-counted per tile, profiles/r0*_kde_pmc*.json):
//   0: d <= 8, folded accumulation   -- 5 MFMA, 16 exp, 23 other VALU
//   1: d = 20, split accumulation    -- 11 MFMA, 16 exp, 40 other VALU
//      (the bf16 piece scheme of rounds 1-3)
//   2: d = 20, f16 pieces, split     --  9 MFMA, 16 exp, 40 other VALU
//      (the f16 and bf16 32x32x16 MFMAs issue alike)
//   3: d <= 8, f16 pieces, folded (round 4 default) -- 4 MFMA, 16 exp, 21
//      (19 in round 4; PMC, profiles/r04_kde_pmc.json: 21.5 other VALU)
//   4: d = 20, f16 pieces, folded (round 4 default) -- 9 MFMA, 16 exp, 19
//   12: mix 3 with 22 other VALU: bench.py averages 3 (21 since round 5)
//       and 12 for the PMC's 21.5 (profiles/r04_kde_pmc.json: 37.5 VALU
//       incl. 16 TRANS)
//   13: d = 20, f16 folded, the PMC's mix -- 9 MFMA, 16 exp, 28 other VALU
//       (profiles/r04_kde_d20_pmc.json: 44.2 VALU incl. 16 TRANS)
//   14-17: mix 13 plus the d = 20 kernel's memory path step by step (14 five
//       ds_read_b128 per step, 15 + a barrier per 4 steps, 16 + the LDS-DMA
//       refill of 18 fragments per barrier, 17 as 14 with four reads)
//   5-7: mix 3 plus the headline kernel's memory path (mix_mem_kernel):
//      5 two ds_read_b128 per step, 6 + a block barrier every 2 steps,
//      7 + the LDS-DMA refill of the other buffer before each barrier;
//      8 / 9 as 6 / 7 with the barrier every 4 steps (the kernel's 64-row
//      chunk: 2 j-tiles x IB = 2), 10 / 11 every 8 steps (128-row chunks)
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC issue_probe.hip \
//         -o libabc_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define ABC_EXP(a) asm volatile("v_exp_f32 %0, %0" : "+v"(a));
#define ABC_ADD(a, s) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(s));

template <int NM, int NE, int NA>
__global__ __launch_bounds__(256) void mix_kernel(float* out, int iters,
                                                  unsigned long long* cyc) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  // random-looking bf16 operands (all-zero operands raise the clock)
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
  bf16x8 a, b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h ^= h >> 13; h *= 0x5bd1e995u;
    a[e] = static_cast<short>(0x3C00 | (h & 0x7F));
    b[e] = static_cast<short>(0xBC00 | ((h >> 8) & 0x7F));
  }
  f32x16 acc = {};
  float v[16];
  const float s = 1e-7f * (threadIdx.x & 7);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = -1e-3f * (threadIdx.x + k);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
      for (int k = m * NE / NM; k < (m + 1) * NE / NM; ++k) ABC_EXP(v[k & 15])
#pragma unroll
      for (int k = m * NA / NM; k < (m + 1) * NA / NM; ++k)
        ABC_ADD(v[(k + 5) & 15], s)
    }
  }
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += v[k] + acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = t;
  if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
}

// The same mix with the headline kernel's memory path added step by step
// (variants 5-7): DSR ds_read_b128 A fragments per step (read one step
// ahead, feeding the MFMAs), a block barrier every BAR steps, and with DMA
// the LDS-DMA refill of the other buffer (8 KB per block from an L2-resident
// source, waited with vmcnt(0) before the barrier) -- the per-64-row-chunk
// pattern of kde_mfma_lds2g_kernel.
template <int NM, int NE, int NA, int DSR, int BAR, int DMA, int NF = 8>
__global__ __launch_bounds__(256) void mix_mem_kernel(float* out, int iters,
                                                      const bf16x8* __restrict__ src) {
  __shared__ bf16x8 As[2][NF][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
  for (int f = wave; f < 2 * NF; f += 4) {
    bf16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      h ^= h >> 13; h *= 0x5bd1e995u;
      x[e] = static_cast<short>(0x3C00 | (h & 0x7F));
    }
    As[f / NF][f % NF][lane] = x;
  }
  bf16x8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h ^= h >> 13; h *= 0x5bd1e995u;
    b[e] = static_cast<short>(0xBC00 | ((h >> 8) & 0x7F));
  }
  __syncthreads();
  f32x16 acc = {};
  float v[16];
  const float s = 1e-7f * (threadIdx.x & 7);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = -1e-3f * (threadIdx.x + k);
  int buf = 0;
  bf16x8 a = As[0][0][lane];
  for (int i = 0; i < iters; ++i) {
    if (BAR > 0 && i % BAR == 0) {
      if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (DMA) {
        const bf16x8* g = src + (i & 1023) * NF * 64;  // src: 1024 x 32 KiB
        for (int f = wave; f < NF; f += 4)
          __builtin_amdgcn_global_load_lds(
              g + f * 64 + lane,
              (__attribute__((address_space(3))) void*)&As[buf ^ 1][f][0], 16, 0, 0);
      }
      buf ^= 1;
    }
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      if (m < DSR) a = As[buf][(i * DSR + m + 1) % NF][lane];
#pragma unroll
      for (int k = m * NE / NM; k < (m + 1) * NE / NM; ++k) ABC_EXP(v[k & 15])
#pragma unroll
      for (int k = m * NA / NM; k < (m + 1) * NA / NM; ++k)
        ABC_ADD(v[(k + 5) & 15], s)
    }
  }
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += v[k] + acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NM, int NE, int NA, int DSR, int BAR, int DMA, int NF = 8>
double time_mem_mix(int waves_per_simd, int iters, int cus, float* out,
                    const bf16x8* src) {
  const int blocks = cus * waves_per_simd;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((mix_mem_kernel<NM, NE, NA, DSR, BAR, DMA, NF>), dim3(blocks),
                       dim3(256), 0, 0, out, iters, src);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best * 1e6 / (static_cast<double>(waves_per_simd) * iters);
}

// mean over blocks of the shader-clock cycles a wave ran (s_memtime), per
// launch millisecond: the clock the chip held under the mix (GHz)
double g_clock_ghz = 0.0;

double mean_clock_ghz(const unsigned long long* cyc, int blocks, float ms) {
  unsigned long long* h = new unsigned long long[blocks];
  double c = 0.0;
  if (hipMemcpy(h, cyc, static_cast<size_t>(blocks) * 8, hipMemcpyDeviceToHost) ==
      hipSuccess) {
    for (int b = 0; b < blocks; ++b) c += static_cast<double>(h[b]);
    c /= blocks;
  }
  delete[] h;
  return ms > 0.0f ? c / (ms * 1e6) : 0.0;
}

// The same work in the v_mfma_f32_16x16x32_f16 shape (variants 20-21, VERDICT
// r05 item 2): a 32 x 32 tile step becomes four 16 x 16 tiles, each one hi
// and (NM / 4 - 1) lo MFMAs chained on its own accumulator (the hi and lo
// products may not share a K = 32 chunk), the four
// chains interleaved so no MFMA waits on its predecessor's result.  A lane
// owns one new row and 4 j's of each 16 x 16 tile: 16 exps and the same
// adds per 1024 pairs as the 32 x 32 mix.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NM, int NE, int NA>
__global__ __launch_bounds__(256) void mix16_kernel(float* out, int iters,
                                                    unsigned long long* cyc) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
  f16x8 a, b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h ^= h >> 13; h *= 0x5bd1e995u;
    a[e] = static_cast<_Float16>(1.0f + (h & 0x7F) * (1.0f / 128));
    b[e] = static_cast<_Float16>(-1.0f - ((h >> 8) & 0x7F) * (1.0f / 128));
  }
  f32x4 acc[4] = {};
  float v[16];
  const float s = 1e-7f * (threadIdx.x & 7);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = -1e-3f * (threadIdx.x + k);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
      for (int k = m * NE / NM; k < (m + 1) * NE / NM; ++k) ABC_EXP(v[k & 15])
#pragma unroll
      for (int k = m * NA / NM; k < (m + 1) * NA / NM; ++k)
        ABC_ADD(v[(k + 5) & 15], s)
    }
  }
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += v[k];
#pragma unroll
  for (int q = 0; q < 4; ++q) t += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * 256 + threadIdx.x] = t;
  if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
}

template <int NM, int NE, int NA>
double time_mix16(int waves_per_simd, int iters, int cus, float* out) {
  const int blocks = cus * waves_per_simd;
  unsigned long long* cyc = nullptr;
  (void)hipMalloc(&cyc, static_cast<size_t>(blocks) * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((mix16_kernel<NM, NE, NA>), dim3(blocks), dim3(256), 0, 0,
                       out, iters, cyc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) {
      best = ms;
      g_clock_ghz = mean_clock_ghz(cyc, blocks, ms);
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(cyc);
  return best * 1e6 / (static_cast<double>(waves_per_simd) * iters);
}

template <int NM, int NE, int NA>
double time_mix(int waves_per_simd, int iters, int cus, float* out) {
  const int blocks = cus * waves_per_simd;
  unsigned long long* cyc = nullptr;
  (void)hipMalloc(&cyc, static_cast<size_t>(blocks) * 8);  // 4 waves per block, 1 per SIMD
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {  // rep 0 warms the clock
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((mix_kernel<NM, NE, NA>), dim3(blocks), dim3(256), 0, 0,
                       out, iters, cyc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) {
      best = ms;
      g_clock_ghz = mean_clock_ghz(cyc, blocks, ms);
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(cyc);
  // every SIMD runs waves_per_simd waves of iters steps
  return best * 1e6 / (static_cast<double>(waves_per_simd) * iters);
}

}  // namespace

extern "C" {

// the clock (GHz, s_memtime cycles / launch time) of the last mix timed by
// abc_probe_kde_mix (variants 0-4, 12, 13, 18-21; 0 for the memory mixes)
double abc_probe_last_clock_ghz() { return g_clock_ghz; }

// ns per step per SIMD of mix `variant` at `waves_per_simd` waves per SIMD
// (< 0 on error).  Blocks: one per CU per wave slot.
double abc_probe_kde_mix(int variant, int waves_per_simd, int iters) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1.0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess)
    return -1.0;
  if (waves_per_simd < 1 || waves_per_simd > 8 || iters < 1) return -1.0;
  float* out = nullptr;
  if (hipMalloc(&out, static_cast<size_t>(cus) * 8 * 256 * 4) != hipSuccess)
    return -1.0;
  // DMA source: 1024 chunks of up to 32 fragments (32 MB; the probes read
  // NF <= 18 KiB of each chunk)
  bf16x8* src = nullptr;
  const size_t src_bytes = size_t{1024} * 32 * 64 * 16;
  if (hipMalloc(&src, src_bytes) != hipSuccess) {
    (void)hipFree(out);
    return -1.0;
  }
  (void)hipMemset(src, 0x3C, src_bytes);
  double ns = -1.0;
  g_clock_ghz = 0.0;
  switch (variant) {
    case 0: ns = time_mix<5, 16, 23>(waves_per_simd, iters, cus, out); break;
    case 1: ns = time_mix<11, 16, 40>(waves_per_simd, iters, cus, out); break;
    case 2: ns = time_mix<9, 16, 40>(waves_per_simd, iters, cus, out); break;
    case 3: ns = time_mix<4, 16, 21>(waves_per_simd, iters, cus, out); break;
    case 4: ns = time_mix<9, 16, 19>(waves_per_simd, iters, cus, out); break;
    case 5: ns = time_mem_mix<4, 16, 19, 2, 0, 0>(waves_per_simd, iters, cus, out, src); break;
    case 6: ns = time_mem_mix<4, 16, 19, 2, 2, 0>(waves_per_simd, iters, cus, out, src); break;
    case 7: ns = time_mem_mix<4, 16, 19, 2, 2, 1>(waves_per_simd, iters, cus, out, src); break;
    case 8: ns = time_mem_mix<4, 16, 19, 2, 4, 0>(waves_per_simd, iters, cus, out, src); break;
    case 9: ns = time_mem_mix<4, 16, 19, 2, 4, 1>(waves_per_simd, iters, cus, out, src); break;
    case 10: ns = time_mem_mix<4, 16, 19, 2, 8, 0>(waves_per_simd, iters, cus, out, src); break;
    case 11: ns = time_mem_mix<4, 16, 19, 2, 8, 1>(waves_per_simd, iters, cus, out, src); break;
    case 12: ns = time_mix<4, 16, 22>(waves_per_simd, iters, cus, out); break;
    case 13: ns = time_mix<9, 16, 28>(waves_per_simd, iters, cus, out); break;
    // the d = 20 ladder (mix 13 plus the folded LDS pass's memory path at
    // IB = 2: 4.5 ds_read_b128 per (tile, i-tile) step -- 4 and 5
    // alternating is not expressible, 5 bounds it --, a barrier per 2-tile
    // stage = 4 steps, 18 KiB of LDS-DMA refill per stage)
    case 14: ns = time_mem_mix<9, 16, 28, 5, 0, 0, 18>(waves_per_simd, iters, cus, out, src); break;
    case 15: ns = time_mem_mix<9, 16, 28, 5, 4, 0, 18>(waves_per_simd, iters, cus, out, src); break;
    case 16: ns = time_mem_mix<9, 16, 28, 5, 4, 1, 18>(waves_per_simd, iters, cus, out, src); break;
    case 17: ns = time_mem_mix<9, 16, 28, 4, 0, 0, 18>(waves_per_simd, iters, cus, out, src); break;
    // LocalTransition z-form density (lz_kernel, d = 6): per (particle tile,
    // point tile) product 3 MFMAs, 2 v_exp_f32 and 17 other VALU (12
    // squares, 2 fma, 2 adds, the flush) -- 19 bounds the flush's share
    case 18: ns = time_mix<3, 2, 17>(waves_per_simd, iters, cus, out); break;
    case 19: ns = time_mix<3, 2, 19>(waves_per_simd, iters, cus, out); break;
    // mix 13's work (d = 20, f16 folded) in the 16x16x32 shape: 4 tiles x
    // (1 hi + 4 lo) = 20 MFMAs per 1024 pairs, 16 exps, 28 other VALU
    case 20: ns = time_mix16<20, 16, 28>(waves_per_simd, iters, cus, out); break;
    // the d = 8 mix 12 in that shape: 4 x (1 hi + 2 lo) = 12 MFMAs
    case 21: ns = time_mix16<12, 16, 22>(waves_per_simd, iters, cus, out); break;
    // round 6: the kernels' PMC mixes with SQ_INSTS_VALU's MFMAs taken out
    // (the counter includes them: this probe's mix 12 reads 42.0 VALU per
    // step = 4 MFMA + 16 exp + 22 adds): d = 8 4 MFMA, 16 exp, 17.5 other
    // (22 / 23 average it), d = 20 9 MFMA, 16 exp, 18 other (24)
    case 22: ns = time_mix<4, 16, 17>(waves_per_simd, iters, cus, out); break;
    case 23: ns = time_mix<4, 16, 18>(waves_per_simd, iters, cus, out); break;
    case 24: ns = time_mix<9, 16, 18>(waves_per_simd, iters, cus, out); break;
    default: break;
  }
  (void)hipFree(src);
  (void)hipFree(out);
  return ns;
}

}  // extern "C"
