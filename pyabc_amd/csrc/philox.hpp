// Philox4x32-10 counter-based RNG (Salmon, Moraes, Dror, Shaw, SC'11).
//
// Stream layout shared with oracle/ref_cpu.py (philox_block/philox_uniform/
// philox_normal): block i of stream s under seed k is
//   counter = (i_lo, i_hi, s_lo, s_hi), key = (k_lo, k_hi).
// Uniform u[i] takes words (0,1) of block i/2 for even i and (2,3) for odd i,
// as a 53-bit value (hi << 21 | lo >> 11) * 2^-53 in [0,1).
// Normal z[i] is Box-Muller on block i/2: u1 = 1 - U(w0,w1) in (0,1],
// u2 = U(w2,w3); even i -> r cos(2 pi u2), odd i -> r sin(2 pi u2).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace abc {

struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0,
                                                uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = static_cast<uint64_t>(M0) * c.x;
    const uint64_t p1 = static_cast<uint64_t>(M1) * c.z;
    const uint32_t hi0 = static_cast<uint32_t>(p0 >> 32);
    const uint32_t lo0 = static_cast<uint32_t>(p0);
    const uint32_t hi1 = static_cast<uint32_t>(p1 >> 32);
    const uint32_t lo1 = static_cast<uint32_t>(p1);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

__host__ __device__ inline u32x4 philox_block(uint64_t seed, uint64_t stream,
                                               uint64_t i) {
  u32x4 c{static_cast<uint32_t>(i), static_cast<uint32_t>(i >> 32),
          static_cast<uint32_t>(stream), static_cast<uint32_t>(stream >> 32)};
  return philox4x32_10(c, static_cast<uint32_t>(seed),
                       static_cast<uint32_t>(seed >> 32));
}

__host__ __device__ inline double u53(uint32_t hi, uint32_t lo) {
  const uint64_t v = (static_cast<uint64_t>(hi) << 21) | (lo >> 11);
  return static_cast<double>(v) * (1.0 / 9007199254740992.0);
}

// four normals from one Philox block for the synthetic simulators' noise:
// 24-bit uniforms from each word (w >> 8) * 2^-24, Box-Muller in fp32 on the
// transcendental unit (v_log_f32 = log2, v_sin/cos_f32 of revolutions):
// words (0,1) -> z0 = r cos, z1 = r sin; words (2,3) -> z2, z3, with
// u1 = 1 - U in (0,1] (|z| <= 5.77).  ~1 fp32 ulp from the exact transform.
__device__ inline void box_muller4_f32(u32x4 b, float (&z)[4]) {
  constexpr float k24 = 5.9604644775390625e-08f;  // 2^-24
  constexpr float kM2Ln2 = -1.3862943611198906f;  // -2 ln 2
  const float u1a = 1.0f - static_cast<float>(b.x >> 8) * k24;
  const float u2a = static_cast<float>(b.y >> 8) * k24;
  const float u1b = 1.0f - static_cast<float>(b.z >> 8) * k24;
  const float u2b = static_cast<float>(b.w >> 8) * k24;
  const float ra = __builtin_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u1a));
  const float rb = __builtin_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u1b));
  z[0] = ra * __builtin_amdgcn_cosf(u2a);
  z[1] = ra * __builtin_amdgcn_sinf(u2a);
  z[2] = rb * __builtin_amdgcn_cosf(u2b);
  z[3] = rb * __builtin_amdgcn_sinf(u2b);
}

// pair of normals (cos branch, sin branch) from one Philox block
__device__ inline void box_muller(u32x4 b, double& z0, double& z1) {
  const double u1 = 1.0 - u53(b.x, b.y);
  const double u2 = u53(b.z, b.w);
  const double r = sqrt(-2.0 * log(u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// normals zi0 .. zi0 + d - 1 of one stream into z[0 .. d) (z[k] = 0 for
// k >= d): normal zi is branch zi & 1 of the Box-Muller pair of block zi / 2,
// and each pair the range touches is computed ONCE (the per-element form
// evaluated every pair twice and kept one branch).  Same values bit for bit.
template <int D>
__device__ inline void philox_normals(uint64_t seed, uint64_t stream,
                                      uint64_t zi0, int d, double (&z)[D]) {
#pragma unroll
  for (int k = 0; k < D; ++k) z[k] = 0.0;
  const uint64_t p0 = zi0 >> 1;
  if ((zi0 & 1) == 0) {  // pair q covers k = 2q (cos), 2q + 1 (sin)
#pragma unroll
    for (int q = 0; q < (D + 1) / 2; ++q) {
      if (2 * q < d) {
        double c0, c1;
        box_muller(philox_block(seed, stream, p0 + q), c0, c1);
        z[2 * q] = c0;
        if (2 * q + 1 < D && 2 * q + 1 < d) z[2 * q + 1] = c1;
      }
    }
  } else {  // pair q covers k = 2q - 1 (cos), 2q (sin)
#pragma unroll
    for (int q = 0; q < D / 2 + 1; ++q) {
      if (2 * q - 1 < d) {
        double c0, c1;
        box_muller(philox_block(seed, stream, p0 + q), c0, c1);
        if (q > 0 && 2 * q - 1 < D) z[2 * q - 1] = c0;
        if (2 * q < D && 2 * q < d) z[2 * q] = c1;
      }
    }
  }
}

}  // namespace abc
