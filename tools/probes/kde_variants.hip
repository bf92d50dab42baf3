// Probe: variants of the fp32 KDE main loop (d = 8 and 20) on synthetic
// whitened data; prints ms, pairs/s and the max relative deviation of each
// variant's row sums from variant 0.  Not part of the product build.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 kde_variants.hip -o kde_variants_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cmath>
#include <algorithm>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ inline float hrand(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (x >> 8) * (1.0f / 16777216.0f);
}
__global__ void fill(float* Y, int64_t n, int D, int stride, float sc, uint32_t seed, bool lw) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  for (int k = 0; k < D; ++k) {
    float u1 = hrand(seed + i * 977 + k * 13 + 1) + 1e-7f, u2 = hrand(seed ^ (i * 31 + k * 7 + 5));
    Y[i * stride + k] = sc * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
  }
  if (lw) Y[i * stride + D] = log2f(0.5f + hrand(seed * 3 + i)) - 0.6f;
}

// ---- baseline structure (as in kde.hip) with knobs --------------------------
template <int D, int R, int U, int CH, bool PF>
__global__ __launch_bounds__(256) void kde_v(const float* __restrict__ Ynew, int64_t M,
                                             const float* __restrict__ P, int64_t npad,
                                             int split, int64_t jchunk, double* __restrict__ partial) {
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t j0 = (int64_t)s * jchunk;
  int64_t j1 = j0 + jchunk; if (j1 > npad) j1 = npad;
  float yi[R][D];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int64_t row = rb * 256 * R + r * 256 + threadIdx.x; if (row >= M) row = M - 1;
#pragma unroll
    for (int k = 0; k < D; ++k) yi[r][k] = Ynew[row * D + k];
  }
  double S[R];
#pragma unroll
  for (int r = 0; r < R; ++r) S[r] = 0.0;
  const int nj = (int)(j1 - j0);
  const float* __restrict__ base = P + j0 * (D + 1);
  constexpr int W = U * (D + 1);
  float nx[W];
  if (PF) {
#pragma unroll
    for (int q = 0; q < W; ++q) nx[q] = base[q];
  }
  for (int jc = 0; jc < nj; jc += CH) {
    const int je = min(jc + CH, nj);
    float sacc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) sacc[r] = 0.f;
    for (int j = jc; j < je; j += U) {
      float cu[W];
      if (PF) {
#pragma unroll
        for (int q = 0; q < W; ++q) cu[q] = nx[q];
        const int jn = min(j + U, nj - U);
        const float* __restrict__ pn = base + (int64_t)jn * (D + 1);
#pragma unroll
        for (int q = 0; q < W; ++q) nx[q] = pn[q];
      } else {
        const float* __restrict__ pj = base + (int64_t)j * (D + 1);
#pragma unroll
        for (int q = 0; q < W; ++q) cu[q] = pj[q];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float acc = cu[u * (D + 1) + D];
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const float df = yi[r][k] - cu[u * (D + 1) + k];
            acc = __builtin_fmaf(-df, df, acc);
          }
          sacc[r] += __builtin_amdgcn_exp2f(acc);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) S[r] += (double)sacc[r];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = rb * 256 * R + r * 256 + threadIdx.x;
    if (row < M) partial[(int64_t)s * M + row] = S[r];
  }
}

// ---- packed: pairs of rows in float2 lanes (v_pk_add_f32 / v_pk_fma_f32) ----
template <int D, int R2, int U, int CH>
__global__ __launch_bounds__(256) void kde_pk(const float* __restrict__ Ynew, int64_t M,
                                              const float* __restrict__ P, int64_t npad,
                                              int split, int64_t jchunk, double* __restrict__ partial) {
  constexpr int R = 2 * R2;
  const int s = blockIdx.x % split;
  const int64_t rb = blockIdx.x / split;
  const int64_t j0 = (int64_t)s * jchunk;
  int64_t j1 = j0 + jchunk; if (j1 > npad) j1 = npad;
  f2 yi[R2][D];
#pragma unroll
  for (int r = 0; r < R2; ++r) {
    int64_t ra = rb * 256 * R + (2 * r) * 256 + threadIdx.x; if (ra >= M) ra = M - 1;
    int64_t rbb = rb * 256 * R + (2 * r + 1) * 256 + threadIdx.x; if (rbb >= M) rbb = M - 1;
#pragma unroll
    for (int k = 0; k < D; ++k) yi[r][k] = f2{Ynew[ra * D + k], Ynew[rbb * D + k]};
  }
  double S[R];
#pragma unroll
  for (int r = 0; r < R; ++r) S[r] = 0.0;
  const int nj = (int)(j1 - j0);
  const float* __restrict__ base = P + j0 * (D + 1);
  constexpr int W = U * (D + 1);
  for (int jc = 0; jc < nj; jc += CH) {
    const int je = min(jc + CH, nj);
    f2 sacc[R2];
#pragma unroll
    for (int r = 0; r < R2; ++r) sacc[r] = f2{0.f, 0.f};
    for (int j = jc; j < je; j += U) {
      const float* __restrict__ pj = base + (int64_t)j * (D + 1);
      float cu[W];
#pragma unroll
      for (int q = 0; q < W; ++q) cu[q] = pj[q];
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int r = 0; r < R2; ++r) {
          const float l = cu[u * (D + 1) + D];
          f2 acc = f2{l, l};
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const float p = cu[u * (D + 1) + k];
            const f2 df = yi[r][k] - f2{p, p};
            acc = __builtin_elementwise_fma(-df, df, acc);
          }
          sacc[r] += f2{__builtin_amdgcn_exp2f(acc.x), __builtin_amdgcn_exp2f(acc.y)};
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) { S[2 * r] += (double)sacc[r].x; S[2 * r + 1] += (double)sacc[r].y; }
  }
#pragma unroll
  for (int r = 0; r < R2; ++r) {
    const int64_t ra = rb * 256 * R + (2 * r) * 256 + threadIdx.x;
    const int64_t rbb = rb * 256 * R + (2 * r + 1) * 256 + threadIdx.x;
    if (ra < M) partial[(int64_t)s * M + ra] = S[2 * r];
    if (rbb < M) partial[(int64_t)s * M + rbb] = S[2 * r + 1];
  }
}

__global__ void finalize(const double* part, int64_t M, int split, double* out) {
  int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= M) return;
  double s = 0; for (int k = 0; k < split; ++k) s += part[k * M + i];
  out[i] = s;
}

static int pick_split(int64_t M, int64_t npad, int R, int CH) {
  int64_t rbk = (M + 256 * R - 1) / (256 * R);
  int64_t split = (8192 + rbk - 1) / rbk;
  if (split > 8) split = (split + 7) / 8 * 8;
  int64_t mx = npad / CH; if (split > mx) split = mx; if (split < 1) split = 1;
  return (int)split;
}

template <int D>
void run_all(int64_t N) {
  const int64_t M = N, npad = (N + 63) / 64 * 64;
  float *Y, *P; double *part, *out;
  hipMalloc(&Y, M * D * 4); hipMalloc(&P, npad * (D + 1) * 4);
  hipMalloc(&part, 64 * M * 8 * 4); hipMalloc(&out, M * 8);
  const float sc = sqrtf(8.6f * 8 / D);
  hipLaunchKernelGGL(fill, dim3((M + 255) / 256), dim3(256), 0, 0, Y, M, D, D, sc, 11u, false);
  hipLaunchKernelGGL(fill, dim3((npad + 255) / 256), dim3(256), 0, 0, P, npad, D, D + 1, sc, 77u, true);
  std::vector<double> ref(M), got(M);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto launch = [&](const char* name, auto kern, int R, int CH, bool first) {
    const int split = pick_split(M, npad, R, CH);
    const int64_t rbk = (M + 256 * R - 1) / (256 * R);
    const int64_t jchunk = ((npad + split - 1) / split + CH - 1) / CH * CH;
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(rbk * split), dim3(256), 0, 0, Y, M, P, npad, split, jchunk, part);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); best = std::min(best, ms);
    }
    hipLaunchKernelGGL(finalize, dim3((M + 255) / 256), dim3(256), 0, 0, part, M, split, out);
    hipMemcpy(first ? ref.data() : got.data(), out, M * 8, hipMemcpyDeviceToHost);
    double dev = 0;
    if (!first) for (int64_t i = 0; i < M; ++i) dev = std::max(dev, std::fabs(got[i] / ref[i] - 1));
    const double pairs = (double)M * npad;
    printf("D=%2d %-26s %8.2f ms  %.3e pairs/s  %.3f of FP32 peak  maxdev %.1e  split %d\n", D, name, best,
           pairs / best * 1e3, pairs * (3 * D + 4) / best * 1e3 / 157.3e12, dev, split);
  };
  launch("base R4 U2 CH64", kde_v<D, 4, 2, 64, false>, 4, 64, true);
  launch("pk R2x2 U2 CH64", kde_pk<D, 2, 2, 64>, 4, 64, false);
  launch("pk R2x2 U1 CH64", kde_pk<D, 2, 1, 64>, 4, 64, false);
  launch("pk R3x2 U2 CH64", kde_pk<D, 3, 2, 64>, 6, 64, false);
  launch("pk R3x2 U1 CH64", kde_pk<D, 3, 1, 64>, 6, 64, false);
  launch("pk R4x2 U2 CH64", kde_pk<D, 4, 2, 64>, 8, 64, false);
  launch("pk R4x2 U1 CH64", kde_pk<D, 4, 1, 64>, 8, 64, false);
  launch("pk R4x2 U2 CH128", kde_pk<D, 4, 2, 128>, 8, 128, false);
  launch("pk R1x2 U4 CH64", kde_pk<D, 1, 4, 64>, 2, 64, false);
  hipFree(Y); hipFree(P); hipFree(part); hipFree(out);
}

int main() {
  run_all<8>(1000000);
  run_all<20>(400000);
  run_all<4>(400000);
  run_all<16>(400000);
  return 0;
}
