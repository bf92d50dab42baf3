// Probe: issue rate of v_mfma_f64_16x16x4_f64 and of the VALU epilogue
// (add_f64, cvt_f32_f64, exp_f32) on gfx950.  Build:
//   hipcc --offload-arch=gfx950 -O3 mfma_f64_rate.hip -o mfma_f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(const double* in, double* out, int iters) {
  double a = in[threadIdx.x], b = in[threadIdx.x + 64];
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void valu_loop(const double* in, double* out, int iters) {
  double c = in[threadIdx.x];
  double e0 = in[threadIdx.x + 1], e1 = in[threadIdx.x + 2], e2 = in[threadIdx.x + 3], e3 = in[threadIdx.x + 4];
  float s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int it = 0; it < iters; ++it) {
    s0 += __builtin_amdgcn_exp2f((float)(e0 + c));
    s1 += __builtin_amdgcn_exp2f((float)(e1 + c));
    s2 += __builtin_amdgcn_exp2f((float)(e2 + c));
    s3 += __builtin_amdgcn_exp2f((float)(e3 + c));
    e0 -= 1e-9; e1 -= 1e-9; e2 -= 1e-9; e3 -= 1e-9;
  }
  out[blockIdx.x * 256 + threadIdx.x] = s0 + s1 + s2 + s3;
}

int main() {
  double *in, *out;
  hipMalloc(&in, 4096 * 8);
  hipMalloc(&out, 4096 * 1024 * 8);
  hipMemset(in, 0, 4096 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 4096;
  float ms;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    mfma_loop<4><<<blocks, 256>>>(in, out, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 16 * 16 * 4 * 4.0 * iters * blocks * 4;
    printf("mfma_f64_16x16x4: %.2f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    valu_loop<<<blocks, 256>>>(in, out, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double el = 4.0 * iters * blocks * 256;
    printf("epilogue (add_f64+cvt+exp+add_f32 + sub_f64): %.2f ms  %.3e elem/s  %.2f cyc/elem/SIMD-lane-group\n",
           ms, el / ms * 1e3, (ms * 1e-3 * 2.4e9 * 1024) / (el / 64));
  }
  return 0;
}
