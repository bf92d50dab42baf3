// Probe: does v_mfma_f32_32x32x16_f16 keep fp16 subnormal inputs (exact
// products) or flush them?  A = subnormal fp16 values in slot 0 of every
// lane, B = 1.0 in slot 0, everything else 0: D[i][j] = A_i.
//   hipcc --offload-arch=gfx950 -O3 mfma_f16_denorm.hip -o mfma_f16_denorm
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(float* out) {
  const int lane = threadIdx.x;
  f16x8 a = {}, b = {};
  // lanes 0-31 hold k = 0..7 of row (lane & 31): slot 0 = subnormal 2^-(15+lane%10)
  if (lane < 32) {
    a[0] = (_Float16)__builtin_ldexpf(1.0f, -15 - (lane % 10));
    b[0] = (_Float16)1.0f;
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int v = 0; v < 16; ++v) out[lane * 16 + v] = c[v];
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 16 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[64 * 16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // print the distinct nonzero magnitudes found
  int nz = 0;
  float mn = 1e30f, mx = 0;
  for (int i = 0; i < 64 * 16; ++i)
    if (h[i] != 0.0f) { ++nz; mn = fminf(mn, h[i]); mx = fmaxf(mx, h[i]); }
  printf("nonzero outputs %d, min %g (2^-24 = %g), max %g (2^-15 = %g)\n", nz, mn,
         5.9604645e-08f, mx, 3.0517578e-05f);
  return 0;
}
