// Probe: wave64 issue throughput of v_fma_f32, v_sub_f32, v_pk_add_f32,
// v_pk_fma_f32, v_exp_f32 on gfx950 with 8 waves/SIMD (many blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

#define BODY8(X) X X X X X X X X
__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
    BODY8(a0 = __builtin_fmaf(a0, s, s); a1 = __builtin_fmaf(a1, s, s); a2 = __builtin_fmaf(a2, s, s); a3 = __builtin_fmaf(a3, s, s);
          a4 = __builtin_fmaf(a4, s, s); a5 = __builtin_fmaf(a5, s, s); a6 = __builtin_fmaf(a6, s, s); a7 = __builtin_fmaf(a7, s, s);)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, int iters, float s) {
  f2 a0 = {(float)threadIdx.x, 1}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f2 ss = {s, s};
  for (int i = 0; i < iters; ++i) {
    BODY8(asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a0) : "v"(ss)); asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a1) : "v"(ss));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a2) : "v"(ss)); asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a3) : "v"(ss));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a4) : "v"(ss)); asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a5) : "v"(ss));
          asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a6) : "v"(ss)); asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a7) : "v"(ss));)
  }
  f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_pkadd(float* out, int iters, float s) {
  f2 a0 = {(float)threadIdx.x, 1}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f2 ss = {s, s};
  for (int i = 0; i < iters; ++i) {
    BODY8(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a0) : "v"(ss)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a1) : "v"(ss));
          asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a2) : "v"(ss)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a3) : "v"(ss));
          asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a4) : "v"(ss)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a5) : "v"(ss));
          asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a6) : "v"(ss)); asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a7) : "v"(ss));)
  }
  f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_sub(float* out, int iters, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
    BODY8(asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a0) : "v"(s)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a1) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a2) : "v"(s)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a3) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a4) : "v"(s)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a5) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a6) : "v"(s)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a7) : "v"(s));)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_exp(float* out, int iters, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
    BODY8(asm volatile("v_exp_f32 %0, %0" : "+v"(a0)); asm volatile("v_exp_f32 %0, %0" : "+v"(a1));
          asm volatile("v_exp_f32 %0, %0" : "+v"(a2)); asm volatile("v_exp_f32 %0, %0" : "+v"(a3));
          asm volatile("v_exp_f32 %0, %0" : "+v"(a4)); asm volatile("v_exp_f32 %0, %0" : "+v"(a5));
          asm volatile("v_exp_f32 %0, %0" : "+v"(a6)); asm volatile("v_exp_f32 %0, %0" : "+v"(a7));)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
// mixed: 1 exp per 4 sub/fma (exp co-issue test)
__global__ __launch_bounds__(256) void k_mix(float* out, int iters, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, e0 = a0 + 4, e1 = a0 + 5;
  for (int i = 0; i < iters; ++i) {
    BODY8(asm volatile("v_exp_f32 %0, %0" : "+v"(e0)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a0) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a1) : "v"(s)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a2) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a3) : "v"(s));
          asm volatile("v_exp_f32 %0, %0" : "+v"(e1)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a0) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a1) : "v"(s)); asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a2) : "v"(s));
          asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a3) : "v"(s));)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + e0 + e1;
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 1024 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 2048;
  const double instr = 64.0 * iters * blocks * 4;  // wave-instructions
  float ms;
  auto run = [&](const char* name, void (*k)(float*, int, float), double per) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    // cycles per wave-instruction per SIMD at 2.4 GHz
    double cyc = ms * 1e-3 * 2.4e9 * 1024 / (instr * per);
    printf("%-10s %.3f ms  %.2f cyc per wave64 instr per SIMD (@2.4GHz)\n", name, ms, cyc);
  };
  run("fma", k_fma, 1); run("sub", k_sub, 1); run("pk_add", k_pkadd, 1);
  run("pk_fma", k_pkfma, 1); run("exp", k_exp, 1); run("mix 1e:4s", k_mix, 1.25);
  return 0;
}
