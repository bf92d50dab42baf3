// Probe: how does v_mfma_f32_32x32x16_{f16,bf16} round when 16 small
// products land on a LARGE accumulator (the folded KDE passes add each lo
// chunk onto e itself)?  Random C in +-[16, 64), random 16-bit pieces whose
// products span 2^-2 .. 2^-18; the output is compared with
//   rne1  C + sum(products) exact, rounded once (nearest even)
//   rz1   the same, rounded toward zero
//   seq   C + p0 + p1 + ... in fp32, nearest even after each add
//   two   fp32(sum(products)) then + C, nearest even (two roundings)
// and the signed error in ulps of the output is summarised (a bias means
// truncation somewhere inside).
//   hipcc --offload-arch=gfx950 -O3 mfma_acc_round.hip -o mfma_acc_round
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 2048;

// A[w][row 32][k 16], B[w][k 16][col 32], C/D[w][row 32][col 32], 16-bit patterns
template <bool F16>
__global__ void probe(const unsigned short* A, const unsigned short* B, const float* C,
                      float* D) {
  const int w = blockIdx.x, l = threadIdx.x;
  const int r = l & 31, h = l >> 5;
  s16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = static_cast<short>(A[(w * 32 + r) * 16 + 8 * h + e]);
    b[e] = static_cast<short>(B[(w * 16 + 8 * h + e) * 32 + r]);
  }
  f32x16 c;
  for (int v = 0; v < 16; ++v) c[v] = C[(w * 32 + 8 * (v >> 2) + 4 * h + (v & 3)) * 32 + r];
  if constexpr (F16)
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                               __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int v = 0; v < 16; ++v) D[(w * 32 + 8 * (v >> 2) + 4 * h + (v & 3)) * 32 + r] = c[v];
}

static double h2d(unsigned short b, bool f16) {
  if (!f16) {
    unsigned u = static_cast<unsigned>(b) << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
  }
  const int s = b >> 15, e = (b >> 10) & 31, m = b & 1023;
  double v = e == 0 ? std::ldexp(m, -24) : std::ldexp(1024 + m, e - 25);
  return s ? -v : v;
}
static unsigned short d2h(double v, bool f16) {  // v exactly representable
  if (!f16) {
    float f = static_cast<float>(v);
    unsigned u;
    memcpy(&u, &f, 4);
    return static_cast<unsigned short>(u >> 16);
  }
  const _Float16 x = static_cast<_Float16>(static_cast<float>(v));
  unsigned short b;
  memcpy(&b, &x, 2);
  return b;
}
static float rz(double x) {
  float f = static_cast<float>(x);
  if (std::fabs(static_cast<double>(f)) > std::fabs(x)) f = std::nextafter(f, 0.0f);
  return f;
}

template <bool F16>
void run(const char* name) {
  const int bits = F16 ? 11 : 8;
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  const size_t nA = size_t(kWaves) * 32 * 16, nC = size_t(kWaves) * 32 * 32;
  std::vector<unsigned short> A(nA), B(nA);
  std::vector<float> C(nC), D(nC);
  auto piece = [&](int emin, int emax) {
    const int e = emin + static_cast<int>(U(g) * (emax - emin + 1));
    const double m = std::floor(std::ldexp(1.0 + U(g), bits - 1)) / std::ldexp(1.0, bits - 1);
    const double v = std::ldexp(m, e) * (U(g) < 0.5 ? -1.0 : 1.0);
    return d2h(v, F16);
  };
  for (size_t i = 0; i < nA; ++i) {
    A[i] = piece(-9, -1);
    B[i] = piece(-9, -1);
  }
  for (size_t i = 0; i < nC; ++i)
    C[i] = static_cast<float>((16.0 + 48.0 * U(g)) * (U(g) < 0.5 ? -1.0 : 1.0));
  unsigned short *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, nA * 2);
  hipMalloc(&dB, nA * 2);
  hipMalloc(&dC, nC * 4);
  hipMalloc(&dD, nC * 4);
  hipMemcpy(dA, A.data(), nA * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), nA * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), nC * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe<F16>, dim3(kWaves), dim3(64), 0, 0, dA, dB, dC, dD);
  hipMemcpy(D.data(), dD, nC * 4, hipMemcpyDeviceToHost);
  size_t eq_rne = 0, eq_rz = 0, eq_seq = 0, eq_two = 0;
  double bias = 0.0, maxerr = 0.0;
  for (int w = 0; w < kWaves; ++w)
    for (int r = 0; r < 32; ++r)
      for (int c = 0; c < 32; ++c) {
        const size_t o = (size_t(w) * 32 + r) * 32 + c;
        double ex = C[o], ps = 0.0;
        float seq = C[o];
        for (int k = 0; k < 16; ++k) {
          const double p = h2d(A[(size_t(w) * 32 + r) * 16 + k], F16) *
                           h2d(B[(size_t(w) * 16 + k) * 32 + c], F16);
          ex += p;
          ps += p;
          seq = static_cast<float>(static_cast<double>(seq) + p);
        }
        const float rne1 = static_cast<float>(ex);
        const float two = static_cast<float>(static_cast<double>(static_cast<float>(ps)) + C[o]);
        eq_rne += D[o] == rne1;
        eq_rz += D[o] == rz(ex);
        eq_seq += D[o] == seq;
        eq_two += D[o] == two;
        const double ulp = std::ldexp(1.0, std::ilogb(rne1) - 23);
        const double err = (static_cast<double>(D[o]) - ex) / ulp;
        bias += err * (ex < 0 ? -1.0 : 1.0);  // toward +|x| positive
        maxerr = std::fmax(maxerr, std::fabs(err));
      }
  const double n = static_cast<double>(nC);
  printf("%s: %zu outputs  match rne1 %.4f  rz1 %.4f  seq %.4f  two %.4f  "
         "mean signed err (away from 0) %.4f ulp  max |err| %.3f ulp\n",
         name, nC, eq_rne / n, eq_rz / n, eq_seq / n, eq_two / n, bias / n, maxerr);
  hipFree(dA);
  hipFree(dB);
  hipFree(dC);
  hipFree(dD);
}

int main() {
  run<true>("f16 ");
  run<false>("bf16");
  return 0;
}
