// probe: per-lane scale operand mapping of v_mfma_scale_f32_16x16x128_f8f6f4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cmath>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t* A, const uint8_t* B, const int* SA, const int* SB, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  for (int d = 0; d < 8; ++d) {
    uint32_t wa = 0, wb = 0;
    for (int e = 0; e < 4; ++e) {
      const int kk = 32 * (l >> 4) + 4 * d + e;
      wa |= (uint32_t)A[(l & 15) * 128 + kk] << (8 * e);
      wb |= (uint32_t)B[kk * 16 + (l & 15)] << (8 * e);
    }
    a[d] = (int)wa; b[d] = (int)wb;
  }
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, SA[l], 0, SB[l]);
  for (int j = 0; j < 4; ++j) C[(4 * (l >> 4) + j) * 16 + (l & 15)] = c[j];
}
static float e4m3(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r = e ? std::ldexp(1.0f + m / 8.0f, e - 7) : std::ldexp(m / 8.0f, -6);
  return s ? -r : r;
}
int main() {
  std::vector<uint8_t> A(16 * 128), B(128 * 16);
  unsigned x = 777;
  auto rnd = [&]() { x = x * 1103515245 + 12345; return (x >> 16) & 0x7fff; };
  for (auto& v : A) { v = rnd() & 0x3f; if (rnd() & 1) v |= 0x80; }
  for (auto& v : B) { v = rnd() & 0x3f; if (rnd() & 1) v |= 0x80; }
  std::vector<int> SA(64), SB(64);
  for (int l = 0; l < 64; ++l) { SA[l] = 124 + (rnd() % 7); SB[l] = 124 + (rnd() % 7); }
  uint8_t *dA, *dB; int *dSA, *dSB; float* dC;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size()); hipMalloc(&dC, 1024); hipMalloc(&dSA, 256); hipMalloc(&dSB, 256);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dSA, SA.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(dSB, SB.data(), 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dSA, dSB, dC);
  std::vector<float> C(256);
  hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost);
  // hypotheses for the scale of (row i, k-block q) of A: lane = H(i, q)
  const char* names[4] = {"lane=i+16q (row,kblock)", "lane=i (one scale per row)", "lane=q*16+i hmm same", "lane=i+16*(q) B col"};
  for (int h = 0; h < 2; ++h) {
    double maxerr = 0, maxref = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      double r = 0;
      for (int kk = 0; kk < 128; ++kk) {
        const int q = kk / 32;
        const int la = h == 0 ? i + 16 * q : i;
        const int lb = h == 0 ? j + 16 * q : j;
        r += (double)e4m3(A[i * 128 + kk]) * e4m3(B[kk * 16 + j]) * std::ldexp(1.0, SA[la] - 127) * std::ldexp(1.0, SB[lb] - 127);
      }
      maxerr = std::fmax(maxerr, std::fabs(r - C[i * 16 + j])); maxref = std::fmax(maxref, std::fabs(r));
    }
    printf("%s: max err %g (max |ref| %g)\n", names[h], maxerr, maxref);
  }
  return 0;
}
