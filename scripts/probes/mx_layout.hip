// probe: lane -> (row, k) map of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cmath>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t* A, const uint8_t* B, float* C, int sa, int sb) {
  // hypothesis H1: lane l holds row l&15, k = 32*(l>>4) + j (j = 0..31) for A; col l&15 same k for B
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
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  for (int j = 0; j < 4; ++j) C[(4 * (l >> 4) + j) * 16 + (l & 15)] = c[j];
}
static float e4m3(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r = e ? std::ldexp(1.0f + m / 8.0f, e - 7) : std::ldexp(m / 8.0f, -6);
  return s ? -r : r;
}
int main() {
  std::vector<uint8_t> A(16 * 128), B(128 * 16);
  unsigned x = 12345;
  auto rnd = [&]() { x = x * 1103515245 + 12345; return (x >> 16) & 0x7f; };
  for (auto& v : A) { v = rnd() & 0x3f; if (rnd() & 1) v |= 0x80; }   // small magnitudes, both signs
  for (auto& v : B) { v = rnd() & 0x3f; if (rnd() & 1) v |= 0x80; }
  uint8_t *dA, *dB; float* dC;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size()); hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  for (int scale : {127, 128, 126}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, scale, 127);
    std::vector<float> C(256);
    hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost);
    double maxerr = 0, maxref = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      double r = 0;
      for (int kk = 0; kk < 128; ++kk) r += (double)e4m3(A[i * 128 + kk]) * e4m3(B[kk * 16 + j]);
      r *= std::ldexp(1.0, scale - 127);
      maxerr = std::fmax(maxerr, std::fabs(r - C[i * 16 + j])); maxref = std::fmax(maxref, std::fabs(r));
    }
    printf("scale_a=%d: H1 max err %g (max |ref| %g)\n", scale, maxerr, maxref);
  }
  return 0;
}
