// probe: v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands
//  (1) operand map H1: lane l holds row (l & 31), k = 32 (l >> 5) + 4d + e (d = 0..7, byte e)
//      C map: element j of lane l = C[row 8 (j >> 2) + 4 (l >> 5) + (j & 3)][col l & 31]
//  (2) scale map: which (lane, byte) of the first scale operand scales which (row, 32-k block)
// build: hipcc --offload-arch=gfx950 -O2 mx32_layout.hip -o mx32_layout
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <set>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void layout(const uint8_t* A, const uint8_t* B, float* C, int sa) {
  const int l = threadIdx.x;
  v8i a, b;
  for (int d = 0; d < 8; ++d) {
    uint32_t wa = 0, wb = 0;
    for (int e = 0; e < 4; ++e) {
      const int kk = 32 * (l >> 5) + 4 * d + e;
      wa |= (uint32_t)A[(l & 31) * 64 + kk] << (8 * e);
      wb |= (uint32_t)B[kk * 32 + (l & 31)] << (8 * e);
    }
    a[d] = (int)wa;
    b[d] = (int)wb;
  }
  f16v c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 0x7f7f7f7f);
  for (int j = 0; j < 16; ++j) C[(8 * (j >> 2) + 4 * (l >> 5) + (j & 3)) * 32 + (l & 31)] = c[j];
}

__global__ void scalemap(int k0, int L, int byte, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  for (int d = 0; d < 8; ++d) {
    uint32_t wa = 0, wb = 0;
    for (int e = 0; e < 4; ++e) {
      const int kk = 32 * (l >> 5) + 4 * d + e;
      wa |= 0x38u << (8 * e);                              // A = 1.0 everywhere
      wb |= (uint32_t)(kk == k0 ? 0x38 : 0) << (8 * e);    // B one-hot at k0
    }
    a[d] = (int)wa;
    b[d] = (int)wb;
  }
  int sa = 0x7f7f7f7f;
  if (l == L) sa = (sa & ~(0xff << (8 * byte))) | (0x80 << (8 * byte));
  f16v c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 0x7f7f7f7f);
  for (int j = 0; j < 16; ++j) C[(8 * (j >> 2) + 4 * (l >> 5) + (j & 3)) * 32 + (l & 31)] = c[j];
}

static float e4m3(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r = e ? std::ldexp(1.0f + m / 8.0f, e - 7) : std::ldexp(m / 8.0f, -6);
  return s ? -r : r;
}

int main() {
  std::vector<uint8_t> A(32 * 64), B(64 * 32);
  unsigned x = 12345;
  auto rnd = [&]() { x = x * 1103515245 + 12345; return (x >> 16) & 0x7f; };
  for (auto& v : A) { v = rnd() & 0x3f; if (rnd() & 1) v |= 0x80; }
  for (auto& v : B) { v = rnd() & 0x3f; if (rnd() & 1) v |= 0x80; }
  uint8_t *dA, *dB;
  float* dC;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dC, 1024 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  for (int scale : {127, 128}) {
    hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, dA, dB, dC, scale);
    std::vector<float> C(1024);
    hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
    double maxerr = 0, maxref = 0;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        double r = 0;
        for (int kk = 0; kk < 64; ++kk) r += (double)e4m3(A[i * 64 + kk]) * e4m3(B[kk * 32 + j]);
        r *= std::ldexp(1.0, scale - 127);
        maxerr = std::fmax(maxerr, std::fabs(r - C[i * 32 + j]));
        maxref = std::fmax(maxref, std::fabs(r));
      }
    printf("layout H1, scale_a=%d (uniform): max err %g (max |ref| %g)\n", scale, maxerr, maxref);
  }
  std::vector<float> C(1024);
  for (int L = 0; L < 64; ++L)
    for (int byte = 0; byte < 4; ++byte) {
      std::set<std::pair<int, int>> hit;
      for (int q = 0; q < 2; ++q) {
        hipLaunchKernelGGL(scalemap, dim3(1), dim3(64), 0, 0, q * 32 + 5, L, byte, dC);
        hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
        for (int i = 0; i < 32; ++i)
          if (C[i * 32 + 3] != 1.0f) hit.insert({i, q});
      }
      if (!hit.empty()) {
        printf("lane %2d byte %d ->", L, byte);
        for (auto& h : hit) printf(" (row %d, kblk32 %d)", h.first, h.second);
        printf("\n");
      }
    }
  return 0;
}
