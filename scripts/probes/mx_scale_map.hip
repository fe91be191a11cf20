// probe: which (lane, byte) of the A-scale operand scales which (row i, k-block q)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <set>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(int k0, int L, int byte, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  for (int d = 0; d < 8; ++d) {
    uint32_t wa = 0, wb = 0;
    for (int e = 0; e < 4; ++e) {
      const int kk = 32 * (l >> 4) + 4 * d + e;
      wa |= 0x38u << (8 * e);                       // A = 1.0 everywhere
      wb |= (uint32_t)(kk == k0 ? 0x38 : 0) << (8 * e);  // B one-hot at k0
    }
    a[d] = (int)wa; b[d] = (int)wb;
  }
  int sa = 0x7f7f7f7f;
  if (l == L) sa = (sa & ~(0xff << (8 * byte))) | (0x80 << (8 * byte));
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 0x7f7f7f7f);
  for (int j = 0; j < 4; ++j) C[(4 * (l >> 4) + j) * 16 + (l & 15)] = c[j];
}
int main() {
  float* dC; hipMalloc(&dC, 1024);
  std::vector<float> C(256);
  for (int L = 0; L < 64; ++L) for (int byte = 0; byte < 4; ++byte) {
    std::set<std::pair<int,int>> hit;
    for (int q = 0; q < 4; ++q) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, q * 32 + 5, L, byte, dC);
      hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost);
      for (int i = 0; i < 16; ++i) if (C[i * 16 + 3] != 1.0f) hit.insert({i, q});
    }
    if (!hit.empty()) {
      printf("lane %2d byte %d ->", L, byte);
      for (auto& h : hit) printf(" (row %d, kblk %d)", h.first, h.second);
      printf("\n");
    }
  }
  return 0;
}
