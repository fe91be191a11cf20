// Device helpers shared by the rank kernels (rank.hip, rank_mirror.hip):
// order keys, the row-norm reciprocal, and the data-independent bitonic
// top-16 list update (see rank.hip's rank_stream comment).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

// Row block / query block of a ranking workgroup.  The grid is (query blocks,
// row blocks): the workgroups that share a row range are dispatched back to
// back, so with Q > 32 a range is read from HBM once and by the other query
// blocks from L2 / the Infinity Cache instead of once per query block.
#define RB ((int)blockIdx.y)
#define QB ((int)blockIdx.x)
#define NRB ((int)gridDim.y)

namespace miclip {
namespace rankk {

__device__ __forceinline__ uint32_t score_key(float s, int nan_first) {
  if (s != s) return nan_first ? 0xFFFFFFFFu : 0u;
  if (s == 0.0f) s = 0.0f;  // -0 == +0
  const uint32_t u = __float_as_uint(s);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float decode_key(uint32_t bk, int nan_first) {
  if ((bk == 0xFFFFFFFFu && nan_first) || (bk == 0u && !nan_first)) return __uint_as_float(0x7fc00000u);
  return __uint_as_float((bk & 0x80000000u) ? (bk & 0x7fffffffu) : ~bk);
}

template <typename I>
__device__ __forceinline__ bool better(uint32_t ka, I ia, uint32_t kb, I ib) {
  return ka > kb || (ka == kb && ia < ib);
}

template <int KC, typename I>
__device__ __forceinline__ void list_insert(uint32_t (&lk)[KC], I (&li)[KC], uint32_t c, I ci) {
#pragma unroll
  for (int p = 0; p < KC; ++p) {
    const bool sw = better(c, ci, lk[p], li[p]);
    const uint32_t tk = lk[p];
    const I ti = li[p];
    lk[p] = sw ? c : tk;
    li[p] = sw ? ci : ti;
    c = sw ? tk : c;
    ci = sw ? ti : ci;
  }
}

// Row normalisation as a reciprocal computed once per row (score = dot * inv):
// MI_NORM_L2 inv = 1/||e|| (a zero row gives 0 * inf = NaN, as E/||E|| does at
// embedding_service.py:210); MI_NORM_L2_GUARD inv = 1 when ||e|| <= 1e-8
// (compare_models.py:1168-1171); MI_NORM_NONE inv = 1.  Every kernel that
// scores rows uses these two helpers, so all paths give identical scores.
__device__ __forceinline__ float inv_norm(float ss, int norm_mode) {
  if (norm_mode == 2) return 1.f;
  const float n = sqrtf(ss);
  if (norm_mode == 1) return n > 1e-8f ? 1.f / n : 1.f;
  return 1.f / n;
}

__device__ __forceinline__ float apply_norm(float dot, float ss, int norm_mode) {
  return norm_mode == 2 ? dot : dot * inv_norm(ss, norm_mode);
}

__device__ __forceinline__ void ce_desc(uint64_t& a, uint64_t& b) {  // a >= b afterwards
  const uint64_t x = a > b ? a : b, y = a > b ? b : a;
  a = x;
  b = y;
}

__device__ __forceinline__ void bitonic_sort16_desc(uint64_t (&c)[16]) {
#pragma unroll
  for (int size = 2; size <= 16; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int j = i ^ stride;
        if (j > i) {
          if ((i & size) == 0) ce_desc(c[i], c[j]);
          else ce_desc(c[j], c[i]);
        }
      }
}

// L sorted desc, c sorted desc -> L = the 16 best of both, sorted desc
__device__ __forceinline__ void merge16_desc(uint64_t (&L)[16], const uint64_t (&c)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) L[i] = L[i] > c[15 - i] ? L[i] : c[15 - i];   // bitonic (max of desc, asc)
#pragma unroll
  for (int stride = 8; stride > 0; stride >>= 1)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = i ^ stride;
      if (j > i) ce_desc(L[i], L[j]);
    }
}

// 16 consecutive elements of a row (f32 / bf16 / f16 storage) as f32
template <int DT>
__device__ __forceinline__ void load_chunk(const void* corpus, int64_t row, int64_t D, int k0, float (&v)[16]) {
  if (DT == 0) {
    const float4* p = (const float4*)((const float*)corpus + row * D + k0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 t = p[i];
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else {
    const uint4* p = (const uint4*)((const uint16_t*)corpus + row * D + k0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint4 t = p[i];
      const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (DT == 1) {
          v[8 * i + 2 * e] = bf2f((uint16_t)(w[e] & 0xffff));
          v[8 * i + 2 * e + 1] = bf2f((uint16_t)(w[e] >> 16));
        } else {
          union { uint32_t u; _Float16 h[2]; } cv;
          cv.u = w[e];
          v[8 * i + 2 * e] = (float)cv.h[0];
          v[8 * i + 2 * e + 1] = (float)cv.h[1];
        }
      }
    }
  }
}

}  // namespace rankk
}  // namespace miclip
