// Fused corpus ranking kernels (gfx950).
//
// Replaces the host NumPy ranking of the reference:
//   EmbeddingService.get_embeddings  E / ||E||                 embedding_service.py:209-210
//   EmbeddingService.search_top_frames  np.dot(E, t.T) +
//       np.argsort(s)[::-1][:top_k]                           embedding_service.py:314-320
//   search_top_frames_by_image (same with an image vector)     embedding_service.py:365-372
//   compare_models S = I @ T.T, rank of ground truth           compare_models.py:999-1016, 1045-1062
//
// rank_stage1: one pass over the corpus.  A wave owns a 32-row x 32-query
// tile; the dot products run on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32:
// bit-for-bit a k-ordered fmaf chain, no reduced precision), each lane
// streaming 64 contiguous bytes of its row per k-chunk (a full 128-B line per
// row across the two half-waves) with the next chunk prefetched; the row's
// sum of squares rides along for the L2 norm.  Each lane keeps a sorted
// top-KC list per (query, lane subset) in registers with a threshold test;
// the workgroup merges its 8 lists per query and writes k candidates per
// (chunk, query).  rank_merge reduces the chunks (or the RCCL all-gathered
// per-shard lists) to the final k.  Order: score desc, index asc; NaN first or
// last by policy (np.argsort(s)[::-1] vs np.argsort(-s)).
#include <hip/hip_runtime.h>

#include <climits>

#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int RQ = 32;          // queries per workgroup (MFMA N)
constexpr int ROWS_WAVE = 32;   // corpus rows per wave tile (MFMA M)

__device__ __forceinline__ uint32_t score_key(float s, int nan_first) {
  if (s != s) return nan_first ? 0xFFFFFFFFu : 0u;
  if (s == 0.0f) s = 0.0f;  // -0 == +0
  const uint32_t u = __float_as_uint(s);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
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

__device__ __forceinline__ float apply_norm(float dot, float ss, int norm_mode) {
  if (norm_mode == 2) return dot;
  const float n = sqrtf(ss);
  if (norm_mode == 1) return n > 1e-8f ? dot / n : dot;
  return dot / n;
}

// Computes the 32x32 f32 score tile of (rows row0.., queries of this block)
// for one wave.  Returns acc (C layout: col = query = lane&31,
// row = (r&3) + 8*(r>>2) + 4*(lane>>5)) and the per-row sum of squares in
// nrm (LDS, 32 floats for this wave).
template <int DT>
__device__ __forceinline__ void score_tile(const void* corpus, int64_t N, int64_t D, int64_t row0,
                                           const float* Ts, int ts_stride, float* nrm, f32x16& acc) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t row = min(row0 + r, N - 1);
  acc = f32x16{};
  float ss = 0.f;
  float cur[16], nxt[16];
  load_chunk<DT>(corpus, row, D, 16 * h, cur);
  const int nch = (int)(D / 32);
  const float* tq = Ts + r * ts_stride + 16 * h;
  for (int j = 0; j < nch; ++j) {
    if (j + 1 < nch) load_chunk<DT>(corpus, row, D, 32 * (j + 1) + 16 * h, nxt);
    float tb[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 t = *(const float4*)(tq + 32 * j + 4 * i);
      tb[4 * i] = t.x; tb[4 * i + 1] = t.y; tb[4 * i + 2] = t.z; tb[4 * i + 3] = t.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[i], tb[i], acc, 0, 0, 0);
      ss = fmaf(cur[i], cur[i], ss);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) cur[i] = nxt[i];
  }
  ss += __shfl_xor(ss, 32, 64);
  if (h == 0) nrm[r] = ss;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// stage-1 LDS: queries [32][D+4] f32, per-wave norms [4][32]; the lists
// [256 lanes][KC] (key u32, idx i32) reuse the query area after a barrier.
template <int KC, int DT>
__global__ __launch_bounds__(256) void rank_stage1(const void* __restrict__ corpus, int64_t N, int64_t D,
                                                   const float* __restrict__ queries, int64_t Q, int k,
                                                   int64_t rows_per_wg, int norm_mode, int nan_first,
                                                   int64_t index_base, float* __restrict__ ws_s,
                                                   int64_t* __restrict__ ws_i, int64_t C) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ts_stride = (int)D + 4;
  float* Ts = (float*)smem;
  float* nrm_all = Ts + RQ * ts_stride;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t q0 = (int64_t)blockIdx.y * RQ;

  for (int64_t e = tid; e < RQ * D; e += 256) {
    const int qq = (int)(e / D);
    const int64_t d = e % D;
    Ts[qq * ts_stride + d] = (q0 + qq < Q) ? queries[(q0 + qq) * D + d] : 0.f;
  }
  __syncthreads();

  const int64_t r_begin = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r_end = min(N, r_begin + rows_per_wg);
  float* nrm = nrm_all + wave * 32;

  uint32_t lk[KC];
  int32_t li[KC];
#pragma unroll
  for (int p = 0; p < KC; ++p) { lk[p] = 0u; li[p] = INT_MAX; }

  const int qcol = lane & 31, h = lane >> 5;
  const bool qvalid = q0 + qcol < Q;
  for (int64_t t0 = r_begin + wave * ROWS_WAVE; t0 < r_end; t0 += 4 * ROWS_WAVE) {
    f32x16 acc;
    score_tile<DT>(corpus, N, D, t0, Ts, ts_stride, nrm, acc);
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
      const int64_t row = t0 + rr;
      const float sc = apply_norm(acc[rg], nrm[rr], norm_mode);
      const uint32_t key = score_key(sc, nan_first);
      const int32_t li_row = (int32_t)(row - r_begin);
      const bool ok = qvalid && row < r_end && better(key, li_row, lk[KC - 1], li[KC - 1]);
      if (__builtin_expect(__any(ok), 0)) {
        if (ok) list_insert<KC, int32_t>(lk, li, key, li_row);
      }
    }
  }
  __syncthreads();  // query area free -> lists
  uint32_t* Lk = (uint32_t*)smem;
  int32_t* Li = (int32_t*)(smem + 256 * KC * 4);
#pragma unroll
  for (int p = 0; p < KC; ++p) {
    Lk[tid * KC + p] = lk[p];
    Li[tid * KC + p] = li[p];
  }
  __syncthreads();
  if (tid < RQ && q0 + tid < Q) {
    // 8 sorted lists: lanes {w*64 + tid, w*64 + 32 + tid}
    int pos[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) pos[l] = 0;
    float* os = ws_s + (q0 + tid) * C + (int64_t)blockIdx.x * k;
    int64_t* oi = ws_i + (q0 + tid) * C + (int64_t)blockIdx.x * k;
    for (int o = 0; o < k; ++o) {
      uint32_t bk = 0u;
      int32_t bi = INT_MAX;
      int bl = 0;
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const int src = (l >> 1) * 64 + (l & 1) * 32 + tid;
        if (pos[l] < KC) {
          const uint32_t kk = Lk[src * KC + pos[l]];
          const int32_t ii = Li[src * KC + pos[l]];
          if (better(kk, ii, bk, bi)) { bk = kk; bi = ii; bl = l; }
        }
      }
#pragma unroll
      for (int l = 0; l < 8; ++l) pos[l] += (l == bl) ? 1 : 0;
      if (bi == INT_MAX) {
        os[o] = -INFINITY;
        oi[o] = -1;
      } else {
        // decode: exact inverse of score_key for non-NaN keys
        float s;
        if ((bk == 0xFFFFFFFFu && nan_first) || (bk == 0u && !nan_first)) s = __uint_as_float(0x7fc00000u);
        else s = __uint_as_float((bk & 0x80000000u) ? (bk & 0x7fffffffu) : ~bk);
        os[o] = s;
        oi[o] = index_base + r_begin + bi;
      }
    }
  }
}

// One workgroup per query: threads keep strided top-KC lists, then a tree
// merge through LDS.
template <int KC, int NT>
__global__ __launch_bounds__(NT) void rank_merge_kernel(const float* __restrict__ cs, const int64_t* __restrict__ ci,
                                                        int64_t C, int k, int nan_first, float* __restrict__ out_s,
                                                        int64_t* __restrict__ out_i) {
  __shared__ uint32_t Lk[NT * KC];
  __shared__ int64_t Li[NT * KC];
  const int tid = threadIdx.x;
  const int64_t q = blockIdx.x;
  uint32_t lk[KC];
  int64_t li[KC];
#pragma unroll
  for (int p = 0; p < KC; ++p) { lk[p] = 0u; li[p] = LLONG_MAX; }
  for (int64_t c = tid; c < C; c += NT) {
    const int64_t idx = ci[q * C + c];
    if (idx < 0) continue;
    const uint32_t key = score_key(cs[q * C + c], nan_first);
    if (better(key, idx, lk[KC - 1], li[KC - 1])) list_insert<KC, int64_t>(lk, li, key, idx);
  }
#pragma unroll
  for (int p = 0; p < KC; ++p) { Lk[tid * KC + p] = lk[p]; Li[tid * KC + p] = li[p]; }
  __syncthreads();
  for (int stride = NT / 2; stride >= 1; stride >>= 1) {
    if (tid < stride) {
      const int a = tid * KC, b = (tid + stride) * KC;
      int pa = 0, pb = 0;
#pragma unroll
      for (int o = 0; o < KC; ++o) {
        const bool ta = better(Lk[a + pa], Li[a + pa], Lk[b + pb], Li[b + pb]);
        lk[o] = ta ? Lk[a + pa] : Lk[b + pb];
        li[o] = ta ? Li[a + pa] : Li[b + pb];
        pa += ta ? 1 : 0;
        pb += ta ? 0 : 1;
        // pa + pb == o + 1 <= KC, so neither index can run past its list
      }
    }
    __syncthreads();
    if (tid < stride) {
#pragma unroll
      for (int p = 0; p < KC; ++p) { Lk[tid * KC + p] = lk[p]; Li[tid * KC + p] = li[p]; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    for (int o = 0; o < k; ++o) {
      const uint32_t bk = Lk[o];
      const int64_t bi = Li[o];
      if (bi == LLONG_MAX) {
        out_s[q * k + o] = -INFINITY;
        out_i[q * k + o] = -1;
      } else {
        float s;
        if ((bk == 0xFFFFFFFFu && nan_first) || (bk == 0u && !nan_first)) s = __uint_as_float(0x7fc00000u);
        else s = __uint_as_float((bk & 0x80000000u) ? (bk & 0x7fffffffu) : ~bk);
        out_s[q * k + o] = s;
        out_i[q * k + o] = bi;
      }
    }
  }
}

template <int DT>
__global__ __launch_bounds__(256) void score_matrix_kernel(const void* __restrict__ corpus, int64_t N, int64_t D,
                                                           const float* __restrict__ queries, int64_t Q,
                                                           int norm_mode, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ts_stride = (int)D + 4;
  float* Ts = (float*)smem;
  float* nrm_all = Ts + RQ * ts_stride;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t q0 = (int64_t)blockIdx.y * RQ;
  for (int64_t e = tid; e < RQ * D; e += 256) {
    const int qq = (int)(e / D);
    const int64_t d = e % D;
    Ts[qq * ts_stride + d] = (q0 + qq < Q) ? queries[(q0 + qq) * D + d] : 0.f;
  }
  __syncthreads();
  const int64_t t0 = ((int64_t)blockIdx.x * 4 + wave) * ROWS_WAVE;
  if (t0 >= N) return;
  f32x16 acc;
  score_tile<DT>(corpus, N, D, t0, Ts, ts_stride, nrm_all + wave * 32, acc);
  const int qcol = lane & 31, h = lane >> 5;
  if (q0 + qcol >= Q) return;
#pragma unroll
  for (int rg = 0; rg < 16; ++rg) {
    const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
    if (t0 + rr < N) out[(q0 + qcol) * N + t0 + rr] = apply_norm(acc[rg], nrm_all[wave * 32 + rr], norm_mode);
  }
}

__global__ __launch_bounds__(256) void rank_of_targets_kernel(const float* __restrict__ S, int64_t N,
                                                              const int64_t* __restrict__ pq,
                                                              const int64_t* __restrict__ pt, int64_t T,
                                                              int64_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const float* row = S + pq[t] * N;
  const int64_t g = pt[t];
  const uint32_t kg = score_key(row[g], 0);
  int64_t total = 0;
  for (int64_t n = lane; n < N; n += 64) {
    const uint32_t kn = score_key(row[n], 0);
    total += (kn > kg || (kn == kg && n < g)) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) total += __shfl_xor(total, o, 64);
  if (lane == 0) out[t] = total + 1;
}

}  // namespace

// ------------------------------------------------------------ host helpers
static int kc_for(int k) { return k <= 16 ? 16 : 64; }

int64_t rank_chunks(int64_t N) {
  // rows per workgroup: multiples of 128, enough workgroups to fill 256 CUs
  const int64_t tiles = (N + 127) / 128;
  return tiles < 1024 ? tiles : 1024;
}

size_t rank_workspace_bytes(int64_t N, int64_t Q, int k) {
  const int64_t nch = N > 0 ? rank_chunks(N) : 1;
  return (size_t)(Q * nch * k) * (sizeof(float) + sizeof(int64_t));
}

static size_t stage1_lds(int64_t D, int KC) {
  const size_t qa = (size_t)RQ * (D + 4) * 4 + 4 * 32 * 4;
  const size_t la = (size_t)256 * KC * 8;
  return qa > la ? qa : la;
}

template <int KC, int DT>
static hipError_t launch_stage1(dim3 grid, size_t lds, hipStream_t s, const void* corpus, int64_t N, int64_t D,
                                const float* q, int64_t Q, int k, int64_t rpw, int nm, int nf, int64_t base,
                                float* ws_s, int64_t* ws_i, int64_t C) {
  auto fn = rank_stage1<KC, DT>;
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fn, grid, dim3(256), lds, s, corpus, N, D, q, Q, k, rpw, nm, nf, base, ws_s, ws_i, C);
  return hipGetLastError();
}

hipError_t rank_merge(const float* cs, const int64_t* ci, int64_t Q, int64_t C, int k, int nan_first, float* out_s,
                      int64_t* out_i, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  if (kc_for(k) == 16)
    hipLaunchKernelGGL((rank_merge_kernel<16, 256>), dim3((unsigned)Q), dim3(256), 0, s, cs, ci, C, k, nan_first,
                       out_s, out_i);
  else
    hipLaunchKernelGGL((rank_merge_kernel<64, 64>), dim3((unsigned)Q), dim3(64), 0, s, cs, ci, C, k, nan_first,
                       out_s, out_i);
  return hipGetLastError();
}

hipError_t rank_topk(const void* corpus, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int k,
                     int64_t base, int norm_mode, int nan_first, float* out_s, int64_t* out_i, void* ws,
                     hipStream_t s) {
  const int64_t nch = rank_chunks(N);
  const int64_t rpw = ((N + nch - 1) / nch + 127) / 128 * 128;
  const int64_t nwg = (N + rpw - 1) / rpw;
  const int64_t C = nwg * k;
  float* ws_s = (float*)ws;
  int64_t* ws_i = (int64_t*)((char*)ws + (size_t)(Q * nch * k) * sizeof(float));
  const dim3 grid((unsigned)nwg, (unsigned)((Q + RQ - 1) / RQ));
  const int KC = kc_for(k);
  const size_t lds = stage1_lds(D, KC);
  hipError_t e;
#define MI_S1(KCV, DTV) \
  launch_stage1<KCV, DTV>(grid, lds, s, corpus, N, D, q, Q, k, rpw, norm_mode, nan_first, base, ws_s, ws_i, C)
  if (KC == 16) e = dt == 0 ? MI_S1(16, 0) : dt == 1 ? MI_S1(16, 1) : MI_S1(16, 2);
  else e = dt == 0 ? MI_S1(64, 0) : dt == 1 ? MI_S1(64, 1) : MI_S1(64, 2);
#undef MI_S1
  if (e != hipSuccess) return e;
  return rank_merge(ws_s, ws_i, Q, C, k, nan_first, out_s, out_i, s);
}

hipError_t score_matrix(const void* corpus, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int norm_mode,
                        float* out, hipStream_t s) {
  const dim3 grid((unsigned)((N + 127) / 128), (unsigned)((Q + RQ - 1) / RQ));
  const size_t lds = (size_t)RQ * (D + 4) * 4 + 4 * 32 * 4;
  const void* fn = dt == 0 ? (const void*)score_matrix_kernel<0>
                           : dt == 1 ? (const void*)score_matrix_kernel<1> : (const void*)score_matrix_kernel<2>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (dt == 0) hipLaunchKernelGGL(score_matrix_kernel<0>, grid, dim3(256), lds, s, corpus, N, D, q, Q, norm_mode, out);
  else if (dt == 1) hipLaunchKernelGGL(score_matrix_kernel<1>, grid, dim3(256), lds, s, corpus, N, D, q, Q, norm_mode, out);
  else hipLaunchKernelGGL(score_matrix_kernel<2>, grid, dim3(256), lds, s, corpus, N, D, q, Q, norm_mode, out);
  return hipGetLastError();
}

hipError_t rank_of_targets(const float* S, int64_t Q, int64_t N, const int64_t* pq, const int64_t* pt, int64_t T,
                           int64_t* out, hipStream_t s) {
  (void)Q;
  if (T <= 0) return hipSuccess;
  hipLaunchKernelGGL(rank_of_targets_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, S, N, pq, pt, T, out);
  return hipGetLastError();
}

}  // namespace miclip
