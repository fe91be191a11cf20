// Mirrored-corpus ranking: an fp16 ranking mirror of
// the corpus, HBM-streamed at half the f32 bytes on the fp16 MFMA, plus an exact
// re-score of the mirror's candidates against the f32 master.
//
// Replaces, like rank.hip, the ranking of EmbeddingService.search_top_frames
// (embedding_service.py:314-320: np.dot(E / ||E||, t.T) + argsort(s)[::-1][:k])
// for a corpus that is ranked many times (the service's per-video .npy rows,
// embedding_service.py:186-217, kept in HBM).
//
// mirror_build: m = fp16(c * inv), inv = the rank kernels' 1/||c|| (the same
//   fmaf order, rank_keys.hpp inv_norm), so mirror rows are unit vectors and the
//   ranking pass needs no norm.
// rank_mirror: rank_reg's structure (one wave per SIMD, per-wave LDS ring of
//   32-row x 64-k chunks by buffer-descriptor DMA, counted waits, queries held
//   as MFMA B operands, bitonic top-16 lists, shared k-th threshold tau) on
//   v_mfma_f32_32x32x16_f16, 2 B per element instead of 4.  The f32 query is split
//   into fp16 hi + lo (SPLIT, D <= 512) so the query side is exact to ~2^-22.
//   Output: the exact top-kc (kc = 16) of the MIRROR scores per query.
// mirror_rescore: per query, the exact f32 scores of its kc candidates with the
//   arithmetic of every exact rank path (exact-f32 MFMA chain in k order, fmaf
//   sum of squares, inv_norm; rank.hip score_tile), their top-k by (score desc,
//   index asc), and a certificate.  With |s_mirror - s_exact| <= delta for
//   every row, every row outside the candidates has
//       s_exact <= s_mirror <= s_mirror[kc-1] + delta,
//   so once the exact k-th candidate score exceeds s_mirror[kc-1] + delta no
//   outside row can reach (or tie) the top-k: the result is then bit-identical
//   to mi_rank_topk over the master.  Uncertified queries (near-ties across the
//   candidate edge, non-finite scores) are flagged for the exact pass.
// delta (per query, |q| its f32 norm): the mirror rounding 2^-11 (fp16 RNE of
//   a unit row: the unit roundoff of an 11-bit significand, per element
//   |m_i - u_i| <= 2^-11 |u_i|, so |q.m - q.u| <= 2^-11 |q| by Cauchy-Schwarz), the query split (2^-22 SPLIT / 2^-11 hi only), the
//   f32 accumulation of both paths (bounded by 8 D 2^-24, covering the fp16
//   MFMA's internal sums), the subnormal floor 2^-25 sqrt(D) on both sides; the
//   sum is scaled by 1.25.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>

#include "common.hpp"
#include "internal.hpp"
#include "rank_keys.hpp"

namespace miclip {
namespace {
using namespace rankk;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int MQ = 32;   // queries per workgroup (MFMA N)

// ---- mirror build: 32 rows per wave (lane = (row, half) as the rank kernels load them)
template <int DT>
__global__ __launch_bounds__(256) void mirror_build_kernel(const void* __restrict__ master, int64_t N, int64_t D,
                                                           uint16_t* __restrict__ mirror) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * 32 + r;
  const bool valid = row < N;
  const int64_t rr = valid ? row : N - 1;
  const int nch = (int)(D / 32);
  float ss = 0.f;
  for (int j = 0; j < nch; ++j) {
    float v[16];
    load_chunk<DT>(master, rr, D, 32 * j + 16 * h, v);
#pragma unroll
    for (int i = 0; i < 16; ++i) ss = fmaf(v[i], v[i], ss);
  }
  ss += __shfl_xor(ss, 32, 64);
  const float inv = inv_norm(ss, 0);
  if (!valid) return;
  for (int j = 0; j < nch; ++j) {
    float v[16];
    load_chunk<DT>(master, rr, D, 32 * j + 16 * h, v);
    uint32_t w[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const _Float16 a = (_Float16)(v[2 * e] * inv), b = (_Float16)(v[2 * e + 1] * inv);
      w[e] = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
    }
    uint4* o = (uint4*)(mirror + row * D + 32 * j + 16 * h);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

// ---- mirror ranking pass (see the file comment)
// ILV: interleaved tile order (rank.hip rank_reg); otherwise each workgroup
// streams rows_per_wg contiguous rows
// PIPE: fragments read one chunk ahead (rank.hip rank_reg)
template <int D, bool SPLIT, bool ILV = false, bool PIPE = true, int NB = 8, int PF = 6, bool SPLITM = true>
__global__ __launch_bounds__(256) void rank_mirror_kernel(const uint16_t* __restrict__ mirror, int64_t N,
                                                          const float* __restrict__ queries, int64_t Q, int k,
                                                          int64_t rows_per_wg, int nan_first, FoldWs f,
                                                          float* __restrict__ out_s, int64_t* __restrict__ out_i) {
  constexpr int NW = 4, NT = 64 * NW, KC = 16, NCH = D / 64, NS = D / 16;
  constexpr int SLOT = 32 * 128;   // 32 rows x 64 k fp16
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;   // [NW][NB][SLOT]
  uint32_t* tau = (uint32_t*)(smem + NW * NB * SLOT);
  uint32_t* lead = tau + MQ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int64_t q0 = (int64_t)QB * MQ;
  const bool qvalid = q0 + r < Q;

  // queries -> fp16 B fragments: step s holds k = 16 s + 8 h + e (e = 0..7) of query r
  f16x8 qh[NS], ql[SPLIT ? NS : 1];
  {
    const float* qp = queries + (qvalid ? (q0 + r) : 0) * D + 8 * h;
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const float4 a = *(const float4*)(qp + 16 * st), b = *(const float4*)(qp + 16 * st + 4);
      const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = qvalid ? x[e] : 0.f;
        const _Float16 hi = (_Float16)xv;
        qh[st][e] = hi;
        if (SPLIT) ql[st][e] = (_Float16)(xv - (float)hi);
      }
    }
  }
  if (tid < MQ) tau[tid] = 0u;
  lead[tid] = 0u;   // 256 = 32 x 8
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // tile t of this wave: 32-row tile sid + t * sstep of rows [r_begin, r_end)
  const int G = NRB;
  const int64_t r_begin = ILV ? 0 : (int64_t)RB * rows_per_wg;
  const int64_t r_end = ILV ? N : min(N, r_begin + rows_per_wg);
  const int64_t nrows = r_end - r_begin;
  const int ntw = (int)((nrows + 31) / 32);
  const int sid = ILV ? wave * G + (int)RB : wave, sstep = ILV ? NW * G : NW;
  const int my_tiles = ntw > sid ? (ntw - 1 - sid) / sstep + 1 : 0;
  char* wring = ring + wave * NB * SLOT;

  // DMA: 4 x 1 KB per chunk; instruction m covers image rows 8m .. 8m + 7,
  // lane l row 8m + (l >> 3), LDS slot (l & 7), source piece (l & 7) ^ ((row >> 1) & 7)
  uint32_t voff[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int row = 8 * m + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    voff[m] = (uint32_t)(row * D * 2 + c * 16);
  }
  int lt = 0, lj = 0, lslot = 0;
  __amdgpu_buffer_rsrc_t rs;
  auto make_rs = [&]() {
    const int64_t trow = (int64_t)(sid + sstep * lt) * 32;   // relative to r_begin
    const int rows = (int)max((int64_t)0, min((int64_t)32, nrows - trow));
    const uint64_t base = (uint64_t)(uintptr_t)(mirror + (r_begin + (rows ? trow : 0)) * (int64_t)D);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const int nrec = __builtin_amdgcn_readfirstlane(rows * D * 2);
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0, nrec, 0x00020000);
  };
  make_rs();
  auto issue = [&]() {
    char* dst = wring + lslot * SLOT;
#pragma unroll
    for (int m = 0; m < 4; ++m)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(dst + m * 1024), 16, voff[m], lj * 128, 0, 0);
    lslot = lslot == NB - 1 ? 0 : lslot + 1;
    if (++lj == NCH) {
      lj = 0;
      ++lt;
      make_rs();
    }
  };
  const int rbase = r * 128;
  const int sw = (r >> 1) & 7;
  uint64_t L[KC];
#pragma unroll
  for (int p = 0; p < KC; ++p) L[p] = 0ull;
  uint32_t kk = 0u;   // running k-th key of this query's lists (own threshold)

  auto read_frag = [&](int slot, f32x4v (&v)[4]) {
    const char* src = wring + slot * SLOT + rbase;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t a = (uint32_t)(uintptr_t)(const LDS_AS char*)(src + (((2 * t + h) ^ sw) << 4));
      asm volatile("ds_read_b128 %0, %1" : "=v"(v[t]) : "v"(a) : "memory");
    }
  };
  if (my_tiles > 0) {
#pragma unroll
    for (int p = 0; p < PF; ++p) issue();
    int cslot = 0;
    f32x4v vb[2][4];
    if (PIPE) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (PF - 1)) : "memory");
      read_frag(0, vb[0]);
      cslot = 1;
    }
    for (int ct = 0; ct < my_tiles; ++ct) {
      f32x16 acc = f32x16{};
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        issue();
        f32x4v (&v)[4] = vb[PIPE ? (j & 1) : 0];
        if (PIPE) {
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(4 * (PF - 1)) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          read_frag(cslot, vb[(j + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PF) : "memory");
          read_frag(cslot, v);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f16x8 av = __builtin_bit_cast(f16x8, v[t]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, qh[4 * j + t], acc, 0, 0, 0);
          if (SPLIT) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, ql[4 * j + t], acc, 0, 0, 0);
        }
        cslot = cslot == NB - 1 ? 0 : cslot + 1;
      }
      const int tr0 = (sid + sstep * ct) * 32;
      const uint32_t tq_thr = tau[r];
      const uint32_t own = kk;   // the query's two half-lists' k-th: a lower bound of its k-th
      const uint32_t thr0 = own > tq_thr ? own : tq_thr;
      const uint32_t lb = lead_min(lead, r);
      const uint32_t thr = lb > thr0 ? lb : thr0;
      uint64_t c[16];
      bool any = false;
      uint32_t okm = 0u;
#pragma unroll
      for (int rg = 0; rg < 16; ++rg) {
        const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
        const int64_t gr = (int64_t)tr0 + rr;   // relative to r_begin
        const uint32_t key = score_key(acc[rg], nan_first);
        const bool ok = qvalid && gr < nrows && key >= thr;
        c[rg] = ok ? (((uint64_t)key << 32) | (uint32_t)~(uint32_t)gr) : 0ull;
        any |= ok;
        okm |= ok ? 1u << rg : 0u;
      }
      if (__any(any)) {
        list_update16(L, c, okm);
        lead_publish(lead, r, 2 * wave + h, (uint32_t)(L[1] >> 32));
        uint32_t kth = (uint32_t)(L[KC - 1] >> 32);   // k = kc = KC candidates
        const uint32_t other = (uint32_t)__shfl_xor((int)kth, 32, 64);
        kth = kth > other ? kth : other;
        kk = kth;
        if (h == 0 && qvalid && kth > tq_thr) tau_max(&tau[r], kth);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (SPLITM) {   // split merge: the lists raw, then fold_merge_kernel (rank_keys.hpp)
    lines_publish<NW>(L, smem, wave, lane, q0, Q, k, r_begin, f);
    return;
  }
  __syncthreads();   // ring free -> lists
  uint32_t* Lk = (uint32_t*)smem;
  int32_t* Li = (int32_t*)(smem + NT * KC * 4);
#pragma unroll
  for (int p = 0; p < KC; ++p) {
    const bool real = L[p] != 0ull;
    Lk[tid * KC + p] = real ? (uint32_t)(L[p] >> 32) : 0u;
    Li[tid * KC + p] = real ? (int32_t)~(uint32_t)L[p] : INT_MAX;
  }
  __syncthreads();
  fold_publish<2 * NW>(Lk, Li, KC, q0, Q, k, r_begin, f);
  fold_reduce<NT>(smem, f, q0, Q, k, nan_first, 0, out_s, out_i);
}

// ---- exact re-score of each query's kc mirror candidates (one wave per query)
// Lane (r, h) scores candidate slot r (rows past the list repeat slot 0) with
// rank.hip score_tile's arithmetic; every column of the MFMA B operand is the
// query, so lanes 0 and 32 hold the 32 slots' dot products.  The candidate
// rows are loaded whole up front (D / 2 VGPRs), one HBM latency per query.
template <int DT, int D>
__global__ __launch_bounds__(64) void mirror_rescore_kernel(const void* __restrict__ master, int64_t N,
                                                            const float* __restrict__ queries, int k, int kc,
                                                            const float* __restrict__ ms,
                                                            const int64_t* __restrict__ mi, int64_t index_base,
                                                            float d_rel, float d_abs, int norm_mode, int nan_first,
                                                            const int32_t* __restrict__ unsafe,
                                                            float* __restrict__ out_s, int64_t* __restrict__ out_i,
                                                            int32_t* __restrict__ cert, uint32_t* __restrict__ zero,
                                                            int64_t zero_words) {
  // the next launch's merge counters (the gated exact pass after a certified pass): cleared
  // here instead of by a memset dispatch of their own
  if (zero && blockIdx.x == 0)
    for (int64_t i = threadIdx.x; i < zero_words; i += 64) zero[i] = 0u;
  constexpr int NCH = D / 32;
  __shared__ float Tq[D];
  __shared__ float nrm[32];
  __shared__ float sc[32];
  __shared__ int64_t cid[32];
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int64_t q = blockIdx.x;
  float qq = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float x = queries[q * D + d];
    Tq[d] = x;
    qq = fmaf(x, x, qq);
  }
  qq = wave_sum(qq);
  const int64_t* cand = mi + q * kc;
  if (lane < 32) cid[lane] = lane < kc ? cand[lane] : -1;
  __syncthreads();
  const int64_t i0 = cid[0];
  const int64_t my = cid[r] >= 0 ? cid[r] : (i0 >= 0 ? i0 : 0);
  float row[NCH][16];
#pragma unroll
  for (int j = 0; j < NCH; ++j) load_chunk<DT>(master, my, D, 32 * j + 16 * h, row[j]);
  f32x16 acc = f32x16{};
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(row[j][i], Tq[32 * j + 16 * h + i], acc, 0, 0, 0);
      ss = fmaf(row[j][i], row[j][i], ss);
    }
  ss += __shfl_xor(ss, 32, 64);
  if (h == 0) nrm[r] = inv_norm(ss, norm_mode);
  __syncthreads();
  if (r == 0) {
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
      sc[rr] = acc[rg] * nrm[rr];
    }
  }
  __syncthreads();
  // lane j < nv: its rank among the candidates by (exact score desc, index asc)
  int nv = 0;
  while (nv < kc && cid[nv] >= 0) ++nv;
  const bool mine = lane < nv;
  const float s_me = mine ? sc[lane] : 0.f;
  const uint32_t k_me = score_key(s_me, nan_first);
  int rank = 0;
  for (int j = 0; j < nv; ++j) rank += (mine && j != lane && better(score_key(sc[j], nan_first), cid[j], k_me, cid[lane])) ? 1 : 0;
  if (mine && rank < k) {
    out_s[q * k + rank] = s_me;
    out_i[q * k + rank] = index_base + cid[lane];
  }
  if (lane >= nv && lane < k) {   // fewer candidates than k (N < k)
    out_s[q * k + lane] = -INFINITY;
    out_i[q * k + lane] = -1;
  }
  const bool fin = !mine || (isfinite(s_me) && isfinite(ms[q * kc + lane]));
  const bool all_fin = __all(fin);
  const float kth = __shfl(s_me, __ffsll((unsigned long long)__ballot(mine && rank == k - 1)) - 1, 64);
  if (lane == 0) {
    int ok;
    if (nv < kc) {
      ok = 1;   // the mirror returned every row: the candidates are the corpus
    } else {
      const float delta = d_rel * sqrtf(qq) + d_abs;
      ok = all_fin && nv >= k && kth > ms[q * kc + kc - 1] + delta;
    }
    if (unsafe && *unsafe) ok = 0;   // the pass met a row its bound does not cover (rank_cert.hip)
    cert[q] = ok;
  }
}

}  // namespace

constexpr int MIRROR_KC = 16;

static int64_t mirror_wgs(int64_t N) {
  int64_t nwg = (N + 127) / 128;
  return nwg < 256 ? nwg : 256;
}

size_t rank_mirror_workspace_bytes(int64_t N, int64_t Q) {
  const int64_t nwg = N > 0 ? mirror_wgs(N) : 1;
  return al128((size_t)(Q * MIRROR_KC) * (sizeof(float) + sizeof(int64_t))) + fold_ws_bytes(nwg, Q);
}

int rank_mirror_supported(int64_t D) { return D == 512 || D == 768; }

hipError_t mirror_build(const void* master, int64_t N, int64_t D, int dt, uint16_t* mirror, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const dim3 grid((unsigned)((N + 127) / 128));
  if (dt == 0) hipLaunchKernelGGL(mirror_build_kernel<0>, grid, dim3(256), 0, s, master, N, D, mirror);
  else if (dt == 1) hipLaunchKernelGGL(mirror_build_kernel<1>, grid, dim3(256), 0, s, master, N, D, mirror);
  else hipLaunchKernelGGL(mirror_build_kernel<2>, grid, dim3(256), 0, s, master, N, D, mirror);
  return hipGetLastError();
}

// delta = d_rel |q| + d_abs (file comment)
static void mirror_delta(int64_t D, bool split, float& d_rel, float& d_abs) {
  const double sq = std::sqrt((double)D) * std::ldexp(1.0, -25);
  const double rel = std::ldexp(1.0, -11) + (split ? std::ldexp(1.0, -22) : std::ldexp(1.0, -11)) +
                     8.0 * (double)D * std::ldexp(1.0, -24) + sq;
  d_rel = (float)(1.25 * rel);
  d_abs = (float)(1.25 * sq);
}

}  // namespace miclip

// Diagnostics (not part of include/miclip.h): the certificate's delta terms, so
// a host test can hold them against the analytic worst case (tests/test_abi.py).
extern "C" int mi_debug_mirror_delta(int64_t D, int split, float* d_rel, float* d_abs) {
  if (!d_rel || !d_abs || D < 1) return -1;   // MI_ERR_ARG
  miclip::mirror_delta(D, split != 0, *d_rel, *d_abs);
  return 0;
}

namespace miclip {

template <int D, bool SPLIT>
static hipError_t launch_mirror(const uint16_t* mirror, int64_t N, const float* q, int64_t Q, int kc, int nf,
                                void* fws, float* out_s, int64_t* out_i, int64_t nwg, hipStream_t s) {
  const size_t lds = (size_t)4 * 8 * 4096 + MQ * 4 + LEAD_LDS;
  const int64_t rpw = ((N + nwg - 1) / nwg + 127) / 128 * 128;   // whole tiles per wave round
  // MICLIP_MIRROR_VAR (A/B): 1 fragments read after the wait (no PIPE), 2 seven chunks in
  // flight, 3 interleaved tiles
#if MICLIP_AB
  const char* var = getenv("MICLIP_MIRROR_VAR");
  const int v = var ? atoi(var) : 0;
  // MICLIP_RANK_FOLD=1 (A/B): the in-launch merge instead of the split merge
  const char* fold = getenv("MICLIP_RANK_FOLD");
  const bool inl = fold && fold[0] == '1';
  auto fn = inl ? rank_mirror_kernel<D, SPLIT, false, true, 8, 6, false>
            : v == 1 ? rank_mirror_kernel<D, SPLIT, false, false>
            : v == 2 ? rank_mirror_kernel<D, SPLIT, false, true, 8, 7>
            : v == 3 ? rank_mirror_kernel<D, SPLIT, true> : rank_mirror_kernel<D, SPLIT>;
#else
  auto fn = rank_mirror_kernel<D, SPLIT>;
  constexpr bool inl = false;
#endif
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const dim3 grid((unsigned)((Q + MQ - 1) / MQ), (unsigned)nwg);   // (query blocks, row blocks): RB / QB
  const FoldWs f = fold_ws(fws, nwg, Q);
  if ((e = fold_zero(f, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(fn, grid, dim3(256), lds, s, mirror, N, q, Q, kc, rpw, nf, f, out_s, out_i);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return inl ? hipSuccess : fold_merge(f, nwg, Q, kc, nf, 0, out_s, out_i, nullptr, s);
}

hipError_t rank_mirror(const uint16_t* mirror, const void* master, int64_t N, int64_t D, int dt, const float* q,
                       int64_t Q, int k, int64_t base, int nan_first, float* out_s, int64_t* out_i, int32_t* cert,
                       void* ws, hipStream_t s) {
  const int kc = MIRROR_KC;
  const int64_t nwg = mirror_wgs(N);
  // the mirror's merged top-kc per query, then the in-launch merge's area
  float* m_s = (float*)ws;
  int64_t* m_i = (int64_t*)((char*)ws + (size_t)(Q * kc) * sizeof(float));
  void* fws = (char*)ws + al128((size_t)(Q * kc) * (sizeof(float) + sizeof(int64_t)));
  const bool split = D <= 512;
  hipError_t e = D == 512 ? launch_mirror<512, true>(mirror, N, q, Q, kc, nan_first, fws, m_s, m_i, nwg, s)
                          : launch_mirror<768, false>(mirror, N, q, Q, kc, nan_first, fws, m_s, m_i, nwg, s);
  if (e != hipSuccess) return e;
  float d_rel, d_abs;
  mirror_delta(D, split, d_rel, d_abs);
  return rank_rescore(master, N, D, dt, q, Q, k, kc, m_s, m_i, base, d_rel, d_abs, 0, nan_first, nullptr, out_s, out_i,
                      cert, s, nullptr, 0);
}

hipError_t rank_rescore(const void* master, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int k, int kc,
                        const float* m_s, const int64_t* m_i, int64_t base, float d_rel, float d_abs, int norm_mode,
                        int nan_first, const int32_t* unsafe, float* out_s, int64_t* out_i, int32_t* cert,
                        hipStream_t s, uint32_t* zero, int64_t zero_words) {
  if (Q <= 0) return hipSuccess;
  const dim3 grid((unsigned)Q);
#define MI_RS(DTV, DV)                                                                                                \
  hipLaunchKernelGGL((mirror_rescore_kernel<DTV, DV>), grid, dim3(64), 0, s, master, N, q, k, kc, m_s, m_i, base, \
                     d_rel, d_abs, norm_mode, nan_first, unsafe, out_s, out_i, cert, zero, zero_words)
  if (D == 512) {
    if (dt == 0) MI_RS(0, 512);
    else if (dt == 1) MI_RS(1, 512);
    else MI_RS(2, 512);
  } else if (D == 768) {
    if (dt == 0) MI_RS(0, 768);
    else if (dt == 1) MI_RS(1, 768);
    else MI_RS(2, 768);
  } else {
    return hipErrorInvalidValue;
  }
#undef MI_RS
  return hipGetLastError();
}

}  // namespace miclip
