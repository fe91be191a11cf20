// Certified ranking pass for large corpora (f32 / bf16 rows, D = 512, k <= 12):
// the ranking of EmbeddingService.search_top_frames (embedding_service.py:314-320:
// np.dot(E / ||E||, t.T) + argsort(s)[::-1][:k]) at bf16 MFMA rate, with results
// bit-identical to the exact pass (rank.hip rank_reg).
//
// The exact pass scores every row on the exact-f32 MFMA (157 TF): at Q = 32 its
// 2 N D Q flops take longer than streaming the rows (1M x 512 f32: 214 us of
// MFMA at peak beside 2 GB of HBM; bf16 rows: 1 GB, so the MFMA alone is twice
// the stream).  Here the rows go through bf16 MFMAs instead, as the fp16 mirror
// does (rank_mirror.hip), but from the caller's corpus itself, with no mirror:
//   * the f32 query is split into bf16 q1 + q2 (residual <= 2^-18 |q_i|), held
//     as MFMA B operands for the whole kernel (D / 2 VGPRs);
//   * bf16 rows are exact bf16 MFMA A operands; f32 rows are split in registers
//     into c_hi = bf16(c), c_lo = bf16(c - c_hi) (residual <= 2^-18 |c_i|), and
//     c_hi q1 + c_hi q2 + c_lo q1 are accumulated (c_lo q2 <= 2^-18 |c||q|);
//   * the row's sum of squares comes from the same fragments (fmaf in f32), so
//     the approximate score is dot * inv_norm(ss) with rank_keys' inv_norm;
//   * rank_reg's streaming structure: one wave per SIMD, a per-wave LDS ring of
//     4-KB chunks (32 rows x 32 k f32 or x 64 k bf16) by buffer-descriptor DMA
//     PF chunks ahead, counted waits, the bitonic top-16 lists, the shared
//     threshold tau and the in-launch merge (fold_publish / fold_reduce).
// Output: the top-16 rows of the APPROXIMATE scores per query.  rank_rescore
// (rank_mirror.hip) then scores those 16 with the exact pass's arithmetic, ranks
// them, and certifies a query when its exact k-th score exceeds the approximate
// 16th + delta: with |s_approx - s_exact| <= delta for every row, no row outside
// the candidates can then reach or tie the top-k, so the result is the exact
// pass's.  Uncertified queries (near-ties across the candidate edge) and every
// query of a call that met a row the bound does not cover (non-finite approximate
// score, sum of squares outside [1e-15, 1e36]: zero rows, overflow, the guarded
// norm's threshold) are re-ranked by the exact pass (rank_reg gated by the
// certificates: fully certified 32-query blocks exit at once).
//
// delta = d_rel |q| + d_abs, per term (|s| <= |q| for the cosine):
//   query split 2^-18 and, f32 rows, row split 2^-18 plus the dropped c_lo q2
//   2^-18; accumulation: the bf16 MFMA path sums P = 2 D (bf16) / 3 D (f32)
//   products (2 P 2^-24, allowing internal truncation), the exact chain D 2^-24;
//   the norm: both sums of squares within D 2^-24 relatively, sqrt and the
//   reciprocal 2^-21 -> D 2^-24 + 2^-20 of |s|; the subnormal floor 2^-25 sqrt(D)
//   on both sides; all scaled by 1.25.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "internal.hpp"
#include "rank_keys.hpp"

namespace miclip {
namespace {
using namespace rankk;

typedef float f32x4c __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));
constexpr int CD = 512;   // supported D
constexpr int CKC = 16;   // candidates per query

template <int... Is, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): a loop whose index is a constant expression
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// a lane's four fragment pieces of the ring slot at byte offset OFF
template <int OFF>
__device__ __forceinline__ void read_frag(const uint32_t (&fa)[4], f32x4c (&v)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[t]) : "v"(fa[t]), "n"(OFF) : "memory");
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// the ring, per-wave row reciprocals [4][32], tau [32], the lead keys [32][8], the
// per-wave candidate buckets [4][CBK][64] u64
constexpr int CNB = 8, CBK = 12;
constexpr size_t cert_bucket_off() { return (size_t)4 * CNB * 4096 + 4 * 32 * 4 + 32 * 4 + LEAD_LDS; }
constexpr size_t cert_lds_bytes() { return cert_bucket_off() + (size_t)4 * CBK * 64 * 8; }

// per wave (row block y < 256, wave w): tile-epilogue cycles, tiles, tiles with candidates, bucket flushes,
// updates, multi-candidate insertion updates (ABL 5, A/B build; mi_debug_cert_probe)
__device__ unsigned long long g_cert_probe[256 * 4 * 5];

// ABL (A/B timing probes, wrong results): 1 = no Gram MFMAs (unit norms), 2 = no MFMAs at
// all, 3 = no list update, 7 = no bucket writes; 5 = the epilogue stamp probe, 6 = the bucket
// writes at the tile end instead of spread over the next tile (correct results)
template <int DT, int ABL = 0, bool SPLITM = true>
__global__ __launch_bounds__(256) void rank_cert_kernel(const void* __restrict__ corpus, int64_t N,
                                                        const float* __restrict__ queries, int64_t Q, int kc,
                                                        int64_t rows_per_wg, int norm_mode, int nan_first, FoldWs f,
                                                        int32_t* __restrict__ unsafe, float* __restrict__ out_s,
                                                        int64_t* __restrict__ out_i) {
  constexpr int D = CD, NW = 4, NT = 64 * NW, KC = CKC, NB = CNB;
  // chunks in flight: bf16 rows read their fragments one chunk ahead, so a slot is free once
  // its fragments have arrived (PF = NB); f32 rows read the chunk itself (PF = NB - 1)
  constexpr int PF = DT ? NB : NB - 1;
  constexpr int ES = DT ? 2 : 4;           // bytes per element
  constexpr int KCH = 128 / ES;            // k per 4-KB chunk (32 rows x 128 B)
  constexpr int NCH = D / KCH;             // chunks per 32-row tile
  constexpr int NS = D / 16;               // bf16 MFMA k-steps
  constexpr int SLOT = 32 * 128;
  static_assert(NB >= PF + (DT ? 0 : 1), "rank_cert: a refilled ring slot must have been read in an earlier chunk");
  static_assert(4 * PF <= 63, "rank_cert: vmcnt(4 PF) exceeds the counter");
  static_assert(cert_lds_bytes() <= 160 * 1024, "rank_cert: ring exceeds the LDS");
  static_assert(cert_lds_bytes() >= (size_t)NT * KC * 8, "rank_cert: list merge area exceeds the allocation");
  static_assert(cert_lds_bytes() >= fold_lds(NT), "rank_cert: in-launch merge area exceeds the allocation");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* nrm_all = (float*)(smem + NW * NB * SLOT);
  uint32_t* tau = (uint32_t*)(nrm_all + NW * 32);
  uint32_t* lead = tau + 32;
  const int tid = threadIdx.x, lane = tid & 63;
  // this lane's candidate bucket: slot j at bkt + 512 j (slot-major, conflict-free)
  const uint32_t bkt = (uint32_t)(uintptr_t)(LDS_AS char*)(smem + cert_bucket_off()) +
                       (uint32_t)((tid >> 6) * CBK * 512 + (tid & 63) * 8);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int64_t q0 = (int64_t)QB * FQ;
  const bool qvalid = q0 + r < Q;

  // queries -> bf16 B fragments q1 + q2: step s holds k = 16 s + 8 h + e of query r
  bf16x8 q1[NS], q2[NS];
  bool qbad = false;
  {
    const float* qp = queries + (qvalid ? (q0 + r) : 0) * D + 8 * h;
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const float4 a = *(const float4*)(qp + 16 * st), b = *(const float4*)(qp + 16 * st + 4);
      const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = qvalid ? x[e] : 0.f;
        qbad |= !(__builtin_fabsf(xv) <= 1e15f);   // non-finite or huge: scores could overflow
        const __bf16 hi = (__bf16)xv;
        q1[st][e] = hi;
        q2[st][e] = (__bf16)(xv - (float)hi);
      }
    }
  }
  if (tid < FQ) tau[tid] = 0u;
  lead[tid] = 0u;   // 256 = 32 x 8
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int64_t r_begin = (int64_t)RB * rows_per_wg;
  const int64_t r_end = min(N, r_begin + rows_per_wg);
  const int64_t nrows = r_end - r_begin;
  const int ntw = (int)((nrows + 31) / 32);
  const int my_tiles = ntw > wave ? (ntw - 1 - wave) / NW + 1 : 0;
  char* wring = ring + wave * NB * SLOT;
  float* nrm = nrm_all + wave * 32;

  // DMA: 4 x 1 KB per chunk; instruction m covers image rows 8m .. 8m + 7,
  // lane l row 8m + (l >> 3), LDS slot (l & 7), source piece (l & 7) ^ ((row >> 1) & 7)
  uint32_t voff[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int row = 8 * m + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    voff[m] = (uint32_t)(row * D * ES + c * 16);
  }
  int lt = 0, lj = 0, lslot = 0;
  __amdgpu_buffer_rsrc_t rs;
  auto make_rs = [&]() {
    const int64_t trow = (int64_t)(wave + NW * lt) * 32;   // relative to r_begin
    const int rows = (int)max((int64_t)0, min((int64_t)32, nrows - trow));
    const uint64_t base = (uint64_t)(uintptr_t)((const char*)corpus + (r_begin + (rows ? trow : 0)) * (int64_t)D * ES);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const int nrec = __builtin_amdgcn_readfirstlane(rows * D * ES);
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
  // fragment pieces of this lane in a chunk: bf16 rows, k-step t: piece 2t + h;
  // f32 rows, k-step t: pieces 4t + 2h and 4t + 2h + 1
  // The 16-row tile takes NCH chunks and NCH is a multiple of NB, so the slot a chunk
  // reads is a compile-time function of its position in the tile: the slot goes in the
  // ds_read's immediate offset, and the per-lane part (4 addresses) is fixed for the kernel
  // (hipcc otherwise kept all 8 x 4 slot addresses live across the tile loop).
  static_assert(NCH % NB == 0, "rank_cert: the ring slot of a chunk must be static");
  uint32_t fa[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int piece = DT ? 2 * t + h : 4 * (t >> 1) + 2 * h + (t & 1);
    fa[t] = (uint32_t)(uintptr_t)(const LDS_AS char*)(wring + rbase + ((piece ^ sw) << 4));
  }
  uint64_t L[KC];
#pragma unroll
  for (int p = 0; p < KC; ++p) L[p] = 0ull;
  unsigned long long pr_cyc = 0ull, pr_t0 = 0ull;   // ABL 5 probe
  unsigned pr_n[4] = {0u, 0u, 0u, 0u};
  uint32_t kk = 0u;   // running k-th key of this query's lists (own threshold)
  uint32_t bcnt = 0u;  // entries in this lane's bucket
  bool bad = qbad;
  // the bucket's entries into L, one insertion round per slot (an entry at a time: the
  // 64-bit sort of a whole bucket would need registers the query fragments hold)
  auto flush = [&]() {
    for (uint32_t j = 0; __any(j < bcnt); ++j) {
      uint64_t e;
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(e) : "v"(bkt + 512u * j) : "memory");
      e = j < bcnt ? e : 0ull;
#pragma unroll
      for (int p = 15; p > 0; --p) L[p] = e > L[p - 1] ? L[p - 1] : (e > L[p] ? e : L[p]);
      L[0] = e > L[0] ? e : L[0];
    }
    bcnt = 0u;
  };

  // The previous tile's scores P and candidate mask pokm (rows ptr0 + rr): their bucket
  // writes are spread over the next tile's chunks (PPC per chunk, after its MFMAs), so
  // the DMA issue keeps its pace and the writes' VALU issues beside the MFMAs.
  constexpr int PPC = 16 / NCH;
  f32x16 P = f32x16{};
  uint32_t pokm = 0u;
  int ptr0 = 0;
  auto put = [&](int rg) {   // candidate rg of the previous tile -> this lane's bucket
    if ((pokm >> rg) & 1u) {
      const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
      const uint64_t e = ((uint64_t)score_key(P[rg], nan_first) << 32) | (uint32_t)~(uint32_t)(ptr0 + rr);
      asm volatile("ds_write_b64 %0, %1" ::"v"(bkt + 512u * bcnt), "v"(e) : "memory");
      ++bcnt;
    }
  };

  if (my_tiles > 0) {
#pragma unroll
    for (int p = 0; p < PF; ++p) issue();
    // bf16 rows: fragments read one chunk ahead (two register buffers, as the mirror pass);
    // f32 rows: one buffer, read after the chunk's wait (the split's temporaries need the VGPRs)
    constexpr bool PIPE = DT != 0;
    f32x4c vb[PIPE ? 2 : 1][4];
    if (PIPE) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (PF - 1)) : "memory");
      read_frag<0>(fa, vb[0]);
    }
    for (int ct = 0; ct < my_tiles; ++ct) {
      // two accumulators (the q2 terms apart): two independent MFMA chains per chunk
      f32x16 acc = f32x16{}, acc2 = f32x16{};
      f32x16 gram = ABL == 1 ? f32x16{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f}
                             : f32x16{};   // bf16 rows
      float ss = 0.f;           // f32 rows (this lane's half of row r)
      static_for<NCH>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        // bf16: this chunk's fragments (read in the previous chunk) have arrived before its
        // slot is refilled with chunk j + PF (PF = NB)
        if (PIPE) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue();
        f32x4c (&v)[4] = vb[PIPE ? (j & 1) : 0];
        if (PIPE) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (PF - 1)) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          read_frag<(j + 1) % NB * SLOT>(fa, vb[PIPE ? ((j + 1) & 1) : 0]);
          __builtin_amdgcn_sched_barrier(0);
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PF) : "memory");
          read_frag<j % NB * SLOT>(fa, v);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
        if (DT) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const bf16x8 av = __builtin_bit_cast(bf16x8, v[t]);
            if (ABL == 2) {
              asm volatile("" ::"v"(av));
              continue;
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, q1[4 * j + t], acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, q2[4 * j + t], acc2, 0, 0, 0);
            // the tile's Gram matrix: the A fragment is also the B fragment of the
            // transposed rows, so its diagonal is each row's sum of squares
            if (ABL != 1) gram = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, av, gram, 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const float x[8] = {v[2 * t][0], v[2 * t][1], v[2 * t][2], v[2 * t][3],
                                v[2 * t + 1][0], v[2 * t + 1][1], v[2 * t + 1][2], v[2 * t + 1][3]};
            uint32_t ph[4], pl[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              ph[e] = pack_bf16x2(x[2 * e], x[2 * e + 1]);
              pl[e] = pack_bf16x2(x[2 * e] - bf_lo(ph[e]), x[2 * e + 1] - bf_hi(ph[e]));
            }
            const bf16x8 ah = __builtin_bit_cast(bf16x8, (u32x4c){ph[0], ph[1], ph[2], ph[3]});
            const bf16x8 al = __builtin_bit_cast(bf16x8, (u32x4c){pl[0], pl[1], pl[2], pl[3]});
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, q1[2 * j + t], acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, q2[2 * j + t], acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, q1[2 * j + t], acc, 0, 0, 0);
#pragma unroll
            for (int e = 0; e < 8; ++e) ss = fmaf(x[e], x[e], ss);
            // pinned here: hipcc sank the whole tile's fmaf chain to the tile end and kept
            // the 256 row values it needs live (in AGPRs), spilling the query fragments
            asm volatile("" : "+v"(ss));
          }
        }
        if (ABL != 3 && ABL != 6 && ABL != 7) {
#pragma unroll
          for (int i = 0; i < PPC; ++i) put(PPC * j + i);
        }
      });
      if (ABL == 6) {   // probe: the previous tile's bucket writes here, not spread over the chunks
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) put(rg);
      }
      // row r's reciprocal norm (lanes r and r + 32 hold its two halves) -> the wave's
      // LDS slots, read back in the accumulator's row order
      if (DT) {
        // Gram diagonal: G[row i][col c] sits in lane c + 32 h at register rho with
        // i = (rho & 3) + 8 (rho >> 2) + 4 h, so row c's sum of squares G[c][c] is in lane
        // c + 32 bit2(c), register (c & 3) + 4 (c >> 3); the other lane of column c fetches it
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int cc = ln & 31, hh = ln >> 5, rho = (cc & 3) + 4 * (cc >> 3);
        float d = gram[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) d = rho == i ? gram[i] : d;
        const bool holds = ((cc >> 2) & 1) == hh;
        const float o = __shfl(d, cc + 32 * (1 - hh), 64);
        ss = holds ? d : o;
      } else {
        ss += __shfl_xor(ss, 32, 64);
      }
      const int tr0 = (wave + NW * ct) * 32;
      const bool rvalid = (int64_t)tr0 + r < nrows;
      // also the scores' guard: with the sum of squares in range and a finite query of
      // moderate norm (checked at entry) every score is finite
      bad |= rvalid && !(ss >= 1e-15f && ss <= 1e36f);
      {
        // the lane id recomputed here (v_mbcnt) rather than kept live across the tile:
        // hipcc otherwise spills this LDS address, and the reload's vmcnt(0) drains the ring
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        if (ln < 32) nrm[ln] = inv_norm(ss, norm_mode);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      if (ABL == 5) pr_t0 = __builtin_amdgcn_s_memtime();
      const uint32_t tq_thr = tau[r];
      const uint32_t own = kk;   // the query's two half-lists' k-th: a lower bound of its k-th
      const uint32_t thr0 = own > tq_thr ? own : tq_thr;
      const uint32_t lb = lead_min(lead, r);
      const uint32_t thr = lb > thr0 ? lb : thr0;
      // the key threshold as a score: score_key is monotone on finite scores (-0 = +0), so
      // key >= thr <=> s >= tf; keys below key(-inf) admit every finite score
      const float tf = thr < 0x00800000u ? -INFINITY
                                         : __uint_as_float((thr & 0x80000000u) ? (thr & 0x7fffffffu) : ~thr);
      const int vrows = (int)min((int64_t)32, nrows - tr0);   // valid rows of this tile
      // the 16 rows' reciprocals: rows (rg & 3) + 8 (rg >> 2) + 4 h are four 16-byte runs
      f32x4c nv[4];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) nv[q4] = *(const f32x4c*)(nrm + 8 * q4 + 4 * h);
      uint32_t okm = 0u;
#pragma unroll
      for (int rg = 0; rg < 16; ++rg) {
        const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
        const float sc = (acc[rg] + acc2[rg]) * nv[rg >> 2][rg & 3];
        P[rg] = sc;
        okm |= (qvalid && rr < vrows && sc >= tf) ? 1u << rg : 0u;
      }
      ptr0 = tr0;
      if (ABL == 5) {
        pr_n[1] += __any(okm != 0u) ? 1u : 0u;
        pr_n[3] += __all(__builtin_popcount(okm) <= 1) ? 0u : 1u;
      }
      // a bucket that this tile's candidates could overflow: merge it into the lists now and
      // refresh the thresholds; a tile with more candidates than a bucket holds (the first
      // ones, before the thresholds rise) is inserted directly, one candidate per round
      const uint32_t pc = (uint32_t)__builtin_popcount(okm);
      if (ABL != 3 && __any(bcnt + pc > (uint32_t)CBK)) {
        if (ABL == 5) pr_n[2] += 1u;
        if (__any(bcnt != 0u)) flush();
        if (__any(pc > (uint32_t)CBK)) {
          uint32_t m = okm;
          while (__any(m != 0u)) {
            const int i = m ? __builtin_ctz(m) : 0;
            float sc = P[0];
#pragma unroll
            for (int rg = 1; rg < 16; ++rg) sc = rg == i ? P[rg] : sc;
            const int rr = (i & 3) + 8 * (i >> 2) + 4 * h;
            const uint64_t e = m ? (((uint64_t)score_key(sc, nan_first) << 32) | (uint32_t)~(uint32_t)(tr0 + rr)) : 0ull;
#pragma unroll
            for (int p = 15; p > 0; --p) L[p] = e > L[p - 1] ? L[p - 1] : (e > L[p] ? e : L[p]);
            L[0] = e > L[0] ? e : L[0];
            m &= m - 1u;
          }
          okm = 0u;
        }
        {
          // lane id recomputed (v_mbcnt): a live-across-the-tile LDS address gets spilled, and
          // its reload's vmcnt(0) would drain the ring
          const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
          lead_publish(lead, ln & 31, 2 * wave + (ln >> 5), (uint32_t)(L[1] >> 32));
        }
        uint32_t kth = (uint32_t)(L[KC - 1] >> 32);   // k = kc = KC candidates
        const uint32_t other = (uint32_t)__shfl_xor((int)kth, 32, 64);
        kth = kth > other ? kth : other;
        kk = kth;
        if (h == 0 && qvalid && kth > tq_thr) tau_max(&tau[r], kth);
      }
      pokm = okm;
      if (ABL == 5) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pr_cyc += __builtin_amdgcn_s_memtime() - pr_t0;
        pr_n[0] += 1u;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the norm reads, before the slots are rewritten
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (ABL != 3) {
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) put(rg);   // the last tile's candidates
  }
  if (ABL != 3 && __any(bcnt != 0u)) flush();
  if (ABL == 5 && lane == 0 && (int)blockIdx.y < 256) {
    unsigned long long* o = g_cert_probe + ((int)blockIdx.y * 4 + wave) * 5;
    o[0] = pr_cyc;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[1 + i] = pr_n[i];
  }
  if (__any(bad) && lane == 0) __hip_atomic_store(unsafe, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (SPLITM) {   // split merge: the lists raw, then fold_merge_kernel (rank_keys.hpp)
    lines_publish<NW>(L, smem, wave, lane, q0, Q, kc, r_begin, f);
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
  fold_publish<2 * NW>(Lk, Li, KC, q0, Q, kc, r_begin, f);
  fold_reduce<NT>(smem, f, q0, Q, kc, nan_first, 0, out_s, out_i);
}

}  // namespace

int64_t rank_cert_min_rows() {
#if MICLIP_AB
  // MICLIP_RANK_CERT (A/B): 0 = never, 2 = every eligible call regardless of N (tests)
  const char* e = getenv("MICLIP_RANK_CERT");
  if (e && e[0] == '0') return INT64_MAX;
  if (e && e[0] == '2') return 1;
#endif
  // below ~256k rows the fixed re-score and merge cost eat the gain (the mirror's threshold)
  return 262144;
}

bool rank_cert_eligible(int64_t N, int64_t D, int dt, int k, int norm_mode) {
  return D == CD && (dt == 0 || dt == 1) && k >= 1 && k <= 12 && norm_mode != 2 && N >= rank_cert_min_rows();
}

static int64_t cert_wgs(int64_t N) {
  int64_t nwg = (N + 127) / 128;
  return nwg < 256 ? nwg : 256;
}

// [m_s Q x 16 f32][m_i Q x 16 i64][cert Q i32][unsafe][fold workspace]
size_t rank_cert_ws_bytes(int64_t N, int64_t Q) {
  const int64_t nwg = N > 0 ? cert_wgs(N) : 1;
  return al128((size_t)(Q * CKC) * (sizeof(float) + sizeof(int64_t))) + al128((size_t)Q * 4 + 4) + fold_ws_bytes(nwg, Q);
}

void rank_cert_delta(int dt, float& d_rel, float& d_abs) {
  const double D = CD, u = std::ldexp(1.0, -24);
  const double sq = std::sqrt(D) * std::ldexp(1.0, -25);
  const double split = dt == 0 ? 3.0 * std::ldexp(1.0, -18) : std::ldexp(1.0, -18);
  const double P = dt == 0 ? 3.0 * D : 2.0 * D;
  const double rel = split + (2.0 * P + D) * u + (D * u + std::ldexp(1.0, -20)) + sq;
  d_rel = (float)(1.25 * rel);
  d_abs = (float)(1.25 * sq);
}

hipError_t rank_cert_topk(const void* corpus, int64_t N, int dt, const float* q, int64_t Q, int k, int64_t base,
                          int norm_mode, int nan_first, float* out_s, int64_t* out_i, void* ws, int32_t** cert_out,
                          hipStream_t s, uint32_t* zero, int64_t zero_words) {
  const int64_t nwg = cert_wgs(N);
  float* m_s = (float*)ws;
  int64_t* m_i = (int64_t*)((char*)ws + (size_t)(Q * CKC) * sizeof(float));
  int32_t* cert = (int32_t*)((char*)ws + al128((size_t)(Q * CKC) * (sizeof(float) + sizeof(int64_t))));
  void* fws = (char*)cert + al128((size_t)Q * 4 + 4);
  *cert_out = cert;
  hipError_t e;
  const int64_t rpw = ((N + nwg - 1) / nwg + 127) / 128 * 128;   // whole tiles per wave round
  const int64_t nwg_used = (N + rpw - 1) / rpw;                  // <= nwg (the workspace's count)
  const FoldWs fu = fold_ws(fws, nwg_used, Q);
  // one memset for the merge counters, gtau and the unsafe flag (the fold workspace's aux word):
  // each fill is a ~5 us dispatch of its own at this size (scripts/gpu_r4p.sh trace)
  int32_t* unsafe = (int32_t*)fu.aux;
  if ((e = fold_zero(fu, s)) != hipSuccess) return e;
  const size_t lds = cert_lds_bytes();
  const dim3 grid((unsigned)((Q + FQ - 1) / FQ), (unsigned)nwg_used);   // (query blocks, row blocks)
#if MICLIP_AB
  const char* ab = getenv("MICLIP_RANK_CERT_ABL");   // timing probes (wrong results)
  const int abl = ab ? atoi(ab) : 0;
#endif
  auto fn = dt == 0 ? rank_cert_kernel<0> : rank_cert_kernel<1>;
  bool inl = false;   // the in-launch merge (A/B: MICLIP_RANK_FOLD=1)
#if MICLIP_AB
  const char* fold = getenv("MICLIP_RANK_FOLD");
  inl = fold && fold[0] == '1';
  if (inl) fn = dt == 0 ? rank_cert_kernel<0, 0, false> : rank_cert_kernel<1, 0, false>;
  if (abl == 1) fn = dt == 0 ? rank_cert_kernel<0, 1> : rank_cert_kernel<1, 1>;
  else if (abl == 2) fn = dt == 0 ? rank_cert_kernel<0, 2> : rank_cert_kernel<1, 2>;
  else if (abl == 3) fn = dt == 0 ? rank_cert_kernel<0, 3> : rank_cert_kernel<1, 3>;
  else if (abl == 5) fn = dt == 0 ? rank_cert_kernel<0, 5> : rank_cert_kernel<1, 5>;
  else if (abl == 6) fn = dt == 0 ? rank_cert_kernel<0, 6> : rank_cert_kernel<1, 6>;
  else if (abl == 7) fn = dt == 0 ? rank_cert_kernel<0, 7> : rank_cert_kernel<1, 7>;
#endif
  if ((e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(fn, grid, dim3(256), lds, s, corpus, N, q, Q, CKC, rpw, norm_mode, nan_first, fu, unsafe, m_s, m_i);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (!inl && (e = fold_merge(fu, nwg_used, Q, CKC, nan_first, 0, m_s, m_i, nullptr, s)) != hipSuccess) return e;
  float d_rel, d_abs;
  rank_cert_delta(dt, d_rel, d_abs);
  return rank_rescore(corpus, N, CD, dt, q, Q, k, CKC, m_s, m_i, base, d_rel, d_abs, norm_mode, nan_first, unsafe,
                      out_s, out_i, cert, s, zero, zero_words);
}

}  // namespace miclip

// Diagnostics (not part of include/miclip.h): the certificate's delta terms for
// f32 (dt 0) and bf16 (dt 1) rows at D = 512, for a host test (tests/test_abi.py).
extern "C" int mi_debug_cert_probe(unsigned long long* host, int n) {
#if MICLIP_AB
  if (n > 256 * 4 * 5) n = 256 * 4 * 5;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(miclip::g_cert_probe), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
#else
  (void)host;
  (void)n;
  return -2;   // A/B build only
#endif
}

extern "C" int mi_debug_cert_delta(int dt, float* d_rel, float* d_abs) {
  if (!d_rel || !d_abs || (dt != 0 && dt != 1)) return -1;   // MI_ERR_ARG
  miclip::rank_cert_delta(dt, *d_rel, *d_abs);
  return 0;
}
