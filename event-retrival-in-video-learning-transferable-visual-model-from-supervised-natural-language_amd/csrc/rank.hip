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
#include <cstdlib>

#include "common.hpp"
#include "internal.hpp"
#include "rank_keys.hpp"

namespace miclip {
namespace {
using namespace rankk;

constexpr int RQ = 32;          // queries per workgroup (MFMA N)
constexpr int ROWS_WAVE = 32;   // corpus rows per wave tile (MFMA M)




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

// Streaming stage 1 (the default for k <= 16, rank_stream): the same
// 32-row x 32-query wave tiles and exact-f32 MFMA arithmetic as rank_stage1,
// rebuilt around the memory stream and a data-independent top-k update:
//  * a wave's tiles are ONE continuous stream of 32-k chunks (tile after
//    tile), loaded two chunks ahead into three register buffers used in place
//    (the chunk loop is unrolled by 3, so no buffer is copied: a copy of a
//    freshly loaded register waits for its load and caps the lookahead at one
//    chunk); the next tile's first chunks are in flight while a tile finishes;
//  * NW waves per workgroup share one LDS copy of the 32 queries;
//  * top-k: a candidate is one u64, (score key << 32) | ~row, so "better"
//    (key desc, row asc) is a single unsigned compare.  After each tile a
//    lane sorts its 16 new candidates with a bitonic network and merges them
//    into its sorted list of 16 (max of the list and the reversed candidates,
//    then a bitonic clean-up): ~112 compare-exchanges per tile whatever the
//    data.  rank_stage1 inserted candidate by candidate under a wave vote,
//    which fires on nearly every row of the first tiles (64 independent lists)
//    and cost 3x the MFMA issue in VALU (PMC: 126M VALU vs 8M MFMA at 1M
//    rows);
//  * the tile is skipped when no lane has a candidate above
//    max(its list's 16th key, tau[q]), tau[q] (LDS) = max over the workgroup's
//    lists of their k-th key: a score below it cannot reach the workgroup's
//    top-k (that list already holds k better rows).
// LDS: queries [32][D+4] f32, row norms [NW][32], tau [32]; the lists
// [64*NW lanes][16] (key u32, idx i32) reuse the query area after a barrier.

template <int DT, int NW, bool SPLITM = true>
__global__ __launch_bounds__(64 * NW) void rank_stream(const void* __restrict__ corpus, int64_t N, int64_t D,
                                                       const float* __restrict__ queries, int64_t Q, int k,
                                                       int64_t rows_per_wg, int norm_mode, int nan_first,
                                                       int64_t index_base, FoldWs f, float* __restrict__ out_s,
                                                       int64_t* __restrict__ out_i) {
  constexpr int NT = 64 * NW, KC = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ts_stride = (int)D + 4;
  float* Ts = (float*)smem;
  float* nrm_all = Ts + RQ * ts_stride;
  uint32_t* tau = (uint32_t*)(nrm_all + NW * 32);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t q0 = (int64_t)QB * RQ;

  for (int64_t e = tid; e < RQ * D; e += NT) {
    const int qq = (int)(e / D);
    const int64_t d = e % D;
    Ts[qq * ts_stride + d] = (q0 + qq < Q) ? queries[(q0 + qq) * D + d] : 0.f;
  }
  if (tid < RQ) tau[tid] = 0u;
  __syncthreads();

  const int64_t r_begin = (int64_t)RB * rows_per_wg;
  const int64_t r_end = min(N, r_begin + rows_per_wg);
  float* nrm = nrm_all + wave * 32;
  const int64_t ntw = (r_end - r_begin + 31) / 32;
  const int my_tiles = ntw > wave ? (int)((ntw - 1 - wave) / NW + 1) : 0;
  const int nch = (int)(D / 32);
  const int64_t total = (int64_t)my_tiles * nch;
  const int nrows = (int)(r_end - r_begin);

  uint64_t L[KC];
#pragma unroll
  for (int p = 0; p < KC; ++p) L[p] = 0ull;      // (key 0, row ~0): below every real candidate
  const bool qvalid = q0 + r < Q;
  const float* tq = Ts + r * ts_stride + 16 * h;

  int lt = 0, lj = 0;  // load cursor (tile ordinal, chunk); loads past the end re-read a valid row
  auto next_load = [&](float (&buf)[16]) {
    const int64_t row = min(r_begin + (int64_t)(wave + NW * lt) * 32 + r, N - 1);
    load_chunk<DT>(corpus, row, D, 32 * lj + 16 * h, buf);
    if (++lj == nch) { lj = 0; ++lt; }
  };
  int ct = 0, cj = 0;  // compute cursor
  f32x16 acc = f32x16{};
  float ss = 0.f;
  auto finalize = [&]() {
    ss += __shfl_xor(ss, 32, 64);
    if (h == 0) nrm[r] = inv_norm(ss, norm_mode);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int tr0 = (wave + NW * ct) * 32;           // tile's first row, relative to r_begin
    const uint32_t tq_thr = tau[r];
    const uint32_t own = (uint32_t)(L[KC - 1] >> 32);
    const uint32_t thr = own > tq_thr ? own : tq_thr;
    uint64_t c[16];
    bool any = false;
    uint32_t okm = 0u;
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
      const int lr = tr0 + rr;
      const float sc = norm_mode == 2 ? acc[rg] : acc[rg] * nrm[rr];
      const uint32_t key = score_key(sc, nan_first);
      const bool ok = qvalid && lr < nrows && key >= thr;
      c[rg] = ok ? (((uint64_t)key << 32) | (uint32_t)~(uint32_t)lr) : 0ull;
      any |= ok;
      okm |= ok ? 1u << rg : 0u;
    }
    if (__any(any)) {
      list_update16(L, c, okm);
      // publish this list's k-th key (a lower bound of the query's k-th best)
      uint32_t kth = (uint32_t)(L[0] >> 32);
#pragma unroll
      for (int p = 1; p < KC; ++p) kth = (p == k - 1) ? (uint32_t)(L[p] >> 32) : kth;
      const uint32_t other = (uint32_t)__shfl_xor((int)kth, 32, 64);
      kth = kth > other ? kth : other;
      if (h == 0 && qvalid && kth > tq_thr) tau_max(&tau[r], kth);
    }
    __builtin_amdgcn_wave_barrier();
    acc = f32x16{};
    ss = 0.f;
    ++ct;
    cj = 0;
  };
  auto consume = [&](const float (&buf)[16]) {
    float tb[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 t = *(const float4*)(tq + 32 * cj + 4 * i);
      tb[4 * i] = t.x; tb[4 * i + 1] = t.y; tb[4 * i + 2] = t.z; tb[4 * i + 3] = t.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(buf[i], tb[i], acc, 0, 0, 0);
      ss = fmaf(buf[i], buf[i], ss);
    }
    if (++cj == nch) finalize();
  };

  // Three register buffers used in place, loaded two chunks ahead (hipcc's
  // own counted waits; measured 3.8-4.0 TB/s at 1M rows).  Tried and
  // rejected: a padded exit-free body with sched_barriers (hipcc then drained
  // the ring at the back-edge) and inline-asm loads with hand-counted waits
  // (hipcc copies the in-flight registers).
  if (total > 0) {
    float b0[16], b1[16], b2[16];
    next_load(b0);
    next_load(b1);
    for (int64_t c = 0; c < total; c += 3) {
      next_load(b2);
      consume(b0);
      if (c + 1 >= total) break;
      next_load(b0);
      consume(b1);
      if (c + 2 >= total) break;
      next_load(b1);
      consume(b2);
    }
  }
  if (SPLITM) {   // split merge: the workgroup's top-k published, then fold_merge_kernel
    lines_publish<NW>(L, smem, wave, lane, q0, Q, k, r_begin, f);   // (its first barrier: the query area is free)
    return;
  }
  __syncthreads();  // query area free -> lists
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
  fold_reduce<NT>(smem, f, q0, Q, k, nan_first, index_base, out_s, out_i);
}

// Register-query streaming stage 1 (f32 corpus, D = 512, k <= 16:
// rank_reg; rank_stream otherwise).  PMC of rank_stream at 1M x 512, Q = 32
// (profiles/r02_rank_pmc.json): FETCH = 1.02x the corpus bytes but MFMA busy
// 44 %, 8.75 VALU per MFMA, and hipcc compiled its register ring into a
// vmcnt(0) per chunk plus 32 buffer copies per chunk.  Here:
//  * one wave per SIMD (4 per workgroup, one workgroup per CU), the 32
//    queries of the block held in registers as MFMA B operands for the whole
//    kernel (lane l: query l & 31, k = 32j + 16h + i: D / 2 VGPRs), so no LDS
//    query reads at all;
//  * the corpus streams through a per-wave LDS ring (NB slots of one 32-row x
//    32-k chunk, 4 KB) by buffer-descriptor DMA, PF chunks ahead, with counted
//    vmcnt waits and no barriers (each wave fills and reads only its own
//    slots).  The descriptor base is the 32-row tile's first row and its range
//    the tile's valid rows, so rows past the workgroup's range read zeros.
//    Image row r at r * 128 B, 16-byte slot s at s ^ ((r >> 1) & 7) (the
//    GEMM's conflict-free image; the DMA permutes its source pieces);
//  * the same arithmetic as rank_stream (k order within and across the
//    v_mfma_f32_32x32x2_f32 chain, the fmaf sum of squares, inv_norm, keys,
//    bitonic list update, tau threshold, workgroup list merge), so the
//    candidates are bit-identical.
// NOMFMA: timing probe (the stream and the fragment reads without the MFMAs; wrong scores)
// ILV (A/B, slower: see launch_reg): interleaved tile order.  Tile t of wave w
// in workgroup g is global 32-row tile (t * NW + w) * G + g, so the whole grid
// streams one contiguous band of NW * G tiles instead of G row ranges
// rows_per_wg apart.  Candidates then carry global rows.
// PIPE: a chunk's fragments are read from the ring one chunk ahead (two
// register buffers), so the LDS latency hides under the previous chunk's MFMAs
// instead of sitting between the wait and the MFMAs; the DMA lookahead is then
// PF - 1 chunks beyond the one being read.
// Dynamic LDS of rank_reg<.., NB, ..>: the ring [NW = 4][NB][4 KB], the per-wave
// row norms [4][32] f32, tau [RQ] u32 and the lead keys [RQ][8].  The launcher sizes the allocation
// with this same function: a kernel whose ring is larger than the allocation
// puts its norms (and the last wave's slots) past the end of the workgroup's
// LDS, where reads return zero — every score comes out 0.
constexpr size_t rank_reg_lds_bytes(int NB) { return (size_t)4 * NB * (32 * 128) + 4 * 32 * 4 + RQ * 4 + LEAD_LDS; }

// STAMP (A/B build, MICLIP_RANK_STAMP=1): s_memrealtime (100 MHz) per workgroup at entry, after the query
// load, after the stream, after fold_publish and at exit (mi_debug_rank_stamp)
__device__ unsigned long long g_rank_stamp[256 * 10];

template <int D, int NB = 8, int PF = 6, bool NOMFMA = false, bool ILV = false, bool PIPE = false, int DT = 0,
          bool STAMP = false, bool SPLITM = true>
__global__ __launch_bounds__(256) void rank_reg(const void* __restrict__ corpus, int64_t N,
                                                const float* __restrict__ queries, int64_t Q, int k,
                                                int64_t rows_per_wg, int norm_mode, int nan_first, int64_t index_base,
                                                FoldWs f, float* __restrict__ out_s, int64_t* __restrict__ out_i,
                                                const int32_t* __restrict__ gate) {
  // gate (nullable): per-query certificates of the certified pass (rank_cert.hip); a query
  // block whose queries are all certified already holds its results and exits here, before
  // any barrier or merge-counter update (uniformly over the block's workgroups).
  // DT 0: f32 rows, a ring chunk = 32 k; DT 1 / 2 (bf16 / fp16 rows): a ring chunk = 64 k, two
  // 32-k MFMA groups, converted to f32 (exactly) after the fragment read — the arithmetic of
  // rank_stream<DT> (load_chunk's conversion, the same k order), so its candidates bit for bit.
  constexpr int ES = DT ? 2 : 4, NG = DT ? 2 : 1, NCH = D / (32 * NG), NQ = D / 32;
  constexpr int NW = 4, NT = 64 * NW, KC = 16;
  // NB ring slots per wave, PF chunks in flight (NB >= PF + 1: a refilled slot was read, and its
  // reads waited for, in an earlier chunk iteration)
  constexpr int SLOT = 32 * 128;           // 4 KB
  // the invariants the ring's correctness rests on:
  //  * a slot is refilled (chunk c + PF into slot (c + PF) % NB, issued at the top of chunk c's
  //    iteration) only after the chunk it held, c + PF - NB, was read and its reads waited for
  //    (lgkmcnt(0) in that chunk's iteration): c + PF - NB <= c - 1;
  //  * the counted wait vmcnt(4 PF) (4 DMA instructions per chunk) fits the 6-bit vmcnt field;
  //  * the ring, norms and tau fit the CU's 160 KB of LDS (and the launcher allocates exactly
  //    rank_reg_lds_bytes(NB), which the list merge's 32 KB also fits in).
  static_assert(NB >= PF + 1, "rank_reg: a refilled ring slot must have been read in an earlier chunk");
  static_assert(4 * PF <= 63, "rank_reg: vmcnt(4 PF) exceeds the counter");
  static_assert(rank_reg_lds_bytes(NB) <= 160 * 1024, "rank_reg: ring exceeds the LDS");
  static_assert(rank_reg_lds_bytes(NB) >= (size_t)NT * KC * 8, "rank_reg: list merge area exceeds the allocation");
  static_assert(rank_reg_lds_bytes(NB) >= fold_lds(NT), "rank_reg: in-launch merge area exceeds the allocation");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;                       // [NW][NB][SLOT]
  float* nrm_all = (float*)(smem + NW * NB * SLOT);
  uint32_t* tau = (uint32_t*)(nrm_all + NW * 32);
  uint32_t* lead = tau + RQ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int64_t q0 = (int64_t)QB * RQ;
  const bool qvalid = q0 + r < Q;
  if (gate && __all(!qvalid || gate[q0 + r] != 0)) return;
  unsigned long long* stamp = g_rank_stamp + 10 * ((int)RB & 255);
  if (STAMP && tid == 0) stamp[0] = __builtin_amdgcn_s_memrealtime();

  // queries -> registers (zeros past Q)
  float qv[NQ][16];
  {
    const float* qp = queries + (qvalid ? (q0 + r) : 0) * D + 16 * h;
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
      for (int i4 = 0; i4 < 4; ++i4) {
        const float4 t = *(const float4*)(qp + 32 * j + 4 * i4);
        qv[j][4 * i4] = qvalid ? t.x : 0.f;
        qv[j][4 * i4 + 1] = qvalid ? t.y : 0.f;
        qv[j][4 * i4 + 2] = qvalid ? t.z : 0.f;
        qv[j][4 * i4 + 3] = qvalid ? t.w : 0.f;
      }
  }
  if (tid < RQ) tau[tid] = 0u;
  lead[tid] = 0u;   // 256 = 32 x 8
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (STAMP && tid == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();

  const int G = NRB;
  const int64_t r_begin = ILV ? 0 : (int64_t)RB * rows_per_wg;
  const int64_t r_end = ILV ? N : min(N, r_begin + rows_per_wg);
  const int nrows = (int)(r_end - r_begin);
  const int ntw = (nrows + 31) / 32;
  // ILV: tiles (t * NW + wave) * G + blockIdx.x < ntw
  const int sid = ILV ? wave * G + (int)RB : wave;
  const int sstep = ILV ? NW * G : NW;
  const int my_tiles = ntw > sid ? (ntw - 1 - sid) / sstep + 1 : 0;
  float* nrm = nrm_all + wave * 32;
  char* wring = ring + wave * NB * SLOT;

  // DMA: 4 x 1 KB per chunk; instruction m covers image rows 8m .. 8m + 7,
  // lane l row 8m + (l >> 3), LDS slot (l & 7), source piece (l & 7) ^ ((row >> 1) & 7)
  uint32_t voff[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int row = 8 * m + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    voff[m] = (uint32_t)(row * D * ES + c * 16);
  }
  int lt = 0, lj = 0, lslot = 0;           // load cursor: tile ordinal, chunk, ring slot
  __amdgpu_buffer_rsrc_t rs;
  auto make_rs = [&]() {
    const int trow = (sid + sstep * lt) * 32;   // relative to r_begin
    const int rows = max(0, min(32, nrows - trow));
    // wave-uniform by construction; readfirstlane makes it provable (no waterfall loop per load, guide T20)
    const uint64_t base = (uint64_t)(uintptr_t)((const char*)corpus + (r_begin + (rows ? trow : 0)) * (int64_t)D * ES);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const int nrec = __builtin_amdgcn_readfirstlane(rows * D * ES);
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0, nrec, 0x00020000);
  };
  make_rs();
  auto issue = [&]() {   // chunk (lt, lj) -> slot lslot; past this wave's tiles: range 0, zeros
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
  // fragment read: row r, f32: k 16h .. 16h + 15 = slots 4h .. 4h + 3; 16-bit: k 32g + 16h .. + 15 =
  // slots 4g + 2h, 4g + 2h + 1 for g = 0, 1 (permuted)
  const int rbase = r * 128;
  const int sw = (r >> 1) & 7;
  uint64_t L[KC];
#pragma unroll
  for (int p = 0; p < KC; ++p) L[p] = 0ull;
  uint32_t kk = 0u;   // running k-th key of this query's lists (own threshold)

  auto read_frag = [&](int slot, float4 (&v)[4]) {
    const char* src = wring + slot * SLOT + rbase;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      const int sl = DT ? (i4 >> 1) * 4 + 2 * h + (i4 & 1) : 4 * h + i4;
      const uint32_t a = (uint32_t)(uintptr_t)(const LDS_AS char*)(src + ((sl ^ sw) << 4));
      asm volatile("ds_read_b128 %0, %1" : "=v"(v[i4]) : "v"(a) : "memory");
    }
  };
  if (my_tiles > 0) {
#pragma unroll
    for (int p = 0; p < PF; ++p) issue();
    int cslot = 0;
    float4 vb[2][4];
    if (PIPE) {   // chunk 0's fragments
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (PF - 1)) : "memory");
      read_frag(0, vb[0]);
      cslot = 1;
    }
    for (int ct = 0; ct < my_tiles; ++ct) {
      f32x16 acc = f32x16{};
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        issue();   // chunk PF ahead (the ring slot it fills was read NB - PF chunks ago)
        float4 (&v)[4] = vb[PIPE ? (j & 1) : 0];
        if (PIPE) {
          // the next chunk landed (PF - 1 younger); this chunk's fragments (read one chunk ago) are in v
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(4 * (PF - 1)) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          read_frag(cslot, vb[(j + 1) & 1]);   // (past the last tile: a zero-range chunk, never used)
          __builtin_amdgcn_sched_barrier(0);
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PF) : "memory");   // this chunk landed
          read_frag(cslot, v);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          float cur[16];
          if (DT == 0) {
            const float c0[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                                  v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
#pragma unroll
            for (int i = 0; i < 16; ++i) cur[i] = c0[i];
          } else {
            const float4 a = v[2 * g], b = v[2 * g + 1];
            const uint32_t w[8] = {__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(a.z), __float_as_uint(a.w),
                                   __float_as_uint(b.x), __float_as_uint(b.y), __float_as_uint(b.z), __float_as_uint(b.w)};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              if (DT == 1) {
                cur[2 * e] = __uint_as_float(w[e] << 16);
                cur[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
              } else {
                union { uint32_t u; _Float16 hh[2]; } cv;
                cv.u = w[e];
                cur[2 * e] = (float)cv.hh[0];
                cur[2 * e + 1] = (float)cv.hh[1];
              }
            }
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            if (NOMFMA) asm volatile("" ::"v"(cur[i]), "v"(qv[j * NG + g][i]));
            else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[i], qv[j * NG + g][i], acc, 0, 0, 0);
            ss = fmaf(cur[i], cur[i], ss);
          }
        }
        cslot = cslot == NB - 1 ? 0 : cslot + 1;
      }
      // ---- tile finished: scores, threshold test, list update (rank_stream's finalize)
      ss += __shfl_xor(ss, 32, 64);
      if (h == 0) nrm[r] = inv_norm(ss, norm_mode);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int tr0 = (sid + sstep * ct) * 32;
      const uint32_t tq_thr = tau[r];
      const uint32_t own = kk;   // the query's two half-lists' k-th: a lower bound of its k-th
      const uint32_t thr0 = own > tq_thr ? own : tq_thr;
      const uint32_t lb = lead_min(lead, r);
      const uint32_t thr = lb > thr0 ? lb : thr0;
      uint64_t c[16];
      bool any = false;
      uint32_t okm = 0u;
      // the 16 rows' reciprocals: rows (rg & 3) + 8 (rg >> 2) + 4 h are four 16-byte runs
      f32x4 nv[4];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) nv[q4] = *(const f32x4*)(nrm + 8 * q4 + 4 * h);
#pragma unroll
      for (int rg = 0; rg < 16; ++rg) {
        const int rr = (rg & 3) + 8 * (rg >> 2) + 4 * h;
        const int lr = tr0 + rr;
        const float sc = norm_mode == 2 ? acc[rg] : acc[rg] * nv[rg >> 2][rg & 3];
        const uint32_t key = score_key(sc, nan_first);
        const bool ok = qvalid && lr < nrows && key >= thr;
        c[rg] = ok ? (((uint64_t)key << 32) | (uint32_t)~(uint32_t)lr) : 0ull;
        any |= ok;
        okm |= ok ? 1u << rg : 0u;
      }
      if (__any(any)) {
        list_update16(L, c, okm);
        lead_publish(lead, r, 2 * wave + h, (uint32_t)(L[1] >> 32));
        uint32_t kth = (uint32_t)(L[0] >> 32);
#pragma unroll
        for (int p = 1; p < KC; ++p) kth = (p == k - 1) ? (uint32_t)(L[p] >> 32) : kth;
        const uint32_t other = (uint32_t)__shfl_xor((int)kth, 32, 64);
        kth = kth > other ? kth : other;
        kk = kth;
        if (h == 0 && qvalid && kth > tq_thr) tau_max(&tau[r], kth);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  // trailing (zero-range) DMAs and the pipelined read past the last chunk complete before the ring is reused
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (SPLITM) {   // split merge: the lists raw, then fold_merge_kernel (rank_keys.hpp)
    lines_publish<NW>(L, smem, wave, lane, q0, Q, k, r_begin, f);
    return;
  }
  __syncthreads();   // ring free -> lists
  if (STAMP && tid == 0) stamp[2] = __builtin_amdgcn_s_memrealtime();
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
  if (STAMP && tid == 0) stamp[3] = __builtin_amdgcn_s_memrealtime();
  fold_reduce<NT>(smem, f, q0, Q, k, nan_first, index_base, out_s, out_i, STAMP ? stamp : nullptr);
  if (STAMP && tid == 0) stamp[4] = __builtin_amdgcn_s_memrealtime();
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
  const int64_t q0 = (int64_t)QB * RQ;

  for (int64_t e = tid; e < RQ * D; e += 256) {
    const int qq = (int)(e / D);
    const int64_t d = e % D;
    Ts[qq * ts_stride + d] = (q0 + qq < Q) ? queries[(q0 + qq) * D + d] : 0.f;
  }
  __syncthreads();

  const int64_t r_begin = (int64_t)RB * rows_per_wg;
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
    float* os = ws_s + (q0 + tid) * C + (int64_t)RB * k;
    int64_t* oi = ws_i + (q0 + tid) * C + (int64_t)RB * k;
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

// The split merge's second launch (rank_keys.hpp lines_publish): one workgroup per query
// reduces the pass's nlines slab lines (one per pass workgroup: its top-k, sorted desc), thread
// w loading line w whole.  A cut first: the k-th largest PACKED entry (key, ~index) among a wave's
// 64 line heads (k distinct rows rank at least that high, so the query's k-th does too), the
// largest such over the waves and gtau (the largest workgroup k-th key); sorting the heads across
// the lanes is a 21-step bitonic network of 64-bit (two 32-bit) shuffles.  Each line's prefix at
// or above the cut is appended to LDS, and thread j ranks appended entry j by counting the entries
// that beat it (packed entries are unique: index asc breaks ties) -- the in-launch reducer's rule,
// so results are bit-identical.  gtau alone kept ~800 of 2450 entries at 125k rows (a 117-us
// count).  The cut is on the packed entry, not its 32-bit key alone: under mass ties
// (duplicate or static frames: every line's prefix ties the cut key) a key cut kept all nlines x k
// entries and the quadratic count took milliseconds; the packed cut keeps the ~k lines whose heads
// beat the k-th head, ~k^2 entries.
// gate (nullable): a query block whose queries are all certified holds its results (the
// gated exact pass skipped it), so its queries are skipped here too.
template <int NT>
__global__ __launch_bounds__(NT) void fold_merge_kernel(const uint64_t* __restrict__ lines, const uint32_t* __restrict__ gtau,
                                                        int64_t Qpad, int nlines, int64_t Q, int k, int nan_first,
                                                        int64_t index_base, float* __restrict__ out_s,
                                                        int64_t* __restrict__ out_i, const int32_t* __restrict__ gate) {
  extern __shared__ __attribute__((aligned(16))) char fm_lds[];   // cnt, cut, then nlines x k entries
  uint32_t& cnt = *(uint32_t*)fm_lds;
  unsigned long long& cut64 = *((unsigned long long*)fm_lds + 1);
  uint64_t* buf = (uint64_t*)(fm_lds + 16);
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t q = blockIdx.x;
  if (gate) {   // the same 32 reads in every wave: a uniform exit
    const int64_t qq = q / FQ * FQ + (lane & 31);
    if (__all(qq >= Q || gate[qq] != 0)) return;
  }
  if (tid == 0) {
    cnt = 0u;
    cut64 = (unsigned long long)gtau[q] << 32;   // every entry below has a key below gtau
  }
  const int nld = (k + 1) >> 1;   // 16-byte pieces of a line holding k entries
  typedef unsigned int u32x4m __attribute__((ext_vector_type(4)));
  uint64_t e[16];
  {
    const int w = tid < nlines ? tid : 0;   // (nlines <= NT: one line per thread)
    const u32x4m* lp = (const u32x4m*)(lines + ((int64_t)w * Qpad + q) * 16);
    u32x4m pc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) pc[c] = (c < nld && tid < nlines) ? lp[c] : (u32x4m){0u, 0u, 0u, 0u};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      e[2 * c] = ((uint64_t)pc[c][1] << 32) | pc[c][0];
      e[2 * c + 1] = ((uint64_t)pc[c][3] << 32) | pc[c][2];
    }
  }
  // the wave's line heads sorted descending across the lanes (an empty head -- and a missing line --
  // sorts as 0; a real entry with key 0 is a NaN-last row, whose head then only makes the cut 0: none)
  uint64_t hk = e[0];
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint32_t olo = (uint32_t)__shfl_xor((int)(uint32_t)hk, stride, 64);
      const uint32_t ohi = (uint32_t)__shfl_xor((int)(uint32_t)(hk >> 32), stride, 64);
      const uint64_t o = ((uint64_t)ohi << 32) | olo;
      const bool lower = (lane & stride) == 0;        // this lane holds the pair's first position
      const bool desc = (lane & size) == 0 || size == 64;
      const uint64_t mx = hk > o ? hk : o, mn = hk > o ? o : hk;
      hk = (lower == desc) ? mx : mn;
    }
  const uint32_t klo = (uint32_t)__shfl((int)(uint32_t)hk, k - 1, 64);
  const uint32_t khi = (uint32_t)__shfl((int)(uint32_t)(hk >> 32), k - 1, 64);
  const uint64_t kth_head = ((uint64_t)khi << 32) | klo;
  __syncthreads();   // cnt / cut64 initialised
  if (lane == 0 && kth_head) atomicMax(&cut64, (unsigned long long)kth_head);
  __syncthreads();
  const uint64_t cut = cut64;
  int m = 0;   // the line's prefix at or above the cut (sorted desc, zeros after)
#pragma unroll
  for (int p = 0; p < 16; ++p) m += (p < k && e[p] != 0ull && e[p] >= cut) ? 1 : 0;
  if (m) {
    const uint32_t at = atomicAdd(&cnt, (uint32_t)m);
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (p < m) buf[at + p] = e[p];
  }
  __syncthreads();
  const int n = (int)cnt;
  for (int j = tid; j < n; j += NT) {
    const uint64_t x = buf[j];
    int rk = 0;
    for (int i = 0; i < n; ++i) rk += buf[i] > x ? 1 : 0;
    if (rk < k) {
      out_s[q * k + rk] = decode_key((uint32_t)(x >> 32), nan_first);
      out_i[q * k + rk] = index_base + (int64_t)(uint32_t)~(uint32_t)x;
    }
  }
  for (int r = n + tid; r < k; r += NT) {   // fewer than k rows in all
    out_s[q * k + r] = -INFINITY;
    out_i[q * k + r] = -1;
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

// ---------------------------------------------------------------------------
// Large k (k > 64: the register top-k lists stop there).  The reference's
// np.argsort(s)[::-1][:top_k] with top_k = 3 x the UI request (query_strategies.py:55)
// exceeds 64 from a request of 22 results on; top_k >= N is a full sort
// (embedding_service.py:317-318).  Path: the exact-f32 score matrix
// (score_matrix_kernel, the same score_tile arithmetic as rank_stage1), then
// per query
//   select_kernel   radix select of the k-th best key (4 passes of 8-bit
//                   digit histograms over the row's keys), then a compaction of
//                   every key above it plus the lowest-index ties equal to it
//                   (waves own contiguous index ranges, so ballot prefixes
//                   number the ties in index order) -> k candidates;
//   sort_chunks     bitonic sort of chunks of <= SORT_CHUNK candidates in LDS
//                   by (key desc, index asc);
//   merge_pass      merge-path merges of sorted runs (k > SORT_CHUNK);
//   finalize        decode keys -> scores, global indices.
constexpr int SEL_NT = 1024;
constexpr int SORT_CHUNK = 8192;
constexpr int MERGE_ITEMS = 16;

__global__ __launch_bounds__(SEL_NT) void select_kernel(const float* __restrict__ S, int64_t N, int k, int nan_first,
                                                        uint32_t* __restrict__ ck, int32_t* __restrict__ ci,
                                                        int64_t kp) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t sh[4];          // prefix, krem, gt counter
  __shared__ uint32_t wcnt[SEL_NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t q = blockIdx.x;
  const float* s = S + q * N;
  uint32_t* okey = ck + q * kp;
  int32_t* oidx = ci + q * kp;
  uint32_t prefix = 0, mask = 0, krem = (uint32_t)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += SEL_NT) hist[i] = 0;
    __syncthreads();
    for (int64_t i = tid; i < N; i += SEL_NT) {
      const uint32_t key = score_key(s[i], nan_first);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= krem) break;
        acc += hist[d];
      }
      sh[0] = prefix | ((uint32_t)d << shift);
      sh[1] = krem - acc;
    }
    __syncthreads();
    prefix = sh[0];
    krem = sh[1];
    mask |= 255u << shift;
    __syncthreads();
  }
  // prefix = T, the k-th best key; k - krem keys are above it, krem ties at T
  // are taken in index order.  Wave w owns indices [w*per, (w+1)*per).
  const uint32_t T = prefix, n_gt = (uint32_t)k - krem;
  const int64_t per = ((N + SEL_NT / 64 - 1) / (SEL_NT / 64) + 63) / 64 * 64;
  const int64_t b0 = wave * per, b1 = min(N, b0 + per);
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t neq = 0;
  for (int64_t i = b0; i < b1; i += 64) {
    const bool eq = i + lane < b1 && score_key(s[i + lane], nan_first) == T;
    neq += (uint32_t)__popcll(__ballot(eq));
  }
  if (lane == 0) wcnt[wave] = neq;
  if (tid == 0) sh[2] = 0;
  __syncthreads();
  uint32_t run = 0;
  for (int w = 0; w < wave; ++w) run += wcnt[w];
  for (int64_t i = b0; i < b1; i += 64) {
    const bool valid = i + lane < b1;
    const uint32_t key = valid ? score_key(s[i + lane], nan_first) : 0u;
    const bool gt = valid && key > T, eq = valid && key == T;
    const uint64_t bg = __ballot(gt), be = __ballot(eq);
    if (bg) {
      const int lead = __ffsll((unsigned long long)bg) - 1;
      uint32_t base = 0;
      if (lane == lead) base = atomicAdd(&sh[2], (uint32_t)__popcll(bg));
      base = __shfl(base, lead, 64);
      if (gt) {
        const uint32_t p = base + (uint32_t)__popcll(bg & lt);
        okey[p] = key;
        oidx[p] = (int32_t)(i + lane);
      }
    }
    if (eq) {
      const uint32_t r = run + (uint32_t)__popcll(be & lt);
      if (r < krem) {
        okey[n_gt + r] = key;
        oidx[n_gt + r] = (int32_t)(i + lane);
      }
    }
    run += (uint32_t)__popcll(be);
  }
  for (int64_t p = k + tid; p < kp; p += SEL_NT) {  // padding sorts after every real candidate
    okey[p] = 0u;
    oidx[p] = INT_MAX;
  }
}

// Bitonic sort of one chunk of `n` (power of two, <= SORT_CHUNK) candidates in
// LDS into "best first" order.
__global__ __launch_bounds__(1024) void sort_chunks_kernel(uint32_t* __restrict__ ck, int32_t* __restrict__ ci,
                                                           int64_t kp, int n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* K = (uint32_t*)smem;
  int32_t* I = (int32_t*)(smem + SORT_CHUNK * 4);
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.y * kp + (int64_t)blockIdx.x * n;
  for (int i = tid; i < n; i += 1024) {
    K[i] = ck[base + i];
    I[i] = ci[base + i];
  }
  __syncthreads();
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < n / 2; t += 1024) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;
        const bool up = (i & size) == 0;
        const uint32_t ki = K[i], kj = K[j];
        const int32_t ii = I[i], ij = I[j];
        if (up ? better(kj, ij, ki, ii) : better(ki, ii, kj, ij)) {
          K[i] = kj; K[j] = ki;
          I[i] = ij; I[j] = ii;
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < n; i += 1024) {
    ck[base + i] = K[i];
    ci[base + i] = I[i];
  }
}

// One merge-path pass: sorted runs of `run` elements -> runs of 2*run.
__global__ __launch_bounds__(256) void merge_pass_kernel(const uint32_t* __restrict__ sk, const int32_t* __restrict__ si,
                                                         uint32_t* __restrict__ dk, int32_t* __restrict__ di,
                                                         int64_t kp, int64_t run) {
  const int64_t o0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * MERGE_ITEMS;
  if (o0 >= kp) return;
  const int64_t qb = (int64_t)blockIdx.y * kp;
  const int64_t a0 = o0 / (2 * run) * (2 * run);
  const int64_t la = min(run, kp - a0);
  const int64_t b0 = a0 + la;
  const int64_t lb = max((int64_t)0, min(run, kp - b0));
  const int64_t d = o0 - a0;
  const uint32_t* AK = sk + qb + a0;
  const int32_t* AI = si + qb + a0;
  const uint32_t* BK = sk + qb + b0;
  const int32_t* BI = si + qb + b0;
  int64_t lo = max((int64_t)0, d - lb), hi = min(d, la);
  while (lo < hi) {  // i = number of the first d outputs taken from A (A first on equal elements)
    const int64_t mid = (lo + hi) >> 1;
    if (!better(BK[d - 1 - mid], BI[d - 1 - mid], AK[mid], AI[mid])) lo = mid + 1;
    else hi = mid;
  }
  int64_t ia = lo, ib = d - lo;
  for (int t = 0; t < MERGE_ITEMS && o0 + t < kp; ++t) {
    const bool takeA = ib >= lb || (ia < la && !better(BK[ib], BI[ib], AK[ia], AI[ia]));
    dk[qb + o0 + t] = takeA ? AK[ia] : BK[ib];
    di[qb + o0 + t] = takeA ? AI[ia] : BI[ib];
    ia += takeA ? 1 : 0;
    ib += takeA ? 0 : 1;
  }
}

__global__ __launch_bounds__(256) void finalize_large_kernel(const uint32_t* __restrict__ ck,
                                                             const int32_t* __restrict__ ci, int64_t kp, int k, int kk,
                                                             int nan_first, int64_t base, float* __restrict__ out_s,
                                                             int64_t* __restrict__ out_i) {
  const int64_t q = blockIdx.y;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < k; o += gridDim.x * 256) {
    if (o < kk) {
      out_s[q * k + o] = decode_key(ck[q * kp + o], nan_first);
      out_i[q * k + o] = base + ci[q * kp + o];
    } else {
      out_s[q * k + o] = -INFINITY;
      out_i[q * k + o] = -1;
    }
  }
}

}  // namespace

// ------------------------------------------------------------ host helpers
static int kc_for(int k) { return k <= 16 ? 16 : 64; }

static int64_t large_kp(int64_t kk) {  // padded candidate count per query
  if (kk <= SORT_CHUNK) {
    int64_t p = 2;
    while (p < kk) p <<= 1;
    return p;
  }
  return (kk + SORT_CHUNK - 1) / SORT_CHUNK * SORT_CHUNK;
}

static size_t large_ws_bytes(int64_t N, int64_t Q, int k) {
  const int64_t kk = k < N ? k : N;
  const size_t sbytes = ((size_t)(Q * N) * 4 + 255) / 256 * 256;
  return sbytes + (size_t)(2 * Q * large_kp(kk)) * 8;
}

hipError_t rank_fill_empty(int64_t Q, int k, float* out_s, int64_t* out_i, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  const unsigned fb = (unsigned)((k + 255) / 256 < 64 ? (k + 255) / 256 : 64);
  hipLaunchKernelGGL(finalize_large_kernel, dim3(fb, (unsigned)Q), dim3(256), 0, s, nullptr, nullptr, (int64_t)0, k,
                     0, 0, (int64_t)0, out_s, out_i);
  return hipGetLastError();
}

static hipError_t rank_topk_large(const void* corpus, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int k,
                                  int64_t base, int norm_mode, int nan_first, float* out_s, int64_t* out_i, void* ws,
                                  hipStream_t s) {
  const int kk = (int)(k < N ? k : N);
  const int64_t kp = large_kp(kk);
  float* S = (float*)ws;
  char* p = (char*)ws + ((size_t)(Q * N) * 4 + 255) / 256 * 256;
  uint32_t* k0 = (uint32_t*)p;
  int32_t* i0 = (int32_t*)(p + (size_t)(Q * kp) * 4);
  uint32_t* k1 = (uint32_t*)(p + (size_t)(Q * kp) * 8);
  int32_t* i1 = (int32_t*)(p + (size_t)(Q * kp) * 12);
  hipError_t e = score_matrix(corpus, N, D, dt, q, Q, norm_mode, S, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(select_kernel, dim3((unsigned)Q), dim3(SEL_NT), 0, s, S, N, kk, nan_first, k0, i0, kp);
  const int chunk = (int)(kp < SORT_CHUNK ? kp : SORT_CHUNK);
  const size_t lds = (size_t)SORT_CHUNK * 8;
  e = hipFuncSetAttribute((const void*)sort_chunks_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sort_chunks_kernel, dim3((unsigned)(kp / chunk), (unsigned)Q), dim3(1024), lds, s, k0, i0, kp,
                     chunk);
  for (int64_t run = chunk; run < kp; run *= 2) {
    const unsigned nb = (unsigned)((kp + 256 * MERGE_ITEMS - 1) / (256 * MERGE_ITEMS));
    hipLaunchKernelGGL(merge_pass_kernel, dim3(nb, (unsigned)Q), dim3(256), 0, s, k0, i0, k1, i1, kp, run);
    uint32_t* tk = k0; k0 = k1; k1 = tk;
    int32_t* ti = i0; i0 = i1; i1 = ti;
  }
  const unsigned fb = (unsigned)((k + 255) / 256 < 64 ? (k + 255) / 256 : 64);
  hipLaunchKernelGGL(finalize_large_kernel, dim3(fb, (unsigned)Q), dim3(256), 0, s, k0, i0, kp, k, kk, nan_first,
                     base, out_s, out_i);
  return hipGetLastError();
}

int64_t rank_chunks(int64_t N) {
  // one workgroup per CU-slot pair (512) once the corpus is large, so each
  // wave streams several 32-row tiles; rows per workgroup are multiples of 384
  // (one tile round of 12 waves)
  const int64_t tiles = (N + 383) / 384;
  return tiles < 512 ? tiles : 512;
}

size_t rank_workspace_bytes(int64_t N, int64_t Q, int k) {
  if (k > RANK_REG_K) return large_ws_bytes(N, Q, k);
  const int64_t nch = N > 0 ? rank_chunks(N) : 1;
  const size_t lists = (size_t)(Q * nch * k) * (sizeof(float) + sizeof(int64_t));   // rank_stage1 + rank_merge
  const size_t fold = kc_for(k) == 16 ? fold_ws_bytes(nch, Q) : 0;                   // in-launch merge (k <= 16)
  const size_t exact = lists > fold ? lists : fold;
  // the certified pass (rank_cert.hip) ahead of the gated exact pass: its own area first
  const bool cert = k <= 12 && N >= rank_cert_min_rows();
  return cert ? al128(rank_cert_ws_bytes(N, Q)) + exact : exact;
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
  // (64 / 128 threads per query measured slower at C = 2560-4096, Q = 1-1000)
  if (kc_for(k) == 16)
    hipLaunchKernelGGL((rank_merge_kernel<16, 256>), dim3((unsigned)Q), dim3(256), 0, s, cs, ci, C, k, nan_first,
                       out_s, out_i);
  else
    hipLaunchKernelGGL((rank_merge_kernel<64, 64>), dim3((unsigned)Q), dim3(64), 0, s, cs, ci, C, k, nan_first,
                       out_s, out_i);
  return hipGetLastError();
}

namespace rankk {
hipError_t fold_merge(const FoldWs& f, int64_t nwg, int64_t Q, int k, int nan_first, int64_t index_base, float* out_s,
                      int64_t* out_i, const int32_t* gate, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  // one slab line per thread: 256 threads (rank_reg / rank_cert / the mirror: <= 256 workgroups)
  // or 512 (rank_stream: up to 512)
  if (nwg > 512) return hipErrorInvalidValue;
  const size_t lds = 16 + (size_t)nwg * k * 8;
  if (nwg <= 256) {
    hipLaunchKernelGGL((fold_merge_kernel<256>), dim3((unsigned)Q), dim3(256), lds, s, f.slab, f.gtau, f.Qpad, (int)nwg,
                       Q, k, nan_first, index_base, out_s, out_i, gate);
  } else {
    static bool attr = false;   // > 64 KB of LDS at nwg = 512, k = 16
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)fold_merge_kernel<512>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 16 + 512 * 16 * 8);
      if (e != hipSuccess) return e;
      attr = true;
    }
    hipLaunchKernelGGL((fold_merge_kernel<512>), dim3((unsigned)Q), dim3(512), lds, s, f.slab, f.gtau, f.Qpad, (int)nwg,
                       Q, k, nan_first, index_base, out_s, out_i, gate);
  }
  return hipGetLastError();
}
}  // namespace rankk

// rank_reg's workgroups: one per CU (LDS ring 128 KB), rows per workgroup a multiple of 128
// (one 32-row tile per wave); never more workgroups than rank_chunks (workspace)
static int64_t reg_rows_per_wg(int64_t N) {
  int64_t nwg = rank_chunks(N);
  if (nwg > 256) nwg = 256;
  if (nwg > (N + 127) / 128) nwg = (N + 127) / 128;
  return ((N + nwg - 1) / nwg + 127) / 128 * 128;
}

static FoldWs reg_fold(int64_t N, int64_t Q, void* ws) {
  const int64_t rpw = reg_rows_per_wg(N);
  return fold_ws(ws, (N + rpw - 1) / rpw, Q);
}

// prezeroed: the merge counters were cleared by the kernel before (the certified route's re-score)
template <int D, int DT>
static hipError_t launch_reg(int64_t N, const void* corpus, const float* q, int64_t Q, int k, int nm, int nf,
                             int64_t base, void* ws, float* out_s, int64_t* out_i, hipStream_t s,
                             const int32_t* gate = nullptr, bool prezeroed = false) {
  const int64_t rpw = reg_rows_per_wg(N);
  const int64_t nwg = (N + rpw - 1) / rpw;
  const FoldWs f = fold_ws(ws, nwg, Q);
  // interleaved tile order: A/B only (MICLIP_RANK_ILV=1).  scripts/rank_micro.py: 1M x 512 494 us
  // against 479 with contiguous row ranges, 1M x 768 729 against 717: not the stream's limit
#if MICLIP_AB
  const char* ilv = getenv("MICLIP_RANK_ILV");
  const bool il = ilv && ilv[0] == '1';
  // ring slots: MICLIP_RANK_NB=9 selects a 9-slot ring with 7 chunks in flight (A/B; round 2's
  // 9-slot attempt kept this allocation at 8 slots' size, so its norms sat past the end of the
  // LDS and read as zeros: every test failed, N = 1 included).  The size now follows NB.
  const char* nbs = getenv("MICLIP_RANK_NB");
  const bool nb9 = nbs && atoi(nbs) == 9;
  const size_t lds = rank_reg_lds_bytes(nb9 ? 9 : 8);
  const char* probe = getenv("MICLIP_RANK_PROBE");
  // (7 chunks in flight measured the same: the stream alone, NOMFMA, reads 5.3 TB/s either way)
  // fragment reads one chunk ahead: A/B only (MICLIP_RANK_PIPE=1; 1M x 512 552 us against 558,
  // within noise: the wait before the MFMAs is not where this kernel loses time)
  const char* pipe = getenv("MICLIP_RANK_PIPE");
  const bool pp = pipe && pipe[0] == '1';
  const char* stp = getenv("MICLIP_RANK_STAMP");
  // in-launch merge (the round-4 tail) instead of the split merge: A/B (MICLIP_RANK_FOLD=1)
  const char* fold = getenv("MICLIP_RANK_FOLD");
  const bool inl = fold && fold[0] == '1';
  auto fn = (stp && stp[0] == '1') ? rank_reg<D, 8, 6, false, false, false, DT, true, false>
            : inl ? rank_reg<D, 8, 6, false, false, false, DT, false, false>
            : nb9 ? rank_reg<D, 9, 7, false, false, false, DT>
            : (probe && probe[0] == '1') ? (il ? rank_reg<D, 8, 6, true, true, false, DT> : rank_reg<D, 8, 6, true, false, false, DT>)
            : il ? (pp ? rank_reg<D, 8, 6, false, true, true, DT> : rank_reg<D, 8, 6, false, true, false, DT>)
                 : (pp ? rank_reg<D, 8, 6, false, false, true, DT> : rank_reg<D, 8, 6, false, false, false, DT>);
#else   // product: the measured default (8 slots, 6 chunks in flight, contiguous row ranges)
  const size_t lds = rank_reg_lds_bytes(8);
  auto fn = rank_reg<D, 8, 6, false, false, false, DT>;
  constexpr bool inl = false;
#endif
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (!prezeroed && (e = fold_zero(f, s)) != hipSuccess) return e;
  const dim3 grid((unsigned)((Q + RQ - 1) / RQ), (unsigned)nwg);   // (query blocks, row blocks): RB / QB
  hipLaunchKernelGGL(fn, grid, dim3(256), lds, s, corpus, N, q, Q, k, rpw, nm, nf, base, f, out_s, out_i, gate);
  if ((e = hipGetLastError()) != hipSuccess) return e;
#if MICLIP_AB
  if (inl || (stp && stp[0] == '1')) return hipSuccess;
#endif
  return inl ? hipSuccess : fold_merge(f, nwg, Q, k, nf, base, out_s, out_i, gate, s);
}

template <int DT, int NW>
static hipError_t launch_stream(dim3 grid, size_t lds, hipStream_t s, const void* corpus, int64_t N, int64_t D,
                                const float* q, int64_t Q, int k, int64_t rpw, int nm, int nf, int64_t base,
                                void* ws, float* out_s, int64_t* out_i) {
  bool inl = false;   // the in-launch merge (A/B: MICLIP_RANK_FOLD=1)
#if MICLIP_AB
  const char* fold = getenv("MICLIP_RANK_FOLD");
  inl = fold && fold[0] == '1';
#endif
  auto fn = inl ? rank_stream<DT, NW, false> : rank_stream<DT, NW, true>;
  const size_t l = lds > fold_lds(64 * NW) ? lds : fold_lds(64 * NW);
  hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l);
  if (e != hipSuccess) return e;
  const FoldWs f = fold_ws(ws, grid.y, Q);
  if ((e = fold_zero(f, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(fn, grid, dim3(64 * NW), l, s, corpus, N, D, q, Q, k, rpw, nm, nf, base, f, out_s, out_i);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return inl ? hipSuccess : fold_merge(f, grid.y, Q, k, nf, base, out_s, out_i, nullptr, s);
}

hipError_t rank_topk(const void* corpus, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int k,
                     int64_t base, int norm_mode, int nan_first, float* out_s, int64_t* out_i, void* ws,
                     hipStream_t s) {
  if (k > RANK_REG_K) return rank_topk_large(corpus, N, D, dt, q, Q, k, base, norm_mode, nan_first, out_s, out_i, ws, s);
  const int64_t nch = rank_chunks(N);
  const int64_t rpw = ((N + nch - 1) / nch + 383) / 384 * 384;
  const int64_t nwg = (N + rpw - 1) / rpw;
  const int64_t C = nwg * k;
  float* ws_s = (float*)ws;
  int64_t* ws_i = (int64_t*)((char*)ws + (size_t)(Q * nch * k) * sizeof(float));
  const dim3 grid((unsigned)((Q + RQ - 1) / RQ), (unsigned)nwg);   // (query blocks, row blocks): RB / QB
  const int KC = kc_for(k);
  // streaming kernel for k <= 16 (KC = 16 lists stay in registers); 8 or 12
  // waves per workgroup (MICLIP_RANK_NW A/B), one workgroup per CU either way
  // (~150 VGPRs, LDS = the list area).  KC = 64 keeps rank_stage1 (its 64-deep
  // lists would go to scratch in the streaming kernel).
#if MICLIP_AB
  const char* nwenv = getenv("MICLIP_RANK_NW");
  const int NW = nwenv && atoi(nwenv) == 8 ? 8 : 12;
  const char* legacy = getenv("MICLIP_RANK_STAGE1");   // A/B: the previous one-tile-at-a-time kernel
  const char* noreg = getenv("MICLIP_RANK_REG");        // A/B: 0 = rank_stream for f32 D = 512 too
#else
  constexpr int NW = 12;
  const char* legacy = nullptr;
  const char* noreg = nullptr;
#endif
  const size_t qa = (size_t)RQ * (D + 4) * 4 + (size_t)NW * 32 * 4 + RQ * 4;
  const size_t la = (size_t)64 * NW * KC * 8;
  const size_t lds = qa > la ? qa : la;
  hipError_t e;
  if (KC == 16 && D == 512 && !(legacy && legacy[0] == '1') && !(noreg && noreg[0] == '0')) {
    if (rank_cert_eligible(N, D, dt, k, norm_mode)) {
      // certified bf16-MFMA pass + exact re-score of its candidates, then the exact pass for
      // the query blocks it could not certify (results identical to the exact pass alone)
      int32_t* cert = nullptr;
      void* ws2 = (char*)ws + al128(rank_cert_ws_bytes(N, Q));
      const FoldWs f2 = reg_fold(N, Q, ws2);   // the gated exact pass's counters: the re-score clears them
      hipError_t ec = rank_cert_topk(corpus, N, dt, q, Q, k, base, norm_mode, nan_first, out_s, out_i, ws, &cert, s,
                                     fold_zero_base(f2), fold_zero_words(f2));
      if (ec != hipSuccess) return ec;
      return dt == 0 ? launch_reg<512, 0>(N, corpus, q, Q, k, norm_mode, nan_first, base, ws2, out_s, out_i, s, cert, true)
                     : launch_reg<512, 1>(N, corpus, q, Q, k, norm_mode, nan_first, base, ws2, out_s, out_i, s, cert, true);
    }
    // (D = 768 would hold 384 query VGPRs: hipcc spills ~230, so it keeps rank_stream)
    return dt == 0   ? launch_reg<512, 0>(N, corpus, q, Q, k, norm_mode, nan_first, base, ws, out_s, out_i, s)
           : dt == 1 ? launch_reg<512, 1>(N, corpus, q, Q, k, norm_mode, nan_first, base, ws, out_s, out_i, s)
                     : launch_reg<512, 2>(N, corpus, q, Q, k, norm_mode, nan_first, base, ws, out_s, out_i, s);
  }
  if (KC == 64 || (legacy && legacy[0] == '1')) {
#define MI_S1(KCV, DTV) \
  launch_stage1<KCV, DTV>(grid, stage1_lds(D, KCV), s, corpus, N, D, q, Q, k, rpw, norm_mode, nan_first, base, ws_s, \
                          ws_i, C)
    if (KC == 16) e = dt == 0 ? MI_S1(16, 0) : dt == 1 ? MI_S1(16, 1) : MI_S1(16, 2);
    else e = dt == 0 ? MI_S1(64, 0) : dt == 1 ? MI_S1(64, 1) : MI_S1(64, 2);
#undef MI_S1
    if (e != hipSuccess) return e;
    return rank_merge(ws_s, ws_i, Q, C, k, nan_first, out_s, out_i, s);
  }
  // k <= 16: rank_stream with the in-launch merge
#define MI_RS(DTV, NWV) \
  launch_stream<DTV, NWV>(grid, lds, s, corpus, N, D, q, Q, k, rpw, norm_mode, nan_first, base, ws, out_s, out_i)
#if MICLIP_AB
  if (NW == 8) return dt == 0 ? MI_RS(0, 8) : dt == 1 ? MI_RS(1, 8) : MI_RS(2, 8);
#endif
  return dt == 0 ? MI_RS(0, 12) : dt == 1 ? MI_RS(1, 12) : MI_RS(2, 12);
#undef MI_RS
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

// Diagnostics (A/B build): the rank_reg stamps of the last MICLIP_RANK_STAMP launch, 256 x 10
extern "C" int mi_debug_rank_stamp(unsigned long long* host, int n) {
#if MICLIP_AB
  if (!host || n < 0) return -1;
  if (n > 256 * 10) n = 256 * 10;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(miclip::g_rank_stamp), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
#else
  (void)host;
  (void)n;
  return -2;   // A/B build only
#endif
}
