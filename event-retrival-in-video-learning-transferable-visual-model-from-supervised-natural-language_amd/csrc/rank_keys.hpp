// Device helpers shared by the rank kernels (rank.hip, rank_mirror.hip):
// order keys, the row-norm reciprocal, and the data-independent bitonic
// top-16 list update (see rank.hip's rank_stream comment).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <cmath>

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

// Branch-free (selects only): in the streaming kernels' per-tile score loop an
// early return here became an exec-masked branch per score, which also split
// the row-norm LDS reads into 16 serialised read + wait pairs.
__device__ __forceinline__ uint32_t score_key(float s, int nan_first) {
  const uint32_t u = __float_as_uint(s == 0.0f ? 0.0f : s);   // -0 == +0
  const uint32_t key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  const uint32_t nan_key = nan_first ? 0xFFFFFFFFu : 0u;
  return s != s ? nan_key : key;
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

// The shared threshold's LDS atomic max, as inline asm: hipcc orders a
// compiler-visible LDS atomic after every LDS-DMA it cannot prove disjoint, i.e.
// an s_waitcnt vmcnt(0) ahead of it, and in the streaming kernels that drained
// the whole DMA ring (PF chunks in flight) each time a wave raised tau.  tau
// shares no bytes with the ring.
__device__ __forceinline__ void tau_max(uint32_t* p, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)(LDS_AS uint32_t*)p;
  asm volatile("ds_max_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// Lead bound, the streaming kernels' second threshold.  A workgroup holds 8
// lists per query (4 waves x 2 lane halves) over disjoint rows; each publishes
// its 2nd-best key in lead[q][list].  Then 8 lists x 2 rows = 16 distinct rows
// score at least the smallest of the 8 keys, a lower bound of the query's
// 16th-best key (so of its k-th for every k <= 16): far tighter than one list's
// 16th-best (tau) while each list has seen an eighth of the rows, so fewer
// candidates reach the list update.  LDS: [32 queries][8] u32, zeroed at entry;
// inline asm so that hipcc adds no LDS-DMA ordering wait.
constexpr size_t LEAD_LDS = 32 * 8 * 4;
__device__ __forceinline__ uint32_t lead_min(const uint32_t* lead, int r) {
  typedef unsigned int u32x4l __attribute__((ext_vector_type(4)));
  const uint32_t a = (uint32_t)(uintptr_t)(LDS_AS const uint32_t*)(lead + r * 8);
  u32x4l x, y;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x), "=&v"(y) : "v"(a) : "memory");
  const uint32_t m0 = min(min(x[0], x[1]), min(x[2], x[3]));
  const uint32_t m1 = min(min(y[0], y[1]), min(y[2], y[3]));
  return min(m0, m1);
}
__device__ __forceinline__ void lead_publish(uint32_t* lead, int r, int list, uint32_t key) {
  const uint32_t a = (uint32_t)(uintptr_t)(LDS_AS uint32_t*)(lead + r * 8 + list);
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(key) : "memory");
}

// A tile's candidates c[0..15] (0 = none; m: the non-empty ones) into the
// sorted (desc) top-16 list L.  Once the threshold has settled a lane has 0 or
// 1 candidate per tile, and a full bitonic sort + merge (~1000 instructions of
// 64-bit compare/select) for that one entry was the per-tile cost that bounded
// the streaming rank kernels (one wave per SIMD: nothing hides it).  So: while
// no lane has more than 6, each round inserts every lane's next candidate with
// one branch-free pass over L (~120 instructions; an empty lane inserts 0, a
// no-op), for as many rounds as the lane with the most; otherwise sort + merge.
// Same final list either way: the packed keys are unique.
__device__ __forceinline__ void list_update16(uint64_t (&L)[16], uint64_t (&c)[16], uint32_t m) {
  const int pc = __builtin_popcount(m);
  if (__any(pc > 6)) {
    bitonic_sort16_desc(c);
    merge16_desc(L, c);
    return;
  }
  if (__all(pc <= 1)) {   // the common case: one insertion, the entry is the OR of the slots
    uint64_t e = 0ull;
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) e |= c[rg];
#pragma unroll
    for (int p = 15; p > 0; --p) L[p] = e > L[p - 1] ? L[p - 1] : (e > L[p] ? e : L[p]);
    L[0] = e > L[0] ? e : L[0];
    return;
  }
  while (__any(m != 0u)) {
    const int i = m ? __builtin_ctz(m) : 16;
    uint64_t e = 0ull;
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) e = rg == i ? c[rg] : e;
#pragma unroll
    for (int p = 15; p > 0; --p) L[p] = e > L[p - 1] ? L[p - 1] : (e > L[p] ? e : L[p]);
    L[0] = e > L[0] ? e : L[0];
    m &= m - 1u;
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

constexpr int FQ = 32;   // queries per ranking workgroup (MFMA N)

// ---- in-launch merge (rank_stream / rank_reg / rank_mirror_kernel, k <= 16):
// replaces the rank_merge_kernel launch after them.  Each workgroup publishes, per query of
// its block, its sorted top-k as 16 packed entries (key << 32 | ~row, row
// relative to index_base; 0 = no entry) in a 128-B slab line of its own, and
// raises the query's global threshold gtau[q] to its k-th key (a lower bound of
// the query's final k-th key: that workgroup alone holds k rows at or above
// it).  The last workgroup of the query block to arrive (agent-scope release,
// ticket fetch_add, acquire: cdna_hip_programming.md §6 G16's counter form)
// reduces: per query a group of threads reads the slabs' heads, keeps the
// entries at or above gtau in a register top-16 each, appends those to LDS,
// and ranks every appended entry by counting the entries that beat it
// (packed keys are unique: index asc breaks ties).  The counters and gtau
// are zeroed by a hipMemsetAsync ahead of the launch.
constexpr size_t fold_lds(int NT) { return 256 + (size_t)NT * 16 * 8; }

// Two levels: workgroups are grouped by FOLD_GS consecutive row blocks; the last arrival of
// a group merges the group's slabs into a group slab, and the last group to finish merges
// the group slabs into the result.  One reducer over ~250 slabs read 32 slabs per thread
// in dependent batches: 60-100 us at the end of every large call (scripts/rank_stamp.py).
constexpr int FOLD_GS = 32;

struct FoldWs {
  uint64_t* slab;    // [nwg][Qpad][16]
  uint64_t* gslab;   // [groups][Qpad][16]
  uint32_t* cnt;     // [query blocks]: groups finished
  uint32_t* gcnt;    // [query blocks][groups]: workgroups of a group finished
  uint32_t* gtau;    // [Qpad]
  uint32_t* aux;     // [32] zeroed with the counters (the certified pass's unsafe flag)
  int64_t Qpad;
  int ngrp;
};

template <int NL>
__device__ __forceinline__ void fold_publish(const uint32_t* Lk, const int32_t* Li, int KC, int64_t q0, int64_t Q,
                                             int k, int64_t r_begin, const FoldWs& f) {
  const int tid = threadIdx.x;
  if (tid < FQ && q0 + tid < Q) {
    int pos[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) pos[l] = 0;
    uint64_t* dst = f.slab + ((int64_t)RB * f.Qpad + q0 + tid) * 16;
    uint32_t kth = 0u;
    bool full = false;
    for (int o = 0; o < 16; ++o) {
      uint64_t e = 0ull;
      if (o < k) {
        uint32_t bk = 0u;
        int32_t bi = INT_MAX;
        int bl = 0;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          const int src = (l >> 1) * 64 + (l & 1) * 32 + tid;
          if (pos[l] < KC) {
            const uint32_t kk = Lk[src * KC + pos[l]];
            const int32_t ii = Li[src * KC + pos[l]];
            if (better(kk, ii, bk, bi)) { bk = kk; bi = ii; bl = l; }
          }
        }
#pragma unroll
        for (int l = 0; l < NL; ++l) pos[l] += (l == bl) ? 1 : 0;
        if (bi != INT_MAX) {
          e = ((uint64_t)bk << 32) | (uint32_t)~(uint32_t)(r_begin + bi);
          if (o == k - 1) { kth = bk; full = true; }
        }
      }
      dst[o] = e;
    }
    if (full) __hip_atomic_fetch_max(&f.gtau[q0 + tid], kth, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// smem: at least FOLD_LDS(NT) bytes (the caller's list area, free here)
template <int NT>
__device__ __forceinline__ void fold_reduce(char* smem, const FoldWs& f, int64_t q0, int64_t Q, int k, int nan_first,
                                            int64_t index_base, float* __restrict__ out_s,
                                            int64_t* __restrict__ out_i, unsigned long long* stamp = nullptr) {
  const int tid = threadIdx.x;
  uint32_t* hdr = (uint32_t*)smem;
  const int nwg = NRB, grp = (int)RB / FOLD_GS, g0 = grp * FOLD_GS;
  const int gsz = nwg - g0 < FOLD_GS ? nwg - g0 : FOLD_GS;
  // ticket: agent-scope release of this workgroup's stores, counter, and on the last arrival an
  // acquire of everyone else's (cdna_hip_programming.md §6 G16's counter form)
  auto last_arrival = [&](uint32_t* counter, uint32_t total) -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's slab stores and gtau atomics
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      hdr[FQ] = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const bool last = hdr[FQ] == total - 1;
    if (last && tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();   // every thread has read the ticket before hdr is reused
    return last;
  };
  if (!last_arrival(f.gcnt + (int64_t)QB * f.ngrp + grp, (uint32_t)gsz)) {
    if (stamp && tid == 0) stamp[5] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  uint64_t* buf = (uint64_t*)(smem + 256);
  const int nq = (int)(Q - q0 < FQ ? Q - q0 : FQ);
  int g = 1;
  while (g < nq) g <<= 1;
  const int tpq = NT / g;                              // threads per query (>= NT / 32)
  const int qi = tid / tpq, sub = tid - qi * tpq;
  const bool act = qi < nq;
  const int64_t q = q0 + qi;
  const int nld = (k + 1) >> 1;                        // 16-byte pieces of a slab line holding k entries

  // merge `count` slab lines (slab w of query q at base[(w Qpad + q) 16]) into the query's top-k:
  // into gdst's line (sorted packed keys, zeros after) or, final, into out_s / out_i
  auto reduce = [&](const uint64_t* base, int count, uint64_t* gdst) {
    if (tid < FQ) hdr[tid] = 0u;
    __syncthreads();
    uint64_t L[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) L[p] = 0ull;
    auto take = [&](uint64_t e, uint64_t tauP) {        // into the sorted (desc) top-16
      if (e < tauP || e <= L[15]) return;
#pragma unroll
      for (int p = 15; p > 0; --p) L[p] = e > L[p - 1] ? L[p - 1] : (e > L[p] ? e : L[p]);
      L[0] = e > L[0] ? e : L[0];
    };
    if (act) {
      // after the acquire a plain (atomic) load sees every workgroup's raise; the fetch_max(0) it
      // replaces was a device-scope RMW per lane, tpq lanes to one address
      const uint64_t tauP = (uint64_t)__hip_atomic_load(&f.gtau[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 32;
      // whole slab lines, unconditionally, a batch at a time (all pieces in flight together)
      constexpr int BATCH = 4;
      for (int w0 = sub; w0 < count; w0 += BATCH * tpq) {
        uint4 hv[BATCH][8];
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
          const int w = w0 + b * tpq;
          const uint4* p = (const uint4*)(base + ((int64_t)(w < count ? w : 0) * f.Qpad + q) * 16);
#pragma unroll
          for (int c = 0; c < 8; ++c) hv[b][c] = p[c];
        }
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
          if (w0 + b * tpq >= count) continue;
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            if (c >= nld) break;
            take(((uint64_t)hv[b][c].y << 32) | hv[b][c].x, tauP);
            take(((uint64_t)hv[b][c].w << 32) | hv[b][c].z, tauP);
          }
        }
      }
    }
    // cut: the largest k-th key among the query's tpq threads (one of them holds k entries at or
    // above it, so the query's k-th is too); entries below it cannot rank, so fewer are appended
    // and counted.  Ties on the key stay in (the cut compares keys only).
    uint64_t lk = 0ull;
#pragma unroll
    for (int p = 0; p < 16; ++p) lk = p == k - 1 ? L[p] : lk;
    uint32_t tk = (uint32_t)(lk >> 32);
    if (tpq <= 64 && (tpq & (tpq - 1)) == 0) {   // the query's threads: an aligned power-of-two lane group
      for (int off = 1; off < tpq; off <<= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)tk, off, 64);
        tk = o > tk ? o : tk;
      }
    } else {
      tk = 0u;
    }
    const uint64_t cut = (uint64_t)tk << 32;
    int m = 0;
#pragma unroll
    for (int p = 0; p < 16; ++p) m += (L[p] != 0ull && L[p] >= cut) ? 1 : 0;   // a prefix: L is sorted
    uint64_t* qb = buf + (int64_t)qi * tpq * 16;
    if (act && m) {
      const uint32_t at = atomicAdd(&hdr[qi], (uint32_t)m);   // LDS
#pragma unroll
      for (int p = 0; p < 16; ++p)
        if (p < m) qb[at + p] = L[p];
    }
    __syncthreads();
    if (act) {
      const int n = (int)hdr[qi];
      int rk[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) rk[p] = 0;
      for (int j = 0; j < n; ++j) {
        const uint64_t e = qb[j];
#pragma unroll
        for (int p = 0; p < 16; ++p) rk[p] += e > L[p] ? 1 : 0;
      }
      if (gdst) {   // the group's top-k as a slab line: ranks 0 .. k - 1, zeros after
        uint64_t* line = gdst + ((int64_t)q) * 16;
#pragma unroll
        for (int p = 0; p < 16; ++p)
          if (p < m && rk[p] < k) line[rk[p]] = L[p];
        for (int r = (n < k ? n : k) + sub; r < 2 * nld; r += tpq) line[r] = 0ull;
      } else {
#pragma unroll
        for (int p = 0; p < 16; ++p)
          if (p < m && rk[p] < k) {
            out_s[q * k + rk[p]] = decode_key((uint32_t)(L[p] >> 32), nan_first);
            out_i[q * k + rk[p]] = index_base + (int64_t)(uint32_t)~(uint32_t)L[p];
          }
        for (int r = n + sub; r < k; r += tpq) {           // fewer than k rows in all
          out_s[q * k + r] = -INFINITY;
          out_i[q * k + r] = -1;
        }
      }
    }
    __syncthreads();
  };

  if (stamp && tid == 0) stamp[5] = __builtin_amdgcn_s_memrealtime();
  if (f.ngrp == 1) {                                   // one group: its last arrival writes the result
    if (stamp && tid == 0) stamp[6] = __builtin_amdgcn_s_memrealtime();
    reduce(f.slab, nwg, nullptr);
    if (stamp && tid == 0) stamp[8] = __builtin_amdgcn_s_memrealtime();
    return;
  }
  reduce(f.slab + (int64_t)g0 * f.Qpad * 16, gsz, f.gslab + (int64_t)grp * f.Qpad * 16);
  if (stamp && tid == 0) stamp[6] = __builtin_amdgcn_s_memrealtime();
  if (!last_arrival(f.cnt + QB, (uint32_t)f.ngrp)) return;
  if (stamp && tid == 0) stamp[7] = __builtin_amdgcn_s_memrealtime();
  reduce(f.gslab, f.ngrp, nullptr);
  if (stamp && tid == 0) stamp[8] = __builtin_amdgcn_s_memrealtime();
}


// ---- split merge (round 5): the pass publishes its workgroup's top-k, a second launch merges.
// The in-launch merge above chains global round trips after the stream (a ticket, the group
// reducer's slab lines, a second ticket, the final reducer: ~60-90 us at 125k-1M rows,
// scripts/rank_stamp.py), and its fold_publish merged the 8 lists of a query with one thread
// per query (~10-20 us).  Here each query's 8 lists (4 waves x 2 lane halves) merge as a tree:
// the two halves by shuffles (merge16_desc), then wave 0 folds the other waves' lists from LDS;
// the workgroup's top-k goes to its slab line (rows global) and raises gtau[q] to its k-th key.
// fold_merge_kernel (rank.hip) then reduces each query's nwg lines in one workgroup.
// smem: >= 4 waves x 32 queries x 16 entries x 8 B = 16 KB, free (the caller's ring, after the
// stream's last wait); every thread of the workgroup calls this.
__device__ __forceinline__ void merge16_xor(uint64_t (&L)[16], int off) {
  uint64_t c[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)L[j], off, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(L[j] >> 32), off, 64);
    c[j] = ((uint64_t)hi << 32) | lo;
  }
  merge16_desc(L, c);
}

template <int NW>
__device__ __forceinline__ void lines_publish(uint64_t (&L)[16], char* smem, int wave, int lane, int64_t q0, int64_t Q,
                                              int k, int64_t r_begin, const FoldWs& f) {
  const int r = lane & 31;
#pragma unroll
  for (int p = 0; p < 16; ++p) {   // rows relative to the workgroup's range -> global (same order)
    const uint64_t e = L[p];
    L[p] = e ? ((e & 0xffffffff00000000ull) | (uint32_t)~(uint32_t)(r_begin + (int64_t)~(uint32_t)e)) : 0ull;
  }
  merge16_xor(L, 32);              // the wave's two half-lists of query r (both halves get it)
  uint64_t* wl = (uint64_t*)smem;  // [NW][32][16]
  __syncthreads();                 // every wave is done with its ring slots
  if (wave > 0 && lane < 32) {
#pragma unroll
    for (int p = 0; p < 16; ++p) wl[((wave * 32) + r) * 16 + p] = L[p];
  }
  __syncthreads();
  if (wave == 0 && lane < 32) {
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      uint64_t c[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) c[p] = wl[((w * 32) + r) * 16 + p];
      merge16_desc(L, c);
    }
    if (q0 + r < Q) {
      typedef unsigned int u32x4lp __attribute__((ext_vector_type(4)));
      u32x4lp* dst = (u32x4lp*)(f.slab + ((int64_t)RB * f.Qpad + q0 + r) * 16);
      const int nld = (k + 1) >> 1;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (c >= nld) break;
        dst[c] = (u32x4lp){(uint32_t)L[2 * c], (uint32_t)(L[2 * c] >> 32), (uint32_t)L[2 * c + 1],
                           (uint32_t)(L[2 * c + 1] >> 32)};
      }
      uint64_t kth = L[0];
#pragma unroll
      for (int p = 1; p < 16; ++p) kth = p == k - 1 ? L[p] : kth;
      if (kth) __hip_atomic_fetch_max(&f.gtau[q0 + r], (uint32_t)(kth >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static inline int64_t qpad(int64_t Q) { return (Q + FQ - 1) / FQ * FQ; }
static inline size_t al128(size_t b) { return (b + 127) / 128 * 128; }

// in-launch merge workspace: slabs [nwg][Qpad][16] u64, group slabs [groups][Qpad][16] u64,
// counters [Qpad / 32] u32, group counters [Qpad / 32][groups] u32, gtau [Qpad] u32, aux [32]
// u32 (the last four contiguous: fold_zero clears them with one memset, or a preceding kernel
// with fold_zero_words / fold_zero_base)
static inline int64_t fold_groups(int64_t nwg) { return (nwg + FOLD_GS - 1) / FOLD_GS; }

static inline size_t fold_ws_bytes(int64_t nwg, int64_t Q) {
  const int64_t qp = qpad(Q), ng = fold_groups(nwg);
  return (size_t)((nwg + ng) * qp) * 128 + al128((size_t)(qp / FQ) * 4) + al128((size_t)(qp / FQ * ng) * 4) +
         al128((size_t)qp * 4) + 128;
}

static inline FoldWs fold_ws(void* ws, int64_t nwg, int64_t Q) {
  const int64_t qp = qpad(Q), ng = fold_groups(nwg);
  FoldWs f;
  f.slab = (uint64_t*)ws;
  f.gslab = (uint64_t*)((char*)ws + (size_t)(nwg * qp) * 128);
  f.cnt = (uint32_t*)((char*)f.gslab + (size_t)(ng * qp) * 128);
  f.gcnt = (uint32_t*)((char*)f.cnt + al128((size_t)(qp / FQ) * 4));
  f.gtau = (uint32_t*)((char*)f.gcnt + al128((size_t)(qp / FQ * ng) * 4));
  f.aux = (uint32_t*)((char*)f.gtau + al128((size_t)qp * 4));
  f.Qpad = qp;
  f.ngrp = (int)ng;
  return f;
}

// the split merge's second launch (rank.hip): grid Q, results into out_s / out_i [Q][k]
hipError_t fold_merge(const FoldWs& f, int64_t nwg, int64_t Q, int k, int nan_first, int64_t index_base, float* out_s,
                      int64_t* out_i, const int32_t* gate, hipStream_t s);

static inline int64_t fold_zero_words(const FoldWs& f) { return (int64_t)((f.aux + 32) - f.cnt); }
static inline uint32_t* fold_zero_base(const FoldWs& f) { return f.cnt; }

static inline hipError_t fold_zero(const FoldWs& f, hipStream_t s) {
  return hipMemsetAsync(f.cnt, 0, (size_t)fold_zero_words(f) * 4, s);
}

}  // namespace rankk
}  // namespace miclip
