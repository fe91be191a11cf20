// Multi-head attention core of openai/CLIP's nn.MultiheadAttention
// (softmax(q k^T / sqrt(64)) v per 64-wide head, causal mask for the text
// tower), restated in oracle/clip_ref.py::_mha.  Built with -fno-honor-nans
// (Makefile): the softmax max/sum chains then compile to v_max3 without NaN
// canonicalisation; -inf masking is unaffected.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace miclip {

namespace {

// --------------------------------------------------------------- attention
// One wave per (sequence, head), head dim 64, whole padded sequence (SP rows,
// multiple of 32) per wave; no workgroup barriers.
//   S = Q K^T : Q (A operand) and K (B operand) fragments are loaded straight
//     from the packed qkv rows as 16-byte pieces (the 16x16x32 operand map
//     wants 8 consecutive head dims of one row per lane), rows past S clamped;
//   softmax over keys in f32 registers (scale 1/8, key >= S and causal masks),
//     rows reduced across the 16 lanes that hold them; P normalised, to bf16,
//     through a per-wave LDS tile (C layout -> operand layout);
//   O^T = V^T P^T with V^T (A operand) from a per-wave transposed LDS image
//     and P (B operand), so each lane holds 4 consecutive head dims of one
//     query row -> one 8-byte store.
// LDS rows are padded to an odd number of 16-byte slots.
template <int SP>
__global__ __launch_bounds__(64) void attention_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                                       int S, int W, int H, int causal, int items) {
  constexpr int TS = SP + 8;  // bf16 per V^T / P row (odd number of 16-byte slots)
  __shared__ __attribute__((aligned(16))) uint16_t lds[64 * TS + 16 * TS];
  uint16_t* Vt = lds;
  uint16_t* Pw = lds + 64 * TS;
  const int item = blockIdx.x;
  if (item >= items) return;
  const int bseq = item / H, h = item % H;
  const int lane = threadIdx.x;
  const int64_t ld = 3 * (int64_t)W;
  const uint16_t* qb = qkv + (int64_t)bseq * S * ld + h * 64;
  const uint16_t* kb = qb + W;
  const uint16_t* vb = qb + 2 * W;

  // V^T image: lane (ch = lane>>3, r8 = lane&7) loads 8 head dims of key
  // row r and scatters them down column r of V^T (consecutive lanes ->
  // consecutive keys, so the 2-byte writes of an instruction are contiguous).
  for (int r0 = 0; r0 < SP; r0 += 8) {
    const int r = r0 + (lane & 7), ch = lane >> 3;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < S) v = *(const uint4*)(vb + (int64_t)r * ld + ch * 8);
    const uint16_t* vv = (const uint16_t*)&v;
#pragma unroll
    for (int e = 0; e < 8; ++e) Vt[(ch * 8 + e) * TS + r] = vv[e];
  }

  constexpr int NKT = SP / 16;
  const float scale = 0.125f;  // 64 ** -0.5
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int nqt = (S + 15) / 16;
  for (int qt = 0; qt < nqt; ++qt) {
    const int64_t qrow = min(qt * 16 + fr, S - 1);
    bf16x8 qa[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) qa[s] = *(const bf16x8*)(qb + qrow * ld + 32 * s + fk);
    f32x4 sc[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int64_t krow = min(kt * 16 + fr, S - 1);
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 kf = *(const bf16x8*)(kb + krow * ld + 32 * s + fk);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[s], kf, c, 0, 0, 0);
      }
      sc[kt] = c;
    }
    // sc[kt][j]: query row qt*16 + 4*(lane>>4) + j, key kt*16 + (lane&15)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = qt * 16 + 4 * (lane >> 4) + j;
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const int key = kt * 16 + fr;
        float v = sc[kt][j] * scale;
        if (key >= S || (causal && key > row)) v = -INFINITY;
        sc[kt][j] = v;
        m = fmaxf(m, v);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const float p = __expf(sc[kt][j] - m);
        sc[kt][j] = p;
        sum += p;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
      const float inv = 1.0f / sum;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) Pw[(4 * (lane >> 4) + j) * TS + kt * 16 + fr] = f2bf_hw(sc[kt][j] * inv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // O^T[d][q] = sum_key V^T[d][key] P[q][key]
    uint2 ov[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < SP / 32; ++s) {
        const bf16x8 va = *(const bf16x8*)(Vt + (dt * 16 + fr) * TS + 32 * s + fk);
        const bf16x8 pb = *(const bf16x8*)(Pw + fr * TS + 32 * s + fk);
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o, 0, 0, 0);
      }
      ov[dt] = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
    }
    // lane: query row qt*16 + (lane&15), head dims dt*16 + 4*(lane>>4) + 0..3
    const int row = qt * 16 + fr;
    if (row < S) {
      uint16_t* dst = out + ((int64_t)bseq * S + row) * W + h * 64 + 4 * (lane >> 4);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) *(uint2*)(dst + dt * 16) = ov[dt];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------ attention, long sequences, K/V in LDS
// One workgroup of NW waves per (sequence, head); wave w owns the NT query
// tiles w, w + NW, ... (16 rows each) for the whole key sweep, so every 64-key
// chunk of K and V is fetched from HBM/L2 ONCE per (sequence, head) and shared
// by all waves through a two-slot LDS ring (a wave-per-query-tile design
// re-reads K per tile: 37 x the K bytes at 577 tokens, 1.8x slower).  Per chunk:
//   stage   : each thread register-loads 16 B of K and of V of chunk c + 1
//             (issued before chunk c's math, written to the other ring slot
//             after it; one barrier per chunk).  K lands row-major (144-byte
//             rows: the 16 rows of an A-operand read hit disjoint banks), V
//             transposed (V^T rows of 64 keys, 136-byte rows).
//   frags   : the chunk's K (A operand of S^T = K Q^T) and V^T (A operand of
//             O^T = V^T P^T) fragments are read from LDS once per chunk into
//             registers and reused by the wave's NT tiles.
//   softmax : scores in the log2 domain u = s * log2(e)/8 (one FMA per score
//             with the reference max folded in); the running max is only
//             moved (and O, l rescaled) when the chunk max exceeds it by more
//             than 2^8 - lazy rescaling: P <= 256, exact after the final 1/l;
//             row max across the 4 lane groups by permlane16/32 swaps.
// Keys >= S are masked (only in the last chunk, and 16-key tiles past S skip
// their MFMAs; skipping their exponentials too measured 10% slower - the extra
// uniform branches split the softmax block); V^T columns >= S are 0.
// SLOTS = 1: S <= 64 (one chunk; B/32's 50 tokens): a single LDS slot and no
// look-ahead staging, which halves the LDS footprint and frees the staging
// registers, so more workgroups fit per CU for this latency-bound case.
// NW = blockDim / 64 waves (8, or 4 for the single-slot S <= 64 instance);
// PP = 16-byte staging pieces of K (and of V) per thread per chunk (1 for 8
// waves, 2 for 4).
// HP heads per workgroup (A/B: 2 = adjacent heads of one sequence, their 128-byte row segments
// read together as 256 bytes), each on its own NW waves and LDS slots.
// PIPE (S <= 64: NT = 1, SLOTS = 1, HP = 1): persistent workgroups walk items blockIdx.x,
// + gridDim.x, ... and load the next item's Q fragments and K / V pieces into registers before
// computing the current one, so a workgroup always has an item's qkv reads in flight.
// VB (S <= 64 instance): the V^T fragments' eight LDS reads issued together and waited for once
// before the P V MFMAs (hipcc otherwise waits for each read right before its MFMA)
template <int NT, int PP, int SLOTS, int HP = 1, bool PIPE = false, bool VB = false>
__device__ __forceinline__ void attention_flash_body(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                                     int S, int W, int H, int causal, uint8_t* __restrict__ q8,
                                                     uint8_t* __restrict__ qs, int64_t rows_pad, int items = 0) {
  static_assert(!PIPE || (NT == 1 && SLOTS == 1 && HP == 1), "PIPE: the single-chunk instance only");
  // causal bit 11: the first 16-query tile only (the last vision block, whose outputs are read at the
  // CLS rows alone, api.cpp last_block_cls); the other tiles' waves still stage K / V
  const bool q0only = (causal >> 11) & 1;
  causal &= 1;
  constexpr int KS = 72, VS = 68;  // LDS row strides (bf16)
  const int NW = PP == 1 ? 8 : (int)(blockDim.x >> 6) / HP;  // PP = 1 is launched with 8 waves
  __shared__ __attribute__((aligned(16))) uint16_t Ksh[HP][SLOTS][64 * KS];
  __shared__ __attribute__((aligned(16))) uint16_t Vsh[HP][SLOTS][64 * VS];
  const int hh = HP == 1 ? 0 : (int)(threadIdx.x >> 6) / NW;   // this thread's head of the workgroup's HP
  uint16_t(*Ks)[64 * KS] = Ksh[hh];
  uint16_t(*Vs)[64 * VS] = Vsh[hh];
  const int tid = threadIdx.x - hh * 64 * NW, lane = tid & 63, wave = tid >> 6;
  const int64_t ld = 3 * (int64_t)W;
  int item = blockIdx.x;
  bool first = true;
  uint4 kr_n[PP], vr_n[PP];   // PIPE: the next item's K / V pieces and Q fragments
  bf16x8 qf_n[2];
  for (;;) {
  const int bseq = item / (H / HP), h = (item % (H / HP)) * HP + hh;
  const uint16_t* qb = qkv + (int64_t)bseq * S * ld + h * 64;
  const uint16_t* kb = qb + W;
  const uint16_t* vb = qb + 2 * W;
  const int nch = (S + 63) / 64, nqt = q0only ? 1 : (S + 15) / 16;
  const int fr = lane & 15, g = lane >> 4, fk = 8 * g;
  const float sl2 = 0.125f * 1.4426950408889634f;  // head_dim^-0.5 * log2(e)
  constexpr float RESCALE = 8.0f;                  // lazy-rescale threshold (log2 units)

  uint4 kr[PP], vr[PP];
#define FA_STAGE_LOAD(c)                                                                  \
  _Pragma("unroll") for (int i = 0; i < PP; ++i) {                                        \
    const int p_ = tid + i * 64 * NW, r_ = (c) * 64 + (p_ >> 3), ch_ = p_ & 7;            \
    kr[i] = make_uint4(0, 0, 0, 0);                                                       \
    vr[i] = make_uint4(0, 0, 0, 0);                                                       \
    if ((PP == 1 || p_ < 512) && r_ < S) {                                                \
      kr[i] = *(const uint4*)(kb + (int64_t)r_ * ld + ch_ * 8);                           \
      vr[i] = *(const uint4*)(vb + (int64_t)r_ * ld + ch_ * 8);                           \
    }                                                                                     \
  }
#define FA_STAGE_WRITE(slot)                                                              \
  _Pragma("unroll") for (int i = 0; i < PP; ++i) {                                        \
    const int p_ = tid + i * 64 * NW, r_ = p_ >> 3, ch_ = p_ & 7;                         \
    if (PP == 1 || p_ < 512) {                                                            \
      *(uint4*)(&Ks[slot][r_ * KS + ch_ * 8]) = kr[i];                                    \
      const uint16_t* vv_ = (const uint16_t*)&vr[i];                                      \
      _Pragma("unroll") for (int e = 0; e < 8; ++e) Vs[slot][(ch_ * 8 + e) * VS + r_] = vv_[e]; \
    }                                                                                     \
  }

  bf16x8 qf[NT][2];
  float m[NT], l[NT];
  f32x4 o[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int qrow = min((wave + NW * t) * 16 + fr, S - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[t][s] = (!PIPE || first) ? *(const bf16x8*)(qb + (int64_t)qrow * ld + 32 * s + fk) : qf_n[s];
    m[t] = -INFINITY;
    l[t] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (!PIPE || first) {
    FA_STAGE_LOAD(0);
  } else {
#pragma unroll
    for (int i = 0; i < PP; ++i) {
      kr[i] = kr_n[i];
      vr[i] = vr_n[i];
    }
  }
  // (PIPE: the previous item's LDS reads ended at the chunk loop's closing barrier)
  FA_STAGE_WRITE(0);
  __syncthreads();
  if (PIPE && item + (int)gridDim.x < items) {   // the next item's operands, in flight during this one
    const int nx = item + (int)gridDim.x;
    const uint16_t* nq = qkv + (int64_t)(nx / H) * S * ld + (nx % H) * 64;
    const int qrow = min(wave * 16 + fr, S - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) qf_n[s] = *(const bf16x8*)(nq + (int64_t)qrow * ld + 32 * s + fk);
#pragma unroll
    for (int i = 0; i < PP; ++i) {
      const int p_ = tid + i * 64 * NW, r_ = p_ >> 3, ch_ = p_ & 7;
      kr_n[i] = make_uint4(0, 0, 0, 0);
      vr_n[i] = make_uint4(0, 0, 0, 0);
      if ((PP == 1 || p_ < 512) && r_ < S) {
        kr_n[i] = *(const uint4*)(nq + W + (int64_t)r_ * ld + ch_ * 8);
        vr_n[i] = *(const uint4*)(nq + 2 * W + (int64_t)r_ * ld + ch_ * 8);
      }
    }
  }

  for (int c = 0; c < nch; ++c) {
    const int slot = SLOTS == 1 ? 0 : (c & 1);
    if (SLOTS > 1 && c + 1 < nch) FA_STAGE_LOAD(c + 1);
    const int kvalid = min(64, S - c * 64);  // keys of this chunk < S
    bf16x8 kf[4][2], vf[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) kf[kt][s] = *(const bf16x8*)(&Ks[slot][(kt * 16 + fr) * KS + 32 * s + fk]);
    auto read_vf = [&]() {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint16_t* vrow = &Vs[slot][(dt * 16 + fr) * VS + 32 * s + 4 * g];
          const uint2 lo = *(const uint2*)vrow;
          const uint2 hi = *(const uint2*)(vrow + 16);
          vf[dt][s] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        }
    };
    // NT > 1: V^T fragments read once per chunk for all tiles; single-tile
    // (S <= 64) instance: read after the softmax, so K and V^T fragments are
    // never live together (fewer VGPRs -> more resident workgroups)
    if (SLOTS > 1) read_vf();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int qt = wave + NW * t;
      if (qt >= nqt || (causal && c * 64 > qt * 16 + 15)) continue;  // wave-uniform
      const int qrow = qt * 16 + fr;
      f32x4 sc[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if (kt * 16 < kvalid) {
#pragma unroll
          for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][s], qf[t][s], acc, 0, 0, 0);
        }
        sc[kt] = acc;
      }
      // sc[kt][j]: query qrow, key c*64 + kt*16 + 4g + j
      if (kvalid < 64 || (causal && (c + 1) * 64 > qt * 16)) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int key = c * 64 + kt * 16 + 4 * g + j;
            if (key >= S || (causal && key > qrow)) sc[kt][j] = -INFINITY;
          }
      }
      float cm = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                       fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
      cm = fmaxf(cm, fmaxf(fmaxf(fmaxf(sc[2][0], sc[2][1]), fmaxf(sc[2][2], sc[2][3])),
                           fmaxf(fmaxf(sc[3][0], sc[3][1]), fmaxf(sc[3][2], sc[3][3]))));
      {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
      }
      const float cmu = cm * sl2;  // finite: chunk 0 holds key 0 <= every row
      if (cmu > m[t] + RESCALE) {
        const float alpha = __builtin_amdgcn_exp2f(m[t] - cmu);
        l[t] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[t][dt] *= alpha;
        m[t] = cmu;
      }
      const float mu = m[t];
      float ps[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sc[kt][j] = __builtin_amdgcn_exp2f(fmaf(sc[kt][j], sl2, -mu));
        ps[kt] = (sc[kt][0] + sc[kt][1]) + (sc[kt][2] + sc[kt][3]);
      }
      l[t] += (ps[0] + ps[1]) + (ps[2] + ps[3]);
      if (SLOTS == 1) {
        __builtin_amdgcn_sched_barrier(0);
        read_vf();
        if (VB) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 1 && kvalid <= 32) break;  // keys past round32(S): P = 0, V^T = 0
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[j] = (__bf16)sc[2 * s][j];
          pb[4 + j] = (__bf16)sc[2 * s + 1][j];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[t][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt][s], pb, o[t][dt], 0, 0, 0);
      }
    }
    if (SLOTS > 1 && c + 1 < nch) FA_STAGE_WRITE(slot ^ 1);
    __syncthreads();
  }
#undef FA_STAGE_LOAD
#undef FA_STAGE_WRITE

#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int qt = wave + NW * t;
    if (qt >= nqt) continue;
    const int qrow = qt * 16 + fr;
    float lt = l[t];
    {
      const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
      lt = __uint_as_float(a[0]) + __uint_as_float(a[1]);
      const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
      lt = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
    const float inv = 1.0f / lt;
    // o[t][dt][j]: query qrow, head dim dt*16 + 4g + j
    if (q8) {  // MX-fp8 output: this head's 64 dims are one 64-k block of out_proj
      float amax = 0.f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fabsf(o[t][dt][j] * inv));
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      const int X = mx_block_exp(amax);
      const float scl = ldexpf(1.0f, -X);
      if (qrow < S) {
        const int64_t row = (int64_t)bseq * S + qrow;
        uint8_t* dst = q8 + row * W + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          *(uint32_t*)(dst + dt * 16) =
              mx_pack4(o[t][dt][0] * inv, o[t][dt][1] * inv, o[t][dt][2] * inv, o[t][dt][3] * inv, scl);
        if (g == 0) qs[mx_scale_index(row, h, rows_pad)] = (uint8_t)(X + 127);
      }
      continue;
    }
    if (qrow < S) {
      uint16_t* dst = out + ((int64_t)bseq * S + qrow) * W + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *(uint2*)(dst + dt * 16) = make_uint2(pack_bf16x2(o[t][dt][0] * inv, o[t][dt][1] * inv),
                                              pack_bf16x2(o[t][dt][2] * inv, o[t][dt][3] * inv));
    }
  }
  if (!PIPE) break;
  item += (int)gridDim.x;
  if (item >= items) break;
  first = false;
  }   // items
}

template <int NT, int PP, int SLOTS = 2>
__global__ __launch_bounds__(512) void attention_flash_kernel(const uint16_t* __restrict__ qkv,
                                                                uint16_t* __restrict__ out, int S, int W, int H,
                                                                int causal, uint8_t* __restrict__ q8,
                                                                uint8_t* __restrict__ qs, int64_t rows_pad) {
  attention_flash_body<NT, PP, SLOTS>(qkv, out, S, W, H, causal, q8, qs, rows_pad);
}

#if MICLIP_AB
// A/B variants of the S <= 64 case (B/32's 50 tokens; the default is attention_flash_kernel<1, 2, 1>
// on 4 waves).  Timed in interleaved rounds at 10k frames (scripts/attn_micro.py,
// profiles/r04_ai_attn_micro.log), all bit-identical: default 603 us; an occupancy target of 6 waves
// per SIMD (72 instead of 74 VGPRs, MICLIP_ATTN_SHORT=3) 604 us; two adjacent heads per 8-wave
// workgroup, their 128-byte qkv / output row segments together (=2) 616 us.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void attention_short_kernel(
    const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out, int S, int W, int H, int causal,
    uint8_t* __restrict__ q8, uint8_t* __restrict__ qs, int64_t rows_pad) {
  attention_flash_body<1, 2, 1>(qkv, out, S, W, H, causal, q8, qs, rows_pad);
}

__global__ __launch_bounds__(256) void attention_pipe_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                                             int S, int W, int H, int causal, uint8_t* __restrict__ q8,
                                                             uint8_t* __restrict__ qs, int64_t rows_pad, int items) {
  attention_flash_body<1, 2, 1, 1, true>(qkv, out, S, W, H, causal, q8, qs, rows_pad, items);
}

__global__ __launch_bounds__(256) void attention_vb_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                                           int S, int W, int H, int causal, uint8_t* __restrict__ q8,
                                                           uint8_t* __restrict__ qs, int64_t rows_pad) {
  attention_flash_body<1, 2, 1, 1, false, true>(qkv, out, S, W, H, causal, q8, qs, rows_pad);
}

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(6))) void attention_short2_kernel(
    const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out, int S, int W, int H, int causal,
    uint8_t* __restrict__ q8, uint8_t* __restrict__ qs, int64_t rows_pad) {
  attention_flash_body<1, 2, 1, 2>(qkv, out, S, W, H, causal, q8, qs, rows_pad);
}
#endif


// ----------------------------- attention, vision towers: K/V resident in LDS
// 64 < S <= 640, non-causal (ViT-L/14 257 tokens, L/14@336 577).  One
// workgroup of NW waves per (sequence, head).  The whole head's K and V
// (rows padded to 32, rows >= S clamped copies: masked / multiplied by P = 0)
// are DMA'd into LDS ONCE (global_load_lds, 8 rows x 128 B per instruction),
// then every wave runs its query tiles (16 rows: w, w + NW, ...) over all keys
// with no further workgroup barrier — a straggler wave no longer parks the
// other seven at a per-chunk barrier, and a second workgroup on the CU
// (S = 257: 72 KB of LDS each) fills the SIMDs meanwhile.
//   K image : 16-byte chunk c of key row r at slot c ^ ((r >> 1) & 7) (the 16
//             rows of a ds_read_b128 A-operand read hit all 16 slots);
//   V image : row-major [key][64 dims], 8-byte unit u at u ^ (((r >> 1) & 3) << 2),
//             read transposed by ds_read_b64_tr_b16 into the V^T A operand of
//             O^T = V^T P^T (a 32-lane half = 8 consecutive keys x 4 units:
//             all 32 8-byte bank pairs once) — no transposing LDS writes;
//   per 64-key chunk: S^T = K Q^T (8 MFMA), online softmax in the log2
//   domain with lazy rescale (flash kernel above), P to bf16, 8 PV MFMAs;
//   the partial last chunk runs only its valid 16-key tiles (NKT template).
// SPLIT (S % 16 small, e.g. L/14's 257 = 16 x 16 + 1): the last, nearly empty query tile
// would add a third tile to wave 0 while the other waves idle with two; instead every wave
// runs it over its share of the 16-key tiles (w, w + NW, ...) and wave 0 merges the partial
// softmax states (m, l, o) of its valid rows through LDS.
template <int NW, bool TT2 = true, bool SPLIT = false, bool SFIRST = false, bool QPF = false>
__global__ __launch_bounds__(NW * 64) void attention_res_kernel(const uint16_t* __restrict__ qkv,
                                                                uint16_t* __restrict__ out, int S, int W, int H,
                                                                uint8_t* __restrict__ q8, uint8_t* __restrict__ qs,
                                                                int64_t rows_pad) {
  extern __shared__ __attribute__((aligned(16))) char res_lds[];
  const int spad = (S + 31) & ~31;
  char* Kimg = res_lds;
  char* Vimg = res_lds + spad * 128;
  const int item = blockIdx.x;
  const int bseq = item / H, h = item % H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ld = 3 * (int64_t)W;
  const uint16_t* qb = qkv + (int64_t)bseq * S * ld + h * 64;
  const uint16_t* kb = qb + W;
  const uint16_t* vb = qb + 2 * W;

  // ---- K, V -> LDS (one DMA instruction = 8 rows)
  {
    const int nr8 = spad >> 3;
    const int slot = lane & 7;
    for (int i = wave; i < 2 * nr8; i += NW) {
      const bool isv = i >= nr8;
      const int i8 = isv ? i - nr8 : i;
      const int r = i8 * 8 + (lane >> 3);
      const int c = isv ? (slot ^ (((r >> 1) & 3) << 1)) : (slot ^ ((r >> 1) & 7));
      glds16((isv ? vb : kb) + (int64_t)min(r, S - 1) * ld + c * 8, (isv ? Vimg : Kimg) + i8 * 1024);
    }
  }

  const int nqt = (S + 15) / 16, nch = (S + 63) / 64;
  const int last_kvalid = S - (nch - 1) * 64;   // 1..64
  const int fr = lane & 15, g = lane >> 4;
  const float sl2 = 0.125f * 1.4426950408889634f;  // head_dim^-0.5 * log2(e)
  constexpr float RESCALE = 8.0f;
  const int rk0 = fr * 128 + (((0 + g) ^ (fr >> 1)) << 4);
  const int rk1 = fr * 128 + (((4 + g) ^ (fr >> 1)) << 4);
  const int vq = (lane & 15) >> 2, vp = lane & 3;
  const int vx = (2 * g + (vq >> 1)) & 3;
  const int rvb = (4 * g + vq) * 128 + vp * 8;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  auto tr_read = [&](const char* p) -> s16x4 {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(LDS_AS char*)(uintptr_t)(const LDS_AS char*)p);
  };

  // QPF (A/B): a tile's Q fragments are loaded one tile ahead (the wave's first tile's beside the
  // K/V load), so their latency is not exposed at the head of every tile
  bf16x8 qn[2];
  auto load_q = [&](int t, bf16x8 (&q)[2]) {
    const int qrow = min(t * 16 + fr, S - 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) q[s2] = *(const bf16x8*)(qb + (int64_t)qrow * ld + 32 * s2 + 8 * g);
  };
  if (QPF) load_q(wave, qn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // A wave's query tiles are w, w + NW, w + 2 NW, ...; it runs them two at a
  // time (TT = 2): each K / V^T fragment read from LDS feeds both tiles' MFMAs,
  // and one tile's softmax VALU has the other tile's MFMAs beside it (one tile
  // at a time, the QK MFMA -> max -> exp -> PV MFMA chain left the matrix pipe
  // idle behind its own dependencies).  An odd last tile runs alone (TT = 1).
  auto tiles = [&](auto tt_c, int t0, int t1) {
    constexpr int TT = decltype(tt_c)::value;
    const int tq[2] = {t0, t1};
    bf16x8 qf[TT][2];
    if (QPF && TT == 1) {
      qf[0][0] = qn[0];
      qf[0][1] = qn[1];
      if (t0 + NW < (SPLIT ? nqt - 1 : nqt)) load_q(t0 + NW, qn);   // the wave's next tile
    } else {
#pragma unroll
      for (int u = 0; u < TT; ++u) {
        const int qrow = min(tq[u] * 16 + fr, S - 1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) qf[u][s2] = *(const bf16x8*)(qb + (int64_t)qrow * ld + 32 * s2 + 8 * g);
      }
    }
    float m[TT], l[TT];
    f32x4 o[TT][4];
#pragma unroll
    for (int u = 0; u < TT; ++u) {
      m[u] = -INFINITY;
      l[u] = 0.f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[u][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // one 64-key chunk; NKT valid 16-key tiles, MASK: keys >= S inside them
    auto chunk = [&](auto nkt_c, auto mask_c, int c) {
      constexpr int NKT = decltype(nkt_c)::value;
      constexpr bool MASK = decltype(mask_c)::value;
      const char* kc = Kimg + c * 64 * 128;
      f32x4 sc[TT][NKT];
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const bf16x8 k0 = *(const bf16x8*)(kc + kt * 16 * 128 + rk0);
        const bf16x8 k1 = *(const bf16x8*)(kc + kt * 16 * 128 + rk1);
#pragma unroll
        for (int u = 0; u < TT; ++u) {
          const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[u][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          sc[u][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[u][1], acc, 0, 0, 0);
        }
      }
      // sc[u][kt][j]: query tq[u]*16 + fr, key c*64 + kt*16 + 4g + j
#pragma unroll
      for (int u = 0; u < TT; ++u) {
        if (MASK) {
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (c * 64 + kt * 16 + 4 * g + j >= S) sc[u][kt][j] = -INFINITY;
        }
        float cm = fmaxf(fmaxf(sc[u][0][0], sc[u][0][1]), fmaxf(sc[u][0][2], sc[u][0][3]));
#pragma unroll
        for (int kt = 1; kt < NKT; ++kt)
          cm = fmaxf(cm, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
        {
          const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
          cm = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
          const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
          cm = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
        }
        const float cmu = cm * sl2;   // finite: chunk 0 holds key 0 for every row
        if (cmu > m[u] + RESCALE) {
          const float alpha = __builtin_amdgcn_exp2f(m[u] - cmu);
          l[u] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[u][dt] *= alpha;
          m[u] = cmu;
        }
        float ps = 0.f;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
          for (int j = 0; j < 4; ++j) sc[u][kt][j] = __builtin_amdgcn_exp2f(fmaf(sc[u][kt][j], sl2, -m[u]));
          ps += (sc[u][kt][0] + sc[u][kt][1]) + (sc[u][kt][2] + sc[u][kt][3]);
        }
        l[u] += ps;
      }
#pragma unroll
      for (int s2 = 0; s2 < (NKT + 1) / 2; ++s2) {
        bf16x8 pb[TT];
#pragma unroll
        for (int u = 0; u < TT; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pb[u][j] = (__bf16)sc[u][2 * s2][j];
            pb[u][4 + j] = 2 * s2 + 1 < NKT ? (__bf16)sc[u][(2 * s2 + 1) < NKT ? 2 * s2 + 1 : 0][j] : (__bf16)0.f;
          }
        const char* vc = Vimg + (c * 64 + 32 * s2) * 128 + rvb;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const s16x4 lo = tr_read(vc + ((dt ^ vx) << 5));
          const s16x4 hi = tr_read(vc + 16 * 128 + ((dt ^ vx) << 5));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 v8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          const bf16x8 vf = __builtin_bit_cast(bf16x8, v8);
#pragma unroll
          for (int u = 0; u < TT; ++u) o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[u], o[u][dt], 0, 0, 0);
        }
      }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using BF = std::integral_constant<bool, false>;
    using BT = std::integral_constant<bool, true>;
    for (int c = 0; c < nch - 1; ++c) chunk(I4{}, BF{}, c);
    {
      const int c = nch - 1;
      if (last_kvalid > 48) chunk(I4{}, BT{}, c);
      else if (last_kvalid > 32) chunk(I3{}, BT{}, c);
      else if (last_kvalid > 16) chunk(I2{}, BT{}, c);
      else chunk(I1{}, BT{}, c);
    }

#pragma unroll
    for (int u = 0; u < TT; ++u) {
      float lt = l[u];
      {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
        lt = __uint_as_float(a[0]) + __uint_as_float(a[1]);
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
        lt = __uint_as_float(b[0]) + __uint_as_float(b[1]);
      }
      const float inv = 1.0f / lt;
      const int qrow = tq[u] * 16 + fr;
      // o[u][dt][j]: query qrow, head dim dt*16 + 4g + j
      if (q8) {  // MX-fp8 output: this head's 64 dims are one 64-k block of out_proj
        float amax = 0.f;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fabsf(o[u][dt][j] * inv));
        amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        const int X = mx_block_exp(amax);
        const float scl = ldexpf(1.0f, -X);
        if (qrow < S) {
          const int64_t row = (int64_t)bseq * S + qrow;
          uint8_t* dst = q8 + row * W + h * 64 + 4 * g;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            *(uint32_t*)(dst + dt * 16) =
                mx_pack4(o[u][dt][0] * inv, o[u][dt][1] * inv, o[u][dt][2] * inv, o[u][dt][3] * inv, scl);
          if (g == 0) qs[mx_scale_index(row, h, rows_pad)] = (uint8_t)(X + 127);
        }
        continue;
      }
      if (qrow < S) {
        uint16_t* dst = out + ((int64_t)bseq * S + qrow) * W + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          *(uint2*)(dst + dt * 16) = make_uint2(pack_bf16x2(o[u][dt][0] * inv, o[u][dt][1] * inv),
                                                pack_bf16x2(o[u][dt][2] * inv, o[u][dt][3] * inv));
      }
    }
  };
  // SPLIT: the last tile's rows over this wave's key tiles, partial states to LDS (SFIRST: before the
  // full tiles, so every wave reaches the merge barrier with the same work behind it)
  auto split_part = [&]() __attribute__((always_inline)) {
    // the last query tile (rows 16 (nqt - 1) .. S - 1, vr <= 16 of them) over this wave's
    // 16-key tiles; the same arithmetic as chunk() per key tile (log2-domain online softmax)
    const int tl = nqt - 1, vr = S - 16 * tl;
    const int nkt = (S + 15) / 16;
    bf16x8 qf[2];
    {
      const int qrow = min(tl * 16 + fr, S - 1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) qf[s2] = *(const bf16x8*)(qb + (int64_t)qrow * ld + 32 * s2 + 8 * g);
    }
    float m = -INFINITY, l = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = wave; kt < nkt; kt += NW) {
      const int kb = kt * 16;
      const bf16x8 k0 = *(const bf16x8*)(Kimg + kb * 128 + rk0);
      const bf16x8 k1 = *(const bf16x8*)(Kimg + kb * 128 + rk1);
      f32x4 sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[1], sc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (kb + 4 * g + j >= S) sc[j] = -INFINITY;
      float cm = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
      {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
        cm = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
      }
      const float cmu = cm * sl2;   // finite: key tile kb < S holds key kb
      if (cmu > m + RESCALE) {
        const float alpha = __builtin_amdgcn_exp2f(m - cmu);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        m = cmu;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) sc[j] = __builtin_amdgcn_exp2f(fmaf(sc[j], sl2, -m));
      l += (sc[0] + sc[1]) + (sc[2] + sc[3]);
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (__bf16)sc[j];
        pb[4 + j] = (__bf16)0.f;
      }
      const char* vc = Vimg + kb * 128 + rvb;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x4 lo = tr_read(vc + ((dt ^ vx) << 5));
        const s16x4 hi = tr_read(vc + 16 * 128 + ((dt ^ vx) << 5));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, v8), pb, o[dt], 0, 0, 0);
      }
    }
    float lt = l;
    {
      const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
      lt = __uint_as_float(a[0]) + __uint_as_float(a[1]);
      const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
      lt = __uint_as_float(b[0]) + __uint_as_float(b[1]);
    }
    // partial states of the valid rows: [wave][row][m, l, o 0..63] after the K / V images
    float* part = (float*)(res_lds + 2 * spad * 128);
    if (fr < vr) {
      float* pw = part + (wave * vr + fr) * 68;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) pw[4 + dt * 16 + 4 * g + j] = o[dt][j];
      if (g == 0) {
        pw[0] = m;
        pw[1] = lt;
      }
    }
  };
  if (SPLIT && SFIRST) split_part();
  const int nfull = SPLIT ? nqt - 1 : nqt;   // SPLIT: the last tile is shared out below
  for (int t = wave; t < nfull; t += 2 * NW) {
    if (TT2 && t + NW < nfull) tiles(std::integral_constant<int, 2>{}, t, t + NW);
    else {
      tiles(std::integral_constant<int, 1>{}, t, t);
      if (!TT2 && t + NW < nfull) tiles(std::integral_constant<int, 1>{}, t + NW, t + NW);
    }
  }
  if (SPLIT && !SFIRST) split_part();
  if (SPLIT) {
    const int tl = nqt - 1, vr = S - 16 * tl;
    float* part = (float*)(res_lds + 2 * spad * 128);
    __syncthreads();
    if (wave == 0 && fr < vr) {
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < NW; ++w) M = fmaxf(M, part[(w * vr + fr) * 68]);
      float L = 0.f;
      f32x4 O[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) O[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float* pw = part + (w * vr + fr) * 68;
        const float sw = pw[0] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(pw[0] - M);
        L += pw[1] * sw;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int j = 0; j < 4; ++j) O[dt][j] += pw[4 + dt * 16 + 4 * g + j] * sw;
      }
      const float inv = 1.0f / L;
      const int qrow = tl * 16 + fr;
      if (q8) {   // never taken: the MX tower's attention runs the 32x32 kernel (SPLIT is bf16 only)
      } else {
        uint16_t* dst = out + ((int64_t)bseq * S + qrow) * W + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          *(uint2*)(dst + dt * 16) = make_uint2(pack_bf16x2(O[dt][0] * inv, O[dt][1] * inv),
                                                pack_bf16x2(O[dt][2] * inv, O[dt][3] * inv));
      }
    }
  }
}

// ------------- attention, vision towers: K/V resident in LDS, 32x32x16 MFMAs
// Same work split and LDS residency as attention_res_kernel, on the 32 x 32
// MFMA shape, whose 32 cycles hold the SIMD's issue for 8 (the 16 x 16 shape
// holds 8 of 16), so the softmax VALU of the other wave on the SIMD finds
// twice the issue slots beside the matrix pipe.  Per wave: query blocks of 32
// rows (two at a time, sharing every K / V^T fragment read), 64-key chunks.
//   S^T = K Q^T : K is the A operand (lane: key r, 8 dims of k-step s at
//     chunk 2s + half), Q^T the B operand held in registers for the block;
//     the result X[key][query] has the query on the lane (r = lane & 31) and
//     16 keys per lane half in registers: key (reg & 3) + 8 (reg >> 2) + 4 half;
//   softmax in the log2 domain with the lazy rescale of the kernels above;
//     a row's max over 64 keys is 32 in-lane values and one permlane32 swap;
//   O^T = V^T P^T : X's registers 8s .. 8s + 7, packed to bf16, ARE the B
//     operand of k-step s (the MFMA's k order inside a step is key
//     16s + 8(j >> 2) + 4 half + (j & 3) for element j), so P never leaves the
//     lane; V^T is the A operand, read transposed (ds_read_b64_tr_b16) in that
//     same key order: two reads of 4 keys x 16 dims per 16-lane group.
//   K image : 16-byte chunk c of key row r at slot c ^ ((r >> 1) & 7) (a
//             16-lane group of the A-operand read covers all 64 banks);
//   V image : chunk c of row r at slot c ^ (((r >> 1) & 1) << 2): the four rows
//             of a transposed read (r0 .. r0 + 3, r0 % 4 == 0) put their 64
//             bytes in four disjoint quarter-banks.
// s_waitcnt vmcnt(n) for a wave-uniform n in [0, N] (the count is an immediate)
template <int N>
__device__ __forceinline__ void vm_wait_younger(int n) {
  if constexpr (N > 0) {
    if (n >= N) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
      return;
    }
    vm_wait_younger<N - 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// ABL (A/B timing probes only): 1 = no exponentials, 2 = no K/V DMA, 3 = no softmax VALU.
// PH2: the K/V load in two phases, keys [0, 64 c0) (c0 = spad / 128 chunks) first; the wave's first query
// block, its Q loaded ahead of the DMAs, starts on the first phase's keys after one
// barrier and takes a second barrier (vmcnt(0)) before chunk c0, so the second half of
// the 148 KB load (S = 577) arrives under the first half's math instead of before it.
template <int NW, bool TT2 = true, int ABL = 0, bool PH2 = false>
__global__ __launch_bounds__(NW * 64) void attention_r32_kernel(const uint16_t* __restrict__ qkv,
                                                                uint16_t* __restrict__ out, int S, int W, int H,
                                                                uint8_t* __restrict__ q8, uint8_t* __restrict__ qs,
                                                                int64_t rows_pad, int stagger_ticks) {
  extern __shared__ __attribute__((aligned(16))) char r32_lds[];
  const int spad = (S + 31) & ~31;
  char* Kimg = r32_lds;
  char* Vimg = r32_lds + spad * 128;
  const int item = blockIdx.x;
  const int bseq = item / H, head = item % H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ld = 3 * (int64_t)W;
  const uint16_t* qb = qkv + (int64_t)bseq * S * ld + head * 64;
  const uint16_t* kb = qb + W;
  const uint16_t* vb = qb + 2 * W;

  // ---- K, V -> LDS (one DMA instruction = 8 rows; rows >= S clamped copies)
  // The first workgroups on the CUs start together and, all taking the same
  // time, would keep issuing their K/V loads (148 KB each at S = 577) in
  // chip-wide bursts; a start delay of 0-3 quarters of a workgroup's time on
  // the first workgroup of each CU spreads them out for the rest of the grid.
  if (stagger_ticks > 0 && (int)blockIdx.x < 256) {
    const int ph = (blockIdx.x >> 3) & 3;
    if (ph) {
      const uint64_t until = __builtin_amdgcn_s_memrealtime() + (uint64_t)ph * stagger_ticks;
      while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(8);
    }
  }
  const int nch = (S + 63) >> 6;
  const int nr8 = spad >> 3;
  const int c0 = PH2 ? max(1, nr8 >> 4) : nch;   // chunks of the first load phase (nr8 >= 12 for S > 64)
  static_assert(!PH2 || (NW == 12 && !TT2), "attention_r32: the two-phase load's slot count assumes 12 waves");
  // NI2 (below) x 12 waves >= 2 nr8 for spad <= 640
  bf16x8 qf0[4];
  if (PH2) {   // the first block's Q, ahead of the DMAs: waiting for it drains none of them
    const int qrow = min(wave * 32 + (lane & 31), S - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) qf0[s] = *(const bf16x8*)(qb + (int64_t)qrow * ld + 16 * s + 8 * (lane >> 5));
  }
  // PH2: NI2 DMA slots per wave in global order g = wave + 12 k, so each wave issues its
  // first-phase blocks (g < 2 h0: K then V blocks of keys < 64 c0) before its second-phase
  // ones; slots past the 2 nr8 blocks re-load the last block (identical bytes, same place)
  constexpr int NI2 = 14;
  const int h0 = 8 * c0;
  if (ABL != 2 && PH2) {
    const int slot = lane & 7;
    const int n1 = nr8 - h0;
#pragma unroll
    for (int k = 0; k < NI2; ++k) {
      const int g = min(wave + NW * k, 2 * nr8 - 1);
      const bool ph = g >= 2 * h0;
      const int j = ph ? g - 2 * h0 : g, cnt = ph ? n1 : h0;
      const bool isv = j >= cnt;
      const int i8 = (ph ? h0 : 0) + (isv ? j - cnt : j);
      const int rr = i8 * 8 + (lane >> 3);
      const int cc = isv ? (slot ^ (((rr >> 1) & 1) << 2)) : (slot ^ ((rr >> 1) & 7));
      glds16((isv ? vb : kb) + (int64_t)min(rr, S - 1) * ld + cc * 8, (isv ? Vimg : Kimg) + i8 * 1024);
    }
  }
  if (ABL != 2 && !PH2) {
    const int slot = lane & 7;
    for (int i = wave; i < 2 * nr8; i += NW) {
      const bool isv = i >= nr8;
      const int i8 = isv ? i - nr8 : i;
      const int rr = i8 * 8 + (lane >> 3);
      const int cc = isv ? (slot ^ (((rr >> 1) & 1) << 2)) : (slot ^ ((rr >> 1) & 7));
      glds16((isv ? vb : kb) + (int64_t)min(rr, S - 1) * ld + cc * 8, (isv ? Vimg : Kimg) + i8 * 1024);
    }
  }

  const int r = lane & 31, hh = lane >> 5;
  const int ksw = (r >> 1) & 7;
  // transposed V^T reads: lane 4q + p of each 16-lane group gives row q
  // (key 4 half + q of the 8-key half-step), dims 16 g + 4p .. + 3 of the
  // 32-dim block
  const int i16 = lane & 15, gq = (lane >> 4) & 1, tq = i16 >> 2, tp = i16 & 3;
  const int vrow = (4 * hh + tq) * 128 + 8 * (tp & 1);
  const int vof0 = vrow + 16 * ((0 + 2 * gq + (tp >> 1)) ^ ((tq >> 1) << 2));
  const int vof1 = vrow + 16 * ((4 + 2 * gq + (tp >> 1)) ^ ((tq >> 1) << 2));
  const float sl2 = 0.125f * 1.4426950408889634f;   // head_dim^-0.5 * log2(e)
  constexpr float RESCALE = 8.0f;
  const int nqb = (S + 31) >> 5;
  const int last_keys = S - (nch - 1) * 64;   // 1..64
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  auto tr_read = [&](const char* p) -> s16x4 {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(LDS_AS char*)(uintptr_t)(const LDS_AS char*)p);
  };
  auto vfrag = [&](const char* p) -> bf16x8 {
    const s16x4 lo = tr_read(p);
    const s16x4 hi = tr_read(p + 8 * 128);
    return __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  if (PH2) {   // this wave's first-phase DMAs (and Q): the NI2 - n0 younger ones may stay in flight
    const int n0 = 2 * h0 > wave ? (2 * h0 - wave + NW - 1) / NW : 0;
    vm_wait_younger<NI2>(NI2 - min(n0, NI2));
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  auto blocks = [&](auto tt_c, int b0, int b1, bool first) {
    constexpr int TT = decltype(tt_c)::value;
    const int bq[2] = {b0, b1};
    bf16x8 qf[TT][4];
#pragma unroll
    for (int u = 0; u < TT; ++u) {
      const int qrow = min(bq[u] * 32 + r, S - 1);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        qf[u][s] = PH2 && first ? qf0[s] : *(const bf16x8*)(qb + (int64_t)qrow * ld + 16 * s + 8 * hh);
    }
    float m[TT], l[TT];
    f32x16 o[TT][2];
#pragma unroll
    for (int u = 0; u < TT; ++u) {
      m[u] = -INFINITY;
      l[u] = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) o[u][0][i] = o[u][1][i] = 0.f;
    }

    // one 64-key chunk: NKB valid 32-key blocks, MASK: keys >= S inside them
    auto chunk = [&](auto nkb_c, auto mask_c, int c) {
      constexpr int NKB = decltype(nkb_c)::value;
      constexpr bool MASK = decltype(mask_c)::value;
      f32x16 x[TT][NKB];
#pragma unroll
      for (int kt = 0; kt < NKB; ++kt) {
        const char* kp = Kimg + (c * 64 + kt * 32 + r) * 128;
        bf16x8 kf[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) kf[s] = *(const bf16x8*)(kp + 16 * ((2 * s + hh) ^ ksw));
#pragma unroll
        for (int u = 0; u < TT; ++u) {
          f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[0], qf[u][0], f32x16{}, 0, 0, 0);
#pragma unroll
          for (int s = 1; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s], qf[u][s], acc, 0, 0, 0);
          x[u][kt] = acc;
        }
      }
#pragma unroll
      for (int u = 0; u < TT && ABL != 3; ++u) {
        if (MASK) {
#pragma unroll
          for (int kt = 0; kt < NKB; ++kt)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (c * 64 + kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh >= S) x[u][kt][i] = -INFINITY;
        }
        float cm = x[u][0][0];
#pragma unroll
        for (int kt = 0; kt < NKB; ++kt)
#pragma unroll
          for (int i = (kt ? 0 : 1); i < 16; ++i) cm = fmaxf(cm, x[u][kt][i]);
        {
          const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(cm), __float_as_uint(cm), false, false);
          cm = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
        }
        const float cmu = cm * sl2;   // finite: chunk 0 holds key 0 for every row
        if (cmu > m[u] + RESCALE) {
          const float alpha = __builtin_amdgcn_exp2f(m[u] - cmu);
          l[u] *= alpha;
          o[u][0] *= alpha;
          o[u][1] *= alpha;
          m[u] = cmu;
        }
        float ps = 0.f;
#pragma unroll
        for (int kt = 0; kt < NKB; ++kt) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            x[u][kt][i] = ABL == 1 ? fmaf(x[u][kt][i], sl2, -m[u]) : __builtin_amdgcn_exp2f(fmaf(x[u][kt][i], sl2, -m[u]));
#pragma unroll
          for (int i = 0; i < 16; i += 4) ps += (x[u][kt][i] + x[u][kt][i + 1]) + (x[u][kt][i + 2] + x[u][kt][i + 3]);
        }
        l[u] += ps;
      }
#pragma unroll
      for (int kt = 0; kt < NKB; ++kt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const char* vp = Vimg + (c * 64 + kt * 32 + 16 * s) * 128;
          const bf16x8 v0 = vfrag(vp + vof0);
          const bf16x8 v1 = vfrag(vp + vof1);
#pragma unroll
          for (int u = 0; u < TT; ++u) {
            uint32_t pk[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) pk[j] = pack_bf16x2(x[u][kt][8 * s + 2 * j], x[u][kt][8 * s + 2 * j + 1]);
            typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
            const bf16x8 pb = __builtin_bit_cast(bf16x8, (u32x4_t){pk[0], pk[1], pk[2], pk[3]});
            o[u][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v0, pb, o[u][0], 0, 0, 0);
            o[u][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v1, pb, o[u][1], 0, 0, 0);
          }
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using BF = std::integral_constant<bool, false>;
    using BT = std::integral_constant<bool, true>;
    for (int c = 0; c < nch - 1; ++c) {
      if (PH2 && first && c == c0) {   // the second load phase (every wave passes here once)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      chunk(I2{}, BF{}, c);
    }
    if (PH2 && first && c0 >= nch - 1) {   // short sequences: the second phase before the last chunk
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (last_keys > 32) chunk(I2{}, BT{}, nch - 1);
    else chunk(I1{}, BT{}, nch - 1);

#pragma unroll
    for (int u = 0; u < TT; ++u) {
      float lt = l[u];
      {
        const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
        lt = __uint_as_float(b[0]) + __uint_as_float(b[1]);
      }
      const float inv = 1.0f / lt;
      const int qrow = bq[u] * 32 + r;
      // o[u][db][i]: query qrow, head dim 32 db + (i & 3) + 8 (i >> 2) + 4 hh
      if (q8) {   // MX-fp8 output: this head's 64 dims are one 64-k block of out_proj
        float amax = 0.f;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) amax = fmaxf(amax, fabsf(o[u][db][i] * inv));
        {
          const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
          amax = fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
        }
        const int X = mx_block_exp(amax);
        const float scl = ldexpf(1.0f, -X);
        if (qrow < S) {
          const int64_t row = (int64_t)bseq * S + qrow;
          uint8_t* dst = q8 + row * W + head * 64 + 4 * hh;
#pragma unroll
          for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int t = 0; t < 4; ++t)
              *(uint32_t*)(dst + 32 * db + 8 * t) = mx_pack4(o[u][db][4 * t] * inv, o[u][db][4 * t + 1] * inv,
                                                             o[u][db][4 * t + 2] * inv, o[u][db][4 * t + 3] * inv, scl);
          if (hh == 0) qs[mx_scale_index(row, head, rows_pad)] = (uint8_t)(X + 127);
        }
        continue;
      }
      if (qrow < S) {
        uint16_t* dst = out + ((int64_t)bseq * S + qrow) * W + head * 64 + 4 * hh;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            *(uint2*)(dst + 32 * db + 8 * t) = make_uint2(pack_bf16x2(o[u][db][4 * t] * inv, o[u][db][4 * t + 1] * inv),
                                                          pack_bf16x2(o[u][db][4 * t + 2] * inv, o[u][db][4 * t + 3] * inv));
      }
    }
  };
  if (TT2) {
    for (int b = wave; b < nqb; b += 2 * NW) {
      if (b + NW < nqb) blocks(std::integral_constant<int, 2>{}, b, b + NW, false);
      else blocks(std::integral_constant<int, 1>{}, b, b, false);
    }
  } else {
    if (PH2 && wave >= nqb) {   // no block: the second phase's barrier all the same
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int b = wave; b < nqb; b += NW) blocks(std::integral_constant<int, 1>{}, b, b, b == wave);
  }
}

}  // namespace

hipError_t attention(const uint16_t* qkv, uint16_t* out, int B, int S, int W, int causal, hipStream_t s, uint8_t* q8,
                     uint8_t* qs) {
  const int H = W / 64;
  const int items = B * H;
  if (items <= 0) return hipSuccess;
  if (S > 640) return hipErrorInvalidValue;
  // Every length runs attention_flash_kernel (scripts/attn_micro.py, this
  // round: B/32 S=50 177 vs 181 us for the one-wave kernel, text S=77 25.9 vs
  // 30.0, L/14 408 vs 572 and L/14@336 547 vs 1004 for the per-query-tile-K
  // kernel it replaced).  Causal bit 8 selects the one-wave kernel for S <= 96
  // (A/B and parity tests of both paths; it has no fp8 output).
#if MICLIP_AB
  const bool one_wave = ((causal >> 8) & 1) && S <= 96 && !q8;
#else
  if ((causal >> 8) & 1) return hipErrorNotSupported;   // the one-wave kernel is in the A/B build only
  constexpr bool one_wave = false;
#endif
  const bool old_flash = (causal >> 9) & 1;   // A/B: the chunk-streaming flash kernel for S > 64
  const int q0only = (causal >> 11) & 1;      // the first query tile only (S <= 64 kernel; others compute all)
  causal &= 1;
  const dim3 grid(items);
#if MICLIP_AB
  // A/B: MICLIP_ATTN_SHORT=1 runs S <= 64 (non-causal) on the resident-K/V kernel with 4 waves
  const char* se = std::getenv("MICLIP_ATTN_SHORT");
  // 5x: persistent workgroups with the next item's operands prefetched, x workgroups per CU (default 4:
  // 128 VGPRs)
  if (se && se[0] == '5' && !one_wave && !old_flash && S <= 64) {
    const int per = se[1] ? std::atoi(se + 1) : 4;
    const int gp = std::min(items, cu_count() * (per > 0 ? per : 5));
    hipLaunchKernelGGL(attention_pipe_kernel, dim3(gp), dim3(256), 0, s, qkv, out, S, W, H, causal, q8, qs,
                       ((int64_t)B * S + 1) & ~1, items);
    return hipGetLastError();
  }
  // 6: the V^T fragment reads batched (attention_vb_kernel)
  if (se && se[0] == '6' && !one_wave && !old_flash && S <= 64) {
    hipLaunchKernelGGL(attention_vb_kernel, grid, dim3(256), 0, s, qkv, out, S, W, H, causal | (q0only << 11), q8, qs,
                       ((int64_t)B * S + 1) & ~1);
    return hipGetLastError();
  }
  // 2: two heads per workgroup; 3: the occupancy-targeted single-head kernel
  if (se && (se[0] == '2' || se[0] == '3') && !one_wave && !old_flash && S <= 64) {
    if (se[0] == '2' && H % 2 == 0)
      hipLaunchKernelGGL(attention_short2_kernel, dim3(items / 2), dim3(512), 0, s, qkv, out, S, W, H, causal, q8, qs,
                         ((int64_t)B * S + 1) & ~1);
    else
      hipLaunchKernelGGL(attention_short_kernel, grid, dim3(256), 0, s, qkv, out, S, W, H, causal, q8, qs,
                         ((int64_t)B * S + 1) & ~1);
    return hipGetLastError();
  }
  if (se && se[0] == '1' && !one_wave && !old_flash && !(causal & 1) && S <= 64) {
    const size_t lds = 2 * (size_t)((S + 31) & ~31) * 128;
    hipLaunchKernelGGL((attention_res_kernel<4, false>), dim3(B * (W / 64)), dim3(256), lds, s, qkv, out, S, W, W / 64,
                       q8, qs, ((int64_t)B * S + 1) & ~1);
    return hipGetLastError();
  }
#endif
  if (!one_wave && !old_flash && !causal && S > 64) {
    // vision towers (257 / 577 tokens): K/V resident in LDS, no per-chunk barriers
    const int spad = (S + 31) & ~31;
    const size_t lds = 2 * (size_t)spad * 128;
    // Defaults (scripts/attn_micro.py, r03): S <= 320 (L/14, 257 tokens) attention_res_kernel
    // with 8 waves, one 16-row query tile at a time; S > 320 (L/14@336, 577 tokens) the
    // 32x32x16 kernel with 12 waves, one 32-row block each (2157 us per 1000-frame chunk
    // against 2392 for attention_res_kernel).  A/B variants (MICLIP_ATTN_VAR): 1 res 8 waves
    // x 1 tile, 2 res 8 waves x 2 tiles, 3 res 16 waves, 4 r32 8 waves x 2 blocks, 5 r32
    // 12 waves, 6 / 7 r32 12 waves with a start stagger of 1 / 2 quarter workgroup times,
    // 8 / 9 r32 timing probes (no K/V load / no exponentials: wrong results), 10 r32 12 waves
    // with the two-phase K/V load
#if MICLIP_AB
    const char* ve = std::getenv("MICLIP_ATTN_VAR");   // A/B
    int var = ve ? std::atoi(ve) : 0;
#else
    int var = 0;
#endif
    if (var < 1 || var > 14) var = S > 320 ? 5 : 1;
    const int64_t rp = ((int64_t)B * S + 1) & ~1;
    auto set_lds = [&](const void* fn, int slot) -> hipError_t {
      static bool attr_set[13] = {false, false, false, false, false, false, false, false, false, false, false, false, false};
      if (attr_set[slot]) return hipSuccess;
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e == hipSuccess) attr_set[slot] = true;
      return e;
    };
    hipError_t e = hipSuccess;
#define ATT_LAUNCH(SLOT, KERNEL, THREADS, ...)                                  \
  {                                                                             \
    if ((e = set_lds((const void*)KERNEL, SLOT)) != hipSuccess) return e;       \
    hipLaunchKernelGGL(KERNEL, grid, dim3(THREADS), lds, s, __VA_ARGS__);       \
  }
#if MICLIP_AB
    // A/B variant 12: the nearly empty last query tile (S % 16 in 1..4, bf16 output) split over
    // the 8 waves' key tiles (attention_res_kernel SPLIT).  Measured at L/14 (scripts/attn_micro.py,
    // r04): 1074 vs 1031 us per 1667-frame chunk -- the second workgroup on the CU already fills
    // the idle waves -- so the unsplit kernel stays the default.  Variant 11 = variant 1.
    const int vr = S - 16 * ((S + 15) / 16 - 1);
    if (var == 12 && vr <= 4 && !q8) {
      const size_t lds_s = lds + (size_t)8 * vr * 68 * 4;
      if ((e = set_lds((const void*)attention_res_kernel<8, false, true>, 0)) != hipSuccess) return e;
      hipLaunchKernelGGL((attention_res_kernel<8, false, true>), grid, dim3(512), lds_s, s, qkv, out, S, W, H, q8, qs,
                         rp);
      return hipGetLastError();
    }
    if (var == 13 && vr <= 4 && !q8) {   // A/B: the split tile first, then the full tiles, then the merge
      const size_t lds_s = lds + (size_t)8 * vr * 68 * 4;
      if ((e = set_lds((const void*)attention_res_kernel<8, false, true, true>, 11)) != hipSuccess) return e;
      hipLaunchKernelGGL((attention_res_kernel<8, false, true, true>), grid, dim3(512), lds_s, s, qkv, out, S, W, H, q8,
                         qs, rp);
      return hipGetLastError();
    }
    if (var == 14) {   // A/B: Q fragments one tile ahead
      if ((e = set_lds((const void*)attention_res_kernel<8, false, false, false, true>, 12)) != hipSuccess) return e;
      hipLaunchKernelGGL((attention_res_kernel<8, false, false, false, true>), grid, dim3(512), lds, s, qkv, out, S, W,
                         H, q8, qs, rp);
      return hipGetLastError();
    }
#endif
    if (var == 11 || var == 12 || var == 13) var = 1;
    if (var == 1) ATT_LAUNCH(1, (attention_res_kernel<8, false>), 512, qkv, out, S, W, H, q8, qs, rp)
    else if (var == 5) ATT_LAUNCH(5, (attention_r32_kernel<12, false>), 768, qkv, out, S, W, H, q8, qs, rp, 0)
#if MICLIP_AB
    else if (var == 2) ATT_LAUNCH(2, (attention_res_kernel<8, true>), 512, qkv, out, S, W, H, q8, qs, rp)
    else if (var == 3) ATT_LAUNCH(3, (attention_res_kernel<16, false>), 1024, qkv, out, S, W, H, q8, qs, rp)
    else if (var == 4) ATT_LAUNCH(4, (attention_r32_kernel<8, true>), 512, qkv, out, S, W, H, q8, qs, rp, 0)
    else if (var == 6 || var == 7)
      ATT_LAUNCH(var, (attention_r32_kernel<12, false>), 768, qkv, out, S, W, H, q8, qs, rp, (var - 5) * (S * S / 378))
    else if (var == 8) ATT_LAUNCH(8, (attention_r32_kernel<12, false, 2>), 768, qkv, out, S, W, H, q8, qs, rp, 0)
    else if (var == 10) ATT_LAUNCH(10, (attention_r32_kernel<12, false, 0, true>), 768, qkv, out, S, W, H, q8, qs, rp, 0)
    else ATT_LAUNCH(9, (attention_r32_kernel<12, false, 1>), 768, qkv, out, S, W, H, q8, qs, rp, 0)
#else
    else return hipErrorNotSupported;
#endif
#undef ATT_LAUNCH
    return hipGetLastError();
  }
#if MICLIP_AB
  if (one_wave) {
    if (S <= 32) hipLaunchKernelGGL(attention_kernel<32>, grid, dim3(64), 0, s, qkv, out, S, W, H, causal, items);
    else if (S <= 64) hipLaunchKernelGGL(attention_kernel<64>, grid, dim3(64), 0, s, qkv, out, S, W, H, causal, items);
    else hipLaunchKernelGGL(attention_kernel<96>, grid, dim3(64), 0, s, qkv, out, S, W, H, causal, items);
    return hipGetLastError();
  }
#endif
  // NT = ceil(tiles / 8) query tiles per wave on 8 waves; S <= 64: one tile on
  // each of 4 waves, single slot.  Fewer waves with fewer idle tile slots
  // measured slower (L/14 257 tokens on 6 waves x 3 tiles: 470 vs 421 us; text
  // 77 on 5 x 1: 45 vs 31 us): a workgroup lasts as long as its busiest wave
  // either way, and 8 waves spread that wave's SIMD over fewer partners.
  const int nqt = (S + 15) / 16;
  const int64_t rp = ((int64_t)B * S + 1) & ~1;
#define FLASH(T) \
  hipLaunchKernelGGL((attention_flash_kernel<T, 1>), grid, dim3(512), 0, s, qkv, out, S, W, H, causal, q8, qs, rp)
  if (nqt <= 4)
    hipLaunchKernelGGL((attention_flash_kernel<1, 2, 1>), grid, dim3(256), 0, s, qkv, out, S, W, H, causal | (q0only << 11),
                       q8, qs, rp);
  else if (nqt <= 8) FLASH(1);
  else if (nqt <= 16) FLASH(2);
  else if (nqt <= 24) FLASH(3);
  else if (nqt <= 32) FLASH(4);
  else FLASH(5);
#undef FLASH
  return hipGetLastError();
}

}  // namespace miclip
