// Baseline JPEG decode on the GPU (gfx950), bit-exact to Pillow's decoder —
// the decode step of the reference's frame ingest
//   Image.open(path).convert("RGB")        embedding_service.py:472-480, embedding.py:46
// (SURVEY.md §8(f) item 1).  Pillow hands YCbCr JPEGs to libjpeg(-turbo) with
// its defaults (JDCT_ISLOW, fancy upsampling, JCS_RGB output), so the three
// kernels below restate those integer algorithms:
//   jpeg_entropy_kernel  one lane per frame (or per restart interval):
//                        sequential Huffman decode of the interleaved scan
//                        (tables in LDS, stream words prefetched), DC
//                        prediction, de-zigzag -> int16 coefficients;
//   jpeg_idct_kernel     one thread per 8x8 block: dequantise + the
//                        LL&M integer IDCT of jidctint.c (CONST_BITS 13,
//                        PASS1_BITS 2) with its 1024-entry range-limit
//                        wrap -> uint8 component planes;
//   jpeg_color_kernel    one thread per output pixel: h2v1 / h2v2 "fancy"
//                        triangular chroma upsampling (jdsample.c, edge rows
//                        and columns replicated as libjpeg's context rows do)
//                        and the fixed-point YCbCr -> RGB of jdcolor.c.
// The host (miclip/jpeg.py) parses the headers, builds the Huffman look-up
// tables and batches frames of one geometry; progressive / arithmetic /
// 12-bit / CMYK / other sampling layouts stay on the host decoder.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "internal.hpp"
#include "miclip.h"

namespace miclip {
namespace {

__constant__ uint8_t kZigzag[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    // extra entries so a corrupt run past 63 lands in position 63 (libjpeg's jpeg_natural_order + 16)
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// One decode table (JpegHuff, host-built, libjpeg d_derived_tbl layout):
//   look[512]: (length << 8) | symbol for codes of <= 9 bits (0: longer code)
//   maxcode[18]: largest code of each length (-1 none; [17] sentinel)
//   valoff[18]: values index offset per length (value = vals[code + valoff[l]])
//   vals[256]
//   l2base, l2n, look2[1024]: (length << 8) | symbol for the 16-bit windows
//     [l2base, l2base + l2n) of the 10..16-bit codes (0: corrupt); l2n = 0: walk maxcode
struct JpegHuff {
  uint16_t look[512];
  int32_t maxcode[18];
  int32_t valoff[18];
  uint8_t vals[256];
  int32_t l2base, l2n;
  uint16_t look2[1024];
};
static_assert(sizeof(JpegHuff) == MI_JPEG_HUFF_BYTES, "table layout shared with miclip/jpeg.py");

// Entropy-coded bytes of one segment as a left-aligned bit buffer.  A lane
// decodes its frame serially, and a wave waits on a load for all its lanes
// (and, vmcnt being in order, for every coefficient store issued before it).
// So raw bytes come from a per-lane queue of up to 64 bytes in registers that
// the WHOLE wave tops up at once (refill(): every lane loads as many aligned
// 16-byte blocks as fit, all issued before the one wait) when any lane runs
// low: one memory wait per ~40 bytes of the fastest lane instead of one per
// byte.  Un-stuffing happens in registers; at a marker or the segment end it
// feeds zeros (libjpeg's "insufficient data" behaviour).
struct BitReader {
  static constexpr int QW = 16, QB = 4 * QW;   // queue: 16 dwords = 64 bytes
  static constexpr int LOW = 12;   // a trip reads <= 9 raw bytes (<= 4 data bytes, stuffed, + a marker peek)
  // (the queue then always holds the 4 bytes the dword path reads when rem >= 4)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* fp;         // next aligned 16-byte block to load
  const u32x4* flast;      // last block holding segment bytes (loads clamp to it)
  uint32_t q[QW];          // raw byte queue, stream order from q[0]'s top byte
  int nq;                  // bytes in the queue
  int64_t rem;             // unread segment bytes
  uint64_t buf;            // left-aligned bit buffer
  int nbits;
  bool marker;             // hit a marker: feed zeros

  __device__ __forceinline__ u32x4 load_block() {
    typedef __attribute__((address_space(1))) const u32x4 gu4;
    const u32x4 v = *(gu4*)(fp < flast ? fp : flast);
    ++fp;
    return v;
  }
  // append 16 bytes (memory order) at byte position nq (nq <= QB - 16)
  __device__ __forceinline__ void append(u32x4 v) {
    const uint32_t a[4] = {__builtin_bswap32(v[0]), __builtin_bswap32(v[1]), __builtin_bswap32(v[2]),
                           __builtin_bswap32(v[3])};
    const int ws = nq >> 2, bs = (nq & 3) * 8;
    uint32_t t[5];
    t[0] = a[0] >> bs;
#pragma unroll
    for (int j = 1; j < 4; ++j) t[j] = (a[j] >> bs) | (bs ? a[j - 1] << (32 - bs) : 0u);
    t[4] = bs ? a[3] << (32 - bs) : 0u;
#pragma unroll
    for (int i = 0; i < QW; ++i) {
      uint32_t x = 0;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (i - j >= 0 && i - j <= QW - 4) x |= (ws == i - j) ? t[j] : 0u;
      q[i] |= x;
    }
    nq += 16;
  }
  __device__ __forceinline__ void init(const uint8_t* p, const uint8_t* end) {
    buf = 0;
    nbits = 0;
    marker = false;
    rem = end - p;
#pragma unroll
    for (int i = 0; i < QW; ++i) q[i] = 0;
    nq = 0;
    if (rem <= 0) {
      rem = 0;
      fp = flast = nullptr;
      return;
    }
    const int sh = (int)((uintptr_t)p & 15);
    fp = (const u32x4*)((uintptr_t)p - sh);
    flast = (const u32x4*)(((uintptr_t)end - 1) & ~(uintptr_t)15);
    const u32x4 v0 = load_block(), v1 = load_block();
    append(v0);
    append(v1);
    // drop the sh bytes before p: whole dwords, then the byte remainder
    const int dw = sh >> 2, bs = (sh & 3) * 8;
#pragma unroll
    for (int i = 0; i < QW; ++i) {
      uint32_t x = q[i];
#pragma unroll
      for (int d = 1; d < 4; ++d) x = (dw == d) ? (i + d < QW ? q[i + d] : 0u) : x;
      q[i] = x;   // in place is safe: q[i + d] is read before it is written (increasing i)
    }
    if (bs) {
#pragma unroll
      for (int i = 0; i < QW; ++i) q[i] = (q[i] << bs) | (i + 1 < QW ? q[i + 1] >> (32 - bs) : 0u);
    }
    nq = 32 - sh;
  }
  __device__ __forceinline__ bool low() const { return nq < LOW && rem > nq; }
  __device__ __forceinline__ void refill() {
    // the loads first (independent), then the appends: one wait for all
    // (all three loads unconditional and waited for together: a load left
    // pending on some path makes the compiler wait inside the main loop)
    const int n = rem > nq ? min((QB - nq) >> 4, 3) : 0;
    const u32x4* f0 = fp;
    const u32x4 v0 = load_block(), v1 = load_block(), v2 = load_block();
    fp = f0 + n;
    __builtin_amdgcn_s_waitcnt(0);
    if (n > 0) append(v0);
    if (n > 1) append(v1);
    if (n > 2) append(v2);
  }
  __device__ __forceinline__ uint32_t next_byte() {
    const uint32_t c = q[0] >> 24;
#pragma unroll
    for (int i = 0; i + 1 < QW; ++i) q[i] = (q[i] << 8) | (q[i + 1] >> 24);
    q[QW - 1] <<= 8;
    --nq;
    --rem;
    return c;
  }
  // Ensure >= 32 buffered bits (a symbol takes <= 16 + 15).  Usual case: the
  // next 4 raw bytes hold no 0xFF and go in as one dword; otherwise byte by
  // byte with un-stuffing.
  __device__ __forceinline__ void fill() {
    if (nbits >= 32) return;
    const uint32_t d = q[0], nd = ~d;
    const bool ff = ((nd - 0x01010101u) & ~nd & 0x80808080u) != 0u;
    if (!ff && !marker && rem >= 4) {
      buf |= (uint64_t)d << (32 - nbits);
      nbits += 32;
#pragma unroll
      for (int i = 0; i + 1 < QW; ++i) q[i] = q[i + 1];
      q[QW - 1] = 0;
      nq -= 4;
      rem -= 4;
      return;
    }
    while (nbits < 32) {
      uint32_t c = 0;
      if (!marker && rem > 0) {
        c = next_byte();
        if (c == 0xFF) {
          const uint32_t n = rem > 0 ? (q[0] >> 24) : 0xD9;
          if (n == 0x00) {
            next_byte();         // stuffed zero byte
          } else {
            marker = true;       // a marker: zeros from here
            c = 0;
          }
        }
      }
      buf |= (uint64_t)c << (56 - nbits);
      nbits += 8;
    }
  }
  __device__ __forceinline__ uint32_t peek(int n) { return (uint32_t)(buf >> (64 - n)); }
  __device__ __forceinline__ void skip(int n) {
    buf <<= n;
    nbits -= n;
  }
};

// Decode one symbol (after fill(): >= 32 bits buffered, a code takes <= 16)
__device__ __forceinline__ int huff_decode(BitReader& br, const JpegHuff* __restrict__ t) {
  const uint32_t lk = t->look[br.peek(9)];
  if (lk) {
    br.skip(lk >> 8);
    return lk & 0xFF;
  }
  // longer code: one second-level lookup, or libjpeg jpeg_huff_decode's walk (lengths 10..16)
  const int i2 = (int)br.peek(16) - t->l2base;
  if ((unsigned)i2 < (unsigned)t->l2n) {
    const uint32_t l2 = t->look2[i2];
    br.skip(l2 ? (int)(l2 >> 8) : 16);   // 0: corrupt data, libjpeg returns 0 (and warns)
    return l2 & 0xFF;
  }
  int l = 10;
  uint32_t code = br.peek(10);
  while (l <= 16 && (int32_t)code > t->maxcode[l]) {
    ++l;
    code = br.peek(l);
  }
  if (l > 16) {   // corrupt data: libjpeg returns 0 (and warns)
    br.skip(16);
    return 0;
  }
  br.skip(l);
  return t->vals[(code + t->valoff[l]) & 0xFF];
}

__device__ __forceinline__ int extend(uint32_t v, int s) {
  return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

// Per frame f: entropy-coded bytes at data + off[f] (len[f] bytes), tables at
// huff[set * 4 + {dc0, ac0, dc1, ac1}] with set = huff_idx[f] (f without
// huff_idx), coefficient output coef + f * blocks_per_frame * 64 (zeroed by the
// caller; only nonzero coefficients are written).
// Geometry (all frames of a launch share it): ncomp components, component c with
// sampling (hs[c], vs[c]), block grid width bw[c] (blocks), block base cbase[c]
// (blocks, within the frame), table selectors dcsel[c] / acsel[c]; MCU grid mcux x mcuy;
// restart interval ri MCUs (0: none).  Segment s of frame f (restart interval s) starts
// at byte seg_off[f * nseg + s] (host-located RSTn positions), so every segment is
// independent: one lane per (frame, segment).
struct JpegGeom {
  int ncomp, mcux, mcuy, ri, nseg;
  int hs[3], vs[3], bw[3], cbase[3], dcsel[3], acsel[3];
  int64_t blocks_per_frame;
};

template <typename T>
__device__ __forceinline__ T pick3(int c, T a, T b, T d) {
  return c == 0 ? a : (c == 1 ? b : d);
}

// One symbol per loop trip (DC or AC of whichever block the lane is in), so
// lanes of a wave decoding different frames never wait on each other's block
// structure: a wave runs as many trips as its longest segment has symbols.
// LDS_T: the launch's table sets (nsets <= JPEG_LDS_SETS) are staged in LDS.
template <bool LDS_T>
__global__ __launch_bounds__(64) void jpeg_entropy_kernel(const uint8_t* __restrict__ data,
                                                          const int64_t* __restrict__ seg_off,
                                                          const int64_t* __restrict__ seg_end,
                                                          const JpegHuff* __restrict__ huff,
                                                          const int32_t* __restrict__ huff_idx, int nsets,
                                                          JpegGeom g, int nframes, int16_t* __restrict__ coef) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  JpegHuff* sh = (JpegHuff*)smem;
  uint8_t* zz = (uint8_t*)smem + (LDS_T ? nsets * 4 * (int)sizeof(JpegHuff) : 0);
  if (LDS_T) {
    const uint32_t* src = (const uint32_t*)huff;
    uint32_t* dst = (uint32_t*)smem;
    const int nw = nsets * 4 * (int)sizeof(JpegHuff) / 4;
    for (int i = threadIdx.x; i < nw; i += 64) dst[i] = src[i];
  }
  for (int i = threadIdx.x; i < 80; i += 64) zz[i] = kZigzag[i];
  __syncthreads();
  const int64_t lane = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (lane >= (int64_t)nframes * g.nseg) return;
  const int f = (int)(lane / g.nseg), s = (int)(lane % g.nseg);
  BitReader br;
  br.init(data + seg_off[lane], data + seg_end[lane]);
  const int set = huff_idx ? huff_idx[f] : f;
  const JpegHuff* T = (LDS_T ? (const JpegHuff*)sh : huff) + (int64_t)set * 4;
  int16_t* out = coef + (int64_t)f * g.blocks_per_frame * 64;
  const int total = g.mcux * g.mcuy;
  int m = g.ri ? s * g.ri : 0;
  const int m1 = g.ri ? min(total, m + g.ri) : total;
  int mx = m % g.mcux, my = m / g.mcux;
  int c = 0, bv = 0, bh = 0, k = 0;
  int p0 = 0, p1 = 0, p2 = 0;
  const JpegHuff *d0 = T + g.dcsel[0] * 2, *a0 = T + g.acsel[0] * 2 + 1;
  const JpegHuff *d1 = T + g.dcsel[1] * 2, *a1 = T + g.acsel[1] * 2 + 1;
  const JpegHuff *d2 = T + g.dcsel[2] * 2, *a2 = T + g.acsel[2] * 2 + 1;
  int hs_c = g.hs[0], vs_c = g.vs[0];
  int16_t* blk = out + (g.cbase[0] + (int64_t)(my * vs_c) * g.bw[0] + mx * hs_c) * 64;
  // Nothing may be in flight when the loop starts: a load still pending at the
  // loop entry makes the compiler place a vmcnt(0) wait inside the loop body,
  // which then drains every coefficient store on every trip.
  __builtin_amdgcn_s_waitcnt(0);
  while (m < m1) {
    const JpegHuff* tp = k ? pick3(c, a0, a1, a2) : pick3(c, d0, d1, d2);
    if (__any(br.low())) br.refill();   // one wave-wide load for every lane with room
    br.fill();
    const int sym = huff_decode(br, tp);
    const int sz = sym & 15;   // DC: the size category (<= 15, host-checked)
    const int r = k ? (sym >> 4) : 0;
    const uint32_t bits = sz ? br.peek(sz) : 0u;
    br.skip(sz);
    const int val = sz ? extend(bits, sz) : 0;
    bool endblk;
    if (k == 0) {
      const int pv = pick3(c, p0, p1, p2) + val;
      p0 = c == 0 ? pv : p0;
      p1 = c == 1 ? pv : p1;
      p2 = c == 2 ? pv : p2;
      blk[0] = (int16_t)pv;
      k = 1;
      endblk = false;
    } else if (sz) {
      k += r;
      blk[zz[k]] = (int16_t)val;
      ++k;
      endblk = k >= 64;
    } else if (r == 15) {
      k += 16;
      endblk = k >= 64;
    } else {
      endblk = true;   // EOB
    }
    if (endblk) {
      k = 0;
      if (++bh == hs_c) {
        bh = 0;
        if (++bv == vs_c) {
          bv = 0;
          if (++c == g.ncomp) {
            c = 0;
            ++m;
            if (++mx == g.mcux) {
              mx = 0;
              ++my;
            }
          }
          hs_c = pick3(c, g.hs[0], g.hs[1], g.hs[2]);
          vs_c = pick3(c, g.vs[0], g.vs[1], g.vs[2]);
        }
      }
      const int bw_c = pick3(c, g.bw[0], g.bw[1], g.bw[2]), cb_c = pick3(c, g.cbase[0], g.cbase[1], g.cbase[2]);
      blk = out + (cb_c + (int64_t)(my * vs_c + bv) * bw_c + (mx * hs_c + bh)) * 64;
    }
  }
}

// ---- IDCT (jidctint.c jpeg_idct_islow) -----------------------------------
constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

// libjpeg-turbo computes in JLONG (64-bit on LP64): the same here, so extreme
// (corrupt) coefficients wrap exactly as there
__device__ __forceinline__ int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }

// libjpeg's post-IDCT range limit: table[(x) & 1023] around CENTERJSAMPLE
__device__ __forceinline__ uint8_t range_limit_idct(int32_t x) {
  const int v = x & 1023;
  return (uint8_t)(v < 128 ? v + 128 : v < 512 ? 255 : v < 896 ? 0 : v - 896);
}

__device__ __forceinline__ void idct_1d(const int32_t* in, int stride_in, int32_t* o, int n_out_shift) {
  // even part
  int64_t z2 = in[2 * stride_in], z3 = in[6 * stride_in];
  int64_t z1 = (z2 + z3) * F0541;
  int64_t tmp2 = z1 + z3 * (-F1847);
  int64_t tmp3 = z1 + z2 * F0765;
  z2 = in[0];
  z3 = in[4 * stride_in];
  int64_t tmp0 = (z2 + z3) * ((int64_t)1 << CONST_BITS);
  int64_t tmp1 = (z2 - z3) * ((int64_t)1 << CONST_BITS);
  const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  // odd part
  tmp0 = in[7 * stride_in];
  tmp1 = in[5 * stride_in];
  tmp2 = in[3 * stride_in];
  tmp3 = in[1 * stride_in];
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  int64_t z4 = tmp1 + tmp3;
  const int64_t z5 = (z3 + z4) * F1175;
  tmp0 = tmp0 * F0298;
  tmp1 = tmp1 * F2053;
  tmp2 = tmp2 * F3072;
  tmp3 = tmp3 * F1501;
  z1 = z1 * (-F0899);
  z2 = z2 * (-F2562);
  z3 = z3 * (-F1961);
  z4 = z4 * (-F0390);
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  o[0] = descale(tmp10 + tmp3, n_out_shift);
  o[7] = descale(tmp10 - tmp3, n_out_shift);
  o[1] = descale(tmp11 + tmp2, n_out_shift);
  o[6] = descale(tmp11 - tmp2, n_out_shift);
  o[2] = descale(tmp12 + tmp1, n_out_shift);
  o[5] = descale(tmp12 - tmp1, n_out_shift);
  o[3] = descale(tmp13 + tmp0, n_out_shift);
  o[4] = descale(tmp13 - tmp0, n_out_shift);
}

// block b of frame f -> component plane bytes.  Planes: component c of frame f at
// planes + f * plane_frame_bytes + pbase[c], row stride pstride[c] = bw[c] * 8.
struct JpegPlanes {
  int64_t plane_frame_bytes;
  int64_t pbase[3];
  int pstride[3], bh[3];
  int qsel[3];
};

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coef,
                                                        const uint16_t* __restrict__ qtab, JpegGeom g, JpegPlanes pl,
                                                        int nframes, uint8_t* __restrict__ planes) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)nframes * g.blocks_per_frame) return;
  const int f = (int)(t / g.blocks_per_frame);
  const int64_t b = t % g.blocks_per_frame;
  int c = 0;
  while (c + 1 < g.ncomp && b >= g.cbase[c + 1]) ++c;
  const int64_t lb = b - g.cbase[c];
  const int by = (int)(lb / g.bw[c]), bx = (int)(lb % g.bw[c]);
  const uint16_t* q = qtab + ((int64_t)f * 4 + pl.qsel[c]) * 64;
  int32_t ws[64];
  const uint4* cb4 = (const uint4*)(coef + t * 64);
  int32_t in[64];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint4 v = cb4[j];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      in[8 * j + 2 * e] = (int32_t)(int16_t)(w[e] & 0xFFFF) * (int32_t)q[8 * j + 2 * e];
      in[8 * j + 2 * e + 1] = (int32_t)(int16_t)(w[e] >> 16) * (int32_t)q[8 * j + 2 * e + 1];
    }
  }
  // pass 1: columns -> ws (DC-only columns: libjpeg's shortcut gives the same values)
#pragma unroll
  for (int col = 0; col < 8; ++col) {
    int32_t o[8];
    idct_1d(in + col, 8, o, CONST_BITS - PASS1_BITS);
#pragma unroll
    for (int r = 0; r < 8; ++r) ws[r * 8 + col] = o[r];
  }
  uint8_t* dst = planes + (int64_t)f * pl.plane_frame_bytes + pl.pbase[c] + (int64_t)(by * 8) * pl.pstride[c] + bx * 8;
#pragma unroll
  for (int row = 0; row < 8; ++row) {
    int32_t o[8];
    idct_1d(ws + row * 8, 1, o, CONST_BITS + PASS1_BITS + 3);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) lo |= (uint32_t)range_limit_idct(o[i]) << (8 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) hi |= (uint32_t)range_limit_idct(o[4 + i]) << (8 * i);
    *(uint2*)(dst + (int64_t)row * pl.pstride[c]) = make_uint2(lo, hi);
  }
}

// ---- upsampling + colour (jdsample.c fancy upsampling, jdcolor.c ycc_rgb_convert)
__device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// fancy-upsampled chroma sample at output (x, y); the component has dw x dh samples
// (libjpeg downsampled_width / _height) with row stride ps; mode: 0 = 1x1 (no
// upsampling), 1 = h2v1, 2 = h2v2
__device__ __forceinline__ int chroma_at(const uint8_t* __restrict__ P, int ps, int dw, int dh, int x, int y, int mode) {
  if (mode == 0) return P[(int64_t)y * ps + x];
  const int cc = x >> 1;
  if (mode == 1) {   // h2v1_fancy_upsample
    const uint8_t* row = P + (int64_t)y * ps;
    const int v = row[cc];
    if ((x & 1) == 0) return cc == 0 ? v : (v * 3 + row[cc - 1] + 1) >> 2;
    return cc == dw - 1 ? v : (v * 3 + row[cc + 1] + 2) >> 2;
  }
  // h2v2_fancy_upsample: near row = y >> 1, far row above (even y) or below (odd y),
  // replicated at the top / bottom edge (libjpeg context rows)
  const int r = y >> 1;
  const int rf = (y & 1) ? min(r + 1, dh - 1) : max(r - 1, 0);
  const uint8_t* n = P + (int64_t)r * ps;
  const uint8_t* fr = P + (int64_t)rf * ps;
  const int th = n[cc] * 3 + fr[cc];
  if ((x & 1) == 0) {
    if (cc == 0) return (th * 4 + 8) >> 4;
    const int la = n[cc - 1] * 3 + fr[cc - 1];
    return (th * 3 + la + 8) >> 4;
  }
  if (cc == dw - 1) return (th * 4 + 7) >> 4;
  const int nx = n[cc + 1] * 3 + fr[cc + 1];
  return (th * 3 + nx + 7) >> 4;
}

__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t* __restrict__ planes, JpegPlanes pl, int W, int H,
                                                         int ncomp, int cmode, int cdw, int cdh, int nframes,
                                                         uint8_t* __restrict__ rgb) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t px = (int64_t)W * H;
  if (t >= (int64_t)nframes * px) return;
  const int f = (int)(t / px);
  const int64_t p = t % px;
  const int y = (int)(p / W), x = (int)(p % W);
  const uint8_t* base = planes + (int64_t)f * pl.plane_frame_bytes;
  const int Y = base[pl.pbase[0] + (int64_t)y * pl.pstride[0] + x];
  uint8_t* o = rgb + t * 3;
  if (ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)Y;
    return;
  }
  const int cb = chroma_at(base + pl.pbase[1], pl.pstride[1], cdw, cdh, x, y, cmode) - 128;
  const int cr = chroma_at(base + pl.pbase[2], pl.pstride[2], cdw, cdh, x, y, cmode) - 128;
  // FIX(x) = (int)(x * 65536 + 0.5); ONE_HALF = 1 << 15; arithmetic right shifts
  const int r = Y + ((91881 * cr + 32768) >> 16);
  const int gch = Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
  const int b = Y + ((116130 * cb + 32768) >> 16);
  o[0] = (uint8_t)clamp255(r);
  o[1] = (uint8_t)clamp255(gch);
  o[2] = (uint8_t)clamp255(b);
}

}  // namespace

// Host launch: see include/miclip.h mi_jpeg_decode for the argument contract.
hipError_t jpeg_decode(const uint8_t* data, const int64_t* seg_off, const int64_t* seg_end, const void* huff,
                       const int32_t* huff_idx, int nsets, const uint16_t* qtab, const int32_t* geom, int nframes, uint8_t* out_rgb, void* ws,
                       size_t ws_bytes, hipStream_t s) {
  // geom: [W, H, ncomp, ri, nseg, hs0, vs0, hs1, vs1, hs2, vs2, q0, q1, q2, dc0, dc1, dc2, ac0, ac1, ac2]
  const int W = geom[0], H = geom[1], ncomp = geom[2];
  JpegGeom g{};
  g.ncomp = ncomp;
  g.ri = geom[3];
  g.nseg = geom[4];
  int hmax = 1, vmax = 1;
  for (int c = 0; c < ncomp; ++c) {
    g.hs[c] = geom[5 + 2 * c];
    g.vs[c] = geom[6 + 2 * c];
    hmax = g.hs[c] > hmax ? g.hs[c] : hmax;
    vmax = g.vs[c] > vmax ? g.vs[c] : vmax;
  }
  if (ncomp == 1) {   // single-component scan: MCU = one block over ceil(W/8) x ceil(H/8)
    g.hs[0] = g.vs[0] = 1;
    hmax = vmax = 1;
  }
  g.mcux = (W + 8 * hmax - 1) / (8 * hmax);
  g.mcuy = (H + 8 * vmax - 1) / (8 * vmax);
  JpegPlanes pl{};
  int64_t blocks = 0, bytes = 0;
  for (int c = 0; c < ncomp; ++c) {
    g.bw[c] = g.mcux * g.hs[c];
    pl.bh[c] = g.mcuy * g.vs[c];
    g.cbase[c] = (int)blocks;
    blocks += (int64_t)g.bw[c] * pl.bh[c];
    pl.pstride[c] = g.bw[c] * 8;
    pl.pbase[c] = bytes;
    bytes += (int64_t)pl.pstride[c] * pl.bh[c] * 8;
    pl.qsel[c] = geom[11 + c];
    g.dcsel[c] = geom[14 + c];
    g.acsel[c] = geom[17 + c];
  }
  g.blocks_per_frame = blocks;
  pl.plane_frame_bytes = bytes;
  const size_t coef_bytes = (size_t)nframes * blocks * 64 * sizeof(int16_t);
  if (ws_bytes < coef_bytes + (size_t)nframes * bytes) return hipErrorInvalidValue;
  int16_t* coef = (int16_t*)ws;
  uint8_t* planes = (uint8_t*)ws + coef_bytes;
  hipError_t e = hipMemsetAsync(coef, 0, coef_bytes, s);
  if (e != hipSuccess) return e;
  const int64_t lanes = (int64_t)nframes * g.nseg;
  const dim3 eg((unsigned)((lanes + 63) / 64));
  if (huff_idx && nsets >= 1 && nsets <= JPEG_LDS_SETS)
    hipLaunchKernelGGL(jpeg_entropy_kernel<true>, eg, dim3(64), nsets * 4 * sizeof(JpegHuff) + 80, s, data, seg_off,
                       seg_end, (const JpegHuff*)huff, huff_idx, nsets, g, nframes, coef);
  else
    hipLaunchKernelGGL(jpeg_entropy_kernel<false>, eg, dim3(64), 80, s, data, seg_off, seg_end,
                       (const JpegHuff*)huff, huff_idx, nsets, g, nframes, coef);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // A dispatch counts its work-items in 32 bits (grid x block < 2^32): the
  // per-block and per-pixel kernels run over frame chunks of < 2^31 items.
  const int64_t fc_idct = blocks > 0 ? std::max<int64_t>(1, ((int64_t)1 << 31) / blocks) : nframes;
  for (int64_t f0 = 0; f0 < nframes; f0 += fc_idct) {
    const int nfc = (int)std::min<int64_t>(fc_idct, nframes - f0);
    const int64_t nb = (int64_t)nfc * blocks;
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s,
                       coef + f0 * blocks * 64, qtab + f0 * 4 * 64, g, pl, nfc, planes + f0 * bytes);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  // chroma layout relative to luma (components 1, 2 share it)
  int cmode = 0, cdw = W, cdh = H;
  if (ncomp == 3) {
    const int hr = hmax / g.hs[1], vr = vmax / g.vs[1];
    cmode = (hr == 1 && vr == 1) ? 0 : (hr == 2 && vr == 1) ? 1 : 2;
    cdw = (W * g.hs[1] + hmax - 1) / hmax;   // libjpeg downsampled_width
    cdh = (H * g.vs[1] + vmax - 1) / vmax;
  }
  const int64_t px = (int64_t)W * H;
  const int64_t fc_px = std::max<int64_t>(1, ((int64_t)1 << 31) / px);
  for (int64_t f0 = 0; f0 < nframes; f0 += fc_px) {
    const int nfc = (int)std::min<int64_t>(fc_px, nframes - f0);
    const int64_t np = (int64_t)nfc * px;
    hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, planes + f0 * bytes, pl,
                       W, H, ncomp, cmode, cdw, cdh, nfc, out_rgb + f0 * px * 3);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

size_t jpeg_workspace_bytes(const int32_t* geom, int nframes) {
  const int W = geom[0], H = geom[1], ncomp = geom[2];
  int hmax = 1, vmax = 1, hs[3] = {1, 1, 1}, vs[3] = {1, 1, 1};
  for (int c = 0; c < ncomp && ncomp == 3; ++c) {
    hs[c] = geom[5 + 2 * c];
    vs[c] = geom[6 + 2 * c];
    hmax = hs[c] > hmax ? hs[c] : hmax;
    vmax = vs[c] > vmax ? vs[c] : vmax;
  }
  const int64_t mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
  int64_t blocks = 0;
  for (int c = 0; c < ncomp; ++c) blocks += mcux * hs[c] * mcuy * vs[c];
  return (size_t)nframes * blocks * 64 * (sizeof(int16_t) + 1);
}

}  // namespace miclip
