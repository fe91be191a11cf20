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
#include <cstdlib>

#include "common.hpp"
#include "internal.hpp"
#include "miclip.h"

namespace miclip {
namespace {

// The coefficient workspace holds each block in ZIGZAG order (coefficient k at slot min(k, 63):
// a corrupt run past 63 lands in natural position 63 = zigzag slot 63, as libjpeg's
// jpeg_natural_order + 16).  The entropy passes then write a block's coefficients in increasing
// slot order, 16-byte windows at a time (jp_run), and the IDCT reads natural position n from
// slot kIzz[n] (a compile-time register permutation).
constexpr uint8_t kIzz[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                              3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                              10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                              21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

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
template <bool STUFFED>
struct BitReaderT {
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
  uint32_t pos;            // (unstuffed streams) bit position of the next unconsumed bit

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
    if (rem <= 0) {   // nothing to read: the (unconditional) refill loads stay on a valid address
      rem = 0;
      fp = flast = (const u32x4*)((uintptr_t)p & ~(uintptr_t)15);
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
    const bool ff = STUFFED && ((nd - 0x01010101u) & ~nd & 0x80808080u) != 0u;
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
        if (STUFFED && c == 0xFF) {
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
    if (!STUFFED) pos += n;
  }
  // unstuffed stream of `len` bytes at base, positioned at bit p (zeros past the end)
  __device__ __forceinline__ void init_at(const uint8_t* base, uint32_t len, uint32_t p) {
    const uint32_t b0 = min(p >> 3, len);
    init(base + b0, base + len);
    pos = b0 * 8;
    while (pos < p) {   // bits before p in the first byte (or past the end: zeros)
      fill();
      skip((int)min(p - pos, 24u));
    }
  }
};
typedef BitReaderT<true> BitReader;

// Decode one symbol (after fill(): >= 32 bits buffered, a code takes <= 16)
template <typename BR>
__device__ __forceinline__ int huff_decode(BR& br, const JpegHuff* __restrict__ t) {
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
                                                          JpegGeom g, int nframes, int16_t* __restrict__ coef,
                                                          int64_t data_bytes, const uint8_t* __restrict__ skip) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  JpegHuff* sh = (JpegHuff*)smem;
  if (LDS_T) {
    const uint32_t* src = (const uint32_t*)huff;
    uint32_t* dst = (uint32_t*)smem;
    const int nw = nsets * 4 * (int)sizeof(JpegHuff) / 4;
    for (int i = threadIdx.x; i < nw; i += 64) dst[i] = src[i];
  }
  __syncthreads();
  const int64_t lane = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (lane >= (int64_t)nframes * g.nseg) return;
  const int f = (int)(lane / g.nseg), s = (int)(lane % g.nseg);
  if (skip && skip[f]) return;   // the chunked decode's frames (the fix-up pass takes the others)
  BitReader br;
  const int64_t so = min(max(seg_off[lane], (int64_t)0), data_bytes);
  br.init(data + so, data + min(max(seg_end[lane], so), data_bytes));
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
      blk[k < 63 ? k : 63] = (int16_t)val;   // zigzag slot (see kIzz)
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

// ---- speculative parallel entropy decode (scans without restart markers) --
// A lane per frame leaves the chip mostly idle (8192 frames = 128 waves) and a
// frame takes ~0.3 s of one lane.  For a scan without restart markers the
// frame's entropy-coded data is instead split into chunks of JP_CHUNK bytes,
// decoded by one lane each (Weissenberger & Schmidt's self-synchronising
// parallel Huffman decoding, extended with JPEG's block state):
//   1. unstuff: the scan's bytes with the 0x00 after each 0xFF removed and
//      everything from the first marker on dropped (libjpeg then feeds zeros,
//      as BitReader does) -> a plain bit stream per frame (jp_unstuff_*);
//   2. phase 1: the lane of chunk t starts at the chunk's first bit GUESSING
//      the state "block 0 of an MCU, coefficient 0" and decodes up to the
//      first symbol boundary at or past the chunk's end: its exit state
//      (bit position, block within the MCU, coefficient index), the blocks it
//      completed and its DC-difference sums per component (jp_sync, round 0);
//   3. rounds: the lane of chunk t re-decodes from the exit state of chunk
//      t - 1 whenever that changed in the previous round; a chunk whose exit
//      state does not change is consistent with its predecessor.  Chunk 0
//      starts at the true state, so after a round with no change every chunk
//      is, and its exit states are the true ones.  Huffman codes resynchronise
//      within a few symbols: on the reference frames, 224 of 225 1-KB chunks
//      had the true exit state after phase 1 (scripts/jpeg_sync_proto.py);
//   4. prefix sums of the block counts and DC sums per frame give each chunk
//      its first block index and DC predictors (jp_prefix);
//   5. the final pass decodes every chunk from its true entry state and writes
//      the coefficients (jp_final).  A frame still changing after the last
//      round (never seen) is decoded serially by its chunk-0 lane instead, so
//      the output is always the serial decode's.
// Same table look-ups, symbol semantics, zero feed and block walk as
// jpeg_entropy_kernel, so the coefficients are bit-identical to it.
constexpr int JP_CHUNK = 1024;    // unstuffed bytes per chunk (scripts/jpeg_sync_proto.py)
constexpr int JP_ROUNDS = 4;      // consistency rounds after phase 1

// The MCU's block walk: block b of an MCU belongs to component comp[b] at
// (dh[b], dv[b]) within that component's hs x vs blocks.
struct JpegMcu {
  int bpm;
  int8_t comp[16], dh[16], dv[16];
};


// Checkpoints of a chunk's recorded decode path (the sync rounds).  A decode that restarts
// from a corrected entry state usually joins the recorded path after a few hundred bits
// (scripts/jpeg_sync_proto.py: median 838 bits on the reference frames); from a shared state
// (bit position, block within the MCU, coefficient index) on, the two decodes are identical, so
// the re-decode stops at the first checkpoint where its state equals the recorded one and takes
// the rest -- exit state, blocks, DC sums -- from the record.  Checkpoint j is the path's first
// symbol boundary at or past first + JP_CP_FIRST + j * JP_CP_STEP bits; its counts are relative
// to the start of the path that recorded it, as are the path totals tn / td.
constexpr int JP_NCP = 8;
constexpr uint32_t JP_CP_FIRST = 512, JP_CP_STEP = 1024;
struct JpCps {
  uint64_t* x;   // [nmax * JP_NCP] packed state, ~0: none
  int32_t* nb;   // [nmax * JP_NCP] blocks completed from the path's start
  int32_t* dc;   // [nmax * JP_NCP * 3] DC-difference sums from the path's start
  int32_t* tn;   // [nmax] the path's blocks, start -> exit
  int32_t* td;   // [nmax * 3]
};
struct JpCpRun {
  uint32_t first, thr;   // the chunk's first bit; the next checkpoint's position
  int j;                 // the next checkpoint
  int hit;               // -1, or the recorded checkpoint this decode joined
  bool cmp;              // compare with the recorded path (a re-decode) or only record (round 0)
  int64_t slot;          // ci * JP_NCP
  JpCps cp;
};

__device__ __forceinline__ uint64_t pack_state(uint32_t pos, int b, int k) {
  return ((uint64_t)pos << 16) | ((uint64_t)b << 8) | (uint64_t)k;
}

// Decode from the reader's position in state (b, k) until the position reaches
// `stop` (at a symbol boundary) or, when writing, the frame's last block is
// done.  nblk counts completed blocks; dc[] accumulates DC differences (WRITE:
// the running predictors, stored as each block's coefficient 0).
typedef BitReaderT<false> UReader;

template <bool WRITE, bool CP = false>
__device__ __forceinline__ void jp_run(UReader& br, const JpegHuff* __restrict__ T, const JpegGeom& g,
                                       const JpegMcu& mc, int& b, int& k, uint32_t stop, int64_t blk, int64_t total,
                                       int& nblk, int (&dc)[3], int16_t* __restrict__ out, bool st = true,
                                       JpCpRun* cr = nullptr) {
  // the block's MCU coordinates, advanced per block (block_addr's 64-bit divisions once per
  // call, not at every block end: in the wave's lockstep some lane ends a block nearly every trip)
  int mx = 0, my = 0;
  if (WRITE) {
    const int64_t m = blk / mc.bpm;
    my = (int)(m / g.mcux);
    mx = (int)(m - (int64_t)my * g.mcux);
  }
  auto addr = [&](int bb) -> int64_t {
    const int c = mc.comp[bb];
    const int hs_c = pick3(c, g.hs[0], g.hs[1], g.hs[2]), vs_c = pick3(c, g.vs[0], g.vs[1], g.vs[2]);
    const int bw_c = pick3(c, g.bw[0], g.bw[1], g.bw[2]), cb_c = pick3(c, g.cbase[0], g.cbase[1], g.cbase[2]);
    return cb_c + (int64_t)(my * vs_c + mc.dv[bb]) * bw_c + mx * hs_c + mc.dh[bb];
  };
  int16_t* bp = WRITE ? out + addr(b) * 64 : nullptr;
  // WRITE: coefficients gather in a 16-byte window of 8 zigzag slots (w[4], slot-pair per dword)
  // that goes out as ONE 16-byte store when the block leaves it -- ~3-4 stores per block instead
  // of a 2-byte store per coefficient.  The workspace is zeroed, so skipped windows need no store.
  // A chunk boundary inside a block splits one window between two lanes: the chunk's first
  // window from slot lo0 (its entry k) and its last from slot ... up to the exit k are written
  // slot by slot, so neither lane's zeros overwrite the other's coefficients.
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  int wk = -1;                                  // window in w (slot >> 3), -1: none
  int lo0 = WRITE && (k & 7) ? k : -1;          // entry slot inside a window (first block only)
  auto flush_range = [&](int lo, int hi) {      // slots [lo, hi) of window wk
    const int s0 = wk * 8;
    if (lo <= s0 && hi >= s0 + 8) {
      if (st) {
        typedef uint32_t u32x4w __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) u32x4w gu4;
        *(gu4*)(bp + s0) = (u32x4w){w[0], w[1], w[2], w[3]};
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (st && s0 + j >= lo && s0 + j < hi) bp[s0 + j] = (int16_t)(w[j >> 1] >> ((j & 1) * 16));
  };
  auto flush = [&]() {
    if (wk < 0) return;
    flush_range(lo0 >= 0 && wk == (lo0 >> 3) ? lo0 : 0, 64);
    w[0] = w[1] = w[2] = w[3] = 0u;
    wk = -1;
  };
  auto put = [&](int slot, int v) {
    const int wi = slot >> 3;
    if (wi != wk) {
      flush();
      wk = wi;
    }
    const int d = (slot >> 1) & 3;
    const uint32_t sh = (uint32_t)(slot & 1) * 16u;
    const uint32_t m = 0xFFFFu << sh, x = ((uint32_t)v & 0xFFFFu) << sh;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = d == i ? (w[i] & ~m) | x : w[i];   // replace: a corrupt run rewrites 63
  };
  while (br.pos < stop && (!WRITE || blk < total)) {
    if (CP && br.pos >= cr->thr) {   // checkpoint cr->j: join the recorded path, or record this one
      const uint64_t xs = pack_state(br.pos, b, k);
      const int64_t sl = cr->slot + cr->j;
      if (cr->cmp && cr->cp.x[sl] == xs) {
        cr->hit = cr->j;
        break;
      }
      cr->cp.x[sl] = xs;
      cr->cp.nb[sl] = nblk;
      cr->cp.dc[3 * sl] = dc[0];
      cr->cp.dc[3 * sl + 1] = dc[1];
      cr->cp.dc[3 * sl + 2] = dc[2];
      ++cr->j;
      cr->thr = cr->j < JP_NCP ? cr->first + JP_CP_FIRST + JP_CP_STEP * (uint32_t)cr->j : 0xFFFFFFFFu;
    }
    const int c = mc.comp[b];
    const JpegHuff* tp = k ? T + pick3(c, g.acsel[0], g.acsel[1], g.acsel[2]) * 2 + 1
                           : T + pick3(c, g.dcsel[0], g.dcsel[1], g.dcsel[2]) * 2;
    if (__any(br.low())) br.refill();   // one wave-wide load for every lane with room
    br.fill();
    const int sym = huff_decode(br, tp);
    const int sz = sym & 15;
    const int r = k ? (sym >> 4) : 0;
    const uint32_t bits = sz ? br.peek(sz) : 0u;
    br.skip(sz);
    const int val = sz ? extend(bits, sz) : 0;
    bool endblk;
    if (k == 0) {
      const int pv = pick3(c, dc[0], dc[1], dc[2]) + val;
      dc[0] = c == 0 ? pv : dc[0];
      dc[1] = c == 1 ? pv : dc[1];
      dc[2] = c == 2 ? pv : dc[2];
      if (WRITE) put(0, pv);
      k = 1;
      endblk = false;
    } else if (sz) {
      k += r;
      if (WRITE) put(k < 63 ? k : 63, val);
      ++k;
      endblk = k >= 64;
    } else if (r == 15) {
      k += 16;
      endblk = k >= 64;
    } else {
      endblk = true;
    }
    if (endblk) {
      k = 0;
      b = b + 1 == mc.bpm ? 0 : b + 1;
      ++nblk;
      ++blk;
      if (WRITE) {
        flush();
        lo0 = -1;
        if (b == 0) {
          mx = mx + 1 == g.mcux ? 0 : mx + 1;
          my += mx == 0 ? 1 : 0;
        }
        if (blk < total) bp = out + addr(b) * 64;
      }
    }
  }
  if (WRITE && wk >= 0) {   // stopped inside a block: the next chunk owns slots from k on
    const int hi = (k & 7) && wk == (k >> 3) ? k : 64;
    flush_range(lo0 >= 0 && wk == (lo0 >> 3) ? lo0 : 0, hi);
  }
}

// frame bookkeeping shared by the chunk kernels
struct JpChunks {
  const int64_t* cbase;    // [B + 1] first chunk of each frame
  const int32_t* cframe;   // [nchunks] frame of each chunk
  const int64_t* ubase;    // [B] unstuffed stream of frame f at ustuff + ubase[f] (4-byte aligned)
  const uint32_t* ulen;    // [B] unstuffed bytes of frame f
};

// chunk layout: T_f = max(1, ceil(raw bytes / JP_CHUNK)) chunks per frame; one workgroup.
// The caller's segments are sanitised first (mi_jpeg_decode's contract: disjoint, in
// frame order, inside [0, data_bytes)): each is clipped to [0, data_bytes), and a frame
// whose segment starts before the end of an earlier frame's (a repeated or out-of-order
// frame) gets no chunks -- vf[f] = 0 -- and is decoded afterwards by the serial kernel,
// which only reads the data.  So sum T_f <= data_bytes / JP_CHUNK + B = the workspace's
// nmax, and the valid frames' unstuffed streams (at their own byte offsets) never overlap.
__global__ __launch_bounds__(1024) void jp_layout_kernel(const int64_t* __restrict__ seg_off,
                                                         const int64_t* __restrict__ seg_end, int nframes,
                                                         int64_t data_bytes, int64_t* __restrict__ cbase,
                                                         int64_t* __restrict__ ubase, int64_t* __restrict__ sso,
                                                         int64_t* __restrict__ sse, uint8_t* __restrict__ vf) {
  __shared__ int64_t part[1024];
  const int tid = threadIdx.x;
  const int per = (nframes + 1023) / 1024;
  const int f0 = tid * per, f1 = min(nframes, f0 + per);
  auto clip = [&](int f, int64_t& o, int64_t& e) {
    o = min(max(seg_off[f], (int64_t)0), data_bytes);
    e = min(max(seg_end[f], o), data_bytes);
  };
  // prefix max of the clipped segment ends over all earlier frames
  int64_t mx = -1;
  for (int f = f0; f < f1; ++f) {
    int64_t o, e;
    clip(f, o, e);
    mx = max(mx, e);
  }
  part[tid] = mx;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {   // inclusive Hillis-Steele max scan
    const int64_t v = tid >= o ? part[tid - o] : -1;
    __syncthreads();
    part[tid] = max(part[tid], v);
    __syncthreads();
  }
  int64_t runmax = tid > 0 ? part[tid - 1] : -1;
  __syncthreads();
  int64_t sum = 0;
  for (int f = f0; f < f1; ++f) {
    int64_t o, e;
    clip(f, o, e);
    const bool ok = o >= runmax;
    runmax = max(runmax, e);
    sso[f] = o;
    sse[f] = ok ? e : o;
    vf[f] = ok ? 1 : 0;
    const int64_t len = e - o;
    sum += ok ? (len > JP_CHUNK ? (len + JP_CHUNK - 1) / JP_CHUNK : 1) : 0;
  }
  part[tid] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {   // inclusive Hillis-Steele scan
    const int64_t v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int64_t run = part[tid] - sum;
  for (int f = f0; f < f1; ++f) {
    cbase[f] = run;
    const int64_t len = sse[f] - sso[f];
    run += vf[f] ? (len > JP_CHUNK ? (len + JP_CHUNK - 1) / JP_CHUNK : 1) : 0;
    // unstuffed stream: 4-byte aligned, never past the next frame's start (unstuffed <= raw bytes)
    ubase[f] = (sso[f] + 4 * (int64_t)f + 3) & ~(int64_t)3;
  }
  if (tid == 1023) cbase[nframes] = part[1023];
}

__global__ __launch_bounds__(256) void jp_chunk_frame_kernel(const int64_t* __restrict__ cbase, int nframes,
                                                             int32_t* __restrict__ cframe) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= nframes) return;
  for (int64_t c = cbase[f]; c < cbase[f + 1]; ++c) cframe[c] = f;
}

// raw byte i of a frame's scan [s, e): kept unless it is the 0x00 after a 0xFF;
// the first 0xFF not followed by 0x00 (a marker, or the segment's last byte)
// ends the data.  One workgroup per raw chunk, a thread per 4 consecutive
// bytes (coalesced byte reads).
struct JpBytes {   // this thread's 4 bytes: kept mask and the chunk's first marker
  uint8_t c[4];
  int keep;        // bit j: byte j kept (before the marker test)
  int64_t mpos;    // first marker position seen by this thread (INT64_MAX: none)
};

__device__ __forceinline__ JpBytes jp_bytes(const uint8_t* __restrict__ data, int64_t fs, int64_t fe, int64_t i0,
                                            int64_t e) {
  JpBytes r;
  r.keep = 0;
  r.mpos = INT64_MAX;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = i0 + j;
    r.c[j] = 0;
    if (i >= e) continue;
    const uint8_t c = data[i];
    r.c[j] = c;
    if (c == 0x00 && i > fs && data[i - 1] == 0xFF) continue;   // stuffing
    if (c == 0xFF && !(i + 1 < fe && data[i + 1] == 0x00)) {    // a marker: the data ends here
      r.mpos = min(r.mpos, i);
      continue;
    }
    r.keep |= 1 << j;
  }
  return r;
}

// workgroup min of an int64 and exclusive scan of an int over 256 threads
__device__ __forceinline__ int64_t wg_min64(int64_t v, int64_t* sh) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int64_t u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const int64_t m = min(min(sh[0], sh[1]), min(sh[2], sh[3]));
  __syncthreads();
  return m;
}

__device__ __forceinline__ int wg_excl_scan(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += sh[i];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return base + x - v;
}

static_assert(JP_CHUNK == 256 * 4, "one workgroup of 256 threads x 4 bytes per raw chunk");

__global__ __launch_bounds__(256) void jp_unstuff_count_kernel(const uint8_t* __restrict__ data,
                                                               const int64_t* __restrict__ seg_off,
                                                               const int64_t* __restrict__ seg_end, JpChunks ch,
                                                               int32_t* __restrict__ cnt, uint8_t* __restrict__ mk) {
  __shared__ int64_t shm[4];
  __shared__ int shs[4];
  const int64_t ci = blockIdx.x;
  const int f = ch.cframe[ci];
  if (f < 0) return;   // workgroup-uniform
  const int64_t t = ci - ch.cbase[f];
  const int64_t fs = seg_off[f], fe = seg_end[f];
  const int64_t s = fs + t * JP_CHUNK, e = min(fe, s + JP_CHUNK);
  const JpBytes b = jp_bytes(data, fs, fe, s + 4 * threadIdx.x, e);
  const int64_t mpos = wg_min64(b.mpos, shm);
  int n = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) n += ((b.keep >> j) & 1) && s + 4 * (int64_t)threadIdx.x + j < mpos;
  int total;
  (void)wg_excl_scan(n, shs, total);
  if (threadIdx.x == 0) {
    cnt[ci] = total;
    mk[ci] = mpos < e ? 1 : 0;
  }
}

// per frame: exclusive offsets of the chunks' kept bytes (chunks after a marker keep nothing)
__global__ __launch_bounds__(256) void jp_unstuff_scan_kernel(JpChunks ch, int nframes, int32_t* __restrict__ cnt,
                                                              const uint8_t* __restrict__ mk,
                                                              uint32_t* __restrict__ coff, uint32_t* __restrict__ ulen) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= nframes) return;
  uint32_t run = 0;
  bool dead = false;
  for (int64_t c = ch.cbase[f]; c < ch.cbase[f + 1]; ++c) {
    coff[c] = run;
    if (dead) {
      cnt[c] = 0;
      continue;
    }
    run += (uint32_t)cnt[c];
    dead = mk[c] != 0;
  }
  ulen[f] = run;
}

__global__ __launch_bounds__(256) void jp_unstuff_scatter_kernel(const uint8_t* __restrict__ data,
                                                                 const int64_t* __restrict__ seg_off,
                                                                 const int64_t* __restrict__ seg_end, JpChunks ch,
                                                                 const int32_t* __restrict__ cnt,
                                                                 const uint32_t* __restrict__ coff,
                                                                 uint8_t* __restrict__ ustuff) {
  __shared__ int64_t shm[4];
  __shared__ int shs[4];
  const int64_t ci = blockIdx.x;
  const int f = ch.cframe[ci];
  if (f < 0 || cnt[ci] <= 0) return;   // workgroup-uniform (dead chunks keep nothing)
  const int64_t t = ci - ch.cbase[f];
  const int64_t fs = seg_off[f], fe = seg_end[f];
  const int64_t s = fs + t * JP_CHUNK, e = min(fe, s + JP_CHUNK);
  const int64_t i0 = s + 4 * threadIdx.x;
  const JpBytes b = jp_bytes(data, fs, fe, i0, e);
  const int64_t mpos = wg_min64(b.mpos, shm);
  int n = 0, keep = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (((b.keep >> j) & 1) && i0 + j < mpos) {
      keep |= 1 << j;
      ++n;
    }
  int total;
  const int o0 = wg_excl_scan(n, shs, total);
  uint8_t* o = ustuff + ch.ubase[f] + coff[ci] + o0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if ((keep >> j) & 1) *o++ = b.c[j];
}

struct JpState {        // per chunk, per buffer: exit state, blocks completed, DC sums
  uint64_t* x;          // pos << 16 | b << 8 | k  (pos: bit index in the frame's unstuffed stream)
  int32_t* nb;
  int32_t* dc;          // [3] per chunk
  uint8_t* changed;
};

// round 0: every chunk from its first bit in the guessed state (block 0, coefficient 0);
// round r >= 1: chunks whose predecessor's exit changed in round r - 1 re-decode from it
template <bool LDS_T>
__global__ __launch_bounds__(256) void jp_sync_kernel(const uint8_t* __restrict__ ustuff, JpChunks ch,
                                                      int64_t nchunks_max, const JpegHuff* __restrict__ huff,
                                                      const int32_t* __restrict__ huff_idx, int nsets, JpegGeom g,
                                                      JpegMcu mc, int round, JpState src, JpState dst,
                                                      int32_t* __restrict__ frame_changed /* this round's [B] */,
                                                      JpCps cps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (LDS_T) {
    const uint32_t* s = (const uint32_t*)huff;
    uint32_t* d = (uint32_t*)smem;
    const int nw = nsets * 4 * (int)sizeof(JpegHuff) / 4;
    for (int i = threadIdx.x; i < nw; i += 256) d[i] = s[i];
    __syncthreads();
  }
  const int64_t ci = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ci >= nchunks_max) return;
  const int f = ch.cframe[ci];
  if (f < 0) return;
  const int64_t t = ci - ch.cbase[f];
  const uint32_t L = ch.ulen[f];
  const uint32_t first = (uint32_t)t * (JP_CHUNK * 8u);
  if ((uint64_t)t * JP_CHUNK >= L) {   // an empty chunk (the stream is shorter than the raw bytes)
    dst.x[ci] = pack_state(first, 0, 0);
    dst.nb[ci] = 0;
    dst.dc[3 * ci] = dst.dc[3 * ci + 1] = dst.dc[3 * ci + 2] = 0;
    dst.changed[ci] = 0;
    return;
  }
  uint32_t start = first;
  int b = 0, k = 0;
  bool redo = round == 0;
  if (round > 0 && t > 0 && src.changed[ci - 1]) {
    const uint64_t xs = src.x[ci - 1];
    start = (uint32_t)(xs >> 16);
    b = (int)((xs >> 8) & 0xFF);
    k = (int)(xs & 0xFF);
    redo = true;
  }
  if (!redo) {   // nothing upstream changed: keep the state
    dst.x[ci] = src.x[ci];
    dst.nb[ci] = src.nb[ci];
    dst.dc[3 * ci] = src.dc[3 * ci];
    dst.dc[3 * ci + 1] = src.dc[3 * ci + 1];
    dst.dc[3 * ci + 2] = src.dc[3 * ci + 2];
    dst.changed[ci] = 0;
    return;
  }
  const int set = huff_idx ? huff_idx[f] : f;
  const JpegHuff* T = (LDS_T ? (const JpegHuff*)smem : huff) + (int64_t)set * 4;
  const uint32_t stop = (uint64_t)(t + 1) * JP_CHUNK >= L ? L * 8u : first + JP_CHUNK * 8u;
  UReader br;
  br.init_at(ustuff + ch.ubase[f], L, start);
  int nblk = 0;
  int dc[3] = {0, 0, 0};
  JpCpRun cr{first, first + JP_CP_FIRST, 0, -1, round > 0, ci * JP_NCP, cps};
  __builtin_amdgcn_s_waitcnt(0);   // nothing in flight entering the loop (see jpeg_entropy_kernel)
  jp_run<false, true>(br, T, g, mc, b, k, stop, 0, 0, nblk, dc, nullptr, true, &cr);
  uint64_t x;
  if (cr.hit >= 0) {
    // joined the recorded path at checkpoint hit: its exit, and its counts from there on.
    // Re-base the recorded checkpoints from hit on (and the totals) to this decode's start;
    // those before hit were just re-recorded by this decode.
    const int64_t sh = cr.slot + cr.hit;
    const int dn = nblk - cps.nb[sh];
    const int d0 = dc[0] - cps.dc[3 * sh], d1 = dc[1] - cps.dc[3 * sh + 1], d2 = dc[2] - cps.dc[3 * sh + 2];
    for (int jj = cr.hit; jj < JP_NCP; ++jj) {
      const int64_t sl = cr.slot + jj;
      cps.nb[sl] += dn;
      cps.dc[3 * sl] += d0;
      cps.dc[3 * sl + 1] += d1;
      cps.dc[3 * sl + 2] += d2;
    }
    cps.tn[ci] += dn;
    cps.td[3 * ci] += d0;
    cps.td[3 * ci + 1] += d1;
    cps.td[3 * ci + 2] += d2;
    x = src.x[ci];
    nblk = cps.tn[ci];
    dc[0] = cps.td[3 * ci];
    dc[1] = cps.td[3 * ci + 1];
    dc[2] = cps.td[3 * ci + 2];
  } else {   // decoded to the chunk's end: this path is the record now
    for (int jj = cr.j; jj < JP_NCP; ++jj) cps.x[cr.slot + jj] = ~0ull;
    cps.tn[ci] = nblk;
    cps.td[3 * ci] = dc[0];
    cps.td[3 * ci + 1] = dc[1];
    cps.td[3 * ci + 2] = dc[2];
    x = pack_state(br.pos, b, k);
  }
  dst.x[ci] = x;
  dst.nb[ci] = nblk;
  dst.dc[3 * ci] = dc[0];
  dst.dc[3 * ci + 1] = dc[1];
  dst.dc[3 * ci + 2] = dc[2];
  const bool ch_ = round == 0 ? true : x != src.x[ci];
  dst.changed[ci] = ch_ ? 1 : 0;
  if (ch_ && round > 0) frame_changed[f] = 1;
}

// per frame: each chunk's first block and DC predictors (exclusive prefix sums)
__global__ __launch_bounds__(256) void jp_prefix_kernel(JpChunks ch, int nframes, JpState st,
                                                        int64_t* __restrict__ bfirst, int32_t* __restrict__ pred) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= nframes) return;
  int64_t blk = 0;
  int p0 = 0, p1 = 0, p2 = 0;
  for (int64_t c = ch.cbase[f]; c < ch.cbase[f + 1]; ++c) {
    bfirst[c] = blk;
    pred[3 * c] = p0;
    pred[3 * c + 1] = p1;
    pred[3 * c + 2] = p2;
    blk += st.nb[c];
    p0 += st.dc[3 * c];
    p1 += st.dc[3 * c + 1];
    p2 += st.dc[3 * c + 2];
  }
}

template <bool LDS_T>
__global__ __launch_bounds__(256) void jp_final_kernel(const uint8_t* __restrict__ ustuff, JpChunks ch,
                                                       int64_t nchunks_max, const JpegHuff* __restrict__ huff,
                                                       const int32_t* __restrict__ huff_idx, int nsets, JpegGeom g,
                                                       JpegMcu mc, JpState st, const int64_t* __restrict__ bfirst,
                                                       const int32_t* __restrict__ pred,
                                                       const int32_t* __restrict__ frame_changed,
                                                       int16_t* __restrict__ coef, int abl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  JpegHuff* sh = (JpegHuff*)smem;
  if (LDS_T) {
    const uint32_t* s = (const uint32_t*)huff;
    uint32_t* d = (uint32_t*)smem;
    const int nw = nsets * 4 * (int)sizeof(JpegHuff) / 4;
    for (int i = threadIdx.x; i < nw; i += 256) d[i] = s[i];
  }
  __syncthreads();
  const int64_t ci = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ci >= nchunks_max) return;
  const int f = ch.cframe[ci];
  if (f < 0) return;
  const int64_t t = ci - ch.cbase[f];
  const uint32_t L = ch.ulen[f];
  const bool serial = frame_changed[f] != 0;   // still changing after the last round: decode the frame serially
  if (serial && t > 0) return;
  if (!serial && t > 0 && (uint64_t)t * JP_CHUNK >= L) return;   // empty chunk
  const int64_t total = (int64_t)g.mcux * g.mcuy * mc.bpm;
  uint32_t start = 0;
  int b = 0, k = 0;
  int64_t blk = 0;
  int dc[3] = {0, 0, 0};
  if (!serial && t > 0) {
    const uint64_t xs = st.x[ci - 1];
    start = (uint32_t)(xs >> 16);
    b = (int)((xs >> 8) & 0xFF);
    k = (int)(xs & 0xFF);
    blk = bfirst[ci];
    dc[0] = pred[3 * ci];
    dc[1] = pred[3 * ci + 1];
    dc[2] = pred[3 * ci + 2];
  }
  const bool last = serial || (uint64_t)(t + 1) * JP_CHUNK >= L;
  const uint32_t stop = last ? 0xFFFFFFFFu : (uint32_t)(t + 1) * (JP_CHUNK * 8u);
  const int set = huff_idx ? huff_idx[f] : f;
  const JpegHuff* T = (LDS_T ? (const JpegHuff*)sh : huff) + (int64_t)set * 4;
  UReader br;
  br.init_at(ustuff + ch.ubase[f], L, start);
  int nblk = 0;
  __builtin_amdgcn_s_waitcnt(0);
  jp_run<true>(br, T, g, mc, b, k, stop, blk, total, nblk, dc, coef + (int64_t)f * g.blocks_per_frame * 64,
               !(abl & 1));
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
  int32_t zv[64], in[64];   // zv: the block's zigzag slots; in: natural order, dequantised
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint4 v = cb4[j];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      zv[8 * j + 2 * e] = (int32_t)(int16_t)(w[e] & 0xFFFF);
      zv[8 * j + 2 * e + 1] = (int32_t)(int16_t)(w[e] >> 16);
    }
  }
#pragma unroll
  for (int n = 0; n < 64; ++n) in[n] = zv[kIzz[n]] * (int32_t)q[n];
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

// RGB of output pixel t (frame-major over nframes x W x H)
__device__ __forceinline__ uint32_t color_px(const uint8_t* __restrict__ planes, const JpegPlanes& pl, int W,
                                             int64_t px, int ncomp, int cmode, int cdw, int cdh, int64_t t) {
  const int f = (int)(t / px);
  const int64_t p = t - (int64_t)f * px;
  const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
  const uint8_t* base = planes + (int64_t)f * pl.plane_frame_bytes;
  const int Y = base[pl.pbase[0] + (int64_t)y * pl.pstride[0] + x];
  if (ncomp == 1) return (uint32_t)Y * 0x010101u;
  const int cb = chroma_at(base + pl.pbase[1], pl.pstride[1], cdw, cdh, x, y, cmode) - 128;
  const int cr = chroma_at(base + pl.pbase[2], pl.pstride[2], cdw, cdh, x, y, cmode) - 128;
  // FIX(x) = (int)(x * 65536 + 0.5); ONE_HALF = 1 << 15; arithmetic right shifts
  const int r = Y + ((91881 * cr + 32768) >> 16);
  const int gch = Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
  const int b = Y + ((116130 * cb + 32768) >> 16);
  return (uint32_t)clamp255(r) | ((uint32_t)clamp255(gch) << 8) | ((uint32_t)clamp255(b) << 16);
}

// one thread per 4 consecutive output pixels: 12 bytes as three dword stores
// (the per-pixel byte stores ran the kernel at ~0.5 TB/s of output)
__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t* __restrict__ planes, JpegPlanes pl, int W, int H,
                                                         int ncomp, int cmode, int cdw, int cdh, int nframes,
                                                         uint8_t* __restrict__ rgb) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t px = (int64_t)W * H, n = (int64_t)nframes * px;
  const int64_t t0 = 4 * g;
  if (t0 >= n) return;
  if (t0 + 4 <= n && ((uintptr_t)(rgb + t0 * 3) & 3) == 0) {
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = color_px(planes, pl, W, px, ncomp, cmode, cdw, cdh, t0 + j);
    uint32_t* o = (uint32_t*)(rgb + t0 * 3);
    o[0] = c[0] | (c[1] << 24);
    o[1] = (c[1] >> 8) | (c[2] << 16);
    o[2] = (c[2] >> 16) | (c[3] << 8);
    return;
  }
  for (int64_t t = t0; t < n && t < t0 + 4; ++t) {   // tail
    const uint32_t c = color_px(planes, pl, W, px, ncomp, cmode, cdw, cdh, t);
    rgb[t * 3] = (uint8_t)c;
    rgb[t * 3 + 1] = (uint8_t)(c >> 8);
    rgb[t * 3 + 2] = (uint8_t)(c >> 16);
  }
}

// ---- fused colour conversion + Pillow resample + crop + ToTensor/Normalize (mi_jpeg_decode_transform)
// The RGB frame of jpeg_color_kernel never reaches HBM: one workgroup per (frame, band of
// output rows) converts the source rows the band's vertical taps need (only the crop's source
// columns) into LDS a few rows at a time, resamples each horizontally into LDS, then resamples
// vertically and normalises.  Every step is the same integer arithmetic as color_px and
// preprocess.hip's resample_h / resample_v kernels, so the output is bit-identical to decode +
// mi_preprocess_frames (and so to Pillow + torchvision).
constexpr int XF_PREC = 22;   // Pillow PRECISION_BITS
constexpr int XF_RPI = 8;     // source rows converted per step
constexpr int XF_NT = 512;    // threads per workgroup (two workgroups per CU: <= XF_LDS2 bytes of LDS each)
constexpr int XF_IPT = 3;     // 4-pixel groups per thread whose loads go out together in a conversion step
constexpr size_t XF_LDS2 = 78 * 1024;

__device__ __forceinline__ uint32_t xf_clip8(int acc) {
  acc >>= XF_PREC;
  return acc < 0 ? 0u : (acc > 255 ? 255u : (uint32_t)acc);
}

// RGB of pixel (x, y) of one frame's planes (color_px without the frame-major index)
__device__ __forceinline__ uint32_t color_xy(const uint8_t* __restrict__ base, const JpegPlanes& pl, int ncomp,
                                             int cmode, int cdw, int cdh, int x, int y) {
  const int Y = base[pl.pbase[0] + (int64_t)y * pl.pstride[0] + x];
  if (ncomp == 1) return (uint32_t)Y * 0x010101u;
  const int cb = chroma_at(base + pl.pbase[1], pl.pstride[1], cdw, cdh, x, y, cmode) - 128;
  const int cr = chroma_at(base + pl.pbase[2], pl.pstride[2], cdw, cdh, x, y, cmode) - 128;
  const int r = Y + ((91881 * cr + 32768) >> 16);
  const int gch = Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
  const int b = Y + ((116130 * cb + 32768) >> 16);
  return (uint32_t)clamp255(r) | ((uint32_t)clamp255(gch) << 8) | ((uint32_t)clamp255(b) << 16);
}

// RGB of the 4 pixels x0 .. x0 + 3 of row y (x0 % 4 == 0, 1 <= x0, x0 + 4 < W: no chroma edge
// column): one dword of Y and one (unaligned) dword per chroma row instead of a byte load per
// sample; the same fancy-upsampling / colour arithmetic as chroma_at + color_px
// 4 bytes at any address as one value: the two aligned dwords around them, byte-aligned
__device__ __forceinline__ uint32_t load4u(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}

// color4 in two halves, so that a thread's loads for several 4-pixel groups are all in
// flight before the first group's arithmetic waits: the raw dwords (Y, then the chroma words
// the fancy upsampling reads, by cmode), then the colour conversion from them
struct Raw4 {
  uint32_t y, b0, b1, r0, r1;   // cmode 0: b0 / r0; 1: b0 / r0 (c0 .. c0 + 3); 2: near b0 / r0, far b1 / r1
};

__device__ __forceinline__ Raw4 color4_load(const uint8_t* __restrict__ base, const JpegPlanes& pl, int cmode,
                                            int cdh, int x0, int y) {
  Raw4 w;
  // planes are 64-byte aligned with row strides of whole blocks: the Y dword is aligned
  w.y = *(const uint32_t*)(base + pl.pbase[0] + (int64_t)y * pl.pstride[0] + x0);
  w.b1 = w.r1 = 0u;
  if (cmode == 0) {
    w.b0 = *(const uint32_t*)(base + pl.pbase[1] + (int64_t)y * pl.pstride[1] + x0);
    w.r0 = *(const uint32_t*)(base + pl.pbase[2] + (int64_t)y * pl.pstride[2] + x0);
  } else {
    const int c0 = (x0 >> 1) - 1;   // chroma columns c0 .. c0 + 3 serve the 4 pixels
    const int r = cmode == 1 ? y : y >> 1;
    w.b0 = load4u(base + pl.pbase[1] + (int64_t)r * pl.pstride[1] + c0);
    w.r0 = load4u(base + pl.pbase[2] + (int64_t)r * pl.pstride[2] + c0);
    if (cmode == 2) {
      const int rf = (y & 1) ? min(r + 1, cdh - 1) : max(r - 1, 0);
      w.b1 = load4u(base + pl.pbase[1] + (int64_t)rf * pl.pstride[1] + c0);
      w.r1 = load4u(base + pl.pbase[2] + (int64_t)rf * pl.pstride[2] + c0);
    }
  }
  return w;
}

// RGB of the 4 pixels x0 .. x0 + 3 of row y (x0 % 4 == 0, 1 <= x0, x0 + 4 < W: no chroma edge
// column) from color4_load's words; the same fancy-upsampling / colour arithmetic as
// chroma_at + color_px
__device__ __forceinline__ void color4_math(const Raw4& w, int cmode, uint32_t* __restrict__ o) {
  int cb[4], cr[4];
  if (cmode == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cb[i] = (int)((w.b0 >> (8 * i)) & 255u);
      cr[i] = (int)((w.r0 >> (8 * i)) & 255u);
    }
  } else {
    int tb[4], tr[4];
    if (cmode == 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tb[k] = (int)((w.b0 >> (8 * k)) & 255u);
        tr[k] = (int)((w.r0 >> (8 * k)) & 255u);
      }
      // h2v1_fancy_upsample: even pixel (v * 3 + left + 1) >> 2, odd (v * 3 + right + 2) >> 2
      cb[0] = (tb[1] * 3 + tb[0] + 1) >> 2;
      cb[1] = (tb[1] * 3 + tb[2] + 2) >> 2;
      cb[2] = (tb[2] * 3 + tb[1] + 1) >> 2;
      cb[3] = (tb[2] * 3 + tb[3] + 2) >> 2;
      cr[0] = (tr[1] * 3 + tr[0] + 1) >> 2;
      cr[1] = (tr[1] * 3 + tr[2] + 2) >> 2;
      cr[2] = (tr[2] * 3 + tr[1] + 1) >> 2;
      cr[3] = (tr[2] * 3 + tr[3] + 2) >> 2;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tb[k] = (int)((w.b0 >> (8 * k)) & 255u) * 3 + (int)((w.b1 >> (8 * k)) & 255u);
        tr[k] = (int)((w.r0 >> (8 * k)) & 255u) * 3 + (int)((w.r1 >> (8 * k)) & 255u);
      }
      // h2v2_fancy_upsample: even pixel (th * 3 + left + 8) >> 4, odd (th * 3 + right + 7) >> 4
      cb[0] = (tb[1] * 3 + tb[0] + 8) >> 4;
      cb[1] = (tb[1] * 3 + tb[2] + 7) >> 4;
      cb[2] = (tb[2] * 3 + tb[1] + 8) >> 4;
      cb[3] = (tb[2] * 3 + tb[3] + 7) >> 4;
      cr[0] = (tr[1] * 3 + tr[0] + 8) >> 4;
      cr[1] = (tr[1] * 3 + tr[2] + 7) >> 4;
      cr[2] = (tr[2] * 3 + tr[1] + 8) >> 4;
      cr[3] = (tr[2] * 3 + tr[3] + 7) >> 4;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int Y = (int)((w.y >> (8 * i)) & 255u);
    const int b_ = cb[i] - 128, r_ = cr[i] - 128;
    const int r = Y + ((91881 * r_ + 32768) >> 16);
    const int gch = Y + ((-22554 * b_ + 32768 - 46802 * r_) >> 16);
    const int b = Y + ((116130 * b_ + 32768) >> 16);
    o[i] = (uint32_t)clamp255(r) | ((uint32_t)clamp255(gch) << 8) | ((uint32_t)clamp255(b) << 16);
  }
}

struct XformK {
  const int32_t *kh, *bh, *kv, *bv;   // preprocess.hip's tables (ResampleTables)
  int ksh, ksv, n, xlo, xw, W;        // xlo % 4 == 0, xw % 4 == 0 (the span rounded out)
  int band, nbands, rows_max;         // output rows per workgroup; LDS rows for the widest band
  int i24;                            // every |coefficient| < 2^23: 24-bit multiplies are exact
  float mean[3], sd[3];
};

// pixel (0..255) x Pillow coefficient: with |w| < 2^23 both fit 24-bit signed operands and the
// product 31 bits, so v_mul_i32_i24 (full rate; v_mul_lo_u32 is quarter rate) is exact
template <bool I24>
__device__ __forceinline__ int xf_mul(uint32_t pix, int w) {
  // (w << 8) >> 8 is w itself when it fits 24 bits; it tells the backend so (v_mul_i32_i24 / v_mad_i32_i24)
  return I24 ? (int)pix * ((w << 8) >> 8) : (int)pix * w;
}

template <bool OUT_BF16, bool I24>
__global__ __launch_bounds__(XF_NT) void jpeg_transform_kernel(const uint8_t* __restrict__ planes, JpegPlanes pl,
                                                             int ncomp, int cmode, int cdw, int cdh, XformK xk,
                                                             void* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char xsm[];
  const int f = (int)(blockIdx.x / xk.nbands), band = (int)(blockIdx.x % xk.nbands);
  const int n = xk.n, xw = xk.xw;   // xw: the crop's source span rounded out to whole 4-pixel groups
  const int y0 = band * xk.band, y1 = min(n, y0 + xk.band), ny = y1 - y0;
  const int ra = xk.bv[2 * y0];
  int rb = ra;
  for (int y = y0; y < y1; ++y) rb = max(rb, xk.bv[2 * y] + xk.bv[2 * y + 1]);
  // LDS: the filter tables (the band's rows of the vertical one), then the converted source
  // rows of one step, then the band's horizontally resampled rows
  int32_t* skh = (int32_t*)xsm;                      // [n][ksh]
  int32_t* sbh = skh + n * xk.ksh;                   // [n] xmin - xlo | xsize << 16
  int32_t* skv = sbh + n;                            // [band][ksv]
  int32_t* sbv = skv + xk.band * xk.ksv;             // [band] ymin - ra | ysize << 16
  uint32_t* crow = (uint32_t*)(sbv + xk.band);       // [XF_RPI][xw] packed RGB of the source rows
  uint32_t* hrow = crow + XF_RPI * xw;               // [rb - ra][n] the horizontal pass's rows
  for (int i = threadIdx.x; i < n * xk.ksh; i += XF_NT) skh[i] = xk.kh[i];
  for (int i = threadIdx.x; i < n; i += XF_NT) sbh[i] = (xk.bh[2 * i] - xk.xlo) | (xk.bh[2 * i + 1] << 16);
  for (int i = threadIdx.x; i < ny * xk.ksv; i += XF_NT) skv[i] = xk.kv[(int64_t)y0 * xk.ksv + i];
  for (int i = threadIdx.x; i < ny; i += XF_NT) sbv[i] = (xk.bv[2 * (y0 + i)] - ra) | (xk.bv[2 * (y0 + i) + 1] << 16);
  const uint8_t* base = planes + (int64_t)f * pl.plane_frame_bytes;
  const int xq = xw >> 2;
  // source rows per step: as many as one thread's XF_IPT 4-pixel groups cover (<= XF_RPI, the
  // LDS rows), so a step's conversion loads go out together, before the previous step's
  // horizontal pass, which then runs under their latency
  const int rps = max(1, min(XF_RPI, XF_NT * XF_IPT / xq));
  Raw4 raw[XF_IPT];
  int ix[XF_IPT];
  auto issue = [&](int r0) {
    const int items = min(rps, rb - r0) * xq;
#pragma unroll
    for (int m = 0; m < XF_IPT; ++m) {
      const int i = threadIdx.x + m * XF_NT;
      const int rr = i / xq, x0 = xk.xlo + 4 * (i - rr * xq);
      ix[m] = i < items ? (ncomp == 3 && x0 >= 4 && x0 + 8 <= xk.W ? 1 : 2) : 0;   // 1 fast, 2 edge
      if (ix[m] == 1) raw[m] = color4_load(base, pl, cmode, cdh, x0, r0 + rr);
    }
  };
  auto convert = [&](int r0) {
#pragma unroll
    for (int m = 0; m < XF_IPT; ++m) {
      if (ix[m] != 1) continue;
      const int i = threadIdx.x + m * XF_NT;
      const int rr = i / xq, x0 = xk.xlo + 4 * (i - rr * xq);
      uint32_t c4[4];
      color4_math(raw[m], cmode, c4);
      *(uint4*)(crow + rr * xw + (x0 - xk.xlo)) = make_uint4(c4[0], c4[1], c4[2], c4[3]);
    }
    // groups at the frame's left / right edge (or one-component frames): pixel by pixel, rolled
#pragma unroll 1
    for (int m = 0; m < XF_IPT; ++m) {
      if (ix[m] != 2) continue;
      const int i = threadIdx.x + m * XF_NT;
      const int rr = i / xq, x0 = xk.xlo + 4 * (i - rr * xq), y = r0 + rr;
      uint32_t* o = crow + rr * xw + (x0 - xk.xlo);
#pragma unroll 1
      for (int j = 0; j < 4; ++j)
        o[j] = x0 + j < xk.W ? color_xy(base, pl, ncomp, cmode, cdw, cdh, x0 + j, y) : 0u;
    }
  };
  issue(ra);
  for (int r0 = ra; r0 < rb; r0 += rps) {
    const int nr = min(rps, rb - r0);
    convert(r0);
    __syncthreads();
    if (r0 + rps < rb) issue(r0 + rps);
    for (int i = threadIdx.x; i < nr * n; i += XF_NT) {   // resample_h_kernel's sums
      const int rr = i / n, ox = i - rr * n;
      const int bh = sbh[ox], xb = bh & 0xFFFF, xs = bh >> 16;
      const int32_t* k = skh + ox * xk.ksh;
      const uint32_t* p = crow + rr * xw + xb;
      int s0 = 1 << (XF_PREC - 1), s1 = s0, s2 = s0;
      for (int j = 0; j < xs; ++j) {
        const uint32_t v = p[j];
        const int w = k[j];
        s0 += xf_mul<I24>(v & 255u, w);
        s1 += xf_mul<I24>((v >> 8) & 255u, w);
        s2 += xf_mul<I24>((v >> 16) & 255u, w);
      }
      hrow[(r0 - ra + rr) * n + ox] = xf_clip8(s0) | (xf_clip8(s1) << 8) | (xf_clip8(s2) << 16);
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < ny * n; i += XF_NT) {   // resample_v_kernel's sums + ToTensor / Normalize
    const int yy = i / n, x = i - yy * n, y = y0 + yy;
    const int bv = sbv[yy], yb = bv & 0xFFFF, ys = bv >> 16;
    const int32_t* k = skv + yy * xk.ksv;
    int sc[3] = {1 << (XF_PREC - 1), 1 << (XF_PREC - 1), 1 << (XF_PREC - 1)};
    for (int j = 0; j < ys; ++j) {
      const uint32_t v = hrow[(yb + j) * n + x];
      const int w = k[j];
      sc[0] += xf_mul<I24>(v & 255u, w);
      sc[1] += xf_mul<I24>((v >> 8) & 255u, w);
      sc[2] += xf_mul<I24>((v >> 16) & 255u, w);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = ((float)xf_clip8(sc[c]) / 255.0f - xk.mean[c]) / xk.sd[c];
      const int64_t o = (((int64_t)f * 3 + c) * n + y) * (int64_t)n + x;
      if (OUT_BF16) ((uint16_t*)out)[o] = f2bf(v);
      else ((float*)out)[o] = v;
    }
  }
}

}  // namespace

// Workspace of the chunked entropy decode (after the coefficients and planes).
struct JpWs {
  size_t bytes;
  size_t o_ustuff, o_cbase, o_ubase, o_ulen, o_cframe, o_cnt, o_coff, o_mk, o_x[2], o_nb[2], o_dc[2], o_ch[2],
      o_bfirst, o_pred, o_fch, o_sso, o_sse, o_vf, o_cpx, o_cpn, o_cpd, o_tn, o_td;
  int64_t nmax;
};

static JpWs jp_layout(int nframes, int64_t data_bytes) {
  JpWs w{};
  size_t off = 0;
  auto carve = [&](size_t n) { const size_t o = off; off += (n + 255) & ~(size_t)255; return o; };
  const int64_t B = nframes;
  w.nmax = data_bytes / JP_CHUNK + B + 1;   // >= sum over frames of max(1, ceil(raw bytes / JP_CHUNK))
  w.o_ustuff = carve((size_t)data_bytes + 4 * (size_t)B + 64);
  w.o_cbase = carve((size_t)(B + 1) * 8);
  w.o_ubase = carve((size_t)B * 8);
  w.o_ulen = carve((size_t)B * 4);
  w.o_cframe = carve((size_t)w.nmax * 4);
  w.o_cnt = carve((size_t)w.nmax * 4);
  w.o_coff = carve((size_t)w.nmax * 4);
  w.o_mk = carve((size_t)w.nmax);
  for (int i = 0; i < 2; ++i) {
    w.o_x[i] = carve((size_t)w.nmax * 8);
    w.o_nb[i] = carve((size_t)w.nmax * 4);
    w.o_dc[i] = carve((size_t)w.nmax * 12);
    w.o_ch[i] = carve((size_t)w.nmax);
  }
  w.o_bfirst = carve((size_t)w.nmax * 8);
  w.o_pred = carve((size_t)w.nmax * 12);
  w.o_fch = carve((size_t)(JP_ROUNDS + 1) * B * 4);
  w.o_sso = carve((size_t)B * 8);
  w.o_sse = carve((size_t)B * 8);
  w.o_vf = carve((size_t)B);
  w.o_cpx = carve((size_t)w.nmax * JP_NCP * 8);
  w.o_cpn = carve((size_t)w.nmax * JP_NCP * 4);
  w.o_cpd = carve((size_t)w.nmax * JP_NCP * 12);
  w.o_tn = carve((size_t)w.nmax * 4);
  w.o_td = carve((size_t)w.nmax * 12);
  w.bytes = off;
  return w;
}

// A/B timing probes (MICLIP_JPEG_ABL): bit 0 = the final pass decodes without storing coefficients
static int jp_abl() {
#if MICLIP_AB
  const char* e = getenv("MICLIP_JPEG_ABL");
  return e ? atoi(e) : 0;
#else
  return 0;
#endif
}

static bool jp_serial_forced() {
#if MICLIP_AB
  const char* e = getenv("MICLIP_JPEG_SERIAL");   // A/B: the lane-per-frame entropy kernel for every scan
  return e && e[0] == '1';
#else
  return false;
#endif
}

// The fused transform's launch shape: output rows per workgroup (band) and LDS bytes -- the
// filter tables, XF_RPI converted source rows and the widest band's source rows of horizontal
// output -- the widest band (16, halved) that fits two workgroups per CU, else one.
hipError_t jpeg_xform_plan(int H, int W, int n, int mode, XformK& xk, size_t& lds) {
  ResampleTables t;
  const hipError_t e = resample_tables(H, W, n, mode, t);
  if (e != hipSuccess) return e;
  xk.kh = t.kh;
  xk.bh = t.bh;
  xk.kv = t.kv;
  xk.bv = t.bv;
  xk.ksh = t.ksh;
  xk.ksv = t.ksv;
  xk.n = n;
  xk.xlo = t.xlo & ~3;                          // whole 4-pixel groups (color4); columns past W
  xk.xw = ((t.xlo + t.xw + 3) & ~3) - xk.xlo;   // are never read by the taps
  xk.W = W;
  xk.i24 = t.wmax < (1 << 23);
  if (xk.xw / 4 > XF_NT * XF_IPT) return hipErrorInvalidValue;   // wider than one step's row: decode + preprocess
  // torchvision's Normalize constants: Python floats -> float32 (preprocess.hip)
  const float mean[3] = {(float)0.48145466, (float)0.4578275, (float)0.40821073};
  const float sd[3] = {(float)0.26862954, (float)0.26130258, (float)0.27577711};
  for (int c = 0; c < 3; ++c) {
    xk.mean[c] = mean[c];
    xk.sd[c] = sd[c];
  }
  // the widest band that leaves two workgroups per CU (<= XF_LDS2), else one (<= 150 KB)
  for (const size_t cap : {XF_LDS2, (size_t)150 * 1024}) {
    for (int band = 16; band >= 1; band /= 2) {
      int rows_max = 0;
      for (int y0 = 0; y0 < n; y0 += band) {
        const int y1 = std::min(n, y0 + band);
        int rb = t.hbv[2 * y0];
        for (int y = y0; y < y1; ++y) rb = std::max(rb, t.hbv[2 * y] + t.hbv[2 * y + 1]);
        rows_max = std::max(rows_max, rb - t.hbv[2 * y0]);
      }
      lds = ((size_t)n * (xk.ksh + 1) + (size_t)band * (xk.ksv + 1) + (size_t)XF_RPI * xk.xw + (size_t)rows_max * n) * 4;
      if (lds <= cap && xk.xw < 65536 && rows_max < 65536) {
        xk.band = band;
        xk.nbands = (n + band - 1) / band;
        xk.rows_max = rows_max;
        return hipSuccess;
      }
    }
  }
  return hipErrorInvalidValue;   // a source too wide / tall for one band in LDS: decode + preprocess instead
}

// Whether the fused transform has a launch plan for H x W -> n (mi_jpeg_decode_transform checks
// this before any decode work is queued)
bool jpeg_xform_fits(int H, int W, int n, int mode) {
  XformK xk{};
  size_t lds = 0;
  return jpeg_xform_plan(H, W, n, mode, xk, lds) == hipSuccess;
}

// Host launch: see include/miclip.h mi_jpeg_decode for the argument contract.
hipError_t jpeg_decode(const uint8_t* data, int64_t data_bytes, const int64_t* seg_off, const int64_t* seg_end,
                       const void* huff, const int32_t* huff_idx, int nsets, const uint16_t* qtab, const int32_t* geom,
                       int nframes, uint8_t* out_rgb, void* ws, size_t ws_bytes, hipStream_t s, const JpegXform* xf) {
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
  const size_t base_bytes = (coef_bytes + (size_t)nframes * bytes + 255) & ~(size_t)255;
  const bool chunked = g.nseg == 1 && !jp_serial_forced();
  const JpWs jw = jp_layout(nframes, data_bytes);
  if (ws_bytes < base_bytes + (chunked ? jw.bytes : 0)) return hipErrorInvalidValue;
  int16_t* coef = (int16_t*)ws;
  uint8_t* planes = (uint8_t*)ws + coef_bytes;
  hipError_t e = hipMemsetAsync(coef, 0, coef_bytes, s);
  if (e != hipSuccess) return e;
  const bool lds_t = huff_idx && nsets >= 1 && nsets <= JPEG_LDS_SETS;
  if (chunked) {
    char* w = (char*)ws + base_bytes;
    uint8_t* ustuff = (uint8_t*)(w + jw.o_ustuff);
    int64_t* cbase = (int64_t*)(w + jw.o_cbase);
    int64_t* ubase = (int64_t*)(w + jw.o_ubase);
    uint32_t* ulen = (uint32_t*)(w + jw.o_ulen);
    int32_t* cframe = (int32_t*)(w + jw.o_cframe);
    int32_t* cnt = (int32_t*)(w + jw.o_cnt);
    uint32_t* coff = (uint32_t*)(w + jw.o_coff);
    uint8_t* mk = (uint8_t*)(w + jw.o_mk);
    JpState st[2];
    for (int i = 0; i < 2; ++i)
      st[i] = JpState{(uint64_t*)(w + jw.o_x[i]), (int32_t*)(w + jw.o_nb[i]), (int32_t*)(w + jw.o_dc[i]),
                      (uint8_t*)(w + jw.o_ch[i])};
    int64_t* bfirst = (int64_t*)(w + jw.o_bfirst);
    int32_t* pred = (int32_t*)(w + jw.o_pred);
    int32_t* fch = (int32_t*)(w + jw.o_fch);
    int64_t* sso = (int64_t*)(w + jw.o_sso);
    int64_t* sse = (int64_t*)(w + jw.o_sse);
    uint8_t* vf = (uint8_t*)(w + jw.o_vf);
    const JpCps cps{(uint64_t*)(w + jw.o_cpx), (int32_t*)(w + jw.o_cpn), (int32_t*)(w + jw.o_cpd),
                    (int32_t*)(w + jw.o_tn), (int32_t*)(w + jw.o_td)};
    const int64_t nmax = jw.nmax;
    if ((e = hipMemsetAsync(cframe, 0xFF, (size_t)nmax * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(fch, 0, (size_t)(JP_ROUNDS + 1) * nframes * 4, s)) != hipSuccess) return e;
    // block walk of one MCU (component order, then rows, then columns within the component)
    JpegMcu mc{};
    for (int c = 0; c < ncomp; ++c)
      for (int bv = 0; bv < g.vs[c]; ++bv)
        for (int bh = 0; bh < g.hs[c]; ++bh) {
          mc.comp[mc.bpm] = (int8_t)c;
          mc.dh[mc.bpm] = (int8_t)bh;
          mc.dv[mc.bpm] = (int8_t)bv;
          ++mc.bpm;
        }
    const dim3 fg((unsigned)((nframes + 255) / 256)), cg((unsigned)((nmax + 255) / 256)),
        fg4((unsigned)((nframes + 63) / 64));
    hipLaunchKernelGGL(jp_layout_kernel, dim3(1), dim3(1024), 0, s, seg_off, seg_end, nframes, data_bytes, cbase, ubase,
                       sso, sse, vf);
    hipLaunchKernelGGL(jp_chunk_frame_kernel, fg, dim3(256), 0, s, cbase, nframes, cframe);
    const JpChunks ch{cbase, cframe, ubase, ulen};
    hipLaunchKernelGGL(jp_unstuff_count_kernel, dim3((unsigned)nmax), dim3(256), 0, s, data, sso, sse, ch, cnt, mk);
    hipLaunchKernelGGL(jp_unstuff_scan_kernel, fg, dim3(256), 0, s, ch, nframes, cnt, mk, coff, ulen);
    hipLaunchKernelGGL(jp_unstuff_scatter_kernel, dim3((unsigned)nmax), dim3(256), 0, s, data, sso, sse, ch, cnt, coff,
                       ustuff);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const size_t tl = lds_t ? nsets * 4 * sizeof(JpegHuff) : 0;
    for (int r = 0; r <= JP_ROUNDS; ++r) {
      const JpState& src = st[(r + 1) & 1];   // round r reads round r - 1's buffer
      const JpState& dst = st[r & 1];
      if (lds_t)
        hipLaunchKernelGGL(jp_sync_kernel<true>, cg, dim3(256), tl, s, ustuff, ch, nmax, (const JpegHuff*)huff,
                           huff_idx, nsets, g, mc, r, src, dst, fch + (int64_t)r * nframes, cps);
      else
        hipLaunchKernelGGL(jp_sync_kernel<false>, cg, dim3(256), 0, s, ustuff, ch, nmax, (const JpegHuff*)huff,
                           huff_idx, nsets, g, mc, r, src, dst, fch + (int64_t)r * nframes, cps);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const JpState& fin = st[JP_ROUNDS & 1];
    hipLaunchKernelGGL(jp_prefix_kernel, fg, dim3(256), 0, s, ch, nframes, fin, bfirst, pred);
    const int32_t* last_changed = fch + (int64_t)JP_ROUNDS * nframes;
    if (lds_t)
      hipLaunchKernelGGL(jp_final_kernel<true>, cg, dim3(256), tl, s, ustuff, ch, nmax, (const JpegHuff*)huff,
                         huff_idx, nsets, g, mc, fin, bfirst, pred, last_changed, coef, jp_abl());
    else
      hipLaunchKernelGGL(jp_final_kernel<false>, cg, dim3(256), 0, s, ustuff, ch, nmax, (const JpegHuff*)huff,
                         huff_idx, nsets, g, mc, fin, bfirst, pred, last_changed, coef, jp_abl());
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // frames outside the chunk layout (repeated / out-of-order segments): the serial decode
    hipLaunchKernelGGL(jpeg_entropy_kernel<false>, fg4, dim3(64), 0, s, data, seg_off, seg_end, (const JpegHuff*)huff,
                       huff_idx, nsets, g, nframes, coef, data_bytes, (const uint8_t*)vf);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  } else {
    const int64_t lanes = (int64_t)nframes * g.nseg;
    const dim3 eg((unsigned)((lanes + 63) / 64));
    if (lds_t)
      hipLaunchKernelGGL(jpeg_entropy_kernel<true>, eg, dim3(64), nsets * 4 * sizeof(JpegHuff), s, data, seg_off,
                         seg_end, (const JpegHuff*)huff, huff_idx, nsets, g, nframes, coef, data_bytes,
                         (const uint8_t*)nullptr);
    else
      hipLaunchKernelGGL(jpeg_entropy_kernel<false>, eg, dim3(64), 0, s, data, seg_off, seg_end,
                         (const JpegHuff*)huff, huff_idx, nsets, g, nframes, coef, data_bytes, (const uint8_t*)nullptr);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
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
  if (xf) {   // fused colour + resample + crop + normalise (jpeg_transform_kernel)
    XformK xk{};
    size_t lds = 0;
    if ((e = jpeg_xform_plan(H, W, xf->n, xf->mode, xk, lds)) != hipSuccess) return e;
    const int64_t per_launch = std::max<int64_t>(1, (int64_t)0x7fffffff / ((int64_t)xk.nbands * XF_NT));
    for (int64_t f0 = 0; f0 < nframes; f0 += per_launch) {
      const int nfc = (int)std::min<int64_t>(per_launch, nframes - f0);
      char* o = (char*)xf->out + f0 * 3 * (int64_t)xf->n * xf->n * (xf->out_bf16 ? 2 : 4);
      const dim3 grid((unsigned)((int64_t)nfc * xk.nbands));
#define XF_LAUNCH(BF, I24_)                                                                                      \
  hipLaunchKernelGGL((jpeg_transform_kernel<BF, I24_>), grid, dim3(XF_NT), lds, s, planes + f0 * bytes, pl, ncomp, \
                     cmode, cdw, cdh, xk, (void*)o)
      if (xf->out_bf16) {
        if (xk.i24) XF_LAUNCH(true, true);
        else XF_LAUNCH(true, false);
      } else {
        if (xk.i24) XF_LAUNCH(false, true);
        else XF_LAUNCH(false, false);
      }
#undef XF_LAUNCH
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const int64_t px = (int64_t)W * H;
  const int64_t fc_px = std::max<int64_t>(1, ((int64_t)1 << 31) / px);
  for (int64_t f0 = 0; f0 < nframes; f0 += fc_px) {
    const int nfc = (int)std::min<int64_t>(fc_px, nframes - f0);
    const int64_t np = (int64_t)nfc * px;
    hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((np / 4 + 256) / 256)), dim3(256), 0, s, planes + f0 * bytes, pl,
                       W, H, ncomp, cmode, cdw, cdh, nfc, out_rgb + f0 * px * 3);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

size_t jpeg_workspace_bytes(const int32_t* geom, int nframes, int64_t data_bytes) {
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
  const size_t base = ((size_t)nframes * blocks * 64 * (sizeof(int16_t) + 1) + 255) & ~(size_t)255;
  return base + (geom[4] == 1 ? jp_layout(nframes, data_bytes < 0 ? 0 : data_bytes).bytes : 0);
}

}  // namespace miclip
