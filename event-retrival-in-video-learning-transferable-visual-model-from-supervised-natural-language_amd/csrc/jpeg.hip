// Baseline JPEG decode on the GPU (gfx950), bit-exact to Pillow's decoder —
// the decode step of the reference's frame ingest
//   Image.open(path).convert("RGB")        embedding_service.py:472-480, embedding.py:46
// (SURVEY.md §8(f) item 1).  Pillow hands YCbCr JPEGs to libjpeg(-turbo) with
// its defaults (JDCT_ISLOW, fancy upsampling, JCS_RGB output), so the three
// kernels below restate those integer algorithms:
//   jpeg_entropy_kernel  one lane per frame (or per restart interval):
//                        sequential Huffman decode of the interleaved scan,
//                        DC prediction, de-zigzag -> int16 coefficients;
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

#include <cstdint>

#include "internal.hpp"

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
struct JpegHuff {
  uint16_t look[512];
  int32_t maxcode[18];
  int32_t valoff[18];
  uint8_t vals[256];
};

struct BitReader {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf;     // left-aligned bit buffer
  int nbits;
  bool marker;      // hit a marker: feed zeros (libjpeg "insufficient data")

  __device__ __forceinline__ void fill() {
    while (nbits <= 56) {
      uint32_t c = 0;
      if (!marker && p < end) {
        c = *p++;
        if (c == 0xFF) {
          const uint32_t n = p < end ? *p : 0xD9;
          if (n == 0x00) {
            ++p;                 // stuffed zero byte
          } else {
            marker = true;       // a marker: stop consuming, zeros from here
            --p;
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
  __device__ __forceinline__ uint32_t get(int n) {
    if (n == 0) return 0;
    const uint32_t v = peek(n);
    skip(n);
    return v;
  }
};

__device__ __forceinline__ int huff_decode(BitReader& br, const JpegHuff* __restrict__ t) {
  br.fill();
  const uint32_t lk = t->look[br.peek(9)];
  if (lk) {
    br.skip(lk >> 8);
    return lk & 0xFF;
  }
  // longer code: libjpeg jpeg_huff_decode (lengths 10..16)
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
// huff[f * 4 + {dc0, ac0, dc1, ac1}], coefficient output coef + f * blocks_per_frame * 64
// (zeroed by the caller; only nonzero coefficients are written).
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

__global__ __launch_bounds__(64) void jpeg_entropy_kernel(const uint8_t* __restrict__ data,
                                                          const int64_t* __restrict__ seg_off,
                                                          const int64_t* __restrict__ seg_end,
                                                          const JpegHuff* __restrict__ huff, JpegGeom g, int nframes,
                                                          int16_t* __restrict__ coef) {
  const int64_t lane = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (lane >= (int64_t)nframes * g.nseg) return;
  const int f = (int)(lane / g.nseg), s = (int)(lane % g.nseg);
  BitReader br;
  br.p = data + seg_off[lane];
  br.end = data + seg_end[lane];
  br.buf = 0;
  br.nbits = 0;
  br.marker = false;
  const JpegHuff* T = huff + (int64_t)f * 4;
  int16_t* out = coef + (int64_t)f * g.blocks_per_frame * 64;
  const int total = g.mcux * g.mcuy;
  const int m0 = g.ri ? s * g.ri : 0;
  const int m1 = g.ri ? min(total, m0 + g.ri) : total;
  int pred[3] = {0, 0, 0};
  for (int m = m0; m < m1; ++m) {
    const int mx = m % g.mcux, my = m / g.mcux;
    for (int c = 0; c < g.ncomp; ++c) {
      const JpegHuff* dc = T + g.dcsel[c] * 2;
      const JpegHuff* ac = T + g.acsel[c] * 2 + 1;
      for (int v = 0; v < g.vs[c]; ++v)
        for (int h = 0; h < g.hs[c]; ++h) {
          int16_t* blk = out + (g.cbase[c] + (int64_t)(my * g.vs[c] + v) * g.bw[c] + (mx * g.hs[c] + h)) * 64;
          int t = huff_decode(br, dc);
          int diff = 0;
          if (t) {
            br.fill();
            diff = extend(br.get(t), t);
          }
          pred[c] += diff;
          blk[0] = (int16_t)pred[c];
          for (int k = 1; k < 64;) {
            const int rs = huff_decode(br, ac);
            const int r = rs >> 4, sz = rs & 15;
            if (sz) {
              k += r;
              br.fill();
              blk[kZigzag[k]] = (int16_t)extend(br.get(sz), sz);
              ++k;
            } else {
              if (r != 15) break;   // EOB
              k += 16;
            }
          }
        }
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
                       const uint16_t* qtab, const int32_t* geom, int nframes, uint8_t* out_rgb, void* ws,
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
  hipLaunchKernelGGL(jpeg_entropy_kernel, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, s, data, seg_off, seg_end,
                     (const JpegHuff*)huff, g, nframes, coef);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t nb = (int64_t)nframes * blocks;
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, coef, qtab, g, pl, nframes,
                     planes);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // chroma layout relative to luma (components 1, 2 share it)
  int cmode = 0, cdw = W, cdh = H;
  if (ncomp == 3) {
    const int hr = hmax / g.hs[1], vr = vmax / g.vs[1];
    cmode = (hr == 1 && vr == 1) ? 0 : (hr == 2 && vr == 1) ? 1 : 2;
    cdw = (W * g.hs[1] + hmax - 1) / hmax;   // libjpeg downsampled_width
    cdh = (H * g.vs[1] + vmax - 1) / vmax;
  }
  const int64_t np = (int64_t)nframes * W * H;
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, planes, pl, W, H, ncomp,
                     cmode, cdw, cdh, nframes, out_rgb);
  return hipGetLastError();
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
