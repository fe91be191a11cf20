// CLIP tower support kernels (gfx950): LayerNorm, embeddings, im2col,
// small-sequence multi-head attention, output finalisation.
//
// Reference semantics (openai/CLIP model.py, restated in oracle/clip_ref.py
// and pinned to transformers/models/clip/modeling_clip.py):
//   LayerNorm in fp32, eps 1e-5 (OpenAI LayerNorm casts to fp32)      V2/V3/V6/V8
//   vision embeddings: [CLS | conv1 patches] + pos -> ln_pre            V1-V2 (:202-218)
//   text embeddings: token_embedding[t] + positional_embedding          T1
//   attention: softmax(q k^T / sqrt(64) [+ causal mask]) v per head     V4/T2 (:280-335)
//   text pooling at argmax(tokens) then ln_final                        T3 (:559-571)
// The residual stream stays f32 in HBM; GEMM operands are bf16.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {

namespace {

constexpr float LN_EPS = 1e-5f;

// ---------------------------------------------------------------- LayerNorm
// One wave per row, W <= 1024 (4 float4 per lane), two-pass mean/variance.
struct RowVals {
  float4 v[4];
};

__device__ __forceinline__ void ln_stats(RowVals& r, int n4, int lane, int W, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < n4) s += (r.v[i].x + r.v[i].y) + (r.v[i].z + r.v[i].w);
  mean = wave_sum(s) / (float)W;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (lane + 64 * i < n4) {
      const float a = r.v[i].x - mean, b = r.v[i].y - mean, c = r.v[i].z - mean, d = r.v[i].w - mean;
      ss += (a * a + b * b) + (c * c + d * d);
    }
  const float var = wave_sum(ss) / (float)W;
  rstd = 1.0f / sqrtf(var + LN_EPS);
}

// LN output of one row: bf16 (out) or, when q != nullptr, MX-fp8 for the MX
// GEMM (q codes + stage-major e8m0 scales, one per 64 columns).  Lane holds
// columns 4*(lane + 64 i) .. +3, so a 64-column block is 16 consecutive lanes:
// its max is reduced with xor 1, 2, 4, 8.
__device__ __forceinline__ void ln_store(const RowVals& r, float mean, float rstd, const float* __restrict__ g,
                                         const float* __restrict__ b, uint16_t* __restrict__ out_row,
                                         uint8_t* __restrict__ q, uint8_t* __restrict__ qs, int64_t row,
                                         int64_t rows_pad, int lane, int n4) {
  const float4* g4 = (const float4*)g;
  const float4* b4 = (const float4*)b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = lane + 64 * i;
    float y0 = 0.f, y1 = 0.f, y2 = 0.f, y3 = 0.f;
    if (idx < n4) {
      const float4 gg = g4[idx], bb = b4[idx];
      y0 = (r.v[i].x - mean) * rstd * gg.x + bb.x;
      y1 = (r.v[i].y - mean) * rstd * gg.y + bb.y;
      y2 = (r.v[i].z - mean) * rstd * gg.z + bb.z;
      y3 = (r.v[i].w - mean) * rstd * gg.w + bb.w;
    }
    if (!q) {
      if (idx < n4) ((uint2*)out_row)[idx] = make_uint2(pack_bf16x2(y0, y1), pack_bf16x2(y2, y3));
      continue;
    }
    if (64 * i >= n4) continue;  // wave-uniform: no column of this lane group exists
    float amax = fmaxf(fmaxf(fabsf(y0), fabsf(y1)), fmaxf(fabsf(y2), fabsf(y3)));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    const int X = mx_block_exp(amax);
    if (idx < n4) {
      ((uint32_t*)(q + row * (int64_t)(4 * n4)))[idx] = mx_pack4(y0, y1, y2, y3, ldexpf(1.0f, -X));
      if ((idx & 15) == 0) qs[mx_scale_index(row, idx >> 4, rows_pad)] = (uint8_t)(X + 127);
    }
  }
}

__global__ __launch_bounds__(256) void ln_bf16_kernel(const float* __restrict__ x, int64_t in_stride,
                                                      const float* __restrict__ g, const float* __restrict__ b,
                                                      uint16_t* __restrict__ out, int64_t out_stride, int rows, int W,
                                                      uint8_t* __restrict__ q, uint8_t* __restrict__ qs) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int n4 = W >> 2;
  const float4* xr = (const float4*)(x + (int64_t)row * in_stride);
  RowVals r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.v[i] = (lane + 64 * i < n4) ? xr[lane + 64 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
  float mean, rstd;
  ln_stats(r, n4, lane, W, mean, rstd);
  ln_store(r, mean, rstd, g, b, out + (int64_t)row * out_stride, q, qs, row, (rows + 1) & ~1, lane, n4);
}

// Residual add + LayerNorm: xr = x[r*stride] + delta[r*stride] (delta = the
// bf16 out_proj / c_proj GEMM output, bias included); optionally x is
// written back (f32 residual stream), and out[r] = LN(xr) in bf16.
// This is `x = x + attn(ln_1(x)); h = ln_2(x)` (and `x = x + mlp(..);
// h = ln_1'(x)` / `ln_post(x[:, 0])`) of openai/CLIP ResidualAttentionBlock.
__global__ __launch_bounds__(256) void residual_ln_kernel(float* __restrict__ x, const uint16_t* __restrict__ delta,
                                                          int64_t stride, int write_x, const float* __restrict__ g,
                                                          const float* __restrict__ b, uint16_t* __restrict__ out,
                                                          int rows, int W, uint8_t* __restrict__ q,
                                                          uint8_t* __restrict__ qs) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int n4 = W >> 2;
  float4* xr = (float4*)(x + (int64_t)row * stride);
  const uint2* dr = (const uint2*)(delta + (int64_t)row * stride);
  RowVals r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = lane + 64 * i;
    if (idx < n4) {
      const float4 v = xr[idx];
      const uint2 d = dr[idx];
      r.v[i] = make_float4(v.x + bf2f((uint16_t)(d.x & 0xffff)), v.y + bf2f((uint16_t)(d.x >> 16)),
                           v.z + bf2f((uint16_t)(d.y & 0xffff)), v.w + bf2f((uint16_t)(d.y >> 16)));
      if (write_x) xr[idx] = r.v[i];
    } else {
      r.v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  float mean, rstd;
  ln_stats(r, n4, lane, W, mean, rstd);
  ln_store(r, mean, rstd, g, b, out + (int64_t)row * W, q, qs, row, (rows + 1) & ~1, lane, n4);
}

__global__ __launch_bounds__(256) void vision_embed_ln_kernel(float* __restrict__ x, const float* __restrict__ cls,
                                                              const float* __restrict__ pos, const float* __restrict__ g,
                                                              const float* __restrict__ b, int rows, int S, int W) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int t = row % S, n4 = W >> 2;
  float4* xr = (float4*)(x + (int64_t)row * W);
  const float4* src = t == 0 ? (const float4*)cls : (const float4*)xr;
  const float4* p4 = (const float4*)(pos + (int64_t)t * W);
  RowVals r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = lane + 64 * i;
    if (idx < n4) {
      const float4 s = src[idx], p = p4[idx];
      r.v[i] = make_float4(s.x + p.x, s.y + p.y, s.z + p.z, s.w + p.w);
    } else {
      r.v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  float mean, rstd;
  ln_stats(r, n4, lane, W, mean, rstd);
  const float4* g4 = (const float4*)g;
  const float4* b4 = (const float4*)b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = lane + 64 * i;
    if (idx < n4) {
      const float4 gg = g4[idx], bb = b4[idx];
      xr[idx] = make_float4((r.v[i].x - mean) * rstd * gg.x + bb.x, (r.v[i].y - mean) * rstd * gg.y + bb.y,
                            (r.v[i].z - mean) * rstd * gg.z + bb.z, (r.v[i].w - mean) * rstd * gg.w + bb.w);
    }
  }
}

__global__ __launch_bounds__(256) void text_embed_kernel(const int32_t* __restrict__ tokens,
                                                         const float* __restrict__ tok_emb,
                                                         const float* __restrict__ pos, float* __restrict__ x,
                                                         int64_t total4, int S, int W, int vocab) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const int n4 = W >> 2;
  const int64_t row = i / n4;
  const int c = (int)(i % n4);
  const int t = (int)(row % S);
  int tok = tokens[row];
  tok = tok < 0 ? 0 : (tok >= vocab ? vocab - 1 : tok);
  const float4 e = ((const float4*)(tok_emb + (int64_t)tok * W))[c];
  const float4 p = ((const float4*)(pos + (int64_t)t * W))[c];
  ((float4*)x)[i] = make_float4(e.x + p.x, e.y + p.y, e.z + p.z, e.w + p.w);
}

__global__ __launch_bounds__(256) void eot_gather_ln_kernel(const int32_t* __restrict__ tokens,
                                                            const float* __restrict__ x,
                                                            const uint16_t* __restrict__ delta,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ b, uint16_t* __restrict__ out,
                                                            int Q, int S, int W) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= Q) return;
  // argmax with first-index tie break (torch.argmax)
  int best = -2147483647 - 1, bi = 0x7fffffff;
  for (int t = lane; t < S; t += 64) {
    const int v = tokens[(int64_t)q * S + t];
    if (v > best || (v == best && t < bi)) { best = v; bi = t; }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int ov = __shfl_xor(best, o, 64), oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  const int n4 = W >> 2;
  const float4* xr = (const float4*)(x + ((int64_t)q * S + bi) * W);
  const uint2* dr = delta ? (const uint2*)(delta + ((int64_t)q * S + bi) * W) : nullptr;
  RowVals r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r.v[i] = (lane + 64 * i < n4) ? xr[lane + 64 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (dr && lane + 64 * i < n4) {
      const uint2 d = dr[lane + 64 * i];
      r.v[i].x += bf2f((uint16_t)(d.x & 0xffff));
      r.v[i].y += bf2f((uint16_t)(d.x >> 16));
      r.v[i].z += bf2f((uint16_t)(d.y & 0xffff));
      r.v[i].w += bf2f((uint16_t)(d.y >> 16));
    }
  }
  float mean, rstd;
  ln_stats(r, n4, lane, W, mean, rstd);
  const float4* g4 = (const float4*)g;
  const float4* b4 = (const float4*)b;
  uint2* o = (uint2*)(out + (int64_t)q * W);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = lane + 64 * i;
    if (idx < n4) {
      const float4 gg = g4[idx], bb = b4[idx];
      o[idx] = make_uint2((uint32_t)f2bf((r.v[i].x - mean) * rstd * gg.x + bb.x) |
                              ((uint32_t)f2bf((r.v[i].y - mean) * rstd * gg.y + bb.y) << 16),
                          (uint32_t)f2bf((r.v[i].z - mean) * rstd * gg.z + bb.z) |
                              ((uint32_t)f2bf((r.v[i].w - mean) * rstd * gg.w + bb.w) << 16));
    }
  }
}

// ------------------------------------------------------------------ im2col
// One thread per 8 consecutive k of one patch row.
// Vector form for P % 8 == 0 (B/32, B/16): the 8 k of a thread are 8
// consecutive pixels of one image row -> one 16-byte (bf16) or two 16-byte
// (f32) loads and one 16-byte store; consecutive threads walk a patch row.
template <bool IN_BF16>
__global__ __launch_bounds__(256) void im2col8_kernel(const void* __restrict__ pixels, uint16_t* __restrict__ out,
                                                      int64_t total8, int R, int P, int G, int Kp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total8) return;
  const int k8 = Kp >> 3;
  const int64_t prow = i / k8;
  const int kb = (int)(i % k8) * 8;
  const int PP = P * P;
  uint4 o = make_uint4(0, 0, 0, 0);
  if (kb < 3 * PP) {
    const int64_t bimg = prow / (G * G);
    const int p = (int)(prow % (G * G));
    const int gy = p / G, gx = p % G;
    const int c = kb / PP, rem = kb % PP, kh = rem / P, kw = rem % P;
    const int64_t off = ((bimg * 3 + c) * R + (gy * P + kh)) * (int64_t)R + gx * P + kw;
    if (IN_BF16) {
      o = *(const uint4*)((const uint16_t*)pixels + off);
    } else {
      const float4 a = *(const float4*)((const float*)pixels + off);
      const float4 b = *(const float4*)((const float*)pixels + off + 4);
      o = make_uint4(pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w), pack_bf16x2(b.x, b.y), pack_bf16x2(b.z, b.w));
    }
  }
  *(uint4*)(out + prow * Kp + kb) = o;
}

template <bool IN_BF16>
__global__ __launch_bounds__(256) void im2col_kernel(const void* __restrict__ pixels, uint16_t* __restrict__ out,
                                                     int64_t total8, int R, int P, int G, int Kp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total8) return;
  const int k8 = Kp >> 3;
  const int64_t prow = i / k8;
  const int kb = (int)(i % k8) * 8;
  const int64_t bimg = prow / (G * G);
  const int p = (int)(prow % (G * G));
  const int gy = p / G, gx = p % G;
  const int PP = P * P, K = 3 * PP;
  uint32_t packed[4];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    float v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = kb + e + u;
      if (k < K) {
        const int c = k / PP, rem = k % PP, kh = rem / P, kw = rem % P;
        const int64_t off = ((bimg * 3 + c) * R + (gy * P + kh)) * (int64_t)R + gx * P + kw;
        v[u] = IN_BF16 ? bf2f(((const uint16_t*)pixels)[off]) : ((const float*)pixels)[off];
      } else {
        v[u] = 0.f;
      }
    }
    packed[e >> 1] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  }
  *(uint4*)(out + prow * Kp + kb) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
}

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

// ------------------------------------------------- attention, long sequences
// One 512-thread workgroup (8 waves) per (sequence, head) for S > 96
// (B/16: 197, L/14: 257, L/14@336: 577 tokens).  V^T of the whole padded
// sequence (SP keys, multiple of 64) is staged once in LDS and shared by the 8
// waves (SP multiple of 32 and <= 608 keeps two workgroups per CU for
// L/14@336); wave w takes query tiles w, w+8, ... and streams the keys in chunks
// of 64 with an online (flash) softmax.  Everything is computed TRANSPOSED so
// that a lane owns one query row end to end:
//   S^T = K Q^T   A = K rows, B = Q rows (16-byte loads straight from the
//                 packed qkv rows; the next chunk's K is loaded before the
//                 current chunk's softmax so its latency hides).  C layout:
//                 lane -> query fr = lane&15, keys kt*16 + 4*(lane>>4) + j.
//   row max / sum: 16 registers in-lane + two cross-group shuffles;
//   m' = max(m, rowmax); alpha = 2^(m - m'); P = 2^(S^T - m')  (log2e/8 folded
//   into the scores); l = alpha l + rowsum P;
//   O^T = alpha O^T + V^T P^T   B = P^T straight from the S^T registers (the
//                 MFMA k order is a permutation: lane group g holds keys
//                 {32s + 4g + j, 32s + 16 + 4g + j}), A = V^T rows from LDS read
//                 with the same key permutation (two 8-byte reads).
// O^T's C layout gives each lane 4 consecutive head dims of its query row per
// 16-dim tile: 8-byte row stores.  Keys >= S are masked to -inf (and their V^T
// columns are 0, so 0 * pad never makes a NaN).
template <int SP, int NW>
__global__ __launch_bounds__(64 * NW) void attention_long_kernel(const uint16_t* __restrict__ qkv,
                                                             uint16_t* __restrict__ out, int S, int W, int H,
                                                             int causal, uint8_t* __restrict__ q8,
                                                             uint8_t* __restrict__ qs, int64_t rows_pad) {
  static_assert(SP % 32 == 0, "key padding");
  constexpr int TS = SP + 4;  // V^T row: +8 bytes staggers the banks of consecutive head dims
  __shared__ __attribute__((aligned(16))) uint16_t Vt[64 * TS];
  const int item = blockIdx.x;
  const int bseq = item / H, h = item % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t ld = 3 * (int64_t)W;
  const uint16_t* qb = qkv + (int64_t)bseq * S * ld + h * 64;
  const uint16_t* kb = qb + W;
  const uint16_t* vb = qb + 2 * W;

  for (int i = wave; i < 8 * ((SP + 63) / 64); i += NW) {
    const int r = (i >> 3) * 64 + lane, ch = i & 7;
    if (r < SP) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < S) v = *(const uint4*)(vb + (int64_t)r * ld + ch * 8);
      const uint16_t* vv = (const uint16_t*)&v;
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(ch * 8 + e) * TS + r] = vv[e];
    }
  }
  __syncthreads();

  const float sl2 = 0.125f * 1.4426950408889634f;  // head_dim^-0.5 * log2(e)
  const int fr = lane & 15, g = lane >> 4, fk = 8 * g;
  const int nqt = (S + 15) / 16;
  for (int qt = wave; qt < nqt; qt += NW) {
    const int qrow = qt * 16 + fr;  // this lane's query row
    bf16x8 qf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[s] = *(const bf16x8*)(qb + (int64_t)min(qrow, S - 1) * ld + 32 * s + fk);
    const int last_key = causal ? min(qt * 16 + 15, S - 1) : S - 1;
    const int nch = last_key / 64 + 1;
    float m = -INFINITY, l = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 kf[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const int64_t krow = min(kt * 16 + fr, S - 1);
#pragma unroll
      for (int s = 0; s < 2; ++s) kf[kt][s] = *(const bf16x8*)(kb + krow * ld + 32 * s + fk);
    }
    for (int c = 0; c < nch; ++c) {
      f32x4 sc[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][s], qf[s], acc, 0, 0, 0);
        sc[kt] = acc;
      }
      if (SP > 64 && c + 1 < nch) {  // prefetch the next chunk's K fragments
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const int64_t krow = min((c + 1) * 64 + kt * 16 + fr, S - 1);
#pragma unroll
          for (int s = 0; s < 2; ++s) kf[kt][s] = *(const bf16x8*)(kb + krow * ld + 32 * s + fk);
        }
      }
      // sc[kt][j]: query qrow, key c*64 + kt*16 + 4g + j
      float cm = -INFINITY;
      const bool edge = (c + 1) * 64 > S || (causal && (c + 1) * 64 > qt * 16);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = sc[kt][j] * sl2;
          if (edge) {
            const int key = c * 64 + kt * 16 + 4 * g + j;
            if (key >= S || (causal && key > qrow)) v = -INFINITY;
          }
          sc[kt][j] = v;
          cm = fmaxf(cm, v);
        }
      cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
      cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
      // finite: chunk 0 holds key 0 <= every row
      const float mn = fmaxf(m, cm);
      const float alpha = exp2f(m - mn);
      m = mn;
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = exp2f(sc[kt][j] - mn);
          sc[kt][j] = p;
          sum += p;
        }
      l = l * alpha + sum;  // partial (this lane group's keys); reduced once at the end
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 1 && c * 64 + 32 >= S) break;  // keys past round32(S) <= SP: P = 0, no V^T columns
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[j] = (__bf16)sc[2 * s][j];
          pb[4 + j] = (__bf16)sc[2 * s + 1][j];
        }
        const uint16_t* vrow = Vt + fr * TS + c * 64 + 32 * s + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const uint2 lo = *(const uint2*)(vrow + dt * 16 * TS);
          const uint2 hi = *(const uint2*)(vrow + dt * 16 * TS + 16);
          const uint4 va4 = make_uint4(lo.x, lo.y, hi.x, hi.y);
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, va4), pb, o[dt], 0, 0, 0);
        }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    // o[dt][j]: query qrow, head dim dt*16 + 4g + j
    if (q8) {  // MX-fp8 output: this head's 64 dims are one 64-k block of out_proj
      float amax = 0.f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fabsf(o[dt][j] * inv));
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      const int X = mx_block_exp(amax);
      const float sc = ldexpf(1.0f, -X);
      if (qrow < S) {
        const int64_t row = (int64_t)bseq * S + qrow;
        uint8_t* dst = q8 + row * W + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          *(uint32_t*)(dst + dt * 16) = mx_pack4(o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv, sc);
        if (g == 0) qs[mx_scale_index(row, h, rows_pad)] = (uint8_t)(X + 127);
      }
      continue;
    }
    if (qrow < S) {
      uint16_t* dst = out + ((int64_t)bseq * S + qrow) * W + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *(uint2*)(dst + dt * 16) = make_uint2(pack_bf16x2(o[dt][0] * inv, o[dt][1] * inv),
                                              pack_bf16x2(o[dt][2] * inv, o[dt][3] * inv));
    }
  }
}

// ---------------------------------------------------------------- finalize
__global__ __launch_bounds__(256) void finalize_kernel(const float* __restrict__ y, void* __restrict__ out,
                                                       int out_dtype, int rows, int D, int l2) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* yr = y + (int64_t)row * D;
  float inv = 1.f;
  if (l2) {
    float ss = 0.f;
    for (int c = lane; c < D; c += 64) ss += yr[c] * yr[c];
    const float n = sqrtf(wave_sum(ss));
    // l2 == 2: compare_models.py:1168-1171 guard (norm <= 1e-8 -> divide by 1)
    inv = (l2 == 2 && !(n > 1e-8f)) ? 1.0f : 1.0f / n;
  }
  for (int c = lane; c < D; c += 64) {
    const float v = l2 ? yr[c] * inv : yr[c];
    if (out_dtype == 0) ((float*)out)[(int64_t)row * D + c] = v;
    else if (out_dtype == 1) ((uint16_t*)out)[(int64_t)row * D + c] = f2bf(v);
    else ((_Float16*)out)[(int64_t)row * D + c] = (_Float16)v;
  }
}

}  // namespace

hipError_t layernorm_bf16(const float* x, int64_t in_stride, const float* g, const float* b, uint16_t* out,
                          int64_t out_stride, int rows, int W, hipStream_t s, uint8_t* q, uint8_t* qs) {
  if (rows <= 0) return hipSuccess;
  if (W % 4 || W > 1024 || (q && W % 128)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_bf16_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, in_stride, g, b, out, out_stride,
                     rows, W, q, qs);
  return hipGetLastError();
}

hipError_t vision_embed_ln(float* x, const float* cls, const float* pos, const float* g, const float* b, int B,
                           int S, int W, hipStream_t s) {
  const int rows = B * S;
  if (rows <= 0) return hipSuccess;
  if (W % 4 || W > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vision_embed_ln_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, cls, pos, g, b, rows, S, W);
  return hipGetLastError();
}

hipError_t text_embed(const int32_t* tokens, const float* tok_emb, const float* pos, float* x, int Q, int S, int W,
                      int vocab, hipStream_t s) {
  const int64_t total4 = (int64_t)Q * S * (W / 4);
  if (total4 <= 0) return hipSuccess;
  hipLaunchKernelGGL(text_embed_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, tokens, tok_emb,
                     pos, x, total4, S, W, vocab);
  return hipGetLastError();
}

hipError_t eot_gather_ln(const int32_t* tokens, const float* x, const uint16_t* delta, const float* g,
                         const float* b, uint16_t* out, int Q, int S, int W, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  hipLaunchKernelGGL(eot_gather_ln_kernel, dim3((Q + 3) / 4), dim3(256), 0, s, tokens, x, delta, g, b, out, Q, S,
                     W);
  return hipGetLastError();
}

hipError_t residual_ln(float* x, const uint16_t* delta, int64_t stride, int write_x, const float* g, const float* b,
                       uint16_t* out, int rows, int W, hipStream_t s, uint8_t* q, uint8_t* qs) {
  if (rows <= 0) return hipSuccess;
  if (W % 4 || W > 1024 || (q && W % 128)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(residual_ln_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, delta, stride, write_x, g, b, out,
                     rows, W, q, qs);
  return hipGetLastError();
}

hipError_t im2col(const void* pixels, int in_bf16, uint16_t* out, int B, int R, int P, int Kp, hipStream_t s) {
  const int G = R / P;
  const int64_t total8 = (int64_t)B * G * G * (Kp / 8);
  if (total8 <= 0) return hipSuccess;
  const dim3 grid((unsigned)((total8 + 255) / 256));
  const bool vec = P % 8 == 0 && ((uintptr_t)pixels & 15) == 0;
  if (vec && in_bf16)
    hipLaunchKernelGGL(im2col8_kernel<true>, grid, dim3(256), 0, s, pixels, out, total8, R, P, G, Kp);
  else if (vec)
    hipLaunchKernelGGL(im2col8_kernel<false>, grid, dim3(256), 0, s, pixels, out, total8, R, P, G, Kp);
  else if (in_bf16)
    hipLaunchKernelGGL(im2col_kernel<true>, grid, dim3(256), 0, s, pixels, out, total8, R, P, G, Kp);
  else
    hipLaunchKernelGGL(im2col_kernel<false>, grid, dim3(256), 0, s, pixels, out, total8, R, P, G, Kp);
  return hipGetLastError();
}

hipError_t attention(const uint16_t* qkv, uint16_t* out, int B, int S, int W, int causal, hipStream_t s, uint8_t* q8,
                     uint8_t* qs) {
  const int H = W / 64;
  const int items = B * H;
  if (items <= 0) return hipSuccess;
  // S <= 96 (B/32 50, text 77): the one-wave LDS-P kernel, measured faster there
  // (scripts/attn_micro.py: 179 vs 195-203 us at B/32) than the flash kernel
  // with 1, 2 or 4 waves; causal bit 8 selects the 4-wave flash kernel instead
  // (A/B measurements, parity tests of both paths).
  bool flash_short = (causal >> 8) & 1;
  causal &= 1;
  const dim3 grid(items), b64(64), b256(256), b512(512);
#define LONG_ATTN(SP, NW, blk)                                                                                   \
  hipLaunchKernelGGL((attention_long_kernel<SP, NW>), grid, blk, 0, s, qkv, out, S, W, H, causal, q8, qs, \
                     ((int64_t)B * S + 1) & ~1)
  if (q8 && S <= 96) flash_short = true;  // the fp8 output lives in the flash kernel
  if (!flash_short && S <= 96) {
    if (S <= 32) hipLaunchKernelGGL(attention_kernel<32>, grid, b64, 0, s, qkv, out, S, W, H, causal, items);
    else if (S <= 64) hipLaunchKernelGGL(attention_kernel<64>, grid, b64, 0, s, qkv, out, S, W, H, causal, items);
    else hipLaunchKernelGGL(attention_kernel<96>, grid, b64, 0, s, qkv, out, S, W, H, causal, items);
  } else if (S <= 32) LONG_ATTN(32, 4, b256);
  else if (S <= 64) LONG_ATTN(64, 4, b256);
  else if (S <= 96) LONG_ATTN(96, 4, b256);
  else if (S <= 128) LONG_ATTN(128, 8, b512);
  else if (S <= 224) LONG_ATTN(224, 8, b512);
  else if (S <= 288) LONG_ATTN(288, 8, b512);
  else if (S <= 384) LONG_ATTN(384, 8, b512);
  else if (S <= 608) LONG_ATTN(608, 8, b512);
  else if (S <= 640) LONG_ATTN(640, 8, b512);
  else return hipErrorInvalidValue;
#undef LONG_ATTN
  return hipGetLastError();
}

hipError_t finalize_rows(const float* y, void* out, int out_dtype, int rows, int D, int l2, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(finalize_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, y, out, out_dtype, rows, D, l2);
  return hipGetLastError();
}

}  // namespace miclip
