// fp32 tower kernels (gfx950): the weight_dtype MI_F32 mode of mi_clip_create.
//
// openai/CLIP computes in fp32 when its weights are fp32: on the CPU
// (clip.load(device="cpu") calls model.float(); Backend/embedding.py:21-22 is
// BASELINE configs[0]) and after `clip_model.float()` (CLIPWithClassifier,
// Backend/services/embedding_service.py:22).  compare_models.py's R@K flow
// (:908-1100) run on a CPU is this arithmetic too.  This mode keeps every
// activation and weight in f32 so that encoder outputs sit within f32 rounding
// of the reference's and R@1/5/10 come out identical (miclip/evaluate.py,
// tests/test_gpu_rk_flow.py), at the f32 MFMA rate (157 TF, 1/16 of bf16).
//
//   gemm_f32   out = A[M,K] . W[N,K]^T (+bias) on v_mfma_f32_32x32x2_f32 (exact f32
//              products, f32 accumulation); epilogues: store, QuickGELU, residual add
//   ln_f32     LayerNorm rows in f32 -> f32 (optionally the EOT row of each token row)
//   attn_f32   softmax(q k^T / 8 [+ causal]) v per (sequence, head), f32
//   im2col_f32 conv1 patches in f32
#include <cstdlib>

#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr float LN_EPS = 1e-5f;

// ------------------------------------------------------------------ GEMM
// 128 x 128 tile, K staged 32 wide through LDS (register prefetch of the next
// stage), 4 waves as 2 x 2, each wave 64 x 64 = 2 x 2 blocks of the 32x32x2
// MFMA.  Lane (r = lane & 31, h = lane >> 5) feeds A[row r][k = 16h + i] and
// W[col r][k = 16h + i] to MFMA i, so 16 MFMAs cover the stage's 32 k.
constexpr int GT = 128, GK = 32, GLD = GK + 4;

template <int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ W, int64_t ldw,
                                                       const float* __restrict__ bias, float* __restrict__ out,
                                                       int64_t ldo, int M, int N, int K, int group, int gstride,
                                                       int goffset) {
  __shared__ __attribute__((aligned(16))) float As[GT * GLD];
  __shared__ __attribute__((aligned(16))) float Ws[GT * GLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  // staging: thread t loads rows t/8 + 32 j (j = 0..3), 4 k at 4 (t % 8)
  const int lr = tid >> 3, lk = (tid & 7) * 4;
  const float* ap[4];
  const float* wp[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = lr + 32 * j;
    ap[j] = A + (int64_t)min(m0 + r, M - 1) * lda + lk;
    wp[j] = W + (int64_t)min(n0 + r, N - 1) * ldw + lk;
  }
  float4 ra[4], rw[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ra[j] = *(const float4*)(ap[j] + k0);
      rw[j] = *(const float4*)(wp[j] + k0);
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *(float4*)&As[(lr + 32 * j) * GLD + lk] = ra[j];
      *(float4*)&Ws[(lr + 32 * j) * GLD + lk] = rw[j];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  const int r = lane & 31, h = lane >> 5;
  const int nk = K / GK;
  gload(0);
  sstore();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload((kt + 1) * GK);
    float fa[2][16], fw[2][16];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 va = *(const float4*)&As[(64 * wm + 32 * a + r) * GLD + 16 * h + 4 * i];
        const float4 vw = *(const float4*)&Ws[(64 * wn + 32 * a + r) * GLD + 16 * h + 4 * i];
        fa[a][4 * i] = va.x; fa[a][4 * i + 1] = va.y; fa[a][4 * i + 2] = va.z; fa[a][4 * i + 3] = va.w;
        fw[a][4 * i] = vw.x; fw[a][4 * i + 1] = vw.y; fw[a][4 * i + 2] = vw.z; fw[a][4 * i + 3] = vw.w;
      }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a][i], fw[b][i], acc[a][b], 0, 0, 0);
    __syncthreads();
    if (kt + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
  // epilogue: C layout col = lane & 31, row = (q & 3) + 8 (q >> 2) + 4 h
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int n = n0 + 64 * wn + 32 * b + r;
    if (n >= N) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + 64 * wm + 32 * a + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (m >= M) continue;
        const int64_t orow = group ? (int64_t)(m / group) * gstride + goffset + m % group : m;
        float v = acc[a][b][q] + bv;
        float* o = out + orow * ldo + n;
        if (EPI == EPI_GELU_BF16) v = v * (1.0f / (1.0f + expf(-1.702f * v)));   // QuickGELU x * sigmoid(1.702 x)
        if (EPI == EPI_RELU_F32) v = fmaxf(v, 0.f);
        if (EPI == EPI_RESID_F32) *o = *o + v;
        else *o = v;
      }
  }
}

// ------------------------------------------------------------- split-bf16 operands
// (internal.hpp split6_rows) one thread per 4 consecutive values of a row
__device__ __forceinline__ void split3(float x, u16& x1, u16& x2, u16& x3) {
  x1 = f2bf(x);
  if (!__builtin_isfinite(x)) {   // inf / NaN: carried by x1 alone (x - x1 would be NaN)
    x2 = x3 = 0;
    return;
  }
  if ((x1 & 0x7fffu) == 0x7f80u) x1 = (u16)((x1 & 0x8000u) | 0x7f7fu);   // finite x past bf16's range: largest bf16
  const float r1 = x - bf2f(x1);    // exact: x1 holds x's leading 8 significand bits
  x2 = f2bf(r1);
  x3 = f2bf(r1 - bf2f(x2));
}

__global__ __launch_bounds__(256) void split6_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int K,
                                                     int role, int gelu, uint16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int k4 = K >> 2;
  if (i >= rows * k4) return;
  const int64_t r = i / k4;
  const int c = (int)(i - r * k4) * 4;
  float4 v = *(const float4*)(x + r * ldx + c);
  if (gelu) {
    v.x = v.x * (1.0f / (1.0f + expf(-1.702f * v.x)));
    v.y = v.y * (1.0f / (1.0f + expf(-1.702f * v.y)));
    v.z = v.z * (1.0f / (1.0f + expf(-1.702f * v.z)));
    v.w = v.w * (1.0f / (1.0f + expf(-1.702f * v.w)));
  }
  u16 p[3][4];
  split3(v.x, p[0][0], p[1][0], p[2][0]);
  split3(v.y, p[0][1], p[1][1], p[2][1]);
  split3(v.z, p[0][2], p[1][2], p[2][2]);
  split3(v.w, p[0][3], p[1][3], p[2][3]);
  // K-block j holds term t_a[j] (activations) or t_w[j] (weights)
  constexpr int t_a[6] = {0, 1, 2, 0, 1, 0}, t_w[6] = {0, 0, 0, 1, 1, 2};
  uint16_t* o = out + r * 6 * (int64_t)K + c;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int t = role ? t_w[j] : t_a[j];
    const uint2 w = make_uint2((uint32_t)p[t][0] | ((uint32_t)p[t][1] << 16), (uint32_t)p[t][2] | ((uint32_t)p[t][3] << 16));
    *(uint2*)(o + (int64_t)j * K) = w;
  }
}

// ------------------------------------------------------------- split-f16 operands
// (internal.hpp split2h_rows; round 5, the default GEMM operands of the fp32 tower).  A row x
// of K values is scaled by a power of two s, max |x s| in [2^13, 2^14), and split as
//   x s = x1 + x2 + r,  x1 = f16(x s),  x2 = f16(x s - x1),  |r| <= 2^-11 |x s - x1| <= 2^-22 |x s|
// (x s - x1 is exact in f32; f16's subnormal floor adds at most 2^-25, i.e. 2^-39 of the row's
// largest value).  Activations are stored [x1 | x1 | x2] and weights [w1 | w2 | w1], so ONE f16
// GEMM over K' = 3K sums a1 w1 + a1 w2 + a2 w1 with f32 accumulation -- the dropped a2 w2 is
// <= 2^-22 |a w| -- and the epilogue multiplies by 1 / (s_row s_col) (powers of two: exact).
// Against the split-bf16 form (split6_rows, K' = 6K) that halves the MFMA work and the operand
// bytes at the same accuracy (numpy simulation at K = 768 / 3072: 7.1e-7 / 4.7e-7 of max |ref|
// for f16 x 3 against 3.2e-7 / 5.8e-7 for bf16 x 6).
__device__ __forceinline__ int split_exp(float mx) {   // s = 2^e: mx * s in [2^13, 2^14)
  if (!(mx > 0.f) || !__builtin_isfinite(mx)) return 0;   // zero / non-finite row: unscaled
  int ex;
  (void)frexpf(mx, &ex);                                 // mx = f 2^ex, f in [0.5, 1)
  const int e = 14 - ex;
  return e > 126 ? 126 : (e < -126 ? -126 : e);          // 1 / s stays a normal float
}

__device__ __forceinline__ void split2h(float xs, _Float16& x1, _Float16& x2) {
  x1 = (_Float16)xs;
  const float f1 = (float)x1;
  // inf / NaN (only in rows left unscaled): carried by x1 alone
  x2 = __builtin_isfinite(f1) ? (_Float16)(xs - f1) : (_Float16)0.f;
}

__device__ __forceinline__ float quick_gelu_f32(float v) { return v * (1.0f / (1.0f + expf(-1.702f * v))); }

__device__ __forceinline__ float absmax4(float m, float4 v) {
  return fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
}

typedef _Float16 f16x4_p __attribute__((ext_vector_type(4)));

// the lane's 4 values (columns c..c+3) of a row scaled by 2^e into the K-blocks of out: role 0
// [x1 | x1 | x2], role 1 [x1 | x2 | x1] (row stride 3K), role 2 [x1 | x2] (row stride 2K: the
// activations once, read as [x1 | x1 | x2] by the 8-phase GEMM, GemmArgs a_dup)
__device__ __forceinline__ void store_split4(float4 v, int e, int role, _Float16* o, int K, int c) {
  _Float16 a0, a1, a2, a3, b0, b1, b2, b3;
  split2h(ldexpf(v.x, e), a0, b0);
  split2h(ldexpf(v.y, e), a1, b1);
  split2h(ldexpf(v.z, e), a2, b2);
  split2h(ldexpf(v.w, e), a3, b3);
  const f16x4_p h1 = {a0, a1, a2, a3}, h2 = {b0, b1, b2, b3};
  *(f16x4_p*)(o + c) = h1;
  if (role == 2) {
    *(f16x4_p*)(o + K + c) = h2;
    return;
  }
  *(f16x4_p*)(o + K + c) = role ? h2 : h1;
  *(f16x4_p*)(o + 2 * K + c) = role ? h1 : h2;
}

// One wave per row, a lane's float4 at columns 4 lane + 256 i (K % 4 == 0, K <= 256 NV).
// sc[row] = 1 / s (the GEMM epilogue's factor for this row / column).
template <int NV>
__global__ __launch_bounds__(256) void split2h_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int K,
                                                      int role, int gelu, _Float16* __restrict__ out,
                                                      float* __restrict__ sc) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + row * ldx;
  float4 v[NV];
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    v[i] = c < K ? *(const float4*)(xr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (gelu) v[i] = make_float4(quick_gelu_f32(v[i].x), quick_gelu_f32(v[i].y), quick_gelu_f32(v[i].z),
                                 quick_gelu_f32(v[i].w));
    mx = absmax4(mx, v[i]);
  }
  const int e = split_exp(wave_max(mx));
  if (lane == 0) sc[row] = ldexpf(1.f, -e);
  _Float16* o = out + row * (role == 2 ? 2 : 3) * (int64_t)K;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    if (c < K) store_split4(v[i], e, role, o, K, c);
  }
}

// LayerNorm (ln_f32_kernel's statistics: two-pass mean / variance in f32) straight into the
// split operand of the following GEMM: no f32 LN output is written or re-read.  W <= 1024.
__global__ __launch_bounds__(256) void ln_split2h_kernel(const float* __restrict__ x, int64_t in_stride,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         int rows, int W, _Float16* __restrict__ out,
                                                         float* __restrict__ sc, float* __restrict__ rmax, int dup) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * in_stride;
  float4 v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * lane + 256 * i;
    v[i] = c < W ? *(const float4*)(xr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / (float)W;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * lane + 256 * i;
    if (c < W) {
      const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
      ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)W + LN_EPS);
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * lane + 256 * i;
    if (c < W) {
      const float4 gg = *(const float4*)(g + c), bb = *(const float4*)(b + c);
      v[i] = make_float4((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y,
                         (v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
      mx = absmax4(mx, v[i]);
    }
  }
  const float rm = wave_max(mx);
  const int e = split_exp(rm);
  if (lane == 0) {
    sc[row] = ldexpf(1.f, -e);
    if (rmax) rmax[row] = rm;
  }
  _Float16* o = out + (int64_t)row * (dup ? 2 : 3) * W;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * lane + 256 * i;
    if (c < W) store_split4(v[i], e, dup ? 2 : 0, o, W, c);
  }
}

// ------------------------------------------------------------- LayerNorm
// One wave per row, W <= 1024, two-pass mean / variance in f32 (torch's
// LayerNorm on fp32).  tokens != nullptr: row q of the output is the row
// q * S + argmax(tokens[q]) of x (text pooling at EOT, first index on ties).
__global__ __launch_bounds__(256) void ln_f32_kernel(const float* __restrict__ x, int64_t in_stride,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float* __restrict__ out, int64_t out_stride, int rows, int W,
                                                     const int32_t* __restrict__ tokens, int S) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  int64_t src = (int64_t)row * in_stride;
  if (tokens) {
    int best = -2147483647 - 1, bi = 0x7fffffff;
    for (int t = lane; t < S; t += 64) {
      const int v = tokens[(int64_t)row * S + t];
      if (v > best || (v == best && t < bi)) { best = v; bi = t; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const int ov = __shfl_xor(best, o, 64), oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    src = ((int64_t)row * S + bi) * in_stride;
  }
  const float* xr = x + src;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < W ? xr[c] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)W;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    if (c < W) ss += (v[i] - mean) * (v[i] - mean);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)W + LN_EPS);
  float* o = out + (int64_t)row * out_stride;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane + 64 * i;
    if (c < W) o[c] = (v[i] - mean) * rstd * g[c] + b[c];
  }
}

// ------------------------------------------------------------- attention
// One workgroup per (sequence, head); a thread owns one query row (q scaled
// by 1/8 = head_dim^-1/2, exact), keys and values stream through LDS in
// chunks of 64 with an online softmax (per-chunk max, one rescale per chunk).
template <int NT>
__global__ __launch_bounds__(NT) void attn_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out, int S,
                                                      int W, int causal) {
  __shared__ float Ks[64 * 64];
  __shared__ float Vs[64 * 64];
  const int H = W / 64;
  const int bseq = blockIdx.x / H, head = blockIdx.x % H;
  const int64_t ld = 3 * (int64_t)W;
  const float* base = qkv + (int64_t)bseq * S * ld;
  const int tid = threadIdx.x;
  for (int q0 = 0; q0 < S; q0 += NT) {
    const int qi = q0 + tid;
    const bool valid = qi < S;
    float qv[64], acc[64];
    float m = -INFINITY, l = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) {
      qv[d] = valid ? base[(int64_t)qi * ld + head * 64 + d] * 0.125f : 0.f;
      acc[d] = 0.f;
    }
    const int kend = causal ? min(S, q0 + NT) : S;
    for (int k0 = 0; k0 < kend; k0 += 64) {
      __syncthreads();
      for (int e = tid; e < 64 * 64; e += NT) {
        const int j = e >> 6, d = e & 63;
        const bool in = k0 + j < S;
        Ks[e] = in ? base[(int64_t)(k0 + j) * ld + W + head * 64 + d] : 0.f;
        Vs[e] = in ? base[(int64_t)(k0 + j) * ld + 2 * W + head * 64 + d] : 0.f;
      }
      __syncthreads();
      float s[64];
      float cmax = -INFINITY;
#pragma unroll
      for (int j = 0; j < 64; ++j) {
        float t = 0.f;
#pragma unroll
        for (int d = 0; d < 64; ++d) t = fmaf(qv[d], Ks[j * 64 + d], t);
        const bool ok = k0 + j < S && (!causal || k0 + j <= qi);
        s[j] = ok ? t : -INFINITY;
        cmax = fmaxf(cmax, s[j]);
      }
      if (!valid || cmax == -INFINITY) continue;
      const float mn = fmaxf(m, cmax);
      const float corr = expf(m - mn);
      l *= corr;
#pragma unroll
      for (int d = 0; d < 64; ++d) acc[d] *= corr;
#pragma unroll
      for (int j = 0; j < 64; ++j) {
        const float p = expf(s[j] - mn);
        l += p;
#pragma unroll
        for (int d = 0; d < 64; ++d) acc[d] = fmaf(p, Vs[j * 64 + d], acc[d]);
      }
      m = mn;
    }
    if (valid) {
      const float inv = 1.0f / l;
      float* o = out + ((int64_t)bseq * S + qi) * W + head * 64;
#pragma unroll
      for (int d = 0; d < 64; ++d) o[d] = acc[d] * inv;
    }
  }
}

// ------------------------------------------------------------- attention (MFMA)
// S <= 32 NKT (<= 128: B/32's 50 tokens, the text tower's 77): one wave per (sequence, head),
// every operand in registers, on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32: exact products,
// f32 accumulation, as fmaf chains).  The 32x32 C layout puts column (lane & 31) in the lane
// and rows rho(r, h) = (r & 3) + 8 (r >> 2) + 4 h, h = lane >> 5, in its registers r = 0..15.
//   S^T = K Q^T per key tile kt and 32-query block: A = K (lane (key i, h) gives K[i][32 h + s]
//     at step s), B = Q (lane (query j, h) gives q[j][32 h + s] / 8): lane (query j, h) then
//     holds its query's scores against keys rho(r, h) -- the softmax over keys is in-lane over
//     16 NKT values plus the partner lane j + 32.
//   O = P V per 32-dim tile dt: A = P, and the k pair of step s is keys {rho(s, 0), rho(s, 1)},
//     so lane (query i, h) gives its own register s (no data movement); B = V (lane (dim j, h)
//     gives V[rho(s, h)][32 dt + j]).  C: lane (dim j, h) holds queries rho(r, h), so each
//     register's 32 lanes store one 128-byte row segment.
// Replaces attn_f32_kernel (a thread per query row, scalar fmaf over LDS; 10.4 ms per B/32 layer
// at 10k frames, profiles/r05_a_fp32_bench_kernel_stats.csv).
// CL: loads and stores through buffer descriptors whose range ends at the sequence's last row, so
// the padding rows read zeros and their stores drop with no branch (a conditional load or store
// compiles to an exec-masked branch around each one: 119 branches per wave and SGPR spills through
// v_writelane in the NKT = 2 kernel); the same values, bit-identical
template <int NKT, int MINB = 1, bool CL = true>
__global__ __launch_bounds__(256, MINB) void attn_f32_mfma_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                            int nseq, int S, int W, int causal) {
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int H = W / 64;
  const int item = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform: SGPR descriptors)
  if (item >= nseq * H) return;
  // causal bit 11: the first 32-query block only (the last vision block: outputs read at the CLS rows)
  const int qend = ((causal >> 11) & 1) ? min(S, 32) : S;
  causal &= 1;
  const int bseq = item / H, head = item % H;
  const int64_t ld = 3 * (int64_t)W;
  const float* base = qkv + (int64_t)bseq * S * ld + head * 64;
  float* obase = out + (int64_t)bseq * S * W + head * 64;
  auto rho = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
  // (CL: p's row r is passed too; offsets from the sequence's first row, rows >= S out of range)
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(qkv + (int64_t)bseq * S * ld), (short)0, S * (int)ld * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (int64_t)bseq * S * W), (short)0, S * W * 4, 0x00020000);
  auto ld4 = [&](const float* p, bool ok, int r, int col) {
    if (CL) {
      typedef unsigned int u32x4a __attribute__((ext_vector_type(4)));
      const u32x4a t = __builtin_bit_cast(u32x4a, __builtin_amdgcn_raw_buffer_load_b128(rin, (uint32_t)((r * (int)ld + col) * 4), 0, 0));
      return make_float4(__uint_as_float(t[0]), __uint_as_float(t[1]), __uint_as_float(t[2]), __uint_as_float(t[3]));
    }
    return ok ? *(const float4*)p : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto ld1 = [&](const float* p, bool ok, int r, int col) {
    if (CL) return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rin, (uint32_t)((r * (int)ld + col) * 4), 0, 0));
    return ok ? *p : 0.f;
  };
  for (int q0 = 0; q0 < qend; q0 += 32) {
    const int qi = q0 + j;   // this lane's query in the S^T layout
    float qv[32];
    {
      const float* qp = base + (int64_t)min(qi, S - 1) * ld + 32 * h;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float4 t = ld4(qp + 4 * c, qi < S, qi, head * 64 + 32 * h + 4 * c);
        qv[4 * c] = t.x * 0.125f; qv[4 * c + 1] = t.y * 0.125f; qv[4 * c + 2] = t.z * 0.125f; qv[4 * c + 3] = t.w * 0.125f;
      }
    }
    f32x16 sc[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      sc[kt] = f32x16{};
      if (kt * 32 >= S) continue;
      const int ki = kt * 32 + j;   // this lane's key as an A-operand row
      const float* kp = base + W + (int64_t)min(ki, S - 1) * ld + 32 * h;
      float kv[32];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float4 t = ld4(kp + 4 * c, ki < S, ki, W + head * 64 + 32 * h + 4 * c);
        kv[4 * c] = t.x; kv[4 * c + 1] = t.y; kv[4 * c + 2] = t.z; kv[4 * c + 3] = t.w;
      }
#pragma unroll
      for (int st = 0; st < 32; ++st) sc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[st], qv[st], sc[kt], 0, 0, 0);
    }
    // masks and the softmax statistics of query qi (keys rho(r, h) of every tile, with lane ^ 32)
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + rho(r);
        if (key >= S || (causal && key > qi)) sc[kt][r] = -INFINITY;
        m = fmaxf(m, sc[kt][r]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = expf(sc[kt][r] - m);   // masked keys: exp(-inf) = 0
        sc[kt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      f32x16 o = f32x16{};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt * 32 >= S) continue;
        float vv[16];
#pragma unroll
        for (int st = 0; st < 16; ++st) {
          const int key = kt * 32 + (st & 3) + 8 * (st >> 2) + 4 * h;
          vv[st] = ld1(base + 2 * W + (int64_t)min(key, S - 1) * ld + 32 * dt + j, key < S, key, 2 * W + head * 64 + 32 * dt + j);
        }
#pragma unroll
        for (int st = 0; st < 16; ++st) o = __builtin_amdgcn_mfma_f32_32x32x2f32(sc[kt][st], vv[st], o, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = q0 + rho(r);
        const float iv = __shfl(inv, rho(r), 64);   // 1 / l of query rho(r) (held by lane rho(r))
        if (CL)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[r] * iv), rout, (uint32_t)((qr * W + head * 64 + 32 * dt + j) * 4), 0, 0);
        else if (qr < S)
          obase[(int64_t)qr * W + 32 * dt + j] = o[r] * iv;
      }
    }
  }
}

// The S <= 64 form with its loads batched (round 6; B/32's 50 tokens, the fp32 tower's attention).
// attn_f32_mfma_kernel above lets hipcc place each load next to its first use: at two waves per
// SIMD its scheduler keeps two of a key tile's eight K loads in flight and issues V one MFMA ahead,
// so a wave waits for ~20 dependent L2 round trips per query block.  Here each query block issues
// Q, both key tiles' K and the first dim tile's V (8 + 16 + 32 loads) together, then a scheduling
// barrier; the second dim tile's V goes out after the softmax, ahead of the first dim tile's MFMAs.
// Rows stay in the per-lane offset (rows >= S read zeros and drop their stores by the descriptor's
// range, which the scalar offset does not enter); the head's column base is the scalar offset.
// Same MFMAs in the same order, masks, expf and stores: bit-identical to attn_f32_mfma_kernel<2>
// (tests/test_gpu_ops.py::test_attention_f32_batched_bit_identical).
__global__ __launch_bounds__(256, 2) void attn_f32_mfma_b_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                                int nseq, int S, int W, int causal) {
  constexpr int NKT = 2;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int H = W / 64;
  const int item = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform)
  if (item >= nseq * H) return;
  const int qend = ((causal >> 11) & 1) ? min(S, 32) : S;   // (bit 11: the first query block only)
  causal &= 1;
  const int bseq = item / H, head = item % H;
  const int ld = 3 * W;
  auto rho = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(qkv + (int64_t)bseq * S * ld), (short)0, S * ld * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (int64_t)bseq * S * W), (short)0, S * W * 4, 0x00020000);
  typedef unsigned int u32x4a __attribute__((ext_vector_type(4)));
  // row r's 32 columns 32 h .. 32 h + 31 of the block at column cb (Q: head * 64, K: W + head * 64)
  auto ld_row32 = [&](int r, int cb, float* v, float mul) {
    const uint32_t vo = (uint32_t)((r * ld + 32 * h) * 4);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const u32x4a t = __builtin_bit_cast(u32x4a, __builtin_amdgcn_raw_buffer_load_b128(rin, vo + 16 * c, cb * 4, 0));
      v[4 * c] = __uint_as_float(t[0]) * mul; v[4 * c + 1] = __uint_as_float(t[1]) * mul;
      v[4 * c + 2] = __uint_as_float(t[2]) * mul; v[4 * c + 3] = __uint_as_float(t[3]) * mul;
    }
  };
  // V[key rho(st, h) of key tile kt][32 dt + j], the B operand of step st
  auto ld_v = [&](int dt, float (&vv)[NKT][16]) {
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key = kt * 32 + (st & 3) + 8 * (st >> 2) + 4 * h;
        vv[kt][st] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rin, (uint32_t)((key * ld + j) * 4), (2 * W + head * 64 + 32 * dt) * 4, 0));
      }
  };
  for (int q0 = 0; q0 < qend; q0 += 32) {
    const int qi = q0 + j;   // this lane's query in the S^T layout
    float qv[32], kv[NKT][32], v0[NKT][16], v1[NKT][16];
    ld_row32(qi, head * 64, qv, 0.125f);
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) ld_row32(kt * 32 + j, W + head * 64, kv[kt], 1.0f);
    ld_v(0, v0);
    __builtin_amdgcn_sched_barrier(0);
    f32x16 sc[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      sc[kt] = f32x16{};
      if (kt * 32 >= S) continue;
#pragma unroll
      for (int st = 0; st < 32; ++st) sc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[kt][st], qv[st], sc[kt], 0, 0, 0);
    }
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + rho(r);
        if (key >= S || (causal && key > qi)) sc[kt][r] = -INFINITY;
        m = fmaxf(m, sc[kt][r]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = expf(sc[kt][r] - m);   // masked keys: exp(-inf) = 0
        sc[kt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    ld_v(1, v1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      f32x16 o = f32x16{};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt * 32 >= S) continue;
#pragma unroll
        for (int st = 0; st < 16; ++st)
          o = __builtin_amdgcn_mfma_f32_32x32x2f32(sc[kt][st], dt ? v1[kt][st] : v0[kt][st], o, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = q0 + rho(r);
        const float iv = __shfl(inv, rho(r), 64);   // 1 / l of query rho(r) (held by lane rho(r))
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[r] * iv), rout, (uint32_t)((qr * W + j) * 4),
                                              (head * 64 + 32 * dt) * 4, 0);
      }
    }
  }
}

// The fp32 tower's S <= 64 attention on the f16 MFMA over split operands (round 6; VERDICT r5 item
// 5): the operands of both products are split as the tower GEMMs' are (split2h: x s = x1 + x2 + r,
// |r| <= 2^-22 |x s|), and each product runs as three f16 MFMAs, a1 b1 + a1 b2 + a2 b1, with f32
// accumulation (the dropped a2 b2 <= 2^-22 |a b|): f32-GEMM-grade scores and outputs, like every
// other product of the tower.  Scales (powers of two, undone exactly after the MFMAs):
//   Q  per query row (the lane's 32 dims + its partner lane's: max |q s| in [2^13, 2^14));
//   K  one per (sequence, head) block: an element's error stays <= max(2^-22 |k|, 2^-39 max |K|),
//      so a key row far below the block's largest loses nothing that reaches a score at f32 grade;
//   V  per dim (the C layout of O keeps a dim in one lane);
//   P  2^14 (softmax values are in [0, 1], the row's largest exactly 1).
// Layout and loads as attn_f32_mfma_b_kernel: S^T = K Q^T then O = P V with v_mfma_f32_32x32x16_f16
// (k slot e of step c in lane half h = dim 32 h + 8 c + e; P straight from the S^T registers),
// 3 x (8 + 4) MFMAs of 32 cycles per 32-query block against 64 + 64 exact-f32 ones of 64.
typedef _Float16 f16x8_s __attribute__((ext_vector_type(8)));
typedef float f32x2_s __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_s __attribute__((ext_vector_type(2)));

typedef unsigned int u32x4_s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split8_s(const float* v, float s, f16x8_s& hi, f16x8_s& lo) {
  u32x4_s a4, b4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const f32x2_s x = (f32x2_s){v[2 * e] * s, v[2 * e + 1] * s};
    const f16x2_s a = __builtin_convertvector(x, f16x2_s);
    const f16x2_s b = __builtin_convertvector(x - __builtin_convertvector(a, f32x2_s), f16x2_s);
    a4[e] = __builtin_bit_cast(unsigned int, a);
    b4[e] = __builtin_bit_cast(unsigned int, b);
  }
  hi = __builtin_bit_cast(f16x8_s, a4);
  lo = __builtin_bit_cast(f16x8_s, b4);
}

// OUT 0: f32 out [rows][W].  OUT 1 / 2: out_proj's split operand straight from the registers
// (the split pass over the f32 output, split2h_rows role 0 / 2, folded in): o s = x1 + x2 stored as
// [x1 | x1 | x2] / [x1 | x2] fp16 rows (a3, row stride 3W / 2W) and rsc[row] = 1 / s.  A row's scale
// has to be one for all its heads (out_proj sums over them), so it comes from a bound instead of
// the row's max: |o[r][d]| <= max_k |V[k][d]| (softmax weights are a convex combination) and
// |V[k][d]| <= rmax[k] max_d sum_k' |W_v[d][k']| + max |b_v| (rmax: ln_1's row max |h|, bw / bb:
// the weight constants api.cpp computes at load), maximised over the sequence's rows and padded by
// 2^-8 for the rounding of the computed values; every head's wave derives the same power of two.
// A loose bound only lowers the split's subnormal floor (|o s| < 2^14 always), as EPI_SPLIT_GELU's.
template <int OUT, bool LATE = false>
__global__ __launch_bounds__(256, 2) void attn_f32s_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                          int nseq, int S, int W, int causal,
                                                          const float* __restrict__ rmax, float bw, float bb,
                                                          uint16_t* __restrict__ a3, float* __restrict__ rsc) {
  constexpr int NKT = 2;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int H = W / 64;
  const int item = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform)
  if (item >= nseq * H) return;
  const int qend = ((causal >> 11) & 1) ? min(S, 32) : S;   // (bit 11: the first query block only)
  causal &= 1;
  const int bseq = item / H, head = item % H;
  const int ld = 3 * W;
  auto rho = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(qkv + (int64_t)bseq * S * ld), (short)0, S * ld * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (int64_t)bseq * S * W), (short)0, OUT == 0 ? S * W * 4 : 0, 0x00020000);
  // OUT 1 / 2: the sequence's rows of the split operand, and their scale (see above)
  const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a3 + (OUT == 0 ? 0 : (int64_t)bseq * S * (OUT == 2 ? 2 : 3) * W)), (short)0,
      OUT == 0 ? 0 : S * (OUT == 2 ? 2 : 3) * W * 2, 0x00020000);
  // (the bound first: placed after the K / V loads it measured slower, 1737 vs 1578 us at 10k
  // frames, profiles/r06_za_bench.json)
  // (LATE, A/B MICLIP_F32_ATTN_LATE=1: the row-max load issued first and reduced where the first
  // query block's outputs are split, off the path to the K / V loads -- measured slower, 1537 vs
  // 1427 us at 10k frames, profiles/r06_ze_attn_split_micro.log: it holds 7 more registers)
  float so = 1.0f, rm = 0.f;
  auto bound_scale = [&]() {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rm = fmaxf(rm, __shfl_xor(rm, o, 64));
    const float bound = (rm * bw + bb) * (1.0f + 1.0f / 256.0f);
    const int eo = __builtin_amdgcn_readfirstlane(split_exp(bound));
    so = ldexpf(1.0f, eo);
    if (head == 0 && lane < S) rsc[(int64_t)bseq * S + lane] = ldexpf(1.0f, -eo);
  };
  if constexpr (OUT != 0) {
    rm = lane < S ? rmax[(int64_t)bseq * S + lane] : 0.f;
    if constexpr (!LATE) bound_scale();
  }
  typedef unsigned int u32x4a __attribute__((ext_vector_type(4)));
  auto ld_row32 = [&](int r, int cb, float* v) {   // row r, columns cb + 32 h .. + 31 (rows >= S: zeros)
    const uint32_t vo = (uint32_t)((r * ld + 32 * h) * 4);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const u32x4a t = __builtin_bit_cast(u32x4a, __builtin_amdgcn_raw_buffer_load_b128(rin, vo + 16 * c, cb * 4, 0));
      v[4 * c] = __uint_as_float(t[0]); v[4 * c + 1] = __uint_as_float(t[1]);
      v[4 * c + 2] = __uint_as_float(t[2]); v[4 * c + 3] = __uint_as_float(t[3]);
    }
  };
  // K of both key tiles and V of both dim tiles, once per (sequence, head)
  float kf[NKT][32], vf[2][NKT][16];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) ld_row32(kt * 32 + j, W + head * 64, kf[kt]);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key = kt * 32 + (st & 3) + 8 * (st >> 2) + 4 * h;
        vf[dt][kt][st] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rin, (uint32_t)((key * ld + j) * 4), (2 * W + head * 64 + 32 * dt) * 4, 0));
      }
  float km = 0.f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int i = 0; i < 32; ++i) km = fmaxf(km, fabsf(kf[kt][i]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) km = fmaxf(km, __shfl_xor(km, o, 64));
  const int ek = __builtin_amdgcn_readfirstlane(split_exp(km));
  const float sk = ldexpf(1.0f, ek), isk = ldexpf(1.0f, -ek);
  f16x8_s k1[NKT][4], k2[NKT][4];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int c = 0; c < 4; ++c) split8_s(&kf[kt][8 * c], sk, k1[kt][c], k2[kt][c]);
  f16x8_s v1[2][NKT][2], v2[2][NKT][2];
  float isv[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    float vm = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int st = 0; st < 16; ++st) vm = fmaxf(vm, fabsf(vf[dt][kt][st]));
    vm = fmaxf(vm, __shfl_xor(vm, 32, 64));
    const int ev = split_exp(vm);
    isv[dt] = ldexpf(1.0f, -ev - 14);   // (and P's 2^14)
    const float sv = ldexpf(1.0f, ev);
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int u = 0; u < 2; ++u) split8_s(&vf[dt][kt][8 * u], sv, v1[dt][kt][u], v2[dt][kt][u]);
  }
  for (int q0 = 0; q0 < qend; q0 += 32) {
    const int qi = q0 + j;   // this lane's query in the S^T layout
    float qv[32];
    ld_row32(qi, head * 64, qv);
    float qm = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) qm = fmaxf(qm, fabsf(qv[i]));
    qm = fmaxf(qm, __shfl_xor(qm, 32, 64));
    const int eq = split_exp(qm);
    const float sq = ldexpf(1.0f, eq), isq8 = ldexpf(0.125f, -eq);
    f16x8_s q1[4], q2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) split8_s(&qv[8 * c], sq, q1[c], q2[c]);
    f32x16 sc[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      sc[kt] = f32x16{};
      if (kt * 32 >= S) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1[kt][c], q1[c], sc[kt], 0, 0, 0);
        sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k1[kt][c], q2[c], sc[kt], 0, 0, 0);
        sc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k2[kt][c], q1[c], sc[kt], 0, 0, 0);
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + rho(r);
        sc[kt][r] = (sc[kt][r] * isk) * isq8;
        if (key >= S || (causal && key > qi)) sc[kt][r] = -INFINITY;
        m = fmaxf(m, sc[kt][r]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = expf(sc[kt][r] - m);   // masked keys: exp(-inf) = 0
        sc[kt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    f16x8_s p1[NKT][2], p2[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float pv[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) pv[t] = sc[kt][8 * u + t];
        split8_s(pv, 16384.0f, p1[kt][u], p2[kt][u]);
      }
    if constexpr (OUT != 0 && LATE) if (q0 == 0) bound_scale();
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      f32x16 o = f32x16{};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt * 32 >= S) continue;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          o = __builtin_amdgcn_mfma_f32_32x32x16_f16(p1[kt][u], v1[dt][kt][u], o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_f16(p1[kt][u], v2[dt][kt][u], o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_f16(p2[kt][u], v1[dt][kt][u], o, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = q0 + rho(r);
        const float iv = __shfl(inv, rho(r), 64);   // 1 / l of query rho(r) (held by lane rho(r))
        const float y = (o[r] * isv[dt]) * iv;
        if constexpr (OUT == 0) {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), rout, (uint32_t)((qr * W + j) * 4),
                                                (head * 64 + 32 * dt) * 4, 0);
        } else {
          // split2h's arithmetic; lanes j, j ^ 1 (dims d, d ^ 1 of row qr) pair their halves into
          // dwords: the even lane stores x1 of both, the odd lane x2 of both
          _Float16 x1, x2;
          split2h(y * so, x1, x2);
          const uint32_t b1 = __builtin_bit_cast(uint16_t, x1), b2 = __builtin_bit_cast(uint16_t, x2);
          const uint32_t mine = (j & 1) ? b1 : b2;   // what the partner lane needs
          const uint32_t got = (uint32_t)__builtin_amdgcn_mov_dpp((int)mine, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
          const uint32_t pk = (j & 1) ? (got | (b2 << 16)) : (b1 | (got << 16));
          // (no branch: the odd lane's offset selects the x2 block; OUT 1's second x1 copy is
          // stored by the even lanes, the odd lanes' copy goes out of the descriptor's range)
          const uint32_t ro = (uint32_t)((qr * (OUT == 2 ? 2 : 3) * W + (j & ~1)) * 2);
          const uint32_t xo = (j & 1) ? (uint32_t)((OUT == 2 ? 1 : 2) * W * 2) : 0u;
          __builtin_amdgcn_raw_buffer_store_b32(pk, rsp, ro + xo, (head * 64 + 32 * dt) * 2, 0);
          if (OUT == 1)
            __builtin_amdgcn_raw_buffer_store_b32(pk, rsp, (j & 1) ? 0x80000000u : ro + (uint32_t)(W * 2),
                                                  (head * 64 + 32 * dt) * 2, 0);
        }
      }
    }
  }
}

// The same kernel for S <= 64 (B/32's 50 tokens: the fp32 tower's attention) with every load of a
// (sequence, head) issued before its first MFMA (round 6).  attn_f32_mfma_kernel loads K and V
// inside its query-block loop (twice at S > 32), each key tile's K and each (dim tile, key tile)'s
// V as a batch that the next MFMAs wait for, and at 254 VGPRs hipcc reuses the load destinations,
// so the Q loads went out one at a time (a load, then vmcnt(0)): ~7 serialized HBM round trips per
// wave.  Here K and V of both key tiles (64 + 64 VGPRs) and the first query block's Q are in flight
// together, once per (sequence, head); the second block's Q goes out behind the first block's
// scores.  The MFMAs, their order, the masks, expf and the stores are attn_f32_mfma_kernel's, so
// the output is bit-identical (tests/test_gpu_ops.py::test_attention_f32_prefetch_bit_identical).
// Measured slower (scripts/attn_f32_micro.py, 10k B/32 frames: 2754 vs 2365 us,
// profiles/r06_n_attn_f32_micro.log): at 350 VGPRs one wave per SIMD, and nothing overlaps a
// wave's loads with another's MFMAs.  A/B only (MICLIP_ATTN_F32_V=3).
#if MICLIP_AB
template <int MINB>
__global__ __launch_bounds__(256, MINB) void attn_f32_mfma_pre_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                                int nseq, int S, int W, int causal) {
  constexpr int NKT = 2;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int H = W / 64;
  const int item = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform: SGPR descriptors)
  if (item >= nseq * H) return;
  const int qend = ((causal >> 11) & 1) ? min(S, 32) : S;   // (bit 11: the first query block only)
  causal &= 1;
  const int bseq = item / H, head = item % H;
  const int ld = 3 * W;
  auto rho = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(qkv + (int64_t)bseq * S * ld), (short)0, S * ld * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (int64_t)bseq * S * W), (short)0, S * W * 4, 0x00020000);
  typedef unsigned int u32x4a __attribute__((ext_vector_type(4)));
  auto ld4 = [&](int r, int col) {   // rows >= S are out of the descriptor's range: zeros
    const u32x4a t = __builtin_bit_cast(u32x4a, __builtin_amdgcn_raw_buffer_load_b128(rin, (uint32_t)((r * ld + col) * 4), 0, 0));
    return make_float4(__uint_as_float(t[0]), __uint_as_float(t[1]), __uint_as_float(t[2]), __uint_as_float(t[3]));
  };
  auto ld1 = [&](int r, int col) { return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rin, (uint32_t)((r * ld + col) * 4), 0, 0)); };
  auto load_q = [&](int q0, float (&qv)[32]) {   // (rows past S: zeros)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float4 t = ld4(q0 + j, head * 64 + 32 * h + 4 * c);
      qv[4 * c] = t.x * 0.125f; qv[4 * c + 1] = t.y * 0.125f; qv[4 * c + 2] = t.z * 0.125f; qv[4 * c + 3] = t.w * 0.125f;
    }
  };
  // every load of the item, ahead of the first MFMA: Q of block 0, K and V of both key tiles
  float qv[32], kv[NKT][32], vv[2][NKT][16];
  load_q(0, qv);
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float4 t = ld4(kt * 32 + j, W + head * 64 + 32 * h + 4 * c);
      kv[kt][4 * c] = t.x; kv[kt][4 * c + 1] = t.y; kv[kt][4 * c + 2] = t.z; kv[kt][4 * c + 3] = t.w;
    }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key = kt * 32 + (st & 3) + 8 * (st >> 2) + 4 * h;
        vv[dt][kt][st] = ld1(key, 2 * W + head * 64 + 32 * dt + j);
      }
  for (int q0 = 0; q0 < qend; q0 += 32) {
    const int qi = q0 + j;   // this lane's query in the S^T layout
    if (q0) load_q(q0, qv);
    f32x16 sc[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      sc[kt] = f32x16{};
      if (kt * 32 >= S) continue;
#pragma unroll
      for (int st = 0; st < 32; ++st) sc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[kt][st], qv[st], sc[kt], 0, 0, 0);
    }
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + rho(r);
        if (key >= S || (causal && key > qi)) sc[kt][r] = -INFINITY;
        m = fmaxf(m, sc[kt][r]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = expf(sc[kt][r] - m);   // masked keys: exp(-inf) = 0
        sc[kt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      f32x16 o = f32x16{};
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt * 32 >= S) continue;
#pragma unroll
        for (int st = 0; st < 16; ++st) o = __builtin_amdgcn_mfma_f32_32x32x2f32(sc[kt][st], vv[dt][kt][st], o, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = q0 + rho(r);
        const float iv = __shfl(inv, rho(r), 64);   // 1 / l of query rho(r) (held by lane rho(r))
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o[r] * iv), rout, (uint32_t)((qr * W + head * 64 + 32 * dt + j) * 4), 0, 0);
      }
    }
  }
}

#endif  // MICLIP_AB

// ------------------------------------------------------------------ im2col + split
// conv1's split-f16 operand straight from the pixels (P % 4 == 0, Kp = 3 P^2; B/32, B/16): one
// wave per patch row, its 3 P^2 values gathered as float4s (kw .. kw + 3 of one image row), then
// split2h_kernel's arithmetic (role 0, the same max / exponent / split) -- the values im2col_f32
// + split2h_rows produce, bit for bit, without writing and re-reading the f32 patches (6 GB at
// 10k B/32 frames: 5.7 + 2.8 ms -> one pass).
template <int NV>
__global__ __launch_bounds__(256) void im2col_split2h_kernel(const void* __restrict__ pixels, int in_bf16, int64_t rows,
                                                             int R, int P, int G, int K, _Float16* __restrict__ out,
                                                             float* __restrict__ sc) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int64_t bimg = row / (G * G);
  const int p = (int)(row % (G * G));
  const int gy = p / G, gx = p % G, PP = P * P;
  float4 v[NV];
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < K) {
      const int ch = c / PP, rem = c % PP, kh = rem / P, kw = rem % P;
      const int64_t off = ((bimg * 3 + ch) * R + (gy * P + kh)) * (int64_t)R + gx * P + kw;
      if (in_bf16) {
        const uint2 u = *(const uint2*)((const uint16_t*)pixels + off);
        v[i] = make_float4(bf2f((uint16_t)(u.x & 0xffff)), bf2f((uint16_t)(u.x >> 16)), bf2f((uint16_t)(u.y & 0xffff)),
                           bf2f((uint16_t)(u.y >> 16)));
      } else {
        v[i] = *(const float4*)((const float*)pixels + off);
      }
    }
    mx = absmax4(mx, v[i]);
  }
  const int e = split_exp(wave_max(mx));
  if (lane == 0) sc[row] = ldexpf(1.f, -e);
  _Float16* o = out + row * 3 * (int64_t)K;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    if (c < K) store_split4(v[i], e, 0, o, K, c);
  }
}

// ------------------------------------------------------------------ im2col
// patches [B*G*G, Kp] f32, k = c*P*P + kh*P + kw (conv1 weight order), zero pad.
__global__ __launch_bounds__(256) void im2col_f32_kernel(const void* __restrict__ pixels, int in_bf16,
                                                         float* __restrict__ out, int64_t total, int R, int P, int G,
                                                         int Kp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t prow = i / Kp;
  const int k = (int)(i % Kp);
  const int PP = P * P;
  float v = 0.f;
  if (k < 3 * PP) {
    const int64_t bimg = prow / (G * G);
    const int p = (int)(prow % (G * G));
    const int gy = p / G, gx = p % G;
    const int c = k / PP, rem = k % PP, kh = rem / P, kw = rem % P;
    const int64_t off = ((bimg * 3 + c) * R + (gy * P + kh)) * (int64_t)R + gx * P + kw;
    v = in_bf16 ? bf2f(((const uint16_t*)pixels)[off]) : ((const float*)pixels)[off];
  }
  out[i] = v;
}

}  // namespace

hipError_t gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, float* out,
                    int64_t ldo, int M, int N, int K, int epi, hipStream_t s, int group, int gstride, int goffset) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % GK || lda % 4 || ldw % 4) return hipErrorInvalidValue;
  const dim3 grid((N + GT - 1) / GT, (M + GT - 1) / GT), block(256);
  if (epi == EPI_F32)
    hipLaunchKernelGGL(gemm_f32_kernel<EPI_F32>, grid, block, 0, s, A, lda, W, ldw, bias, out, ldo, M, N, K, group,
                       gstride, goffset);
  else if (epi == EPI_GELU_BF16)
    hipLaunchKernelGGL(gemm_f32_kernel<EPI_GELU_BF16>, grid, block, 0, s, A, lda, W, ldw, bias, out, ldo, M, N, K,
                       group, gstride, goffset);
  else if (epi == EPI_RELU_F32)
    hipLaunchKernelGGL(gemm_f32_kernel<EPI_RELU_F32>, grid, block, 0, s, A, lda, W, ldw, bias, out, ldo, M, N, K,
                       group, gstride, goffset);
  else if (epi == EPI_RESID_F32)
    hipLaunchKernelGGL(gemm_f32_kernel<EPI_RESID_F32>, grid, block, 0, s, A, lda, W, ldw, bias, out, ldo, M, N, K,
                       group, gstride, goffset);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t split6_rows(const float* x, int64_t ldx, int64_t rows, int K, int role, int gelu, uint16_t* out,
                       hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (K % 4 || ldx % 4 || K < 4) return hipErrorInvalidValue;
  const int64_t n = rows * (K / 4);
  hipLaunchKernelGGL(split6_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ldx, rows, K, role, gelu, out);
  return hipGetLastError();
}

hipError_t split2h_rows(const float* x, int64_t ldx, int64_t rows, int K, int role, int gelu, uint16_t* out,
                        float* sc, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (K % 4 || ldx % 4 || K < 4 || K > 4096 || !sc) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((rows + 3) / 4));
  _Float16* o = (_Float16*)out;
  if (K <= 1024) hipLaunchKernelGGL(split2h_kernel<4>, grid, dim3(256), 0, s, x, ldx, rows, K, role, gelu, o, sc);
  else if (K <= 3072) hipLaunchKernelGGL(split2h_kernel<12>, grid, dim3(256), 0, s, x, ldx, rows, K, role, gelu, o, sc);
  else hipLaunchKernelGGL(split2h_kernel<16>, grid, dim3(256), 0, s, x, ldx, rows, K, role, gelu, o, sc);
  return hipGetLastError();
}

hipError_t layernorm_split2h(const float* x, int64_t in_stride, const float* g, const float* b, int rows, int W,
                             uint16_t* out, float* sc, hipStream_t s, float* rmax, int dup) {
  if (rows <= 0) return hipSuccess;
  if (W > 1024 || W < 4 || W % 4 || in_stride % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_split2h_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, in_stride, g, b, rows, W,
                     (_Float16*)out, sc, rmax, dup ? 1 : 0);
  return hipGetLastError();
}

hipError_t layernorm_f32(const float* x, int64_t in_stride, const float* g, const float* b, float* out,
                         int64_t out_stride, int rows, int W, hipStream_t s, const int32_t* tokens, int S) {
  if (rows <= 0) return hipSuccess;
  if (W > 1024 || W < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_f32_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, in_stride, g, b, out, out_stride, rows,
                     W, tokens, S);
  return hipGetLastError();
}

// the MFMA attention (S <= 128) is the default; MICLIP_ATTN_F32_MFMA=0 (A/B build) keeps the
// scalar kernel for comparison
static bool attn_f32_mfma_on() {
#if MICLIP_AB
  const char* e = std::getenv("MICLIP_ATTN_F32_MFMA");
  if (e) return std::atoi(e) != 0;
#endif
  return true;
}
static int attn_f32_variant() {
#if MICLIP_AB
  const char* e = std::getenv("MICLIP_ATTN_F32_V");
  if (e) return std::atoi(e);
#endif
  return 0;
}

hipError_t attention_f32(const float* qkv, float* out, int B, int S, int W, int causal, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (W % 64 || S < 1) return hipErrorInvalidValue;
  const int cq = causal;   // (bit 11: the first query block only, MFMA kernels; the scalar kernels compute all)
  causal &= 1;
  const dim3 grid((unsigned)B * (W / 64));
  const dim3 grid4((unsigned)(((int64_t)B * (W / 64) + 3) / 4));
#if MICLIP_AB
  if (attn_f32_mfma_on() && attn_f32_variant() == 1 && S <= 128) {   // 1: conditional loads / stores (A/B)
    if (S <= 64) hipLaunchKernelGGL((attn_f32_mfma_kernel<2, 1, false>), grid4, dim3(256), 0, s, qkv, out, B, S, W, causal);
    else if (S <= 96) hipLaunchKernelGGL((attn_f32_mfma_kernel<3, 1, false>), grid4, dim3(256), 0, s, qkv, out, B, S, W, causal);
    else hipLaunchKernelGGL((attn_f32_mfma_kernel<4, 1, false>), grid4, dim3(256), 0, s, qkv, out, B, S, W, causal);
    return hipGetLastError();
  }
#endif
#if MICLIP_AB   // 3: every load ahead of the first MFMA (attn_f32_mfma_pre_kernel; measured slower)
  if (attn_f32_mfma_on() && S <= 64 && attn_f32_variant() == 3) {
    hipLaunchKernelGGL((attn_f32_mfma_pre_kernel<1>), grid4, dim3(256), 0, s, qkv, out, B, S, W, cq);
    return hipGetLastError();
  }
#endif
  if (attn_f32_mfma_on() && S <= 64 && attn_f32_variant() == 0)   // split-f16 operands (round 6)
    hipLaunchKernelGGL(attn_f32s_kernel<0>, grid4, dim3(256), 0, s, qkv, out, B, S, W, cq, nullptr, 0.f, 0.f,
                       nullptr, nullptr);
  else if (attn_f32_mfma_on() && S <= 64 && attn_f32_variant() == 4)   // exact f32, batched loads (A/B)
    hipLaunchKernelGGL(attn_f32_mfma_b_kernel, grid4, dim3(256), 0, s, qkv, out, B, S, W, cq);
  else if (attn_f32_mfma_on() && S <= 64)   // (A/B MICLIP_ATTN_F32_V=2; held to 256 registers: two waves per SIMD)
    hipLaunchKernelGGL((attn_f32_mfma_kernel<2, 2>), grid4, dim3(256), 0, s, qkv, out, B, S, W, cq);
  else if (attn_f32_mfma_on() && S <= 96)
    hipLaunchKernelGGL(attn_f32_mfma_kernel<3>, grid4, dim3(256), 0, s, qkv, out, B, S, W, cq);
  else if (attn_f32_mfma_on() && S <= 128)
    hipLaunchKernelGGL(attn_f32_mfma_kernel<4>, grid4, dim3(256), 0, s, qkv, out, B, S, W, cq);
  else if (S <= 64)
    hipLaunchKernelGGL(attn_f32_kernel<64>, grid, dim3(64), 0, s, qkv, out, S, W, causal);
  else
    hipLaunchKernelGGL(attn_f32_kernel<256>, grid, dim3(256), 0, s, qkv, out, S, W, causal);
  return hipGetLastError();
}

hipError_t attention_f32_split(const float* qkv, const float* rmax, float bw, float bb, uint16_t* a3, int role,
                               float* rsc, int B, int S, int W, int causal, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (W % 64 || S < 1 || S > 64 || (role != 0 && role != 2)) return hipErrorInvalidValue;
  const dim3 grid4((unsigned)(((int64_t)B * (W / 64) + 3) / 4));
#if MICLIP_AB
  if (const char* le = std::getenv("MICLIP_F32_ATTN_LATE"); le && std::atoi(le) && role == 2) {
    hipLaunchKernelGGL((attn_f32s_kernel<2, true>), grid4, dim3(256), 0, s, qkv, nullptr, B, S, W, causal, rmax, bw, bb,
                       a3, rsc);
    return hipGetLastError();
  }
#endif
  if (role == 2)
    hipLaunchKernelGGL(attn_f32s_kernel<2>, grid4, dim3(256), 0, s, qkv, nullptr, B, S, W, causal, rmax, bw, bb, a3, rsc);
  else
    hipLaunchKernelGGL(attn_f32s_kernel<1>, grid4, dim3(256), 0, s, qkv, nullptr, B, S, W, causal, rmax, bw, bb, a3, rsc);
  return hipGetLastError();
}

hipError_t im2col_split2h(const void* pixels, int in_bf16, int B, int R, int P, int Kp, uint16_t* out, float* sc,
                          hipStream_t s) {
  const int G = R / P;
  const int64_t rows = (int64_t)B * G * G;
  if (rows <= 0) return hipSuccess;
  // float4 / 4 x bf16 loads of one image row: P % 4 == 0 (and R % 4 == 0 for their alignment), Kp = 3 P^2 <= 4096
  if (P % 4 || R % 4 || Kp != 3 * P * P || Kp > 4096 || !sc) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((rows + 3) / 4));
  _Float16* o = (_Float16*)out;
  if (Kp <= 1024) hipLaunchKernelGGL(im2col_split2h_kernel<4>, grid, dim3(256), 0, s, pixels, in_bf16, rows, R, P, G, Kp, o, sc);
  else if (Kp <= 3072) hipLaunchKernelGGL(im2col_split2h_kernel<12>, grid, dim3(256), 0, s, pixels, in_bf16, rows, R, P, G, Kp, o, sc);
  else hipLaunchKernelGGL(im2col_split2h_kernel<16>, grid, dim3(256), 0, s, pixels, in_bf16, rows, R, P, G, Kp, o, sc);
  return hipGetLastError();
}

hipError_t im2col_f32(const void* pixels, int in_bf16, float* out, int B, int R, int P, int Kp, hipStream_t s) {
  const int G = R / P;
  const int64_t total = (int64_t)B * G * G * Kp;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(im2col_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, pixels, in_bf16, out,
                     total, R, P, G, Kp);
  return hipGetLastError();
}

}  // namespace miclip
