// Host-side launchers shared between the kernel translation units and api.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef MICLIP_AB   // 1: the A/B build (common.hpp)
#define MICLIP_AB 0
#endif

namespace miclip {

enum GemmEpi {
  EPI_BF16 = 0,        // out bf16 = acc + bias
  EPI_GELU_BF16 = 1,   // out bf16 = quick_gelu(acc + bias)
  EPI_RESID_F32 = 2,   // out f32 += acc + bias   (residual stream, in place)
  EPI_F32 = 3,         // out f32 = acc (+ bias)
  EPI_GELU_MX = 4,     // MX-fp8 GEMM only: out e4m3 = MX(quick_gelu(acc + bias)), scales -> o_scale
  EPI_RELU_F32 = 5,    // f32 GEMM only: out f32 = max(acc + bias, 0)
  // LayerNorm folded into the GEMM (gemm_8q.hip, fp16 operands: A = the fp16 residual stream x,
  // W' = f16(W * gamma)): out bf16 = rstd_r * acc + (c_n - rstd_r * mean_r * s_n), c_n = bias
  // (= b + W beta), s_n = colv[n] (= sum_k W'[n][k]), (rstd_r, rstd_r * mean_r) = rs[r]
  EPI_LN_BF16 = 6,
  EPI_LN_GELU_BF16 = 7,    // the same, then QuickGELU
  // residual add fused (gemm_8q.hip, bf16 operands): out is the fp16 residual stream x16 (row
  // stride ldo), x16 = f16(x16 + bf16(acc + bias)) — residual_stats' arithmetic — and ps[r][n / 64]
  // = (sum, sum of squared deviations from that sum's mean) of the 64 stored values of row r,
  // columns n .. n + 63; residual_finalize turns a row's N / 64 partials into rs
  EPI_RES16_BF16 = 8,
  // split-f16 GEMM only (a_f16; the fp32 tower's c_fc): y = QuickGELU(acc * rsc[m] * csc[n] + b[n])
  // (the f32 expf form) written as the NEXT GEMM's split-f16 operand (role 0, fp16 [M][3N] at out,
  // ldo = 3N) with a per-row power-of-two scale from the bound |y| <= rmax[m] * bnd_w + bnd_b, and
  // rsc_out[m] = 1 / that scale (the n-tile-0 workgroups write it)
  EPI_SPLIT_GELU = 10
};

// MX block quantisation shared by the fp8 producers (gemm_mx.hip, encoder.hip):
// X = floor(log2 amax) - 8 clamped to [-127, 127] (amax = 0 -> -127);
// element = RNE e4m3 of clamp(v * 2^-X, +-448); scale byte = X + 127.
__device__ __forceinline__ int mx_block_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  int ex;
  (void)frexpf(amax, &ex);
  const int X = ex - 1 - 8;
  return X < -127 ? -127 : (X > 127 ? 127 : X);
}
__device__ __forceinline__ uint32_t mx_pack4(float a, float b, float c, float d, float inv) {
  a = fminf(fmaxf(a * inv, -448.f), 448.f);
  b = fminf(fmaxf(b * inv, -448.f), 448.f);
  c = fminf(fmaxf(c * inv, -448.f), 448.f);
  d = fminf(fmaxf(d * inv, -448.f), 448.f);
  uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
// scale byte index of (row r, 64-k block b) in the stage-major layout [K/128][rows_pad][2]
__device__ __forceinline__ int64_t mx_scale_index(int64_t r, int b, int64_t rows_pad) {
  return ((int64_t)(b >> 1) * rows_pad + r) * 2 + (b & 1);
}

struct GemmArgs {
  const uint16_t* A;  // [M, K] bf16, row stride lda
  const uint16_t* W;  // [N, K] bf16 (nn.Linear layout), row stride ldw
  const float* bias;  // [N] or nullptr
  void* out;          // see epilogue
  int64_t lda, ldw, ldo;
  int M, N, K;
  // output row remap: r -> (r / group) * gstride + goffset + r % group (group == 0: identity)
  int group, gstride, goffset;
  int variant;  // main-loop schedule (0 = default choice; see gemm.hip)
  const uint8_t *a_scale, *w_scale;  // MX-fp8 GEMM: e8m0 per 64 k, stage-major [K/128][rows_pad][2] (gemm_mx.hip)
  uint8_t* o_scale;                  // EPI_GELU_MX: scales of the fp8 output (same layout, rows = M)
  int ngroup;   // tile order: n-blocks per group (0 = m-major raster; gemm.hip tile_coords)
  // Fused patch gather (gemm.hip, bf16 A only): patch_R > 0 makes A the bf16
  // NCHW pixels [B,3,R,R] and row m the patch (m / G^2, m % G^2) of a P = 32
  // grid (K = 3*32*32, one 32-pixel image-row segment per BK = 32 stage), so
  // no im2col buffer is written or read.  0 = plain row-major A.
  int patch_R = 0;
  // persistent 8-phase kernels (gemm_8q.hip): workgroups start (blockIdx / 8) % stagger_phases x
  // stagger_ticks (100 MHz) late, so the CUs' tile epilogues (all 16 stores) do not coincide
  int stagger_phases = 0, stagger_ticks = 0;
  // EPI_LN_* (gemm_8q.hip): operands are fp16 (f16 MFMA) when a_f16; rs is readable for
  // 256 rows past M (the tile stages whole tiles' rows)
  int a_f16 = 0;
  const float* rs = nullptr;     // [M + 256][2] (rstd, rstd * mean) per row
  const float* colv = nullptr;   // [N] s_n
  float* ps = nullptr;           // EPI_RES16_BF16: [M][N / 64][2] row partial statistics
  // split-f16 operands (split2h_rows; a_f16 with EPI_F32 / EPI_RESID_F32): the accumulator is
  // multiplied by rsc[m] * csc[n] (powers of two) before the bias
  const float* rsc = nullptr;
  const float* csc = nullptr;
  // EPI_SPLIT_GELU: the input rows' max |a| (layernorm_split2h), the weights' max row 1-norm and
  // max |bias|, and the output row scales
  const float* rmax = nullptr;
  float bnd_w = 0.f, bnd_b = 0.f;
  float* rsc_out = nullptr;
  // split-f16 A operand stored once as [x1 | x2] (2 a_dup wide) for the logical [x1 | x1 | x2]
  // (K = 3 a_dup): K-tiles at k >= a_dup read from k - a_dup (gemm_8q only); 0 = the full layout
  int a_dup = 0;
  // EPI_SPLIT_GELU output in that layout ([y1 | y2], ldo = 2N; gemm_8q only)
  int o_dup = 0;
};

// Requirements: K % 64 == 0, N % 128 == 0, A/W 16-byte aligned rows.
hipError_t gemm_bf16(const GemmArgs& a, int epi, hipStream_t s);
// one-wave-per-SIMD 256x256x64 persistent kernel (gemm_w4.hip); bf16 epilogues only
int gemm_w4_ok(const GemmArgs& a);
hipError_t gemm_w4(const GemmArgs& a, int epi, hipStream_t s, int cus);
// 8-phase interleaved ping-pong, 256x256x64 persistent (gemm_8p.hip); bf16 epilogues, K % 128 == 0
int gemm_8p_ok(const GemmArgs& a);
hipError_t gemm_8p(const GemmArgs& a, int epi, hipStream_t s, int cus, int abl = 0);
// 8-phase, second schedule: descriptor DMAs, template-form waits, quadrant-split epilogue (gemm_8q.hip)
// LN-folded c_fc with the epilogue deferred into the next tile's MFMAs, one wave per SIMD
// (gemm_1d.hip, A/B build only); abl 4 = no-epilogue probe
int gemm_1d_ok(const GemmArgs& a);
hipError_t gemm_1d(const GemmArgs& a, int abl, hipStream_t s, int cus);
int gemm_8q_ok(const GemmArgs& a);
hipError_t gemm_8q(const GemmArgs& a, int epi, hipStream_t s, int cus, int mode = 0);
hipError_t gemm8q_probe_read(unsigned long long* host, int n);   // ABL 9 stamps (gemm_8q.hip)
// baseline JPEG decode (jpeg.hip); geom as mi_jpeg_decode
constexpr int JPEG_LDS_SETS = 4;   // table sets staged in LDS (4 x 3480 B each, <= 64 KB)
// fused output of jpeg_decode: out [B][3][n][n] (f32 / bf16) = mi_preprocess_frames(decoded RGB, n, mode)
struct JpegXform {
  int n, mode, out_bf16;
  void* out;
};
bool jpeg_xform_fits(int H, int W, int n, int mode);
hipError_t jpeg_decode(const uint8_t* data, int64_t data_bytes, const int64_t* seg_off, const int64_t* seg_end,
                       const void* huff, const int32_t* huff_idx, int nsets, const uint16_t* qtab, const int32_t* geom,
                       int nframes, uint8_t* out_rgb, void* ws, size_t ws_bytes, hipStream_t s,
                       const JpegXform* xf = nullptr);
size_t jpeg_workspace_bytes(const int32_t* geom, int nframes, int64_t data_bytes);
// 256 x 128 tiles, deferred (drained) epilogue, three-slot ring (gemm_8r.hip)
int gemm_8r_ok(const GemmArgs& a);
hipError_t gemm_8r(const GemmArgs& a, int epi, hipStream_t s, int cus, int mode = 0);
// variant 19's per-workgroup timestamps (gemm.hip g_gemm_probe) -> host
hipError_t gemm_probe_read(unsigned long long* host, int n);
// MX-fp8: A, W e4m3 bytes (row strides lda/ldw in BYTES), a_scale/w_scale e8m0; K % 128 == 0, N % 256 == 0
hipError_t gemm_mx(const GemmArgs& a, int epi, hipStream_t s);
// MX-fp8 on gemm_8q's 8-phase persistent schedule (gemm_mx8q.hip): bf16 / GELU-bf16 / GELU-MX epilogues
int gemm_mx8q_ok(const GemmArgs& a, int epi);
hipError_t gemm_mx8q(const GemmArgs& a, int epi, hipStream_t s, int cus);
int cu_count();   // compute units of the current device (gemm.hip)
// bf16 [rows][K] -> e4m3 [rows][K] + e8m0 scales [K/128][rows_pad][2] (one per 64 k; K % 128 == 0)
hipError_t quantize_mx(const uint16_t* in, int64_t ld_in, uint8_t* q, int64_t ld_q, uint8_t* sc, int rows, int K,
                       hipStream_t s);

// out[r] = LN(x[r * in_stride]) over W features; out is bf16 (row stride out_stride).
// q != nullptr: MX-fp8 output instead (q [rows][W] e4m3 + qs stage-major scales, W % 128 == 0)
hipError_t layernorm_bf16(const float* x, int64_t in_stride, const float* g, const float* b,
                          uint16_t* out, int64_t out_stride, int rows, int W, hipStream_t s,
                          uint8_t* q = nullptr, uint8_t* qs = nullptr);
// x[b*S + t] = LN((t == 0 ? cls : x[b*S + t]) + pos[t]) in place (f32); with
// h != nullptr also h = LN_{g1,b1}(x) in bf16 (the first block's ln_1, fused)
hipError_t vision_embed_ln(float* x, const float* cls, const float* pos, const float* g,
                           const float* b, int B, int S, int W, hipStream_t s, const float* g1 = nullptr,
                           const float* b1 = nullptr, uint16_t* h = nullptr);
// LayerNorm-folded vision tower (EPI_LN_*): x = ln_pre([CLS | patches] + pos) written as fp16
// into the first half of each f32 row slot (element (r, j) at ((half*)x)[2 r W + j]) and
// rs[r] = (rstd, rstd * mean) of those fp16 values (the first block's ln_1 statistics)
hipError_t vision_embed_ln16(float* x, const float* cls, const float* pos, const float* g, const float* b, int B,
                             int S, int W, float* rs, hipStream_t s);
// x16[r] = f16(x16[r] + delta[r]) in that half-row layout and rs[r] = (rstd, rstd * mean) of the
// stored fp16 values: the residual add of residual_ln without its LayerNorm output (the
// consumer GEMM applies the LayerNorm in its epilogue, EPI_LN_*)
hipError_t residual_stats(float* x, const uint16_t* delta, float* rs, int rows, int W, hipStream_t s);
// rs[r] = (rstd, rstd * mean) from the W / 64 partials ps[r][j] = (sum, M2) of EPI_RES16_BF16
// (Chan's pairwise combination of equal-count groups), W % 128 == 0, W <= 1024
hipError_t residual_finalize(const float* ps, float* rs, int rows, int W, hipStream_t s);
// x[q*S + t] = tok_emb[tokens[q*S + t]] + pos[t]
hipError_t text_embed(const int32_t* tokens, const float* tok_emb, const float* pos, float* x,
                      int Q, int S, int W, int vocab, hipStream_t s);
// out[q] = LN(x[r] (+ delta[r])), r = q*S + argmax_t tokens[q*S + t]; bf16
hipError_t eot_gather_ln(const int32_t* tokens, const float* x, const uint16_t* delta, const float* g,
                         const float* b, uint16_t* out, int Q, int S, int W, hipStream_t s);
// row r = i*stride: xr = x[r] + delta[r] (bf16); if write_x: x[r] = xr; out[i] = LN(xr) bf16 [rows, W].
// xmode: 0 residual f32; 1 f32 in, fp16 out (half-row layout); 2 fp16 in/out (encoder.hip)
hipError_t residual_ln(float* x, const uint16_t* delta, int64_t stride, int write_x, const float* g, const float* b,
                       uint16_t* out, int rows, int W, hipStream_t s, uint8_t* q = nullptr, uint8_t* qs = nullptr,
                       int xmode = 0);
// pixels [B,3,R,R] (f32 or bf16) -> patches [B*G*G, Kp] bf16, k = c*P*P + kh*P + kw, zero pad to Kp
hipError_t im2col(const void* pixels, int in_bf16, uint16_t* out, int B, int R, int P, int Kp,
                  hipStream_t s);
// multi-head attention over qkv [B*S, 3W] bf16 -> out [B*S, W] bf16, head dim 64
// q8 != nullptr: MX-fp8 output (one 64-k block per head) instead of bf16 out
hipError_t attention(const uint16_t* qkv, uint16_t* out, int B, int S, int W, int causal,
                     hipStream_t s, uint8_t* q8 = nullptr, uint8_t* qs = nullptr);
// y [rows, D] f32 -> out (f32/bf16/f16), optional L2 normalisation
hipError_t finalize_rows(const float* y, void* out, int out_dtype, int rows, int D, int l2,
                         hipStream_t s);

// ---- fp32 tower (precise.hip; weight_dtype MI_F32) ----
// out = A[M,K] . W[N,K]^T (+bias), all f32, K % 32 == 0; epi EPI_F32 (store),
// EPI_GELU_BF16 (QuickGELU, stored f32), EPI_RESID_F32 (out += ...); group /
// gstride / goffset remap output rows as GemmArgs does
hipError_t gemm_f32(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, float* out,
                    int64_t ldo, int M, int N, int K, int epi, hipStream_t s, int group = 0, int gstride = 0,
                    int goffset = 0);
// out[r] = LN(x[r * in_stride]) f32; tokens != nullptr: source row r*S + argmax(tokens[r]) (EOT pooling)
hipError_t layernorm_f32(const float* x, int64_t in_stride, const float* g, const float* b, float* out,
                         int64_t out_stride, int rows, int W, hipStream_t s, const int32_t* tokens = nullptr,
                         int S = 0);
// MHA core over qkv f32 [B*S, 3W] -> out f32 [B*S, W], head dim 64
hipError_t attention_f32(const float* qkv, float* out, int B, int S, int W, int causal, hipStream_t s);
// S <= 64: the attention output as out_proj's split operand (role 0 [x1 x1 x2] / role 2 [x1 x2],
// a3 row stride 3W / 2W fp16) and rsc[row] = 1 / s, s from the bound rmax[row] * bw + bb over the
// sequence's rows (precise.hip attn_f32s_kernel)
hipError_t attention_f32_split(const float* qkv, const float* rmax, float bw, float bb, uint16_t* a3, int role,
                               float* rsc, int B, int S, int W, int causal, hipStream_t s);
// pixels [B,3,R,R] (f32 / bf16) -> patches f32 [B*G*G, Kp]
hipError_t im2col_f32(const void* pixels, int in_bf16, float* out, int B, int R, int P, int Kp, hipStream_t s);
// im2col_f32 + split2h_rows (role 0) in one pass: conv1's split operand [B G^2][3 Kp] fp16 and its
// row scales straight from the pixels (bit-identical); P % 4 == 0, R % 4 == 0, Kp == 3 P^2 <= 4096
hipError_t im2col_split2h(const void* pixels, int in_bf16, int B, int R, int P, int Kp, uint16_t* out, float* sc,
                          hipStream_t s);
// Split-bf16 operands of the fp32 tower's GEMMs (precise.hip): each f32 value x = x1 + x2 + x3
// + O(2^-24 |x|) with x1 = bf16(x), x2 = bf16(x - x1), x3 = bf16(x - x1 - x2); a row of K values
// becomes 6K bf16 in six K-blocks, activations (role 0) as [x1 x2 x3 x1 x2 x1] and weights
// (role 1) as [w1 w1 w1 w2 w2 w3], so ONE bf16 GEMM over K' = 6K sums a1w1 + a2w1 + a3w1 +
// a1w2 + a2w2 + a1w3: every product term down to 2^-16 relative, f32 accumulation.
// gelu: QuickGELU (the fp32 epilogue's expf form) applied to x first (c_proj's input).
hipError_t split6_rows(const float* x, int64_t ldx, int64_t rows, int K, int role, int gelu, uint16_t* out,
                       hipStream_t s);
// Split-f16 operands (precise.hip; the fp32 tower's default since round 5): row r of x scaled by
// a power of two s_r (max |x s_r| in [2^13, 2^14)) becomes 3K fp16 as [x1 x1 x2] (role 0,
// activations) or [x1 x2 x1] (role 1, weights), x1 = f16(x s), x2 = f16(x s - x1), and
// sc[r] = 1 / s_r; ONE f16 GEMM over K' = 3K with epilogue factor rsc[m] * csc[n] (GemmArgs)
// then gives a1 w1 + a1 w2 + a2 w1 in f32: every term to 2^-22 relative.  K % 4 == 0, K <= 4096.
// role 2: activations stored once, [x1 x2] (row stride 2K), for the 8-phase GEMM's A_DUP read of
// the logical [x1 x1 x2] (GemmArgs a_dup).
hipError_t split2h_rows(const float* x, int64_t ldx, int64_t rows, int K, int role, int gelu, uint16_t* out,
                        float* sc, hipStream_t s);
// LayerNorm (f32 statistics) written directly as the split-f16 operand (role 0) + its row scales
// rmax (nullable): the row's max |LN(x)| (EPI_SPLIT_GELU's bound)
// (dup: the [x1 x2] layout of role 2)
hipError_t layernorm_split2h(const float* x, int64_t in_stride, const float* g, const float* b, int rows, int W,
                             uint16_t* out, float* sc, hipStream_t s, float* rmax = nullptr, int dup = 0);

}  // namespace miclip

namespace miclip {
constexpr int RANK_REG_K = 64;          // register top-k lists (rank_stage1) up to this k
constexpr int RANK_MAX_K = 1 << 24;     // select + sort path above it (rank.hip)
constexpr int RANK_MAX_D = 1024;        // 32 queries x (D + 4) f32 staged in LDS
size_t rank_workspace_bytes(int64_t N, int64_t Q, int k);
hipError_t rank_topk(const void* corpus, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int k,
                     int64_t base, int norm_mode, int nan_first, float* out_s, int64_t* out_i, void* ws,
                     hipStream_t s);
hipError_t rank_merge(const float* cs, const int64_t* ci, int64_t Q, int64_t C, int k, int nan_first, float* out_s,
                      int64_t* out_i, hipStream_t s);
// out_s = -inf, out_i = -1 for all Q x k slots (empty corpus)
hipError_t rank_fill_empty(int64_t Q, int k, float* out_s, int64_t* out_i, hipStream_t s);
hipError_t score_matrix(const void* corpus, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int norm_mode,
                        float* out, hipStream_t s);
hipError_t rank_of_targets(const float* S, int64_t Q, int64_t N, const int64_t* pq, const int64_t* pt, int64_t T,
                           int64_t* out, hipStream_t s);
// mirrored corpus (rank_mirror.hip): fp16 unit-row mirror + certified exact re-score, k <= 16
constexpr int MIRROR_MAX_K = 16;
int rank_mirror_supported(int64_t D);
size_t rank_mirror_workspace_bytes(int64_t N, int64_t Q);
hipError_t mirror_build(const void* master, int64_t N, int64_t D, int dt, uint16_t* mirror, hipStream_t s);
hipError_t rank_mirror(const uint16_t* mirror, const void* master, int64_t N, int64_t D, int dt, const float* q,
                       int64_t Q, int k, int64_t base, int nan_first, float* out_s, int64_t* out_i, int32_t* cert,
                       void* ws, hipStream_t s);
// exact re-score + certificate of kc candidates per query (rank_mirror.hip): out = their exact top-k,
// cert[q] = 1 when no row outside them can reach the top-k (|s_cand - s_exact| <= d_rel |q| + d_abs);
// unsafe (nullable): a device flag that uncertifies every query when set
hipError_t rank_rescore(const void* master, int64_t N, int64_t D, int dt, const float* q, int64_t Q, int k, int kc,
                        const float* m_s, const int64_t* m_i, int64_t base, float d_rel, float d_abs, int norm_mode,
                        int nan_first, const int32_t* unsafe, float* out_s, int64_t* out_i, int32_t* cert,
                        hipStream_t s, uint32_t* zero = nullptr, int64_t zero_words = 0);
// (zero / zero_words: words the re-score kernel clears for the launch after it)
// certified bf16-MFMA ranking pass (rank_cert.hip): f32 / bf16 rows, D = 512, k <= 12, L2 norms
int64_t rank_cert_min_rows();
bool rank_cert_eligible(int64_t N, int64_t D, int dt, int k, int norm_mode);
size_t rank_cert_ws_bytes(int64_t N, int64_t Q);
void rank_cert_delta(int dt, float& d_rel, float& d_abs);
// certified queries' results in out; *cert_out = the per-query certificates (in ws) for the gated exact pass
hipError_t rank_cert_topk(const void* corpus, int64_t N, int dt, const float* q, int64_t Q, int k, int64_t base,
                          int norm_mode, int nan_first, float* out_s, int64_t* out_i, void* ws, int32_t** cert_out,
                          hipStream_t s, uint32_t* zero = nullptr, int64_t zero_words = 0);
// float16 corpus rows normalised as NumPy does it in float16 (corpus.hip;
// embedding_service.py:209-210): the host-planned pairwise-summation tree of
// the row's squares (leaves <= 128 elements, ops 0 = next leaf, 1 = add)
struct PairwisePlan {
  int32_t nleaf, nops;
  int16_t start[8], len[8];
  int8_t ops[16];
};
PairwisePlan pairwise_plan(int D);
// out[r] = f16(in[r] / f16 norm(in[r])) per NumPy float16; D in [1, 1024]; in == out allowed
hipError_t normalize_rows_f16(const uint16_t* in, int64_t N, int D, uint16_t* out, hipStream_t s);
}  // namespace miclip

#include <vector>
namespace miclip {
// Pillow ImagingResample coefficients (csrc/preprocess.hip): filter 0 bicubic,
// 1 bilinear; returns ksize (< 0 on error), kk [out_size][ksize] int32 (22
// fractional bits), bounds [out_size][2] = (first tap, tap count).
int resample_coeffs(int in_size, double in0, double in1, int out_size, int filter, std::vector<int32_t>& kk,
                    std::vector<int32_t>& bounds);
size_t preprocess_workspace_bytes(int64_t B, int H, int W, int n, int mode);
// the device coefficient tables of mi_preprocess_frames' resample (H x W -> n x n crop, mode as
// there): horizontal kh [n][ksh] / bh [n][2], vertical kv [n][ksv] / bv [n][2] (Pillow's int32
// coefficients and (first tap, taps)); the crop's source columns [xlo, xlo + xw); bv on the host
struct ResampleTables {
  const int32_t *kh = nullptr, *bh = nullptr, *kv = nullptr, *bv = nullptr;
  int ksh = 0, ksv = 0, xlo = 0, xw = 0;
  std::vector<int32_t> hbv;
  int32_t wmax = 0;   // largest |coefficient|
};
hipError_t resample_tables(int H, int W, int n, int mode, ResampleTables& t);
// frames uint8 [B,H,W,3] -> out [B,3,n,n] f32 / bf16; mode 0 CLIP _transform, 1 squash (bilinear)
hipError_t preprocess_frames(const uint8_t* frames, int64_t B, int H, int W, int n, int mode, void* out,
                             int out_bf16, void* ws, hipStream_t s);
}  // namespace miclip
