// C-ABI of libmiclip (include/miclip.h): model context, weight upload,
// encode orchestration and the ranking entry points.
//
// encode_image follows openai/CLIP VisionTransformer.forward (restated in
// oracle/clip_ref.py::encode_image): im2col + conv1 GEMM -> [CLS|patches]+pos
// -> ln_pre -> L x {LN -> QKV GEMM -> attention -> out-proj GEMM (+residual)
// -> LN -> c_fc GEMM (+QuickGELU) -> c_proj GEMM (+residual)} -> ln_post(CLS)
// -> proj GEMM.  encode_text: token gather + pos -> L causal blocks ->
// ln_final at argmax(tokens) -> text_projection GEMM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/miclip.h"
#include "src_hash.h"   // MICLIP_SRC_HASH / MICLIP_SRC_FILES (Makefile)
#include "internal.hpp"

using namespace miclip;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail(MI_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                                      \
  } while (0)

#define MI_TRY(expr)      \
  do {                    \
    const int r_ = (expr); \
    if (r_) return r_;    \
  } while (0)

uint16_t f2bf_host(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct Layer {
  const float *ln1_g, *ln1_b, *b_qkv, *b_out, *ln2_g, *ln2_b, *b_fc, *b_proj;
  const uint16_t *w_qkv, *w_out, *w_fc, *w_proj;
  // f32 GEMM weights (weight_dtype MI_F32): the same [N][K] matrices kept in f32
  const float *f_qkv = nullptr, *f_out = nullptr, *f_fc = nullptr, *f_proj = nullptr;
  // ... and split into three bf16 terms, [N][6K] (split6_rows role 1): the split-bf16 GEMMs
  const uint16_t *s6_qkv = nullptr, *s6_out = nullptr, *s6_fc = nullptr, *s6_proj = nullptr;
  // ... or split into two fp16 terms, [N][3K] (split2h_rows role 1) + their column scales: the
  // split-f16 GEMMs (the default since round 5)
  const uint16_t *h3_qkv = nullptr, *h3_out = nullptr, *h3_fc = nullptr, *h3_proj = nullptr;
  const float *c3_qkv = nullptr, *c3_out = nullptr, *c3_fc = nullptr, *c3_proj = nullptr;
  // c_fc's output bound for the fused split (EPI_SPLIT_GELU): max_n sum_k |W_fc| and max |b_fc|
  float fc_bw = 0.f, fc_bb = 0.f;
  // the same for attention's output split (attention_f32_split): max over V's rows of sum_k |W_v|
  // and max |b_v| (rows 2W .. 3W of in_proj)
  float v_bw = 0.f, v_bb = 0.f;
  // MX-fp8 copies (weight_dtype MI_FP8, vision tower): e4m3 codes + stage-major e8m0 scales
  const uint8_t *q_qkv = nullptr, *s_qkv = nullptr, *q_out = nullptr, *s_out = nullptr;
  const uint8_t *q_fc = nullptr, *s_fc = nullptr, *q_proj = nullptr, *s_proj = nullptr;
  // LayerNorm-folded copies (bf16 vision tower, run_tower_fold): W' = f16(W * gamma) of
  // in_proj (ln_1) and c_fc (ln_2), their column sums s_n and c_n = b_n + W beta
  const uint16_t *lw_qkv = nullptr, *lw_fc = nullptr;
  const float *ls_qkv = nullptr, *lc_qkv = nullptr, *ls_fc = nullptr, *lc_fc = nullptr;
};

// Device weight image: bf16 GEMM weights and f32 vectors in one allocation.
// Built by walking the canonical host blob (DESIGN.md "Weight blob").
struct Builder {
  const float* src;   // host blob
  int64_t pos = 0;    // elements consumed
  int64_t numel;
  std::vector<char> img;  // host copy of the device image
  bool ok = true;

  const float* take(int64_t n) {
    if (pos + n > numel) { ok = false; return nullptr; }
    const float* p = src + pos;
    pos += n;
    return p;
  }
  size_t align() {
    size_t o = (img.size() + 255) & ~(size_t)255;
    img.resize(o);
    return o;
  }
  size_t f32(int64_t n) {  // copy n floats as-is
    const float* p = take(n);
    size_t o = align();
    img.resize(o + n * 4);
    if (p) memcpy(img.data() + o, p, n * 4);
    return o;
  }
  // rows x cols fp32 matrix -> f32 [rows][ldp] (zero padded columns)
  size_t f32_pad(int64_t rows, int64_t cols, int64_t ldp) {
    const float* p = take(rows * cols);
    size_t o = align();
    img.resize(o + rows * ldp * 4);
    float* d = (float*)(img.data() + o);
    for (int64_t r = 0; r < rows; ++r)
      for (int64_t c = 0; c < ldp; ++c) d[r * ldp + c] = (p && c < cols) ? p[r * cols + c] : 0.f;
    return o;
  }
  // [rows][cols] fp32 used as x @ P  ->  f32 P^T [cols][rows]
  size_t f32_t(int64_t rows, int64_t cols) {
    const float* p = take(rows * cols);
    size_t o = align();
    img.resize(o + rows * cols * 4);
    float* d = (float*)(img.data() + o);
    for (int64_t c = 0; c < cols; ++c)
      for (int64_t r = 0; r < rows; ++r) d[c * rows + r] = p ? p[r * cols + c] : 0.f;
    return o;
  }
  // GEMM weight in the context's precision
  size_t mat(bool full, int64_t rows, int64_t cols, int64_t ldp) {
    return full ? f32_pad(rows, cols, ldp) : bf16(rows, cols, ldp);
  }
  size_t mat_t(bool full, int64_t rows, int64_t cols) { return full ? f32_t(rows, cols) : bf16_t(rows, cols); }
  // rows x cols fp32 matrix -> bf16 [rows][ldp] (zero padded columns)
  size_t bf16(int64_t rows, int64_t cols, int64_t ldp) {
    const float* p = take(rows * cols);
    size_t o = align();
    img.resize(o + rows * ldp * 2);
    uint16_t* d = (uint16_t*)(img.data() + o);
    for (int64_t r = 0; r < rows; ++r)
      for (int64_t c = 0; c < ldp; ++c) d[r * ldp + c] = (p && c < cols) ? f2bf_host(p[r * cols + c]) : 0;
    return o;
  }
  // [rows][cols] fp32 used as x @ P  ->  bf16 P^T [cols][rows]
  size_t bf16_t(int64_t rows, int64_t cols) {
    const float* p = take(rows * cols);
    size_t o = align();
    img.resize(o + rows * cols * 2);
    uint16_t* d = (uint16_t*)(img.data() + o);
    for (int64_t c = 0; c < cols; ++c)
      for (int64_t r = 0; r < rows; ++r) d[c * rows + r] = p ? f2bf_host(p[r * cols + c]) : 0;
    return o;
  }
};

struct LayerOff {
  size_t ln1_g, ln1_b, w_qkv, b_qkv, w_out, b_out, ln2_g, ln2_b, w_fc, b_fc, w_proj, b_proj;
  // blob positions of the tensors the LayerNorm fold reads
  int64_t p_ln1_g, p_ln1_b, p_w_qkv, p_b_qkv, p_ln2_g, p_ln2_b, p_w_fc, p_b_fc;
  size_t lw_qkv = 0, ls_qkv = 0, lc_qkv = 0, lw_fc = 0, ls_fc = 0, lc_fc = 0;   // 0: not folded
};

void build_tower(Builder& b, int W, int L, std::vector<LayerOff>& out, bool full) {
  out.resize(L);
  for (int i = 0; i < L; ++i) {
    LayerOff& l = out[i];
    l.p_ln1_g = b.pos;
    l.ln1_g = b.f32(W);
    l.p_ln1_b = b.pos;
    l.ln1_b = b.f32(W);
    l.p_w_qkv = b.pos;
    l.w_qkv = b.mat(full, 3 * W, W, W);
    l.p_b_qkv = b.pos;
    l.b_qkv = b.f32(3 * W);
    l.w_out = b.mat(full, W, W, W);
    l.b_out = b.f32(W);
    l.p_ln2_g = b.pos;
    l.ln2_g = b.f32(W);
    l.p_ln2_b = b.pos;
    l.ln2_b = b.f32(W);
    l.p_w_fc = b.pos;
    l.w_fc = b.mat(full, 4 * W, W, W);
    l.p_b_fc = b.pos;
    l.b_fc = b.f32(4 * W);
    l.w_proj = b.mat(full, W, 4 * W, 4 * W);
    l.b_proj = b.f32(W);
  }
}

uint16_t f2h_host(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

// LayerNorm folded into the following GEMM (ln_1 -> in_proj, ln_2 -> c_fc; gemm_8q.hip EPI_LN_*):
//   LN(x) W^T + b = rstd * (x W'^T) - rstd * mean * s + c,
//   W'[n][k] = f16(W[n][k] * gamma[k]),  s_n = sum_k W'[n][k],  c_n = b_n + sum_k beta[k] W[n][k]
// (s from the rounded W', so that x W'^T - mean s = (x - mean) W'^T exactly; sums in double).
// Appends W' (f16 [N][K]), s and c (f32 [N]) to the image; returns their offsets.
// Returns false when a product W * gamma leaves the fp16 range (|W'| > 65504 rounds to inf) or a
// column sum / constant is not finite: the caller then keeps the unfolded tower.
bool fold_ln(Builder& b, int64_t p_g, int64_t p_beta, int64_t p_w, int64_t p_bias, int N, int K, size_t& ow,
             size_t& os, size_t& oc) {
  const float* g = b.src + p_g;
  const float* be = b.src + p_beta;
  const float* w = b.src + p_w;
  const float* bias = b.src + p_bias;
  ow = b.align();
  b.img.resize(ow + (size_t)N * K * 2);
  std::vector<float> sv(N), cv(N);
  bool finite = true;
  for (int n = 0; n < N; ++n) {
    uint16_t* d = (uint16_t*)(b.img.data() + ow) + (size_t)n * K;
    double ss = 0, cc = bias[n];
    for (int k = 0; k < K; ++k) {
      const float wv = w[(size_t)n * K + k];
      const uint16_t h = f2h_host(wv * g[k]);
      d[k] = h;
      _Float16 hv;
      memcpy(&hv, &h, 2);
      finite = finite && std::isfinite((float)hv);
      ss += (double)(float)hv;
      cc += (double)be[k] * (double)wv;
    }
    sv[n] = (float)ss;
    cv[n] = (float)cc;
    finite = finite && std::isfinite(sv[n]) && std::isfinite(cv[n]);
  }
  os = b.align();
  b.img.resize(os + (size_t)N * 4);
  memcpy(b.img.data() + os, sv.data(), (size_t)N * 4);
  oc = b.align();
  b.img.resize(oc + (size_t)N * 4);
  memcpy(b.img.data() + oc, cv.data(), (size_t)N * 4);
  return finite;
}

int64_t tower_numel(int64_t W, int64_t L) { return L * (W * 2 + 3 * W * W + 3 * W + W * W + W + 2 * W + 4 * W * W + 4 * W + 4 * W * W + W); }

}  // namespace

struct mi_clip {
  mi_clip_arch a;
  int device = 0;
  int S_v = 0, G = 0, Kp = 0;
  char* wdev = nullptr;
  bool fp8 = false;       // vision tower GEMMs on the MX-fp8 MFMA
  bool f32 = false;       // weight_dtype MI_F32: every GEMM, activation and the residual stream in f32 (precise.hip)
  int Kp32 = 0;           // f32 mode: conv1 K padded to the f32 GEMM's 32-k stage
  const float *conv_f = nullptr, *vproj_f = nullptr, *tproj_f = nullptr;
  char* wq = nullptr;     // MX-fp8 weight copies
  char* w6 = nullptr;     // f32 mode, A/B: split-bf16 weight copies (Layer::s6_*)
  char* w3 = nullptr;     // f32 mode: split-f16 weight copies + column scales (Layer::h3_* / c3_*, conv_h3)
  const uint16_t* conv_h3 = nullptr;
  const float* conv_c3 = nullptr;
  float* rsc = nullptr;   // f32 mode: row scales of the split-f16 activations (workspace, 3 x rsc_rows)
  int64_t rsc_rows = 0;
  uint16_t* a6 = nullptr; // f32 mode: split-bf16 activations of one GEMM, [M][6K] (workspace)
  // vision
  const uint16_t* conv_w = nullptr;
  const float *cls = nullptr, *vpos = nullptr, *ln_pre_g = nullptr, *ln_pre_b = nullptr, *ln_post_g = nullptr,
              *ln_post_b = nullptr;
  const uint16_t* vproj_t = nullptr;
  std::vector<Layer> vl, tl;
  // text
  const float *tok_emb = nullptr, *tpos = nullptr, *lnf_g = nullptr, *lnf_b = nullptr;
  const uint16_t* tproj_t = nullptr;
  // workspace
  int64_t img_chunk = 0, txt_chunk = 0;
  char* ws = nullptr;
  float* x = nullptr;
  uint16_t *h = nullptr, *qkv = nullptr, *att = nullptr, *mlp = nullptr, *patches = nullptr, *cls_ln = nullptr;
  uint16_t* delta = nullptr;  // bf16 GEMM output added to x by the next residual_ln
  float* rs = nullptr;        // LayerNorm-folded tower: per-row (rstd, rstd * mean), 256 rows of padding
  float* y = nullptr;
  // MX-fp8 activations (fp8 mode): LN outputs, attention output, QuickGELU(c_fc) + their scales
  uint8_t *hq = nullptr, *hqs = nullptr, *attq = nullptr, *attqs = nullptr, *mlpq = nullptr, *mlpqs = nullptr;
  std::mutex mu;
  // workspace ordering across streams: the encoders' kernels run on the caller's stream, the
  // mutex only covers their launch, so a call on another stream first waits for the event
  // recorded after the previous call's last kernel
  hipEvent_t ws_evt = nullptr;
  // kernel timing (mi_clip_kernel_events): start / stop events around the launches of one tower GEMM
  int ev_kind = 0, ev_cap = 0, ev_n = 0;
  std::vector<hipEvent_t> ev;
  hipStream_t ws_stream = nullptr;
  bool ws_used = false;
};

static hipError_t ws_acquire(mi_clip* c, hipStream_t s) {
  if (c->ws_used && c->ws_stream != s) return hipStreamWaitEvent(s, c->ws_evt, 0);
  return hipSuccess;
}

static hipError_t ws_release(mi_clip* c, hipStream_t s) {
  if (!c->ws_evt) {
    hipError_t e = hipEventCreateWithFlags(&c->ws_evt, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  c->ws_stream = s;
  c->ws_used = true;
  return hipEventRecord(c->ws_evt, s);
}

static int f32_gemm_mode();

extern "C" {

int mi_abi_version(void) { return MICLIP_ABI_VERSION; }
const char* mi_build_id(void) { return MICLIP_SRC_HASH; }
const char* mi_build_sources(void) { return MICLIP_SRC_FILES; }

const char* mi_last_error(void) { return g_err.c_str(); }

int64_t mi_clip_weights_numel(const mi_clip_arch* a) {
  if (!a) return -1;
  // sizes the blob's tensors from the arch: no field may be negative or divide by zero
  if (a->embed_dim < 1 || a->image_resolution < 1 || a->vision_layers < 0 || a->vision_width < 1 ||
      a->vision_patch_size < 1 || a->image_resolution % a->vision_patch_size || a->context_length < 1 ||
      a->vocab_size < 1 || a->text_width < 1 || a->text_heads < 1 || a->text_layers < 0)
    return -1;
  const int64_t W = a->vision_width, P = a->vision_patch_size, G = a->image_resolution / a->vision_patch_size;
  const int64_t S = G * G + 1, E = a->embed_dim, TW = a->text_width;
  int64_t n = W * 3 * P * P + W + S * W + 2 * W + tower_numel(W, a->vision_layers) + 2 * W + W * E;
  n += (int64_t)a->vocab_size * TW + (int64_t)a->context_length * TW + tower_numel(TW, a->text_layers) + 2 * TW +
       TW * E + 1;
  return n;
}

int mi_clip_create(const mi_clip_arch* arch, const float* weights, int64_t numel, int device, int weight_dtype,
                   mi_clip** out) {
  if (!arch || !weights || !out) return fail(MI_ERR_ARG, "mi_clip_create: null argument");
  *out = nullptr;
  if (weight_dtype != MI_BF16 && weight_dtype != MI_FP8 && weight_dtype != MI_F32)
    return fail(MI_ERR_UNSUPPORTED, "mi_clip_create: weight_dtype must be MI_BF16, MI_FP8 or MI_F32");
  const bool full = weight_dtype == MI_F32;
  const mi_clip_arch& a = *arch;
  if (a.vision_width % 128 || a.text_width % 128 || a.vision_width > 1024 || a.text_width > 1024)
    return fail(MI_ERR_UNSUPPORTED, "widths must be multiples of 128 and <= 1024 (got %d/%d)", a.vision_width,
                a.text_width);
  if (a.embed_dim % 128) return fail(MI_ERR_UNSUPPORTED, "embed_dim must be a multiple of 128");
  if (weight_dtype == MI_FP8 && a.vision_width % 256)
    return fail(MI_ERR_UNSUPPORTED, "MI_FP8 needs vision_width %% 256 == 0 (MX GEMM N tiles), got %d", a.vision_width);
  if (a.image_resolution % a.vision_patch_size) return fail(MI_ERR_ARG, "resolution not divisible by patch");
  if (a.text_heads * 64 != a.text_width) return fail(MI_ERR_UNSUPPORTED, "text head dim must be 64");
  const int G = a.image_resolution / a.vision_patch_size;
  if (G * G + 1 > 640 || a.context_length > 640)
    return fail(MI_ERR_UNSUPPORTED, "sequences longer than 640 tokens are not supported");
  const int64_t expect = mi_clip_weights_numel(arch);
  if (numel != expect) return fail(MI_ERR_ARG, "weight blob has %lld elements, expected %lld", (long long)numel,
                                   (long long)expect);
  HIP_TRY(hipSetDevice(device));

  auto* c = new mi_clip();
  c->a = a;
  c->device = device;
  c->G = G;
  c->S_v = G * G + 1;
  const int W = a.vision_width, TW = a.text_width, E = a.embed_dim;
  const int K = 3 * a.vision_patch_size * a.vision_patch_size;
  c->Kp = (K + 63) / 64 * 64;
  c->Kp32 = (K + 31) / 32 * 32;
  c->f32 = full;

  Builder b;
  b.src = weights;
  b.numel = numel;
  b.img.reserve((size_t)numel * (full ? 4 : 2) + (size_t)a.vocab_size * TW * 2 + (1 << 20));
  const size_t o_conv = b.mat(full, W, K, full ? c->Kp32 : c->Kp);
  const size_t o_cls = b.f32(W);
  const size_t o_vpos = b.f32((int64_t)c->S_v * W);
  const size_t o_lnpre_g = b.f32(W), o_lnpre_b = b.f32(W);
  std::vector<LayerOff> vlo, tlo;
  build_tower(b, W, a.vision_layers, vlo, full);
  const size_t o_lnpost_g = b.f32(W), o_lnpost_b = b.f32(W);
  const size_t o_vproj = b.mat_t(full, W, E);
  const size_t o_tok = b.f32((int64_t)a.vocab_size * TW);
  const size_t o_tpos = b.f32((int64_t)a.context_length * TW);
  build_tower(b, TW, a.text_layers, tlo, full);
  const size_t o_lnf_g = b.f32(TW), o_lnf_b = b.f32(TW);
  const size_t o_tproj = b.mat_t(full, TW, E);
  const float* ls = b.take(1);
  if (!b.ok || b.pos != numel || !ls) {
    delete c;
    return fail(MI_ERR_ARG, "weight blob layout mismatch (consumed %lld of %lld)", (long long)b.pos,
                (long long)numel);
  }
  // bf16 vision tower: the LayerNorm-folded GEMM weights (run_tower_fold); W % 256 == 0 so
  // that all four GEMMs take the 8-phase kernel
  // (all layers or none: a product W * gamma outside fp16's range, or a non-finite column sum,
  // keeps the whole tower unfolded, run_tower)
  if (weight_dtype == MI_BF16 && W % 256 == 0) {
    const size_t img0 = b.img.size();
    bool ok = true;
    for (LayerOff& l : vlo) {
      ok = fold_ln(b, l.p_ln1_g, l.p_ln1_b, l.p_w_qkv, l.p_b_qkv, 3 * W, W, l.lw_qkv, l.ls_qkv, l.lc_qkv) && ok;
      ok = fold_ln(b, l.p_ln2_g, l.p_ln2_b, l.p_w_fc, l.p_b_fc, 4 * W, W, l.lw_fc, l.ls_fc, l.lc_fc) && ok;
    }
    if (!ok) {
      for (LayerOff& l : vlo) l.lw_qkv = l.ls_qkv = l.lc_qkv = l.lw_fc = l.ls_fc = l.lc_fc = 0;
      b.img.resize(img0);
    }
  }
  hipError_t e = hipMalloc(&c->wdev, b.img.size());
  if (e == hipSuccess) e = hipMemcpy(c->wdev, b.img.data(), b.img.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (c->wdev) (void)hipFree(c->wdev);
    delete c;
    return fail(MI_ERR_HIP, "weight upload: %s", hipGetErrorString(e));
  }
  char* d = c->wdev;
  auto F = [&](size_t o) { return (const float*)(d + o); };
  auto H = [&](size_t o) { return (const uint16_t*)(d + o); };
  c->conv_w = full ? nullptr : H(o_conv);
  c->conv_f = full ? F(o_conv) : nullptr;
  c->cls = F(o_cls);
  c->vpos = F(o_vpos);
  c->ln_pre_g = F(o_lnpre_g);
  c->ln_pre_b = F(o_lnpre_b);
  c->ln_post_g = F(o_lnpost_g);
  c->ln_post_b = F(o_lnpost_b);
  c->vproj_t = full ? nullptr : H(o_vproj);
  c->vproj_f = full ? F(o_vproj) : nullptr;
  c->tok_emb = F(o_tok);
  c->tpos = F(o_tpos);
  c->lnf_g = F(o_lnf_g);
  c->lnf_b = F(o_lnf_b);
  c->tproj_t = full ? nullptr : H(o_tproj);
  c->tproj_f = full ? F(o_tproj) : nullptr;
  auto conv_layers = [&](const std::vector<LayerOff>& lo, std::vector<Layer>& L) {
    L.resize(lo.size());
    for (size_t i = 0; i < lo.size(); ++i) {
      const LayerOff& o = lo[i];
      if (full) {
        L[i] = Layer{F(o.ln1_g), F(o.ln1_b), F(o.b_qkv), F(o.b_out), F(o.ln2_g), F(o.ln2_b), F(o.b_fc), F(o.b_proj),
                     nullptr, nullptr, nullptr, nullptr};
        L[i].f_qkv = F(o.w_qkv);
        L[i].f_out = F(o.w_out);
        L[i].f_fc = F(o.w_fc);
        L[i].f_proj = F(o.w_proj);
        {   // EPI_SPLIT_GELU's bound constants, from the host blob (rounded up to stay bounds)
          const int64_t Wd = (int64_t)(&lo == &vlo ? a.vision_width : a.text_width);
          const float* wfc = b.src + o.p_w_fc;
          const float* bfc = b.src + o.p_b_fc;
          double bw = 0, bb = 0;
          for (int64_t n = 0; n < 4 * Wd; ++n) {
            double r = 0;
            for (int64_t k = 0; k < Wd; ++k) r += std::fabs((double)wfc[n * Wd + k]);
            bw = r > bw ? r : bw;
            bb = std::fabs((double)bfc[n]) > bb ? std::fabs((double)bfc[n]) : bb;
          }
          L[i].fc_bw = (float)(bw * (1.0 + 1e-6));
          L[i].fc_bb = (float)(bb * (1.0 + 1e-6));
          const float* wq = b.src + o.p_w_qkv;
          const float* bq = b.src + o.p_b_qkv;
          bw = bb = 0;
          for (int64_t n = 2 * Wd; n < 3 * Wd; ++n) {
            double r = 0;
            for (int64_t k = 0; k < Wd; ++k) r += std::fabs((double)wq[n * Wd + k]);
            bw = r > bw ? r : bw;
            bb = std::fabs((double)bq[n]) > bb ? std::fabs((double)bq[n]) : bb;
          }
          L[i].v_bw = (float)(bw * (1.0 + 1e-6));
          L[i].v_bb = (float)(bb * (1.0 + 1e-6));
        }
      } else {
        L[i] = Layer{F(o.ln1_g), F(o.ln1_b), F(o.b_qkv), F(o.b_out), F(o.ln2_g), F(o.ln2_b), F(o.b_fc), F(o.b_proj),
                     H(o.w_qkv), H(o.w_out), H(o.w_fc), H(o.w_proj)};
        if (o.lw_qkv) {
          L[i].lw_qkv = H(o.lw_qkv);
          L[i].ls_qkv = F(o.ls_qkv);
          L[i].lc_qkv = F(o.lc_qkv);
          L[i].lw_fc = H(o.lw_fc);
          L[i].ls_fc = F(o.ls_fc);
          L[i].lc_fc = F(o.lc_fc);
        }
      }
    }
  };
  conv_layers(vlo, c->vl);
  conv_layers(tlo, c->tl);
  if (full) {
    // the GEMM operands of the fp32 tower (run_tower_f32): split-f16 copies of every tower GEMM
    // weight and of conv1 ([N][3K] fp16 + column scales, 72 W^2 bytes per layer; the default), or
    // split-bf16 copies ([N][6K] bf16, 144 W^2; A/B, MICLIP_F32_SPLIT=6).  They need N % 128 == 0
    // and K' % 32 == 0 (gemm_bf16), true for W % 128 == 0.  When the copies cannot be built the
    // exact-f32 GEMM runs instead (it needs none of them).
    const int64_t Wv = a.vision_width, Wt = a.text_width;
    const int mode = f32_gemm_mode();
    hipError_t e3 = hipSuccess;
    if (mode == 3) {
      const int64_t Kc = c->Kp32;
      size_t bytes = (size_t)(Wv * 3 * Kc * 2 + Wv * 4 + 512);
      for (int t = 0; t < 2; ++t) {
        const int64_t W = t ? Wt : Wv;
        bytes += (size_t)(t ? c->tl.size() : c->vl.size()) * (size_t)(72 * W * W + 36 * W + 8 * 256);
      }
      e3 = hipMalloc(&c->w3, bytes);
      char* p3 = c->w3;
      auto split = [&](const float* w, int64_t N, int64_t K, const uint16_t** o, const float** cs) {
        uint16_t* ow = (uint16_t*)p3;
        p3 += ((size_t)N * 3 * K * 2 + 255) & ~(size_t)255;
        float* oc = (float*)p3;
        p3 += ((size_t)N * 4 + 255) & ~(size_t)255;
        if (e3 == hipSuccess) e3 = split2h_rows(w, K, N, (int)K, 1, 0, ow, oc, nullptr);
        *o = ow;
        *cs = oc;
      };
      if (e3 == hipSuccess) {
        split(c->conv_f, Wv, Kc, &c->conv_h3, &c->conv_c3);
        for (int t = 0; t < 2; ++t) {
          const int64_t W = t ? Wt : Wv;
          for (Layer& L : t ? c->tl : c->vl) {
            split(L.f_qkv, 3 * W, W, &L.h3_qkv, &L.c3_qkv);
            split(L.f_out, W, W, &L.h3_out, &L.c3_out);
            split(L.f_fc, 4 * W, W, &L.h3_fc, &L.c3_fc);
            split(L.f_proj, W, 4 * W, &L.h3_proj, &L.c3_proj);
          }
        }
      }
      if (e3 == hipSuccess) e3 = hipDeviceSynchronize();
    } else if (mode == 6) {
      const size_t bytes = (size_t)(144 * Wv * Wv * (int64_t)c->vl.size() + 144 * Wt * Wt * (int64_t)c->tl.size());
      e3 = hipMalloc(&c->w6, bytes);
      char* p6 = c->w6;
      auto split = [&](const float* w, int64_t N, int64_t K) -> const uint16_t* {
        uint16_t* o = (uint16_t*)p6;
        p6 += (size_t)N * 6 * K * 2;
        if (e3 == hipSuccess) e3 = split6_rows(w, K, N, (int)K, 1, 0, o, nullptr);
        return o;
      };
      for (int t = 0; t < 2 && e3 == hipSuccess; ++t) {
        const int64_t W = t ? Wt : Wv;
        for (Layer& L : t ? c->tl : c->vl) {
          L.s6_qkv = split(L.f_qkv, 3 * W, W);
          L.s6_out = split(L.f_out, W, W);
          L.s6_fc = split(L.f_fc, 4 * W, W);
          L.s6_proj = split(L.f_proj, W, 4 * W);
        }
      }
      if (e3 == hipSuccess) e3 = hipDeviceSynchronize();
    }
    if (e3 != hipSuccess) {
      // no room (or no split): the exact-f32 GEMMs need none of these copies, so the context is
      // still usable
      (void)hipGetLastError();
      if (c->w6) (void)hipFree(c->w6);
      if (c->w3) (void)hipFree(c->w3);
      c->w6 = c->w3 = nullptr;
      c->conv_h3 = nullptr;
      c->conv_c3 = nullptr;
      for (int t = 0; t < 2; ++t)
        for (Layer& L : t ? c->tl : c->vl) {
          L.s6_qkv = L.s6_out = L.s6_fc = L.s6_proj = nullptr;
          L.h3_qkv = L.h3_out = L.h3_fc = L.h3_proj = nullptr;
        }
      fprintf(stderr, "miclip: split GEMM weights unavailable (%s); fp32 tower on the exact-f32 GEMM\n",
              hipGetErrorString(e3));
    }
  }
  if (weight_dtype == MI_FP8) {
    // MX-fp8 copies of the vision tower GEMM weights, quantised on the device
    // from the bf16 image (the text tower and the projections stay bf16)
    const int64_t Wv = a.vision_width;
    const int64_t per_layer = 12 * Wv * Wv + 4 * (12 * Wv * Wv / 64) + 4 * 256;
    e = hipMalloc(&c->wq, per_layer * c->vl.size() + 256);
    if (e != hipSuccess) {
      (void)hipFree(c->wdev);
      delete c;
      return fail(MI_ERR_HIP, "fp8 weight allocation: %s", hipGetErrorString(e));
    }
    size_t off = 0;
    auto carve = [&](size_t bytes) { char* p = c->wq + off; off += (bytes + 255) & ~(size_t)255; return (uint8_t*)p; };
    for (Layer& L : c->vl) {
      struct { const uint16_t* w; int64_t n, k; const uint8_t** q; const uint8_t** sc; } mats[4] = {
          {L.w_qkv, 3 * Wv, Wv, &L.q_qkv, &L.s_qkv}, {L.w_out, Wv, Wv, &L.q_out, &L.s_out},
          {L.w_fc, 4 * Wv, Wv, &L.q_fc, &L.s_fc}, {L.w_proj, Wv, 4 * Wv, &L.q_proj, &L.s_proj}};
      for (auto& m : mats) {
        uint8_t* q = carve(m.n * m.k);
        uint8_t* sc = carve((m.k / 128) * ((m.n + 1) & ~1) * 2);
        if (e == hipSuccess) e = quantize_mx(m.w, m.k, q, m.k, sc, (int)m.n, (int)m.k, nullptr);
        *m.q = q;
        *m.sc = sc;
      }
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      (void)hipFree(c->wq);
      (void)hipFree(c->wdev);
      delete c;
      return fail(MI_ERR_HIP, "fp8 weight quantisation: %s", hipGetErrorString(e));
    }
    c->fp8 = true;
  }
  *out = c;
  return MI_OK;
}

int mi_clip_destroy(mi_clip* c) {
  if (!c) return MI_OK;
  {
    std::lock_guard<std::mutex> g(c->mu);
    (void)hipSetDevice(c->device);
    if (c->ws) (void)hipFree(c->ws);
    if (c->wdev) (void)hipFree(c->wdev);
    if (c->wq) (void)hipFree(c->wq);
    if (c->w6) (void)hipFree(c->w6);
    if (c->w3) (void)hipFree(c->w3);
    if (c->ws_evt) (void)hipEventDestroy(c->ws_evt);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  }
  delete c;
  return MI_OK;
}

static int reserve_locked(mi_clip* c, int64_t ic, int64_t tc) {
  if (ic <= c->img_chunk && tc <= c->txt_chunk && c->ws) return MI_OK;
  ic = ic > c->img_chunk ? ic : c->img_chunk;
  tc = tc > c->txt_chunk ? tc : c->txt_chunk;
  const mi_clip_arch& a = c->a;
  const int64_t Mv = ic * c->S_v, Mt = tc * a.context_length;
  const int64_t Wv = a.vision_width, Wt = a.text_width;
  auto mx = [](int64_t p, int64_t q) { return p > q ? p : q; };
  const int64_t xw = mx(Mv * Wv, Mt * Wt);
  const int64_t rows_max = mx(ic, tc);
  size_t off = 0;
  auto carve = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t es = c->f32 ? 4 : 2;   // activation element size (f32 mode: every buffer f32)
  const size_t o_x = carve(xw * 4);
  const size_t o_h = carve(xw * es);
  const size_t o_qkv = carve(3 * xw * es);
  const size_t o_att = carve(xw * es);
  const size_t o_delta = c->f32 ? carve(0) : carve(xw * 2);
  const size_t o_mlp = carve(4 * xw * es);
  const size_t o_pat = carve((size_t)ic * c->G * c->G * (c->f32 ? c->Kp32 * 4 : c->Kp * 2));
  const size_t o_cls = carve((size_t)rows_max * mx(Wv, Wt) * es);
  const size_t o_y = carve((size_t)rows_max * a.embed_dim * 4);
  const size_t o_rs = carve((size_t)(Mv + 256) * 8);
  // f32 mode, split GEMM operands: the widest A operand, c_proj's [M][6 * 4W] bf16 (split-bf16)
  // or [M][3 * 4W] fp16 (split-f16), and conv1's patches [ic G^2][3 Kp32] fp16; + row scales
  const bool split_ops = c->w6 || c->w3;
  const size_t o_a6 = split_ops ? carve((size_t)mx(mx(Mv * Wv, Mt * Wt) * 24 * 2, ic * c->G * c->G * 3 * c->Kp32 * 2))
                                : carve(0);
  // row scales: the split operand's (rsc), the fused c_fc split's (rsc + rows) and the LN rows' max |h|
  const size_t o_rsc = c->w3 ? carve((size_t)mx(mx(Mv, Mt), ic * c->G * c->G) * 4 * 3) : carve(0);
  size_t o_hq = 0, o_hqs = 0, o_attq = 0, o_attqs = 0, o_mlpq = 0, o_mlpqs = 0;
  if (c->fp8) {
    const size_t mp = (size_t)((Mv + 1) & ~1);
    o_hq = carve(Mv * Wv);
    o_hqs = carve((Wv / 128) * mp * 2);
    o_attq = carve(Mv * Wv);
    o_attqs = carve((Wv / 128) * mp * 2);
    o_mlpq = carve(4 * Mv * Wv);
    o_mlpqs = carve((4 * Wv / 128) * mp * 2);
  }
  HIP_TRY(hipSetDevice(c->device));
  char* ws = nullptr;
  HIP_TRY(hipMalloc(&ws, off));
  if (c->ws) {
    (void)hipDeviceSynchronize();
    (void)hipFree(c->ws);
  }
  c->ws = ws;
  c->x = (float*)(ws + o_x);
  c->h = (uint16_t*)(ws + o_h);
  c->qkv = (uint16_t*)(ws + o_qkv);
  c->att = (uint16_t*)(ws + o_att);
  c->delta = (uint16_t*)(ws + o_delta);
  c->mlp = (uint16_t*)(ws + o_mlp);
  c->patches = (uint16_t*)(ws + o_pat);
  c->cls_ln = (uint16_t*)(ws + o_cls);
  c->y = (float*)(ws + o_y);
  c->rs = (float*)(ws + o_rs);
  c->a6 = split_ops ? (uint16_t*)(ws + o_a6) : nullptr;
  c->rsc = c->w3 ? (float*)(ws + o_rsc) : nullptr;
  c->rsc_rows = mx(mx(Mv, Mt), ic * c->G * c->G);
  if (c->fp8) {
    c->hq = (uint8_t*)(ws + o_hq);
    c->hqs = (uint8_t*)(ws + o_hqs);
    c->attq = (uint8_t*)(ws + o_attq);
    c->attqs = (uint8_t*)(ws + o_attqs);
    c->mlpq = (uint8_t*)(ws + o_mlpq);
    c->mlpqs = (uint8_t*)(ws + o_mlpqs);
  }
  c->img_chunk = ic;
  c->txt_chunk = tc;
  return MI_OK;
}

int mi_clip_reserve(mi_clip* c, int64_t image_chunk, int64_t text_chunk) {
  if (!c || image_chunk < 1 || text_chunk < 1) return fail(MI_ERR_ARG, "mi_clip_reserve: bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  return reserve_locked(c, image_chunk, text_chunk);
}

// A/B switches (MICLIP_* environment overrides of the measured defaults) are
// read only by the A/B build (scripts/ab, MICLIP_AB=1); the product library
// always runs the defaults.
static const char* ab_getenv(const char* name) {
#if MICLIP_AB
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// GEMM main-loop schedule (gemm.hip): MICLIP_GEMM_VARIANT overrides the default.
static int gemm_variant() {
  static int v = -1;
  if (v < 0) {
    const char* e = ab_getenv("MICLIP_GEMM_VARIANT");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// Per-GEMM schedule overrides for A/B runs of the whole encoder
// (MICLIP_GEMM_VARIANT_{QKV,OUT,FC,PROJ}; 0 = MICLIP_GEMM_VARIANT / default).
enum { GV_QKV = 0, GV_OUT = 1, GV_FC = 2, GV_PROJ = 3 };
static int gemm_variant_for(int which) {
  static int v[4] = {-1, -1, -1, -1};
  static const char* names[4] = {"MICLIP_GEMM_VARIANT_QKV", "MICLIP_GEMM_VARIANT_OUT", "MICLIP_GEMM_VARIANT_FC",
                                 "MICLIP_GEMM_VARIANT_PROJ"};
  if (v[which] < 0) {
    const char* e = ab_getenv(names[which]);
    v[which] = e ? atoi(e) : 0;
  }
  return v[which];
}

static GemmArgs with_variant(GemmArgs g, int which) {
  const int v = gemm_variant_for(which);
  if (v) g.variant = v;
  return g;
}

static GemmArgs gargs(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const float* bias, void* out,
                      int64_t ldo, int M, int N, int K) {
  GemmArgs g;
  g.A = A; g.lda = lda; g.W = W; g.ldw = ldw; g.bias = bias; g.out = out; g.ldo = ldo;
  g.M = M; g.N = N; g.K = K; g.group = 0; g.gstride = 0; g.goffset = 0; g.ngroup = 0; g.a_scale = nullptr; g.w_scale = nullptr; g.o_scale = nullptr;
  g.patch_R = 0;
  g.variant = gemm_variant();
  return g;
}

// Vision residual stream storage: fp16 after the first residual add (2 B
// instead of 4 per element on each of the 24 residual LayerNorms' read and
// write); MICLIP_RESID16=0 keeps it f32 (A/B, parity comparisons).
static int resid16() {
  static int v = -1;
  if (v < 0) {
    const char* e = ab_getenv("MICLIP_RESID16");
    v = e ? atoi(e) != 0 : 1;
  }
  return v;
}
// Patch embedding reads the bf16 pixels straight from the GEMM's A-operand DMA
// (B/32: one 32-pixel row segment per k stage) instead of through an im2col
// buffer; MICLIP_PATCH_FUSED=0 keeps the im2col pass (A/B).
static int patch_fused() {
  static int v = -1;
  if (v < 0) {
    const char* e = ab_getenv("MICLIP_PATCH_FUSED");
    v = e ? atoi(e) != 0 : 1;
  }
  return v;
}
// The first block's ln_1 fused into the vision embedding kernel (bf16 tower);
// MICLIP_EMBED_LN1=0 keeps the separate LayerNorm pass (A/B).
static int embed_ln1() {
  static int v = -1;
  if (v < 0) {
    const char* e = ab_getenv("MICLIP_EMBED_LN1");
    v = e ? atoi(e) != 0 : 1;
  }
  return v;
}
// xmode of a layer's first residual_ln: the f32 stream from ln_pre is converted at layer 0
static int xmode_at(int r16, size_t l) { return r16 ? (l == 0 ? 1 : 2) : 0; }

// One tower.  On return x + delta is the final residual stream (the last
// c_proj output is left in delta; the caller's final LayerNorm adds it).
// Per block (openai/CLIP ResidualAttentionBlock):
//   qkv = h W_qkv^T + b ; att = MHA(qkv) ; delta = att W_o^T + b_o
//   x += delta ; h = ln_2(x)                      (residual_ln)
//   m = QuickGELU(h W_fc^T + b_fc) ; delta = m W_pr^T + b_pr
//   x += delta ; h = ln_1'(x)  (next block)       (residual_ln)
// h_ready: the caller already wrote h = ln_1(x) of the first block (the
// vision embedding kernel fuses it).
static int run_tower(mi_clip* c, const std::vector<Layer>& layers, int B, int S, int W, int causal, hipStream_t s,
                     int r16 = 0, bool h_ready = false) {
  const int M = B * S;
  if (!h_ready) HIP_TRY(layernorm_bf16(c->x, W, layers[0].ln1_g, layers[0].ln1_b, c->h, W, M, W, s));
  for (size_t l = 0; l < layers.size(); ++l) {
    const Layer& L = layers[l];
    HIP_TRY(gemm_bf16(with_variant(gargs(c->h, W, L.w_qkv, W, L.b_qkv, c->qkv, 3 * W, M, 3 * W, W), GV_QKV), EPI_BF16,
                      s));
    HIP_TRY(attention(c->qkv, c->att, B, S, W, causal, s));
    HIP_TRY(gemm_bf16(with_variant(gargs(c->att, W, L.w_out, W, L.b_out, c->delta, W, M, W, W), GV_OUT), EPI_BF16, s));
    HIP_TRY(residual_ln(c->x, c->delta, W, 1, L.ln2_g, L.ln2_b, c->h, M, W, s, nullptr, nullptr, xmode_at(r16, l)));
    HIP_TRY(gemm_bf16(with_variant(gargs(c->h, W, L.w_fc, W, L.b_fc, c->mlp, 4 * W, M, 4 * W, W), GV_FC),
                      EPI_GELU_BF16, s));
    HIP_TRY(gemm_bf16(with_variant(gargs(c->mlp, 4 * W, L.w_proj, 4 * W, L.b_proj, c->delta, W, M, W, 4 * W), GV_PROJ),
                      EPI_BF16, s));
    if (l + 1 < layers.size())
      HIP_TRY(residual_ln(c->x, c->delta, W, 1, layers[l + 1].ln1_g, layers[l + 1].ln1_b, c->h, M, W, s, nullptr, nullptr,
                          r16 ? 2 : 0));
  }
  return MI_OK;
}

// LayerNorm folded into the in_proj / c_fc GEMMs (bf16 vision tower): the GEMMs read the fp16
// residual stream x16 directly (half-slot layout, row stride 2W elements) and apply ln_1 / ln_2
// in their epilogues from per-row (rstd, rstd * mean) (gemm_8q.hip EPI_LN_*), so the residual
// adds only write x16 and the statistics (residual_stats: 6 instead of residual_ln's 8 bytes per
// element, no h buffer).  MICLIP_LNFOLD=0 keeps run_tower (A/B).
// Default: folded for W <= 1024.  Before the residual add moved into the out_proj / c_proj
// epilogues the fold only paid for W <= 768 (B/32: 101.9k -> 103.6k frames/s; at W = 1024 the
// folded c_fc / qkv run 10 % / 5 % slower than the plain GEMMs, and residual_stats did not make that
// up: configs[2] 16.25 -> 16.32 s per step, profiles/r04_v_config2.json).  With the fused residual
// it pays at L/14 too: 6566 frames/s against 6160 unfolded and 6107 folded without the fusion
// (10k frames x 256 queries, profiles/r04_al_l14_fold.log).
static int lnfold(int W) {
  const char* e = ab_getenv("MICLIP_LNFOLD");   // read per call (A/B tests switch it within one process)
  return e ? atoi(e) != 0 : W <= 1024;
}

static GemmArgs ln_args(mi_clip* c, const uint16_t* wf, const float* sv, const float* cv, void* out, int N, int M,
                        int W) {
  GemmArgs g = gargs((const uint16_t*)c->x, 2 * W, wf, W, cv, out, N, M, N, W);
  g.variant = 0;   // the folded GEMMs have one schedule (gemm_bf16 rejects EPI_LN_* with a variant)
  g.a_f16 = 1;
  g.rs = c->rs;
  g.colv = sv;
  return g;
}

// Residual add fused into out_proj / c_proj (gemm_8q EPI_RES16_BF16): the GEMM epilogue adds its
// bf16 output into x16 in place and stores per-row partial statistics of each 64 columns; the
// tiny residual_finalize pass turns them into rs.  The GEMM reads and writes x16 (4 B per
// element) instead of writing delta and residual_stats re-reading it (8 B).  The partials live
// in the h buffer, which the folded tower does not otherwise use.  MICLIP_RESFUSE=0 keeps the
// separate residual_stats pass (A/B).
static int resfuse() {
  const char* e = ab_getenv("MICLIP_RESFUSE");   // read per call (A/B tests switch it within one process)
  return e ? atoi(e) != 0 : 1;
}

// out_proj / c_proj with the residual add fused: x16 += bf16(A W^T + b), partials into c->h
static int gemm_residual(mi_clip* c, const uint16_t* A, int64_t lda, const uint16_t* w, const float* b, int M, int W,
                         int K, hipStream_t s) {
  GemmArgs g = gargs(A, lda, w, K, b, c->x, 2 * W, M, W, K);
  g.ps = (float*)c->h;
  HIP_TRY(gemm_bf16(g, EPI_RES16_BF16, s));
  HIP_TRY(residual_finalize((const float*)c->h, c->rs, M, W, s));
  return MI_OK;
}

// The last block after its attention on the CLS rows only.  encode_image reads the tower at
// x[:, 0] alone (ln_post(x[:, 0]) @ proj, openai/CLIP VisionTransformer.forward), and every op of
// the block after attention is row-wise (out_proj, the residual add, ln_2, c_fc, c_proj), so the
// other S - 1 rows of each sequence are never read: the CLS rows of att and of the fp16 stream
// are gathered (B rows) and the rest of the block runs on them with the same kernels -- the
// values of the full pass's CLS rows bit for bit (each GEMM row's arithmetic does not depend on
// the rows beside it).  Needs the 8-phase kernel's 256 rows (B >= 256); the compact rows live in
// the qkv buffer, dead after attention.  MICLIP_CLS_LAST=0 (A/B) runs the full block.
static int cls_last() {
  const char* e = ab_getenv("MICLIP_CLS_LAST");
  return e ? atoi(e) != 0 : 1;
}

static int last_block_cls(mi_clip* c, const Layer& L, int B, int S, int W, float** xpost, hipStream_t s) {
  uint16_t* att_c = c->qkv;                                                  // [B][W] bf16
  float* x_c = (float*)((char*)c->qkv + (((size_t)B * W * 2 + 255) & ~(size_t)255));   // [B] fp16 row slots
  HIP_TRY(hipMemcpy2DAsync(att_c, (size_t)W * 2, c->att, (size_t)S * W * 2, (size_t)W * 2, B, hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemcpy2DAsync(x_c, (size_t)W * 4, c->x, (size_t)S * W * 4, (size_t)W * 2, B, hipMemcpyDeviceToDevice, s));
  GemmArgs o = gargs(att_c, W, L.w_out, W, L.b_out, x_c, 2 * W, B, W, W);
  o.ps = (float*)c->h;
  HIP_TRY(gemm_bf16(o, EPI_RES16_BF16, s));
  HIP_TRY(residual_finalize((const float*)c->h, c->rs, B, W, s));
  GemmArgs f = gargs((const uint16_t*)x_c, 2 * W, L.lw_fc, W, L.lc_fc, c->mlp, 4 * W, B, 4 * W, W);
  f.variant = 0;
  f.a_f16 = 1;
  f.rs = c->rs;
  f.colv = L.ls_fc;
  HIP_TRY(gemm_bf16(f, EPI_LN_GELU_BF16, s));
  HIP_TRY(gemm_bf16(with_variant(gargs(c->mlp, 4 * W, L.w_proj, 4 * W, L.b_proj, c->delta, W, B, W, 4 * W), GV_PROJ),
                    EPI_BF16, s));
  *xpost = x_c;
  return MI_OK;
}

// x16 / rs hold the embedding output and ln_1's statistics (vision_embed_ln16).  On return x16
// + delta is the final residual stream (the last c_proj output stays in delta, as run_tower), at
// rows r * post_stride of (*xpost, delta): the full stream's CLS rows (stride S), or the last
// block's compact CLS rows (stride 1, last_block_cls).
static int run_tower_fold(mi_clip* c, const std::vector<Layer>& layers, int B, int S, int W, hipStream_t s,
                          float** xpost, int64_t* post_stride) {
  const int M = B * S;
  const bool fuse = resfuse() && !gemm_variant_for(GV_OUT) && !gemm_variant_for(GV_PROJ) && !gemm_variant();
  *xpost = c->x;
  *post_stride = S;
  for (size_t l = 0; l < layers.size(); ++l) {
    const Layer& L = layers[l];
    const bool last = l + 1 == layers.size();
    const bool cls = last && fuse && B >= 256 && S > 1 && cls_last();
    if (cls) {
      // the last block reads attention at the CLS queries only: K and V for every row, Q for the
      // CLS rows (strided A and output rows, their LN statistics gathered); the other rows' Q
      // columns keep stale finite values, which reach only their own queries' outputs (a query's
      // scores, softmax and P V use its own Q row alone), never read
      GemmArgs kv = ln_args(c, L.lw_qkv + (size_t)W * W, L.ls_qkv + W, L.lc_qkv + W, c->qkv + W, 2 * W, M, W);
      kv.ldo = 3 * W;
      HIP_TRY(gemm_bf16(kv, EPI_LN_BF16, s));
      float* rs_c = (float*)c->h;
      HIP_TRY(hipMemcpy2DAsync(rs_c, 8, c->rs, (size_t)S * 8, 8, B, hipMemcpyDeviceToDevice, s));
      GemmArgs q = ln_args(c, L.lw_qkv, L.ls_qkv, L.lc_qkv, c->qkv, W, B, W);
      q.lda = (int64_t)S * 2 * W;
      q.ldo = (int64_t)S * 3 * W;
      q.rs = rs_c;
      HIP_TRY(gemm_bf16(q, EPI_LN_BF16, s));
    } else {
      HIP_TRY(gemm_bf16(ln_args(c, L.lw_qkv, L.ls_qkv, L.lc_qkv, c->qkv, 3 * W, M, W), EPI_LN_BF16, s));
    }
    HIP_TRY(attention(c->qkv, c->att, B, S, W, cls ? 0x800 : 0, s));   // (cls: the CLS queries' tile only)
    if (cls) {
      MI_TRY(last_block_cls(c, L, B, S, W, xpost, s));
      *post_stride = 1;
      break;
    }
    if (fuse) {
      MI_TRY(gemm_residual(c, c->att, W, L.w_out, L.b_out, M, W, W, s));
    } else {
      HIP_TRY(gemm_bf16(with_variant(gargs(c->att, W, L.w_out, W, L.b_out, c->delta, W, M, W, W), GV_OUT), EPI_BF16, s));
      HIP_TRY(residual_stats(c->x, c->delta, c->rs, M, W, s));
    }
    const bool tm = c->ev_kind == MI_KERNEL_C_FC && c->ev_n < c->ev_cap;
    if (tm) HIP_TRY(hipEventRecord(c->ev[2 * c->ev_n], s));
    HIP_TRY(gemm_bf16(ln_args(c, L.lw_fc, L.ls_fc, L.lc_fc, c->mlp, 4 * W, M, W), EPI_LN_GELU_BF16, s));
    if (tm) HIP_TRY(hipEventRecord(c->ev[2 * c->ev_n++ + 1], s));
    if (fuse && !last) {
      MI_TRY(gemm_residual(c, c->mlp, 4 * W, L.w_proj, L.b_proj, M, W, 4 * W, s));
    } else {
      HIP_TRY(gemm_bf16(with_variant(gargs(c->mlp, 4 * W, L.w_proj, 4 * W, L.b_proj, c->delta, W, M, W, 4 * W), GV_PROJ),
                        EPI_BF16, s));
      if (!last) HIP_TRY(residual_stats(c->x, c->delta, c->rs, M, W, s));
    }
  }
  return MI_OK;
}

// MX-fp8 GEMM arguments: A / W e4m3 with their stage-major scales
static GemmArgs margs(const uint8_t* A, const uint8_t* as, const uint8_t* W, const uint8_t* ws, const float* bias,
                      void* out, int64_t ldo, int M, int N, int K) {
  GemmArgs g = gargs((const uint16_t*)A, K, (const uint16_t*)W, K, bias, out, ldo, M, N, K);
  g.a_scale = as;
  g.w_scale = ws;
  return g;
}

// The vision tower with MX-fp8 GEMMs (weight_dtype MI_FP8): the same block as
// run_tower, every GEMM on the block-scaled MFMA; the producers of GEMM A
// operands (the LayerNorms, attention, c_fc's QuickGELU epilogue) emit MX-fp8
// directly, so no separate quantisation pass runs.
// xpost / post_stride: where ln_post reads the CLS rows (the last block after attention runs on
// them alone at >= 256 frames, as run_tower_fold's last_block_cls: the CLS rows of the MX-fp8
// attention output -- codes and their stage-major scales -- and of the residual stream gathered)
static int run_tower_mx(mi_clip* c, const std::vector<Layer>& layers, int B, int S, int W, hipStream_t s, int r16,
                        float** xpost, int64_t* post_stride) {
  const int M = B * S;
  *xpost = c->x;
  *post_stride = S;
  HIP_TRY(layernorm_bf16(c->x, W, layers[0].ln1_g, layers[0].ln1_b, c->h, W, M, W, s, c->hq, c->hqs));
  for (size_t l = 0; l < layers.size(); ++l) {
    const Layer& L = layers[l];
    HIP_TRY(gemm_mx(margs(c->hq, c->hqs, L.q_qkv, L.s_qkv, L.b_qkv, c->qkv, 3 * W, M, 3 * W, W), EPI_BF16, s));
    HIP_TRY(attention(c->qkv, c->att, B, S, W, 0, s, c->attq, c->attqs));
    int Mr = M;
    const uint8_t *aq = c->attq, *aqs = c->attqs;
    float* xr = c->x;
    if (l + 1 == layers.size() && B >= 256 && S > 1 && W % 128 == 0 && cls_last()) {
      uint8_t* aq_c = (uint8_t*)c->qkv;                                    // [B][W] e4m3
      uint8_t* aqs_c = aq_c + (((size_t)B * W + 255) & ~(size_t)255);       // [W / 128][Bp][2]
      float* x_c = (float*)(aqs_c + ((((size_t)W / 128) * (B + 2) * 2 + 255) & ~(size_t)255));
      const size_t mp = (size_t)((M + 1) & ~1), bp = (size_t)((B + 1) & ~1);
      HIP_TRY(hipMemcpy2DAsync(aq_c, W, c->attq, (size_t)S * W, W, B, hipMemcpyDeviceToDevice, s));
      for (int st = 0; st < W / 128; ++st)
        HIP_TRY(hipMemcpy2DAsync(aqs_c + st * bp * 2, 2, c->attqs + st * mp * 2, (size_t)S * 2, 2, B,
                                 hipMemcpyDeviceToDevice, s));
      HIP_TRY(hipMemcpy2DAsync(x_c, (size_t)W * 4, c->x, (size_t)S * W * 4, (size_t)W * 4, B, hipMemcpyDeviceToDevice, s));
      Mr = B;
      aq = aq_c;
      aqs = aqs_c;
      xr = x_c;
      *xpost = x_c;
      *post_stride = 1;
    }
    HIP_TRY(gemm_mx(margs(aq, aqs, L.q_out, L.s_out, L.b_out, c->delta, W, Mr, W, W), EPI_BF16, s));
    HIP_TRY(residual_ln(xr, c->delta, W, 1, L.ln2_g, L.ln2_b, c->h, Mr, W, s, c->hq, c->hqs, xmode_at(r16, l)));
    GemmArgs fc = margs(c->hq, c->hqs, L.q_fc, L.s_fc, L.b_fc, c->mlpq, 4 * W, Mr, 4 * W, W);
    fc.o_scale = c->mlpqs;
    HIP_TRY(gemm_mx(fc, EPI_GELU_MX, s));
    HIP_TRY(gemm_mx(margs(c->mlpq, c->mlpqs, L.q_proj, L.s_proj, L.b_proj, c->delta, W, Mr, W, 4 * W), EPI_BF16, s));
    if (l + 1 < layers.size())
      HIP_TRY(residual_ln(c->x, c->delta, W, 1, layers[l + 1].ln1_g, layers[l + 1].ln1_b, c->h, M, W, s, c->hq,
                          c->hqs, r16 ? 2 : 0));
  }
  return MI_OK;
}

static size_t dtype_size(int dt) { return dt == MI_F32 ? 4 : 2; }

// The fp32 tower's GEMMs (run_tower_f32): 3 = split-f16 operands on the f16 MFMA (the
// default since round 5, K' = 3K), 6 = split-bf16 operands (round 4, K' = 6K), 0 = the exact-f32
// MFMA GEMM (precise.hip gemm_f32).  MICLIP_F32_SPLIT selects one in the A/B build (read when a
// context is created: the weight copies are built for the mode).
static int f32_gemm_mode() {
  const char* e = ab_getenv("MICLIP_F32_SPLIT");
  if (!e) return 3;
  const int v = atoi(e);
  return v == 0 || v == 6 ? v : 3;
}

// The fp32 tower (weight_dtype MI_F32; kernels in precise.hip).  openai/CLIP
// ResidualAttentionBlock with every tensor f32, the residual adds in the
// out_proj / c_proj GEMM epilogues:
//   h = ln_1(x) ; qkv = h W_qkv^T + b ; att = MHA(qkv) ; x += att W_o^T + b_o
//   h = ln_2(x) ; m = QuickGELU(h W_fc^T + b_fc) ; x += m W_pr^T + b_pr
// xpost / post_stride (vision): where ln_post reads the CLS rows (the last block may run on them
// alone, as run_tower_fold's last_block_cls)
static int run_tower_f32(mi_clip* c, const std::vector<Layer>& layers, int B, int S, int W, int causal,
                         hipStream_t s, float** xpost = nullptr, int64_t* post_stride = nullptr) {
  const int M = B * S;
  if (xpost) {
    *xpost = c->x;
    *post_stride = S;
  }
  float* h = (float*)c->h;
  float* qkv = (float*)c->qkv;
  float* att = (float*)c->att;
  float* mlp = (float*)c->mlp;
  if (c->a6 && c->rsc && layers.size() && layers[0].h3_qkv) {
    // split-f16 GEMMs (split2h_rows): one f16 GEMM over K' = 3K per linear layer, a1 w1 + a1 w2 +
    // a2 w1 in f32 with the row / column scales in the epilogue -- f32-grade results; ln_1 / ln_2
    // write the split operand directly (layernorm_split2h), attention's and c_fc's outputs are
    // split by one pass each (c_proj's with QuickGELU applied first)
    uint16_t* a3 = c->a6;
    float* rsc = c->rsc;
    // the fused c_fc split (the default; MICLIP_F32_FUSED_SPLIT=0 in the A/B build keeps the f32
    // pre-activation + split pass): c_proj's operand [M][12W] after c_fc's [M][3W] in the workspace
    const char* fe = ab_getenv("MICLIP_F32_FUSED_SPLIT");
    const bool fuse_split = !fe || atoi(fe) != 0;
    uint16_t* a3o = a3 + (int64_t)M * 3 * W;
    float* rsc_o = rsc + c->rsc_rows;
    float* rmax = rsc + 2 * c->rsc_rows;
    int Mr = M;   // the rows the block's row-wise part runs on (B for the last block's CLS rows)
    // The activations' split operand stored once, [x1 | x2] (role 2, row stride 2K), where the
    // consumer GEMM is the 8-phase kernel (its A_DUP read gives the logical [x1 | x1 | x2]): a third
    // less written by the split passes and by c_fc's split epilogue (o_dup), bit-identical.
    // MICLIP_F32_DUP=0 (A/B) keeps the full layout everywhere.
    // (MICLIP_F32_DUP=mask in the A/B build: 1 ln_1's split, 2 attention's, 4 ln_2's, 8 c_fc's output)
    const char* de = ab_getenv("MICLIP_F32_DUP");
    const char* e8 = ab_getenv("MICLIP_F32_8Q");
    const int dmask = de ? atoi(de) : 15;
    // MICLIP_F32_ATTN_FUSED=0 (A/B): attention's f32 output and the split pass (round 5)
    const char* ae = ab_getenv("MICLIP_F32_ATTN_FUSED");
    const bool att_fused = !ae || atoi(ae) != 0;
    const bool dup_on = dmask != 0 && (!e8 || atoi(e8) != 0);
    auto sargs = [&](const uint16_t* A, int64_t lda_rows, bool dup, const uint16_t* w3, const float* c3, const float* b,
                     float* out, int64_t ldo, int rows, int N, int K) {   // lda_rows: row stride in rows of the operand
      GemmArgs g = gargs(A, lda_rows * (dup ? 2 : 3) * K, w3, 3 * K, b, out, ldo, rows, N, 3 * K);
      g.a_f16 = 1;
      g.rsc = rsc;
      g.csc = c3;
      g.a_dup = dup ? K : 0;
      return g;
    };
    auto dup_ok = [&](int rows, int N, int K, int64_t lda_rows = 1) {   // the consumer takes the 8-phase kernel
      if (!dup_on) return false;
      GemmArgs t = sargs(a3, lda_rows, true, nullptr, nullptr, nullptr, nullptr, N, rows, N, K);
      return gemm_8q_ok(t) != 0;
    };
    auto gemm3 = [&](int K, const uint16_t* w3, const float* c3, const float* b, float* out, int N, int epi,
                     bool dup) -> int {
      HIP_TRY(gemm_bf16(sargs(a3, 1, dup, w3, c3, b, out, N, Mr, N, K), epi, s));
      return MI_OK;
    };
    for (size_t li = 0; li < layers.size(); ++li) {
      const Layer& L = layers[li];
      Mr = M;
      const bool cls = xpost && li + 1 == layers.size() && !causal && B >= 256 && S > 1 && cls_last();
      // ln_1's operand feeds in_proj (every row; in the CLS-row last block K / V for every row and Q
      // for the CLS rows, read with a row stride of S)
      const bool d1 = (dmask & 1) && (cls ? dup_ok(M, 2 * W, W) && dup_ok(B, W, W, S) : dup_ok(M, 3 * W, W));
      // S <= 64: attention writes out_proj's split operand itself (attention_f32_split, its scale
      // bounded through ln_1's row max; round 6), in place of its f32 output and a split pass
      const bool fuse_att = S <= 64 && att_fused;
      HIP_TRY(layernorm_split2h(c->x, W, L.ln1_g, L.ln1_b, M, W, a3, rsc, s, fuse_att ? rmax : nullptr, d1));
      if (cls) {   // K and V for every row, Q for the CLS rows only (as run_tower_fold's last block)
        GemmArgs kv = sargs(a3, 1, d1, L.h3_qkv + (size_t)W * 3 * W, L.c3_qkv + W, L.b_qkv + W, qkv + W, 3 * W, M, 2 * W, W);
        HIP_TRY(gemm_bf16(kv, EPI_F32, s));
        float* rsc_c = (float*)c->h;
        HIP_TRY(hipMemcpy2DAsync(rsc_c, 4, rsc, (size_t)S * 4, 4, B, hipMemcpyDeviceToDevice, s));
        GemmArgs q = sargs(a3, S, d1, L.h3_qkv, L.c3_qkv, L.b_qkv, qkv, (int64_t)S * 3 * W, B, W, W);
        q.rsc = rsc_c;
        HIP_TRY(gemm_bf16(q, EPI_F32, s));
      } else {
        MI_TRY(gemm3(W, L.h3_qkv, L.c3_qkv, L.b_qkv, qkv, 3 * W, EPI_F32, d1));
      }
      float* xr = c->x;
      if (fuse_att) {
        // out_proj reads the operand in place: the CLS rows with a row stride of S in the CLS-row
        // last block (their scales gathered, as the CLS Q GEMM's above)
        const bool da = (dmask & 2) && (cls ? dup_ok(B, W, W, S) : dup_ok(M, W, W));
        HIP_TRY(attention_f32_split(qkv, rmax, L.v_bw, L.v_bb, a3, da ? 2 : 0, rsc, B, S, W,
                                    causal | (cls ? 0x800 : 0), s));
        if (cls) {
          float* x_c = qkv + (((size_t)B * W + 63) & ~(size_t)63);
          float* rsc_c = (float*)c->h;
          HIP_TRY(hipMemcpy2DAsync(x_c, (size_t)W * 4, c->x, (size_t)S * W * 4, (size_t)W * 4, B, hipMemcpyDeviceToDevice, s));
          HIP_TRY(hipMemcpy2DAsync(rsc_c, 4, rsc, (size_t)S * 4, 4, B, hipMemcpyDeviceToDevice, s));
          Mr = B;
          xr = x_c;
          *xpost = x_c;
          *post_stride = 1;
          GemmArgs g = sargs(a3, S, da, L.h3_out, L.c3_out, L.b_out, xr, W, B, W, W);
          g.rsc = rsc_c;
          HIP_TRY(gemm_bf16(g, EPI_RESID_F32, s));
        } else {
          MI_TRY(gemm3(W, L.h3_out, L.c3_out, L.b_out, xr, W, EPI_RESID_F32, da));
        }
      } else {
      HIP_TRY(attention_f32(qkv, att, B, S, W, causal | (cls ? 0x800 : 0), s));   // (cls: the CLS queries' block)
      const float* ar = att;
      if (cls) {
        // the last block after attention on the CLS rows only (see last_block_cls), gathered into
        // the qkv buffer (dead after attention)
        float* att_c = qkv;
        float* x_c = qkv + (((size_t)B * W + 63) & ~(size_t)63);
        HIP_TRY(hipMemcpy2DAsync(att_c, (size_t)W * 4, att, (size_t)S * W * 4, (size_t)W * 4, B, hipMemcpyDeviceToDevice, s));
        HIP_TRY(hipMemcpy2DAsync(x_c, (size_t)W * 4, c->x, (size_t)S * W * 4, (size_t)W * 4, B, hipMemcpyDeviceToDevice, s));
        Mr = B;
        xr = x_c;
        ar = att_c;
        *xpost = x_c;
        *post_stride = 1;
      }
      const bool da = (dmask & 2) && dup_ok(Mr, W, W);          // attention's split -> out_proj
      HIP_TRY(split2h_rows(ar, W, Mr, W, da ? 2 : 0, 0, a3, rsc, s));
      MI_TRY(gemm3(W, L.h3_out, L.c3_out, L.b_out, xr, W, EPI_RESID_F32, da));
      }
      const bool df = (dmask & 4) && dup_ok(Mr, 4 * W, W);      // ln_2's split -> c_fc
      const bool dp = (dmask & 8) && dup_ok(Mr, W, 4 * W);      // c_fc's output split -> c_proj
      if (fuse_split) {   // c_fc's epilogue writes c_proj's split operand (EPI_SPLIT_GELU)
        HIP_TRY(layernorm_split2h(xr, W, L.ln2_g, L.ln2_b, Mr, W, a3, rsc, s, rmax, df));
        GemmArgs g = sargs(a3, 1, df, L.h3_fc, L.c3_fc, L.b_fc, nullptr, 0, Mr, 4 * W, W);
        g.out = a3o;
        g.ldo = (dp ? 2 : 3) * 4 * W;
        g.o_dup = dp ? 1 : 0;
        g.rmax = rmax;
        g.bnd_w = L.fc_bw;
        g.bnd_b = L.fc_bb;
        g.rsc_out = rsc_o;
        HIP_TRY(gemm_bf16(g, EPI_SPLIT_GELU, s));
        GemmArgs p = sargs(a3o, 1, dp, L.h3_proj, L.c3_proj, L.b_proj, xr, W, Mr, W, 4 * W);
        p.rsc = rsc_o;
        HIP_TRY(gemm_bf16(p, EPI_RESID_F32, s));
        continue;
      }
      HIP_TRY(layernorm_split2h(xr, W, L.ln2_g, L.ln2_b, Mr, W, a3, rsc, s, nullptr, df));
      MI_TRY(gemm3(W, L.h3_fc, L.c3_fc, L.b_fc, mlp, 4 * W, EPI_F32, df));   // pre-activation
      HIP_TRY(split2h_rows(mlp, 4 * W, Mr, 4 * W, dp ? 2 : 0, 1, a3, rsc, s));   // QuickGELU, then split
      MI_TRY(gemm3(4 * W, L.h3_proj, L.c3_proj, L.b_proj, xr, W, EPI_RESID_F32, dp));
    }
    return MI_OK;
  }
  if (c->a6 && layers.size() && layers[0].s6_qkv) {
    // split-bf16 GEMMs (split6_rows): one bf16 GEMM over K' = 6K per linear layer, every product
    // term to 2^-16 relative, f32 accumulation -- f32-grade results at bf16 MFMA rates
    uint16_t* a6 = c->a6;
    auto lin = [&](const float* in, int K, const uint16_t* w6, const float* b, float* out, int N, int epi,
                   int gelu) -> int {
      HIP_TRY(split6_rows(in, K, M, K, 0, gelu, a6, s));
      HIP_TRY(gemm_bf16(gargs(a6, 6 * K, w6, 6 * K, b, out, N, M, N, 6 * K), epi, s));
      return MI_OK;
    };
    for (const Layer& L : layers) {
      HIP_TRY(layernorm_f32(c->x, W, L.ln1_g, L.ln1_b, h, W, M, W, s));
      MI_TRY(lin(h, W, L.s6_qkv, L.b_qkv, qkv, 3 * W, EPI_F32, 0));
      HIP_TRY(attention_f32(qkv, att, B, S, W, causal, s));
      MI_TRY(lin(att, W, L.s6_out, L.b_out, c->x, W, EPI_RESID_F32, 0));
      HIP_TRY(layernorm_f32(c->x, W, L.ln2_g, L.ln2_b, h, W, M, W, s));
      MI_TRY(lin(h, W, L.s6_fc, L.b_fc, mlp, 4 * W, EPI_F32, 0));   // pre-activation: the split applies QuickGELU
      MI_TRY(lin(mlp, 4 * W, L.s6_proj, L.b_proj, c->x, W, EPI_RESID_F32, 1));
    }
    return MI_OK;
  }
  for (const Layer& L : layers) {
    HIP_TRY(layernorm_f32(c->x, W, L.ln1_g, L.ln1_b, h, W, M, W, s));
    HIP_TRY(gemm_f32(h, W, L.f_qkv, W, L.b_qkv, qkv, 3 * W, M, 3 * W, W, EPI_F32, s));
    HIP_TRY(attention_f32(qkv, att, B, S, W, causal, s));
    HIP_TRY(gemm_f32(att, W, L.f_out, W, L.b_out, c->x, W, M, W, W, EPI_RESID_F32, s));
    HIP_TRY(layernorm_f32(c->x, W, L.ln2_g, L.ln2_b, h, W, M, W, s));
    HIP_TRY(gemm_f32(h, W, L.f_fc, W, L.b_fc, mlp, 4 * W, M, 4 * W, W, EPI_GELU_BF16, s));
    HIP_TRY(gemm_f32(mlp, 4 * W, L.f_proj, 4 * W, L.b_proj, c->x, W, M, W, 4 * W, EPI_RESID_F32, s));
  }
  return MI_OK;
}

static int encode_image_f32(mi_clip* c, const char* px, int nb, int in_dtype, char* out, int out_dtype,
                            int l2_normalize, hipStream_t s) {
  const mi_clip_arch& a = c->a;
  const int W = a.vision_width, E = a.embed_dim, S = c->S_v, R = a.image_resolution, P = a.vision_patch_size;
  const int G2 = c->G * c->G;
  float* patches = (float*)c->patches;
  // conv1 as a split-f16 GEMM (rows remapped past CLS); its operand straight from the pixels where
  // the patch rows are float4-aligned (P % 4 == 0: B/32, B/16; MICLIP_IM2COL_SPLIT=0 in the A/B
  // build keeps im2col_f32 + split2h_rows)
  const char* fe = ab_getenv("MICLIP_IM2COL_SPLIT");
  const bool fused = (!fe || atoi(fe) != 0) && P % 4 == 0 && R % 4 == 0 && c->Kp32 == 3 * P * P && c->Kp32 <= 4096 &&
                     ((uintptr_t)px & 15) == 0;
  const bool split3 = c->conv_h3 && c->a6 && c->rsc;
  if (!(split3 && fused)) HIP_TRY(im2col_f32(px, in_dtype == MI_BF16, patches, nb, R, P, c->Kp32, s));
  if (split3) {
    const int K = c->Kp32;
    if (fused) HIP_TRY(im2col_split2h(px, in_dtype == MI_BF16, nb, R, P, K, c->a6, c->rsc, s));
    else HIP_TRY(split2h_rows(patches, K, (int64_t)nb * G2, K, 0, 0, c->a6, c->rsc, s));
    GemmArgs g = gargs(c->a6, 3 * K, c->conv_h3, 3 * K, nullptr, c->x, W, nb * G2, W, 3 * K);
    g.a_f16 = 1;
    g.rsc = c->rsc;
    g.csc = c->conv_c3;
    g.group = G2;
    g.gstride = S;
    g.goffset = 1;
    HIP_TRY(gemm_bf16(g, EPI_F32, s));
  } else {
    HIP_TRY(gemm_f32(patches, c->Kp32, c->conv_f, c->Kp32, nullptr, c->x, W, nb * G2, W, c->Kp32, EPI_F32, s, G2, S,
                     1));
  }
  HIP_TRY(vision_embed_ln(c->x, c->cls, c->vpos, c->ln_pre_g, c->ln_pre_b, nb, S, W, s));
  float* xpost = c->x;
  int64_t post_stride = S;
  int r = run_tower_f32(c, c->vl, nb, S, W, 0, s, &xpost, &post_stride);
  if (r) return r;
  float* cls = (float*)c->cls_ln;
  HIP_TRY(layernorm_f32(xpost, post_stride * W, c->ln_post_g, c->ln_post_b, cls, W, nb, W, s));
  HIP_TRY(gemm_f32(cls, W, c->vproj_f, W, nullptr, c->y, E, nb, E, W, EPI_F32, s));
  HIP_TRY(finalize_rows(c->y, out, out_dtype, nb, E, l2_normalize, s));
  return MI_OK;
}

static int encode_text_f32(mi_clip* c, const int32_t* tk, int nq, char* out, int out_dtype, int l2_normalize,
                           hipStream_t s) {
  const mi_clip_arch& a = c->a;
  const int W = a.text_width, E = a.embed_dim, S = a.context_length;
  HIP_TRY(text_embed(tk, c->tok_emb, c->tpos, c->x, nq, S, W, a.vocab_size, s));
  int r = run_tower_f32(c, c->tl, nq, S, W, 1, s);
  if (r) return r;
  float* cls = (float*)c->cls_ln;
  HIP_TRY(layernorm_f32(c->x, W, c->lnf_g, c->lnf_b, cls, W, nq, W, s, tk, S));
  HIP_TRY(gemm_f32(cls, W, c->tproj_f, W, nullptr, c->y, E, nq, E, W, EPI_F32, s));
  HIP_TRY(finalize_rows(c->y, out, out_dtype, nq, E, l2_normalize, s));
  return MI_OK;
}

int mi_clip_encode_image(mi_clip* c, const void* pixels, int64_t B, int in_dtype, void* out, int out_dtype,
                         int l2_normalize, void* stream) {
  if (!c || (!pixels && B > 0) || (!out && B > 0) || B < 0) return fail(MI_ERR_ARG, "encode_image: bad arguments");
  if (in_dtype != MI_F32 && in_dtype != MI_BF16) return fail(MI_ERR_ARG, "encode_image: in_dtype must be f32/bf16");
  if (out_dtype < MI_F32 || out_dtype > MI_F16) return fail(MI_ERR_ARG, "encode_image: bad out_dtype");
  if (l2_normalize < 0 || l2_normalize > 2) return fail(MI_ERR_ARG, "encode_image: l2_normalize must be 0, 1 or 2");
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->ws) {
    int r = reserve_locked(c, 256, 64);
    if (r) return r;
  }
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(ws_acquire(c, s));
  const mi_clip_arch& a = c->a;
  const int W = a.vision_width, E = a.embed_dim, S = c->S_v, R = a.image_resolution, P = a.vision_patch_size;
  const int G2 = c->G * c->G;
  const size_t in_img = (size_t)3 * R * R * dtype_size(in_dtype);
  for (int64_t c0 = 0; c0 < B; c0 += c->img_chunk) {
    const int nb = (int)((B - c0) < c->img_chunk ? (B - c0) : c->img_chunk);
    const char* px = (const char*)pixels + c0 * in_img;
    if (c->f32) {
      int r = encode_image_f32(c, px, nb, in_dtype, (char*)out + c0 * E * dtype_size(out_dtype), out_dtype,
                               l2_normalize, s);
      if (r) return r;
      continue;
    }
    const bool fused = patch_fused() && in_dtype == MI_BF16 && P == 32 && c->Kp == 3 * P * P && R % 8 == 0 &&
                       ((uintptr_t)px & 15) == 0 && (int64_t)nb * G2 >= 1024;
    GemmArgs pg;
    if (fused) {
      pg = gargs((const uint16_t*)px, 0, c->conv_w, c->Kp, nullptr, c->x, W, nb * G2, W, c->Kp);
      pg.patch_R = R;
    } else {
      HIP_TRY(im2col(px, in_dtype == MI_BF16, c->patches, nb, R, P, c->Kp, s));
      pg = gargs(c->patches, c->Kp, c->conv_w, c->Kp, nullptr, c->x, W, nb * G2, W, c->Kp);
    }
    pg.group = G2;
    pg.gstride = S;
    pg.goffset = 1;
    HIP_TRY(gemm_bf16(pg, EPI_F32, s));
    // LayerNorm-folded tower: bf16 weights folded at create (W % 256 == 0), whole 256-row tiles
    const bool fold = !c->fp8 && !c->vl.empty() && c->vl[0].lw_qkv && lnfold(W) && (int64_t)nb * S >= 256;
    int r;
    float* xpost = c->x;
    int64_t post_stride = S;
    if (fold) {
      HIP_TRY(vision_embed_ln16(c->x, c->cls, c->vpos, c->ln_pre_g, c->ln_pre_b, nb, S, W, c->rs, s));
      r = run_tower_fold(c, c->vl, nb, S, W, s, &xpost, &post_stride);
    } else {
      const bool fuse_ln1 = !c->fp8 && !c->vl.empty() && embed_ln1();  // the MX tower's first LN writes fp8 itself
      HIP_TRY(vision_embed_ln(c->x, c->cls, c->vpos, c->ln_pre_g, c->ln_pre_b, nb, S, W, s,
                              fuse_ln1 ? c->vl[0].ln1_g : nullptr, fuse_ln1 ? c->vl[0].ln1_b : nullptr,
                              fuse_ln1 ? c->h : nullptr));
      r = c->fp8 ? run_tower_mx(c, c->vl, nb, S, W, s, resid16() && !c->vl.empty(), &xpost, &post_stride)
                 : run_tower(c, c->vl, nb, S, W, 0, s, resid16() && !c->vl.empty(), fuse_ln1);
    }
    if (r) return r;
    const int r16 = fold || (resid16() && !c->vl.empty());
    // ln_post(x[:, 0] + last c_proj delta) over the CLS rows only
    HIP_TRY(residual_ln(xpost, c->delta, post_stride * W, 0, c->ln_post_g, c->ln_post_b, c->cls_ln, nb, W, s, nullptr,
                        nullptr, r16 ? 2 : 0));
    HIP_TRY(gemm_bf16(gargs(c->cls_ln, W, c->vproj_t, W, nullptr, c->y, E, nb, E, W), EPI_F32, s));
    HIP_TRY(finalize_rows(c->y, (char*)out + c0 * E * dtype_size(out_dtype), out_dtype, nb, E, l2_normalize, s));
  }
  HIP_TRY(ws_release(c, s));
  return MI_OK;
}

int mi_clip_encode_text(mi_clip* c, const int32_t* tokens, int64_t Q, void* out, int out_dtype, int l2_normalize,
                        void* stream) {
  if (!c || (!tokens && Q > 0) || (!out && Q > 0) || Q < 0) return fail(MI_ERR_ARG, "encode_text: bad arguments");
  if (out_dtype < MI_F32 || out_dtype > MI_F16) return fail(MI_ERR_ARG, "encode_text: bad out_dtype");
  if (l2_normalize < 0 || l2_normalize > 2) return fail(MI_ERR_ARG, "encode_text: l2_normalize must be 0, 1 or 2");
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->ws) {
    int r = reserve_locked(c, 256, 64);
    if (r) return r;
  }
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(ws_acquire(c, s));
  const mi_clip_arch& a = c->a;
  const int W = a.text_width, E = a.embed_dim, S = a.context_length;
  for (int64_t c0 = 0; c0 < Q; c0 += c->txt_chunk) {
    const int nq = (int)((Q - c0) < c->txt_chunk ? (Q - c0) : c->txt_chunk);
    const int32_t* tk = tokens + c0 * S;
    if (c->f32) {
      int r = encode_text_f32(c, tk, nq, (char*)out + c0 * E * dtype_size(out_dtype), out_dtype, l2_normalize, s);
      if (r) return r;
      continue;
    }
    HIP_TRY(text_embed(tk, c->tok_emb, c->tpos, c->x, nq, S, W, a.vocab_size, s));
    int r = run_tower(c, c->tl, nq, S, W, 1, s);
    if (r) return r;
    HIP_TRY(eot_gather_ln(tk, c->x, c->delta, c->lnf_g, c->lnf_b, c->cls_ln, nq, S, W, s));
    HIP_TRY(gemm_bf16(gargs(c->cls_ln, W, c->tproj_t, W, nullptr, c->y, E, nq, E, W), EPI_F32, s));
    HIP_TRY(finalize_rows(c->y, (char*)out + c0 * E * dtype_size(out_dtype), out_dtype, nq, E, l2_normalize, s));
  }
  HIP_TRY(ws_release(c, s));
  return MI_OK;
}

size_t mi_rank_workspace_bytes(int64_t N, int64_t Q, int32_t k) {
  if (N < 0 || Q < 0 || k < 1) return 0;
  return rank_workspace_bytes(N, Q, k);
}

static int check_rank_args(int64_t N, int64_t D, int dt, int64_t Q, int32_t k, int norm_mode, int nan_policy) {
  if (N < 0 || Q < 0) return fail(MI_ERR_ARG, "negative size");
  if (k < 1 || k > RANK_MAX_K) return fail(MI_ERR_UNSUPPORTED, "k must be in [1, %d] (got %d)", RANK_MAX_K, k);
  if (D < 32 || D % 32 || D > RANK_MAX_D)
    return fail(MI_ERR_UNSUPPORTED, "D must be a multiple of 32 in [32, %d] (queries are staged in LDS)", RANK_MAX_D);
  if (dt != MI_F32 && dt != MI_BF16 && dt != MI_F16) return fail(MI_ERR_ARG, "bad corpus dtype");
  if (norm_mode < 0 || norm_mode > 2) return fail(MI_ERR_ARG, "bad norm_mode");
  if (nan_policy != MI_NAN_FIRST && nan_policy != MI_NAN_LAST) return fail(MI_ERR_ARG, "bad nan_policy");
  if (N >= (int64_t)1 << 31) return fail(MI_ERR_UNSUPPORTED, "N >= 2^31 per call: shard the corpus");
  return MI_OK;
}

int mi_rank_topk(const void* corpus, int64_t N, int64_t D, int corpus_dtype, const float* queries, int64_t Q,
                 int32_t k, int64_t index_base, int norm_mode, int nan_policy, float* out_scores, int64_t* out_index,
                 void* workspace, size_t workspace_bytes, void* stream) {
  int r = check_rank_args(N, D, corpus_dtype, Q, k, norm_mode, nan_policy);
  if (r) return r;
  if (Q == 0) return MI_OK;
  if (!queries || !out_scores || !out_index || (N > 0 && !corpus))
    return fail(MI_ERR_ARG, "mi_rank_topk: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nf = nan_policy == MI_NAN_FIRST;
  if (N == 0) {
    HIP_TRY(rank_fill_empty(Q, k, out_scores, out_index, s));
    return MI_OK;
  }
  const size_t need = rank_workspace_bytes(N, Q, k);
  if (!workspace || workspace_bytes < need)
    return fail(MI_ERR_ARG, "mi_rank_topk: workspace too small (%zu < %zu)", workspace_bytes, need);
  HIP_TRY(rank_topk(corpus, N, D, corpus_dtype, queries, Q, k, index_base, norm_mode, nf, out_scores, out_index,
                    workspace, s));
  return MI_OK;
}

int mi_mirror_build(const void* corpus, int64_t N, int64_t D, int corpus_dtype, void* mirror, void* stream) {
  int r = check_rank_args(N, D, corpus_dtype, 1, 1, MI_NORM_L2, MI_NAN_FIRST);
  if (r) return r;
  if (!rank_mirror_supported(D)) return fail(MI_ERR_UNSUPPORTED, "mi_mirror_build: D must be 512 or 768 (got %lld)", (long long)D);
  if (N == 0) return MI_OK;
  if (!corpus || !mirror) return fail(MI_ERR_ARG, "mi_mirror_build: null pointer");
  HIP_TRY(mirror_build(corpus, N, D, corpus_dtype, (uint16_t*)mirror, (hipStream_t)stream));
  return MI_OK;
}

int mi_normalize_rows_f16(const void* rows, int64_t N, int64_t D, void* out, void* stream) {
  if (N < 0) return fail(MI_ERR_ARG, "negative size");
  if (D < 1 || D > 1024) return fail(MI_ERR_UNSUPPORTED, "mi_normalize_rows_f16: D must be in [1, 1024] (got %lld)", (long long)D);
  if (N == 0) return MI_OK;
  if (!rows || !out) return fail(MI_ERR_ARG, "mi_normalize_rows_f16: null pointer");
  if (N > ((int64_t)1 << 40)) return fail(MI_ERR_UNSUPPORTED, "mi_normalize_rows_f16: N too large");
  HIP_TRY(normalize_rows_f16((const uint16_t*)rows, N, (int)D, (uint16_t*)out, (hipStream_t)stream));
  return MI_OK;
}

size_t mi_rank_mirror_workspace_bytes(int64_t N, int64_t Q) {
  if (N < 0 || Q < 0) return 0;
  return rank_mirror_workspace_bytes(N, Q);
}

int mi_rank_mirror(const void* mirror, const void* master, int64_t N, int64_t D, int master_dtype,
                   const float* queries, int64_t Q, int32_t k, int64_t index_base, int nan_policy, float* out_scores,
                   int64_t* out_index, int32_t* out_certified, void* workspace, size_t workspace_bytes,
                   void* stream) {
  int r = check_rank_args(N, D, master_dtype, Q, k, MI_NORM_L2, nan_policy);
  if (r) return r;
  if (!rank_mirror_supported(D)) return fail(MI_ERR_UNSUPPORTED, "mi_rank_mirror: D must be 512 or 768 (got %lld)", (long long)D);
  if (k > MIRROR_MAX_K) return fail(MI_ERR_UNSUPPORTED, "mi_rank_mirror: k must be in [1, %d] (got %d)", MIRROR_MAX_K, k);
  if (Q == 0) return MI_OK;
  if (N == 0) return fail(MI_ERR_ARG, "mi_rank_mirror: empty corpus");
  if (!mirror || !master || !queries || !out_scores || !out_index || !out_certified)
    return fail(MI_ERR_ARG, "mi_rank_mirror: null pointer");
  const size_t need = rank_mirror_workspace_bytes(N, Q);
  if (!workspace || workspace_bytes < need)
    return fail(MI_ERR_ARG, "mi_rank_mirror: workspace too small (%zu < %zu)", workspace_bytes, need);
  HIP_TRY(rank_mirror((const uint16_t*)mirror, master, N, D, master_dtype, queries, Q, k, index_base,
                      nan_policy == MI_NAN_FIRST, out_scores, out_index, out_certified, workspace, (hipStream_t)stream));
  return MI_OK;
}

int mi_rank_merge(const float* cs, const int64_t* ci, int64_t Q, int64_t C, int32_t k, int nan_policy, float* out_s,
                  int64_t* out_i, void* stream) {
  if (Q < 0 || C < 0) return fail(MI_ERR_ARG, "negative size");
  if (k < 1 || k > RANK_REG_K) return fail(MI_ERR_UNSUPPORTED, "k must be in [1, %d] (got %d)", RANK_REG_K, k);
  if (nan_policy != MI_NAN_FIRST && nan_policy != MI_NAN_LAST) return fail(MI_ERR_ARG, "bad nan_policy");
  if (Q == 0) return MI_OK;
  if ((C > 0 && (!cs || !ci)) || !out_s || !out_i) return fail(MI_ERR_ARG, "mi_rank_merge: null pointer");
  HIP_TRY(rank_merge(cs, ci, Q, C, k, nan_policy == MI_NAN_FIRST, out_s, out_i, (hipStream_t)stream));
  return MI_OK;
}

int mi_score_matrix(const void* corpus, int64_t N, int64_t D, int corpus_dtype, const float* queries, int64_t Q,
                    int norm_mode, float* out, void* stream) {
  int r = check_rank_args(N, D, corpus_dtype, Q, 1, norm_mode, MI_NAN_FIRST);
  if (r) return r;
  if (N == 0 || Q == 0) return MI_OK;
  if (!corpus || !queries || !out) return fail(MI_ERR_ARG, "mi_score_matrix: null pointer");
  HIP_TRY(score_matrix(corpus, N, D, corpus_dtype, queries, Q, norm_mode, out, (hipStream_t)stream));
  return MI_OK;
}

int mi_rank_of_targets(const float* scores, int64_t Q, int64_t N, const int64_t* pq, const int64_t* pt, int64_t T,
                       int64_t* out, void* stream) {
  if (Q < 0 || N < 0 || T < 0) return fail(MI_ERR_ARG, "negative size");
  if (T == 0) return MI_OK;
  if (!scores || !pq || !pt || !out) return fail(MI_ERR_ARG, "mi_rank_of_targets: null pointer");
  HIP_TRY(rank_of_targets(scores, Q, N, pq, pt, T, out, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_gemm(const void* A, const void* W, const float* bias, void* out, int32_t M, int32_t N, int32_t K,
               int32_t epi, void* stream) {
  if (!A || !W || !out || M < 0) return fail(MI_ERR_ARG, "mi_op_gemm: bad arguments");
  if (K % 64 || N % 128 || K <= 0) return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm: needs K %% 64 == 0, N %% 128 == 0");
  const int variant = epi >> 8;  // bits 8+: schedule override for A/B measurements
  if (variant && !MICLIP_AB) return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm: schedule overrides need the A/B build (make ab)");
  epi &= 0xff;
  if (epi < 0 || epi > 3) return fail(MI_ERR_ARG, "mi_op_gemm: bad epilogue");
  GemmArgs g = gargs((const uint16_t*)A, K, (const uint16_t*)W, K, bias, out, N, M, N, K);
  if (variant) g.variant = variant;
  HIP_TRY(gemm_bf16(g, epi, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_gemm_f32(const float* A, const float* W, const float* bias, float* out, int32_t M, int32_t N, int32_t K,
                   int32_t epi, void* stream) {
  if (!A || !W || !out || M < 0 || N < 1) return fail(MI_ERR_ARG, "mi_op_gemm_f32: bad arguments");
  if (K % 32 || K <= 0) return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_f32: needs K %% 32 == 0");
  static const int epis[4] = {EPI_F32, EPI_GELU_BF16, EPI_RESID_F32, EPI_RELU_F32};
  if (epi < 0 || epi > 3) return fail(MI_ERR_ARG, "mi_op_gemm_f32: epilogue 0 (store), 1 (QuickGELU), 2 (+=), 3 (ReLU)");
  HIP_TRY(gemm_f32(A, K, W, K, bias, out, N, M, N, K, epis[epi], (hipStream_t)stream));
  return MI_OK;
}

// Diagnostics: timestamps of the GEMM timing-probe variant (19), 4 per
// workgroup (not part of include/miclip.h; scripts/gemm_micro.py only).
extern "C" int mi_debug_gemm_probe(unsigned long long* host, int32_t n) {
  if (!host || n < 0) return fail(MI_ERR_ARG, "mi_debug_gemm_probe: bad arguments");
  HIP_TRY(gemm_probe_read(host, n));
  return MI_OK;
}

extern "C" int mi_debug_gemm8q_probe(unsigned long long* host, int32_t n) {
  if (!host || n < 0) return fail(MI_ERR_ARG, "mi_debug_gemm8q_probe: bad arguments");
  HIP_TRY(gemm8q_probe_read(host, n));
  return MI_OK;
}

int mi_op_layernorm(const float* x, const float* g, const float* b, void* out, int32_t rows, int32_t W,
                    void* stream) {
  if (!x || !g || !b || !out || rows < 0) return fail(MI_ERR_ARG, "mi_op_layernorm: bad arguments");
  if (W % 4 || W > 1024) return fail(MI_ERR_UNSUPPORTED, "mi_op_layernorm: W must be a multiple of 4, <= 1024");
  HIP_TRY(layernorm_bf16(x, W, g, b, (uint16_t*)out, W, rows, W, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_residual_ln(void* x, const void* delta, const float* g, const float* b, void* out, int32_t rows, int32_t W,
                      int32_t xmode, void* stream) {
  if (!x || !delta || !g || !b || !out || rows < 0) return fail(MI_ERR_ARG, "mi_op_residual_ln: bad arguments");
  if (W % 4 || W > 1024) return fail(MI_ERR_UNSUPPORTED, "mi_op_residual_ln: W must be a multiple of 4, <= 1024");
  if (xmode < 0 || xmode > 2) return fail(MI_ERR_ARG, "mi_op_residual_ln: xmode must be 0, 1 or 2");
  HIP_TRY(residual_ln((float*)x, (const uint16_t*)delta, W, 1, g, b, (uint16_t*)out, rows, W, (hipStream_t)stream,
                      nullptr, nullptr, xmode));
  return MI_OK;
}

int mi_op_split6(const float* x, int64_t ldx, int64_t rows, int32_t K, int32_t role, int32_t gelu, void* out,
                 void* stream) {
  if (!x || !out || rows < 0 || (role & ~1) || (gelu & ~1)) return fail(MI_ERR_ARG, "mi_op_split6: bad arguments");
  if (K < 4 || K % 4 || ldx < K || ldx % 4) return fail(MI_ERR_UNSUPPORTED, "mi_op_split6: K %% 4 == 0, ldx >= K, ldx %% 4 == 0");
  HIP_TRY(split6_rows(x, ldx, rows, K, role, gelu, (uint16_t*)out, (hipStream_t)stream));
  return MI_OK;
}

int mi_clip_kernel_events(mi_clip* c, int32_t kind, int32_t capacity) {
  if (!c || kind < 0 || kind > MI_KERNEL_C_FC || capacity < 0 || capacity > (1 << 16))
    return fail(MI_ERR_ARG, "mi_clip_kernel_events: bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  while ((int)c->ev.size() < 2 * capacity) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    c->ev.push_back(e);
  }
  c->ev_kind = capacity ? kind : 0;
  c->ev_cap = capacity;
  c->ev_n = 0;
  return MI_OK;
}

int mi_clip_kernel_times(mi_clip* c, float* us, int32_t n) {
  if (!c || (!us && n > 0) || n < 0) return fail(MI_ERR_ARG, "mi_clip_kernel_times: bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  const int m = c->ev_n < n ? c->ev_n : n;
  for (int i = 0; i < m; ++i) {
    HIP_TRY(hipEventSynchronize(c->ev[2 * i + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[2 * i], c->ev[2 * i + 1]));
    us[i] = ms * 1e3f;
  }
  return m;
}

int mi_op_split2h(const float* x, int64_t ldx, int64_t rows, int32_t K, int32_t role, int32_t gelu, void* out,
                  float* scale, void* stream) {
  if (!x || !out || !scale || rows < 0 || role < 0 || role > 2 || (gelu & ~1))
    return fail(MI_ERR_ARG, "mi_op_split2h: bad arguments");
  if (K < 4 || K > 4096 || K % 4 || ldx < K || ldx % 4)
    return fail(MI_ERR_UNSUPPORTED, "mi_op_split2h: 4 <= K <= 4096, K %% 4 == 0, ldx >= K, ldx %% 4 == 0");
  HIP_TRY(split2h_rows(x, ldx, rows, K, role, gelu, (uint16_t*)out, scale, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_gemm_split2h(const void* A3, const void* W3, const float* a_scale, const float* w_scale, const float* bias,
                       float* out, int32_t M, int32_t N, int32_t K3, int32_t epi, void* stream) {
  const int dup = (epi >> 8) & 1;
  epi &= ~0x100;
  if (!A3 || !W3 || !a_scale || !w_scale || !out || M < 0 || N < 1 || K3 < 1 || (epi != EPI_F32 && epi != EPI_RESID_F32))
    return fail(MI_ERR_ARG, "mi_op_gemm_split2h: bad arguments");
  if (N % 128 || K3 % 32) return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_split2h: N %% 128 == 0, K3 %% 32 == 0");
  GemmArgs g = gargs((const uint16_t*)A3, dup ? 2 * (K3 / 3) : K3, (const uint16_t*)W3, K3, bias, out, N, M, N, K3);
  g.variant = 0;
  g.a_f16 = 1;
  g.rsc = a_scale;
  g.csc = w_scale;
  g.a_dup = dup ? K3 / 3 : 0;
  if (dup && (K3 % 3 || !bias || !gemm_8q_ok(g)))
    return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_split2h: the [x1 x2] layout needs M >= 256, N %% 256 == 0, K %% 64 == 0");
  HIP_TRY(gemm_bf16(g, epi, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_attention_f32_split(const float* qkv, const float* rmax, float bw, float bb, void* out, int32_t role,
                              float* scale, int32_t B, int32_t S, int32_t W, int32_t causal, void* stream) {
  if (!qkv || !rmax || !out || !scale || B < 0 || S < 1 || W < 64 || (causal & ~1) || (role != 0 && role != 2))
    return fail(MI_ERR_ARG, "mi_op_attention_f32_split: bad arguments");
  if (W % 64 || S > 64) return fail(MI_ERR_UNSUPPORTED, "mi_op_attention_f32_split: W %% 64 == 0 and S <= 64");
  HIP_TRY(attention_f32_split(qkv, rmax, bw, bb, (uint16_t*)out, role, scale, B, S, W, causal, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_attention_f32(const float* qkv, float* out, int32_t B, int32_t S, int32_t W, int32_t causal, void* stream) {
  if (!qkv || !out || B < 0 || S < 1 || W < 64 || (causal & ~1)) return fail(MI_ERR_ARG, "mi_op_attention_f32: bad arguments");
  if (W % 64) return fail(MI_ERR_UNSUPPORTED, "mi_op_attention_f32: W %% 64 == 0");
  HIP_TRY(attention_f32(qkv, out, B, S, W, causal, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_residual_stats(void* x, const void* delta, float* rs, int32_t rows, int32_t W, void* stream) {
  if (!x || !delta || !rs || rows < 0) return fail(MI_ERR_ARG, "mi_op_residual_stats: bad arguments");
  if (W % 4 || W > 1024) return fail(MI_ERR_UNSUPPORTED, "mi_op_residual_stats: W must be a multiple of 4, <= 1024");
  HIP_TRY(residual_stats((float*)x, (const uint16_t*)delta, rs, rows, W, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_gemm_ln(const void* x16, int64_t lda, const float* rs, const void* wf, const float* colsum,
                  const float* colc, void* out, int32_t M, int32_t N, int32_t K, int32_t gelu, void* stream) {
  if (!x16 || !rs || !wf || !colsum || !colc || !out || M < 0 || (gelu & ~1))
    return fail(MI_ERR_ARG, "mi_op_gemm_ln: bad arguments");
  if (M == 0) return MI_OK;
  GemmArgs g = gargs((const uint16_t*)x16, lda, (const uint16_t*)wf, K, colc, out, N, M, N, K);
  g.variant = 0;   // one schedule for the folded GEMMs (an A/B MICLIP_GEMM_VARIANT does not apply)
  g.a_f16 = 1;
  g.rs = rs;
  g.colv = colsum;
  if (lda < K || lda % 8 || !gemm_8q_ok(g))
    return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_ln: needs N %% 256 == 0, K %% 128 == 0, K >= 256, M >= 256, "
                                    "lda >= K with lda %% 8 == 0");
  HIP_TRY(gemm_bf16(g, gelu ? EPI_LN_GELU_BF16 : EPI_LN_BF16, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_gemm_residual(void* x16, int64_t ldx, const void* A, int64_t lda, const void* w, const float* bias,
                        float* ps, float* rs, int32_t M, int32_t W, int32_t K, void* stream) {
  if (!x16 || !A || !w || !ps || !rs || M < 0) return fail(MI_ERR_ARG, "mi_op_gemm_residual: bad arguments");
  if (M == 0) return MI_OK;
  GemmArgs g = gargs((const uint16_t*)A, lda, (const uint16_t*)w, K, bias, x16, ldx, M, W, K);
  g.ps = ps;
  if (lda < K || lda % 8 || ldx < W || ldx % 8 || W > 1024 || ((uintptr_t)x16 & 15) || !gemm_8q_ok(g))
    return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_residual: needs W %% 256 == 0, W <= 1024, K %% 128 == 0, K >= 256, "
                                    "M >= 256, lda >= K and ldx >= W multiples of 8, x16 16-byte aligned");
  HIP_TRY(gemm_bf16(g, EPI_RES16_BF16, (hipStream_t)stream));
  HIP_TRY(residual_finalize(ps, rs, M, W, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_attention(const void* qkv, void* out, int32_t B, int32_t S, int32_t W, int32_t causal, void* stream) {
  if (!qkv || !out || B < 0 || S < 1) return fail(MI_ERR_ARG, "mi_op_attention: bad arguments");
  if (W % 64 || S > 640 || (causal & ~0x301)) return fail(MI_ERR_UNSUPPORTED, "mi_op_attention: W %% 64 == 0 and S <= 640");
  if ((causal & 0x100) && !MICLIP_AB) return fail(MI_ERR_UNSUPPORTED, "mi_op_attention: the one-wave kernel (bit 8) is in the A/B build");
  HIP_TRY(attention((const uint16_t*)qkv, (uint16_t*)out, B, S, W, causal, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_gemm_mx(const void* A, const void* a_scale, const void* W, const void* w_scale, const float* bias, void* out,
                  int32_t M, int32_t N, int32_t K, int32_t epi, void* stream) {
  if (!A || !W || !a_scale || !w_scale || !out || M < 0) return fail(MI_ERR_ARG, "mi_op_gemm_mx: bad arguments");
  if (K % 128 || N % 256 || K <= 0) return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_mx: needs K %% 128 == 0, N %% 256 == 0");
  const int variant = epi >> 8;  // bits 8+: kernel override for A/B (gemm_mx: 1 = 16x16x128, 3 = ping-pong)
  if (variant && !MICLIP_AB) return fail(MI_ERR_UNSUPPORTED, "mi_op_gemm_mx: kernel overrides need the A/B build (make ab)");
  epi &= 0xff;
  if (epi != 0 && epi != 1 && epi != 3 && epi != 4)
    return fail(MI_ERR_ARG, "mi_op_gemm_mx: epilogue 0 (bf16), 1 (GELU), 3 (f32) or 4 (GELU -> MX-fp8)");
  GemmArgs g = gargs((const uint16_t*)A, K, (const uint16_t*)W, K, bias, out, N, M, N, K);
  g.variant = variant;
  g.a_scale = (const uint8_t*)a_scale;
  g.w_scale = (const uint8_t*)w_scale;
  if (epi == 4) g.o_scale = (uint8_t*)out + ((int64_t)M * N + 255) / 256 * 256;   // e4m3 [M,N] then its scales
  HIP_TRY(gemm_mx(g, epi, (hipStream_t)stream));
  return MI_OK;
}

int mi_op_quantize_mx(const void* in, void* q, void* scales, int32_t rows, int32_t K, void* stream) {
  if (!in || !q || !scales || rows < 0) return fail(MI_ERR_ARG, "mi_op_quantize_mx: bad arguments");
  if (K % 128 || K <= 0) return fail(MI_ERR_UNSUPPORTED, "mi_op_quantize_mx: K %% 128 == 0");
  HIP_TRY(quantize_mx((const uint16_t*)in, K, (uint8_t*)q, K, (uint8_t*)scales, rows, K, (hipStream_t)stream));
  return MI_OK;
}

int mi_resample_coeffs(int32_t in_size, double in0, double in1, int32_t out_size, int filter, int32_t* kk,
                       int64_t kk_cap, int32_t* bounds) {
  if (!kk || !bounds || in_size < 1 || out_size < 1 || (filter != MI_RESAMPLE_BICUBIC && filter != MI_RESAMPLE_BILINEAR))
    return fail(MI_ERR_ARG, "mi_resample_coeffs: bad arguments");
  std::vector<int32_t> k, b;
  const int ks = resample_coeffs(in_size, in0, in1, out_size, filter, k, b);
  if (ks < 0) return fail(MI_ERR_ARG, "mi_resample_coeffs: bad arguments");
  if ((int64_t)k.size() > kk_cap) return fail(MI_ERR_ARG, "mi_resample_coeffs: kk needs %zu entries", k.size());
  memcpy(kk, k.data(), k.size() * 4);
  memcpy(bounds, b.data(), b.size() * 4);
  return ks;
}

size_t mi_preprocess_workspace_bytes(int64_t B, int32_t H, int32_t W, int32_t n, int mode) {
  return preprocess_workspace_bytes(B, H, W, n, mode);
}

int mi_preprocess_frames(const uint8_t* frames, int64_t B, int32_t H, int32_t W, int32_t n, int mode, void* out,
                         int out_dtype, void* workspace, size_t workspace_bytes, void* stream) {
  if (B < 0 || H < 1 || W < 1 || n < 1 || n > 4096) return fail(MI_ERR_ARG, "mi_preprocess_frames: bad sizes");
  if (mode != MI_PREP_CLIP && mode != MI_PREP_SQUASH) return fail(MI_ERR_ARG, "mi_preprocess_frames: bad mode");
  if (out_dtype != MI_F32 && out_dtype != MI_BF16) return fail(MI_ERR_ARG, "mi_preprocess_frames: out_dtype f32/bf16");
  if (B == 0) return MI_OK;
  if (!frames || !out) return fail(MI_ERR_ARG, "mi_preprocess_frames: null pointer");
  const size_t need = preprocess_workspace_bytes(B, H, W, n, mode);
  if (!workspace || workspace_bytes < need)
    return fail(MI_ERR_ARG, "mi_preprocess_frames: workspace too small (%zu < %zu)", workspace_bytes, need);
  HIP_TRY(preprocess_frames(frames, B, H, W, n, mode, out, out_dtype == MI_BF16, workspace, (hipStream_t)stream));
  return MI_OK;
}

size_t mi_jpeg_workspace_bytes(const int32_t* geom, int32_t B, int64_t data_bytes) {
  if (!geom || B < 0) return 0;
  return jpeg_workspace_bytes(geom, B, data_bytes);
}

static int check_jpeg_args(const char* fn, const uint8_t* data, int64_t data_bytes, const int64_t* seg_off,
                           const int64_t* seg_end, const void* huff, const int32_t* huff_idx, int32_t nsets,
                           const uint16_t* qtab, const int32_t* geom, int32_t B, const void* out, void* workspace,
                           size_t workspace_bytes) {
  if (!geom || B < 0 || data_bytes < 0) return fail(MI_ERR_ARG, "%s: bad arguments", fn);
  if (huff_idx && nsets < 1) return fail(MI_ERR_ARG, "%s: huff_idx needs nsets >= 1", fn);
  if (B == 0) return MI_OK;
  if (!data || !seg_off || !seg_end || !huff || !qtab || !out) return fail(MI_ERR_ARG, "%s: null pointer", fn);
  const int W = geom[0], H = geom[1], nc = geom[2], ri = geom[3], nseg = geom[4];
  if (W < 1 || H < 1 || W > 65535 || H > 65535 || (nc != 1 && nc != 3) || ri < 0 || nseg < 1)
    return fail(MI_ERR_ARG, "%s: bad geometry", fn);
  if (nc == 3) {
    const int h0 = geom[5], v0 = geom[6];
    const bool luma_ok = (h0 == 1 && v0 == 1) || (h0 == 2 && v0 == 1) || (h0 == 2 && v0 == 2);
    for (int c = 1; c < 3; ++c)
      if (geom[5 + 2 * c] != 1 || geom[6 + 2 * c] != 1 || !luma_ok)
        return fail(MI_ERR_UNSUPPORTED, "%s: sampling must be luma 1x1/2x1/2x2 with chroma 1x1", fn);
  }
  for (int c = 0; c < nc; ++c)
    if (geom[11 + c] < 0 || geom[11 + c] > 3 || geom[14 + c] < 0 || geom[14 + c] > 1 || geom[17 + c] < 0 ||
        geom[17 + c] > 1)
      return fail(MI_ERR_ARG, "%s: bad table selector", fn);
  const size_t need = jpeg_workspace_bytes(geom, B, data_bytes);
  if (!workspace || workspace_bytes < need)
    return fail(MI_ERR_ARG, "%s: workspace too small (%zu < %zu)", fn, workspace_bytes, need);
  return MI_OK;
}

int mi_jpeg_decode(const uint8_t* data, int64_t data_bytes, const int64_t* seg_off, const int64_t* seg_end, const void* huff,
                   const int32_t* huff_idx, int32_t nsets, const uint16_t* qtab, const int32_t* geom, int32_t B,
                   uint8_t* out_rgb, void* workspace, size_t workspace_bytes, void* stream) {
  const int r = check_jpeg_args("mi_jpeg_decode", data, data_bytes, seg_off, seg_end, huff, huff_idx, nsets, qtab, geom,
                                B, out_rgb, workspace, workspace_bytes);
  if (r || B == 0) return r;
  HIP_TRY(jpeg_decode(data, data_bytes, seg_off, seg_end, huff, huff_idx, nsets, qtab, geom, B, out_rgb, workspace, workspace_bytes,
                      (hipStream_t)stream));
  return MI_OK;
}

int mi_jpeg_decode_transform(const uint8_t* data, int64_t data_bytes, const int64_t* seg_off, const int64_t* seg_end,
                             const void* huff, const int32_t* huff_idx, int32_t nsets, const uint16_t* qtab,
                             const int32_t* geom, int32_t B, int32_t n, int mode, void* out, int out_dtype,
                             void* workspace, size_t workspace_bytes, void* stream) {
  const int r = check_jpeg_args("mi_jpeg_decode_transform", data, data_bytes, seg_off, seg_end, huff, huff_idx, nsets,
                                qtab, geom, B, out, workspace, workspace_bytes);
  if (r) return r;
  if (n < 1 || n > 4096 || (mode != MI_PREP_CLIP && mode != MI_PREP_SQUASH))
    return fail(MI_ERR_ARG, "mi_jpeg_decode_transform: bad size / mode");
  if (out_dtype != MI_F32 && out_dtype != MI_BF16) return fail(MI_ERR_ARG, "mi_jpeg_decode_transform: out_dtype must be f32/bf16");
  if (B == 0) return MI_OK;
  // the fit check comes first, so no decode work is queued for a geometry the fused transform
  // cannot take; every error after it is a HIP error
  if (!jpeg_xform_fits(geom[1], geom[0], n, mode))
    return fail(MI_ERR_UNSUPPORTED, "mi_jpeg_decode_transform: %dx%d -> %d does not fit one LDS band: use "
                "mi_jpeg_decode + mi_preprocess_frames", geom[0], geom[1], n);
  const JpegXform xf{n, mode, out_dtype == MI_BF16, out};
  HIP_TRY(jpeg_decode(data, data_bytes, seg_off, seg_end, huff, huff_idx, nsets, qtab, geom, B, nullptr, workspace,
                      workspace_bytes, (hipStream_t)stream, &xf));
  return MI_OK;
}

int mi_host_gather(void* dst, const void* const* src, const int64_t* len, int64_t n, int32_t threads) {
  if (!dst || n < 0 || (n > 0 && (!src || !len))) return fail(MI_ERR_ARG, "mi_host_gather: bad arguments");
  // no C++ exception may cross the C ABI (std::bad_alloc, std::system_error from a thread
  // that cannot be created, e.g. under a tight cgroup pids limit)
  try {
  std::vector<int64_t> off((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (len[i] < 0 || (len[i] > 0 && !src[i])) return fail(MI_ERR_ARG, "mi_host_gather: bad piece %lld", (long long)i);
    off[i + 1] = off[i] + len[i];
  }
  const int64_t total = off[n];
  int T = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  if (total < (1 << 22)) T = 1;
  // thread t copies the byte range [t * total / T, (t + 1) * total / T) of the output,
  // piece by piece (pieces split across two threads are copied in two parts)
  auto work = [&](int64_t b0, int64_t b1) {
    int64_t i = std::upper_bound(off.begin(), off.end(), b0) - off.begin() - 1;
    for (int64_t b = b0; b < b1 && i < n; ++i) {
      const int64_t e = std::min(b1, off[i + 1]);
      if (e > b) memcpy((char*)dst + b, (const char*)src[i] + (b - off[i]), (size_t)(e - b));
      b = e;
    }
  };
  if (T == 1) {
    work(0, total);
    return MI_OK;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  int started = 0;
  for (; started < T; ++started) {
    try {
      th.emplace_back(work, total * started / T, total * (started + 1) / T);
    } catch (const std::system_error&) {
      break;   // no more threads: the calling thread copies the remaining ranges
    }
  }
  if (started < T) work(total * started / T, total);
  for (auto& x : th) x.join();
  return MI_OK;
  } catch (const std::exception& ex) {
    return fail(MI_ERR_STATE, "mi_host_gather: %s", ex.what());
  }
}

}  // extern "C"
