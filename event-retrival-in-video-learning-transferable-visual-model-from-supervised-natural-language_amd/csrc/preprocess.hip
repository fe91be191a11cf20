// Frame preprocessing on the GPU (gfx950): Pillow-exact resize + center crop +
// ToTensor + Normalize of decoded RGB frames, producing encode_image's input.
//
// Replaces the per-frame host transforms the reference runs before
// encode_image:
//   mode 0  openai/CLIP _transform(n): Resize(n, BICUBIC) on the short side ->
//           CenterCrop(n) -> ToTensor -> Normalize(CLIP mean/std)
//           (Backend/embedding.py:46, Backend/services/embedding_service.py:406,475);
//   mode 1  compare_models.py:387-391: Resize((n, n)) (torchvision's default
//           BILINEAR) -> ToTensor -> Normalize.
// torchvision resizes PIL images with Pillow's ImagingResample; that algorithm
// is restated in oracle/preprocess_ref.py (pinned bit-exactly against PIL) and
// here: the host computes the same int32 coefficients (22 fractional bits,
// double-precision normalisation — resample_coeffs below), the kernels do
// Pillow's integer accumulation, so the uint8 image before ToTensor is
// bit-identical to Pillow's and the f32 output to torchvision's.
//   pass h: tmp[b][r][x][c] = clip8(2^21 + sum_j src[b][r0+r][xb(x)+j][c] * kh[x][j])
//           for the n crop columns x and the source rows the crop rows need;
//   pass v: out[b][c][y][x] = (clip8(2^21 + sum_j tmp[b][yb(y)+j][x][c] * kv[y][j]) / 255
//                              - mean[c]) / std[c]
// clip8(a) = clamp(a >> 22, 0, 255).  A pass Pillow skips (size unchanged) is
// an identity coefficient row (2^22), which reproduces the input exactly.
// Roofline HBM: per frame H*W*3 bytes read (once, the tap overlap is served
// by L1/L2) + the crop's rows*n*3 tmp bytes written and read + 3*n*n*out bytes.
#include "common.hpp"
#include "internal.hpp"

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace miclip {

namespace {

constexpr int PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ uint32_t clip8(int acc) {
  acc >>= PREC;
  return acc < 0 ? 0u : (acc > 255 ? 255u : (uint32_t)acc);
}

// one thread per (frame, tmp row, crop column), 3 channels
__global__ __launch_bounds__(256) void resample_h_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ tmp,
                                                         const int32_t* __restrict__ kh,
                                                         const int32_t* __restrict__ bh, int ksize, int H, int W,
                                                         int n, int r0, int rows, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % n);
  const int64_t t = i / n;  // b * rows + r
  const int r = (int)(t % rows);
  const int64_t b = t / rows;
  const int xb = bh[2 * x], xs = bh[2 * x + 1];
  const int32_t* k = kh + (int64_t)x * ksize;
  const uint8_t* p = src + ((b * H + r0 + r) * (int64_t)W + xb) * 3;
  int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
  for (int j = 0; j < xs; ++j) {
    const int w = k[j];
    s0 += (int)p[3 * j] * w;
    s1 += (int)p[3 * j + 1] * w;
    s2 += (int)p[3 * j + 2] * w;
  }
  uint8_t* o = tmp + (t * n + x) * 3;
  o[0] = (uint8_t)clip8(s0);
  o[1] = (uint8_t)clip8(s1);
  o[2] = (uint8_t)clip8(s2);
}

struct Norm {
  float mean[3], std[3];
};

// one thread per (frame, crop row y, column x), 3 channels -> planar output
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void resample_v_kernel(const uint8_t* __restrict__ tmp, void* __restrict__ out,
                                                         const int32_t* __restrict__ kv,
                                                         const int32_t* __restrict__ bv, int ksize, int rows,
                                                         int n, int r0, Norm nm, int64_t total) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % n);
  const int y = (int)((i / n) % n);
  const int64_t b = i / ((int64_t)n * n);
  const int yb = bv[2 * y] - r0, ys = bv[2 * y + 1];
  const int32_t* k = kv + (int64_t)y * ksize;
  const uint8_t* p = tmp + ((b * rows + yb) * (int64_t)n + x) * 3;
  int s[3] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
  for (int j = 0; j < ys; ++j) {
    const int w = k[j];
    const uint8_t* q = p + (int64_t)j * n * 3;
    s[0] += (int)q[0] * w;
    s[1] += (int)q[1] * w;
    s[2] += (int)q[2] * w;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    // torchvision ToTensor (x / 255) then Normalize ((x - mean) / std), f32, no contraction
    const float v = ((float)clip8(s[c]) / 255.0f - nm.mean[c]) / nm.std[c];
    const int64_t o = ((b * 3 + c) * n + y) * (int64_t)n + x;
    if (OUT_BF16) ((uint16_t*)out)[o] = f2bf(v);
    else ((float*)out)[o] = v;
  }
}

double bicubic(double x) {  // Pillow bicubic_filter, a = -0.5
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

double bilinear(double x) {  // Pillow bilinear_filter
  if (x < 0.0) x = -x;
  if (x < 1.0) return 1.0 - x;
  return 0.0;
}

struct Geometry {
  int nw, nh, left, top, filter;
};

Geometry geometry(int H, int W, int n, int mode) {
  Geometry g;
  if (mode == 1) {
    g.nw = g.nh = n;
    g.left = g.top = 0;
    g.filter = 1;
    return g;
  }
  // torchvision Resize(n): short side n, long side int(n * long / short);
  // CenterCrop(n): offsets int(round((size - n) / 2.0)) (round half to even)
  if (W <= H) {
    g.nw = n;
    g.nh = (int)((double)n * H / W);
  } else {
    g.nw = (int)((double)n * W / H);
    g.nh = n;
  }
  g.left = (int)std::nearbyint((g.nw - n) / 2.0);
  g.top = (int)std::nearbyint((g.nh - n) / 2.0);
  g.filter = 0;
  return g;
}

// Device copies of the coefficient tables per (device, H, W, n, mode),
// uploaded once (the only allocation of the preprocessing path).
struct Tables {
  int32_t *kh = nullptr, *bh = nullptr, *kv = nullptr, *bv = nullptr;
  int ksh = 0, ksv = 0, r0 = 0, rows = 0;
  int xlo = 0, xw = 0;            // source columns the crop's taps read: [xlo, xlo + xw)
  std::vector<int32_t> hbv;       // host copy of bv (the fused JPEG transform sizes its row bands from it)
  int32_t wmax = 0;               // largest |coefficient| of kh / kv (24-bit multiplies apply below 2^23)
};

std::mutex g_tab_mu;
std::map<std::tuple<int, int, int, int, int>, Tables> g_tables;

// coefficients of the crop's outputs [off, off + n) of an in_size -> out_size resize
int crop_coeffs(int in_size, int out_size, int off, int n, int filter, std::vector<int32_t>& kk,
                std::vector<int32_t>& bounds) {
  std::vector<int32_t> k_all, b_all;
  int ks;
  if (in_size == out_size) {  // the pass Pillow skips: identity rows
    ks = 1;
    k_all.assign(out_size, 1 << PREC);
    b_all.resize(2 * out_size);
    for (int i = 0; i < out_size; ++i) {
      b_all[2 * i] = i;
      b_all[2 * i + 1] = 1;
    }
  } else {
    ks = resample_coeffs(in_size, 0.0, (double)in_size, out_size, filter, k_all, b_all);
    if (ks < 0) return ks;
  }
  kk.assign(k_all.begin() + (size_t)off * ks, k_all.begin() + (size_t)(off + n) * ks);
  bounds.assign(b_all.begin() + 2 * off, b_all.begin() + 2 * (off + n));
  return ks;
}

hipError_t get_tables(int H, int W, int n, int mode, Tables& out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(g_tab_mu);
  auto key = std::make_tuple(dev, H, W, n, mode);
  auto it = g_tables.find(key);
  if (it != g_tables.end()) {
    out = it->second;
    return hipSuccess;
  }
  const Geometry g = geometry(H, W, n, mode);
  std::vector<int32_t> kh, bh, kv, bv;
  Tables t;
  t.ksh = crop_coeffs(W, g.nw, g.left, n, g.filter, kh, bh);
  t.ksv = crop_coeffs(H, g.nh, g.top, n, g.filter, kv, bv);
  if (t.ksh < 0 || t.ksv < 0) return hipErrorInvalidValue;
  t.r0 = bv[0];
  int hi = 0;
  for (int y = 0; y < n; ++y) hi = std::max(hi, bv[2 * y] + bv[2 * y + 1]);
  t.rows = hi - t.r0;
  int xlo = W, xhi = 0;
  for (int x = 0; x < n; ++x) {
    xlo = std::min(xlo, bh[2 * x]);
    xhi = std::max(xhi, bh[2 * x] + bh[2 * x + 1]);
  }
  t.xlo = xlo;
  t.xw = xhi - xlo;
  t.hbv = bv;
  for (const int32_t w : kh) t.wmax = std::max(t.wmax, w < 0 ? -w : w);
  for (const int32_t w : kv) t.wmax = std::max(t.wmax, w < 0 ? -w : w);
  const size_t nb = (kh.size() + bh.size() + kv.size() + bv.size()) * 4;
  char* d = nullptr;
  if ((e = hipMalloc(&d, nb)) != hipSuccess) return e;
  std::vector<int32_t> all;
  all.insert(all.end(), kh.begin(), kh.end());
  all.insert(all.end(), bh.begin(), bh.end());
  all.insert(all.end(), kv.begin(), kv.end());
  all.insert(all.end(), bv.begin(), bv.end());
  if ((e = hipMemcpy(d, all.data(), nb, hipMemcpyHostToDevice)) != hipSuccess) {
    (void)hipFree(d);
    return e;
  }
  t.kh = (int32_t*)d;
  t.bh = t.kh + kh.size();
  t.kv = t.bh + bh.size();
  t.bv = t.kv + kv.size();
  g_tables[key] = t;
  out = t;
  return hipSuccess;
}

}  // namespace

int resample_coeffs(int in_size, double in0, double in1, int out_size, int filter, std::vector<int32_t>& kk,
                    std::vector<int32_t>& bounds) {
  if (in_size < 1 || out_size < 1 || (filter != 0 && filter != 1)) return -1;
  // the box inside the input, as Pillow's resize requires ("box can't exceed original image
  // size"); outside it the bounds below would run past the row (and NaN edges fail here too)
  if (!(in0 >= 0.0 && in1 <= (double)in_size && in1 > in0)) return -1;
  double (*fn)(double) = filter == 0 ? bicubic : bilinear;
  const double fsupport = filter == 0 ? 2.0 : 1.0;
  // Pillow precompute_coeffs: the box edges are C floats, their difference is
  // taken in float and then widened
  double filterscale, scale;
  filterscale = scale = (double)((float)in1 - (float)in0) / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = fsupport * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  std::vector<double> pre((size_t)out_size * ksize, 0.0);
  bounds.assign(2 * (size_t)out_size, 0);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (float)in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double* k = &pre[(size_t)xx * ksize];
    for (int x = 0; x < xmax; ++x) {
      const double w = fn((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  // normalize_coeffs_8bpc: round half away from zero to 22 fractional bits
  kk.assign(pre.size(), 0);
  for (size_t i = 0; i < pre.size(); ++i)
    kk[i] = pre[i] < 0 ? (int32_t)(-0.5 + pre[i] * (1 << PREC)) : (int32_t)(0.5 + pre[i] * (1 << PREC));
  return ksize;
}

hipError_t resample_tables(int H, int W, int n, int mode, ResampleTables& r) {
  Tables t;
  const hipError_t e = get_tables(H, W, n, mode, t);
  if (e != hipSuccess) return e;
  r.kh = t.kh;
  r.bh = t.bh;
  r.kv = t.kv;
  r.bv = t.bv;
  r.ksh = t.ksh;
  r.ksv = t.ksv;
  r.xlo = t.xlo;
  r.xw = t.xw;
  r.hbv = t.hbv;
  r.wmax = t.wmax;
  return hipSuccess;
}

size_t preprocess_workspace_bytes(int64_t B, int H, int W, int n, int mode) {
  if (B < 0 || H < 1 || W < 1 || n < 1) return 0;
  (void)mode;  // the crop needs at most all H source rows
  return (size_t)B * H * n * 3 + 256;
}

hipError_t preprocess_frames(const uint8_t* frames, int64_t B, int H, int W, int n, int mode, void* out,
                             int out_bf16, void* ws, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  Tables t;
  hipError_t e = get_tables(H, W, n, mode, t);
  if (e != hipSuccess) return e;
  // the constants as torchvision builds them: Python floats (double) -> float32
  const Norm nm = {{(float)0.48145466, (float)0.4578275, (float)0.40821073},
                   {(float)0.26862954, (float)0.26130258, (float)0.27577711}};
  // A dispatch counts its work-items in 32 bits (grid x block < 2^32): big
  // batches run as several launches of at most 2^31 work-items each.
  const int64_t per = (int64_t)t.rows * n > (int64_t)n * n ? (int64_t)t.rows * n : (int64_t)n * n;
  const int64_t bc = per > 0 ? (((int64_t)1 << 31) / per > 0 ? ((int64_t)1 << 31) / per : 1) : B;
  for (int64_t f0 = 0; f0 < B; f0 += bc) {
    const int64_t nb = B - f0 < bc ? B - f0 : bc;
    const uint8_t* src = frames + f0 * H * W * 3;
    uint8_t* tmp = (uint8_t*)ws + f0 * t.rows * n * 3;
    char* dst = (char*)out + f0 * 3 * n * n * (out_bf16 ? 2 : 4);
    const int64_t th = nb * t.rows * n;
    hipLaunchKernelGGL(resample_h_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, src, tmp, t.kh,
                       t.bh, t.ksh, H, W, n, t.r0, t.rows, th);
    const int64_t tv = nb * n * n;
    if (out_bf16)
      hipLaunchKernelGGL(resample_v_kernel<true>, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s, tmp, dst,
                         t.kv, t.bv, t.ksv, t.rows, n, t.r0, nm, tv);
    else
      hipLaunchKernelGGL(resample_v_kernel<false>, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s, tmp, dst,
                         t.kv, t.bv, t.ksv, t.rows, n, t.r0, nm, tv);
    const hipError_t le = hipGetLastError();
    if (le != hipSuccess) return le;
  }
  return hipSuccess;
}

}  // namespace miclip
