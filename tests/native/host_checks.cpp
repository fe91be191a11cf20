// Host-side checks of libmiclip's C-ABI under AddressSanitizer + UBSan (built by
// `make san` in the package's csrc/, run by tests/test_native_sanitize.py; no GPU):
// every entry point whose work is host code (Pillow resample coefficients, the
// multithreaded entropy-byte gather, workspace sizing, the weight-blob size, the
// certificate's delta terms) over sweeps of sizes and edge cases, and the argument
// validation that every GPU entry point performs before it touches the device.
// Exit status 0 = all checks passed (a sanitizer report aborts with its own status).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "miclip.h"

extern "C" int mi_debug_cert_delta(int dt, float* d_rel, float* d_abs);

static int g_fail = 0;
#define CHECK(cond, ...)                                         \
  do {                                                           \
    if (!(cond)) {                                               \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);  \
      std::fprintf(stderr, __VA_ARGS__);                         \
      std::fprintf(stderr, "\n");                                \
      ++g_fail;                                                  \
    }                                                            \
  } while (0)

// Pillow's coefficient table for every (in, out) pair of a sweep: the returned
// support, the bounds inside the input, the table exactly as large as reported.
static void check_resample() {
  std::vector<int32_t> kk, bounds;
  const int ins[] = {1, 2, 3, 7, 31, 224, 225, 336, 337, 720, 1080, 1280, 1920, 3840, 4096};
  const int outs[] = {1, 2, 3, 17, 224, 336, 500, 1024};
  int tables = 0;
  for (int filter = 0; filter < 2; ++filter)
    for (int in : ins)
      for (int out : outs)
        for (int crop = 0; crop < 3; ++crop) {
          // whole input, a centred crop, a window past both edges (rejected: Pillow's box must lie
          // inside the image, and outside it the bounds would run past the row)
          const double in0 = crop == 0 ? 0.0 : crop == 1 ? in * 0.125 : -0.5 * in;
          const double in1 = crop == 0 ? in : crop == 1 ? in * 0.875 : 1.5 * in;
          int64_t cap = 0;
          if (crop == 2) {
            kk.assign(1 << 16, 0);
            bounds.assign(2 * (size_t)out, 0);
            CHECK(mi_resample_coeffs(in, in0, in1, out, filter, kk.data(), 1 << 16, bounds.data()) == MI_ERR_ARG,
                  "resample %d->%d: a box past the input accepted", in, out);
            continue;
          }
          // first call with no room: it must fail and say so, not write
          kk.assign(1, -7);
          bounds.assign(2 * (size_t)out, -7);
          int ks = mi_resample_coeffs(in, in0, in1, out, filter, kk.data(), 0, bounds.data());
          if (ks >= 0) {   // a table of zero entries is impossible: support >= 1
            CHECK(false, "resample %d->%d filter %d: accepted a zero-capacity table", in, out, filter);
            continue;
          }
          CHECK(kk[0] == -7, "resample: wrote past a zero-capacity table");
          for (cap = 16; cap < (int64_t)1 << 26; cap *= 4) {
            kk.assign((size_t)cap + 64, INT32_MIN);   // guard entries after the capacity
            ks = mi_resample_coeffs(in, in0, in1, out, filter, kk.data(), cap, bounds.data());
            if (ks >= 0) break;
          }
          CHECK(ks >= 1, "resample %d->%d filter %d crop %d: no table (%s)", in, out, filter, crop, mi_last_error());
          if (ks < 1) continue;
          for (int64_t i = cap; i < cap + 64; ++i) CHECK(kk[(size_t)i] == INT32_MIN, "resample: wrote past the capacity");
          for (int o = 0; o < out; ++o) {
            const int x0 = bounds[2 * o], n = bounds[2 * o + 1];
            CHECK(x0 >= 0 && n >= 0 && n <= ks && x0 + n <= in, "resample %d->%d: bounds [%d, +%d) outside the input", in,
                  out, x0, n);
          }
          ++tables;
        }
  CHECK(tables >= 2 * 15 * 8 * 2, "resample: only %d tables", tables);
  // invalid arguments fail without writing
  int32_t one = 0, b2[2] = {0, 0};
  CHECK(mi_resample_coeffs(0, 0, 1, 1, 0, &one, 1, b2) == MI_ERR_ARG, "resample in_size 0");
  CHECK(mi_resample_coeffs(4, 0, 4, 0, 0, &one, 1, b2) == MI_ERR_ARG, "resample out_size 0");
  CHECK(mi_resample_coeffs(4, 0, 4, 2, 7, &one, 1, b2) == MI_ERR_ARG, "resample filter 7");
  CHECK(mi_resample_coeffs(4, 0, 4, 2, 0, nullptr, 1, b2) == MI_ERR_ARG, "resample null table");
  CHECK(mi_resample_coeffs(4, 2, 2, 2, 0, &one, 1, b2) == MI_ERR_ARG, "resample empty box");
  CHECK(mi_resample_coeffs(4, NAN, 4, 2, 0, &one, 1, b2) == MI_ERR_ARG, "resample NaN box");
}

// The gather against a serial concatenation: piece counts and lengths (zero-length
// pieces, pieces split across threads), 1 .. 64+ threads, below and above the
// multithreading threshold (4 MB).
static void check_gather() {
  std::mt19937_64 rng(7);
  for (int trial = 0; trial < 40; ++trial) {
    const int n = trial < 5 ? trial : 1 + (int)(rng() % 300);
    const bool big = trial % 3 == 2;
    std::vector<std::vector<uint8_t>> pieces((size_t)n);
    std::vector<const void*> src((size_t)n);
    std::vector<int64_t> len((size_t)n);
    int64_t total = 0;
    for (int i = 0; i < n; ++i) {
      const int64_t L = (rng() % 5 == 0) ? 0 : (int64_t)(rng() % (big ? 200000 : 3000));
      pieces[(size_t)i].resize((size_t)L);
      for (auto& b : pieces[(size_t)i]) b = (uint8_t)rng();
      src[(size_t)i] = L ? pieces[(size_t)i].data() : nullptr;
      len[(size_t)i] = L;
      total += L;
    }
    std::vector<uint8_t> want;
    want.reserve((size_t)total);
    for (auto& p : pieces) want.insert(want.end(), p.begin(), p.end());
    for (int threads : {0, 1, 3, 16, 100}) {
      std::vector<uint8_t> got((size_t)total + 32, 0xA5);
      const int rc = mi_host_gather(got.data(), src.data(), len.data(), n, threads);
      CHECK(rc == MI_OK, "gather n %d threads %d: %s", n, threads, mi_last_error());
      CHECK(total == 0 || std::memcmp(got.data(), want.data(), (size_t)total) == 0, "gather n %d threads %d: wrong bytes",
            n, threads);
      for (size_t i = (size_t)total; i < got.size(); ++i) CHECK(got[i] == 0xA5, "gather: wrote past the total");
    }
  }
  uint8_t d[4];
  const void* s1[1] = {nullptr};
  int64_t l1[1] = {3};
  CHECK(mi_host_gather(nullptr, s1, l1, 1, 1) == MI_ERR_ARG, "gather null dst");
  CHECK(mi_host_gather(d, s1, l1, 1, 1) == MI_ERR_ARG, "gather null piece of length 3");
  l1[0] = -1;
  CHECK(mi_host_gather(d, s1, l1, 1, 1) == MI_ERR_ARG, "gather negative length");
  CHECK(mi_host_gather(d, nullptr, nullptr, 0, 4) == MI_OK, "gather of nothing");
}

static void check_sizes() {
  const mi_clip_arch b32 = {512, 224, 12, 768, 32, 77, 49408, 512, 8, 12};
  const mi_clip_arch l14 = {768, 224, 24, 1024, 14, 77, 49408, 768, 12, 12};
  const mi_clip_arch l336 = {768, 336, 24, 1024, 14, 77, 49408, 768, 12, 12};
  // the OpenAI state dicts' element counts (sum of every tensor the blob carries)
  const int64_t nb = mi_clip_weights_numel(&b32), nl = mi_clip_weights_numel(&l14), n3 = mi_clip_weights_numel(&l336);
  CHECK(nb == 151277313, "B/32 blob %lld (151,277,313 parameters)", (long long)nb);
  CHECK(nl == 427616513, "L/14 blob %lld (427,616,513 parameters)", (long long)nl);
  CHECK(n3 - nl == (577 - 257) * 1024, "L/14@336 blob differs from L/14 by the positional table: %lld", (long long)(n3 - nl));
  mi_clip_arch bad = b32;
  bad.vision_patch_size = 0;   // would divide by zero
  CHECK(mi_clip_weights_numel(&bad) < 0, "patch size 0 accepted");
  bad = b32;
  bad.text_layers = -1;
  CHECK(mi_clip_weights_numel(&bad) < 0, "negative layer count accepted");
  bad = b32;
  bad.image_resolution = 230;  // not a multiple of the patch
  CHECK(mi_clip_weights_numel(&bad) < 0, "resolution not divisible by the patch accepted");
  CHECK(mi_clip_weights_numel(nullptr) < 0, "null arch accepted");

  // workspace sizes: monotone in the corpus / query counts, finite at the extremes
  size_t prev = 0;
  for (int64_t N = 1; N <= ((int64_t)1 << 34); N *= 7) {
    const size_t w = mi_rank_workspace_bytes(N, 32, 10);
    CHECK(w >= prev, "rank workspace not monotone at N %lld", (long long)N);
    prev = w;
  }
  CHECK(mi_rank_workspace_bytes(1000000, 1000, 10) >= mi_rank_workspace_bytes(1000000, 32, 10), "rank workspace in Q");
  CHECK(mi_rank_workspace_bytes(1000000, 32, 200) > 0, "large-k workspace");
  CHECK(mi_rank_mirror_workspace_bytes(1000000, 32) > 0, "mirror workspace");
  CHECK(mi_preprocess_workspace_bytes(256, 720, 1280, 224, MI_PREP_CLIP) > 0, "preprocess workspace");
  CHECK(mi_preprocess_workspace_bytes(0, 720, 1280, 224, MI_PREP_CLIP) == 0 ||
            mi_preprocess_workspace_bytes(0, 720, 1280, 224, MI_PREP_CLIP) < ((size_t)1 << 20),
        "preprocess workspace of nothing");
  int32_t geom[32] = {1280, 720, 3, 0, 1, 2, 2, 1, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1};
  CHECK(mi_jpeg_workspace_bytes(geom, 8192, (int64_t)8192 * 228000) > 0, "jpeg workspace");
  CHECK(mi_jpeg_workspace_bytes(nullptr, 4, 100) == 0, "jpeg workspace of no geometry");
  CHECK(mi_jpeg_workspace_bytes(geom, -1, 100) == 0, "jpeg workspace of -1 frames");

  float dr = 0, da = 0;
  for (int dt = 0; dt < 2; ++dt) {
    CHECK(mi_debug_cert_delta(dt, &dr, &da) == 0, "cert delta %d", dt);
    CHECK(dr > 0 && dr < 1e-3f && da > 0 && da < 1e-5f && std::isfinite(dr), "cert delta %d: %g %g", dt, dr, da);
  }
  CHECK(mi_debug_cert_delta(2, &dr, &da) == MI_ERR_ARG, "cert delta dt 2");
  CHECK(mi_debug_cert_delta(0, nullptr, &da) == MI_ERR_ARG, "cert delta null");
}

// Argument validation ahead of any device work: each call fails with MI_ERR_ARG (or
// MI_ERR_UNSUPPORTED) and a message, and none touches the null / bogus pointers.
static void check_validation() {
  float q[4] = {0, 0, 0, 0};
  float s[4];
  int64_t idx[4];
  CHECK(mi_rank_topk(nullptr, 10, 512, MI_F32, q, 1, 1, 0, MI_NORM_L2, MI_NAN_FIRST, s, idx, nullptr, 0, nullptr) < 0,
        "rank_topk null corpus");
  CHECK(std::strlen(mi_last_error()) > 0, "rank_topk: no message");
  CHECK(mi_rank_topk(q, 10, 0, MI_F32, q, 1, 1, 0, MI_NORM_L2, MI_NAN_FIRST, s, idx, nullptr, 0, nullptr) < 0,
        "rank_topk D 0");
  CHECK(mi_rank_topk(q, 10, 512, 9, q, 1, 1, 0, MI_NORM_L2, MI_NAN_FIRST, s, idx, nullptr, 0, nullptr) < 0,
        "rank_topk dtype 9");
  CHECK(mi_rank_topk(q, 10, 512, MI_F32, q, 1, 0, 0, MI_NORM_L2, MI_NAN_FIRST, s, idx, nullptr, 0, nullptr) < 0,
        "rank_topk k 0");
  CHECK(mi_preprocess_frames(nullptr, 2, 0, 1280, 224, MI_PREP_CLIP, nullptr, MI_BF16, nullptr, 0, nullptr) ==
            MI_ERR_ARG, "preprocess H 0");
  CHECK(mi_preprocess_frames(nullptr, 2, 720, 1280, 224, 5, nullptr, MI_BF16, nullptr, 0, nullptr) == MI_ERR_ARG,
        "preprocess mode 5");
  CHECK(mi_preprocess_frames(nullptr, 2, 720, 1280, 224, MI_PREP_CLIP, nullptr, MI_BF16, nullptr, 0, nullptr) ==
            MI_ERR_ARG, "preprocess null frames");
  CHECK(mi_preprocess_frames((const uint8_t*)q, 2, 720, 1280, 224, MI_PREP_CLIP, s, MI_BF16, nullptr, 0, nullptr) ==
            MI_ERR_ARG, "preprocess no workspace");
  int32_t geom[32] = {1280, 720, 3, 0, 1, 2, 2, 1, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1};
  const uint8_t data[8] = {0};
  const int64_t so[1] = {0}, se[1] = {8};
  const uint16_t qt[64] = {0};
  const uint8_t huff[16] = {0};
  CHECK(mi_jpeg_decode(data, 8, so, se, huff, nullptr, 0, qt, geom, 1, nullptr, nullptr, 0, nullptr) == MI_ERR_ARG,
        "jpeg null output");
  int32_t g2[32];
  std::memcpy(g2, geom, sizeof g2);
  g2[0] = 0;
  CHECK(mi_jpeg_decode(data, 8, so, se, huff, nullptr, 0, qt, g2, 1, (uint8_t*)s, nullptr, 0, nullptr) == MI_ERR_ARG,
        "jpeg width 0");
  std::memcpy(g2, geom, sizeof g2);
  g2[7] = 2;   // chroma 2x1: unsupported sampling
  CHECK(mi_jpeg_decode(data, 8, so, se, huff, nullptr, 0, qt, g2, 1, (uint8_t*)s, nullptr, 0, nullptr) ==
            MI_ERR_UNSUPPORTED, "jpeg chroma 2x1");
  std::memcpy(g2, geom, sizeof g2);
  g2[11] = 4;  // Huffman table selector out of range
  CHECK(mi_jpeg_decode(data, 8, so, se, huff, nullptr, 0, qt, g2, 1, (uint8_t*)s, nullptr, 0, nullptr) == MI_ERR_ARG,
        "jpeg table selector 4");
  CHECK(mi_jpeg_decode(data, 8, so, se, huff, nullptr, 0, qt, geom, 1, (uint8_t*)s, nullptr, 0, nullptr) == MI_ERR_ARG,
        "jpeg no workspace");
  CHECK(mi_clip_create(nullptr, nullptr, 0, 0, MI_BF16, nullptr) < 0, "clip_create null arch");
  CHECK(mi_clip_destroy(nullptr) == MI_OK, "clip_destroy null");
}

int main() {
  CHECK(mi_abi_version() == MICLIP_ABI_VERSION, "abi version %d", mi_abi_version());
  check_resample();
  check_gather();
  check_sizes();
  check_validation();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host checks passed\n");
  return 0;
}
