// Corpus-file row normalisation in the file's own dtype (gfx950).
//
// EmbeddingService.get_embeddings (Backend/services/embedding_service.py:209-210)
// normalises the loaded `.npy` rows with
//     embeddings / np.linalg.norm(embeddings, axis=-1, keepdims=True)
// and NumPy evaluates that in the array's dtype.  The reference's default
// corpus files are float16 (Backend/embedding/video_test_3_embeddings.npy and
// image_embeddings.npy, [360,512], written by the GPU path of
// Backend/embedding.py), so the rows that search_top_frames ranks
// (:314-320) and extract_query_confidence scores (:277) are NumPy float16
// arithmetic, not f32 unit vectors.  np.linalg.norm(x, axis=-1) for a float
// array is sqrt(add.reduce((x.conj() * x).real, axis)) (numpy/linalg), which in
// float16 is (NumPy 2.2 loops, pinned bit for bit against NumPy itself by
// tests/test_oracle.py::test_f16_norm_plan_matches_numpy):
//   sq_i  = f16(f32(x_i) * f32(x_i))                      HALF_multiply
//   sum   = f16(0 + pairwise_f32(sq_0 .. sq_{D-1}))        HALF_add reduce: the
//           identity 0 as initial value, then NumPy's pairwise summation in f32:
//           n < 8 sequential; n <= 128 eight strided accumulators combined
//           ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus a sequential tail;
//           otherwise split at n2 = n/2 - (n/2 % 8) and add the halves
//   norm  = f16(sqrtf(f32(sum)))                          HALF_sqrt
//   y_i   = f16(f32(x_i) / f32(norm))                     HALF_divide
// so a zero row becomes NaN (0/0) and an overflowing one 0 or NaN, exactly as
// the reference's arrays do.  One wave per row; the pairwise tree is planned
// on the host (leaves <= 128 elements, <= 8 of them for D <= 1024, so one lane
// per strided accumulator) and replayed in the same order on the device.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {

namespace {

constexpr int kMaxD = 1024;
constexpr int kWaves = 4;

__device__ __forceinline__ float h2f(u16 h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ u16 f2h(float f) { return __builtin_bit_cast(u16, (_Float16)f); }

__global__ __launch_bounds__(256) void normalize_rows_f16_kernel(const u16* in, u16* out,
                                                                 int64_t N, int D, PairwisePlan p) {
  __shared__ float sq[kWaves][kMaxD];
  __shared__ u16 xs[kWaves][kMaxD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWaves + wave;
  const bool valid = row < N;
  if (valid) {
    const u16* src = in + row * D;
    for (int i = lane; i < D; i += 64) {
      const u16 x = src[i];
      const float f = h2f(x);
      xs[wave][i] = x;
      sq[wave][i] = h2f(f2h(f * f));        // f16 square (the f32 product of two f16 is exact)
    }
  }
  __syncthreads();
  if (!valid) return;                       // no barrier below: the rest is wave-local
  const float* s = sq[wave];
  // leaf sums: lane (leaf, j) owns accumulator r[j] of leaf `leaf`
  const int leaf = lane >> 3, j = lane & 7;
  float r = 0.f;
  int start = 0, len = 0;
  if (leaf < p.nleaf) {
    start = p.start[leaf];
    len = p.len[leaf];
    if (len >= 8) {
      r = s[start + j];
      const int body = len - len % 8;
      for (int i = 8; i < body; i += 8) r += s[start + i + j];
    }
  }
  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) on lane j == 0 (float + is commutative bit for bit)
  r += __shfl_xor(r, 1, 64);
  r += __shfl_xor(r, 2, 64);
  r += __shfl_xor(r, 4, 64);
  if (len < 8) {
    r = 0.f;
    for (int i = 0; i < len; ++i) r += s[start + i];
  } else {
    for (int i = len - len % 8; i < len; ++i) r += s[start + i];
  }
  // replay the tree: ops[t] == 0 pushes the next leaf, 1 adds the top two (left + right)
  float leafsum[8];
#pragma unroll
  for (int l = 0; l < 8; ++l) leafsum[l] = __shfl(r, l * 8, 64);
  float st[8];
  int sp = 0, nl = 0;
  for (int t = 0; t < p.nops; ++t) {
    if (p.ops[t] == 0) {
      st[sp++] = leafsum[nl++];
    } else {
      const float right = st[--sp];
      st[sp - 1] = st[sp - 1] + right;
    }
  }
  const float total = 0.f + st[0];          // the reduction's initial value is the identity 0
  const float nrm = h2f(f2h(__builtin_sqrtf(h2f(f2h(total)))));
  u16* dst = out + row * D;
  for (int i = lane; i < D; i += 64) dst[i] = f2h(h2f(xs[wave][i]) / nrm);
}

void plan_rec(int off, int n, PairwisePlan& p) {
  if (n <= 128) {
    if (p.nleaf >= 8) {                     // more leaves than lanes per row: refuse (never for D <= 1024)
      p.nleaf = 9;
      return;
    }
    p.start[p.nleaf] = (int16_t)off;
    p.len[p.nleaf] = (int16_t)n;
    ++p.nleaf;
    if (p.nops < 16) p.ops[p.nops++] = 0;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  plan_rec(off, n2, p);
  plan_rec(off + n2, n - n2, p);
  if (p.nops < 16) p.ops[p.nops++] = 1;
}

}  // namespace

PairwisePlan pairwise_plan(int D) {
  PairwisePlan p{};
  if (D >= 1 && D <= kMaxD) plan_rec(0, D, p);
  return p;
}

hipError_t normalize_rows_f16(const uint16_t* in, int64_t N, int D, uint16_t* out, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const PairwisePlan p = pairwise_plan(D);
  if (p.nleaf < 1 || p.nleaf > 8 || p.nops > 16) return hipErrorInvalidValue;
  const int64_t blocks = (N + kWaves - 1) / kWaves;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(normalize_rows_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, out, N, D, p);
  return hipGetLastError();
}

}  // namespace miclip
