// bf16 MFMA GEMM, one wave per SIMD (gfx950): C[M,N] = A[M,K] . W[N,K]^T
// (+ bias, QuickGELU), bf16 out — the tower GEMMs of openai/CLIP's
// encode_image / encode_text.
//
// Why this shape (measured on the ping-pong kernel, gemm.hip, variants
// 31-35): its MFMA + fragment-read structure alone runs at 93 % of the bf16
// peak, its LDS-DMA operand stream alone at ~45 GB/s per CU; combined the
// stage time is neither, because the stream is only issued in the partner
// wave's load sections and the 32-k stages fetch half 128-byte lines.
// Here
//   * 4 waves, one per SIMD, each owning a 128 x 128 block of the 256 x 256
//     tile (8 x 8 16x16x32 MFMA accumulators = 256 AGPRs): every fragment read
//     from LDS feeds 8 MFMAs (4 in the ping-pong kernel);
//   * K is staged 64 wide: a stage is the tile's 256 A rows and 256 W rows x
//     128 bytes, i.e. whole lines; each LDS-DMA instruction moves 8 rows x
//     128 B (lane = row (lane>>3), 16-byte slot lane&7);
//   * two stage buffers (2 x 64 KB); stage g+2 is issued right after the
//     barrier in the middle of stage g, so it has a full stage of MFMA work
//     to land;
//   * fragments are double-buffered in registers per 32-k step: the 16
//     ds_reads of the next step are issued ahead of the 64 MFMAs of the
//     current one;
//   * persistent: one workgroup per CU walks its tiles; the stage stream runs
//     across tile boundaries, so the next tile's first stages are in flight
//     during this tile's epilogue, and the epilogue's stores are counted in
//     the next wait (vmcnt) instead of drained.
// LDS image: row r of a stage part at r * 128 B, 16-byte slot s of the row at
// physical slot s ^ ((r >> 1) & 7) — a ds_read_b128 lane group (16 distinct
// rows, one slot) then covers all 16 bank slots (conflict-free); the DMA
// applies the same permutation on its source address (the LDS side of an
// LDS-DMA is lane-linear, guide §5.4 rule 21).
#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int BM = 256, BN = 256, BKW = 64;
constexpr int PART = 256 * BKW * 2;      // 32 KB: one operand's rows of a stage
constexpr int STAGE = 2 * PART;          // 64 KB
constexpr int NSTORE = 32;               // epilogue store instructions per wave (full tile)

__device__ __forceinline__ float quick_gelu_w4(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v));
}

__device__ __forceinline__ float4 lds_read_f4_w4(const float* p) {
  float4 v;
  const uint32_t addr = (uint32_t)(uintptr_t)(const LDS_AS float*)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// logical tile t -> (m-block, n-block): n-blocks walked in groups of ng
// (ng <= 0 or >= tiles_n: m-major raster), as gemm.hip tile_coords
__device__ __forceinline__ void tile_coords_w4(int t, int tiles_m, int tiles_n, int ng, int& mb, int& nb) {
  if (ng <= 0 || ng >= tiles_n) {
    mb = t / tiles_n;
    nb = t % tiles_n;
    return;
  }
  const int per = tiles_m * ng;
  const int gg = t / per, r = t - gg * per;
  const int ngg = min(ng, tiles_n - gg * ng);
  mb = r / ngg;
  nb = gg * ng + r % ngg;
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_w4_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2 * BN * 4];
  float* sbias = (float*)(smem + 2 * STAGE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int nk = a.K / BKW;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntiles) return;

  auto coords = [&](int v, int& mm, int& nn) {
    const int t = xcd_remap(v, ntiles);
    int mb, nb;
    tile_coords_w4(t, tiles_m, tiles_n, a.ngroup, mb, nb);
    mm = mb * BM;
    nn = nb * BN;
  };

  // ---- DMA issue side: cursor (itile, ikt) runs two stages ahead of compute
  const int drow = lane >> 3, dp = lane & 7;
  // per-lane 16-byte slot of the source row: the LDS permutation s ^ ((row >> 1) & 7)
  // depends on the row only through (instruction parity, drow) -> two values
  const int s_even = dp ^ ((drow >> 1) & 7), s_odd = dp ^ ((4 + (drow >> 1)) & 7);
  int iv = blockIdx.x, ikt = 0, ipar = 0;   // tile (virtual id), k-step, bias slot parity of the issue cursor
  int im0 = 0, in0 = 0;
  coords(iv, im0, in0);
  auto load_bias = [&](int slot, int nn) {
    if (wave == 0 && a.bias) glds16(a.bias + nn + lane * 4, sbias + slot * BN);
  };
  load_bias(0, in0);
  // returns false when the stream is exhausted (nothing issued)
  auto issue = [&](int buf) -> bool {
    if (iv >= ntiles) return false;
    char* base = smem + buf * STAGE + wave * 8 * 1024;
    const int64_t ko = (int64_t)ikt * BKW;
    // addresses recomputed per stage (a few VALU each) instead of 16 live 64-bit pointers
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = (wave * 8 + j) * 8 + drow;
      const int sl = (j & 1) ? s_odd : s_even;
      glds16(a.A + (int64_t)min(im0 + row, a.M - 1) * a.lda + ko + sl * 8, base + j * 1024);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = (wave * 8 + j) * 8 + drow;
      const int sl = (j & 1) ? s_odd : s_even;
      glds16(a.W + (int64_t)(in0 + row) * a.ldw + ko + sl * 8, base + PART + j * 1024);
    }
    if (++ikt == nk) {
      ikt = 0;
      iv += G;
      ipar ^= 1;
      if (iv < ntiles) {
        coords(iv, im0, in0);
        load_bias(ipar, in0);
      }
    }
    return true;
  };

  // ---- compute side
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = fr >> 1;                        // ((row >> 1) & 7) for row = 16 x + fr
  const int rd0 = fr * 128 + (((0 * 4 + fq) ^ sw) << 4);   // k-step 0 (k 0..31)
  const int rd1 = fr * 128 + (((1 * 4 + fq) ^ sw) << 4);   // k-step 1 (k 32..63)
  const int arow = (128 * wm) * 128, wrow = PART + (128 * wn) * 128;
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  auto read_frags = [&](int buf, int rd, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 8; ++i) fb[i] = *(const bf16x8*)(base + wrow + i * 16 * 128 + rd);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *(const bf16x8*)(base + arow + i * 16 * 128 + rd);
  };
  f32x4 acc[8][8];
  auto mfma_step = [&](const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ni], fa[mi], acc[mi][ni], 0, 0, 0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: stages 0 and 1 in flight, stage 0 landed, its k-step 0 fragments read
  issue(0);
  const bool two = issue(1);
  if (two) vm_wait<16>(); else vm_wait<0>();
  barrier();
  read_frags(0, rd0, fa0, fb0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  int g = 0;           // global stage index of the compute cursor
  int pend = 0;        // epilogue stores of the previous tile still counted in vmcnt
  int cpar = 0;        // bias slot of the tile being computed
  for (int v = blockIdx.x; v < ntiles; v += G) {
    int cm0, cn0;
    coords(v, cm0, cn0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const int buf = g & 1;
      // k-step 0: next fragments (k-step 1 of this stage) read while the MFMAs run
      read_frags(buf, rd1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      mfma_step(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every read of this buffer is done
      // stage g+1 has landed (its 16 DMAs are the oldest outstanding, or only the stores are older)
      if (pend) vm_wait<NSTORE>(); else vm_wait<0>();
      // the stores above stay counted only while they are younger than stage g+1's DMAs
      pend = 0;
      barrier();
      // k-step 1: stage g+2 into this buffer, next stage's k-step 0 fragments, MFMAs
      issue(buf);
      __builtin_amdgcn_sched_barrier(0);
      read_frags(buf ^ 1, rd0, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      mfma_step(fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: bias (+ QuickGELU), bf16, permlane16-swapped 16-byte row stores
    const int gq = fq;
    float4 bias[8];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni)
      bias[ni] = a.bias ? lds_read_f4_w4(sbias + cpar * BN + 128 * wn + ni * 16 + 4 * gq)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    const bool full = cm0 + BM <= a.M;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = cm0 + 128 * wm + mi * 16 + fr;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint2 pk[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ni = 2 * p + q;
          float v0 = acc[mi][ni][0] + bias[ni].x, v1 = acc[mi][ni][1] + bias[ni].y;
          float v2 = acc[mi][ni][2] + bias[ni].z, v3 = acc[mi][ni][3] + bias[ni].w;
          if (EPI == EPI_GELU_BF16) {
            v0 = quick_gelu_w4(v0); v1 = quick_gelu_w4(v1); v2 = quick_gelu_w4(v2); v3 = quick_gelu_w4(v3);
          }
          pk[q] = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        }
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
        const int col = cn0 + 128 * wn + (2 * p + (gq & 1)) * 16 + (gq >> 1) * 8;
        if (m < a.M) *(uint4*)((uint16_t*)a.out + (int64_t)m * a.ldo + col) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
      }
      __builtin_amdgcn_sched_barrier(0);   // one 16-row block at a time (keeps the AGPR reads from piling up)
    }
    cpar ^= 1;
    if (full) {
      pend = 1;
    } else {
      vm_wait<0>();   // a partial tile issued fewer stores than NSTORE
      pend = 0;
    }
  }
  vm_wait<0>();
}

}  // namespace

int gemm_w4_ok(const GemmArgs& a) {
  return a.N % BN == 0 && a.K % BKW == 0 && a.K / BKW >= 2 && a.M >= BM && !a.group && !a.patch_R;
}

hipError_t gemm_w4(const GemmArgs& a, int epi, hipStream_t s, int cus) {
  const int nt = ((a.M + BM - 1) / BM) * (a.N / BN);
  const int grid = nt < cus ? nt : cus;
  if (epi == EPI_GELU_BF16) hipLaunchKernelGGL(gemm_w4_kernel<EPI_GELU_BF16>, dim3(grid), dim3(256), 0, s, a);
  else if (epi == EPI_BF16) hipLaunchKernelGGL(gemm_w4_kernel<EPI_BF16>, dim3(grid), dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace miclip
