// bf16 MFMA GEMM, 8-phase interleaved ping-pong (gfx950): C[M,N] = A[M,K] . W[N,K]^T
// (+ bias, QuickGELU), bf16 out — the tower GEMMs of openai/CLIP's
// encode_image / encode_text.
//
// Why (gemm.hip variants 31-35, PMC in DESIGN.md §4): on the 32-k ping-pong
// kernel the operand stream (LDS-DMA) and the MFMA work each fit in well
// under the measured stage time, but they serialise — every wave issues its
// stage's DMAs in one burst after a barrier, the texture addresser backs up
// (TA busy 60 % of the kernel) and the partner group's MFMAs wait at the next
// barrier.  Here the stream is cut into half-tiles (128 rows x 64 k = 16 KB,
// two 1-KB DMAs per thread) and ONE half-tile is issued per phase, beside 16
// MFMAs per wave, so the DMA issue is spread evenly over the main loop
// (cdna_hip_programming.md §5 "The 256² 8-phase template": the per-phase
// ds_read ∥ DMA ∥ MFMA interleave is the lever).
//
// Geometry: 256 x 256 tile, K staged 64 wide (whole 128-byte lines), 8 waves
// as 2 (M) x 4 (N), each owning 128 x 64 outputs = 8 x 4 16x16x32 fragments.
// A wave's 128 x 64 block is computed in four quadrants (64 rows x 32 cols x
// 64 k = 16 MFMAs), one per phase, in the order (m0,n0) (m0,n1) (m1,n1)
// (m1,n0): A fragments are re-read every other phase, B fragments every
// phase but the third.  The four half-tiles of a K-tile are exactly
// what one quadrant phase reads across the workgroup:
//   A_m0 = A rows {0..63, 128..191}, A_m1 = {64..127, 192..255},
//   B_n0 = W rows {wc*64 + 0..31}, B_n1 = {wc*64 + 32..63} (wc = 0..3),
// so a half-tile is free for restaging one phase after the last phase that read it.
// Two K-tile buffers (even / odd K-tile, 64 KB each); one iteration = 8
// phases = 2 K-tiles:
//   phase  reads (buffer)        restages (the next pair unless noted)
//   1      even A_m0 + B_n0      odd  B_n0 (of the CURRENT pair)
//   2      even B_n1             even A_m0
//   3      even A_m1             even B_n1
//   4      even B_n0             even A_m1   + vmcnt(6): odd buffer landed
//   5      odd  A_m0 + B_n0      even B_n0
//   6      odd  B_n1             odd  A_m0
//   7      odd  A_m1             odd  B_n1
//   8      odd  B_n0             odd  A_m1   + vmcnt(6): even buffer landed
// RAW: a buffer is read only in phases after the wait that retires it (and
// after a barrier every issuing wave passed behind that wait); WAR: each
// phase ends its reads with lgkmcnt(0) before its first barrier, so a
// half-tile may be restaged in the next phase.  Every phase is
//   ds_reads; 2 DMAs; [vmcnt]; lgkmcnt(0); s_barrier; 16 MFMA; s_barrier
// with the two M-groups staggered by one barrier: while one group runs its
// MFMAs, the other reads fragments and issues its DMAs.
// Persistent: one workgroup per CU walks its tiles (XCD-contiguous runs,
// xcd_remap); the half-tile stream runs across tile boundaries (stream
// positions past the last tile re-load valid addresses into buffers nobody
// reads again, which keeps every wait count exact), and a tile's epilogue
// (bias, QuickGELU, bf16 row stores) sits in the memory section of the next
// tile's first phase, overlapped with the partner group's MFMAs.
// LDS image of a half-tile: image row r at r * 128 B, 16-byte slot s at
// s ^ ((r >> 1) & 7) (conflict-free ds_read_b128 lane groups); the DMA applies
// the same permutation to its per-lane SOURCE address (lane-linear LDS side,
// guide §5.4 rule 21).
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int BM = 256, BN = 256, BK8 = 64;
constexpr int HALF = 128 * BK8 * 2;   // 16 KB half-tile
constexpr int BUF = 4 * HALF;         // 64 KB K-tile buffer
// half-tile ids (issue/read order) and their slots in a buffer
constexpr int H_A0 = 0, H_B0 = 1, H_B1 = 2, H_A1 = 3;

// QuickGELU x * sigmoid(1.702 x) on a pair: packed FP32 multiplies/adds
// (v_pk_*), one v_exp_f32 (2^x, the 1.702 * log2(e) scale folded) and one
// v_rcp_f32 per value
__device__ __forceinline__ f32x2 quick_gelu2_8p(f32x2 v) {
  const f32x2 t = v * (f32x2){-2.45546696f, -2.45546696f};
  f32x2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  e = e + 1.0f;
  return v * (f32x2){__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}

// bias read the compiler does not see (a plain LDS read would make hipcc
// drain the in-flight DMAs with vmcnt(0), gemm.hip lds_read_f4)
__device__ __forceinline__ float4 lds_read_f4_8p(const float* p) {
  float4 v;
  const uint32_t addr = (uint32_t)(uintptr_t)(const LDS_AS float*)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

__device__ __forceinline__ void tile_coords_8p(int t, int tiles_m, int tiles_n, int ng, int& mb, int& nb) {
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

template <int P>
using PhaseC = std::integral_constant<int, P>;

// ABL (timing probes, gemm.hip variants 91-96): 1 = no operand DMAs, 2 = no MFMAs, 3 = no output
// stores, 4 = no epilogue (bias/activation/pack/stores), 6 = full-line store shape (wrong layout),
// 7 = neither DMAs nor epilogue, 8 = no epilogue and no DMA waits (reads race the DMAs)
template <int EPI, int ABL = 0, bool ALN = false, bool EARLY = false>
__global__ __launch_bounds__(512) void gemm_8p_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 2 * BN * 4];
  float* sbias = (float*)(smem + 2 * BUF);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int npairs = a.K / (2 * BK8);
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntiles) return;

  auto coords = [&](int v, int& mm, int& nn) {
    const int t = xcd_remap(v, ntiles);
    int mb, nb;
    tile_coords_8p(t, tiles_m, tiles_n, a.ngroup, mb, nb);
    mm = mb * BM;
    nn = nb * BN;
  };

  // ---- restage cursor: K-tile pair rpp of tile rv (origin rm0, rn0)
  int rv = blockIdx.x, rpp = 0, rm0, rn0;
  coords(rv, rm0, rn0);
  auto advance = [&]() {
    if (++rpp == npairs) {
      rpp = 0;
      rv += G;
      if (rv < ntiles) coords(rv, rm0, rn0);   // past the end: keep re-loading valid rows
    }
  };
  const int drow = lane >> 3;
  const int c0 = (lane & 7) ^ (lane >> 4), c1 = (lane & 7) ^ (4 + (lane >> 4));
  // one half-tile h of K-tile (2 * rpp + b) into buffer b: two 1-KB DMAs per thread
  auto issue = [&](int h, int b) {
    if (ABL == 1 || ABL == 7) return;
    const int kofs = (2 * rpp + b) * BK8;
    char* dst = smem + b * BUF + h * HALF + (2 * wave) * 1024;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ir = (2 * wave + j) * 8 + drow;      // image row 0..127
      const int c = j ? c1 : c0;
      const uint16_t* src;
      if (h == H_A0 || h == H_A1) {
        const int row = (ir >> 6) * 128 + (h == H_A1 ? 64 : 0) + (ir & 63);
        src = a.A + (int64_t)min(rm0 + row, a.M - 1) * a.lda + kofs + c * 8;
      } else {
        const int row = (ir >> 5) * 64 + (h == H_B1 ? 32 : 0) + (ir & 31);
        src = a.W + (int64_t)(rn0 + row) * a.ldw + kofs + c * 8;
      }
      glds16(src, dst + j * 1024);
    }
  };

  // ---- fragment side
  const int fr = lane & 15, fq = lane >> 4;
  const int rd0 = fr * 128 + (((0 + fq) ^ (fr >> 1)) << 4);   // k 0..31 of the K-tile
  const int rd1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);   // k 32..63
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](const char* half) {   // this wave's 64 rows of an A half-tile
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const char* p = half + (wr * 64 + mi * 16) * 128;
      fa[mi][0] = *(const bf16x8*)(p + rd0);
      fa[mi][1] = *(const bf16x8*)(p + rd1);
    }
  };
  auto read_b = [&](const char* half, bf16x8 (&fb)[2][2]) {   // this wave's 32 rows of a B half-tile
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const char* p = half + (wc * 32 + ni * 16) * 128;
      fb[ni][0] = *(const bf16x8*)(p + rd0);
      fb[ni][1] = *(const bf16x8*)(p + rd1);
    }
  };
  f32x4 acc[8][4];
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  int cm0 = 0, cn0 = 0, cpar = 0;   // tile being computed, its bias slot
  int nxt_n0 = 0;
  bool has_next = false;
  bool pre = false;   // EARLY: this tile's first phase-1 DMAs went out ahead of the previous epilogue
  bool first_pair = true;

  auto phase = [&](auto pc, bool last_pair) {
    constexpr int P = decltype(pc)::value;
    constexpr int b = P <= 4 ? 0 : 1;
    constexpr int q = (P - 1) & 3;
    const char* rbuf = smem + b * BUF;
    if (q == 0) {
      read_a(rbuf + H_A0 * HALF);
      read_b(rbuf + H_B0 * HALF, fb0);
    } else if (q == 1) {
      read_b(rbuf + H_B1 * HALF, fb1);
    } else if (q == 2) {
      read_a(rbuf + H_A1 * HALF);
    } else {
      read_b(rbuf + H_B0 * HALF, fb0);   // re-read (16 fewer live VGPRs than keeping it from phase 1)
    }
    __builtin_amdgcn_sched_barrier(0);
    if (P == 1 && !(EARLY && pre && first_pair)) issue(H_B0, 1);
    if (P == 2) { advance(); issue(H_A0, 0); }
    if (P == 3) issue(H_B1, 0);
    if (P == 4) issue(H_A1, 0);
    if (P == 5) issue(H_B0, 0);
    if (P == 6) issue(H_A0, 1);
    if (P == 7) issue(H_B1, 1);
    if (P == 8) issue(H_A1, 1);
    __builtin_amdgcn_sched_barrier(0);
    // the awaited half-tile has 3 phases of DMAs younger than it (EARLY, first
    // pair: + the previous tile's 16 epilogue stores)
    if (ABL == 8) {   // timing probe: never wait for the DMAs (reads race them)
    } else if (P == 4 && EARLY && pre && first_pair) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
    else if (P == 4 || P == 8) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    if (P == 8 && last_pair && has_next && wave == 0 && a.bias)   // next tile's bias, older than phase 1's DMAs
      glds16(a.bias + nxt_n0 + lane * 4, sbias + (cpar ^ 1) * BN);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    constexpr int mh = q >= 2 ? 1 : 0, nh = (q == 1 || q == 2) ? 1 : 0;
    auto& fb = nh ? fb1 : fb0;
    if (ABL == 2) {   // keep the fragments live, skip the MFMAs
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) asm volatile("" ::"v"(fa[mi][0]), "v"(fa[mi][1]));
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) asm volatile("" ::"v"(fb[ni][0]), "v"(fb[ni][1]));
    } else
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mh * 4 + mi][nh * 2 + ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ni][ks], fa[mi][ks], acc[mh * 4 + mi][nh * 2 + ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
  };

  // ---- prologue: tile 0's bias, the whole even K-tile and three odd half-tiles of pair 0
  {
    int m0, n0;
    coords(blockIdx.x, m0, n0);
    if (wave == 0 && a.bias) glds16(a.bias + n0 + lane * 4, sbias);
  }
  issue(H_A0, 0);
  issue(H_B1, 0);
  issue(H_A1, 0);
  issue(H_B0, 0);
  issue(H_A0, 1);
  issue(H_B1, 1);
  issue(H_A1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  barrier();
  if (wr == 1) barrier();   // stagger the two M-groups by one barrier

  const int g = fq;
  for (int v = blockIdx.x; v < ntiles; v += G) {
    coords(v, cm0, cn0);
    has_next = v + G < ntiles;
    if (has_next) {
      int nm0;
      coords(v + G, nm0, nxt_n0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int pp = 0; pp < npairs; ++pp) {
      first_pair = pp == 0;
      const bool lastp = pp == npairs - 1;
      phase(PhaseC<1>{}, lastp);
      phase(PhaseC<2>{}, lastp);
      phase(PhaseC<3>{}, lastp);
      phase(PhaseC<4>{}, lastp);
      phase(PhaseC<5>{}, lastp);
      phase(PhaseC<6>{}, lastp);
      phase(PhaseC<7>{}, lastp);
      phase(PhaseC<8>{}, lastp);
    }
    if (ALN && wr == 0) barrier();   // ALN: both M-groups run the epilogue in the same interval
    if (EARLY) {
      // the next tile's phase-1 DMAs go out now (the restage cursor is at its
      // first pair), so this epilogue's stores are younger than them and stay
      // in flight through the next phase-4 wait (vmcnt(22) there)
      pre = has_next;
      if (has_next) issue(H_B0, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue (in the next phase's memory section): bias (+ QuickGELU),
    // bf16, permlane16-swapped 16-byte row stores (gemm.hip DIRECT form)
    float4 bias[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      bias[ni] = a.bias ? lds_read_f4_8p(sbias + cpar * BN + wc * 64 + ni * 16 + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = cm0 + wr * 128 + mi * 16 + fr;
      if (ABL == 4 || ABL == 7 || ABL == 8) {   // no epilogue work at all: keep the accumulators live
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
        continue;
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint2 pk[2];
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const int ni = 2 * p + qq;
          f32x2 lo = (f32x2){acc[mi][ni][0], acc[mi][ni][1]} + (f32x2){bias[ni].x, bias[ni].y};
          f32x2 hi = (f32x2){acc[mi][ni][2], acc[mi][ni][3]} + (f32x2){bias[ni].z, bias[ni].w};
          if (EPI == EPI_GELU_BF16) {
            lo = quick_gelu2_8p(lo);
            hi = quick_gelu2_8p(hi);
          }
          pk[qq] = make_uint2(pack_bf16x2(lo), pack_bf16x2(hi));
        }
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
        const int col = cn0 + wc * 64 + (2 * p + (g & 1)) * 16 + (g >> 1) * 8;
        if (ABL == 3) {
          asm volatile("" ::"v"(sx[0]), "v"(sy[0]), "v"(sx[1]), "v"(sy[1]));
        } else if (ABL == 6) {   // 8 rows x 128-B full lines per store instruction (timing only)
          const int mr = cm0 + wr * 128 + mi * 16 + p * 8 + (lane >> 3);
          if (mr < a.M)
            *(uint4*)((uint16_t*)a.out + (int64_t)mr * a.ldo + cn0 + wc * 64 + (lane & 7) * 8) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        } else if (m < a.M) {
          *(uint4*)((uint16_t*)a.out + (int64_t)m * a.ldo + col) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // a partial tile may skip whole store instructions: the counted wait needs all 16
    if (EARLY && cm0 + BM > a.M) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    cpar ^= 1;
    if (ALN && wr == 1 && v + G < ntiles) barrier();   // re-stagger
  }
  if (!ALN && wr == 0) barrier();   // the M-groups' barrier counts meet
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing (dummy) DMAs land before the workgroup's LDS is released
}

}  // namespace

int gemm_8p_ok(const GemmArgs& a) {
  return a.N % BN == 0 && a.K % (2 * BK8) == 0 && a.M >= BM && !a.group && !a.patch_R;
}

template <int EPI>
static hipError_t launch_probe(const GemmArgs& a, hipStream_t s, int grid, int abl) {
  if (abl == 1) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 1>), dim3(grid), dim3(512), 0, s, a);
  else if (abl == 2) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 2>), dim3(grid), dim3(512), 0, s, a);
  else if (abl == 3) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 3>), dim3(grid), dim3(512), 0, s, a);
  else if (abl == 4) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 4>), dim3(grid), dim3(512), 0, s, a);
  else if (abl == 6) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 6>), dim3(grid), dim3(512), 0, s, a);
  else if (abl == 7) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 7>), dim3(grid), dim3(512), 0, s, a);
  else if (abl == 8) hipLaunchKernelGGL((gemm_8p_kernel<EPI, 8>), dim3(grid), dim3(512), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t gemm_8p(const GemmArgs& a, int epi, hipStream_t s, int cus, int abl) {
  const int nt = ((a.M + BM - 1) / BM) * (a.N / BN);
  const int grid = nt < cus ? nt : cus;
  if (abl == 101) {   // early phase-1 DMAs
    if (epi == EPI_GELU_BF16) hipLaunchKernelGGL((gemm_8p_kernel<EPI_GELU_BF16, 0, false, true>), dim3(grid), dim3(512), 0, s, a);
    else if (epi == EPI_BF16) hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 0, false, true>), dim3(grid), dim3(512), 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (abl == 102) {   // early phase-1 DMAs + aligned epilogue
    if (epi == EPI_GELU_BF16) hipLaunchKernelGGL((gemm_8p_kernel<EPI_GELU_BF16, 0, true, true>), dim3(grid), dim3(512), 0, s, a);
    else if (epi == EPI_BF16) hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 0, true, true>), dim3(grid), dim3(512), 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (abl == 100) {   // aligned epilogue
    if (epi == EPI_GELU_BF16) hipLaunchKernelGGL((gemm_8p_kernel<EPI_GELU_BF16, 0, true>), dim3(grid), dim3(512), 0, s, a);
    else if (epi == EPI_BF16) hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 0, true>), dim3(grid), dim3(512), 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (abl) {
    if (epi == EPI_GELU_BF16) return launch_probe<EPI_GELU_BF16>(a, s, grid, abl);
    if (epi == EPI_BF16) return launch_probe<EPI_BF16>(a, s, grid, abl);
    return hipErrorInvalidValue;
  }
  if (epi == EPI_GELU_BF16) hipLaunchKernelGGL(gemm_8p_kernel<EPI_GELU_BF16>, dim3(grid), dim3(512), 0, s, a);
  else if (epi == EPI_BF16) hipLaunchKernelGGL(gemm_8p_kernel<EPI_BF16>, dim3(grid), dim3(512), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace miclip
