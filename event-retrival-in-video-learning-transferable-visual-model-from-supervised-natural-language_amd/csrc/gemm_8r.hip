// bf16 MFMA GEMM with a deferred epilogue (gfx950): C[M,N] = A[M,K] . W[N,K]^T
// (+ bias, QuickGELU), bf16 out — the tower GEMMs of openai/CLIP's
// encode_image / encode_text.
//
// Why (scripts/gemm_probe8q.py, in-kernel s_memtime stamps of gemm_8q): on the
// 256 x 256 tile the epilogue runs twice per tile (once per M-group) with
// nothing beside it — QuickGELU's VALU (~4.2k cycles per wave: 128 values x
// (exp + rcp + 3 plain ops)) on c_fc, the store issue (~48 cycles per 1-KB
// store instruction per CU, 64 per group) on the others — ~28 % of a K = 768
// tile.  Hiding it under the next tile's MFMAs needs the finished tile's
// accumulators to stay in registers while the next one accumulates, which a
// 128 x 64 wave tile (128 accumulator VGPRs) cannot afford at two waves per
// SIMD.  Here each wave owns 64 x 64 outputs (64 accumulator VGPRs), so a
// second set holds the previous tile (`pend`) and is drained one 16 x 32
// chunk (8 values per lane: bias, QuickGELU, bf16, one permlane16-swapped
// 16-byte row store) per K-tile over the next tile's first 8 K-tiles, in the
// memory section of the K-tile's second phase.
//
// Geometry: 256 x 128 tile, K staged 64 wide (128-byte image rows), 8 waves as
// 4 (M) x 2 (N); wave (wr, wc) owns rows wr*64.., cols wc*64.. as 4 x 4
// 16x16x32 fragments.  A K-tile buffer (48 KB) holds A0 (rows 0-127, read only
// by M-group 0 = waves 0-3), A1 (rows 128-255, group 1), Bh0 (W rows
// {0-31, 64-95}: the ni = 0,1 fragments of both wave columns) and Bh1 (W rows
// {32-63, 96-127}).  Two phases per K-tile, 16 MFMAs each:
//   phase 0: read A (own 64 rows, kept for phase 1) + Bh0; restage A0 + Bh0 of K-tile kt+2
//   phase 1: read Bh1; restage A1 + Bh1 of K-tile kt+2; vmcnt: K-tile kt+1 landed
// in a three-slot ring (144 KB): K-tile kt+2 reuses the slot of K-tile kt-1,
// whose pieces were last read two phases before their restaging phase (WAR
// for the template-form waits: fragment reads are waited for after the
// phase's first barrier), and K-tile kt+1 is read one phase after the wait
// that retires it (RAW).  Every phase:
//   ds_reads; DMAs; [drain chunk]; [vmcnt]; s_barrier; lgkmcnt(0); 16 MFMA; s_barrier
// with the two M-groups staggered by one barrier (ping-pong).  The wait count
// is 6 (two phases of 3 DMAs) plus the drain stores and the bias DMA that sit
// between K-tile kt+1's last DMA and the wait.
// DMAs are buffer-descriptor loads (gemm_8q.hip): lane row offsets fixed for
// the kernel, the tile origin in the descriptor base, rows past M out of its
// range (zeros); stores likewise (rows past M dropped).  Persistent: one
// workgroup per CU walks XCD-contiguous tiles; the DMA cursor runs two
// K-tiles ahead across tile boundaries.  A tile's first MFMA into each
// accumulator takes C = 0 (no zeroing pass).  Arithmetic per output element is
// gemm_8p's (same k order, bias added after the sum), so results are bit-identical.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int BM = 256, BN = 128, BK = 64;
constexpr int PA = 128 * BK * 2;   // 16 KB A piece (128 image rows)
constexpr int PB = 64 * BK * 2;    // 8 KB B piece (64 image rows)
constexpr int KT = 2 * PA + 2 * PB;   // 48 KB K-tile slot
constexpr int OFF_A0 = 0, OFF_A1 = PA, OFF_B0 = 2 * PA, OFF_B1 = 2 * PA + PB;
constexpr int NSLOT = 3;
constexpr int NCHUNK = 8;   // 16 x 32 drain chunks per wave tile

__device__ __forceinline__ f32x2 quick_gelu2_8r(f32x2 v) {
  const f32x2 t = v * (f32x2){-2.45546696f, -2.45546696f};   // -1.702 * log2(e)
  f32x2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  e = e + 1.0f;
  return v * (f32x2){__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}

__device__ __forceinline__ void tile_coords_8r(int t, int tiles_n, int& mb, int& nb) {
  mb = t / tiles_n;
  nb = t % tiles_n;
}

template <bool V>
struct BC8r {
  static constexpr bool value = V;
};

// ABL (timing probes): 2 = no MFMAs, 4 = no drain work (accumulators kept live)
template <int EPI, int ABL = 0>
__global__ __launch_bounds__(512) void gemm_8r_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * KT + 2 * BN * 4];
  float* sbias = (float*)(smem + NSLOT * KT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1, grp = wave >> 2;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int nkt = a.K / BK;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntiles) return;

  auto coords = [&](int v, int& mm, int& nn) {
    int mb, nb;
    tile_coords_8r(xcd_remap(v, ntiles), tiles_n, mb, nb);
    mm = mb * BM;
    nn = nb * BN;
  };

  // ---- DMA cursor: K-tile dk of tile dv (origin dm0, dn0) into ring slot dslot
  int dv = blockIdx.x, dk = 0, dslot = 0, dm0, dn0;
  coords(dv, dm0, dn0);
  const int drow = lane >> 3;
  const int c0 = (lane & 7) ^ (lane >> 4), c1 = (lane & 7) ^ (4 + (lane >> 4));
  uint32_t voA[2][2], voB;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ir = (2 * wave + j) * 8 + drow;   // image row 0..127 of an A piece
    const int c = j ? c1 : c0;
#pragma unroll
    for (int p = 0; p < 2; ++p) voA[p][j] = (uint32_t)((p * 128 + ir) * a.lda * 2 + c * 16);
  }
  {
    const int ir = wave * 8 + drow;   // image row 0..63 of a B piece
    const int c = (wave & 1) ? c1 : c0;
    voB = (uint32_t)(((ir >> 5) * 64 + (ir & 31)) * a.ldw * 2 + c * 16);
  }
  const int bh1_sofs = 32 * (int)a.ldw * 2;
  __amdgpu_buffer_rsrc_t rsA, rsW;
  auto make_rs = [&]() {
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(a.A + (int64_t)dm0 * a.lda), (short)0,
                                            min(a.M - dm0, BM) * (int)a.lda * 2, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(a.W + (int64_t)dn0 * a.ldw), (short)0, BN * (int)a.ldw * 2, 0x00020000);
  };
  make_rs();
  // pieces h of the cursor's K-tile: h = 0: A0 + Bh0, h = 1: A1 + Bh1 (3 DMAs per thread)
  auto issue = [&](int h) {
    char* sb = smem + dslot * KT;
    const int kb = dk * BK * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (LDS_AS void*)(sb + (h ? OFF_A1 : OFF_A0) + (2 * wave + j) * 1024), 16,
                                               voA[h][j], kb, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (LDS_AS void*)(sb + (h ? OFF_B1 : OFF_B0) + wave * 1024), 16, voB,
                                             kb + (h ? bh1_sofs : 0), 0, 0);
  };
  auto advance = [&]() {
    dslot = dslot == NSLOT - 1 ? 0 : dslot + 1;
    if (++dk == nkt) {
      dk = 0;
      dv += G;
      if (dv < ntiles) {   // past the end: keep re-loading the last tile's valid rows
        coords(dv, dm0, dn0);
        make_rs();
      }
    }
  };

  // ---- fragment side
  const int fr = lane & 15, fq = lane >> 4, g = fq;
  const int rd0 = fr * 128 + (((0 + fq) ^ (fr >> 1)) << 4);   // k 0..31 of the K-tile
  const int rd1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);   // k 32..63
  const int a_off = (wr >> 1 ? OFF_A1 : OFF_A0) + (wr & 1) * 64 * 128;
  bf16x8 fa[4][2], fb[2][2];
  f32x4 acc[4][4], pend[4][4];
  float4 bpend[4];

  // ---- drain (the previous tile): chunk c = (mi, p): fragments ni = 2p, 2p + 1 of row block mi
  typedef unsigned int u32x4_8r __attribute__((ext_vector_type(4)));
  const uint32_t voO = (uint32_t)(((wr * 64 + fr) * a.ldo + wc * 64 + (g & 1) * 16 + (g >> 1) * 8) * 2);
  const uint32_t blkO = (uint32_t)(16 * a.ldo * 2);
  int pm0 = 0, pn0 = 0;
  __amdgpu_buffer_rsrc_t rsO;
  auto drain = [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    constexpr int mi = c >> 1, p = c & 1;
    if (ABL == 4) {
      asm volatile("" ::"v"(pend[mi][2 * p]), "v"(pend[mi][2 * p + 1]));
      return;
    }
    uint2 pk[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int ni = 2 * p + qq;
      f32x2 lo = (f32x2){pend[mi][ni][0], pend[mi][ni][1]} + (f32x2){bpend[ni].x, bpend[ni].y};
      f32x2 hi = (f32x2){pend[mi][ni][2], pend[mi][ni][3]} + (f32x2){bpend[ni].z, bpend[ni].w};
      if (EPI == EPI_GELU_BF16) {
        lo = quick_gelu2_8r(lo);
        hi = quick_gelu2_8r(hi);
      }
      pk[qq] = make_uint2(pack_bf16x2(lo), pack_bf16x2(hi));
    }
    const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
    const u32x4_8r d = {sx[0], sy[0], sx[1], sy[1]};
    __builtin_amdgcn_raw_buffer_store_b128(d, rsO, voO + mi * blkO + p * 64, 0, 0);
  };
  auto drain_rt = [&](int c) {   // runtime chunk index -> compile-time instance
    switch (c) {
      case 0: drain(std::integral_constant<int, 0>{}); break;
      case 1: drain(std::integral_constant<int, 1>{}); break;
      case 2: drain(std::integral_constant<int, 2>{}); break;
      case 3: drain(std::integral_constant<int, 3>{}); break;
      case 4: drain(std::integral_constant<int, 4>{}); break;
      case 5: drain(std::integral_constant<int, 5>{}); break;
      case 6: drain(std::integral_constant<int, 6>{}); break;
      default: drain(std::integral_constant<int, 7>{}); break;
    }
  };
  // bias of the finished tile (LDS slot par) -> registers, four reads under one wait,
  // invisible to the compiler (a plain LDS read makes hipcc drain the DMAs with vmcnt(0))
  auto load_bpend = [&](int par) {
    if (!a.bias) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bpend[ni] = make_float4(0.f, 0.f, 0.f, 0.f);
      return;
    }
    const uint32_t ba = (uint32_t)(uintptr_t)(const LDS_AS float*)(sbias + par * BN + wc * 64 + 4 * g);
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                 "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(bpend[0]), "=&v"(bpend[1]), "=&v"(bpend[2]), "=&v"(bpend[3]) : "v"(ba) : "memory");
  };

  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_section = [&](int nh, auto zc) {
    constexpr bool zero_c = decltype(zc)::value;
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if (ABL == 2) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) asm volatile("" ::"v"(fa[mi][0]), "v"(fa[mi][1]));
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) asm volatile("" ::"v"(fb[ni][0]), "v"(fb[ni][1]));
    } else if (nh == 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fb[ni][ks], fa[mi][ks], (zero_c && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][2 + ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fb[ni][ks], fa[mi][ks], (zero_c && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][2 + ni], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    barrier();
  };
  // s_waitcnt vmcnt(6 + extra) with extra in 0..3 (runtime, wave-uniform)
  auto wait_vm = [&](int extra) {
    if (extra == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (extra == 1) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else if (extra == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  };

  // ---- prologue: tile 0's bias, K-tiles 0 and 1
  {
    int m0, n0;
    coords(blockIdx.x, m0, n0);
    if (wave == 0 && a.bias && lane < 32) glds16(a.bias + n0 + lane * 4, sbias);   // 128 floats: lanes 0..31 x 16 B
  }
  issue(0);
  issue(1);
  advance();
  issue(0);
  issue(1);
  advance();
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  barrier();
  if (grp == 1) barrier();   // stagger the two M-groups by one barrier

  int kslot = 0;         // ring slot of the K-tile being computed
  int sprev = 0;         // drain stores issued in the previous K-tile (behind its last DMAs)
  bool has_prev = false;
  int par = 0;           // bias slot of the tile being computed
  for (int v = blockIdx.x; v < ntiles; v += G) {
    int cm0, cn0;
    coords(v, cm0, cn0);
    for (int kt = 0; kt < nkt; ++kt) {
      const char* sb = smem + kslot * KT;
      const bool first = kt == 0;
      // ---- phase 0: A + Bh0
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        fa[mi][0] = *(const bf16x8*)(sb + a_off + mi * 16 * 128 + rd0);
        fa[mi][1] = *(const bf16x8*)(sb + a_off + mi * 16 * 128 + rd1);
      }
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        fb[ni][0] = *(const bf16x8*)(sb + OFF_B0 + (wc * 32 + ni * 16) * 128 + rd0);
        fb[ni][1] = *(const bf16x8*)(sb + OFF_B0 + (wc * 32 + ni * 16) * 128 + rd1);
      }
      __builtin_amdgcn_sched_barrier(0);
      // this tile's bias (not tile 0's: the prologue loaded it), ahead of the DMAs
      int bias_dma = 0;
      if (first && v != (int)blockIdx.x && wave == 0 && a.bias) {
        if (lane < 32) glds16(a.bias + cn0 + lane * 4, sbias + par * BN);
        bias_dma = 1;
      }
      issue(0);
      __builtin_amdgcn_sched_barrier(0);
      if (first && has_prev) {   // the finished tile's accumulators move to the drain set
        load_bpend(par ^ 1);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) pend[mi][ni] = acc[mi][ni];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (first) mfma_section(0, BC8r<true>{});
      else mfma_section(0, BC8r<false>{});
      // ---- phase 1: Bh1
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        fb[ni][0] = *(const bf16x8*)(sb + OFF_B1 + (wc * 32 + ni * 16) * 128 + rd0);
        fb[ni][1] = *(const bf16x8*)(sb + OFF_B1 + (wc * 32 + ni * 16) * 128 + rd1);
      }
      __builtin_amdgcn_sched_barrier(0);
      issue(1);
      advance();
      __builtin_amdgcn_sched_barrier(0);
      int scur = 0;
      if (has_prev && kt < NCHUNK) {
        drain_rt(kt);
        scur = 1;
      }
      __builtin_amdgcn_sched_barrier(0);
      // K-tile kt + 1 landed: younger than its last DMA are the previous K-tile's drain
      // store, this K-tile's bias DMA, 2 x 3 DMAs and this K-tile's drain store
      wait_vm(sprev + bias_dma + scur);
      sprev = scur;
      if (first) mfma_section(1, BC8r<true>{});
      else mfma_section(1, BC8r<false>{});
      kslot = kslot == NSLOT - 1 ? 0 : kslot + 1;
    }
    // the finished tile becomes the drain set at the next tile's first K-tile
    pm0 = cm0;
    pn0 = cn0;
    rsO = __builtin_amdgcn_make_buffer_rsrc((void*)((uint16_t*)a.out + (int64_t)pm0 * a.ldo + pn0), (short)0,
                                            min(a.M - pm0, BM) * (int)a.ldo * 2, 0x00020000);
    has_prev = true;
    par ^= 1;
  }
  if (grp == 0) barrier();   // the M-groups' barrier counts meet
  // the last tile: drain all of it
  load_bpend(par ^ 1);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) pend[mi][ni] = acc[mi][ni];
  drain(std::integral_constant<int, 0>{});
  drain(std::integral_constant<int, 1>{});
  drain(std::integral_constant<int, 2>{});
  drain(std::integral_constant<int, 3>{});
  drain(std::integral_constant<int, 4>{});
  drain(std::integral_constant<int, 5>{});
  drain(std::integral_constant<int, 6>{});
  drain(std::integral_constant<int, 7>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing (dummy) DMAs land before the LDS is released
}

}  // namespace

int gemm_8r_ok(const GemmArgs& a) {
  return a.N % BN == 0 && a.K % BK == 0 && a.K >= NCHUNK * BK && a.M >= BM && !a.group && !a.patch_R &&
         (int64_t)BM * a.lda * 2 < (1LL << 31) && (int64_t)BN * a.ldw * 2 < (1LL << 31) &&
         (int64_t)BM * a.ldo * 2 < (1LL << 31) && (int64_t)(BM + 128) * a.lda * 2 < (1LL << 32);
}

// mode: 0 = default, 2 = no-MFMA probe, 4 = no-drain probe
hipError_t gemm_8r(const GemmArgs& a, int epi, hipStream_t s, int cus, int mode) {
  const int nt = ((a.M + BM - 1) / BM) * (a.N / BN);
  const int grid = nt < cus ? nt : cus;
#define L8R(E, ABL_) hipLaunchKernelGGL((gemm_8r_kernel<E, ABL_>), dim3(grid), dim3(512), 0, s, a)
#define L8R_ALL(E)                 \
  if (mode == 0) L8R(E, 0);        \
  else if (mode == 2) L8R(E, 2);   \
  else if (mode == 4) L8R(E, 4);   \
  else return hipErrorInvalidValue;
  if (epi == EPI_GELU_BF16) {
    L8R_ALL(EPI_GELU_BF16)
  } else if (epi == EPI_BF16) {
    L8R_ALL(EPI_BF16)
  } else {
    return hipErrorInvalidValue;
  }
#undef L8R_ALL
#undef L8R
  return hipGetLastError();
}

}  // namespace miclip
