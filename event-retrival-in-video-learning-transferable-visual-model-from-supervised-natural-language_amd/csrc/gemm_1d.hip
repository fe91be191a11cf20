// LayerNorm-folded c_fc GEMM with a DEFERRED epilogue, one wave per SIMD (gfx950):
// C[M,N] = QuickGELU(rstd * (x16 . W'^T) - rstd * mean * s + c), bf16 out — c_fc of openai/CLIP's
// vision tower on gemm_8q.hip's LN-folded fp16 operands (EPI_LN_GELU_BF16).
// A/B only (MICLIP_8Q_F=1000, scripts/gemm_micro.py lnfc500).
//
// Why: on gemm_8q the epilogue of a 256 x 256 tile (two exponentials per value, stores) takes
// ~25 % of the tile, the main loop alone ran at 1530 TF against 1110 with it, and
// its two waves per SIMD hold 249 VGPRs, so a finished tile cannot stay live beside the next
// one.  Here one wave per SIMD gets 512 registers: a 256 x 128 tile, each wave 128 x 64 (128
// accumulators), and TWO accumulator sets.  Tile t accumulates into one set while the other
// set's values (tile t - 1) go through the epilogue one 16-row block per K-stage, between the
// stage's MFMAs (a wave issues vector work while its own MFMAs run: 16 cycles per 16x16x32
// MFMA, the epilogue needs ~2 instructions per MFMA).
//
// Stage = 64 k: A 256 rows x 128 B + W 128 rows x 128 B (48 KB), three stage buffers.  Per
// stage g (two 32-k steps, 32 MFMAs each, fragments double-buffered in registers):
//   [k-step 1 fragments of g read]  [k-step 0 MFMAs + columns 0-31 of epilogue block g]
//   wait: k-step 1 fragments, stage g + 1 landed (counted vmcnt), barrier
//   [stage g + 3 issued into g's buffer (+ the tile's LN vectors at its stage 0)]
//   [k-step 0 fragments of stage g + 1 read]  [k-step 1 MFMAs + columns 32-63, the block's stores]
// LDS images, DMA permutation, k order of the MFMA chain (C = 0 at a tile's first k-step)
// and the epilogue's arithmetic are gemm_8q's, so the output is bit-identical to it.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int D_BM = 256, D_BN = 128, D_BK = 64, D_NS = 3;
#ifndef D_IL
#define D_IL 2   // vector instructions per MFMA slot in the epilogue stages
#endif
constexpr int D_ABYTES = D_BM * D_BK * 2;     // 32 KB
constexpr int D_STAGE = D_ABYTES + D_BN * D_BK * 2;   // 48 KB
constexpr int D_VEC = 2 * D_BN * 4 * 2 + 2 * D_BM * 8;   // bias, colv [2][BN]; rs [2][BM][2]
constexpr int D_LDS = D_NS * D_STAGE + D_VEC;

typedef _Float16 f16x8_d __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void tile_coords_d(int t, int tiles_m, int tiles_n, int ng, int& mb, int& nb) {
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

// QuickGELU in stage order over 4 pairs, "+ 1" as packed adds (gemm_8q quick_gelu_stage_8q's
// arithmetic per value: bit-identical whatever the group size)
__device__ __forceinline__ void quick_gelu8_d(f32x2 (&v)[4]) {
  float e[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 t = v[k] * (f32x2){-2.45546696f, -2.45546696f};
    e[2 * k] = t.x;
    e[2 * k + 1] = t.y;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) e[k] = __builtin_amdgcn_exp2f(e[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 p = (f32x2){e[2 * k], e[2 * k + 1]} + (f32x2){1.0f, 1.0f};
    e[2 * k] = p.x;
    e[2 * k + 1] = p.y;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) e[k] = __builtin_amdgcn_rcpf(e[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = v[k] * (f32x2){e[2 * k], e[2 * k + 1]};
}

// lane id through asm: opaque to CSE / LICM, so offsets derived from it are rebuilt where used
// instead of hoisted out of the tile loop and held (or spilled) for the kernel's life
__device__ __forceinline__ int lane_d() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

template <int N>
__device__ __forceinline__ void vmwait_d() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int ABL, int NST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_1d_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[D_LDS];
  float* sbias = (float*)(smem + D_NS * D_STAGE);   // [2][BN]
  float* scol = sbias + 2 * D_BN;                   // [2][BN]
  float* srs = scol + 2 * D_BN;                     // [2][BM][2]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = a.N / D_BN;
  const int tiles_m = (a.M + D_BM - 1) / D_BM;
  const int ntiles = tiles_m * tiles_n;
  constexpr int nst = NST;   // K / 64 (the stage sequence is unrolled)
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntiles) return;

  auto coords = [&](int v, int& mm, int& nn) __attribute__((always_inline)) {
    const int t = xcd_remap(v, ntiles);
    int mb, nb;
    tile_coords_d(t, tiles_m, tiles_n, a.ngroup, mb, nb);
    mm = mb * D_BM;
    nn = nb * D_BN;
  };

  // ---- DMA cursor: stage ls of tile lv (origin lm0, ln0); past the last tile it keeps
  // re-loading the last tile's stages (uniform counts; those buffers are never read)
  int lv = blockIdx.x, ls = 0, lm0, ln0;
  coords(lv, lm0, ln0);
  __amdgpu_buffer_rsrc_t rsA, rsW;
  auto make_rs = [&]() __attribute__((always_inline)) {
    const int rows = min(a.M - lm0, D_BM);
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(a.A + (int64_t)lm0 * a.lda), (short)0, rows * (int)a.lda * 2, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(a.W + (int64_t)ln0 * a.ldw), (short)0, D_BN * (int)a.ldw * 2, 0x00020000);
  };
  make_rs();
  // stage (lv, ls) into buffer `buf`: A rows 64 wave .. + 63 (8 x 1 KB), W rows 32 wave .. + 31 (4 x 1 KB)
  auto issue = [&](int buf) __attribute__((always_inline)) {
    char* dst = smem + buf * D_STAGE;
    const int kofs = ls * D_BK * 2;
    // per-lane source offsets from the opaque lane id (row 8 i + (l >> 3) of the operand, 16-byte
    // chunk (l & 7) ^ ((row >> 1) & 7)): VALU per DMA instead of 12 hoisted row offsets in SGPRs
    const int l = lane_d(), drow = l >> 3;
    const int ce = (l & 7) ^ (l >> 4), co = (l & 7) ^ (4 + (l >> 4));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = wave * 8 + j;
      const uint32_t vo = (uint32_t)((i * 8 + drow) * (int)a.lda * 2 + ((j & 1) ? co : ce) * 16);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (LDS_AS void*)(dst + i * 1024), 16, vo, kofs, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = wave * 4 + j;
      const uint32_t vo = (uint32_t)((i * 8 + drow) * (int)a.ldw * 2 + ((j & 1) ? co : ce) * 16);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (LDS_AS void*)(dst + D_ABYTES + i * 1024), 16, vo, kofs, 0, 0);
    }
    if (++ls == nst) {
      ls = 0;
      if (lv + G < ntiles) {
        lv += G;
        coords(lv, lm0, ln0);
        make_rs();
      }
    }
  };
  // the LN vectors of tile (m0, n0) into parity par: one DMA per wave (wave 0 bias, 1 colv, 2 / 3
  // rows 0-127 / 128-255 of rs); the 128-float vectors by lanes 0-31
  auto stage_vectors = [&](int m0, int n0, int par) __attribute__((always_inline)) {
    if (wave < 2) {
      if (lane < 32) {
        const float* src = (wave == 0 ? a.bias : a.colv) + n0;
        float* dst = (wave == 0 ? sbias : scol) + par * D_BN;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 512, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)dst, 16, (uint32_t)lane_d() * 16, 0, 0, 0);
      }
    } else {
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.rs + (int64_t)(m0 + (wave - 2) * 128) * 2), (short)0, 1024, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(srs + par * D_BM * 2 + (wave - 2) * 256), 16,
                                               (uint32_t)lane_d() * 16, 0, 0, 0);
    }
  };

  // ---- fragments: lane (fr, fq) reads row fr of a 16-row block, k 8 fq .. + 7 (k-step 0) or
  // 32 + 8 fq .. (k-step 1), slot permuted by (fr >> 1)
  auto rdof = [&](int ks) __attribute__((always_inline)) {
    const int l = lane_d(), lfr = l & 15, lfq = l >> 4;
    return lfr * 128 + (((4 * ks + lfq) ^ (lfr >> 1)) << 4);
  };
  bf16x8 fa0[8], fb0[4], fa1[8], fb1[4];
  // asm reads (one base VGPR per operand, the block in the offset field; compiler-visible reads
  // had their 24 per-buffer addresses hoisted and spilled), so their waits are explicit below
  auto read_frags = [&](int buf, int rd, bf16x8 (&fa)[8], bf16x8 (&fb)[4]) __attribute__((always_inline)) {
    const uint32_t b0 = (uint32_t)(uintptr_t)(LDS_AS char*)smem + (uint32_t)(buf * D_STAGE + rd);
    const uint32_t ba = b0 + (uint32_t)(wm * 128 * 128), bb = b0 + (uint32_t)(D_ABYTES + wn * 64 * 128);
    asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:2048\n\tds_read_b128 %2, %8 offset:4096\n\t"
                 "ds_read_b128 %3, %8 offset:6144\n\tds_read_b128 %4, %8 offset:8192\n\tds_read_b128 %5, %8 offset:10240\n\t"
                 "ds_read_b128 %6, %8 offset:12288\n\tds_read_b128 %7, %8 offset:14336"
                 : "=&v"(fa[0]), "=&v"(fa[1]), "=&v"(fa[2]), "=&v"(fa[3]), "=&v"(fa[4]), "=&v"(fa[5]), "=&v"(fa[6]),
                   "=&v"(fa[7])
                 : "v"(ba)
                 : "memory");
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:2048\n\tds_read_b128 %2, %4 offset:4096\n\t"
                 "ds_read_b128 %3, %4 offset:6144"
                 : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3])
                 : "v"(bb)
                 : "memory");
  };
#define D_FWAIT(N, FA, FB)                                                                                  \
  asm volatile("s_waitcnt lgkmcnt(" #N ")"                                                                  \
               : "+v"(FA[0]), "+v"(FA[1]), "+v"(FA[2]), "+v"(FA[3]), "+v"(FA[4]), "+v"(FA[5]), "+v"(FA[6]), \
                 "+v"(FA[7]), "+v"(FB[0]), "+v"(FB[1]), "+v"(FB[2]), "+v"(FB[3])                            \
               :                                                                                            \
               : "memory")
  auto barrier = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 accX[8][4], accY[8][4];
  // MFMAs of one k-step into acc (first: a tile's first k-step, C = 0)
  auto mfma_step = [&](f32x4 (&acc)[8][4], const bf16x8 (&fa)[8], const bf16x8 (&fb)[4], bool first) __attribute__((always_inline)) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(f16x8_d, fb[ni]), __builtin_bit_cast(f16x8_d, fa[mi]),
            first ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni], 0, 0, 0);
  };

  // ---- epilogue of 16-row block mi of the finished tile (pm0, pn0), vectors at parity pp:
  // gemm_8q's EPI_LN_GELU_BF16 with F_GSTAGE16 | F_GPK | F_FULL | F_ONT, wave (wm, wn) in place of
  // (wr, wc), in two halves: columns ni 0-1 (store piece p = 0) beside a stage's k-step 0 MFMAs,
  // ni 2-3 (p = 1), the whole-row exchange and the two stores beside its k-step 1 MFMAs
  int pm0 = 0, pn0 = 0, pp = 0;
  f32x4 ecol[2], ebias[2];
  f32x2 erab;
  u32x4_d dp0;   // the block's p = 0 piece, from half 0 to half 1
  // the half's LN vectors (asm LDS reads, issued before the 12 fragment reads: lgkmcnt(12) waits)
  auto epi_vectors = [&](int mi, int h) __attribute__((always_inline)) {
    const int l = lane_d(), fr = l & 15, fq = l >> 4;
    const uint32_t ba = (uint32_t)(uintptr_t)(const LDS_AS float*)(sbias + pp * D_BN + wn * 64 + 32 * h + 4 * fq);
    const uint32_t ca = (uint32_t)(uintptr_t)(const LDS_AS float*)(scol + pp * D_BN + wn * 64 + 32 * h + 4 * fq);
    const uint32_t ra = (uint32_t)(uintptr_t)(const LDS_AS float*)(srs + pp * D_BM * 2 + (wm * 128 + mi * 16 + fr) * 2);
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %5\n\t"
                 "ds_read_b128 %3, %5 offset:64"
                 : "=&v"(ebias[0]), "=&v"(ebias[1]), "=&v"(ecol[0]), "=&v"(ecol[1]) : "v"(ba), "v"(ca) : "memory");
    asm volatile("ds_read_b64 %0, %1" : "=v"(erab) : "v"(ra) : "memory");
  };
#define D_VWAIT(N)                                                                                         \
  asm volatile("s_waitcnt lgkmcnt(" #N ")"                                                                 \
               : "+v"(ebias[0]), "+v"(ebias[1]), "+v"(ecol[0]), "+v"(ecol[1]), "+v"(erab)                  \
               :                                                                                           \
               : "memory")
  // columns ni = 2 h, 2 h + 1 of block mi: LN affine, QuickGELU, bf16, permlane16 swap -> piece p = h
  auto epi_half = [&](const f32x4 (&acc)[8][4], const int mi, const int h) __attribute__((always_inline)) -> u32x4_d {
    f32x2 gw[4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ni = 2 * h + q;
      const f32x2 ar = (f32x2){erab.x, erab.x}, br = (f32x2){-erab.y, -erab.y};
      f32x2 lo = (f32x2){acc[mi][ni][0], acc[mi][ni][1]};
      f32x2 hi = (f32x2){acc[mi][ni][2], acc[mi][ni][3]};
      lo = ar * lo + (br * (f32x2){ecol[q].x, ecol[q].y} + (f32x2){ebias[q].x, ebias[q].y});
      hi = ar * hi + (br * (f32x2){ecol[q].z, ecol[q].w} + (f32x2){ebias[q].z, ebias[q].w});
      gw[2 * q] = lo;
      gw[2 * q + 1] = hi;
    }
    quick_gelu8_d(gw);
    const uint32_t x0 = pack_bf16x2(gw[0]), y0 = pack_bf16x2(gw[1]);
    const uint32_t x1 = pack_bf16x2(gw[2]), y1 = pack_bf16x2(gw[3]);
    const auto sx = __builtin_amdgcn_permlane16_swap(x0, x1, false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(y0, y1, false, false);
    return (u32x4_d){sx[0], sy[0], sx[1], sy[1]};
  };
  auto epi_first = [&](const f32x4 (&acc)[8][4], const int mi) __attribute__((always_inline)) {
    if (ABL == 4) {   // probe: accumulators kept live, no epilogue work
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) asm volatile("" ::"a"(acc[mi][ni]));
      return;
    }
    dp0 = epi_half(acc, mi, 0);
  };
  auto epi_second = [&](const f32x4 (&acc)[8][4], const int mi) __attribute__((always_inline)) {
    if (ABL == 4) return;
    const u32x4_d dp1 = epi_half(acc, mi, 1);
    // whole 128-B rows: lane fr < 8 keeps its p = 0 piece of row fr and takes row fr + 8's p = 0
    // piece for store 2; lane fr >= 8 takes row fr - 8's p = 1 piece for store 1 (gemm_8q F_FULL)
    const int l = lane_d(), fr = l & 15, fq = l >> 4;
    const bool top = fr < 8;
    u32x4_d s1, s2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dp0[e], 0x128, 0xf, 0xf, false);
      const uint32_t r1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dp1[e], 0x128, 0xf, 0xf, false);
      s1[e] = top ? dp0[e] : r1;
      s2[e] = top ? r0 : dp1[e];
    }
    const int rows = min(a.M - pm0, D_BM);
    const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((uint16_t*)a.out + (int64_t)pm0 * a.ldo + pn0), (short)0, rows * (int)a.ldo * 2, 0x00020000);
    const uint32_t voF =
        (uint32_t)(((wm * 128 + (fr & 7)) * a.ldo + wn * 64 + 8 * ((fq & 1) * 2 + (fq >> 1)) + 32 * (fr >> 3)) * 2);
    const uint32_t blk = (uint32_t)(mi * 16 * a.ldo * 2);
    __builtin_amdgcn_raw_buffer_store_b128(s1, rsO, voF + blk, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(s2, rsO, voF + blk + (uint32_t)(8 * a.ldo * 2), 0, 2);
  };

  // ---- prologue: tile 0's vectors, stages 0-2 in flight, stage 0 landed, its k-step 0 fragments
  {
    int m0, n0;
    coords(blockIdx.x, m0, n0);
    stage_vectors(m0, n0, 0);
  }
  issue(0);
  issue(1);
  issue(2);
  vmwait_d<24>();
  barrier();
  read_frags(0, rdof(0), fa0, fb0);

  int g = 0;   // global stage index (buffer g % 3)
  int cpar = 0;
  // one MFMA, then up to D_IL vector instructions (transcendentals included), 32 times: the
  // epilogue's VALU between the MFMAs instead of in runs that leave the matrix pipe idle
  auto interleave = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x402, D_IL, 0);
    }
  };
  // stage S of a tile (S = 10: any stage >= 10) into acc; HP: a previous tile exists, whose block
  // S (S < 8) is finished from prv beside this stage's MFMAs
  auto stage = [&](auto hp_c, auto s_c, f32x4 (&acc)[8][4], const f32x4 (&prv)[8][4], int cm0, int cn0) __attribute__((always_inline)) {
    constexpr bool HP = decltype(hp_c)::value;
    constexpr int S = decltype(s_c)::value;
    constexpr bool EPI = HP && S < 8;
    const int buf = g % 3;
    D_FWAIT(0, fa0, fb0);   // k-step 0 fragments (read one MFMA group ago)
    if (EPI) epi_vectors(S, 0);
    read_frags(buf, rdof(1), fa1, fb1);
    if (EPI) D_VWAIT(12);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(acc, fa0, fb0, S == 0);
    if (EPI) {
      epi_first(prv, S);
      interleave();
    }
    __builtin_amdgcn_sched_barrier(0);
    D_FWAIT(0, fa1, fb1);
    // stage g + 1 landed.  Younger than its DMAs (issued in the middle of stage g - 2): the tile's
    // vectors (issued after the DMAs of a tile's stage 0), the epilogue stores of stages g - 2 and
    // g - 1 (2 each, after their middles), stage g + 2's 12 DMAs
    if (!HP) {
      if (S == 1 || S == 2) vmwait_d<13>();
      else vmwait_d<12>();
    } else if (S == 0 || S >= 10) {
      vmwait_d<12>();
    } else if (S == 1) {
      vmwait_d<15>();
    } else if (S == 2) {
      vmwait_d<17>();
    } else if (S == 9) {
      vmwait_d<14>();
    } else {   // 3 .. 8
      vmwait_d<16>();
    }
    barrier();
    issue(buf);   // stage g + 3 into the buffer just read
    if (S == 0) stage_vectors(cm0, cn0, cpar);
    if (EPI) epi_vectors(S, 1);
    read_frags((g + 1) % 3, rdof(0), fa0, fb0);
    if (EPI) D_VWAIT(12);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(acc, fa1, fb1, false);
    if (EPI) {
      epi_second(prv, S);
      interleave();
    }
    __builtin_amdgcn_sched_barrier(0);
    ++g;
  };
  auto tile = [&](auto hp_c, f32x4 (&acc)[8][4], const f32x4 (&prv)[8][4], int cm0, int cn0) __attribute__((always_inline)) {
    stage(hp_c, std::integral_constant<int, 0>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 1>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 2>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 3>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 4>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 5>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 6>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 7>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 8>{}, acc, prv, cm0, cn0);
    stage(hp_c, std::integral_constant<int, 9>{}, acc, prv, cm0, cn0);
#pragma unroll
    for (int s = 10; s < NST; ++s) stage(hp_c, std::integral_constant<int, 10>{}, acc, prv, cm0, cn0);
    pm0 = cm0;
    pn0 = cn0;
    pp = cpar;
    cpar ^= 1;
  };
  auto drain = [&](const f32x4 (&acc)[8][4]) __attribute__((always_inline)) {   // the last tile's epilogue, no MFMAs beside it
#define D_DRAIN(MI)   \
  epi_vectors(MI, 0); \
  D_VWAIT(0);         \
  epi_first(acc, MI); \
  epi_vectors(MI, 1); \
  D_VWAIT(0);         \
  epi_second(acc, MI);
    D_DRAIN(0) D_DRAIN(1) D_DRAIN(2) D_DRAIN(3) D_DRAIN(4) D_DRAIN(5) D_DRAIN(6) D_DRAIN(7)
#undef D_DRAIN
  };
  using BF = std::integral_constant<bool, false>;
  using BT = std::integral_constant<bool, true>;
  // tiles of this workgroup: blockIdx.x + t G, t < mt; X holds the last finished tile at the loop head
  const int mt = (ntiles - (int)blockIdx.x + G - 1) / G;
  int cm0, cn0;
  coords(blockIdx.x, cm0, cn0);
  tile(BF{}, accX, accY, cm0, cn0);
  int t = 1;
  for (; t + 1 < mt; t += 2) {
    coords(blockIdx.x + t * G, cm0, cn0);
    tile(BT{}, accY, accX, cm0, cn0);
    coords(blockIdx.x + (t + 1) * G, cm0, cn0);
    tile(BT{}, accX, accY, cm0, cn0);
  }
  if (t < mt) {
    coords(blockIdx.x + t * G, cm0, cn0);
    tile(BT{}, accY, accX, cm0, cn0);
    drain(accY);
  } else {
    drain(accX);
  }
#undef D_VWAIT
#undef D_FWAIT
  vmwait_d<0>();   // trailing DMAs land before the workgroup's LDS is released; stores retire
}

}  // namespace

int gemm_1d_ok(const GemmArgs& a) {
  return a.a_f16 && a.rs && a.colv && a.bias && a.N % D_BN == 0 && a.K % D_BK == 0 && (a.K / D_BK == 12 || a.K / D_BK == 16) &&
         a.M >= D_BM && !a.group && !a.patch_R && (int64_t)D_BM * a.lda * 2 < (1LL << 31) &&
         (int64_t)D_BN * a.ldw * 2 < (1LL << 31) && (int64_t)D_BM * a.ldo * 2 < (1LL << 31);
}

// EPI_LN_GELU_BF16 only (A/B: MICLIP_8Q_F=1000; 1004 = the no-epilogue probe)
hipError_t gemm_1d(const GemmArgs& a0, int abl, hipStream_t s, int cus) {
  GemmArgs a = a0;
  if (!gemm_1d_ok(a)) return hipErrorInvalidValue;
  if (a.ngroup == 0) {   // n-tiles in groups whose weight panel is <= 2.4 MB (gemm_8q's rule)
    const int tn = a.N / D_BN;
    for (int ng = tn / 2; ng >= 6; --ng)
      if (tn % ng == 0 && (int64_t)ng * D_BN * a.K * 2 <= 2400000) {
        a.ngroup = ng;
        break;
      }
  }
  const int nt = ((a.M + D_BM - 1) / D_BM) * (a.N / D_BN);
  const int grid = nt < cus ? nt : cus;
  const int nst = a.K / D_BK;
  if (nst == 12 && abl == 4) hipLaunchKernelGGL((gemm_1d_kernel<4, 12>), dim3(grid), dim3(256), 0, s, a);
  else if (nst == 12) hipLaunchKernelGGL((gemm_1d_kernel<0, 12>), dim3(grid), dim3(256), 0, s, a);
  else if (nst == 16) hipLaunchKernelGGL((gemm_1d_kernel<0, 16>), dim3(grid), dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace miclip
