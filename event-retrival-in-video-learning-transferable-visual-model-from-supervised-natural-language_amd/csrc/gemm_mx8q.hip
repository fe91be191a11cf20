// MX-fp8 GEMM on gemm_8q's 8-phase persistent schedule (gfx950), the vision
// tower of weights="fp8" (BASELINE.json configs[4], ViT-L/14@336px).  A/B only
// (MICLIP_GEMM_VARIANT=8 / mi_op_gemm_mx variant 8): bit-identical to the 16x16x128
// kernel but 8-30 % slower than the ping-pong kernel at the L/14@336 shapes
// (scripts/gemm_mx_micro.py: qkv 489 vs 446 us, fc 670 vs 627, c_proj 578 vs 453):
// at fp8 rate a K = 1024 tile's MFMAs take half the bf16 time while the epilogue
// placed between tiles does not shrink.
//
//   C[M,N] = (A[M,K] * 2^sa) . (W[N,K] * 2^sw)^T  (+ bias, QuickGELU)
//
// A K-tile is 128 k of e4m3 = 128 bytes per row, so the LDS image, the
// half-tile DMAs (128 rows x 128 B = 16 KB), the descriptor addressing, the
// phase table, the template-form waits and the epilogue placement are
// gemm_8q.hip's byte for byte (see its header).  What differs:
//  * one v_mfma_scale_f32_16x16x128_f8f6f4 per (mi, ni) and K-tile: 8 MFMAs
//    of 2x the cycles of a 16x16x32 bf16 per phase, the same 256 MFMA cycles
//    per phase at twice the FLOPs per staged byte.  Operands as gemm_mx.hip's
//    16x16x128 kernel (lane l: row l & 15, k = 32 (l >> 4) .. +31 = 16-byte
//    chunks 2g, 2g + 1 of the row), so the k order and the results are
//    bit-identical to it (tests/test_gpu_mx.py);
//  * the e8m0 scales (one per 64 k per row; stage-major [K/128][rows_pad][2],
//    gemm_mx.hip) of a K-tile, 512 B for the 256 A rows + 512 B for the 256 W
//    rows, ride one dword LDS-DMA per wave (waves 4-7 repeat waves 0-3's).
//    Every phase of a buffer reads scales, so the scale block is restaged two
//    phases after its last read by either M-group (the half-tiles' WAR rule):
//    even in phase 6, odd in phase 2, or in phase 1 of a tile's first pair
//    (the last pair skips phase 8's re-read, so phase 7 read them last), where
//    it goes ahead of the previous tile's epilogue stores.  Each is older than
//    the DMAs its K-tile's wait leaves in flight: gemm_8q's wait thresholds;
//  * epilogues: bf16 (+ QuickGELU) as gemm_8q, and EPI_GELU_MX (c_fc -> c_proj):
//    a wave's 64 columns of a row are one 64-k block of the consumer, so the
//    block max is the lane's 16 values then xor 16 / 32 across the lane groups;
//    e4m3 dword and scale-byte stores go through descriptors whose range drops
//    rows past M (and the scale stores of lanes 16-63), with no branch, so the
//    store count the phase-4 wait allows for is exact.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int BM = 256, BN = 256, BKB = 128;   // K-tile: 128 e4m3 = 128 bytes per row
constexpr int HALF = 128 * BKB;                 // 16 KB half-tile
constexpr int BUF = 4 * HALF;                   // 64 KB K-tile buffer
constexpr int SCB = 1024;                       // a K-tile's scales: 256 A + 256 W rows x 2 B
constexpr int H_A0 = 0, H_B0 = 1, H_B1 = 2, H_A1 = 3;

typedef int v8i_q __attribute__((ext_vector_type(8)));
typedef int v4i_q __attribute__((ext_vector_type(4)));

// QuickGELU exactly as gemm_mx.hip's mx_gelu (the MX kernels' results stay bit-identical)
__device__ __forceinline__ float quick_gelu_mx(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v)); }
__device__ __forceinline__ f32x2 quick_gelu2_mx(f32x2 v) { return (f32x2){quick_gelu_mx(v.x), quick_gelu_mx(v.y)}; }

// lane id through asm: opaque to CSE/LICM, so values derived from it are rebuilt where used
__device__ __forceinline__ int mx8q_lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// byte offset of this lane's 16-byte DMA piece j of a half-tile (gemm_8q's image: image row
// (2 wave + j) * 8 + lane / 8, 16-byte slot permuted on the source)
__device__ __forceinline__ uint32_t mx8q_dma_off(int wave, int j, bool wside, int ld) {
  const int l = mx8q_lane_id();
  const int ir = (2 * wave + j) * 8 + (l >> 3);
  const int c = (l & 7) ^ ((j ? 4 : 0) + (l >> 4));
  const int row = wside ? (ir >> 5) * 64 + (ir & 31) : (ir >> 6) * 128 + (ir & 63);
  return (uint32_t)(row * ld + c * 16);
}

template <int P>
struct PhMx {
  static constexpr int value = P;
};
template <bool V>
struct BoolMx {
  static constexpr bool value = V;
};

// stores a tile's epilogue leaves in flight into the next tile's phase 4 (per wave)
template <int EPI>
struct EpiStores {
  static constexpr int value = EPI == EPI_GELU_MX ? 8 * 4 + 8 : 16;
};

template <int EPI>
__global__ __launch_bounds__(512) void gemm_mx8q_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 2 * SCB + 2 * BN * 4];
  char* ssc = smem + 2 * BUF;                       // [2][SCB]
  float* sbias = (float*)(smem + 2 * BUF + 2 * SCB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int npairs = a.K / (2 * BKB);
  const int G = gridDim.x;
  const int m_pad = (a.M + 1) & ~1;
  if ((int)blockIdx.x >= ntiles) return;
  const uint8_t* A8 = (const uint8_t*)a.A;
  const uint8_t* W8 = (const uint8_t*)a.W;

  auto coords = [&](int v, int& mm, int& nn) {
    const int t = xcd_remap(v, ntiles);
    mm = (t / tiles_n) * BM;
    nn = (t % tiles_n) * BN;
  };

  // ---- restage cursor: K-tile pair rpp of tile rv (origin rm0, rn0)
  int rv = blockIdx.x, rpp = 0, rm0, rn0;
  coords(rv, rm0, rn0);
  // Per-lane DMA offsets, rebuilt at each issue from an opaque lane id (a few VALU in the memory
  // section) instead of 4 VGPRs held for the kernel's life: at 256 VGPRs hipcc otherwise spills
  // them and reloads them with vmcnt(0) ahead of a DMA, draining the stream.  A_m1 rows sit 64
  // rows below A_m0's and B_n1's 32 below B_n0's (soffset).
  auto lane_id = []() { return mx8q_lane_id(); };
  auto dma_off = [&](int j, bool wside_) { return mx8q_dma_off(wave, j, wside_, wside_ ? (int)a.ldw : (int)a.lda); };
  const int a1_sofs = 64 * (int)a.lda;
  const int b1_sofs = 32 * (int)a.ldw;
  __amdgpu_buffer_rsrc_t rsA, rsW;
  auto make_rs = [&]() {
    const int rows = min(a.M - rm0, BM);
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(A8 + (int64_t)rm0 * a.lda), (short)0, rows * (int)a.lda, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(W8 + (int64_t)rn0 * a.ldw), (short)0, BN * (int)a.ldw, 0x00020000);
  };
  make_rs();
  auto advance = [&]() {
    if (++rpp == npairs) {
      rpp = 0;
      rv += G;
      if (rv < ntiles) {
        coords(rv, rm0, rn0);
        make_rs();
      }
    }
  };
  auto issue = [&](int h, int b) {
    const int kofs = (2 * rpp + b) * BKB;
    char* dst = smem + b * BUF + h * HALF + (2 * wave) * 1024;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool ws = !(h == H_A0 || h == H_A1);
      const uint32_t vo = dma_off(j, ws);
      if (!ws)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (LDS_AS void*)(dst + j * 1024), 16, vo,
                                                 kofs + (h == H_A1 ? a1_sofs : 0), 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (LDS_AS void*)(dst + j * 1024), 16, vo,
                                                 kofs + (h == H_B1 ? b1_sofs : 0), 0, 0);
    }
  };
  // scales of K-tile (2 rpp + b) into ssc[b]: wave w & 3 moves 256 B (waves 0-1 A rows, 2-3 W rows)
  // through a descriptor over the whole scale tensor (rows past the padded M read the next stage's
  // bytes or, past the end, zeros: they only feed output rows past M); lane offset fixed, the
  // (K-tile, tile row) offset in soffset
  const bool wside = (wave & 2) != 0;
  const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(wside ? a.w_scale : a.a_scale), (short)0,
      (int)((int64_t)(a.K / BKB) * (wside ? a.N : m_pad) * 2), 0x00020000);
  auto issue_sc = [&](int b) {
    const int kt = 2 * rpp + b;
    const int so = (wside ? (kt * a.N + rn0) * 2 : (kt * m_pad + rm0) * 2) + (wave & 1) * 256;
    // (the operands as locals: a call inside the builtin's argument list made hipcc's host pass
    // drop this kernel's launch stubs)
    const uint32_t vo = (uint32_t)lane_id() * 4;
    const int sof = __builtin_amdgcn_readfirstlane(so);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsS, (LDS_AS void*)(ssc + b * SCB + (wave & 3) * 256), 4, vo, sof, 0, 0);
  };

  // ---- fragment side: lane (fr, g) reads 16-byte chunks 2g, 2g + 1 of row fr (k = 32 g .. +31)
  // (the read offsets are rebuilt per phase from the opaque lane id, like the DMA offsets)
  int rd0 = 0, rd1 = 0, sro = 0;
  auto frag_offsets = [&]() {
    const int l = lane_id(), lfr = l & 15, lfq = l >> 4;
    rd0 = lfr * 128 + (((2 * lfq) ^ (lfr >> 1)) << 4);
    rd1 = lfr * 128 + (((2 * lfq + 1) ^ (lfr >> 1)) << 4);
    sro = lfr * 2 + (lfq & 1);
  };
  auto frag = [&](const char* p, v8i_q& f) {   // straight into the operand tuple's halves
    v4i_q* h = (v4i_q*)&f;
    h[0] = *(const v4i_q*)(p + rd0);
    h[1] = *(const v4i_q*)(p + rd1);
  };
  // scale bytes: plain (compiler-visible) LDS byte loads, one per VGPR (opsel 0), at the lane's
  // row / k-block offset sro rebuilt per phase with the fragment offsets
  auto sbyte = [&](int off) -> int { return (int)*((const uint8_t*)ssc + off + sro); };
  v8i_q fa[4], fb0[2], fb1[2];
  int sa[4], sw0[2], sw1[2];
  auto read_a = [&](const char* half, auto bc, auto mhc) {
    constexpr int b = decltype(bc)::value, mh = decltype(mhc)::value;
    frag(half + (wr * 64) * 128, fa[0]);
    frag(half + (wr * 64 + 16) * 128, fa[1]);
    frag(half + (wr * 64 + 32) * 128, fa[2]);
    frag(half + (wr * 64 + 48) * 128, fa[3]);
    const int ao = b * SCB + wr * 256 + mh * 128;
    sa[0] = sbyte(ao);
    sa[1] = sbyte(ao + 32);
    sa[2] = sbyte(ao + 64);
    sa[3] = sbyte(ao + 96);
  };
  auto read_b = [&](const char* half, auto bc, auto nhc, v8i_q (&fb)[2], int (&sw)[2]) {
    constexpr int b = decltype(bc)::value, nh = decltype(nhc)::value;
    frag(half + (wc * 32) * 128, fb[0]);
    frag(half + (wc * 32 + 16) * 128, fb[1]);
    const int wo = b * SCB + 512 + wc * 128 + nh * 64;
    sw[0] = sbyte(wo);
    sw[1] = sbyte(wo + 32);
  };
  f32x4 acc[8][4];
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  int pm0 = 0, pn0 = 0, ppar = 0;
  bool has_prev = false;
  int nxt_n0 = 0, cpar = 0;
  bool has_next = false;

  typedef unsigned int u32x4_mx __attribute__((ext_vector_type(4)));
  // wait states after a store before its data registers can be rewritten: hipcc rewrote a
  // dwordx4 store's data with the very next VALU and lanes 12-15 / 44-47 of the stored dword 1
  // came out corrupt (scripts/mx8q_debug.py)
  auto store_gap = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 4");
    __builtin_amdgcn_sched_barrier(0);
  };
  // MX8Q_DRAIN probe: wait states between the last MFMAs and the epilogue's reads of their results
  auto mfma_drain = []() {
#ifdef MX8Q_DRAIN
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
    __builtin_amdgcn_sched_barrier(0);
#endif
  };
  // v_permlane*_swap reading a VGPR written by the VALU two instructions earlier (hipcc's spacing:
  // one s_nop) came out stale in lanes 12-15 / 44-47 of some rows (tests/test_gpu_mx.py); five
  // wait states between the producers and the swaps
  auto permlane_gap = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 4");
    __builtin_amdgcn_sched_barrier(0);
  };
  // the epilogue's per-lane offsets come from the opaque lane id too (used once per tile: held
  // for the kernel they are the first values hipcc spills)
  auto epilogue = [&]() {
    mfma_drain();
    const int el = lane_id(), efr = el & 15, eg = el >> 4;
    float4 bias[4];
    if (a.bias) {
      const uint32_t ba = (uint32_t)(uintptr_t)(const LDS_AS float*)(sbias + ppar * BN + wc * 64 + 4 * eg);
      asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                   "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(bias[0]), "=&v"(bias[1]), "=&v"(bias[2]), "=&v"(bias[3]) : "v"(ba) : "memory");
    } else {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bias[ni] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int rows = min(a.M - pm0, BM);
    if (EPI == EPI_GELU_MX) {
      // e4m3 out [M][ldo bytes], one dword per (mi, ni): row wr*128 + mi*16 + fr, cols wc*64 + ni*16 + 4g
      const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((uint8_t*)a.out + (int64_t)pm0 * a.ldo + pn0), (short)0, rows * (int)a.ldo, 0x00020000);
      // scale bytes: o_scale[((blk >> 1) * m_pad + m) * 2 + (blk & 1)], blk = the wave's 64-column block
      const int blk = (pn0 + wc * 64) >> 6;
      const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.o_scale + ((int64_t)(blk >> 1) * m_pad + pm0) * 2 + (blk & 1)), (short)0, rows * 2, 0x00020000);
      const uint32_t voD = (uint32_t)((wr * 128 + efr) * a.ldo + wc * 64 + 4 * eg);
      // lanes 0-15 store the row's scale byte; the others aim past the range (dropped, no branch)
      const uint32_t soS = eg == 0 ? (uint32_t)((wr * 128 + efr) * 2) : 0x7fff0000u;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        f32x2 v[4][2];
        float amax = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          v[ni][0] = quick_gelu2_mx((f32x2){acc[mi][ni][0], acc[mi][ni][1]} + (f32x2){bias[ni].x, bias[ni].y});
          v[ni][1] = quick_gelu2_mx((f32x2){acc[mi][ni][2], acc[mi][ni][3]} + (f32x2){bias[ni].z, bias[ni].w});
          amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[ni][0].x), fabsf(v[ni][0].y)), fmaxf(fabsf(v[ni][1].x), fabsf(v[ni][1].y))));
        }
        // max with lanes ^ 16 and ^ 32 by permlane swaps (no bpermute address registers)
        permlane_gap();
        const auto x16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(x16[0]), __uint_as_float(x16[1]));
        permlane_gap();
        const auto x32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(x32[0]), __uint_as_float(x32[1]));
        const int X = mx_block_exp(amax);
        const float inv = ldexpf(1.0f, -X);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
        {
          const uint32_t pk = mx_pack4(v[ni][0].x, v[ni][0].y, v[ni][1].x, v[ni][1].y, inv);
          const int sof = __builtin_amdgcn_readfirstlane(mi * 16 * (int)a.ldo + ni * 16);
          __builtin_amdgcn_raw_buffer_store_b32(pk, rsO, voD, sof, 0);
          store_gap();
        }
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(X + 127), rsS, soS, mi * 32, 0);
      }
      return;
    }
    const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((uint16_t*)a.out + (int64_t)pm0 * a.ldo + pn0), (short)0, rows * (int)a.ldo * 2, 0x00020000);
    const uint32_t voO = (uint32_t)(((wr * 128 + efr) * a.ldo + wc * 64 + (eg & 1) * 16 + (eg >> 1) * 8) * 2);
    const uint32_t blkO = (uint32_t)(16 * a.ldo * 2);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint2 pk[2];
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const int ni = 2 * p + qq;
          f32x2 lo = (f32x2){acc[mi][ni][0], acc[mi][ni][1]} + (f32x2){bias[ni].x, bias[ni].y};
          f32x2 hi = (f32x2){acc[mi][ni][2], acc[mi][ni][3]} + (f32x2){bias[ni].z, bias[ni].w};
          if (EPI == EPI_GELU_BF16) {
            lo = quick_gelu2_mx(lo);
            hi = quick_gelu2_mx(hi);
          }
          pk[qq] = make_uint2(pack_bf16x2(lo), pack_bf16x2(hi));
        }
        permlane_gap();
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
        const u32x4_mx d = {sx[0], sy[0], sx[1], sy[1]};
        const int sof = __builtin_amdgcn_readfirstlane((int)(mi * blkO + p * 64));
        __builtin_amdgcn_raw_buffer_store_b128(d, rsO, voO, sof, 0);
        store_gap();
      }
    }
  };

  auto phase = [&](auto pc, auto firstc, auto lastc) {
    constexpr int P = decltype(pc)::value;
    constexpr bool FIRST = decltype(firstc)::value, LAST = decltype(lastc)::value;
    constexpr int b = P <= 4 ? 0 : 1;
    constexpr int q = (P - 1) & 3;
    const char* rbuf = smem + b * BUF;
    if (P == 1) {
      // a tile's first pair: the odd K-tile's scales, oldest of the phase (older than the
      // previous tile's stores); the last pair read them last in phase 7 (no phase-8 re-read)
      if (FIRST) issue_sc(1);
      issue(H_A1, 1);
      if (FIRST) issue(H_B0, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (FIRST && has_prev) {
        epilogue();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (!(LAST && P == 8)) frag_offsets();
    if (q == 0) {
      read_a(rbuf + H_A0 * HALF, PhMx<b>{}, PhMx<0>{});
      read_b(rbuf + H_B0 * HALF, PhMx<b>{}, PhMx<0>{}, fb0, sw0);
    } else if (q == 1) {
      read_b(rbuf + H_B1 * HALF, PhMx<b>{}, PhMx<1>{}, fb1, sw1);
    } else if (q == 2) {
      read_a(rbuf + H_A1 * HALF, PhMx<b>{}, PhMx<1>{});
    } else if (!(LAST && P == 8)) {
      read_b(rbuf + H_B0 * HALF, PhMx<b>{}, PhMx<0>{}, fb0, sw0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (P == 2 && !FIRST) { issue_sc(1); issue(H_B0, 1); }   // two phases after phase 8's read
    if (P == 3) { advance(); issue(H_A0, 0); }
    if (P == 4) issue(H_B1, 0);
    if (P == 5) issue(H_A1, 0);
    if (P == 6) { issue_sc(0); issue(H_B0, 0); }   // the next pair's even scales, two phases after phase 4's read
    if (P == 7) issue(H_A0, 1);
    if (P == 8) issue(H_B1, 1);
    __builtin_amdgcn_sched_barrier(0);
    if (P == 4) {
      if (FIRST && has_prev) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + EpiStores<EPI>::value) : "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    if (P == 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    if (P == 8 && LAST && has_next && wave == 0 && a.bias)
      glds16(a.bias + nxt_n0 + lane_id() * 4, sbias + (cpar ^ 1) * BN);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    constexpr int mh = q >= 2 ? 1 : 0, nh = (q == 1 || q == 2) ? 1 : 0;
    auto& fb = nh ? fb1 : fb0;
    auto& sw = nh ? sw1 : sw0;
    // The MFMAs as inline asm accumulating in place (dst = srcC) and, on a tile's first K-tile,
    // into an early-clobber destination from C = 0.  Through the builtin hipcc gave the
    // block-scaled MFMA destinations inside its own dying srcA / srcB tuple, or retired srcC
    // early and reused its registers, and the results came out corrupt in lanes 12-15 / 44-47
    // (tests/test_gpu_mx.py, scripts/mx8q_debug.py).  The operands and results are consumed
    // phases later, behind barriers, so the hazards hipcc cannot see through the asm do not arise.
#define MX8Q_MFMA(MI, NI)                                                                                  \
  if (FIRST && P <= 4)                                                                                     \
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, 0, %3, %4"                                  \
                 : "=&v"(acc[mh * 4 + MI][nh * 2 + NI])                                                     \
                 : "v"(fb[NI]), "v"(fa[MI]), "v"(sw[NI]), "v"(sa[MI]));                                     \
  else                                                                                                     \
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4"                                 \
                 : "+v"(acc[mh * 4 + MI][nh * 2 + NI])                                                      \
                 : "v"(fb[NI]), "v"(fa[MI]), "v"(sw[NI]), "v"(sa[MI]))
    MX8Q_MFMA(0, 0); MX8Q_MFMA(0, 1); MX8Q_MFMA(1, 0); MX8Q_MFMA(1, 1);
    MX8Q_MFMA(2, 0); MX8Q_MFMA(2, 1); MX8Q_MFMA(3, 0); MX8Q_MFMA(3, 1);
#undef MX8Q_MFMA
    // pin the quadrant's MFMAs inside this section: without a use here hipcc sinks a tile's first
    // (C = 0) MFMAs into later phases, and the fragments they hold stay live (~350 VGPRs spilled)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) asm volatile("" : "+v"(acc[mh * 4 + mi][nh * 2 + ni]));
    // keep the operands live past the MFMAs: hipcc otherwise gives an MFMA a destination inside
    // its own dying srcA / srcB tuple (v[116:119] = mfma(v[112:119], ...)), which the block-scaled
    // MFMA does not tolerate (lanes 12-15 / 44-47 of the result came out corrupt)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) asm volatile("" ::"v"(fa[mi]));
    asm volatile("" ::"v"(fb[0]), "v"(fb[1]));
    __builtin_amdgcn_s_setprio(0);
    barrier();
  };
  auto pair = [&](auto firstc, auto lastc) {
    phase(PhMx<1>{}, firstc, lastc);
    phase(PhMx<2>{}, firstc, lastc);
    phase(PhMx<3>{}, firstc, lastc);
    phase(PhMx<4>{}, firstc, lastc);
    phase(PhMx<5>{}, firstc, lastc);
    phase(PhMx<6>{}, firstc, lastc);
    phase(PhMx<7>{}, firstc, lastc);
    phase(PhMx<8>{}, firstc, lastc);
  };

  // ---- prologue: tile 0's bias, the even K-tile's scales and halves, the odd A_m0 / B_n1 of pair 0
  {
    int m0, n0;
    coords(blockIdx.x, m0, n0);
    if (wave == 0 && a.bias) glds16(a.bias + n0 + lane * 4, sbias);
  }
  issue_sc(0);
  issue(H_A0, 0);
  issue(H_B1, 0);
  issue(H_A1, 0);
  issue(H_B0, 0);
  issue(H_A0, 1);
  issue(H_B1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  barrier();
  if (wr == 1) barrier();

  for (int v = blockIdx.x; v < ntiles; v += G) {
    int cm0, cn0;
    coords(v, cm0, cn0);
    has_next = v + G < ntiles;
    if (has_next) {
      int nm0;
      coords(v + G, nm0, nxt_n0);
    }
    pair(BoolMx<true>{}, BoolMx<false>{});
    for (int pp = 1; pp < npairs - 1; ++pp) pair(BoolMx<false>{}, BoolMx<false>{});
    pair(BoolMx<false>{}, BoolMx<true>{});
    pm0 = cm0;
    pn0 = cn0;
    ppar = cpar;
    has_prev = true;
    cpar ^= 1;
  }
  if (wr == 0) barrier();
  epilogue();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

int gemm_mx8q_ok(const GemmArgs& a, int epi) {
  return (epi == EPI_BF16 || epi == EPI_GELU_BF16 || (epi == EPI_GELU_MX && a.o_scale)) && a.N % BN == 0 &&
         a.K % (2 * BKB) == 0 && a.K >= 4 * BKB && a.M >= BM && !a.group && a.lda % 16 == 0 && a.ldw % 16 == 0 &&
         (int64_t)BM * a.lda < (1LL << 31) && (int64_t)BN * a.ldw < (1LL << 31) &&
         (int64_t)(BM + 64) * a.lda < (1LL << 32) && (int64_t)BM * a.ldo * 2 < (1LL << 31);
}

hipError_t gemm_mx8q(const GemmArgs& a, int epi, hipStream_t s, int cus) {
  const int nt = ((a.M + BM - 1) / BM) * (a.N / BN);
  const int grid = nt < cus ? nt : cus;
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_mx8q_kernel<EPI_BF16>, dim3(grid), dim3(512), 0, s, a); break;
    case EPI_GELU_BF16: hipLaunchKernelGGL(gemm_mx8q_kernel<EPI_GELU_BF16>, dim3(grid), dim3(512), 0, s, a); break;
    case EPI_GELU_MX: hipLaunchKernelGGL(gemm_mx8q_kernel<EPI_GELU_MX>, dim3(grid), dim3(512), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace miclip
