// bf16 MFMA GEMM, 8-phase interleaved ping-pong, second schedule (gfx950):
// C[M,N] = A[M,K] . W[N,K]^T (+ bias, QuickGELU), bf16 out — the tower GEMMs
// of openai/CLIP's encode_image / encode_text.
//
// Same tile geometry, LDS image and quadrant order as gemm_8p.hip (256 x 256
// tile, K staged 64 wide, 8 waves as 2 (M) x 4 (N), each wave 128 x 64 in
// four 64 x 32 quadrants, one quadrant x 64 k = 16 MFMAs per phase, two
// K-tile buffers, one iteration = 8 phases = 2 K-tiles).  Three changes,
// each measured against gemm_8p (scripts/gpu_8p_abl.sh ablations: there the
// no-MFMA build ran at 90 % of the full kernel's time, i.e. the memory
// sections, not the MFMAs, set the phase length):
//
// 1. Buffer-descriptor DMAs (buffer_load_dwordx4 ... lds).  Each lane's row
//    offsets inside a tile are fixed for the kernel's lifetime (6 VGPRs);
//    the tile origin lives in the descriptor base (rebuilt by scalar code
//    when the restage cursor changes tiles) and the k offset in soffset, so
//    a DMA costs one M0 write and the load — gemm_8p spends ~8 VALU (64-bit
//    multiply-adds) per DMA on the address.  Rows past M are out of the
//    descriptor's range (num_records = the tile's valid rows x row bytes)
//    and load zeros instead of a clamped row.
// 2. Template-form waits (cdna_hip_programming.md §5 "The 256² 8-phase
//    template"): a phase's fragment reads are waited for AFTER its first
//    barrier (lgkmcnt(0) at the head of the MFMA section), so their latency
//    overlaps the barrier instead of lengthening the memory section.  That
//    needs every half-tile restaged two phases after its last read (WAR),
//    so the issue table shifts by one phase and each K-tile is waited for
//    with vmcnt(4) (two phases of DMAs younger than it; Vm8q::YOUNGER):
//      phase  reads (buffer)      restages
//      1      even A_m0 + B_n0    odd  A_m1   (current pair)
//      2      even B_n1           odd  B_n0   (current pair)
//      3      even A_m1           even A_m0   (next pair; the cursor advances here)
//      4      even B_n0           even B_n1   + vmcnt(4): odd buffer landed
//      5      odd  A_m0 + B_n0    even A_m1
//      6      odd  B_n1           even B_n0
//      7      odd  A_m1           odd  A_m0   (next pair)
//      8      odd  B_n0           odd  B_n1   + vmcnt(4): even buffer landed
//    RAW: a buffer is read one phase after the wait that retires it (one
//    barrier more than the stagger needs).  WAR: a half-tile's last reader
//    (either M-group) has passed its lgkmcnt(0) before the barrier that
//    precedes the restaging section of both groups.
// 3. Epilogue: the previous tile's (bias, QuickGELU, bf16, permlane16-swapped
//    16-byte row stores) opens the next tile's first phase, behind that
//    phase's DMAs — which on a tile's first pair are BOTH odd half-tiles
//    (A_m1 and B_n0): the last pair does not re-read B_n0 in phase 8 (it keeps
//    phase 5's fragments), so B_n0's last read is three phases back.  The 16
//    stores are then younger than every DMA the first pair's phase-4 wait
//    needs (vmcnt(20) = Vm8q::FIRST_P4) and have until phase 8 to complete.  Stores go through
//    a descriptor whose range is the tile's valid rows (no per-store branch or
//    64-bit address math), the four bias reads share one wait, and a tile's
//    first MFMA into each accumulator takes C = 0 (no zeroing pass).
//    Measured alternatives: the epilogue split by quadrant over phases 1-4
//    (+12 % on fc500: each quadrant's VALU lengthens a memory section the
//    partner's 16 MFMAs cannot cover); a start stagger of half the workgroups
//    (+-1 %: the store cost is per CU, ~48 cycles per 1-KB store instruction,
//    not a chip-wide write burst; scripts/gemm_probe8q.py stamps).
// Result (scripts/gemm_micro.py, M = 500k, interleaved with v98 in one process):
// fc -4..-7 %, qkv -3..-4 %, proj -6 %, out +-3 %; bit-identical to gemm_8p.
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "internal.hpp"

namespace miclip {
namespace {

constexpr int BM = 256, BN = 256, BK8 = 64;
constexpr int HALF = 128 * BK8 * 2;   // 16 KB half-tile
constexpr int BUF = 4 * HALF;         // 64 KB K-tile buffer
constexpr int H_A0 = 0, H_B0 = 1, H_B1 = 2, H_A1 = 3;
// flags
constexpr int F_GLDS = 1;   // flat global_load_lds with per-DMA address math (gemm_8p's) instead of descriptors
constexpr int F_FULL = 2;   // epilogue stores of 8 whole 128-B rows (lane pairs fr, fr ^ 8 swap halves by DPP)
constexpr int F_VOREC = 4;  // epilogue store offsets recomputed from the lane id (EPI_RES16 always)
constexpr int F_GSTAGE = 8; // QuickGELU over a store's 8 values in stage order (quick_gelu8_8q)
constexpr int F_GSTAGE16 = 32;   // the same over a 16-row block's 16 values (A/B)
constexpr int F_ANT = 64;   // A-operand DMAs non-temporal (A/B: keep the weight panel in L2 against the A stream)
constexpr int F_ONT = 128;  // output stores non-temporal (A/B)
constexpr int F_GPK = 256;  // QuickGELU's "+ 1" as packed adds (v_pk_add_f32: 5.1 cycles per pair vs 4.7 per value)
// F_BEARLY: the lagging M-group (wr = 1) runs its epilogue right after its last MFMA section of
// the tile (the same barrier interval as the leading group's epilogue) instead of one interval
// later, so the two waves of each SIMD issue their epilogue VALU concurrently (two waves: 2x the
// plain-VALU and 1.37x the transcendental issue rate of one, scripts/probes/valu_rate.hip)
constexpr int F_BEARLY = 512;
// F_ODUP (EPI_SPLIT_GELU): the output split stored once, [y1 | y2] (GemmArgs o_dup).  A compile-time
// flag: the same choice as a runtime branch around the second y1 store made the in-loop epilogues of
// large grids produce non-finite rows at random (measured, scripts/gpu_r5zq.sh)
constexpr int F_ODUP = 1024;
// F_DYN (A/B): tiles handed out in order by a per-XCD counter instead of the static stride G, so
// the CUs that share an m-block's A rows (its n-tiles on consecutive CUs of one XCD) cannot drift
// apart over the launch: each CU takes the XCD's next unclaimed tile when it starts one.  The
// claim for the tile after next goes out at a tile's start (one lane's atomic, before phase 1's
// DMAs: older than the awaited K-tile, so the phase-4 wait retires it) and reaches the other waves
// through an LDS slot
constexpr int F_DYN = 2048;
// F_WARM (EPI_RES16, A/B): after the last pair's phase-4 wait each wave issues two 4-byte LDS-DMAs
// per lane into a throw-away LDS slot, one per 128-byte line of the tile's x16 rows (1024 lines
// over the 8 waves), so the epilogue's x16 loads five phases later find their lines in L2 (the
// probes put the x16 loads' exposed latency at ~100 us of resout500's ~710).  The two extra VMEM
// ops are older than every later wait's awaited DMAs, so those waits also retire them (vmcnt
// completes in order): correct, and four phases after their issue
constexpr int F_WARM = 4096;
__device__ unsigned g_dyn8q[8];   // F_DYN: per-XCD claim counters, zeroed before each launch

__device__ __forceinline__ f32x2 quick_gelu2_8q(f32x2 v) {
  const f32x2 t = v * (f32x2){-2.45546696f, -2.45546696f};   // -1.702 * log2(e)
  f32x2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  e = e + 1.0f;
  return v * (f32x2){__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}

// QuickGELU of 8 values in stage order (all multiplies, all exponentials, all adds, all
// reciprocals, all products), so consecutive transcendental ops are independent (F_GSTAGE)
// (PK: the adds as packed pairs -- the same additions, bit-identical; one wave alone issues a
// v_pk_add_f32 in 5.1 cycles against 4.7 for a v_add_f32, scripts/probes/valu_rate.hip)
template <int NP, bool PK = false>
__device__ __forceinline__ void quick_gelu_stage_8q(f32x2 (&v)[NP]) {
  float e[2 * NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const f32x2 t = v[k] * (f32x2){-2.45546696f, -2.45546696f};
    e[2 * k] = t.x;
    e[2 * k + 1] = t.y;
  }
#pragma unroll
  for (int k = 0; k < 2 * NP; ++k) e[k] = __builtin_amdgcn_exp2f(e[k]);
  if (PK) {
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const f32x2 p = (f32x2){e[2 * k], e[2 * k + 1]} + (f32x2){1.0f, 1.0f};
      e[2 * k] = p.x;
      e[2 * k + 1] = p.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 2 * NP; ++k) e[k] = e[k] + 1.0f;
  }
#pragma unroll
  for (int k = 0; k < 2 * NP; ++k) e[k] = __builtin_amdgcn_rcpf(e[k]);
#pragma unroll
  for (int k = 0; k < NP; ++k) v[k] = v[k] * (f32x2){e[2 * k], e[2 * k + 1]};
}
__device__ __forceinline__ void quick_gelu8_8q(f32x2 (&v)[4]) { quick_gelu_stage_8q<4>(v); }

// EPI_SPLIT_GELU's row exponent (gemm.hip split_exp_g): 2^e scales the row bound into [2^13, 2^14)
__device__ __forceinline__ int split_exp_8q(float mx) {
  if (!(mx > 0.f) || !__builtin_isfinite(mx)) return 0;
  int ex;
  (void)frexpf(mx, &ex);
  const int e = 14 - ex;
  return e > 126 ? 126 : (e < -126 ? -126 : e);
}

__device__ __forceinline__ void tile_coords_8q(int t, int tiles_m, int tiles_n, int ng, int& mb, int& nb) {
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

// timing probe (ABL 9, scripts/gemm_probe.py 8q): per workgroup and M-group, s_memtime stamps
// of its third tile (see the S* comments) + two s_memrealtime stamps for the clock
__device__ unsigned long long g_probe8q[1024 * 2 * 9];

template <int P>
struct Ph8q {
  static constexpr int value = P;
};
template <bool V>
struct BoolC {
  static constexpr bool value = V;
};

// ABL (timing probes): 2 = no MFMAs, 4 = no epilogue work (accumulators kept live), 9 = stamps
typedef _Float16 f16x8_8q __attribute__((ext_vector_type(8)));

template <int EPI>
struct EpiKind8q {
  static constexpr bool LN = EPI == EPI_LN_BF16 || EPI == EPI_LN_GELU_BF16;   // LayerNorm folded in (fp16 operands)
  static constexpr bool GELU = EPI == EPI_GELU_BF16 || EPI == EPI_LN_GELU_BF16;
  static constexpr bool RES = EPI == EPI_RES16_BF16;   // residual add + row partial statistics fused
  // split-f16 operands of the fp32 tower (split2h_rows; OPF16): f32 epilogues with the row / column
  // scales rsc[m] * csc[n] (EPI_F32: in_proj; EPI_RESID_F32: out_proj / c_proj into the f32
  // stream; EPI_SPLIT_GELU: c_fc's QuickGELU split into c_proj's operand), gemm.hip's arithmetic
  static constexpr bool SPL = EPI == EPI_F32 || EPI == EPI_RESID_F32 || EPI == EPI_SPLIT_GELU;
  // LDS: 2 K-tile buffers, bias [2][BN]; LN: + row statistics [2][BM][2] + column sums [2][BN];
  // SPL: + rsc / rmax [2][2][BM] in the row-statistics slot + csc [2][BN] in the column-sum slot
  static constexpr int LDS = 2 * BUF + 2 * BN * 4 + (LN || SPL ? 2 * BM * 8 + 2 * BN * 4 : 0);
};

// The kernel's counted waits (common.hpp vm_wait), every immediate derived from the VMEM ops the code
// issues.  VERDICT r5: a hand-kept immediate (60, the [y1 | y1 | y2] store count) outlived a change
// that issued 16 fewer epilogue stores per wave (o_dup), so the first pair's phase-4 wait released
// while up to 16 of the awaited K-tile's DMAs were in flight and stale LDS reached the MFMAs in the
// in-loop epilogues of large grids.  Now the epilogue counts the ops it issues and vm_count_check
// ties the count to EPI_VMEM at compile time (a mismatch fails the device link).
template <int EPI, int ABL, int F>
struct Vm8q {
  using EK = EpiKind8q<EPI>;
  static constexpr int DMA_PER_HALF = 2;   // issue(): two 1-KB DMAs per thread and half-tile
  // a phase-4 / phase-8 wait (and the prologue's) retires the K-tile whose last half-tile was
  // restaged before the two preceding phases; those two phases' half-tiles (3-4 / 7-8) are younger
  static constexpr int YOUNGER = 2 * DMA_PER_HALF;
  static constexpr int BLOCKS = 8;         // the epilogue's 16-row blocks (a wave's 128 rows)
  // the epilogue's VMEM ops per block, all issued after phase 1's DMAs (EPI_RES16's x16 loads go out
  // ahead of them, in phase 6 / ahead of phase 1's DMAs: older than the awaited K-tile, not counted)
  static constexpr int PER_BLOCK =
      ABL == 4 ? 0                                                 // probe: no epilogue work
      : EPI == EPI_F32 ? 4                                         // four f32 16-byte row pieces
      : EPI == EPI_RESID_F32 ? 4 + 4                               // the stream's four pieces (loaded a block ahead) + four stores
      : EPI == EPI_SPLIT_GELU ? 2 * ((F & F_ODUP) ? 2 : 3) + 1      // per column half p: y1 (, y1), y2; + rsc_out
      : EK::RES ? 2 + (ABL == 11 ? 0 : 1)                          // two row stores + the 64-column partial
      : (ABL == 10 && !(F & F_FULL)) ? 0                           // stamp probe without stores
      : 2;                                                         // two row stores (F_FULL: rows 0-7, 8-15)
  static constexpr int EPI_VMEM = BLOCKS * PER_BLOCK;
  // the first pair's phase-4 wait when the previous tile's epilogue ran in phase 1 (after that
  // phase's DMAs): the epilogue's ops are younger too.  Saturated at VM_MAX it over-waits (the oldest
  // epilogue ops retire with the K-tile): correct, only slower (EPI_RESID_F32: 64 + 4)
  static constexpr int FIRST_P4 = YOUNGER + EPI_VMEM < VM_MAX ? YOUNGER + EPI_VMEM : VM_MAX;
  static_assert(YOUNGER > 0 && YOUNGER <= VM_MAX && FIRST_P4 >= YOUNGER, "counted waits out of range");
};

template <int EPI, int ABL = 0, int F = 0, bool OPF16 = false>
__global__ __launch_bounds__(512) void gemm_8q_kernel(GemmArgs a) {
  using EK = EpiKind8q<EPI>;
  using VM = Vm8q<EPI, ABL, F>;
  __shared__ __attribute__((aligned(16))) char smem[EK::LDS + ((F & F_DYN) ? 16 : 0) + ((F & F_WARM) ? 256 : 0)];
  float* sbias = (float*)(smem + 2 * BUF);
  float* srs = (float*)(smem + 2 * BUF + 2 * BN * 4);              // LN: [2][BM][2]
  float* scol = (float*)(smem + 2 * BUF + 2 * BN * 4 + 2 * BM * 8);  // LN: [2][BN]
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
    tile_coords_8q(t, tiles_m, tiles_n, a.ngroup, mb, nb);
    mm = mb * BM;
    nn = nb * BN;
  };

  // F_DYN: this XCD's logical tile range [dxs, dxe) (xcd_remap's), tiles in logical order
  constexpr bool DYN = (F & F_DYN) != 0;
  const int dxcd = blockIdx.x & 7;
  const int dq = ntiles >> 3, dr = ntiles & 7;
  const int dxs = dxcd < dr ? dxcd * (dq + 1) : dr * (dq + 1) + (dxcd - dr) * dq;
  const int dxe = dxs + dq + (dxcd < dr ? 1 : 0);
  auto coords_l = [&](int t, int& mm, int& nn) {
    int mb, nb;
    tile_coords_8q(t, tiles_m, tiles_n, a.ngroup, mb, nb);
    mm = mb * BM;
    nn = nb * BN;
  };
  const uint32_t dyn_slot = (uint32_t)(uintptr_t)(const LDS_AS char*)(smem + EK::LDS);
  // claim the XCD's next tile: lane 0's atomic, in asm with exec = lane 0 (no branch): hipcc's own
  // waitcnt pass drained every VMEM op in flight right after a compiler-visible atomic.  The
  // caller retires it with a counted wait (an op older than the awaited DMAs: vmcnt retires in
  // order, and an op the compiler does not see only makes its own waits over-wait)
  auto dyn_claim = [&]() {
    unsigned got = 0;
    unsigned long long sv;
    const unsigned one = 1u;
    unsigned* ctr = &g_dyn8q[dxcd];
    asm volatile("s_mov_b64 %1, exec\n\ts_mov_b64 exec, 1\n\tglobal_atomic_add %0, %2, %3, off sc0\n\ts_mov_b64 exec, %1"
                 : "+v"(got), "=&s"(sv) : "v"(ctr), "v"(one) : "memory");
    return got;
  };
  auto dyn_publish = [&](unsigned got) {   // wave 0, after the wait that retired the claim
    asm volatile("" : "+v"(got));
    const int t = dxs + (G >> 3) + (int)__builtin_amdgcn_readlane(got, 0);
    asm volatile("ds_write_b32 %0, %1" ::"v"(dyn_slot), "v"(t) : "memory");
  };
  auto dyn_read = [&]() {
    int t;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(dyn_slot) : "memory");
    return __builtin_amdgcn_readfirstlane(t);
  };
  int dyn_next = 0;   // F_DYN: the tile after the current one (the restage cursor's next)
  unsigned dyn_got = 0;
  // ---- restage cursor: K-tile pair rpp of tile rv (origin rm0, rn0)
  int rv = DYN ? dxs + (int)(blockIdx.x >> 3) : (int)blockIdx.x, rpp = 0, rm0, rn0;
  if constexpr (DYN) coords_l(rv, rm0, rn0);
  else coords(rv, rm0, rn0);
  const int drow = lane >> 3;
  const int c0 = (lane & 7) ^ (lane >> 4), c1 = (lane & 7) ^ (4 + (lane >> 4));
  // per-lane byte offsets of this thread's two DMA rows in each half-tile
  // (image row ir = (2 * wave + j) * 8 + drow, 16-byte slot c permuted on the source)
  uint32_t voA0[2], voA1[2], voB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ir = (2 * wave + j) * 8 + drow;
    const int c = j ? c1 : c0;
    const int ra = (ir >> 6) * 128 + (ir & 63);
    voA0[j] = (uint32_t)(ra * a.lda * 2 + c * 16);
    voA1[j] = (uint32_t)((ra + 64) * a.lda * 2 + c * 16);
    voB[j] = (uint32_t)(((ir >> 5) * 64 + (ir & 31)) * a.ldw * 2 + c * 16);
  }
  const int b1_sofs = 32 * (int)a.ldw * 2;   // B_n1 rows sit 32 rows below B_n0's
  __amdgpu_buffer_rsrc_t rsA, rsW;
  auto make_rs = [&]() {
    const int rows = min(a.M - rm0, BM);
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(a.A + (int64_t)rm0 * a.lda), (short)0, rows * (int)a.lda * 2, 0x00020000);
    rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(a.W + (int64_t)rn0 * a.ldw), (short)0, BN * (int)a.ldw * 2, 0x00020000);
  };
  if (!(F & F_GLDS)) make_rs();
  auto advance = [&]() {
    if (++rpp == npairs) {
      rpp = 0;
      if constexpr (DYN) {
        rv = dyn_next;
        if (rv < dxe) {   // past the end: keep re-loading the last tile's valid rows
          coords_l(rv, rm0, rn0);
          make_rs();
        }
      } else {
        rv += G;
        if (rv < ntiles) {   // past the end: keep re-loading the last tile's valid rows
          coords(rv, rm0, rn0);
          if (!(F & F_GLDS)) make_rs();
        }
      }
    }
  };
  // one half-tile h of K-tile (2 * rpp + b) into buffer b: two 1-KB DMAs per thread
  auto issue = [&](int h, int b) {
    const int kofs = (2 * rpp + b) * BK8;
    char* dst = smem + b * BUF + h * HALF + (2 * wave) * 1024;
#pragma unroll
    for (int j = 0; j < VM::DMA_PER_HALF; ++j) {
      if (F & F_GLDS) {
        const int ir = (2 * wave + j) * 8 + drow;
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
      } else if (h == H_A0 || h == H_A1) {
        // (a_dup: the split operand's [x1 | x2] read as [x1 | x1 | x2]: K-tiles past a_dup from k - a_dup)
        const int ka = (a.a_dup && kofs >= a.a_dup) ? kofs - a.a_dup : kofs;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (LDS_AS void*)(dst + j * 1024), 16, h == H_A1 ? voA1[j] : voA0[j],
                                                 ka * 2, 0, (F & F_ANT) ? 2 : 0);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (LDS_AS void*)(dst + j * 1024), 16, voB[j],
                                                 kofs * 2 + (h == H_B1 ? b1_sofs : 0), 0, 0);
      }
    }
  };

  // per-tile vectors into LDS parity `par`: bias (wave 0); LN: column sums (wave 1) and the
  // tile's 256 rows of (rstd, rstd * mean) (waves 2, 3; rs is readable 256 rows past M)
  // (buffer-descriptor DMAs: the base is scalar, the lane offset lane * 16 -- no 64-bit
  // per-lane address kept live across the tile)
  auto dma_vec = [&](const float* base, float* lds, int bytes = 1024) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)lds, 16, (uint32_t)lane * 16, 0, 0, 0);
  };
  auto stage_vectors = [&](int m0, int n0, int par) {
    if (wave == 0 && a.bias) dma_vec(a.bias + n0, sbias + par * BN);
    if (EK::LN) {
      if (wave == 1) dma_vec(a.colv + n0, scol + par * BN);
      if (wave == 2) dma_vec(a.rs + (int64_t)m0 * 2, srs + par * BM * 2);
      if (wave == 3) dma_vec(a.rs + (int64_t)(m0 + 128) * 2, srs + par * BM * 2 + 256);
    }
    if (EK::SPL) {   // rows past M read zeros (the descriptor's range ends at row M)
      const int rb = min(a.M - m0, BM) * 4;
      if (wave == 1) dma_vec(a.csc + n0, scol + par * BN);
      if (wave == 2) dma_vec(a.rsc + m0, srs + par * BM * 2, rb);
      if (EPI == EPI_SPLIT_GELU && wave == 3) dma_vec(a.rmax + m0, srs + par * BM * 2 + BM, rb);
    }
  };

  // ---- fragment side
  const int fr = lane & 15, fq = lane >> 4, g = fq;
  const int rd0 = fr * 128 + (((0 + fq) ^ (fr >> 1)) << 4);   // k 0..31 of the K-tile
  const int rd1 = fr * 128 + (((4 + fq) ^ (fr >> 1)) << 4);   // k 32..63
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](const char* half) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const char* p = half + (wr * 64 + mi * 16) * 128;
      fa[mi][0] = *(const bf16x8*)(p + rd0);
      fa[mi][1] = *(const bf16x8*)(p + rd1);
    }
  };
  auto read_b = [&](const char* half, bf16x8 (&fb)[2][2]) {
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

  unsigned long long st[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int ti = 0;   // this workgroup's tile index
  auto stamp = [&](int i) {
    if ((ABL == 9 || ABL == 10) && ti == 2) {
      __builtin_amdgcn_sched_barrier(0);
      st[i] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // previous tile (its epilogue runs in this tile's phases 1-4)
  int pm0 = 0, pn0 = 0, ppar = 0;
  bool has_prev = false;
  int nxt_m0 = 0, nxt_n0 = 0, cpar = 0;
  bool has_next = false;

  // the previous tile's epilogue: bias (+ QuickGELU), bf16, permlane16-swapped
  // 16-byte row stores through a descriptor whose range is the tile's valid
  // rows (rows past M are dropped by the range check: no per-store branch),
  // each lane's row/column offset fixed for the kernel, the 16-row block in a
  // scalar multiple, the column half in the instruction offset
  typedef unsigned int u32x4_8q __attribute__((ext_vector_type(4)));
  const uint32_t voO = (uint32_t)(((wr * 128 + fr) * a.ldo + wc * 64 + (g & 1) * 16 + (g >> 1) * 8) * 2);
  const uint32_t blkO = (uint32_t)(16 * a.ldo * 2);
  // F_FULL: store 1 covers rows 0-7 of the 16-row block, store 2 rows 8-15, each row's 64
  // columns whole: lane (fr < 8) keeps its p = 0 piece of row fr and takes the p = 0 piece of
  // row fr + 8 for store 2; lane (fr >= 8) takes the p = 1 piece of row fr - 8 for store 1
  const uint32_t voF = (uint32_t)(((wr * 128 + (fr & 7)) * a.ldo + wc * 64 + 8 * ((g & 1) * 2 + (g >> 1)) + 32 * (fr >> 3)) * 2);
  const uint32_t rows8 = (uint32_t)(8 * a.ldo * 2);
  auto out_rsrc_at = [&](int m0, int n0) {
    const int rows = min(a.M - m0, BM);
    return __builtin_amdgcn_make_buffer_rsrc((void*)((uint16_t*)a.out + (int64_t)m0 * a.ldo + n0), (short)0,
                                             rows * (int)a.ldo * 2, 0x00020000);
  };
  auto out_rsrc = [&]() { return out_rsrc_at(pm0, pn0); };
  int cur_m0 = 0, cur_n0 = 0;   // the tile in the main loop (EPI_RES16: its x16 blocks 0-1 load in its last pair)
  // EPI_RES16: the x16 pieces a tile's epilogue stores over (16 bytes per lane and 16-row block),
  // loaded ahead so that no wait for them also waits for a DMA issued just before: blocks 0-1 at
  // the head of the tile's LAST pair's phase 6 (16 VGPRs live across phases 6-8), blocks 2-7 at
  // the head of the next tile's phase 1, AHEAD of that phase's DMAs (the fragment registers are
  // dead until phase 1's reads).  Rows past M read zeros (descriptor range) and are not stored.
  // Measured (scripts/gemm_micro.py resout500 / resproj500, profiles/r04_a[cdeq]_*): this order
  // 684 / 1833 us; blocks 0-3 before phase 1's DMAs and 4-7 behind them (each of those waits then
  // also waited for phase 1's DMAs) 702-724 / 1867-1890 us; all eight before phase 1's DMAs 711 /
  // 1890 us; blocks 0-1 in phase 6 with 4-7 behind the DMAs 729 us.  Non-temporal x16 accesses
  // (probe ABL 13) 742-760 / 1888-1935 us.  The statistics, partial stores and residual_finalize
  // cost ~30-50 us (probe ABL 11).
  typedef _Float16 h2_8q __attribute__((ext_vector_type(2)));
  u32x4_8q xin[8][2];
  // lane id from an opaque asm, so offsets derived from it are computed where used (the 16
  // store offsets voO + mi * blkO, derived from a kernel-scope constant, are otherwise hoisted
  // out of the tile loop and held in 16 VGPRs for the kernel's life)
  auto lane_id = [&]() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
  };
  auto vo_out = [&](int l) {
    return (uint32_t)(((wr * 128 + (l & 15)) * a.ldo + wc * 64 + ((l >> 4) & 1) * 16 + (l >> 5) * 8) * 2);
  };
  auto res_load = [&](const __amdgpu_buffer_rsrc_t& r, uint32_t vo, int mi) {
    // (ABL 13: non-temporal x16 loads and stores, probe of L2 pollution)
    xin[mi][0] = __builtin_bit_cast(u32x4_8q, __builtin_amdgcn_raw_buffer_load_b128(r, vo + mi * blkO, 0, ABL == 13 ? 2 : 0));
    xin[mi][1] = __builtin_bit_cast(u32x4_8q, __builtin_amdgcn_raw_buffer_load_b128(r, vo + mi * blkO + 64, 0, ABL == 13 ? 2 : 0));
  };
  auto res_warm = [&](int m0, int n0) {   // F_WARM (see above)
    const __amdgpu_buffer_rsrc_t r = out_rsrc_at(m0, n0);
    const int l = lane_id();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int L = wave * 64 + l + i * 512;   // line L of the 256 rows x 512 bytes
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(smem + EK::LDS + ((F & F_DYN) ? 16 : 0)), 4,
                                               (uint32_t)((L >> 2) * a.ldo * 2 + (L & 3) * 128), 0, 0, 0);
    }
  };
  auto res_prefetch = [&](int mlo, int mhi, int m0, int n0) {
    if (!EK::RES || ABL == 12) return;
    const __amdgpu_buffer_rsrc_t r = out_rsrc_at(m0, n0);
    const uint32_t vo = vo_out(lane_id());
#pragma unroll
    for (int mi = mlo; mi < mhi; ++mi) res_load(r, vo, mi);
  };
  // sum across the four lanes (fr + 16 g) that hold one row's 64 columns: every lane gets the
  // same value (each level adds one commutative pair)
  auto row_sum4 = [](float x) {
    const auto a2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a2[0]) + __uint_as_float(a2[1]);
    const auto b2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b2[0]) + __uint_as_float(b2[1]);
  };
  // SPL: the split-f16 GEMM's f32 epilogues with gemm.hip's arithmetic (v = acc * (rsc[m] csc[n]) + b;
  // then the f32 store, the in-place add o + v, or split_gelu_store's QuickGELU split), so the
  // results are bit-identical to gemm_pp_kernel's.  A lane holds 4 consecutive columns of one row
  // per 16 x 16 block: the f32 pieces are 16-byte row stores straight from the accumulators, the
  // split's fp16 pieces pair blocks ni / ni + 1 by permlane16 swaps (the bf16 epilogue's layout)
  // VMEM ops issued by the running epilogue, checked against VM::EPI_VMEM in the counting build
  // (MICLIP_VMCHECK: `make` compiles it beside the product objects; the counters fold away)
  int vm_epi = 0;
#if MICLIP_VMCHECK
#define MI_VM_ISSUED(n) (vm_epi += (n))
#else
#define MI_VM_ISSUED(n) ((void)0)
#endif
  auto epilogue_spl = [&]() __attribute__((always_inline)) {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    const int lr = l & 15, lg = l >> 4;
    float4 bias[4], cs[4];
    const uint32_t ca = (uint32_t)(uintptr_t)(const LDS_AS float*)(scol + ppar * BN + wc * 64 + 4 * lg);
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                 "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(cs[0]), "=&v"(cs[1]), "=&v"(cs[2]), "=&v"(cs[3]) : "v"(ca) : "memory");
    {   // (SPL launches carry a bias, gemm_8q host: no runtime branch inside the epilogue, see F_ODUP)
      const uint32_t ba = (uint32_t)(uintptr_t)(const LDS_AS float*)(sbias + ppar * BN + wc * 64 + 4 * lg);
      asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                   "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(bias[0]), "=&v"(bias[1]), "=&v"(bias[2]), "=&v"(bias[3]) : "v"(ba) : "memory");
    }
    // the lane's 8 rows' rsc (and rmax for the split's bound), one row per 16-row block
    float rsv[8], rmv[8];
    const uint32_t ra = (uint32_t)(uintptr_t)(const LDS_AS float*)(srs + ppar * BM * 2 + wr * 128 + lr);
    asm volatile("ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:64\n\tds_read_b32 %2, %8 offset:128\n\t"
                 "ds_read_b32 %3, %8 offset:192\n\tds_read_b32 %4, %8 offset:256\n\tds_read_b32 %5, %8 offset:320\n\t"
                 "ds_read_b32 %6, %8 offset:384\n\tds_read_b32 %7, %8 offset:448\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(rsv[0]), "=&v"(rsv[1]), "=&v"(rsv[2]), "=&v"(rsv[3]), "=&v"(rsv[4]), "=&v"(rsv[5]),
                   "=&v"(rsv[6]), "=&v"(rsv[7])
                 : "v"(ra) : "memory");
    if (EPI == EPI_SPLIT_GELU)
      asm volatile("ds_read_b32 %0, %8 offset:1024\n\tds_read_b32 %1, %8 offset:1088\n\tds_read_b32 %2, %8 offset:1152\n\t"
                   "ds_read_b32 %3, %8 offset:1216\n\tds_read_b32 %4, %8 offset:1280\n\tds_read_b32 %5, %8 offset:1344\n\t"
                   "ds_read_b32 %6, %8 offset:1408\n\tds_read_b32 %7, %8 offset:1472\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(rmv[0]), "=&v"(rmv[1]), "=&v"(rmv[2]), "=&v"(rmv[3]), "=&v"(rmv[4]), "=&v"(rmv[5]),
                     "=&v"(rmv[6]), "=&v"(rmv[7])
                   : "v"(ra) : "memory");
    const int rows = min(a.M - pm0, BM);
    auto scaled = [&](int mi, int ni) {   // acc * (rsc[m] csc[n]) + b
      f32x4 v = acc[mi][ni] * (f32x4){rsv[mi] * cs[ni].x, rsv[mi] * cs[ni].y, rsv[mi] * cs[ni].z, rsv[mi] * cs[ni].w};
      return (f32x4){v[0] + bias[ni].x, v[1] + bias[ni].y, v[2] + bias[ni].z, v[3] + bias[ni].w};
    };
    if constexpr (EPI == EPI_F32 || EPI == EPI_RESID_F32) {
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((float*)a.out + (int64_t)pm0 * a.ldo + pn0), (short)0, rows * (int)a.ldo * 4, 0x00020000);
      const uint32_t vo = (uint32_t)(((wr * 128 + lr) * (int)a.ldo + wc * 64 + 4 * lg) * 4);
      const uint32_t blk = (uint32_t)(16 * a.ldo * 4);
      u32x4_8q xo[2][4];   // EPI_RESID_F32: the stream's values, one 16-row block ahead
      auto load_blk = [&](int mi) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          xo[mi & 1][ni] = __builtin_bit_cast(u32x4_8q, __builtin_amdgcn_raw_buffer_load_b128(ro, vo + mi * blk + ni * 64, 0, 0));
          MI_VM_ISSUED(1);
        }
      };
      if (EPI == EPI_RESID_F32) load_blk(0);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        if (EPI == EPI_RESID_F32 && mi < 7) load_blk(mi + 1);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          f32x4 v = scaled(mi, ni);
          if (EPI == EPI_RESID_F32) {
            const u32x4_8q ov = xo[mi & 1][ni];
            const f32x4 o = {__uint_as_float(ov[0]), __uint_as_float(ov[1]), __uint_as_float(ov[2]), __uint_as_float(ov[3])};
            v = (f32x4){o[0] + v[0], o[1] + v[1], o[2] + v[2], o[3] + v[3]};
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_8q, v), ro, vo + mi * blk + ni * 64, 0, 0);
          MI_VM_ISSUED(1);
        }
      }
    } else {   // EPI_SPLIT_GELU: [y1 | y1 | y2] at columns n, n + N, n + 2N; rsc_out[m] by the n = 0 tile
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((uint16_t*)a.out + (int64_t)pm0 * a.ldo + pn0), (short)0, rows * (int)a.ldo * 2, 0x00020000);
      const uint32_t vo = (uint32_t)(((wr * 128 + lr) * (int)a.ldo + wc * 64 + (lg & 1) * 16 + (lg >> 1) * 8) * 2);
      const uint32_t blk = (uint32_t)(16 * a.ldo * 2);
      // byte offsets of the second and third column blocks (soffset); F_ODUP: [y1 | y2] only
      const int n2 = a.N * 2, n4 = (F & F_ODUP) ? a.N * 2 : a.N * 4;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.rsc_out + pm0), (short)0, rows * 4, 0x00020000);
      // one writer per row (the n = 0 tile's columns 0-3); other lanes store out of range (dropped)
      const uint32_t vr = (pn0 == 0 && wc == 0 && lg == 0) ? (uint32_t)((wr * 128 + lr) * 4) : 0x7ff00000u;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const float bound = (rmv[mi] * a.bnd_w + a.bnd_b) * (1.0f + 0.00390625f);
        const int e = split_exp_8q(bound);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          uint2 k1[2], k2[2];
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) {
            const f32x4 v = scaled(mi, 2 * p + qq);
            uint32_t h1[4], h2[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float y = v[i] * (1.0f / (1.0f + expf(-1.702f * v[i])));
              const float ys = ldexpf(y, e);
              const _Float16 p1 = (_Float16)ys;
              const float f1 = (float)p1;
              const _Float16 p2 = __builtin_isfinite(f1) ? (_Float16)(ys - f1) : (_Float16)0.f;
              h1[i] = __builtin_bit_cast(uint16_t, p1);
              h2[i] = __builtin_bit_cast(uint16_t, p2);
            }
            k1[qq] = make_uint2(h1[0] | (h1[1] << 16), h1[2] | (h1[3] << 16));
            k2[qq] = make_uint2(h2[0] | (h2[1] << 16), h2[2] | (h2[3] << 16));
          }
          const auto ax = __builtin_amdgcn_permlane16_swap(k1[0].x, k1[1].x, false, false);
          const auto ay = __builtin_amdgcn_permlane16_swap(k1[0].y, k1[1].y, false, false);
          const auto bx = __builtin_amdgcn_permlane16_swap(k2[0].x, k2[1].x, false, false);
          const auto by = __builtin_amdgcn_permlane16_swap(k2[0].y, k2[1].y, false, false);
          const u32x4_8q d1 = {ax[0], ay[0], ax[1], ay[1]}, d2 = {bx[0], by[0], bx[1], by[1]};
          __builtin_amdgcn_raw_buffer_store_b128(d1, ro, vo + mi * blk + p * 64, 0, 0);
          MI_VM_ISSUED(1);
          if constexpr (!(F & F_ODUP)) {
            __builtin_amdgcn_raw_buffer_store_b128(d1, ro, vo + mi * blk + p * 64, n2, 0);
            MI_VM_ISSUED(1);
          }
          __builtin_amdgcn_raw_buffer_store_b128(d2, ro, vo + mi * blk + p * 64, n4, 0);
          MI_VM_ISSUED(1);
        }
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ldexpf(1.f, -e)), rr, vr + mi * 64, 0, 0);
        MI_VM_ISSUED(1);
      }
    }
  };
  auto epilogue_body = [&]() __attribute__((always_inline)) {
    if constexpr (EK::SPL) {
      if (ABL != 4) epilogue_spl();
      return;
    }
    if (ABL == 4) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
      return;
    }
    float4 bias[4];
    if (a.bias) {   // four reads under one wait, invisible to the compiler (gemm.hip lds_read_f4)
      const uint32_t ba = (uint32_t)(uintptr_t)(const LDS_AS float*)(sbias + ppar * BN + wc * 64 + 4 * g);
      asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                   "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(bias[0]), "=&v"(bias[1]), "=&v"(bias[2]), "=&v"(bias[3]) : "v"(ba) : "memory");
    } else {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bias[ni] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // LN: the column sums s_n beside c_n (= bias) and the lane's 8 rows' (rstd, rstd * mean)
    // LN: the column sums s_n beside c_n (= bias); the lane's rows' (rstd, rstd * mean) are read
    // per 16-row block below (one block ahead)
    float4 col[4];
    // lane offsets recomputed here (a lane constant kept from kernel entry is spilled around the
    // tile loop, and its reload's vmcnt(0) would drain the DMAs in flight)
    constexpr bool VOREC = EK::RES || (F & F_VOREC);
    int ln_ = 0;
    if (EK::LN || VOREC) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln_));
    uint32_t vo = voO;
    if constexpr (VOREC) vo = vo_out(ln_);
    // (asm LDS reads: a compiler-visible LDS read waits vmcnt(0) for the LDS-DMAs in flight)
    const uint32_t rab_a = (uint32_t)(uintptr_t)(const LDS_AS float*)(srs + ppar * BM * 2 + (wr * 128 + (ln_ & 15)) * 2);
    f32x2 rab_c = (f32x2){0.f, 0.f}, rab_n = (f32x2){0.f, 0.f};
    if (EK::LN) {
      const uint32_t ca = (uint32_t)(uintptr_t)(const LDS_AS float*)(scol + ppar * BN + wc * 64 + 4 * (ln_ >> 4));
      asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
                   "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(col[0]), "=&v"(col[1]), "=&v"(col[2]), "=&v"(col[3]) : "v"(ca) : "memory");
      asm volatile("ds_read_b64 %0, %1" : "=v"(rab_c) : "v"(rab_a) : "memory");
    }
    const __amdgpu_buffer_rsrc_t rsO = out_rsrc();
    // EPI_RES16 partials: ps row stride pstr bytes, the wave's 64 columns at entry pn0 / 64 + wc;
    // lanes g != 0 hold copies of their row's partial and store out of range (dropped)
    const int pstr = (a.N / 64) * 8;
    __amdgpu_buffer_rsrc_t rsP;
    uint32_t voP = 0;
    if (EK::RES) {
      const int rows = min(a.M - pm0, BM);
      rsP = __builtin_amdgcn_make_buffer_rsrc((void*)(a.ps + ((int64_t)pm0 * (a.N / 64) + pn0 / 64) * 2), (short)0,
                                              (rows - 1) * pstr + 32, 0x00020000);
      voP = (ln_ >> 4) ? 0x7ff00000u : (uint32_t)((wr * 128 + (ln_ & 15)) * pstr + wc * 8);
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      u32x4_8q dp[2];
      if (EK::LN) {   // block mi's row statistics landed; block mi + 1's read goes out
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rab_c) : : "memory");
        if (mi < 7) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(rab_n) : "v"(rab_a), "i"((mi + 1) * 128) : "memory");
      }
      uint2 pkb[2][2];   // F_GSTAGE16: the block's 16 values through QuickGELU in one stage order
      if (EK::GELU && (F & F_GSTAGE16)) {
        f32x2 gw[8];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          f32x2 lo = (f32x2){acc[mi][ni][0], acc[mi][ni][1]};
          f32x2 hi = (f32x2){acc[mi][ni][2], acc[mi][ni][3]};
          if (EK::LN) {
            const f32x2 ar = (f32x2){rab_c.x, rab_c.x}, br = (f32x2){-rab_c.y, -rab_c.y};
            lo = ar * lo + (br * (f32x2){col[ni].x, col[ni].y} + (f32x2){bias[ni].x, bias[ni].y});
            hi = ar * hi + (br * (f32x2){col[ni].z, col[ni].w} + (f32x2){bias[ni].z, bias[ni].w});
          } else {
            lo = lo + (f32x2){bias[ni].x, bias[ni].y};
            hi = hi + (f32x2){bias[ni].z, bias[ni].w};
          }
          gw[2 * ni] = lo;
          gw[2 * ni + 1] = hi;
        }
        quick_gelu_stage_8q<8, (F & F_GPK) != 0>(gw);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) pkb[ni >> 1][ni & 1] = make_uint2(pack_bf16x2(gw[2 * ni]), pack_bf16x2(gw[2 * ni + 1]));
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint2 pk[2];
        f32x2 gv[4];   // F_GSTAGE: the 8 values of this p, QuickGELU in stage order
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const int ni = 2 * p + qq;
          if (EK::GELU && (F & F_GSTAGE16)) {
            pk[qq] = pkb[p][qq];
            continue;
          }
          f32x2 lo = (f32x2){acc[mi][ni][0], acc[mi][ni][1]};
          f32x2 hi = (f32x2){acc[mi][ni][2], acc[mi][ni][3]};
          if (EK::LN) {   // rstd * acc + (c_n - rstd * mean * s_n)
            const f32x2 ar = (f32x2){rab_c.x, rab_c.x}, br = (f32x2){-rab_c.y, -rab_c.y};
            lo = ar * lo + (br * (f32x2){col[ni].x, col[ni].y} + (f32x2){bias[ni].x, bias[ni].y});
            hi = ar * hi + (br * (f32x2){col[ni].z, col[ni].w} + (f32x2){bias[ni].z, bias[ni].w});
          } else {
            lo = lo + (f32x2){bias[ni].x, bias[ni].y};
            hi = hi + (f32x2){bias[ni].z, bias[ni].w};
          }
          if (EK::GELU && (F & F_GSTAGE) && !(F & F_GSTAGE16)) {
            gv[2 * qq] = lo;
            gv[2 * qq + 1] = hi;
            continue;
          }
          if (EK::GELU) {
            lo = quick_gelu2_8q(lo);
            hi = quick_gelu2_8q(hi);
          }
          pk[qq] = make_uint2(pack_bf16x2(lo), pack_bf16x2(hi));
        }
        if (EK::GELU && (F & F_GSTAGE) && !(F & F_GSTAGE16)) {
          quick_gelu8_8q(gv);
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) pk[qq] = make_uint2(pack_bf16x2(gv[2 * qq]), pack_bf16x2(gv[2 * qq + 1]));
        }
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
        u32x4_8q d = {sx[0], sy[0], sx[1], sy[1]};
        if (EK::RES) {   // x16 = f16(x16 + bf16 delta), as residual_stats_kernel
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t dv = d[e];
            // (vector elements are copied out before __builtin_bit_cast: on an element lvalue,
            // this hipcc reads element 0 whatever the index)
            const uint32_t xv = ABL == 12 ? 0u : xin[mi][p][e];   // ABL 12: x16 loads ablated
            const h2_8q xh = __builtin_bit_cast(h2_8q, xv);
            const f32x2 sm = (f32x2){(float)xh.x, (float)xh.y} +
                             (f32x2){__uint_as_float(dv << 16), __uint_as_float(dv & 0xffff0000u)};
            const h2_8q oh = {(_Float16)sm.x, (_Float16)sm.y};
            d[e] = __builtin_bit_cast(uint32_t, oh);
          }
        }
        dp[p] = d;
        if (F & F_FULL) continue;
        if (ABL == 10) asm volatile("" ::"v"(d));   // stamp probe without the stores
        else {
          if (p == 0) __builtin_amdgcn_raw_buffer_store_b128(d, rsO, vo + mi * blkO, 0, (ABL == 13 || (F & F_ONT)) ? 2 : 0);
          else __builtin_amdgcn_raw_buffer_store_b128(d, rsO, vo + mi * blkO + 64, 0, (ABL == 13 || (F & F_ONT)) ? 2 : 0);
          MI_VM_ISSUED(1);
        }
      }
      if (F & F_FULL) {
        const bool top = fr < 8;
        u32x4_8q s1, s2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // row_ror:8 inside each 16-lane row: lane fr takes lane fr ^ 8's value
          const uint32_t r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dp[0][e], 0x128, 0xf, 0xf, false);
          const uint32_t r1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dp[1][e], 0x128, 0xf, 0xf, false);
          s1[e] = top ? dp[0][e] : r1;
          s2[e] = top ? r0 : dp[1][e];
        }
        __builtin_amdgcn_raw_buffer_store_b128(s1, rsO, voF + mi * blkO, 0, (F & F_ONT) ? 2 : 0);
        __builtin_amdgcn_raw_buffer_store_b128(s2, rsO, voF + mi * blkO + rows8, 0, (F & F_ONT) ? 2 : 0);
        MI_VM_ISSUED(2);
      }
      if (EK::RES && ABL == 11) {   // timing probe: no statistics, no partial stores
        __builtin_amdgcn_sched_barrier(0);
      } else if (EK::RES) {   // the row's 64-column partial: sum, then squared deviations from its mean
        // (the stored values re-read from dp in each pass: 16 f32 kept live across the passes spill)
        auto val = [&](int k) {
          const uint32_t w = dp[k >> 2][k & 3];
          const h2_8q h = __builtin_bit_cast(h2_8q, w);
          return (f32x2){(float)h.x, (float)h.y};
        };
        const f32x2 t = ((val(0) + val(1)) + (val(2) + val(3))) + ((val(4) + val(5)) + (val(6) + val(7)));
        const float s = row_sum4(t.x + t.y);
        const f32x2 mu = (f32x2){s * (1.0f / 64.0f), s * (1.0f / 64.0f)};
        f32x2 q = (f32x2){0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const f32x2 dv = val(k) - mu;
          q = dv * dv + q;
        }
        const float m2 = row_sum4(q.x + q.y);
        typedef unsigned int u32x2_8q __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((u32x2_8q){__float_as_uint(s), __float_as_uint(m2)}, rsP,
                                              voP + (uint32_t)(mi * 16 * pstr), 0, 0);
        MI_VM_ISSUED(1);
        __builtin_amdgcn_sched_barrier(0);
      }
      rab_c = rab_n;
    }
  };
  // every epilogue instance issues exactly the VMEM ops its waits were derived from
#if MICLIP_VMCHECK
  auto epilogue = [&]() __attribute__((always_inline)) {
    vm_epi = 0;
    epilogue_body();
    vm_count_check<VM::EPI_VMEM>(vm_epi);
  };
#else
  auto& epilogue = epilogue_body;
  (void)vm_epi;
#endif
#undef MI_VM_ISSUED

  // FIRST / LAST: the tile's first / last K-tile pair (compile-time: separate code paths)
  auto phase = [&](auto pc, auto firstc, auto lastc) {
    constexpr int P = decltype(pc)::value;
    constexpr bool FIRST = decltype(firstc)::value, LAST = decltype(lastc)::value;
    constexpr int b = P <= 4 ? 0 : 1;
    constexpr int q = (P - 1) & 3;
    const char* rbuf = smem + b * BUF;
    if constexpr (DYN) if (P == 1 && FIRST && wave == 0 && has_next) {   // the tile after next, before phase 1's DMAs
      dyn_got = dyn_claim();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (P == 1 && FIRST) {
      stamp(0);   // S0: tile start
      if ((ABL == 9 || ABL == 10) && ti == 2) st[7] = __builtin_amdgcn_s_memrealtime();
    }
    if (P == 1 && !(EK::RES && FIRST)) {
      issue(H_A1, 1);
      // a tile's first pair restages the odd B_n0 here too, ahead of the
      // previous tile's stores: the last pair did not re-read it in phase 8
      if (FIRST) issue(H_B0, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (FIRST && has_prev && !((F & F_BEARLY) && wr == 1)) {
        // the previous tile's whole epilogue, ahead of this phase's fragment
        // reads (its bias reads wait lgkmcnt(0)), behind the phase's DMAs
        epilogue();
        __builtin_amdgcn_sched_barrier(0);
      }
      if (FIRST) stamp(1);   // S1: epilogue issued
    }
    if (P == 1 && EK::RES && FIRST) {
      if (has_prev && !((F & F_BEARLY) && wr == 1)) {
        // the previous tile's x16 blocks 0-3 ahead of the phase's DMAs (one conditional block
        // from the loads to the epilogue: split across two, the loads' registers spilled)
        res_prefetch(2, 8, pm0, pn0);
        __builtin_amdgcn_sched_barrier(0);
        issue(H_A1, 1);
        issue(H_B0, 1);
        __builtin_amdgcn_sched_barrier(0);
        epilogue();
        __builtin_amdgcn_sched_barrier(0);
      } else {
        issue(H_A1, 1);
        issue(H_B0, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (P == 6 && LAST && EK::RES) {   // this tile's x16 blocks 0-1, ahead of the phase's DMA
      res_prefetch(0, 2, cur_m0, cur_n0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (q == 0) {
      read_a(rbuf + H_A0 * HALF);
      read_b(rbuf + H_B0 * HALF, fb0);
    } else if (q == 1) {
      read_b(rbuf + H_B1 * HALF, fb1);
    } else if (q == 2) {
      read_a(rbuf + H_A1 * HALF);
    } else if (!(LAST && P == 8)) {
      read_b(rbuf + H_B0 * HALF, fb0);   // re-read (16 fewer live VGPRs than keeping it from the q = 0 phase)
    }
    __builtin_amdgcn_sched_barrier(0);
    if (P == 2 && !FIRST) issue(H_B0, 1);
    if (P == 3) { advance(); issue(H_A0, 0); }
    if (P == 4) issue(H_B1, 0);
    if (P == 5) issue(H_A1, 0);
    if (P == 6) issue(H_B0, 0);
    if (P == 7) issue(H_A0, 1);
    if (P == 8) issue(H_B1, 1);
    __builtin_amdgcn_sched_barrier(0);
    // the awaited K-tile has two phases of DMAs younger than it; on a tile's
    // first pair the previous tile's 16 epilogue stores are younger as well
    // (they then have until phase 8 to complete)
    if (P == 4) {
      // on a tile's first pair the previous tile's epilogue (phase 1, after its DMAs) is younger than
      // the awaited K-tile as well: VM::FIRST_P4.  (F_BEARLY, lagging group: its epilogue ran at the
      // previous tile's phase 8, OLDER than phase 1's DMAs, so VM::YOUNGER also retires it --
      // issued three barrier intervals earlier)
      if (FIRST && has_prev && !((F & F_BEARLY) && wr == 1)) vm_wait<VM::FIRST_P4>();
      else vm_wait<VM::YOUNGER>();
      if constexpr ((F & F_WARM) && EK::RES) if (LAST) res_warm(cur_m0, cur_n0);
      if constexpr (DYN) if (FIRST && wave == 0 && has_next) dyn_publish(dyn_got);   // (retired: older than phase 1's DMAs)
      if (FIRST) stamp(3);   // S3: first pair's phase-4 wait passed
    }
    if (P == 8 && FIRST) stamp(4);   // S4: before the first pair's phase-8 wait (the stores must be done)
    if (P == 8) vm_wait<VM::YOUNGER>();
    if (P == 8 && FIRST) stamp(5);   // S5: after it
    if (P == 8 && LAST && has_next)   // next tile's bias (+ LN vectors), older than phase 1's DMAs
      stage_vectors(nxt_m0, nxt_n0, cpar ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (P == 1 && FIRST) stamp(2);   // S2: phase 1's MFMA section starts
    __builtin_amdgcn_s_setprio(1);
    constexpr int mh = q >= 2 ? 1 : 0, nh = (q == 1 || q == 2) ? 1 : 0;
    auto& fb = nh ? fb1 : fb0;
    if (ABL == 2) {
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
            // a tile's first MFMA into each accumulator (first pair, phases 1-4, k-step 0)
            // takes C = 0 as an inline constant: no zeroing pass between tiles
            if (OPF16)   // fp16 operands (the LN-folded GEMMs: x16 rows and W' = f16(W * gamma))
              acc[mh * 4 + mi][nh * 2 + ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                  __builtin_bit_cast(f16x8_8q, fb[ni][ks]), __builtin_bit_cast(f16x8_8q, fa[mi][ks]),
                  (FIRST && P <= 4 && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mh * 4 + mi][nh * 2 + ni], 0, 0, 0);
            else
              acc[mh * 4 + mi][nh * 2 + ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  fb[ni][ks], fa[mi][ks], (FIRST && P <= 4 && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mh * 4 + mi][nh * 2 + ni],
                  0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if constexpr ((F & F_BEARLY) && P == 8 && LAST) {
      if (wr == 1) {   // this tile's epilogue now, beside the leading group's (see F_BEARLY)
        pm0 = cur_m0;
        pn0 = cur_n0;
        ppar = cpar;
        __builtin_amdgcn_sched_barrier(0);
        // EPI_RES16: x16 blocks 2-7 here, after the MFMA section (blocks 0-1 went out in phase 6;
        // the fragment registers are dead, so all eight blocks fit); their latency runs beside the
        // leading group's epilogue in the same barrier interval
        res_prefetch(2, 8, pm0, pn0);
        __builtin_amdgcn_sched_barrier(0);
        epilogue();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    barrier();
  };
  auto pair = [&](auto firstc, auto lastc) {
    phase(Ph8q<1>{}, firstc, lastc);
    phase(Ph8q<2>{}, firstc, lastc);
    phase(Ph8q<3>{}, firstc, lastc);
    phase(Ph8q<4>{}, firstc, lastc);
    phase(Ph8q<5>{}, firstc, lastc);
    phase(Ph8q<6>{}, firstc, lastc);
    phase(Ph8q<7>{}, firstc, lastc);
    phase(Ph8q<8>{}, firstc, lastc);
  };

  if (a.stagger_phases > 1) {   // start stagger (see GemmArgs)
    const int ph = (blockIdx.x >> 3) % a.stagger_phases;
    if (ph) {
      const uint64_t until = __builtin_amdgcn_s_memrealtime() + (uint64_t)ph * a.stagger_ticks;
      while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(8);
    }
  }
  // ---- prologue: tile 0's bias, the whole even K-tile and the odd A_m0 / B_n1 of pair 0
  {
    int m0, n0;
    if constexpr (DYN) coords_l(rv, m0, n0);
    else coords(blockIdx.x, m0, n0);
    stage_vectors(m0, n0, 0);
  }
  if constexpr (DYN) if (wave == 0) dyn_got = dyn_claim();   // the second tile, retired by the prologue's wait
  issue(H_A0, 0);
  issue(H_B1, 0);
  issue(H_A1, 0);
  issue(H_B0, 0);
  issue(H_A0, 1);
  issue(H_B1, 1);
  vm_wait<VM::YOUNGER>();   // the even K-tile (and the vectors) landed
  if constexpr (DYN) if (wave == 0) {   // (landed before the barrier: the other waves read it right after)
    dyn_publish(dyn_got);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  barrier();
  if (wr == 1) barrier();   // stagger the two M-groups by one barrier

  int dcur = rv, dnext = DYN ? dyn_read() : 0;   // F_DYN: the current and the next tile
  for (int v = blockIdx.x; DYN ? dcur < dxe : v < ntiles; v += G) {
    int cm0, cn0;
    if constexpr (DYN) {
      coords_l(dcur, cm0, cn0);
      has_next = dnext < dxe;
      if (has_next) coords_l(dnext, nxt_m0, nxt_n0);
      dyn_next = dnext;
    } else {
      coords(v, cm0, cn0);
      has_next = v + G < ntiles;
      if (has_next) coords(v + G, nxt_m0, nxt_n0);
    }
    cur_m0 = cm0;
    cur_n0 = cn0;
    // (npairs >= 2, gemm_8q_ok: a one-pair instance beside these made hipcc spill ~200 VGPRs)
    pair(BoolC<true>{}, BoolC<false>{});
    for (int pp = 1; pp < npairs - 1; ++pp) pair(BoolC<false>{}, BoolC<false>{});
    pair(BoolC<false>{}, BoolC<true>{});
    stamp(6);   // S6: tile end
    if ((ABL == 9 || ABL == 10) && ti == 2) st[8] = __builtin_amdgcn_s_memrealtime();
    ++ti;
    pm0 = cm0;
    pn0 = cn0;
    ppar = cpar;
    has_prev = true;
    cpar ^= 1;
    if constexpr (DYN) {   // the claim published in this tile's first pair: the tile after next
      dcur = dnext;
      if (has_next) dnext = dyn_read();
    }
  }
  // the last tile's epilogue
  if (wr == 0) barrier();   // the M-groups' barrier counts meet
  if (!((F & F_BEARLY) && wr == 1)) {   // (F_BEARLY: the lagging group's is done)
    res_prefetch(2, 8, pm0, pn0);
    epilogue();
  }
  if ((ABL == 9 || ABL == 10) && lane == 0 && (wave & 3) == 0 && blockIdx.x < 1024) {
#pragma unroll
    for (int i = 0; i < 9; ++i) g_probe8q[(blockIdx.x * 2 + wr) * 9 + i] = st[i];
  }
  vm_wait<0>();   // trailing (dummy) DMAs land before the workgroup's LDS is released
}

}  // namespace

int gemm_8q_ok(const GemmArgs& a) {
  // descriptors: a tile's rows x row bytes must fit num_records (int)
  return a.N % BN == 0 && a.K % (2 * BK8) == 0 && a.K >= 4 * BK8 && a.M >= BM && !a.group && !a.patch_R &&
         (!a.a_dup || (a.a_f16 && a.a_dup % BK8 == 0 && a.K == 3 * a.a_dup && a.lda >= 2 * (int64_t)a.a_dup)) &&
         (int64_t)BM * a.lda * 2 < (1LL << 31) && (int64_t)BN * a.ldw * 2 < (1LL << 31) &&
         (int64_t)(BM + 64) * a.lda * 2 < (1LL << 32);
}

// mode: 0 = default (descriptors), 2 = no-MFMA probe,
// 3 = flat global_load_lds addressing, 4 = no-epilogue probe, 10 = whole-row epilogue stores (F_FULL)
// Tile order: n-tiles walked in groups of ng over all m-tiles, so each XCD's
// L2 (4 MB) keeps its group's weight panel (ng x 256 x K bf16) while the
// activation rows stream through: chosen when the tiles split into >= 6-wide
// groups of <= 2.4 MB.  Measured at the B/32 c_fc shape (M = 500k, N = 3072,
// K = 768, ng = 6): FETCH 7.8 -> 3.6 GB per launch, shader clock ~1.6 ->
// ~1.85 GHz, 2282 -> 2207 us (scripts/gpu_gemm_group.sh).  Narrower groups,
// and qkv's 9 n-tiles in groups of 3, were slower; ngroup < 0 forces the raster.
// Wide GEMMs whose n-tiles split evenly over the 8 XCDs take one group per XCD: the ViT-L/14 c_fc
// ([428459, 4096, 1024], 16 n-tiles) in groups of 2 (a 1-MB panel per XCD's L2) ran 3006-3011 us
// against 3145-3164 m-major, groups of 4 3065 and of 8 3095 (profiles/r05_y_ngroup.log,
// r05_x_ngroup.log); B/32's 12 n-tiles keep groups of 6 (2185 us; 2, 3, 4 and m-major 2235-2359)
// and L/14's in_proj (12 n-tiles) m-major (2292 us; groups of 4 or 8 2304-2377).
int default_ngroup_8q(int tiles_n, int K) {
  if (tiles_n >= 16 && tiles_n % 8 == 0 && (int64_t)(tiles_n / 8) * 256 * K * 2 <= 2400000) return tiles_n / 8;
  if (tiles_n < 12) return 0;
  for (int ng = tiles_n / 2; ng >= 6; --ng)
    if (tiles_n % ng == 0 && (int64_t)ng * 256 * K * 2 <= 2400000) return ng;
  return 0;
}

hipError_t gemm_8q(const GemmArgs& a0, int epi, hipStream_t s, int cus, int mode) {
  GemmArgs a = a0;
#if MICLIP_AB   // A/B: MICLIP_8Q_NG forces the tile-order group width (-1 = m-major raster)
  if (const char* ng = std::getenv("MICLIP_8Q_NG")) a.ngroup = std::atoi(ng);
#endif
  if (a.ngroup == 0) a.ngroup = default_ngroup_8q(a.N / BN, a.K);
  if (mode == 5 || mode == 6 || mode == 7 || mode == 8) {   // start-stagger probes: 2 / 4 / 2 phases of ~1/2, 1/4, 1/4 tile
    const int tile_ticks = (int)(2200LL * a.K / 768);   // ~22 us per 256 x 256 tile at K = 768
    a.stagger_phases = mode == 6 ? 4 : 2;
    a.stagger_ticks = (mode == 5 || mode == 8) ? tile_ticks / 2 : tile_ticks / 4;
    mode = mode == 8 ? 9 : 0;   // 8: the stamp probe, staggered
  }
  const int nt = ((a.M + BM - 1) / BM) * (a.N / BN);
  const int grid = nt < cus ? nt : cus;
  // the LayerNorm-folded GEMMs read fp16 operands; their vectors must be present
  if (epi == EPI_LN_BF16 || epi == EPI_LN_GELU_BF16) {
    if (!a.a_f16 || !a.rs || !a.colv || !a.bias || mode) return hipErrorInvalidValue;
#if MICLIP_AB   // A/B (MICLIP_8Q_F): epilogue flags F_VOREC (4) / F_GSTAGE (8) / both (12); 1 = none
    const char* fe = std::getenv("MICLIP_8Q_F");
    const int ff = fe ? std::atoi(fe) : 0;
    // 1000: the deferred-epilogue one-wave kernel (gemm_1d.hip), 1004 its no-epilogue probe
    if ((ff == 1000 || ff == 1004) && epi == EPI_LN_GELU_BF16) return gemm_1d(a0, ff - 1000, s, cus);
    if (ff == 1 && epi == EPI_LN_GELU_BF16) {
      hipLaunchKernelGGL((gemm_8q_kernel<EPI_LN_GELU_BF16, 0, 0, true>), dim3(grid), dim3(512), 0, s, a);
      return hipGetLastError();
    }
    // + 64: A DMAs non-temporal (F_ANT), + 128: output stores non-temporal (F_ONT)
    // + 2: whole-line (128-B) row stores (F_FULL), alone (46 / 2) or non-temporal (174 / 130)
    if (ff == 4 || ff == 8 || ff == 12 || ff == 44 || ff == 64 || ff == 192 || ff == 76 || ff == 204 || ff == 108 ||
        ff == 140 || ff == 46 || ff == 174 || ff == 2 || ff == 130 || ff == 300 || ff == 430 || ff == 942 ||
        ff == 642) {
#define LNF(E, FL) hipLaunchKernelGGL((gemm_8q_kernel<E, 0, FL, true>), dim3(grid), dim3(512), 0, s, a)
      if (epi == EPI_LN_BF16) {
        if (ff == 2 || ff == 46) LNF(EPI_LN_BF16, F_FULL);
        else if (ff == 130 || ff == 174) LNF(EPI_LN_BF16, F_FULL | F_ONT);
        else if (ff == 642 || ff == 942) LNF(EPI_LN_BF16, F_BEARLY | F_FULL | F_ONT);
        else if (ff == 64 || ff == 76) LNF(EPI_LN_BF16, F_ANT);
        else if (ff == 192 || ff == 204) LNF(EPI_LN_BF16, F_ANT | F_ONT);
        else LNF(EPI_LN_BF16, F_VOREC);   // (no GELU: F_GSTAGE has nothing to reorder)
      } else if (ff == 4) LNF(EPI_LN_GELU_BF16, F_VOREC);
      else if (ff == 8) LNF(EPI_LN_GELU_BF16, F_GSTAGE);
      else if (ff == 44) LNF(EPI_LN_GELU_BF16, F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else if (ff == 76 || ff == 64) LNF(EPI_LN_GELU_BF16, F_ANT | F_GSTAGE | F_VOREC);
      else if (ff == 204 || ff == 192) LNF(EPI_LN_GELU_BF16, F_ONT | F_ANT | F_GSTAGE | F_VOREC);
      else if (ff == 140) LNF(EPI_LN_GELU_BF16, F_ONT | F_GSTAGE | F_VOREC);
      else if (ff == 108) LNF(EPI_LN_GELU_BF16, F_ANT | F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else if (ff == 46 || ff == 2) LNF(EPI_LN_GELU_BF16, F_FULL | F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else if (ff == 174 || ff == 130) LNF(EPI_LN_GELU_BF16, F_ONT | F_FULL | F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else if (ff == 300) LNF(EPI_LN_GELU_BF16, F_GPK | F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else if (ff == 430) LNF(EPI_LN_GELU_BF16, F_GPK | F_ONT | F_FULL | F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else if (ff == 942 || ff == 642)
        LNF(EPI_LN_GELU_BF16, F_BEARLY | F_GPK | F_ONT | F_FULL | F_GSTAGE16 | F_GSTAGE | F_VOREC);
      else LNF(EPI_LN_GELU_BF16, F_GSTAGE | F_VOREC);
#undef LNF
      return hipGetLastError();
    }
#endif
    // c_fc: QuickGELU in stage order over each 16-row block's 16 values, its "+ 1" as packed adds,
    // store offsets from the lane id, and whole-line (128-B) non-temporal row stores -- all
    // bit-identical (lnfc500 2281 vs 2318 us for the 8-value order against none,
    // profiles/r04_ag_lnflags.log; the 16-value order 2296 vs 2354 us, profiles/r05_a_lnfc.log;
    // + packed adds + whole-line non-temporal stores 2239-2259 vs 2304-2311 us,
    // profiles/r05_d_lnfc.log).  in_proj: whole-line non-temporal stores, 1646 vs 1690 us
    // (r05_d_lnqkv.log; FETCH 5.4 -> 3.7x the operand bytes: the output no longer displaces the
    // weight panel from L2, profiles/r05_b_fullnt_gemm_traffic_ab.json).  Both: the lagging
    // M-group's epilogue beside the leading one's (F_BEARLY): c_fc 2143-2149 vs 2230 us, qkv 1606
    // vs 1615 us, bit-identical (profiles/r05_f_lnfc.log, r05_f_lnqkv.log)
#if MICLIP_AB   // A/B (MICLIP_8Q_DYN=1): the product flags + per-XCD claimed tile order (F_DYN)
    if (const char* dy = std::getenv("MICLIP_8Q_DYN")) {
      if (std::atoi(dy) == 1 && grid % 8 == 0 && nt >= grid) {
        void* ctr = nullptr;
        if (hipGetSymbolAddress(&ctr, HIP_SYMBOL(g_dyn8q)) != hipSuccess) return hipErrorInvalidSymbol;
        const hipError_t e = hipMemsetAsync(ctr, 0, sizeof(unsigned) * 8, s);
        if (e != hipSuccess) return e;
        if (epi == EPI_LN_BF16)
          hipLaunchKernelGGL((gemm_8q_kernel<EPI_LN_BF16, 0, F_DYN | F_BEARLY | F_FULL | F_ONT, true>), dim3(grid), dim3(512), 0, s, a);
        else
          hipLaunchKernelGGL(
              (gemm_8q_kernel<EPI_LN_GELU_BF16, 0, F_DYN | F_BEARLY | F_GPK | F_ONT | F_FULL | F_GSTAGE16 | F_GSTAGE | F_VOREC, true>),
              dim3(grid), dim3(512), 0, s, a);
        return hipGetLastError();
      }
    }
#endif
    if (epi == EPI_LN_BF16)
      hipLaunchKernelGGL((gemm_8q_kernel<EPI_LN_BF16, 0, F_BEARLY | F_FULL | F_ONT, true>), dim3(grid), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL(
          (gemm_8q_kernel<EPI_LN_GELU_BF16, 0, F_BEARLY | F_GPK | F_ONT | F_FULL | F_GSTAGE16 | F_GSTAGE | F_VOREC, true>),
          dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  // the fp32 tower's split-f16 GEMMs (K' = 3K; gemm.hip launch checks the vectors)
  if (epi == EPI_F32 || epi == EPI_RESID_F32 || epi == EPI_SPLIT_GELU) {
    if (!a.a_f16 || !a.rsc || !a.csc || !a.bias || mode || a.group || (a.ldo % 4) || (int64_t)BM * a.ldo * 4 >= (1LL << 31))
      return hipErrorInvalidValue;
    if (epi == EPI_SPLIT_GELU && (!a.rmax || !a.rsc_out || a.ldo != (a.o_dup ? 2 : 3) * (int64_t)a.N))
      return hipErrorInvalidValue;
#if MICLIP_AB   // A/B (MICLIP_F32_8Q=2): the lagging M-group's epilogue beside the leading one's (F_BEARLY)
    const char* fv = std::getenv("MICLIP_F32_8Q");
    if (fv && std::atoi(fv) == 2 && !a.o_dup) {
      if (epi == EPI_SPLIT_GELU) hipLaunchKernelGGL((gemm_8q_kernel<EPI_SPLIT_GELU, 0, F_BEARLY, true>), dim3(grid), dim3(512), 0, s, a);
      else if (epi == EPI_RESID_F32) hipLaunchKernelGGL((gemm_8q_kernel<EPI_RESID_F32, 0, F_BEARLY, true>), dim3(grid), dim3(512), 0, s, a);
      else hipLaunchKernelGGL((gemm_8q_kernel<EPI_F32, 0, F_BEARLY, true>), dim3(grid), dim3(512), 0, s, a);
      return hipGetLastError();
    }
#endif
    if (epi == EPI_SPLIT_GELU && a.o_dup) {
      hipLaunchKernelGGL((gemm_8q_kernel<EPI_SPLIT_GELU, 0, F_ODUP, true>), dim3(grid), dim3(512), 0, s, a);
    } else if (epi == EPI_SPLIT_GELU) {
      hipLaunchKernelGGL((gemm_8q_kernel<EPI_SPLIT_GELU, 0, 0, true>), dim3(grid), dim3(512), 0, s, a);
    } else if (epi == EPI_RESID_F32) {
      hipLaunchKernelGGL((gemm_8q_kernel<EPI_RESID_F32, 0, 0, true>), dim3(grid), dim3(512), 0, s, a);
    } else {
      hipLaunchKernelGGL((gemm_8q_kernel<EPI_F32, 0, 0, true>), dim3(grid), dim3(512), 0, s, a);
    }
    return hipGetLastError();
  }
  if (a.a_f16) return hipErrorInvalidValue;
  if (epi == EPI_RES16_BF16) {   // fused residual add: out = x16 (fp16), ps = row partial statistics
    if (!a.ps || mode || a.N % 64 || (a.ldo % 8)) return hipErrorInvalidValue;
#if MICLIP_AB   // timing probes (scripts/gemm_micro.py resout500 / resproj500): 11 no statistics, 12 no x16 loads
    const char* ab = std::getenv("MICLIP_RES_ABL");
    const int abl = ab ? std::atoi(ab) : 0;
    // start stagger (A/B, MICLIP_RES_STAGGER=phases:ticks): workgroups start (blockIdx / 8) % phases
    // x ticks (100 MHz) late, so the CUs' epilogue x16 read bursts do not coincide chip-wide
    if (const char* st = std::getenv("MICLIP_RES_STAGGER")) {
      a.stagger_phases = std::atoi(st);
      const char* c = std::strchr(st, ':');
      a.stagger_ticks = c ? std::atoi(c + 1) : 0;
    }
    if (abl == 11) hipLaunchKernelGGL((gemm_8q_kernel<EPI_RES16_BF16, 11, 0>), dim3(grid), dim3(512), 0, s, a);
    else if (abl == 12) hipLaunchKernelGGL((gemm_8q_kernel<EPI_RES16_BF16, 12, 0>), dim3(grid), dim3(512), 0, s, a);
    else if (abl == 13) hipLaunchKernelGGL((gemm_8q_kernel<EPI_RES16_BF16, 13, 0>), dim3(grid), dim3(512), 0, s, a);
    else if (abl == 14) hipLaunchKernelGGL((gemm_8q_kernel<EPI_RES16_BF16, 0, F_BEARLY>), dim3(grid), dim3(512), 0, s, a);
    else if (abl == 15) hipLaunchKernelGGL((gemm_8q_kernel<EPI_RES16_BF16, 0, F_WARM>), dim3(grid), dim3(512), 0, s, a);
    else
#endif
    hipLaunchKernelGGL((gemm_8q_kernel<EPI_RES16_BF16, 0, 0>), dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
#define L8Q(E, ABL_, F_) hipLaunchKernelGGL((gemm_8q_kernel<E, ABL_, F_>), dim3(grid), dim3(512), 0, s, a)
#if MICLIP_AB   // ablation / stamp probes: A/B build only
#define L8Q_ALL(E)                   \
  if (mode == 0) L8Q(E, 0, 0);       \
  else if (mode == 10) L8Q(E, 0, F_FULL); \
  else if (mode == 2) L8Q(E, 2, 0);  \
  else if (mode == 3) L8Q(E, 0, F_GLDS); \
  else if (mode == 4) L8Q(E, 4, 0);  \
  else if (mode == 9) L8Q(E, 9, 0);  \
  else if (mode == 1) L8Q(E, 10, 0);  \
  else return hipErrorInvalidValue;
#else
#define L8Q_ALL(E)                   \
  if (mode == 0) L8Q(E, 0, 0);       \
  else return hipErrorNotSupported;
#endif
#if MICLIP_AB
  {   // A/B (MICLIP_8Q_F): epilogue flags on the plain GELU kernel (text tower / unfolded c_fc)
    const char* fe = std::getenv("MICLIP_8Q_F");
    const int ff = fe ? std::atoi(fe) : 0;
    if (mode == 0 && epi == EPI_GELU_BF16 && (ff == 4 || ff == 8 || ff == 12)) {
      if (ff == 4) L8Q(EPI_GELU_BF16, 0, F_VOREC);
      else if (ff == 8) L8Q(EPI_GELU_BF16, 0, F_GSTAGE);
      else L8Q(EPI_GELU_BF16, 0, F_GSTAGE | F_VOREC);
      return hipGetLastError();
    }
    if (mode == 0 && epi == EPI_BF16 && ff == 4) {
      L8Q(EPI_BF16, 0, F_VOREC);
      return hipGetLastError();
    }
  }
#endif
  if (epi == EPI_GELU_BF16) {
    L8Q_ALL(EPI_GELU_BF16)
  } else if (epi == EPI_BF16) {
    L8Q_ALL(EPI_BF16)
  } else {
    return hipErrorInvalidValue;
  }
#undef L8Q_ALL
#undef L8Q
  return hipGetLastError();
}

}  // namespace miclip

namespace miclip {
hipError_t gemm8q_probe_read(unsigned long long* host, int n) {
#if MICLIP_AB
  if (n > 1024 * 2 * 9) n = 1024 * 2 * 9;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_probe8q), n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost);
#else
  (void)host;
  (void)n;
  return hipErrorNotSupported;   // stamp probe: A/B build only
#endif
}
}  // namespace miclip
