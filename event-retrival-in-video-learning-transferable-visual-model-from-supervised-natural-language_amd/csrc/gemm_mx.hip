// MX-fp8 GEMM (gfx950 block-scaled MFMA) for the "fp8 MFMA weights" tower
// configuration (BASELINE.json configs[4]: ViT-L/14@336px).
//
//   C[M,N] = (A[M,K] * 2^sa) . (W[N,K] * 2^sw)^T  (+ bias, QuickGELU)
//
// A and W are OCP e4m3 with one e8m0 scale per 64 consecutive k of a row;
// v_mfma_scale_f32_16x16x128_f8f6f4 applies the scales in hardware and runs at
// twice the bf16 MFMA rate (MI355X_MICROARCH.md "Matrix cores").  Probed on
// hardware (scripts/probes/):
//   operands (mx_layout.hip): lane l holds row (l & 15) and k = 32 (l >> 4) ..
//     +31 of the 128-k step, dword d = k 4d..4d+3; C/D is the common 16x16 map;
//   scales (mx_scale_map.hip, .out.txt): with opsel 0, byte 0 of lane l < 32
//     scales row (l & 15) over k = 64 (l >> 4) .. +63 — one e8m0 per 64 k, so
//     that is this format's block (the OCP MX block is 32);
//   LDS-DMA of 1- or 2-byte elements lands at a 4-byte lane stride, so scales
//     are moved as dwords: the scale tensor is stage-major, [K/128][rows_pad][2]
//     (rows_pad = rows rounded up to even; byte (kb & 1) of row r in stage
//     kb >> 1 is the e8m0 of k-block kb), one dword = 2 rows of one stage.
//
// Tile 256x256, 512 threads = 8 waves (2 M x 4 N), 128x64 per wave; the MFMA
// computes C^T (A operand = W fragment, B operand = activation fragment) so a
// lane holds 4 consecutive output columns (same epilogue as gemm.hip).
// Stage = 128 k = 128 bytes per row: 64 KB of operands + 2 KB of scales,
// double buffered by LDS-DMA one stage ahead; one barrier per stage.
// LDS row image: 16-byte chunk c of row r sits in slot c ^ ((r >> 1) & 5), so
// the two 16-byte reads of every fragment (chunks 2g, 2g+1 for lane group g)
// hit 16 distinct bank quads per ds_read_b128 lane group (exhaustive search).
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "internal.hpp"

namespace miclip {

namespace {

constexpr int MX_BK = 128;                              // k (bytes) per stage
constexpr int MX_STAGE = 512 * MX_BK;                   // 256 A rows + 256 W rows
constexpr int MX_SC_STAGE = 512 * 2;                    // 2 e8m0 (64-k blocks) per row per stage

typedef int v8i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int mx_swz(int r) { return (r >> 1) & 5; }

__device__ __forceinline__ float mx_gelu(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v)); }

__device__ __forceinline__ void glds4(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)lds_base, 4, 0, 0);
}

template <int EPI>
__global__ __launch_bounds__(512) void gemm_mx_kernel(GemmArgs a) {
  constexpr int BM = 256, BN = 256, WTM = 128, WTN = 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * MX_STAGE + 2 * MX_SC_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int nk = a.K / MX_BK;
  const int m_pad = (a.M + 1) & ~1;
  const uint8_t* A = (const uint8_t*)a.A;
  const uint8_t* Wt = (const uint8_t*)a.W;

  // ---- DMA geometry: instruction j (0..3) of wave w moves 8 rows x 128 B:
  // rows (w*4 + j)*8 + (lane >> 3), LDS slot lane & 7 <- global chunk slot ^ swz
  const uint8_t* asrc[4];
  const uint8_t* wsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wave * 4 + j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ mx_swz(r);
    asrc[j] = A + (int64_t)min(m0 + r, a.M - 1) * a.lda + c * 16;
    wsrc[j] = Wt + (int64_t)(n0 + r) * a.ldw + c * 16;
  }
  // scales: waves 0-1 move A row pairs, waves 2-3 W row pairs (one dword = 2 rows)
  const int spair = (wave & 1) * 64 + lane;
  const uint8_t* ssrc = wave < 2 ? a.a_scale + (int64_t)min(m0 + 2 * spair, m_pad - 2) * 2
                                 : a.w_scale + (int64_t)(n0 + 2 * spair) * 2;
  const int64_t sstage = wave < 2 ? (int64_t)m_pad * 2 : (int64_t)a.N * 2;  // bytes per stage
  auto issue = [&](int st) {
    char* base = smem + (st & 1) * MX_STAGE;
    const int kofs = st * MX_BK;
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(asrc[j] + kofs, base + (wave * 4 + j) * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(wsrc[j] + kofs, base + 256 * MX_BK + (wave * 4 + j) * 1024);
    if (wave < 4) glds4(ssrc + st * sstage, smem + 2 * MX_STAGE + (st & 1) * MX_SC_STAGE + wave * 256);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read: row fr of a 16-row block, chunks 2g and 2g+1
  const int fr = lane & 15, g = lane >> 4;
  const int rdo0 = fr * MX_BK + (((2 * g) ^ mx_swz(fr)) * 16);
  const int rdo1 = fr * MX_BK + (((2 * g + 1) ^ mx_swz(fr)) * 16);

  issue(0);
  for (int st = 0; st < nk; ++st) {
    // stage st landed (this wave's share), every wave's reads of the other
    // buffer (stage st-1) are done -> barrier -> prefetch st+1 into it
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (st + 1 < nk) issue(st + 1);
    const char* As = smem + (st & 1) * MX_STAGE + (wr * WTM) * MX_BK;
    const char* Ws = smem + (st & 1) * MX_STAGE + 256 * MX_BK + (wc * WTN) * MX_BK;
    const uint16_t* Ssa = (const uint16_t*)(smem + 2 * MX_STAGE + (st & 1) * MX_SC_STAGE) + wr * WTM;
    const uint16_t* Ssw = (const uint16_t*)(smem + 2 * MX_STAGE + (st & 1) * MX_SC_STAGE) + 256 + wc * WTN;
    v8i bw[4];
    int sw[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const char* p = Ws + ni * 16 * MX_BK;
      const uint4 lo = *(const uint4*)(p + rdo0), hi = *(const uint4*)(p + rdo1);
      bw[ni] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      sw[ni] = (int)((Ssw[ni * 16 + fr] >> (8 * (g & 1))) & 0xff);  // lanes >= 32: unused
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v8i av[4];
      int sa[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int mi = 4 * h + q;
        const char* p = As + mi * 16 * MX_BK;
        const uint4 lo = *(const uint4*)(p + rdo0), hi = *(const uint4*)(p + rdo1);
        av[q] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        sa[q] = (int)((Ssa[mi * 16 + fr] >> (8 * (g & 1))) & 0xff);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[4 * h + q][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw[ni], av[q], acc[4 * h + q][ni], 0,
                                                                                0, 0, sw[ni], 0, sa[q]);
    }
  }

  // ---- epilogue: lane holds rows m0 + wr*128 + mi*16 + fr, columns n0 + wc*64 + ni*16 + 4g .. +3
  float4 bias[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wc * WTN + ni * 16 + 4 * g;
    bias[ni] = a.bias ? *(const float4*)(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (EPI == EPI_GELU_MX) {
    // fp8 output for the next MX GEMM (mlp.c_fc -> c_proj): a wave's 64
    // columns of a row are exactly one 64-k block of the consumer: max over the
    // lane's 16 values, then across the 4 lane groups (xor 16, 32)
    const int blk = (n0 + wc * WTN) >> 6;
    const int64_t m_pad = (a.M + 1) & ~1;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = m0 + wr * WTM + mi * 16 + fr;
      float v[4][4];
      float amax = 0.f;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        v[ni][0] = mx_gelu(acc[mi][ni][0] + bias[ni].x);
        v[ni][1] = mx_gelu(acc[mi][ni][1] + bias[ni].y);
        v[ni][2] = mx_gelu(acc[mi][ni][2] + bias[ni].z);
        v[ni][3] = mx_gelu(acc[mi][ni][3] + bias[ni].w);
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[ni][0]), fabsf(v[ni][1])), fmaxf(fabsf(v[ni][2]), fabsf(v[ni][3]))));
      }
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      const int X = mx_block_exp(amax);
      const float inv = ldexpf(1.0f, -X);
      if (m < a.M) {
        uint8_t* o = (uint8_t*)a.out + (int64_t)m * a.ldo + n0 + wc * WTN + 4 * g;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) *(uint32_t*)(o + ni * 16) = mx_pack4(v[ni][0], v[ni][1], v[ni][2], v[ni][3], inv);
        if (g == 0) a.o_scale[mx_scale_index(m, blk, m_pad)] = (uint8_t)(X + 127);
      }
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int m = m0 + wr * WTM + mi * 16 + fr;
    if (EPI == EPI_F32) {
      if (m < a.M)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int n = n0 + wc * WTN + ni * 16 + 4 * g;
          *(float4*)((float*)a.out + (int64_t)m * a.ldo + n) =
              make_float4(acc[mi][ni][0] + bias[ni].x, acc[mi][ni][1] + bias[ni].y, acc[mi][ni][2] + bias[ni].z,
                          acc[mi][ni][3] + bias[ni].w);
        }
      continue;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint2 pk[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ni = 2 * p + q;
        float v0 = acc[mi][ni][0] + bias[ni].x, v1 = acc[mi][ni][1] + bias[ni].y;
        float v2 = acc[mi][ni][2] + bias[ni].z, v3 = acc[mi][ni][3] + bias[ni].w;
        if (EPI == EPI_GELU_BF16) {
          v0 = mx_gelu(v0); v1 = mx_gelu(v1); v2 = mx_gelu(v2); v3 = mx_gelu(v3);
        }
        pk[q] = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
      }
      // 16-lane-row exchange -> 8 consecutive columns per lane (gemm.hip DIRECT epilogue)
      const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
      const int col = n0 + wc * WTN + (2 * p + (g & 1)) * 16 + (g >> 1) * 8;
      if (m < a.M) *(uint4*)((uint16_t*)a.out + (int64_t)m * a.ldo + col) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
    }
  }
}

// ---------------------------------------------------------------------------
// Ping-pong MX-fp8 GEMM (the default for K >= 192): gemm.hip's gemm_pp_kernel
// schedule on the 32x32x64 block-scaled MFMA.  A stage is 64 k = 64 bytes per
// row, so the LDS geometry is byte-for-byte the bf16 kernel's (512 rows x 64 B
// = 32 KB per stage, 4-deep ring, LDS-DMA three stages ahead with counted
// vmcnt, the {0,2,3,1} chunk XOR), and a stage's 8 MFMAs per wave (4 M x 2 N
// blocks of 32x32, 2x the cycles of a bf16 32x32x16) fill the same 512
// cycles as the bf16 kernel's 32 16x16x32 MFMAs: twice the FLOPs per staged
// byte.  The two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one
// barrier apart, so one wave per SIMD issues MFMAs while its partner issues
// its DMA share and fragment reads.
//   operands (scripts/probes/mx32_layout.hip, .out.txt): lane l holds row
//     (l & 31), k = 32 (l >> 5) .. +31 of the stage (chunks 2h, 2h+1 of the
//     64-byte row); C element j of lane l is C[8 (j >> 2) + 4 (l >> 5) + (j & 3)][l & 31];
//   scales: byte 0 of lane l < 32 scales row l over the whole 64 k -> the
//     e8m0 of (row, stage) straight from the stage-major scale tensor.  The
//     stage pair's 1 KB scale block (256 A + 256 W rows x 2 B) rides in a
//     4-slot ring, one dword LDS-DMA per stage from waves 0-3.
// The MFMA computes C^T (A operand = W fragment) so lane l holds output row
// m = l & 31 and columns 8i + 4h .. +3 (h = l >> 5) of each 32-column block:
// permlane32_swap pairs give 16-byte bf16 row stores (T21).
__device__ __forceinline__ int pp_swz(int x) { return (0x1320 >> (4 * x)) & 0xF; }  // {0,2,3,1}

// LDS reads the compiler does not see (gemm.hip lds_read_f4): with plain
// loads from the shared array hipcc drains every in-flight LDS-DMA
// (s_waitcnt vmcnt(0)) before the section's first read, serialising the
// stage pipeline.  The section's lgkmcnt(0) + barrier covers the reads.
// Caveat of untracked reads: nothing may copy their destination registers
// before that wait; the emitted code reads straight into the MFMA operand
// tuples (checked in the .s: no v_mov between the ds_reads and the
// lgkmcnt(0)), and tests/test_gpu_mx.py would catch a stale operand.
__device__ __forceinline__ int lds_u8(const uint8_t* p) {
  int v;
  const uint32_t addr = (uint32_t)(uintptr_t)(const LDS_AS uint8_t*)p;
  asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

// 32-byte operand fragment (two 16-byte chunks of one LDS row), read with
// the same invisible-to-the-waitcnt-pass asm for the same reason
__device__ __forceinline__ v8i lds_frag32(const char* p, int rd0, int rd1) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i lo, hi;
  const uint32_t a0 = (uint32_t)(uintptr_t)(const LDS_AS char*)(p + rd0);
  const uint32_t a1 = (uint32_t)(uintptr_t)(const LDS_AS char*)(p + rd1);
  asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(a0));
  asm volatile("ds_read_b128 %0, %1" : "=v"(hi) : "v"(a1));
  return v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// The same reads with the LDS address split into a VGPR base and an immediate offset (the
// persistent kernel's lean stage body: one base add per operand per stage instead of one per read)
template <int OFF>
__device__ __forceinline__ v8i lds_frag32_o(uint32_t a0, uint32_t a1) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i lo, hi;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "i"(OFF));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "i"(OFF));
  return v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
template <int OFF>
__device__ __forceinline__ int lds_u8_o(uint32_t a) {
  int v;
  asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return v;
}

// Logical tile t -> (m-block, n-block) in groups of ng n-blocks (ng <= 0 or >= tiles_n: m-major):
// within a group every m-block, so an XCD's contiguous run of tiles keeps its group's weight panel
// (ng x 256 rows x K bytes of e4m3) in its 4-MB L2 (gemm_8q.hip tile_coords_8q)
__device__ __forceinline__ void tile_coords_mx(int t, int tiles_m, int tiles_n, int ng, int& mb, int& nb) {
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

template <int EPI>
__global__ __launch_bounds__(512) void gemm_mxpp_kernel(GemmArgs a) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  constexpr int BM = 256, BN = 256, WTM = 128, WTN = 64;
  constexpr int SB = 64;                               // k bytes per stage
  constexpr int RING = 4, LEAD = 3;
  constexpr int A_BYTES = BM * SB, STAGE = (BM + BN) * SB;
  constexpr int SC = 1024;                             // scale ring slot
  __shared__ __attribute__((aligned(16))) char smem[RING * STAGE + RING * SC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int mb_, nb_;
  tile_coords_mx(t, tiles_m, tiles_n, a.ngroup, mb_, nb_);
  const int m0 = mb_ * BM, n0 = nb_ * BN;
  const int nk = a.K / SB;
  const int m_pad = (a.M + 1) & ~1;
  const uint8_t* A = (const uint8_t*)a.A;
  const uint8_t* Wt = (const uint8_t*)a.W;

  // DMA: instruction j (0, 1) of wave w moves rows (w*2 + j)*16 + (lane >> 2), 4 lanes x 16 B per row
  const int lrow = lane >> 2;
  const int lchunk = ((lane & 3) ^ pp_swz(lane >> 4)) * 16;
  const uint8_t* asrc[2];
  const uint8_t* wsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    asrc[j] = A + (int64_t)min(m0 + (wave * 2 + j) * 16 + lrow, a.M - 1) * a.lda + lchunk;
    wsrc[j] = Wt + (int64_t)(n0 + (wave * 2 + j) * 16 + lrow) * a.ldw + lchunk;
  }
  // scales (waves 0-3): waves 0-1 move A row pairs, 2-3 W row pairs (one dword = 2 rows x {kb even, odd})
  const int spair = (wave & 1) * 64 + lane;
  const uint8_t* ssrc = (wave & 2) ? a.w_scale + (int64_t)(n0 + 2 * spair) * 2
                                   : a.a_scale + (int64_t)min(m0 + 2 * spair, m_pad - 2) * 2;
  const int64_t sstage = (wave & 2) ? (int64_t)a.N * 2 : (int64_t)m_pad * 2;
  // counted waits (common.hpp vm_wait): a stage is OPS_AW row DMAs per wave (DMA_ROWS instructions
  // of 16 rows for A and for W) plus, in group 0, one scale dword; vmcnt retires in issue order
  constexpr int DMA_ROWS = 2;
  constexpr int OPS_AW = 2 * DMA_ROWS, OPS_SC = 1;
  constexpr int OPS0 = OPS_AW + OPS_SC, OPS1 = OPS_AW;
  static_assert((LEAD - 1) * OPS0 <= VM_MAX, "the stages in flight exceed vmcnt's 6-bit field");
  auto issue = [&](int st) {
    char* base = smem + (st % RING) * STAGE;
    int n = 0;
#pragma unroll
    for (int j = 0; j < DMA_ROWS; ++j, ++n) glds16(asrc[j] + st * SB, base + (wave * 2 + j) * 1024);
#pragma unroll
    for (int j = 0; j < DMA_ROWS; ++j, ++n) glds16(wsrc[j] + st * SB, base + A_BYTES + (wave * 2 + j) * 1024);
    if (MICLIP_VMCHECK) vm_count_check<OPS_AW>(n);
    if (grp == 0) glds4(ssrc + (st >> 1) * sstage, smem + RING * STAGE + (st % RING) * SC + (wave & 3) * 256);   // OPS_SC
  };
  auto wait_stage = [&](int g1) {  // retire this wave's DMAs for stage g1: up to LEAD - 1 younger stages
    const int younger = min(LEAD - 1, nk - 1 - g1);
    if (grp == 0) vm_wait_stages<OPS0, LEAD - 1>(younger);
    else vm_wait_stages<OPS1, LEAD - 1>(younger);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lgkm_barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

#pragma unroll
  for (int st = 0; st < LEAD; ++st)
    if (st < nk) issue(st);
  wait_stage(0);
  barrier();
  if (grp == 1) barrier();

  const int lr = lane & 31, h = lane >> 5;
  const int rd0 = lr * SB + (((2 * h) ^ pp_swz((lr >> 2) & 3)) * 16);
  const int rd1 = lr * SB + (((2 * h + 1) ^ pp_swz((lr >> 2) & 3)) * 16);
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  v8i wf[2], af[4];
  int sw[2], sa[4];
  for (int g = 0; g < nk; ++g) {
    const char* As = smem + (g % RING) * STAGE + (grp * WTM) * SB;
    const char* Ws = smem + (g % RING) * STAGE + A_BYTES + (wc * WTN) * SB;
    const uint8_t* Sc = (const uint8_t*)(smem + RING * STAGE + (g % RING) * SC) + (g & 1);
    // ---- L: DMA share of stage g+3, this stage's fragments and scales
    if (g + LEAD < nk) issue(g + LEAD);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      wf[ni] = lds_frag32(Ws + ni * 32 * SB, rd0, rd1);
      sw[ni] = lds_u8(Sc + 512 + (wc * WTN + ni * 32 + lr) * 2);
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      af[mi] = lds_frag32(As + mi * 32 * SB, rd0, rd1);
      sa[mi] = lds_u8(Sc + (grp * WTM + mi * 32 + lr) * 2);
    }
    if (grp == 1 && g + 1 < nk) wait_stage(g + 1);
    lgkm_barrier();
    // ---- C: 8 MFMAs (4 M x 2 N blocks of 32x32x64)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[ni], af[mi], acc[mi][ni], 0, 0, 0, sw[ni], 0,
                                                                      sa[mi]);
    if (grp == 0 && g + 1 < nk) wait_stage(g + 1);
    barrier();
  }
  if (grp == 0) barrier();

  // ------------------------------------------------ epilogue (no LDS, no barrier)
  // lane: output row m0 + grp*128 + mi*32 + lr; element j of block (mi, ni) is
  // column n0 + wc*64 + ni*32 + 8 (j >> 2) + 4h + (j & 3)
  float4 bias[2][4];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wc * WTN + ni * 32 + 8 * i + 4 * h;
      bias[ni][i] = a.bias ? *(const float4*)(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  auto val = [&](int mi, int ni, int j) -> float {
    const float4 b = bias[ni][j >> 2];
    const float bb = (j & 3) == 0 ? b.x : (j & 3) == 1 ? b.y : (j & 3) == 2 ? b.z : b.w;
    const float v = acc[mi][ni][j] + bb;
    return (EPI == EPI_GELU_BF16 || EPI == EPI_GELU_MX) ? mx_gelu(v) : v;
  };
  if (EPI == EPI_GELU_MX) {
    // fp8 output for the next MX GEMM: the wave's 64 columns of a row are one
    // 64-k block of the consumer; this lane holds 32 of them, its partner
    // (lane ^ 32) the other 32
    const int blk = (n0 + wc * WTN) >> 6;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int m = m0 + grp * WTM + mi * 32 + lr;
      float v[2][16];
      float amax = 0.f;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          v[ni][j] = val(mi, ni, j);
          amax = fmaxf(amax, fabsf(v[ni][j]));
        }
      const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
      amax = fmaxf(__uint_as_float(sx[0]), __uint_as_float(sx[1]));
      const int X = mx_block_exp(amax);
      const float inv = ldexpf(1.0f, -X);
      // dword i of block ni holds bytes ni*32 + 8i + 4h .. +3 of the row; a half swap gives lanes
      // 0-31 bytes ni*32 + 0..15 and lanes 32-63 bytes ni*32 + 16..31, so each lane stores 16
      // contiguous bytes (2 store instructions per row block instead of 8 dword stores: the
      // per-CU store issue, not the bytes, set the epilogue's time)
      uint4 q16[2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        uint32_t d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = mx_pack4(v[ni][4 * i], v[ni][4 * i + 1], v[ni][4 * i + 2], v[ni][4 * i + 3], inv);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 4");   // wait states between the packs and the swaps (gemm_mx8q.hip permlane_gap)
        __builtin_amdgcn_sched_barrier(0);
        const auto s02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
        const auto s13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
        q16[ni] = make_uint4(s02[0], s02[1], s13[0], s13[1]);
      }
      if (m < a.M) {
        uint8_t* o = (uint8_t*)a.out + (int64_t)m * a.ldo + n0 + wc * WTN + 16 * h;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) *(uint4*)(o + ni * 32) = q16[ni];
        if (h == 0) a.o_scale[mx_scale_index(m, blk, m_pad)] = (uint8_t)(X + 127);
      }
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = m0 + grp * WTM + mi * 32 + lr;
    if (EPI == EPI_F32) {
      if (m < a.M)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            *(float4*)((float*)a.out + (int64_t)m * a.ldo + n0 + wc * WTN + ni * 32 + 8 * i + 4 * h) =
                make_float4(val(mi, ni, 4 * i), val(mi, ni, 4 * i + 1), val(mi, ni, 4 * i + 2), val(mi, ni, 4 * i + 3));
      continue;
    }
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int ip = 0; ip < 2; ++ip) {
        // groups 2ip (cols 16ip + 4h ..) and 2ip+1 (cols 16ip + 8 + 4h ..): after the
        // half swap lanes 0-31 hold cols 16ip .. +7, lanes 32-63 cols 16ip + 8 .. +15
        const int j0 = 8 * ip, j1 = 8 * ip + 4;
        const uint32_t ax = pack_bf16x2(val(mi, ni, j0), val(mi, ni, j0 + 1));
        const uint32_t ay = pack_bf16x2(val(mi, ni, j0 + 2), val(mi, ni, j0 + 3));
        const uint32_t bx = pack_bf16x2(val(mi, ni, j1), val(mi, ni, j1 + 1));
        const uint32_t by = pack_bf16x2(val(mi, ni, j1 + 2), val(mi, ni, j1 + 3));
        const auto sx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
        if (m < a.M)
          *(uint4*)((uint16_t*)a.out + (int64_t)m * a.ldo + n0 + wc * WTN + ni * 32 + 16 * ip + 8 * h) =
              make_uint4(sx[0], sy[0], sx[1], sy[1]);
      }
  }
}

// ---------------------------------------------------------------------------
// Persistent MX-fp8 ping-pong (round 6; configs[4]): gemm_mxpp_kernel's
// stage, fragment, MFMA and epilogue arithmetic (bit-identical results) with one workgroup per
// CU walking its tiles as gemm.hip's gemm_ppp_kernel does for bf16.  At K = 1024 a non-persistent
// tile paid a fixed ~8.6 us of its ~25 us (launch, the first LEAD stages' DMA latency exposed,
// the ring draining over its last LEAD stages) -- the K sweep of round 5: c_proj (K = 4096) ran
// at 0.37 of the fp8 peak, c_fc (K = 1024) at 0.27.  Here the stages of all of a workgroup's
// tiles are one stream through the ring: the next tile's first LEAD stages (with its bias, by
// LDS-DMA into a parity slot) are issued in this tile's last LEAD iterations, so they land under
// this tile's MFMAs and epilogue.  Counted waits: a stage is OPS_AW row DMAs (+ the scale dword in
// group 0); the previous tile's NSTORE epilogue stores are younger than the next tile's first
// LEAD stages and older than every later one, so the waits add them while waiting for stages
// < LEAD; a partial last m-tile (an unknown store count) drains with vmcnt(0) instead.
__device__ __forceinline__ float4 mx_lds_f4(const float* p) {   // (an LDS read hipcc does not see)
  float4 v;
  const uint32_t addr = (uint32_t)(uintptr_t)(const LDS_AS float*)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// LEAN (round 6, A/B MICLIP_MX_PERSIST=4; measured no faster, see below): the stage loop split
// into its head (the waits that may include the previous tile's stores), a steady part and its
// tail, each with its wait immediate known at compile time, and instantiated per M-group, so a
// steady stage carries no runtime wait chain and no group branch (the PMC pass of the first form,
// profiles/r06_w_mx_fc_pmc.txt: per wave and tile 903 SALU, 200 branches and 2444 VALU beside 128
// MFMAs, MFMA busy 0.32 -- the ping-pong's load-and-read section, not the MFMAs, set each stage's
// length); the fragment reads address LDS as one base per operand plus immediate offsets.  Same
// DMAs, reads, MFMAs and epilogue: bit-identical.  At the configs[4] shapes (scripts/mx_persist_micro.py,
// profiles/r06_x_mx_lean.log) c_fc -> MX-fp8 2806 vs 2777 us, qkv 1944 vs 1976, out_proj 698 vs 709:
// within noise, so the scalar work was not what bounds the stage (and the GELU -> MX-fp8 instance
// spills 4 registers); the first form stays the default.
template <int EPI, bool LEAN = false>
__global__ __launch_bounds__(512) void gemm_mxppp_kernel(GemmArgs a) {
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  constexpr int BM = 256, BN = 256, WTM = 128, WTN = 64;
  constexpr int SB = 64;                               // k bytes per stage
  constexpr int RING = 4, LEAD = 3;
  constexpr int A_BYTES = BM * SB, STAGE = (BM + BN) * SB;
  constexpr int SC = 1024;                             // scale ring slot
  // epilogue store instructions per wave of a full tile: GELU_MX 2 row pieces + the scale byte per
  // 32-row block; bf16 2 (ni) x 2 (ip) per block; f32 2 (ni) x 4 per block
  constexpr int NSTORE = EPI == EPI_GELU_MX ? 4 * (2 + 1) : EPI == EPI_F32 ? 4 * 2 * 4 : 4 * 2 * 2;
  constexpr int DMA_ROWS = 2;
  constexpr int OPS_AW = 2 * DMA_ROWS, OPS_SC = 1;
  constexpr int OPS0 = OPS_AW + OPS_SC, OPS1 = OPS_AW;
  static_assert((LEAD - 1) * OPS0 + NSTORE <= VM_MAX, "the ops in flight exceed vmcnt's 6-bit field");
  __shared__ __attribute__((aligned(16))) char smem[RING * STAGE + RING * SC + 2 * BN * 4];
  float* sbias = (float*)(smem + RING * STAGE + RING * SC);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int nk = a.K / SB;
  const int m_pad = (a.M + 1) & ~1;
  const uint8_t* A = (const uint8_t*)a.A;
  const uint8_t* Wt = (const uint8_t*)a.W;
  auto coords = [&](int v, int& mm, int& nn) {   // grid % 8 == 0 keeps a WG's tiles on its XCD's run
    const int t = xcd_remap(v, ntiles);
    int mb, nb;
    tile_coords_mx(t, tiles_m, tiles_n, a.ngroup, mb, nb);
    mm = mb * BM;
    nn = nb * BN;
  };
  int vb = blockIdx.x, m0, n0;
  coords(vb, m0, n0);

  const int lrow = lane >> 2;
  const int lchunk = ((lane & 3) ^ pp_swz(lane >> 4)) * 16;
  const int spair = (wave & 1) * 64 + lane;
  const int64_t sstage = (wave & 2) ? (int64_t)a.N * 2 : (int64_t)m_pad * 2;
  const uint8_t* asrc[2];
  const uint8_t* wsrc[2];
  const uint8_t* ssrc;
  auto set_src = [&](int mm, int nn) {
#pragma unroll
    for (int j = 0; j < DMA_ROWS; ++j) {
      asrc[j] = A + (int64_t)min(mm + (wave * 2 + j) * 16 + lrow, a.M - 1) * a.lda + lchunk;
      wsrc[j] = Wt + (int64_t)(nn + (wave * 2 + j) * 16 + lrow) * a.ldw + lchunk;
    }
    ssrc = (wave & 2) ? a.w_scale + (int64_t)(nn + 2 * spair) * 2
                      : a.a_scale + (int64_t)min(mm + 2 * spair, m_pad - 2) * 2;
  };
  auto issue = [&](int st, int slot) {   // stage st of the tile set_src points at -> ring slot
    char* base = smem + slot * STAGE;
    int n = 0;
#pragma unroll
    for (int j = 0; j < DMA_ROWS; ++j, ++n) glds16(asrc[j] + st * SB, base + (wave * 2 + j) * 1024);
#pragma unroll
    for (int j = 0; j < DMA_ROWS; ++j, ++n) glds16(wsrc[j] + st * SB, base + A_BYTES + (wave * 2 + j) * 1024);
    if (MICLIP_VMCHECK) vm_count_check<OPS_AW>(n);
    if (grp == 0) glds4(ssrc + (st >> 1) * sstage, smem + RING * STAGE + slot * SC + (wave & 3) * 256);   // OPS_SC
  };
  bool pend = false;   // the previous tile's NSTORE stores are in flight, younger than stages 0..LEAD-1
  int rb = 0, nm0 = 0, nn0 = 0;   // rb: ring slot of this tile's stage 0
  bool has_next = false;
  auto wait_stage = [&](int g1) {
    const int younger = has_next ? LEAD - 1 : min(LEAD - 1, nk - 1 - g1);
    if (grp == 0) {
      if (g1 < LEAD && pend) vm_wait_stages<OPS0, LEAD - 1, NSTORE>(younger);
      else vm_wait_stages<OPS0, LEAD - 1>(younger);
    } else {
      if (g1 < LEAD && pend) vm_wait_stages<OPS1, LEAD - 1, NSTORE>(younger);
      else vm_wait_stages<OPS1, LEAD - 1>(younger);
    }
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lgkm_barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  int tpar = 0;   // tile parity: bias slot
  auto load_bias = [&](int slot, int nn) {   // wave 0: 64 lanes x 16 B = the tile's 256 bias values
    if (wave == 0 && a.bias) glds16(a.bias + nn + lane * 4, sbias + slot * BN);
  };
  load_bias(0, n0);
  set_src(m0, n0);
#pragma unroll
  for (int st = 0; st < LEAD; ++st)
    if (st < nk) issue(st, st);

  const int lr = lane & 31, h = lane >> 5;
  const int rd0 = lr * SB + (((2 * h) ^ pp_swz((lr >> 2) & 3)) * 16);
  const int rd1 = lr * SB + (((2 * h + 1) ^ pp_swz((lr >> 2) & 3)) * 16);
  static_assert(RING == 4 && 96 * SB < 65536, "LEAN: ring slot by mask, read offsets in the 16-bit field");
  while (true) {
    const int nvb = vb + (int)gridDim.x;
    has_next = nvb < ntiles;
    if (has_next) coords(nvb, nm0, nn0);
    wait_stage(0);
    barrier();
    if (grp == 1) barrier();
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    v8i wf[2], af[4];
    int sw[2], sa[4];
    if constexpr (!LEAN) {
    for (int gs = 0; gs < nk; ++gs) {
      const int slot = (rb + gs) % RING;
      const char* As = smem + slot * STAGE + (grp * WTM) * SB;
      const char* Ws = smem + slot * STAGE + A_BYTES + (wc * WTN) * SB;
      const uint8_t* Sc = (const uint8_t*)(smem + RING * STAGE + slot * SC) + (gs & 1);
      if (gs + LEAD < nk) {
        issue(gs + LEAD, (rb + gs + LEAD) % RING);
      } else if (has_next) {   // the next tile's stage gs + LEAD - nk, the same ring position in the stream
        const int st = gs + LEAD - nk;
        if (st == 0) {
          load_bias(tpar ^ 1, nn0);
          set_src(nm0, nn0);
        }
        issue(st, (rb + gs + LEAD) % RING);
      }
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        wf[ni] = lds_frag32(Ws + ni * 32 * SB, rd0, rd1);
        sw[ni] = lds_u8(Sc + 512 + (wc * WTN + ni * 32 + lr) * 2);
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        af[mi] = lds_frag32(As + mi * 32 * SB, rd0, rd1);
        sa[mi] = lds_u8(Sc + (grp * WTM + mi * 32 + lr) * 2);
      }
      if (grp == 1 && gs + 1 < nk) wait_stage(gs + 1);
      lgkm_barrier();
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[ni], af[mi], acc[mi][ni], 0, 0, 0, sw[ni], 0,
                                                                        sa[mi]);
      if (grp == 0 && gs + 1 < nk) wait_stage(gs + 1);
      barrier();
    }
    } else {
    // the per-wave LDS bases of the fragment and scale reads (a stage adds its ring slot), derived
    // per tile from an opaque lane id so that they are not held across the epilogue
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int lr_ = ln & 31, h_ = ln >> 5;
    const int sw_ = pp_swz((lr_ >> 2) & 3);
    // (three VGPRs: A's chunk-0 address, the lane's chunk-1 distance and the A-scale address; the W
    // addresses differ from the A ones by wave-uniform amounts)
    const int wcu = __builtin_amdgcn_readfirstlane(wc);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const LDS_AS char*)smem;
    const uint32_t vA0 = lds0 + (uint32_t)(lr_ * SB + (((2 * h_) ^ sw_) * 16) + grp * WTM * SB);
    const uint32_t vD = (uint32_t)((((2 * h_ + 1) ^ sw_) - ((2 * h_) ^ sw_)) * 16);
    const uint32_t vSA = lds0 + (uint32_t)(RING * STAGE + (grp * WTM + lr_) * 2);
    const uint32_t dW = (uint32_t)(A_BYTES + wcu * WTN * SB - grp * WTM * SB);
    const uint32_t dSW = (uint32_t)(512 + wcu * WTN * 2 - grp * WTM * 2);
    // one stage; G the M-group, ST a steady stage: gs in [LEAD - 1, nk - LEAD), where this stage's
    // DMA issue is the current tile's and the wait for stage gs + 1 has LEAD - 1 younger stages and
    // no stores behind it (wait_stage's general case)
    auto body = [&](auto g_c, const bool ST, int gs) __attribute__((always_inline)) {
      constexpr int G = decltype(g_c)::value;
      const int slot = (rb + gs) & (RING - 1);
      if (ST || gs + LEAD < nk) {
        issue(gs + LEAD, (rb + gs + LEAD) & (RING - 1));
      } else if (has_next) {
        const int st = gs + LEAD - nk;
        if (st == 0) {
          load_bias(tpar ^ 1, nn0);
          set_src(nm0, nn0);
        }
        issue(st, (rb + gs + LEAD) & (RING - 1));
      }
      const uint32_t so = (uint32_t)(slot * STAGE), sso = (uint32_t)(slot * SC + (gs & 1));
      const uint32_t a0 = vA0 + so, a1 = a0 + vD, w0 = a0 + dW, w1 = a1 + dW;
      const uint32_t ssa = vSA + sso, ssw = ssa + dSW;
      wf[0] = lds_frag32_o<0>(w0, w1);
      wf[1] = lds_frag32_o<32 * SB>(w0, w1);
      sw[0] = lds_u8_o<0>(ssw);
      sw[1] = lds_u8_o<64>(ssw);
      af[0] = lds_frag32_o<0>(a0, a1);
      af[1] = lds_frag32_o<32 * SB>(a0, a1);
      af[2] = lds_frag32_o<64 * SB>(a0, a1);
      af[3] = lds_frag32_o<96 * SB>(a0, a1);
      sa[0] = lds_u8_o<0>(ssa);
      sa[1] = lds_u8_o<64>(ssa);
      sa[2] = lds_u8_o<128>(ssa);
      sa[3] = lds_u8_o<192>(ssa);
      if (G == 1 && (ST || gs + 1 < nk)) {
        if (ST) vm_wait<(LEAD - 1) * OPS1>();
        else wait_stage(gs + 1);
      }
      lgkm_barrier();
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[ni], af[mi], acc[mi][ni], 0, 0, 0, sw[ni], 0,
                                                                        sa[mi]);
      if (G == 0 && (ST || gs + 1 < nk)) {
        if (ST) vm_wait<(LEAD - 1) * OPS0>();
        else wait_stage(gs + 1);
      }
      barrier();
    };
    auto run = [&](auto g_c) __attribute__((always_inline)) {
      for (int gs = 0; gs < nk; ++gs) body(g_c, gs >= LEAD - 1 && gs < nk - LEAD, gs);
    };
    if (grp == 0) run(std::integral_constant<int, 0>{});
    else run(std::integral_constant<int, 1>{});
    }
    if (grp == 0) barrier();   // groups realigned; every ring read of this tile is done

    // ---- epilogue of tile (cm0, cn0) (gemm_mxpp_kernel's arithmetic; bias from its LDS slot)
    const int cm0 = m0, cn0 = n0;
    int vm_st = 0;   // store instructions of a full tile (MICLIP_VMCHECK: checked against NSTORE)
    float4 bias[2][4];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        bias[ni][i] = a.bias ? mx_lds_f4(sbias + tpar * BN + wc * WTN + ni * 32 + 8 * i + 4 * h)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    auto val = [&](int mi, int ni, int j) -> float {
      const float4 b = bias[ni][j >> 2];
      const float bb = (j & 3) == 0 ? b.x : (j & 3) == 1 ? b.y : (j & 3) == 2 ? b.z : b.w;
      const float v = acc[mi][ni][j] + bb;
      return (EPI == EPI_GELU_BF16 || EPI == EPI_GELU_MX) ? mx_gelu(v) : v;
    };
    if constexpr (EPI == EPI_GELU_MX) {
      const int blk = (cn0 + wc * WTN) >> 6;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int m = cm0 + grp * WTM + mi * 32 + lr;
        // QuickGELU in stage order over the block's 32 values (each value's operations are
        // mx_gelu's, so the result is bit-identical; consecutive transcendentals are independent,
        // as gemm_8q's F_GSTAGE16)
        float v[2][16];
        float amax = 0.f;
        if constexpr (LEAN) {   // (one 16-value stage order per ni: 16 fewer live registers, same values)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            float e[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const float4 b = bias[ni][j >> 2];
              v[ni][j] = acc[mi][ni][j] + ((j & 3) == 0 ? b.x : (j & 3) == 1 ? b.y : (j & 3) == 2 ? b.z : b.w);
              e[j] = __expf(-1.702f * v[ni][j]);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) e[j] = __builtin_amdgcn_rcpf(1.0f + e[j]);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              v[ni][j] = v[ni][j] * e[j];
              amax = fmaxf(amax, fabsf(v[ni][j]));
            }
          }
        } else {
        float e[2][16];
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const float4 b = bias[ni][j >> 2];
            v[ni][j] = acc[mi][ni][j] + ((j & 3) == 0 ? b.x : (j & 3) == 1 ? b.y : (j & 3) == 2 ? b.z : b.w);
            e[ni][j] = __expf(-1.702f * v[ni][j]);
          }
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 16; ++j) e[ni][j] = __builtin_amdgcn_rcpf(1.0f + e[ni][j]);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            v[ni][j] = v[ni][j] * e[ni][j];
            amax = fmaxf(amax, fabsf(v[ni][j]));
          }
        }
        const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(amax), __float_as_uint(amax), false, false);
        amax = fmaxf(__uint_as_float(sx[0]), __uint_as_float(sx[1]));
        const int X = mx_block_exp(amax);
        const float inv = ldexpf(1.0f, -X);
        uint4 q16[2];
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          uint32_t d[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) d[i] = mx_pack4(v[ni][4 * i], v[ni][4 * i + 1], v[ni][4 * i + 2], v[ni][4 * i + 3], inv);
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_nop 4");   // wait states between the packs and the swaps (gemm_mx8q.hip permlane_gap)
          __builtin_amdgcn_sched_barrier(0);
          const auto s02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
          const auto s13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
          q16[ni] = make_uint4(s02[0], s02[1], s13[0], s13[1]);
        }
        if (MICLIP_VMCHECK) vm_st += 3;
        if (m < a.M) {
          uint8_t* o = (uint8_t*)a.out + (int64_t)m * a.ldo + cn0 + wc * WTN + 16 * h;
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) *(uint4*)(o + ni * 32) = q16[ni];
          if (h == 0) a.o_scale[mx_scale_index(m, blk, m_pad)] = (uint8_t)(X + 127);
        }
      }
    } else {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int m = cm0 + grp * WTM + mi * 32 + lr;
        if constexpr (EPI == EPI_F32) {
          if (MICLIP_VMCHECK) vm_st += 2 * 4;
          if (m < a.M)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
              for (int i = 0; i < 4; ++i)
                *(float4*)((float*)a.out + (int64_t)m * a.ldo + cn0 + wc * WTN + ni * 32 + 8 * i + 4 * h) =
                    make_float4(val(mi, ni, 4 * i), val(mi, ni, 4 * i + 1), val(mi, ni, 4 * i + 2), val(mi, ni, 4 * i + 3));
          continue;
        }
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int ip = 0; ip < 2; ++ip) {
            const int j0 = 8 * ip, j1 = 8 * ip + 4;
            const uint32_t ax = pack_bf16x2(val(mi, ni, j0), val(mi, ni, j0 + 1));
            const uint32_t ay = pack_bf16x2(val(mi, ni, j0 + 2), val(mi, ni, j0 + 3));
            const uint32_t bx = pack_bf16x2(val(mi, ni, j1), val(mi, ni, j1 + 1));
            const uint32_t by = pack_bf16x2(val(mi, ni, j1 + 2), val(mi, ni, j1 + 3));
            const auto sx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
            const auto sy = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
            if (MICLIP_VMCHECK) ++vm_st;
            if (m < a.M)
              *(uint4*)((uint16_t*)a.out + (int64_t)m * a.ldo + cn0 + wc * WTN + ni * 32 + 16 * ip + 8 * h) =
                  make_uint4(sx[0], sy[0], sx[1], sy[1]);
          }
      }
    }
    if (MICLIP_VMCHECK) vm_count_check<NSTORE>(vm_st);
    if (!has_next) break;
    vb = nvb;
    m0 = nm0;
    n0 = nn0;
    rb = (rb + nk) % RING;
    tpar ^= 1;
    if (cm0 + BM <= a.M) {
      pend = true;
    } else {   // partial tile: an unknown number of stores issued
      pend = false;
      vm_wait_all();
    }
  }
}

// ---------------------------------------------------------------------------
// bf16 -> MX-fp8 (OCP e4m3 + one e8m0 scale per 64 consecutive k): one lane
// per 64-element block.  Shared exponent X = floor(log2(amax)) - 8 (e4m3's
// largest exponent), element = RNE e4m3 of v * 2^-X, saturated to +-448;
// scale byte = X + 127 (amax = 0 -> X = -127).
__global__ __launch_bounds__(256) void quantize_mx_kernel(const uint16_t* __restrict__ in, int64_t ld_in,
                                                          uint8_t* __restrict__ q, int64_t ld_q,
                                                          uint8_t* __restrict__ s, int rows, int K) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nb = K / 64;
  if (i >= (int64_t)rows * nb) return;
  const int64_t r = i / nb;
  const int b = (int)(i % nb);
  const uint4* src = (const uint4*)(in + r * ld_in + b * 64);
  const int rows_pad = (rows + 1) & ~1;
  float v[64];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint4 u = src[c];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[8 * c + 2 * e] = bf2f((uint16_t)(w[e] & 0xffff));
      v[8 * c + 2 * e + 1] = bf2f((uint16_t)(w[e] >> 16));
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 64; ++e) amax = fmaxf(amax, fabsf(v[e]));
  const int X = mx_block_exp(amax);
  const float inv = ldexpf(1.0f, -X);
  uint32_t packed[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) packed[d] = mx_pack4(v[4 * d], v[4 * d + 1], v[4 * d + 2], v[4 * d + 3], inv);
  uint4* dst = (uint4*)(q + r * ld_q + b * 64);
#pragma unroll
  for (int c = 0; c < 4; ++c) dst[c] = make_uint4(packed[4 * c], packed[4 * c + 1], packed[4 * c + 2], packed[4 * c + 3]);
  s[mx_scale_index(r, b, rows_pad)] = (uint8_t)(X + 127);
}

}  // namespace

hipError_t gemm_mx(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  if (a.K % MX_BK || a.N % 256 || a.K <= 0 || !a.a_scale || !a.w_scale) return hipErrorInvalidValue;
  if ((a.lda % 16) || (a.ldw % 16) || (a.ldo % 8) || ((uintptr_t)a.out & 15)) return hipErrorInvalidValue;
  if (epi == EPI_GELU_MX && (a.ldo % 16)) return hipErrorInvalidValue;   // 16-byte fp8 row stores
  const int nt = ((a.M + 255) / 256) * (a.N / 256);
  // default: the ping-pong 32x32x64 kernel (needs K / 64 >= 3 stages).  A/B variants:
  // 1 the double-buffered 16x16x128 kernel; 8 the 8-phase persistent kernel (gemm_mx8q.hip:
  // bit-identical to 1, but 8-30 % slower than the ping-pong kernel at the L/14@336 shapes,
  // scripts/gemm_mx_micro.py — at fp8 rate a K = 1024 tile's MFMAs take half the bf16 time
  // while its epilogue does not shrink)
#if MICLIP_AB
  if (a.variant == 8 && gemm_mx8q_ok(a, epi)) return gemm_mx8q(a, epi, s, cu_count());
  const bool force_dbuf = a.variant == 1;
#else
  if (a.variant != 0) return hipErrorNotSupported;   // kernel overrides exist in the A/B build only
  const bool force_dbuf = false;
#endif
  // persistent ping-pong (round 6; A/B MICLIP_MX_PERSIST=0 keeps one workgroup per tile): at least
  // one tile per CU, whole XCD runs (grid % 8 == 0) and K <= 2048.  At the configs[4] pass shapes
  // (M = 497951, scripts/mx_persist_micro.py, profiles/r06_d_mx_persist_micro.log; bit-identical):
  // c_fc -> MX-fp8 2831 vs 2947 us, qkv 1966 vs 2002, out_proj 686 vs 738; c_proj (K = 4096, a
  // 64-stage main loop) 2119 vs 2009 us, so long-K GEMMs keep one workgroup per tile
  const int cus = cu_count();
  bool persist = nt >= cus && cus % 8 == 0 && a.K <= 2048;
#if MICLIP_AB   // (2: persistent whatever K)
  if (const char* pe = std::getenv("MICLIP_MX_PERSIST"))
    persist = std::atoi(pe) == 2 ? nt >= cus && cus % 8 == 0 : persist && std::atoi(pe) != 0;   // (4: see below)
#endif
  if (!force_dbuf && a.K / 64 >= 3 && persist) {
    // tile order: n-tiles in groups of 6 when there are >= 12 and a group's e4m3 panel fits 2.4 MB
    // (an XCD's 32 concurrent tiles then hold a 1.5-MB panel at K = 1024, not the m-major walk's
    // whole 3-4 MB, which the L2 re-fetched per m-block: FETCH 9x the operand bytes on c_fc,
    // profiles/r06_h_fp8_gemm_traffic.json).  configs[4] shapes, bit-identical
    // (profiles/r06_i_mx_ng.log): c_fc -> MX-fp8 2756 vs 2854 us m-major (groups of 8 2801, 4 2819,
    // 2 2864), qkv 1961 vs 1986 (4: 2049, 2: 2070); out_proj's 4 n-tiles stay m-major
    GemmArgs g = a;
    const int tn = a.N / 256;
    if (g.ngroup == 0) g.ngroup = (tn >= 12 && (int64_t)6 * 256 * a.K <= 2400000) ? 6 : -1;
    bool lean = false;
#if MICLIP_AB   // MICLIP_MX_NG forces the tile-order group width (-1 = m-major); MICLIP_MX_PERSIST=4
                // runs the lean stage loop
    if (const char* ng = std::getenv("MICLIP_MX_NG")) g.ngroup = std::atoi(ng);
    if (const char* pe = std::getenv("MICLIP_MX_PERSIST")) lean = std::atoi(pe) == 4;
#endif
#define MX_PPP(E)                                                                    \
  do {                                                                               \
    if (lean) hipLaunchKernelGGL((gemm_mxppp_kernel<E, true>), dim3(cus), dim3(512), 0, s, g);   \
    else hipLaunchKernelGGL((gemm_mxppp_kernel<E, false>), dim3(cus), dim3(512), 0, s, g);       \
  } while (0)
    switch (epi) {
      case EPI_BF16: MX_PPP(EPI_BF16); break;
      case EPI_GELU_BF16: MX_PPP(EPI_GELU_BF16); break;
      case EPI_F32: MX_PPP(EPI_F32); break;
      case EPI_GELU_MX:
        if (!a.o_scale) return hipErrorInvalidValue;
        MX_PPP(EPI_GELU_MX);
        break;
      default: return hipErrorInvalidValue;
    }
#undef MX_PPP
    return hipGetLastError();
  }
  if (!force_dbuf && a.K / 64 >= 3) {
    GemmArgs g = a;   // (the per-tile kernel walks m-major unless asked: A/B MICLIP_MX_NG)
#if MICLIP_AB
    if (const char* ng = std::getenv("MICLIP_MX_NG")) g.ngroup = std::atoi(ng);
#endif
    switch (epi) {
      case EPI_BF16: hipLaunchKernelGGL(gemm_mxpp_kernel<EPI_BF16>, dim3(nt), dim3(512), 0, s, g); break;
      case EPI_GELU_BF16: hipLaunchKernelGGL(gemm_mxpp_kernel<EPI_GELU_BF16>, dim3(nt), dim3(512), 0, s, g); break;
      case EPI_F32: hipLaunchKernelGGL(gemm_mxpp_kernel<EPI_F32>, dim3(nt), dim3(512), 0, s, g); break;
      case EPI_GELU_MX:
        if (!a.o_scale) return hipErrorInvalidValue;
        hipLaunchKernelGGL(gemm_mxpp_kernel<EPI_GELU_MX>, dim3(nt), dim3(512), 0, s, g);
        break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_mx_kernel<EPI_BF16>, dim3(nt), dim3(512), 0, s, a); break;
    case EPI_GELU_BF16: hipLaunchKernelGGL(gemm_mx_kernel<EPI_GELU_BF16>, dim3(nt), dim3(512), 0, s, a); break;
    case EPI_F32: hipLaunchKernelGGL(gemm_mx_kernel<EPI_F32>, dim3(nt), dim3(512), 0, s, a); break;
    case EPI_GELU_MX:
      if (!a.o_scale) return hipErrorInvalidValue;
      hipLaunchKernelGGL(gemm_mx_kernel<EPI_GELU_MX>, dim3(nt), dim3(512), 0, s, a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t quantize_mx(const uint16_t* in, int64_t ld_in, uint8_t* q, int64_t ld_q, uint8_t* sc, int rows, int K,
                       hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (K % 128 || (ld_in % 8) || (ld_q % 16)) return hipErrorInvalidValue;
  const int64_t n = (int64_t)rows * (K / 64);
  hipLaunchKernelGGL(quantize_mx_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, ld_in, q, ld_q, sc,
                     rows, K);
  return hipGetLastError();
}

}  // namespace miclip
