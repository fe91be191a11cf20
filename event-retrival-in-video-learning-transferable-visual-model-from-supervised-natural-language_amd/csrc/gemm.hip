// bf16 MFMA GEMM with fused CLIP epilogues (gfx950).
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ bias, QuickGELU)
//
// Replaces the nn.Linear / conv1 GEMMs that openai/CLIP's encode_image /
// encode_text run inside PyTorch:
// attn.in_proj (+bias), attn.out_proj (+bias), mlp.c_fc (+bias +QuickGELU,
// transformers/activations.py:117-123), mlp.c_proj (+bias), conv1 as an
// im2col GEMM, and the bias-free CLS projections.  The residual additions
// x += out_proj(..) / c_proj(..) are done by the following LayerNorm kernel
// (encoder.hip residual_ln), so every GEMM epilogue is a pure store.
//
// Tiles (mfma_f32_16x16x32_bf16):
//   256x256, 512 threads = 8 waves (2 M x 4 N), 128x64 per wave — the tower
//     GEMMs: 128 FLOP per staged byte keeps the operand stream at ~half the
//     L2 bandwidth at full MFMA rate (a 128^2 tile would need more than L2 has);
//   128x128, 256 threads = 4 waves (2 x 2), 64x64 per wave — small / ragged N.
//
// Persistent grid, one continuous staging pipeline per workgroup: K is
// consumed in BK = 32 stages held in a 4-deep LDS ring, each loaded by
// 16-byte LDS-DMA (global_load_lds_dwordx4) THREE stages ahead of its use —
// across tile boundaries, so the next tile's first stages are in flight while
// the current tile finishes and stores.  One raw s_barrier per stage, preceded
// by a COUNTED vmcnt that retires only the stage about to be read (a
// __syncthreads() would drain every in-flight load, cdna_hip_programming.md §5
// "Pipelining across barriers").  The epilogue's global stores are younger
// than the next tile's first three stages, so they drain under its first
// three stages of MFMA work (the counts below include them).  Bias lives in
// LDS, so the epilogue issues no vector-memory load.
//
// LDS image: rows of 64 bytes (32 bf16) = four 16-byte chunks; chunk c of row
// r is stored in slot c ^ g[(r >> 2) & 3], g = {0,2,3,1}, which makes the
// 16-lane groups of every ds_read_b128 fragment read hit 16 distinct bank
// slots.  The DMA destination is lane-linear, so the permutation is applied to
// each lane's SOURCE address and again on the read (guide §5.4 rule 21).
//
// The MFMA computes the transposed tile (A operand = W fragment, B operand =
// activation fragment) so each lane holds 4 consecutive output columns of one
// row: 8-byte (bf16) / 16-byte (f32) stores, a wave writing whole 128/256-byte
// row segments over its 4 column fragments.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {

namespace {

constexpr int BK = 32;       // k per stage
constexpr int RING = 4;      // LDS stages
constexpr int LEAD = 3;      // stages in flight ahead of the one being read
// counted waits (common.hpp vm_wait_stages): VMEM ops per wave and stage -- issue_half(st, 0) and
// issue_half(st, 1) (gemm_ppp_kernel's issue: j = 0, 1), each one A and one W 16-row DMA
constexpr int STAGE_OPS = 2 * 2;
static_assert((LEAD - 1) * STAGE_OPS + 16 <= VM_MAX, "counted waits exceed vmcnt's 6-bit field");
constexpr int MAX_N = 4096;  // bias staged in LDS
constexpr int EPI_NONE = 9;  // timing probe (variant 8): main loop only

// QuickGELU x * sigmoid(1.702 x) with the hardware exp/rcp (~1 ulp; output is bf16)
__device__ __forceinline__ float quick_gelu(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v));
}

__device__ __forceinline__ int swz(int x) { return (0x1320 >> (4 * x)) & 0xF; }  // g = {0,2,3,1}

// LDS read the compiler does not see: a plain ds_read of the bias would make
// hipcc wait vmcnt(0) (it cannot prove the read misses the in-flight LDS-DMA
// of the next tile's stages), draining the prefetch at every epilogue.
__device__ __forceinline__ float4 lds_read_f4(const float* p) {
  float4 v;
  const uint32_t addr = (uint32_t)(uintptr_t)(const LDS_AS float*)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// Logical tile t -> (m-block, n-block).  Tiles are taken in groups of `ng`
// n-blocks (ng >= tiles_n: plain m-major raster): within a group all m-blocks
// are swept with the group's n-blocks innermost, so the W column panel of the
// group stays L2-resident while the XCD streams A (each A panel is re-read by
// the ng concurrent tiles of its row).  With xcd_remap each XCD owns a
// contiguous run of t, i.e. one group and a contiguous range of m-blocks.
__device__ __forceinline__ void tile_coords(int t, int tiles_m, int tiles_n, int ng, int& mb, int& nb) {
  if (ng <= 0 || ng >= tiles_n) {
    mb = t / tiles_n;
    nb = t % tiles_n;
    return;
  }
  const int per = tiles_m * ng;
  const int g = t / per, r = t - g * per;
  const int ngg = min(ng, tiles_n - g * ng);
  mb = r / ngg;
  nb = g * ng + r % ngg;
}

template <bool V>
struct BoolT {};

// EPI_SPLIT_GELU (split-f16 GEMM, fp32 tower c_fc): QuickGELU of the f32 pre-activations v
// (columns n .. n + 3 of row m; the f32 epilogue's expf form) scaled by the row's power of two
// and split into the next GEMM's operand [y1 | y1 | y2] (precise.hip split2h_rows, role 0).  The
// scale comes from a bound instead of the row's max, which this tile cannot see:
// |y| <= |v| <= max|a_m| * max_n sum_k |W_nk| + max|b| (with 2^-8 of slack for the f32 rounding
// of v), so |y s| < 2^14 (1 + 2^-8); a loose bound only lowers the subnormal floor's share.
__device__ __forceinline__ int split_exp_g(float mx) {
  if (!(mx > 0.f) || !__builtin_isfinite(mx)) return 0;
  int ex;
  (void)frexpf(mx, &ex);
  const int e = 14 - ex;
  return e > 126 ? 126 : (e < -126 ? -126 : e);
}
__device__ __forceinline__ void split_gelu_store(const GemmArgs& a, int m, int n, float4 v) {
  const float bound = (a.rmax[m] * a.bnd_w + a.bnd_b) * (1.0f + 0.00390625f);
  const int e = split_exp_g(bound);
  const float y[4] = {v.x * (1.0f / (1.0f + expf(-1.702f * v.x))), v.y * (1.0f / (1.0f + expf(-1.702f * v.y))),
                      v.z * (1.0f / (1.0f + expf(-1.702f * v.z))), v.w * (1.0f / (1.0f + expf(-1.702f * v.w)))};
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  _Float16 p1[4], p2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float ys = ldexpf(y[i], e);
    p1[i] = (_Float16)ys;
    const float f1 = (float)p1[i];
    p2[i] = __builtin_isfinite(f1) ? (_Float16)(ys - f1) : (_Float16)0.f;
  }
  const h4 h1 = {p1[0], p1[1], p1[2], p1[3]}, h2 = {p2[0], p2[1], p2[2], p2[3]};
  _Float16* o = (_Float16*)a.out + (int64_t)m * a.ldo + n;
  const int N = a.N;
  *(h4*)o = h1;
  *(h4*)(o + N) = h1;
  *(h4*)(o + 2 * N) = h2;
  if (n == 0) a.rsc_out[m] = ldexpf(1.f, -e);
}
typedef _Float16 f16x8_g __attribute__((ext_vector_type(8)));
// one 16x16x32 MFMA on bf16 or (split-f16 operands) fp16 fragments of the same bytes
__device__ __forceinline__ f32x4 mfma16(BoolT<false>, bf16x8 b, bf16x8 a, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(BoolT<true>, bf16x8 b, bf16x8 a, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_g, b), __builtin_bit_cast(f16x8_g, a), c, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  // retire all but the N youngest vector-memory ops of this wave, then a raw
  // workgroup barrier; "memory" keeps the compiler from moving LDS accesses across
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}

// F16: fp16 operands on the f16 MFMA (split-f16 operands of the fp32 tower, GemmArgs rsc / csc)
template <int EPI, int BM, int BN, int WAVES_M, int WAVES_N, bool F16 = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_kernel(GemmArgs a) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int NWAVES = WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;  // per-wave tile
  constexpr int MI = WTM / 16, NI = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, STAGE_BYTES = (BM + BN) * BK * 2;
  constexpr int GA = BM / 16 / NWAVES;     // A DMA instructions per wave per stage (16 rows each)
  constexpr int GB = BN / 16 / NWAVES;
  constexpr int PS = GA + GB;              // vmcnt units per stage
  constexpr int S = MI * NI;               // epilogue stores per lane
  static_assert(2 * PS + S <= 63, "vmcnt field is 6 bits");
  __shared__ __attribute__((aligned(16))) char smem[RING * STAGE_BYTES + MAX_N * 4];
  float* sbias = (float*)(smem + RING * STAGE_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);  // XCD-contiguous runs of tiles per round
  if (slot >= ntiles) return;
  const int my_tiles = (ntiles - 1 - slot) / G + 1;
  const int nk = a.K / BK;
  const int T = my_tiles * nk;                 // stages this workgroup consumes

  for (int i = tid; i < a.N; i += NT) sbias[i] = a.bias ? a.bias[i] : 0.f;
  __syncthreads();

  // ---- issuer: DMA geometry — instruction j of wave w fills LDS bytes
  // [(w*G+j)*1024, +1024) = tile rows (w*G+j)*16 .. +15; lane i -> row +(i>>2),
  // slot (i&3) holding global chunk (i&3) ^ g[i>>4]  ((row>>2)&3 == i>>4).
  const int lrow = lane >> 2;
  const int lchunk = ((lane & 3) ^ swz(lane >> 4)) * 8;
  const uint16_t* asrc[GA];
  const uint16_t* wsrc[GB];
  int is_g = 0, is_kt = 0, is_tile = 0;
  auto set_src = [&](int t) {
    const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
#pragma unroll
    for (int j = 0; j < GA; ++j)
      asrc[j] = a.A + (int64_t)min(m0 + (wave * GA + j) * 16 + lrow, a.M - 1) * a.lda + lchunk;
#pragma unroll
    for (int j = 0; j < GB; ++j) wsrc[j] = a.W + (int64_t)(n0 + (wave * GB + j) * 16 + lrow) * a.ldw + lchunk;
  };
  auto issue = [&]() {
    char* base = smem + (is_g % RING) * STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < GA; ++j) glds16(asrc[j] + is_kt * BK, base + (wave * GA + j) * 1024);
#pragma unroll
    for (int j = 0; j < GB; ++j) glds16(wsrc[j] + is_kt * BK, base + A_BYTES + (wave * GB + j) * 1024);
    ++is_g;
    if (++is_kt == nk) {
      is_kt = 0;
      if (++is_tile < my_tiles) set_src(slot + is_tile * G);
    }
  };
  set_src(slot);
  for (int s = 0; s < LEAD; ++s)
    if (is_g < T) issue();

  // ---- consumer
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  // fragment read: row (lane&15) of a 16-row block, chunk (lane>>4)
  const int rd = (lane & 15) * 64 + (((lane >> 4) ^ swz((lane >> 2) & 3)) * 16);
  bool pend = false;  // previous tile's S stores are still counted in vmcnt
  int g = 0;
  for (int ti = 0; ti < my_tiles; ++ti) {
    const int t = slot + ti * G;
    const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
    f32x4 acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt, ++g) {
      // stage g must have landed; younger ops: up to LEAD-1 stages, plus the
      // previous epilogue's stores while stage g predates them (kt < LEAD)
      const int ys = min(LEAD - 1, T - 1 - g);
      const bool st = pend && kt < LEAD;
      if (nk < LEAD) wait_vm_barrier<0>();
      else if (ys == 2) { if (st) wait_vm_barrier<2 * PS + S>(); else wait_vm_barrier<2 * PS>(); }
      else if (ys == 1) { if (st) wait_vm_barrier<PS + S>(); else wait_vm_barrier<PS>(); }
      else { if (st) wait_vm_barrier<S>(); else wait_vm_barrier<0>(); }
      if (is_g < T) issue();
      const char* As = smem + (g % RING) * STAGE_BYTES;
      const char* Ws = As + A_BYTES;
      bf16x8 bfr[NI], af[MI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bfr[ni] = *(const bf16x8*)(Ws + (wc * WTN + ni * 16) * 64 + rd);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) af[mi] = *(const bf16x8*)(As + (wr * WTM + mi * 16) * 64 + rd);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = mfma16(BoolT<F16>{}, bfr[ni], af[mi], acc[mi][ni]);
    }

    // ---------------------------------------------------------- epilogue
    // lane: output row m = m0 + wr*WTM + mi*16 + (lane&15),
    //       columns  n = n0 + wc*WTN + ni*16 + 4*(lane>>4) + 0..3
    const bool tail = m0 + BM > a.M;
    float4 bias[NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bias[ni] = lds_read_f4(sbias + n0 + wc * WTN + ni * 16 + 4 * (lane >> 4));
    float4 csc[NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
      csc[ni] = F16 ? *(const float4*)(a.csc + n0 + wc * WTN + ni * 16 + 4 * (lane >> 4)) : make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = m0 + wr * WTM + mi * 16 + (lane & 15);
      if (tail && m >= a.M) continue;
      int64_t orow = m;
      if (a.group) orow = (int64_t)(m / a.group) * a.gstride + a.goffset + m % a.group;
      const float rs = F16 ? a.rsc[m] : 1.f;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int n = n0 + wc * WTN + ni * 16 + 4 * (lane >> 4);
        if (F16) {   // split-f16 operands: 1 / (s_row s_col), exact (powers of two)
          acc[mi][ni][0] *= rs * csc[ni].x; acc[mi][ni][1] *= rs * csc[ni].y;
          acc[mi][ni][2] *= rs * csc[ni].z; acc[mi][ni][3] *= rs * csc[ni].w;
        }
        float v0 = acc[mi][ni][0] + bias[ni].x, v1 = acc[mi][ni][1] + bias[ni].y;
        float v2 = acc[mi][ni][2] + bias[ni].z, v3 = acc[mi][ni][3] + bias[ni].w;
        if (EPI == EPI_BF16 || EPI == EPI_GELU_BF16) {
          if (EPI == EPI_GELU_BF16) {
            v0 = quick_gelu(v0); v1 = quick_gelu(v1); v2 = quick_gelu(v2); v3 = quick_gelu(v3);
          }
          *(uint2*)((uint16_t*)a.out + orow * a.ldo + n) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        } else if (EPI == EPI_F32) {
          *(float4*)((float*)a.out + orow * a.ldo + n) = make_float4(v0, v1, v2, v3);
        } else if constexpr (EPI == EPI_SPLIT_GELU) {
          split_gelu_store(a, m, n, make_float4(v0, v1, v2, v3));
        } else {  // EPI_RESID_F32 (operator API only): read-modify-write, not overlapped
          float4* dst = (float4*)((float*)a.out + orow * a.ldo + n);
          const float4 o = *dst;
          *dst = make_float4(o.x + v0, o.y + v1, o.z + v2, o.w + v3);
        }
      }
    }
    // a tail tile issues fewer than S stores (and the residual form issues
    // loads): drain so the counted waits stay exact
    if (tail || EPI == EPI_RESID_F32 || EPI == EPI_SPLIT_GELU) {   // (the split form: 3 stores + a load each)
      vm_wait_all();
      pend = false;
    } else {
      pend = true;
    }
  }
}

// ---------------------------------------------------------------------------
// Ping-pong schedule (variant 2): the 8 waves form two groups (waves 0-3 and
// 4-7; waves w and w+4 share a SIMD), each owning 128 rows of the 256x256
// tile.  A wave alternates LOAD sections (issue its share of the LDS-DMA for a
// stage three ahead, ds_read the fragments of its next MFMA cluster,
// lgkmcnt(0)) and COMPUTE sections (16 MFMAs); every section ends at a
// workgroup barrier.  Group 1 runs one section behind group 0, so in every
// section one wave of each SIMD feeds the matrix pipe while its partner loads
// (cdna_hip_programming.md §5 "8-phase template", MI355X_MICROARCH.md "Two
// waves per SIMD").  Per BK=32 stage: L_a (A frags 0-3, B frags) | C_a (16
// MFMA) | L_b (A frags 4-7) | C_b (16 MFMA).  RAW on a stage: every wave
// retires its DMA for stage g+1 (counted vmcnt) before the barrier that opens
// stage g+1's first LOAD section — group 0 at the end of C_b(g), group 1 at
// the end of L_b(g).  WAR: stage g+3 is issued in L sections of stage g, after
// every read of the buffer it overwrites (stage g-1, last read by group 1 in
// L_b(g-1), which ends with lgkmcnt(0) + barrier).
//
// PATCH (patch embedding, a.patch_R = R > 0): A is the bf16 NCHW pixel tensor
// and output row m is patch m % G^2 of frame m / G^2 (G = R / 32).  With
// P = 32 a BK = 32 stage st is one contiguous 32-pixel segment of an image
// row (channel st / 32, patch row st % 32), so the DMA source of row m at
// stage st is pix(m) + (st >> 5) * R^2 + (st & 31) * R: the im2col gather
// rides on the LDS-DMA address and no patch matrix is written or read.
template <int EPI, int CL, bool PRIO, bool DIRECT = false, bool NTS = false, bool PATCH = false, bool F16 = false>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs a) {
  constexpr int BM = 256, BN = 256, NT = 512;
  constexpr int WTM = 128, WTN = 64;
  constexpr int A_BYTES = BM * BK * 2, STAGE_BYTES = (BM + BN) * BK * 2;
  constexpr int LDS = (RING * STAGE_BYTES > BM * (BN * 2 + 16) ? RING * STAGE_BYTES : BM * (BN * 2 + 16)) >
                              (WTM * (BN * 4 + 16))
                          ? (RING * STAGE_BYTES > BM * (BN * 2 + 16) ? RING * STAGE_BYTES : BM * (BN * 2 + 16))
                          : (WTM * (BN * 4 + 16));
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  int m0, n0;
  tile_coords(xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, a.ngroup, m0, n0);
  m0 *= BM;
  n0 *= BN;
  const int nk = a.K / BK;

  // DMA: per stage each wave issues A rows (wave*2+j)*16.. and W rows likewise (j = 0,1)
  const int lrow = lane >> 2;
  const int lchunk = ((lane & 3) ^ swz(lane >> 4)) * 8;
  const uint16_t* asrc[2];
  const uint16_t* wsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = min(m0 + (wave * 2 + j) * 16 + lrow, a.M - 1);
    if (PATCH) {
      const int R = a.patch_R, G = R >> 5, p = m % (G * G);
      asrc[j] = a.A + ((int64_t)(m / (G * G)) * 3 * R + (p / G) * 32) * R + (p % G) * 32 + lchunk;
    } else {
      asrc[j] = a.A + (int64_t)m * a.lda + lchunk;
    }
    wsrc[j] = a.W + (int64_t)(n0 + (wave * 2 + j) * 16 + lrow) * a.ldw + lchunk;
  }
  auto a_off = [&](int st) -> int64_t {
    if (PATCH) return (int64_t)(st >> 5) * a.patch_R * a.patch_R + (st & 31) * a.patch_R;
    return (int64_t)st * BK;
  };
  auto issue_half = [&](int st, int j) {
    char* base = smem + (st % RING) * STAGE_BYTES;
    glds16(asrc[j] + a_off(st), base + (wave * 2 + j) * 1024);
    glds16(wsrc[j] + st * BK, base + A_BYTES + (wave * 2 + j) * 1024);
  };
  auto wait_stage = [&](int g1) {  // retire this wave's DMA for stage g1 (STAGE_OPS per younger stage)
    const int younger = min(LEAD - 1, nk - 1 - g1);
    vm_wait_stages<STAGE_OPS, LEAD - 1>(younger);
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
  for (int s = 0; s < LEAD; ++s)
    if (s < nk) { issue_half(s, 0); issue_half(s, 1); }
  wait_stage(0);
  barrier();
  if (grp == 1) barrier();

  const int rd = (lane & 15) * 64 + (((lane >> 4) ^ swz((lane >> 2) & 3)) * 16);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 bfr[4], af[8 / CL];

  auto mfma_cluster = [&](int mbase, int count) {
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[mbase + mi][ni] = mfma16(BoolT<F16>{}, bfr[ni], af[(mbase % (8 / CL)) + mi], acc[mbase + mi][ni]);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    (void)count;
  };
  for (int g = 0; g < nk; ++g) {
    const char* As = smem + (g % RING) * STAGE_BYTES + (grp * WTM) * 64;
    const char* Ws = smem + (g % RING) * STAGE_BYTES + A_BYTES + (wc * WTN) * 64;
    if (CL == 2) {
      // ---- L_a
      if (g + LEAD < nk) issue_half(g + LEAD, 0);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = *(const bf16x8*)(Ws + ni * 16 * 64 + rd);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi] = *(const bf16x8*)(As + mi * 16 * 64 + rd);
      lgkm_barrier();
      // ---- C_a
      mfma_cluster(0, 16);
      barrier();
      // ---- L_b
      if (g + LEAD < nk) issue_half(g + LEAD, 1);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi] = *(const bf16x8*)(As + (mi + 4) * 16 * 64 + rd);
      if (grp == 1 && g + 1 < nk) wait_stage(g + 1);
      lgkm_barrier();
      // ---- C_b
      mfma_cluster(4, 16);
      if (grp == 0 && g + 1 < nk) wait_stage(g + 1);
      barrier();
    } else {
      // ---- L: all fragments of the stage + the whole DMA share of stage g+3
      if (g + LEAD < nk) { issue_half(g + LEAD, 0); issue_half(g + LEAD, 1); }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = *(const bf16x8*)(Ws + ni * 16 * 64 + rd);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) af[mi] = *(const bf16x8*)(As + mi * 16 * 64 + rd);
      if (grp == 1 && g + 1 < nk) wait_stage(g + 1);
      lgkm_barrier();
      // ---- C: 32 MFMAs
      mfma_cluster(0, 16);
      mfma_cluster(4, 16);
      if (grp == 0 && g + 1 < nk) wait_stage(g + 1);
      barrier();
    }
  }
  if (grp == 0) barrier();
  if (!DIRECT) __syncthreads();
  if (EPI == EPI_NONE) {  // timing probe: nothing stored, every accumulator kept live
    float t = 0.f;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) t += acc[mi][ni][0] + acc[mi][ni][1] + acc[mi][ni][2] + acc[mi][ni][3];
    if (t == 12345.f && a.M < 0) *(float*)a.out = t;
    return;
  }

  // ------------------------------------------------ epilogue
  const int wr = grp;
  float4 bias[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wc * WTN + ni * 16 + 4 * (lane >> 4);
    bias[ni] = a.bias ? *(const float4*)(a.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto out_row = [&](int m) -> int64_t {
    return a.group ? (int64_t)(m / a.group) * a.gstride + a.goffset + m % a.group : (int64_t)m;
  };
  if (DIRECT && (EPI == EPI_BF16 || EPI == EPI_GELU_BF16)) {
    // Direct row stores, no LDS round trip or workgroup barrier.  Fragments
    // ni and ni+1 of a 16-row block are exchanged across 16-lane rows with
    // v_permlane16_swap (odd row of the first <-> even row of the second), so
    // lane (r, g) ends up with 8 consecutive bf16 columns of row r:
    //   g = 0: ni*16 + 0..7   g = 1: (ni+1)*16 + 0..7
    //   g = 2: ni*16 + 8..15  g = 3: (ni+1)*16 + 8..15
    // -> one 16-byte store per lane per fragment pair, 64 contiguous bytes per
    // row per instruction (cdna_hip_programming.md T21, 16-lane form).
    const int g = lane >> 4;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = m0 + wr * WTM + mi * 16 + (lane & 15);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint2 pk[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ni = 2 * p + q;
          float v0 = acc[mi][ni][0] + bias[ni].x, v1 = acc[mi][ni][1] + bias[ni].y;
          float v2 = acc[mi][ni][2] + bias[ni].z, v3 = acc[mi][ni][3] + bias[ni].w;
          if (EPI == EPI_GELU_BF16) {
            v0 = quick_gelu(v0); v1 = quick_gelu(v1); v2 = quick_gelu(v2); v3 = quick_gelu(v3);
          }
          pk[q] = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        }
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
        const int col = n0 + wc * WTN + (2 * p + (g & 1)) * 16 + (g >> 1) * 8;
        if (m < a.M) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          u32x4* dst = (u32x4*)((uint16_t*)a.out + out_row(m) * a.ldo + col);
          const u32x4 val = {sx[0], sy[0], sx[1], sy[1]};
          if (NTS) __builtin_nontemporal_store(val, dst);
          else *dst = val;
        }
      }
    }
  } else if (EPI == EPI_BF16 || EPI == EPI_GELU_BF16) {
    constexpr int RS = BN * 2 + 16;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        float v0 = acc[mi][ni][0] + bias[ni].x, v1 = acc[mi][ni][1] + bias[ni].y;
        float v2 = acc[mi][ni][2] + bias[ni].z, v3 = acc[mi][ni][3] + bias[ni].w;
        if (EPI == EPI_GELU_BF16) {
          v0 = quick_gelu(v0); v1 = quick_gelu(v1); v2 = quick_gelu(v2); v3 = quick_gelu(v3);
        }
        const int r = wr * WTM + mi * 16 + (lane & 15);
        const int c = wc * WTN + ni * 16 + 4 * (lane >> 4);
        *(uint2*)(smem + r * RS + c * 2) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
      }
    __syncthreads();
    constexpr int CH = BN / 8;
#pragma unroll 4
    for (int f = tid; f < BM * CH; f += NT) {
      const int r = f / CH, c8 = f % CH;
      const int m = m0 + r;
      if (m < a.M)
        *(uint4*)((uint16_t*)a.out + out_row(m) * a.ldo + n0 + c8 * 8) = *(const uint4*)(smem + r * RS + c8 * 16);
    }
  } else {
    constexpr int RS = BN * 4 + 16;
    float4 csc[4];   // split-f16 operands: 1 / (s_row s_col) on the accumulator (exact)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      csc[ni] = F16 ? *(const float4*)(a.csc + n0 + wc * WTN + ni * 16 + 4 * (lane >> 4)) : make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (wr == p) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
          const int mr = min(m0 + wr * WTM + mi * 16 + (lane & 15), a.M - 1);
          const float rs = F16 ? a.rsc[mr] : 1.f;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            const int r = mi * 16 + (lane & 15);
            const int c = wc * WTN + ni * 16 + 4 * (lane >> 4);
            f32x4 v = acc[mi][ni];
            if (F16) v = v * (f32x4){rs * csc[ni].x, rs * csc[ni].y, rs * csc[ni].z, rs * csc[ni].w};
            *(float4*)(smem + r * RS + c * 4) =
                make_float4(v[0] + bias[ni].x, v[1] + bias[ni].y, v[2] + bias[ni].z, v[3] + bias[ni].w);
          }
        }
      }
      __syncthreads();
      constexpr int C4 = BN / 4;
#pragma unroll 4
      for (int f = tid; f < WTM * C4; f += NT) {
        const int r = f / C4, c4 = f % C4;
        const int m = m0 + p * WTM + r;
        if (m < a.M) {
          const float4 v = *(const float4*)(smem + r * RS + c4 * 16);
          if constexpr (EPI == EPI_SPLIT_GELU) {
            split_gelu_store(a, m, n0 + c4 * 4, v);
            continue;
          }
          float4* dst = (float4*)((float*)a.out + out_row(m) * a.ldo + n0 + c4 * 4);
          if (EPI == EPI_RESID_F32) {
            const float4 o = *dst;
            *dst = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
          } else {
            *dst = v;
          }
        }
      }
      if (p == 0) __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// Main-loop ablation probes (variants 31-33, scripts/gemm_micro.py; no
// epilogue, like variant 8): gemm_pp_kernel<EPI_NONE, 1>'s schedule with one
// component removed, to see which one sets the stage time.
//   31: no LDS-DMA (the MFMAs read whatever the ring holds)
//   32: no fragment ds_reads (the MFMAs reuse the first stage's fragments)
//   33: no MFMAs (the fragments are kept live by an empty asm)
template <int ABL>
__global__ __launch_bounds__(512) void gemm_abl_kernel(GemmArgs a) {
  constexpr int BM = 256, BN = 256;
  constexpr int WTM = 128, WTN = 64;
  constexpr int A_BYTES = BM * BK * 2, STAGE_BYTES = (BM + BN) * BK * 2;
  __shared__ __attribute__((aligned(16))) char smem[RING * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  int m0, n0;
  tile_coords(xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, 0, m0, n0);
  m0 *= BM;
  n0 *= BN;
  const int nk = a.K / BK;
  const int lrow = lane >> 2;
  const int lchunk = ((lane & 3) ^ swz(lane >> 4)) * 8;
  const uint16_t* asrc[2];
  const uint16_t* wsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    asrc[j] = a.A + (int64_t)min(m0 + (wave * 2 + j) * 16 + lrow, a.M - 1) * a.lda + lchunk;
    wsrc[j] = a.W + (int64_t)(n0 + (wave * 2 + j) * 16 + lrow) * a.ldw + lchunk;
  }
  // ABL 4/5: the same bytes per stage, fetched as full 128-byte row lines
  // (8 rows x 128 B per instruction: rows of half (st & 1), k in [64*(st>>1), +64))
  // instead of 16 rows x 64 B; the data is wrong, the timing shows the cost of
  // half-line pieces.
  const int frow = lane >> 3, fcol = (lane & 7) * 8;
  auto issue_half = [&](int st, int j) {
    if (ABL == 1) return;
    char* base = smem + (st % RING) * STAGE_BYTES;
    if (ABL == 4 || ABL == 5) {
      const int r0 = (st & 1) * 128 + (wave * 2 + j) * 8 + frow;
      const int64_t k0 = (int64_t)(st >> 1) * 64 + fcol;
      glds16(a.A + (int64_t)min(m0 + r0, a.M - 1) * a.lda + k0, base + (wave * 2 + j) * 1024);
      glds16(a.W + (int64_t)(n0 + r0) * a.ldw + k0, base + A_BYTES + (wave * 2 + j) * 1024);
      return;
    }
    glds16(asrc[j] + (int64_t)st * BK, base + (wave * 2 + j) * 1024);
    glds16(wsrc[j] + st * BK, base + A_BYTES + (wave * 2 + j) * 1024);
  };
  auto wait_stage = [&](int g1) {  // retire this wave's DMA for stage g1 (STAGE_OPS per younger stage)
    const int younger = min(LEAD - 1, nk - 1 - g1);
    vm_wait_stages<STAGE_OPS, LEAD - 1>(younger);
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
  for (int s = 0; s < LEAD; ++s)
    if (s < nk) { issue_half(s, 0); issue_half(s, 1); }
  wait_stage(0);
  barrier();
  if (grp == 1) barrier();
  const int rd = (lane & 15) * 64 + (((lane >> 4) ^ swz((lane >> 2) & 3)) * 16);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 bfr[4], af[8];
  {
    const char* As = smem + (grp * WTM) * 64;
    const char* Ws = smem + A_BYTES + (wc * WTN) * 64;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) bfr[ni] = *(const bf16x8*)(Ws + ni * 16 * 64 + rd);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) af[mi] = *(const bf16x8*)(As + mi * 16 * 64 + rd);
  }
  for (int g = 0; g < nk; ++g) {
    const char* As = smem + (g % RING) * STAGE_BYTES + (grp * WTM) * 64;
    const char* Ws = smem + (g % RING) * STAGE_BYTES + A_BYTES + (wc * WTN) * 64;
    if (g + LEAD < nk) { issue_half(g + LEAD, 0); issue_half(g + LEAD, 1); }
    if (ABL != 2) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = *(const bf16x8*)(Ws + ni * 16 * 64 + rd);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) af[mi] = *(const bf16x8*)(As + mi * 16 * 64 + rd);
    }
    if (grp == 1 && g + 1 < nk) wait_stage(g + 1);
    lgkm_barrier();
    if (ABL == 3 || ABL == 4) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) asm volatile("" ::"v"(bfr[ni]));
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) asm volatile("" ::"v"(af[mi]));
    } else {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
    }
    if (grp == 0 && g + 1 < nk) wait_stage(g + 1);
    barrier();
  }
  if (grp == 0) barrier();
  float t = 0.f;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) t += acc[mi][ni][0] + acc[mi][ni][1] + acc[mi][ni][2] + acc[mi][ni][3];
  if (t == 12345.f && a.M < 0) *(float*)a.out = t;
}

// ---------------------------------------------------------------------------
// Persistent ping-pong (variant 18, bf16 outputs): gemm_pp_kernel's schedule
// (CL = 1) with one workgroup per CU walking its tiles, so a tile's epilogue
// overlaps the next tile's prologue and store drain:
//   the stages of all of a workgroup's tiles are one stream through the ring:
//   the NEXT tile's first LEAD stages (and its bias) are issued in this tile's
//   last LEAD main-loop iterations, into the ring slots a continuous pipeline
//   would use (same WAR rule as inside a tile), so they have landed by the end
//   of this tile's direct-store epilogue.  The 16 stores per wave are younger
//   than those three stages and older than every later one, so the counted
//   waits of the next tile add the stores only while waiting for stages < LEAD;
//   the first wait that has to cover them is stage LEAD's, three stages (~3k
//   cycles) after they issued.  (Issuing the next tile's stages only after the
//   main loop, the previous form, measured 0-4 % slower.)
//   A partial last m-tile (lanes with m >= M skip their stores) drains with
//   vmcnt(0) instead, since its store count is not the fixed 16.
//   A tile's bias (256 f32) is LDS-DMA'd by wave 0 into one of two LDS slots
//   (tile parity; the previous tile's epilogue finished reading the slot
//   before this tile started) just before that tile's first stages are issued: older than
//   them, it has landed once the tile's first stage wait + barrier return, and
//   the epilogue reads it with an LDS read hipcc does not see.  A plain global
//   load of the bias there made hipcc drain the prefetch with vmcnt(0).
// Timing probe (variant 19, scripts/gemm_micro.py): s_memrealtime stamps
// (100 MHz) of each workgroup's third tile - main loop start, main loop end,
// epilogue stores issued, next tile's main loop start - kept in SGPRs and
// written once at kernel end (a mid-loop store would break the counted waits).
__device__ unsigned long long g_gemm_probe[4096 * 4];

// EARLY (variant 20): group 0, one section ahead, issues its epilogue during
// group 1's last MFMA section and realigns afterwards (same barrier count).
template <int EPI, bool PROBE = false, bool EARLY = false, bool NTS = false>
__global__ __launch_bounds__(512) void gemm_ppp_kernel(GemmArgs a) {
  constexpr int BM = 256, BN = 256;
  constexpr int WTM = 128, WTN = 64;
  constexpr int A_BYTES = BM * BK * 2, STAGE_BYTES = (BM + BN) * BK * 2;
  constexpr int NSTORE = 8 * 2;  // epilogue store instructions per wave of a full tile: (mi, p)
  __shared__ __attribute__((aligned(16))) char smem[RING * STAGE_BYTES + 2 * BN * 4];
  float* sbias = (float*)(smem + RING * STAGE_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wave >> 2), wc = wave & 3;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int nk = a.K / BK;
  int vb = blockIdx.x;
  int m0, n0;
  auto coords = [&](int v, int& mm, int& nn) {
    const int t = xcd_remap(v, ntiles);  // grid % 8 == 0 keeps a WG's tiles on its XCD's contiguous run
    int mb, nb;
    tile_coords(t, tiles_m, tiles_n, a.ngroup, mb, nb);   // ngroup 0: m-major raster
    mm = mb * BM;
    nn = nb * BN;
  };
  coords(vb, m0, n0);

  const int lrow = lane >> 2;
  const int lchunk = ((lane & 3) ^ swz(lane >> 4)) * 8;
  const uint16_t* asrc[2];
  const uint16_t* wsrc[2];
  auto set_src = [&](int mm, int nn) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      asrc[j] = a.A + (int64_t)min(mm + (wave * 2 + j) * 16 + lrow, a.M - 1) * a.lda + lchunk;
      wsrc[j] = a.W + (int64_t)(nn + (wave * 2 + j) * 16 + lrow) * a.ldw + lchunk;
    }
  };
  auto issue = [&](int st, int slot) {  // stage st of the tile set_src points at -> ring slot
    char* base = smem + slot * STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      glds16(asrc[j] + st * BK, base + (wave * 2 + j) * 1024);
      glds16(wsrc[j] + st * BK, base + A_BYTES + (wave * 2 + j) * 1024);
    }
  };
  bool pend = false;  // the previous tile's NSTORE stores are in flight, younger than stages 0..LEAD-1
  // The stages of a workgroup's tiles form ONE stream through the ring: the
  // next tile's first LEAD stages are issued in this tile's last LEAD main-loop
  // iterations (where a single tile's pipeline would run dry), so they have
  // landed before the epilogue ends.  rb = ring slot of this tile's stage 0.
  int rb = 0, nm0 = 0, nn0 = 0;
  bool has_next = false;
  auto wait_stage = [&](int g1) {   // STAGE_OPS per younger stage (+ the previous tile's NSTORE stores)
    const int younger = has_next ? LEAD - 1 : min(LEAD - 1, nk - 1 - g1);
    if (g1 < LEAD && pend) vm_wait_stages<STAGE_OPS, LEAD - 1, NSTORE>(younger);
    else vm_wait_stages<STAGE_OPS, LEAD - 1>(younger);
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

  const int g = lane >> 4;
  int tpar = 0;  // tile parity: bias slot
  auto load_bias = [&](int slot, int nn) {  // wave 0: 64 lanes x 16 B = the tile's 256 bias values
    if (wave == 0 && a.bias) glds16(a.bias + nn + lane * 4, sbias + slot * BN);
  };
  load_bias(0, n0);
  set_src(m0, n0);
#pragma unroll
  for (int st = 0; st < LEAD; ++st)
    if (st < nk) issue(st, st);
  const int rd = (lane & 15) * 64 + (((lane >> 4) ^ swz((lane >> 2) & 3)) * 16);
  int ti = 0;
  unsigned long long ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0;
  while (true) {
    const int nvb = vb + gridDim.x;
    has_next = nvb < ntiles;
    if (has_next) coords(nvb, nm0, nn0);
    wait_stage(0);
    barrier();
    if (grp == 1) barrier();
    if (PROBE) {
      if (ti == 2) ts0 = __builtin_amdgcn_s_memrealtime();
      if (ti == 3) ts3 = __builtin_amdgcn_s_memrealtime();
    }
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 bfr[4], af[8];
    for (int gs = 0; gs < nk; ++gs) {
      const int slot = (rb + gs) % RING;
      const char* As = smem + slot * STAGE_BYTES + (grp * WTM) * 64;
      const char* Ws = smem + slot * STAGE_BYTES + A_BYTES + (wc * WTN) * 64;
      if (gs + LEAD < nk) {
        issue(gs + LEAD, (rb + gs + LEAD) % RING);
      } else if (has_next) {  // the next tile's stage gs + LEAD - nk, same ring position in the stream
        const int st = gs + LEAD - nk;
        if (st == 0) {
          load_bias(tpar ^ 1, nn0);
          set_src(nm0, nn0);
        }
        issue(st, (rb + gs + LEAD) % RING);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = *(const bf16x8*)(Ws + ni * 16 * 64 + rd);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) af[mi] = *(const bf16x8*)(As + mi * 16 * 64 + rd);
      if (grp == 1 && gs + 1 < nk) wait_stage(gs + 1);
      lgkm_barrier();
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
      if (grp == 0 && gs + 1 < nk) wait_stage(gs + 1);
      barrier();
    }
    if (!EARLY && grp == 0) barrier();  // groups realigned; every ring read of this tile is done
    if (PROBE && ti == 2) ts1 = __builtin_amdgcn_s_memrealtime();

    // the next tile's first stages are already in flight (issued in the main loop)
    const int cm0 = m0, cn0 = n0;
    // ---- epilogue of tile (cm0, cn0): direct permlane-swapped row stores (gemm_pp_kernel DIRECT)
    int vm_st = 0;   // store instructions of a full tile (MICLIP_VMCHECK: checked against NSTORE)
    float4 bias[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      bias[ni] = a.bias ? lds_read_f4(sbias + tpar * BN + wc * WTN + ni * 16 + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = cm0 + grp * WTM + mi * 16 + (lane & 15);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint2 pk[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ni = 2 * p + q;
          float v0 = acc[mi][ni][0] + bias[ni].x, v1 = acc[mi][ni][1] + bias[ni].y;
          float v2 = acc[mi][ni][2] + bias[ni].z, v3 = acc[mi][ni][3] + bias[ni].w;
          if (EPI == EPI_GELU_BF16) {
            v0 = quick_gelu(v0); v1 = quick_gelu(v1); v2 = quick_gelu(v2); v3 = quick_gelu(v3);
          }
          pk[q] = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        }
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[0].x, pk[1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[0].y, pk[1].y, false, false);
        const int col = cn0 + wc * WTN + (2 * p + (g & 1)) * 16 + (g >> 1) * 8;
        if (MICLIP_VMCHECK) ++vm_st;
        if (m < a.M) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          u32x4* dst = (u32x4*)((uint16_t*)a.out + (int64_t)m * a.ldo + col);
          const u32x4 val = {sx[0], sy[0], sx[1], sy[1]};
          if (NTS) __builtin_nontemporal_store(val, dst);
          else *dst = val;
        }
      }
    }
    if (MICLIP_VMCHECK) vm_count_check<NSTORE>(vm_st);
    if (EARLY && grp == 0) barrier();
    if (PROBE && ti == 2) ts2 = __builtin_amdgcn_s_memrealtime();
    ++ti;
    if (!has_next) break;
    vb = nvb;
    m0 = nm0;
    n0 = nn0;
    rb = (rb + nk) % RING;
    tpar ^= 1;
    if (cm0 + BM <= a.M) {
      pend = true;
    } else {  // partial tile: an unknown number of stores issued
      pend = false;
      vm_wait_all();
    }
  }
  if (PROBE && wave == 0 && lane == 0 && blockIdx.x < 4096) {
    unsigned long long* d = g_gemm_probe + blockIdx.x * 4;
    d[0] = ts0; d[1] = ts1; d[2] = ts2; d[3] = ts3;
  }
}

}  // namespace

int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

namespace {

// n-blocks per tile group (tile_coords): the largest divisor of tiles_n whose
// W panel (ng x 256 rows x K bf16) fits ~1.6 MB of the XCD's 4 MB L2; 0 (plain
// m-major) when even one n-block's panel does not fit or all of W fits.
int n_group(int tiles_n, int K) {
  const int64_t panel = 256LL * K * 2;
  if (tiles_n * panel <= (1 << 21)) return 0;
  for (int ng = tiles_n - 1; ng >= 2; --ng)
    if (tiles_n % ng == 0 && ng * panel <= 1677722) return ng;
  return 0;
}

#if MICLIP_AB
// A/B build (scripts/ab, MICLIP_AB=1): every schedule, ablation and probe
// variant of rounds 1-2 stays selectable by GemmArgs::variant for
// scripts/gemm_micro.py and the bit-identity tests; the product library
// (MICLIP_AB=0) compiles only the default path below.
template <int EPI>
hipError_t launch_ab(const GemmArgs& a, hipStream_t s) {
  const bool big = a.N % 256 == 0 && a.M >= 1024;
  // variant 0 (default): ping-pong, one 32-MFMA cluster per stage, direct
  // permlane-swapped row stores for bf16 outputs (16, or its persistent form
  // 18 on wide N) / LDS-staged rows for f32 (3) (scripts/gemm_micro.py);
  // 1 = persistent ring; 8 = main-loop-only timing probe (no epilogue).
  const bool bf16_out = EPI == EPI_BF16 || EPI == EPI_GELU_BF16;
  // default for bf16 outputs: the persistent ping-pong (18) on wide GEMMs (N >= 2048:
  // qkv, c_fc; +1.7-3 % in scripts/gemm_micro.py) and on K <= 1024 (out_proj),
  // the one-tile-per-workgroup ping-pong (16) on N = 768 with long K (c_proj:
  // the persistent kernel's static tile split loses 3.8 % there against the
  // dispatcher's dynamic one)
  if (a.patch_R) {  // fused patch gather: f32 output rows, ping-pong only
    if (!big || a.K != 3 * 32 * 32 || (a.patch_R & 31)) return hipErrorInvalidValue;
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false, false, false, true>), dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  // (N = 768: persistent on K = 768 since the stage streaming, +5 % on out500;
  // c_proj, K = 3072, stays one tile per workgroup: -3.8 % persistent)
  int v = a.variant == 0 ? (bf16_out ? ((a.N >= 2048 || a.K <= 1024) && !a.group ? 18 : 16) : 3) : a.variant;
  // default for bf16 outputs since the 8-phase kernel (gemm_8p.hip): +12-18 % over 16/18 on all four
  // B/32 tower shapes at M = 500k, bit-identical (scripts/gemm_micro.py); 16/18 stay for K % 128 != 0 / grouped rows
  if (a.variant == 0 && bf16_out && gemm_8p_ok(a)) v = 98;   // (+ early phase-1 DMAs: 0-3 % over 80)
  // default since gemm_8q.hip (descriptor DMAs, template-form waits, descriptor-store epilogue):
  // fc500 -4..-7 %, qkv500 -3..-4 %, proj500 -6 %, out500 +-3 % against v98, bit-identical
  if (a.variant == 0 && bf16_out && gemm_8q_ok(a)) v = 110;
  if (v == 16 && !bf16_out) v = 3;
  if (big && v == 16 && a.K / BK >= LEAD) {
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false, true>), dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (v >= 131 && v <= 139 && bf16_out && gemm_8q_ok(a)) {   // 8-phase, n-tiles in groups of (v - 130); 131: raster
    GemmArgs ga = a;
    ga.ngroup = v == 131 ? -1 : v - 130;
    return gemm_8q(ga, EPI, s, cu_count(), 0);
  }
  if (v == 125 && bf16_out && gemm_8q_ok(a)) return gemm_8q(a, EPI, s, cu_count(), 10);   // whole-row epilogue stores
  if (v >= 120 && v <= 124 && bf16_out) {   // 256 x 128 tiles, deferred epilogue (v98 where it does not apply)
    if (gemm_8r_ok(a)) return gemm_8r(a, EPI, s, cu_count(), v - 120);
    v = 98;
  }
  if (v >= 110 && v <= 119 && bf16_out) {   // 8-phase, second schedule (gemm_8p's v98 where it does not apply)
    if (gemm_8q_ok(a)) return gemm_8q(a, EPI, s, cu_count(), v - 110);
    v = 98;
  }
  if (v == 70 && bf16_out && gemm_w4_ok(a)) return gemm_w4(a, EPI, s, cu_count());   // one wave per SIMD, BK 64
  if (((v >= 91 && v <= 96 && v != 95) || v == 87 || v == 88) && bf16_out && gemm_8p_ok(a)) return gemm_8p(a, EPI, s, cu_count(), v < 90 ? v - 80 : v - 90);   // 8-phase probes
  if (v == 97 && bf16_out && gemm_8p_ok(a)) return gemm_8p(a, EPI, s, cu_count(), 100);   // 8-phase, aligned epilogue
  if (v == 98 && bf16_out && gemm_8p_ok(a)) return gemm_8p(a, EPI, s, cu_count(), 101);   // 8-phase, early phase-1 DMAs
  if (v == 99 && bf16_out && gemm_8p_ok(a)) return gemm_8p(a, EPI, s, cu_count(), 102);   // both
  if (v >= 80 && v < 90 && bf16_out && gemm_8p_ok(a)) {   // 8-phase interleave; n-groups of (v - 80)
    GemmArgs ga = a;
    ga.ngroup = v - 80;
    return gemm_8p(ga, EPI, s, cu_count());
  }
  if (big && v >= 60 && v < 70 && bf16_out && a.K / BK >= LEAD && !a.group) {
    // persistent kernel, non-temporal output stores, n-blocks in groups of (v - 60)
    GemmArgs ga = a;
    ga.ngroup = v - 60;
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_ppp_kernel<EPI, false, false, true>), dim3(grid), dim3(512), 0, s, ga);
    return hipGetLastError();
  }
  if (big && v >= 40 && v < 60 && bf16_out && a.K / BK >= LEAD && !a.group) {
    // tile-order probe: the persistent kernel with n-blocks walked in groups of (v - 40)
    GemmArgs ga = a;
    ga.ngroup = v - 40;
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_ppp_kernel<EPI>), dim3(grid), dim3(512), 0, s, ga);
    return hipGetLastError();
  }
  if (big && v == 18 && bf16_out && a.K / BK >= LEAD && !a.group) {  // persistent ping-pong
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_ppp_kernel<EPI>), dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (big && v == 20 && bf16_out && a.K / BK >= LEAD && !a.group) {  // persistent, early group-0 epilogue
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_ppp_kernel<EPI, false, true>), dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (big && v == 19 && bf16_out && a.K / BK >= LEAD && !a.group) {  // persistent + timing probe
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_ppp_kernel<EPI, true>), dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (big && v == 17 && bf16_out && a.K / BK >= LEAD) {  // experiment: non-temporal output stores
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false, true, true>), dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (big && v >= 31 && v <= 33 && a.K / BK >= LEAD) {  // main-loop ablation probes
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    if (v == 31) hipLaunchKernelGGL(gemm_abl_kernel<1>, dim3(nt), dim3(512), 0, s, a);
    else if (v == 32) hipLaunchKernelGGL(gemm_abl_kernel<2>, dim3(nt), dim3(512), 0, s, a);
    else hipLaunchKernelGGL(gemm_abl_kernel<3>, dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (big && (v == 34 || v == 35) && a.K / BK >= LEAD && (a.K / BK) % 2 == 0) {  // full-line fetch probes
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    if (v == 34) hipLaunchKernelGGL(gemm_abl_kernel<4>, dim3(nt), dim3(512), 0, s, a);
    else hipLaunchKernelGGL(gemm_abl_kernel<5>, dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (big && v == 8 && a.K / BK >= LEAD) {
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    hipLaunchKernelGGL((gemm_pp_kernel<EPI_NONE, 1, false>), dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (v == 16) v = 3;
  GemmArgs ga = a;
  if (v == 6) {  // ping-pong with the grouped (L2-resident W panel) tile order
    v = 3;
    ga.ngroup = n_group(a.N / 256, a.K);
  }
  if (big && v >= 2 && v <= 5 && a.K / BK >= LEAD) {
    const GemmArgs& a = ga;
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    if (v == 2) hipLaunchKernelGGL((gemm_pp_kernel<EPI, 2, false>), dim3(nt), dim3(512), 0, s, a);
    else if (v == 3) hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false>), dim3(nt), dim3(512), 0, s, a);
    else if (v == 4) hipLaunchKernelGGL((gemm_pp_kernel<EPI, 2, true>), dim3(nt), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, true>), dim3(nt), dim3(512), 0, s, a);
  } else if (big) {
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    const int g = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_kernel<EPI, 256, 256, 2, 4>), dim3(g), dim3(512), 0, s, a);
  } else {
    const int nt = ((a.M + 127) / 128) * (a.N / 128);
    const int g = nt < 2 * cu_count() ? nt : 2 * cu_count();
    hipLaunchKernelGGL((gemm_kernel<EPI, 128, 128, 2, 2>), dim3(g), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

#endif  // MICLIP_AB

// Product dispatch: the 8-phase kernel (gemm_8q.hip) for bf16 outputs whenever
// it applies (every tower GEMM of B/32, L/14, L/14@336 and the text towers
// with >= 256 rows); otherwise the ping-pong kernels — persistent (18) on wide
// N or K <= 1024, one tile per workgroup (16) on N = 768 with long K, LDS-staged
// rows (3) for f32 outputs (patch embedding, projections) — and the generic
// tiled kernel for shapes too small for them.
template <int EPI>
hipError_t launch(const GemmArgs& a, hipStream_t s) {
  const bool big = a.N % 256 == 0 && a.M >= 1024;
  const bool bf16_out = EPI == EPI_BF16 || EPI == EPI_GELU_BF16;
  if (a.patch_R) {  // fused patch gather: f32 output rows, ping-pong only
    if (!big || a.K != 3 * 32 * 32 || (a.patch_R & 31)) return hipErrorInvalidValue;
    const int nt = ((a.M + 255) / 256) * (a.N / 256);
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false, false, false, true>), dim3(nt), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (a.a_f16) {   // split-f16 operands (fp32 tower): f32 epilogues with the rsc / csc factors
    if ((EPI != EPI_F32 && EPI != EPI_RESID_F32 && EPI != EPI_SPLIT_GELU) || !a.rsc || !a.csc || a.variant)
      return hipErrorInvalidValue;
    if (EPI == EPI_SPLIT_GELU && (!a.rmax || !a.rsc_out || a.group || a.ldo != (a.o_dup ? 2 : 3) * (int64_t)a.N))
      return hipErrorInvalidValue;
    if constexpr (EPI == EPI_F32 || EPI == EPI_RESID_F32 || EPI == EPI_SPLIT_GELU) {
      // the 8-phase kernel (gemm_8q.hip) wherever it applies; MICLIP_F32_8Q=0 (A/B build) keeps the
      // ping-pong kernel below
#if MICLIP_AB
      // (MICLIP_F32_8Q=1 + MICLIP_F32_8Q_MASK: 1 EPI_F32, 2 EPI_RESID_F32, 4 EPI_SPLIT_GELU on the 8-phase kernel)
      const char* e8 = std::getenv("MICLIP_F32_8Q");
      const char* em = std::getenv("MICLIP_F32_8Q_MASK");
      const int bit = EPI == EPI_F32 ? 1 : (EPI == EPI_RESID_F32 ? 2 : 4);
      const bool use8q = (!e8 || std::atoi(e8) != 0) && (!em || (std::atoi(em) & bit));
#else
      const bool use8q = true;
#endif
      // (the 8-phase kernel's f32 epilogues assume a bias: bias-less calls take the ping-pong kernel)
      if (use8q && a.bias && gemm_8q_ok(a)) return gemm_8q(a, EPI, s, cu_count(), 0);
      if (a.a_dup || a.o_dup) return hipErrorInvalidValue;   // the [x1 | x2] layouts: the 8-phase kernel only
      const int ntf = ((a.M + 255) / 256) * (a.N / 256);
      if (big && a.K / BK >= LEAD) {
        hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false, false, false, false, true>), dim3(ntf), dim3(512), 0, s, a);
      } else if (big) {
        const int g = ntf < cu_count() ? ntf : cu_count();
        hipLaunchKernelGGL((gemm_kernel<EPI, 256, 256, 2, 4, true>), dim3(g), dim3(512), 0, s, a);
      } else {
        const int nt2 = ((a.M + 127) / 128) * (a.N / 128);
        const int g = nt2 < 2 * cu_count() ? nt2 : 2 * cu_count();
        hipLaunchKernelGGL((gemm_kernel<EPI, 128, 128, 2, 2, true>), dim3(g), dim3(256), 0, s, a);
      }
    }
    return hipGetLastError();
  }
#if MICLIP_AB
  if (a.variant != 0) return launch_ab<EPI>(a, s);
#else
  if (a.variant != 0) return hipErrorNotSupported;   // schedule overrides exist in the A/B build only
#endif
  // Small grids (fewer than 64 tiles of 256 x 256: the text tower's in_proj / out_proj / c_proj at
  // 32 queries, small image batches) take 128 x 128 tiles: 4x the workgroups on a chip of 256
  // CUs, the same k order and epilogue arithmetic (bit-identical for EPI_BF16).  B/32 encode_text
  // of 32 queries 1272 -> 1134 us (scripts/text_micro.py, profiles/r05_zl_text_micro.log).
  // MICLIP_SMALLM=t (A/B build) moves the threshold (0: off).
  int small_t = 64;
#if MICLIP_AB
  if (const char* sm = std::getenv("MICLIP_SMALLM")) small_t = std::atoi(sm);
#endif
  // Fewer 128 x 128 tiles than CUs (the text tower's in_proj / out_proj / c_proj at 32 queries):
  // 64 x 64 tiles, bit-identical again (round 6: encode_text of 32 queries 1131 -> 1006 us,
  // scripts/text_micro.py, profiles/r06_v_text_micro.log).  A/B MICLIP_SMALL64=u moves the
  // threshold to u tiles of 128 x 128 (0: off).
  int small64 = cu_count();
#if MICLIP_AB
  if (const char* sm = std::getenv("MICLIP_SMALL64")) small64 = std::atoi(sm);
#endif
  if (EPI == EPI_BF16 && ((a.M + 255) / 256) * (a.N / 256) < small_t && a.N % 128 == 0 && !a.group) {
    const int nt2 = ((a.M + 127) / 128) * (a.N / 128);
    if (nt2 < small64) {
      const int nt3 = ((a.M + 63) / 64) * (a.N / 64);
      const int g = nt3 < 4 * cu_count() ? nt3 : 4 * cu_count();
      hipLaunchKernelGGL((gemm_kernel<EPI, 64, 64, 2, 2>), dim3(g), dim3(256), 0, s, a);
      return hipGetLastError();
    }
    const int g = nt2 < 2 * cu_count() ? nt2 : 2 * cu_count();
    hipLaunchKernelGGL((gemm_kernel<EPI, 128, 128, 2, 2>), dim3(g), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (bf16_out && gemm_8q_ok(a)) return gemm_8q(a, EPI, s, cu_count(), 0);
  const int nt = ((a.M + 255) / 256) * (a.N / 256);
  const bool staged = big && a.K / BK >= LEAD;
  if (staged && bf16_out && !a.group && (a.N >= 2048 || a.K <= 1024)) {   // persistent ping-pong (18)
    const int grid = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_ppp_kernel<EPI>), dim3(grid), dim3(512), 0, s, a);
  } else if (staged && bf16_out) {                                         // ping-pong, direct row stores (16)
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false, true>), dim3(nt), dim3(512), 0, s, a);
  } else if (staged) {                                                     // ping-pong, LDS-staged f32 rows (3)
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, 1, false>), dim3(nt), dim3(512), 0, s, a);
  } else if (big) {
    const int g = nt < cu_count() ? nt : cu_count();
    hipLaunchKernelGGL((gemm_kernel<EPI, 256, 256, 2, 4>), dim3(g), dim3(512), 0, s, a);
  } else {
    const int nt2 = ((a.M + 127) / 128) * (a.N / 128);
    const int g = nt2 < 2 * cu_count() ? nt2 : 2 * cu_count();
    hipLaunchKernelGGL((gemm_kernel<EPI, 128, 128, 2, 2>), dim3(g), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t gemm_probe_read(unsigned long long* host, int n) {
#if MICLIP_AB
  if (n > 4096 * 4) n = 4096 * 4;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_probe), n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost);
#else
  (void)host;
  (void)n;
  return hipErrorNotSupported;   // the timing probe (variant 19) is in the A/B build only
#endif
}

hipError_t gemm_bf16(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  if (a.K % BK || a.N % 128 || a.K <= 0 || a.N > MAX_N) return hipErrorInvalidValue;
  if ((a.ldo % 8) || ((uintptr_t)a.out & 15)) return hipErrorInvalidValue;
  switch (epi) {
    case EPI_BF16: return launch<EPI_BF16>(a, s);
    case EPI_GELU_BF16: return launch<EPI_GELU_BF16>(a, s);
    case EPI_RESID_F32: return launch<EPI_RESID_F32>(a, s);
    case EPI_F32: return launch<EPI_F32>(a, s);
    case EPI_SPLIT_GELU: return launch<EPI_SPLIT_GELU>(a, s);
    case EPI_LN_BF16:
    case EPI_LN_GELU_BF16:   // LayerNorm-folded vision tower: the 8-phase kernel only
    case EPI_RES16_BF16:
      if (!gemm_8q_ok(a) || a.variant != 0) return hipErrorInvalidValue;
      return gemm_8q(a, epi, s, cu_count(), 0);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace miclip
