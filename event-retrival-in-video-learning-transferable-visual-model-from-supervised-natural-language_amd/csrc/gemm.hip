// bf16 MFMA GEMM with fused CLIP epilogues (gfx950).
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ bias, QuickGELU, residual add)
//
// Replaces the nn.Linear / conv1 GEMMs that openai/CLIP's encode_image /
// encode_text run inside PyTorch:
// attn.in_proj (+bias), attn.out_proj (+bias +residual), mlp.c_fc (+bias
// +QuickGELU, transformers/activations.py:117-123), mlp.c_proj (+bias
// +residual), conv1 as an im2col GEMM, and the bias-free CLS projections.
//
// Tile: 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 =
// 4x4 x mfma_f32_16x16x32_bf16.  Operands are staged global->LDS with
// 16-byte LDS-DMA (global_load_lds_dwordx4) into two buffers; the LDS image
// is lane-linear, so the bank-conflict XOR swizzle (slot ^= row & 7 on the
// 16-byte chunk of a 128-byte row) is applied to the per-lane SOURCE address
// and again on the ds_read (cdna_hip_programming.md §5.4 rule 21).  Block ids
// are remapped XCD-aware so tiles sharing an A row-panel share an L2.
#include "common.hpp"
#include "internal.hpp"

namespace miclip {

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int STAGE_BYTES = (BM + BN) * BK * 2;  // 32 KiB: A tile then W tile

__device__ __forceinline__ float quick_gelu(float v) { return v / (1.0f + __expf(-1.702f * v)); }

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = a.N / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;

  // --- LDS-DMA source addresses: instruction j of wave w fills LDS bytes
  // [(w*4+j)*1024, +1024) = rows (w*4+j)*8 .. +7 of the tile; lane i -> row
  // +(i>>3), LDS slot (i&7) which holds global chunk (i&7) ^ (row&7).
  const uint16_t* asrc[4];
  const uint16_t* wsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (wave * 4 + j) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ (row & 7);
    const int ra = min(m0 + row, a.M - 1);
    asrc[j] = a.A + (int64_t)ra * a.lda + chunk * 8;
    wsrc[j] = a.W + (int64_t)(n0 + row) * a.ldw + chunk * 8;
  }
  auto stage = [&](int kt, int buf) {
    char* base = smem + buf * STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      glds16(asrc[j] + kt * BK, base + (wave * 4 + j) * 1024);
      glds16(wsrc[j] + kt * BK, base + BM * BK * 2 + (wave * 4 + j) * 1024);
    }
  };

  const int wr = wave >> 1, wc = wave & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
  stage(0, 0);
  vm_wait_all();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const char* As = smem + (kt & 1) * STAGE_BYTES;
    const char* Ws = As + BM * BK * 2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // fragment: row (lane&15) of a 16-row block, k chunk 4s + (lane>>4)
      const int slot = ((4 * s + (lane >> 4)) ^ (lane & 7)) * 16;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
        af[mi] = *(const bf16x8*)(As + (wr * 64 + mi * 16 + (lane & 15)) * 128 + slot);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        bfr[ni] = *(const bf16x8*)(Ws + (wc * 64 + ni * 16 + (lane & 15)) * 128 + slot);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    vm_wait_all();
    __syncthreads();
  }

  // --- epilogue: C/D map col = lane&15, row = 4*(lane>>4) + j
  float bias[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wc * 64 + ni * 16 + (lane & 15);
    bias[ni] = a.bias ? a.bias[n] : 0.f;
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wr * 64 + mi * 16 + 4 * (lane >> 4) + j;
      if (m >= a.M) continue;
      const int64_t orow = a.group ? (int64_t)(m / a.group) * a.gstride + a.goffset + m % a.group : m;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int n = n0 + wc * 64 + ni * 16 + (lane & 15);
        float v = acc[mi][ni][j] + bias[ni];
        if (EPI == EPI_BF16) {
          ((uint16_t*)a.out)[orow * a.ldo + n] = f2bf(v);
        } else if (EPI == EPI_GELU_BF16) {
          ((uint16_t*)a.out)[orow * a.ldo + n] = f2bf(quick_gelu(v));
        } else if (EPI == EPI_RESID_F32) {
          float* p = (float*)a.out + orow * a.ldo + n;
          *p = *p + v;
        } else {
          ((float*)a.out)[orow * a.ldo + n] = v;
        }
      }
    }
  }
}

}  // namespace

hipError_t gemm_bf16(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  if (a.K % BK || a.N % BN || a.K <= 0) return hipErrorInvalidValue;
  const int nwg = ((a.M + BM - 1) / BM) * (a.N / BN);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_kernel<EPI_BF16>, dim3(nwg), dim3(256), 0, s, a); break;
    case EPI_GELU_BF16: hipLaunchKernelGGL(gemm_kernel<EPI_GELU_BF16>, dim3(nwg), dim3(256), 0, s, a); break;
    case EPI_RESID_F32: hipLaunchKernelGGL(gemm_kernel<EPI_RESID_F32>, dim3(nwg), dim3(256), 0, s, a); break;
    case EPI_F32: hipLaunchKernelGGL(gemm_kernel<EPI_F32>, dim3(nwg), dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace miclip
