// Shared device helpers for libmiclip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// MICLIP_AB = 1 builds the A/B library (scripts/ab/libmiclip_ab.so, `make ab`):
// every measured alternative schedule, ablation and timing probe of the
// kernels plus their MICLIP_* environment switches.  The product library
// (libmiclip.so, MICLIP_AB = 0) holds the measured defaults only.
#ifndef MICLIP_AB
#define MICLIP_AB 0
#endif
// MICLIP_VMCHECK = 1: the counting build of the kernels with counted waits (vm_count_check below;
// `make` compiles it for the device only, next to the product objects, and fails on a mismatch)
#ifndef MICLIP_VMCHECK
#define MICLIP_VMCHECK 0
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16;

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

// f32 -> bf16 round-to-nearest-even (NaN stays NaN: quiet bit forced).
__device__ __host__ __forceinline__ u16 f2bf(float f) {
  union { float f; uint32_t u; } v;
  v.f = f;
  uint32_t u = v.u;
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (u16)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (u16)(u >> 16);
}

// Hardware RNE conversion (v_cvt_pk_bf16_f32; keeps NaN a NaN).
__device__ __forceinline__ u16 f2bf_hw(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 for the pair (two scalar conversions + shift/or otherwise)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2_t));
}
__device__ __forceinline__ uint32_t pack_bf16x2(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

__device__ __host__ __forceinline__ float bf2f(u16 h) {
  union { uint32_t u; float f; } v;
  v.u = ((uint32_t)h) << 16;
  return v.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// async 16-byte global -> LDS copy: LDS destination is lds_base + lane*16
// (wave-uniform base), the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Counted waits.  vmcnt retires a wave's VMEM ops in issue order and its field holds 0..63, so the
// wait for one DMA names how many VMEM ops the wave issued AFTER it.  Kernels that count waits derive
// each immediate from constexpr op counts (VM_MAX bounds them) and wait through vm_wait<N>.
constexpr int VM_MAX = 63;
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N <= VM_MAX, "vmcnt immediate outside the 6-bit field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// A ring of stages of OPS ops each: wait until at most `younger` (0..Y, runtime) stages younger than
// the awaited one -- plus EXTRA younger ops of another kind (an epilogue's stores) -- are in flight:
// vmcnt(younger * OPS + EXTRA) through a chain of compile-time immediates
template <int OPS, int Y, int EXTRA = 0>
__device__ __forceinline__ void vm_wait_stages(int younger) {
  if constexpr (Y == 0) {
    vm_wait<EXTRA>();
  } else {
    if (younger >= Y) vm_wait<Y * OPS + EXTRA>();
    else vm_wait_stages<OPS, Y - 1, EXTRA>(younger);
  }
}
// Compile-time check of an issued-op count: `n` is a local counter bumped at every VMEM op a code
// section issues, which the optimiser folds to a constant (fully unrolled, template-selected code).
// When it differs from the constexpr N that a counted wait was derived from, the call to this
// never-defined function survives and the device link fails -- the count and the code cannot drift
// apart silently.
extern "C" __device__ void miclip_vmcnt_count_mismatch();
template <int N>
__device__ __forceinline__ void vm_count_check(int n) {
  if (n != N) miclip_vmcnt_count_mismatch();
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks that share an XCD (b % 8) get a contiguous run of
// logical tile ids, so neighbouring tiles (which share operand panels) hit the
// same L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
