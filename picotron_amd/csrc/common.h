// Shared device helpers for the picotron_amd gfx950 (CDNA4 / MI355X) kernels.
//
// Everything in csrc/ is plain HIP written for gfx950 only: 64-lane wavefronts,
// MFMA bf16 tiles, LDS staging.  Host entry points are `extern "C"` and take
// plain device pointers, sizes and a hipStream_t (see include/picotron_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_WAVE 64

// The C ABI (and the PT_* error codes: 0 ok, negative = argument error found before launch,
// positive = hipError_t of the launch).  Included here so every definition is checked against it.
#include "../../include/picotron_hip.h"

// measurement variants (pt_set_variant, csrc/variants.hip): read by the launchers, never the kernels
enum PtVariant { PT_VAR_ATTN_PAIR = 0, PT_VAR_ATTN_SPLIT, PT_VAR_GEMM_MIX, PT_VAR_GEMM_KH,
                 PT_VAR_ATTN_KV_CHUNK, PT_VAR_COUNT };
int pt_variant(PtVariant v);

#define PT_CHECK_LAUNCH()                          \
  do {                                             \
    hipError_t _e = hipGetLastError();             \
    if (_e != hipSuccess) return (int)_e;          \
  } while (0)

// ---- bf16 <-> f32 -----------------------------------------------------------
// bf16 is carried as raw uint16 bits.  f32->bf16 is round-to-nearest-even via
// the native __bf16 cast (hipcc emits v_cvt_pk_bf16_f32, NaN-preserving).
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
// round an f32 through bf16 and back (models a bf16 storage round trip)
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }
// sigmoid(x) = 1 / (1 + e^-x) with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of the IEEE
// division sequence (v_div_scale / fmas / fixup, ~10 instructions): every SwiGLU kernel uses this
// one expression, so the fused epilogues and csrc/swiglu.hip stay bit-identical
__device__ __forceinline__ float pt_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// 8 x bf16 in one 16-byte vector
struct __attribute__((aligned(16))) bf16x8 { uint32_t w[4]; };

__device__ __forceinline__ void unpack8(const bf16x8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[2 * i] = lo_bf(v.w[i]); f[2 * i + 1] = hi_bf(v.w[i]); }
}
__device__ __forceinline__ bf16x8 pack8(const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v.w[i] = pack_bf2(f[2 * i], f[2 * i + 1]);
  return v;
}
__device__ __forceinline__ bf16x8 ld8(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void st8(uint16_t* p, const bf16x8& v) { *reinterpret_cast<bf16x8*>(p) = v; }
// non-temporal forms for data touched once (streaming optimizer state, split-K partials): the guide's
// nt stream measured 6.5-6.8 TB/s against 6.4 with the default cache policy
// (global address space explicitly: pointers read from a device-side table would otherwise be flat)
typedef uint32_t pt_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) pt_u32x4 pt_g_u32x4;
__device__ __forceinline__ bf16x8 ld8_nt(const uint16_t* p) {
  const pt_u32x4 r = __builtin_nontemporal_load((const pt_g_u32x4*)(p));
  return bf16x8{{r.x, r.y, r.z, r.w}};
}
__device__ __forceinline__ void st8_nt(uint16_t* p, const bf16x8& v) {
  const pt_u32x4 r = {v.w[0], v.w[1], v.w[2], v.w[3]};
  __builtin_nontemporal_store(r, (pt_g_u32x4*)(p));
}

// ---- wave reductions (64 lanes) ---------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- LDS-DMA from inline asm ----------------------------------------------------
// global -> LDS copies (saddr form: wave-uniform base + per-lane byte offset; M0 = the LDS
// destination of lane 0).  Issued from asm so the compiler does not treat them as pending LDS
// writes: it otherwise cannot prove ds_read_b64_tr_b16 reads disjoint from an in-flight LDS-DMA
// and puts an `s_waitcnt vmcnt(0)` in front of them, draining every prefetch.  The kernels order
// the copies themselves (counted `s_waitcnt vmcnt(N)` + barrier before the first read).  M0 is
// written here and read by nothing else in those kernels.
__device__ __forceinline__ uint64_t pt_uniform_u64(uint64_t p) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void pt_glds16(const void* base, uint32_t voff_bytes,
                                          __attribute__((address_space(3))) void* dst) {
  const uint64_t sb = pt_uniform_u64((uint64_t)(uintptr_t)base);
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(m0), "v"(voff_bytes), "s"(sb) : "memory");
}
__device__ __forceinline__ void pt_glds4(const void* base, uint32_t voff_bytes,
                                         __attribute__((address_space(3))) void* dst) {
  const uint64_t sb = pt_uniform_u64((uint64_t)(uintptr_t)base);
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, %2" ::"s"(m0), "v"(voff_bytes), "s"(sb) : "memory");
}

static inline bool pt_aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Grid cap for streaming (HBM-bound) kernels: 256 CUs x 8 blocks.
static constexpr int PT_STREAM_GRID_CAP = 2048;
