// The ring-attention output / LSE merge as a standalone op.
//
// Replaces (reference, /root/reference): picotron/context_parallel/context_parallel.py:157-187
// update_out_and_lse -- the pure function RingAttentionFunc calls after every block:
//   out <- out - sigmoid(block_lse - lse) * (out - block_out)
//   lse <- lse - logsigmoid(lse - block_lse)
// with `out` fp32 and `lse` kept in the dtype of the block LSE (bf16 for a bf16 ring: SURVEY §8c
// caveat 1).  The ring itself (context_parallel.ring_forward) merges inside the attention kernel's
// epilogue; this entry point serves the reference's pure-function API with the reference's
// roundings: in bf16 mode every lse-side intermediate is rounded to bf16 as torch's bf16 ops do.
//
// Two stream-ordered elementwise passes (out first, from the OLD lse; then lse), each coalesced over
// the contiguous [rows, D] / [rows] buffers.  HBM-bound: 4 + 2|4 + 4 bytes per out element.
#include "common.h"

// torch evaluates these expressions op by op (sub, then mul, then sub); keep the compiler from
// contracting them into fmas so the f32 path rounds as the reference does
#pragma clang fp contract(off)

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float ld_lse(const void* p, int64_t i, int bf) {
  return bf ? bf2f(((const uint16_t*)p)[i]) : ((const float*)p)[i];
}

// torch's CPU / CUDA log_sigmoid: min(x, 0) - log1p(exp(-|x|))
__device__ __forceinline__ float log_sigmoid(float x) { return fminf(x, 0.f) - log1pf(expf(-fabsf(x))); }
__device__ __forceinline__ float sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(kThreads) void merge_out_kernel(const float* __restrict__ out, const void* __restrict__ bo,
                                                             int bo_bf, const void* __restrict__ lse,
                                                             const void* __restrict__ blse, int lse_bf,
                                                             float* __restrict__ out_new, int64_t rows, int64_t D) {
  const int64_t n = rows * D;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const int64_t r = i / D;
    const float L = ld_lse(lse, r, lse_bf), B = ld_lse(blse, r, lse_bf);
    float d = B - L;
    if (lse_bf) d = round_bf(d);
    float w = sigmoid(d);
    if (lse_bf) w = round_bf(w);   // F.sigmoid of a bf16 tensor is a bf16 tensor
    const float b = bo_bf ? bf2f(((const uint16_t*)bo)[i]) : ((const float*)bo)[i];
    const float o = out[i];
    out_new[i] = o - w * (o - b);
  }
}

__global__ __launch_bounds__(kThreads) void merge_lse_kernel(const void* __restrict__ lse, const void* __restrict__ blse,
                                                             int lse_bf, void* __restrict__ lse_new, int64_t rows) {
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < rows; r += (int64_t)gridDim.x * kThreads) {
    const float L = ld_lse(lse, r, lse_bf), B = ld_lse(blse, r, lse_bf);
    if (lse_bf) {
      const float ls = round_bf(log_sigmoid(round_bf(L - B)));
      ((uint16_t*)lse_new)[r] = f2bf(L - ls);
    } else {
      ((float*)lse_new)[r] = L - log_sigmoid(L - B);
    }
  }
}

inline unsigned grid_for(int64_t n) {
  const int64_t g = (n + kThreads - 1) / kThreads;
  return (unsigned)(g < PT_STREAM_GRID_CAP ? (g > 0 ? g : 1) : PT_STREAM_GRID_CAP);
}

}  // namespace

extern "C" int pt_lse_merge(const float* out, const void* block_out, int block_out_dtype, const void* lse,
                            const void* block_lse, int lse_dtype, float* out_new, void* lse_new, int64_t rows,
                            int64_t D, hipStream_t stream) {
  if (!out || !block_out || !lse || !block_lse || !out_new || !lse_new || rows <= 0 || D <= 0) return PT_EINVAL;
  if ((block_out_dtype != 0 && block_out_dtype != 1) || (lse_dtype != 0 && lse_dtype != 1)) return PT_EINVAL;
  merge_out_kernel<<<grid_for(rows * D), kThreads, 0, stream>>>(out, block_out, block_out_dtype == 0, lse, block_lse,
                                                                lse_dtype == 0, out_new, rows, D);
  PT_CHECK_LAUNCH();
  merge_lse_kernel<<<grid_for(rows), kThreads, 0, stream>>>(lse, block_lse, lse_dtype == 0, lse_new, rows);
  PT_CHECK_LAUNCH();
  return PT_OK;
}
