// SwiGLU activation forward / backward:  h = silu(g) * u   (the MLP core).
//
// Replaces (reference, /root/reference): picotron/model.py:186  `F.silu(self.gate_proj(x)) * self.up_proj(x)`
// in bf16.  torch rounds silu(g) to bf16 and then the product, so we do too:
//   fwd:  h  = bf16( bf16(silu(g)) * u )
//   bwd:  du = bf16( dh * bf16(silu(g)) )
//         dg = bf16( bf16(dh * u) * sig(g) * (1 + g * (1 - sig(g))) )
//
// g, u, h, dh, dg, du are [rows, cols] views with independent row strides (elements), so the
// gate/up halves of a fused [rows, 2*cols] projection output are consumed in place.  One thread
// per 8 columns.  HBM-bound: fwd 6 bytes/element, bwd 10 bytes/element.
#include "common.h"

namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return pt_sigmoid(x); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const uint16_t* __restrict__ g, int64_t gs,
                                                         const uint16_t* __restrict__ u, int64_t us,
                                                         uint16_t* __restrict__ h, int64_t hs, int64_t rows,
                                                         int cols) {
  const int cpr = cols >> 3;
  const int64_t total = rows * cpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr) * 8;
    float a[8], b[8], o[8];
    unpack8(ld8(g + r * gs + c), a);
    unpack8(ld8(u + r * us + c), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = round_bf(a[j] * sigmoidf_(a[j])) * b[j];
    st8(h + r * hs + c, pack8(o));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const uint16_t* __restrict__ dh, int64_t dhs,
                                                         const uint16_t* __restrict__ g, int64_t gs,
                                                         const uint16_t* __restrict__ u, int64_t us,
                                                         uint16_t* __restrict__ dg, int64_t dgs,
                                                         uint16_t* __restrict__ du, int64_t dus, int64_t rows,
                                                         int cols) {
  const int cpr = cols >> 3;
  const int64_t total = rows * cpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr) * 8;
    float d[8], a[8], b[8], og[8], ou[8];
    unpack8(ld8(dh + r * dhs + c), d);
    unpack8(ld8(g + r * gs + c), a);
    unpack8(ld8(u + r * us + c), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoidf_(a[j]);
      ou[j] = d[j] * round_bf(a[j] * s);
      og[j] = round_bf(d[j] * b[j]) * (s * (1.0f + a[j] * (1.0f - s)));
    }
    st8(dg + r * dgs + c, pack8(og));
    st8(du + r * dus + c, pack8(ou));
  }
}

// out = bf16(x + r) over n contiguous elements (n % 8 == 0): the residual add of model.py:208
// (`x = x + self.mlp(...)`, torch's bf16 add: the fp32 sum rounded once) where it cannot ride in a
// GEMM epilogue -- the sequence-parallel TP layer adds the residual to the reduce-scattered MLP
// output.  HBM-bound, 6 bytes per element.
__global__ __launch_bounds__(256) void residual_add_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ r,
                                                           uint16_t* __restrict__ out, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float a[8], b[8], o[8];
    unpack8(ld8(x + i * 8), a);
    unpack8(ld8(r + i * 8), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = a[j] + b[j];
    st8(out + i * 8, pack8(o));
  }
}

int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g < PT_STREAM_GRID_CAP * 2 ? g : PT_STREAM_GRID_CAP * 2);
}

}  // namespace

extern "C" {

int pt_swiglu_fwd(const void* g, int64_t g_stride, const void* u, int64_t u_stride, void* h, int64_t h_stride,
                  int64_t rows, int64_t cols, hipStream_t stream) {
  if (!g || !u || !h || rows <= 0 || cols <= 0) return PT_EINVAL;
  if ((cols & 7) || (g_stride & 7) || (u_stride & 7) || (h_stride & 7)) return PT_EALIGN;
  if (!pt_aligned16(g) || !pt_aligned16(u) || !pt_aligned16(h)) return PT_EALIGN;
  swiglu_fwd_kernel<<<grid_for(rows * (cols / 8)), 256, 0, stream>>>(
      (const uint16_t*)g, g_stride, (const uint16_t*)u, u_stride, (uint16_t*)h, h_stride, rows, (int)cols);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

int pt_swiglu_bwd(const void* dh, int64_t dh_stride, const void* g, int64_t g_stride, const void* u,
                  int64_t u_stride, void* dg, int64_t dg_stride, void* du, int64_t du_stride, int64_t rows,
                  int64_t cols, hipStream_t stream) {
  if (!dh || !g || !u || !dg || !du || rows <= 0 || cols <= 0) return PT_EINVAL;
  if ((cols & 7) || (dh_stride & 7) || (g_stride & 7) || (u_stride & 7) || (dg_stride & 7) || (du_stride & 7))
    return PT_EALIGN;
  if (!pt_aligned16(dh) || !pt_aligned16(g) || !pt_aligned16(u) || !pt_aligned16(dg) || !pt_aligned16(du))
    return PT_EALIGN;
  swiglu_bwd_kernel<<<grid_for(rows * (cols / 8)), 256, 0, stream>>>(
      (const uint16_t*)dh, dh_stride, (const uint16_t*)g, g_stride, (const uint16_t*)u, u_stride, (uint16_t*)dg,
      dg_stride, (uint16_t*)du, du_stride, rows, (int)cols);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

int pt_residual_add(const void* x, const void* r, void* out, int64_t n, hipStream_t stream) {
  if (!x || !r || !out || n <= 0) return PT_EINVAL;
  if ((n & 7) || !pt_aligned16(x) || !pt_aligned16(r) || !pt_aligned16(out)) return PT_EALIGN;
  residual_add_kernel<<<grid_for(n / 8), 256, 0, stream>>>((const uint16_t*)x, (const uint16_t*)r, (uint16_t*)out,
                                                           n / 8);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

}  // extern "C"
