// RMSNorm forward / backward for gfx950, with an optional fused residual add.
//
// Replaces (reference, /root/reference):
//   * picotron/model.py:51-65  TritonRMSNorm.forward -> flash-attn layer_norm_fn(is_rms_norm=True)
//     mode 0:  y = bf16(x * rstd * w)                (all f32 math, one rounding)
//   * picotron/model.py:81-86  LlamaRMSNorm.forward (FLASH_ATTEN=0 / CPU path)
//     mode 1:  y = bf16(w * bf16(x * rstd))          (extra rounding before the weight)
//   * picotron/model.py:207-208 the residual `x + f(x)` in bf16, fused in front of the
//     following norm:   z = bf16(x + r), y = norm(z); z is written out as the new residual stream.
//
// Layout: rows x cols, row-major bf16, cols % 8 == 0.  One wavefront owns one row
// (grid-strided); each lane holds NCH 16-byte chunks of the row in registers, so x
// is read from HBM exactly once.  HBM-bound: fwd moves 4*rows*cols bytes (6 with the
// residual), bwd 6*rows*cols (+2 with the fused residual gradient).
#include "common.h"

namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kThreads = kWavesPerBlock * PT_WAVE;

template <int NCH>
__global__ __launch_bounds__(kThreads) void rmsnorm_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ y, uint16_t* __restrict__ z_out, float* __restrict__ rstd_out,
    int64_t rows, int cols, float eps, int mode) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
  const int nchunk = cols >> 3;
  const float inv_cols = 1.0f / (float)cols;

  // weight chunks are row-invariant: keep them in registers across rows
  float wf[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * PT_WAVE;
    if (c < nchunk) unpack8(ld8(w + c * 8), wf[i]);
  }

  for (int64_t row = wave; row < rows; row += nwaves) {
    const uint16_t* xr = x + row * cols;
    float v[NCH][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        unpack8(ld8(xr + c * 8), v[i]);
        if (res) {
          float r[8];
          unpack8(ld8(res + row * cols + c * 8), r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] = round_bf(v[i][j] + r[j]);  // bf16 residual stream
          st8(z_out + row * cols + c * 8, pack8(v[i]));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
      }
    }
    ss = wave_sum(ss);
    const float rstd = rsqrtf(ss * inv_cols + eps);
    if (lane == 0) rstd_out[row] = rstd;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float o[8];
        if (mode == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wf[i][j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = wf[i][j] * round_bf(v[i][j] * rstd);
        }
        st8(y + row * cols + c * 8, pack8(o));
      }
    }
  }
}

// dz = rstd * (dxh - xh * mean(dxh * xh)),  dxh = dy * w,  xh = z * rstd
// dx = dz (+ dres when the residual branch gradient is fused in)
// dw partial per block: sum over this block's rows of dy * xh (mode 1: dy * bf16(xh))
template <int NCH>
__global__ __launch_bounds__(kThreads) void rmsnorm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ z, const uint16_t* __restrict__ w,
    const float* __restrict__ rstd_in, const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
    float* __restrict__ dw_partial, int64_t rows, int cols, int mode) {
  __shared__ float red[kWavesPerBlock][NCH * PT_WAVE * 8 > 4096 ? 1 : NCH * PT_WAVE * 8];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
  const int nchunk = cols >> 3;
  const float inv_cols = 1.0f / (float)cols;

  float wf[NCH][8], dwacc[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * PT_WAVE;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = 0.f;
    if (c < nchunk) unpack8(ld8(w + c * 8), wf[i]);
  }

  for (int64_t row = wave; row < rows; row += nwaves) {
    const float rstd = rstd_in[row];
    float xh[NCH][8], g[NCH][8];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float zz[8], d[8];
        unpack8(ld8(z + row * cols + c * 8), zz);
        unpack8(ld8(dy + row * cols + c * 8), d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = zz[j] * rstd;
          g[i][j] = d[j] * wf[i][j];
          dot += g[i][j] * xh[i][j];
          dwacc[i][j] += d[j] * (mode == 0 ? xh[i][j] : round_bf(xh[i][j]));
        }
      }
    }
    dot = wave_sum(dot) * inv_cols;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[i][j] - xh[i][j] * dot);
        if (dres) {
          float r[8];
          unpack8(ld8(dres + row * cols + c * 8), r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        st8(dx + row * cols + c * 8, pack8(o));
      }
    }
  }

  // combine the block's waves, then one partial row per block
  if (NCH * PT_WAVE * 8 <= 4096) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wid][c * 8 + j] = dwacc[i][j];
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < cols; col += kThreads) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kWavesPerBlock; ++k) s += red[k][col];
      dw_partial[(int64_t)blockIdx.x * cols + col] = s;
    }
  } else {
    // wide rows: one partial row per wave instead
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float* dst = dw_partial + ((int64_t)blockIdx.x * kWavesPerBlock + wid) * cols + c * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[j] = dwacc[i][j];
      }
    }
  }
}

// dw[col] = bf16(sum_p partial[p][col])  -- fixed summation order, deterministic.
// A block owns 32 columns; its 8 row groups (one per 32 threads) stride over the partial rows
// with coalesced 128-B reads, then combine through LDS in a fixed order.
constexpr int kColsumCols = 32, kColsumGroups = 8;
__global__ __launch_bounds__(256) void colsum_to_bf16_kernel(const float* __restrict__ partial, int nparts,
                                                             int cols, uint16_t* __restrict__ out,
                                                             float* __restrict__ out_f32) {
  __shared__ float red[kColsumGroups][kColsumCols];
  const int c = threadIdx.x % kColsumCols, g = threadIdx.x / kColsumCols;
  const int col = blockIdx.x * kColsumCols + c;
  float s = 0.f;
  if (col < cols)
    for (int p = g; p < nparts; p += kColsumGroups) s += partial[(int64_t)p * cols + col];
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < cols) {
#pragma unroll
    for (int k = 1; k < kColsumGroups; ++k) s += red[k][c];
    if (out) out[col] = f2bf(s);
    if (out_f32) out_f32[col] = s;
  }
}

int nch_for(int cols) {
  const int chunks = cols / 8;
  if (chunks <= 64) return 1;
  if (chunks <= 128) return 2;
  if (chunks <= 256) return 4;
  if (chunks <= 512) return 8;
  return -1;
}

int fwd_grid(int64_t rows) {
  int64_t g = (rows + kWavesPerBlock - 1) / kWavesPerBlock;
  return (int)(g < PT_STREAM_GRID_CAP ? g : PT_STREAM_GRID_CAP);
}

}  // namespace

extern "C" {

int pt_rmsnorm_bwd_partials(int64_t rows, int cols) {
  const int nch = nch_for(cols);
  if (nch < 0) return PT_EUNSUPPORTED;
  // bwd grid is fixed at 256 blocks (one per CU); wide rows keep one partial per wave
  const int grid = (int)(rows < 256 * kWavesPerBlock ? (rows + kWavesPerBlock - 1) / kWavesPerBlock : 256);
  return (nch * PT_WAVE * 8 <= 4096) ? grid : grid * kWavesPerBlock;
}

int pt_rmsnorm_fwd(const void* x, const void* residual, const void* weight, void* y, void* z_out,
                   float* rstd, int64_t rows, int64_t cols, float eps, int mode, hipStream_t stream) {
  if (!x || !weight || !y || !rstd || rows <= 0 || cols <= 0 || (cols & 7)) return PT_EINVAL;
  if (residual && !z_out) return PT_EINVAL;
  if (!pt_aligned16(x) || !pt_aligned16(weight) || !pt_aligned16(y)) return PT_EALIGN;
  if (residual && (!pt_aligned16(residual) || !pt_aligned16(z_out))) return PT_EALIGN;
  const int nch = nch_for((int)cols);
  const auto* X = (const uint16_t*)x;
  const auto* R = (const uint16_t*)residual;
  const auto* W = (const uint16_t*)weight;
  auto* Y = (uint16_t*)y;
  auto* Z = (uint16_t*)z_out;
  const dim3 grid(fwd_grid(rows)), block(kThreads);
  switch (nch) {
    case 1: rmsnorm_fwd_kernel<1><<<grid, block, 0, stream>>>(X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    case 2: rmsnorm_fwd_kernel<2><<<grid, block, 0, stream>>>(X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    case 4: rmsnorm_fwd_kernel<4><<<grid, block, 0, stream>>>(X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    case 8: rmsnorm_fwd_kernel<8><<<grid, block, 0, stream>>>(X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    default: return PT_EUNSUPPORTED;
  }
  PT_CHECK_LAUNCH();
  return PT_OK;
}

int pt_rmsnorm_bwd(const void* dy, const void* z, const void* weight, const float* rstd, const void* dres,
                   void* dx, void* dweight, float* dw_partial, int64_t rows, int64_t cols, int mode,
                   hipStream_t stream) {
  if (!dy || !z || !weight || !rstd || !dx || !dw_partial || rows <= 0 || cols <= 0 || (cols & 7))
    return PT_EINVAL;
  if (!pt_aligned16(dy) || !pt_aligned16(z) || !pt_aligned16(dx) || (dres && !pt_aligned16(dres)))
    return PT_EALIGN;
  const int nch = nch_for((int)cols);
  if (nch < 0) return PT_EUNSUPPORTED;
  const int grid = (int)(rows < 256 * kWavesPerBlock ? (rows + kWavesPerBlock - 1) / kWavesPerBlock : 256);
  const int nparts = pt_rmsnorm_bwd_partials(rows, (int)cols);
  const auto* DY = (const uint16_t*)dy;
  const auto* Z = (const uint16_t*)z;
  const auto* W = (const uint16_t*)weight;
  const auto* DR = (const uint16_t*)dres;
  auto* DX = (uint16_t*)dx;
  switch (nch) {
    case 1: rmsnorm_bwd_kernel<1><<<grid, kThreads, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, mode); break;
    case 2: rmsnorm_bwd_kernel<2><<<grid, kThreads, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, mode); break;
    case 4: rmsnorm_bwd_kernel<4><<<grid, kThreads, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, mode); break;
    case 8: rmsnorm_bwd_kernel<8><<<grid, kThreads, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, mode); break;
    default: return PT_EUNSUPPORTED;
  }
  PT_CHECK_LAUNCH();
  if (dweight) {
    colsum_to_bf16_kernel<<<(int)((cols + kColsumCols - 1) / kColsumCols), 256, 0, stream>>>(dw_partial, nparts, (int)cols,
                                                                        (uint16_t*)dweight, nullptr);
    PT_CHECK_LAUNCH();
  }
  return PT_OK;
}

}  // extern "C"
