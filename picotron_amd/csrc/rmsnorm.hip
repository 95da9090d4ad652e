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
// One row per wave at a time, kBwdWaves(NCH) waves per block (rows grid-strided): every load of a
// row (z, dy, dres) is issued before the row's reduction, and many waves per SIMD keep HBM busy
// (the kernel is HBM-bound: 8 bytes per element with the fused residual gradient).
template <int NCH>
constexpr int bwd_waves() { return NCH <= 4 ? 8 : 4; }
constexpr int kBwdGridCap = 1024;

template <int NCH>
__global__ __launch_bounds__(bwd_waves<NCH>() * 64) void rmsnorm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ z, const uint16_t* __restrict__ w,
    const float* __restrict__ rstd_in, const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
    float* __restrict__ dw_partial, int64_t rows, int cols, int mode) {
  constexpr int WPB = bwd_waves<NCH>();
  __shared__ float red[WPB][NCH * PT_WAVE * 8];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nchunk = cols >> 3;
  const float inv_cols = 1.0f / (float)cols;

  bf16x8 wv[NCH];
  float dwacc[NCH][8];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * PT_WAVE;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = 0.f;
    if (c < nchunk) wv[i] = ld8(w + c * 8);
  }

  for (int64_t row = (int64_t)blockIdx.x * WPB + wid; row < rows; row += (int64_t)gridDim.x * WPB) {
    bf16x8 zr[NCH], dr[NCH], rr[NCH];
    const float rstd = rstd_in[row];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        zr[i] = ld8(z + row * cols + c * 8);
        dr[i] = ld8(dy + row * cols + c * 8);
        if (dres) rr[i] = ld8(dres + row * cols + c * 8);
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float zz[8], d[8], wf[8];
        unpack8(zr[i], zz);
        unpack8(dr[i], d);
        unpack8(wv[i], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = zz[j] * rstd;
          dot += d[j] * wf[j] * xh;
          dwacc[i][j] += d[j] * (mode == 0 ? xh : round_bf(xh));
        }
      }
    }
    dot = wave_sum(dot) * inv_cols;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float zz[8], d[8], wf[8], o[8];
        unpack8(zr[i], zz);
        unpack8(dr[i], d);
        unpack8(wv[i], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = zz[j] * rstd;
          o[j] = rstd * (d[j] * wf[j] - xh * dot);
        }
        if (dres) {
          float r[8];
          unpack8(rr[i], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        st8(dx + row * cols + c * 8, pack8(o));
      }
    }
  }

  // combine the block's waves (fixed order), one partial row per block
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * PT_WAVE;
    if (c < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][c * 8 + j] = dwacc[i][j];
    }
  }
  __syncthreads();
  for (int col = threadIdx.x; col < cols; col += WPB * 64) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WPB; ++k) s += red[k][col];
    dw_partial[(int64_t)blockIdx.x * cols + col] = s;
  }
}

template <int NCH>
int bwd_grid(int64_t rows) {
  const int64_t g = (rows + bwd_waves<NCH>() - 1) / bwd_waves<NCH>();
  return (int)(g < kBwdGridCap ? g : kBwdGridCap);
}

// dw[col] = sum_p partial[p][col]  -- fixed summation order, deterministic.  One block per 8
// columns (256 blocks for cols 2048: every CU): thread t sums partial rows t, t + 256, ... of its
// block's 8 columns (two 16-B loads per row), then a fixed-shape LDS tree over the 256 threads.
// Sink (flags): 0 store bf16, DW_ACC_BF16 bf16 accumulate (= autograd's grad + bf16(new)),
// DW_ACC_F32 f32 accumulate (DataParallelBucket main_grad).
constexpr int kColsumThreads = 256;
__global__ __launch_bounds__(kColsumThreads) void colsum_kernel(const float* __restrict__ partial, int nparts,
                                                                int cols, void* __restrict__ out, int sink) {
  __shared__ float red[kColsumThreads][9];  // +1 pad
  const int t = threadIdx.x;
  const int col0 = blockIdx.x * 8;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  for (int p = t; p < nparts; p += kColsumThreads) {
    const float4 a = *(const float4*)(partial + (int64_t)p * cols + col0);
    const float4 b = *(const float4*)(partial + (int64_t)p * cols + col0 + 4);
    s[0] += a.x; s[1] += a.y; s[2] += a.z; s[3] += a.w;
    s[4] += b.x; s[5] += b.y; s[6] += b.z; s[7] += b.w;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = s[j];
  __syncthreads();
  for (int w = kColsumThreads / 2; w >= 8; w >>= 1) {
    if (t < w) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[t][j] += red[t + w][j];
    }
    __syncthreads();
  }
  if (t < 8) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += red[k][t];
    const int col = col0 + t;
    if (sink == PT_DW_ACC_F32) {
      ((float*)out)[col] += v;
    } else if (sink == PT_DW_ACC_BF16) {
      uint16_t* o = (uint16_t*)out;
      o[col] = f2bf(bf2f(o[col]) + round_bf(v));
    } else {
      ((uint16_t*)out)[col] = f2bf(v);
    }
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
  switch (nch_for(cols)) {  // one partial row per bwd block
    case 1: return bwd_grid<1>(rows);
    case 2: return bwd_grid<2>(rows);
    case 4: return bwd_grid<4>(rows);
    case 8: return bwd_grid<8>(rows);
    default: return PT_EUNSUPPORTED;
  }
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
  const int nmode = mode & 3;
  if (nmode > 1 || (mode & PT_DW_ACC_BF16 && mode & PT_DW_ACC_F32)) return PT_EINVAL;
  const int nparts = pt_rmsnorm_bwd_partials(rows, (int)cols);
  const auto* DY = (const uint16_t*)dy;
  const auto* Z = (const uint16_t*)z;
  const auto* W = (const uint16_t*)weight;
  const auto* DR = (const uint16_t*)dres;
  auto* DX = (uint16_t*)dx;
  switch (nch) {
    case 1: rmsnorm_bwd_kernel<1><<<bwd_grid<1>(rows), bwd_waves<1>() * 64, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    case 2: rmsnorm_bwd_kernel<2><<<bwd_grid<2>(rows), bwd_waves<2>() * 64, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    case 4: rmsnorm_bwd_kernel<4><<<bwd_grid<4>(rows), bwd_waves<4>() * 64, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    case 8: rmsnorm_bwd_kernel<8><<<bwd_grid<8>(rows), bwd_waves<8>() * 64, 0, stream>>>(DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    default: return PT_EUNSUPPORTED;
  }
  PT_CHECK_LAUNCH();
  if (dweight) {
    if (cols % 8) return PT_EUNSUPPORTED;
    colsum_kernel<<<(int)(cols / 8), kColsumThreads, 0, stream>>>(dw_partial, nparts, (int)cols, dweight,
                                                                  mode & (PT_DW_ACC_BF16 | PT_DW_ACC_F32));
    PT_CHECK_LAUNCH();
  }
  return PT_OK;
}

}  // extern "C"
