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
// Layout: rows x cols, row-major bf16, cols % 8 == 0.  One wavefront owns one row at a time; each
// lane holds NCH 16-byte chunks of the row in registers, so every input is read from HBM exactly
// once.  HBM-bound: fwd moves 4*rows*cols bytes (8 with the residual: x, r in; z, y out), bwd
// 8*rows*cols with the fused residual gradient (dy, z, dres in; dx out).
//
// Rows are grid-strided over a grid sized so that every block is resident at once (at the layer's
// 4096 rows: one row per wave, all loads in flight from the start); the register budget is kept
// at <= 128 VGPRs for that (see the backward's second pass).
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int kCUs = 256;

// launch shape: waves per block and blocks per CU (grid cap) of the forward and backward kernels.
// Measured at T 4096 (tools/norm_bench.py, profiles/r02_norm_bench.log, r02_notes.md): forward 4
// waves x 4 blocks per CU; backward 16 waves x 1 block per CU (backward + column sum 17.5-18.4 us vs
// 19.2 with 8 x 2: one 1024-thread block per CU halves the partial rows), 4 waves for the 8-chunk
// rows (cols > 2048: 16 waves of those would not fit the LDS row buffers and spill).
// Below 4096 rows (the TP sequence-parallel shards: T / tp rows per rank, 512 at TP = 8) those
// shapes leave most CUs idle -- 32 backward blocks of 16 waves for 512 rows, 10.4 us -- so the
// blocks shrink with the rows until they cover the 256 CUs: 16 / 4 / 2 waves per backward block at
// >= 4096 / >= 1024 / fewer rows, and 4 / 1 waves per forward block at >= 4096 / fewer rows.
constexpr int kFwdWpb = 4, kFwdBpc = 4, kBwdBpc = 1;
constexpr int fwd_wpb(int64_t rows) { return rows >= 4096 ? kFwdWpb : 1; }
constexpr int bwd_wpb(int nch, int64_t rows) { return nch == 8 ? (rows >= 1024 ? 4 : 2) : (rows >= 4096 ? 16 : rows >= 1024 ? 4 : 2); }

template <int NCH>
__device__ __forceinline__ void load_row(const uint16_t* __restrict__ p, int lane, int nchunk, bf16x8 (&v)[NCH]) {
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * PT_WAVE;
    if (c < nchunk) v[i] = ld8(p + c * 8);
  }
}

// waves per SIMD the register allocation must allow: every block resident at once (NCH <= 4)
template <int NCH>
constexpr int min_waves() { return NCH <= 4 ? 4 : 2; }

template <int NCH, int WPB>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(min_waves<NCH>()))) void rmsnorm_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ y, uint16_t* __restrict__ z_out, float* __restrict__ rstd_out,
    int64_t rows, int cols, float eps, int mode) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * WPB;
  int64_t row = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int nchunk = cols >> 3;
  const float inv_cols = 1.0f / (float)cols;

  bf16x8 wv[NCH];  // row-invariant weight chunks
  load_row<NCH>(w, lane, nchunk, wv);

  for (; row < rows; row += stride) {
    bf16x8 xc[NCH], rc[NCH];
    load_row<NCH>(x + row * cols, lane, nchunk, xc);
    if (res) load_row<NCH>(res + row * cols, lane, nchunk, rc);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float v[8];
        unpack8(xc[i], v);
        if (res) {
          float r[8];
          unpack8(rc[i], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + r[j]);  // bf16 residual stream
          xc[i] = pack8(v);                                           // exact: v is bf16-valued
          st8(z_out + row * cols + c * 8, xc[i]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
      }
    }
    // keep the row packed (bf16) across the reduction, not as 8*NCH f32 registers
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(xc[i].w[k]), "+v"(wv[i].w[k]));
    ss = wave_sum(ss);
    const float rstd = rsqrtf(ss * inv_cols + eps);
    if (lane == 0) rstd_out[row] = rstd;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float v[8], o[8], wf[8];
        unpack8(xc[i], v);
        unpack8(wv[i], wf);
        if (mode == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[j] * rstd * wf[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = wf[j] * round_bf(v[j] * rstd);
        }
        st8(y + row * cols + c * 8, pack8(o));
      }
    }
  }
}

// dz = rstd * (dxh - xh * mean(dxh * xh)),  dxh = dy * w,  xh = z * rstd
// dx = dz (+ dres when the residual branch gradient is fused in)
// dw partial per block: sum over this block's rows of dy * xh (mode 1: dy * bf16(xh)), the block's
// waves combined through LDS in a fixed order -> one partial row per block (deterministic).
// SPLIT: dy arrives as the two f32 K halves of a split-K dX GEMM (gemm.hip splitk_sum2_kernel's
// inputs) and is formed here as bf16(p0 + p1) -- the sum pass's own rounding -- so the bf16 dy is
// never written and re-read (dy_p1 = the second half; dy = the first, as float)
template <int NCH>
__device__ __forceinline__ void load_split_row(const float* __restrict__ p0, const float* __restrict__ p1, int lane,
                                               int nchunk, bf16x8 (&v)[NCH]) {
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + i * PT_WAVE;
    if (c < nchunk) {
      const float4 a0 = *(const float4*)(p0 + c * 8), a1 = *(const float4*)(p0 + c * 8 + 4);
      const float4 b0 = *(const float4*)(p1 + c * 8), b1 = *(const float4*)(p1 + c * 8 + 4);
      float f[8] = {a0.x + b0.x, a0.y + b0.y, a0.z + b0.z, a0.w + b0.w,
                    a1.x + b1.x, a1.y + b1.y, a1.z + b1.z, a1.w + b1.w};
      v[i] = pack8(f);
    }
  }
}

template <int NCH, int WPB, bool SPLIT = false>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(min_waves<NCH>()))) void rmsnorm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ z, const uint16_t* __restrict__ w,
    const float* __restrict__ rstd_in, const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
    float* __restrict__ dw_partial, int64_t rows, int cols, int mode, const float* __restrict__ dy_p1 = nullptr) {
  extern __shared__ float red[];  // [WPB][cols]
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nchunk = cols >> 3;
  const float inv_cols = 1.0f / (float)cols;
  const int64_t stride = (int64_t)gridDim.x * WPB;
  int64_t row = (int64_t)blockIdx.x * WPB + wid;

  bf16x8 wv[NCH];
  load_row<NCH>(w, lane, nchunk, wv);
  // the wave's dw accumulator is its own LDS row (not 8*NCH registers): read-modify-written once
  // per chunk per row, no barrier needed until the cross-wave combine.  Planar: columns 0-3 of
  // chunk c at [4c], columns 4-7 at [cols / 2 + 4c], so a wave's 16-byte accesses are lane-
  // contiguous (chunk-interleaved 32-byte lanes were 2-way bank conflicts)
  float* dwrow = red + wid * cols;
  const int half = cols >> 1;
  for (int c = lane; c < nchunk; c += PT_WAVE) {
    *(float4*)(dwrow + c * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(dwrow + half + c * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  for (; row < rows; row += stride) {
    bf16x8 zc[NCH], dc[NCH], rc[NCH];
    load_row<NCH>(z + row * cols, lane, nchunk, zc);
    if constexpr (SPLIT)
      load_split_row<NCH>((const float*)dy + row * cols, dy_p1 + row * cols, lane, nchunk, dc);
    else
      load_row<NCH>(dy + row * cols, lane, nchunk, dc);
    if (dres) load_row<NCH>(dres + row * cols, lane, nchunk, rc);
    const float rstd = rstd_in[row];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float zz[8], d[8], wf[8], g[8];
        unpack8(zc[i], zz);
        unpack8(dc[i], d);
        unpack8(wv[i], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = zz[j] * rstd;
          dot += d[j] * wf[j] * xh;
          g[j] = d[j] * (mode == 0 ? xh : round_bf(xh));
        }
        float4* acc0 = (float4*)(dwrow + c * 4);
        float4* acc1 = (float4*)(dwrow + half + c * 4);
        float4 a0 = *acc0, a1 = *acc1;
        a0.x += g[0]; a0.y += g[1]; a0.z += g[2]; a0.w += g[3];
        a1.x += g[4]; a1.y += g[5]; a1.z += g[6]; a1.w += g[7];
        *acc0 = a0; *acc1 = a1;
      }
    }
    // the f32 unpacked row is not kept live across the reduction (it would double the VGPRs
    // and halve the waves per CU): the second pass re-expands the packed chunks
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(zc[i].w[k]), "+v"(dc[i].w[k]), "+v"(wv[i].w[k]));
    dot = wave_sum(dot) * inv_cols;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + i * PT_WAVE;
      if (c < nchunk) {
        float zz[8], d[8], wf[8], o[8];
        unpack8(zc[i], zz);
        unpack8(dc[i], d);
        unpack8(wv[i], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = zz[j] * rstd;
          o[j] = rstd * (d[j] * wf[j] - xh * dot);
        }
        if (dres) {
          float r[8];
          unpack8(rc[i], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        st8(dx + row * cols + c * 8, pack8(o));
      }
    }
  }

  // combine the block's waves (fixed order), one partial row per block
  __syncthreads();
  for (int col = threadIdx.x; col < cols; col += WPB * 64) {
    const int at = ((col & 7) >> 2) * half + (col >> 3) * 4 + (col & 3);   // the planar slot
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WPB; ++k) s += red[k * cols + at];
    dw_partial[(int64_t)blockIdx.x * cols + col] = s;
  }
}

// ------------------------------------------------------------------ rows wider than 4096 columns
// (Llama-2-13B 5120, 70B 8192: more 16-byte chunks per lane than the register-resident kernels
// hold).  One wave per row, the row streamed in 512-column passes twice: the sum of squares (the
// backward's dot) first, then the output from a second read of the same bytes (L2-resident by then;
// the residual form re-reads the z it wrote).  The backward's dW partial stays one LDS row per wave
// (planar, as above), combined per block in a fixed order: one partial row per block.
constexpr int kWideWpb = 4;   // waves per block; 2 above 8192 columns (LDS: WPB x cols x 4 B)
constexpr int kWideMax = 16384;
inline int wide_wpb(int cols) { return cols > 8192 ? 2 : kWideWpb; }

__global__ __launch_bounds__(kWideWpb * 64) void rmsnorm_fwd_wide_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ y, uint16_t* z_out, float* __restrict__ rstd_out, int64_t rows, int cols, float eps,
    int mode) {
  const int lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const int nchunk = cols >> 3;
  const float inv_cols = 1.0f / (float)cols;
  for (int64_t row = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); row < rows; row += (int64_t)gridDim.x * wpb) {
    float ss = 0.f;
    for (int c = lane; c < nchunk; c += PT_WAVE) {
      float v[8];
      unpack8(ld8(x + row * cols + c * 8), v);
      if (res) {
        float r[8];
        unpack8(ld8(res + row * cols + c * 8), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + r[j]);   // bf16 residual stream
        st8(z_out + row * cols + c * 8, pack8(v));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    }
    ss = wave_sum(ss);
    const float rstd = rsqrtf(ss * inv_cols + eps);
    if (lane == 0) rstd_out[row] = rstd;
    const uint16_t* src = res ? z_out : x;   // the lane re-reads what it read (or wrote) above
    for (int c = lane; c < nchunk; c += PT_WAVE) {
      float v[8], wf[8], o[8];
      unpack8(ld8(src + row * cols + c * 8), v);
      unpack8(ld8(w + c * 8), wf);
      if (mode == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[j] * rstd * wf[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = wf[j] * round_bf(v[j] * rstd);
      }
      st8(y + row * cols + c * 8, pack8(o));
    }
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(kWideWpb * 64) void rmsnorm_bwd_wide_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ z, const uint16_t* __restrict__ w,
    const float* __restrict__ rstd_in, const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
    float* __restrict__ dw_partial, int64_t rows, int cols, int mode, const float* __restrict__ dy_p1) {
  extern __shared__ float red[];  // [wpb][cols], planar as rmsnorm_bwd_kernel's
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const int nchunk = cols >> 3, half = cols >> 1;
  const float inv_cols = 1.0f / (float)cols;
  float* dwrow = red + wid * cols;
  for (int c = lane; c < nchunk; c += PT_WAVE) {
    *(float4*)(dwrow + c * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    *(float4*)(dwrow + half + c * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto load_dy = [&](int64_t row, int c, float (&d)[8]) {
    if constexpr (SPLIT) {
      const float* p0 = (const float*)dy + row * cols + c * 8;
      const float* p1 = dy_p1 + row * cols + c * 8;
      const float4 a0 = *(const float4*)p0, a1 = *(const float4*)(p0 + 4);
      const float4 b0 = *(const float4*)p1, b1 = *(const float4*)(p1 + 4);
      float f[8] = {a0.x + b0.x, a0.y + b0.y, a0.z + b0.z, a0.w + b0.w,
                    a1.x + b1.x, a1.y + b1.y, a1.z + b1.z, a1.w + b1.w};
      unpack8(pack8(f), d);   // bf16(p0 + p1): the split-K sum pass's own rounding
    } else {
      unpack8(ld8(dy + row * cols + c * 8), d);
    }
  };
  for (int64_t row = (int64_t)blockIdx.x * wpb + wid; row < rows; row += (int64_t)gridDim.x * wpb) {
    const float rstd = rstd_in[row];
    float dot = 0.f;
    for (int c = lane; c < nchunk; c += PT_WAVE) {
      float zz[8], d[8], wf[8];
      unpack8(ld8(z + row * cols + c * 8), zz);
      load_dy(row, c, d);
      unpack8(ld8(w + c * 8), wf);
      float4* acc0 = (float4*)(dwrow + c * 4);
      float4* acc1 = (float4*)(dwrow + half + c * 4);
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = zz[j] * rstd;
        dot += d[j] * wf[j] * xh;
        g[j] = d[j] * (mode == 0 ? xh : round_bf(xh));
      }
      float4 a0 = *acc0, a1 = *acc1;
      a0.x += g[0]; a0.y += g[1]; a0.z += g[2]; a0.w += g[3];
      a1.x += g[4]; a1.y += g[5]; a1.z += g[6]; a1.w += g[7];
      *acc0 = a0; *acc1 = a1;
    }
    dot = wave_sum(dot) * inv_cols;
    for (int c = lane; c < nchunk; c += PT_WAVE) {
      float zz[8], d[8], wf[8], o[8];
      unpack8(ld8(z + row * cols + c * 8), zz);
      load_dy(row, c, d);
      unpack8(ld8(w + c * 8), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rstd * (d[j] * wf[j] - zz[j] * rstd * dot);
      if (dres) {
        float r[8];
        unpack8(ld8(dres + row * cols + c * 8), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += r[j];
      }
      st8(dx + row * cols + c * 8, pack8(o));
    }
  }
  __syncthreads();
  for (int col = threadIdx.x; col < cols; col += blockDim.x) {
    const int at = ((col & 7) >> 2) * half + (col >> 3) * 4 + (col & 3);
    float s = 0.f;
    for (int k = 0; k < wpb; ++k) s += red[k * cols + at];
    dw_partial[(int64_t)blockIdx.x * cols + col] = s;
  }
}

int wide_grid(int64_t rows, int wpb, int bpc) {
  const int64_t g = (rows + wpb - 1) / wpb, cap = (int64_t)kCUs * bpc;
  return (int)(g < cap ? g : cap);
}

void launch_bwd_wide(bool split, int grid, hipStream_t s, const uint16_t* DY, const uint16_t* Z, const uint16_t* W,
                     const float* rstd, const uint16_t* DR, uint16_t* DX, float* part, int64_t rows, int cols,
                     int mode, const float* P1) {
  const int wpb = wide_wpb(cols);
  const size_t lds = (size_t)wpb * cols * sizeof(float);
  static bool attr[2] = {false, false};
  if (!attr[split]) {
    (void)hipFuncSetAttribute(split ? (const void*)rmsnorm_bwd_wide_kernel<true> : (const void*)rmsnorm_bwd_wide_kernel<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr[split] = true;
  }
  if (split)
    rmsnorm_bwd_wide_kernel<true><<<grid, wpb * 64, lds, s>>>(DY, Z, W, rstd, DR, DX, part, rows, cols, mode, P1);
  else
    rmsnorm_bwd_wide_kernel<false><<<grid, wpb * 64, lds, s>>>(DY, Z, W, rstd, DR, DX, part, rows, cols, mode, P1);
}

// dw[col] = sum_p partial[p][col]  -- fixed summation order, deterministic.  One block per 32
// columns: 8 lanes x 16 B cover a partial row's 32 columns (128 contiguous bytes per row), the 128
// lane groups of the 1024-thread block take every 128th partial row (all of a thread's rows loaded
// before any is added), then a fixed-order two-level sum over the groups (4 groups per thread, then
// 32).  (256 threads and 32 groups: 16 dependent rows per thread, one wave per CU -- 4.9 us for
// the 4 MB of partials at T 4096.)
// Sink (flags): 0 store bf16, DW_ACC_BF16 bf16 accumulate (= autograd's grad + bf16(new)),
// DW_ACC_F32 f32 accumulate (DataParallelBucket main_grad).
constexpr int kCsCols = 32, kCsThreads = 1024, kCsGroups = kCsThreads / (kCsCols / 4);
__device__ __forceinline__ void colsum_block(const float* __restrict__ partial, int nparts, int cols,
                                             void* __restrict__ out, int sink) {
  __shared__ float red[kCsGroups][kCsCols + 1];
  __shared__ float red2[kCsThreads / kCsCols][kCsCols + 1];
  const int t = threadIdx.x, ch = t & 7, grp = t >> 3;
  const int col4 = blockIdx.x * kCsCols + ch * 4;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col4 < cols) {
    constexpr int kPre = 4;  // rows in flight per thread (nparts <= 4 x 128 at the layer's shapes)
    int p = grp;
    for (; p + (kPre - 1) * kCsGroups < nparts; p += kPre * kCsGroups) {
      float4 a[kPre];
#pragma unroll
      for (int k = 0; k < kPre; ++k) a[k] = *(const float4*)(partial + (int64_t)(p + k * kCsGroups) * cols + col4);
#pragma unroll
      for (int k = 0; k < kPre; ++k) { s0 += a[k].x; s1 += a[k].y; s2 += a[k].z; s3 += a[k].w; }
    }
    for (; p < nparts; p += kCsGroups) {
      const float4 a = *(const float4*)(partial + (int64_t)p * cols + col4);
      s0 += a.x; s1 += a.y; s2 += a.z; s3 += a.w;
    }
  }
  red[grp][ch * 4 + 0] = s0; red[grp][ch * 4 + 1] = s1;
  red[grp][ch * 4 + 2] = s2; red[grp][ch * 4 + 3] = s3;
  __syncthreads();
  {  // level 1: thread (part, c) sums groups 4 part .. 4 part + 3 of column c
    const int c = t & (kCsCols - 1), part = t / kCsCols;
    constexpr int per = kCsGroups / (kCsThreads / kCsCols);
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < per; ++g) v += red[part * per + g][c];
    red2[part][c] = v;
  }
  __syncthreads();
  const int col = blockIdx.x * kCsCols + t;
  if (t < kCsCols && col < cols) {
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < kCsThreads / kCsCols; ++g) v += red2[g][t];
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

__global__ __launch_bounds__(kCsThreads) void colsum_kernel(const float* __restrict__ partial, int nparts,
                                                            int cols, void* __restrict__ out, int sink) {
  colsum_block(partial, nparts, cols, out, sink);
}

// several norms' column sums in one launch (blockIdx.y = the norm): the backward of a micro-batch
// defers its 2 L norms' sums to one launch at its end (picotron_amd/functional.py norm_bwd)
constexpr int kCsBatch = 32;
struct ColsumBatch {
  const float* partial[kCsBatch];
  void* out[kCsBatch];
  int nparts[kCsBatch];
  int sink[kCsBatch];
};
__global__ __launch_bounds__(kCsThreads) void colsum_batch_kernel(const ColsumBatch b, int cols) {
  const int i = blockIdx.y;
  colsum_block(b.partial[i], b.nparts[i], cols, b.out[i], b.sink[i]);
}

int nch_for(int cols) {
  const int chunks = cols / 8;
  if (chunks <= 64) return 1;
  if (chunks <= 128) return 2;
  if (chunks <= 256) return 4;
  if (chunks <= 512) return 8;
  return -1;
}

int grid_for(int64_t rows, int wpb, int bpc) {
  const int64_t g = (rows + wpb - 1) / wpb, cap = (int64_t)kCUs * bpc;
  return (int)(g < cap ? g : cap);
}

template <int NCH>
void launch_fwd(hipStream_t s, const uint16_t* X, const uint16_t* R, const uint16_t* W, uint16_t* Y,
                uint16_t* Z, float* rstd, int64_t rows, int cols, float eps, int mode) {
  if (fwd_wpb(rows) == kFwdWpb)
    rmsnorm_fwd_kernel<NCH, kFwdWpb><<<grid_for(rows, kFwdWpb, kFwdBpc), kFwdWpb * 64, 0, s>>>(X, R, W, Y, Z, rstd,
                                                                                              rows, cols, eps, mode);
  else
    rmsnorm_fwd_kernel<NCH, 1><<<grid_for(rows, 1, kFwdBpc * kFwdWpb), 64, 0, s>>>(X, R, W, Y, Z, rstd, rows, cols,
                                                                                  eps, mode);
}

// LDS: wpb * cols * 4 (128 KiB at 16 waves x 2048 columns)
template <int NCH, int WPB, bool SPLIT>
void launch_bwd_w(int grid, hipStream_t s, const uint16_t* DY, const uint16_t* Z, const uint16_t* W,
                  const float* rstd, const uint16_t* DR, uint16_t* DX, float* part, int64_t rows, int cols, int mode,
                  const float* P1) {
  const size_t lds = (size_t)WPB * cols * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)rmsnorm_bwd_kernel<NCH, WPB, SPLIT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  rmsnorm_bwd_kernel<NCH, WPB, SPLIT><<<grid, WPB * 64, lds, s>>>(DY, Z, W, rstd, DR, DX, part, rows, cols, mode, P1);
}

template <int NCH, bool SPLIT = false>
void launch_bwd(int grid, hipStream_t s, const uint16_t* DY, const uint16_t* Z, const uint16_t* W,
                const float* rstd, const uint16_t* DR, uint16_t* DX, float* part, int64_t rows, int cols, int mode,
                const float* P1 = nullptr) {
  switch (bwd_wpb(NCH, rows)) {
    case 16:
      if constexpr (NCH != 8) launch_bwd_w<NCH, 16, SPLIT>(grid, s, DY, Z, W, rstd, DR, DX, part, rows, cols, mode, P1);
      break;
    case 4: launch_bwd_w<NCH, 4, SPLIT>(grid, s, DY, Z, W, rstd, DR, DX, part, rows, cols, mode, P1); break;
    default: launch_bwd_w<NCH, 2, SPLIT>(grid, s, DY, Z, W, rstd, DR, DX, part, rows, cols, mode, P1); break;
  }
}

}  // namespace

extern "C" {

int pt_rmsnorm_bwd_partials(int64_t rows, int cols) {
  const int nch = nch_for(cols);
  if (nch < 0) {
    if (cols > kWideMax || (cols & 7)) return PT_EUNSUPPORTED;
    return wide_grid(rows, wide_wpb(cols), 1);   // the wide-row backward: one partial row per block
  }
  return grid_for(rows, bwd_wpb(nch, rows), kBwdBpc);  // one partial row per bwd block
}

int pt_rmsnorm_fwd(const void* x, const void* residual, const void* weight, void* y, void* z_out,
                   float* rstd, int64_t rows, int64_t cols, float eps, int mode, hipStream_t stream) {
  if (!x || !weight || !y || !rstd || rows <= 0 || cols <= 0 || (cols & 7)) return PT_EINVAL;
  if (residual && !z_out) return PT_EINVAL;
  if (!pt_aligned16(x) || !pt_aligned16(weight) || !pt_aligned16(y)) return PT_EALIGN;
  if (residual && (!pt_aligned16(residual) || !pt_aligned16(z_out))) return PT_EALIGN;
  const auto* X = (const uint16_t*)x;
  const auto* R = (const uint16_t*)residual;
  const auto* W = (const uint16_t*)weight;
  auto* Y = (uint16_t*)y;
  auto* Z = (uint16_t*)z_out;
  switch (nch_for((int)cols)) {
    case 1: launch_fwd<1>(stream, X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    case 2: launch_fwd<2>(stream, X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    case 4: launch_fwd<4>(stream, X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    case 8: launch_fwd<8>(stream, X, R, W, Y, Z, rstd, rows, (int)cols, eps, mode); break;
    default:
      if (cols > kWideMax) return PT_EUNSUPPORTED;
      rmsnorm_fwd_wide_kernel<<<wide_grid(rows, kWideWpb, 4), kWideWpb * 64, 0, stream>>>(X, R, W, Y, Z, rstd, rows,
                                                                                         (int)cols, eps, mode);
      break;
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
  if (nch < 0 && cols > kWideMax) return PT_EUNSUPPORTED;
  const int nmode = mode & 3;
  if (nmode > 1 || (mode & PT_DW_ACC_BF16 && mode & PT_DW_ACC_F32)) return PT_EINVAL;
  const int grid = nch < 0 ? wide_grid(rows, wide_wpb((int)cols), 1) : grid_for(rows, bwd_wpb(nch, rows), kBwdBpc);
  const auto* DY = (const uint16_t*)dy;
  const auto* Z = (const uint16_t*)z;
  const auto* W = (const uint16_t*)weight;
  const auto* DR = (const uint16_t*)dres;
  auto* DX = (uint16_t*)dx;
  switch (nch) {
    case 1: launch_bwd<1>(grid, stream, DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    case 2: launch_bwd<2>(grid, stream, DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    case 4: launch_bwd<4>(grid, stream, DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    case 8: launch_bwd<8>(grid, stream, DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode); break;
    default: launch_bwd_wide(false, grid, stream, DY, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode, nullptr);
  }
  PT_CHECK_LAUNCH();
  if (dweight) {
    colsum_kernel<<<(int)((cols + kCsCols - 1) / kCsCols), kCsThreads, 0, stream>>>(
        dw_partial, grid, (int)cols, dweight, mode & (PT_DW_ACC_BF16 | PT_DW_ACC_F32));
    PT_CHECK_LAUNCH();
  }
  return PT_OK;
}

// pt_rmsnorm_bwd with dy = bf16(dy_p0 + dy_p1): the two f32 K halves [rows, cols] (contiguous) of a
// split-K dX GEMM, summed here instead of by pt_gemm_splitk_sum (bit-identical to that sum followed
// by pt_rmsnorm_bwd)
int pt_rmsnorm_bwd_splitk(const float* dy_p0, const float* dy_p1, const void* z, const void* weight,
                          const float* rstd, const void* dres, void* dx, void* dweight, float* dw_partial,
                          int64_t rows, int64_t cols, int mode, hipStream_t stream) {
  if (!dy_p0 || !dy_p1 || !z || !weight || !rstd || !dx || !dw_partial || rows <= 0 || cols <= 0 || (cols & 7))
    return PT_EINVAL;
  if (!pt_aligned16(dy_p0) || !pt_aligned16(dy_p1) || !pt_aligned16(z) || !pt_aligned16(dx) ||
      (dres && !pt_aligned16(dres)))
    return PT_EALIGN;
  const int nch = nch_for((int)cols);
  if (nch < 0 && cols > kWideMax) return PT_EUNSUPPORTED;
  const int nmode = mode & 3;
  if (nmode > 1 || (mode & PT_DW_ACC_BF16 && mode & PT_DW_ACC_F32)) return PT_EINVAL;
  const int grid = nch < 0 ? wide_grid(rows, wide_wpb((int)cols), 1) : grid_for(rows, bwd_wpb(nch, rows), kBwdBpc);
  const auto* P0 = (const uint16_t*)dy_p0;  // reinterpreted as float inside the SPLIT kernel
  const auto* Z = (const uint16_t*)z;
  const auto* W = (const uint16_t*)weight;
  const auto* DR = (const uint16_t*)dres;
  auto* DX = (uint16_t*)dx;
  switch (nch) {
    case 1: launch_bwd<1, true>(grid, stream, P0, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode, dy_p1); break;
    case 2: launch_bwd<2, true>(grid, stream, P0, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode, dy_p1); break;
    case 4: launch_bwd<4, true>(grid, stream, P0, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode, dy_p1); break;
    case 8: launch_bwd<8, true>(grid, stream, P0, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode, dy_p1); break;
    default: launch_bwd_wide(true, grid, stream, P0, Z, W, rstd, DR, DX, dw_partial, rows, (int)cols, nmode, dy_p1);
  }
  PT_CHECK_LAUNCH();
  if (dweight) {
    colsum_kernel<<<(int)((cols + kCsCols - 1) / kCsCols), kCsThreads, 0, stream>>>(
        dw_partial, grid, (int)cols, dweight, mode & (PT_DW_ACC_BF16 | PT_DW_ACC_F32));
    PT_CHECK_LAUNCH();
  }
  return PT_OK;
}

// dweight[i] (+)= column sums of partials[i] ([nparts[i], cols] f32, from pt_rmsnorm_bwd called with
// dweight = NULL) for n <= 32 norms of the same width, one launch; sinks[i] as pt_rmsnorm_bwd's
// PT_DW_ACC_* bits (0 = bf16 store).  Bit-identical to the per-norm sums.
int pt_rmsnorm_colsum_batch(const float* const* partials, const int* nparts, void* const* dweights,
                            const int* sinks, int n, int64_t cols, hipStream_t stream) {
  if (!partials || !nparts || !dweights || !sinks || n <= 0 || n > kCsBatch || cols <= 0 || (cols & 7))
    return PT_EINVAL;
  ColsumBatch b{};
  for (int i = 0; i < n; ++i) {
    if (!partials[i] || !dweights[i] || nparts[i] <= 0) return PT_EINVAL;
    if (sinks[i] != 0 && sinks[i] != PT_DW_ACC_BF16 && sinks[i] != PT_DW_ACC_F32) return PT_EINVAL;
    b.partial[i] = partials[i];
    b.out[i] = dweights[i];
    b.nparts[i] = nparts[i];
    b.sink[i] = sinks[i];
  }
  const dim3 grid((unsigned)((cols + kCsCols - 1) / kCsCols), (unsigned)n);
  colsum_batch_kernel<<<grid, kCsThreads, 0, stream>>>(b, (int)cols);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

}  // extern "C"
