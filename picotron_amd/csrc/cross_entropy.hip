// Fused cross-entropy forward + backward over bf16 logits (one read, one in-place write).
//
// Replaces (reference, /root/reference): train.py:48-49
//   loss = F.cross_entropy(logits.view(-1, V), targets, reduction='mean') / grad_acc_steps
// and its autograd backward (softmax - onehot), and the PP variant pipeline_parallel.py:103,153.
//
//   row_loss[r] = lse_r - x[r, t_r]            (0 for t_r == ignore_index)
//   dlogits[r,:] = (softmax(x[r,:]) - onehot(t_r)) * scale * (*inv_count if given)
// where the caller sets scale = 1/grad_acc and inv_count = 1/#valid rows (on device, so the
// host never synchronises).  dlogits may alias logits (in place: the logits are dead after the
// loss, which saves a 384 MiB buffer at SmolLM-1.7B mbs4 seq1024).
//
// Targets are range-checked: a target outside [0, V) that is not ignore_index gives a NaN row loss
// (and, through the saved NaN LSE, a NaN gradient row), never an out-of-bounds read, and sets bit
// PT_STATUS_BAD_TARGET of *status (when given) -- torch's device-side assert, made observable
// without a trap (kernels.device_status / functional.check_device_status read it).
//
// One 256-thread workgroup per row; the row is held in registers (NC 16-byte chunks per
// thread) so HBM sees exactly one read and one write of the logits: 4*V bytes per row, the
// roofline figure in DESIGN.md.  Rows longer than 256*8*32 elements take the two-pass variant.
#include "common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < kThreads / 64; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  __syncthreads();
  return r;
}

template <int NC>
__global__ __launch_bounds__(kThreads) void ce_kernel(const uint16_t* __restrict__ logits, int64_t ls,
                                                      const int64_t* __restrict__ tgt, uint16_t* dlogits,
                                                      int64_t ds, float* __restrict__ row_loss, int V,
                                                      float scale, const float* __restrict__ inv_count,
                                                      int64_t ignore_index, int* __restrict__ status) {
  __shared__ float red[kThreads / 64];
  const int64_t row = blockIdx.x;
  const uint16_t* x = logits + row * ls;
  const int nch = V >> 3;
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  const bool bad = valid && (t < 0 || t >= V);
  // read the target logit before any barrier: later writes may overwrite x in place
  const float xt = (threadIdx.x == 0 && valid && !bad) ? bf2f(x[t]) : 0.f;
  if (bad && threadIdx.x == 0 && status) status[0] = PT_STATUS_BAD_TARGET;
  bf16x8 v[NC];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = threadIdx.x + i * kThreads;
    if (c < nch) {
      v[i] = ld8(x + c * 8);
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, f[j]);
    }
  }
  mx = block_reduce(mx, red, true);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = threadIdx.x + i * kThreads;
    if (c < nch) {
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) se += __expf(f[j] - mx);
    }
  }
  se = block_reduce(se, red, false);
  const float lse = bad ? __builtin_nanf("") : mx + __logf(se);
  const float g = valid ? scale * (inv_count ? *inv_count : 1.0f) : 0.f;
  if (threadIdx.x == 0) row_loss[row] = valid ? lse - xt : 0.f;
  if (!dlogits) return;  // loss-only (forward) launch
  uint16_t* d = dlogits + row * ds;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = threadIdx.x + i * kThreads;
    if (c < nch) {
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __expf(f[j] - lse);
        f[j] = (p - ((int64_t)(c * 8 + j) == t ? 1.f : 0.f)) * g;
      }
      st8(d + c * 8, pack8(f));
    }
  }
}

// long rows: online max/sum in one read, gradient in a second read
__global__ __launch_bounds__(kThreads) void ce_kernel_2pass(const uint16_t* __restrict__ logits, int64_t ls,
                                                            const int64_t* __restrict__ tgt, uint16_t* dlogits,
                                                            int64_t ds, float* __restrict__ row_loss, int V,
                                                            float scale, const float* __restrict__ inv_count,
                                                            int64_t ignore_index, int* __restrict__ status) {
  __shared__ float red[kThreads / 64];
  __shared__ float red2[kThreads / 64];
  const int64_t row = blockIdx.x;
  const uint16_t* x = logits + row * ls;
  const int nch = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nch; c += kThreads) {
    float f[8];
    unpack8(ld8(x + c * 8), f);
    float cm = m;
#pragma unroll
    for (int j = 0; j < 8; ++j) cm = fmaxf(cm, f[j]);
    s *= __expf(m - cm);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(f[j] - cm);
    m = cm;
  }
  // combine (m, s) pairs across the block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) { red[wid] = m; red2[wid] = s; }
  __syncthreads();
  float M = red[0];
  for (int i = 1; i < kThreads / 64; ++i) M = fmaxf(M, red[i]);
  float S = 0.f;
  for (int i = 0; i < kThreads / 64; ++i) S += red2[i] * __expf(red[i] - M);
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  const bool bad = valid && (t < 0 || t >= V);
  const float lse = bad ? __builtin_nanf("") : M + __logf(S);
  const float g = valid ? scale * (inv_count ? *inv_count : 1.0f) : 0.f;
  if (threadIdx.x == 0) row_loss[row] = valid ? lse - (bad ? 0.f : bf2f(x[t])) : 0.f;
  if (bad && threadIdx.x == 0 && status) status[0] = PT_STATUS_BAD_TARGET;
  __syncthreads();  // x[t] read before any in-place write
  if (!dlogits) return;
  uint16_t* d = dlogits + row * ds;
  for (int c = threadIdx.x; c < nch; c += kThreads) {
    float f[8];
    unpack8(ld8(x + c * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (__expf(f[j] - lse) - ((int64_t)(c * 8 + j) == t ? 1.f : 0.f)) * g;
    st8(d + c * 8, pack8(f));
  }
}

// ---- streaming pair: the autograd forward saves the row LSE so the backward needs no reduction
//
// fwd: one 256-thread workgroup per row, online (max, sum-exp) over 4 chunks (32 logits) at a time
// with the 4 loads issued together -- a handful of registers, so many rows stream at once (the
// register-resident ce_kernel above caps occupancy at ~4 waves per SIMD for V = 49152).
// bwd: purely elementwise  dl = (exp(x - lse_row) - onehot) * g,  4 chunks in flight per thread.
constexpr int kUnroll = 4;
constexpr float kLog2e = 1.4426950408889634f;

__global__ __launch_bounds__(kThreads) void ce_fwd_stream_kernel(const uint16_t* __restrict__ logits, int64_t ls,
                                                                 const int64_t* __restrict__ tgt,
                                                                 float* __restrict__ row_loss,
                                                                 float* __restrict__ row_lse, int V,
                                                                 int64_t ignore_index, int* __restrict__ status) {
  __shared__ float red[kThreads / 64];
  __shared__ float red2[kThreads / 64];
  const int64_t row = blockIdx.x;
  const uint16_t* x = logits + row * ls;
  const int nch = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (int c0 = threadIdx.x; c0 < nch; c0 += kThreads * kUnroll) {
    bf16x8 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int c = c0 + u * kThreads;
      if (c < nch) v[u] = ld8(x + c * 8);
    }
    float f[kUnroll][8];
    float cm = m;
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int c = c0 + u * kThreads;
      if (c < nch) {
        unpack8(v[u], f[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) cm = fmaxf(cm, f[u][j]);
      }
    }
    if (cm == -INFINITY) continue;  // nothing finite seen yet
    // base-2 domain: exp(x - cm) = exp2(x log2e - cm log2e), one fma + one v_exp per logit
    const float ncl = -cm * kLog2e;
    s *= __builtin_amdgcn_exp2f(fmaf(m, kLog2e, ncl));
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int c = c0 + u * kThreads;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) s += __builtin_amdgcn_exp2f(fmaf(f[u][j], kLog2e, ncl));
      }
    }
    m = cm;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) { red[wid] = m; red2[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red[0];
    for (int i = 1; i < kThreads / 64; ++i) M = fmaxf(M, red[i]);
    float S = 0.f;
    for (int i = 0; i < kThreads / 64; ++i) S += red2[i] * __expf(red[i] - M);
    const int64_t t = tgt[row];
    const bool valid = t != ignore_index;
    const bool bad = valid && (t < 0 || t >= V);
    const float lse = bad ? __builtin_nanf("") : M + __logf(S);
    row_lse[row] = lse;
    row_loss[row] = valid ? lse - (bad ? 0.f : bf2f(x[t])) : 0.f;
    if (bad && status) status[0] = PT_STATUS_BAD_TARGET;
  }
}

// Forward from the lm_head GEMM's statistics (gemm.hip EPI_CE_STATS): float2 stats[b][row] =
// (m_b, s_b = sum exp(x - m_b)) over the nblk column tiles -> lse = M + log(sum_b s_b exp(m_b - M)),
// M = max_b m_b; row_loss = lse - x[t].  A block = 32 rows x 8 tile groups: each lane merges every
// 8th tile of its row online (32 lanes read 256 contiguous bytes of one tile's pairs), then the 8
// partial merges of a row are combined in a fixed order.  The [rows, V] logits are not read again
// (only x[t]).
constexpr int kStatRows = 32, kStatGroups = 8;
__global__ __launch_bounds__(kStatRows * kStatGroups) void ce_fwd_stats_kernel(
    const uint16_t* __restrict__ logits, int64_t ls, const int64_t* __restrict__ tgt,
    const float2* __restrict__ stats, int nblk, float* __restrict__ row_loss, float* __restrict__ row_lse,
    int64_t rows, int V, int64_t ignore_index, int* __restrict__ status) {
  __shared__ float2 part[kStatGroups][kStatRows];
  const int r = threadIdx.x % kStatRows, grp = threadIdx.x / kStatRows;
  const int64_t row = (int64_t)blockIdx.x * kStatRows + r;
  float m = -INFINITY, s = 0.f;
  if (row < rows) {
    for (int b = grp; b < nblk; b += kStatGroups) {
      const float2 p = stats[(int64_t)b * rows + row];
      const float nm = fmaxf(m, p.x);
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (p.x == -INFINITY ? 0.f : p.y * __expf(p.x - nm));
      m = nm;
    }
  }
  part[grp][r] = make_float2(m, s);
  __syncthreads();
  if (grp == 0 && row < rows) {
    for (int g = 1; g < kStatGroups; ++g) {
      const float2 p = part[g][r];
      const float nm = fmaxf(m, p.x);
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (p.x == -INFINITY ? 0.f : p.y * __expf(p.x - nm));
      m = nm;
    }
    const int64_t t = tgt[row];
    const bool valid = t != ignore_index;
    const bool bad = valid && (t < 0 || t >= V);
    const float lse = bad ? __builtin_nanf("") : m + __logf(s);
    row_lse[row] = lse;
    row_loss[row] = valid ? lse - (bad ? 0.f : bf2f(logits[row * ls + t])) : 0.f;
    if (bad && status) status[0] = PT_STATUS_BAD_TARGET;
  }
}

// mean over the valid rows (train.py:49's reduction='mean'): loss = sum(row_loss) / #valid, in ONE
// block with a fixed-shape reduction (deterministic); also 1/#valid for the backward and the loss in
// the logits' dtype.  #valid == 0 gives 0 * inf = NaN, as F.cross_entropy's mean does.
constexpr int kMeanThreads = 1024;
__global__ __launch_bounds__(kMeanThreads) void ce_mean_kernel(const float* __restrict__ row_loss,
                                                               const int64_t* __restrict__ tgt, int64_t rows,
                                                               int64_t ignore_index, float* __restrict__ loss_f32,
                                                               float* __restrict__ inv_count, void* __restrict__ out,
                                                               int out_bf16, int reduce_sum) {
  __shared__ float ssum[kMeanThreads];
  __shared__ int scnt[kMeanThreads];
  float s = 0.f;
  int c = 0;
  for (int64_t r = threadIdx.x; r < rows; r += kMeanThreads) {
    s += row_loss[r];
    c += tgt[r] != ignore_index;
  }
  ssum[threadIdx.x] = s;
  scnt[threadIdx.x] = c;
  __syncthreads();
  for (int w = kMeanThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      ssum[threadIdx.x] += ssum[threadIdx.x + w];
      scnt[threadIdx.x] += scnt[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float inv = reduce_sum ? 1.0f : 1.0f / (float)scnt[0];
    const float loss = reduce_sum ? ssum[0] : ssum[0] * inv;
    inv_count[0] = inv;
    if (loss_f32) loss_f32[0] = loss;
    if (out) {
      if (out_bf16) *(uint16_t*)out = f2bf(loss);
      else *(float*)out = loss;
    }
  }
}

__global__ __launch_bounds__(kThreads) void ce_bwd_stream_kernel(const uint16_t* __restrict__ logits, int64_t ls,
                                                                 const int64_t* __restrict__ tgt,
                                                                 const float* __restrict__ row_lse,
                                                                 uint16_t* __restrict__ dl, int64_t ds, int V,
                                                                 const float* __restrict__ scale_dev,
                                                                 int64_t scale_stride, int64_t ignore_index,
                                                                 int64_t vocab_lo) {
  const int64_t row = blockIdx.x;
  const uint16_t* x = logits + row * ls;
  uint16_t* d = dl + row * ds;
  const int nch = V >> 3;
  const int64_t t = tgt[row] - vocab_lo;   // a vocab shard [vocab_lo, vocab_lo + V): its own columns
  const float nl2 = -row_lse[row] * kLog2e;   // exp(x - lse) = exp2(x log2e - lse log2e)
  const float g = tgt[row] != ignore_index ? scale_dev[row * scale_stride] : 0.f;
  for (int c0 = threadIdx.x; c0 < nch; c0 += kThreads * kUnroll) {
    bf16x8 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int c = c0 + u * kThreads;
      if (c < nch) v[u] = ld8(x + c * 8);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int c = c0 + u * kThreads;
      if (c < nch) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          f[j] = (__builtin_amdgcn_exp2f(fmaf(f[j], kLog2e, nl2)) - ((int64_t)(c * 8 + j) == t ? 1.f : 0.f)) * g;
        st8(d + c * 8, pack8(f));
      }
    }
  }
}

// ---- vocab-parallel cross-entropy (the lm_head as a ColumnParallelLinear over tp ranks, each holding
// the logits of vocab columns [vocab_lo, vocab_lo + Vs)): instead of gathering the [rows, V] logits
// (tp_communications.py:51-72, 7/8 of them crossing xGMI at tp 8) every rank reduces its shard to a
// per-row float4 (m, s = sum exp(x - m), x[target] if the target is in the shard else 0, 1 / 0 flag),
// the tp group all-gathers those 16 bytes per row, and every rank combines them in rank order.
__global__ __launch_bounds__(kStatRows * kStatGroups) void ce_vp_partial_kernel(
    const uint16_t* __restrict__ logits, int64_t ls, const int64_t* __restrict__ tgt,
    const float2* __restrict__ stats, int nblk, float4* __restrict__ part_out, int64_t rows, int Vs,
    int64_t vocab_lo) {
  __shared__ float2 part[kStatGroups][kStatRows];
  const int r = threadIdx.x % kStatRows, grp = threadIdx.x / kStatRows;
  const int64_t row = (int64_t)blockIdx.x * kStatRows + r;
  float m = -INFINITY, s = 0.f;
  if (row < rows) {
    for (int b = grp; b < nblk; b += kStatGroups) {   // ce_fwd_stats_kernel's merge
      const float2 p = stats[(int64_t)b * rows + row];
      const float nm = fmaxf(m, p.x);
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (p.x == -INFINITY ? 0.f : p.y * __expf(p.x - nm));
      m = nm;
    }
  }
  part[grp][r] = make_float2(m, s);
  __syncthreads();
  if (grp == 0 && row < rows) {
    for (int g = 1; g < kStatGroups; ++g) {
      const float2 p = part[g][r];
      const float nm = fmaxf(m, p.x);
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (p.x == -INFINITY ? 0.f : p.y * __expf(p.x - nm));
      m = nm;
    }
    const int64_t t = tgt[row] - vocab_lo;
    const bool own = t >= 0 && t < Vs;
    part_out[row] = make_float4(m, s, own ? bf2f(logits[row * ls + t]) : 0.f, own ? 1.f : 0.f);
  }
}

// every rank's partials [tp][rows] -> row_lse, row_loss (lse - x[target]); the range check of
// ce_fwd_stats_kernel against the global vocab (NaN row + PT_STATUS_BAD_TARGET)
__global__ __launch_bounds__(256) void ce_vp_combine_kernel(const float4* __restrict__ parts, int tp,
                                                            const int64_t* __restrict__ tgt, float* __restrict__ row_loss,
                                                            float* __restrict__ row_lse, int64_t rows, int64_t V,
                                                            int64_t ignore_index, int* __restrict__ status) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float m = -INFINITY, s = 0.f, xt = 0.f;
  for (int q = 0; q < tp; ++q) {
    const float4 p = parts[(int64_t)q * rows + row];
    const float nm = fmaxf(m, p.x);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (p.x == -INFINITY ? 0.f : p.y * __expf(p.x - nm));
    m = nm;
    xt += p.z;
  }
  const int64_t t = tgt[row];
  const bool valid = t != ignore_index;
  const bool bad = valid && (t < 0 || t >= V);
  const float lse = bad ? __builtin_nanf("") : m + __logf(s);
  row_lse[row] = lse;
  row_loss[row] = valid ? lse - xt : 0.f;
  if (bad && status) status[0] = PT_STATUS_BAD_TARGET;
}

}  // namespace

extern "C" int pt_cross_entropy_vp_partial(const void* logits, int64_t logits_stride, const int64_t* targets,
                                           const float* stats, int64_t nblk, float* part, int64_t rows,
                                           int64_t vocab_shard, int64_t vocab_lo, hipStream_t stream) {
  if (!logits || !targets || !stats || !part || rows <= 0 || vocab_shard <= 0 || nblk <= 0) return PT_EINVAL;
  if (vocab_shard % nblk || !pt_aligned16(stats) || !pt_aligned16(part)) return PT_EINVAL;
  if (rows > INT32_MAX || vocab_shard > INT32_MAX) return PT_EUNSUPPORTED;
  const unsigned grid = (unsigned)((rows + kStatRows - 1) / kStatRows);
  ce_vp_partial_kernel<<<grid, kStatRows * kStatGroups, 0, stream>>>((const uint16_t*)logits, logits_stride, targets,
                                                                   (const float2*)stats, (int)nblk, (float4*)part,
                                                                   rows, (int)vocab_shard, vocab_lo);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

extern "C" int pt_cross_entropy_vp_combine(const float* parts, int64_t tp, const int64_t* targets, float* row_loss,
                                           float* row_lse, int64_t rows, int64_t vocab, int64_t ignore_index,
                                           int* status, hipStream_t stream) {
  if (!parts || !targets || !row_loss || !row_lse || rows <= 0 || vocab <= 0 || tp <= 0) return PT_EINVAL;
  if (!pt_aligned16(parts)) return PT_EALIGN;
  ce_vp_combine_kernel<<<(unsigned)((rows + 255) / 256), 256, 0, stream>>>((const float4*)parts, (int)tp, targets,
                                                                          row_loss, row_lse, rows, vocab,
                                                                          ignore_index, status);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

extern "C" int pt_cross_entropy_bwd_lse_shard(const void* logits, int64_t logits_stride, const int64_t* targets,
                                              const float* row_lse, void* dlogits, int64_t dlogits_stride,
                                              int64_t rows, int64_t vocab_shard, int64_t vocab_lo, const float* scale,
                                              int64_t scale_stride, int64_t ignore_index, hipStream_t stream) {
  if (!logits || !targets || !row_lse || !dlogits || !scale || rows <= 0 || vocab_shard <= 0) return PT_EINVAL;
  if (scale_stride != 0 && scale_stride != 1) return PT_EINVAL;
  if ((vocab_shard & 7) || (logits_stride & 7) || (dlogits_stride & 7)) return PT_EALIGN;
  if (!pt_aligned16(logits) || !pt_aligned16(dlogits)) return PT_EALIGN;
  if (rows > INT32_MAX || vocab_shard > INT32_MAX) return PT_EUNSUPPORTED;
  ce_bwd_stream_kernel<<<(unsigned)rows, kThreads, 0, stream>>>((const uint16_t*)logits, logits_stride, targets,
                                                               row_lse, (uint16_t*)dlogits, dlogits_stride,
                                                               (int)vocab_shard, scale, scale_stride, ignore_index,
                                                               vocab_lo);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

extern "C" int pt_cross_entropy_fwd_lse(const void* logits, int64_t logits_stride, const int64_t* targets,
                                        float* row_loss, float* row_lse, int64_t rows, int64_t vocab,
                                        int64_t ignore_index, int* status, hipStream_t stream) {
  if (!logits || !targets || !row_loss || !row_lse || rows <= 0 || vocab <= 0) return PT_EINVAL;
  if ((vocab & 7) || (logits_stride & 7) || !pt_aligned16(logits)) return PT_EALIGN;
  if (rows > INT32_MAX || vocab > INT32_MAX) return PT_EUNSUPPORTED;
  ce_fwd_stream_kernel<<<(unsigned)rows, kThreads, 0, stream>>>((const uint16_t*)logits, logits_stride, targets,
                                                               row_loss, row_lse, (int)vocab, ignore_index, status);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

extern "C" int pt_cross_entropy_bwd_lse(const void* logits, int64_t logits_stride, const int64_t* targets,
                                        const float* row_lse, void* dlogits, int64_t dlogits_stride, int64_t rows,
                                        int64_t vocab, const float* scale, int64_t scale_stride,
                                        int64_t ignore_index, hipStream_t stream) {
  if (!logits || !targets || !row_lse || !dlogits || !scale || rows <= 0 || vocab <= 0) return PT_EINVAL;
  if (scale_stride != 0 && scale_stride != 1) return PT_EINVAL;
  if ((vocab & 7) || (logits_stride & 7) || (dlogits_stride & 7)) return PT_EALIGN;
  if (!pt_aligned16(logits) || !pt_aligned16(dlogits)) return PT_EALIGN;
  if (rows > INT32_MAX || vocab > INT32_MAX) return PT_EUNSUPPORTED;
  ce_bwd_stream_kernel<<<(unsigned)rows, kThreads, 0, stream>>>((const uint16_t*)logits, logits_stride, targets,
                                                               row_lse, (uint16_t*)dlogits, dlogits_stride,
                                                               (int)vocab, scale, scale_stride, ignore_index, 0);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

extern "C" int pt_cross_entropy_fwd_bwd(const void* logits, int64_t logits_stride, const int64_t* targets,
                                        void* dlogits, int64_t dlogits_stride, float* row_loss, int64_t rows,
                                        int64_t vocab, float scale, const float* inv_count, int64_t ignore_index,
                                        int* status, hipStream_t stream) {
  if (!logits || !targets || !row_loss || rows <= 0 || vocab <= 0) return PT_EINVAL;
  if ((vocab & 7) || (logits_stride & 7) || (dlogits && (dlogits_stride & 7))) return PT_EALIGN;
  if (!pt_aligned16(logits) || (dlogits && !pt_aligned16(dlogits))) return PT_EALIGN;
  const auto* L = (const uint16_t*)logits;
  auto* D = (uint16_t*)dlogits;
  const int nc = (int)((vocab / 8 + kThreads - 1) / kThreads);
  const dim3 grid((unsigned)rows);
#define PT_CE(N) ce_kernel<N><<<grid, kThreads, 0, stream>>>(L, logits_stride, targets, D, dlogits_stride, row_loss, (int)vocab, scale, inv_count, ignore_index, status)
  if (nc <= 4) PT_CE(4);
  else if (nc <= 8) PT_CE(8);
  else if (nc <= 16) PT_CE(16);
  else if (nc <= 24) PT_CE(24);
  else if (nc <= 32) PT_CE(32);
  else ce_kernel_2pass<<<grid, kThreads, 0, stream>>>(L, logits_stride, targets, D, dlogits_stride, row_loss,
                                                      (int)vocab, scale, inv_count, ignore_index, status);
#undef PT_CE
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// Forward (per-row loss + LSE) from the lm_head GEMM's statistics (pt_gemm_ce_stats): float2
// stats[b * rows + row] = (max, sum exp(x - max)) of the row's logits in column tile b < nblk.
extern "C" int pt_cross_entropy_fwd_stats(const void* logits, int64_t logits_stride, const int64_t* targets,
                                          const float* stats, int64_t nblk, float* row_loss, float* row_lse,
                                          int64_t rows, int64_t vocab, int64_t ignore_index, int* status,
                                          hipStream_t stream) {
  if (!logits || !targets || !stats || !row_loss || !row_lse || rows <= 0 || vocab <= 0 || nblk <= 0) return PT_EINVAL;
  if (vocab % nblk || !pt_aligned16(stats)) return PT_EINVAL;
  const unsigned grid = (unsigned)((rows + kStatRows - 1) / kStatRows);
  ce_fwd_stats_kernel<<<grid, kStatRows * kStatGroups, 0, stream>>>((const uint16_t*)logits, logits_stride, targets,
                                                                  (const float2*)stats, (int)nblk, row_loss, row_lse,
                                                                  rows, (int)vocab, ignore_index, status);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// loss = mean of row_loss over the rows whose target is not ignore_index; inv_count = 1 / #valid
// (reduce_sum: loss = the sum, inv_count = 1 -- F.cross_entropy's reduction='sum');
// out (optional) = loss in bf16 (out_bf16) or f32.  One launch, deterministic.
extern "C" int pt_cross_entropy_mean(const float* row_loss, const int64_t* targets, int64_t rows, int64_t ignore_index,
                                     float* loss_f32, float* inv_count, void* out, int out_bf16, int reduce_sum,
                                     hipStream_t stream) {
  if (!row_loss || !targets || !inv_count || rows <= 0) return PT_EINVAL;
  ce_mean_kernel<<<1, kMeanThreads, 0, stream>>>(row_loss, targets, rows, ignore_index, loss_f32, inv_count, out,
                                                 out_bf16, reduce_sum);
  PT_CHECK_LAUNCH();
  return PT_OK;
}
