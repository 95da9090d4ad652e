// Rotary position embedding (NeoX "rotate-half", non-interleaved) forward / backward.
//
// Replaces (reference, /root/reference):
//   * picotron/model.py:136-137  flash-attn apply_rotary_emb(x, cos[:, :d/2], sin[:, :d/2], interleaved=False)
//   * picotron/model.py:12-19    apply_rotary_pos_emb (eager path): x*cos + rotate_half(x)*sin
//   cos/sin tables come from get_cos_sin (model.py:21-31): [S, d] bf16 with the two halves equal,
//   sliced per CP rank by update_rope_for_context_parallel (context_parallel.py:189-195).
//
//   fwd:  o1 = x1*c - x2*s,   o2 = x2*c + x1*s      (f32 math, one bf16 rounding)
//   bwd:  rotation by -theta: d1 = g1*c + g2*s,  d2 = g2*c - g1*s
//
// Layout: token-major rows ([B*S, row_stride] bf16, the natural output of the fused
// QKV projection).  The first `nheads` heads of every row are rotated in place; with the
// fused [q | k | v] row that is q and k together in one launch.  Row r has position
// r % seq_len.  One thread = 8 rotation pairs (two 16-byte loads + two 16-byte stores).
// HBM-bound: 4 bytes read + 4 written per rotated bf16 pair-half... i.e. 4*T*nheads*d bytes.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void rope_kernel(uint16_t* __restrict__ x, int64_t rows, int64_t row_stride,
                                                   int nheads, int head_dim, const uint16_t* __restrict__ cos_t,
                                                   const uint16_t* __restrict__ sin_t, int seq_len, int tab_stride,
                                                   float sign) {
  const int half = head_dim >> 1;
  const int cph = half >> 3;  // 8-wide chunks per half head
  const int64_t per_row = (int64_t)nheads * cph;
  const int64_t total = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / per_row;
    const int rem = (int)(i - row * per_row);
    const int head = rem / cph;
    const int ch = rem - head * cph;
    const int pos = (int)(row % seq_len);
    uint16_t* p1 = x + row * row_stride + (int64_t)head * head_dim + ch * 8;
    uint16_t* p2 = p1 + half;
    float a[8], b[8], c[8], s[8], o1[8], o2[8];
    unpack8(ld8(p1), a);
    unpack8(ld8(p2), b);
    unpack8(ld8(cos_t + (int64_t)pos * tab_stride + ch * 8), c);
    unpack8(ld8(sin_t + (int64_t)pos * tab_stride + ch * 8), s);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sj = sign * s[j];
      o1[j] = fmaf(a[j], c[j], -(b[j] * sj));  // explicit contraction: the GEMM / attention
      o2[j] = fmaf(b[j], c[j], a[j] * sj);     // epilogues that fuse RoPE round identically
    }
    st8(p1, pack8(o1));
    st8(p2, pack8(o2));
  }
}

}  // namespace

extern "C" int pt_rope(void* x, int64_t rows, int64_t row_stride, int64_t nheads, int64_t head_dim,
                       const void* cos_table, const void* sin_table, int64_t seq_len, int64_t table_stride,
                       int inverse, hipStream_t stream) {
  if (!x || !cos_table || !sin_table || rows <= 0 || nheads <= 0 || seq_len <= 0) return PT_EINVAL;
  if (head_dim % 16 != 0 || row_stride % 8 != 0 || table_stride % 8 != 0) return PT_EALIGN;
  if (!pt_aligned16(x) || !pt_aligned16(cos_table) || !pt_aligned16(sin_table)) return PT_EALIGN;
  const int64_t total = rows * nheads * (head_dim / 16);
  int64_t g = (total + 255) / 256;
  if (g > PT_STREAM_GRID_CAP * 2) g = PT_STREAM_GRID_CAP * 2;
  rope_kernel<<<(int)g, 256, 0, stream>>>((uint16_t*)x, rows, row_stride, (int)nheads, (int)head_dim,
                                          (const uint16_t*)cos_table, (const uint16_t*)sin_table, (int)seq_len,
                                          (int)table_stride, inverse ? -1.0f : 1.0f);
  PT_CHECK_LAUNCH();
  return PT_OK;
}
