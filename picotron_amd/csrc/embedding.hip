// Token embedding lookup and its backward for gfx950 (bf16 table).
//
// Replaces (reference, /root/reference):
//   * picotron/model.py:224-225  Embedding -> F.embedding(ids, W)   (and autograd's dense backward)
//   * picotron/tensor_parallel/tensor_parallel.py:246-270  VocabParallelEmbedding.forward: the
//     masked lookup into this rank's vocab slice [vocab_lo, vocab_hi) (rows of other ranks' tokens
//     are zero and, in the backward, contribute nothing)
//
// fwd:  out[t, :] = W[ids[t] - vocab_lo, :]  (0 when ids[t] is outside the slice)
// bwd:  for every vocab row r touched by the micro-batch: dW[r] (op)= bf16(sum_{t: ids[t] = r} dY[t])
//       the sum in f32 over the tokens in ascending position order (ids sorted stably on the host),
//       rounded to bf16 once -- torch's embedding_dense_backward -- then applied to the gradient
//       sink: bf16 store / bf16 accumulate (autograd's grad + new) / f32 accumulate (main_grad).
//       Rows no token touches are not read or written (the reference materialises a dense
//       [V, H] gradient and adds all of it: 600 MB of traffic per micro-batch at V 49152).
// fwd: one thread per 16-B chunk; bwd: one wave per touched row.  H % 8 == 0.  HBM-bound.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void embedding_fwd_kernel(const int64_t* __restrict__ ids, int64_t T,
                                                            const uint16_t* __restrict__ w, int64_t ldw,
                                                            int64_t lo, int64_t hi, uint16_t* __restrict__ out,
                                                            int64_t ldo, int H) {
  const int cpr = H >> 3;
  const int64_t total = T * cpr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / cpr;
    const int c = (int)(i - t * cpr) * 8;
    const int64_t id = ids[t];
    bf16x8 v;
    if (id >= lo && id < hi) {
      v = ld8(w + (id - lo) * ldw + c);
    } else {
      v.w[0] = v.w[1] = v.w[2] = v.w[3] = 0u;
    }
    st8(out + t * ldo + c, v);
  }
}

// sorted_ids[i] (ascending; -1 = skip), perm[i] = the token position of sorted entry i.  A wave
// owns the segment that starts at sorted entry i (i == 0 or a new id) and walks it.
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ perm, int64_t T,
                                                            const uint16_t* __restrict__ dy, int64_t ldy,
                                                            int64_t lo, void* __restrict__ dw, int64_t lddw,
                                                            int H, int sink) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < T; i += nw) {
    const int64_t id = sorted_ids[i];
    if (id < 0 || (i > 0 && sorted_ids[i - 1] == id)) continue;  // not a segment start
    int64_t end = i + 1;
    while (end < T && sorted_ids[end] == id) ++end;
    const int64_t row = id - lo;
    for (int c = lane * 8; c < H; c += 64 * 8) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int64_t j = i; j < end; ++j) {
        float x[8];
        unpack8(ld8(dy + perm[j] * ldy + c), x);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += x[e];
      }
      if (sink == PT_DW_ACC_F32) {
        float* d = (float*)dw + row * lddw + c;
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] += round_bf(acc[e]);
      } else {
        uint16_t* d = (uint16_t*)dw + row * lddw + c;
        if (sink == PT_DW_ACC_BF16) {
          float o[8];
          unpack8(ld8(d), o);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] = o[e] + round_bf(acc[e]);
        }
        st8(d, pack8(acc));
      }
    }
  }
}

// The backward's key preparation + stable sort in ONE single-workgroup launch (T <= 16384): key =
// 0 for a skipped token (outside [lo, hi) or padding_idx), id - lo + 1 otherwise, carried with its
// position as (key << 32 | position).  LSD radix sort, 4 key bits per pass (passes = bit length of
// hi - lo, rounded up to 4): each pass is a stable 16-way split, an element's destination = the
// elements of smaller digits + those of its digit in earlier (round, wave) slots + those before it in
// its wave (4 ballots of the digit bits give each digit's lane mask), one block-wide exclusive scan
// over the (digit, round, wave) counts, scattered through LDS.  Stable by construction, so equal ids
// keep ascending positions (== torch.sort(stable=True) of the keyed ids; the backward's fixed
// summation order).  Element i = r * 1024 + tid lives in thread tid's register r.  Writes sorted_ids
// (-1 = skip, first) and perm as int64.  (One bit per pass: 16 passes, 35 us at T 4096.)
constexpr int kSortThreads = 1024, kSortMax = 16384, kSortRounds = kSortMax / kSortThreads, kSortDigits = 16;
__global__ __launch_bounds__(kSortThreads) void embedding_sort_kernel(const int64_t* __restrict__ ids, int T,
                                                                      int rounds, int bits, int64_t lo, int64_t hi,
                                                                      int has_pad, int64_t pad,
                                                                      int64_t* __restrict__ sorted_ids,
                                                                      int64_t* __restrict__ perm) {
  extern __shared__ uint64_t buf[];                          // [rounds * 1024]
  __shared__ int cnt[kSortDigits * kSortRounds * 16];        // (digit, round, wave) counts -> offsets
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt_mask = (1ull << lane) - 1;
  uint64_t c[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = r * kSortThreads + tid;
    c[r] = ~0ull;  // padding: all key bits set -> sorts last
    if (r < rounds && i < T) {
      const int64_t id = ids[i];
      const bool skip = id < lo || id >= hi || (has_pad && id == pad);
      c[r] = ((uint64_t)(skip ? 0 : (uint32_t)(id - lo + 1)) << 32) | (uint32_t)i;
    }
  }
  const int n = kSortDigits * rounds * 16;   // scan entries, (digit, round, wave) order
  for (int shift = 0; shift < bits; shift += 4) {
    int rk[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      if (r < rounds) {
        const int dg = (int)(c[r] >> (32 + shift)) & 15;
        const uint64_t b0 = __ballot(dg & 1), b1 = __ballot(dg & 2), b2 = __ballot(dg & 4), b3 = __ballot(dg & 8);
        // the lanes holding digit d: per lane, from the four bit masks (own digit: rank; lane < 16:
        // that digit's count in the wave)
        auto lanes_of = [&](int d) {
          return ((d & 1) ? b0 : ~b0) & ((d & 2) ? b1 : ~b1) & ((d & 4) ? b2 : ~b2) & ((d & 8) ? b3 : ~b3);
        };
        rk[r] = __popcll(lanes_of(dg) & lt_mask);
        if (lane < kSortDigits) cnt[(lane * rounds + r) * 16 + wave] = __popcll(lanes_of(lane));
      }
    }
    __syncthreads();
    {  // block-wide exclusive scan of cnt[0, n): 4 consecutive entries per thread
      int v4[4], run = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid * 4 + k;
        v4[k] = e < n ? cnt[e] : 0;
        run += v4[k];
      }
      int x = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) wsum[wave] = x;
      __syncthreads();
      int before = 0;
      for (int w = 0; w < wave; ++w) before += wsum[w];
      int acc = before + x - run;   // exclusive prefix of this thread's first entry
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid * 4 + k;
        if (e < n) cnt[e] = acc;
        acc += v4[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      if (r < rounds) {
        const int dg = (int)(c[r] >> (32 + shift)) & 15;
        buf[cnt[(dg * rounds + r) * 16 + wave] + rk[r]] = c[r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r)
      if (r < rounds) c[r] = buf[r * kSortThreads + tid];
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = r * kSortThreads + tid;
    if (r < rounds && i < T) {
      const uint32_t key = (uint32_t)(c[r] >> 32);
      sorted_ids[i] = key == 0 ? -1 : (int64_t)key - 1 + lo;
      perm[i] = (int64_t)(uint32_t)c[r];
    }
  }
}

int grid_for(int64_t work, int per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < 4 * PT_STREAM_GRID_CAP ? g : 4 * PT_STREAM_GRID_CAP);
}

}  // namespace

extern "C" {

int pt_embedding_fwd(const int64_t* ids, int64_t T, const void* weight, int64_t ldw, int64_t vocab_lo, int64_t vocab_hi,
                     void* out, int64_t ldo, int64_t H, hipStream_t stream) {
  if (!ids || !weight || !out || T < 0 || H <= 0 || vocab_hi < vocab_lo) return PT_EINVAL;
  if ((H & 7) || (ldw & 7) || (ldo & 7) || !pt_aligned16(weight) || !pt_aligned16(out)) return PT_EALIGN;
  if (T == 0) return PT_OK;
  embedding_fwd_kernel<<<grid_for(T * (H / 8), 256), 256, 0, stream>>>(ids, T, (const uint16_t*)weight, ldw, vocab_lo,
                                                                       vocab_hi, (uint16_t*)out, ldo, (int)H);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

int pt_embedding_bwd(const int64_t* sorted_ids, const int64_t* perm, int64_t T, const void* dy, int64_t ldy,
                     int64_t vocab_lo, void* dweight, int64_t lddw, int64_t H, int sink, hipStream_t stream) {
  if (!sorted_ids || !perm || !dy || !dweight || T < 0 || H <= 0) return PT_EINVAL;
  if (sink != 0 && sink != PT_DW_ACC_BF16 && sink != PT_DW_ACC_F32) return PT_EINVAL;
  if ((H & 7) || (ldy & 7) || (lddw & 7) || !pt_aligned16(dy) || !pt_aligned16(dweight)) return PT_EALIGN;
  if (T == 0) return PT_OK;
  embedding_bwd_kernel<<<grid_for(T, 4), 256, 0, stream>>>(sorted_ids, perm, T, (const uint16_t*)dy, ldy, vocab_lo,
                                                           dweight, lddw, (int)H, sink);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// Key preparation + stable sort of the backward's token ids (embedding_sort_kernel): T <= 16384
// (PT_EUNSUPPORTED above; the caller sorts otherwise).  has_padding / padding_idx: F.embedding's.
int pt_embedding_sort(const int64_t* ids, int64_t T, int64_t vocab_lo, int64_t vocab_hi, int has_padding,
                      int64_t padding_idx, int64_t* sorted_ids, int64_t* perm, hipStream_t stream) {
  if (!ids || !sorted_ids || !perm || T < 0 || vocab_hi < vocab_lo || vocab_hi - vocab_lo >= (1ll << 31) - 1)
    return PT_EINVAL;
  if (T > kSortMax) return PT_EUNSUPPORTED;
  if (T == 0) return PT_OK;
  const int rounds = (int)((T + kSortThreads - 1) / kSortThreads);
  int bits = 1;
  while (bits < 31 && ((vocab_hi - vocab_lo) >> bits) != 0) ++bits;  // keys <= hi - lo
  const int smem = rounds * kSortThreads * (int)sizeof(uint64_t);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)embedding_sort_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kSortMax * (int)sizeof(uint64_t));
    attr = true;
  }
  embedding_sort_kernel<<<1, kSortThreads, smem, stream>>>(ids, (int)T, rounds, bits, vocab_lo, vocab_hi,
                                                           has_padding, padding_idx, sorted_ids, perm);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

}  // extern "C"
