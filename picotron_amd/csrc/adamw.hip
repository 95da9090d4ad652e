// Fused AdamW step for gfx950: one pass over (param, grad, exp_avg, exp_avg_sq) per tensor.
//
// Replaces (reference, /root/reference): picotron/train.py:205-209 -- `torch.optim.AdamW(
// model.parameters(), lr=learning_rate)` (the reference's own fused switch at :205-207 is dead
// code), i.e. torch's multi-tensor Adam with decoupled weight decay, which on bf16 tensors runs
// eight foreach passes, each computing in f32 and rounding its result to the tensor dtype:
//   p  = r(p * decay)                       _foreach_mul_      decay = 1 - lr * wd
//   m  = r(m + w1 * (g - m))                _foreach_lerp_     w1 = 1 - beta1 (|w| < .5 form)
//   v  = r(v * beta2)                       _foreach_mul_
//   v  = r(v + c2 * (g * g))                _foreach_addcmul_  c2 = 1 - beta2
//   s  = r(sqrt(v)); s = r(s / bc2s); s = r(s + eps)   _foreach_sqrt / div_ / add_
//   p  = r(p + step * (m / s))              _foreach_addcdiv_  step = -lr / (1 - beta1^t)
// r() = round to the storage dtype.  This kernel performs exactly that sequence per element, with
// the roundings, so its result matches torch's bit for bit up to f32 contraction differences --
// but reads each of the four tensors once and writes three (14 bytes per bf16 parameter instead
// of ~44 over the eight passes).  Scalars arrive as f32, as torch's foreach kernels cast them.
#include "common.h"

namespace {

struct AdamScalars {
  float decay, w1, beta2, c2, bc2s, eps, step;
};

template <typename T>
__device__ __forceinline__ float ld_as_f(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld_as_f<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float ld_as_f<float>(const float* p, int64_t i) { return p[i]; }

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamScalars& s, bool bf) {
  auto r = [bf](float x) { return bf ? round_bf(x) : x; };
  p = r(p * s.decay);
  m = r(m + s.w1 * (g - m));
  v = r(v * s.beta2);
  v = r(v + s.c2 * (g * g));
  float d = r(sqrtf(v));
  d = r(d / s.bc2s);
  d = r(d + s.eps);
  p = r(p + s.step * (m / d));
}

// bf16 tensors: 8 elements per thread (16-byte loads / stores on all four streams)
__global__ __launch_bounds__(256) void adamw_bf16_kernel(uint16_t* __restrict__ param, const uint16_t* __restrict__ grad,
                                                         uint16_t* __restrict__ m, uint16_t* __restrict__ v,
                                                         int64_t n8, AdamScalars s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float p[8], g[8], a[8], b[8];
    unpack8(ld8(param + i * 8), p);
    unpack8(ld8(grad + i * 8), g);
    unpack8(ld8(m + i * 8), a);
    unpack8(ld8(v + i * 8), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) adam_elem(p[j], g[j], a[j], b[j], s, true);
    st8(param + i * 8, pack8(p));
    st8(m + i * 8, pack8(a));
    st8(v + i * 8, pack8(b));
  }
}

// scalar tail (n % 8) of a bf16 tensor, and f32 tensors
template <typename T>
__global__ __launch_bounds__(256) void adamw_scalar_kernel(T* __restrict__ param, const T* __restrict__ grad,
                                                           T* __restrict__ m, T* __restrict__ v, int64_t n,
                                                           AdamScalars s) {
  constexpr bool bf = sizeof(T) == 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float p = ld_as_f(param, i), g = ld_as_f(grad, i), a = ld_as_f(m, i), b = ld_as_f(v, i);
    adam_elem(p, g, a, b, s, bf);
    if (bf) {
      ((uint16_t*)param)[i] = f2bf(p);
      ((uint16_t*)m)[i] = f2bf(a);
      ((uint16_t*)v)[i] = f2bf(b);
    } else {
      ((float*)param)[i] = p;
      ((float*)m)[i] = a;
      ((float*)v)[i] = b;
    }
  }
}

// Multi-tensor form: ONE launch per step over every bf16 parameter (torch's foreach AdamW works on
// the whole list too).  The tensors are a virtual concatenation of 8-element chunks; workgroup b
// owns a contiguous run of chunks, finds the tensor its run starts in by binary search over the
// chunk prefix sums (read from the caller's descriptor table), then walks forward.  A tensor whose
// length is not a multiple of 8 finishes its last chunk element by element.
struct AdamTensor {   // pt_adam_tensor (include/picotron_hip.h)
  uint16_t* p;
  const uint16_t* g;
  uint16_t* m;
  uint16_t* v;
  int64_t n;
};

__global__ __launch_bounds__(256) void adamw_multi_bf16_kernel(const AdamTensor* __restrict__ ts,
                                                               const int64_t* __restrict__ chunk_start, int nt,
                                                               int64_t per_block, AdamScalars s) {
  const int64_t total = chunk_start[nt];
  const int64_t lo = (int64_t)blockIdx.x * per_block;
  const int64_t hi = lo + per_block < total ? lo + per_block : total;
  if (lo >= hi) return;
  // the tensor holding chunk lo: largest t with chunk_start[t] <= lo
  int a = 0, b = nt - 1;
  while (a < b) {
    const int mid = (a + b + 1) >> 1;
    if (chunk_start[mid] <= lo) a = mid; else b = mid - 1;
  }
  for (int t = a; t < nt && chunk_start[t] < hi; ++t) {
    const AdamTensor T = ts[t];
    const int64_t c0 = chunk_start[t], c1 = chunk_start[t + 1];
    const int64_t from = (lo > c0 ? lo : c0) - c0, to = (hi < c1 ? hi : c1) - c0;   // chunk range in t
    const int64_t full = T.n >> 3;
    const int64_t end = to < full ? to : full;   // this run's full chunks in tensor t
    // software-pipelined: the loads of a thread's next two chunks are issued before the current
    // chunk's stores, so every wait for a load sits behind loads only -- vmcnt counts stores too,
    // and loads issued after the previous chunk's stores waited out their write latency (5.0 TB/s)
    int64_t c = from + threadIdx.x;
    const int64_t bd = blockDim.x;
    bf16x8 cur[4], nx1[4], nx2[4];
    auto load4 = [&](int64_t cc, bf16x8 (&r)[4]) {
      r[0] = ld8_nt(T.p + cc * 8); r[1] = ld8_nt(T.g + cc * 8); r[2] = ld8_nt(T.m + cc * 8);
      r[3] = ld8_nt(T.v + cc * 8);
    };
    if (c < end) load4(c, cur);
    if (c + bd < end) load4(c + bd, nx1);
    for (; c < end; c += bd) {
      if (c + 2 * bd < end) load4(c + 2 * bd, nx2);
      float p[8], g[8], m[8], v[8];
      unpack8(cur[0], p); unpack8(cur[1], g); unpack8(cur[2], m); unpack8(cur[3], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) adam_elem(p[j], g[j], m[j], v[j], s, true);
      st8_nt(T.p + c * 8, pack8(p));
      st8_nt(T.m + c * 8, pack8(m));
      st8_nt(T.v + c * 8, pack8(v));
#pragma unroll
      for (int q = 0; q < 4; ++q) { cur[q] = nx1[q]; nx1[q] = nx2[q]; }
    }
    for (; c < to; c += blockDim.x) {
      if (c < full) {
        float p[8], g[8], m[8], v[8];
        unpack8(ld8(T.p + c * 8), p);
        unpack8(ld8(T.g + c * 8), g);
        unpack8(ld8(T.m + c * 8), m);
        unpack8(ld8(T.v + c * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) adam_elem(p[j], g[j], m[j], v[j], s, true);
        st8(T.p + c * 8, pack8(p));
        st8(T.m + c * 8, pack8(m));
        st8(T.v + c * 8, pack8(v));
      } else {   // the ragged last chunk
        for (int64_t i = c * 8; i < T.n; ++i) {
          float p = bf2f(T.p[i]), g = bf2f(T.g[i]), m = bf2f(T.m[i]), v = bf2f(T.v[i]);
          adam_elem(p, g, m, v, s, true);
          T.p[i] = f2bf(p);
          T.m[i] = f2bf(m);
          T.v[i] = f2bf(v);
        }
      }
    }
  }
}

int grid_for(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (int)(g < PT_STREAM_GRID_CAP ? (g < 1 ? 1 : g) : PT_STREAM_GRID_CAP);
}

}  // namespace

extern "C" {

int pt_adamw_step(void* param, const void* grad, void* exp_avg, void* exp_avg_sq, int64_t n, int dtype,
                  float decay, float w1, float beta2, float c2, float bc2_sqrt, float eps, float step_size,
                  hipStream_t stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || n < 0) return PT_EINVAL;
  if (n == 0) return PT_OK;
  const AdamScalars s{decay, w1, beta2, c2, bc2_sqrt, eps, step_size};
  if (dtype == 0) {  // bf16
    auto* P = (uint16_t*)param;
    auto* G = (const uint16_t*)grad;
    auto* M = (uint16_t*)exp_avg;
    auto* V = (uint16_t*)exp_avg_sq;
    const bool vec = pt_aligned16(P) && pt_aligned16(G) && pt_aligned16(M) && pt_aligned16(V);
    const int64_t n8 = vec ? n / 8 : 0;
    if (n8) {
      adamw_bf16_kernel<<<grid_for(n8), 256, 0, stream>>>(P, G, M, V, n8, s);
      PT_CHECK_LAUNCH();
    }
    const int64_t done = n8 * 8;
    if (done < n) {
      adamw_scalar_kernel<uint16_t><<<grid_for(n - done), 256, 0, stream>>>(P + done, G + done, M + done, V + done,
                                                                             n - done, s);
      PT_CHECK_LAUNCH();
    }
  } else if (dtype == 1) {  // f32
    adamw_scalar_kernel<float><<<grid_for(n), 256, 0, stream>>>((float*)param, (const float*)grad, (float*)exp_avg,
                                                                (float*)exp_avg_sq, n, s);
    PT_CHECK_LAUNCH();
  } else {
    return PT_EINVAL;
  }
  return PT_OK;
}

// bf16 tensors (every pointer 16-byte aligned), one launch.  tensors: device array of ntensors
// pt_adam_tensor; chunk_start: device int64 [ntensors + 1], chunk_start[i] = sum over j < i of
// ceil(n_j / 8) -- both built (and cached) by the caller.  total_chunks = chunk_start[ntensors].
int pt_adamw_step_multi(const void* tensors, const int64_t* chunk_start, int ntensors, int64_t total_chunks,
                        float decay, float w1, float beta2, float c2, float bc2_sqrt, float eps, float step_size,
                        hipStream_t stream) {
  if (!tensors || !chunk_start || ntensors <= 0 || total_chunks < 0) return PT_EINVAL;
  if (total_chunks == 0) return PT_OK;
  const AdamScalars s{decay, w1, beta2, c2, bc2_sqrt, eps, step_size};
  // one resident round: 4 blocks of 4 waves per CU at <= 128 VGPRs (2 chunks per thread in flight)
  const int64_t cap = 1024, want = (total_chunks + 511) / 512;
  const int64_t blocks = want < 1 ? 1 : (want < cap ? want : cap);
  const int64_t per_block = (total_chunks + blocks - 1) / blocks;
  adamw_multi_bf16_kernel<<<(unsigned)blocks, 256, 0, stream>>>((const AdamTensor*)tensors, chunk_start, ntensors,
                                                                per_block, s);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

}  // extern "C"
