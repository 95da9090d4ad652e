// Micro-benchmark: f32 global atomic-add throughput for a dQ accumulated by the dK/dV workgroups of
// a fused attention backward (d64, causal, B 4 x H 32 x S 1024: 9216 (key block, q tile) pairs, each
// adding a 64 x 64 f32 tile), against plain stores of the same tiles.
//
//   hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics tools/atomic_probe.hip -o tools/ab/atomic_probe
//   ./tools/ab/atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int B = 4, H = 32, S = 1024, D = 64, QT = 64, KB = 128;

struct Pair { int bh, qt; };

template <int MODE>  // 0 store, 1 atomic add (no return)
__global__ __launch_bounds__(256) void probe(const Pair* pairs, float* dq) {
  const Pair p = pairs[blockIdx.x];
  float* base = dq + ((int64_t)p.bh * S + p.qt * QT) * D;
  const float v = 1.0f + threadIdx.x * 1e-3f;
#pragma unroll
  for (int i = 0; i < QT * D / 256; ++i) {
    float* a = base + i * 256 + threadIdx.x;
    if (MODE == 0) *a = v;
    else unsafeAtomicAdd(a, v);
  }
}

template <int MODE>  // float4 vector form: 4 consecutive floats per lane
__global__ __launch_bounds__(256) void probe4(const Pair* pairs, float* dq) {
  const Pair p = pairs[blockIdx.x];
  float* base = dq + ((int64_t)p.bh * S + p.qt * QT) * D;
  const float v = 1.0f + threadIdx.x * 1e-3f;
#pragma unroll
  for (int i = 0; i < QT * D / 1024; ++i) {
    float* a = base + i * 1024 + threadIdx.x * 4;
    if (MODE == 0) {
      *(float4*)a = make_float4(v, v, v, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) unsafeAtomicAdd(a + j, v);
    }
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  // the pairs a causal dK/dV launch would visit, in its XCD-grouped order: per (b, h) each key block
  // kb of 128 keys meets the q tiles 2 kb .. S / 64 - 1
  std::vector<Pair> pairs;
  for (int bh = 0; bh < B * H; ++bh)
    for (int kb = 0; kb < S / KB; ++kb)
      for (int qt = kb * KB / QT; qt < S / QT; ++qt) pairs.push_back({bh, qt});
  const int n = (int)pairs.size();
  Pair* dp;
  float* dq;
  CK(hipMalloc(&dp, n * sizeof(Pair)));
  CK(hipMalloc(&dq, (size_t)B * H * S * D * 4));
  CK(hipMemcpy(dp, pairs.data(), n * sizeof(Pair), hipMemcpyHostToDevice));
  CK(hipMemset(dq, 0, (size_t)B * H * S * D * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)n * QT * D * 4;
  auto run = [&](const char* name, auto kern) {
    for (int w = 0; w < 3; ++w) kern<<<n, 256>>>(dp, dq);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      kern<<<n, 256>>>(dp, dq);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-22s pairs %d  %.2f MB  %.1f us  %.2f TB/s\n", name, n, bytes / 1e6, best * 1e3, bytes / (best * 1e-3) / 1e12);
    return 0;
  };
  run("store f32", probe<0>);
  run("atomic f32", probe<1>);
  run("store f32x4", probe4<0>);
  run("atomic f32 (x4/lane)", probe4<1>);
  return 0;
}
