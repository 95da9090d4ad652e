// Probe ds_read_b64_tr_b16 semantics in several address patterns.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef short short4_t __attribute__((ext_vector_type(4)));
// mode 0: lane 16g+4q+p -> &img[4g+q][4p]         (probe of the guide's description)
// mode 1: lane 16g+4q+p -> &img[8g+q][4p]
// mode 2: lane 16g+4q+p -> &img[q][16g+4p]
// mode 3: same as 0 but image filled by global_load_lds
__global__ void k(const uint16_t* src, int* out, int mode) {
  __shared__ __attribute__((aligned(16))) uint16_t img[64 * 64];
  if (mode == 3) {
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds(src + i * 512 + threadIdx.x * 8,
                                       (__attribute__((address_space(3))) void*)(img + i * 512), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int i = threadIdx.x; i < 64 * 64; i += 64) img[i] = (uint16_t)((i / 64) * 256 + (i % 64));
  }
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  int off;
  if (mode == 0 || mode == 3) off = (4 * g + q) * 64 + 4 * p;
  else if (mode == 1) off = (8 * g + q) * 64 + 4 * p;
  else off = q * 64 + 16 * g + 4 * p;
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(img + off));
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = (uint16_t)v[j];
}
extern "C" int probe(const uint16_t* src, int* out, int mode) {
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, src, out, mode);
  return (int)hipDeviceSynchronize();
}
