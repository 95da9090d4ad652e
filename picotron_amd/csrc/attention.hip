// Flash attention forward / backward for gfx950 (MFMA 32x32x16 bf16, f32 softmax), with the
// ring-attention LSE merge fused into the forward epilogue.
//
// Replaces (reference, /root/reference):
//   * picotron/model.py:33-37,154   flash_attention -> flash_attn_func(q, k, v, causal=True)  (fwd + FA2 bwd)
//   * picotron/model.py:157         F.scaled_dot_product_attention(q, k, v, is_causal=True)   (FLASH_ATTEN=0)
//   * picotron/context_parallel/context_parallel.py:112-128  ring_attention_forward (block attention + LSE)
//   * context_parallel.py:130-155   ring_attention_backward (block bwd from the global out/LSE)
//   * context_parallel.py:157-187   update_out_and_lse (fused: merge=1 epilogue)
//   * model.py:142-143              repeat_interleave for GQA (elided: kv head = q head / group)
//
// Layout: q/k/v/o are token-major [B, S, H, D] strided views (d contiguous), e.g. slices of the
// fused [T, (h + 2*hkv) * D] projection output -- no transposes, no copies.  lse is f32 [B, H, Sq]
// with rows lse_ld apart (a slice of a longer sequence's LSE: the zig-zag ring's half blocks).
// mask: 0 = full, 1 = causal (key j visible to query i iff j <= i; Sq == Sk).
//
// Fragment scheme (all v_mfma_f32_32x32x16_bf16): scores are computed "key on the row",
// S^T = K . Q^T, so a lane owns one query column and softmax statistics are lane-local (plus one
// lane^32 exchange).  The S^T / dS^T accumulators are re-used directly as the B operand of the
// next product (O^T += V^T P^T, dQ^T += K^T dS^T); the matching A operands come from
// ds_read_b64_tr_b16 transposed reads of the row-major K/V tiles.  The dK/dV kernel uses the
// mirror scheme (S = Q . K^T, key on the lane) so dV^T += dO^T P and dK^T += Q^T dS take their
// B operands from accumulators as well.  One LDS image per tile serves both the row reads and
// the transposed reads (XOR swizzle from tools/lds_swizzle_search.py, conflict-free for both).
// K/V (fwd, dq) and Q/dO (dkdv) tiles arrive by global_load_lds_dwordx4 into a 2-deep ring.
#include "common.h"

#include <stdlib.h>

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));   // v_pk_fma_f32 / v_pk_add_f32 operands
typedef __attribute__((address_space(3))) uint8_t lds_u8;

// the d64 forward: a batch of LDS operand reads stays ahead of the MFMAs that consume it (no
// scheduling across; 34.3 vs 34.9 us at the SmolLM layer shape; at d128 and in the backward kernels
// the compiler's own interleave measured equal or faster).
#define PT_BATCH_BARRIER(D) do { if constexpr ((D) == 64) __builtin_amdgcn_sched_barrier(0); } while (0)

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleLog2 = 8.0f;
constexpr int KT = 64;  // rows per staged K/V (or Q/dO) tile
constexpr int NW = 4;   // waves per workgroup, 32 rows each

struct AttnArgs {
  const uint16_t* q; int64_t q_sb, q_ss, q_sh;
  const uint16_t* k; int64_t k_sb, k_ss, k_sh;
  const uint16_t* v; int64_t v_sb, v_ss, v_sh;
  void* o; int64_t o_sb, o_ss, o_sh;            // bf16 output, or f32 accumulator when merge
  float* lse;                                    // [B, H, Sq] rows lse_ld apart
  const uint16_t* dout; int64_t do_sb, do_ss, do_sh;
  const float* delta;                            // [B, H, Sq] rowsum(dO * O), rows lse_ld apart
  int64_t lse_ld;   // elements between consecutive (b, h) rows of lse / delta (Sq when dense)
  void* dq; int64_t dq_sb, dq_ss, dq_sh;
  void* dk; int64_t dk_sb, dk_ss, dk_sh;
  void* dv; int64_t dv_sb, dv_ss, dv_sh;
  int B, H, HKV, Sq, Sk;
  float scale;
  int causal;
  int merge;      // fwd: merge into (o f32, lse) accumulators
  int grad_f32;   // bwd: dq/dk/dv are f32 accumulators (+=) instead of bf16 stores
  // bwd: when set, dq and dk are rotated back by -theta (the RoPE backward, model.py:136-137)
  // before their bf16 store, position = the query / key index; tables [Sq, rope_ld] bf16
  const uint16_t* rope_cos;
  const uint16_t* rope_sin;
  int64_t rope_ld;
  // causal load balance: each workgroup runs block x and block (n - 1 - x) one after the other,
  // so every workgroup gets the same number of tiles whatever CU slot it lands in
  int pair;
  // bwd: when set, the dQ kernel (launched first) computes D = rowsum(dO * O) of its own rows from
  // O (a.o, bf16) and writes it here for the dK/dV kernel -- no separate delta pass
  float* delta_w;
  // few-head split forms (pt_attn_split_plan): work items of split_ck K (Q) tiles each, split_per_bh
  // items per (batch, head) row; f32 partials [item][rows of the block][D] (split_o: O / dQ / dK,
  // split_dv: dV) and the forward's per-row LSE [item][rows]
  int split_ck, split_per_bh;
  float* split_o;
  float* split_dv;
  float* split_lse;
};

template <int D>
__device__ __forceinline__ int aswz(int r) {
  if (D == 64) return (((r >> 1) & 1) << 2) | ((r >> 3) & 1) | (((r >> 4) & 1) << 1);
  return ((r & 1) << 2) | (((r >> 1) & 1) << 3) | ((r >> 3) & 1) | (((r >> 4) & 1) << 1);
}

// stage a [KT][D] bf16 tile (rows `row_stride` elements apart) into a swizzled LDS image
template <int D, int NWK = NW>
__device__ __forceinline__ void stage_rows(const uint16_t* __restrict__ g, int64_t row_stride, lds_u8* dst,
                                           int wave, int lane) {
  constexpr int RB = D * 2, RC = RB / 16, RPI = 1024 / RB;  // rows per 1 KiB wave instruction
  constexpr int NI = KT * RB / 1024;
  static_assert(NI % NWK == 0, "tile instructions split evenly over the waves");
#pragma unroll
  for (int it = 0; it < NI / NWK; ++it) {
    const int i = it * NWK + wave;
    const int r = i * RPI + lane / RC, c = lane % RC;
    pt_glds16(g, (uint32_t)((r * row_stride + 8 * (c ^ aswz<D>(r))) * 2),
              (__attribute__((address_space(3))) void*)(dst + i * 1024));
  }
}

// A operand (rows of the tile): lane -> row row0 + (lane & 31), k = 16 ks + 8 (lane >> 5) + j
template <int D>
__device__ __forceinline__ bf16x8_t rd_row(const lds_u8* t, int row0, int ks, int lane) {
  const int r = row0 + (lane & 31), ch = 2 * ks + (lane >> 5);
  return *(const __attribute__((address_space(3))) bf16x8_t*)(t + r * (D * 2) + 16 * (ch ^ aswz<D>(r)));
}

// A operand X^T (sum over tile rows) for 16-row step s and 32-column tile dt:
// element j <-> tile row 16 s + 8 (j >> 2) + 4 (lane >> 5) + (j & 3), column 32 dt + (lane & 31)
template <int D>
__device__ __forceinline__ bf16x8_t rd_tr(const lds_u8* t, int s, int dt, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = 32 * dt + 16 * (g & 1) + 4 * p;
  bf16x4_t v[2];  // whole-vector concat (element-wise bit_cast of short4 miscompiles, see gemm.hip)
#pragma unroll
  for (int sec = 0; sec < 2; ++sec) {
    const int r = 16 * s + 8 * sec + 4 * (g >> 1) + q;
    const int off = r * (D * 2) + 16 * ((col >> 3) ^ aswz<D>(r)) + 8 * ((col >> 2) & 1);
    v[sec] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(t + off));
  }
  return __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7);
}

// B operand from a C-layout 32x32 accumulator, k-step s (rows 16 s .. 16 s + 15)
__device__ __forceinline__ bf16x8_t acc_as_b(const f32x16_t& x, int s) {
  bf16x8_t out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (__bf16)x[8 * s + j];
  return out;
}

// B operand straight from a global row: lane -> row (lane & 31) of `base`, k = 16 ks + 8 (lane >> 5) + j
__device__ __forceinline__ bf16x8_t ld_row_frag(const uint16_t* row_ptr, int ks, int lane) {
  return *(const bf16x8_t*)(row_ptr + 16 * ks + 8 * (lane >> 5));
}

// C layout row index of register r for this lane
__device__ __forceinline__ int crow(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// XCD-aware block order.  The dispatcher deals workgroups round-robin over the 8 XCDs (linear id
// mod 8), which would spread the 8-16 blocks of one (batch, head) -- all re-reading that head's
// K/V (or Q/dO) tiles -- over 8 different L2s.  Remap so each XCD gets a contiguous range of
// (block, head, batch) ids, blocks of one head adjacent: a head's tiles are fetched into one L2
// and re-read from there (a head's K+V at S 1024, d 64 is 256 KiB; an XCD's L2 is 4 MiB).
__device__ __forceinline__ void attn_coords(const AttnArgs& a, int& x, int& y, int& z) {
  const int nx = gridDim.x, ny = gridDim.y, nwg = nx * ny * gridDim.z;
  const int id = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
  const int pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  x = pid % nx;
  y = (pid / nx) % ny;
  z = pid / (nx * ny);
}

__device__ __forceinline__ int nqb_of(const AttnArgs& a) { return a.Sq / (NW * 32); }

// v + (v of lane ^ 32) and max(v, v of lane ^ 32): one v_permlane32_swap (no LDS round trip)
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ f32x16_t zero16() {
  f32x16_t z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ f32x16_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// store a 32(d) x 32(row) C-layout tile transposed into row-major memory: lane owns row
// (lane & 31), d = 32 dt + crow(r); 4 consecutive d per 8-byte store
// Widened (guide T21): the 4-column chunks of lanes l and l ^ 32 sit side by side in the row, so
// for each pair of groups (g4, g4 + 1) one v_permlane32_swap per dword (vdst = the g4 chunk, src =
// the g4 + 1 chunk: lanes 32-63 of vdst trade with lanes 0-31 of src) leaves the lower lanes
// [own g4 | upper's g4] and the upper lanes [lower's g4 + 1 | own g4 + 1]: 8 consecutive columns per
// lane, one 16-byte store instead of two 8-byte ones (the epilogue tail is store-issue-bound).  The
// stored values are those of the 8-byte form.
__device__ __forceinline__ void store_T_bf16(uint16_t* row_ptr, int dt, const f32x16_t& x, float mul, int lane) {
#pragma unroll
  for (int gp = 0; gp < 4; gp += 2) {
    uint32_t a[2], b[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t c0 = pack_bf2(x[4 * gp + 2 * u] * mul, x[4 * gp + 2 * u + 1] * mul);
      const uint32_t c1 = pack_bf2(x[4 * gp + 4 + 2 * u] * mul, x[4 * gp + 4 + 2 * u + 1] * mul);
      const auto r = __builtin_amdgcn_permlane32_swap(c0, c1, false, false);
      a[u] = r[0];
      b[u] = r[1];
    }
    *(uint4*)(row_ptr + 32 * dt + 8 * gp + (lane >= 32 ? 8 : 0)) = make_uint4(a[0], a[1], b[0], b[1]);
  }
}
// store_T_bf16 of all DT tiles of one row with the inverse RoPE rotation applied to the bf16
// values, exactly as csrc/rope.hip's backward (sj = -s; o1 = fma(g1, c, -(g2 sj)), o2 = fma(g2, c, g1 sj))
template <int DT>
__device__ __forceinline__ void store_T_bf16_unrope(uint16_t* row_ptr, const f32x16_t (&x)[DT], float mul,
                                                    const uint16_t* cos_row, const uint16_t* sin_row, int lane) {
  constexpr int HD = DT / 2;  // (d, d + 32 HD) pairs sit in tiles dt and dt + HD
  uint32_t e1[2], e2[2];      // the even group's packed chunks, waiting for the odd one
#pragma unroll
  for (int dt = 0; dt < HD; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = 32 * dt + 8 * g4 + 4 * (lane >> 5);
      const uint2 cw = *(const uint2*)(cos_row + d), sw = *(const uint2*)(sin_row + d);
      const float c[4] = {lo_bf(cw.x), hi_bf(cw.x), lo_bf(cw.y), hi_bf(cw.y)};
      const float sn[4] = {lo_bf(sw.x), hi_bf(sw.x), lo_bf(sw.y), hi_bf(sw.y)};
      float o1[4], o2[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g1 = round_bf(x[dt][4 * g4 + e] * mul), g2 = round_bf(x[dt + HD][4 * g4 + e] * mul);
        const float sj = -sn[e];
        o1[e] = fmaf(g1, c[e], -(g2 * sj));
        o2[e] = fmaf(g2, c[e], g1 * sj);
      }
      uint32_t p1[2] = {pack_bf2(o1[0], o1[1]), pack_bf2(o1[2], o1[3])};
      uint32_t p2[2] = {pack_bf2(o2[0], o2[1]), pack_bf2(o2[2], o2[3])};
      if ((g4 & 1) == 0) {   // hold group g4's chunks; the odd group completes the pair (store_T_bf16)
#pragma unroll
        for (int u = 0; u < 2; ++u) { e1[u] = p1[u]; e2[u] = p2[u]; }
        continue;
      }
      uint32_t a1[2], b1[2], a2[2], b2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const auto r1 = __builtin_amdgcn_permlane32_swap(e1[u], p1[u], false, false);
        const auto r2 = __builtin_amdgcn_permlane32_swap(e2[u], p2[u], false, false);
        a1[u] = r1[0]; b1[u] = r1[1];
        a2[u] = r2[0]; b2[u] = r2[1];
      }
      const int dw = 32 * dt + 8 * (g4 - 1) + (lane >= 32 ? 8 : 0);
      *(uint4*)(row_ptr + dw) = make_uint4(a1[0], a1[1], b1[0], b1[1]);
      *(uint4*)(row_ptr + dw + 32 * HD) = make_uint4(a2[0], a2[1], b2[0], b2[1]);
    }
}

__device__ __forceinline__ void accum_T_f32(float* row_ptr, int dt, const f32x16_t& x, float mul, int lane) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int d = 32 * dt + 8 * g4 + 4 * (lane >> 5);
    float4 o = *(float4*)(row_ptr + d);
    o.x += x[4 * g4 + 0] * mul; o.y += x[4 * g4 + 1] * mul;
    o.z += x[4 * g4 + 2] * mul; o.w += x[4 * g4 + 3] * mul;
    *(float4*)(row_ptr + d) = o;
  }
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else static_assert(N == 0, "vm_wait: add the count");
}

// K/V (Q/dO) staging ring of NS LDS stages: tile t lives in stage t % NS and its LDS-DMA pieces (OPS
// per wave) are issued NS - 1 tiles ahead; before tile t + 1 is read, every piece older than the
// `younger` tiles issued after it must have landed.  Attention workgroups of one XCD walk the same
// K/V tiles in step, so a tile's first touch is an HBM miss they all wait on: with one tile of
// look-ahead that latency was most of the d64 kernels' time (the forward's DMA / barrier skeleton
// alone: 21 of 37 us).
template <int OPS, int NS>
__device__ __forceinline__ void ring_wait(int younger) {
  if constexpr (NS >= 4) {
    if (younger >= 2) { vm_wait<2 * OPS>(); return; }
  }
  if constexpr (NS >= 3) {
    if (younger >= 1) { vm_wait<OPS>(); return; }
  }
  vm_wait<0>();
}

// A wave's tiles [0, nkt) in three loops -- below the causal diagonal (kind 0), on it (1), past it
// (2: only the ring's refill / wait / barrier) -- so no per-tile branch joins two versions of the
// accumulators (such a join cost 16-32 register copies on every tile) and the diagonal mask is
// compiled into its own loop only.
template <typename Step>
__device__ __forceinline__ void tile_loops(int n_nd, int n_c, int nkt, Step&& step) {
  for (int kt = 0; kt < n_nd; ++kt) step(std::integral_constant<int, 0>{}, kt);
  for (int kt = n_nd; kt < n_c; ++kt) step(std::integral_constant<int, 1>{}, kt);
  for (int kt = n_c; kt < nkt; ++kt) step(std::integral_constant<int, 2>{}, kt);
}

// the loop bounds for a wave whose 32 query rows start at q0, over key tiles kt0 .. kt0 + nkt - 1:
// n_c tiles hold a key <= q0 + 31, the first n_nd of them only keys <= q0
__device__ __forceinline__ void causal_split(bool causal, int q0, int kt0, int nkt, int& n_nd, int& n_c) {
  if (!causal) { n_nd = n_c = nkt; return; }
  n_c = min(nkt, max(0, (q0 + 31) / KT - kt0 + 1));
  n_nd = min(n_c, max(0, (q0 + 1) / KT - kt0));
}

// ring depth per kernel and head dim (LDS: a d64 K|V stage is 16 KiB, d128 32 KiB).  Measured
// (tools/attn_bench.py, in-process A/B): d64 forward 4 stages 36.0 -> 35.1 us with the widened stores
// (ring alone -2 %); the d128 forward slower with 3 (138.5 vs 145.8 us), so it keeps 2.
template <int D, int NWK>
constexpr int fwd_stages() { return D == 64 ? 4 : 2; }
template <int D>
constexpr int dq_stages() { return D == 64 ? 4 : 2; }

// ============================================================================ forward
// NWK waves per workgroup (32 query rows each): 4, or 8 at d 128 (the K/V tiles staged once for
// twice the queries; measured 7-8 % faster at S_local 4096, equal at d 64)
template <int D, int NWK>
__device__ __forceinline__ void attn_fwd_block(const AttnArgs& a, int bx, int h_or_hk, int b, int kt_lo = 0,
                                               int kt_hi = -1, int item = -1) {
  constexpr int DT = D / 32, KS = D / 16;
  constexpr int TILE_B = KT * D * 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: an SGPR
  const int nqb = a.Sq / (NWK * 32);
  const int h = h_or_hk;
  const int qb = a.causal ? nqb - 1 - bx : bx;  // heavy blocks first
  const int hk = h / (a.H / a.HKV);
  const int q0 = qb * NWK * 32 + wave * 32;
  const int myq = q0 + (lane & 31);

  bf16x8_t qf[KS];
  if constexpr (D != 64) {
    const uint16_t* qrow = a.q + b * a.q_sb + (int64_t)myq * a.q_ss + h * a.q_sh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = ld_row_frag(qrow, ks, lane);
  }

  const uint16_t* kbase = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vbase = a.v + b * a.v_sb + hk * a.v_sh;
  const int kv_end = a.causal ? (qb + 1) * NWK * 32 : a.Sk;
  // this call's K/V tiles: all of the block's, or a split work item's [kt_lo, kt_hi)
  const int kt0 = kt_lo, nkt = (kt_hi < 0 ? kv_end / KT : kt_hi) - kt_lo;
  const float c2 = a.scale * kLog2e;

  f32x16_t o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = zero16();
  float m = -INFINITY, l = 0.f;

  constexpr int NS = fwd_stages<D, NWK>(), OPS = 2 * (KT * D * 2 / 1024) / NWK;
  auto stage = [&](int kt, int buf) {
    lds_u8* sk = smem + buf * 2 * TILE_B;
    stage_rows<D, NWK>(kbase + (int64_t)(kt0 + kt) * KT * a.k_ss, a.k_ss, sk, wave, lane);
    stage_rows<D, NWK>(vbase + (int64_t)(kt0 + kt) * KT * a.v_ss, a.v_ss, sk + TILE_B, wave, lane);
  };
  const int pre = nkt < NS - 1 ? nkt : NS - 1;
  if constexpr (D == 64) {
    // the block's Q rows by LDS-DMA too, into the ring stages the last prefetched tiles would use
    // (one stage at 4 waves, two at 8), so the prologue waits for Q and tile 0 only -- with Q as
    // compiler-tracked loads its vmcnt(0) drained every prefetched tile; those stages' tiles are
    // issued once every wave holds its Q fragments
    constexpr int QI = NWK * 32 / KT, QS = QI / 2;   // 64-row Q images, K|V stages they take
    static_assert(QI % 2 == 0 && QS < NS, "Q images fill whole K|V stages");
    lds_u8* qimg = smem + (NS - QS) * 2 * TILE_B;
    const uint16_t* qbase = a.q + b * a.q_sb + h * a.q_sh + (int64_t)qb * NWK * 32 * a.q_ss;
#pragma unroll
    for (int i = 0; i < QI; ++i) stage_rows<D, NWK>(qbase + (int64_t)i * KT * a.q_ss, a.q_ss, qimg + i * TILE_B, wave, lane);
    const int pre0 = nkt < NS - QS ? nkt : NS - QS;   // tiles in flight beside Q
    for (int t = 0; t < pre0; ++t) stage(t, t);
    if (pre0 >= 3) vm_wait<2 * OPS>();   // the younger tiles 1 .. pre0 - 1 may stay in flight
    else if (pre0 == 2) vm_wait<OPS>();
    else vm_wait<0>();
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = rd_row<D>(qimg + (wave >> 1) * TILE_B, 32 * (wave & 1), ks, lane);
    __syncthreads();   // every wave has its Q fragments before the tiles' DMA reuses those stages
    for (int t = pre0; t < pre; ++t) stage(t, t);
  } else {
    for (int t = 0; t < pre; ++t) stage(t, t);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler: its own fragment loads are done
    __syncthreads();
  }

  // one K/V tile.  d64: the diagonal tile's mask is a separate instantiation (dg 1), run by its own
  // loop (tile_loops) -- as a runtime branch the compiler if-converted it (60 compares / selects on
  // every tile) and the join copied the accumulators; d128 keeps one body with the skip and the mask
  // as runtime branches (dg 3: its split loops measured 5 % slower)
  auto tile = [&](auto dg, const lds_u8* sk, int kv0) {
    const lds_u8* sv = sk + TILE_B;
    if constexpr (decltype(dg)::value == 3)
      if (a.causal && kv0 > q0 + 31) return;  // wave-uniform: skip tiles fully above the diagonal
    {
      f32x16_t s[2];
      // the tile's K operands in one batch of LDS reads ahead of the MFMAs (left to itself the
      // compiler re-uses one register pair and waits out the LDS latency every MFMA or two)
      bf16x8_t ka[2][KS];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) ka[kh][ks] = rd_row<D>(sk, 32 * kh, ks, lane);
      PT_BATCH_BARRIER(D);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        s[kh] = zero16();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[kh] = mfma(ka[kh][ks], qf[ks], s[kh]);
      }
      // causal mask, diagonal tiles only: key row 32 kh + crow(r) visible iff <= thr
      if (decltype(dg)::value == 1 || (decltype(dg)::value == 3 && a.causal && kv0 + KT - 1 > q0)) {
        const int thr = myq - kv0 - 4 * (lane >> 5);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (32 * kh + (r & 3) + 8 * (r >> 2) > thr) s[kh][r] = -INFINITY;
      }
      float mt = -INFINITY;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kh][r]);
      mt = xor32_max(mt) * c2;  // log2 units (c2 > 0)
      // lazy rescale (FA-style deferred max): only when some query's max grew by > 2^8; P may then
      // exceed 1 by at most 2^8, harmless in f32 accumulation and in bf16 (relative precision)
      // d64 branch-free: alpha = exp2(0) = 1 exactly when no row grew, and x * 1 = x, so the result
      // is the lazy form's; as a branch the two paths' copies of O cost 16 v_mov_b64 per tile.  d128
      // (64 O registers, 8-wave workgroups) keeps the branch: its unconditional multiply measured 6 %
      // slower
      if (D == 64 || __any(mt > m + kRescaleLog2)) {
        const float mn = __any(mt > m + kRescaleLog2) ? fmaxf(m, mt) : m;
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      }
      // P = exp2(S c2 - m), summed into l: the exponent arguments as packed pairs (v_pk_fma_f32) and
      // the row sum in four packed partial sums (v_pk_add_f32, a dependency chain of 8 instead of
      // 32 serial adds), combined once at the end of the tile
      const f32x2_t c22 = {c2, c2}, nm2 = {-m, -m};
      f32x2_t ls[4];   // each partial starts as its first pair (= 0 + p: exp2 is never -0)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f32x2_t x = {s[kh][r], s[kh][r + 1]};
          x = __builtin_elementwise_fma(x, c22, nm2);
          const f32x2_t p = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
          s[kh][r] = p.x;
          s[kh][r + 1] = p.y;
          if (kh == 0 && r < 8) ls[r / 2] = p;
          else ls[(kh * 8 + r / 2) & 3] += p;
        }
      const f32x2_t lt = (ls[0] + ls[1]) + (ls[2] + ls[3]);
      l += lt.x + lt.y;
#pragma unroll
      for (int half = 0; half < 2; ++half) {  // V operands of two k-steps per batch
        bf16x8_t va[2][DT];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) va[u][dt] = rd_tr<D>(sv, 2 * half + u, dt, lane);
        PT_BATCH_BARRIER(D);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8_t pb = acc_as_b(s[half], u);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] = mfma(va[u][dt], pb, o[dt]);
        }
      }
    }
  };

  int n_nd, n_c;
  causal_split(a.causal, q0, kt0, nkt, n_nd, n_c);
  auto step = [&](auto kind, int kt) {
    if (kt + NS - 1 < nkt)  // into the stage tile kt - 1 used (every wave passed its barrier)
      stage(kt + NS - 1, (kt + NS - 1) % NS);
    if constexpr (decltype(kind)::value != 2) tile(kind, smem + (kt % NS) * 2 * TILE_B, (kt0 + kt) * KT);
    const int issued = kt + NS - 1 < nkt ? kt + NS - 1 : nkt - 1;   // the last tile issued so far
    ring_wait<OPS, NS>(issued - (kt + 1));
    __syncthreads();
  };
  if constexpr (D == 64) tile_loops(n_nd, n_c, nkt, step);
  else for (int kt = 0; kt < nkt; ++kt) step(std::integral_constant<int, 3>{}, kt);

  l = xor32_sum(l);
  if (item >= 0) {
    // a split work item: its normalised partial O (f32) and LSE, merged by attn_split_merge_kernel
    // (every query row sees at least one key of every item: split_ck is even)
    const float inv_l = l > 0.f ? 1.0f / l : 0.f;
    const int row = wave * 32 + (lane & 31);
    float* orow = a.split_o + ((int64_t)item * (NWK * 32) + row) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * (lane >> 5);
        *(float4*)(orow + d) = make_float4(o[dt][4 * g4] * inv_l, o[dt][4 * g4 + 1] * inv_l,
                                           o[dt][4 * g4 + 2] * inv_l, o[dt][4 * g4 + 3] * inv_l);
      }
    if (lane < 32) a.split_lse[(int64_t)item * (NWK * 32) + row] = l > 0.f ? m * kLn2 + __logf(l) : -INFINITY;
    return;
  }
  const float inv_l = 1.0f / l;
  const float lse = m * kLn2 + __logf(l);
  float* lse_p = a.lse + ((int64_t)b * a.H + h) * a.lse_ld + myq;
  if (!a.merge) {
    uint16_t* orow = (uint16_t*)a.o + b * a.o_sb + (int64_t)myq * a.o_ss + h * a.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_T_bf16(orow, dt, o[dt], inv_l, lane);
    if (lane < 32) *lse_p = lse;
  } else {
    // update_out_and_lse: out <- out*exp(lse_old - lse_new) + blk*exp(lse_blk - lse_new)
    float* orow = (float*)a.o + b * a.o_sb + (int64_t)myq * a.o_ss + h * a.o_sh;
    const float lold = *lse_p;
    const float lnew = fmaxf(lold, lse) + log1pf(__expf(-fabsf(lold - lse)));
    const float wold = lold == -INFINITY ? 0.f : __expf(lold - lnew);
    const float wblk = __expf(lse - lnew) * inv_l;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * (lane >> 5);
        float4 ov = *(float4*)(orow + d);
        ov.x = ov.x * wold + o[dt][4 * g4 + 0] * wblk;
        ov.y = ov.y * wold + o[dt][4 * g4 + 1] * wblk;
        ov.z = ov.z * wold + o[dt][4 * g4 + 2] * wblk;
        ov.w = ov.w * wold + o[dt][4 * g4 + 3] * wblk;
        *(float4*)(orow + d) = ov;
      }
    __syncthreads();  // both lane halves have read lse_old before it is overwritten
    if (lane < 32) *lse_p = lnew;
  }
}

template <int D, int NWK>
__global__ __launch_bounds__(NWK * 64) void attn_fwd_kernel(AttnArgs a) {
  int bx, hh, b;
  attn_coords(a, bx, hh, b);
  for (int pass = 0; pass <= a.pair; ++pass) {  // one inlined body: no register growth
    if (pass) __syncthreads();
    attn_fwd_block<D, NWK>(a, pass ? a.Sq / (NWK * 32) - 1 - bx : bx, hh, b);
  }
}

// ================================================================= few-head split work items
// With few (batch, head) rows -- a TP = 8 shard of SmolLM-1.7B has 4 heads: 16 rows x 8 query blocks,
// paired into 64 workgroups on the 256 CUs -- the forward and dQ kernels run work items of split_ck
// K/V tiles of one query block (the dK/dV kernel: split_ck (head, Q tile) steps of one key block),
// each writing an f32 partial that a merge / reduce pass combines.  Items per (batch, head): the
// blocks heaviest first (query blocks descending, key blocks ascending), each cut into chunks.
__device__ __forceinline__ int split_nq_tiles(const AttnArgs& a, int qb) {   // K tiles of query block qb
  return a.causal ? (qb + 1) * (NW * 32 / KT) : a.Sk / KT;
}
__device__ __forceinline__ int split_nk_steps(const AttnArgs& a, int kb) {   // (head, Q tile) steps of key block kb
  const int qt_begin = a.causal ? (kb * NW * 32) / KT : 0;
  return (a.Sq / KT - qt_begin) * (a.H / a.HKV);
}
// work item i -> (row bh, block, chunk c); q_side: the forward / dQ enumeration, else dK/dV's
__device__ __forceinline__ void split_item(const AttnArgs& a, int i, bool q_side, int& bh, int& blk, int& c) {
  bh = i / a.split_per_bh;
  int r = i - bh * a.split_per_bh;
  const int nb = q_side ? a.Sq / (NW * 32) : a.Sk / (NW * 32);
  for (int j = 0; j < nb; ++j) {
    blk = q_side ? nb - 1 - j : j;
    const int n = ((q_side ? split_nq_tiles(a, blk) : split_nk_steps(a, blk)) + a.split_ck - 1) / a.split_ck;
    if (r < n) { c = r; return; }
    r -= n;
  }
  c = 0;
}
// first item of (bh, blk) and its chunk count
__device__ __forceinline__ int split_base(const AttnArgs& a, int bh, int blk, bool q_side, int& nch) {
  int s = bh * a.split_per_bh;
  const int nb = q_side ? a.Sq / (NW * 32) : a.Sk / (NW * 32);
  for (int j = 0; j < nb; ++j) {
    const int bb = q_side ? nb - 1 - j : j;
    const int n = ((q_side ? split_nq_tiles(a, bb) : split_nk_steps(a, bb)) + a.split_ck - 1) / a.split_ck;
    if (bb == blk) { nch = n; return s; }
    s += n;
  }
  nch = 0;
  return s;
}
// XCD-aware item order (attn_coords' remap on a 1-D grid): an XCD takes a contiguous item range,
// so the items of one (batch, head) share that XCD's L2
__device__ __forceinline__ int split_item_id() {
  const int nwg = gridDim.x, id = blockIdx.x;
  const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
}

template <int D>
__global__ __launch_bounds__(NW * 64) void attn_fwd_split_kernel(AttnArgs a) {
  const int i = split_item_id();
  int bh, qb, c;
  split_item(a, i, true, bh, qb, c);
  const int nqb = a.Sq / (NW * 32);
  const int lo = c * a.split_ck, hi = min(lo + a.split_ck, split_nq_tiles(a, qb));
  attn_fwd_block<D, NW>(a, a.causal ? nqb - 1 - qb : qb, bh % a.H, bh / a.H, lo, hi, i);
}

// O = sum_c exp(lse_c - lse) O_c, lse = log sum_c exp(lse_c): one thread per (query row, 8 columns),
// rows in (batch, head, query) order (coalesced partial reads), bf16 O into its strided view
__global__ __launch_bounds__(256) void attn_split_merge_kernel(AttnArgs a, int D) {
  const int cpr = D / 8;
  const int64_t total = (int64_t)a.B * a.H * a.Sq * cpr;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(t % cpr);
    const int64_t r = t / cpr;
    const int q = (int)(r % a.Sq), bh = (int)(r / a.Sq);
    const int qb = q / (NW * 32), rl = q % (NW * 32);
    int n;
    const int base = split_base(a, bh, qb, true, n);
    float mx = -INFINITY;
    for (int c = 0; c < n; ++c) mx = fmaxf(mx, a.split_lse[(int64_t)(base + c) * (NW * 32) + rl]);
    float sum = 0.f;
    for (int c = 0; c < n; ++c) sum += __expf(a.split_lse[(int64_t)(base + c) * (NW * 32) + rl] - mx);
    const float lse = mx + __logf(sum);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < n; ++c) {
      const float w = __expf(a.split_lse[(int64_t)(base + c) * (NW * 32) + rl] - lse);
      const float* p = a.split_o + ((int64_t)(base + c) * (NW * 32) + rl) * D + ch * 8;
      const float4 x0 = *(const float4*)p, x1 = *(const float4*)(p + 4);
      acc[0] += w * x0.x; acc[1] += w * x0.y; acc[2] += w * x0.z; acc[3] += w * x0.w;
      acc[4] += w * x1.x; acc[5] += w * x1.y; acc[6] += w * x1.z; acc[7] += w * x1.w;
    }
    const int b = bh / a.H, h = bh % a.H;
    st8((uint16_t*)a.o + b * a.o_sb + (int64_t)q * a.o_ss + h * a.o_sh + ch * 8, pack8(acc));
    if (ch == 0) a.lse[(int64_t)bh * a.lse_ld + q] = lse;
  }
}

// ======================================================================= delta = rowsum(dO * O)
// one thread per (b, h, q) row; d in 16-byte chunks.  D is passed in a.dq_sh.
// rows in memory order (b, s, h: one row = D contiguous bf16 of the token-major layout), D/8 lanes
// per row each loading one 16-B chunk of dO and O, the row's partial dots reduced over those lanes
// by shuffles -- every wave instruction reads whole contiguous rows (coalesced), no serial chain
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnArgs a, const uint16_t* __restrict__ o) {
  const int Dh = (int)a.dq_sh;
  const int lpr = Dh / 8;  // lanes per row (8 or 16)
  const int64_t rows = (int64_t)a.B * a.Sq * a.H;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = tid; t < rows * lpr; t += nthreads) {
    const int64_t row = t / lpr;
    const int c = (int)(t - row * lpr);
    const int h = (int)(row % a.H);
    const int64_t bs = row / a.H;
    const int qq = (int)(bs % a.Sq);
    const int b = (int)(bs / a.Sq);
    float x[8], y[8];
    unpack8(ld8(a.dout + b * a.do_sb + (int64_t)qq * a.do_ss + h * a.do_sh + c * 8), x);
    unpack8(ld8(o + b * a.o_sb + (int64_t)qq * a.o_ss + h * a.o_sh + c * 8), y);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
    for (int off = lpr >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (c == 0) a.lse[((int64_t)b * a.H + h) * a.lse_ld + qq] = acc;  // the delta buffer travels in the lse slot
  }
}

// ============================================================================ dK / dV
template <int D>
__device__ __forceinline__ void attn_bwd_dkdv_block(const AttnArgs& a, int bx, int h_or_hk, int b, int it_lo = 0,
                                                    int it_hi = -1, int item = -1) {
  constexpr int DT = D / 32, KS = D / 16;
  constexpr int TILE_B = KT * D * 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: an SGPR
  const int kb = bx, hk = h_or_hk;
  const int k0 = kb * NW * 32 + wave * 32;
  const int mykey = k0 + (lane & 31);
  const int group = a.H / a.HKV;

  const uint16_t* krow = a.k + b * a.k_sb + (int64_t)mykey * a.k_ss + hk * a.k_sh;
  const uint16_t* vrow = a.v + b * a.v_sb + (int64_t)mykey * a.v_ss + hk * a.v_sh;
  bf16x8_t kf[KS], vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    kf[ks] = ld_row_frag(krow, ks, lane);
    vf[ks] = ld_row_frag(vrow, ks, lane);
  }
  f32x16_t dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) { dk[i] = zero16(); dv[i] = zero16(); }
  const float c2 = a.scale * kLog2e;

  // q tiles: causal -> only those that can see this block's keys
  const int qt_begin = a.causal ? (kb * NW * 32) / KT : 0;
  const int nqt = a.Sq / KT;
  const int nq = nqt - qt_begin;  // q tiles per query head
  // this call's (head, q tile) steps: all, or a split work item's [it_lo, it_hi)
  const int it0 = it_lo, n_iter = (it_hi < 0 ? nq * group : it_hi) - it_lo;
  // LDS: 2 x {Q tile, dO tile, lse * log2(e) [64], delta[64]}
  constexpr int STAGE_B = 2 * TILE_B + 2 * KT * 4;

  // the LSE rows go through wave 0's registers (one load per lane, scaled by log2(e) and written to
  // LDS at the end of the iteration): the exponent below is then one fma per score, not two ops
  float lse_next = 0.f;
  auto stage = [&](int hq, int qt, int buf) {
    lds_u8* sq = smem + buf * STAGE_B;
    stage_rows<D>(a.q + b * a.q_sb + (int64_t)qt * KT * a.q_ss + hq * a.q_sh, a.q_ss, sq, wave, lane);
    stage_rows<D>(a.dout + b * a.do_sb + (int64_t)qt * KT * a.do_ss + hq * a.do_sh, a.do_ss, sq + TILE_B, wave, lane);
    if (wave == 0) {  // 64 delta floats = 256 B: one 4-byte DMA per lane
      const int64_t ro = ((int64_t)b * a.H + hq) * a.lse_ld + qt * KT;
      lse_next = a.lse[ro + lane];
      pt_glds4(a.delta + ro, lane * 4u, (__attribute__((address_space(3))) void*)(sq + 2 * TILE_B + KT * 4));
    }
  };
  auto put_lse = [&](int buf) {  // after the iteration's vmcnt(0), before its barrier
    if (wave == 0) ((__attribute__((address_space(3))) float*)(smem + buf * STAGE_B + 2 * TILE_B))[lane] = lse_next * kLog2e;
  };

  // one (query head, q tile) step; edge (the causal block's first NW * 32 / KT q tiles of a head: halves
  // before my keys skipped, the diagonal one masked) and full steps are separate instantiations, run
  // by separate loops below (as the forward's tile_loops)
  auto tile = [&](auto edge, const lds_u8* sq, int qt) {
    const lds_u8* sdo = sq + TILE_B;
    const float* sl2 = (const float*)(sq + 2 * TILE_B);
    const float* sdel = sl2 + KT;
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int qs = qt * KT + 32 * qh;
      if (decltype(edge)::value && a.causal && qs + 31 < k0) continue;  // wave-uniform: all these queries precede my keys
      // S = Q K^T and dP = dO V^T  (C layout: col = key = lane, row = query)
      f32x16_t s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma(rd_row<D>(sq, 32 * qh, ks, lane), kf[ks], s);
        dp = mfma(rd_row<D>(sdo, 32 * qh, ks, lane), vf[ks], dp);
      }
      if (decltype(edge)::value && a.causal && (qs < k0 + 31)) {  // diagonal: query row crow(r) sees my key iff >= thr
        const int thr = mykey - qs - 4 * (lane >> 5);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((r & 3) + 8 * (r >> 2) < thr) s[r] = -INFINITY;
      }
      // P = exp2(S c2 - lse log2e), dS = P (dP - D): packed pairs of rows (v_pk_fma / v_pk_add / v_pk_mul)
      const f32x2_t c22 = {c2, c2};
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int qi = 32 * qh + crow(r, lane), qj = 32 * qh + crow(r + 1, lane);
        f32x2_t x = {s[r], s[r + 1]};
        x = __builtin_elementwise_fma(x, c22, (f32x2_t){-sl2[qi], -sl2[qj]});
        const f32x2_t pp = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
        const f32x2_t ds = pp * ((f32x2_t){dp[r], dp[r + 1]} - (f32x2_t){sdel[qi], sdel[qj]});
        s[r] = pp.x;                          // P
        s[r + 1] = pp.y;
        dp[r] = ds.x;                         // dS
        dp[r + 1] = ds.y;
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8_t pb = acc_as_b(s, st), db = acc_as_b(dp, st);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dv[dt] = mfma(rd_tr<D>(sdo, 2 * qh + st, dt, lane), pb, dv[dt]);
          dk[dt] = mfma(rd_tr<D>(sq, 2 * qh + st, dt, lane), db, dk[dt]);
        }
      }
    }
  };

  // (head, tile) counters for this step and the staged one (no divisions in the loop)
  int cur_h = hk * group + it0 / nq, cur_t = it0 % nq, nxt_h = cur_h, nxt_t = cur_t;
  if (n_iter > 0) stage(cur_h, qt_begin + cur_t, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler: its own fragment loads are done
  if (n_iter > 0) put_lse(0);
  __syncthreads();

  auto step = [&](auto edge, int it) {
    const int buf = it & 1;
    if (++nxt_t == nq) { nxt_t = 0; ++nxt_h; }
    if (it + 1 < n_iter) stage(nxt_h, qt_begin + nxt_t, buf ^ 1);
    const lds_u8* sq = smem + buf * STAGE_B;
    tile(edge, sq, qt_begin + cur_t);
    cur_h = nxt_h; cur_t = nxt_t;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (it + 1 < n_iter) put_lse(buf ^ 1);
    __syncthreads();
  };
  const int n_edge = a.causal ? NW * 32 / KT : 0;   // q tiles of a head that reach the diagonal
  for (int it = 0; it < n_iter;) {   // per query head: its edge steps, then its full ones
    const int h_end = min(n_iter, it + (nq - cur_t));   // this head's last step + 1
    const int e_end = min(h_end, it + max(0, n_edge - cur_t));
    for (; it < e_end; ++it) step(std::true_type{}, it);
    for (; it < h_end; ++it) step(std::false_type{}, it);
  }

  if (item >= 0) {   // a split work item: dK (scaled) and dV partials (f32), summed by attn_split_reduce_kernel
    const int64_t ro = ((int64_t)item * (NW * 32) + wave * 32 + (lane & 31)) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * (lane >> 5);
        *(float4*)(a.split_o + ro + d) = make_float4(dk[dt][4 * g4] * a.scale, dk[dt][4 * g4 + 1] * a.scale,
                                                     dk[dt][4 * g4 + 2] * a.scale, dk[dt][4 * g4 + 3] * a.scale);
        *(float4*)(a.split_dv + ro + d) = make_float4(dv[dt][4 * g4], dv[dt][4 * g4 + 1], dv[dt][4 * g4 + 2],
                                                      dv[dt][4 * g4 + 3]);
      }
    return;
  }
  if (!a.grad_f32) {
    uint16_t* dkr = (uint16_t*)a.dk + b * a.dk_sb + (int64_t)mykey * a.dk_ss + hk * a.dk_sh;
    uint16_t* dvr = (uint16_t*)a.dv + b * a.dv_sb + (int64_t)mykey * a.dv_ss + hk * a.dv_sh;
    if (a.rope_cos) {
      store_T_bf16_unrope<DT>(dkr, dk, a.scale, a.rope_cos + (int64_t)mykey * a.rope_ld,
                              a.rope_sin + (int64_t)mykey * a.rope_ld, lane);
    } else {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_T_bf16(dkr, dt, dk[dt], a.scale, lane);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_T_bf16(dvr, dt, dv[dt], 1.0f, lane);
  } else {
    float* dkr = (float*)a.dk + b * a.dk_sb + (int64_t)mykey * a.dk_ss + hk * a.dk_sh;
    float* dvr = (float*)a.dv + b * a.dv_sb + (int64_t)mykey * a.dv_ss + hk * a.dv_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      accum_T_f32(dkr, dt, dk[dt], a.scale, lane);
      accum_T_f32(dvr, dt, dv[dt], 1.0f, lane);
    }
  }
}

template <int D>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(D == 64 ? 2 : 1)))
void attn_bwd_dkdv_split_kernel(AttnArgs a) {
  const int i = split_item_id();
  int bh, kb, c;
  split_item(a, i, false, bh, kb, c);
  const int lo = c * a.split_ck, hi = min(lo + a.split_ck, split_nk_steps(a, kb));
  attn_bwd_dkdv_block<D>(a, kb, bh % a.HKV, bh / a.HKV, lo, hi, i);
}

template <int D>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(D == 64 ? 2 : 1)))
void attn_bwd_dkdv_kernel(AttnArgs a) {
  int bx, hh, b;
  attn_coords(a, bx, hh, b);
  for (int pass = 0; pass <= a.pair; ++pass) {  // one inlined body: no register growth
    if (pass) __syncthreads();
    attn_bwd_dkdv_block<D>(a, pass ? a.Sk / (NW * 32) - 1 - bx : bx, hh, b);
  }
}

// ================================================================ dK / dV, split over wave pairs
// The same products as attn_bwd_dkdv_block, divided between the two waves of a pair so that one
// SIMD holds a VALU-heavy and an MFMA-only wave side by side (8-wave workgroups; 128 keys = 4
// pairs x 32; waves w and w + 4 share a SIMD).  Wave p < 4 ("score wave") keeps K and V of the
// pair's keys in registers and runs S = Q K^T, dP = dO V^T, P = exp2(S c2 - lse log2e),
// dS = P (dP - delta); it hands P and dS, already rounded to bf16 in the MFMA B-operand layout, to
// wave p + 4 ("accumulator wave") through LDS; wave p + 4 keeps dV^T and dK^T and runs
// dV^T += dO^T P, dK^T += Q^T dS one step behind.  A step is half a Q/dO tile (32 queries); a
// tile is read in steps 2t .. 2t + 2.  Staging is a 3-deep ring: the DMA of tile t + 2 is issued
// in step 2t + 1 and waited for (counted vmcnt: the younger tile's pieces stay in flight) at the
// end of step 2t + 3, so a tile has three steps to arrive -- the workgroups of one XCD walk the
// same Q/dO tiles together, and each tile's first touch is an HBM miss all of them wait on.
// Each wave executes the same number of barriers (one per step) on its own branch.  The MFMA
// operands and their order per accumulator are those of attn_bwd_dkdv_block: dK and dV are
// bit-identical.
constexpr int kXchB = 4 * 2 * 2 * 1024;  // one step's P|dS hand-off: 4 pairs x 2 k-steps x 2 kinds x 1 KiB
constexpr int kStampB = 0;


template <int D>
__device__ __forceinline__ void attn_bwd_dkdv_pair_block(const AttnArgs& a, int bx, int hk, int b) {
  constexpr int DT = D / 32, KS = D / 16;
  constexpr int TILE_B = KT * D * 2;
  constexpr int STAGE_B = 2 * TILE_B + 2 * KT * 4;  // Q tile, dO tile, lse [64], delta [64]
  constexpr int NSTG = 3;
  // LDS-DMA pieces one tile's staging issues per wave (the lse and delta rows: wave 0)
  constexpr int OPS = 2 * (KT * D * 2 / 1024) / 8, OPS0 = OPS + 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;
  lds_u8* xch = smem + NSTG * STAGE_B;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: an SGPR
  const bool score = wave < 4;
  const int pr = wave & 3;
  const int k0 = bx * 128 + pr * 32;
  const int mykey = k0 + (lane & 31);
  const int group = a.H / a.HKV;
  const float c2 = a.scale * kLog2e;

  const int qt_begin = a.causal ? (bx * 128) / KT : 0;
  const int nq = a.Sq / KT - qt_begin;  // q tiles per query head
  const int n_tiles = nq * group;
  const int n_steps = 2 * n_tiles;

  // staging: tile t = (query head hk * group + t / nq, q tile qt_begin + t % nq), counters advanced
  // per staged tile (no divisions in the loop)
  int st_hq = hk * group, st_qt = qt_begin, st_buf = 0;
  auto stage_next = [&]() {
    lds_u8* sq = smem + st_buf * STAGE_B;
    stage_rows<D, 8>(a.q + b * a.q_sb + (int64_t)st_qt * KT * a.q_ss + st_hq * a.q_sh, a.q_ss, sq, wave, lane);
    stage_rows<D, 8>(a.dout + b * a.do_sb + (int64_t)st_qt * KT * a.do_ss + st_hq * a.do_sh, a.do_ss, sq + TILE_B,
                     wave, lane);
    if (wave == 0) {
      const int64_t ro = ((int64_t)b * a.H + st_hq) * a.lse_ld + st_qt * KT;
      pt_glds4(a.lse + ro, lane * 4u, (__attribute__((address_space(3))) void*)(sq + 2 * TILE_B));
      pt_glds4(a.delta + ro, lane * 4u, (__attribute__((address_space(3))) void*)(sq + 2 * TILE_B + KT * 4));
    }
    if (++st_qt == qt_begin + nq) { st_qt = qt_begin; ++st_hq; }
    if (++st_buf == NSTG) st_buf = 0;
  };
  // wait for every staged tile but the youngest one (when `keep`), then the barrier
  auto wait_keep = [&](bool keep) {
    if (keep) {
      if (wave == 0) vm_wait<OPS0>(); else vm_wait<OPS>();
    } else {
      vm_wait<0>();
    }
  };
  // step j (odd, j = 2t + 1) issues tile t + 2; its end waits for tile t + 1 (used from step 2t + 2)
  auto issue = [&](int j) { return (j & 1) && (j >> 1) + 2 < n_tiles; };
  auto stamp = [&](int, int) {};
  auto end_step = [&](int j) {
    stamp(j, 3);
    if (j & 1) wait_keep(issue(j));
    __syncthreads();
  };

  if (n_tiles > 0) stage_next();
  if (n_tiles > 1) stage_next();
  // the q tile of the step this wave works on (A: step j, B: step j - 1), advanced every second step
  int qt = qt_begin;
  if (score) {
    const uint16_t* krow = a.k + b * a.k_sb + (int64_t)mykey * a.k_ss + hk * a.k_sh;
    const uint16_t* vrow = a.v + b * a.v_sb + (int64_t)mykey * a.v_ss + hk * a.v_sh;
    bf16x8_t kf[KS], vf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = ld_row_frag(krow, ks, lane);
      vf[ks] = ld_row_frag(vrow, ks, lane);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler: K / V and tiles 0, 1
    __syncthreads();
    int buf = 0;
    for (int j = 0; j <= n_steps; ++j) {
      stamp(j, 0);
      if (issue(j)) stage_next();
      const int qh = j & 1;
      const int qs = qt * KT + 32 * qh;
      // causal: every query of the half tile precedes the pair's keys (wave-uniform; the partner
      // wave skips the same step)
      if (j < n_steps && !(a.causal && qs + 31 < k0)) {
        const lds_u8* sq = smem + buf * STAGE_B;
        const lds_u8* sdo = sq + TILE_B;
        const float* sl = (const float*)(sq + 2 * TILE_B);
        const float* sdel = sl + KT;
        // every LDS operand of the step is read up front (the compiler otherwise re-uses one register
        // pair and waits out the LDS latency every two MFMAs), then the MFMA chains
        bf16x8_t qa[KS], da[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          qa[ks] = rd_row<D>(sq, 32 * qh, ks, lane);
          da[ks] = rd_row<D>(sdo, 32 * qh, ks, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        f32x16_t s = zero16(), dp = zero16();
        // the score wave's MFMAs go first on the SIMD (its softmax then runs beside the partner's
        // MFMAs instead of after them)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          s = mfma(qa[ks], kf[ks], s);
          dp = mfma(da[ks], vf[ks], dp);
        }
        __builtin_amdgcn_s_setprio(0);
        // the row constants, read while the MFMAs run
        float lr[16], dr[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = 32 * qh + crow(r, lane);
          lr[r] = sl[qi];
          dr[r] = sdel[qi];
        }
        if (a.causal && (qs < k0 + 31)) {  // diagonal: query row crow(r) sees my key iff >= thr
          const int thr = mykey - qs - 4 * (lane >> 5);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if ((r & 3) + 8 * (r >> 2) < thr) s[r] = -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -(lr[r] * kLog2e)));
          s[r] = p;
          dp[r] = p * (dp[r] - dr[r]);
        }
        lds_u8* x = xch + (j & 1) * kXchB + pr * 4096 + lane * 16;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          *(__attribute__((address_space(3))) bf16x8_t*)(x + st * 2048) = acc_as_b(s, st);
          *(__attribute__((address_space(3))) bf16x8_t*)(x + st * 2048 + 1024) = acc_as_b(dp, st);
        }
      }
      if (qh) {
        if (++qt == qt_begin + nq) qt = qt_begin;
        if (++buf == NSTG) buf = 0;
      }
      end_step(j);
    }
  } else {
    f32x16_t dk[DT], dv[DT];
#pragma unroll
    for (int i = 0; i < DT; ++i) { dk[i] = zero16(); dv[i] = zero16(); }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    int buf = 0;
    for (int j = 0; j <= n_steps; ++j) {
      stamp(j, 0);
      if (issue(j)) stage_next();
      const int h = j - 1, qh = h & 1;
      if (j > 0 && !(a.causal && qt * KT + 32 * qh + 31 < k0)) {
        const lds_u8* sq = smem + buf * STAGE_B;
        const lds_u8* sdo = sq + TILE_B;
        const lds_u8* x = xch + (h & 1) * kXchB + pr * 4096 + lane * 16;
        {
          // each k-step's LDS operands are read in one batch (the compiler otherwise re-uses one
          // register pair and waits out the LDS latency every two MFMAs): k-step 1's batch is
          // issued behind k-step 0's MFMAs
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            bf16x8_t ta[DT], tq[DT];
            const bf16x8_t pb = *(const __attribute__((address_space(3))) bf16x8_t*)(x + st * 2048);
            const bf16x8_t db = *(const __attribute__((address_space(3))) bf16x8_t*)(x + st * 2048 + 1024);
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              ta[dt] = rd_tr<D>(sdo, 2 * qh + st, dt, lane);
              tq[dt] = rd_tr<D>(sq, 2 * qh + st, dt, lane);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              dv[dt] = mfma(ta[dt], pb, dv[dt]);
              dk[dt] = mfma(tq[dt], db, dk[dt]);
            }
          }
        }
      }
      if (j > 0 && qh) {
        if (++qt == qt_begin + nq) qt = qt_begin;
        if (++buf == NSTG) buf = 0;
      }
      end_step(j);
    }
    if (!a.grad_f32) {
      uint16_t* dkr = (uint16_t*)a.dk + b * a.dk_sb + (int64_t)mykey * a.dk_ss + hk * a.dk_sh;
      uint16_t* dvr = (uint16_t*)a.dv + b * a.dv_sb + (int64_t)mykey * a.dv_ss + hk * a.dv_sh;
      if (a.rope_cos) {
        store_T_bf16_unrope<DT>(dkr, dk, a.scale, a.rope_cos + (int64_t)mykey * a.rope_ld,
                                a.rope_sin + (int64_t)mykey * a.rope_ld, lane);
      } else {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) store_T_bf16(dkr, dt, dk[dt], a.scale, lane);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_T_bf16(dvr, dt, dv[dt], 1.0f, lane);
    } else {
      float* dkr = (float*)a.dk + b * a.dk_sb + (int64_t)mykey * a.dk_ss + hk * a.dk_sh;
      float* dvr = (float*)a.dv + b * a.dv_sb + (int64_t)mykey * a.dv_ss + hk * a.dv_sh;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        accum_T_f32(dkr, dt, dk[dt], a.scale, lane);
        accum_T_f32(dvr, dt, dv[dt], 1.0f, lane);
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(8 * 64) void attn_bwd_dkdv_pair_kernel(AttnArgs a) {
  int bx, hh, b;
  attn_coords(a, bx, hh, b);
  for (int pass = 0; pass <= a.pair; ++pass) {
    if (pass) __syncthreads();
    attn_bwd_dkdv_pair_block<D>(a, pass ? a.Sk / 128 - 1 - bx : bx, hh, b);
  }
}

// ============================================================================ dQ
template <int D>
__device__ __forceinline__ void attn_bwd_dq_block(const AttnArgs& a, int bx, int h_or_hk, int b, int kt_lo = 0,
                                                  int kt_hi = -1, int item = -1) {
  constexpr int DT = D / 32, KS = D / 16;
  constexpr int TILE_B = KT * D * 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: an SGPR
  const int nqb = a.Sq / (NW * 32);
  const int h = h_or_hk;
  const int qb = a.causal ? nqb - 1 - bx : bx;
  const int hk = h / (a.H / a.HKV);
  const int q0 = qb * NW * 32 + wave * 32;
  const int myq = q0 + (lane & 31);

  const uint16_t* qrow = a.q + b * a.q_sb + (int64_t)myq * a.q_ss + h * a.q_sh;
  const uint16_t* dorow = a.dout + b * a.do_sb + (int64_t)myq * a.do_ss + h * a.do_sh;
  bf16x8_t qf[KS], dof[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = ld_row_frag(qrow, ks, lane);
    dof[ks] = ld_row_frag(dorow, ks, lane);
  }
  const int64_t ri = ((int64_t)b * a.H + h) * a.lse_ld + myq;
  const float nlse2 = -a.lse[ri] * kLog2e;
  // D of this lane's row (a.delta_w: computed here from O; its half of d in this lane, the other
  // half in lane ^ 32).  The O loads are issued now and consumed after the first K/V tile's DMA
  // has been queued, so the two latencies overlap.
  bf16x8_t of[KS];
  float del = 0.f;
  if (a.delta_w) {
    const uint16_t* orow = (const uint16_t*)a.o + b * a.o_sb + (int64_t)myq * a.o_ss + h * a.o_sh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) of[ks] = ld_row_frag(orow, ks, lane);
  } else {
    del = a.delta[ri];
  }
  const float c2 = a.scale * kLog2e;

  const uint16_t* kbase = a.k + b * a.k_sb + hk * a.k_sh;
  const uint16_t* vbase = a.v + b * a.v_sb + hk * a.v_sh;
  const int kv_end = a.causal ? (qb + 1) * NW * 32 : a.Sk;
  // this call's K/V tiles: all of the block's, or a split work item's [kt_lo, kt_hi)
  const int kt0 = kt_lo, nkt = (kt_hi < 0 ? kv_end / KT : kt_hi) - kt_lo;
  f32x16_t dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dq[i] = zero16();

  constexpr int NS = dq_stages<D>(), OPS = 2 * (KT * D * 2 / 1024) / NW;
  auto stage = [&](int kt, int buf) {
    lds_u8* sk = smem + buf * 2 * TILE_B;
    stage_rows<D>(kbase + (int64_t)(kt0 + kt) * KT * a.k_ss, a.k_ss, sk, wave, lane);
    stage_rows<D>(vbase + (int64_t)(kt0 + kt) * KT * a.v_ss, a.v_ss, sk + TILE_B, wave, lane);
  };
  const int pre = nkt < NS - 1 ? nkt : NS - 1;
  for (int t = 0; t < pre; ++t) stage(t, t);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler: its own fragment loads are done
  if (a.delta_w) {
    float part = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)dof[ks][j] * (float)of[ks][j];
    del = xor32_sum(part);
    // (split work items: every item of the block forms D itself; the first one stores it)
    if (lane < 32 && kt0 == 0) a.delta_w[ri] = del;
  }
  __syncthreads();

  // one K/V tile; the diagonal tile's mask is its own instantiation (dg 1), as in the forward, at d64;
  // d128 keeps one body with the skip and the mask as runtime branches (dg 3: its 256-VGPR budget
  // spilled the split loops)
  auto tile = [&](auto dg, const lds_u8* sk, int kv0) {
    const lds_u8* sv = sk + TILE_B;
    if constexpr (decltype(dg)::value == 3)
      if (a.causal && kv0 > q0 + 31) return;  // wave-uniform: every key of the tile is after my queries
    // each 32-key half's dS feeds its two dQ k-steps right away: one dS tile live, not two
    // (16 VGPRs: d128's dQ kernel fits 2 waves per SIMD)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      f32x16_t s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma(rd_row<D>(sk, 32 * kh, ks, lane), qf[ks], s);
        dp = mfma(rd_row<D>(sv, 32 * kh, ks, lane), dof[ks], dp);
      }
      if (decltype(dg)::value == 1 || (decltype(dg)::value == 3 && a.causal && kv0 + KT - 1 > q0)) {
        // key row 32 kh + crow(r) visible iff <= thr
        const int thr = myq - kv0 - 32 * kh - 4 * (lane >> 5);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((r & 3) + 8 * (r >> 2) > thr) s[r] = -INFINITY;
      }
      // dS = P (dP - D), P = exp2(S c2 - lse log2e): at d64 as packed pairs (v_pk_fma / v_pk_add /
      // v_pk_mul); d128 keeps the scalar form (its 256-VGPR budget spilled the packed one)
      if constexpr (D == 64) {
        const f32x2_t c22 = {c2, c2}, nl2 = {nlse2, nlse2}, nd2 = {-del, -del};
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f32x2_t x = {s[r], s[r + 1]};
          x = __builtin_elementwise_fma(x, c22, nl2);
          const f32x2_t pp = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
          const f32x2_t dd = (f32x2_t){dp[r], dp[r + 1]} + nd2;
          const f32x2_t ds = pp * dd;
          s[r] = ds.x;
          s[r + 1] = ds.y;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[r], c2, nlse2));
          s[r] = p * (dp[r] - del);
        }
      }
#pragma unroll
      for (int sh = 0; sh < 2; ++sh) {
        const int st = 2 * kh + sh;
        const bf16x8_t db = acc_as_b(s, sh);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dq[dt] = mfma(rd_tr<D>(sk, st, dt, lane), db, dq[dt]);
      }
    }
  };

  int n_nd, n_c;   // the forward's ring (ring_wait) and loop split (tile_loops)
  causal_split(a.causal, q0, kt0, nkt, n_nd, n_c);
  auto step = [&](auto kind, int kt) {
    if (kt + NS - 1 < nkt) stage(kt + NS - 1, (kt + NS - 1) % NS);
    if constexpr (decltype(kind)::value != 2) tile(kind, smem + (kt % NS) * 2 * TILE_B, (kt0 + kt) * KT);
    const int issued = kt + NS - 1 < nkt ? kt + NS - 1 : nkt - 1;
    ring_wait<OPS, NS>(issued - (kt + 1));
    __syncthreads();
  };
  if constexpr (D == 64) {
    tile_loops(n_nd, n_c, nkt, step);
  } else {   // one loop: at d128 the three loops' extra copies of the body spilled (256-VGPR budget)
    for (int kt = 0; kt < nkt; ++kt) step(std::integral_constant<int, 3>{}, kt);
  }

  if (item >= 0) {   // a split work item: its dQ partial (scaled, f32), summed by attn_split_reduce_kernel
    float* prow = a.split_o + ((int64_t)item * (NW * 32) + wave * 32 + (lane & 31)) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * (lane >> 5);
        *(float4*)(prow + d) = make_float4(dq[dt][4 * g4] * a.scale, dq[dt][4 * g4 + 1] * a.scale,
                                           dq[dt][4 * g4 + 2] * a.scale, dq[dt][4 * g4 + 3] * a.scale);
      }
    return;
  }
  if (!a.grad_f32) {
    // the row index re-derived behind an opaque copy: the epilogue's row pointers (and the RoPE
    // tables') are then formed here, not hoisted into the prologue and held across the loop (at d128
    // that spilled them to scratch)
    int myq_e = myq, lane_e = lane;
    asm volatile("" : "+v"(myq_e), "+v"(lane_e));
    uint16_t* dqr = (uint16_t*)a.dq + b * a.dq_sb + (int64_t)myq_e * a.dq_ss + h * a.dq_sh;
    if (a.rope_cos) {
      store_T_bf16_unrope<DT>(dqr, dq, a.scale, a.rope_cos + (int64_t)myq_e * a.rope_ld,
                              a.rope_sin + (int64_t)myq_e * a.rope_ld, lane_e);
    } else {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_T_bf16(dqr, dt, dq[dt], a.scale, lane);
    }
  } else {
    float* dqr = (float*)a.dq + b * a.dq_sb + (int64_t)myq * a.dq_ss + h * a.dq_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) accum_T_f32(dqr, dt, dq[dt], a.scale, lane);
  }
}

template <int D>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(D == 128 ? 2 : 1)))
void attn_bwd_dq_kernel(AttnArgs a) {
  int bx, hh, b;
  attn_coords(a, bx, hh, b);
  for (int pass = 0; pass <= a.pair; ++pass) {  // one inlined body: no register growth
    if (pass) __syncthreads();
    attn_bwd_dq_block<D>(a, pass ? nqb_of(a) - 1 - bx : bx, hh, b);
  }
}

template <int D>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(D == 128 ? 2 : 1)))
void attn_bwd_dq_split_kernel(AttnArgs a) {
  const int i = split_item_id();
  int bh, qb, c;
  split_item(a, i, true, bh, qb, c);
  const int nqb = a.Sq / (NW * 32);
  const int lo = c * a.split_ck, hi = min(lo + a.split_ck, split_nq_tiles(a, qb));
  attn_bwd_dq_block<D>(a, a.causal ? nqb - 1 - qb : qb, bh % a.H, bh / a.H, lo, hi, i);
}

// dQ (q_side) or dK | dV of the split work items summed in item order, rounded to bf16 and stored
// into their strided views -- dq / dk rotated back by RoPE when tables are given, with the same
// bf16-operand arithmetic as store_T_bf16_unrope.  One thread per (row, 8 columns of each half of
// the head: d and d + D / 2), rows in (batch, head, position) order.
__global__ __launch_bounds__(256) void attn_split_reduce_kernel(AttnArgs a, int D, int q_side) {
  const int hd = D / 2, cpr = hd / 8;
  const int heads = q_side ? a.H : a.HKV, S = q_side ? a.Sq : a.Sk;
  const int64_t total = (int64_t)a.B * heads * S * cpr;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(t % cpr);
    const int64_t r = t / cpr;
    const int pos = (int)(r % S), bh = (int)(r / S);
    const int blk = pos / (NW * 32), rl = pos % (NW * 32);
    int n;
    const int base = split_base(a, bh, blk, q_side != 0, n);
    const int d0 = ch * 8;
    for (int part = 0; part < (q_side ? 1 : 2); ++part) {   // dq | (dk, dv)
      const float* src = part ? a.split_dv : a.split_o;
      float lo[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, hi[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < n; ++c) {
        const float* p = src + ((int64_t)(base + c) * (NW * 32) + rl) * D + d0;
        const float4 x0 = *(const float4*)p, x1 = *(const float4*)(p + 4);
        const float4 y0 = *(const float4*)(p + hd), y1 = *(const float4*)(p + hd + 4);
        lo[0] += x0.x; lo[1] += x0.y; lo[2] += x0.z; lo[3] += x0.w;
        lo[4] += x1.x; lo[5] += x1.y; lo[6] += x1.z; lo[7] += x1.w;
        hi[0] += y0.x; hi[1] += y0.y; hi[2] += y0.z; hi[3] += y0.w;
        hi[4] += y1.x; hi[5] += y1.y; hi[6] += y1.z; hi[7] += y1.w;
      }
      const int b = bh / heads, h = bh % heads;
      uint16_t* dst = part ? (uint16_t*)a.dv + b * a.dv_sb + (int64_t)pos * a.dv_ss + h * a.dv_sh
                           : (uint16_t*)(q_side ? a.dq : a.dk) + b * (q_side ? a.dq_sb : a.dk_sb) +
                                 (int64_t)pos * (q_side ? a.dq_ss : a.dk_ss) + h * (q_side ? a.dq_sh : a.dk_sh);
      if (!part && a.rope_cos) {
        float c[8], sn[8], o1[8], o2[8];
        unpack8(ld8(a.rope_cos + (int64_t)pos * a.rope_ld + d0), c);
        unpack8(ld8(a.rope_sin + (int64_t)pos * a.rope_ld + d0), sn);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float g1 = round_bf(lo[e]), g2 = round_bf(hi[e]);
          const float sj = -sn[e];
          o1[e] = fmaf(g1, c[e], -(g2 * sj));
          o2[e] = fmaf(g2, c[e], g1 * sj);
        }
        st8(dst + d0, pack8(o1));
        st8(dst + d0 + hd, pack8(o2));
      } else {
        st8(dst + d0, pack8(lo));
        st8(dst + d0 + hd, pack8(hi));
      }
    }
  }
}

template <typename K>
void set_smem(K kern, int bytes) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// causal block pairing (variant "attn_pair"; 0 = off, A/B measurement only)
bool pair_enabled() { return pt_variant(PT_VAR_ATTN_PAIR) == 1; }

// dK/dV kernel form per head dim (variant "attn_split"): bit 0 = d64, bit 1 = d128 use the wave-pair
// split; default d128 only
int split_mask() { return pt_variant(PT_VAR_ATTN_SPLIT); }

int check_common(const AttnArgs& a, int D) {
  if (D != 64 && D != 128) return PT_EUNSUPPORTED;
  if (a.B <= 0 || a.H <= 0 || a.HKV <= 0 || a.H % a.HKV) return PT_EINVAL;
  if (a.Sq % (NW * 32) || a.Sk % KT) return PT_EUNSUPPORTED;
  if (a.causal && a.Sq != a.Sk) return PT_EUNSUPPORTED;
  return PT_OK;
}

int attn_bwd_impl(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                  const int64_t* v_str, const void* dout, const int64_t* do_str, const float* lse,
                  const float* delta, void* dq, const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv,
                  const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D,
                  float scale, int causal, int grad_f32, const void* rope_cos, const void* rope_sin,
                  int64_t rope_stride, const void* o, const int64_t* o_str, float* delta_w, int64_t lse_ld,
                  hipStream_t stream, int parts = 3);

}  // namespace

extern "C" {

// q/k/v/o: base pointer + (batch, seq, head) strides in elements; d contiguous.
// merge = 0: o is bf16, lse written.  merge = 1: o is an f32 accumulator and lse holds the running
// LSE (initialise o = 0, lse = -inf); this block's result is merged in (update_out_and_lse).
int pt_attn_fwd(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                const int64_t* v_str, void* o, const int64_t* o_str, float* lse, int64_t B, int64_t H, int64_t HKV,
                int64_t Sq, int64_t Sk, int64_t D, float scale, int causal, int merge, int64_t lse_ld,
                hipStream_t stream) {
  if (!q || !k || !v || !o || !lse) return PT_EINVAL;
  if (lse_ld != 0 && lse_ld < Sq) return PT_EINVAL;
  AttnArgs a{};
  a.lse_ld = lse_ld ? lse_ld : Sq;
  a.q = (const uint16_t*)q; a.q_sb = q_str[0]; a.q_ss = q_str[1]; a.q_sh = q_str[2];
  a.k = (const uint16_t*)k; a.k_sb = k_str[0]; a.k_ss = k_str[1]; a.k_sh = k_str[2];
  a.v = (const uint16_t*)v; a.v_sb = v_str[0]; a.v_ss = v_str[1]; a.v_sh = v_str[2];
  a.o = o; a.o_sb = o_str[0]; a.o_ss = o_str[1]; a.o_sh = o_str[2];
  a.lse = lse;
  a.B = (int)B; a.H = (int)H; a.HKV = (int)HKV; a.Sq = (int)Sq; a.Sk = (int)Sk;
  a.scale = scale; a.causal = causal; a.merge = merge;
  int rc = check_common(a, (int)D);
  if (rc) return rc;
  // 8-wave workgroups (the K|V tiles staged once for 256 queries) at d128; at d64 measured equal or
  // slower (round 5: 35.6 vs 34.8 us, bit-identical), so 4
  const int nwk = (D == 128 && Sq % (8 * 32) == 0) ? 8 : NW;
  const int nqb = (int)(Sq / (nwk * 32));
  a.pair = causal && nqb % 2 == 0 && pair_enabled();
  const dim3 grid((unsigned)(a.pair ? nqb / 2 : nqb), (unsigned)H, (unsigned)B);
  const int stage_b = 2 * KT * (int)D * 2;
  if (D == 64) {
    const int smem = fwd_stages<64, NW>() * stage_b;   // the Q image shares the last stage
    set_smem(attn_fwd_kernel<64, NW>, smem);
    attn_fwd_kernel<64, NW><<<grid, NW * 64, smem, stream>>>(a);
  } else if (nwk == 8) {
    const int smem = fwd_stages<128, 8>() * stage_b;
    set_smem(attn_fwd_kernel<128, 8>, smem);
    attn_fwd_kernel<128, 8><<<grid, 8 * 64, smem, stream>>>(a);
  } else {
    const int smem = fwd_stages<128, NW>() * stage_b;
    set_smem(attn_fwd_kernel<128, NW>, smem);
    attn_fwd_kernel<128, NW><<<grid, NW * 64, smem, stream>>>(a);
  }
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// delta[b, h, q] = sum_d dO * O   (f32, [B, H, Sq])
int pt_attn_bwd_delta(const void* dout, const int64_t* do_str, const void* o, const int64_t* o_str, float* delta,
                      int64_t B, int64_t H, int64_t Sq, int64_t D, int64_t lse_ld, hipStream_t stream) {
  if (!dout || !o || !delta || D % 8) return PT_EINVAL;
  if (lse_ld != 0 && lse_ld < Sq) return PT_EINVAL;
  AttnArgs a{};
  a.lse_ld = lse_ld ? lse_ld : Sq;
  a.dout = (const uint16_t*)dout; a.do_sb = do_str[0]; a.do_ss = do_str[1]; a.do_sh = do_str[2];
  a.o_sb = o_str[0]; a.o_ss = o_str[1]; a.o_sh = o_str[2];
  a.lse = delta;
  a.dq_sh = D;
  a.B = (int)B; a.H = (int)H; a.Sq = (int)Sq;
  if (D != 64 && D != 128) return PT_EUNSUPPORTED;
  const int64_t total = B * H * Sq * (D / 8);  // one thread per 16-B chunk
  int64_t g = (total + 255) / 256;
  if (g > 4 * PT_STREAM_GRID_CAP) g = 4 * PT_STREAM_GRID_CAP;
  attn_delta_kernel<<<(int)g, 256, 0, stream>>>(a, (const uint16_t*)o);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// Backward from (global) out/lse: dq, dk, dv.  grad_f32 = 1 makes dq/dk/dv f32 accumulators (+=),
// used by the ring, where blocks of one query/key shard arrive over several steps.
int pt_attn_bwd(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                const int64_t* v_str, const void* dout, const int64_t* do_str, const float* lse, const float* delta,
                void* dq, const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv, const int64_t* dv_str,
                int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D, float scale, int causal,
                int grad_f32, const void* rope_cos, const void* rope_sin, int64_t rope_stride, int64_t lse_ld,
                hipStream_t stream) {
  if (!delta) return PT_EINVAL;
  return attn_bwd_impl(q, q_str, k, k_str, v, v_str, dout, do_str, lse, delta, dq, dq_str, dk, dk_str, dv, dv_str,
                       B, H, HKV, Sq, Sk, D, scale, causal, grad_f32, rope_cos, rope_sin, rope_stride, nullptr,
                       nullptr, nullptr, lse_ld, stream);
}

}  // extern "C"

namespace {

int attn_bwd_impl(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                  const int64_t* v_str, const void* dout, const int64_t* do_str, const float* lse,
                  const float* delta, void* dq, const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv,
                  const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D,
                  float scale, int causal, int grad_f32, const void* rope_cos, const void* rope_sin,
                  int64_t rope_stride, const void* o, const int64_t* o_str, float* delta_w, int64_t lse_ld,
                  hipStream_t stream, int parts) {
  if (!q || !k || !v || !dout || !lse || parts < 1 || parts > 3) return PT_EINVAL;
  if (((parts & 1) && (!dq || !dq_str)) || ((parts & 2) && (!dk || !dv || !dk_str || !dv_str))) return PT_EINVAL;
  if (delta_w && parts != 3) return PT_EINVAL;   // the fused delta comes from the dQ kernel, for dK/dV
  if (lse_ld != 0 && lse_ld < Sq) return PT_EINVAL;
  if (rope_cos && (!rope_sin || grad_f32 || Sq != Sk || (rope_stride & 3) || !pt_aligned16(rope_cos) ||
                   !pt_aligned16(rope_sin)))
    return PT_EINVAL;
  AttnArgs a{};
  a.q = (const uint16_t*)q; a.q_sb = q_str[0]; a.q_ss = q_str[1]; a.q_sh = q_str[2];
  a.k = (const uint16_t*)k; a.k_sb = k_str[0]; a.k_ss = k_str[1]; a.k_sh = k_str[2];
  a.v = (const uint16_t*)v; a.v_sb = v_str[0]; a.v_ss = v_str[1]; a.v_sh = v_str[2];
  a.dout = (const uint16_t*)dout; a.do_sb = do_str[0]; a.do_ss = do_str[1]; a.do_sh = do_str[2];
  a.lse = (float*)lse; a.delta = delta;
  a.lse_ld = lse_ld ? lse_ld : Sq;
  if (parts & 1) { a.dq = dq; a.dq_sb = dq_str[0]; a.dq_ss = dq_str[1]; a.dq_sh = dq_str[2]; }
  if (parts & 2) {
    a.dk = dk; a.dk_sb = dk_str[0]; a.dk_ss = dk_str[1]; a.dk_sh = dk_str[2];
    a.dv = dv; a.dv_sb = dv_str[0]; a.dv_ss = dv_str[1]; a.dv_sh = dv_str[2];
  }
  a.B = (int)B; a.H = (int)H; a.HKV = (int)HKV; a.Sq = (int)Sq; a.Sk = (int)Sk;
  a.scale = scale; a.causal = causal; a.grad_f32 = grad_f32;
  a.rope_cos = (const uint16_t*)rope_cos; a.rope_sin = (const uint16_t*)rope_sin; a.rope_ld = rope_stride;
  if (delta_w) {
    a.o = const_cast<void*>(o); a.o_sb = o_str[0]; a.o_ss = o_str[1]; a.o_sh = o_str[2];
    a.delta_w = delta_w;
  }
  int rc = check_common(a, (int)D);
  if (rc) return rc;
  if (Sk % (NW * 32)) return PT_EUNSUPPORTED;
  const int smem_kv = (D == 64 ? dq_stages<64>() : dq_stages<128>()) * 2 * KT * (int)D * 2;
  const int smem_q = 2 * (2 * KT * (int)D * 2 + 2 * KT * 4);
  const int nqb = (int)(Sq / (NW * 32)), nkb = (int)(Sk / (NW * 32));
  a.pair = causal && nqb % 2 == 0 && nkb % 2 == 0 && pair_enabled();
  const dim3 gq((unsigned)(a.pair ? nqb / 2 : nqb), (unsigned)H, (unsigned)B);
  const dim3 gk((unsigned)(a.pair ? nkb / 2 : nkb), (unsigned)HKV, (unsigned)B);
  const int smem_pair = 3 * (2 * KT * (int)D * 2 + 2 * KT * 4) + 2 * kXchB + kStampB;
  const bool split = (split_mask() >> (D == 64 ? 0 : 1)) & 1;
  // dQ first: with delta_w set it produces the D the dK/dV kernel reads (same stream, in order)
  if (D == 64) {
    if (parts & 1) {
      set_smem(attn_bwd_dq_kernel<64>, smem_kv);
      attn_bwd_dq_kernel<64><<<gq, NW * 64, smem_kv, stream>>>(a);
      PT_CHECK_LAUNCH();
    }
    a.delta = a.delta_w ? a.delta_w : a.delta;
    a.delta_w = nullptr;
    if (!(parts & 2)) {
    } else if (split) {
      set_smem(attn_bwd_dkdv_pair_kernel<64>, smem_pair);
      attn_bwd_dkdv_pair_kernel<64><<<gk, 8 * 64, smem_pair, stream>>>(a);
    } else {
      set_smem(attn_bwd_dkdv_kernel<64>, smem_q);
      attn_bwd_dkdv_kernel<64><<<gk, NW * 64, smem_q, stream>>>(a);
    }
  } else {
    if (parts & 1) {
      set_smem(attn_bwd_dq_kernel<128>, smem_kv);
      attn_bwd_dq_kernel<128><<<gq, NW * 64, smem_kv, stream>>>(a);
      PT_CHECK_LAUNCH();
    }
    a.delta = a.delta_w ? a.delta_w : a.delta;
    a.delta_w = nullptr;
    if (!(parts & 2)) {
    } else if (split) {
      set_smem(attn_bwd_dkdv_pair_kernel<128>, smem_pair);
      attn_bwd_dkdv_pair_kernel<128><<<gk, 8 * 64, smem_pair, stream>>>(a);
    } else {
      set_smem(attn_bwd_dkdv_kernel<128>, smem_q);
      attn_bwd_dkdv_kernel<128><<<gk, NW * 64, smem_q, stream>>>(a);
    }
  }
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// ---- few-head split forms: plan and launches
// the work-item chunk when the split forms apply (0: they do not): d64, and the regular launch (one
// workgroup per causal block pair) would put fewer than 128 workgroups on the 256 CUs
int split_ck_for(int64_t B, int64_t H, int64_t Sq, int64_t Sk, int64_t D, int causal) {
  const int ck = pt_variant(PT_VAR_ATTN_KV_CHUNK);
  if (ck <= 0 || (ck & 1) || D != 64 || Sq % (NW * 32) || Sk % (NW * 32) || (causal && Sq != Sk)) return 0;
  const int64_t nqb = Sq / (NW * 32);
  const int64_t wgs = B * H * ((causal && nqb % 2 == 0) ? nqb / 2 : nqb);
  return wgs < 128 ? ck : 0;
}
// items per (batch, head) row: forward / dQ (q_side) or dK / dV (per (batch, kv head))
int64_t split_row_items(int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int causal, int ck, bool q_side) {
  int64_t n = 0;
  if (q_side) {
    for (int64_t qb = 0; qb < Sq / (NW * 32); ++qb) {
      const int64_t nt = causal ? (qb + 1) * (NW * 32 / KT) : Sk / KT;
      n += (nt + ck - 1) / ck;
    }
  } else {
    for (int64_t kb = 0; kb < Sk / (NW * 32); ++kb) {
      const int64_t qt_begin = causal ? (kb * NW * 32) / KT : 0;
      const int64_t steps = (Sq / KT - qt_begin) * (H / HKV);
      n += (steps + ck - 1) / ck;
    }
  }
  return n;
}
inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

}  // namespace

extern "C" {

// Few-head attention (a TP shard's 4 heads): whether the split work-item forms apply to this shape and
// the f32 workspace they need -- forward (backward = 0): partial O and LSE per item; backward: partial
// dQ, dK, dV per item.  Returns 1 (ws_bytes set) or 0 (the regular launches; ws_bytes = 0).
int pt_attn_split_plan(int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D, int causal, int backward,
                       int64_t* ws_bytes) {
  if (!ws_bytes || B <= 0 || H <= 0 || HKV <= 0 || H % HKV) return PT_EINVAL;
  *ws_bytes = 0;
  const int ck = split_ck_for(B, H, Sq, Sk, D, causal);
  if (!ck) return 0;
  const int64_t iq = B * H * split_row_items(H, HKV, Sq, Sk, causal, ck, true);
  const int64_t rows = NW * 32;
  if (!backward) {
    *ws_bytes = align256(iq * rows * D * 4) + align256(iq * rows * 4);
  } else {
    const int64_t ik = B * HKV * split_row_items(H, HKV, Sq, Sk, causal, ck, false);
    *ws_bytes = align256(iq * rows * D * 4) + 2 * align256(ik * rows * D * 4);
  }
  return 1;
}

// pt_attn_fwd (merge = 0, dense lse) in the split form: work items of attn_kv_chunk K/V tiles of
// one query block, then the merge pass (O bf16 and lse)
int pt_attn_fwd_split(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                      const int64_t* v_str, void* o, const int64_t* o_str, float* lse, int64_t B, int64_t H,
                      int64_t HKV, int64_t Sq, int64_t Sk, int64_t D, float scale, int causal, void* ws,
                      int64_t ws_bytes, hipStream_t stream) {
  if (!q || !k || !v || !o || !lse || !ws) return PT_EINVAL;
  int64_t need = 0;
  if (pt_attn_split_plan(B, H, HKV, Sq, Sk, D, causal, 0, &need) != 1) return PT_EUNSUPPORTED;
  if (ws_bytes < need || !pt_aligned16(ws)) return PT_EINVAL;
  if ((o_str[0] & 7) || (o_str[1] & 7) || (o_str[2] & 7) || !pt_aligned16(o)) return PT_EALIGN;
  AttnArgs a{};
  a.lse_ld = Sq;
  a.q = (const uint16_t*)q; a.q_sb = q_str[0]; a.q_ss = q_str[1]; a.q_sh = q_str[2];
  a.k = (const uint16_t*)k; a.k_sb = k_str[0]; a.k_ss = k_str[1]; a.k_sh = k_str[2];
  a.v = (const uint16_t*)v; a.v_sb = v_str[0]; a.v_ss = v_str[1]; a.v_sh = v_str[2];
  a.o = o; a.o_sb = o_str[0]; a.o_ss = o_str[1]; a.o_sh = o_str[2];
  a.lse = lse;
  a.B = (int)B; a.H = (int)H; a.HKV = (int)HKV; a.Sq = (int)Sq; a.Sk = (int)Sk;
  a.scale = scale; a.causal = causal;
  int rc = check_common(a, (int)D);
  if (rc) return rc;
  a.split_ck = split_ck_for(B, H, Sq, Sk, D, causal);
  a.split_per_bh = (int)split_row_items(H, HKV, Sq, Sk, causal, a.split_ck, true);
  const int64_t items = B * H * a.split_per_bh;
  a.split_o = (float*)ws;
  a.split_lse = (float*)((char*)ws + align256(items * NW * 32 * D * 4));
  const int smem = fwd_stages<64, NW>() * 2 * KT * 64 * 2;   // the Q image shares the last stage
  set_smem(attn_fwd_split_kernel<64>, smem);
  attn_fwd_split_kernel<64><<<(unsigned)items, NW * 64, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  const int64_t total = B * H * Sq * (D / 8);
  int64_t g = (total + 255) / 256;
  if (g > 4 * PT_STREAM_GRID_CAP) g = 4 * PT_STREAM_GRID_CAP;
  attn_split_merge_kernel<<<(unsigned)g, 256, 0, stream>>>(a, (int)D);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// pt_attn_bwd_fused_delta in the split form: dQ items (each forms D from O; the first of a block
// stores it), then dK/dV items of attn_kv_chunk (head, Q tile) steps, then one reduce pass each
int pt_attn_bwd_split(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                      const int64_t* v_str, const void* o, const int64_t* o_str, const void* dout, const int64_t* do_str,
                      const float* lse, float* delta_out, void* dq, const int64_t* dq_str, void* dk,
                      const int64_t* dk_str, void* dv, const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV,
                      int64_t Sq, int64_t Sk, int64_t D, float scale, int causal, const void* rope_cos,
                      const void* rope_sin, int64_t rope_stride, void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (!q || !k || !v || !o || !dout || !lse || !delta_out || !dq || !dk || !dv || !ws) return PT_EINVAL;
  int64_t need = 0;
  if (pt_attn_split_plan(B, H, HKV, Sq, Sk, D, causal, 1, &need) != 1) return PT_EUNSUPPORTED;
  if (ws_bytes < need || !pt_aligned16(ws)) return PT_EINVAL;
  if (!pt_aligned16(o) || (o_str[0] & 7) || (o_str[1] & 7) || (o_str[2] & 7)) return PT_EALIGN;
  for (const int64_t* st : {dq_str, dk_str, dv_str})
    if ((st[0] & 7) || (st[1] & 7) || (st[2] & 7)) return PT_EALIGN;
  if (!pt_aligned16(dq) || !pt_aligned16(dk) || !pt_aligned16(dv)) return PT_EALIGN;
  if (rope_cos && (!rope_sin || Sq != Sk || (rope_stride & 7) || !pt_aligned16(rope_cos) || !pt_aligned16(rope_sin)))
    return PT_EINVAL;
  AttnArgs a{};
  a.q = (const uint16_t*)q; a.q_sb = q_str[0]; a.q_ss = q_str[1]; a.q_sh = q_str[2];
  a.k = (const uint16_t*)k; a.k_sb = k_str[0]; a.k_ss = k_str[1]; a.k_sh = k_str[2];
  a.v = (const uint16_t*)v; a.v_sb = v_str[0]; a.v_ss = v_str[1]; a.v_sh = v_str[2];
  a.dout = (const uint16_t*)dout; a.do_sb = do_str[0]; a.do_ss = do_str[1]; a.do_sh = do_str[2];
  a.o = const_cast<void*>(o); a.o_sb = o_str[0]; a.o_ss = o_str[1]; a.o_sh = o_str[2];
  a.lse = (float*)lse; a.lse_ld = Sq;
  a.delta_w = delta_out;
  a.dq = dq; a.dq_sb = dq_str[0]; a.dq_ss = dq_str[1]; a.dq_sh = dq_str[2];
  a.dk = dk; a.dk_sb = dk_str[0]; a.dk_ss = dk_str[1]; a.dk_sh = dk_str[2];
  a.dv = dv; a.dv_sb = dv_str[0]; a.dv_ss = dv_str[1]; a.dv_sh = dv_str[2];
  a.B = (int)B; a.H = (int)H; a.HKV = (int)HKV; a.Sq = (int)Sq; a.Sk = (int)Sk;
  a.scale = scale; a.causal = causal;
  a.rope_cos = (const uint16_t*)rope_cos; a.rope_sin = (const uint16_t*)rope_sin; a.rope_ld = rope_stride;
  int rc = check_common(a, (int)D);
  if (rc) return rc;
  const int ck = split_ck_for(B, H, Sq, Sk, D, causal);
  const int64_t per_q = split_row_items(H, HKV, Sq, Sk, causal, ck, true);
  const int64_t per_k = split_row_items(H, HKV, Sq, Sk, causal, ck, false);
  const int64_t iq = B * H * per_q, ik = B * HKV * per_k;
  char* w = (char*)ws;
  float* pdq = (float*)w;
  float* pdk = (float*)(w + align256(iq * NW * 32 * D * 4));
  float* pdv = (float*)((char*)pdk + align256(ik * NW * 32 * D * 4));
  a.split_ck = ck;
  // dQ items
  a.split_per_bh = (int)per_q;
  a.split_o = pdq;
  const int smem_kv = dq_stages<64>() * 2 * KT * 64 * 2;
  set_smem(attn_bwd_dq_split_kernel<64>, smem_kv);
  attn_bwd_dq_split_kernel<64><<<(unsigned)iq, NW * 64, smem_kv, stream>>>(a);
  PT_CHECK_LAUNCH();
  const int64_t tq = B * H * Sq * (D / 16);
  int64_t g = (tq + 255) / 256;
  if (g > 4 * PT_STREAM_GRID_CAP) g = 4 * PT_STREAM_GRID_CAP;
  attn_split_reduce_kernel<<<(unsigned)g, 256, 0, stream>>>(a, (int)D, 1);
  PT_CHECK_LAUNCH();
  // dK / dV items read the D the dQ items stored
  a.delta = delta_out;
  a.delta_w = nullptr;
  a.split_per_bh = (int)per_k;
  a.split_o = pdk;
  a.split_dv = pdv;
  const int smem_q = 2 * (2 * KT * 64 * 2 + 2 * KT * 4);
  set_smem(attn_bwd_dkdv_split_kernel<64>, smem_q);
  attn_bwd_dkdv_split_kernel<64><<<(unsigned)ik, NW * 64, smem_q, stream>>>(a);
  PT_CHECK_LAUNCH();
  const int64_t tk = B * HKV * Sk * (D / 16);
  g = (tk + 255) / 256;
  if (g > 4 * PT_STREAM_GRID_CAP) g = 4 * PT_STREAM_GRID_CAP;
  attn_split_reduce_kernel<<<(unsigned)g, 256, 0, stream>>>(a, (int)D, 0);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// pt_attn_bwd computing only dQ (parts 1) or only dK / dV (parts 2): the full-mesh context-parallel
// backward runs each rank's dQ against the visiting K / V and its own keys' dK / dV against the
// visiting queries (the other pointers may be NULL)
int pt_attn_bwd_part(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                     const int64_t* v_str, const void* dout, const int64_t* do_str, const float* lse,
                     const float* delta, void* dq, const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv,
                     const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D,
                     float scale, int causal, int grad_f32, int64_t lse_ld, int parts, hipStream_t stream) {
  if (!delta) return PT_EINVAL;
  return attn_bwd_impl(q, q_str, k, k_str, v, v_str, dout, do_str, lse, delta, dq, dq_str, dk, dk_str, dv, dv_str,
                       B, H, HKV, Sq, Sk, D, scale, causal, grad_f32, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                       lse_ld, stream, parts);
}

// pt_attn_bwd with D = rowsum(dO * O) computed inside the dQ kernel from o (bf16, strides o_str)
// and written to delta_out [B, H, Sq] f32 (replaces the separate pt_attn_bwd_delta pass)
int pt_attn_bwd_fused_delta(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str,
                            const void* v, const int64_t* v_str, const void* o, const int64_t* o_str,
                            const void* dout, const int64_t* do_str, const float* lse, float* delta_out, void* dq,
                            const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv,
                            const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk,
                            int64_t D, float scale, int causal, const void* rope_cos, const void* rope_sin,
                            int64_t rope_stride, int64_t lse_ld, hipStream_t stream) {
  if (!o || !delta_out || !o_str) return PT_EINVAL;
  if (!pt_aligned16(o) || (o_str[0] & 7) || (o_str[1] & 7) || (o_str[2] & 7)) return PT_EALIGN;
  return attn_bwd_impl(q, q_str, k, k_str, v, v_str, dout, do_str, lse, nullptr, dq, dq_str, dk, dk_str, dv,
                       dv_str, B, H, HKV, Sq, Sk, D, scale, causal, 0, rope_cos, rope_sin, rope_stride, o, o_str,
                       delta_out, lse_ld, stream);
}

}  // extern "C"
