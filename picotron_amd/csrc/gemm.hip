// bf16 MFMA GEMM for gfx950 with fp32 accumulation: the dense contractions of the decoder layer.
//
// Replaces (reference, /root/reference): every F.linear / matmul on the hot path --
//   picotron/model.py:124-126,161,186,270 (q/k/v/out, up/gate/down, lm_head),
//   picotron/tensor_parallel/tp_communications.py:105 (ColumnParallel), tensor_parallel.py:186 (RowParallel),
//   tp_communications.py:79,93,98 (LinearWithAsyncAllReduce fwd/bwd).
//
//   C[M,N] (op)= A[M,K] . B[K,N]
//   A is K-contiguous ("row", X[T,K]) or M-contiguous (dY^T for dW = dY^T X)
//   B is K-contiguous (weight W[N,K] -> Y = X W^T) or N-contiguous (W[K,N] for dX = dY W; X for dW)
//
// Segmented operands (one launch instead of several, and enough tiles to fill 256 CUs):
//   * B may be split into up to 4 pointers along N (fused q|k|v or gate|up forward) or along K
//     (dX = [dq|dk|dv] . [Wq;Wk;Wv]);  * C may be split along M (dW of q,k,v in one launch).
//   Segment boundaries must be multiples of the tile (checked on the host).
//
// Kernels (all v_mfma_f32_16x16x32_bf16, fp32 accumulators, operands staged global->LDS by
// global_load_lds_dwordx4: LDS-DMA, lane-linear 1 KiB per wave instruction; the XOR swizzle is
// applied to the per-lane SOURCE address and undone on the ds_read -- tools/lds_swizzle_search.py:
// conflict-free for ds_read_b128 on K-contiguous images and ds_read_b64_tr_b16 on MN-contiguous
// images):
//  * gemm_8ph_kernel (tile 12, 256x256) and gemm_4ph_kernel (tile 13, 256x128): phased,
//    wave-group ping-pong schedules with one counted vmcnt per K-tile (see each kernel) -- every
//    projection of the layer, 1.0-1.38 PF/s (profiles/r01_gemm_tiles_8ph.md).
//  * gemm_kernel (tiles 2 / 3 / 4 / 5 / 8 / 9): the simple two-stage loop, for shapes the phased
//    kernels do not divide.
// One launch may carry up to 4 independent problems (pt_gemm_grouped) to fill the CUs.
//
// Epilogue: the wave's tile is staged through LDS as bf16 rows and written as whole 16-byte row
// segments; fp32 epilogues (main_grad accumulation) write the accumulator directly.
#include "common.h"

#include <limits.h>
#include <stdlib.h>
#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;

namespace {

constexpr int BK = 64;

// Accumulator layout.  Every MFMA is fed (B fragment, A fragment), so a 16x16 accumulator holds
// C^T of its block: lane l has row (l & 15), columns 4 (l >> 4) .. +3 -- four consecutive columns
// of one row.  The epilogue then stages each (i, j) fragment with ONE 8-byte (bf16) / 16-byte
// (f32) LDS write instead of four 2- / 4-byte ones (a wave's 128 x 64 bf16 tile: 32 instead of
// 128 LDS write instructions).  Same products and summation order as the (A, B) order.
__device__ __forceinline__ int acc_row(int i, int lane) { return i * 16 + (lane & 15); }
__device__ __forceinline__ int acc_col(int j, int r, int lane) { return j * 16 + (lane >> 4) * 4 + r; }
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
template <typename V, typename A>
__device__ __forceinline__ A mfma16(const V& a, const V& b, const A& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, 0, 0, 0);
}

// EPI_BF16_RES: C = bf16(R + bf16(acc)) -- the residual add of model.py:207-208 fused into the
// producing GEMM (R may alias C).
// EPI_SWIGLU_FWD: the gate|up projection with SwiGLU (model.py:186) in its epilogue: B = {W_gate,
//   W_up} consumed in PAIRED tiles (output tile n = gate rows and up rows 128n..128n+127), writes
//   C[0] = h = bf16(bf16(silu(g)) * u) [M, N] and C[1] = the [M, 2N] g|u buffer the backward reads.
// EPI_SWIGLU_BWD: dh = dY . W_down with the SwiGLU backward in its epilogue: R = g|u [M, 2N];
//   C[0] = dg|du [M, 2N] (dh itself is never written).
enum Epilogue {
  EPI_BF16 = 0, EPI_BF16_ACC = 1, EPI_F32 = 2, EPI_F32_ACC = 3, EPI_BF16_RES = 4,
  EPI_SWIGLU_FWD = 5, EPI_SWIGLU_BWD = 6,
  // EPI_ROPE: the q|k|v projection with RoPE (model.py:136-137) on its q|k columns in the
  // epilogue; head_dim 64 = the wave tile's width, so (d, d + 32) pairs sit in one lane
  EPI_ROPE = 7,
  // EPI_CE_STATS: the lm_head (model.py:270) storing bf16 logits AND, per row and per output tile
  // (BN = 256 / 128 columns), the cross-entropy forward's statistics of the stored bf16 values:
  // (max m, sum exp(x - m)) as float2 stats[(col / BN) * M + row] (tile-major: each workgroup
  // writes its rows' pairs as one contiguous run) -- the CE forward (train.py:49) then combines
  // N / BN pairs per row instead of streaming the [M, N] logits again
  EPI_CE_STATS = 8
};

// SwiGLU element math, the same expressions as csrc/swiglu.hip (torch's bf16 roundings)
__device__ __forceinline__ float silu_sig(float x) { return pt_sigmoid(x); }

struct GemmArgs {
  const uint16_t* A;
  int64_t lda;
  // A's second K-segment: k >= ak2 reads A2 (same lda) -- a weight gradient over two micro-batches'
  // token rows (dY of both, K = 2 T); ak2 = INT32_MAX: none.  The 256x256 8-phase kernel only.
  const uint16_t* A2;
  int ak2;
  const uint16_t* B[4];
  int64_t ldb[4];
  int64_t bseg[5];  // boundaries along N (bdim 0) or K (bdim 1)
  int nbseg;
  int bdim;
  void* C[4];
  int64_t ldc[4];
  int64_t cseg[5];  // boundaries along M
  int ncseg;
  const uint16_t* R;  // residual (EPI_BF16_RES), indexed like C segment 0
  int64_t ldr;
  const uint16_t* rope_cos;  // EPI_ROPE: [seq, rope_ld] bf16 tables (get_cos_sin, model.py:21-31)
  const uint16_t* rope_sin;
  int64_t rope_ld;
  int rope_seq, rope_cols;   // position = row % rope_seq; columns [0, rope_cols) are rotated
  float* stats;              // EPI_CE_STATS: float2 [N / BN][M], (max, sumexp) per row and tile
  int M, N, K;
  int tiles_m, tiles_n;
  int group_m;
  // split-K: the launch computes ksplit K-slices of K / ksplit each (EPI_F32 only); slice s writes
  // its f32 partial at C + s * kpart_stride (pt_gemm_splitk_reduce sums them into the real sink)
  int ksplit;
  int64_t kpart_stride;
};

// swizzles (chunk = 16 bytes); see tools/lds_swizzle_search.py
__device__ __forceinline__ int swz_k(int r) { return (r >> 1) & 7; }                    // 128-B rows
__device__ __forceinline__ int swz_mn(int r, int row_bytes) {
  return row_bytes >= 256 ? 2 * ((r & 3) | ((r >> 1) & 4)) : 2 * (((r >> 1) & 1) | ((r >> 2) & 2));
}

__device__ __forceinline__ void glds16(const void* gsrc, lds_u8* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Stage one operand image (ROWS x 64 if K-contiguous, 64 x ROWS if MN-contiguous) into LDS.
// `g` points at element (image row/col 0, k0) of the operand; ld is its leading dimension.
template <int ROWS, bool KCONTIG, int NTHREADS>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ g, int64_t ld, lds_u8* lds, int tid) {
  constexpr int kInstr = ROWS * BK * 2 / 1024;  // 1 KiB per wave instruction
  constexpr int kWaves = NTHREADS / 64;
  static_assert(kInstr % kWaves == 0, "tile must split evenly over waves");
  const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int it = 0; it < kInstr / kWaves; ++it) {
    const int i = it * kWaves + wave;
    if (KCONTIG) {
      const int r = i * 8 + (lane >> 3), c = lane & 7;
      glds16(g + (int64_t)r * ld + 8 * (c ^ swz_k(r)), lds + i * 1024);
    } else {
      constexpr int rb = ROWS * 2;           // bytes per k-row of the image
      constexpr int rc = rb / 16;            // 16-B chunks per k-row
      constexpr int rows_per = 1024 / rb;    // k-rows per instruction
      const int r = i * rows_per + lane / rc, c = lane % rc;
      glds16(g + (int64_t)r * ld + 8 * (c ^ swz_mn(r, rb)), lds + i * 1024);
    }
  }
}

// one 16x32 (A) or 32x16 (B) bf16 fragment for k-substep s (k = 32s .. 32s+31)
template <int ROWS, bool KCONTIG>
__device__ __forceinline__ bf16x8_t read_frag(const lds_u8* lds, int rbase, int s, int lane) {
  if (KCONTIG) {
    const int r = rbase + (lane & 15);
    const int C = 4 * s + (lane >> 4);
    return *(const __attribute__((address_space(3))) bf16x8_t*)(lds + r * 128 + 16 * (C ^ swz_k(r)));
  } else {
    constexpr int rb = ROWS * 2;
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = rbase + 4 * p;
    // NB: read as bf16x4 and concatenate whole vectors; an element-wise bit_cast of a short4
    // result miscompiles on ROCm 7.2 (the halves were duplicated; tools/probe_tr.*)
    bf16x4_t t[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kr = 32 * s + 8 * g + 4 * h + q;
      const int off = kr * rb + 16 * ((col >> 3) ^ swz_mn(kr, rb)) + 8 * ((col >> 2) & 1);
      t[h] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4_t*)(lds + off));
    }
    return __builtin_shufflevector(t[0], t[1], 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

__device__ __forceinline__ int find_seg(const int64_t* bounds, int n, int64_t x) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < n && x >= bounds[i]) s = i;
  return s;
}

// bijective XCD-aware remap: consecutive tile ids land on the same XCD (blocks b, b+8 share one)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// A launch runs up to kMaxProb independent problems ("grouped GEMM": e.g. dW of q|k|v and dW of
// o_proj, 192 + 64 tiles, fill the 256 CUs together where each alone leaves CUs idle).  Problems
// share the kernel instantiation (layouts, epilogue, tile); their tiles are numbered
// consecutively (start[i] = first tile id of problem i).
constexpr int kMaxProb = 4;
struct GemmGroup {
  GemmArgs p[kMaxProb];
  int start[kMaxProb + 1];
  int nprob;
};

// tile order: XCD remap over the whole grid (consecutive ids share an XCD), then the problem,
// then group `group_m` tile-rows so an XCD's consecutive tiles form a compact block of the
// output (A and B panels shared through that XCD's L2): 6 rows (group_m_for: measured faster
// than the 8 / 4 rows that made 32 tiles one 2048 x 1024 / 1024 x 1024 block)
// tile id pid_all (already in XCD order) of group g -> its problem and (tile_m, tile_n)
// (split-K: the K-slice is the outermost index of a problem's tiles, so an XCD's consecutive tiles
// share one slice's A / B panels)
__device__ __forceinline__ const GemmArgs& select_problem_pid(const GemmGroup& g, int pid_all, int& tile_m,
                                                              int& tile_n, int& kslice) {
  int pi = 0;
#pragma unroll
  for (int i = 1; i < kMaxProb; ++i)
    if (i < g.nprob && pid_all >= g.start[i]) pi = i;
  const GemmArgs& a = g.p[pi];
  int pid = pid_all - g.start[pi];
  const int per_slice = a.tiles_m * a.tiles_n;
  kslice = a.ksplit > 1 ? pid / per_slice : 0;
  pid -= kslice * per_slice;
  const int GROUP = a.group_m;
  const int group_span = GROUP * a.tiles_n;
  const int gid = pid / group_span;
  const int first_m = gid * GROUP;
  const int gsize = min(a.tiles_m - first_m, GROUP);
  tile_m = first_m + (pid % group_span) % gsize;
  tile_n = (pid % group_span) / gsize;
  return a;
}

__device__ __forceinline__ const GemmArgs& select_problem(const GemmGroup& g, int& tile_m, int& tile_n, int& kslice,
                                                          int bid = -1, int nwg = -1) {
  const int pid_all = bid < 0 ? xcd_remap(blockIdx.x, gridDim.x) : xcd_remap(bid, nwg);
  return select_problem_pid(g, pid_all, tile_m, tile_n, kslice);
}

// K range of split-K slice ks: first element, and the slice's K-tile count
__device__ __forceinline__ int kslice_begin(const GemmArgs& a, int ks) { return a.ksplit > 1 ? ks * (a.K / a.ksplit) : 0; }
__device__ __forceinline__ int kslice_tiles(const GemmArgs& a) { return (a.ksplit > 1 ? a.K / a.ksplit : a.K) / BK; }

// Write the wave's TM x TN accumulator tile (FM x FN 16x16 fragments) at output (m0 + wm*TM,
// n0 + wn*TN).  `st` is this wave's private LDS staging area (TM * (2*TN + 16) bytes).
// sum / max over the 8 consecutive lanes of a lane's group (lane & ~7): DPP, no LDS round trip
template <int CTRL>
__device__ __forceinline__ float dpp8(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float max8(float v) {
  v = fmaxf(v, dpp8<0xB1>(v));    // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp8<0x4E>(v));    // quad_perm [2,3,0,1]
  return fmaxf(v, dpp8<0x141>(v));  // row_half_mirror: lane i <-> 7 - i, the other quad
}
__device__ __forceinline__ float sum8(float v) {
  v += dpp8<0xB1>(v);
  v += dpp8<0x4E>(v);
  return v + dpp8<0x141>(v);
}

// EPI_CE_STATS, after every wave's epilogue wrote its rows' (max, sumexp) over its TN columns into
// xs[(wm * WN + wn) * TM + row] (and a barrier): the WN = 0 waves merge the WN pairs of each of
// their TM rows and store them contiguously at stats[(n0 / (WN * TN)) * M + row].
template <int WN, int TM, int TN>
__device__ __forceinline__ void ce_stats_merge(const GemmArgs& a, const float2* xs, int m0, int n0, int wm, int lane) {
  float2* out = (float2*)a.stats + (int64_t)(n0 / (WN * TN)) * a.M + m0 + wm * TM;
#pragma unroll
  for (int r = lane; r < TM; r += 64) {
    float2 p[WN];
#pragma unroll
    for (int w = 0; w < WN; ++w) p[w] = xs[(wm * WN + w) * TM + r];
    float M = p[0].x;
#pragma unroll
    for (int w = 1; w < WN; ++w) M = fmaxf(M, p[w].x);
    float S = 0.f;
#pragma unroll
    for (int w = 0; w < WN; ++w) S += p[w].y * __expf(p[w].x - M);
    out[r] = make_float2(M, S);
  }
}

// EPI_SWIGLU_BWD tail: the wave's TM x TN dh tile is staged (bf16) in `st`; read g|u, write
// dg|du (swiglu.hip's backward), SG chunks of g and u per group, row-group bases in SGPRs (one
// address VGPR per lane).  The tail is HBM-bound -- the 256 tiles of a round reach it together and
// move 134 MB at ~4.5 TB/s -- and a stream that alternates loads and stores runs it fastest:
// issuing all 2 x NIT loads before any math measured 3 % slower than 2 chunks per group
// (profiles/r02_notes.md).
constexpr int kSwigluGroup = 2;   // chunks per load group (4: equal, 16: -0.4 %; profiles/r04/notes_r04.md)
template <int TM, int TN>
__device__ __forceinline__ void swiglu_bwd_tail(const GemmArgs& a, const lds_u8* st, int64_t mrow0, int ncol0,
                                                int64_t ldc, uint16_t* C, int lane) {
  constexpr int ROWB = TN * 2 + 16, CPR = TN / 8, RPI = 64 / CPR, NIT = TM / RPI, SG = kSwigluGroup;
  static_assert(NIT % SG == 0, "chunk groups");
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  const int lrow = lane / CPR, ch = lane % CPR;
  const uint32_t roff = (uint32_t)(lrow * a.ldr + ch * 8) * 2u;  // bytes from the row group's base
  const uint32_t coff = (uint32_t)(lrow * ldc + ch * 8) * 2u;
  const int64_t r0 = (int64_t)__builtin_amdgcn_readfirstlane((int)mrow0);
  const int c0 = __builtin_amdgcn_readfirstlane(ncol0);
  const uint8_t* gbase = (const uint8_t*)(a.R + r0 * a.ldr + c0);
  uint8_t* cbase = (uint8_t*)(C + r0 * ldc + c0);
  const int64_t rstep = (int64_t)RPI * a.ldr * 2, cstep = (int64_t)RPI * ldc * 2, ustep = (int64_t)a.N * 2;
#pragma unroll
  for (int q0 = 0; q0 < NIT; q0 += SG) {
    bf16x8 g[SG], u[SG];
#pragma unroll
    for (int k = 0; k < SG; ++k) {
      // g|u: the forward's activations, read once here -- non-temporal, beside the dual launch's
      // weight-gradient tiles and their operand panels
      g[k] = ld8_nt((const uint16_t*)(gbase + (q0 + k) * rstep + roff));
      u[k] = ld8_nt((const uint16_t*)(gbase + (q0 + k) * rstep + ustep + roff));
    }
#pragma unroll
    for (int k = 0; k < SG; ++k) {
      const int q = q0 + k, row = q * RPI + lrow;
      const u32x4_t raw = *(const __attribute__((address_space(3))) u32x4_t*)(st + row * ROWB + ch * 16);
      bf16x8 v;
      v.w[0] = raw[0]; v.w[1] = raw[1]; v.w[2] = raw[2]; v.w[3] = raw[3];
      float d[8], gg[8], uu[8], og[8], ou[8];
      unpack8(v, d);
      unpack8(g[k], gg);
      unpack8(u[k], uu);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sg = silu_sig(gg[e]);
        ou[e] = d[e] * round_bf(gg[e] * sg);
        og[e] = round_bf(d[e] * uu[e]) * (sg * (1.0f + gg[e] * (1.0f - sg)));
      }
      st8((uint16_t*)(cbase + q * cstep + coff), pack8(og));
      st8((uint16_t*)(cbase + q * cstep + ustep + coff), pack8(ou));
    }
  }
}

// EPI_F32_ACC (the f32 main_grad sink of DataParallelBucket): C += acc in two TM / 2-row passes
// through this wave's LDS staging area (TM / 2 x 64 f32 + pad fits the TM x (64 bf16 + pad) area
// the bf16 epilogues use) so that every global access is a
// whole 16-byte chunk of a row (the accumulator layout gives 4-byte pieces of 16 rows); the old
// values of BOTH passes are loaded before the first store (one memory round trip per wave, was
// one per 16-row fragment row), pass 1's loads issued once pass 0's accumulators are staged.
// ACC = false: EPI_F32, store only (the split-K dgrad's f32 partials), the same row-chunk writes.
template <int TM, int TN, bool ACC = true>
__device__ __forceinline__ void f32_acc_tail(const f32x4_t (&acc)[TM / 16][TN / 16], lds_u8* st, int64_t mrow0,
                                             int ncol0, int64_t ldc, float* C, int lane) {
  constexpr int HR = TM / 2, NP = 2, FP = HR / 16, FN = TN / 16;
  static_assert(HR * (TN * 4 + 16) <= TM * (TN * 2 + 16), "f32 pass fits the staging area");
  constexpr int ROWB = TN * 4 + 16, CPR = TN / 4, RPI = 64 / CPR, NIT = HR / RPI;
  const int lrow = lane / CPR, ch = lane % CPR;
  const int64_t r0 = (int64_t)__builtin_amdgcn_readfirstlane((int)mrow0);
  const int c0 = __builtin_amdgcn_readfirstlane(ncol0);
  uint8_t* cbase = (uint8_t*)(C + r0 * ldc + c0);
  const uint32_t coff = (uint32_t)(lrow * ldc + ch * 4) * 4u;
  const int64_t rstep = (int64_t)RPI * ldc * 4;
  f32x4_t old[NP][NIT];
  // the f32 main_grad is read-modify-written once per micro-batch, nothing re-reads it soon: non-
  // temporal loads / stores, so it does not push the GEMMs' operand panels out of L2 / Infinity Cache
  typedef __attribute__((address_space(1))) f32x4_t g_f32x4_t;
  auto load_pass = [&](int p) {
#pragma unroll
    for (int q = 0; q < NIT; ++q)
      old[p][q] = __builtin_nontemporal_load((const g_f32x4_t*)(cbase + (p * NIT + q) * rstep + coff));
  };
  auto stage_pass = [&](int p) {
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)  // the fragment's 4 columns of one row: one 16-byte write
        *(__attribute__((address_space(3))) f32x4_t*)(st + acc_row(i, lane) * ROWB + acc_col(j, 0, lane) * 4) =
            acc[p * FP + i][j];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private staging
  };
  if (ACC) load_pass(0);
  stage_pass(0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int p = 1; p < NP; ++p)
    if (ACC) load_pass(p);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (p > 0) stage_pass(p);
#pragma unroll
    for (int q = 0; q < NIT; ++q) {
      const f32x4_t v = *(const __attribute__((address_space(3))) f32x4_t*)(st + (q * RPI + lrow) * ROWB + ch * 16);
      if (ACC) {
        asm volatile("" : "+v"(old[p][q]));
        __builtin_nontemporal_store(old[p][q] + v, (g_f32x4_t*)(cbase + (p * NIT + q) * rstep + coff));
      } else {
        *(f32x4_t*)(cbase + (p * NIT + q) * rstep + coff) = v;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // this pass's LDS reads done before the next staging
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int TM, int TN, int EPI>
__device__ __forceinline__ void epilogue(const GemmArgs& a, const f32x4_t (&acc)[TM / 16][TN / 16], lds_u8* st,
                                         int m0, int n0, int wm, int wn, int lane, float2* xs_wave = nullptr,
                                         int64_t c_off = 0) {
  constexpr int FM = TM / 16, FN = TN / 16;
  const int cs = find_seg(a.cseg, a.ncseg, m0);
  const int64_t ldc = a.ldc[cs];
  const int64_t mrow0 = m0 - a.cseg[cs] + wm * TM;
  const int ncol0 = n0 + wn * TN;
  if (EPI == EPI_BF16 || EPI == EPI_BF16_ACC || EPI == EPI_BF16_RES || EPI == EPI_SWIGLU_BWD || EPI == EPI_ROPE ||
      EPI == EPI_CE_STATS) {
    constexpr int ROWB = TN * 2 + 16;  // +16 B pad: spreads the staging writes over banks
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {  // 4 consecutive columns of one row: one 8-byte write
        const u32x2_t w = {pack_bf2(acc[i][j][0], acc[i][j][1]), pack_bf2(acc[i][j][2], acc[i][j][3])};
        *(__attribute__((address_space(3))) u32x2_t*)(st + acc_row(i, lane) * ROWB + acc_col(j, 0, lane) * 2) = w;
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private staging, no barrier needed
    // keep the epilogue's loads below the staging (the accumulators die there): hoisted above it,
    // they would be live next to all of acc and spill
    __builtin_amdgcn_sched_barrier(0);
    uint16_t* C = (uint16_t*)a.C[cs];
    if constexpr (EPI == EPI_SWIGLU_BWD) {
      swiglu_bwd_tail<TM, TN>(a, st, mrow0, ncol0, ldc, C, lane);
      return;
    }
    if constexpr (EPI == EPI_ROPE && TN == 64) {
      if (ncol0 < a.rope_cols) {
        // the wave's 64 columns are one head: lane = (row, chunk ch < 4) rotates chunk ch with
        // its partner ch + 4 (d, d + 32) from the bf16 staging, as csrc/rope.hip does
        typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
        // every row's cos / sin chunk loaded before the first store (C may alias the tables as far
        // as the compiler knows: loaded per row, they were one table round trip per 16 rows)
        constexpr int NR = TM / 16;
        bf16x8 cv[NR], sv[NR];
#pragma unroll
        for (int it = 0; it < NR; ++it) {
          const int row = it * 16 + lane / 4, ch = lane % 4;
          const int64_t pos = (mrow0 + row) % a.rope_seq;
          cv[it] = ld8(a.rope_cos + pos * a.rope_ld + ch * 8);
          sv[it] = ld8(a.rope_sin + pos * a.rope_ld + ch * 8);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int it = 0; it < NR; ++it) {
          const int row = it * 16 + lane / 4, ch = lane % 4;
          asm volatile("" : "+v"(cv[it].w[0]), "+v"(cv[it].w[1]), "+v"(cv[it].w[2]), "+v"(cv[it].w[3]));
          asm volatile("" : "+v"(sv[it].w[0]), "+v"(sv[it].w[1]), "+v"(sv[it].w[2]), "+v"(sv[it].w[3]));
          const u32x4_t r1 = *(const __attribute__((address_space(3))) u32x4_t*)(st + row * ROWB + ch * 16);
          const u32x4_t r2 = *(const __attribute__((address_space(3))) u32x4_t*)(st + row * ROWB + (ch + 4) * 16);
          float x1[8], x2[8], c[8], sn[8], o1[8], o2[8];
          bf16x8 v1, v2;
          v1.w[0] = r1[0]; v1.w[1] = r1[1]; v1.w[2] = r1[2]; v1.w[3] = r1[3];
          v2.w[0] = r2[0]; v2.w[1] = r2[1]; v2.w[2] = r2[2]; v2.w[3] = r2[3];
          unpack8(v1, x1);
          unpack8(v2, x2);
          unpack8(cv[it], c);
          unpack8(sv[it], sn);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            o1[e] = fmaf(x1[e], c[e], -(x2[e] * sn[e]));
            o2[e] = fmaf(x2[e], c[e], x1[e] * sn[e]);
          }
          uint16_t* dst = C + (mrow0 + row) * ldc + ncol0 + ch * 8;
          st8(dst, pack8(o1));
          st8(dst + 32, pack8(o2));
        }
        return;
      }
    }
    constexpr int CPR = TN / 8;          // 16-B chunks per row
    constexpr int RPI = 64 / CPR;        // rows per wave instruction
    constexpr int NIT = TM / RPI;
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    // the epilogues that READ memory (g|u, the residual, the accumulated gradient) issue all their
    // loads first, then consume them: C may alias R / the old gradient, so the compiler would keep
    // every load behind the previous iteration's store -- one HBM round trip per row group
    // (all NIT chunks -- 4 NIT VGPRs, the accumulators are dead once staged -- before any store,
    // so the wave's epilogue is one memory round trip)
    constexpr bool RD = EPI == EPI_BF16_ACC || EPI == EPI_BF16_RES;
    constexpr int GRP = NIT;
#pragma unroll
    for (int g0 = 0; g0 < NIT; g0 += GRP) {
      bf16x8 pre[GRP][1];
      if constexpr (RD) {
#pragma unroll
        for (int q = 0; q < GRP; ++q) {
          const int row = (g0 + q) * RPI + lane / CPR, ch = lane % CPR;
          const uint16_t* src = EPI == EPI_BF16_ACC ? C + (mrow0 + row) * ldc + ncol0 + ch * 8
                                                    : a.R + (mrow0 + row) * a.ldr + ncol0 + ch * 8;
          // the accumulated weight gradient (.grad): read-modify-written once per micro-batch,
          // non-temporal (as the f32 main_grad in f32_acc_tail); the residual: read once, too
          pre[q][0] = ld8_nt(src);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < GRP; ++q) {
        const int row = (g0 + q) * RPI + lane / CPR, ch = lane % CPR;
        const u32x4_t raw = *(const __attribute__((address_space(3))) u32x4_t*)(st + row * ROWB + ch * 16);
        bf16x8 v;
        v.w[0] = raw[0]; v.w[1] = raw[1]; v.w[2] = raw[2]; v.w[3] = raw[3];
        uint16_t* dst = C + (mrow0 + row) * ldc + ncol0 + ch * 8;
        if constexpr (EPI == EPI_CE_STATS) {
          // the row's TN = 64 columns of this wave are the CPR = 8 consecutive lanes sharing
          // lane / 8: max and sum-exp of the stored (bf16) values over the 8 x 8, one pair per row
          static_assert(TN == 64, "CE statistics: 64-column wave tiles (8 lanes per row)");
          float f[8];
          unpack8(v, f);
          const float mx = max8(fmaxf(fmaxf(fmaxf(f[0], f[1]), fmaxf(f[2], f[3])),
                                      fmaxf(fmaxf(f[4], f[5]), fmaxf(f[6], f[7]))));
          const float nm = -mx * 1.4426950408889634f;
          float se = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) se += __builtin_amdgcn_exp2f(fmaf(f[e], 1.4426950408889634f, nm));
          se = sum8(se);
          if (ch == 0) xs_wave[row] = make_float2(mx, se);
        }
        if constexpr (EPI == EPI_BF16_ACC || EPI == EPI_BF16_RES) {
          // opaque: keeps chunk q's unpacking (and so its wait) here, after every load is issued
          asm volatile("" : "+v"(pre[q][0].w[0]), "+v"(pre[q][0].w[1]), "+v"(pre[q][0].w[2]), "+v"(pre[q][0].w[3]));
          float o[8], f[8];
          unpack8(v, f);
          unpack8(pre[q][0], o);
          // acc was rounded to bf16 once above; add in f32 and round again (== torch's bf16 add)
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += f[e];
          v = pack8(o);
        }
        if constexpr (EPI == EPI_BF16_ACC) st8_nt(dst, v);
        else st8(dst, v);
      }
    }
  } else {
    float* C = (float*)a.C[cs] + c_off;   // c_off: this split-K slice's partial (EPI_F32)
    if constexpr (EPI == EPI_F32_ACC && TN == 64) {
      f32_acc_tail<TM, TN>(acc, st, mrow0, ncol0, ldc, C, lane);
      return;
    }
    if constexpr (EPI == EPI_F32 && TN == 64) {  // store only (the split-K partials): whole 16-B row chunks
      if ((ldc & 3) == 0 && ((uintptr_t)C & 15) == 0) {
        f32_acc_tail<TM, TN, false>(acc, st, mrow0, ncol0, ldc, C, lane);
        return;
      }
    }
    // f32 store (and accumulate for other wave tiles): one fragment row (FN x 4 values) of old
    // values loaded before any of its stores
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      float old[FN][4];
      if (EPI == EPI_F32_ACC) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            old[j][r] = C[(mrow0 + acc_row(i, lane)) * ldc + ncol0 + acc_col(j, r, lane)];
      }
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mrow0 + acc_row(i, lane);
          const int col = ncol0 + acc_col(j, r, lane);
          C[row * ldc + col] = EPI == EPI_F32_ACC ? old[j][r] + acc[i][j][r] : acc[i][j][r];
        }
    }
  }
}

// Stage a 128 x 32 bf16 tile (value f(i, j, r) at wave row acc_row(i), column acc_col(j, r))
// through this wave's LDS area and write it at dst (+ row * ld) as 16-B row segments.
template <typename F>
__device__ __forceinline__ void write_128x32(lds_u8* st, int lane, uint16_t* dst, int64_t ld, F f) {
  constexpr int ROWB = 32 * 2 + 16;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const u32x2_t w = {pack_bf2(f(i, j, 0), f(i, j, 1)), pack_bf2(f(i, j, 2), f(i, j, 3))};
      *(__attribute__((address_space(3))) u32x2_t*)(st + acc_row(i, lane) * ROWB + acc_col(j, 0, lane) * 2) = w;
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
#pragma unroll
  for (int it = 0; it < 128 / 16; ++it) {
    const int row = it * 16 + lane / 4, ch = lane % 4;
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    const u32x4_t raw = *(const __attribute__((address_space(3))) u32x4_t*)(st + row * ROWB + ch * 16);
    bf16x8 v;
    v.w[0] = raw[0]; v.w[1] = raw[1]; v.w[2] = raw[2]; v.w[3] = raw[3];
    st8(dst + row * ld + ch * 8, v);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // the staging area is reused by the next call
}

// EPI_SWIGLU_FWD: the wave's 128 x 64 accumulators are 32 gate columns (acc[.][0..1]) and the
// SAME 32 up columns (acc[.][2..3]) of output columns hc0 .. hc0+31.
__device__ __forceinline__ void epilogue_swiglu_fwd(const GemmArgs& a, f32x4_t (&acc)[8][4], lds_u8* st, int64_t row0,
                                                    int hc0, int lane) {
  uint16_t* H = (uint16_t*)a.C[0];
  uint16_t* GU = (uint16_t*)a.C[1];
  const int64_t ldh = a.ldc[0], ldgu = a.ldc[1];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = round_bf(acc[i][j][r]);  // g, u are bf16 tensors
  write_128x32(st, lane, GU + row0 * ldgu + hc0, ldgu, [&](int i, int j, int r) { return acc[i][j][r]; });
  write_128x32(st, lane, GU + row0 * ldgu + a.N + hc0, ldgu, [&](int i, int j, int r) { return acc[i][j + 2][r]; });
  write_128x32(st, lane, H + row0 * ldh + hc0, ldh, [&](int i, int j, int r) {
    const float g = acc[i][j][r];
    return round_bf(g * silu_sig(g)) * acc[i][j + 2][r];
  });
}

// B operand image base for the tile at (n0, k0) (+ n_off columns inside the tile)
// Segment selection by a compare chain on constant indices: every kernarg load is loop-invariant
// (hoisted into SGPRs) -- an indexed a.B[s] load would put a dependent scalar-memory round trip
// in front of every DMA issue.
__device__ __forceinline__ const uint16_t* b_image_ptr(const GemmArgs& a, bool bkc, int n0, int k0, int n_off,
                                                       int64_t& ldb) {
  const int64_t x = a.bdim == 0 ? n0 : k0;
  const uint16_t* Bp = a.B[0];
  int64_t ld = a.ldb[0], base = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const bool in = i < a.nbseg && x >= a.bseg[i];
    Bp = in ? a.B[i] : Bp;
    ld = in ? a.ldb[i] : ld;
    base = in ? a.bseg[i] : base;
  }
  ldb = ld;
  const int64_t nl = (a.bdim == 0 ? n0 - base : n0) + n_off;
  const int64_t kl = a.bdim == 1 ? k0 - base : k0;
  return bkc ? Bp + nl * ld + kl : Bp + kl * ld + nl;
}

// B image base of K-tile k0 for the tile at n0, with the B segments (N- or K-split) read from the
// kernarg ONCE, before the K loop, into registers.  (Calling b_image_ptr per K-tile re-issued its
// kernarg loads after every inline-asm wait -- the "memory" clobber -- behind an s_waitcnt
// lgkmcnt(0) that also drained the phase's in-flight LDS reads: every K-segmented launch, i.e.
// every dX GEMM, ran 20-30 % slow.)
struct BImg {
  // element (k = 0, n = n0) of the first segment; a K-segment i >= 1 adds d_i elements to the
  // base from k = s_i on (INT_MAX: no such segment) -- independent selects against 0 on plain
  // integers: pointer selects over an array / nested chain were materialised in scratch memory
  // (a scratch load per K-tile).  K-segments share one ld (checked on the host).
  const uint16_t* b0;
  int64_t d1, d2, d3;
  int s1, s2, s3;
  int64_t ld;
};

__device__ __forceinline__ int64_t bimg_seg_base(const GemmArgs& a, bool bkc, int n0, int i, int& start) {
  const bool kseg = a.bdim == 1 && i < a.nbseg;
  const int64_t k0 = kseg ? a.bseg[i] : 0;
  // element (k, n0) of segment i = B_i + (k - k0) ld + n0  (N-contig) / B_i + n0 ld + (k - k0)
  const int64_t off = bkc ? (int64_t)n0 * a.ldb[i] - k0 : (int64_t)n0 - k0 * a.ldb[i];
  start = kseg ? (int)k0 : INT_MAX;
  return kseg ? (int64_t)((intptr_t)a.B[i] + off * 2) : 0;
}

__device__ __forceinline__ BImg bimg_make(const GemmArgs& a, bool bkc, int n0) {
  BImg r;
  int64_t ld;
  r.b0 = b_image_ptr(a, bkc, n0, 0, 0, ld);
  r.ld = ld;
  const int64_t p0 = (int64_t)(intptr_t)r.b0;
  const int64_t p1 = bimg_seg_base(a, bkc, n0, 1, r.s1);
  const int64_t p2 = bimg_seg_base(a, bkc, n0, 2, r.s2);
  const int64_t p3 = bimg_seg_base(a, bkc, n0, 3, r.s3);
  r.d1 = r.s1 == INT_MAX ? 0 : p1 - p0;
  r.d2 = r.s2 == INT_MAX ? 0 : p2 - p1;
  r.d3 = r.s3 == INT_MAX ? 0 : p3 - p2;
  return r;
}

__device__ __forceinline__ const uint16_t* bimg_ptr(const BImg& b, bool bkc, int k0) {
  const int64_t e1 = k0 >= b.s1 ? b.d1 : 0;
  const int64_t e2 = k0 >= b.s2 ? b.d2 : 0;
  const int64_t e3 = k0 >= b.s3 ? b.d3 : 0;
  const int64_t k_off = bkc ? (int64_t)k0 : (int64_t)k0 * b.ld;
  return (const uint16_t*)((intptr_t)b.b0 + e1 + e2 + e3 + k_off * 2);
}

// ============================================================================ 8-phase 256x256
// 256x256 tile, BK = 64, 8 waves as 2(M) x 4(N), each wave a 128 x 64 output (8 x 4 accumulators
// of 16x16).  Each operand tile is held as two "half images" of 128 rows (A) / columns (B) x 64 k,
// split so that one half holds exactly the fragments every wave reads in one phase:
//   At = tile rows {0-63, 128-191}   (rows 0-63 of each M-wave's 128)   read in phase 1
//   Ab = tile rows {64-127, 192-255}                                    read in phase 3
//   Bl = tile cols {0-31, 64-95, 128-159, 192-223} (cols 0-31 of each N-wave's 64)   phase 1
//   Br = the other 128 columns                                          read in phase 2
// K-tile t = 4 phases (one 64x32 quadrant of the wave's output each: (0,0) (0,1) (1,1) (1,0)),
// each { LDS reads; one half-image LDS-DMA; lgkmcnt(0); barrier; 16 MFMAs; barrier }.  A half
// image is re-staged the phase after its last read (the reads were retired before that phase's
// first barrier): At, Bl, Br of K-tile t+2 in phases 2-4 of t (into t's buffer), Ab of t+1 in
// phase 1 of t.  The single wait per K-tile (phase 4, before its first barrier) is vmcnt(6): it
// retires K-tile t+1 and leaves t+2's three halves in flight.  Wave group 1 (waves 4-7) runs one
// barrier behind group 0, so on each SIMD one wave multiplies while the other reads and stages
// (cdna_hip_programming.md §5 "The 256² 8-phase template"; RAW: data is read >= 2 barriers after
// the wait that retired it).  LDS: 2 buffers x 4 halves x 16 KiB = 128 KiB (+ epilogue staging).
template <bool KC, int SPAN>
__device__ __forceinline__ uint32_t himg_voff(int i, int lane, int64_t ld, int off) {
  // element offset (from the operand's (tile row/col 0, k0) element) of lane's 16-B chunk of
  // 1-KiB DMA instruction i of a half image whose image row/col r maps to tile row/col
  // (r / SPAN) * 2 SPAN + r % SPAN + off
  if (KC) {
    const int r = i * 8 + (lane >> 3), c = lane & 7;
    const int row = (r / SPAN) * 2 * SPAN + r % SPAN + off;
    return (uint32_t)(row * ld + 8 * (c ^ swz_k(r)));
  } else {
    const int r = i * 4 + (lane >> 4), c = lane & 15;
    const int col = 8 * (c ^ swz_mn(r, 256));
    const int tc = (col / SPAN) * 2 * SPAN + col % SPAN + off;
    return (uint32_t)(r * ld + tc);
  }
}

__device__ __forceinline__ void glds16_asm(const uint16_t* base, uint32_t voff_elems, lds_u8* dst) {
  pt_glds16(base, voff_elems * 2u, (__attribute__((address_space(3))) void*)dst);  // common.h
}

// one 256x256 output tile (tile_m, tile_n) of problem `a` by the whole 512-thread workgroup
template <bool AK, bool BKC, int EPI>
__device__ __forceinline__ void gemm_8ph_tile(const GemmArgs& a, const int tile_m, const int tile_n, const int ks = 0) {
  constexpr int TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int HALF = 128 * BK * 2;          // 16 KiB
  constexpr int BUF = 4 * HALF;               // At, Bl, Br, Ab
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: an SGPR
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = tile_m * 256, n0 = tile_n * 256;

  // B segment for this tile (N-segments) or the first K-segment; ld is per tile (host checks
  // that K-segments share one ld)
  constexpr bool PAIR = EPI == EPI_SWIGLU_FWD;  // Bl = W_gate rows, Br = W_up rows of tile n
  const BImg bi = bimg_make(a, BKC, PAIR ? 0 : n0);
  const int64_t ldb = PAIR ? a.ldb[0] : bi.ld;
  const uint16_t* const pairB0 = a.B[0];
  const uint16_t* const pairB1 = a.B[1];
  const int64_t lda = a.lda;
  // loop-invariant per-lane element offsets of this wave's 2 DMA instructions per half image
  uint32_t vA[2][2], vB[2][2];  // [half][it]
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 8 + wave;
    vA[0][it] = himg_voff<AK, 64>(i, lane, lda, 0);
    vA[1][it] = himg_voff<AK, 64>(i, lane, lda, 64);
    if (PAIR) {
      vB[0][it] = vB[1][it] = himg_voff<BKC, 128>(i, lane, ldb, 0);
    } else {
      vB[0][it] = himg_voff<BKC, 32>(i, lane, ldb, 0);
      vB[1][it] = himg_voff<BKC, 32>(i, lane, ldb, 32);
    }
  }
  const int kb = kslice_begin(a, ks);        // this split-K slice's first k (0 unsplit)
  const uint16_t* Ab0 = AK ? a.A + (int64_t)m0 * lda + kb : a.A + m0 + (int64_t)kb * lda;
  // A's second K-segment (a two-micro-batch weight gradient): from k = ak2 on, element (k, m) is
  // A2's (k - ak2, m): the same address plus one element offset, read once into registers
  const int ak2 = a.ak2;
  const int64_t a_d2 = a.A2 ? ((int64_t)(intptr_t)a.A2 - (int64_t)(intptr_t)a.A) / 2 -
                                  (AK ? (int64_t)ak2 : (int64_t)ak2 * lda)
                            : 0;
  auto a_ptr = [&](int t) {
    const int64_t e2 = kb + t * BK >= ak2 ? a_d2 : 0;
    return (AK ? Ab0 + t * BK : Ab0 + (int64_t)t * BK * lda) + e2;
  };
  auto b_ptr = [&](int t) { return bimg_ptr(bi, BKC, kb + t * BK); };
  // paired: rows tile_n * 128 .. +127 of W_gate (Bl) and W_up (Br), K-contiguous
  auto pair_ptr = [&](int t, int which) {
    return (which ? pairB1 : pairB0) + (int64_t)tile_n * 128 * ldb + kb + t * BK;
  };
  // half image h (0 At, 1 Bl, 2 Br, 3 Ab) of K-tile t into buffer buf
  auto stage = [&](int t, int buf, int h) {
    lds_u8* dst = smem + buf * BUF + h * HALF;
    const bool isA = h == 0 || h == 3;
    const uint16_t* base = isA ? a_ptr(t) : (PAIR ? pair_ptr(t, h == 2) : b_ptr(t));
    const int sel = (h == 0 || h == 1) ? 0 : 1;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const uint32_t vo = isA ? vA[sel][it] : vB[sel][it];
      glds16_asm(base, vo, dst + (it * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = kslice_tiles(a);
  stage(0, 0, 0); stage(0, 0, 1); stage(0, 0, 2); stage(0, 0, 3);
  if (nk > 1) {
    stage(1, 1, 0); stage(1, 1, 1); stage(1, 1, 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  bf16x8_t af[4][2], b0[2][2], b1[2][2];
  auto mma = [&](int i0, int j0, const bf16x8_t (&A)[4][2], const bf16x8_t (&Bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = mfma16(A[i][s], Bf[j][s], acc[i0 + i][j0 + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  const bool late = __builtin_amdgcn_readfirstlane(wm) == 1;
  if (late) bar();

  auto ktile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    const lds_u8* sAt = smem + buf * BUF;
    const lds_u8* sBl = sAt + HALF;
    const lds_u8* sBr = sAt + 2 * HALF;
    const lds_u8* sAb = sAt + 3 * HALF;
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // phase 1: At rows + Bl cols; stage Ab(t+1); quadrant (0, 0)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = read_frag<128, AK>(sAt, wm * 64 + i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[j][s] = read_frag<128, BKC>(sBl, wn * 32 + j * 16, s, lane);
    if (n1) stage(t + 1, buf ^ 1, 3);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(0, 0, af, b0);
    bar();
    // phase 2: Br cols; stage At(t+2); quadrant (0, 1)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) b1[j][s] = read_frag<128, BKC>(sBr, wn * 32 + j * 16, s, lane);
    if (n2) stage(t + 2, buf, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(0, 2, af, b1);
    bar();
    // phase 3: Ab rows; stage Bl(t+2); quadrant (1, 1)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = read_frag<128, AK>(sAb, wm * 64 + i * 16, s, lane);
    if (n2) stage(t + 2, buf, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(4, 2, af, b1);
    bar();
    // phase 4: no reads; stage Br(t+2); retire K-tile t+1; quadrant (1, 0)
    if (n2) {
      stage(t + 2, buf, 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (n1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    mma(4, 0, af, b0);
    bar();
  };

  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  if (!late) bar();  // balance the barrier count of the two wave groups
  __syncthreads();
  if constexpr (PAIR) {
    epilogue_swiglu_fwd(a, acc, smem + wave * (TM * (32 * 2 + 16)), m0 + wm * TM, tile_n * 128 + wn * 32, lane);
  } else {
    // EPI_CE_STATS: per-wave row statistics beside the 8 staging areas (launch_8ph sizes the LDS)
    float2* xs = (float2*)(smem + 8 * (TM * (TN * 2 + 16)));
    epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane, xs + wave * TM,
                          (int64_t)ks * a.kpart_stride);
    if constexpr (EPI == EPI_CE_STATS) {
      __syncthreads();
      if (wn == 0) ce_stats_merge<4, TM, TN>(a, xs, m0, n0, wm, lane);
    }
  }
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(512) void gemm_8ph_kernel(const GemmGroup g) {
  int tile_m, tile_n, ks;
  const GemmArgs& a = select_problem(g, tile_m, tile_n, ks);
  gemm_8ph_tile<AK, BKC, EPI>(a, tile_m, tile_n, ks);
}

// ---------------------------------------------------------------------------- dual launch
// Two INDEPENDENT groups in one launch of 256x256 8-phase tiles, each with its own layouts and
// epilogue: the down_proj dX with the SwiGLU backward in its epilogue beside the down_proj dW
// (both read only dY and saved activations).  One launch instead of two: the dX tiles' HBM-bound
// epilogue tail (the g|u read and dg|du write, ~4.5 TB/s while every CU is in it) shares the launch
// with the dW tiles' main loops -- measured 271 vs 280 us for the two launches at SmolLM-1.7B
// shapes.  Each XCD (blocks b, b + 8, ... share one) takes an equal, contiguous share of each
// group's tiles (n0 / n1 per XCD), so both keep their XCD-grouped L2 reuse; `order` 0 runs an
// XCD's group-0 tiles first, 1 its group-1 tiles first.  (Interleaving the groups inside an XCD,
// in proportion or with the CUs split between them by work, measured 4-7 % slower: two GEMMs'
// panels then share each L2; profiles/r02_notes.md.)
struct DualMap {
  int n0, n1, order;
};

// order 2 (staggered): even XCDs run their group-0 tiles first, odd XCDs their group-1 tiles first,
// so the dX tiles' HBM-bound SwiGLU-backward tails of half the chip overlap the other half's dW
// main loops instead of all 256 CUs reaching them together (each XCD still works on one GEMM at a
// time: its L2 grouping is kept)
__device__ __forceinline__ int dual_select(const DualMap& m, int& pid) {
  const int bid = blockIdx.x, xcd = bid & 7, li = bid >> 3;
  const int ord = m.order == 2 ? (xcd & 1) : m.order;
  const int nfirst = ord == 0 ? m.n0 : m.n1;
  const bool first = li < nfirst;
  const int which = (ord == 0) ? !first : first;
  const int local = first ? li : li - nfirst;
  pid = xcd * (which ? m.n1 : m.n0) + local;
  return which;
}

template <bool AK0, bool BKC0, int EPI0, bool AK1, bool BKC1, int EPI1>
__global__ __launch_bounds__(512) void gemm_8ph_dual_kernel(const GemmGroup g0, const GemmGroup g1, const DualMap m) {
  int pid, tile_m, tile_n, ks;
  if (dual_select(m, pid) == 0) {
    const GemmArgs& a = select_problem_pid(g0, pid, tile_m, tile_n, ks);
    gemm_8ph_tile<AK0, BKC0, EPI0>(a, tile_m, tile_n, ks);
  } else {
    const GemmArgs& a = select_problem_pid(g1, pid, tile_m, tile_n, ks);
    gemm_8ph_tile<AK1, BKC1, EPI1>(a, tile_m, tile_n, ks);
  }
}

// ============================================================================ 4-phase 256x128
// For the N = 2048 shapes (o_proj, down_proj forward, every dX GEMM of the layer, the lm_head dX),
// where 256x256 tiles put only 128 workgroups on the 256 CUs.  256x128 tile, BK = 64, 8 waves as
// 4(M) x 2(N), each wave a 64 x 64 output (4 x 4 accumulators): the same A + B fragment bytes per
// MFMA as the 8-wave 256x256 kernel's 128 x 64 wave tiles.  Three images per K-tile:
//   At = tile rows {0-31, 64-95, 128-159, 192-223} (rows 0-31 of each M-wave's 64)  read in phase 1
//   Ab = the other 128 rows                                                           read in phase 2
//   B  = all 128 columns                                                              read in phase 1
// K-tile t = 2 phases (upper / lower 32 x 64 half of the wave's output, 16 MFMAs each), same
// phase anatomy and wave-group stagger as the 8-phase kernel.  With 48 KiB per K-tile the LDS holds
// THREE K-tiles (144 KiB): K-tile t+2 is staged during K-tile t into the buffer K-tile t-1 freed
// (At in phase 1, B and Ab in phase 2), and the one wait per K-tile (phase 2, vmcnt(6)) retires
// K-tile t+1 with t+2 in flight -- every DMA has >= 1.5 K-tiles to land.
template <bool AK, bool BKC, int EPI>
__device__ __forceinline__ void gemm_4ph_tile(const GemmArgs& a, const int tile_m, const int tile_n, const int ks = 0) {
  constexpr int TM = 64, TN = 64, FM = 4, FN = 4;
  constexpr int IMG = 128 * BK * 2;           // 16 KiB
  constexpr int BUF = 3 * IMG;                // At, B, Ab
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: an SGPR
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = tile_m * 256, n0 = tile_n * 128;

  const BImg bi = bimg_make(a, BKC, n0);
  const int64_t ldb = bi.ld;
  const int64_t lda = a.lda;
  uint32_t vA[2][2], vB[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 8 + wave;
    vA[0][it] = himg_voff<AK, 32>(i, lane, lda, 0);
    vA[1][it] = himg_voff<AK, 32>(i, lane, lda, 32);
    vB[it] = himg_voff<BKC, 128>(i, lane, ldb, 0);
  }
  const int kb = kslice_begin(a, ks);
  const uint16_t* Ab0 = AK ? a.A + (int64_t)m0 * lda + kb : a.A + m0 + (int64_t)kb * lda;
  auto a_ptr = [&](int t) { return AK ? Ab0 + t * BK : Ab0 + (int64_t)t * BK * lda; };
  auto b_ptr = [&](int t) { return bimg_ptr(bi, BKC, kb + t * BK); };
  // image h (0 At, 1 B, 2 Ab) of K-tile t into buffer buf
  // DMA instruction `it` (of 2 per wave) of image h (0 At, 1 B, 2 Ab) of K-tile t into buffer buf
  auto stage1 = [&](int t, int buf, int h, int it) {
    lds_u8* dst = smem + buf * BUF + h * IMG;
    const uint16_t* base = h == 1 ? b_ptr(t) : a_ptr(t);
    const uint32_t vo = h == 1 ? vB[it] : vA[h == 2 ? 1 : 0][it];
    glds16_asm(base, vo, dst + (it * 8 + wave) * 1024);
  };
  auto stage = [&](int t, int buf, int h) {
    stage1(t, buf, h, 0);
    stage1(t, buf, h, 1);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = kslice_tiles(a);
  stage(0, 0, 0); stage(0, 0, 1); stage(0, 0, 2);
  if (nk > 1) {
    stage(1, 1, 0); stage(1, 1, 1); stage(1, 1, 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  bf16x8_t af[2][2], bf[4][2];
  auto mma = [&](int i0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i0 + i][j] = mfma16(af[i][s], bf[j][s], acc[i0 + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  const bool late = __builtin_amdgcn_readfirstlane(wm) >= 2;
  if (late) bar();

  auto ktile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    constexpr int nbuf = (buf + 2) % 3;  // K-tile t+2's buffer (freed by K-tile t-1)
    const lds_u8* sAt = smem + buf * BUF;
    const lds_u8* sB = sAt + IMG;
    const lds_u8* sAb = sAt + 2 * IMG;
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // phase 1: At rows + all B cols; stage At(t+2); upper half
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = read_frag<128, AK>(sAt, wm * 32 + i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) bf[j][s] = read_frag<128, BKC>(sB, wn * 64 + j * 16, s, lane);
    if (n2) stage(t + 2, nbuf, 0);  // (measured: moving DMA between the phases only loses)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(0);
    bar();
    // phase 2: Ab rows; stage B, Ab of t+2; retire K-tile t+1; lower half
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = read_frag<128, AK>(sAb, wm * 32 + i * 16, s, lane);
    if (n2) {
      stage(t + 2, nbuf, 1);
      stage(t + 2, nbuf, 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (n1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(2);
    bar();
  };

  int t = 0;
  for (; t + 2 < nk; t += 3) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
    ktile(t + 2, std::integral_constant<int, 2>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  if (t + 1 < nk) ktile(t + 1, std::integral_constant<int, 1>{});
  if (!late) bar();
  __syncthreads();
  float2* xs = (float2*)(smem + 8 * (TM * (TN * 2 + 16)));  // EPI_CE_STATS row statistics
  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane, xs + wave * TM,
                        (int64_t)ks * a.kpart_stride);
  if constexpr (EPI == EPI_CE_STATS) {
    __syncthreads();
    if (wn == 0) ce_stats_merge<2, TM, TN>(a, xs, m0, n0, wm, lane);
  }
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(512) void gemm_4ph_kernel(const GemmGroup g) {
  int tile_m, tile_n, ks;
  const GemmArgs& a = select_problem(g, tile_m, tile_n, ks);
  gemm_4ph_tile<AK, BKC, EPI>(a, tile_m, tile_n, ks);
}

// ================================================================ 256x128, K-halves (tile 14)
// The 4-phase kernel's tile and images with the 8-phase kernel's wave tile: the two wave groups
// (waves 0-3, 4-7) take the two k-substeps of every K-tile (k 0-31 / 32-63), and inside a group
// 2(M) x 2(N) waves each own a 128 x 64 output (8 x 4 accumulators) -- 12 LDS fragment reads per
// 32 MFMAs instead of the 4-phase kernel's 16 (64 x 64 wave tiles), the LDS read rate the 8-phase
// kernel runs at.  Images per K-tile: At / Ab = the 8-phase kernel's A half images (rows 0-63 /
// 64-127 of each M-wave's 128), B = all 128 columns; the 4-phase kernel's three-K-tile ring, phase
// anatomy, single counted wait per K-tile and wave-group stagger, unchanged.  After the K loop the
// groups swap halves through LDS: group 0 finishes rows 0-63 of each wave tile, group 1 rows
// 64-127 (each adds the other group's partial: g0 + g1 for every element), and each wave writes
// its 64 x 64 through the common epilogue.
template <bool AK, bool BKC, int EPI>
__device__ __forceinline__ void gemm_kh_tile(const GemmArgs& a, const int tile_m, const int tile_n, const int ks = 0) {
  constexpr int IMG = 128 * BK * 2;           // 16 KiB
  constexpr int BUF = 3 * IMG;                // At, B, Ab
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: an SGPR
  const int grp = wave >> 2, wm = (wave >> 1) & 1, wn = wave & 1;
  const int m0 = tile_m * 256, n0 = tile_n * 128;

  const BImg bi = bimg_make(a, BKC, n0);
  const int64_t ldb = bi.ld;
  const int64_t lda = a.lda;
  uint32_t vA[2][2], vB[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 8 + wave;
    vA[0][it] = himg_voff<AK, 64>(i, lane, lda, 0);
    vA[1][it] = himg_voff<AK, 64>(i, lane, lda, 64);
    vB[it] = himg_voff<BKC, 128>(i, lane, ldb, 0);
  }
  const int kb = kslice_begin(a, ks);
  const uint16_t* Ab0 = AK ? a.A + (int64_t)m0 * lda + kb : a.A + m0 + (int64_t)kb * lda;
  auto a_ptr = [&](int t) { return AK ? Ab0 + t * BK : Ab0 + (int64_t)t * BK * lda; };
  auto b_ptr = [&](int t) { return bimg_ptr(bi, BKC, kb + t * BK); };
  // image h (0 At, 1 B, 2 Ab) of K-tile t into buffer buf: 2 DMA instructions per wave
  auto stage = [&](int t, int buf, int h) {
    lds_u8* dst = smem + buf * BUF + h * IMG;
    const uint16_t* base = h == 1 ? b_ptr(t) : a_ptr(t);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const uint32_t vo = h == 1 ? vB[it] : vA[h == 2 ? 1 : 0][it];
      glds16_asm(base, vo, dst + (it * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = kslice_tiles(a);
  stage(0, 0, 0); stage(0, 0, 1); stage(0, 0, 2);
  if (nk > 1) {
    stage(1, 1, 0); stage(1, 1, 1); stage(1, 1, 2);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  const int s = __builtin_amdgcn_readfirstlane(grp);  // this group's k-substep
  bf16x8_t af[4], bf[4];
  auto mma = [&](int i0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i0 + i][j] = mfma16(af[i], bf[j], acc[i0 + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  const bool late = s == 1;
  if (late) bar();

  auto ktile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    constexpr int nbuf = (buf + 2) % 3;  // K-tile t+2's buffer (freed by K-tile t-1)
    const lds_u8* sAt = smem + buf * BUF;
    const lds_u8* sB = sAt + IMG;
    const lds_u8* sAb = sAt + 2 * IMG;
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // phase 1: At rows + B cols of substep s; stage At(t+2); rows 0-63 of the wave tile
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag<128, AK>(sAt, wm * 64 + i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = read_frag<128, BKC>(sB, wn * 64 + j * 16, s, lane);
    if (n2) stage(t + 2, nbuf, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(0);
    bar();
    // phase 2: Ab rows; stage B, Ab of t+2; retire K-tile t+1; rows 64-127
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag<128, AK>(sAb, wm * 64 + i * 16, s, lane);
    if (n2) {
      stage(t + 2, nbuf, 1);
      stage(t + 2, nbuf, 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (n1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(4);
    bar();
  };

  int t = 0;
  for (; t + 2 < nk; t += 3) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
    ktile(t + 2, std::integral_constant<int, 2>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  if (t + 1 < nk) ktile(t + 1, std::integral_constant<int, 1>{});
  if (!late) bar();
  __syncthreads();
  // swap halves: wave w hands the 4 x 4 fragments the partner wave (w ^ 4) finishes -- group 0 its
  // rows 64-127, group 1 its rows 0-63 -- through slot w (16 B per lane, lane-contiguous)
  typedef __attribute__((address_space(3))) f32x4_t lds_f4;
  lds_f4* slot = (lds_f4*)smem + wave * 16 * 64 + lane;
  // (constant accumulator indices in each branch: an index that depends on the group would put
  // the accumulators in scratch)
  if (s == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) slot[(i * 4 + j) * 64] = acc[4 + i][j];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) slot[(i * 4 + j) * 64] = acc[i][j];
  }
  __syncthreads();
  const lds_f4* peer = (const lds_f4*)smem + (wave ^ 4) * 16 * 64 + lane;
  f32x4_t out[4][4];
  if (s == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) out[i][j] = acc[i][j] + peer[(i * 4 + j) * 64];       // g0 + g1
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) out[i][j] = peer[(i * 4 + j) * 64] + acc[4 + i][j];   // g0 + g1
  }
  __syncthreads();
  // the wave's 64 x 64 output: tile rows wm * 128 + s * 64 .., columns wn * 64 ..
  epilogue<64, 64, EPI>(a, out, smem + wave * (64 * (64 * 2 + 16)), m0, n0, wm * 2 + s, wn, lane, nullptr,
                        (int64_t)ks * a.kpart_stride);
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(512) void gemm_kh_kernel(const GemmGroup g) {
  int tile_m, tile_n, ks;
  const GemmArgs& a = select_problem(g, tile_m, tile_n, ks);
  gemm_kh_tile<AK, BKC, EPI>(a, tile_m, tile_n, ks);
}

// ================================================================ 128x128, k-substep groups (tile 15)
// For the few-tile problems of the TP shards (TP = 8 at SmolLM-1.7B: q|k|v 4096 x 768, o_proj
// 4096 x 256, the weight gradients 768 x 2048 / 2048 x 2048 at K 4096): a 128x128 tile puts four
// times the 256x256 kernel's workgroups on the 256 CUs at the same K, so the launch fills the chip
// without K-slices and their f32 partial round trip.  8 waves: the two wave groups (waves 0-3, 4-7)
// take the two k-substeps of every K-tile (k 0-31 / 32-63), and inside a group 2(M) x 2(N) waves own
// a 64 x 64 output (4 x 4 accumulators): 8 LDS fragment reads per 16 MFMAs, the 4-phase kernel's
// ratio.  Per K-tile the images A (128 rows x 64 k) and B (128 columns x 64 k), 32 KiB, in a 4-deep
// ring (128 KiB: one workgroup per CU): K-tile t + 3 is staged during K-tile t into the buffer
// K-tile t - 1 freed, and the one counted wait per K-tile retires t + 1 with t + 2 and t + 3 in
// flight.  One phase per K-tile { reads; DMA; waits; barrier; 16 MFMAs; barrier } with group 1 one
// barrier behind (its reads beside group 0's MFMAs on every SIMD, and vice versa).  After the loop
// the groups swap halves through LDS as tile 14 does: group 0 finishes rows 0-31 of each wave tile,
// group 1 rows 32-63 (g0 + g1 for every element), through the common epilogue.
template <bool AK, bool BKC, int EPI>
__device__ __forceinline__ void gemm_hq_tile(const GemmArgs& a, const int tile_m, const int tile_n, const int ks = 0) {
  constexpr int IMG = 128 * BK * 2;           // 16 KiB
  constexpr int BUF = 2 * IMG;                // A, B
  constexpr int NS = 4;                       // ring depth (K-tiles resident)
  constexpr int OPS = 4;                      // DMA instructions per wave and K-tile
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: an SGPR
  const int grp = wave >> 2, wm = (wave >> 1) & 1, wn = wave & 1;
  const int m0 = tile_m * 128, n0 = tile_n * 128;

  const BImg bi = bimg_make(a, BKC, n0);
  const int64_t ldb = bi.ld;
  const int64_t lda = a.lda;
  uint32_t vA[2], vB[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 8 + wave;
    vA[it] = himg_voff<AK, 128>(i, lane, lda, 0);
    vB[it] = himg_voff<BKC, 128>(i, lane, ldb, 0);
  }
  const int kb = kslice_begin(a, ks);
  const uint16_t* Ab0 = AK ? a.A + (int64_t)m0 * lda + kb : a.A + m0 + (int64_t)kb * lda;
  auto a_ptr = [&](int t) { return AK ? Ab0 + t * BK : Ab0 + (int64_t)t * BK * lda; };
  auto b_ptr = [&](int t) { return bimg_ptr(bi, BKC, kb + t * BK); };
  // K-tile t's two images into buffer buf: OPS = 4 DMA instructions per wave
  auto stage = [&](int t, int buf) {
    lds_u8* dst = smem + buf * BUF;
    const uint16_t* ap = a_ptr(t);
    const uint16_t* bp = b_ptr(t);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      glds16_asm(ap, vA[it], dst + (it * 8 + wave) * 1024);
      glds16_asm(bp, vB[it], dst + IMG + (it * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = kslice_tiles(a);
  const int pre = nk < NS - 1 ? nk : NS - 1;
  for (int t = 0; t < pre; ++t) stage(t, t);
  // K-tile 0 landed; the ones after it stay in flight
  if (pre >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (pre == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  const int s = __builtin_amdgcn_readfirstlane(grp);  // this group's k-substep
  const bool late = s == 1;
  if (late) bar();
  bf16x8_t af[4], bf[4];

  auto ktile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    const lds_u8* sA = smem + buf * BUF;
    const lds_u8* sB = sA + IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag<128, AK>(sA, wm * 64 + i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = read_frag<128, BKC>(sB, wn * 64 + j * 16, s, lane);
    // K-tile t + 3 into the buffer K-tile t - 1 used (every wave's reads of it retired before the
    // barrier that ended its phase)
    const int tn = t + NS - 1;
    if (tn < nk) stage(tn, (buf + NS - 1) % NS);
    // K-tile t + 1 must have landed before the next phase's reads: the younger K-tiles in flight
    // (issued so far, after t + 1) may stay
    const int issued = tn < nk ? tn : nk - 1;
    const int younger = issued - (t + 1);
    if (t + 1 < nk) {
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };

  int t = 0;
  for (; t + 3 < nk; t += 4) {
    ktile(t, std::integral_constant<int, 0>{});
    ktile(t + 1, std::integral_constant<int, 1>{});
    ktile(t + 2, std::integral_constant<int, 2>{});
    ktile(t + 3, std::integral_constant<int, 3>{});
  }
  if (t < nk) ktile(t, std::integral_constant<int, 0>{});
  if (t + 1 < nk) ktile(t + 1, std::integral_constant<int, 1>{});
  if (t + 2 < nk) ktile(t + 2, std::integral_constant<int, 2>{});
  if (!late) bar();
  __syncthreads();
  // swap halves: wave w hands the 2 x 4 fragments its partner (w ^ 4) finishes -- group 0 its rows
  // 32-63, group 1 its rows 0-31 -- through slot w (16 B per lane, lane-contiguous)
  typedef __attribute__((address_space(3))) f32x4_t lds_f4;
  lds_f4* slot = (lds_f4*)smem + wave * 8 * 64 + lane;
  if (s == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) slot[(i * 4 + j) * 64] = acc[2 + i][j];
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) slot[(i * 4 + j) * 64] = acc[i][j];
  }
  __syncthreads();
  const lds_f4* peer = (const lds_f4*)smem + (wave ^ 4) * 8 * 64 + lane;
  f32x4_t out[2][4];
  if (s == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) out[i][j] = acc[i][j] + peer[(i * 4 + j) * 64];       // g0 + g1
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) out[i][j] = peer[(i * 4 + j) * 64] + acc[2 + i][j];   // g0 + g1
  }
  __syncthreads();
  // the wave's 32 x 64 output: tile rows wm * 64 + s * 32 .., columns wn * 64 ..
  epilogue<32, 64, EPI>(a, out, smem + wave * (32 * (64 * 2 + 16)), m0, n0, wm * 2 + s, wn, lane, nullptr,
                        (int64_t)ks * a.kpart_stride);
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(512) void gemm_hq_kernel(const GemmGroup g) {
  int tile_m, tile_n, ks;
  const GemmArgs& a = select_problem(g, tile_m, tile_n, ks);
  gemm_hq_tile<AK, BKC, EPI>(a, tile_m, tile_n, ks);
}

// ------------------------------------------------------------------- mixed-tile launch (q|k|v)
// One problem whose output columns [0, n_split) are covered by 256x256 8-phase tiles and
// [n_split, N) by 256x128 4-phase tiles, in ONE launch.  For the q|k|v projection with RoPE
// (q|k = 2/3 of the columns at H = HKV): 768 tiles of 256x128 are 3 rounds of the 256 CUs; 256
// tiles of 256x256 over q|k plus 256 tiles of 256x128 over v are 2 rounds, the 4-phase tiles
// filling CUs as the 8-phase ones finish.  Tile order as the dual launch: each XCD takes an equal
// contiguous share of each part, 8-phase tiles first; inside a part the usual grouped raster.
struct MixMap {
  DualMap d;                  // n0 / n1 = tiles per XCD of the 8-phase / 4-phase part
  int tiles_m, tn0, tn1;      // tile grid of each part
  int nsplit_t1;              // n_split / 128: the 4-phase part's first tile column
};

__device__ __forceinline__ void grouped_tile(int pid, int tiles_m, int tiles_n, int group, int& tm, int& tn) {
  const int span = group * tiles_n, gid = pid / span, first = gid * group;
  const int gsize = min(tiles_m - first, group);
  tm = first + (pid % span) % gsize;
  tn = (pid % span) / gsize;
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(512) void gemm_mix_kernel(const GemmArgs a, const MixMap m) {
  int pid, tile_m, tile_n;
  if (dual_select(m.d, pid) == 0) {
    grouped_tile(pid, m.tiles_m, m.tn0, 8, tile_m, tile_n);
    gemm_8ph_tile<AK, BKC, EPI>(a, tile_m, tile_n);
  } else {
    grouped_tile(pid, m.tiles_m, m.tn1, 4, tile_m, tile_n);
    gemm_4ph_tile<AK, BKC, EPI>(a, tile_m, m.nsplit_t1 + tile_n);
  }
}

// ================================================================================= simple
template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, int SCHED>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(const GemmGroup g) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: an SGPR
  const int wm = wave / WN, wn = wave % WN;
  int tile_m, tile_n, ks;
  const GemmArgs& a = select_problem(g, tile_m, tile_n, ks);
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kb = kslice_begin(a, ks);
  const uint16_t* Abase = AK ? a.A + (int64_t)m0 * a.lda + kb : a.A + m0 + (int64_t)kb * a.lda;

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const BImg bi = bimg_make(a, BKC, n0);
  const int64_t lda = a.lda;
  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BK;
    lds_u8* sa = smem + buf * STAGE_BYTES;
    lds_u8* sb = sa + A_BYTES;
    const uint16_t* ga = AK ? Abase + k0 : Abase + (int64_t)k0 * lda;
    stage_tile<BM, AK, NT>(ga, lda, sa, tid);
    stage_tile<BN, BKC, NT>(bimg_ptr(bi, BKC, kb + k0), bi.ld, sb, tid);
  };

  const int nk = kslice_tiles(a);
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const lds_u8* sa = smem + buf * STAGE_BYTES;
    const lds_u8* sb = sa + A_BYTES;
    if (SCHED == 0) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8_t af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, AK>(sa, wm * TM + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, BKC>(sb, wn * TN + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    } else {
      // both k-substeps' fragments in flight at once (two register sets, B first so the first
      // MFMA row can start after FN + 1 reads), MFMAs in one prioritised cluster, raw barrier
      bf16x8_t a0[FM], b0[FN], a1[FM], b1[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) b0[j] = read_frag<BN, BKC>(sb, wn * TN + j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) a0[i] = read_frag<BM, AK>(sa, wm * TM + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) b1[j] = read_frag<BN, BKC>(sb, wn * TN + j * 16, 1, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) a1[i] = read_frag<BM, AK>(sa, wm * TM + i * 16, 1, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane, nullptr,
                        (int64_t)ks * a.kpart_stride);
}

// ================================================================================== launch
template <typename Kern>
void set_smem_once(Kern k, int smem) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
}

// per-problem tile grid + consecutive tile ids; returns the total tile count
// tile-rows per group of the tile order: 6 for both phased tiles.  Whole-step A/B (round 4,
// profiles/r04/group_m/, two boxes, interleaved): 6 -> 156.6-157.5 k, 5 / 7 -> 156.2-157.8 k,
// 4 -> 155.4-155.9 k, the previous 8 (256x256) / 4 (256x128) -> 154.9-155.0 k tokens/s
// (the A/B variant that overrode it is retired: every other count measured slower)
// round 6 (weight-gradient pairing on), same box, 2 interleaved rounds (profiles/r06/notes_r06.md):
// 6 -> 164.7 / 165.4 k, 4 -> 165.4 / 165.0 k, 8 -> 163.7 / 164.0 k.  -DPT_GROUP_M=n builds the A/B form.
#ifndef PT_GROUP_M
#define PT_GROUP_M 6
#endif
int group_m_for(int bm, int bn) {
  (void)bm; (void)bn;
  return PT_GROUP_M;
}

inline int group_tiles(GemmGroup& g, int bm, int bn) {
  int n = 0;
  const int gm = group_m_for(bm, bn);
  for (int i = 0; i < g.nprob; ++i) {
    g.p[i].tiles_m = g.p[i].M / bm;
    g.p[i].tiles_n = g.p[i].N / bn;
    g.p[i].group_m = gm;
    g.start[i] = n;
    n += g.p[i].tiles_m * g.p[i].tiles_n * (g.p[i].ksplit > 1 ? g.p[i].ksplit : 1);
  }
  for (int i = g.nprob; i <= kMaxProb; ++i) g.start[i] = n;
  return n;
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, int SCHED = 0>
int launch_t(GemmGroup g, hipStream_t stream) {
  const int tiles = group_tiles(g, BM, BN);
  constexpr int smem_main = 2 * (BM + BN) * BK * 2;
  constexpr int smem_epi = WM * WN * (BM / WM) * ((BN / WN) * 2 + 16);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_kernel<BM, BN, WM, WN, AK, BKC, EPI, SCHED>, smem);
    attr_set = true;
  }
  gemm_kernel<BM, BN, WM, WN, AK, BKC, EPI, SCHED><<<tiles, WM * WN * 64, smem, stream>>>(g);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_8ph(GemmGroup g, hipStream_t stream) {
  const int tiles = group_tiles(g, 256, EPI == EPI_SWIGLU_FWD ? 128 : 256);
  constexpr int smem_main = 8 * 128 * BK * 2;
  constexpr int smem_epi = 8 * 128 * (64 * 2 + 16) + (EPI == EPI_CE_STATS ? 8 * 128 * 8 : 0);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_8ph_kernel<AK, BKC, EPI>, smem);
    attr_set = true;
  }
  gemm_8ph_kernel<AK, BKC, EPI><<<tiles, 512, smem, stream>>>(g);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK0, bool BKC0, int EPI0, bool AK1, bool BKC1, int EPI1>
int launch_dual_t(GemmGroup g0, GemmGroup g1, int order, hipStream_t stream) {
  const int t0 = group_tiles(g0, 256, 256), t1 = group_tiles(g1, 256, 256);  // (x ksplit)
  if (t0 % 8 || t1 % 8) return PT_EUNSUPPORTED;  // equal per-XCD shares of both groups
  const DualMap m{t0 / 8, t1 / 8, order};
  constexpr int smem = 8 * 128 * (64 * 2 + 16);  // epilogue staging (> the 128 KiB main loop)
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_8ph_dual_kernel<AK0, BKC0, EPI0, AK1, BKC1, EPI1>, smem);
    attr_set = true;
  }
  gemm_8ph_dual_kernel<AK0, BKC0, EPI0, AK1, BKC1, EPI1><<<t0 + t1, 512, smem, stream>>>(g0, g1, m);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_4ph(GemmGroup g, hipStream_t stream) {
  const int tiles = group_tiles(g, 256, 128);
  constexpr int smem_main = 9 * 128 * BK * 2;
  constexpr int smem_epi = 8 * 64 * (64 * 2 + 16) + (EPI == EPI_CE_STATS ? 8 * 64 * 8 : 0);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_4ph_kernel<AK, BKC, EPI>, smem);
    attr_set = true;
  }
  gemm_4ph_kernel<AK, BKC, EPI><<<tiles, 512, smem, stream>>>(g);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_kh(GemmGroup g, hipStream_t stream) {
  static_assert(EPI != EPI_CE_STATS && EPI != EPI_SWIGLU_FWD && EPI != EPI_SWIGLU_BWD, "tile 14 epilogues");
  const int tiles = group_tiles(g, 256, 128);
  constexpr int smem = 9 * 128 * BK * 2;  // 144 KiB: the ring; the half swap (128 KiB) and staging fit
  static_assert(8 * 16 * 64 * 16 <= smem && 8 * 64 * (64 * 2 + 16) <= smem && smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_kh_kernel<AK, BKC, EPI>, smem);
    attr_set = true;
  }
  gemm_kh_kernel<AK, BKC, EPI><<<tiles, 512, smem, stream>>>(g);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_hq(GemmGroup g, hipStream_t stream) {
  static_assert(EPI != EPI_CE_STATS && EPI != EPI_SWIGLU_FWD && EPI != EPI_SWIGLU_BWD && EPI != EPI_ROPE,
                "tile 15 epilogues");
  const int tiles = group_tiles(g, 128, 128);
  constexpr int smem = 4 * 2 * 128 * BK * 2;  // 128 KiB: the ring; the half swap (64 KiB) and staging fit
  static_assert(8 * 8 * 64 * 16 <= smem && 8 * 32 * (64 * 2 + 16) <= smem && smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_hq_kernel<AK, BKC, EPI>, smem);
    attr_set = true;
  }
  gemm_hq_kernel<AK, BKC, EPI><<<tiles, 512, smem, stream>>>(g);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// tile ids: 2 = simple 128x128, 3 = simple 64x64 (the TP shards' few-tile problems),
//           12 = 8-phase 256x256 (two half-image wave groups, one wait per K-tile)
//           13 = 4-phase 256x128 (three K-tiles resident)
//           14 = 256x128 with the K-tile's two k-substeps over two wave groups (128 x 64 wave tiles)
//           15 = 128x128 with the K-tile's two k-substeps over two wave groups (64 x 64 wave tiles,
//                a 4-deep ring): the TP shards' few-tile problems
//           (ids 4, 5, 8, 9 -- the simple 256x256 / 256x128 kernels and their two-substep forms --
//           were never picked once the phased kernels existed, and the 256x256 ones spilled: dropped
//           from the library in round 4; ids 0, 1, 6, 7, 10, 11 were pipelining experiments, measured slower and retired; so
//           was round 2's 14: the 8-phase tile with ONE barrier per K-tile and free-running
//           phases, 3-13 % slower on every layer shape -- the per-phase ping-pong pays for its
//           barriers)
constexpr int kNumTiles = 16;
const int kTileBM[kNumTiles] = {0, 0, 128, 64, 0, 0, 0, 0, 0, 0, 0, 0, 256, 256, 256, 128};
const int kTileBN[kNumTiles] = {0, 0, 128, 64, 0, 0, 0, 0, 0, 0, 0, 0, 256, 128, 128, 128};

template <bool AK, bool BKC, int EPI>
int launch_layout(const GemmGroup& a, int tile, hipStream_t s) {
  if constexpr (!AK && BKC) {  // A M-contiguous with B K-contiguous: no layer GEMM takes this layout,
    switch (tile) {            // so only the simple tiles are built for it (pick_group_tile knows)
      case 2: return launch_t<128, 128, 2, 2, AK, BKC, EPI>(a, s);
      case 3: return launch_t<64, 64, 2, 2, AK, BKC, EPI>(a, s);
      default: return PT_EUNSUPPORTED;
    }
  } else {
    switch (tile) {
      case 12: return launch_8ph<AK, BKC, EPI>(a, s);
      case 13: return launch_4ph<AK, BKC, EPI>(a, s);
      case 14: return launch_kh<AK, BKC, EPI>(a, s);
      case 15: return launch_hq<AK, BKC, EPI>(a, s);
      case 2: return launch_t<128, 128, 2, 2, AK, BKC, EPI>(a, s);
      case 3: return launch_t<64, 64, 2, 2, AK, BKC, EPI>(a, s);
      default: return PT_EUNSUPPORTED;
    }
  }
}

template <int EPI>
int launch_epi(const GemmGroup& a, int a_kcontig, int b_kcontig, int tile, hipStream_t s) {
  if (a_kcontig && b_kcontig) return launch_layout<true, true, EPI>(a, tile, s);
  if (a_kcontig && !b_kcontig) return launch_layout<true, false, EPI>(a, tile, s);
  if (!a_kcontig && !b_kcontig) return launch_layout<false, false, EPI>(a, tile, s);
  return launch_layout<false, true, EPI>(a, tile, s);
}

}  // namespace

namespace {

// split-K fields of a grouped problem: ksplit slices of K / ksplit (a multiple of BK) written as f32
// partials kpart_stride elements apart (EPI_F32 only).
int fill_split(GemmArgs& a, const pt_gemm_problem& q, int epilogue) {
  a.A2 = nullptr;
  a.ak2 = INT32_MAX;
  if (q.A2) {   // A K-segmented at a_k2 (a BK multiple inside K; A2 aligned like A)
    if (q.a_k2 <= 0 || q.a_k2 >= a.K || q.a_k2 % BK) return PT_EINVAL;
    if (!pt_aligned16(q.A2)) return PT_EALIGN;
    a.A2 = (const uint16_t*)q.A2;
    a.ak2 = (int)q.a_k2;
  }
  a.ksplit = q.ksplit > 1 ? q.ksplit : 1;
  a.kpart_stride = q.kpart_stride;
  if (a.ksplit == 1) return PT_OK;
  if (epilogue != EPI_F32 || q.kpart_stride <= 0 || a.ksplit > 64) return PT_EINVAL;
  if (a.K % (a.ksplit * BK)) return PT_EUNSUPPORTED;
  if (a.bdim == 1)  // a K-tile never straddles a K-segment boundary (segments are BK multiples)
    for (int i = 0; i <= a.nbseg; ++i)
      if (a.bseg[i] % BK) return PT_EUNSUPPORTED;
  return PT_OK;
}

// Validate one problem and fill its kernel arguments.  Returns PT_OK or a PT_E* code.
int fill_args(GemmArgs& a, const void* A, int64_t lda, const void* const* B, const int64_t* ldb,
              const int64_t* b_bounds, int nb, int b_seg_dim, void* const* C, const int64_t* ldc,
              const int64_t* c_bounds, int nc, int64_t M, int64_t N, int64_t K, int epilogue, const void* residual,
              int64_t ldr) {
  if (!A || !B || !C || nb < 1 || nb > 4 || nc < 1 || nc > 4 || M <= 0 || N <= 0 || K <= 0) return PT_EINVAL;
  if (epilogue == EPI_BF16_RES && (!residual || nc != 1 || !pt_aligned16(residual) || (ldr & 7))) return PT_EINVAL;
  if (epilogue == EPI_SWIGLU_FWD) {
    // B = {W_gate, W_up} ([N/2, K] each, same ld), C = {h [M, N/2], g|u [M, N]}; N = 2 I
    if (nb != 2 || b_seg_dim != 0 || nc != 2 || (N & 1) || ldb[0] != ldb[1]) return PT_EINVAL;
    if (b_bounds && (b_bounds[0] != 0 || b_bounds[1] != N / 2 || b_bounds[2] != N)) return PT_EINVAL;
    a = GemmArgs{};
    a.A = (const uint16_t*)A;
    a.lda = lda;
    a.nbseg = 2;
    for (int i = 0; i < 2; ++i) {
      if (!B[i] || !pt_aligned16(B[i]) || (ldb[i] & 7) || !C[i] || !pt_aligned16(C[i]) || (ldc[i] & 7))
        return PT_EALIGN;
      a.B[i] = (const uint16_t*)B[i];
      a.ldb[i] = ldb[i];
      a.C[i] = C[i];
      a.ldc[i] = ldc[i];
    }
    a.bseg[1] = N / 2;
    for (int i = 2; i < 5; ++i) a.bseg[i] = N;
    a.ncseg = 1;
    for (int i = 1; i < 5; ++i) a.cseg[i] = M;
    if (!pt_aligned16(A) || (lda & 7) || K % BK) return PT_EALIGN;
    a.M = (int)M;
    a.N = (int)(N / 2);  // h columns; the tile grid is 256 x 128 of h
    a.K = (int)K;
    return PT_OK;
  }
  if (epilogue == EPI_SWIGLU_BWD && (!residual || nc != 1 || !pt_aligned16(residual) || (ldr & 7) || (ldc[0] & 7)))
    return PT_EINVAL;
  if (K % BK) return PT_EUNSUPPORTED;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return PT_EUNSUPPORTED;
  a = GemmArgs{};
  a.A = (const uint16_t*)A;
  a.lda = lda;
  a.nbseg = nb;
  a.bdim = b_seg_dim;
  for (int i = 0; i < nb; ++i) {
    if (!B[i] || !pt_aligned16(B[i]) || (ldb[i] & 7)) return PT_EALIGN;
    a.B[i] = (const uint16_t*)B[i];
    a.ldb[i] = ldb[i];
  }
  for (int i = 0; i <= nb; ++i) a.bseg[i] = b_bounds ? b_bounds[i] : (i == 0 ? 0 : (b_seg_dim ? K : N));
  if (a.bseg[0] != 0 || a.bseg[nb] != (b_seg_dim ? K : N)) return PT_EINVAL;
  a.ncseg = nc;
  for (int i = 0; i < nc; ++i) {
    if (!C[i] || !pt_aligned16(C[i])) return PT_EALIGN;
    a.C[i] = C[i];
    a.ldc[i] = ldc[i];
  }
  for (int i = 0; i <= nc; ++i) a.cseg[i] = c_bounds ? c_bounds[i] : (i == 0 ? 0 : M);
  if (a.cseg[0] != 0 || a.cseg[nc] != M) return PT_EINVAL;
  for (int i = nc + 1; i < 5; ++i) a.cseg[i] = M;
  for (int i = nb + 1; i < 5; ++i) a.bseg[i] = b_seg_dim ? K : N;
  if (!pt_aligned16(A) || (lda & 7)) return PT_EALIGN;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.R = (const uint16_t*)residual;
  a.ldr = ldr;
  if (b_seg_dim == 1)  // K-segment boundaries must be multiples of BK
    for (int i = 0; i <= nb; ++i)
      if (a.bseg[i] % BK) return PT_EUNSUPPORTED;
  return PT_OK;
}

bool args_fit(const GemmArgs& a, int tile) {
  if (tile < 0 || tile >= kNumTiles || kTileBM[tile] == 0) return false;
  const int bm = kTileBM[tile], bn = kTileBN[tile];
  if (a.M % bm || a.N % bn) return false;
  for (int i = 0; i <= a.ncseg; ++i)
    if (a.cseg[i] % bm) return false;
  if (a.bdim == 0)
    for (int i = 0; i <= a.nbseg; ++i)
      if (a.bseg[i] % bn) return false;
  if (tile >= 12 && a.bdim == 1)  // the phased kernels keep one B ld per tile
    for (int i = 1; i < a.nbseg; ++i)
      if (a.ldb[i] != a.ldb[0]) return false;
  return true;
}

// auto tile for a group.  The phased kernels (256x256 8-phase, 256x128 4-phase), whichever fills the
// CUs' last round better (ties -> 256x256), as long as that puts at least 128 tiles on the 256 CUs:
// on the SmolLM-1.7B / Llama-2-7B TP=1 shapes they measure fastest (profiles/r01_gemm_tiles_8ph.md).
// Below that -- the TP shards (N 256-1024 at TP=8: 24-96 phased tiles) -- the candidate with the
// smallest modelled time, rounds x tile work / the kernel's sustained rate (one CU per workgroup:
// ceil(tiles / 256) rounds; in-situ TF/s 1.30 / 1.20 / 0.85 / 0.45 for 256x256 / 256x128 / 128x128
// / 64x64), which trades the phased kernels' rate for the smaller tiles' parallelism.
int pick_group_tile(const GemmGroup& g, bool simple_only = false) {
  auto fits = [&](int t) {
    for (int i = 0; i < g.nprob; ++i)
      if (!args_fit(g.p[i], t)) return false;
    return true;
  };
  auto ntiles = [&](int t) {
    int64_t tiles = 0;
    for (int i = 0; i < g.nprob; ++i)
      tiles += (int64_t)(g.p[i].M / kTileBM[t]) * (g.p[i].N / kTileBN[t]) * (g.p[i].ksplit > 1 ? g.p[i].ksplit : 1);
    return tiles;
  };
  auto fill = [&](int t) {
    const int64_t tiles = ntiles(t);
    return (double)tiles / (double)(((tiles + 255) / 256) * 256);
  };
  const bool f12 = !simple_only && fits(12), f13 = !simple_only && fits(13);
  const int phased = f12 && (!f13 || fill(12) >= fill(13)) ? 12 : (f13 ? 13 : -1);
  if (phased >= 0 && ntiles(phased) >= 128) return phased;
  const int cand[4] = {12, 13, 2, 3};
  const double rate[4] = {1.30, 1.20, 0.85, 0.45};
  int best = -1;
  double best_cost = 0.0;
  for (int i = simple_only ? 2 : 0; i < 4; ++i) {
    if (!fits(cand[i])) continue;
    const double c = (double)((ntiles(cand[i]) + 255) / 256) * kTileBM[cand[i]] * kTileBN[cand[i]] / rate[i];
    if (best < 0 || c < best_cost) best = cand[i], best_cost = c;
  }
  return best;
}

int launch_swiglu(GemmGroup& g, int a_kcontig, int b_kcontig, int epilogue, int tile, hipStream_t stream);

// variant "gemm_mix" = 0 turns the mixed-tile q|k|v launch off (A/B measurement only)
bool mix_enabled() { return pt_variant(PT_VAR_GEMM_MIX) == 1; }
// variant "gemm_kh": where the auto pick chose 256x128 tiles, tile 14 (K-halves) instead of 13 --
// 2 (default): when every problem's K (per split slice) is >= 4096, 1: always, 0: never.  Measured
// (tools/gemm_bench.py, profiles/r04/notes_r04.md): +2-11 % at K 4096-49152 (down_proj forward
// 1309 vs 1253 TF/s), equal or -4.5 % at K 2048 (o_proj forward / dX), where the half swap
// through LDS is a larger share of a short K loop.
bool kh_enabled(const GemmGroup& g) {
  // 0: never (A/B); otherwise (2, default) the K >= 4096 rule -- "always" (1) measured equal to it at
  // the step (profiles/r04/notes_r04.md) and was retired
  if (pt_variant(PT_VAR_GEMM_KH) == 0) return false;
  for (int i = 0; i < g.nprob; ++i)
    if (g.p[i].K / (g.p[i].ksplit > 1 ? g.p[i].ksplit : 1) < 4096) return false;
  return true;
}

// q|k|v + RoPE as one mixed-tile launch: the rotated columns [0, rope_cols) in 256x256 tiles, the
// rest (v) in 256x128 tiles.  PT_EUNSUPPORTED when the shape does not split that way (the caller
// then launches one tile shape as before).
int launch_mix_rope(const GemmArgs& a0, hipStream_t stream) {
  const int ns = a0.rope_cols;
  if (ns <= 0 || ns >= a0.N || ns % 256 || (a0.N - ns) % 128) return PT_EUNSUPPORTED;
  if (!args_fit(a0, 12) || !args_fit(a0, 13)) return PT_EUNSUPPORTED;
  MixMap m{};
  m.tiles_m = a0.M / 256;
  m.tn0 = ns / 256;
  m.tn1 = (a0.N - ns) / 128;
  m.nsplit_t1 = ns / 128;
  const int t0 = m.tiles_m * m.tn0, t1 = m.tiles_m * m.tn1;
  // the two parts must each divide over the 8 XCDs; the 8-phase part at most one round: the gain is
  // the round quantization (SmolLM-1.7B: 3 rounds -> 2, +0.8 % step); Llama-2-7B's 512 + 512 tiles
  // (6 whole rounds either way) measured neutral, the CP=8 proxy's 4096 + 4096 within noise
  if (t0 % 8 || t1 % 8 || t0 > 256) return PT_EUNSUPPORTED;
  m.d = DualMap{t0 / 8, t1 / 8, 0};
  GemmArgs a = a0;
  constexpr int smem = 8 * 128 * (64 * 2 + 16);  // = the 4-phase main loop's 144 KiB
  static_assert(smem >= 9 * 128 * BK * 2 && smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_mix_kernel<true, true, EPI_ROPE>, smem);
    attr_set = true;
  }
  gemm_mix_kernel<true, true, EPI_ROPE><<<t0 + t1, 512, smem, stream>>>(a, m);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

int launch_group(GemmGroup& g, int a_kcontig, int b_kcontig, int epilogue, int tile, hipStream_t stream) {
  if (epilogue == EPI_SWIGLU_FWD || epilogue == EPI_SWIGLU_BWD)
    return launch_swiglu(g, a_kcontig, b_kcontig, epilogue, tile, stream);
  // RoPE: wave tiles 64 columns wide, the phased kernels only; the 256x128 one (twice the tiles) when
  // it divides -- the q|k|v projection never fills more than a few rounds of 256x256 tiles
  if (epilogue == EPI_ROPE && tile < 0 && a_kcontig && b_kcontig && g.nprob == 1 && mix_enabled()) {
    const int rc = launch_mix_rope(g.p[0], stream);
    if (rc != PT_EUNSUPPORTED) return rc;
  }
  const bool auto_tile = tile < 0;
  if (epilogue == EPI_ROPE && tile < 0) tile = args_fit(g.p[0], 13) ? 13 : 12;
  if (tile < 0) tile = pick_group_tile(g, !a_kcontig && b_kcontig);
  if (auto_tile && tile == 13 && kh_enabled(g) && epilogue != EPI_CE_STATS) tile = 14;
  if (epilogue == EPI_ROPE) {
    if (!a_kcontig || !b_kcontig) return PT_EUNSUPPORTED;
    for (int i = 0; i < g.nprob; ++i)
      if (!args_fit(g.p[i], tile)) return PT_EUNSUPPORTED;
    if (tile == 12) return launch_8ph<true, true, EPI_ROPE>(g, stream);
    if (tile == 13) return launch_4ph<true, true, EPI_ROPE>(g, stream);
    if (tile == 14) return launch_kh<true, true, EPI_ROPE>(g, stream);
    return PT_EUNSUPPORTED;
  }
  for (int i = 0; i < g.nprob; ++i)
    if (!args_fit(g.p[i], tile) || (g.p[i].A2 && tile != 12)) return PT_EUNSUPPORTED;
  switch (epilogue) {
    case EPI_BF16: return launch_epi<EPI_BF16>(g, a_kcontig, b_kcontig, tile, stream);
    case EPI_BF16_ACC: return launch_epi<EPI_BF16_ACC>(g, a_kcontig, b_kcontig, tile, stream);
    case EPI_F32: return launch_epi<EPI_F32>(g, a_kcontig, b_kcontig, tile, stream);
    case EPI_F32_ACC: return launch_epi<EPI_F32_ACC>(g, a_kcontig, b_kcontig, tile, stream);
    case EPI_BF16_RES:  // forward projections only (weights K-contiguous)
      if (!a_kcontig || !b_kcontig) return PT_EUNSUPPORTED;
      return launch_layout<true, true, EPI_BF16_RES>(g, tile, stream);
    case EPI_CE_STATS:  // the lm_head forward: the phased kernels (64-column wave tiles)
      if (!a_kcontig || !b_kcontig) return PT_EUNSUPPORTED;
      if (tile == 12) return launch_8ph<true, true, EPI_CE_STATS>(g, stream);
      if (tile == 13) return launch_4ph<true, true, EPI_CE_STATS>(g, stream);
      return PT_EUNSUPPORTED;
    default: return PT_EINVAL;
  }
}

// the SwiGLU-fused projections: 8-phase kernel only (tile 12)
int launch_swiglu(GemmGroup& g, int a_kcontig, int b_kcontig, int epilogue, int tile, hipStream_t stream) {
  if (tile != -1 && tile != 12) return PT_EUNSUPPORTED;
  for (int i = 0; i < g.nprob; ++i) {
    const GemmArgs& a = g.p[i];
    if (a.M % 256 || a.N % (epilogue == EPI_SWIGLU_FWD ? 128 : 256)) return PT_EUNSUPPORTED;
    if (epilogue == EPI_SWIGLU_BWD && (a.ncseg != 1 || a.bdim != 0 || a.nbseg != 1)) return PT_EUNSUPPORTED;
  }
  if (epilogue == EPI_SWIGLU_FWD) {
    if (!a_kcontig || !b_kcontig) return PT_EUNSUPPORTED;
    return launch_8ph<true, true, EPI_SWIGLU_FWD>(g, stream);
  }
  if (!a_kcontig || b_kcontig) return PT_EUNSUPPORTED;
  return launch_8ph<true, false, EPI_SWIGLU_BWD>(g, stream);
}

// group 0: dX (A = dY K-contiguous, B = W N-contiguous) with EPI_BF16 or EPI_SWIGLU_BWD;
// group 1: wgrad (dY^T X: both operands MN-contiguous) into a bf16 / bf16-accumulate / f32-accumulate sink
template <int EPI0>
int launch_dual_e1(GemmGroup& g0, GemmGroup& g1, int e1, int order, hipStream_t s) {
  switch (e1) {
    case EPI_BF16: return launch_dual_t<true, false, EPI0, false, false, EPI_BF16>(g0, g1, order, s);
    case EPI_BF16_ACC: return launch_dual_t<true, false, EPI0, false, false, EPI_BF16_ACC>(g0, g1, order, s);
    case EPI_F32_ACC: return launch_dual_t<true, false, EPI0, false, false, EPI_F32_ACC>(g0, g1, order, s);
    case EPI_F32: return launch_dual_t<true, false, EPI0, false, false, EPI_F32>(g0, g1, order, s);  // split-K dW
    default: return PT_EUNSUPPORTED;
  }
}

int launch_dual(GemmGroup& g0, int ak0, int bk0, int e0, GemmGroup& g1, int ak1, int bk1, int e1, int order,
                hipStream_t s) {
  if (!ak0 || bk0 || ak1 || bk1 || order < 0 || order > 2) return PT_EUNSUPPORTED;
  for (int i = 0; i < g0.nprob; ++i) {
    if (!args_fit(g0.p[i], 12)) return PT_EUNSUPPORTED;
    if (e0 == EPI_SWIGLU_BWD && (g0.p[i].ncseg != 1 || g0.p[i].bdim != 0 || g0.p[i].nbseg != 1)) return PT_EUNSUPPORTED;
  }
  for (int i = 0; i < g1.nprob; ++i)
    if (!args_fit(g1.p[i], 12)) return PT_EUNSUPPORTED;
  if (e0 == EPI_BF16) return launch_dual_e1<EPI_BF16>(g0, g1, e1, order, s);
  if (e0 == EPI_SWIGLU_BWD) return launch_dual_e1<EPI_SWIGLU_BWD>(g0, g1, e1, order, s);
  if (e0 == EPI_F32) return launch_dual_e1<EPI_F32>(g0, g1, e1, order, s);  // split-K dX halves
  return PT_EUNSUPPORTED;
}

}  // namespace

extern "C" {

// C = A . B  (see header comment).  a_kcontig: A is [M,K] (ld=lda) else stored [K,M];
// b_kcontig: B is stored [N,K] (weights) else [K,N].  b_seg_dim: 0 = segments along N, 1 = along K.
// b_bounds / c_bounds: n+1 boundaries (first 0, last = N/K or M).  epilogue: 0 bf16 store,
// 1 bf16 accumulate (C = bf16(C + bf16(acc))), 2 fp32 store, 3 fp32 accumulate,
// 4 bf16 residual (C = bf16(R + bf16(acc))).  tile: -1 = auto.
int pt_gemm(const void* A, int64_t lda, int a_kcontig, const void* const* B, const int64_t* ldb,
            const int64_t* b_bounds, int nb, int b_kcontig, int b_seg_dim, void* const* C, const int64_t* ldc,
            const int64_t* c_bounds, int nc, int64_t M, int64_t N, int64_t K, int epilogue,
            const void* residual, int64_t ldr, int tile, hipStream_t stream) {
  GemmGroup g{};
  g.nprob = 1;
  const int rc = fill_args(g.p[0], A, lda, B, ldb, b_bounds, nb, b_seg_dim, C, ldc, c_bounds, nc, M, N, K, epilogue,
                           residual, ldr);
  if (rc) return rc;
  return launch_group(g, a_kcontig, b_kcontig, epilogue, tile, stream);
}

// Several independent problems in one launch (same layouts / epilogue; see include/picotron_hip.h).
int pt_gemm_grouped(const pt_gemm_problem* probs, int nprob, int a_kcontig, int b_kcontig, int epilogue, int tile,
                    hipStream_t stream) {
  if (!probs || nprob < 1 || nprob > kMaxProb) return PT_EINVAL;
  GemmGroup g{};
  g.nprob = nprob;
  for (int i = 0; i < nprob; ++i) {
    const pt_gemm_problem& q = probs[i];
    int rc = fill_args(g.p[i], q.A, q.lda, q.B, q.ldb, q.b_bounds, q.nb, q.b_seg_dim, q.C, q.ldc, q.c_bounds,
                       q.nc, q.M, q.N, q.K, epilogue, q.residual, q.ldr);
    if (!rc) rc = fill_split(g.p[i], q, epilogue);
    if (rc) return rc;
  }
  return launch_group(g, a_kcontig, b_kcontig, epilogue, tile, stream);
}

}  // extern "C"

namespace {

// Split-K finish for nparts f32 partials [nparts][M][N] (ld N, part stride M N): out = the sum in
// part order (deterministic), through the sink's epilogue -- 0 bf16 store, 1 bf16 accumulate
// (bf16(C + bf16(sum)), the wgrad's .grad accumulation), 2 f32 store, 3 f32 accumulate (main_grad),
// 4 bf16 residual (bf16(R + bf16(sum))), 6 the SwiGLU backward of a split-K down_proj dX (sum = dh,
// R = g|u [M, 2N], C = dg|du [M, 2N]: the fused epilogue's math) -- into up to 4 row segments of C
// (c_bounds), each with its own pointer and leading dimension.  4 columns per thread-iteration
// (16-B partial loads).
struct ReduceArgs {
  const float* parts;
  int nparts;
  int64_t M, N, part_stride;
  void* C[4];
  int64_t ldc[4];
  int64_t cseg[5];
  int nc;
  const uint16_t* R;
  int64_t ldr;
};

template <int MODE>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const ReduceArgs r) {
  const int64_t n4 = r.N / 4, total = r.M * n4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / n4, c4 = i - row * n4;
    const float* p = r.parts + row * r.N + c4 * 4;
    float4 acc = *(const float4*)p;
    for (int k = 1; k < r.nparts; ++k) {
      const float4 v = *(const float4*)(p + k * r.part_stride);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    int seg = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (j < r.nc && row >= r.cseg[j]) seg = j;
    const int64_t off = (row - r.cseg[seg]) * r.ldc[seg] + c4 * 4;
    const float v[4] = {acc.x, acc.y, acc.z, acc.w};
    if (MODE == EPI_SWIGLU_BWD) {
      // the sum is dh (rounded to bf16 as the fused epilogue stages it); R = g|u, C = dg|du [M, 2N]
      const uint16_t* gr = r.R + row * r.ldr + c4 * 4;
      const uint2 gw = *(const uint2*)gr, uw = *(const uint2*)(gr + r.N);
      const float g[4] = {lo_bf(gw.x), hi_bf(gw.x), lo_bf(gw.y), hi_bf(gw.y)};
      const float u[4] = {lo_bf(uw.x), hi_bf(uw.x), lo_bf(uw.y), hi_bf(uw.y)};
      float og[4], ou[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = round_bf(v[e]), sg = silu_sig(g[e]);
        ou[e] = d * round_bf(g[e] * sg);
        og[e] = round_bf(d * u[e]) * (sg * (1.0f + g[e] * (1.0f - sg)));
      }
      uint16_t* o = (uint16_t*)r.C[0] + off;
      *(uint2*)o = make_uint2(pack_bf2(og[0], og[1]), pack_bf2(og[2], og[3]));
      *(uint2*)(o + r.N) = make_uint2(pack_bf2(ou[0], ou[1]), pack_bf2(ou[2], ou[3]));
    } else if (MODE == EPI_F32 || MODE == EPI_F32_ACC) {
      float4* o = (float4*)((float*)r.C[seg] + off);
      float4 w = make_float4(v[0], v[1], v[2], v[3]);
      if (MODE == EPI_F32_ACC) {
        const float4 old = *o;
        w.x += old.x; w.y += old.y; w.z += old.z; w.w += old.w;
      }
      *o = w;
    } else {
      uint2* o = (uint2*)((uint16_t*)r.C[seg] + off);
      float f[4] = {v[0], v[1], v[2], v[3]};
      if (MODE == EPI_BF16_ACC || MODE == EPI_BF16_RES) {
        const uint2 old = MODE == EPI_BF16_ACC ? *o : *(const uint2*)(r.R + row * r.ldr + c4 * 4);
        const float of[4] = {lo_bf(old.x), hi_bf(old.x), lo_bf(old.y), hi_bf(old.y)};
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = of[e] + round_bf(f[e]);
      }
      uint2 w;
      w.x = pack_bf2(f[0], f[1]);
      w.y = pack_bf2(f[2], f[3]);
      *o = w;
    }
  }
}

}  // namespace

extern "C" {

int pt_gemm_splitk_reduce(const float* parts, int nparts, int64_t part_stride, int64_t M, int64_t N, void* const* C,
                          const int64_t* ldc, const int64_t* c_bounds, int nc, int mode, const void* residual,
                          int64_t ldr, hipStream_t stream) {
  if (!parts || nparts < 1 || M <= 0 || N <= 0 || (N & 3) || !C || nc < 1 || nc > 4) return PT_EINVAL;
  if (part_stride < M * N || !pt_aligned16(parts) || (part_stride & 3)) return PT_EALIGN;
  if ((mode == EPI_BF16_RES || mode == EPI_SWIGLU_BWD) && (!residual || ((uintptr_t)residual & 7) || (ldr & 3)))
    return PT_EINVAL;
  if (mode == EPI_SWIGLU_BWD && nc != 1) return PT_EINVAL;   // one dg|du [M, 2N] output
  ReduceArgs r{};
  r.parts = parts; r.nparts = nparts; r.M = M; r.N = N; r.part_stride = part_stride;
  r.nc = nc;
  for (int i = 0; i <= nc; ++i) r.cseg[i] = c_bounds ? c_bounds[i] : (i == 0 ? 0 : M);
  if (r.cseg[0] != 0 || r.cseg[nc] != M) return PT_EINVAL;
  const int esz = (mode == EPI_F32 || mode == EPI_F32_ACC) ? 4 : 2;
  for (int i = 0; i < nc; ++i) {
    if (!C[i] || ((uintptr_t)C[i] & (esz * 4 - 1)) || (ldc[i] & 3)) return PT_EALIGN;
    r.C[i] = C[i];
    r.ldc[i] = ldc[i];
  }
  r.R = (const uint16_t*)residual;
  r.ldr = ldr;
  const int64_t total = M * (N / 4);
  int64_t grid = (total + 255) / 256;
  if (grid > PT_STREAM_GRID_CAP) grid = PT_STREAM_GRID_CAP;
  switch (mode) {
    case EPI_BF16: splitk_reduce_kernel<EPI_BF16><<<(int)grid, 256, 0, stream>>>(r); break;
    case EPI_BF16_ACC: splitk_reduce_kernel<EPI_BF16_ACC><<<(int)grid, 256, 0, stream>>>(r); break;
    case EPI_F32: splitk_reduce_kernel<EPI_F32><<<(int)grid, 256, 0, stream>>>(r); break;
    case EPI_F32_ACC: splitk_reduce_kernel<EPI_F32_ACC><<<(int)grid, 256, 0, stream>>>(r); break;
    case EPI_BF16_RES: splitk_reduce_kernel<EPI_BF16_RES><<<(int)grid, 256, 0, stream>>>(r); break;
    case EPI_SWIGLU_BWD: splitk_reduce_kernel<EPI_SWIGLU_BWD><<<(int)grid, 256, 0, stream>>>(r); break;
    default: return PT_EINVAL;
  }
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// Split-K finish: out = bf16(p0 + p1), 4 elements per thread-iteration (16-B loads, 8-B store).
// For the long-K dX GEMMs of N = 2048 (gate|up dX, K 16384; lm_head dX, K 49152): 256x256 8-phase
// tiles over two K halves fill the 256 CUs as one round and run ~17 % above the 256x128 4-phase
// rate per FLOP at that K (tools/gemm_kscan.py), which pays for the f32 partials and this pass.
__global__ __launch_bounds__(256) void splitk_sum2_kernel(const float4* __restrict__ p0, const float4* __restrict__ p1,
                                                          const uint2* res, uint2* out, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 a = p0[i], b = p1[i];
    float v[4] = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
    if (res) {  // EPI_BF16_RES: bf16(R + bf16(acc))
      const uint2 r = res[i];
      const float rf[4] = {lo_bf(r.x), hi_bf(r.x), lo_bf(r.y), hi_bf(r.y)};
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = rf[k] + round_bf(v[k]);
    }
    uint2 w;
    w.x = pack_bf2(v[0], v[1]);
    w.y = pack_bf2(v[2], v[3]);
    out[i] = w;
  }
}

int pt_gemm_splitk_sum(const float* p0, const float* p1, const void* residual, void* out, int64_t n,
                       hipStream_t stream) {
  if (!p0 || !p1 || !out || n <= 0 || (n & 3)) return PT_EINVAL;
  if (!pt_aligned16(p0) || !pt_aligned16(p1) || ((uintptr_t)out & 7) || ((uintptr_t)residual & 7)) return PT_EALIGN;
  const int64_t n4 = n / 4;
  int64_t grid = (n4 + 255) / 256;
  if (grid > PT_STREAM_GRID_CAP) grid = PT_STREAM_GRID_CAP;
  splitk_sum2_kernel<<<(int)grid, 256, 0, stream>>>((const float4*)p0, (const float4*)p1, (const uint2*)residual,
                                                    (uint2*)out, n4);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// Two independent groups in ONE launch of 256x256 8-phase tiles (see gemm_8ph_dual_kernel): a dX
// group and a wgrad group of the same layer, each with its own epilogue.  PT_EUNSUPPORTED when a
// problem does not tile by 256x256 or a group's tile count is not a multiple of 8 (the caller
// then launches the two groups separately).
int pt_gemm_dual(const pt_gemm_problem* p0, int n0, int a_kcontig0, int b_kcontig0, int epilogue0,
                 const pt_gemm_problem* p1, int n1, int a_kcontig1, int b_kcontig1, int epilogue1, int order,
                 hipStream_t stream) {
  if (!p0 || !p1 || n0 < 1 || n0 > kMaxProb || n1 < 1 || n1 > kMaxProb) return PT_EINVAL;
  GemmGroup g[2]{};
  const pt_gemm_problem* ps[2] = {p0, p1};
  const int ns[2] = {n0, n1}, es[2] = {epilogue0, epilogue1};
  for (int k = 0; k < 2; ++k) {
    g[k].nprob = ns[k];
    for (int i = 0; i < ns[k]; ++i) {
      const pt_gemm_problem& q = ps[k][i];
      int rc = fill_args(g[k].p[i], q.A, q.lda, q.B, q.ldb, q.b_bounds, q.nb, q.b_seg_dim, q.C, q.ldc,
                         q.c_bounds, q.nc, q.M, q.N, q.K, es[k], q.residual, q.ldr);
      if (!rc) rc = fill_split(g[k].p[i], q, es[k]);
      if (rc) return rc;
    }
  }
  return launch_dual(g[0], a_kcontig0, b_kcontig0, epilogue0, g[1], a_kcontig1, b_kcontig1, epilogue1, order,
                     stream);
}

// q|k|v projection with RoPE fused (EPI_ROPE): C[M,N] = A[M,K] . [B_0; ...]^T with columns
// [0, rot_cols) rotated by the [seq, table_stride] cos/sin tables at position row % seq_len.
int pt_gemm_rope(const void* A, int64_t lda, const void* const* B, const int64_t* ldb, const int64_t* b_bounds, int nb,
                 void* C, int64_t ldc, int64_t M, int64_t N, int64_t K, const void* cos_table, const void* sin_table,
                 int64_t table_stride, int64_t seq_len, int64_t rot_cols, int64_t head_dim, int tile,
                 hipStream_t stream) {
  if (!cos_table || !sin_table || seq_len <= 0 || rot_cols < 0 || rot_cols > N) return PT_EINVAL;
  if (head_dim != 64 || rot_cols % 64) return PT_EUNSUPPORTED;
  GemmGroup g{};
  g.nprob = 1;
  void* const Cs[1] = {C};
  const int64_t ldcs[1] = {ldc};
  const int rc = fill_args(g.p[0], A, lda, B, ldb, b_bounds, nb, 0, Cs, ldcs, nullptr, 1, M, N, K, EPI_ROPE, nullptr, 0);
  if (rc) return rc;
  GemmArgs& a = g.p[0];
  a.rope_cos = (const uint16_t*)cos_table;
  a.rope_sin = (const uint16_t*)sin_table;
  a.rope_ld = table_stride;
  a.rope_seq = (int)seq_len;
  a.rope_cols = (int)rot_cols;
  return launch_group(g, 1, 1, EPI_ROPE, tile, stream);
}

// lm_head with the cross-entropy forward statistics fused (EPI_CE_STATS): logits C[M, N] = A[M, K] .
// W[N, K]^T stored bf16, and float2 stats[N / block][M] = (max, sum exp(x - max)) of the stored
// values per row and block-column tile (block 256: the 8-phase 256x256 kernel, 128: the 4-phase
// 256x128 one).  M % 256 == 0, N % block == 0.
int pt_gemm_ce_stats(const void* A, int64_t lda, const void* W, int64_t ldw, void* C, int64_t ldc, float* stats,
                     int64_t block, int64_t M, int64_t N, int64_t K, hipStream_t stream) {
  if (!stats || !pt_aligned16(stats)) return PT_EINVAL;
  if (block != 256 && block != 128) return PT_EUNSUPPORTED;
  const int tile = block == 256 ? 12 : 13;
  GemmGroup g{};
  g.nprob = 1;
  const void* const Bs[1] = {W};
  const int64_t ldbs[1] = {ldw};
  void* const Cs[1] = {C};
  const int64_t ldcs[1] = {ldc};
  const int rc = fill_args(g.p[0], A, lda, Bs, ldbs, nullptr, 1, 0, Cs, ldcs, nullptr, 1, M, N, K, EPI_CE_STATS,
                           nullptr, 0);
  if (rc) return rc;
  if (!args_fit(g.p[0], tile)) return PT_EUNSUPPORTED;
  if (ldc & 7) return PT_EALIGN;
  g.p[0].stats = stats;
  return launch_group(g, 1, 1, EPI_CE_STATS, tile, stream);
}

// Tile the auto-pick chooses for one [M, N] problem with the given segment boundaries (see
// pick_group_tile: the phased 256x256 / 256x128 kernels by last-round fill, then 128x128, 64x64).
int pt_gemm_pick_tile(int64_t M, int64_t N, const int64_t* mseg, int nmseg, const int64_t* nseg, int nnseg) {
  GemmGroup g{};
  g.nprob = 1;
  GemmArgs& a = g.p[0];
  a.M = (int)M;
  a.N = (int)N;
  a.ncseg = nmseg > 1 ? nmseg - 1 : 1;
  a.cseg[0] = 0;
  a.cseg[a.ncseg] = M;
  for (int i = 0; i < nmseg && i < 5; ++i) a.cseg[i] = mseg[i];
  a.nbseg = nnseg > 1 ? nnseg - 1 : 1;
  a.bseg[0] = 0;
  a.bseg[a.nbseg] = N;
  for (int i = 0; i < nnseg && i < 5; ++i) a.bseg[i] = nseg[i];
  return pick_group_tile(g);
}

}  // extern "C"
