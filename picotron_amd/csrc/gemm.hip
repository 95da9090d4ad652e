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
// Two kernel structures, both v_mfma_f32_16x16x32_bf16 with operands staged global->LDS by
// global_load_lds_dwordx4 (LDS-DMA, lane-linear 1 KiB per wave instruction; the XOR swizzle is
// applied to the per-lane SOURCE address and undone on the ds_read -- tools/lds_swizzle_search.py:
// conflict-free for ds_read_b128 on K-contiguous images and ds_read_b64_tr_b16 on MN-contiguous
// images):
//
//  * gemm_pipe_kernel (tiles 256x256 and 256x128, 8 waves as 2(M) x 4(N), the large shapes):
//    each K-tile is four phases, one per quadrant of the wave's output tile, each closed by a raw
//    s_barrier.  The operand tiles are kept as four independent "half images" (A rows 0-127 /
//    128-255, B cols 0-BN/2 / BN/2-BN) so a buffer is refilled half by half: the DMA of K-tile
//    t+1's halves is issued in phases 1-3 of tile t and the first half of t+2 in phase 4 (the
//    moment all waves have finished reading tile t's buffer), and the single wait per K-tile is a
//    counted `s_waitcnt vmcnt(2)` that leaves that half in flight across the barrier -- the load
//    path never drains (cdna_hip_programming.md §5 "Pipelining across barriers", T3+T4).  Wave
//    fragments are read quadrant by quadrant (A rows 0-63 + B cols 0-31, B cols 32-63, A rows
//    64-127, registers reused for the 4th) and the MFMA cluster of each phase is bracketed with
//    s_setprio (T5).
//  * gemm_kernel (tiles 128x128, 64x64; small / ragged shapes): the simple two-stage loop.
//
// Epilogue (both): the wave's tile is staged through LDS as bf16 rows and written as whole 16-byte
// row segments; fp32 epilogues (main_grad accumulation) write the accumulator directly.
#include "common.h"

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;

namespace {

constexpr int BK = 64;

// EPI_BF16_RES: C = bf16(R + bf16(acc)) -- the residual add of model.py:207-208 fused into the
// producing GEMM (R may alias C).
enum Epilogue { EPI_BF16 = 0, EPI_BF16_ACC = 1, EPI_F32 = 2, EPI_F32_ACC = 3, EPI_BF16_RES = 4 };

struct GemmArgs {
  const uint16_t* A;
  int64_t lda;
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
  int M, N, K;
  int tiles_m, tiles_n;
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

// tile order: XCD remap, then group 8 tile-rows so an XCD's neighbours share A/B panels
__device__ __forceinline__ void tile_coords(const GemmArgs& a, int& tile_m, int& tile_n) {
  const int nwg = a.tiles_m * a.tiles_n;
  const int pid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int group_span = GROUP * a.tiles_n;
  const int gid = pid / group_span;
  const int first_m = gid * GROUP;
  const int gsize = min(a.tiles_m - first_m, GROUP);
  tile_m = first_m + (pid % group_span) % gsize;
  tile_n = (pid % group_span) / gsize;
}

// Write the wave's TM x TN accumulator tile (FM x FN 16x16 fragments) at output (m0 + wm*TM,
// n0 + wn*TN).  `st` is this wave's private LDS staging area (TM * (2*TN + 16) bytes).
template <int TM, int TN, int EPI>
__device__ __forceinline__ void epilogue(const GemmArgs& a, const f32x4_t (&acc)[TM / 16][TN / 16], lds_u8* st,
                                         int m0, int n0, int wm, int wn, int lane) {
  constexpr int FM = TM / 16, FN = TN / 16;
  const int cs = find_seg(a.cseg, a.ncseg, m0);
  const int64_t ldc = a.ldc[cs];
  const int64_t mrow0 = m0 - a.cseg[cs] + wm * TM;
  const int ncol0 = n0 + wn * TN;
  if (EPI == EPI_BF16 || EPI == EPI_BF16_ACC || EPI == EPI_BF16_RES) {
    constexpr int ROWB = TN * 2 + 16;  // +16 B pad: spreads the column-wise 2-B writes over banks
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + (lane >> 4) * 4 + r, col = j * 16 + (lane & 15);
          *(__attribute__((address_space(3))) uint16_t*)(st + row * ROWB + col * 2) = f2bf(acc[i][j][r]);
        }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-private staging, no barrier needed
    uint16_t* C = (uint16_t*)a.C[cs];
    constexpr int CPR = TN / 8;          // 16-B chunks per row
    constexpr int RPI = 64 / CPR;        // rows per wave instruction
#pragma unroll
    for (int it = 0; it < TM / RPI; ++it) {
      const int row = it * RPI + lane / CPR, ch = lane % CPR;
      typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
      const u32x4_t raw = *(const __attribute__((address_space(3))) u32x4_t*)(st + row * ROWB + ch * 16);
      bf16x8 v;
      v.w[0] = raw[0]; v.w[1] = raw[1]; v.w[2] = raw[2]; v.w[3] = raw[3];
      uint16_t* dst = C + (mrow0 + row) * ldc + ncol0 + ch * 8;
      if (EPI == EPI_BF16_ACC || EPI == EPI_BF16_RES) {
        float o[8], f[8];
        unpack8(v, f);
        unpack8(ld8(EPI == EPI_BF16_ACC ? dst : a.R + (mrow0 + row) * a.ldr + ncol0 + ch * 8), o);
        // acc was rounded to bf16 once above; add in f32 and round again (== torch's bf16 add)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += f[e];
        v = pack8(o);
      }
      st8(dst, v);
    }
  } else {
    float* C = (float*)a.C[cs];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mrow0 + i * 16 + (lane >> 4) * 4 + r;
          const int col = ncol0 + j * 16 + (lane & 15);
          float* d = C + row * ldc + col;
          if (EPI == EPI_F32_ACC) *d += acc[i][j][r];
          else *d = acc[i][j][r];
        }
  }
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

// =============================================================================== pipelined
// LDS holds two rings of half images: A halves (128 rows x 64 k, 16 KiB) in 5 slots and B halves
// (BN/2 cols x 64 k) in 5 slots -- 2.5 K-tiles, 160 KiB at BN = 256.  Half images of K-tile u are
// issued during the four phases of K-tile u-2, in the order A0, B0, B1, A1, each into the slot of
// a half image whose last read retired at least one barrier earlier:
//   A slot (2u + a) % 5 last held A1 of u-3 (a = 0) or A0 of u-2 (a = 1: read until phase 3 of
//   u-2, re-staged in phase 4);  B slot (2u + b) % 5 last held B1 of u-3 or B0 of u-2 (read until
//   phase 2, re-staged in phase 3).
// DMAs are issued at the start of M-sections and LDS reads are retired inside the following
// M-section (not before the barrier), so a slot is re-staged >= 2 barriers after its last read even
// across the staggered wave groups.  The wait for K-tile u+1 (end of phase 3's M-section of u)
// leaves K-tile u+2's first three halves in flight: vmcnt(6) (BN 256) / vmcnt(4) (BN 128).
template <int BN, bool AK, bool BKC, int EPI, bool STAG>
__global__ __launch_bounds__(512) void gemm_pipe_kernel(GemmArgs a) {
  constexpr int BM = 256, NT = 512;
  constexpr int TM = 128, TN = BN / 4;            // wave tile (2 x 4 waves)
  constexpr int FM = TM / 16, FN = TN / 16;       // 8 x (4 or 2) accumulators
  constexpr int QM = FM / 2, QN = FN / 2;         // fragments per quadrant
  constexpr int HB = BN / 2;                      // columns per B half image
  constexpr int A_HALF = 128 * BK * 2, B_HALF = HB * BK * 2;
  constexpr int NSLOT = 5;
  constexpr int B_RING = NSLOT * A_HALF;          // byte offset of the B ring
  constexpr int B_INSTR = B_HALF / 1024 / 8;      // DMA instructions per wave per B half (2 or 1)
  constexpr int AHEAD = 2 * 2 + 2 * B_INSTR;      // a K-tile's DMA instructions per wave
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int tile_m, tile_n;
  tile_coords(a, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  auto a_slot = [&](int u, int h) { return smem + ((2 * u + h) % NSLOT) * A_HALF; };
  auto b_slot = [&](int u, int h) { return smem + B_RING + ((2 * u + h) % NSLOT) * B_HALF; };
  auto stage_a = [&](int u, int h) {
    const int k0 = u * BK, r0 = m0 + 128 * h;
    const uint16_t* g = AK ? a.A + (int64_t)r0 * a.lda + k0 : a.A + (int64_t)k0 * a.lda + r0;
    stage_tile<128, AK, NT>(g, a.lda, a_slot(u, h), tid);
  };
  auto stage_b = [&](int u, int h) {
    int64_t ldb;
    const uint16_t* g = b_image_ptr(a, BKC, n0, u * BK, HB * h, ldb);
    stage_tile<HB, BKC, NT>(g, ldb, b_slot(u, h), tid);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
  // prologue: K-tiles 0 and 1 issued, K-tile 0 waited for
  stage_a(0, 0); stage_b(0, 0); stage_b(0, 1); stage_a(0, 1);
  if (nk > 1) {
    stage_a(1, 0); stage_b(1, 0); stage_b(1, 1); stage_a(1, 1);
    if (B_INSTR == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  const int brow = (wn & 1) * TN;  // the wave's first column inside its B half image
  bf16x8_t af[QM][2], b0[QN][2], b1[QN][2];

  // Every phase = R-section (LDS reads, left in flight across the barrier) + M-section (one half
  // image DMA + the quadrant's 16 / 8 MFMAs), each closed by a raw s_barrier.
  // STAG: waves 4-7 run one barrier behind waves 0-3, so on each SIMD one wave multiplies while
  // the other reads (ping-pong).
  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mma = [&](int i0, int j0, const bf16x8_t (&A)[QM][2], const bf16x8_t (&Bf)[QN][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < QM; ++i)
#pragma unroll
        for (int j = 0; j < QN; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i][s], Bf[j][s], acc[i0 + i][j0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  const bool late = STAG && __builtin_amdgcn_readfirstlane(wm) == 1;
  if (late) bar();

  for (int kt = 0; kt < nk; ++kt) {
    const lds_u8* sa = a_slot(kt, wm);
    const lds_u8* sb = b_slot(kt, wn >> 1);
    const bool pre = kt + 2 < nk;

    // ---- phase 1: R: A rows 0..63, B cols 0..TN/2 | M: DMA A0 of kt+2, quadrant (0, 0)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = read_frag<128, AK>(sa, i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < QN; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[j][s] = read_frag<HB, BKC>(sb, brow + j * 16, s, lane);
    bar();
    if (pre) stage_a(kt + 2, 0);
    mma(0, 0, af, b0);
    bar();

    // ---- phase 2: R: B cols TN/2..TN (last B reads) | M: DMA B0 of kt+2, quadrant (0, 1)
#pragma unroll
    for (int j = 0; j < QN; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) b1[j][s] = read_frag<HB, BKC>(sb, brow + (QN + j) * 16, s, lane);
    bar();
    if (pre) stage_b(kt + 2, 0);
    mma(0, QN, af, b1);
    bar();

    // ---- phase 3: R: A rows 64..127 (last A reads) | M: DMA B1 of kt+2 (into B0 of kt),
    //      quadrant (1, 1), then wait for K-tile kt+1 (all but kt+2's three halves in flight)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[i][s] = read_frag<128, AK>(sa, (QM + i) * 16, s, lane);
    bar();
    if (pre) stage_b(kt + 2, 1);
    mma(QM, QN, af, b1);
    if (pre) {
      if (B_INSTR == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();

    // ---- phase 4: R: nothing | M: DMA A1 of kt+2 (into A0 of kt), quadrant (1, 0)
    bar();
    if (pre) stage_a(kt + 2, 1);
    mma(QM, 0, af, b0);
    bar();
  }
  if (STAG && !late) bar();  // balance the barrier count of the two wave groups
  (void)AHEAD;

  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane);
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

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(512) void gemm_8ph_kernel(GemmArgs a) {
  constexpr int NT = 512, TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int HALF = 128 * BK * 2;          // 16 KiB
  constexpr int BUF = 4 * HALF;               // At, Bl, Br, Ab
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int tile_m, tile_n;
  tile_coords(a, tile_m, tile_n);
  const int m0 = tile_m * 256, n0 = tile_n * 256;

  // B segment for this tile (N-segments) or the first K-segment; ld is per tile (host checks
  // that K-segments share one ld)
  int64_t ldb;
  const uint16_t* Bt0 = b_image_ptr(a, BKC, n0, 0, 0, ldb);
  const int64_t lda = a.lda;
  // loop-invariant per-lane element offsets of this wave's 2 DMA instructions per half image
  uint32_t vA[2][2], vB[2][2];  // [half][it]
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 8 + wave;
    vA[0][it] = himg_voff<AK, 64>(i, lane, lda, 0);
    vA[1][it] = himg_voff<AK, 64>(i, lane, lda, 64);
    vB[0][it] = himg_voff<BKC, 32>(i, lane, ldb, 0);
    vB[1][it] = himg_voff<BKC, 32>(i, lane, ldb, 32);
  }
  const uint16_t* Ab0 = AK ? a.A + (int64_t)m0 * lda : a.A + m0;
  auto a_ptr = [&](int t) { return AK ? Ab0 + t * BK : Ab0 + (int64_t)t * BK * lda; };
  auto b_ptr = [&](int t) {
    if (a.bdim == 0) return BKC ? Bt0 + t * BK : Bt0 + (int64_t)t * BK * ldb;
    int64_t ld;
    return b_image_ptr(a, BKC, n0, t * BK, 0, ld);
  };
  // half image h (0 At, 1 Bl, 2 Br, 3 Ab) of K-tile t into buffer buf
  auto stage = [&](int t, int buf, int h) {
    lds_u8* dst = smem + buf * BUF + h * HALF;
    const bool isA = h == 0 || h == 3;
    const uint16_t* base = isA ? a_ptr(t) : b_ptr(t);
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

  const int nk = a.K / BK;
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
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i][s], Bf[j][s], acc[i0 + i][j0 + j], 0, 0, 0);
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
  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane);
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
__global__ __launch_bounds__(512) void gemm_4ph_kernel(GemmArgs a) {
  constexpr int TM = 64, TN = 64, FM = 4, FN = 4;
  constexpr int IMG = 128 * BK * 2;           // 16 KiB
  constexpr int BUF = 3 * IMG;                // At, B, Ab
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tile_m, tile_n;
  tile_coords(a, tile_m, tile_n);
  const int m0 = tile_m * 256, n0 = tile_n * 128;

  int64_t ldb;
  const uint16_t* Bt0 = b_image_ptr(a, BKC, n0, 0, 0, ldb);
  const int64_t lda = a.lda;
  uint32_t vA[2][2], vB[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = it * 8 + wave;
    vA[0][it] = himg_voff<AK, 32>(i, lane, lda, 0);
    vA[1][it] = himg_voff<AK, 32>(i, lane, lda, 32);
    vB[it] = himg_voff<BKC, 128>(i, lane, ldb, 0);
  }
  const uint16_t* Ab0 = AK ? a.A + (int64_t)m0 * lda : a.A + m0;
  auto a_ptr = [&](int t) { return AK ? Ab0 + t * BK : Ab0 + (int64_t)t * BK * lda; };
  auto b_ptr = [&](int t) {
    if (a.bdim == 0) return BKC ? Bt0 + t * BK : Bt0 + (int64_t)t * BK * ldb;
    int64_t ld;
    return b_image_ptr(a, BKC, n0, t * BK, 0, ld);
  };
  // image h (0 At, 1 B, 2 Ab) of K-tile t into buffer buf
  auto stage = [&](int t, int buf, int h) {
    lds_u8* dst = smem + buf * BUF + h * IMG;
    const uint16_t* base = h == 1 ? b_ptr(t) : a_ptr(t);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const uint32_t vo = h == 1 ? vB[it] : vA[h == 2 ? 1 : 0][it];
      glds16_asm(base, vo, dst + (it * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
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
          acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bf[j][s], acc[i0 + i][j], 0, 0, 0);
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
    if (n2) stage(t + 2, nbuf, 0);
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
  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane);
}

// ================================================================================= simple
template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, int SCHED>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(GemmArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int tile_m, tile_n;
  tile_coords(a, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const uint16_t* Abase = AK ? a.A + (int64_t)m0 * a.lda : a.A + m0;

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BK;
    lds_u8* sa = smem + buf * STAGE_BYTES;
    lds_u8* sb = sa + A_BYTES;
    const uint16_t* ga = AK ? Abase + k0 : Abase + (int64_t)k0 * a.lda;
    stage_tile<BM, AK, NT>(ga, a.lda, sa, tid);
    int64_t ldb;
    const uint16_t* gb = b_image_ptr(a, BKC, n0, k0, 0, ldb);
    stage_tile<BN, BKC, NT>(gb, ldb, sb, tid);
  };

  const int nk = a.K / BK;
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
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane);
}

// ============================================================================ 4-wave 256x256
// One workgroup of 4 waves (2 x 2) per CU, each wave owning a 128 x 128 output tile: 256 fp32
// accumulators per lane held across the unified 512-entry register file (one wave per SIMD,
// amdgpu_waves_per_eu(1, 1)).  Per K-tile a wave reads its A and B panels once (32 KiB; 128 KiB
// per CU instead of the 192 KiB an 8-wave 128 x 64 decomposition reads) for 128 MFMAs.
// Latency is hidden inside the wave: the K-tile is two MFMA blocks of 64 (k-substeps 0 and 1)
// and each block carries the LDS reads of the NEXT block's fragments (second register set):
//   block A(kt): MFMA(kt, s0)  ||  ds_read(kt, s1)
//   s_waitcnt vmcnt(0); s_barrier    <- K-tile kt+1 landed; every wave done reading K-tile kt
//   block B(kt): MFMA(kt, s1)  ||  ds_read(kt+1, s0), DMA(kt+2 -> the buffer kt just freed)
// so there is one barrier per K-tile and no read or DMA sits on the critical path.
template <bool AK, bool BKC, int EPI, int ABL = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void gemm_w4_kernel(GemmArgs a) {
  constexpr int BM = 256, BN = 256, NT = 256;
  constexpr int TM = 128, TN = 128, FM = 8, FN = 8;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int tile_m, tile_n;
  tile_coords(a, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const uint16_t* Abase = AK ? a.A + (int64_t)m0 * a.lda : a.A + m0;

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BK;
    lds_u8* sa = smem + buf * STAGE;
    const uint16_t* ga = AK ? Abase + k0 : Abase + (int64_t)k0 * a.lda;
    stage_tile<BM, AK, NT>(ga, a.lda, sa, tid);
    int64_t ldb;
    const uint16_t* gb = b_image_ptr(a, BKC, n0, k0, 0, ldb);
    stage_tile<BN, BKC, NT>(gb, ldb, sa + A_BYTES, tid);
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  bf16x8_t a0[FM], b0[FN], a1[FM], b1[FN];
  auto read_set = [&](int buf, int s, bf16x8_t (&A)[FM], bf16x8_t (&Bf)[FN]) {
    const lds_u8* sa = smem + buf * STAGE;
    const lds_u8* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < FM; ++i) A[i] = read_frag<BM, AK>(sa, wm * TM + i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) Bf[j] = read_frag<BN, BKC>(sb, wn * TN + j * 16, s, lane);
  };
  auto mma = [&](const bf16x8_t (&A)[FM], const bf16x8_t (&Bf)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], Bf[j], acc[i][j], 0, 0, 0);
  };

  const int nk = a.K / BK;
  stage(0, 0);
  if (nk > 1) stage(1, 1);
  if (nk > 1) {
    // K-tile 0's DMA instructions are the older half: wait for them only
    constexpr int PER_TILE = (A_BYTES + B_BYTES) / 1024 / (NT / 64);
    static_assert(PER_TILE == 16, "DMA instructions per wave per K-tile");
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  read_set(0, 0, a0, b0);

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    // block A: MFMA(kt, s0) with the reads of (kt, s1)
    read_set(buf, 1, a1, b1);
    mma(a0, b0);
    // K-tile kt+1 landed (its DMA is the only one outstanding); all reads of buffer `buf` retired
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // block B: MFMA(kt, s1) with the reads of (kt+1, s0) and the DMA of kt+2 into `buf`
    if (kt + 1 < nk) read_set(buf ^ 1, 0, a0, b0);
    if (ABL == 0 && kt + 2 < nk) stage(kt + 2, buf);   // ABL = 1: timing ablation without the DMA
    mma(a1, b1);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  epilogue<TM, TN, EPI>(a, acc, smem + wave * (TM * (TN * 2 + 16)), m0, n0, wm, wn, lane);
}

template <bool AK, bool BKC, int EPI, int ABL = 0>
int launch_w4(const GemmArgs& a0, hipStream_t stream) {
  GemmArgs a = a0;
  a.tiles_m = a.M / 256;
  a.tiles_n = a.N / 256;
  constexpr int smem_main = 2 * (256 + 256) * BK * 2;
  constexpr int smem_epi = 4 * 128 * (128 * 2 + 16);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_w4_kernel<AK, BKC, EPI, ABL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  gemm_w4_kernel<AK, BKC, EPI, ABL><<<a.tiles_m * a.tiles_n, 256, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// ================================================================================== launch
template <typename Kern>
void set_smem_once(Kern k, int smem) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
}

template <int BN, bool AK, bool BKC, int EPI, bool STAG>
int launch_pipe(const GemmArgs& a0, hipStream_t stream) {
  GemmArgs a = a0;
  a.tiles_m = a.M / 256;
  a.tiles_n = a.N / BN;
  constexpr int smem_main = 5 * (128 * BK * 2 + (BN / 2) * BK * 2);
  constexpr int smem_epi = 8 * 128 * ((BN / 4) * 2 + 16);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_pipe_kernel<BN, AK, BKC, EPI, STAG>, smem);
    attr_set = true;
  }
  gemm_pipe_kernel<BN, AK, BKC, EPI, STAG><<<a.tiles_m * a.tiles_n, 512, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI, int SCHED = 0>
int launch_t(const GemmArgs& a0, hipStream_t stream) {
  GemmArgs a = a0;
  a.tiles_m = a.M / BM;
  a.tiles_n = a.N / BN;
  constexpr int smem_main = 2 * (BM + BN) * BK * 2;
  constexpr int smem_epi = WM * WN * (BM / WM) * ((BN / WN) * 2 + 16);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_kernel<BM, BN, WM, WN, AK, BKC, EPI, SCHED>, smem);
    attr_set = true;
  }
  gemm_kernel<BM, BN, WM, WN, AK, BKC, EPI, SCHED><<<a.tiles_m * a.tiles_n, WM * WN * 64, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

// tile ids: 0 = pipelined 256x256, 1 = pipelined 256x128 (ping-pong wave groups), 2 = simple
//           128x128, 3 = simple 64x64, 4 = simple 256x256, 5 = simple 256x128, 6 / 7 = pipelined
//           256x256 / 256x128 without the ping-pong stagger (kept for A/B measurement)
//           12 = 8-phase 256x256 (two half-image wave groups, one wait per K-tile)
//           13 = 4-phase 256x128 (three K-tiles resident)
constexpr int kNumTiles = 14;
const int kTileBM[kNumTiles] = {256, 256, 128, 64, 256, 256, 256, 256, 256, 128, 256, 256, 256, 256};
const int kTileBN[kNumTiles] = {256, 128, 128, 64, 256, 128, 256, 128, 256, 128, 256, 256, 256, 128};

template <bool AK, bool BKC, int EPI>
int launch_8ph(const GemmArgs& a0, hipStream_t stream) {
  GemmArgs a = a0;
  a.tiles_m = a.M / 256;
  a.tiles_n = a.N / 256;
  constexpr int smem_main = 8 * 128 * BK * 2;
  constexpr int smem_epi = 8 * 128 * (64 * 2 + 16);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_8ph_kernel<AK, BKC, EPI>, smem);
    attr_set = true;
  }
  gemm_8ph_kernel<AK, BKC, EPI><<<a.tiles_m * a.tiles_n, 512, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_4ph(const GemmArgs& a0, hipStream_t stream) {
  GemmArgs a = a0;
  a.tiles_m = a.M / 256;
  a.tiles_n = a.N / 128;
  constexpr int smem_main = 9 * 128 * BK * 2;
  constexpr int smem_epi = 8 * 64 * (64 * 2 + 16);
  constexpr int smem = smem_main > smem_epi ? smem_main : smem_epi;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    set_smem_once(gemm_4ph_kernel<AK, BKC, EPI>, smem);
    attr_set = true;
  }
  gemm_4ph_kernel<AK, BKC, EPI><<<a.tiles_m * a.tiles_n, 512, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_layout(const GemmArgs& a, int tile, hipStream_t s) {
  switch (tile) {
    case 0: return launch_pipe<256, AK, BKC, EPI, true>(a, s);
    case 1: return launch_pipe<128, AK, BKC, EPI, true>(a, s);
    case 6: return launch_pipe<256, AK, BKC, EPI, false>(a, s);
    case 7: return launch_pipe<128, AK, BKC, EPI, false>(a, s);
    case 8: return launch_t<256, 256, 2, 4, AK, BKC, EPI, 1>(a, s);
    case 9: return launch_t<128, 128, 2, 2, AK, BKC, EPI, 1>(a, s);
    case 10: return launch_w4<AK, BKC, EPI>(a, s);
    case 11: return launch_w4<AK, BKC, EPI, 1>(a, s);
    case 12: return launch_8ph<AK, BKC, EPI>(a, s);
    case 13: return launch_4ph<AK, BKC, EPI>(a, s);
    case 2: return launch_t<128, 128, 2, 2, AK, BKC, EPI>(a, s);
    case 3: return launch_t<64, 64, 2, 2, AK, BKC, EPI>(a, s);
    case 4: return launch_t<256, 256, 2, 4, AK, BKC, EPI>(a, s);
    case 5: return launch_t<256, 128, 4, 2, AK, BKC, EPI>(a, s);
    default: return PT_EUNSUPPORTED;
  }
}

template <int EPI>
int launch_epi(const GemmArgs& a, int a_kcontig, int b_kcontig, int tile, hipStream_t s) {
  if (a_kcontig && b_kcontig) return launch_layout<true, true, EPI>(a, tile, s);
  if (a_kcontig && !b_kcontig) return launch_layout<true, false, EPI>(a, tile, s);
  if (!a_kcontig && !b_kcontig) return launch_layout<false, false, EPI>(a, tile, s);
  return launch_layout<false, true, EPI>(a, tile, s);
}

}  // namespace

extern "C" {

// Tile choice, from the measured sweep over the decoder layer's shapes (tools/gemm_bench.py,
// profiles/r01_gemm_tiles_8ph.md): the phased kernels whenever the shape divides -- 256x256 (tile
// 12) or 256x128 (tile 13), whichever fills the 256 CUs' last round better (ties -> 256x256: fewer
// operand bytes per MFMA); 1.0-1.38 PF/s on every projection of the layer.  Else the 128x128
// two-stage kernel, else 64x64.
static bool tile_fits(int t, int64_t M, int64_t N, const int64_t* mseg, int nmseg, const int64_t* nseg, int nnseg) {
  const int bm = kTileBM[t], bn = kTileBN[t];
  if (M % bm || N % bn) return false;
  for (int i = 0; i < nmseg; ++i)
    if (mseg[i] % bm) return false;
  for (int i = 0; i < nnseg; ++i)
    if (nseg[i] % bn) return false;
  return true;
}

static int pick_tile(int64_t M, int64_t N, const int64_t* mseg, int nmseg, const int64_t* nseg, int nnseg,
                     int b_kcontig) {
  (void)b_kcontig;
  auto fill = [&](int t) {  // fraction of the CU-rounds this tile grid keeps busy
    const int64_t tiles = (M / kTileBM[t]) * (N / kTileBN[t]);
    const int64_t rounds = (tiles + 255) / 256;
    return (double)tiles / (double)(rounds * 256);
  };
  const bool f12 = tile_fits(12, M, N, mseg, nmseg, nseg, nnseg);
  const bool f13 = tile_fits(13, M, N, mseg, nmseg, nseg, nnseg);
  if (f12 && (!f13 || fill(12) >= fill(13))) return 12;
  if (f13) return 13;
  if (tile_fits(2, M, N, mseg, nmseg, nseg, nnseg)) return 2;
  if (tile_fits(3, M, N, mseg, nmseg, nseg, nnseg)) return 3;
  return -1;
}

int pt_gemm_pick_tile(int64_t M, int64_t N, const int64_t* mseg, int nmseg, const int64_t* nseg, int nnseg) {
  return pick_tile(M, N, mseg, nmseg, nseg, nnseg, 1);
}

// C = A . B  (see header comment).  a_kcontig: A is [M,K] (ld=lda) else stored [K,M];
// b_kcontig: B is stored [N,K] (weights) else [K,N].  b_seg_dim: 0 = segments along N, 1 = along K.
// b_bounds / c_bounds: n+1 boundaries (first 0, last = N/K or M).  epilogue: 0 bf16 store,
// 1 bf16 accumulate (C = bf16(C + bf16(acc))), 2 fp32 store, 3 fp32 accumulate,
// 4 bf16 residual (C = bf16(R + bf16(acc))).  tile: -1 = auto.
int pt_gemm(const void* A, int64_t lda, int a_kcontig, const void* const* B, const int64_t* ldb,
            const int64_t* b_bounds, int nb, int b_kcontig, int b_seg_dim, void* const* C, const int64_t* ldc,
            const int64_t* c_bounds, int nc, int64_t M, int64_t N, int64_t K, int epilogue,
            const void* residual, int64_t ldr, int tile, hipStream_t stream) {
  if (!A || !B || !C || nb < 1 || nb > 4 || nc < 1 || nc > 4 || M <= 0 || N <= 0 || K <= 0) return PT_EINVAL;
  if (epilogue == EPI_BF16_RES && (!residual || nc != 1 || !pt_aligned16(residual) || (ldr & 7))) return PT_EINVAL;
  if (K % BK) return PT_EUNSUPPORTED;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return PT_EUNSUPPORTED;
  GemmArgs a{};
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
  // K-segment boundaries must be multiples of BK
  if (b_seg_dim == 1)
    for (int i = 0; i <= nb; ++i)
      if (a.bseg[i] % BK) return PT_EUNSUPPORTED;
  if (tile < 0) {
    int64_t nsegs[5], msegs[5];
    for (int i = 0; i <= nb; ++i) nsegs[i] = b_seg_dim == 0 ? a.bseg[i] : 0;
    for (int i = 0; i <= nc; ++i) msegs[i] = a.cseg[i];
    tile = pick_tile(M, N, msegs, nc + 1, nsegs, nb + 1, b_kcontig);
    if ((tile == 12 || tile == 13) && b_seg_dim == 1)
      for (int i = 1; i < nb; ++i)
        if (a.ldb[i] != a.ldb[0]) tile = tile_fits(2, M, N, msegs, nc + 1, nsegs, nb + 1) ? 2 : 3;
  }
  if (tile < 0 || tile >= kNumTiles) return PT_EUNSUPPORTED;
  const int bm = kTileBM[tile], bn = kTileBN[tile];
  if (M % bm || N % bn) return PT_EUNSUPPORTED;
  for (int i = 0; i <= nc; ++i)
    if (a.cseg[i] % bm) return PT_EUNSUPPORTED;
  if (b_seg_dim == 0)
    for (int i = 0; i <= nb; ++i)
      if (a.bseg[i] % bn) return PT_EUNSUPPORTED;
  if ((tile == 12 || tile == 13) && b_seg_dim == 1)  // one B leading dimension per tile
    for (int i = 1; i < nb; ++i)
      if (a.ldb[i] != a.ldb[0]) return PT_EUNSUPPORTED;
  switch (epilogue) {
    case EPI_BF16: return launch_epi<EPI_BF16>(a, a_kcontig, b_kcontig, tile, stream);
    case EPI_BF16_ACC: return launch_epi<EPI_BF16_ACC>(a, a_kcontig, b_kcontig, tile, stream);
    case EPI_F32: return launch_epi<EPI_F32>(a, a_kcontig, b_kcontig, tile, stream);
    case EPI_F32_ACC: return launch_epi<EPI_F32_ACC>(a, a_kcontig, b_kcontig, tile, stream);
    case EPI_BF16_RES:  // forward projections only (weights K-contiguous)
      if (!a_kcontig || !b_kcontig) return PT_EUNSUPPORTED;
      return launch_layout<true, true, EPI_BF16_RES>(a, tile, stream);
    default: return PT_EINVAL;
  }
}

}  // extern "C"
