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
// Structure: BMxBNx64 tiles, WMxWN waves (wave tile (BM/WM)x(BN/WN)), v_mfma_f32_16x16x32_bf16.
// Global->LDS by global_load_lds_dwordx4 (LDS-DMA, lane-linear 1 KiB per wave instruction) into a
// double-buffered LDS image; the XOR swizzle is applied to the per-lane SOURCE address and undone
// on the ds_read (tools/lds_swizzle_search.py: conflict-free for ds_read_b128 on K-contiguous
// images and ds_read_b64_tr_b16 on MN-contiguous images).  The next K-tile's DMA is in flight
// while the current one is multiplied.  Epilogue stages the tile through LDS and writes whole
// 16-byte row segments.
#include "common.h"

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

// Stage one operand tile (ROWS x 64 if K-contiguous, 64 x ROWS if MN-contiguous) into LDS.
// `g` points at element (tile row/col 0, k0) of the operand; ld is its leading dimension.
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

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI>
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

  // tile order: XCD remap, then group 8 tile-rows so an XCD's neighbours share A/B panels
  const int nwg = a.tiles_m * a.tiles_n;
  const int pid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int group_span = GROUP * a.tiles_n;
  const int gid = pid / group_span;
  const int first_m = gid * GROUP;
  const int gsize = min(a.tiles_m - first_m, GROUP);
  const int tile_m = first_m + (pid % group_span) % gsize;
  const int tile_n = (pid % group_span) / gsize;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // operand bases for this tile
  const uint16_t* Abase = AK ? a.A + (int64_t)m0 * a.lda : a.A + m0;
  int bs_n = 0;
  if (a.bdim == 0) bs_n = find_seg(a.bseg, a.nbseg, n0);
  const uint16_t* Bn = a.B[bs_n];
  const int64_t ldb_n = a.ldb[bs_n];
  const int64_t nloc = n0 - a.bseg[bs_n];

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
    const uint16_t* Bp = Bn;
    int64_t ldb = ldb_n, kl = k0, nl = nloc;
    if (a.bdim == 1) {
      const int s = find_seg(a.bseg, a.nbseg, k0);
      Bp = a.B[s];
      ldb = a.ldb[s];
      kl = k0 - a.bseg[s];
      nl = n0;
    }
    const uint16_t* gb = BKC ? Bp + nl * ldb + kl : Bp + kl * ldb + nl;
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
  }

  // ---- epilogue ---------------------------------------------------------------------------
  const int cs = find_seg(a.cseg, a.ncseg, m0);
  const int64_t ldc = a.ldc[cs];
  const int64_t mrow0 = m0 - a.cseg[cs] + wm * TM;
  const int ncol0 = n0 + wn * TN;
  if (EPI == EPI_BF16 || EPI == EPI_BF16_ACC || EPI == EPI_BF16_RES) {
    // stage this wave's TM x TN tile as bf16 rows in LDS, then write 16-B row segments
    constexpr int ROWB = TN * 2 + 16;  // +16 B pad: spreads the column-wise 2-B writes over banks
    lds_u8* st = smem + wave * (TM * ROWB);
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

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, int EPI>
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
    (void)hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, WM, WN, AK, BKC, EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  gemm_kernel<BM, BN, WM, WN, AK, BKC, EPI><<<a.tiles_m * a.tiles_n, WM * WN * 64, smem, stream>>>(a);
  PT_CHECK_LAUNCH();
  return PT_OK;
}

template <bool AK, bool BKC, int EPI>
int launch_layout(const GemmArgs& a, int tile, hipStream_t s) {
  switch (tile) {
    case 0: return launch_t<256, 256, 2, 4, AK, BKC, EPI>(a, s);
    case 1: return launch_t<256, 128, 4, 2, AK, BKC, EPI>(a, s);
    case 2: return launch_t<128, 128, 2, 2, AK, BKC, EPI>(a, s);
    case 3: return launch_t<64, 64, 2, 2, AK, BKC, EPI>(a, s);
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

const int kTileBM[4] = {256, 256, 128, 64};
const int kTileBN[4] = {256, 128, 128, 64};

}  // namespace

extern "C" {

// Pick the largest tile that divides the problem and still puts >= 256 tiles on the chip
// (one per CU); fall back to the largest that divides.
int pt_gemm_pick_tile(int64_t M, int64_t N, const int64_t* mseg, int nmseg, const int64_t* nseg, int nnseg) {
  int best_div = -1;
  for (int t = 0; t < 4; ++t) {
    const int bm = kTileBM[t], bn = kTileBN[t];
    if (M % bm || N % bn) continue;
    bool ok = true;
    for (int i = 0; i < nmseg && ok; ++i) ok = (mseg[i] % bm) == 0;
    for (int i = 0; i < nnseg && ok; ++i) ok = (nseg[i] % bn) == 0;
    if (!ok) continue;
    if (best_div < 0) best_div = t;
    if ((M / bm) * (N / bn) >= 256) return t;
  }
  return best_div;
}

// C = A . B  (see header comment).  a_kcontig: A is [M,K] (ld=lda) else stored [K,M];
// b_kcontig: B is stored [N,K] (weights) else [K,N].  b_seg_dim: 0 = segments along N, 1 = along K.
// b_bounds / c_bounds: n+1 boundaries (first 0, last = N/K or M).  epilogue: 0 bf16 store,
// 1 bf16 accumulate (C = bf16(C + bf16(acc))), 2 fp32 store, 3 fp32 accumulate.  tile: -1 = auto.
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
    tile = pt_gemm_pick_tile(M, N, msegs, nc + 1, nsegs, nb + 1);
  }
  if (tile < 0 || tile > 3) return PT_EUNSUPPORTED;
  if (M % kTileBM[tile] || N % kTileBN[tile]) return PT_EUNSUPPORTED;
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
