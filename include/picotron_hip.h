/* picotron_hip.h -- C ABI of the picotron_amd gfx950 (MI355X) kernels.
 *
 * Every entry point takes plain device pointers, element counts / strides (in ELEMENTS, not
 * bytes) and a hipStream_t, launches asynchronously on that stream, never allocates, and returns
 * 0 on success, a negative PT_E* code for an argument error detected before launch, or a
 * positive hipError_t from the launch.  bf16 tensors are passed as raw 16-bit storage.
 *
 * Each function names the reference interface it replaces (paths relative to the reference
 * checkout, okoge-kaz/picotron @ 2025-03-02).  The Python host layer (picotron_amd/_C.py) binds
 * these with ctypes; INTEGRATION.md shows the binding a picotron maintainer would add.
 */
#ifndef PICOTRON_HIP_H
#define PICOTRON_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

#define PT_OK 0
#define PT_EINVAL (-1)
#define PT_EALIGN (-2)
#define PT_EUNSUPPORTED (-3)

/* Device status word (int32, caller-owned, zeroed by the caller): kernels that validate DATA (not
 * shapes) set a bit here instead of trapping -- the analogue of torch's device-side assert.  The
 * host reads it when it synchronises anyway (picotron_amd.kernels.device_status). */
#define PT_STATUS_BAD_TARGET 1

/* ---- RMSNorm ------------------------------------------------------------------------------
 * replaces picotron/model.py:51-65 (TritonRMSNorm -> flash-attn layer_norm_fn, mode 0) and
 * picotron/model.py:81-86 (LlamaRMSNorm, mode 1); `residual` fuses the bf16 residual add of
 * picotron/model.py:207-208 (z_out = bf16(x + residual) is normalised and written out).
 * x, residual, y, z_out: [rows, cols] bf16; weight [cols] bf16; rstd [rows] f32 (saved for bwd). */
int pt_rmsnorm_fwd(const void* x, const void* residual, const void* weight, void* y, void* z_out, float* rstd,
                   int64_t rows, int64_t cols, float eps, int mode, hipStream_t stream);
/* number of f32 rows of `cols` the bwd needs in dw_partial */
int pt_rmsnorm_bwd_partials(int64_t rows, int cols);
/* autograd backward of the above: dx = d/dz (+ dres), dweight [cols] (may be NULL).
 * mode = norm mode (0 / 1) | dweight sink: 0 store bf16; PT_DW_ACC_BF16 dweight = bf16(dweight +
 * bf16(dw)) (autograd's accumulation into a bf16 .grad); PT_DW_ACC_F32 dweight is f32, += dw
 * (DataParallelBucket main_grad).  The weight sum is in a fixed order (deterministic). */
#define PT_DW_ACC_BF16 4
#define PT_DW_ACC_F32 8
int pt_rmsnorm_bwd(const void* dy, const void* z, const void* weight, const float* rstd, const void* dres,
                   void* dx, void* dweight, float* dw_partial, int64_t rows, int64_t cols, int mode,
                   hipStream_t stream);
/* pt_rmsnorm_bwd with dy given as the two f32 K halves of a split-K dX GEMM (pt_gemm_dual / pt_gemm
 * with EPI_F32 partials: contiguous [rows, cols]): dy = bf16(dy_p0 + dy_p1) is formed in the kernel,
 * bit-identical to pt_gemm_splitk_sum followed by pt_rmsnorm_bwd without writing and re-reading dy.
 * (The post_attention_layernorm backward behind the gate|up dX, model.py:206-208.) */
int pt_rmsnorm_bwd_splitk(const float* dy_p0, const float* dy_p1, const void* z, const void* weight,
                          const float* rstd, const void* dres, void* dx, void* dweight, float* dw_partial,
                          int64_t rows, int64_t cols, int mode, hipStream_t stream);
/* the dweight column sums of n <= 32 pt_rmsnorm_bwd calls made with dweight = NULL (their
 * dw_partial buffers, pt_rmsnorm_bwd_partials rows each), one launch; sinks[i] as the dweight sink
 * bits of pt_rmsnorm_bwd's mode.  Bit-identical to passing dweight to each call.  (An
 * implementation detail of the same LlamaRMSNorm backward: a micro-batch's norms sum their weight
 * gradients together at the end of its backward.) */
int pt_rmsnorm_colsum_batch(const float* const* partials, const int* nparts, void* const* dweights,
                            const int* sinks, int n, int64_t cols, hipStream_t stream);

/* ---- RoPE (rotate-half, non-interleaved) --------------------------------------------------
 * replaces picotron/model.py:136-137 (flash-attn apply_rotary_emb) and model.py:12-19
 * (apply_rotary_pos_emb).  In place on the first `nheads` heads of every row of x
 * ([rows, row_stride] bf16); row r has position r % seq_len in the [seq_len, table_stride]
 * cos/sin tables of get_cos_sin (model.py:21-31).  inverse = 1 rotates by -theta (backward). */
int pt_rope(void* x, int64_t rows, int64_t row_stride, int64_t nheads, int64_t head_dim, const void* cos_table,
            const void* sin_table, int64_t seq_len, int64_t table_stride, int inverse, hipStream_t stream);

/* ---- SwiGLU: h = silu(g) * u --------------------------------------------------------------
 * replaces picotron/model.py:186 F.silu(gate_proj(x)) * up_proj(x) (fwd and autograd bwd). */
int pt_swiglu_fwd(const void* g, int64_t g_stride, const void* u, int64_t u_stride, void* h, int64_t h_stride,
                  int64_t rows, int64_t cols, hipStream_t stream);
int pt_swiglu_bwd(const void* dh, int64_t dh_stride, const void* g, int64_t g_stride, const void* u,
                  int64_t u_stride, void* dg, int64_t dg_stride, void* du, int64_t du_stride, int64_t rows,
                  int64_t cols, hipStream_t stream);

/* ---- residual add: out = bf16(x + r), n contiguous bf16 (n % 8 == 0, 16-B aligned) ------------
 * replaces picotron/model.py:208 `x + self.mlp(...)` where the sequence-parallel TP layer adds the
 * residual to its reduce-scattered MLP output (no GEMM epilogue can carry it there). */
int pt_residual_add(const void* x, const void* r, void* out, int64_t n, hipStream_t stream);

/* ---- fused cross-entropy forward + backward -----------------------------------------------
 * replaces train.py:49 F.cross_entropy(logits, targets, 'mean') / grad_acc (+ autograd bwd) and
 * pipeline_parallel.py:103,153.  row_loss[r] = lse - logit[target]; dlogits (may alias logits) =
 * (softmax - onehot) * scale * (*inv_count if non-NULL).  targets int64, ignore_index rows -> 0;
 * a target outside [0, vocab) (not ignore_index) gives a NaN row and sets PT_STATUS_BAD_TARGET in
 * *status (may be NULL).  dlogits == NULL: loss only (one read of the logits). */
int pt_cross_entropy_fwd_bwd(const void* logits, int64_t logits_stride, const int64_t* targets, void* dlogits,
                             int64_t dlogits_stride, float* row_loss, int64_t rows, int64_t vocab, float scale,
                             const float* inv_count, int64_t ignore_index, int* status, hipStream_t stream);
/* The autograd pair (train.py:49 forward, loss.backward() at train.py:51): the forward streams the
 * logits once with an online max / sum-exp and writes row_loss and row_lse [rows] f32; the
 * backward is elementwise from the saved LSE: dlogits = (exp(x - row_lse) - onehot) *
 * scale[row * scale_stride] (scale_stride 0: one device scalar, grad_output / #valid for 'mean',
 * grad_output for 'sum'; 1: a per-row f32 gradient, reduction='none'), ignore_index rows -> 0.
 * dlogits may alias logits. */
int pt_cross_entropy_fwd_lse(const void* logits, int64_t logits_stride, const int64_t* targets, float* row_loss,
                             float* row_lse, int64_t rows, int64_t vocab, int64_t ignore_index, int* status,
                             hipStream_t stream);
int pt_cross_entropy_bwd_lse(const void* logits, int64_t logits_stride, const int64_t* targets, const float* row_lse,
                             void* dlogits, int64_t dlogits_stride, int64_t rows, int64_t vocab, const float* scale,
                             int64_t scale_stride, int64_t ignore_index, hipStream_t stream);
/* The same forward from the lm_head GEMM's statistics (pt_gemm_ce_stats) instead of a second pass
 * over the logits: float2 stats[b * rows + row] = (max, sum exp(x - max)) of the row's bf16 logits
 * in column tile b < nblk (vocab / nblk columns each); only x[row, target] is read. */
int pt_cross_entropy_fwd_stats(const void* logits, int64_t logits_stride, const int64_t* targets,
                               const float* stats, int64_t nblk, float* row_loss, float* row_lse, int64_t rows,
                               int64_t vocab, int64_t ignore_index, int* status, hipStream_t stream);

/* Vocab-parallel form (the lm_head as ColumnParallelLinear(gather_output=True), tensor_parallel.py:
 * 50 + tp_communications.py:51-72, whose logits all-gather it replaces): each tp rank reduces its
 * shard logits [rows, vocab_shard] (global columns vocab_lo ..) with the GEMM statistics to a float4
 * part[row] = (max, sum exp(x - max), x[target] if target in the shard else 0, 1 / 0); the caller
 * all-gathers the parts [tp][rows][4] and combines them (rank order) into row_loss / row_lse as
 * pt_cross_entropy_fwd_stats returns them for the whole vocabulary (same range check against
 * `vocab`).  The backward on the shard: pt_cross_entropy_bwd_lse with the one-hot at target - vocab_lo. */
int pt_cross_entropy_vp_partial(const void* logits, int64_t logits_stride, const int64_t* targets,
                                const float* stats, int64_t nblk, float* part, int64_t rows, int64_t vocab_shard,
                                int64_t vocab_lo, hipStream_t stream);
int pt_cross_entropy_vp_combine(const float* parts, int64_t tp, const int64_t* targets, float* row_loss,
                                float* row_lse, int64_t rows, int64_t vocab, int64_t ignore_index, int* status,
                                hipStream_t stream);
int pt_cross_entropy_bwd_lse_shard(const void* logits, int64_t logits_stride, const int64_t* targets,
                                   const float* row_lse, void* dlogits, int64_t dlogits_stride, int64_t rows,
                                   int64_t vocab_shard, int64_t vocab_lo, const float* scale, int64_t scale_stride,
                                   int64_t ignore_index, hipStream_t stream);

/* train.py:49's reduction='mean' over the per-row losses: loss = sum(row_loss) / #(target !=
 * ignore_index) in one deterministic launch; inv_count = 1 / #valid (the backward's scale);
 * reduce_sum != 0: reduction='sum' (loss = sum(row_loss), inv_count = 1);
 * loss_f32 / out (bf16 when out_bf16, else f32) optional. */
int pt_cross_entropy_mean(const float* row_loss, const int64_t* targets, int64_t rows, int64_t ignore_index,
                          float* loss_f32, float* inv_count, void* out, int out_bf16, int reduce_sum,
                          hipStream_t stream);

/* ---- token embedding ----------------------------------------------------------------------
 * replaces model.py:224-225 (F.embedding + autograd's dense backward) and the masked lookup of
 * VocabParallelEmbedding (tensor_parallel.py:246-270): rows of ids outside [vocab_lo, vocab_hi)
 * are zero.  ids int64 [T]; weight [vocab_hi - vocab_lo, H] bf16 (leading dim ldw).
 * bwd: ids sorted ascending with their token positions perm (stable; -1 = token to skip);
 * dweight[id - vocab_lo] (sink: 0 store bf16, PT_DW_ACC_BF16, PT_DW_ACC_F32) gets the f32 sum of
 * the dY rows of each id rounded to bf16 once; untouched rows are not accessed. */
int pt_embedding_fwd(const int64_t* ids, int64_t T, const void* weight, int64_t ldw, int64_t vocab_lo, int64_t vocab_hi,
                     void* out, int64_t ldo, int64_t H, hipStream_t stream);
int pt_embedding_bwd(const int64_t* sorted_ids, const int64_t* perm, int64_t T, const void* dy, int64_t ldy,
                     int64_t vocab_lo, void* dweight, int64_t lddw, int64_t H, int sink, hipStream_t stream);
/* The backward's segment order: ids keyed (0 = skipped: outside [vocab_lo, vocab_hi) or padding_idx
 * when has_padding; else id - vocab_lo + 1) and stably sorted in one launch -> sorted_ids (-1 =
 * skip) and perm (token positions), the inputs of pt_embedding_bwd.  T <= 16384 (else
 * PT_EUNSUPPORTED). */
int pt_embedding_sort(const int64_t* ids, int64_t T, int64_t vocab_lo, int64_t vocab_hi, int has_padding,
                      int64_t padding_idx, int64_t* sorted_ids, int64_t* perm, hipStream_t stream);

/* ---- fused AdamW step ---------------------------------------------------------------------
 * replaces train.py:209 torch.optim.AdamW(...).step() for one tensor: the eight foreach passes of
 * torch's multi-tensor Adam (decoupled weight decay) in one, same per-op rounding to the storage
 * dtype (dtype 0 bf16, 1 f32).  Scalars as torch casts them: decay = 1 - lr*wd, w1 = 1 - beta1,
 * c2 = 1 - beta2, bc2_sqrt = sqrt(1 - beta2^t), step_size = -lr / (1 - beta1^t). */
int pt_adamw_step(void* param, const void* grad, void* exp_avg, void* exp_avg_sq, int64_t n, int dtype,
                  float decay, float w1, float beta2, float c2, float bc2_sqrt, float eps, float step_size,
                  hipStream_t stream);
/* The same update over a LIST of bf16 tensors in one launch (torch's foreach AdamW is a list op
 * too): `tensors` is a device array of pt_adam_tensor (every pointer 16-byte aligned),
 * `chunk_start` a device int64 [ntensors + 1] of prefix sums of ceil(n / 8), total_chunks its last
 * entry.  The caller builds and caches both (the pointers only change when tensors are re-made). */
typedef struct {
  void* param;
  const void* grad;
  void* exp_avg;
  void* exp_avg_sq;
  int64_t n;
} pt_adam_tensor;
int pt_adamw_step_multi(const void* tensors, const int64_t* chunk_start, int ntensors, int64_t total_chunks,
                        float decay, float w1, float beta2, float c2, float bc2_sqrt, float eps, float step_size,
                        hipStream_t stream);

/* ---- bf16 GEMM, f32 accumulate -------------------------------------------------------------
 * replaces every F.linear / matmul of the layer: model.py:124-126,161,186,270,
 * tensor_parallel.py:186, tp_communications.py:79,93,98,105.
 * C[M,N] (op)= A[M,K] B[K,N].  a_kcontig: A stored [M,K] (else [K,M]); b_kcontig: B stored
 * [N,K] (weights; else [K,N]).  B may be split into nb pointer segments along N (b_seg_dim 0)
 * or K (1), C into nc segments along M; *_bounds hold n+1 boundaries (NULL = one segment).
 * epilogue 0: C bf16 = acc, 1: C bf16 += acc, 2: C f32 = acc, 3: C f32 += acc,
 * 4: C bf16 = residual + acc (residual [M, N] bf16, leading dim ldr; the residual add of
 * model.py:207-208 fused into the producing projection).  tile -1 = auto. */
int pt_gemm(const void* A, int64_t lda, int a_kcontig, const void* const* B, const int64_t* ldb,
            const int64_t* b_bounds, int nb, int b_kcontig, int b_seg_dim, void* const* C, const int64_t* ldc,
            const int64_t* c_bounds, int nc, int64_t M, int64_t N, int64_t K, int epilogue,
            const void* residual, int64_t ldr, int tile, hipStream_t stream);
int pt_gemm_pick_tile(int64_t M, int64_t N, const int64_t* mseg, int nmseg, const int64_t* nseg, int nnseg);
/* The q|k|v projection with RoPE fused into its epilogue (model.py:124-126 + 136-137): columns
 * [0, rot_cols) of C = A . [B_0; ...]^T (B K-contiguous, segments along N) are rotated like
 * pt_rope (position = row % seq_len in the [seq, table_stride] bf16 cos/sin tables); head_dim 64. */
int pt_gemm_rope(const void* A, int64_t lda, const void* const* B, const int64_t* ldb, const int64_t* b_bounds, int nb,
                 void* C, int64_t ldc, int64_t M, int64_t N, int64_t K, const void* cos_table, const void* sin_table,
                 int64_t table_stride, int64_t seq_len, int64_t rot_cols, int64_t head_dim, int tile,
                 hipStream_t stream);
/* The lm_head (model.py:270, logits consumed by F.cross_entropy at train.py:49) with the CE forward's
 * statistics fused into its epilogue: C[M, N] = A[M, K] . W[N, K]^T stored bf16, and per row and
 * `block`-column tile b the (max, sum exp(x - max)) of the stored values as float2
 * stats[b * M + row] (block 256 or 128; M % 256 == 0, N % block == 0, K % 64 == 0). */
int pt_gemm_ce_stats(const void* A, int64_t lda, const void* W, int64_t ldw, void* C, int64_t ldc, float* stats,
                     int64_t block, int64_t M, int64_t N, int64_t K, hipStream_t stream);
/* Grouped GEMM: nprob (<= 4) independent problems in ONE launch, each described like pt_gemm's
 * arguments, sharing layouts (a_kcontig, b_kcontig), epilogue and tile (-1 = auto over the
 * group).  Used where one problem alone would leave CUs idle (dW of q|k|v + dW of o_proj).
 * ksplit > 1 (epilogue 2 only): the problem runs as ksplit K-slices of K / ksplit (a multiple of 64)
 * whose f32 partials land kpart_stride elements apart from C (slice s at C + s kpart_stride) -- for
 * the few-tile TP-shard GEMMs (24-128 tiles on 256 CUs); pt_gemm_splitk_reduce finishes them. */
typedef struct {
  const void* A;
  int64_t lda;
  const void* B[4];
  int64_t ldb[4];
  int64_t b_bounds[5];
  int nb;
  int b_seg_dim;
  void* C[4];
  int64_t ldc[4];
  int64_t c_bounds[5];
  int nc;
  int64_t M, N, K;
  const void* residual;
  int64_t ldr;
  int ksplit;              /* 0 / 1: not split */
  int64_t kpart_stride;    /* elements between two slices' f32 partials */
  /* A K-segmented: k >= a_k2 (a multiple of 64 inside K) reads A2 (same lda) -- a weight gradient
   * over two micro-batches' token rows (dY of both; B K-segmented the same way through b_seg_dim 1,
   * b_bounds {0, a_k2, K}): one K = 2 T launch instead of two accumulating ones (data_parallel.py:
   * 122-144's main_grad read-modify-written once per two micro-batches).  NULL: not segmented.  The
   * 256x256 8-phase tile only (pt_gemm_grouped tile 12 / auto, pt_gemm_dual). */
  const void* A2;
  int64_t a_k2;
} pt_gemm_problem;
int pt_gemm_grouped(const pt_gemm_problem* probs, int nprob, int a_kcontig, int b_kcontig, int epilogue, int tile,
                    hipStream_t stream);

/* Two independent groups in ONE launch of 256x256 tiles, each with its own layouts and epilogue:
 * group 0 = dX (A = dY [M, K] K-contiguous, B = W [K, N] N-contiguous; epilogue 0 or 6 = the
 * SwiGLU backward, residual = g|u), group 1 = wgrad (dY^T X; both operands MN-contiguous;
 * epilogue 0, 1 or 3; or 2 with ksplit problems: a split-K dW's f32 slices, pt_gemm_splitk_reduce).  The dX of a layer's projection beside its dW (both read only dY and saved
 * activations): the down_proj dX's HBM-bound SwiGLU-backward tail overlaps the dW's MFMA work.
 * Group 0's epilogue: 0 (bf16), 6 (SwiGLU backward) or 2 (f32: the two K halves of a split-K dX,
 * finished by pt_gemm_splitk_sum).
 * order: 0 group 0 first, 1 group 1 first, inside each XCD's share; 2 staggered (even XCDs group 0 first,
 * odd XCDs group 1 first).
 * PT_EUNSUPPORTED when a problem does not tile by 256 x 256 or a group's tile count % 8 != 0. */
int pt_gemm_dual(const pt_gemm_problem* p0, int n0, int a_kcontig0, int b_kcontig0, int epilogue0,
                 const pt_gemm_problem* p1, int n1, int a_kcontig1, int b_kcontig1, int epilogue1, int order,
                 hipStream_t stream);
/* out (bf16, n contiguous elements) = bf16(p0 + p1), or bf16(residual + bf16(p0 + p1)) when
 * residual (bf16, n contiguous) is given (= the EPI_BF16_RES epilogue): the finishing pass of a GEMM
 * split in two K halves (two f32 problems of one pt_gemm_grouped launch, 256x256 tiles).  n % 4 == 0,
 * p0 / p1 16-byte, out / residual 8-byte aligned; residual may alias out. */
int pt_gemm_splitk_sum(const float* p0, const float* p1, const void* residual, void* out, int64_t n,
                       hipStream_t stream);
/* Split-K finish for nparts f32 partials [nparts][M][N] (ld N, part_stride >= M N elements apart):
 * the sum in part order through `mode` = the GEMM epilogue it completes -- 0 bf16 store, 1 bf16
 * accumulate, 2 f32 store, 3 f32 accumulate (main_grad), 4 bf16 residual (residual [M, N], ld ldr),
 * 6 SwiGLU backward (the sum is dh of a split-K down_proj dX, model.py:186; residual = g|u [M, 2N]
 * ld ldr; C[0] = dg|du [M, 2N], nc = 1) -- into nc (<= 4) row segments of C (c_bounds, NULL = one),
 * each with its own ld.  N % 4 == 0. */
int pt_gemm_splitk_reduce(const float* parts, int nparts, int64_t part_stride, int64_t M, int64_t N, void* const* C,
                          const int64_t* ldc, const int64_t* c_bounds, int nc, int mode, const void* residual,
                          int64_t ldr, hipStream_t stream);

/* ---- ring-attention merge ------------------------------------------------------------------
 * replaces picotron/context_parallel/context_parallel.py:157-187 update_out_and_lse (its non-first
 * call): out_new = out - sigmoid(blse - lse) * (out - block_out), lse_new = lse - logsigmoid(lse -
 * blse).  out / out_new f32 [rows, D]; block_out [rows, D] (dtype 0 bf16, 1 f32); lse, block_lse,
 * lse_new [rows] in lse_dtype (0 bf16: every lse-side op rounded to bf16 as the reference's bf16
 * ring does; 1 f32).  All contiguous; rows = B * H * S.  (The ring's own merge is fused into
 * pt_attn_fwd's merge mode.) */
int pt_lse_merge(const float* out, const void* block_out, int block_out_dtype, const void* lse, const void* block_lse,
                 int lse_dtype, float* out_new, void* lse_new, int64_t rows, int64_t D, hipStream_t stream);

/* ---- flash attention ----------------------------------------------------------------------
 * replaces model.py:33-37,154 flash_attn_func(causal=True) / model.py:157 SDPA, and the ring
 * blocks context_parallel.py:112-155 with update_out_and_lse (:157-187) fused (merge = 1).
 * q/k/v/o/dout/dq/dk/dv: token-major [B, S, H, D] views given as base + 3 strides
 * {batch, seq, head} (elements; d contiguous).  lse, delta: f32 [B, H, Sq] whose (b, h) rows are
 * lse_ld elements apart (0: Sq, dense; larger: the Sq rows are a slice of a longer sequence's LSE,
 * as the zig-zag ring's half-sequence blocks use).  D in {64, 128},
 * Sq % 128 == 0, Sk % 64 == 0 (bwd: Sk % 128 == 0).  causal: key j visible to query i iff j <= i.
 * bwd rope_cos/rope_sin (may be NULL): [S, rope_stride] bf16 tables; dq and dk are then stored
 * rotated back by -theta (pt_rope inverse fused; positions = query / key index, Sq == Sk, bf16). */
int pt_attn_fwd(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                const int64_t* v_str, void* o, const int64_t* o_str, float* lse, int64_t B, int64_t H, int64_t HKV,
                int64_t Sq, int64_t Sk, int64_t D, float scale, int causal, int merge, int64_t lse_ld,
                hipStream_t stream);
int pt_attn_bwd_delta(const void* dout, const int64_t* do_str, const void* o, const int64_t* o_str, float* delta,
                      int64_t B, int64_t H, int64_t Sq, int64_t D, int64_t lse_ld, hipStream_t stream);
int pt_attn_bwd(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                const int64_t* v_str, const void* dout, const int64_t* do_str, const float* lse, const float* delta,
                void* dq, const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv, const int64_t* dv_str,
                int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D, float scale, int causal,
                int grad_f32, const void* rope_cos, const void* rope_sin, int64_t rope_stride, int64_t lse_ld,
                hipStream_t stream);
/* pt_attn_bwd computing only dQ (parts = 1) or only dK / dV (parts = 2), or both (3); the pointers
 * of a gradient not computed may be NULL.  The context-parallel mesh backward
 * (context_parallel.py:72-106's ring, restated for the xGMI full mesh) runs each rank's dQ against
 * the visiting K / V and its own keys' dK / dV against the visiting queries, so no dK / dV partial
 * travels. */
int pt_attn_bwd_part(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                     const int64_t* v_str, const void* dout, const int64_t* do_str, const float* lse,
                     const float* delta, void* dq, const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv,
                     const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D,
                     float scale, int causal, int grad_f32, int64_t lse_ld, int parts, hipStream_t stream);
/* pt_attn_bwd with the FA2 'D' = rowsum(dO * O) computed inside the dQ kernel (run first) from o
 * (bf16 [B, S, H, D] strides o_str) and written to delta_out [B, H, Sq] f32, which the dK/dV kernel
 * then reads: the separate pt_attn_bwd_delta pass disappears.  bf16 gradients only (no grad_f32). */
int pt_attn_bwd_fused_delta(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str,
                            const void* v, const int64_t* v_str, const void* o, const int64_t* o_str,
                            const void* dout, const int64_t* do_str, const float* lse, float* delta_out, void* dq,
                            const int64_t* dq_str, void* dk, const int64_t* dk_str, void* dv,
                            const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk,
                            int64_t D, float scale, int causal, const void* rope_cos, const void* rope_sin,
                            int64_t rope_stride, int64_t lse_ld, hipStream_t stream);
/* Few-head attention (a TP shard's heads: the regular launch -- one workgroup per causal query-block
 * pair -- would put fewer than 128 workgroups on the 256 CUs): the same flash_attn_func forward /
 * backward as work items of "attn_kv_chunk" K/V (Q) tiles, f32 partials in a caller-owned workspace,
 * and a merge / reduce pass.  pt_attn_split_plan: 1 and the workspace bytes when the split forms
 * apply to the shape (d64), else 0.  pt_attn_fwd_split = pt_attn_fwd with merge = 0 and a dense lse;
 * pt_attn_bwd_split = pt_attn_bwd_fused_delta with a dense lse.  Results equal the regular kernels' up
 * to the f32 summation order. */
int pt_attn_split_plan(int64_t B, int64_t H, int64_t HKV, int64_t Sq, int64_t Sk, int64_t D, int causal,
                       int backward, int64_t* ws_bytes);
int pt_attn_fwd_split(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                      const int64_t* v_str, void* o, const int64_t* o_str, float* lse, int64_t B, int64_t H,
                      int64_t HKV, int64_t Sq, int64_t Sk, int64_t D, float scale, int causal, void* ws,
                      int64_t ws_bytes, hipStream_t stream);
int pt_attn_bwd_split(const void* q, const int64_t* q_str, const void* k, const int64_t* k_str, const void* v,
                      const int64_t* v_str, const void* o, const int64_t* o_str, const void* dout, const int64_t* do_str,
                      const float* lse, float* delta_out, void* dq, const int64_t* dq_str, void* dk,
                      const int64_t* dk_str, void* dv, const int64_t* dv_str, int64_t B, int64_t H, int64_t HKV,
                      int64_t Sq, int64_t Sk, int64_t D, float scale, int causal, const void* rope_cos,
                      const void* rope_sin, int64_t rope_stride, void* ws, int64_t ws_bytes, hipStream_t stream);

/* ---- measurement variants ------------------------------------------------------------------
 * Not a reference interface: selects between kernel forms with identical results, for A/B runs and
 * the bit-identity tests.  The library reads no environment; the host sets these (picotron_amd/
 * switches.py reads PICOTRON_<NAME> once at import and pushes them here).  Names and defaults:
 *   "attn_pair"     1   causal attention: pair query/key blocks (i, n-1-i) per workgroup
 *   "attn_split"    2   dK/dV kernel form per head dim: bit 0 = d64, bit 1 = d128 use the wave pair
 *   "gemm_mix"      1   q|k|v + RoPE GEMM as one mixed 256x256 / 256x128 launch
 *   "gemm_kh"       2   auto-picked 256x128 tiles as tile 14 (K-halves) when K >= 4096; 0 never
 *   "attn_kv_chunk" 4   few-head attention (pt_attn_split_plan): K / Q tiles per work item (even;
 *                       0 = never split)
 * Returns PT_EINVAL for an unknown name.  pt_get_variant returns the value (or PT_EINVAL). */
int pt_set_variant(const char* name, int value);
int pt_get_variant(const char* name);

#ifdef __cplusplus
}
#endif
#endif /* PICOTRON_HIP_H */
