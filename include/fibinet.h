/*
 * fibinet.h -- C ABI of libfibinet_hip.so, the MI355X (gfx950) kernels behind the FiBiNET
 * training path of YOUNESELBOUKNIFY/Ctr_recommendation.
 *
 * The reference is pure Python: its "interface" for this path is the PyTorch module
 * src/model_fibinet.py (build_model / MM_FiBiNET.forward + autograd backward) and the per-step
 * optimizer code of src/train_fibinet.py.  Each entry point below replaces the implicit ATen
 * op(s) named in its comment (reference file:line).  The Python binding is
 * ctr_recommendation_amd/_lib.py (ctypes); INTEGRATION.md shows the reference-side wiring.
 *
 * Conventions
 *  - all tensors are device pointers owned by the caller (torch); the library allocates
 *    nothing persistent.  Scratch is passed in; size it with the *_workspace_size queries.
 *  - every call is asynchronous on `stream` (a hipStream_t), takes no locks and keeps no
 *    global mutable state except a thread-local error string -> reentrant, graph-capturable.
 *  - return 0 on success, otherwise FBN_ERR_*; fbn_last_error() describes the failure.
 *  - id range violations never fault: kernels set a sticky int flag (*err) that the caller
 *    checks lazily (the reference raises IndexError in nn.Embedding).
 *  - fp32 storage everywhere; `bf16` flags select bf16 MFMA operands with fp32 accumulation.
 */
#ifndef FIBINET_H
#define FIBINET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FBN_OK 0
#define FBN_ERR_ARG 1
#define FBN_ERR_LAUNCH 2
#define FBN_ERR_UNSUPPORTED 3

const char* fbn_last_error(void);
/* Kernel-span probes (bench.py's rooflines): between fbn_probe_arm(slot) and fbn_probe_disarm() the
 * library's kernel launches record slot's event pair -- start at the first kernel's start, stop at
 * each kernel's end (hipExtLaunchKernelGGL; timing events without the system-scope fence).  Both are
 * ordinary entry points, so a step program can record them (probes inside the timed replays).
 * fbn_probe_elapsed(slot): the span in ms once those kernels completed, -1 if none took the slot. */
int fbn_probe_arm(int slot);
int fbn_probe_disarm(void);
float fbn_probe_elapsed(int slot);
int fbn_version(void);
int fbn_device_ok(void); /* 1 if the current HIP device is gfx950 */

/* ---------------------------------------------------------------- GEMM (MFMA)
 * C[m][rC(n)] = sum_k A(m,k) B(k,n) + bias[n] + beta*C ; remap r(i) = i + (i < seg ? off0 : off1)
 * (seg = INT32_MAX: identity).  Replaces addmm/matmul of
 *   mm_proj Linear           src/model_fibinet.py:105-106,162
 *   bilinear x @ W            src/model_fibinet.py:72
 *   MLP Linear x3             src/model_fibinet.py:126,130,134,197
 * and all of their autograd backward GEMMs.  Split-K slabs need ws >= fbn_gemm_workspace_size. */
size_t fbn_gemm_workspace_size(int M, int N, int K, int bf16);
/* a16 / b16: operand A / B is bf16 in memory (bf16 = 1, ld % 8 == 0, no rB remap); otherwise fp32.
 * bf16 = 2: split-bf16 x3 over fp32 operands (a16 = b16 = 0): each operand x = hi + lo, hi = bf16(x),
 * lo = bf16(x - hi), and C = Ahi Bhi + Ahi Blo + Alo Bhi on the bf16 MFMA with fp32 accumulation
 * (~2^-16 relative per product) -- the fp32-gradient GEMMs of the bf16-forward mode.
 * stats (optional): [ceil(M/64)][N][2] per-64-row-tile column (sum, M2) of C for the fused
 * BatchNorm statistics, from the MFMA epilogue (no split-K: 64-row tiles) or the split-K reduce;
 * C is bit-identical with or without it. */
int fbn_gemm(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int lda, int ldb,
             int ldc, int transA, int transB, int rB_seg, int rB_off0, int rB_off1, int rC_seg, int rC_off0,
             int rC_off1, float beta, int bf16, int a16, int b16, float* stats, float* ws, size_t ws_bytes,
             void* stream);
/* bf16 GEMM over a split operand (LDS-DMA path): A2/kseg -- a k-contiguous A is [A | A2] along K
 * (A(m,k), k >= kseg, at A2[m*lda2 + k - kseg]); B2/nseg -- a k-major B is [B | B2] along N
 * (B(k,n), n >= nseg, at B2[k*ldb2 + n - nseg]); segments multiples of 128.  The MLP input
 * [V_1..V_5 | pairs] is read from the bf16 fields (Vc16) and the pair block of c without a copy. */
/* Slab mode (bf16 LDS-DMA path): op(A) op(B) whose split-K partial products stay in ws as
 * *nsplit slabs [nsplit][M][N] f32 (ws >= fbn_gemm_slabs_size(M, N, K) bytes) -- no reduce launch;
 * the caller sums them with fbn_sum_jobs2 beside the step's other deferred reductions (the
 * trainer's weight-gradient GEMMs, autograd of src/model_fibinet.py:72,105,126,130).  No bias,
 * beta, remap or statistics; A2/kseg, B2/nseg as fbn_gemm_split. */
size_t fbn_gemm_slabs_size(int M, int N, int K);
int fbn_gemm_slabs(const void* A, const void* B, int M, int N, int K, int lda, int ldb, int transA, int transB,
                   float* ws, size_t ws_bytes, const void* A2, int lda2, int kseg, const void* B2, int ldb2, int nseg,
                   int* nsplit, void* stream);
/* The K-slab count fbn_gemm_slabs takes for an M x N x K product (its *nsplit), host-only. */
int fbn_gemm_slabs_split(int M, int N, int K);
/* n <= 6 slab-mode GEMMs in ONE launch (the step's weight gradients, deferred to the end of the
 * backward: one tail instead of one per GEMM).  descs = host array of n records
 * {const void* A, *B; float* ws; size_t ws_bytes; const void* A2, *B2;
 *  int M, N, K, lda, ldb, transA, transB, lda2, kseg, ldb2, nseg, s3k0; long long lo_a, lo_b;}
 * with the meaning of fbn_gemm_slabs's arguments; each ws receives fbn_gemm_slabs_group_split(M, N, K)
 * K-slabs (3/4 of fbn_gemm_slabs_split's, rounded, by default; with FBN_GROUP_SPLIT_DIV=1 exactly the slabs
 * fbn_gemm_slabs writes, bit for bit).  Every problem: transA = 1, transB = 0, K % 64 == 0,
 * M, N, lda, ldb % 8 == 0, no A2.  s3k0 > 0 (on every problem or none): split-bf16 x3 as
 * fbn_gemm_s3, K = 3 s3k0 over the hi images A / B and the lo images lo_a / lo_b elements past them. */
int fbn_gemm_slabs_group(const void* descs, int n, void* stream);
/* The K-slab count a problem takes inside fbn_gemm_slabs_group, host-only. */
int fbn_gemm_slabs_group_split(int M, int N, int K);
/* bf16 operands (as fbn_gemm with bf16 = a16 = b16 = 1), C stored in bf16 (C[m * ldc + n], rounded
 * once from the f32 accumulators); no bias, beta, remap or statistics.  The bf16-mode dgrad
 * dc = dh1 Wa of the MLP input (src/model_fibinet.py:126-130 autograd), read only by
 * fbn_bilinear_bwd. */
int fbn_gemm_bf16out(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                     int transA, int transB, void* stream);
/* Split-bf16 x3 (the bf16_fwd backward GEMMs, src/model_fibinet.py:126-134 autograd at ~fp32 accuracy):
 * C = beta C + A_hi B_hi + A_hi B_lo + A_lo B_hi as ONE bf16 MFMA GEMM over K = 3 K0 (LDS-DMA path).
 * A / B are the hi images (bf16, layout as fbn_gemm's bf16 operands), the lo images (x - hi rounded to
 * bf16: fbn_convert_bf16 part 2 writes both) lie lo_a / lo_b elements past them.  K0 % 64 == 0,
 * lda, ldb % 8 == 0, k-major extents % 8; ws: fbn_gemm_workspace_size(M, N, 3 K0, 1) bytes. */
int fbn_gemm_s3(const void* A, const void* B, float* C, int M, int N, int K0, int lda, int ldb, int ldc, int transA,
                int transB, long long lo_a, long long lo_b, float beta, float* ws, size_t ws_bytes, void* stream);
/* bf16 dgrad GEMM C = op(A) op(B) (f32 C, no bias) whose epilogue also computes the first pass of
 * the BatchNorm backward that follows it (src/model_fibinet.py:127-129 autograd: the BN1 backward
 * of the MLP, whose input gradient source G is this C): part = fbn_bn_bwd_fused's column partials
 * ([fbn_bn_bwd_chunks(M, N)][3][N] doubles) from the accumulators, the activation's bf16 image
 * hact16 (its sign is the ReLU / dropout mask), the BN input xpre and mean; hand part to
 * fbn_bn_bwd_fused as part_pre.  _supported: 1 when the shape's tiling gives one row chunk per
 * wave (else FBN_ERR_UNSUPPORTED: run fbn_gemm and the fused BN backward's own pass). */
int fbn_gemm_bn_bwd_part_supported(int M, int N, int K, int lda, int ldb, int transA, int transB);
int fbn_gemm_bn_bwd_part(const void* A, const void* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                         int transA, int transB, const short* hact16, const float* xpre, const float* mean, float scale,
                         double* part, void* stream);
int fbn_gemm_split(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, int lda, int ldb,
                   int ldc, int transA, int transB, int rC_seg, int rC_off0, int rC_off1, float beta, float* stats,
                   float* ws, size_t ws_bytes, const void* A2, int lda2, int kseg, const void* B2, int ldb2, int nseg,
                   void* stream);

/* ---------------------------------------------------------------- K1 + K4: fields + SENET forward
 * Replaces: nn.Embedding lookups (src/model_fibinet.py:155,156,159,167), masked history mean
 * (:165-176), LayerNorm+ReLU of mm_proj (:107-108), torch.stack (:180-182), SENetLayer.forward
 * (:24-35).  table = E [V][D] (pos == NULL) or an exchanged row buffer addressed by
 * pos[B][L+1] (multi-GPU).  map (optional) registers rows for the sparse gradient: the
 * first entry e = b*(L+1)+t touching row r claims it (map[r] = e, slot_row[e] = r; slot_row
 * pre-filled with -1).  D in {16,32,64,128,256}; L <= 32. */
int fbn_fields_fwd(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes, const int64_t* views,
                   const float* hmm, const float* ln_g, const float* ln_b, float ln_eps, const float* cate, int n_cate,
                   const float* table, long long V, const int* pos, const float* w1, const float* b1, const float* w2,
                   const float* b2, int R, float* X, float* Vc, short* Vc16, void* c, int ldc, int c_bf16, float* a_out,
                   float* cnt_out,
                   int* err, int* map, int* slot_row, int B, int L, int D, int rows_bf16, void* stream);
/* Hot-row LDS staging (A/B variant of the gather; single GPU, f32 table under 4 GB).
 * fbn_hot_rows(clear = 0): each batch entry counts its row in cnt [V] (int32, zero on entry) and
 * the entry that brings a row's count to tau appends it to hot [H] (hot_n: count, may exceed H);
 * clear = 1 zeroes those counts and hot_n again.  fbn_fields_fwd_hot = fbn_fields_fwd (pos = NULL,
 * f32 rows) whose workgroups first stage min(hot_n, H, 8192/D) listed rows in LDS and read those
 * from there. */
int fbn_hot_rows(const int64_t* item, const int64_t* seq, int B, int L, long long V, int* cnt, int* hot, int* hot_n,
                 int H, int tau, int clear, void* stream);
int fbn_fields_fwd_hot(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes, const int64_t* views,
                       const float* hmm, const float* ln_g, const float* ln_b, float ln_eps, const float* cate,
                       int n_cate, const float* table, long long V, const float* w1, const float* b1, const float* w2,
                       const float* b2, int R, float* X, float* Vc, short* Vc16, void* c, int ldc, int c_bf16,
                       float* a_out, float* cnt_out, int* err, int* map, int* slot_row, int B, int L, int D,
                       const int* hot, const int* hot_n, int H, void* stream);

/* ---------------------------------------------------------------- K2 + K4 backward
 * Replaces the autograd of the lines above, including embedding_dense_backward with
 * padding_idx=0 (src/model_fibinet.py:100).  Table gradient: dense gtab[V][D] by f32 atomics
 * (gvec == NULL, drop-in), two per-sample vectors gvec[B][2][D] = {dX3, dX5/count} (native
 * trainer: rows resolve through map/slot_row, see fbn_sparse_fixup), or one row per routed
 * entry into sendbuf at pos (multi-GPU).
 * param_grads: host array of 8 device pointers that receive the gradients of {senet W1, b1,
 * W2, b2, LN gamma, beta, cate table, mm_proj bias (may be NULL)}; partials: [fbn_fields_bwd_grid(B,D)][P] scratch with
 * P = fbn_fields_bwd_partials_size.  param_grads == NULL: no reduction launch -- the caller sums
 * the partial rows' segments (6R, R, 6R, 6, D, D, n_cate*D, D columns) with fbn_sum_jobs2 (ld = P). */
int fbn_fields_bwd_partials_size(int D, int R, int n_cate);
int fbn_fields_bwd_grid(int B, int D);
/* Vc16 / dhmm16 / dU16 (optional, may be NULL): bf16 copies written beside the fp32 outputs,
 * the operands of the bf16 GEMMs that consume them (compute_dtype bf16). */
int fbn_fields_bwd(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes, const int64_t* views,
                   const float* hmm, const float* ln_g, const float* ln_b, float ln_eps, const float* w1,
                   const float* b1, const float* w2, int R, int n_cate, const float* cate, const float* X, const float* a, const float* cnt, const float* dV, float* dhmm,
                   short* dhmm16, float* partials, float* const* param_grads, float* gtab, float* gvec,
                   double* gnorm, long long V, const int* pos, void* sendbuf, int send_bf16, int B, int L, int D,
                   void* stream);
/* fbn_fields_bwd with the bf16 copy of dhmm as split images (bf16_fwd training): dhmm_img = bf16(dhmm),
 * lo = bf16(dhmm - hi) B*D elements further (the split-bf16 x3 mm_proj weight gradient's operand). */
int fbn_fields_bwd_img(const int64_t* item_id, const int64_t* item_seq, const int64_t* likes, const int64_t* views,
                       const float* hmm, const float* ln_g, const float* ln_b, float ln_eps, const float* w1,
                       const float* b1, const float* w2, int R, int n_cate, const float* cate, const float* X,
                       const float* a, const float* cnt, const float* dV, float* dhmm, void* dhmm_img,
                       float* partials, float* const* param_grads, float* gtab, float* gvec, double* gnorm,
                       long long V, const int* pos, void* sendbuf, int send_bf16, int B, int L, int D, void* stream);
/* gnorm (optional, with gvec): [B][2] float64 sums of squares of the two per-sample vectors,
 * read by fbn_sumsq_sparse_norms for the clip_grad_norm_ total (src/train_fibinet.py:119).
 * pos / sendbuf (N > 1): one gradient row per routed entry, f32, or bf16 when send_bf16 (the bf16
 * mode's wire format: half the sparse reduce-scatter's bytes; the owner widens on receipt). */

/* ---------------------------------------------------------------- K5 bilinear pair products
 * Replaces the pair loop + stack + cat of src/model_fibinet.py:75-79,89,191-194 ("all", mode 0)
 * and :81-86 ("each", mode 1).  Pairs (0,j) are structurally zero and not stored. */
/* V is read from Vc (fp32) or, when Vc16 is given, from the bf16 copy (bf16 mode; fbn_fields_fwd
 * then writes no fp32 Vc). */
int fbn_pairs_fwd(const float* Vc, const short* Vc16, const float* U, void* c, int B, int D, int ldc, int mode,
                  int c_bf16, void* stream);
/* bf16_fwd training, bilinear "all" (src/model_fibinet.py:60-66 pair products): the MLP input c =
 * [V | pairs] written ONLY as split-bf16 images (bf16 hi at c_img[b*ldc + j], lo = bf16(x - hi)
 * B*ldc elements further) -- the operands of the layer-1 GEMM (hi) and of fbn_gemm_s3 / the
 * split-bf16 x3 slab GEMMs; and the lo image of V (vc_img: [B][5][D] hi = fbn_fields_fwd's Vc16,
 * lo 5*B*D further, written here; vc_img may be null). */
int fbn_pairs_fwd_img(const float* Vc, const float* U, void* c_img, void* vc_img, int B, int D, int ldc, void* stream);
/* fbn_pairs_bwd (bilinear "all") with dU written only as split-bf16 images (hi [B][5][D], lo 5*B*D
 * elements further). */
int fbn_pairs_bwd_img(const float* dc, const float* Vc, const float* U, float* dV, void* dU_img, int B, int D, int ldc,
                      void* stream);
int fbn_pairs_bwd(const float* dc, const float* Vc, const short* Vc16, const float* U, float* dV, float* dU,
                  short* dU16, int B, int D, int ldc, int mode, void* stream);

/* ---------------------------------------------------------------- K6 BatchNorm + ReLU + dropout
 * Replaces nn.BatchNorm1d / ReLU / Dropout(0.2) of src/model_fibinet.py:127-133.  The stats
 * entry points split into local passes and finalize so that a SyncBN all-reduce of the
 * float64 sums can run in between (multi-GPU). */
size_t fbn_bn_workspace_size(int B, int C);
int fbn_bn_stats_pass(const float* X, int B, int C, const double* mean_d, double* out_d, void* ws, void* stream);
int fbn_bn_mean(const double* sum_d, double ntot, int C, double* mean_d, void* stream);
int fbn_bn_finalize(const double* m2_d, const double* mean_d, double ntot, int C, float* mean, float* invstd,
                    float* run_mean, float* run_var, float momentum, float eps, int update_running, void* stream);
int fbn_bn_stats(const float* X, int B, int C, float* mean, float* invstd, float* run_mean, float* run_var,
                 float momentum, float eps, int update_running, void* ws, void* stream);
/* BN statistics from fbn_gemm tile partials: mean_d == NULL -> out = column sums; else
 * out = column sums of squared deviations about mean_d (Chan merge, f64). */
int fbn_bn_tile_stats(const float* part, int M, int C, const double* mean_d, double* out_d, void* stream);
/* Single-process form of the above + fbn_bn_mean + fbn_bn_finalize in one launch (same f64
 * operations in the same order; the multi-GPU path needs the all-reduces in between). */
/* SyncBN (multi-GPU) with one all-reduce per layer: per-rank raw moments out[2C] = {sum x,
 * sum x^2} from the tile partials, all-reduced by the caller, then the finalize. */
int fbn_bn_tile_moments(const float* part, int M, int C, double* out_d, void* stream);
int fbn_bn_moments_finalize(const double* mom_d, double ntot, int C, float* mean, float* invstd, float* run_mean,
                            float* run_var, float momentum, float eps, int update_running, void* stream);
int fbn_bn_tile_finalize(const float* part, int M, int C, double ntot, float* mean, float* invstd, float* run_mean,
                         float* run_var, float momentum, float eps, int update_running, void* stream);
int fbn_bn_eval_params(const float* run_mean, const float* run_var, float* mean, float* invstd, int C, float eps,
                       void* stream);
/* Y (f32) or Y16 (bf16) may be null (not both). */
int fbn_bn_act_fwd(const float* X, float* Y, int B, int C, const float* mean, const float* invstd, const float* g,
                   const float* b, float p_drop, const unsigned long long* rng, unsigned stream_id,
                   unsigned char* mask_out, const unsigned char* mask_in, short* Y16, void* stream);
/* fbn_bn_act_fwd with the bf16 output as split images (bf16_fwd training): Y_img = bf16(y) (the
 * layer-2 GEMM operand), lo = bf16(y - hi) B*C elements further; Y (fp32) may be null. */
int fbn_bn_act_fwd_img(const float* X, float* Y, int B, int C, const float* mean, const float* invstd, const float* g,
                       const float* b, float p_drop, const unsigned long long* rng, unsigned stream_id,
                       unsigned char* mask_out, const unsigned char* mask_in, void* Y_img, void* stream);
/* fbn_bn_act_fwd of the last hidden layer (C = 256) fused with fbn_head_fwd (same outputs).
 * bwd_part (optional, with labels / gout; fbn_bn_bwd_chunks(B, C) * 3 * C doubles): the first pass
 * of this layer's BN backward (rank-1 source gout x hw, dropout scale bwd_scale), handed to
 * fbn_bn_bwd_fused as part_pre. */
int fbn_bn_act_head_fwd(const float* X, float* Y, int B, int C, const float* mean, const float* invstd, const float* g,
                        const float* b, float p_drop, const unsigned long long* rng, unsigned stream_id,
                        unsigned char* mask_out, const unsigned char* mask_in, const float* hw, const float* hbias,
                        float* logits, float* probs, const float* labels, float* loss_terms, float* gout, float denom,
                        double* bwd_part, float bwd_scale, void* stream);
int fbn_bn_bwd_reduce(const float* G, const float* gvec, const float* w, const float* hact, float scale,
                      const float* Xpre, const float* mean, int B, int C, double* red_d, void* ws, void* stream);
int fbn_bn_bwd_apply(const float* G, const float* gvec, const float* w, const float* hact, float scale,
                     const float* Xpre, const float* mean, const float* invstd, const float* gamma, int B, int C,
                     const double* red_d, double ntot, float* dXpre, short* dXpre16, float* dgamma, float* dbeta,
                     float* dw, void* ws, void* stream);
int fbn_bn_bwd(const float* G, const float* gvec, const float* w, const float* hact, float scale, const float* Xpre,
               const float* mean, const float* invstd, const float* gamma, int B, int C, float* dXpre, float* dgamma,
               float* dbeta, float* dw, void* ws, void* stream);
/* Single-process BN backward in three launches (partials -> reduce + finalize -> vectorised
 * apply).  colpart (optional, fbn_bn_colpart_size bytes): per-row-chunk column sums of dXpre =
 * the partials of the preceding Linear's bias gradient (finalised by fbn_sum_jobs). */
size_t fbn_bn_colpart_size(int B, int C);
int fbn_row_chunks(int B);
/* row chunks of fbn_bn_bwd_fused (its colpart is [fbn_bn_bwd_chunks(B, C)][C]) */
int fbn_bn_bwd_chunks(int B, int C);
/* hact16 (bf16 image of the activation) may replace hact (null) for a matrix source G: the ReLU /
 * dropout mask needs only the sign.  dXpre or dXpre16 may be null (not both). */
int fbn_bn_bwd_fused(const float* G, const float* gvec, const float* w, const float* hact, const short* hact16,
                     float scale, const float* Xpre, const float* mean, const float* invstd, const float* gamma, int B,
                     int C, double ntot, float* dXpre, short* dXpre16, float* dgamma, float* dbeta, float* dw,
                     float* colpart, const double* part_pre, void* ws, void* stream);
/* fbn_bn_bwd_fused with the bf16 output as split images (bf16_fwd training): dXpre_img = bf16(dx),
 * lo = bf16(dx - hi) B*C elements further -- the operands of the split-bf16 x3 backward GEMMs. */
int fbn_bn_bwd_fused_img(const float* G, const float* gvec, const float* w, const float* hact, const short* hact16,
                         float scale, const float* Xpre, const float* mean, const float* invstd, const float* gamma,
                         int B, int C, double ntot, float* dXpre, void* dXpre_img, float* dgamma, float* dbeta,
                         float* dw, float* colpart, const double* part_pre, void* ws, void* stream);
/* bf16 images: jobs = host array of n <= 16 records
 * {const float* src; short* dst; int rows, cols, ld, trans, seg, off0, off1, part, dld, pst;}
 * x = trans ? src[j*ld + rm(i)] : src[i*ld + rm(j)], rm(x) = x + (x < seg ? off0 : off1);
 * hi = bf16(x), lo = bf16(x - float(hi));  dst[i*dld + j] = part ? lo : hi  (dld = 0: cols).  part 1
 * is the rounding residual: hi + lo carry 16 significant bits.  part 2 writes both from one read,
 * lo pst elements past hi: the operand images of fbn_gemm_s3 / split-bf16 x3 slab GEMMs. */
int fbn_convert_bf16(const void* jobs, int n, void* stream);
size_t fbn_colsum_workspace_size(int B, int C);
int fbn_colsum(const float* X, int B, int C, int ldx, float* out, float beta, void* ws, void* stream);
/* column partials only: part[fbn_row_chunks(B)][C] (finalised by fbn_sum_jobs) */
int fbn_colsum_partial(const float* X, int B, int C, int ldx, float* part, void* stream);
/* Deferred sums of one step in ONE launch: jobs = host array of n <= 16 records
 * {const float* part; float* out; int nch, C; float scale, beta; int ld, pad;}:
 * out[c] = beta * out[c] + scale * sum_{k < nch} part[k * ld + c]   (ld 0 = C; fixed-order tree).
 * Used for the bias gradients (sum over the batch, autograd of src/model_fibinet.py:105,126,130,134),
 * the fields' small parameter gradients and the mean BCE loss (src/train_fibinet.py:115).
 * fbn_sum_jobs2 adds, in the same launch, ns <= 8 slab jobs {const float* ws; float* out; int M, N,
 * ldc, nsplit, seg, off0, off1; float beta;}: out[m*ldc + n + (n < seg ? off0 : off1)] =
 * beta*out + sum_{z < nsplit} ws[z][m][n] -- the split-K slabs fbn_gemm_slabs left (N, ldc and the
 * remap multiples of 4, buffers 16-B aligned). */
int fbn_sum_jobs(const void* jobs, int n, void* stream);
int fbn_sum_jobs2(const void* jobs, int n, const void* slabs, int ns, void* stream);

/* ---------------------------------------------------------------- K7 head: Linear(256,1)+sigmoid+BCE
 * Replaces src/model_fibinet.py:134,136,199 and nn.BCELoss fwd/bwd (src/train_fibinet.py:79,115). */
int fbn_head_fwd(const float* H, const float* w, const float* bias, int B, int C, float* logits, float* probs,
                 const float* labels, float* loss_terms, float* gout, float denom, void* stream);
int fbn_sigmoid_bwd(const float* gp, const float* probs, float* gout, int B, void* stream);
int fbn_outer(const float* g, const float* w, float* out, int B, int C, void* stream);
int fbn_sum(const float* x, int n, float* out, float scale, void* stream);

/* ---------------------------------------------------------------- K8 + K9 clip + Adam
 * Replaces clip_grad_norm_(10) (src/train_fibinet.py:119) and torch.optim.Adam with coupled L2
 * (:78,121); the schedule table carries OneCycleLR's lr/beta1 per step (:84-92,122): 8 floats per
 * step {1-beta1, -lr/bc1, sqrt(bc2), 1/sqrt(bc2), dmul, 0, 0, 0}, dmul = 1 - lr*wd for the opt-in
 * AdamW (config/fibinet_config.yaml:62; pass wd = 0 then), 1 for Adam. */
int fbn_sumsq(const float* x, long long n, const int* n_rows, int row_len, double* out, void* stream);
int fbn_clip_coef(const double* sumsq, float max_norm, float* coef, float* norm, void* stream);
/* sumsq (optional): the FBN_SUMSQ_SLOTS norm accumulators -- the kernel then applies
 * clip_grad_norm_(max_norm) itself (same arithmetic as fbn_clip_coef) and writes the coefficient
 * and the total norm to coef_out / norm_out for the table passes that follow; else coef is read. */
int fbn_adam_dense(float* p, const float* g, float* m, float* v, long long n, const float* coef,
                   const void* consts_table, const int* step, float wd, float beta2, float eps, const double* sumsq,
                   float max_norm, float* coef_out, float* norm_out, void* stream);
/* Sparse table gradient.  Slots are entry indices; gvec is the per-sample vector buffer of
 * fbn_fields_bwd (Lp1 = L+1) or the owner's received per-entry rows (Lp1 = 1).  fixup folds
 * entries whose row was claimed by another entry into that claimer (extra[] + a flag bit in
 * slot_row for the single-GPU layout, in place for the owner layout); sumsq_sparse and
 * adam_table read the gradient of row r as gvec-slot(map[r]) (+ extra). */
int fbn_sparse_fixup(const int64_t* item, const int64_t* seq, const int* ids, int n, int L, long long V, int rank,
                     const int* map, const float* gvec, float* extra, int* slot_row, int Lp1, int D, void* stream);
int fbn_sumsq_sparse(const float* gvec, float* extra, int* slot_row, int Lp1, int n, int D, double* out,
                     void* stream);
/* Single-GPU fast forms: fixup from the claim-time duplicate list dup[n] of fbn_claim_rows (no
 * id re-resolution through map), and the table-gradient sum of squares from fbn_fields_bwd's
 * per-sample norms gnorm[B][2] (vectors re-read only for rows with duplicates). */
int fbn_sparse_fixup_dup(const int* dup, int n, const float* gvec, float* extra, int* slot_row, int Lp1, int D,
                         void* stream);
/* dense (optional, n_dense % 4 == 0, 16-B aligned): also adds the squares of a dense gradient
 * vector to out (fbn_sumsq's work in the same launch). */
int fbn_sumsq_sparse_norms(const double* gnorm, const float* gvec, float* extra, int* slot_row, int Lp1, int n, int D,
                           double* out, unsigned long long* fx, const float* dense, long long n_dense, void* stream);
/* Deterministic mode (no float atomics on the table gradient): every entry of a row several
 * entries hit -- claimer included -- adds its vector into acc[claimer] ([n][D] int64 fixed point,
 * scale 2^40: order-independent sums); claimers are flagged.  fbn_sumsq_sparse_norms(fx = acc)
 * then writes the FULL row gradient to extra[claimer] (and resets acc): pass Lp1 | FBN_GRAD_FULL
 * to the table-Adam entry points so they read it as the whole gradient.  hasdup [n]: set by the
 * row claims (fbn_claim_rows / fbn_adam_claim_catchup), cleared here. */
#define FBN_GRAD_FULL 0x10000
/* Lp1 | FBN_GRAD_CELL: the gradient-row pointer argument is the address of a device cell holding the
 * row pointer (written by fbn_ring_slot) -- readers resolve it on the device */
#define FBN_GRAD_CELL 0x20000
/* Lp1 | FBN_GRAD_BF16 (per-entry rows, Lp1 == 1): the rows are bf16 -- the sharded owner's deferred-gradient
 * ring in bf16 mode keeps the wire's bf16 gradient rows as they arrived (widened on every read: the same
 * f32 values as a widened f32 ring, half its bytes). */
#define FBN_GRAD_BF16 0x40000
/* ring_n | FBN_RING_BF16 wherever a deferred-gradient ring is passed (pend / ring / coef_hist / ring_stride /
 * ring_n argument groups, fbn_owner_fold): the ring's rows are bf16 and ring_stride counts bf16 elements
 * (sharded owner, Lp1 == 1 only; fbn_ring_slot and fbn_sparse_fixup refuse it). */
#define FBN_RING_BF16 0x40000000
int fbn_sparse_fold_fx(const int* dup, int* hasdup, int n, const float* gvec, int* slot_row, int Lp1, int D,
                       unsigned long long* acc, void* stream);
/* adam_table mode 0: every row (touched rows read their gradient through map); mode 1: only the
 * rows the batch did not touch -- their gradient is 0, so the update is independent of the
 * backward and the clip coefficient and runs on a side stream concurrently with the backward;
 * adam_touched then updates the claimed rows (one group per claiming entry) and resets map. */
int fbn_adam_table(float* p, float* m, float* v, long long nrows, int D, int* map, const float* gvec, float* extra,
                   int* slot_row, int Lp1, const float* coef, const void* consts_table, const int* step, float wd,
                   float beta2, float eps, int mode, void* stream);
int fbn_adam_touched(float* p, float* m, float* v, int D, int* map, const float* gvec, float* extra, int* slot_row,
                     int Lp1, int n, const float* coef, const void* consts_table, const int* step, float wd,
                     float beta2, float eps, int* last, void* stream);
/* Row-state record.  Every `last`, `pend` and `preclaim` argument below is a FIELD of one 16-B
 * record per table row, {uint64 preclaim; int32 last; int32 pend} (FBN_ROW_STATE_BYTES): pass the
 * record array's base as preclaim, base + 8 B as last, base + 12 B as pend; the kernels index each
 * field with the 16-B record stride, so a claim reads a row's whole state in one sector. */
#define FBN_ROW_STATE_BYTES 16
/* Lazy table Adam (bit-identical to the eager table pass): last[r] = Adam steps applied to row r.  fbn_adam_catchup replays the
 * zero-loss-gradient steps (coupled L2 decay only: g = 0*coef + wd*p) of the rows claimed in
 * slot_row and of rolling window (step mod F) (ceil(nrows/F) rows) up to *step, with the same
 * float operations in the same order as stepping them (bit-identical); fbn_adam_touched(last)
 * then applies the step with the gradient; fbn_adam_flush brings every row up to date.
 * Replaces the per-step dense Adam pass of torch.optim.Adam over item_emb.weight
 * (src/train_fibinet.py:78,121) by O(touched + nrows/F) rows per step.  F <= 512. */
/* parts: 1 = claimed rows (before the gather), 2 = rolling window (unclaimed rows; may overlap the
 * step on another stream), 3 = both. */
/* Deferred gradients (single GPU; pend == NULL disables): pend[r] = index b*2+slot of the
 * per-sample gradient vector row r received at step last[r] (-1 = none); ring [ring_n][B][2][D]
 * holds step s's vectors in slot s % ring_n (ring_stride = B*2*D floats, ring_n > F);
 * coef_hist[s] = step s's clip coefficient.  A replay applies that step with the gradient first. */
/* decoupled: the opt-in AdamW mode (weight decay by the schedule table's dmul = 1 - lr*wd per
 * step, wd = 0 in the gradient); 0 = Adam with coupled L2, the reference's optimizer. */
int fbn_adam_catchup(float* p, float* m, float* v, long long nrows, int D, const int* slot_row, int n_ent,
                     const int* map, int F, int parts, int* last, const void* consts_table, const int* step, float wd,
                     float beta2, float eps, int* pend, const float* ring, const float* coef_hist,
                     long long ring_stride, int ring_n, int decoupled, void* stream);
/* Single GPU: fbn_claim_rows + fbn_adam_catchup(parts = 1) in ONE launch -- each entry claims its
 * row (first CAS wins: map, slot_row, dup as fbn_claim_rows) and a winning entry's row is brought
 * up to date at once.  preclaim (optional, [V] u64, zero-initialised): tagged claims made for THIS
 * batch by the previous step's fbn_adam_prefetch -- an entry whose tag is the current step takes
 * the claim from it without a CAS (the smallest entry index of each row claims); pass it only when
 * that prefetch was given this very batch. */
/* N > 1 owner (the fixed-capacity exchange): claims of the received local rows lids [n] (negative =
 * empty slot; skip0: rank 0's row 0 is padding) + the claimed-row catch-up in one launch; preclaim
 * (optional): fbn_adam_prefetch_rows' tags for this very routing -- a row tagged for this step is
 * claimed by its smallest slot without a CAS. */
int fbn_adam_owner_claim_catchup(const int* lids, int n, int skip0, int* map, int* slot_row,
                                 unsigned long long* preclaim, float* p, float* m, float* v, long long nrows, int D,
                                 int F, int* last, const void* consts_table, const int* step, float wd, float beta2,
                                 float eps, int* pend, const float* ring, const float* coef_hist, long long ring_stride,
                                 int ring_n, int decoupled, void* stream);
int fbn_adam_claim_catchup(const int64_t* item, const int64_t* seq, int B, int L, long long V, int* map, int* slot_row,
                           int* dup, int* hasdup, unsigned long long* preclaim, float* p, float* m, float* v,
                           long long nrows, int D, int F, int* last,
                           const void* consts_table, const int* step, float wd, float beta2, float eps, int* pend,
                           const float* ring, const float* coef_hist, long long ring_stride, int ring_n, int decoupled,
                           void* stream);
/* fbn_adam_claim_catchup with the step's bf16 image conversion (fbn_convert_bf16's n_conv <= 16
 * job records) in the same launch (claim blocks, then conversion blocks) -- the two are
 * independent: the images are of the weights the previous step's tail wrote and of this batch's
 * item_emb_d128 (src/model_fibinet.py:162). */
int fbn_adam_claim_catchup_conv(const int64_t* item, const int64_t* seq, int B, int L, long long V, int* map,
                                int* slot_row, int* dup, int* hasdup, unsigned long long* preclaim, float* p,
                                float* m, float* v, long long nrows, int D, int F, int* last,
                                const void* consts_table, const int* step, float wd, float beta2, float eps,
                                int* pend, const float* ring, const float* coef_hist, long long ring_stride,
                                int ring_n, int decoupled, const void* conv_jobs, int n_conv, void* stream);
/* Single GPU, D = 128 / 256: ahead-of-time catch-up of the NEXT batch's rows during this step, on
 * the rolling window's stream after this step's claims and before its step tail.  A next-batch row
 * that this batch does not touch (map == -1) takes only zero-gradient steps through the current
 * step inclusive, so it is brought to last = step + 1 now (bit-identical to eager Adam); the next
 * step's claimed-row catch-up then finds it up to date.  Replaces the reference's dense Adam over
 * item_emb.weight (train_fibinet.py:78,121) for those rows, one step early.  preclaim (optional):
 * every next-batch entry also records its tagged claim there (non-returning atomic max), for the
 * next step's fbn_adam_claim_catchup. */
int fbn_adam_prefetch(const int64_t* item, const int64_t* seq, int B, int L, long long V, const int* map,
                      unsigned long long* preclaim, float* p, float* m, float* v, int D, int* last,
                      const void* consts_table, const int* step, float wd, float beta2, float eps, int* pend,
                      const float* ring, const float* coef_hist, long long ring_stride, int ring_n, int decoupled,
                      void* stream);

/* fbn_adam_prefetch (two-pass form: preclaim required; D = 128 / 256) with the replay balanced
 * longest-first: a binning pass makes the same claims and appends each owned row's record to a bin
 * by replay length (one 128-B counter line per (bin, block % 8)); the replay pass hands every wave a
 * chunk of 64 records of one bin, longest bins first.  Bit-identical to fbn_adam_prefetch.
 * ws: fbn_adam_prefetch_binned_ws_size(B * (L + 1)) bytes of device scratch (reused every call). */
size_t fbn_adam_prefetch_binned_ws_size(long long n);
int fbn_adam_prefetch_binned(const int64_t* item, const int64_t* seq, int B, int L, long long V, const int* map,
                             unsigned long long* preclaim, float* p, float* m, float* v, int D, int* last,
                             const void* consts_table, const int* step, float wd, float beta2, float eps, int* pend,
                             const float* ring, const float* coef_hist, long long ring_stride, int ring_n,
                             int decoupled, void* ws, size_t ws_bytes, void* stream);

/* N > 1, the owner's side, D = 128 / 256: fbn_adam_prefetch over local rows lids [n] (-1 = none;
 * skip0: row 0 is the padding id, rank 0) -- the rows the NEXT step's requests name, received
 * through fbn_pad_routes + an equal-split all-to-all during this step.  preclaim (the row-state
 * records' tag field, optional): the two-pass form -- tagged pre-claims decide each row's entry with
 * one non-returning atomic, the four-row engine replays; NULL: the one-pass kernel. */
int fbn_adam_prefetch_rows(const int* lids, int n, int skip0, long long nrows, const int* map,
                           unsigned long long* preclaim, float* p, float* m, float* v, int D, int* last,
                           const void* consts_table, const int* step, float wd, float beta2, float eps, int* pend,
                           const float* ring, const float* coef_hist, long long ring_stride, int ring_n,
                           int decoupled, void* stream);
int fbn_adam_flush(float* p, float* m, float* v, long long nrows, int D, int* last, const void* consts_table,
                   const int* step, float wd, float beta2, float eps, int* pend, const float* ring,
                   const float* coef_hist, long long ring_stride, int ring_n, int decoupled, void* stream);
/* Single-GPU step tail in ONE launch: fbn_adam_dense (clip from the sumsq slots) on the flat dense
 * parameters + fbn_adam_commit on the table + fbn_step_end; ticket = FBN_TICKET_WORDS device
 * unsigneds, zero before the first call (the kernel resets them); max_step / err as fbn_step_end. */
#define FBN_TICKET_WORDS 17
int fbn_adam_step_tail(float* dp, const float* dg, float* dm, float* dv, long long n_dense, const double* sumsq,
                       float max_norm, float* coef_out, float* norm_out, float* p, float* m, float* v, int D, int* map,
                       const float* gvec, float* extra, int* slot_row, int Lp1, int n, const void* consts_table,
                       int* step, float wd, float beta2, float eps, int* last, int* pend, float* ring,
                       float* coef_hist, int ring_n, long long ring_stride, int B, unsigned long long* rng,
                       long long* nbt0, long long* nbt1, unsigned* ticket, int max_step, int* err, void* stream);
/* (step tail) Lp1 >= 2: per-sample vectors gvec [B][2][D] copied into ring slot step % ring_n
 * (ring_stride = B*2*D); Lp1 == 1 (N > 1 owner): per-entry rows gvec [n][D] already received into
 * that ring slot (ring_stride = the slot's row capacity x D), pend[r] = the claiming entry. */
/* Self-test of the table-row Adam step (hardware sqrt / rcp, fused moment updates; used by every
 * item_emb.weight kernel) against the IEEE element step of fbn_adam_dense: n x 4 random operands
 * in training ranges; dev[0..2] = max deviation of m, v, p in 1/16 ulp of each update's largest
 * term (device counters, caller zeroes). */
int fbn_adam_selftest(int n, unsigned seed, unsigned long long* dev, void* stream);
/* Single-GPU end of step with deferred table gradients (replaces fbn_adam_touched + the slot_row
 * reset): a claiming entry without duplicates records its vector in pend (applied at the row's
 * next replay); one with duplicates (FLAG) is updated now; map and slot_row are reset; the step's
 * vectors go to ring slot step % ring_n and the clip coefficient to coef_hist[step]. */
int fbn_adam_commit(float* p, float* m, float* v, int D, int* map, const float* gvec, float* extra, int* slot_row,
                    int Lp1, int n, const float* coef, const void* consts_table, const int* step, float wd,
                    float beta2, float eps, int* last, int* pend, float* ring, float* coef_hist, int ring_n, int B,
                    void* stream);

/* sumsq accumulators are FBN_SUMSQ_SLOTS (= 64) doubles; fbn_clip_coef sums them and
 * fbn_step_end zeroes them.  fbn_claim_rows registers the rows of a batch in map/slot_row (the
 * same claims fbn_fields_fwd makes when given a map), as a tiny kernel at the start of a step. */
#define FBN_SUMSQ_SLOTS 64
/* dup (optional, [B*(L+1)]): the claiming entry of each entry's row when another entry claimed
 * it, else -1 (input of fbn_sparse_fixup_dup). */
int fbn_claim_rows(const int64_t* item, const int64_t* seq, int B, int L, long long V, int* map, int* slot_row,
                   int* dup, int* hasdup, void* stream);
/* Multi-GPU: pack {loss, this rank's table-gradient sumsq (slots zeroed)} into the two floats
 * appended to the dense-gradient all-reduce buffer; unpack after it (sumsq[0] += table norms). */
int fbn_pack_extras(const float* loss, double* tab_slots, float* out, void* stream);
int fbn_unpack_extras(const float* in, float* loss, double* sumsq, void* stream);
/* fbn_unpack_extras + fbn_sumsq(x, n) in one launch (N > 1: after the all-reduce, the dense
 * gradients' sum of squares beside the unpacked table sumsq). */
int fbn_unpack_sumsq(const float* in, float* loss, const float* x, long long n, double* sumsq, void* stream);
/* end of step: step counter, dropout counter, zero the sumsq slots, and the BatchNorm
 * num_batches_tracked buffers (nbt0 / nbt1 may be NULL; model_fibinet.py:127,131 BN1d).
 * max_step (= total_steps): the counter saturates there and sets bit 2 of *err (err may be NULL)
 * -- OneCycleLR raises past total_steps (train_fibinet.py:84-92); a replayed hipGraph cannot, so
 * the device keeps every schedule read in bounds and the host raises at its next check. */
int fbn_step_end(int* step, unsigned long long* rng, double* sumsq, long long* nbt0, long long* nbt1, int max_step,
                 int* err, void* stream);

/* ---------------------------------------------------------------- row-sharded exchange (multi-GPU)
 * Replaces torch.nn.DataParallel's replicate/scatter of the whole table (src/train_fibinet.py:69-70)
 * by routing ids to the owner of each row block; RCCL all-to-all runs between these calls. */
int fbn_route(const int64_t* item, const int64_t* seq, int B, int L, long long V, long long Vl, int nranks,
              int* counts, int* offsets, int* cursor, int* send_ids, int* pos, int* err, void* stream);
/* The fixed-capacity exchange (RowExchange, default at N > 1): every requester -> owner block has
 * cap + 1 slots, so the ids, the looked-up rows and the gradient rows cross as equal-split
 * all-to-alls and no split size ever reaches the host (the step can be recorded as a step program).
 * send_ids [nranks][cap + 1]: owner o's block holds the local rows routed to o in slots 0..cap-1,
 * -1 in unused slots; pos[b][t] = o * (cap + 1) + k (-1 = not routed).  An entry past slot cap - 1
 * is not routed: stat[0] = 1 and every block's last slot is -2 (the flag travels in-band).
 * stat [nranks + 1] = {overflow, entries requested from owner 0 .. nranks-1}.  Owner-side kernels
 * (fbn_owner_claim / fbn_owner_gather / fbn_sparse_fixup / fbn_adam_prefetch_rows) skip negative ids.
 * fbn_route_fc_status (after the ids all-to-all, recv_ids as received): stat[0] |= any requester's
 * flag -- the same on every rank -- and stat[0 .. nranks] is copied to host (pinned, may be NULL) on
 * the stream: a set flag makes every rank exchange that step with host-side split sizes instead.
 * send_ids non-NULL: the all-to-all skipped the caller's own block (fbn_comm_alltoall_peers), which
 * is copied from send_ids into recv_ids first. */
int fbn_route_fc(const int64_t* item, const int64_t* seq, int B, int L, long long V, long long Vl, int nranks,
                 int cap, int* send_ids, int* pos, int* stat, int* err, void* stream);
int fbn_route_fc_status(const int* send_ids, int* recv_ids, int nranks, int rank, int cap, int* stat, int* host,
                        void* stream);
/* fbn_owner_gather with the caller's own block redirected: entries [self_lo, self_lo + self_n) are
 * written to self_out (same index) -- the requester's row buffer, so that block never crosses RCCL
 * (the fixed-capacity exchange's all-to-alls skip it: fbn_comm_alltoall_peers). */
int fbn_owner_gather_self(const int* ids, int n, const float* E, void* out, int* map, int* slot_row, int rank, int D,
                          int out_bf16, void* self_out, int self_lo, int self_n, void* stream);
/* claims only (the lazy table Adam replays the claimed rows before fbn_owner_gather(map = NULL)) */
int fbn_owner_claim(const int* ids, int n, int* map, int* slot_row, int rank, void* stream);
/* out_bf16: reply rows as bf16 (the bf16 mode's wire format; fbn_fields_fwd(rows_bf16 = 1) reads them) */
int fbn_owner_gather(const int* ids, int n, const float* E, void* out, int* map, int* slot_row, int rank, int D,
                     int out_bf16, void* stream);
/* N > 1 owner with deferred table gradients: the received gradient rows `wire` (n floats; bf16 when
 * wire_bf16, else f32; n % 8 == 0, n <= stride) widened / copied into ring slot (*step % ring_n) of
 * ring [ring_n][stride]; *cell = that slot's address (pass cell with Lp1 | FBN_GRAD_CELL to
 * fbn_sparse_fixup / fbn_sumsq_sparse / fbn_adam_step_tail) -- the slot is chosen on the device, so
 * a recorded step program replays with the right slot.  Elements [self_lo, self_lo + self_n) are read
 * from wire_self instead (the caller's own block, never sent: the requester's gradient rows). */
int fbn_ring_slot(float* ring, int ring_n, long long stride, const int* step, void* cell, const void* wire,
                  int wire_bf16, long long n, const void* wire_self, long long self_lo, long long self_n,
                  void* stream);
/* N > 1 owner, the fixed-capacity exchange: fbn_ring_slot + the duplicate fold in one pass.  Slot e
 * (local row ids[e]; negative = empty; rank 0's row 0 = padding): the claimer of its row
 * (map[row] == e) stores its widened row into ring slot (*step % ring_n) [stride floats per slot;
 * *cell = its address]; a duplicate adds its row into extra[claimer] (zero at rest) and flags the
 * claimer in slot_row (FBN_SLOT_FLAG).  Readers take (cell, extra, Lp1 = 1 | FBN_GRAD_CELL); the step
 * tail applies flagged claimers at once and zeroes their extra rows.  Rows [self_lo, self_lo +
 * self_n) come from wire_self (the caller's own block, never sent). */
int fbn_owner_fold(const int* ids, int n, int rank, const int* map, int* slot_row, const void* wire, int wire_bf16,
                   const void* wire_self, long long self_lo, long long self_n, float* ring, int ring_n,
                   long long stride, const int* step, void* cell, float* extra, int D, double* part,
                   unsigned long long* fx, void* stream);
/* part (optional, 8192 doubles): fbn_owner_fold leaves one partial sum of the claimers' own rows' squares
 * per workgroup; fbn_sumsq_flagged (same n and D) folds them and adds each flagged claimer's
 * |x + extra|^2 - |x|^2 (x read through the ring slot's pointer cell) into sumsq (FBN_SUMSQ_SLOTS
 * doubles): together the table gradient's sum of squares (clip_grad_norm_, src/train_fibinet.py:119)
 * without a pass over every row.
 * fx (optional, [n][D] int64, zero at rest): deterministic mode (src/utils.py:15-16).
 * fbn_owner_fold adds each duplicate's row into fx[claimer] as fixed point (2^-40) instead of float
 * atomics into extra; fbn_sumsq_flagged (same fx) adds the claimer's own row, writes the FULL row
 * gradient float(total) to extra[claimer] and resets fx -- readers then take Lp1 = 1 | FBN_GRAD_CELL |
 * FBN_GRAD_FULL.  The fold is bitwise reproducible and equal to the single-GPU deterministic fold on
 * the same entries; with fx, fbn_sumsq_flagged runs on at most FBN_SUMSQ_SLOTS workgroups (one f64
 * addition per norm slot).  ring_bf16: the claimers' own rows behind `cell` are bf16 (FBN_RING_BF16). */
int fbn_sumsq_flagged(const int* slot_row, int n, const void* cell, float* extra, int D, const double* part,
                      double* sumsq, unsigned long long* fx, int ring_bf16, void* stream);
/* bf16 -> f32 (n % 8 == 0, 16-B aligned): the owner's received bf16 gradient rows (bf16 mode). */
int fbn_widen_bf16(const void* in, float* out, long long n, void* stream);
/* out [world][cap + 1]: out[o][j] = send_ids[offsets[o] + j] for j < counts[o], else -1, and
 * out[o][cap] = -2 - counts[o] -- the routing of the NEXT batch as ONE equal-split all-to-all (no
 * host-side counts, no counts all-to-all); negative slots read as "no row" in
 * fbn_adam_prefetch_rows (n = world * (cap + 1)). */
int fbn_pad_routes(const int* send_ids, const int* offsets, const int* counts, int world, int cap, int* out,
                   void* stream);
/* The owner's side of that exchange (padded [world][cap + 1] as received): counts[r] = entries rank r
 * requests, ids = the requests packed in rank order (= the host-split ids all-to-all's result);
 * 1 <= world <= 64. */
int fbn_compact_routes(const int* padded, int world, int cap, int* ids, int* counts, void* stream);
/* Up to 8 device-to-device copies in one launch (bytes and addresses multiples of 16): a step's
 * inputs into the static buffers of the trainer's captured compute segments (N > 1). */
int fbn_copy_jobs(const void* const* src, void* const* dst, const long long* bytes, int n, void* stream);

/* ---------------------------------------------------------------- fused bilinear (bf16 mode, "all")
 * Replaces BilinearInteraction "all" (src/model_fibinet.py:60-79,89) and its autograd in ONE launch
 * each way, MFMA for the W contraction, pair products in the epilogue:
 *   fwd: c[:, 5D + k*D + n] (bf16) = V_i (.) (V_j W) for pair k = (i, j)   (V16 [B][5][D] bf16,
 *        WT16 = W^T [D][D] bf16); U = V W is never stored;
 *   bwd: dU16 [B][5][D] (bf16) and dV [B][5][D] (f32) = dc_V + pair terms + dU W^T from dc [B][ldc]
 *        (V block at 0, pairs at 5D; f32, or bf16 when dc_bf16 -- fbn_gemm_bf16out's output),
 *        recomputing U on the MFMA (W16 = W [D][D] bf16).
 * fbn_bilinear_supported(D): 1 for the D these kernels are built for (64, 128). */
int fbn_bilinear_supported(int D);
int fbn_bilinear_fwd(const short* V16, const short* WT16, short* c, int B, int D, int ldc, void* stream);
int fbn_bilinear_bwd(const void* dc, int ldc, int dc_bf16, const short* V16, const short* WT16, const short* W16,
                     float* dV, short* dU16, int B, int D, void* stream);

/* ---------------------------------------------------------------- device collator
 * Replaces BatchCollator.__call__ (src/dataloader.py:69-121) and InferenceCollator.__call__
 * (src/Prediction.py:28-52): batch row b = dataset row perm[b] of HBM-resident columns item [N],
 * seq [N][Ls] (the last L columns are kept: src/dataloader.py:111-116), likes, views, user [N]
 * int64 and label [N] f32 (any of those may be NULL), and o_emb[b] = emb[slot_of_id[item]] (the
 * item_info lookup of :91-95; E floats per row).  An item id without an item_info row gets a zero
 * row and sets *missing (the training collator's KeyError, raised by the host when it checks).
 * sorted_ids == NULL: slot_of_id is a dense index [n_ids] by id; else sorted_ids [n_ids] holds the
 * item_info ids ascending and slot_of_id[k] the row of sorted_ids[k] (sparse or hashed ids, where a
 * dense index would be sized by the largest id): a binary search per sample. */
int fbn_collate(const int64_t* perm, int B, const int64_t* item, const int64_t* seq, int Ls, int L,
                const int64_t* likes, const int64_t* views, const int64_t* user, const float* label,
                const int* slot_of_id, long long n_ids, const int64_t* sorted_ids, const float* emb, int E,
                int64_t* o_item, int64_t* o_seq,
                int64_t* o_likes, int64_t* o_views, int64_t* o_user, float* o_label, float* o_emb, int* missing,
                void* stream);
/* x[0:n] = 0 when *flag != 0: the inference collator's whole-batch zero fallback
 * (src/Prediction.py:39-42) on the batch's own missing flag, with no host round trip. */
int fbn_collate_zero_if(float* x, long long n, const int* flag, void* stream);

/* ---------------------------------------------------------------- step programs (native step driver)
 * Replaces the Python loop body that issues one training step (src/train_fibinet.py:113-123): the
 * host records a step's calls of this library -- entry point, arguments, and the cross-stream
 * edges (event record + stream wait) -- once while running the step, and replays them natively
 * (the same launches, streams and order: a replay is bit-identical to the eager step).  A recorded
 * call names its entry point; replay goes through a packed-argument thunk generated from this
 * header (csrc/plan_thunks.inc) that makes a well-typed call of the declared prototype.  Every
 * int-returning fbn_* entry point below (except the program and communicator set-up calls) with
 * <= 48 integer-class and <= 8 floating arguments can be recorded.
 *   fbn_plan_create(&plan); fbn_plan_add_call(plan, "fbn_...", iargs, ni, fargs, nf)  -- iargs: the
 *   integer-class arguments in order (pointers / ints as 64-bit, sign-extended); fargs: the float /
 *   double arguments in order as doubles (a float argument: a double whose low 32 bits are the
 *   float's); ni / nf must match the prototype (else FBN_ERR_ARG);
 *   fbn_plan_add_record(plan, slot, stream) / fbn_plan_add_wait(plan, stream, slot): a stream edge
 *   through the program's event `slot`; fbn_plan_run(plan, &failed_op): 0, or the failing entry
 *   point's code (message in fbn_last_error). */
int fbn_plan_create(void** plan);
int fbn_plan_destroy(void* plan);
int fbn_plan_size(void* plan);
int fbn_plan_add_call(void* plan, const char* name, const unsigned long long* iargs, int ni, const double* fargs,
                      int nf);
int fbn_plan_add_record(void* plan, int slot, void* stream);
int fbn_plan_add_wait(void* plan, void* stream, int slot);
int fbn_plan_run(void* plan, int* failed);
/* host: wait for event `slot` of the program's last replay (hipEventSynchronize) */
int fbn_plan_event_sync(void* plan, int slot);

/* ---------------------------------------------------------------- RCCL on the step's stream (N > 1)
 * The row exchange's all-to-alls and the dense all-reduce as RCCL calls on the stream the step's
 * kernels run on (csrc/comm.cpp) instead of torch.distributed's internal stream -- replaces the
 * process-group collectives the reference gets from nn.DataParallel (src/train_fibinet.py:69-70).
 *   fbn_comm_load(path): bind torch's own librccl.so (dlopen + dlsym; one RCCL runtime per process)
 *   fbn_comm_unique_id(out[fbn_comm_id_bytes()]) on rank 0, broadcast by the host, then
 *   fbn_comm_init(&comm, id, world, rank) on every rank (collective).
 *   fbn_comm_alltoallv: rows of row_bytes bytes, host int counts per peer (read at call time),
 *   blocks packed in rank order; fbn_comm_alltoall: equal split; fbn_comm_allreduce: in-place sum,
 *   dtype 0 f32 / 1 f64 / 2 i32.  Errors: 1 bad arguments / not loaded, 3 an RCCL error. */
int fbn_comm_load(const char* path);
int fbn_comm_id_bytes(void);
int fbn_comm_unique_id(void* out);
int fbn_comm_init(void** comm, const void* id, int world, int rank);
int fbn_comm_destroy(void* comm);
int fbn_comm_alltoallv(void* comm, const void* send, const int* send_counts, void* recv, const int* recv_counts,
                       long long row_bytes, void* stream);
int fbn_comm_alltoall(void* comm, const void* send, void* recv, long long bytes_per_peer, void* stream);
/* the equal-split all-to-all WITHOUT the caller's own block (grouped send / recv to the peers; a
 * no-op at one rank): the fixed-capacity exchange keeps a rank's requests to itself in place */
int fbn_comm_alltoall_peers(void* comm, const void* send, void* recv, long long bytes_per_peer, void* stream);
int fbn_comm_allreduce(void* comm, void* buf, long long n, int dtype, void* stream);
/* Watchdog (torch.distributed's collective timeout, which these communicators bypass).
 * fbn_comm_watch(timeout_ms): start the process's monitor thread (timeout_ms <= 0 disarms it).
 * fbn_comm_heartbeat(stream): the end of a step -- the host time now, and an event recorded on
 * `stream` (recordable: a step program's replays post it too).  Once the last heartbeat is older than
 * the timeout while its event has not completed, the monitor aborts every live communicator
 * (ncclCommAbort: RCCL's kernels exit, the stream and the host blocked on it drain) and every later
 * call on them fails with error 3 and the watchdog's message.  fbn_comm_abort(comm): abort one now.
 * fbn_comm_watchdog_fired(NULL): 1 once the watchdog fired; (comm): 1 if that communicator is aborted. */
/* Deterministic mode's all-reduce (replaces the sum of torch.distributed / ncclAllReduce, whose
 * reduction order follows the algorithm RCCL picks): fbn_comm_allgather (bytes_per_rank from every rank,
 * rank order) then fbn_sum_slices(in, ns, n, dtype 0 f32 / 1 f64, out) = the slices summed in rank order. */
int fbn_comm_allgather(void* comm, const void* send, void* recv, long long bytes_per_rank, void* stream);
int fbn_sum_slices(const void* in, int ns, long long n, int dtype, void* out, void* stream);
int fbn_comm_watch(long long timeout_ms);
int fbn_comm_heartbeat(void* stream);
int fbn_comm_abort(void* comm);
int fbn_comm_watchdog_fired(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* FIBINET_H */
