/*
 * vqgnn.h — C-ABI of the MI355X-native VQ-GNN per-layer hot path.
 *
 * The reference (devnkong/VQ-GNN, vq_gnn_v2) is pure Python: its hot path is
 * VectorQuantizerEMA (vq.py), the codebook gather in LowRankGNNLayer.forward
 * (models.py:157-177) and the sparse aggregation OurGCNConv / OurGATConv
 * (convs.py), whose arithmetic runs in third-party kernels (ATen, torch_sparse
 * spmm_sum, torch_scatter segment_csr).  Each entry point below replaces one
 * of those steps; the comment on each cites the reference line(s) it replaces.
 * The Python host layer (vq-gnn_amd/vq.py, convs.py, models.py) keeps the
 * reference's module API and calls these functions through ctypes; the
 * bindings a maintainer would add on the reference side are in INTEGRATION.md.
 *
 * Conventions
 *  - All pointers are DEVICE pointers (HBM) unless stated otherwise; every call
 *    is asynchronous on the given stream (a hipStream_t passed as void*; NULL =
 *    the legacy default stream).  Nothing here synchronises the device.
 *  - The library never allocates.  Functions that need scratch space take a
 *    workspace pointer whose size is returned by the matching *_workspace()
 *    function (host-only arithmetic, no device access).
 *  - Return value: 0 (VQGNN_OK) or a vqgnn_status code; the message of the
 *    last failure on the calling thread is returned by vqgnn_last_error().
 *  - Reentrant, no global mutable state: calls may come from any host thread
 *    (e.g. the autograd engine's device thread during backward).
 *  - Index types: CSR rowptr/col are int32 (nnz < 2^31); node ids int64 as in
 *    the reference (subset / batch_idx are LongTensors); codeword codes int16
 *    as the reference's c_indices buffer (models.py:27).
 */
#ifndef VQGNN_H
#define VQGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vqgnn_stream_t;

enum vqgnn_status {
  VQGNN_OK = 0,
  VQGNN_ERR_INVALID = 1,     /* bad argument (shape, null pointer, alignment) */
  VQGNN_ERR_LAUNCH = 2,      /* hipLaunch / hipMemsetAsync failure           */
  VQGNN_ERR_UNSUPPORTED = 3  /* shape outside what the kernels implement     */
};

/* Thread-local text of the last error on this thread ("" if none). */
const char* vqgnn_last_error(void);
/* ABI version (major*100 + minor). */
int vqgnn_version(void);

/* ------------------------------------------------------------------------ *
 * 1. BatchNorm1d sufficient statistics of the VQ inputs.
 *    Replaces the batch-stat half of BatchNorm1d(train) in
 *    vq.py:162 (feature_update) and vq.py:208-223 (update).
 *    Columns: F = nb*D feature columns of X, and (with_grad) F columns of G.
 *    sums[4][F] (fp64): sum x, sum x^2, sum g, sum g^2 over the B rows.
 *    These are the quantities a multi-GPU caller all-reduces.
 * ------------------------------------------------------------------------ */
size_t vqgnn_bn_stats_workspace(int32_t B, int32_t F);
int vqgnn_bn_stats(const float* X, int64_t ldx, const float* G, int64_t ldg,
                   int32_t B, int32_t F, int32_t with_grad,
                   double* sums, void* workspace, vqgnn_stream_t stream);
/* Multi-GPU form: sums is a flat [4F + 2] buffer; after the four sums it
 * holds sums[4F] = B (the row count every rank's all-reduce adds up, read by
 * vqgnn_bn_finalize with count = 0) and sums[4F + 1] = 0 (the over-capacity
 * flag a caller may set before the all-reduce) -- written on the device, so
 * the caller issues no fill of its own.  Without grads the g sums are 0. */
int vqgnn_bn_stats_count(const float* X, int64_t ldx, const float* G, int64_t ldg,
                         int32_t B, int32_t F, int32_t with_grad,
                         double* sums, void* workspace, vqgnn_stream_t stream);

/* 2. BatchNorm finalize: batch statistics -> per-column normalisation
 *    coefficients and the running-stat EMA update.
 *    Replaces BatchNorm1d.forward's stat update (vq.py:162, :223) and the
 *    first-call running-stat initialisation of update() (vq.py:216-221).
 *    mode: 0 = eval (coefficients from running stats, no update)
 *          1 = train (batch stats, running stats updated with momentum)
 *          2 = train + init_from_batch (vq.py:216-221, then as 1)
 *          3 = eval  + init_from_batch (vq.py:216-221, then as 0)
 *    arith_x / arith_g: the arithmetic of the feature / gradient columns,
 *    i.e. which of ATen's CPU BatchNorm paths the reference takes for that
 *    input (oracle/bn_ref.py restates both):
 *      VQGNN_BN_FP64    fp64 sums; deterministic and independent of the
 *                       number of ranks (the multi-GPU path, whose sums are
 *                       all-reduced)
 *      VQGNN_BN_STRIDED ATen on a non-contiguous [B, D] input: the reference
 *                       layers' x[:, D*i:D*(i+1)] slices (models.py:162-165)
 *      VQGNN_BN_CONTIG  ATen on a contiguous [B, D] input with ref_threads
 *                       CPU threads (its row chunks depend on them)
 *    vqgnn_bn_finalize takes fp64 sums, so its batch modes use FP64; arith
 *    only picks the form of the eval coefficients.
 *    count = rows over all ranks; count <= 0 reads it from sums[4F] (a
 *    double on the device: the multi-GPU path appends the local row count to
 *    the sums, so the one all-reduce also yields the global count without a
 *    host round trip).  momenta and eps are the reference's
 *    Python floats (double).
 *    coef[6][F]: alpha_f, beta_f, alpha_g, beta_g, shift_f, shift_g; every
 *    consumer normalises x as fma(x - shift, alpha, beta), which is ATen's
 *    expression on either path ((x - mean) * invstd, or
 *    fma(x, invstd, -mean * invstd)).
 *    batch_out[4][F] (optional, may be NULL): mean_f, std_f, mean_g, std_g with
 *    mean = torch.mean and std = sqrt(torch.var + eps_std) (vq.py:208-211
 *    logging stash).
 *    nbt_f / nbt_g (optional, [F / nbt_d] int64): BatchNorm1d's
 *    num_batches_tracked of each branch (nbt_d columns per branch) += 1 in
 *    the training modes.                                                      */
#define VQGNN_BN_FP64 0
#define VQGNN_BN_STRIDED 1
#define VQGNN_BN_CONTIG 2
int vqgnn_bn_finalize(const double* sums, int64_t count, int32_t F, int32_t with_grad,
                      int32_t mode, int32_t arith_x, int32_t arith_g,
                      double momentum_f, double eps_f, double momentum_g, double eps_g,
                      double eps_std, float* rm_f, float* rv_f, float* rm_g, float* rv_g,
                      float* coef, float* batch_out,
                      int64_t* nbt_f, int64_t* nbt_g, int32_t nbt_d,
                      vqgnn_stream_t stream);

/* 2b. Single-process statistics + finalize (count = B), any arithmetic.
 *     FP64: the vqgnn_bn_stats partials with the reduce and the finalize
 *     fused (same summation order and bits as the two calls); sums
 *     (optional) receives the fp64 sums.  STRIDED / CONTIG: the cascade-sum
 *     and row-chunk statistics of ATen's paths (sums must be NULL);
 *     ref_threads (1..1024) is the reference's torch.get_num_threads(), used
 *     by CONTIG columns only.  B <= 2^23.  Multi-GPU callers use FP64 and
 *     all-reduce the sums between vqgnn_bn_stats and vqgnn_bn_finalize. */
int vqgnn_bn_stats_finalize(const float* X, int64_t ldx, const float* G, int64_t ldg,
                            int32_t B, int32_t F, int32_t with_grad, double* sums, int32_t mode,
                            int32_t arith_x, int32_t arith_g, int32_t ref_threads,
                            double momentum_f, double eps_f, double momentum_g, double eps_g,
                            double eps_std, float* rm_f, float* rv_f, float* rm_g, float* rv_g,
                            float* coef, float* batch_out, int64_t* nbt_f, int64_t* nbt_g,
                            int32_t nbt_d, void* workspace, vqgnn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * 3. Product-quantised nearest-codeword assignment for nb branches at once,
 *    plus (ema_parts != NULL) the EMA sufficient statistics.
 *    Replaces, per branch b, vq.py:166-173 (feature_update, W = D) or
 *    vq.py:223-238 (update, W = 2D): normalise, d = (|x|^2 + |e|^2) - 2 x.e,
 *    argmin (first index on ties), and the one-hot reductions of
 *    vq.py:177-178/191 and :242-243/256 (counts, encodings^T @ x_norm).
 *    Branch b reads X[:, b*D:(b+1)*D] (and G[:, b*D:(b+1)*D] when W = 2D).
 *    embedding: [nb][M][ldw] (vq._embedding, ldw = 2D), branch stride
 *    emb_bstride floats.  coef: output of vqgnn_bn_finalize.
 *    Outputs (each optional):
 *      idx_out   [nb][B] int64   — encoding_indices per branch
 *      codes     [*][ldc] int16  — codes[batch_idx[i]][b] = idx (models.py:63/46)
 *      ema_parts [P][nb][M][W+1] int64 — P = vqgnn_vq_ema_parts(B, nb, M, W)
 *                (currently 1): (count, sum of normalised x) per codeword in
 *                fixed point; the workgroups' partials are added into it with
 *                int64 atomics (from the assign's LDS slab when the codebook
 *                and the slab share the LDS; else from a second kernel that
 *                holds one codeword range's slab in LDS per workgroup).
 *                ema_zeroed = 0: the call zeroes it first;
 *                1: the caller guarantees it is zero (e.g. left so by
 *                vqgnn_vq_ema_finalize with zero_after = 1).
 *    stat_count: rows the BatchNorm batch statistics were taken over (all
 *    ranks); it bounds |normalised x| <= sqrt(stat_count) and so fixes the
 *    fixed-point scale, vqgnn_vq_stat_shifts: column k < D of a slab is in
 *    units of 2^-shift_f, k >= D of 2^-shift_g, the count column of 1.  Each
 *    normalised value is rounded once (half an ulp of 2^-shift); the sums are
 *    exact, so the statistic does not depend on thread order, the number of
 *    parts or ranks (an int64 all-reduce of the slabs is exact).
 * ------------------------------------------------------------------------ */
void vqgnn_vq_stat_shifts(int64_t stat_count, float grad_scale, int32_t* shift_f,
                          int32_t* shift_g);
int32_t vqgnn_vq_ema_parts(int32_t B, int32_t nb, int32_t M, int32_t W);
size_t vqgnn_vq_assign_workspace(int32_t B, int32_t nb, int32_t M, int32_t W);
int vqgnn_vq_assign(const float* X, int64_t ldx, const float* G, int64_t ldg,
                    int32_t B, int32_t nb, int32_t D, int32_t M, int32_t W,
                    const float* coef, float grad_scale,
                    const float* embedding, int32_t ldw, int64_t emb_bstride,
                    int64_t* idx_out, int16_t* codes, int64_t ldc,
                    const int64_t* batch_idx, int64_t* ema_parts, int32_t ema_zeroed,
                    int64_t stat_count, void* workspace, vqgnn_stream_t stream);

/* 3a. The assign with the BatchNorm finalize folded into its prologue
 *     (single process, FP64 / STRIDED arithmetic): vqgnn_bn_stats_partial is
 *     vqgnn_bn_stats_finalize's statistics pass alone (its workspace:
 *     vqgnn_bn_stats_workspace(B, F)); vqgnn_vq_assign_bn takes that
 *     workspace and the finalize's parameters (as vqgnn_bn_stats_finalize;
 *     with_grad = (W == 2D), F = nb * D) in place of coef.  Every workgroup
 *     of branch b folds b's columns itself -- the finalize kernel's arithmetic,
 *     bit for bit -- and the first row part's workgroups update the running
 *     statistics and num_batches_tracked and write coef / batch_out, so the
 *     results equal vqgnn_bn_stats_finalize + vqgnn_vq_assign with one launch
 *     fewer (the host layer's default stays the two calls: every row part
 *     re-reads the partials).  The columns' arithmetic is that call's cascade form: at least
 *     one half STRIDED (all-FP64 statistics take the fp64-sum path there, and
 *     are rejected here); CONTIG has no fold.
 *     vqgnn_vq_assign_bn_supported says whether a shape has the fold
 *     (the filter path, W <= 8, B <= 2^23, and the fold's scratch within the
 *     codebook planes' LDS).                                                   */
int32_t vqgnn_vq_assign_bn_supported(int32_t B, int32_t nb, int32_t D, int32_t M, int32_t W);
int vqgnn_bn_stats_partial(const float* X, int64_t ldx, const float* G, int64_t ldg,
                           int32_t B, int32_t F, int32_t with_grad, void* workspace,
                           vqgnn_stream_t stream);
int vqgnn_vq_assign_bn(const float* X, int64_t ldx, const float* G, int64_t ldg,
                       int32_t B, int32_t nb, int32_t D, int32_t M, int32_t W,
                       float grad_scale, const float* embedding, int32_t ldw,
                       int64_t emb_bstride, int64_t* idx_out, int16_t* codes, int64_t ldc,
                       const int64_t* batch_idx, int64_t* ema_parts, int32_t ema_zeroed,
                       int64_t stat_count, void* workspace, const void* bn_workspace,
                       int32_t mode, int32_t arith_x, int32_t arith_g, double momentum_f,
                       double eps_f, double momentum_g, double eps_g, double eps_std,
                       float* rm_f, float* rv_f, float* rm_g, float* rv_g, float* coef,
                       float* batch_out, int64_t* nbt_f, int64_t* nbt_g, int32_t nbt_d,
                       vqgnn_stream_t stream);

/* 3b. Fold P partial slabs into one: out[i] = sum_p parts[p][i] (exact).
 *     Multi-GPU callers fold, then all-reduce (sum) the single int64 slab.    */
int vqgnn_vq_ema_reduce(const int64_t* parts, int32_t nparts, int64_t part_elems,
                        int64_t* out, vqgnn_stream_t stream);

/* 4. EMA codebook finalize for nb branches (vq.py:177-200 / :242-277):
 *    cluster size EMA, Laplace smoothing (laplace != 0, vq.py:182-186),
 *    'Bad Init!' detection (*bad_init |= 1, vq.py:188, and the branch is left
 *    with only cluster_size updated, as the reference raises there), ema_w EMA,
 *    embedding = ema_w / cs, and the de-normalised _embedding_output.  W = D
 *    updates the feature half only (feature_update); W = 2D all columns.
 *    ema_parts: nparts int64 slabs of [nb][M][W+1] (vqgnn_vq_assign), decoded
 *    with the shifts of the same stat_count / grad_scale; zero_after != 0
 *    clears every entry once read (ready for the next assign).
 *    Running stats (rm_f, rv_f, rm_g, rv_g) are [nb][D].  Per-branch arrays use
 *    strides cs_bstride (cluster_size) and emb_bstride (ema_w, embedding, out). */
int vqgnn_vq_ema_finalize(int64_t* ema_parts, int32_t nparts, int32_t zero_after,
                          int64_t stat_count,
                          int32_t nb, int32_t M,
                          int32_t D, int32_t W, int32_t ldw,
                          float decay, int32_t laplace, float grad_scale, float epsilon,
                          float* cluster_size, int64_t cs_bstride,
                          float* ema_w, float* embedding, float* embedding_output,
                          int64_t emb_bstride,
                          const float* rm_f, const float* rv_f,
                          const float* rm_g, const float* rv_g,
                          int32_t* bad_init, vqgnn_stream_t stream);

/* 4b. The operands of vqgnn_vq_ema_finalize as one record, for the
 *     aggregation entry that runs the finalize inside its own fix-up launch
 *     (vqgnn_spmm_task_cb_fin, §6b).  Same meaning, same checks.            */
typedef struct vqgnn_ema_finalize_args {
  int64_t* ema_parts;
  int32_t nparts, zero_after;
  int64_t stat_count;
  int32_t nb, M, D, W, ldw;
  float decay;
  int32_t laplace;
  float grad_scale, epsilon;
  float* cluster_size;
  int64_t cs_bstride;
  float* ema_w;
  float* embedding;
  float* embedding_output;
  int64_t emb_bstride;
  const float* rm_f;
  const float* rv_f;
  const float* rm_g;
  const float* rv_g;
  int32_t* bad_init;
} vqgnn_ema_finalize_args;

/* ------------------------------------------------------------------------ *
 * 5. Out-of-batch codeword gather (models.py:158, :168-173): for j in [0, n-B)
 *    and b < nb, with node = subset[B+j] and code = codes[node][b]:
 *      xt[j][b*D + k] = emb_out[b][code][col_offset + k],  k < D
 *      lcodes[j][b]   = code                               (optional)
 *    col_offset = 0 gives x_first_order (feature halves), col_offset = D the
 *    grad halves (grad_first_order).  codes [n_nodes][ldc] (c_indices);
 *    emb_out [n_branches][M][ldw], branch stride emb_bstride; xt [n-B][ldt].
 *    xt may be NULL (codes only).  nb (the code columns read) must not exceed
 *    n_branches (VQGNN_ERR_INVALID): the gather never reads past the codebook.
 *    A node outside [0, n_nodes) or a code outside [0, M) reads nothing: its
 *    D values are zeros (lcodes: -1 for a bad node).  (The reference raises
 *    IndexError there; c_indices written by vqgnn_vq_assign are always in
 *    range.)
 * ------------------------------------------------------------------------ */
int vqgnn_gather_codewords(const int64_t* subset, int32_t B, int32_t n,
                           const int16_t* codes, int64_t ldc, int64_t n_nodes,
                           int32_t nb, int32_t D, const float* emb_out,
                           int32_t n_branches, int32_t M, int32_t ldw, int64_t emb_bstride,
                           int32_t col_offset, float* xt, int64_t ldt,
                           int16_t* lcodes, vqgnn_stream_t stream);

/* 5b. Code scatter (models.py:63 / :46 across ranks): for i in [0, B),
 *     codes[batch_idx[i]][b] = local[i][b]  (batch_idx[i] < 0: skipped).
 *     Multi-GPU callers all-gather the (batch_idx, local codes) of every rank
 *     and scatter them with this so all replicas' c_indices stay identical.  */
int vqgnn_scatter_codes(const int64_t* batch_idx, int32_t B, const int16_t* local,
                        int32_t nb, int16_t* codes, int64_t ldc, vqgnn_stream_t stream);

/* 6. Task-split two-source CSR SpMM (sum), the aggregation of OurGCNConv
 *    (convs.py:95 -> torch_sparse.matmul(adj, x_input, reduce='add')):
 *      out[i][:] = sum_{e in row i} val[e] * xin[col[e]][:]
 *    with xin[j] = X[j] for j < B and X2[j - B] for j >= B, i.e.
 *    x_input = cat([x, x_first_order]) (models.py:174) without the copy.
 *    X2 == NULL: xin = X (plain SpMM; B ignored) -- also the transpose product
 *    of the backward pass.  n_cols = rows of xin (X rows, or B + X2 rows);
 *    every col[e] must be < n_cols < 2^26.  F a multiple of 4 (column tiles of
 *    128 floats; a partial last tile loads nothing past F); X/X2/out 16-byte
 *    aligned; out [n_rows][ldo].
 *    The nnz range is cut into tasks of K edges; 32 lanes walk one task (a
 *    wave: two tasks in lock-step, balanced whatever the row lengths),
 *    gathering each source row as 512-byte lines (dwordx4 per lane, 16 edges
 *    in flight per task) and accumulating with fma; rows that span tasks are
 *    finished by a fix-up in task order, empty rows written as zeros.  Each
 *    row is a sequential fma chain over its edges in CSR order: deterministic,
 *    independent of the launch geometry, within 1e-5 relative of the fp64 sum
 *    (north_star tolerance; not spmm_sum's separate multiply/add bit pattern).
 *    Plan (once per batch adjacency, any F): vqgnn_spmm_task_plan fills
 *    plan [vqgnn_spmm_task_size(nnz, K, n_rows)] int32 (each task's first
 *    edge and row -- a row of at most K/2 edges is never cut, so tasks hold
 *    K/2..3K/2 edges -- then the fix-up jobs: cut rows and empty rows),
 *    records [nnz] int64 (source column, row-end flag, weight) and
 *    counts[2] (device int32: cut rows, empty rows), which the caller reads
 *    once per plan and passes to every vqgnn_spmm_task call as n_jobs /
 *    n_empty.  K = 64 (multiple of 4 in [8, 4096]); nnz < 2^31.  A call may
 *    cover the first n_rows rows of the planned CSR (edges
 *    [0, rowptr[n_rows])), e.g. the backward's batch rows.  Workspace:
 *    vqgnn_spmm_task_workspace(nnz, K, F) bytes.
 *    vqgnn_spmm_task_records rewrites only the records for other values on
 *    the same structure (the plan's task starts and fix-up jobs depend on
 *    rowptr alone), e.g. GAT's coefficients on the transposed CSR in the
 *    backward, without a new plan or a host read.                            */
int64_t vqgnn_spmm_task_size(int64_t nnz, int32_t K, int32_t n_rows);
int vqgnn_spmm_task_plan(const int32_t* rowptr, const int32_t* col, const float* val,
                         int32_t n_rows, int64_t nnz, int32_t K, int32_t* plan,
                         int64_t* records, int32_t* counts, vqgnn_stream_t stream);
int vqgnn_spmm_task_records(const int32_t* rowptr, const int32_t* col, const float* val,
                            int32_t n_rows, int64_t nnz, int64_t* records,
                            vqgnn_stream_t stream);
size_t vqgnn_spmm_task_workspace(int64_t nnz, int32_t K, int32_t F);
int vqgnn_spmm_task(const int32_t* rowptr, int32_t n_rows, int32_t n_cols, int64_t nnz,
                    int32_t B, const float* X, int64_t ldx, const float* X2, int64_t ldx2,
                    int32_t F, float* out, int64_t ldo, const int32_t* plan,
                    const int64_t* records, int32_t K, int32_t n_jobs, int32_t n_empty,
                    void* workspace, vqgnn_stream_t stream);

/* 6b. Codebook-source SpMM: the layer's aggregation A @ [X ; x_first_order]
 *    (models.py:168-174 + convs.py:95) with the out-of-batch rows read from
 *    the codebook instead of a materialised x_first_order — row j >= B of
 *    x_in is, for every branch b and feature d < D, emb_out[b][codes[subset[j]][b]][d]
 *    (gather_codewords' values, include §4), served from an LDS image of the
 *    codebook's feature halves.  Same records, fma chain and fix-up as
 *    vqgnn_spmm_task over [X ; gather_codewords(...)]: the same output.
 *    vqgnn_spmm_task_records_cb: copy of a plan's records (vqgnn_spmm_task_plan)
 *      rewritten in place: a column j >= B becomes B + subset[j] (the node
 *      whose codes give the row); requires B + n_nodes <= 2^26.  A column
 *      past the subset or a node outside [0, n_nodes) gets weight 0 (its
 *      code reads as 0): it adds 0 x codeword 0 -- the zero row
 *      vqgnn_gather_codewords writes for it, for a finite codebook.
 *    vqgnn_spmm_task_cb: out = A @ x_in for the rewritten records; codes
 *      [n_nodes][ldc] int16 (c_indices; a code outside [0, M) reads the
 *      image's zero row, gather's zero row), codewords =
 *      emb_out [n_branches][M][ldw] (branch stride bstride, 16-byte aligned
 *      rows); the F / D code columns read must not exceed n_branches; D a
 *      multiple of 4; the image of a column tile of 4G columns is (M + 1) x
 *      16G bytes (the codewords and a zero row) <= 160 KiB with 4G dividing
 *      F (G = 32: M <= 319 at F % 128 == 0; G = 16: M <= 639 at F % 64 ==
 *      0; G = 8: M <= 1,279 at F % 32 == 0), vqgnn_spmm_task_cb_lds; X and
 *      out on the 32-bit near path.  Any
 *      other shape: VQGNN_ERR_INVALID (use vqgnn_gather_codewords +
 *      vqgnn_spmm_task, which has a 64-bit path).
 *    vqgnn_spmm_task_cb_supported: 1 iff vqgnn_spmm_task_cb accepts this
 *      shape (the same checks, no launch), so a host falls back before the
 *      call instead of catching its error.
 *    Speed: each column tile walks every edge once, so the narrow tiles (G <
 *      32) are slower than gather + vqgnn_spmm_task on arxiv-like batches;
 *      the package's host layer uses this entry only when
 *      vqgnn_spmm_task_cb_lds(M) == (M + 1) * 512 (the 128-column tile fits).
 *    vqgnn_spmm_task_cb_fin: vqgnn_spmm_task_cb, then the EMA finalize of
 *      *fin (§4, the update whose statistics the walk's codebook predates:
 *      models.py:181-185 runs it after the aggregation) inside the fix-up
 *      launch -- its first fin->nb workgroups finalize the branches beside
 *      the cut-row sums, one launch and one kernel boundary fewer than the
 *      two calls.  The finalize overwrites embedding_output, which the walk
 *      has read by then (same stream order as the two calls).  Same outputs
 *      and state, bit for bit, as vqgnn_spmm_task_cb followed by
 *      vqgnn_vq_ema_finalize; fin == NULL is vqgnn_spmm_task_cb.  For
 *      M >= 1,024 (the finalize's two-kernel form) the finalize runs as its
 *      own launches after the fix-up.  Single process: a multi-GPU update
 *      finalizes after its statistics' all-reduce instead.
 *    vqgnn_spmm_task_cb_walk + vqgnn_spmm_task_cb_fixup: vqgnn_spmm_task_cb_fin
 *      as two calls with the same arguments (the same workspace): the walk
 *      (every row that ends inside a task, and the cut rows' partials) and
 *      the fix-up (cut and empty rows, plus *fin's finalize when fin is not
 *      NULL).  The caller orders them: the fix-up after the walk (same
 *      stream, or an event).  Between them the walk may share the GPU with
 *      work that does not write what it reads (X, the out-of-batch nodes'
 *      codes, the codewords) -- the VQ update of the batch rows: its assign
 *      writes only the batch nodes' codes, its finalize runs in the fix-up.
 *      Same outputs, bit for bit, as the one-call entries.                 */
int vqgnn_spmm_task_records_cb(int64_t* records, int64_t nnz, int32_t B, const int64_t* subset,
                               int32_t n_cols, int64_t n_nodes, vqgnn_stream_t stream);
size_t vqgnn_spmm_task_cb_lds(int32_t M);
int32_t vqgnn_spmm_task_cb_supported(int32_t n_rows, int32_t B, int64_t ldx, int32_t F,
                                     int64_t ldo, int64_t n_nodes, int64_t ldc,
                                     int32_t n_branches, int32_t M, int32_t D);
int vqgnn_spmm_task_cb(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t B,
                       const float* X, int64_t ldx, int32_t F, const int16_t* codes, int64_t ldc,
                       int64_t n_nodes, const float* codewords, int64_t ldw, int64_t bstride,
                       int32_t n_branches, int32_t M, int32_t D, float* out, int64_t ldo,
                       const int32_t* plan, const int64_t* records_cb, int32_t K, int32_t n_jobs,
                       int32_t n_empty, void* workspace, vqgnn_stream_t stream);
int vqgnn_spmm_task_cb_fin(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t B,
                           const float* X, int64_t ldx, int32_t F, const int16_t* codes,
                           int64_t ldc, int64_t n_nodes, const float* codewords, int64_t ldw,
                           int64_t bstride, int32_t n_branches, int32_t M, int32_t D, float* out,
                           int64_t ldo, const int32_t* plan, const int64_t* records_cb, int32_t K,
                           int32_t n_jobs, int32_t n_empty, void* workspace,
                           const vqgnn_ema_finalize_args* fin, vqgnn_stream_t stream);
int vqgnn_spmm_task_cb_walk(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t B,
                            const float* X, int64_t ldx, int32_t F, const int16_t* codes,
                            int64_t ldc, int64_t n_nodes, const float* codewords, int64_t ldw,
                            int64_t bstride, int32_t n_branches, int32_t M, int32_t D, float* out,
                            int64_t ldo, const int32_t* plan, const int64_t* records_cb, int32_t K,
                            int32_t n_jobs, int32_t n_empty, void* workspace,
                            vqgnn_stream_t stream);
int vqgnn_spmm_task_cb_fixup(const int32_t* rowptr, int32_t n_rows, int64_t nnz, int32_t B,
                             const float* X, int64_t ldx, int32_t F, const int16_t* codes,
                             int64_t ldc, int64_t n_nodes, const float* codewords, int64_t ldw,
                             int64_t bstride, int32_t n_branches, int32_t M, int32_t D, float* out,
                             int64_t ldo, const int32_t* plan, const int64_t* records_cb, int32_t K,
                             int32_t n_jobs, int32_t n_empty, void* workspace,
                             const vqgnn_ema_finalize_args* fin, vqgnn_stream_t stream);

/* 7. CSR transpose (structure + values) for the backward product
 *    dX = A^T dOut (torch_sparse matmul autograd, convs.py:95).  Output CSR of
 *    A^T with rows sorted by column of A; within a row, entries ordered by
 *    row of A (canonical, deterministic).  t_val and t_perm are optional;
 *    t_perm[k] = index in the input CSR of transposed entry k (to carry other
 *    per-edge values, e.g. GAT coefficients, into transposed order).
 *    vqgnn_csr_expand_rows: rows[e] = row of edge e (COO row indices).       */
size_t vqgnn_csr_transpose_workspace(int32_t n_rows, int32_t n_cols, int64_t nnz);
int vqgnn_csr_transpose(const int32_t* rowptr, const int32_t* col, const float* val,
                        int32_t n_rows, int32_t n_cols, int64_t nnz,
                        int32_t* t_rowptr, int32_t* t_col, float* t_val,
                        int32_t* t_perm, void* workspace, vqgnn_stream_t stream);
int vqgnn_csr_expand_rows(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                          int32_t* rows, vqgnn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * 8. GAT attention aggregation (OurGATConv, convs.py:165-266, vq_softmax
 *    utils/vq_softmax.py:33-57, normalisation models.py:178-179/:187-189).
 *    x_in = [X (rows < B) ; X2 (rows >= B) ; ones column if ones != 0].
 *    gat_alpha: alpha_l/r[i] = x_in[i] . att_l/r (att length F + ones) and
 *      params[5] = {max_l, max_r, s, ds/dmax_l, ds/dmax_r} with
 *      s = sqrt(max_l^2+1) * sqrt(max_r^2+1)                  (convs.py:209-211)
 *      and, when alpha_l_s / alpha_r_s are given (both or neither), the
 *      per-node scaled scalars alpha_l_s[i] = alpha_l[i] / s, alpha_r_s[i] =
 *      alpha_r[i] / s, as the reference divides once per node
 *      (convs.py:209-211) and only adds per edge (:256).  Every per-edge
 *      consumer below takes these scaled arrays.
 *    gat_coef: coef[e] = exp(leaky(alpha_l_s[col] + alpha_r_s[row])) * val[e]
 *      (no max shift, no softmax normalisation), den[i] = sum_e coef[e] in
 *      CSR order (the ones column of the aggregation)         (convs.py:249-266)
 *    (gat_coef + vqgnn_spmm_task on records of coef + gat_normalize is the
 *    unfused form of vqgnn_gat_spmm_task, 8b, kept as its test reference.)
 *    gat_normalize: rows < B: out[i][:F] /= den[i] + eps       (models.py:188)
 *    gat_edge_grad: backward of the coefficient chain for every edge:
 *      a = alpha_l_s[col] + alpha_r_s[row] (s = params[2]);
 *      dcoef = dy[row] . x_in[col][:F] + dden[row];  da = dcoef*coef*leaky'(a);
 *      dalpha_l[col] += da/s; dalpha_r[row] += da/s; ds_row[row] += -da*a/s
 *      (atomic adds: the caller zeroes dalpha_l, dalpha_r, ds_row).
 * ------------------------------------------------------------------------ */
size_t vqgnn_gat_alpha_workspace(int32_t n);
int vqgnn_gat_alpha(const float* X, int64_t ldx, const float* X2, int64_t ldx2,
                    int32_t B, int32_t n, int32_t F, int32_t ones,
                    const float* att_l, const float* att_r, float* alpha_l, float* alpha_r,
                    float* alpha_l_s, float* alpha_r_s, float* params, void* workspace,
                    vqgnn_stream_t stream);
int vqgnn_gat_coef(const int32_t* rowptr, const int32_t* col, const float* val,
                   int32_t n_rows, int64_t nnz, const float* alpha_l_s, const float* alpha_r_s,
                   float negative_slope, float* coef, float* den, vqgnn_stream_t stream);
int vqgnn_gat_normalize(float* out, int64_t ldo, int32_t B, int32_t F, const float* den,
                        float eps, vqgnn_stream_t stream);
int vqgnn_gat_edge_grad(const int32_t* rows, const int32_t* col, const float* coef,
                        int64_t nnz, const float* X, int64_t ldx, const float* X2,
                        int64_t ldx2, int32_t B, int32_t F, const float* dy, int64_t lddy,
                        const float* dden, const float* alpha_l_s, const float* alpha_r_s,
                        const float* params, float negative_slope, float* dalpha_l,
                        float* dalpha_r, float* ds_row, vqgnn_stream_t stream);

/* 8b. Fused GAT aggregation (the default GAT forward): the task-split SpMM of
 *     6e with each edge's coefficient exp(leaky(alpha_l_s[j] + alpha_r_s[i]))
 *     * w computed in the kernel (the op order of vqgnn_gat_coef; the scaled
 *     scalars of vqgnn_gat_alpha), the ones column as a per-row
 *     coefficient sum, and rows < norm_B normalised by that sum + 1e-16
 *     before the store (models.py:188; norm_B = 0: no normalisation) -- as
 *     ONE v_rcp_f32 of (sum + 1e-16) times each column, not the reference's
 *     IEEE division: within 2^-20 relative (measured <= 5 ulp) of
 *     vqgnn_gat_normalize's true quotient
 *     (pinned in tests/test_gpu_gat.py), and the same bits for a row whether
 *     the plan cuts it across tasks (fix-up) or not (walker).  Replaces
 *     vqgnn_gat_coef + vqgnn_spmm_task + vqgnn_gat_normalize; the coefficients are
 *     never materialised unless coef (optional, [nnz], CSR order) is given for
 *     the backward; den (optional, [n_rows]) receives the sums.  erow: the
 *     COO row of every edge (vqgnn_csr_expand_rows); the default kernel
 *     derives each edge's row from the plan's row-end records and reads erow
 *     only for blocks after 31 or more consecutive empty rows (and the G = 8
 *     shape), but it must always be valid.  Plan and workspace as 6e
 *     (records hold the adjacency values w).                                 */
int vqgnn_gat_spmm_task(const int32_t* rowptr, int32_t n_rows, int32_t n_cols, int64_t nnz,
                        int32_t B, const float* X, int64_t ldx, const float* X2, int64_t ldx2,
                        int32_t F, float* out, int64_t ldo, const int32_t* plan,
                        const int64_t* records, int32_t K, int32_t n_jobs, int32_t n_empty,
                        const int32_t* erow, const float* alpha_l_s, const float* alpha_r_s,
                        float negative_slope, int32_t norm_B, float* den,
                        float* coef, void* workspace, vqgnn_stream_t stream);

/* 8b. GAT backward helper: vqgnn_gat_att_grad: d att_l / d att_r [F + ones]
 *       = x_in^T d alpha_l / d alpha_r with x_in = [X (rows < B) ; X2 ; ones
 *       column if ones] (the alpha = x_in . att of convs.py:189-190), F % 4 ==
 *       0, rows 16-byte aligned; fixed-order two-stage reduction; workspace
 *       vqgnn_gat_att_grad_workspace(n, F, ones) bytes.
 *     (vqgnn_gat_edge_grad runs 16 lanes per edge with coalesced row reads
 *     when F % 4 == 0, F <= 512 and the rows are 16-byte aligned.)            */
size_t vqgnn_gat_att_grad_workspace(int32_t n, int32_t F, int32_t ones);
int vqgnn_gat_att_grad(const float* X, int64_t ldx, const float* X2, int64_t ldx2, int32_t B,
                       int32_t n, int32_t F, int32_t ones, const float* dalpha_l,
                       const float* dalpha_r, float* datt_l, float* datt_r, void* workspace,
                       vqgnn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * 9. Mini-batch construction on the device.
 *    Replaces OurDataLoader._k_hop_subgraph (dataloader.py:98-148; num_hops,
 *    relabel_nodes=True, train_flag) and the SparseTensor build of
 *    prepare_batch_input (utils/misc.py:73).
 *    Full graph (data.adj_t, the normalised adjacency): rowptr int64 [N+1],
 *    col int32 [nnz_g < 2^31], val fp32.  node_idx int64 [B] (batch nodes).
 *
 *    vqgnn_khop_subset: node_map [N] (local id or -1), subset [capacity N]
 *      = [node_idx ; B' in ascending global id] (dataloader.py:121-126),
 *      out_rowptr [capacity N+1] of the rows emitted, and
 *      sizes [4] on the device = {n, nnz, rows emitted, status}; status =
 *      VQGNN_KHOP_OUT_OF_RANGE if a node id is outside [0, N).  A node
 *      repeated in node_idx behaves as in the reference: every copy stays in
 *      subset[:B], the last copy is its local id (node_idx[subset] = arange,
 *      :144), the rows of earlier copies are empty.
 *      order VQGNN_KHOP_ORDER_CSR: rows = subset order (every local row).
 *      order VQGNN_KHOP_ORDER_REF: rows = the reference's edge_index row order
 *      (ascending global id; eval: the batch nodes only), written to rows
 *      [capacity N].
 *      Kept entries: train -> both ends in subset (:132-133); eval -> rows
 *      of batch nodes (:136-138).
 *    vqgnn_khop_edges: after the caller read sizes (n, nnz, rows emitted):
 *      ORDER_CSR: out_col / out_val sorted by local column in every row -> the
 *      batch CSR the layer consumes (local row r = subset[r]);
 *      ORDER_REF: entries in edge_index[:, edge_mask] order (global row, then
 *      global column), out_row = local row (edge_index[0]).
 *      rows = subset (ORDER_CSR) or the rows array of vqgnn_khop_subset.
 *    vqgnn_coo_to_csr: SparseTensor(row=, col=, value=, sparse_sizes) ->
 *      CSR sorted by (row, col), stable for repeated (row, col) pairs; status
 *      (device int64) = VQGNN_KHOP_OUT_OF_RANGE if an index is outside.
 * ------------------------------------------------------------------------ */
enum vqgnn_khop_order { VQGNN_KHOP_ORDER_CSR = 0, VQGNN_KHOP_ORDER_REF = 1 };
enum vqgnn_khop_status { VQGNN_KHOP_OUT_OF_RANGE = 2 };
size_t vqgnn_khop_workspace(int64_t N);
int vqgnn_khop_subset(const int64_t* rowptr, const int32_t* col, int64_t N,
                      const int64_t* node_idx, int32_t B, int32_t num_hops, int32_t train_flag,
                      int32_t order, int32_t* node_map, int64_t* subset, int64_t* rows,
                      int32_t* out_rowptr, int64_t* sizes, void* workspace,
                      vqgnn_stream_t stream);
size_t vqgnn_khop_edges_workspace(int64_t nrows, int64_t nnz);
int vqgnn_khop_edges(const int64_t* rowptr, const int32_t* col, const float* val, int64_t N,
                     const int32_t* node_map, const int64_t* rows, int64_t nrows, int64_t n,
                     int32_t B, int32_t train_flag, int32_t order, const int32_t* out_rowptr,
                     int64_t nnz, int32_t* out_col, float* out_val, int32_t* out_row,
                     void* workspace, vqgnn_stream_t stream);
size_t vqgnn_coo_to_csr_workspace(int64_t nnz, int64_t n_rows, int64_t n_cols);
int vqgnn_coo_to_csr(const int64_t* row, const int64_t* col, const float* val, int64_t nnz,
                     int64_t n_rows, int64_t n_cols, int32_t* out_rowptr, int32_t* out_col,
                     float* out_val, int64_t* status, void* workspace, vqgnn_stream_t stream);

/* 9b. Uniform random walks for the 'edge', 'rw' and 'cont' samplers
 *     (dataloader.py:70-90: SparseTensor.random_walk -> torch_cluster
 *     random_walk with p = q = 1; torch_cluster is not vendored in the
 *     reference).  out [n_start][walk_length + 1] int64: out[i][0] =
 *     start[i]; step l moves from v to col[rowptr[v] + (int64)(u * (float)
 *     deg(v))] with u in [0, 1), or stays on v when deg(v) = 0 — torch_cluster's
 *     uniform step.  u = (splitmix64(splitmix64(seed ^ splitmix64(i)) + l)
 *     >> 40) * 2^-24: deterministic per seed, not torch's CPU RNG stream
 *     (oracle/subgraph_ref.walk_uniforms restates it).  status (device
 *     int64) = VQGNN_KHOP_OUT_OF_RANGE if a start node is outside [0, N). */
int vqgnn_random_walk(const int64_t* rowptr, const int32_t* col, int64_t N, const int64_t* start,
                      int64_t n_start, int32_t walk_length, uint64_t seed, int64_t* out,
                      int64_t* status, vqgnn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * 10. Full-graph preprocessing.  Graph CSR as in §9:
 *     rowptr int64 [N+1], col int32 (sorted within rows), val fp32 or NULL
 *     (no values: every entry 1).
 *   vqgnn_norm_adj: norm_adj (utils/misc.py:14-34).  GCN / GAT: set_diag()
 *     (the diagonal replaced by, or inserted as, 1), deg = sequential row
 *     sum, GCN: v = (deg^-1/2[row] * v) * deg^-1/2[col] (ATen pow(-0.5) =
 *     1/sqrt), SAGE / GAT: v = deg^-1[row] * v; inf -> 0.  Output capacity
 *     nnz + N (GCN, GAT) or nnz (SAGE); out_rowptr[N] = the output nnz.
 *   vqgnn_to_symmetric: SparseTensor.to_symmetric() (misc.py:190, :211): A
 *     and A^T merged, repeated (row, col) summed (val NULL: pattern, 1).
 *     Capacity 2*nnz; out_nnz (device int64) = the output nnz.
 *   vqgnn_csr_permute: SparseTensor.permute(perm) (misc.py:113-130): new node
 *     i = old node perm[i]; rows sorted by the new columns.  status (device
 *     int64) = 1 if perm holds an index outside [0, N).
 *   vqgnn_partition: the METIS substitute for metis() (misc.py:93-111; METIS
 *     is absent): connected components by min-label propagation, a BFS from
 *     each component's smallest node, nodes ordered by (component, level,
 *     id) -> perm [N]; ptr [num_parts+1] = equal contiguous bands.  Host-
 *     synchronous (one readback per propagation / BFS step); iterations
 *     (host, may be NULL) = the number of steps.
 * ------------------------------------------------------------------------ */
enum vqgnn_conv_type { VQGNN_CONV_GCN = 0, VQGNN_CONV_SAGE = 1, VQGNN_CONV_GAT = 2 };
size_t vqgnn_norm_adj_workspace(int64_t N);
int vqgnn_norm_adj(const int64_t* rowptr, const int32_t* col, const float* val, int64_t N,
                   int32_t conv_type, int64_t* out_rowptr, int32_t* out_col, float* out_val,
                   void* workspace, vqgnn_stream_t stream);
size_t vqgnn_to_symmetric_workspace(int64_t N, int64_t nnz);
int vqgnn_to_symmetric(const int64_t* rowptr, const int32_t* col, const float* val, int64_t N,
                       int64_t nnz, int64_t* out_rowptr, int32_t* out_col, float* out_val,
                       int64_t* out_nnz, void* workspace, vqgnn_stream_t stream);
size_t vqgnn_csr_permute_workspace(int64_t N, int64_t nnz);
int vqgnn_csr_permute(const int64_t* rowptr, const int32_t* col, const float* val, int64_t N,
                      int64_t nnz, const int64_t* perm, int64_t* out_rowptr, int32_t* out_col,
                      float* out_val, int64_t* status, void* workspace, vqgnn_stream_t stream);
size_t vqgnn_partition_workspace(int64_t N);
int vqgnn_partition(const int64_t* rowptr, const int32_t* col, int64_t N, int32_t num_parts,
                    int64_t* perm, int64_t* ptr, int32_t* iterations, void* workspace,
                    vqgnn_stream_t stream);

/* 5a. Measurement (bench.py): vqgnn_assign_timing(1) starts recording every
 *     vq_assign_kernel launch with a start/stop event pair taken by
 *     hipExtLaunchKernel (the kernel's own duration); _read syncs on them and
 *     writes up to cap durations in ms, returns the count; (0) stops and
 *     frees the events.                                                       */
int vqgnn_assign_timing(int32_t enable);
int32_t vqgnn_assign_timing_read(float* ms, int32_t cap);

/* 5b. Multi-GPU code exchange wire format (keeps every replica's c_indices
 *     identical; models.py:46/:63 across ranks).  A record per batch row:
 *     int32 node id (-1 = padding), then nb codes as uint8 (M <= 256) or
 *     int16, padded to 4 bytes (vqgnn_codes_wire_record).
 *     vqgnn_pack_codes: rows [0, B) of (batch_idx, local [B][nb]) and
 *     padding up to max_B into send; with codes != NULL also scatters them
 *     into this rank's own c_indices at once.
 *     vqgnn_scatter_wire: all ranks' records (rank-major, as
 *     all_gather_into_tensor lays them out) into codes; a node held by
 *     several records takes the LAST record's codes (deterministic: a
 *     per-node atomicMax of (epoch << 32 | record index), then only the
 *     winner writes).  winner: int64 [N], zero-initialised once and never
 *     reset; epoch: 1, 2, 3, ... per call on the same table (< 2^31), so
 *     earlier stamps always lose.  n_records < 2^32.                          */
int32_t vqgnn_codes_wire_record(int32_t nb, int32_t M);
int vqgnn_pack_codes(const int64_t* batch_idx, int32_t B, const int16_t* local, int32_t nb,
                     int32_t M, int32_t max_B, uint8_t* send, int16_t* codes, int64_t ldc,
                     vqgnn_stream_t stream);
int vqgnn_scatter_wire(const uint8_t* recv, int64_t n_records, int32_t nb, int32_t M,
                       int64_t* winner, int64_t epoch, int64_t N, int16_t* codes, int64_t ldc,
                       vqgnn_stream_t stream);

/* ------------------------------------------------------------------------ *
 * 11. VQ-GNN v1 compressed adjacency: mapper(batch, c,
 *     num_M, gnn_type) of vq_gnn_v1/utils/dataloader.py:144-192, called per
 *     branch at vq_gnn_v1/models.py:170.  Inputs (device): A_BN COO (bn_row =
 *     local batch row, bn_col = global node, bn_val) of E entries; nb_val
 *     (A_NB_v, may be NULL); A_BB COO in local ids (bb_* NULL: no A_BB) of E2
 *     entries with batch_idx [B]; codes: int16 codeword of node j at
 *     codes[j*ldc] (one branch of the node-major c_indices); deg_inv [B]
 *     (self-loop values; unused for SAGE).  Output: CSR of dim = B + M,
 *     out_rowptr int64 [dim+1], out_col int32 / out_val fp32 of capacity
 *     vqgnn_mapper_capacity(...), out_nnz (device int64).  Coalescing sums
 *     repeated (row, col) sequentially in concatenation order (stable radix
 *     sort + one thread per key = torch_sparse coalesce's segment_csr);
 *     status (device int64) = 1 if a code is outside [0, M).
 * ------------------------------------------------------------------------ */
int64_t vqgnn_mapper_capacity(int64_t E, int64_t E2, int32_t B, int32_t has_nb, int32_t has_bb,
                              int32_t conv_type);
size_t vqgnn_mapper_workspace(int64_t E, int64_t E2, int32_t B, int32_t has_nb, int32_t has_bb);
int vqgnn_mapper(const int32_t* bn_row, const int32_t* bn_col, const float* bn_val, int64_t E,
                 const float* nb_val, const int32_t* bb_row, const int32_t* bb_col,
                 const float* bb_val, int64_t E2, const int64_t* batch_idx, int32_t B,
                 const int16_t* codes, int64_t ldc, int32_t M, const float* deg_inv,
                 int32_t conv_type, int64_t* out_rowptr, int32_t* out_col, float* out_val,
                 int64_t* out_nnz, int64_t* status, void* workspace, vqgnn_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* VQGNN_H */
