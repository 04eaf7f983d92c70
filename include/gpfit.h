/*
 * gpfit.h — C-ABI of the MI355X GP-fit hot path (libgpfit.so).
 *
 * The reference (rferguson22/Gaussian-Process) is pure Python: its "plugin
 * surface" for this path is a set of Python functions, not an FFI. Each entry
 * point below replaces one of those seams; the Python drop-in modules in
 * gaussian-process_amd/ bind them through ctypes.
 *
 *   gpf_eval_batch  replaces the particle fan-out
 *                     list(executor.map(evaluate_loss_helper, args))
 *                   at find_len_scales.py:77, :103, :134 — i.e. P calls of
 *                   evaluate_loss (:181) -> wass_loss (:154-177) -> GP(x,y,e,x,l,
 *                   batch_size=N) (GP_func.py:12-45, called at :159).
 *   gpf_predict     replaces GP(x_known,y_known,e_known,x_fit,lengths,batch_size)
 *                   (GP_func.py:12-45) for arbitrary query points (GP_fit.py:32).
 *   gpf_kernel      replaces kernel_func(x1,x2,l) (GP_func.py:49-65).
 *
 * Conventions (mirroring the reference):
 *   - all floating point is IEEE fp64;
 *   - x arrays are dims-major (d, N), C-contiguous (the Python side calls
 *     np.ascontiguousarray on the reference's F-order view, read_in.py:229);
 *   - host buffers are caller-owned; data set by gpf_set_data stays resident
 *     on the device until the next gpf_set_data / gpf_close;
 *   - a context drives ONE device and is not thread-safe (one host thread per
 *     context); one process per GPU, the swarm exchange between them is in this
 *     library (gpf_comm_*: RCCL over xGMI, or a host transport).
 *
 * Return codes: GPF_OK, GPF_NOT_PD (Cholesky pivot <= 0 or NaN: the Python side
 * raises numpy.linalg.LinAlgError("Matrix is not positive definite") exactly
 * like numpy.linalg.cholesky at GP_func.py:22), GPF_HIP_ERROR, GPF_BAD_ARG.
 */
#ifndef GPFIT_H
#define GPFIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPF_OK 0
#define GPF_NOT_PD 1
#define GPF_HIP_ERROR 2
#define GPF_BAD_ARG 3

#define GPF_ABI_VERSION 2  /* 2 (r6): gpf_plan_check's stats carry 11 entries */

typedef struct gpf_ctx gpf_ctx;

/* ABI version of the loaded library (== GPF_ABI_VERSION). */
int gpf_version(void);

/* Open a context on HIP device `device` (after HIP_VISIBLE_DEVICES). */
int gpf_open(int device, gpf_ctx** out);
void gpf_close(gpf_ctx* ctx);

/* Message for the last non-OK return on this context ("" if none). */
const char* gpf_last_error(gpf_ctx* ctx);

/* Training data: x_dN is (d, N) dims-major; y, e are (N,).
 * Reference: the (x_known, y_known, e_known) tuple members pickled per task at
 * find_len_scales.py:76,102,133; here uploaded once per len_scale_opt call. */
int gpf_set_data(gpf_ctx* ctx, const double* x_dN, const double* y,
                 const double* e, int64_t N, int d);

/* Objective grid and search box: sigma_vals/expected are the K-point grid of
 * find_len_scales.py:66-67 (K = 1000 in the reference), lo/hi the (d,) bounds of
 * :56-61. */
int gpf_set_grid(gpf_ctx* ctx, const double* sigma_vals, const double* expected,
                 int K, const double* lo, const double* hi);

/* Batched objective. ls_Pd is (P, d) row-major particle positions. Writes
 * loss_P[p] = evaluate_loss(ls[p], ...) (find_len_scales.py:181); sentinel
 * particles (any ls <= lo or ls >= hi, :156-157) get 1e13 without touching the
 * GPU. mu_PN / sd_PN (nullable, (P, N) row-major) receive the GP mean / sd at
 * the training points (GP_func.py:36-40 with x_fit = x_known); rows of
 * sentinel particles are filled with NaN. On GPF_NOT_PD *bad_idx is the first
 * particle whose covariance is not positive definite. */
int gpf_eval_batch(gpf_ctx* ctx, const double* ls_Pd, int P, double* loss_P,
                   double* mu_PN, double* sd_PN, int* bad_idx);

/* GP prediction at M query points xfit_dM (d, M), chunked by `batch` like
 * GP_func.py:28-30 (the chunking does not change the result here). */
int gpf_predict(gpf_ctx* ctx, const double* ls, const double* xfit_dM,
                int64_t M, int64_t batch, double* mu_M, double* sd_M);

/* kernel_func(x1, x2, l) (GP_func.py:49-65): out is (N1, N2) row-major. */
int gpf_kernel(gpf_ctx* ctx, const double* x1_dN1, int64_t N1,
               const double* x2_dN2, int64_t N2, int d, const double* l,
               double* out);

/* Diagnostic log marginal likelihood from the same factor (the reference has
 * none): -1/2 y^T alpha - sum log L_ii - N/2 log(2 pi). */
int gpf_log_marginal_likelihood(gpf_ctx* ctx, const double* ls, double* out);

/* Probability surface of merged GP results (replaces calc_prob_surf.py:15-30,67-81; SURVEY.md
 * §8f row 4). tails: M rows x E entries (row-major) = each merged-frame row after its kinematic
 * columns, non-finite = missing. Per row: y[100] (the numpy.linspace grid), p[100] (bin
 * probabilities of the equal-weight Gaussian mixture), ok = 0 if the row is skipped (fewer than
 * 2 or an odd number of finite entries, calc_prob_surf.py:71-73), else 1. E <= 1024. */
int gpf_prob_surface(gpf_ctx* ctx, const double* tails, int64_t M, int E, double* y, double* p, int* ok);

/* Convex-hull grid fill (replaces the fill passes of convex_hull.py:122-155,203-224; SURVEY.md
 * §8f row 3). shell: n x d rows (row-major) = the rasterised hull facets (the reference's
 * concatenated facet surfaces, convex_hull.py:215-217); res: the d resolutions; decimals: the
 * digits after the point of str(res[j]) (numpy.around in round_to_res, convex_hull.py:13-24).
 * Runs the d sort + scan-fill passes and keeps the grid; *m = its row count. gpf_hull_fetch
 * copies it (m x d, rows sorted lexicographically, as fill_convex_hull returns them). */
int gpf_hull_fill(gpf_ctx* ctx, const double* shell, int64_t n, int d, const double* res, const int* decimals,
                  int64_t* m);
int gpf_hull_fetch(gpf_ctx* ctx, double* out);

/* KMeans subsample (the Lloyd iterations of find_len_scales.py:27-31, sklearn KMeans(n_clusters,
 * n_init='auto', random_state=0)). gpf_kmeans_set keeps n points x d
 * (row-major, already centred by their mean as sklearn's fit does) on the device. One
 * gpf_kmeans_step = the E-step (and with update != 0 the M-step sums) of sklearn's
 * lloyd_iter_chunked_dense with unit weights against k centres (k x d, row-major; k*(d+1) <= 8192,
 * else GPF_BAD_ARG and gpfit.kmeans keeps sklearn's host fit):
 * labels[i] = the first j minimising ||c_j||^2 - 2 x_i.c_j; sums (k x d) and counts (k) of each
 * cluster's members; dist[i] = ||x_i - c_labels[i]||^2 (optional, may be NULL). The host runs
 * sklearn's loop around it (gaussian-process_amd/gpfit/kmeans.py). */
int gpf_kmeans_set(gpf_ctx* ctx, const double* X, int64_t n, int d);
int gpf_kmeans_step(gpf_ctx* ctx, const double* centers, int k, int update, int* labels, double* sums, double* counts,
                    double* dist);

/* ---- swarm exchange across ranks (one process per GPU) ----
 *
 * Replaces the cross-process half of the particle fan-out: the reference's single process
 * scatters the swarm over a fork pool and gathers the scores (find_len_scales.py:73-77,
 * 102-104,133-135); here every rank scores its contiguous rows [rP/G, (r+1)P/G) and one
 * all-reduce (sum) of a zero-initialised [P + G] float64 vector hands every rank the full
 * score vector (exact: one non-zero contributor per entry), so all ranks take the same
 * first-index argmin (:81,110). The G trailing entries carry each rank's status, so a non-PD
 * particle or a device error on one rank is reported on every rank (same bad_idx, same code)
 * instead of leaving the others blocked in the collective.
 *
 * Transports: GPF_COMM_RCCL = ncclAllReduce on the context's device (RCCL over xGMI; rank 0
 * hands out the ncclUniqueId over TCP); GPF_COMM_HOST = the same exchange over the TCP
 * rendezvous sockets (rank 0 combines in rank order; needs no device). Rendezvous: rank 0
 * listens on host:port, the others connect (retrying until GPF_COMM_TIMEOUT_S, default 600 s).
 * A communicator is not thread-safe. */
#define GPF_COMM_RCCL 1
#define GPF_COMM_HOST 2
#define GPF_OP_SUM 0
#define GPF_OP_MAX 1

typedef struct gpf_comm gpf_comm;

/* Join rank `rank` of `nranks`. ctx: the rank's context (required for GPF_COMM_RCCL: the
 * communicator lives on its device; may be NULL for GPF_COMM_HOST). */
int gpf_comm_open(gpf_ctx* ctx, int rank, int nranks, const char* host, int port, int transport, gpf_comm** out);
void gpf_comm_close(gpf_comm* comm);
int gpf_comm_rank(const gpf_comm* comm);
int gpf_comm_size(const gpf_comm* comm);
const char* gpf_comm_last_error(const gpf_comm* comm);
/* Cumulative wall time spent inside gpf_comm_exchange_scores on this rank (the all-reduce,
 * including the wait for the slowest rank) and the number of exchanges. */
int gpf_comm_stats(const gpf_comm* comm, double* exchange_ms, long long* exchanges);

/* In-place all-reduce of n host doubles (GPF_OP_SUM or GPF_OP_MAX) across the ranks: the
 * seed broadcast of the PSO driver, the bench's barrier and max-over-ranks timing. */
int gpf_comm_allreduce(gpf_comm* comm, double* buf, int64_t n, int op);

/* The exchange step alone, given this rank's results for its rows [rP/G, (r+1)P/G):
 * local (hi - lo scores; ignored unless local_rc == GPF_OK), local_rc (GPF_OK / GPF_NOT_PD /
 * other), local_bad (the row, relative to lo, of the first non-PD particle). Fills loss_P on
 * every rank, or returns on every rank GPF_NOT_PD with *bad_idx = the smallest failing row of
 * the whole swarm (the particle the reference's in-order map would raise on first), or the
 * error code of the first failed rank. */
int gpf_comm_exchange_scores(gpf_comm* comm, int P, const double* local, int local_rc, int local_bad,
                             double* loss_P, int* bad_idx);

/* Sharded gpf_eval_batch: this rank scores its rows of ls_Pd (P, d) on its context, then
 * gpf_comm_exchange_scores. Every rank passes the same ls_Pd and receives the same loss_P. */
int gpf_eval_batch_sharded(gpf_ctx* ctx, gpf_comm* comm, const double* ls_Pd, int P, double* loss_P,
                           int* bad_idx);

/* Wait until all work queued by this library on the context's device has finished
 * (hipDeviceSynchronize on that device): the bench's timing fence. */
int gpf_sync(gpf_ctx* ctx);

/* ---- measurement hooks (bench.py) ---- */

/* Enable per-kernel-class HIP event timing on the context's stream. */
int gpf_set_profiling(gpf_ctx* ctx, int on);

/* Fill out[0..n) with accumulated counters since the last reset:
 *  [0] panel kernel ms   [1] panel launches  [2] panel algorithmic flops
 *  [3] diag kernel ms    [4] diag launches   [5] diag algorithmic flops
 *  [6] K-build ms        [7] K-build launches[8] K-build algorithmic bytes
 *  [9] loss kernel ms    [10] loss launches  [11] evals (non-sentinel)
 *  [12] factorisation wall ms (K build + diag + steps of all particle groups, which run
 *       on concurrent streams, so [0]/[3]/[6] may overlap)  [13] calls  [14] its flops
 *  [15] prediction V = U K_s kernel ms  [16] launches  [17] algorithmic flops
 *  [18] prediction cross-covariance ms  [19] launches  [20] algorithmic bytes
 *  [21] probability-surface kernel ms  [22] launches  [23] algorithmic bytes
 *  [24] shader clock (MHz) the factor kernels held while they ran (every workgroup's span in
 *       s_memtime clocks over its span in the 100 MHz s_memrealtime clock; profiled batches only)
 *  [25] compute units  [26] FP64 matrix ceiling at that clock, TFLOP/s (128 flop / CU / clock)
 * Returns the number of values written. */
int gpf_get_profile(gpf_ctx* ctx, double* out, int n);
int gpf_reset_profile(gpf_ctx* ctx);

/* Tile edge used by the factorisation (padding granule). */
int gpf_tile(void);

/* Build provenance baked in at compile time by __graft_entry__.build(): "src=<sha256 of the
 * csrc .hip and include .h sources> hipcc=<compiler version line>" ("unknown" if compiled by
 * hand). Tests compare it with the hash of the sources in the tree. */
const char* gpf_build_info(void);

/* Host-only structural check of the k_step dispatch plan (needs no device and no context):
 * for a chunk of pc particles with nt block columns, under the current GPF_GROUPS /
 * GPF_SPLIT_K / GPF_STEP_GROUP environment, builds the
 * launch list run_factor issues and decodes every workgroup of every launch with the kernel's
 * own decoder (gpf::step_decode). Checks that every (block column, particle, tile) is computed
 * exactly once (one whole-tile workgroup, or all S depth pieces exactly once, whose S arrivals
 * on a zeroed counter elect exactly one finisher), that pieces stay inside the split-K buffers,
 * and that concurrent particle groups never share partial slots or counters.
 * With the early diagonal factor it also checks that every launch starts with exactly one
 * diagonal workgroup per particle, ahead of all tiles; with the deferred diagonal update
 * (GPF_DEFER_SYRK, default on) that launches 1 .. nt-2 without the all-tile split carry exactly
 * one SYRK workgroup per particle right behind the diagonal workgroups, and no other launch any.
 * Under the persistent factorisation (GPF_PERSIST; default for chunks with more tiles per block
 * column than 512 workgroup slots) it instead decodes every ticket of every work queue with the
 * kernel's own decoder (gpf::p_decode): every (block column, particle, tile) exactly once, one
 * SYRK item per particle and block column 1 .. nt-2, and every item's inputs produced by items
 * earlier in its queue (what makes the persistent launch deadlock-free).
 * Paired block columns (GPF_PAIR; gpf::pair_decode): a lead launch J carries, per particle, every
 * tile of column J once, its SYRK workgroup, one look-ahead partial per tile of column J+1 that
 * exists (the tile's 8 or 16 ids behind, on the same XCD), and the partial SYRK of block J+2; it is
 * followed on its stream by the follow launch J+1, whose tiles read those partials (slots inside
 * the group's buffer).
 * stats (nullable, 11 entries): launches, workgroups (persistent: items), whole tiles, split
 * tiles, S (all-tile split factor), largest split factor, particle groups, diagonal
 * workgroups, SYRK workgroups (items), persistent (0/1), lead launches of paired block columns. Returns GPF_OK, or
 * GPF_BAD_ARG with a description of the first violation in msg. */
int gpf_plan_check(int pc, int nt, long long* stats, char* msg, int msg_len);

/* Self-test of the f64 MFMA fragment layout: C = A(16x4) B(4x16) on device,
 * compared on the host by the caller. a: 16x4 row-major, b: 4x16 row-major,
 * c: 16x16 row-major. */
int gpf_selftest_mfma(gpf_ctx* ctx, const double* a, const double* b, double* c);

/* Diagnostic: factorise one particle and copy back its Npad x Npad L and
 * U = L^-1 (row-major; the strict upper triangles hold scratch), the
 * forward-substituted RHS z (Npad) and alpha (N). Npad = ceil(N/128)*128. */
int gpf_debug_factor(gpf_ctx* ctx, const double* ls, double* L, double* U, double* z, double* alpha);

/* Diagnostic / measurement: the 128x128 diagonal-block factor of the factorisation (factor128 in
 * csrc/gpf_diag.hip) on n blocks, one workgroup each. A: n x 128 x 128 row-major (lower triangles
 * read), y: n x 128. Out: L (zeros above the diagonal), U = L^-1 (likewise), z = U y, s2 / sz =
 * the column partials colsum(U o U) and U^T z, bad[b] = 1 where a pivot was not > 0, cycles
 * (nullable): each workgroup's shader cycles. */
int gpf_debug_factor128(gpf_ctx* ctx, const double* A, const double* y, int n, double* L, double* U, double* z,
                        double* s2, double* sz, int* bad, double* cycles);

/* Diagnostic: measured FP64 MFMA throughput (TFLOP/s) of a register-only
 * v_mfma_f64_16x16x4_f64 loop over `blocks` workgroups of 4 waves. */
int gpf_mfma_peak(gpf_ctx* ctx, int blocks, int iters, double* tflops);

/* The shader clock (MHz) the timed launches of the last gpf_mfma_peak or gpf_gemm_bench call
 * held (every workgroup's span in s_memtime clocks over its span in the 100 MHz s_memrealtime
 * clock; 0 before any such call). */
int gpf_bench_clock(gpf_ctx* ctx, double* mhz);

/* Measurement hook: TF/s of the block-column GEMM core alone (no factorisation):
 * P particles' Npad x Npad matrices, `tiles` workgroups per particle, depth D, `iters`
 * timed launches; mode 0 = per-particle operands, mode 1 = one shared (L2-resident) pair; mode
 * bit 2 (4): U-tile-shaped operands; bit 3 (8): zero operands instead of hashed values in [-1, 1);
 * bit 4 (16) / bit 5 (32): the 3- / 4-stage LDS pipeline (one workgroup per CU). */
int gpf_gemm_bench(gpf_ctx* ctx, int mode, int Npad, int P, int tiles, int D, int iters, double* tflops);

#ifdef __cplusplus
}
#endif

#endif /* GPFIT_H */
