/*
 * glx.h — C ABI of libglx.so, the MI355X-native group-lasso first-order solver.
 *
 * Problem:  min_x  1/2 ||A x - b||_F^2 + mu * sum_i ||x_i||_2,   A: m x n, b: m x l, x: n x l
 * (row-major, contiguous; group i = row i of x, contiguous along l).
 *
 * This ABI replaces the bodies of the reference's solver functions, which all share the
 * signature  gl_<method>(x0, A, b, mu_0, opts) -> (x, iters, out):
 *   GLX_PROXGD  <- code/gl_ProxGD_primal.py:9-146   (proximal gradient + Armijo line search)
 *   GLX_FPROXGD <- code/gl_FProxGD_primal.py:9-161  (FISTA + backtracking)
 *   GLX_SGD     <- code/gl_SGD_primal.py:9-109      (subgradient)
 *   GLX_GD      <- code/gl_GD_primal.py:9-112       (gradient on the smoothed problem)
 *   GLX_FGD     <- code/gl_FGD_primal.py:9-163      (Nesterov on the smoothed problem)
 * and the dense products inside them (A @ x at gl_ProxGD_primal.py:25,61,129 and
 * A.T @ r at :129), which NumPy sends to host BLAS.
 *
 * Conventions
 *   - Every pointer named "device" is HBM memory on the current HIP device; the library never
 *     allocates it: callers (the Python layer, through PyTorch) own A, b, x and the workspace.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream). All calls are
 *     stream-ordered; glx_session_run() additionally synchronises the stream to read the
 *     scalars its control flow needs (line-search tests, the stop rule).
 *   - Return value: 0 on success, a GLX_E* code otherwise; glx_last_error() describes the
 *     failure (thread-local). No C++ exception crosses the ABI.
 *   - dtype is the compute type: GLX_F64 (double) or GLX_F32 (float). Scalars cross the ABI as
 *     double and are rounded to dtype where the reference's NumPy would (NEP 50 weak scalars).
 */
#ifndef GLX_H_
#define GLX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GLX_ABI_VERSION 2

enum glx_dtype { GLX_F32 = 0, GLX_F64 = 1 };
enum glx_method { GLX_PROXGD = 0, GLX_FPROXGD = 1, GLX_SGD = 2, GLX_GD = 3, GLX_FGD = 4 };
/* step_type option (gl_ProxGD_primal.py:78-101) */
enum glx_step { GLX_STEP_LINE_SEARCH = 0, GLX_STEP_FIXED = 1, GLX_STEP_DIMINISHING = 2,
                GLX_STEP_DIMINISHING2 = 3 };
enum glx_status { GLX_OK = 0, GLX_E_INVALID = 1, GLX_E_HIP = 2, GLX_E_RCCL = 3,
                  GLX_E_WORKSPACE = 4, GLX_E_STATE = 5 };

/* Solver options; field names and defaults follow the reference's default_opts dicts
 * (gl_ProxGD_primal.py:10-19 etc.). glx_default_opts() fills the per-method defaults. */
typedef struct glx_opts {
  int32_t maxit;                  /* iterations per continuation phase                   */
  double  thres;                  /* hard threshold / prox denominator switch (1e-3)      */
  int32_t step_type;              /* enum glx_step                                        */
  double  alpha0;                 /* initial / fixed step                                 */
  double  ftol;                   /* stop rule relative tolerance                         */
  int32_t stable_len_threshold;   /* stop after this many consecutive stable iterations   */
  double  ls_coeff;               /* line_search_attenuation_coeffi                       */
  int32_t ls_maxit;               /* maxit_line_search_iter                               */
  double  delta;                  /* smoothing parameter (GD / FGD)                       */
  int32_t continuous_subgradient; /* SGD/GD: alpha0 = 1/lambda_max(A^T A) (caller-computed:
                                     pass alpha0 accordingly; kept for ABI completeness)   */
  /* ---- build-only keys (the reference has no equivalent) ---- */
  int32_t exact_objective;        /* ProxGD: 1 = evaluate the next objective at the accepted
                                     x = prox(x - t*grad) itself (a third right-hand side in
                                     the same pass over A: A@[z | p_thr | p]), bit-faithful to
                                     the reference's evaluation order; 0 = reuse the accepted
                                     line-search residual A@z, z = x - t*G_t (ulp-level
                                     difference, SURVEY.md §8a reuse table)                   */
  int32_t profile;                /* k > 0: time every k-th A@x / A^T r launch (HIP events) */
  int64_t max_total_iters;        /* stop after this many iterations in total (0 = off)     */
  int32_t ax_variant;             /* A@x kernel variant for A/B tests (0 = auto)            */
  int32_t split_cand;             /* fp64 ProxGD / FProxGD split-candidate trial (A p = A p_thr
                                     + A e, A e gathered from a transposed copy of A): 0 = auto
                                     (on when this rank's A is >= 768 MiB; GLX_SPLIT_CAND env
                                     overrides), 1 = on at any size, 2 = off. On adds an m x n
                                     copy of A to the workspace (glx_workspace_bytes counts it) */
  int32_t dc_window;              /* device-controlled line search (ProxGD / FProxGD): 0 = auto
                                     (GLX_DC_BATCH env, else the measured default: 8 for
                                     FProxGD with a communicator, off otherwise), -1 = off,
                                     k in 1..32 = up to k iterations queued ahead of the host   */
  int32_t shard_rows;             /* ProxGD with a communicator of G > 1 ranks: 0 = auto (on),
                                     1 = on, 2 = off. On: the row-sharded schedule — the gradient
                                     is reduce-scattered, the prox / trial runs on this rank's
                                     n / G rows and the new iterate's rows are all-gathered
                                     (needs n % G == 0); off: the gradient is all-reduced and
                                     every rank runs the row-wise step on all n rows            */
  int32_t shard_model;            /* BENCHMARK ONLY (bench.py --shard-model): G > 1 with a world-1
                                     communicator runs the per-rank timing model of G ranks of the
                                     row-sharded ProxGD schedule (the trial on n / G rows, every
                                     line-search test accepted). Its iterates are NOT a solve:
                                     glx_solve refuses it and glx_session_describe says
                                     "(timing model)". 0 = off                                  */
  int32_t reserved[3];
} glx_opts;

/* One problem instance. For multi-GPU runs A and b are this rank's row shard
 * (m = local rows) and `comm` is a communicator from glx_comm_create(); x, mu and the
 * options are replicated on every rank. */
typedef struct glx_problem {
  int32_t dtype;        /* enum glx_dtype                                    */
  int32_t method;       /* enum glx_method                                   */
  int64_t m, n, l;      /* local rows of A, columns of A (= groups), columns of b/x */
  const void* A;        /* device, m x n row-major                          */
  const void* b;        /* device, m x l                                    */
  void* x;              /* device, n x l: x0 on entry, the iterate on return */
  double mu0;           /* mu_0                                             */
  void* comm;           /* glx_comm* or NULL                                */
} glx_problem;

typedef struct glx_result {
  int64_t iters;        /* k: total iterations (the reference's second return value) */
  double fval;          /* objective of the returned x (out["fval"])                 */
  double tt;            /* seconds spent in the iteration loop, stream-synchronised   */
  double* f_hist;       /* host, capacity f_cap: objective per iteration (out["f_hist"]) */
  double* f_hist_best;  /* host, capacity f_cap (out["f_hist_best"])                 */
  int64_t f_cap;
  int64_t n_fhist;      /* entries written                                           */
  int64_t ax_calls;     /* passes of A@x issued (executed-work accounting)            */
  int64_t atr_calls;    /* passes of A^T r issued                                     */
  int64_t syncs;        /* host readbacks the device queue drains behind (the host decides
                           before queuing more work; a device-controlled batch counts one) */
  int64_t ax_sources;   /* right-hand sides batched into those A@x passes (>= ax_calls) */
  double stats[8];      /* diagnostics: [0] threshold-changed entries and [1] rows summed over
                           accepted ProxGD steps, [2] accepted steps; split-candidate
                           FProxGD: [3] gathered batches, [4] dense batches, [5] nnz(e_c)
                           summed over the gathered ones, [6] A thr(x_k) restores;
                           [7] iterations whose line-search decision ran on the device  */
  int64_t record_waits; /* device-controlled batches: decision records the host read while
                           later iterations stayed queued on the device                   */
} glx_result;

typedef struct glx_session glx_session;
typedef struct glx_comm glx_comm;

int         glx_abi_version(void);
const char* glx_last_error(void);
int         glx_default_opts(int method, glx_opts* out);

/* Workspace (device bytes) a session needs for this problem and these options (includes the
 * transposed copy of A of the split-candidate trial, opts.split_cand, and the gradient-set ring
 * of device control with a communicator, opts.dc_window). Environment overrides (GLX_*) are read
 * here and at create: keep them unchanged in between. */
int glx_workspace_bytes(const glx_problem* prob, const glx_opts* opts, size_t* bytes);

/* Session API: the reference loop split so that a caller can time exactly K iterations.
 * create  — validates shapes, carves the workspace, copies nothing (x is used in place).
 * run     — runs up to max_steps further iterations (<=0: to completion); *done = steps run.
 *           *finished = 1 once all continuation phases are over.
 * finish  — evaluates fval of the current x and copies the histories into res.
 * destroy — frees host-side state (pinned buffers, events). */
int  glx_session_create(glx_session** out, const glx_problem* prob, const glx_opts* opts,
                        void* workspace, size_t workspace_bytes, void* stream);
int  glx_session_run(glx_session* s, int64_t max_steps, int64_t* done, int32_t* finished);
int  glx_session_finish(glx_session* s, glx_result* res);
/* launches timed and their total device time (ms) for A@x (kind 0: the dense pass) / A^T r
 * (kind 1) / the split-candidate A e gather (kind 2), sampled every opts.profile-th launch of that
 * kind; resets the accumulators. */
int  glx_session_kernel_time(glx_session* s, int kind, int64_t* launches, double* total_ms);
/* executed-work counters since create: out = {A@x passes, right-hand sides in them, A^T r
 * passes, host readbacks (glx_result.syncs)} (cumulative; the caller differences them around a
 * timed region). */
int  glx_session_counters(glx_session* s, int64_t out[4]);
/* Progress record, safe to call from ANOTHER thread while glx_session_run() is in progress (a
 * watchdog's diagnostic, round 6): out = {iterations recorded so far (k), continuation phase
 * (0..2), what the host is waiting on (0 nothing, 1 a scalar packet, 2 a device decision record),
 * collectives issued on the session's communicator (0 without one)}. */
int  glx_session_progress(glx_session* s, int64_t out[4]);
/* After glx_session_finish: what the reference's 'opt' logger prints, so a host can replay it
 * without touching the hot loop (gl_ProxGD_primal.py:54 `new mu=` per phase, :134-136 the line
 * every 100 iterations; same in gl_FProxGD_primal.py:56,149-151 and gl_SGD_primal.py:49,98-99).
 * sparsity_after[i] = sparsity of the iterate after iteration i+1's update (NaN where not
 * recorded: SGD/GD record it at every 100th iteration only); *n = entries written (with
 * sparsity_after == NULL: entries available). phase_info[p] = k at the start of phase p (-1 if
 * never entered), phase_info[3 + p] = 1 if the stop rule ended phase p (that iteration logs
 * nothing, :118-125). */
int  glx_session_trace(glx_session* s, double* sparsity_after, int64_t cap, int64_t* n,
                       int64_t phase_info[6]);
/* One-line description of the kernels this session launches (the planner's tiles and splits
 * after the session's own choices: the fused trial, the split-candidate form, the device-control
 * window), NUL-terminated, truncated to cap. */
int  glx_session_describe(glx_session* s, char* out, size_t cap);
/* The split-candidate trials' sparsity, one value per trial batch so far (diagnostic): ProxGD the
 * rows of e = p - p_thr (accepted trials), FProxGD nnz(e_c) of a gathered batch (flagged rows in
 * the row form) or -1 for a dense batch. *n = the count; up to cap values copied to out. */
int  glx_session_split_trace(glx_session* s, double* out, int64_t cap, int64_t* n);
void glx_session_destroy(glx_session* s);

/* One-shot solve: create + run to completion + finish + destroy. */
int glx_solve(const glx_problem* prob, const glx_opts* opts, void* workspace,
              size_t workspace_bytes, glx_result* res, void* stream);

/* ---- single kernels (test / composition surface) ---- */
/* R = A X - B (m x l); *half_sumsq_dev = 1/2 ||R||^2 (device double). */
int glx_residual(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* X,
                 const void* B, void* R, void* half_sumsq_dev, void* workspace,
                 size_t workspace_bytes, int variant, void* stream);
/* Batched right-hand sides in one pass over A: R[i] = A X[i] - B for i < nsrc (nsrc <= 3);
 * sumsq_dev[i] = ||R[i]||^2 (device doubles, 4 slots). */
int glx_residual_batch(int dtype, int64_t m, int64_t n, int64_t l, const void* A, int nsrc,
                       const void* const* X, const void* B, void* const* R, void* sumsq_dev,
                       void* workspace, size_t workspace_bytes, int variant, void* stream);
/* G = A^T R (n x l). */
int glx_gradient(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* R,
                 void* G, void* workspace, size_t workspace_bytes, void* stream);
/* X_out = prox_{t*mu*||.||_{1,2}}(W) with the reference's (||w_i|| < thres) + ||w_i||
 * denominator (gl_ProxGD_primal.py:65-71); sums_dev[0] = sum_i ||X_out_i||,
 * sums_dev[1] = max |X_out| (device doubles). */
int glx_prox(int dtype, int64_t n, int64_t l, const void* W, double t, double mu, double thres,
             void* X_out, void* sums_dev, void* workspace, size_t workspace_bytes, void* stream);
/* R = A X - B (m x l) and G = A^T R (n x l) (reference gl_ProxGD_primal.py:129
 * `A.T @ (A @ x - b)`). one_pass = 0: A @ X, then A^T R (two passes over A, the faster path on
 * MI355X); one_pass = 1: the fused residual-gradient kernel reads A from HBM once
 *  where the shape and device allow it (fp64, l = 32, n = 512 P with P a power
 * of two in 2..128, m a multiple of 16 * 256 / P, >= 256 CUs), else two passes. The one-pass
 * kernel is a cooperative launch (its workgroups wait for each other); if the runtime refuses it,
 * or a hand-off wait inside it times out (error flag read back: the one-pass call is synchronous),
 * R and G are recomputed with two passes. *one_pass_ran (may be NULL) = 1 when the returned R
 * and G come from the fused kernel. */
int glx_residual_gradient(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* X,
                          const void* B, void* R, void* G, void* workspace, size_t workspace_bytes,
                          int one_pass, int* one_pass_ran, void* stream);
/* The line-search trial's batch and the next gradient (round 4, SURVEY §8f row 1 at l = 16):
 * R0 = A X0 - B, R1 = A X1 - B (the reference's A @ z and A @ p_thr, gl_ProxGD_primal.py:89-92,
 * :112) and G = A^T R1 (:129 at the candidate). one_pass = 1: one read of A by the role-split
 * kernel (kernels_rg2.hip) where the shape allows it (fp64, l = 16, n = 256 P with P a power of
 * two in 2..128, m a multiple of 64 * 256 / P, >= 256 CUs; slower than two passes on MI355X,
 * DESIGN.md (f), so the solver does not use it); a timed-out hand-off wait inside it
 * (error flag read back: the one-pass call is synchronous) or another shape runs A @ [X0 | X1],
 * then A^T R1. *one_pass_ran (may be NULL) = 1 when the outputs come from the one-pass kernel. */
int glx_residual_gradient2(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* X0,
                           const void* X1, const void* B, void* R0, void* R1, void* G,
                           void* workspace, size_t workspace_bytes, int one_pass,
                           int* one_pass_ran, void* stream);
/* The thresholded part of the split-candidate line-search trial (round 5, SURVEY §8a row a9:
 * A e with e = p - p_thr nonzero only in the rows the hard threshold touched,
 * gl_ProxGD_primal.py:91,112,127; FProxGD's A e_c, gl_FProxGD_primal.py:92-97,136):
 *   Y (m x l) = sum over the rows k with row_masks[k] != 0 of At[k,:]^T E[k,:],  At = A^T (n x m).
 * row_masks[k] (device uint32, n + 3 readable) = the column mask of row k of E (bit c = E[k][c] != 0,
 * as the trial kernels write it). form 0: the MFMA row form (k_at_rows; FProxGD's default in the
 * solver, m % 64 == 0); form 1: the VALU column-list gather of rounds 2-4; form 2: the bitmap gather
 * (ProxGD's default in the solver since round 5, bit-identical to form 1). Forms 1, 2 need the exact
 * column masks. NOTE: these form codes are this entry point's own; they are NOT the codes of the
 * GLX_GATHER environment variable (bm / rows / lists). */
int glx_flagged_rows_product(int dtype, int64_t m, int64_t n, int64_t l, const void* At,
                             const void* E, const uint32_t* row_masks, void* Y, int form,
                             void* workspace, size_t workspace_bytes, void* stream);
/* Workspace bytes for the single-kernel entry points above. */
int glx_kernel_workspace_bytes(int dtype, int64_t m, int64_t n, int64_t l, size_t* bytes);
/* One-line description of the kernels (tile, split) the planner picks for this shape, for
 * A @ X with 1, 2, 3 right-hand sides and for A^T R (NUL-terminated, truncated to cap). */
int glx_plan_describe(int dtype, int64_t m, int64_t n, int64_t l, char* out, size_t cap);

/* ---- multi-GPU (row-sharded A; A^T r all-reduced, or reduce-scattered with the row-sharded step) ---- */
#define GLX_COMM_ID_BYTES 128
int  glx_comm_unique_id(uint8_t id[GLX_COMM_ID_BYTES]);
int  glx_comm_create(glx_comm** out, const uint8_t id[GLX_COMM_ID_BYTES], int nranks, int rank);
/* Host-staged transport (testing: several ranks sharing one GPU, which RCCL refuses). Each
 * all-reduce synchronises the stream, copies the buffer to pinned host memory, calls
 * fn(host_buf, count, dtype, user) — which must sum it in place across ranks and return 0 —
 * and copies it back. Not a performance path. */
typedef int (*glx_host_allreduce_fn)(void* host_buf, int64_t count, int dtype, void* user);
int  glx_comm_create_host(glx_comm** out, int nranks, int rank, glx_host_allreduce_fn fn, void* user);
/* in-place sum all-reduce of `count` elements of dtype on `stream` (exposed for tests) */
int  glx_comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, void* stream);
/* The row-sharded schedule's collectives (round 5, exposed for tests), in place over nranks
 * chunks of `count` elements: reduce-scatter leaves in chunk `rank` the sum over ranks of that
 * chunk (other chunks undefined); all-gather sends chunk `rank` and receives every chunk. The
 * host transport runs both through the all-reduce callback (all-gather exactly: the chunks it
 * does not own are -0.0). */
int  glx_comm_reduce_scatter(glx_comm* c, void* buf, int64_t count, int dtype, void* stream);
int  glx_comm_all_gather(glx_comm* c, void* buf, int64_t count, int dtype, void* stream);
/* Progress record, safe to call from another thread (round 6): out = {collectives issued,
 * collectives the host transport completed (-1 for RCCL), kind of the last one issued (1 all-reduce,
 * 2 reduce-scatter, 3 all-gather), RCCL's asynchronous error (ncclCommGetAsyncError; 0 none, -1
 * aborted)}. A session whose host wait on RCCL sees an asynchronous error, or waits longer than
 * GLX_WAIT_TIMEOUT_S (default 300 s), aborts the communicator and fails with GLX_E_RCCL and this
 * record in glx_last_error(). */
int  glx_comm_progress(glx_comm* c, int64_t out[4]);
void glx_comm_destroy(glx_comm* c);

#ifdef __cplusplus
}
#endif
#endif /* GLX_H_ */
