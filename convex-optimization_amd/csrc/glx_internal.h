// glx_internal.h — declarations shared by the HIP kernels and the host-side driver.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <string>
#include <tuple>
#include <utility>

#include "glx.h"

namespace glx {

// error carried to the C ABI boundary (never crosses it)
struct Error {
  int code;
  std::string msg;
};
extern thread_local std::string g_last_error;

// Kernel-attached HIP-event timing (solver.cpp prof_begin / prof_end). A sampled A@X / A^T R /
// gather launch sets this slot; the next glx_launch on the thread hands the two events to
// hipExtLaunchKernel, which stamps them with that kernel's own start and end, and clears it.
// Round 3: hipEventRecord around the launch instead put two marker packets in the queue, each
// opening a ~6 us gap before the next kernel (profiles/r3_timeline/: the driver-form command,
// every second launch timed, ran 5 gaps per two iterations, ~3-4 % of its time).
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchTiming g_launch_timing;

template <typename... P, std::size_t... I>
inline hipError_t ext_launch(void (*kern)(P...), dim3 g, dim3 b, uint32_t sh, hipStream_t st,
                             std::tuple<P...>& t, std::index_sequence<I...>, hipEvent_t e0,
                             hipEvent_t e1) {
  void* args[sizeof...(P) > 0 ? sizeof...(P) : 1] = {static_cast<void*>(&std::get<I>(t))...};
  return hipExtLaunchKernel(reinterpret_cast<const void*>(kern), g, b, args, sh, st, e0, e1, 0);
}
// hipLaunchKernelGGL, or the timed form when a timing slot is pending. The arguments are
// converted to the kernel's own parameter types first (hipExtLaunchKernel takes raw pointers
// to them, so an int passed for an int64_t must not reach it unconverted).
template <typename... P, typename... A>
inline void glx_launch(void (*kern)(P...), dim3 g, dim3 b, uint32_t sh, hipStream_t st, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "argument count");
  LaunchTiming& lt = g_launch_timing;
  if (lt.start != nullptr) {
    std::tuple<P...> t(static_cast<P>(std::forward<A>(a))...);
    const hipEvent_t e0 = lt.start, e1 = lt.stop;
    lt = LaunchTiming{};
    const hipError_t e = ext_launch(kern, g, b, sh, st, t, std::index_sequence_for<P...>{}, e0, e1);
    if (e != hipSuccess) {
      // the events were not taken: hand the slot back, so prof_end (or the session's destructor)
      // returns them to the pool instead of losing them
      lt = LaunchTiming{e0, e1};
      throw Error{GLX_E_HIP, std::string("timed kernel launch: ") + hipGetErrorString(e)};
    }
    return;
  }
  hipLaunchKernelGGL(kern, g, b, sh, st, std::forward<A>(a)...);
}

constexpr int kMaxBlocks = 1024;   // grid cap of every reducing kernel (size of a partials row)
constexpr int kMaxRedVals = 6;     // max scalars one reducing kernel produces
constexpr int kMaxL = 128;         // largest l (columns of x) supported by the row kernels
// Arrival tickets: kTicketShards per-XCD counters plus one final counter, each on its own
// 128-B line (32 unsigned words apart). Word 0 = final counter, shard s at (1 + s) * 32.
constexpr int kTicketShards = 8;
constexpr int kTicketStride = 32;
constexpr int kTicketBytes = 2048;  // >= (kTicketShards + 1) * 128, keeps 256-B alignment

// Deterministic grid-wide reduction target: each block writes its partial to
// part[v * kMaxBlocks + block]; the last block (arrival ticket) sums them in block order
// and writes out[v]. `ticket` (kTicketBytes) must be zero before the first launch; the last
// block resets it.
struct Red {
  double* part;
  unsigned* ticket;
  double* out;     // kMaxRedVals consecutive doubles (caller picks the slots)
  // device-controlled batches (solver.cpp dc_run): the whole launch is skipped, uniformly over
  // the grid (nobody touches a ticket or counter), when skip != NULL and *skip is neither 0 nor
  // skip_pass
  const int* skip = nullptr;
  int skip_pass = 0;
  // 1: every workgroup stores its NV block values at part[slot * NV + j] and returns (no tickets,
  // no out): the row-sharded trial's partials ride the all-gather (ShardPub)
  int parts_only = 0;
};

// Device-side line-search decision of a device-controlled ProxGD batch (solver.cpp dc_batch),
// run by the last block of the trial's residual finalize once the residual sums are final
// (gl_ProxGD_primal.py:86-99 Armijo test, :118-125 stop rule). ring == NULL: off.
//   state[0..3] = gx (1/2 ||A thr(x) - b||^2), f and sparsity of the last record, stable count
//   tr = the trial's six sums (k_prox_pgd / k_atr_prox), t = the trial's step
// On acceptance the next record (f, s) and the stop rule are evaluated and the state advances.
// *abort = 0 (accepted), pass (accepted, the next record stops the phase, or code 3), -1 (rejected):
// the speculative gradient queued right behind this decision runs on 0 and on this tag
// (Red::skip_pass), the rest of the batch only on 0. ring[10] = 0, 1 (stop), 2 (rejected),
// 3 (FProxGD: accepted, nnz budget exceeded).
// rec[0..10] (device) = the four residual sums, the six trial sums and the code as a double.
// The speculative kernel queued behind the decision hands rec to the host from its publisher
// workgroup (Pub), also when the decision cancels it, so the PCIe write latency stays off the
// finalize's critical path.
//
// mode 1 = FProxGD's backtracking test (gl_FProxGD_primal.py:89-103): state[0] = ||A y - b||^2 of
// the current y (not halved), the test g(xc) <= g(y) + <g, xc - y> + ||xc - y||^2 / (2t) from the
// batch's residual sums and the trial's four sums, and on acceptance state[0] = ||A y_next - b||^2.
// A gathered (split-candidate) batch also checks nnz(e_c) = out[2] against nnz_budget (>= 0): above
// it the next batches are dense on the host path (solver.cpp kFistaDenseRun), so the decision
// cancels the batch behind it like a stop (code 3: accepted, the speculative kernel runs).
struct Ctl {
  double* rec = nullptr;
  double* state = nullptr;
  int* abort = nullptr;
  const double* tr = nullptr;
  double tag = 0.0, t = 0.0, mu0 = 0.0, ftol = 0.0, nl = 1.0;
  double nnz_budget = -1.0;
  int stable_thr = 0, use_sp = 1, emode = 0;
  int mode = 0;    // 0 ProxGD, 1 FProxGD
  int pass = 0;    // nonzero; the abort word's value for "stop" (Red::skip_pass of the kernel behind)
};
constexpr int kCtlRec = 16;        // doubles per ring record
constexpr int kCtlMaxBatch = 64;   // ring records

// A scalar packet for the host (what k_publish writes) carried by a kernel launch as one extra
// workgroup (publisher_first, glx_device.h); host == NULL: none.
struct Pub {
  const double* s = nullptr;
  int ns = 0;
  double* host = nullptr;
  unsigned* host_seq = nullptr;
  unsigned seq = 0;
  const double* s2 = nullptr;   // host[off2 .. off2 + n2) come from s2 instead of s
  int off2 = 0, n2 = 0;
  const double* s3 = nullptr;   // host[off3 .. off3 + n3) come from s3 (a snapshot)
  int off3 = 0, n3 = 0;
  // Round 5, deferred reductions: workgroup partials (Red::parts_only layout: dnv values per
  // slot, dnp slots) that the publishing workgroup reduces (dmax bit j: max) into dout[0, dnv)
  // before it copies the packet, so the kernels that produced them skip their grid reduction's
  // serial tail (solver.cpp defer_)
  const double* dpart[2] = {nullptr, nullptr};
  int dnp[2] = {0, 0}, dnv[2] = {0, 0};
  unsigned dmax[2] = {0u, 0u};
  double* dout[2] = {nullptr, nullptr};
};

// Launch plan of the two dense products for one (dtype, m, n, l).
struct GemmPlan {
  int esize;        // 4 or 8
  int64_t m, n, l;
  // A @ X  ->  P[ax_S][m][l] partial slabs (summed by finalize_residual)
  int ax_kind;      // 1 = MFMA direct row loads, 2 = MFMA quad loads + bpermute, 3 = VALU
  int ax_mt, ax_pf; // MFMA: 16-row tiles per wave, chunks in flight per wave
  int ax_code;      // MFMA variant code (kind*1000 + MT*100 + PF*10 + non-temporal)
  int ax_S;         // K (= n) splits across workgroups
  int ax_xmap;      // MFMA: group K splits by XCD (L2 locality of X)
  int ax_lb;        // VALU: column block width (1,2,4,8); ax_ncb = ceil(l / ax_lb)
  int ax_vec;       // VALU: 16-byte loads
  // per number of batched right-hand sides (index 1..3; [1] mirrors ax_code / ax_S):
  // MFMA variant code (kind 5 = X staged in LDS: 5 MT PF VPL WAVES) and its K split
  int axb_code[4];
  int axb_S[4];
  // A^T R  ->  Gp[atr_S][n][l]
  int atr_kind;     // 1 = MFMA, 3 = VALU
  int atr_wl, atr_pf; // MFMA: wave layout (0 = waves split rows, 1 = waves split columns), ring depth
  int atr_ntl;      // non-temporal A loads
  int atr_S;        // M (= m) splits across workgroups
  int atr_lb, atr_vec;
  // Infinity-Cache hand-off between the two non-temporal passes (Session sets them; 0 = off):
  // the last ~that many MiB a pass reads load with the default policy (kernel arguments, so
  // every session and device gets its own value)
  int ax_keep_mib = 0, atr_keep_mib = 0;
};

GemmPlan make_plan(int esize, int64_t m, int64_t n, int64_t l, int ax_variant);
// K split (number of partial slabs per source) of an A@X launch with nsrc right-hand sides
inline int ax_split(const GemmPlan& p, int nsrc) { return nsrc > 1 ? p.axb_S[nsrc] : p.ax_S; }
inline int ax_split_max(const GemmPlan& p) {
  int s = p.ax_S;
  for (int k = 2; k <= 3; ++k) s = s > p.axb_S[k] ? s : p.axb_S[k];
  return s;
}
// largest K split any A@X variant (single or batched) plans for this shape
int max_ax_split(int esize, int64_t m, int64_t n, int64_t l);
// one-line description of the kernels and splits a plan launches (glx_plan_describe)
std::string describe_plan(const GemmPlan& p);

// ---- dense products (kernels_gemm.hip) ----
// A @ [X[0] | .. | X[nsrc-1]] (nsrc <= 3, each n x l) in one pass over A: partial slabs
// P[src][ax_split(p, nsrc)][m][l]; skipped entirely unless gate == NULL or *gate == epoch.
// pub.host != NULL: the launch also hands that scalar packet to the host from its first
// workgroup (needs ax_pub_ok: the kind-5 LDS tile for nsrc).
bool ax_pub_ok(const GemmPlan& p, int nsrc);
template <typename T>
void launch_ax(const GemmPlan& p, int nsrc, const T* A, const T* const* X, T* P, const int* gate,
               int epoch, hipStream_t st, Pub pub = Pub{});
// the kind-8 (LDS-DMA, f64) A @ X tile of `code` (kernels_axdma.hip); false: unknown code.
// dma_lds_need: its LDS bytes for l columns and nsrc right-hand sides (<= 160 KiB to launch).
template <typename T>
bool launch_ax_dma(const GemmPlan& p, int code, int nsrc, int S, const T* A, const T* const* X, T* P,
                   const int* gate, int epoch, hipStream_t st, Pub pub);
int dma_lds_need(int code, int64_t l, int nsrc, int esize);
// Round 6: the split-candidate trial's A e inside its dense pass (NS's one-source f64 LDS-DMA tile
// 92278): the pass streams A p (X = the candidate p) on MFMA and, for the entries the column
// bitmaps behind zf flag (glx_device.h zf_bitmaps; there e = p), accumulates A[:, k] e[k, c] on
// VALU from the A and p chunks already in LDS: no transposed copy of A, no gather pass, no second
// source. P[S][m][l] = A p slabs, Pe[S][m][l] = the A e slabs (one per K split); the finalize's
// chain mode 2 forms A p - b and A p_thr - b = (A p - b) - A e.
struct EGat {
  const void* E = nullptr;               // unused (e is read from the staged p)
  const unsigned short* bm = nullptr;    // zf_bitmaps(zf, n): column c's u16 words at c * bstride
  int64_t bstride = 0;                   // zf_npad(n) / 16
  void* Pe = nullptr;
};
bool ax_egat_ok(const GemmPlan& p, int esize);
template <typename T>
bool launch_ax_egat(const GemmPlan& p, const T* A, const T* X, T* P, const int* gate, int epoch,
                    hipStream_t st, Pub pub, const EGat& eg);
int dma_waves(int code);   // waves per workgroup of a kind-8/9 code (last digit; 1 = 16)
int dma_mt(int code);      // 16-row tiles per wave (kind 9: 2)
// Infinity-Cache hand-off between the passes (tuning experiment; MiB of A fetched with the
// default policy at the end of a non-temporal pass; 0 = off): A@X (LDS-DMA tile) / A^T R
template <typename T>
void launch_atr(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st);
// ProxGD trial fused into A^T R (needs atr_prox_ok: MFMA panels, WL 0, at most 8 K splits):
// G = A^T R, then p = prox(x - t G), p_thr, z and the six trial sums of k_prox_pgd into red
// (zf != NULL: z = e = p - p_thr and its row flags, as launch_prox_pgd).
// With S = atr_S > 1 K splits the blocks write slabs Gp[S][n][l] and the last block of each
// 64-row panel (counter pcnt[panel], zero before the first launch, reset by that block) sums
// them in slab order and runs the trial.
bool atr_prox_ok(const GemmPlan& p);
template <typename T>
void launch_atr_prox(const GemmPlan& p, const T* A, const T* R, T* G, const T* x, T* pp, T* pthr,
                     T* z, double t, double mu, double thres, Red red, hipStream_t st, Pub pub = Pub{},
                     T* Gp = nullptr, unsigned* pcnt = nullptr, unsigned* zf = nullptr);
// FISTA trial fused into A^T R (same plan condition): G = A^T R, then xc, v_next, y_next and the
// four trial sums of k_fista_trial (PROX) into red (ec, zf: as launch_fista_trial).
template <typename T>
void launch_atr_fista(const GemmPlan& p, const T* A, const T* R, T* G, const T* y, const T* xk,
                      T* xc, T* vn, T* yn, double t, double mu, double thres, double theta,
                      double theta_next, Red red, hipStream_t st, Pub pub = Pub{},
                      T* Gp = nullptr, unsigned* pcnt = nullptr, T* ec = nullptr,
                      unsigned* zf = nullptr);

// ---- split-candidate A e from a transposed copy of A (kernels_gather.hip) ----
// gather_ok: the shape supports it (l in {16, 32}, n < 65536); gather_split: K splits of the
// flagged-row list for m output rows (slabs P[S][m][l]).
bool gather_ok(int64_t n, int64_t l);
// round 5: the MFMA row form (k_at_rows): the shapes it takes, the solver's default (GLX_GATHER=valu:
// the column-list gather, ONE slab), and its K splits for this shape (1 where it does not apply)
bool gather_rows_ok(int64_t m, int64_t n);
int gather_form();   // GLX_GATHER: 0 bitmaps, 1 MFMA rows, 2 k_e_lists + k_at_gather, -1 unset
int gather_split(int64_t m, int64_t n);
// zf: the per-row column masks of e and, behind them, the per-column row bitmaps (glx_device.h)
size_t zf_bytes(int64_t n);
// A e from the column bitmaps behind zf (ONE slab at P; the column list lengths to gather_counts)
template <typename T>
void launch_at_gather_bm(const T* At, const T* E, unsigned* zf, int64_t m, int64_t n, int64_t l, T* P,
                         void* lists_ws, hipStream_t st, const int* skip = nullptr);
// the column bitmaps behind zf from its row masks (where no trial kernel wrote them)
void launch_zf_bitmaps(unsigned* zf, int64_t n, int64_t l, hipStream_t st);
// P[s][r][c] = sum over the flagged rows k (zf[k] != 0) of K range s, ascending:
// At[k][r] E[k][c], s < gather_split(m, n); counts[s] (gather_counts) = the flagged rows of range s
template <typename T>
void launch_at_rows(const T* At, const T* E, const unsigned* zf, int64_t m, int64_t n, int64_t l,
                    T* P, void* lists_ws, hipStream_t st, const int* skip = nullptr);
// At (n x m) = A^T
template <typename T>
void launch_transpose(const T* A, T* At, int64_t m, int64_t n, hipStream_t st);
// launch_e_lists: per column c the ascending k with bit c of zm[k] set (zm: the per-row column
// masks of e the trial kernels write), into lists_ws (gather_lists_bytes(n));
// launch_at_gather: P[r][c] = sum over column c's list of At[k][r] E[k][c] (one slab)
size_t gather_lists_bytes(int64_t n);
// the l per-column list lengths inside lists_ws (device)
const unsigned* gather_counts(const void* lists_ws, int64_t n);
void launch_e_lists(const unsigned* zm, int64_t n, int64_t l, void* lists_ws, hipStream_t st,
                    const int* skip = nullptr);
template <typename T>
void launch_at_gather(const T* At, const T* E, int64_t m, int64_t n, int64_t l, T* P, void* lists_ws,
                      hipStream_t st, const int* skip = nullptr);

// ---- fused residual + gradient in one pass over A (kernels_fused.hip) ----
// Sraw = A X (m x 32) and Gs[RG][n][32] with G = A^T (A X - B) = sum of the RG slabs in order.
// resgrad_shape_ok: fp64, l = 32, n % 512 == 0, m % (16 RG) == 0; resgrad_device_ok: all 256
// workgroups can be resident (>= 256 CUs). ws: resgrad_ws_bytes; its counters must be zeroed
// (resgrad_reset) before launch_count 1, and launch_count must grow by one per launch.
bool resgrad_shape_ok(int esize, int64_t m, int64_t n, int64_t l);
bool resgrad_device_ok();
int resgrad_groups(int64_t n);
size_t resgrad_ws_bytes(int64_t m, int64_t n);
void resgrad_reset(void* ws, int64_t m, int64_t n, hipStream_t st);
// returns false (nothing launched) when the runtime refuses the cooperative launch; *err != 0
// after the launch: a hand-off wait timed out or the XCD grouping failed, R / G are invalid
// ---- the trial's batch + the next gradient in one pass, l = 16 (kernels_rg2.hip, round 4) ----
// P0 = A X0, P1 = A X1 (one m x 16 slab each), Gs[RG][n][16] with G = A^T (P1 - B) = the sum of the
// RG slabs in order. resgrad2_shape_ok: fp64, l = 16, n = 256 P (P a power of two in 2..128),
// m % (16 kRAB RG) == 0 (kRAB = 4 A-tiles per hand-off: 64 * 256 / P), m / RG >= 32 (RG = 256 / P). Plain launch of 256 workgroups that wait for each
// other with bounded spins (*err = 1 on a timeout: outputs invalid); resgrad2_device_ok checks
// that all of them can be resident. ws: resgrad2_ws_bytes, zeroed (resgrad2_reset) before
// launch_count 1; launch_count grows by one per launch on the same workspace.
bool resgrad2_shape_ok(int esize, int64_t m, int64_t n, int64_t l);
bool resgrad2_device_ok();
int resgrad2_groups(int64_t n);
size_t resgrad2_ws_bytes(int64_t n);
void resgrad2_reset(void* ws, int64_t n, hipStream_t st);
void launch_resgrad2(const double* A, const double* X0, const double* X1, const double* B,
                     double* P0, double* P1, double* Gs, void* ws, unsigned launch_count, int64_t m,
                     int64_t n, int* err, hipStream_t st);
bool launch_resgrad(const double* A, const double* X, const double* B, double* Sraw, double* Gs,
                    void* ws, unsigned launch_count, int64_t m, int64_t n, int* err, hipStream_t st);

// ---- row / elementwise kernels (kernels_elem.hip) ----
// Gradient inputs `g` with an `S` argument are S split-K slabs of n*l values summed in slab
// order on the fly (S = 1: an already-summed array).
//
// R[src] = sum_s P[src][s] - B for src < nsrc (if gate == NULL or *gate == epoch);
// out[src] = sum R[src]^2 (out[0..2]), out[3] = count(|cx| > 1e-6 * (*cmax)) when cx != NULL;
// fh != NULL: *fh = 0.5 out[0] + fh_mu * (*fh_rn) (device-side objective history).
// gate_mode: when gated off, 0 = do nothing, 1 = recompute out[0] from R[0] (nsrc = 1).
// chain (nsrc = 2, split-candidate mode): source 0 is a correction on top of source 1,
// R[0] = (sum_s P[1][s] - B) + sum_s P[0][s]; R[0] may then be NULL (only its sum is kept).
// With chain, source 0 has S0 slabs (0: S) at P and source 1 has S slabs at P + S0 * ml.
template <typename T>
void launch_finalize_residual(const T* P, int S, const T* B, int nsrc, T* const* R, int64_t ml,
                              const int* gate, int epoch, int gate_mode, const T* cx, int64_t cn,
                              const double* cmax, double* fh, double fh_mu, const double* fh_rn,
                              Red red, hipStream_t st, const double* snap_src = nullptr,
                              double* snap_dst = nullptr, int nsnap = 0, int chain = 0, int S0 = 0,
                              Ctl ctl = Ctl{}, const double* cmax_parts = nullptr, int cmax_np = 0,
                              int cmax_nv = 6);
// (cmax_parts: *cmax is still pending as the max column (index 3) of cmax_np trial partials,
// Red::parts_only layout of cmax_nv values, reduced by every workgroup for itself)
// state[0..3] = s0..s3, *abort = 0 (one thread; the seed of a device-controlled batch)
// the decision of a device-controlled ProxGD iteration with a communicator (one thread): out =
// the all-reduced residual sums (a gradient set's tail); no-op once *c.abort != 0; the record
// goes to c.rec and to the host ring (host[0..11), then *host_seq = seq)
void launch_ctl_decide(const Ctl& c, const double* out, double* host, unsigned* host_seq,
                       unsigned seq, hipStream_t st);
void launch_ctl_seed(double* state, int* abort, double s0, double s1, double s2, double s3,
                     hipStream_t st);
template <typename T>
void launch_sum_partials(const T* Gp, int S, T* G, int64_t nl, hipStream_t st);
// ProxGD trial: p = prox(x - t g, t), G_t = (x - p)/t, z = x - t G_t, pthr = p thresholded.
// out: [sum g*G_t, sum G_t^2, sum_i ||p_i||, max |p|, #changed by the threshold]
// zf != NULL (split-candidate mode): z receives e = p - p_thr instead and zf[i] = the column mask
// of row i of e (bit c = e[i][c] != 0).
template <typename T>
void launch_prox_pgd(const T* x, const T* g, int S, T* gout, T* p, T* pthr, T* z, int64_t n,
                     int64_t l, double t, double mu, double thres, Red red, hipStream_t st,
                     Pub pub = Pub{}, unsigned* zf = nullptr);
// The row-sharded trial's all-gathered sums: blk holds nranks chunks of `chunk` doubles, from
// kShardPartOff the workgroup partials (Red::parts_only) of the trial (launch_prox_pgd's out, 6
// per workgroup, nbp workgroups) and then of its finalize (launch_finalize_residual's out, 4 per
// workgroup, nbf workgroups). Combined in a
// fixed order (sums; trial slot 3: max, NaN-propagating), identical on every rank: mask & 1 ->
// tr[0, 6), mask & 2 -> rt[0, 4); with pub.host the scalar packet follows with these values.
constexpr int kShardPartOff = 16;
struct ShardPub {
  const double* blk = nullptr;
  int nranks = 1, chunk = 0, nbp = 0, nbf = 0, mask = 0;
  int tv = 6;                   // values per trial partial (ProxGD 6, FProxGD 4; the max is value 3)
  double* tr = nullptr;
  double* rt = nullptr;
  int tr_off = 0, rt_off = 0;   // their packet slots
  Pub pub{};
};
void launch_shard_combine(const ShardPub& sp, hipStream_t st);
// workgroups of launch_prox_pgd over n rows of l columns (without a packet)
int prox_blocks(int64_t n, int64_t l);
// reducing slots of launch_atr_prox (Red::parts_only partials: 6 values each)
int atr_prox_slots(const GemmPlan& p, bool pub);
// workgroups of launch_finalize_residual for these slabs and count length
int finalize_blocks(int64_t ml, int S, int S0, int64_t cn);
int finalize_fista_blocks(int64_t ml, int S, int S0, int64_t cn);
// Row-sharded schedule (round 5, solver.cpp iter_proxgd_shard): the replicated half of a ProxGD
// trial, from the all-gathered p (n x l): pthr = p with |p| < thres zeroed; z = e = p - pthr
// (emode) or z = xt - t (xt - p) / t (launch_prox_pgd's dense z, xt = the thresholded iterate);
// zf != NULL: zf[i] = the column mask of row i of e and the column bitmaps behind the masks —
// the same bits launch_prox_pgd writes.
// z == NULL: not written. sp.blk != NULL: one more workgroup runs launch_shard_combine's work
// beside the rows.
template <typename T>
void launch_trial_split(const T* p, const T* xt, T* pthr, T* z, unsigned* zf, int64_t n, int64_t l,
                        double t, double thres, bool emode, const ShardPub& sp, hipStream_t st);
// Row-sharded FProxGD (round 6, solver.cpp iter_fista_shard): the replicated half of a FISTA
// trial from the all-gathered xc (n x l): v_next = thr(xk) + (xc - thr(xk)) / theta and
// y_next = (1 - theta') thr(xc) + theta' v_next with k_fista_trial's arithmetic (fista_row), so
// the bits equal the ones that kernel would have written for the whole of xc. sp.blk != NULL: one
// more workgroup combines the gathered sums (launch_shard_combine's work) beside the elements.
template <typename T>
void launch_fista_split(const T* xc, const T* xk, T* vnext, T* ynext, int64_t nl, double thres,
                        double theta, double theta_next, const ShardPub& sp, hipStream_t st);
// Round 6: the ProxGD half above (emode, e = p, no z) fused into the split-candidate dense pass
// A p_thr (kernels_gemm.hip k_ax_lds_drv, the 8-wave shard tile 51328 at l = 32, f64): the pass
// reads the gathered p and thresholds it on the way into LDS; nd extra workgroups write p_thr,
// ggx * l more compute the trial's A e (k_at_gather_bm's work and bits) into the slab Pe beside
// the MFMA work — column c's row list from the bitmap words every rank's k_prox_pgd wrote for its
// srows rows into its sums chunk (blk + rank * bstride + moff: srows row masks, then the column
// bitmaps; all-gathered with the sums, so ready before the pass starts; bstride 0 in the one-GPU
// timing model: rank 0's words for every rank); the publisher workgroup combines sp's sums and
// publishes the packet (pub, required). False: the plan or the shape does not take it.
struct AxDerive {
  void* pthr = nullptr;
  double thres = 0.0;
  ShardPub sp{};
  int ggx = 0;                   // gather row blocks (kDrvGatRows rows each)
  int nd = 0, thr0 = 0, gat0 = 0;   // set by the launcher: p_thr workgroups, first p_thr / A e one
  const void* At = nullptr;
  const void* E = nullptr;       // e where its masks are set (the gathered p)
  void* Pe = nullptr;
  const double* blk = nullptr;
  int64_t bstride = 0, moff = 0, srows = 0;
};
bool ax_derive_ok(const GemmPlan& p, int esize);
// rows of A per gather workgroup of the fused dense pass (AxDerive::ggx = ceil(m / this)), and
// its p_thr workgroups
constexpr int kDrvGatRows = 512;
constexpr int kDrvThrBlocks = 64;
template <typename T>
bool launch_ax_derive(const GemmPlan& p, const T* A, const T* Xp, T* P, hipStream_t st, Pub pub,
                      const AxDerive& d);

// FISTA (prox = true) / FGD (prox = false: identity) trial fused with the next combine:
// xc = prox(y - t g, t); vnext = thr(xk) + (xc - thr(xk))/theta;
// ynext = (1 - theta_next) thr(xc) + theta_next vnext.
// out: prox: [sum g*(xc-y), sum (xc-y)^2, sum ||xc_i||, max |xc|]
//      FGD : [sum g*(xc-y), sum (xc-y)^2, sum (sqrt(||xc_i||^2+d^2)-d), sum ||xc_i||, max |xc|]
// ec != NULL (split-candidate mode): ec = xc - thr(xc) and zf[i] = the column mask of row i of ec.
template <typename T>
void launch_fista_trial(bool prox, const T* y, const T* g, int S, T* gout, const T* xk, T* xc,
                        T* vnext, T* ynext, int64_t n, int64_t l, double t, double mu, double thres,
                        double theta, double theta_next, double delta, Red red, hipStream_t st,
                        Pub pub = Pub{}, T* ec = nullptr, unsigned* zf = nullptr);
// split-candidate FISTA batch finalize (k_finalize_fista): P = S slabs of A xc, Pe = S0 slabs of
// A e_c, sxo = A thr(xk); Ry = A y_next - b with y_next = a1 thr(xc) + b1 (thr(xk) + (xc -
// thr(xk)) / theta), sxo_out = A thr(xc). out: [sum (A xc - b)^2, sum Ry^2,
// sum counts[0..nl) (nnz of e_c, gather_counts), count as above].
template <typename T>
void launch_finalize_fista(const T* P, int S, const T* Pe, int S0, const T* B, T* Ry, const T* sxo,
                           T* sxo_out, int64_t ml, double a1, double b1, double theta, const T* cx,
                           int64_t cn, const double* cmax, const unsigned* counts, int nl, Red red,
                           hipStream_t st, Ctl ctl = Ctl{}, const double* cmax_parts = nullptr,
                           int cmax_np = 0, int cmax_nv = 4);
// plain prox of W (glx_prox): out: [sum ||x_i||, max |x|]
template <typename T>
void launch_prox_plain(const T* w, T* x, int64_t n, int64_t l, double t, double mu, double thres,
                       Red red, hipStream_t st);
// out[0] = count(|x| > 1e-6 * (*maxv))
template <typename T>
void launch_count_above(const T* x, int64_t nl, const double* maxv, Red red, hipStream_t st);
// xo = x with |x| < thres zeroed (xo may alias x); *flag = epoch if any value changed
template <typename T>
void launch_threshold(const T* x, T* xo, int64_t nl, double thres, int* flag, int epoch, hipStream_t st);
// xk[|xk| < thres] = 0 in place; y = a*xk + b*vk
template <typename T>
void launch_thr_axpby(T* xk, const T* vk, T* y, int64_t nl, double thres, double a, double b,
                      hipStream_t st);
// v = xk + (x - xk)/theta
template <typename T>
void launch_fista_v(const T* xk, const T* x, T* v, int64_t nl, double theta, hipStream_t st);
// SGD (mode 0) / GD (mode 1) step from the thresholded iterate xt: x = xt - alpha (g + mu xt/d),
// xt = thr(x). out: [sum ||x_new_i||]
template <typename T>
void launch_descent(T* x, T* xt, const T* g, int S, int64_t n, int64_t l, double alpha, double mu,
                    double thres, double delta, int mode, Red red, hipStream_t st);
// out: [sum ||x_i||, max |x|]
template <typename T>
void launch_rownorm_max(const T* x, int64_t n, int64_t l, Red red, hipStream_t st);
// FGD: g = sum(gp slabs) + mu * y / sqrt(||y_i||^2 + delta^2);
// out: [sum (sqrt(||y_i||^2+delta^2) - delta)]
template <typename T>
void launch_fgd_grad(const T* y, const T* gp, int S, T* g, int64_t n, int64_t l, double mu,
                     double delta, Red red, hipStream_t st);
// fh[idx] = 0.5 * s[i_sumsq] + mu * s[i_reg]
void launch_record_f(const double* s, int i_sumsq, int i_reg, double mu, double* fh, int64_t idx,
                     hipStream_t st);
// l = 1 descent pass in one sweep of A (kernels_gemv.hip): Gp[blocks][n] = per-workgroup
// A^T (A xt - b) slabs, red.out[0..1] = sum (A x - b)^2, sum (A xt - b)^2, fh[0] (if non-null)
// = 0.5 out[0] + fh_mu * rn[0]. gemv_fused_blocks() = workgroups to launch, 0 = not applicable.
int gemv_fused_blocks(int esize, int64_t m, int64_t n, int64_t l);
template <typename T>
void launch_gemv_fused(int blocks, const T* A, const T* x, const T* xt, const T* b, T* Gp, int64_t m,
                       int64_t n, double* fh, double fh_mu, const double* rn, Red red,
                       hipStream_t st);
// G[j] = sum_{s<S} Gp[s][j] (slab order, deterministic)
template <typename T>
void launch_sum_cols(const T* Gp, int S, T* G, int64_t n, hipStream_t st);
// host[0..ns) = s[0..ns) except host[off2..off2+n2) = s2[0..n2) when s2 != NULL, then
// *host_seq = seq (system-scope release); host memory is mapped
// the packet of `pub` with its deferred reductions first (pub.host == NULL: the reductions only)
void launch_publish_pub(const Pub& pub, hipStream_t st);
void launch_publish(const double* s, int ns, double* host, unsigned* host_seq, unsigned seq,
                    hipStream_t st, const double* s2 = nullptr, int off2 = 0, int n2 = 0);

}  // namespace glx
