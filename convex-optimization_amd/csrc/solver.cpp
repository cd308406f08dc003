// solver.cpp — the iteration driver behind gl_<method>(x0, A, b, mu_0, opts), native C++.
//
// The reference runs each solver as a Python loop over NumPy calls; here the same control
// flow (continuation over mu in [100 mu0, 10 mu0, mu0], the stability stop rule, Armijo /
// backtracking line searches, step schedules) runs in C++ and drives the HIP kernels on one
// stream. The host reads back a packet of device scalars only where a branch needs them:
// once per line-search trial (ProxGD / FProxGD / FGD) and never for SGD / GD, whose objective
// history is recorded on the device.
//
// Work per iteration (passes over A; reference counts from SURVEY §3):
//   ProxGD  reference 5.7 A@x + 1 A^T r;  here 1 A@[e | p_thr] per trial + 1 A^T r (e: the
//           entries the threshold zeroed, MFMAs on flagged K chunks only)
//           (+1 A@x when the hard threshold changed x, +1 A@x in exact_objective mode)
//   FProxGD reference 4 A@x + 1 A^T r;    here 1 A@y + 1 A@x per trial + 1 A^T r
//   SGD/GD  reference 2 A@x + 1 A^T r;    here 1 A@x (+1 when the threshold changed x) + 1 A^T r
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "glx.h"
#include "glx_comm.h"
#include "glx_internal.h"

namespace glx {

thread_local std::string g_last_error;
thread_local LaunchTiming g_launch_timing;

#define GLX_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) throw Error{GLX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
  } while (0)

static inline void check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw Error{GLX_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e)};
}

// scalar slots in the device scalar array
enum {
  S_TR = 0,     // trial kernel outputs, up to 6 values (0..5)
  S_RT = 6,     // trial-pass finalize: [sum r_src0^2, r_src1^2, r_src2^2, count(candidate)]
  S_RO = 10,    // prologue finalize:   [sum r_x^2, sum r_xt^2, -, count(x)]
  S_XRN = 14,   // sum ||x_i|| of the current iterate   } rownorm_max: [sum, max]
  S_XMAX = 15,  // max |x|
  S_RG = 16,    // standalone residual finalize (FISTA y): [sum r^2, ...]
  S_TRN = 16,   // row-sharded ProxGD: the speculated next trial's sums (6; the FISTA / SGD slots)
  S_REGY = 20,  // FGD smooth regulariser at y
  S_DRN = 21,   // row-norm sum written by the SGD/GD step (+1: max)
  NSCAL = 24,   // the host packet copies slots [0, NSCAL)
  S_SNAP = 24,  // snapshot of S_TR..S_TR+5 taken by a finalize (packet remap, not copied itself)
  S_SPX = 30,   // SGD/GD log sparsity every 100 iterations: [sum ||x_i||, max |x|] of the new x
  NSCAL_DEV = 32
};

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  void* take(size_t bytes) {
    off = (off + 255) & ~size_t(255);
    void* p = base ? base + off : nullptr;
    off += bytes;
    return p;
  }
};

static int method_bufs(int method) {
  switch (method) {
    case GLX_PROXGD: return 7;   // (x, x_thr), (p, p_thr), z + two spares (speculative trial)
    case GLX_FPROXGD: return 9;  // (x_k, v_k, y) current + (x, v, y) of the trial + 3 spares
    case GLX_FGD: return 6;
    default: return 2;           // SGD / GD: x, thr(x)
  }
}
constexpr int kBufs = 9;
constexpr int kTailBytes = 64;   // behind each gradient set: scalars that ride its all-reduce
constexpr int kRes = 4;
constexpr int kDcWindow = 8;     // device-controlled line search: iterations in flight (GLX_DC_BATCH)
constexpr int kKeepMiB = 192;    // Infinity-Cache hand-off between the non-temporal passes
// gradient sets: 2 (current, speculative); with a communicator and device control a ring of
// window + 2, so that the all-reduces queued behind a cancelling decision (they cannot be
// gated) never land in the set the host resumes from
constexpr int kMaxGSets = kCtlMaxBatch / 2 + 2;
// row-sharded ProxGD (iter_proxgd_shard): each rank's chunk of sums that rides the all-gather
// (the finalize's at [6, 10), the trial's workgroup partials from kShardPartOff, ShardPub), for
// up to kMaxShardRanks ranks
constexpr int kShardChunkMax = kShardPartOff + (6 + 4) * kMaxBlocks;
constexpr int kMaxShardRanks = 64;
// round 6: flagged rows from which ProxGD's split-candidate A e takes the fused form (GLX_AE_HYB_ROWS)
constexpr double kHybRows = 2000.0;
// the chunks' doubles: the sums of up to kMaxShardRanks ranks, plus (round 6, sderive_) every rank's
// row masks and column bitmaps of e for its rows (n / 2 + l n / 64 doubles over all ranks)
static int64_t shard_blk_doubles(int64_t n, int64_t l) {
  return (int64_t)kShardChunkMax * kMaxShardRanks + n / 2 + l * n / 64 + 64;
}

// device-controlled batches' window: opts.dc_window (> 0: that window, < 0: off), else
// GLX_DC_BATCH, else the measured default (0 = the host decides every iteration): kDcWindow for
// FProxGD with a communicator, off elsewhere. Same box, 200-step windows, host control against
// window 8 (profiles/r3_dc/): ProxGD NS 2374-2382 vs 2344-2354 it/s, C2 9003-9010 vs 8894-8910,
// the comm-path shards 6922-11023 vs 6735-10612 (its speculative A@X already hides the host's
// turn); FProxGD NS 2454-2478 vs 2456-2465 (whole solve 2058-2060 vs 2036-2038), C3 3702 vs
// 3687-3703, C5's shard 1227-1231 vs 1230-1234, the 1024-row comm shard 9802-9829 vs 10517-10587
// (+7.5 %: the host path leaves the GPU idle while it decides behind the short speculative trial).
// Round 5: also kDcWindow for ProxGD on the unfused speculative form (unfused: Session's
// dc_unfused_ok) when A is at most kDcSmallBytes — launch-bound shapes, where the host's turn per
// iteration is a large share: C1 (512, 1024, 2) 200-step windows 24 250 / 24 253 it/s with host
// control against 25 477 / 25 591 with window 8 (and 22 079 / 21 752 on the rounds-1-4 form;
// profiles/r5_unfused/).
static constexpr double kDcSmallBytes = 64.0 * 1024 * 1024;
static int dc_window_opt(const glx_problem& P, const glx_opts& O, bool unfused = false) {
  int w = (P.method == GLX_FPROXGD && P.comm != nullptr) ? kDcWindow : 0;
  if (unfused && (double)P.m * (double)P.n * 8.0 <= kDcSmallBytes) w = kDcWindow;
  if (O.dc_window != 0) {
    w = O.dc_window;
  } else if (const char* dc = std::getenv("GLX_DC_BATCH")) {
    w = std::atoi(dc);
  }
  return std::max(0, std::min(w, kCtlMaxBatch / 2));
}

static void validate(const glx_problem* P, const glx_opts* O) {
  if (!P || !O) throw Error{GLX_E_INVALID, "null problem/opts"};
  if (P->dtype != GLX_F32 && P->dtype != GLX_F64) throw Error{GLX_E_INVALID, "dtype must be GLX_F32 or GLX_F64"};
  if (P->method < GLX_PROXGD || P->method > GLX_FGD) throw Error{GLX_E_INVALID, "unknown method"};
  if (P->m <= 0 || P->n <= 0 || P->l <= 0) throw Error{GLX_E_INVALID, "m, n, l must be positive"};
  if (P->l > kMaxL) throw Error{GLX_E_INVALID, "l > 128 is not supported"};
  if (!P->A || !P->b || !P->x) throw Error{GLX_E_INVALID, "A, b and x must be device pointers"};
  if (O->step_type < GLX_STEP_LINE_SEARCH || O->step_type > GLX_STEP_DIMINISHING2)
    throw Error{GLX_E_INVALID, "Unsupported step_type"};
  if ((P->method == GLX_SGD || P->method == GLX_GD) && O->step_type == GLX_STEP_LINE_SEARCH)
    throw Error{GLX_E_INVALID, "SGD/GD have no line search (reference logs 'Unsupported type.')"};
  if (O->maxit < 0 || O->ls_maxit < 0) throw Error{GLX_E_INVALID, "negative iteration limit"};
  if ((reinterpret_cast<uintptr_t>(P->A) | reinterpret_cast<uintptr_t>(P->b) |
       reinterpret_cast<uintptr_t>(P->x)) & 15)
    throw Error{GLX_E_INVALID, "A, b, x must be 16-byte aligned"};
}

// ------------------------------------------------------------------------------------------
// The solver's plan: the shape's GEMM plan, plus one method-level choice. fp32 ProxGD/FProxGD
// on one GPU take the 4-wave panel AᵀR with 2 K splits (code 1008) instead of the 4-panel
// tile (1114), so that the line-search trial fuses into it (atr_split_combine): the AᵀR pass
// is ≈13 µs slower but the trial launch and its boundary go. Same box: C3 (8192,16384,32)
// FProxGD 3669–3691 → 3743–3749 it/s, ProxGD 3654–3657 → 3744–3752, FProxGD at (4096,8192,16)
// 11 362–11 366 → 13 200–13 215 (profiles/r1_tuning/small_kernels/atr_f32_fused.log).
// Round 3: with the PF 8 ring (1008) instead of PF 4 the C3 pass reads 5.0 instead of 4.7 TB/s
// (A^T R 106.6–107.1 vs 113–114.5 us), FProxGD 3627–3680 → 3725–3763 it/s over 200 steps;
// S = 1 / 4 and the default load policy measured level or slower (profiles/r3_c3atr/sweep.txt).
// Split-candidate ProxGD (the fast objective mode, see iter_proxgd): 0 = off (exact mode, other
// methods, shapes the gather does not cover, or GLX_SPLIT_CAND=0 / glx_opts.split_cand = 0: the
// dense [z | p_thr] batch of round 1); 1 = A e from the transposed copy of A (kernels_gather.hip;
// costs an extra m x n copy of A in the workspace, glx_session_workspace_bytes).
// ProxGD: fp64 only. In fp32 its regrouped sum (A p_thr - b) + A e IS the recorded objective
// and moves f by ~1e-6 relative on short unconverged runs (measured 1.5e-6 on mid_384x640x16
// against the 1e-6 fp32 bar); no fp32 ProxGD configuration is on the benchmark path.
// FProxGD in fp32 (C3): the objective is A xc computed directly; only A y_next is regrouped.
// Round 4 kept it opt-in because one whole C3 solve ended 3.4e-5 from the reference's fp32 run
// against 3.4e-7 for the dense batch. Round 5 measured the band (scripts/c3_band.py,
// profiles/r5_d/c3_band.jsonl): eleven summation orders of the two forms (K splits, tiles, A e
// forms) end 3.4e-7 .. 8.7e-5 (dense) and 1.6e-5 .. 8.9e-5 (split) from the reference's fp32
// objective, all 7.0e-3 .. 7.1e-3 from its fp64 one (the reference's own fp32 run: 7.0e-3).
// Round 6: the dense batch is the fp32 default again — its default order ends
// 3.4e-7 from the reference's fp32 run, inside the 1e-6 fp32 bar, the split form's 1.6e-5 does
// not, and whole solves run level (3897 it/s both: late in a solve e_c fills and the budget runs
// dense batches; only 200-step windows gain, +17 %). GLX_SPLIT_F32=1: the split form (opt-in).
// (The size gate counts elements as fp64.)
// FProxGD with line search takes the gather form too (iter_fista: A y_next by linearity from
// A xc, A e_c and the kept A thr(x_k)); GLX_SPLIT_FISTA=0 keeps its dense [xc | y_next] batch.
// Only for A of at least kSplitMinBytes (this rank's rows): the column lists and the gather
// carry a fixed ~70 + 50 us that a short dense pass cannot hide. Measured against the dense
// batch (profiles/r2_splitgate/): NS (1 GiB) 2295 vs 2080 it/s, (4096,16384,32) 3894 vs 3832,
// but C2 (4096,8192,16) 7329 vs 8948 and the comm-path shards of 4096 / 2048 / 1024 rows
// 3543 / 6756 / 9748 vs 3623 / 6884 / 11162. GLX_SPLIT_CAND=1 forces it at any size (tests).
// Round 5 (the bitmap gather: no lists kernel, ~5 us fixed): ProxGD at l = 32 takes it from
// 64 MiB of A on this rank. Measured against the dense batch (profiles/r5_e/, profiles/r5_f/;
// 200-step windows / whole solves): (4096, 16384, 32) 4844 / 4894 vs 3987 / 4069 it/s; the
// communicator-path shards of 1024 / 2048 / 4096 rows 12114 / 8016 / 4759 vs 11122 / 6931 / 3915
// (whole solves at 1024 / 4096 rows 12082 / 4848 vs 11226 / 4015). C2 (l = 16, A in the Infinity
// Cache, where At would evict it) stays dense: 8411 / 8205 vs 9127 / 9151; FProxGD's shards too
// (whole solves 10480 / 3943 vs 10847 / 4000: e_c fills late in a solve).
static constexpr double kSplitMinBytesL32 = 64.0 * 1024 * 1024;
static constexpr double kSplitMinBytes = 768.0 * 1024 * 1024;
// Round 6: row-sharded FProxGD (iter_fista_shard) — the gradient
// reduce-scattered, k_fista_trial on this rank's n / G rows, xc's rows all-gathered and v_next,
// y_next re-derived from it on every rank (k_fista_split). Returns G where it applies, else 0.
// opts.shard_rows (GLX_SHARD_ROWS): 1 on (needs n % G == 0), 2 off, 0 auto: on where this rank's
// A is below kFistaShardMaxBytes and no device-control window is asked for. Host control only:
// the device-controlled FISTA batch (fista_dc_run) decides from all-reduced gradient tails; the
// sharded form would need its decision behind the all-gather, one more collective per queued
// iteration, so big shards (C5: 2 GiB per rank, where the replicated row work is ~2 % of an
// iteration) keep the all-reduce schedule with device control.
static constexpr double kFistaShardMaxBytes = 768.0 * 1024 * 1024;
static int shard_rows_opt(const glx_opts& O) {
  int want = O.shard_rows;
  if (const char* e = std::getenv("GLX_SHARD_ROWS")) {
    want = std::atoi(e);
    if (want < 0 || want > 2) throw Error{GLX_E_INVALID, "GLX_SHARD_ROWS must be 0 (auto), 1 (on) or 2 (off)"};
  }
  return want;
}
static int fista_shard_ranks(const glx_problem& P, const glx_opts& O) {
  if (P.comm == nullptr || P.method != GLX_FPROXGD) return 0;
  if (O.step_type != GLX_STEP_LINE_SEARCH && O.step_type != GLX_STEP_FIXED) return 0;
  const int want = shard_rows_opt(O);
  if (want == 2) return 0;
  const glx_comm* c = static_cast<const glx_comm*>(P.comm);
  const int vr = comm_size(c) == 1 ? std::max(1, O.shard_model) : comm_size(c);
  if (vr <= 1) return 0;
  const bool fits = vr <= 64 && P.n % vr == 0;
  if (want == 1 && !fits)
    throw Error{GLX_E_INVALID, "row-sharded FProxGD needs n % ranks == 0 and at most 64 ranks "
                               "(opts.shard_rows = 0 / 2: the all-reduce schedule)"};
  if (!fits) return 0;
  if (want == 0 && ((double)P.m * (double)P.n * 8.0 >= kFistaShardMaxBytes || O.dc_window > 0)) return 0;
  return vr;
}

static int split_mode(const glx_problem& P, const glx_opts& O) {
  if (O.exact_objective != 0) return 0;
  if (P.method != GLX_PROXGD && P.method != GLX_FPROXGD) return 0;
  if (P.dtype != GLX_F64) {   // fp32: FProxGD only, opt-in (GLX_SPLIT_F32=1, above)
    const char* f = std::getenv("GLX_SPLIT_F32");
    if (P.method != GLX_FPROXGD || !(f && std::strcmp(f, "1") == 0)) return 0;
  }
  if (O.split_cand == 2) return 0;
  const char* sc = O.split_cand == 0 ? std::getenv("GLX_SPLIT_CAND") : nullptr;
  if (sc && std::strcmp(sc, "0") == 0) return 0;
  const bool force = O.split_cand == 1 || (sc && std::strcmp(sc, "1") == 0);
  const double gate = (P.method == GLX_PROXGD && P.l == 32) ? kSplitMinBytesL32 : kSplitMinBytes;
  if (!force && (double)P.m * (double)P.n * 8.0 < gate) return 0;
  if (P.method == GLX_FPROXGD) {
    if (fista_shard_ranks(P, O) > 0) return 0;   // the row-sharded FISTA runs the dense batch
    const char* sf = std::getenv("GLX_SPLIT_FISTA");
    if (sf && std::strcmp(sf, "0") == 0) return 0;
    const bool ls = O.step_type == GLX_STEP_LINE_SEARCH && O.ls_maxit > 0;
    return (ls && gather_ok(P.n, P.l)) ? 1 : 0;
  }
  return gather_ok(P.n, P.l) ? 1 : 0;
}

// Round 6: ProxGD's split-candidate trial with A e fused into the dense pass (launch_ax_egat,
// kernels_axdma.hip: A p on MFMA, A e on VALU from the same LDS chunks; no transposed copy of A,
// no gather launch) where the session's one-source pass is the f64 LDS-DMA tile 92278 (NS).
// Opt-in (GLX_AE_FUSED=1): same box, 200-step windows / whole solves (profiles/r6_egat/): NS
// 2 452-2 467 / 2 461-2 467 it/s fused against 2 454-2 470 / 2 427-2 434 with the gather — level
// in the window, +1.5 % over a solve (the gather grows late in a solve), but the fused pass runs
// 210-218 µs against 174-176 µs: its A e (VALU, after the chunk's MFMAs) leaves the MFMA pipe of
// both waves of a SIMD idle. Interleaving it into the MFMA stream (straight-line, or on opposite
// sides of the two waves' MFMAs) spilled 16-208 VGPRs at 256. Throughout a solve it stays opt-in
// (it also halves the session's workspace: no m x n copy of A); by default the session takes it
// per trial once many rows are flagged (hyb_rows_, below).
static bool egat_mode(const glx_problem& P, const GemmPlan& plan, int smode) {
  if (smode != 1 || P.method != GLX_PROXGD || P.dtype != GLX_F64) return false;
  if (gather_form() >= 0) return false;
  const char* e = std::getenv("GLX_AE_FUSED");
  if (!(e && std::strcmp(e, "1") == 0)) return false;
  return ax_egat_ok(plan, 8);
}

static GemmPlan session_plan(const glx_problem& P, const glx_opts& O) {
  const int es = P.dtype == GLX_F64 ? 8 : 4;
  GemmPlan p = make_plan(es, P.m, P.n, P.l, O.ax_variant);
  const bool trial_method = (P.method == GLX_PROXGD || P.method == GLX_FPROXGD) &&
                            (O.step_type == GLX_STEP_LINE_SEARCH || O.step_type == GLX_STEP_FIXED);
  if (es == 4 && P.comm == nullptr && trial_method && p.atr_kind == 1 &&
      (P.l == 16 || P.l == 32) && P.n % 64 == 0 && P.m >= 128 && (P.n / 64) * 2 < kMaxBlocks &&
      !std::getenv("GLX_ATR_VARIANT") && !std::getenv("GLX_ATR_S") &&
      !std::getenv("GLX_FUSED_TRIAL")) {
    GemmPlan f = p;
    f.atr_wl = 0;
    f.atr_ntl = 1;
    f.atr_pf = 8;   // round 3: the PF 8 ring (1008), see above
    f.atr_S = 2;
    // Round 4: with at least one panel per CU, the eight-wave panel (WL 2: two waves per SIMD)
    // with one K split, no slab combine: C3 FProxGD A^T R + trial 101.2-101.4 us against
    // 107.4-107.6, 3815-3825 against 3741-3748 it/s over 200 steps (profiles/r4_c3atr/; with
    // two K splits it measured 119 us, with the PF 4 ring 104 us)
    if (P.n / 64 >= 256) {
      f.atr_wl = 2;
      f.atr_S = 1;
      // (round 6: a sixteen-step ring, twice the A bytes in flight per wave, measured slower:
      // A^T R + trial 120.9 against 101.3 us at C3, 3 628 against 3 862 it/s, profiles/r6_egat/)
    }
    if (atr_prox_ok(f)) return f;   // only where the trial actually fuses (GLX_ATR_FUSE_SPLIT)
  }
  // Round 5: fp64 with fewer than 256 64-column panels (C2: 128, planned as 2 K splits) takes
  // the 32-column panel without K splits (WL 3): 256+ workgroups and no slab combine in front of
  // the fused trial. GLX_ATR_NARROW=0: off. (Its eight-wave form, WL 4, measured slower and is no
  // longer built, round 6.)
  if (es == 8 && P.comm == nullptr && trial_method && p.atr_kind == 1 && (P.l == 16 || P.l == 32) &&
      P.n % 32 == 0 && P.n / 64 < 256 && P.n / 32 >= 256 && !std::getenv("GLX_ATR_VARIANT") &&
      !std::getenv("GLX_ATR_S") && !std::getenv("GLX_FUSED_TRIAL")) {
    const char* nw = std::getenv("GLX_ATR_NARROW");
    if (!(nw && std::strcmp(nw, "0") == 0)) {
      GemmPlan f = p;
      f.atr_wl = 3;
      f.atr_pf = 8;
      f.atr_S = 1;
      if (atr_prox_ok(f)) return f;
    }
  }
  return p;
}

class SessionBase {
 public:
  virtual ~SessionBase() {}
  virtual void run(int64_t max_steps, int64_t* done, int32_t* finished) = 0;
  virtual void finish(glx_result* res) = 0;
  virtual void kernel_time(int kind, int64_t* launches, double* ms) = 0;
  virtual void counters(int64_t out[4]) const = 0;
  // thread-safe progress record (a watchdog thread reads it while run() is in progress)
  virtual void progress(int64_t out[4]) const = 0;
  virtual void trace(double* sp_after, int64_t cap, int64_t* n, int64_t phase_info[6]) const = 0;
  virtual std::string describe() const = 0;
  virtual int64_t split_trace(double* out, int64_t cap) const = 0;
};

template <typename T>
class Session : public SessionBase {
 public:
  // workspace layout; with ws == nullptr only computes the size
  static size_t carve(const glx_problem& P, const glx_opts& O, const GemmPlan& plan, int64_t fh_cap,
                      int smode, void* ws, Session* s) {
    Carver c(ws);
    const int64_t nl = P.n * P.l, ml = P.m * P.l;
    const int nb = method_bufs(P.method);
    T* bufs[kBufs] = {static_cast<T*>(P.x)};
    for (int i = 1; i < nb; ++i) bufs[i] = static_cast<T*>(c.take(sizeof(T) * nl));
    T* res[kRes];
    for (int i = 0; i < kRes; ++i) res[i] = static_cast<T*>(c.take(sizeof(T) * ml));
    // gradient sets (G, its split-K slabs): the current one and the speculative one (a ring with
    // a communicator and device control, gsets_for)
    const int ngs = gsets_for(P, O, plan);
    T* g[kMaxGSets];
    T* gp[kMaxGSets];
    for (int k = 0; k < ngs; ++k) {
      g[k] = static_cast<T*>(c.take(sizeof(T) * nl + kTailBytes));   // + scalar tail (comm)
      gp[k] = plan.atr_S > 1 ? static_cast<T*>(c.take(sizeof(T) * nl * plan.atr_S)) : g[k];
    }
    // A@X slabs of up to 3 batched sources; split-candidate gather: the A e slabs + A p_thr's
    const int64_t pslabs = std::max<int64_t>((int64_t)ax_split_max(plan) * 3,
                                             smode == 1 ? gather_split(P.m, P.n) + ax_split(plan, 1) : 0);
    T* pp = static_cast<T*>(c.take(sizeof(T) * ml * pslabs));
    const bool eg = egat_mode(P, plan, smode);
    T* at = (smode == 1 && !eg) ? static_cast<T*>(c.take(sizeof(T) * P.m * P.n)) : nullptr;   // A^T
    void* glists = smode == 1 ? c.take(gather_lists_bytes(P.n)) : nullptr;
    // split-candidate FISTA: e_c and a ring of three A thr(x) (x_k's, the trial's, the
    // speculated next trial's)
    const bool fsp = smode == 1 && P.method == GLX_FPROXGD;
    T* ec = fsp ? static_cast<T*>(c.take(sizeof(T) * nl)) : nullptr;
    T* sxo[3] = {nullptr, nullptr, nullptr};
    for (int k = 0; k < 3 && fsp; ++k) sxo[k] = static_cast<T*>(c.take(sizeof(T) * ml));
    double* scal = static_cast<double*>(c.take(sizeof(double) * NSCAL_DEV));
    double* part = static_cast<double*>(c.take(sizeof(double) * kMaxRedVals * kMaxBlocks));
    unsigned* ticket = static_cast<unsigned*>(c.take(kTicketBytes));
    // per-panel arrival counters of the fused A^T R with K splits (atr_split_combine)
    unsigned* pcnt = static_cast<unsigned*>(c.take(sizeof(unsigned) * (P.n / 64 + 64)));
    int* flag = static_cast<int*>(c.take(256));
    // device-controlled batches: Ctl::state (4 doubles) and the abort word; decision records
    double* dcs = static_cast<double*>(c.take(256));
    double* dcr = static_cast<double*>(c.take(sizeof(double) * kCtlRec * kCtlMaxBatch));
    // split-candidate mode: per-row column masks of e = p - p_thr (z's buffer; bit c = e[k][c] != 0)
    unsigned* zf = static_cast<unsigned*>(c.take(zf_bytes(P.n)));   // + the column bitmaps
    // deferred reductions (defer_): two trial partial buffers (the kernel that reduces one may run
    // beside the next trial writing the other) and the finalize's
    double* tpart = static_cast<double*>(c.take(sizeof(double) * 2 * 6 * kMaxBlocks));
    double* fpart = static_cast<double*>(c.take(sizeof(double) * 4 * kMaxBlocks));
    double* sblk = P.comm != nullptr && (P.method == GLX_PROXGD || P.method == GLX_FPROXGD)
                       ? static_cast<double*>(c.take(sizeof(double) * shard_blk_doubles(P.n, P.l)))
                       : nullptr;
    double* fh = static_cast<double*>(c.take(sizeof(double) * (fh_cap + 1)));
    double* sp100 = static_cast<double*>(c.take(sizeof(double) * (fh_cap / 100 + 2)));
    const int gb = gemv_blocks_for(P);
    T* gs = gb > 0 ? static_cast<T*>(c.take(sizeof(T) * nl * gb)) : nullptr;   // fused l = 1 slabs
    if (s) {
      for (int i = 0; i < kBufs; ++i) s->X_[i] = bufs[i];
      for (int i = 0; i < kRes; ++i) s->R_[i] = res[i];
      for (int k = 0; k < ngs; ++k) { s->Gs_[k] = g[k]; s->Gps_[k] = gp[k]; }
      s->nsets_ = ngs;
      s->G_ = g[0]; s->Gp_ = gp[0]; s->Pp_ = pp; s->At_ = at; s->glists_ = glists;
      s->scal_ = scal; s->part_ = part; s->ticket_ = ticket; s->flag_ = flag; s->fh_dev_ = fh;
      s->pcnt_ = pcnt;
      s->dc_state_ = dcs;
      s->dc_abort_ = reinterpret_cast<int*>(dcs + 8);
      s->dc_rec_ = dcr;
      s->zf_ = zf;
      s->blk_ = sblk;
      s->tpart_[0] = tpart;
      s->tpart_[1] = tpart + 6 * kMaxBlocks;
      s->fpart_ = fpart;
      s->E_ = ec;
      for (int k = 0; k < 3; ++k) s->SXO_[k] = sxo[k];
      s->sp100_ = sp100;
      s->gemv_slabs_ = gs;
      s->gemv_blocks_ = gb;
    }
    return c.off + 256;
  }

  // SGD / GD with l = 1: the descent pass reads A once (kernels_gemv.hip); GLX_GEMV_FUSED=0
  // selects the two-pass path (A @ [x | thr(x)], then A^T r)
  static int gemv_blocks_for(const glx_problem& P) {
    if (P.method != GLX_SGD && P.method != GLX_GD) return 0;
    const char* e = std::getenv("GLX_GEMV_FUSED");
    if (e && std::strcmp(e, "0") == 0) return 0;
    return gemv_fused_blocks((int)sizeof(T), P.m, P.n, P.l);
  }

  // Round 5: ProxGD on one GPU whose plan cannot fuse the trial into A^T r (l not in {16, 32},
  // n % 64 != 0, ...; C1's (512, 1024, 2)) runs the communicator path's form instead: A^T r, then
  // k_prox_pgd from its slabs, queued speculatively the same way (the packet riding k_prox_pgd),
  // so device control (dc_queue_comm) applies to these shapes too. GLX_UNFUSED_SPEC=0: off (the
  // gradient and the trial as separate host-driven steps, rounds 1-4).
  static bool unfused_spec_ok(const glx_problem& P, const glx_opts& O, const GemmPlan& plan) {
    const char* e = std::getenv("GLX_UNFUSED_SPEC");
    const char* fz = std::getenv("GLX_FUSED_TRIAL");
    return P.comm == nullptr && P.method == GLX_PROXGD && !atr_prox_ok(plan) &&
           (O.step_type == GLX_STEP_LINE_SEARCH || O.step_type == GLX_STEP_FIXED) &&
           !(e && std::strcmp(e, "0") == 0) && !(fz && std::strcmp(fz, "0") == 0);
  }
  // device control on that form: as with a communicator (fp64: the finalize's sums go to the
  // gradient set's tail, read as doubles), line search, fast objective mode
  static bool dc_unfused_ok(const glx_problem& P, const glx_opts& O, const GemmPlan& plan) {
    return unfused_spec_ok(P, O, plan) && P.dtype == GLX_F64 && O.step_type == GLX_STEP_LINE_SEARCH &&
           O.ls_maxit > 0 && O.exact_objective == 0;
  }
  // device control with a communicator: ProxGD, fp64 (the trial sums ride the gradient
  // all-reduce), line search, fast objective mode
  static bool dc_comm_ok(const glx_problem& P, const glx_opts& O) {
    return P.comm != nullptr && (P.method == GLX_PROXGD || P.method == GLX_FPROXGD) && P.dtype == GLX_F64 &&
           O.step_type == GLX_STEP_LINE_SEARCH && O.ls_maxit > 0 && O.exact_objective == 0;
  }
  static bool env_is(const char* name, const char* v) {
    const char* e = std::getenv(name);
    return e && std::strcmp(e, v) == 0;
  }
  // the device-control window that takes effect for this plan: the requested one
  // (dc_window_opt) where the fused speculative path, the spinning readback and, with a
  // communicator, the attached packet are all on; else 0 (the host decides)
  static int dc_window_eff(const glx_problem& P, const glx_opts& O, const GemmPlan& plan) {
    if (fista_shard_ranks(P, O) > 0) return 0;   // row-sharded FProxGD: host control
    const bool ls = O.step_type == GLX_STEP_LINE_SEARCH && O.ls_maxit > 0;
    const bool spin = !env_is("GLX_READBACK", "sync");
    const bool attach = spin && !env_is("GLX_ATTACH_PUB", "0");
    const bool fuse_any = (P.comm != nullptr || atr_prox_ok(plan)) &&
                          (O.step_type == GLX_STEP_LINE_SEARCH || O.step_type == GLX_STEP_FIXED) &&
                          !env_is("GLX_FUSED_TRIAL", "0");
    const bool method = P.method == GLX_PROXGD || P.method == GLX_FPROXGD;
    const bool unf = dc_unfused_ok(P, O, plan) && attach;
    if (!((fuse_any || unf) && method && spin && O.exact_objective == 0 && ls &&
          (P.comm == nullptr || (dc_comm_ok(P, O) && attach))))
      return 0;
    return dc_window_opt(P, O, unf && P.comm == nullptr);
  }
  // a ring of window + 2 gradient sets only where device control with a communicator actually
  // runs (it was sized on the request, not on the window that takes effect)
  static int gsets_for(const glx_problem& P, const glx_opts& O, const GemmPlan& plan) {
    const int w = dc_window_eff(P, O, plan);
    return (w > 0 && (dc_comm_ok(P, O) || dc_unfused_ok(P, O, plan))) ? w + 2 : 2;
  }

  static int64_t fh_capacity(const glx_problem& P, const glx_opts& O) {
    int64_t cap = 3 * (int64_t)O.maxit;
    if (O.max_total_iters > 0) cap = std::min<int64_t>(cap, O.max_total_iters);
    return cap;
  }

  Session(const glx_problem& P, const glx_opts& O, void* ws, size_t ws_bytes, hipStream_t st)
      : P_(P), O_(O), st_(st) {
    m_ = P.m; n_ = P.n; l_ = P.l;
    nl_ = n_ * l_; ml_ = m_ * l_;
    plan_ = session_plan(P, O);
    {   // Infinity-Cache hand-off between the two non-temporal passes: the last ~192 MiB each
        // pass reads stay in the 256 MiB Infinity Cache for the other pass. NS, same box, two
        // interleaved rounds: 2307 / 2318 it/s against 2252 / 2272 with both off, either alone
        // in between (profiles/r3_keep/). GLX_AX_KEEP_MIB / GLX_ATR_KEEP_MIB = 0: off. Kernel
        // arguments through the plan, so every session and device has its own value.
      const char* ka = std::getenv("GLX_AX_KEEP_MIB");
      const char* kr = std::getenv("GLX_ATR_KEEP_MIB");
      plan_.ax_keep_mib = std::max(0, ka ? std::atoi(ka) : kKeepMiB);
      plan_.atr_keep_mib = std::max(0, kr ? std::atoi(kr) : kKeepMiB);
    }
    comm_ = static_cast<glx_comm*>(P.comm);
    fh_cap_ = fh_capacity(P, O);
    smode_ = split_mode(P, O);
    const size_t need = carve(P, O, plan_, fh_cap_, smode_, nullptr, nullptr);
    if (!ws || ws_bytes < need) throw Error{GLX_E_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes"};
    if (reinterpret_cast<uintptr_t>(ws) & 255) throw Error{GLX_E_WORKSPACE, "workspace must be 256-byte aligned"};
    carve(P, O, plan_, fh_cap_, smode_, ws, this);
    A_ = static_cast<const T*>(P.A);
    B_ = static_cast<const T*>(P.b);
    // scalar packet: host-mapped, coherent memory the GPU writes directly (k_publish)
    GLX_HIP(hipHostMalloc(reinterpret_cast<void**>(&hs_), sizeof(double) * 32,
                          hipHostMallocMapped | hipHostMallocCoherent));
    hseq_ = reinterpret_cast<unsigned*>(hs_ + NSCAL + 2);
    *hseq_ = 0;
    GLX_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&hs_dev_), hs_, 0));
    hseq_dev_ = reinterpret_cast<unsigned*>(hs_dev_ + NSCAL + 2);
    const char* rb = std::getenv("GLX_READBACK");
    spin_readback_ = !(rb && std::strcmp(rb, "sync") == 0);
    // the scalar packet rides the speculative kernel queued right behind it (one extra
    // workgroup, publisher_first) instead of a k_publish launch in front of it
    const char* ap = std::getenv("GLX_ATTACH_PUB");
    attach_ok_ = spin_readback_ && !(ap && std::strcmp(ap, "0") == 0);
    const char* sp = std::getenv("GLX_SPEC_GRAD");
    spec_off_env_ = (sp && std::strcmp(sp, "0") == 0);
    const char* sa = std::getenv("GLX_SPEC_AX_PUB");
    spec_ax_pub_ = !(sa && std::strcmp(sa, "0") == 0);
    const char* fz = std::getenv("GLX_FUSED_TRIAL");
    // With a communicator the trial cannot live in the A^T r epilogue (the gradient is summed
    // over ranks first): it runs as A^T r, all-reduce, then k_prox_pgd / k_fista_trial, and is
    // queued speculatively the same way (see atr_prox).
    const bool fuse_any = (comm_ != nullptr || atr_prox_ok(plan_)) &&
                          (O.step_type == GLX_STEP_LINE_SEARCH || O.step_type == GLX_STEP_FIXED) &&
                          !(fz && std::strcmp(fz, "0") == 0);
    unfused_spec_ = unfused_spec_ok(P, O, plan_);
    fused_ok_ = (fuse_any || unfused_spec_) && P.method == GLX_PROXGD;
    // ProxGD's fast objective mode evaluates the candidate as A p = A p_thr + A e, e = p - p_thr
    // nonzero only where the hard threshold zeroed p (see iter_proxgd, split_mode)
    emode_ = smode_ != 0 && P.method == GLX_PROXGD;
    fsplit_ = smode_ == 1 && P.method == GLX_FPROXGD;
    // A e form (round 5, scripts/ec_distribution.py over whole NS solves, profiles/r5_c/): ProxGD's
    // e has ~1.1 nonzeros per flagged row (27 % of the rows), so the VALU bitmap gather does 1/30
    // of the row form's MFMA work (whole solve 2206 against 2128 it/s for the row form, 2185 for
    // the round-4 lists); FProxGD's e_c reaches 96 % of the rows with ~7.5 nonzeros each late in
    // a solve, where the row form reads every flagged At row once (whole solves 2131-2143 against
    // 2114-2121 bitmap, 2122-2124 lists).
    gform_ = gather_form();
    if (gform_ < 0) gform_ = P.method == GLX_FPROXGD ? 1 : 0;
    if (gform_ == 1 && !gather_rows_ok(m_, n_)) gform_ = 0;
    rows_form_ = gform_ == 1;
    gsplit_ = rows_form_ ? gather_split(m_, n_) : 1;
    egat_ = egat_mode(P, plan_, smode_);
    if (egat_) gsplit_ = ax_split(plan_, 1);   // the A e slabs: one per K split of the dense pass
    {   // the VALU gather's budget counts nonzeros of e_c, the row form's flagged rows (round 5)
      const char* nb = std::getenv("GLX_SPLIT_NNZ");
      nnz_budget_ = (nb ? std::atof(nb) : (rows_form_ ? kRowsBudget : 0.35)) * (double)n_;
    }
    if (smode_ == 1 && !egat_) {
      launch_transpose<T>(static_cast<const T*>(P.A), At_, m_, n_, st_);   // once
    }
    fused_fista_ok_ = fuse_any && P.method == GLX_FPROXGD;
    // (Round 5's folded finalize — the split-candidate trial's finalize inside its dense pass,
    // GLX_AX_FIN=1 — measured slower, 2376 against 2537-2543 it/s at NS, and was removed in round 6;
    // DESIGN.md keeps the numbers.)
    // device-controlled batches (dc_run / fista_dc_run): ProxGD / FProxGD with line search on
    // the fused speculative path; GLX_DC_BATCH = iterations in flight (0: the host decides every
    // iteration). With a communicator fp64 only (the trial sums ride the gradient all-reduce).
    dc_window_ = dc_window_eff(P, O, plan_);
    if (dc_window_ > 0 && !((fused_ok_ || fused_fista_ok_) && spin_readback_ && (comm_ == nullptr || attach_ok_)))
      throw Error{GLX_E_STATE, "device-control window and the session's fused path disagree"};
    if (dc_window_ > 0) {
      GLX_HIP(hipHostMalloc(reinterpret_cast<void**>(&dc_ring_), sizeof(double) * kCtlRec * kCtlMaxBatch,
                            hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(dc_ring_, 0, sizeof(double) * kCtlRec * kCtlMaxBatch);   // tags start at 1
      GLX_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dc_ring_dev_), dc_ring_, 0));
    }
    // Row-sharded ProxGD (round 5, iter_proxgd_shard): with a communicator of G > 1 ranks the
    // gradient is reduce-scattered, the trial runs on this rank's n / G rows and p's rows are
    // all-gathered (opts.shard_rows: 0 auto = on where n % G == 0, 1 on, 2 off; GLX_SHARD_ROWS,
    // same codes, overrides). Host control only (a device-control window keeps the all-reduce
    // schedule). opts.shard_model = G at world size 1 (bench.py --shard-model, with --force-comm):
    // the per-rank timing model of G ranks — the trial on n / G rows, every line-search test
    // accepted — whose iterates are NOT a solve (glx_solve refuses it; ADVICE round 5: no
    // environment variable turns it on inside the library).
    if (comm_ != nullptr && P.method == GLX_FPROXGD) {
      const int fr = fista_shard_ranks(P, O);
      cranks_ = comm_size(comm_);
      if (fr > 0) {
        shard_ = true;
        fshard_ = true;
        shard_model_ = cranks_ == 1;
        sranks_ = fr;
        srank_ = shard_model_ ? 0 : comm_rank(comm_);
        srows_ = n_ / fr;
        srow0_ = (int64_t)srank_ * srows_;
        nbp_ = prox_blocks(srows_, l_);   // k_fista_trial's grid is k_prox_pgd's
        nbf_ = finalize_blocks(ml_, ax_split(plan_, 2), 0, srows_ * l_);
        stv_ = 4;
        schunk_ = kShardPartOff + stv_ * nbp_ + 4 * nbf_;
      }
    }
    if (comm_ != nullptr && P.method == GLX_PROXGD && dc_window_ == 0) {
      const int want = shard_rows_opt(O);
      cranks_ = comm_size(comm_);
      int vr = cranks_;
      if (cranks_ == 1) {
        vr = std::max(1, O.shard_model);
        shard_model_ = vr > 1;
      }
      const bool fits = vr <= kMaxShardRanks && n_ % vr == 0;
      if (want == 1 && vr > 1 && !fits)
        throw Error{GLX_E_INVALID, "row-sharded ProxGD needs n % ranks == 0 and at most 64 ranks "
                                   "(opts.shard_rows = 0 / 2: the all-reduce schedule)"};
      if (want != 2 && vr > 1 && fits) {   // auto: the all-reduce schedule where it does not fit
        shard_ = true;
        sranks_ = vr;
        srank_ = shard_model_ ? 0 : comm_rank(comm_);
        srows_ = n_ / vr;
        srow0_ = (int64_t)srank_ * srows_;
        nbp_ = prox_blocks(srows_, l_);
        // the trial finalize's workgroups (its sources: 2 in the split / dense modes, 3 exact)
        const int fsrc = O.exact_objective != 0 ? 3 : 2;
        nbf_ = finalize_blocks(ml_, emode_ && smode_ == 1 ? ax_split(plan_, 1) : ax_split(plan_, fsrc),
                               emode_ && smode_ == 1 ? gsplit_ : 0, srows_ * l_);
        schunk_ = kShardPartOff + stv_ * nbp_ + 4 * nbf_;
        // A e from the bitmap / list gathers reads e only where its masks are set, where e = p:
        // the gathered p serves as e and z is not re-derived (the row form reads whole rows)
        zskip_ = emode_ && gform_ != 1;
        // Round 6: that derive (k_trial_split) fused into the next trial's dense pass where the
        // plan's one-source tile takes it (k_ax_lds DRV: the 8-wave shard tile, f64, l = 32) and
        // the packet rides the pass (iter_proxgd_shard's speculative step). GLX_SHARD_DERIVE=0: off.
        // With it the A e gather (AxDerive: extra workgroups of that pass): k_prox_pgd writes the
        // masks and bitmaps of its rows into the rank's sums chunk (behind the partials, moff_),
        // all-gathered with them, so the gather needs nothing the pass writes.
        sderive_ = zskip_ && smode_ == 1 && !egat_ && gform_ == 0 && ax_derive_ok(plan_, (int)sizeof(T)) &&
                   n_ % 64 == 0 && srows_ % 64 == 0 && n_ <= 65536 && !env_is("GLX_SHARD_DERIVE", "0");
        moff_ = schunk_;
        if (sderive_) schunk_ += srows_ / 2 + l_ * srows_ / 64;
      } else {
        shard_model_ = false;
      }
    }
    // Round 5, deferred reductions (single GPU, host control, ProxGD): the fused trial (k_atr_prox)
    // and the residual finalize leave their sums as workgroup partials (Red::parts_only) instead
    // of running the grid reduction's serial tail (two arrival counters, the last workgroup's
    // loads: ~3 us at the end of each kernel); the workgroup that publishes the next packet
    // reduces them first (Pub::dpart, defer_reduce), and the finalize takes max |p| from the
    // trial's partials itself. GLX_DEFER_RED=0: off.
    // Only where the packet that follows is carried by the next speculative kernel (carry_): a
    // standalone k_publish_pub that reduces them and then writes the packet measured 17-19 us
    // against 4 us for k_publish (profiles/r5_probe/), so the non-speculative paths keep the
    // in-kernel reduction.
    // ProxGD only: FProxGD's k_atr_fista measured no gain (NS FProxGD 2583 / 2582, C3 4527 / 4535
    // it/s over 200 steps, profiles/r5_defer3/) and lost 8 % on the rejection-heavy probe
    // (its publisher's reduction stretched the 33 us fused kernel by ~4 us); that opt-in form
    // (GLX_DEFER_RED=2) was removed in round 6.
    const bool dmeth = P.method == GLX_PROXGD;
    // Round 6: ProxGD's split-candidate A e chosen per trial on one GPU under host control: the
    // bitmap gather while few rows are flagged (its cost grows with them: 12 us at ~570 rows,
    // ~50 us averaged over a solve), A e fused into the dense pass (launch_ax_egat, a near-constant
    // extra) once the last accepted trial flagged at least hyb_rows_ rows. NS whole solves 2 538-
    // 2 541 it/s at 1 500-2 500 rows against 2 463-2 465 with the gather throughout, the 20-step
    // window unchanged (profiles/r6_hyb/). GLX_AE_HYB_ROWS: the threshold, 0 = off (the gather
    // throughout); GLX_AE_FUSED=1 keeps the fused form throughout.
    if (smode_ == 1 && !egat_ && gform_ == 0 && comm_ == nullptr && dc_window_ == 0 &&
        P.method == GLX_PROXGD && P.dtype == GLX_F64 && ax_egat_ok(plan_, 8)) {
      const char* e = std::getenv("GLX_AE_HYB_ROWS");
      hyb_rows_ = e ? std::atof(e) : kHybRows;
    }
    defer_ = comm_ == nullptr && dc_window_ == 0 && dmeth && spin_readback_ && attach_ok_ &&
             !env_is("GLX_DEFER_RED", "0");
    GLX_HIP(hipMemsetAsync(ticket_, 0, kTicketBytes, st_));
    GLX_HIP(hipMemsetAsync(pcnt_, 0, sizeof(unsigned) * (P.n / 64 + 64), st_));
    GLX_HIP(hipMemsetAsync(flag_, 0, 256, st_));
    GLX_HIP(hipMemsetAsync(scal_, 0, sizeof(double) * NSCAL_DEV, st_));
    // the column bitmaps' words no trial visits (rows in [ceil16(n), ceil64(n)), the upper half
    // of a narrow panel's last u64) must read as 0 (glx_device.h zf_bitmaps)
    GLX_HIP(hipMemsetAsync(zf_, 0, zf_bytes(P.n), st_));
    if (blk_) GLX_HIP(hipMemsetAsync(blk_, 0, sizeof(double) * shard_blk_doubles(n_, l_), st_));
    mus_[0] = 100 * P.mu0;
    mus_[1] = 10 * P.mu0;
    mus_[2] = P.mu0;
    mu_ = mus_[0];
    fbest_ = INFINITY;
    tk_ = O.alpha0;
    method_ = P.method;
    use_sparsity_ = (method_ == GLX_PROXGD || method_ == GLX_FPROXGD || method_ == GLX_FGD);
    device_hist_ = (method_ == GLX_SGD || method_ == GLX_GD);
    if (method_ == GLX_FPROXGD || method_ == GLX_FGD) copy_x(iv_, ix_);  // v_k = copy(x_k)
    phase_start_[0] = 0;
  }

  ~Session() override {
    if (hs_) (void)hipHostFree(hs_);
    if (dc_ring_) (void)hipHostFree(dc_ring_);
    if (rb_event_) (void)hipEventDestroy(rb_event_);
    for (auto& v : ev_)
      for (auto& p : v) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
    // a timing slot this session opened whose launch threw: never hand its events to a later
    // launch on this thread
    if (g_launch_timing.stop != nullptr && g_launch_timing.stop == prof_stop_) {
      (void)hipEventDestroy(g_launch_timing.start);
      (void)hipEventDestroy(g_launch_timing.stop);
      g_launch_timing = LaunchTiming{};
    }
  }

  // ------------------------------------------------------------------ run loop
  void run(int64_t max_steps, int64_t* done, int32_t* finished) override {
    const auto t0 = std::chrono::steady_clock::now();
    int64_t steps = 0;
    while (!finished_ && (max_steps <= 0 || steps < max_steps)) {
      if (inner_ >= O_.maxit) { end_phase(); continue; }
      // iterations a device-controlled batch may run from here (each records once)
      step_room_ = max_steps > 0 ? max_steps - steps : INT64_MAX;
      const int64_t k0 = k_;
      switch (method_) {
        case GLX_PROXGD: iter_proxgd(); break;
        case GLX_FPROXGD: iter_fista(false); break;
        case GLX_FGD: iter_fista(true); break;
        default: iter_descent(); break;
      }
      steps += k_ - k0;
      prog_k_.store(k_, std::memory_order_relaxed);
      prog_phase_.store(phase_, std::memory_order_relaxed);
      if (O_.max_total_iters > 0 && k_ >= O_.max_total_iters) finished_ = true;
    }
    GLX_HIP(hipStreamSynchronize(st_));
    tt_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (done) *done = steps;
    if (finished) *finished = finished_ ? 1 : 0;
  }

  void finish(glx_result* res) override {
    if (!res) throw Error{GLX_E_INVALID, "null result"};
    // fval = objective of the returned x (gl_ProxGD_primal.py:141). SGD uses its phase mu.
    const double mu_obj = (method_ == GLX_SGD) ? mu_ : P_.mu0;
    objective_of(X_[ix_]);
    res->fval = 0.5 * hs_[S_RO] + mu_obj * hs_[S_XRN];
    const double final_sp = hs_[S_RO + 3] / (double)nl_;   // count(x) when use_sparsity_
    if (ix_ != 0) copy_buf(X_[0], X_[ix_]);
    if (device_hist_ && k_ > 0) {
      fh_.resize(k_);
      GLX_HIP(hipMemcpyAsync(fh_.data(), fh_dev_, sizeof(double) * k_, hipMemcpyDeviceToHost, st_));
    }
    std::vector<double> sp100;
    if (device_hist_ && k_ >= 100) {
      sp100.resize(k_ / 100 + 1);
      GLX_HIP(hipMemcpyAsync(sp100.data(), sp100_, sizeof(double) * sp100.size(), hipMemcpyDeviceToHost, st_));
    }
    GLX_HIP(hipStreamSynchronize(st_));
    // sparsity of the iterate after iteration i's update (the reference's 100-iteration debug
    // line, gl_ProxGD_primal.py:134-136): the next recorded sparsity, the returned x's for the
    // last one; SGD/GD record it on the device at every 100th iteration only (NaN elsewhere)
    trace_sp_.assign(k_, NAN);
    for (int64_t i = 0; i < k_; ++i) {
      if (use_sparsity_) trace_sp_[i] = (i + 1 < (int64_t)sp_hist_.size()) ? sp_hist_[i + 1] : final_sp;
      else if ((i + 1) % 100 == 0 && (size_t)((i + 1) / 100) < sp100.size())
        trace_sp_[i] = sp100[(i + 1) / 100] / (double)nl_;
    }
    if (device_hist_) {
      fhb_.resize(fh_.size());
      double best = INFINITY;
      for (size_t i = 0; i < fh_.size(); ++i) {
        if (fh_[i] < best) best = fh_[i];
        fhb_[i] = best;
      }
    }
    res->iters = k_;
    res->tt = tt_;
    const int64_t cnt = std::min<int64_t>(res->f_cap, (int64_t)fh_.size());
    if (res->f_hist && cnt > 0) std::memcpy(res->f_hist, fh_.data(), sizeof(double) * cnt);
    if (res->f_hist_best && cnt > 0) std::memcpy(res->f_hist_best, fhb_.data(), sizeof(double) * cnt);
    res->n_fhist = cnt;
    res->ax_calls = ax_calls_;
    res->ax_sources = ax_cols_;
    for (int i = 0; i < 8; ++i) res->stats[i] = stats_[i];
    res->atr_calls = atr_calls_;
    res->syncs = syncs_;
    res->record_waits = record_waits_;
    // finish() overwrote residual buffers: rebuild the iteration state if run() is called again
    state_valid_ = false;
    y_ready_ = false;
    spec_ready_ = false;
    spec_trial_ready_ = false;
    ax_queued_ = false;
    kslot_ = -1;
  }

  void trace(double* sp_after, int64_t cap, int64_t* n, int64_t phase_info[6]) const override {
    const int64_t cnt = std::min<int64_t>(cap, (int64_t)trace_sp_.size());
    if (sp_after && cnt > 0) std::memcpy(sp_after, trace_sp_.data(), sizeof(double) * cnt);
    if (n) *n = sp_after ? cnt : (int64_t)trace_sp_.size();
    if (phase_info)
      for (int p = 0; p < 3; ++p) { phase_info[p] = phase_start_[p]; phase_info[3 + p] = phase_break_[p]; }
  }

  // per trial batch of the split-candidate form: ProxGD the rows of e (rows the threshold
  // changed, accepted trials), FProxGD nnz(e_c) of a gathered batch (row form: flagged rows) or -1
  // for a dense batch; returns the count, copies up to cap
  int64_t split_trace(double* out, int64_t cap) const override {
    const int64_t cnt = std::min<int64_t>(cap, (int64_t)split_hist_.size());
    if (out && cnt > 0) std::memcpy(out, split_hist_.data(), sizeof(double) * cnt);
    return (int64_t)split_hist_.size();
  }

  // the kernels this session actually launches (bench.py re-derived the plan)
  std::string describe() const override {
    std::string s = describe_plan(plan_);
    if (comm_ == nullptr && fused_ok_) s += unfused_spec_ ? " +trial (k_prox_pgd behind A^T r)" : " +trial (k_atr_prox)";
    if (comm_ == nullptr && fused_fista_ok_) s += " +trial (k_atr_fista)";
    s += "; split=";
    if (smode_ == 0) s += "dense";
    else if (egat_) s += "A e fused into the dense pass (k_ax_dma EG), S0=" + std::to_string(gsplit_);
    else if (hyb_rows_ > 0.0)
      s += "gather k_at_gather_bm, A e fused into the dense pass (k_ax_dma EG) from " +
           std::to_string((int64_t)hyb_rows_) + " flagged rows";
    else if (rows_form_) s += "rows k_at_rows S0=" + std::to_string(gsplit_);
    else if (gform_ == 2) s += "gather k_e_lists+k_at_gather";
    else s += "gather k_at_gather_bm";
    if (shard_ && fshard_)
      s += "; rows=sharded x" + std::to_string(sranks_) + (shard_model_ ? " (timing model)" : "") +
           " (reduce-scatter of A^T r, k_fista_trial on n/" + std::to_string(sranks_) +
           " rows, all-gather of xc, k_fista_split)";
    else if (shard_)
      s += "; rows=sharded x" + std::to_string(sranks_) + (shard_model_ ? " (timing model)" : "") +
           " (reduce-scatter of A^T r, k_prox_pgd on n/" + std::to_string(sranks_) +
           " rows, all-gather of p, " + (sderive_ ? "derive and A e in the dense pass" : "k_trial_split") + ")";
    s += "; dc_window=" + std::to_string(dc_window_);
    return s;
  }

  void progress(int64_t out[4]) const override {
    out[0] = prog_k_.load(std::memory_order_relaxed);
    out[1] = prog_phase_.load(std::memory_order_relaxed);
    out[2] = prog_wait_.load(std::memory_order_relaxed);
    out[3] = comm_ != nullptr ? comm_issued(comm_) : 0;
  }

  void counters(int64_t out[4]) const override {
    out[0] = ax_calls_;
    out[1] = ax_cols_;
    out[2] = atr_calls_;
    out[3] = syncs_;
  }

  void kernel_time(int kind, int64_t* launches, double* ms) override {
    if (kind < 0 || kind > 2)
      throw Error{GLX_E_INVALID, "kind must be 0 (A@x), 1 (A^T r) or 2 (split-candidate A e gather)"};
    auto& v = ev_[kind];
    double total = 0.0;
    if (!v.empty()) GLX_HIP(hipEventSynchronize(v.back().b));
    for (auto& p : v) {
      float t = 0.f;
      GLX_HIP(hipEventElapsedTime(&t, p.a, p.b));
      total += t;
      ev_pool_.push_back(p.a);
      ev_pool_.push_back(p.b);
    }
    if (launches) *launches = (int64_t)v.size();
    if (ms) *ms = total;
    v.clear();
  }

 private:
  // ------------------------------------------------------------------ helpers
  // while a device-controlled batch is queued every reduction carries its abort word: the launch
  // is skipped once a decision has cancelled the rest of the batch (*skip not 0 and not pass)
  Red red(int slot, int pass = 0) { return red_to(scal_ + slot, pass); }
  Red red_to(double* out, int pass = 0) {
    Red r{part_, ticket_, out};
    r.skip = dc_gate_;
    r.skip_pass = pass;
    return r;
  }

  // HIP-event timing of A@X (kind 0) / A^T R (kind 1) / gather (kind 2) launches. opts.profile =
  // k > 0 times every k-th launch of each kind. The events ride on the kernel itself
  // (hipExtLaunchKernel through glx_launch, see LaunchTiming): the next glx_launch takes them, so
  // the pair brackets exactly that kernel and adds nothing to the queue.
  // Launches queued inside a device-controlled batch carry the batch segment's tag; when a
  // decision cancels segments, their samples are dropped (prof_drop_from): a cancelled launch
  // exits at once and would report a near-zero kernel time.
  hipEvent_t prof_begin(int kind) {
    if (O_.profile <= 0 || (prof_n_[kind]++ % O_.profile) != 0) return nullptr;
    hipEvent_t e0 = get_event();
    prof_stop_ = get_event();
    prof_tag_ = dc_gate_ != nullptr ? dc_tag_ : 0;
    g_launch_timing = LaunchTiming{e0, prof_stop_};
    return e0;
  }
  // drop the samples of batch segments tagged >= tag (those a device-side decision cancelled)
  void prof_drop_from(int64_t tag) {
    for (auto& v : ev_) {
      size_t keep = 0;
      for (size_t i = 0; i < v.size(); ++i) {
        if (v[i].tag != 0 && v[i].tag >= tag) {
          ev_pool_.push_back(v[i].a);
          ev_pool_.push_back(v[i].b);
        } else {
          v[keep++] = v[i];
        }
      }
      v.resize(keep);
    }
  }
  void prof_end(int kind, hipEvent_t e0) {
    if (e0 == nullptr) return;
    const LaunchTiming lt = g_launch_timing;
    g_launch_timing = LaunchTiming{};
    if (lt.start == nullptr) {   // taken by the launch: keep the sample
      ev_[kind].push_back({e0, prof_stop_, prof_tag_});
    } else {                     // the launch path had no timed kernel: no sample
      ev_pool_.push_back(lt.start);
      ev_pool_.push_back(lt.stop);
    }
  }

  hipEvent_t prof_stop_ = nullptr;   // the stop event of the open prof_begin
  int64_t prof_tag_ = 0;             // its batch segment (0: not in a device-controlled batch)
  // Timing-only events (round 4): hipEventDisableSystemFence drops the system-scope release /
  // acquire the runtime otherwise wraps around an event-stamped launch (an L2 writeback and
  // invalidate, "the cost of cache writeback and invalidation, and the performance impact of
  // those actions on the execution of following work", hip_runtime_api.h). The pair still
  // brackets exactly that kernel; nothing reads the events but hipEventElapsedTime.
  // GLX_EVENT_FENCE=1 restores plain events.
  hipEvent_t get_event() {
    if (ev_pool_.empty()) {   // grow in batches: never create events inside a timed loop's steady state
      static const bool fence = [] {
        const char* e = std::getenv("GLX_EVENT_FENCE");
        return e && std::strcmp(e, "1") == 0;
      }();
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        GLX_HIP(hipEventCreateWithFlags(&e, fence ? hipEventDefault : hipEventDisableSystemFence));
        ev_pool_.push_back(e);
      }
    }
    hipEvent_t e = ev_pool_.back();
    ev_pool_.pop_back();
    return e;
  }

  void copy_buf(T* dst, const T* src) {
    GLX_HIP(hipMemcpyAsync(dst, src, sizeof(T) * nl_, hipMemcpyDeviceToDevice, st_));
  }
  void copy_x(int dst, int src) { copy_buf(X_[dst], X_[src]); }

  void allreduce_scalar(int slot) {
    if (comm_) comm_allreduce(comm_, scal_ + slot, 1, GLX_F64, st_);
  }

  // R[src] = A X[src] - b for src < nsrc in one pass over A; scal[slot + src] = sum R[src]^2
  // (summed over ranks), scal[slot + 3] = count(|cx| > 1e-6 * *cmax); fh: device f record.
  // pub_seq != NULL: also enqueue the scalar packet for the host once the sums are final
  // (after the all-reduce with a communicator); *pub_seq receives the sequence number to wait
  // for (wait_readback), so more work can be queued before the host blocks.
  // defer != NULL (communicator, f64): the sums go to `defer` (a gradient set's tail) instead
  // of scal[slot..], are NOT all-reduced here and nothing is published — they ride the next
  // gradient all-reduce and publish (atr_prox / atr_fista), saving one all-reduce per iteration.
  // skip_ax: the slabs are already in Pp_ (queued speculatively with the trial, spec_ax);
  // only the finalize runs.
  // chain (split-candidate ProxGD trial, nsrc = 2): xs = [e | p_thr] with e flagged by zf_;
  // the finalize forms A p - b = (A p_thr - b) + A e and keeps only its sum (rs[0] unused).
  void residuals(int nsrc, const T* const* xs, T* const* rs, int slot, const T* cx = nullptr,
                 const double* cmax = nullptr, double* fh = nullptr, double fh_mu = 0.0,
                 unsigned* pub_seq = nullptr, double* defer = nullptr, bool skip_ax = false,
                 bool snap_trial = false, bool chain = false) {
    const bool gat = chain && smode_ == 1;
    if (!skip_ax) {
      if (gat) cand_ax(xs);
      else spec_ax(nsrc, xs);
    }
    T* rsc[3] = {chain ? nullptr : rs[0], rs[1], rs[2]};
    Red rd = defer ? red_to(defer) : red(slot);
    const bool dfin = defer_ && carry_ && pub_seq == nullptr && defer == nullptr && !snap_trial &&
                      (comm_ ? nullptr : fh) == nullptr && dc_ctl_.rec == nullptr;
    // max |p| of a trial whose sums are still partials
    const bool dmax = cx != nullptr && ptr_.part != nullptr && cmax == ptr_.out + 3;
    const int S = gat ? ax_split(plan_, 1) : ax_split(plan_, nsrc);
    if (dfin) {
      flush_fin_pending();
      rd.part = fpart_;
      rd.parts_only = 1;
    }
    launch_finalize_residual<T>(Pp_, S, B_, nsrc, rsc,
                                ml_, nullptr, 0, 1, cx,
                                cx ? nl_ : 0, cmax, comm_ ? nullptr : fh, fh_mu, scal_ + S_DRN,
                                rd, st_,
                                snap_trial ? scal_ + S_TR : nullptr,
                                snap_trial ? scal_ + S_SNAP : nullptr, snap_trial ? 6 : 0,
                                chain ? (qeg_ ? 2 : 1) : 0, gat ? gs_of(qeg_) : 0, dc_ctl_,
                                dmax ? ptr_.part : nullptr, dmax ? ptr_.np : 0, dmax ? ptr_.nv : 6);
    check_launch();
    if (dfin) pfin_ = Pend{fpart_, finalize_blocks(ml_, S, gat ? gs_of(qeg_) : 0, cx ? nl_ : 0), 4, 0u, scal_ + slot};
    if (defer) return;
    if (comm_) {
      comm_allreduce(comm_, scal_ + slot, nsrc, GLX_F64, st_);
      if (fh) {
        launch_record_f(scal_, slot, S_DRN, fh_mu, fh, 0, st_);
        check_launch();
      }
    }
    if (pub_seq != nullptr) *pub_seq = post_readback();
  }
  // A @ [xs] into the slabs Pp_; pb: the launch also carries that scalar packet (ax_pub_ok)
  // In a device-controlled batch the A@X passes, the column lists and the gather are gated by the
  // abort word too (live only while it is 0): after a rejection, stop or nnz-budget decision the
  // queued passes of the cancelled iterations would otherwise stream A for nothing (up to
  // window - 1 dense passes per cancellation).
  void spec_ax(int nsrc, const T* const* xs, Pub pb = Pub{}) {
    hipEvent_t e0 = prof_begin(0);
    launch_ax<T>(plan_, nsrc, A_, xs, Pp_, dc_gate_, 0, st_, pb);
    check_launch();
    prof_end(0, e0);
    ++ax_calls_;
    ax_cols_ += nsrc;   // dense right-hand sides
  }
  // Split-candidate trial, gather form: A p_thr (one dense source, slabs behind the A e slab)
  // and A e from the transposed copy (one slab at Pp_); xs = [e | p_thr]. The column lists of e
  // are built first on the same stream, from the row masks the trial wrote (a few us; round 2 ran
  // them on a side stream beside the dense pass, where they waited for CUs until the pass drained
  // and the cross-stream wait left the queue idle, see kernels_gather.hip). The dense pass and the
  // gather are timed apart (kinds 0 and 2), so each event pair brackets one kernel of the trace.
  // pb: the dense launch carries that scalar packet.
  // Round 5 (rows_form_): A e is the A^T R panel over the flagged rows of At (k_at_rows: gsplit_
  // slabs, each workgroup compacts its K range's row flags itself), so no column lists.
  // dv (row-sharded ProxGD, sderive_): the dense pass reads p (xs[2]) and derives p_thr into xs[1]
  // itself, with the masks and bitmaps the gather reads (k_ax_lds DRV)
  void cand_ax(const T* const* xs, Pub pb = Pub{}, const AxDerive* dv = nullptr) {
    const T* xd[3] = {xs[1], nullptr, nullptr};
    qeg_ = dv == nullptr && egat_now();
    if (qeg_) {   // round 6: A p and A e in one pass (S slabs each: A e at Pp_, A p behind)
      EGat eg;
      eg.E = xs[0];
      const int64_t npad = (n_ + 63) / 64 * 64;   // glx_device.h zf_npad
      eg.bm = reinterpret_cast<const unsigned short*>(zf_ + npad);
      eg.bstride = npad / 16;
      eg.Pe = Pp_;
      hipEvent_t e0 = prof_begin(0);
      if (!launch_ax_egat<T>(plan_, A_, xs[2], Pp_ + (size_t)gs_of(true) * ml_, dc_gate_, 0, st_, pb, eg))
        throw Error{GLX_E_STATE, "fused A e: the plan does not take it"};
      check_launch();
      prof_end(0, e0);
      ++ax_calls_;
      ax_cols_ += 1;
      return;
    }
    if (gform_ == 2) {
      launch_e_lists(zf_, n_, l_, glists_, st_, dc_gate_);
      check_launch();
    }
    hipEvent_t e0 = prof_begin(0);
    if (dv != nullptr) {
      if (pb.s2 != nullptr || pb.dpart[0] != nullptr || pb.dpart[1] != nullptr || dc_gate_ != nullptr ||
          !launch_ax_derive<T>(plan_, A_, xs[2], Pp_ + (size_t)gsplit_ * ml_, st_, pb, *dv))
        throw Error{GLX_E_STATE, "row-sharded derive: the dense pass does not take it"};
    } else {
      launch_ax<T>(plan_, 1, A_, xd, Pp_ + (size_t)gsplit_ * ml_, dc_gate_, 0, st_, pb);
    }
    check_launch();
    prof_end(0, e0);
    if (dv != nullptr) {   // A e ran inside the dense pass
      ++ax_calls_;
      ax_cols_ += 1;
      return;
    }
    hipEvent_t e2 = prof_begin(2);
    if (gform_ == 1) launch_at_rows<T>(At_, xs[0], zf_, m_, n_, l_, Pp_, glists_, st_, dc_gate_);
    else if (gform_ == 2) launch_at_gather<T>(At_, xs[0], m_, n_, l_, Pp_, glists_, st_, dc_gate_);
    else launch_at_gather_bm<T>(At_, xs[0], zf_, m_, n_, l_, Pp_, glists_, st_, dc_gate_);
    check_launch();
    prof_end(2, e2);
    ++ax_calls_;
    ax_cols_ += 1;
  }
  void residual1(const T* x, T* r, int slot, const T* cx = nullptr, const double* cmax = nullptr,
                 unsigned* pub_seq = nullptr) {
    const T* xs[3] = {x, nullptr, nullptr};
    T* rs[3] = {r, nullptr, nullptr};
    residuals(1, xs, rs, slot, cx, cmax, nullptr, 0.0, pub_seq);
  }

  // G = A^T r as slabs of gradient set `set` (default: the current one); returns (source, S)
  // for the consumer. With a communicator the slabs are summed and all-reduced first (S = 1).
  // tail_n > 0 (communicator, f64): the all-reduce also sums the first tail_n doubles of the
  // set's tail (deferred residual sums, see residuals()).
  std::pair<const T*, int> gradient(const T* r, int set = -1, int tail_n = 0) {
    if (set < 0) set = gset_;
    T* G = Gs_[set];
    T* Gp = Gps_[set];
    hipEvent_t e0 = prof_begin(1);
    launch_atr<T>(plan_, A_, r, Gp, st_);
    check_launch();
    prof_end(1, e0);
    ++atr_calls_;
    if (!comm_) return {Gp, plan_.atr_S};
    if (plan_.atr_S > 1) {
      launch_sum_partials<T>(Gp, plan_.atr_S, G, nl_, st_);
      check_launch();
    }
    comm_allreduce(comm_, G, nl_ + tail_n, P_.dtype, st_);
    return {G, 1};
  }
  void use_gset(int set) { gset_ = set; G_ = Gs_[set]; Gp_ = Gps_[set]; }
  int nset(int set) const { return set + 1 == nsets_ ? 0 : set + 1; }   // the next set of the ring
  double* tail(int set) { return reinterpret_cast<double*>(Gs_[set] + nl_); }
  // merge a speculated trial's residual sums into the next gradient all-reduce
  bool merge_tail() const { return comm_ != nullptr && sizeof(T) == 8; }

  // Speculative gradient (ProxGD / FISTA with line search). The next iteration's gradient
  // residual is produced by the trial's batched A@X, and the next gradient depends only on
  // whether that trial is accepted. So A^T r of the candidate is queued behind the trial
  // and runs while the host reads the trial's scalars and decides, into the other gradient
  // set. If the trial is rejected it is dropped. Used only while the previous iteration
  // accepted its first trial, so a rejecting regime pays no extra passes.
  std::pair<const T*, int> take_gradient(const T* r) {
    if (spec_ready_) {
      spec_ready_ = false;
      use_gset(spec_set_);
      return spec_g_;
    }
    return gradient(r);
  }
  bool want_spec(int trial_it) const {
    return spec_on_ && trial_it == 0 && O_.step_type == GLX_STEP_LINE_SEARCH && !spec_off_env_;
  }

  // Scalar readback in two halves so that work can be queued between them (the speculative
  // gradient): post_readback enqueues the packet copy behind everything queued so far and
  // returns its sequence number; wait_readback spins on the host-mapped sequence word.
  // extra != NULL: the packet's S_RT..S_RT+3 come from extra[0..4) (a gradient set's tail)
  unsigned post_readback(const double* extra = nullptr) {
    ++syncs_;
    if (pending()) {   // deferred reductions: reduced by the publishing kernel first
      Pub pb;
      pb.s = scal_;
      pb.ns = NSCAL;
      pb.s2 = extra;
      pb.off2 = S_RT;
      pb.n2 = extra ? 4 : 0;
      attach_pending(pb);
      if (spin_readback_) {
        pb.host = hs_dev_;
        pb.host_seq = hseq_dev_;
        pb.seq = ++seq_;
      }
      launch_publish_pub(pb, st_);
      check_launch();
      if (spin_readback_) return pb.seq;
    }
    if (!spin_readback_) {   // GLX_READBACK=sync: stream-ordered copies, then an event wait
      GLX_HIP(hipMemcpyAsync(hs_, scal_, sizeof(double) * NSCAL, hipMemcpyDeviceToHost, st_));
      if (extra) GLX_HIP(hipMemcpyAsync(hs_ + S_RT, extra, 4 * sizeof(double), hipMemcpyDeviceToHost, st_));
      if (!rb_event_) GLX_HIP(hipEventCreateWithFlags(&rb_event_, hipEventDisableTiming));
      GLX_HIP(hipEventRecord(rb_event_, st_));
      return 0;
    }
    const unsigned seq = ++seq_;
    launch_publish(scal_, NSCAL, hs_dev_, hseq_dev_, seq, st_, extra, S_RT, 4);
    check_launch();
    return seq;
  }
  // The packet as a Pub for the next launch to carry (attach_ok_); *seq_out = its number.
  Pub make_pub(const double* extra, unsigned* seq_out) {
    ++syncs_;
    Pub pb;
    pb.s = scal_;
    pb.ns = NSCAL;
    pb.host = hs_dev_;
    pb.host_seq = hseq_dev_;
    pb.seq = ++seq_;
    pb.s2 = extra;
    pb.off2 = S_RT;
    pb.n2 = extra ? 4 : 0;
    attach_pending(pb);
    *seq_out = pb.seq;
    return pb;
  }
  // deferred reductions (defer_): partials not yet reduced into their scalar slots
  struct Pend {
    const double* part = nullptr;
    int np = 0, nv = 0;
    unsigned mx = 0;
    double* out = nullptr;
  };
  bool pending() const { return ptr_.part != nullptr || pfin_.part != nullptr; }
  // a finalize's partials still pending when the next finalize would overwrite them (FProxGD's
  // g(y) residual ahead of the trial's batch): reduced on their own first
  void flush_fin_pending() {
    if (pfin_.part == nullptr) return;
    Pub pb;
    pb.dpart[0] = pfin_.part;
    pb.dnp[0] = pfin_.np;
    pb.dnv[0] = pfin_.nv;
    pb.dmax[0] = pfin_.mx;
    pb.dout[0] = pfin_.out;
    pfin_ = Pend{};
    launch_publish_pub(pb, st_);
    check_launch();
  }
  // the kernel carrying pb reduces the pending partials before it copies the packet
  void attach_pending(Pub& pb) {
    int d = 0;
    for (Pend* q : {&ptr_, &pfin_}) {
      if (q->part == nullptr) continue;
      pb.dpart[d] = q->part;
      pb.dnp[d] = q->np;
      pb.dnv[d] = q->nv;
      pb.dmax[d] = q->mx;
      pb.dout[d] = q->out;
      ++d;
      *q = Pend{};
    }
  }
  void wait_readback(unsigned seq) {
    if (!spin_readback_) {
      GLX_HIP(hipEventSynchronize(rb_event_));
      return;
    }
    // spin on the sequence word the GPU writes after the packet (system-scope release)
    volatile unsigned* hs = hseq_;
    uint64_t spins = 0;
    auto t0 = std::chrono::steady_clock::time_point{};
    prog_wait_.store(1, std::memory_order_relaxed);
    while (*hs != seq) {
      __builtin_ia32_pause();
      if ((++spins & 0xFFFFF) == 0) {
        if (spins == 0x100000) t0 = std::chrono::steady_clock::now();
        else stalled_wait(t0, [&] { return *hs == seq; }, "scalar readback");
      }
    }
    prog_wait_.store(0, std::memory_order_relaxed);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  // A host wait that has spun for over ~5 s. Without a communicator the stream is synchronised
  // (it surfaces a device error) and the wait fails if the word still has not come. With RCCL
  // (round 6) a collective may be waiting for a peer: the stream is only
  // queried, RCCL's asynchronous error is polled (an error aborts the communicator, so the
  // blocked RCCL kernels return and the stream drains, then throws), and after GLX_WAIT_TIMEOUT_S
  // (default 300 s) the communicator is aborted too and the wait fails with the progress record
  // (iteration, collectives issued) — a diagnostic instead of a silent hang.
  template <typename Done>
  void stalled_wait(std::chrono::steady_clock::time_point t0, Done done, const char* what) {
    if (comm_ == nullptr || !comm_is_rccl(comm_)) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        GLX_HIP(hipStreamSynchronize(st_));   // surfaces a device error, if any
        if (!done()) throw Error{GLX_E_HIP, std::string(what) + " timed out"};
      }
      return;
    }
    const int aerr = comm_async_error(comm_);
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    static const double limit = [] {
      const char* e = std::getenv("GLX_WAIT_TIMEOUT_S");
      return e ? std::atof(e) : 300.0;
    }();
    if (aerr == 0 && (limit <= 0 || waited < limit)) return;
    const std::string why =
        std::string(what) + (aerr != 0 ? " failed: RCCL asynchronous error " + std::to_string(aerr)
                                       : " stalled for " + std::to_string((int)waited) + " s") +
        " on rank " + std::to_string(comm_rank(comm_)) + " of " + std::to_string(comm_size(comm_)) +
        " at iteration " + std::to_string(k_) + " (phase " + std::to_string(phase_) + "), after " +
        std::to_string(comm_issued(comm_)) + " collectives issued; the communicator was aborted";
    comm_abort(comm_);
    (void)hipStreamSynchronize(st_);   // the aborted RCCL kernels return
    throw Error{GLX_E_RCCL, why};
  }
  void readback() { wait_readback(post_readback()); }

  // objective of x (used by finish and as the FISTA prologue): S_XRN, S_XMAX, S_RO (sum r^2),
  // S_RO + 3 (count); r = A x - b -> R_[0]
  void objective_of(T* x) {
    launch_rownorm_max<T>(x, n_, l_, red(S_XRN), st_);
    check_launch();
    unsigned seq = 0;
    residual1(x, R_[0], S_RO, use_sparsity_ ? x : nullptr, scal_ + S_XMAX, &seq);
    wait_readback(seq);
  }

  void record(double f, double s) {
    fh_.push_back(f);
    if (f < fbest_) fbest_ = f;   // Python min(f_best, f): NaN never becomes the best
    fhb_.push_back(fbest_);
    if (use_sparsity_) { sp_prev_ = sp_cur_; sp_cur_ = s; sp_hist_.push_back(s); }
    ++k_;
    ++inner_;
  }

  // stability rule (gl_ProxGD_primal.py:118-125); true = break
  bool stop_rule() {
    const size_t k = fh_.size();
    bool ok = false;
    if (k > 1) {
      ok = std::fabs(fh_[k - 1] - fh_[k - 2]) / std::fabs(fh_[k - 2]) < O_.ftol;
      if (ok && use_sparsity_) ok = std::fabs(sp_cur_ - sp_prev_) / std::fabs(sp_prev_) < O_.ftol;
    }
    stable_ = ok ? stable_ + 1 : 0;
    return stable_ > O_.stable_len_threshold;
  }

  void end_phase(bool by_stop_rule = false) {
    if (phase_ < 3) phase_break_[phase_] = by_stop_rule ? 1 : 0;
    ++phase_;
    inner_ = 0;
    stable_ = 0;
    if (phase_ >= 3) { finished_ = true; return; }
    phase_start_[phase_] = k_;
    mu_ = mus_[phase_];
    if (method_ == GLX_FPROXGD || method_ == GLX_FGD) {  // gl_FProxGD_primal.py:68-69
      copy_x(iv_, ix_);
      tk_ = O_.alpha0;
      y_ready_ = false;
      spec_ready_ = false;   // y is re-formed from the reset v: its gradient was not speculated
      spec_trial_ready_ = false;
    }
  }

  double schedule(int64_t inner) const {  // gl_ProxGD_primal.py:78-85
    const double it_hat = (double)(std::max<int64_t>(inner, 1000) - 999);
    switch (O_.step_type) {
      case GLX_STEP_FIXED: return O_.alpha0;
      case GLX_STEP_DIMINISHING: return O_.alpha0 / std::sqrt(it_hat);
      case GLX_STEP_DIMINISHING2: return O_.alpha0 / it_hat;
      default: return O_.alpha0;
    }
  }

  // ------------------------------------------------------------------ ProxGD
  // Invariants between iterations (state_valid_): X_[ix_] = x (unthresholded, what is recorded
  // and returned), X_[ixt_] = thr(x) (:127), R_[irg_] = A thr(x) - b (the gradient residual,
  // :129, exact), gx_ = 1/2 ||R_[irg_]||^2, f_cur_/s_cur_ = objective and sparsity of x.
  void proxgd_prologue(bool have_thr) {
    spec_ready_ = false;   // the gradient is recomputed from the rebuilt residual
    spec_trial_ready_ = false;
    ax_queued_ = false;
    if (!have_thr) {
      launch_threshold<T>(X_[ix_], X_[ixt_], nl_, O_.thres, flag_, ++epoch_, st_);
      check_launch();
    }
    launch_rownorm_max<T>(X_[ix_], n_, l_, red(S_XRN), st_);
    check_launch();
    const int ro = (irg_ + 1) % kRes;
    const T* xs[3] = {X_[ix_], X_[ixt_], nullptr};
    T* rs[3] = {R_[ro], R_[irg_], nullptr};
    unsigned seq = 0;
    residuals(2, xs, rs, S_RO, X_[ix_], scal_ + S_XMAX, nullptr, 0.0, &seq);   // A @ [x | thr(x)]
    wait_readback(seq);
    f_cur_ = 0.5 * hs_[S_RO] + P_.mu0 * hs_[S_XRN];
    s_cur_ = hs_[S_RO + 3] / (double)nl_;
    gx_ = 0.5 * hs_[S_RO + 1];
    state_valid_ = true;
  }

  // First-trial sources: (1) a speculative fused kernel of the previous iteration left G and
  // this trial ready (same mu and t); (2) otherwise A^T r with the trial fused into it
  // (launch_atr_prox); (3) otherwise the gradient (speculative or not) and k_prox_pgd.
  void iter_proxgd() {
    if (shard_) { iter_proxgd_shard(); return; }
    if (!state_valid_) proxgd_prologue(thr_from_trial_);
    record(f_cur_, s_cur_);
    if (stop_rule()) { end_phase(true); return; }
    if (dc_ready()) { dc_run(); return; }
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    const double t0 = ls ? O_.alpha0 : schedule(inner_);
    std::pair<const T*, int> g{nullptr, 0};
    bool first_done = false;
    if (spec_trial_ready_) {
      spec_trial_ready_ = false;
      use_gset(spec_set_);
      g = {G_, 1};
      first_done = (spec_trial_mu_ == mu_ && spec_trial_t_ == t0);   // else: a phase change
      if (!first_done) ax_queued_ = false;
    } else if (fused_ok_) {
      carry_ = want_spec(0);   // the batch's packet will ride the speculative kernel
      atr_prox(R_[irg_], gset_, X_[ixt_], ip_, ipt_, iz_, t0);
      carry_ = false;
      g = {G_, 1};
      first_done = true;
    } else {
      g = take_gradient(R_[irg_]);
    }
    proxgd_trials(g, first_done, t0, 0);
  }

  // The line search from trial it0 (it0 = 1: the first trial was rejected by a device-side
  // decision, dc_run; t0 is then already alpha0 * ls_coeff), or the fixed step, and the update.
  void proxgd_trials(std::pair<const T*, int> g, bool first_done, double t0, int it0) {
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    const T* xt = X_[ixt_];
    const bool exact = O_.exact_objective != 0;
    // trial residual buffers: never the gradient residual
    const int rz = (irg_ + 1) % kRes, rpt = (irg_ + 2) % kRes, rp = (irg_ + 3) % kRes;
    double t;
    bool accepted = false, spec_trial = false;
    auto trial = [&](double tt, bool first) {
      launch_prox_pgd<T>(xt, first ? g.first : G_, first ? g.second : 1,
                         (first && g.first != G_) ? G_ : nullptr, X_[ip_], X_[ipt_], X_[iz_], n_,
                         l_, tt, mu_, O_.thres, red(S_TR), st_, Pub{}, ezf());
      check_launch();
      ptr_ = Pend{};   // S_TR holds this trial's sums
    };
    if (ls) {
      t = t0;
      for (int it = it0; it < O_.ls_maxit; ++it) {
        if (!(it == 0 && first_done)) trial(t, it == 0);
        // one pass: the candidate's g for the test (:91) + the next iteration's residual
        // A p_thr (exact mode: g(z) and A p as a third source). Split-candidate mode (emode_,
        // the default fast mode): the batch is [e | p_thr], e = p - p_thr, and the test and the
        // next objective use g(p) = 1/2 ||(A p_thr - b) + A e||^2. z = x - t G_t equals p up to
        // the rounding of x - t((x - p)/t), the same order as the GEMMs' own summation-order
        // differences, while e is nonzero only in the rows the hard threshold touched, so A e
        // costs MFMAs only on those K chunks (k_ax_lds SP) instead of a second dense source.
        const T* xs[3] = {X_[iz_], X_[ipt_], X_[ip_]};
        T* rs[3] = {R_[rz], R_[rpt], R_[rp]};
        const int nsrc = exact ? 3 : 2;
        unsigned seq = 0;
        const bool spec = want_spec(it);
        const bool merge = spec && fused_ok_ && merge_tail();
        // the packet rides the speculative kernel (no communicator; with one only when merged)
        const bool late_pub = merge || (spec && fused_ok_ && attach_ok_ && comm_ == nullptr);
        const bool skip_ax = it == 0 && first_done && ax_queued_;   // queued with the trial
        ax_queued_ = false;
        // with a communicator the speculative next trial is a short k_prox_pgd: its A@X is
        // queued right behind it and carries this trial's packet, whose trial sums (which
        // that k_prox_pgd overwrites) come from a snapshot this finalize takes
        const bool axp = spec && fused_ok_ && comm_ != nullptr && late_pub && attach_ok_ &&
                         spec_ax_pub_ && ax_pub_ok(plan_, smode_ == 1 ? 1 : nsrc);
        carry_ = late_pub;
        residuals(nsrc, xs, rs, S_RT, X_[ip_], scal_ + S_TR + 3, nullptr, 0.0,
                  late_pub ? nullptr : &seq, merge ? tail(nset(gset_)) : nullptr, skip_ax, axp, emode_);
        carry_ = false;
        std::pair<const T*, int> sg;
        if (spec && fused_ok_) {
          // the next iteration's A^T r and first trial at the candidate p_thr, into the other
          // gradient set and the spare buffers (z is free once this trial's A@X has read it)
          Pub pbx;
          atr_prox(R_[rpt], nset(gset_), X_[ipt_], if1_, if2_, iz_, O_.alpha0, merge ? nsrc : 0,
                   late_pub ? &seq : nullptr, axp ? &pbx : nullptr);
          spec_trial = true;
          if (axp) {
            pbx.s3 = scal_ + S_SNAP;
            pbx.off3 = S_TR;
            pbx.n3 = 6;
            const T* sx[3] = {X_[iz_], X_[if2_], X_[if1_]};   // [z | p_thr | p] of that trial
            if (smode_ == 1) cand_ax(sx, pbx);
            else spec_ax(nsrc, sx, pbx);
            ax_queued_ = true;
          }
        } else if (spec) {
          sg = gradient(R_[rpt], nset(gset_));   // gradient at the candidate p_thr
        }
        wait_readback(seq);
        const double gz = 0.5 * hs_[S_RT];
        if (gz <= gx_ - t * hs_[S_TR + 0] + 0.5 * t * hs_[S_TR + 1]) {
          accepted = true;
          if (spec && !spec_trial) { spec_ready_ = true; spec_g_ = sg; spec_set_ = nset(gset_); }
          spec_on_ = (it == 0);
          break;
        }
        spec_trial = false;
        spec_on_ = false;
        ax_queued_ = false;   // the speculated trial and its A@X are dropped
        t *= O_.ls_coeff;
      }
      // after ls_maxit failures the reference returns alpha0*coeff^maxit untested (:99)
      if (!accepted) trial(t, false);
    } else {
      t = t0;
      if (!first_done) trial(t, true);
    }
    if (accepted) {   // the packet holds the accepted trial's sums (read before any speculation)
      proxgd_accept(rpt, exact);
    } else {
      state_valid_ = false;
      thr_from_trial_ = true;                     // x_thr came out of the trial kernel
    }
    // x = prox(x - t grad, t)  (:132)
    if (spec_trial) {   // x <- p, x_thr <- p_thr, the speculative outputs become the trial's
      proxgd_spec_rotate();
    } else {
      std::swap(ix_, ip_);
      std::swap(ixt_, ipt_);
    }
  }

  // accepted trial: the packet (hs_) holds its sums
  // trs: the packet slots that hold the trial's sums (S_TR; row-sharded: S_TR or S_TRN)
  void proxgd_accept(int rpt, bool exact, int trs = S_TR) {
    stats_[0] += hs_[trs + 4];
    stats_[1] += hs_[trs + 5];
    stats_[2] += 1;
    split_hist_.push_back(hs_[trs + 5]);
    last_rows_ = hs_[trs + 5];
    irg_ = rpt;
    gx_ = 0.5 * hs_[S_RT + 1];
    // exact: A p from the batch; split-candidate: A p - b = (A p_thr - b) + A e; dense z
    // batch (GLX_SPLIT_CAND=0): A z - b (z = x - t G_t is ulp-close to p) unless the
    // threshold changed nothing, in which case A p_thr - b == A p - b exactly
    const double sq_x = exact ? hs_[S_RT + 2]
                              : ((emode_ || hs_[trs + 4] != 0) ? hs_[S_RT] : hs_[S_RT + 1]);
    f_cur_ = 0.5 * sq_x + P_.mu0 * hs_[trs + 2];
    s_cur_ = hs_[S_RT + 3] / (double)nl_;
    state_valid_ = true;
  }
  // x <- p, x_thr <- p_thr; the speculative outputs become the next iteration's first trial
  // (z's buffer already holds its z)
  void proxgd_spec_rotate() {
    const int ox = ix_, oxt = ixt_;
    ix_ = ip_; ixt_ = ipt_; ip_ = if1_; ipt_ = if2_;
    if1_ = ox; if2_ = oxt;
    spec_trial_ready_ = true;
    spec_set_ = nset(gset_);
    spec_trial_mu_ = mu_;
    spec_trial_t_ = O_.alpha0;
  }

  // ------------------------------------------------------------------ row-sharded ProxGD
  // (round 5; VERDICT round 4: reduce-scatter -> prox on n/G rows -> all-gather). Per iteration
  // on every rank: A@[e | p_thr] over this rank's rows of A and its finalize (partial residual
  // sums, the sparsity count over this rank's rows of p); A^T r of the candidate, reduce-scattered
  // (this rank's n / G rows of the gradient); the next trial, k_prox_pgd on those rows (partial
  // trial sums); one RCCL group that all-gathers p's rows and every rank's block of partial sums,
  // combined in rank order (k_shard_combine: every rank holds the same bits); then the replicated
  // k_trial_split re-derives p_thr, z and the masks of e from the gathered p. The host decides
  // from the combined sums, with the next trial and its A@X already queued (the speculative path
  // of iter_proxgd). The all-gathered blocks replace the 8-byte all-reduces of the residual sums.
  // Bytes per iteration and rank: reduce-scatter + all-gather of n x l, the same as one ring
  // all-reduce of the gradient; the row-wise work (k_prox_pgd, the count) is divided by G.
  double* blk_own() { return blk_ + (int64_t)(shard_model_ ? 0 : srank_) * schunk_; }
  // the speculated next trial's sums: ProxGD S_TRN; FProxGD S_RO (S_TRN = S_RG holds g(y) of a
  // prologue until the host has read it; S_RO is read right behind its own objective)
  int tr_other() const { return tr_slot_ == S_TR ? (fshard_ ? S_RO : S_TRN) : S_TR; }
  void shard_gradient(const T* r, int set) {
    T* G = Gs_[set];
    T* Gp = Gps_[set];
    hipEvent_t e0 = prof_begin(1);
    launch_atr<T>(plan_, A_, r, Gp, st_);
    check_launch();
    prof_end(1, e0);
    ++atr_calls_;
    if (plan_.atr_S > 1) {
      launch_sum_partials<T>(Gp, plan_.atr_S, G, nl_, st_);
      check_launch();
    }
    comm_reduce_scatter(comm_, G, srows_ * l_, P_.dtype, st_);
  }
  // the trial on this rank's rows: p, p_thr, z rows into X_[op], X_[opt], X_[oz]; its workgroup
  // partials into this rank's chunk (Red::parts_only)
  void shard_prox(const T* xt, const T* G, int op, int opt, int oz, double t) {
    const int64_t o = srow0_ * l_;
    Red rd = red_to(scal_ + S_TR);
    rd.part = blk_own() + kShardPartOff;
    rd.parts_only = 1;
    // sderive_: the masks and bitmaps of e for these rows into the chunk (the third output is then e)
    unsigned* czf = sderive_ ? reinterpret_cast<unsigned*>(blk_own() + moff_) : nullptr;
    launch_prox_pgd<T>(xt + o, G + o, 1, nullptr, X_[op] + o, X_[opt] + o, X_[oz] + o, srows_, l_, t,
                       mu_, O_.thres, rd, st_, Pub{}, czf);
    check_launch();
  }
  // one RCCL group: p's rows (op >= 0) and every rank's chunk of sums
  void shard_exchange(int op) {
    comm_group_begin(comm_);
    if (op >= 0) comm_all_gather(comm_, X_[op], srows_ * l_, P_.dtype, st_);
    comm_all_gather(comm_, blk_, schunk_, GLX_F64, st_);
    comm_group_end(comm_);
  }
  // mask & 1: the trial's sums -> scal_[tr_dst], mask & 2: the finalize's -> scal_[S_RT];
  // seq != NULL: the packet follows (*seq = its number)
  ShardPub shard_pub(int mask, int tr_dst, unsigned* seq) {
    ShardPub sp;
    sp.blk = blk_;
    sp.nranks = cranks_;
    sp.chunk = schunk_;
    sp.nbp = nbp_;
    sp.nbf = nbf_;
    sp.mask = mask;
    sp.tv = stv_;
    sp.tr = scal_ + tr_dst;
    sp.rt = scal_ + S_RT;
    sp.tr_off = tr_dst;
    sp.rt_off = S_RT;
    if (seq != nullptr) sp.pub = make_pub(nullptr, seq);
    return sp;
  }
  // p_thr, z (unless zskip_) and e's masks from the gathered p, the sums combined beside the rows
  void shard_derive(int ixt, int op, int opt, int oz, double t, const ShardPub& sp) {
    launch_trial_split<T>(X_[op], X_[ixt], X_[opt], zskip_ ? nullptr : X_[oz], ezf(), n_, l_, t,
                          O_.thres, emode_, sp, st_);
    check_launch();
  }
  // the trial's pass over this rank's rows of A and its finalize: sums -> the chunk's [6, 10), the
  // count over this rank's rows of cx against the combined max at cmax
  void shard_fin(int nsrc, const T* const* xs, T* const* rs, const T* cx, const double* cmax, bool skip_ax) {
    const bool chain = emode_;
    const bool gat = chain && smode_ == 1;
    if (!skip_ax) {
      if (gat) cand_ax(xs);
      else spec_ax(nsrc, xs);
    }
    T* rsc[3] = {chain ? nullptr : rs[0], rs[1], rs[2]};
    const int64_t o = srow0_ * l_;
    Red rd = red_to(scal_ + S_RT);   // its workgroup partials ride the all-gather too
    rd.part = blk_own() + kShardPartOff + stv_ * nbp_;
    rd.parts_only = 1;
    launch_finalize_residual<T>(Pp_, gat ? ax_split(plan_, 1) : ax_split(plan_, nsrc), B_, nsrc, rsc,
                                ml_, nullptr, 0, 1, cx + o, srows_ * l_, cmax, nullptr, 0.0,
                                scal_ + S_DRN, rd, st_, nullptr, nullptr, 0,
                                chain ? (qeg_ ? 2 : 1) : 0, gat ? gs_of(qeg_) : 0, Ctl{});
    check_launch();
  }
  void iter_proxgd_shard() {
    if (!state_valid_) proxgd_prologue(thr_from_trial_);   // x replicated: all-reduced sums
    record(f_cur_, s_cur_);
    if (stop_rule()) { end_phase(true); return; }
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    const double t0 = ls ? O_.alpha0 : schedule(inner_);
    bool first_done = false;
    if (spec_trial_ready_) {   // the previous iteration's speculated trial (its sums in tr_slot_)
      spec_trial_ready_ = false;
      use_gset(spec_set_);
      first_done = (spec_trial_mu_ == mu_ && spec_trial_t_ == t0);
      if (!first_done) ax_queued_ = false;
    } else {
      shard_gradient(R_[irg_], gset_);
    }
    const bool exact = O_.exact_objective != 0;
    const int rz = (irg_ + 1) % kRes, rpt = (irg_ + 2) % kRes, rp = (irg_ + 3) % kRes;
    const int nsrc = exact ? 3 : 2;
    auto trial = [&](double tt) {
      shard_prox(X_[ixt_], G_, ip_, ipt_, iz_, tt);
      shard_exchange(ip_);
      shard_derive(ixt_, ip_, ipt_, iz_, tt, shard_pub(1, tr_slot_, nullptr));
    };
    double t = t0;
    bool accepted = false, spec_trial = false;
    if (ls) {
      for (int it = 0; it < O_.ls_maxit; ++it) {
        if (!(it == 0 && first_done)) trial(t);
        const T* xs[3] = {zskip_ ? X_[ip_] : X_[iz_], X_[ipt_], X_[ip_]};
        T* rs[3] = {R_[rz], R_[rpt], R_[rp]};
        const bool skip_ax = it == 0 && first_done && ax_queued_;
        ax_queued_ = false;
        shard_fin(nsrc, xs, rs, X_[ip_], scal_ + tr_slot_ + 3, skip_ax);
        unsigned seq = 0;
        if (want_spec(it)) {
          // the next iteration's gradient and first trial at the candidate p_thr (the other
          // gradient set, the spare buffers, the other trial slot); their exchange carries this
          // trial's residual sums, and the next trial's A@X is queued before the host waits
          const int ns = nset(gset_);
          const int ot = tr_other();
          shard_gradient(R_[rpt], ns);
          shard_prox(X_[ipt_], Gs_[ns], if1_, if2_, iz_, O_.alpha0);
          shard_exchange(if1_);
          // the packet (this trial's residual sums, the next trial's sums) rides the next trial's
          // dense pass as its publisher workgroup: a workgroup of the 8 MiB-writing k_trial_split
          // that stores to host memory stretched that kernel from 5.6 to 17.8 us (its end-of-
          // kernel release), a separate k_publish costs ~4.5 us (profiles/r5_shard/)
          const bool carry = spin_readback_ && attach_ok_ && ax_pub_ok(plan_, smode_ == 1 ? 1 : nsrc);
          const bool fused = carry && sderive_;   // round 6: the derive inside the dense pass
          if (!fused) shard_derive(ipt_, if1_, if2_, iz_, O_.alpha0, shard_pub(3, ot, nullptr));
          const T* sx[3] = {zskip_ ? X_[if1_] : X_[iz_], X_[if2_], X_[if1_]};
          Pub pb;
          if (carry) pb = make_pub(nullptr, &seq);
          else seq = post_readback();
          if (fused) {
            AxDerive dv;
            dv.pthr = X_[if2_];
            dv.thres = O_.thres;
            dv.sp = shard_pub(3, ot, nullptr);
            dv.ggx = (int)((m_ + kDrvGatRows - 1) / kDrvGatRows);
            dv.At = At_;
            dv.E = sx[0];
            dv.Pe = Pp_;
            dv.blk = blk_;
            dv.bstride = shard_model_ ? 0 : schunk_;
            dv.moff = moff_;
            dv.srows = srows_;
            cand_ax(sx, pb, &dv);
          } else if (smode_ == 1) {
            cand_ax(sx, pb);
          } else {
            spec_ax(nsrc, sx, pb);
          }
          ax_queued_ = true;
          spec_trial = true;
        } else {
          // the combine and a plain k_publish: one kernel that combines and then writes the packet
          // measured 17-19 us against ~4 us for k_publish (as k_publish_pub, profiles/r5_probe/)
          shard_exchange(-1);
          launch_shard_combine(shard_pub(2, tr_slot_, nullptr), st_);
          check_launch();
          seq = post_readback();
        }
        wait_readback(seq);
        const double gz = 0.5 * hs_[S_RT];
        if (shard_model_ || gz <= gx_ - t * hs_[tr_slot_ + 0] + 0.5 * t * hs_[tr_slot_ + 1]) {
          accepted = true;
          spec_on_ = (it == 0);
          break;
        }
        spec_trial = false;
        spec_on_ = false;
        ax_queued_ = false;   // the speculated trial and its A@X are dropped
        t *= O_.ls_coeff;
      }
      if (!accepted) trial(t);   // the untested last step (:99)
    } else if (!first_done) {
      trial(t);
    }
    if (accepted) {
      proxgd_accept(rpt, exact, tr_slot_);
    } else {
      state_valid_ = false;
      thr_from_trial_ = true;
    }
    if (spec_trial) {
      proxgd_spec_rotate();
      tr_slot_ = tr_other();
    } else {
      std::swap(ix_, ip_);
      std::swap(ixt_, ipt_);
    }
  }

  // ------------------------------------------------------------------ device-controlled ProxGD
  // SURVEY 8f row 2. In the speculative steady state (the previous first trial was accepted and
  // its fused kernel left G and this iteration's first trial ready) every iteration launches the
  // same kernels on buffer roles that rotate the same way: A@[e | p_thr] (+ the A e gather),
  // its finalize, and the fused A^T r + next trial. So up to dc_window_ iterations are queued
  // ahead of the host. The Armijo test (gl_ProxGD_primal.py:89-92), the next record and the stop
  // rule (:118-125) run in the finalize's last block (ctl_decide, kernels_elem.hip), which writes
  // a decision record to host-mapped memory and an abort word every later launch of the batch
  // tests first: a rejection cancels everything behind it, a stop lets only the speculative
  // gradient finish (the next phase starts from it, as on the host path). The host reads the
  // records in order — re-deriving every decision from the record's sums and checking it —
  // and tops the window up; it never blocks the GPU. A rejection continues on the host path at
  // the second trial; a stop ends the phase there. Results are bit-identical to host control.
  struct Roles { int ix, ixt, ip, ipt, if1, if2, iz, irg, gset; };
  bool dc_ready() const {
    // (with a communicator the first trial's A@X is normally already queued: the batch uses it)
    return dc_window_ > 0 && spec_trial_ready_ && spec_trial_mu_ == mu_ &&
           spec_trial_t_ == O_.alpha0 && want_spec(0) && (comm_ != nullptr || unfused_spec_ || !ax_queued_);
  }
  // Gated (cancellable) launches: the finalize (it would overwrite the decision state and the
  // gradient residual of the iteration the host resumes) and the speculative fused kernel (the
  // next gradient set and iterate buffers). A@X and the gather only write the scratch slabs, so
  // a cancelled one runs to no effect instead of testing the flag.
  Ctl dc_make_ctl(int64_t tag) const {
    Ctl c{};
    const int64_t slot = (tag % kCtlMaxBatch) * kCtlRec;
    c.rec = dc_rec_ + slot;
    c.state = dc_state_;
    c.abort = dc_abort_;
    c.tr = scal_ + S_TR;
    c.tag = (double)tag;
    c.t = O_.alpha0;
    c.mu0 = P_.mu0;
    c.ftol = O_.ftol;
    c.nl = (double)nl_;
    c.stable_thr = O_.stable_len_threshold;
    c.use_sp = use_sparsity_ ? 1 : 0;
    c.emode = emode_ ? 1 : 0;
    c.pass = 1 + (int)(tag % 0x3FFFFFFF);
    return c;
  }
  // With a communicator (f64): the trial's A@X is queued already (the previous segment, or the
  // host path before the batch); its finalize defers the residual sums into the next gradient
  // set's tail; A^T r of the candidate and the all-reduce of [G | tail] (not gated: a ring of
  // gradient sets, kMaxGSets); the decision (k_ctl_decide, gated) from the all-reduced sums and
  // the trial sums k_prox_pgd left in S_TR; then the next trial (k_prox_pgd, gated) and its
  // A@X (not gated: scratch slabs). A stop cancels everything behind it too: the next phase
  // starts from the gradient set the all-reduce in front of the decision completed.
  void dc_queue_comm(Roles& q, int64_t tag, bool first) {
    const int rz = (q.irg + 1) % kRes, rpt = (q.irg + 2) % kRes, rp = (q.irg + 3) % kRes;
    const T* xs[3] = {X_[q.iz], X_[q.ipt], X_[q.ip]};
    T* rs[3] = {R_[rz], R_[rpt], R_[rp]};
    if (first && !ax_queued_) {
      if (smode_ == 1) cand_ax(xs);
      else spec_ax(2, xs);
    }
    dc_gate_ = dc_abort_;
    const int ns = nset(q.gset);
    residuals(2, xs, rs, S_RT, X_[q.ip], scal_ + S_TR + 3, nullptr, 0.0, nullptr, tail(ns), true,
              false, emode_);
    const std::pair<const T*, int> g = gradient(R_[rpt], ns, 2);   // (one GPU: A^T r's slabs)
    const int64_t slot = (tag % kCtlMaxBatch) * kCtlRec;
    launch_ctl_decide(dc_make_ctl(tag), tail(ns), dc_ring_dev_ + slot,
                      reinterpret_cast<unsigned*>(dc_ring_dev_ + slot + kCtlRec - 1), (unsigned)tag, st_);
    check_launch();
    launch_prox_pgd<T>(X_[q.ipt], g.first, g.second, g.first != Gs_[ns] ? Gs_[ns] : nullptr, X_[q.if1],
                       X_[q.if2], X_[q.iz], n_, l_, O_.alpha0, mu_, O_.thres, red(S_TR), st_, Pub{}, ezf());
    check_launch();
    const T* sx[3] = {X_[q.iz], X_[q.if2], X_[q.if1]};   // [z | p_thr | p] of that trial
    if (smode_ == 1) cand_ax(sx);
    else spec_ax(2, sx);
    dc_gate_ = nullptr;
    q.irg = rpt;
    const int ox = q.ix, oxt = q.ixt;
    q.ix = q.ip; q.ixt = q.ipt; q.ip = q.if1; q.ipt = q.if2;
    q.if1 = ox; q.if2 = oxt;
    q.gset = ns;
  }
  void dc_queue(Roles& q, int64_t tag) {
    const int rz = (q.irg + 1) % kRes, rpt = (q.irg + 2) % kRes, rp = (q.irg + 3) % kRes;
    const T* xs[3] = {X_[q.iz], X_[q.ipt], X_[q.ip]};
    T* rs[3] = {R_[rz], R_[rpt], R_[rp]};
    dc_gate_ = dc_abort_;
    dc_ctl_ = dc_make_ctl(tag);
    const int64_t slot = (tag % kCtlMaxBatch) * kCtlRec;
    residuals(2, xs, rs, S_RT, X_[q.ip], scal_ + S_TR + 3, nullptr, 0.0, nullptr, nullptr, false,
              false, emode_);
    dc_ctl_ = Ctl{};
    dc_pass_ = 1 + (int)(tag % 0x3FFFFFFF);
    dc_pub_ = Pub{};
    dc_pub_.s = dc_rec_ + slot;
    dc_pub_.ns = 11;
    dc_pub_.host = dc_ring_dev_ + slot;
    dc_pub_.host_seq = reinterpret_cast<unsigned*>(dc_ring_dev_ + slot + kCtlRec - 1);
    dc_pub_.seq = (unsigned)tag;
    atr_prox(R_[rpt], nset(q.gset), X_[q.ipt], q.if1, q.if2, q.iz, O_.alpha0);
    dc_pub_ = Pub{};
    dc_pass_ = 0;
    dc_gate_ = nullptr;
    // the roles after an accepted first trial (proxgd_accept + proxgd_spec_rotate + use_gset)
    q.irg = rpt;
    const int ox = q.ix, oxt = q.ixt;
    q.ix = q.ip; q.ixt = q.ipt; q.ip = q.if1; q.ipt = q.if2;
    q.if1 = ox; q.if2 = oxt;
    q.gset = nset(q.gset);
  }
  const double* dc_wait(int64_t tag) {
    const double* rec = dc_ring_ + (tag % kCtlMaxBatch) * kCtlRec;
    volatile const unsigned* tp = reinterpret_cast<const unsigned*>(rec + kCtlRec - 1);
    const unsigned want = (unsigned)tag;
    uint64_t spins = 0;
    auto t0 = std::chrono::steady_clock::time_point{};
    prog_wait_.store(2, std::memory_order_relaxed);
    while (*tp != want) {
      __builtin_ia32_pause();
      if ((++spins & 0xFFFFF) == 0) {
        if (spins == 0x100000) t0 = std::chrono::steady_clock::now();
        else stalled_wait(t0, [&] { return *tp == want; }, "device-controlled batch: decision record");
      }
    }
    prog_wait_.store(0, std::memory_order_relaxed);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return rec;
  }
  void dc_run() {
    // iterations from here (this one is recorded): to the phase's maxit, max_total_iters and
    // the steps run() may still take
    int64_t budget = O_.maxit - inner_ + 1;
    if (O_.max_total_iters > 0) budget = std::min<int64_t>(budget, O_.max_total_iters - k_ + 1);
    budget = std::max<int64_t>(1, std::min<int64_t>(budget, step_room_));
    ++syncs_;   // the host's one blocking read per batch is this batch's records
    launch_ctl_seed(dc_state_, dc_abort_, gx_, f_cur_, s_cur_, (double)stable_, st_);
    check_launch();
    Roles q{ix_, ixt_, ip_, ipt_, if1_, if2_, iz_, irg_, spec_set_};
    const int64_t tag0 = dc_tag_;
    int64_t queued = 0;
    const int64_t w = std::min<int64_t>(dc_window_, budget);
    auto push = [&]() {   // tags are never reused: dc_tag_ = the last one queued
      dc_tag_ = tag0 + 1 + queued++;
      if (comm_ || unfused_spec_) dc_queue_comm(q, dc_tag_, queued == 1);
      else dc_queue(q, dc_tag_);
    };
    while (queued < w) push();
    int prev = 0;
    for (int64_t d = 0; d < budget; ++d) {
      if (d > 0) {
        record(f_cur_, s_cur_);
        const bool stop = stop_rule();
        if (stop != (prev == 1))
          throw Error{GLX_E_STATE, "device-controlled batch: stop rule differs from the host's"};
        if (stop) {
          // With a communicator the stopping decision cancelled the next trial (its gated
          // k_prox_pgd and everything behind it), which proxgd_spec_rotate declared ready: keep
          // its gradient set (the all-reduce in front of the decision completed) but never its
          // trial, even where the next phase's mu equals this one's (mu0 = 0).
          if (comm_ || unfused_spec_) {
            spec_trial_mu_ = NAN;
            ax_queued_ = false;
          }
          prof_drop_from(tag0 + d + 1);   // the segments behind the stopping decision
          end_phase(true);
          return;
        }
      }
      const double* rec = dc_wait(tag0 + 1 + d);
      ++record_waits_;
      if (queued < budget) push();
      for (int i = 0; i < 4; ++i) hs_[S_RT + i] = rec[i];
      for (int i = 0; i < 6; ++i) hs_[S_TR + i] = rec[4 + i];
      const int code = (int)rec[10];
      spec_trial_ready_ = false;   // iteration start: the speculated gradient set
      use_gset(spec_set_);
      const int rpt = (irg_ + 2) % kRes;
      const double t = O_.alpha0;
      const double gz = 0.5 * hs_[S_RT];
      const bool acc = gz <= gx_ - t * hs_[S_TR + 0] + 0.5 * t * hs_[S_TR + 1];
      if (acc != (code != 2))
        throw Error{GLX_E_STATE, "device-controlled batch: Armijo decision differs from the host's"};
      stats_[7] += 1;
      if (!acc) {   // everything queued behind this decision was cancelled on the device
        prof_drop_from(tag0 + 1 + d);
        spec_on_ = false;
        ax_queued_ = false;
        proxgd_trials({G_, 1}, true, t * O_.ls_coeff, 1);
        return;
      }
      spec_on_ = true;
      proxgd_accept(rpt, false);
      proxgd_spec_rotate();
      prev = code;
    }
    // with a communicator the last segment queued the next trial's A@X
    ax_queued_ = comm_ != nullptr || unfused_spec_;
  }

  // A^T r fused with a ProxGD trial at x (gradient set `set`, outputs X_[op], X_[opt], X_[oz]).
  // With a communicator: A^T r, the all-reduce (also summing tail_n deferred residual sums of
  // the set's tail), the scalar packet if pub_seq (so the host reads those sums while the trial
  // runs), then k_prox_pgd — the same arithmetic as the fused epilogue.
  // pub_out (communicator): the packet is returned for the caller's next launch to carry
  // instead of riding k_prox_pgd.
  void atr_prox(const T* r, int set, const T* x, int op, int opt, int oz, double t, int tail_n = 0,
                unsigned* pub_seq = nullptr, Pub* pub_out = nullptr) {
    const double* extra = tail_n ? tail(set) : nullptr;
    if (comm_ || unfused_spec_) {
      const std::pair<const T*, int> g = gradient(r, set, tail_n);
      Pub pb;
      if (pub_seq && pub_out) *pub_out = make_pub(extra, pub_seq);
      else if (pub_seq && attach_ok_) pb = make_pub(extra, pub_seq);
      else if (pub_seq) *pub_seq = post_readback(extra);
      // (one GPU: g is A^T r's slabs; the trial stores their sum as the set's G for retrials)
      launch_prox_pgd<T>(x, g.first, g.second, g.first != Gs_[set] ? Gs_[set] : nullptr, X_[op], X_[opt],
                         X_[oz], n_, l_, t, mu_, O_.thres, red(S_TR, dc_pass_), st_, pb, ezf());
      check_launch();
      ptr_ = Pend{};   // S_TR holds this trial's sums
      return;
    }
    Pub pb = dc_pub_;   // without a communicator pub_seq is only passed when attaching
    if (pub_seq) pb = make_pub(extra, pub_seq);
    hipEvent_t e0 = prof_begin(1);
    // in a device-controlled batch this speculative kernel also runs when the decision before it
    // stops the phase (abort = that decision's tag): the next phase starts from its gradient, as
    // on the host path; the speculative kernels queued after it do not run
    Red rd = red(S_TR, dc_pass_);
    // its trial sums stay partials (the other buffer than the one pb may reduce) when the packet
    // that needs them is carried by a later speculative kernel: this one's own trial is the next
    // iteration's (pub_seq), or the caller's batch is carried (carry_)
    const bool dtr = defer_ && (pub_seq != nullptr || carry_);
    if (dtr) {
      tb_ ^= 1;
      rd.part = tpart_[tb_];
      rd.parts_only = 1;
    }
    launch_atr_prox<T>(plan_, A_, r, Gs_[set], x, X_[op], X_[opt], X_[oz], t, mu_, O_.thres,
                       rd, st_, pb, Gps_[set], pcnt_, ezf());
    check_launch();
    ptr_ = dtr ? Pend{tpart_[tb_], atr_prox_slots(plan_, pb.host != nullptr), 6, 0x8u, scal_ + S_TR} : Pend{};
    prof_end(1, e0);
    ++atr_calls_;
  }

  // ------------------------------------------------------------------ FProxGD / FGD
  // Between iterations: X_[ix_] = x_k, X_[iv_] = v_k; when y_ready_, X_[iy_] = y of the next
  // iteration (formed by the accepted trial, bit-identical to :136/:139) and R_[iry_] = A y - b.
  void iter_fista(bool smooth) {
    if (!f_known_) {
      objective_of(X_[ix_]);
      f_cur_ = 0.5 * hs_[S_RO] + P_.mu0 * hs_[S_XRN];
      s_cur_ = hs_[S_RO + 3] / (double)nl_;
      f_known_ = true;
    }
    record(f_cur_, s_cur_);
    if (stop_rule()) { end_phase(true); return; }
    const double theta = 2.0 / (double)(inner_ + 1);       // gl_FProxGD_primal.py:138
    const double theta_next = 2.0 / (double)(inner_ + 2);
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    const double t0 = ls ? tk_ : schedule(inner_);
    if (fshard_) { iter_fista_shard(theta, theta_next); return; }
    const bool fuse = fused_fista_ok_ && !smooth;
    if (fsplit_ && ls && kslot_ < 0 && dense_left_ == 0) fista_split_prologue();
    if (!smooth && fista_dc_ready(t0, theta)) { fista_dc_run(); return; }
    // first trial: from the previous iteration's speculative fused kernel, fused into this
    // iteration's A^T r, or (FGD / unfusable plans) the gradient and k_fista_trial
    std::pair<const T*, int> g{nullptr, 0};
    bool first_done = false;
    if (spec_trial_ready_) {   // only ever set after an accepted trial: y and A y - b are ready
      spec_trial_ready_ = false;
      use_gset(spec_set_);
      g = {G_, 1};
      first_done = spec_trial_mu_ == mu_ && spec_trial_t_ == t0 && spec_trial_theta_ == theta;
    } else {
      if (!y_ready_) {
        launch_thr_axpby<T>(X_[ix_], X_[iv_], X_[iy_], nl_, O_.thres, 1.0 - theta, theta, st_);
        check_launch();
        residual1(X_[iy_], R_[iry_], S_RG);               // g(y) and the gradient residual
        gy_pending_ = true;
      }
      if (fuse) {
        carry_ = want_spec(0);
        atr_fista(R_[iry_], gset_, X_[iy_], X_[ix_], ic_, ivn_, iyn_, t0, theta, theta_next);
        carry_ = false;
        g = {G_, 1};
        first_done = true;
      } else {
        g = take_gradient(R_[iry_]);
      }
    }
    fista_trials(g, first_done, t0, 0, theta, theta_next, smooth);
  }

  // The backtracking search from trial it0 (it0 = 1: the first trial was rejected by a
  // device-side decision, fista_dc_run; t0 is then already tk * ls_coeff), or the untested
  // step, and the update (x_k, v_k, y and the split-candidate bookkeeping).
  void fista_trials(std::pair<const T*, int> g, bool first_done, double t0, int it0, double theta,
                    double theta_next, bool smooth) {
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    const bool fuse = fused_fista_ok_ && !smooth;
    const T* y = X_[iy_];
    if (smooth) {                                         // G = A^T r + mu y / sqrt(|y_i|^2 + d^2)
      launch_fgd_grad<T>(y, g.first, g.second, G_, n_, l_, mu_, O_.delta, red(S_REGY), st_);
      check_launch();
      g = {G_, 1};
    }
    const int rc = (iry_ + 1) % kRes, ryn = (iry_ + 2) % kRes;
    double t;
    bool accepted = false, spec_trial = false;
    auto trial = [&](double tt, bool first) {
      launch_fista_trial<T>(!smooth, y, first ? g.first : G_, first ? g.second : 1,
                            (first && g.first != G_) ? G_ : nullptr, X_[ix_], X_[ic_], X_[ivn_],
                            X_[iyn_], n_, l_, tt, mu_, O_.thres, theta, theta_next, O_.delta,
                            red(S_TR), st_, Pub{}, fec(), fzf());
      check_launch();
      ptr_ = Pend{};   // S_TR holds this trial's sums
    };
    const int i_rn = smooth ? 3 : 2, i_max = smooth ? 4 : 3;
    bool fs_batch = false;
    if (ls) {
      t = t0;
      for (int it = it0; it < O_.ls_maxit; ++it) {
        if (!(it == 0 && first_done)) trial(t, it == 0);
        const T* xs[3] = {X_[ic_], X_[iyn_], nullptr};
        T* rs[3] = {R_[rc], R_[ryn], nullptr};
        unsigned seq = 0;
        const bool spec = want_spec(it);
        const bool merge = spec && fuse && merge_tail();
        const bool late_pub = merge || (spec && fuse && attach_ok_ && comm_ == nullptr);
        fs_batch = fsplit_ && kslot_ >= 0 && dense_left_ == 0;
        carry_ = late_pub;
        if (fs_batch) {   // A xc dense, A e_c gathered, A y_next by linearity
          fista_split_batch(R_[ryn], theta, theta_next, S_RT, X_[ic_], scal_ + S_TR + i_max,
                            late_pub ? nullptr : &seq, merge ? tail(nset(gset_)) : nullptr);
        } else {
          residuals(2, xs, rs, S_RT, X_[ic_], scal_ + S_TR + i_max, nullptr, 0.0,   // A @ [x | y_next]
                    late_pub ? nullptr : &seq, merge ? tail(nset(gset_)) : nullptr);
        }
        carry_ = false;
        std::pair<const T*, int> sg;
        if (spec && fuse) {
          // the next iteration's gradient at y_next and its first trial (t, theta' = theta_next)
          atr_fista(R_[ryn], nset(gset_), X_[iyn_], X_[ic_], ff1_, ff2_, ff3_, t, theta_next,
                    2.0 / (double)(inner_ + 3), merge ? 2 : 0, late_pub ? &seq : nullptr);
          spec_trial = true;
        } else if (spec) {
          sg = gradient(R_[ryn], nset(gset_));   // gradient at the next y
        }
        wait_readback(seq);
        if (gy_pending_) { gy_sq_ = hs_[S_RG]; gy_pending_ = false; }
        double gy = 0.5 * gy_sq_, gxc = 0.5 * hs_[S_RT];
        if (smooth) {
          gy = gy + mu_ * hs_[S_REGY];
          gxc = gxc + mu_ * hs_[S_TR + 2];
        }
        if (gxc <= gy + hs_[S_TR + 0] + hs_[S_TR + 1] / (2 * t)) {
          accepted = true;
          if (spec && !spec_trial) { spec_ready_ = true; spec_g_ = sg; spec_set_ = nset(gset_); }
          spec_on_ = (it == 0);
          break;
        }
        spec_trial = false;
        spec_on_ = false;
        t *= O_.ls_coeff;
      }
      if (!accepted) trial(t, false);
    } else {
      t = t0;
      if (!first_done) trial(t, true);
    }
    fista_update(accepted, spec_trial, t, fs_batch, theta_next, ryn, i_rn);
  }

  // After the search: x_k <- x, v_k <- v (:145, :147), y <- y_next; the packet (hs_) holds the
  // last trial's sums. spec_trial: the speculative fused kernel left the next first trial.
  void fista_update(bool accepted, bool spec_trial, double t, bool fs_batch, double theta_next,
                    int ryn, int i_rn, int trs = S_TR) {
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    if (spec_trial) {   // the speculative outputs become the next iteration's trial buffers
      const int ox = ix_, ov = iv_, oy = iy_;
      ix_ = ic_; iv_ = ivn_; iy_ = iyn_;
      ic_ = ff1_; ivn_ = ff2_; iyn_ = ff3_;
      ff1_ = ox; ff2_ = ov; ff3_ = oy;
      spec_trial_ready_ = true;
      spec_set_ = nset(gset_);
      spec_trial_mu_ = mu_;
      spec_trial_t_ = t;
      spec_trial_theta_ = theta_next;
    } else {
      std::swap(ix_, ic_);
      std::swap(iv_, ivn_);
      std::swap(iy_, iyn_);
    }
    tk_ = t;
    kslot_ = (accepted && fs_batch) ? (kslot_ + 1) % 3 : -1;
    if (fsplit_ && ls) {
      split_hist_.push_back(fs_batch ? hs_[S_RT + 2] : -1.0);
      if (fs_batch) {
        stats_[3] += 1;
        stats_[5] += hs_[S_RT + 2];
        if (accepted && hs_[S_RT + 2] > nnz_budget_) dense_left_ = kFistaDenseRun;
      } else {
        stats_[4] += 1;
        if (dense_left_ > 0) --dense_left_;
      }
    }
    if (accepted) {
      iry_ = ryn;
      gy_sq_ = hs_[S_RT + 1];
      y_ready_ = true;
      f_cur_ = 0.5 * hs_[S_RT] + P_.mu0 * hs_[trs + i_rn];   // A x exact: same x as recorded
      s_cur_ = hs_[S_RT + 3] / (double)nl_;
      f_known_ = true;
    } else {
      y_ready_ = false;
      f_known_ = false;
    }
  }

  // ------------------------------------------------------------------ row-sharded FProxGD
  // (round 6; gl_FProxGD_primal.py:138-147 row-sharded). Per trial on
  // every rank: k_fista_trial on this rank's n / G rows of y and the reduce-scattered gradient
  // (xc's rows and the four trial sums as workgroup partials into this rank's chunk); one RCCL
  // group all-gathers xc's rows and every rank's chunk; k_fista_split re-derives v_next and y_next
  // of every row from the gathered xc (fista_row's arithmetic) and combines the sums in rank
  // order; A @ [xc | y_next] over this rank's rows of A and its finalize (sums into the chunk, the
  // count over this rank's rows of xc). As iter_proxgd_shard, the next gradient and first trial
  // are queued speculatively behind the trial (their exchange carries its residual sums) and the
  // packet rides the next trial's dense pass. Host control only (see fista_shard_ranks).
  void fshard_trial(int ix, int iy, const T* G, int oc, int ovn, int oyn, double t, double theta,
                    double theta_next) {
    const int64_t o = srow0_ * l_;
    Red rd = red_to(scal_ + S_TR);
    rd.part = blk_own() + kShardPartOff;
    rd.parts_only = 1;
    launch_fista_trial<T>(true, X_[iy] + o, G + o, 1, nullptr, X_[ix] + o, X_[oc] + o, X_[ovn] + o,
                          X_[oyn] + o, srows_, l_, t, mu_, O_.thres, theta, theta_next, O_.delta, rd, st_,
                          Pub{}, nullptr, nullptr);
    check_launch();
  }
  void fshard_derive(int ix, int oc, int ovn, int oyn, double theta, double theta_next, const ShardPub& sp) {
    launch_fista_split<T>(X_[oc], X_[ix], X_[ovn], X_[oyn], nl_, O_.thres, theta, theta_next, sp, st_);
    check_launch();
  }
  void iter_fista_shard(double theta, double theta_next) {
    const bool ls = O_.step_type == GLX_STEP_LINE_SEARCH && O_.ls_maxit > 0;
    const double t0 = ls ? tk_ : schedule(inner_);
    bool first_done = false;
    if (spec_trial_ready_) {   // the previous iteration's speculated trial (its sums in tr_slot_)
      spec_trial_ready_ = false;
      use_gset(spec_set_);
      first_done = spec_trial_mu_ == mu_ && spec_trial_t_ == t0 && spec_trial_theta_ == theta;
      if (!first_done) ax_queued_ = false;
    } else {
      if (!y_ready_) {
        launch_thr_axpby<T>(X_[ix_], X_[iv_], X_[iy_], nl_, O_.thres, 1.0 - theta, theta, st_);
        check_launch();
        residual1(X_[iy_], R_[iry_], S_RG);   // g(y): its sums all-reduced (8 B)
        gy_pending_ = true;
      }
      shard_gradient(R_[iry_], gset_);
    }
    const int rc = (iry_ + 1) % kRes, ryn = (iry_ + 2) % kRes;
    auto trial = [&](double tt) {
      fshard_trial(ix_, iy_, G_, ic_, ivn_, iyn_, tt, theta, theta_next);
      shard_exchange(ic_);
      fshard_derive(ix_, ic_, ivn_, iyn_, theta, theta_next, shard_pub(1, tr_slot_, nullptr));
    };
    double t = t0;
    bool accepted = false, spec_trial = false;
    if (ls) {
      for (int it = 0; it < O_.ls_maxit; ++it) {
        if (!(it == 0 && first_done)) trial(t);
        const T* xs[3] = {X_[ic_], X_[iyn_], nullptr};
        T* rs[3] = {R_[rc], R_[ryn], nullptr};
        const bool skip_ax = it == 0 && first_done && ax_queued_;
        ax_queued_ = false;
        shard_fin(2, xs, rs, X_[ic_], scal_ + tr_slot_ + 3, skip_ax);
        unsigned seq = 0;
        if (want_spec(it)) {
          // the next iteration's gradient at y_next and its first trial (t, theta_next and the one
          // after), into the other gradient set, the spare buffers and the other trial slot
          const int ns = nset(gset_);
          const int ot = tr_other();
          const double thnn = 2.0 / (double)(inner_ + 3);
          shard_gradient(R_[ryn], ns);
          fshard_trial(ic_, iyn_, Gs_[ns], ff1_, ff2_, ff3_, t, theta_next, thnn);
          shard_exchange(ff1_);
          fshard_derive(ic_, ff1_, ff2_, ff3_, theta_next, thnn, shard_pub(3, ot, nullptr));
          const T* sx[3] = {X_[ff1_], X_[ff3_], nullptr};
          const bool carry = spin_readback_ && attach_ok_ && ax_pub_ok(plan_, 2);
          Pub pb;
          if (carry) pb = make_pub(nullptr, &seq);
          else seq = post_readback();
          spec_ax(2, sx, pb);
          ax_queued_ = true;
          spec_trial = true;
        } else {
          shard_exchange(-1);
          launch_shard_combine(shard_pub(2, tr_slot_, nullptr), st_);
          check_launch();
          seq = post_readback();
        }
        wait_readback(seq);
        if (gy_pending_) { gy_sq_ = hs_[S_RG]; gy_pending_ = false; }
        const double gy = 0.5 * gy_sq_, gxc = 0.5 * hs_[S_RT];
        if (shard_model_ || gxc <= gy + hs_[tr_slot_ + 0] + hs_[tr_slot_ + 1] / (2 * t)) {
          accepted = true;
          spec_on_ = (it == 0);
          break;
        }
        spec_trial = false;
        spec_on_ = false;
        ax_queued_ = false;   // the speculated trial and its A@X are dropped
        t *= O_.ls_coeff;
      }
      if (!accepted) trial(t);   // the untested last step
    } else if (!first_done) {
      trial(t);
    }
    fista_update(accepted, spec_trial, t, false, theta_next, ryn, 2, tr_slot_);
    if (spec_trial) tr_slot_ = tr_other();
  }

  // ------------------------------------------------------------------ device-controlled FProxGD
  // SURVEY 8f row 2 for FISTA (round 3), the counterpart of dc_run. In the speculative steady
  // state (the previous first trial accepted, the step t unchanged, theta = 2/(k+1) known ahead)
  // every iteration launches the same kernels on rotating roles: the trial's batch (A@[xc |
  // y_next] and its finalize, or the split-candidate A xc + A e_c gather and k_finalize_fista),
  // then the fused A^T r at y_next + the next first trial (k_atr_fista). The backtracking test
  // (gl_FProxGD_primal.py:92-97), the next record and the stop rule (:127-134) run in the
  // finalize's last block (ctl_decide, mode 1); with a communicator in k_ctl_decide behind the
  // gradient all-reduce that carries the trial's residual sums, followed by k_fista_trial. A
  // gathered batch whose nnz(e_c) exceeds the budget ends the device batch (code 3): the host
  // path then runs kFistaDenseRun dense batches, which device control queues again (each batch
  // at most until the A thr(x_k) restore). The host re-derives every decision from the records
  // and checks it; results are bit-identical to host control.
  struct FRoles { int ix, iv, iy, ic, ivn, iyn, f1, f2, f3, iry, gset, ks; };
  bool fista_dc_ready(double t0, double theta) const {
    return dc_window_ > 0 && method_ == GLX_FPROXGD && fused_fista_ok_ && spec_trial_ready_ &&
           y_ready_ && !gy_pending_ && spec_trial_mu_ == mu_ && spec_trial_t_ == t0 &&
           spec_trial_theta_ == theta && want_spec(0) && !(fsplit_ && kslot_ < 0 && dense_left_ == 0);
  }
  // one segment of a device-controlled FISTA batch; th = theta of the iteration, thn / thnn the
  // next two (the speculative trial's theta and theta_next)
  void fista_dc_queue(FRoles& q, int64_t tag, bool split, double t, double th, double thn,
                      double thnn) {
    const int rc = (q.iry + 1) % kRes, ryn = (q.iry + 2) % kRes;
    Ctl c = dc_make_ctl(tag);
    c.mode = 1;
    c.t = t;
    c.nnz_budget = split ? nnz_budget_ : -1.0;
    dc_gate_ = dc_abort_;
    const int ns = nset(q.gset);
    double* defer = comm_ ? tail(ns) : nullptr;
    if (split) {
      const T* xs[3] = {E_, X_[q.ic], nullptr};
      cand_ax(xs);
      launch_finalize_fista<T>(Pp_ + (size_t)gsplit_ * ml_, ax_split(plan_, 1), Pp_, gsplit_, B_,
                               R_[ryn], SXO_[q.ks], SXO_[(q.ks + 1) % 3], ml_, 1.0 - thn, thn, th,
                               X_[q.ic], nl_, scal_ + S_TR + 3, gather_counts(glists_, n_), gcount_n(),
                               defer ? red_to(defer) : red(S_RT), st_, comm_ ? Ctl{} : c);
      check_launch();
      q.ks = (q.ks + 1) % 3;
    } else {
      const T* xs[3] = {X_[q.ic], X_[q.iyn], nullptr};
      T* rs[3] = {R_[rc], R_[ryn], nullptr};
      if (!comm_) dc_ctl_ = c;
      residuals(2, xs, rs, S_RT, X_[q.ic], scal_ + S_TR + 3, nullptr, 0.0, nullptr, defer);
      dc_ctl_ = Ctl{};
    }
    if (comm_) {
      gradient(R_[ryn], ns, 2);
      const int64_t slot = (tag % kCtlMaxBatch) * kCtlRec;
      launch_ctl_decide(c, tail(ns), dc_ring_dev_ + slot,
                        reinterpret_cast<unsigned*>(dc_ring_dev_ + slot + kCtlRec - 1), (unsigned)tag, st_);
      check_launch();
      // the next first trial runs also behind a stop / budget decision (the host path needs it)
      launch_fista_trial<T>(true, X_[q.iyn], Gs_[ns], 1, nullptr, X_[q.ic], X_[q.f1], X_[q.f2],
                            X_[q.f3], n_, l_, t, mu_, O_.thres, thn, thnn, O_.delta,
                            red(S_TR, c.pass), st_, Pub{}, fec(), fzf());
      check_launch();
    } else {
      dc_pass_ = c.pass;
      dc_pub_ = Pub{};
      const int64_t slot = (tag % kCtlMaxBatch) * kCtlRec;
      dc_pub_.s = dc_rec_ + slot;
      dc_pub_.ns = 11;
      dc_pub_.host = dc_ring_dev_ + slot;
      dc_pub_.host_seq = reinterpret_cast<unsigned*>(dc_ring_dev_ + slot + kCtlRec - 1);
      dc_pub_.seq = (unsigned)tag;
      atr_fista(R_[ryn], ns, X_[q.iyn], X_[q.ic], q.f1, q.f2, q.f3, t, thn, thnn);
      dc_pub_ = Pub{};
      dc_pass_ = 0;
    }
    dc_gate_ = nullptr;
    q.iry = ryn;
    const int ox = q.ix, ov = q.iv, oy = q.iy;
    q.ix = q.ic; q.iv = q.ivn; q.iy = q.iyn;
    q.ic = q.f1; q.ivn = q.f2; q.iyn = q.f3;
    q.f1 = ox; q.f2 = ov; q.f3 = oy;
    q.gset = ns;
  }
  void fista_dc_run() {
    int64_t budget = O_.maxit - inner_ + 1;
    if (O_.max_total_iters > 0) budget = std::min<int64_t>(budget, O_.max_total_iters - k_ + 1);
    budget = std::max<int64_t>(1, std::min<int64_t>(budget, step_room_));
    const bool split = fsplit_ && kslot_ >= 0 && dense_left_ == 0;
    // dense batches: at most until the A thr(x_k) restore the host path runs after the last one
    if (fsplit_ && dense_left_ > 0) budget = std::min<int64_t>(budget, dense_left_);
    ++syncs_;   // the host's one drain point per batch (its records are read while it runs)
    launch_ctl_seed(dc_state_, dc_abort_, gy_sq_, f_cur_, s_cur_, (double)stable_, st_);
    check_launch();
    FRoles q{ix_, iv_, iy_, ic_, ivn_, iyn_, ff1_, ff2_, ff3_, iry_, spec_set_, kslot_};
    const int64_t tag0 = dc_tag_, in0 = inner_;
    const double t = tk_;
    int64_t queued = 0;
    const int64_t w = std::min<int64_t>(dc_window_, budget);
    auto push = [&]() {
      const int64_t d = queued;
      dc_tag_ = tag0 + 1 + queued++;
      fista_dc_queue(q, dc_tag_, split, t, 2.0 / (double)(in0 + d + 1), 2.0 / (double)(in0 + d + 2),
                     2.0 / (double)(in0 + d + 3));
    };
    while (queued < w) push();
    int prev = 0;
    for (int64_t d = 0; d < budget; ++d) {
      if (d > 0) {
        record(f_cur_, s_cur_);
        const bool stop = stop_rule();
        if (stop != (prev == 1))
          throw Error{GLX_E_STATE, "device-controlled batch: stop rule differs from the host's"};
        if (stop) {
          prof_drop_from(tag0 + d + 1);   // the segments behind the stopping decision
          end_phase(true);
          return;
        }
      }
      const double* rec = dc_wait(tag0 + 1 + d);
      ++record_waits_;
      if (queued < budget) push();
      for (int i = 0; i < 4; ++i) hs_[S_RT + i] = rec[i];
      for (int i = 0; i < 6; ++i) hs_[S_TR + i] = rec[4 + i];
      const int code = (int)rec[10];
      spec_trial_ready_ = false;
      use_gset(spec_set_);
      const double theta = 2.0 / (double)(inner_ + 1), theta_next = 2.0 / (double)(inner_ + 2);
      const double gy = 0.5 * gy_sq_, gxc = 0.5 * hs_[S_RT];
      const bool acc = gxc <= gy + hs_[S_TR + 0] + hs_[S_TR + 1] / (2 * t);
      if (acc != (code != 2))
        throw Error{GLX_E_STATE, "device-controlled batch: backtracking decision differs from the host's"};
      stats_[7] += 1;
      if (!acc) {   // everything behind this decision was cancelled on the device
        prof_drop_from(tag0 + 1 + d);
        spec_on_ = false;
        fista_trials({G_, 1}, true, t * O_.ls_coeff, 1, theta, theta_next, false);
        return;
      }
      spec_on_ = true;
      const bool trip = split && hs_[S_RT + 2] > nnz_budget_;
      if ((code == 3) != (trip && code != 1))
        throw Error{GLX_E_STATE, "device-controlled batch: nnz budget decision differs from the host's"};
      fista_update(true, true, t, split, theta_next, (iry_ + 2) % kRes, 2);
      prev = code;
      if (code == 3) {   // the batch behind was cancelled; dense batches follow
        prof_drop_from(tag0 + 2 + d);
        return;
      }
    }
  }

  // Split-candidate FProxGD. The batch of a trial needs A xc (the objective, exact) and
  // A y_next (the next gradient residual and g(y)). y_next = a1 thr(xc) + b1 v_next with
  // v_next = thr(x_k) + (xc - thr(x_k))/theta (fista_row) is linear in xc, e_c = xc - thr(xc)
  // and thr(x_k), so one dense source suffices:
  //   A y_next = a1 (A xc - A e_c) + b1 (A thr(x_k) + (A xc - A thr(x_k))/theta)
  // with A e_c gathered from the transposed copy of A over the rows the threshold touched
  // (cand_ax) and A thr(x_k) = the previous accepted trial's A xc - A e_c, kept in a ring of
  // three (x_k's, this trial's, the speculated next trial's). The regrouping changes A y_next at
  // the rounding level only (the GEMMs' own summation order does as much); A xc, hence the
  // recorded objective, is computed directly. Without a kept A thr(x_k) (first iteration, after
  // an untested step or finish) one dense pass restores it.
  //
  // The gather reads one m-vector of At per nonzero of e_c, so it beats the second dense source
  // only while nnz(e_c) stays below a fraction of n (gather bytes / A bytes = nnz / n). FISTA's
  // candidates can carry many small entries late in a phase: each gathered batch reports its
  // nnz, and above the budget (GLX_SPLIT_NNZ, a fraction of n, default 0.35) the next
  // kFistaDenseRun batches are the dense [xc | y_next] pair, then A thr(x_k) is restored and
  // the gather form tried again.
  static constexpr int kFistaDenseRun = 128;
  // the row form reads one At row per flagged row: its cost passes the dense second source's
  // (~0.7 of a pass at NS) near 0.65 n flagged rows
  static constexpr double kRowsBudget = 0.6;
  void fista_split_prologue() {
    T* scratch = X_[ff1_];   // free between iterations (the speculation's spare)
    launch_threshold<T>(X_[ix_], scratch, nl_, O_.thres, flag_, ++epoch_, st_);
    check_launch();
    const T* xs[3] = {scratch, nullptr, nullptr};
    spec_ax(1, xs);
    launch_sum_partials<T>(Pp_, ax_split(plan_, 1), SXO_[0], ml_, st_);
    check_launch();
    kslot_ = 0;
    stats_[6] += 1;
  }
  void fista_split_batch(T* ry, double theta, double theta_next, int slot, const T* cx,
                         const double* cmax, unsigned* pub_seq, double* defer) {
    const T* xs[3] = {E_, X_[ic_], nullptr};
    cand_ax(xs);
    Red rd = defer ? Red{part_, ticket_, defer} : red(slot);
    const bool dfin = defer_ && carry_ && pub_seq == nullptr && defer == nullptr;
    const bool dmax = cx != nullptr && ptr_.part != nullptr && cmax == ptr_.out + 3;
    if (dfin) {
      flush_fin_pending();
      rd.part = fpart_;
      rd.parts_only = 1;
    }
    launch_finalize_fista<T>(Pp_ + (size_t)gsplit_ * ml_, ax_split(plan_, 1), Pp_, gsplit_, B_, ry,
                             SXO_[kslot_], SXO_[(kslot_ + 1) % 3], ml_, 1.0 - theta_next,
                             theta_next, theta, cx, nl_, cmax, gather_counts(glists_, n_), gcount_n(),
                             rd, st_, Ctl{}, dmax ? ptr_.part : nullptr, dmax ? ptr_.np : 0,
                             dmax ? ptr_.nv : 4);
    check_launch();
    if (dfin)
      pfin_ = Pend{fpart_, finalize_fista_blocks(ml_, ax_split(plan_, 1), gsplit_, cx ? nl_ : 0), 4, 0u,
                   scal_ + slot};
    if (defer) return;
    if (comm_) comm_allreduce(comm_, scal_ + slot, 2, GLX_F64, st_);
    if (pub_seq != nullptr) *pub_seq = post_readback();
  }

  // A^T r fused with a FISTA trial at y (gradient set `set`; x_k = xk; outputs X_[oc], X_[ov],
  // X_[oy])
  // (with a communicator: as atr_prox, the trial as k_fista_trial after the all-reduce)
  void atr_fista(const T* r, int set, const T* yv, const T* xk, int oc, int ov, int oy, double t,
                 double theta, double theta_next, int tail_n = 0, unsigned* pub_seq = nullptr) {
    const double* extra = tail_n ? tail(set) : nullptr;
    if (comm_) {
      const std::pair<const T*, int> g = gradient(r, set, tail_n);
      Pub pb;
      if (pub_seq && attach_ok_) pb = make_pub(extra, pub_seq);
      else if (pub_seq) *pub_seq = post_readback(extra);
      launch_fista_trial<T>(true, yv, g.first, g.second, nullptr, xk, X_[oc], X_[ov], X_[oy], n_,
                            l_, t, mu_, O_.thres, theta, theta_next, O_.delta, red(S_TR), st_, pb,
                            fec(), fzf());
      check_launch();
      return;
    }
    Pub pb = dc_pub_;   // in a device-controlled batch: the decision record (fista_dc_queue)
    if (pub_seq) pb = make_pub(extra, pub_seq);
    hipEvent_t e0 = prof_begin(1);
    Red rd = red(S_TR, dc_pass_);
    const bool dtr = defer_ && (pub_seq != nullptr || carry_);   // (as atr_prox)
    if (dtr) {
      tb_ ^= 1;
      rd.part = tpart_[tb_];
      rd.parts_only = 1;
    }
    launch_atr_fista<T>(plan_, A_, r, Gs_[set], yv, xk, X_[oc], X_[ov], X_[oy], t, mu_, O_.thres,
                        theta, theta_next, rd, st_, pb, Gps_[set], pcnt_, fec(), fzf());
    check_launch();
    ptr_ = dtr ? Pend{tpart_[tb_], atr_prox_slots(plan_, pb.host != nullptr), 4, 0x8u, scal_ + S_TR} : Pend{};
    prof_end(1, e0);
    ++atr_calls_;
  }

  // ------------------------------------------------------------------ SGD / GD (no syncs)
  // Between iterations: X_[0] = x, X_[1] = thr(x) (:93), R_[0] = A x - b, R_[1] = A thr(x) - b,
  // fh_dev_[k_] = the objective of x (recorded on the device by the finalize kernel).
  double descent_mu_obj(int64_t phase) const {
    return method_ == GLX_GD ? P_.mu0 : mus_[std::min<int64_t>(phase, 2)];
  }
  void descent_residuals(int64_t phase) {
    const T* xs[3] = {X_[0], X_[1], nullptr};
    T* rs[3] = {R_[0], R_[1], nullptr};
    residuals(2, xs, rs, S_RO, nullptr, nullptr, fh_dev_ + k_, descent_mu_obj(phase));
  }
  // l = 1, one pass over A: the objective of x (recorded at fh[k]) and the slabs of the
  // gradient A^T (A thr(x) - b) (kernels_gemv.hip)
  void descent_pass(int64_t phase) {
    hipEvent_t e0 = prof_begin(0);
    launch_gemv_fused<T>(gemv_blocks_, A_, X_[0], X_[1], B_, gemv_slabs_, m_, n_,
                         comm_ ? nullptr : fh_dev_ + k_, descent_mu_obj(phase), scal_ + S_DRN,
                         red(S_RO), st_);
    check_launch();
    prof_end(0, e0);
    ++ax_calls_;
    ax_cols_ += 2;
    if (comm_) {
      comm_allreduce(comm_, scal_ + S_RO, 2, GLX_F64, st_);
      launch_record_f(scal_, S_RO, S_DRN, descent_mu_obj(phase), fh_dev_ + k_, 0, st_);
      check_launch();
    }
  }
  std::pair<const T*, int> descent_gradient() {
    if (gemv_blocks_ == 0) return gradient(R_[1]);
    launch_sum_cols<T>(gemv_slabs_, gemv_blocks_, G_, n_, st_);   // l = 1: n x l = n
    check_launch();
    if (comm_) comm_allreduce(comm_, G_, nl_, P_.dtype, st_);
    return {G_, 1};
  }
  void iter_descent() {
    const bool gd = (method_ == GLX_GD);
    if (!state_valid_) {
      launch_rownorm_max<T>(X_[0], n_, l_, red(S_DRN), st_);
      check_launch();
      launch_threshold<T>(X_[0], X_[1], nl_, O_.thres, flag_, ++epoch_, st_);
      check_launch();
      if (gemv_blocks_) descent_pass(phase_);
      else descent_residuals(phase_);
      state_valid_ = true;
    }
    ++k_;
    ++inner_;
    const std::pair<const T*, int> g = descent_gradient();
    const double alpha = (O_.step_type == GLX_STEP_FIXED || mu_ > P_.mu0) ? O_.alpha0 : schedule(inner_);
    launch_descent<T>(X_[0], X_[1], g.first, g.second, n_, l_, alpha, mu_, O_.thres, O_.delta,
                      gd ? 1 : 0, red(S_DRN), st_);
    check_launch();
    if (k_ % 100 == 0 && k_ / 100 <= fh_cap_ / 100 + 1) {   // sparsity_func(x) of the debug line (:99)
      launch_rownorm_max<T>(X_[0], n_, l_, red(S_SPX), st_);
      check_launch();
      launch_count_above<T>(X_[0], nl_, scal_ + S_SPX + 1, Red{part_, ticket_, sp100_ + k_ / 100}, st_);
      check_launch();
    }
    // next iteration's objective residual and gradient residual, one pass
    const int64_t next_phase = (inner_ >= O_.maxit) ? phase_ + 1 : phase_;
    if (gemv_blocks_) descent_pass(next_phase);
    else descent_residuals(next_phase);
  }

 public:
  // state (public for carve)
  glx_problem P_;
  glx_opts O_;
  hipStream_t st_;
  GemmPlan plan_{};
  glx_comm* comm_ = nullptr;
  bool ax_queued_ = false;     // the pending first trial's A@X is already queued (spec_ax)
  bool spec_ax_pub_ = true;    // GLX_SPEC_AX_PUB=0: the packet rides k_prox_pgd instead
  int64_t m_ = 0, n_ = 0, l_ = 0, nl_ = 0, ml_ = 0;
  const T* A_ = nullptr;
  const T* B_ = nullptr;
  T* X_[kBufs] = {};
  T* R_[kRes] = {nullptr, nullptr, nullptr, nullptr};
  T *G_ = nullptr, *Gp_ = nullptr, *Pp_ = nullptr;
  T* Gs_[kMaxGSets] = {};
  T* Gps_[kMaxGSets] = {};
  int nsets_ = 2;
  double *scal_ = nullptr, *part_ = nullptr, *fh_dev_ = nullptr;
  double *hs_ = nullptr, *hs_dev_ = nullptr;
  unsigned *hseq_ = nullptr, *hseq_dev_ = nullptr;
  unsigned* ticket_ = nullptr;
  unsigned* pcnt_ = nullptr;   // per-panel counters (fused A^T R with K splits)
  unsigned* zf_ = nullptr;     // per-row column masks of e (split-candidate mode)
  // row-sharded ProxGD (iter_proxgd_shard): this rank's rows [srow0_, srow0_ + srows_) of n,
  // sranks_ row blocks (cranks_ communicator ranks; they differ only in the timing model)
  bool shard_ = false, shard_model_ = false;
  bool fshard_ = false;        // round 6: row-sharded FProxGD (iter_fista_shard)
  int stv_ = 6;                // values per trial workgroup partial in the chunk (FProxGD: 4)
  int srank_ = 0, sranks_ = 1, cranks_ = 1;
  int64_t srow0_ = 0, srows_ = 0;
  int nbp_ = 0, nbf_ = 0;      // k_prox_pgd's workgroups on srows_ rows, the trial finalize's
  int schunk_ = 0;             // doubles per rank's chunk
  bool zskip_ = false;         // the gathered p serves as e (bitmap / list gathers)
  bool sderive_ = false;       // round 6: the speculative derive inside the dense pass (AxDerive)
  int64_t moff_ = 0;           // doubles into a rank's chunk: its row masks + column bitmaps (sderive_)
  double* blk_ = nullptr;      // kMaxShardRanks chunks of sums (kShardChunkMax doubles each)
  // deferred reductions (defer_, single GPU): the trial's and the finalize's pending partials
  bool defer_ = false;
  double* tpart_[2] = {nullptr, nullptr};
  double* fpart_ = nullptr;
  int tb_ = 0;
  Pend ptr_, pfin_;
  bool unfused_spec_ = false;  // one GPU, a plan without the fused trial: the communicator form
  bool carry_ = false;         // while queuing: the next packet rides the speculative kernel
  int tr_slot_ = S_TR;         // the packet slots of the current trial's sums
  T* At_ = nullptr;            // A^T (split-candidate gather form)
  void* glists_ = nullptr;     // the gather's per-column index lists of e
  int smode_ = 0, gsplit_ = 1;
  int gform_ = 0;              // A e: 0 bitmap gather, 1 k_at_rows, 2 lists + gather (gather_form)
  bool rows_form_ = false;     // gform_ == 1: A e by k_at_rows (round 5), gsplit_ slabs
  bool egat_ = false;          // round 6: A e inside the dense pass (launch_ax_egat), gsplit_ = its S
  double hyb_rows_ = 0.0;      // round 6: > 0: the fused form per trial from this many flagged rows
  double last_rows_ = 0.0;     // flagged rows of the last accepted trial
  bool qeg_ = false;           // the queued split-candidate A@X is the fused form (its finalize reads it)
  // the fused A e form for the next trial; its A e slabs (one per K split) in front of A p
  bool egat_now() const { return egat_ || (hyb_rows_ > 0.0 && last_rows_ >= hyb_rows_); }
  int gs_of(bool eg) const { return eg ? ax_split(plan_, 1) : gsplit_; }
  // entries of the gather counts the FISTA finalize sums: flagged rows per K range (row form) or
  // nonzeros per column (VALU gather)
  int gcount_n() const { return rows_form_ ? gsplit_ : (int)l_; }
  bool emode_ = false;         // split-candidate ProxGD: trials write e = p - p_thr, not z
  unsigned* ezf() const { return emode_ ? zf_ : nullptr; }
  // split-candidate FProxGD (iter_fista): trials also write e_c = xc - thr(xc) to E_ and its
  // row flags to zf_; SXO_[kslot_] = A thr(x_k) (kslot_ < 0: not known)
  bool fsplit_ = false;
  T* E_ = nullptr;
  T* SXO_[3] = {nullptr, nullptr, nullptr};
  int kslot_ = -1;
  double nnz_budget_ = 0;      // nnz(e_c) above which the dense batch is cheaper
  int dense_left_ = 0;         // dense batches before the gather form is tried again
  T* fec() const { return fsplit_ ? E_ : nullptr; }
  unsigned* fzf() const { return fsplit_ ? zf_ : nullptr; }
  int* flag_ = nullptr;
  // device-controlled ProxGD batches (dc_run)
  double* dc_state_ = nullptr;    // Ctl::state
  int* dc_abort_ = nullptr;       // 0 live, a decision's tag: stop at the next record, -1 rejected
  int dc_pass_ = 0;               // while queuing: the tag the speculative kernel also runs on
  double* dc_rec_ = nullptr;      // device decision records (Ctl::rec), kCtlMaxBatch slots
  Pub dc_pub_{};                  // while queuing: the record's hand-off, carried by atr_prox
  double* dc_ring_ = nullptr;     // host-mapped decision records
  double* dc_ring_dev_ = nullptr;
  int dc_window_ = 0;             // iterations in flight (0: off)
  int64_t dc_tag_ = 0;            // decision records issued
  int64_t step_room_ = INT64_MAX;
  const int* dc_gate_ = nullptr;  // while queuing a batch: the abort word the launches test
  Ctl dc_ctl_{};                  // while queuing a batch: the finalize's decision epilogue
  int64_t fh_cap_ = 0;
  // progress record for glx_session_progress (read by other threads): iterations, phase, what
  // the host is waiting on (0 nothing, 1 a scalar packet, 2 a decision record)
  std::atomic<int64_t> prog_k_{0};
  std::atomic<int> prog_phase_{0}, prog_wait_{0};
  double* sp100_ = nullptr;   // SGD/GD: count(|x| > 1e-6 max|x|) after every 100th iteration
  T* gemv_slabs_ = nullptr;
  int gemv_blocks_ = 0;

 private:
  int method_ = 0;
  bool use_sparsity_ = true, device_hist_ = false, spin_readback_ = true;
  unsigned seq_ = 0;
  bool attach_ok_ = true;
  hipEvent_t rb_event_ = nullptr;
  int epoch_ = 0;
  // buffer roles
  int ix_ = 0, iv_ = 1, iy_ = 2, ic_ = 3, ivn_ = 4, iyn_ = 5;   // FISTA
  int ff1_ = 6, ff2_ = 7, ff3_ = 8;                               // FISTA spares (speculation)
  int ixt_ = 1, ip_ = 2, ipt_ = 3, iz_ = 4, if1_ = 5, if2_ = 6;   // ProxGD (+ two spares)
  int irg_ = 0, iry_ = 0;
  bool state_valid_ = false, thr_from_trial_ = false, y_ready_ = false, gy_pending_ = false;
  // speculative gradient (take_gradient)
  int gset_ = 0, spec_set_ = 1;
  bool spec_on_ = true, spec_ready_ = false, spec_off_env_ = false;
  // ProxGD trial fused into A^T r (launch_atr_prox): fused_ok_ = the plan allows it; a
  // speculative fused kernel leaves G and the next iteration's first trial (t, mu) ready
  bool fused_ok_ = false, fused_fista_ok_ = false, spec_trial_ready_ = false;
  double spec_trial_mu_ = 0, spec_trial_t_ = 0, spec_trial_theta_ = 0;
  std::pair<const T*, int> spec_g_{nullptr, 0};
  double gx_ = 0, gy_sq_ = 0;
  // algorithm state
  int phase_ = 0;
  int64_t inner_ = 0, k_ = 0;
  int stable_ = 0;
  bool finished_ = false, f_known_ = false, rn_known_ = false;
  double mus_[3] = {0, 0, 0}, mu_ = 0, tk_ = 0;
  double f_cur_ = 0, s_cur_ = 0, fbest_ = 0, sp_cur_ = 0, sp_prev_ = 0;
  std::vector<double> fh_, fhb_, sp_hist_, trace_sp_;
  int64_t phase_start_[3] = {-1, -1, -1};
  int64_t phase_break_[3] = {0, 0, 0};
  double tt_ = 0;
  // syncs_: host readbacks the queue drains behind (the host decides before queuing more; one
  // per device-controlled batch); record_waits_: decision records read while the device keeps
  // later iterations queued (device-controlled batches)
  int64_t ax_calls_ = 0, ax_cols_ = 0, atr_calls_ = 0, syncs_ = 0, record_waits_ = 0;
  double stats_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  std::vector<double> split_hist_;
  struct EvSample { hipEvent_t a, b; int64_t tag; };
  std::vector<EvSample> ev_[3];
  int64_t prof_n_[3] = {0, 0, 0};
  std::vector<hipEvent_t> ev_pool_;
};

static size_t session_bytes(const glx_problem& P, const glx_opts& O) {
  const GemmPlan plan = session_plan(P, O);
  const int sm = split_mode(P, O);
  if (P.dtype == GLX_F64)
    return Session<double>::carve(P, O, plan, Session<double>::fh_capacity(P, O), sm, nullptr, nullptr);
  return Session<float>::carve(P, O, plan, Session<float>::fh_capacity(P, O), sm, nullptr, nullptr);
}

template <typename F>
static int guarded(F&& f) {
  try {
    f();
    return GLX_OK;
  } catch (const Error& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return GLX_E_STATE;
  } catch (...) {
    g_last_error = "unknown error";
    return GLX_E_STATE;
  }
}

// ---- single-kernel workspace: P slabs + Gp slabs + reduction scratch
struct KernelWs {
  void* pp; void* gp; double* part; unsigned* ticket; double* scal;
  void* rg_ws; double* rg_s; double* rg_g; int* rg_err;   // fused residual-gradient pass
  void* rg2_ws; double* rg2_g;                              // its l = 16 two-source form
  void* fr_slabs; void* fr_lists; void* fr_zf;              // glx_flagged_rows_product
};
static size_t kernel_ws(int es, const GemmPlan& p, void* base, KernelWs* out) {
  Carver c(base);
  // room for the largest split any variant of this shape plans (MFMA tiles, VALU)
  int64_t s_ax = 1, s_atr = 1;
  for (int v : {0, 3}) s_atr = std::max<int64_t>(s_atr, make_plan(es, p.m, p.n, p.l, v).atr_S);
  s_ax = std::max<int64_t>(max_ax_split(es, p.m, p.n, p.l), ax_split_max(p));
  s_atr = std::max<int64_t>(s_atr, p.atr_S);
  void* pp = c.take((size_t)es * p.m * p.l * s_ax * 3);
  void* gp = c.take((size_t)es * p.n * p.l * s_atr);
  double* part = static_cast<double*>(c.take(sizeof(double) * kMaxRedVals * kMaxBlocks));
  unsigned* ticket = static_cast<unsigned*>(c.take(kTicketBytes));
  double* scal = static_cast<double*>(c.take(sizeof(double) * NSCAL));
  void* rg_ws = nullptr;
  double *rg_s = nullptr, *rg_g = nullptr;
  int* rg_err = nullptr;
  if (resgrad_shape_ok(es, p.m, p.n, p.l)) {
    rg_ws = c.take(resgrad_ws_bytes(p.m, p.n));
    rg_s = static_cast<double*>(c.take(sizeof(double) * p.m * p.l));
    rg_g = static_cast<double*>(c.take(sizeof(double) * p.n * p.l * resgrad_groups(p.n)));
    rg_err = static_cast<int*>(c.take(256));
  }
  void* rg2_ws = nullptr;
  double* rg2_g = nullptr;
  if (resgrad2_shape_ok(es, p.m, p.n, p.l)) {
    rg2_ws = c.take(resgrad2_ws_bytes(p.n));
    rg2_g = static_cast<double*>(c.take(sizeof(double) * p.n * p.l * resgrad2_groups(p.n)));
    if (!rg_err) rg_err = static_cast<int*>(c.take(256));
  }
  // the flagged-row product (A e of the split-candidate trial): its slabs and lists / counts
  void* fr_slabs = nullptr;
  void* fr_lists = nullptr;
  void* fr_zf = nullptr;
  if (gather_ok(p.n, p.l)) {
    fr_slabs = c.take((size_t)es * p.m * p.l * std::max(1, gather_split(p.m, p.n)));
    fr_lists = c.take(gather_lists_bytes(p.n));
    fr_zf = c.take(zf_bytes(p.n));
  }
  if (out)
    *out = KernelWs{pp, gp, part, ticket, scal, rg_ws, rg_s, rg_g, rg_err, rg2_ws, rg2_g, fr_slabs, fr_lists,
                    fr_zf};
  return c.off + 256;
}

}  // namespace glx

// ============================================================================================
// C ABI
// ============================================================================================
using namespace glx;

struct glx_session {
  std::unique_ptr<SessionBase> impl;
};

extern "C" {

int glx_abi_version(void) { return GLX_ABI_VERSION; }

const char* glx_last_error(void) { return g_last_error.c_str(); }

int glx_default_opts(int method, glx_opts* o) {
  return guarded([&] {
    if (!o) throw Error{GLX_E_INVALID, "null opts"};
    std::memset(o, 0, sizeof(*o));
    o->thres = 1e-3;
    o->ls_maxit = 5;
    o->delta = 1e-3;
    switch (method) {
      case GLX_PROXGD:   // gl_ProxGD_primal.py:10-19
        o->maxit = 2500; o->step_type = GLX_STEP_LINE_SEARCH; o->alpha0 = 2e-3; o->ftol = 1e-6;
        o->stable_len_threshold = 70; o->ls_coeff = 0.9; break;
      case GLX_FPROXGD:  // gl_FProxGD_primal.py:10-19
        o->maxit = 1500; o->step_type = GLX_STEP_LINE_SEARCH; o->alpha0 = 1e-3; o->ftol = 1e-6;
        o->stable_len_threshold = 70; o->ls_coeff = 0.98; break;
      case GLX_SGD:      // gl_SGD_primal.py:10-18
        o->maxit = 2100; o->step_type = GLX_STEP_DIMINISHING; o->alpha0 = 1e-3; o->ftol = 1e-5;
        o->stable_len_threshold = 100; o->ls_coeff = 0.9; break;
      case GLX_GD:       // gl_GD_primal.py:10-19
        o->maxit = 2500; o->step_type = GLX_STEP_DIMINISHING; o->alpha0 = 1e-3; o->ftol = 1e-5;
        o->stable_len_threshold = 100; o->ls_coeff = 0.9; o->delta = 1e-3; break;
      case GLX_FGD:      // gl_FGD_primal.py:10-19
        o->maxit = 1500; o->step_type = GLX_STEP_LINE_SEARCH; o->alpha0 = 1e-3; o->ftol = 1e-6;
        o->stable_len_threshold = 70; o->ls_coeff = 0.98; o->delta = 1e-6; break;
      default: throw Error{GLX_E_INVALID, "unknown method"};
    }
  });
}

int glx_workspace_bytes(const glx_problem* prob, const glx_opts* opts, size_t* bytes) {
  return guarded([&] {
    validate(prob, opts);
    if (!bytes) throw Error{GLX_E_INVALID, "null bytes"};
    *bytes = session_bytes(*prob, *opts);
  });
}

int glx_session_create(glx_session** out, const glx_problem* prob, const glx_opts* opts,
                       void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!out) throw Error{GLX_E_INVALID, "null out"};
    *out = nullptr;
    validate(prob, opts);
    auto s = std::make_unique<glx_session>();
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (prob->dtype == GLX_F64)
      s->impl = std::make_unique<Session<double>>(*prob, *opts, workspace, workspace_bytes, st);
    else
      s->impl = std::make_unique<Session<float>>(*prob, *opts, workspace, workspace_bytes, st);
    *out = s.release();
  });
}

int glx_session_run(glx_session* s, int64_t max_steps, int64_t* done, int32_t* finished) {
  return guarded([&] {
    if (!s || !s->impl) throw Error{GLX_E_INVALID, "null session"};
    s->impl->run(max_steps, done, finished);
  });
}

int glx_session_finish(glx_session* s, glx_result* res) {
  return guarded([&] {
    if (!s || !s->impl) throw Error{GLX_E_INVALID, "null session"};
    s->impl->finish(res);
  });
}

int glx_session_kernel_time(glx_session* s, int kind, int64_t* launches, double* total_ms) {
  return guarded([&] {
    if (!s || !s->impl) throw Error{GLX_E_INVALID, "null session"};
    s->impl->kernel_time(kind, launches, total_ms);
  });
}

int glx_session_counters(glx_session* s, int64_t out[4]) {
  return guarded([&] {
    if (!s || !s->impl || !out) throw Error{GLX_E_INVALID, "null session/out"};
    s->impl->counters(out);
  });
}

int glx_session_progress(glx_session* s, int64_t out[4]) {
  return guarded([&] {
    if (!s || !s->impl || !out) throw Error{GLX_E_INVALID, "null session/out"};
    s->impl->progress(out);
  });
}

int glx_session_trace(glx_session* s, double* sparsity_after, int64_t cap, int64_t* n,
                      int64_t phase_info[6]) {
  return guarded([&] {
    if (!s || !s->impl) throw Error{GLX_E_INVALID, "null session"};
    s->impl->trace(sparsity_after, cap, n, phase_info);
  });
}

int glx_session_split_trace(glx_session* s, double* out, int64_t cap, int64_t* n) {
  return guarded([&] {
    if (!s || !s->impl) throw Error{GLX_E_INVALID, "null session"};
    const int64_t k = s->impl->split_trace(out, cap);
    if (n) *n = k;
  });
}

int glx_session_describe(glx_session* s, char* out, size_t cap) {
  return guarded([&] {
    if (!s || !s->impl || !out || cap == 0) throw Error{GLX_E_INVALID, "null session/out"};
    std::snprintf(out, cap, "%s", s->impl->describe().c_str());
  });
}

void glx_session_destroy(glx_session* s) { delete s; }

int glx_solve(const glx_problem* prob, const glx_opts* opts, void* workspace,
              size_t workspace_bytes, glx_result* res, void* stream) {
  if (opts != nullptr && opts->shard_model > 1) {   // a timing model is not a solve
    g_last_error = "opts.shard_model is a benchmark timing model whose iterates are not a solve; "
                   "glx_solve refuses it (use the session API, as bench.py does)";
    return GLX_E_INVALID;
  }
  glx_session* s = nullptr;
  int rc = glx_session_create(&s, prob, opts, workspace, workspace_bytes, stream);
  if (rc != GLX_OK) return rc;
  rc = glx_session_run(s, 0, nullptr, nullptr);
  if (rc == GLX_OK) rc = glx_session_finish(s, res);
  glx_session_destroy(s);
  return rc;
}

int glx_kernel_workspace_bytes(int dtype, int64_t m, int64_t n, int64_t l, size_t* bytes) {
  return guarded([&] {
    if (dtype != GLX_F32 && dtype != GLX_F64) throw Error{GLX_E_INVALID, "bad dtype"};
    if (m <= 0 || n <= 0 || l <= 0 || l > kMaxL || !bytes) throw Error{GLX_E_INVALID, "bad shape"};
    const int es = dtype == GLX_F64 ? 8 : 4;
    *bytes = kernel_ws(es, make_plan(es, m, n, l, 0), nullptr, nullptr);
  });
}

int glx_plan_describe(int dtype, int64_t m, int64_t n, int64_t l, char* out, size_t cap) {
  return guarded([&] {
    if (dtype != GLX_F32 && dtype != GLX_F64) throw Error{GLX_E_INVALID, "bad dtype"};
    if (m <= 0 || n <= 0 || l <= 0 || l > kMaxL || !out || cap == 0) throw Error{GLX_E_INVALID, "bad arguments"};
    const std::string d = describe_plan(make_plan(dtype == GLX_F64 ? 8 : 4, m, n, l, 0));
    std::snprintf(out, cap, "%s", d.c_str());
  });
}

static KernelWs kernel_setup(int dtype, int64_t m, int64_t n, int64_t l, void* ws, size_t wsb,
                             int variant, hipStream_t st, GemmPlan* plan) {
  if (dtype != GLX_F32 && dtype != GLX_F64) throw Error{GLX_E_INVALID, "bad dtype"};
  if (m <= 0 || n <= 0 || l <= 0 || l > kMaxL) throw Error{GLX_E_INVALID, "bad shape"};
  const int es = dtype == GLX_F64 ? 8 : 4;
  *plan = make_plan(es, m, n, l, variant);
  if (!ws || wsb < kernel_ws(es, *plan, nullptr, nullptr)) throw Error{GLX_E_WORKSPACE, "workspace too small"};
  if (reinterpret_cast<uintptr_t>(ws) & 255) throw Error{GLX_E_WORKSPACE, "workspace must be 256-byte aligned"};
  KernelWs k;
  kernel_ws(es, *plan, ws, &k);
  GLX_HIP(hipMemsetAsync(k.ticket, 0, kTicketBytes, st));
  return k;
}

int glx_residual(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* X,
                 const void* B, void* R, void* half_sumsq_dev, void* ws, size_t wsb, int variant,
                 void* stream) {
  return guarded([&] {
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, m, n, l, ws, wsb, variant, st, &p);
    Red r{k.part, k.ticket, k.scal};
    if (dtype == GLX_F64) {
      const double* xs[3] = {(const double*)X, nullptr, nullptr};
      double* rs[3] = {(double*)R, nullptr, nullptr};
      launch_ax<double>(p, 1, (const double*)A, xs, (double*)k.pp, nullptr, 0, st);
      launch_finalize_residual<double>((const double*)k.pp, p.ax_S, (const double*)B, 1, rs, m * l,
                                       nullptr, 0, 1, nullptr, 0, nullptr, nullptr, 0.0, nullptr, r, st);
    } else {
      const float* xs[3] = {(const float*)X, nullptr, nullptr};
      float* rs[3] = {(float*)R, nullptr, nullptr};
      launch_ax<float>(p, 1, (const float*)A, xs, (float*)k.pp, nullptr, 0, st);
      launch_finalize_residual<float>((const float*)k.pp, p.ax_S, (const float*)B, 1, rs, m * l,
                                      nullptr, 0, 1, nullptr, 0, nullptr, nullptr, 0.0, nullptr, r, st);
    }
    check_launch();
    if (half_sumsq_dev) {
      // 0.5 * sum: scale on device with a tiny record kernel (fh[0] = 0.5*s + 0*s)
      launch_record_f(k.scal, 0, 0, 0.0, static_cast<double*>(half_sumsq_dev), 0, st);
      check_launch();
    }
  });
}

int glx_residual_batch(int dtype, int64_t m, int64_t n, int64_t l, const void* A, int nsrc,
                       const void* const* X, const void* B, void* const* R, void* sumsq_dev,
                       void* ws, size_t wsb, int variant, void* stream) {
  return guarded([&] {
    if (nsrc < 1 || nsrc > 3 || !X || !R) throw Error{GLX_E_INVALID, "nsrc must be 1..3"};
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, m, n, l, ws, wsb, variant, st, &p);
    Red r{k.part, k.ticket, sumsq_dev ? static_cast<double*>(sumsq_dev) : k.scal};
    if (dtype == GLX_F64) {
      const double* xs[3] = {nullptr, nullptr, nullptr};
      double* rs[3] = {nullptr, nullptr, nullptr};
      for (int i = 0; i < nsrc; ++i) { xs[i] = (const double*)X[i]; rs[i] = (double*)R[i]; }
      launch_ax<double>(p, nsrc, (const double*)A, xs, (double*)k.pp, nullptr, 0, st);
      launch_finalize_residual<double>((const double*)k.pp, ax_split(p, nsrc), (const double*)B, nsrc, rs, m * l,
                                       nullptr, 0, 1, nullptr, 0, nullptr, nullptr, 0.0, nullptr, r, st);
    } else {
      const float* xs[3] = {nullptr, nullptr, nullptr};
      float* rs[3] = {nullptr, nullptr, nullptr};
      for (int i = 0; i < nsrc; ++i) { xs[i] = (const float*)X[i]; rs[i] = (float*)R[i]; }
      launch_ax<float>(p, nsrc, (const float*)A, xs, (float*)k.pp, nullptr, 0, st);
      launch_finalize_residual<float>((const float*)k.pp, ax_split(p, nsrc), (const float*)B, nsrc, rs, m * l,
                                      nullptr, 0, 1, nullptr, 0, nullptr, nullptr, 0.0, nullptr, r, st);
    }
    check_launch();
  });
}

int glx_gradient(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* R,
                 void* G, void* ws, size_t wsb, void* stream) {
  return guarded([&] {
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, m, n, l, ws, wsb, 0, st, &p);
    if (dtype == GLX_F64) {
      double* gp = p.atr_S > 1 ? (double*)k.gp : (double*)G;
      launch_atr<double>(p, (const double*)A, (const double*)R, gp, st);
      if (p.atr_S > 1) launch_sum_partials<double>(gp, p.atr_S, (double*)G, n * l, st);
    } else {
      float* gp = p.atr_S > 1 ? (float*)k.gp : (float*)G;
      launch_atr<float>(p, (const float*)A, (const float*)R, gp, st);
      if (p.atr_S > 1) launch_sum_partials<float>(gp, p.atr_S, (float*)G, n * l, st);
    }
    check_launch();
  });
}

int glx_flagged_rows_product(int dtype, int64_t m, int64_t n, int64_t l, const void* At,
                             const void* E, const uint32_t* row_masks, void* Y, int form,
                             void* ws, size_t wsb, void* stream) {
  return guarded([&] {
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, m, n, l, ws, wsb, 0, st, &p);
    if (!gather_ok(n, l) || k.fr_slabs == nullptr) throw Error{GLX_E_INVALID, "needs l in {16, 32}, n < 65536"};
    if (form < 0 || form > 2) throw Error{GLX_E_INVALID, "form must be 0 (MFMA rows), 1 (lists), 2 (bitmaps)"};
    if (form == 0 && !gather_rows_ok(m, n)) throw Error{GLX_E_INVALID, "the row form needs m % 64 == 0"};
    const int S0 = form == 0 ? gather_split(m, n) : 1;
    auto go = [&](auto* tag) {
      typedef std::remove_pointer_t<decltype(tag)> T;
      T* slabs = static_cast<T*>(k.fr_slabs);
      if (form == 0) {
        launch_at_rows<T>(static_cast<const T*>(At), static_cast<const T*>(E), row_masks, m, n, l, slabs,
                          k.fr_lists, st);
      } else if (form == 1) {
        launch_e_lists(row_masks, n, l, k.fr_lists, st);
        launch_at_gather<T>(static_cast<const T*>(At), static_cast<const T*>(E), m, n, l, slabs, k.fr_lists, st);
      } else {   // the masks copied into a zf-shaped buffer, its bitmaps built, then the gather
        unsigned* zf = static_cast<unsigned*>(k.fr_zf);
        GLX_HIP(hipMemcpyAsync(zf, row_masks, sizeof(unsigned) * n, hipMemcpyDeviceToDevice, st));
        launch_zf_bitmaps(zf, n, l, st);
        launch_at_gather_bm<T>(static_cast<const T*>(At), static_cast<const T*>(E), zf, m, n, l, slabs,
                               k.fr_lists, st);
      }
      launch_sum_partials<T>(slabs, S0, static_cast<T*>(Y), m * l, st);
    };
    if (dtype == GLX_F64) go(static_cast<double*>(nullptr));
    else go(static_cast<float*>(nullptr));
    check_launch();
  });
}

int glx_residual_gradient(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* X,
                          const void* B, void* R, void* G, void* ws, size_t wsb, int one_pass,
                          int* fused_out, void* stream) {
  return guarded([&] {
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, m, n, l, ws, wsb, 0, st, &p);
    const bool fused = one_pass != 0 && dtype == GLX_F64 && k.rg_ws != nullptr && resgrad_device_ok();
    if (fused_out) *fused_out = fused ? 1 : 0;
    if (fused) {
      resgrad_reset(k.rg_ws, m, n, st);
      GLX_HIP(hipMemsetAsync(k.rg_err, 0, sizeof(int), st));
      if (launch_resgrad((const double*)A, (const double*)X, (const double*)B, k.rg_s, k.rg_g, k.rg_ws,
                         1, m, n, k.rg_err, st)) {
        double* rs[3] = {(double*)R, nullptr, nullptr};
        launch_finalize_residual<double>(k.rg_s, 1, (const double*)B, 1, rs, m * l, nullptr, 0, 1,
                                         nullptr, 0, nullptr, nullptr, 0.0, nullptr,
                                         Red{k.part, k.ticket, k.scal}, st);
        launch_sum_partials<double>(k.rg_g, resgrad_groups(n), (double*)G, n * l, st);
        check_launch();
        // the one-pass result is valid only if no hand-off wait timed out: read the flag back
        // (this makes the one-pass call synchronous) and recompute with two passes otherwise
        int herr = 0;
        GLX_HIP(hipMemcpyAsync(&herr, k.rg_err, sizeof(int), hipMemcpyDeviceToHost, st));
        GLX_HIP(hipStreamSynchronize(st));
        if (herr == 0) return;
      }
      if (fused_out) *fused_out = 0;
    }
    const int es = dtype == GLX_F64 ? 8 : 4;
    (void)es;
    if (dtype == GLX_F64) {
      const double* xs[3] = {(const double*)X, nullptr, nullptr};
      double* rs[3] = {(double*)R, nullptr, nullptr};
      launch_ax<double>(p, 1, (const double*)A, xs, (double*)k.pp, nullptr, 0, st);
      launch_finalize_residual<double>((const double*)k.pp, p.ax_S, (const double*)B, 1, rs, m * l,
                                       nullptr, 0, 1, nullptr, 0, nullptr, nullptr, 0.0, nullptr,
                                       Red{k.part, k.ticket, k.scal}, st);
      double* gp = p.atr_S > 1 ? (double*)k.gp : (double*)G;
      launch_atr<double>(p, (const double*)A, (const double*)R, gp, st);
      if (p.atr_S > 1) launch_sum_partials<double>(gp, p.atr_S, (double*)G, n * l, st);
    } else {
      const float* xs[3] = {(const float*)X, nullptr, nullptr};
      float* rs[3] = {(float*)R, nullptr, nullptr};
      launch_ax<float>(p, 1, (const float*)A, xs, (float*)k.pp, nullptr, 0, st);
      launch_finalize_residual<float>((const float*)k.pp, p.ax_S, (const float*)B, 1, rs, m * l,
                                      nullptr, 0, 1, nullptr, 0, nullptr, nullptr, 0.0, nullptr,
                                      Red{k.part, k.ticket, k.scal}, st);
      float* gp = p.atr_S > 1 ? (float*)k.gp : (float*)G;
      launch_atr<float>(p, (const float*)A, (const float*)R, gp, st);
      if (p.atr_S > 1) launch_sum_partials<float>(gp, p.atr_S, (float*)G, n * l, st);
    }
    check_launch();
  });
}

int glx_residual_gradient2(int dtype, int64_t m, int64_t n, int64_t l, const void* A, const void* X0,
                           const void* X1, const void* B, void* R0, void* R1, void* G, void* ws,
                           size_t wsb, int one_pass, int* one_pass_ran, void* stream) {
  return guarded([&] {
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, m, n, l, ws, wsb, 0, st, &p);
    const bool fused = one_pass != 0 && dtype == GLX_F64 && k.rg2_ws != nullptr && resgrad2_device_ok();
    if (one_pass_ran) *one_pass_ran = fused ? 1 : 0;
    if (fused) {
      resgrad2_reset(k.rg2_ws, n, st);
      GLX_HIP(hipMemsetAsync(k.rg_err, 0, sizeof(int), st));
      double* pp = static_cast<double*>(k.pp);   // two slabs: A X0, A X1
      launch_resgrad2((const double*)A, (const double*)X0, (const double*)X1, (const double*)B, pp,
                      pp + m * l, k.rg2_g, k.rg2_ws, 1, m, n, k.rg_err, st);
      check_launch();
      double* rs[3] = {(double*)R0, (double*)R1, nullptr};
      launch_finalize_residual<double>(pp, 1, (const double*)B, 2, rs, m * l, nullptr, 0, 1,
                                       nullptr, 0, nullptr, nullptr, 0.0, nullptr,
                                       Red{k.part, k.ticket, k.scal}, st);
      launch_sum_partials<double>(k.rg2_g, resgrad2_groups(n), (double*)G, n * l, st);
      check_launch();
      int herr = 0;   // valid only if no hand-off wait timed out (the call is synchronous)
      GLX_HIP(hipMemcpyAsync(&herr, k.rg_err, sizeof(int), hipMemcpyDeviceToHost, st));
      GLX_HIP(hipStreamSynchronize(st));
      if (std::getenv("GLX_RG_VERBOSE")) std::fprintf(stderr, "glx_residual_gradient2: one-pass err flag %d\n", herr);
      if (herr == 0) return;
      if (one_pass_ran) *one_pass_ran = 0;
    }
    auto two = [&](auto* Ap) {
      typedef std::remove_const_t<std::remove_pointer_t<decltype(Ap)>> T;
      const T* xs[3] = {(const T*)X0, (const T*)X1, nullptr};
      T* rs[3] = {(T*)R0, (T*)R1, nullptr};
      launch_ax<T>(p, 2, Ap, xs, (T*)k.pp, nullptr, 0, st);
      launch_finalize_residual<T>((const T*)k.pp, ax_split(p, 2), (const T*)B, 2, rs, m * l, nullptr, 0,
                                  1, nullptr, 0, nullptr, nullptr, 0.0, nullptr,
                                  Red{k.part, k.ticket, k.scal}, st);
      T* gp = p.atr_S > 1 ? (T*)k.gp : (T*)G;
      launch_atr<T>(p, Ap, (const T*)R1, gp, st);
      if (p.atr_S > 1) launch_sum_partials<T>(gp, p.atr_S, (T*)G, n * l, st);
    };
    if (dtype == GLX_F64) two((const double*)A);
    else two((const float*)A);
    check_launch();
  });
}

int glx_prox(int dtype, int64_t n, int64_t l, const void* W, double t, double mu, double thres,
             void* X_out, void* sums_dev, void* ws, size_t wsb, void* stream) {
  return guarded([&] {
    hipStream_t st = static_cast<hipStream_t>(stream);
    GemmPlan p;
    KernelWs k = kernel_setup(dtype, 1, n, l, ws, wsb, 0, st, &p);
    Red r{k.part, k.ticket, sums_dev ? static_cast<double*>(sums_dev) : k.scal};
    if (dtype == GLX_F64)
      launch_prox_plain<double>((const double*)W, (double*)X_out, n, l, t, mu, thres, r, st);
    else
      launch_prox_plain<float>((const float*)W, (float*)X_out, n, l, t, mu, thres, r, st);
    check_launch();
  });
}

}  // extern "C"
