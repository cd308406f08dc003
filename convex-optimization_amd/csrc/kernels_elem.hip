// kernels_elem.hip — per-group (row of x) and elementwise kernels of the solvers, each fused
// with the scalar reductions the host control flow needs.
//
// Everything here is HBM/L2 streaming over n*l or m*l elements (4 MiB at the north-star
// size); the work per element is a handful of flops. Rows of x (groups, l contiguous values)
// are owned by LPR lanes (LPR = min(16, next_pow2(l))), each lane holding EPL elements strided
// by LPR, so a group's l2 norm is an in-register sum plus log2(LPR) xor-shuffles.
//
// Floating-point expressions keep the reference's NumPy evaluation order (the library is
// built with -ffp-contract=off, so a*b+c is never fused behind our back):
//   prox   (gl_ProxGD_primal.py:65-71)  p = (w * max(||w_i|| - t*mu, 0)) / ((||w_i|| < thres) + ||w_i||)
//   G_t    (gl_ProxGD_primal.py:73-74)  G = (x - p) / t,  trial point z = x - t*G  (:91)
//   FISTA  (gl_FProxGD_primal.py:139,145)  y = (1-θ) x + θ v,  v = x + (x_new - x)/θ
//   SGD    (gl_SGD_primal.py:56-61,96)  x - α (g + μ x/((||x_i||<thres)+||x_i||))
//   GD     (gl_GD_primal.py:59-63,98)   x - α (g + μ x/sqrt(Σx_i² + δ²))
// Scalars (t, μ, α, thres …) arrive as double and are rounded to T first, as NumPy does with
// Python-float operands of a T array (NEP 50 weak scalars).
//
// Reductions are deterministic: block partials in a fixed tree order, then the last block to
// arrive (sc1 partials + a two-level agent-scope arrival ticket, see grid_reduce) sums the
// block partials in block order. max() propagates NaN like np.max.
#include <cstdlib>

#include "glx.h"
#include "glx_device.h"

namespace glx {

static inline unsigned grid_for(int64_t work, int per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > kMaxBlocks) g = kMaxBlocks;
  return (unsigned)g;
}



// ------------------------------------------------------------------------------------------
// residual finalize: R = sum_s P[s] - B; out[0] = sum R^2, out[1] = count(|c| > 1e-6 *cmax)
// over a second array c (the candidate iterate, fused here to save a launch); the last block
// optionally records f = 0.5 out[0] + mu * (*rn) into fh (SGD/GD device-side history).
//
// The S slabs of one residual element are split over G adjacent lanes (G = 1, 2, 4 or 8, so a
// lane takes at most 8 slabs). A lane issues its loads back to back and adds them in slab
// order; the G partial sums then combine by an xor butterfly, which gives every lane of the
// group the same bits ((p0 + p1) + (p2 + p3) ...). The order is fixed, so the result is
// deterministic, and G = 1 is the plain sequential sum. With few rows and a deep split (the
// per-rank shards of a multi-GPU run: m = 1024, S = 32) this spreads the slab reads over the
// whole grid instead of leaving them to m*l threads with S-long load chains (22 -> 11.6 us at
// m = 1024). Splitting further than 8 slabs per lane measured slower (NS: 13.7 -> 17.9 us).
// ------------------------------------------------------------------------------------------
constexpr int kSlabLoads = 8;
static inline int finalize_groups(int S) {
  int g = 1;
  while (g * kSlabLoads < S) g *= 2;
  return g;
}

// group_slab_sum in two halves, so a caller can issue the loads of several sources before the
// first add (round 5: the finalize's two sources, one round trip instead of two)
template <typename T, int G>
__device__ inline int group_slab_load(const T* __restrict__ P, int S, int64_t ml, int64_t idx, int sub,
                                      T (&a)[kSlabLoads]) {
  const int per = (S + G - 1) / G;
  const int k0 = sub * per;
  const int cnt = S - k0 < per ? S - k0 : per;   // <= 0 for an empty trailing lane
#pragma unroll
  for (int k = 0; k < kSlabLoads; ++k) a[k] = k < cnt ? P[(int64_t)(k0 + k) * ml + idx] : T(0);
  return cnt;
}
template <typename T, int G>
__device__ inline T group_slab_fold(const T (&a)[kSlabLoads], int cnt) {
  T v = a[0];
#pragma unroll
  for (int k = 1; k < kSlabLoads; ++k)
    if (k < cnt) v = v + a[k];
#pragma unroll
  for (int off = 1; off < G; off <<= 1) v = v + __shfl_xor(v, off);
  return v;
}
template <typename T, int G>
__device__ inline T group_slab_sum(const T* __restrict__ P, int S, int64_t ml, int64_t idx, int sub) {
  T a[kSlabLoads];
  const int cnt = group_slab_load<T, G>(P, S, ml, idx, sub, a);
  return group_slab_fold<T, G>(a, cnt);
}

// Device-controlled ProxGD with a communicator (solver.cpp dc_queue): the trial's residual sums
// are final only after the gradient all-reduce that carries them (a gradient set's tail), so the
// decision runs as its own one-thread launch right behind that all-reduce. Skipped once an earlier
// decision of the batch has cancelled it; hands its record straight to the host ring.
__global__ void k_ctl_decide(Ctl c, const double* __restrict__ out, double* host, unsigned* host_seq,
                             unsigned seq) {
  if (threadIdx.x != 0) return;
  if (*c.abort != 0) return;
  double pre[10];
  for (int k = 0; k < 6; ++k) pre[k] = c.tr[k];
  for (int k = 0; k < 4; ++k) pre[6 + k] = c.state[k];
  double o[4];
  for (int k = 0; k < 4; ++k) o[k] = out[k];
  ctl_decide(c, o, pre);
  publish_packet(c.rec, 11, host, host_seq, seq);
}

__global__ void k_ctl_seed(double* state, int* abort, double s0, double s1, double s2, double s3) {
  if (threadIdx.x == 0) {
    state[0] = s0;
    state[1] = s1;
    state[2] = s2;
    state[3] = s3;
    *abort = 0;
  }
}

// *cmax, or (cmp != NULL: the trial's sums still pending as Red::parts_only partials, cmnv values
// per slot) the max of their column 3 over cmnp slots, by every workgroup for itself (all 256
// threads call this; the result is order-independent)
__device__ inline double pending_max(const double* cmax, const double* __restrict__ cmp, int cmnp, int cmnv) {
  if (cmp == nullptr) return *cmax;
  __shared__ double wmax[4];
  double mv = -__builtin_inf();
  for (int i = threadIdx.x; i < cmnp; i += 256) mv = nan_max(mv, cmp[i * cmnv + 3]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mv = nan_max(mv, __shfl_xor(mv, off));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mv;
  __syncthreads();
  return nan_max(nan_max(wmax[0], wmax[1]), nan_max(wmax[2], wmax[3]));
}

// count(|cx| > 1e-6 cm) over this thread's indices tid, tid + stride, ...: the first kCountAhead
// values already in cxv (loaded ahead), the rest read here
constexpr int kCountAhead = 2;
template <typename T>
__device__ inline double count_above(const T* __restrict__ cx, int64_t cn, const T (&cxv)[kCountAhead],
                                     int64_t tid, int64_t stride, double cm) {
  const T thr = (T)1e-6 * (T)cm;
  double c = 0.0;
#pragma unroll
  for (int q = 0; q < kCountAhead; ++q)
    if (tid + q * stride < cn) c += (tabs(cxv[q]) > thr) ? 1.0 : 0.0;
  for (int64_t idx = tid + kCountAhead * stride; idx < cn; idx += stride) c += (tabs(cx[idx]) > thr) ? 1.0 : 0.0;
  return c;
}

template <typename T, int NSRC, int G>
__global__ __launch_bounds__(256) void k_finalize_residual(
    const T* __restrict__ P, int S, const T* __restrict__ B, T* __restrict__ R0, T* __restrict__ R1,
    T* __restrict__ R2, int64_t ml, const int* __restrict__ gate, int epoch, int gate_mode,
    const T* __restrict__ cx, int64_t cn, const double* __restrict__ cmax, double* __restrict__ fh,
    double fh_mu, const double* __restrict__ fh_rn, Red red, const double* __restrict__ snap_src,
    double* __restrict__ snap_dst, int nsnap, int chain, const T* __restrict__ P0, int S0, Ctl ctl,
    const double* __restrict__ cmp, int cmnp, int cmnv) {
  // a cancelled launch (device-controlled batch) stores nothing and returns before the
  // reduction; the flag is tested at the first store, so its load overlaps the slab loads
  const bool skipped = red_skipped(red);
  double pre[10];
  if (ctl.rec != nullptr && threadIdx.x == 0) {
    for (int k = 0; k < 6; ++k) pre[k] = ctl.tr[k];
    for (int k = 0; k < 4; ++k) pre[6 + k] = ctl.state[k];
  }
  const bool live = (gate == nullptr) || (*gate == epoch);
  if (!live && gate_mode == 0) return;  // uniform over the grid: nobody touches the ticket
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  T* rs[3] = {R0, R1, R2};
  const int sub = threadIdx.x % G;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  // the count's first kCountAhead values are loaded before the slab loads (their latencies
  // overlap); the threshold (max |cx|) is known only later
  T cxv[kCountAhead];
#pragma unroll
  for (int q = 0; q < kCountAhead; ++q)
    cxv[q] = (cx != nullptr && tid + q * stride < cn) ? cx[tid + q * stride] : T(0);
  // residual elements: G lanes per element; the lanes of a group share idx, so they enter and
  // leave the loop together and the butterfly only reads active partners
  for (int64_t idx = tid / G; idx < ml; idx += stride / G) {
    const T bv = B[idx];
    if (NSRC == 2 && chain) {   // split-candidate: R0 = (A p_thr - b) + A e (always live)
      // chain 2 (round 6, the fused A e pass): the slabs behind P0 are A p, so R0 = A p - b and
      // R1 = A p_thr - b = R0 - A e
      T a1[kSlabLoads], a0[kSlabLoads];
      const int c1 = group_slab_load<T, G>(P + (int64_t)S0 * ml, S, ml, idx, sub, a1);
      const int c0 = group_slab_load<T, G>(P0, S0, ml, idx, sub, a0);
      T r1, r0;
      if (chain == 2) {
        r0 = group_slab_fold<T, G>(a1, c1) - bv;
        r1 = r0 - group_slab_fold<T, G>(a0, c0);
      } else {
        r1 = group_slab_fold<T, G>(a1, c1) - bv;
        r0 = r1 + group_slab_fold<T, G>(a0, c0);
      }
      if (skipped) return;
      if (sub == 1 % G) rs[1][idx] = r1;
      if (R0 != nullptr && sub == 0) rs[0][idx] = r0;
      if (sub == 0) {
        v[0] += (double)(r0 * r0);
        v[1] += (double)(r1 * r1);
      }
      continue;
    }
    T a[NSRC][kSlabLoads];   // every source's slab loads issued before the first add
    int cs[NSRC];
    if (live) {
#pragma unroll
      for (int sr = 0; sr < NSRC; ++sr)
        cs[sr] = group_slab_load<T, G>(P + (int64_t)sr * S * ml, S, ml, idx, sub, a[sr]);
    }
#pragma unroll
    for (int sr = 0; sr < NSRC; ++sr) {
      T r;
      if (live) {
        r = group_slab_fold<T, G>(a[sr], cs[sr]) - bv;
        if (skipped) return;
        if (sub == sr % G) rs[sr][idx] = r;
      } else {
        r = rs[sr][idx];
      }
      if (sub == 0) v[sr] += (double)(r * r);
    }
  }
  if (skipped) return;   // (threads without a residual element; uniform over the grid)
  if (cx != nullptr) v[3] = count_above(cx, cn, cxv, tid, stride, pending_max(cmax, cmp, cmnp, cmnv));
  const bool last = grid_reduce<4, 0u>(v, red);
  if (last && fh != nullptr && threadIdx.x == 0) *fh = 0.5 * red.out[0] + fh_mu * (*fh_rn);
  // snapshot of the preceding trial's sums for a packet published after the next trial has
  // overwritten them (the A@X-carried packet of the multi-GPU path)
  if (last && (int)threadIdx.x < nsnap) snap_dst[threadIdx.x] = snap_src[threadIdx.x];
  if (last && ctl.rec != nullptr && threadIdx.x == 0) ctl_decide(ctl, red.out, pre);
}

// Split-candidate FISTA batch (solver.cpp iter_fista): the dense source is A xc (S slabs at P),
// the gather slab(s) hold A e_c (S0 at Pe), and A y_next follows from the linearity of
// y_next = a1 thr(xc) + b1 (thr(xk) + (xc - thr(xk)) / theta)   (fista_row):
//   A thr(xc) = A xc - A e_c,   A y_next = a1 A thr(xc) + b1 (A thr(xk) + (A xc - A thr(xk)) / theta)
// with A thr(xk) (sxo) kept from the previous accepted trial. Writes R_y = A y_next - b and
// sxo_out = A thr(xc); out: [sum (A xc - b)^2, sum R_y^2, nnz(e_c) = sum of the nl list
// lengths `counts` (written by k_at_gather), count(|cx| > 1e-6 *cmax)].
template <typename T, int G>
__global__ __launch_bounds__(256) void k_finalize_fista(
    const T* __restrict__ P, int S, const T* __restrict__ Pe, int S0, const T* __restrict__ B,
    T* __restrict__ Ry, const T* __restrict__ sxo, T* __restrict__ sxo_out, int64_t ml, double a1_,
    double b1_, double theta_, const T* __restrict__ cx, int64_t cn, const double* __restrict__ cmax,
    const unsigned* __restrict__ counts, int nl, Red red, Ctl ctl, const double* __restrict__ cmp,
    int cmnp, int cmnv) {
  const bool skipped = red_skipped(red);   // cancelled in a device-controlled batch
  double pre[10];
  if (ctl.rec != nullptr && threadIdx.x == 0) {
    for (int k = 0; k < 6; ++k) pre[k] = ctl.tr[k];
    for (int k = 0; k < 4; ++k) pre[6 + k] = ctl.state[k];
  }
  const T a1 = (T)a1_, b1 = (T)b1_, theta = (T)theta_;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  if (blockIdx.x == 0 && (int)threadIdx.x < nl) v[2] = (double)counts[threadIdx.x];
  const int sub = threadIdx.x % G;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  T cxv[kCountAhead];   // (as k_finalize_residual)
#pragma unroll
  for (int q = 0; q < kCountAhead; ++q)
    cxv[q] = (cx != nullptr && tid + q * stride < cn) ? cx[tid + q * stride] : T(0);
  for (int64_t idx = tid / G; idx < ml; idx += stride / G) {
    const T bv = B[idx];
    const T sx = group_slab_sum<T, G>(P, S, ml, idx, sub);
    const T apt = sx - group_slab_sum<T, G>(Pe, S0, ml, idx, sub);
    const T so = sxo[idx];
    const T avn = so + (sx - so) / theta;
    const T ry = (a1 * apt + b1 * avn) - bv;
    const T rx = sx - bv;
    if (skipped) return;
    if (sub == 0) {
      Ry[idx] = ry;
      sxo_out[idx] = apt;
      v[0] += (double)(rx * rx);
      v[1] += (double)(ry * ry);
    }
  }
  if (skipped) return;
  if (cx != nullptr) v[3] = count_above(cx, cn, cxv, tid, stride, pending_max(cmax, cmp, cmnp, cmnv));
  const bool last = grid_reduce<4, 0u>(v, red);
  if (last && ctl.rec != nullptr && threadIdx.x == 0) ctl_decide(ctl, red.out, pre);
}

template <typename T>
__global__ __launch_bounds__(256) void k_sum_partials(const T* __restrict__ Gp, int S, T* __restrict__ G,
                                                      int64_t nl) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < nl; idx += stride)
    G[idx] = slab_sum(Gp, S, nl, idx);
}

// Iterate over rows: each group of LPR lanes owns one row per trip.
// NB = the workgroups that share the rows, BI = this workgroup's index among them (all but a
// publisher workgroup, see Pub)
#define GLX_ROW_LOOP_BEGIN_NBI(LPR, NB, BI)                                            \
  const int sub = threadIdx.x & ((LPR)-1);                                             \
  const int64_t rows_per_block = 256 / (LPR);                                          \
  const int64_t row_stride = (int64_t)(NB) * rows_per_block;                           \
  const int64_t n_trips = (n + row_stride - 1) / row_stride;                           \
  for (int64_t trip = 0; trip < n_trips; ++trip) {                                     \
    const int64_t row = trip * row_stride + (int64_t)(BI) * rows_per_block +           \
                        (threadIdx.x / (LPR));                                         \
    const bool rv = row < n;                                                           \
    const int64_t base = (rv ? row : 0) * l;
#define GLX_ROW_LOOP_BEGIN_NB(LPR, NB) GLX_ROW_LOOP_BEGIN_NBI(LPR, NB, blockIdx.x)
#define GLX_ROW_LOOP_BEGIN(LPR) GLX_ROW_LOOP_BEGIN_NB(LPR, gridDim.x)
#define GLX_ROW_LOOP_END }

// ------------------------------------------------------------------------------------------
// ProxGD line-search trial (gl_ProxGD_primal.py:73-74, 89-92)
// g = sum of S gradient slabs (written to gout when non-null so later trials read one array);
// outputs p, p_thr = p with |p| < thres zeroed (the next iteration's x after :127), z.
// out: [sum g*G_t, sum G_t^2, sum_i ||p_i||, max |p|, #{p changed by the threshold},
//       #{rows of p changed by the threshold}]
// ------------------------------------------------------------------------------------------
template <typename T, int LPR, int EPL>
__global__ __launch_bounds__(256) void k_prox_pgd(const T* __restrict__ x, const T* __restrict__ g,
                                                  int S, T* __restrict__ gout, T* __restrict__ p,
                                                  T* __restrict__ pthr, T* __restrict__ z,
                                                  unsigned* __restrict__ zf, int64_t n,
                                                  int64_t l, double t_, double tmu_, double thres_,
                                                  Red red, Pub pub) {
  // a launch of a device-controlled batch cancelled by an earlier decision (communicator path,
  // solver.cpp dc_queue_comm): nothing is written, no ticket touched (uniform over the grid)
  if (red_skipped(red)) {
    if (pub.host != nullptr && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
      publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq);
    return;
  }
  if (publisher_last<6, 0x8u>(pub, red)) return;
  const T t = (T)t_, tmu = (T)tmu_, thres = (T)thres_;
  const int64_t nl = n * l;
  double acc[6] = {0.0, 0.0, 0.0, -__builtin_inf(), 0.0, 0.0};
  GLX_ROW_LOOP_BEGIN_NB(LPR, gridDim.x - (pub.host ? 1u : 0u))
  T xv[EPL], gv[EPL], pv[EPL], pth[EPL], zv[EPL];
  bool ok[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    ok[e] = rv && j < l;
    xv[e] = ok[e] ? x[base + j] : T(0);
    gv[e] = ok[e] ? slab_sum(g, S, nl, base + j) : T(0);
    if (ok[e] && gout != nullptr) gout[base + j] = gv[e];
  }
  const unsigned rowe = prox_pgd_row<T, LPR, EPL>(xv, gv, ok, rv, sub, t, tmu, thres, pv, pth, zv, acc,
                                              zf != nullptr);
  if (zf != nullptr && rv && sub == 0) zf[row] = rowe;
  if constexpr (LPR == 16) {   // the split-candidate shapes (l in {16, 32}): the column bitmaps
    __shared__ unsigned msk[16];
    if (zf != nullptr) zf_store_group16(msk, rowe, rv, sub, zf, n, (int)l, row - (threadIdx.x >> 4));
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    if (ok[e]) {
      p[base + j] = pv[e];
      pthr[base + j] = pth[e];
      z[base + j] = zv[e];
    }
  }
  GLX_ROW_LOOP_END
  grid_reduce<6, 0x8u>(acc, red);
}

__global__ __launch_bounds__(256) void k_shard_combine(ShardPub sp) { shard_combine_block(sp); }

// Row-sharded ProxGD trial, the replicated half (solver.cpp iter_proxgd_shard): each rank ran
// k_prox_pgd on its n / G rows and the rows of p were all-gathered; every rank re-derives p_thr,
// z and the masks of e from p with the comparisons and arithmetic k_prox_pgd uses, so the bits
// equal the ones the trial kernel would have written for the whole of p. With sp.blk the last
// workgroup combines the gathered sums (and publishes the packet) beside the rows.
template <typename T, int LPR, int EPL>
__global__ __launch_bounds__(256) void k_trial_split(const T* __restrict__ p, const T* __restrict__ xt,
                                                     T* __restrict__ pthr, T* __restrict__ z,
                                                     unsigned* __restrict__ zf, int64_t n, int64_t l,
                                                     double t_, double thres_, int emode, ShardPub sp) {
  if (sp.blk != nullptr && blockIdx.x == gridDim.x - 1) {
    shard_combine_block(sp);
    return;
  }
  const T t = (T)t_, thres = (T)thres_;
  GLX_ROW_LOOP_BEGIN_NB(LPR, gridDim.x - (sp.blk != nullptr ? 1u : 0u))
  T pth[EPL], zv[EPL];
  bool ok[EPL];
  unsigned mk = 0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    ok[e] = rv && j < l;
    const T pv = ok[e] ? p[base + j] : T(0);
    const bool small = tabs(pv) < thres;
    pth[e] = small ? T(0) : pv;
    if (emode) {
      zv[e] = small ? pv : T(0);
    } else {
      const T xv = ok[e] ? xt[base + j] : T(0);
      const T G = (xv - pv) / t;
      zv[e] = xv - t * G;
    }
    if (ok[e] && small && pv != T(0) && sub + e * LPR < 32) mk |= 1u << (sub + e * LPR);
  }
  const unsigned rowe = row_or<LPR>(mk);
  if (zf != nullptr && rv && sub == 0) zf[row] = rowe;
  if constexpr (LPR == 16) {
    __shared__ unsigned msk[16];
    if (zf != nullptr) zf_store_group16(msk, rowe, rv, sub, zf, n, (int)l, row - (threadIdx.x >> 4));
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    if (ok[e]) {
      pthr[base + j] = pth[e];
      if (z != nullptr) z[base + j] = zv[e];
    }
  }
  GLX_ROW_LOOP_END
}

// Row-sharded FISTA trial, the replicated half (solver.cpp iter_fista_shard): v_next and y_next of
// every element from the all-gathered xc with fista_row's comparisons and arithmetic; the last
// workgroup (sp.blk) combines the gathered sums beside them.
template <typename T>
__global__ __launch_bounds__(256) void k_fista_split(const T* __restrict__ xc, const T* __restrict__ xk,
                                                     T* __restrict__ vnext, T* __restrict__ ynext,
                                                     int64_t nl, double thres_, double theta_, double a1_,
                                                     double b1_, ShardPub sp) {
  if (sp.blk != nullptr && blockIdx.x == gridDim.x - 1) {
    shard_combine_block(sp);
    return;
  }
  const T thres = (T)thres_, theta = (T)theta_, a1 = (T)a1_, b1 = (T)b1_;
  const int64_t nb = gridDim.x - (sp.blk != nullptr ? 1 : 0);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nl; i += nb * 256) {
    const T pv = xc[i];
    T xo = xk[i];
    if (tabs(xo) < thres) xo = T(0);
    const T vn = xo + (pv - xo) / theta;
    const T pt = tabs(pv) < thres ? T(0) : pv;
    vnext[i] = vn;
    ynext[i] = a1 * pt + b1 * vn;
  }
}

// FISTA / FGD trial (gl_FProxGD_primal.py:92-102, gl_FGD_primal.py:209-212), fused with the
// next iteration's combine so that A @ [xc | y_next] is one pass over A:
//   xc     = prox(y - t g, t)        (PROX) or y - t g (FGD's identity prox)
//   v_next = xk_thr + (xc - xk_thr) / theta                           (:145)
//   y_next = (1 - theta') thr(xc) + theta' v_next                     (:136, :139 of the next step)
// with xk_thr = xk with |xk| < thres zeroed (xk itself is left untouched; :136).
// out: PROX: [sum g*(xc-y), sum (xc-y)^2, sum ||xc_i||, max |xc|]
//      FGD : [sum g*(xc-y), sum (xc-y)^2, sum (sqrt(||xc_i||^2+d^2)-d), sum ||xc_i||, max |xc|]
template <typename T, int LPR, int EPL, bool PROX>
__global__ __launch_bounds__(256) void k_fista_trial(
    const T* __restrict__ y, const T* __restrict__ g, int S, T* __restrict__ gout,
    const T* __restrict__ xk, T* __restrict__ xc, T* __restrict__ vnext, T* __restrict__ ynext,
    int64_t n, int64_t l, double t_, double tmu_, double thres_, double theta_, double a1_,
    double b1_, double dd_, double delta_, Red red, Pub pub, T* __restrict__ ec,
    unsigned* __restrict__ zf) {
  constexpr int NV = PROX ? 4 : 5;
  if (red_skipped(red)) {   // cancelled in a device-controlled batch (as k_prox_pgd)
    if (pub.host != nullptr && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
      publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq);
    return;
  }
  if (publisher_last<NV, (1u << (NV - 1))>(pub, red)) return;
  const T t = (T)t_, tmu = (T)tmu_, thres = (T)thres_, theta = (T)theta_, a1 = (T)a1_, b1 = (T)b1_;
  const T dd = (T)dd_, delta = (T)delta_;
  const int64_t nl = n * l;
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = 0.0;
  acc[NV - 1] = -__builtin_inf();
  GLX_ROW_LOOP_BEGIN_NB(LPR, gridDim.x - (pub.host ? 1u : 0u))
  T yv[EPL], gv[EPL], xkv[EPL], xcv[EPL], vnv[EPL], ynv[EPL], ecv[EPL];
  bool ok[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    ok[e] = rv && j < l;
    yv[e] = ok[e] ? y[base + j] : T(0);
    gv[e] = ok[e] ? slab_sum(g, S, nl, base + j) : T(0);
    xkv[e] = ok[e] ? xk[base + j] : T(0);
    if (ok[e] && gout != nullptr) gout[base + j] = gv[e];
  }
  const unsigned rowe = fista_row<T, LPR, EPL, PROX>(yv, gv, xkv, ok, rv, sub, t, tmu, thres, theta, a1,
                                                  b1, dd, delta, xcv, vnv, ynv, acc,
                                                  ec != nullptr ? ecv : nullptr);
  if (zf != nullptr && rv && sub == 0) zf[row] = rowe;
  if constexpr (LPR == 16) {   // the split-candidate shapes (l in {16, 32}): the column bitmaps
    __shared__ unsigned msk[16];
    if (zf != nullptr) zf_store_group16(msk, rowe, rv, sub, zf, n, (int)l, row - (threadIdx.x >> 4));
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    if (ok[e]) {
      xc[base + j] = xcv[e];
      vnext[base + j] = vnv[e];
      ynext[base + j] = ynv[e];
      if (ec != nullptr) ec[base + j] = ecv[e];
    }
  }
  GLX_ROW_LOOP_END
  grid_reduce<NV, (1u << (NV - 1))>(acc, red);
}

// plain prox (C-ABI glx_prox): out [sum ||x_i||, max |x|]
template <typename T, int LPR, int EPL>
__global__ __launch_bounds__(256) void k_prox_plain(const T* __restrict__ wsrc, T* __restrict__ xo,
                                                    int64_t n, int64_t l, double tmu_, double thres_,
                                                    Red red) {
  const T tmu = (T)tmu_, thres = (T)thres_;
  double acc[2] = {0.0, -__builtin_inf()};
  GLX_ROW_LOOP_BEGIN(LPR)
  T w[EPL];
  T sq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    w[e] = (rv && j < l) ? wsrc[base + j] : T(0);
    sq = sq + w[e] * w[e];
  }
  const T nrm = __builtin_sqrt(row_allsum<LPR>(sq));
  T c = nrm - tmu;
  c = (c < T(0)) ? T(0) : c;
  const T d = ((nrm < thres) ? T(1) : T(0)) + nrm;
  T psq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    const T pv = (w[e] * c) / d;
    if (rv && j < l) {
      xo[base + j] = pv;
      acc[1] = nan_max(acc[1], (double)tabs(pv));
      psq = psq + pv * pv;
    }
  }
  const T pn = __builtin_sqrt(row_allsum<LPR>(psq));
  if (rv && sub == 0) acc[0] += (double)pn;
  GLX_ROW_LOOP_END
  grid_reduce<2, 0x2u>(acc, red);
}

// row-norm sum and max|x| (objective + sparsity of the current iterate)
template <typename T, int LPR, int EPL>
__global__ __launch_bounds__(256) void k_rownorm_max(const T* __restrict__ x, int64_t n, int64_t l, Red red) {
  double acc[2] = {0.0, -__builtin_inf()};
  GLX_ROW_LOOP_BEGIN(LPR)
  T sq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    if (rv && j < l) {
      const T v = x[base + j];
      sq = sq + v * v;
      acc[1] = nan_max(acc[1], (double)tabs(v));
    }
  }
  const T nr = __builtin_sqrt(row_allsum<LPR>(sq));
  if (rv && sub == 0) acc[0] += (double)nr;
  GLX_ROW_LOOP_END
  grid_reduce<2, 0x2u>(acc, red);
}

// SGD (MODE 0, gl_SGD_primal.py:56-61) / GD (MODE 1, gl_GD_primal.py:59-63) step, in place.
// reads the thresholded iterate xt; writes x = x_new and xt = thr(x_new) (the next
// iteration's threshold, :93, precomputed so A @ [x | xt] is one pass). out: [sum ||x_new_i||]
template <typename T, int LPR, int EPL, int MODE>
__global__ __launch_bounds__(256) void k_descent(T* __restrict__ x, T* __restrict__ xt,
                                                 const T* __restrict__ g, int S,
                                                 int64_t n, int64_t l, double alpha_, double mu_,
                                                 double thres_, double dd_, Red red) {
  const T alpha = (T)alpha_, mu = (T)mu_, thres = (T)thres_, dd = (T)dd_;
  const int64_t nl = n * l;
  double acc[1] = {0.0};
  GLX_ROW_LOOP_BEGIN(LPR)
  T xv[EPL], gv[EPL];
  T sq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    const bool ok = rv && j < l;
    xv[e] = ok ? xt[base + j] : T(0);
    gv[e] = ok ? slab_sum(g, S, nl, base + j) : T(0);
    sq = sq + xv[e] * xv[e];
  }
  const T s = row_allsum<LPR>(sq);
  T d;
  if (MODE == 0) {
    const T nrm = __builtin_sqrt(s);
    d = ((nrm < thres) ? T(1) : T(0)) + nrm;
  } else {
    d = __builtin_sqrt(s + dd);
  }
  T nsq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    const T sub_g = gv[e] + mu * (xv[e] / d);
    const T xn = xv[e] - alpha * sub_g;
    if (rv && j < l) {
      x[base + j] = xn;
      xt[base + j] = (tabs(xn) < thres) ? T(0) : xn;
      nsq = nsq + xn * xn;
    }
  }
  const T nn = __builtin_sqrt(row_allsum<LPR>(nsq));
  if (rv && sub == 0) acc[0] += (double)nn;
  GLX_ROW_LOOP_END
  grid_reduce<1, 0u>(acc, red);
}

// FGD: g += mu * y / sqrt(sum y^2 + delta^2) (gl_FGD_primal.py:69-72);
//      out: sum_i (sqrt(sum y_i^2 + delta^2) - delta) (:64-67)
template <typename T, int LPR, int EPL>
__global__ __launch_bounds__(256) void k_fgd_grad(const T* __restrict__ y, const T* __restrict__ gp,
                                                  int S, T* __restrict__ g, int64_t n, int64_t l,
                                                  double mu_, double dd_, double delta_, Red red) {
  const T mu = (T)mu_, dd = (T)dd_, delta = (T)delta_;
  const int64_t nl = n * l;
  double acc[1] = {0.0};
  GLX_ROW_LOOP_BEGIN(LPR)
  T yv[EPL];
  T sq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    yv[e] = (rv && j < l) ? y[base + j] : T(0);
    sq = sq + yv[e] * yv[e];
  }
  const T s = row_allsum<LPR>(sq);
  const T d = __builtin_sqrt(s + dd);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t j = sub + (int64_t)e * LPR;
    if (rv && j < l) g[base + j] = slab_sum(gp, S, nl, base + j) + mu * (yv[e] / d);
  }
  if (rv && sub == 0) acc[0] += (double)(d - delta);
  GLX_ROW_LOOP_END
  grid_reduce<1, 0u>(acc, red);
}

// ------------------------------------------------------------------------------------------
// flat elementwise kernels
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_count_above(const T* __restrict__ x, int64_t nl,
                                                     const double* __restrict__ maxv, Red red) {
  const T thr = (T)1e-6 * (T)(*maxv);
  double v[1] = {0.0};
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < nl; idx += stride)
    v[0] += (tabs(x[idx]) > thr) ? 1.0 : 0.0;
  grid_reduce<1, 0u>(v, red);
}

// xo = x with |x| < thres zeroed (xo may alias x); *flag = epoch when any value changed
template <typename T>
__global__ __launch_bounds__(256) void k_threshold(const T* x, T* xo, int64_t nl, double thres_,
                                                   int* flag, int epoch) {
  const T thres = (T)thres_;
  int changed = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < nl; idx += stride) {
    const T v = x[idx];
    if (tabs(v) < thres) {
      if (v != T(0)) changed = 1;
      xo[idx] = T(0);
    } else if (xo != x) {
      xo[idx] = v;
    }
  }
  if (__any(changed) && (threadIdx.x & 63) == 0) *flag = epoch;   // same value from every writer
}

// FISTA: x_k[|x_k| < thres] = 0 in place (gl_FProxGD_primal.py:136), then
// y = (1 - theta) x_k + theta v_k (:139)
template <typename T>
__global__ __launch_bounds__(256) void k_thr_axpby(T* __restrict__ xk, const T* __restrict__ vk,
                                                   T* __restrict__ y, int64_t nl, double thres_,
                                                   double a_, double b_) {
  const T thres = (T)thres_, a = (T)a_, b = (T)b_;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < nl; idx += stride) {
    T v = xk[idx];
    if (tabs(v) < thres) {
      v = T(0);
      xk[idx] = v;
    }
    y[idx] = a * v + b * vk[idx];
  }
}

// the deferred reductions of a packet, then the packet (host == NULL: the reductions only)
__global__ __launch_bounds__(256) void k_publish_pub(Pub pub) {
  defer_reduce<4>(pub);
  if (threadIdx.x == 0 && pub.host != nullptr)
    publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq, pub.s2, pub.off2, pub.n2, pub.s3,
                   pub.off3, pub.n3);
}

// publish the scalar packet to host-mapped memory: data, then (system-scope release) seq
__global__ void k_publish(const double* __restrict__ s, int ns, double* host, unsigned* host_seq,
                          unsigned seq, const double* __restrict__ s2, int off2, int n2) {
  if (threadIdx.x == 0) publish_packet(s, ns, host, host_seq, seq, s2, off2, n2);
}

template <typename T>
__global__ __launch_bounds__(256) void k_fista_v(const T* __restrict__ xk, const T* __restrict__ x,
                                                 T* __restrict__ v, int64_t nl, double theta_) {
  const T theta = (T)theta_;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < nl; idx += stride) {
    const T xo = xk[idx];
    v[idx] = xo + (x[idx] - xo) / theta;
  }
}

__global__ void k_record_f(const double* __restrict__ s, int i_sumsq, int i_reg, double mu,
                           double* __restrict__ fh, int64_t idx) {
  if (threadIdx.x == 0) fh[idx] = 0.5 * s[i_sumsq] + mu * s[i_reg];
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <int LPR, typename F>
static void dispatch_epl(int64_t l, F&& f) {
  const int64_t epl = (l + LPR - 1) / LPR;
  switch (epl) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 7: f(std::integral_constant<int, 7>{}); break;
    default: f(std::integral_constant<int, 8>{}); break;
  }
}
// F receives (lpr_constant, epl_constant)
template <typename F>
static void dispatch_row(int64_t l, F&& f) {
  if (l <= 1) f(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
  else if (l <= 2) f(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
  else if (l <= 4) f(std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{});
  else if (l <= 8) f(std::integral_constant<int, 8>{}, std::integral_constant<int, 1>{});
  else dispatch_epl<16>(l, [&](auto epl) { f(std::integral_constant<int, 16>{}, epl); });
}
// Work workgroups of the row kernels, at most kRowBlocks (GLX_ROW_BLOCKS overrides): at n = 16384
// two 16-row trips per workgroup instead of one halve the grid reduction's fan-in. Round 4, the
// 8-GPU shard model (1024 rows, communicator path, where the trial kernel runs every iteration;
// two interleaved rounds, profiles/r4_exp8/, profiles/r4_exp9/): k_prox_pgd 14.4 -> 12.4 us,
// ProxGD 10853-10898 -> 11109-11149 it/s, FProxGD 10621-10671 -> 10783-10817; caps 768 / 384 /
// 256 / 128 measured between or below; NS level (its trial is fused into A^T R).
constexpr unsigned kRowBlocks = 512;
static inline unsigned row_grid(int64_t n, int lpr) {
  static const unsigned cap = [] {
    const char* e = std::getenv("GLX_ROW_BLOCKS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? (unsigned)v : kRowBlocks;
  }();
  const unsigned g = grid_for(n, 256 / lpr);
  return g < cap ? g : cap;
}
// + one publisher workgroup when the launch carries the scalar packet (the grid reduction's
// partials hold at most kMaxBlocks workgroups). The work workgroups are capped at kMaxBlocks - 1
// with or without the packet, so the rows each workgroup sums, and with them the rounding of the
// trial's sums, do not depend on whether the launch carries it (a device-controlled batch runs
// the same trial without a packet: at n >= 16368 the two grids used to differ by one workgroup
// and the sums by an ulp)
static inline unsigned row_grid_pub(int64_t n, int lpr, const Pub& pub) {
  return std::min<unsigned>(row_grid(n, lpr), (unsigned)kMaxBlocks - 1) + (pub.host ? 1u : 0u);
}

// work items per workgroup of k_finalize_residual (GLX_FIN_PER_BLOCK): one per thread, within
// the 1024-block cap. Measured (profiles/r2_fin*): 512 -> 256 takes C2 from 256 to 512 workgroups,
// +2.3 %; NS and the 1024-row shape sit at the cap either way; 1024-4096 lost 0-24 %.
static int finalize_per_block() {
  static const int per_block = [] {
    const char* e = std::getenv("GLX_FIN_PER_BLOCK");
    const int v = e ? std::atoi(e) : 0;
    return v >= 256 ? v : 256;
  }();
  return per_block;
}
template <typename T>
void launch_finalize_residual(const T* P, int S, const T* B, int nsrc, T* const* R, int64_t ml,
                              const int* gate, int epoch, int gate_mode, const T* cx, int64_t cn,
                              const double* cmax, double* fh, double fh_mu, const double* fh_rn,
                              Red red, hipStream_t st, const double* snap_src, double* snap_dst,
                              int nsnap, int chain, int S0, Ctl ctl, const double* cmax_parts,
                              int cmax_np, int cmax_nv) {
  if (chain && (nsrc != 2 || gate != nullptr)) throw Error{GLX_E_INVALID, "finalize: chain needs 2 ungated sources"};
  if (S0 <= 0) S0 = S;
  const int G = finalize_groups(S > S0 ? S : S0);
  if (G > 8) throw Error{GLX_E_INVALID, "finalize: more than 64 K-split slabs"};
  const int64_t work = ml * G > cn ? ml * G : cn;
  const dim3 grid(grid_for(work, finalize_per_block()));
  T* r1 = nsrc > 1 ? R[1] : nullptr;
  T* r2 = nsrc > 2 ? R[2] : nullptr;
  auto go = [&](auto ns, auto g) {
    hipLaunchKernelGGL((k_finalize_residual<T, decltype(ns)::value, decltype(g)::value>), grid,
                       dim3(256), 0, st, P, S, B, R[0], r1, r2, ml, gate, epoch, gate_mode, cx, cn,
                       cmax, fh, fh_mu, fh_rn, red, snap_src, snap_dst, nsnap, chain, P, S0, ctl,
                       cmax_parts, cmax_np, cmax_nv);
  };
  auto by_g = [&](auto ns) {
    if (G == 1) go(ns, std::integral_constant<int, 1>{});
    else if (G == 2) go(ns, std::integral_constant<int, 2>{});
    else if (G == 4) go(ns, std::integral_constant<int, 4>{});
    else go(ns, std::integral_constant<int, 8>{});
  };
  if (nsrc == 1) by_g(std::integral_constant<int, 1>{});
  else if (nsrc == 2) by_g(std::integral_constant<int, 2>{});
  else by_g(std::integral_constant<int, 3>{});
}
template <typename T>
void launch_finalize_fista(const T* P, int S, const T* Pe, int S0, const T* B, T* Ry, const T* sxo,
                           T* sxo_out, int64_t ml, double a1, double b1, double theta, const T* cx,
                           int64_t cn, const double* cmax, const unsigned* counts, int nl, Red red,
                           hipStream_t st, Ctl ctl, const double* cmax_parts, int cmax_np,
                           int cmax_nv) {
  const int G = finalize_groups(S > S0 ? S : S0);
  if (G > 8) throw Error{GLX_E_INVALID, "finalize: more than 64 K-split slabs"};
  const int64_t work = ml * G > cn ? ml * G : cn;
  const dim3 grid(grid_for(work, 256 * 2));
  auto go = [&](auto g) {
    hipLaunchKernelGGL((k_finalize_fista<T, decltype(g)::value>), grid, dim3(256), 0, st, P, S, Pe,
                       S0, B, Ry, sxo, sxo_out, ml, a1, b1, theta, cx, cn, cmax, counts, nl, red, ctl,
                       cmax_parts, cmax_np, cmax_nv);
  };
  if (G == 1) go(std::integral_constant<int, 1>{});
  else if (G == 2) go(std::integral_constant<int, 2>{});
  else if (G == 4) go(std::integral_constant<int, 4>{});
  else go(std::integral_constant<int, 8>{});
}
template <typename T>
void launch_sum_partials(const T* Gp, int S, T* G, int64_t nl, hipStream_t st) {
  hipLaunchKernelGGL(k_sum_partials<T>, dim3(grid_for(nl, 256 * 4)), dim3(256), 0, st, Gp, S, G, nl);
}
template <typename T>
void launch_prox_pgd(const T* x, const T* g, int S, T* gout, T* p, T* pthr, T* z, int64_t n,
                     int64_t l, double t, double mu, double thres, Red red, hipStream_t st, Pub pub,
                     unsigned* zf) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    hipLaunchKernelGGL((k_prox_pgd<T, decltype(lpr)::value, decltype(epl)::value>),
                       dim3(row_grid_pub(n, lpr, pub)), dim3(256), 0, st, x, g, S, gout, p, pthr, z, zf,
                       n, l, t, t * mu, thres, red, pub);
  });
}
template <typename T>
void launch_trial_split(const T* p, const T* xt, T* pthr, T* z, unsigned* zf, int64_t n, int64_t l,
                        double t, double thres, bool emode, const ShardPub& sp, hipStream_t st) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    hipLaunchKernelGGL((k_trial_split<T, decltype(lpr)::value, decltype(epl)::value>),
                       dim3(row_grid(n, lpr) + (sp.blk != nullptr ? 1u : 0u)), dim3(256), 0, st, p, xt,
                       pthr, z, zf, n, l, t, thres, emode ? 1 : 0, sp);
  });
}
template <typename T>
void launch_fista_split(const T* xc, const T* xk, T* vnext, T* ynext, int64_t nl, double thres,
                        double theta, double theta_next, const ShardPub& sp, hipStream_t st) {
  const int64_t nb = std::min<int64_t>((nl + 255) / 256, 1024);
  hipLaunchKernelGGL(k_fista_split<T>, dim3((unsigned)nb + (sp.blk != nullptr ? 1u : 0u)), dim3(256), 0, st, xc,
                     xk, vnext, ynext, nl, thres, theta, 1.0 - theta_next, theta_next, sp);
}
void launch_shard_combine(const ShardPub& sp, hipStream_t st) {
  hipLaunchKernelGGL(k_shard_combine, dim3(1), dim3(256), 0, st, sp);
}
int finalize_blocks(int64_t ml, int S, int S0, int64_t cn) {
  if (S0 <= 0) S0 = S;
  const int G = finalize_groups(S > S0 ? S : S0);
  const int64_t work = ml * G > cn ? ml * G : cn;
  return (int)grid_for(work, finalize_per_block());
}
int finalize_fista_blocks(int64_t ml, int S, int S0, int64_t cn) {
  const int G = finalize_groups(S > S0 ? S : S0);
  const int64_t work = ml * G > cn ? ml * G : cn;
  return (int)grid_for(work, 256 * 2);
}
int prox_blocks(int64_t n, int64_t l) {
  int b = 0;
  dispatch_row(l, [&](auto lpr, auto) { b = (int)row_grid_pub(n, lpr, Pub{}); });
  return b;
}
template <typename T>
void launch_fista_trial(bool prox, const T* y, const T* g, int S, T* gout, const T* xk, T* xc,
                        T* vnext, T* ynext, int64_t n, int64_t l, double t, double mu, double thres,
                        double theta, double theta_next, double delta, Red red, hipStream_t st,
                        Pub pub, T* ec, unsigned* zf) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    if (prox)
      hipLaunchKernelGGL((k_fista_trial<T, decltype(lpr)::value, decltype(epl)::value, true>),
                         dim3(row_grid_pub(n, lpr, pub)), dim3(256), 0, st, y, g, S, gout, xk, xc,
                         vnext, ynext, n, l, t, t * mu, thres, theta, 1.0 - theta_next, theta_next,
                         delta * delta, delta, red, pub, ec, zf);
    else
      hipLaunchKernelGGL((k_fista_trial<T, decltype(lpr)::value, decltype(epl)::value, false>),
                         dim3(row_grid_pub(n, lpr, pub)), dim3(256), 0, st, y, g, S, gout, xk, xc,
                         vnext, ynext, n, l, t, t * mu, thres, theta, 1.0 - theta_next, theta_next,
                         delta * delta, delta, red, pub, ec, zf);
  });
}
template <typename T>
void launch_prox_plain(const T* w, T* x, int64_t n, int64_t l, double t, double mu, double thres,
                       Red red, hipStream_t st) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    hipLaunchKernelGGL((k_prox_plain<T, decltype(lpr)::value, decltype(epl)::value>),
                       dim3(row_grid(n, lpr)), dim3(256), 0, st, w, x, n, l, t * mu, thres, red);
  });
}
template <typename T>
void launch_rownorm_max(const T* x, int64_t n, int64_t l, Red red, hipStream_t st) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    hipLaunchKernelGGL((k_rownorm_max<T, decltype(lpr)::value, decltype(epl)::value>),
                       dim3(row_grid(n, lpr)), dim3(256), 0, st, x, n, l, red);
  });
}
template <typename T>
void launch_descent(T* x, T* xt, const T* g, int S, int64_t n, int64_t l, double alpha, double mu,
                    double thres, double delta, int mode, Red red, hipStream_t st) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    if (mode == 0)
      hipLaunchKernelGGL((k_descent<T, decltype(lpr)::value, decltype(epl)::value, 0>),
                         dim3(row_grid(n, lpr)), dim3(256), 0, st, x, xt, g, S, n, l, alpha, mu, thres,
                         delta * delta, red);
    else
      hipLaunchKernelGGL((k_descent<T, decltype(lpr)::value, decltype(epl)::value, 1>),
                         dim3(row_grid(n, lpr)), dim3(256), 0, st, x, xt, g, S, n, l, alpha, mu, thres,
                         delta * delta, red);
  });
}
template <typename T>
void launch_fgd_grad(const T* y, const T* gp, int S, T* g, int64_t n, int64_t l, double mu,
                     double delta, Red red, hipStream_t st) {
  dispatch_row(l, [&](auto lpr, auto epl) {
    hipLaunchKernelGGL((k_fgd_grad<T, decltype(lpr)::value, decltype(epl)::value>),
                       dim3(row_grid(n, lpr)), dim3(256), 0, st, y, gp, S, g, n, l, mu, delta * delta,
                       delta, red);
  });
}
template <typename T>
void launch_count_above(const T* x, int64_t nl, const double* maxv, Red red, hipStream_t st) {
  hipLaunchKernelGGL(k_count_above<T>, dim3(grid_for(nl, 256 * 4)), dim3(256), 0, st, x, nl, maxv, red);
}
template <typename T>
void launch_threshold(const T* x, T* xo, int64_t nl, double thres, int* flag, int epoch, hipStream_t st) {
  hipLaunchKernelGGL(k_threshold<T>, dim3(grid_for(nl, 256 * 4)), dim3(256), 0, st, x, xo, nl, thres,
                     flag, epoch);
}
template <typename T>
void launch_thr_axpby(T* xk, const T* vk, T* y, int64_t nl, double thres, double a, double b,
                      hipStream_t st) {
  hipLaunchKernelGGL(k_thr_axpby<T>, dim3(grid_for(nl, 256 * 4)), dim3(256), 0, st, xk, vk, y, nl, thres,
                     a, b);
}
template <typename T>
void launch_fista_v(const T* xk, const T* x, T* v, int64_t nl, double theta, hipStream_t st) {
  hipLaunchKernelGGL(k_fista_v<T>, dim3(grid_for(nl, 256 * 4)), dim3(256), 0, st, xk, x, v, nl, theta);
}
void launch_record_f(const double* s, int i_sumsq, int i_reg, double mu, double* fh, int64_t idx,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_record_f, dim3(1), dim3(64), 0, st, s, i_sumsq, i_reg, mu, fh, idx);
}
void launch_ctl_decide(const Ctl& c, const double* out, double* host, unsigned* host_seq,
                       unsigned seq, hipStream_t st) {
  hipLaunchKernelGGL(k_ctl_decide, dim3(1), dim3(64), 0, st, c, out, host, host_seq, seq);
}

void launch_ctl_seed(double* state, int* abort, double s0, double s1, double s2, double s3,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_ctl_seed, dim3(1), dim3(64), 0, st, state, abort, s0, s1, s2, s3);
}

void launch_publish_pub(const Pub& pub, hipStream_t st) {
  hipLaunchKernelGGL(k_publish_pub, dim3(1), dim3(256), 0, st, pub);
}
void launch_publish(const double* s, int ns, double* host, unsigned* host_seq, unsigned seq,
                    hipStream_t st, const double* s2, int off2, int n2) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, s, ns, host, host_seq, seq, s2, off2,
                     s2 ? n2 : 0);
}

#define GLX_INST(T)                                                                                  \
  template void launch_finalize_residual<T>(const T*, int, const T*, int, T* const*, int64_t,       \
                                            const int*, int, int, const T*, int64_t, const double*, \
                                            double*, double, const double*, Red, hipStream_t,       \
                                            const double*, double*, int, int, int, Ctl,             \
                                            const double*, int, int);                               \
  template void launch_sum_partials<T>(const T*, int, T*, int64_t, hipStream_t);                    \
  template void launch_finalize_fista<T>(const T*, int, const T*, int, const T*, T*, const T*, T*,  \
                                         int64_t, double, double, double, const T*, int64_t,        \
                                         const double*, const unsigned*, int, Red, hipStream_t, Ctl,\
                                         const double*, int, int);                                  \
  template void launch_trial_split<T>(const T*, const T*, T*, T*, unsigned*, int64_t, int64_t,       \
                                      double, double, bool, const ShardPub&, hipStream_t);            \
  template void launch_fista_split<T>(const T*, const T*, T*, T*, int64_t, double, double, double,   \
                                      const ShardPub&, hipStream_t);                                  \
  template void launch_prox_pgd<T>(const T*, const T*, int, T*, T*, T*, T*, int64_t, int64_t,       \
                                   double, double, double, Red, hipStream_t, Pub, unsigned*);       \
  template void launch_fista_trial<T>(bool, const T*, const T*, int, T*, const T*, T*, T*, T*,      \
                                      int64_t, int64_t, double, double, double, double, double,     \
                                      double, Red, hipStream_t, Pub, T*, unsigned*);                \
  template void launch_prox_plain<T>(const T*, T*, int64_t, int64_t, double, double, double, Red,   \
                                     hipStream_t);                                                  \
  template void launch_rownorm_max<T>(const T*, int64_t, int64_t, Red, hipStream_t);                \
  template void launch_descent<T>(T*, T*, const T*, int, int64_t, int64_t, double, double, double,  \
                                  double, int, Red, hipStream_t);                                   \
  template void launch_fgd_grad<T>(const T*, const T*, int, T*, int64_t, int64_t, double, double,   \
                                   Red, hipStream_t);                                               \
  template void launch_count_above<T>(const T*, int64_t, const double*, Red, hipStream_t);          \
  template void launch_threshold<T>(const T*, T*, int64_t, double, int*, int, hipStream_t);        \
  template void launch_thr_axpby<T>(T*, const T*, T*, int64_t, double, double, double, hipStream_t);\
  template void launch_fista_v<T>(const T*, const T*, T*, int64_t, double, hipStream_t);

GLX_INST(double)
GLX_INST(float)

}  // namespace glx
