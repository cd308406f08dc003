// kernels_atr.hip — the gradient contraction A^T R (reference: gl_ProxGD_primal.py:129
// `A.T @ (A @ x - b)`; gl_FProxGD_primal.py:65-66) on MFMA, with the ProxGD / FISTA line-search
// trial fused into its epilogue (k_atr_prox, k_atr_fista), and the VALU fallback for small l.
//
// The K index (rows of A) is on l>>4 and the 16-wide M index (columns of A) on l&15, so lanes
// 0..15 read consecutive columns: a lane loads 4 columns of one row (atr_col) and feeds 4 MFMAs
// whose output rows are those columns. Split-K partials (waves through LDS, workgroups as
// slabs) are summed in a fixed order, so every result is deterministic run to run.
#include <cstdio>

#include "glx_mfma.h"

namespace glx {

// ------------------------------------------------------------------------------------------
// A^T R on MFMA: a wave owns 64 columns of A (= 64 rows of G) x NT 16-col tiles of G.
//   WL = 0: a block = one 64-column panel, its 4 waves split the block's rows (LDS-reduced);
//   WL = 1: a block = four adjacent panels (256 columns) sharing one row range, so the four
//           waves read the same R fragments (L1 hits) and write their slabs directly;
//   WL = 2: as WL 0 with eight waves (512 threads, two waves per SIMD): the block's rows split
//           eight ways, waves 4..7 folded into 0..3 through LDS first (round 4);
//   WL = 3: as WL 0 with a 32-column panel (f64; round 5): twice the panels, so a shape with
//           n / 64 < 256 (C2: 128) fills the chip without K splits and their slab combine.
// blockIdx.y = row split. Needs n % 64 == 0 (n % 256 for WL = 1), m % 4 == 0.
// Gp[split][n][16*NT].
// ------------------------------------------------------------------------------------------
// One 64-column panel of A^T R over this wave's (WL 1: this block's) row range; returns the
// panel's first column. acc[e][nt] holds rows col0 + atr_col(M::row(lane, r), e). For WL 0 the
// block's four waves split the rows (K) and are summed through LDS in the fixed order
// ((w0 + w1) + w2) + w3; afterwards wave w holds the complete sum for e == w in acc[w][*]
// (the other e of a wave are partial and unused), so the four waves share the epilogue.
// (pbx, pby) = (panel, K split) of this block: (blockIdx.x, blockIdx.y) for k_atr_mfma.
// Infinity-Cache hand-off (GemmPlan::atr_keep_mib, a kernel argument; the solver's default is
// kKeepMiB = 192, GLX_ATR_KEEP_MIB overrides it, 0 = off): the last rows a non-temporal A^T R
// pass reads are loaded with the default policy, so that about that many MiB of A stay in the
// 256 MiB Infinity Cache for the next pass over A (A@X) to hit.

// panel width (columns of A = rows of G) of a wave layout, and its MFMA output groups e
template <int WL> constexpr int atr_pw() { return (WL == 3 || WL == 4) ? 32 : 64; }
// waves per workgroup: WL 2 (64-column panel) and WL 4 (32-column panel, round 5) have eight
template <int WL> constexpr int atr_waves() { return (WL == 2 || WL == 4) ? 8 : 4; }
template <int WL> constexpr int atr_ne() { return atr_pw<WL>() / 16; }

template <typename T, int NT, int PF, int WL, bool NTL>
__device__ inline int64_t atr_panel(const T* __restrict__ A, const T* __restrict__ R, int64_t m,
                                    int64_t n, int S, typename MF<T>::acc_t (&acc)[4][NT],
                                    int64_t pbx, int64_t pby, int keep_mib) {
  typedef MF<T> M;
  typedef typename M::acc_t C;
  constexpr int L = 16 * NT;
  constexpr bool RW = WL != 1;   // the block's waves split the rows of one panel
  constexpr int NWV = atr_waves<WL>();
  constexpr int PW = atr_pw<WL>(), NE = atr_ne<WL>();
  static_assert((WL != 3 && WL != 4) || sizeof(T) == 8, "the 32-column panel is f64 (one 16-B load per row)");
  __shared__ C red[RW ? 4 : 1][RW ? 4 * NT : 1][64];   // [wave][e * NT + nt][lane]

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t col0 = RW ? pbx * PW : pbx * 256 + wave * 64;
  const int64_t steps = m / 4;
  const int64_t W = RW ? (int64_t)S * NWV : (int64_t)S;
  const int64_t w = RW ? pby * NWV + wave : pby;
  const int64_t sb = steps * w / W, se = steps * (w + 1) / W;

  const T* ap = A + (sb * 4 + q) * n + col0 + atr_col<T>(i, 0);
  const T* rp = R + (sb * 4 + q) * L + i;

#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[e][nt] = C{};

  // Ring of PF row steps, consumed in place: a step's fragments feed its MFMAs and are then
  // refilled with step s + PF in the same registers, at a clamped offset so that the main
  // loop carries no load predicates (a predicate or a register copy at the loop's back edge
  // makes the compiler drain vmcnt to 0 there). Lookahead = PF - 1 steps.
  const int64_t nst = se - sb;
  T a[PF][4], rb[PF][NT];
  auto lda = [&](const T* p, T (&dst)[4], auto ntl) {
    if constexpr (NE == 2) {   // columns 2i, 2i + 1 (atr_col for e < 2): one 16-B load
      const typename M::vec_t v = load_vec<T, decltype(ntl)::value>(p);
      dst[0] = v[0];
      dst[1] = v[1];
    } else {
      Load4<T, decltype(ntl)::value>::go(p, dst);
    }
  };
  auto ld = [&](int p, int64_t off) {
    off = off < nst ? off : nst - 1;
    lda(ap + off * 4 * n, a[p], std::integral_constant<bool, NTL>{});
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) rb[p][nt] = rp[off * 4 * L + nt * 16];
  };
  auto ld_def = [&](int p, int64_t off) {   // default policy (the Infinity-Cache hand-off)
    off = off < nst ? off : nst - 1;
    lda(ap + off * 4 * n, a[p], std::integral_constant<bool, false>{});
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) rb[p][nt] = rp[off * 4 * L + nt * 16];
  };
  // steps [kt, nst) load with the default policy: keep MiB over the grid's W * (n / 64) waves of
  // 4 rows x 64 columns per step (WL 1: 4 x 256 columns per block step)
  int64_t keep = 0;
  if constexpr (NTL) {
    const int64_t kb = (int64_t)keep_mib << 20;
    keep = kb / ((int64_t)(RW ? W * (n / PW) : W * (n / 256)) * 4 * (RW ? PW : 256) * (int64_t)sizeof(T));
  }
  const int64_t kt = nst - keep;
  auto mma_step = [&](int p) {
#pragma unroll
    for (int e = 0; e < NE; ++e)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[e][nt] = M::mma(a[p][e], rb[p][nt], acc[e][nt]);
  };
  GLX_CLK(1);
  if (nst > 0) {
#pragma unroll
    for (int p = 0; p < PF; ++p) ld(p, p);
    // Trip bounds as wave-uniform 32-bit scalars (readfirstlane): round 3's fused condition
    // `s0 + PF <= nst && (keep == 0 || s0 + 2 PF <= kt)` compiled into an exec-masked loop with
    // an s_nop per MFMA group, and k_atr_prox ran 180 us against round 2's 168 us on one box
    // (profiles/r4_diag/). Loop 1 runs while s0 + PF <= min(nst, kt - PF).
    const int nsti = __builtin_amdgcn_readfirstlane((int)nst);
    const int lim1 = __builtin_amdgcn_readfirstlane(
        keep == 0 ? (int)nst : (int)(kt - PF < nst ? kt - PF : nst));
    int s0 = 0;
    for (; s0 + PF <= lim1; s0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        mma_step(p);
        ld(p, s0 + p + PF);
      }
    }
    for (; s0 + PF <= nsti; s0 += PF) {   // the kept tail (only with keep > 0)
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        mma_step(p);
        ld_def(p, s0 + p + PF);
      }
    }
#pragma unroll
    for (int p = 0; p < PF - 1; ++p)
      if (s0 + p < nst) mma_step(p);
  }
  GLX_CLK(2);

  if constexpr (WL == 2 || WL == 4) {   // waves 4..7 into 0..3: acc(w) + acc(w + 4)
    if (wave >= 4) {
#pragma unroll
      for (int e = 0; e < NE; ++e)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) red[wave - 4][e * NT + nt][lane] = acc[e][nt];
    }
    __syncthreads();
    if (wave < 4) {
#pragma unroll
      for (int e = 0; e < NE; ++e)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[e][nt] += red[wave][e * NT + nt][lane];
    }
    __syncthreads();
  }
  if (RW) {
    if (wave < 4) {
#pragma unroll
      for (int e = 0; e < NE; ++e)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) red[wave][e * NT + nt][lane] = acc[e][nt];
    }
    __syncthreads();
    if (wave < NE) {   // (WL 2: waves 4..7 hold no rows from here on; WL 3: waves 2, 3)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        C v = red[0][wave * NT + nt][lane];
#pragma unroll
        for (int s = 1; s < 4; ++s) v += red[s][wave * NT + nt][lane];
#pragma unroll
        for (int e = 0; e < NE; ++e)
          if (e == wave) acc[e][nt] = v;   // static register index; e == wave selects one
      }
    }
  }
  return col0;
}

// K splits of a fused A^T R (WL 0, S > 1): a 1-D grid of n/64 panels x S splits (+ the
// publisher). Every block stores its panel rows (wave w: rows e == w) into slab `split` of Gp;
// the block that arrives last on its panel's counter sums the S slabs in slab order (the
// order of slab_sum, so G is bit-identical to the unfused path) and runs the trial epilogue.
// Hand-off: sc1 (agent-scope) stores, vmcnt(0), a workgroup barrier, one agent-scope add per
// block; the last arriver loads with sc1 after a barrier (MI355X_MICROARCH.md "Valid forms",
// row 1). Returns false in the blocks that are not last: they leave the kernel without joining
// the grid reduction, which counts only the n/64 panel owners (+ the publisher; grid_reduce's
// nparts), so S is not bounded by the kMaxBlocks partials row (round 3: C2 takes more splits).
// *slot = the panel: the trial's scalar sums come out in panel order, bit-identical from run to
// run whatever the arrival order (a last arriver at its own block slot made their summation
// order depend on timing), and equal to the earlier form that also reduced identity partials.
template <typename T, int NT>
__device__ inline bool atr_split_combine(typename MF<T>::acc_t (&acc)[4][NT], T* __restrict__ Gp,
                                         int64_t n, int S, int64_t panel, int64_t split,
                                         unsigned* __restrict__ pcnt, int* slot) {
  typedef MF<T> M;
  constexpr int L = 16 * NT;
  __shared__ int last;
  __shared__ unsigned arrival;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15;
  const int64_t col0 = panel * 64;
  const int64_t nl = n * L;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (e != wave) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = col0 + atr_col<T>(M::row(lane, r), e);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        __hip_atomic_store(Gp + split * nl + row * L + nt * 16 + i, acc[e][nt][r], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    arrival = __hip_atomic_fetch_add(pcnt + panel, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = arrival == (unsigned)S - 1;
  }
  __syncthreads();
  if (!last) return false;
  *slot = (int)panel;
  // Round 5: every slab load of the wave's 4 x NT elements issued before the first add (S <= 8,
  // atr_prox_ok), one round trip instead of S - 1 dependent ones per element; same slab order
  constexpr int KS = NT == 1 ? 8 : 4;   // slabs per load batch (register budget)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (e != wave) continue;
    for (int k0 = 0; k0 < S; k0 += KS) {
      T sv[4][NT][KS];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = col0 + atr_col<T>(M::row(lane, r), e);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const T* g = Gp + row * L + nt * 16 + i;
#pragma unroll
          for (int k = 0; k < KS; ++k)
            sv[r][nt][k] = k0 + k < S ? __hip_atomic_load(g + (int64_t)(k0 + k) * nl, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : T(0);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          T v = k0 == 0 ? sv[r][nt][0] : acc[e][nt][r] + sv[r][nt][0];
#pragma unroll
          for (int k = 1; k < KS; ++k)
            if (k0 + k < S) v = v + sv[r][nt][k];
          acc[e][nt][r] = v;
        }
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(pcnt + panel, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

template <typename T, int NT, int PF, int WL, bool NTL>
__global__ __launch_bounds__(atr_waves<WL>() * 64) void k_atr_mfma(const T* __restrict__ A, const T* __restrict__ R,
                                                  T* __restrict__ Gp, int64_t m, int64_t n, int S,
                                                  int keep_mib) {
  typedef MF<T> M;
  constexpr int L = 16 * NT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15;
  typename M::acc_t acc[4][NT];
  const int64_t col0 = atr_panel<T, NT, PF, WL, NTL>(A, R, m, n, S, acc, blockIdx.x, blockIdx.y, keep_mib);
  T* gout = Gp + (int64_t)blockIdx.y * n * L;
#pragma unroll
  for (int e = 0; e < atr_ne<WL>(); ++e) {
    if (WL != 1 && e != wave) continue;   // WL 0 / 2 / 3: wave w < NE owns the rows e == w
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t grow = col0 + atr_col<T>(M::row(lane, r), e);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) gout[grow * L + nt * 16 + i] = acc[e][nt][r];
    }
  }
}

// ProxGD's line-search trial fused into A^T R (WL 0, one K split): once the block's LDS
// reduction leaves each wave w the 16 gradient rows e == w of its panel — lane (i, q) holding
// columns i and 16 + i of 4 rows, exactly the 16-lanes-per-row layout of k_prox_pgd — every
// wave writes its rows of G and runs the trial on them (prox_pgd_row, the same arithmetic as
// k_prox_pgd) with x = the thresholded iterate; the six trial sums are reduced over the grid.
template <typename T, int NT, int PF, bool NTL, bool SPLIT, int WL>
__global__ __launch_bounds__(atr_waves<WL>() * 64, ((WL == 0 || WL == 3) && sizeof(T) == 8) ? 2 : 1) void k_atr_prox(const T* __restrict__ A, const T* __restrict__ R,
                                                  T* __restrict__ G, int64_t m, int64_t n,
                                                  const T* __restrict__ x, T* __restrict__ p,
                                                  T* __restrict__ pthr, T* __restrict__ z,
                                                  double t_, double tmu_, double thres_, Red red,
                                                  Pub pub, int S, T* __restrict__ Gp,
                                                  unsigned* __restrict__ pcnt,
                                                  unsigned* __restrict__ zf, int keep_mib) {
  // Cancelled by a device-side decision (solver.cpp dc_run): nothing is computed or stored, no
  // counter or ticket is touched. (Testing the flag after the main loop instead measured no
  // faster and would spend a whole pass per cancelled launch.) The decision record still goes
  // to the host: the cancelling decision's own.
  GLX_CLK(0);
  if (red_skipped(red)) {
    if (pub.host != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
      publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq);
    return;
  }
  // the extra workgroup (n / 64 * S + 1 in all); with K splits only the panel owners and the
  // publisher reduce (nparts)
  const int nparts = SPLIT ? (int)(n / 64) + (pub.host ? 1 : 0) : -1;
  constexpr int NW = atr_waves<WL>();
  if (publisher_first<6, 0x8u, NW>(pub, red, nparts)) return;
  typedef MF<T> M;
  constexpr int L = 16 * NT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15;
  typename M::acc_t acc[4][NT];
  const int64_t bid = (int64_t)blockIdx.x - (pub.host ? 1 : 0);
  const int64_t panel = SPLIT ? bid / S : bid, split = SPLIT ? bid % S : 0;
  // Round 4: the row results are stored after the trial sums have been handed to grid_reduce,
  // whose vmcnt(0) drain then waits for six partials instead of wave 0's G / p / p_thr / z stores
  // (the fused epilogue took 8-10 us of the kernel at NS and C2, profiles/r4_clk). Loading the
  // iterate rows before the main loop instead of after it measured 4-5 us slower at NS (+18
  // VGPRs live through the ring, profiles/r4_ab2).
  const int64_t col0 = atr_panel<T, NT, PF, WL, NTL>(A, R, m, n, SPLIT ? S : 1, acc, panel, split, keep_mib);
  GLX_CLK(4);
  T xa[4][NT];
#pragma unroll
  for (int e = 0; e < atr_ne<WL>(); ++e) {
    if (e != wave) continue;   // wave w owns the rows e == w (4 per lane group)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = col0 + atr_col<T>(M::row(lane, r), e);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) xa[r][nt] = x[row * L + nt * 16 + i];
    }
  }
  double accr[6] = {0.0, 0.0, 0.0, -__builtin_inf(), 0.0, 0.0};
  int slot = work_slot(pub);
  if constexpr (SPLIT) {   // a separate instantiation: the S = 1 kernel keeps 2 blocks per CU
    if (!atr_split_combine<T, NT>(acc, Gp, n, S, panel, split, pcnt, &slot)) return;
  }
  const T t = (T)t_, tmu = (T)tmu_, thres = (T)thres_;
  T gs[4][NT], ps[4][NT], pts[4][NT], zs[4][NT];
  unsigned rows_e[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int e = 0; e < atr_ne<WL>(); ++e) {
    if (e != wave) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bool ok[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        gs[r][nt] = acc[e][nt][r];
        ok[nt] = true;
      }
      rows_e[r] = prox_pgd_row<T, 16, NT>(xa[r], gs[r], ok, true, i, t, tmu, thres, ps[r], pts[r], zs[r],
                                          accr, zf != nullptr);
    }
  }
  GLX_CLK(5);
  grid_reduce<6, 0x8u, NW>(accr, red, slot, nparts);
  __shared__ unsigned msk[64];   // the panel's row masks of e (column bitmaps, zf_store_panel)
#pragma unroll
  for (int e = 0; e < atr_ne<WL>(); ++e) {
    if (e != wave) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = col0 + atr_col<T>(M::row(lane, r), e);
      if (zf != nullptr && i == 0) {
        zf[row] = rows_e[r];
        msk[row - col0] = rows_e[r];
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        G[row * L + nt * 16 + i] = gs[r][nt];
        p[row * L + nt * 16 + i] = ps[r][nt];
        pthr[row * L + nt * 16 + i] = pts[r][nt];
        z[row * L + nt * 16 + i] = zs[r][nt];
      }
    }
  }
  if (zf != nullptr) {
    __syncthreads();
    zf_store_panel<atr_pw<WL>()>(msk, zf, n, L, col0);
  }
  GLX_CLK(3);
}

// FISTA's backtracking trial fused into A^T R the same way (WL 0, one K split): each wave runs
// fista_row (the arithmetic of k_fista_trial) on its 16 gradient rows, with y the extrapolated
// point and xk the current iterate; writes G, xc, v_next, y_next and reduces the four sums.
template <typename T, int NT, int PF, bool NTL, bool SPLIT, int WL>
__global__ __launch_bounds__(atr_waves<WL>() * 64, ((WL == 0 || WL == 3) && sizeof(T) == 8) ? 2 : 1) void k_atr_fista(const T* __restrict__ A, const T* __restrict__ R,
                                                   T* __restrict__ G, int64_t m, int64_t n,
                                                   const T* __restrict__ y, const T* __restrict__ xk,
                                                   T* __restrict__ xc, T* __restrict__ vnext,
                                                   T* __restrict__ ynext, double t_, double tmu_,
                                                   double thres_, double theta_, double a1_,
                                                   double b1_, Red red, Pub pub, int S,
                                                   T* __restrict__ Gp, unsigned* __restrict__ pcnt,
                                                   T* __restrict__ ec, unsigned* __restrict__ zf,
                                                   int keep_mib) {
  if (red_skipped(red)) {   // cancelled by a device-side decision (as k_atr_prox)
    if (pub.host != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
      publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq);
    return;
  }
  const int nparts = SPLIT ? (int)(n / 64) + (pub.host ? 1 : 0) : -1;   // see k_atr_prox
  constexpr int NW = atr_waves<WL>();
  if (publisher_first<4, 0x8u, NW>(pub, red, nparts)) return;
  typedef MF<T> M;
  constexpr int L = 16 * NT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15;
  typename M::acc_t acc[4][NT];
  const int64_t bid = (int64_t)blockIdx.x - (pub.host ? 1 : 0);
  const int64_t panel = SPLIT ? bid / S : bid, split = SPLIT ? bid % S : 0;
  const int64_t col0 = atr_panel<T, NT, PF, WL, NTL>(A, R, m, n, SPLIT ? S : 1, acc, panel, split, keep_mib);
  double accr[4] = {0.0, 0.0, 0.0, -__builtin_inf()};
  int slot = work_slot(pub);
  if constexpr (SPLIT) {   // fixed reduction slots, see atr_split_combine
    if (!atr_split_combine<T, NT>(acc, Gp, n, S, panel, split, pcnt, &slot)) return;
  }
  const T t = (T)t_, tmu = (T)tmu_, thres = (T)thres_, theta = (T)theta_, a1 = (T)a1_, b1 = (T)b1_;
  __shared__ unsigned msk[64];   // the panel's row masks of e_c (column bitmaps, zf_store_panel)
#pragma unroll
  for (int e = 0; e < atr_ne<WL>(); ++e) {
    if (e != wave) continue;   // wave w owns the rows e == w
    T ya[4][NT], xa[4][NT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = col0 + atr_col<T>(M::row(lane, r), e);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        ya[r][nt] = y[row * L + nt * 16 + i];
        xa[r][nt] = xk[row * L + nt * 16 + i];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = col0 + atr_col<T>(M::row(lane, r), e);
      T gv[NT], xcv[NT], vnv[NT], ynv[NT], ecv[NT];
      bool ok[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        gv[nt] = acc[e][nt][r];
        ok[nt] = true;
        G[row * L + nt * 16 + i] = gv[nt];
      }
      const unsigned rowe = fista_row<T, 16, NT, true>(ya[r], gv, xa[r], ok, true, i, t, tmu, thres, theta,
                                                   a1, b1, T(0), T(0), xcv, vnv, ynv, accr,
                                                   ec != nullptr ? ecv : nullptr);
      if (zf != nullptr && i == 0) {
        zf[row] = rowe;
        msk[row - col0] = rowe;
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        xc[row * L + nt * 16 + i] = xcv[nt];
        vnext[row * L + nt * 16 + i] = vnv[nt];
        ynext[row * L + nt * 16 + i] = ynv[nt];
        if (ec != nullptr) ec[row * L + nt * 16 + i] = ecv[nt];
      }
    }
  }
  grid_reduce<4, 0x8u, NW>(accr, red, slot, nparts);
  if (zf != nullptr) {   // (grid_reduce's barriers ordered the msk stores above)
    __syncthreads();
    zf_store_panel<atr_pw<WL>()>(msk, zf, n, L, col0);
  }
}

// A^T R on VALU: a thread owns E consecutive columns of A over a row range; R[row][c0..c0+LB)
// is wave-uniform (scalar loads). Gp[blockIdx.y][n][l].
template <typename T, int LB, bool VEC>
__global__ __launch_bounds__(256) void k_atr_valu(const T* __restrict__ A, const T* __restrict__ R,
                                                  T* __restrict__ Gp, int64_t m, int64_t n,
                                                  int64_t l, int c0, int S) {
  constexpr int E = VEC ? (16 / (int)sizeof(T)) : 1;
  const int64_t col = ((int64_t)blockIdx.x * 256 + threadIdx.x) * E;
  const int s = blockIdx.y;
  const int64_t rb = m * s / S, re = m * (s + 1) / S;
  const int nc = (int)((l - c0) < LB ? (l - c0) : LB);
  const bool active = col < n;
  const int64_t ccol = active ? col : 0;

  T acc[E][LB];
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int c = 0; c < LB; ++c) acc[e][c] = T(0);

  const T* ap = A + rb * n + ccol;
  const T* rp = R + rb * l + c0;
#pragma unroll 4
  for (int64_t row = rb; row < re; ++row) {
    T a[E];
    if constexpr (VEC) {
      typedef typename MF<T>::vec_t V;
      const V v = *reinterpret_cast<const V*>(ap);
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] = v[e];
    } else {
      a[0] = *ap;
    }
    T rv[LB];
#pragma unroll
    for (int c = 0; c < LB; ++c) rv[c] = (c < nc) ? rp[c] : T(0);
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int c = 0; c < LB; ++c) acc[e][c] = __builtin_fma(a[e], rv[c], acc[e][c]);
    ap += n;
    rp += l;
  }
  if (!active) return;
  T* gout = Gp + (int64_t)s * n * l;
#pragma unroll
  for (int e = 0; e < E; ++e)
#pragma unroll
    for (int c = 0; c < LB; ++c)
      if (c < nc) gout[(col + e) * l + c0 + c] = acc[e][c];
}


template <typename T, int LB>
static void atr_valu_lb(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int64_t cols_per_block = 256 * (p.atr_vec ? E : 1);
  const dim3 grid((unsigned)cdiv(p.n, cols_per_block), (unsigned)p.atr_S);
  for (int64_t c0 = 0; c0 < p.l; c0 += LB) {
    if (p.atr_vec)
      glx_launch((k_atr_valu<T, LB, true>), grid, dim3(256), 0, st, A, R, Gp, p.m, p.n,
                         p.l, (int)c0, p.atr_S);
    else
      glx_launch((k_atr_valu<T, LB, false>), grid, dim3(256), 0, st, A, R, Gp, p.m, p.n,
                         p.l, (int)c0, p.atr_S);
  }
}

template <typename T, int NT, int PF, int WL, bool NTL>
static void atr_mfma_go(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st) {
  const dim3 grid((unsigned)(p.n / (WL == 1 ? 256 : atr_pw<WL>())), (unsigned)p.atr_S);
  static const size_t pad = lds_pad(k_atr_mfma<T, NT, PF, WL, NTL>, "GLX_ATR_LDS_PAD");
  glx_launch((k_atr_mfma<T, NT, PF, WL, NTL>), grid, dim3(atr_waves<WL>() * 64), pad, st, A, R, Gp, p.m, p.n, p.atr_S,
             p.atr_keep_mib);
}

// Round 6: only the tiles the planner picks are built — the f64
// default (WL 0, PF 8; non-temporal A beyond the Infinity Cache), the f32 default (WL 1, PF 4,
// non-temporal), the fp32 fused trial's eight-wave panel (WL 2) and the f64 32-column panel
// (WL 3). The measured-slower ring depths (PF 2-6) and the 8-wave 32-column panel (WL 4) of
// rounds 1-5 are gone; their numbers stay in DESIGN.md's tuning record.
// the switch key of a plan's A^T R tile: NTL * 1000 + WL * 100 + PF
static inline int atr_key(const GemmPlan& p) { return p.atr_ntl * 1000 + p.atr_wl * 100 + p.atr_pf; }

template <typename T, int NT>
static void atr_mfma_nt(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st) {
  switch (atr_key(p)) {
    case 8: atr_mfma_go<T, NT, 8, 0, false>(p, A, R, Gp, st); break;
    case 1008: atr_mfma_go<T, NT, 8, 0, true>(p, A, R, Gp, st); break;
    case 1104: atr_mfma_go<T, NT, 4, 1, true>(p, A, R, Gp, st); break;
    case 1208: atr_mfma_go<T, NT, 8, 2, true>(p, A, R, Gp, st); break;
    case 308:
    case 1308:
      if constexpr (sizeof(T) == 8) {
        if (p.atr_ntl) atr_mfma_go<T, NT, 8, 3, true>(p, A, R, Gp, st);
        else atr_mfma_go<T, NT, 8, 3, false>(p, A, R, Gp, st);
        break;
      }
      throw Error{GLX_E_INVALID, "A^T R: the 32-column panel is f64"};
    default:
      throw Error{GLX_E_INVALID, "A^T R: tile WL" + std::to_string(p.atr_wl) + " PF" + std::to_string(p.atr_pf) +
                                     " NTL" + std::to_string(p.atr_ntl) + " is not built (round 6 pruning)"};
  }
}

template <typename T>
void launch_atr(const GemmPlan& p, const T* A, const T* R, T* Gp, hipStream_t st) {
  if (p.atr_kind == 3) {
    switch (p.atr_lb) {
      case 1: atr_valu_lb<T, 1>(p, A, R, Gp, st); break;
      case 2: atr_valu_lb<T, 2>(p, A, R, Gp, st); break;
      case 4: atr_valu_lb<T, 4>(p, A, R, Gp, st); break;
      default: atr_valu_lb<T, 8>(p, A, R, Gp, st); break;
    }
    return;
  }
  if (p.l == 16) atr_mfma_nt<T, 1>(p, A, R, Gp, st);
  else atr_mfma_nt<T, 2>(p, A, R, Gp, st);
}


int atr_prox_slots(const GemmPlan& p, bool pub) {
  return (int)(p.n / (p.atr_wl == 3 ? 32 : 64)) + (pub ? 1 : 0);
}

bool atr_prox_ok(const GemmPlan& p) {
  if (p.atr_wl == 3)   // the 32-column panel: f64, no K splits (session_plan)
    return p.atr_kind == 1 && p.esize == 8 && p.atr_S == 1 && (p.l == 16 || p.l == 32) &&
           p.n % 32 == 0 && p.n / 32 < kMaxBlocks;
  return p.atr_kind == 1 && (p.atr_wl == 0 || p.atr_wl == 2) && p.atr_S >= 1 && p.atr_S <= 8 &&
         (p.l == 16 || p.l == 32) && p.n % 64 == 0 &&
         p.n / 64 < kMaxBlocks &&   // reducing slots (one per panel) + the publisher
         (p.atr_S == 1 || env_int("GLX_ATR_FUSE_SPLIT", 1) != 0);
}

template <typename T, int NT, int PF, bool NTL, int WL>
static void atr_prox_go(const GemmPlan& p, const T* A, const T* R, T* G, const T* x, T* pp,
                        T* pthr, T* z, double t, double mu, double thres, Red red, hipStream_t st,
                        Pub pub, T* Gp, unsigned* pcnt, unsigned* zf) {
  const dim3 grid((unsigned)(p.n / atr_pw<WL>() * p.atr_S + (pub.host ? 1 : 0)));
  const dim3 block(atr_waves<WL>() * 64);
  if (WL != 3 && WL != 4 && p.atr_S > 1) {
    glx_launch((k_atr_prox<T, NT, PF, NTL, true, WL>), grid, block, 0, st, A, R, G, p.m,
                       p.n, x, pp, pthr, z, t, t * mu, thres, red, pub, p.atr_S, Gp, pcnt, zf, p.atr_keep_mib);
    return;
  }
  static const size_t pad = lds_pad(k_atr_prox<T, NT, PF, NTL, false, WL>, "GLX_ATR_LDS_PAD");
  glx_launch((k_atr_prox<T, NT, PF, NTL, false, WL>), grid, block, pad, st, A, R, G, p.m,
                     p.n, x, pp, pthr, z, t, t * mu, thres, red, pub, 1, Gp, pcnt, zf, p.atr_keep_mib);
}
template <typename T, int NT>
static void atr_prox_nt(const GemmPlan& p, const T* A, const T* R, T* G, const T* x, T* pp,
                        T* pthr, T* z, double t, double mu, double thres, Red red, hipStream_t st,
                        Pub pub, T* Gp, unsigned* pcnt, unsigned* zf) {
  // the planner's fused tiles only (see atr_mfma_nt): f64 WL 0 PF 8 (+ non-temporal), WL 3
  // (32-column panel); WL 2 non-temporal (fp32's eight-wave panel; f64 through GLX_ATR_VARIANT)
  const int code = atr_key(p);
  if constexpr (sizeof(T) == 8) {
    switch (code) {
      case 8: atr_prox_go<T, NT, 8, false, 0>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf); return;
      case 308: atr_prox_go<T, NT, 8, false, 3>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf); return;
      case 1308: atr_prox_go<T, NT, 8, true, 3>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf); return;
      default: break;
    }
  }
  switch (code) {
    case 1008: atr_prox_go<T, NT, 8, true, 0>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf); return;
    case 1208: atr_prox_go<T, NT, 8, true, 2>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf); return;
    default:
      throw Error{GLX_E_INVALID, "fused A^T R + trial: tile code " + std::to_string(code) + " is not built"};
  }
}
template <typename T>
void launch_atr_prox(const GemmPlan& p, const T* A, const T* R, T* G, const T* x, T* pp, T* pthr,
                     T* z, double t, double mu, double thres, Red red, hipStream_t st, Pub pub,
                     T* Gp, unsigned* pcnt, unsigned* zf) {
  if (p.atr_S > 1 && (Gp == nullptr || pcnt == nullptr))
    throw Error{GLX_E_INVALID, "fused A^T R with K splits needs slab and counter buffers"};
  if (p.l == 16) atr_prox_nt<T, 1>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf);
  else atr_prox_nt<T, 2>(p, A, R, G, x, pp, pthr, z, t, mu, thres, red, st, pub, Gp, pcnt, zf);
}

template <typename T, int NT, int PF, bool NTL, int WL>
static void atr_fista_go(const GemmPlan& p, const T* A, const T* R, T* G, const T* y, const T* xk,
                         T* xc, T* vn, T* yn, double t, double mu, double thres, double theta,
                         double theta_next, Red red, hipStream_t st, Pub pub, T* Gp, unsigned* pcnt,
                         T* ec, unsigned* zf) {
  const dim3 grid((unsigned)(p.n / atr_pw<WL>() * p.atr_S + (pub.host ? 1 : 0)));
  const dim3 block(atr_waves<WL>() * 64);
  if (WL != 3 && WL != 4 && p.atr_S > 1) {
    glx_launch((k_atr_fista<T, NT, PF, NTL, true, WL>), grid, block, 0, st, A, R, G, p.m,
                       p.n, y, xk, xc, vn, yn, t, t * mu, thres, theta, 1.0 - theta_next,
                       theta_next, red, pub, p.atr_S, Gp, pcnt, ec, zf, p.atr_keep_mib);
    return;
  }
  static const size_t pad = lds_pad(k_atr_fista<T, NT, PF, NTL, false, WL>, "GLX_ATR_LDS_PAD");
  glx_launch((k_atr_fista<T, NT, PF, NTL, false, WL>), grid, block, pad, st, A, R, G, p.m,
                     p.n, y, xk, xc, vn, yn, t, t * mu, thres, theta, 1.0 - theta_next, theta_next,
                     red, pub, 1, Gp, pcnt, ec, zf, p.atr_keep_mib);
}
template <typename T, int NT>
static void atr_fista_nt(const GemmPlan& p, const T* A, const T* R, T* G, const T* y, const T* xk,
                         T* xc, T* vn, T* yn, double t, double mu, double thres, double theta,
                         double theta_next, Red red, hipStream_t st, Pub pub, T* Gp, unsigned* pcnt,
                         T* ec, unsigned* zf) {
  const int code = atr_key(p);   // the tiles of atr_prox_nt
  if constexpr (sizeof(T) == 8) {
    switch (code) {
      case 8: atr_fista_go<T, NT, 8, false, 0>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf); return;
      case 308: atr_fista_go<T, NT, 8, false, 3>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf); return;
      case 1308: atr_fista_go<T, NT, 8, true, 3>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf); return;
      default: break;
    }
  }
  switch (code) {
    case 1008: atr_fista_go<T, NT, 8, true, 0>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf); return;
    case 1208: atr_fista_go<T, NT, 8, true, 2>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf); return;
    default:
      throw Error{GLX_E_INVALID, "fused A^T R + FISTA trial: tile code " + std::to_string(code) + " is not built"};
  }
}
template <typename T>
void launch_atr_fista(const GemmPlan& p, const T* A, const T* R, T* G, const T* y, const T* xk,
                      T* xc, T* vn, T* yn, double t, double mu, double thres, double theta,
                      double theta_next, Red red, hipStream_t st, Pub pub, T* Gp, unsigned* pcnt,
                         T* ec, unsigned* zf) {
  if (p.atr_S > 1 && (Gp == nullptr || pcnt == nullptr))
    throw Error{GLX_E_INVALID, "fused A^T R with K splits needs slab and counter buffers"};
  if (p.l == 16) atr_fista_nt<T, 1>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf);
  else atr_fista_nt<T, 2>(p, A, R, G, y, xk, xc, vn, yn, t, mu, thres, theta, theta_next, red, st, pub, Gp, pcnt, ec, zf);
}

template void launch_atr<double>(const GemmPlan&, const double*, const double*, double*, hipStream_t);
template void launch_atr_fista<double>(const GemmPlan&, const double*, const double*, double*,
                                       const double*, const double*, double*, double*, double*,
                                       double, double, double, double, double, Red, hipStream_t, Pub,
                                       double*, unsigned*, double*, unsigned*);
template void launch_atr_fista<float>(const GemmPlan&, const float*, const float*, float*,
                                      const float*, const float*, float*, float*, float*, double,
                                      double, double, double, double, Red, hipStream_t, Pub,
                                      float*, unsigned*, float*, unsigned*);
template void launch_atr_prox<double>(const GemmPlan&, const double*, const double*, double*,
                                      const double*, double*, double*, double*, double, double,
                                      double, Red, hipStream_t, Pub, double*, unsigned*, unsigned*);
template void launch_atr_prox<float>(const GemmPlan&, const float*, const float*, float*,
                                     const float*, float*, float*, float*, double, double, double,
                                     Red, hipStream_t, Pub, float*, unsigned*, unsigned*);
template void launch_atr<float>(const GemmPlan&, const float*, const float*, float*, hipStream_t);


}  // namespace glx

GLX_CLK_READER(glx_probe_clock_atr)
