// kernels_gemm.hip — the residual contraction of the prox-grad iteration on CDNA4 (gfx950) and
// the launch planner of both dense products.
//
//   A @ X   (reference: gl_ProxGD_primal.py:25,61,129 — `A @ x`):   M = m, K = n, N = l
//   A^T R   (reference: gl_ProxGD_primal.py:129 — `A.T @ (...)`):  M = n, K = m, N = l
//           (kernels in kernels_atr.hip; the LDS-DMA A @ X tile in kernels_axdma.hip)
//
// Both stream A (m x n, row-major, 1 GiB at the north-star size) once per launch. A^T R and
// A @ X with one right-hand side (l/4 flop/B in fp64) are HBM-bound; A @ X batching 2-3
// right-hand sides per pass (the line-search trial and the next gradient residual) is
// MFMA-bound at l = 32 (v_mfma_f64_16x16x4f64 / v_mfma_f32_16x16x4f32).
//
// MFMA 16x16x4 operand maps (cdna_hip_programming.md §3): lane l supplies A_op[l&15][l>>4] and
// B_op[l>>4][l&15]; the C/D map is row=(l>>4)+4r (f64) or 4(l>>4)+r (f32), col=l&15.
//
// A @ X: the K index sits on l>>4, i.e. the 16 lanes of a k-slice live in 16 different rows of
// A. Each lane loads VPL x 16 contiguous bytes of its row and feeds them to consecutive MFMAs
// (k permuted inside a chunk; X is read with the same permutation, so the sum is unchanged).
//   kind 1/2 — X gathered by every wave into registers (2: quad loads + ds_bpermute);
//   kind 5   — X staged once per block in LDS, natural [k][col] order, conflict-free padding;
//              the default (f64: 8-wave blocks, f32: 4-wave blocks with a 3-deep ring);
//   kind 8   — (f64) A AND X staged in LDS by LDS-DMA, whole 256-B row pieces per wave
//              instruction (k_ax_dma). Kinds 6/7 (pipelined X, sparse barriers) measured slower
//              in round 1 and were removed (tuning record).
// All main loops keep their register rings predicate-free and consume each ring slot in place
// (no vmcnt(0) drain at the back edge). Split-K partials (waves through LDS, workgroups as
// slabs) are summed in a fixed order, so every result is deterministic run to run.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "glx_mfma.h"

namespace glx {


template <typename T, int MT, int NT, int NSRC, int PF, bool QUAD, bool NTL, int VPL>
__global__ __launch_bounds__(256) void k_ax_mfma(const T* __restrict__ A, const T* __restrict__ X0,
                                                 const T* __restrict__ X1, const T* __restrict__ X2,
                                                 T* __restrict__ P, int64_t m, int64_t n,
                                                 int64_t chunks, int S, int gx, int xmap,
                                                 const int* __restrict__ gate, int epoch) {
  typedef MF<T> M;
  typedef typename M::vec_t V;
  typedef typename M::acc_t C;
  constexpr int E = M::E;
  constexpr int EL = VPL * E;   // contiguous k values a lane streams from its row per chunk
  constexpr int CK = 4 * EL;    // k per chunk
  constexpr int L = 16 * NT;    // == l
  constexpr int NC = NT * NSRC;
  if (!gate_live(gate, epoch)) return;
  int bx, by;
  if (!ax_block(xmap, gx, S, bx, by)) return;   // padding block of the XCD map (block-uniform)
  __shared__ C red[MT * NC][64];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t row0 = (int64_t)bx * (16 * MT);
  const int64_t W = (int64_t)S * 4;
  const int64_t w = (int64_t)by * 4 + wave;
  const int64_t cb = chunks * w / W, ce = chunks * (w + 1) / W;

  const int lrow = QUAD ? (lane >> 2) : i;
  const int lchk = QUAD ? (lane & 3) : q;
  const int src = i * 4 + q;  // QUAD: lane holding (row i, chunk q)
  const T* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int64_t r = row0 + mt * 16 + lrow;
    r = r < m ? r : m - 1;
    ap[mt] = A + r * n + cb * CK + (int64_t)lchk * EL;
  }
  const int64_t xoff = (cb * CK + (int64_t)q * EL) * L + i;
  const T* xp[NSRC];
  xp[0] = X0 + xoff;
  if (NSRC > 1) xp[1] = X1 + xoff;
  if (NSRC > 2) xp[2] = X2 + xoff;

  C acc[MT][NC];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[mt][c] = C{};

  V a[PF][MT][VPL];
  T xb[PF][EL][NC];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    if (cb + p < ce) {
      const int64_t off = (int64_t)p * CK;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int v = 0; v < VPL; ++v) a[p][mt][v] = load_vec<T, NTL>(ap[mt] + off + v * E);
#pragma unroll
      for (int e = 0; e < EL; ++e)
#pragma unroll
        for (int c = 0; c < NC; ++c) xb[p][e][c] = xp[c / NT][off * L + e * L + (c % NT) * 16];
    }
  }
  for (int64_t c0 = cb; c0 < ce; c0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int64_t c = c0 + p;
      if (c < ce) {
        V av[MT][VPL];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int v = 0; v < VPL; ++v) av[mt][v] = QUAD ? bpermute_vec(a[p][mt][v], src) : a[p][mt][v];
        T xv[EL][NC];
#pragma unroll
        for (int e = 0; e < EL; ++e)
#pragma unroll
          for (int cc = 0; cc < NC; ++cc) xv[e][cc] = xb[p][e][cc];
        if (c + PF < ce) {   // refill this ring slot with chunk c + PF
          const int64_t off = (c + PF - cb) * CK;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int v = 0; v < VPL; ++v) a[p][mt][v] = load_vec<T, NTL>(ap[mt] + off + v * E);
#pragma unroll
          for (int e = 0; e < EL; ++e)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) xb[p][e][cc] = xp[cc / NT][off * L + e * L + (cc % NT) * 16];
        }
#pragma unroll
        for (int v = 0; v < VPL; ++v)
#pragma unroll
          for (int e = 0; e < E; ++e)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
              for (int cc = 0; cc < NC; ++cc)
                acc[mt][cc] = M::mma(av[mt][v][e], xv[v * E + e][cc], acc[mt][cc]);
      }
    }
  }

  // fixed-order reduction of the 4 waves: ((w0 + w1) + w2) + w3
#pragma unroll
  for (int s = 1; s < 4; ++s) {
    __syncthreads();
    if (wave == s) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) red[mt * NC + cc][lane] = acc[mt][cc];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) acc[mt][cc] += red[mt * NC + cc][lane];
    }
  }
  if (wave != 0) return;
#pragma unroll
  for (int sr = 0; sr < NSRC; ++sr) {
    T* pout = P + ((int64_t)sr * S + by) * m * L;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row0 + mt * 16 + M::row(lane, r);
        if (row < m) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) pout[row * L + nt * 16 + i] = acc[mt][sr * NT + nt][r];
        }
      }
  }
}

// ------------------------------------------------------------------------------------------
// A @ X with X staged through LDS (kind 5). A block of WAVES waves walks ONE K range; wave w
// owns rows row0 + 16*MT*w .. +16*MT, so there is no cross-wave reduction. Each K chunk of X
// (CK rows x 16NT columns per source, 8 KiB at l = 32 with two sources) is loaded from L2 once
// per block, one 16-B vector per thread, and kept in LDS in its natural [k][column] order with
// a padded row of LP = L + 4 (f64) / L + 2 (f32) elements: the MFMA B-operand reads (lane
// (i, q) <- X[q*EL + e][16nt + i], ds_read_b64 / _b32) and the staging stores (ds_write_b128,
// or 2 x _b64 when the f32 row is not 16-B aligned) are then free of bank conflicts under the
// CDNA4 LDS lane-group model (MI355X_MICROARCH.md §LDS; checked with a small simulator).
// Compared with kind 1/2 (every wave gathers its own X chunk into registers) this cuts the
// L2->CU traffic of X by WAVES and frees the X register ring: the f64 2-RHS tile fits 2 waves
// per SIMD. Pipeline per chunk c: write X(c+1) (loaded PF-1 chunks ago) to the other LDS slot,
// issue X(c+PF), read X(c) from this slot, then per row tile its MFMAs followed by the refill
// of that tile's A registers with chunk c+PF; one barrier. A is read exactly once.
// ------------------------------------------------------------------------------------------
// one 16-B X vector into LDS: a b128 store, or two 8-B stores when the row is only 8-B aligned
template <typename T, bool W16>
__device__ inline void lds_put(T* dst, typename MF<T>::vec_t v) {
  typedef typename MF<T>::vec_t V;
  if constexpr (W16) {
    *reinterpret_cast<V*>(dst) = v;
  } else {
    typedef T h2 __attribute__((ext_vector_type(2)));
    constexpr int E = MF<T>::E;
#pragma unroll
    for (int h = 0; h < E / 2; ++h) *reinterpret_cast<h2*>(dst + 2 * h) = h2{v[2 * h], v[2 * h + 1]};
  }
}

// p_thr = p with |p| < thres zeroed over the n l elements (k_trial_split's comparison), 16-B
// vectors strided over the AxDerive::nd workgroups of the fused dense pass
template <typename T, int NTHR>
__device__ inline void drv_thr_item(const T* __restrict__ p, const AxDerive& d, int64_t nl, int item) {
  typedef typename MF<T>::vec_t V;
  constexpr int E = MF<T>::E;
  const T thres = (T)d.thres;
  const V* src = reinterpret_cast<const V*>(p);
  V* dst = reinterpret_cast<V*>(static_cast<T*>(d.pthr));
  const int64_t nv = nl / E;
  for (int64_t i = (int64_t)item * NTHR + threadIdx.x; i < nv; i += (int64_t)d.nd * NTHR) {
    V v = src[i];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = tabs(v[e]) < thres ? T(0) : v[e];
    dst[i] = v;
  }
}

// One (row block, column) item of the split-candidate A e inside the fused dense pass (AxDerive
// with ggx > 0): k_at_gather_bm's work (kernels_gather.hip) by a 512-thread workgroup, one output
// row per thread — column c's ascending list of flagged rows built in LDS from its bitmap words,
// then At's rows walked in that order with the same arithmetic, so A e has the same bits — with the
// words read from the all-gathered sums chunks (d.blk) instead of zf.
template <typename T, int L, int NTHR>
__device__ inline void drv_gather_item(const AxDerive& d, int64_t m, int64_t n, int item) {
  constexpr int SEGW = 256, NW = NTHR / 64, U = 8;
  static_assert(NTHR >= SEGW, "one bitmap word per thread and segment");
  __shared__ unsigned short lst[64 * SEGW];
  __shared__ unsigned wsum[NW];
  const T* At = static_cast<const T*>(d.At);
  const T* E = static_cast<const T*>(d.E);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rb = item % d.ggx, c = item / d.ggx;
  const int64_t nw = n / 64;             // n % 64 == 0 and srows % 64 == 0 (solver.cpp sderive_)
  const int64_t wpr = d.srows / 64;      // bitmap words per rank
  const int64_t r = (int64_t)rb * NTHR + tid;
  const int64_t rr = r < m ? r : m - 1;
  T acc = T(0);
  for (int64_t w0 = 0; w0 < nw; w0 += SEGW) {
    const int64_t w = w0 + tid;
    uint64_t bits = 0;
    if (tid < SEGW && w < nw) {
      const int64_t rk = w / wpr, lw = w - rk * wpr;
      const unsigned* zr = reinterpret_cast<const unsigned*>(d.blk + rk * d.bstride + d.moff);
      const unsigned short* bm = reinterpret_cast<const unsigned short*>(zr + d.srows) + (int64_t)c * (d.srows / 16);
      bits = reinterpret_cast<const uint64_t*>(bm)[lw];
    }
    const unsigned cnt = (unsigned)__builtin_popcountll(bits);
    unsigned inc = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned v = __shfl_up(inc, off);
      if (lane >= off) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    unsigned pos = inc - cnt, total = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      if (q < wave) pos += wsum[q];
      total += wsum[q];
    }
    while (bits != 0) {
      const int j = __builtin_ctzll(bits);
      bits &= bits - 1;
      lst[pos++] = (unsigned short)((w - w0) * 64 + j);   // row - 64 w0
    }
    __syncthreads();
    const int tot = (int)total;
    const int64_t kb = w0 * 64;
    int idx = 0;
    for (; idx + U <= tot; idx += U) {
      T a[U], ev[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k = kb + lst[idx + u];
        a[u] = __builtin_nontemporal_load(At + k * m + rr);
        ev[u] = E[k * L + c];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc = acc + a[u] * ev[u];
    }
    for (; idx < tot; ++idx) {
      const int64_t k = kb + lst[idx];
      acc = acc + __builtin_nontemporal_load(At + k * m + rr) * E[k * L + c];
    }
    __syncthreads();   // lst and wsum are rewritten by the next segment
  }
  if (r < m) static_cast<T*>(d.Pe)[r * L + c] = acc;
}

//
// DRV (round 6, the row-sharded ProxGD trial; solver.cpp iter_proxgd_shard): X0 is the all-gathered
// p and the launch does the trial's replicated half itself. The dense workgroups threshold the
// MFMA operands as they leave LDS (|p| < thres -> 0, k_trial_split's comparison; stores and
// branches in the ring loop made the compiler drain vmcnt at its join points: +15 us per pass,
// and thresholding the staged vectors before their LDS store shortened the X prefetch: +6 us),
// so the MFMAs read p_thr; behind them AxDerive::nd workgroups write
// p_thr (drv_thr_item) and ggx * l workgroups compute A e (drv_gather_item) beside the MFMA work;
// the publisher workgroup combines the all-gathered sums (shard_combine_block) and publishes the
// packet with them. Replaces k_trial_split and the k_at_gather_bm launch between the all-gather
// and this pass.
template <typename T, int MT, int NT, int NSRC, int PF, int VPL, int WAVES, int DRV>
__device__ __forceinline__ void ax_lds_body(const T* __restrict__ A,
                                                      const T* __restrict__ X0,
                                                      const T* __restrict__ X1,
                                                      const T* __restrict__ X2,
                                                      T* __restrict__ P, int64_t m, int64_t n,
                                                      int64_t chunks, int S, int gx, int xmap,
                                                      const int* __restrict__ gate, int epoch,
                                                      Pub pub, AxDerive drv) {
  typedef MF<T> M;
  typedef typename M::vec_t V;
  typedef typename M::acc_t C;
  constexpr int E = M::E;
  constexpr int EL = VPL * E;             // k per lane per chunk
  constexpr int CK = 4 * EL;              // k per chunk
  constexpr int L = 16 * NT;              // == l
  constexpr int NC = NT * NSRC;
  constexpr int LP = L + (sizeof(T) == 8 ? 4 : 2);   // padded LDS row (see header)
  constexpr bool W16 = (LP * sizeof(T)) % 16 == 0;    // rows 16-B aligned: one b128 store
  constexpr int XCH = NSRC * CK * LP;     // elements of one staged chunk
  constexpr int NTHR = 64 * WAVES;
  constexpr int XV = NSRC * CK * L / E;   // 16-B vectors of X per chunk
  constexpr int XPT = (XV + NTHR - 1) / NTHR;
  constexpr bool XFULL = (XV % NTHR) == 0; // every thread moves XPT vectors: no predicate
  constexpr int VPR = L / E;              // vectors per X row
  static_assert(PF >= 2, "X(c+1) must sit in another ring slot than X(c + PF)");
  static_assert(!DRV || NSRC == 1, "the derive: one source");
  __shared__ __attribute__((aligned(16))) T xs[2][XCH];
  // pub.host: workgroup 0 hands the scalar packet to the host (no reduction to join here) while
  // the others run; with a short kernel in front (the N > 1 trial) a packet carried by THAT
  // kernel held up this launch by ~4 us (profiles/r1_tuning/small_kernels/ax_publisher.log)
  if (pub.host != nullptr && blockIdx.x == 0) {
    if constexpr (DRV) {
      shard_combine_block(drv.sp);   // drv.sp.pub == pub
    } else if (threadIdx.x == 0) {
      publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq, pub.s2, pub.off2, pub.n2,
                     pub.s3, pub.off3, pub.n3);
    }
    return;
  }
  if constexpr (DRV) {
    if ((int)blockIdx.x >= drv.gat0) {   // the A e workgroups (block-uniform)
      drv_gather_item<T, L, 64 * WAVES>(drv, m, n, (int)blockIdx.x - drv.gat0);
      return;
    }
    if ((int)blockIdx.x >= drv.thr0) {   // the p_thr workgroups
      drv_thr_item<T, 64 * WAVES>(X0, drv, n * L, (int)blockIdx.x - drv.thr0);
      return;
    }
  }
  if (!gate_live(gate, epoch)) return;
  int bx, by;
  if (!ax_block(xmap, gx, S, bx, by, pub.host != nullptr ? 1 : 0)) return;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t row0 = (int64_t)bx * (16 * MT * WAVES) + (int64_t)wave * (16 * MT);
  const int64_t cb = chunks * by / S, ce = chunks * (by + 1) / S;
  const int64_t nch = ce - cb;
  if (nch <= 0) return;   // block-uniform
  const int64_t rot = ax_rot(xmap, bx, gx, nch);
  // chunk `off` of the walk (clamped past the end: a re-read of the last one, see below) is
  // chunk (off + rot) mod nch of the block's K range
  auto kch = [&](int64_t off) -> int64_t {
    off = (off < nch ? off : nch - 1) + rot;
    return off >= nch ? off - nch : off;
  };

  const T* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int64_t r = row0 + mt * 16 + i;
    r = r < m ? r : m - 1;
    ap[mt] = A + r * n + cb * CK + (int64_t)q * EL;
  }
  // X staging: thread t moves vectors t, t + NTHR, ... of the chunk (src, k, column vector)
  const T* xg[XPT];
  int xo[XPT];
  bool xon[XPT];
#pragma unroll
  for (int j = 0; j < XPT; ++j) {
    const int v = threadIdx.x + NTHR * j;
    xon[j] = XFULL || v < XV;
    const int vv = xon[j] ? v : 0;
    const int src = vv / (CK * VPR), rem = vv % (CK * VPR);
    const int k = rem / VPR, c = (rem % VPR) * E;
    const T* xb = src == 0 ? X0 : (src == 1 ? X1 : X2);
    xg[j] = xb + (cb * CK + k) * L + c;
    xo[j] = src * CK * LP + k * LP + c;
  }

  C acc[MT][NC];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[mt][c] = C{};

  // Ring loads at a clamped chunk offset: past the end they re-read the last chunk (unused),
  // so the main loop has no load predicates. A predicate at a loop join point makes the
  // compiler drain vmcnt to 0 there, which empties the prefetch ring every chunk.
  V a[PF][MT][VPL];
  V xr[PF][XPT];
  auto load_x = [&](V (&dst)[XPT], int64_t off) {
    off = kch(off);
#pragma unroll
    for (int j = 0; j < XPT; ++j)
      if (XFULL || xon[j]) dst[j] = *reinterpret_cast<const V*>(xg[j] + off * CK * L);
  };
  auto load_a = [&](V (&dst)[MT][VPL], int64_t off) {
    off = kch(off);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int v = 0; v < VPL; ++v)
        dst[mt][v] = load_vec<T, false>(ap[mt] + off * CK + v * E);
  };
  auto put_x = [&](int slot, V (&src)[XPT]) {
#pragma unroll
    for (int j = 0; j < XPT; ++j)
      if (XFULL || xon[j]) lds_put<T, W16>(&xs[slot][xo[j]], src[j]);
  };
  // X(c) from LDS slot into registers
  auto read_x = [&](int slot, T (&xv)[NC][EL]) {
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
      const int src = cc / NT, nt = cc % NT;
      const T* xp = &xs[slot][src * CK * LP + q * EL * LP + nt * 16 + i];
#pragma unroll
      for (int e = 0; e < EL; ++e) xv[cc][e] = xp[e * LP];
      if constexpr (DRV == 1) {   // p -> p_thr as the operands leave LDS (see the header)
        const T thres = (T)drv.thres;
#pragma unroll
        for (int e = 0; e < EL; ++e) xv[cc][e] = tabs(xv[cc][e]) < thres ? T(0) : xv[cc][e];
      }
    }
  };
  // MFMAs of row tile mt for one chunk, column tiles [C0, C1)
  auto mma_cols = [&](int mt, const V (&av)[VPL], const T (&xv)[NC][EL], int c0, int c1) {
#pragma unroll
    for (int v = 0; v < VPL; ++v)
#pragma unroll
      for (int e = 0; e < E; ++e)
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
          if (cc >= c0 && cc < c1) acc[mt][cc] = M::mma(av[v][e], xv[cc][v * E + e], acc[mt][cc]);
  };
  auto mma_tile = [&](int mt, const V (&av)[VPL], const T (&xv)[NC][EL]) {
    mma_cols(mt, av, xv, 0, NC);
  };

#pragma unroll
  for (int p = 0; p < PF; ++p) {   // X first, then A, in every ring step (see header)
    load_x(xr[p], p);
    load_a(a[p], p);
  }
  put_x(0, xr[0]);                 // chunk 0 -> slot 0
  __syncthreads();

  // Main loop: PF chunks per trip, no predicates. Registers are consumed in place: a tile's
  // A fragments feed its MFMAs and are then refilled with chunk c + PF in the same registers
  // (copying them out first would force the refill loads to complete at the loop's back edge).
  int64_t c0 = 0;
  for (; c0 + PF <= nch; c0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int64_t c = c0 + p;
      const int slot = (int)(c & 1);
      put_x(slot ^ 1, xr[(p + 1) % PF]);   // X(c+1), loaded PF-1 chunks ago
      load_x(xr[p], c + PF);       // xr[p] (X(c)) has been in LDS since chunk c-1
      T xv[NC][EL];
      read_x(slot, xv);
      const int64_t off = kch(c + PF);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        mma_tile(mt, a[p][mt], xv);
#pragma unroll
        for (int v = 0; v < VPL; ++v) a[p][mt][v] = load_vec<T, false>(ap[mt] + off * CK + v * E);
      }
      __syncthreads();
    }
  }
  // tail: fewer than PF chunks left (their data is already in the ring)
#pragma unroll
  for (int p = 0; p < PF - 1; ++p) {
    const int64_t c = c0 + p;
    if (c < nch) {
      const int slot = (int)(c & 1);
      if (c + 1 < nch) put_x(slot ^ 1, xr[(p + 1) % PF]);
      T xv[NC][EL];
      read_x(slot, xv);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) mma_tile(mt, a[p][mt], xv);
      __syncthreads();
    }
  }

#pragma unroll
  for (int sr = 0; sr < NSRC; ++sr) {
    T* pout = P + ((int64_t)sr * S + by) * m * L;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row0 + mt * 16 + M::row(lane, r);
        if (row < m) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) pout[row * L + nt * 16 + i] = acc[mt][sr * NT + nt][r];
        }
      }
  }
}

#define GLX_AX_LDS_ARGS                                                                          \
  const T* __restrict__ A, const T* __restrict__ X0, const T* __restrict__ X1,                 \
      const T* __restrict__ X2, T* __restrict__ P, int64_t m, int64_t n, int64_t chunks, int S, \
      int gx, int xmap, const int* __restrict__ gate, int epoch, Pub pub, AxDerive drv
template <typename T, int MT, int NT, int NSRC, int PF, int VPL, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_ax_lds(GLX_AX_LDS_ARGS) {
  ax_lds_body<T, MT, NT, NSRC, PF, VPL, WAVES, 0>(A, X0, X1, X2, P, m, n, chunks, S, gx, xmap, gate,
                                                     epoch, pub, drv);
}
// the derive form (its own kernel: the extra workgroups' code and LDS stay out of k_ax_lds)
template <typename T, int MT, int NT, int NSRC, int PF, int VPL, int WAVES, int DRV>
__global__ __launch_bounds__(64 * WAVES) void k_ax_lds_drv(
    GLX_AX_LDS_ARGS) {
  ax_lds_body<T, MT, NT, NSRC, PF, VPL, WAVES, DRV>(A, X0, X1, X2, P, m, n, chunks, S, gx, xmap, gate,
                                                    epoch, pub, drv);
}
#undef GLX_AX_LDS_ARGS

template <typename T, int LB, int RW, bool VEC, int NSRC>
__global__ __launch_bounds__(256) void k_ax_valu(const T* __restrict__ A, const T* __restrict__ X0,
                                                 const T* __restrict__ X1, const T* __restrict__ X2,
                                                 T* __restrict__ P, int64_t m, int64_t n,
                                                 int64_t l, int c0, int S,
                                                 const int* __restrict__ gate, int epoch) {
  constexpr int E = VEC ? (16 / (int)sizeof(T)) : 1;
  if (!gate_live(gate, epoch)) return;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * RW;
  if (row0 >= m) return;  // wave-uniform; no barriers below
  const int s = blockIdx.y;
  const int64_t nv = n / E;
  const int64_t kb = E * (nv * s / S);
  const int64_t ke = (s == S - 1) ? n : E * (nv * (s + 1) / S);
  const int nc = (int)((l - c0) < LB ? (l - c0) : LB);
  const T* xs[3] = {X0, X1, X2};

  const T* arow[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    int64_t rr = row0 + r;
    rr = rr < m ? rr : m - 1;
    arow[r] = A + rr * n;
  }
  T acc[NSRC][RW][LB];
#pragma unroll
  for (int sr = 0; sr < NSRC; ++sr)
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int c = 0; c < LB; ++c) acc[sr][r][c] = T(0);

  for (int64_t k = kb + (int64_t)lane * E; k < ke; k += 64 * E) {
    T a[RW][E];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      if constexpr (VEC) {
        typedef typename MF<T>::vec_t V;
        const V v = *reinterpret_cast<const V*>(arow[r] + k);
#pragma unroll
        for (int e = 0; e < E; ++e) a[r][e] = v[e];
      } else {
        a[r][0] = arow[r][k];
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int sr = 0; sr < NSRC; ++sr) {
        T xv[LB];
#pragma unroll
        for (int c = 0; c < LB; ++c) xv[c] = (c < nc) ? xs[sr][(k + e) * l + c0 + c] : T(0);
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int c = 0; c < LB; ++c) acc[sr][r][c] = __builtin_fma(a[r][e], xv[c], acc[sr][r][c]);
      }
    }
  }
#pragma unroll
  for (int sr = 0; sr < NSRC; ++sr)
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int c = 0; c < LB; ++c) acc[sr][r][c] = wave_sum(acc[sr][r][c]);
  if (lane == 0) {
#pragma unroll
    for (int sr = 0; sr < NSRC; ++sr) {
      T* pout = P + ((int64_t)sr * S + s) * m * l;
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int64_t row = row0 + r;
        if (row < m) {
#pragma unroll
          for (int c = 0; c < LB; ++c)
            if (c < nc) pout[row * l + c0 + c] = acc[sr][r][c];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// planning + launch
// ------------------------------------------------------------------------------------------
// tiles below when the shape does not fit them (l not 16/32, n not a multiple of 4*E*VPL).
static constexpr int kAxDefault = 52228;       // f64 single RHS: LDS, MT 2, PF 2, VPL 2, 8 waves
static constexpr int kAxFallback = 21820;      // f64: VPL 2, direct loads, MT 8, PF 2
static constexpr int kAxDefault32 = 21410;     // f32: VPL 2, direct loads, MT 4, PF 1
static constexpr int kAxDma32 = 92478;         // f32 one RHS, A beyond the Infinity Cache (LDS-DMA)
// A^T R code: NTL*1000 + WL*10 + PF (WL 1 = four panels of a block share rows, PF = ring depth)
static constexpr int kAtrDefault = 108;        // f64: WL 0, PF 8 (A that stays in the MALL)
static constexpr int kAtrDefaultBig = 1008;    // f64: non-temporal A, WL 0, PF 8
// Non-temporal A loads pay only when A cannot stay in the 256 MiB Infinity Cache between the
// passes: NS (1 GiB) 2278 -> 2326 it/s, FProxGD 2397 -> 2451, but C2 (256 MiB) 7477 -> 6250 and
// the 1024-row shard (128 MiB) 9477 -> 8323 (profiles/r2_axat/)
static constexpr double kAtrNtBytes = 384.0 * 1024 * 1024;
static constexpr int kAtrDefault32 = 1114;     // f32: non-temporal A, WL 1, PF 4
// batched right-hand sides (MFMA-bound at l = 32, both dtypes): the LDS tile, 2 waves per SIMD
// (end-to-end sweep, profiles/r1_tuning: f64 8-wave blocks, f32 4-wave blocks with PF 3)
static int axb_default(int nsrc, int esize) {
  (void)nsrc;
  return esize == 8 ? 52228 : 52324;
}

// the tiles the planner picks (lds_plan); the LDS-DMA sweep's other codes are in DESIGN.md
static constexpr int kLdsCodes[] = {52224, 52324, 52228, 51328,
                                     // kind 9 (LDS-DMA, two row tiles per wave): 9 NS KC/16 flags WAVES;
                                     // 92278 / 92268 f64, 92478 f32 (one source)
                                     92278, 92268, 92478};
static inline bool dma_kind(int c) { return c / 10000 == 8 || c / 10000 == 9; }
static inline bool lds_kind(int c) { return c / 10000 == 5 || dma_kind(c); }
static bool lds_code_ok(int c, int64_t n, int64_t l, int esize, int nsrc = 1) {
  bool known = false;
  for (int k : kLdsCodes) known |= (k == c);
  if (!known) return false;
  if (dma_kind(c))
    return (c == kAxDma32 ? (esize == 4 && nsrc == 1) : esize == 8) && (l == 16 || l == 32) &&
           n % (16 * ((c / 100) % 10)) == 0 && dma_lds_need(c, l, nsrc, esize) <= 160 * 1024;
  const int E = 16 / esize, vpl = (c / 10) % 10;
  return (l == 16 || l == 32) && n % (4 * E * vpl) == 0;
}
// K split of a kind-5/8 launch: enough blocks for 2 (4-wave) blocks per CU
static int lds_split(int esize, int64_t m, int64_t n, int code, int64_t target = 0) {
  const int E = 16 / esize, waves = code % 10;
  int64_t rb, chunks;
  if (dma_kind(code)) {   // MT 16-row tiles per wave, KC = 16 * digit-3 columns per chunk
    rb = cdiv(m, 16 * dma_mt(code) * dma_waves(code));
    chunks = n / (16 * ((code / 100) % 10));
  } else {
    const int mt = (code / 1000) % 10, vpl = (code / 10) % 10;
    rb = cdiv(m, 16 * mt * waves);
    chunks = n / (4 * E * vpl);
  }
  if (target <= 0) target = env_int("GLX_AXL_BLOCKS", (waves == 8 || waves == 1) ? 256 : 512);
  return (int)clampi(cdiv(target, rb), 1, std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, chunks / 8)));
}
// A K-split launch writes S partial slabs of m x (nsrc*l) that the finalize kernel reads back.
// With few rows (the per-rank shards of a multi-GPU run) a 256-block target lets S reach 64 and
// the slabs rival A itself. When they exceed 1/6 of A, use the 4-wave tile at 256 blocks, which
// halves them. Shard-shape sweep (profiles/r1_tuning/shard_shapes.txt): at m = 1024 this is
// +10 % end to end despite a slower A@X; at m >= 2048 the default tile stays ahead.
//
// Per-rank shards at l = 32 (m <= 2048: the 4- and 8-GPU runs of the north-star size) take the
// 8-wave tile with ONE 16-row tile per wave and a 3-deep ring (51328): at these row counts the
// K splits are short, and two waves per SIMD with half the rows per block keep the slab volume
// of the 4-wave tile. Measured end to end with the communicator path
// (profiles/r1_tuning/small_kernels/ax_shard_tile.log): +4.7 % at m = 1024, +3 % at 2048,
// neutral at 4096; at m = 8192 the default tile stays ahead (A@X 290 vs 306 us).
//
// One right-hand side at l = 32, f64 (round 2: the split-candidate trial's dense pass A p_thr is
// HBM-bound): 51328 with its 4 K splits, A@X 246-250 vs 252-254 us incl. the A e gather, NS
// ProxGD 2266-2269 vs 2231-2232 it/s on one box (profiles/r2_axtile/).
//
// Round 3, the LDS-DMA tile (kernels_axdma.hip): one right-hand side in fp64 with A beyond the
// Infinity Cache (the split-candidate dense pass A p_thr at NS, FProxGD's A xc, C5's shard) takes
// 92278 (two 16-row tiles per wave, 256-B row pieces, 2-slot ring, non-temporal A, DMA issues and
// operand reads interleaved into the MFMA stream): NS 164 vs 193-196 us (6.57 TB/s), the 16384-row
// shard 334 vs 399 us. fp64 C2 (two right-hand sides, l = 16, A in the Infinity Cache) takes
// 92268 (default policy): 46.2 vs 49.3 us. Interleaved kernel-trace A/B, profiles/r3_axdma/.
static void lds_plan(int esize, int64_t m, int64_t n, int64_t l, int nsrc, int& code, int& S) {
  S = lds_split(esize, m, n, code);
  if (std::getenv("GLX_AXL_BLOCKS") || std::getenv("GLX_AXB_VARIANT")) return;
  const bool big = (double)m * (double)n * esize > kAtrNtBytes;
  if (esize == 8 && nsrc == 1 && big && code == 52228 && lds_code_ok(92278, n, l, esize, 1) &&
      env_int("GLX_AX_DMA", 1) != 0 && !std::getenv("GLX_AX_VARIANT")) {
    code = 92278;
    S = lds_split(esize, m, n, code);
    return;
  }
  if (esize == 8 && nsrc == 2 && l == 16 && !big && code == 52228 &&
      lds_code_ok(92268, n, l, esize, 2) && env_int("GLX_AX_DMA", 1) != 0) {
    code = 92268;
    S = lds_split(esize, m, n, code);
    return;
  }
  if (esize == 8 && nsrc == 1 && l == 32 && code == 52228 && lds_code_ok(51328, n, l, esize) &&
      !std::getenv("GLX_AX_VARIANT")) {
    code = 51328;
    S = lds_split(esize, m, n, code);
    return;
  }
  if (esize == 8 && nsrc == 2 && l == 32 && m <= 2048 && code == 52228 &&
      lds_code_ok(51328, n, l, esize) && env_int("GLX_SHARD_TILE", 1) != 0) {
    code = 51328;
    S = lds_split(esize, m, n, code);
    return;
  }
  if ((double)S * (double)m * nsrc * l * 6.0 <= (double)m * n) return;
  const int c4 = esize == 8 ? 52224 : 52324;
  if (!lds_code_ok(c4, n, l, esize)) return;
  const int S4 = lds_split(esize, m, n, c4, 256);
  if (S4 < S) { code = c4; S = S4; }
}

static bool valid_ax_code(int c) { return c == 21820 || c == 21410 || c == 1820; }

GemmPlan make_plan(int esize, int64_t m, int64_t n, int64_t l, int ax_variant) {
  GemmPlan p{};
  p.esize = esize;
  p.m = m; p.n = n; p.l = l;
  const int E = 16 / esize;
  const bool mfma_l = (l == 16 || l == 32);
  // ---- A @ X ----
  if (ax_variant == 0) ax_variant = env_int("GLX_AX_VARIANT", 0);
  if (ax_variant == 1 || ax_variant == 2) ax_variant = esize == 8 ? kAxFallback : kAxDefault32;
  const bool ax_mfma_ok = mfma_l && (n % (4 * E) == 0);
  if (ax_variant == 3 || !ax_mfma_ok) {
    p.ax_kind = 3;
    p.ax_lb = l >= 8 ? 8 : (l >= 4 ? 4 : (l >= 2 ? 2 : 1));
    if (l == 3) p.ax_lb = 4;
    if (l > 4 && l < 8) p.ax_lb = 8;
    p.ax_vec = (n % E == 0) ? 1 : 0;
    const int64_t waves = cdiv(m, 4);                    // RW = 4 rows per wave
    const int64_t kunits = n / (64 * (p.ax_vec ? E : 1)); // 64-lane strides per row
    p.ax_S = (int)clampi(cdiv(kTargetWaves, waves), 1, std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, kunits / 4)));
  } else if (esize == 4 && ax_variant == 0 && (double)m * (double)n * esize > kAtrNtBytes &&
             lds_code_ok(kAxDma32, n, l, esize, 1) && env_int("GLX_AX_DMA", 1) != 0 &&
             env_int("GLX_AX_DMA32", 1) != 0) {
    // Round 4: f32 with one right-hand side and A beyond the Infinity Cache (C3's split-candidate
    // dense pass A xc) on the LDS-DMA tile, as 92278 does for f64: 85-88 us = 6.1-6.3 TB/s
    // against 115 us for the direct-load tile 21410 (profiles/r4_exp3/). GLX_AX_DMA32=0: off.
    p.ax_code = kAxDma32;
    p.ax_kind = 5;
    p.ax_S = lds_split(esize, m, n, kAxDma32);
    p.ax_mt = 2;
    p.ax_pf = 0;
  } else if (lds_code_ok(ax_variant ? ax_variant : (esize == 8 ? kAxDefault : kAxDefault32), n, l, esize)) {
    int code = ax_variant ? ax_variant : (esize == 8 ? kAxDefault : kAxDefault32);
    if (ax_variant) p.ax_S = lds_split(esize, m, n, code);
    else lds_plan(esize, m, n, l, 1, code, p.ax_S);
    p.ax_code = code;
    p.ax_kind = 5;
    p.ax_mt = (code / 1000) % 10;
    p.ax_pf = (code / 100) % 10;
  } else {
    int code = valid_ax_code(ax_variant) ? ax_variant : (esize == 8 ? kAxFallback : kAxDefault32);
    int vpl = code / 10000 ? code / 10000 : 1;
    if (n % (4 * E * vpl) != 0) { code = 1820; vpl = 1; }   // wider chunks need n % 4*E*VPL
    p.ax_code = code;
    p.ax_kind = (code / 1000) % 10;
    p.ax_mt = (code / 100) % 10;
    p.ax_pf = (code / 10) % 10;
    const int64_t blocks = cdiv(m, 16 * p.ax_mt);
    const int64_t chunks = n / (4 * E * vpl);
    // sweep (scripts/kbench.py): f64 at MT 8 wants 1024 waves, f32 4096
    const int64_t target = esize == 8 ? (p.ax_mt == 8 ? kTargetWaves / 2 : kTargetWaves) : 2 * kTargetWaves;
    p.ax_S = (int)clampi(cdiv(target, blocks * 4), 1,
                         std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, chunks / 16)));
  }
  const int s_ax = env_int("GLX_AX_S", 0);
  if (s_ax > 0) p.ax_S = (int)std::min<int64_t>(s_ax, kMaxSplit);
  p.ax_xmap = (env_int("GLX_AX_XCD", 1) ? 1 : 0) | (env_int("GLX_AX_ROT", 1) ? 2 : 0);
  // batched right-hand sides
  p.axb_code[0] = p.axb_code[1] = p.ax_code;
  p.axb_S[0] = p.axb_S[1] = p.ax_S;
  for (int ns = 2; ns <= 3; ++ns) {
    int code = env_int("GLX_AXB_VARIANT", axb_default(ns, esize));
    int S = p.ax_S;
    if (p.ax_kind == 3) {
      code = 0;
    } else if (lds_kind(code)) {
      if (lds_code_ok(code, n, l, esize, ns)) lds_plan(esize, m, n, l, ns, code, S);
      else code = ns == 2 ? 1420 : 1220;
    } else if (code >= 10000 && n % (4 * E * (code / 10000)) != 0) {
      code = ns == 2 ? 1420 : 1220;
    }
    const int s_axb = env_int("GLX_AXB_S", 0);
    if (s_axb > 0 && lds_kind(code)) S = (int)std::min<int64_t>(s_axb, kMaxSplit);
    p.axb_code[ns] = code;
    p.axb_S[ns] = S;
  }
  // ---- A^T R ----
  int atr_code = env_int("GLX_ATR_VARIANT", 0);
  if (atr_code == 0)
    atr_code = esize == 8 ? ((double)m * n * esize > kAtrNtBytes ? kAtrDefaultBig : kAtrDefault)
                          : kAtrDefault32;
  int ntl = atr_code >= 1000 ? 1 : 0;
  int wl = (atr_code / 10) % 10;
  int pf = atr_code % 10;
  if (wl == 1 && n % 256 != 0) wl = 0;   // four shared-row panels need n % 256: one panel per block
  if (wl > 3 || (wl == 3 && (esize != 8 || n % 32 != 0))) wl = 0;   // 3: the 32-column f64 panel (4 waves)
  // Round 6: only the planner's tiles are built (kernels_atr.hip atr_mfma_nt): WL 0 / 3 with the
  // PF 8 ring, WL 2 with PF 8 and non-temporal A, WL 1 with PF 4 and non-temporal A
  if (wl == 1) { pf = 4; ntl = 1; }
  else { pf = 8; if (wl == 2) ntl = 1; }
  const bool atr_mfma_ok = mfma_l && (n % 64 == 0) && (m % 4 == 0);
  if (ax_variant == 3 || atr_code == 3 || !atr_mfma_ok) {
    p.atr_kind = 3;
    p.atr_lb = l >= 8 ? 8 : (l >= 4 ? 4 : (l >= 2 ? 2 : 1));
    if (l == 3) p.atr_lb = 4;
    if (l > 4 && l < 8) p.atr_lb = 8;
    p.atr_vec = (n % E == 0) ? 1 : 0;
    const int64_t cols_per_block = 256 * (p.atr_vec ? E : 1);
    const int64_t blocks = cdiv(n, cols_per_block);
    p.atr_S = (int)clampi(cdiv(kTargetWaves / 4, blocks), 1, std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, m / 16)));
  } else {
    p.atr_kind = 1;
    p.atr_wl = wl;   // 0: 4 waves split a panel's rows, 1: 4 panels per block, 2: 8 waves
    p.atr_pf = (pf >= 2 && pf <= 8) ? pf : 2;   // in-place ring: lookahead PF - 1 steps
    p.atr_ntl = ntl;
    const int64_t steps = m / 4;
    if (p.atr_wl != 1) {
      const int64_t blocks = n / (p.atr_wl == 3 ? 32 : 64);
      // f64: one wave per SIMD is enough with the PF-8 ring (and S = 1 at n = 16384 lets the
      // ProxGD trial fuse into the kernel); f32 wants 4 per SIMD
      const int64_t target = esize == 8 ? kTargetWaves / 2 : 2 * kTargetWaves;
      p.atr_S = (int)clampi(cdiv(target, blocks * 4), 1,
                            std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, steps / 16)));
    } else {
      const int64_t blocks = n / 256;
      p.atr_S = (int)clampi(cdiv(kTargetWaves / 4, blocks), 1,
                            std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, steps / 16)));
    }
  }
  const int s_atr = env_int("GLX_ATR_S", 0);
  if (s_atr > 0) p.atr_S = (int)std::min<int64_t>(s_atr, kMaxSplit);
  return p;
}

static std::string ax_name(const GemmPlan& p, int nsrc) {
  const int code = p.axb_code[nsrc];
  char buf[128];
  if (p.ax_kind == 3 || code == 0) {
    std::snprintf(buf, sizeof buf, "k_ax_valu<LB%d,VEC%d> S=%d", p.ax_lb, p.ax_vec, ax_split(p, nsrc));
  } else if (dma_kind(code)) {
    std::snprintf(buf, sizeof buf, "k_ax_dma<MT%d,NS%d,KC%d,NTL%d,HOIST%d(2:PIPE),W%d> S=%d", dma_mt(code), (code / 1000) % 10,
                  16 * ((code / 100) % 10), (code / 10) % 2, (code / 20) % 2 + 2 * ((code / 40) % 2),
                  dma_waves(code),
                  ax_split(p, nsrc));
  } else if (code / 10000 == 5) {
    std::snprintf(buf, sizeof buf, "k_ax_lds<MT%d,PF%d,VPL%d,W%d> S=%d", (code / 1000) % 10,
                  (code / 100) % 10, (code / 10) % 10, code % 10, ax_split(p, nsrc));
  } else {
    const int vpl = code / 10000 ? code / 10000 : 1;
    std::snprintf(buf, sizeof buf, "k_ax_mfma<kind%d,MT%d,PF%d,NTL%d,VPL%d> S=%d", (code / 1000) % 10,
                  (code / 100) % 10, (code / 10) % 10, code % 10, vpl, ax_split(p, nsrc));
  }
  return buf;
}

std::string describe_plan(const GemmPlan& p) {
  std::string s;
  for (int ns = 1; ns <= 3; ++ns) s += "ax" + std::to_string(ns) + "=" + ax_name(p, ns) + "; ";
  char buf[128];
  if (p.atr_kind == 3)
    std::snprintf(buf, sizeof buf, "atr=k_atr_valu<LB%d,VEC%d> S=%d", p.atr_lb, p.atr_vec, p.atr_S);
  else
    std::snprintf(buf, sizeof buf, "atr=k_atr_mfma<WL%d,PF%d,NTL%d> S=%d%s", p.atr_wl, p.atr_pf, p.atr_ntl, p.atr_S,
                  p.atr_wl == 3 ? " (32-column panels)" : "");
  return s + buf;
}

int max_ax_split(int esize, int64_t m, int64_t n, int64_t l) {
  int s = 1;
  for (int v : {0, 3, 1820, 21820, 21410}) s = std::max(s, ax_split_max(make_plan(esize, m, n, l, v)));
  for (int v : kLdsCodes) s = std::max(s, ax_split_max(make_plan(esize, m, n, l, v)));
  return s;
}

template <typename T, int LB, int NSRC>
static void ax_valu_lb(const GemmPlan& p, const T* A, const T* const* X, T* P, const int* gate,
                       int epoch, hipStream_t st) {
  const dim3 grid((unsigned)cdiv(cdiv(p.m, 4), 4), (unsigned)p.ax_S);
  for (int64_t c0 = 0; c0 < p.l; c0 += LB) {
    if (p.ax_vec)
      glx_launch((k_ax_valu<T, LB, 4, true, NSRC>), grid, dim3(256), 0, st, A, X[0], X[1],
                         X[2], P, p.m, p.n, p.l, (int)c0, p.ax_S, gate, epoch);
    else
      glx_launch((k_ax_valu<T, LB, 4, false, NSRC>), grid, dim3(256), 0, st, A, X[0], X[1],
                         X[2], P, p.m, p.n, p.l, (int)c0, p.ax_S, gate, epoch);
  }
}

template <typename T, int NSRC>
static void ax_valu_src(const GemmPlan& p, const T* A, const T* const* X, T* P, const int* gate,
                        int epoch, hipStream_t st) {
  switch (p.ax_lb) {
    case 1: ax_valu_lb<T, 1, NSRC>(p, A, X, P, gate, epoch, st); break;
    case 2: ax_valu_lb<T, 2, NSRC>(p, A, X, P, gate, epoch, st); break;
    case 4: ax_valu_lb<T, 4, NSRC>(p, A, X, P, gate, epoch, st); break;
    default: ax_valu_lb<T, 8, NSRC>(p, A, X, P, gate, epoch, st); break;
  }
}

template <typename T, int NT, int NSRC, int MT, int PF, bool QUAD, bool NTL, int VPL = 1>
static void ax_mfma_go(const GemmPlan& p, const T* A, const T* const* X, T* P, const int* gate,
                       int epoch, hipStream_t st) {
  constexpr int E = 16 / sizeof(T);
  const int gx = (int)cdiv(p.m, 16 * MT);
  const int xmap = ((p.ax_xmap & 1) && ax_xmap_ok(p.ax_S)) ? 1 : 0;
  const dim3 grid((unsigned)ax_grid(xmap, gx, p.ax_S));
  glx_launch((k_ax_mfma<T, MT, NT, NSRC, PF, QUAD, NTL, VPL>), grid, dim3(256), 0, st, A,
                     X[0], X[1], X[2], P, p.m, p.n, p.n / (4 * VPL * E), p.ax_S, gx, xmap, gate,
                     epoch);
}

template <typename T, int NT, int NSRC, int MT, int PF, int VPL, int WAVES, int DRV = 0>
static void ax_lds_go(const GemmPlan& p, int S, const T* A, const T* const* X, T* P,
                      const int* gate, int epoch, hipStream_t st, Pub pub = Pub{},
                      const AxDerive& drv = AxDerive{}) {
  constexpr int E = 16 / sizeof(T);
  const int gx = (int)cdiv(p.m, 16 * MT * WAVES);
  const int xmap = ax_xmap_flags(p, S);
  const unsigned dense = (unsigned)ax_grid(xmap, gx, S) + (pub.host ? 1u : 0u);
  AxDerive dv = drv;
  dv.thr0 = (int)dense;
  dv.gat0 = (int)dense + dv.nd;
  const dim3 grid(dense + (DRV ? (unsigned)(dv.nd + dv.ggx * p.l) : 0u));
  if constexpr (DRV) {
    static const size_t pad = lds_pad(k_ax_lds_drv<T, MT, NT, NSRC, PF, VPL, WAVES, DRV>, "GLX_AX_LDS_PAD");
    glx_launch((k_ax_lds_drv<T, MT, NT, NSRC, PF, VPL, WAVES, DRV>), grid, dim3(64 * WAVES), pad, st, A, X[0],
               X[1], X[2], P, p.m, p.n, p.n / (4 * VPL * E), S, gx, xmap, gate, epoch, pub, dv);
  } else {
    static const size_t pad = lds_pad(k_ax_lds<T, MT, NT, NSRC, PF, VPL, WAVES>, "GLX_AX_LDS_PAD");
    glx_launch((k_ax_lds<T, MT, NT, NSRC, PF, VPL, WAVES>), grid, dim3(64 * WAVES), pad, st, A, X[0], X[1],
               X[2], P, p.m, p.n, p.n / (4 * VPL * E), S, gx, xmap, gate, epoch, pub, dv);
  }
}

// the planner's kind-5 tiles (lds_plan): 52228 (f64 batched / one RHS in the Infinity Cache),
// 52224 (its 4-wave form for deep-split shards), 51328 (one 16-row tile per wave: the
// one-RHS and shard tile at l = 32), 52324 (f32 batched)
template <typename T, int NT, int NSRC>
static void ax_lds_code(const GemmPlan& p, int code, int S, const T* A, const T* const* X, T* P,
                        const int* gate, int epoch, hipStream_t st, Pub pub) {
  if (dma_kind(code)) {
    if (!launch_ax_dma<T>(p, code, NSRC, S, A, X, P, gate, epoch, st, pub))
      throw Error{GLX_E_INVALID, "A@X: unknown LDS-DMA tile code"};
    return;
  }
  switch (code) {
    case 52228: ax_lds_go<T, NT, NSRC, 2, 2, 2, 8>(p, S, A, X, P, gate, epoch, st, pub); break;
    case 51328: ax_lds_go<T, NT, NSRC, 1, 3, 2, 8>(p, S, A, X, P, gate, epoch, st, pub); break;
    case 52324: ax_lds_go<T, NT, NSRC, 2, 3, 2, 4>(p, S, A, X, P, gate, epoch, st, pub); break;
    case 52224: ax_lds_go<T, NT, NSRC, 2, 2, 2, 4>(p, S, A, X, P, gate, epoch, st, pub); break;
    default: throw Error{GLX_E_INVALID, "A@X: unknown LDS tile code"};
  }
}

// Direct-load tiles (kinds 1/2) only where no LDS tile fits the shape (lds_code_ok: l not 16/32
// is VALU; n not a multiple of the LDS chunk): 21820 / 1820 (f64, or any n % 4E), 21410 (f32),
// and for batched sources 1420 / 1220.
template <typename T, int NT>
static void ax_mfma_nt(const GemmPlan& p, int nsrc, const T* A, const T* const* X, T* P,
                       const int* gate, int epoch, hipStream_t st, Pub pub) {
  const int code = p.axb_code[nsrc];
  if (lds_kind(code)) {
    if (nsrc == 1) ax_lds_code<T, NT, 1>(p, code, p.axb_S[1], A, X, P, gate, epoch, st, pub);
    else if (nsrc == 2) ax_lds_code<T, NT, 2>(p, code, p.axb_S[2], A, X, P, gate, epoch, st, pub);
    else ax_lds_code<T, NT, 3>(p, code, p.axb_S[3], A, X, P, gate, epoch, st, pub);
    return;
  }
  if (pub.host != nullptr) throw Error{GLX_E_INVALID, "A@X: this tile cannot carry the scalar packet"};
  if (nsrc == 2) {
    ax_mfma_go<T, NT, 2, 4, 2, false, false>(p, A, X, P, gate, epoch, st);
    return;
  }
  if (nsrc == 3) {
    ax_mfma_go<T, NT, 3, 2, 2, false, false>(p, A, X, P, gate, epoch, st);
    return;
  }
  switch (p.ax_code) {
    case 21820: ax_mfma_go<T, NT, 1, 8, 2, false, false, 2>(p, A, X, P, gate, epoch, st); break;
    case 21410: ax_mfma_go<T, NT, 1, 4, 1, false, false, 2>(p, A, X, P, gate, epoch, st); break;
    default: ax_mfma_go<T, NT, 1, 8, 2, false, false>(p, A, X, P, gate, epoch, st); break;   // 1820
  }
}

bool ax_pub_ok(const GemmPlan& p, int nsrc) {
  return p.ax_kind != 3 && (p.l == 16 || p.l == 32) && nsrc >= 1 && nsrc <= 3 &&
         lds_kind(p.axb_code[nsrc]);
}

template <typename T>
void launch_ax(const GemmPlan& p, int nsrc, const T* A, const T* const* X, T* P, const int* gate,
               int epoch, hipStream_t st, Pub pub) {
  if (pub.host != nullptr && !ax_pub_ok(p, nsrc))
    throw Error{GLX_E_INVALID, "A@X: this plan cannot carry the scalar packet"};
  if (p.ax_kind == 3) {
    if (nsrc == 1) ax_valu_src<T, 1>(p, A, X, P, gate, epoch, st);
    else if (nsrc == 2) ax_valu_src<T, 2>(p, A, X, P, gate, epoch, st);
    else ax_valu_src<T, 3>(p, A, X, P, gate, epoch, st);
    return;
  }
  if (p.l == 16) ax_mfma_nt<T, 1>(p, nsrc, A, X, P, gate, epoch, st, pub);
  else ax_mfma_nt<T, 2>(p, nsrc, A, X, P, gate, epoch, st, pub);
}

bool ax_derive_ok(const GemmPlan& p, int esize) {
  return esize == 8 && p.ax_kind == 5 && p.axb_code[1] == 51328 && p.l == 32 && p.n % 16 == 0;
}

template <typename T>
bool launch_ax_derive(const GemmPlan& p, const T* A, const T* Xp, T* P, hipStream_t st, Pub pub,
                      const AxDerive& d) {
  if constexpr (sizeof(T) != 8) {
    return false;
  } else {
    if (!ax_derive_ok(p, 8) || pub.host == nullptr || d.pthr == nullptr) return false;
    if (d.ggx <= 0 || p.n % 64 != 0 || d.srows % 64 != 0 || d.srows <= 0 || d.blk == nullptr ||
        (int64_t)d.ggx * kDrvGatRows < p.m || p.n > 65536)
      return false;
    AxDerive dd = d;
    dd.sp.pub = pub;
    dd.nd = kDrvThrBlocks;
    const T* xs[3] = {Xp, nullptr, nullptr};
    ax_lds_go<T, 2, 1, 1, 3, 2, 8, 1>(p, p.axb_S[1], A, xs, P, nullptr, 0, st, pub, dd);
    return true;
  }
}
template bool launch_ax_derive<double>(const GemmPlan&, const double*, const double*, double*, hipStream_t, Pub,
                                       const AxDerive&);
template bool launch_ax_derive<float>(const GemmPlan&, const float*, const float*, float*, hipStream_t, Pub,
                                      const AxDerive&);

template void launch_ax<double>(const GemmPlan&, int, const double*, const double* const*, double*, const int*, int, hipStream_t, Pub);
template void launch_ax<float>(const GemmPlan&, int, const float*, const float* const*, float*, const int*, int, hipStream_t, Pub);
}  // namespace glx
