// kernels_gather.hip — the thresholded part of ProxGD's line-search candidate, A e, read from a
// transposed copy of A (split-candidate mode, solver.cpp iter_proxgd).
//
// The candidate p of a ProxGD trial is recorded (objective, gl_ProxGD_primal.py:112) before the
// hard threshold (:127) turns it into the next iterate p_thr, so one trial needs A p and A p_thr.
// Here A p = A p_thr + A e with e = p - p_thr: e is exactly p in the entries |p| < thres and 0
// elsewhere, and only a fraction of the rows of x have such entries (≈ 3 000 of 16 384 at the
// north-star size, ≈ 560 in the first iterations). A p_thr streams A once (the dense A@X tile
// with one right-hand side, HBM-bound); A e needs column k of A for every flagged row k of e,
// which is row k of At = A^T (n x m, one contiguous m-vector), built once per session:
//
//   P[r][c] = sum over the k with e[k][c] != 0 (ascending):  At[k][r] * e[k][c]
//
// e has about one nonzero per flagged row, so A e is computed column by column on the VALU
// (k_at_gather below), reading At only for the nonzeros: ≈ 230 MB at 3 500 nonzeros instead of a
// second dense pass (1 GiB of MFMA-bound work). The result goes to the finalize kernel, which
// forms A p - b = (A p_thr - b) + A e. (A 16x16x4 MFMA form over the flagged rows measured 72 us
// a trial at NS, round 2: its flops were ~97 % zeros.)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "glx.h"
#include "glx_device.h"
#include "glx_mfma.h"

namespace glx {

namespace {
constexpr int kGW = 4;                  // waves per workgroup
constexpr int kGThreads = 64 * kGW;
}  // namespace

// At = A^T through 64 x 64 LDS tiles (padded rows: conflict-free transposed reads)
template <typename T>
__global__ __launch_bounds__(256) void k_transpose(const T* __restrict__ A, T* __restrict__ At,
                                                   int64_t m, int64_t n) {
  __shared__ T tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = ty + 4 * k;
    const int64_t r = r0 + rr, c = c0 + tx;
    tile[rr][tx] = (r < m && c < n) ? A[r * n + c] : T(0);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int cc = ty + 4 * k;
    const int64_t c = c0 + cc, r = r0 + tx;
    if (c < n && r < m) At[c * m + r] = tile[tx][cc];
  }
}

// Column lists of e (one workgroup per column c): the ascending k whose column mask zm[k] (written
// by the trial kernels, bit c = e[k][c] != 0) has bit c. Thread t owns the masks
// [t * per, (t + 1) * per) as 16-B vectors, up to 16 in flight; a count, one block scan, and a
// write pass over the same vectors (L1/L2 hits); no LDS beyond the scan's 16 B. It runs on the
// solver's stream right before the dense pass. Round 2 ran the lists on a side stream beside the
// dense pass (byte row flags, then e[k][c] of every flagged row, 32 KiB of LDS): the kernel trace
// showed them getting CUs only once the dense pass drained (the LDS-DMA tile fills every CU's
// LDS), and the cross-stream wait ordering the gather behind them left 11-19 us idle per trial.
// Building each column's list inside every gather workgroup instead made the gather 40 us
// instead of 13 (profiles/r3_gather/).
__global__ __launch_bounds__(kGThreads) void k_e_lists(const unsigned* __restrict__ zm, int64_t n,
                                                       unsigned short* __restrict__ lists,
                                                       unsigned* __restrict__ counts,
                                                       const int* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  __shared__ unsigned wsum[kGW];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const unsigned c = blockIdx.x;
  constexpr int V = 16;   // vectors in flight per thread
  const int64_t per = (((n + kGThreads - 1) / kGThreads) + 3) & ~int64_t(3);
  const int64_t f0 = tid * per;
  const int64_t f1 = f0 + per < n ? f0 + per : (f0 < n ? n : f0);
  auto chunk = [&](int64_t k0, unsigned (&w)[4 * V]) {
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t k = k0 + 4 * u;
      const uint4 v = k < f1 ? *reinterpret_cast<const uint4*>(zm + k) : uint4{0u, 0u, 0u, 0u};
      w[4 * u] = v.x; w[4 * u + 1] = v.y; w[4 * u + 2] = v.z; w[4 * u + 3] = v.w;
    }
  };
  // the first 4V masks of the thread's range stay in registers for the write pass (the whole
  // range at n <= 4V * 256 = 16384: one load round per kernel instead of two)
  unsigned w0[4 * V];
  chunk(f0, w0);
  unsigned cnt = 0;
#pragma unroll
  for (int j = 0; j < 4 * V; ++j)
    if (f0 + j < f1 && ((w0[j] >> c) & 1u)) ++cnt;
  for (int64_t k0 = f0 + 4 * V; k0 < f1; k0 += 4 * V) {
    unsigned w[4 * V];
    chunk(k0, w);
#pragma unroll
    for (int j = 0; j < 4 * V; ++j)
      if (k0 + j < f1 && ((w[j] >> c) & 1u)) ++cnt;
  }
  // block-exclusive scan of the counts
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
  for (int w = 0; w < kGW; ++w) {
    if (w < wave) pos += wsum[w];
    total += wsum[w];
  }
  unsigned short* out = lists + (int64_t)c * n;
  if (cnt != 0) {
#pragma unroll
    for (int j = 0; j < 4 * V; ++j)
      if (f0 + j < f1 && ((w0[j] >> c) & 1u)) out[pos++] = (unsigned short)(f0 + j);
    for (int64_t k0 = f0 + 4 * V; k0 < f1; k0 += 4 * V) {
      unsigned w[4 * V];
      chunk(k0, w);
#pragma unroll
      for (int j = 0; j < 4 * V; ++j)
        if (k0 + j < f1 && ((w[j] >> c) & 1u)) out[pos++] = (unsigned short)(k0 + j);
    }
  }
  if (tid == 0) counts[c] = total;
}

// One workgroup per (256-row block, column c) of A e. e has few nonzeros per flagged row (about
// one of the 32 columns at the north-star size), so a dense 16x16x4 MFMA over all 32 columns
// would spend ~97 % of its flops on zeros: here every output element is a fp64 VALU dot product
// over column c's list (k_e_lists) in its ascending order (deterministic); thread t (row
// r = 256 rb + t) keeps 8 loads in flight and the 64 lanes of a wave read 512 contiguous bytes
// of one At row. out[r][c] = the sum (one slab: no K split).
// NT: At read with the non-temporal policy (each of its rows is read at most once per trial;
// GLX_GATHER_NT)
// GW waves per workgroup (round 4, GLX_GATHER_WAVES): with 1-wave workgroups the grid has 4x as
// many, so the dispatcher keeps refilling CUs as the short columns finish instead of every CU
// holding four workgroups that all wait for the longest list of their columns.
template <typename T, int L, bool NT, int GW>
__global__ __launch_bounds__(64 * GW) void k_at_gather(const T* __restrict__ At,
                                                         const T* __restrict__ E,
                                                         const unsigned short* __restrict__ lists,
                                                         const unsigned* __restrict__ counts,
                                                         int64_t m, int64_t n, T* __restrict__ P,
                                                         int gx, const int* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int rb = (int)blockIdx.x % gx, c = (int)blockIdx.x / gx;
  const int total = (int)counts[c];
  const unsigned short* lst = lists + (int64_t)c * n;
  const int64_t r = (int64_t)rb * (64 * GW) + threadIdx.x;
  const int64_t rr = r < m ? r : m - 1;
  constexpr int U = 8;
  T acc = T(0);
  int idx = 0;
  for (; idx + U <= total; idx += U) {
    T a[U], ev[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = lst[idx + u];
      a[u] = NT ? __builtin_nontemporal_load(At + k * m + rr) : At[k * m + rr];
      ev[u] = E[k * L + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = acc + a[u] * ev[u];
  }
  for (; idx < total; ++idx) {
    const int64_t k = lst[idx];
    acc = acc + (NT ? __builtin_nontemporal_load(At + k * m + rr) : At[k * m + rr]) * E[k * L + c];
  }
  if (r < m) P[r * L + c] = acc;
}

// The same with two output rows per thread (round 4, GLX_GATHER_VEC=1): each thread loads
// At[k][r], At[k][r + 1] as one 16-B vector, so a wave-instruction reads 1 KiB of the At row
// instead of 512 B (8-B loads read at 0.54-0.70x the 16-B rate, MI355X_MICROARCH.md visibility
// table). Per output element the same ascending-k sum: bit-identical to k_at_gather. Measured
// over whole NS solves: 56.6 us against 53.8 us for k_at_gather (half the waves in flight),
// so it is not the default (profiles/r4_gvec/). Needs m even (16-B alignment of every At row).
template <typename T, int L, bool NT>
__global__ __launch_bounds__(kGThreads) void k_at_gather2(const T* __restrict__ At,
                                                          const T* __restrict__ E,
                                                          const unsigned short* __restrict__ lists,
                                                          const unsigned* __restrict__ counts,
                                                          int64_t m, int64_t n, T* __restrict__ P,
                                                          int gx, const int* __restrict__ skip) {
  static_assert(sizeof(T) == 8, "fp64: two rows = one 16-B vector");
  if (skip != nullptr && *skip != 0) return;
  const int rb = (int)blockIdx.x % gx, c = (int)blockIdx.x / gx;
  const int total = (int)counts[c];
  const unsigned short* lst = lists + (int64_t)c * n;
  const int64_t r = ((int64_t)rb * kGThreads + threadIdx.x) * 2;
  const int64_t rr = r < m ? r : m - 2;
  constexpr int U = 8;
  T acc0 = T(0), acc1 = T(0);
  int idx = 0;
  for (; idx + U <= total; idx += U) {
    d2_t a[U];
    T ev[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = lst[idx + u];
      const d2_t* ap = reinterpret_cast<const d2_t*>(At + k * m + rr);
      a[u] = NT ? __builtin_nontemporal_load(ap) : *ap;
      ev[u] = E[k * L + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc0 = acc0 + a[u][0] * ev[u];
      acc1 = acc1 + a[u][1] * ev[u];
    }
  }
  for (; idx < total; ++idx) {
    const int64_t k = lst[idx];
    const d2_t* ap = reinterpret_cast<const d2_t*>(At + k * m + rr);
    const d2_t a = NT ? __builtin_nontemporal_load(ap) : *ap;
    const T ev = E[k * L + c];
    acc0 = acc0 + a[0] * ev;
    acc1 = acc1 + a[1] * ev;
  }
  if (r < m) {
    P[r * L + c] = acc0;
    P[(r + 1) * L + c] = acc1;
  }
}

// Round 5: the same gather without k_e_lists (k_at_gather_bm, the default). The trial kernels
// also write per-column row bitmaps of e (glx_device.h zf_store_panel / zf_store_group16), and
// each workgroup (row block rb, column c) builds column c's ascending row list itself, in LDS:
// thread t takes the u64 bitmap words t, t + 256, ... of a 256-word segment (16 384 rows), a
// popcount, one block scan, the set bits written in order; then the same walk as k_at_gather
// with the indices read from LDS. Same list, same order, same arithmetic: bit-identical to
// k_e_lists + k_at_gather, one launch and ~8 us fewer per trial (the lists kernel's 32
// workgroups ran alone on the chip). counts[c] (rb == 0) = the list length (FProxGD's budget).
// U: At loads in flight per thread; SEGW: bitmap words per segment (64 SEGW rows, its list in
// 128 SEGW bytes of LDS; 128: twice the workgroups per CU). Neither changes the summation order.
// VEC: each thread owns E = 16 / sizeof(T) consecutive output rows and reads them with one 16-B
// load per list entry (1 KiB per wave-instruction instead of 512 B; 8-B loads stream at ~0.54-0.70
// of the 16-B rate, MI355X_MICROARCH.md), each row's sum in the same order (needs m % E == 0).
template <typename T, int L, bool NT, int U, int SEGW, bool VEC = false>
__global__ __launch_bounds__(kGThreads) void k_at_gather_bm(const T* __restrict__ At,
                                                            const T* __restrict__ E,
                                                            unsigned* __restrict__ zf, int64_t m,
                                                            int64_t n, T* __restrict__ P,
                                                            unsigned* __restrict__ counts, int gx,
                                                            const int* __restrict__ skip) {
  static_assert(SEGW <= kGThreads, "one bitmap word per thread and segment");
  if (skip != nullptr && *skip != 0) return;
  __shared__ unsigned short lst[64 * SEGW];   // one segment: SEGW words x 64 rows
  __shared__ unsigned wsum[kGW];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int rb = (int)blockIdx.x % gx, c = (int)blockIdx.x / gx;
  const int64_t nw = zf_npad(n) / 64;
  const uint64_t* words = reinterpret_cast<const uint64_t*>(zf_bitmaps(zf, n) + (int64_t)c * (zf_npad(n) / 16));
  typedef typename MF<T>::vec_t V;
  constexpr int RW = VEC ? MF<T>::E : 1;   // output rows per thread
  const int64_t r = ((int64_t)rb * kGThreads + tid) * RW;
  const int64_t rr = r < m ? r : m - RW;
  T acc[RW];
#pragma unroll
  for (int j = 0; j < RW; ++j) acc[j] = T(0);
  auto ldat = [&](int64_t k, T (&a)[RW]) {
    if constexpr (VEC) {
      const V* ap = reinterpret_cast<const V*>(At + k * m + rr);
      const V v = NT ? __builtin_nontemporal_load(ap) : *ap;
#pragma unroll
      for (int j = 0; j < RW; ++j) a[j] = v[j];
    } else {
      a[0] = NT ? __builtin_nontemporal_load(At + k * m + rr) : At[k * m + rr];
    }
  };
  unsigned all = 0;
  for (int64_t w0 = 0; w0 < nw; w0 += SEGW) {
    const int64_t w = w0 + tid;
    uint64_t bits = (tid < SEGW && w < nw) ? words[w] : uint64_t(0);
    if (w == nw - 1 && (n & 63) != 0) bits &= (uint64_t(1) << (n & 63)) - 1;   // rows >= n: never
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
    for (int q = 0; q < kGW; ++q) {
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
      T a[U][RW], ev[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k = kb + lst[idx + u];
        ldat(k, a[u]);
        ev[u] = E[k * L + c];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < RW; ++j) acc[j] = acc[j] + a[u][j] * ev[u];
    }
    for (; idx < tot; ++idx) {
      const int64_t k = kb + lst[idx];
      T a[RW];
      ldat(k, a);
      const T ev = E[k * L + c];
#pragma unroll
      for (int j = 0; j < RW; ++j) acc[j] = acc[j] + a[j] * ev;
    }
    all += total;
    __syncthreads();   // lst and wsum are rewritten by the next segment
  }
#pragma unroll
  for (int j = 0; j < RW; ++j)
    if (r + j < m) P[(r + j) * L + c] = acc[j];
  if (rb == 0 && tid == 0) counts[c] = all;
}

// zf's column bitmaps from its n row masks (glx_flagged_rows_product's bitmap form, where no
// trial kernel wrote them): thread (c, word g) ORs bit c of the 16 masks of rows 16 g .. 16 g + 15
__global__ void k_zf_bitmaps(unsigned* __restrict__ zf, int64_t n, int l) {
  const int64_t ng = zf_npad(n) / 16;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ng * l) return;
  const int c = (int)(t / ng);
  const int64_t g = t % ng;
  unsigned b = 0;
  for (int j = 0; j < 16; ++j) {
    const int64_t k = 16 * g + j;
    if (k < n) b |= ((zf[k] >> c) & 1u) << j;
  }
  zf_bitmaps(zf, n)[(int64_t)c * ng + g] = (unsigned short)b;
}

// ------------------------------------------------------------------------------------------
// Round 5: A e as the A^T R panel over the flagged rows of e (k_at_rows, the default).
//
//   P[s][r][c] = sum over the flagged rows k of K range s (ascending):  At[k][r] * e[k][c]
//
// i.e. Y = At_F^T e_F, the gradient contraction's shape (kernels_atr.hip atr_panel) with its K
// index (rows of A there, rows of At here) drawn from the list F of rows whose column mask zf[k]
// (written by the trial kernels) is nonzero. The VALU gather above reads one At row per NONZERO
// of e and one 512-B piece per wave-instruction at ~4.5 TB/s; this form reads each flagged row
// once, whatever its nonzero count, in the 512-B pieces of the A^T R panel (4 rows x 2 x 256 B per
// wave-instruction pair, non-temporal), and multiplies all l columns on MFMA: FProxGD's e_c
// (flagged rows ~0.4 n late in a solve) is dense enough that the zero products cost nothing
// beside the bytes, and ProxGD's e (~1.1 nonzeros per flagged row) pays 2 m l flops per row at
// l / 4 flop/B, still HBM-bound. No column lists: every workgroup compacts the flags of its own
// K range into an ascending list in LDS (a block scan over n / S0 masks, L2 hits), so k_e_lists
// goes too.
// Grid: (m / 64 panels) x S0 K splits; block = 4 waves splitting the K range's list (WL 0 of
// atr_panel), reduced through LDS in the fixed order ((w0 + w1) + w2) + w3. Slab s of P holds K
// range s; the finalize sums the S0 slabs in order: deterministic. counts[s] = the flagged rows
// of range s (panel 0's workgroup): FProxGD's budget input (nnz of e_c counted in rows).
// Needs m % 64 == 0 (whole panels, 16-B aligned At rows) and a K range of at most kRowsListMax
// rows (S0 >= n / kRowsListMax); else the VALU gather runs.
constexpr int kRowsListMax = 16384;   // u16 row indices (n <= 65535), 32 KiB of LDS

template <typename T, int NT, int PF, bool NTL>
__global__ __launch_bounds__(256, 2) void k_at_rows(const T* __restrict__ At, const T* __restrict__ E,
                                                    const unsigned* __restrict__ zf, int64_t m,
                                                    int64_t n, int S0, T* __restrict__ P,
                                                    unsigned* __restrict__ counts,
                                                    const int* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  typedef MF<T> M;
  typedef typename M::acc_t C;
  constexpr int L = 16 * NT;
  constexpr int kRedBytes = 4 * 4 * NT * 64 * (int)sizeof(C);
  constexpr int kLdsBytes = kRedBytes > 2 * (kRowsListMax + 8) ? kRedBytes : 2 * (kRowsListMax + 8);
  // the list lives through the main loop, the wave partials after it: one buffer
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLdsBytes];
  __shared__ unsigned wsum[4];
  unsigned short* lst = reinterpret_cast<unsigned short*>(lds);
  C(*red)[4 * NT][64] = reinterpret_cast<C(*)[4 * NT][64]>(lds);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int64_t gp = m / 64;
  const int64_t panel = (int64_t)blockIdx.x % gp, split = (int64_t)blockIdx.x / gp;
  const int64_t col0 = panel * 64;
  // K range of this split in whole 64-row chunks (16-B aligned mask loads)
  const int64_t nch = (n + 63) / 64;
  const int64_t k0 = 64 * (nch * split / S0);
  const int64_t k1e = 64 * (nch * (split + 1) / S0);
  const int64_t k1 = k1e < n ? k1e : n;

  // ---- compaction: thread t owns the masks [k0 + t per, k0 + (t + 1) per), per % 4 == 0
  const int64_t len = k1 - k0;
  const int64_t per = (((len + 255) / 256) + 3) & ~int64_t(3);   // <= 64 (len <= 16384)
  const int64_t f0 = k0 + tid * per;
  uint64_t bits = 0;   // bit j: row f0 + j flagged
  for (int64_t j = 0; j < per; j += 4) {
    const int64_t k = f0 + j;
    if (k < k1) {
      const uint4 v = *reinterpret_cast<const uint4*>(zf + k);
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k + u < k1 && w[u] != 0u) bits |= uint64_t(1) << (j + u);
    }
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
  unsigned pos = inc - cnt, R = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (w < wave) pos += wsum[w];
    R += wsum[w];
  }
  while (bits != 0) {
    const int j = __builtin_ctzll(bits);
    bits &= bits - 1;
    lst[pos++] = (unsigned short)(f0 + j);
  }
  __syncthreads();
  // pad the last row step: positions R .. R + 3 repeat a valid row, their e is taken as 0
  if (tid < 4) lst[R + tid] = (unsigned short)(R > 0 ? lst[R - 1] : k0);
  if (panel == 0 && tid == 0) counts[split] = R;
  __syncthreads();

  // ---- the A^T R panel over the list (atr_panel, WL 0): wave w takes row steps [sb, se)
  const int Ri = __builtin_amdgcn_readfirstlane((int)R);
  const int steps = (Ri + 3) / 4;
  const int sb = steps * wave / 4, se = steps * (wave + 1) / 4;
  const int nst = __builtin_amdgcn_readfirstlane(se - sb);
  C acc[4][NT];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[e][nt] = C{};
  T a[PF][4], rb[PF][NT];
  // ring slot p's next row: its index is read from the LDS list one ring cycle ahead of the
  // global loads that use it, so no LDS wait sits in front of a load issue
  int kx[PF];
  bool lv[PF];
  auto fetch = [&](int p, int off) {
    off = off < nst ? off : nst - 1;   // past the end: the last step again (never consumed)
    const int pos = (sb + off) * 4 + q;
    kx[p] = lst[pos];
    lv[p] = pos < Ri;
  };
  auto ld = [&](int p) {
    const int64_t k = kx[p];
    Load4<T, NTL>::go(At + k * m + col0 + atr_col<T>(i, 0), a[p]);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const T ev = E[k * L + nt * 16 + i];
      rb[p][nt] = lv[p] ? ev : T(0);
    }
  };
  auto mma_step = [&](int p) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[e][nt] = M::mma(a[p][e], rb[p][nt], acc[e][nt]);
  };
  if (nst > 0) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      fetch(p, p);
      ld(p);
      fetch(p, p + PF);
    }
    int s0 = 0;
    for (; s0 + PF <= nst; s0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        mma_step(p);
        ld(p);
        fetch(p, s0 + p + 2 * PF);
      }
    }
#pragma unroll
    for (int p = 0; p < PF - 1; ++p)
      if (s0 + p < nst) mma_step(p);
  }
  __syncthreads();   // the list is dead: its LDS takes the wave partials
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) red[wave][e * NT + nt][lane] = acc[e][nt];
  __syncthreads();
  T* out = P + split * m * L;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    C v = red[0][wave * NT + nt][lane];
#pragma unroll
    for (int s = 1; s < 4; ++s) v += red[s][wave * NT + nt][lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = col0 + atr_col<T>(M::row(lane, r), wave);
      out[row * L + nt * 16 + i] = v[r];
    }
  }
}

static int env_rows_s() {
  const char* e = std::getenv("GLX_ATROWS_S");
  return e ? std::atoi(e) : 0;
}
// the shapes the MFMA row form (k_at_rows) takes: whole 64-row panels of At
bool gather_rows_ok(int64_t m, int64_t n) { return m % 64 == 0 && m > 0 && n <= 65535; }
// the A e form GLX_GATHER asks for: 0 = the bitmap gather ("bm", k_at_gather_bm), 1 = the MFMA
// row form ("rows", where gather_rows_ok), 2 = k_e_lists + k_at_gather ("lists", rounds 2-4),
// -1 = unset (the solver's per-method default)
int gather_form() {
  const char* e = std::getenv("GLX_GATHER");
  if (e && std::strcmp(e, "rows") == 0) return 1;
  if (e && (std::strcmp(e, "lists") == 0 || std::strcmp(e, "valu") == 0)) return 2;
  if (e && std::strcmp(e, "bm") == 0) return 0;
  return -1;
}
// K splits of the row form: about two workgroups per CU (512 on 256 CUs), each K range within
// the LDS list; GLX_ATROWS_S overrides (clamped to that bound)
int gather_split(int64_t m, int64_t n) {
  if (!gather_rows_ok(m, n)) return 1;   // the VALU gather: ONE slab
  const int64_t gp = m / 64;
  const int64_t need = (n + kRowsListMax - 1) / kRowsListMax;
  int64_t s = env_rows_s() > 0 ? env_rows_s() : (512 + gp - 1) / gp;
  s = s < 1 ? 1 : (s > 16 ? 16 : s);
  return (int)(s < need ? need : s);
}

bool gather_ok(int64_t n, int64_t l) { return (l == 16 || l == 32) && n <= 65535; }

template <typename T>
void launch_transpose(const T* A, T* At, int64_t m, int64_t n, hipStream_t st) {
  const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((m + 63) / 64));
  hipLaunchKernelGGL(k_transpose<T>, grid, dim3(256), 0, st, A, At, m, n);
}

size_t gather_lists_bytes(int64_t n);

static unsigned* list_counts(void* lists_ws, int64_t n) {
  return reinterpret_cast<unsigned*>(static_cast<char*>(lists_ws) + gather_lists_bytes(n) - 256);
}
const unsigned* gather_counts(const void* lists_ws, int64_t n) {
  return list_counts(const_cast<void*>(lists_ws), n);
}

void launch_e_lists(const unsigned* zm, int64_t n, int64_t l, void* lists_ws, hipStream_t st,
                    const int* skip) {
  if (!gather_ok(n, l)) throw Error{GLX_E_INVALID, "A e gather: needs l in {16, 32}, n < 65536"};
  hipLaunchKernelGGL(k_e_lists, dim3((unsigned)l), dim3(kGThreads), 0, st, zm, n,
                     static_cast<unsigned short*>(lists_ws), list_counts(lists_ws, n), skip);
}

template <typename T>
void launch_at_gather(const T* At, const T* E, int64_t m, int64_t n, int64_t l, T* P, void* lists_ws,
                      hipStream_t st, const int* skip) {
  if (!gather_ok(n, l)) throw Error{GLX_E_INVALID, "A e gather: needs l in {16, 32}, n < 65536"};
  const unsigned short* lists = static_cast<const unsigned short*>(lists_ws);
  static const bool nt = [] {
    const char* e = std::getenv("GLX_GATHER_NT");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  const int gw = [] {   // read per launch (tests switch it within one process)
    const char* e = std::getenv("GLX_GATHER_WAVES");
    const int v = e ? std::atoi(e) : 4;
    return (v == 1 || v == 2) ? v : 4;
  }();
  auto go = [&](auto kern, int waves) {
    const int gx = (int)((m + 64 * waves - 1) / (64 * waves));
    glx_launch(kern, dim3((unsigned)(gx * l)), dim3(64 * waves), 0, st, At, E, lists,
                       list_counts(lists_ws, n), m, n, P, gx, skip);
  };
  auto go_l = [&](auto kern4, auto kern2, auto kern1) {
    if (gw == 1) go(kern1, 1);
    else if (gw == 2) go(kern2, 2);
    else go(kern4, 4);
  };
  const bool vec = [] {   // measured slower over whole NS solves (56.6 vs 53.8 us): off
    const char* e = std::getenv("GLX_GATHER_VEC");
    return e && std::strcmp(e, "1") == 0;
  }();
  if constexpr (sizeof(T) == 8) {
    if (vec && m % 2 == 0) {   // two rows per thread, 16-B loads
      const int gx = (int)((m / 2 + kGThreads - 1) / kGThreads);
      auto g2 = [&](auto kern) {
        glx_launch(kern, dim3((unsigned)(gx * l)), dim3(kGThreads), 0, st, At, E, lists,
                   list_counts(lists_ws, n), m, n, P, gx, skip);
      };
      if (l == 32) nt ? g2(k_at_gather2<T, 32, true>) : g2(k_at_gather2<T, 32, false>);
      else nt ? g2(k_at_gather2<T, 16, true>) : g2(k_at_gather2<T, 16, false>);
      return;
    }
  }
  if (l == 32) {
    if (nt) go_l(k_at_gather<T, 32, true, 4>, k_at_gather<T, 32, true, 2>, k_at_gather<T, 32, true, 1>);
    else go_l(k_at_gather<T, 32, false, 4>, k_at_gather<T, 32, false, 2>, k_at_gather<T, 32, false, 1>);
  } else {
    if (nt) go_l(k_at_gather<T, 16, true, 4>, k_at_gather<T, 16, true, 2>, k_at_gather<T, 16, true, 1>);
    else go_l(k_at_gather<T, 16, false, 4>, k_at_gather<T, 16, false, 2>, k_at_gather<T, 16, false, 1>);
  }
}

// A e by the column bitmaps the trial kernels wrote behind zf (k_at_gather_bm): ONE slab at P,
// the column list lengths into the counts area of lists_ws (gather_counts). GLX_GATHER_BM =
// "U,SEGW,VEC" selects the loads in flight, the segment and the 16-B row form (default 8,256,1:
// NS 200-step windows 42.2-42.4 against 44.7 us for 8-B loads, whole solves 2456-2458 against
// 2433-2436 it/s, profiles/r5_h/; 16 loads in flight or 128-word segments measured slower).
template <typename T, int L, bool NT>
static void at_gather_bm_go(int code, int64_t m, hipStream_t st, const T* At, const T* E, unsigned* zf,
                            int64_t n, int64_t l, T* P, unsigned* cnt, const int* skip) {
  const bool vec = (code % 10) == 1 && m % MF<T>::E == 0;
  const int rpb = kGThreads * (vec ? MF<T>::E : 1);   // output rows per workgroup
  const int gx = (int)((m + rpb - 1) / rpb);
  const dim3 g((unsigned)(gx * l));
  switch (vec ? code : code / 10 * 10) {
    case 162560: glx_launch(k_at_gather_bm<T, L, NT, 16, 256>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    case 81280: glx_launch(k_at_gather_bm<T, L, NT, 8, 128>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    case 161280: glx_launch(k_at_gather_bm<T, L, NT, 16, 128>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    case 82561: glx_launch(k_at_gather_bm<T, L, NT, 8, 256, true>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    case 162561: glx_launch(k_at_gather_bm<T, L, NT, 16, 256, true>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    case 81281: glx_launch(k_at_gather_bm<T, L, NT, 8, 128, true>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    case 161281: glx_launch(k_at_gather_bm<T, L, NT, 16, 128, true>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
    default: glx_launch(k_at_gather_bm<T, L, NT, 8, 256>, g, dim3(kGThreads), 0, st, At, E, zf, m, n, P, cnt, gx, skip); break;
  }
}
template <typename T>
void launch_at_gather_bm(const T* At, const T* E, unsigned* zf, int64_t m, int64_t n, int64_t l, T* P,
                         void* lists_ws, hipStream_t st, const int* skip) {
  if (!gather_ok(n, l)) throw Error{GLX_E_INVALID, "A e gather: needs l in {16, 32}, n < 65536"};
  static const bool nt = [] {
    const char* e = std::getenv("GLX_GATHER_NT");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  const int code = [] {   // read per launch (tests switch it within one process)
    const char* e = std::getenv("GLX_GATHER_BM");
    int u = 8, w = 256, v = 1;   // round 5: the 16-B row form (42.2-42.4 vs 44.7 us at NS)
    if (e && *e) std::sscanf(e, "%d,%d,%d", &u, &w, &v);
    return ((u == 16 ? 16 : 8) * 1000 + (w == 128 ? 128 : 256)) * 10 + (v == 1 ? 1 : 0);
  }();
  unsigned* cnt = list_counts(lists_ws, n);
  if (l == 32) {
    if (nt) at_gather_bm_go<T, 32, true>(code, m, st, At, E, zf, n, l, P, cnt, skip);
    else at_gather_bm_go<T, 32, false>(code, m, st, At, E, zf, n, l, P, cnt, skip);
  } else {
    if (nt) at_gather_bm_go<T, 16, true>(code, m, st, At, E, zf, n, l, P, cnt, skip);
    else at_gather_bm_go<T, 16, false>(code, m, st, At, E, zf, n, l, P, cnt, skip);
  }
}
void launch_zf_bitmaps(unsigned* zf, int64_t n, int64_t l, hipStream_t st) {
  const int64_t t = zf_npad(n) / 16 * l;
  hipLaunchKernelGGL(k_zf_bitmaps, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, zf, n, (int)l);
}
// bytes of zf: the row masks (zf_npad(n) words) and the column bitmaps behind them
size_t zf_bytes(int64_t n) { return (((size_t)zf_npad(n) * 8) + 255) & ~size_t(255); }

// A e over the flagged rows (k_at_rows): S0 = gather_split(m, n) slabs at P, the flagged rows of
// each K range into the counts area of lists_ws (gather_counts)
template <typename T>
void launch_at_rows(const T* At, const T* E, const unsigned* zf, int64_t m, int64_t n, int64_t l,
                    T* P, void* lists_ws, hipStream_t st, const int* skip) {
  if (!gather_ok(n, l) || !gather_rows_ok(m, n))
    throw Error{GLX_E_INVALID, "A e row form: needs l in {16, 32}, m % 64 == 0, n < 65536"};
  const int S0 = gather_split(m, n);
  const dim3 grid((unsigned)(m / 64 * S0));
  unsigned* cnt = list_counts(lists_ws, n);
  static const bool nt = [] {
    const char* e = std::getenv("GLX_GATHER_NT");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  if (l == 32) {
    if (nt) glx_launch(k_at_rows<T, 2, 8, true>, grid, dim3(256), 0, st, At, E, zf, m, n, S0, P, cnt, skip);
    else glx_launch(k_at_rows<T, 2, 8, false>, grid, dim3(256), 0, st, At, E, zf, m, n, S0, P, cnt, skip);
  } else {
    if (nt) glx_launch(k_at_rows<T, 1, 8, true>, grid, dim3(256), 0, st, At, E, zf, m, n, S0, P, cnt, skip);
    else glx_launch(k_at_rows<T, 1, 8, false>, grid, dim3(256), 0, st, At, E, zf, m, n, S0, P, cnt, skip);
  }
}

// workspace of the column lists: l * n indices + 256 B of counts
size_t gather_lists_bytes(int64_t n) { return (((size_t)32 * n * 2 + 255) & ~size_t(255)) + 256; }

template void launch_at_rows<double>(const double*, const double*, const unsigned*, int64_t, int64_t,
                                     int64_t, double*, void*, hipStream_t, const int*);
template void launch_at_rows<float>(const float*, const float*, const unsigned*, int64_t, int64_t,
                                    int64_t, float*, void*, hipStream_t, const int*);
template void launch_at_gather_bm<double>(const double*, const double*, unsigned*, int64_t, int64_t,
                                          int64_t, double*, void*, hipStream_t, const int*);
template void launch_at_gather_bm<float>(const float*, const float*, unsigned*, int64_t, int64_t,
                                         int64_t, float*, void*, hipStream_t, const int*);
template void launch_transpose<double>(const double*, double*, int64_t, int64_t, hipStream_t);
template void launch_transpose<float>(const float*, float*, int64_t, int64_t, hipStream_t);
template void launch_at_gather<double>(const double*, const double*, int64_t, int64_t, int64_t, double*,
                                       void*, hipStream_t, const int*);
template void launch_at_gather<float>(const float*, const float*, int64_t, int64_t, int64_t, float*,
                                      void*, hipStream_t, const int*);

}  // namespace glx
