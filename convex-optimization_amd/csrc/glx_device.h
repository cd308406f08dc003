// glx_device.h — device-side helpers shared by kernels_elem.hip and kernels_gemm.hip:
// deterministic grid reductions, slab sums, per-row shuffles, and the ProxGD trial's per-row
// arithmetic (used by the standalone trial kernel and by the A^T R epilogue that fuses it, so
// both produce bit-identical results).
#ifndef GLX_DEVICE_H_
#define GLX_DEVICE_H_

#include "glx_internal.h"

namespace glx {

enum { OP_SUM = 0, OP_MAX = 1 };

__device__ inline double nan_max(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return a > b ? a : b;
}
__device__ inline double combine(int op, double a, double b) { return op == OP_MAX ? nan_max(a, b) : a + b; }
__device__ inline double identity(int op) { return op == OP_MAX ? -__builtin_inf() : 0.0; }

// Fixed-order combine of NW per-wave values: ((w0 + w1) + (w2 + w3)) [+ the same for w4..w7].
template <int NW>
__device__ inline double waves_combine(int op, const double* w) {
  double a = combine(op, combine(op, w[0], w[1]), combine(op, w[2], w[3]));
  if constexpr (NW == 8) a = combine(op, a, combine(op, combine(op, w[4], w[5]), combine(op, w[6], w[7])));
  return a;
}

// A launch of a device-controlled batch that an earlier decision has cancelled (Red::skip);
// the flag was written by an earlier kernel in the stream, so every workgroup reads the same value
__device__ inline bool red_skipped(const Red& red) {
  if (red.skip == nullptr) return false;
  const int v = *red.skip;
  return v != 0 && v != red.skip_pass;
}

// Reduce NV per-thread values over the grid; block size must be 64 * NW (NW = 4 or 8).
// MAXMASK bit v = max op. slot = this block's partials slot (default blockIdx.x): a launch
// whose first workgroup is a publisher (publisher_first) puts that one last and the others at
// blockIdx.x - 1, so the sums come out bit-identical with and without the packet.
// nparts >= 0: only nparts workgroups of the launch take part, each with a distinct slot in
// [0, nparts) (the K-split A^T R kernels: one per panel + the publisher, so the split count is
// not bounded by the partials row); the arrival shards are then keyed by slot, not blockIdx.
template <int NV, unsigned MAXMASK, int NW = 4>
__device__ bool grid_reduce(double (&v)[NV], const Red& red, int slot = -1, int nparts = -1) {
  static_assert(NW == 4 || NW == 8, "4- or 8-wave blocks");
  constexpr int NTHR = 64 * NW;
  __shared__ double sh[NV][NW];
  __shared__ int is_last;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int op = (MAXMASK >> j) & 1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[j] = combine(op, v[j], __shfl_xor(v[j], off));
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) sh[j][wave] = v[j];
  }
  __syncthreads();
  if (red.parts_only) {   // uniform over the grid: the block values are the result
    if (threadIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j)
        red.part[(slot < 0 ? (int)blockIdx.x : slot) * NV + j] = waves_combine<NW>((MAXMASK >> j) & 1, sh[j]);
    }
    return false;
  }
  if (threadIdx.x == 0) {
    // write-through (sc1) partial stores + drained vmcnt before the ticket: no release fence
    // (MI355X_MICROARCH.md, visibility "Valid forms" table, row 1)
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int op = (MAXMASK >> j) & 1;
      const double bv = waves_combine<NW>(op, sh[j]);
      __hip_atomic_store(&red.part[j * kMaxBlocks + (slot < 0 ? (int)blockIdx.x : slot)], bv,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // Two-level arrival: one device-scope counter costs ~12 ns per arriving block
    // (MI355X_MICROARCH.md, "fanin"), so 1024 blocks on one word serialise for ~12 us. Blocks
    // arrive on the counter of their shard (blockIdx % 8, i.e. their XCD under round-robin
    // dispatch); the last arriver of each shard, whose add returned after every add of its
    // shard, arrives on the final counter, and the last arriver there owns the sum.
    const unsigned G = nparts >= 0 ? (unsigned)nparts : gridDim.x;
    const unsigned sh = (nparts >= 0 ? (unsigned)slot : blockIdx.x) & (kTicketShards - 1);
    const unsigned nsh = G < (unsigned)kTicketShards ? G : (unsigned)kTicketShards;
    const unsigned cnt = (G - sh + kTicketShards - 1) / kTicketShards;
    const unsigned prev = __hip_atomic_fetch_add(red.ticket + (1 + sh) * kTicketStride, 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = 0;
    if (prev == cnt - 1)
      last = __hip_atomic_fetch_add(red.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1;
    is_last = last;
  }
  __syncthreads();
  if (!is_last) return false;
  // every load of the partials is an sc1 load (L1 bypass): no acquire fence needed. All of them
  // are issued before the first is consumed (clamped index, select afterwards), so the last
  // block pays one round trip instead of one per partial.
  constexpr int PER = kMaxBlocks / NTHR;
  const unsigned np = nparts >= 0 ? (unsigned)nparts : gridDim.x;
  double pv[NV][PER];
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const unsigned b = threadIdx.x + (unsigned)NTHR * t;
      const unsigned bc = b < np ? b : np - 1;
      pv[j][t] = __hip_atomic_load(&red.part[j * kMaxBlocks + bc], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int op = (MAXMASK >> j) & 1;
    acc[j] = identity(op);
#pragma unroll
    for (int t = 0; t < PER; ++t)
      if (threadIdx.x + (unsigned)NTHR * t < np) acc[j] = combine(op, acc[j], pv[j][t]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[j] = combine(op, acc[j], __shfl_xor(acc[j], off));
  }
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) sh[j][wave] = acc[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int op = (MAXMASK >> j) & 1;
      red.out[j] = waves_combine<NW>(op, sh[j]);
    }
    for (int k = 0; k <= kTicketShards; ++k)
      __hip_atomic_store(red.ticket + k * kTicketStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

// Hand ns scalars to the host through the mapped, fine-grained (uncached) packet: system-scope
// stores (sc0 sc1, straight to host memory), drained with vmcnt(0) so every packet store is
// acknowledged, then the sequence word the host spins on; no L2 writeback is needed for it.
// All loads are issued before the first store (one latency, not ns). Either its own tiny kernel
// (k_publish) or the publisher workgroup of the next kernel (publisher_first). Done by the last
// block of the preceding reduction instead it measured ~15 us slower (profiles/r1_tuning,
// fused-publish attribution) than a separate launch (~5.5 us).
constexpr int kPublishMax = 32;
__device__ inline void publish_packet(const double* s, int ns, double* host, unsigned* host_seq,
                                      unsigned seq, const double* s2 = nullptr, int off2 = 0,
                                      int n2 = 0, const double* s3 = nullptr, int off3 = 0,
                                      int n3 = 0) {
  double v[kPublishMax];
#pragma unroll
  for (int k = 0; k < kPublishMax; ++k)
    v[k] = (k >= off3 && k < off3 + n3) ? s3[k - off3]
                                        : ((k >= off2 && k < off2 + n2) ? s2[k - off2] : (k < ns ? s[k] : 0.0));
#pragma unroll
  for (int k = 0; k < kPublishMax; ++k)
    if (k < ns) __hip_atomic_store(host + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(host_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pub's deferred reductions, by the publishing workgroup (all its threads call this; the first
// 256 work): each value over its partials strided over 256 threads in slot order, the butterfly,
// the four waves in order — grid_reduce's order for a 256-thread launch, whichever kernel (4 or 8
// waves) publishes. Thread 0 stores the results to dout (and then reads them back itself when it
// copies the packet).
template <int NW>
__device__ inline void defer_reduce(const Pub& pub) {
  static_assert(NW == 4 || NW == 8, "4- or 8-wave workgroups");
  if (pub.dpart[0] == nullptr && pub.dpart[1] == nullptr) return;
  __shared__ double dsh[2][6][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < 256) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      if (pub.dpart[d] == nullptr) continue;
      const int nv = pub.dnv[d];
      double acc[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[j] = identity((pub.dmax[d] >> j) & 1);
      for (int i = threadIdx.x; i < pub.dnp[d]; i += 256)
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (j < nv) acc[j] = combine((pub.dmax[d] >> j) & 1, acc[j], pub.dpart[d][i * nv + j]);
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
          acc[j] = combine((pub.dmax[d] >> j) & 1, acc[j], __shfl_xor(acc[j], off));
      if (lane == 0)
#pragma unroll
        for (int j = 0; j < 6; ++j) dsh[d][j][wave] = acc[j];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int d = 0; d < 2; ++d)
      if (pub.dpart[d] != nullptr)
        for (int j = 0; j < pub.dnv[d]; ++j) pub.dout[d][j] = waves_combine<4>((pub.dmax[d] >> j) & 1, dsh[d][j]);
}

// A launch that carries the scalar packet gets one extra workgroup, the FIRST (blockIdx.x 0;
// the other workgroups index themselves with blockIdx.x - 1), that writes it and then joins the
// grid reduction with identity values (the reduction counts every workgroup). Workgroups are
// dispatched in index order, so the packet leaves at the start of the launch, while the
// kernel's other workgroups work, instead of as a separate k_publish launch in front of it —
// also when only one workgroup fits per CU (a last-index publisher then waited for the first
// workgroups to retire: a 4 us gap before the next kernel). Returns true in the publisher.
// nparts >= 0: the launch reduces over nparts slots (grid_reduce); the publisher takes the last.
template <int NV, unsigned MAXMASK, int NW = 4>
__device__ inline bool publisher_first(const Pub& pub, const Red& red, int nparts = -1) {
  if (pub.host == nullptr || blockIdx.x != 0) return false;
  defer_reduce<NW>(pub);
  if (threadIdx.x == 0)
    publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq, pub.s2, pub.off2, pub.n2,
                   pub.s3, pub.off3, pub.n3);
  double v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = identity((MAXMASK >> j) & 1);
  grid_reduce<NV, MAXMASK, NW>(v, red, (nparts >= 0 ? nparts : (int)gridDim.x) - 1, nparts);
  return true;
}
// partials slot of a non-publisher workgroup of such a launch
__device__ inline int work_slot(const Pub& pub) { return (int)blockIdx.x - (pub.host ? 1 : 0); }

// The row kernels (k_prox_pgd, k_fista_trial: at N > 1 the speculative kernel that carries the
// packet) keep the publisher as their LAST workgroup: they fit many workgroups per CU, so it
// starts at once anyway, and a first-index publisher measured 2-5 % slower end to end on the
// multi-GPU shards (profiles/r1_tuning/small_kernels/publisher_first_rows.log).
template <int NV, unsigned MAXMASK, int NW = 4>
__device__ inline bool publisher_last(const Pub& pub, const Red& red) {
  if (pub.host == nullptr || blockIdx.x != gridDim.x - 1) return false;
  defer_reduce<NW>(pub);
  if (threadIdx.x == 0)
    publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq, pub.s2, pub.off2, pub.n2,
                   pub.s3, pub.off3, pub.n3);
  double v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = identity((MAXMASK >> j) & 1);
  grid_reduce<NV, MAXMASK, NW>(v, red);
  return true;
}

// g = sum_s slabs[s][idx] in slab order (S = 1: a plain load)
template <typename T>
__device__ inline T slab_sum(const T* __restrict__ g, int S, int64_t stride, int64_t idx) {
  T v = g[idx];
  for (int k = 1; k < S; ++k) v = v + g[(int64_t)k * stride + idx];
  return v;
}


template <typename T> __device__ inline T tabs(T v) { return v < T(0) ? -v : v; }

// Device-side control of a ProxGD (mode 0) / FProxGD (mode 1) line-search iteration (struct Ctl,
// solver.cpp dc_run / fista_dc_run): the Armijo test of gl_ProxGD_primal.py:89-92 (FProxGD's
// backtracking test, gl_FProxGD_primal.py:92-97) with t = the trial's step, then — on acceptance — the
// next record's objective and sparsity (:132-133 via the split-candidate/dense residual sums) and
// the stop rule of :118-125. The expressions are the host's (solver.cpp iter_proxgd, stop_rule)
// term for term, so with -ffp-contract=off the decision is the host's bit for bit; the host
// re-derives it from the record and checks it. out = the four residual sums of this finalize.
// pre = tr[0..5], state[0..3], loaded when the kernel starts (they were final before it began),
// so the last block's decision costs no dependent global loads at the end of the kernel
__device__ inline void ctl_decide(const Ctl& c, const double* out, const double (&pre)[10]) {
  double* st = c.state;
  const double* tr = pre;
  double rec[kCtlRec];
  for (int k = 0; k < 4; ++k) rec[k] = out[k];
  for (int k = 0; k < 6; ++k) rec[4 + k] = tr[k];
  bool acc;
  if (c.mode == 1) {   // FProxGD (solver.cpp fista_trials): g(xc) <= g(y) + <g, xc - y> + |xc - y|^2/(2t)
    const double gy = 0.5 * pre[6], gxc = 0.5 * out[0];
    acc = gxc <= gy + tr[0] + tr[1] / (2 * c.t);
  } else {             // ProxGD (iter_proxgd): g(z) <= g(x) - t <g, G_t> + t/2 |G_t|^2
    const double gz = 0.5 * out[0];
    acc = gz <= pre[6] - c.t * tr[0] + 0.5 * c.t * tr[1];
  }
  int code = 2;
  if (acc) {
    double f;
    if (c.mode == 1) {
      f = 0.5 * out[0] + c.mu0 * tr[2];
    } else {
      const double sqx = (c.emode || tr[4] != 0) ? out[0] : out[1];
      f = 0.5 * sqx + c.mu0 * tr[2];
    }
    const double s = out[3] / c.nl;
    const double fl = pre[7], sl = pre[8];
    bool ok = fabs(f - fl) / fabs(fl) < c.ftol;
    if (ok && c.use_sp) ok = fabs(s - sl) / fabs(sl) < c.ftol;
    const double stable = ok ? pre[9] + 1.0 : 0.0;
    st[0] = c.mode == 1 ? out[1] : 0.5 * out[1];
    st[1] = f;
    st[2] = s;
    st[3] = stable;
    code = stable > (double)c.stable_thr ? 1 : 0;
    if (code == 0 && c.nnz_budget >= 0.0 && out[2] > c.nnz_budget) code = 3;
  }
  *c.abort = code == 0 ? 0 : (code == 2 ? -1 : c.pass);
  rec[10] = (double)code;
  for (int k = 0; k <= 10; ++k) c.rec[k] = rec[k];
}

// The all-gathered sums of the row-sharded trial, combined by one workgroup in a fixed order (the
// same bits on every rank): the trial's nranks * nbp workgroup partials strided over 256 threads
// in (rank, workgroup) order, then the butterfly and the four waves in order; the finalize's sums
// rank by rank. Writes tr / rt and, with sp.pub.host, the scalar packet with these values in
// place (read from LDS, not back from memory). Called by every thread of a 256- or 512-thread
// workgroup (k_trial_split's extra workgroup, round 6 also the publisher of the fused dense pass,
// kernels_gemm.hip k_ax_lds DRV): threads past 256 only pass the barrier, so the bits are the
// same whichever kernel combines.
__device__ inline void shard_combine_block(const ShardPub& sp) {
  __shared__ double wv[10][4];
  __shared__ double fin[10];
  __shared__ double pre[kPublishMax];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc[10] = {0.0, 0.0, 0.0, -__builtin_inf(), 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const bool in = threadIdx.x < 256;
  const int np1 = (sp.mask & 1) ? sp.nranks * sp.nbp : 0;
  const int np2 = (sp.mask & 2) ? sp.nranks * sp.nbf : 0;
  const int npm = np1 > np2 ? np1 : np2;
  // Round 6 (this block publishes from the fused dense pass, where the packet's latency is on the
  // host's critical path): every load of a batch — KB trial and finalize partials per thread, and
  // the packet's other scalars — is issued before the first add, one round trip instead of three;
  // the adds keep the per-thread order i = t, t + 256, ... (the same bits as before)
  const bool pubp = sp.pub.host != nullptr && sp.pub.ns <= kPublishMax;
  const double pv = (pubp && (int)threadIdx.x < sp.pub.ns) ? sp.pub.s[threadIdx.x] : 0.0;
  constexpr int KB = 4;
  for (int i0 = (int)threadIdx.x; in && i0 < npm; i0 += 256 * KB) {
    double q1[KB][6], q2[KB][4];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int i = i0 + 256 * k;
      const int r1 = i < np1 ? i / sp.nbp : 0, b1 = i < np1 ? i - r1 * sp.nbp : 0;
      const double* p1 = sp.blk + (int64_t)r1 * sp.chunk + kShardPartOff + b1 * sp.tv;
#pragma unroll
      for (int j = 0; j < 6; ++j) q1[k][j] = (i < np1 && j < sp.tv) ? p1[j] : 0.0;
      const int r2 = i < np2 ? i / sp.nbf : 0, b2 = i < np2 ? i - r2 * sp.nbf : 0;
      const double* p2 = sp.blk + (int64_t)r2 * sp.chunk + kShardPartOff + sp.tv * sp.nbp + b2 * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) q2[k][j] = i < np2 ? p2[j] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int i = i0 + 256 * k;
      if (i < np1)
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (j < sp.tv) acc[j] = combine(j == 3 ? OP_MAX : OP_SUM, acc[j], q1[k][j]);
      if (i < np2)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[6 + j] += q2[k][j];
    }
  }
  if (pubp && (int)threadIdx.x < sp.pub.ns) pre[threadIdx.x] = pv;
#pragma unroll
  for (int j = 0; j < 10; ++j)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
      acc[j] = combine(j == 3 ? OP_MAX : OP_SUM, acc[j], __shfl_xor(acc[j], off));
  if (lane == 0 && in)
#pragma unroll
    for (int j = 0; j < 10; ++j) wv[j][wave] = acc[j];
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int j = 0; j < 10; ++j) fin[j] = waves_combine<4>(j == 3 ? OP_MAX : OP_SUM, wv[j]);
  if (sp.mask & 1)
    for (int j = 0; j < sp.tv; ++j) sp.tr[j] = fin[j];
  if (sp.mask & 2)
    for (int j = 0; j < 4; ++j) sp.rt[j] = fin[6 + j];
  if (sp.pub.host != nullptr)
    publish_packet(pubp ? pre : sp.pub.s, sp.pub.ns, sp.pub.host, sp.pub.host_seq, sp.pub.seq, fin,
                   sp.tr_off, (sp.mask & 1) ? sp.tv : 0, fin + 6, sp.rt_off, (sp.mask & 2) ? 4 : 0);
}

// ------------------------------------------------------------------------------------------
// Split-candidate column bitmaps (round 5). Behind the n per-row column masks zf[k] of e (bit c =
// e[k][c] != 0) the trial kernels also write, per column c, a bitmap of the rows whose mask has
// bit c: u16 word g of column c = rows 16 g .. 16 g + 15 (bit j = row 16 g + j), at
// zf_bitmaps(zf, n)[c * zf_npad(n) / 16 + g]; read as u64, word w of column c covers the 64 rows
// of panel w. The A e gather builds its ascending per-column row lists from them in LDS
// (kernels_gather.hip k_at_gather_bm) instead of a k_e_lists launch over all n masks. A trial
// rewrites the words of the row groups it visits: the 16-row groups below ceil16(n) (row kernels)
// or the 64 / 32-row panels (A^T R epilogues). Words it never visits — the groups in
// [ceil16(n), ceil64(n)), the upper half of the last u64 of a 32-row panel — keep what the session
// cleared at creation (Session's constructor zeroes the whole zf region), and the gather also
// masks the bits of rows >= n of the last word itself (stale bits there made it
// read At and E beyond n).
// ------------------------------------------------------------------------------------------
__host__ __device__ inline int64_t zf_npad(int64_t n) { return (n + 63) / 64 * 64; }
__device__ inline unsigned short* zf_bitmaps(unsigned* zf, int64_t n) {
  return reinterpret_cast<unsigned short*>(zf + zf_npad(n));
}
// A PW-row panel [col0, col0 + PW) of masks (PW = 64, or 32 for the narrow A^T R panel), held
// one per row in the LDS array msk (all of the workgroup's waves wrote theirs and passed a
// barrier): wave 0 transposes it with one ballot per column and lane c < l stores column c's
// u64 (u32) word. Called by the whole workgroup.
template <int PW = 64>
__device__ inline void zf_store_panel(const unsigned* msk, unsigned* zf, int64_t n, int l,
                                      int64_t col0) {
  static_assert(PW == 64 || PW == 32, "64- or 32-row panels");
  if ((threadIdx.x >> 6) != 0) return;
  const int lane = threadIdx.x & 63;
  const unsigned v = lane < PW ? msk[lane] : 0u;
  uint64_t mine = 0;
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    const uint64_t b = __ballot((v >> c) & 1u);
    if (lane == c) mine = b;
  }
  if (lane < l) {
    unsigned short* col = zf_bitmaps(zf, n) + (int64_t)lane * (zf_npad(n) / 16);
    if constexpr (PW == 64) reinterpret_cast<uint64_t*>(col)[col0 / 64] = mine;
    else reinterpret_cast<unsigned*>(col)[col0 / 32] = (unsigned)mine;
  }
}
// The row kernels' form (16 lanes per row, so a 256-thread workgroup holds the 16 rows of one
// 16-row group per trip): the lane sub == 0 of each row puts its mask in msk[16], a barrier, then
// thread c < l stores column c's u16 word of the group starting at row0; a second barrier frees
// msk for the next trip. Called by the whole workgroup (the trip count is uniform).
__device__ inline void zf_store_group16(unsigned* msk, unsigned rowe, bool rv, int sub, unsigned* zf,
                                        int64_t n, int l, int64_t row0) {
  if (sub == 0) msk[threadIdx.x >> 4] = rv ? rowe : 0u;
  __syncthreads();
  if ((int)threadIdx.x < l && row0 < zf_npad(n)) {
    unsigned b = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) b |= ((msk[j] >> threadIdx.x) & 1u) << j;
    zf_bitmaps(zf, n)[(int64_t)threadIdx.x * (zf_npad(n) / 16) + row0 / 16] = (unsigned short)b;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// row helpers
// ------------------------------------------------------------------------------------------
template <int LPR>
__device__ inline double row_allsum(double v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
template <int LPR>
__device__ inline unsigned row_or(unsigned v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v |= __shfl_xor(v, off);
  return v;
}
template <int LPR>
__device__ inline float row_allsum(float v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}


// ------------------------------------------------------------------------------------------
// ProxGD trial arithmetic for one row (gl_ProxGD_primal.py:65-74, 89-92), for a lane that
// holds EPL elements of the row (columns sub + e*LPR; ok[e] = column exists): w = x - t g,
// p = w * max(||w|| - t mu, 0) / ((||w|| < thres) + ||w||), G_t = (x - p)/t, z = x - t G_t,
// p_thr = p with |p| < thres zeroed. acc (per thread, reduced over the grid by the caller):
// [sum g*G_t, sum G_t^2, sum_i ||p_i||, max |p|, #{p changed by the threshold},
//  #{rows of p changed by the threshold}]. rv = the row exists (all LPR lanes call this).
//
// emode (the split-candidate form of the fast objective mode, see solver.cpp iter_proxgd):
// instead of z the third output is e = p - p_thr, i.e. p where the threshold zeroed it and 0
// elsewhere (exact: p_thr is either p or 0, and NaN is never "small"), so A p = A p_thr + A e
// with e nonzero only in the rows the threshold touched. Returns the row's column mask of e
// (bit j = e[j] != 0, columns j < 32; every lane of the row gets the same mask), which the
// split-candidate gather's column lists are built from (kernels_gather.hip k_e_lists).
// ------------------------------------------------------------------------------------------
template <typename T, int LPR, int EPL>
__device__ inline unsigned prox_pgd_row(const T (&xv)[EPL], const T (&gv)[EPL], const bool (&ok)[EPL],
                                    bool rv, int sub, T t, T tmu, T thres, T (&pv)[EPL],
                                    T (&pth)[EPL], T (&zv)[EPL], double (&acc)[6],
                                    bool emode = false) {
  T w[EPL];
  T sq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    w[e] = xv[e] - t * gv[e];
    sq = sq + w[e] * w[e];
  }
  const T nrm = __builtin_sqrt(row_allsum<LPR>(sq));
  T c = nrm - tmu;
  c = (c < T(0)) ? T(0) : c;                        // np.clip(., 0, None): NaN stays NaN
  const T d = ((nrm < thres) ? T(1) : T(0)) + nrm;
  T psq = T(0);
  bool rch = false;
  unsigned mk = 0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    pv[e] = (w[e] * c) / d;
    const T G = (xv[e] - pv[e]) / t;
    const bool small = tabs(pv[e]) < thres;
    pth[e] = small ? T(0) : pv[e];
    zv[e] = emode ? (small ? pv[e] : T(0)) : xv[e] - t * G;
    if (ok[e]) {
      acc[0] += (double)(gv[e] * G);
      acc[1] += (double)(G * G);
      acc[3] = nan_max(acc[3], (double)tabs(pv[e]));
      const bool ch = small && pv[e] != T(0);
      acc[4] += ch ? 1.0 : 0.0;
      rch = rch || ch;
      if (ch && sub + e * LPR < 32) mk |= 1u << (sub + e * LPR);
      psq = psq + pv[e] * pv[e];
    }
  }
  const T pn = __builtin_sqrt(row_allsum<LPR>(psq));
  const double rowch = row_allsum<LPR>(rch ? 1.0 : 0.0);
  if (rv && sub == 0) {
    acc[2] += (double)pn;
    acc[5] += rowch > 0.0 ? 1.0 : 0.0;
  }
  return emode ? row_or<LPR>(mk) : 0u;
}

// ------------------------------------------------------------------------------------------
// FISTA / FGD trial arithmetic for one row (gl_FProxGD_primal.py:92-102, :136-145): with
// w = y - t g, xc = prox(w, t) (PROX) or w (FGD), xk_thr = xk with |xk| < thres zeroed,
// v_next = xk_thr + (xc - xk_thr)/theta, y_next = a1 thr(xc) + b1 v_next.
// acc: PROX [sum g*(xc-y), sum (xc-y)^2, sum ||xc_i||, max |xc|];
//      FGD  [sum g*(xc-y), sum (xc-y)^2, sum (sqrt(||xc_i||^2+d^2)-d), sum ||xc_i||, max |xc|].
// ------------------------------------------------------------------------------------------
// ecv (split form, when non-null): e_c = xc - thr(xc), i.e. xc where the threshold zeroes it and
// 0 elsewhere; returns the row's column mask of e_c (as prox_pgd_row; 0 without ecv).
template <typename T, int LPR, int EPL, bool PROX>
__device__ inline unsigned fista_row(const T (&yv)[EPL], const T (&gv)[EPL], const T (&xkv)[EPL],
                                 const bool (&ok)[EPL], bool rv, int sub, T t, T tmu, T thres,
                                 T theta, T a1, T b1, T dd, T delta, T (&xcv)[EPL],
                                 T (&vnv)[EPL], T (&ynv)[EPL], double (&acc)[PROX ? 4 : 5],
                                 T* ecv = nullptr) {
  constexpr int NV = PROX ? 4 : 5;
  T w[EPL];
  T sq = T(0);
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    w[e] = yv[e] - t * gv[e];
    sq = sq + w[e] * w[e];
  }
  T c = T(1), d = T(1);
  if (PROX) {
    const T nrm = __builtin_sqrt(row_allsum<LPR>(sq));
    c = nrm - tmu;
    c = (c < T(0)) ? T(0) : c;
    d = ((nrm < thres) ? T(1) : T(0)) + nrm;
  }
  T psq = T(0);
  unsigned mk = 0;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const T pv = PROX ? (w[e] * c) / d : w[e];
    const T dl = pv - yv[e];
    T xo = xkv[e];
    if (tabs(xo) < thres) xo = T(0);
    const T vn = xo + (pv - xo) / theta;
    const bool small = tabs(pv) < thres;
    const T pt = small ? T(0) : pv;
    xcv[e] = pv;
    vnv[e] = vn;
    ynv[e] = a1 * pt + b1 * vn;
    if (ecv != nullptr) {
      ecv[e] = small ? pv : T(0);
      if (ok[e] && small && pv != T(0) && sub + e * LPR < 32) mk |= 1u << (sub + e * LPR);
    }
    if (ok[e]) {
      acc[0] += (double)(gv[e] * dl);
      acc[1] += (double)(dl * dl);
      acc[NV - 1] = nan_max(acc[NV - 1], (double)tabs(pv));
      psq = psq + pv * pv;
    }
  }
  const T ps = row_allsum<LPR>(psq);
  if (rv && sub == 0) {
    if (PROX) {
      acc[2] += (double)__builtin_sqrt(ps);
    } else {
      acc[2] += (double)(__builtin_sqrt(ps + dd) - delta);
      acc[3] += (double)__builtin_sqrt(ps);
    }
  }
  return ecv != nullptr ? row_or<LPR>(mk) : 0u;
}

}  // namespace glx
#endif  // GLX_DEVICE_H_
