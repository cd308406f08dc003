// kernels_rg2.hip — the trial's batch AND the next gradient in ONE pass over A (SURVEY §8f row 1 at
// l = 16; reference gl_ProxGD_primal.py:89-92 + :112 `A @ z`, `A @ p_thr` and :129
// `A.T @ (A @ x - b)` at the candidate):
//
//   S0 = A z,  S1 = A p_thr        (the line-search trial's two right-hand sides, m x 16 each)
//   r  = S1 - b                    (the next gradient residual, if the trial is accepted)
//   G  = A^T r                     (the next gradient, n x 16)
//
// Round 4. The l = 32 kernel (kernels_fused.hip) puts the residual exchange on the MFMA waves'
// critical path; DESIGN.md's probe-backed ceiling at C2 (4096, 8192, 16) says a one-pass form
// wins there only with the exchange taken off them. Here the workgroup's eight waves split by role:
//
//   * 256 workgroups (one per CU, 512 threads), RG row groups x P column panels of 256 columns
//     (n = 8192: P = 32, RG = 8). A-waves 0..3 and B-waves 4..7; wave w and w + 4 own the same 64
//     columns (and share a SIMD: the dispatcher puts a workgroup's waves on SIMDs cyclically).
//   * A-wave (phase A): for every 16-row block b of its row group, its 16 x 64 tile of A (16-B
//     loads, prefetched one block ahead) times the matching 64 x 32 slice of X = [z | p_thr] (in
//     LDS for the whole launch) on v_mfma_f64_16x16x4f64 -> a 16 x 32 partial, written to an LDS
//     ring slot; then it moves on. It never waits for another workgroup.
//   * B-wave (exchange + phase B), pipelined over blocks (iteration j):
//       1. block j: the four A-wave partials summed in a fixed order (each B-wave a quarter), the
//          workgroup's partial handed out as tagged 8-byte granules;
//       2. block j - 1, hop 1 (reduce-scatter): this workgroup owns 512 / P of the block's 512
//          values: sums the P panels' partials in a fixed butterfly order, writes S0 / S1 for
//          the finalize, and hands out r = S1 - b (the same subtraction the finalize does);
//       3. block j - 2, hop 2 (all-gather): r of the block into LDS, then phase B:
//          G[its 64 columns] += tile^T r, the tile re-read from L2 / the Infinity Cache.
//     The G accumulators stay in registers; at the end each B-wave writes its rows of slab rg.
//   * LDS flags between the roles (monotone counters, polled with s_sleep); every wait is bounded:
//     on a timeout the wave sets *err and carries on (results invalid; the host recomputes with
//     two passes). Granule tags are epoch-based, so nothing is reset between launches.
//
// Outputs: P0 = S0, P1 = S1 (one slab each, the A@X slab layout the finalize reads) and
// Gs[rg][n][16] (the consumer sums the RG slabs in slab order). Deterministic: every sum has a
// fixed order independent of timing.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "glx.h"
#include "glx_device.h"
#include "glx_mfma.h"

namespace glx {

namespace {
typedef unsigned long long u64;
constexpr int kRW = 8;                  // waves per workgroup: 4 A-waves + 4 B-waves
constexpr int kRThreads = 64 * kRW;
constexpr int kRCols = 64;              // columns per wave
constexpr int kRPanel = 4 * kRCols;     // 256 columns per workgroup
constexpr int kRLA = 32;                // phase-A columns: z | p_thr
constexpr int kRLB = 16;                // phase-B columns (l)
constexpr int kRBlk = 16 * kRLA;        // 512 values of a block's partial
constexpr int kRSlot = 3;               // LDS partial ring (A-waves may run 3 blocks ahead)
#ifndef GLX_RG2_AB
#define GLX_RG2_AB 4
#endif
constexpr int kRAB = GLX_RG2_AB;        // A-wave tile buffers (kRAB - 1 blocks of A in flight)
// B-wave lags (template D1, D2): iteration j publishes block j's partial, runs hop 1 of block
// j - D1 and hop 2 + phase B of block j - D2. Granule rings per row group (memory): a workgroup Y
// publishes block j only after its hop 2 of j - 1 - D2, which needed r of that block, which needed
// every panel's partial of it; a workgroup W that far behind is still to read block
// j - 1 - D2 - D1 at most, so D1 + D2 + 2 slots keep them apart. r of block k is published after
// W's partial of k (W's iteration k), when W is still to read r of k - D2: D2 + 1 slots.
__host__ __device__ constexpr int pg_ring(int d1, int d2) { return d1 + d2 + 2; }
__host__ __device__ constexpr int rg_ring(int d2) { return d2 + 1; }
constexpr int kRMaxPg = pg_ring(3, 6), kRMaxRg = rg_ring(6);
constexpr int kRGrid = 256;

// XL (XCD-local hand-off, as kernels_fused.hip's put_value): every reader of a row group's
// granules runs on the writer's XCD, so a plain store (the vector L1 is write-through: the line
// lands in that XCD's L2) is enough for the readers' sc1 loads; otherwise sc1 (write-through)
// stores, visible on every XCD.
template <bool XL>
__device__ inline void put_gran(u64* g, unsigned tag, double v) {
  const u64 u = (u64)__double_as_longlong(v);
  constexpr int scope = XL ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT;
  __hip_atomic_store(g, ((u64)tag << 32) | (u & 0xffffffffull), __ATOMIC_RELAXED, scope);
  __hip_atomic_store(g + 1, ((u64)tag << 32) | (u >> 32), __ATOMIC_RELAXED, scope);
}
struct Gr { u64 w0, w1; };
__device__ inline Gr get_gran(const u64* g) {
  return Gr{__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
            __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
}
__device__ inline bool gr_ok(const Gr& x, unsigned tag) {
  return (unsigned)(x.w0 >> 32) == tag && (unsigned)(x.w1 >> 32) == tag;
}
__device__ inline double gr_val(const Gr& x) {
  return __longlong_as_double((long long)((x.w1 << 32) | (x.w0 & 0xffffffffull)));
}
// LDS counters shared by the roles. Every counter guards LDS data only (the partial ring, r of
// a block), and one wave's LDS operations execute in issue order, so relaxed atomics with
// compiler-only fences suffice: acquire / release at workgroup scope also made the compiler
// drain vmcnt (s_waitcnt vmcnt(0)) at every counter access, i.e. wait for the A-waves' tile
// prefetch and the B-waves' granule and tile loads each block (round 4: 146-158 us at C2
// whatever the lags or the prefetch depth).
__device__ inline unsigned lds_get(const unsigned* p) {
  const unsigned v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);   // later LDS reads stay behind the counter read
  return v;
}
// one add per wave (lane 0), behind the wave's earlier LDS accesses (issue order)
__device__ inline void lds_add(unsigned* p) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
}  // namespace

template <int D1, int D2, bool XL>
__global__ __launch_bounds__(kRThreads, 1) void k_resgrad2(
    const double* __restrict__ A, const double* __restrict__ X0, const double* __restrict__ X1,
    const double* __restrict__ B, double* __restrict__ P0, double* __restrict__ P1,
    double* __restrict__ Gs, u64* Pg, u64* Rg, unsigned* xslot, unsigned epoch0, int64_t m,
    int64_t n, int RG, int NB, int* err, unsigned spin_max) {
  __shared__ __attribute__((aligned(16))) double xs[4][kRCols * kRLA];          // 64 KiB
  __shared__ __attribute__((aligned(16))) double part[kRSlot][4][kRBlk];        // 48 KiB
  __shared__ __attribute__((aligned(16))) double rsh[2][16 * kRLB];             // 4 KiB
  __shared__ unsigned cnt_part[kRSlot], cnt_free[kRSlot], cnt_r[2], cnt_rfree[2];
  __shared__ int bad;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int P = (int)(n / kRPanel);
  // XL: the row group is this workgroup's XCD (HW_REG_XCC_ID; RG = 8) and the panel its arrival
  // order there (xslot, zeroed before the launch); a workgroup beyond P on one XCD flags err = 2
  // and leaves, the others of its XCD then time out (bad: every later wait returns at once) and
  // the host recomputes with two passes.
  __shared__ int xl_id[2];
  if (XL) {
    if (tid == 0) {
      const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);   // HW_REG_XCC_ID[3:0]
      xl_id[0] = xcc;
      xl_id[1] = (int)__hip_atomic_fetch_add(xslot + xcc * 32, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  const int rg = XL ? xl_id[0] : (int)blockIdx.x % RG;
  const int pnl = XL ? xl_id[1] : (int)blockIdx.x / RG;
  if (XL && (pnl >= P || rg >= RG)) {
    if (tid == 0) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int64_t rbase = (int64_t)rg * (m / RG);
  const int wc = wave & 3;                                   // column slot of the wave
  const int64_t col0 = (int64_t)pnl * kRPanel + (int64_t)wc * kRCols;
  auto tag_of = [&](int b) { return epoch0 + (unsigned)b + 1u; };

  if (tid < kRSlot) { cnt_part[tid] = 0; cnt_free[tid] = 0; }
  if (tid < 2) { cnt_r[tid] = 0; cnt_rfree[tid] = 0; }
  if (tid == 0) bad = 0;
  // X slice of the workgroup (256 rows of [z | p_thr]) in LDS: row k of column slot s at
  // xs[s][k * 32 + (c ^ (((k >> 2) & 1) << 4))] (the halves swap with bit 2 of k: the B-operand
  // reads of lane groups q and q + 1 land on different banks, as in kernels_fused.hip)
  for (int idx = tid; idx < kRPanel * kRLA; idx += kRThreads) {
    const int kk = idx / kRLA, c = idx % kRLA;
    const int s = kk / kRCols, k = kk % kRCols;
    const int64_t row = (int64_t)pnl * kRPanel + kk;
    const double v = c < 16 ? X0[row * 16 + c] : X1[row * 16 + (c - 16)];
    xs[s][k * kRLA + (c ^ (((k >> 2) & 1) << 4))] = v;
  }
  __syncthreads();

  // a timed-out wait flags the launch (any lane that saw it) and carries on
  auto fail = [&] {
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bad = 1;
  };
  auto spin_wait = [&](const unsigned* ctr, unsigned want) {
    unsigned spins = 0;
    while (!__all(lds_get(ctr) >= want)) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin_max || bad) {
        fail();
        return;
      }
    }
  };

  if (wave < 4) {
    // ------------------------------------------------------------------ A-wave: phase A
    const double* xw = &xs[wc][0];
    // AB tile buffers, AB - 1 blocks in flight (round 4: with one block ahead the A-waves waited
    // a whole HBM latency per block); [chunk][e], row rbase + 16 b + i, cols col0 + 16 ch + 4 q + e
    double a[kRAB][4][4];
    auto load_tile = [&](double (&t)[4][4], int b) {
      b = b < NB ? b : NB - 1;
      const double* ap = A + (rbase + 16 * (int64_t)b + i) * n + col0 + 4 * q;
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const d2_t v0 = *reinterpret_cast<const d2_t*>(ap + 16 * ch);
        const d2_t v1 = *reinterpret_cast<const d2_t*>(ap + 16 * ch + 2);
        t[ch][0] = v0[0]; t[ch][1] = v0[1]; t[ch][2] = v1[0]; t[ch][3] = v1[1];
      }
    };
    auto phase_a = [&](const double (&t)[4][4], int b) {
      d4_t c0[2] = {d4_t{0.0, 0.0, 0.0, 0.0}, d4_t{0.0, 0.0, 0.0, 0.0}};
      d4_t c1[2] = {d4_t{0.0, 0.0, 0.0, 0.0}, d4_t{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
      for (int ch = 0; ch < 4; ch += 2)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 16 * ch + 4 * q + e;   // (k >> 2) & 1 == q & 1
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const int cx = 16 * (nt ^ (q & 1)) + i;
            c0[nt] = MF<double>::mma(t[ch][e], xw[k * kRLA + cx], c0[nt]);
            c1[nt] = MF<double>::mma(t[ch + 1][e], xw[(k + 16) * kRLA + cx], c1[nt]);
          }
        }
      const int s = b % kRSlot;
      // the slot's previous block was summed by all four B-waves
      if (b >= kRSlot) spin_wait(&cnt_free[s], 4u * (unsigned)(b / kRSlot));
      double* dst = &part[s][wc][0];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const d4_t v = c0[nt] + c1[nt];
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(q + 4 * r) * kRLA + 16 * nt + i] = v[r];
      }
      lds_add(&cnt_part[s]);
    };
    // in block order (the scheduler would otherwise issue block 0's loads last, and the loop
    // head's wait would cover all of them on every trip)
#pragma unroll
    for (int d = 0; d < kRAB - 1; ++d) {
      load_tile(a[d], d);
      __builtin_amdgcn_sched_barrier(0);
    }
    // NB % kRAB == 0 (resgrad2_shape_ok): no early exit inside the trip, so the compiler's
    // waitcnt state at the loop head keeps kRAB - 1 tiles in flight (an exit edge made it drain
    // vmcnt to 0 at the top of every trip)
    for (int b = 0; b < NB; b += kRAB) {
#pragma unroll
      for (int h = 0; h < kRAB; ++h) {
        load_tile(a[(h + kRAB - 1) % kRAB], b + h + kRAB - 1);
        phase_a(a[h], b + h);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped re-loads, before exit
    return;
  }

  // -------------------------------------------------------------------- B-wave
  const int bw = wave - 4;          // 0..3
  const int bl = bw * 64 + lane;    // 0..255 within the B-waves
  d4_t gacc[4];                     // G rows col0 + 16 ct + q + 4 r, column i
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) gacc[ct] = d4_t{0.0, 0.0, 0.0, 0.0};

  // hop 1: the 512 (value, panel) pairs of this workgroup's slice, two per B-lane: value
  // v1 = pnl * (512 / P) + bl * 2 / P, panels k0 = (2 bl) % P, k0 + 1; the P / 2 lanes of a value
  // are consecutive (P <= 128: within one wave)
  constexpr int kPg = pg_ring(D1, D2), kRg = rg_ring(D2);
  const int pl = 2 * bl;
  const int vloc = pl / P, k0 = pl % P;
  const int v1 = pnl * (kRBlk / P) + vloc;
  const int vrow = v1 / kRLA, vcol = v1 % kRLA;
  auto pg_at = [&](int b, int panel, int v) {
    return Pg + ((((int64_t)rg * kPg + (b % kPg)) * P + panel) * kRBlk + v) * 2;
  };
  auto rg_at = [&](int b, int v) {   // r granules: 16 rows x 16 columns (the p_thr half)
    return Rg + (((int64_t)rg * kRg + (b % kRg)) * (16 * kRLB) + v) * 2;
  };
  auto sweep = [&](const u64* g, unsigned tag, Gr x) -> double {
    unsigned spins = 0;
    while (!__all(gr_ok(x, tag))) {
      __builtin_amdgcn_s_sleep(1);
      if (!gr_ok(x, tag)) x = get_gran(g);
      if (++spins > spin_max || bad) {
        if (!gr_ok(x, tag)) fail();
        break;
      }
    }
    return gr_val(x);
  };
  // phase B tile of block b: lane (i, q) holds A[row 4 s + q][col0 + 16 ct + i]; two tiles,
  // loaded two blocks ahead (their latency overlaps two iterations of hop waits)
  double at[2][4][4];
  auto load_at = [&](double (&t)[4][4], int b) {
    b = b < NB ? b : NB - 1;
    const double* ap = A + (rbase + 16 * (int64_t)b + q) * n + col0 + i;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) t[s][ct] = ap[(int64_t)4 * s * n + 16 * ct];
  };

  load_at(at[0], 0);
  load_at(at[1], 1);
  // The remote reads of iteration j (hop-1 granules of block j - D1, b, the r granule of block
  // j - D2) are issued at the end of iteration j - 1, BEFORE that iteration's phase-B tile
  // prefetch: loads retire in order, so waiting for them then leaves the tile loads in flight.
  struct Pre {
    Gr h1[2];
    double bv;
    Gr h2;
  };
  auto issue = [&](int j, Pre& p) {
    const int b1 = j - D1, b2 = j - D2;
    if (b1 >= 0 && b1 < NB) {
      p.h1[0] = get_gran(pg_at(b1, k0, v1));
      p.h1[1] = get_gran(pg_at(b1, k0 + 1, v1));
      p.bv = (k0 == 0 && vcol >= 16) ? B[(rbase + 16 * b1 + vrow) * kRLB + (vcol - 16)] : 0.0;
    }
    if (b2 >= 0 && b2 < NB) p.h2 = get_gran(rg_at(b2, bl));
  };
  // one B iteration; tb = the tile buffer of block j - D2 (constant after inlining: the loop
  // below runs two iterations per trip); cur: this iteration's remote reads, nxt: the next one's
  auto iter = [&](int j, double (&tb)[4][4], Pre& cur, Pre& nxt) {
    const int b1 = j - D1, b2 = j - D2;
    const bool do1 = b1 >= 0 && b1 < NB, do2 = b2 >= 0 && b2 < NB;
    // 1. block j: the four A-wave partials (fixed order), handed out as granules
    if (j < NB) {
      const int s = j % kRSlot;
      spin_wait(&cnt_part[s], 4u * (unsigned)(j / kRSlot + 1));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int v = bl + 256 * h;
        const double sv = ((part[s][0][v] + part[s][1][v]) + part[s][2][v]) + part[s][3][v];
        put_gran<XL>(pg_at(j, pnl, v), tag_of(j), sv);
      }
      lds_add(&cnt_free[s]);
    }
    // 2. block b1, hop 1: slice sums in a fixed butterfly order; S to the output slabs, r out
    if (do1) {
      double sum = sweep(pg_at(b1, k0, v1), tag_of(b1), cur.h1[0]) +
                   sweep(pg_at(b1, k0 + 1, v1), tag_of(b1), cur.h1[1]);
      for (int off = 1; off < P / 2; off <<= 1) sum = sum + __shfl_xor(sum, off);
      if (k0 == 0) {
        const int64_t row = rbase + 16 * b1 + vrow;
        if (vcol < 16) {
          P0[row * kRLB + vcol] = sum;
        } else {
          P1[row * kRLB + (vcol - 16)] = sum;
          put_gran<XL>(rg_at(b1, vrow * kRLB + (vcol - 16)), tag_of(b1), sum - cur.bv);
        }
      }
    }
    // 3. block b2, hop 2 + phase B
    if (do2) {
      const int rs = b2 & 1;
      if (b2 >= 2) spin_wait(&cnt_rfree[rs], 4u * (unsigned)(b2 / 2));
      rsh[rs][bl] = sweep(rg_at(b2, bl), tag_of(b2), cur.h2);
      lds_add(&cnt_r[rs]);
      spin_wait(&cnt_r[rs], 4u * (unsigned)(b2 / 2 + 1));
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double rr = rsh[rs][(4 * s + q) * kRLB + i];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) gacc[ct] = MF<double>::mma(tb[s][ct], rr, gacc[ct]);
      }
      lds_add(&cnt_rfree[rs]);
    }
    issue(j + 1, nxt);
    __builtin_amdgcn_sched_barrier(0);   // (the scheduler would hoist the tile loads above them)
    if (do2 && b2 + 2 < NB) load_at(tb, b2 + 2);
  };
  constexpr int p0 = D2 & 1;   // tile buffer of block j - D2 for even j
  Pre pa, pb;
  issue(0, pa);
  for (int j = 0; j < NB + D2; j += 2) {
    iter(j, at[p0], pa, pb);
    if (j + 1 < NB + D2) iter(j + 1, at[p0 ^ 1], pb, pa);
  }
  double* gout = Gs + (int64_t)rg * n * kRLB;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double v = bad ? __builtin_nan("") : gacc[ct][r];
      gout[(col0 + 16 * ct + q + 4 * r) * kRLB + i] = v;
    }
}

// ---------------------------------------------------------------------------------------------
// shape / device checks and launch
// ---------------------------------------------------------------------------------------------
struct Rg2Layout {
  size_t pg, rg, xs, total;
};
static Rg2Layout rg2_layout(int64_t n) {
  const int64_t P = n / kRPanel, RG = kRGrid / P;
  auto up = [](size_t v) { return (v + 255) & ~size_t(255); };
  Rg2Layout L;
  L.pg = 0;
  L.rg = up(sizeof(u64) * 2 * (size_t)RG * kRMaxPg * P * kRBlk);
  L.xs = L.rg + up(sizeof(u64) * 2 * (size_t)RG * kRMaxRg * 16 * kRLB);
  L.total = L.xs + 8 * 32 * sizeof(unsigned) + 256;
  return L;
}

bool resgrad2_shape_ok(int esize, int64_t m, int64_t n, int64_t l) {
  if (esize != 8 || l != kRLB || n % kRPanel != 0) return false;
  const int64_t P = n / kRPanel;
  if (P < 2 || P > 128 || (P & (P - 1)) != 0) return false;
  const int64_t RG = kRGrid / P;
  return m % (RG * 16 * kRAB) == 0 && m / RG >= 32;   // NB = m / RG / 16, a multiple of kRAB
}

int resgrad2_groups(int64_t n) { return (int)(kRGrid / (n / kRPanel)); }

bool resgrad2_device_ok() {
  // per device (one process-wide answer was taken from whichever device was
  // current at the first call)
  static int ok[64];
  static bool init = false;
  if (!init) {
    for (int& v : ok) v = -1;
    init = true;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (ok[dev] < 0) {
    int cus = 0, occ = 0;
    ok[dev] = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(k_resgrad2<2, 4, true>),
                                                     kRThreads, 0) == hipSuccess)
      ok[dev] = (cus >= kRGrid && occ >= 1) ? 1 : 0;
  }
  return ok[dev] == 1;
}

size_t resgrad2_ws_bytes(int64_t n) { return rg2_layout(n).total; }

void resgrad2_reset(void* ws, int64_t n, hipStream_t st) {
  (void)hipMemsetAsync(ws, 0, rg2_layout(n).total - 256, st);
}

// launch_count >= 1 grows by one per launch on the same workspace (granule tags never repeat)
void launch_resgrad2(const double* A, const double* X0, const double* X1, const double* B,
                     double* P0, double* P1, double* Gs, void* ws, unsigned launch_count, int64_t m,
                     int64_t n, int* err, hipStream_t st) {
  const int64_t P = n / kRPanel, RG = kRGrid / P, NB = m / RG / 16;
  const Rg2Layout L = rg2_layout(n);
  char* w = static_cast<char*>(ws);
  u64* pg = reinterpret_cast<u64*>(w + L.pg);
  u64* rgp = reinterpret_cast<u64*>(w + L.rg);
  unsigned* xs = reinterpret_cast<unsigned*>(w + L.xs);
  const unsigned ep = (unsigned)((launch_count - 1) * (unsigned)(NB + 8));
  static const unsigned spin_max = [] {
    const char* v = std::getenv("GLX_RG_SPIN");
    const int lg = v && *v ? std::atoi(v) : 22;
    return lg <= 0 ? 0u : (1u << (lg > 30 ? 30 : lg));
  }();
  // B-wave lags D1 D2 (GLX_RG2_LAG = two digits; default 24)
  static const int lag = [] {
    const char* v = std::getenv("GLX_RG2_LAG");
    const int x = v && *v ? std::atoi(v) : 24;
    return (x == 12 || x == 23 || x == 24 || x == 36) ? x : 24;
  }();
  // XCD-local hand-off where the row groups are the 8 XCDs (GLX_RG_XCD=0: the agent-scope form)
  static const bool xcd = [] {
    const char* v = std::getenv("GLX_RG_XCD");
    return !(v && v[0] == '0');
  }();
  const bool xl = xcd && RG == 8;
  auto go = [&](auto kern) {
    glx_launch(kern, dim3((unsigned)(RG * P)), dim3(kRThreads), 0, st, A, X0, X1, B, P0, P1, Gs, pg, rgp,
               xs, ep, m, n, (int)RG, (int)NB, err, spin_max);
  };
  auto lags = [&](auto k12, auto k23, auto k24, auto k36) {
    switch (lag) {
      case 12: go(k12); break;
      case 23: go(k23); break;
      case 36: go(k36); break;
      default: go(k24); break;
    }
  };
  if (xl)
    lags(k_resgrad2<1, 2, true>, k_resgrad2<2, 3, true>, k_resgrad2<2, 4, true>, k_resgrad2<3, 6, true>);
  else
    lags(k_resgrad2<1, 2, false>, k_resgrad2<2, 3, false>, k_resgrad2<2, 4, false>, k_resgrad2<3, 6, false>);
}

}  // namespace glx
