// kernels_fused.hip — the residual AND the gradient of one right-hand side in ONE pass over A
// (reference gl_ProxGD_primal.py:129 `A.T @ (A @ x - b)`):
//
//   S = A X            (X = the thresholded candidate p_thr, n x 32, fp64)
//   r = S - b          (the next gradient residual)
//   G = A^T r          (the next gradient)
//
// Two launches read A twice (A@X, then A^T r). Here every 16-row block of A is read from HBM once
// and used for both products while it is in registers / LDS:
//
//   * 256 workgroups (one per CU, 8 waves = two per SIMD), arranged as RG row groups x P column
//     panels (n = 16384: 8 x 32, a panel = 512 columns, a wave = 64 of them).
//     Workgroup (rg, p) walks the 16-row blocks of row group rg over its panel.
//   * phase A: a wave multiplies its 16 x 64 tile of A by the matching 64 x 32 slice of X
//     (LDS-resident for the whole launch) on v_mfma_f64_16x16x4f64; the eight waves' partial
//     residual rows are summed through LDS in a fixed order into the workgroup's 16 x 32 partial.
//   * the P partials of a block are exchanged through memory in two hops (reduce-scatter, then
//     all-gather, see hop1 / hop2): sc1 (write-through) stores, every wave's vmcnt drain, a
//     workgroup barrier, one agent-scope counter add per workgroup; a consumer polls the counter
//     with sc1 loads and reads the values with sc1 loads (MI355X_MICROARCH.md "Valid forms",
//     row 1 — the form grid_reduce already uses). Each value of r is summed by ONE workgroup in a
//     fixed butterfly order, so r is identical everywhere and deterministic.
//   * phase B: the tile, read again from L2 / the Infinity Cache in the transposed operand
//     layout two blocks later (phase B lags phase A by two blocks), meets r on MFMA:
//     G[panel columns] += tile^T r. The G accumulators (64 x 32 per wave) stay in registers over
//     all blocks of the row group; at the end each workgroup writes its rows of G slab rg.
//   * pipelining: phase A of block b+1 is issued (and published) before the wait for block b's
//     partials, so the exchange hides behind one block of MFMA work; the A loads of block b+2 are
//     in flight meanwhile. Partials live in a ring of 4 slots per row group: a workgroup can be at
//     most two blocks behind any other (it cannot pass the wait of block b-1 before every
//     workgroup has published it), so slot (b+1) % 4 is never still being read.
//   * counters: cnt[rg][b] gains P per launch; the host passes target = P * launch_count, so no
//     counter is reset inside the launch. Every spin is bounded: on timeout the workgroup sets
//     *err and carries on (its results are then wrong); glx_residual_gradient reads *err back
//     and recomputes R and G with two passes when it is set.
//
// Outputs: Sraw = S (the finalize kernel forms r = S - b with the same subtraction, bit-identical
// to the r used for G here) and Gs[rg] = the row group's part of G; the consumer sums the RG
// slabs in slab order (slab_sum), so G is deterministic. All 256 workgroups must be resident at
// once (they wait for each other): the host launches this only when the device has >= 256 CUs
// (resgrad_device_ok), as a cooperative launch, which the runtime refuses when the grid cannot
// be co-resident.
//
// XL mode relies on gfx950's write-through vector L1 and on the readers sharing the writer's XCD
// L2: the granules are stored with workgroup-scope (plain) atomic stores, which the HIP memory
// model does not make visible to other workgroups; on gfx950 they reach the XCD's L2, where the
// readers' sc1 loads find them (measured correct at every tested shape, and a wrong placement
// is caught: a granule never observed times the wait out, *err is set and the host recomputes).
// GLX_RG_XCD=0 selects the placement-independent agent-scope form.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "glx.h"
#include "glx_device.h"

namespace glx {

namespace {
typedef double fd2 __attribute__((ext_vector_type(2)));
typedef double fd4 __attribute__((ext_vector_type(4)));

constexpr int kFW = 8;                 // waves per workgroup (two per SIMD)
constexpr int kFThreads = 64 * kFW;
constexpr int kFCols = 64;             // columns of A per wave
constexpr int kFCh = kFCols / 16;      // 16-column chunks per wave
constexpr int kFPanel = kFW * kFCols;  // 512 columns per workgroup
constexpr int kFRows = 16;             // rows per block
constexpr int kFRing = 4;              // partial slots per row group
constexpr int kFL = 32;                // l
constexpr int kFBlk = kFRows * kFL;    // 512 values per partial
constexpr int kFPerCU = 1;             // workgroups per CU
constexpr int kFGrid = 256 * kFPerCU;

__device__ inline fd4 mfma(double a, double b, fd4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// A double handed to other workgroups as two 8-byte granules {tag, 32-bit half}, each stored by
// one agent-scope (sc1) atomic store: the data is its own flag (cdna_hip_programming.md §6
// Guideline 16, R2). A reader accepts the value once both tags equal the expected one.
typedef unsigned long long u64;
// XL (XCD-local exchange): every workgroup that reads these granules shares the writer's XCD (the
// grouping is taken from HW_REG_XCC_ID at run time, see k_resgrad), so a plain 8-byte store,
// which keeps the line in that XCD's L2, is enough: the readers' sc1 loads bypass their L1 and
// are served by the same L2. Otherwise sc1 (write-through) stores, visible on every XCD.
// Architecture dependence: the HIP memory model does not promise that a
// workgroup-scope store becomes visible to another workgroup. XL relies on two gfx950 facts:
// the vector L1 is write-through (a store reaches the XCD's L2 without a writeback), and every
// reader is on the writer's XCD and loads with sc1 (L1 bypass). Each granule carries its own tag,
// so there is no separate flag whose ordering a fence would have to provide. The solver never
// launches this kernel (glx_residual_gradient(one_pass = 1) only); the portable form is XL = 0.
template <bool XL>
__device__ inline void put_value(u64* g, unsigned tag, double v) {
  const u64 u = (u64)__double_as_longlong(v);
  constexpr int scope = XL ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT;
  __hip_atomic_store(g, ((u64)tag << 32) | (u & 0xffffffffull), __ATOMIC_RELAXED, scope);
  __hip_atomic_store(g + 1, ((u64)tag << 32) | (u >> 32), __ATOMIC_RELAXED, scope);
}
struct Gran {
  u64 w0, w1;
};
__device__ inline Gran get_gran(const u64* g) {
  return Gran{__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
              __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
}
__device__ inline bool gran_ok(const Gran& x, unsigned tag) {
  return (unsigned)(x.w0 >> 32) == tag && (unsigned)(x.w1 >> 32) == tag;
}
__device__ inline double gran_value(const Gran& x) {
  return __longlong_as_double((long long)((x.w1 << 32) | (x.w0 & 0xffffffffull)));
}
}  // namespace

// Phase timestamps of workgroup 0 (scripts/rg_probe.hip builds this file with GLX_RG_TRACE and
// sets the buffer; the library build has no tracing).
#ifdef GLX_RG_TRACE
__device__ unsigned long long* g_rg_trace = nullptr;
#define RG_STAMP(b, k)                                                                        \
  do {                                                                                        \
    if (g_rg_trace != nullptr && blockIdx.x == 0 && threadIdx.x == 0)                         \
      g_rg_trace[(b) * 8 + (k)] = __builtin_amdgcn_s_memtime();                                \
  } while (0)
#else
#define RG_STAMP(b, k) do {} while (0)
#endif
#ifndef GLX_RG_KB
#define GLX_RG_KB 8
#endif

template <bool XL>
__global__ __launch_bounds__(kFThreads, kFPerCU) void k_resgrad(
    const double* __restrict__ A, const double* __restrict__ X, const double* __restrict__ B,
    double* __restrict__ Sraw, double* __restrict__ Gs, u64* Pg, u64* Rg, unsigned* xslot,
    unsigned epoch0,
    int64_t m, int64_t n, int RG, int NB, int* err, unsigned spin_max) {
  __shared__ __attribute__((aligned(16))) double xs[kFW][kFCols * kFL];     // X slices
  __shared__ __attribute__((aligned(16))) double red[kFW / 2][kFBlk];        // wave partials
  __shared__ __attribute__((aligned(16))) double rb[kFBlk];                  // r of the block
  __shared__ int bad;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int P = (int)(n / kFPanel);
  // XL: the row group is this workgroup's XCD (HW_REG_XCC_ID) and the panel its arrival order
  // there (xslot, zeroed before the launch); a workgroup beyond P on one XCD flags an error.
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
  if (XL && (pnl >= (int)(n / kFPanel) || rg >= RG)) {
    if (tid == 0) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;   // the others of its XCD time out and flag; the host falls back to two passes
  }
  const int64_t col0 = (int64_t)pnl * kFPanel + (int64_t)wave * kFCols;
  const int64_t rbase = (int64_t)rg * (m / RG);
  if (tid == 0) bad = 0;

  // X slice of this wave (rows col0 .. col0 + 63) in LDS for the whole launch. Row k's two
  // 16-column halves swap when bit 2 of k is set, so that the B-operand reads of phase A (lane
  // (i, q): row 16 ch + 4 q + e, column 16 nt + i) put lane groups q and q + 1 on different banks.
  double* xw = &xs[wave][0];
  for (int idx = lane; idx < kFCols * kFL; idx += 64) {
    const int k = idx / kFL, c = idx % kFL;
    xw[k * kFL + (c ^ (((k >> 2) & 1) << 4))] = X[(col0 + k) * kFL + c];
  }
  __syncthreads();

  fd4 gacc[kFCh][2];   // G rows col0 + 16 ct + (q + 4 r), columns 16 nt + i
#pragma unroll
  for (int ct = 0; ct < kFCh; ++ct)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) gacc[ct][nt] = fd4{0.0, 0.0, 0.0, 0.0};

  // A tile of block b, A-operand layout: row rbase + 16 b + i, columns col0 + 16 ch + 4 q + e
  double a[kFCh][4];
  auto load_tile = [&](int64_t b) {
    b = b < NB ? b : NB - 1;
    const double* ap = A + (rbase + 16 * b + i) * n + col0 + 4 * q;
#pragma unroll
    for (int ch = 0; ch < kFCh; ++ch) {
      const fd2 v0 = *reinterpret_cast<const fd2*>(ap + 16 * ch);
      const fd2 v1 = *reinterpret_cast<const fd2*>(ap + 16 * ch + 2);
      a[ch][0] = v0[0]; a[ch][1] = v0[1]; a[ch][2] = v1[0]; a[ch][3] = v1[1];
    }
  };
  auto tag_of = [&](int64_t b) { return epoch0 + (unsigned)b + 1u; };
  // re-read the two granules at g until their tags match (every lane of the wave); bounded
  auto sweep = [&](const u64* g, unsigned tag, Gran x) -> double {
    unsigned spins = 0;
    while (!__all(gran_ok(x, tag))) {
      __builtin_amdgcn_s_sleep(1);
      x = get_gran(g);
      if (++spins > spin_max) {   // bounded: flag and continue with whatever is there
        if (lane == 0) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bad = 1;
        }
        break;
      }
    }
    return gran_value(x);
  };

  // phase A of block b, MFMA part: the wave's 16 x 32 partial of S = A X
  auto phase_a_mma = [&](fd4 (&sp)[2]) {
    // two accumulator sets (even / odd chunks): four independent MFMA chains
    fd4 c0[2] = {fd4{0.0, 0.0, 0.0, 0.0}, fd4{0.0, 0.0, 0.0, 0.0}};
    fd4 c1[2] = {fd4{0.0, 0.0, 0.0, 0.0}, fd4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int ch = 0; ch < kFCh; ch += 2)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 16 * ch + 4 * q + e;   // (k >> 2) & 1 == q & 1
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int cx = 16 * (nt ^ (q & 1)) + i;
          c0[nt] = mfma(a[ch][e], xw[k * kFL + cx], c0[nt]);
          c1[nt] = mfma(a[ch + 1][e], xw[(k + 16) * kFL + cx], c1[nt]);
        }
      }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) sp[nt] = c0[nt] + c1[nt];
  };
  // phase A of block b, the rest: the wave partials summed through LDS in a fixed order (the
  // first half of the waves store, the second half add theirs: w + (w + W/2), then in wave
  // order) and the workgroup's partial handed out as granules
  auto phase_a_rest = [&](const fd4 (&sp)[2], int64_t b) {
    if (wave < kFW / 2) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave][(q + 4 * r) * kFL + 16 * nt + i] = sp[nt][r];
    }
    __syncthreads();
    if (wave >= kFW / 2) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double* d = &red[wave - kFW / 2][(q + 4 * r) * kFL + 16 * nt + i];
          *d = *d + sp[nt][r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < kFBlk / kFThreads; ++h) {
      const int v = tid + kFThreads * h;
      double sv = red[0][v];
#pragma unroll
      for (int w = 1; w < kFW / 2; ++w) sv = sv + red[w][v];
      u64* slot = Pg + ((((int64_t)rg * kFRing + (b % kFRing)) * P + pnl) * kFBlk + v) * 2;
      put_value<XL>(slot, tag_of(b), sv);
    }
    RG_STAMP(b, 5);
  };

  // Exchange of block b in two hops, each value read by ONE workgroup in the first and by all in
  // the second (2 x 512 values per workgroup per block instead of P x 512):
  //   hop 1 (reduce-scatter): workgroup p sums slice p of the block (512 / P values) over the P
  //     partials in a fixed butterfly order (P lanes per value, one partial per lane), subtracts
  //     b and hands out r of its slice (granules) and writes S (Sraw, for the finalize);
  //   hop 2 (all-gather): every workgroup reads the 512 values of r into LDS.
  // hop 1: slice of 512 / P values; T = kFThreads / slice consecutive lanes per value, each lane
  // adding kPL = P / T partials (lane sub: partials kPL sub .. kPL sub + kPL - 1, in order)
  const int T = kFThreads / (kFBlk / P);
  const int sub = tid % T, vl = tid / T;
  const int v1 = pnl * (kFBlk / P) + vl;
  constexpr int kPL = kFBlk / kFThreads;   // = P / T
  auto hop1_g = [&](int64_t b, int k) {
    return Pg + ((((int64_t)rg * kFRing + (b % kFRing)) * P + kPL * sub + k) * kFBlk + v1) * 2;
  };
  struct Gr2 { Gran x[kPL]; };
  auto hop1_issue = [&](int64_t b) -> Gr2 {
    Gr2 r;
#pragma unroll
    for (int k = 0; k < kPL; ++k) r.x[k] = get_gran(hop1_g(b, k));
    return r;
  };
  // the b value hop 1 subtracts (issued with the first read of the partials)
  auto hop1_b = [&](int64_t b) -> double {
    return sub == 0 ? B[(rbase + 16 * b + v1 / kFL) * kFL + v1 % kFL] : 0.0;
  };
  auto hop1_finish = [&](int64_t b, Gr2 x, double bv) {
    double sum = sweep(hop1_g(b, 0), tag_of(b), x.x[0]);
#pragma unroll
    for (int k = 1; k < kPL; ++k) sum = sum + sweep(hop1_g(b, k), tag_of(b), x.x[k]);
    RG_STAMP(b, 4);
    for (int off = 1; off < T; off <<= 1) sum = sum + __shfl_xor(sum, off);
    if (sub == 0) {
      const int64_t row = rbase + 16 * b + v1 / kFL;
      const int col = v1 % kFL;
      put_value<XL>(Rg + (((int64_t)rg * kFRing + (b % kFRing)) * kFBlk + v1) * 2, tag_of(b),
                sum - bv);
      Sraw[row * kFL + col] = sum;
    }
  };
  auto hop2 = [&](int64_t b) {
    __syncthreads();   // rb: the previous phase B has read it
    Gran x[kPL];
#pragma unroll
    for (int h = 0; h < kPL; ++h)
      x[h] = get_gran(Rg + (((int64_t)rg * kFRing + (b % kFRing)) * kFBlk + tid + kFThreads * h) * 2);
#pragma unroll
    for (int h = 0; h < kPL; ++h) {
      const u64* g = Rg + (((int64_t)rg * kFRing + (b % kFRing)) * kFBlk + tid + kFThreads * h) * 2;
      rb[tid + kFThreads * h] = sweep(g, tag_of(b), x[h]);
    }
    __syncthreads();
  };

  // phase B of block b: G[col0 + 16 ct + .., :] += tile^T r (K = the block's 16 rows). The
  // tile is read a second time, in the transposed operand layout (lane (i, q): row 4 s + q,
  // column 16 ct + i; 16 lanes = 128 contiguous bytes), from L2 / the Infinity Cache: phase A
  // streamed it from HBM two blocks earlier.
  double at[4][kFCh];
  auto load_at = [&](int64_t b) {
    const double* ap = A + (rbase + 16 * b + q) * n + col0 + i;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int ct = 0; ct < kFCh; ++ct) at[s4][ct] = ap[(int64_t)4 * s4 * n + 16 * ct];
  };
  auto phase_b = [&]() {
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      double rr[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) rr[nt] = rb[(4 * s4 + q) * kFL + 16 * nt + i];
#pragma unroll
      for (int ct = 0; ct < kFCh; ++ct)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) gacc[ct][nt] = mfma(at[s4][ct], rr[nt], gacc[ct][nt]);
    }
  };

  // Schedule, iteration j (phase B lags phase A by two blocks, so every exchange it waits for was
  // produced one iteration earlier): the loads of the transposed tile j - 1 and the first read of
  // block j's partials are issued, phase A's MFMAs of block j + 1 run while they fly, hop 1 of
  // block j finishes, phase A of j + 1 is handed out, hop 2 collects r of j - 1, the loads of
  // tile j + 2 are issued (after the exchange's loads: vmcnt retires in order) and phase B of
  // j - 1 runs.
  {
    fd4 sp[2];
    load_tile(0);
    phase_a_mma(sp);
    phase_a_rest(sp, 0);
    if (NB > 1) load_tile(1);
  }
  for (int64_t j = 0; j <= NB; ++j) {
    RG_STAMP(j, 0);
    // hop 1's reads first: vmcnt retires in order, so its check then does not wait for the
    // transposed-tile loads issued behind it
    Gr2 x;
    double bv = 0.0;
    if (j < NB) {
      x = hop1_issue(j);
      bv = hop1_b(j);
    }
    if (j >= 1) load_at(j - 1);
    fd4 sp[2];
    if (j + 1 < NB) phase_a_mma(sp);
    RG_STAMP(j, 1);
    if (j < NB) hop1_finish(j, x, bv);
    RG_STAMP(j, 7);
    if (j + 1 < NB) phase_a_rest(sp, j + 1);
    RG_STAMP(j, 6);
    if (j >= 1) hop2(j - 1);
    RG_STAMP(j, 2);
    if (j + 2 < NB) load_tile(j + 2);
    if (j >= 1) phase_b();
    RG_STAMP(j, 3);
  }

  // this workgroup's rows of G slab rg (C map: rows col0 + 16 ct + q + 4 r, column 16 nt + i)
  double* gout = Gs + (int64_t)rg * n * kFL;
#pragma unroll
  for (int ct = 0; ct < kFCh; ++ct)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double v = bad ? __builtin_nan("") : gacc[ct][nt][r];
        gout[(col0 + 16 * ct + q + 4 * r) * kFL + 16 * nt + i] = v;
      }
}

// ---------------------------------------------------------------------------------------------
// shape / device checks and launch
// ---------------------------------------------------------------------------------------------
// workspace: partial granules (ring) | r granules (ring) | XCD arrival counters; tags start at
// 1, so zeroed granules never match
struct RgLayout {
  size_t pg, rg, xs, total;
};
static RgLayout rg_layout(int64_t m, int64_t n) {
  const int64_t P = n / kFPanel, RG = kFGrid / P;
  (void)m;
  auto up = [](size_t v) { return (v + 255) & ~size_t(255); };
  RgLayout L;
  L.pg = 0;
  L.rg = up(sizeof(u64) * 2 * (size_t)RG * kFRing * P * kFBlk);
  L.xs = L.rg + up(sizeof(u64) * 2 * (size_t)RG * kFRing * kFBlk);
  L.total = L.xs + up(sizeof(unsigned) * 8 * 32) + 256;
  return L;
}

bool resgrad_shape_ok(int esize, int64_t m, int64_t n, int64_t l) {
  if (esize != 8 || l != kFL || n % kFPanel != 0) return false;
  const int64_t P = n / kFPanel;
  // hop 1 puts P / 2 lanes (a power of two, <= 64: one wave) on each of the 512 / P values of a
  // slice
  if (P < 2 || P > 128 || (P & (P - 1)) != 0) return false;
  const int64_t RG = kFGrid / P;
  return m % (RG * kFRows) == 0 && m / RG >= 2 * kFRows;
}

int resgrad_groups(int64_t n) { return (int)(kFGrid / (n / kFPanel)); }

// every workgroup of the launch must be resident at once: kFPerCU per CU on >= 256 CUs
bool resgrad_device_ok() {
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
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(k_resgrad<true>),
                                                     kFThreads, 0) == hipSuccess)
      ok[dev] = (cus * kFPerCU >= kFGrid && occ >= kFPerCU) ? 1 : 0;
  }
  return ok[dev] == 1;
}

size_t resgrad_ws_bytes(int64_t m, int64_t n) { return rg_layout(m, n).total; }

// XCD-local exchange where the row groups can be the XCDs (8 row groups; GLX_RG_XCD=0: off)
static bool rg_xcd_mode(int64_t n) {
  static const int env = [] { const char* v = std::getenv("GLX_RG_XCD"); return v ? std::atoi(v) : 1; }();
  return env != 0 && kFGrid / (n / kFPanel) == 8;
}

bool launch_resgrad(const double* A, const double* X, const double* B, double* Sraw, double* Gs,
                    void* ws, unsigned launch_count, int64_t m, int64_t n, int* err, hipStream_t st) {
  const int64_t P = n / kFPanel, RG = kFGrid / P, NB = m / RG / kFRows;
  const RgLayout L = rg_layout(m, n);
  char* w = static_cast<char*>(ws);
  unsigned* xslot = reinterpret_cast<unsigned*>(w + L.xs);
  unsigned ep = (unsigned)((launch_count - 1) * NB);
  // spin bound of every hand-off wait (GLX_RG_SPIN = log2 of it, default 22; the tests force
  // the error path with a tiny bound)
  static const unsigned spin_max = [] {
    const char* v = std::getenv("GLX_RG_SPIN");
    const int lg = v && *v ? std::atoi(v) : 22;
    return lg <= 0 ? 0u : (1u << (lg > 30 ? 30 : lg));
  }();
  unsigned smax = spin_max;
  u64* pg = reinterpret_cast<u64*>(w + L.pg);
  u64* rgp = reinterpret_cast<u64*>(w + L.rg);
  int rgi = (int)RG, nbi = (int)NB;
  void* args[] = {(void*)&A, (void*)&X, (void*)&B, (void*)&Sraw, (void*)&Gs, (void*)&pg, (void*)&rgp,
                  (void*)&xslot, (void*)&ep, (void*)&m, (void*)&n, (void*)&rgi, (void*)&nbi,
                  (void*)&err, (void*)&smax};
  // cooperative launch: the workgroups wait for each other, so a grid that cannot be resident at
  // once is refused at launch (the caller then runs two passes) instead of spinning
  const bool xl = rg_xcd_mode(n);
  if (xl) (void)hipMemsetAsync(xslot, 0, sizeof(unsigned) * 8 * 32, st);
  const void* kern = xl ? reinterpret_cast<const void*>(k_resgrad<true>)
                        : reinterpret_cast<const void*>(k_resgrad<false>);
  const hipError_t e = hipLaunchCooperativeKernel(kern, dim3((unsigned)(RG * P)), dim3(kFThreads), args, 0, st);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}

// the granules must be zero before the first launch (launch_count 1)
void resgrad_reset(void* ws, int64_t m, int64_t n, hipStream_t st) {
  (void)hipMemsetAsync(ws, 0, rg_layout(m, n).total - 256, st);
}

}  // namespace glx
