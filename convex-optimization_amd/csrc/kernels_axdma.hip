// kernels_axdma.hip — A @ X (reference: gl_ProxGD_primal.py:25,61,129 `A @ x`) with A and X
// staged in LDS by LDS-DMA, f64 and f32 (kinds 8/9 of the A @ X planner, kernels_gemm.hip).
#include "glx_mfma.h"

namespace glx {

// ------------------------------------------------------------------------------------------
// A @ X, kind 8 (f64): A and X staged in LDS by LDS-DMA (global_load_lds_dwordx4). The kind-5
// tile loads A straight into the MFMA operand registers, so one wave-instruction can only
// cover 16 rows x 64 B (a lane's bytes must be its own row's); the streaming probe
// (scripts/stream_probe.hip, profiles/r2_stream/) caps that shape at 5.9-6.2 TB/s against
// 6.3-7.3 TB/s for whole 256-512-B pieces. Here the wave-instruction that fetches A is decoupled
// from the lane that consumes it: each instruction lands 4 rows x 256 B (KC = 32) in LDS and
// the lanes read their MFMA operands back with ds_read_b128.
//
// Block = WAVES waves; wave w owns 16 rows (row0 .. row0 + 15) and streams them itself; the
// block's X chunk (KC rows of every source) is fetched by one 1-KiB instruction per wave and
// shared. A ring of NS LDS slots, NS - 1 chunks in flight. Per chunk every wave waits for its
// own DMAs of that chunk with a counted vmcnt, then ONE raw s_barrier (never __syncthreads(),
// whose fence waits for vmcnt(0) and would drain the ring) makes every wave's DMAs visible,
// then the next chunk is issued into the slot the previous chunk used (every wave has read it:
// its ds_reads completed before the wave reached the barrier, lgkmcnt(0) in the same wait).
//
// LDS images (one __shared__ array; the DMA destination is lane-linear, so swizzles go on the
// SOURCE address, cdna_hip_programming.md §5.4 rule 21):
//   A: wave's [16][SLR] 16-B slots (SLR = KC / EV, EV = 16 / sizeof(T) values per slot), slot s
//      of row i stored at s ^ sw(i). Lane (i, q) reads slots s = q + 4j (j < SLR / 4), i.e.
//      k = EV s + e — conflict-free ds_read_b128 for every 4 x 16-lane group
//      (MI355X_MICROARCH.md §LDS), checked by scripts/lds_banks.py. f32 with KC = 64 has the
//      same byte image as f64 with KC = 32 (256-B row pieces).
//   X: per source KC rows of l values as 16-value units of UB = 16 sizeof(T) bytes (k * NT +
//      half); unit u stored at u ^ ((k / EV) & (EV - 1)). f64 (ds_read_b64): the two 16-lane
//      halves of a group (lane groups q = 0/1 and 2/3 read rows k = 2(q + 4j) + e) fall on
//      different bank halves; f32 (ds_read_b32, all 64 lanes at once): the four lane groups'
//      64-B units (rows k = 4(q + 4j) + e) land on the four different 16-bank quarters.
// MFMA operand maps as in kind 5 (k permuted inside a chunk, X read with the same permutation).
// Past the end of a block's K range the ring re-issues the last chunk (an L2 hit, discarded),
// so every wave's DMA count per chunk is the same constant the counted vmcnt needs.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) void g_void_t;
typedef __attribute__((address_space(3))) void l_void_t;

// one 16-B-per-lane LDS-DMA wave-instruction: lane j writes lds_base + 16 j (lds_base uniform)
template <bool NTL>
__device__ inline void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((g_void_t*)src, (l_void_t*)lds_base, 16, 0, NTL ? 2 : 0);
}

// LDS bytes of a kind-8 tile: NS slots of WAVES 16-row A chunks + the X chunk of every source
// (+ 1 KiB dummy when the X pieces do not divide evenly among the waves)
template <typename T, int NT, int NSRC, int NS, int KC, int WAVES, int MT = 1>
constexpr int dma_lds_bytes() {
  constexpr int es = (int)sizeof(T);
  return NS * (WAVES * 16 * MT * KC * es + NSRC * KC * 16 * NT * es) +
         ((NSRC * KC * 16 * NT * es / 1024) % WAVES ? 1024 : 0);
}

// Infinity-Cache hand-off (GemmPlan::ax_keep_mib, a kernel argument; the solver's default is
// kKeepMiB = 192, GLX_AX_KEEP_MIB overrides it, 0 = off): with NTL, the last chunks of every
// block's walk are fetched with the default policy instead, about that many MiB of A over the
// grid, so they stay in the 256 MiB Infinity Cache for the next pass (A^T R).

// A slot swizzle of row i for SLR 16-B slots per row piece
template <int SLR>
__device__ inline int dma_sw(int i) { return SLR >= 16 ? (i & 15) : ((i >> 1) & 7); }

template <typename T, int NT, int NSRC, int NS, int KC, int WAVES, bool NTL, bool HOIST, bool PIPE,
          int MT, bool EG = false>
__global__ __launch_bounds__(64 * WAVES) void k_ax_dma(const T* __restrict__ A,
                                                      const T* __restrict__ X0,
                                                      const T* __restrict__ X1,
                                                      const T* __restrict__ X2,
                                                      T* __restrict__ P, int64_t m, int64_t n,
                                                      int64_t chunks, int S, int gx, int xmap,
                                                      const int* __restrict__ gate, int epoch,
                                                      Pub pub, int keep_mib, EGat eg) {
  typedef MF<T> M;
  typedef typename M::acc_t C;
  typedef typename M::vec_t V;                      // one 16-B slot of A
  constexpr int ES = (int)sizeof(T);
  constexpr int EV = 16 / ES;                       // values per 16-B slot (2 f64, 4 f32)
  constexpr int UB = 16 * ES;                       // bytes of one 16-value X unit
  constexpr int LPU = UB / 16;                      // DMA lanes per X unit
  constexpr int UPI = 1024 / UB;                    // X units per DMA wave-instruction
  constexpr int L = 16 * NT;
  constexpr int NC = NT * NSRC;
  constexpr int SLR = KC / EV;                      // 16-B slots per row of an A chunk
  constexpr int AW = 16 * MT * KC * (int)sizeof(T); // one wave's A chunk (MT 16-row tiles)
  constexpr int NIA = AW / 1024;                    // its LDS-DMA instructions
  constexpr int XS = KC * L * (int)sizeof(T);       // one source's X chunk
  constexpr int XB = NSRC * XS;
  constexpr int NXT = XB / 1024;                    // the block's X instructions per chunk
  constexpr int NIX = (NXT + WAVES - 1) / WAVES;    // per wave (surplus ones load a dummy)
  constexpr bool XDUP = NIX * WAVES != NXT;
  constexpr int SLOT = WAVES * AW + XB;
  constexpr int LDSB = NS * SLOT + (XDUP ? 1024 : 0);
  constexpr int NI = NIA + NIX;                     // DMA instructions per wave and chunk
  constexpr int D = NS - 1;                         // chunks in flight beyond the computed one
  constexpr int JN = SLR / 4;                       // ds_read_b128 of A per lane and chunk
  constexpr int WAITN = (D - 1) * NI;
  static_assert(KC == 16 || KC == 32 || KC == 64, "chunk of 16, 32 or 64 columns");
  static_assert(XS % 1024 == 0 && AW % 1024 == 0, "whole 1-KiB pieces");
  static_assert(D >= 1 && WAITN <= 63, "vmcnt range");
  static_assert(LDSB <= 160 * 1024, "LDS");
  static_assert(MT == 1 || PIPE, "two row tiles per wave: pipelined form only");
  static_assert(!EG || (NSRC == 1 && PIPE && HOIST && NS == 2 && KC == 32 && 64 % L == 0),
                "the fused A e: one MFMA source, the pipelined two-slot tile");
  // PIPE && HOIST: the pipelined loop with the DMA issues and operand reads interleaved into
  // the MFMA stream (sched_group_barrier) instead of all issued in front of it
  // s_waitcnt vmcnt(WAITN) expcnt(7) lgkmcnt(0) (gfx9 encoding: vmcnt[3:0] bits 3:0, expcnt
  // bits 6:4, lgkmcnt bits 11:8, vmcnt[5:4] bits 15:14)
  constexpr int kWaitVmLgkm0 = (WAITN & 15) | (7 << 4) | ((WAITN >> 4) << 14);
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];

  GLX_CLK(0);
  if (pub.host != nullptr && blockIdx.x == 0) {   // as k_ax_lds: workgroup 0 carries the packet
    if (threadIdx.x == 0)
      publish_packet(pub.s, pub.ns, pub.host, pub.host_seq, pub.seq, pub.s2, pub.off2, pub.n2,
                     pub.s3, pub.off3, pub.n3);
    return;
  }
  if (!gate_live(gate, epoch)) return;
  int bx, by;
  if (!ax_block(xmap, gx, S, bx, by, pub.host != nullptr ? 1 : 0)) return;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int64_t row0 = (int64_t)bx * (16 * MT * WAVES) + (int64_t)wave * (16 * MT);
  const int64_t cb = chunks * by / S, ce = chunks * (by + 1) / S;
  const int64_t nch = ce - cb;
  if (nch <= 0) return;   // block-uniform

  // A piece t of this wave: linear slot 64 t + lane of the [16][SLR] image
  const T* asrc[NIA];
#pragma unroll
  for (int t = 0; t < NIA; ++t) {
    const int ls = 64 * t + lane, ri = ls / SLR, p = ls % SLR;
    int64_t r = row0 + ri;
    r = r < m ? r : m - 1;
    asrc[t] = A + r * n + cb * KC + EV * (p ^ dma_sw<SLR>(ri & 15));
  }
  // X pieces: instruction tx = wave + WAVES r of the block covers the UPI units UPI tx ..
  const T* xsrc[NIX];
  int xdst[NIX];
#pragma unroll
  for (int r = 0; r < NIX; ++r) {
    const int tx = wave + WAVES * r;
    const int txc = tx % NXT;                        // surplus: a real piece into the dummy
    const int pu = UPI * txc + lane / LPU;
    const int src = pu / (KC * NT), u = pu % (KC * NT);
    const int k = u / NT;
    const int us = u ^ ((k / EV) & (EV - 1));
    const T* xb = src == 0 ? X0 : (src == 1 ? X1 : X2);
    xsrc[r] = xb + (cb * KC + us / NT) * L + (us % NT) * 16 + (lane % LPU) * EV;
    xdst[r] = tx < NXT ? WAVES * AW + tx * 1024 : -1;
  }
  const int64_t rot = ax_rot(xmap, bx, gx, nch);
  int64_t kt = nch;   // walk chunks [kt, nch) load with the default policy (the hand-off)
  if constexpr (NTL) {
    const int64_t kb = (int64_t)keep_mib << 20;
    if (kb > 0) kt = nch - kb / ((int64_t)gridDim.x * WAVES * AW);
  }
  auto issue = [&](int64_t c, int slot) {
    c = c < nch ? c : nch - 1;
    const bool nt = c < kt;
    c += rot;                            // the walk starts at chunk rot (mod nch)
    c = c >= nch ? c - nch : c;
    char* sb = lds + slot * SLOT;
    if (NTL && nt) {
#pragma unroll
      for (int t = 0; t < NIA; ++t) glds16<NTL>(asrc[t] + c * KC, sb + wave * AW + t * 1024);
    } else {
#pragma unroll
      for (int t = 0; t < NIA; ++t) glds16<false>(asrc[t] + c * KC, sb + wave * AW + t * 1024);
    }
#pragma unroll
    for (int r = 0; r < NIX; ++r)
      glds16<false>(xsrc[r] + c * KC * L, XDUP && xdst[r] < 0 ? lds + NS * SLOT : sb + xdst[r]);
  };

  C acc[MT][NC];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[mt][c] = C{};

  // lane (i, q): A slots q + 4j of row i; X units of rows k = EV (q + 4j) + e, whose swizzle
  // (k / EV) & (EV - 1) = q & (EV - 1)
  const int aoff = wave * AW + i * (SLR * 16);
  int asl[MT][JN];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int j = 0; j < JN; ++j) asl[mt][j] = aoff + mt * 16 * SLR * 16 + 16 * ((q + 4 * j) ^ dma_sw<SLR>(i));
  const int xoff = WAVES * AW + ES * i;
  const int xq = q & (EV - 1);
  auto compute = [&](int slot) {
    const char* sb = lds + slot * SLOT;
    V av[JN];
#pragma unroll
    for (int j = 0; j < JN; ++j) av[j] = *reinterpret_cast<const V*>(sb + asl[0][j]);
    if constexpr (HOIST) {
      // every LDS read of the chunk first, in MFMA order, then the MFMAs: the compiler's counted
      // lgkmcnt waits then retire them progressively instead of a wait per small read group
      T xv[JN][EV][NSRC][NT];
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int e = 0; e < EV; ++e)
#pragma unroll
          for (int src = 0; src < NSRC; ++src)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              const int k = EV * (q + 4 * j) + e;
              const int unit = (k * NT + nt) ^ xq;
              xv[j][e][src][nt] = *reinterpret_cast<const T*>(sb + xoff + src * XS + unit * UB);
            }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int e = 0; e < EV; ++e)
#pragma unroll
          for (int src = 0; src < NSRC; ++src)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              acc[0][src * NT + nt] = M::mma(av[j][e], xv[j][e][src][nt], acc[0][src * NT + nt]);
      return;
    }
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const int k = EV * (q + 4 * j) + e;
#pragma unroll
        for (int src = 0; src < NSRC; ++src)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const int unit = (k * NT + nt) ^ xq;
            const T xv = *reinterpret_cast<const T*>(sb + xoff + src * XS + unit * UB);
            acc[0][src * NT + nt] = M::mma(av[j][e], xv, acc[0][src * NT + nt]);
          }
      }
  };

  // ---- EG: the MFMA source X0 is the candidate p itself (A p: the objective and the Armijo test)
  // and A e, e = p where the hard threshold zeroes it, is accumulated on VALU from the staged
  // chunks: lane (c, h) owns column c = lane % L of e and the RPL rows h RPL .. h RPL + RPL - 1 of
  // the wave's 16 MT rows. Per chunk the lane reads the u32 of column c's bitmap that covers the
  // chunk's 32 k (loaded one chunk ahead, like the DMA ring, so the barrier's wait covers it) and,
  // for every set bit k (ascending), adds A[row][k] p[k][c] for its rows, A and p read from the
  // chunk's LDS image. Order: per K split, the block's (rotated) chunk walk, ascending k within a
  // chunk; the finalize sums the S slabs in order and forms A p_thr - b = (A p - b) - A e.
  constexpr int RPL = EG ? (16 * MT * L) / 64 : 1;
  T accE[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) accE[r] = T(0);
  const int ecol_c = lane % L;
  const int rb0 = (lane / L) * RPL;
  const unsigned short* ecol = EG ? eg.bm + (int64_t)ecol_c * eg.bstride : nullptr;
  auto ebits = [&](int64_t c) -> unsigned {   // bitmap word of walk step c (0 past the range)
    if constexpr (!EG) {
      return 0u;
    } else {
      if (c >= nch) return 0u;
      c += rot;
      c = c >= nch ? c - nch : c;
      return *reinterpret_cast<const unsigned*>(ecol + (cb + c) * (KC / 16));
    }
  };
  auto ework = [&](int slot, unsigned bits) {
    if constexpr (EG) {
      const char* sb = lds + slot * SLOT;
      while (bits != 0u) {
        const int kk = __builtin_ctz(bits);
        bits &= bits - 1u;
        const int unit = (kk * NT + (ecol_c >> 4)) ^ ((kk / EV) & (EV - 1));
        // e[k][c] = p[k][c] where the bitmap is set: read from the staged X chunk (source 0 = p)
        const T ev = *reinterpret_cast<const T*>(sb + WAVES * AW + unit * UB + (ecol_c & 15) * ES);
        T ar[RPL];
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          const int w = rb0 + r, ri = w & 15;
          ar[r] = *reinterpret_cast<const T*>(sb + wave * AW + w * (SLR * 16) + 16 * ((kk / EV) ^ dma_sw<SLR>(ri)) +
                                              ES * (kk % EV));
        }
#pragma unroll
        for (int r = 0; r < RPL; ++r) accE[r] = accE[r] + ar[r] * ev;
      }
    }
  };
  unsigned ebr[2] = {0u, 0u};   // bitmap words of the next two walk steps
  (void)ebr;

  if constexpr (PIPE) {
    // Software-pipelined: the operands of chunk c sit in registers (read one iteration earlier)
    // when chunk c's MFMAs issue, so the MFMA pipe does not idle on the LDS read latency after
    // each barrier (the two waves of a SIMD reach it in lockstep); chunk c + 1's reads are
    // issued in front of those MFMAs and complete behind them. Same ring: after the barrier of
    // iteration c every wave has landed chunk c + 1 and finished reading chunk c, whose slot
    // takes chunk c + 1 + D.
    // (fp64 MFMA on live data holds the clock near 2.05-2.2 GHz, where A@X's 2 m n l flops
    // need ~125 us of MFMA pipe against ~158 us of streaming: scripts/axdma_ablate.hip.)
    V av[2][MT][JN];
    T xv[2][JN][EV][NSRC][NT];
    auto read_ops = [&](int slot, V (&a)[MT][JN], T (&x)[JN][EV][NSRC][NT]) {
      const char* sb = lds + slot * SLOT;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < JN; ++j) a[mt][j] = *reinterpret_cast<const V*>(sb + asl[mt][j]);
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int e = 0; e < EV; ++e)
#pragma unroll
          for (int src = 0; src < NSRC; ++src)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              const int k = EV * (q + 4 * j) + e;
              const int unit = (k * NT + nt) ^ xq;
              x[j][e][src][nt] = *reinterpret_cast<const T*>(sb + xoff + src * XS + unit * UB);
            }
    };
    auto mma_ops = [&](const V (&a)[MT][JN], const T (&x)[JN][EV][NSRC][NT]) {
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int e = 0; e < EV; ++e)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int src = 0; src < NSRC; ++src)
#pragma unroll
              for (int nt = 0; nt < NT; ++nt)
                acc[mt][src * NT + nt] = M::mma(a[mt][j][e], x[j][e][src][nt], acc[mt][src * NT + nt]);
    };
    GLX_CLK(1);
    if constexpr (EG) ebr[0] = ebits(0);
#pragma unroll
    for (int d = 0; d < D; ++d) issue(d, d);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAITN) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (EG) ebr[1] = ebits(1);
    issue(D, D);          // NS = D + 1: slot D is free
    read_ops(0, av[0], xv[0]);
    if constexpr (EG) ework(0, ebr[0]);   // chunk 0 before the loop's first barrier frees slot 0
    int cs = 1;           // slot of chunk c + 1
    int64_t c = 0;
    // two chunks per trip so the register sets keep static indices
    for (; c + 1 < nch; c += 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // chunk c + h + 1 landed everywhere, chunk c + h no longer read by anyone. The builtin
        // (not inline asm) so that the compiler's own wait insertion knows the operand reads of
        // the previous iteration are complete and adds no lgkmcnt(0) in front of the MFMAs
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(kWaitVmLgkm0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const int is = cs == 0 ? NS - 1 : cs - 1;   // slot of chunk c + h = slot of c + h + 1 + D
        unsigned eb_use = 0u;
        if constexpr (EG) {   // this step's word (chunk c + h + 1) out, the word of c + h + 2 in
          eb_use = ebr[h ^ 1];
          ebr[h] = ebits(c + h + 1 + D);
        }
        issue(c + h + 1 + D, is);
        read_ops(cs, av[h ^ 1], xv[h ^ 1]);         // next chunk's operands ...
        if constexpr (!HOIST) {
          __builtin_amdgcn_sched_barrier(0);        // (DMA and reads issue before the MFMAs)
          mma_ops(av[h], xv[h]);                    // ... in flight behind this chunk's MFMAs
        } else {
          // An LDS-DMA issue costs its wave ~60-185 cycles (MI355X_MICROARCH.md constants):
          // spread the NI DMAs over the first MFMAs (one after each), then the operand reads two
          // per MFMA, so the issue costs hide under the MFMA pipe instead of delaying it
          mma_ops(av[h], xv[h]);
          constexpr int NMF = MT * JN * EV * NSRC * NT;      // MFMAs per chunk and wave
          constexpr int NRD = MT * JN + JN * EV * NSRC * NT; // operand reads per chunk and wave
#pragma unroll
          for (int g = 0; g < NI; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // 1 VMEM read (the DMA)
          }
#pragma unroll
          for (int g = 0; g < (NRD + 1) / 2; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // 2 DS reads
          }
          __builtin_amdgcn_sched_group_barrier(0x008, NMF - NI - (NRD + 1) / 2, 0);
        }
        if constexpr (EG) {   // behind this chunk's MFMAs: chunk c + h + 1's A e (slot cs)
          __builtin_amdgcn_sched_barrier(0);
          if (c + h + 1 < nch) ework(cs, eb_use);
        }
        cs = cs + 1 == NS ? 0 : cs + 1;
      }
    }
    if (c < nch) mma_ops(av[0], xv[0]);   // odd count: the last chunk is in set 0
    GLX_CLK(2);
  } else {
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d, d);
  int cs = 0;
  for (int64_t c = 0; c < nch; ++c) {
    // this wave's DMAs of chunk c have landed (the D - 1 younger chunks may be in flight) and
    // its reads of chunk c - 1 are done; the barrier publishes both block-wide
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WAITN) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int is = cs == 0 ? NS - 1 : cs - 1;   // slot of chunk c - 1 = slot of chunk c + D
    issue(c + D, is);
    compute(cs);
    cs = cs + 1 == NS ? 0 : cs + 1;
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the surplus re-issues, before exit
  if constexpr (EG) {
    T* pe = static_cast<T*>(eg.Pe) + (int64_t)by * m * L;
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int64_t row = row0 + rb0 + r;
      if (row < m) pe[row * L + ecol_c] = accE[r];
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
  GLX_CLK(3);
}

template <typename T, int NT, int NSRC, int NS, int KC, int WAVES, bool NTL, bool HOIST = false,
          bool PIPE = false, int MT = 1, bool EG = false>
static void ax_dma_go(const GemmPlan& p, int S, const T* A, const T* const* X, T* P,
                      const int* gate, int epoch, hipStream_t st, Pub pub, const EGat& eg = EGat{}) {
  if constexpr (dma_lds_bytes<T, NT, NSRC, NS, KC, WAVES, MT>() > 160 * 1024) {
    throw Error{GLX_E_INVALID, "A@X: this LDS-DMA tile does not fit (160 KiB of LDS)"};
  } else {
    const int gx = (int)cdiv(p.m, 16 * MT * WAVES);
    const int xmap = ax_xmap_flags(p, S);
    const dim3 grid((unsigned)ax_grid(xmap, gx, S) + (pub.host ? 1u : 0u));
    glx_launch((k_ax_dma<T, NT, NSRC, NS, KC, WAVES, NTL, HOIST, PIPE, MT, EG>), grid, dim3(64 * WAVES), 0, st,
                       A, X[0], X[1], X[2], P, p.m, p.n, p.n / KC, S, gx, xmap, gate, epoch, pub,
                       p.ax_keep_mib, eg);
  }
}

// The planner's LDS-DMA tiles (kernels_gemm.hip lds_plan). Code: 9 NS KC/16 flags WAVES, kind 9 =
// two 16-row tiles per wave; flags 7 = non-temporal A + hoisted, pipelined operand reads with the
// DMA issues interleaved into the MFMAs, 6 = the same with the default load policy. The round-3
// sweep's other forms (one row tile per wave, 3-4 ring slots, 16-wave blocks, 16-column chunks,
// no hoisting / pipelining) measured slower and are no longer instantiated.
template <typename T, int NT, int NSRC>
static bool dma_code(const GemmPlan& p, int code, int S, const T* A, const T* const* X, T* P,
                     const int* gate, int epoch, hipStream_t st, Pub pub) {
  switch (code) {
    case 92278: ax_dma_go<T, NT, NSRC, 2, 32, 8, true, true, true, 2>(p, S, A, X, P, gate, epoch, st, pub); return true;
    case 92268: ax_dma_go<T, NT, NSRC, 2, 32, 8, false, true, true, 2>(p, S, A, X, P, gate, epoch, st, pub); return true;
    // f32 (round 4): 64-column chunks, the same 256-B row pieces and LDS image as 92278 in f64
    case 92478:
      if constexpr (sizeof(T) == 4 && NSRC == 1) {
        ax_dma_go<T, NT, NSRC, 2, 64, 8, true, true, true, 2>(p, S, A, X, P, gate, epoch, st, pub);
        return true;
      }
      return false;
    default: return false;
  }
}

int dma_waves(int code) { return code % 10 == 1 ? 16 : code % 10; }

int dma_mt(int code) { return code / 10000 == 9 ? 2 : 1; }

int dma_lds_need(int code, int64_t l, int nsrc, int esize) {
  const int ns = (code / 1000) % 10, kc = 16 * ((code / 100) % 10), waves = dma_waves(code);
  const int xb = nsrc * kc * (int)l * esize;
  return ns * (waves * 16 * dma_mt(code) * kc * esize + xb) + ((xb / 1024) % waves ? 1024 : 0);
}

template <typename T>
bool launch_ax_dma(const GemmPlan& p, int code, int nsrc, int S, const T* A, const T* const* X, T* P,
                   const int* gate, int epoch, hipStream_t st, Pub pub) {
  if (p.l == 16) {
    if (nsrc == 1) return dma_code<T, 1, 1>(p, code, S, A, X, P, gate, epoch, st, pub);
    if (nsrc == 2) return dma_code<T, 1, 2>(p, code, S, A, X, P, gate, epoch, st, pub);
    return dma_code<T, 1, 3>(p, code, S, A, X, P, gate, epoch, st, pub);
  }
  if (nsrc == 1) return dma_code<T, 2, 1>(p, code, S, A, X, P, gate, epoch, st, pub);
  if (nsrc == 2) return dma_code<T, 2, 2>(p, code, S, A, X, P, gate, epoch, st, pub);
  return dma_code<T, 2, 3>(p, code, S, A, X, P, gate, epoch, st, pub);
}

// the fused A e form of the one-source f64 pass 92278 (EGat)
bool ax_egat_ok(const GemmPlan& p, int esize) {
  return esize == 8 && p.ax_kind != 3 && p.axb_code[1] == 92278 && (p.l == 16 || p.l == 32) && p.n % 32 == 0 &&
         p.n <= 65535;
}
template <typename T>
bool launch_ax_egat(const GemmPlan& p, const T* A, const T* X, T* P, const int* gate, int epoch,
                    hipStream_t st, Pub pub, const EGat& eg) {
  if constexpr (sizeof(T) != 8) {
    return false;
  } else {
    if (!ax_egat_ok(p, 8)) return false;
    const T* xs[3] = {X, nullptr, nullptr};
    const int S = p.axb_S[1];
    if (p.l == 16)
      ax_dma_go<T, 1, 1, 2, 32, 8, true, true, true, 2, true>(p, S, A, xs, P, gate, epoch, st, pub, eg);
    else
      ax_dma_go<T, 2, 1, 2, 32, 8, true, true, true, 2, true>(p, S, A, xs, P, gate, epoch, st, pub, eg);
    return true;
  }
}
template bool launch_ax_egat<double>(const GemmPlan&, const double*, const double*, double*, const int*, int,
                                     hipStream_t, Pub, const EGat&);
template bool launch_ax_egat<float>(const GemmPlan&, const float*, const float*, float*, const int*, int,
                                    hipStream_t, Pub, const EGat&);

template bool launch_ax_dma<double>(const GemmPlan&, int, int, int, const double*, const double* const*,
                                    double*, const int*, int, hipStream_t, Pub);
template bool launch_ax_dma<float>(const GemmPlan&, int, int, int, const float*, const float* const*,
                                   float*, const int*, int, hipStream_t, Pub);

}  // namespace glx

GLX_CLK_READER(glx_probe_clock_ax)
