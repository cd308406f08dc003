"""Host-side check of k_ax_dma's address arithmetic (kernels_axdma.hip) for every kind-8 code,
l in {16, 32}, 1-3 right-hand sides and the kernel-test shapes: every LDS-DMA source index must
lie inside A (m x n) / its X source (n x l, a source that exists), every LDS destination and
every ds_read inside the tile's LDS, before the kernel ever runs on a GPU.

    python scripts/axdma_addr_check.py
"""
import itertools
import sys

CODES = [84208, 84218, 83208, 83218, 82408, 82418, 88108, 88118, 84204, 84214, 83238, 84238, 83228,
         84131, 84111, 82231, 83258, 84258, 83248, 84151, 94158, 94148, 93158, 92258,
         83278, 93178, 92278, 93168, 92268, 94178, 94168]
SHAPES = [(512, 1024), (1000, 1024), (192, 4096), (129, 64), (64, 128), (4096, 8192), (129, 640),
          (8192, 16384), (1024, 16384), (2048, 16384), (256, 512)]


def sw(kc, i):
    return (i & 15) if kc >= 32 else ((i >> 1) & 7)


def lds_need(ns, kc, w, nt, nsrc, mt=1):
    xb = nsrc * kc * 16 * nt * 8
    return ns * (w * 16 * mt * kc * 8 + xb) + (1024 if (xb // 1024) % w else 0)


def check(code, m, n, nt, nsrc, S):
    ns, kc, w = (code // 1000) % 10, 16 * ((code // 100) % 10), (16 if code % 10 == 1 else code % 10)
    mt = 2 if code // 10000 == 9 else 1
    if n % kc or lds_need(ns, kc, w, nt, nsrc, mt) > 160 * 1024:
        return None
    L = 16 * nt
    slr, aw = kc // 2, 16 * mt * kc * 8
    nia, xs = aw // 1024, kc * L * 8
    nxt = nsrc * xs // 1024
    nix = -(-nxt // w)
    slot = w * aw + nsrc * xs
    ldsb = lds_need(ns, kc, w, nt, nsrc, mt)
    chunks = n // kc
    gx = -(-m // (16 * mt * w))
    for bx, by in itertools.product(sorted({0, gx - 1}), range(S)):   # first and last row block
        cb, ce = chunks * by // S, chunks * (by + 1) // S
        nch = ce - cb
        if nch <= 0:
            continue
        for wave in range(w):
            row0 = bx * 16 * mt * w + wave * 16 * mt
            for c in (0, nch - 1):
                for t in range(nia):
                    assert slot * (ns - 1) + wave * aw + t * 1024 + 1024 <= ldsb
                    for lane in range(64):
                        ls = 64 * t + lane
                        ri, p = ls // slr, ls % slr
                        r = min(row0 + ri, m - 1)
                        col = cb * kc + 2 * (p ^ sw(kc, ri & 15)) + c * kc
                        assert 0 <= col and col + 1 < n, (code, m, n, col)
                        assert 0 <= r < m
                for rr in range(nix):
                    tx = wave + w * rr
                    txc = tx % nxt
                    dst = w * aw + tx * 1024 if tx < nxt else None
                    if dst is not None:
                        assert slot * (ns - 1) + dst + 1024 <= ldsb
                    for lane in range(64):
                        pu = 8 * txc + (lane >> 3)
                        src, u = pu // (kc * nt), pu % (kc * nt)
                        k = u // nt
                        us = u ^ ((k >> 1) & 1)
                        assert src < nsrc, (code, nt, nsrc, tx, txc)
                        row = cb * kc + us // nt + c * kc
                        assert 0 <= row < n
                        assert (us % nt) * 16 + (lane & 7) * 2 + 1 < L
            # ds_reads
            for lane in range(64):
                i, q = lane & 15, lane >> 4
                for t in range(mt):
                    for j in range(kc // 8):
                        a = wave * aw + (16 * t + i) * slr * 16 + 16 * ((q + 4 * j) ^ sw(kc, i))
                        assert wave * aw <= a and a + 16 <= (wave + 1) * aw
                for j in range(kc // 8):
                    for e in range(2):
                        kk = 2 * (q + 4 * j) + e
                        for src in range(nsrc):
                            for h in range(nt):
                                unit = (kk * nt + h) ^ (q & 1)
                                a = w * aw + src * xs + unit * 128 + 8 * i
                                assert w * aw <= a and a + 8 <= slot
    return True


def main():
    ok = 0
    for code in CODES:
        for (m, n) in SHAPES:
            for nt in (1, 2):
                for nsrc in (1, 2, 3):
                    for S in (1, 2, 3, 4, 8):
                        if check(code, m, n, nt, nsrc, S):
                            ok += 1
    print("address checks passed:", ok)


if __name__ == "__main__":
    sys.exit(main())
