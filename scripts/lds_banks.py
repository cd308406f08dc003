"""Bank-conflict check of k_ax_dma's LDS reads (kernels_axdma.hip), by the CDNA4 lane-group model
of MI355X_MICROARCH.md §LDS: a wave64 access is serviced in fixed lane groups, one LDS cycle per
group when no two lanes of a group hit the same bank (64 banks of 4 B) at different addresses.

    python scripts/lds_banks.py        # prints the extra cycles per wave-instruction (0 = free)

A image: wave's [16][KC/2] 16-B slots, slot s of row i at s ^ sw(i); lane (i, q) reads slots
q + 4j with ds_read_b128. X image: 128-B units (k * NT + half) stored at u ^ ((k >> 1) & 1);
lane (i, q) reads row k = 2 (q + 4j) + e, column 16 nt + i with ds_read_b64.
"""
B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128 += [[x + 32 for x in g] for g in B128]
B64 = [list(range(0, 32)), list(range(32, 64))]


def extra_cycles(addrs, groups, width):
    worst = 0
    for g in groups:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for d in range(width // 4):
                banks.setdefault(((a // 4) + d) % 64, set()).add(a)
        worst += max(len(v) for v in banks.values()) - 1
    return worst


def sw(kc, i):
    return (i & 15) if kc >= 32 else ((i >> 1) & 7)


def check(kc, nt):
    slr = kc // 2
    out = 0
    for j in range(kc // 8):
        addrs = [(l & 15) * slr * 16 + 16 * ((l >> 4) + 4 * j ^ sw(kc, l & 15)) for l in range(64)]
        out += extra_cycles(addrs, B128, 16)
    for j in range(kc // 8):
        for e in range(2):
            for h in range(nt):
                addrs = []
                for l in range(64):
                    i, q = l & 15, l >> 4
                    k = 2 * (q + 4 * j) + e
                    unit = (k * nt + h) ^ ((k >> 1) & 1)
                    addrs.append(unit * 128 + 8 * i)
                out += extra_cycles(addrs, B64, 8)
    return out


if __name__ == "__main__":
    bad = 0
    for kc in (16, 32, 64):
        for nt in (1, 2):
            c = check(kc, nt)
            bad += c
            print("KC=%d NT=%d: extra LDS cycles per chunk and wave = %d" % (kc, nt, c))
    raise SystemExit(1 if bad else 0)
