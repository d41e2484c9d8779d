#!/usr/bin/env python3
"""Exhaustive LDS bank-conflict check of csrc/hip/gemm.hip's operand images (CPU, no GPU needed).

Bank model (MI355X_MICROARCH.md §LDS): bank of byte address a = (a/4) mod 64; ds_read_b128 is serviced
in four non-contiguous 16-lane groups, ds_read_b64_tr_b16 in two 32-lane halves; N distinct dwords on
one bank within a group = N-way.  Prints the worst case over every fragment read of a K step."""
G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[l + 32 for l in g] for g in G128]
HALVES = [list(range(32)), list(range(32, 64))]


def worst_way(addrs, groups, width):
    worst = 0
    for g in groups:
        banks = {}
        for l in g:
            for w in range(width // 4):
                dw = addrs[l] // 4 + w
                banks.setdefault(dw % 64, set()).add(dw)
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


def kc(swz):
    """KC image: 128-B rows, chunk c of row r at slot c ^ swz(r); fragment read: lane l -> row l&15,
    chunk 4s + (l>>4)."""
    w = 0
    for r0 in range(0, 144, 16):
        for s in range(2):
            addrs = [(r0 + (l & 15)) * 128 + (((4 * s + (l >> 4)) ^ swz(r0 + (l & 15))) << 4) for l in range(64)]
            w = max(w, worst_way(addrs, G128, 16))
    return w


def mc(swt):
    """MC image: 256-B k-rows, chunk c of k-row k at slot c ^ swt(k); ds_read_b64_tr_b16: lane 4q+p of
    16-lane group g reads k-row 32s + 8g + 4h + q, columns cc + 4p .. +3."""
    w = 0
    for cc in range(0, 128, 16):
        for s in range(2):
            for h in range(2):
                addrs = []
                for l in range(64):
                    g, i = l >> 4, l & 15
                    q, p = i >> 2, i & 3
                    k = 32 * s + 8 * g + 4 * h + q
                    ch = cc // 8 + (p >> 1)
                    addrs.append(k * 256 + ((ch ^ swt(k)) << 4) + 8 * (p & 1))
                w = max(w, worst_way(addrs, HALVES, 8))
    return w


if __name__ == "__main__":
    print("KC  chunk ^ (row & 7)           :", kc(lambda r: r & 7), "-way")
    print("KC  unswizzled                  :", kc(lambda r: 0), "-way")
    print("MC  chunk ^ 2((k&3)|((k>>1)&4)) :", mc(lambda k: ((k & 3) | ((k >> 1) & 4)) << 1), "-way")
    print("MC  unswizzled                  :", mc(lambda k: 0), "-way")
