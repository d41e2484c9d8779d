"""CPU emulation of csrc/hip/gemm.hip bnred_epilogue's indexing (tile rows, per-wave expert slots k % 3, the
second statistics group of a straddling tile, the wave-order combine and the partial-row layout) against a
direct per-(group, channel) reduction.  Pins the index math the GPU test checks numerically."""
import numpy as np
import pytest


def emulate(U, B, HW, cols, BM=144, BN=256, NW=8, seed=0):
    rng = np.random.default_rng(seed)
    E, EC, K, M = 3, 96, 32 * HW, U * B * 3
    dh = rng.standard_normal((M, K))
    z = rng.standard_normal((M, K))
    st = rng.standard_normal((U, EC, 8))
    st[..., 1] = np.abs(st[..., 1]) + 0.5
    MT = M // BM
    part = np.zeros((U, MT, 2, EC))
    span = HW // 4
    for ti in range(MT):
        for tj in range(cols // BN):
            i0, j0 = ti * BM, tj * BN
            ub = 3 * B
            u_lo, rb = i0 // ub, (i0 // ub + 1) * ub - i0
            u_hi = min(u_lo + 1, U - 1)
            red = {}
            for wave in range(NW):
                for lane in range(64):
                    col = j0 + 4 * lane
                    c = col // HW
                    s = np.zeros((2, 3, 2))
                    for k in range(BM // NW):
                        row, j = wave + NW * k, k % 3
                        e = (wave + NW * j) % 3
                        hi = row >= rb
                        u = u_hi if hi else u_lo
                        mu, inv, a, b = st[u, e * 32 + c, :4]
                        d, zz = dh[i0 + row, col:col + 4], z[i0 + row, col:col + 4]
                        g = np.where(a * zz + b > 0, d, 0)
                        s[int(hi), j, 0] += g.sum()
                        s[int(hi), j, 1] += (g * (zz - mu) * inv).sum()
                    red[(wave, lane // span)] = red.get((wave, lane // span), 0) + s
            for half in range(64 // span):
                for us in range(2):
                    uu = u_lo + us
                    if not (rb > 0 if us == 0 else (rb < BM and uu < U)):
                        continue
                    for e in range(3):
                        for k in range(2):
                            t = 0.0
                            for w in range(NW):
                                j = next(j for j in range(3) if (w + NW * j) % 3 == e)
                                t += red[(w, half)][us, j, k]
                            part[uu, ti, k, e * 32 + (j0 + half * span * 4) // HW] = t
    ref = np.zeros((U, 2, EC))
    for r in range(M):
        u, e = r // (3 * B), r % 3
        for c in range(cols // HW):
            mu, inv, a, b = st[u, e * 32 + c, :4]
            d, zz = dh[r, c * HW:(c + 1) * HW], z[r, c * HW:(c + 1) * HW]
            g = np.where(a * zz + b > 0, d, 0)
            ref[u, 0, e * 32 + c] += g.sum()
            ref[u, 1, e * 32 + c] += (g * (zz - mu) * inv).sum()
    return part.sum(1), ref


@pytest.mark.parametrize("U,B,HW,NW", [(3, 64, 128, 8), (2, 48, 256, 8), (2, 96, 128, 4)])
def test_bnred_epilogue_index_math(U, B, HW, NW):
    got, ref = emulate(U, B, HW, cols=512, NW=NW)
    assert np.allclose(got, ref, rtol=1e-9, atol=1e-9)
