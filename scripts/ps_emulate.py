"""CPU emulation of the pair-sum stencil kernel (lens_amd/csrc/vk_stencil_ps.h):
the same lanes, ring slots, stage schedule (fill / steady / nested tail) and
edge handling, in numpy, for debugging the kernel's bookkeeping without a GPU.

    python scripts/ps_emulate.py          # checks against oracle/cpu_kinetics.c's stencil
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dpp_above(x):          # lane l <- lane l+1 (bound_ctrl: 0 from outside the wave)
    y = np.zeros_like(x)
    y[:-1] = x[1:]
    return y


def dpp_below(x):          # lane l <- lane l-1
    y = np.zeros_like(x)
    y[1:] = x[:-1]
    return y


def pass_ps(src, dst, K, PD, C, out_lo, out_hi, in_lo, in_hi, top, bot, coef, rows_per_chunk, force_general=False):
    ny = src.shape[1]
    KH = (K + C - 1) // C * C
    W = 64 * C - 2 * KH
    tiles_x = (ny + W - 1) // W
    chunks_y = (out_hi - out_lo + rows_per_chunk - 1) // rows_per_chunk
    c4 = 1.0 - 4.0 * coef
    SC = abs(c4) >= 1e-3
    q_coef = coef / c4 if SC else coef
    cK = c4 ** K if SC else 1.0
    if SC:
        cK = 1.0
        for _ in range(K):
            cK *= c4
    lane = np.arange(64)
    NR = PD + 2
    for ty in range(chunks_y):
        for tx in range(tiles_x):
            c0 = out_lo + ty * rows_per_chunk
            c1 = min(c0 + rows_per_chunk, out_hi)
            x0 = tx * W
            cA = x0 - KH + C * lane
            writer = (lane >= KH // C) & (lane < 64 - KH // C)
            cols = cA[:, None] + np.arange(C)[None, :]
            wmask = writer[:, None] & (cols >= 0) & (cols < ny)
            last = np.where((ny - 1 - cA >= 0) & (ny - 1 - cA < C), ny - 1 - cA, -1)
            gl = cA + C - 1 == -1
            gx = x0 - KH <= 0 or x0 - KH + 64 * C >= ny
            ey = (c0 - 2 * K - 2 <= top <= c1 + 2 * K) or (c0 - 2 * K - 2 <= bot <= c1 + 2 * K)
            general = force_general or not SC or ey or gx or ny % C != 0

            def load(r):
                rr = min(max(r, in_lo), in_hi - 1)
                if general:
                    return src[rr][np.clip(cols, 0, ny - 1)].copy()
                inb = (cols >= 0) & (cols < ny)
                out = np.zeros((64, C))
                out[inb] = src[rr][cols[inb]]
                return out

            ring = [np.zeros((64, C)) for _ in range(NR)]
            Wa = [np.zeros((64, C)) for _ in range(K)]
            Wb = [np.zeros((64, C)) for _ in range(K)]
            Da = [np.zeros((64, C)) for _ in range(K)]
            Db = [np.zeros((64, C)) for _ in range(K)]
            is_ = c0 - K + 1
            ring[NR - 1] = load(is_ - 1)
            for u in range(PD):
                ring[u] = load(is_ + u)

            def stage(cn, fr, dold, first, r):
                t = general and r == top
                b = general and r == bot
                right = dpp_above(cn[:, 0])
                e = np.empty((64, C))
                for j in range(C):
                    e[:, j] = cn[:, j + 1] if j + 1 < C else right
                    if general:
                        e[:, j] = np.where(last == j, cn[:, j], e[:, j])
                s_ = fr.copy()
                if general and first:
                    s_[:, C - 1] = np.where(gl, dpp_above(fr[:, 0]), fr[:, C - 1])
                h = cn + e
                dnew = h.copy() if b else s_ + e
                dp = h.copy() if t else dold
                left = dpp_below(dp[:, C - 1])
                v = np.empty((64, C))
                for j in range(C):
                    s = (left if j == 0 else dp[:, j - 1]) + dnew[:, j]
                    v[:, j] = (q_coef * s + cn[:, j]) if SC else (coef * s + c4 * cn[:, j])
                if general:
                    v[:, C - 1] = np.where(gl, dpp_above(v[:, 0]), v[:, C - 1])
                return dnew, v

            def iteration(i, U, act, store):
                P = U & 1
                ring[(U + PD) % NR] = load(i + PD)
                for q in range(act):
                    r = i - 1 - q
                    cn = ring[(U + NR - 1) % NR] if q == 0 else (Wa[q] if P == 0 else Wb[q])
                    fr = ring[U] if q == 0 else (Wb[q] if P == 0 else Wa[q])
                    dold = Da[q] if P == 0 else Db[q]
                    dnew, v = stage(cn, fr, dold, q == 0, r)
                    if P == 0:
                        Db[q] = dnew
                    else:
                        Da[q] = dnew
                    if q + 1 < K:
                        if P == 0:
                            Wb[q + 1] = v
                        else:
                            Wa[q + 1] = v
                    elif store:
                        if SC:
                            v = v * cK
                        row = i - K
                        m = wmask if general else np.repeat(writer[:, None] & (cA[:, None] >= 0) & (cA[:, None] + C <= ny), C, axis=1)
                        dst[row][cols[m]] = v[m]

            for T in range(2 * K - 1):
                iteration(is_ + T, T % NR, min(T // 2 + 1, K), False)
            PH = (2 * K - 1) % NR
            i, i1 = c0 + K, c1 + K
            while i + NR <= i1:
                for u in range(NR):
                    iteration(i + u, (PH + u) % NR, K, True)
                i += NR
            for u in range(NR - 1):
                if u < i1 - i:
                    iteration(i + u, (PH + u) % NR, K, True)
                else:
                    break


def diffuse_ps(f0, coef, n_sub, K, PD=4, C=2, rows=16, **kw):
    """Whole-plane passes of depth K (n_sub a multiple of K) through the emulator."""
    nx, ny = f0.shape
    a = f0.copy()
    b = np.empty_like(a)
    for _ in range(n_sub // K):
        pass_ps(a, b, K, PD, C, 0, nx, 0, nx, 0, nx - 1, coef, rows, **kw)
        a, b = b, a
    return a


if __name__ == '__main__':
    from oracle import cpu
    rng = np.random.default_rng(1)
    ok = True
    for (nx, ny, K, rows, gen) in [(17, 23, 3, 16, False), (40, 260, 3, 16, False), (40, 260, 5, 8, False),
                                   (40, 260, 5, 8, True), (33, 300, 10, 12, False)]:
        f0 = rng.random((nx, ny)) + 0.5
        n_sub = 2 * K
        got = diffuse_ps(f0, 0.05, n_sub, K, rows=rows, force_general=gen)
        ref = np.ascontiguousarray(f0.copy())
        cpu.diffuse(ref, 0.05, n_sub)
        err = np.abs(got - ref).max() / np.abs(ref).max()
        bad = np.argwhere(np.abs(got - ref) > 1e-12 * np.abs(ref).max())
        print((nx, ny, K, rows, gen), 'rel err %.3g' % err, 'bad rows', sorted(set(bad[:, 0].tolist()))[:10],
              'bad cols', sorted(set(bad[:, 1].tolist()))[:10])
        ok &= err < 1e-13
    print('OK' if ok else 'MISMATCH')
