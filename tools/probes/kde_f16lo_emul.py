"""numpy emulation: the d > 8 MFMA KDE pass with the lo pieces in f16
instead of bf16 (fewer matrix-pipe cycles per tile).

Current scheme (kde_mfma.hip): y = y1 + y2 + y3 (y1 on the grid g, 8 bits;
y2, y3 bf16), lo = the seven cross products y1.y2, y1.y3, y2.y1, y3.y1,
y2.y2, y2.y3, y3.y2 per dimension + aL + bL: 7D + 4 slots (KL = 9 MFMAs of
K = 16 at D = 20).

f16 scheme: r = y - y1 split as r2 = f16(r), r3 = f16(r - r2) (22 bits
below g/2), the r pieces scaled by 2^10 (r2.r2 by 2^5 on each side) so
every piece that matters is a NORMAL f16 whatever the hardware does with
f16 denormals (emulated here as flushed), lo = y1.r2, y1.r3, r2.y1, r3.y1, r2.r2 per dimension + aL + bL:
5D + 4 slots (KL = 7 at D = 20); e = hi + lo_acc * 2^-10 (one fma on the
VALU in place of the add).  Dropped: r2.r3, r3.r2 (<= g^2 2^-13 each).

Both are emulated with exact products (bf16 x bf16 and f16 x f16 products
are exact in fp32), each 16-slot chunk summed exactly and rounded to fp32,
then added to the fp32 accumulator (the MFMA's chunk rounding), hi exact.
Reported: max / p99 relative error of the row sums sum_j 2^e_ij against
fp64, over rows of the population's own KDE and rows displaced outward.

    python tools/probes/kde_f16lo_emul.py [N] [M] [d]
"""
import json
import math
import sys

import numpy as np

LOG2E = 1.4426950408889634


def bf16(x):
    x = np.asarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def f16(x):
    return np.asarray(x, dtype=np.float64).astype(np.float16).astype(np.float64)


def f16z(x):
    """f16 with subnormals flushed (if the MFMA flushes them)."""
    v = f16(x)
    return np.where(np.abs(v) < 2.0 ** -14, 0.0, v)


def grid(ymax):
    E = math.frexp(ymax)[1] if ymax > 0 else 0
    return max(math.ldexp(1.0, E - 7), 0.015625)


def chunked_fp32(prod, K=16):
    """prod [..., slots]: per 16-slot chunk an exact sum rounded to fp32,
    chunks accumulated in fp32."""
    s = prod.shape[-1]
    acc = np.zeros(prod.shape[:-1], dtype=np.float32)
    for c in range(0, s, K):
        part = prod[..., c:c + K].sum(-1).astype(np.float32)
        acc = (acc + part).astype(np.float32)
    return acc.astype(np.float64)


def split_value(v, G):
    q = np.clip(np.rint(v / G), -8388607, 8388607)
    return q * G, v - q * G


def emulate(yj, lw2, yi, scheme):
    N, D = yj.shape
    if scheme in ("f16n", "f16fold"):
        # norm grid: |y_j| < 2^E -> g = 2^(E - 10), |y1/g| <= 1024 (f16 ints)
        E = math.frexp(np.sqrt((yj ** 2).sum(1)).max())[1]
        g = max(math.ldexp(1.0, E - 10), 2.0 ** -10)
    else:
        g = grid(np.abs(yj).max())
    G = g * g
    if scheme == "f16fold":
        # unscaled f16 pieces, subnormals kept (if the MFMA keeps them)
        y2j = f16(yj - np.rint(yj / g) * g)
        y2i = f16(yi - np.rint(yi / g) * g)
    y1j = np.rint(yj / g) * g
    y1i = np.rint(yi / g) * g
    rj, ri = yj - y1j, yi - y1i
    if scheme == "bf16":
        y2j = bf16(rj); y3j = bf16(rj - y2j)
        y2i = bf16(ri); y3i = bf16(ri - y2i)
        ytj, yti = y1j + y2j + y3j, y1i + y2i + y3i
    elif scheme == "f16fold":
        y2j = f16(rj); y3j = f16(rj - y2j)
        y2i = f16(ri); y3i = f16(ri - y2i)
        ytj, yti = y1j + y2j + y3j, y1i + y2i + y3i
    else:
        # absolute scale 2^10 (the kernel has no g): pieces of r * 2^10
        y2j = f16z(rj * 1024) / 1024
        y3j = f16z((rj - y2j) * 1024) / 1024
        y2i = f16z(ri * 1024) / 1024
        y3i = f16z((ri - y2i) * 1024) / 1024
        ytj, yti = y1j + y2j + y3j, y1i + y2i + y3i
    if scheme == "f16n":
        assert np.abs(y1j / g).max() <= 2048 and np.abs(y1i / g).max() <= 2048
    a = lw2 - (ytj ** 2).sum(1)
    b = -(yti ** 2).sum(1)
    aH, aL = split_value(a, G)
    bH, bL = split_value(b, G)
    if scheme == "bf16":
        aL1 = bf16(aL); aL2 = bf16(aL - aL1)
        bL1 = bf16(bL); bL2 = bf16(bL - bL1)
    elif scheme == "f16fold":
        aL1 = f16(aL); aL2 = f16(aL - aL1)
        bL1 = f16(bL); bL2 = f16(bL - bL1)
    else:
        aL1 = f16z(aL * 1024) / 1024
        aL2 = f16z((aL - aL1) * 1024) / 1024
        bL1 = f16z(bL * 1024) / 1024
        bL2 = f16z((bL - bL1) * 1024) / 1024
    M = yi.shape[0]
    out = np.empty(M)
    for i in range(M):
        hi = 2 * (y1i[i] * y1j).sum(1) + aH + bH[i]     # exact (multiples of G)
        if scheme == "bf16":
            terms = [y2j * 2 * y1i[i], y3j * 2 * y1i[i], y1j * 2 * y2i[i],
                     y1j * 2 * y3i[i], y2j * 2 * y2i[i], y3j * 2 * y2i[i],
                     y2j * 2 * y3i[i]]
        elif scheme == "f16fold":
            terms = [y2j * 2 * y1i[i], y3j * 2 * y1i[i], y1j * 2 * y2i[i],
                     y1j * 2 * y3i[i], f16(y2j) * f16(2 * y2i[i])]
        else:
            # r2.r2 with 2^5 on each side: a side below the f16 normal
            # range is flushed (the hardware's worst case)
            r2r2 = f16z(y2j * 32) * f16z(2 * y2i[i] * 32) / 1024
            terms = [y2j * 2 * y1i[i], y3j * 2 * y1i[i], y1j * 2 * y2i[i],
                     y1j * 2 * y3i[i], r2r2]
        prod = np.stack(terms, -1).reshape(N, -1)
        prod = np.concatenate([prod, np.stack(
            [aL1, aL2, np.full(N, bL1[i]), np.full(N, bL2[i])], -1)], 1)
        if scheme == "f16fold":
            # folded: hi (exact) first, then each 16-slot lo chunk rounded
            # onto the same fp32 accumulator
            acc = hi.astype(np.float32)
            for c in range(0, prod.shape[1], 16):
                acc = (acc.astype(np.float64) + prod[:, c:c + 16].sum(1)
                       ).astype(np.float32)
            t = np.exp2(acc).astype(np.float32)
            out[i] = t.astype(np.float64).sum()
            continue
        if scheme != "bf16":
            prod = prod * 1024.0                 # the scaled accumulator
        lo = chunked_fp32(prod)
        if scheme != "bf16":
            e = (hi + lo / 1024.0).astype(np.float32)   # fma(lo, 2^-10, hi)
        else:
            e = (hi.astype(np.float32) + lo.astype(np.float32)).astype(np.float32)
        t = np.exp2(e.astype(np.float32)).astype(np.float32)
        out[i] = t.astype(np.float64).sum()
    return out


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rng = np.random.default_rng(0)
    h = (4.0 / (N * (d + 2))) ** (1.0 / (d + 4))
    # C5-like: the kernel covariance is h^2 Sigma; at N = 1e6 the whitened
    # spread is 1/h(1e6) -- emulate that spread with N particles
    hs = (4.0 / (1e6 * (d + 2))) ** (1.0 / (d + 4))
    s = math.sqrt(0.5 * LOG2E)
    yj = rng.normal(size=(N, d)) / hs * s
    lw = rng.normal(scale=0.3, size=N)
    lw2 = (lw - lw.max()) * LOG2E
    par = rng.integers(0, N, size=M)
    yi = yj[par] + rng.normal(size=(M, d)) * s
    far = yi[:M // 8] * 1.8                         # rows outward
    yi = np.concatenate([yi, far])
    exact = np.array([np.exp2(lw2 - ((yj - r) ** 2).sum(1)).sum() for r in yi])
    res = {"N": N, "M": len(yi), "d": d, "g_bf16": grid(np.abs(yj).max()),
           "max_abs_y": float(np.abs(yj).max())}
    schemes = sys.argv[4].split(",") if len(sys.argv) > 4 else \
        ["bf16", "f16", "f16n"]
    for scheme in schemes:
        got = emulate(yj, lw2, yi, scheme)
        ok = exact > 2.0 ** -32
        rel = np.abs(got[ok] / exact[ok] - 1)
        res[scheme] = {"max": float(rel.max()), "p99": float(np.quantile(rel, 0.99)),
                       "mean": float(rel.mean())}
        print(scheme, res[scheme], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
