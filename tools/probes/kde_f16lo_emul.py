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
    if scheme in ("f16n", "f16fold", "f16foldS", "f16foldR", "f16loA", "f16loB",
                  "f16foldX"):
        # norm grid: |y_j| < 2^E -> g = 2^(E - 10), |y1/g| <= 1024 (f16 ints)
        E = math.frexp(np.sqrt((yj ** 2).sum(1)).max())[1]
        g = max(math.ldexp(1.0, E - 10), 2.0 ** -10)
    else:
        g = grid(np.abs(yj).max())
    G = g * g
    if scheme in ("f16fold", "f16foldR", "f16loA", "f16loB"):
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
    elif scheme == "f16foldX":
        # r2 unscaled (normal), r3 carried x 2^10 against y1 x 2^-10 (both
        # exact, normal or exact subnormal)
        y2j = f16(rj); y3j = f16((rj - y2j) * 1024) / 1024
        y2i = f16(ri); y3i = f16((ri - y2i) * 1024) / 1024
        ytj, yti = y1j + y2j + y3j, y1i + y2i + y3i
    elif scheme in ("f16fold", "f16foldR", "f16loA", "f16loB"):
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
    if scheme in ("f16n", "f16foldS"):
        assert np.abs(y1j / g).max() <= 2048 and np.abs(y1i / g).max() <= 2048
    a = lw2 - (ytj ** 2).sum(1)
    b = -(yti ** 2).sum(1)
    aH, aL = split_value(a, G)
    bH, bL = split_value(b, G)
    if scheme == "bf16":
        aL1 = bf16(aL); aL2 = bf16(aL - aL1)
        bL1 = bf16(bL); bL2 = bf16(bL - bL1)
    elif scheme in ("f16fold", "f16foldR", "f16loA", "f16loB"):
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
        elif scheme in ("f16fold", "f16foldR", "f16loA", "f16loB", "f16foldX"):
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
        if scheme in ("f16loA", "f16loB"):
            # chunk-aligned, lo chunks first (pure lo, onto 0), then the hi
            # chunks onto them: A = y1.y1[0:16] | y1.y1[16:] aH aH bH bH,
            # B = aH aH bH bH y1.y1[0:12] | y1.y1[12:]
            qa = np.rint(aH / G); qb = np.rint(bH[i] / G)
            qa0 = np.trunc(qa / 2048) * 2048; qb0 = np.trunc(qb / 2048) * 2048
            ab = np.stack([qa0 * G, (qa - qa0) * G, np.full(N, qb0 * G),
                           np.full(N, (qb - qb0) * G)], -1)
            yy = 2 * y1i[i] * y1j
            if scheme == "f16loA":
                h0 = yy[:, :16]; h1 = np.concatenate([yy[:, 16:], ab], 1)
            else:
                h0 = np.concatenate([ab, yy[:, :12]], 1); h1 = yy[:, 12:]
            acc = np.zeros(N, dtype=np.float32)
            for c in range(0, prod.shape[1], 16):
                acc = (acc.astype(np.float64) + prod[:, c:c + 16].sum(1)
                       ).astype(np.float32)
            for h in (h0, h1):
                acc = (acc.astype(np.float64) + h.sum(1)).astype(np.float32)
            out[i] = np.exp2(acc).astype(np.float32).astype(np.float64).sum()
            continue
        if scheme == "f16foldR":
            # packed slots, lo first: the 5D + 4 lo slots, then the D + 4 hi
            # slots (y1.y1 per dimension, aH x2, bH x2), 16-slot chunks
            # rounded onto one fp32 accumulator starting from 0
            qa = np.rint(aH / G); qb = np.rint(bH[i] / G)
            qa0 = np.trunc(qa / 2048) * 2048; qb0 = np.trunc(qb / 2048) * 2048
            hiv = np.concatenate([2 * y1i[i] * y1j, np.stack(
                [qa0 * G, (qa - qa0) * G, np.full(N, qb0 * G),
                 np.full(N, (qb - qb0) * G)], -1)], 1)
            allp = np.concatenate([prod, hiv], 1)
            acc = np.zeros(N, dtype=np.float32)
            for c in range(0, allp.shape[1], 16):
                acc = (acc.astype(np.float64) + allp[:, c:c + 16].sum(1)
                       ).astype(np.float32)
            out[i] = np.exp2(acc).astype(np.float32).astype(np.float64).sum()
            continue
        if scheme == "f16foldS":
            # folded in units of 2^-10: hi (exact, x 2^10) first, then each
            # 16-slot chunk of the scaled lo products rounded onto the same
            # fp32 accumulator; e = acc * 2^-10 (exact)
            allp = np.concatenate([prod * 1024.0], 1)
            acc = (hi * 1024.0).astype(np.float32)
            # merged slots: hi fills D + 4 slots, the lo slots follow
            nh = (D + 4) % 16
            first = 16 - nh if nh else 0
            cuts = [0, first] + list(range(first + 16, allp.shape[1], 16))
            cuts = sorted(set(c for c in cuts if c < allp.shape[1])) + [allp.shape[1]]
            for c0, c1 in zip(cuts[:-1], cuts[1:]):
                if c1 > c0:
                    acc = (acc.astype(np.float64) + allp[:, c0:c1].sum(1)
                           ).astype(np.float32)
            t = np.exp2((acc * np.float32(2.0 ** -10)).astype(np.float32)).astype(np.float32)
            out[i] = t.astype(np.float64).sum()
            continue
        if scheme in ("f16fold", "f16foldX"):
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
    if len(sys.argv) > 5:      # force the grid: one particle at this norm
        yj[0] *= float(sys.argv[5]) / np.sqrt((yj[0] ** 2).sum())
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
