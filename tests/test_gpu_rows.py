"""Round-6 data-movement kernels of the hot path, checked against numpy:

* the accepted-row selection (abc_gather_words / abc_gather_cols_words):
  the first-n-by-id population of the reference's samplers
  (sampler/multicore_evaluation_parallel.py:131-132, singlecore.py:19-38)
  gathered straight into column / row blocks of one buffer, bit for bit;
* the spatial index's stable radix sort (abc_radix_sort_pairs_u64, the
  Hilbert-key sort that replaces cKDTree's build, local_transition.py:
  82-83) against numpy's stable argsort, ties and edge sizes included.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.as_tensor(a, device="cuda")


@pytest.mark.parametrize("n,B,d", [(0, 5, 3), (1, 1, 1), (777, 5000, 8),
                                   (4099, 4100, 21)])
def test_gather_words_selection(n, B, d):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels as K
    rng = np.random.default_rng(n + d)
    theta = rng.normal(size=(B, d))
    pid = rng.integers(0, 2 ** 40, size=B).astype(np.int64)
    dist = rng.normal(size=B)
    sel = np.sort(rng.choice(B, n, replace=False)).astype(np.int64)
    # theta and the int64 parent as an extra column of ONE fp64 buffer, at a
    # row offset (a later round's block)
    off = 3
    buf = torch.full((off + n, d + 1), np.nan, dtype=torch.float64,
                     device="cuda")
    K.gather_words(_dev(theta), _dev(sel), n, buf[off:, :d])
    K.gather_words(_dev(pid), _dev(sel), n, buf[off:, d:])
    out = buf.cpu().numpy()
    np.testing.assert_array_equal(out[off:, :d], theta[sel])
    np.testing.assert_array_equal(out[off:, d].view(np.int64), pid[sel])
    assert np.isnan(out[:off]).all()
    dd = torch.empty(n, dtype=torch.float64, device="cuda")
    K.gather_words(_dev(dist), _dev(sel), n, dd)
    np.testing.assert_array_equal(dd.cpu().numpy(), dist[sel])
    # identity (strided copy): the parent column back out as int64
    par = torch.empty((n, 1), dtype=torch.int64, device="cuda")
    K.gather_words(buf[off:, d:], None, n, par)
    np.testing.assert_array_equal(par.cpu().numpy()[:, 0], pid[sel])


@pytest.mark.parametrize("S,B,n", [(100, 3000, 1200), (1, 10, 10), (7, 50, 0)])
def test_gather_cols_selection(S, B, n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels as K
    rng = np.random.default_rng(S + B)
    big = rng.normal(size=(S, B + 17))
    src = _dev(big)[:, :B]                      # a column slice, ld = B + 17
    sel = np.sort(rng.choice(B, n, replace=False)).astype(np.int64)
    out = torch.full((S, n + 5), np.nan, dtype=torch.float64, device="cuda")
    K.gather_cols(src, _dev(sel), n, out[:, 5:])
    o = out.cpu().numpy()
    np.testing.assert_array_equal(o[:, 5:], big[:, sel])
    assert np.isnan(o[:, :5]).all()
    cp = torch.empty((S, n), dtype=torch.float64, device="cuda")
    K.gather_cols(out[:, 5:], None, n, cp)
    np.testing.assert_array_equal(cp.cpu().numpy(), big[:, sel])


@pytest.mark.parametrize("n,end_bit,kind", [
    (1, 60, "random"), (255, 60, "random"), (2048, 60, "random"),
    (2049, 60, "ties"), (200_000, 60, "ties"), (100_003, 64, "random"),
    (65_536, 8, "random"), (300_000, 36, "sorted"), (50_000, 60, "reversed"),
    # either side of the switch from 2 to 8 rounds of keys per block (2^19)
    (524_287, 37, "ties"), (524_288, 60, "random"),
    (4_000_000, 60, "ties")])
def test_radix_sort_stable(n, end_bit, kind):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels as K
    rng = np.random.default_rng(n)
    mask = np.uint64((1 << end_bit) - 1) if end_bit < 64 else \
        np.uint64(0xFFFFFFFFFFFFFFFF)
    if kind == "ties":      # few distinct keys: stability decides the order
        keys = rng.integers(0, 37, size=n).astype(np.uint64) * \
            np.uint64(0x0123456789AB)
    else:
        keys = rng.integers(0, 2 ** 63, size=n, dtype=np.int64).astype(
            np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n).astype(
                np.uint64)
    if kind == "sorted":
        keys = np.sort(keys & mask)
    elif kind == "reversed":
        keys = np.sort(keys & mask)[::-1].copy()
    vals = np.arange(n, dtype=np.int32)
    ko, vo = K.radix_sort_pairs(_dev(keys.view(np.int64)), _dev(vals),
                                end_bit)
    km = keys & mask
    order = np.argsort(km, kind="stable")
    got_v = vo.cpu().numpy()
    np.testing.assert_array_equal(got_v, order.astype(np.int32))
    got_k = ko.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got_k & mask, km[order])
    # the bits above end_bit travel with the key
    np.testing.assert_array_equal(got_k, keys[order])


@pytest.mark.parametrize("d", [1, 2, 3, 5, 8, 9, 12, 17, 20, 23, 31, 32])
def test_propose_group_equals_single_lane(d):
    """The indexed entry's proposal kernel (four lanes per proposal, CDF
    bucket table) against the unindexed entry's one-lane kernel and plain
    binary search: theta, resample indices and support flags bit for bit
    (multivariatenormal.py:87-95 restated in-kernel), an odd B so the last
    group is partial."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels as K
    rng = np.random.default_rng(d)
    N, B = 5000, 70_001
    X = _dev(rng.normal(size=(N, d)))
    w = rng.pareto(1.5, size=N) + 0.01
    cdf = K.resample_cdf(_dev(w / w.sum()))
    tab = K.cdf_index(cdf)
    A = _dev(rng.normal(size=(d, d)) * 0.3)
    lo = _dev(np.full(d, -2.5))
    sc = _dev(np.full(d, 5.0))
    ref = K.propose_philox(X, cdf, A, lo, sc, 11, 3, 12345, B)
    got = K.propose_philox(X, cdf, A, lo, sc, 11, 3, 12345, B, tab=tab)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    assert 0.001 < float(ref[2].float().mean()) < 0.999


@pytest.mark.parametrize("d", [3, 8, 20])
def test_propose_group_support_edges(d):
    """The group kernel forms (theta - lo) / scale only near the support's
    edges; with a zero factor theta = X, so rows placed on, just inside and
    just outside [lo, lo + scale] (and a tiny negative offset whose quotient
    underflows) must get the single-lane kernel's flags bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyabc_amd import kernels as K
    lo = np.linspace(-3.0, 2.0, d)
    sc = np.linspace(0.5, 7.0, d)
    hi = lo + sc
    cand = [lo, hi, np.nextafter(lo, -np.inf), np.nextafter(lo, np.inf),
            np.nextafter(hi, np.inf), np.nextafter(hi, -np.inf),
            lo + sc * (1 - 2.0 ** -21), lo + sc * (1 - 2.0 ** -19),
            lo + sc * 0.5, lo - 1e-300, lo + 1e-300]
    rows = []
    rng = np.random.default_rng(d)
    for _ in range(400):   # mixed rows: each column from a random candidate
        pick = rng.integers(0, len(cand), size=d)
        rows.append(np.array([cand[p][j] for j, p in enumerate(pick)]))
    rows += [c.copy() for c in cand]
    X = _dev(np.array(rows))
    N = X.shape[0]
    cdf = K.resample_cdf(_dev(np.full(N, 1.0 / N)))
    tab = K.cdf_index(cdf)
    A = _dev(np.zeros((d, d)))
    ref = K.propose_philox(X, cdf, A, _dev(lo), _dev(sc), 5, 1, 77, 50_001)
    got = K.propose_philox(X, cdf, A, _dev(lo), _dev(sc), 5, 1, 77, 50_001,
                           tab=tab)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    # theta = X of the drawn row, and the flag the exact quotient gives
    th = got[0].cpu().numpy()
    Xn = np.array(rows)
    np.testing.assert_array_equal(th, Xn[got[1].cpu().numpy()])
    x = (th - lo) / sc
    np.testing.assert_array_equal(got[2].cpu().numpy().astype(bool),
                                  ((x >= 0) & (x <= 1)).all(axis=1))
    frac = float(got[2].float().mean())
    assert 0.0 < frac < 1.0
