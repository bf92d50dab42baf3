"""Build-time resource check of the hot kernels (no GPU): register spills and
scratch read from the gfx950 code objects' metadata in the built library
(tools/spill_report.py).  Two kernels lost most of their time this round to
SGPR spills (DESIGN.md section 4 "Proposal kernel", section 8); this keeps
the hot path's kernels from regressing silently."""
import os

import pytest

from tools import spill_report as sr

pytestmark = pytest.mark.skipif(
    not os.path.exists(sr.DEFAULT_LIB) or sr.readelf() is None,
    reason="built library or llvm-readelf missing")


@pytest.fixture(scope="module")
def kernels():
    res = sr.kernel_resources()
    dm = sr.demangle(list(res))
    return {sr.kernel_label(dm[k]): v for k, v in res.items()}


def _select(kernels, prefix):
    got = {k: v for k, v in kernels.items() if k.startswith(prefix)}
    assert got, f"no kernel named {prefix}*"
    return got


# (kernel name prefix, max SGPR spills, max VGPR spills, max scratch bytes)
HOT = [
    # the MFMA KDE passes: d = 20 default (pipelined, IB = 3), the d = 8
    # headline form (unpipelined, IB = 4 since round 6: 167 VGPRs, three
    # waves per SIMD) and the d = 5, 6 form (IB = 3; two VGPRs spilled
    # outside the loop to hold four waves per SIMD)
    ("void abc::kde_mfma_lds2g_kernel<2, 7, 3, 2, true, 4>", 0, 0, 0),
    ("void abc::kde_mfma_lds2g_kernel<1, 3, 4, 2, false, 4>", 0, 0, 0),
    ("void abc::kde_mfma_lds2g_kernel<1, 3, 3, 2, false, 4>", 0, 2, 12),
    # LocalTransition density (z form) at every dimension and shape
    ("void abc::lz_kernel<", 0, 0, 0),
    # the MVN proposal (A staged in LDS since round 5: no SGPR spills), and
    # the four-lanes-per-proposal default of round 6 (44-59 VGPRs: eight
    # waves per SIMD)
    ("void abc::propose_philox_kernel<", 0, 0, 0),
    ("void abc::propose_group_kernel<", 0, 0, 0),
    # the kNN default (4 rows per wave): spills outside the tile loop only;
    # the ceiling guards against the round-5 regression (the row pinned to
    # VGPRs, DESIGN.md section 4 "LocalTransition kNN design")
    ("void abc::knn_kernel<6, 1, 4>", 48, 0, 0),
    # the previous population's pack (rows and matrix staged in LDS)
    ("void abc::pack_prev_kernel<", 0, 0, 0),
    # the spatial index's radix sort (round 6, replaces rocPRIM)
    ("abc::rs_", 0, 0, 0),
    # the accepted-row word gathers
    ("abc::gather_words_kernel", 0, 0, 0),
    ("abc::gather_cols_kernel", 0, 0, 0),
] + [
    # the LocalTransition proposal, one instantiation per d <= 8: the
    # Cholesky factor in registers (the runtime-d form kept it in scratch)
    (f"void abc::propose_local_kernel<{d}, true>", 0, 0, 0) for d in range(1, 9)
]


@pytest.mark.parametrize("prefix,sgpr,vgpr,scratch", HOT)
def test_hot_kernel_spills(kernels, prefix, sgpr, vgpr, scratch):
    for name, r in _select(kernels, prefix).items():
        assert r.get("sgpr_spill_count", 0) <= sgpr, (name, r)
        assert r.get("vgpr_spill_count", 0) <= vgpr, (name, r)
        assert r.get("private_segment_fixed_size", 0) <= scratch, (name, r)


def test_report_reads_every_code_object(kernels):
    # one bundle per translation unit with device code; every kernel carries
    # its register counts
    assert len(sr.code_objects(sr.DEFAULT_LIB)) >= 9
    assert len(kernels) > 500
    assert all("vgpr_count" in r and "sgpr_count" in r for r in kernels.values())
