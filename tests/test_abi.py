"""The C-ABI library loads here (no GPU) and exports exactly what include/nais.h declares;
argument validation fails loudly before any device work."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from poi_recommendation_models_amd import build, _capi
    build.build()
    return _capi.load()


def declared():
    src = open(os.path.join(ROOT, "include", "nais.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nais_[a-z0-9_]+)\s*\(", src)))


def test_exports_match_header(lib):
    from poi_recommendation_models_amd import _capi
    names = declared()
    assert set(names) == set(_capi.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r" T (nais_\w+)", out))
    assert set(names) <= exported, set(names) - exported
    # and nothing beyond the header: no A/B entry points left in the product library
    internal = {"nais_internal_fail", "nais_internal_check_launch"}
    assert exported - internal == set(names), exported - internal - set(names)
    for n in names:
        assert hasattr(lib, n)


def test_abi_version_and_struct_layout(lib):
    from poi_recommendation_models_amd import _capi
    assert lib.nais_abi_version() == _capi.ABI_VERSION
    P = _capi.NaisParams
    assert P.num_pois.offset == 24 and P.beta.offset == 40 and P.embed_history.offset == 48
    assert ctypes.sizeof(P) == 48 + 8 * 8


def test_validation_errors_without_device(lib):
    from poi_recommendation_models_amd import _capi
    rc = lib.nais_forward(None, None, 1, 1, 1, None, None, 0, None, None, 0, None, None, 1, None)
    assert rc == -1 and b"params" in lib.nais_last_error()
    p = _capi.NaisParams()
    p.variant, p.embed_dim, p.item_dim, p.din, p.hidden, p.num_pois = 0, 264, 264, 264, 16, 10
    for f in ("embed_history", "embed_target", "w1", "b1", "w2"):
        setattr(p, f, 16)
    rc = lib.nais_forward(p, 16, 1, 1, 1, 16, None, 0, None, None, 0, 16, None, 1, None)
    assert rc == -2 and b"256" in lib.nais_last_error()   # any embed_dim <= 256 (ABI 12)
    p.variant, p.embed_dim, p.item_dim, p.din = 1, 12, 5, 12        # region: item_dim == embed_dim/2
    rc = lib.nais_forward(p, 16, 1, 1, 1, 16, None, 0, None, None, 0, 16, None, 1, None)
    assert rc == -1 and b"region" in lib.nais_last_error()
    p.variant = 0
    p.embed_dim = p.item_dim = p.din = 16
    p.hidden = 0
    rc = lib.nais_forward(p, 16, 1, 1, 1, 16, None, 0, None, None, 0, 16, None, 1, None)
    assert rc == -2 and b"hidden" in lib.nais_last_error()
    p.hidden = 16
    assert lib.nais_score_topk(p, 16, 16, 16, 1, 2000, None, None, None, None, 16, 16, None, None,
                               16, 1 << 30, None) == -2
    assert lib.nais_score_topk(p, 16, 16, 16, 1, 50, None, None, None, None, 16, 16, None, None,
                               None, 0, None) == -4
    assert lib.nais_gather_rows(None, 1, 1, None, 1, None, None) == -1
