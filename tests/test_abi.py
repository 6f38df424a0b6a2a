"""The C-ABI library loads and exports every symbol include/geomesa_hip.h declares (no GPU calls)."""
import ctypes
import os
import re

from geomesa_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(_lib.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_path():
    syms = declared_symbols()
    for s in ["gm_z3_index_key", "gm_z3_invert", "gm_z2_index", "gm_xz2_index", "gm_z3_ranges", "gm_xz3_ranges",
              "gm_z3filter_scan", "gm_pip_join"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from geomesa_amd import build
    build.build(verbose=False)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_library_is_gfx950():
    from geomesa_amd import build
    build.build(verbose=False)
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_load_without_gpu_fails_loudly():
    import torch
    import pytest
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.GeomesaHipUnavailable):
        _lib.context()


def test_product_build_refuses_timing_hooks():
    """The GM_JX_* stage-ablation hooks (wrong results by design) cannot reach the shipped library:
    build.py refuses them for its output path (no compile runs), and the product build defines
    GM_PRODUCT_BUILD, under which gm_pip.hip #errors on any of them."""
    import pytest
    from geomesa_amd import build as B
    with pytest.raises(ValueError):
        B.build(defines=("GM_JX_NOBLOB",), verbose=False)
    src = open(os.path.join(ROOT, "geomesa_amd", "csrc", "gm_pip.hip")).read()
    hooks = set(re.findall(r"GM_JX_[A-Z0-9]+", src))
    guard = src[src.index("#if defined(GM_PRODUCT_BUILD)"):src.index("#error")]
    assert hooks and all(h in guard for h in hooks), hooks
