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
    """Timing-variant defines (stage ablations, the reference checks compiled out, the inline-word
    ablations) never reach the shipped library: build.py refuses them for its output path before any
    compile runs, and no product source carries a GM_JX_ hook."""
    import pytest
    from geomesa_amd import build as B
    for d in ("GM_JX_NOBLOB", "GM_NO_REF_CHECKS"):
        with pytest.raises(ValueError):
            B.build(defines=(d,), verbose=False)
    for src in B.sources():
        assert "GM_JX_" not in open(src).read(), src


def test_no_environment_selected_kernel_paths():
    """Which kernel answers a product call is never chosen by the process environment: the library
    reads only diagnostics (GM_PIP_DEBUG) and the host build's thread count; every knob that changes
    a kernel path is a gm_ctx_set_param parameter."""
    csrc = os.path.join(ROOT, "geomesa_amd", "csrc")
    names = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".hpp")):
            names |= set(re.findall(r'getenv\(\s*"([A-Z0-9_]+)"', open(os.path.join(csrc, f)).read()))
            assert "getenv(v)" not in open(os.path.join(csrc, f)).read() or f == "gm_pip_build.hip", f
    assert names <= {"GM_PIP_DEBUG"}, names


def test_header_constants_match_binding():
    """Every GM_PARAM_* / GM_JOIN_* / GM_SPATIAL_* value of the header is the binding's."""
    src = open(_lib.HEADER).read()
    defs = dict((k, int(v)) for k, v in re.findall(r"#define\s+(GM_(?:PARAM|JOIN|SPATIAL)_[A-Z0-9_]+)\s+(-?\d+)", src))
    assert len(defs) >= 12
    for k, v in defs.items():
        assert getattr(_lib, k) == v, k
