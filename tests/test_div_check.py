"""The XZ keys' corrected-reciprocal division (gm_keys.hpp div_span / div_time) equals IEEE a / b:
tools/div_check.c at a reduced draw count (the full 2.3e9-quotient run is documented in DESIGN.md §3).
Host-only: x86 fma is IEEE-exact, the same operation the device's v_fma_f64 performs."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_span_division_is_ieee(tmp_path):
    exe = str(tmp_path / "div_check")
    subprocess.check_call(["gcc", "-O2", "-mfma", "-o", exe, os.path.join(ROOT, "tools", "div_check.c"), "-lm"])
    out = subprocess.run([exe, "3000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("bad 0"), out.stdout
