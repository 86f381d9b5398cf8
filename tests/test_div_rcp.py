"""The shared-reciprocal quotient the device Riccati uses (bmpc_core.h div_rcp): with r = 1 / y
correctly rounded, q0 = x r and q = fma(fma(-q0, y, x), r, q0) is the correctly rounded x / y
(Markstein's theorem), so replacing the column solves' divisions by it keeps every bit.  Checked
here on random pairs by tools/markstein_check.c (the committed run: 2e8 pairs);
the GPU side is covered by the seeded batches being bit-identical before and after the change
(profiles/r06/r06v_*)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_markstein_quotient_equals_ieee_division(tmp_path):
    exe = str(tmp_path / "mk")
    subprocess.check_call(["gcc", "-O2", "-mfma", "-o", exe, os.path.join(REPO, "tools", "markstein_check.c"), "-lm"])
    out = subprocess.check_output([exe, "5000000"], text=True)
    assert "mismatches 0 of 5000000" in out, out
