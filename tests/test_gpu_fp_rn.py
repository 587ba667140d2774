"""The kernel's correctly rounded fp32 helpers (raytracing-clj_amd/csrc/fp_rn.h)
against the compiler's IEEE `1.0f / b` and `sqrtf`, on every one of the 2^32
fp32 inputs on the GPU (tools/fp_rn_exhaustive.hip, built by the package
Makefile as lib/fp_rn_exhaustive).  The kernel's bit-exact contract with the
fp32 mirror rests on these being the same bits everywhere.
"""
import re
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

EXE = Path(__file__).resolve().parent.parent / "raytracing-clj_amd" / "lib" / "fp_rn_exhaustive"


def test_fp_rn_equals_ieee_on_every_input():
    assert EXE.exists(), f"{EXE} missing: run `make -C raytracing-clj_amd`"
    out = subprocess.run([str(EXE)], capture_output=True, text=True, timeout=180, check=True).stdout
    counts = {m.group(1).strip(): int(m.group(2)) for m in re.finditer(r"^(.*?)\s+mismatches (\d+)", out, re.M)}
    for name in ("rcp_rn_normal (2^-126 <= b < 2^126)", "rcp_rn (all 2^32 patterns)",
                 "sqrt_rn (all 2^32 patterns)", "sqrt_rn_normal (2^-96 <= x <= inf)"):
        assert counts.get(name) == 0, (name, out)
    # the checker sees differences where they exist: the bare v_rcp_f32 (1 ulp)
    # and the Newton step outside its range both differ somewhere
    assert counts["v_rcp_f32 alone (positive normals)"] > 0, out
    assert counts["rcp + 1 newton (positive normals)"] > 0, out
