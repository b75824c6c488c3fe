"""Host-side (CPU) checks of device helper functions, compiled with hipcc and run without a GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_ref_avail_mask_matches_unit_loop(tmp_path):
    """intra.h: ref_avail_mask (analytic, used by intra_prep_kernel) == nb_available_wh per unit,
    exhaustively over CTB sizes, TB sizes/positions, neighbour-CTU flags and picture edges."""
    exe = str(tmp_path / "avail_check")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", os.path.join(ROOT, "tools", "avail_check.hip"), "-o", exe],
                   check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout
