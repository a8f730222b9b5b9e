"""Checks on the built gfx950 code objects (CPU only: disassembly, no GPU)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "protein-structure-tokenizer_amd", "pst_amd", "_lib")
OBJS = [os.path.join(LIB, f) for f in ("pst_kernels.o", "pst_decode.o", "pst_fsq_aux.o")]


@pytest.mark.skipif(not all(os.path.exists(o) for o in OBJS), reason="libpst objects not built")
def test_no_valu_to_mfma_operand_hazard():
    """hipcc pads the 2 wait states an MFMA needs before reading a VGPR a VALU just wrote, except
    after inline asm. The packed GELU's asm output is an MFMA B operand; tools/mfma_hazard_scan.py
    finds every VALU write followed by an MFMA A/B read of that register too early (round 5: one
    such pair made k_mpnn_q<1,4> compute with stale operands)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_hazard_scan.py")] + OBJS,
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "hazard hits: 0" in out.stdout
