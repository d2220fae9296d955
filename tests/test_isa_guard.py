"""The built libsesa carries no packed-fp32 instruction with a source op_sel (tools/isa_guard.py): on gfx950 those
return wrong values while another wave on the CU executes MFMAs -- the root cause of the rounds 4-5 cross-stream
discrepancy.  CPU-only: disassembles the in-tree library's gfx950 code objects."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
LIB = os.path.join(REPO, "sesa-audio-separation_amd", "sesa", "_native", "libsesa.so")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built libsesa and the ROCm LLVM tools")
def test_no_packed_fp32_op_sel():
    import isa_guard
    n, hits = isa_guard.scan(LIB)
    assert n >= 8, "expected one gfx950 code object per HIP translation unit"
    assert not hits, f"{len(hits)} v_pk_*_f32 with op_sel, e.g. {hits[:3]}"
