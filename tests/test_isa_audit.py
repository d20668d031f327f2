"""The built gfx950 kernels carry no packed-fp32 op with a high-element op_sel (tools/isa_audit.py; the fused-SE
data-parallel discrepancy of rounds 3-4, profiles/r4_se_dp_rootcause.md).  CPU-only: disassembles build/hip."""
import glob
import os

import pytest

from tools import isa_audit


def _objects():
    return isa_audit.current_objects()


@pytest.mark.skipif(not isa_audit.tools_available() or not _objects(), reason="ROCm LLVM tools or build/hip missing")
def test_no_packed_fp32_op_sel_in_built_kernels():
    bad = isa_audit.audit(_objects())
    assert not bad, "\n".join(f"{o}: {f[:90]}: {i}" for o, f, i in bad[:20])


@pytest.mark.skipif(not isa_audit.tools_available() or not _objects(), reason="ROCm LLVM tools or build/hip missing")
def test_audit_sees_the_se_kernels():
    # the audit must actually be reading code: the SE weight-sum kernel is in se.hip.o's disassembly
    import tempfile
    se = [o for o in _objects() if os.path.basename(o).startswith("se.hip")]
    assert se
    with tempfile.TemporaryDirectory() as tmp:
        text = isa_audit.disassemble(se[0], tmp)
    assert "se_wsum_part_kernel" in text and ("v_fma" in text or "v_pk_fma_f32" in text)
