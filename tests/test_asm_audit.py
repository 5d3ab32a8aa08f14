"""The inline-asm hazard audit (tools/asm_audit.py) on the
CPU: hipcc cross-compiles gfx950 assembly here. It must flag both planted
hazards of tests/fixtures/asm_hazard_fixture.hip (an in-flight inline-asm
ds_read destination copied before its retiring s_waitcnt; inline asm reading
an MFMA result without wait states), pass their correct twins, and find no
hazard and no hot-loop spill in any product score_scan_kernel /
mmr_pick_kernel instantiation (csrc/score_scan.h:188-202 ds_read_b128_asm +
lds_wait, csrc/mmr.hip's asm round loop)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import asm_audit  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")


def test_audit_flags_planted_hazards(tmp_path):
    text = asm_audit.compile_asm(os.path.join(ROOT, "tests", "fixtures", "asm_hazard_fixture.hip"),
                                 str(tmp_path / "fx.s"))
    found = {}
    for k in ("planted_bad_inflight", "planted_good_inflight", "planted_bad_mfma",
              "planted_good_mfma"):
        _, haz = asm_audit.audit_text(text, (k,), quiet=True)
        found[k] = haz
    assert len(found["planted_bad_inflight"]) == 1 and "in flight" in found["planted_bad_inflight"][0][3]
    assert len(found["planted_bad_mfma"]) == 1 and "wait states" in found["planted_bad_mfma"][0][3]
    assert not found["planted_good_inflight"] and not found["planted_good_mfma"]


@pytest.mark.parametrize("src", asm_audit.PRODUCT_SOURCES)
def test_product_kernels_have_no_asm_hazards(src, tmp_path):
    text = asm_audit.compile_asm(os.path.join(asm_audit.PKG, "csrc", src + ".hip"),
                                 str(tmp_path / (src + ".s")))
    kernels = [n for f in asm_audit.KERNELS for n, _ in asm_audit.functions(text, f)]
    assert kernels, "no product kernel found in the assembly"
    n_reads = 0
    for f in asm_audit.KERNELS:
        for _, lines in asm_audit.functions(text, f):
            ins = asm_audit.instructions(lines)
            n_reads += sum(1 for (_, mn, _, a) in ins if a and mn.startswith("ds_read"))
    if src.startswith("score_scan"):
        assert n_reads > 0  # the audit saw the inline A-fragment reads
    spills, haz = asm_audit.audit_text(text, quiet=True)
    assert spills == 0
    assert not haz, haz[:3]
