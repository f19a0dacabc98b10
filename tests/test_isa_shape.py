"""The hot kernels' register allocation, pinned (CPU test).

The fused cfg-2 kernel and the long-horizon kernel are held in shape by empty-asm register
steering points (29 `asm volatile("")` in solve_big.hip / solve_wave.hip / solve_phases.h) and by
code placement: DESIGN.md records that edits outside the ADMM loop move its register assignment
by +-1 %, and spills or `v_readlane` reloads that appeared only on the GPU.  This test reads the
code objects that ship in python-mpc_amd/osqp_amd/libmpcqp.so (tests/isa_shape.py) and fails when
any of the recorded shapes moves:

* VGPR / AGPR counts, spilled VGPRs, the scratch bytes per lane (12 B on cfg 2, 20 B on cfg 5:
  the callee-saved spill lanes of the out-of-line phases; 44 B with 5 spilled VGPRs on the
  slack layouts' eliminated-column kernel), SGPR spills at most the recorded count;
* the ADMM loop: its instruction count, its workgroup barriers, no scratch access, and its
  `v_readlane` count (none in the four-wave loops);
* k_solve_b's two-sided sweep steps: no `v_readlane` and no scratch access in them.

An intended change to these kernels updates the numbers here (`python tests/isa_shape.py`
prints them) together with the same-box A/B that justified it.
"""
import os

import pytest

import isa_shape

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "python-mpc_amd", "osqp_amd", "libmpcqp.so")

PINNED = {
    "cfg2": dict(vgpr_count=256, agpr_count=0, vgpr_spill_count=0, private_segment_fixed_size=12, sgpr_spill_max=185,
                 loop=dict(instructions=197, barriers=4, readlane=0, scratch=0)),
    "cfg3": dict(vgpr_count=256, agpr_count=0, vgpr_spill_count=5, private_segment_fixed_size=44, sgpr_spill_max=212,
                 loop=dict(instructions=233, barriers=4, readlane=0, scratch=0)),
    # cfg 5, round 6: the LDS factorisation chain and the unrolled Gauss-Jordan rows moved the
    # callee-saved spill lanes of factorize2_nl (12 -> 20 B, once per factorisation) and the
    # loop's register assignment (1617 -> 1606 instructions, 46 -> 39 v_readlane); same-box
    # A/Bs 251.6 k -> 254.7 k -> 266.7 k solves/s (profiles/r6/lchain_ab.txt, gj_unroll_ab.txt)
    "cfg5": dict(vgpr_count=254, agpr_count=0, vgpr_spill_count=0, private_segment_fixed_size=20, sgpr_spill_max=238,
                 loop=dict(instructions=1606, barriers=21, readlane=39, scratch=0),
                 step_readlane=0, step_scratch=0),
    # cfg 5's persistent form (round 6, the batch path: the instance body inside the work loop,
    # the lane id and the parameter block laundered per instance -- 29 spilled VGPRs without):
    # v_readlane reloads of one spilled 64-bit scalar in the sweep steps, no scratch access in
    # them; 294.2 k against the plain kernel's 275 k a launch (no dispatcher wait,
    # profiles/r6/dispatch.txt).  Pinned so that a change that makes it worse shows
    "cfg5p": dict(vgpr_count=256, agpr_count=0, vgpr_spill_count=0, private_segment_fixed_size=20,
                  sgpr_spill_max=232, loop=dict(instructions=1659, barriers=21, readlane=90, scratch=0),
                  step_readlane=50, step_scratch=0),
}


@pytest.fixture(scope="module")
def shapes():
    if not isa_shape.tools_present():
        pytest.skip("ROCm LLVM tools (llvm-objcopy, clang-offload-bundler, llvm-readelf, llvm-objdump) absent")
    if not os.path.exists(LIB):
        pytest.skip("libmpcqp.so not built")
    return isa_shape.report(LIB, isa_shape.HOT)


@pytest.mark.parametrize("key", sorted(PINNED))
def test_hot_kernel_shape_is_pinned(shapes, key):
    got, want = shapes[key], PINNED[key]
    for f in ("vgpr_count", "agpr_count", "vgpr_spill_count", "private_segment_fixed_size"):
        assert got[f] == want[f], (key, f, got[f], want[f], got["symbol"])
    assert got["sgpr_spill_count"] <= want["sgpr_spill_max"], (key, got["sgpr_spill_count"])
    assert got["loop"] == want["loop"], (key, got["loop"], want["loop"])
    if "step_readlane" in want:
        assert got["step_loops"] >= 8, got  # the forward / backward step runs of the sweep were found
        assert got["step_readlane"] == want["step_readlane"] and got["step_scratch"] == want["step_scratch"], got


@pytest.mark.skipif(not isa_shape.tools_present() or not os.path.exists(LIB), reason="no llvm tools or library")
def test_wide_setup_has_no_spills():
    """The wide batch setup (setup_wide.h, round 6): every instantiation of k_setup_wide keeps its
    registers -- the 512-thread form at most 128 VGPRs (two instances per CU) with no spilled
    VGPR (8 spilled VGPRs cost 4.5 % of its time: profiles/r6/setup_ab.txt item 8), the 1024-thread
    form at most 128 (one workgroup of 16 waves per CU)."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        md = {}
        for co in isa_shape.code_objects(LIB, d):
            md.update({k: v for k, v in isa_shape.metadata(co).items() if "k_setup_wide" in k})
    assert len(md) == 6, sorted(md)
    for name, v in md.items():
        assert v["vgpr_spill_count"] == 0, (name, v)
        assert v["sgpr_spill_count"] <= 32, (name, v)  # (SGPR spills go to VGPR lanes: 26 in the 512 form)
        assert v["vgpr_count"] + v["agpr_count"] <= 128, (name, v)
