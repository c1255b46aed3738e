"""CPU: the engine build's assembly pass (mpc-tsid_amd/csrc/asmpass): the DPP hazard scan,
the nop elision's rules, and the hipcc wrapper end to end on a small kernel."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASMPASS = os.path.join(REPO, "mpc-tsid_amd", "csrc", "asmpass")
sys.path.insert(0, ASMPASS)
import dpp_hazards  # noqa: E402
import nop_elide  # noqa: E402

DPP = "\tv_fmac_f64_dpp v[10:11], v[2:3], v[4:5] row_newbcast:1 row_mask:0xf bank_mask:0xf"


def block(pre):
    """`pre` instructions, then an asm region opening with s_nop 1 whose DPP reads v[2:3]."""
    return pre + ["\t;;#ASMSTART", "\ts_nop 1", DPP, "\t;;#ASMEND", "\ts_endpgm"]


def hazards(lines):
    return [(no, av) for no, s, need, av in dpp_hazards.scan(enumerate(lines, 1)) if av < need]


def test_scan_flags_a_dpp_read_right_after_its_write():
    assert hazards(["\tv_add_f64 v[2:3], v[6:7], v[8:9]", DPP])
    assert hazards(["\tv_add_f64 v[2:3], v[6:7], v[8:9]", "\tv_mov_b32 v20, 0", DPP])
    assert not hazards(["\tv_add_f64 v[2:3], v[6:7], v[8:9]", "\ts_nop 1", DPP])
    assert not hazards(["\tv_add_f64 v[2:3], v[6:7], v[8:9]", "\tv_mov_b32 v20, 0", "\tv_mov_b32 v21, 0", DPP])
    # a write of another register is no hazard
    assert not hazards(["\tv_add_f64 v[6:7], v[6:7], v[8:9]", DPP])


def test_scan_counts_both_operands_of_a_swap_and_the_exec_rule():
    # v_swap_b32 writes both operands (as v_permlane): its second operand is a DPP source here
    assert hazards(["\tv_swap_b32 v20, v2", DPP])
    assert hazards(["\tv_swap_b32 v2, v20", DPP])
    assert not hazards(["\tv_swap_b32 v20, v21", DPP])
    # a VALU write of EXEC needs five wait states before a DPP instruction
    cmpx = "\tv_cmpx_gt_f64_e32 vcc, v[6:7], v[8:9]"
    mov = "\tv_mov_b32 v20, 0"
    assert hazards([cmpx, mov, mov, DPP])
    assert hazards([cmpx, mov, mov, mov, mov, DPP])
    assert not hazards([cmpx, mov, mov, mov, mov, mov, DPP])
    assert not hazards([cmpx, "\ts_nop 4", DPP])


def test_elides_when_nothing_before_writes_the_inputs():
    src = block(["\tv_add_f64 v[2:3], v[6:7], v[8:9]", "\tv_mov_b32 v20, 0", "\tv_mov_b32 v21, 0"])
    out, removed, kept = nop_elide.elide(src)
    assert (removed, kept) == (1, 0)
    assert not hazards(out)


@pytest.mark.parametrize("pre", [
    ["\tv_mov_b32 v20, 0", "\tv_add_f64 v[2:3], v[6:7], v[8:9]"],  # writes the DPP source
    ["\tv_add_f64 v[2:3], v[6:7], v[8:9]", "\tv_mov_b32 v20, 0"],  # one instruction between
    ["\tv_mov_b32 v20, 0", "\tv_rcp_f64_e32 v[4:5], v[6:7]"],  # writes another operand (trans)
    ["\tv_mov_b32 v20, 0", "\tv_mov_b32 v10, 0"],  # writes the accumulator
    ["\tv_mov_b32 v20, 0", ".LBB0_3:                 ; %loop", "\tv_mov_b32 v21, 0"],  # a branch target
    ["\tv_cmpx_gt_f64 s[0:1], v[6:7], v[8:9]", "\tv_mov_b32 v20, 0", "\tv_mov_b32 v21, 0"],  # EXEC write
    ["\tv_mov_b32 v20, 0", "\ts_nop 0"],
    ["\tv_mov_b32 v20, 0", "\ts_cbranch_scc1 .LBB0_4"],
])
def test_keeps_the_nop_when_needed_or_unsure(pre):
    out, removed, kept = nop_elide.elide(block(pre))
    assert (removed, kept) == (0, 1)
    assert out == block(pre)


def test_a_swap_writing_the_dpp_source_keeps_the_nop():
    pre = ["\tv_mov_b32 v20, 0", "\tv_swap_b32 v21, v3"]  # writes v3, half of the DPP source v[2:3]
    out, removed, kept = nop_elide.elide(block(pre))
    assert (removed, kept) == (0, 1)


def test_a_label_is_no_stop_where_the_program_writes_exec_by_valu():
    """A label two instructions back ends the walk only if nothing in the program writes EXEC
    by VALU: a branch from elsewhere could land right after such a write."""
    pre = ["\tv_mov_b32 v20, 0", ".LBB0_3:", "\tv_mov_b32 v21, 0", "\tv_mov_b32 v22, 0"]
    out, removed, kept = nop_elide.elide(block(pre))
    assert (removed, kept) == (1, 0)
    elsewhere = ["\tv_cmpx_gt_f64_e32 vcc, v[6:7], v[8:9]", "\ts_cbranch_execz .LBB0_3"]
    out, removed, kept = nop_elide.elide(elsewhere + block(pre))
    assert (removed, kept) == (0, 1)


def test_an_earlier_asm_region_is_read_as_instructions():
    first = ["\t;;#ASMSTART", "\tv_fmac_f64_dpp v[2:3], v[12:13], v[14:15] row_newbcast:0 row_mask:0xf bank_mask:0xf",
             "\t;;#ASMEND"]
    out, removed, kept = nop_elide.elide(block(first))  # writes the next block's DPP source
    assert (removed, kept) == (0, 1)
    other = ["\t;;#ASMSTART", "\tv_fmac_f64_dpp v[30:31], v[12:13], v[14:15] row_newbcast:0 row_mask:0xf bank_mask:0xf",
             "\tv_fmac_f64_dpp v[32:33], v[12:13], v[14:15] row_newbcast:0 row_mask:0xf bank_mask:0xf", "\t;;#ASMEND"]
    out, removed, kept = nop_elide.elide(block(other))
    assert (removed, kept) == (1, 0)
    assert not hazards(out)


KERNEL = r"""
#include <hip/hip_runtime.h>
__device__ __forceinline__ double bc1(double acc, double v, double g) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(v), "v"(g));
  return acc;
}
__global__ void k(const double* x, double* y) {
  const int l = threadIdx.x;
  double v = x[l] * 3.0, g = x[l + 64], a = 0.0, b = 1.0;
  a = bc1(a, v, g);      // v written just before: the nop stays (or the schedule separates them)
  b = bc1(b, g, v);
  y[l] = a + b;
}
"""


def test_hipcc_wrapper_builds_and_leaves_no_hazard(tmp_path):
    src = tmp_path / "k.hip"
    src.write_text(KERNEL)
    r = subprocess.run([sys.executable, os.path.join(ASMPASS, "hipcc_elide.py"), "-O3", "--offload-arch=gfx950",
                        "-c", "-o", str(tmp_path / "k.o"), str(src)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "0 DPP hazards after" in r.stdout
    assert (tmp_path / "k.o").stat().st_size > 0


def test_shipped_library_has_no_dpp_hazard():
    """The library the GPU runs: its N = 16 and N = 32 engine code objects (the C2 / C3
    kernels) extracted from .hip_fatbin, disassembled, and scanned as the build scanned
    their assembly."""
    import codeobj
    so = os.path.join(REPO, "mpc-tsid_amd", "mpcq", "libmpcq.so")
    if not os.path.exists(so):
        pytest.skip("libmpcq.so not built")
    seen = set()
    for _, code in codeobj.extract(so):
        ns = {n for n in (16, 32) if f"engine_kernelILi{n}E".encode() in code}  # (symbol names)
        if not ns:
            continue
        funcs = codeobj.kernels(codeobj.disassemble(code))
        seen |= ns
        ndpp = 0
        for name, lines in funcs.items():
            found = list(dpp_hazards.scan(lines))
            ndpp += len(found)
            assert all(av >= need for _, _, need, av in found), name
        assert ndpp > 1000  # the solve kernels' v_fmac_f64_dpp chains were scanned
    assert seen == {16, 32}
