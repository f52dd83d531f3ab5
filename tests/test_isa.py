"""ISA check of the hand-counted vmcnt / lgkmcnt waits in the rmb kernels (csrc/enc_gemm.hip).

rmb_front3 / trans4 issue their K-loop loads (weight fragments, depthwise taps,
prefetches, LDS-DMA) as asm statements and retire them with counted s_waitcnt vmcnt(N).
The compiler does not know those loads are in flight: if it moved or reused a
destination register before the covering wait, the kernel would read (or clobber) a
value still being loaded, and only some code generations would show it.  This test
compiles the file for gfx950 and runs both scans of tools/isa_vmem_check.py (vector memory
vs vmcnt, LDS vs lgkmcnt) over each kernel's control-flow graph: no instruction may name a
pending load's destination VGPRs on any path.  The r05 front variant that faulted on the GPU
(tools/exp/enc_gemm_r05_prio_variant.hip.txt) is compiled the same way and must be flagged:
its X prefetch load into v0 is still in flight when the compiler copies v0 away and reuses it
(DESIGN.md §5).  CPU only (hipcc cross-compiles); skipped without hipcc.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import isa_vmem_check as IC  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"


def test_scanner_flags_an_early_use():
    body = ["\tglobal_load_dwordx4 v[4:7], v[0:1], off",
            "\tglobal_load_dwordx4 v[8:11], v[0:1], off offset:1024",
            "\ts_waitcnt vmcnt(1)",
            "\tv_add_f32_e32 v12, v4, v5",      # v[4:7] retired by vmcnt(1): fine
            "\tv_add_f32_e32 v13, v8, v9",      # v[8:11] still in flight: reported
            "\ts_waitcnt vmcnt(0)",
            "\tv_add_f32_e32 v14, v8, v9"]
    bad = IC.scan(body)
    assert [b[0] for b in bad] == [4]
    # an ALU write into a pending destination is reported; a younger load into it is not
    # (loads return in issue order), but one addressed through a pending register is
    assert IC.scan(["\tglobal_load_dword v3, v[0:1], off", "\tv_mov_b32_e32 v3, 0"])
    assert not IC.scan(["\tglobal_load_dword v3, v[0:1], off", "\tscratch_load_dword v3, off, off offset:4"])
    assert IC.scan(["\tglobal_load_dword v0, v[0:1], off", "\tglobal_load_dword v3, v[0:1], off"])
    # LDS reads against lgkmcnt: in-order retirement, and nothing retires but lgkmcnt(0) while a
    # scalar load (out of order) is outstanding
    lds = ["\tds_read_b128 v[4:7], v0", "\tds_read_b128 v[8:11], v0 offset:1024", "\ts_waitcnt lgkmcnt(1)",
           "\tv_mfma_f32_16x16x32_bf16 v[20:23], v[12:15], v[4:7], v[20:23]",
           "\tv_mfma_f32_16x16x32_bf16 v[24:27], v[12:15], v[8:11], v[24:27]"]
    assert [b[0] for b in IC.scan_lds(lds)] == [4]
    assert not IC.scan_lds(lds[:2] + ["\ts_waitcnt lgkmcnt(0)"] + lds[3:])
    assert IC.scan_lds(["\tds_read_b32 v4, v0", "\ts_load_dword s4, s[0:1], 0x0", "\ts_waitcnt lgkmcnt(1)",
                        "\tv_add_f32_e32 v5, v4, v4"])


def test_scanner_follows_control_flow():
    """Pending loads cross compiler block labels (the r05 scanner dropped them there): along a
    fall-through edge, along a taken branch, and around a loop's back edge; at a join the worst
    predecessor counts.  A wait on every path clears them."""
    ld = "\tglobal_load_dword v3, v[0:1], off"
    # fall-through into a labelled block
    assert IC.scan([ld, ".LBB0_1:", "\tv_mov_b32_e32 v3, 0"])
    # conditional branch: the load is pending on both edges; the taken one uses it
    body = [ld, "\ts_cbranch_scc1 .LBB0_2", "\ts_waitcnt vmcnt(0)", "\ts_branch .LBB0_3",
            ".LBB0_2:", "\tv_mov_b32_e32 v4, v3", ".LBB0_3:", "\ts_endpgm"]
    assert [b[0] for b in IC.scan(body)] == [5]
    body[4:6] = [".LBB0_2:", "\ts_waitcnt vmcnt(0)", "\tv_mov_b32_e32 v4, v3"]
    assert not IC.scan(body)
    # join: one path retires the load, the other does not -> pending after the join
    join = [ld, "\ts_cbranch_scc1 .LBB0_2", "\ts_waitcnt vmcnt(0)", ".LBB0_2:", "\tv_mov_b32_e32 v3, 1"]
    assert [b[0] for b in IC.scan(join)] == [4]
    # loop: a load at the bottom of the body is pending at the top on the next iteration
    loop = [".LBB0_1:", "\tv_add_f32_e32 v5, v3, v3", ld, "\ts_cbranch_scc1 .LBB0_1", "\ts_endpgm"]
    assert [b[0] for b in IC.scan(loop)] == [1]
    # inline asm numeric labels (rf2_wait's poll loop): resolved, and its lgkmcnt(0) clears LDS reads
    poll = ["\tds_read_b128 v[4:7], v0", "1:", "\tds_read_b32 v9, v8", "\ts_waitcnt lgkmcnt(0)",
            "\ts_cbranch_scc1 2f", "\ts_sleep 1", "\ts_branch 1b", "2:", "\tv_mov_b32_e32 v10, v4"]
    assert not IC.scan_lds(poll)
    assert IC.scan_lds(poll[:1] + ["\tv_mov_b32_e32 v10, v4"] + poll[1:])


def _compile_asm(tmp_path, src_file, out_name):
    src = os.path.join(REPO, "a-lightweight-unsupervised-feature-extractor-_amd", "csrc")
    # the sources include ../../include/trk_amd.h: mirror that layout
    c = tmp_path / "p" / "c"
    if not c.exists():
        shutil.copytree(src, c, ignore=shutil.ignore_patterns("build", "*.o"))
        shutil.copytree(os.path.join(REPO, "include"), tmp_path / "include")
    if src_file != "enc_gemm.hip":
        shutil.copy(src_file, c / "variant.hip")
        src_file = "variant.hip"
    asm = tmp_path / out_name
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "--offload-device-only", "-S", "-o", str(asm),
                    src_file], cwd=c, check=True, capture_output=True)
    return asm.read_text().splitlines()


@pytest.mark.timeout(900)
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_rmb_kernels_wait_before_using_asm_loads(tmp_path):
    lines = _compile_asm(tmp_path, "enc_gemm.hip", "enc_gemm.s")
    found = 0
    for name, body in IC.kernels(lines, ["rmb_front3_kernel", "trans4_kernel"]):
        found += 1
        bad = IC.scan(body)
        assert not bad, (name, bad[:5])
        bad = IC.scan_lds(body)
        assert not bad, (name, bad[:5])
    assert found == 3  # rmb_front3 (with and without the fragment read-ahead) + trans4
    # no VGPR spills in the two register-bound kernels (the faulting r05 variant spilled 14)
    text = "\n".join(lines)
    for k in ("rmb_front3_kernel", "trans4_kernel"):
        meta = [m for m in re.finditer(r"\.name:\s+\S*" + k + r"\S*(.*?)\.vgpr_spill_count:\s+(\d+)", text, re.S)]
        assert meta, k
        assert all(int(m.group(2)) == 0 for m in meta), (k, [m.group(2) for m in meta])
    # the r05 variant that faulted in one of three pipeline runs: the scan must flag it.  Its X
    # prefetch (`global_load_dword v0` under `tid < 288`, issued before the depthwise) is still
    # pending when the compiler, out of registers, copies v0 to v157 and loads v0 with another
    # value; the prefetch then lands in v0 over that value
    var = _compile_asm(tmp_path, os.path.join(REPO, "tools", "exp", "enc_gemm_r05_prio_variant.hip.txt"),
                       "variant.s")
    name, body = next(IC.kernels(var, ["rmb_front3_kernel"]))
    bad = IC.scan(body)
    assert bad, "the scanner misses the r05 variant's hazard"
    assert all(re.match(r"v_mov_b32_e32 v\d+, v\d+$", s) for _, s, _ in bad), bad
