"""Build-time guard for sqmp_gemm_fq7 (CPU, no GPU needed).

The kernel keeps its weight loads in flight in VGPRs across hand-counted s_waitcnt; the
compiler does not know those registers are still being written, so a spill (or any copy
of them before the wait) would read them early.  Every fq7 kernel variant must therefore
compile with zero VGPR spills (the timing-diagnostic DIAG variants are exempt) and no scratch (the ISA was also checked for copies of the
in-flight registers when the loop structure was written)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(ROOT, "smoothquant-mixedprecision_amd", "csrc", "sqmp_gemm_fq7.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_fq7_kernels_do_not_spill(tmp_path):
    # (the device assembly for the SGPR hazard scan, compiled alongside)
    asm = subprocess.Popen([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                            "-S", "-I", os.path.join(ROOT, "include"), SRC, "-o", str(tmp_path / "fq7.s")],
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I",
                        os.path.join(ROOT, "include"), "-c", SRC, "-o", str(tmp_path / "fq7.o"),
                        "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert asm.wait(timeout=600) == 0
    # no hand-written VMEM instruction reads an SGPR a VALU instruction (a spill restore by
    # v_readlane) wrote fewer than 5 wait states before: the compiler pads only the VMEM
    # instructions it can see (tools/check_asm_sgpr_hazard.py)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_asm_sgpr_hazard as H
    assert H.main(str(tmp_path / "fq7.s")) == 0
    blocks = re.split(r"remark: Function Name: ", r.stderr)
    seen = 0
    for b in blocks[1:]:
        name = b.split()[0]
        # template <DT, GB, TM, J, DIAG>: product kernels only (DIAG = 0)
        m = re.search(r"gemm_fq7_kernelI.*?ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", name)
        if not m or m.group(4) != "0":
            continue
        seen += 1
        spill = int(re.search(r"VGPRs Spill: (\d+)", b).group(1))
        scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", b).group(1))
        assert spill == 0 and scratch == 0, f"{name}: {spill} VGPR spills, {scratch} B scratch"
    assert seen >= 14



@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_h2d_kernels_do_not_spill(tmp_path):
    """sqmp_gemm_h2d holds the next stage's weight planes in VGPRs across hand-counted
    s_waitcnt (as fq7): every variant (COLMAX x TM 128 / 64) compiles without spills or
    scratch, at two waves per SIMD."""
    src = os.path.join(ROOT, "smoothquant-mixedprecision_amd", "csrc", "sqmp_gemm_h2d.hip")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I",
                        os.path.join(ROOT, "include"), "-c", src, "-o", str(tmp_path / "h2d.o"),
                        "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    blocks = re.split(r"remark: Function Name: ", r.stderr)
    seen = 0
    for b in blocks[1:]:
        if "gemm_h2d_kernel" not in b.split()[0]:
            continue
        seen += 1
        spill = int(re.search(r"VGPRs Spill: (\d+)", b).group(1))
        scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", b).group(1))
        vgprs = int(re.search(r"VGPRs: (\d+)", b).group(1))
        assert spill == 0 and scratch == 0 and vgprs <= 256, (b.split()[0], spill, scratch, vgprs)
    assert seen == 4


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_asm_sgpr_hazard_other_kernels(tmp_path):
    """The same inline-asm SGPR hazard scan (tools/check_asm_sgpr_hazard.py) on the other
    sources whose kernels issue hand-written buffer loads / LDS-DMA / stores from asm."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_asm_sgpr_hazard as H
    csrc = os.path.dirname(SRC)
    names = ["sqmp_gemm_f8", "sqmp_gemm_h2d", "sqmp_actquant_lc", "sqmp_gemm_fast",
             "sqmp_gemm_x3"]

    def asm(n):
        out = str(tmp_path / (n + ".s"))
        extra = ["-fno-slp-vectorize"] if n == "sqmp_gemm_f8" else []
        r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                            "-S", *extra, "-I", os.path.join(ROOT, "include"),
                            os.path.join(csrc, n + ".hip"), "-o", out],
                           capture_output=True, text=True, timeout=900)
        return n, r.returncode, out

    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        results = list(ex.map(asm, names))
    for n, rc, out in results:
        assert rc == 0, n
        assert H.main(out) == 0, n


_FIXTURE = """_Z6kernelv:
{body}
.Lfunc_end0:
"""


@pytest.mark.parametrize("body,want", [
    # straight line: a v_readlane restore 2 wait states before an asm buffer_load reading it
    ("  v_readlane_b32 s12, v3, 4\n  s_nop 0\n  ;;#ASMSTART\n"
     "  buffer_load_dword v5, v6, s[8:11], s12 offen\n  ;;#ASMEND", 1),
    # the same padded by s_nop 4 (5 wait states): clean
    ("  v_readlane_b32 s12, v3, 4\n  s_nop 4\n  ;;#ASMSTART\n"
     "  buffer_load_dword v5, v6, s[8:11], s12 offen\n  ;;#ASMEND", 0),
    # the write at the end of a loop body reaches the load at the loop head by the back edge
    (".LBB0_1:\n  ;;#ASMSTART\n  buffer_load_dword v5, v6, s[8:11], s12 offen\n  ;;#ASMEND\n"
     "  s_nop 7\n  s_nop 7\n  v_readfirstlane_b32 s12, v7\n  s_cbranch_scc1 .LBB0_1", 1),
    # a VOP3b carry-out (the second operand) into the load's soffset
    ("  v_add_co_u32 v1, s[12:13], v2, v3\n  ;;#ASMSTART\n"
     "  buffer_load_dword v5, v6, s[8:11], s12 offen\n  ;;#ASMEND", 1),
    # a VGPR-destination VALU op and an SALU write of the register: no hazard
    ("  v_add_co_u32 v1, vcc, v2, v3\n  s_mov_b32 s12, 0\n  ;;#ASMSTART\n"
     "  buffer_load_dword v5, v6, s[8:11], s12 offen\n  ;;#ASMEND", 0),
])
def test_asm_hazard_scan_fixtures(tmp_path, body, want):
    """tools/check_asm_sgpr_hazard.py on synthetic assembly: straight-line and back-edge
    paths, VOP3b carry-out destinations, and the clean cases."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_asm_sgpr_hazard as H
    p = tmp_path / "k.s"
    p.write_text(_FIXTURE.format(body=body))
    assert H.main(str(p)) == want
