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

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(ROOT, "smoothquant-mixedprecision_amd", "csrc", "sqmp_gemm_fq7.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_fq7_kernels_do_not_spill(tmp_path):
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I",
                        os.path.join(ROOT, "include"), "-c", SRC, "-o", str(tmp_path / "fq7.o"),
                        "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
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
@pytest.mark.parametrize("name,ns,mfma", [("fqt8", "fqt8", 512), ("fqt9", "fqt9", 256)])
def test_one_wave_gemm_accumulators_stay_in_agprs(tmp_path, name, ns, mfma):
    """sqmp_gemm_fqt8 / _fqt9 name their 256 accumulators as literal a[0:255] in asm
    statements that hipcc cannot see into: the compiler must neither spill nor emit a
    v_accvgpr_* of its own (that would land in an accumulator it does not know is live), and
    the kernels must issue every MFMA of 2 x 2 stages (the steady code-stage loop and the
    general one): 128 16x16x32 or 64 32x32x16 per stage."""
    src = os.path.join(ROOT, "smoothquant-mixedprecision_amd", "csrc", f"sqmp_gemm_{name}.hip")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I",
                        os.path.join(ROOT, "include"), "-c", src, "-o", str(tmp_path / "f8.o"),
                        "-save-temps=obj", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    spills = [int(v) for v in re.findall(r"VGPRs Spill: (\d+)", r.stderr)]
    scratch = [int(v) for v in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", r.stderr)]
    assert len(spills) >= 2 and not any(spills) and not any(scratch), r.stderr[-3000:]
    asm = [f for f in os.listdir(tmp_path) if f.endswith(".s") and "gfx950" in f]
    assert asm
    text = open(tmp_path / asm[0]).read()
    kernels = re.split(r"\n(?=_ZN4sqmp4" + ns + r"\w+:)", text)[1:]
    assert len(kernels) >= 2
    for k in kernels:
        inasm, own, n_mfma = False, 0, 0
        for line in k.split("\n"):
            if ";;#ASMSTART" in line:
                inasm = True
            elif ";;#ASMEND" in line:
                inasm = False
            elif "accvgpr" in line and not inasm:
                own += 1
            elif "v_mfma" in line:
                n_mfma += 1
        assert own == 0, "compiler-emitted accumulator moves"
        assert n_mfma == mfma


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
