"""The MFMA rate probe (tools/probes/fp6_mfma_probe.hip) times what it claims: each rate_asm
loop body is exactly 16 MFMAs of the named operand format on the fixed accumulators
a[0:3] .. a[28:31] plus the scalar counter -- no accumulator moves, no s_nop (the compiler
padding that made round 5's builtin loops time the same dependency pattern for e4m3 and
e2m3).  Cross-compiles for gfx950 (no GPU needed)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "probes", "fp6_mfma_probe.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# template argument (mangled) -> (instruction, format modifiers, operand dwords)
FORMATS = {"0": ("v_mfma_scale_f32_16x16x128_f8f6f4", "", 8),
           "2": ("v_mfma_scale_f32_16x16x128_f8f6f4", "cbsz:2 blgp:2", 6),
           "4": ("v_mfma_scale_f32_16x16x128_f8f6f4", "cbsz:4 blgp:4", 4),
           "n1": ("v_mfma_f32_16x16x32_bf16", "", 4)}


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    out = tmp_path_factory.mktemp("probe") / "probe.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", SRC,
                    "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


def _loops(asm):
    out = {}
    for m in re.finditer(r"^_Z8rate_asmIL(i\w+?)EEvPfii:", asm, re.M):
        body = asm[m.start():asm.index(".Lfunc_end", m.start())]
        i = body.index("\n1:")
        j = body.index("s_cbranch_scc1", i)
        lines = [ln.split(";")[0].strip() for ln in body[i + 3:j].split("\n")]
        out[m.group(1)[1:]] = [ln for ln in lines if ln]
    return out


def test_rate_loops_are_pure_mfma(asm):
    loops = _loops(asm)
    assert set(loops) == set(FORMATS), loops.keys()
    for key, (op, mods, nd) in FORMATS.items():
        body = loops[key]
        mf = [ln for ln in body if ln.startswith("v_mfma")]
        rest = [ln for ln in body if not ln.startswith("v_mfma")]
        assert len(mf) == 16, (key, body)
        assert rest == [rest[0], rest[1]] and rest[0].startswith("s_sub_u32") \
            and rest[1].startswith("s_cmp_lg_u32"), (key, rest)
        accs = []
        for ln in mf:
            assert ln.split()[0] == op, (key, ln)
            assert ln.endswith(mods) if mods else ("cbsz" not in ln and "blgp" not in ln), (key, ln)
            ops = [o.strip() for o in ln.split(None, 1)[1].split(",")]
            assert ops[0] == ops[3] and ops[0].startswith("a["), (key, ln)  # C = D, fixed AGPRs
            lo, hi = (int(v) for v in re.match(r"v\[(\d+):(\d+)\]", ops[1]).groups())
            assert hi - lo + 1 == nd, (key, ln)
            accs.append(ops[0])
        # the eight accumulators, each reused only 8 MFMAs later
        assert accs[:8] == [f"a[{4 * i}:{4 * i + 3}]" for i in range(8)] and accs[8:] == accs[:8]
