"""Scan device assembly (hipcc -S) for the VALU-writes-SGPR -> VMEM-reads-that-SGPR hazard
inside inline asm: the compiler pads its own VMEM instructions (5 wait states) but cannot
see into an asm statement, so a spilled SGPR restored by v_readlane (or a v_readfirstlane /
VOP3 compare result) just before a hand-written buffer_load/store reaches it stale.
Usage: check_asm_sgpr_hazard.py file.s [kernel-substring]"""
import re
import sys

NEED = 5
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def sregs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path, sub=""):
    name, insts, in_asm, bad = None, [], False, {}
    for raw in open(path):
        line = raw.rstrip("\n")
        if re.match(r"^_Z\S*:", line):
            name, insts = line.split(":")[0], []
            continue
        if name is None:
            continue
        if line.startswith(".Lfunc_end"):
            name = None
            continue
        s = line.strip()
        if ";;#ASMSTART" in s:
            in_asm = True
            continue
        if ";;#ASMEND" in s:
            in_asm = False
            continue
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            if s.endswith(":"):
                insts.append(("LABEL", set(), 0))   # conservatively reset nothing; labels cost 0
            continue
        op = s.split()[0]
        ws = int(re.match(r"s_nop (\d+)", s).group(1)) + 1 if op == "s_nop" else 1
        written = set()
        if op.startswith("v_") and ("readlane" in op or "readfirstlane" in op or "_e64" in op or op.startswith("v_cmp")):
            dst = s.split(None, 1)[1].split(",")[0].strip() if " " in s else ""
            if dst.startswith("s"):
                written = sregs(dst)
        if in_asm and (op.startswith("buffer_") or op.startswith("global_")) and (sub in name):
            reads = sregs(s.split(None, 1)[1])
            acc = 0
            for pop, pw, pws in reversed(insts[-12:]):
                if pop == "LABEL":
                    continue
                if pw & reads and acc < NEED:
                    bad.setdefault(name, []).append(f"{pop} -> {s} after {acc} wait states")
                    break
                acc += pws
                if acc >= NEED:
                    break
        insts.append((op if op != "s_nop" else s, written, ws))
    for k, v in bad.items():
        print(f"{k[:110]}: {len(v)}")
        for e in v[:4]:
            print("   ", e)
    print("kernels with hazards:", len(bad))
    return len(bad)


if __name__ == "__main__":
    sys.exit(1 if main(*sys.argv[1:]) else 0)
