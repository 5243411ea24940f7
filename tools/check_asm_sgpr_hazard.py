"""Scan device assembly (hipcc -S) for the VALU-writes-SGPR -> VMEM-reads-that-SGPR hazard
inside inline asm: the compiler pads its own VMEM instructions (5 wait states) but cannot
see into an asm statement, so a spilled SGPR restored by v_readlane (or a v_readfirstlane /
VOP3 compare result / VOP3b carry-out) just before a hand-written buffer_load/store reaches it
stale.

Every path into an asm VMEM instruction is walked backwards until 5 wait states have passed:
the lexical predecessors, and at a label also the instructions in front of every branch that
targets it (a VALU write at the end of a loop body reaches the loop head's load through the
back edge).  SGPR destinations of a VALU instruction: its first operand (v_readlane,
v_readfirstlane, VOP3 compares with an SGPR sdst) and, for the VOP3b forms (v_add_co_u32,
v_sub_co_u32, v_addc_co_u32, ..., v_div_scale, v_mad_u64_u32), the carry-out / sdst operand.
Usage: check_asm_sgpr_hazard.py file.s [kernel-substring]"""
import re
import sys

NEED = 5
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
VOP3B = re.compile(r"^v_(add|sub|subrev)_co_|^v_(addc|subb|subbrev)_co_|^v_div_scale_|"
                   r"^v_mad_(u64_u32|i64_i32)")
BRANCH = re.compile(r"^s_(branch|cbranch_\w+)$")


def sregs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _operands(s):
    parts = s.split(None, 1)
    return [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []


def valu_sgpr_writes(s):
    """SGPRs a VALU instruction writes (empty for every other instruction)."""
    op = s.split()[0]
    if not op.startswith("v_"):
        return set()
    ops = _operands(s)
    out = set()
    if ops and ops[0].startswith("s"):
        out |= sregs(ops[0])
    if VOP3B.match(op) and len(ops) > 1 and ops[1].startswith("s"):
        out |= sregs(ops[1])
    return out


def parse(path):
    """{kernel: [(kind, text, written, wait_states, in_asm)]}; kind is "LABEL" (text = the
    label) or the opcode."""
    funcs, name, insts, in_asm = {}, None, None, False
    for raw in open(path):
        line = raw.split("//")[0].rstrip("\n")
        if re.match(r"^_Z\S*:", line):
            name, insts = line.split(":")[0], []
            funcs[name] = insts
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
        if not s or s.startswith(";"):
            continue
        if s.endswith(":"):
            insts.append(("LABEL", s[:-1], set(), 0, False))
            continue
        if s.startswith("."):
            continue
        op = s.split()[0]
        ws = int(re.match(r"s_nop (\d+)", s).group(1)) + 1 if op == "s_nop" else 1
        insts.append((op, s, valu_sgpr_writes(s), ws, in_asm))
    return funcs


def hazards(insts):
    """[(writer, reader, wait states)] for every asm VMEM instruction reached by a VALU SGPR
    write within NEED wait states on some path."""
    branches_to = {}
    for i, (kind, text, _, _, _) in enumerate(insts):
        if BRANCH.match(kind):
            ops = _operands(text)
            if ops:
                branches_to.setdefault(ops[-1], []).append(i)
    out = []

    def walk(i, reads, acc, seen, reader):
        # instructions before index i (exclusive), acc wait states already passed
        while i > 0 and acc < NEED:
            i -= 1
            kind, text, written, ws, _ = insts[i]
            if kind == "LABEL":
                for b in branches_to.get(text, []):
                    if (b, acc) not in seen:
                        seen.add((b, acc))
                        # the branch itself takes a wait state before the label
                        walk(b, reads, acc + 1, seen, reader)
                continue
            if written & reads:
                out.append((text, reader, acc))
                return
            acc += ws
            if kind in ("s_branch", "s_endpgm", "s_setpc_b64"):
                return  # no fallthrough into what follows

    for i, (kind, text, _, _, in_asm) in enumerate(insts):
        if in_asm and (kind.startswith("buffer_") or kind.startswith("global_")):
            reads = sregs(text.split(None, 1)[1]) if " " in text else set()
            if reads:
                walk(i, reads, 0, set(), text)
    return out


def main(path, sub=""):
    bad = {}
    for name, insts in parse(path).items():
        if sub not in name:
            continue
        h = hazards(insts)
        if h:
            bad[name] = h
    for k, v in bad.items():
        print(f"{k[:110]}: {len(v)}")
        for w, r, acc in v[:4]:
            print(f"    {w} -> {r} after {acc} wait states")
    print("kernels with hazards:", len(bad))
    return len(bad)


if __name__ == "__main__":
    sys.exit(1 if main(*sys.argv[1:]) else 0)
