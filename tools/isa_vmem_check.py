"""Scan gfx950 assembly for uses of a vector-memory load's destination VGPRs before an
s_waitcnt vmcnt that retires the load (the hazard hand-counted vmcnt waits can hide if
the compiler moves or reuses an asm load's destination).  Linear scan of each kernel:
every global_/buffer_/flat_ memory op counts in vmcnt in issue order; a load's destination
stays pending until a vmcnt(N) leaves at most N younger ops outstanding; any other
instruction naming a pending VGPR is reported (a younger load into the same destination is
not: loads return in issue order).  Pending state is dropped at compiler
basic-block labels (paths are interleaved in the layout).  usage: isa_vmem_check.py file.s [kernel-substring ...]"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for a, b, c in VREG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def kernels(lines, pats):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and ln.startswith(".Lfunc_end"):
            if any(p in cur for p in pats):
                yield cur, body
            cur = None
            continue
        if cur:
            body.append(ln)


def scan(body):
    out, bad = [], []  # out: outstanding vmem ops in issue order, each (dest regs or empty, line)
    for i, ln in enumerate(body):
        s = ln.split(";")[0].strip()
        if s.startswith(".LBB") and s.endswith(":"):
            # a compiler basic block: its predecessors' outstanding ops are not tracked (the
            # linear layout interleaves paths), so the scan covers straight-line regions --
            # the unrolled K loops, where hand-counted waits live
            out = []
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", s)
            if m:
                n = int(m.group(1))
                while len(out) > n:
                    out.pop(0)
            continue
        pending = set().union(*[d for d, _ in out]) if out else set()
        used = regs(s)
        dest = set()
        if VMEM.match(op) and "load" in op and "_lds" not in op:
            dest = regs(s[len(op):].split(",")[0])
            # a younger load into a pending destination is ordered behind it (vector memory
            # loads return in issue order on gfx9), so only its address operands count
            used -= dest
        if pending & used:
            bad.append((i, s, sorted(pending & used)[:4]))
        if VMEM.match(op):
            out.append((dest, s))
    return bad


DS = re.compile(r"^ds_")
SMEM = re.compile(r"^s_(load|buffer_load|memtime|memrealtime|getpc|dcache)")


def scan_lds(body):
    """The same scan for LDS reads and lgkmcnt: ds_* ops count in lgkmcnt in issue order and
    return in order; a ds_read (or ds_bpermute / ds_swizzle / a returning ds atomic)
    destination stays pending until an lgkmcnt(N) leaves at most N younger ops.  Scalar
    memory ops also count in lgkmcnt but may return out of order: while one is outstanding
    only lgkmcnt(0) retires anything."""
    out, bad = [], []  # (dest regs, is_smem)
    for i, ln in enumerate(body):
        s = ln.split(";")[0].strip()
        if s.startswith(".LBB") and s.endswith(":"):
            out = []
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        if op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", s)
            if m:
                n = int(m.group(1))
                if n == 0:
                    out = []
                elif not any(sm for _, sm in out):
                    while len(out) > n:
                        out.pop(0)
            continue
        pending = set().union(*[d for d, _ in out]) if out else set()
        used = regs(s)
        dest = set()
        is_ds = bool(DS.match(op))
        returns = is_ds and ("read" in op or "bpermute" in op or "swizzle" in op or "rtn" in op)
        if returns:
            dest = regs(s[len(op):].split(",")[0])
            used -= dest
        if pending & used:
            bad.append((i, s, sorted(pending & used)[:4]))
        if is_ds:
            out.append((dest, False))
        elif SMEM.match(op):
            out.append((set(), True))
    return bad


def main():
    lines = open(sys.argv[1]).read().splitlines()
    pats = sys.argv[2:] or ["rmb_"]
    total = 0
    for name, body in kernels(lines, pats):
        bad = scan(body) + scan_lds(body)
        total += len(bad)
        print(f"{name}: {len(body)} lines, {len(bad)} early uses of in-flight load destinations")
        for i, s, r in bad[:10]:
            print(f"  line {i}: {s}   (v{r})")
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
