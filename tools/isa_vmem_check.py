"""Scan gfx950 assembly for uses of an in-flight load's destination VGPRs before the
s_waitcnt that retires the load (the hazard hand-counted vmcnt / lgkmcnt waits can hide if
the compiler moves, spills or reuses an asm load's destination).

Dataflow over the kernel's control-flow graph (since r06; the r05 scanner was linear and
dropped all pending state at every compiler block label, so a hazard that crossed a block
boundary was invisible to it):

* blocks start at labels (compiler `.LBB` labels and the numeric local labels of inline asm,
  `1:` / `s_branch 1b`) and after branches; edges are the branch targets (`s_branch`,
  `s_cbranch_*`) and the fall-through of every block not ending in `s_branch` / `s_setpc` /
  `s_endpgm`;
* vector memory (`scan`): every global_/buffer_/flat_/scratch_ op counts in vmcnt in issue
  order; a load's destination registers carry the number of vector-memory ops issued after
  it ("younger"); `s_waitcnt vmcnt(N)` retires every load with at least N younger ops;
* LDS (`scan_lds`): ds_* ops count in lgkmcnt in issue order, a returning ds op's
  destination is pending the same way; scalar memory ops also count in lgkmcnt but may
  return out of order, so while one may be outstanding only lgkmcnt(0) retires anything;
* at a join the state is the worst case over the predecessors (a register is pending if it
  is pending on any path, with the fewest younger ops of any path); iterated to a fixed point
  (back edges included);
* any instruction naming a pending register is reported (a younger load into a pending
  destination is not: loads return in issue order, so only its address operands count).

usage: isa_vmem_check.py file.s [kernel-substring ...]"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
DS = re.compile(r"^ds_")
SMEM = re.compile(r"^s_(load|buffer_load|memtime|memrealtime|getpc|dcache)")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
CAP = 1 << 10  # younger-op counts saturate here (no wait counter is that wide)


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


# ------------------------------------------------------------------ CFG --
def _items(body):
    """[(kind, text, line index)]: kind 'label' (name made unique for numeric asm labels) or
    'inst'; branch targets of numeric labels resolved to those unique names"""
    raw = []
    for i, ln in enumerate(body):
        s = ln.split(";")[0].strip()
        if not s:
            continue
        m = re.match(r"^([.\w$]+):(.*)$", s)
        if m and not s.startswith("s_"):
            raw.append(["label", m.group(1), i])
            rest = m.group(2).strip()
            if rest:
                raw.append(["inst", rest, i])
            continue
        if s.startswith("."):
            continue  # directive
        raw.append(["inst", s, i])
    # numeric local labels: unique names; "Nb" / "Nf" operands resolved by position
    for k, it in enumerate(raw):
        if it[0] == "label" and it[1].isdigit():
            it[1] = f"{it[1]}@{k}"
    for k, it in enumerate(raw):
        if it[0] != "inst":
            continue
        m = re.match(r"^(s_branch|s_cbranch_\w+)\s+(\d+)([bf])$", it[1])
        if m:
            n, d = m.group(2), m.group(3)
            rng = range(k - 1, -1, -1) if d == "b" else range(k + 1, len(raw))
            tgt = next((raw[j][1] for j in rng if raw[j][0] == "label" and raw[j][1].split("@")[0] == n), None)
            if tgt is not None:
                it[1] = f"{m.group(1)} {tgt}"
    return [tuple(x) for x in raw]


def cfg(body):
    """blocks [(label or None, [(inst, line index)])] and successor lists"""
    items = _items(body)
    blocks, cur = [], None

    def new(label):
        blocks.append((label, []))
        return blocks[-1]

    cur = new(None)
    for kind, text, i in items:
        if kind == "label":
            if not cur[1] and cur[0] is None:
                blocks.pop()  # an empty unlabeled block (after a branch): the label starts it
            cur = new(text)
            continue
        cur[1].append((text, i))
        op = text.split()[0]
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op in ("s_endpgm", "s_setpc_b64"):
            cur = new(None)
    index = {b[0]: k for k, b in enumerate(blocks) if b[0] is not None}
    succ = []
    for k, (label, insts) in enumerate(blocks):
        s = []
        last = insts[-1][0] if insts else ""
        op = last.split()[0] if last else ""
        if op in ("s_branch", ) or op.startswith("s_cbranch"):
            tgt = last.split()[1] if len(last.split()) > 1 else None
            if tgt in index:
                s.append(index[tgt])
        falls = op not in ("s_branch", "s_endpgm", "s_setpc_b64")
        if falls and k + 1 < len(blocks):
            s.append(k + 1)
        succ.append(s)
    return blocks, succ


# ------------------------------------------------------ transfer functions --
def _vm_step(state, s, bad, i):
    """state: {reg: younger vmem ops}; one instruction"""
    op = s.split()[0]
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", s)
        if m:
            n = int(m.group(1))
            for r in [r for r, y in state.items() if y >= n]:
                del state[r]
        return
    used = regs(s)
    dest = set()
    if VMEM.match(op) and "load" in op and "_lds" not in op:
        dest = regs(s[len(op):].split(",")[0])
        used -= dest
    hit = used & state.keys()
    if hit and bad is not None:
        bad.append((i, s, sorted(hit)[:4]))
    if VMEM.match(op):
        for r in state:
            state[r] = min(CAP, state[r] + 1)
        for r in dest:
            state[r] = 0


def _lds_step(state, s, bad, i):
    """state: ({reg: younger lgkm ops}, smem may be outstanding)"""
    pend, smem = state
    op = s.split()[0]
    if op == "s_waitcnt":
        m = re.search(r"lgkmcnt\((\d+)\)", s)
        if m:
            n = int(m.group(1))
            if n == 0:
                pend.clear()
                smem = False
            elif not smem:
                for r in [r for r, y in pend.items() if y >= n]:
                    del pend[r]
        return pend, smem
    used = regs(s)
    dest = set()
    is_ds = bool(DS.match(op))
    if is_ds and ("read" in op or "bpermute" in op or "swizzle" in op or "rtn" in op):
        dest = regs(s[len(op):].split(",")[0])
        used -= dest
    hit = used & pend.keys()
    if hit and bad is not None:
        bad.append((i, s, sorted(hit)[:4]))
    if is_ds or SMEM.match(op):
        for r in pend:
            pend[r] = min(CAP, pend[r] + 1)
        for r in dest:
            pend[r] = 0
        smem = smem or bool(SMEM.match(op))
    return pend, smem


def _merge_map(a, b):
    out = dict(a)
    for r, y in b.items():
        out[r] = min(out.get(r, CAP), y)
    return out


def _dataflow(body, init, step, merge, copy):
    blocks, succ = cfg(body)
    n = len(blocks)
    ins = [None] * n
    ins[0] = init()
    work = [0]
    while work:
        k = work.pop()
        st = copy(ins[k])
        for s, i in blocks[k][1]:
            st = step(st, s, None, i)
        for j in succ[k]:
            m = st if ins[j] is None else merge(ins[j], st)
            if ins[j] is None or m != ins[j]:
                ins[j] = copy(m)
                work.append(j)
    bad = []
    for k in range(n):
        if ins[k] is None:
            continue  # unreachable
        st = copy(ins[k])
        for s, i in blocks[k][1]:
            st = step(st, s, bad, i)
    return sorted(bad)


def scan(body):
    """vector-memory loads vs vmcnt; returns [(line index, instruction, regs)]"""
    def step(st, s, bad, i):
        _vm_step(st, s, bad, i)
        return st
    return _dataflow(body, dict, step, _merge_map, dict)


def scan_lds(body):
    """LDS reads (and scalar memory, out of order) vs lgkmcnt"""
    return _dataflow(body, lambda: ({}, False), _lds_step,
                     lambda a, b: (_merge_map(a[0], b[0]), a[1] or b[1]),
                     lambda st: (dict(st[0]), st[1]))


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
