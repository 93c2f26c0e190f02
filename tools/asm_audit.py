"""Audit of the inline-asm LDS reads in the device assembly (cdna_hip_programming.md "What hipcc does not do",
item 1: an asm load's VGPR destination counts as written at ;;#ASMEND, so the compiler may read, copy, spill or
reuse it before the data lands).

Per function of a hipcc -S output: the basic blocks and their successors (labels, branches, fall-through), then a
forward dataflow of the outstanding inline-asm ds_reads (destination register ranges, oldest first): an asm
block's ds_read adds one, its `s_waitcnt lgkmcnt(N)` retires all but the N youngest (LDS reads complete in
order).  Any compiler-generated instruction that names a register of an outstanding read -- a read, a copy, a
write -- on any path is a violation (this covers a rewrite hoisted above an MFMA that reads the old fragment:
that MFMA would name an outstanding read's registers).  Alongside, the MFMAs' SrcA/B registers: an asm ds_read
that rewrites them fewer than MFMA_GAP wait states after the MFMA, with no s_barrier between, is a violation too.
Every distinct state is propagated (the states are finite: capped lists).  Prints one line per function with asm
reads and exits 1 on any violation.

usage: python tools/asm_audit.py build/dkg_kernels.s [more.s ...]
"""
import re
import sys

# An asm ds_read may rewrite an MFMA's SrcA/B registers only MFMA_GAP wait states after that MFMA on every path, or
# after an s_barrier (the MFMA must have read them: the hazard recognizer does not see inline asm).  Wait states
# counted: an MFMA 4 (one pass), s_nop N N + 1, any other instruction 1.
MFMA_GAP = 16


def wait_states(ins):
    if ins.startswith("v_mfma"):
        return 4
    m = re.match(r"s_nop\s+(\d+)", ins)
    return int(m.group(1)) + 1 if m else 1
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.LBB[\w.]+|\.Ltmp[\w.]*):")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return frozenset(out)


def functions(path):
    """(name, [(line number, kind, payload)]): kind 'label', 'asm' (list of asm lines), 'ins' (text)."""
    fn, items, inasm, block = None, [], False, []
    for ln, raw in enumerate(open(path), 1):
        s = raw.strip()
        if re.match(r"^_Z\w+:", raw):
            if fn:
                yield fn, items
            fn, items = raw.split(":")[0], []
            continue
        if fn is None:
            continue
        if s.startswith(".Lfunc_end"):
            yield fn, items
            fn, items = None, []
            continue
        m = LABEL.match(raw)
        if m:
            items.append((ln, "label", m.group(1)))
            continue
        if s == ";;#ASMSTART":
            inasm, block = True, []
            continue
        if s == ";;#ASMEND":
            inasm = False
            items.append((ln, "asm", block))
            continue
        code = s.split(";", 1)[0].strip()
        if inasm:
            if code:
                block.append(code)
            continue
        if not code or code.startswith("."):
            continue
        items.append((ln, "ins", code))
    if fn:
        yield fn, items


def audit_fn(items):
    # basic blocks: split at labels and after branches
    blocks, cur, names = [], [], {}
    for it in items:
        if it[1] == "label":
            if cur:
                blocks.append(cur)
            cur = []
            names[it[2]] = len(blocks)
            cur.append(it)
            continue
        cur.append(it)
        if it[1] == "ins" and re.match(r"s_(c?branch|setpc|endpgm)", it[2]):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    # label names may start a block that follows a branch-ended one: re-index
    names = {}
    for i, b in enumerate(blocks):
        if b and b[0][1] == "label":
            names[b[0][2]] = i
    succ = []
    for i, b in enumerate(blocks):
        s = []
        last = b[-1] if b else None
        if last and last[1] == "ins":
            op = last[2].split()[0]
            if op.startswith("s_branch") or op.startswith("s_cbranch"):
                tgt = last[2].split()[-1]
                if tgt in names:
                    s.append(names[tgt])
            if op.startswith("s_branch") or op.startswith("s_endpgm") or op.startswith("s_setpc"):
                succ.append(s)
                continue
        if i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    nreads = sum(sum(1 for x in it[2] if x.startswith("ds_read")) for b in blocks for it in b if it[1] == "asm")
    if nreads == 0:
        return 0, 0, [], []
    # state: (outstanding asm reads, recent MFMA SrcA/B reads as (registers, line, wait states since))
    seen = {0: {((), ())}}
    work = [(0, ((), ()))]
    viol, close = {}, {}
    steps = 0
    while work and steps < 200000:
        steps += 1
        i, (p0, m0) = work.pop()
        pend, mf = list(p0), list(m0)
        for ln, kind, pay in blocks[i]:
            if kind == "asm":
                for ins in pay:
                    m = re.match(r"s_waitcnt\s+lgkmcnt\((\d+)\)", ins)
                    if m:
                        keep = int(m.group(1))
                        pend = pend[len(pend) - keep:] if 0 < keep < len(pend) else ([] if keep == 0 else pend)
                    elif ins.startswith("ds_read"):
                        dst = regs(ins.split(None, 1)[1].split(",")[0])
                        for r, mln, since in mf:
                            if r & dst and since < MFMA_GAP:
                                close[(ln, mln)] = ins
                        pend.append((dst, ln))
                    elif ins.startswith("s_barrier"):
                        mf = []
                        continue
                    ws = wait_states(ins)
                    mf = [(r, mln, min(since + ws, MFMA_GAP)) for r, mln, since in mf if since < MFMA_GAP]
                continue
            if kind != "ins":
                continue
            if pend:
                if re.match(r"s_waitcnt\b.*lgkmcnt\(0\)", pay):  # a compiler wait retires everything
                    pend = []
                else:
                    used = regs(pay)
                    for dst, aln in pend:
                        if used & dst:
                            viol[(ln, aln)] = pay
            if pay.startswith("s_barrier"):
                mf = []
                continue
            ws = wait_states(pay)
            mf = [(r, mln, min(since + ws, MFMA_GAP)) for r, mln, since in mf if since < MFMA_GAP]
            if pay.startswith("v_mfma"):
                ops = [o.strip() for o in pay.split(None, 1)[1].split(",")]
                mf.append((regs(ops[1]) | regs(ops[2]), ln, 0))
        out = (tuple(pend[-16:]), tuple(mf))  # (lgkmcnt counts at most 15 outstanding LGKM operations)
        for j in succ[i]:
            if out not in seen.setdefault(j, set()):
                seen[j].add(out)
                work.append((j, out))
    return nreads, len(viol), sorted(viol.items()), sorted(close.items())


def main():
    total = 0
    for p in sys.argv[1:]:
        for fn, items in functions(p):
            nreads, nviol, viol, close = audit_fn(items)
            if nreads:
                print(f"{fn}: {nreads} inline-asm LDS reads, {nviol} instructions naming an outstanding read's "
                      f"registers, {len(close)} rewrites within {MFMA_GAP} wait states of an MFMA reading them")
                for (ln, aln), ins in viol[:10]:
                    print(f"  {p}:{ln}: `{ins}` before the wait of the ds_read at line {aln}")
                for (ln, mln), ins in close[:10]:
                    print(f"  {p}:{ln}: `{ins}` rewrites operands of the MFMA at line {mln}")
                total += nviol + len(close)
    print("asm audit:", "OK" if total == 0 else f"{total} violations")
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
