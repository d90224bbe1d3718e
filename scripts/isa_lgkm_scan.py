"""Find `s_waitcnt lgkmcnt(N>0)` issued while scalar-memory loads may be in
flight (gfx9 ISA: SMEM returns out of order, so with an `s_load*` /
`s_buffer_load*` outstanding only lgkmcnt(0) retires a given LDS read).

    python scripts/isa_lgkm_scan.py file.s [...]

Per kernel in a `hipcc --cuda-device-only -S` listing: basic blocks from the
labels and branches, then a forward dataflow over "an SMEM load may be
outstanding" (set by s_load / s_buffer_load, cleared by any wait with
lgkmcnt(0)), joined with OR at block entries until it is stable. Reports every
lgkmcnt(N>0) wait reached with the flag set. Used by tests/test_isa.py on the
default-path kernels and by DESIGN.md §2's account of the round-1 gcn0 bisect.
"""
import re
import sys


def kernels(lines):
    """(name, [lines]) per kernel body of an assembly listing."""
    out, name, body = [], None, []
    for l in lines:
        m = re.match(r"^(_Z\S+):", l)
        if m:
            if name:
                out.append((name, body))
            name, body = m.group(1), []
            continue
        if name:
            body.append(l)
            if re.match(r"^\s+s_endpgm", l) and False:
                pass
            if re.match(r"^\.Lfunc_end", l):
                out.append((name, body))
                name, body = None, []
    if name:
        out.append((name, body))
    return out


def scan_kernel(body):
    """[(line_index, instruction)] of the lgkmcnt(N>0) waits reachable with an SMEM load outstanding."""
    instrs = []   # (idx, text) of instructions and labels
    for i, l in enumerate(body):
        s = l.split(";")[0].strip()
        if s:
            instrs.append((i, s))
    # basic blocks: start at labels and after branches / endpgm
    blocks, cur, labels = [], [], {}
    for i, s in instrs:
        if re.match(r"^\.?\w+:$", s) or re.match(r"^\.LBB\S+:", s):
            if cur:
                blocks.append(cur)
            cur = [(i, s)]
            labels[s.rstrip(":")] = len(blocks)
            continue
        cur.append((i, s))
        if s.startswith("s_branch") or s.startswith("s_cbranch") or s.startswith("s_endpgm") or s.startswith("s_setpc"):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    # successors
    succ = []
    for b, blk in enumerate(blocks):
        last = blk[-1][1]
        ss = []
        m = re.match(r"^s_c?branch\w*\s+(\S+)", last)
        if m and m.group(1) in labels:
            ss.append(labels[m.group(1)])
        if not (last.startswith("s_branch") or last.startswith("s_endpgm") or last.startswith("s_setpc")):
            if b + 1 < len(blocks):
                ss.append(b + 1)
        succ.append(ss)
    entry = [False] * len(blocks)
    changed = True
    while changed:
        changed = False
        for b, blk in enumerate(blocks):
            f = entry[b]
            for _, s in blk:
                if s.startswith("s_load") or s.startswith("s_buffer_load"):
                    f = True
                m = re.search(r"lgkmcnt\((\d+)\)", s)
                if s.startswith("s_waitcnt") and m and int(m.group(1)) == 0:
                    f = False
            for t in succ[b]:
                if f and not entry[t]:
                    entry[t] = True
                    changed = True
    bad = []
    for b, blk in enumerate(blocks):
        f = entry[b]
        for i, s in blk:
            if s.startswith("s_load") or s.startswith("s_buffer_load"):
                f = True
            m = re.search(r"lgkmcnt\((\d+)\)", s)
            if s.startswith("s_waitcnt") and m:
                if int(m.group(1)) == 0:
                    f = False
                elif f:
                    bad.append((i, s))
    return bad


def scan_file(path):
    """{kernel: (n_lgkm_waits, [suspicious waits])} for an assembly listing."""
    lines = open(path).read().split("\n")
    res = {}
    for name, body in kernels(lines):
        n = sum(1 for l in body if "lgkmcnt(" in l and l.strip().startswith("s_waitcnt"))
        res[name] = (n, scan_kernel(body))
    return res


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for k, (n, bad) in scan_file(p).items():
            print(f"{p}: {k}: {n} lgkmcnt waits, {len(bad)} with SMEM outstanding")
            for i, s in bad[:10]:
                print(f"    line {i}: {s}")
