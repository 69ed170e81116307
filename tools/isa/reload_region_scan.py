"""Register-cap reproducer (DESIGN.md \"Register-cap hazard\"): scratch reloads inside an
s_and_saveexec region whose register is read after the region's s_or_b64 exec join, in
straight-line code (stops at the first branch).  Input: a kernel's assembly (-S).

    python tools/isa/reload_region_scan.py kernel.s
"""
import re, sys
L = open(sys.argv[1]).read().split("\n")
def vset(tok):
    tok = tok.strip()
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m: return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    if m: return {int(m.group(1))}
    return set()
def parse(line):
    s = line.split(";")[0].strip()
    if not s or s.startswith(".") or s.endswith(":"): return None, [], s
    p = s.split(None, 1)
    ops = [t.strip() for t in re.split(r",(?![^\[]*\])", p[1])] if len(p) > 1 else []
    return p[0], ops, s
NODEST = ("scratch_store", "global_store", "buffer_store", "ds_write", "flat_store", "global_atomic", "ds_add", "s_")
stack = []
pending = []   # (line, regs, key)
flags = []
for i, l in enumerate(L):
    op, ops, s = parse(l)
    if op is None:
        continue
    m = re.match(r"s_and_saveexec_b64 (s\[\d+:\d+\])", s)
    if m: stack.append((m.group(1), i)); continue
    m = re.match(r"s_or_b64 exec, exec, (s\[\d+:\d+\])", s)
    if m:
        key = m.group(1)
        for k in range(len(stack) - 1, -1, -1):
            if stack[k][0] == key:
                opened = stack[k][1]
                # loads inside [opened, i) become candidates
                for (ln, regs, depth) in list(pending):
                    if ln > opened:
                        flags.append([ln, set(regs), i, key])
                pending = [p for p in pending if p[0] <= opened]
                del stack[k:]
                break
        continue
    if op.startswith("scratch_load") and stack:
        pending.append((i, vset(ops[0]), len(stack)))
# for each flagged load, scan forward from the join: read before write?
for ln, regs, join, key in flags:
    live = set(regs)
    res = []
    for j in range(join + 1, min(join + 3000, len(L))):
        op, ops, s = parse(L[j])
        if op is None: continue
        if op.startswith("s_endpgm"): break
        dst = set()
        srcs = ops
        if ops and not op.startswith(NODEST) and not op.startswith("v_cmp") and not op.startswith("v_readlane"):
            dst = vset(ops[0]); srcs = ops[1:]
        rd = set().union(*[vset(t) for t in srcs]) if srcs else set()
        hit = live & rd
        if hit:
            res.append((j + 1, sorted(hit), s[:70])); live -= hit
        live -= dst
        if not live: break
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            res.append((j + 1, "ctrl", s[:50])); break
    print(f"load@{ln+1} v{sorted(regs)} region {key} joined@{join+1}: {res[:3]}")
