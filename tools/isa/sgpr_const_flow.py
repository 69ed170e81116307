"""Register-cap reproducer (DESIGN.md \"Register-cap hazard\"): forward data flow over a
kernel's disassembly (llvm-objdump -d, with encodings) on its real control-flow graph:
does any v_mul_lo_u32 read SGPR <reg> at a point where it may not hold <const>?

    python tools/isa/sgpr_const_flow.py kernel.s s80 0x846ca68b
"""
import re, sys
L = open(sys.argv[1]).read().split('\n')
REG = sys.argv[2] if len(sys.argv) > 2 else 's80'
CONST = sys.argv[3] if len(sys.argv) > 3 else '0x846ca68b'
rn = int(REG[1:])
ins = []
for l in L:
    m = re.match(r'\s+(\S.*?)\s*//\s*([0-9A-F]+):\s*([0-9A-F ]+)$', l)
    if not m: continue
    text, addr, enc = m.group(1), int(m.group(2), 16), m.group(3).split()
    ins.append((addr, 4 * len(enc), text))
idx = {a: i for i, (a, _, _) in enumerate(ins)}
def covers(tok):
    tok = tok.strip()
    if tok == REG: return True
    m = re.match(r's\[(\d+):(\d+)\]$', tok)
    return bool(m) and int(m.group(1)) <= rn <= int(m.group(2))
def split_ops(t):
    p = t.split(None, 1)
    return p[0], ([x.strip() for x in re.split(r",(?![^\[]*\])", p[1])] if len(p) > 1 else [])
NODST = ('s_cmp', 'ds_write', 'global_store', 'scratch_store', 'buffer_store', 's_cbranch', 's_waitcnt', 's_branch', 's_nop', 's_endpgm', 's_setprio', 's_barrier', 'v_writelane', 's_sleep')
succ = []
for i, (a, sz, t) in enumerate(ins):
    op, ops = split_ops(t)
    s = []
    if op.startswith('s_branch') or op.startswith('s_cbranch'):
        off = int(ops[0]); off = off - 65536 if off > 32767 else off
        tgt = a + 4 + 4 * off
        s.append(idx.get(tgt))
        if op.startswith('s_cbranch'): s.append(i + 1)
    elif op.startswith('s_endpgm'):
        pass
    else:
        s.append(i + 1)
    succ.append([x for x in s if x is not None and x < len(ins)])
# state: 0 = const, 1 = maybe non-const; entry: non-const (unset)
N = len(ins)
state_in = [None] * N
state_in[0] = 1
work = [0]
def transfer(i, st):
    op, ops = split_ops(ins[i][2])
    if ops and not op.startswith(NODST) and covers(ops[0]):
        if op == 's_mov_b32' and ops[1] == CONST: return 0
        return 1
    return st
while work:
    i = work.pop()
    out = transfer(i, state_in[i])
    for j in succ[i]:
        new = out if state_in[j] is None else max(state_in[j], out)
        if new != state_in[j]:
            state_in[j] = new; work.append(j)
bad = 0
for i, (a, sz, t) in enumerate(ins):
    op, ops = split_ops(t)
    srcs = ops[1:] if ops and not op.startswith(NODST) else ops
    if any(covers(x) for x in srcs) and op.startswith('v_mul_lo_u32') and state_in[i] != 0:
        bad += 1
        print(f'maybe-non-const {REG} at {a:x}: {t[:60]}  state={state_in[i]}')
print('instructions', N, 'flagged multiplier reads', bad)
