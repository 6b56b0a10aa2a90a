"""Instruction mix of the innermost loops of one kernel in a disassembly
(tools/disasm.sh output).  Usage: python tools/loopmix.py file.dis KERNEL_SUBSTR"""
import re
import sys
from collections import Counter

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split('\n')
starts = [i for i, l in enumerate(lines) if re.match(r'^[0-9a-f]+ <.*>:', l)]
k = [i for i in starts if sub in lines[i]][0]
end = next((i for i in starts if i > k), len(lines))
body = lines[k + 1:end]
ins = []
for l in body:
    m = re.match(r'^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):(.*)$', l)
    if m:
        ins.append((int(m.group(3), 16), m.group(1), m.group(4)))
addr_idx = {a: n for n, (a, _, _) in enumerate(ins)}
# backward branches = loops
loops = []
for n, (a, op, args) in enumerate(ins):
    if op.startswith('s_cbranch') or op == 's_branch':
        m = re.search(r'<.*\+0x([0-9a-f]+)>', args)
        tgt = None
        if m:
            base = int(re.match(r'^([0-9a-f]+)', lines[k]).group(1), 16)
            tgt = base + int(m.group(1), 16)
        if tgt is not None and tgt <= a and tgt in addr_idx:
            loops.append((addr_idx[tgt], n))
print(f"{len(ins)} instructions, {len(loops)} backward branches")
for s, e in loops:
    c = Counter()
    for _, op, _ in ins[s:e + 1]:
        cls = ('valu' if op.startswith('v_') else 'nop' if op == 's_nop' else
               'wait' if op.startswith('s_waitcnt') else 'salu' if op.startswith('s_') else
               'lds' if op.startswith('ds_') else 'vmem' if op.startswith(('global', 'buffer', 'flat')) else op)
        c[cls] += 1
    print(f"loop [{s}:{e}] {e - s + 1} instrs: {dict(c)}")
