"""Instruction mix per basic block of one kernel in a --save-temps .s file:
    python tools/isa_blocks.py <file.s> <mangled-name-substring> [min-instructions]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
sub = sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 30
name = next(m.group(1) for m in re.finditer(r"^(\S+):(?:\s|$)", s, re.M) if sub in m.group(1) and not m.group(1).startswith('.'))
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
blocks, cur = [], None
for l in s[a:b].split('\n'):
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    t = l.strip()
    if cur and t and not t.startswith(';') and not t.startswith('.'):
        cur[1].append(t)
tot = Counter()
for nm, ins in blocks:
    c = Counter(x.split()[0] for x in ins)
    v = sum(n for k, n in c.items() if k.startswith('v_'))
    if len(ins) >= mn:
        print(nm, len(ins), 'valu', v, 'br:', [x for x in ins if 'branch' in x][-2:])
        print('   ', ', '.join(f'{k}:{n}' for k, n in c.most_common(14)))
