"""Loops of a kernel in a hipcc -S listing and their instruction mix:
python tools/isa_loops.py file.s name"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
m = re.search(r'^(_Z[\w]*%s[\w]*):[^\n]*\n(.*?)^\.Lfunc_end' % re.escape(sys.argv[2]), s, re.S | re.M)
lines = m.group(2).splitlines()
labels = {l.strip()[:-1]: i for i, l in enumerate(lines) if l.strip().startswith('.LBB') and l.strip().endswith(':')}


def ops(seg):
    return [x.strip().split()[0] for x in seg
            if x.strip() and not x.strip().startswith(('.', ';')) and not x.strip().endswith(':')]


print(m.group(1), 'instructions', len(ops(lines)))
for i, l in enumerate(lines):
    t = l.strip()
    if 'branch' in t:
        tgt = t.split()[-1]
        if tgt in labels and labels[tgt] < i:
            o = ops(lines[labels[tgt]:i + 1])
            c = Counter(o)
            print('loop', tgt, 'instructions', len(o))
            print('  ', sorted(c.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30])
