"""Static instruction mix of a kernel in a hipcc -S listing:
python tools/isa_mix.py file.s name [name ...]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for name in sys.argv[2:]:
    m = re.search(r'^(_Z[\w]*%s[\w]*):[^\n]*\n(.*?)s_endpgm' % re.escape(name), s, re.S | re.M)
    ins = []
    for l in m.group(2).splitlines():
        t = l.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':') or not l.startswith(('\t', ' ')):
            continue
        ins.append(t.split()[0])
    c = Counter()
    for x in ins:
        if x.startswith('s_waitcnt'):
            c['wait'] += 1
        elif x.startswith('s_') and 'branch' in x:
            c['br'] += 1
        elif x.startswith('s_'):
            c['salu'] += 1
        elif x.startswith('v_'):
            c['valu'] += 1
        else:
            c[x.split('_')[0]] += 1
    print(m.group(1)[:60], len(ins), dict(c))
