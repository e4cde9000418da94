"""Instructions between consecutive MFMAs in the kernel's loop with the most
MFMAs (a backward branch's target up to the branch):
python tools/isa_gaps.py file.s name"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r'^(_Z[\w]*%s[\w]*):[^\n]*\n(.*?)^\.Lfunc_end' % re.escape(sys.argv[2]), s, re.S | re.M)
lines = [l.strip() for l in m.group(2).splitlines()]
labels = {l.split()[0][:-1]: i for i, l in enumerate(lines) if l.startswith('.LBB') and l.split()[0].endswith(':')}


def ops(seg):
    return [l.split()[0] for l in seg if l and not l.startswith(('.', ';')) and not l.split()[0].endswith(':')]


best = []
for i, l in enumerate(lines):
    if 'branch' in l and l.split()[-1] in labels and labels[l.split()[-1]] < i:
        seq = ops(lines[labels[l.split()[-1]]:i + 1])
        if sum(o.startswith('v_mfma') for o in seq) > sum(o.startswith('v_mfma') for o in best):
            best = seq
out, run = [], []
for op in best:
    if op.startswith('v_mfma'):
        out.append(run)
        run = []
    else:
        run.append(op)
out.append(run)
print('mfma', len(out) - 1, 'instructions', len(best))
for i, r in enumerate(out):
    short = {}
    for op in r:
        k = 'wait' if op.startswith('s_waitcnt') else ('nop' if op == 's_nop' else
            ('vmem' if op.startswith(('global_', 'buffer_')) else ('salu' if op.startswith('s_') else 'valu')))
        short[k] = short.get(k, 0) + 1
    print(i, len(r), short)
