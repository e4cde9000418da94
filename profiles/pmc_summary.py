import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
for r in rows:
    k=r['Kernel_Name']
    k=k[k.find('k_'):].split('(')[0] if 'k_' in k else k[:30]
    agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
    cnt[(k,r['Counter_Name'])]+=1
for k,v in agg.items():
    if not k.startswith('k_'): continue
    n=max(cnt[(k,c)] for c in v)
    print(k, n, {c.replace('SQ_',''): f"{x/n:.3g}" for c,x in sorted(v.items())})
