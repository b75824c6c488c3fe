import csv, collections, sys
for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in rows:
        k = r['Kernel_Name'].split('(')[0][-40:]
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); cnt[(k, r['Counter_Name'])] += 1
    for k, d in agg.items():
        n = max(cnt[(k, c)] for c in d)
        print(f.split('/')[-2], k, 'dispatches', n)
        print('   ', {c: '%.4g' % (v / n) for c, v in sorted(d.items())})
