import csv, sys, glob, collections
d = sys.argv[1]
agg = collections.defaultdict(list)
durs = {}
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if 'conv' not in r.get('Kernel_Name', ''): continue
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    print(f"{k:28s} mean/dispatch {sum(v)/len(v):16.1f}  n={len(v)}")
