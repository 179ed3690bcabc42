import csv, glob, collections, sys
kern = sys.argv[1] if len(sys.argv) > 1 else "rt_pixel"
for f in sorted(glob.glob('gpurun_out/sq_*/sq_counter_collection.csv')):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(f"{k:32s} {sum(v)/len(v):16.1f}")
