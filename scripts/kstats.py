"""Print rocprofv3 kernel_stats CSVs compactly: python scripts/kstats.py gpurun_out/prof_*/..."""
import csv, glob, sys
for pat in sys.argv[1:] or ["gpurun_out/prof_*/*_kernel_stats.csv"]:
    for f in sorted(glob.glob(pat)):
        print(f)
        for r in csv.DictReader(open(f)):
            print(f"  {r['Name'][:70]:70s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.2f}")
