"""Summarise rocprofv3 PMC passes (gpurun_out/pmc_<wl>_<CTR>/) into profiles/pmc_summary.json.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE
reads exactly half the bytes of a wide (16 B/lane) streaming read on gfx950, so the corrected
figure doubles it (an upper bound for narrower accesses); WRITE_SIZE is exact for 16-B stores.
"""
import collections, csv, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = {"rt": ["rt_lattice_kernel"], "rast": ["rast_clip_kernel", "rast_setup_kernel", "rast_rows_kernel", "rast_fill_kernel",
                                                 "rast_post_kernel"]}


def per_kernel(wl, ctr):
    path = os.path.join(ROOT, "gpurun_out", f"pmc_{wl}_{ctr}", "pmc_counter_collection.csv")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        agg[name.split("::")[-1]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


path = os.path.join(ROOT, "profiles", "pmc_summary.json")
try:
    out = json.load(open(path))          # keep other sections (e.g. the SQ figures)
except (OSError, ValueError):
    out = {}
out.update({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --steps 20",
            "units": "bytes per launch", "round": sys.argv[1] if len(sys.argv) > 1 else "r01"})
for wl, kernels in DOMINANT.items():
    f, w = per_kernel(wl, "FETCH_SIZE"), per_kernel(wl, "WRITE_SIZE")
    det = {k: {"fetch_kib_raw": f.get(k), "write_kib": w.get(k),
               "hbm_bytes_corrected": (2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024} for k in kernels}
    out.setdefault(wl, {}).update({"kernels": det,
                                   "frames_per_launch": int(os.environ.get("CG_PMC_RT_FRAMES", "32")) if wl == "rt" else 1,
                                   "hbm_bytes_per_launch": sum(d["hbm_bytes_corrected"] for d in det.values())})
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
with open(path, "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps(out, indent=1))
