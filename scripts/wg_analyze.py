"""Summarise scripts/wg_timing.py's per-workgroup stamps (gpurun_out/wgt/*.npy, 100 MHz).
Per case: the certificate kernel's span and per-phase medians, the gap to the lattice kernel,
the lattice kernel's span, its workgroups' durations, peak concurrency, the time after the last
workgroup started (the launch tail), and list-scheduling makespans on the peak concurrency for
the observed start order and for longest-first order (the tail an ordering could remove).
Usage: python scripts/wg_analyze.py [DIR] > summary.json"""
import glob
import heapq
import json
import os
import sys

import numpy as np

DIR = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                          "gpurun_out", "wgt")
US = 0.01   # 100 MHz ticks -> us


def makespan(d, slots):
    h = [0.0] * slots
    for x in d:
        t = heapq.heappop(h)
        heapq.heappush(h, t + x)
    return max(h)


def peak_conc(t0, t1):
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    return int(np.max(np.cumsum(ev[:, 1])))


out = {}
for f in sorted(glob.glob(os.path.join(DIR, "*.npy"))):
    r = np.load(f).astype(np.int64)
    kind = (r[:, 0] >> 56) & 0xFF
    res = {}
    base = r[:, 1].min()
    c = r[kind == 1]
    if len(c):
        res["cert"] = {"workgroups": len(c), "span_us": float((c[:, 4].max() - c[:, 1].min()) * US),
                       "wg_us_median": float(np.median(c[:, 4] - c[:, 1]) * US),
                       "wg_us_max": float((c[:, 4] - c[:, 1]).max() * US),
                       "super_us_median": float(np.median(c[:, 2] - c[:, 1]) * US),
                       "phase1_us_median": float(np.median(c[:, 3] - c[:, 2]) * US),
                       "phase2_us_median": float(np.median(c[:, 4] - c[:, 3]) * US),
                       "peak_concurrency": peak_conc(c[:, 1], c[:, 4]),
                       "start_us": float((c[:, 1].min() - base) * US)}
    lt = r[kind == 2]
    if len(lt):
        d = (lt[:, 2] - lt[:, 1]) * US
        order = np.argsort(lt[:, 1], kind="stable")
        slots = peak_conc(lt[:, 1], lt[:, 2])
        span = float((lt[:, 2].max() - lt[:, 1].min()) * US)
        res["lattice"] = {"workgroups": len(lt), "span_us": span,
                          "start_us": float((lt[:, 1].min() - base) * US),
                          "wg_us_mean": float(d.mean()), "wg_us_median": float(np.median(d)),
                          "wg_us_p90": float(np.percentile(d, 90)), "wg_us_max": float(d.max()),
                          "work_us": float(d.sum()), "peak_concurrency": slots,
                          "packed_span_us": float(d.sum() / slots),
                          "tail_after_last_start_us": float((lt[:, 2].max() - lt[:, 1].max()) * US),
                          "sim_observed_order_us": makespan(d[order], slots),
                          "sim_longest_first_us": makespan(np.sort(d)[::-1], slots)}
        if len(c):
            res["gap_cert_end_to_lattice_start_us"] = float((lt[:, 1].min() - c[:, 4].max()) * US)
    out[os.path.basename(f)[:-4]] = res
print(json.dumps(out, indent=1))
