"""Per-CU view of scripts/wg_timing.py's lattice records (diagnostic build with hardware ids):
for each CU (XCC, SE, SH, CU from HW_ID), the workgroups it ran, its mean resident count over
the launch's steady middle (10-80 % of the span), and the gap between a workgroup's end and the
next start on the same CU (how long a freed slot stays empty); for a queued launch, the gap
between a workgroup's consecutive tiles.  Usage: wg_slots.py DIR [queued]"""
import glob
import os
import sys

import numpy as np

DIR = sys.argv[1]
US = 0.01
for f in sorted(glob.glob(os.path.join(DIR, "*.npy"))):
    r = np.load(f).astype(np.int64)
    kind = (r[:, 0] >> 56) & 0xFF
    lt = r[kind == 2]
    if not len(lt):
        continue
    hw = (lt[:, 5] >> 24) & 0xFFFFFFFF
    xcc = (lt[:, 5] >> 56) & 0xF
    cu = xcc * 256 + ((hw >> 8) & 0x7F)
    wg = lt[:, 5] & 0xFFFFFF
    t0, t1 = lt[:, 1], lt[:, 2]
    base, span = t0.min(), t1.max() - t0.min()
    lo, hi = base + 0.1 * span, base + 0.8 * span
    gaps, resid = [], []
    grid = np.linspace(lo, hi, 200)
    queued = len(sys.argv) > 2 and sys.argv[2] == "queued"
    for c in np.unique(cu):
        m = cu == c
        s, e = np.sort(t0[m]), np.sort(t1[m])
        resid.append(np.mean([((t0[m] <= g) & (t1[m] > g)).sum() for g in grid]))
        if queued:   # per workgroup: the gap between its consecutive tiles
            for w in np.unique(wg[m]):
                mm = m & (wg == w)
                o = np.argsort(t0[mm])
                a, b = t0[mm][o], t1[mm][o]
                gaps.extend((a[1:] - b[:-1]).tolist())
        else:
            first_end = e[0]
            for x in s[s > first_end]:
                k = np.searchsorted(e, x, side="right") - 1
                gaps.append(x - e[k])
    g = np.array(gaps) * US
    print(f"{os.path.basename(f)[:-4]}: {'queued' if queued else 'grid'} CUs {len(np.unique(cu))}, "
          f"resident mean {np.mean(resid):.2f} (min {np.min(resid):.2f}), "
          f"slot gap median {np.median(g):.2f} us p90 {np.percentile(g, 90):.2f} mean {g.mean():.2f}, "
          f"tiles per CU {len(lt) / len(np.unique(cu)):.0f}")
