"""The CPU restatement's C1 frame time (SURVEY.md 6's reference figure: 268 ms for the
reference's own -O3 build, timed by the survey in its container), repeated in this container:
the band the bench's cpu_baseline is uncertain by.  Writes
profiles/<round>_cpu_restatement_timing.json."""
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import oracle  # noqa: E402

rnd = sys.argv[1] if len(sys.argv) > 1 else "r04"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
oracle.build()
p = oracle.rt_params(320, 256)
oracle.rt_draw(p)                                   # warm
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    oracle.rt_draw(p)
    ts.append(1e3 * (time.perf_counter() - t0))
ts = np.array(ts)
model = platform.processor()
try:
    model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
except (OSError, StopIteration):
    pass
ref = 268.0
rec = {"config": "C1: RT 320x256, f 256, camera (0, 0, -3, 1), 1 thread, -O3 no -march",
       "restatement_ms": {"min": float(ts.min()), "median": float(np.median(ts)), "max": float(ts.max()),
                          "runs": ts.round(2).tolist()},
       "reference_ms_survey": ref,
       "ratio_restatement_over_reference": {"min": float(ts.min() / ref), "median": float(np.median(ts) / ref),
                                            "max": float(ts.max() / ref)},
       "cpu": model,
       "note": "different containers and hosts: the reference figure comes from the survey's container; the "
               "ratio band mixes host speed with code speed, so it bounds rather than certifies the restatement"}
out = os.path.join(ROOT, "profiles", f"{rnd}_cpu_restatement_timing.json")
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec, indent=1))
