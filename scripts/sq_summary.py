"""Add executed-work figures to profiles/pmc_summary.json from the SQ counter passes of
scripts/profile_round.sh (gpurun_out/sq_<workload>_*/):

  python3 scripts/sq_summary.py KERNEL "gpurun_out/sq_c5_*/sq_counter_collection.csv" SECTION FPL

* sq_kernels[KERNEL]: the dominant kernel's counters per launch, VALU issue fraction and
  wave states (as before);
* frame_sq: every library kernel the profiled frames ran (rt_* / rast_* / jpeg_*), each with
  its executed lane-ops per launch, its launches per launch of KERNEL and its machine-code
  hash, and their sum per frame -- bench.py's `frac_frame` (every kernel's executed VALU
  work over the frame's time).

Per MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8 XCDs; a wave64 FP32 VALU
instruction issues in 2 cycles on a SIMD32; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are
quad-cycles and WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = sys.argv[1] if len(sys.argv) > 1 else "rt_lattice_kernel"
SRC = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "sq_*", "sq_counter_collection.csv")
SECTION = sys.argv[3] if len(sys.argv) > 3 else "rt"
FPL = int(sys.argv[4]) if len(sys.argv) > 4 else 32     # frames per launch of the profiled kernel
SIMDS = 256 * 4
PREFIXES = ("rt_", "rast_", "jpeg_", "star_")


def base_name(k):
    return k.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1].strip()


def code_sha256(kernel):
    """The profiled kernel's machine code identity: gpurun_out/code_sha256.json written on the
    GPU box by scripts/profile_round.sh (the library the counters ran on), else this tree's build."""
    sys.path.insert(0, os.path.join(ROOT, "computer-graphics_amd"))
    import codeobj
    try:
        rec = json.load(open(os.path.join(ROOT, "gpurun_out", "code_sha256.json")))
        if kernel in rec:
            return rec[kernel]
    except (OSError, ValueError):
        pass
    return codeobj.kernel_sha256(kernel)


agg = collections.defaultdict(list)                               # dominant kernel: counter -> values
valu = collections.defaultdict(list)                              # every kernel: SQ_INSTS_VALU per dispatch
for f in sorted(glob.glob(SRC)):
    for r in csv.DictReader(open(f)):
        k = base_name(r["Kernel_Name"])
        if k == KERNEL:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "SQ_INSTS_VALU" and k.startswith(PREFIXES):
            valu[k].append(float(r["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in agg.items()}
cycles = c["GRBM_GUI_ACTIVE"] / 8.0
wave = c["SQ_WAVE_CYCLES"]
sq = {"kernel": KERNEL, "counters_per_launch": c,
      "valu_issue_frac": c["SQ_INSTS_VALU"] * 2.0 / (cycles * SIMDS),
      "valu_lane_ops_per_launch": c["SQ_INSTS_VALU"] * 64,
      "wave_state_frac": {"active": c["SQ_ACTIVE_INST_ANY"] / wave, "issue_stall": c["SQ_WAIT_INST_ANY"] / wave,
                          "waiting": c["SQ_WAIT_ANY"] / wave},
      "frames_per_launch": FPL,
      "code_sha256": code_sha256(KERNEL),
      "note": "valu_issue_frac = SQ_INSTS_VALU x 2 cyc / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)"}
path = os.path.join(ROOT, "profiles", "pmc_summary.json")
out = json.load(open(path))
sec = out.setdefault(SECTION, {})
sqs = sec.setdefault("sq_kernels", {})
sqs[KERNEL] = sq
if SECTION == "rt":
    out["rt"]["sq"] = sq
# the whole frame: each kernel's median lane-ops per dispatch (a first frame's sizing passes
# repeat the list kernels on the same frame) x its dispatches per dispatch of KERNEL.  The
# dispatch ratios come from the longer kernel-trace run of the same workload when there is one
# (gpurun_out/prof_<section>/<section>_kernel_stats.csv: 20+ frames dilute the sizing passes),
# else from the counter passes themselves.
calls = {}
stats = os.path.join(ROOT, "gpurun_out", f"prof_{SECTION}", f"{SECTION}_kernel_stats.csv")
if os.path.exists(stats):
    for r in csv.DictReader(open(stats)):
        calls[base_name(r["Name"])] = int(r["Calls"])
n_dom = calls.get(KERNEL) or len(valu.get(KERNEL, [])) or 1
kern = {}
for k, v in sorted(valu.items()):
    n_k = calls.get(k, len(v)) if calls else len(v)
    kern[k] = {"valu_lane_ops_per_launch": 64.0 * sorted(v)[len(v) // 2],
               "launches_per_frame_launch": max(1, round(n_k / n_dom)), "code_sha256": code_sha256(k)}
per_frame = sum(r["valu_lane_ops_per_launch"] * r["launches_per_frame_launch"] for r in kern.values()) / FPL
sec["frame_sq"] = {"dominant": KERNEL, "frames_per_launch": FPL, "kernels": kern,
                   "valu_lane_ops_per_frame": per_frame,
                   "note": "every library kernel of the profiled frames: SQ_INSTS_VALU x 64 per dispatch x "
                           "dispatches per dispatch of the dominant kernel / frames per dominant launch"}
json.dump(out, open(path, "w"), indent=1)
print(json.dumps({"sq": sq, "frame_valu_lane_ops_per_frame": per_frame,
                  "frame_kernels": {k: round(v["valu_lane_ops_per_launch"] * v["launches_per_frame_launch"] / FPL / 1e9, 3)
                                    for k, v in kern.items()}}, indent=1))
