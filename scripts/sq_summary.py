"""Add executed-work figures of the RT pixel kernel to profiles/pmc_summary.json from the SQ
counter passes of scripts/pmc_sq.sh (gpurun_out/sq_*/).

Per MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8 XCDs; a wave64 FP32 VALU
instruction issues in 2 cycles on a SIMD32; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are
quad-cycles and WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES.
"""
import collections, csv, glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = sys.argv[1] if len(sys.argv) > 1 else "rt_lattice_kernel"
SRC = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "sq_*", "sq_counter_collection.csv")
SECTION = sys.argv[3] if len(sys.argv) > 3 else "rt"
FPL = int(sys.argv[4]) if len(sys.argv) > 4 else 32     # frames per launch of the profiled kernel
SIMDS = 256 * 4



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


agg = collections.defaultdict(list)
for f in sorted(glob.glob(SRC)):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1] == KERNEL:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
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
sqs = out.setdefault(SECTION, {}).setdefault("sq_kernels", {})
sqs[KERNEL] = sq
if SECTION == "rt":
    out["rt"]["sq"] = sq
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(sq, indent=1))
