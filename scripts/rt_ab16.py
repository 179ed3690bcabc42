"""A/B timing of libcgamd.so variants on the C2 workload as bench.py runs it
(16 frames per cg_rt_render_frames_device call; us_per_frame synchronises
after every call, stream_us_per_frame times 8 calls back to back).  Each variant runs in its own
process (CGAMD_LIB), rounds interleaved; prints the median us per frame and
whether frame 0 equals the golden C2 frame.
usage: python scripts/rt_ab16.py [lib.so ...]   (default: the in-tree build)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, json, hashlib
sys.path[:0] = [{pkg!r}]
import numpy as np, torch, cgamd
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx = cgamd.Context(0); t, n, s = cgamd.rt_scene(); ctx.rt_set_scene(t, n, s, 1)
K = 16
cams = [cgamd.rt_camera(1920, 1080, 1080.0)] * K
buf = torch.zeros(K * 1920 * 1080, dtype=torch.int32, device="cuda")
for _ in range(3): ctx.rt_render_frames_device(cams, buf.data_ptr(), None, st.cuda_stream)
ts = []
for _ in range({reps}):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(st); ctx.rt_render_frames_device(cams, buf.data_ptr(), None, st.cuda_stream); b.record(st)
    b.synchronize(); ts.append(a.elapsed_time(b))
bs = []   # back-to-back calls (what bench.py times): certificates overlap
for _ in range(5):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(8): ctx.rt_render_frames_device(cams, buf.data_ptr(), None, st.cuda_stream)
    b.record(st); b.synchronize(); bs.append(a.elapsed_time(b))
f0 = buf[:1920 * 1080].cpu().numpy().view(np.uint32)
want = json.load(open({golden!r}))["rt"]["rt_1920x1080_f1080"]["argb_sha256"]
print(json.dumps(dict(us_per_frame=float(np.median(ts)) * 1e3 / K, min=float(np.min(ts)) * 1e3 / K,
                      stream_us_per_frame=float(np.median(bs)) * 1e3 / (8 * K),
                      exact=hashlib.sha256(f0.tobytes()).hexdigest() == want)))
"""


def run(lib, reps=30):
    env = dict(os.environ)
    if lib:
        env["CGAMD_LIB"] = os.path.abspath(lib)
    code = CODE.format(pkg=os.path.join(ROOT, "computer-graphics_amd"), reps=reps,
                       golden=os.path.join(ROOT, "tests", "golden", "golden.json"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    if r.returncode:
        return {"lib": lib, "error": r.stderr[-1500:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d["lib"] = lib or "default"
    return d


if __name__ == "__main__":
    libs = sys.argv[1:] or [""]
    for rnd in range(2):
        for lib in libs:
            print(json.dumps(run(lib)), flush=True)
