"""A/B timing of RT variants in one process (interleaved rounds, median)."""
import os, sys, time, json, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]
import numpy as np
import torch
import cgamd

def run(spec, W=1920, H=1080, F=1080.0, n=50):
    # spec = "<cull mode>[@<libcgamd.so path>]"
    mode, _, lib = str(spec).partition("@")
    env = dict(os.environ, CG_RT_CULL=mode)
    if lib:
        env["CGAMD_LIB"] = os.path.join(ROOT, lib)
    code = f"""
import sys; sys.path[:0]=[{os.path.join(ROOT, 'computer-graphics_amd')!r}]
import torch, numpy as np, cgamd, hashlib, json
st=torch.cuda.Stream(); torch.cuda.set_stream(st)
ctx=cgamd.Context(0); t,n,s=cgamd.rt_scene(); ctx.rt_set_scene(t,n,s,1)
cam=cgamd.rt_camera({W},{H},{F}); buf=torch.zeros({W*H},dtype=torch.int32,device='cuda')
for _ in range(5): ctx.rt_render_device(cam, buf.data_ptr(), None, st.cuda_stream)
ts=[]
for _ in range({n}):
    a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    a.record(st); ctx.rt_render_device(cam, buf.data_ptr(), None, st.cuda_stream); b.record(st); b.synchronize(); ts.append(a.elapsed_time(b))
h=hashlib.sha256(buf.cpu().numpy().tobytes()).hexdigest()
print(json.dumps(dict(spec={spec!r}, med=float(np.median(ts)), min=float(np.min(ts)), sha=h[:16])))
"""
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    return r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-2000:]

if __name__ == "__main__":
    modes = sys.argv[1:] or ["0", "1", "2"]
    for rnd in range(2):
        for m in modes:
            print(run(m), flush=True)
