"""Per-rank render time of each RT sharding on ONE GPU (multi-GPU planning).

For N ranks, every rank's shard is rendered in turn on cuda:0 and timed with
HIP events (median of `reps`); prints max/mean per layout.  Layouts:
  stripeS  -- S-row stripes dealt round-robin (needs the unstripe kernel)
  band     -- one contiguous band per rank (stripe_h = ceil(H/N) rounded up to
              the kernel's tile height): the gather lands in place.
Also times the batched unstripe kernel per frame.
usage: python scripts/shard_balance.py [rt|c4|c5] [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cgamd  # noqa: E402
import cgdist  # noqa: E402
from bench import RT_WORKLOADS  # noqa: E402


def main():
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "rt"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    wl = RT_WORKLOADS[wl_name]
    W, H = wl["W"], wl["H"]
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    ctx = cgamd.Context(0)
    if wl["random"]:
        ctx.rt_set_scene(cgamd.random_scene(wl["random"], 0x5EED), wl["random"], None, 0)
    else:
        t, n, s = cgamd.rt_scene()
        ctx.rt_set_scene(t, n, s, 1)
    cam = cgamd.rt_camera(W, H, wl["F"])
    lights = cgamd.area_lights(None, *wl["area"]) if wl["area"] else cgamd.default_lights()

    K = int(os.environ.get("CG_BAL_FRAMES", "1"))   # frames per render call (batched launch)
    buf = torch.zeros(K * (W * H + 64 * W), dtype=torch.int32, device="cuda")

    def time_shard(shard):
        """Device time per frame of this shard, K frames per call."""
        def call():
            if K == 1:
                ctx.rt_render_device(cam, buf.data_ptr(), shard, st.cuda_stream, lights)
            else:
                ctx.rt_render_frames_device([cam] * K, buf.data_ptr(), shard, st.cuda_stream, lights)
        for _ in range(3):
            call()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            call()
            b.record(st)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts)) * 1e3 / K

    tile = wl["stripe"]
    res = {"workload": wl_name, "frames_per_call": K, "whole_us": time_shard(None)}
    for N in (2, 4, 8):
        band = -(-(-(-H // N)) // tile) * tile
        for name, S in ((f"stripe{tile}", tile), ("band", band)):
            us = [time_shard(cgamd.RtShard(r, N, S)) for r in range(N)]
            res[f"N{N}_{name}"] = {"per_rank_us": [round(x, 1) for x in us],
                                   "max_over_mean": max(us) / float(np.mean(us)), "max_us": max(us)}
    # the batched unstripe kernel, per frame (K = 8 frames, N = 8)
    N, KU, S = 8, 8, tile
    rows = cgdist.shard_rows(H, N, S)
    g = torch.zeros(N * KU * rows * W, dtype=torch.int32, device="cuda")
    fr = torch.zeros(KU * H * W, dtype=torch.int32, device="cuda")
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        ctx.rt_unstripe_batch_device(g.data_ptr(), W, H, N, S, KU, fr.data_ptr(), st.cuda_stream)
        b.record(st)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    res["unstripe_us_per_frame"] = float(np.median(ts)) * 1e3 / KU
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
