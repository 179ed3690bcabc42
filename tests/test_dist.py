"""CPU, world_size 2 (gloo): the multi-GPU raytracer's stripe sharding + gather +
unstripe reassembles exactly the single-process frame.  Each rank renders its
shard's rows with the oracle (test infrastructure stands in for the GPU
kernel here; the GPU form is exercised by tests/test_rt_gpu.py and bench.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import cgdist

W, H, F = 96, 64, 64.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, stripe, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "computer-graphics_amd"), os.path.join(root, "oracle")]
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = oracle.rt_params(W, H, F)
        rows = cgdist.shard_row_map(H, rank, world, stripe)
        full = oracle.rt_draw(p).reshape(H, W)
        shard = np.zeros((len(rows), W), np.uint32)
        valid = rows < H
        shard[valid] = full[rows[valid]]
        t = torch.from_numpy(shard.view(np.int32))
        gl = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, gl, dst=0)
        if rank == 0:
            g = np.stack([x.numpy().view(np.uint32) for x in gl])
            frame = cgdist.unstripe_np(g, H, world, stripe)
            q.put(bool(np.array_equal(frame, full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe", [(2, 8), (2, 16)])
def test_stripe_gather_unstripe_gloo(world, stripe):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, stripe, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
        assert pr.exitcode == 0
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("S", [cgdist.DEFAULT_STRIPE, cgdist.LATTICE_STRIPE, 32])
def test_row_maps_partition_the_frame(S):
    for H_ in (64, 256, 1080, 2160, 1001):
        for n in (1, 2, 3, 4, 8):
            rows = np.concatenate([cgdist.shard_row_map(H_, r, n, S) for r in range(n)])
            real = np.sort(rows[rows < H_])
            assert np.array_equal(real, np.arange(H_))
            # equal-size shards, balanced to within one stripe
            sizes = [int((cgdist.shard_row_map(H_, r, n, S) < H_).sum()) for r in range(n)]
            assert max(sizes) - min(sizes) <= S
    # C2 at 8 GPUs: 15-row stripes split 1080 rows exactly (9 stripes per rank)
    assert cgdist.shard_rows(1080, 8, cgdist.LATTICE_STRIPE) * 8 == 1080


# ---- balanced bands (bench.py's default N > 1 layout) ------------------------

def _band_worker(rank, world, port, q):
    """Rank r renders its band (oracle), ranks > 0 send it as RGB24 with gloo
    p2p, rank 0 assembles: == the single-process frame.  Bands come from the
    library's native partition (cg_dist_band_partition) over all-gathered,
    skewed timings, so they are uneven."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "computer-graphics_amd"), os.path.join(root, "oracle")]
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Fb = 40.0   # a focal length at which the scene leaves black columns to crop
        full = oracle.rt_draw(oracle.rt_params(W, H, Fb)).reshape(H, W)
        import cgamd
        # the library's rebalance, as cg_dist_rebalance runs it: every rank
        # contributes its measured per-frame time (skewed here), the times are
        # all-gathered, each rank spreads its time over its band's rows and
        # calls the native partition (cg_dist_band_partition) -- every rank
        # must arrive at the same bands
        eq = cgdist.equal_bands(H, world)
        t = torch.tensor([1.0 + 0.7 * rank, 0.3 if rank == 0 else 0.0], dtype=torch.float64)
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        cost = np.zeros(H)
        for r, (a, n) in enumerate(eq):
            cost[a:a + n] = float(allt[r][0]) / n
        bands = cgamd.band_partition_native(cost, world, np.array([float(x[1]) for x in allt]))
        assert bands == cgdist.rebalance(eq, [float(x[0]) for x in allt], [float(x[1]) for x in allt], H)
        mine_b = torch.tensor([v for b_ in bands for v in b_], dtype=torch.int64)
        allb = [torch.empty_like(mine_b) for _ in range(world)]
        dist.all_gather(allb, mine_b)
        assert all(torch.equal(x, mine_b) for x in allb)
        r0, nr = bands[rank]
        mine = full[r0:r0 + nr].reshape(-1)
        # the RGB24 window: columns the camera can see anything in
        t_, n_, s_ = cgamd.rt_scene()
        c0, c1 = cgamd.frame_columns(t_, n_, s_, 1, cgamd.rt_camera(W, H, Fb))
        cols = c1 - c0
        if rank == 0:
            frames = np.zeros((1, H * W), np.uint32)
            frames[0, r0 * W:(r0 + nr) * W] = mine
            parts = []
            for p in range(1, world):
                buf = torch.empty(bands[p][1] * cols * 3, dtype=torch.uint8)
                dist.recv(buf, src=p)
                parts.append(buf.numpy())
            cgdist.assemble_np(np.concatenate(parts), 3, bands[1:], W, H, 1, frames, col0=c0, cols=cols)
            q.put(bool(np.array_equal(frames[0], full.reshape(-1))) and 0 < cols < W)
        else:
            dist.send(torch.from_numpy(cgdist.pack_rgb24_np(cgdist.window_np(mine, W, c0, cols))), dst=0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_band_p2p_rgb24_assemble_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
        assert pr.exitcode == 0
    assert q.get(timeout=5) is True


def test_band_partition_properties():
    rng = np.random.default_rng(3)
    for H_ in (7, 64, 1080, 2160):
        for n in (1, 2, 3, 8):
            for cost in (np.ones(H_), rng.random(H_) + 0.1, np.linspace(1, 5, H_)):
                o = rng.random(n) * cost.sum() / n * 0.2
                bands = cgdist.band_partition(cost, n, o)
                # contiguous, rank-ordered, covering every row exactly once
                assert bands[0][0] == 0 and sum(nr for _, nr in bands) == H_
                for (a, na), (b, _) in zip(bands, bands[1:]):
                    assert a + na == b
                if H_ >= n:
                    assert all(nr >= 1 for _, nr in bands)
                # makespan within one row's cost of the continuous optimum's lower bound
                span = max(cost[a:a + na].sum() + o[r] for r, (a, na) in enumerate(bands))
                lb = max((cost.sum() + o.sum()) / n, o.max())
                assert span <= lb + cost.max() * 1.0001 + 1e-9
    # equal_bands: tile-aligned boundaries (C2 at 8 GPUs: 135 = 9 lattice tiles)
    assert cgdist.equal_bands(1080, 8, 15) == [(135 * r, 135) for r in range(8)]


def test_rgb24_pack_assemble_roundtrip():
    rng = np.random.default_rng(5)
    Wd, Hd, nf = 24, 10, 3
    frames_ref = (0x80000000 | rng.integers(0, 1 << 24, (nf, Hd * Wd), dtype=np.uint32)).astype(np.uint32)
    bands = [(0, 3), (3, 4), (7, 3)]
    src = np.concatenate([cgdist.pack_rgb24_np(frames_ref[f, a * Wd:(a + n) * Wd])
                          for a, n in bands for f in range(nf)])
    got = cgdist.assemble_np(src, 3, bands, Wd, Hd, nf, np.zeros_like(frames_ref))
    assert np.array_equal(got, frames_ref)


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_native_band_partition_matches_python(nranks):
    """cg_dist_band_partition (the library's rebalance) == cgdist.band_partition."""
    import cgamd
    rng = np.random.default_rng(nranks)
    for H in (1, 5, 64, 1080):
        for _ in range(5):
            cost = rng.random(H) * rng.choice([0.0, 1.0], H, p=[0.3, 0.7])
            ovh = rng.random(nranks) * cost.sum() / nranks * 0.3
            for o in (None, ovh):
                want = cgdist.band_partition(cost, nranks, o)
                got = cgamd.band_partition_native(cost, nranks, o)
                assert got == want, (H, nranks, got, want)
                assert sum(n for _, n in got) == H and got[0][0] == 0
