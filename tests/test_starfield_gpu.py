"""GPU: the starfield program's Draw (starfield/Source/skeleton.cpp:66-79) against
the oracle over a scripted session of frame times (the reference reads them
from SDL_GetTicks)."""
import numpy as np
import pytest

import cgamd
import oracle

pytestmark = pytest.mark.gpu


def test_starfield_frames_match_oracle(ctx):
    a, b = cgamd.starfield_init(1000), oracle.starfield_init(1000)
    for dt in (0.0, 16.0, 17.0, 400.0, 1300.0, 16.0, 2000.0):
        got = ctx.starfield_draw(a)
        ref = oracle.starfield_draw(b)
        assert np.array_equal(got, ref), dt
        assert (got == 0x80FFFFFF).sum() > 100          # stars on screen
        cgamd.starfield_update(a, dt)
        oracle.starfield_update(b, dt)


def test_starfield_other_sizes(ctx):
    s = cgamd.starfield_init(5000)
    for W, H in ((640, 480), (1920, 1080), (7, 5)):
        assert np.array_equal(ctx.starfield_draw(s, W, H), oracle.starfield_draw(s.copy(), W, H))
