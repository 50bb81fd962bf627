"""CPU tests of bench.py's CPU baseline (oracle/prk_cpu_avx.c) — no GPU.

The AVX2 restatement of FillLineOptimized must produce the scalar oracle's
frame bit for bit (z, colour, winners, span statistics) under both schedules:
"banded" (row bands per thread) and "queue" (the reference's producer AET ->
per-span work queue -> workers with the per-8-px ZMask spinlock,
projekt.cpp:3615-3871 / 2211-2237).  Random soups have no exactly equal z at a
pixel, so the queue schedule's order freedom cannot show here.
"""
import numpy as np
import pytest

import oracle as O
from prk import abi, scenes

pytestmark = pytest.mark.skipif(O.cpu_lib() is None, reason="host has no AVX2")


def same(a, b):
    """Equal frames and span statistics.  `writes` (z-test passes) depends on
    the order spans run in, so the queue schedule may count differently."""
    return ((a[0] == b[0]).all() and (a[1].view(np.uint32) == b[1].view(np.uint32)).all()
            and (a[2] == b[2]).all() and a[3]["spans"] == b[3]["spans"]
            and a[3]["span_pixels"] == b[3]["span_pixels"])


@pytest.mark.parametrize("cpu,threads", [("banded", 1), ("banded", 3), ("queue", 1), ("queue", 4), ("rows", 1),
                                         ("rows", 4)])
@pytest.mark.parametrize("seed,R,lights", [(1, 16, 1), (2, 60, 2), (3, 6, 0)])
def test_avx2_baseline_matches_oracle(cpu, threads, seed, R, lights):
    kw = {} if lights == 1 else dict(lights=scenes.LIGHTS_TWO[:lights], ambient=scenes.AMBIENT_TWO)
    s = scenes.random_soup(2000, 256, 192, radius=R, seed=seed, textured=True, **kw)
    assert same(O.render(s, threads=1), O.render(s, threads=threads, cpu=cpu))


def test_avx2_baseline_clipping_and_prior_contents():
    """Triangles over every screen edge (XOffset, right clamp, start/end
    masks) drawn over non-clear prior contents."""
    s = scenes.random_soup(300, 128, 96, radius=70, seed=9, textured=True, centroid_margin=60,
                           z_range=(-3.5, 3.0))
    rng = np.random.default_rng(4)
    col = rng.integers(0, 2**32, (96, 128), dtype=np.uint32)
    z = rng.uniform(-2, 2, (96, 128)).astype(np.float32)
    a = O.render(s, color=col, z=z)
    for cpu, th in (("banded", 2), ("queue", 3), ("rows", 3)):
        assert same(a, O.render(s, color=col, z=z, threads=th, cpu=cpu))


def test_avx2_baseline_bilinear():
    s = scenes.random_soup(1500, 128, 128, radius=20, seed=11, textured=True)
    s.texture.filter = abi.PRK_FILTER_BILINEAR
    assert same(O.render(s), O.render(s, threads=2, cpu="banded"))


@pytest.mark.parametrize("cpu", ["queue", "rows"])
def test_avx2_baseline_whole_objects(cpu):
    """Objects of several triangles (one AET per object, edges of different
    triangles paired into spans): the rows schedule's per-row tasks hold
    several pairs."""
    s = scenes.random_soup(1200, 160, 128, radius=18, seed=21, textured=True)
    ref = O.render(s, tris_per_object=6)
    assert same(ref, O.render(s, tris_per_object=6, threads=3, cpu=cpu))
