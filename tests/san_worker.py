"""Worker for tests/test_sanitizers.py: runs the AVX2 CPU baseline's three
schedules (banded, queue = the reference's span work queue with per-8-px
ZMask spinlocks, rows = the DrawModelOptimizedLines per-row tasks) on small
scenes and checks each frame bit for bit against the scalar restatement.

Run in a child process with the TSan runtime preloaded and
PRK_ORACLE_LIBDIR=oracle/_san/tsan (liborcpu.so built -fsanitize=thread);
the scalar restatement comes from the ordinary oracle/liboracle.so.
TEST INFRASTRUCTURE ONLY."""
import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "oracle"))
sys.path.insert(0, os.path.join(_ROOT, "cpu-renderer_amd"))
import oracle as O  # noqa: E402
from prk import scenes  # noqa: E402


def main():
    assert "_san" in O.cpu_lib()._name, O.cpu_lib()._name
    cases = [
        (scenes.random_soup(300, 128, 128, radius=24, seed=3), 1),
        (scenes.random_soup(400, 160, 96, radius=40, seed=5, centroid_margin=-30), 1),
        (scenes.random_soup(240, 128, 128, radius=20, seed=7), 6),  # whole objects of 6 triangles
    ]
    for sc, tpo in cases:
        ref = O.render(sc, tris_per_object=tpo, winners=False)
        for cpu in ("queue", "rows", "banded"):
            for threads in (3, 8):
                c, z, _, _ = O.render(sc, cpu=cpu, threads=threads, winners=False, tris_per_object=tpo)
                assert (z.view(np.uint32) == ref[1].view(np.uint32)).all(), (cpu, threads, tpo)
                assert (c == ref[0]).all(), (cpu, threads, tpo)
    print("san_worker ok")


if __name__ == "__main__":
    main()
