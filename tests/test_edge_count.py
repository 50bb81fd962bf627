"""The drop-in header's inline edge count (include/prk_edge_count.h).

projekt.h's FillEdgeTable returns the reference's visible-edge count
(projekt.cpp:3882-4121, 4119) from prk_tri_edge_count_sse, the three vertices
projected side by side in SSE lanes; libprk_hip.so's prk_fill_edge_count loops
over the scalar prk_tri_edge_count (pinned to the oracle by
test_abi.test_fill_edge_count_matches_oracle).  Here both are compiled into one
program, built the way a caller might build the drop-in (plain -O2, and -O2
-march=haswell -ffp-contract=fast where FMA contraction is allowed), and must
agree triangle for triangle -- and with the library -- on a soup with
back-facing and degenerate triangles, near-plane vertices, horizontal edges
and extreme magnitudes.
"""
import os
import subprocess

import numpy as np
import pytest

import prk

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHECK_SRC = r"""
#include <cstdio>
#include <vector>
#include "prk_edge_count.h"
int main(int argc, char **argv) {
    FILE *f = std::fopen(argv[1], "rb");
    float cam[5], P[3];
    unsigned n = 0;
    if (std::fread(cam, 4, 5, f) != 5 || std::fread(P, 4, 3, f) != 3 || std::fread(&n, 4, 1, f) != 1) return 2;
    std::vector<float> v(9 * (size_t)n + 3);
    if (std::fread(v.data(), 4, 9 * (size_t)n, f) != 9 * (size_t)n) return 2;
    std::fclose(f);
    prk_transform T = {cam[0], cam[1], cam[2], {cam[3], cam[4]}};
    FILE *o = std::fopen(argv[2], "wb");
    for (unsigned t = 0; t < n; ++t) {
        const float *p = v.data() + 9 * (size_t)t;
        unsigned r[2] = {prk_tri_edge_count(p, P[0], P[1], P[2], &T),
                         prk_tri_edge_count_sse(_mm_loadu_ps(p), _mm_loadu_ps(p + 4), _mm_load_ss(p + 8), P[0],
                                                P[1], P[2], &T)};
        std::fwrite(r, 4, 2, o);
    }
    std::fclose(o);
    return 0;
}
"""


def _soup(seed=7, n=20000):
    from prk import scenes
    s = scenes.random_soup(n, 256, 192, radius=60, seed=seed, centroid_margin=80)
    rng = np.random.default_rng(seed)
    v = s.vertices.reshape(-1, 3, 3).copy()
    flip = rng.random(n) < 0.4  # back-facing
    v[flip, 1], v[flip, 2] = v[flip, 2].copy(), v[flip, 1].copy()
    v[rng.random(n) < 0.05, 0, 2] = 3.9                     # a vertex at the near plane (D - z = 0.1)
    v[rng.random(n) < 0.02, 1, 2] = s.prk_transform().DistanceAboveTarget - 0.2  # exactly on it
    flat = rng.random(n) < 0.05                             # a horizontal edge
    v[flat, 1, 1] = v[flat, 0, 1]
    col = rng.random(n) < 0.03                              # collinear: the facing test's slow path
    v[col, 2] = 0.5 * (v[col, 0] + v[col, 1])
    tiny = rng.random(n) < 0.02                             # sub-2^-40 screen extent
    v[tiny, 1] = v[tiny, 0] * np.float32(1 + 1e-7)
    v[tiny, 2] = v[tiny, 0]
    big = rng.random(n) < 0.02                              # far off screen, huge magnitudes
    v[big, :, :2] *= np.float32(1e12)
    return s, v.astype(np.float32)


def _compile(tmp_path, name, extra):
    src = tmp_path / "ec_check.cpp"
    src.write_text(CHECK_SRC)
    exe = tmp_path / name
    r = subprocess.run(["g++", "-std=c++17", "-O2", *extra, "-I", os.path.join(ROOT, "include"), str(src), "-o",
                        str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def _cpu_has(flag):
    try:
        with open("/proc/cpuinfo") as f:
            return any(flag in line.split() for line in f if line.startswith("flags"))
    except OSError:
        return False


@pytest.mark.parametrize("build", ["plain", "fma_contract"])
def test_inline_sse_count_matches_scalar_and_library(tmp_path, build):
    extra = []
    if build == "fma_contract":
        if not (_cpu_has("fma") and _cpu_has("avx2")):
            pytest.skip("CPU without FMA")
        extra = ["-march=haswell", "-ffp-contract=fast"]
    exe = _compile(tmp_path, "ec_" + build, extra)
    s, v = _soup()
    T = s.prk_transform()
    P = np.asarray(s.P, np.float32)
    inp = tmp_path / "tris.bin"
    with open(inp, "wb") as f:
        f.write(np.array([T.DistanceAboveTarget, T.FocalLength, T.MetersToPixels, T.ScreenCenter[0],
                          T.ScreenCenter[1]], np.float32).tobytes())
        f.write(P.tobytes())
        f.write(np.uint32(v.shape[0]).tobytes())
        f.write(v.tobytes())
    out = tmp_path / "counts.bin"
    r = subprocess.run([str(exe), str(inp), str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, np.uint32).reshape(-1, 2)
    assert np.array_equal(got[:, 0], got[:, 1]), np.nonzero(got[:, 0] != got[:, 1])[0][:10]
    assert got[:, 0].sum() > 0 and (got[:, 0] == 0).sum() > 0  # both facings present
    # ... and the library's count (the scalar path, built by hipcc) agrees
    flat = v.reshape(-1, 3)
    for t0 in range(0, v.shape[0], 997):
        n = min(997, v.shape[0] - t0)
        want = int(got[t0:t0 + n, 0].sum())
        assert prk.fill_edge_count(flat[3 * t0:3 * (t0 + n)], tuple(map(float, P)), T) == want, t0
