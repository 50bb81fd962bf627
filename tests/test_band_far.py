"""The quick band test of k_bin_band (band_far, cpu-renderer_amd/csrc/prk_bin.hip)
drops a triangle only when the exact test would (tri_tile_range_proj's first
line: no row of the band, after ProjectVertex, projekt.cpp:74-93).

band_far uses the hardware reciprocal (v_rcp_f32, <= 1 ulp) where
ProjectVertex divides; this restates both in float32 (numpy: IEEE single,
no contraction, as the kernels are built) and checks the implication with
the reciprocal rounded down, exact and rounded up, on random and hostile
vertices: near the band edges, near the camera plane (D - z <= 0.2 projects
to 0), huge and tiny magnitudes, inf and NaN.  The GPU side of the claim is
tests/test_gpu_parity.py::test_band_edges_quick_test."""
import numpy as np

f32 = np.float32


def project_y(cy, cz, D, F, M2P, Cy, rcp_ulps=None):
    """ProjectVertex's y (exact: 1/d; else the reciprocal moved by rcp_ulps ulps)."""
    with np.errstate(all="ignore"):
        d = f32(D) - cz
        ok = d > f32(0.2)
        r = f32(1.0) / d
        if rcp_ulps is not None:
            r = np.where(rcp_ulps < 0, np.nextafter(r, f32(-np.inf)),
                         np.where(rcp_ulps > 0, np.nextafter(r, f32(np.inf)), r)).astype(np.float32)
        t = f32(M2P) * ((r * f32(F)) * cy)
        y = f32(Cy) + t
        return np.where(ok, y, f32(0.0)).astype(np.float32), np.where(ok, t, f32(0.0)).astype(np.float32)


def exact_reject(ys, row0, row1):
    """tri_tile_range_proj: fr1 + 1 <= row0 || fr0 >= row1 (fminf / fmaxf skip NaN)."""
    with np.errstate(all="ignore"):
        ymin = np.fmin(ys[0], np.fmin(ys[1], ys[2]))
        ymax = np.fmax(ys[0], np.fmax(ys[1], ys[2]))
        fr0, fr1 = np.floor(ymin), np.ceil(ymax)
        return (fr1 + f32(1.0) <= f32(row0)) | (fr0 >= f32(row1))


def band_far(cys, czs, D, F, M2P, Cy, row0, row1, ulps):
    above = np.ones(cys[0].shape, bool)
    below = np.ones(cys[0].shape, bool)
    with np.errstate(all="ignore"):
        for k in range(3):
            y, t = project_y(cys[k], czs[k], D, F, M2P, Cy, ulps[k])
            d = f32(D) - czs[k]
            m = np.where(d > f32(0.2), (np.abs(t) + np.abs(f32(Cy))) * f32(2.0 ** -18), f32(0.0)).astype(np.float32)
            above &= (y + m) + f32(2.0) < f32(row0)
            below &= (y - m) >= f32(row1) + f32(1.0)
    return above | below


def _vertices(rng, n, H, D, F, M2P, Cy, edges):
    """Camera-space (y, z) of n triangles' vertices: screen rows around the
    band edges and everywhere, unprojected; some at or behind the camera
    plane, some huge, some tiny, some non-finite."""
    z = rng.uniform(-3.0, 3.5, (3, n)).astype(np.float32)
    centre = np.where(rng.random(n) < 0.6, rng.choice(edges, n) + rng.uniform(-4, 4, n), rng.uniform(-2 * H, 3 * H, n))
    rows = centre + rng.uniform(-1, 1, (3, n)) * rng.choice([2.0, 16.0, 300.0], n)
    y = ((rows - Cy) * (D - z) / M2P / F).astype(np.float32)
    k = rng.random((3, n))
    z = np.where(k < 0.03, rng.uniform(3.79, 4.3, (3, n)), z).astype(np.float32)  # near / behind the camera plane
    y = np.where((k >= 0.03) & (k < 0.05), y * f32(1e30), y).astype(np.float32)  # huge
    y = np.where((k >= 0.05) & (k < 0.06), y * f32(1e-30), y).astype(np.float32)  # tiny
    y = np.where((k >= 0.06) & (k < 0.062), np.float32(np.inf), y).astype(np.float32)
    y = np.where((k >= 0.062) & (k < 0.064), np.float32(np.nan), y).astype(np.float32)
    z = np.where((k >= 0.064) & (k < 0.066), np.float32(-np.inf), z).astype(np.float32)
    return y, z


def test_band_far_implies_exact_reject():
    rng = np.random.default_rng(2024)
    cams = [(4.0, 1.0, 2048.0, 2048.0, 4096), (4.0, 1.0, 256.0, 256.0, 512), (7.5, 1.7, 3000.0, 1800.0, 3600),
            (4.0, 1.0, 4096.0, 4096.0, 8192)]
    rejected = dropped = 0
    for D, F, M2P, Cy, H in cams:
        for row0, row1 in [(0, H // 8), (H // 8, H // 4), (H // 2, H // 2 + 1), (H - H // 8, H), (37, 91)]:
            edges = np.array([row0, row1], float)
            ys, zs = _vertices(rng, 40000, H, D, F, M2P, Cy, edges)
            ex = exact_reject([project_y(ys[k], zs[k], D, F, M2P, Cy)[0] for k in range(3)], row0, row1)
            for ul in (-1, 0, 1):
                ulps = [np.full(ys.shape[1], ul)] * 3 if ul else [rng.integers(-1, 2, ys.shape[1]) for _ in range(3)]
                far = band_far(ys, zs, D, F, M2P, Cy, row0, row1, ulps)
                bad = far & ~ex
                assert not bad.any(), (D, F, M2P, Cy, row0, row1, ul, int(bad.sum()),
                                       ys[:, bad][:, :3], zs[:, bad][:, :3])
                rejected += int(ex.sum())
                dropped += int(far.sum())
    # and it drops most of what the exact test rejects (the point of it)
    assert dropped > 0.8 * rejected, (dropped, rejected)


def test_band_far_keeps_non_finite():
    """inf / NaN projected values fail every comparison: never dropped here."""
    for y in (np.inf, -np.inf, np.nan):
        ys = np.full((3, 1), np.float32(y))
        zs = np.zeros((3, 1), np.float32)
        far = band_far(ys, zs, 4.0, 1.0, 2048.0, 2048.0, 0, 512, [np.zeros(1, int)] * 3)
        assert not far.any(), y
