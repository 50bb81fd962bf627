"""Occlusion-cull upper bounds for k_vis on the headline scene (CPU model).

VERDICT r05 item 1 asked for an exact occlusion cull inside k_vis: depth-
ordered tile bins, per-(row, 32-px segment) z floors, and skipping whole bin
entries / rows whose z upper bound is below the floor.  Before building it,
this model measures what such a cull can remove at all on C3b's geometry.

Model (numpy, a 1024x512 window of the C3b soup at C3b's density: 31 k of the
1 M triangles' density, radius 16 px, z0 in [-1, 1] +- 0.15 per vertex):
  * coverage by pixel centres, z the triangle's screen-space plane (the
    kernels' z is that plane up to the DDA's rounding);
  * 256x8 tiles, one bin per tile, entries ordered nearest-first by the
    entry's z upper bound (max vertex z + 0.5 px * |dz/dx|: the +-0.5-px
    span-end rounding) or in bin order;
  * k_vis's concurrency: 4 waves take 64-entry chunks in turn, so chunk k can
    only see the keys of chunks <= k - 4 ("in flight" = 3); 0 is a sequential
    tile (one wave, no other chunk in flight).
Culling tests, from weakest to the exact bound:
  segfloor   entry culled if its bound < min key z over the (row, 32-px
             segment) cells its bbox touches (the verdict's floors);
  perpixel   entry / row culled if its bound < the current key z of EVERY
             pixel it covers (the best any conservative test can do);
  twophase   the nearest P of a tile's entries first (all waves, barrier),
             then the rest tested per pixel against those keys only.
usage: python tools/cull_sim.py [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
from prk import scenes  # noqa: E402

TW, TH, W, H = 256, 8, 1024, 512


def build(seed=1):
    n = int(1_000_000 * W * H / 4096 ** 2)
    sc = scenes.random_soup(n, W, H, radius=16.0, seed=seed, textured=True)
    D, F, M2P, cx, cy = sc.transform
    v = sc.vertices.reshape(-1, 3, 3).astype(np.float64)
    z = v[..., 2]
    sx = cx + M2P * F * v[..., 0] / (D - z)
    sy = cy + M2P * F * v[..., 1] / (D - z)
    x0, y0 = sx[:, 0], sy[:, 0]
    e1x, e1y, e2x, e2y = sx[:, 1] - x0, sy[:, 1] - y0, sx[:, 2] - x0, sy[:, 2] - y0
    dz1, dz2 = z[:, 1] - z[:, 0], z[:, 2] - z[:, 0]
    det = e1x * e2y - e1y * e2x
    a = (dz1 * e2y - dz2 * e1y) / det
    b = (e1x * dz2 - e2x * dz1) / det
    zb = z.max(1) + 0.5 * np.abs(a) + 1e-4  # the entry's z upper bound
    ntx = W // TW
    bins = [[] for _ in range(ntx * (H // TH))]
    frag = {}
    for t in range(n):
        r0 = max(0, int(np.ceil(sy[t].min() - 0.5)))
        r1 = min(H - 1, int(np.floor(sy[t].max() - 0.5)))
        c0 = max(0, int(np.floor(sx[t].min())))
        c1 = min(W - 1, int(np.ceil(sx[t].max())))
        if r0 > r1 or c0 > c1:
            continue
        yy, xx = np.mgrid[r0:r1 + 1, c0:c1 + 1]
        px, py = xx + 0.5, yy + 0.5

        def ef(i, j):
            return (sx[t, j] - sx[t, i]) * (py - sy[t, i]) - (sy[t, j] - sy[t, i]) * (px - sx[t, i])
        e0, e1_, e2_ = ef(0, 1), ef(1, 2), ef(2, 0)
        m = ((e0 >= 0) & (e1_ >= 0) & (e2_ >= 0)) | ((e0 <= 0) & (e1_ <= 0) & (e2_ <= 0))
        if not m.any():
            continue
        X, Y = xx[m], yy[m]
        Z = z[t, 0] + a[t] * (px[m] - x0[t]) + b[t] * (py[m] - y0[t])
        tid = (Y // TH) * ntx + X // TW
        for T in np.unique(tid):
            s = tid == T
            ty, tx = T // ntx, T % ntx
            box = (max(r0, ty * TH) % TH, min(r1, ty * TH + TH - 1) % TH,
                   max(c0, tx * TW) % TW, min(c1, tx * TW + TW - 1) % TW)
            bins[T].append(t)
            frag[(t, T)] = (Y[s] % TH, X[s] % TW, Z[s], box)
    return n, bins, frag, zb


def ordered(b, zb, order, rng):
    b = np.array(b)
    if order == "z":
        return b[np.argsort(-zb[b], kind="stable")]
    if order == "rand":
        return rng.permutation(b)
    return b


def sim_chunks(bins, frag, zb, inflight, order, test, seg=32):
    rng = np.random.default_rng(0)
    tot = dict(entries=0, culled=0, rows=0, rows_culled=0, frags=0, frags_hidden=0)
    for T, b in enumerate(bins):
        if not b:
            continue
        b = ordered(b, zb, order, rng)
        keys = np.full((TH, TW), -np.inf)
        snaps = []
        for c0 in range(0, len(b), 64):
            k = c0 // 64
            st = snaps[k - inflight - 1] if k - inflight - 1 >= 0 else np.full((TH, TW), -np.inf)
            fl = st.reshape(TH, TW // seg, seg).min(2)
            for t in b[c0:c0 + 64]:
                yr, xr, zz, (r0, r1, q0, q1) = frag[(t, T)]
                tot["entries"] += 1
                tot["frags"] += len(zz)
                rows = np.unique(yr)
                tot["rows"] += len(rows)
                if test == "segfloor":
                    if zb[t] < fl[r0:r1 + 1, q0 // seg:q1 // seg + 1].min():
                        tot["culled"] += 1
                        tot["rows_culled"] += len(rows)
                    continue
                hid = zb[t] < st[yr, xr]
                tot["frags_hidden"] += int(hid.sum())
                if hid.all():
                    tot["culled"] += 1
                tot["rows_culled"] += sum(bool(hid[yr == r].all()) for r in rows)
            for t in b[c0:c0 + 64]:
                yr, xr, zz, _ = frag[(t, T)]
                np.maximum.at(keys, (yr, xr), zz)
            snaps.append(keys.copy())
    return tot


def sim_twophase(bins, frag, zb, p):
    tot = dict(entries=0, culled=0, rows=0, rows_culled=0)
    for T, b in enumerate(bins):
        if not b:
            continue
        b = ordered(b, zb, "z", None)
        n1 = int(np.ceil(p * len(b)))
        keys = np.full((TH, TW), -np.inf)
        for t in b:
            yr, xr, zz, _ = frag[(t, T)]
            rows = np.unique(yr)
            tot["entries"] += 1
            tot["rows"] += len(rows)
        for t in b[:n1]:
            yr, xr, zz, _ = frag[(t, T)]
            np.maximum.at(keys, (yr, xr), zz)
        for t in b[n1:]:
            yr, xr, zz, _ = frag[(t, T)]
            hid = zb[t] < keys[yr, xr]
            if hid.all():
                tot["culled"] += 1
            tot["rows_culled"] += sum(bool(hid[yr == r].all()) for r in np.unique(yr))
    return tot


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    n, bins, frag, zb = build()
    nfrag = sum(len(f[0]) for f in frag.values())
    res = dict(model=dict(window="%dx%d" % (W, H), triangles=n, entries=sum(len(b) for b in bins),
                          fragments=nfrag, depth_complexity=nfrag / (W * H), tile="%dx%d" % (TW, TH)),
               runs=[])
    for test, inflight, order in (("segfloor", 3, "z"), ("segfloor", 0, "z"), ("perpixel", 3, "z"),
                                  ("perpixel", 3, "bin"), ("perpixel", 0, "z"), ("perpixel", 0, "rand")):
        t = sim_chunks(bins, frag, zb, inflight, order, test)
        row = dict(test=test, inflight=inflight, order=order, entries_culled=t["culled"] / t["entries"],
                   rows_culled=t["rows_culled"] / t["rows"])
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    for p in (0.25, 0.35, 0.5):
        t = sim_twophase(bins, frag, zb, p)
        row = dict(test="twophase", first=p, entries_culled=t["culled"] / t["entries"],
                   rows_culled=t["rows_culled"] / t["rows"])
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
