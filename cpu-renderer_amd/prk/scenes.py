"""Deterministic synthetic scenes.

The reference ships no meshes, textures or benchmark scenes; its only asset
is ConstructSphere (projekt.cpp:4123-4289, exposed by the library as
prk_construct_sphere).  These generators produce the configs of
BASELINE.json from seeded numpy RNG, in float32, non-indexed SoA exactly like
render_entry_3d_object (projekt.h:2-15): 3 vertices per triangle, positions
v3, colours v4, normals v3, uvs v2.

Camera for every scene: D = 4, F = 1, M2P = W/2, C = (W/2, H/2).  Triangles
are generated in screen space and unprojected (x = (sx - Cx)(D - z)/M2P) with
their winding forced front-facing for the reference's cull
(projekt.cpp:3926-3943: keep iff -(cross.z) > 0 on projected points).
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi

FLT_MAX = float(np.finfo(np.float32).max)
CLEAR_COLOR = 0xFF000000
CLEAR_Z = -FLT_MAX


@dataclass
class Texture:
    """loaded_bitmap with the zeroed guard row (Height+1 rows)."""
    texels: np.ndarray  # uint32 [Height+1, Pitch//4], last row zero
    width: int
    height: int
    filter: int = abi.PRK_FILTER_NEAREST  # PRK_FILTER_BILINEAR: extension (AVX only)

    @property
    def pitch(self):
        return self.texels.shape[1] * 4


@dataclass
class Scene:
    width: int
    height: int
    vertices: np.ndarray  # float32 [3T, 3]
    colors: np.ndarray    # float32 [3T, 4]
    normals: np.ndarray   # float32 [3T, 3]
    uvs: np.ndarray       # float32 [3T, 2]
    transform: tuple      # (D, F, M2P, cx, cy)
    lights: list          # [((px,py,pz),(r,g,b,a)), ...]
    ambient: tuple
    texture: Optional[Texture] = None
    P: tuple = (0.0, 0.0, 0.0)
    name: str = "scene"
    meta: dict = field(default_factory=dict)
    # Multi-draw scenes: [(first_tri, tri_count, Texture or None[, semantics
    # [, tris_per_object]]), ...] drawn in order into one frame (one DrawModel*
    # call each; semantics PRK_SEM_* / tris_per_object override the frame's);
    # None = one draw of every triangle with `texture`.
    draws: Optional[list] = None

    @property
    def tri_count(self):
        return self.vertices.shape[0] // 3

    def prk_transform(self):
        return abi.make_transform(*self.transform)

    def prk_lights(self):
        return abi.make_lights(self.lights, self.ambient)

    def subset(self, t0, t1):
        s = slice(3 * t0, 3 * t1)
        return Scene(self.width, self.height, self.vertices[s].copy(), self.colors[s].copy(),
                     self.normals[s].copy(), self.uvs[s].copy(), self.transform, self.lights,
                     self.ambient, self.texture, self.P, self.name + "[%d:%d]" % (t0, t1),
                     dict(self.meta))


def default_camera(width, height):
    return (4.0, 1.0, width / 2.0, width / 2.0, height / 2.0)


LIGHTS_ONE = [((1.0, 1.0, 3.0), (0.8, 0.8, 0.8, 1.0))]
AMBIENT_ONE = (0.2, 0.2, 0.2, 1.0)
LIGHTS_TWO = [((1.0, 1.0, 3.0), (0.8, 0.7, 0.6, 1.0)),
              ((-2.0, 0.5, 2.0), (0.3, 0.5, 0.9, 0.5))]
AMBIENT_TWO = (0.2, 0.2, 0.2, 0.2)


def random_texture(rng, w=256, h=256):
    tex = np.zeros((h + 1, w), dtype=np.uint32)
    tex[:h] = rng.integers(0, 2**32, size=(h, w), dtype=np.uint64).astype(np.uint32)
    return Texture(tex, w, h)


def _unproject(sx, sy, z, cam):
    D, F, M2P, cx, cy = cam
    x = (sx - cx) * (D - z) / M2P / F
    y = (sy - cy) * (D - z) / M2P / F
    return x, y


def random_soup(n_tris, width, height, radius=16.0, seed=0, textured=True, lights=None,
                ambient=None, centroid_margin=None, z_range=(-1.0, 1.0), jitter=0.15,
                tex_size=256):
    """C3-style soup: centroids uniform over the screen (+margin), vertex
    offsets uniform in [-radius, radius] px, per-vertex z = z0 +- jitter with
    z0 uniform in z_range, random unit normals, uniform uvs/colours."""
    rng = np.random.default_rng(seed)
    cam = default_camera(width, height)
    m = radius if centroid_margin is None else centroid_margin
    n = int(n_tris)
    cxy = np.stack([rng.uniform(-m, width + m, n), rng.uniform(-m, height + m, n)], 1)
    off = rng.uniform(-radius, radius, (n, 3, 2))
    s = cxy[:, None, :] + off
    e1 = s[:, 1] - s[:, 0]
    e2 = s[:, 2] - s[:, 0]
    cz = e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0]
    flip = cz > 0  # want cross.z < 0 so that Inner((0,0,-1), cross) > 0
    s[flip, 1], s[flip, 2] = s[flip, 2].copy(), s[flip, 1].copy()
    z0 = rng.uniform(z_range[0], z_range[1], n)
    z = z0[:, None] + rng.uniform(-jitter, jitter, (n, 3))
    x, y = _unproject(s[..., 0], s[..., 1], z, cam)
    verts = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    nrm = rng.normal(size=(3 * n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    uvs = rng.uniform(0.0, 1.0, (3 * n, 2)).astype(np.float32)
    cols = rng.uniform(0.0, 1.0, (3 * n, 4)).astype(np.float32)
    cols[:, 3] = 1.0
    tex = random_texture(rng, tex_size, tex_size) if textured else None
    return Scene(width, height, verts, cols, nrm.astype(np.float32), uvs, cam,
                 LIGHTS_ONE if lights is None else lights,
                 AMBIENT_ONE if ambient is None else ambient, tex,
                 name="soup%d_%dx%d_r%g_s%d" % (n, width, height, radius, seed),
                 meta=dict(kind="soup", radius=radius, seed=seed))


def single_triangle(width=256, height=256, textured=False, gouraud_only=True):
    """C1: one RGB triangle at 256x256.  With ambient = 1 and I = 0 the
    Gouraud setup (projekt.cpp:4020-4063) reduces to pure vertex colours."""
    cam = default_camera(width, height)
    s = np.array([[40.3, 30.7], [220.6, 90.2], [100.1, 230.4]], dtype=np.float64)
    e1, e2 = s[1] - s[0], s[2] - s[0]
    if e1[0] * e2[1] - e1[1] * e2[0] > 0:
        s[[1, 2]] = s[[2, 1]]
    z = np.array([0.1, -0.2, 0.3])
    x, y = _unproject(s[:, 0], s[:, 1], z, cam)
    verts = np.stack([x, y, z], -1).astype(np.float32)
    cols = np.array([[1, 0, 0, 1], [0, 1, 0, 1], [0, 0, 1, 1]], dtype=np.float32)
    nrm = np.array([[0, 0, 1], [0.3, 0, 0.95], [0, 0.3, 0.95]], dtype=np.float32)
    uvs = np.array([[0.05, 0.05], [0.95, 0.1], [0.4, 0.95]], dtype=np.float32)
    tex = random_texture(np.random.default_rng(1), 64, 64) if textured else None
    if gouraud_only:
        lights, amb = [((1.0, 1.0, 3.0), (0.0, 0.0, 0.0, 0.0))], (1.0, 1.0, 1.0, 1.0)
    else:
        lights, amb = LIGHTS_ONE, AMBIENT_ONE
    return Scene(width, height, verts, cols, nrm, uvs, cam, lights, amb, tex,
                 name="triangle_%dx%d" % (width, height), meta=dict(kind="triangle"))


def displaced_sphere(n_target, width, height, seed=0, radius=0.9, bumps=0.08):
    """C2 stand-in (no mesh files exist in this container): a closed, displaced
    UV sphere of ~n_target triangles centred on screen, generalising
    ConstructSphere (projekt.cpp:4123-4289).  Smooth per-vertex normals."""
    rng = np.random.default_rng(seed)
    cam = default_camera(width, height)
    steps = max(4, int(round(np.sqrt(n_target / 4.0))))
    n_inc, n_az = steps, 2 * steps
    th = np.linspace(0, np.pi, n_inc + 1)
    ph = np.linspace(0, 2 * np.pi, n_az + 1)
    T, Ph = np.meshgrid(th, ph, indexing="ij")
    k = rng.normal(size=(6, 3))
    dirs = np.stack([np.sin(T) * np.cos(Ph), np.cos(T), np.sin(T) * np.sin(Ph)], -1)
    disp = 1.0 + bumps * np.sin(3 * dirs @ k[0] + 1.0) * np.cos(2 * dirs @ k[1])
    P = dirs * (radius * disp)[..., None]
    Nrm = dirs  # approximate smooth normals (unit)
    UV = np.stack([Ph / (2 * np.pi), T / np.pi], -1)
    tris = []
    for i in range(n_inc):
        for j in range(n_az):
            a, b, c, d = (i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)
            tris.append((a, b, c))
            tris.append((a, c, d))
    idx = np.array(tris)  # [T,3,2]
    V = P[idx[..., 0], idx[..., 1]]
    N = Nrm[idx[..., 0], idx[..., 1]]
    U = UV[idx[..., 0], idx[..., 1]]
    # Place in front of the camera: camera looks down -z from z = D = 4
    # (projekt.cpp:80: distance = D - z), so larger z is nearer.
    V = V.copy()
    V[..., 2] += 0.5
    col = np.concatenate([0.5 + 0.5 * N, np.ones(N.shape[:-1] + (1,))], -1)
    # Drop degenerate polar triangles, then force the reference's winding on the rest.
    verts = V.reshape(-1, 3).astype(np.float32)
    return Scene(width, height, verts, col.reshape(-1, 4).astype(np.float32),
                 N.reshape(-1, 3).astype(np.float32), U.reshape(-1, 2).astype(np.float32),
                 cam, LIGHTS_ONE, AMBIENT_ONE, None,
                 name="sphere%d_%dx%d" % (len(tris), width, height),
                 meta=dict(kind="displaced_sphere"))


def slivers(n_tris, width, height, seed=0, textured=True):
    """Edge cases of the AET order: near-vertical slivers far right on the
    screen whose two top edges have gradients below half an ulp of X, so
    X + G rounds back to X and the two edges tie in X on every row.  The list
    order then comes from the insertion tie-break (G, then Left;
    projekt.cpp:3663-3667) carried through rows without a crossing swap
    (3831-3841).  DrawModel's inclusive span draws the one pixel at X with the
    LEFT edge's attributes, so a wrong order shows in z and colour."""
    rng = np.random.default_rng(seed)
    cam = default_camera(width, height)
    n = int(n_tris)
    x0 = rng.uniform(width * 0.75, width - 4.0, n)
    y0 = rng.uniform(0.0, height - 48.0, n)
    h1 = rng.uniform(4.0, 24.0, n)
    h2 = h1 + rng.uniform(4.0, 24.0, n)
    ulp = np.spacing(np.float32(width)).astype(np.float64)
    # |dx / h| well below half an ulp: both top edges stick at X = x0.
    s = np.empty((n, 3, 2))
    s[:, 0] = np.stack([x0, y0], 1)
    s[:, 1] = np.stack([x0 + rng.uniform(0.5, 4.0, n) * ulp, y0 + h1], 1)
    s[:, 2] = np.stack([x0 + rng.uniform(-4.0, 4.0, n) * ulp, y0 + h2], 1)
    # a quarter of them widen below the middle vertex (spans of several pixels)
    wide = rng.random(n) < 0.25
    s[wide, 1, 0] += rng.uniform(2.0, 10.0, wide.sum())
    e1 = s[:, 1] - s[:, 0]
    e2 = s[:, 2] - s[:, 0]
    flip = e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0] > 0
    s[flip, 1], s[flip, 2] = s[flip, 2].copy(), s[flip, 1].copy()
    z = rng.uniform(-0.8, 0.8, n)[:, None] + rng.uniform(-0.1, 0.1, (n, 3))
    x, y = _unproject(s[..., 0], s[..., 1], z, cam)
    verts = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    nrm = rng.normal(size=(3 * n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    uvs = rng.uniform(0.0, 1.0, (3 * n, 2)).astype(np.float32)
    cols = rng.uniform(0.0, 1.0, (3 * n, 4)).astype(np.float32)
    cols[:, 3] = 1.0
    tex = random_texture(rng, 64, 64) if textured else None
    return Scene(width, height, verts, cols, nrm.astype(np.float32), uvs, cam, LIGHTS_ONE, AMBIENT_ONE, tex,
                 name="slivers%d_%dx%d_s%d" % (n, width, height, seed), meta=dict(kind="slivers", seed=seed))


def procedural_texture(rng, size, kind):
    """A 1024^2-style material texture (uint32 ARGB, zeroed guard row):
    checker / brick / stripes / noise patterns with per-texel noise."""
    y, x = np.mgrid[0:size, 0:size]
    base = rng.integers(40, 200, size=3)
    alt = rng.integers(40, 220, size=3)
    if kind == 0:    # checker
        m = ((x // 64) + (y // 64)) & 1
    elif kind == 1:  # bricks
        row = y // 48
        m = (((x + (row & 1) * 64) % 128) < 6) | ((y % 48) < 5)
    elif kind == 2:  # stripes
        m = ((x + y) // 40) & 1
    else:            # blobs
        m = (np.sin(x / 37.0) * np.cos(y / 23.0)) > 0.2
    m = m.astype(np.int64)
    noise = rng.integers(-18, 19, size=(size, size, 3))
    rgb = np.clip(base[None, None, :] * (1 - m[..., None]) + alt[None, None, :] * m[..., None] + noise, 0, 255)
    tex = np.zeros((size + 1, size), np.uint32)
    tex[:size] = ((0xFF << 24) | (rgb[..., 0].astype(np.uint32) << 16) | (rgb[..., 1].astype(np.uint32) << 8)
                  | rgb[..., 2].astype(np.uint32)).astype(np.uint32)
    return Texture(tex, size, size)


def _grid_quads(p0, du, dv, nu, nv, normal):
    """nu x nv quads on the parallelogram p0 + s*du + t*dv; each quad maps the
    whole texture (UVs in [0, 1], as the AVX path's UV mask requires)."""
    s = np.arange(nu)[:, None]
    t = np.arange(nv)[None, :]
    a = p0 + (s[..., None] / nu) * du + (t[..., None] / nv) * dv
    b = a + du / nu
    c = b + dv / nv
    d = a + dv / nv
    quads = np.stack([a, b, c, d], 2).reshape(-1, 4, 3)
    tris = np.concatenate([quads[:, [0, 1, 2]], quads[:, [0, 2, 3]]], 0)
    uv = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float64)
    tuv = np.concatenate([np.repeat(uv[None, [0, 1, 2]], len(quads), 0), np.repeat(uv[None, [0, 2, 3]], len(quads), 0)], 0)
    nrm = np.repeat(np.asarray(normal, np.float64)[None, None, :], len(tris), 0).repeat(3, 1)
    return tris, tuv, nrm


def _cylinder(cx, cz, r, y0, y1, n_around, n_up, outward=True):
    ang = np.linspace(0, 2 * np.pi, n_around + 1)
    ys = np.linspace(y0, y1, n_up + 1)
    A, Y = np.meshgrid(ang, ys, indexing="ij")
    P = np.stack([cx + r * np.cos(A), Y, cz + r * np.sin(A)], -1)
    N = np.stack([np.cos(A), np.zeros_like(A), np.sin(A)], -1)
    UV = np.stack([A / (2 * np.pi), (Y - y0) / (y1 - y0)], -1)
    return _mesh_from_grid(P, N, UV)


def _arch(x0, x1, cz, y_base, thickness, n_seg, n_w):
    """Half-torus-like arch spanning x0..x1 at depth cz (a curved band)."""
    cx, rad = 0.5 * (x0 + x1), 0.5 * (x1 - x0)
    ang = np.linspace(0, np.pi, n_seg + 1)
    w = np.linspace(-thickness, thickness, n_w + 1)
    A, Wd = np.meshgrid(ang, w, indexing="ij")
    P = np.stack([cx + rad * np.cos(A), y_base + rad * np.sin(A), cz + Wd], -1)
    N = np.stack([-np.cos(A), -np.sin(A), np.zeros_like(A)], -1)  # underside faces down/in
    UV = np.stack([A / np.pi, (Wd + thickness) / (2 * thickness)], -1)
    return _mesh_from_grid(P, N, UV)


def _mesh_from_grid(P, N, UV):
    """Triangles of a (nu+1) x (nv+1) vertex grid, two per cell, UVs rescaled
    so that every cell maps the whole texture."""
    nu, nv = P.shape[0] - 1, P.shape[1] - 1
    i, j = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    i, j = i.ravel(), j.ravel()
    cells = [(i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)]
    cp = [P[a, b] for a, b in cells]
    cn = [N[a, b] for a, b in cells]
    uvc = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float64)
    tris = np.concatenate([np.stack([cp[0], cp[1], cp[2]], 1), np.stack([cp[0], cp[2], cp[3]], 1)], 0)
    nrm = np.concatenate([np.stack([cn[0], cn[1], cn[2]], 1), np.stack([cn[0], cn[2], cn[3]], 1)], 0)
    tuv = np.concatenate([np.repeat(uvc[None, [0, 1, 2]], len(i), 0), np.repeat(uvc[None, [0, 2, 3]], len(i), 0)], 0)
    return tris, tuv, nrm


def sponza_like(width=3840, height=2160, seed=0, detail=1.56, tex_size=1024, filt=abi.PRK_FILTER_BILINEAR):
    """C4 stand-in ("textured Sponza-style scene, ~250k tris", no asset files
    exist here): a procedural atrium — floor, ceiling, side and back walls, two
    rows of pillars and arches between them — in 8 materials of one
    tex_size^2 texture each, drawn as 8 draws (one DrawModelOptimized call per
    material).  Every triangle is oriented so that the reference's back-face
    cull (projekt.cpp:3926-3943) keeps the faces toward the camera and drops
    the rest (pillar backs, arch tops).  `filt`: texture sampling of all 8
    materials (bilinear is the build's extension, BASELINE config 4)."""
    rng = np.random.default_rng(seed)
    cam = default_camera(width, height)
    D = cam[0]
    X, Yf, Yc, Z0, Z1 = 6.0, -2.5, 3.5, 3.0, -34.0
    g = lambda n: max(2, int(round(n * detail)))  # noqa: E731
    parts = []  # (tris, uv, nrm) per material
    parts.append(_grid_quads(np.array([-X, Yf, Z0]), np.array([2 * X, 0, 0]), np.array([0, 0, Z1 - Z0]), g(60), g(110), (0, 1, 0)))    # floor
    parts.append(_grid_quads(np.array([-X, Yc, Z0]), np.array([2 * X, 0, 0]), np.array([0, 0, Z1 - Z0]), g(40), g(80), (0, -1, 0)))   # ceiling
    parts.append(_grid_quads(np.array([-X, Yf, Z0]), np.array([0, Yc - Yf, 0]), np.array([0, 0, Z1 - Z0]), g(40), g(110), (1, 0, 0)))  # left
    parts.append(_grid_quads(np.array([X, Yf, Z0]), np.array([0, Yc - Yf, 0]), np.array([0, 0, Z1 - Z0]), g(40), g(110), (-1, 0, 0)))  # right
    parts.append(_grid_quads(np.array([-X, Yf, Z1]), np.array([2 * X, 0, 0]), np.array([0, Yc - Yf, 0]), g(60), g(40), (0, 0, 1)))    # back
    cols = []
    zs = np.linspace(-2.0, -30.0, 8)
    for side in (-3.5, 3.5):
        for cz in zs:
            cols.append(_cylinder(side, cz, 0.45, Yf, 1.5, g(48), g(32)))
    parts.append(tuple(np.concatenate([c[k] for c in cols], 0) for k in range(3)))  # pillars
    arches = []
    for side in (-3.5, 3.5):
        for a, b in zip(zs[:-1], zs[1:]):
            # arch between consecutive pillars of one row (spans along z, rotate: swap axes)
            t, uv, n = _arch(b, a, 0.0, 1.5, 0.4, g(40), g(8))
            t = t[..., [2, 1, 0]].copy()
            t[..., 0] += side
            n = n[..., [2, 1, 0]].copy()
            arches.append((t, uv, n))
    parts.append(tuple(np.concatenate([c[k] for c in arches], 0) for k in range(3)))  # arches
    # cross arches over the nave
    xarch = [_arch(-3.5, 3.5, cz, 1.5, 0.3, g(64), g(6)) for cz in zs[::2]]
    parts.append(tuple(np.concatenate([c[k] for c in xarch], 0) for k in range(3)))
    verts, uvs, nrms, draws = [], [], [], []
    first = 0
    textures = [procedural_texture(rng, tex_size, k % 4) for k in range(len(parts))]
    for k, (tris, tuv, nrm) in enumerate(parts):
        # Screen rows grow with +y (projekt.cpp:86): build y-up, then flip.
        tris = tris * np.array([1.0, -1.0, 1.0])
        nrm = nrm * np.array([1.0, -1.0, 1.0])
        # Orient: faces whose normal looks at the eye (origin after projection:
        # distance D - z) keep the reference's front winding (projected
        # cross.z < 0), the others get the back winding and are culled.
        eye = np.array([0.0, 0.0, D])
        cen = tris.mean(1)
        front = (nrm.mean(1) * (eye - cen)).sum(-1) > 0
        d = D - tris[..., 2]
        sx = tris[..., 0] / d
        sy = tris[..., 1] / d
        cz = (sx[:, 1] - sx[:, 0]) * (sy[:, 2] - sy[:, 0]) - (sy[:, 1] - sy[:, 0]) * (sx[:, 2] - sx[:, 0])
        flip = (cz > 0) == front
        tris[flip, 1], tris[flip, 2] = tris[flip, 2].copy(), tris[flip, 1].copy()
        tuv[flip, 1], tuv[flip, 2] = tuv[flip, 2].copy(), tuv[flip, 1].copy()
        nrm[flip, 1], nrm[flip, 2] = nrm[flip, 2].copy(), nrm[flip, 1].copy()
        textures[k].filter = filt
        verts.append(tris.reshape(-1, 3))
        uvs.append(tuv.reshape(-1, 2))
        nrms.append(nrm.reshape(-1, 3))
        draws.append((first, len(tris), textures[k]))
        first += len(tris)
    V = np.concatenate(verts).astype(np.float32)
    N = np.concatenate(nrms).astype(np.float32)
    UV = np.concatenate(uvs).astype(np.float32)
    C = np.ones((V.shape[0], 4), np.float32)
    lights = [((0.0, -2.5, -6.0), (0.9, 0.85, 0.7, 1.0)), ((-3.0, -1.0, -20.0), (0.4, 0.5, 0.9, 1.0))]
    return Scene(width, height, V, C, N, UV, cam, lights, (0.25, 0.25, 0.25, 1.0), None,
                 name="sponza_like%d_%dx%d" % (V.shape[0] // 3, width, height),
                 meta=dict(kind="sponza_like", seed=seed), draws=draws)


def draw_spec(d, semantics, tris_per_object=1):
    """(first, count, texture, semantics, tris_per_object) of a Scene.draws
    entry (first, count, texture[, semantics[, tris_per_object]])."""
    return (d[0], d[1], d[2], d[3] if len(d) > 3 and d[3] is not None else semantics,
            d[4] if len(d) > 4 and d[4] is not None else tris_per_object)


def with_ties(scene, frac=0.5, seed=0):
    """The scene plus exact positional duplicates of a random `frac` of its
    triangles (new normals, uvs and colours, so the tie's two fragments shade
    differently), each inserted at a random later position: equal-z
    fragments decide the z-test's tie rule (projekt.cpp:2219 strict '>' vs
    3205 '>=')."""
    rng = np.random.default_rng(seed)
    T = scene.tri_count
    pick = np.sort(rng.choice(T, int(T * frac), replace=False))
    order = list(range(T))
    for k in pick[::-1]:
        order.insert(int(rng.integers(k + 1, len(order) + 1)), T + int(np.searchsorted(pick, k)))
    V = scene.vertices.reshape(T, 3, 3)
    Vd = np.concatenate([V, V[pick]])
    def fresh(a, lo, hi):
        a = a.reshape(T, 3, -1)
        b = rng.uniform(lo, hi, a[pick].shape).astype(np.float32)
        return np.concatenate([a, b])
    N = fresh(scene.normals, -1.0, 1.0)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    UV = fresh(scene.uvs, 0.0, 1.0)
    C = fresh(scene.colors, 0.0, 1.0)
    o = np.array(order)
    return Scene(scene.width, scene.height, Vd[o].reshape(-1, 3).copy(), C[o].reshape(-1, 4).copy(),
                 N[o].reshape(-1, 3).astype(np.float32).copy(), UV[o].reshape(-1, 2).copy(), scene.transform,
                 scene.lights, scene.ambient, scene.texture, scene.P, scene.name + "+ties", dict(scene.meta))
