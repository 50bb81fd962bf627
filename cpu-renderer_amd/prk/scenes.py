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
