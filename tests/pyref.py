"""pyref — a second, independent restatement of the hot path in plain Python
(numpy float32 scalars, one op at a time: IEEE single rounding, no FMA).

TEST INFRASTRUCTURE ONLY (slow; small cases).  It is written from
projekt.cpp directly, separately from oracle/prk_oracle.c, so that the two
restatements check each other.  Covers per-triangle submission of
FillEdgeTable (3882-4121) + MergeSort (2-72) + the AET of
DrawModelOptimized(RenderQueue,...) (3615-3871, with P3) + FillLineOptimized
(1492-2320, Phong + texture) or DrawModel's span loop (298-538).
"""
import math

import numpy as np

f32 = np.float32
INT_MIN = -2**31


def cvtt(x):
    x = float(x)
    if not (-2147483648.0 <= x < 2147483648.0):
        return INT_MIN
    return int(x)  # truncation toward zero


def roundf(x):
    x = float(x)
    if x != x or math.isinf(x):
        return x
    return math.copysign(math.floor(abs(x) + 0.5), x)


def round_s32(x):
    return cvtt(roundf(x))


def round_u32(x):
    r = roundf(x)
    if not (-9.2233720368547758e18 <= r < 9.2233720368547758e18):
        return 0
    return int(r) & 0xFFFFFFFF


def rne(x):
    x = float(x)
    if not (-2147483648.0 <= x < 2147483648.0):
        return INT_MIN
    return int(np.rint(x))


def mx(a, b):  # MAXPS
    return a if a > b else b


def mn(a, b):  # MINPS
    return a if a < b else b


def clamp01(x):
    return f32(0) if x < 0 else (f32(1) if x > 1 else x)


def norm_rcp(v):
    s = f32(1) / np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    return [s * v[0], s * v[1], s * v[2]]


def norm_div(v):
    ln = np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    return [v[0] / ln, v[1] / ln, v[2] / ln]


def mul16(y, p):
    ylo, yhi = y & 0xFFFF, (y >> 16) & 0xFFFF
    plo, phi = p & 0xFFFF, (p >> 16) & 0xFFFF
    lo = (ylo * plo) & 0xFFFF
    hmlo = (yhi * phi) & 0xFFFF
    s16 = lambda v: v - 0x10000 if v & 0x8000 else v  # noqa: E731
    hmhi = ((s16(ylo) * s16(plo)) >> 16) & 0xFFFF
    r = lo | (((hmlo | hmhi) & 0xFFFF) << 16)
    return r - (1 << 32) if r & 0x80000000 else r


def texel(tex, off):
    limit = tex.pitch * (tex.height + 1) - 4
    if off < 0 or off > limit:
        off = 0
    flat = tex.texels.reshape(-1).view(np.uint8)
    return int(flat[off:off + 4].view(np.uint32)[0])


def bilinear(tex, fu, fv):
    """The build's bilinear extension (no reference): centres at +0.5,
    clamp to edge, fp32.  Returns [R, G, B, A] in [0, 1]."""
    x = f32(tex.width) * fu - f32(0.5)
    y = f32(tex.height) * fv - f32(0.5)
    fx, fy = f32(np.floor(x)), f32(np.floor(y))
    ax, ay = x - fx, y - fy
    x0, y0 = int(fx), int(fy)
    xs = [min(max(x0, 0), tex.width - 1), min(max(x0 + 1, 0), tex.width - 1)]
    ys = [min(max(y0, 0), tex.height - 1), min(max(y0 + 1, 0), tex.height - 1)]
    rows = tex.texels
    bx, by = f32(1) - ax, f32(1) - ay
    out = []
    for sh in (16, 8, 0, 24):
        c = [[f32((int(rows[yy, xx]) >> sh) & 255) / f32(255) for xx in xs] for yy in ys]
        top = bx * c[0][0] + ax * c[0][1]
        bot = bx * c[1][0] + ax * c[1][1]
        out.append(by * top + ay * bot)
    return out


class Cam:
    """Commands->Transform and LightData of a scene, as float32."""

    def __init__(self, scene):
        self.D, self.F, self.M2P, self.cx, self.cy = [f32(v) for v in scene.transform]
        self.lights = [([f32(c) for c in p], [f32(c) for c in i]) for p, i in scene.lights]
        self.amb = [f32(c) for c in scene.ambient]


class Ctx:
    def __init__(self, scene, semantics, phong, color=None, z=None, setup=None, setup_camera=None):
        self.s = scene
        # the camera FillEdgeTable saw (project + Gouraud lighting); the spans
        # shade with the scene's own (Commands at DrawModel*, 452-458, 2042-2046)
        self.su = Cam(scene if setup_camera is None else setup_camera)
        # FillEdgeTable's own PhongShading / Object->Bitmap (projekt.cpp:4012-4089);
        # None: as the draw (PhongShading, the draw's Bitmap)
        self.fe_phong = phong if setup is None else bool(setup & 1)
        self.fe_bitmap = (scene.texture is not None) if setup is None else bool(setup & 2)
        self.W, self.H = scene.width, scene.height
        D, F, M2P, cx, cy = [f32(v) for v in scene.transform]
        self.D, self.F, self.M2P, self.cx, self.cy = D, F, M2P, cx, cy
        self.lights = [([f32(c) for c in p], [f32(c) for c in i]) for p, i in scene.lights]
        self.amb = [f32(c) for c in scene.ambient]
        self.avx = semantics in (1, 2)
        self.st = semantics == 2  # DrawModelOptimized(Buffer,...) projekt.cpp:2350-3358
        self.phong = phong
        self.tex = scene.texture
        self.color = np.full((self.H, self.W), 0xFF000000, np.uint32) if color is None else color
        self.z = np.full((self.H, self.W), -np.finfo(np.float32).max, np.float32) if z is None else z
        self.win = np.full((self.H, self.W), -1, np.int64)


def project(ctx, c):
    d = ctx.D - c[2]
    if d > f32(0.2):
        k = (f32(1) / d) * ctx.F
        return [ctx.cx + ctx.M2P * (k * c[0]), ctx.cy + ctx.M2P * (k * c[1]), d + ctx.M2P * f32(0)]
    return [f32(0), f32(0), f32(0)]


def edge_table(ctx, t):
    s = ctx.s
    P = [f32(v) for v in s.P]
    cam = [[s.vertices[3 * t + k][i] + P[i] for i in range(3)] for k in range(3)]
    proj = [project(ctx.su, c) for c in cam]
    a = norm_rcp([proj[1][i] - proj[0][i] for i in range(3)])
    b = norm_rcp([proj[2][i] - proj[0][i] for i in range(3)])
    cross = [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]
    inner = (f32(0) * cross[0] + f32(0) * cross[1]) + f32(-1) * cross[2]
    if not inner > 0:
        return []
    textured = ctx.fe_bitmap  # Object->Bitmap (4034-4054, 4078)
    edges = []
    for i0, i1 in ((0, 1), (1, 2), (2, 0)):
        mi, ma = i0, i1
        if proj[mi][1] > proj[ma][1]:
            mi, ma = ma, mi
        Mn, Mx = proj[mi], proj[ma]
        if not Mx[1] > 0:
            continue
        e = {}
        e["YMax"] = round_s32(Mx[1])
        clip, tt = f32(0), f32(0)
        if Mn[1] < f32(0):
            clip = -Mn[1]
            tt = (-Mn[1]) / (Mx[1] - Mn[1])
        r = f32(round_s32(Mn[1]))
        e["YMin"] = int(f32(0) if f32(0) > r else r)
        e["X"] = Mn[0]
        e["Z"] = cam[mi][2]
        uv0 = [f32(v) for v in s.uvs[3 * t + mi]]
        uv1 = [f32(v) for v in s.uvs[3 * t + ma]]
        e["U"] = uv0[0] / Mn[2]
        e["V"] = uv0[1] / Mn[2]
        e["W"] = f32(1) / Mn[2]
        s2 = f32(1) / Mx[2]
        uv1 = [uv1[0] * s2, uv1[1] * s2]
        s1 = f32(1) / Mn[2]
        uv0 = [uv0[0] * s1, uv0[1] * s1]
        c0 = [f32(v) for v in s.colors[3 * t + mi]]
        c1 = [f32(v) for v in s.colors[3 * t + ma]]
        n0 = [f32(v) for v in s.normals[3 * t + mi]]
        n1 = [f32(v) for v in s.normals[3 * t + ma]]
        if ctx.fe_phong:  # FillEdgeTable's PhongShading (4012)
            minc, maxc, minn, maxn = c0, c1, n0, [n1[0], n1[1], n1[2]]
        else:
            minc, maxc = [f32(0)] * 4, [f32(0)] * 4
            minn, maxn = [f32(0)] * 3, [f32(0)] * 3
            for li, (lp, lint) in enumerate(ctx.su.lights):
                fv = norm_rcp([lp[k] - cam[mi][k] for k in range(3)])
                sv = norm_rcp([lp[k] - cam[ma][k] for k in range(3)])
                if li == 0:
                    minc = [(f32(1) if textured else c0[k]) * ctx.su.amb[k] for k in range(4)]
                    maxc = [(f32(1) if textured else c1[k]) * ctx.su.amb[k] for k in range(4)]
                fd = clamp01((fv[0] * n0[0] + fv[1] * n0[1]) + fv[2] * n0[2])
                sd = clamp01((sv[0] * n1[0] + sv[1] * n1[1]) + sv[2] * n1[2])
                minc = [clamp01(minc[k] + fd * ((f32(1) if textured else c0[k]) * lint[k])) for k in range(4)]
                maxc = [clamp01(maxc[k] + sd * ((f32(1) if textured else c1[k]) * lint[k])) for k in range(4)]
        if Mn[1] - Mx[1] == 0:
            continue
        yd = f32(e["YMax"]) - f32(e["YMin"])
        with np.errstate(all="ignore"):
            e["ZG"] = (cam[ma][2] - cam[mi][2]) / yd
            e["G"] = (Mx[0] - Mn[0]) / (Mx[1] - Mn[1])
            e["X"] = e["X"] + clip * e["G"]
            e["Z"] = e["Z"] + clip * e["ZG"]
            if textured:
                e["UG"] = (uv1[0] - uv0[0]) / yd
                e["VG"] = (uv1[1] - uv0[1]) / yd
                e["U"] = e["U"] + clip * e["UG"]
                e["V"] = e["V"] + clip * e["VG"]
                e["WG"] = ((f32(1) / Mx[2]) - e["W"]) / yd
                e["W"] = e["W"] + clip * e["WG"]
            else:
                e["U"] = e["V"] = e["W"] = e["UG"] = e["VG"] = e["WG"] = f32(0)
            minc = [(f32(1) - tt) * minc[k] + tt * maxc[k] for k in range(4)]
            e["C"] = minc
            e["CG"] = [(maxc[k] - minc[k]) / yd for k in range(4)]
            e["N"] = list(minn)
            e["NG"] = [(maxn[k] - minn[k]) / yd for k in range(3)]
        e["Left"] = 1 if e["YMin"] == round_s32(proj[i0][1]) else 0
        edges.append(e)
    # MergeSort (projekt.cpp:2-72) for <= 3 edges.
    if len(edges) == 2 and edges[0]["YMin"] > edges[1]["YMin"]:
        edges = [edges[1], edges[0]]
    elif len(edges) == 3:
        h1 = edges[1:]
        if h1[0]["YMin"] > h1[1]["YMin"]:
            h1 = [h1[1], h1[0]]
        out, a, i = [], [edges[0]], 0
        while a or i < 2:
            if not a:
                out.append(h1[i]); i += 1
            elif i == 2:
                out.append(a.pop())
            elif a[0]["YMin"] < h1[i]["YMin"]:
                out.append(a.pop())
            else:
                out.append(h1[i]); i += 1
        edges = out
    return edges


def before(a, b):
    return a["X"] < b["X"] or (a["X"] == b["X"] and (a["G"] < b["G"] or (a["G"] == b["G"] and a["Left"] < b["Left"])))


def step(e):
    with np.errstate(all="ignore"):
        e["X"] = e["X"] + e["G"]
        e["Z"] = e["Z"] + e["ZG"]
        e["C"] = [e["C"][k] + e["CG"][k] for k in range(4)]
        e["N"] = norm_rcp([e["N"][k] + e["NG"][k] for k in range(3)])
        e["U"] = e["U"] + e["UG"]
        e["V"] = e["V"] + e["VG"]
        e["W"] = e["W"] + e["WG"]


def walk(ctx, t, edges):
    if not edges:
        return
    first = edges[0]["YMin"]
    maxy = min(max(e["YMax"] for e in edges), ctx.H)
    lst = []
    for row in range(first, maxy):
        for e in edges:
            if e["YMin"] == row:
                pos = len(lst)
                for j, o in enumerate(lst):
                    if before(e, o):
                        pos = j
                        break
                lst.insert(pos, e)
        lst = [e for e in lst if not e["YMax"] <= row]
        if len(lst) >= 2:
            L = {k: (list(v) if isinstance(v, list) else v) for k, v in lst[0].items()}
            R = {k: (list(v) if isinstance(v, list) else v) for k, v in lst[1].items()}
            (span_avx if ctx.avx else span_scalar)(ctx, t, L, R, row)
            step(lst[0])
            step(lst[1])
            if lst[0]["X"] > lst[1]["X"]:
                lst[0], lst[1] = lst[1], lst[0]


def shade_phong_avx(ctx, C, P, n):
    F = [f32(0)] * 4
    for li, (lp, I) in enumerate(ctx.lights):
        if li == 0:
            F = [C[k] * ctx.amb[k] for k in range(4)]
        L = norm_div([lp[k] - P[k] for k in range(3)])
        cos = mn(f32(1), mx(f32(0), (n[0] * L[0] + n[1] * L[1]) + n[2] * L[2]))
        V = norm_div([f32(0) - P[k] for k in range(3)])
        Hh = norm_div([L[k] + V[k] for k in range(3)])
        ph = mn(f32(1), mx(f32(0), (n[0] * Hh[0] + n[1] * Hh[1]) + n[2] * Hh[2]))
        for _ in range(4):
            ph = ph * ph
        F = [F[k] + ((cos * (C[k] * I[k])) + (ph * (f32(1) * I[k]))) for k in range(4)]
    return [mx(mn(F[k], f32(1)), f32(0)) for k in range(4)]


def span_avx(ctx, t, L, R, row):
    W = ctx.W
    xoff = f32(0)
    lx = L["X"]
    if lx < 0:
        xoff, lx = (-xoff if ctx.st else -L["X"]), f32(0)  # single-thread: XOffset = -XOffset (2508)
    elif lx >= W:
        lx = f32(W) - f32(1)
    rx = R["X"]
    if rx < 0:
        rx = f32(0)
    elif rx >= W:
        rx = f32(W) - f32(1)
    if lx != lx or rx != rx:
        return
    xd = (round_s32(R["X"]) - round_s32(L["X"]) + 2**31) % 2**32 - 2**31
    mnx, mxx = round_s32(lx), round_s32(rx)
    left = mnx
    if mnx & 7:
        left = mnx & ~7
        xoff = xoff - f32(mnx & 7) * f32(1)
    fxd = f32(xd)
    with np.errstate(all="ignore"):
        inc = {}
        for q in ("W", "U", "V", "Z"):
            inc[q] = (R[q] - L[q]) / fxd if xd != 0 else f32(0)
        incn = [(R["N"][k] - L["N"][k]) / fxd if xd != 0 else f32(0) for k in range(3)]
        for x in range(max(mnx, 0), mxx):
            rel = x - left
            i, b = rel & 7, rel >> 3
            o = xoff + f32(i)
            v = {q: L[q] + o * inc[q] for q in inc}
            n = norm_div([L["N"][k] + o * incn[k] for k in range(3)])
            for _ in range(b):
                n = norm_div([n[k] + incn[k] * f32(8) for k in range(3)])
                v["Z"] = v["Z"] + f32(8) * inc["Z"]
                for q in ("W", "U", "V"):
                    v[q] = v[q] + inc[q] * f32(8)
            iw = f32(1) / v["W"]
            fu, fv = iw * v["U"], iw * v["V"]
            if not (fu >= 0 and fu <= 1 and fv >= 0 and fv <= 1):
                continue
            z = v["Z"]
            if not (z >= ctx.z[row, x] if ctx.st else z > ctx.z[row, x]):  # GE_OQ (3205) / GT_OQ (2219)
                continue
            tx = ctx.tex
            fx = (cvtt(f32(tx.width) * fu) << 2) & 0xFFFFFFFF
            fy = mul16(cvtt(f32(tx.height) * fv) & 0xFFFFFFFF, tx.pitch) & 0xFFFFFFFF
            off = (fx + fy) & 0xFFFFFFFF
            off = off - (1 << 32) if off & 0x80000000 else off
            if getattr(tx, "filter", 0) == 1:
                C = bilinear(tx, fu, fv)
            else:
                tv = texel(tx, off)
                C = [f32((tv >> 16) & 255) / f32(255), f32((tv >> 8) & 255) / f32(255), f32(tv & 255) / f32(255),
                     f32((tv >> 24) & 255) / f32(255)]
            d = ctx.D - z
            X0 = x - i
            ax = ((f32(X0) + f32(i)) - ctx.cx) * (f32(1) / ctx.M2P)
            ay = ((f32(row) + f32(0)) - ctx.cy) * (f32(1) / ctx.M2P)
            P = [(d / ctx.F) * ax, (d / ctx.F) * ay, z]
            F = shade_phong_avx(ctx, C, P, n)
            col = ((rne(F[0] * f32(255)) << 16) | (rne(F[1] * f32(255)) << 8) | rne(F[2] * f32(255)) |
                   (rne(F[3] * f32(255)) << 24)) & 0xFFFFFFFF
            ctx.z[row, x] = z
            ctx.color[row, x] = col
            ctx.win[row, x] = t


def span_scalar(ctx, t, L, R, row):
    W = ctx.W
    xoff = f32(0)
    xd = f32(roundf(R["X"] - L["X"]))
    with np.errstate(all="ignore"):
        def inc(a, b):
            return (b - a) / xd if xd != 0 else f32(0)
        iz, iw, iu, iv = inc(L["Z"], R["Z"]), inc(L["W"], R["W"]), inc(L["U"], R["U"]), inc(L["V"], R["V"])
        ic = [inc(L["C"][k], R["C"][k]) for k in range(4)]
        inn = [inc(L["N"][k], R["N"][k]) for k in range(3)]
        lx = L["X"]
        if lx < 0:
            xoff, lx = -L["X"], f32(0)
        elif lx >= W:
            lx = f32(W) - f32(1)
        rx = R["X"]
        if rx < 0:
            rx = f32(0)
        elif rx >= W:
            rx = f32(W) - f32(1)
        if lx != lx or rx != rx:
            return
        mnx, mxx = round_s32(lx), round_s32(rx)
        z = L["Z"] + xoff * iz
        w, u, v = L["W"] + xoff * iw, L["U"] + xoff * iu, L["V"] + xoff * iv
        n = [L["N"][k] + xoff * inn[k] for k in range(3)]
        c = [L["C"][k] + xoff * ic[k] for k in range(4)]
        for x in range(mnx, mxx + 1):
            lin = row * W + x
            if lin < W * ctx.H:
                rr, xx = divmod(lin, W)
                C = list(c)
                if ctx.tex is not None:
                    sc = f32(1) / w
                    fu, fv = sc * u, sc * v
                    tx_ = round_s32(fu * f32(ctx.tex.width - 1))
                    ty_ = round_s32(fv * f32(ctx.tex.height - 1))
                    off = (tx_ * 4 + ty_ * ctx.tex.pitch) & 0xFFFFFFFF
                    off = off - (1 << 32) if off & 0x80000000 else off
                    tv = texel(ctx.tex, off)
                    C = [f32((tv >> 16) & 255) / f32(255), f32((tv >> 8) & 255) / f32(255),
                         f32(tv & 255) / f32(255), f32((tv >> 24) & 255) / f32(255)]
                if ctx.phong:
                    d = ctx.D - z
                    P = [(d / ctx.F) * ((f32(x) - ctx.cx) * (f32(1) / ctx.M2P)),
                         (d / ctx.F) * ((f32(row) - ctx.cy) * (f32(1) / ctx.M2P)), z]
                    F = [f32(0)] * 4
                    for li, (lp, I) in enumerate(ctx.lights):
                        if li == 0:
                            F = [C[k] * ctx.amb[k] for k in range(4)]
                        Lv = norm_rcp([lp[k] - P[k] for k in range(3)])
                        cos = clamp01((n[0] * Lv[0] + n[1] * Lv[1]) + n[2] * Lv[2])
                        Vv = norm_rcp([-P[0], -P[1], -P[2]])
                        Hv = norm_rcp([Lv[k] + Vv[k] for k in range(3)])
                        ph = clamp01((n[0] * Hv[0] + n[1] * Hv[1]) + n[2] * Hv[2])
                        ph = f32(math.pow(float(ph), 16.0))
                        F = [F[k] + ((cos * (C[k] * I[k])) + (ph * (f32(1) * I[k]))) for k in range(4)]
                    F = [clamp01(F[k]) for k in range(4)]
                else:
                    F = C
                col = ((round_u32(F[3] * f32(255)) << 24) | (round_u32(F[0] * f32(255)) << 16) |
                       (round_u32(F[1] * f32(255)) << 8) | round_u32(F[2] * f32(255))) & 0xFFFFFFFF
                if z > ctx.z[rr, xx]:
                    ctx.z[rr, xx] = z
                    ctx.color[rr, xx] = col
                    ctx.win[rr, xx] = t
            if ctx.phong:
                n = norm_rcp([n[k] + inn[k] for k in range(3)])
            c = [c[k] + ic[k] for k in range(4)]
            z = z + iz
            w, u, v = w + iw, u + iu, v + iv


def render(scene, semantics=1, phong=True, setup=None, setup_camera=None):
    ctx = Ctx(scene, semantics, phong, setup=setup, setup_camera=setup_camera)
    with np.errstate(all="ignore"):
        for t in range(scene.tri_count):
            walk(ctx, t, edge_table(ctx, t))
    return ctx.color, ctx.z, ctx.win
