"""bench.py — headline benchmark of the MI355X rasterizer.

Metric (BASELINE.json): Mpixels/s shaded at 4096x4096, 1M triangles (+ Mtri/s),
on 1/2/4/8 GPUs.  Workload = config C3b of SURVEY §8(d): 1M random front-facing
triangles (vertex offsets +-16 px), Phong + 256^2 texture, one light, drawn with
FillLineOptimized semantics (DrawModelOptimized(RenderQueue,...) +
FillLineOptimized, projekt.cpp:3615-3871 / 1492-2320), per-triangle submission.

One step = one frame: clear colour + z (fused into the frame's kernels,
prk_target_clear_on_flush), then bin + raster + shade every triangle into the
frame (inputs already resident in HBM).  With N GPUs the
frame is split into N row bands (rank r owns rows [r*H/N, (r+1)*H/N)), every
rank bins all triangles against its band, and the colour strips are gathered
to rank 0 over RCCL ("scaling": "strong": total work fixed).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # frames are ~1 ms: ~0.1 s timed
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--height", type=int, default=4096)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--radius", type=float, default=16.0)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--tile", type=str, default="")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU path (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-max-tris", type=int, default=1_000_000,
                    help="bound on the CPU sample (triangles of the same scene)")
    ap.add_argument("--check", type=int, default=0, help="compare the frame with the oracle")
    ap.add_argument("--comm", choices=("torch", "prk"), default="torch",
                    help="N > 1 strip gather: torch.distributed P2P (RCCL) or the C-ABI's prk_gather_frame "
                         "(RCCL from libprk_hip.so)")
    return ap.parse_args()


def algorithmic_bytes(T, W, rows, tex_texels):
    """Algorithmic bytes of one frame, SURVEY §8(d): the geometry read once
    (144 B/triangle: v3 position + v4 colour + v3 normal + v2 uv per vertex),
    z and colour of every pixel written once (8 B/pixel: the frame starts
    from a clear fused into its kernels, so no prior z is read), each texel
    read once.  (FillLineOptimized never reads vertex colours, so the bytes
    the AVX path must move are 48 B/triangle fewer; DESIGN.md §5 gives both.)"""
    return 144 * T + 8 * W * rows + 4 * tex_texels


def load_traffic(cfg_key):
    """HBM bytes per frame measured with rocprofv3 PMC passes
    (tools/profile_round.sh -> tools/pmc_traffic.py -> profiles/pmc_traffic.json,
    committed with the round's profiles), or (None, None).  NOT measured by
    this run: the counters need their own rocprofv3 passes."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(cfg_key)
        if e is None:
            return None, None
        return float(e["hbm_bytes_per_frame"]), "profiles/pmc_traffic.json[%s] (%s)" % (cfg_key, e.get("round", "?"))
    except Exception:
        return None, None


def load_valu(cfg_key, kernel, ms_frame=None):
    """The dominant kernel's issued-VALU time estimate and lane utilisation
    from the round's SQ counter passes (tools/profile_round.sh ->
    tools/sqsum.py --json -> profiles/sq_valu.json), or None, and that VALU
    time's share of this run's frame (`valu_frac_of_frame`).  NOT measured by
    this run: SQ counters need their own rocprofv3 passes."""
    p = os.path.join(ROOT, "profiles", "sq_valu.json")
    try:
        with open(p) as f:
            e = json.load(f)[cfg_key]
        k = next(v for n, v in e["per_kernel"].items() if n.startswith(kernel + "<") or n == kernel)
        vt = k.get("valu_time_estimate_ms")
        return dict(kernel=kernel, valu_time_estimate_ms=vt, lane_utilisation=k.get("lane_utilisation"),
                    valu_issue_floor_ms=k.get("valu_issue_floor_ms"), valu_insts=k.get("insts_valu"),
                    valu_frac_of_frame=(vt / ms_frame) if (vt and ms_frame) else None,
                    source="profiles/sq_valu.json[%s] (%s)" % (cfg_key, e.get("round", "?")))
    except (OSError, ValueError, KeyError, StopIteration):
        return None


def load_valu_frame(cfg_key, ms_frame):
    """The frame's issued-VALU time: the sum over every kernel of the round's
    SQ counter passes (profiles/sq_valu.json, as load_valu) of its VALU time
    estimate, and that sum's share of this run's ms_per_step -- how far the
    frame as a whole is from its VALU-issue floor.  None without the file."""
    p = os.path.join(ROOT, "profiles", "sq_valu.json")
    try:
        with open(p) as f:
            e = json.load(f)[cfg_key]
        per = {n: v.get("valu_time_estimate_ms") or 0.0 for n, v in e["per_kernel"].items()}
        tot = sum(per.values())
        return dict(valu_time_ms=tot, frac_of_frame=tot / ms_frame if ms_frame else None, kernels=len(per),
                    source="profiles/sq_valu.json[%s] (%s)" % (cfg_key, e.get("round", "?")))
    except (OSError, ValueError, KeyError):
        return None


def cpu_topology():
    """Host CPUs this process may run on, their physical cores and SMT, and
    the cgroup CPU quota (the box's share of the host)."""
    aff = sorted(os.sched_getaffinity(0))
    cores, model = set(), None
    try:
        cur = {}
        with open("/proc/cpuinfo") as f:
            for ln in f.read().split("\n\n"):
                kv = dict((a.strip(), b.strip()) for a, b in
                          (x.split(":", 1) for x in ln.split("\n") if ":" in x))
                if "processor" not in kv:
                    continue
                model = model or kv.get("model name")
                if int(kv["processor"]) in aff:
                    cores.add((kv.get("physical id", "0"), kv.get("core id", kv["processor"])))
                cur = kv
        del cur
    except (OSError, ValueError, KeyError):
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    phys = len(cores) or None
    return dict(affinity_cpus=len(aff), physical_cores=phys,
                smt=(len(aff) / phys) if phys else None, cgroup_cpu_quota=quota, cpu_model=model,
                host_cpus=os.cpu_count())


def _cpu_share(threads, topo):
    """The CPUs the baseline actually had: its thread count, capped by the
    cgroup CPU quota (on the GPU box 16 CPUs of a 256-CPU host: 64 threads
    there time-share 16 CPUs' worth)."""
    q = topo.get("cgroup_cpu_quota")
    return min(float(threads), float(q)) if q else float(threads)


def cpu_baseline(scene, threads, max_tris, frames=3, scan=(16, 64)):
    """The CPU path on the same scene, on the host cores (SURVEY §8(d) "CPU
    path timing"): the AVX2 restatement (oracle/prk_cpu_avx.c, bit-exact to
    the scalar oracle), scanned up to `threads` = every CPU of this process's
    affinity mask, under three schedules:
      banded  row bands per thread, no locks (median of `frames` full frames
              after one warm-up);
      queue   the reference's DrawModelOptimized(RenderQueue,...): a producer
              AET posts one task per span, workers take the per-8-px ZMask
              spinlock (projekt.cpp:3615-3871, 2202-2239);
      rows    DrawModelOptimizedLines + FillLinesOptimized: one task per row
              of an object (projekt.cpp:3362-3613, 629-1490).
    queue / rows are timed on a bounded sample (the scene's first triangles)
    and scaled to the scene.  The banded schedule runs at every count of
    `scan`, the cgroup CPU quota and `threads`; `value` is the fastest
    schedule at the fastest count (on the GPU box the cgroup quota is 16 CPUs
    of 256, and 256 threads run slower than 64)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from prk import abi
    T = scene.tri_count
    px = scene.width * scene.height
    topo = cpu_topology()
    if O.cpu_lib() is None:  # no AVX2 on this host: the scalar port, banded
        n = min(T, max_tris)
        sub = scene if n == T else scene.subset(0, n)
        t0 = time.perf_counter()
        _, _, _, st = O.render(sub, semantics=abi.PRK_SEM_AVX, phong=True, threads=threads, winners=False)
        frame = (time.perf_counter() - t0) * (T / n)
        return dict(value=px / frame / 1e6, unit="Mpixels/s", cores=_cpu_share(threads, topo), threads=threads,
                    kind="port",
                    sample="scalar oracle (no AVX2 on this host), %d of %d triangles, banded over %d threads"
                           % (n, T, threads), frame_s=frame, span_pixels=st["span_pixels"] if n == T else None,
                    **topo)

    def timed(sub, cpu, th, nframes):
        ts, st = [], None
        for i in range(nframes + 1):
            t0 = time.perf_counter()
            _, _, _, st = O.render(sub, semantics=abi.PRK_SEM_AVX, phong=True, threads=th, winners=False, cpu=cpu)
            if i:
                ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), st

    n = min(T, max_tris)
    sub = scene if n == T else scene.subset(0, n)
    # banded thread scan: 16, 64, the cgroup CPU quota (the box's share of
    # the host), every CPU of the affinity mask; the fastest count is the
    # one the other schedules run at and the one `cores` reports.
    counts = sorted({th for th in scan if th < threads} | {threads} |
                    ({int(topo["cgroup_cpu_quota"])} if topo.get("cgroup_cpu_quota") and
                     1 <= topo["cgroup_cpu_quota"] < threads else set()))
    scan_out, st = {}, None
    for th in counts:
        f, s_ = timed(sub, "banded", th, frames)
        st = st or s_
        f *= T / n
        scan_out[str(th)] = {"frame_ms": f * 1e3, "mpixels_s": px / f / 1e6}
    tbest = int(min(scan_out, key=lambda k: scan_out[k]["frame_ms"]))
    fb = scan_out[str(tbest)]["frame_ms"] * 1e-3
    variants = {"banded": {"threads": tbest, "frame_ms": fb * 1e3, "mpixels_s": px / fb / 1e6,
                           "sample": "%d of %d triangles, median of %d frames" % (n, T, frames)}}
    nq = min(n, 20_000)
    subq = scene.subset(0, nq) if nq < T else scene
    for sched in ("queue", "rows"):
        fq, _ = timed(subq, sched, tbest, 2)
        fq *= T / nq
        variants[sched] = {"threads": tbest, "frame_ms": fq * 1e3, "mpixels_s": px / fq / 1e6,
                           "sample": "first %d triangles, median of 2 frames, scaled to T" % nq}
    best = min(variants, key=lambda k: variants[k]["frame_ms"])
    frame = variants[best]["frame_ms"] * 1e-3
    return dict(value=px / frame / 1e6, unit="Mpixels/s", cores=_cpu_share(tbest, topo), threads=tbest, kind="port",
                sample="AVX2 restatement of FillLineOptimized (oracle/prk_cpu_avx.c); banded schedule scanned "
                       "over %s threads (%d = every CPU of the affinity mask), value = fastest schedule (%s) at "
                       "the fastest count (%d threads); banded: %s; queue/rows: %s"
                       % ("/".join(map(str, counts)), threads, best, tbest, variants["banded"]["sample"],
                          variants["queue"]["sample"]),
                variants=variants, banded_thread_scan=scan_out, frame_s=frame,
                span_pixels=st["span_pixels"] if n == T else None, **topo)


def main():
    a = parse()
    import torch
    import prk
    from prk import abi, scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.stderr.write("bench: --gpus %d needs torch.distributed.run (WORLD_SIZE)\n" % a.gpus)
            sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    W, H = a.width, a.height
    scene = scenes.random_soup(a.tris, W, H, radius=a.radius, seed=a.seed, textured=True)
    from prk.dist import band_rows
    row0, row1 = band_rows(rank, world, H)
    rows = row1 - row0

    # N > 1: two strip (and, on rank 0, frame) buffers, so frame k's RCCL
    # gather runs on the communicator's stream while frame k+1 renders into the
    # other buffer; a buffer is reused only after its gather completed.
    nbuf = 2 if world > 1 else 1
    frames = [torch.empty((H, W), dtype=torch.int32, device=dev) if (world > 1 and rank == 0) else None
              for _ in range(nbuf)]
    # rank 0 renders its band straight into its slice of the gathered frame
    colors = [f[row0:row1] if f is not None else torch.empty((rows, W), dtype=torch.int32, device=dev)
              for f in frames]
    color = colors[0]
    zbuf = torch.empty((rows, W), dtype=torch.float32, device=dev)
    r = prk.Renderer(dev)
    r.target_bind(color.data_ptr(), W * 4, zbuf.data_ptr(), W, H, row0, row1)
    if a.tile:
        tw, th = [int(x) for x in a.tile.split("x")]
        r.set_tile(tw, th)
    r.set_camera(scene.prk_transform(), scene.prk_lights())
    torch.cuda.synchronize()
    t_up = time.perf_counter()
    geom = r.geometry(scene.vertices, None, scene.normals, scene.uvs)  # AVX path: no colours read
    tex = r.texture(scene.texture)
    torch.cuda.synchronize()
    ms_upload = (time.perf_counter() - t_up) * 1e3  # host -> HBM, once per scene (not in `value`)
    stream = torch.cuda.current_stream().cuda_stream
    from prk import dist as pdist
    zmin = -float(np.finfo(np.float32).max)

    pending = [[] for _ in range(nbuf)]
    nstep = [0]
    comm = comm_stream = None
    if a.comm == "prk":  # the C-ABI's RCCL gather (prk_comm_init / prk_gather_frame)
        uid = [prk.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        comm = prk.Comm.init(r, uid[0], world, rank)
        comm_stream = torch.cuda.Stream()

    def step():
        b = nstep[0] % nbuf
        nstep[0] += 1
        for req in pending[b]:  # this buffer's previous gather has landed
            req.wait()
        pending[b] = []
        if nbuf > 1:
            r.target_bind(colors[b].data_ptr(), W * 4, zbuf.data_ptr(), W, H, row0, row1)
        # clear colour + z (the reference's clear values), fused into the
        # frame's kernels: every pixel of the band is written by the frame
        r.clear_on_flush(0xFF000000, zmin)
        r.draw_model_optimized(geom, scene.tri_count, bitmap=tex, phong=True)
        r.complete_all_work(stream)
        if world > 1 and comm is not None:  # prk_gather_frame on its own stream
            ev = torch.cuda.Event()
            ev.record()
            comm_stream.wait_event(ev)
            comm.gather(r, frames[b].data_ptr() if rank == 0 else None, None, with_z=False,
                        stream=comm_stream.cuda_stream)
            done = torch.cuda.Event()
            done.record(comm_stream)
            pending[b] = [done]  # Event.wait(): the render stream waits for it
        elif world > 1:  # RCCL over xGMI: strips -> rank 0's frame
            r.resolve(stream)  # an overflowed frame is re-run before its strip is sent
            _, pending[b] = pdist.gather_strips_start(dist, colors[b], rank, world, H, out=frames[b])

    def drain():
        for b in range(nbuf):
            for req in pending[b]:
                req.wait()
            pending[b] = []

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    r.timing_reset()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()  # every frame's gather is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # Per-kernel device time in the timed (pipelined) frames: HIP events
    # recorded on the launch streams; frames overlap, so these are stretched
    # spans, not serial shares of a frame.
    stats = r.stats()
    nt = max(1, stats["frames_timed"])
    ms_bin = stats["sum_ms_bin"] / nt
    ms_raster = stats["sum_ms_raster"] / nt
    ms_vis = stats["sum_ms_vis"] / nt
    ms_span = stats["sum_ms_span"] / nt
    ms_pix = ms_raster - ms_vis - ms_span
    # Serial kernel times (outside the timed region): the same frame with the
    # host waiting for each frame, so no kernel overlaps another frame's.
    r.timing_reset()
    for _ in range(5):
        step()
        drain()
        torch.cuda.synchronize()
    ss = r.stats()
    ns = max(1, ss["frames_timed"])
    serial = {"k_bin_phase": ss["sum_ms_bin"] / ns, "k_vis": ss["sum_ms_vis"] / ns,
              "k_walk": ss["sum_ms_span"] / ns,
              "k_pix": (ss["sum_ms_raster"] - ss["sum_ms_vis"] - ss["sum_ms_span"]) / ns,
              "raster": ss["sum_ms_raster"] / ns}
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt * 1000.0 / a.steps
    # Frame download (colour + z of this rank's band, HBM -> host), outside
    # the timed region: reported separately.
    r.synchronize()  # the last frame's bin count is read (an overflowed frame re-run) before torch reads the target
    host_c = torch.empty(color.shape, dtype=color.dtype, pin_memory=True)
    host_z = torch.empty(zbuf.shape, dtype=zbuf.dtype, pin_memory=True)
    torch.cuda.synchronize()
    t_dn = time.perf_counter()
    host_c.copy_(color, non_blocking=True)
    host_z.copy_(zbuf, non_blocking=True)
    torch.cuda.synchronize()
    ms_download = (time.perf_counter() - t_dn) * 1e3

    check = None
    if a.check and rank == 0 and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        oc, oz, _, _ = O.render(scene, threads=min(16, os.cpu_count() or 1), winners=False)
        gc = color.cpu().numpy().view(np.uint32)
        gz = zbuf.cpu().numpy()
        check = dict(z_mismatch=int((gz.view(np.uint32) != oz.view(np.uint32)).sum()),
                     color_mismatch=int((gc != oc).sum()))

    if rank != 0:
        if comm is not None:
            comm.close()
        if dist is not None:
            dist.destroy_process_group()
        return
    T = scene.tri_count
    tex_texels = scene.texture.width * scene.texture.height
    alg = algorithmic_bytes(T, W, rows, tex_texels)
    # Roofline of the whole frame (every kernel of the step): SURVEY §8(d)'s
    # algorithmic bytes per frame over the measured time per frame.
    achieved = alg / (ms * 1e-3) / 1e9
    cfg_key = "%dx%d_T%d_r%g_N%d" % (W, H, T, a.radius, world)
    traffic, traffic_src = load_traffic(cfg_key)
    out = {
        "metric": "Mpixels/s shaded (+ Mtri/s) at 4096x4096, 1M tris; 1/2/4/8 GPUs",
        "value": W * H / (ms * 1e-3) / 1e6,
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded random triangle soup + random 256x256 texture; SURVEY C3b)",
        "config": {"workload": "C3b: %dx%d, %d random triangles (offsets +-%g px), Phong + texture, "
                               "FillLineOptimized semantics, per-triangle submission"
                               % (W, H, T, a.radius),
                   "width": W, "height": H, "triangles": T, "radius_px": a.radius,
                   "lights": len(scene.lights), "texture": "256x256",
                   "parallelism": ("row bands x%d + RCCL gather (%s)" % (world, "prk_gather_frame" if comm
                                                                          else "torch.distributed")
                                   if world > 1 else "1 GPU"),
                   "tile": a.tile or "256x8"},
        "mtri_per_s": T / (ms * 1e-3) / 1e6,
        # binning runs on its own stream, overlapping the previous frame's
        # raster: ms_bin is its (stretched) span, not a serial share of the frame
        # pipelined frames: HIP-event spans stretched by the overlap with the
        # neighbouring frames' kernels (not serial shares of ms_per_step)
        "ms_bin_overlapped": ms_bin,
        "ms_raster_overlapped": ms_raster,
        "ms_kernels_overlapped": {"k_vis": ms_vis, "k_walk": ms_span, "k_pix": ms_pix},
        # serial: 5 more frames with the host waiting after each one
        "ms_kernels_serial": serial,
        "bin_entries": int(stats["bin_entries"]),
        "ms_upload": ms_upload,
        "ms_download": ms_download,
        # Whole frame against HBM: SURVEY §8(d) algorithmic bytes / ms_per_step.
        # `bound` names the roofline `frac` is priced on (the contract's
        # hbm|mfma); what actually limits the frame is `limiter`: the dominant
        # kernel (k_vis) is VALU-issue-bound, not HBM-bound (DESIGN.md §5,
        # profiles/r04/sq_summary.txt), its VALU time and that time's share
        # of the frame are in `valu`.
        "roofline": {"bound": "hbm", "limiter": "valu-issue (k_vis); no kernel of the frame is HBM-bound",
                     "kernel": "whole frame (binning + k_vis + k_walk + k_pix)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src, "algorithmic_bytes": alg,
                     "dominant_kernel": {"name": "k_vis", "ms_serial": serial["k_vis"],
                                         "share_of_serial_frame": serial["k_vis"] / max(
                                             1e-9, serial["raster"] + serial["k_bin_phase"])},
                     # the frame's algorithmic bytes over the dominant kernel's
                     # own serial time (HIP events on its stream, host-synchronised
                     # frames; rocprofv3 of the same frames:
                     # profiles/r06/kernel_stats_serial.csv)
                     "dominant_frac": alg / (serial["k_vis"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     # the binding resource of the dominant kernel: issued VALU
                     # (SQ counters of the committed round profile)
                     "valu": load_valu(cfg_key, "k_vis", ms),
                     # every kernel's VALU time over the frame (SQ counters)
                     "valu_frame": load_valu_frame(cfg_key, ms)},
    }
    if check is not None:
        out["check"] = check
    if a.cpu_baseline and world == 1:
        threads = a.cpu_threads or len(os.sched_getaffinity(0))
        cb = cpu_baseline(scene, threads, a.cpu_max_tris)
        out["cpu_baseline"] = cb
        cb.pop("frame_s", None)
        spx = cb.pop("span_pixels", None)
        if spx:  # the reference's unit of work: span pixels
            out["mfrag_per_s"] = spx / (ms * 1e-3) / 1e6
            out["span_pixels"] = int(spx)
        out["gpu_vs_cpu"] = out["value"] / cb["value"]
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out))
    if comm is not None:
        comm.close()
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
