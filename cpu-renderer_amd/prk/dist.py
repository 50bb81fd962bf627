"""Row-band sharding of one frame over N ranks.

Rank r of N owns frame rows [r*H/N, (r+1)*H/N).  Every rank bins all
triangles against its own band (no pixel belongs to two ranks, triangles stay
in submission order), so the only exchange is the final gather of the colour
(and optionally z) strips to rank 0.  On GPUs this runs over RCCL (backend
"nccl"), on CPUs over gloo; both use the same calls below.
"""


def band_rows(rank, world, height):
    """Rank `rank`'s rows: the C-ABI's prk_band_rows, the same split the C++
    drop-in (PRK_InitDevices) and prk_gather_frame use."""
    from . import band_rows as c_band_rows
    return c_band_rows(height, rank, world)


def max_band_rows(world, height):
    return max(band_rows(r, world, height)[1] - band_rows(r, world, height)[0] for r in range(world))


def gather_strips(dist, strip, rank, world, height, out=None):
    """Blocking form of gather_strips_start: the current stream (GPU) or the
    host (CPU) waits for the gather."""
    out, reqs = gather_strips_start(dist, strip, rank, world, height, out=out)
    for req in reqs:
        req.wait()
    return out


def gather_strips_start(dist, strip, rank, world, height, out=None):
    """Gather every rank's [rows_r, W] strip into rank 0's [H, W] frame.

    Point to point: every rank r > 0 sends its strip to rank 0, which
    receives it straight into its slice of the frame (one message per peer,
    each on its own xGMI link; no padding, no all-gather of the whole frame
    to every rank).  Rank 0's own strip is copied unless it already is that
    slice (bench.py renders rank 0's band in place).  Returns (the frame on
    rank 0 / None elsewhere, the pending requests): on RCCL the transfers run
    on the communicator's stream, so rendering the next frame into another
    strip buffer overlaps them; req.wait() orders the current stream after
    them (call it before the strip or frame is reused).

    When `strip` is a prk target just flushed, call Renderer.resolve(stream)
    (prk_resolve) first: a frame whose bin entries overflowed the scratch is
    re-run when its count is resolved, and the sends must come after that
    (prk_gather_frame does this itself)."""
    import torch

    W = strip.shape[1]
    if rank == 0:
        if out is None:
            out = torch.empty((height, W), dtype=strip.dtype, device=strip.device)
        a, b = band_rows(0, world, height)
        if out[a:b].data_ptr() != strip.data_ptr():
            out[a:b].copy_(strip)
        ops = []
        for r in range(1, world):
            a, b = band_rows(r, world, height)
            ops.append(dist.P2POp(dist.irecv, out[a:b], r))
    else:
        ops = [dist.P2POp(dist.isend, strip.contiguous(), 0)]
    reqs = dist.batch_isend_irecv(ops) if ops else []
    return (out if rank == 0 else None), reqs
