"""Row-band sharding of one frame over N ranks.

Rank r of N owns frame rows [r*H/N, (r+1)*H/N).  Every rank bins all
triangles against its own band (no pixel belongs to two ranks, triangles stay
in submission order), so the only exchange is the final gather of the colour
(and optionally z) strips to rank 0.  On GPUs this runs over RCCL (backend
"nccl"), on CPUs over gloo; both use the same calls below.
"""


def band_rows(rank, world, height):
    return height * rank // world, height * (rank + 1) // world


def max_band_rows(world, height):
    return max(band_rows(r, world, height)[1] - band_rows(r, world, height)[0] for r in range(world))


def gather_strips(dist, strip, rank, world, height, out=None):
    """Gather every rank's [rows_r, W] strip into rank 0's [H, W] frame.

    Strips are padded to the largest band so one all_gather_into_tensor
    moves them (one message per peer over xGMI); rank 0 then drops the
    padding.  Returns the full frame on rank 0, None elsewhere."""
    import torch

    W = strip.shape[1]
    rows = strip.shape[0]
    mr = max_band_rows(world, height)
    if rows == mr:
        send = strip.contiguous()
    else:
        send = torch.zeros((mr, W), dtype=strip.dtype, device=strip.device)
        send[:rows] = strip
    recv = torch.empty((world * mr, W), dtype=strip.dtype, device=strip.device)
    dist.all_gather_into_tensor(recv, send)
    if rank != 0:
        return None
    if out is None:
        out = torch.empty((height, W), dtype=strip.dtype, device=strip.device)
    for r in range(world):
        a, b = band_rows(r, world, height)
        out[a:b] = recv[r * mr: r * mr + (b - a)]
    return out
