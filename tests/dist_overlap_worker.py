"""Worker for tests/test_dist.py: the double-buffered, overlapped gather of
bench.py on CPU (gloo).  Frame k is drawn (here: filled with a per-rank,
per-frame pattern) into strip buffer k % 2 while frame k-1's gather may still
be in flight; a buffer is reused only after its previous gather's requests
completed.  Rank 0 checks the last two gathered frames.
usage: torch.distributed.run ... tests/dist_overlap_worker.py FRAMES"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from prk import dist as pdist  # noqa: E402


def main():
    nframes = int(sys.argv[1])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    H, W = 37, 16
    r0, r1 = pdist.band_rows(rank, world, H)
    frames = [torch.full((H, W), -1, dtype=torch.int32) if rank == 0 else None for _ in range(2)]
    strips = [f[r0:r1] if f is not None else torch.empty((r1 - r0, W), dtype=torch.int32) for f in frames]
    pending = [[], []]
    for k in range(nframes):
        b = k % 2
        for req in pending[b]:
            req.wait()
        strips[b].fill_(1000 * k + rank)  # "render" frame k into its buffer
        _, pending[b] = pdist.gather_strips_start(dist, strips[b], rank, world, H, out=frames[b])
    for b in range(2):
        for req in pending[b]:
            req.wait()
    if rank == 0:
        for k in (nframes - 2, nframes - 1):
            f = frames[k % 2]
            for r in range(world):
                a, c = pdist.band_rows(r, world, H)
                assert (f[a:c] == 1000 * k + r).all(), (k, r)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
