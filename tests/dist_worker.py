"""Worker for tests/test_dist.py: one rank of a row-band sharded frame on CPU
(gloo).  Each rank draws its band with the CPU restatement (standing in for
the GPU kernel, which uses the same band and the same gather over RCCL in
bench.py), then the strips are gathered to rank 0 with prk.dist.
usage: torch.distributed.run ... tests/dist_worker.py OUT.npz SEMANTICS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle as O  # noqa: E402
from prk import dist as pdist  # noqa: E402
from prk import scenes  # noqa: E402


def main():
    out, sem = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    s = scenes.random_soup(4000, 200, 150, radius=20, seed=99, textured=True)
    r0, r1 = pdist.band_rows(rank, world, s.height)
    col, z, win, _ = O.render(s, semantics=sem, phong=sem == 1, rows=(r0, r1))
    strips = [torch.from_numpy(np.ascontiguousarray(a[r0:r1]).view(np.int32)) for a in (col, z, win)]
    full = [pdist.gather_strips(dist, t, rank, world, s.height) for t in strips]
    if rank == 0:
        np.savez(out, color=full[0].numpy().view(np.uint32), z=full[1].numpy().view(np.float32),
                 winners=full[2].numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
