"""Multi-rank path on CPU (gloo, world_size 2 and 3): row bands + strip gather
reproduce the single-rank frame bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from prk import abi, scenes
from prk import dist as pdist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_band_rows_c_abi():
    """prk_band_rows (C-ABI) is the split r*H/N in 64-bit arithmetic and
    rejects bad arguments."""
    import prk
    for world in (1, 2, 3, 5, 8):
        for H in (1, 7, 150, 4096, 4097, 8192, 2**31 - 1):
            for r in range(world):
                assert prk.band_rows(H, r, world) == (H * r // world, H * (r + 1) // world)
    for bad in ((0, 0, 1), (16, 2, 2), (16, -1, 2), (16, 0, 0)):
        with pytest.raises(prk.PrkError):
            prk.band_rows(*bad)


def test_band_rows_partition():
    for world in (1, 2, 3, 8):
        for H in (150, 4096, 4097):
            bands = [pdist.band_rows(r, world, H) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == H
            assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("world,sem", [(2, abi.PRK_SEM_AVX), (3, abi.PRK_SEM_SCALAR)])
def test_gloo_band_gather_matches_single_rank(tmp_path, world, sem):
    out = str(tmp_path / "frame.npz")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), out, str(sem)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    s = scenes.random_soup(4000, 200, 150, radius=20, seed=99, textured=True)
    col, z, win, _ = O.render(s, semantics=sem, phong=sem == abi.PRK_SEM_AVX)
    assert (got["color"] == col).all()
    assert (got["z"].view(np.uint32) == z.view(np.uint32)).all()
    assert (got["winners"] == win).all()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_overlapped_double_buffered_gather(world):
    """bench.py's N > 1 loop: gathers left in flight while the next frame is
    drawn into the other buffer land intact."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "dist_overlap_worker.py"), "7"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
