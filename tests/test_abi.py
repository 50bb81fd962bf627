"""CPU tests of the C-ABI boundary (no GPU compute).

* libprk_hip.so loads and exports every entry point include/prk.h declares.
* The product library does not link the oracle.
* Host-only entry points work without a device (ConstructSphere, argument
  checks); compute entry points fail loudly (PRK_ERR_DEVICE) when no GPU is
  visible instead of falling back to the CPU.
* The C++ drop-in header (include/projekt.h) compiles against the reference's
  call pattern (examples/dropin_demo.cpp) and links against the library.
"""
import ast
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import prk
from prk import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    with open(os.path.join(ROOT, "include", "prk.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(prk_[a-z_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    names = declared()
    assert len(names) >= 20
    lib = prk.lib()  # (the binding's load order: torch's ROCm first)
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(prk.exported_symbols())
    out = subprocess.run(["nm", "-D", "--defined-only", prk.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(r"\bT %s$" % n, out, re.M), n


def test_product_does_not_link_the_oracle():
    out = subprocess.run(["readelf", "-d", prk.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    assert "libamdhip64" in out  # the HIP runtime is the compute path


def test_struct_layouts_match_header():
    assert C.sizeof(abi.PrkTransform) == 20
    assert C.sizeof(abi.PrkLightInfo) == 28
    assert C.sizeof(abi.PrkLightData) == 4 + 16 + 8 * 28
    assert C.sizeof(abi.PrkBitmap) == 8 + 12 + 4  # pointer + 3 ints (+ tail padding)


def test_argument_errors_without_device():
    L = prk.lib()
    assert L.prk_destroy(None) == abi.PRK_ERR_ARG
    assert L.prk_device_count(None) == abi.PRK_ERR_ARG
    assert L.prk_create(0, None) == abi.PRK_ERR_ARG
    assert L.prk_construct_sphere(None, None, None, None, None) == abi.PRK_ERR_ARG
    assert L.prk_resolve(None, None) == abi.PRK_ERR_ARG
    assert L.prk_synchronize(None) == abi.PRK_ERR_ARG
    assert L.prk_version() .startswith(b"prk")


def test_construct_sphere_host():
    V, Cc, N, UV = prk.construct_sphere()
    assert V.shape == (6624, 3)
    r = np.linalg.norm(V, axis=1)
    assert np.allclose(r, 0.5, atol=1e-5)           # Radius*FirstVertex, r = 0.5 (4127)
    assert np.allclose(np.linalg.norm(N, axis=1), 1.0, atol=1e-5)
    assert np.array_equal(Cc[0], np.array([1, 0, 1, 1], np.float32))  # UpColor + Blue(az 0)


@pytest.mark.skipif(os.environ.get("PRK_EXPECT_GPU") == "1", reason="GPU box")
def test_compute_fails_loudly_without_gpu():
    if prk.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(prk.PrkError) as e:
        prk.Renderer()
    assert e.value.code == abi.PRK_ERR_DEVICE


def test_dropin_header_builds_and_links(tmp_path):
    exe = tmp_path / "dropin_demo"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "examples", "dropin_demo.cpp"), "-L",
                        os.path.join(ROOT, "cpu-renderer_amd"), "-lprk_hip",
                        "-Wl,-rpath," + os.path.join(ROOT, "cpu-renderer_amd"), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    if prk.device_count() == 0:
        run = subprocess.run([str(exe), str(tmp_path / "c"), str(tmp_path / "z")], capture_output=True, text=True)
        assert run.returncode == 2 and "no HIP device" in run.stderr


@pytest.mark.parametrize("per", [1, 5, 60])
def test_fill_edge_count_matches_oracle(per):
    """prk_fill_edge_count (what the drop-in's FillEdgeTable returns,
    projekt.cpp:4119) equals the oracle's FillEdgeTable edge count for every
    object: back-facing objects (0), the near plane, clipping on every side,
    horizontal edges."""
    import oracle as O
    from prk import scenes
    s = scenes.random_soup(1200, 256, 192, radius=60, seed=31, centroid_margin=80)
    rng = np.random.default_rng(3)
    v = s.vertices.reshape(-1, 3, 3)
    flip = rng.random(v.shape[0]) < 0.3  # back-facing: swap two vertices
    v[flip, 1], v[flip, 2] = v[flip, 2].copy(), v[flip, 1].copy()
    v[rng.random(v.shape[0]) < 0.05, 0, 2] = 3.9  # a vertex at the near plane
    flat = rng.random(v.shape[0]) < 0.05  # a horizontal edge
    v[flat, 1, 1] = v[flat, 0, 1]
    s.vertices = v.reshape(-1, 3)
    T = s.prk_transform()
    for t0 in range(0, s.tri_count, per):
        n = min(per, s.tri_count - t0)
        want = len(O.fill_edge_table(s, t0, n))
        got = prk.fill_edge_count(s.vertices[3 * t0:3 * (t0 + n)], s.P, T)
        assert got == want, (t0, n, got, want)


ROCM_MAP_RE = r"(/\S*(?:libamdhip64|librccl|librocm_smi64|libhsa-runtime64)\S*)"
LOAD_ORDER_CHILD = """
import re, sys
sys.path.insert(0, {pkg!r})
import prk
assert prk.comm_available()  # dlopens librccl, as prk.Comm does
import torch  # noqa: F401
print(sorted(set(re.findall({rx!r}, open('/proc/self/maps').read()))))
"""


def _needs_torch_and_rccl():
    pytest.importorskip("torch")
    if not prk.comm_available():
        pytest.skip("librccl not loadable here")


REVERSED_ORDER_CHILD = """
import ctypes, sys
L = ctypes.CDLL({lib!r})                       # /opt/rocm's HIP runtime, first
assert L.prk_comm_available() == 1             # dlopens /opt/rocm's librccl (+ librocm_smi64)
import torch  # noqa: F401                     # torch's own copies beside them
h = ctypes.c_void_p()
print("create", L.prk_create(0, ctypes.byref(h)), "check", L.prk_runtime_check())
"""


def test_reversed_load_order_reported_and_exit_guarded():
    """libprk_hip.so and RCCL loaded BEFORE torch (the order the binding
    avoids): prk_create returns PRK_ERR_RUNTIME_MIX, names the fix on stderr,
    and the process still exits 0 -- the on_exit guard ends it before the two
    librocm_smi64 copies' destructors free one map twice."""
    _needs_torch_and_rccl()
    code = REVERSED_ORDER_CHILD.format(lib=prk.LIB_PATH)
    run = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0 and "double free" not in run.stderr, (run.returncode, run.stderr[-2000:])
    assert "create %d check %d" % (abi.PRK_ERR_RUNTIME_MIX, abi.PRK_ERR_RUNTIME_MIX) in run.stdout, run.stdout
    assert "BEFORE libprk_hip.so" in run.stderr
    # ... and with an exit status of its own, that status survives the guard
    run = subprocess.run([sys.executable, "-c", code + "sys.exit(3)\n"], capture_output=True, text=True,
                         timeout=300)
    assert run.returncode == 3, (run.returncode, run.stderr[-2000:])


def test_runtime_check_clean_process():
    """One ROCm stack (this test process, the binding's load order): OK."""
    assert prk.lib().prk_runtime_check() == abi.PRK_OK


def test_one_rocm_runtime_per_process():
    """The binding loads torch's ROCm libraries before libprk_hip.so, so a
    process that uses both maps one HIP runtime, one RCCL and one
    librocm_smi64: loaded the other way round, the process maps
    /opt/rocm's copies and torch's side by side, and the two librocm_smi64
    copies' exit-time destructors free one interposed static map twice (glibc
    "double free or corruption", rc 134 — the round-3/4 exit aborts)."""
    _needs_torch_and_rccl()
    code = LOAD_ORDER_CHILD.format(pkg=os.path.join(ROOT, "cpu-renderer_amd"), rx=ROCM_MAP_RE)
    run = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0 and "double free" not in run.stderr, (run.returncode, run.stderr[-2000:])
    libs = ast.literal_eval(run.stdout.strip().splitlines()[-1])
    for name in ("libamdhip64", "librccl", "librocm_smi64", "libhsa-runtime64"):
        assert len([p for p in libs if name in os.path.basename(p)]) == 1, libs
