"""Sanitizer runs of the CPU-side code (CPU only, no GPU).

* TSan: the AVX2 baseline (`oracle/prk_cpu_avx.c`: lock-free span ring and
  per-8-px ZMask byte spinlocks of the reference's work queue, the per-row
  task schedule, the banded threads) built `-fsanitize=thread`, driven by
  tests/san_worker.py in a child process with the TSan runtime preloaded.
* ASan + UBSan: the scalar restatement and the AVX2 baseline built
  `-fsanitize=address,undefined`, running the oracle tests (golden fixtures,
  clipping, near plane, edge tables, caller edge / span lists) and the
  baseline tests in a child pytest.

The libraries come from `make -C oracle san` (oracle/_san/, git-ignored);
oracle.py loads them when PRK_ORACLE_LIBDIR points there.
"""
import os
import subprocess
import sys

import pytest

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ORACLE = os.path.join(_ROOT, "oracle")


def _runtime(name):
    try:
        p = subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True,
                           check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def san_libs():
    if _runtime("libtsan.so") is None or _runtime("libasan.so") is None:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", _ORACLE, "san"], check=True)
    return os.path.join(_ORACLE, "_san")


def _env(runtime, libdir, **extra):
    env = dict(os.environ)
    env["LD_PRELOAD"] = _runtime(runtime)
    env["PRK_ORACLE_LIBDIR"] = libdir
    env.update(extra)
    return env


def test_tsan_cpu_schedules(san_libs):
    env = _env("libtsan.so", os.path.join(san_libs, "tsan"),
               TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0")
    p = subprocess.run([sys.executable, os.path.join(_ROOT, "tests", "san_worker.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0 and "ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "san_worker ok" in p.stdout


def test_asan_ubsan_oracle_and_baseline(san_libs):
    env = _env("libasan.so", os.path.join(san_libs, "asan"), ASAN_OPTIONS="detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    probe = ("import sys; sys.path.insert(0, 'oracle'); import oracle as O; "
             "assert '_san' in O.lib()._name and '_san' in O.cpu_lib()._name; print('asan libs')")
    p = subprocess.run([sys.executable, "-c", probe], env=env, cwd=_ROOT, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0 and "asan libs" in p.stdout, p.stderr[-4000:]
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_oracle.py", "tests/test_cpu_baseline.py"],
                       env=env, cwd=_ROOT, capture_output=True, text=True, timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0 and "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
