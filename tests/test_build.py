"""The CMake build (csrc/CMakeLists.txt) describes the same library and CLI as
csrc/Makefile: configure into a scratch directory and check the build graph (ninja dry run)
compiles every engine source for gfx950 and links both targets. (A full `cmake --build` takes
about a minute; it was run by hand and its CLI gives the same report as the Makefile build.)"""
import os
import shutil
import sys
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None,
                    reason="cmake/ninja not installed")
def test_cmake_configure_and_plan(tmp_path):
    b = tmp_path / "build"
    r = subprocess.run(["cmake", "-S", os.path.join(ROOT, "csrc"), "-B", str(b), "-G", "Ninja",
                        f"-DMSBFS_OUT_DIR={tmp_path / 'out'}"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(["ninja", "-C", str(b), "-n", "-v"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    plan = r.stdout
    for src in ("bitpar_solver.hip", "bitpar_push.hip", "bitpar_pull.hip", "bitpar_hybrid.hip",
                "dist.hip", "gen.hip", "io.cpp", "capi.cpp", "main.cpp"):
        assert src in plan, src
    assert plan.count("--offload-arch=gfx950") >= 3
    assert "libmsbfs.so" in plan and "_bin/msbfs" in plan


def test_bench_rejects_world_size_mismatch():
    """bench.py --gpus N under a launcher with a different WORLD_SIZE fails before touching the
    GPU (a silently smaller job would report the wrong whole-node number)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    env.pop("MSBFS_FORCE_DIST", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=60, env=env, cwd=ROOT)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr
