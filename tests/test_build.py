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


def test_level_record_layout(tmp_path):
    """The ctypes mirrors of the C API's structs (msbfs_level, msbfs_stats, msbfs_options in
    msbfs.h) have the C compiler's size and field offsets: the per-level records, run stats and
    solver options cross the FFI by memory layout."""
    import ctypes

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no host C compiler")
    from msbfs.ops import native as N

    structs = {"msbfs_level": N.Level, "msbfs_stats": N.Stats, "msbfs_options": N.Options}
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "msbfs/msbfs.h"',
             "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    inc = os.path.join(ROOT, "csrc", "include")
    subprocess.run([cc, "-std=c11", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    seen = 0
    for line in filter(None, out):
        cname, what, val = line.split()
        py = structs[cname]
        got = ctypes.sizeof(py) if what == "size" else getattr(py, what).offset
        assert got == int(val), (cname, what, got, val)
        seen += 1
    assert seen == sum(1 + len(p._fields_) for p in structs.values())
