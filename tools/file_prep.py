#!/usr/bin/env python3
"""File-input preprocessing at scale: the reference's printed "Preprocessing time"
(main.cu:235-298: rank-0 file read + CSR build + broadcasts + device allocation and upload) on a
legacy binary edge list, against the device-generator path (--gen, no file at all).

    python tools/file_prep.py --scale 26 --groups 1024 --dir /tmp/msbfs_fp

Writes a Graph500 RMAT edge list in the reference's format (int32 n, int64 m, m x (int32, int32);
8.6 GB at scale 26) and a query file (extended format for K > 255), then runs the drop-in CLI
(`_bin/msbfs -g G -q Q -gn 1`) cold and warm, with and without the CSR sidecar cache (--cache:
the first run writes it, the second reads it), and with --gen. The plain file runs build the CSR
on the device (the mapped edge list streamed to HBM, device count / scan / scatter);
--host-csr is the host build of rounds 1-3 for comparison. "cold" is the first read after the
file was written (the page cache is not dropped: that needs root). Prints one JSON line per run and
a summary; the answers (minimum group, F) must agree across every run.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import re
import shutil
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_cli(cli, args, env):
    t = time.perf_counter()
    r = subprocess.run([cli] + args, capture_output=True, text=True, env=env, timeout=1500)
    wall = time.perf_counter() - t
    if r.returncode != 0:
        raise SystemExit(f"CLI failed ({r.returncode}): {r.stderr[-2000:]}")
    out = {"wall_s": round(wall, 3)}
    for line in r.stdout.splitlines():
        m = re.match(r"(Preprocessing|Computation) time: ([0-9.]+) s", line)
        if m:
            out[m.group(1).lower() + "_s"] = float(m.group(2))
        m = re.match(r"Query number \(k\) with minimum F value: (-?\d+)", line)
        if m:
            out["min_k"] = int(m.group(1))
        m = re.match(r"Minimum F value: (-?\d+)", line)
        if m:
            out["min_f"] = int(m.group(1))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "msbfs_fp"))
    ap.add_argument("--keep", action="store_true", help="keep the written files")
    args = ap.parse_args()

    import msbfs
    from msbfs.ops import native

    os.makedirs(args.dir, exist_ok=True)
    gpath = os.path.join(args.dir, f"rmat{args.scale}.bin")
    qpath = os.path.join(args.dir, f"q{args.groups}.bin")
    print(json.dumps({"disk_free_GB": round(shutil.disk_usage(args.dir).free / 2**30, 1)}),
          flush=True)
    L = native.lib()
    t = time.perf_counter()
    pu, pv = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
    n, m = C.c_int64(), C.c_int64()
    native.check(L.msbfs_gen_rmat_host(args.scale, args.edgefactor, 1, 0.57, 0.19, 0.19, 1,
                                       C.byref(pu), C.byref(pv), C.byref(n), C.byref(m)))
    t_gen = time.perf_counter() - t
    t = time.perf_counter()
    native.check(L.msbfs_write_edge_list(gpath.encode(), n.value, m.value, pu, pv))
    t_write = time.perf_counter() - t
    L.msbfs_free(C.cast(pu, C.c_void_p))
    L.msbfs_free(C.cast(pv, C.c_void_p))
    qs = msbfs.QuerySet.random(n.value, args.groups, args.group_size, 7)
    qs.write(qpath)
    size = os.path.getsize(gpath)
    print(json.dumps({"n": n.value, "m": m.value, "file_GB": round(size / 1e9, 3),
                      "host_gen_s": round(t_gen, 2), "write_s": round(t_write, 2)}), flush=True)

    cli = native.CLI_PATH
    env = dict(os.environ, MSBFS_NO_MPI="1")
    base = ["-g", gpath, "-q", qpath, "-gn", "1"]
    runs = [("file_cold", base), ("file_warm", base), ("file_host_csr", base + ["--host-csr"]),
            ("cache_build", base + ["--cache"]), ("cache_read", base + ["--cache"]),
            ("gen", ["--gen", f"rmat:{args.scale}:{args.edgefactor}:1", "--qgen",
                     f"{args.groups}:{args.group_size}:7", "-gn", "1"])]
    res = {}
    for name, a in runs:
        res[name] = run_cli(cli, a, env)
        print(json.dumps({"run": name, **res[name]}), flush=True)
    answers = {(r["min_k"], r["min_f"]) for r in res.values()}
    print(json.dumps({"summary": {k: v.get("preprocessing_s") for k, v in res.items()},
                      "computation_s": {k: v.get("computation_s") for k, v in res.items()},
                      "answers_agree": len(answers) == 1, "answer": sorted(answers)[0]}),
          flush=True)
    if not args.keep:
        for p in (gpath, qpath, gpath + ".csr"):
            if os.path.exists(p):
                os.remove(p)
    return 0 if len(answers) == 1 else 3


if __name__ == "__main__":
    sys.exit(main())
