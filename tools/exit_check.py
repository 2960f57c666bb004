#!/usr/bin/env python3
"""Process-exit check under rocprofv3 --runtime-trace (round-4 verdict: bench.py finished, then
died with SIGSEGV in __cxa_finalize when run under the runtime tracer).

    rocprofv3 --runtime-trace -d gpurun_out/ex -o run -- python tools/exit_check.py MODE

MODE narrows down which teardown crashes:
  load    load libmsbfs.so (registers its code objects with the HIP runtime), touch no device
  device  + create a device graph and free it
  solve   + one small bit-parallel solve (the smoke path), every handle closed before exit
  leak    the same solve, handles left to the interpreter's teardown
  torch   import torch and initialise its HIP context only (no msbfs)
  tsolve  torch's context, then the solve of `solve`
  tbig    torch's context, an RMAT-24 device graph and a 1024-group solve (bench.py's shape)
Each mode prints "exit_check MODE done" just before the interpreter exits; a crash after that
line is a teardown crash.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(mode: str) -> int:
    if mode.startswith("t"):
        import torch
        torch.cuda.init()
        torch.cuda.synchronize(0)
        if mode == "torch":
            print(f"exit_check {mode} done", flush=True)
            return 0
    import msbfs
    from msbfs.ops import native
    assert native.available()
    if mode in ("device", "solve", "leak", "tsolve", "tbig"):
        big = mode == "tbig"
        g = msbfs.DeviceGraph.rmat(24 if big else 12, 16, 1, device=0)
        if big:
            g.relabel_by_degree()
        if mode != "device":
            qs = msbfs.QuerySet.random(g.n, 1024 if big else 100, 16 if big else 4, 7)
            s = msbfs.Solver(g, "bitpar", max_groups=qs.K)
            s.prepare()
            r = s.run(qs)
            print("F[0] =", int(r.F[0]))
            if mode != "leak":
                s.close()
        if mode != "leak":
            g.close()
    # the executable mappings, to name the frames of a teardown crash's stack afterwards
    os.makedirs("gpurun_out", exist_ok=True)
    with open("/proc/self/maps") as f, open(f"gpurun_out/maps_{mode}.txt", "w") as o:
        o.writelines(l for l in f if " r-xp " in l)
    print(f"exit_check {mode} done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "solve"))
