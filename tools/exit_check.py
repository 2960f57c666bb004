#!/usr/bin/env python3
"""Process-exit check under rocprofv3 --runtime-trace (round-4 verdict: bench.py finished, then
died with SIGSEGV in __cxa_finalize when run under the runtime tracer).

    rocprofv3 --runtime-trace -d gpurun_out/ex -o run -- python tools/exit_check.py MODE

MODE narrows down which teardown crashes:
  load    load libmsbfs.so (registers its code objects with the HIP runtime), touch no device
  device  + create a device graph and free it
  solve   + one small bit-parallel solve (the smoke path), every handle closed before exit
  leak    the same solve, handles left to the interpreter's teardown
Each mode prints "exit_check MODE done" just before the interpreter exits; a crash after that
line is a teardown crash.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(mode: str) -> int:
    import msbfs
    from msbfs.ops import native
    assert native.available()
    if mode in ("device", "solve", "leak"):
        g = msbfs.DeviceGraph.rmat(12, 16, 1, device=0)
        if mode in ("solve", "leak"):
            qs = msbfs.QuerySet.random(g.n, 100, 4, 7)
            s = msbfs.Solver(g, "bitpar", max_groups=qs.K)
            r = s.run(qs)
            print("F[0] =", int(r.F[0]))
            if mode == "solve":
                s.close()
        if mode != "leak":
            g.close()
    print(f"exit_check {mode} done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "solve"))
