#!/usr/bin/env python3
"""Per-rank cost of the hybrid decomposition on ONE GPU (no multi-GPU box needed).

Runs every rank's phase A (levels 1-2, own residue class of vertices) and phase C (own groups, levels >= 3)
sequentially on one GPU (parallel/hybrid.py emulate_ranks), checks F against the single-GPU
solver, and prints per-rank device times plus the all-to-all volume. The estimated N-GPU step
is max_r(A_r) + exposed exchange + max_r(C_r): with --chunks > 1 phase A hands its vertex ranges to
the exchange as they are done (parallel/hybrid.py, the overlapped exchange), and only the part of
the exchange still running when phase A ends is counted; the exchange (dense; zero-word coded with --coded) is priced at
--a2a-gbps per GPU (max of send and receive side), an assumption to be replaced by the driver's measured 8-GPU runs. For comparison it also
times round-robin (each rank runs ceil(K/N) groups on the whole graph).

    python tools/hybrid_sim.py --scale 26 --groups 1024 --ranks 2 4 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--groups", type=int, default=1024)
    ap.add_argument("--group-size", type=int, default=16)
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--no-roundrobin", action="store_true")
    ap.add_argument("--a2a-gbps", type=float, default=300.0,
                    help="assumed per-GPU all-to-all bandwidth (GB/s, max of send and receive)")
    ap.add_argument("--coded", action="store_true", help="zero-word coded exchange")
    ap.add_argument("--chunks", type=int, default=4,
                    help="overlapped exchange: phase A hands out its vertex ranges in this many "
                         "pieces (1 = the whole exchange after phase A)")
    ap.add_argument("--rccl-pieces", action="store_true",
                    help="start a one-rank RCCL all-to-all of each piece's size as it is packed "
                         "(its kernels then compete with phase A's for the CUs, as on a node)")
    args = ap.parse_args()

    import msbfs
    from msbfs.parallel import distributed as D
    from msbfs.parallel import hybrid as H

    g = msbfs.DeviceGraph.rmat(args.scale, args.edgefactor, 1, device=0, relabel=True)
    qs = msbfs.QuerySet.random(g.n, args.groups, args.group_size, 7)
    hook = None
    if args.rccl_pieces:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        scratch = [torch.zeros(1 << 27, dtype=torch.int64, device="cuda:0") for _ in range(2)]

        def hook(c, nbytes):
            n = min(int(nbytes) // 8, scratch[0].numel())
            dist.all_to_all_single(scratch[1][:n], scratch[0][:n], async_op=True)
    with msbfs.Solver(g, "bitpar", max_groups=qs.K) as s:
        ref = s.run(qs)
        t = time.perf_counter()
        ref = s.run(qs)
        one = (time.perf_counter() - t) * 1e3
        print(json.dumps({"ranks": 1, "ms": round(one, 3), "device_ms": ref.stats["device_ms"]}),
              flush=True)
        for N in args.ranks:
            H.emulate_ranks(s, qs, N, coded=args.coded, chunks=args.chunks,
                            piece_hook=hook)  # warm
            tim = []
            F = H.emulate_ranks(s, qs, N, timings=tim, coded=args.coded, chunks=args.chunks,
                                piece_hook=hook)
            ok = bool(np.array_equal(F, ref.F))
            a = max(x["phase_a_ms"] for x in tim)
            c = max(x["phase_c_ms"] + x.get("decode_ms", 0.0) for x in tim)  # decode: receiver
            rb = max(max(x["recv_bytes"], x["send_bytes"]) for x in tim)
            x_ms = rb / (args.a2a_gbps * 1e9) * 1e3
            # overlapped: every rank's pieces leave as they are packed; the exchange is done when
            # the last rank's last piece is out (the receive side priced like the send side)
            if args.chunks > 1 and not args.coded:
                done = max(H.overlapped_exchange_ms(
                    x["phase_a_ms"], [p[0] for p in x["pieces"]],
                    [p[1] * max(x["recv_bytes"], x["send_bytes"]) / max(1, x["send_bytes"])
                     for p in x["pieces"]], args.a2a_gbps) for x in tim)
                x_exposed = max(0.0, done - a)
            else:
                x_exposed = x_ms
            rr = [0.0]
            for r in ([] if args.no_roundrobin else range(N)):
                sub = qs.subset(D.round_robin(qs.K, r, N))
                rr.append(s.run(sub).stats["device_ms"])
            print(json.dumps({
                "ranks": N, "correct": ok, "phase_a_ms_max": round(a, 3),
                "phase_c_ms_max": round(c, 3), "a2a_MB_max": round(rb / 2**20, 1),
                "a2a_dense_MB_max": round(max(x["dense_send_bytes"] for x in tim) / 2**20, 1),
                "coded": args.coded,
                "a2a_ms_est": round(x_ms, 3), "a2a_exposed_ms_est": round(x_exposed, 3),
                "chunks": args.chunks if not args.coded else 1,
                "hybrid_est_ms": round(a + x_exposed + c, 3),
                "phase_a_wall_ms_max": round(max(x["phase_a_wall_ms"] for x in tim), 3),
                "phase_c_wall_ms_max": round(max(x["phase_c_wall_ms"] for x in tim), 3),
                "roundrobin_ms_max": round(max(rr), 3),
                "per_rank": [{k: (round(v, 3) if isinstance(v, float) else v)
                              for k, v in x.items() if k != "pieces"} for x in tim],
                "pieces_ms": [[round(p[0], 3) for p in x["pieces"]] for x in tim]}), flush=True)


if __name__ == "__main__":
    main()
