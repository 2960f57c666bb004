"""python -m msbfs -g <graph.bin> -q <query.bin> -gn <numGPU> [options]

The torch.distributed twin of the native CLI (`_bin/msbfs`, launched with mpirun): launch with
`torchrun --nproc-per-node N -m msbfs ...` for one rank per GPU over RCCL (or gloo on CPU).
Same flags and the same 7-line report as the reference (main.cu:203-224, 403-414); unknown
tokens are ignored; fewer than 4 arguments print the usage line and exit 255.
"""
import sys


def main(argv=None) -> int:
    argv = list(sys.argv if argv is None else argv)
    from .parallel import distributed as D
    if len(argv) < 5:
        import os
        if int(os.environ.get("RANK", "0")) == 0:
            print(f"Usage: mpirun -np <ranks> {argv[0]} -g <graph.bin> -q <query.bin> -gn <numGPU>",
                  file=sys.stderr)
        return 255
    from .engine import Engine, JobConfig
    cfg = JobConfig()
    json_out = False
    i = 1
    while i < len(argv):
        a = argv[i]
        has = i + 1 < len(argv)
        if a == "-g" and has:
            cfg.graph = argv[i + 1]; i += 1
        elif a == "-q" and has:
            cfg.query = argv[i + 1]; i += 1
        elif a == "-gn" and has:
            cfg.num_gpu = int(argv[i + 1]); i += 1
        elif a == "--algo" and has:
            cfg.algo = argv[i + 1]; i += 1
        elif a == "--gen" and has:
            cfg.gen = argv[i + 1]; i += 1
        elif a == "--qgen" and has:
            cfg.qgen = argv[i + 1]; i += 1
        elif a == "--cache":
            cfg.use_cache = True
        elif a == "--sort-rows":
            cfg.sort_rows = True
        elif a == "--no-relabel":
            cfg.relabel = False
        elif a == "--json":
            json_out = True
            cfg.count_edges = True
        i += 1
    if cfg.num_gpu <= 0:
        print("msbfs: -gn must be >= 1", file=sys.stderr)
        return 1
    import torch
    use_gpu = cfg.algo != "cpu" and torch.cuda.is_available()
    ctx = D.init_from_env(gpus_per_node=cfg.num_gpu, use_gpu=use_gpu)
    eng = Engine(cfg, ctx)
    try:
        eng.preprocess()
    except Exception as e:  # e.g. "Could not open graph file X"
        print(str(e), file=sys.stderr)
        D.shutdown(ctx)
        return 1
    D.barrier(ctx)
    r = eng.compute(gather=json_out)
    if ctx.rank == 0:
        sys.stdout.write(eng.report(r))
        if json_out:
            import json
            print(json.dumps({"K": eng.queries.K, "n": eng.n, "ranks": ctx.world,
                              "backend": ctx.backend, "traversed_edges": r.traversed_edges,
                              "F": [int(x) for x in r.F]}))
        sys.stdout.flush()
    eng.close()
    D.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
