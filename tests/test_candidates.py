"""bench.py's candidate selection (distributed.evaluate_candidates) on CPU ranks over gloo: a
candidate that raises on one rank only, or whose gathered F differs from the round-robin pass,
is excluded on EVERY rank (no rank left alone in a collective) and reported; round robin is still
timed (the first real 8-GPU run must yield a number)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from msbfs.parallel import distributed as D
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    ref = np.arange(10, dtype=np.int64)

    def run(name):
        local = np.zeros(10, np.int64)
        local[rank::world] = ref[rank::world]
        if name == "wrong":
            local[rank::world] += 1
        def work():  # rank-local part of the step
            if name == "raises_on_last" and rank == world - 1:
                raise RuntimeError("boom")
            return local
        F = D.allreduce_sum_i64(D.checked(work, ctx), ctx)  # then a collective, like gather_F
        return F, {}

    ms, errors = D.evaluate_candidates(["roundrobin", "raises_on_last", "wrong", "good"], run, ref,
                                       ctx, reps=2)
    devs = D.allgather_int(100 + rank, ctx)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), names=np.array(sorted(ms)),
             errs=np.array(sorted(errors)), devs=np.array(devs),
             msg=np.array(errors.get("raises_on_last", "")))
    D.shutdown(ctx)


@pytest.mark.parametrize("world", [2, 3])
def test_evaluate_candidates_excludes_collectively(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert list(z["names"]) == ["good", "roundrobin"]
        assert list(z["errs"]) == ["raises_on_last", "wrong"]
        assert list(z["devs"]) == [100 + i for i in range(world)]
        # the raising rank names the exception, the others learn it failed elsewhere
        msg = str(z["msg"])
        assert ("boom" in msg) if r == world - 1 else ("another rank" in msg)


def test_evaluate_candidates_single_process():
    from msbfs.parallel import distributed as D
    ctx = D.DistContext()
    ref = np.array([3, 1, 2])
    ms, errors = D.evaluate_candidates(
        ["roundrobin", "bad"], lambda n: (ref if n == "roundrobin" else ref + 1, {}), ref, ctx)
    assert set(ms) == {"roundrobin"} and set(errors) == {"bad"}
