"""bench.py's multi-GPU code paths on the one-GPU box: MSBFS_FORCE_DIST=1 makes a one-rank
torch.distributed process group over RCCL ("nccl") that still runs every collective (barrier,
all-reduces, the hybrid exchange's point-to-point pieces), and bench.py checks each
decomposition's F vector against the round-robin pass before timing (exit status 3 on a
mismatch). Several ranks share the one GPU over gloo; the RCCL run with one GPU per rank needs a
box with two or more GPUs and is skipped otherwise."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("dist", ["hybrid", "hybrid-coded", "roundrobin", "auto"])
def test_bench_forced_rccl_one_rank(dist):
    env = dict(os.environ, MSBFS_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--scale", "18",
                        "--groups", "300", "--steps", "2", "--warmup", "1", "--dist", dist,
                        "--verify", "8"],
                       capture_output=True, text=True, env=env, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["n_gpus"] == 1 and js["value"] > 0
    if dist.startswith("hybrid"):
        assert js["config"]["parallelism"].startswith("hybrid1")
        assert ("coded" in js["config"]["parallelism"]) == (dist == "hybrid-coded")
    if dist == "auto":
        assert set(js["config"]["candidates_ms"]) == {"roundrobin", "hybrid", "hybrid-coded"}


def test_bench_graph_forced_rccl_one_rank(msbfs_pkg):
    """tools/bench_graph.py (secondary BASELINE configs) through a one-rank RCCL group: round
    robin split, the packed all-reduce(MIN), the answer equal to the CPU oracle's."""
    msbfs = msbfs_pkg
    env = dict(os.environ, MSBFS_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_graph.py"), "--graph",
                        "grid:200:200:0.7", "--groups", "100", "--group-size", "4", "--steps", "2",
                        "--verify", "4"], capture_output=True, text=True, env=env, timeout=110,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    g = msbfs.Graph.grid(200, 200, 0.7, 0, 1)
    ref = msbfs.cpu_bfs(g, msbfs.QuerySet.random(g.n, 100, 4, 7), count_edges=True)
    k = msbfs.argmin_first(ref.F)
    assert js["n_gpus"] == 1 and js["min_k"] == k + 1 and js["min_f"] == int(ref.F[k])
    assert js["traversed_edges"] == int(ref.edges.sum())


def test_bench_graph_two_ranks_gloo(msbfs_pkg):
    """Two ranks sharing the GPU (gloo host collectives): each rank runs half of the groups."""
    msbfs = msbfs_pkg
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(_port()), os.path.join(ROOT, "tools", "bench_graph.py"), "--graph",
                        "rmat:14:8", "--relabel", "1", "--groups", "130", "--group-size", "3",
                        "--steps", "1", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    g = msbfs.Graph.rmat(14, 8, 1)
    ref = msbfs.cpu_bfs(g, msbfs.QuerySet.random(g.n, 130, 3, 7), count_edges=True)
    k = msbfs.argmin_first(ref.F)
    assert js["n_gpus"] == 2 and js["min_k"] == k + 1 and js["min_f"] == int(ref.F[k])
    assert js["traversed_edges"] == int(ref.edges.sum())


@pytest.mark.parametrize("ranks,dist", [(2, "hybrid"), (3, "hybrid"), (2, "hybrid-coded"),
                                        (3, "auto")])
def test_bench_multi_rank_gloo_shared_gpu(ranks, dist):
    """bench.py with several ranks on the one GPU (gloo collectives, the hybrid exchange staged
    through host memory): every rank runs its own solver, the hybrid phases exchange real
    buffers, and bench.py checks each decomposition's F against the round-robin pass."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", str(ranks), "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus",
                        str(ranks), "--scale", "16", "--groups", "200", "--steps", "2", "--warmup", "1", "--dist", dist,
                        "--backend", "gloo", "--verify", "4"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["n_gpus"] == ranks and js["value"] > 0
    cfg = js["config"]
    assert cfg["devices"] == [0] * ranks and cfg["process_group_size"] == ranks
    assert cfg["candidate_errors"] == {}
    if dist.startswith("hybrid"):
        assert cfg["parallelism"].startswith(f"hybrid{ranks}")
        ph = cfg["phases"]  # per-phase wall ms (max over ranks) and the exchange rate
        assert ph["phase_a_wall_ms"] > 0 and ph["phase_c_wall_ms"] > 0 and ph["exchange_ms"] > 0
        assert ph["alltoall_GBps_per_rank"] is None or ph["alltoall_GBps_per_rank"] > 0
        # the dense exchange overlaps phase A in point-to-point pieces under gloo too
        assert ph["chunks"] == (1 if dist == "hybrid-coded" else 8)
    else:
        assert set(cfg["candidates_ms"]) == {"roundrobin", "hybrid", "hybrid-coded"}


def _visible_gpus():
    import torch
    return torch.cuda.device_count()  # (counts devices without creating a context)


@pytest.mark.parametrize("dist", ["hybrid", "auto"])
def test_bench_two_ranks_rccl(dist):
    """Two ranks, one GPU each, over RCCL: the overlapped hybrid exchange's grouped P2P pieces
    between real peers, the async argmin, and the candidates' F checked against round robin."""
    if _visible_gpus() < 2:
        pytest.skip("needs two GPUs (one per RCCL rank)")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--scale",
                        "18", "--groups", "300", "--steps", "2", "--warmup", "1", "--dist", dist,
                        "--verify", "4"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    cfg = js["config"]
    assert js["n_gpus"] == 2 and cfg["devices"] == [0, 1] and cfg["candidate_errors"] == {}
    if dist == "hybrid":
        assert cfg["phases"]["chunks"] == 8


@pytest.mark.parametrize("bad", ["hybrid", "hybrid-coded"])
def test_bench_excludes_wrong_candidate(bad):
    """A decomposition whose F is wrong (bench.py --test-corrupt, tests only) is excluded on
    every rank and reported in candidate_errors; the run still times a verified one (exit 0)."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus",
                        "2", "--scale", "16", "--groups", "200", "--steps", "2", "--warmup", "1",
                        "--backend", "gloo", "--verify", "4", "--test-corrupt", bad],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    cfg = js["config"]
    assert list(cfg["candidate_errors"]) == [bad] and "F differs" in cfg["candidate_errors"][bad]
    assert bad not in cfg["candidates_ms"] and "roundrobin" in cfg["candidates_ms"]
    assert js["value"] > 0 and cfg["timed_F_equals_untimed"]


def test_bench_wrong_roundrobin_fails():
    """Round robin itself wrong: no number (exit 3), whatever the other candidates say."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus",
                        "2", "--scale", "14", "--groups", "100", "--steps", "1", "--warmup", "0",
                        "--backend", "gloo", "--test-corrupt", "roundrobin"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode != 0


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher around it starts the two ranks itself (the driver's
    plain `python3 bench.py --gpus N` must measure N ranks, not one): n_gpus 2 in the JSON line,
    the timed F equal to the untimed pass, groups checked against the distance solver."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--scale", "16", "--groups", "200", "--steps", "2",
                        "--warmup", "1", "--verify", "8"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["n_gpus"] == 2 and js["value"] > 0
    assert js["verified"] == 8 and js["config"]["timed_F_equals_untimed"]


def test_bench_one_gpu_self_verifies():
    """The default headline run checks itself: verified >= 8 groups against the distance solver
    (untimed) and the last timed step's F equal to the untimed pass."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--scale", "18",
                        "--groups", "256", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["verified"] >= 8 and js["n_gpus"] == 1
