"""The drop-in CLI's GPU paths: device CSR upload from a graph file, every device
algorithm, and the multi-rank decompositions (round-robin over MPI, hybrid with ranks that own
no 64-group word) — each checked against the CPU oracle through the 7-line report and --json F.

Several ranks share the box's one GPU (-gn 1), so the CLI keeps host MPI collectives (RCCL
refuses two ranks on one device); the hybrid all-to-all then runs through alltoallv_host_u64."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"

pytestmark = pytest.mark.gpu


def _cli(m):
    p = m.native.CLI_PATH
    if not os.path.exists(p):
        pytest.fail("native CLI not built (make -C csrc)")
    return p


def _files(tmp_path, m, K, size, seed=3):
    g = m.Graph.rmat(12, 8, seed)
    gp, qp = str(tmp_path / "g.bin"), str(tmp_path / "q.bin")
    g.write(gp)
    qs = m.QuerySet.random(g.n, K, size, seed + 4)
    qs.write(qp)
    return g, qs, gp, qp


def _check(r, ref, m, ranks):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 8, r.stdout
    k = m.argmin_first(ref.F)
    assert lines[2] == f"Query number (k) with minimum F value: {k + 1}"
    assert lines[3] == f"Minimum F value: {ref.F[k]}"
    js = json.loads(lines[7])
    assert js["F"] == list(map(int, ref.F))
    assert js["ranks"] == ranks
    return js


def _run(cmd, env=None, timeout=110):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, env=e, timeout=timeout)


@pytest.mark.parametrize("algo", ["bitpar", "dist", "topdown", "sweep", "auto"])
def test_cli_gpu_single_rank(tmp_path, msbfs_pkg, algo):
    m = msbfs_pkg
    K = 6 if algo == "sweep" else 70
    g, qs, gp, qp = _files(tmp_path, m, K, 3)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([_cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", algo, "--json"],
             {"MSBFS_NO_MPI": "1"})
    js = _check(r, ref, m, 1)
    assert js["traversed_edges"] == int(ref.edges.sum())


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("ranks,K,dist", [(2, 64, "hybrid"), (3, 64, "hybrid"), (3, 130, "hybrid"),
                                          (2, 70, "roundrobin"), (3, 64, "auto")])
def test_cli_gpu_multi_rank(tmp_path, msbfs_pkg, ranks, K, dist):
    """K = 64 is one word: with 2-3 ranks, ranks >= 1 own no groups in hybrid mode (phase C
    skipped, their F slice empty) but still take part in every collective."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, K, 4)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([MPIEXEC, "-n", str(ranks), _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo",
              "bitpar", "--dist", dist, "--json"])
    js = _check(r, ref, m, ranks)
    assert js["comm"] == "mpi"
    assert js["traversed_edges"] == int(ref.edges.sum())


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
def test_cli_gpu_generator_mode_multi_rank(msbfs_pkg):
    """--gen: every rank generates the identical graph in its own HBM (no broadcast)."""
    m = msbfs_pkg
    r = _run([MPIEXEC, "-n", "2", _cli(m), "--gen", "rmat:11:8:5", "--qgen", "100:3:9", "-gn", "1",
              "--json"])
    g = m.Graph.rmat(11, 8, 5)
    ref = m.cpu_bfs(g, m.QuerySet.random(g.n, 100, 3, 9), count_edges=True)
    _check(r, ref, m, 2)


@pytest.mark.parametrize("dist", ["hybrid", "roundrobin"])
def test_cli_gpu_rccl_one_rank(tmp_path, msbfs_pkg, dist):
    """--comm rccl with one rank: the graph broadcast (ncclBroadcast), the hybrid exchange
    (grouped ncclSend/ncclRecv) and the result reductions (ncclAllReduce) all run through a real
    one-rank RCCL communicator — the device-collective code of the 8-GPU runs, on one GPU."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 200, 4)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([MPIEXEC, "-n", "1", _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "bitpar",
              "--comm", "rccl", "--dist", dist, "--json"])
    js = _check(r, ref, m, 1)
    assert js["comm"] == "rccl"


@pytest.mark.parametrize("extra", [[], ["--no-relabel"], ["--sort-rows"]])
def test_python_cli_gpu(tmp_path, msbfs_pkg, extra):
    """`python -m msbfs` (the torch.distributed twin) on the GPU: degree relabelling on by
    default, the 7-line report and the F vector equal to the CPU oracle."""
    import sys
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 90, 3)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([sys.executable, "-m", "msbfs", "-g", gp, "-q", qp, "-gn", "1", "--algo", "bitpar",
              "--json"] + extra, {"PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    k = m.argmin_first(ref.F)
    assert lines[2] == f"Query number (k) with minimum F value: {k + 1}"
    assert lines[3] == f"Minimum F value: {ref.F[k]}"
    js = json.loads(lines[7])
    assert js["F"] == list(map(int, ref.F)) and js["traversed_edges"] == int(ref.edges.sum())


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("ranks,K,comm", [(3, 300, "mpi"), (2, 130, "mpi"), (1, 200, "rccl")])
def test_cli_gpu_hybrid_coded_exchange(tmp_path, msbfs_pkg, ranks, K, comm):
    """--dist hybrid-coded: the hybrid all-to-all carries zero-word coded segments (sizes from the
    coded-length matrix in the phase-A all-reduce) and every rank decodes them on the GPU; the
    report and F vector must equal the CPU oracle's (host MPI staging and a real RCCL group)."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, K, 4)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([MPIEXEC, "-n", str(ranks), _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo",
              "bitpar", "--dist", "hybrid-coded", "--comm", comm, "--json"])
    js = _check(r, ref, m, ranks)
    assert js["comm"] == comm


@pytest.mark.parametrize("spmd,comm,dist,K", [(1, "rccl", "roundrobin", 2100),
                                              (1, "rccl", "hybrid", 200),
                                              (2, "auto", "hybrid", 300),
                                              (3, "auto", "roundrobin", 700)])
def test_cli_gpu_spmd(tmp_path, msbfs_pkg, spmd, comm, dist, K):
    """--spmd N: the job in one process, ranks as threads. One rank with --comm rccl makes its
    communicator with ncclCommInitAll (the single-process multi-GPU bootstrap) and runs the
    round-robin passes (K = 2100: several 64*W-group passes) with their packed MIN reductions
    issued asynchronously on the communicator's stream while the next pass computes;
    --repeat 3 re-runs the timed region on the same persistent buffers. Several threads on the
    box's one GPU use the in-process ThreadComm (device all-to-all by peer copies)."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, K, 4)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([_cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "bitpar", "--spmd", str(spmd),
              "--comm", comm, "--dist", dist, "--repeat", "3", "--json"], {"MSBFS_NO_MPI": "1"})
    js = _check(r, ref, m, spmd)
    assert js["comm"] == ("rccl" if comm == "rccl" else "threads")
    assert js["traversed_edges"] == int(ref.edges.sum())


def test_cli_gpu_spmd_rccl_shared_gpu_refused(tmp_path, msbfs_pkg):
    """--spmd 2 --comm rccl on one GPU (repeated devices, which RCCL rejects) fails
    with a message instead of running over host collectives unannounced."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 100, 4)
    r = subprocess.run([_cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "bitpar", "--spmd", "2",
                        "--comm", "rccl"], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "MSBFS_NO_MPI": "1"})
    assert r.returncode != 0 and "one GPU per --spmd rank" in (r.stderr + r.stdout)


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
def test_cli_gpu_rccl_repeat_multipass(tmp_path, msbfs_pkg):
    """One-rank RCCL over MPI with several solver passes and --repeat 3: the asynchronous
    per-pass reductions and the persistent device scratch give the exact answer every time."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 1500, 3)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([MPIEXEC, "-n", "1", _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "bitpar",
              "--comm", "rccl", "--repeat", "3", "--json"])
    js = _check(r, ref, m, 1)
    assert js["comm"] == "rccl"


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("ranks,comm", [(1, "rccl"), (2, "mpi")])
def test_cli_gpu_many_passes_drain(tmp_path, msbfs_pkg, ranks, comm):
    """more solver passes than asynchronous reduction slots. --max-words 1 makes every
    pass 64 groups (700 groups: 11 passes on one rank, 6 on each of two) and --async-slots 2
    drains the in-flight MIN reductions every 2 passes into the running minimum; the answer must
    still be the oracle's (before, more passes than slots aborted the job)."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 700, 3)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([MPIEXEC, "-n", str(ranks), _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo",
              "bitpar", "--comm", comm, "--dist", "roundrobin", "--max-words", "1",
              "--async-slots", "2", "--repeat", "2", "--json"])
    js = _check(r, ref, m, ranks)
    assert js["comm"] == comm


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("ranks,comm,chunks", [(2, "mpi", 3), (3, "mpi", 2), (1, "rccl", 4),
                                               (1, "rccl", 0)])
def test_cli_gpu_hybrid_chunked_exchange(tmp_path, msbfs_pkg, ranks, comm, chunks):
    """--chunks N: the overlapped hybrid exchange (phase A hands out its vertex ranges, one
    all-to-all piece each; RCCL: grouped send/recv on the communicator's stream while phase A
    goes on; host MPI: staged pieces). chunks 0 = the default (8 with RCCL)."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 300, 4)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([MPIEXEC, "-n", str(ranks), _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo",
              "bitpar", "--dist", "hybrid", "--comm", comm, "--chunks", str(chunks), "--repeat",
              "2", "--json"])
    js = _check(r, ref, m, ranks)
    assert js["comm"] == comm


def test_cli_gpu_spmd_hybrid_chunked(tmp_path, msbfs_pkg):
    """--spmd 3 threads (ThreadComm) with the chunked hybrid exchange: every piece staged through
    the in-process collectives, in the same order on every thread."""
    m = msbfs_pkg
    g, qs, gp, qp = _files(tmp_path, m, 300, 4)
    ref = m.cpu_bfs(g, qs, count_edges=True)
    r = _run([_cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "bitpar", "--spmd", "3",
              "--dist", "hybrid", "--chunks", "3", "--json"], {"MSBFS_NO_MPI": "1"})
    js = _check(r, ref, m, 3)
    assert js["comm"] == "threads"
