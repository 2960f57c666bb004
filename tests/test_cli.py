"""The native CLI keeps the reference contract: flags, usage/exit code, 7-line report, errors,
and identical answers for every MPI world size (round-robin invariance, main.cu:305)."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

from golden import CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"


def _cli(msbfs):
    p = msbfs.native.CLI_PATH
    if not os.path.exists(p):
        pytest.skip("native CLI not built")
    return p


def _write_case(tmp_path, m, case, idx):
    (n, edges), groups = case[0], case[1]
    g = m.Graph.from_edges(n, np.array([e[0] for e in edges], np.int32),
                           np.array([e[1] for e in edges], np.int32))
    gp, qp = str(tmp_path / f"g{idx}.bin"), str(tmp_path / f"q{idx}.bin")
    g.write(gp)
    m.QuerySet.from_groups(groups).write(qp)
    return gp, qp


def _run(cmd, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, env=e, timeout=300)


@pytest.mark.parametrize("idx", range(len(CASES)))
def test_cli_golden_report(tmp_path, msbfs_pkg, idx):
    m = msbfs_pkg
    gp, qp = _write_case(tmp_path, m, CASES[idx], idx)
    r = _run([_cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "cpu", "--no-cache"],
             {"MSBFS_NO_MPI": "1"})
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 7
    assert lines[0] == f"Graph: {gp}" and lines[1] == f"Query: {qp}"
    assert lines[2] == f"Query number (k) with minimum F value: {CASES[idx][3]}"
    assert lines[3] == f"Minimum F value: {CASES[idx][4]}"
    assert lines[4] == "GPU # : 1 GPU"
    assert lines[5].startswith("Preprocessing time: ") and lines[5].endswith(" s")
    assert len(lines[5].split()[2].split(".")[1]) == 9  # fixed << setprecision(9)
    assert lines[6].startswith("Computation time: ")


def test_cli_usage_and_errors(tmp_path, msbfs_pkg):
    cli = _cli(msbfs_pkg)
    r = _run([cli, "-g", "x"], {"MSBFS_NO_MPI": "1"})
    assert r.returncode == 255 and "Usage: mpirun -np <ranks>" in r.stderr
    assert "-g <graph.bin> -q <query.bin> -gn <numGPU>" in r.stderr
    r = _run([cli, "-g", str(tmp_path / "nope.bin"), "-q", "q", "-gn", "1", "--algo", "cpu"],
             {"MSBFS_NO_MPI": "1"})
    assert r.returncode != 0 and "Could not open graph file" in r.stderr


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("ranks", [1, 2, 3, 5])
def test_cli_mpi_world_size_invariance(tmp_path, msbfs_pkg, ranks):
    m = msbfs_pkg
    g = m.Graph.rmat(10, 8, 4)
    gp, qp = str(tmp_path / "r.bin"), str(tmp_path / "q.bin")
    g.write(gp)
    qs = m.QuerySet.random(g.n, 4, 2, 3)  # K=4 < ranks=5 -> idle ranks (main.cu:305)
    qs.write(qp)
    ref = m.cpu_bfs(g, qs)
    k = m.argmin_first(ref.F)
    r = _run([MPIEXEC, "-n", str(ranks), _cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "cpu",
              "--no-cache", "--json"])
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[2] == f"Query number (k) with minimum F value: {k + 1}"
    assert lines[3] == f"Minimum F value: {ref.F[k]}"
    import json
    js = json.loads(lines[7])
    assert js["F"] == list(map(int, ref.F)) and js["ranks"] == ranks and js["comm"] == "mpi"


def test_cli_generator_mode(msbfs_pkg):
    m = msbfs_pkg
    r = _run([_cli(m), "--gen", "rmat:9:8:2", "--qgen", "20:3:5", "-gn", "1", "--algo", "cpu",
              "--json"], {"MSBFS_NO_MPI": "1"})
    assert r.returncode == 0, r.stderr
    g = m.Graph.rmat(9, 8, 2)
    ref = m.cpu_bfs(g, m.QuerySet.random(g.n, 20, 3, 5))
    import json
    assert json.loads(r.stdout.splitlines()[7])["F"] == list(map(int, ref.F))


def test_python_cli_matches(tmp_path, msbfs_pkg):
    m = msbfs_pkg
    gp, qp = _write_case(tmp_path, m, CASES[1], 1)
    r = _run([sys.executable, "-m", "msbfs", "-g", gp, "-q", qp, "-gn", "1", "--algo", "cpu"],
             {"PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[2] == "Query number (k) with minimum F value: 2" and lines[3] == "Minimum F value: 3"
    r = _run([sys.executable, "-m", "msbfs", "-g"], {"PYTHONPATH": ROOT})
    assert r.returncode == 255 and "Usage" in r.stderr


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="no mpiexec")
@pytest.mark.parametrize("fault", ["load:0", "load:2", "compute:1"])
def test_cli_fault_takes_job_down(tmp_path, msbfs_pkg, fault):
    """A failure on any rank ends the whole job promptly with an error (MPI_Abort), instead of
    leaving the other ranks blocked in a collective as the reference's rank-0 exit() does
    (main.cu:95-99). MSBFS_FAULT=<where>:<rank> injects the failure."""
    cli = _cli(msbfs_pkg)
    rank = fault.split(":")[1]
    r = subprocess.run([MPIEXEC, "-n", "3", "-errfile-pattern", str(tmp_path / "err.%r"), cli,
                        "--gen", "rmat:9:8:2", "--qgen", "20:3:5", "-gn", "1", "--algo", "cpu"],
                       capture_output=True, text=True, timeout=60,
                       env={**os.environ, "MSBFS_FAULT": fault})
    assert r.returncode != 0
    # the faulting rank's message: in its error file, unless the abort tore the job down before
    # the launcher wrote that file (seen under a loaded machine)
    msg = f"injected fault: {fault.split(':')[0]} on rank {rank}"
    texts = [p.read_text() for p in tmp_path.glob("err.*")] + [r.stderr]
    assert any(msg in t for t in texts) or not (tmp_path / f"err.{rank}").exists(), texts


def test_cli_baseline_config1_serial_cpu(msbfs_pkg):
    """BASELINE config 1: 1K-vertex / 10K-edge random graph, 4 single-source queries, serial CPU
    BFS on one rank (plumbing, no GPU) — checked against the numpy oracle of the reference
    semantics (ops/reference.py)."""
    m = msbfs_pkg
    r = _run([_cli(m), "--gen", "uniform:1000:10000:1", "--qgen", "4:1:7", "-gn", "1", "--algo",
              "cpu", "--threads", "1", "--json"], {"MSBFS_NO_MPI": "1"})
    assert r.returncode == 0, r.stderr
    g = m.Graph.uniform(1000, 10000, 1)
    qs = m.QuerySet.random(g.n, 4, 1, 7)
    from msbfs.ops.reference import bfs_F_numpy
    F = [bfs_F_numpy(g.n, g.rowptr, g.col, qs.group(k))[0] for k in range(qs.K)]
    import json
    js = json.loads(r.stdout.splitlines()[7])
    assert js["F"] == F and js["K"] == 4 and js["n"] == 1000
    k = int(np.argmin(F))
    assert r.stdout.splitlines()[2] == f"Query number (k) with minimum F value: {k + 1}"


@pytest.mark.parametrize("ranks", [1, 2, 3, 5])
def test_cli_spmd_threads_world_size_invariance(tmp_path, msbfs_pkg, ranks):
    """--spmd N: the whole job in ONE process, N ranks as N threads (the in-process ThreadComm:
    shared-memory broadcasts, all-reduces, all-to-all; SURVEY C8 single-process mode). Same
    report and F vector as the oracle for every N, idle ranks included (K=4 < 5)."""
    m = msbfs_pkg
    g = m.Graph.rmat(10, 8, 4)
    gp, qp = str(tmp_path / "r.bin"), str(tmp_path / "q.bin")
    g.write(gp)
    qs = m.QuerySet.random(g.n, 4, 2, 3)
    qs.write(qp)
    ref = m.cpu_bfs(g, qs)
    k = m.argmin_first(ref.F)
    r = _run([_cli(m), "-g", gp, "-q", qp, "-gn", "1", "--algo", "cpu", "--spmd", str(ranks),
              "--json"], {"MSBFS_NO_MPI": "1"})
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 8  # the 7-line report once (rank 0) + the JSON line
    assert lines[2] == f"Query number (k) with minimum F value: {k + 1}"
    assert lines[3] == f"Minimum F value: {ref.F[k]}"
    import json
    js = json.loads(lines[7])
    assert js["F"] == list(map(int, ref.F)) and js["ranks"] == ranks and js["comm"] == "threads"


def test_cli_spmd_fault_takes_process_down(msbfs_pkg):
    """A failure in one rank-thread ends the whole single-process job with an error (its peers
    would otherwise wait in a collective forever)."""
    r = _run([_cli(msbfs_pkg), "--gen", "rmat:9:8:2", "--qgen", "20:3:5", "-gn", "1", "--algo",
              "cpu", "--spmd", "3"], {"MSBFS_NO_MPI": "1", "MSBFS_FAULT": "compute:1"})
    assert r.returncode != 0 and "injected fault: compute on rank 1" in r.stderr
