"""The MPI control plane (MpiCtrl): ranks started by an MPI launcher, the reference's launch model
(mpirun -n N, MPI_COMM_WORLD collectives: src/sequence.cpp:88-125, src/benchmarker.cpp:45-145).
CPU only; skipped when the image has no MPI launcher (this one ships MPICH 3.3 in /opt/conda)."""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = shutil.which("mpiexec") or ("/opt/conda/bin/mpiexec"
                                      if os.path.exists("/opt/conda/bin/mpiexec") else None)
needs_mpi = pytest.mark.skipif(MPIEXEC is None, reason="no MPI launcher in this image")

BODY = r"""
import json, sys
sys.path.insert(0, {root!r})
import tenzing_amd as tz
from tenzing_amd.parallel import init_ctrl
from tenzing_amd.parallel.dist import env

c = init_ctrl()
assert type(c).__name__ == "MpiCtrl", type(c)
c.barrier()
got = c.bcast("hello" if c.rank == 0 else "", 0).decode()
got2 = c.bcast("x" * 100000 if c.rank == 2 else "", 2).decode()
mx = c.allreduce_max([float(c.rank), -float(c.rank)])
sm = c.allreduce_sum([1.0, 2.0])
ag = [x.decode() for x in c.allgather("r" * c.rank)]
# personalized exchange (MPI_Alltoallv): element j to rank j, of varying sizes incl. empty
a2a = [x.decode() for x in c.alltoallv([f"{{c.rank}}>{{j}}" * j for j in range(c.size)])]
# a collective search on top of it: rank 0 owns the tree, every rank benchmarks every candidate
g = tz.Graph()
a, b = tz.SimGpuOp("a", 20.0), tz.SimGpuOp("b", 30.0)
g.start_then(a); g.start_then(b); g.then_finish(a); g.then_finish(b)
o = tz.MctsOpts(); o.n_iters = 8; o.bench = tz.BenchOpts(n_iters=3)
r = tz.mcts_explore(g, tz.Platform(2), tz.SimBenchmarker(2), c, o)
print(json.dumps(dict(rank=c.rank, size=c.size, local=env().local_rank, got=got,
                      got2=len(got2), mx=mx, sm=sm, ag=ag, a2a=a2a, n=len(r.sims))), flush=True)
"""


def _mpiexec(n, argv, timeout=180):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return subprocess.run([MPIEXEC, "-n", str(n)] + argv, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd="/tmp")


@needs_mpi
def test_mpi_ctrl_collectives_and_search():
    p = _mpiexec(3, [sys.executable, "-c", BODY.format(root=ROOT)])
    assert p.returncode == 0, p.stdout + p.stderr
    rs = sorted((json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")),
                key=lambda r: r["rank"])
    assert [r["rank"] for r in rs] == [0, 1, 2]
    for r in rs:
        assert r["size"] == 3 and r["local"] == r["rank"]
        assert r["got"] == "hello" and r["got2"] == 100000
        assert r["mx"] == [2.0, 0.0] and r["sm"] == [3.0, 6.0]
        assert r["ag"] == ["", "r", "rr"]
        assert r["a2a"] == [f"{src}>{r['rank']}" * r["rank"] for src in range(3)]
    assert rs[0]["n"] == 8 and rs[1]["n"] == 0  # only rank 0 holds results


@needs_mpi
def test_native_cli_under_mpiexec():
    """tz-search picks the MPI control plane when an MPI launcher started it (--ctrl auto)"""
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    if not os.path.exists(exe):
        pytest.skip("tz-search not built")
    p = _mpiexec(2, [exe, "--workload", "diamond", "--sim", "--iters", "6", "--streams", "2"])
    assert p.returncode == 0, p.stdout + p.stderr
    summary = [json.loads(ln) for ln in p.stderr.splitlines() if ln.startswith('{"best')]
    assert summary and summary[0]["ranks"] == 2 and summary[0]["candidates"] == 6
    # the results CSV comes from rank 0 only
    assert sum(ln.startswith("0|") for ln in p.stdout.splitlines()) == 1


@pytest.mark.parametrize("env,launched", [
    ({}, False),
    ({"PMI_RANK": "0", "PMI_SIZE": "1"}, False),       # one rank under a PMI batch wrapper
    ({"PMIX_RANK": "0", "SLURM_NTASKS": "1"}, False),
    ({"PMI_RANK": "1", "PMI_SIZE": "4"}, True),
    ({"OMPI_COMM_WORLD_RANK": "0", "OMPI_COMM_WORLD_SIZE": "2"}, False),  # not MPICH ABI
    ({"PMIX_RANK": "3", "SLURM_NTASKS": "8"}, True),
    # Open MPI inside a Slurm allocation also exports PMIX_RANK: still not an MPICH launch
    ({"PMIX_RANK": "3", "SLURM_NTASKS": "8", "OMPI_COMM_WORLD_RANK": "3",
      "OMPI_COMM_WORLD_SIZE": "8"}, False),
])
def test_mpi_launch_detection(env, launched):
    """MPI is picked only for several launcher ranks; a single process keeps the plain path
    (no MPI library is opened)"""
    code = ("import sys; sys.path.insert(0, %r); import tenzing_amd as tz; "
            "print(tz._tz.MpiCtrl.launched(), tz._tz.MpiCtrl.launcher_size())" % ROOT)
    e = {k: v for k, v in os.environ.items()
         if not k.startswith(("PMI", "OMPI_", "MV2_", "SLURM_", "MPI_LOCAL"))}
    e.update(env)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=e,
                         timeout=120).stdout.split()
    assert out[0] == str(launched)
