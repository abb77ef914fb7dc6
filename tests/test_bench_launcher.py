"""bench.py's own launcher: a multi-GPU run must never lose its scaling point
to how it was launched. Without a launcher in the environment, `bench.py --gpus N` starts N rank
processes itself; a launcher whose rank count differs from --gpus is a hard error."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
_LAUNCH = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
           "PMI_SIZE", "PMI_RANK", "PMIX_RANK", "OMPI_COMM_WORLD_SIZE", "MV2_COMM_WORLD_SIZE")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in _LAUNCH}
    e.update(kw)
    return e


def test_world_size_mismatch_is_a_hard_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], capture_output=True, text=True,
                       timeout=60, env=_env(WORLD_SIZE="2", RANK="0"), cwd="/tmp")
    assert r.returncode == 2, (r.stdout, r.stderr)
    assert "--gpus 4" in r.stderr and "2 rank(s)" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_mpi_launcher_mismatch_is_a_hard_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8"], capture_output=True, text=True,
                       timeout=60, env=_env(PMI_SIZE="2", PMI_RANK="0"), cwd="/tmp")
    assert r.returncode == 2 and "2 rank(s)" in r.stderr, (r.stdout, r.stderr)


def test_one_rank_under_a_launcher_that_says_more_is_refused():
    r = subprocess.run([sys.executable, BENCH], capture_output=True, text=True, timeout=60,
                       env=_env(WORLD_SIZE="8", RANK="0"), cwd="/tmp")
    assert r.returncode == 2 and "--gpus 1" in r.stderr, (r.stdout, r.stderr)


def test_self_spawned_ranks_rendezvous_and_the_failure_is_relayed():
    """no launcher: two fresh rank processes start, meet over the native TCP control plane
    (RANK / WORLD_SIZE / MASTER_* set by the parent), find no GPU here and exit 2; the parent
    exits non-zero and prints one partial result line that names the rank count"""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--deadline-s", "90"], capture_output=True, text=True, timeout=150,
                       env=_env(), cwd="/tmp")
    assert r.returncode == 2, (r.stdout, r.stderr[-3000:])
    for rank in (0, 1):
        assert f"rank {rank}: no GPU visible" in r.stderr, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["partial"] is True and j["launcher"] == "bench.py"
    assert "[2, 2]" in j["error"]


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("tz_bench", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_spmv_transport_of_a_schedule():
    b = _bench_module()
    assert b.spmv_via(["a_Pack", "a_yl_i4", "a_exchange", "a_yr"]) == "rccl"
    assert b.spmv_via(["spmv_i_put", "spmv_i_wait", "spmv_yl_w8", "he_put_dx1_dy0_dz0"]) == "ipc"
    # halo puts are not the SpMV's transport
    assert b.spmv_via(["spmv_yl_w8", "he_put_dx1_dy0_dz0"]) == "local"


def test_launcher_world_from_each_launcher(monkeypatch):
    b = _bench_module()
    for k in _LAUNCH + ("SLURM_NTASKS",):
        monkeypatch.delenv(k, raising=False)
    assert b.launched_world() is None
    monkeypatch.setenv("PMI_RANK", "0")
    assert b.launched_world() == 1  # srun without a task count: one rank
    monkeypatch.setenv("SLURM_NTASKS", "4")
    assert b.launched_world() == 4
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "3")
    assert b.launched_world() == 3
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert b.launched_world() == 8  # torchrun's variables win
