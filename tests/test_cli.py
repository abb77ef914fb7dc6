"""CLI drivers (Python and native) without hardware."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(*args, timeout=300):
    r = subprocess.run([sys.executable, "-m", "tenzing_amd", *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_python_cli_sim_then_replay_then_rules(tmp_path):
    csv = tmp_path / "s.csv"
    out = _py("search", "--workload", "spmv", "--solver", "dfs", "--sim", "--streams", "2",
              "--bench-iters", "3", "--csv", str(csv))
    s = json.loads(out.strip().splitlines()[-1])
    assert s["candidates"] > 10 and s["best_pct10_ms"] > 0
    out = _py("search", "--workload", "spmv", "--replay", str(csv), "--streams", "2",
              "--iters", "30")
    r = json.loads(out.strip().splitlines()[-1])
    assert r["best_pct10_ms"] >= s["best_pct10_ms"] - 1e-12
    out = _py("rules", str(csv), "--out", str(tmp_path / "x_"))
    assert (tmp_path / "x_rules.txt").exists()


def test_python_cli_fused_sim():
    out = _py("search", "--workload", "fused", "--sim", "--streams", "4", "--iters", "20",
              "--neighbors", "26", "--bench-iters", "2")
    s = json.loads(out.strip().splitlines()[-1])
    names = {op["name"] for op in s["best_schedule"]}
    assert any(n.startswith("he_") for n in names) and any(n.startswith("spmv_") for n in names)


def test_native_cli_sim(tmp_path):
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    r = subprocess.run([exe, "--sim", "--workload", "halo", "--neighbors", "26", "--streams", "4",
                        "--iters", "20", "--bench-iters", "2", "--csv", str(tmp_path / "h.csv")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    summary = json.loads(r.stderr.strip().splitlines()[-1])
    assert summary["candidates"] == 20
    lines = (tmp_path / "h.csv").read_text().splitlines()
    assert json.loads(lines[0])["mcts__Opts"]["nIters"] == 20 and len(lines) == 21


def test_env_report():
    out = _py("env")
    j = json.loads(out)
    assert "tenzing_amd" in j and "rccl" in j
