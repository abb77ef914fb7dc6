"""CLI drivers (Python and native) without hardware."""
import json
import os
import signal
import subprocess
import sys
import time

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


def test_links_single_process():
    """`links` in one process: no pairs to measure, no GPU touched, still one JSON line"""
    j = json.loads(_py("links", "--mib", "1", "--iters", "1").strip().splitlines()[-1])
    assert j["ranks"] == 1 and j["link_matrix"]["why"] == "one rank: no pairs"
    assert j["peer_devices"]["summary"] == "no peers"


def test_env_report():
    out = _py("env")
    j = json.loads(out)
    assert "tenzing_amd" in j and "rccl_library" in j and "hip_runtime" in j
    # the runtime actually mapped into the process, not /opt/rocm's version file
    assert j["hip_runtime"]["path"] and "libamdhip64" in j["hip_runtime"]["path"]
    assert j["rccl_library"]["path"] and "librccl" in j["rccl_library"]["path"]
    assert j["rccl_library"]["version"].count(".") == 2


def test_native_cli_sigint_dumps_partial_csv():
    """reference trap.cpp:26-30 / mcts.hpp:175-178: SIGINT during a search prints the results
    gathered so far as CSV and exits 1"""
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    p = subprocess.Popen([exe, "--sim", "--workload", "halo", "--neighbors", "26", "--streams", "4",
                          "--iters", "100000000", "--bench-iters", "2"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    time.sleep(4.0)
    p.send_signal(signal.SIGINT)
    out, err = p.communicate(timeout=60)
    assert p.returncode == 1, err[-2000:]
    lines = out.strip().splitlines()
    assert json.loads(lines[0])["mcts__Opts"]["nIters"] == 100000000
    rows = lines[1:]
    assert len(rows) >= 1
    for r in rows:
        f = r.split("|")
        assert int(f[0]) >= 0 and float(f[2]) > 0
        json.loads(f[7])  # first op of the schedule


def test_cpulist_parsing_and_binding(monkeypatch):
    """GPU-local CPU binding (the reference's dead NUMA binding, numa.cpp:13): sysfs cpulist
    parsing, and binding restricted to the CPUs this process may use"""
    from tenzing_amd.utils import env

    assert env.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert env.parse_cpulist("") == []
    allowed = sorted(os.sched_getaffinity(0))
    mine = allowed[:4]
    monkeypatch.setattr(env, "local_cpus", lambda dev: mine + [10 ** 6])
    try:
        assert env.bind_local_cpus(0) == mine
        assert os.sched_getaffinity(0) == set(mine)
    finally:
        os.sched_setaffinity(0, allowed)
    if len(allowed) >= 4:
        # one usable local CPU out of several allowed: too few to pin the process to
        monkeypatch.setattr(env, "local_cpus", lambda dev: [allowed[0], 10 ** 6])
        assert env.bind_local_cpus(0) == []
        assert sorted(os.sched_getaffinity(0)) == allowed
    monkeypatch.setattr(env, "local_cpus", lambda dev: [])
    assert env.bind_local_cpus(0) == []
    assert sorted(os.sched_getaffinity(0)) == allowed


def test_example_sim_design_rules(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "sim_design_rules.py"),
                        "--out", str(tmp_path / "ex_")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "24 schedules" in r.stdout and "b and c same stream" in r.stdout
    assert (tmp_path / "ex_rules.txt").exists()


def test_cpp_library_example_sim():
    """examples/cpp/custom_kernel_op.hip: a user-defined kernel op searched through the C++
    library (built against build/libtenzing_amd.a), hardware-free"""
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-example-custom-op")
    r = subprocess.run([exe, "--sim"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["candidates"] == 24 and j["best_us"] < j["worst_us"]


def test_trace_best_chrome_json_sim(tmp_path):
    """--trace-best: the best schedule's timeline as Chrome trace events (here the discrete-event
    model's): one complete event per GPU op, on the track of its stream"""
    out = tmp_path / "best.json"
    _py("search", "--workload", "halo", "--sim", "--neighbors", "26", "--halo-n", "32",
        "--streams", "3", "--iters", "10", "--bench-iters", "2", "--fuse", "none",
        "--trace-best", str(out))
    ev = json.loads(out.read_text())["traceEvents"]
    ops = [e for e in ev if e["ph"] == "X"]
    names = {e["args"]["name"] for e in ev if e["ph"] == "M"}
    assert len(ops) == 26 and all(e["name"].startswith("he_direct_") for e in ops)
    assert all(e["dur"] > 0 and e["ts"] >= 0 for e in ops)
    assert "host" in names and {f"stream {e['tid'] - 1}" for e in ops} <= names


def test_save_best_then_load(tmp_path):
    """search --save-best writes a self-contained schedule; `run`'s loader rebuilds the graph
    from the saved options and proves the schedule race-free on it (no GPU: graph only)"""
    import tenzing_amd as tz
    from tenzing_amd import cli

    path = tmp_path / "best.json"
    out = _py("search", "--workload", "fused", "--sim", "--streams", "3", "--iters", "15",
              "--neighbors", "26", "--bench-iters", "2", "--save-best", str(path))
    s = json.loads(out.strip().splitlines()[-1])
    doc = json.loads(path.read_text())
    assert doc["ranks"] == 1 and doc["args"]["workload"] == "fused" and doc["args"]["streams"] == 3
    assert abs(doc["pct10_ms"] - s["best_pct10_ms"]) < 1e-9
    assert all("in_graph" in op for op in doc["schedule"])
    w, g, wl, seq = cli.load_schedule(doc, tz.SelfCtrl(), -1, False)
    assert w.neighbors == 26 and len(seq) == len(doc["schedule"])
    # a tampered schedule (a cross-stream wait removed) is refused
    waits = [i for i, op in enumerate(doc["schedule"]) if op.get("kind") == "CudaStreamWaitEvent"]
    if waits:
        bad = dict(doc, schedule=[op for i, op in enumerate(doc["schedule"]) if i != waits[0]])
        import pytest

        with pytest.raises(SystemExit, match="race-free"):
            cli.load_schedule(bad, tz.SelfCtrl(), -1, False)


def test_native_save_best_loads_in_python(tmp_path):
    """tz-search --save-best writes the same document format as the Python CLI (python-style
    option keys, the reference's schedule JSON), so either CLI can run the other's schedules"""
    import tenzing_amd as tz
    from tenzing_amd import cli

    path = tmp_path / "nbest.json"
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    r = subprocess.run([exe, "--sim", "--workload", "halo+spmv", "--neighbors", "26", "--streams",
                        "3", "--iters", "12", "--bench-iters", "2", "--fuse", "choice",
                        "--save-best", str(path), "--csv", str(tmp_path / "n.csv")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    doc = json.loads(path.read_text())
    assert doc["args"]["halo_n"] == 512 and doc["args"]["workload"] == "halo+spmv"
    assert doc["args"]["fuse"] == "choice" and doc["args"]["stencil"] is False
    w, g, wl, seq = cli.load_schedule(doc, tz.SelfCtrl(), -1, False)
    assert w.workload == "fused" and w.streams == 3 and len(seq) == len(doc["schedule"])


def test_seed_schedule_flag_both_clis(tmp_path):
    """search --save-best, then a new search seeded with that schedule measures it first (both
    CLIs read either CLI's document)"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    best = tmp_path / "best.json"
    r = subprocess.run([sys.executable, "-m", "tenzing_amd", "search", "--workload", "diamond", "--sim",
                 "--iters", "5", "--save-best", str(best)], cwd=root, capture_output=True, text=True,
                timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "tenzing_amd", "search", "--workload", "diamond", "--sim",
                 "--iters", "4", "--seed-schedule", str(best)], cwd=root, capture_output=True,
                text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["candidates"] == 5
    exe = os.path.join(root, "tenzing_amd", "bin", "tz-search")
    if os.path.exists(exe):
        r = subprocess.run([exe, "--workload", "diamond", "--sim", "--iters", "4", "--seed-schedule",
                     str(best)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [ln for ln in r.stderr.splitlines() if ln.startswith('{"best')][-1]
        assert json.loads(line)["candidates"] == 5


def test_native_cli_deadline_prints_partial_csv():
    """--deadline: past it the native CLI prints the results CSV so far (opts line + rows) and
    exits 5, the reference's partial dump on the Slurm script's early SIGABRT
    (scripts/perlmutter/spmv.sh:12, src/trap.cpp:26-30)"""
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    r = subprocess.run([exe, "--sim", "--workload", "halo", "--neighbors", "26", "--streams", "4",
                        "--iters", "100000000", "--bench-iters", "50", "--deadline", "3"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 5, (r.returncode, r.stderr[-2000:])
    lines = r.stdout.strip().splitlines()
    assert json.loads(lines[0])["mcts__Opts"]["nIters"] == 100000000
    rows = lines[1:]
    assert len(rows) >= 1 and all(len(x.split("|")) > 7 for x in rows)
    assert [int(x.split("|")[0]) for x in rows] == list(range(len(rows)))
    assert "run deadline" in r.stderr


def test_native_cli_two_ranks_port_rendezvous():
    """tz-search started the torchrun way (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, no
    file): the native control plane's port rendezvous, a collective simulated search, the
    results CSV from rank 0 only"""
    import socket

    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = []
    for r in (0, 1):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        ps.append(subprocess.Popen([exe, "--workload", "diamond", "--sim", "--iters", "6",
                                    "--streams", "2"], env=env, stdout=subprocess.PIPE,
                                   stderr=subprocess.PIPE, text=True))
    try:
        outs = [p.communicate(timeout=120) for p in ps]
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in ps), [e[-1500:] for _, e in outs]
    best = [json.loads(ln) for ln in outs[0][1].splitlines() if ln.startswith('{"best')]
    assert best and best[0]["ranks"] == 2 and best[0]["candidates"] == 6
    assert sum(ln.startswith("0|") for ln in outs[0][0].splitlines()) == 1
    assert not any(ln.startswith("0|") for ln in outs[1][0].splitlines())


def test_saved_wide_put_schedule_loads_where_auto_would_not_offer_it():
    """a schedule searched on a node, where "auto" offered the wide put, loads anywhere: the
    saved options say "auto", the schedule's he_putw_ ops turn the wide put on again"""
    import tenzing_amd as tz
    from tenzing_amd.cli import load_schedule
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.search import greedy_schedule

    class EightRanks:  # graph-only builds read the rank and the size
        rank, size = 0, 8

    cfg = HaloConfig(n=16, neighbors=26, fuse="all", transport="auto", wide_puts="on",
                     relay="off", hostsplit="off")
    _, g = build_halo(cfg, EightRanks(), setup=False)
    s = greedy_schedule(g, tz.Platform(2), {"he_remote": "he_via_ipcw"})
    assert any(o.name.startswith("he_putw_") for o in s.ops())
    doc = {"ranks": 8, "args": {"workload": "halo", "streams": 2, "halo_n": 16, "neighbors": 26,
                                "fuse": "all", "transport": "auto", "relay": "off",
                                "hostsplit": "off", "wide_puts": "auto"},
           "schedule": json.loads(s.json(True))}
    w, g2, wl, seq = load_schedule(doc, EightRanks(), -1, False)
    assert w.wide_puts == "on" and any(o.name.startswith("he_putw_") for o in seq.ops())


def test_bench_names_the_transport_of_a_schedule():
    """bench.py's transport label per schedule (op-name prefixes): kernel puts of either width,
    copy engines, the mix, relay and host-split shares"""
    from tenzing_amd.utils import benchkit as bench

    assert bench.remote_via(["he_direct_self", "he_put_ipc_all"]) == "ipc"
    assert bench.remote_via(["he_direct_self", "he_putw_w_all", "he_wait_w_remote"]) == "ipc_wide"
    assert bench.remote_via(["he_put_mx", "he_copyput_mx"]) == "mixed"
    assert bench.remote_via(["he_rl20_putd", "he_rl20_putc"]) == "relay20"
    assert bench.remote_via(["he_hs30_putd", "he_hs30_puth"]) == "hostsplit30"
    assert bench.remote_via(["he_direct_all"]) is None
    assert bench.schedule_via(["he_direct_a", "he_putw_x"]) == ["direct", "ipc_wide"]


def test_grid_memory_option_in_both_clis():
    """both CLIs take --grid-memory, and the native one refuses a bad value"""
    out = _py("search", "--workload", "halo", "--sim", "--streams", "2", "--iters", "4",
              "--halo-n", "16", "--bench-iters", "2", "--grid-memory", "fine")
    assert json.loads(out.strip().splitlines()[-1])["candidates"] == 4
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    ok = subprocess.run([exe, "--sim", "--workload", "halo", "--halo-n", "16", "--streams", "2",
                         "--iters", "4", "--bench-iters", "2", "--grid-memory", "coarse"],
                        capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stderr[-2000:]
    bad = subprocess.run([exe, "--sim", "--workload", "halo", "--halo-n", "16", "--iters", "2",
                          "--grid-memory", "bogus"], capture_output=True, text=True, timeout=300)
    assert bad.returncode != 0 and "--grid-memory" in bad.stderr
