"""Several ranks on one MI355X (loopback): the ipc transport's pack-free peer puts, arrival
waits and the collective search, with every ghost cell verified on every rank.

Each rank is its own process (one process per rank, as on a multi-GPU node); here all ranks
share GPU 0, so their grids are IPC-mapped on the same device.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    """a MASTER_PORT whose control-plane port (MASTER_PORT + 1) is free as well"""
    for _ in range(100):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        t = socket.socket()
        try:
            t.bind(("0.0.0.0", p + 1))
        except OSError:
            continue
        finally:
            t.close()
        return p
    raise RuntimeError("no free port pair")


# RCCL between loopback ranks goes through RCCL's socket transport with every rank's kernels on
# one GPU. Part of the default suite again since round 4 (whole-schedule capture; every rank's
# log kept as it runs); TZ_TEST_NO_RCCL_LOOPBACK=1 skips them
rccl_loopback = pytest.mark.skipif(os.environ.get("TZ_TEST_NO_RCCL_LOOPBACK") == "1",
                                   reason="RCCL across loopback ranks skipped (TZ_TEST_NO_RCCL_LOOPBACK=1)")


def _tails(logs, n=40):
    out = []
    for r, path in enumerate(logs):
        try:
            with open(path) as f:
                lines = f.read().splitlines()
        except OSError:
            lines = ["(no log)"]
        out.append(f"== rank {r} ({path}), last {n} lines:\n" + "\n".join(lines[-n:]))
    return "\n".join(out)


def _launch(case, world, timeout=150, extra_env=None, tmp_path=None):
    """W rank processes of gpu_rank_body.py; each rank's output goes to its own file AS IT RUNS
    (TZ_TEST_VERBOSE progress lines, watchdog and [tz] messages), so a rank that hangs or dies
    still leaves its trace: on a failure or a timeout every rank's tail is printed. The files go
    under TZ_TEST_LOGDIR when set (e.g. gpurun_out/..., so they come back from the GPU box even
    when the whole run is killed). The limits are below the GPU box's 180 s silence limit: a
    rank blocked in a control-plane collective fails after TZ_CTRL_TIMEOUT_S (90 s here), and
    the test itself after `timeout`, each with the ranks' tails."""
    import tempfile

    port = _free_port()
    base = os.environ.get("TZ_TEST_LOGDIR")
    if base:
        os.makedirs(base, exist_ok=True)
        logdir = tempfile.mkdtemp(prefix=f"{case}_w{world}_", dir=base)
    else:
        logdir = str(tmp_path) if tmp_path is not None else tempfile.mkdtemp(prefix=f"tz_{case}_")
    procs, logs = [], []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TZ_TEST_VERBOSE="1",
                   PYTHONFAULTHANDLER="1", TZ_CTRL_TIMEOUT_S=os.environ.get("TZ_CTRL_TIMEOUT_S", "90"),
                   **(extra_env or {}))
        path = os.path.join(logdir, f"{case}_rank{r}.log")
        logs.append(path)
        f = open(path, "w")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "gpu_rank_body.py"), case],
                                      env=env, stdout=f, stderr=subprocess.STDOUT, text=True))
        f.close()
    import time

    t0 = time.time()
    try:
        for p in procs:
            try:
                p.wait(timeout=max(1.0, timeout - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                pytest.fail(f"{case} on {world} ranks: no exit within {timeout} s\n" + _tails(logs))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    res = []
    for r, p in enumerate(procs):
        if p.returncode != 0:
            pytest.fail(f"{case}: rank {r} exited with {p.returncode}\n" + _tails(logs))
        with open(logs[r]) as f:
            lines = [x for x in f.read().splitlines() if x.startswith("RESULT ")]
        assert lines, _tails(logs)
        res.append(json.loads(lines[-1][len("RESULT "):]))
    return res


@pytest.mark.parametrize("world,mode", [(2, "grid"), (4, "grid"), (2, "buffers"), (8, "grid"),
                                        (8, "buffers")])
def test_ipc_halo_loopback(gpu, world, mode):
    """8 ranks form the 2x2x2 grid of the driver's 8-GPU run: no self-neighbours, both
    neighbours along every axis are one rank, and 26 directions reach 7 distinct peers"""
    extra = {"TZ_IPC_GRID": "1" if mode == "grid" else "0"}
    if world == 8:
        extra.update(TZ_TEST_N="24", TZ_TEST_FUSES="choice")
    res = _launch("ipc_halo", world, extra_env=extra)
    nf = 1 if world == 8 else 2
    for r in res:
        assert r["size"] == world
        # only rank 0 holds the search results; every rank ran every candidate
        assert r["mcts"] == ([4] * nf if r["rank"] == 0 else [0] * nf)
        assert r["mcts_err"] == [0] * nf
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run
            # 2 ranks: grid 1x1x2 (x, y self-neighbours move directly); 4 ranks: 1x2x2;
            # 8 ranks: 2x2x2, every direction remote
            assert run["transport"] == ("ipc" if world == 8 else "direct+ipc")
        # peers store into the grid itself in grid mode: fine-grained memory there
        assert r["grid_memory"] == ("fine" if mode == "grid" else "coarse"), r["grid_memory"]
        # buffers mode also offers copy-engine (SDMA) puts: some schedules must have used them
        used = any(run["copyput"] for run in r["runs"])
        if mode == "grid" or world < 8:  # (8 ranks sample too few schedules to insist)
            assert used == (mode == "buffers"), [run["copyput"] for run in r["runs"]]


@pytest.mark.parametrize("world", [2, 8])
def test_mixed_engines_loopback(gpu, world):
    """buffers mode's mixed transport: the + face of every axis by CU stores, the - face by the
    copy engines, into the same receive buffers and arrival counters; every ghost right, eager
    and as hipGraphs, over repeated exchanges"""
    extra = {"TZ_IPC_GRID": "0", "TZ_TEST_FUSES": "choice", "TZ_TEST_REQUIRE": "he_copyput_mx",
             "TZ_TEST_SEEDS": "2", "TZ_TEST_NO_MCTS": "1"}
    if world == 8:
        extra.update(TZ_TEST_N=os.environ.get("TZ_HS_N", "24"), TZ_TEST_RELAY="off")
    res = _launch("ipc_halo", world, extra_env=extra)
    for r in res:
        assert r["runs"], r
        for run in r["runs"]:
            assert run["mixed"] and run["copyput"], run
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


def test_copy_puts_over_two_engines_loopback(gpu):
    """copy-engine puts cut over two engine streams (copy_engines=2: a fork to a side stream
    and a join back inside the op): exact eager and inside whole-schedule hipGraph captures,
    where the side stream's capture dependencies are set per op (no false edge between copy ops
    of different schedule streams)"""
    extra = {"TZ_IPC_GRID": "0", "TZ_TEST_COPY_ENGINES": "2", "TZ_TEST_FUSES": "choice",
             "TZ_TEST_REQUIRE": "he_copyput_", "TZ_TEST_SEEDS": "3", "TZ_TEST_NO_MCTS": "1"}
    res = _launch("ipc_halo", 2, extra_env=extra)
    for r in res:
        assert r["runs"] and all(run["copyput"] for run in r["runs"]), r["runs"]
        assert {run["mode"] for run in r["runs"]} == {"ExecMode.Eager", "ExecMode.Graph"}
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


@pytest.mark.parametrize("grid_mode", ["1", "0"])
def test_wide_puts_loopback(gpu, grid_mode):
    """wide kernel puts (256 workgroups per box, forced on: loopback ranks share one GPU, where
    "auto" does not offer them): preflighted at setup, then exact eager and as hipGraphs over
    repeated exchanges, in grid and buffers mode"""
    extra = {"TZ_IPC_GRID": grid_mode, "TZ_TEST_WIDE": "on", "TZ_TEST_FUSES": "none,choice",
             "TZ_TEST_REQUIRE": "he_putw_", "TZ_TEST_SEEDS": "2", "TZ_TEST_NO_MCTS": "1"}
    res = _launch("ipc_halo", 2, extra_env=extra)
    for r in res:
        assert r["transports"]["wide_put"].startswith("ok"), r["transports"]
        assert "he_via_ipcw" in r["graph_ops"]
        assert r["runs"] and all(run["wide"] for run in r["runs"]), r["runs"]
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


def test_relay_routing_loopback(gpu):
    """the 2x2x2 grid with every remote direction through relay routing (a share of each face
    via the corner peer, forwarded over its edge-diagonal link): every ghost right on all 8
    ranks, eager and as hipGraphs, over repeated exchanges, and in a collective search"""
    extra = {"TZ_IPC_GRID": "0", "TZ_TEST_N": "24", "TZ_TEST_FUSES": "choice",
             "TZ_TEST_RELAY": "force"}
    res = _launch("ipc_halo", 8, extra_env=extra)
    for r in res:
        assert r["relay_ready"] and r["mcts_err"] == [0]
        assert r["mcts"] == ([4] if r["rank"] == 0 else [0])
        for run in r["runs"]:
            assert run["relay"], run
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


def test_ipc_abort_recovery_loopback(gpu):
    """a candidate hangs on one rank: every rank's watchdog aborts it (device waits released),
    the benchmarker fails it on both ranks, the recovery hooks reset the IPC put / wait counters
    everywhere, and the next candidate's exchanges are exact again"""
    res = _launch("ipc_abort", 2, extra_env={"TZ_IPC_GRID": "0"})
    for r in res:
        assert r["hang_first"] and r["failed"] and r["recovered"], r
        assert r["fail_s"] < 60, r
        assert r["bad"] == 0 and r["bad2"] == 0 and r["err"] == 0, r
    assert res[0]["fired"] >= 1


@pytest.mark.parametrize("world,chunks", [(2, 1), (2, 4), (8, 1), (8, 4)])
def test_hostsplit_loopback(gpu, world, chunks):
    """host split: a share of every face through node shared host memory (POSIX shm mapped for
    each rank's GPU: kernel stores into the receiver's inbox, single-writer flag stores, DMA
    back out), the rest as IPC puts; both shares offered; every ghost right on every rank, eager
    and as hipGraphs, over repeated exchanges, and in a collective search"""
    extra = {"TZ_IPC_GRID": "0", "TZ_TEST_FUSES": "choice", "TZ_TEST_HOSTSPLIT": "force",
             "TZ_TEST_HS_CHUNKS": str(chunks)}
    if world == 8:
        extra.update(TZ_TEST_N=os.environ.get("TZ_HS_N", "24"), TZ_TEST_RELAY="off")
    res = _launch("ipc_halo", world, extra_env=extra)
    for r in res:
        assert r["hostsplit_ready"] and r["mcts_err"] == [0], r
        assert r["mcts"] == ([4] if r["rank"] == 0 else [0])
        for run in r["runs"]:
            assert run["hostsplit"], run
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


@pytest.mark.parametrize("mode", ["grid", "buffers"])
def test_bench_two_ranks_loopback(gpu, tmp_path, mode):
    """the driver's multi-GPU bench flow (torchrun, one process per rank, collective search,
    best-schedule broadcast, device-side verification, eager + hipGraph timing, max over ranks,
    per-link transport probes) with both ranks on this one GPU. RCCL refuses two ranks on one
    device, so this also checks the collective fallback to the IPC transport."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--cells", "64", "--mcts-iters", "6", "--bench-iters", "3", "--deadline-s", "240", "--subrecords", "off"]
    env = dict(os.environ, TZ_IPC_GRID="1" if mode == "grid" else "0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=160, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    j = json.loads(line)
    assert j["n_gpus"] == 2 and j["steps"] == 6 and j["verified_bad_cells"] == 0
    assert j["transport"] == "direct+ipc" and j["config"]["rank_grid"] == [1, 1, 2]
    assert j["value"] > 0 and j["higher_is_better"] is False
    assert j["ipc_mode"] == mode
    # the timed schedule once more against the independent torch model, every rank's block
    tm = j["torch_model_check"]
    assert tm.get("bad_cells") == 0 and sum(tm["by_ghost_class"]) == 0, tm
    # self-describing multi-GPU record: RCCL refused (two ranks on one device), its reason
    # recorded, no communicator size; IPC passed its preflight
    assert j["partial"] is False and j["phase"] == "done"
    ta = j["transports_available"]
    assert ta["ipc"] == "ok" and ta["rccl"] != "ok" and ta["rccl"] != "not offered", ta
    assert j["rccl_nranks"] is None
    assert j["transport_by_group"]["remote"]["dirs"] == 18
    assert j["transport_by_group"]["local"] == {"dirs": 8, "via": "direct"}
    assert j["transport_by_group"]["remote"]["via"] in ("ipc", "sdma", "memcpy", "mixed",
                                                        "hostsplit10", "hostsplit20", "hostsplit30", "hostsplit40")
    assert j["watchdog"]["fired"] == 0 and j["dead_domains"] == []
    # device-pair facts: on one GPU every peer is this rank's own device, and the IPC-mapped
    # peer memory says so; the record names the HIP runtime / RCCL actually mapped
    pd = j["peer_devices"]
    assert pd["peers"] and all(p["same_device"] and p["ipc_mapping_consistent"]
                               for p in pd["peers"].values()), pd
    assert ta["peer_access"].endswith("(loopback)")
    assert "libamdhip64" in j["runtime"]["hip_runtime"]["path"]
    assert "librccl" in j["runtime"]["rccl_library"]["path"]
    # the link-aware model's best structures seeded too, each measured (loopback rates say
    # nothing about xGMI: only the plumbing is checked here)
    ms = j["model_seeded"]
    assert ms and len(ms) <= 2 and all(d["model_us"] > 0 and d["measured_ms"] > 0 for d in ms), ms
    if mode == "buffers":
        # one seed per remote transport, each measured before the search
        assert set(j["seeded_pct10_ms"]) == {"ipc", "sdma", "memcpy", "mixed", "hostsplit10",
                                             "hostsplit20", "hostsplit30", "hostsplit40"}, j["seeded_pct10_ms"]
        assert j["transports_available"]["hostsplit"] == "ok"
    p = j["link_probe"]
    # kernel puts always; copy-engine puts need receive buffers; RCCL is refused in loopback
    assert p["GBps"]["put"] > 0 and "rccl" not in p["GBps"]
    # the wide kernel put is probed everywhere but offered to the search only where peers sit on
    # other devices ("auto")
    assert p["GBps"]["put_wide"] > 0 and p["pair_GBps"]["put_wide"] > 0
    assert j["wide_puts_offered"] is False
    assert set(p["put_GBps_by_blocks_per_box"]) == {"16", "64", "256", "1024"}
    # all pairs, both engines: 2 x 2 with the diagonal unmeasured
    lm = j["link_matrix"]
    assert lm["why"] == "", lm
    for key in ("put_GBps", "sdma_GBps"):
        m = lm[key]
        assert len(m) == 2 and m[0][0] == m[1][1] == -1 and m[0][1] > 0 and m[1][0] > 0, lm
    assert lm["summary"]["put"]["pairs"] == 2 and lm["summary"]["sdma"]["spread"] >= 1.0, lm
    assert all(v > 0 for v in p["put_GBps_by_blocks_per_box"].values()), p
    assert (p["GBps"]["sdma"] is not None) == (mode == "buffers")
    assert (p["GBps"]["memcpy"] is not None) == (mode == "buffers")
    # both z faces at once (2 ranks: one peer): kernel puts always, copy engines and the
    # kernel + copy-engine mix in buffers mode
    assert p["pair_GBps"]["put"] > 0
    # 2 ranks: 1x1x2, only the z faces are remote
    assert set(p["put_GBps_by_axis"]) == {"z"}
    assert (p["pair_GBps"]["sdma"] is not None) == (p["pair_GBps"]["mixed"] is not None) == (mode == "buffers")
    assert p["busiest_link_MB"] > p["face_MB"] > 0 and p["busiest_link_at_probe_rate_ms"] > 0
    # the model calibrated on these rates, beside the measured per-transport seeds
    assert j["post_timing"]["done"] == ["torch_model", "link_probe", "link_matrix", "topology", "model_check"]
    mc = j["model_check"]
    assert "error" not in mc, mc
    seeded = {r["transport"]: r for r in mc["seeds"] if r["measured_us"] is not None}
    # (grid mode offers the kernel puts alone: nothing seeded, nothing to compare)
    assert set(seeded) == set(j["seeded_pct10_ms"] or {}), mc
    assert mc["seeds"] and all(r["model_us"] > 0 for r in mc["seeds"]), mc
    assert mc["best_measured"] in (seeded or {None: 0})


def test_bench_two_ranks_under_mpiexec(gpu):
    """the same bench flow started the reference's way, by an MPI launcher: the control plane is
    MPI_COMM_WORLD (MpiCtrl), so the schedule broadcasts, max-reductions and the IPC handle
    exchange all go over MPI, while the transfers stay on the GPU"""
    import shutil

    mpiexec = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
    if not os.path.exists(mpiexec):
        pytest.skip("no MPI launcher")
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [mpiexec, "-n", "2", sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "6", "--warmup", "2", "--cells", "64", "--mcts-iters", "6",
           "--bench-iters", "3", "--deadline-s", "240", "--subrecords", "off", "--link-probe-iters", "0"]
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=160, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one result line
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["verified_bad_cells"] == 0 and j["verified_bad_cells_after_timing"] == 0
    # 6 search iterations plus the seeds measured before them (one per transport, the model's)
    seeds = len(j["seeded_pct10_ms"] or {}) + len(j["model_seeded"] or [])
    assert j["config"]["rank_grid"] == [1, 1, 2] and 6 <= j["mcts_candidates"] <= 6 + seeds, j


def test_native_cli_two_ranks_under_mpiexec(gpu):
    """tz-search started by mpiexec (no torchrun): MPI control plane, IPC puts between the two
    loopback ranks, a collective search and the final check of the best schedule"""
    import shutil

    mpiexec = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
    exe = os.path.join(ROOT, "tenzing_amd", "bin", "tz-search")
    if not os.path.exists(mpiexec) or not os.path.exists(exe):
        pytest.skip("no MPI launcher or tz-search")
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([mpiexec, "-n", "2", exe, "--workload", "halo", "--halo-n", "48",
                        "--neighbors", "26", "--transport", "ipc", "--iters", "6", "--streams", "2",
                        "--bench-iters", "3", "--target-secs", "0.001"],
                       cwd="/tmp", capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = [x for x in r.stderr.splitlines() if x.startswith('{"best')][-1]
    j = json.loads(line)
    assert j["ranks"] == 2 and j["candidates"] == 6


def test_links_cli_three_ranks_loopback(gpu, tmp_path):
    """`python -m tenzing_amd links` on 3 ranks started the torchrun way (RANK / WORLD_SIZE /
    MASTER_*): the all-pairs matrix covers all 6 ordered pairs by kernel put and SDMA, and the
    peer facts say loopback (every peer on this rank's GPU)"""
    port = _free_port()
    procs, logs = [], []
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TZ_CTRL_TIMEOUT_S="60")
        path = tmp_path / f"links{r}.log"
        logs.append(str(path))
        with open(path, "w") as f:
            procs.append(subprocess.Popen([sys.executable, "-m", "tenzing_amd", "links", "--mib", "8",
                                           "--iters", "3"], cwd=ROOT, env=env, stdout=f,
                                          stderr=subprocess.STDOUT, text=True))
    try:
        for p in procs:
            p.wait(timeout=120)
    except subprocess.TimeoutExpired:
        pytest.fail("links: no exit within 120 s\n" + _tails(logs))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert all(p.returncode == 0 for p in procs), _tails(logs)
    with open(logs[0]) as f:
        j = json.loads([x for x in f.read().splitlines() if x.startswith('{"ranks"')][-1])
    lm = j["link_matrix"]
    assert j["ranks"] == 3 and lm["why"] == "" and lm["iters"] == 3, j
    for key in ("put_GBps", "sdma_GBps"):
        m = lm[key]
        assert all((m[r][q] > 0) == (r != q) for r in range(3) for q in range(3)), lm
    assert all(f["same_device"] for f in j["peer_devices"]["peers"].values()), j["peer_devices"]


@pytest.mark.parametrize("world,case", [(2, "spmv"), (4, "spmv"), (8, "spmv"), (2, "fused")])
def test_spmv_ipc_loopback(gpu, world, case):
    """distributed SpMV (and SpMV + halo in one graph, BASELINE config 5) on several ranks of
    one GPU: RCCL refuses the shared device, so the x halo goes through IPC puts; every rank's
    y is checked against the host reference after every schedule"""
    res = _launch(case, world)
    for r in res:
        assert r["size"] == world and r["transport"] == "ipc"
        assert r["mcts"] == (6 if r["rank"] == 0 else 0)
        for run in r["runs"]:
            assert run["err1"] < 1e-4 and run["err2"] < 1e-4, run
            assert run["bad"] == 0 and run["ipc_err"] == 0 and run["ipc"], run


def test_stencil_mode_loopback(gpu):
    """exchange + stencil on 2 ranks of one GPU (IPC): ghosts and every stencil output cell are
    right on both ranks, whichever stencil alternative a schedule takes"""
    res = _launch("ipc_halo", 2, extra_env={"TZ_TEST_STENCIL": "1", "TZ_TEST_FUSES": "choice"})
    for r in res:
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


def test_bench_host_fallback_loopback(gpu, tmp_path):
    """neither device transport available (RCCL refuses two ranks on one device, IPC is made
    to fail its setup): the remote directions go through the host-staged transport (device ->
    host -> control plane -> host -> device), and the run still produces a verified number"""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--cells", "48", "--mcts-iters", "6", "--bench-iters", "2", "--deadline-s", "240", "--subrecords", "off",
           "--link-probe-iters", "0", "--copy-puts", "off"]
    env = dict(os.environ, TZ_FAIL_TRANSPORTS="ipc")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=160, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    j = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert j["verified_bad_cells"] == 0 and j["value"] > 0
    assert j["transport"] == "direct+host", j["transport"]
    ta = j["transports_available"]
    assert ta["host"] == "ok" and "simulated" in ta["ipc"] and ta["rccl"] != "ok", ta
    assert j["schedule_transport"] == "direct+host"
    assert j["transport_by_group"]["remote"]["via"] == "host"
    assert j["rccl_nranks"] is None
    # host ops cannot be captured: the candidates and the timing ran eagerly
    assert j["timed_mode"] == "eager"


def test_copy_preflight_failure_drops_only_that_variant_loopback(gpu):
    """the SDMA copy-engine put fails its own verified preflight (simulated): every rank drops
    that variant (and the mixed puts and relay copy forwards built on it) with the reason
    recorded, the runtime-engine copy puts and kernel puts stay, and every schedule is exact"""
    extra = {"TZ_IPC_GRID": "0", "TZ_FAIL_TRANSPORTS": "sdma_put", "TZ_TEST_FUSES": "choice",
             "TZ_TEST_SEEDS": "4", "TZ_TEST_NO_MCTS": "1"}
    res = _launch("ipc_halo", 2, extra_env=extra)
    for r in res:
        ta = r["transports"]
        assert "simulated" in ta["sdma_put"] and ta["memcpy_put"] == "ok" and ta["ipc"] == "ok", ta
        assert not any(o.startswith(("he_via_sdma", "he_via_mixed")) for o in r["graph_ops"])
        assert "he_via_memcpy" in r["graph_ops"]
        for run in r["runs"]:
            assert not run["copyput"] and not run["mixed"], run
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0 and run["err"] == 0, run


def test_bench_rejected_finalist_loopback(gpu):
    """a finalist that fails the bench's verification (forced: TZ_BENCH_REJECT=1) is rejected
    and the next one verified and timed; the record lists the rejection"""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--cells", "48", "--mcts-iters", "8", "--bench-iters", "2", "--deadline-s", "240", "--subrecords", "off",
           "--link-probe-iters", "0", "--hostsplit", "off"]
    env = dict(os.environ, TZ_IPC_GRID="0", TZ_BENCH_REJECT="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=160, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    j = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert j["verified_bad_cells"] == 0 and j["verified_bad_cells_after_timing"] == 0
    assert j["partial"] is False and j["value"] > 0
    rej = j["verify_rejected"]
    assert len(rej) == 1 and rej[0]["rank_in_rerank"] == 0 and rej[0]["bad"] >= 1, rej
    assert j["transports_available"]["sdma_put"] == "ok"
    assert j["transports_available"]["memcpy_put"] == "ok"


@rccl_loopback
def test_rccl_node_overlaps_kernels_loopback(gpu):
    """an RCCL send/recv between two real ranks as a node of a whole-schedule-captured hipGraph,
    beside two independent ~200 us kernels on two other streams: exact data over three value
    generations; the RCCL node (a kernel plus its network proxy's host node) is an ordinary
    branch of the graph, so the two kernels still overlap (round 3's child graphs serialized
    every node: 424 us for the two kernels alone). HIP's graph executor runs a third branch of
    any kind partly behind the first two (~295 us with a 50 us kernel instead of RCCL,
    profiles/archive/r4_capture/), which the bound allows for"""
    res = _launch("rccl_overlap", 2, extra_env={"TZ_RCCL_LOOPBACK": "1"})
    for r in res:
        assert r["effective_mode"] == "ExecMode.Graph" and r["bad"] == [0, 0, 0], r
        # 2 busy kernels + the RCCL kernel (RCCL may add a kernel node of its own)
        assert r["node_types"].get("kernel") in (3, 4) and "child_graph" not in r["node_types"], r
        # concurrent kernels: never the serial sum of the two
        assert r["iter_us"] < 1.75 * r["one_kernel_us"], r


def test_rccl_node_overlaps_kernels_one_process(gpu):
    """the same probe in one process (a 1-rank communicator sending to itself): no second process
    shares the GPU and RCCL needs no network proxy, so its captured node is one kernel. The RCCL
    node beside two independent 200 us kernels then costs what any short third branch does:
    231.6-244.4 us per launch measured on different boxes (profiles/archive/r4_self_overlap/), within
    VERDICT r3's 250 us; the assertion leaves box-to-box variance some room (1.3 x one kernel)"""
    res = _launch("rccl_overlap", 1, extra_env={"TZ_TEST_COMMS": "1"})
    r = res[0]
    assert r["effective_mode"] == "ExecMode.Graph" and r["bad"] == [0, 0, 0], r
    assert r["node_types"] == {"kernel": 3}, r
    assert r["iter_us"] <= 1.3 * r["one_kernel_us"], r


@rccl_loopback
@pytest.mark.parametrize("world", [2, 4])
def test_rccl_halo_across_ranks_loopback(gpu, world):
    """RCCL between real ranks: each rank gets a host id of its own (TZ_RCCL_LOOPBACK=1), so
    RCCL accepts several ranks on one GPU and connects them through its network transport. The
    halo's RCCL transport (per-direction and fused send/recv groups on the ordering domain's
    communicator) then runs across rank boundaries, eagerly and captured into hipGraphs, after
    the verified RCCL preflight, and (2 ranks) in a collective search; every ghost cell is
    checked.

    4 ranks run the seeded schedules only, eager and as hipGraphs: in round 6 one full-suite run
    of 3 hung in the search's random candidates, where 4 processes' RCCL kernels of up to 3
    communicators spin on one GPU's queues for data that their peers' proxies move over
    sockets (every rank's watchdog fired at its 60 s floor). On a node each rank has a GPU of
    its own; the 2-rank case keeps the search across real RCCL rank boundaries"""
    extra = {"TZ_RCCL_LOOPBACK": "1", "TZ_TEST_TRANSPORT": "rccl", "TZ_TEST_SEEDS": "2"}
    if world > 2:
        extra["TZ_TEST_NO_MCTS"] = "1"
    res = _launch("ipc_halo", world, extra_env=extra)
    for r in res:
        # "ok", or "ok (eager only: ...)" when RCCL inside hipGraphs failed its preflight (then
        # the graph-mode runs below ran eagerly, and must still be exact)
        assert r["transports"]["rccl"].startswith("ok"), r["transports"]
        assert r["rccl_nranks"] == world
        if world <= 2:
            assert r["mcts"] == ([4, 4] if r["rank"] == 0 else [0, 0]) and r["mcts_err"] == [0, 0]
        for run in r["runs"]:
            assert run["transport"] == "rccl", run
            assert run["bad1"] == run["bad2"] == run["bad3"] == 0, run


@rccl_loopback
def test_bench_rccl_across_ranks_loopback(gpu):
    """the driver's bench flow with RCCL working between the two ranks (TZ_RCCL_LOOPBACK=1):
    RCCL passes its preflight, the record shows a 2-rank communicator, RCCL is seeded and
    measured beside the IPC transports, and the timed schedule is verified"""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--cells", "48", "--mcts-iters", "8", "--bench-iters", "2", "--deadline-s", "240", "--subrecords", "off",
           "--link-probe-iters", "2", "--link-probe-rccl", "--hostsplit", "off"]
    env = dict(os.environ, TZ_IPC_GRID="0", TZ_RCCL_LOOPBACK="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=160, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    j = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert j["verified_bad_cells"] == 0 and j["verified_bad_cells_after_timing"] == 0
    assert j["transports_available"]["rccl"].startswith("ok") and j["rccl_nranks"] == 2
    assert j["transport"] == "direct+rccl+ipc", j["transport"]
    assert "rccl" in j["seeded_pct10_ms"], j["seeded_pct10_ms"]
    assert j["link_probe"]["GBps"]["rccl"] > 0


@rccl_loopback
@pytest.mark.parametrize("fail_schedule", [False, True])
def test_spmv_rccl_across_ranks_loopback(gpu, fail_schedule):
    """the distributed SpMV's x halo through RCCL between real ranks (TZ_RCCL_LOOPBACK=1):
    its preflight verifies the exchange compiled into hipGraphs (whole-schedule capture, or
    child capture when the former is forced to deliver wrong data), then every schedule's y is
    checked against the host reference, eagerly and as hipGraphs, then a collective search"""
    env = {"TZ_RCCL_LOOPBACK": "1", "TZ_TEST_SPMV_TRANSPORT": "rccl"}
    if fail_schedule:
        env["TZ_FAIL_TRANSPORTS"] = "rccl_graph_schedule"
    res = _launch("spmv", 2, extra_env=env)
    for r in res:
        assert r["transport"] == "rccl", r["transport"]
        assert r["rccl_graph_ok"], r["rccl_capture"]
        if fail_schedule:
            assert r["rccl_capture"].startswith("child capture (schedule capture: "), r["rccl_capture"]
        else:
            assert r["rccl_capture"] == "schedule capture", r["rccl_capture"]
        assert r["mcts"] == (6 if r["rank"] == 0 else 0)
        for run in r["runs"]:
            assert run["err1"] < 1e-4 and run["err2"] < 1e-4, run
            assert not run["ipc"], run


@pytest.mark.parametrize("how", ["phase", "transfer"])
def test_bench_stall_after_headline_loopback(gpu, how):
    """a diagnostic after the headline stalls on every rank (phase: the link-matrix phase never
    returns; transfer: every link-matrix transfer never completes): the final line still comes
    out complete (partial false) with exit status 0 on every rank, within the post-timing
    budget, and says which diagnostic did not finish"""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--cells", "48", "--mcts-iters", "4", "--bench-iters", "3", "--deadline-s", "300",
           "--link-probe-iters", "2", "--post-budget-s", "25", "--link-matrix-wait-s", "3"]
    env = dict(os.environ)
    if how == "phase":
        env["TZ_BENCH_STALL"] = "link_matrix"
    else:
        env["TZ_FAIL_TRANSPORTS"] = "link_matrix_stall"
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=170, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    j = json.loads(lines[0])
    assert j["partial"] is False and j["phase"] == "done" and j["verified_bad_cells"] == 0
    assert j["value"] > 0 and "link_probe" in j["post_timing"]["done"]
    if how == "phase":
        assert j["post_timing"]["running"] == "link_matrix" and "link_matrix" not in j
    else:
        lm = j["link_matrix"]
        assert lm["stuck"] is True and "did not complete" in lm["why"], lm
        assert "link_matrix" in j["post_timing"]["done"]


def test_bench_self_launched_two_ranks_with_subrecords_loopback(gpu):
    """`bench.py --gpus 2` with no launcher in the environment starts
    its own two rank processes (one line, n_gpus 2, rank grid 1x1x2), and the multi-GPU record
    carries BASELINE configs 2 and 5 searched over the ranks' transports, each verified exact,
    with the transport its winner used, the matrix's nnz summed over ranks and the RCCL
    communicator size (RCCL is refused for two ranks on one device, so the SpMV halo goes over
    IPC puts here)"""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "PMI_SIZE", "PMI_RANK", "PMIX_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
           "--warmup", "5", "--cells", "64", "--mcts-iters", "6", "--bench-iters", "3",
           "--deadline-s", "280", "--link-probe-iters", "2"]
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["launcher"] == "bench.py" and j["config"]["rank_grid"] == [1, 1, 2]
    assert j["partial"] is False and j["verified_bad_cells"] == 0
    assert j["verified_bad_cells_after_timing"] == 0
    assert j["torch_model_check"].get("bad_cells") == 0, j["torch_model_check"]
    assert "baseline_configs" in j["post_timing"]["done"], j["post_timing"]
    assert "reference_layout" not in j  # one-rank only
    bc = j["baseline_configs"]
    assert "error" not in bc, bc
    sp, fu = bc["spmv_c2"], bc["fused_c5"]
    for rec in (sp, fu):
        assert "error" not in rec, rec
        assert rec["verified_bad"] == 0 and rec["verified_bad_after_timing"] == 0, rec
        assert rec["ms_per_step"] > 0 and rec["config"]["ranks"] == 2
        assert rec["config"]["nnz"] == 1_500_000 and rec["config"]["bw"] == 75_000
        assert rec["config"]["spmv_transport"] in ("ipc", "rccl"), rec["config"]
    assert sp["config"]["rccl_nranks"] is None  # (loopback: RCCL refused)
    assert fu["config"]["halo_transport"] not in (None, "direct"), fu["config"]


@pytest.mark.parametrize("world", [2, 8])
def test_exchange_matches_independent_torch_model_loopback(gpu, world):
    """IPC puts between real ranks against the torch model of the exchange (random field,
    circular padding, strides as reported): 2 ranks (1x1x2, x and y wrap onto the rank itself)
    and 8 ranks (2x2x2, the driver's node, every direction remote), both orders, 6 and 26
    neighbours, eager and as hipGraphs"""
    res = _launch("parity", world, timeout=170,
                  extra_env={"TZ_TEST_ORDERS": "qxyz,xyzq" if world == 2 else "qxyz",
                             "TZ_TEST_SEEDS": "2" if world == 2 else "1",
                             # 8 ranks: the hashed field, each rank evaluating its own block
                             "TZ_TEST_FIELD": "random" if world == 2 else "hashed"})
    coords = set()
    for r in res:
        assert r["runs"], r
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == 0, run
            assert run["transport"] == ("ipc" if world == 8 else "direct+ipc"), run
        coords.add(tuple(r["runs"][0]["coords"]))
    assert len(coords) == world


@rccl_loopback
def test_rccl_exchange_matches_independent_torch_model_loopback(gpu):
    """the RCCL transport between 2 real ranks against the same model"""
    res = _launch("parity", 2, timeout=170,
                  extra_env={"TZ_RCCL_LOOPBACK": "1", "TZ_TEST_TRANSPORT": "rccl",
                             "TZ_TEST_ORDERS": "qxyz", "TZ_TEST_SEEDS": "1"})
    for r in res:
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == 0 and run["transport"] == "rccl", run


@pytest.mark.parametrize("world", [2, 4])
def test_odd_shape_exchange_matches_independent_torch_model_loopback(gpu, world):
    """odd interior size, 2 quantities, ghost 2, both orders, IPC puts between real ranks
    (1x1x2 and 1x2x2), against the torch model's hashed field"""
    res = _launch("parity", world, timeout=170,
                  extra_env={"TZ_TEST_N": "17", "TZ_TEST_NQ": "2", "TZ_TEST_GHOST": "2",
                             "TZ_TEST_SEEDS": "1", "TZ_TEST_FIELD": "hashed"})
    for r in res:
        assert r["runs"], r
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == 0, run


@rccl_loopback
def test_cross_node_directions_over_rccl_beside_ipc_loopback(gpu):
    """4 ranks posing as 2 nodes (node tags a, a, b, b; 1x2x2 grid): the z directions cross
    "nodes" and go over RCCL on every rank, the y directions stay on IPC puts, in one schedule;
    every rank's whole block against the torch model, eager and as hipGraphs"""
    res = _launch("parity", 4, timeout=170,
                  extra_env={"TZ_RCCL_LOOPBACK": "1", "TZ_TEST_TRANSPORT": "auto",
                             "TZ_TEST_NODE_TAGS": "a,a,b,b", "TZ_TEST_ORDERS": "qxyz",
                             "TZ_TEST_SEEDS": "1", "TZ_TEST_FIELD": "hashed"})
    for r in res:
        assert r["runs"], r
        for run in r["runs"]:
            assert run["bad1"] == run["bad2"] == 0, run
            assert run["transport"] == "direct+rccl+ipc", run
            # off-node: every direction with dz != 0 (18 of 26; with 6 neighbours the two z faces)
            assert run["off_node"] == (18 if run["neighbors"] == 26 else 2), run
