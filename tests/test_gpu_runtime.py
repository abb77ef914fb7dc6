"""HIP runtime, workloads and solvers on a real MI355X (1 GPU)."""
import json

import pytest

pytestmark = pytest.mark.gpu


def _small_halo(tz, neighbors=26, fuse="none", order="xyzq", transport="auto", n=24):
    from tenzing_amd.models import HaloConfig, build_halo

    cfg = HaloConfig(n=n, neighbors=neighbors, fuse=fuse, order=order, transport=transport)
    return build_halo(cfg, tz.SelfCtrl(), device=0)


def test_device_and_native_loaded(tz, gpu):
    rt = tz.HipRuntime(device=0, n_streams=2)
    assert "gfx950" in rt.device_name()
    assert tz.native_loaded().endswith(".so")


def test_gpu_graph_decisions_real_streams(tz, gpu):
    """reference test/test_gpu_graph.cu:41-118 with real HIP streams and an empty kernel."""
    g = tz.Graph()
    k1, k2, k3 = (tz.EmptyKernelOp(f"kernel{i}") for i in (1, 2, 3))
    g.start_then(k1)
    g.then(k1, k2)
    g.then(k1, k3)
    g.then_finish(k2)
    g.then_finish(k3)
    plat = tz.Platform(2, symmetric_streams=False)
    s = tz.State(g, plat)
    ds = s.get_decisions()
    assert sorted(d.stream for d in ds if d.kind == "Assign") == [0, 1]
    seqs = tz.get_all_sequences(g, tz.Platform(2))
    rt = tz.HipRuntime(device=0, n_streams=2)
    for seq in seqs:
        rt.prepare(seq)
        rt.run(3)
    rt.device_sync()


@pytest.mark.parametrize("transport", ["copy", "direct"])
@pytest.mark.parametrize("mode", ["eager", "graph"])
@pytest.mark.parametrize("fuse", ["none", "pack", "all", "groups", "choice"])
@pytest.mark.parametrize("neighbors", [6, 26])
def test_halo_exchange_correct(tz, gpu, mode, fuse, neighbors, transport):
    halo, g = _small_halo(tz, neighbors=neighbors, fuse=fuse, transport=transport)
    assert halo.transport() == transport
    m = tz.ExecMode.Graph if mode == "graph" else tz.ExecMode.Eager
    rt = tz.HipRuntime(device=0, n_streams=3, mode=m)
    for seed in range(3):
        final = _rollout_state(tz, g, 3, seed)
        seq, _ = tz.remove_redundant_syncs(final.sequence, final.graph, 3)
        halo.init_grid(gen=seed + 1)  # new values each time: nothing stale passes
        rt.device_sync()
        assert halo.check_grid() > 0  # ghosts not yet filled
        rt.prepare(seq)
        assert rt.effective_mode == m
        rt.run(1)
        rt.device_sync()
        assert halo.check_grid() == 0, seq.desc()


def _rollout_state(tz, g, streams, seed):
    import random

    rng = random.Random(seed)
    s = tz.State(g, tz.Platform(streams))
    while not s.complete():
        s = s.apply(rng.choice(s.get_decisions()))
    return s


def _final_graph(tz, g):
    g2 = g.clone()
    g2.normalize()
    return g2


def test_grid_generations(tz, gpu):
    """value generations (what lets the multi-rank tests catch data left over from an earlier
    exchange): every generation exchanges correctly after the other, the ghosts are reset by
    each init, and only 0..3 exist"""
    halo, g = _small_halo(tz, neighbors=26, order="qxyz")
    rt = tz.HipRuntime(device=0, n_streams=2)
    seq = tz.random_rollout(tz.State(g, tz.Platform(2)), 0)
    rt.prepare(seq)
    for gen in (2, 3, 1, 1, 0):
        halo.init_grid(gen=gen)
        assert halo.check_grid() > 0  # ghosts reset to -1, not yet exchanged
        rt.run(1)
        rt.device_sync()
        assert halo.check_grid() == 0
    with pytest.raises(Exception, match="generation"):
        halo.init_grid(gen=4)


def test_halo_qxyz_order(tz, gpu):
    halo, g = _small_halo(tz, neighbors=26, order="qxyz")
    rt = tz.HipRuntime(device=0, n_streams=2)
    seq = tz.random_rollout(tz.State(g, tz.Platform(2)), 1)
    halo.init_grid()
    rt.prepare(seq)
    rt.run(2)
    rt.device_sync()
    assert halo.check_grid() == 0


@pytest.mark.parametrize("unroll", [1, 3])
def test_graph_mode_iteration_count(tz, gpu, unroll):
    """every iteration of a compiled (and unrolled) graph executes every op exactly once"""
    torch = pytest.importorskip("torch")
    n = 4096
    ones = torch.ones(n, dtype=torch.float64, device="cuda")
    y = torch.zeros(3, n, dtype=torch.float64, device="cuda")  # one counter per op (b, c may overlap)
    K = tz._tz.kernels

    def adder(i):
        return lambda stream: K.axpy_f64(n, 1.0, ones.data_ptr(), y[i].data_ptr(), stream)

    g = tz.Graph()
    a, b, c = tz.PyGpuOp("a", adder(0)), tz.PyGpuOp("b", adder(1)), tz.PyGpuOp("c", adder(2))
    g.start_then(a)
    g.then(a, b)
    g.then(a, c)
    g.then_finish(b)
    g.then_finish(c)
    rt = tz.HipRuntime(device=0, n_streams=2, mode=tz.ExecMode.Graph, graph_unroll=unroll)
    for seed in range(3):
        y.zero_()
        torch.cuda.synchronize()
        seq = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
        rt.prepare(seq)
        assert rt.effective_mode == tz.ExecMode.Graph
        rt.run(7)
        rt.device_sync()
        assert torch.all(y == 7.0), y[:, 0]
        # the unroll's remainder compiled as one graph (precompile): run(n) still executes n
        # iterations, whether n has that remainder or another one
        # (`runs`, not `n`: the ops' closures read `n`, the vector length)
        for runs in (8, 7, 8, 11):
            rt.precompile(8)
            y.zero_()
            torch.cuda.synchronize()
            rt.run(runs)
            rt.device_sync()
            assert torch.all(y == float(runs)), (runs, y[:, 0])


@pytest.mark.parametrize("kind", ["cu_partition", "priorities"])
def test_distinct_streams_halo_correct(tz, gpu, kind):
    """CU-masked (disjoint, XCD-balanced) or prioritized streams as distinct resources: the
    search platform keeps stream bindings apart and every schedule still exchanges correctly"""
    halo, g = _small_halo(tz, neighbors=26, fuse="groups", order="qxyz", n=48)
    kw = {"cu_partition": True} if kind == "cu_partition" else {"priorities": [-1, 0, 0]}
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=3, mode=m, **kw)
        plat = tz.Platform(3, symmetric_streams=False)
        for seed in range(3):
            seq = tz.random_rollout(tz.State(g, plat), seed)
            halo.init_grid()
            rt.prepare(seq)
            assert rt.effective_mode == m
            rt.run(2)
            rt.device_sync()
            assert halo.check_grid() == 0


def test_benchmark_many_graph_slots(tz, gpu):
    """interleaved benchmarking keeps one compiled hipGraph per schedule (switching slots does
    not rebuild), and the runtime returns to single-schedule use afterwards"""
    halo, g = _small_halo(tz, neighbors=26, fuse="choice", order="qxyz", n=64)
    seqs = [tz.random_rollout(tz.State(g, tz.Platform(3)), s) for s in range(4)]
    rt = tz.HipRuntime(device=0, n_streams=3, mode=tz.ExecMode.Graph, graph_unroll=4)
    bench = tz.EmpiricalBenchmarker(rt, tz.SelfCtrl())
    res = bench.benchmark_many(seqs, tz.BenchOpts(n_iters=5, max_retries=1, target_secs=0.001))
    assert len(res) == 4 and all(0 < r.pct10 < 5e-3 for r in res)
    assert rt.effective_mode == tz.ExecMode.Graph
    for seq in seqs:
        halo.init_grid()
        rt.prepare(seq)
        rt.run(3)
        rt.device_sync()
        assert halo.check_grid() == 0


def test_halo_rccl_self_exchange(tz, gpu):
    """RCCL transport on a 1-rank communicator (self send/recv in a group)."""
    halo, g = _small_halo(tz, neighbors=6, transport="rccl")
    assert halo.uses_rccl()
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=2, mode=m, graph_unroll=3)
        for seed in (4, 5):
            seq = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
            halo.init_grid()
            rt.prepare(seq)
            # RCCL send/recv must capture into the schedule's hipGraph (no silent eager fallback)
            assert rt.effective_mode == m
            rt.run(1)
            rt.device_sync()
            assert halo.check_grid() == 0
            rt.run(7)  # unrolled graph launches + remainder
            rt.device_sync()
            assert halo.check_grid() == 0


@pytest.mark.parametrize("form", ["split", "accum", "choice"])
def test_spmv_workload_correct(tz, gpu, form):
    from tenzing_amd.models import SpmvConfig, build_spmv

    sp, g = build_spmv(SpmvConfig(m=20000, form=form), tz.SelfCtrl(), device=0)
    rt = tz.HipRuntime(device=0, n_streams=2)
    seqs = tz.get_all_sequences(g, tz.Platform(2), max_seqs=40)
    assert len(seqs) >= 4
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt.set_mode(m)
        for seq in seqs[:10]:
            sp.reset_y()
            rt.prepare(seq)
            rt.run(1)
            rt.device_sync()
            assert sp.check() < 1e-4


@pytest.mark.parametrize("form", ["split", "accum"])
def test_spmv_every_local_kernel_variant(tz, gpu, form):
    """each alternative of the local-product ChoiceOp (wave64 kernels and the rocSPARSE
    library variant) computes the right y, eagerly and captured into a hipGraph"""
    from tenzing_amd.models import SpmvConfig, build_spmv

    sp, g = build_spmv(SpmvConfig(m=30000, form=form), tz.SelfCtrl(), device=0)
    by_variant = {}
    for seed in range(400):
        seq = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
        names = [o.name for o in seq.ops()]
        v = [n for n in names if n.startswith("yl_")]
        assert len(v) == 1, names
        by_variant.setdefault(v[0], seq)
    assert any("rocsparse" in k for k in by_variant), sorted(by_variant)
    # lane-group kernels, CSR-stream, the ILP kernels (1 / 2 / 4 lanes) and rocSPARSE
    assert {"yl_i1", "yl_i2", "yl_i4", "yl_stream"} <= set(by_variant), sorted(by_variant)
    assert len(by_variant) == 8, sorted(by_variant)
    rt = tz.HipRuntime(device=0, n_streams=2)
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt.set_mode(m)
        for name, seq in sorted(by_variant.items()):
            sp.reset_y()
            rt.prepare(seq)
            assert rt.effective_mode == m, name
            rt.run(2)
            rt.device_sync()
            assert sp.check() < 1e-4, (name, m)


def test_mcts_halo_on_gpu(tz, gpu):
    halo, g = _small_halo(tz, neighbors=6, n=64)
    rt = tz.HipRuntime(device=0, n_streams=2, watchdog_s=60.0)
    ctrl = tz.SelfCtrl()
    bench = tz.EmpiricalBenchmarker(rt, ctrl)
    o = tz.MctsOpts()
    o.n_iters = 8
    o.bench = tz.BenchOpts(n_iters=5, max_retries=1, target_secs=0.001)
    res = tz.mcts_explore(g, tz.Platform(2), bench, ctrl, o)
    assert len(res.sims) == 8
    best = res.sims[res.best()]
    assert 0 < best.res.pct10 < 0.01
    csv = res.dump_csv().splitlines()
    assert json.loads(csv[0])["mcts__Opts"]["nIters"] == 8
    assert len(csv) == 9


def test_dfs_spmv_on_gpu(tz, gpu):
    """BASELINE config 2: CSR SpMV op-graph on 1 MI355X, DFS over 2 HIP streams."""
    from tenzing_amd.models import SpmvConfig, build_spmv

    sp, g = build_spmv(SpmvConfig(m=150_000), tz.SelfCtrl(), device=0)
    rt = tz.HipRuntime(device=0, n_streams=2)
    o = tz.DfsOpts()
    o.max_seqs = 30
    o.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
    res = tz.dfs_explore(g, tz.Platform(2), tz.EmpiricalBenchmarker(rt, tz.SelfCtrl()), tz.SelfCtrl(), o)
    assert len(res.sims) == 30
    assert min(s.res.pct10 for s in res.sims) > 0


def test_pygpuop_torch_on_schedule_stream(tz, gpu):
    torch = pytest.importorskip("torch")
    x = torch.zeros(1 << 20, device="cuda")

    def add_one(stream_ptr):
        s = torch.cuda.ExternalStream(stream_ptr)
        with torch.cuda.stream(s):
            x.add_(1.0)

    g = tz.Graph()
    a = tz.PyGpuOp("a", add_one, 5.0, False)
    b = tz.PyGpuOp("b", add_one, 5.0, False)
    g.start_then(a)
    g.then(a, b)
    g.then_finish(b)
    rt = tz.HipRuntime(device=0, n_streams=2)
    seq = tz.random_rollout(tz.State(g, tz.Platform(2)), 0)
    rt.prepare(seq)
    rt.run(3)
    rt.device_sync()
    assert float(x[0]) == 6.0


def test_native_cli_halo_and_spmv_on_gpu(tz, gpu, tmp_path):
    """tz-search (the native driver, reference tenzing-mcts/examples/halo_*.cu and
    tenzing-dfs/examples/spmv.cu): search, then verify the winning halo schedule on the device"""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tenzing_amd", "bin", "tz-search")
    r = subprocess.run([exe, "--workload", "halo", "--halo-n", "64", "--neighbors", "26", "--order", "qxyz",
                        "--fuse", "choice", "--iters", "6", "--streams", "3", "--bench-iters", "3",
                        "--target-secs", "0.001", "--mode", "graph", "--graph-unroll", "4",
                        "--csv", str(tmp_path / "h.csv")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    summary = json.loads(r.stderr.strip().splitlines()[-1])
    assert summary["candidates"] == 6 and summary["verified_bad_cells"] == 0
    r = subprocess.run([exe, "--workload", "spmv", "--solver", "dfs", "--max-seqs", "12", "--streams", "2",
                        "--bench-iters", "3", "--target-secs", "0.001"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stderr.strip().splitlines()[-1])["candidates"] == 12


def test_example_torch_overlap(gpu):
    """examples/torch_overlap.py: MCTS over torch ops (hipBLASLt GEMM, DMA copy, reductions)
    finds the two-stream overlap"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "examples", "torch_overlap.py"),
                        "--iters", "16"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["candidates"] == 16
    # overlapping the copy chain with the GEMM chain beats running them back to back
    assert j["best_ms"] < 0.9 * j["worst_ms"], j
    bs = j["best_streams"]
    assert bs["gemm"] != bs["h2d"], j


def test_example_grad_allreduce_overlap(gpu):
    """examples/grad_allreduce_overlap.py: backward GEMMs and per-bucket RCCL all-reduces (one
    rank here), searched by MCTS through the communication ops"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "examples", "grad_allreduce_overlap.py"),
                        "--iters", "10", "--layers", "3", "--n", "2048"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["ranks"] == 1 and j["candidates"] == 10 and j["best_ms"] > 0
    assert {"bwd0", "allreduce0"} <= set(j["best_streams"])


def test_cpp_library_example_on_gpu(tz, gpu):
    """the C++ library example on the device: its own HIP kernel op, MCTS over 2 streams, the
    winning schedule's results checked by the program (exit 1 on a wrong element)"""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tenzing_amd", "bin", "tz-example-custom-op")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    # the two chains overlap on two streams
    assert j["best_us"] < 0.8 * j["worst_us"], j


def test_cpp_ring_example_on_gpu(tz, gpu):
    """the C++ multi-rank example (examples/cpp/ring_overlap.hip) on one rank: RCCL send/recv and
    all-reduce ops in a user graph, searched as hipGraph candidates; the program checks the
    winning schedule's results (exit 1 on a wrong element) and the search overlaps the interior
    kernel with the communication chain"""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tenzing_amd", "bin", "tz-example-ring")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["ranks"] == 1 and j["bad"] == 0 and j["candidates"] == 20
    assert j["interior_stream"] != j["xfer_stream"], j
    assert j["best_us"] < j["worst_us"], j


@pytest.mark.parametrize("order", ["qxyz", "xyzq"])
def test_halo_stencil_mode_correct(tz, gpu, order):
    """exchange + 7-point stencil: for random schedules of both alternatives (interior beside
    the exchange, or everything after it), eager and as hipGraphs, the ghosts and every stencil
    output cell are right"""
    from tenzing_amd.models import HaloConfig, build_halo

    halo, g = build_halo(HaloConfig(n=40, neighbors=26, order=order, fuse="choice", stencil=True),
                         tz.SelfCtrl(), device=0)
    kinds = set()
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=3, mode=m, graph_unroll=2)
        for seed in range(6):
            seq = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
            kinds.add("st_full" in [o.name for o in seq.ops()])
            halo.init_grid()
            rt.prepare(seq)
            assert rt.effective_mode == m
            rt.run(3)
            rt.device_sync()
            assert halo.check_grid() == 0
            assert halo.check_stencil() == 0
    assert kinds == {True, False}


def test_spmv_workload_from_matrix_market_file(tz, gpu, tmp_path):
    """a square matrix read from a Matrix Market file (symmetric storage, irregular rows)
    instead of the band matrix: every candidate schedule computes y = A x"""
    from tenzing_amd.models import SpmvConfig, build_spmv
    import random

    rnd = random.Random(5)
    n, lines = 4000, []
    for r in range(1, n + 1):
        for _ in range(rnd.choice([0, 1, 3, 40])):  # empty, short and long rows
            c = rnd.randint(1, r)
            lines.append(f"{r} {c} {rnd.uniform(-1, 1):.6f}")
    f = tmp_path / "sym.mtx"
    f.write_text("%%MatrixMarket matrix coordinate real symmetric\n"
                 f"{n} {n} {len(lines)}\n" + "\n".join(lines) + "\n")
    sp, g = build_spmv(SpmvConfig(matrix=str(f)), tz.SelfCtrl(), device=0)
    assert sp.args.m == n
    rt = tz.HipRuntime(device=0, n_streams=2)
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt.set_mode(m)
        for seed in range(6):
            seq = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
            sp.reset_y()
            rt.prepare(seq)
            rt.run(1)
            rt.device_sync()
            assert sp.check() < 1e-4, seq.desc()


def test_runtime_trace_timeline(tz, gpu):
    """HipRuntime.trace: measured device start/end of every GPU op (timing events around each
    launch), host spans for the syncs; ops on one stream do not overlap, dependent ops start
    after their producers end; the prepared schedule and mode are left as they were"""
    halo, g = _small_halo(tz, neighbors=26, transport="direct")
    rt = tz.HipRuntime(device=0, n_streams=2, mode=tz.ExecMode.Graph, graph_unroll=2)
    seq = tz.random_rollout(tz.State(g, tz.Platform(2)), 3)
    rt.prepare(seq)
    gpu_ops = [o.name for o in seq.ops() if isinstance(o, tz._tz.BoundGpuOp)]
    spans = rt.trace(seq, 3)
    dev = [s for s in spans if s[1] >= 0]
    assert len(dev) == 3 * len(gpu_ops)
    for name, st, it, t0, t1 in dev:
        assert 0 <= t0 <= t1 and name in gpu_ops
    for st in (0, 1):
        on = sorted((t0, t1) for _, s, _, t0, t1 in dev if s == st)
        assert all(a[1] <= b[0] + 1e-3 for a, b in zip(on, on[1:]))
    # iterations follow each other (the schedule ends with host syncs)
    last0 = max(t1 for _, _, it, _, t1 in dev if it == 0)
    first1 = min(t0 for _, _, it, t0, _ in dev if it == 1)
    assert last0 <= first1 + 1e-3
    assert rt.effective_mode == tz.ExecMode.Graph
    halo.init_grid()
    rt.run(1)
    rt.device_sync()
    assert halo.check_grid() == 0
    j = json.loads(tz._tz.chrome_trace(spans))
    assert sum(e["ph"] == "X" for e in j["traceEvents"]) == len(spans)


def test_watchdog_turns_a_hang_into_an_error(tz, gpu):
    """an iteration longer than the watchdog limit: the watchdog aborts the RCCL
    communicators (here: a live one-rank communicator) and the run raises instead of ending the
    process; the runtime stays usable and the benchmarker reports a skippable failure"""
    comm = tz._tz.RcclComm(tz.SelfCtrl(), 0)
    g = tz.Graph()
    slow = tz.BusyKernelOp("slow", 1.5e6)
    g.start_then(slow)
    g.then_finish(slow)
    rt = tz.HipRuntime(device=0, n_streams=1, watchdog_s=0.3)
    seq = tz.random_rollout(tz.State(g, tz.Platform(1)), 0)
    rt.prepare(seq)
    with pytest.raises(Exception, match="watchdog"):
        rt.run(1)
    assert comm.aborted
    with pytest.raises(Exception, match="aborted"):
        comm.sendrecv(0, 0, 0, 0, 0, 0, 1, 0)
    # a failing run inside a benchmark is a CandidateFailed every search skips
    o = tz.DfsOpts()
    o.bench = tz.BenchOpts(n_iters=1, max_retries=1, target_secs=0.001)
    r = tz.dfs_explore(g, tz.Platform(1), tz.EmpiricalBenchmarker(rt, tz.SelfCtrl()), tz.SelfCtrl(), o)
    assert r.failed == 1 and len(r.sims) == 0
    fast = tz.Graph()
    k = tz.BusyKernelOp("fast", 10.0)
    fast.start_then(k)
    fast.then_finish(k)
    rt.prepare(tz.random_rollout(tz.State(fast, tz.Platform(1)), 0))
    rt.run(3)


def test_device_timer_measures_gpu_time(tz, gpu):
    """BenchOpts(device_timer=True): each measurement is the device time between events around
    the batch, so a 200 us kernel measures ~200 us without the host's issue and wake-up cost
    (host wall clock is never below it)"""
    g = tz.Graph()
    k = tz.BusyKernelOp("k", 200.0)
    g.start_then(k)
    g.then_finish(k)
    seq = tz.random_rollout(tz.State(g, tz.Platform(1)), 0)
    res = {}
    for dev in (False, True):
        for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
            rt = tz.HipRuntime(device=0, n_streams=1, mode=mode)
            b = tz.EmpiricalBenchmarker(rt, tz.SelfCtrl())
            r = b.benchmark(seq, tz.BenchOpts(n_iters=5, max_retries=1, target_secs=0.005,
                                              device_timer=dev))
            res[(dev, str(mode))] = r.pct10
    for mode in ("ExecMode.Eager", "ExecMode.Graph"):
        d, h = res[(True, mode)], res[(False, mode)]
        assert 190e-6 < d < 260e-6, res
        assert h >= d * 0.98, res


@pytest.mark.parametrize("workload", ["halo", "fused"])
def test_search_save_best_then_run(tz, gpu, tmp_path, workload):
    """search once, deploy many: the saved schedule is rebuilt by name in a fresh process,
    proven race-free, checked for correct results and timed as a hipGraph"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = tmp_path / "best.json"

    def cli(*args):
        r = subprocess.run([sys.executable, "-m", "tenzing_amd", *args], cwd=root,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    s = cli("search", "--workload", workload, "--halo-n", "64", "--neighbors", "26", "--order",
            "qxyz", "--spmv-m", "20000", "--streams", "3", "--iters", "8", "--bench-iters", "3",
            "--target-secs", "0.001", "--mode", "graph", "--graph-unroll", "4",
            "--save-best", str(path))
    assert path.exists() and s["best_pct10_ms"] > 0
    r = cli("run", str(path), "--iters", "200", "--warmup", "10")
    assert r["correct"] and r["mode"] == "graph" and r["ms_per_iter"] > 0
    assert r["torch_model_check"]["bad_cells"] == 0, r["torch_model_check"]
    if workload == "halo":
        assert r["halo_bad_cells"] == 0
    else:
        assert r["halo_bad_cells"] == 0 and r["spmv_max_rel_err"] < 1e-4
    # the native CLI runs the same document
    exe = os.path.join(root, "tenzing_amd", "bin", "tz-search")
    n = subprocess.run([exe, "--run", str(path), "--run-iters", "200", "--run-warmup", "10"],
                       cwd=root, capture_output=True, text=True, timeout=240)
    assert n.returncode == 0, n.stderr[-3000:]
    rn = json.loads(n.stdout.strip().splitlines()[-1])
    assert rn["correct"] and rn["mode"] == "graph" and rn["halo_bad_cells"] == 0


def test_graph_mode_many_prepares(tz, gpu):
    """regression: a prepare/run loop over many schedules in graph mode (with and without
    unrolling) crashed inside hipGraphLaunch while each source hipGraph was destroyed right after
    instantiation; source graphs now live as long as their execs"""
    halo, g = _small_halo(tz, neighbors=26, fuse="choice", order="qxyz", n=128)
    seqs = [tz.random_rollout(tz.State(g, tz.Platform(4)), s) for s in range(24)]
    for unroll in (1, 6):
        rt = tz.HipRuntime(device=0, n_streams=4, mode=tz.ExecMode.Graph, graph_unroll=unroll)
        for seq in seqs:
            halo.init_grid()
            rt.prepare(seq)
            assert rt.effective_mode == tz.ExecMode.Graph
            rt.run(unroll + 1)
            rt.device_sync()
            assert halo.check_grid() == 0, seq.desc()
        del rt


def test_search_then_run_user_graph(tz, gpu):
    """tz.search on a user graph of busy kernels, then tz.run of the best schedule read back
    from JSON: the two-stream overlap holds in the replay"""
    g = tz.Graph()
    k = [tz.BusyKernelOp(f"k{i}", us) for i, us in enumerate((10, 60, 60, 10), 1)]
    g.start_then(k[0])
    g.then(k[0], k[1])
    g.then(k[0], k[2])
    g.then(k[1], k[3])
    g.then(k[2], k[3])
    g.then_finish(k[3])
    res = tz.search(g, streams=2, solver="dfs", bench_iters=3, target_secs=0.002,
                    ctrl=tz.SelfCtrl(), device=0)
    best = res.sims[res.best()]
    ms = tz.run(g, best.seq.json(True), streams=2, iters=200, ctrl=tz.SelfCtrl(), device=0)
    # k2 and k3 overlap: well under the 140 us of running all four back to back
    assert 0.07 < ms < 0.125, ms
    assert abs(ms - best.res.pct10 * 1e3) < 0.3 * ms


def test_bench_save_best_then_run(tz, gpu, tmp_path):
    """the driver bench's best schedule, saved, runs again through `python -m tenzing_amd run`
    (the same workload rebuilt from the saved options, verified, checked, timed)"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = tmp_path / "bench_best.json"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--cells", "64",
                        "--mcts-iters", "6", "--steps", "5", "--warmup", "2", "--rerank", "1",
                        "--subrecords", "off", "--save-best", str(path)], cwd=root, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    tm = json.loads(r.stdout.strip().splitlines()[-1])["torch_model_check"]
    assert tm.get("bad_cells") == 0 and tm["field"] == "hashed", tm
    doc = json.loads(path.read_text())
    assert doc["ranks"] == 1 and doc["args"]["halo_n"] == 64 and doc["args"]["neighbors"] == 26
    r = subprocess.run([sys.executable, "-m", "tenzing_amd", "run", str(path), "--iters", "50",
                        "--warmup", "5"], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["correct"] and j["halo_bad_cells"] == 0 and j["ms_per_iter"] > 0
    assert j["torch_model_check"]["bad_cells"] == 0, j["torch_model_check"]


@pytest.mark.parametrize("alt", ["hs_onelaunch_i4", "hs_onelaunch_i2", "hs_separate"])
def test_config5_one_launch_schedule_is_exact(tz, gpu, alt):
    """BASELINE config 5 on one GPU: each hs_launches alternative, eager and compiled to a
    hipGraph, leaves every ghost cell exact and y = A x (the workloads' own checks), from two grid
    generations"""
    from tenzing_amd.models import HaloConfig, SpmvConfig, build_fused
    from tenzing_amd.search import greedy_schedule

    h, s, g = build_fused(HaloConfig(n=48, neighbors=26, order="qxyz", fuse="choice"),
                          SpmvConfig(m=20_000), tz.SelfCtrl(), 0)
    seq = greedy_schedule(g, tz.Platform(4), {"hs_launches": alt, "*": ["allfused", "accum"]},
                          stream_for=lambda n: 1 if n.startswith("he_") else 0)
    names = [o.name for o in seq.ops() if isinstance(o, tz._tz.BoundGpuOp)]
    assert (names == [alt]) == alt.startswith("hs_onelaunch"), names
    for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=4, mode=mode, graph_unroll=3)
        for gen in (1, 2):
            h.init_grid(gen=gen)
            s.reset_y()
            rt.device_sync()
            rt.prepare(seq)
            rt.run(1)
            rt.device_sync()
            assert h.check_grid() == 0, (alt, mode, gen)
            assert s.check() < 1e-4, (alt, mode, gen)
        del rt


@pytest.mark.parametrize("mode", ["eager", "graph"])
@pytest.mark.parametrize("ghost_align", [-1, -2])
@pytest.mark.parametrize("transport", ["copy", "direct"])
@pytest.mark.parametrize("neighbors", [6, 26])
@pytest.mark.parametrize("order", ["xyzq", "qxyz"])
@pytest.mark.parametrize("n,field", [(20, "random"), (24, "hashed")])
def test_exchange_matches_independent_torch_model(tz, gpu, n, field, order, neighbors, transport,
                                                  ghost_align, mode):
    """the exchange against a model that shares no code with it (tenzing_amd/utils/halo_ref.py):
    a random field, torch's circular padding, the grid read back through the reported strides.
    Every ghost cell the exchange fills must equal the model, every other cell must be untouched,
    over random schedules of the search's choice graph and repeated exchanges. n = 24 puts the
    high x ghost run of the row-start layout on a 64-B boundary, n = 20 does not; n = 24 also
    uses the hashed field (each rank's block computed on its own)."""
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.utils.halo_ref import ExchangeCheck

    cfg = HaloConfig(n=n, neighbors=neighbors, order=order, transport=transport, fuse="choice",
                     ghost_align=ghost_align)
    halo, g = build_halo(cfg, tz.SelfCtrl(), device=0)
    rt = tz.HipRuntime(device=0, n_streams=3,
                       mode=tz.ExecMode.Graph if mode == "graph" else tz.ExecMode.Eager)
    for seed in range(2):
        seq = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
        chk = ExchangeCheck(halo, seed=seed, field=field)
        chk.load()
        before = chk.mismatches()
        assert before[0] == 0 and before[1] > 0  # interior loaded, ghosts not yet filled
        rt.prepare(seq)
        rt.run(1)
        rt.device_sync()
        assert chk.mismatches() == {0: 0, 1: 0, 2: 0, 3: 0}, seq.desc()
        rt.run(3)
        rt.device_sync()
        assert chk.mismatches() == {0: 0, 1: 0, 2: 0, 3: 0}, seq.desc()


def test_headline_exchange_matches_independent_torch_model(tz, gpu):
    """the headline's shape (512^3 x 3q, ghost 3, 26 neighbours, QXYZ, line-aligned ghosts) and
    the bench's flow (MCTS over the choice graph on 4 streams, then the chosen schedule as a
    hipGraph), checked against the torch model on the device"""
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.utils.halo_ref import ExchangeCheck

    halo, g = build_halo(HaloConfig(n=512, neighbors=26, order="qxyz", fuse="choice",
                                    transport="direct"), tz.SelfCtrl(), device=0)
    rt = tz.HipRuntime(device=0, n_streams=4, mode=tz.ExecMode.Graph)
    o = tz.MctsOpts()
    o.n_iters = 8
    o.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
    ctrl = tz.SelfCtrl()
    res = tz.mcts_explore(g, tz.Platform(4), tz.EmpiricalBenchmarker(rt, ctrl), ctrl, o)
    best = res.sims[res.best()].seq
    chk = ExchangeCheck(halo, seed=7, device="cuda:0", field="hashed")
    chk.load()
    rt.prepare(best)
    rt.run(2)
    rt.device_sync()
    assert chk.mismatches() == {0: 0, 1: 0, 2: 0, 3: 0}, best.desc()


@pytest.mark.parametrize("shape", [(17, 1, 1), (16, 5, 2), (13, 2, 4), (9, 3, 3), (30, 4, 5)])
@pytest.mark.parametrize("ghost_align", [-1, -2])
@pytest.mark.parametrize("transport", ["copy", "direct"])
@pytest.mark.parametrize("order", ["xyzq", "qxyz"])
def test_odd_shapes_match_independent_torch_model(tz, gpu, shape, ghost_align, transport, order):
    """interior sizes, quantity counts and ghost widths away from the headline's (odd n, one
    quantity, ghost 1 to 5) against the torch model, 26 neighbours, eager and as hipGraphs"""
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.utils.halo_ref import ExchangeCheck

    n, nq, ghost = shape
    cfg = HaloConfig(n=n, nq=nq, ghost=ghost, neighbors=26, order=order, transport=transport,
                     fuse="choice", ghost_align=ghost_align)
    halo, g = build_halo(cfg, tz.SelfCtrl(), device=0)
    for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=3, mode=mode)
        seq = tz.random_rollout(tz.State(g, tz.Platform(3)), n + nq + ghost)
        chk = ExchangeCheck(halo, seed=n * 7 + ghost, field="hashed")
        chk.load()
        rt.prepare(seq)
        rt.run(2)
        rt.device_sync()
        assert chk.mismatches() == {0: 0, 1: 0, 2: 0, 3: 0}, (shape, str(mode), seq.desc())
