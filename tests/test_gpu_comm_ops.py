"""RCCL communication ops in user graphs (the reference's Isend/Irecv/Ialltoallv/Wait ops,
include/tenzing/mpi/ops_mpi.hpp:17-192), on a 1-rank communicator set: every op runs its real
RCCL path (self send/recv, 1-rank collectives), eagerly and captured into hipGraphs, under every
enumerated schedule. Multi-rank matching is covered by the halo/SpMV RCCL transports, which use
the same communicator-per-stream rule."""
import pytest

pytestmark = pytest.mark.gpu


def _pipeline(tz, comms, n):
    torch = pytest.importorskip("torch")
    from tenzing_amd.ops import comm

    K = tz._tz.kernels
    f64 = dict(dtype=torch.float64, device="cuda")
    a, b, c, e, f, g, h = (torch.zeros(n, **f64) for _ in range(7))

    produce = tz.PyGpuOp("produce", lambda s: K.iota_f64(n, 1.0, 1.0, a.data_ptr(), s))
    ar = comm.all_reduce("ar", comms, a, b)                      # b = a
    sr = comm.send_recv("sr", comms, a, 0, c, 0)                 # c = a
    consume = tz.PyGpuOp("consume", lambda s: K.axpy_f64(n, 1.0, b.data_ptr(), c.data_ptr(), s))
    ag = comm.all_gather("ag", comms, c, e)                      # e = c = 2a
    bc = comm.broadcast("bc", comms, e, 0, f)                    # f = e
    rs = comm.reduce_scatter("rs", comms, f, g, op="max")        # g = f
    a2a = comm.alltoallv("a2a", comms, [(g, 0)], [(h, 0)])       # h = g

    gr = tz.Graph()
    gr.start_then(produce)
    for x in (ar, sr):
        gr.then(produce, x)
        gr.then(x, consume)
    gr.then(consume, ag)
    gr.then(ag, bc)
    gr.then(bc, rs)
    gr.then(rs, a2a)
    gr.then_finish(a2a)
    want = 2.0 * (1.0 + torch.arange(n, **f64))
    return gr, (a, b, c, e, f, g, h), want


def test_comm_ops_every_schedule(tz, gpu):
    torch = pytest.importorskip("torch")
    comms = tz._tz.make_rccl_comms(tz.SelfCtrl(), 0, 2)
    n = 1 << 16
    gr, bufs, want = _pipeline(tz, comms, n)
    seqs = tz.get_all_sequences(gr, tz.Platform(2), max_seqs=24)
    assert len(seqs) >= 4
    kinds = {op.kind for op in seqs[0].ops()}
    assert {"RcclAllReduce", "RcclSendRecv", "RcclAllGather", "RcclBroadcast",
            "RcclReduceScatter", "RcclAlltoallv"} <= kinds
    for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=2, mode=mode, graph_unroll=2)
        for seq in seqs:
            for t in bufs:
                t.zero_()
            torch.cuda.synchronize()
            rt.prepare(seq)
            assert rt.effective_mode == mode  # RCCL ops capture: no silent eager fallback
            rt.run(3)
            rt.device_sync()
            assert torch.equal(bufs[-1], want), seq.desc()


def test_comm_ops_search_and_json(tz, gpu):
    """an MCTS search over a graph of comm ops benchmarks collectively; schedules round-trip
    through the reference's JSON format (ops found by name)"""
    comms = tz._tz.make_rccl_comms(tz.SelfCtrl(), 0, 2)
    gr, bufs, want = _pipeline(tz, comms, 1 << 12)
    rt = tz.HipRuntime(device=0, n_streams=2, mode=tz.ExecMode.Graph)
    opts = tz.MctsOpts()
    opts.n_iters = 8
    opts.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
    res = tz.mcts_explore(gr, tz.Platform(2), tz.EmpiricalBenchmarker(rt, tz.SelfCtrl()),
                          tz.SelfCtrl(), opts)
    best = res.sims[res.best()]
    assert best.res.pct10 > 0
    text = best.seq.json(True)
    assert '"kind": "RcclSendRecv"' in text or '"kind":"RcclSendRecv"' in text
    back = tz.OpIndex(gr).sequence_from_json(text)
    assert back.canonical_key() == best.seq.canonical_key()


def test_comm_ops_host_checks(tz, gpu):
    torch = pytest.importorskip("torch")
    from tenzing_amd.ops import comm

    comms = tz._tz.make_rccl_comms(tz.SelfCtrl(), 0, 1)
    x = torch.zeros(8, dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError):
        comm.all_gather("ag", comms, x, torch.zeros(4, dtype=torch.float32, device="cuda"))
    with pytest.raises(TypeError):
        comm.all_reduce("ar", comms, x, torch.zeros(8, dtype=torch.float64, device="cuda"))
    with pytest.raises(tz.TzError):
        comm.send_recv("sr", comms, x, 3, x, 0)  # peer outside the 1-rank communicator
    with pytest.raises(ValueError):
        comm.all_reduce("ar", comms, x, op="avg")
