"""Rank body for tests/test_gpu_multirank.py: one process per rank, all ranks on GPU 0 (the
loopback setting of the ipc transport). Prints one JSON line with the rank's results."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.parallel import init

    case = sys.argv[1]
    verbose = bool(os.environ.get("TZ_TEST_VERBOSE"))

    import time as _time

    t_start = _time.time()

    def say(*a):
        if verbose:
            print(f"[rank {os.environ.get('RANK', '?')} +{_time.time() - t_start:.1f}s]", *a,
                  file=sys.stderr, flush=True)

    say("start", case)

    ctrl, dev = init(timeout_s=120)
    keep = []  # workloads built by this rank, kept until exit
    say("init done")
    out = {"rank": ctrl.rank, "size": ctrl.size}
    if case == "ipc_halo":
        n = int(os.environ.get("TZ_TEST_N", "48"))
        res = []
        fuses = os.environ.get("TZ_TEST_FUSES", "none,choice").split(",")
        modes = os.environ.get("TZ_TEST_MODES", "eager,graph").split(",")
        for fuse in fuses:
            say("build_halo", n, fuse)
            stencil = bool(os.environ.get("TZ_TEST_STENCIL"))
            relay = os.environ.get("TZ_TEST_RELAY", "auto")
            hostsplit = os.environ.get("TZ_TEST_HOSTSPLIT", "off")
            halo, g = build_halo(HaloConfig(n=n, neighbors=26, order="qxyz",
                                            transport=os.environ.get("TZ_TEST_TRANSPORT", "ipc"),
                                            fuse=fuse, stencil=stencil, relay=relay,
                                            hostsplit=hostsplit,
                                            wide_puts=os.environ.get("TZ_TEST_WIDE", "auto"),
                                            comms=int(os.environ.get("TZ_TEST_COMMS", "0")),
                                            hostsplit_chunks=int(os.environ.get("TZ_TEST_HS_CHUNKS", "1")),
                                            copy_engines=int(os.environ.get("TZ_TEST_COPY_ENGINES", "1"))),
                               ctrl, dev)
            out["relay_ready"] = halo.uses_relay()
            out["transports"] = halo.transport_report()
            out["rccl_nranks"] = halo.rccl_nranks()
            out["grid_memory"] = halo.grid_memory()
            from tenzing_amd.search import choice_alternatives
            out["graph_ops"] = choice_alternatives(g, "he_remote")
            out["hostsplit_ready"] = halo.uses_hostsplit()
            say("built")
            rt = tz.HipRuntime(device=dev, n_streams=3,
                               watchdog_s=float(os.environ.get("TZ_TEST_WATCHDOG", "60")))
            for mode in [tz.ExecMode.Eager if m == "eager" else tz.ExecMode.Graph for m in modes]:
                rt.set_mode(mode)
                rt.set_graph_unroll(int(os.environ.get("TZ_TEST_UNROLL", "3"))
                                    if mode == tz.ExecMode.Graph else 1)
                need = os.environ.get("TZ_TEST_REQUIRE", "")  # an op-name prefix every run uses
                draw = 0
                for seed in range(int(os.environ.get("TZ_TEST_SEEDS", "3"))):
                    msg = ""
                    if ctrl.rank == 0:
                        for _ in range(400):
                            cand = tz.random_rollout(tz.State(g, tz.Platform(3)), draw)
                            draw += 1
                            if not need or any(o.name.startswith(need) for o in cand.ops()):
                                break
                        msg = cand.json(True)
                    seq = tz.OpIndex(g).sequence_from_json(ctrl.bcast(msg, 0).decode())
                    # value generations change from seed to seed and within one: a ghost
                    # filled from a stale buffer or cache line fails the check
                    halo.init_grid(gen=1 + seed % 3)
                    say("init_grid", seed)
                    ctrl.barrier()
                    rt.prepare(seq)
                    say("prepared", seq.desc())
                    rt.run(1)
                    say("ran")
                    rt.device_sync()
                    say("synced")
                    ctrl.barrier()
                    bad1 = halo.check_grid() + (halo.check_stencil() if stencil else 0)
                    say("checked", bad1)
                    ctrl.barrier()
                    rt.run(7)  # repeated exchanges keep the ghosts right
                    rt.device_sync()
                    ctrl.barrier()
                    bad2 = halo.check_grid() + (halo.check_stencil() if stencil else 0)
                    halo.init_grid(gen=1 + (seed + 1) % 3)
                    ctrl.barrier()
                    rt.run(1)
                    rt.device_sync()
                    ctrl.barrier()
                    bad3 = halo.check_grid() + (halo.check_stencil() if stencil else 0)
                    res.append(dict(fuse=fuse, mode=str(mode), seed=seed, bad1=int(bad1),
                                    bad2=int(bad2), bad3=int(bad3), err=halo.ipc_errors(),
                                    transport=halo.transport(), ipc_mode=halo.ipc_mode(),
                                    copyput=any(o.name.startswith("he_copyput_")
                                                for o in seq.ops()),
                                    relay=any(o.name.startswith("he_rl") for o in seq.ops()),
                                    relay_sdma=any(o.name.endswith("_fwdcp") for o in seq.ops()),
                                    hostsplit=any(o.name.startswith("he_hs") for o in seq.ops()),
                                    mixed=any(o.name == "he_copyput_mx" for o in seq.ops()),
                                    wide=any(o.name.startswith("he_putw_") for o in seq.ops())))
            if not os.environ.get("TZ_TEST_NO_MCTS"):
                # a short collective search over ipc schedules
                bench = tz.EmpiricalBenchmarker(rt, ctrl)
                o = tz.MctsOpts()
                o.n_iters = 4
                o.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
                rt.set_mode(tz.ExecMode.Eager)
                r = tz.mcts_explore(g, tz.Platform(3), bench, ctrl, o)
                out.setdefault("mcts", []).append(len(r.sims))
                out.setdefault("mcts_err", []).append(halo.ipc_errors())
                del bench, r
            # release this build on every rank before the next one sets up (see "parity")
            # every workload stays alive until the process ends: RCCL communicators destroyed
            # between two workloads (in use just before, or just after) hung or failed the next
            # workload's first send in RCCL's loopback transport, whichever side of the next
            # setup the teardown fell on
            keep.append((halo, g))
            del rt
        out["runs"] = res
    elif case in ("spmv", "fused"):
        from tenzing_amd.models import SpmvConfig, build_fused, build_spmv

        m = int(os.environ.get("TZ_TEST_M", "30000"))
        sp_transport = os.environ.get("TZ_TEST_SPMV_TRANSPORT", "auto")
        if case == "spmv":
            sp, g = build_spmv(SpmvConfig(m=m, transport=sp_transport), ctrl, dev)
            halo = None
        else:
            halo, sp, g = build_fused(HaloConfig(n=32, neighbors=26, order="qxyz", fuse="choice"),
                                      SpmvConfig(m=m), ctrl, dev)
        out["transport"] = sp.transport()
        out["rccl_capture"] = sp.rccl_capture_note()
        out["rccl_graph_ok"] = sp.rccl_graph_ok()
        rt = tz.HipRuntime(device=dev, n_streams=3, watchdog_s=60.0)
        res = []
        for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
            rt.set_mode(mode)
            rt.set_graph_unroll(3 if mode == tz.ExecMode.Graph else 1)
            for seed in range(4):
                msg = ""
                if ctrl.rank == 0:
                    msg = tz.random_rollout(tz.State(g, tz.Platform(3)), seed).json(True)
                seq = tz.OpIndex(g).sequence_from_json(ctrl.bcast(msg, 0).decode())
                names = [o.name for o in seq.ops()]
                sp.reset_y()
                if halo is not None:
                    halo.init_grid()
                ctrl.barrier()
                rt.prepare(seq)
                rt.run(1)
                rt.device_sync()
                ctrl.barrier()
                err1 = sp.check()
                bad = halo.check_grid() if halo is not None else 0
                ctrl.barrier()
                rt.run(5)  # y = A x is idempotent: repeated iterations keep it right
                rt.device_sync()
                ctrl.barrier()
                res.append(dict(mode=str(mode), seed=seed, err1=err1, err2=sp.check(), bad=int(bad),
                                ipc=any(n.startswith(("i_", "spmv_i_")) for n in names),
                                ipc_err=sp.ipc_errors()))
        bench = tz.EmpiricalBenchmarker(rt, ctrl)
        o = tz.MctsOpts()
        o.n_iters = 6
        o.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
        rt.set_mode(tz.ExecMode.Eager)
        r = tz.mcts_explore(g, tz.Platform(3), bench, ctrl, o)
        out["mcts"] = len(r.sims)
        out["runs"] = res
    elif case == "comm_ops":
        # the user-level RCCL ops between real ranks (TZ_RCCL_LOOPBACK=1): every rank's result
        # depends on its peers' data through each collective and point-to-point op
        import torch
        from tenzing_amd.ops import comm

        K = tz._tz.kernels
        W, R = ctrl.size, ctrl.rank
        n = 1 << 14
        torch.cuda.set_device(dev)
        f64 = dict(dtype=torch.float64, device=f"cuda:{dev}")
        comms = tz._tz.make_rccl_comms(ctrl, dev, 2)
        a, b, c, g, h = (torch.zeros(n, **f64) for _ in range(5))
        e, f = torch.zeros(n * W, **f64), torch.zeros(n * W, **f64)
        nxt, prv = (R + 1) % W, (R - 1) % W
        produce = tz.PyGpuOp("produce", lambda s: K.iota_f64(n, float(R + 1), 1.0, a.data_ptr(), s))
        ar = comm.all_reduce("ar", comms, a, b)                      # b = sum_q a_q
        sr = comm.send_recv("sr", comms, a, nxt, c, prv)             # c = a_{R-1}
        consume = tz.PyGpuOp("consume", lambda s: K.axpy_f64(n, 1.0, b.data_ptr(), c.data_ptr(), s))
        ag = comm.all_gather("ag", comms, c, e)                      # e[q] = c_q
        bc = comm.broadcast("bc", comms, e, 0, f)                    # f = e of rank 0
        rs = comm.reduce_scatter("rs", comms, f, g)                  # g = W * f[R]
        a2a = comm.alltoallv("a2a", comms, [(g, nxt)], [(h, prv)])   # h = g_{R-1}
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
        i = torch.arange(n, **f64)
        bsum = W * (W + 1) / 2 + W * i
        want = W * ((((R - 2) % W) + 1) + i + bsum)
        seqs = tz.get_all_sequences(gr, tz.Platform(2), max_seqs=12)
        index = tz.OpIndex(gr)
        runs = []
        for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
            rt = tz.HipRuntime(device=dev, n_streams=2, mode=mode, graph_unroll=2, watchdog_s=60.0)
            for k in range(len(seqs)):
                seq = index.sequence_from_json(ctrl.bcast(seqs[k].json(True) if R == 0 else "", 0).decode())
                for t in (a, b, c, e, f, g, h):
                    t.zero_()
                torch.cuda.synchronize()
                ctrl.barrier()
                rt.prepare(seq)
                say("schedule", k, str(mode), seq.desc())
                rt.run(3)
                rt.device_sync()
                runs.append(dict(mode=str(mode), k=k, eff=str(rt.effective_mode),
                                 bad=int((h != want).sum())))
                say("schedule", k, "bad", runs[-1]["bad"])
            del rt
        rt = tz.HipRuntime(device=dev, n_streams=2, mode=tz.ExecMode.Graph, watchdog_s=60.0)
        o = tz.MctsOpts()
        o.n_iters = 6
        o.bench = tz.BenchOpts(n_iters=3, max_retries=1, target_secs=0.001)
        res = tz.mcts_explore(gr, tz.Platform(2), tz.EmpiricalBenchmarker(rt, ctrl), ctrl, o)
        out["mcts"] = len(res.sims)
        out["runs"] = runs
        out["nranks"] = comms[0].size if hasattr(comms[0], "size") else None
    elif case == "rccl_overlap":
        # an RCCL send/recv node beside two independent ~200 us kernels, all three on different
        # streams of one hipGraph: with whole-schedule capture the RCCL node must overlap the
        # kernels (one launch ~ one kernel), and the received data must follow every new value
        # generation of the send buffer. Native buffers only: runs without torch (TZ_NO_TORCH=1,
        # the system ROCm runtime) as well as on torch's bundled one
        import time

        import numpy as np

        K = tz._tz.kernels
        W, R = ctrl.size, ctrl.rank
        n = int(os.environ.get("TZ_TEST_N", str(1 << 12)))
        us = float(os.environ.get("TZ_TEST_BUSY_US", "200"))
        comms = tz._tz.make_rccl_comms(ctrl, dev, int(os.environ.get("TZ_TEST_COMMS", "3")))
        a, c = tz._tz.DeviceBuffer(8 * n), tz._tz.DeviceBuffer(8 * n)
        nxt, prv = (R + 1) % W, (R - 1) % W
        sr = tz.SendRecvOp("sr", comms, a.ptr, n, nxt, c.ptr, n, prv, 1, keep=(a, c))
        kernels = [tz.BusyKernelOp("busy_a", us), tz.BusyKernelOp("busy_b", us)]
        kernels = kernels[:int(os.environ.get("TZ_TEST_OVERLAP_KERNELS", "2"))]
        g = tz.Graph()
        for op in kernels + [sr]:
            g.start_then(op)
            g.then_finish(op)
        names = [o.name for o in kernels] + ["sr"]
        msg = ""
        if R == 0:
            for seed in range(400):
                s = tz.random_rollout(tz.State(g, tz.Platform(3)), seed)
                st = {o.name: o.stream for o in s.ops() if o.name in names}
                if len(set(st.values())) == len(names):
                    msg = s.json(True)
                    break
        seq = tz.OpIndex(g).sequence_from_json(ctrl.bcast(msg, 0).decode())
        rt = tz.HipRuntime(device=dev, n_streams=3, mode=tz.ExecMode.Graph, watchdog_s=60.0)
        rt.prepare(seq)
        say("prepared", seq.desc())
        out["effective_mode"] = str(rt.effective_mode)
        out["graph_nodes"] = rt.graph_nodes()
        out["node_types"] = rt.graph_node_types()
        out["kernels"] = len(kernels)
        idx = np.arange(n, dtype=np.float64)
        bad = []
        for gen in (1, 2, 3):
            K.iota_f64(n, 1000.0 * (R + 1) + 7.0 * gen, 1.0, a.ptr, 0)
            c.zero()
            rt.device_sync()
            ctrl.barrier()
            rt.run(1)
            rt.device_sync()
            got = np.frombuffer(c.to_bytes(), dtype=np.float64)
            want = idx + 1000.0 * (prv + 1) + 7.0 * gen
            bad.append(int((got != want).sum()))
            say("gen", gen, "bad", bad[-1])
        out["bad"] = bad
        iters = int(os.environ.get("TZ_TEST_ITERS", "50"))
        rt.run(5)
        rt.device_sync()
        times = []
        for _ in range(3):
            ctrl.barrier()
            t0 = time.perf_counter()
            rt.run(iters)
            rt.device_sync()
            times.append((time.perf_counter() - t0) / iters * 1e6)
        out["iter_us"] = min(times)
        out["iter_us_all"] = times
        out["one_kernel_us"] = us
        # the RCCL op alone, same capture path: what the overlap hides
        g2 = tz.Graph()
        g2.start_then(sr)
        g2.then_finish(sr)
        msg = tz.random_rollout(tz.State(g2, tz.Platform(3)), 0).json(True) if R == 0 else ""
        rt.prepare(tz.OpIndex(g2).sequence_from_json(ctrl.bcast(msg, 0).decode()))
        rt.run(5)
        rt.device_sync()
        ctrl.barrier()
        t0 = time.perf_counter()
        rt.run(iters)
        rt.device_sync()
        out["rccl_alone_us"] = (time.perf_counter() - t0) / iters * 1e6
        out["capture"] = os.environ.get("TZ_GRAPH_CAPTURE", "schedule")
        from tenzing_amd.utils.env import runtime_libraries
        out["runtime"] = runtime_libraries()
        del rt
    elif case == "parity":
        # every transport between real ranks against the independent torch model
        # (tenzing_amd/utils/halo_ref.py): each rank loads its slice of one random global field
        # and checks its whole padded block after the exchange
        from tenzing_amd.utils.halo_ref import ExchangeCheck

        n = int(os.environ.get("TZ_TEST_N", "24"))
        transport = os.environ.get("TZ_TEST_TRANSPORT", "ipc")
        # ranks posing as several nodes: TZ_TEST_NODE_TAGS=a,a,b,b gives rank r the r-th tag
        tags = [t for t in os.environ.get("TZ_TEST_NODE_TAGS", "").split(",") if t]
        node_tag = tags[ctrl.rank] if tags else ""
        res = []
        for order in os.environ.get("TZ_TEST_ORDERS", "qxyz,xyzq").split(","):
            for neighbors in (6, 26):
                halo, g = build_halo(HaloConfig(n=n, neighbors=neighbors, order=order,
                                                nq=int(os.environ.get("TZ_TEST_NQ", "3")),
                                                ghost=int(os.environ.get("TZ_TEST_GHOST", "3")),
                                                transport=transport, fuse="choice",
                                                hostsplit="off", node_tag=node_tag), ctrl, dev)
                rt = tz.HipRuntime(device=dev, n_streams=3, watchdog_s=60.0)
                for mode in (tz.ExecMode.Eager, tz.ExecMode.Graph):
                    rt.set_mode(mode)
                    for seed in range(int(os.environ.get("TZ_TEST_SEEDS", "2"))):
                        msg = ""
                        if ctrl.rank == 0:
                            msg = tz.random_rollout(tz.State(g, tz.Platform(3)), seed).json(True)
                        seq = tz.OpIndex(g).sequence_from_json(ctrl.bcast(msg, 0).decode())
                        chk = ExchangeCheck(halo, seed=17 * seed + neighbors,
                                            field=os.environ.get("TZ_TEST_FIELD", "random"))
                        chk.load()
                        ctrl.barrier()
                        rt.prepare(seq)
                        rt.run(1)
                        rt.device_sync()
                        ctrl.barrier()
                        m1 = chk.mismatches()
                        ctrl.barrier()
                        rt.run(3)
                        rt.device_sync()
                        ctrl.barrier()
                        m2 = chk.mismatches()
                        say(order, neighbors, str(mode), seed, m1, m2)
                        res.append(dict(order=order, neighbors=neighbors, mode=str(mode),
                                        seed=seed, bad1=sum(m1.values()), bad2=sum(m2.values()),
                                        by_class=m1, transport=halo.transport(),
                                        coords=list(halo.coords()),
                                        off_node=len(halo.off_node_dirs()),
                                        schedule_via=sorted({o.name.split("_")[1] for o in seq.ops()
                                                             if o.name.startswith("he_")})))
                        ctrl.barrier()
                # (every workload stays alive until the process ends: see "ipc_halo")
                keep.append((halo, g))
                del rt
        out["runs"] = res
    elif case == "ipc_abort":
        # a candidate that hangs on rank 0 (a spinning kernel ahead of its puts): the watchdogs
        # abort it on every rank, the benchmarker fails it collectively, the recovery hooks reset
        # the IPC counters on every rank, and the next candidate is exact again
        import time

        from tenzing_amd.search import greedy_schedule

        n = int(os.environ.get("TZ_TEST_N", "48"))
        cfg = HaloConfig(n=n, neighbors=26, order="qxyz", transport="ipc", fuse="all",
                         hostsplit="off", relay="off")
        halo, g_ok = build_halo(cfg, ctrl, dev)
        K = tz._tz.kernels

        def hang(stream):
            if ctrl.rank == 0:
                K.busy_wait(1 << 50, 1, stream)

        g_hang = tz.Graph()
        h = tz.PyGpuOp("hang", hang, 1.0)  # added first: executed first, on stream 0
        g_hang.start_then(h)
        g_hang.then_finish(h)
        halo.add_to_graph(g_hang)
        rt = tz.HipRuntime(device=dev, n_streams=2, watchdog_s=4.0)
        bench = tz.EmpiricalBenchmarker(rt, ctrl)
        bo = tz.BenchOpts(n_iters=2, max_retries=1, target_secs=0.001)
        seq_hang = greedy_schedule(g_hang, tz.Platform(2))
        seq_ok = greedy_schedule(g_ok, tz.Platform(2))
        out["hang_first"] = [o.name for o in seq_hang.ops()][1] == "hang"
        t0 = time.time()
        try:
            bench.benchmark(seq_hang, bo)
            out["failed"] = False
        except Exception as e:  # noqa: BLE001
            out["failed"] = True
            say("hang candidate failed:", e)
        out["fail_s"] = time.time() - t0
        out["fired"] = rt.watchdog_fired
        out["recovered"] = tz._tz.recover_after_abort(ctrl)
        r = bench.benchmark(seq_ok, bo)
        out["ok_pct10_ms"] = r.pct10 * 1e3
        halo.init_grid()
        ctrl.barrier()
        rt.prepare(seq_ok)
        rt.run(1)
        rt.device_sync()
        ctrl.barrier()
        out["bad"] = int(halo.check_grid())
        ctrl.barrier()
        rt.run(5)
        rt.device_sync()
        ctrl.barrier()
        out["bad2"] = int(halo.check_grid())
        out["err"] = halo.ipc_errors()
    print("RESULT " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
