"""Multi-rank bootstrap without torch: the native TCP control plane's own rendezvous
(``TcpCtrl.rendezvous`` on MASTER_PORT + 1, handshake-checked), as bench.py uses it at N > 1.
Reference: MPI_Init + MPI_COMM_WORLD (tenzing-mcts/examples/halo_min_time.cu:11)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

BODY = r"""
import json, os, sys
sys.path.insert(0, os.environ["TZ_ROOT"])
from tenzing_amd.parallel import init_ctrl
from tenzing_amd.utils.env import runtime_libraries
c = init_ctrl(timeout_s=60)
c.barrier()
got = c.bcast("hello" if c.rank == 0 else "", 0).decode()
mx = c.allreduce_max([float(c.rank)])[0]
ag = [x.decode() for x in c.allgather(f"r{c.rank}")]
libs = runtime_libraries()
print("RESULT " + json.dumps(dict(rank=c.rank, size=c.size, got=got, mx=mx, ag=ag,
                                  torch="torch" in sys.modules, libs=libs)), flush=True)
"""


def _free_port():
    """a MASTER_PORT whose control port (MASTER_PORT + 1) is free as well"""
    for _ in range(100):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p >= 65535:
            continue
        t = socket.socket()
        try:
            t.bind(("0.0.0.0", p + 1))
        except OSError:
            continue
        finally:
            t.close()
        return p
    raise RuntimeError("no free port pair")


def _launch(world, port, extra=None, timeout=120):
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TZ_NO_TORCH="1",
                   TZ_ROOT=ROOT, **(extra or {}))
        env.pop("TZ_CTRL_BOOTSTRAP", None)
        procs.append(subprocess.Popen([sys.executable, "-c", BODY], env=env, text=True,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return procs, outs


def _results(procs, outs):
    res = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
        line = [x for x in o.splitlines() if x.startswith("RESULT ")][-1]
        res.append(json.loads(line[len("RESULT "):]))
    return res


def test_two_ranks_without_torch():
    """two ranks rendezvous on MASTER_PORT + 1 with torch never imported; every collective
    works, and each rank reports the HIP runtime / RCCL it actually mapped"""
    res = _results(*_launch(2, _free_port()))
    for r in res:
        assert r["size"] == 2 and r["got"] == "hello" and r["mx"] == 1.0 and r["ag"] == ["r0", "r1"]
        assert r["torch"] is False
        # without torch the system ROCm's runtime is the one mapped
        assert r["libs"]["hip_runtime"]["path"].startswith("/opt/rocm")
        assert r["libs"]["rccl_library"]["path"].startswith("/opt/rocm")
        assert r["libs"]["torch_loaded"] is False


def test_four_ranks_explicit_ctrl_port():
    port = _free_port()
    res = _results(*_launch(4, 29000, extra={"TZ_CTRL_PORT": str(port)}))
    assert sorted(r["rank"] for r in res) == [0, 1, 2, 3]
    assert all(r["ag"] == ["r0", "r1", "r2", "r3"] for r in res)


def test_stray_connection_is_dropped():
    """a connection to the control port that does not speak the handshake is dropped, and the
    job's ranks still join"""
    import threading

    port = _free_port()

    def stray():
        t0 = time.time()
        while time.time() - t0 < 30:
            try:
                s = socket.create_connection(("127.0.0.1", port + 1), timeout=1)
                s.sendall(b"GET / HTTP/1.0\r\n\r\n")
                time.sleep(0.2)
                s.close()
                return
            except OSError:
                time.sleep(0.05)

    th = threading.Thread(target=stray)
    th.start()
    res = _results(*_launch(2, port))
    th.join()
    assert [r["got"] for r in res] == ["hello", "hello"]


def test_world_size_mismatch_fails_loudly():
    """a rank of a differently sized job is refused with a clear error, not taken for a rank"""
    port = _free_port()
    env = dict(os.environ, TZ_NO_TORCH="1", TZ_ROOT=ROOT, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    p0 = subprocess.Popen([sys.executable, "-c", BODY], env=dict(env, RANK="0", WORLD_SIZE="2"),
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    p1 = subprocess.Popen([sys.executable, "-c", BODY], env=dict(env, RANK="1", WORLD_SIZE="3"),
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        _, e0 = p0.communicate(timeout=90)
        p1.communicate(timeout=90)
    finally:
        for p in (p0, p1):
            if p.poll() is None:
                p.kill()
    assert p0.returncode != 0 and "of 3" in e0, e0[-2000:]


def test_peer_device_facts_fake_two_device_topology():
    """the device-pair record on a fake 2-GPU node (rank 0 on bus A / device 0, rank 1 on bus B /
    device 1) and on a fake loopback pair (both ranks on bus A)"""
    from tenzing_amd.parallel.topology import peer_device_facts

    class FakeCtrl:
        def __init__(self, rank, buses):
            self.rank, self.buses = rank, buses

        def allgather(self, mine):
            assert mine == self.buses[self.rank]
            return [b.encode() for b in self.buses]

    devs = {"0000:0a:00.0": 0, "0000:1b:00.0": 1}
    f = peer_device_facts(FakeCtrl(0, ["0000:0a:00.0", "0000:1b:00.0"]), 0, [1, 1, 0],
                          bus_of=lambda d: "0000:0a:00.0", device_by_bus=lambda b: devs.get(b, -1),
                          can_access=lambda a, b: (a, b) == (0, 1), ipc_mapped={1: 1})
    p = f["peers"]["1"]
    assert list(f["peers"]) == ["1"]  # self and duplicates dropped
    assert p["same_device"] is False and p["visible_as"] == 1 and p["can_access_peer"] is True
    assert p["ipc_mapped_on_device"] == 1 and p["ipc_mapping_consistent"] is True
    assert f["summary"] == "1 of 1 peer(s) on other devices, 1 with peer access"
    # a mapping that claims this rank's own device for a peer on another GPU is flagged
    g = peer_device_facts(FakeCtrl(0, ["0000:0a:00.0", "0000:1b:00.0"]), 0, [1],
                          bus_of=lambda d: "0000:0a:00.0", device_by_bus=lambda b: devs.get(b, -1),
                          can_access=lambda a, b: True, ipc_mapped={1: 0})
    assert g["peers"]["1"]["ipc_mapping_consistent"] is False and "unexpected" in g["summary"]
    # the peer's GPU hidden from this process (device isolation): no access claim either way
    h = peer_device_facts(FakeCtrl(0, ["0000:0a:00.0", "0000:1b:00.0"]), 0, [1],
                          bus_of=lambda d: "0000:0a:00.0", device_by_bus=lambda b: -1,
                          can_access=lambda a, b: True)
    assert h["peers"]["1"]["can_access_peer"] is None and "not visible" in h["peers"]["1"]["reason"]
    # loopback: both ranks on one device
    lo = peer_device_facts(FakeCtrl(1, ["0000:0a:00.0", "0000:0a:00.0"]), 0, [0],
                           bus_of=lambda d: "0000:0a:00.0", device_by_bus=lambda b: 0,
                           can_access=lambda a, b: False, ipc_mapped={0: 0})
    q = lo["peers"]["0"]
    assert q["same_device"] is True and q["can_access_peer"] is None
    assert q["ipc_mapping_consistent"] is True
    assert lo["summary"] == "all 1 peer(s) on this rank's own device (loopback)"


def test_silent_peer_times_out_with_a_message():
    """a rank that stops talking (hung outside every watchdog) ends its peers' collectives with
    a clear error after TZ_CTRL_TIMEOUT_S, instead of blocking them forever"""
    port = _free_port()
    body = r"""
import os, sys, time
sys.path.insert(0, os.environ["TZ_ROOT"])
from tenzing_amd.parallel import init_ctrl
c = init_ctrl(timeout_s=60)
if c.rank == 1:
    time.sleep(8)
    sys.exit(0)
t0 = time.time()
try:
    c.barrier()
    print("NO-TIMEOUT")
except Exception as e:
    print("TIMEOUT %.1f %s" % (time.time() - t0, e))
"""
    env = dict(os.environ, TZ_NO_TORCH="1", TZ_ROOT=ROOT, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), WORLD_SIZE="2", TZ_CTRL_TIMEOUT_S="1.5")
    ps = [subprocess.Popen([sys.executable, "-c", body], env=dict(env, RANK=str(r)),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (0, 1)]
    try:
        out0 = ps[0].communicate(timeout=60)[0]
        ps[1].communicate(timeout=60)
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    line = [x for x in out0.splitlines() if x.startswith(("TIMEOUT", "NO-TIMEOUT"))][-1]
    assert line.startswith("TIMEOUT"), out0
    assert float(line.split()[1]) < 6.0 and "hung or gone" in line


def _hold_port(port):
    """a foreign program on `port`: accepts connections and never answers"""
    import threading

    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("0.0.0.0", port))
    srv.listen(8)
    held, stop = [], threading.Event()

    def accept_and_hold():
        srv.settimeout(0.2)
        while not stop.is_set():
            try:
                held.append(srv.accept()[0])
            except OSError:
                pass

    th = threading.Thread(target=accept_and_hold)
    th.start()

    def release():
        stop.set()
        th.join()
        for c in held:
            c.close()
        srv.close()
    return release


def _run_pair(port, body, extra=None):
    env = dict(os.environ, TZ_NO_TORCH="1", TZ_ROOT=ROOT, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), WORLD_SIZE="2", **(extra or {}))
    ps = [subprocess.Popen([sys.executable, "-c", body], env=dict(env, RANK=str(r)),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (0, 1)]
    try:
        outs = [p.communicate(timeout=90) for p in ps]
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    return ps, outs


def test_foreign_listener_on_the_control_port_is_skipped():
    """another program holds the control port (it accepts connections and never answers): rank 0
    takes the next candidate port, and rank 1 leaves the foreign listener (no acknowledgement)
    and finds rank 0 there (round 3's unexplained loopback hang had this shape: a port picked as
    free, then taken)"""
    port = _free_port()
    release = _hold_port(port + 1)
    try:
        ps, outs = _run_pair(port, BODY)
    finally:
        release()
    res = _results(ps, outs)
    assert [r["got"] for r in res] == ["hello", "hello"]


def test_foreign_listener_with_one_candidate_port_fails_fast():
    """with a single candidate port (TZ_CTRL_PORTS=1) held by another program: rank 0 cannot bind
    and says so, and rank 1 does not wait on that listener forever: it gives up within its
    rendezvous timeout, naming the cause"""
    port = _free_port()
    release = _hold_port(port + 1)
    body = BODY.replace("init_ctrl(timeout_s=60)", "init_ctrl(timeout_s=8)")
    t0 = time.time()
    try:
        ps, outs = _run_pair(port, body, {"TZ_CTRL_PORTS": "1"})
    finally:
        release()
    errs = [e for _, e in outs]
    assert time.time() - t0 < 60
    assert ps[0].returncode != 0 and "could be bound" in errs[0], errs[0][-1500:]
    assert ps[1].returncode != 0 and "not this job's rank 0" in errs[1], errs[1][-1500:]


def test_graph_capture_info_defaults():
    """the record of how schedules become hipGraphs (bench.py's `graph_capture`): whole-schedule
    capture, 6 streams owned at least; env settings (applied at import) are reported as forced"""
    code = ("import sys, json; sys.path.insert(0, %r); import tenzing_amd as tz; "
            "print(json.dumps(tz._tz.graph_capture_info()))" % ROOT)
    env = {k: v for k, v in os.environ.items()
           if k not in ("TZ_GRAPH_CAPTURE", "TZ_PAD_STREAMS")}
    env["TZ_NO_TORCH"] = "1"
    j = json.loads(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                                  text=True, timeout=120).stdout.strip().splitlines()[-1])
    assert j == {"mode": "schedule", "forced": False, "rccl_mode": "schedule", "pad_streams": 6}, j
    env.update(TZ_GRAPH_CAPTURE="child", TZ_PAD_STREAMS="0")
    j = json.loads(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                                  text=True, timeout=120).stdout.strip().splitlines()[-1])
    assert j["mode"] == "child" and j["forced"] and j["rccl_mode"] == "child" and j["pad_streams"] == 0


def test_link_matrix_summary_finds_the_slow_pair():
    """the record's link-matrix summary on a fake 8-GPU node: 56 ordered pairs, one of them
    (3 -> 5) at half speed, as a pair routed over two hops would be"""
    import importlib.util

    # the module alone (no package import: this file's tests stay torch-free)
    spec = importlib.util.spec_from_file_location(
        "tz_topology", os.path.join(ROOT, "tenzing_amd", "parallel", "topology.py"))
    topo = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(topo)
    matrix_summary = topo.matrix_summary

    m = [[-1.0 if r == q else 70.0 for q in range(8)] for r in range(8)]
    m[3][5] = 35.0
    s = matrix_summary(m)
    assert s["pairs"] == 56 and s["min"] == 35.0 and s["max"] == 70.0 and s["median"] == 70.0
    assert s["slowest_pair"] == [3, 5] and s["spread"] == 2.0
    assert matrix_summary([[-1.0]]) is None


def test_timeout_is_raised_for_long_runs():
    """a run whose watchdog budget is longer than the control plane's receive timeout raises it
    (the benchmarker calls ensure_timeout before every run): a peer that is slow but within that
    budget is waited for, not declared gone"""
    port = _free_port()
    body = r"""
import os, sys, time
sys.path.insert(0, os.environ["TZ_ROOT"])
from tenzing_amd.parallel import init_ctrl
c = init_ctrl(timeout_s=60)
c.ensure_timeout(1.0)   # never lowers
assert abs(c.timeout - 1.5) < 1e-9, c.timeout
c.ensure_timeout(8.0)
if c.rank == 1:
    time.sleep(3)
t0 = time.time()
c.barrier()
print("OK %.1f %.1f" % (time.time() - t0, c.timeout))
"""
    env = dict(os.environ, TZ_NO_TORCH="1", TZ_ROOT=ROOT, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), WORLD_SIZE="2", TZ_CTRL_TIMEOUT_S="1.5")
    ps = [subprocess.Popen([sys.executable, "-c", body], env=dict(env, RANK=str(r)),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (0, 1)]
    try:
        outs = [p.communicate(timeout=60) for p in ps]
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in ps), outs
    line = [x for x in outs[0][0].splitlines() if x.startswith("OK")][-1]
    assert float(line.split()[1]) > 2.0 and float(line.split()[2]) == 8.0, line


def test_rank_that_reconnects_replaces_its_closed_connection():
    """a peer that gave up waiting for its acknowledgement and came back with the same rank is
    taken again (its first connection, now closed, is replaced) instead of failing the whole
    rendezvous as a duplicate rank (3 ranks: rank 0 is still waiting for rank 2 when rank 1
    comes back)"""
    import struct
    import time

    port = _free_port()
    body = r"""
import os, sys
sys.path.insert(0, os.environ["TZ_ROOT"])
import tenzing_amd as tz
c = tz._tz.TcpCtrl(int(os.environ["RANK"]), 3)
c.rendezvous("127.0.0.1", int(os.environ["MASTER_PORT"]), 30.0, 1)
print("JOINED", c.allreduce_max([float(c.rank)])[0])
"""
    env = dict(os.environ, TZ_NO_TORCH="1", TZ_ROOT=ROOT, MASTER_PORT=str(port))
    ps = [subprocess.Popen([sys.executable, "-c", body], env=dict(env, RANK="0"),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)]
    try:
        # the first, abandoned connection of rank 1: handshake, acknowledged, then closed
        deadline = time.time() + 30
        while True:
            try:
                s = socket.create_connection(("127.0.0.1", port), timeout=5)
                break
            except OSError:
                if time.time() > deadline:
                    raise
                time.sleep(0.1)
        s.sendall(struct.pack("<Iiii", 0x545A4331, 3, 1, port))
        assert struct.unpack("<I", s.recv(4))[0] == 0x545A4143
        s.close()
        for r in (1, 2):
            ps.append(subprocess.Popen([sys.executable, "-c", body], env=dict(env, RANK=str(r)),
                                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs = [p.communicate(timeout=60) for p in ps]
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in ps), outs
    assert all("JOINED 2.0" in o[0] for o in outs), outs


def test_runtime_options_flip_both_ways_in_one_process(tz):
    """the kept tuning options are runtime options, not environment
    variables cached in statics: each is set both ways and read back inside one process
    (capture mode, default stream padding, the box kernels' peel / widened unpack / cache
    policies / block order / put cap, and the halo's IPC mode, copy-engine puts, copy engines and
    row-pair moves as HaloArgs fields)"""
    k = tz._tz.kernels
    info = tz._tz.graph_capture_info
    try:
        for mode, forced in (("child", True), ("schedule", True), ("auto", False)):
            tz._tz.set_graph_capture(mode)
            i = info()
            assert i["forced"] is forced and i["mode"] == ("child" if mode == "child" else "schedule")
        for n in (0, 9, 6):
            tz._tz.set_default_pad_streams(n)
            assert info()["pad_streams"] == n
        with pytest.raises(Exception):
            tz._tz.set_graph_capture("bogus")
    finally:
        tz._tz.set_graph_capture("auto")
        tz._tz.set_default_pad_streams(6)
    pairs = ((k.set_peel_moves, k.get_peel_moves), (k.set_widen_unpack, k.get_widen_unpack),
             (k.set_nt_move_store, k.get_nt_move_store))
    for setter, getter in pairs:
        prev = getter()
        for v in (not prev, prev):
            setter(v)
            assert getter() == v
    for setter, getter, vals in ((k.set_xcd_remap, k.get_xcd_remap, (2, 1, 0)),
                                 (k.set_put_max_blocks, k.get_put_max_blocks, (16, 64)),
                                 (k.set_move_unroll, k.get_move_unroll, (2, 1))):
        for v in vals:
            setter(v)
            assert getter() == v
    prev = k.get_box_tuning()
    k.set_box_tuning(prev[0], not prev[1], not prev[2], prev[3], not prev[4])
    assert k.get_box_tuning()[1:3] == (not prev[1], not prev[2])
    k.set_box_tuning(*prev)
    assert k.get_box_tuning() == prev
    # halo options: fields of the arguments, so one process builds both sides
    from tenzing_amd.models import HaloConfig

    for grid in (0, 1):
        for copy in (True, False):
            h = tz._tz.HaloExchange(HaloConfig(n=16, ipc_grid=grid, copy_puts=copy, copy_engines=2,
                                               transport="ipc").args(0, 2, -1))
            assert h.ipc_mode() == ("grid" if grid else "buffers")
            assert h.args.copy_engines == 2 and h.args.copy_puts is copy
    for pairs_on in (True, False):
        a = HaloConfig(n=16, order="xyzq", move_pairs=pairs_on).args(0, 1, -1)
        assert a.move_pairs is pairs_on and '"move_pairs":%s' % str(pairs_on).lower() in a.json().replace(" ", "")
    for mem in (-1, 0, 1):
        a = HaloConfig(n=16, grid_memory=mem).args(0, 1, -1)
        assert a.grid_memory == mem and '"grid_memory":%d' % mem in a.json().replace(" ", "")
    with pytest.raises(Exception, match="grid_memory"):
        tz._tz.HaloExchange(HaloConfig(n=16, grid_memory=2).args(0, 1, -1)).setup(None)
