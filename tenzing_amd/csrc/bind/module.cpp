// Python bindings (pybind11) for the native core, HIP runtime, RCCL transport and workloads.
// The reference listed Python bindings as a roadmap item (README.md:56-58); here they are the
// primary scripting surface, while the search engine itself stays native.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "core/benchmark.hpp"
#include "core/health.hpp"
#include "core/solve.hpp"
#include "hip/comm_ops.hpp"
#include "hip/hip_runtime.hpp"
#include "hip/rccl_comm.hpp"
#include "hip/rocsparse_spmv.hpp"
#include "kernels/kernels.hpp"
#include "workloads/workloads.hpp"

#include <hip/hip_runtime_api.h>

#include <csignal>
#include <cstdlib>
#include <execinfo.h>
#include <sstream>
#include <unistd.h>
#include <vector>

namespace py = pybind11;
using namespace tz;

namespace {

// ---- Python-defined ops

class PyCpuOp : public CpuOp {
public:
  PyCpuOp(std::string name, py::function fn, double cost) : name_(std::move(name)), fn_(std::move(fn)), cost_(cost) {}
  ~PyCpuOp() override {
    py::gil_scoped_acquire g;
    fn_ = py::function();
  }
  std::string name() const override { return name_; }
  std::string kind() const override { return "PyCpuOp"; }
  double cost_us() const override { return cost_; }
  void run(Executor &ex) const override {
    if (!fn_ || ex.simulated()) { // the cost model charges the cost; the callback is not run
      ex.host_busy(cost_);
      return;
    }
    py::gil_scoped_acquire g;
    fn_();
  }

private:
  std::string name_;
  py::function fn_;
  double cost_;
};

class PyGpuOp : public GpuOp {
public:
  PyGpuOp(std::string name, py::function fn, double cost, bool capturable, std::string domain)
      : name_(std::move(name)), fn_(std::move(fn)), cost_(cost), capturable_(capturable),
        domain_(std::move(domain)) {}
  ~PyGpuOp() override {
    py::gil_scoped_acquire g;
    fn_ = py::function();
  }
  std::string name() const override { return name_; }
  std::string kind() const override { return "PyGpuOp"; }
  double cost_us() const override { return cost_; }
  bool capturable() const override { return capturable_; }
  std::string order_domain() const override { return domain_; }
  void launch(void *stream, Executor &) const override {
    py::gil_scoped_acquire g;
    fn_(reinterpret_cast<uintptr_t>(stream));
  }

private:
  std::string name_;
  py::function fn_;
  double cost_;
  bool capturable_;
  std::string domain_;
};

/// a benchmarker written in Python: fn(sequence, bench_opts) -> BenchResult (an analytical
/// model, a remote service, a replay of some other log...). An exception raised by fn counts as
/// a failed candidate (skipped by the solvers unless `skip_failed` is off).
class PyBenchmarker : public Benchmarker {
public:
  explicit PyBenchmarker(py::function fn) : fn_(std::move(fn)) {}
  ~PyBenchmarker() override {
    py::gil_scoped_acquire g;
    fn_ = py::function();
  }
  BenchResult benchmark(const Sequence &seq, const BenchOpts &opts) override {
    py::gil_scoped_acquire g;
    return fn_(seq, opts).cast<BenchResult>();
  }

private:
  py::function fn_;
};

py::dict counters_dict(const Counters &c) {
  py::dict d;
  for (const auto &kv : c.seconds) d[py::str(kv.first)] = kv.second;
  return d;
}

kern::BoxDesc box_from_dict(const py::dict &d) {
  kern::BoxDesc b;
  b.buf = reinterpret_cast<double *>(d["buf"].cast<uintptr_t>());
  b.grid_off = d["grid_off"].cast<int64_t>();
  b.s1 = d["s1"].cast<int64_t>();
  b.s2 = d["s2"].cast<int64_t>();
  b.s3 = d["s3"].cast<int64_t>();
  b.len = d["len"].cast<int>();
  b.n1 = d["n1"].cast<int>();
  b.n2 = d["n2"].cast<int>();
  b.n3 = d["n3"].cast<int>();
  // an unpack box's widening over row padding (unpack_box); absent: exactly the box
  if (d.contains("lead")) b.lead = d["lead"].cast<int>();
  if (d.contains("trail")) b.trail = d["trail"].cast<int>();
  return b;
}

py::dict box_to_dict(const kern::BoxDesc &b) {
  py::dict d;
  d["buf"] = reinterpret_cast<uintptr_t>(b.buf);
  d["grid_off"] = b.grid_off;
  d["s1"] = b.s1;
  d["s2"] = b.s2;
  d["s3"] = b.s3;
  d["len"] = b.len;
  d["lead"] = b.lead;
  d["trail"] = b.trail;
  d["n1"] = b.n1;
  d["n2"] = b.n2;
  d["n3"] = b.n3;
  return d;
}

void *P(uintptr_t p) { return reinterpret_cast<void *>(p); }

/// hold a Python object (the tensors behind an op's raw pointers) from C++; released under
/// the GIL whenever the last C++ owner lets go
std::shared_ptr<void> py_keep(py::object o) {
  if (o.is_none()) return nullptr;
  auto *p = new py::object(std::move(o));
  return std::shared_ptr<void>(p, [](void *q) {
    py::gil_scoped_acquire g;
    delete static_cast<py::object *>(q);
  });
}

// native backtrace on a fatal signal, then chain to the previous handler (Python faulthandler)
struct sigaction g_prevSegv, g_prevAbrt;
void crash_handler(int sig, siginfo_t *si, void *uc) {
  void *frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "\n[tz] fatal signal in native code, backtrace:\n";
  ssize_t w = write(2, msg, sizeof(msg) - 1);
  (void)w;
  backtrace_symbols_fd(frames, n, 2);
  struct sigaction &prev = sig == SIGSEGV ? g_prevSegv : g_prevAbrt;
  sigaction(sig, &prev, nullptr);
  if (prev.sa_flags & SA_SIGINFO) {
    if (prev.sa_sigaction) prev.sa_sigaction(sig, si, uc);
  } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN) {
    prev.sa_handler(sig);
  }
  raise(sig);
}
void install_crash_handler() {
  if (std::getenv("TZ_NO_CRASH_TRACE")) return;
  // an alternate signal stack for this (the main) thread: a stack overflow must still print
  static std::vector<char> altstack(size_t(1) << 16);
  stack_t ss{};
  ss.ss_sp = altstack.data();
  ss.ss_size = altstack.size();
  sigaltstack(&ss, nullptr);
  // warm backtrace() up: its first call loads the unwinder, which a signal handler must not do
  void *warm[2];
  (void)backtrace(warm, 2);
  struct sigaction sa {};
  sa.sa_sigaction = crash_handler;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prevSegv);
  sigaction(SIGABRT, &sa, &g_prevAbrt);
}

} // namespace

PYBIND11_MODULE(_tz, m) {
  m.doc() = "tenzing_amd native core: schedule search over HIP streams / RCCL on MI355X";
  install_crash_handler();

  py::register_exception<tz::Error>(m, "TzError");
  m.def("version", &version_string);
  m.def("reproduce_json", [](const std::vector<std::string> &a) { return reproduce_json(a).dump(); });
  m.def("set_log_level", [](int l) { set_log_level(LogLevel(l)); });
  m.def("set_log_rank", [](int r) { log_rank() = r; });
  m.def("hip_device_count", &hip_device_count);
  m.def("enable_roctx", &enable_roctx, py::arg("on") = true,
        "emit roctx ranges for MCTS phases and eager schedule ops (rocprofv3 --marker-trace)");
  m.def("pci_bus_id", [](int dev) {
    char buf[64] = {0};
    if (hipDeviceGetPCIBusId(buf, sizeof(buf), dev) != hipSuccess) return std::string();
    return std::string(buf);
  });
  m.def("rccl_version", &RcclComm::version);
  m.def("hip_runtime_version", [] {
    int v = 0;
    return hipRuntimeGetVersion(&v) == hipSuccess ? v : -1;
  }, "HIP_VERSION of the libamdhip64 this process actually uses (major*1e7 + minor*1e5 + patch)");
  m.def("graph_capture_info", [] {
    py::dict d;
    d["mode"] = std::string(capture_mode_name(capture_mode()));
    d["forced"] = capture_mode_forced();
    d["rccl_mode"] = std::string(capture_mode_name(rccl_capture_mode()));
    d["pad_streams"] = pad_streams();
    return d;
  }, "how schedules become hipGraphs: capture mode (schedules with RCCL between ranks: the mode "
     "the RCCL preflight settled on), default stream padding");
  m.def("set_graph_capture", &set_graph_capture, py::arg("mode"),
        "schedule | child: every schedule captured that way; auto: whole-schedule capture, RCCL "
        "schedules as their preflight found exact (process-wide)");
  m.def("set_default_pad_streams", &set_default_pad_streams, py::arg("n"),
        "streams a runtime created with pad_streams=-1 owns at least (process-wide, default 6)");
  m.def("device_by_pci_bus_id", [](const std::string &bus) {
    int d = -1;
    return hipDeviceGetByPCIBusId(&d, bus.c_str()) == hipSuccess ? d : -1;
  }, "this process's index of the GPU at PCI bus id `bus` (-1: not visible here)");
  m.def("can_access_peer", [](int a, int b) {
    int v = 0;
    return hipDeviceCanAccessPeer(&v, a, b) == hipSuccess && v != 0;
  }, "hipDeviceCanAccessPeer(a, b)");
  m.def("hip_driver_version", [] {
    int v = 0;
    return hipDriverGetVersion(&v) == hipSuccess ? v : -1;
  });
  m.def("rccl_unique_id", [] { return py::bytes(RcclComm::unique_id()); },
        "a fresh ncclUniqueId as bytes");
  m.def("strategy_names", &strategy_names);
  m.def("prime_factors", &prime_factors);
  m.def("runs_test", [](const std::vector<double> &v, bool rejectSmall) {
    return runs_test(v, rejectSmall ? RunsTestSmall::Reject : RunsTestSmall::Accept);
  }, py::arg("v"), py::arg("reject_small") = false);

  // ------------------------------------------------------------------ ops
  py::class_<OpBase, std::shared_ptr<OpBase>>(m, "OpBase")
      .def_property_readonly("name", &OpBase::name)
      .def_property_readonly("kind", &OpBase::kind)
      .def_property_readonly("op_class", [](const OpBase &o) { return std::string(op_class_name(o.op_class())); })
      .def("json", [](const OpBase &o) { return o.json().dump(); })
      .def("traffic", [](const OpBase &o) {
             const GpuOp *g = dynamic_cast<const GpuOp *>(&o);
             if (auto b = dynamic_cast<const BoundGpuOp *>(&o)) g = b->unbound().get();
             py::list l;
             if (g)
               for (const Traffic &t : g->traffic()) l.append(py::make_tuple(t.resource, t.engine, t.bytes));
             return l;
           }, "(resource, engine, bytes) a GPU op moves, for the link-aware simulator ([] otherwise)")
      .def("desc", &OpBase::desc)
      .def("eq", &OpBase::eq)
      .def_property_readonly("cost_us", &OpBase::cost_us)
      .def_property_readonly("bytes", &OpBase::bytes)
      .def_property_readonly("order_domain", &OpBase::order_domain)
      .def("__repr__", [](const OpBase &o) { return "<" + o.kind() + " " + o.desc() + ">"; });
  py::class_<BoundOp, OpBase, std::shared_ptr<BoundOp>>(m, "BoundOp");
  py::class_<CpuOp, BoundOp, std::shared_ptr<CpuOp>>(m, "CpuOp");
  py::class_<GpuOp, OpBase, std::shared_ptr<GpuOp>>(m, "GpuOp")
      .def("latency_us", &GpuOp::latency_us);
  py::class_<Start, CpuOp, std::shared_ptr<Start>>(m, "Start").def(py::init<>());
  py::class_<Finish, CpuOp, std::shared_ptr<Finish>>(m, "Finish").def(py::init<>());
  py::class_<NoOp, CpuOp, std::shared_ptr<NoOp>>(m, "NoOp")
      .def(py::init<std::string, double>(), py::arg("name"), py::arg("cost_us") = 0.0);
  py::class_<SleepOp, CpuOp, std::shared_ptr<SleepOp>>(m, "SleepOp").def(py::init<std::string, double>());
  py::class_<PyCpuOp, CpuOp, std::shared_ptr<PyCpuOp>>(m, "PyCpuOp")
      .def(py::init<std::string, py::function, double>(), py::arg("name"), py::arg("fn"), py::arg("cost_us") = 0.0);
  py::class_<SimGpuOp, GpuOp, std::shared_ptr<SimGpuOp>>(m, "SimGpuOp")
      .def(py::init([](std::string name, double us, std::string domain, py::list traffic) {
             std::vector<Traffic> tr;
             for (auto h : traffic) {
               auto t = h.cast<py::tuple>();
               tr.push_back({t[0].cast<std::string>(), t[1].cast<std::string>(), t[2].cast<double>()});
             }
             return std::make_shared<SimGpuOp>(std::move(name), us, std::move(domain), std::move(tr));
           }), py::arg("name"), py::arg("us"), py::arg("domain") = "", py::arg("traffic") = py::list(),
           "a GPU op that only models time: `us`, or with `traffic` [(resource, engine, bytes)] "
           "that fixed latency plus its transfers under the link-aware model");
  py::class_<PyGpuOp, GpuOp, std::shared_ptr<PyGpuOp>>(m, "PyGpuOp")
      .def(py::init<std::string, py::function, double, bool, std::string>(), py::arg("name"),
           py::arg("fn"), py::arg("cost_us") = 0.0, py::arg("capturable") = true,
           py::arg("domain") = "");
  py::class_<EmptyKernelOp, GpuOp, std::shared_ptr<EmptyKernelOp>>(m, "EmptyKernelOp").def(py::init<std::string>());
  py::class_<HostFuncOp, GpuOp, std::shared_ptr<HostFuncOp>>(m, "HostFuncOp").def(py::init<std::string>());
  py::class_<BusyKernelOp, GpuOp, std::shared_ptr<BusyKernelOp>>(m, "BusyKernelOp")
      .def(py::init<std::string, double, int>(), py::arg("name"), py::arg("us"), py::arg("blocks") = 1);
  py::class_<BoundGpuOp, BoundOp, std::shared_ptr<BoundGpuOp>>(m, "BoundGpuOp")
      .def(py::init([](std::shared_ptr<GpuOp> op, int s) { return std::make_shared<BoundGpuOp>(op, s); }))
      .def_property_readonly("stream", &BoundGpuOp::stream)
      .def_property_readonly("unbound", [](const BoundGpuOp &b) { return std::const_pointer_cast<GpuOp>(b.unbound()); });
  py::class_<SyncOp, BoundOp, std::shared_ptr<SyncOp>>(m, "SyncOp")
      .def_property_readonly("stream", &SyncOp::stream)
      .def_property_readonly("event", &SyncOp::event);
  py::class_<EventRecord, SyncOp, std::shared_ptr<EventRecord>>(m, "EventRecord")
      .def(py::init<int, int, std::string>(), py::arg("event"), py::arg("stream"), py::arg("name") = "");
  py::class_<StreamWaitEvent, SyncOp, std::shared_ptr<StreamWaitEvent>>(m, "StreamWaitEvent")
      .def(py::init<int, int, std::string>(), py::arg("stream"), py::arg("event"), py::arg("name") = "");
  py::class_<EventSync, SyncOp, std::shared_ptr<EventSync>>(m, "EventSync")
      .def(py::init<int, std::string>(), py::arg("event"), py::arg("name") = "");
  py::class_<StreamSync, SyncOp, std::shared_ptr<StreamSync>>(m, "StreamSync")
      .def(py::init<int, std::string>(), py::arg("stream"), py::arg("name") = "");
  py::class_<StreamWait, SyncOp, std::shared_ptr<StreamWait>>(m, "StreamWait")
      .def(py::init<int, int, std::string>(), py::arg("waiter"), py::arg("waitee"), py::arg("name") = "");
  py::class_<ChoiceOp, OpBase, std::shared_ptr<ChoiceOp>>(m, "ChoiceOp")
      .def("choices", [](const ChoiceOp &c) {
        std::vector<std::shared_ptr<OpBase>> out;
        for (auto &x : c.choices()) out.push_back(std::const_pointer_cast<OpBase>(x));
        return out;
      });
  py::class_<StaticChoiceOp, ChoiceOp, std::shared_ptr<StaticChoiceOp>>(m, "StaticChoiceOp")
      .def(py::init([](std::string name, std::vector<std::shared_ptr<OpBase>> ch) {
        std::vector<OpPtr> c(ch.begin(), ch.end());
        return std::make_shared<StaticChoiceOp>(name, c);
      }));
  py::class_<CompoundOp, OpBase, std::shared_ptr<CompoundOp>>(m, "CompoundOp")
      .def("graph", [](const CompoundOp &c) { return std::const_pointer_cast<Graph>(c.graph()); });
  py::class_<StaticCompoundOp, CompoundOp, std::shared_ptr<StaticCompoundOp>>(m, "StaticCompoundOp")
      .def(py::init([](std::string name, std::shared_ptr<Graph> g) {
        return std::make_shared<StaticCompoundOp>(name, std::make_shared<Graph>(*g));
      }));

  auto cop = [](const std::shared_ptr<OpBase> &o) { return std::const_pointer_cast<const OpBase>(o); };

  // ------------------------------------------------------------------ graph
  py::class_<Graph, std::shared_ptr<Graph>>(m, "Graph")
      .def(py::init<>())
      .def("add", [cop](Graph &g, std::shared_ptr<OpBase> o) { return g.add(cop(o)); })
      .def("then", [cop](Graph &g, std::shared_ptr<OpBase> a, std::shared_ptr<OpBase> b) { g.then(cop(a), cop(b)); })
      .def("start_then", [cop](Graph &g, std::shared_ptr<OpBase> a) { g.start_then(cop(a)); })
      .def("then_finish", [cop](Graph &g, std::shared_ptr<OpBase> a) { g.then_finish(cop(a)); })
      .def("add_edge", &Graph::add_edge)
      .def("erase", [](Graph &g, const std::string &name) {
        const int id = g.find(name);
        TZ_CHECK(id >= 0, "no op named " << name);
        g.erase(id);
      }, py::arg("name"), "remove an op and its edges")
      .def("erase_edge", [](Graph &g, const std::string &a, const std::string &b) {
        const int ia = g.find(a), ib = g.find(b);
        TZ_CHECK(ia >= 0 && ib >= 0, "no op named " << (ia < 0 ? a : b));
        g.erase_edge(ia, ib);
      }, py::arg("a"), py::arg("b"), "remove the edge a -> b (keep both ops)")
      .def("normalize", &Graph::normalize)
      .def("__len__", &Graph::size)
      .def_property_readonly("capacity", &Graph::capacity)
      .def("vertices", &Graph::vertices)
      .def("op", [](const Graph &g, int i) { return std::const_pointer_cast<OpBase>(g.op(i)); })
      .def("preds", &Graph::preds)
      .def("succs", &Graph::succs)
      .def("find", &Graph::find)
      .def("contains", &Graph::contains)
      .def("topo_order", &Graph::topo_order)
      .def("num_edges", &Graph::num_edges)
      .def("clone", [](const Graph &g) { return g.clone(); })
      .def("clone_but_replace", [cop](const Graph &g, int id, std::shared_ptr<OpBase> o) { return g.clone_but_replace(id, cop(o)); })
      .def("clone_but_expand", &Graph::clone_but_expand)
      .def("dump_graphviz", &Graph::dump_graphviz, py::arg("title") = "")
      .def("json", [](const Graph &g) { return g.json().dump(); });

  // ------------------------------------------------------------------ SDP
  py::class_<Platform>(m, "Platform")
      .def(py::init([](int n, bool sym, bool ss) {
        Platform p;
        p.n_streams = n;
        p.symmetric_streams = sym;
        p.offer_stream_sync = ss;
        return p;
      }), py::arg("n_streams") = 2, py::arg("symmetric_streams") = true, py::arg("offer_stream_sync") = false)
      .def_readwrite("n_streams", &Platform::n_streams)
      .def_readwrite("symmetric_streams", &Platform::symmetric_streams)
      .def_readwrite("offer_stream_sync", &Platform::offer_stream_sync);

  py::class_<Sequence>(m, "Sequence")
      .def(py::init<>())
      .def("__len__", &Sequence::size)
      .def("__getitem__", [](const Sequence &s, size_t i) {
        if (i >= s.size()) throw py::index_error();
        return std::const_pointer_cast<BoundOp>(s[i]);
      })
      .def("append", [](Sequence &s, std::shared_ptr<BoundOp> o) { s.push_back(o, -1); })
      .def("ops", [](const Sequence &s) {
        std::vector<std::shared_ptr<BoundOp>> v;
        for (auto &e : s.entries) v.push_back(std::const_pointer_cast<BoundOp>(e.op));
        return v;
      })
      .def("json", [](const Sequence &s, bool ig) { return s.json(ig).dump(); }, py::arg("in_graph") = false)
      .def("desc", &Sequence::desc, py::arg("delim") = ", ")
      .def("canonical_key", &Sequence::canonical_key)
      .def("num_events", &Sequence::num_events)
      .def("num_streams", &Sequence::num_streams)
      .def("count_sync_ops", &Sequence::count_sync_ops)
      .def("equivalent", [](const Sequence &a, const Sequence &b) { return equivalent(a, b); });

  py::class_<Decision>(m, "Decision")
      .def_property_readonly("kind", [](const Decision &d) {
        switch (d.kind) {
        case Decision::Kind::Execute: return "Execute";
        case Decision::Kind::Expand: return "Expand";
        case Decision::Kind::Choose: return "Choose";
        default: return "Assign";
        }
      })
      .def_property_readonly("op", [](const Decision &d) { return std::const_pointer_cast<BoundOp>(d.op); })
      .def_readonly("node", &Decision::node)
      .def_readonly("stream", &Decision::stream)
      .def_readonly("choice", &Decision::choice)
      .def("desc", &Decision::desc)
      .def("__repr__", &Decision::desc);

  py::class_<State>(m, "State")
      .def(py::init([](std::shared_ptr<Graph> g, const Platform &p) { return State(g, p); }),
           py::arg("graph"), py::arg("platform") = Platform())
      .def_property_readonly("sequence", &State::sequence)
      .def_property_readonly("graph", [](const State &s) { return std::const_pointer_cast<Graph>(s.graph_ptr()); })
      .def("frontier", &State::frontier)
      .def("get_decisions", &State::get_decisions)
      .def("apply", &State::apply)
      .def("complete", &State::complete)
      .def("stream_of", &State::stream_of)
      .def("executed", &State::executed)
      .def("canonical_key", &State::canonical_key)
      .def("equivalent", [](const State &a, const State &b) { return equivalent(a, b); });

  m.def("resolve_graph", [](const Graph &g, const Sequence &s) {
    return std::const_pointer_cast<Graph>(resolve_graph(g, s));
  }, py::arg("graph"), py::arg("seq"),
     "the graph `seq` executed: compounds expanded, each choice replaced by the alternative it runs");
  m.def("verify", [](const Sequence &s, const Graph &g, int n) {
    std::vector<std::string> out;
    for (auto &v : verify(s, g, n)) out.push_back(v.desc());
    return out;
  });
  m.def("remove_redundant_syncs", [](Sequence s, const Graph &g, int n) {
    int k = remove_redundant_syncs(s, g, n);
    return py::make_tuple(s, k);
  });
  m.def("random_rollout", [](const State &s, uint64_t seed) {
    std::mt19937_64 rng(seed);
    return random_rollout(s, rng);
  });

  py::class_<OpIndex>(m, "OpIndex")
      .def(py::init<const Graph &>())
      .def("from_json", [](const OpIndex &i, const std::string &j) { return std::const_pointer_cast<BoundOp>(i.from_json(Json::parse(j))); })
      .def("sequence_from_json", [](const OpIndex &i, const std::string &j) { return i.sequence_from_json(Json::parse(j)); });

  // ------------------------------------------------------------------ benchmark
  py::class_<BenchOpts>(m, "BenchOpts")
      .def(py::init([](int64_t n, int r, double t, bool rs, bool dev, double race, double settle) {
        BenchOpts o;
        o.n_iters = n;
        o.max_retries = r;
        o.target_secs = t;
        o.small_sample = rs ? RunsTestSmall::Reject : RunsTestSmall::Accept;
        o.device_timer = dev;
        o.race_ratio = race;
        o.settle_ratio = settle;
        return o;
      }), py::arg("n_iters") = 1000, py::arg("max_retries") = 10, py::arg("target_secs") = 0.01,
         py::arg("reject_small_samples") = false, py::arg("device_timer") = false,
         py::arg("race_ratio") = 0.0, py::arg("settle_ratio") = 0.0)
      .def_readwrite("race_ratio", &BenchOpts::race_ratio)
      .def_readwrite("race_min", &BenchOpts::race_min)
      .def_readwrite("settle_ratio", &BenchOpts::settle_ratio)
      .def_readwrite("settle_min", &BenchOpts::settle_min)
      .def_readwrite("n_iters", &BenchOpts::n_iters)
      .def_readwrite("max_retries", &BenchOpts::max_retries)
      .def_readwrite("target_secs", &BenchOpts::target_secs)
      .def_readwrite("device_timer", &BenchOpts::device_timer);

  py::class_<BenchResult>(m, "BenchResult")
      .def(py::init<>())
      .def_readwrite("pct01", &BenchResult::pct01)
      .def_readwrite("pct10", &BenchResult::pct10)
      .def_readwrite("pct50", &BenchResult::pct50)
      .def_readwrite("pct90", &BenchResult::pct90)
      .def_readwrite("pct99", &BenchResult::pct99)
      .def_readwrite("stddev", &BenchResult::stddev)
      .def_readonly("samples_per_measurement", &BenchResult::samples_per_measurement)
      .def_readonly("retries", &BenchResult::retries)
      .def("json", [](const BenchResult &r) { return r.json().dump(); })
      .def_static("from_times", &BenchResult::from_times);

  py::class_<Benchmarker>(m, "Benchmarker")
      .def("benchmark", &Benchmarker::benchmark, py::call_guard<py::gil_scoped_release>());
  py::class_<SimParams>(m, "SimParams")
      .def(py::init<>())
      .def_readwrite("launch_us", &SimParams::launch_us)
      .def_readwrite("api_us", &SimParams::api_us)
      .def_readwrite("sync_us", &SimParams::sync_us)
      .def_readwrite("noise", &SimParams::noise)
      .def_readwrite("seed", &SimParams::seed)
      .def_readwrite("contention", &SimParams::contention)
      .def_readwrite("link_model", &SimParams::link_model)
      .def_readwrite("graph", &SimParams::graph)
      .def_readwrite("graph_gap_us", &SimParams::graph_gap_us)
      .def_readwrite("graph_join_us", &SimParams::graph_join_us)
      .def_readwrite("graph_wait_us", &SimParams::graph_wait_us)
      .def_readwrite("engine_GBps", &SimParams::engine_GBps)
      .def_readwrite("resource_GBps", &SimParams::resource_GBps);
  py::class_<SimBenchmarker, Benchmarker>(m, "SimBenchmarker")
      .def(py::init<int, SimParams, Ctrl *>(), py::arg("n_streams"), py::arg("params") = SimParams(),
           py::arg("ctrl") = nullptr, py::keep_alive<1, 4>(),
           "discrete-event model; with `ctrl`, every rank simulates its own copy of each schedule "
           "and the result is the max over ranks");
  py::class_<SimExecutor>(m, "SimExecutor")
      .def(py::init<int, SimParams>(), py::arg("n_streams"), py::arg("params") = SimParams())
      .def("run_once", &SimExecutor::run_once)
      .def("trace", [](const SimExecutor &e) {
        py::list l;
        for (auto &s : e.trace()) l.append(py::make_tuple(s.name, s.stream, s.start, s.end));
        return l;
      });
  py::class_<PyBenchmarker, Benchmarker>(m, "PyBenchmarker")
      .def(py::init<py::function>(), py::arg("fn"));
  py::class_<CsvBenchmarker, Benchmarker>(m, "CsvBenchmarker")
      .def(py::init<const std::string &, const Graph &>())
      .def("__len__", &CsvBenchmarker::size);
  py::class_<ExecutorRunner>(m, "ExecutorRunner")
      .def("prepare", &ExecutorRunner::prepare, py::call_guard<py::gil_scoped_release>())
      .def("run", &ExecutorRunner::run, py::call_guard<py::gil_scoped_release>());
  py::class_<HostExecutor, ExecutorRunner>(m, "HostExecutor", py::multiple_inheritance()).def(py::init<int>());
  py::class_<EmpiricalBenchmarker, Benchmarker>(m, "EmpiricalBenchmarker")
      .def(py::init<ExecutorRunner &, Ctrl &>(), py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def_property_readonly("raced", &EmpiricalBenchmarker::raced)
      .def_property_readonly("settled", &EmpiricalBenchmarker::settled)
      .def("reset_race", &EmpiricalBenchmarker::reset_race)
      .def("benchmark_many", &EmpiricalBenchmarker::benchmark_many, py::arg("seqs"), py::arg("opts"),
           py::arg("seed") = 0, py::call_guard<py::gil_scoped_release>(),
           "interleaved measurement of several schedules (random order per iteration)");

  // ------------------------------------------------------------------ control plane
  py::class_<Ctrl, std::shared_ptr<Ctrl>>(m, "Ctrl")
      .def_property_readonly("rank", &Ctrl::rank)
      .def_property_readonly("size", &Ctrl::size)
      .def("barrier", &Ctrl::barrier, py::call_guard<py::gil_scoped_release>())
      .def("bcast", [](Ctrl &c, std::string s, int root) {
        {
          py::gil_scoped_release r;
          c.bcast(s, root);
        }
        return py::bytes(s);
      }, py::arg("data"), py::arg("root") = 0)
      .def("allreduce_max", [](Ctrl &c, std::vector<double> v) {
        py::gil_scoped_release r;
        c.allreduce_max(v.data(), v.size());
        return v;
      })
      .def("allreduce_sum", [](Ctrl &c, std::vector<double> v) {
        py::gil_scoped_release r;
        c.allreduce_sum(v.data(), v.size());
        return v;
      })
      .def("allgather", [](Ctrl &c, const std::string &s) {
        std::vector<std::string> out;
        {
          py::gil_scoped_release r;
          out = c.allgather(s);
        }
        py::list l;
        for (auto &x : out) l.append(py::bytes(x));
        return l;
      })
      .def("alltoallv", [](Ctrl &c, const std::vector<std::string> &outs) {
        std::vector<std::string> in;
        {
          py::gil_scoped_release r;
          in = c.alltoallv(outs);
        }
        py::list l;
        for (auto &x : in) l.append(py::bytes(x));
        return l;
      }, "personalized exchange: element j goes to rank j; returns what each rank sent me");
  py::class_<SelfCtrl, Ctrl, std::shared_ptr<SelfCtrl>>(m, "SelfCtrl").def(py::init<>());
  py::class_<TcpCtrl, Ctrl, std::shared_ptr<TcpCtrl>>(m, "TcpCtrl")
      .def(py::init<int, int>())
      .def("listen", &TcpCtrl::listen, py::arg("port") = 0, py::arg("bind_addr") = "0.0.0.0")
      .def("connect", &TcpCtrl::connect, py::arg("host"), py::arg("port"), py::arg("timeout_s") = 300.0,
           py::call_guard<py::gil_scoped_release>())
      .def("rendezvous", &TcpCtrl::rendezvous, py::arg("host"), py::arg("port"),
           py::arg("timeout_s") = 300.0, py::arg("nports") = 8, py::call_guard<py::gil_scoped_release>(),
           "rank 0 listens on the first free port of port..port+nports-1, the others connect "
           "(handshake-checked): no store, no torch")
      .def("rendezvous_file", &TcpCtrl::rendezvous_file, py::arg("path"), py::arg("host") = "127.0.0.1",
           py::arg("timeout_s") = 300.0, py::call_guard<py::gil_scoped_release>())
      .def("ensure_timeout", &TcpCtrl::ensure_timeout, py::arg("seconds"),
           "raise the peer sockets' receive timeout to at least this (never lowered)")
      .def_property_readonly("timeout", &TcpCtrl::timeout,
                             "the peer sockets' receive timeout in seconds (0 = none)");
  py::class_<MpiCtrl, Ctrl, std::shared_ptr<MpiCtrl>>(m, "MpiCtrl")
      .def(py::init<const std::string &>(), py::arg("lib") = "", py::call_guard<py::gil_scoped_release>())
      .def_static("launched", &MpiCtrl::launched)
      .def_static("launcher_size", &MpiCtrl::launcher_size)
      .def_static("launcher_local_rank", &MpiCtrl::launcher_local_rank)
      .def_property_readonly("library", &MpiCtrl::library);

  // ------------------------------------------------------------------ solvers
  py::class_<MctsOpts>(m, "MctsOpts")
      .def(py::init<>())
      .def_readwrite("n_iters", &MctsOpts::n_iters)
      .def_readwrite("time_budget_s", &MctsOpts::time_budget_s)
      .def_readwrite("max_tree_nodes", &MctsOpts::max_tree_nodes)
      .def_readwrite("seed_schedules", &MctsOpts::seed_schedules)
      .def_readwrite("expand_rollout", &MctsOpts::expand_rollout)
      .def_readwrite("remove_redundant_syncs", &MctsOpts::remove_redundant_syncs)
      .def_readwrite("reuse_measurements", &MctsOpts::reuse_measurements)
      .def_readwrite("verify", &MctsOpts::verify)
      .def_readwrite("dump_tree", &MctsOpts::dump_tree)
      .def_readwrite("dump_tree_prefix", &MctsOpts::dump_tree_prefix)
      .def_readwrite("strategy", &MctsOpts::strategy)
      .def_readwrite("seed", &MctsOpts::seed)
      .def_readwrite("explore_c", &MctsOpts::explore_c)
      .def_readwrite("bench", &MctsOpts::bench)
      .def_readwrite("checkpoint_path", &MctsOpts::checkpoint_path)
      .def_readwrite("checkpoint_every", &MctsOpts::checkpoint_every)
      .def_readwrite("resume_path", &MctsOpts::resume_path)
      .def_readwrite("trap_signals", &MctsOpts::trap_signals)
      .def_readwrite("skip_failed", &MctsOpts::skip_failed)
      .def("json", [](const MctsOpts &o) { return o.json().dump(); });
  py::class_<DfsOpts>(m, "DfsOpts")
      .def(py::init<>())
      .def_readwrite("max_seqs", &DfsOpts::max_seqs)
      .def_readwrite("dedup_states", &DfsOpts::dedup_states)
      .def_readwrite("remove_redundant_syncs", &DfsOpts::remove_redundant_syncs)
      .def_readwrite("bench", &DfsOpts::bench)
      .def_readwrite("trap_signals", &DfsOpts::trap_signals)
      .def_readwrite("skip_failed", &DfsOpts::skip_failed)
      .def("json", [](const DfsOpts &o) { return o.json().dump(); });
  py::class_<SimResult>(m, "SimResult")
      .def_readonly("seq", &SimResult::seq)
      .def_readonly("res", &SimResult::res)
      .def_readonly("cached", &SimResult::cached)
      .def_readonly("seeded", &SimResult::seeded);
  py::class_<SearchResult>(m, "SearchResult")
      .def_readonly("sims", &SearchResult::sims)
      .def_readonly("wall_s", &SearchResult::wall_s)
      .def_readonly("tree_size", &SearchResult::tree_size)
      .def_readonly("tree_fully_visited", &SearchResult::tree_fully_visited)
      .def_readonly("stop_reason", &SearchResult::stop_reason)
      .def_readonly("failed", &SearchResult::failed)
      .def_readonly("dead_domains", &SearchResult::dead_domains)
      .def_readonly("pruned_dead", &SearchResult::pruned_dead)
      .def("best", &SearchResult::best)
      .def("counters", [](const SearchResult &r) { return counters_dict(r.counters); })
      .def("counter_counts", [](const SearchResult &r) {
        py::dict d;
        for (const auto &kv : r.counters.counts) d[py::str(kv.first)] = kv.second;
        return d;
      }, "how often each counter was hit (phases; SEED_IN_TREE: seeds placed in the tree)")
      .def("dump_csv", [](const SearchResult &r) {
        std::ostringstream ss;
        r.dump_csv(ss);
        return ss.str();
      })
      .def("dump_jsonl", [](const SearchResult &r) {
        std::ostringstream ss;
        r.dump_jsonl(ss);
        return ss.str();
      });
  py::class_<RunDeadline>(m, "RunDeadline")
      .def(py::init<double, int>(), py::arg("seconds"), py::arg("exit_code") = 5)
      .def("set_report", &RunDeadline::set_report, py::arg("line"))
      .def("cancel", &RunDeadline::cancel)
      .def("tighten", &RunDeadline::tighten, py::arg("seconds"), py::arg("exit_code"),
           "expire at the latest `seconds` from now, exiting with `exit_code`")
      .def_property_readonly("remaining", &RunDeadline::remaining)
      .def_property_readonly("armed", &RunDeadline::armed);
  m.def("exit_with_report", [](int code, const std::string &why) { exit_with_report(code, why); },
        py::arg("code"), py::arg("why"),
        "leave the process now (no cleanup), printing the armed RunDeadline's report line with "
        "\"exit_reason\" added: what the watchdog does when a hung run cannot be released");
  m.def("mcts_explore", [](std::shared_ptr<Graph> g, const Platform &p, Benchmarker &b, Ctrl &c,
                           const MctsOpts &o, py::object cb) {
    std::function<void(size_t, const SimResult &)> f;
    if (!cb.is_none()) {
      f = [cb](size_t i, const SimResult &r) {
        py::gil_scoped_acquire a;
        cb(i, r);
      };
    }
    py::gil_scoped_release r;
    return mcts_explore(*g, p, b, c, o, f);
  }, py::arg("graph"), py::arg("platform"), py::arg("bench"), py::arg("ctrl"), py::arg("opts"),
     py::arg("callback") = py::none());
  m.def("dfs_explore", [](std::shared_ptr<Graph> g, const Platform &p, Benchmarker &b, Ctrl &c,
                          const DfsOpts &o, py::object cb) {
    std::function<void(size_t, const SimResult &)> f;
    if (!cb.is_none()) {
      f = [cb](size_t i, const SimResult &r) {
        py::gil_scoped_acquire a;
        cb(i, r);
      };
    }
    py::gil_scoped_release r;
    return dfs_explore(*g, p, b, c, o, f);
  }, py::arg("graph"), py::arg("platform"), py::arg("bench"), py::arg("ctrl"), py::arg("opts"),
     py::arg("callback") = py::none());
  m.def("get_all_sequences", [](std::shared_ptr<Graph> g, const Platform &p, int64_t mx, bool dd, bool rr) {
    py::gil_scoped_release r;
    return get_all_sequences(*g, p, mx, dd, rr);
  }, py::arg("graph"), py::arg("platform"), py::arg("max_seqs") = -1, py::arg("dedup_states") = true,
     py::arg("remove_redundant_syncs") = true);

  // ------------------------------------------------------------------ HIP runtime
  py::enum_<ExecMode>(m, "ExecMode").value("Eager", ExecMode::Eager).value("Graph", ExecMode::Graph);
  py::class_<HipRuntime, ExecutorRunner>(m, "HipRuntime", py::multiple_inheritance())
      .def(py::init([](int device, int n, std::vector<int> prio, bool cu, ExecMode mode, double wd,
                       int unroll, double wk, int pad) {
        HipRuntimeOpts o;
        o.pad_streams = pad;
        o.device = device;
        o.n_streams = n;
        o.priorities = prio;
        o.cu_partition = cu;
        o.mode = mode;
        o.watchdog_s = wd;
        o.watchdog_k = wk;
        o.graph_unroll = unroll;
        return new HipRuntime(o);
      }), py::arg("device") = -1, py::arg("n_streams") = 2, py::arg("priorities") = std::vector<int>{},
         py::arg("cu_partition") = false, py::arg("mode") = ExecMode::Eager, py::arg("watchdog_s") = 0.0,
         py::arg("graph_unroll") = 1, py::arg("watchdog_k") = 50.0, py::arg("pad_streams") = -1)
      .def_property_readonly("pad_streams", &HipRuntime::pad_streams,
                             "streams this runtime owns at least (schedule streams + never-used spares)")
      .def("set_graph_unroll", &HipRuntime::set_graph_unroll)
      .def("precompile", &HipRuntime::precompile, py::arg("n"),
           "graph mode: compile the n % unroll remainder of a run(n) as one graph (before timing it)")
      .def_property_readonly("graph_unroll", &HipRuntime::graph_unroll)
      .def("set_mode", &HipRuntime::set_mode)
      .def_property_readonly("mode", &HipRuntime::mode)
      .def_property_readonly("effective_mode", &HipRuntime::effective_mode)
      .def_property_readonly("device", &HipRuntime::device)
      .def("device_name", &HipRuntime::device_name)
      .def("graph_nodes", &HipRuntime::graph_nodes)
      .def("graph_edges", &HipRuntime::graph_edges)
      .def("num_streams", &HipRuntime::num_streams)
      .def("graph_node_types", &HipRuntime::graph_node_types,
           "node count by type of the compiled graph (kernel, host, memcpy, event_record, ...)")
      .def("native_stream", [](HipRuntime &r, int s) { return reinterpret_cast<uintptr_t>(r.native_stream(s)); })
      .def("device_sync", &HipRuntime::device_sync, py::call_guard<py::gil_scoped_release>())
      .def("set_watchdog", &HipRuntime::set_watchdog, py::arg("floor_s"), py::arg("k") = -1.0)
      .def_property_readonly("watchdog_floor", &HipRuntime::watchdog_floor)
      .def_property_readonly("watchdog_k", &HipRuntime::watchdog_k)
      .def_property_readonly("expected_iter_s", &HipRuntime::expected_iter_s)
      .def_property_readonly("watchdog_fired", &HipRuntime::watchdog_fired)
      .def("watchdog_budget", &HipRuntime::watchdog_budget, py::arg("n"),
           "seconds the watchdog gives a run of n iterations of the prepared schedule")
      .def_property("spin_sync", &HipRuntime::spin_sync, &HipRuntime::set_spin_sync)
      .def("trace", [](HipRuntime &r, const Sequence &seq, int iterations) {
             std::vector<HipRuntime::Span> sp;
             {
               py::gil_scoped_release nogil;
               sp = r.trace(seq, iterations);
             }
             py::list l;
             for (const auto &s : sp) l.append(py::make_tuple(s.name, s.stream, s.iteration, s.start_us, s.end_us));
             return l;
           }, py::arg("seq"), py::arg("iterations") = 1,
           "eager run with timing events around every GPU op: [(name, stream (-1 host), iteration, start_us, end_us)]");
  m.def("chrome_trace", [](const std::vector<std::tuple<std::string, int, int, double, double>> &spans) {
    std::vector<HipRuntime::Span> v;
    for (const auto &t : spans)
      v.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t), std::get<4>(t)});
    return chrome_trace(v).dump();
  }, py::arg("spans"), "Chrome trace-event JSON of (name, stream, iteration, start_us, end_us) spans");

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](Ctrl &c, int dev) { return std::make_shared<RcclComm>(c, dev); }))
      .def_static("from_id", [](py::bytes uid, int rank, int size, int dev) {
             std::string u = uid;
             py::gil_scoped_release r;
             return std::make_shared<RcclComm>(u, rank, size, dev);
           }, py::arg("unique_id"), py::arg("rank"), py::arg("size"), py::arg("device"),
           "join a communicator whose unique id was distributed out of band (bounded by "
           "TZ_RCCL_INIT_S: raises if the other ranks do not join in time)")
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def("allreduce_sum", [](const RcclComm &c, uintptr_t buf, size_t n, int dt, uintptr_t s) {
        c.allreduce_sum(P(buf), n, dt, P(s));
      })
      .def("sendrecv", [](const RcclComm &c, uintptr_t sb, size_t sc, int sp, uintptr_t rb, size_t rc, int rp, int dt, uintptr_t s) {
        c.sendrecv(P(sb), sc, sp, P(rb), rc, rp, dt, P(s));
      })
      .def("allreduce", [](const RcclComm &c, uintptr_t sb, uintptr_t rb, size_t n, int dt, int red, uintptr_t s) {
        c.allreduce(P(sb), P(rb), n, dt, red, P(s));
      }, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("red") = 0, py::arg("stream") = 0)
      .def("allgather", [](const RcclComm &c, uintptr_t sb, uintptr_t rb, size_t n, int dt, uintptr_t s) {
        c.allgather(P(sb), P(rb), n, dt, P(s));
      }, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("stream") = 0)
      .def("reduce_scatter", [](const RcclComm &c, uintptr_t sb, uintptr_t rb, size_t n, int dt, int red, uintptr_t s) {
        c.reduce_scatter(P(sb), P(rb), n, dt, red, P(s));
      }, py::arg("send"), py::arg("recv"), py::arg("recv_count"), py::arg("dtype"), py::arg("red") = 0, py::arg("stream") = 0)
      .def("broadcast", [](const RcclComm &c, uintptr_t sb, uintptr_t rb, size_t n, int root, int dt, uintptr_t s) {
        c.broadcast(P(sb), P(rb), n, root, dt, P(s));
      }, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("root"), py::arg("dtype"), py::arg("stream") = 0)
      .def_static("dtype_size", &RcclComm::dtype_size)
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted);
  m.def("rccl_abort_all", &rccl_abort_all, py::call_guard<py::gil_scoped_release>());
  m.def("mark_domain_dead", &mark_domain_dead, py::arg("domain"), py::arg("why") = "",
        "take an ordering domain (a transport, e.g. 'rccl') out of every later search");
  m.def("domain_dead", &domain_dead);
  m.def("dead_domains", [] {
    auto d = dead_domains();
    return std::vector<std::string>(d.begin(), d.end());
  });
  m.def("revive_domains", &revive_domains);
  m.def("agree_dead_domains", [](Ctrl &c) {
    std::set<std::string> d;
    {
      py::gil_scoped_release r;
      d = agree_dead_domains(c);
    }
    return std::vector<std::string>(d.begin(), d.end());
  }, "collective: every rank adopts the union of the ranks' dead domains");
  m.def("device_abort_set", &kern::abort_set, "the device abort flag is set (a watchdog fired)");
  m.def("note_abort", &note_abort, "record an aborted run (the watchdog does this)");
  m.def("aborts_noted", &aborts_noted);
  m.def("add_recovery_hook", [](py::function fn) {
    // the hook list is a static of the library: a hook still registered at exit is destroyed
    // after the interpreter has finalized, when the reference must not be touched any more
    auto keep = std::shared_ptr<py::function>(new py::function(std::move(fn)), [](py::function *p) {
      if (Py_IsInitialized() && !_Py_IsFinalizing()) {
        py::gil_scoped_acquire g;
        delete p;
      } else {
        (void)p->release(); // leak the reference: the interpreter is gone
        delete p;
      }
    });
    return add_recovery_hook([keep](Ctrl &c) {
      py::gil_scoped_acquire g;
      (*keep)(py::cast(&c, py::return_value_policy::reference));
    });
  }, "fn(ctrl) runs on every rank after a failed candidate if any rank aborted a run");
  m.def("remove_recovery_hook", &remove_recovery_hook);
  m.def("recover_after_abort", [](Ctrl &c) {
    py::gil_scoped_release r;
    return recover_after_abort(c);
  });
  m.def("node_identity", []() { return py::bytes(node_identity()); },
        "this machine as exchanged with IPC handles (host name | boot id, fixed size)");
  m.def("link_matrix", [](Ctrl &c, size_t bytes, int iters, double wait_limit_s) {
          LinkMatrix lm;
          {
            py::gil_scoped_release r;
            lm = link_matrix(c, bytes, iters, wait_limit_s);
          }
          py::dict d;
          d["put_GBps"] = lm.put;
          d["sdma_GBps"] = lm.sdma;
          d["bytes"] = lm.bytes;
          d["iters"] = lm.iters;
          d["why"] = lm.why;
          d["stuck"] = lm.stuck;
          return d;
        }, py::arg("ctrl"), py::arg("bytes") = size_t(32) << 20, py::arg("iters") = 10,
        py::arg("wait_limit_s") = 30.0,
        "collective all-pairs link probe: GB/s rank r -> q by kernel put and SDMA, all ranks at once");
  m.def("make_rccl_comms", &make_rccl_comms, py::arg("ctrl"), py::arg("device"), py::arg("n"),
        "n communicators over the same ranks (one per logical stream), one broadcast of ids");

  // device memory without torch (TZ_NO_TORCH runs, tests on the system ROCm runtime)
  py::class_<DeviceBuffer, std::shared_ptr<DeviceBuffer>>(m, "DeviceBuffer")
      .def(py::init([](size_t bytes) {
             TZ_CHECK(bytes > 0, "a device buffer needs at least one byte");
             return std::make_shared<DeviceBuffer>(bytes);
           }), py::arg("bytes"))
      .def_property_readonly("ptr", [](const DeviceBuffer &b) { return reinterpret_cast<uintptr_t>(b.get()); })
      .def_property_readonly("bytes", &DeviceBuffer::bytes)
      .def("zero", [](DeviceBuffer &b) { TZ_HIP(hipMemset(b.get(), 0, b.bytes())); })
      .def("to_bytes", [](const DeviceBuffer &b) {
        std::string s(b.bytes(), '\0');
        {
          py::gil_scoped_release r;
          b.download(&s[0], s.size());
        }
        return py::bytes(s);
      }, "synchronous copy of the whole buffer to the host")
      .def("from_bytes", [](DeviceBuffer &b, const py::bytes &data) {
        const std::string s = data;
        TZ_CHECK(s.size() <= b.bytes(), "from_bytes: " << s.size() << " bytes into " << b.bytes());
        b.upload(s.data(), s.size());
      });

  // ------------------------------------------------------------------ communication ops
  py::class_<CommOp, GpuOp, std::shared_ptr<CommOp>>(m, "CommOp")
      .def_property_readonly("dtype", &CommOp::dtype)
      .def_property_readonly("n_comms", [](const CommOp &o) { return o.comms().size(); });
  py::class_<SendRecvOp, CommOp, std::shared_ptr<SendRecvOp>>(m, "SendRecvOp")
      .def(py::init([](std::string name, CommSet comms, uintptr_t sb, size_t sc, int sp, uintptr_t rb,
                       size_t rc, int rp, int dt, py::object keep) {
             return std::make_shared<SendRecvOp>(std::move(name), std::move(comms), P(sb), sc, sp,
                                                 P(rb), rc, rp, dt, py_keep(std::move(keep)));
           }), py::arg("name"), py::arg("comms"), py::arg("send"), py::arg("send_count"),
           py::arg("send_peer"), py::arg("recv"), py::arg("recv_count"), py::arg("recv_peer"),
           py::arg("dtype"), py::arg("keep") = py::none());
  py::class_<AlltoallvOp, CommOp, std::shared_ptr<AlltoallvOp>>(m, "AlltoallvOp")
      .def(py::init([](std::string name, CommSet comms,
                       const std::vector<std::tuple<uintptr_t, size_t, int, uintptr_t, size_t, int>> &xs,
                       int dt, py::object keep) {
             std::vector<RcclComm::Xfer> v;
             for (const auto &t : xs)
               v.push_back({P(std::get<0>(t)), std::get<1>(t), std::get<2>(t), P(std::get<3>(t)),
                            std::get<4>(t), std::get<5>(t)});
             return std::make_shared<AlltoallvOp>(std::move(name), std::move(comms), std::move(v), dt,
                                                  py_keep(std::move(keep)));
           }), py::arg("name"), py::arg("comms"), py::arg("xfers"), py::arg("dtype"),
           py::arg("keep") = py::none(),
           "xfers: [(send, send_count, send_peer, recv, recv_count, recv_peer)]");
  py::class_<AllReduceOp, CommOp, std::shared_ptr<AllReduceOp>>(m, "AllReduceOp")
      .def(py::init([](std::string name, CommSet comms, uintptr_t sb, uintptr_t rb, size_t n, int dt,
                       int red, py::object keep) {
             return std::make_shared<AllReduceOp>(std::move(name), std::move(comms), P(sb), P(rb), n,
                                                  dt, red, py_keep(std::move(keep)));
           }), py::arg("name"), py::arg("comms"), py::arg("send"), py::arg("recv"), py::arg("count"),
           py::arg("dtype"), py::arg("red") = 0, py::arg("keep") = py::none());
  py::class_<AllGatherOp, CommOp, std::shared_ptr<AllGatherOp>>(m, "AllGatherOp")
      .def(py::init([](std::string name, CommSet comms, uintptr_t sb, uintptr_t rb, size_t n, int dt,
                       py::object keep) {
             return std::make_shared<AllGatherOp>(std::move(name), std::move(comms), P(sb), P(rb), n,
                                                  dt, py_keep(std::move(keep)));
           }), py::arg("name"), py::arg("comms"), py::arg("send"), py::arg("recv"), py::arg("count"),
           py::arg("dtype"), py::arg("keep") = py::none());
  py::class_<ReduceScatterOp, CommOp, std::shared_ptr<ReduceScatterOp>>(m, "ReduceScatterOp")
      .def(py::init([](std::string name, CommSet comms, uintptr_t sb, uintptr_t rb, size_t n, int dt,
                       int red, py::object keep) {
             return std::make_shared<ReduceScatterOp>(std::move(name), std::move(comms), P(sb), P(rb),
                                                      n, dt, red, py_keep(std::move(keep)));
           }), py::arg("name"), py::arg("comms"), py::arg("send"), py::arg("recv"),
           py::arg("recv_count"), py::arg("dtype"), py::arg("red") = 0, py::arg("keep") = py::none());
  py::class_<BroadcastOp, CommOp, std::shared_ptr<BroadcastOp>>(m, "BroadcastOp")
      .def(py::init([](std::string name, CommSet comms, uintptr_t sb, uintptr_t rb, size_t n, int root,
                       int dt, py::object keep) {
             return std::make_shared<BroadcastOp>(std::move(name), std::move(comms), P(sb), P(rb), n,
                                                  root, dt, py_keep(std::move(keep)));
           }), py::arg("name"), py::arg("comms"), py::arg("send"), py::arg("recv"), py::arg("count"),
           py::arg("root"), py::arg("dtype"), py::arg("keep") = py::none());

  // ------------------------------------------------------------------ workloads
  py::class_<HaloArgs>(m, "HaloArgs")
      .def(py::init<>())
      .def_readwrite("nx", &HaloArgs::nx)
      .def_readwrite("ny", &HaloArgs::ny)
      .def_readwrite("nz", &HaloArgs::nz)
      .def_readwrite("nq", &HaloArgs::nq)
      .def_readwrite("ghost", &HaloArgs::ghost)
      .def_readwrite("neighbors", &HaloArgs::neighbors)
      .def_readwrite("order", &HaloArgs::order)
      .def_readwrite("transport", &HaloArgs::transport)
      .def_readwrite("fuse", &HaloArgs::fuse)
      .def_readwrite("comms", &HaloArgs::comms)
      .def_readwrite("rank", &HaloArgs::rank)
      .def_readwrite("size", &HaloArgs::size)
      .def_readwrite("px", &HaloArgs::px)
      .def_readwrite("py", &HaloArgs::py)
      .def_readwrite("pz", &HaloArgs::pz)
      .def_readwrite("pitch_pad", &HaloArgs::pitch_pad)
      .def_readwrite("ghost_align", &HaloArgs::ghost_align)
      .def_readwrite("stencil", &HaloArgs::stencil)
      .def_readwrite("relay", &HaloArgs::relay)
      .def_readwrite("relay_fracs", &HaloArgs::relay_fracs)
      .def_readwrite("hostsplit", &HaloArgs::hostsplit)
      .def_readwrite("hostsplit_fracs", &HaloArgs::hostsplit_fracs)
      .def_readwrite("hostsplit_chunks", &HaloArgs::hostsplit_chunks)
      .def_readwrite("wide_puts", &HaloArgs::wide_puts)
      .def_readwrite("wide_put_blocks", &HaloArgs::wide_put_blocks)
      .def_readwrite("ipc_grid", &HaloArgs::ipc_grid)
      .def_readwrite("copy_puts", &HaloArgs::copy_puts)
      .def_readwrite("copy_engines", &HaloArgs::copy_engines)
      .def_readwrite("move_pairs", &HaloArgs::move_pairs)
      .def_readwrite("grid_memory", &HaloArgs::grid_memory)
      .def_readwrite("node_tag", &HaloArgs::node_tag)
      .def_readwrite("device", &HaloArgs::device)
      .def("json", [](const HaloArgs &a) { return a.json().dump(); });
  py::class_<HaloExchange, std::shared_ptr<HaloExchange>>(m, "HaloExchange")
      .def(py::init([](const HaloArgs &a) { return std::make_shared<HaloExchange>(a); }))
      .def_property_readonly("args", &HaloExchange::args)
      .def("ndirs", &HaloExchange::ndirs)
      .def("dir_name", [](const HaloExchange &h, int i) { return h.dir(i).name(); })
      .def("dir", [](const HaloExchange &h, int i) { auto d = h.dir(i); return py::make_tuple(d.dx, d.dy, d.dz); })
      .def("opposite", &HaloExchange::opposite)
      .def("neighbor", &HaloExchange::neighbor)
      .def("coords", &HaloExchange::coords)
      .def("rank_grid", &HaloExchange::rank_grid)
      .def("box_elems", &HaloExchange::box_elems)
      .def("pack_box", [](const HaloExchange &h, int i) { return box_to_dict(h.pack_box(i)); })
      .def("unpack_box", [](const HaloExchange &h, int i) { return box_to_dict(h.unpack_box(i)); })
      .def_static("chunk_box",
                  [](const py::dict &b, int parts) {
                    py::list out;
                    for (const kern::BoxDesc &c : HaloExchange::chunk_box(box_from_dict(b), parts))
                      out.append(box_to_dict(c));
                    return out;
                  },
                  py::arg("box"), py::arg("parts"))
      .def("grid_elems", &HaloExchange::grid_elems)
      .def("grid_memory", &HaloExchange::grid_memory, "fine or coarse (HaloArgs.grid_memory)")
      .def("off_node_dirs", &HaloExchange::off_node_dirs,
           "remote directions whose neighbour runs on another node (RCCL only)")
      .def("layout", [](const HaloExchange &h) {
             const kern::HaloGeom g = h.geom();
             py::dict d;
             d["order"] = g.order == 0 ? "xyzq" : "qxyz";
             d["x_offset_cells"] = g.xoff;   // padding before x = 0 (the first ghost cell)
             d["row_pitch_elems"] = g.sy;    // doubles per pitched row
             d["grid_bytes"] = double(h.grid_elems()) * 8.0;
             // element strides of the logical (q, z, y, x) index, x counted from the first
             // ghost cell at element offset x_offset_cells * stride x
             const bool q = g.order == 1;
             d["strides_qzyx"] = py::make_tuple(q ? 1 : g.sq, g.sz, g.sy, q ? int64_t(g.nq) : 1);
             d["shape_qzyx"] = py::make_tuple(g.nq, g.nz + 2 * g.g, g.ny + 2 * g.g, g.nx + 2 * g.g);
             d["ghost"] = g.g;
             return d;
           }, "storage layout: order, x padding before the first ghost cell, row pitch")
      .def("exchange_bytes", &HaloExchange::exchange_bytes)
      .def("setup", [](HaloExchange &h, Ctrl *c) { h.setup(c); }, py::arg("ctrl") = nullptr,
           py::call_guard<py::gil_scoped_release>())
      .def("ready", &HaloExchange::ready)
      .def("add_to_graph", &HaloExchange::add_to_graph)
      .def("grid_ptr", [](const HaloExchange &h) { return reinterpret_cast<uintptr_t>(h.grid()); })
      .def("read_grid", [](HaloExchange &h, uintptr_t dst, uintptr_t s) { h.copy_grid(P(dst), false, P(s)); },
           py::arg("dst"), py::arg("stream") = 0, "copy grid_elems() doubles of storage to dst")
      .def("write_grid", [](HaloExchange &h, uintptr_t src, uintptr_t s) { h.copy_grid(P(src), true, P(s)); },
           py::arg("src"), py::arg("stream") = 0, "overwrite the grid storage from src")
      .def("init_grid", [](HaloExchange &h, uintptr_t s, int gen) { h.init_grid(P(s), gen); },
           py::arg("stream") = 0, py::arg("gen") = 0)
      .def("check_grid", [](HaloExchange &h, uintptr_t s) { return h.check_grid(P(s)); }, py::arg("stream") = 0)
      .def("check_stencil", [](HaloExchange &h, uintptr_t s) { return h.check_stencil(P(s)); }, py::arg("stream") = 0)
      .def("stencil", [](const HaloExchange &h, int region, uintptr_t s) { h.stencil(region, P(s)); },
           py::arg("region"), py::arg("stream") = 0)
      .def("pack", [](const HaloExchange &h, int i, uintptr_t s) { h.pack(i, P(s)); })
      .def("unpack", [](const HaloExchange &h, int i, uintptr_t s) { h.unpack(i, P(s)); })
      .def("shift", [](const HaloExchange &h, int i, uintptr_t s) { h.shift(i, P(s)); })
      .def("pack_all", [](const HaloExchange &h, uintptr_t s) { h.pack_all(P(s)); })
      .def("unpack_all", [](const HaloExchange &h, uintptr_t s) { h.unpack_all(P(s)); })
      .def("shift_all", [](const HaloExchange &h, uintptr_t s) { h.shift_all(P(s)); })
      .def("direct", [](const HaloExchange &h, int i, uintptr_t s) { h.direct(i, P(s)); })
      .def("direct_group", [](const HaloExchange &h, std::vector<int> d, uintptr_t s) { h.direct_group(d, P(s)); })
      .def("direct_moves", [](const HaloExchange &h, std::vector<int> dirs) {
             py::list l;
             for (const kern::MoveDesc &m : h.direct_moves(dirs)) {
               py::dict d;
               d["src_off"] = m.src_off;
               d["dst_off"] = m.dst_off;
               d["len"] = m.len;
               d["n"] = py::make_tuple(m.n1, m.n2, m.n3);
               d["s"] = py::make_tuple(m.s1, m.s2, m.s3);
               d["pair"] = m.pair;
               // the keys kernels.box_move_many / move_kinds read (pointers 0 before setup)
               d["src"] = reinterpret_cast<uintptr_t>(m.src);
               d["dst"] = reinterpret_cast<uintptr_t>(m.dst);
               d["s1"] = m.s1;
               d["s2"] = m.s2;
               d["s3"] = m.s3;
               d["n1"] = m.n1;
               d["n2"] = m.n2;
               d["n3"] = m.n3;
               l.append(d);
             }
             return l;
           }, "the moves direct_group launches for these directions (no GPU needed)")
      .def("move_roof", &HaloExchange::move_roof, py::arg("iters") = 20, py::call_guard<py::gil_scoped_release>(),
           "the fused direct move against its shape-matched roof (same 128-B lines, whole-line "
           "accesses): us per launch of each, lines read / written, payload (re-inits the grid)")
      .def("uses_rccl", &HaloExchange::uses_rccl)
      .def("rccl_graph_ok", &HaloExchange::rccl_graph_ok, "RCCL ops may be captured into hipGraphs")
      .def("uses_direct", &HaloExchange::uses_direct)
      .def("is_direct", &HaloExchange::is_direct)
      .def("is_ipc", &HaloExchange::is_ipc)
      .def("uses_ipc", &HaloExchange::uses_ipc)
      .def("uses_relay", &HaloExchange::uses_relay)
      .def("uses_hostsplit", &HaloExchange::uses_hostsplit)
      .def("uses_wide_puts", &HaloExchange::uses_wide_puts)
      .def_static("wide_puts_offered", &HaloExchange::wide_puts_offered, py::arg("mode"),
                  py::arg("my_bus"), py::arg("peer_buses"), py::arg("my_device"),
                  py::arg("mapped_devices"))
      .def("hostsplit_parts", &HaloExchange::hs_parts, py::arg("frac"))
      .def("relay_faces", &HaloExchange::relay_faces)
      .def("link_probe", [](HaloExchange &h, int dir, const std::string &via, int iters, Ctrl *c) {
             return h.link_probe(dir, via, iters, c);
           }, py::arg("dir"), py::arg("via"), py::arg("iters"), py::arg("ctrl"),
           py::call_guard<py::gil_scoped_release>())
      .def("ipc_mode", &HaloExchange::ipc_mode)
      .def("put_group", [](const HaloExchange &h, std::vector<int> d, uintptr_t s, int maxBlocks) {
             h.put_group(d, P(s), maxBlocks);
           }, py::arg("dirs"), py::arg("stream"), py::arg("max_blocks") = 0)
      .def("wait_group", [](const HaloExchange &h, std::vector<int> d, uintptr_t s) { h.wait_group(d, P(s)); })
      .def("ipc_errors", &HaloExchange::ipc_errors, py::call_guard<py::gil_scoped_release>())
      .def("pipelined_dirs", &HaloExchange::pipelined_dirs)
      .def("uses_host", &HaloExchange::uses_host)
      .def("rccl_nranks", &HaloExchange::rccl_nranks)
      .def("transport_report", &HaloExchange::transport_report)
      .def("ipc_peer_devices", &HaloExchange::ipc_peer_devices,
           "peer rank -> device its IPC-mapped memory reports (hipPointerGetAttributes)")
      .def("reset_transport_state", &HaloExchange::reset_transport_state, py::arg("ctrl"),
           py::call_guard<py::gil_scoped_release>())
      .def("host_exchange", &HaloExchange::host_exchange, py::call_guard<py::gil_scoped_release>())
      .def("transport", &HaloExchange::transport);

  py::class_<SpmvArgs>(m, "SpmvArgs")
      .def(py::init<>())
      .def_readwrite("matrix", &SpmvArgs::matrix)
      .def_readwrite("m", &SpmvArgs::m)
      .def_readwrite("distribute", &SpmvArgs::distribute)
      .def_readwrite("bw", &SpmvArgs::bw)
      .def_readwrite("nnz", &SpmvArgs::nnz)
      .def_readonly("nnz_actual", &SpmvArgs::nnz_actual)
      .def_readwrite("seed", &SpmvArgs::seed)
      .def_readwrite("rank", &SpmvArgs::rank)
      .def_readwrite("size", &SpmvArgs::size)
      .def_readwrite("device", &SpmvArgs::device)
      .def_readwrite("compound", &SpmvArgs::compound)
      .def_readwrite("kernel_choice", &SpmvArgs::kernel_choice)
      .def_readwrite("form", &SpmvArgs::form)
      .def_readwrite("library", &SpmvArgs::library)
      .def_readwrite("transport", &SpmvArgs::transport)
      .def_readwrite("prefix", &SpmvArgs::prefix)
      .def("json", [](const SpmvArgs &a) { return a.json().dump(); });
  py::class_<DistSpmv, std::shared_ptr<DistSpmv>>(m, "DistSpmv")
      .def(py::init([](const SpmvArgs &a, Ctrl *c) {
             py::gil_scoped_release r; // collective with "root" distribution
             return std::make_shared<DistSpmv>(a, c);
           }), py::arg("args"), py::arg("ctrl") = nullptr)
      .def_property_readonly("args", &DistSpmv::args)
      .def("local_rows", &DistSpmv::local_rows)
      .def("local_nnz", &DistSpmv::local_nnz)
      .def("remote_nnz", &DistSpmv::remote_nnz)
      .def("remote_cols", &DistSpmv::remote_cols)
      .def("send_elems", &DistSpmv::send_elems)
      .def("num_peers", &DistSpmv::num_peers)
      .def("transport", &DistSpmv::transport)
      .def("uses_ipc", &DistSpmv::uses_ipc)
      .def("uses_rccl", &DistSpmv::uses_rccl)
      .def("rccl_graph_ok", &DistSpmv::rccl_graph_ok, "RCCL exchanges may be captured into hipGraphs")
      .def("rccl_capture_note", &DistSpmv::rccl_capture_note,
           "how the RCCL exchange is compiled into hipGraphs (its preflight's verdict), or why not")
      .def("ipc_errors", &DistSpmv::ipc_errors, py::call_guard<py::gil_scoped_release>())
      .def("setup", [](DistSpmv &s, Ctrl *c) { s.setup(c); }, py::arg("ctrl") = nullptr,
           py::call_guard<py::gil_scoped_release>())
      .def("ready", &DistSpmv::ready)
      .def("add_to_graph", &DistSpmv::add_to_graph)
      .def("op_graph", [](DistSpmv &s) { return std::const_pointer_cast<Graph>(s.op_graph()); })
      .def("check", [](DistSpmv &s, uintptr_t st) { return s.check(P(st)); }, py::arg("stream") = 0)
      .def("reset_y", [](DistSpmv &s, uintptr_t st) { s.reset_y(P(st)); }, py::arg("stream") = 0);
  m.def("move_spmv_op", [](std::shared_ptr<HaloExchange> h, std::vector<int> dirs, std::shared_ptr<DistSpmv> s,
                           std::string name, int lanes, bool intoY) {
    return make_move_spmv_op(h, std::move(dirs), s, std::move(name), lanes, intoY);
  }, py::arg("halo"), py::arg("dirs"), py::arg("spmv"), py::arg("name"), py::arg("lanes") = kern::kSpmvIlp + 4,
     py::arg("into_y") = true,
     "one GPU op running the halo's self moves `dirs` and the SpMV's local product in one kernel "
     "(horizontal fusion; the SpMV's workgroups interleaved among the move's)");
  m.def("random_band_matrix", [](int64_t n, int64_t bw, int64_t nnz, uint64_t seed) {
    CsrHost a = random_band_matrix(n, bw, nnz, seed);
    return py::make_tuple(a.rowPtr, a.colInd, a.val);
  });
  m.def("read_matrix_market", [](const std::string &path) {
    CsrHost a = read_matrix_market(path);
    return py::make_tuple(a.rows, a.cols, a.rowPtr, a.colInd, a.val);
  }, py::arg("path"));
  m.def("write_matrix_market", [](int64_t rows, int64_t cols, std::vector<int32_t> rowPtr,
                                  std::vector<int32_t> colInd, std::vector<float> val,
                                  const std::string &path) {
    CsrHost a;
    a.rows = rows;
    a.cols = cols;
    a.rowPtr = std::move(rowPtr);
    a.colInd = std::move(colInd);
    a.val = std::move(val);
    TZ_CHECK(int64_t(a.rowPtr.size()) == rows + 1 && a.colInd.size() == a.val.size() &&
                 int64_t(a.colInd.size()) == int64_t(a.rowPtr.back()),
             "inconsistent CSR arrays");
    write_matrix_market(a, path);
  }, py::arg("rows"), py::arg("cols"), py::arg("row_ptr"), py::arg("col_ind"), py::arg("val"), py::arg("path"));
  m.def("row_partition", &row_partition);

  // ------------------------------------------------------------------ raw kernels
  auto k = m.def_submodule("kernels", "hand-written gfx950 kernels (raw device pointers)");
  k.def("box_copy", [](uintptr_t grid, py::dict d, bool unpack, uintptr_t s) {
    kern::box_copy(reinterpret_cast<double *>(grid), box_from_dict(d), unpack, P(s));
  }, py::arg("grid"), py::arg("box"), py::arg("unpack"), py::arg("stream") = 0);
  k.def("box_copy_many", [](uintptr_t grid, std::vector<py::dict> ds, bool unpack, uintptr_t s) {
    std::vector<kern::BoxDesc> bs;
    for (auto &d : ds) bs.push_back(box_from_dict(d));
    kern::box_copy_many(reinterpret_cast<double *>(grid), bs.data(), int(bs.size()), unpack, P(s));
  }, py::arg("grid"), py::arg("boxes"), py::arg("unpack"), py::arg("stream") = 0);
  k.def("csr_spmv", [](int n, uintptr_t rp, uintptr_t ci, uintptr_t v, uintptr_t x, uintptr_t y, int lanes, bool acc, uintptr_t s) {
    kern::csr_spmv(n, reinterpret_cast<const int32_t *>(rp), reinterpret_cast<const int32_t *>(ci),
                   reinterpret_cast<const float *>(v), reinterpret_cast<const float *>(x),
                   reinterpret_cast<float *>(y), lanes, acc, P(s));
  }, py::arg("n_rows"), py::arg("row_ptr"), py::arg("col_ind"), py::arg("val"), py::arg("x"), py::arg("y"),
     py::arg("lanes") = 0, py::arg("accumulate") = false, py::arg("stream") = 0);
  py::class_<RocsparseCsr, std::shared_ptr<RocsparseCsr>>(
      k, "RocsparseCsr", "rocSPARSE CSR SpMV (library comparison variant): y = A x on raw pointers")
      .def(py::init([](int64_t m, int64_t n, int64_t nnz, uintptr_t rp, uintptr_t ci, uintptr_t v,
                       uintptr_t x, uintptr_t y, const std::string &alg) {
             return std::make_shared<RocsparseCsr>(
                 m, n, nnz, reinterpret_cast<const int32_t *>(rp), reinterpret_cast<const int32_t *>(ci),
                 reinterpret_cast<const float *>(v), reinterpret_cast<const float *>(x),
                 reinterpret_cast<float *>(y), alg.c_str());
           }),
           py::arg("m"), py::arg("n"), py::arg("nnz"), py::arg("row_ptr"), py::arg("col_ind"),
           py::arg("val"), py::arg("x"), py::arg("y"), py::arg("alg") = "adaptive")
      .def("run", [](const RocsparseCsr &r, uintptr_t s, bool acc) { r.run(P(s), acc); },
           py::arg("stream") = 0, py::arg("accumulate") = false);
  k.def("stencil7", [](uintptr_t in, uintptr_t out, int64_t base, int row, int ny, int nz,
                       int nouter, int64_t sy, int64_t sz, int64_t so, int xs, double c0, double c1,
                       bool lds, uintptr_t s) {
    kern::StencilBox b;
    b.in = reinterpret_cast<const double *>(in);
    b.out = reinterpret_cast<double *>(out);
    b.base = base;
    b.row = row;
    b.ny = ny;
    b.nz = nz;
    b.nouter = nouter;
    b.sy = sy;
    b.sz = sz;
    b.so = so;
    b.xs = xs;
    b.c0 = c0;
    b.c1 = c1;
    kern::stencil7(b, lds, P(s));
  }, py::arg("in_"), py::arg("out"), py::arg("base"), py::arg("row"), py::arg("ny"), py::arg("nz"),
     py::arg("nouter"), py::arg("sy"), py::arg("sz"), py::arg("so"), py::arg("xs"),
     py::arg("c0") = 0.4, py::arg("c1") = 0.1, py::arg("lds") = true, py::arg("stream") = 0);
  k.def("set_stencil_tuning", [](int ty, int zc, int pf, bool db) {
    TZ_CHECK(ty == 8 || ty == 16, "stencil ty must be 8 or 16");
    TZ_CHECK(zc == 16 || zc == 32 || zc == 64 || zc == 128, "stencil zc must be 16, 32, 64 or 128");
    TZ_CHECK(zc != 128 || pf == 1, "stencil zc 128 takes pf 1");
    TZ_CHECK(pf == 1 || pf == 2, "stencil pf must be 1 or 2");
    kern::stencil_tuning().ty = ty;
    kern::stencil_tuning().zc = zc;
    kern::stencil_tuning().pf = pf;
    kern::stencil_tuning().db = db;
  }, py::arg("ty") = 16, py::arg("zc") = 64, py::arg("pf") = 1, py::arg("db") = true);
  k.def("set_stencil_xcd_tiles", [](bool on) { kern::stencil_tuning().xcd_tiles = on; }, py::arg("on"),
        "stencil tiles in XCD-contiguous order (each XCD a contiguous range of tiles)");
  k.def("get_stencil_xcd_tiles", []() { return kern::stencil_tuning().xcd_tiles; });
  k.def("gather_f32", [](int n, uintptr_t src, uintptr_t idx, uintptr_t dst, uintptr_t s) {
    kern::gather_f32(n, reinterpret_cast<const float *>(src), reinterpret_cast<const int32_t *>(idx),
                     reinterpret_cast<float *>(dst), P(s));
  }, py::arg("n"), py::arg("src"), py::arg("idx"), py::arg("dst"), py::arg("stream") = 0);
  k.def("vector_add_f32", [](int n, uintptr_t a, uintptr_t b, uintptr_t y, uintptr_t s) {
    kern::vector_add_f32(n, reinterpret_cast<const float *>(a), reinterpret_cast<const float *>(b),
                         reinterpret_cast<float *>(y), P(s));
  }, py::arg("n"), py::arg("a"), py::arg("b"), py::arg("y"), py::arg("stream") = 0);
  k.def("axpy_f64", [](int64_t n, double alpha, uintptr_t x, uintptr_t y, uintptr_t s) {
    kern::axpy_f64(n, alpha, reinterpret_cast<const double *>(x), reinterpret_cast<double *>(y), P(s));
  }, py::arg("n"), py::arg("alpha"), py::arg("x"), py::arg("y"), py::arg("stream") = 0);
  k.def("iota_f64", [](int64_t n, double base, double scale, uintptr_t a, uintptr_t s) {
    kern::iota_f64(n, base, scale, reinterpret_cast<double *>(a), P(s));
  }, py::arg("n"), py::arg("base"), py::arg("scale"), py::arg("a"), py::arg("stream") = 0);
  k.def("empty", [](uintptr_t s) { kern::empty(P(s)); }, py::arg("stream") = 0);
  auto moves_from = [](const std::vector<py::dict> &ds) {
    std::vector<kern::MoveDesc> ms;
    for (auto &d : ds) {
      kern::MoveDesc m;
      m.src = reinterpret_cast<const double *>(d["src"].cast<uintptr_t>());
      m.dst = reinterpret_cast<double *>(d["dst"].cast<uintptr_t>());
      m.src_off = d["src_off"].cast<int64_t>();
      m.dst_off = d["dst_off"].cast<int64_t>();
      m.s1 = d.contains("s1") ? d["s1"].cast<int64_t>() : 0;
      m.s2 = d.contains("s2") ? d["s2"].cast<int64_t>() : 0;
      m.s3 = d.contains("s3") ? d["s3"].cast<int64_t>() : 0;
      m.len = d["len"].cast<int32_t>();
      m.n1 = d.contains("n1") ? d["n1"].cast<int32_t>() : 1;
      m.n2 = d.contains("n2") ? d["n2"].cast<int32_t>() : 1;
      m.n3 = d.contains("n3") ? d["n3"].cast<int32_t>() : 1;
      m.pair = d.contains("pair") && d["pair"].cast<bool>();
      ms.push_back(m);
    }
    return ms;
  };
  k.def("box_move_spmv", [moves_from](std::vector<py::dict> ds, int n, uintptr_t rp, uintptr_t ci, uintptr_t v,
                                      uintptr_t x, uintptr_t y, int lanes, bool acc, uintptr_t s) {
    const std::vector<kern::MoveDesc> ms = moves_from(ds);
    kern::SpmvJob j;
    j.nRows = n;
    j.rowPtr = reinterpret_cast<const int32_t *>(rp);
    j.colInd = reinterpret_cast<const int32_t *>(ci);
    j.val = reinterpret_cast<const float *>(v);
    j.x = reinterpret_cast<const float *>(x);
    j.y = reinterpret_cast<float *>(y);
    j.lanes = lanes;
    j.accumulate = acc;
    kern::box_move_spmv(ms.data(), int(ms.size()), j, P(s));
  }, py::arg("moves"), py::arg("n_rows"), py::arg("row_ptr"), py::arg("col_ind"), py::arg("val"),
     py::arg("x"), py::arg("y"), py::arg("lanes") = kern::kSpmvIlp + 4, py::arg("accumulate") = false,
     py::arg("stream") = 0,
     "the direct moves (as box_move_many) and one ILP CSR SpMV in one launch, workgroups interleaved");
  k.def("move_kinds", [moves_from](std::vector<py::dict> ds) {
    const std::vector<kern::MoveDesc> ms = moves_from(ds);
    return kern::move_kinds(ms.data(), int(ms.size()));
  }, py::arg("moves"), "how box_move_many would move each box (no GPU needed)");
  k.def("box_move_many", [moves_from](std::vector<py::dict> ds, uintptr_t s) {
    const std::vector<kern::MoveDesc> ms = moves_from(ds);
    kern::box_move_many(ms.data(), int(ms.size()), P(s));
  }, py::arg("moves"), py::arg("stream") = 0);
  k.def("set_box_tuning", [](int unroll, bool ntPack, bool ntUnpack, int maxBlocks, bool ntMove) {
    TZ_CHECK(unroll >= 1 && unroll <= 64, "unroll must be 1..64");
    TZ_CHECK(maxBlocks >= 1, "max_blocks must be positive");
    kern::box_tuning().unroll = unroll;
    kern::box_tuning().nt_pack = ntPack;
    kern::box_tuning().nt_unpack = ntUnpack;
    kern::box_tuning().max_blocks = maxBlocks;
    kern::box_tuning().nt_move = ntMove;
  }, py::arg("unroll") = 3, py::arg("nt_pack") = true, py::arg("nt_unpack") = true,
     py::arg("max_blocks") = 4096, py::arg("nt_move") = false);
  k.def("set_xcd_remap", &kern::set_xcd_remap, py::arg("mode"));
  k.def("set_put_max_blocks", [](int b) {
    TZ_CHECK(b >= 1, "put_max_blocks must be positive");
    kern::box_tuning().put_max_blocks = b;
  }, py::arg("blocks"));
  k.def("get_put_max_blocks", []() { return kern::box_tuning().put_max_blocks; });
  k.def("set_nt_move_store", [](bool on) { kern::box_tuning().nt_move_store = on; }, py::arg("on"));
  k.def("get_nt_move_store", []() { return kern::box_tuning().nt_move_store; });
  k.def("get_xcd_remap", []() { return kern::box_tuning().xcd_remap; });
  k.def("set_move_unroll", [](int u) {
    TZ_CHECK(u == 1 || u == 2 || u == 4, "move_unroll must be 1, 2 or 4");
    kern::box_tuning().move_unroll = u;
  }, py::arg("unroll"));
  k.def("get_move_unroll", []() { return kern::box_tuning().move_unroll; });
  k.def("set_move_items", [](int n) {
    TZ_CHECK(n >= 1 && n <= 64, "move_items must be 1..64");
    kern::box_tuning().move_items = n;
  }, py::arg("items"));
  k.def("get_move_items", []() { return kern::box_tuning().move_items; });
  k.def("set_peel_moves", [](bool on) { kern::box_tuning().peel_moves = on; }, py::arg("on"),
        "moves of rows one element past a 16-B boundary: peel it and move the rest 16 B at a time");
  k.def("get_peel_moves", []() { return kern::box_tuning().peel_moves; });
  k.def("set_widen_unpack", [](bool on) { kern::box_tuning().widen_unpack = on; }, py::arg("on"),
        "unpack boxes with lead / trail write their widened rows with 16-B stores");
  k.def("get_widen_unpack", []() { return kern::box_tuning().widen_unpack; });
  k.def("get_box_tuning", []() {
    const auto &t = kern::box_tuning();
    return py::make_tuple(t.unroll, t.nt_pack, t.nt_unpack, t.max_blocks, t.nt_move);
  });
  k.def("copy_bytes", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s) {
    kern::copy_bytes(P(dst), P(src), n, P(s));
  }, py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream") = 0);
  k.def("busy_wait", [](int64_t t, int b, uintptr_t s) { kern::busy_wait(t, b, P(s)); },
        py::arg("ticks"), py::arg("blocks") = 1, py::arg("stream") = 0);
}
