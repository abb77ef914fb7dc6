// tz-search: standalone native driver (no Python) — the MI355X counterpart of the reference's
// example executables halo-mcts-min-time / halo-mcts-coverage / spmv-{random,min-time,coverage}
// (tenzing-mcts/examples/*.cu) and tenzing-dfs/examples/spmv.cu, behind one CLI.
//
//   tz-search --workload halo --solver mcts --strategy FastMin --iters 100 --streams 4
//   torchrun --nproc-per-node 8 ... tz-search (one process per GPU; RANK/WORLD_SIZE/LOCAL_RANK)
//   mpirun -n 8 tz-search ...                 (the reference's launch; control plane over MPI)
//
// Under torchrun the control plane rendezvouses on MASTER_ADDR, rank 0 listening on the first
// free of 8 ports from MASTER_PORT + 1 (TZ_CTRL_PORT / TZ_CTRL_PORTS as in Python), or through a
// file (--rdzv-file, single node; the default without MASTER_PORT); under an MPI launcher it is
// MPI_COMM_WORLD (--ctrl mpi, picked automatically). The data plane is RCCL / IPC puts either way.
#include "core/solve.hpp"
#include "hip/hip_runtime.hpp"
#include "workloads/workloads.hpp"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>

using namespace tz;

namespace {

struct Args {
  std::map<std::string, std::string> kv;
  std::vector<std::string> raw;
  std::string get(const std::string &k, const std::string &d) const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  double num(const std::string &k, double d) const {
    auto it = kv.find(k);
    return it == kv.end() ? d : std::stod(it->second);
  }
  bool flag(const std::string &k) const { return kv.count(k) > 0; }
};

int env_int(const char *a, const char *b, int d) {
  if (const char *e = std::getenv(a)) return std::atoi(e);
  if (b)
    if (const char *e = std::getenv(b)) return std::atoi(e);
  return d;
}

void usage() {
  std::cerr
      << "usage: tz-search [--workload halo|spmv|halo+spmv|diamond] [--solver mcts|dfs]\n"
         "  [--strategy NAME] [--iters N] [--time-budget S] [--max-tree-nodes N] [--streams N] [--bench-iters N]\n"
         "  [--target-secs S] [--mode eager|graph] [--sim] [--seed N] [--no-expand-rollout]\n"
         "  [--halo-n N] [--nq N] [--ghost N] [--neighbors 6|26] [--order xyzq|qxyz]\n"
         "  [--fuse none|pack|all|groups|choice] [--graph-unroll K]\n"
         "  [--transport auto|rccl|ipc|copy|direct] [--rank-grid PXxPYxPZ] [--spmv-m N] [--spmv-matrix F.mtx]\n"
         "  [--spmv-form choice|split|accum] [--spmv-transport auto|rccl|ipc] [--spmv-distribute auto|root|local]\n"
         "  [--spmv-library adaptive|lrb|rowsplit|''] [--cu-partition] [--stencil] [--max-seqs N]\n"
         "  [--relay auto|off|force] [--relay-fracs F1,F2]\n"
         "  [--hostsplit auto|off|force] [--hostsplit-fracs F1,F2,...] [--hostsplit-chunks N]\n"
         "  [--wide-puts auto|on|off] [--wide-put-blocks N]\n"
         "  [--ipc-grid auto|0|1] [--copy-puts on|off] [--copy-engines N] [--move-pairs on|off]\n"
         "  [--grid-memory auto|coarse|fine]\n"
         "  [--horizontal on|off]   halo+spmv on one rank: offer the move + SpMV as one launch\n"
         "  [--ctrl auto|tcp|mpi|self] [--mpi-lib PATH] [--rdzv-file PATH]\n"
         "  [--master-addr HOST] [--csv PATH] [--jsonl PATH] [--dump-graph PATH] [--dump-tree]\n"
         "  [--checkpoint PATH] [--resume PATH] [--seed-schedule PATH] [--watchdog S]\n"
         "  [--deadline S]          past S seconds print the partial results CSV and exit 5\n"
         "  [--race-ratio R] [--settle-ratio R]\n"
         "  [--save-best PATH]      write the best schedule + workload options (JSON)\n"
         "  [--run PATH [--run-iters N] [--run-warmup N]]\n"
         "                          run a saved schedule (this CLI's or python -m tenzing_amd's)\n"
         "                          without searching: verified race-free, checked, timed\n";
}

/// python-style option key ("halo_n") of a CLI option ("halo-n")
std::string py_key(std::string k) {
  for (char &c : k)
    if (c == '-') c = '_';
  return k;
}

/// options of a saved schedule document -> this CLI's options (the document may come from
/// `tz-search --save-best` or `python -m tenzing_amd search --save-best`)
void load_saved_args(const Json &args, Args &a) {
  for (const auto &kv : args.as_object()) {
    std::string k = kv.first;
    for (char &c : k)
      if (c == '_') c = '-';
    const Json &v = kv.second;
    if (v.is_bool()) {
      if (v.as_bool()) a.kv[k] = "1";
      else a.kv.erase(k);
    } else if (v.is_string()) {
      if (v.as_string().empty()) a.kv.erase(k);
      else a.kv[k] = v.as_string();
    } else {
      a.kv[k] = v.dump();
    }
  }
  if (a.get("workload", "") == "fused") a.kv["workload"] = "halo+spmv";
}

} // namespace

int main(int argc, char **argv) {
  Args a;
  for (int i = 1; i < argc; ++i) a.raw.push_back(argv[i]);
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s == "-h" || s == "--help") {
      usage();
      return 0;
    }
    if (s.rfind("--", 0) != 0) {
      std::cerr << "unexpected argument " << s << "\n";
      usage();
      return 2;
    }
    s = s.substr(2);
    auto eq = s.find('=');
    if (eq != std::string::npos) {
      a.kv[s.substr(0, eq)] = s.substr(eq + 1);
    } else if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) {
      a.kv[s] = argv[++i];
    } else {
      a.kv[s] = "1";
    }
  }
  try {
    Json saved;
    if (a.flag("run")) {
      std::ifstream f(a.get("run", ""));
      TZ_CHECK(f, "cannot open " << a.get("run", ""));
      std::stringstream ss;
      ss << f.rdbuf();
      saved = Json::parse(ss.str());
      load_saved_args(saved.at("args"), a);
      // a schedule that uses the wide put needs it offered again wherever it runs now
      if (saved.contains("schedule") && saved.at("schedule").dump().find("he_putw_") != std::string::npos)
        a.kv["wide-puts"] = "on";
      if (!a.flag("mode") && saved.contains("mode")) a.kv["mode"] = saved.at("mode").as_string();
      TZ_CHECK(!a.flag("sim"), "--run needs a GPU");
    }
    // control plane: --ctrl mpi for ranks started by mpirun / srun (the reference's launch
    // model), tcp for torchrun-style RANK / WORLD_SIZE; auto picks mpi when an MPI launcher
    // started this process and no WORLD_SIZE is set
    std::string ctrlKind = a.get("ctrl", "auto");
    TZ_CHECK(ctrlKind == "auto" || ctrlKind == "tcp" || ctrlKind == "mpi" || ctrlKind == "self",
             "--ctrl must be auto, tcp, mpi or self");
    if (ctrlKind == "auto")
      ctrlKind = !std::getenv("WORLD_SIZE") && MpiCtrl::launched() ? "mpi" : "tcp";
    std::shared_ptr<Ctrl> ctrl;
    int rank = env_int("RANK", "OMPI_COMM_WORLD_RANK", 0);
    int size = env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", 1);
    int local = env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", rank);
    if (ctrlKind == "mpi") {
      auto m = std::make_shared<MpiCtrl>(a.get("mpi-lib", ""));
      rank = m->rank();
      size = m->size();
      local = MpiCtrl::launcher_local_rank() >= 0 ? MpiCtrl::launcher_local_rank() : rank;
      ctrl = m;
    } else if (ctrlKind == "self") {
      rank = 0;
      size = 1;
    }
    log_rank() = rank;
    const bool sim = a.flag("sim");
    const int streams = int(a.num("streams", 2));
    const std::string workload = a.get("workload", "halo");

    if (!ctrl && size > 1) {
      auto t = std::make_shared<TcpCtrl>(rank, size);
      const char *mp = std::getenv("MASTER_PORT");
      const char *ma = std::getenv("MASTER_ADDR");
      const std::string host = a.get("master-addr", ma ? ma : "127.0.0.1");
      if (mp && !a.flag("rdzv-file")) {
        const int base = std::getenv("TZ_CTRL_PORT") ? std::atoi(std::getenv("TZ_CTRL_PORT")) : std::atoi(mp) + 1;
        const int nports = std::getenv("TZ_CTRL_PORTS") ? std::atoi(std::getenv("TZ_CTRL_PORTS")) : 8;
        t->rendezvous(host, base, 300.0, nports);
      } else {
        t->rendezvous_file(a.get("rdzv-file", std::string("/tmp/tz_rdzv_") + (mp ? mp : "default")), host);
      }
      ctrl = t;
    } else if (!ctrl) {
      ctrl = std::make_shared<SelfCtrl>();
    }
    if (rank == 0) std::cerr << reproduce_json(a.raw).dump() << "\n";

    int device = -1;
    if (!sim) {
      const int n = hip_device_count();
      TZ_CHECK(n > 0, "no GPU visible (use --sim for a hardware-free search)");
      device = local % n;
      TZ_HIP(hipSetDevice(device));
    }

    if (a.flag("run")) {
      const int64_t want = saved.at("ranks").as_int();
      TZ_CHECK(want == size, "schedule was searched on " << want << " ranks, this run has " << size);
    }
    // the workload options in effect (python-style keys: what --save-best records)
    Json wargs = Json::object();
    auto opt = [&](const std::string &k, const std::string &d) {
      const std::string v = a.get(k, d);
      wargs[py_key(k)] = v;
      return v;
    };
    auto optn = [&](const std::string &k, double d) {
      const double v = a.num(k, d);
      if (v == std::floor(v) && std::fabs(v) < 9e15) wargs[py_key(k)] = int64_t(v);
      else wargs[py_key(k)] = v;
      return v;
    };
    auto optf = [&](const std::string &k) {
      const bool v = a.flag(k);
      wargs[py_key(k)] = v;
      return v;
    };
    wargs["workload"] = workload;
    wargs["streams"] = streams;
    auto g = std::make_shared<Graph>();
    std::shared_ptr<HaloExchange> halo;
    std::shared_ptr<DistSpmv> spmv;
    if (workload == "halo" || workload == "halo+spmv") {
      HaloArgs h;
      h.nx = h.ny = h.nz = int(optn("halo-n", 512));
      h.nq = int(optn("nq", 3));
      h.ghost = int(optn("ghost", 3));
      h.neighbors = int(optn("neighbors", 6));
      h.fuse = opt("fuse", "none");
      h.transport = opt("transport", "auto");
      h.order = opt("order", "xyzq");
      h.stencil = optf("stencil");
      h.relay = opt("relay", "auto");
      {
        // comma-separated relayed shares, e.g. 0.15,0.2
        const std::string fr = opt("relay-fracs", "0.15,0.2,0.25");
        if (!fr.empty()) {
          h.relay_fracs.clear();
          std::stringstream ss(fr);
          std::string tok;
          while (std::getline(ss, tok, ',')) h.relay_fracs.push_back(std::stod(tok));
        }
      }
      h.hostsplit = opt("hostsplit", "auto");
      {
        // comma-separated host shares, e.g. 0.2,0.3,0.4
        const std::string fr = opt("hostsplit-fracs", "0.1,0.2,0.3,0.4");
        if (!fr.empty()) {
          h.hostsplit_fracs.clear();
          std::stringstream ss(fr);
          std::string tok;
          while (std::getline(ss, tok, ',')) h.hostsplit_fracs.push_back(std::stod(tok));
        }
      }
      h.hostsplit_chunks = std::stoi(opt("hostsplit-chunks", "1"));
      h.wide_puts = opt("wide-puts", "auto");
      h.wide_put_blocks = int(optn("wide-put-blocks", 256));
      {
        const std::string ig = opt("ipc-grid", "auto");
        TZ_CHECK(ig == "auto" || ig == "0" || ig == "1", "--ipc-grid must be auto, 0 or 1");
        h.ipc_grid = ig == "auto" ? -1 : std::stoi(ig);
        const std::string cp = opt("copy-puts", "on");
        TZ_CHECK(cp == "on" || cp == "off", "--copy-puts must be on or off");
        h.copy_puts = cp == "on";
        h.copy_engines = int(optn("copy-engines", 1));
        const std::string mp = opt("move-pairs", "on");
        TZ_CHECK(mp == "on" || mp == "off", "--move-pairs must be on or off");
        h.move_pairs = mp == "on";
        const std::string gm = opt("grid-memory", "auto");
        TZ_CHECK(gm == "auto" || gm == "coarse" || gm == "fine", "--grid-memory must be auto, coarse or fine");
        h.grid_memory = gm == "auto" ? -1 : gm == "fine" ? 1 : 0;
      }
      TZ_CHECK(h.order == "xyzq" || h.order == "qxyz", "--order must be xyzq or qxyz");
      h.rank = rank;
      h.size = size;
      const std::string rg = opt("rank-grid", "");
      if (!rg.empty()) {
        TZ_CHECK(std::sscanf(rg.c_str(), "%dx%dx%d", &h.px, &h.py, &h.pz) == 3,
                 "--rank-grid must look like 2x2x2");
      }
      halo = std::make_shared<HaloExchange>(h);
      if (!sim) halo->setup(ctrl.get());
      halo->add_to_graph(*g);
    }
    if (workload == "spmv" || workload == "halo+spmv") {
      SpmvArgs s;
      s.m = int64_t(optn("spmv-m", 150000));
      s.matrix = opt("spmv-matrix", "");
      s.rank = rank;
      s.size = size;
      s.prefix = workload == "halo+spmv" ? "spmv_" : "";
      s.form = opt("spmv-form", "choice");
      s.transport = opt("spmv-transport", "auto");
      s.library = opt("spmv-library", "adaptive");
      s.distribute = opt("spmv-distribute", "auto");
      spmv = std::make_shared<DistSpmv>(s, ctrl.get());
      if (!sim) spmv->setup(ctrl.get());
      spmv->add_to_graph(*g);
    }
    if (workload == "halo+spmv") {
      // horizontal fusion, as the Python builder (tenzing_amd/models/fused.py): on one rank with
      // every halo direction a self move, a top-level choice between the two workloads' own ops
      // and one launch running the move and the SpMV's local product together
      const std::string hz = opt("horizontal", "on");
      TZ_CHECK(hz == "on" || hz == "off", "--horizontal must be on or off");
      std::vector<int> direct;
      for (int i = 0; i < halo->ndirs(); ++i)
        if (halo->is_direct(i)) direct.push_back(i);
      if (hz == "on" && size == 1 && int(direct.size()) == halo->ndirs() && !halo->args().stencil) {
        std::vector<OpPtr> alts = {std::make_shared<StaticCompoundOp>("hs_separate", g)};
        for (int w : {4, 2})
          alts.push_back(make_move_spmv_op(halo, direct, spmv, "hs_onelaunch_i" + std::to_string(w),
                                           kern::kSpmvIlp + w, true));
        auto top = std::make_shared<StaticChoiceOp>("hs_launches", alts);
        g = std::make_shared<Graph>();
        g->start_then(top);
        g->then_finish(top);
      }
    }
    if (workload == "diamond") {
      auto k1 = std::make_shared<BusyKernelOp>("k1", 20), k2 = std::make_shared<BusyKernelOp>("k2", 100),
           k3 = std::make_shared<BusyKernelOp>("k3", 100), k4 = std::make_shared<BusyKernelOp>("k4", 20);
      g->start_then(k1);
      g->then(k1, k2);
      g->then(k1, k3);
      g->then(k2, k4);
      g->then(k3, k4);
      g->then_finish(k4);
    }
    TZ_CHECK(g->size() > 2, "unknown workload " << workload);
    if (rank == 0 && a.flag("dump-graph")) {
      std::ofstream f(a.get("dump-graph", "graph.dot"));
      f << g->dump_graphviz(workload);
    }

    Platform plat = Platform::make_n_streams(streams);
    // CU-partitioned streams are distinguishable resources: no symmetric-stream pruning
    if (optf("cu-partition")) plat.symmetric_streams = false;
    std::unique_ptr<HipRuntime> rt;
    std::unique_ptr<Benchmarker> bench;
    if (sim) {
      SimParams sp;
      sp.graph = a.get("mode", "eager") == "graph"; // a replayed hipGraph's measured costs
      bench = std::make_unique<SimBenchmarker>(streams, sp);
    } else {
      HipRuntimeOpts ro;
      ro.n_streams = streams;
      ro.mode = a.get("mode", "eager") == "graph" ? ExecMode::Graph : ExecMode::Eager;
      ro.watchdog_s = a.num("watchdog", 30); // floor; + 50 x n x expected per run
      ro.graph_unroll = int(a.num("graph-unroll", a.flag("run") ? 20 : 1));
      ro.cu_partition = a.flag("cu-partition");
      rt = std::make_unique<HipRuntime>(ro);
      bench = std::make_unique<EmpiricalBenchmarker>(*rt, *ctrl);
    }
    BenchOpts bo;
    bo.n_iters = int64_t(a.num("bench-iters", 50));
    bo.target_secs = a.num("target-secs", 0.01);
    bo.race_ratio = a.num("race-ratio", 0.0);
    bo.settle_ratio = a.num("settle-ratio", 0.0);

    if (a.flag("run")) {
      // a saved schedule: rebuilt by op name, proven race-free on the graph it executes,
      // checked once from a fresh state, then timed (max over ranks)
      if (halo && !halo->uses_wide_puts() &&
          saved.at("schedule").dump().find("he_putw_") != std::string::npos)
        TZ_THROW("the saved schedule uses wide IPC puts (he_putw_*), which this launch does not "
                 "offer: " << halo->transport_report().at("wide_put")
                           << " (e.g. the put block cap equal to --wide-put-blocks, or its preflight "
                              "failed on this node)");
      const Sequence seq = OpIndex(*g).sequence_from_json(saved.at("schedule"));
      const auto bad = verify(seq, *resolve_graph(*g, seq), streams);
      TZ_CHECK(bad.empty(), "schedule is not race-free on this graph: " << bad.front().desc());
      if (halo) halo->init_grid();
      if (spmv) spmv->reset_y();
      rt->device_sync();
      rt->prepare(seq);
      rt->run(1);
      rt->device_sync();
      double bad_cells = halo ? double(halo->check_grid()) + double(halo->ipc_errors()) : 0.0;
      double err = spmv ? spmv->check() : 0.0;
      ctrl->allreduce_sum(&bad_cells, 1);
      ctrl->allreduce_max(&err, 1);
      const int64_t iters = int64_t(a.num("run-iters", 1000));
      rt->run(int64_t(a.num("run-warmup", 50)));
      rt->device_sync();
      ctrl->barrier();
      const auto t0 = std::chrono::steady_clock::now();
      rt->run(iters);
      rt->device_sync();
      double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      ctrl->allreduce_max(&dt, 1);
      const bool ok = bad_cells == 0 && err < 1e-4;
      if (rank == 0) {
        Json o;
        o["schedule"] = a.get("run", "");
        o["workload"] = workload;
        o["ranks"] = size;
        o["streams"] = streams;
        o["mode"] = rt->effective_mode() == ExecMode::Graph ? "graph" : "eager";
        o["iters"] = iters;
        o["ms_per_iter"] = dt / double(std::max<int64_t>(iters, 1)) * 1e3;
        if (halo) o["halo_bad_cells"] = int64_t(bad_cells);
        if (spmv) o["spmv_max_rel_err"] = err;
        if (saved.contains("pct10_ms")) o["searched_pct10_ms"] = saved.at("pct10_ms");
        o["correct"] = ok;
        std::cout << o.dump() << "\n";
      }
      return ok ? 0 : 3;
    }

    SearchResult res;
    // --deadline S: past S seconds rank 0 prints the results CSV so far (the reference's partial
    // dump on the Slurm script's SIGABRT, scripts/perlmutter/spmv.sh:12) and every rank exits 5,
    // even when a collective or a device wait never returns
    std::unique_ptr<RunDeadline> deadline;
    std::string partialCsv;
    std::function<void(size_t, const SimResult &)> onResult;
    if (a.flag("deadline")) {
      deadline = std::make_unique<RunDeadline>(a.num("deadline", 0), 5);
      onResult = [&](size_t i, const SimResult &sr) {
        partialCsv += csv_row(i, sr.res, sr.seq) + "\n";
        deadline->set_report(partialCsv);
      };
    }
    auto header = [&](const Json &opts) {
      if (!deadline || rank != 0) return;
      partialCsv = opts.dump() + "\n";
      deadline->set_report(partialCsv);
    };
    if (a.get("solver", "mcts") == "dfs") {
      DfsOpts o;
      o.max_seqs = int64_t(a.num("max-seqs", 15000));
      o.bench = bo;
      o.trap_signals = true;
      header(o.json());
      res = dfs_explore(*g, plat, *bench, *ctrl, o, rank == 0 ? onResult : nullptr);
    } else {
      MctsOpts o;
      o.n_iters = int64_t(a.num("iters", 300));
      o.time_budget_s = a.num("time-budget", 0);
      o.max_tree_nodes = int64_t(a.num("max-tree-nodes", 0));
      o.strategy = a.get("strategy", "FastMin");
      o.seed = uint64_t(a.num("seed", 0));
      o.expand_rollout = !a.flag("no-expand-rollout");
      o.dump_tree = a.flag("dump-tree");
      o.checkpoint_path = a.get("checkpoint", "");
      o.checkpoint_every = o.checkpoint_path.empty() ? 0 : 10;
      o.resume_path = a.get("resume", "");
      if (a.flag("seed-schedule") && rank == 0) {
        // a --save-best document or a bare schedule (JSON array of ops of this workload)
        std::ifstream f(a.get("seed-schedule", ""));
        TZ_CHECK(f, "cannot open " << a.get("seed-schedule", ""));
        std::stringstream ss;
        ss << f.rdbuf();
        const Json doc = Json::parse(ss.str());
        o.seed_schedules.push_back(OpIndex(*g).sequence_from_json(doc.is_object() ? doc.at("schedule") : doc));
      }
      o.bench = bo;
      o.trap_signals = true;
      header(o.json());
      res = mcts_explore(*g, plat, *bench, *ctrl, o, rank == 0 ? onResult : nullptr);
    }

    // correctness of the winning halo schedule: one exchange from a fresh grid, every cell
    // checked on every rank (collective)
    int64_t bad = -1;
    if (halo && !sim) {
      std::string js = rank == 0 && res.best() >= 0 ? res.sims[res.best()].seq.json(true).dump() : "";
      ctrl->bcast(js, 0);
      if (!js.empty()) {
        const Sequence best = OpIndex(*g).sequence_from_json(Json::parse(js));
        rt->set_mode(ExecMode::Eager);
        halo->init_grid();
        ctrl->barrier();
        rt->prepare(best);
        rt->run(1);
        rt->device_sync();
        ctrl->barrier();
        double b = double(halo->check_grid()) + double(halo->ipc_errors());
        ctrl->allreduce_sum(&b, 1);
        bad = int64_t(b);
      }
    }

    if (deadline) deadline->cancel(); // finished in time: the full output follows
    if (rank == 0) {
      if (a.flag("csv")) {
        std::ofstream f(a.get("csv", "results.csv"));
        res.dump_csv(f);
      } else {
        res.dump_csv(std::cout);
      }
      if (a.flag("jsonl")) {
        std::ofstream f(a.get("jsonl", "results.jsonl"));
        res.dump_jsonl(f);
      }
      Json s;
      const int b = res.best();
      s["workload"] = workload;
      s["ranks"] = size;
      s["streams"] = streams;
      s["candidates"] = int64_t(res.sims.size());
      s["search_wall_s"] = res.wall_s;
      s["stop_reason"] = res.stop_reason;
      if (b >= 0) {
        s["best_pct10_ms"] = res.sims[b].res.pct10 * 1e3;
        s["best_pct50_ms"] = res.sims[b].res.pct50 * 1e3;
      }
      if (bad >= 0) s["verified_bad_cells"] = bad;
      std::cerr << s.dump() << "\n";
      if (a.flag("save-best") && b >= 0) {
        Json doc;
        doc["tenzing_amd"] = std::string("native");
        doc["ranks"] = size;
        doc["mode"] = a.get("mode", "eager");
        doc["pct10_ms"] = res.sims[b].res.pct10 * 1e3;
        doc["args"] = wargs;
        doc["schedule"] = res.sims[b].seq.json(true);
        std::ofstream f(a.get("save-best", "best.json"));
        f << doc.dump() << "\n";
      }
    }
    return bad > 0 ? 3 : 0;
  } catch (const std::exception &e) {
    std::cerr << "tz-search: error: " << e.what() << "\n";
    return 1;
  }
}
