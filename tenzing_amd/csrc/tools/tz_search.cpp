// tz-search: standalone native driver (no Python) — the MI355X counterpart of the reference's
// example executables halo-mcts-min-time / halo-mcts-coverage / spmv-{random,min-time,coverage}
// (tenzing-mcts/examples/*.cu) and tenzing-dfs/examples/spmv.cu, behind one CLI.
//
//   tz-search --workload halo --solver mcts --strategy FastMin --iters 100 --streams 4
//   torchrun --nproc-per-node 8 ... tz-search (one process per GPU; RANK/WORLD_SIZE/LOCAL_RANK)
//
// Multi-rank control-plane rendezvous goes through a file (--rdzv-file, default under /tmp keyed
// by MASTER_PORT); the data plane is RCCL.
#include "core/solve.hpp"
#include "hip/hip_runtime.hpp"
#include "workloads/workloads.hpp"

#include <hip/hip_runtime_api.h>

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
         "  [--strategy NAME] [--iters N] [--time-budget S] [--streams N] [--bench-iters N]\n"
         "  [--target-secs S] [--mode eager|graph] [--sim] [--seed N] [--no-expand-rollout]\n"
         "  [--halo-n N] [--nq N] [--ghost N] [--neighbors 6|26] [--order xyzq|qxyz]\n"
         "  [--fuse none|pack|all|groups|choice] [--graph-unroll K]\n"
         "  [--transport auto|rccl|ipc|copy|direct] [--rank-grid PXxPYxPZ] [--spmv-m N] [--spmv-matrix F.mtx]\n"
         "  [--spmv-form choice|split|accum] [--spmv-transport auto|rccl|ipc]\n"
         "  [--spmv-library adaptive|lrb|rowsplit|''] [--cu-partition] [--stencil] [--max-seqs N]\n"
         "  [--relay auto|off|force] [--relay-fracs F1,F2]\n"
         "  [--rdzv-file PATH]\n"
         "  [--master-addr HOST] [--csv PATH] [--jsonl PATH] [--dump-graph PATH] [--dump-tree]\n"
         "  [--checkpoint PATH] [--resume PATH] [--watchdog S]\n";
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
    const int rank = env_int("RANK", "OMPI_COMM_WORLD_RANK", 0);
    const int size = env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", 1);
    const int local = env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", rank);
    log_rank() = rank;
    const bool sim = a.flag("sim");
    const int streams = int(a.num("streams", 2));
    const std::string workload = a.get("workload", "halo");

    std::shared_ptr<Ctrl> ctrl;
    if (size > 1) {
      auto t = std::make_shared<TcpCtrl>(rank, size);
      const std::string port = std::getenv("MASTER_PORT") ? std::getenv("MASTER_PORT") : "default";
      t->rendezvous_file(a.get("rdzv-file", "/tmp/tz_rdzv_" + port), a.get("master-addr", "127.0.0.1"));
      ctrl = t;
    } else {
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

    auto g = std::make_shared<Graph>();
    std::shared_ptr<HaloExchange> halo;
    std::shared_ptr<DistSpmv> spmv;
    if (workload == "halo" || workload == "halo+spmv") {
      HaloArgs h;
      h.nx = h.ny = h.nz = int(a.num("halo-n", 512));
      h.nq = int(a.num("nq", 3));
      h.ghost = int(a.num("ghost", 3));
      h.neighbors = int(a.num("neighbors", 6));
      h.fuse = a.get("fuse", "none");
      h.transport = a.get("transport", "auto");
      h.order = a.get("order", "xyzq");
      h.stencil = a.flag("stencil");
      h.relay = a.get("relay", "auto");
      {
        // comma-separated relayed shares, e.g. 0.15,0.2
        const std::string fr = a.get("relay-fracs", "");
        if (!fr.empty()) {
          h.relay_fracs.clear();
          std::stringstream ss(fr);
          std::string tok;
          while (std::getline(ss, tok, ',')) h.relay_fracs.push_back(std::stod(tok));
        }
      }
      TZ_CHECK(h.order == "xyzq" || h.order == "qxyz", "--order must be xyzq or qxyz");
      h.rank = rank;
      h.size = size;
      const std::string rg = a.get("rank-grid", "");
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
      s.m = int64_t(a.num("spmv-m", 150000));
      s.matrix = a.get("spmv-matrix", "");
      s.rank = rank;
      s.size = size;
      s.prefix = workload == "halo+spmv" ? "spmv_" : "";
      s.form = a.get("spmv-form", "choice");
      s.transport = a.get("spmv-transport", "auto");
      s.library = a.get("spmv-library", "adaptive");
      spmv = std::make_shared<DistSpmv>(s);
      if (!sim) spmv->setup(ctrl.get());
      spmv->add_to_graph(*g);
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
    if (a.flag("cu-partition")) plat.symmetric_streams = false;
    std::unique_ptr<HipRuntime> rt;
    std::unique_ptr<Benchmarker> bench;
    if (sim) {
      bench = std::make_unique<SimBenchmarker>(streams, SimParams());
    } else {
      HipRuntimeOpts ro;
      ro.n_streams = streams;
      ro.mode = a.get("mode", "eager") == "graph" ? ExecMode::Graph : ExecMode::Eager;
      ro.watchdog_s = a.num("watchdog", 60);
      ro.graph_unroll = int(a.num("graph-unroll", 1));
      ro.cu_partition = a.flag("cu-partition");
      rt = std::make_unique<HipRuntime>(ro);
      bench = std::make_unique<EmpiricalBenchmarker>(*rt, *ctrl);
    }
    BenchOpts bo;
    bo.n_iters = int64_t(a.num("bench-iters", 50));
    bo.target_secs = a.num("target-secs", 0.01);

    SearchResult res;
    if (a.get("solver", "mcts") == "dfs") {
      DfsOpts o;
      o.max_seqs = int64_t(a.num("max-seqs", 15000));
      o.bench = bo;
      o.trap_signals = true;
      res = dfs_explore(*g, plat, *bench, *ctrl, o);
    } else {
      MctsOpts o;
      o.n_iters = int64_t(a.num("iters", 300));
      o.time_budget_s = a.num("time-budget", 0);
      o.strategy = a.get("strategy", "FastMin");
      o.seed = uint64_t(a.num("seed", 0));
      o.expand_rollout = !a.flag("no-expand-rollout");
      o.dump_tree = a.flag("dump-tree");
      o.checkpoint_path = a.get("checkpoint", "");
      o.checkpoint_every = o.checkpoint_path.empty() ? 0 : 10;
      o.resume_path = a.get("resume", "");
      o.bench = bo;
      o.trap_signals = true;
      res = mcts_explore(*g, plat, *bench, *ctrl, o);
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
    }
    return bad > 0 ? 3 : 0;
  } catch (const std::exception &e) {
    std::cerr << "tz-search: error: " << e.what() << "\n";
    return 1;
  }
}
