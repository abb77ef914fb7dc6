// Solvers: exhaustive DFS and Monte-Carlo tree search over the State decision tree.
//
// Parity:
//   tenzing-dfs: get_all_sequences / explore / Result::dump_csv (tenzing-dfs/src/dfs.cpp:16-105,
//     tenzing-dfs/include/tenzing/dfs/dfs.hpp:78-178)
//   tenzing-mcts: explore (mcts.hpp:154-326), Node select/expand/rollout/backprop
//     (mcts_node.hpp:119-564), dump_graphviz (mcts.hpp:52-127), per-phase counters
//     (mcts/counters.hpp:15-25), strategies FastMin, Coverage, Random (built in the reference),
//     AvgTime, Unvisited, AntiCorrelation, NormalizedAntiCorrelation, NormRootCorr,
//     BalanceHistogram (stale in the reference, all implemented here behind one interface).
// Differences: tree nodes store only their decision and statistics; the State is rebuilt
// incrementally along the selection path (the reference stores a full Graph per node,
// mcts_node.hpp:45); RNG is a seeded mt19937_64 instead of rand(); equivalent final schedules
// are benchmarked once and re-used (cache by canonical key) unless disabled; search can be
// bounded by a wall-clock budget; the tree can be checkpointed to JSON and resumed.
#pragma once

#include "benchmark.hpp"
#include "util.hpp"

#include <functional>
#include <limits>
#include <memory>
#include <ostream>
#include <random>

namespace tz {

struct SimResult {
  Sequence seq;
  BenchResult res;
  bool cached = false;
  bool seeded = false; // one of MctsOpts::seed_schedules, not found by the search
};

struct SearchResult {
  std::vector<SimResult> sims;
  Counters counters;
  Json opts;
  double wall_s = 0;
  size_t tree_size = 0;
  size_t tree_fully_visited = 0;
  std::string stop_reason;
  size_t failed = 0; // candidates that could not be benchmarked (skipped)
  // transports that died during the search (health.hpp) and the decisions taken out of the
  // tree because they need one: no candidate using a dead transport is measured again
  std::vector<std::string> dead_domains;
  size_t pruned_dead = 0;

  /// index of the best (lowest pct10) result, -1 if none
  int best() const;
  /// CSV rows in the reference format, preceded by a one-line JSON of the options
  void dump_csv(std::ostream &os) const;
  /// one JSON object per line: {"i", "result", "seq"}
  void dump_jsonl(std::ostream &os) const;
};

// ------------------------------------------------------------------------ MCTS

struct MctsNode {
  MctsNode *parent = nullptr;
  std::vector<std::unique_ptr<MctsNode>> children;
  Decision decision;
  bool expanded = false;
  bool fully_visited = false;
  bool terminal = false;
  size_t n = 0;
  // strategy statistics
  double tmin = std::numeric_limits<double>::infinity();
  double tmax = -std::numeric_limits<double>::infinity();
  std::vector<double> times; // kept sorted by strategies that need quantiles

  const MctsNode &root() const { return parent ? parent->root() : *this; }
  size_t size() const;
  size_t fully_visited_size() const;
  size_t unvisited_size() const;
  bool is_leaf() const;
};

class Strategy {
public:
  virtual ~Strategy() = default;
  virtual std::string name() const = 0;
  /// exploitation score of `child` in [0,1] (or +inf to force)
  virtual double select(const MctsNode &child) = 0;
  virtual void backprop(MctsNode &node, const BenchResult &br) = 0;
  virtual std::string label(const MctsNode &node) const;
};

std::unique_ptr<Strategy> make_strategy(const std::string &name, uint64_t seed);
std::vector<std::string> strategy_names();

struct MctsOpts {
  int64_t n_iters = 300;        // 0 = until the tree is fully visited / budget exhausted
  double time_budget_s = 0;     // 0 = unlimited
  int64_t max_tree_nodes = 0;   // stop once the tree holds this many nodes (0 = unlimited)
  bool expand_rollout = true;   // keep rollout paths in the tree (reference Opts::expandRollout)
  bool remove_redundant_syncs = true;
  bool reuse_measurements = true; // benchmark each equivalent final schedule once
  bool verify = true;           // race-check every candidate before it runs
  bool skip_failed = true;      // a candidate whose benchmark throws is pruned, not fatal
  bool dump_tree = false;
  std::string dump_tree_prefix = "mcts_";
  std::string strategy = "FastMin";
  uint64_t seed = 0;
  double explore_c = 1.41421356; // UCT exploration constant (reference sqrt(2))
  BenchOpts bench;
  std::string checkpoint_path;  // write tree + results JSON here every checkpoint_every iters
  int64_t checkpoint_every = 0;
  bool trap_signals = false;     // dump partial CSV on SIGINT/SIGTERM/SIGABRT (CLI)
  std::string resume_path;      // resume a checkpointed tree
  // schedules of this graph to measure before the search (the program's current schedule, a
  // previous search's best): they count as results, so the search never reports worse
  std::vector<Sequence> seed_schedules;
  Json json() const;
};

/// Runs on every rank of `ctrl`; rank 0 owns the tree, all ranks benchmark each candidate
/// together. Only rank 0's result holds the simulations.
SearchResult mcts_explore(const Graph &g, const Platform &plat, Benchmarker &bench, Ctrl &ctrl,
                          const MctsOpts &opts,
                          const std::function<void(size_t, const SimResult &)> &onResult = nullptr);

/// graphviz of an MCTS tree (reference mcts.hpp:52-127)
std::string mcts_tree_graphviz(const MctsNode &root, const Strategy &strat, size_t maxNodes = 2000);

// ------------------------------------------------------------------------ DFS

struct DfsOpts {
  int64_t max_seqs = -1; // stop enumerating at this many sequences (reference maxSeqs)
  bool dedup_states = true;
  bool remove_redundant_syncs = true;
  bool trap_signals = false;
  bool skip_failed = true; // a sequence whose benchmark throws is skipped, not fatal
  BenchOpts bench;
  Json json() const;
};

/// all complete, pairwise non-equivalent sequences (reference dfs.cpp:16-82)
std::vector<Sequence> get_all_sequences(const Graph &g, const Platform &plat, int64_t maxSeqs = -1,
                                        bool dedupStates = true, bool removeRedundant = true);

SearchResult dfs_explore(const Graph &g, const Platform &plat, Benchmarker &bench, Ctrl &ctrl,
                         const DfsOpts &opts,
                         const std::function<void(size_t, const SimResult &)> &onResult = nullptr);

// ------------------------------------------------------------------------ misc

/// install SIGINT/SIGTERM/SIGABRT handler that calls fn then exits (reference trap.cpp:11-35)
/// Signal trap (reference src/trap.cpp:11-35): SIGINT/SIGTERM/SIGABRT only set a flag (the
/// handler is async-signal-safe); the solvers poll it between candidates, stop collectively,
/// call `fn` on rank 0 (dump the partial CSV) and exit(1). A second signal exits at once.
void register_handler(std::function<void(int)> fn);
void unregister_handler();
/// the pending trapped signal (0 = none)
int signal_pending();
/// rank 0 after a collective signal stop: run the registered handler, then exit(1)
[[noreturn]] void handle_pending_signal();

/// Wall-clock limit for a whole program run (bench.py, tz-search). Past it, the report line the
/// program set last (its best result so far, in its normal output format, marked partial) is
/// written to stdout with one write(2) and the process exits with `exit_code`, whatever the
/// other threads are blocked in (a hung collective, a device wait): a run that cannot finish
/// still reports. Native, so it fires while Python threads hold or wait for the GIL. Reference
/// analogue: the Slurm script signals SIGABRT 10 s before the wall-clock limit
/// (scripts/perlmutter/spmv.sh:12) and the trap dumps the partial CSV (src/trap.cpp:26-30).
class RunDeadline {
public:
  RunDeadline(double seconds, int exitCode);
  ~RunDeadline();
  RunDeadline(const RunDeadline &) = delete;
  RunDeadline &operator=(const RunDeadline &) = delete;
  /// the line to print if the deadline fires ("" = print nothing)
  void set_report(const std::string &line);
  /// disarm (the program finished in time)
  void cancel();
  /// expire at the latest `seconds` from now (never later than already set) and exit with
  /// `exit_code` then: e.g. once a result is final, a bounded budget for the optional work after
  /// it, whose expiry prints the (complete) report and exits 0
  void tighten(double seconds, int exit_code);
  double remaining() const;
  bool armed() const;

  struct Impl;

private:
  std::unique_ptr<Impl> p_;
};

/// leave the process now with `code` after an unrecoverable failure (e.g. a hung run that the
/// watchdog's abort could not release): the armed RunDeadline's report line is printed first,
/// with `"exit_reason": why` added, so a bench still ends with its partial JSON line
[[noreturn]] void exit_with_report(int code, const std::string &why);

/// {"major","minor","patch","hash","args"} (reference reproduce.cpp:22-37)
Json reproduce_json(const std::vector<std::string> &args);
std::string version_string();

} // namespace tz
