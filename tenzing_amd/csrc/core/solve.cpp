#include "solve.hpp"
#include "health.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <unistd.h>

#include <atomic>
#include <fstream>
#include <iostream>
#include <limits>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#ifndef TZ_VERSION_MAJOR
#define TZ_VERSION_MAJOR 0
#define TZ_VERSION_MINOR 1
#define TZ_VERSION_PATCH 0
#endif
#ifndef TZ_GIT_HASH
#define TZ_GIT_HASH "unknown"
#endif

namespace tz {

static constexpr double kInf = std::numeric_limits<double>::infinity();

/// A benchmark failure the search may skip: one every rank agreed on (CandidateFailed), or any
/// failure when there is a single rank. Anything else may be local to one rank, and skipping it
/// would leave that rank's peers blocked in the benchmark's collectives, so it propagates.
static bool skippable(const std::exception &e, const Ctrl &ctrl) {
  return dynamic_cast<const CandidateFailed *>(&e) != nullptr || ctrl.size() == 1;
}

// ======================================================================== results

int SearchResult::best() const {
  int b = -1;
  for (size_t i = 0; i < sims.size(); ++i)
    if (b < 0 || sims[i].res.pct10 < sims[b].res.pct10) b = int(i);
  return b;
}

void SearchResult::dump_csv(std::ostream &os) const {
  os << opts.dump() << "\n";
  for (size_t i = 0; i < sims.size(); ++i) os << csv_row(i, sims[i].res, sims[i].seq) << "\n";
}

void SearchResult::dump_jsonl(std::ostream &os) const {
  for (size_t i = 0; i < sims.size(); ++i) {
    Json j;
    j["i"] = int64_t(i);
    j["result"] = sims[i].res.json();
    j["cached"] = sims[i].cached;
    if (sims[i].seeded) j["seeded"] = true;
    j["seq"] = sims[i].seq.json();
    os << j.dump() << "\n";
  }
}

// ======================================================================== MCTS nodes

size_t MctsNode::size() const {
  size_t s = 1;
  for (const auto &c : children) s += c->size();
  return s;
}
size_t MctsNode::fully_visited_size() const {
  size_t s = fully_visited ? 1 : 0;
  for (const auto &c : children) s += c->fully_visited_size();
  return s;
}
size_t MctsNode::unvisited_size() const {
  size_t s = n == 0 ? 1 : 0;
  for (const auto &c : children) s += c->unvisited_size();
  return s;
}
bool MctsNode::is_leaf() const {
  if (children.empty()) return true;
  for (const auto &c : children)
    if (c->n == 0) return true;
  return false;
}

// ======================================================================== strategies

std::string Strategy::label(const MctsNode &node) const {
  std::ostringstream ss;
  ss.precision(3);
  ss << std::scientific;
  if (std::isfinite(node.tmin)) ss << node.tmin << " - " << node.tmax;
  else if (!node.times.empty()) ss << node.times.front() << " - " << node.times.back();
  return ss.str();
}

namespace {

double clamp01(double v) {
  if (std::isnan(v)) return 0;
  return v < 0 ? 0 : (v > 1 ? 1 : v);
}

void push_sorted(std::vector<double> &v, double x) { v.insert(std::upper_bound(v.begin(), v.end(), x), x); }

std::vector<uint64_t> histogram(const std::vector<double> &v, double tMin, double tMax, int nBins) {
  std::vector<uint64_t> h(nBins, 0);
  for (double e : v) {
    long i = tMax > tMin ? long((e - tMin) / (tMax - tMin) * nBins) : 0;
    if (i < 0) i = 0;
    if (i >= nBins) i = nBins - 1;
    ++h[i];
  }
  return h;
}

// reference mcts_strategy_fast_min.hpp:40-65
struct FastMin : Strategy {
  std::string name() const override { return "FastMin"; }
  double select(const MctsNode &child) override {
    const MctsNode &root = child.root();
    if (&child == &root) return 1;
    if (root.n < 2 || root.tmax == root.tmin) return 1;
    if (child.n < 1) return select(*child.parent);
    return clamp01(1 - (child.tmin - root.tmin) / (root.tmax - root.tmin));
  }
  void backprop(MctsNode &node, const BenchResult &br) override {
    node.tmin = std::min(node.tmin, br.pct10);
    node.tmax = std::max(node.tmax, br.pct10);
  }
};

// reference mcts_strategy_coverage.hpp:39-101
struct Coverage : Strategy {
  std::string name() const override { return "Coverage"; }
  double select(const MctsNode &child) override {
    const MctsNode &parent = *child.parent;
    const auto &pt = parent.times, &ct = child.times;
    if (pt.size() < 2 || ct.empty()) return 1;
    const double pMin = pt.front(), pMax = pt.back();
    if (pMin == pMax) return 1;
    if (ct.size() < 2) return clamp01(std::max(ct[0] - pMin, pMax - ct[0]) / (pMax - pMin));
    return clamp01((ct.back() - ct.front()) / (pMax - pMin));
  }
  void backprop(MctsNode &node, const BenchResult &br) override {
    push_sorted(node.times, br.pct10);
    node.tmin = node.times.front();
    node.tmax = node.times.back();
  }
};

// reference mcts_strategy_random.hpp:31-54
struct RandomS : Strategy {
  std::mt19937_64 rng;
  std::unordered_map<const MctsNode *, size_t> selected;
  explicit RandomS(uint64_t seed) : rng(seed) {}
  std::string name() const override { return "Random"; }
  double select(const MctsNode &child) override {
    const MctsNode &parent = *child.parent;
    auto it = selected.find(&parent);
    if (it == selected.end()) {
      std::uniform_int_distribution<size_t> u(0, parent.children.size() - 1);
      it = selected.emplace(&parent, u(rng)).first;
    }
    return parent.children[it->second].get() == &child ? kInf : 0;
  }
  void backprop(MctsNode &node, const BenchResult &br) override {
    node.times.push_back(br.pct10);
    if (!node.parent) selected.clear();
  }
};

// reference mcts_strategy_avg_time.hpp:33-58
struct AvgTime : Strategy {
  std::string name() const override { return "AvgTime"; }
  double select(const MctsNode &child) override {
    const MctsNode &root = child.root();
    if (child.n < 1 || root.n < 2 || root.tmax == root.tmin) return 0;
    double acc = 0;
    for (double t : child.times) acc += clamp01(1 - (t - root.tmin) / (root.tmax - root.tmin));
    return acc / double(child.times.size());
  }
  void backprop(MctsNode &node, const BenchResult &br) override {
    node.tmin = std::min(node.tmin, br.pct10);
    node.tmax = std::max(node.tmax, br.pct10);
    node.times.push_back(br.pct10);
  }
};

// reference mcts_strategy_unvisited.hpp:26-36
struct Unvisited : Strategy {
  std::string name() const override { return "Unvisited"; }
  double select(const MctsNode &child) override { return child.times.empty() ? kInf : 0; }
  void backprop(MctsNode &node, const BenchResult &br) override { node.times.push_back(br.pct10); }
};

constexpr int kBins = 10;

// reference mcts_strategy_anti_corr.hpp:25-88
struct AntiCorrelation : Strategy {
  std::string name() const override { return "AntiCorrelation"; }
  double select(const MctsNode &child) override {
    const MctsNode &parent = *child.parent;
    if (parent.times.size() < 2 || child.times.size() < 2) return 0;
    const double tMin = std::min(parent.times.front(), child.times.front());
    const double tMax = std::max(parent.times.back(), child.times.back());
    double v = corr(histogram(parent.times, tMin, tMax, kBins), histogram(child.times, tMin, tMax, kBins));
    return clamp01((2 - (v + 1)) / 2);
  }
  void backprop(MctsNode &node, const BenchResult &br) override { push_sorted(node.times, br.pct10); }
};

// reference mcts_strategy_norm_anti_corr.hpp:45-110 (correlation against the root histogram,
// normalized by the best sibling). `anti` selects anti-correlation vs correlation
// (NormRootCorr, mcts_strategy_norm_root_corr.hpp:46-110).
struct NormCorr : Strategy {
  bool anti;
  explicit NormCorr(bool a) : anti(a) {}
  std::string name() const override { return anti ? "NormalizedAntiCorrelation" : "NormRootCorr"; }
  double score(const std::vector<uint64_t> &rh, const std::vector<double> &times, double tMin, double tMax) const {
    double c = corr(rh, histogram(times, tMin, tMax, kBins)) + 1; // [0,2]
    return anti ? 2 - c : c;
  }
  double select(const MctsNode &child) override {
    const MctsNode &parent = *child.parent;
    const MctsNode &root = child.root();
    if (parent.times.size() < 2 || child.times.size() < 2 || root.times.empty()) return 0;
    const double tMin = root.times.front(), tMax = root.times.back();
    auto rh = histogram(root.times, tMin, tMax, kBins);
    double best = -1;
    for (const auto &sib : parent.children) best = std::max(best, score(rh, sib->times, tMin, tMax));
    if (best <= 0) return 0;
    return clamp01(score(rh, child.times, tMin, tMax) / best);
  }
  void backprop(MctsNode &node, const BenchResult &br) override { push_sorted(node.times, br.pct10); }
};

// reference mcts_strategy_balance_hist.hpp:49-190 (active #if 1 branch)
struct BalanceHistogram : Strategy {
  std::string name() const override { return "BalanceHistogram"; }
  double select(const MctsNode &child) override {
    const MctsNode &parent = *child.parent;
    const MctsNode &root = child.root();
    if (parent.times.empty() || child.times.empty() || root.times.empty()) return 0;
    const double tMin = root.times.front(), tMax = root.times.back();
    auto rh = histogram(root.times, tMin, tMax, kBins);
    auto ch = histogram(child.times, tMin, tMax, kBins);
    long smallest = -1, largest = -1;
    uint64_t cnt = std::numeric_limits<uint64_t>::max();
    for (int i = 0; i < kBins; ++i)
      if (rh[i] > 0 && rh[i] < cnt && ch[i] > 0) {
        smallest = i;
        cnt = rh[i];
      }
    int64_t lc = -1;
    for (int i = 0; i < kBins; ++i)
      if (rh[i] > 0 && int64_t(rh[i]) > lc) {
        largest = i;
        lc = int64_t(rh[i]);
      }
    if (smallest < 0 || largest < 0) return 0;
    return clamp01(1.0 - double(rh[smallest]) / double(rh[largest]));
  }
  void backprop(MctsNode &node, const BenchResult &br) override { push_sorted(node.times, br.pct10); }
};

} // namespace

std::vector<std::string> strategy_names() {
  return {"FastMin", "Coverage", "Random", "AvgTime", "Unvisited", "AntiCorrelation",
          "NormalizedAntiCorrelation", "NormRootCorr", "BalanceHistogram"};
}

std::unique_ptr<Strategy> make_strategy(const std::string &name, uint64_t seed) {
  std::string n = name;
  std::transform(n.begin(), n.end(), n.begin(), ::tolower);
  n.erase(std::remove(n.begin(), n.end(), '_'), n.end());
  if (n == "fastmin" || n == "mintime") return std::make_unique<FastMin>();
  if (n == "coverage") return std::make_unique<Coverage>();
  if (n == "random") return std::make_unique<RandomS>(seed);
  if (n == "avgtime") return std::make_unique<AvgTime>();
  if (n == "unvisited") return std::make_unique<Unvisited>();
  if (n == "anticorrelation" || n == "anticorr") return std::make_unique<AntiCorrelation>();
  if (n == "normalizedanticorrelation" || n == "normanticorr") return std::make_unique<NormCorr>(true);
  if (n == "normrootcorr") return std::make_unique<NormCorr>(false);
  if (n == "balancehistogram" || n == "balancehist") return std::make_unique<BalanceHistogram>();
  TZ_THROW("unknown MCTS strategy '" << name << "'");
}

// ======================================================================== MCTS

Json MctsOpts::json() const {
  Json j, o;
  o["nIters"] = n_iters;
  o["timeBudgetS"] = time_budget_s;
  if (max_tree_nodes > 0) o["maxTreeNodes"] = max_tree_nodes;
  o["expandRollout"] = expand_rollout;
  o["removeRedundantSyncs"] = remove_redundant_syncs;
  o["reuseMeasurements"] = reuse_measurements;
  o["strategy"] = strategy;
  o["seed"] = int64_t(seed);
  o["exploreC"] = explore_c;
  o["benchOpts"] = bench.json();
  j["mcts__Opts"] = o;
  return j;
}

namespace {

struct Tree {
  MctsNode root;
  std::unique_ptr<Strategy> strat;
  std::mt19937_64 rng;
  double c;
  size_t nodes = 1; // nodes created so far (the root included)
  std::set<std::string> dead; // dead transport domains (health.hpp): decisions needing one are pruned
  size_t prunedDead = 0;

  /// does decision `d` (taken in state `st`) commit the schedule to a dead transport? A choice
  /// of an alternative that needs a dead domain, or the execution of an op of one.
  bool dead_decision(const State &st, const Decision &d) const {
    if (dead.empty()) return false;
    if (d.kind == Decision::Kind::Choose) {
      const auto alts = static_cast<const ChoiceOp &>(*st.graph().op(d.node)).choices();
      return uses_domain(alts[size_t(d.choice)], dead);
    }
    if (d.kind == Decision::Kind::Execute && d.op) return uses_domain(d.op, dead);
    if (d.kind == Decision::Kind::Assign) return uses_domain(st.graph().op(d.node), dead);
    return false;
  }

  /// refresh the fully-visited flags from `node` up to the root
  static void propagate_visited(MctsNode *node) {
    for (; node; node = node->parent) {
      if (node->children.empty() || node->fully_visited) continue;
      bool all = true;
      for (auto &ch : node->children) all = all && ch->fully_visited;
      if (!all) break;
      node->fully_visited = true;
    }
  }

  /// take `node`'s children that need a dead transport out of the search (fully visited, never
  /// selected again); true if any child is still live
  bool prune_dead_children(MctsNode &node, const State &st) {
    bool live = false;
    if (!dead.empty())
      for (auto &ch : node.children)
        if (!ch->fully_visited && dead_decision(st, ch->decision)) {
          ch->fully_visited = true;
          ++prunedDead;
        }
    for (auto &ch : node.children) live = live || !ch->fully_visited;
    if (!node.children.empty() && !live) propagate_visited(&node);
    return live || node.children.empty();
  }

  void ensure_children(MctsNode &node, const State &st) {
    if (node.expanded) return;
    node.expanded = true;
    node.terminal = st.complete();
    for (auto &d : st.get_decisions()) {
      ++nodes;
      auto ch = std::make_unique<MctsNode>();
      ch->parent = &node;
      ch->decision = d;
      node.children.push_back(std::move(ch));
    }
  }

  MctsNode *pick_uct(MctsNode &node) {
    std::vector<double> ucts;
    ucts.reserve(node.children.size());
    double m = -kInf;
    for (auto &ch : node.children) {
      double u;
      if (ch->fully_visited) {
        u = -kInf;
      } else {
        const double exploit = strat->select(*ch);
        const double explore = c * std::sqrt(std::log(double(node.n)) / double(ch->n));
        u = exploit + explore;
        if (std::isnan(u)) u = exploit;
      }
      ucts.push_back(u);
      m = std::max(m, u);
    }
    std::vector<size_t> best;
    for (size_t i = 0; i < ucts.size(); ++i)
      if (ucts[i] == m) best.push_back(i);
    std::uniform_int_distribution<size_t> u(0, best.size() - 1);
    return node.children[best[u(rng)]].get();
  }

  /// a candidate that could not be benchmarked: count the visit, take the path out of the
  /// search (fully visited), feed the strategy nothing
  void prune_failed(MctsNode *node) {
    node->fully_visited = true;
    for (; node; node = node->parent) {
      ++node->n;
      if (!node->children.empty()) {
        bool all = true;
        for (auto &ch : node->children) all = all && ch->fully_visited;
        if (all) node->fully_visited = true;
      }
    }
  }

  void backprop(MctsNode *node, const BenchResult &br) {
    for (; node; node = node->parent) {
      ++node->n;
      if (node->children.empty()) {
        if (node->expanded) node->fully_visited = true;
      } else {
        bool all = true;
        for (auto &ch : node->children) all = all && ch->fully_visited;
        if (all) node->fully_visited = true;
      }
      strat->backprop(*node, br);
    }
  }

  Json save(const MctsNode &node) const {
    Json j;
    j["n"] = int64_t(node.n);
    if (std::isfinite(node.tmin)) j["tmin"] = node.tmin;
    if (std::isfinite(node.tmax)) j["tmax"] = node.tmax;
    if (!node.times.empty()) {
      Json t = Json::array();
      for (double x : node.times) t.push_back(x);
      j["times"] = t;
    }
    j["fv"] = node.fully_visited;
    if (node.expanded) {
      Json cs = Json::array();
      for (auto &ch : node.children) cs.push_back(ch->n ? save(*ch) : Json());
      j["c"] = cs;
    }
    return j;
  }

  void load(MctsNode &node, const Json &j, const State &st) {
    if (j.is_null()) return;
    node.n = size_t(j.at("n").as_int());
    if (j.contains("tmin")) node.tmin = j.at("tmin").as_double();
    if (j.contains("tmax")) node.tmax = j.at("tmax").as_double();
    if (j.contains("times"))
      for (auto &x : j.at("times").as_array()) node.times.push_back(x.as_double());
    node.fully_visited = j.at("fv").as_bool();
    if (j.contains("c")) {
      ensure_children(node, st);
      const auto &cs = j.at("c").as_array();
      TZ_CHECK(cs.size() == node.children.size(), "checkpoint does not match this graph");
      for (size_t i = 0; i < cs.size(); ++i) {
        if (cs[i].is_null()) continue;
        load(*node.children[i], cs[i], st.apply(node.children[i]->decision));
      }
    }
  }
};

// every op name inside `op`: itself, a compound's sub-graph, a choice's alternatives
void op_names(const OpPtr &op, std::unordered_set<std::string> &out) {
  out.insert(op->name());
  if (op->op_class() == OpClass::Compound) {
    auto g = static_cast<const CompoundOp &>(*op).graph();
    for (int v : g->vertices()) op_names(g->op(v), out);
  } else if (op->op_class() == OpClass::Choice) {
    for (const auto &c : static_cast<const ChoiceOp &>(*op).choices()) op_names(c, out);
  }
}

// The tree path of a seed schedule, so that its measurement steers the search like any
// rollout's. Descends from the root taking, at every state, the decision that agrees with the
// seed: an Expand; a Choose whose alternative holds ops of the seed; an Assign of a pending op to
// the stream the seed uses for it (seed streams relabeled consistently); then, by the seed's
// next entry: for a sync, the offered sync of the same kind on the same stream, or none (the
// state does not need it); for a graph op its Execute, else a sync the state requires (one the
// seed dropped as redundant). The path is accepted when the descent's schedule, after the
// seed's redundant-sync removal, is equivalent to the seed. Returns the terminal leaf or nullptr.
MctsNode *seed_path(Tree &tree, const State &rootState, const Sequence &seed, bool removeRedundant,
                    int nStreams) {
  std::unordered_map<std::string, int> streamOf; // the seed's stream of each bound GPU op
  std::unordered_set<std::string> names;
  for (const auto &e : seed.entries) {
    const OpClass c = e.op->op_class();
    // (Start / Finish are in every sub-graph: they would match every alternative of a choice)
    if (c == OpClass::Sync || c == OpClass::Start || c == OpClass::Finish) continue;
    names.insert(e.op->name());
    if (c == OpClass::BoundGpu) streamOf[e.op->name()] = static_cast<const BoundGpuOp &>(*e.op).stream();
  }
  auto sync_stream = [](const BoundOp &op) {
    const Json j = op.json();
    return j.contains("stream") ? int(j.at("stream").as_int()) : -1;
  };
  std::unordered_map<int, int> relabel; // seed stream -> state stream
  State st = rootState;
  MctsNode *cur = &tree.root;
  size_t pos = 0;
  while (pos < seed.size() && seed[pos]->op_class() == OpClass::Start) ++pos;
  for (int guard = 0; !st.complete(); ++guard) {
    if (guard > 1000000) return nullptr;
    tree.ensure_children(*cur, st);
    const auto &ch = cur->children;
    int pick = -1;
    bool advance = false;
    for (size_t i = 0; i < ch.size() && pick < 0; ++i)
      if (ch[i]->decision.kind == Decision::Kind::Expand) pick = int(i);
    for (size_t i = 0; i < ch.size() && pick < 0; ++i) {
      const Decision &d = ch[i]->decision;
      if (d.kind != Decision::Kind::Choose) continue;
      const auto alts = static_cast<const ChoiceOp &>(*st.graph().op(d.node)).choices();
      std::unordered_set<std::string> in;
      op_names(alts[size_t(d.choice)], in);
      for (const auto &n : in)
        if (names.count(n)) {
          pick = int(i);
          break;
        }
    }
    for (size_t i = 0; i < ch.size() && pick < 0; ++i) {
      const Decision &d = ch[i]->decision;
      if (d.kind != Decision::Kind::Assign) continue;
      auto it = streamOf.find(st.graph().op(d.node)->name());
      if (it == streamOf.end()) continue;
      auto m = relabel.find(it->second);
      bool taken = false;
      for (const auto &kv : relabel) taken = taken || kv.second == d.stream;
      if ((m != relabel.end() && m->second == d.stream) || (m == relabel.end() && !taken)) {
        relabel[it->second] = d.stream;
        pick = int(i);
      }
    }
    if (pick < 0 && pos < seed.size() && seed[pos]->op_class() == OpClass::Sync) {
      const BoundOp &want = *seed[pos];
      const int ws = sync_stream(want);
      auto m = relabel.find(ws);
      for (size_t i = 0; i < ch.size() && pick < 0; ++i) {
        const Decision &d = ch[i]->decision;
        if (d.kind != Decision::Kind::Execute || d.op->op_class() != OpClass::Sync || d.op->kind() != want.kind())
          continue;
        if (ws < 0 || (m != relabel.end() && m->second == sync_stream(*d.op))) pick = int(i);
      }
      ++pos; // taken, or a sync this state does not need
      if (pick < 0) continue;
    }
    if (pick < 0 && pos < seed.size()) {
      for (size_t i = 0; i < ch.size() && pick < 0; ++i) {
        const Decision &d = ch[i]->decision;
        if (d.kind == Decision::Kind::Execute && d.op->op_class() != OpClass::Sync &&
            d.op->name() == seed[pos]->name()) {
          pick = int(i);
          advance = true;
        }
      }
    }
    for (size_t i = 0; i < ch.size() && pick < 0; ++i) {
      const Decision &d = ch[i]->decision;
      if (d.kind == Decision::Kind::Execute && d.op->op_class() == OpClass::Sync) pick = int(i);
    }
    if (pick < 0) return nullptr;
    if (advance) ++pos;
    st.apply_inplace(ch[size_t(pick)]->decision);
    cur = ch[size_t(pick)].get();
  }
  tree.ensure_children(*cur, st); // terminal: expanded without children
  Sequence s = st.sequence();
  if (removeRedundant) remove_redundant_syncs(s, st.graph(), nStreams);
  return s.canonical_key() == seed.canonical_key() ? cur : nullptr;
}

void graphviz_rec(const MctsNode &node, const Strategy &strat, std::ostream &os, size_t &count,
                  size_t maxNodes, const std::string &id) {
  std::string color = node.fully_visited ? "green" : "black";
  os << "  " << id << " [label=\"" << node.decision.desc() << "\\nn=" << node.n << "\\n"
     << strat.label(node) << "\", color=" << color << "];\n";
  ++count;
  size_t i = 0;
  for (const auto &ch : node.children) {
    ++i;
    if (count >= maxNodes) break;
    // hide unvisited, fully-visited and single-rollout subtrees (reference mcts.hpp:60-100)
    if (ch->n == 0) continue;
    const std::string cid = id + "_" + std::to_string(i);
    if (ch->fully_visited || ch->n == 1) {
      os << "  " << cid << " [label=\"" << ch->decision.desc() << "\\nn=" << ch->n
         << "\", color=" << (ch->fully_visited ? "green" : "gray") << "];\n";
      ++count;
    } else {
      graphviz_rec(*ch, strat, os, count, maxNodes, cid);
    }
    os << "  " << id << " -> " << cid << ";\n";
  }
}

void write_file(const std::string &path, const std::string &s) {
  std::ofstream f(path);
  f << s;
}

} // namespace

std::string mcts_tree_graphviz(const MctsNode &root, const Strategy &strat, size_t maxNodes) {
  std::ostringstream os;
  os << "digraph MCTS {\n";
  size_t count = 0;
  graphviz_rec(root, strat, os, count, maxNodes, "n");
  os << "}\n";
  return os.str();
}

SearchResult mcts_explore(const Graph &g, const Platform &plat, Benchmarker &bench, Ctrl &ctrl,
                          const MctsOpts &opts,
                          const std::function<void(size_t, const SimResult &)> &onResult) {
  const bool root = ctrl.rank() == 0;
  const double t0 = wtime();
  SearchResult result;
  result.opts = opts.json();

  auto gp = std::make_shared<Graph>(g);
  gp->normalize();
  State rootState(gp, plat);
  OpIndex index(*gp);

  Tree tree;
  tree.strat = make_strategy(opts.strategy, opts.seed + 1);
  tree.rng.seed(opts.seed);
  tree.c = opts.explore_c;
  std::unordered_map<std::string, size_t> cache; // canonical key -> sims index

  if (root && !opts.resume_path.empty()) {
    std::ifstream f(opts.resume_path);
    TZ_CHECK(f, "cannot open checkpoint " << opts.resume_path);
    std::stringstream ss;
    ss << f.rdbuf();
    Json ck = Json::parse(ss.str());
    tree.load(tree.root, ck.at("tree"), rootState);
    for (const auto &s : ck.at("sims").as_array()) {
      SimResult sr;
      sr.seq = index.sequence_from_json(s.at("seq"));
      const Json &r = s.at("result");
      sr.res.pct01 = r.at("pct01").as_double();
      sr.res.pct10 = r.at("pct10").as_double();
      sr.res.pct50 = r.at("pct50").as_double();
      sr.res.pct90 = r.at("pct90").as_double();
      sr.res.pct99 = r.at("pct99").as_double();
      sr.res.stddev = r.at("stddev").as_double();
      if (s.contains("seeded")) sr.seeded = s.at("seeded").as_bool();
      cache.emplace(sr.seq.canonical_key(), result.sims.size());
      result.sims.push_back(sr);
    }
    TZ_LOG(Info, "resumed MCTS: tree size " << tree.root.size() << ", " << result.sims.size()
                                            << " results");
  }

  // transports some rank already saw die (an earlier search of this process): agreed before the
  // first candidate, so every rank prunes the same alternatives
  tree.dead = agree_dead_domains(ctrl);
  auto after_failure = [&] {
    // collective (every rank reaches it: failures are agreed on): reset the transports if a
    // run was aborted anywhere, then adopt what any rank saw die
    recover_after_abort(ctrl);
    const size_t before = tree.dead.size();
    tree.dead = agree_dead_domains(ctrl);
    if (root && tree.dead.size() > before)
      TZ_LOG(Warn, "pruning every alternative that needs a dead transport (" << tree.dead.size()
                                                                            << " dead)");
  };
  auto seq_dead = [&](const Sequence &s) {
    for (const auto &e : s.entries)
      if (uses_domain(e.op, tree.dead)) return true;
    return false;
  };

  // seed schedules: every rank measures them first (collectively, like any candidate)
  const int64_t nSeeds = ctrl.bcast_int(root ? int64_t(opts.seed_schedules.size()) : 0, 0);
  for (int64_t k = 0; k < nSeeds; ++k) {
    // rank 0 checks the seed; a refusal travels with the broadcast so every rank throws together
    Json m;
    if (root) {
      const Sequence &s = opts.seed_schedules[size_t(k)];
      try {
        if (opts.verify) {
          auto v = verify(s, *resolve_graph(*gp, s), plat.n_streams);
          TZ_CHECK(v.empty(), "seed schedule " << k << " has a race: " << v[0].desc());
        }
        if (seq_dead(s)) m["dead"] = true;
        else m["seq"] = s.json(true);
      } catch (const std::exception &e) {
        m["err"] = std::string(e.what());
      }
    }
    std::string msg = root ? m.dump() : "";
    ctrl.bcast(msg, 0);
    m = Json::parse(msg);
    if (m.contains("err")) TZ_THROW(m.at("err").as_string());
    if (m.contains("dead")) {
      if (root) TZ_LOG(Warn, "seed schedule " << k << " skipped: it needs a dead transport");
      continue;
    }
    Sequence s = root ? opts.seed_schedules[size_t(k)] : index.sequence_from_json(m.at("seq"));
    SimResult sr;
    sr.seq = s;
    sr.seeded = true;
    try {
      ScopedTimer t(result.counters, "BENCHMARK");
      sr.res = bench.benchmark(s, opts.bench);
    } catch (const std::exception &e) {
      if (!opts.skip_failed || !skippable(e, ctrl)) throw;
      if (root) {
        ++result.failed;
        TZ_LOG(Warn, "seed schedule " << k << " skipped: " << e.what());
      }
      after_failure();
      continue;
    }
    if (root) {
      cache.emplace(s.canonical_key(), result.sims.size());
      // the search looks candidates up after its redundant-sync removal: a seed that still
      // carries a redundant sync is found under the key of its reduced form too
      if (opts.remove_redundant_syncs) {
        try {
          Sequence r = s;
          if (remove_redundant_syncs(r, *resolve_graph(*gp, s), plat.n_streams) > 0)
            cache.emplace(r.canonical_key(), result.sims.size());
        } catch (const std::exception &) {
          // a seed the reduction cannot replay keeps its own key only
        }
      }
      result.sims.push_back(sr);
      if (onResult) onResult(result.sims.size() - 1, sr);
      // its result steers the search from where the seed sits in the tree
      MctsNode *leaf = seed_path(tree, rootState, s, opts.remove_redundant_syncs, plat.n_streams);
      if (leaf) {
        tree.backprop(leaf, sr.res);
        result.counters.add("SEED_IN_TREE", 0.0);
      }
      TZ_LOG(Info, "seed schedule " << k << " pct10=" << sr.res.pct10
                                    << (leaf ? " (in the tree)" : " (no tree path)"));
    }
  }

  std::function<void(int)> dump = [&result](int) { result.dump_csv(std::cout); };
  if (root && opts.trap_signals) register_handler(dump);

  auto checkpoint = [&]() {
    if (!root || opts.checkpoint_path.empty()) return;
    Json ck;
    ck["tree"] = tree.save(tree.root);
    Json sims = Json::array();
    for (const auto &s : result.sims) {
      Json j;
      j["result"] = s.res.json();
      j["seq"] = s.seq.json();
      if (s.seeded) j["seeded"] = true;
      sims.push_back(j);
    }
    ck["sims"] = sims;
    ck["opts"] = opts.json();
    write_file(opts.checkpoint_path + ".tmp", ck.dump());
    std::rename((opts.checkpoint_path + ".tmp").c_str(), opts.checkpoint_path.c_str());
  };

  Counters &C = result.counters;
  for (int64_t iter = 0;; ++iter) {
    int64_t stop = 0;
    if (root) {
      if (tree.root.fully_visited) {
        stop = 1;
        result.stop_reason = "full_tree";
      } else if (opts.n_iters > 0 && iter >= opts.n_iters) {
        stop = 2;
        result.stop_reason = "iterations";
      } else if (opts.time_budget_s > 0 && wtime() - t0 > opts.time_budget_s) {
        stop = 3;
        result.stop_reason = "time_budget";
      } else if (opts.max_tree_nodes > 0 && tree.nodes >= size_t(opts.max_tree_nodes)) {
        // reference Stop::Reason::large_tree (mcts.hpp:131): bounds the host memory of the tree
        stop = 5;
        result.stop_reason = "large_tree";
      }
      if (opts.trap_signals && signal_pending()) {
        stop = 4;
        result.stop_reason = "signal";
      }
    }
    stop = ctrl.bcast_int(stop, 0);
    if (stop == 4) {
      // trapped signal on rank 0: every rank leaves together, rank 0 dumps the partial results
      ctrl.barrier();
      if (root) handle_pending_signal();
      std::exit(1);
    }
    if (stop) break;

    std::string msg;
    MctsNode *bpStart = nullptr;
    size_t cachedIdx = size_t(-1);
    Sequence seq;
    if (root) {
      // one descent: select, expand, roll out. A descent that runs into decisions needing a
      // dead transport prunes them and starts over (bounded); if nothing live is left the
      // iteration measures nothing and the next one stops on the fully visited tree.
      bool found = false;
      for (int attempt = 0; attempt < 64 && !found && !tree.root.fully_visited; ++attempt) {
        State st = rootState;
        MctsNode *node = &tree.root;
        bool dead = false;
        {
          ScopedTimer t(C, "SELECT");
          while (!node->is_leaf() && !node->terminal) {
            if (!tree.prune_dead_children(*node, st)) {
              dead = true;
              break;
            }
            node = tree.pick_uct(*node);
            st.apply_inplace(node->decision);
          }
        }
        if (dead) continue;
        {
          ScopedTimer t(C, "EXPAND");
          tree.ensure_children(*node, st);
          if (!node->children.empty()) {
            if (!tree.prune_dead_children(*node, st)) continue;
            MctsNode *next = nullptr;
            for (auto &ch : node->children)
              if (ch->n == 0 && !ch->fully_visited) {
                next = ch.get();
                break;
              }
            if (!next) next = tree.pick_uct(*node);
            node = next;
            st.apply_inplace(node->decision);
          }
        }
        {
          ScopedTimer t(C, "ROLLOUT");
          bpStart = node;
          MctsNode *cur = node;
          std::vector<size_t> live;
          while (!st.complete() && !dead) {
            if (opts.expand_rollout) {
              tree.ensure_children(*cur, st);
              TZ_CHECK(!cur->children.empty(), "dead-end state during rollout");
              live.clear();
              for (size_t i = 0; i < cur->children.size(); ++i)
                if (!tree.dead_decision(st, cur->children[i]->decision)) live.push_back(i);
              if (live.empty()) {
                tree.prune_dead_children(*cur, st);
                dead = true;
                break;
              }
              std::uniform_int_distribution<size_t> u(0, live.size() - 1);
              cur = cur->children[live[u(tree.rng)]].get();
              st.apply_inplace(cur->decision);
              bpStart = cur;
            } else {
              auto ds = st.get_decisions();
              TZ_CHECK(!ds.empty(), "dead-end state during rollout");
              live.clear();
              for (size_t i = 0; i < ds.size(); ++i)
                if (!tree.dead_decision(st, ds[i])) live.push_back(i);
              if (live.empty()) {
                dead = true;
                break;
              }
              std::uniform_int_distribution<size_t> u(0, live.size() - 1);
              st.apply_inplace(ds[live[u(tree.rng)]]);
            }
          }
          // a rollout that reached a state whose every decision needs a dead transport: that
          // node was pruned (prune_dead_children marks it and its ancestors as far as they are
          // exhausted); try another descent
          if (dead) continue;
          if (opts.expand_rollout) tree.ensure_children(*cur, st);
        }
        seq = st.sequence();
        if (opts.remove_redundant_syncs) {
          ScopedTimer t(C, "REDUNDANT_SYNC");
          remove_redundant_syncs(seq, st.graph(), plat.n_streams);
        }
        if (opts.verify) {
          ScopedTimer t(C, "VERIFY");
          auto v = verify(seq, st.graph(), plat.n_streams);
          if (!v.empty()) TZ_THROW("candidate schedule has a race: " << v[0].desc());
        }
        found = true;
      }
      Json m;
      if (!found) {
        m["skip"] = true;
      } else {
        if (opts.reuse_measurements) {
          auto it = cache.find(seq.canonical_key());
          if (it != cache.end()) cachedIdx = it->second;
        }
        m["cached"] = cachedIdx != size_t(-1);
        m["seq"] = seq.json(true);
      }
      msg = m.dump();
    }
    {
      ScopedTimer t(C, "BCAST");
      ctrl.bcast(msg, 0);
    }
    Json m = Json::parse(msg);
    if (m.contains("skip")) continue; // no live candidate: the next iteration stops
    const bool cached = m.at("cached").as_bool();
    if (!root) seq = index.sequence_from_json(m.at("seq"));

    BenchResult br;
    bool failed = false;
    if (!cached) {
      ScopedTimer t(C, "BENCHMARK");
      if (opts.skip_failed) {
        // preparation and run failures (e.g. a schedule that cannot be compiled to a hipGraph)
        // are agreed on collectively by the benchmarker, so every rank skips the same candidate
        try {
          br = bench.benchmark(seq, opts.bench);
        } catch (const std::exception &e) {
          if (!skippable(e, ctrl)) throw;
          failed = true;
          if (root) TZ_LOG(Warn, "mcts iter " << iter << ": candidate skipped: " << e.what());
        }
      } else {
        br = bench.benchmark(seq, opts.bench);
      }
    }
    if (failed) {
      if (root) {
        ++result.failed;
        tree.prune_failed(bpStart);
      }
      after_failure();
      continue;
    }
    if (root) {
      SimResult sr;
      sr.seq = seq;
      if (cached) {
        sr.res = result.sims[cachedIdx].res;
        sr.cached = true;
      } else {
        sr.res = br;
        cache.emplace(seq.canonical_key(), result.sims.size());
      }
      result.sims.push_back(sr);
      {
        ScopedTimer t(C, "BACKPROP");
        tree.backprop(bpStart, sr.res);
      }
      if (onResult) onResult(result.sims.size() - 1, sr);
      TZ_LOG(Info, "mcts iter " << iter << " pct10=" << sr.res.pct10 << (cached ? " (cached)" : "")
                                << " tree=" << tree.root.size());
      if (opts.dump_tree && (iter < 10 || (iter < 50 && iter % 10 == 0) ||
                             (iter < 100 && iter % 25 == 0))) {
        write_file(opts.dump_tree_prefix + std::to_string(iter) + ".dot",
                   mcts_tree_graphviz(tree.root, *tree.strat));
      }
      if (opts.checkpoint_every > 0 && (iter + 1) % opts.checkpoint_every == 0) checkpoint();
    }
  }
  ctrl.barrier();
  if (root) {
    unregister_handler();
    checkpoint();
    result.tree_size = tree.root.size();
    result.tree_fully_visited = tree.root.fully_visited_size();
  }
  result.dead_domains.assign(tree.dead.begin(), tree.dead.end());
  result.pruned_dead = tree.prunedDead;
  result.wall_s = wtime() - t0;
  return result;
}

// ======================================================================== DFS

Json DfsOpts::json() const {
  Json j, o;
  o["maxSeqs"] = max_seqs;
  j["dfs__Opts"] = o;
  return j;
}

std::vector<Sequence> get_all_sequences(const Graph &g, const Platform &plat, int64_t maxSeqs,
                                        bool dedupStates, bool removeRedundant) {
  auto gp = std::make_shared<Graph>(g);
  gp->normalize();
  std::vector<State> work{State(gp, plat)};
  std::unordered_set<std::string> seenStates, seenSeqs;
  std::vector<Sequence> out;
  while (!work.empty()) {
    if (maxSeqs >= 0 && int64_t(out.size()) >= maxSeqs) break;
    State cur = std::move(work.back());
    work.pop_back();
    if (cur.complete()) {
      Sequence s = cur.sequence();
      if (removeRedundant) remove_redundant_syncs(s, cur.graph(), plat.n_streams);
      if (seenSeqs.insert(s.canonical_key()).second) out.push_back(std::move(s));
      continue;
    }
    auto ds = cur.get_decisions();
    // push in reverse so the first decision is explored first
    for (auto it = ds.rbegin(); it != ds.rend(); ++it) {
      State nx = cur.apply(*it);
      if (dedupStates && !seenStates.insert(nx.canonical_key()).second) continue;
      work.push_back(std::move(nx));
    }
  }
  return out;
}

SearchResult dfs_explore(const Graph &g, const Platform &plat, Benchmarker &bench, Ctrl &ctrl,
                         const DfsOpts &opts,
                         const std::function<void(size_t, const SimResult &)> &onResult) {
  const bool root = ctrl.rank() == 0;
  const double t0 = wtime();
  SearchResult result;
  result.opts = opts.json();
  auto gp = std::make_shared<Graph>(g);
  gp->normalize();
  OpIndex index(*gp);
  std::vector<Sequence> seqs;
  if (root) {
    ScopedTimer t(result.counters, "ENUMERATE");
    seqs = get_all_sequences(*gp, plat, opts.max_seqs, opts.dedup_states, opts.remove_redundant_syncs);
  }
  std::function<void(int)> dump = [&result](int) { result.dump_csv(std::cout); };
  if (root && opts.trap_signals) register_handler(dump);
  std::set<std::string> dead = agree_dead_domains(ctrl);
  auto seq_dead = [&](const Sequence &s) {
    for (const auto &e : s.entries)
      if (uses_domain(e.op, dead)) return true;
    return false;
  };
  for (size_t i = 0;; ++i) {
    // sequences that need a transport that died are not measured (rank 0 decides, the others
    // follow the broadcast sequence)
    while (root && i < seqs.size() && !dead.empty() && seq_dead(seqs[i])) {
      ++i;
      ++result.pruned_dead;
    }
    int64_t stop = root ? int64_t(i >= seqs.size()) : 0;
    if (root && opts.trap_signals && signal_pending()) stop = 4;
    stop = ctrl.bcast_int(stop, 0);
    if (stop == 4) {
      ctrl.barrier();
      if (root) handle_pending_signal();
      std::exit(1);
    }
    if (stop) break;
    std::string msg;
    if (root) msg = seqs[i].json(true).dump();
    ctrl.bcast(msg, 0);
    Sequence seq = root ? seqs[i] : index.sequence_from_json(Json::parse(msg));
    SimResult sr;
    sr.seq = seq;
    {
      ScopedTimer t(result.counters, "BENCHMARK");
      try {
        sr.res = bench.benchmark(seq, opts.bench);
      } catch (const std::exception &e) {
        // collective failure: every rank skips this sequence
        if (!opts.skip_failed || !skippable(e, ctrl)) throw;
        if (root) {
          ++result.failed;
          TZ_LOG(Warn, "dfs sequence " << i << " skipped: " << e.what());
        }
        recover_after_abort(ctrl);
        dead = agree_dead_domains(ctrl);
        continue;
      }
    }
    if (root) {
      result.sims.push_back(sr);
      if (onResult) onResult(result.sims.size() - 1, sr);
    }
  }
  result.dead_domains.assign(dead.begin(), dead.end());
  ctrl.barrier();
  if (root) unregister_handler();
  result.stop_reason = "enumerated";
  result.wall_s = wtime() - t0;
  return result;
}

// ======================================================================== trap / reproduce

namespace {
std::function<void(int)> g_handler;
volatile std::sig_atomic_t g_pending = 0;
struct sigaction g_old[3];
const int kTrapped[3] = {SIGINT, SIGTERM, SIGABRT};
bool g_installed = false;

void trap_fn(int sig) {
  // async-signal-safe: only flag the signal (the search loop dumps between candidates); a
  // second signal while the first is pending ends the process at once
  if (g_pending) {
    static const char msg[] = "[tz] second signal: exiting without dump\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    std::_Exit(1);
  }
  g_pending = sig;
}
} // namespace

void register_handler(std::function<void(int)> fn) {
  g_handler = std::move(fn);
  g_pending = 0;
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = trap_fn;
  sigemptyset(&sa.sa_mask);
  for (int i = 0; i < 3; ++i) sigaction(kTrapped[i], &sa, &g_old[i]);
  g_installed = true;
}

void unregister_handler() {
  // restore whatever was installed before (e.g. Python's own SIGINT handler)
  if (g_installed)
    for (int i = 0; i < 3; ++i) sigaction(kTrapped[i], &g_old[i], nullptr);
  g_installed = false;
  g_handler = nullptr;
}

int signal_pending() { return int(g_pending); }

void handle_pending_signal() {
  const int sig = int(g_pending);
  if (g_handler) g_handler(sig);
  std::cout.flush();
  std::fflush(stdout);
  std::exit(1);
}

struct RunDeadline::Impl {
  std::mutex mu;
  std::condition_variable cv;
  std::string report;
  bool done = false;
  double end = 0;                                // wtime() of expiry (remaining())
  std::chrono::steady_clock::time_point until;   // the same instant, for the waiting thread
  uint64_t gen = 0;                              // bumped by tighten(): re-wait
  int code = 5;
  std::thread th;
};

namespace {
// the armed deadline whose report a fatal exit prints (the newest one armed)
std::atomic<RunDeadline::Impl *> g_armedDeadline{nullptr};

// write a whole line with write(2): no locks other threads might hold, no stdio buffers
void write_all(int fd, const std::string &line) {
  const char *at = line.data();
  size_t left = line.size();
  while (left > 0) {
    const ssize_t w = ::write(fd, at, left);
    if (w <= 0) break;
    at += w;
    left -= size_t(w);
  }
}

// the report line with the reason for the early exit added, if it is a JSON object
std::string with_reason(std::string line, const std::string &why) {
  while (!line.empty() && (line.back() == '\n' || line.back() == ' ')) line.pop_back();
  if (!why.empty() && line.size() > 2 && line.front() == '{' && line.back() == '}') {
    std::string esc;
    for (char c : why) {
      if (c == '"' || c == '\\') esc += '\\';
      if (static_cast<unsigned char>(c) >= 0x20) esc += c;
    }
    line.pop_back();
    line += ", \"exit_reason\": \"" + esc + "\"}";
  }
  if (!line.empty()) line += '\n';
  return line;
}
} // namespace

void exit_with_report(int code, const std::string &why) {
  std::string line;
  if (RunDeadline::Impl *p = g_armedDeadline.load()) {
    // the lock is only ever held for a string copy: a bounded wait for it
    for (int k = 0; k < 200; ++k) {
      std::unique_lock<std::mutex> lk(p->mu, std::try_to_lock);
      if (lk.owns_lock()) {
        if (!p->done) line = p->report;
        p->done = true; // the deadline thread must not print it a second time
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
  if (!line.empty()) write_all(1, with_reason(line, why));
  write_all(2, "[tz] exiting with status " + std::to_string(code) + ": " + why +
                   (line.empty() ? "\n" : " (partial result printed)\n"));
  std::_Exit(code);
}

RunDeadline::RunDeadline(double seconds, int exitCode) : p_(std::make_unique<Impl>()) {
  p_->end = wtime() + seconds;
  p_->until = std::chrono::steady_clock::now() +
              std::chrono::microseconds(int64_t(std::max(0.0, seconds) * 1e6));
  p_->code = exitCode;
  Impl *p = p_.get();
  g_armedDeadline = p;
  p_->th = std::thread([p, seconds] {
    std::unique_lock<std::mutex> lk(p->mu);
    for (;;) {
      const uint64_t gen = p->gen;
      const auto until = p->until;
      if (p->cv.wait_until(lk, until, [p, gen] { return p->done || p->gen != gen; })) {
        if (p->done) return;
        continue; // tightened: wait for the new instant
      }
      break;
    }
    // expired: report and leave; no locks other threads might hold, no stdio buffers
    p->done = true; // (a fatal exit racing this one must not print the line again)
    std::string line = p->report;
    if (!line.empty() && line.back() != '\n') line += '\n';
    write_all(1, line);
    char msg[200];
    const int n = std::snprintf(msg, sizeof(msg),
                                "[tz] run deadline reached (%.0f s from the start): %s; exiting with status %d\n",
                                seconds, p->report.empty() ? "nothing to report" : "report printed",
                                p->code);
    if (n > 0) (void)!::write(2, msg, size_t(std::min<int>(n, int(sizeof(msg) - 1))));
    std::_Exit(p->code);
  });
}

void RunDeadline::tighten(double seconds, int exitCode) {
  {
    std::lock_guard<std::mutex> lk(p_->mu);
    if (p_->done) return;
    const double end = wtime() + std::max(0.0, seconds);
    if (end < p_->end) {
      p_->end = end;
      p_->until = std::chrono::steady_clock::now() +
                  std::chrono::microseconds(int64_t(std::max(0.0, seconds) * 1e6));
    }
    p_->code = exitCode;
    ++p_->gen;
  }
  p_->cv.notify_all();
}

RunDeadline::~RunDeadline() {
  cancel();
  if (p_->th.joinable()) p_->th.join();
  Impl *mine = p_.get();
  g_armedDeadline.compare_exchange_strong(mine, nullptr);
}

void RunDeadline::set_report(const std::string &line) {
  std::lock_guard<std::mutex> lk(p_->mu);
  p_->report = line;
}

void RunDeadline::cancel() {
  {
    std::lock_guard<std::mutex> lk(p_->mu);
    p_->done = true;
  }
  p_->cv.notify_all();
}

double RunDeadline::remaining() const { return p_->end - wtime(); }

bool RunDeadline::armed() const {
  std::lock_guard<std::mutex> lk(p_->mu);
  return !p_->done;
}

std::string version_string() {
  std::ostringstream ss;
  ss << TZ_VERSION_MAJOR << "." << TZ_VERSION_MINOR << "." << TZ_VERSION_PATCH << "+" << TZ_GIT_HASH;
  return ss.str();
}

Json reproduce_json(const std::vector<std::string> &args) {
  Json j;
  j["major"] = TZ_VERSION_MAJOR;
  j["minor"] = TZ_VERSION_MINOR;
  j["patch"] = TZ_VERSION_PATCH;
  j["hash"] = TZ_GIT_HASH;
  Json a = Json::array();
  for (const auto &s : args) a.push_back(s);
  j["args"] = a;
  return j;
}

} // namespace tz
