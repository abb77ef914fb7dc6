// Operation DAG.
//
// Parity: reference include/tenzing/graph.hpp:19-556 + src/graph.cpp:13-420 (Graph<OpBase>:
// start_then / then / then_finish / clone / clone_but_replace / clone_but_expand / frontier /
// dump_graphviz / get_equivalence). Redesign: vertices are integer ids into a vector (names are
// unique keys) instead of maps keyed by op comparison; vertex ids are stable across
// replace/expand (expansion appends and tombstones), so a search State can keep per-vertex
// overlays (stream binding, executed position) as flat arrays and share one immutable Graph
// among all states that did not expand/choose (no whole-graph clone per decision, cf.
// reference state.cpp:84-100).
#pragma once

#include "ops.hpp"

#include <string>
#include <unordered_map>
#include <vector>

namespace tz {

class Graph {
public:
  static constexpr int kStart = 0;
  static constexpr int kFinish = 1;

  Graph();

  // ---- construction (reference graph.hpp:46-73)
  /// add a vertex (or return the existing one with the same name; throws if a different op
  /// already uses the name)
  int add(const OpPtr &op);
  void then(const OpPtr &a, const OpPtr &b);
  void start_then(const OpPtr &op) { then(start_op(), op); }
  void then_finish(const OpPtr &op) { then(op, finish_op()); }
  void add_edge(int a, int b);
  /// connect every vertex without predecessors to Start and without successors to Finish;
  /// if the graph is empty, connect Start to Finish
  void normalize();

  // ---- queries
  int size() const { return n_alive_; }    // number of live vertices
  int capacity() const { return int(nodes_.size()); } // id bound
  bool alive(int id) const { return nodes_[id].alive; }
  const OpPtr &op(int id) const { return nodes_[id].op; }
  const std::vector<int> &preds(int id) const { return nodes_[id].preds; }
  const std::vector<int> &succs(int id) const { return nodes_[id].succs; }
  int find(const std::string &name) const; // -1 if absent
  bool contains(const std::string &name) const { return find(name) >= 0; }
  const OpPtr &start_op() const { return nodes_[kStart].op; }
  const OpPtr &finish_op() const { return nodes_[kFinish].op; }
  std::vector<int> vertices() const; // live ids, ascending
  std::vector<int> topo_order() const;
  int num_edges() const;

  // ---- transforms (return new graphs; ids of untouched vertices are preserved)
  std::shared_ptr<Graph> clone() const { return std::make_shared<Graph>(*this); }
  std::shared_ptr<Graph> clone_but_replace(int id, const OpPtr &replacement) const;
  /// replace vertex `id` by the contents of `sub` (its Start/Finish are merged into id's
  /// predecessors/successors, reference graph.hpp:162-219). New vertices get fresh ids.
  std::shared_ptr<Graph> clone_but_expand(int id, const Graph &sub) const;
  void erase(int id);
  /// remove the edge a -> b if present (reference Graph::erase_edge_only, graph.hpp:448-471)
  void erase_edge(int a, int b);

  // ---- output
  std::string dump_graphviz(const std::string &title = "") const;
  Json json() const;

private:
  struct Node {
    OpPtr op;
    std::vector<int> preds, succs;
    bool alive = true;
  };
  std::vector<Node> nodes_;
  std::unordered_map<std::string, int> by_name_;
  int n_alive_ = 0;
};

using GraphPtr = std::shared_ptr<const Graph>;

/// Collect every op reachable by name from a graph, descending into CompoundOp sub-graphs and
/// ChoiceOp alternatives (used by deserialization, reference operation_serdes.cpp:14-76).
std::unordered_map<std::string, OpPtr> collect_ops(const Graph &g);

} // namespace tz
