#include "graph.hpp"
#include "util.hpp"

#include <algorithm>
#include <functional>
#include <queue>
#include <sstream>

namespace tz {

Graph::Graph() {
  nodes_.push_back(Node{std::make_shared<Start>(), {}, {}, true});
  nodes_.push_back(Node{std::make_shared<Finish>(), {}, {}, true});
  by_name_["Start"] = kStart;
  by_name_["Finish"] = kFinish;
  n_alive_ = 2;
}

int Graph::add(const OpPtr &op) {
  TZ_CHECK(op, "null op");
  if (op->op_class() == OpClass::Start) return kStart;
  if (op->op_class() == OpClass::Finish) return kFinish;
  const std::string n = op->name();
  auto it = by_name_.find(n);
  if (it != by_name_.end()) {
    if (it->second >= 0 && nodes_[it->second].alive) {
      const OpPtr &have = nodes_[it->second].op;
      if (have.get() != op.get() && !have->eq(*op)) {
        TZ_THROW("graph already has a different op named '" << n << "'");
      }
      return it->second;
    }
  }
  int id = int(nodes_.size());
  nodes_.push_back(Node{op, {}, {}, true});
  by_name_[n] = id;
  ++n_alive_;
  return id;
}

void Graph::add_edge(int a, int b) {
  TZ_CHECK(a != b, "self edge on " << nodes_[a].op->name());
  TZ_CHECK(b != kStart, "edge into Start");
  TZ_CHECK(a != kFinish, "edge out of Finish");
  auto &s = nodes_[a].succs;
  if (std::find(s.begin(), s.end(), b) != s.end()) return;
  s.push_back(b);
  nodes_[b].preds.push_back(a);
}

void Graph::then(const OpPtr &a, const OpPtr &b) {
  // copies first: `a` / `b` may alias nodes_ storage (start_op()/finish_op()) that add() can
  // reallocate
  const OpPtr pa = a, pb = b;
  const int ia = add(pa);
  const int ib = add(pb);
  add_edge(ia, ib);
}

void Graph::normalize() {
  for (int id = 2; id < capacity(); ++id) {
    if (!alive(id)) continue;
    if (nodes_[id].preds.empty()) add_edge(kStart, id);
    if (nodes_[id].succs.empty()) add_edge(id, kFinish);
  }
  if (nodes_[kStart].succs.empty()) add_edge(kStart, kFinish);
  // drop a direct Start->Finish edge if other paths exist (reference start_then semantics)
  if (nodes_[kStart].succs.size() > 1) {
    auto &s = nodes_[kStart].succs;
    auto it = std::find(s.begin(), s.end(), kFinish);
    if (it != s.end()) {
      s.erase(it);
      auto &p = nodes_[kFinish].preds;
      p.erase(std::find(p.begin(), p.end(), kStart));
    }
  }
}

int Graph::find(const std::string &name) const {
  auto it = by_name_.find(name);
  if (it == by_name_.end()) return -1;
  return nodes_[it->second].alive ? it->second : -1;
}

std::vector<int> Graph::vertices() const {
  std::vector<int> v;
  for (int i = 0; i < capacity(); ++i)
    if (alive(i)) v.push_back(i);
  return v;
}

int Graph::num_edges() const {
  int n = 0;
  for (const auto &nd : nodes_)
    if (nd.alive) n += int(nd.succs.size());
  return n;
}

std::vector<int> Graph::topo_order() const {
  std::vector<int> indeg(capacity(), 0), out;
  for (int i = 0; i < capacity(); ++i)
    if (alive(i)) indeg[i] = int(nodes_[i].preds.size());
  std::priority_queue<int, std::vector<int>, std::greater<int>> q;
  for (int i = 0; i < capacity(); ++i)
    if (alive(i) && indeg[i] == 0) q.push(i);
  while (!q.empty()) {
    int u = q.top();
    q.pop();
    out.push_back(u);
    for (int v : nodes_[u].succs)
      if (--indeg[v] == 0) q.push(v);
  }
  TZ_CHECK(int(out.size()) == n_alive_, "graph has a cycle");
  return out;
}

void Graph::erase(int id) {
  TZ_CHECK(id != kStart && id != kFinish, "cannot erase Start/Finish");
  Node &n = nodes_[id];
  for (int p : n.preds) {
    auto &s = nodes_[p].succs;
    s.erase(std::remove(s.begin(), s.end(), id), s.end());
  }
  for (int s : n.succs) {
    auto &p = nodes_[s].preds;
    p.erase(std::remove(p.begin(), p.end(), id), p.end());
  }
  n.preds.clear();
  n.succs.clear();
  n.alive = false;
  by_name_.erase(n.op->name());
  --n_alive_;
}

void Graph::erase_edge(int a, int b) {
  TZ_CHECK(a >= 0 && a < capacity() && b >= 0 && b < capacity(), "bad vertex id");
  auto &s = nodes_[a].succs;
  s.erase(std::remove(s.begin(), s.end(), b), s.end());
  auto &p = nodes_[b].preds;
  p.erase(std::remove(p.begin(), p.end(), a), p.end());
}

std::shared_ptr<Graph> Graph::clone_but_replace(int id, const OpPtr &replacement) const {
  auto g = clone();
  TZ_CHECK(id >= 0 && id < capacity() && alive(id), "bad vertex id " << id);
  const std::string oldName = g->nodes_[id].op->name();
  g->by_name_.erase(oldName);
  g->nodes_[id].op = replacement;
  const std::string newName = replacement->name();
  auto it = g->by_name_.find(newName);
  TZ_CHECK(it == g->by_name_.end(), "replacement name '" << newName << "' already in graph");
  g->by_name_[newName] = id;
  return g;
}

std::shared_ptr<Graph> Graph::clone_but_expand(int id, const Graph &subIn) const {
  Graph sub = subIn;
  sub.normalize();
  auto g = clone();
  TZ_CHECK(alive(id), "expand of dead vertex");
  const std::vector<int> outerPreds = nodes_[id].preds;
  const std::vector<int> outerSuccs = nodes_[id].succs;
  g->erase(id);

  // map sub vertex -> new id in g
  std::vector<int> map(sub.capacity(), -1);
  for (int v = 0; v < sub.capacity(); ++v) {
    if (!sub.alive(v) || v == kStart || v == kFinish) continue;
    map[v] = g->add(sub.op(v));
  }
  for (int u = 0; u < sub.capacity(); ++u) {
    if (!sub.alive(u)) continue;
    for (int v : sub.succs(u)) {
      std::vector<int> from, to;
      if (u == kStart) from = outerPreds;
      else from = {map[u]};
      if (v == kFinish) to = outerSuccs;
      else to = {map[v]};
      for (int a : from)
        for (int b : to) g->add_edge(a, b);
    }
  }
  return g;
}

std::string Graph::dump_graphviz(const std::string &title) const {
  std::ostringstream ss;
  ss << "digraph D {\n";
  if (!title.empty()) ss << "  label=\"" << title << "\";\n";
  for (int i = 0; i < capacity(); ++i) {
    if (!alive(i)) continue;
    const OpPtr &op = nodes_[i].op;
    std::string shape = "box";
    switch (op->op_class()) {
    case OpClass::Gpu:
    case OpClass::BoundGpu: shape = "ellipse"; break;
    case OpClass::Compound: shape = "box3d"; break;
    case OpClass::Choice: shape = "diamond"; break;
    case OpClass::Start:
    case OpClass::Finish: shape = "oval"; break;
    default: break;
    }
    ss << "  op_" << i << " [label=\"" << op->desc() << "\", shape=" << shape << "];\n";
  }
  for (int i = 0; i < capacity(); ++i) {
    if (!alive(i)) continue;
    for (int s : nodes_[i].succs) ss << "  op_" << i << " -> op_" << s << ";\n";
  }
  ss << "}\n";
  return ss.str();
}

Json Graph::json() const {
  Json j;
  Json vs = Json::array(), es = Json::array();
  for (int i = 0; i < capacity(); ++i) {
    if (!alive(i)) continue;
    Json v = nodes_[i].op->json();
    v["id"] = i;
    v["class"] = op_class_name(nodes_[i].op->op_class());
    vs.push_back(v);
    for (int s : nodes_[i].succs) {
      Json e = Json::array();
      e.push_back(i);
      e.push_back(s);
      es.push_back(e);
    }
  }
  j["vertices"] = vs;
  j["edges"] = es;
  return j;
}

static void collect_rec(const OpPtr &op, std::unordered_map<std::string, OpPtr> &out) {
  if (op->op_class() == OpClass::Compound) {
    auto c = std::dynamic_pointer_cast<const CompoundOp>(op);
    auto sub = collect_ops(*c->graph());
    for (auto &kv : sub)
      if (kv.second->op_class() != OpClass::Start && kv.second->op_class() != OpClass::Finish)
        out.emplace(kv.first, kv.second);
  } else if (op->op_class() == OpClass::Choice) {
    auto c = std::dynamic_pointer_cast<const ChoiceOp>(op);
    for (const auto &ch : c->choices()) collect_rec(ch, out);
  }
  out.emplace(op->name(), op);
}

std::unordered_map<std::string, OpPtr> collect_ops(const Graph &g) {
  std::unordered_map<std::string, OpPtr> out;
  for (int i = 0; i < g.capacity(); ++i)
    if (g.alive(i)) collect_rec(g.op(i), out);
  return out;
}

} // namespace tz
