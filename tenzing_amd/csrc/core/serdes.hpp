// Schedule (de)serialization in the reference's JSON schema and results CSV format.
//
// Parity: reference include/tenzing/operation_serdes.hpp:14-47, src/operation_serdes.cpp:14-76
// (name lookup in the graph, recursing into CompoundOp graphs and ChoiceOp choices; GPU ops
// re-bound from "stream"; ops absent from the graph rebuilt from "kind"), src/sequence.cpp:88-125
// (sequence broadcast as JSON text), tenzing-dfs/src/dfs.cpp:84-105 and
// tenzing-mcts/src/mcts.cpp:13-31 (CSV rows `i|p01|p10|p50|p90|p99|stddev|op-json|...`).
// Unlike the reference, StreamWait and StreamSync are deserializable too, and "Hip*" kind
// aliases are accepted.
#pragma once

#include "state.hpp"

#include <unordered_map>

namespace tz {

class OpIndex {
public:
  explicit OpIndex(const Graph &g) : ops_(collect_ops(g)) {}
  BoundOpPtr from_json(const Json &j) const;
  Sequence sequence_from_json(const Json &arr) const;
  OpPtr find(const std::string &name) const {
    auto it = ops_.find(name);
    return it == ops_.end() ? nullptr : it->second;
  }

private:
  std::unordered_map<std::string, OpPtr> ops_;
};

/// build a sync op from its JSON (kind must be one of the synchronizer kinds)
BoundOpPtr sync_op_from_json(const Json &j);

} // namespace tz
