#include "serdes.hpp"
#include "util.hpp"

namespace tz {

BoundOpPtr sync_op_from_json(const Json &j) {
  const std::string kind = j.at("kind").as_string();
  const std::string name = j.contains("name") ? j.at("name").as_string() : "";
  if (kind == "CudaEventRecord" || kind == "HipEventRecord")
    return std::make_shared<EventRecord>(int(j.at("event").as_int()), int(j.at("stream").as_int()),
                                         name);
  if (kind == "CudaStreamWaitEvent" || kind == "HipStreamWaitEvent")
    return std::make_shared<StreamWaitEvent>(int(j.at("stream").as_int()),
                                             int(j.at("event").as_int()), name);
  if (kind == "CudaEventSync" || kind == "HipEventSync")
    return std::make_shared<EventSync>(int(j.at("event").as_int()), name);
  if (kind == "StreamSync") return std::make_shared<StreamSync>(int(j.at("stream").as_int()), name);
  if (kind == "StreamWait")
    return std::make_shared<StreamWait>(int(j.at("waiter").as_int()), int(j.at("waitee").as_int()),
                                        name);
  return nullptr;
}

BoundOpPtr OpIndex::from_json(const Json &j) const {
  if (j.contains("kind")) {
    if (auto s = sync_op_from_json(j)) return s;
  }
  const std::string name = j.at("name").as_string();
  OpPtr op = find(name);
  if (!op) TZ_THROW("failure to deserialize (no op named '" << name << "'): " << j.dump());
  if (op->op_class() == OpClass::Gpu) {
    TZ_CHECK(j.contains("stream"), "gpu op " << name << " serialized without a stream");
    return std::make_shared<BoundGpuOp>(std::static_pointer_cast<const GpuOp>(op),
                                        int(j.at("stream").as_int()));
  }
  auto b = std::dynamic_pointer_cast<const BoundOp>(op);
  if (!b) TZ_THROW("op '" << name << "' is not executable (class " << op_class_name(op->op_class())
                          << ")");
  return b;
}

Sequence OpIndex::sequence_from_json(const Json &arr) const {
  Sequence s;
  for (const auto &j : arr.as_array()) s.push_back(from_json(j), -1);
  return s;
}

} // namespace tz
