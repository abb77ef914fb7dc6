#include "ops.hpp"
#include "util.hpp"

#include <chrono>
#include <sstream>
#include <thread>

namespace tz {

const char *op_class_name(OpClass c) {
  switch (c) {
  case OpClass::Start: return "Start";
  case OpClass::Finish: return "Finish";
  case OpClass::Cpu: return "Cpu";
  case OpClass::Gpu: return "Gpu";
  case OpClass::BoundGpu: return "BoundGpu";
  case OpClass::Sync: return "Sync";
  case OpClass::Compound: return "Compound";
  case OpClass::Choice: return "Choice";
  }
  return "?";
}

Json OpBase::json() const {
  Json j;
  j["name"] = name();
  return j;
}

bool OpBase::is_bound() const {
  switch (op_class()) {
  case OpClass::Start:
  case OpClass::Finish:
  case OpClass::Cpu:
  case OpClass::BoundGpu:
  case OpClass::Sync: return true;
  default: return false;
  }
}

bool OpBase::is_cpu_like() const {
  switch (op_class()) {
  case OpClass::Start:
  case OpClass::Finish:
  case OpClass::Cpu:
  case OpClass::Sync: return true;
  default: return false;
  }
}

Json NoOp::json() const {
  Json j;
  j["name"] = name();
  j["kind"] = "NoOp";
  return j;
}

void NoOp::run(Executor &ex) const {
  if (cost_ > 0) ex.host_busy(cost_);
}

void SleepOp::run(Executor &ex) const { ex.host_busy(us_); }

void Executor::host_busy(double us) {
  const double t0 = wtime();
  while ((wtime() - t0) * 1e6 < us) {
  }
}

Json BoundGpuOp::json() const {
  Json j = op_->json();
  j["stream"] = stream_;
  return j;
}

std::string BoundGpuOp::desc() const {
  std::ostringstream ss;
  ss << "{" << name() << ", s:" << stream_ << "}";
  return ss.str();
}

bool BoundGpuOp::eq(const OpBase &o) const {
  auto *b = dynamic_cast<const BoundGpuOp *>(&o);
  return b && b->stream_ == stream_ && b->op_->eq(*op_);
}

void BoundGpuOp::run(Executor &ex) const { ex.launch(*op_, stream_); }

bool SyncOp::eq(const OpBase &o) const {
  auto *s = dynamic_cast<const SyncOp *>(&o);
  return s && s->kind() == kind() && s->stream() == stream() && s->event() == event() &&
         s->stream2() == stream2();
}

EventRecord::EventRecord(int event, int stream, std::string name) : event_(event), stream_(stream) {
  name_ = name.empty() ? "CER-e" + std::to_string(event) + "-s" + std::to_string(stream) : name;
}
Json EventRecord::json() const {
  Json j;
  j["name"] = name();
  j["stream"] = stream_;
  j["event"] = event_;
  j["kind"] = kind();
  return j;
}
std::string EventRecord::desc() const {
  std::ostringstream ss;
  ss << "{" << name() << ", e:" << event_ << ", s:" << stream_ << "}";
  return ss.str();
}
void EventRecord::run(Executor &ex) const { ex.event_record(event_, stream_); }

StreamWaitEvent::StreamWaitEvent(int stream, int event, std::string name)
    : stream_(stream), event_(event) {
  name_ = name.empty() ? "CSWE-s" + std::to_string(stream) + "-e" + std::to_string(event) : name;
}
Json StreamWaitEvent::json() const {
  Json j;
  j["name"] = name();
  j["stream"] = stream_;
  j["event"] = event_;
  j["kind"] = kind();
  return j;
}
std::string StreamWaitEvent::desc() const {
  std::ostringstream ss;
  ss << "{" << name() << ", s:" << stream_ << ", e:" << event_ << "}";
  return ss.str();
}
void StreamWaitEvent::run(Executor &ex) const { ex.stream_wait_event(stream_, event_); }

EventSync::EventSync(int event, std::string name) : event_(event) {
  name_ = name.empty() ? "CES-e" + std::to_string(event) : name;
}
Json EventSync::json() const {
  Json j;
  j["name"] = name();
  j["event"] = event_;
  j["kind"] = kind();
  return j;
}
std::string EventSync::desc() const {
  std::ostringstream ss;
  ss << "{" << name() << ", e:" << event_ << "}";
  return ss.str();
}
void EventSync::run(Executor &ex) const { ex.event_sync(event_); }

StreamSync::StreamSync(int stream, std::string name) : stream_(stream) {
  name_ = name.empty() ? "SS-s" + std::to_string(stream) : name;
}
Json StreamSync::json() const {
  Json j;
  j["name"] = name();
  j["stream"] = stream_;
  j["kind"] = kind();
  return j;
}
std::string StreamSync::desc() const {
  std::ostringstream ss;
  ss << "{" << name() << ", s:" << stream_ << "}";
  return ss.str();
}
void StreamSync::run(Executor &ex) const { ex.stream_sync(stream_); }

StreamWait::StreamWait(int waiter, int waitee, std::string name) : waiter_(waiter), waitee_(waitee) {
  name_ = name.empty() ? "SW-" + std::to_string(waiter) + "-" + std::to_string(waitee) : name;
}
Json StreamWait::json() const {
  Json j;
  j["name"] = name();
  j["waiter"] = waiter_;
  j["waitee"] = waitee_;
  j["kind"] = kind();
  return j;
}
std::string StreamWait::desc() const {
  std::ostringstream ss;
  ss << "{" << name() << ", waiter:" << waiter_ << ", waitee:" << waitee_ << "}";
  return ss.str();
}
void StreamWait::run(Executor &ex) const { ex.stream_wait(waiter_, waitee_); }

} // namespace tz
