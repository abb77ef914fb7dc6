#include "workloads.hpp"

#include <unistd.h>

#include <cstdlib>
#include <fstream>

#include "core/util.hpp"
#include "hip/hip_runtime.hpp"

#include <hip/hip_runtime_api.h>

namespace tz {

DeviceBuffer::DeviceBuffer(size_t bytes) : bytes_(bytes) {
  if (bytes) TZ_HIP(hipMalloc(&p_, bytes));
}

DeviceBuffer::DeviceBuffer(size_t bytes, bool peerWritten) : bytes_(bytes) {
  if (!bytes) return;
  static const bool fine = [] {
    const char *e = std::getenv("TZ_IPC_FINE");
    return !e || std::atoi(e) != 0;
  }();
  if (peerWritten && fine) TZ_HIP(hipExtMallocWithFlags(&p_, bytes, hipDeviceMallocFinegrained));
  else TZ_HIP(hipMalloc(&p_, bytes));
}

DeviceBuffer::~DeviceBuffer() {
  if (p_) (void)hipFree(p_); // teardown: nothing useful to do with an error
}

DeviceBuffer &DeviceBuffer::operator=(DeviceBuffer &&o) noexcept {
  if (this != &o) {
    if (p_) (void)hipFree(p_);
    p_ = o.p_;
    bytes_ = o.bytes_;
    o.p_ = nullptr;
    o.bytes_ = 0;
  }
  return *this;
}

void DeviceBuffer::upload(const void *src, size_t bytes) {
  TZ_CHECK(bytes <= bytes_, "upload overflow");
  if (bytes) TZ_HIP(hipMemcpy(p_, src, bytes, hipMemcpyHostToDevice));
}

void DeviceBuffer::download(void *dst, size_t bytes) const {
  TZ_CHECK(bytes <= bytes_, "download overflow");
  if (bytes) TZ_HIP(hipMemcpy(dst, p_, bytes, hipMemcpyDeviceToHost));
}

std::string node_identity() {
  char host[64] = {0};
  gethostname(host, sizeof(host) - 1);
  std::string id(host);
  std::ifstream f("/proc/sys/kernel/random/boot_id");
  std::string boot;
  if (f) std::getline(f, boot);
  id += "|" + boot;
  id.resize(kNodeIdBytes, '\0');
  return id;
}

void EmptyKernelOp::launch(void *stream, Executor &) const { kern::empty(stream); }

Json BusyKernelOp::json() const {
  Json j;
  j["name"] = name_;
  return j;
}

static int64_t wall_clock_khz() {
  static int64_t khz = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return int64_t(100000);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) != hipSuccess || v <= 0)
      return int64_t(100000);
    return int64_t(v);
  }();
  return khz;
}

void BusyKernelOp::launch(void *stream, Executor &) const {
  kern::busy_wait(int64_t(us_ * double(wall_clock_khz()) / 1000.0), blocks_, stream);
}

} // namespace tz
