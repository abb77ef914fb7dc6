#include "workloads.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

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
  if (peerWritten) TZ_HIP(hipExtMallocWithFlags(&p_, bytes, hipDeviceMallocFinegrained));
  else TZ_HIP(hipMalloc(&p_, bytes));
}

double preflight_limit_s(double dflt) {
  const char *e = std::getenv("TZ_PREFLIGHT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : dflt;
}

SharedHostBuffer SharedHostBuffer::create(const std::string &name, size_t bytes) {
  TZ_CHECK(bytes > 0 && !name.empty() && name[0] == '/', "bad shared buffer " << name);
  SharedHostBuffer b;
  const int fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  TZ_CHECK(fd >= 0, "shm_open(" << name << "): " << std::strerror(errno));
  b.name_ = name;
  b.linked_ = true; // from here on the destructor removes the name on any failure
  const int rc = ::posix_fallocate(fd, 0, off_t(bytes));
  if (rc != 0) {
    ::close(fd);
    TZ_THROW("posix_fallocate(" << name << ", " << bytes << " B): " << std::strerror(rc)
                                << " (/dev/shm too small?)");
  }
  void *p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  TZ_CHECK(p != MAP_FAILED, "mmap(" << name << "): " << std::strerror(errno));
  b.host_ = p;
  b.bytes_ = bytes;
  std::memset(p, 0, bytes);
  TZ_HIP(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  b.registered_ = true;
  TZ_HIP(hipHostGetDevicePointer(&b.dev_, p, 0));
  return b;
}

SharedHostBuffer SharedHostBuffer::open(const std::string &name, size_t bytes) {
  SharedHostBuffer b;
  const int fd = ::shm_open(name.c_str(), O_RDWR, 0600);
  TZ_CHECK(fd >= 0, "shm_open(" << name << "): " << std::strerror(errno));
  struct stat st {};
  if (::fstat(fd, &st) != 0 || size_t(st.st_size) < bytes) {
    ::close(fd);
    TZ_THROW("shared buffer " << name << " is smaller than " << bytes << " B");
  }
  void *p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  TZ_CHECK(p != MAP_FAILED, "mmap(" << name << "): " << std::strerror(errno));
  b.host_ = p;
  b.bytes_ = bytes;
  TZ_HIP(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  b.registered_ = true;
  TZ_HIP(hipHostGetDevicePointer(&b.dev_, p, 0));
  return b;
}

void SharedHostBuffer::unlink() {
  if (linked_) (void)::shm_unlink(name_.c_str());
  linked_ = false;
}

void SharedHostBuffer::swap(SharedHostBuffer &o) noexcept {
  std::swap(host_, o.host_);
  std::swap(dev_, o.dev_);
  std::swap(bytes_, o.bytes_);
  std::swap(name_, o.name_);
  std::swap(linked_, o.linked_);
  std::swap(registered_, o.registered_);
}

SharedHostBuffer::~SharedHostBuffer() {
  // teardown: nothing useful to do with an error
  if (registered_) (void)hipHostUnregister(host_);
  if (host_) (void)::munmap(host_, bytes_);
  unlink();
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

static void host_noop(void *) {}

void HostFuncOp::launch(void *stream, Executor &) const {
  TZ_HIP(hipLaunchHostFunc(static_cast<hipStream_t>(stream), host_noop, nullptr));
}

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
