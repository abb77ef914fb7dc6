// SDMA copy-engine throughput on one GPU: a D2D copy forced onto the copy engines
// (hipMemcpyDeviceToDeviceNoCU) split into k chunks on k streams (forked from and joined back to
// stream 0 through events, as a schedule op does), against the plain D2D copy (blit kernel). Shows whether one copy op needs several engines (streams) to go fast.
//   hipcc --offload-arch=gfx950 -O2 scripts/sdma_probe.hip -o /tmp/sdma_probe && /tmp/sdma_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e = (x);                                                                            \
    if (e != hipSuccess) {                                                                         \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));                                   \
      return 1;                                                                                    \
    }                                                                                              \
  } while (0)

int main() {
  const size_t sizes[] = {size_t(19) << 20, size_t(76) << 20};
  std::vector<hipStream_t> st(8);
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(8);
  for (auto &evk : ev) CK(hipEventCreateWithFlags(&evk, hipEventDisableTiming));
  for (size_t bytes : sizes) {
    void *a = nullptr, *b = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    for (int kind = 0; kind < 2; ++kind) {
      const hipMemcpyKind k = kind ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
      for (int chunks : {1, 2, 4, 8}) {
        const size_t per = (bytes / chunks + 255) / 256 * 256;
        // fork / join through events from stream 0, the way a schedule op spreads its copies
        auto once = [&] {
          (void)hipEventRecord(ev[0], st[0]);
          for (int c = 1; c < chunks; ++c) (void)hipStreamWaitEvent(st[c], ev[0], 0);
          for (int c = 0; c < chunks; ++c) {
            const size_t off = size_t(c) * per;
            if (off >= bytes) break;
            const size_t n = std::min(per, bytes - off);
            (void)hipMemcpyAsync(static_cast<char *>(b) + off, static_cast<char *>(a) + off, n, k, st[c]);
          }
          for (int c = 1; c < chunks; ++c) {
            (void)hipEventRecord(ev[c], st[c]);
            (void)hipStreamWaitEvent(st[0], ev[c], 0);
          }
        };
        once();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) once();
        CK(hipDeviceSynchronize());
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
        std::printf("bytes=%zu MB kind=%s chunks=%d  %.1f GB/s  (%.1f us)\n", bytes >> 20,
                    kind ? "NoCU(SDMA)" : "D2D", chunks, double(bytes) / s / 1e9, s * 1e6);
      }
    }
    CK(hipFree(a));
    CK(hipFree(b));
  }
  return 0;
}
