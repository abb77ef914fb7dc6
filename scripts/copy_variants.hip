// HBM copy roof on gfx950: dwordx4 grid-stride copies of a 3.4 GB buffer (the halo grid's size)
// with plain or non-temporal loads/stores and 4 or 8 vectors in flight per lane, at several grid
// sizes. Rate = (bytes read + bytes written) / time.
//   hipcc --offload-arch=gfx950 -O3 -o copy_variants scripts/copy_variants.hip && ./copy_variants
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                 \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void copy_k(v4i *__restrict__ dst, const v4i *__restrict__ src,
                                              long n16) {
  const long stride = long(gridDim.x) * 256;
  long i = long(blockIdx.x) * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    v4i v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

template <bool NTL, bool NTS, int U>
void run(const char *name, v4i *d, const v4i *s, long n16, int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((copy_k<NTL, NTS, U>), dim3(blocks), dim3(256), 0, 0, d, s, n16);
  CHECK(hipGetLastError());
  float best = 1e30f, sum = 0;
  const int reps = 10;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((copy_k<NTL, NTS, U>), dim3(blocks), dim3(256), 0, 0, d, s, n16);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
    sum += ms;
  }
  const double bytes = 2.0 * 16.0 * double(n16);
  std::printf("{\"kernel\": \"%s\", \"blocks\": %d, \"best_us\": %.1f, \"mean_us\": %.1f, \"TBps_best\": %.2f}\n",
              name, blocks, best * 1e3, sum / reps * 1e3, bytes / (best * 1e-3) / 1e12);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main() {
  const size_t bytes = 3438840384ull; // 518 x 518 x 3*(518+16) doubles: the halo grid
  const long n16 = long(bytes / 16);
  v4i *s, *d;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMemset(s, 1, bytes));
  CHECK(hipMemset(d, 0, bytes));
  for (int blocks : {2048, 4096, 8192, 16384, 65536}) {
    run<false, false, 4>("plain_u4", d, s, n16, blocks);
    run<true, true, 4>("nt_u4", d, s, n16, blocks);
    run<false, true, 4>("ntstore_u4", d, s, n16, blocks);
    run<true, true, 8>("nt_u8", d, s, n16, blocks);
  }
  CHECK(hipFree(s));
  CHECK(hipFree(d));
  return 0;
}
