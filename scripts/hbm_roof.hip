// HBM roof probe: what a streaming copy, a pure read and a pure write reach on this MI355X, and
// which copy shape gets closest (grid-stride vs contiguous chunk per workgroup, loads in flight
// per lane, non-temporal hints, workgroup size). Buffers are far larger than the 256 MB
// Infinity Cache. Rates count every byte read plus every byte written.
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_roof scripts/hbm_roof.hip && ./hbm_roof [GB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                 \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT> __device__ __forceinline__ f4 ld(const f4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT> __device__ __forceinline__ void st(f4 *p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride: lane i of the grid touches i, i + S, i + 2S, ... (U loads in flight)
template <int U, bool NTL, bool NTS>
__global__ void copy_gs(f4 *__restrict__ d, const f4 *__restrict__ s, long n) {
  const long S = long(gridDim.x) * blockDim.x;
  long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * S < n; i += U * S) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(s + i + u * S);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(d + i + u * S, v[u]);
  }
  for (; i < n; i += S) st<NTS>(d + i, ld<NTL>(s + i));
}

// contiguous chunk per workgroup: the workgroup sweeps its own [c0, c1) in block-wide steps
template <int U, bool NTL, bool NTS>
__global__ void copy_chunk(f4 *__restrict__ d, const f4 *__restrict__ s, long n) {
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long c0 = long(blockIdx.x) * per, c1 = std::min(n, c0 + per);
  const int B = blockDim.x;
  long i = c0 + threadIdx.x;
  for (; i + (U - 1) * B < c1; i += U * B) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(s + i + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(d + i + u * B, v[u]);
  }
  for (; i < c1; i += B) st<NTS>(d + i, ld<NTL>(s + i));
}

template <int U> __global__ void read_gs(const f4 *__restrict__ s, long n, float *out) {
  const long S = long(gridDim.x) * blockDim.x;
  long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * S < n; i += U * S) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc += __builtin_nontemporal_load(s + i + u * S);
  }
  for (; i < n; i += S) acc += s[i];
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x; // keeps the loads alive
}

template <int U> __global__ void write_gs(f4 *__restrict__ d, long n) {
  const long S = long(gridDim.x) * blockDim.x;
  long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  const f4 v = {1, 2, 3, 4};
  for (; i + (U - 1) * S < n; i += U * S) {
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * S] = v;
  }
  for (; i < n; i += S) d[i] = v;
}

template <class F> float time_ms(F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int k = 0; k < 2; ++k) launch();
  std::vector<float> ts;
  for (int k = 0; k < reps; ++k) {
    CHECK(hipEventRecord(a, 0));
    launch();
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  CHECK(hipGetLastError());
  std::sort(ts.begin(), ts.end());
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 2.0;
  const long n = long(gb * 1e9) / 16;
  const double bytes = double(n) * 16;
  f4 *s, *d;
  float *out;
  CHECK(hipMalloc(&s, n * 16));
  CHECK(hipMalloc(&d, n * 16));
  CHECK(hipMalloc(&out, 16));
  CHECK(hipMemset(s, 1, n * 16));
  CHECK(hipMemset(d, 0, n * 16));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  std::printf("{\"device\": \"%s\", \"cus\": %d, \"buffer_GB\": %.2f}\n", p.gcnArchName, cus, bytes / 1e9);
  auto report = [&](const char *what, int blocks, int threads, float ms, double traffic) {
    std::printf("{\"kernel\": \"%s\", \"blocks\": %d, \"threads\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", what,
                blocks, threads, ms * 1e3, traffic / (ms * 1e-3) / 1e12);
    std::fflush(stdout);
  };
  const int reps = 10;
#define COPY(K, U, L, S, BL, TH)                                                                   \
  report(#K "<" #U "," #L "," #S ">", BL, TH,                                                      \
         time_ms([&] { hipLaunchKernelGGL((K<U, L, S>), dim3(BL), dim3(TH), 0, 0, d, s, n); }, reps), \
         2 * bytes)
  for (int th : {256, 1024}) {
    for (int mult : {4, 8, 32, 128}) {
      const int bl = cus * mult * 256 / th;
      COPY(copy_gs, 4, false, false, bl, th);
      COPY(copy_gs, 8, false, false, bl, th);
      COPY(copy_gs, 4, true, true, bl, th);
      COPY(copy_gs, 4, true, false, bl, th);
      COPY(copy_chunk, 4, false, false, bl, th);
      COPY(copy_chunk, 8, false, false, bl, th);
      COPY(copy_chunk, 4, true, true, bl, th);
    }
  }
  for (int mult : {4, 8, 32}) {
    const int bl = cus * mult;
    report("read_gs<8>", bl, 256,
           time_ms([&] { hipLaunchKernelGGL((read_gs<8>), dim3(bl), dim3(256), 0, 0, s, n, out); }, reps), bytes);
    report("write_gs<8>", bl, 256,
           time_ms([&] { hipLaunchKernelGGL((write_gs<8>), dim3(bl), dim3(256), 0, 0, d, n); }, reps), bytes);
  }
  report("hipMemcpyDtoD", 0, 0, time_ms([&] { CHECK(hipMemcpyAsync(d, s, n * 16, hipMemcpyDeviceToDevice, 0)); }, reps),
         2 * bytes);
  CHECK(hipFree(s));
  CHECK(hipFree(d));
  CHECK(hipFree(out));
  return 0;
}
