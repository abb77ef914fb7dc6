// CSR SpMV and vector kernels for gfx950.
//
// Reference: include/tenzing/spmv/ops_spmv.cuh:25-186 (a one-thread-per-row `spmv` kernel that
// is never launched; the op calls cuSPARSE CSR_ALG2; `VectorAdd::run` is a no-op;
// `scatter<<<128,100>>>` grid-stride gather). Here:
//  * csr_spmv: W lanes of a wave64 cooperate on one row (W chosen from the average row length,
//    W | 64 so a row group never straddles a wave), strided coalesced loads of col/val, x read
//    through L2/MALL (the band structure keeps x L2-resident), butterfly reduction with
//    __shfl_xor inside the W-lane group, optional accumulate (y += A x) so the remote part can
//    be fused into y without a separate add. CSR SpMV is bandwidth/latency bound (2 flops per
//    8-12 bytes); MFMA does not apply to a general CSR band matrix.
//  * gather (x-halo scatter), f32 vector add with 16-byte accesses, f64 axpy / iota, an empty
//    kernel for launch-overhead probes and a clocked busy kernel for scheduling tests.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "spmv_device.hpp"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace tz {
namespace kern {

namespace {

#define TZ_HIP_LAUNCH_CHECK()                                                                      \
  do {                                                                                             \
    hipError_t e_ = hipGetLastError();                                                             \
    if (e_ != hipSuccess)                                                                          \
      throw std::runtime_error(std::string("kernel launch failed: ") + hipGetErrorString(e_));     \
  } while (0)

constexpr int kThreads = 256;

template <int W>
__global__ __launch_bounds__(kThreads) void csr_spmv_k(int nRows, const int32_t *__restrict__ rowPtr,
                                                       const int32_t *__restrict__ colInd,
                                                       const float *__restrict__ val,
                                                       const float *__restrict__ x,
                                                       float *__restrict__ y, int accumulate) {
  const int gtid = blockIdx.x * kThreads + threadIdx.x;
  const int row = gtid / W;
  const int lane = gtid & (W - 1);
  if (row >= nRows) return; // whole W-lane groups exit together (W divides 64)
  const int b = rowPtr[row], e = rowPtr[row + 1];
  float sum = 0.f;
  for (int j = b + lane; j < e; j += W) sum = fmaf(val[j], x[colInd[j]], sum);
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) sum += __shfl_xor(sum, off, W);
  if (lane == 0) y[row] = accumulate ? y[row] + sum : sum;
}

// CSR with instruction-level parallelism (dev::csr_spmv_ilp_row): W lanes per row as
// csr_spmv_k, every lane issuing all K of its column loads, then all K value loads and x
// gathers, before it uses any. At 150,000 rows the whole grid is resident at once.
template <int W, int K>
__global__ __launch_bounds__(kThreads) void csr_spmv_ilp_k(int nRows, const int32_t *__restrict__ rowPtr,
                                                           const int32_t *__restrict__ colInd,
                                                           const float *__restrict__ val,
                                                           const float *__restrict__ x,
                                                           float *__restrict__ y, int accumulate) {
  dev::csr_spmv_ilp_row<W, K>(blockIdx.x * kThreads + threadIdx.x, nRows, rowPtr, colInd, val, x, y,
                               accumulate);
}

// CSR-stream: a block owns kStreamRows consecutive rows; its nnz range [rowPtr[r0],
// rowPtr[r0+R]) is contiguous, so all 256 lanes stream col/val with unit stride (4 independent
// loads in flight per lane), form val*x[col] into LDS, then 4 lanes per row reduce their row's
// segment out of LDS. For short rows (the band matrices here average 10 nnz) this replaces
// W-lane groups that idle on short rows and issue dependent loads one row at a time.
constexpr int kStreamRows = 64;
constexpr int kStreamCap = 4096; // products staged per pass (16 KB of LDS)

__global__ __launch_bounds__(kThreads) void csr_spmv_stream_k(int nRows,
                                                              const int32_t *__restrict__ rowPtr,
                                                              const int32_t *__restrict__ colInd,
                                                              const float *__restrict__ val,
                                                              const float *__restrict__ x,
                                                              float *__restrict__ y, int accumulate) {
  __shared__ int sPtr[kStreamRows + 1];
  __shared__ float sProd[kStreamCap];
  const int r0 = blockIdx.x * kStreamRows;
  const int nr = min(kStreamRows, nRows - r0);
  for (int i = threadIdx.x; i <= nr; i += kThreads) sPtr[i] = rowPtr[r0 + i];
  __syncthreads();
  const int a = sPtr[0], b = sPtr[nr];
  const int row = threadIdx.x >> 2, sub = threadIdx.x & 3; // 4 lanes per row
  float sum = 0.f;
  for (int c0 = a; c0 < b; c0 += kStreamCap) {
    const int c1 = min(b, c0 + kStreamCap);
    int k = c0 + threadIdx.x;
    for (; k + 3 * kThreads < c1; k += 4 * kThreads) {
      int c[4];
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) c[u] = colInd[k + u * kThreads];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = val[k + u * kThreads];
#pragma unroll
      for (int u = 0; u < 4; ++u) sProd[k + u * kThreads - c0] = v[u] * x[c[u]];
    }
    for (; k < c1; k += kThreads) sProd[k - c0] = val[k] * x[colInd[k]];
    __syncthreads();
    if (row < nr) {
      const int lo = max(sPtr[row], c0), hi = min(sPtr[row + 1], c1);
      for (int j = lo + sub; j < hi; j += 4) sum += sProd[j - c0];
    }
    __syncthreads();
  }
  sum += __shfl_xor(sum, 1, 4);
  sum += __shfl_xor(sum, 2, 4);
  if (row < nr && sub == 0) y[r0 + row] = accumulate ? y[r0 + row] + sum : sum;
}

__global__ __launch_bounds__(kThreads) void gather_k(int n, const float *__restrict__ src,
                                                     const int32_t *__restrict__ idx,
                                                     float *__restrict__ dst) {
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads)
    dst[i] = src[idx[i]];
}

struct DevPutBatch {
  const float *src;
  const int32_t *idx;
  unsigned int *done;
  int32_t nseg;
  uint32_t block_start[kMaxPutPeers + 1];
  PutSeg seg[kMaxPutPeers];
};

// IPC put of the SpMV x halo: each segment gathers x[idx[off + i]] straight into a peer's
// (IPC-mapped) remote-x buffer; the segment's last block publishes it with one system-scope
// increment of the peer's arrival counter (same protocol as the halo puts)
__global__ __launch_bounds__(kThreads) void gather_put_k(DevPutBatch b) {
  int s = 0;
  while (s + 1 < b.nseg && blockIdx.x >= b.block_start[s + 1]) ++s;
  const PutSeg &g = b.seg[s];
  const uint32_t nb = b.block_start[s + 1] - b.block_start[s];
  const uint32_t tid = (blockIdx.x - b.block_start[s]) * kThreads + threadIdx.x;
  for (uint32_t i = tid; i < uint32_t(g.n); i += nb * kThreads) g.dst[i] = b.src[b.idx[g.off + i]];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int prev = atomicAdd(&b.done[s], 1u);
    if (prev == nb - 1) {
      b.done[s] = 0; // ready for the next launch (kernel boundary orders it)
      __threadfence_system();
      __hip_atomic_fetch_add(g.flag, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(kThreads) void vector_add_k(int n, const float *__restrict__ a,
                                                         const float *__restrict__ b,
                                                         float *__restrict__ y) {
  const int n4 = n / 4;
  const float4 *a4 = reinterpret_cast<const float4 *>(a);
  const float4 *b4 = reinterpret_cast<const float4 *>(b);
  float4 *y4 = reinterpret_cast<float4 *>(y);
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n4; i += gridDim.x * kThreads) {
    float4 u = a4[i], v = b4[i];
    y4[i] = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
  }
  for (int i = n4 * 4 + blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads)
    y[i] = a[i] + b[i];
}

__global__ __launch_bounds__(kThreads) void axpy_k(int64_t n, double alpha,
                                                   const double *__restrict__ x,
                                                   double *__restrict__ y) {
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * kThreads)
    y[i] = fma(alpha, x[i], y[i]);
}

__global__ __launch_bounds__(kThreads) void iota_k(int64_t n, double base, double scale,
                                                   double *__restrict__ a) {
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * kThreads)
    a[i] = base + scale * double(i);
}

// 16 B per lane, 4 independent 16-B loads in flight per lane before the stores
__global__ __launch_bounds__(kThreads) void copy16_k(int4 *__restrict__ dst,
                                                     const int4 *__restrict__ src, int64_t n16) {
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const int4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

struct CopyBatch {
  int4 *dst[kMaxBoxes];
  const int4 *src[kMaxBoxes];
  int64_t n16[kMaxBoxes];
  int32_t tail8[kMaxBoxes]; // 1 if an 8-byte remainder follows the 16-byte part
  uint32_t block_start[kMaxBoxes + 1];
  int32_t n;
};

__global__ __launch_bounds__(kThreads) void copy_many_k(CopyBatch b) {
  int c = 0;
  while (c + 1 < b.n && blockIdx.x >= b.block_start[c + 1]) ++c;
  const int64_t nb = b.block_start[c + 1] - b.block_start[c];
  const int64_t stride = nb * kThreads;
  int4 *__restrict__ dst = b.dst[c];
  const int4 *__restrict__ src = b.src[c];
  const int64_t n16 = b.n16[c];
  int64_t i = int64_t(blockIdx.x - b.block_start[c]) * kThreads + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const int4 x0 = src[i], x1 = src[i + stride], x2 = src[i + 2 * stride], x3 = src[i + 3 * stride];
    dst[i] = x0;
    dst[i + stride] = x1;
    dst[i + 2 * stride] = x2;
    dst[i + 3 * stride] = x3;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
  if (b.tail8[c] && blockIdx.x == b.block_start[c] && threadIdx.x == 0)
    reinterpret_cast<double *>(dst + n16)[0] = reinterpret_cast<const double *>(src + n16)[0];
}

__global__ void copy_tail_k(char *__restrict__ dst, const char *__restrict__ src, int n) {
  if (int(threadIdx.x) < n) dst[threadIdx.x] = src[threadIdx.x];
}

__global__ void empty_k() {}

__global__ void busy_k(int64_t ticks, const int *abort) {
  // wall_clock64 runs at a fixed rate (hipDeviceAttributeWallClockRate), unlike the shader clock;
  // the abort flag (host memory, a PCIe round trip) is read every 256 polls
  const int64_t t0 = wall_clock64();
  for (uint32_t k = 1; wall_clock64() - t0 < ticks; ++k) {
    __builtin_amdgcn_s_sleep(1);
    if ((k & 255u) == 0 && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
  }
}

int grid_for(int64_t n, int perThread = 1) {
  int64_t b = (n + int64_t(kThreads) * perThread - 1) / (int64_t(kThreads) * perThread);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return int(b);
}

} // namespace

void csr_spmv(int nRows, const int32_t *rowPtr, const int32_t *colInd, const float *val,
              const float *x, float *y, int lanesPerRow, bool accumulate, void *stream) {
  if (nRows <= 0) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (lanesPerRow < 0) {
    const dim3 g(unsigned((int64_t(nRows) + kStreamRows - 1) / kStreamRows));
    hipLaunchKernelGGL(csr_spmv_stream_k, g, dim3(kThreads), 0, s, nRows, rowPtr, colInd, val, x,
                       y, accumulate ? 1 : 0);
    TZ_HIP_LAUNCH_CHECK();
    return;
  }
  if (lanesPerRow > kSpmvIlp) { // the ILP kernel with W = lanesPerRow - kSpmvIlp lanes per row
    const int W = lanesPerRow - kSpmvIlp;
    const int64_t threads = int64_t(nRows) * W;
    const dim3 g(unsigned((threads + kThreads - 1) / kThreads)), b(kThreads);
    const int acc = accumulate ? 1 : 0;
    switch (W) {
    case 1: hipLaunchKernelGGL((csr_spmv_ilp_k<1, 16>), g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
    case 2: hipLaunchKernelGGL((csr_spmv_ilp_k<2, 8>), g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
    case 4: hipLaunchKernelGGL((csr_spmv_ilp_k<4, 4>), g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
    default: throw std::runtime_error("csr_spmv: the ILP kernel takes 1, 2 or 4 lanes per row");
    }
    TZ_HIP_LAUNCH_CHECK();
    return;
  }
  int W = lanesPerRow;
  if (W <= 0) W = 8;
  const int64_t threads = int64_t(nRows) * W;
  const dim3 g(unsigned((threads + kThreads - 1) / kThreads)), b(kThreads);
  const int acc = accumulate ? 1 : 0;
  switch (W) {
  case 1: hipLaunchKernelGGL(csr_spmv_k<1>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  case 2: hipLaunchKernelGGL(csr_spmv_k<2>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  case 4: hipLaunchKernelGGL(csr_spmv_k<4>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  case 8: hipLaunchKernelGGL(csr_spmv_k<8>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  case 16: hipLaunchKernelGGL(csr_spmv_k<16>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  case 32: hipLaunchKernelGGL(csr_spmv_k<32>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  case 64: hipLaunchKernelGGL(csr_spmv_k<64>, g, b, 0, s, nRows, rowPtr, colInd, val, x, y, acc); break;
  default: throw std::runtime_error("csr_spmv: lanesPerRow must be a power of two <= 64");
  }
  TZ_HIP_LAUNCH_CHECK();
}

void gather_f32(int n, const float *src, const int32_t *idx, float *dst, void *stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_k, dim3(grid_for(n)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), n, src, idx, dst);
  TZ_HIP_LAUNCH_CHECK();
}

void gather_put_signal(const float *src, const int32_t *idx, const PutSeg *segs, int nseg,
                       unsigned int *done, void *stream) {
  if (nseg <= 0) return;
  if (nseg > kMaxPutPeers) throw std::runtime_error("gather_put_signal: too many peers");
  if (!src || !idx || !done) throw std::runtime_error("gather_put_signal: null pointer");
  DevPutBatch b{};
  b.src = src;
  b.idx = idx;
  b.done = done;
  b.nseg = nseg;
  uint32_t total = 0;
  for (int i = 0; i < nseg; ++i) {
    if (!segs[i].dst || !segs[i].flag || segs[i].n <= 0 || segs[i].off < 0)
      throw std::runtime_error("gather_put_signal: bad segment");
    b.seg[i] = segs[i];
    b.block_start[i] = total;
    // enough blocks to stream the segment, few enough that the completion count stays cheap
    total += uint32_t(std::min<int64_t>(64, (int64_t(segs[i].n) + 4 * kThreads - 1) / (4 * kThreads)));
  }
  b.block_start[nseg] = total;
  hipLaunchKernelGGL(gather_put_k, dim3(total), dim3(kThreads), 0, static_cast<hipStream_t>(stream), b);
  TZ_HIP_LAUNCH_CHECK();
}

void vector_add_f32(int n, const float *a, const float *b, float *y, void *stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(vector_add_k, dim3(grid_for(n, 4)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), n, a, b, y);
  TZ_HIP_LAUNCH_CHECK();
}

void axpy_f64(int64_t n, double alpha, const double *x, double *y, void *stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(axpy_k, dim3(grid_for(n, 4)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), n, alpha, x, y);
  TZ_HIP_LAUNCH_CHECK();
}

void iota_f64(int64_t n, double base, double scale, double *a, void *stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(iota_k, dim3(grid_for(n, 4)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), n, base, scale, a);
  TZ_HIP_LAUNCH_CHECK();
}

void copy_bytes(void *dst, const void *src, size_t bytes, void *stream) {
  if (!bytes) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 16)
    throw std::runtime_error("copy_bytes: pointers must be 16-byte aligned");
  const int64_t n16 = int64_t(bytes / 16);
  if (n16) {
    hipLaunchKernelGGL(copy16_k, dim3(grid_for(n16, 4)), dim3(kThreads), 0, s,
                       static_cast<int4 *>(dst), static_cast<const int4 *>(src), n16);
    TZ_HIP_LAUNCH_CHECK();
  }
  const int tail = int(bytes % 16);
  if (tail) {
    hipLaunchKernelGGL(copy_tail_k, dim3(1), dim3(64), 0, s, static_cast<char *>(dst) + n16 * 16,
                       static_cast<const char *>(src) + n16 * 16, tail);
    TZ_HIP_LAUNCH_CHECK();
  }
}

void copy_many(const CopyDesc *d, int n, void *stream) {
  if (n <= 0) return;
  if (n > kMaxBoxes) throw std::runtime_error("copy_many: too many copies");
  CopyBatch b{};
  uint32_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (d[i].bytes == 0) continue;
    if (!d[i].dst || !d[i].src) throw std::runtime_error("copy_many: null pointer");
    if ((reinterpret_cast<uintptr_t>(d[i].dst) | reinterpret_cast<uintptr_t>(d[i].src)) % 16 ||
        d[i].bytes % 8)
      throw std::runtime_error("copy_many: 16-byte aligned pointers and 8-byte sizes required");
    const int k = b.n++;
    b.dst[k] = static_cast<int4 *>(d[i].dst);
    b.src[k] = static_cast<const int4 *>(d[i].src);
    b.n16[k] = int64_t(d[i].bytes / 16);
    b.tail8[k] = int32_t((d[i].bytes % 16) / 8);
    b.block_start[k] = total;
    total += uint32_t(grid_for(std::max<int64_t>(b.n16[k], 1), 4));
  }
  if (b.n == 0) return;
  b.block_start[b.n] = total;
  hipLaunchKernelGGL(copy_many_k, dim3(total), dim3(kThreads), 0, static_cast<hipStream_t>(stream), b);
  TZ_HIP_LAUNCH_CHECK();
}

void empty(void *stream) {
  hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream));
  TZ_HIP_LAUNCH_CHECK();
}

void busy_wait(int64_t cycles, int blocks, void *stream) {
  hipLaunchKernelGGL(busy_k, dim3(blocks > 0 ? blocks : 1), dim3(64), 0,
                     static_cast<hipStream_t>(stream), cycles, abort_flag());
  TZ_HIP_LAUNCH_CHECK();
}

namespace {
int *g_abortHost = nullptr; // host view
int *g_abortDev = nullptr;  // device view of the same bytes
std::once_flag g_abortOnce;
void alloc_abort_flag() {
  // coherent host memory: a host store is visible to spinning kernels without any flush, and a
  // kernel's system-scope load always goes to memory (no stale cache line)
  void *p = nullptr;
  if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess || !p)
    throw std::runtime_error("abort flag: hipHostMalloc failed");
  std::memset(p, 0, 64);
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d)
    throw std::runtime_error("abort flag: hipHostGetDevicePointer failed");
  g_abortHost = static_cast<int *>(p);
  g_abortDev = static_cast<int *>(d);
}
} // namespace

const int *abort_flag() {
  std::call_once(g_abortOnce, alloc_abort_flag);
  return g_abortDev;
}

void set_abort(bool on) {
  std::call_once(g_abortOnce, alloc_abort_flag);
  __atomic_store_n(g_abortHost, on ? 1 : 0, __ATOMIC_SEQ_CST);
}

bool abort_set() {
  if (!g_abortHost) return false;
  return __atomic_load_n(g_abortHost, __ATOMIC_SEQ_CST) != 0;
}

} // namespace kern
} // namespace tz
