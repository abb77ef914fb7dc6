// Halo pack / unpack kernels for gfx950 (CDNA4).
//
// Reference kernels: src/halo_exchange/ops_halo_exchange.cu:519-664 (pack/unpack for QXYZ and
// XYZQ, one CUDA thread block of (32,4,4) per tile; their loops start at 0 without thread
// offsets, so every thread copies the same elements — SURVEY.md §7.4). Design here:
//  * one generic "box <-> dense buffer" copy: the box is rows of `len` contiguous elements
//    (x-runs for XYZQ, (q,x)-runs for QXYZ), so one kernel serves every face/edge/corner and
//    both storage orders;
//  * a flat 1-D work space (item = VEC consecutive doubles of one row, buffer offset =
//    item*VEC exactly) decoded with multiply-high "magic" division (no integer divides), so
//    consecutive lanes touch consecutive addresses of both the grid row and the buffer;
//  * 16-byte (double2) accesses whenever the row and all strides are even — the halo layout
//    (HaloExchange) pads x so interior rows start 64-B aligned, making every y/z face
//    dwordx4-vectorizable; 3-wide x faces fall back to 8-byte accesses (their 24-byte runs at a
//    4 KB pitch are sector-bound either way);
//  * 4 items in flight per lane (all loads issued before the stores) to cover HBM latency on a
//    wave64 machine without relying on occupancy alone;
//  * a multi-box variant packs every face/edge/corner of an exchange in ONE launch: blocks are
//    assigned to boxes through a prefix table in the kernel arguments (scalar loads, wave-
//    uniform), so small edge/corner boxes cost a handful of blocks instead of a launch each;
//  * a box-to-box "move" variant for the direct (pack-free) transfer: interior slab -> ghost
//    region of the same layout in one pass (2 bytes of HBM traffic per payload byte instead of
//    6 for pack -> copy -> unpack).
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "spmv_device.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

namespace tz {
namespace kern {

BoxTuning &box_tuning() {
  // process-wide launch tuning, changed only through its setters (bindings: kernels.set_*);
  // no environment overrides: every option can be flipped both ways inside one process
  static BoxTuning t;
  return t;
}

void set_xcd_remap(int mode) {
  if (mode < 0 || mode > 2)
    throw std::invalid_argument("xcd_remap must be 0 (round-robin), 1 (per-XCD range) or 2 (per-box)");
  box_tuning().xcd_remap = mode;
}

namespace {

#define TZ_HIP_LAUNCH_CHECK()                                                                      \
  do {                                                                                             \
    hipError_t e_ = hipGetLastError();                                                             \
    if (e_ != hipSuccess)                                                                          \
      throw std::runtime_error(std::string("kernel launch failed: ") + hipGetErrorString(e_));     \
  } while (0)

struct FastDiv {
  uint32_t d = 1, m = 0, s = 0;
  FastDiv() = default;
  explicit FastDiv(uint32_t div) : d(div) {
    s = 0;
    while ((uint64_t(1) << s) < div) ++s;
    m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << s) - div)) / div + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint32_t t = __umulhi(n, m);
    return uint32_t((uint64_t(t) + n) >> s);
  }
};

struct DevDesc {
  double *buf;        // pack/unpack: dense buffer; move: destination array
  const double *src;  // move: source array (grid_off indexes it)
  int64_t delta;      // move: destination offset - source offset; widened unpack (make_dev_wide):
                      // buffer row length << 32 | elements of padding before each grid row
  int64_t grid_off, s1, s2, s3;
  uint32_t lvec, n1, n2, items;
  FastDiv dl, d1, d2;
  int32_t vec;
};

struct DevBatch {
  DevDesc d[kMaxBoxes];
  uint32_t block_start[kMaxBoxes + 1];
  int32_t n;
};

// XCD block order of box_move_many_k only (the other batch kernels never read it, so it is a
// kernel argument of its own instead of part of every DevBatch copy)
struct DevRemap {
  uint32_t total;   // logical blocks (the launch may be padded up to a multiple of 8)
  uint32_t per_xcd; // 0: logical block = blockIdx.x; else blocks per XCD of the remap
  uint32_t box_xcd; // per-box remap: block_start padded to multiples of 8, nreal = real blocks
  uint16_t nreal[kMaxBoxes]; // (16 bits: max_blocks <= 65535)
};

// The dispatcher deals workgroups to the 8 XCDs round-robin (hardware block b runs on XCD
// b % 8). With the remap, XCD x runs logical blocks [x * per_xcd, (x + 1) * per_xcd): each
// pass of the grid-stride loop then covers one contiguous span of memory per XCD, so rows that
// cross a block boundary (72-B x-face runs) stay within one L2.
__device__ __forceinline__ uint32_t logical_block(const DevRemap &r) {
  if (r.per_xcd == 0) return blockIdx.x;
  return (blockIdx.x % 8u) * r.per_xcd + blockIdx.x / 8u;
}

constexpr int kThreads = 256;

DevDesc make_dev(const BoxDesc &b) {
  DevDesc d{};
  d.buf = b.buf;
  d.grid_off = b.grid_off;
  d.s1 = b.s1;
  d.s2 = b.s2;
  d.s3 = b.s3;
  const bool even = (b.len % 2 == 0) && (b.grid_off % 2 == 0) && (b.s1 % 2 == 0) &&
                    (b.s2 % 2 == 0) && (b.s3 % 2 == 0) &&
                    (reinterpret_cast<uintptr_t>(b.buf) % 16 == 0);
  d.vec = even ? 2 : 1;
  d.lvec = uint32_t(b.len / d.vec);
  d.n1 = uint32_t(b.n1);
  d.n2 = uint32_t(b.n2);
  const uint64_t items = uint64_t(d.lvec) * b.n1 * b.n2 * b.n3;
  if (items >= (uint64_t(1) << 31)) throw std::runtime_error("box too large for 32-bit indexing");
  d.items = uint32_t(items);
  d.dl = FastDiv(std::max<uint32_t>(d.lvec, 1));
  d.d1 = FastDiv(std::max<uint32_t>(d.n1, 1));
  d.d2 = FastDiv(std::max<uint32_t>(d.n2, 1));
  return d;
}

// An unpack box whose rows may be widened over row padding (BoxDesc::lead / trail): grid rows of
// lead + len + trail elements written with 16-B stores when that makes them 16-B aligned, each
// element read from the dense buffer row (clamped into it for the padding elements, whose values
// nobody reads). Anything else: the plain box.
DevDesc make_dev_wide(const BoxDesc &b, bool unpack) {
  if (!unpack || !box_tuning().widen_unpack || (b.lead <= 0 && b.trail <= 0)) return make_dev(b);
  const int64_t wlen = int64_t(b.lead) + b.len + b.trail;
  const int64_t goff = b.grid_off - b.lead;
  if (b.lead < 0 || b.trail < 0 || b.len <= 0 || wlen % 2 != 0 || goff % 2 != 0 || goff < 0 ||
      b.s1 % 2 != 0 || b.s2 % 2 != 0 || b.s3 % 2 != 0)
    return make_dev(b);
  BoxDesc w = b;
  w.grid_off = goff;
  w.len = int32_t(wlen);
  DevDesc d = make_dev(w);
  d.vec = 2; // the grid side; the buffer is read one element at a time
  d.lvec = uint32_t(wlen / 2);
  const uint64_t items = uint64_t(d.lvec) * b.n1 * b.n2 * b.n3;
  if (items >= (uint64_t(1) << 31)) throw std::runtime_error("box too large for 32-bit indexing");
  d.items = uint32_t(items);
  d.dl = FastDiv(std::max<uint32_t>(d.lvec, 1));
  d.delta = int64_t((uint64_t(uint32_t(b.len)) << 32) | uint32_t(b.lead));
  return d;
}

// `cap`: blocks per box at most (0: BoxTuning::max_blocks); `unroll`: items per lane (0:
// BoxTuning::unroll)
uint32_t blocks_for(const DevDesc &d, int cap = 0, int unroll = 0) {
  const BoxTuning &t = box_tuning();
  const uint64_t per = uint64_t(kThreads) * uint64_t(unroll > 0 ? unroll : t.unroll);
  uint64_t b = (uint64_t(d.items) + per - 1) / per;
  const uint64_t m = uint64_t(std::max(1, cap > 0 ? cap : t.max_blocks));
  return uint32_t(std::max<uint64_t>(1, std::min<uint64_t>(b, m)));
}

typedef double dbl2_t __attribute__((ext_vector_type(2)));
template <int VEC> struct Vec;
template <> struct Vec<1> { using T = double; };
template <> struct Vec<2> { using T = dbl2_t; };

template <bool NT, typename T> __device__ __forceinline__ T ld(const T *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename T> __device__ __forceinline__ void st(T *p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int VEC>
__device__ __forceinline__ int64_t grid_index(const DevDesc &d, uint32_t it) {
  const uint32_t row = d.dl.div(it);
  const uint32_t xv = it - row * d.lvec;
  const uint32_t r1 = d.d1.div(row);
  const uint32_t i1 = row - r1 * d.n1;
  const uint32_t i3 = d.d2.div(r1);
  const uint32_t i2 = r1 - i3 * d.n2;
  return d.grid_off + int64_t(i1) * d.s1 + int64_t(i2) * d.s2 + int64_t(i3) * d.s3 +
         int64_t(xv) * VEC;
}

template <int VEC, bool UNPACK, int U, bool NT>
__device__ __forceinline__ void box_body(double *__restrict__ grid, const DevDesc &d, uint32_t tid,
                                         uint32_t nthreads) {
  using T = typename Vec<VEC>::T;
  T *__restrict__ buf = reinterpret_cast<T *>(d.buf);
  uint32_t it = tid;
  for (; it + (U - 1) * nthreads < d.items; it += U * nthreads) {
    T v[U];
    int64_t g[U];
#pragma unroll
    for (int k = 0; k < U; ++k) g[k] = grid_index<VEC>(d, it + k * nthreads);
    if (UNPACK) {
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = buf[it + k * nthreads];
#pragma unroll
      for (int k = 0; k < U; ++k) st<NT>(reinterpret_cast<T *>(grid + g[k]), v[k]);
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ld<NT>(reinterpret_cast<const T *>(grid + g[k]));
#pragma unroll
      for (int k = 0; k < U; ++k) buf[it + k * nthreads] = v[k];
    }
  }
  for (; it < d.items; it += nthreads) {
    const int64_t g = grid_index<VEC>(d, it);
    if (UNPACK) st<NT>(reinterpret_cast<T *>(grid + g), buf[it]);
    else buf[it] = ld<NT>(reinterpret_cast<const T *>(grid + g));
  }
}

// widened unpack (make_dev_wide): whole 16-B pairs of the widened grid rows, each element from
// the dense buffer row, padding elements clamped to the row's ends
template <int U, bool NT>
__device__ __forceinline__ void unpack_wide_body(double *__restrict__ grid, const DevDesc &d, uint32_t tid,
                                                 uint32_t nthreads) {
  const double *__restrict__ buf = d.buf;
  const uint32_t blen = uint32_t(uint64_t(d.delta) >> 32);
  const int32_t lead = int32_t(uint32_t(uint64_t(d.delta)));
  const int32_t last = int32_t(blen) - 1;
  auto value = [&](uint32_t item) {
    const uint32_t row = d.dl.div(item);
    const int32_t x = int32_t(2 * (item - row * d.lvec)) - lead;
    const double *r = buf + int64_t(row) * blen;
    dbl2_t v;
    v.x = r[min(max(x, 0), last)];
    v.y = r[min(max(x + 1, 0), last)];
    return v;
  };
  uint32_t it = tid;
  for (; it + (U - 1) * nthreads < d.items; it += U * nthreads) {
    dbl2_t v[U];
    int64_t g[U];
#pragma unroll
    for (int k = 0; k < U; ++k) g[k] = grid_index<2>(d, it + k * nthreads);
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = value(it + k * nthreads);
#pragma unroll
    for (int k = 0; k < U; ++k) st<NT>(reinterpret_cast<dbl2_t *>(grid + g[k]), v[k]);
  }
  for (; it < d.items; it += nthreads)
    st<NT>(reinterpret_cast<dbl2_t *>(grid + grid_index<2>(d, it)), value(it));
}

template <bool UNPACK, int U, bool NT>
__global__ __launch_bounds__(kThreads) void box_copy_one_k(double *__restrict__ grid, DevDesc d) {
  const uint32_t tid = blockIdx.x * kThreads + threadIdx.x;
  const uint32_t nth = gridDim.x * kThreads;
  if (UNPACK && d.delta) unpack_wide_body<U, NT>(grid, d, tid, nth);
  else if (d.vec == 2) box_body<2, UNPACK, U, NT>(grid, d, tid, nth);
  else box_body<1, UNPACK, U, NT>(grid, d, tid, nth);
}

template <bool UNPACK, int U, bool NT>
__global__ __launch_bounds__(kThreads) void box_copy_many_k(double *__restrict__ grid, DevBatch b) {
  int box = 0;
  while (box + 1 < b.n && blockIdx.x >= b.block_start[box + 1]) ++box;
  const DevDesc &d = b.d[box];
  const uint32_t nb = b.block_start[box + 1] - b.block_start[box];
  const uint32_t tid = (blockIdx.x - b.block_start[box]) * kThreads + threadIdx.x;
  const uint32_t nth = nb * kThreads;
  if (UNPACK && d.delta) unpack_wide_body<U, NT>(grid, d, tid, nth);
  else if (d.vec == 2) box_body<2, UNPACK, U, NT>(grid, d, tid, nth);
  else box_body<1, UNPACK, U, NT>(grid, d, tid, nth);
}

// direct move: src box -> dst box of the same layout (both rows addressed by one index)
template <int VEC, int U, bool NT, bool NTS = false>
__device__ __forceinline__ void move_body(const DevDesc &d, uint32_t tid, uint32_t nthreads) {
  using T = typename Vec<VEC>::T;
  const double *__restrict__ src = d.src;
  double *__restrict__ dst = d.buf + d.delta;
  uint32_t it = tid;
  for (; it + (U - 1) * nthreads < d.items; it += U * nthreads) {
    T v[U];
    int64_t g[U];
#pragma unroll
    for (int k = 0; k < U; ++k) g[k] = grid_index<VEC>(d, it + k * nthreads);
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = ld<NT>(reinterpret_cast<const T *>(src + g[k]));
#pragma unroll
    for (int k = 0; k < U; ++k) st<NTS>(reinterpret_cast<T *>(dst + g[k]), v[k]);
  }
  for (; it < d.items; it += nthreads) {
    const int64_t g = grid_index<VEC>(d, it);
    st<NTS>(reinterpret_cast<T *>(dst + g), ld<NT>(reinterpret_cast<const T *>(src + g)));
  }
}

// peeled rows (d.vec == 3, or 5 with a tail): a row [x0, x0 + len) with x0 odd (the interior of
// an XYZQ grid with x = 0 at the row start begins at x = 3): element x0 alone, 16-B pairs from
// x0 + 1 (16-B aligned), and the last element alone when len - 1 is odd. Item xv of a row:
// xv < pairs a pair, then the head, then the tail; d.lvec = pairs + 1 + tail.
template <bool NT, bool NTS>
__device__ __forceinline__ void peel_body(const DevDesc &d, uint32_t tid, uint32_t nthreads) {
  const uint32_t tail = d.vec == 5 ? 1u : 0u;
  const uint32_t pairs = d.lvec - 1u - tail;
  const double *__restrict__ src = d.src;
  double *__restrict__ dst = d.buf + d.delta;
  for (uint32_t it = tid; it < d.items; it += nthreads) {
    const uint32_t row = d.dl.div(it);
    const uint32_t xv = it - row * d.lvec;
    const int64_t base = grid_index<1>(d, it) - int64_t(xv); // the row's x0
    if (xv < pairs) {
      const int64_t g = base + 1 + 2 * int64_t(xv);
      st<NTS>(reinterpret_cast<dbl2_t *>(dst + g), ld<NT>(reinterpret_cast<const dbl2_t *>(src + g)));
    } else {
      const int64_t g = xv == pairs ? base : base + 2 * int64_t(pairs) + 1;
      st<NTS>(dst + g, ld<NT>(src + g));
    }
  }
}

// row pair (MoveDesc::pair, d.vec = -len): item (row, k), k < 2 len: k < len moves element k of
// run A (row end -> row start), k >= len element k - len of run B (row start -> row end).
// Consecutive lanes cover consecutive k of a row, as the plain move covers a row's x: per row
// the same 2 line loads and 2 line stores as two separate boxes, but the lines a row's lanes
// load are the lines its lanes store into (x = 0 at the row start), within one wave.
template <int U, bool NTS>
__device__ __forceinline__ void pair_body(const DevDesc &d, uint32_t tid, uint32_t nthreads) {
  const int64_t len = -d.vec;
  const double *__restrict__ src = d.src;
  double *__restrict__ grid = d.buf;
  uint32_t it = tid;
  for (; it + (U - 1) * nthreads < d.items; it += U * nthreads) {
    double v[U];
    int64_t to[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = grid_index<1>(d, it + u * nthreads); // row base + k
      const uint32_t row = d.dl.div(it + u * nthreads);
      const int64_t k = int64_t(it + u * nthreads - row * d.lvec);
      const int64_t base = g - k;
      const int64_t from = k < len ? base + k : base + k + d.delta;          // A: end, B: start
      to[u] = k < len ? base + d.delta + k : base + k;                        // A: start, B: end
      v[u] = src[from];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(grid + to[u], v[u]);
  }
  for (; it < d.items; it += nthreads) {
    const int64_t g = grid_index<1>(d, it);
    const uint32_t row = d.dl.div(it);
    const int64_t k = int64_t(it - row * d.lvec);
    const int64_t base = g - k;
    const int64_t from = k < len ? base + k : base + k + d.delta;
    const int64_t to = k < len ? base + d.delta + k : base + k;
    st<NTS>(grid + to, src[from]);
  }
}

// one logical block `lb` of a batch of moves (box_move_many_k, box_move_spmv_k)
template <int U, bool NT, bool NTS>
__device__ __forceinline__ void move_block(const DevBatch &b, const DevRemap &r, uint32_t lb) {
  int box = 0;
  while (box + 1 < b.n && lb >= b.block_start[box + 1]) ++box;
  const DevDesc &d = b.d[box];
  uint32_t nb = b.block_start[box + 1] - b.block_start[box];
  uint32_t j = lb - b.block_start[box];
  if (r.box_xcd) { // every box spread over all 8 XCDs, one contiguous share of it per XCD
    j = (j % 8u) * (nb / 8u) + j / 8u;
    nb = r.nreal[box];
    if (j >= nb) return;
  }
  const uint32_t tid = j * kThreads + threadIdx.x;
  const uint32_t nth = nb * kThreads;
  if (d.vec == 2) move_body<2, U, NT, NTS>(d, tid, nth);
  else if (d.vec < 0) pair_body<U, NTS>(d, tid, nth);
  else if (d.vec >= 3) peel_body<NT, NTS>(d, tid, nth);
  else move_body<1, U, NT, NTS>(d, tid, nth);
}

template <int U, bool NT, bool NTS>
__global__ __launch_bounds__(kThreads) void box_move_many_k(DevBatch b, DevRemap r) {
  const uint32_t lb = logical_block(r);
  if (lb >= r.total) return; // padding of the remapped launch (no barriers in this kernel)
  move_block<U, NT, NTS>(b, r, lb);
}

// the SpMV half of box_move_spmv_k (kernel arguments: device pointers and sizes)
struct SpmvDev {
  const int32_t *rowPtr, *colInd;
  const float *val, *x;
  float *y;
  int32_t nRows, accumulate;
  uint32_t nBlocks, stride; // SpMV workgroups; one every `stride` workgroups of the launch
};

// horizontal fusion: workgroup b is SpMV workgroup b / stride when b % stride == 0 (and that
// index < nBlocks), else move workgroup b - (SpMV workgroups at or before b). Both kinds are
// dispatched side by side from the first wave on. No barriers: a workgroup returns as soon as
// its part is done.
template <int U, bool NT, bool NTS, int W, int K>
__global__ __launch_bounds__(kThreads) void box_move_spmv_k(DevBatch b, SpmvDev sp) {
  const uint32_t bid = blockIdx.x;
  const uint32_t k = bid / sp.stride;
  if (bid % sp.stride == 0 && k < sp.nBlocks) {
    dev::csr_spmv_ilp_row<W, K>(int(k) * kThreads + int(threadIdx.x), sp.nRows, sp.rowPtr, sp.colInd,
                                sp.val, sp.x, sp.y, sp.accumulate);
    return;
  }
  const uint32_t before = min(sp.nBlocks, k + 1);
  DevRemap r{};
  move_block<U, NT, NTS>(b, r, bid - before);
}

// shape-matched roof (line_roof): whole lines, 16-B accesses; d.vec carries the mode. U items
// per lane in flight (all loads issued before any is used); NTS: non-temporal stores (as the
// move's ghost stores)
template <int U, bool NTS>
__global__ __launch_bounds__(kThreads) void line_roof_k(DevBatch b, double zero, double *sink) {
  int box = 0;
  while (box + 1 < b.n && blockIdx.x >= b.block_start[box + 1]) ++box;
  const DevDesc &d = b.d[box];
  const uint32_t nb = b.block_start[box + 1] - b.block_start[box];
  const uint32_t tid = (blockIdx.x - b.block_start[box]) * kThreads + threadIdx.x;
  const uint32_t nth = nb * kThreads;
  const dbl2_t z = {zero, zero};
  dbl2_t acc = z;
  uint32_t it = tid;
  for (; it + (U - 1) * nth < d.items; it += U * nth) {
    dbl2_t *p[U];
#pragma unroll
    for (int k = 0; k < U; ++k) p[k] = reinterpret_cast<dbl2_t *>(d.buf + grid_index<2>(d, it + k * nth));
    if (d.vec == 1) {
#pragma unroll
      for (int k = 0; k < U; ++k) st<NTS>(p[k], z);
    } else if (d.vec == 3) { // line-to-line copy: p indexes the source, + delta the target
      dbl2_t v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = *reinterpret_cast<const dbl2_t *>(d.src + (reinterpret_cast<double *>(p[k]) - d.buf));
#pragma unroll
      for (int k = 0; k < U; ++k) st<NTS>(reinterpret_cast<dbl2_t *>(reinterpret_cast<double *>(p[k]) + d.delta), v[k]);
    } else {
      dbl2_t v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = *p[k];
      if (d.vec == 0) {
#pragma unroll
        for (int k = 0; k < U; ++k) acc += v[k];
      } else {
#pragma unroll
        for (int k = 0; k < U; ++k) st<NTS>(p[k], v[k] + z); // read, written back by the same lane
      }
    }
  }
  for (; it < d.items; it += nth) {
    dbl2_t *p = reinterpret_cast<dbl2_t *>(d.buf + grid_index<2>(d, it));
    if (d.vec == 0) acc += *p;
    else if (d.vec == 1) st<NTS>(p, z);
    else if (d.vec == 3)
      st<NTS>(reinterpret_cast<dbl2_t *>(reinterpret_cast<double *>(p) + d.delta),
              *reinterpret_cast<const dbl2_t *>(d.src + (reinterpret_cast<double *>(p) - d.buf)));
    else st<NTS>(p, *p + z);
  }
  if (acc.x + acc.y == 1.0e300) sink[0] = acc.x; // keeps the loads; never taken on a probe grid
}

struct DevSignal {
  unsigned int *done;
  unsigned long long *flag[kMaxBoxes];
  unsigned long long *count; // store mode (MoveSignal::count)
  uint64_t store_mask;
};

// explicit kernel arguments are limited to 4 KB; the largest signatures are checked here so a
// new field cannot push a launch over the limit
static_assert(sizeof(DevBatch) + sizeof(DevRemap) <= 4096, "box_move_many_k kernargs over 4 KB");
static_assert(sizeof(DevBatch) + sizeof(DevSignal) <= 4096, "box_move_signal_k kernargs over 4 KB");
static_assert(sizeof(double *) + sizeof(DevBatch) + sizeof(DevSignal) <= 4096,
              "box_pack_signal_k kernargs over 4 KB");

__device__ __forceinline__ void signal_box_done(const DevSignal &sig, int box, uint32_t nb);

// peer put: the move, then the box's last block publishes it with one system-scope signal
template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void box_move_signal_k(DevBatch b, DevSignal sig) {
  int box = 0;
  while (box + 1 < b.n && blockIdx.x >= b.block_start[box + 1]) ++box;
  const DevDesc &d = b.d[box];
  const uint32_t nb = b.block_start[box + 1] - b.block_start[box];
  const uint32_t tid = (blockIdx.x - b.block_start[box]) * kThreads + threadIdx.x;
  const uint32_t nth = nb * kThreads;
  if (d.vec == 2) move_body<2, U, NT>(d, tid, nth);
  else if (d.vec >= 3) peel_body<NT, false>(d, tid, nth);
  else move_body<1, U, NT>(d, tid, nth);
  signal_box_done(sig, box, nb);
}

// the box's last block publishes every block's (peer) stores with one system-scope signal
__device__ __forceinline__ void signal_box_done(const DevSignal &sig, int box, uint32_t nb) {
  __threadfence_system(); // this thread's peer stores are visible system-wide ...
  __syncthreads();        // ... for every thread of the block before it is counted
  if (threadIdx.x == 0) {
    const unsigned int prev = atomicAdd(&sig.done[box], 1u);
    if (prev == nb - 1) { // last block of this box: every block's stores are fenced
      sig.done[box] = 0;  // ready for the next iteration (kernel boundary orders it)
      __threadfence_system();
      if ((sig.store_mask >> box) & 1ull) {
        // single-writer flag (host memory): publish the new count with a plain release store
        const unsigned long long v = sig.count[box] + 1ull;
        sig.count[box] = v;
        __hip_atomic_store(sig.flag[box], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __hip_atomic_fetch_add(sig.flag[box], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// IPC put into a neighbour's receive buffer: pack, then signal
template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void box_pack_signal_k(double *__restrict__ grid, DevBatch b,
                                                              DevSignal sig) {
  int box = 0;
  while (box + 1 < b.n && blockIdx.x >= b.block_start[box + 1]) ++box;
  const DevDesc &d = b.d[box];
  const uint32_t nb = b.block_start[box + 1] - b.block_start[box];
  const uint32_t tid = (blockIdx.x - b.block_start[box]) * kThreads + threadIdx.x;
  const uint32_t nth = nb * kThreads;
  if (d.vec == 2) box_body<2, false, U, NT>(grid, d, tid, nth);
  else box_body<1, false, U, NT>(grid, d, tid, nth);
  signal_box_done(sig, box, nb);
}

constexpr int kMaxWaitSlots = 64;
struct WaitArgs {
  const unsigned long long *arrive;
  unsigned long long *expected;
  int *err;
  const int *abort; // process abort flag (kern::abort_flag): give up when set
  long long timeout_ticks;
  int n;
  int lag;  // wait for arrive[slot] >= expected[slot] + 1 - lag (then expected[slot] += 1)
  int wait; // 0: signal only
  int slot[kMaxWaitSlots];
  unsigned long long *signal[kMaxWaitSlots]; // after the wait: +1 (system scope), if non-null
  unsigned long long *count; // non-null: store ++count[i] into signal[i] instead (store mode)
};

// one wave: lane i waits for slot i, then (optionally) signals a peer's counter. Used for
// arrivals (receiver waits for the peers' puts, lag 0), credits (sender waits until the peer
// has consumed its previous put, lag 1) and releases (signal only).
__global__ __launch_bounds__(64) void ipc_wait_k(WaitArgs a) {
  const int i = threadIdx.x;
  if (i < a.n && a.wait) {
    const int s = a.slot[i];
    const unsigned long long want = a.expected[s] + 1 - (unsigned long long)a.lag;
    a.expected[s] += 1;
    const long long t0 = wall_clock64();
    for (uint32_t k = 1;
         __hip_atomic_load(&a.arrive[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want; ++k) {
      __builtin_amdgcn_s_sleep(2);
      // the abort flag lives in host memory (a PCIe round trip): read it every 64 polls
      if (wall_clock64() - t0 > a.timeout_ticks ||
          ((k & 63u) == 0 && __hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
        atomicOr(a.err, 1);
        break;
      }
    }
  }
  __threadfence_system();
  if (i < a.n && a.signal[i]) {
    if (a.count) {
      const unsigned long long v = a.count[i] + 1ull;
      a.count[i] = v;
      __hip_atomic_store(a.signal[i], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      __hip_atomic_fetch_add(a.signal[i], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// host dispatch over (unpack, unroll, nt)
template <bool UNPACK, int U, bool NT>
void launch_one(dim3 g, hipStream_t s, double *grid, const DevDesc &d) {
  hipLaunchKernelGGL((box_copy_one_k<UNPACK, U, NT>), g, dim3(kThreads), 0, s, grid, d);
}
template <bool UNPACK, int U, bool NT>
void launch_many(dim3 g, hipStream_t s, double *grid, const DevBatch &b) {
  hipLaunchKernelGGL((box_copy_many_k<UNPACK, U, NT>), g, dim3(kThreads), 0, s, grid, b);
}

template <bool UNPACK> bool use_nt() {
  const BoxTuning &t = box_tuning();
  return UNPACK ? t.nt_unpack : t.nt_pack;
}

template <bool UNPACK>
void dispatch_one(dim3 g, hipStream_t s, double *grid, const DevDesc &d) {
  const bool nt = use_nt<UNPACK>();
  if (box_tuning().unroll >= 8) {
    if (nt) launch_one<UNPACK, 8, true>(g, s, grid, d);
    else launch_one<UNPACK, 8, false>(g, s, grid, d);
  } else if (box_tuning().unroll < 4) { // one item in flight, `unroll` items per lane
    if (nt) launch_one<UNPACK, 1, true>(g, s, grid, d);
    else launch_one<UNPACK, 1, false>(g, s, grid, d);
  } else {
    if (nt) launch_one<UNPACK, 4, true>(g, s, grid, d);
    else launch_one<UNPACK, 4, false>(g, s, grid, d);
  }
}

template <bool UNPACK>
void dispatch_many(dim3 g, hipStream_t s, double *grid, const DevBatch &b) {
  const bool nt = use_nt<UNPACK>();
  if (box_tuning().unroll >= 8) {
    if (nt) launch_many<UNPACK, 8, true>(g, s, grid, b);
    else launch_many<UNPACK, 8, false>(g, s, grid, b);
  } else if (box_tuning().unroll < 4) { // one item in flight, `unroll` items per lane
    if (nt) launch_many<UNPACK, 1, true>(g, s, grid, b);
    else launch_many<UNPACK, 1, false>(g, s, grid, b);
  } else {
    if (nt) launch_many<UNPACK, 4, true>(g, s, grid, b);
    else launch_many<UNPACK, 4, false>(g, s, grid, b);
  }
}

// ---- grid initialization / verification (test support; not on the timed path)

__device__ __forceinline__ int64_t wrapi(int64_t a, int64_t n) {
  a %= n;
  return a < 0 ? a + n : a;
}

__device__ __forceinline__ double halo_value(int q, int64_t gx, int64_t gy, int64_t gz, int gen) {
  constexpr int64_t G = 65536;
  // exact in a double for nq <= 8 (below 2^53 with the generation in bits 51-52)
  return double(((int64_t(q) * G + gz) * G + gy) * G + gx + (int64_t(gen & 3) << 51));
}

// classify logical element (x,y,z,q); returns expected value after a complete exchange and
// writes the storage index
__device__ __forceinline__ double halo_expect(const HaloGeom &g, int64_t lin, int64_t &idx,
                                              bool afterExchange) {
  const int64_t X = g.nx + 2 * g.g, Y = g.ny + 2 * g.g, Z = g.nz + 2 * g.g;
  const int64_t x = lin % X;
  int64_t r = lin / X;
  const int64_t y = r % Y;
  r /= Y;
  const int64_t z = r % Z;
  const int q = int(r / Z);
  if (g.order == 0) idx = q * g.sq + z * g.sz + y * g.sy + x + g.xoff;
  else idx = q + int64_t(g.nq) * (x + g.xoff) + y * g.sy + z * g.sz;
  const int gx = (x < g.g || x >= g.nx + g.g), gy = (y < g.g || y >= g.ny + g.g),
            gz = (z < g.g || z >= g.nz + g.g);
  const int k = gx + gy + gz;
  if (k > 0) {
    const bool filled = afterExchange && (g.neighbors == 26 || k == 1);
    if (!filled) return -1.0;
  }
  const int64_t GX = int64_t(g.nx) * g.px, GY = int64_t(g.ny) * g.py, GZ = int64_t(g.nz) * g.pz;
  return halo_value(q, wrapi(int64_t(g.cx) * g.nx + x - g.g, GX),
                    wrapi(int64_t(g.cy) * g.ny + y - g.g, GY),
                    wrapi(int64_t(g.cz) * g.nz + z - g.g, GZ), g.gen);
}

__global__ __launch_bounds__(kThreads) void halo_init_k(double *__restrict__ grid, HaloGeom g) {
  const int64_t total = int64_t(g.nx + 2 * g.g) * (g.ny + 2 * g.g) * (g.nz + 2 * g.g) * g.nq;
  for (int64_t lin = int64_t(blockIdx.x) * kThreads + threadIdx.x; lin < total;
       lin += int64_t(gridDim.x) * kThreads) {
    int64_t idx;
    const double v = halo_expect(g, lin, idx, false);
    grid[idx] = v;
  }
}

__global__ __launch_bounds__(kThreads) void halo_check_k(const double *__restrict__ grid, HaloGeom g,
                                                         unsigned long long *count) {
  const int64_t total = int64_t(g.nx + 2 * g.g) * (g.ny + 2 * g.g) * (g.nz + 2 * g.g) * g.nq;
  unsigned long long bad = 0;
  for (int64_t lin = int64_t(blockIdx.x) * kThreads + threadIdx.x; lin < total;
       lin += int64_t(gridDim.x) * kThreads) {
    int64_t idx;
    const double v = halo_expect(g, lin, idx, true);
    bad += grid[idx] != v;
  }
  // wave64 reduction, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_xor(bad, off);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(count, bad);
}

// stencil mode: out must hold c0 * v + c1 * (6 face neighbours of v) of the initialized field v
// (global coordinates, periodic), for every interior cell; counts the cells that do not
__global__ __launch_bounds__(kThreads) void stencil_check_k(const double *__restrict__ out, HaloGeom g,
                                                            double c0, double c1,
                                                            unsigned long long *count) {
  const int64_t total = int64_t(g.nx) * g.ny * g.nz * g.nq;
  const int64_t GX = int64_t(g.nx) * g.px, GY = int64_t(g.ny) * g.py, GZ = int64_t(g.nz) * g.pz;
  unsigned long long bad = 0;
  for (int64_t lin = int64_t(blockIdx.x) * kThreads + threadIdx.x; lin < total;
       lin += int64_t(gridDim.x) * kThreads) {
    const int64_t x = lin % g.nx;
    int64_t r = lin / g.nx;
    const int64_t y = r % g.ny;
    r /= g.ny;
    const int64_t z = r % g.nz;
    const int q = int(r / g.nz);
    const int64_t X = x + g.g, Y = y + g.g, Z = z + g.g; // storage coordinates
    const int64_t idx = g.order == 0 ? q * g.sq + Z * g.sz + Y * g.sy + X + g.xoff
                                     : q + int64_t(g.nq) * (X + g.xoff) + Y * g.sy + Z * g.sz;
    const int64_t gx = int64_t(g.cx) * g.nx + x, gy = int64_t(g.cy) * g.ny + y,
                  gz = int64_t(g.cz) * g.nz + z;
    auto v = [&](int64_t dx, int64_t dy, int64_t dz) {
      return halo_value(q, wrapi(gx + dx, GX), wrapi(gy + dy, GY), wrapi(gz + dz, GZ), g.gen);
    };
    const double want = c0 * v(0, 0, 0) + c1 * (v(-1, 0, 0) + v(1, 0, 0) + v(0, -1, 0) +
                                                v(0, 1, 0) + v(0, 0, -1) + v(0, 0, 1));
    bad += fabs(out[idx] - want) > 1e-12 * fabs(want) + 1e-9;
  }
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_xor(bad, off);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(count, bad);
}

} // namespace

void stencil_check(const double *out, const HaloGeom &g, unsigned long long *count, void *stream) {
  const StencilBox defaults;
  hipLaunchKernelGGL(stencil_check_k, dim3(4096), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     out, g, defaults.c0, defaults.c1, count);
  TZ_HIP_LAUNCH_CHECK();
}

void halo_init(double *grid, const HaloGeom &g, void *stream) {
  hipLaunchKernelGGL(halo_init_k, dim3(4096), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     grid, g);
  TZ_HIP_LAUNCH_CHECK();
}

void halo_check(const double *grid, const HaloGeom &g, unsigned long long *count, void *stream) {
  hipLaunchKernelGGL(halo_check_k, dim3(4096), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     grid, g, count);
  TZ_HIP_LAUNCH_CHECK();
}

void box_copy(double *grid, const BoxDesc &b, bool unpack, void *stream) {
  if (!grid || !b.buf) throw std::runtime_error("box_copy: null grid or buffer");
  DevDesc d = make_dev_wide(b, unpack);
  if (d.items == 0) return;
  const dim3 grid_dim(blocks_for(d));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (unpack) dispatch_one<true>(grid_dim, s, grid, d);
  else dispatch_one<false>(grid_dim, s, grid, d);
  TZ_HIP_LAUNCH_CHECK();
}

void box_copy_many(double *grid, const BoxDesc *boxes, int n, bool unpack, void *stream) {
  if (n <= 0) return;
  if (n > kMaxBoxes) throw std::runtime_error("box_copy_many: too many boxes");
  DevBatch b{};
  b.n = 0;
  uint32_t total = 0;
  if (!grid) throw std::runtime_error("box_copy_many: null grid");
  for (int i = 0; i < n; ++i) {
    if (!boxes[i].buf) throw std::runtime_error("box_copy_many: null buffer");
    DevDesc d = make_dev_wide(boxes[i], unpack);
    if (d.items == 0) continue;
    b.d[b.n] = d;
    b.block_start[b.n] = total;
    total += blocks_for(d);
    ++b.n;
  }
  if (b.n == 0) return;
  b.block_start[b.n] = total;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (unpack) dispatch_many<true>(dim3(total), s, grid, b);
  else dispatch_many<false>(dim3(total), s, grid, b);
  TZ_HIP_LAUNCH_CHECK();
}

namespace {
// the device batch of a move launch (shared by the plain and the signalling variant);
// `keep` maps batch entries back to input boxes
DevBatch make_move_batch(const MoveDesc *moves, int n, uint32_t &total, std::vector<int> &keep,
                         int cap = 0, int unroll = 0);

template <int U>
void launch_move(const dim3 &g, hipStream_t s, const DevBatch &b, const DevRemap &r, bool ntl, bool nts) {
  if (ntl && nts) hipLaunchKernelGGL((box_move_many_k<U, true, true>), g, dim3(kThreads), 0, s, b, r);
  else if (ntl) hipLaunchKernelGGL((box_move_many_k<U, true, false>), g, dim3(kThreads), 0, s, b, r);
  else if (nts) hipLaunchKernelGGL((box_move_many_k<U, false, true>), g, dim3(kThreads), 0, s, b, r);
  else hipLaunchKernelGGL((box_move_many_k<U, false, false>), g, dim3(kThreads), 0, s, b, r);
}
} // namespace

void box_move_many(const MoveDesc *moves, int n, void *stream) {
  if (n <= 0) return;
  if (n > kMaxBoxes) throw std::runtime_error("box_move_many: too many boxes");
  uint32_t total = 0;
  std::vector<int> keep;
  const int U = box_tuning().move_unroll;
  if (U != 1 && U != 2 && U != 4) throw std::runtime_error("box_move_many: move_unroll must be 1, 2 or 4");
  const int items = std::max(U, box_tuning().move_items);
  DevBatch b = make_move_batch(moves, n, total, keep, 0, items);
  if (b.n == 0) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int mode = box_tuning().xcd_remap;
  DevRemap r{};
  if (mode == 2) { // pad every box to a multiple of 8 blocks, starting on a multiple of 8
    uint32_t t = 0;
    for (int i = 0; i < b.n; ++i) {
      const uint32_t nb = b.block_start[i + 1] - b.block_start[i];
      if (nb > 65535) throw std::runtime_error("box_move_many: too many blocks for the remap");
      r.nreal[i] = uint16_t(nb);
      b.block_start[i] = t;
      t += (nb + 7) / 8 * 8;
    }
    b.block_start[b.n] = t;
    total = t;
    r.box_xcd = 1;
  }
  r.total = total;
  r.per_xcd = mode == 1 ? (total + 7) / 8 : 0;
  const dim3 g(r.per_xcd ? r.per_xcd * 8 : total);
  const BoxTuning &t = box_tuning();
  if (U == 1) launch_move<1>(g, s, b, r, t.nt_move, t.nt_move_store);
  else if (U == 2) launch_move<2>(g, s, b, r, t.nt_move, t.nt_move_store);
  else launch_move<4>(g, s, b, r, t.nt_move, t.nt_move_store);
  TZ_HIP_LAUNCH_CHECK();
}

namespace {
template <int W, int K>
void launch_move_spmv(const dim3 &g, hipStream_t s, const DevBatch &b, const SpmvDev &sp, bool ntl,
                      bool nts) {
  // one item in flight per lane, as the tuned move (BoxTuning::move_unroll 1)
  if (ntl && nts) hipLaunchKernelGGL((box_move_spmv_k<1, true, true, W, K>), g, dim3(kThreads), 0, s, b, sp);
  else if (ntl) hipLaunchKernelGGL((box_move_spmv_k<1, true, false, W, K>), g, dim3(kThreads), 0, s, b, sp);
  else if (nts) hipLaunchKernelGGL((box_move_spmv_k<1, false, true, W, K>), g, dim3(kThreads), 0, s, b, sp);
  else hipLaunchKernelGGL((box_move_spmv_k<1, false, false, W, K>), g, dim3(kThreads), 0, s, b, sp);
}
static_assert(sizeof(DevBatch) + sizeof(SpmvDev) <= 4096, "box_move_spmv_k kernargs over 4 KB");
} // namespace

void box_move_spmv(const MoveDesc *moves, int n, const SpmvJob &job, void *stream) {
  if (n > kMaxBoxes) throw std::runtime_error("box_move_spmv: too many boxes");
  if (job.nRows < 0 || (job.nRows > 0 && (!job.rowPtr || !job.y)))
    throw std::runtime_error("box_move_spmv: bad SpMV job");
  const int W = job.lanes - kSpmvIlp;
  if (W != 1 && W != 2 && W != 4) throw std::runtime_error("box_move_spmv: lanes must be kSpmvIlp + 1, 2 or 4");
  uint32_t total = 0;
  std::vector<int> keep;
  const int items = std::max(1, box_tuning().move_items);
  const DevBatch b = n > 0 ? make_move_batch(moves, n, total, keep, 0, items) : DevBatch{};
  SpmvDev sp{};
  sp.rowPtr = job.rowPtr;
  sp.colInd = job.colInd;
  sp.val = job.val;
  sp.x = job.x;
  sp.y = job.y;
  sp.nRows = job.nRows;
  sp.accumulate = job.accumulate ? 1 : 0;
  sp.nBlocks = uint32_t((int64_t(job.nRows) * W + kThreads - 1) / kThreads);
  const uint64_t all = uint64_t(total) + sp.nBlocks;
  if (all == 0) return;
  if (all >= (uint64_t(1) << 31)) throw std::runtime_error("box_move_spmv: grid too large");
  // an odd stride: the dispatcher deals workgroup b to XCD b % 8, so an even stride would put
  // every SpMV workgroup on the same XCD (a stride of 8: all on XCD 0, 61 instead of 50 us)
  sp.stride = sp.nBlocks ? uint32_t(all / sp.nBlocks) : uint32_t(all + 1);
  if (sp.nBlocks && sp.stride % 2 == 0) sp.stride -= 1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g{unsigned(all)};
  const BoxTuning &t = box_tuning();
  if (W == 1) launch_move_spmv<1, 16>(g, s, b, sp, t.nt_move, t.nt_move_store);
  else if (W == 2) launch_move_spmv<2, 8>(g, s, b, sp, t.nt_move, t.nt_move_store);
  else launch_move_spmv<4, 4>(g, s, b, sp, t.nt_move, t.nt_move_store);
  TZ_HIP_LAUNCH_CHECK();
}

// workgroups per box of a signalling put: the launch's own cap, else the global one
static int put_cap(const MoveSignal &sig) {
  return sig.max_blocks > 0 ? sig.max_blocks : box_tuning().put_max_blocks;
}

void box_move_many_signal(const MoveDesc *moves, int n, const MoveSignal &sig, void *stream) {
  if (n <= 0) return;
  if (n > kMaxBoxes) throw std::runtime_error("box_move_many_signal: too many boxes");
  if (!sig.done) throw std::runtime_error("box_move_many_signal: null block counters");
  uint32_t total = 0;
  std::vector<int> keep;
  for (int i = 0; i < n; ++i)
    if (moves[i].pair) throw std::runtime_error("box_move_many_signal: row pairs are for self moves only");
  const DevBatch b = make_move_batch(moves, n, total, keep, put_cap(sig));
  if (b.n != n) throw std::runtime_error("box_move_many_signal: empty box (nothing to signal)");
  DevSignal ds{};
  ds.done = sig.done;
  for (int i = 0; i < n; ++i) {
    if (!sig.flag[keep[i]]) throw std::runtime_error("box_move_many_signal: null flag");
    ds.flag[i] = sig.flag[keep[i]];
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(total);
  if (box_tuning().nt_move) hipLaunchKernelGGL((box_move_signal_k<4, true>), g, dim3(kThreads), 0, s, b, ds);
  else hipLaunchKernelGGL((box_move_signal_k<4, false>), g, dim3(kThreads), 0, s, b, ds);
  TZ_HIP_LAUNCH_CHECK();
}

void box_pack_many_signal(double *grid, const BoxDesc *boxes, int n, const MoveSignal &sig,
                          void *stream) {
  if (n <= 0) return;
  if (n > kMaxBoxes) throw std::runtime_error("box_pack_many_signal: too many boxes");
  if (!grid || !sig.done) throw std::runtime_error("box_pack_many_signal: null grid or counters");
  DevBatch b{};
  DevSignal ds{};
  ds.done = sig.done;
  ds.count = sig.count;
  ds.store_mask = sig.store_mask;
  if (sig.store_mask && !sig.count) throw std::runtime_error("box_pack_many_signal: store mode without counters");
  uint32_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (!boxes[i].buf || !sig.flag[i]) throw std::runtime_error("box_pack_many_signal: null buffer/flag");
    DevDesc d = make_dev(boxes[i]);
    if (d.items == 0) throw std::runtime_error("box_pack_many_signal: empty box (nothing to signal)");
    b.d[b.n] = d;
    b.block_start[b.n] = total;
    ds.flag[b.n] = sig.flag[i];
    total += blocks_for(d, put_cap(sig));
    ++b.n;
  }
  b.block_start[b.n] = total;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (box_tuning().nt_pack)
    hipLaunchKernelGGL((box_pack_signal_k<4, true>), dim3(total), dim3(kThreads), 0, s, grid, b, ds);
  else
    hipLaunchKernelGGL((box_pack_signal_k<4, false>), dim3(total), dim3(kThreads), 0, s, grid, b, ds);
  TZ_HIP_LAUNCH_CHECK();
}

void ipc_wait(const unsigned long long *arrive, unsigned long long *expected, const int *slots,
              int n, int *err, double timeout_s, void *stream, int lag,
              unsigned long long *const *signal) {
  if (n <= 0) return;
  if (n > kMaxWaitSlots) throw std::runtime_error("ipc_wait: too many slots");
  if (!arrive || !expected || !err) throw std::runtime_error("ipc_wait: null pointer");
  if (lag < 0 || lag > 1) throw std::runtime_error("ipc_wait: lag must be 0 or 1");
  WaitArgs a{};
  a.arrive = arrive;
  a.expected = expected;
  a.err = err;
  a.abort = abort_flag();
  a.timeout_ticks = (long long)(timeout_s * 1.0e8); // wall_clock64 runs at 100 MHz
  a.n = n;
  a.lag = lag;
  a.wait = 1;
  for (int i = 0; i < n; ++i) {
    a.slot[i] = slots[i];
    a.signal[i] = signal ? signal[i] : nullptr;
  }
  hipLaunchKernelGGL(ipc_wait_k, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), a);
  TZ_HIP_LAUNCH_CHECK();
}

void ipc_signal(unsigned long long *const *signal, int n, void *stream, unsigned long long *count) {
  if (n <= 0) return;
  if (n > kMaxWaitSlots) throw std::runtime_error("ipc_signal: too many counters");
  WaitArgs a{};
  a.n = n;
  a.wait = 0;
  a.count = count;
  for (int i = 0; i < n; ++i) {
    if (!signal[i]) throw std::runtime_error("ipc_signal: null counter");
    a.signal[i] = signal[i];
  }
  hipLaunchKernelGGL(ipc_wait_k, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), a);
  TZ_HIP_LAUNCH_CHECK();
}

namespace {
DevBatch make_move_batch(const MoveDesc *moves, int n, uint32_t &total, std::vector<int> &keep,
                         int cap, int unroll) {
  DevBatch b{};
  b.n = 0;
  total = 0;
  for (int i = 0; i < n; ++i) {
    const MoveDesc &m = moves[i];
    if (!m.src || !m.dst) throw std::runtime_error("box_move_many: null array");
    BoxDesc box;
    box.buf = m.dst;
    box.grid_off = m.src_off;
    box.s1 = m.s1;
    box.s2 = m.s2;
    box.s3 = m.s3;
    box.len = m.len;
    box.n1 = m.n1;
    box.n2 = m.n2;
    box.n3 = m.n3;
    DevDesc d = make_dev(box);
    if (d.items == 0) continue;
    d.src = m.src;
    d.delta = m.dst_off - m.src_off;
    if (m.pair) {
      if (m.src != m.dst || m.len < 1 || m.len > kMaxPairLen)
        throw std::runtime_error("box_move_many: a row pair needs src == dst and 1..8 elements per run");
      // items (row, k < 2 len); d.vec < 0 marks the pair and carries the run length
      d.vec = -m.len;
      d.lvec = uint32_t(2 * m.len);
      d.items = uint32_t(uint64_t(d.lvec) * m.n1 * m.n2 * m.n3);
      d.dl = FastDiv(d.lvec);
      b.d[b.n] = d;
      b.block_start[b.n] = total;
      total += blocks_for(d, cap, unroll);
      keep.push_back(i);
      ++b.n;
      continue;
    }
    // 16-B accesses need both rows 16-B aligned: make_dev checked the source side (and the
    // destination base); the destination offset must be even as well
    if (d.vec == 2 && (m.dst_off % 2 != 0 || reinterpret_cast<uintptr_t>(m.src) % 16 != 0)) {
      d.vec = 1;
      d.lvec = uint32_t(m.len);
      d.items = uint32_t(uint64_t(m.len) * m.n1 * m.n2 * m.n3);
      d.dl = FastDiv(std::max<uint32_t>(d.lvec, 1));
    }
    // rows that start one element past a 16-B boundary on both sides (strides even): peel the
    // first element (and an odd last one), move the rest 16 B at a time
    if (d.vec == 1 && box_tuning().peel_moves && m.len >= 3 && m.src_off % 2 != 0 && m.dst_off % 2 != 0 &&
        m.s1 % 2 == 0 && m.s2 % 2 == 0 && m.s3 % 2 == 0 &&
        reinterpret_cast<uintptr_t>(m.src) % 16 == 0 && reinterpret_cast<uintptr_t>(m.dst) % 16 == 0) {
      const uint32_t tail = uint32_t((m.len - 1) % 2), pairs = uint32_t((m.len - 1) / 2);
      d.vec = tail ? 5 : 3;
      d.lvec = pairs + 1 + tail;
      d.items = uint32_t(uint64_t(d.lvec) * m.n1 * m.n2 * m.n3);
      d.dl = FastDiv(d.lvec);
    }
    b.d[b.n] = d;
    b.block_start[b.n] = total;
    total += blocks_for(d, cap, unroll);
    keep.push_back(i);
    ++b.n;
  }
  b.block_start[b.n] = total;
  return b;
}
} // namespace

std::vector<std::string> move_kinds(const MoveDesc *moves, int n) {
  if (n <= 0) return {};
  if (n > kMaxBoxes) throw std::runtime_error("move_kinds: too many boxes");
  uint32_t total = 0;
  std::vector<int> keep;
  const DevBatch b = make_move_batch(moves, n, total, keep);
  std::vector<std::string> out(size_t(n), "empty");
  for (int k = 0; k < b.n; ++k) {
    const int v = b.d[k].vec;
    out[size_t(keep[size_t(k)])] = v < 0 ? "pair" : v >= 3 ? "peeled" : v == 2 ? "vec16" : "vec8";
  }
  return out;
}

std::vector<LineBox> line_boxes(const MoveDesc *moves, int n, bool copies) {
  std::vector<LineBox> reads, writes, moved;
  auto add = [](std::vector<LineBox> &v, const MoveDesc &m, double *base, int64_t off) {
    if (m.s1 % 16 || m.s2 % 16 || m.s3 % 16)
      throw std::runtime_error("line_boxes: row strides must be whole 128-B lines");
    LineBox b;
    b.base = base;
    b.off = off / 16 * 16;
    b.lines = int32_t((off + m.len - 1) / 16 - off / 16 + 1);
    b.s1 = m.s1;
    b.s2 = m.s2;
    b.s3 = m.s3;
    b.n1 = m.n1;
    b.n2 = m.n2;
    b.n3 = m.n3;
    v.push_back(b);
  };
  for (int i = 0; i < n; ++i) {
    const MoveDesc &m = moves[i];
    double *src = const_cast<double *>(m.src);
    if (m.pair) {
      const int64_t delta = m.dst_off - m.src_off;
      add(reads, m, src, m.src_off);
      add(reads, m, src, m.src_off + m.len + delta);
      add(writes, m, m.dst, m.dst_off);
      add(writes, m, m.dst, m.src_off + m.len);
    } else {
      add(reads, m, src, m.src_off);
      add(writes, m, m.dst, m.dst_off);
      const LineBox &r = reads.back(), &w = writes.back();
      if (copies && r.lines == w.lines && m.src_off % 16 == m.dst_off % 16) {
        LineBox c = r;
        c.mode = 3;
        c.dst_base = w.base;
        c.dst_off = w.off;
        moved.push_back(c);
        reads.pop_back();
        writes.pop_back();
      }
    }
  }
  auto same = [](const LineBox &a, const LineBox &b) {
    return a.base == b.base && a.off == b.off && a.lines == b.lines && a.s1 == b.s1 && a.s2 == b.s2 &&
           a.s3 == b.s3 && a.n1 == b.n1 && a.n2 == b.n2 && a.n3 == b.n3;
  };
  std::vector<LineBox> out;
  std::vector<bool> merged(writes.size(), false);
  for (LineBox r : reads) {
    r.mode = 0;
    for (size_t k = 0; k < writes.size(); ++k)
      if (!merged[k] && same(r, writes[k])) {
        r.mode = 2;
        merged[k] = true;
        break;
      }
    out.push_back(r);
  }
  for (size_t k = 0; k < writes.size(); ++k)
    if (!merged[k]) {
      LineBox w = writes[k];
      w.mode = 1;
      out.push_back(w);
    }
  out.insert(out.begin(), moved.begin(), moved.end());
  return out;
}

void line_roof(const LineBox *boxes, int n, void *stream, int variant) {
  if (variant < 0 || variant >= kLineRoofVariants) throw std::runtime_error("line_roof: bad variant");
  static double *sink = nullptr;
  if (!sink && hipMalloc(&sink, 64) != hipSuccess) throw std::runtime_error("line_roof: hipMalloc");
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int k0 = 0; k0 < n; k0 += kMaxBoxes) {
    DevBatch b{};
    uint32_t total = 0;
    for (int i = k0; i < std::min(n, k0 + kMaxBoxes); ++i) {
      BoxDesc box;
      box.buf = boxes[i].base;
      box.grid_off = boxes[i].off;
      box.len = boxes[i].lines * 16;
      box.n1 = boxes[i].n1;
      box.n2 = boxes[i].n2;
      box.n3 = boxes[i].n3;
      box.s1 = boxes[i].s1;
      box.s2 = boxes[i].s2;
      box.s3 = boxes[i].s3;
      DevDesc d = make_dev(box);
      if (d.items == 0) continue;
      if (d.vec != 2) throw std::runtime_error("line_roof: boxes must be whole 128-B lines");
      d.buf = boxes[i].base;
      d.vec = boxes[i].mode;
      if (boxes[i].mode == 3) { // source: base; target: dst_base + dst_off, same geometry
        if (!boxes[i].dst_base) throw std::runtime_error("line_roof: copy box without a target");
        d.src = boxes[i].base;
        d.buf = boxes[i].base;
        d.delta = (boxes[i].dst_base - boxes[i].base) + (boxes[i].dst_off - boxes[i].off);
      }
      b.d[b.n] = d;
      b.block_start[b.n] = total;
      total += blocks_for(d, 0, std::max(1, box_tuning().move_items));
      ++b.n;
    }
    if (b.n == 0) continue;
    b.block_start[b.n] = total;
    switch (variant) { // (items in flight per lane, non-temporal stores)
    case 0: hipLaunchKernelGGL((line_roof_k<1, true>), dim3(total), dim3(kThreads), 0, s, b, 0.0, sink); break;
    case 1: hipLaunchKernelGGL((line_roof_k<4, true>), dim3(total), dim3(kThreads), 0, s, b, 0.0, sink); break;
    case 2: hipLaunchKernelGGL((line_roof_k<1, false>), dim3(total), dim3(kThreads), 0, s, b, 0.0, sink); break;
    default: hipLaunchKernelGGL((line_roof_k<4, false>), dim3(total), dim3(kThreads), 0, s, b, 0.0, sink); break;
    }
    TZ_HIP_LAUNCH_CHECK();
  }
}

} // namespace kern
} // namespace tz
