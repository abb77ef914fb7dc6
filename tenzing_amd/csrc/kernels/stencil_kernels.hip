// 7-point stencil on the halo grid (gfx950): the compute that a halo exchange exists to feed.
//
// Not in the reference (its halo workload stops at the exchange). It lets the
// search do what real stencil codes do with an exchange: update the interior, which needs no
// ghost, while the ghosts are in flight, and the one-cell boundary shell afterwards.
//
// out[e] = c0 * in[e] + c1 * (in[e-xs] + in[e+xs] + in[e-sy] + in[e+sy] + in[e-sz] + in[e+sz])
// for every element e of a box (both storage orders: a "row" is the box's contiguous run, xs
// the distance of the x neighbour: nq for QXYZ, 1 for XYZQ; XYZQ boxes add an outer q loop).
//
// Kernel (2.5-D blocking): a 64 x 8 workgroup (one wave64 per row segment, 8 rows) owns a tile
// of 64 contiguous elements x 8 rows and marches up z through a chunk of planes. Each plane
// goes through LDS with a one-row / xs-column apron, so the x and y neighbours come from LDS;
// the z neighbours live in registers (previous plane, current plane, next plane), and the next
// plane's value is the one global load per element that the kernel needs. Loads of the next
// plane and stores of the output are non-temporal (each element is touched once).
#include <hip/hip_runtime.h>

#include "kernels.hpp"

#include <algorithm>
#include <cstdint>
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

constexpr int TX = 64, XS_MAX = 4;

__device__ __forceinline__ double ldnt(const double *p) { return __builtin_nontemporal_load(p); }

typedef double dbl2_t __attribute__((ext_vector_type(2)));

// VX consecutive elements per thread (VX = 2: 16-B loads/stores of the z queue and the output)
template <int VX> struct VT;
template <> struct VT<1> {
  using T = double;
  __device__ static T zero() { return 0.0; }
  __device__ static double get(const T &v, int) { return v; }
};
template <> struct VT<2> {
  using T = dbl2_t;
  __device__ static T zero() { return T{0.0, 0.0}; }
  __device__ static double get(const T &v, int k) { return k ? v.y : v.x; }
};

// PF: planes prefetched ahead of the z + 1 plane (1: z + 2; 2: z + 2 and z + 3), i.e. the
// loads each lane keeps in flight; the tile is double-buffered, one barrier per plane
// Tile order of the launch: per = 0, the hardware order (blockIdx.x / y / z = x tile, row tile,
// z chunk, so consecutive workgroups -- dealt round-robin to the 8 XCDs -- sit on different XCDs
// and a tile's row apron comes from another XCD's L2 or from memory); per > 0, a 1-D launch of
// 8 * per workgroups where XCD k runs tiles [k * per, (k + 1) * per) in (x, row, z-chunk) order,
// so the tiles above and below a tile run on its own XCD at about the same time
struct TileGrid {
  uint32_t gx, gy, gz, per;
};

template <bool LDS, int VX, int TY, int ZC, int PF, bool DB>
__global__ __launch_bounds__(TX *TY) void stencil7_k(StencilBox b, TileGrid tg) {
  uint32_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (tg.per) {
    const uint32_t l = (blockIdx.x % 8u) * tg.per + blockIdx.x / 8u;
    if (l >= tg.gx * tg.gy * tg.gz) return; // launch padding: the whole workgroup, before any barrier
    bx = l % tg.gx;
    by = (l / tg.gx) % tg.gy;
    bz = l / (tg.gx * tg.gy);
  }
  using V = VT<VX>;
  using T = typename V::T;
  constexpr int W = TX * VX;              // elements per tile row
  constexpr int LW = W + 2 * XS_MAX;      // LDS row width
  __shared__ double tiles[LDS && DB ? 2 : 1][TY + 2][LW];
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int r = int(bx) * W + tx * VX; // first element of this thread within the row
  const int y = int(by) * TY + ty;     // row
  const int zChunks = (b.nz + ZC - 1) / ZC;
  const int outer = int(bz) / zChunks; // XYZQ: quantity
  const int z0 = (int(bz) % zChunks) * ZC;
  const int z1 = min(z0 + ZC, b.nz);
  // VX = 2 launches only when row is even: a thread's two elements are both in or both out
  // output elements of the box (m0 / m1 masked at the row ends); VX = 2 pairs straddling a
  // mask edge store element by element
  const int rlo = b.m0, rhi = b.row - b.m1;
  const bool mine = r + VX > rlo && r < rhi && y < b.ny;
  // the x / y neighbours of the box's last column / row are elements just outside the box:
  // threads there still load their (real) value into the tile (never past the masked ends)
  const int llo = rlo - b.xs, lhi = rhi + b.xs;
  const bool live = LDS ? (r + VX > llo && r < lhi && y <= b.ny) : mine;
  const int64_t e0 = b.base + int64_t(outer) * b.so + int64_t(y) * b.sy + r; // plane 0 offset
  const double *in = b.in;
  auto load = [&](int64_t e) { return *reinterpret_cast<const T *>(in + e); };

  // apron cells of the LDS tile (xs columns left/right, one row above/below): each thread owns
  // up to two, and loads them one plane ahead like the z queue, so no load sits between a
  // plane's barrier and its compute
  constexpr int NAPRON = 2 * LW + 2 * TY * XS_MAX;
  constexpr int NT = TX * TY;
  int alr[2], alc[2], agr[2], agy[2];
  bool aok[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int k = threadIdx.x + a * NT;
    int lr = 0, lc = 0;
    if (k < 2 * LW) {
      lr = k < LW ? 0 : TY + 1;
      lc = k % LW;
    } else if (k < NAPRON) {
      const int j = k - 2 * LW;
      lr = 1 + j / (2 * XS_MAX);
      const int c = j % (2 * XS_MAX);
      lc = c < XS_MAX ? c : W + c; // left apron [0, XS_MAX), right [W+XS_MAX, LW)
    }
    alr[a] = lr;
    alc[a] = lc;
    agr[a] = int(bx) * W + lc - XS_MAX;
    agy[a] = int(by) * TY + lr - 1;
    // apron cells outside [-xs, row + xs) x [-1, ny] feed no stored output: never loaded
    aok[a] = LDS && k < NAPRON && agr[a] >= llo && agr[a] < lhi && agy[a] >= -1 && agy[a] <= b.ny;
  }
  const int64_t pbase = b.base + int64_t(outer) * b.so;
  auto apron = [&](int a, int z) {
    return aok[a] ? in[pbase + int64_t(z) * b.sz + int64_t(agy[a]) * b.sy + agr[a]] : 0.0;
  };

  // register queue: planes z - 1, z, z + 1 of my elements, and z + 2 .. z + 1 + PF in flight
  // (at most plane nz, the ghost plane, of the last chunk)
  auto loadnt = [&](int zz) {
    return live && zz <= b.nz
               ? __builtin_nontemporal_load(reinterpret_cast<const T *>(in + e0 + int64_t(zz) * b.sz))
               : V::zero();
  };
  T prev = mine ? load(e0 + int64_t(z0 - 1) * b.sz) : V::zero();
  T cur = live ? load(e0 + int64_t(z0) * b.sz) : V::zero();
  T next = live ? load(e0 + int64_t(z0 + 1) * b.sz) : V::zero();
  T ahead[PF];
#pragma unroll
  for (int p = 0; p + 1 < PF; ++p) ahead[p] = loadnt(z0 + 2 + p);
  double ap0 = apron(0, z0), ap1 = apron(1, z0);
  for (int z = z0; z < z1; ++z) {
    const int64_t e = e0 + int64_t(z) * b.sz;
    ahead[PF - 1] = loadnt(z + 1 + PF);
    auto &tile = tiles[LDS && DB ? (z - z0) & 1 : 0];
    double xm[VX], xp[VX], ym[VX], yp[VX];
    if (LDS) {
#pragma unroll
      for (int k = 0; k < VX; ++k) tile[ty + 1][XS_MAX + tx * VX + k] = V::get(cur, k);
      if (aok[0]) tile[alr[0]][alc[0]] = ap0;
      if (aok[1]) tile[alr[1]][alc[1]] = ap1;
      // next plane's apron (plane z + 1 <= nz exists)
      if (z + 1 < z1) {
        ap0 = apron(0, z + 1);
        ap1 = apron(1, z + 1);
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < VX; ++k) {
        const int c = XS_MAX + tx * VX + k;
        xm[k] = tile[ty + 1][c - b.xs];
        xp[k] = tile[ty + 1][c + b.xs];
        ym[k] = tile[ty][c];
        yp[k] = tile[ty + 2][c];
      }
    } else {
#pragma unroll
      for (int k = 0; k < VX; ++k) {
        xm[k] = mine ? in[e + k - b.xs] : 0.0;
        xp[k] = mine ? in[e + k + b.xs] : 0.0;
        ym[k] = mine ? in[e + k - b.sy] : 0.0;
        yp[k] = mine ? in[e + k + b.sy] : 0.0;
      }
    }
    if (mine) {
      T o;
      if constexpr (VX == 1) {
        o = b.c0 * cur + b.c1 * (xm[0] + xp[0] + ym[0] + yp[0] + prev + next);
        __builtin_nontemporal_store(o, b.out + e);
      } else {
        o.x = b.c0 * cur.x + b.c1 * (xm[0] + xp[0] + ym[0] + yp[0] + prev.x + next.x);
        o.y = b.c0 * cur.y + b.c1 * (xm[1] + xp[1] + ym[1] + yp[1] + prev.y + next.y);
        if (r >= rlo && r + 1 < rhi) {
          __builtin_nontemporal_store(o, reinterpret_cast<T *>(b.out + e));
        } else {
          if (r >= rlo) b.out[e] = o.x;
          if (r + 1 >= rlo && r + 1 < rhi) b.out[e + 1] = o.y;
        }
      }
    }
    // double-buffered: no second barrier (the next plane writes the other tile, and every
    // thread has left this plane's reads behind before anyone passes the next plane's barrier)
    if (LDS && !DB) __syncthreads();
    prev = cur;
    cur = next;
    next = ahead[0];
#pragma unroll
    for (int p = 0; p + 1 < PF; ++p) ahead[p] = ahead[p + 1];
  }
}

// thin boxes (the one-cell boundary shell): one thread per output element, neighbours from
// global memory (L2) — a z-march or a 64-wide tile would leave most lanes idle on a slab that
// is one cell thick. Up to kMaxFlat boxes in one launch (blocks map to boxes through a prefix
// table), 4 elements in flight per thread.
constexpr int kMaxFlat = 8;
struct FlatBatch {
  StencilBox b[kMaxFlat];
  uint32_t block_start[kMaxFlat + 1];
  int32_t n;
};

__device__ __forceinline__ void flat_one(const StencilBox &b, int64_t it) {
  const int64_t i = it % b.row;
  if (i < b.m0 || i >= b.row - b.m1) return;
  int64_t r = it / b.row;
  const int64_t y = r % b.ny;
  r /= b.ny;
  const int64_t z = r % b.nz;
  const int64_t o = r / b.nz;
  const int64_t e = b.base + o * b.so + z * b.sz + y * b.sy + i;
  const double *in = b.in;
  b.out[e] = b.c0 * in[e] + b.c1 * (in[e - b.xs] + in[e + b.xs] + in[e - b.sy] + in[e + b.sy] +
                                    in[e - b.sz] + in[e + b.sz]);
}

__global__ __launch_bounds__(256) void stencil7_flat_k(FlatBatch fb) {
  int k = 0;
  while (k + 1 < fb.n && blockIdx.x >= fb.block_start[k + 1]) ++k;
  const StencilBox &b = fb.b[k];
  const int64_t total = int64_t(b.row) * b.ny * b.nz * b.nouter;
  const int64_t nth = int64_t(fb.block_start[k + 1] - fb.block_start[k]) * 256;
  int64_t it = int64_t(blockIdx.x - fb.block_start[k]) * 256 + threadIdx.x;
  for (; it + 3 * nth < total; it += 4 * nth) {
#pragma unroll
    for (int u = 0; u < 4; ++u) flat_one(b, it + u * nth);
  }
  for (; it < total; it += nth) flat_one(b, it);
}

} // namespace

bool stencil_thin(const StencilBox &b) { return b.nz < 4 || b.ny < 4 || b.row < 32; }

void stencil7_thin_many(const StencilBox *boxes, int n, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int k0 = 0; k0 < n; k0 += kMaxFlat) {
    FlatBatch fb{};
    uint32_t total = 0;
    for (int k = k0; k < n && fb.n < kMaxFlat; ++k) {
      const StencilBox &b = boxes[k];
      const int64_t items = int64_t(b.row) * b.ny * b.nz * b.nouter;
      if (items <= 0) continue;
      if (!b.in || !b.out) throw std::runtime_error("stencil7: null grid");
      fb.b[fb.n] = b;
      fb.block_start[fb.n] = total;
      total += uint32_t(std::min<int64_t>((items + 1023) / 1024, 8192)); // 4 per thread
      ++fb.n;
    }
    if (fb.n == 0) continue;
    fb.block_start[fb.n] = total;
    hipLaunchKernelGGL(stencil7_flat_k, dim3(total), dim3(256), 0, s, fb);
    TZ_HIP_LAUNCH_CHECK();
  }
}

StencilTuning &stencil_tuning() {
  static StencilTuning t;
  return t;
}

namespace {
template <bool LDS, int VX, int TY, int ZC, int PF, bool DB>
void launch_stencil_db(const StencilBox &b, hipStream_t s) {
  const int W = TX * VX;
  const int zChunks = (b.nz + ZC - 1) / ZC;
  TileGrid tg{unsigned((b.row + W - 1) / W), unsigned((b.ny + TY - 1) / TY), unsigned(zChunks * b.nouter), 0};
  dim3 g(tg.gx, tg.gy, tg.gz);
  if (stencil_tuning().xcd_tiles) {
    const uint64_t total = uint64_t(tg.gx) * tg.gy * tg.gz;
    if (total >= (uint64_t(1) << 31)) throw std::runtime_error("stencil7: too many tiles");
    tg.per = unsigned((total + 7) / 8);
    g = dim3(tg.per * 8);
  }
  hipLaunchKernelGGL((stencil7_k<LDS, VX, TY, ZC, PF, DB>), g, dim3(TX * TY), 0, s, b, tg);
}

template <bool LDS, int VX, int TY, int ZC, int PF>
void launch_stencil(const StencilBox &b, hipStream_t s) {
  if (stencil_tuning().db) launch_stencil_db<LDS, VX, TY, ZC, PF, true>(b, s);
  else launch_stencil_db<LDS, VX, TY, ZC, PF, false>(b, s);
}

template <bool LDS, int VX, int TY>
void launch_zc(const StencilBox &b, hipStream_t s) {
  const StencilTuning &t = stencil_tuning();
  if (t.zc == 64) {
    if (t.pf >= 2) launch_stencil<LDS, VX, TY, 64, 2>(b, s);
    else launch_stencil<LDS, VX, TY, 64, 1>(b, s);
  } else if (t.zc == 128) {
    launch_stencil<LDS, VX, TY, 128, 1>(b, s);
  } else if (t.zc == 16) {
    if (t.pf >= 2) launch_stencil<LDS, VX, TY, 16, 2>(b, s);
    else launch_stencil<LDS, VX, TY, 16, 1>(b, s);
  } else {
    if (t.pf >= 2) launch_stencil<LDS, VX, TY, 32, 2>(b, s);
    else launch_stencil<LDS, VX, TY, 32, 1>(b, s);
  }
}

template <bool LDS, int VX>
void launch_ty(const StencilBox &b, hipStream_t s) {
  const StencilTuning &t = stencil_tuning();
  if (t.ty == 16) launch_zc<LDS, VX, 16>(b, s);
  else launch_zc<LDS, VX, 8>(b, s);
}
} // namespace

void stencil7(const StencilBox &b, bool lds, void *stream) {
  if (b.row <= 0 || b.ny <= 0 || b.nz <= 0 || b.nouter <= 0) return;
  if (!b.in || !b.out) throw std::runtime_error("stencil7: null grid");
  if (b.xs < 1 || b.xs > XS_MAX) throw std::runtime_error("stencil7: x neighbour distance must be 1..4");
  // two elements per thread (16-B accesses) when every row of the box starts 16-B aligned
  const bool v2 = b.row % 2 == 0 && b.base % 2 == 0 && b.sy % 2 == 0 && b.sz % 2 == 0 &&
                  b.so % 2 == 0 && reinterpret_cast<uintptr_t>(b.in) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.out) % 16 == 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (stencil_thin(b)) {
    stencil7_thin_many(&b, 1, stream);
    return;
  }
  if (lds && v2) launch_ty<true, 2>(b, s);
  else if (lds) launch_ty<true, 1>(b, s);
  else if (v2) launch_ty<false, 2>(b, s);
  else launch_ty<false, 1>(b, s);
  TZ_HIP_LAUNCH_CHECK();
}

} // namespace kern
} // namespace tz
