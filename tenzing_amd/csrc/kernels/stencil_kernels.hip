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

constexpr int TX = 64, TY = 8, XS_MAX = 4, ZC = 32;
constexpr int LW = TX + 2 * XS_MAX; // LDS row width (doubles)

__device__ __forceinline__ double ldnt(const double *p) { return __builtin_nontemporal_load(p); }

template <bool LDS>
__global__ __launch_bounds__(TX *TY) void stencil7_k(StencilBox b) {
  __shared__ double tile[TY + 2][LW];
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int r = blockIdx.x * TX + tx;          // element within the row
  const int y = blockIdx.y * TY + ty;          // row
  const int zChunks = (b.nz + ZC - 1) / ZC;
  const int outer = blockIdx.z / zChunks;      // XYZQ: quantity
  const int z0 = (blockIdx.z % zChunks) * ZC;
  const int z1 = min(z0 + ZC, b.nz);
  const bool mine = r < b.row && y < b.ny; // an output element of the box
  // the x / y neighbours of the box's last column / row are elements just outside the box:
  // threads there still load their (real) value into the tile
  const bool live = LDS ? (r < b.row + b.xs && y <= b.ny) : mine;
  const int64_t e0 = b.base + int64_t(outer) * b.so + int64_t(y) * b.sy + r; // plane 0 offset
  const double *in = b.in;

  // registers: z - 1 and z of this element (z + 1 is loaded inside the loop)
  double prev = mine ? in[e0 + int64_t(z0 - 1) * b.sz] : 0.0;
  double cur = live ? in[e0 + int64_t(z0) * b.sz] : 0.0;
  for (int z = z0; z < z1; ++z) {
    const int64_t e = e0 + int64_t(z) * b.sz;
    const double next = live ? ldnt(in + e + b.sz) : 0.0;
    double xm, xp, ym, yp;
    if (LDS) {
      // this plane: my element, plus the apron (xs columns left/right, one row above/below)
      tile[ty + 1][tx + XS_MAX] = cur;
      const int64_t p = b.base + int64_t(outer) * b.so + int64_t(z) * b.sz;
      const int rx0 = blockIdx.x * TX, ry0 = blockIdx.y * TY;
      for (int k = threadIdx.x; k < 2 * LW + 2 * TY * XS_MAX; k += TX * TY) {
        int lr, lc; // LDS row / column
        if (k < 2 * LW) {
          lr = k < LW ? 0 : TY + 1;
          lc = k % LW;
        } else {
          const int j = k - 2 * LW;
          lr = 1 + j / (2 * XS_MAX);
          const int c = j % (2 * XS_MAX);
          lc = c < XS_MAX ? c : TX + c; // left apron [0, XS_MAX), right [TX+XS_MAX, LW)
        }
        const int gr = rx0 + lc - XS_MAX, gy = ry0 + lr - 1;
        // apron cells outside [-xs, row + xs) x [-1, ny] feed no stored output: skip them
        const bool ok = gr >= -b.xs && gr < b.row + b.xs && gy >= -1 && gy <= b.ny;
        tile[lr][lc] = ok ? in[p + int64_t(gy) * b.sy + gr] : 0.0;
      }
      __syncthreads();
      xm = tile[ty + 1][tx + XS_MAX - b.xs];
      xp = tile[ty + 1][tx + XS_MAX + b.xs];
      ym = tile[ty][tx + XS_MAX];
      yp = tile[ty + 2][tx + XS_MAX];
    } else {
      xm = mine ? in[e - b.xs] : 0.0;
      xp = mine ? in[e + b.xs] : 0.0;
      ym = mine ? in[e - b.sy] : 0.0;
      yp = mine ? in[e + b.sy] : 0.0;
    }
    if (mine)
      __builtin_nontemporal_store(b.c0 * cur + b.c1 * (xm + xp + ym + yp + prev + next), b.out + e);
    if (LDS) __syncthreads(); // the tile is rewritten for the next plane
    prev = cur;
    cur = next;
  }
}

} // namespace

void stencil7(const StencilBox &b, bool lds, void *stream) {
  if (b.row <= 0 || b.ny <= 0 || b.nz <= 0 || b.nouter <= 0) return;
  if (!b.in || !b.out) throw std::runtime_error("stencil7: null grid");
  if (b.xs < 1 || b.xs > XS_MAX) throw std::runtime_error("stencil7: x neighbour distance must be 1..4");
  const int zChunks = (b.nz + ZC - 1) / ZC;
  const dim3 g(unsigned((b.row + TX - 1) / TX), unsigned((b.ny + TY - 1) / TY),
               unsigned(zChunks * b.nouter));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (lds) hipLaunchKernelGGL(stencil7_k<true>, g, dim3(TX * TY), 0, s, b);
  else hipLaunchKernelGGL(stencil7_k<false>, g, dim3(TX * TY), 0, s, b);
  TZ_HIP_LAUNCH_CHECK();
}

} // namespace kern
} // namespace tz
