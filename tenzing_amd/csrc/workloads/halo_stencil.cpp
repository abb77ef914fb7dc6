// Halo workload, stencil mode: the 7-point stencil boxes (interior, boundary shell, whole box)
// and their device-side verification.
#include "halo_internal.hpp"

namespace tz {

kern::StencilBox HaloExchange::stencil_box(int x0, int x1, int y0, int y1, int z0, int z1) const {
  // cells [x0,x1) x [y0,y1) x [z0,z1) of the interior (interior coordinates)
  kern::StencilBox b;
  b.in = grid();
  b.out = out_.as<double>();
  const int64_t g = a_.ghost;
  if (a_.order == "xyzq") {
    b.base = (z0 + g) * sz_ + (y0 + g) * sy_ + (x0 + g) + xoff_;
    b.row = x1 - x0;
    b.xs = 1;
    b.so = sq_;
    b.nouter = a_.nq;
  } else {
    b.base = int64_t(a_.nq) * (x0 + g + xoff_) + (y0 + g) * sy_ + (z0 + g) * sz_;
    b.row = a_.nq * (x1 - x0);
    b.xs = a_.nq;
    b.so = 0;
    b.nouter = 1;
  }
  b.sy = sy_;
  b.sz = sz_;
  b.ny = y1 - y0;
  b.nz = z1 - z0;
  return b;
}

void HaloExchange::stencil(int region, void *stream) const {
  TZ_CHECK(ready() && out_.get(), "stencil mode not set up");
  const int X = a_.nx, Y = a_.ny, Z = a_.nz;
  std::vector<kern::StencilBox> boxes;
  if (region == 2) {
    boxes.push_back(stencil_box(0, X, 0, Y, 0, Z));
  } else if (region == 0) {
    // full rows with the first / last x cell masked: rows stay 16-B aligned
    if (X > 2 && Y > 2 && Z > 2) {
      kern::StencilBox b = stencil_box(0, X, 1, Y - 1, 1, Z - 1);
      b.m0 = b.m1 = b.xs;
      boxes.push_back(b);
    }
  } else {
    // the shell: two z planes, two y slabs between them, two x slabs inside those
    boxes.push_back(stencil_box(0, X, 0, Y, 0, 1));
    if (Z > 1) boxes.push_back(stencil_box(0, X, 0, Y, Z - 1, Z));
    if (Z > 2) {
      boxes.push_back(stencil_box(0, X, 0, 1, 1, Z - 1));
      if (Y > 1) boxes.push_back(stencil_box(0, X, Y - 1, Y, 1, Z - 1));
      if (Y > 2) {
        boxes.push_back(stencil_box(0, 1, 1, Y - 1, 1, Z - 1));
        if (X > 1) boxes.push_back(stencil_box(X - 1, X, 1, Y - 1, 1, Z - 1));
      }
    }
  }
  // thin boxes (the shell's slabs) share one launch; the rest go one by one
  std::vector<kern::StencilBox> thin;
  for (const auto &b : boxes) {
    if (kern::stencil_thin(b)) thin.push_back(b);
    else kern::stencil7(b, true, stream);
  }
  if (!thin.empty()) kern::stencil7_thin_many(thin.data(), int(thin.size()), stream);
}

uint64_t HaloExchange::check_stencil(void *stream) {
  TZ_CHECK(ready() && out_.get(), "stencil mode not set up");
  hipStream_t s = static_cast<hipStream_t>(stream);
  TZ_HIP(hipMemsetAsync(count_.get(), 0, sizeof(unsigned long long), s));
  kern::stencil_check(out_.as<double>(), geom(), count_.as<unsigned long long>(), stream);
  unsigned long long n = 0;
  TZ_HIP(hipMemcpyAsync(&n, count_.get(), sizeof(n), hipMemcpyDeviceToHost, s));
  TZ_HIP(hipStreamSynchronize(s));
  return n;
}

} // namespace tz
