#include "rocsparse_spmv.hpp"

#include "core/util.hpp"
#include "hip/hip_runtime.hpp"

#include <hip/hip_runtime_api.h>
#include <rocsparse/rocsparse.h>

#include <cstring>

namespace tz {

#define TZ_RS(x)                                                                                   \
  do {                                                                                             \
    rocsparse_status s_ = (x);                                                                     \
    if (s_ != rocsparse_status_success) TZ_THROW(#x << " failed: rocsparse status " << int(s_));   \
  } while (0)

static rocsparse_spmv_alg parse_alg(const char *a) {
  if (!std::strcmp(a, "adaptive")) return rocsparse_spmv_alg_csr_adaptive;
  if (!std::strcmp(a, "lrb")) return rocsparse_spmv_alg_csr_lrb;
  if (!std::strcmp(a, "rowsplit")) return rocsparse_spmv_alg_csr_rowsplit;
  if (!std::strcmp(a, "nnzsplit")) return rocsparse_spmv_alg_csr_nnzsplit;
  TZ_THROW("unknown rocSPARSE CSR algorithm " << a);
}

RocsparseCsr::RocsparseCsr(int64_t m, int64_t n, int64_t nnz, const int32_t *rowPtr,
                           const int32_t *colInd, const float *val, const float *x, float *y,
                           const char *alg) {
  rocsparse_handle h = nullptr;
  TZ_RS(rocsparse_create_handle(&h));
  handle_ = h;
  rocsparse_spmat_descr A = nullptr;
  TZ_RS(rocsparse_create_csr_descr(&A, m, n, nnz, const_cast<int32_t *>(rowPtr),
                                   const_cast<int32_t *>(colInd), const_cast<float *>(val),
                                   rocsparse_indextype_i32, rocsparse_indextype_i32,
                                   rocsparse_index_base_zero, rocsparse_datatype_f32_r));
  mat_ = A;
  rocsparse_dnvec_descr dx = nullptr, dy = nullptr;
  TZ_RS(rocsparse_create_dnvec_descr(&dx, n, const_cast<float *>(x), rocsparse_datatype_f32_r));
  x_ = dx;
  TZ_RS(rocsparse_create_dnvec_descr(&dy, m, y, rocsparse_datatype_f32_r));
  y_ = dy;
  rocsparse_spmv_descr d = nullptr;
  TZ_RS(rocsparse_create_spmv_descr(&d));
  descr_ = d;
  const rocsparse_spmv_alg a = parse_alg(alg);
  const rocsparse_operation op = rocsparse_operation_none;
  const rocsparse_datatype dt = rocsparse_datatype_f32_r;
  TZ_RS(rocsparse_spmv_set_input(h, d, rocsparse_spmv_input_alg, &a, sizeof(a), nullptr));
  TZ_RS(rocsparse_spmv_set_input(h, d, rocsparse_spmv_input_operation, &op, sizeof(op), nullptr));
  TZ_RS(rocsparse_spmv_set_input(h, d, rocsparse_spmv_input_scalar_datatype, &dt, sizeof(dt), nullptr));
  TZ_RS(rocsparse_spmv_set_input(h, d, rocsparse_spmv_input_compute_datatype, &dt, sizeof(dt), nullptr));
  // analysis once at setup (the reference re-creates its cuSPARSE state per op clone)
  size_t an = 0;
  TZ_RS(rocsparse_v2_spmv_buffer_size(h, d, A, dx, dy, rocsparse_v2_spmv_stage_analysis, &an, nullptr));
  size_t cb = 0;
  TZ_RS(rocsparse_v2_spmv_buffer_size(h, d, A, dx, dy, rocsparse_v2_spmv_stage_compute, &cb, nullptr));
  bufBytes_ = std::max<size_t>({an, cb, 256});
  TZ_HIP(hipMalloc(&buf_, bufBytes_));
  const float one = 1.f, zero = 0.f;
  TZ_RS(rocsparse_v2_spmv(h, d, &one, A, dx, &zero, dy, rocsparse_v2_spmv_stage_analysis, bufBytes_,
                          buf_, nullptr));
  TZ_HIP(hipDeviceSynchronize());
}

RocsparseCsr::~RocsparseCsr() {
  if (descr_) rocsparse_destroy_spmv_descr(static_cast<rocsparse_spmv_descr>(descr_));
  if (x_) rocsparse_destroy_dnvec_descr(static_cast<rocsparse_dnvec_descr>(x_));
  if (y_) rocsparse_destroy_dnvec_descr(static_cast<rocsparse_dnvec_descr>(y_));
  if (mat_) rocsparse_destroy_spmat_descr(static_cast<rocsparse_spmat_descr>(mat_));
  if (handle_) rocsparse_destroy_handle(static_cast<rocsparse_handle>(handle_));
  if (buf_) (void)hipFree(buf_);
}

void RocsparseCsr::run(void *stream, bool accumulate) const {
  rocsparse_handle h = static_cast<rocsparse_handle>(handle_);
  TZ_RS(rocsparse_set_stream(h, static_cast<hipStream_t>(stream)));
  const float one = 1.f, beta = accumulate ? 1.f : 0.f;
  TZ_RS(rocsparse_v2_spmv(h, static_cast<rocsparse_spmv_descr>(descr_), &one,
                          static_cast<rocsparse_spmat_descr>(mat_),
                          static_cast<rocsparse_dnvec_descr>(x_), &beta,
                          static_cast<rocsparse_dnvec_descr>(y_), rocsparse_v2_spmv_stage_compute,
                          bufBytes_, buf_, nullptr));
}

} // namespace tz
