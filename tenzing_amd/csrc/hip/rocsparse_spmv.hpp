// rocSPARSE CSR SpMV as a library comparison variant of the hand-written kernels.
//
// Reference: SpMVKernel wraps cusparseSpMV (CSR_ALG2, alpha 1, beta 0) and creates a handle,
// descriptors and a work buffer per instance (include/tenzing/spmv/ops_spmv.cuh:61-163). Here
// one handle/descriptor set is created at setup (not per op clone) and the search can pick it
// against the hand-written wave64 kernels (SpMV local-product ChoiceOp).
#pragma once

#include <cstddef>
#include <cstdint>

namespace tz {

class RocsparseCsr {
public:
  /// y = A x for an m x n f32 CSR matrix (i32 indices) already resident on the device.
  /// `alg`: "adaptive", "lrb", "rowsplit" or "nnzsplit" (nnzsplit: not implemented for this
  /// configuration by the ROCm 7.2 rocSPARSE)
  RocsparseCsr(int64_t m, int64_t n, int64_t nnz, const int32_t *rowPtr, const int32_t *colInd,
               const float *val, const float *x, float *y, const char *alg = "adaptive");
  ~RocsparseCsr();
  RocsparseCsr(const RocsparseCsr &) = delete;
  RocsparseCsr &operator=(const RocsparseCsr &) = delete;
  /// y = A x (beta 0) or y += A x (accumulate) on `stream` (compute stage only: capturable)
  void run(void *stream, bool accumulate = false) const;

private:
  void *handle_ = nullptr, *mat_ = nullptr, *x_ = nullptr, *y_ = nullptr, *descr_ = nullptr;
  void *buf_ = nullptr;
  size_t bufBytes_ = 0;
};

} // namespace tz
