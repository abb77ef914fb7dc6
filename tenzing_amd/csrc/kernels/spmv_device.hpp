// Device bodies shared by the SpMV kernels (spmv_kernels.hip) and the fused move + SpMV kernel
// (halo_kernels.hip). Device code only: include from .hip translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace tz {
namespace kern {
namespace dev {

// CSR with instruction-level parallelism, for global thread `gtid`: W lanes per row, and every
// lane issues all K of its column loads, then all K value loads and x gathers, before it uses
// any (one pass covers W*K entries of the row). Short rows (10 entries on average here) then cost
// one latency chain per row (row pointers -> columns -> x) with few, loaded waves, instead of one
// chain per W entries on 4-8x as many waves. Whole W-lane groups exit together (W divides 64).
template <int W, int K>
__device__ __forceinline__ void csr_spmv_ilp_row(int gtid, int nRows, const int32_t *__restrict__ rowPtr,
                                                 const int32_t *__restrict__ colInd,
                                                 const float *__restrict__ val,
                                                 const float *__restrict__ x, float *__restrict__ y,
                                                 int accumulate) {
  const int row = gtid / W;
  const int lane = gtid & (W - 1);
  if (row >= nRows) return;
  const int b = rowPtr[row], e = rowPtr[row + 1];
  float sum = 0.f;
  for (int j0 = b + lane; j0 < e; j0 += W * K) {
    int c[K];
    float v[K], xv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = j0 + k * W;
      c[k] = j < e ? colInd[j] : -1;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int j = j0 + k * W;
      v[k] = j < e ? val[j] : 0.f;
      xv[k] = c[k] >= 0 ? x[c[k]] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) sum = fmaf(v[k], xv[k], sum);
  }
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) sum += __shfl_xor(sum, off, W);
  if (lane == 0) y[row] = accumulate ? y[row] + sum : sum;
}

} // namespace dev
} // namespace kern
} // namespace tz
