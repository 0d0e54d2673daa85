// Shared by qnet.hip (k_linear_relu_rows) and fc.hip (k_fc_reduce_rows): one workgroup of the
// device-counted FC1 tail rows.  Rows [r0, min(*n_dev, n_max)) of y = relu(x w^T + b), x [*, F]
// row stride ldx, w [O, F], y row stride ldy; workgroup `blk` = kLrCols output columns; the rows
// go in chunks of kLrRows, each lane a strided float4 slice of F, the partial dots summed by xor
// shuffles and then across the waves in a fixed order (deterministic).
#pragma once

#include "common.hpp"

namespace rth {

constexpr int kLrCols = 4, kLrRows = 8, kLrThreads = 256;
__device__ __forceinline__ void linear_relu_rows_wg(int blk, const float *__restrict__ x, int64_t ldx, int64_t r0,
                                                    int64_t n_max, const int64_t *__restrict__ n_dev,
                                                    const float *__restrict__ w, const float *__restrict__ b, int F,
                                                    int O, float *__restrict__ y, int64_t ldy) {
  int64_t n_end = *n_dev;
  n_end = n_end < n_max ? n_end : n_max;
  if (n_end <= r0) return;  // uniform
  __shared__ float red[kLrThreads / 64][kLrCols * kLrRows];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, F4 = F / 4;
  const int j0 = blk * kLrCols;
  const float4 *w4 = reinterpret_cast<const float4 *>(w);
  for (int64_t rb = r0; rb < n_end; rb += kLrRows) {
    float acc[kLrCols][kLrRows];
#pragma unroll
    for (int c = 0; c < kLrCols; ++c)
#pragma unroll
      for (int u = 0; u < kLrRows; ++u) acc[c][u] = 0.0f;
    for (int f4 = tid; f4 < F4; f4 += kLrThreads) {
      float4 wv[kLrCols];
#pragma unroll
      for (int c = 0; c < kLrCols; ++c)
        wv[c] = j0 + c < O ? w4[(int64_t)(j0 + c) * F4 + f4] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
      for (int u = 0; u < kLrRows; ++u) {
        if (rb + u >= n_end) break;  // uniform
        const float4 xv = reinterpret_cast<const float4 *>(x + (rb + u) * ldx)[f4];
#pragma unroll
        for (int c = 0; c < kLrCols; ++c)
          acc[c][u] = radd(radd(radd(radd(acc[c][u], rmul(xv.x, wv[c].x)), rmul(xv.y, wv[c].y)),
                                rmul(xv.z, wv[c].z)), rmul(xv.w, wv[c].w));
      }
    }
#pragma unroll
    for (int c = 0; c < kLrCols; ++c)
#pragma unroll
      for (int u = 0; u < kLrRows; ++u) {
        float v = acc[c][u];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = radd(v, __shfl_xor(v, o, 64));
        if (lane == 0) red[wave][c * kLrRows + u] = v;
      }
    __syncthreads();
    if (tid < kLrCols * kLrRows) {
      const int c = tid / kLrRows, u = tid % kLrRows;
      if (rb + u < n_end && j0 + c < O) {
        float v = b[j0 + c];
#pragma unroll
        for (int k = 0; k < kLrThreads / 64; ++k) v = radd(v, red[k][tid]);
        y[(rb + u) * ldy + j0 + c] = v > 0.0f ? v : 0.0f;
      }
    }
    __syncthreads();
  }
}

}  // namespace rth
