// Development aid (r06): the actors' counted FC1 tail row (y[j] = relu(b[j] + x . w[j]), one row,
// F = 3136) computed three ways, to tell which cross-lane mechanism loses data while a
// k_fc_x9t launch shares the CUs (scripts/diag_tail_concurrency.py):
//   form 0: xor shuffles (ds_bpermute) within each wave + the 4 waves' sums through LDS
//           (k_linear_relu_rows' scheme);
//   form 1: LDS only -- every lane's partial into LDS, one lane sums them in order;
//   form 2: shuffles only -- one wave per workgroup, no LDS.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/probes/librows_probe.so scripts/probes/rows_probe.hip
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void k_rows_shfl_lds(const float *x, const float *w, const float *b, int F, float *y) {
  __shared__ float red[4];
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float acc = 0.0f;
  for (int f = tid; f < F; f += 256) acc += x[f] * w[(size_t)j * F + f];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (tid == 0) {
    const float v = b[j] + red[0] + red[1] + red[2] + red[3];
    y[j] = v > 0.0f ? v : 0.0f;
  }
}

__global__ __launch_bounds__(256) void k_rows_lds(const float *x, const float *w, const float *b, int F, float *y) {
  __shared__ float part[256];
  const int j = blockIdx.x, tid = threadIdx.x;
  float acc = 0.0f;
  for (int f = tid; f < F; f += 256) acc += x[f] * w[(size_t)j * F + f];
  part[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    float v = b[j];
    for (int k = 0; k < 256; ++k) v += part[k];
    y[j] = v > 0.0f ? v : 0.0f;
  }
}

__global__ __launch_bounds__(64) void k_rows_shfl(const float *x, const float *w, const float *b, int F, float *y) {
  const int j = blockIdx.x, lane = threadIdx.x;
  float acc = 0.0f;
  for (int f = lane; f < F; f += 64) acc += x[f] * w[(size_t)j * F + f];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) {
    const float v = b[j] + acc;
    y[j] = v > 0.0f ? v : 0.0f;
  }
}

extern "C" int rows_probe(int form, const void *x, const void *w, const void *b, int F, int O, void *y, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float *xf = static_cast<const float *>(x), *wf = static_cast<const float *>(w), *bf = static_cast<const float *>(b);
  float *yf = static_cast<float *>(y);
  if (form == 0) hipLaunchKernelGGL(k_rows_shfl_lds, dim3(O), dim3(256), 0, s, xf, wf, bf, F, yf);
  else if (form == 1) hipLaunchKernelGGL(k_rows_lds, dim3(O), dim3(256), 0, s, xf, wf, bf, F, yf);
  else hipLaunchKernelGGL(k_rows_shfl, dim3(O), dim3(64), 0, s, xf, wf, bf, F, yf);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// forms 3..: the tail-row scheme of linear_relu_rows_wg itself (form 3: the library's code,
// included), then variants of it: COLS output columns per workgroup, ROWS rows per chunk,
// VEC4 = float4 loads of x and w
#include "../../reth_amd/csrc/fc_rows.hpp"

__global__ __launch_bounds__(256) void k_rows_exact(const float *x, int64_t ldx, int64_t r0, int64_t n_max,
                                                    const int64_t *n_dev, const float *w, const float *b, int F, int O,
                                                    float *y, int64_t ldy) {
  rth::linear_relu_rows_wg((int)blockIdx.x, x, ldx, r0, n_max, n_dev, w, b, F, O, y, ldy);
}

template <int COLS, int ROWS, bool VEC4>
__global__ __launch_bounds__(256) void k_rows_var(const float *x, int64_t ldx, int64_t r0, const int64_t *n_dev,
                                                  const float *w, const float *b, int F, int O, float *y) {
  const int64_t n_end = *n_dev;
  __shared__ float red[4][COLS * ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * COLS;
  for (int64_t rb = r0; rb < n_end; rb += ROWS) {
    float acc[COLS][ROWS];
    for (int c = 0; c < COLS; ++c)
      for (int u = 0; u < ROWS; ++u) acc[c][u] = 0.0f;
    if (VEC4) {
      const int F4 = F / 4;
      for (int f4 = tid; f4 < F4; f4 += 256) {
        float4 wv[COLS];
        for (int c = 0; c < COLS; ++c) wv[c] = reinterpret_cast<const float4 *>(w + (int64_t)(j0 + c) * F)[f4];
        for (int u = 0; u < ROWS; ++u) {
          if (rb + u >= n_end) break;
          const float4 xv = reinterpret_cast<const float4 *>(x + (rb + u) * ldx)[f4];
          for (int c = 0; c < COLS; ++c)
            acc[c][u] += xv.x * wv[c].x + xv.y * wv[c].y + xv.z * wv[c].z + xv.w * wv[c].w;
        }
      }
    } else {
      for (int f = tid; f < F; f += 256)
        for (int u = 0; u < ROWS; ++u) {
          if (rb + u >= n_end) break;
          for (int c = 0; c < COLS; ++c) acc[c][u] += x[(rb + u) * ldx + f] * w[(int64_t)(j0 + c) * F + f];
        }
    }
    for (int c = 0; c < COLS; ++c)
      for (int u = 0; u < ROWS; ++u) {
        float v = acc[c][u];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) red[wave][c * ROWS + u] = v;
      }
    __syncthreads();
    if (tid < COLS * ROWS) {
      const int c = tid / ROWS, u = tid % ROWS;
      if (rb + u < n_end && j0 + c < O) {
        float v = b[j0 + c];
        for (int k = 0; k < 4; ++k) v += red[k][tid];
        y[(rb + u) * O + j0 + c] = v > 0.0f ? v : 0.0f;
      }
    }
    __syncthreads();
  }
}

extern "C" int rows_probe_ex(int form, const void *x, int64_t r0, const void *n_dev, const void *w, const void *b, int F,
                             int O, void *y, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float *xf = static_cast<const float *>(x), *wf = static_cast<const float *>(w), *bf = static_cast<const float *>(b);
  const int64_t *nd = static_cast<const int64_t *>(n_dev);
  float *yf = static_cast<float *>(y);
  switch (form) {
    case 3: hipLaunchKernelGGL(k_rows_exact, dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, (int64_t)1 << 40, nd, wf, bf, F, O, yf, (int64_t)O); break;
    case 4: hipLaunchKernelGGL((k_rows_var<4, 8, true>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf); break;
    case 5: hipLaunchKernelGGL((k_rows_var<4, 8, false>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf); break;
    case 6: hipLaunchKernelGGL((k_rows_var<4, 1, true>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf); break;
    case 7: hipLaunchKernelGGL((k_rows_var<1, 8, true>), dim3(O), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf); break;
    case 8: hipLaunchKernelGGL((k_rows_var<1, 1, true>), dim3(O), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// forms 9 / 10: linear_relu_rows_wg with one change each -- 9: the weight loads unconditional
// (no `j0 + c < O ? load : 0`); 10: the row loop without the in-loop break (rows past n_end
// read a clamped row and their sums are discarded)
template <bool WCOND, bool RBREAK>
__global__ __launch_bounds__(256) void k_rows_mod(const float *__restrict__ x, int64_t ldx, int64_t r0,
                                                  const int64_t *__restrict__ n_dev, const float *__restrict__ w,
                                                  const float *__restrict__ b, int F, int O, float *__restrict__ y,
                                                  int64_t ldy) {
  using namespace rth;
  int64_t n_end = *n_dev;
  if (n_end <= r0) return;
  __shared__ float red[kLrThreads / 64][kLrCols * kLrRows];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, F4 = F / 4;
  const int j0 = blockIdx.x * kLrCols;
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
        wv[c] = !WCOND || j0 + c < O ? w4[(int64_t)(j0 + c) * F4 + f4] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
      for (int u = 0; u < kLrRows; ++u) {
        if (RBREAK) {
          if (rb + u >= n_end) break;
        }
        const int64_t row = rb + u < n_end ? rb + u : n_end - 1;
        const float4 xv = reinterpret_cast<const float4 *>(x + row * ldx)[f4];
#pragma unroll
        for (int c = 0; c < kLrCols; ++c)
          acc[c][u] = radd(radd(radd(radd(acc[c][u], rmul(xv.x, wv[c].x)), rmul(xv.y, wv[c].y)), rmul(xv.z, wv[c].z)),
                           rmul(xv.w, wv[c].w));
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

extern "C" int rows_probe_mod(int form, const void *x, int64_t r0, const void *n_dev, const void *w, const void *b, int F,
                              int O, void *y, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const float *xf = static_cast<const float *>(x), *wf = static_cast<const float *>(w), *bf = static_cast<const float *>(b);
  const int64_t *nd = static_cast<const int64_t *>(n_dev);
  float *yf = static_cast<float *>(y);
  if (form == 9) hipLaunchKernelGGL((k_rows_mod<false, true>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf, (int64_t)O);
  else if (form == 10) hipLaunchKernelGGL((k_rows_mod<true, false>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf, (int64_t)O);
  else if (form == 11) hipLaunchKernelGGL((k_rows_mod<false, false>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf, (int64_t)O);
  else if (form == 12) hipLaunchKernelGGL((k_rows_mod<true, true>), dim3(O / 4), dim3(256), 0, s, xf, (int64_t)F, r0, nd, wf, bf, F, O, yf, (int64_t)O);
  else return -2;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
