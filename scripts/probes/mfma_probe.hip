// Calibration probe (not product code): f32 MFMA issue rate on this box.
//   mode 0: 4 independent 16x16x4 accumulators, operands in registers
//   mode 1: same + one ds_read_b128 per 4 MFMAs (B from LDS, like the conv loop)
//   mode 2: 2 accumulators only
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int MODE>
__global__ __launch_bounds__(512) void k(float *out, int iters) {
  __shared__ f32x4 lds[4096];
  const int lane = threadIdx.x % 64;
  lds[threadIdx.x] = f32x4{1.f, 2.f, 3.f, 4.f};
  __syncthreads();
  f32x4 acc[4] = {};
  float a = threadIdx.x * 1e-3f, b = 0.5f;
  for (int i = 0; i < iters; ++i) {
    f32x4 bv = MODE == 1 ? lds[(i * 64 + lane) & 4095] : f32x4{b, b, b, b};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[t], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[t], acc[1], 0, 0, 0);
      if (MODE != 2) {
        acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[t], acc[2], 0, 0, 0);
        acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[t], acc[3], 0, 0, 0);
      }
    }
  }
  float s = 0;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(int blocks, int threads, int iters) {
  float *out;
  hipMalloc(&out, blocks * threads * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<MODE><<<blocks, threads>>>(out, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<MODE><<<blocks, threads>>>(out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mf = MODE == 2 ? 8.0 : 16.0;
  const double flops = 5.0 * blocks * (threads / 64) * (double)iters * mf * 2048.0;
  printf("mode %d blocks %d threads %d: %.1f us/launch, %.1f TF\n", MODE, blocks, threads, ms * 1000 / 5,
         flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  run<0>(256, 256, 20000);
  run<0>(256, 512, 20000);
  run<1>(256, 256, 20000);
  run<1>(256, 512, 20000);
  run<2>(256, 256, 20000);
  run<2>(256, 512, 20000);
  return 0;
}
