// Development aid (r06): a kernel that fills and re-reads a fixed amount of LDS per workgroup and
// counts every read that does not return what its own workgroup wrote.  Run beside other kernels
// (scripts/diag_tail_concurrency.py b=hogKB) to see whether workgroups of different kernels
// sharing a CU ever see each other's LDS.  Build:
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/probes/liblds_hog.so scripts/probes/lds_hog.hip
#include <hip/hip_runtime.h>

template <int U4>
__global__ __launch_bounds__(512) void k_lds_hog(int iters, unsigned seed, unsigned *bad) {
  __shared__ uint4 buf[U4];
  unsigned nbad = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < U4; i += 512)
      buf[i] = make_uint4(seed + i, (unsigned)it, (unsigned)i, blockIdx.x);
    __syncthreads();
    for (int i = threadIdx.x; i < U4; i += 512) {
      const int j = (i * 7 + it) % U4;
      const uint4 v = buf[j];
      nbad += (v.x != seed + j || v.y != (unsigned)it || v.z != (unsigned)j || v.w != blockIdx.x) ? 1u : 0u;
    }
    __syncthreads();
  }
  if (nbad) atomicAdd(bad, nbad);
}

template <int KB>
static int launch(int grid, int iters, unsigned seed, unsigned *bad, hipStream_t s) {
  hipLaunchKernelGGL((k_lds_hog<KB * 64>), dim3(grid), dim3(512), 0, s, iters, seed, bad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int lds_hog(int kb, int grid, int iters, unsigned seed, void *bad, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  unsigned *b = static_cast<unsigned *>(bad);
  switch (kb) {
    case 16: return launch<16>(grid, iters, seed, b, s);
    case 32: return launch<32>(grid, iters, seed, b, s);
    case 64: return launch<64>(grid, iters, seed, b, s);
    case 80: return launch<80>(grid, iters, seed, b, s);
    case 96: return launch<96>(grid, iters, seed, b, s);
    case 128: return launch<128>(grid, iters, seed, b, s);
    case 150: return launch<150>(grid, iters, seed, b, s);
    default: return -2;
  }
}
