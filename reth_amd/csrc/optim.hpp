// Shared by optim.hip (clip + Adam) and conv.hip (the norm partials computed by extra
// workgroups of conv1's weight-gradient reduce launch): the parameter segments, the loads and
// the per-workgroup sum of squares of clip_grad_norm_ (reth/reth/algorithm/dqn/dqn_solver.py:118).
#pragma once

#include "common.hpp"

namespace rth {

constexpr int kOptThreads = 256;
// elements per norm-partial workgroup and per Adam workgroup (8 per lane each; r06: 2,048 for
// both -- 22.3-22.4 vs 23.5 us per clip + Adam live with 4,096 / 2,048, the step equal; 1,024 /
// 1,024 22.6-22.7)
constexpr int kOptChunk = 2048;
constexpr int kAdamChunk = 2048;
#ifndef OPT_PART_LOADS
#define OPT_PART_LOADS 5
#endif
// partials each k_adam lane loads up front (all of them up to 1,280: the one-rank step's ~1,200
// since the weight gradients' reduce workgroups add theirs, r06)
constexpr int kPartLoads = OPT_PART_LOADS;
constexpr int kMaxPartials = 1 << 15;

struct OptSeg {
  float *param;
  const float *grad;
  float *m;
  float *v;
  int64_t n;
  int64_t blk0;  // first workgroup of this tensor
  int vec;       // all four pointers 16-byte aligned: float4 accesses
};

constexpr int kOptV = kOptChunk / kOptThreads / 4;    // float4 groups per lane (k_grad_sqsum)
constexpr int kAdamV = kAdamChunk / kOptThreads / 4;  // float4 groups per lane (k_adam)

// the workgroup's sum of one fp64 value per lane in a fixed order (r06: a wavefront shuffle
// tree, then the 4 waves in order; was an 8-step LDS tree with a barrier per step): every
// lane returns the same sum
__device__ __forceinline__ double block_sum(double v, double *red4) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = radd(v, __shfl_down(v, o, 64));
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = red4[0];
#pragma unroll
  for (int w = 1; w < kOptThreads / 64; ++w) t = radd(t, red4[w]);
  return t;
}

// lane's k-th float4 group of the chunk at element base: elements base + 4 (k T + tid) + 0..3,
// zero past n
__device__ __forceinline__ float4 ld4(const float *__restrict__ p, int64_t e, int64_t n, int vec) {
  if (vec && e + 3 < n) return *reinterpret_cast<const float4 *>(p + e);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n) r.x = p[e];
  if (e + 1 < n) r.y = p[e + 1];
  if (e + 2 < n) r.z = p[e + 2];
  if (e + 3 < n) r.w = p[e + 3];
  return r;
}

// the same load from a buffer resource over [p, p + n): one unconditional dwordx4 whose dwords
// past n read zero (the range check), so no load sits under a branch -- the branchy form made
// the compiler wait for each load before issuing the next.  vec segments only (16-byte aligned).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seg_rsrc(const float *p, int64_t n) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);  // wave-uniform (the workgroup's segment)
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane((int)(n * 4));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}
__device__ __forceinline__ float4 ld4b(__amdgpu_buffer_rsrc_t r, int64_t e) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(e * 4), 0, 0));
}

__device__ __forceinline__ void st4(float *__restrict__ p, int64_t e, int64_t n, int vec, float4 v) {
  if (vec && e + 3 < n) {
    *reinterpret_cast<float4 *>(p + e) = v;
    return;
  }
  if (e < n) p[e] = v.x;
  if (e + 1 < n) p[e + 1] = v.y;
  if (e + 2 < n) p[e + 2] = v.z;
  if (e + 3 < n) p[e + 3] = v.w;
}

struct OptArgs {
  OptSeg seg[RTH_MAX_PARAM_TENSORS];
  int32_t nseg;
};

__device__ __forceinline__ int seg_of(const OptArgs &a, int64_t b) {
  int s = 0;
  while (s + 1 < a.nseg && b >= a.seg[s + 1].blk0) ++s;
  return s;
}

// the bias corrections of step t (python-float scalars of adam.py, cast to f32 where they meet
// the f32 tensors): lr / (1 - beta1^t), sqrt(1 - beta2^t)
struct BiasCorr {
  float step_size, bc2_sqrt;
};
__device__ __forceinline__ BiasCorr bias_corr(double lr, double beta1, double beta2, int64_t t) {
  const double bc1 = 1.0 - pow(beta1, (double)t);
  const double bc2 = 1.0 - pow(beta2, (double)t);
  return BiasCorr{(float)(lr / bc1), (float)sqrt(bc2)};
}


// what a norm-partial workgroup 0 updates: the device step count and the new step's bias corrections
struct SqStep {
  int64_t *step;
  BiasCorr *bc;
  double lr, beta1, beta2;
};

// workgroup b's fp64 sum of squares of its kOptChunk gradient elements (every load of the
// chunk in flight before the first use), in part[b]; workgroup 0 also advances the step count
__device__ __forceinline__ void grad_sqsum_wg(const OptArgs &a, int64_t b, double *__restrict__ part, SqStep st) {
  __shared__ double red[kOptThreads / 64];
  const OptSeg &sg = a.seg[seg_of(a, b)];
  const int64_t base = (b - sg.blk0) * kOptChunk;
  float4 gv[kOptV];
  if (sg.vec) {
    const __amdgpu_buffer_rsrc_t rg = seg_rsrc(sg.grad, sg.n);
#pragma unroll
    for (int k = 0; k < kOptV; ++k) gv[k] = ld4b(rg, base + 4 * (k * kOptThreads + threadIdx.x));
  } else {
#pragma unroll
    for (int k = 0; k < kOptV; ++k) gv[k] = ld4(sg.grad, base + 4 * (k * kOptThreads + threadIdx.x), sg.n, 0);
  }
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < kOptV; ++k) {
    const double x = gv[k].x, y = gv[k].y, z = gv[k].z, w = gv[k].w;
    acc = radd(acc, rmul(x, x));
    acc = radd(acc, rmul(y, y));
    acc = radd(acc, rmul(z, z));
    acc = radd(acc, rmul(w, w));
  }
  const double wsum = block_sum(acc, red);
  if (threadIdx.x == 0) {
    part[b] = wsum;
    if (b == 0) {
      const int64_t t = *st.step + 1;
      *st.step = t;
      *st.bc = bias_corr(st.lr, st.beta1, st.beta2, t);
    }
  }
}

// the segments of `tensors` at `chunk` elements per workgroup: returns the workgroup count
inline int64_t opt_segments(const rth_param_tensor *tensors, int n_tensors, int64_t chunk, OptArgs *a) {
  int64_t blocks = 0;
  for (int s = 0; s < n_tensors; ++s) {
    const rth_param_tensor &t = tensors[s];
    const uintptr_t al = reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                         reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq);
    a->seg[s] = OptSeg{t.param, t.grad, t.exp_avg, t.exp_avg_sq, t.n, blocks, (al & 15) == 0 ? 1 : 0};
    blocks += (t.n + chunk - 1) / chunk;
  }
  a->nseg = n_tensors;
  return blocks;
}

}  // namespace rth
