// Learner optimizer step on gfx950: clip_grad_norm_ + Adam as two launches over every
// parameter tensor at once (per-workgroup squared-norm partials; every Adam workgroup sums
// them itself, in the same fixed order, before updating its chunk).
//
// Reference: reth/reth/algorithm/dqn/dqn_solver.py:118-121 -- torch.nn.utils.clip_grad_norm_
// (max_norm = clip_value, 2-norm) then torch.optim.Adam.step() (no weight decay, no amsgrad;
// torch/optim/adam.py single-tensor math):
//   g       = g * min(max_norm / (||g||_2 + 1e-6), 1)
//   m       = lerp(m, g, 1 - beta1)            = m + (1 - beta1) * (g - m)
//   v       = v * beta2 + (1 - beta2) * g * g
//   p       = p - (lr / (1 - beta1^t)) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps)
// The step count t lives on the device (graph replay).  The global norm is a deterministic
// two-stage reduction (per-workgroup fp64 partials, combined in workgroup order); torch's
// fused/foreach kernels chunk 65,536 elements per workgroup (~30 workgroups for the 1.69 M
// Q-net parameters), here every workgroup takes 4,096 elements (~420 workgroups).
#include "common.hpp"

namespace rth {

constexpr int kOptThreads = 256;
constexpr int kOptChunk = 4096;   // elements per k_grad_sqsum workgroup (16 per lane)
constexpr int kAdamChunk = 2048;  // elements per k_adam workgroup (8 per lane): twice the
                                  // workgroups, so one's stores overlap another's loads (r06)
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

// scalars the combine stage hands to the Adam stage (workspace layout after the partials)
struct OptScalars {
  float coef;         // clip coefficient (1 when not clipping)
  float step_size;    // lr / (1 - beta1^t)
  float bc2_sqrt;     // sqrt(1 - beta2^t)
  float total_norm;   // ||g||_2 before clipping (clip_grad_norm_'s return value)
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

// the norm and the clip coefficient from the per-workgroup partials (summed in workgroup
// order: deterministic), `acc` = this lane's in-order sum of partials tid, tid + T, ...  Every
// Adam workgroup computes them itself -- the same values in the same order -- so no workgroup
// waits for another; the step count and the bias corrections were written by k_grad_sqsum's
// first workgroup (a kernel boundary before any read).
__device__ OptScalars opt_scalars(double acc, double *red, int clip, float max_norm, BiasCorr bc) {
  const float total = (float)sqrt(block_sum(acc, red));
  float coef = 1.0f;
  if (clip) {  // clip_coef = max_norm / (total_norm + 1e-6), clamped to 1 (f32 tensor math)
    const float c = max_norm / radd(total, 1e-6f);
    coef = c < 1.0f ? c : 1.0f;
  }
  return OptScalars{coef, bc.step_size, bc.bc2_sqrt, total};
}

struct ScalarArgs {
  int clip;
  float max_norm;
  double lr, beta1, beta2;
  int64_t *step;
  OptScalars *out;
  float *total_out;
  BiasCorr *bc;  // written by k_grad_sqsum's workgroup 0, read by every k_adam workgroup
};

// per-workgroup sums of squares of the gradients (fp64 partials); workgroup 0 advances the
// device step count and writes the new step's bias corrections
__global__ __launch_bounds__(kOptThreads) void k_grad_sqsum(OptArgs a, double *__restrict__ part, ScalarArgs sa) {
  __shared__ double red[kOptThreads / 64];
  const int64_t b = blockIdx.x;
  const OptSeg &sg = a.seg[seg_of(a, b)];
  const int64_t base = (b - sg.blk0) * kOptChunk;
  float4 gv[kOptV];  // every load of the chunk in flight before the first use
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
      const int64_t t = *sa.step + 1;
      *sa.step = t;
      *sa.bc = bias_corr(sa.lr, sa.beta1, sa.beta2, t);
    }
  }
}

__global__ __launch_bounds__(kOptThreads) void k_adam(OptArgs a, const double *__restrict__ part, int nparts,
                                                     ScalarArgs sa, float w1, float beta2, float w2, float eps) {
  __shared__ double red[kOptThreads / 64];
  const int64_t b = blockIdx.x;
  const OptSeg &sg = a.seg[seg_of(a, b)];  // a: the segments at kAdamChunk workgroups
  const int64_t base = (b - sg.blk0) * kAdamChunk;
  // the partials and the bias corrections are loaded first and the chunk's loads issued behind
  // them, so the norm's reduction runs while the chunk is in flight (the load counter is in
  // order: waiting for the partials does not wait for the chunk)
  double pacc = 0.0, pl[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {  // unconditional loads (a clamped index): none waits under a branch
    const int k = threadIdx.x + u * kOptThreads;
    pl[u] = part[k < nparts ? k : nparts - 1];
  }
  const BiasCorr bc = *sa.bc;
  // the partials' in-order sum, in each load path right after its loads are issued (at a merge
  // of the two paths the compiler would wait for every load before it)
  auto sum_parts = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(pl[u]));  // keeps the sum behind the loads
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (threadIdx.x + u * kOptThreads < nparts) pacc = radd(pacc, pl[u]);
    for (int k = threadIdx.x + 4 * kOptThreads; k < nparts; k += kOptThreads) pacc = radd(pacc, part[k]);
  };
  __builtin_amdgcn_sched_barrier(0);
  float4 gv[kAdamV], mv[kAdamV], vv[kAdamV], pv[kAdamV];
  if (sg.vec) {
    const __amdgpu_buffer_rsrc_t rg = seg_rsrc(sg.grad, sg.n), rm = seg_rsrc(sg.m, sg.n), rv = seg_rsrc(sg.v, sg.n),
                                 rp = seg_rsrc(sg.param, sg.n);
#pragma unroll
    for (int k = 0; k < kAdamV; ++k) {
      const int64_t e = base + 4 * (k * kOptThreads + threadIdx.x);
      gv[k] = ld4b(rg, e);
      mv[k] = ld4b(rm, e);
      vv[k] = ld4b(rv, e);
      pv[k] = ld4b(rp, e);
    }
    sum_parts();
  } else {
#pragma unroll
    for (int k = 0; k < kAdamV; ++k) {
      const int64_t e = base + 4 * (k * kOptThreads + threadIdx.x);
      gv[k] = ld4(sg.grad, e, sg.n, 0);
      mv[k] = ld4(sg.m, e, sg.n, 0);
      vv[k] = ld4(sg.v, e, sg.n, 0);
      pv[k] = ld4(sg.param, e, sg.n, 0);
    }
    sum_parts();
  }
  const OptScalars sc = opt_scalars(pacc, red, sa.clip, sa.max_norm, bc);
  if (b == 0 && threadIdx.x == 0) {
    *sa.out = sc;
    if (sa.total_out) *sa.total_out = sc.total_norm;
  }
  const int clip = sa.clip;
  const float coef = sc.coef, step_size = sc.step_size, bc2_sqrt = sc.bc2_sqrt;
  auto adam1 = [&](float g, float &m, float &v, float &p) {
    if (clip) g = rmul(g, coef);  // grad.mul_(clip_coef_clamped)
    m = radd(m, rmul(w1, rsub(g, m)));               // lerp_(g, 1 - beta1), weight < 0.5 branch
    v = radd(rmul(v, beta2), rmul(rmul(w2, g), g));  // mul_(beta2).addcmul_(g, g, 1 - beta2)
    const float denom = radd(sqrtf(v) / bc2_sqrt, eps);
    p = radd(p, rmul(-step_size, m) / denom);  // addcdiv_(m, denom, -step_size)
  };
#pragma unroll
  for (int k = 0; k < kAdamV; ++k) {
    const int64_t e = base + 4 * (k * kOptThreads + threadIdx.x);
    if (e >= sg.n) break;
    adam1(gv[k].x, mv[k].x, vv[k].x, pv[k].x);
    adam1(gv[k].y, mv[k].y, vv[k].y, pv[k].y);
    adam1(gv[k].z, mv[k].z, vv[k].z, pv[k].z);
    adam1(gv[k].w, mv[k].w, vv[k].w, pv[k].w);
    st4(sg.param, e, sg.n, sg.vec, pv[k]);
    st4(sg.m, e, sg.n, sg.vec, mv[k]);
    st4(sg.v, e, sg.n, sg.vec, vv[k]);
  }
}

}  // namespace rth

using namespace rth;

extern "C" {

// [partials: kMaxPartials doubles][OptScalars (the last update's scalars, 16 B)][BiasCorr
// (k_grad_sqsum -> k_adam, 8 B)]
int64_t rth_clip_adam_workspace(void) { return (int64_t)kMaxPartials * 8 + 64; }

int rth_clip_adam(const rth_param_tensor *tensors, int32_t n_tensors, double lr, double beta1, double beta2,
                  double eps, double max_norm, int64_t *step_dev, void *workspace_dev, float *total_norm_out,
                  void *stream) {
  RTH_REQUIRE(tensors && step_dev && workspace_dev, "rth_clip_adam: NULL argument");
  RTH_REQUIRE(n_tensors >= 1 && n_tensors <= RTH_MAX_PARAM_TENSORS, "rth_clip_adam: %d tensors not in [1, %d]",
              n_tensors, RTH_MAX_PARAM_TENSORS);
  OptArgs a{};
  int64_t blocks = 0;
  for (int s = 0; s < n_tensors; ++s) {
    const rth_param_tensor &t = tensors[s];
    RTH_REQUIRE(t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.n >= 1, "rth_clip_adam: tensor %d incomplete", s);
    const uintptr_t al = reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                         reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq);
    a.seg[s] = OptSeg{t.param, t.grad, t.exp_avg, t.exp_avg_sq, t.n, blocks, (al & 15) == 0 ? 1 : 0};
    blocks += (t.n + kOptChunk - 1) / kOptChunk;
  }
  a.nseg = n_tensors;
  RTH_REQUIRE(blocks <= kMaxPartials, "rth_clip_adam: %lld elements exceed the workspace",
              (long long)(blocks * kOptChunk));
  OptArgs ad = a;  // the same segments at k_adam's chunk size
  int64_t ablocks = 0;
  for (int s = 0; s < n_tensors; ++s) {
    ad.seg[s].blk0 = ablocks;
    ablocks += (tensors[s].n + kAdamChunk - 1) / kAdamChunk;
  }
  auto *part = static_cast<double *>(workspace_dev);
  auto *sc = reinterpret_cast<OptScalars *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8);
  const int clip = max_norm >= 0.0;
  hipStream_t s = as_stream(stream);
  auto *bcw = reinterpret_cast<BiasCorr *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8 + 16);
  const ScalarArgs sa{clip, (float)max_norm, lr, beta1, beta2, step_dev, sc, total_norm_out, bcw};
  // r05 tried one launch with a grid barrier through tagged granules (every load issued once):
  // faster alone (16.8 us) but 37-40 us per call in the loop, where its all-resident grid waits
  // for CUs the actor stream's convolutions hold -- removed in r06 (profiles/r05)
  hipLaunchKernelGGL(k_grad_sqsum, dim3((unsigned)blocks), dim3(kOptThreads), 0, s, a, part, sa);
  RTH_LAUNCHED();
  // 1 - beta1 and 1 - beta2 are python floats in adam.py, rounded to f32 once
  hipLaunchKernelGGL(k_adam, dim3((unsigned)ablocks), dim3(kOptThreads), 0, s, ad, part, (int)blocks, sa,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
