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
// Q-net parameters), here every workgroup takes 2,048 elements (~830 workgroups).  On one rank
// the partials can come from the learner's backward instead (rth_conv1_relu_wgrad_norm: extra
// workgroups of conv1's weight-gradient reduce launch), leaving the update alone
// (rth_adam_prenormed, r06).
#include "optim.hpp"

namespace rth {

// scalars the combine stage hands to the Adam stage (workspace layout after the partials)
struct OptScalars {
  float coef;         // clip coefficient (1 when not clipping)
  float step_size;    // lr / (1 - beta1^t)
  float bc2_sqrt;     // sqrt(1 - beta2^t)
  float total_norm;   // ||g||_2 before clipping (clip_grad_norm_'s return value)
};

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

// per-workgroup sums of squares of the gradients (fp64 partials, grad_sqsum_wg); workgroup 0
// advances the device step count and writes the new step's bias corrections
__global__ __launch_bounds__(kOptThreads) void k_grad_sqsum(OptArgs a, double *__restrict__ part, ScalarArgs sa) {
  grad_sqsum_wg(a, blockIdx.x, part, SqStep{sa.step, sa.bc, sa.lr, sa.beta1, sa.beta2});
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
  double pacc = 0.0, pl[kPartLoads];
#pragma unroll
  for (int u = 0; u < kPartLoads; ++u) {  // unconditional loads (a clamped index): none waits under a branch
    const int k = threadIdx.x + u * kOptThreads;
    pl[u] = part[k < nparts ? k : nparts - 1];
  }
  const BiasCorr bc = *sa.bc;
  // the partials' in-order sum, in each load path right after its loads are issued (at a merge
  // of the two paths the compiler would wait for every load before it)
  auto sum_parts = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kPartLoads; ++u) asm volatile("" : "+v"(pl[u]));  // keeps the sum behind the loads
#pragma unroll
    for (int u = 0; u < kPartLoads; ++u)
      if (threadIdx.x + u * kOptThreads < nparts) pacc = radd(pacc, pl[u]);
    for (int k = threadIdx.x + kPartLoads * kOptThreads; k < nparts; k += kOptThreads) pacc = radd(pacc, part[k]);
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

static int adam_launch(const rth_param_tensor *tensors, int32_t n_tensors, double lr, double beta1, double beta2,
                       double eps, double max_norm, int64_t *step_dev, void *workspace_dev, float *total_norm_out,
                       int nparts, bool sqsum, hipStream_t s) {
  RTH_REQUIRE(tensors && step_dev && workspace_dev, "rth_clip_adam: NULL argument");
  RTH_REQUIRE(n_tensors >= 1 && n_tensors <= RTH_MAX_PARAM_TENSORS, "rth_clip_adam: %d tensors not in [1, %d]",
              n_tensors, RTH_MAX_PARAM_TENSORS);
  for (int i = 0; i < n_tensors; ++i)
    RTH_REQUIRE(tensors[i].param && tensors[i].grad && tensors[i].exp_avg && tensors[i].exp_avg_sq && tensors[i].n >= 1,
                "rth_clip_adam: tensor %d incomplete", i);
  OptArgs a{}, ad{};
  const int64_t blocks = opt_segments(tensors, n_tensors, kOptChunk, &a);
  const int64_t ablocks = opt_segments(tensors, n_tensors, kAdamChunk, &ad);  // the same segments at k_adam's chunk
  if (sqsum) nparts = (int)(blocks < kMaxPartials ? blocks : kMaxPartials + 1);
  RTH_REQUIRE(nparts >= 1 && nparts <= kMaxPartials, "rth_clip_adam: %d norm partials (at most %d)", nparts,
              kMaxPartials);
  auto *part = static_cast<double *>(workspace_dev);
  auto *sc = reinterpret_cast<OptScalars *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8);
  const int clip = max_norm >= 0.0;
  auto *bcw = reinterpret_cast<BiasCorr *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8 + 16);
  const ScalarArgs sa{clip, (float)max_norm, lr, beta1, beta2, step_dev, sc, total_norm_out, bcw};
  // r05 tried one launch with a grid barrier through tagged granules (every load issued once):
  // faster alone (16.8 us) but 37-40 us per call in the loop, where its all-resident grid waits
  // for CUs the actor stream's convolutions hold -- removed in r06 (profiles/r05)
  if (sqsum) {
    hipLaunchKernelGGL(k_grad_sqsum, dim3((unsigned)blocks), dim3(kOptThreads), 0, s, a, part, sa);
    RTH_LAUNCHED();
  }
  // 1 - beta1 and 1 - beta2 are python floats in adam.py, rounded to f32 once
  hipLaunchKernelGGL(k_adam, dim3((unsigned)ablocks), dim3(kOptThreads), 0, s, ad, part, nparts, sa,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_clip_adam(const rth_param_tensor *tensors, int32_t n_tensors, double lr, double beta1, double beta2,
                  double eps, double max_norm, int64_t *step_dev, void *workspace_dev, float *total_norm_out,
                  void *stream) {
  return adam_launch(tensors, n_tensors, lr, beta1, beta2, eps, max_norm, step_dev, workspace_dev, total_norm_out, 0,
                     true, as_stream(stream));
}

int rth_adam_prenormed(const rth_param_tensor *tensors, int32_t n_tensors, double lr, double beta1, double beta2,
                       double eps, double max_norm, int32_t nparts, int64_t *step_dev, void *workspace_dev,
                       float *total_norm_out, void *stream) {
  return adam_launch(tensors, n_tensors, lr, beta1, beta2, eps, max_norm, step_dev, workspace_dev, total_norm_out,
                     nparts, false, as_stream(stream));
}

}  // extern "C"
