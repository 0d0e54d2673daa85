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
constexpr int kOptChunk = 4096;  // elements per workgroup (16 per lane)
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

constexpr int kOptV = kOptChunk / kOptThreads / 4;  // float4 groups per lane

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
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kOptThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = radd(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  const float total = (float)sqrt(red[0]);
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
  __shared__ double red[kOptThreads];
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
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kOptThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = radd(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[b] = red[0];
    if (b == 0) {
      const int64_t t = *sa.step + 1;
      *sa.step = t;
      *sa.bc = bias_corr(sa.lr, sa.beta1, sa.beta2, t);
    }
  }
}

__global__ __launch_bounds__(kOptThreads) void k_adam(OptArgs a, const double *__restrict__ part, int nparts,
                                                     ScalarArgs sa, float w1, float beta2, float w2, float eps) {
  __shared__ double red[kOptThreads];
  const int64_t b = blockIdx.x;
  const OptSeg &sg = a.seg[seg_of(a, b)];
  const int64_t base = (b - sg.blk0) * kOptChunk;
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
  float4 gv[kOptV], mv[kOptV], vv[kOptV], pv[kOptV];
  if (sg.vec) {
    const __amdgpu_buffer_rsrc_t rg = seg_rsrc(sg.grad, sg.n), rm = seg_rsrc(sg.m, sg.n), rv = seg_rsrc(sg.v, sg.n),
                                 rp = seg_rsrc(sg.param, sg.n);
#pragma unroll
    for (int k = 0; k < kOptV; ++k) {
      const int64_t e = base + 4 * (k * kOptThreads + threadIdx.x);
      gv[k] = ld4b(rg, e);
      mv[k] = ld4b(rm, e);
      vv[k] = ld4b(rv, e);
      pv[k] = ld4b(rp, e);
    }
    sum_parts();
  } else {
#pragma unroll
    for (int k = 0; k < kOptV; ++k) {
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
  for (int k = 0; k < kOptV; ++k) {
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

// ---------------------------------------------------------------------------------------
// One-launch form (r05): the two launches above read the 6.7 MB of gradients twice (norm
// partials, then Adam) and pay a kernel boundary between them.  Here a grid of at most one
// workgroup per CU (all resident: grid <= CUs, 512 threads, ~100 VGPRs) issues EVERY load of its
// chunks -- gradient, exp_avg, exp_avg_sq, param -- at once, sums its gradient squares, and
// publishes the fp64 partial as two tagged 8-byte granules (cdna_hip_programming.md Guideline
// 16, R2: the data is the flag; {tag = epoch, 32 value bits}, relaxed agent-scope atomic stores
// = write-through).  One wave of every workgroup sweeps all granules until every tag equals
// this call's epoch -- the grid barrier and the norm's data in one -- then every workgroup sums
// the partials in workgroup order (deterministic, the same value everywhere) and updates its
// chunks from the registers the loads landed in.  HBM traffic: the algorithmic 28 B per
// parameter, once.  epoch = a call counter kept in the workspace (read by every workgroup at
// entry, advanced by workgroup 0 after its sweep, when every workgroup has read it), so tags
// left by an earlier call never match; the spin is bounded and a timeout leaves the
// parameters untouched and sets the workspace's error word.
constexpr int kFT = 512;                 // threads per workgroup
constexpr int kFChunk = kFT * 4;         // elements per chunk (one float4 per lane)
constexpr int kFMaxJ = 8;                // chunks per workgroup at most (template J: 2, 4, 8)
constexpr int kFMaxGrid = 256;           // workgroups at most (2 granules each; <= the CUs)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

struct FusedWs {  // after the partials block of the workspace (rth_clip_adam_workspace)
  unsigned int epoch;    // calls completed
  unsigned int timeout;  // nonzero: a call's grid barrier timed out (parameters not updated)
};

struct FusedArgs {
  OptArgs a;
  int64_t nchunks;
  ScalarArgs sa;
  float w1, beta2, w2, eps;
  unsigned long long *gran;  // [2 * grid] tagged granules
  FusedWs *fw;
};

template <int J>
__global__ __launch_bounds__(kFT) void k_clip_adam_fused(FusedArgs fa) {
  __shared__ double red[kFT / 64];
  __shared__ double total_sh;
  __shared__ int ok_sh;
  const OptArgs &a = fa.a;
  gu64 *const gran = (gu64 *)fa.gran;  // agent-scope accesses on global pointers, never flat
  const int G = gridDim.x, wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const unsigned int epoch = *reinterpret_cast<volatile unsigned int *>(&fa.fw->epoch) + 1u;
  const int64_t t = *reinterpret_cast<volatile int64_t *>(fa.sa.step) + 1;  // Adam's step, advanced below
  // t is first used after the grid barrier, but workgroup 0 rewrites *step right after it: the
  // load must have completed before this workgroup publishes (the epoch is in the tags itself)
  asm volatile("" ::"v"((unsigned int)t), "v"((unsigned int)(t >> 32)) : "memory");
  float4 gv[J], mv[J], vv[J], pv[J];
  int segj[J];
  int64_t basej[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int64_t c = blockIdx.x + (int64_t)j * G;
    const int64_t cc = c < fa.nchunks ? c : fa.nchunks - 1;
    const int s = seg_of(a, cc);
    const OptSeg &sg = a.seg[s];
    segj[j] = s;
    // a chunk past the last one reads past its segment's end: the range check returns zeros
    basej[j] = (cc - sg.blk0) * kFChunk + (c < fa.nchunks ? 0 : (int64_t)1 << 40);
    const int64_t e = basej[j] + 4 * threadIdx.x;
    // every segment is 16-byte aligned here (the launcher checks): one unconditional dwordx4
    // per array, the dwords past the segment read zero; the offset fits 32 bits
    const int64_t eb = e < sg.n ? e : sg.n;
    gv[j] = ld4b(seg_rsrc(sg.grad, sg.n), eb);
    mv[j] = ld4b(seg_rsrc(sg.m, sg.n), eb);
    vv[j] = ld4b(seg_rsrc(sg.v, sg.n), eb);
    pv[j] = ld4b(seg_rsrc(sg.param, sg.n), eb);
  }
  // this workgroup's sum of squares (fp64; lane order, then the waves in order)
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const double x = gv[j].x, y = gv[j].y, z = gv[j].z, w = gv[j].w;
    acc = radd(acc, rmul(x, x));
    acc = radd(acc, rmul(y, y));
    acc = radd(acc, rmul(z, z));
    acc = radd(acc, rmul(w, w));
  }
  for (int o = 32; o > 0; o >>= 1) acc = radd(acc, __shfl_down(acc, o, 64));
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double wsum = 0.0;
    for (int w = 0; w < kFT / 64; ++w) wsum = radd(wsum, red[w]);
    const unsigned long long bits = __double_as_longlong(wsum);
    __hip_atomic_store(gran + 2 * blockIdx.x, ((unsigned long long)epoch << 32) | (unsigned int)bits,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gran + 2 * blockIdx.x + 1, ((unsigned long long)epoch << 32) | (unsigned int)(bits >> 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // wave 0 sweeps every granule until all carry this epoch; its values are the partials
  if (wave == 0) {
    constexpr int PER = kFMaxGrid * 2 / 64;  // granules per lane at the largest grid
    unsigned int lo[PER / 2], hi[PER / 2];
    bool ok = false;
    for (unsigned int spins = 0; spins < (1u << 22); ++spins) {
      bool mine = true;
      unsigned long long x0[PER / 2], x1[PER / 2];
#pragma unroll
      for (int k = 0; k < PER / 2; ++k) {  // every load of the pass in flight at once (lanes past
        const int b = lane + 64 * k;       // the grid re-read the last workgroup's granules)
        const int bc = b < G ? b : G - 1;
        x0[k] = __hip_atomic_load(gran + 2 * bc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x1[k] = __hip_atomic_load(gran + 2 * bc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int k = 0; k < PER / 2; ++k) {
        lo[k] = (unsigned int)x0[k];
        hi[k] = (unsigned int)x1[k];
        mine = mine && (lane + 64 * k >= G || ((unsigned int)(x0[k] >> 32) == epoch &&
                                                (unsigned int)(x1[k] >> 32) == epoch));
      }
      if (__all(mine)) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // the partials in workgroup order: lane l holds workgroups l, l + 64, ...; sum k-major per
    // lane, then across lanes in a fixed tree -- the same order in every workgroup
    double part = 0.0;
#pragma unroll
    for (int k = 0; k < PER / 2; ++k) {
      const int b = lane + 64 * k;
      if (b < G) part = radd(part, __longlong_as_double(((long long)hi[k] << 32) | lo[k]));
    }
    for (int o = 32; o > 0; o >>= 1) part = radd(part, __shfl_down(part, o, 64));
    if (lane == 0) {
      total_sh = part;
      ok_sh = ok ? 1 : 0;
      if (!ok) __hip_atomic_store((gu32 *)(&fa.fw->timeout), 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!ok_sh) return;  // the barrier timed out: leave the parameters as they are
  const float total = (float)sqrt(total_sh);
  const int clip = fa.sa.clip;
  float coef = 1.0f;
  if (clip) {
    const float c = fa.sa.max_norm / radd(total, 1e-6f);
    coef = c < 1.0f ? c : 1.0f;
  }
  const double bc1 = 1.0 - pow(fa.sa.beta1, (double)t);
  const double bc2 = 1.0 - pow(fa.sa.beta2, (double)t);
  const float step_size = (float)(fa.sa.lr / bc1), bc2_sqrt = (float)sqrt(bc2);
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // every workgroup has read epoch and step by now
    *fa.sa.step = t;
    fa.fw->epoch = epoch;
    *fa.sa.out = OptScalars{coef, step_size, bc2_sqrt, total};
    if (fa.sa.total_out) *fa.sa.total_out = total;
  }
  const float w1 = fa.w1, beta2 = fa.beta2, w2 = fa.w2, eps = fa.eps;
  auto adam1 = [&](float g, float &m, float &v, float &p) {
    if (clip) g = rmul(g, coef);
    m = radd(m, rmul(w1, rsub(g, m)));
    v = radd(rmul(v, beta2), rmul(rmul(w2, g), g));
    const float denom = radd(sqrtf(v) / bc2_sqrt, eps);
    p = radd(p, rmul(-step_size, m) / denom);
  };
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int64_t c = blockIdx.x + (int64_t)j * G;
    if (c >= fa.nchunks) break;
    const OptSeg &sg = a.seg[segj[j]];
    const int64_t e = basej[j] + 4 * threadIdx.x;
    if (e >= sg.n) continue;
    adam1(gv[j].x, mv[j].x, vv[j].x, pv[j].x);
    adam1(gv[j].y, mv[j].y, vv[j].y, pv[j].y);
    adam1(gv[j].z, mv[j].z, vv[j].z, pv[j].z);
    adam1(gv[j].w, mv[j].w, vv[j].w, pv[j].w);
    st4(sg.param, e, sg.n, sg.vec, pv[j]);
    st4(sg.m, e, sg.n, sg.vec, mv[j]);
    st4(sg.v, e, sg.n, sg.vec, vv[j]);
  }
}

static int cu_count_opt() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n < 1)
      n = 1;
  }
  return n;
}

}  // namespace rth

using namespace rth;

extern "C" {

// [partials: kMaxPartials doubles (the one-launch form: its tagged granules)][OptScalars (the
// last update's scalars, 16 B)][BiasCorr (k_grad_sqsum -> k_adam, 8 B)][FusedWs at +32: call
// counter, timeout word]
int64_t rth_clip_adam_workspace(void) { return (int64_t)kMaxPartials * 8 + 64; }

// the one-launch form's timeout word (nonzero: a grid barrier timed out and that call left
// the parameters as they were); a debug / test read, host-synchronous
int rth_clip_adam_timed_out(const void *workspace_dev) {
  unsigned int w[2] = {0, 0};
  if (!workspace_dev) return -1;
  if (hipMemcpy(w, static_cast<const uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8 + 32, 8,
                hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return w[1] ? 1 : 0;
}

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
  auto *part = static_cast<double *>(workspace_dev);
  auto *sc = reinterpret_cast<OptScalars *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8);
  const int clip = max_norm >= 0.0;
  hipStream_t s = as_stream(stream);
  auto *bcw = reinterpret_cast<BiasCorr *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8 + 16);
  const ScalarArgs sa{clip, (float)max_norm, lr, beta1, beta2, step_dev, sc, total_norm_out, bcw};
  // RTH_ADAM_ONE_PASS=1: one launch when every segment is 16-byte aligned and the chunks fit the
  // resident grid.  Opt-in: alone it is the faster form (16.8 us kernel time for the Q-net), but
  // in the loop its 256 all-resident workgroups wait for CUs the actor stream's convolutions hold
  // and the grid barrier waits for the last of them: 37-40 us per call against 31 for the two
  // launches, and no step-time difference (r05 A/B)
  int64_t nchunks = 0;
  for (int i = 0; i < n_tensors; ++i) nchunks += (tensors[i].n + kFChunk - 1) / kFChunk;
  const int grid = cu_count_opt() < kFMaxGrid ? cu_count_opt() : kFMaxGrid;
  static const bool two_pass = [] {
    const char *e = getenv("RTH_ADAM_ONE_PASS");
    return !(e && atoi(e) != 0);
  }();
  bool aligned = true;
  for (int i = 0; i < n_tensors; ++i) aligned = aligned && a.seg[i].vec;
  if (!two_pass && aligned && nchunks <= (int64_t)grid * kFMaxJ) {
    FusedArgs fa{};
    fa.a = a;
    int64_t b0 = 0;
    for (int i = 0; i < n_tensors; ++i) {  // re-chunked at kFChunk
      fa.a.seg[i].blk0 = b0;
      b0 += (tensors[i].n + kFChunk - 1) / kFChunk;
    }
    fa.nchunks = nchunks;
    fa.sa = sa;
    fa.w1 = (float)(1.0 - beta1);
    fa.beta2 = (float)beta2;
    fa.w2 = (float)(1.0 - beta2);
    fa.eps = (float)eps;
    // workspace: [partials / granules][OptScalars (16 B)][FusedWs (8 B)]
    fa.gran = static_cast<unsigned long long *>(workspace_dev);
    fa.fw = reinterpret_cast<FusedWs *>(static_cast<uint8_t *>(workspace_dev) + (int64_t)kMaxPartials * 8 + 32);
    const int g = nchunks < grid ? (int)nchunks : grid;
    const int64_t per = (nchunks + g - 1) / g;  // chunks per workgroup
    if (per <= 2)
      hipLaunchKernelGGL(k_clip_adam_fused<2>, dim3((unsigned)g), dim3(kFT), 0, s, fa);
    else if (per <= 4)
      hipLaunchKernelGGL(k_clip_adam_fused<4>, dim3((unsigned)g), dim3(kFT), 0, s, fa);
    else
      hipLaunchKernelGGL(k_clip_adam_fused<8>, dim3((unsigned)g), dim3(kFT), 0, s, fa);
    RTH_LAUNCHED();
    return RTH_OK;
  }
  hipLaunchKernelGGL(k_grad_sqsum, dim3((unsigned)blocks), dim3(kOptThreads), 0, s, a, part, sa);
  RTH_LAUNCHED();
  // 1 - beta1 and 1 - beta2 are python floats in adam.py, rounded to f32 once
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(kOptThreads), 0, s, a, part, (int)blocks, sa,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
