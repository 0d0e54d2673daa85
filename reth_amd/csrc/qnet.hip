// Q-network glue on gfx950: the conv epilogue and its backward as single HBM passes.
//
// Reference: reth/reth/algorithm/dqn/dqn_model.py:14-20 -- every Conv2d is followed by a
// ReLU.  PyTorch-ROCm runs MIOpen's convolution without bias, then a broadcast bias add and
// a separate ReLU (two read+write passes over each activation), and in the backward a
// threshold pass plus a per-channel reduction for the bias gradient.  Here:
//   rth_bias_relu      y = relu(y + b[c]) in place, one pass (same fp32 add as torch's, so
//                      the activations are bit-identical to conv(+bias) -> relu);
//   rth_relu_bias_grad gy = (y > 0) ? g : 0 and db[c] = sum of gy over N*H*W in one pass;
//                      the channel sums are deterministic (fixed per-lane order, fixed LDS
//                      tree, per-block partials combined in block order by a second launch).
// Activations are channels-last (NHWC) contiguous: element e has channel e % C.
#include <cstdint>

#include "common.hpp"
#include "fc_rows.hpp"

namespace rth {

constexpr int kEpiThreads = kBiasThreads;
constexpr int kGradBlocks = kBiasSlabs;  // max partial-sum slabs for the bias gradient

__device__ __forceinline__ float relu_f(float v) { return v < 0.0f ? 0.0f : v; }  // NaN passes, like torch

__global__ __launch_bounds__(kEpiThreads) void k_bias_relu(float4 *__restrict__ y, const float *__restrict__ b,
                                                            int64_t n4, int C) {
  const int64_t stride = (int64_t)gridDim.x * kEpiThreads;
  for (int64_t i = (int64_t)blockIdx.x * kEpiThreads + threadIdx.x; i < n4; i += stride) {
    const int c = (int)((4 * i) % C);
    float4 v = y[i];
    v.x = relu_f(radd(v.x, b[c]));
    v.y = relu_f(radd(v.y, b[c + 1]));
    v.z = relu_f(radd(v.z, b[c + 2]));
    v.w = relu_f(radd(v.w, b[c + 3]));
    y[i] = v;
  }
}

// One lane owns channel quad q = tid % (C/4) and walks rows tid / (C/4), + R, + 2R, ... of
// its block's row slab (R = 256 / (C/4) rows per sweep), so each lane's partial sums have a
// fixed order; lanes with the same quad are then summed by a fixed LDS tree.
__global__ __launch_bounds__(kEpiThreads) void k_relu_bias_grad(const float4 *__restrict__ g,
                                                                 const float4 *__restrict__ y,
                                                                 float4 *__restrict__ gy, float *__restrict__ part,
                                                                 int64_t rows, int C) {
  __shared__ float4 red[kEpiThreads];
  const int tid = threadIdx.x;
  const int Q = C / 4;            // quads per row
  const int R = kEpiThreads / Q;  // rows per sweep
  const int q = tid % Q;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = min<int64_t>(rows, r0 + per);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int U = 8;  // rows per round trip: their loads all in flight, summed in row order
                        // (conv2's 128-row slabs: one round trip; the order does not depend on U)
  for (int64_t r = r0 + tid / Q; r < r1; r += U * R) {
    float4 gv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = r + u * R, i = (rr < r1 ? rr : r) * Q + q;  // past r1: a duplicate, unused
      gv[u] = g[i];
      yv[u] = y[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = r + u * R;
      if (rr >= r1) break;
      float4 o;
      o.x = yv[u].x > 0.0f ? gv[u].x : 0.0f;  // threshold_backward(g, y, 0): y <= 0 -> 0
      o.y = yv[u].y > 0.0f ? gv[u].y : 0.0f;
      o.z = yv[u].z > 0.0f ? gv[u].z : 0.0f;
      o.w = yv[u].w > 0.0f ? gv[u].w : 0.0f;
      gy[rr * Q + q] = o;
      acc.x = radd(acc.x, o.x);
      acc.y = radd(acc.y, o.y);
      acc.z = radd(acc.z, o.z);
      acc.w = radd(acc.w, o.w);
    }
  }
  red[tid] = acc;
  __syncthreads();
  for (int s = kEpiThreads / 2; s >= Q; s >>= 1) {  // lanes tid and tid+s share a quad
    if (tid < s) {
      float4 a = red[tid];
      const float4 o = red[tid + s];
      a.x = radd(a.x, o.x);
      a.y = radd(a.y, o.y);
      a.z = radd(a.z, o.z);
      a.w = radd(a.w, o.w);
      red[tid] = a;
    }
    __syncthreads();
  }
  if (tid < Q) reinterpret_cast<float4 *>(part)[(int64_t)blockIdx.x * Q + tid] = red[tid];
}

// The same for the last conv's NCHW output (the FC1 input in the reference's (C, H, W)
// flatten order): g and y are [n, C, P] (P = H*W), gy is written channels-last [n, P, C] for
// the data / weight gradients that follow.  Slab s owns samples [s*n/S, (s+1)*n/S); per
// sample the masked gradient goes through an LDS tile [C][P+1] so the NCHW reads and the
// NHWC writes are both coalesced.  Lane t sums channel t / Q over positions of quarter t % Q
// (Q = 256 / C) across its slab's samples, then the Q quarter sums in fixed order: the same
// slab-partial layout as k_relu_bias_grad, so the combine (or a deferred job) is shared.
constexpr int kNchwMaxTile = 64 * 50;
__global__ __launch_bounds__(kEpiThreads) void k_relu_bias_grad_nchw(const float *__restrict__ g,
                                                                      const float *__restrict__ y,
                                                                      float *__restrict__ gy, float *__restrict__ part,
                                                                      int64_t n, int C, int P) {
  __shared__ float tile[kNchwMaxTile];
  __shared__ float red[kEpiThreads];
  const int tid = threadIdx.x, S = gridDim.x, E = C * P, LP = P + 1;
  const int64_t b0 = (int64_t)blockIdx.x * n / S, b1 = (int64_t)(blockIdx.x + 1) * n / S;
  const int Q = kEpiThreads / C, c_own = tid / Q, qq = tid % Q;
  const int pq = (P + Q - 1) / Q, p0 = qq * pq, p1 = min(P, p0 + pq);
  float acc = 0.0f;
  constexpr int U = (kNchwMaxTile + kEpiThreads - 1) / kEpiThreads;
  float yv[U], gv[U];  // a sample's loads all in flight (a load-then-use loop waited for each)
  auto fetch = [&](int64_t b) {
    const float *gb = g + b * E, *yb = y + b * E;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kEpiThreads, ic = i < E ? i : E - 1;  // past E: a duplicate, unused
      yv[u] = yb[ic];
      gv[u] = gb[ic];
    }
  };
  if (b0 < b1) fetch(b0);
  for (int64_t b = b0; b < b1; ++b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {  // NCHW order: i = c * P + p
      const int i = tid + u * kEpiThreads;
      if (i < E) {
        const int c = i / P, pp = i - c * P;
        tile[c * LP + pp] = yv[u] > 0.0f ? gv[u] : 0.0f;  // threshold_backward(g, y, 0)
      }
    }
    // the next sample's loads go out now and land while this one is summed and stored (the last
    // sample re-reads itself: no load under a branch)
    fetch(b + 1 < b1 ? b + 1 : b);
    __syncthreads();
    for (int p = p0; p < p1; ++p) acc = radd(acc, tile[c_own * LP + p]);
    float *gyb = gy + b * E;
    for (int o = tid; o < E; o += kEpiThreads) {  // NHWC order: o = p * C + c
      const int pp = o / C, c = o - pp * C;
      gyb[o] = tile[c * LP + pp];
    }
    __syncthreads();
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < C) {
    float sum = red[tid * Q];
    for (int k = 1; k < Q; ++k) sum = radd(sum, red[tid * Q + k]);
    part[(int64_t)blockIdx.x * C + tid] = sum;
  }
}

// db[c] = sum of the slabs' partials in slab order: lane t sums slabs t / C, t / C + G, ...
// of channel t % C (G = 1024 / C lanes per channel, 8 loads in flight), then the G lane sums
// of a channel by a fixed LDS tree.  A separate launch: the kernel boundary publishes the
// partials (a per-block agent-scope fence would write back the XCD's whole L2 each time).
constexpr int kCombThreads = 1024;
__global__ __launch_bounds__(kCombThreads) void k_bias_grad_combine(const float *__restrict__ part, int nslabs, int C,
                                                                     float *__restrict__ db) {
  __shared__ float red[kCombThreads];
  const int tid = threadIdx.x;
  const int G = kCombThreads / C;
  const int c = tid % C;
  float s = 0.0f;
  for (int k = tid / C; k < nslabs; k += 8 * G) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kk = k + u * G;
      v[u] = kk < nslabs ? part[(int64_t)kk * C + c] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s = radd(s, v[u]);
  }
  red[tid] = s;
  __syncthreads();
  for (int st = kCombThreads / 2; st >= C; st >>= 1) {
    if (tid < st) red[tid] = radd(red[tid], red[tid + st]);
    __syncthreads();
  }
  if (tid < C) db[tid] = red[tid];
}


// ---------------------------------------------------------------- merged dueling heads
// model.py's merged-heads forward runs the two dueling branches as one FC1 GEMM (rows: the
// advantage then the value branch; columns in the NHWC flatten order of the conv features
// when hwc != 0) and one block-diagonal FC2 GEMM.  One launch builds the merged operands
// from the reference's eight parameters, one launch splits their gradients back.
struct HeadsDims {
  int64_t H, F, A;  // hidden units per branch, features, actions
  int32_t C, P;     // feature map channels and H*W positions (C = 0: no permutation)
  int32_t fc2_only;  // only the second layer (w2, b2): FC1 is held merged by the model
};


constexpr int kRowF4 = 12;  // float4 per thread for one FC1 row in LDS: F <= 12288

// One workgroup per FC1 row (2H rows) + one for the small tail (b1, w2, b2).  A row of the
// NHWC-permuted FC1 weight is a C x P -> P x C transpose of the reference row, done through
// LDS so both the HBM reads and the writes are coalesced.
__global__ __launch_bounds__(256) void k_heads_merge(HeadsDims d, const float *__restrict__ wa1,
                                                     const float *__restrict__ wv1, const float *__restrict__ ba1,
                                                     const float *__restrict__ bv1, const float *__restrict__ wa2,
                                                     const float *__restrict__ wv2, const float *__restrict__ ba2,
                                                     const float *__restrict__ bv2, float *__restrict__ w1,
                                                     float *__restrict__ b1, float *__restrict__ w2,
                                                     float *__restrict__ b2) {
  extern __shared__ float row[];
  const int64_t r = blockIdx.x + (d.fc2_only ? 2 * d.H : 0), F = d.F;
  if (r < 2 * d.H) {
    const float *src = (r < d.H ? wa1 : wv1) + (r % d.H) * F;
    float *dst = w1 + r * F;
    if (d.C == 0) {
      for (int64_t i = threadIdx.x; i < F; i += blockDim.x) dst[i] = src[i];
      return;
    }
    // reference order c * P + p; float4 loads, all issued before the first LDS write
    // (selects, not conditional loads: the array stays in registers)
    {
      const int F4 = (int)(F / 4);
      const float4 *s4 = reinterpret_cast<const float4 *>(src);
      float4 v[kRowF4];
#pragma unroll
      for (int u = 0; u < kRowF4; ++u) {
        const int i = threadIdx.x + u * 256;
        v[u] = s4[i < F4 ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < kRowF4; ++u) {
        const int i = threadIdx.x + u * 256;
        if (i < F4) reinterpret_cast<float4 *>(row)[i] = v[u];
      }
    }
    __syncthreads();
    for (int j4 = threadIdx.x; j4 < F / 4; j4 += 256) {  // merged order p * C + c, 4 c per thread
      const int j = 4 * j4, p = j / d.C, c = j - p * d.C;
      reinterpret_cast<float4 *>(dst)[j4] =
          float4{row[c * d.P + p], row[(c + 1) * d.P + p], row[(c + 2) * d.P + p], row[(c + 3) * d.P + p]};
    }
    return;
  }
  const int64_t H2 = 2 * d.H, A1 = d.A + 1;
  if (!d.fc2_only)
    for (int64_t k = threadIdx.x; k < H2; k += blockDim.x) b1[k] = k < d.H ? ba1[k] : bv1[k - d.H];
  for (int64_t k = threadIdx.x; k < A1 * H2; k += blockDim.x) {
    const int64_t rr = k / H2, j = k - rr * H2;
    float v = 0.0f;
    if (rr < d.A && j < d.H) v = wa2[rr * d.H + j];
    if (rr == d.A && j >= d.H) v = wv2[j - d.H];
    w2[k] = v;
  }
  for (int64_t k = threadIdx.x; k < A1; k += blockDim.x) b2[k] = k < d.A ? ba2[k] : bv2[0];
}

__global__ __launch_bounds__(256) void k_heads_split_grad(HeadsDims d, const float *__restrict__ gw1,
                                                          const float *__restrict__ gb1,
                                                          const float *__restrict__ gw2,
                                                          const float *__restrict__ gb2, float *__restrict__ gwa1,
                                                          float *__restrict__ gwv1, float *__restrict__ gba1,
                                                          float *__restrict__ gbv1, float *__restrict__ gwa2,
                                                          float *__restrict__ gwv2, float *__restrict__ gba2,
                                                          float *__restrict__ gbv2) {
  extern __shared__ float row[];
  const int64_t r = blockIdx.x + (d.fc2_only ? 2 * d.H : 0), F = d.F;
  if (r < 2 * d.H) {
    const float *src = gw1 + r * F;
    float *dst = (r < d.H ? gwa1 : gwv1) + (r % d.H) * F;
    if (d.C == 0) {
      for (int64_t i = threadIdx.x; i < F; i += blockDim.x) dst[i] = src[i];
      return;
    }
    // merged order j = p * C + c, kept at p * (C + 1) + c (padded: conflict-free reads below);
    // float4 loads, all issued before the first LDS write
    {
      const int F4 = (int)(F / 4);
      const float4 *s4 = reinterpret_cast<const float4 *>(src);
      float4 v[kRowF4];
#pragma unroll
      for (int u = 0; u < kRowF4; ++u) {
        const int i = threadIdx.x + u * 256;
        if (i < F4) v[u] = s4[i];
      }
#pragma unroll
      for (int u = 0; u < kRowF4; ++u) {
        const int i = threadIdx.x + u * 256;
        if (i < F4) {
          const int j = 4 * i, p = j / d.C, c = j - p * d.C;  // C % 4 == 0: same p for all 4
          float *o = row + p * (d.C + 1) + c;
          o[0] = v[u].x, o[1] = v[u].y, o[2] = v[u].z, o[3] = v[u].w;
        }
      }
    }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < F; i += 256) {  // reference order c * P + p
      const int c = (int)(i / d.P), p = (int)(i - (int64_t)c * d.P);
      dst[i] = row[p * (d.C + 1) + c];
    }
    return;
  }
  const int64_t H2 = 2 * d.H;
  if (!d.fc2_only)
    for (int64_t k = threadIdx.x; k < H2; k += blockDim.x) {
      if (k < d.H) gba1[k] = gb1[k]; else gbv1[k - d.H] = gb1[k];
    }
  for (int64_t k = threadIdx.x; k < d.A * d.H + d.H; k += blockDim.x) {
    if (k < d.A * d.H) {
      const int64_t rr = k / d.H, j = k - rr * d.H;
      gwa2[k] = gw2[rr * H2 + j];
    } else {
      gwv2[k - d.A * d.H] = gw2[d.A * H2 + d.H + (k - d.A * d.H)];
    }
  }
  for (int64_t k = threadIdx.x; k <= d.A; k += blockDim.x) {
    if (k < d.A) gba2[k] = gb2[k]; else gbv2[0] = gb2[k];
  }
}


// ---------------------------------------------------------------- heads backward
// The merged heads' second layer backward (heads = h @ w2^T + b2, h = relu(FC1)) in one
// launch, from the TD kernel's d(loss)/d(heads):
//   gh  = (h > 0) ? dq @ w2 : 0      (addmm backward -> threshold_backward, [B, H2])
//   gw2 = dq^T @ h  [A1, H2],  gb2 = column sums of dq [A1],  gb1 = column sums of gh [H2]
// Workgroup k < H2 / 16 owns columns 16k .. 16k+15 over all B rows: lane = column tid % 16,
// row group tid / 16 (64 groups), RB rows of h and dq loaded per batch before any use (the
// loop is load-latency bound otherwise); the 64 row-group partials are summed in LDS in a
// fixed order (deterministic).  The last workgroup sums gb2 and, optionally, adds
// mean(|td|) to a device accumulator (Trainer's mean_error, reth/reth/presets/trainer.py:64-69).
constexpr int kHbCols = 16, kHbGroups = 64, kHbThreads = kHbCols * kHbGroups, kHbMaxA1 = kMaxActions + 1;

// The second layer's weights and gradients: merged (w2 [A1, H2] block diagonal, gw2, gb2) or,
// with `branches`, the reference's four parameters read and written in place (wa2 [A, H],
// wv2 [1, H]; gwa2, gwv2, gba2, gbv2) -- no merged copy to build or split per update.  In
// branch form the off-diagonal blocks are zero and their gradients are not produced.
struct Fc2 {
  const float *w2;
  float *gw2, *gb2;
  const float *wa2, *wv2;
  float *gwa2, *gwv2, *gba2, *gbv2;
  int H, A, branches;
};

__device__ __forceinline__ float fc2_w(const Fc2 &f, int a, int j, int H2) {
  if (!f.branches) return f.w2[(int64_t)a * H2 + j];
  if (a < f.A) return j < f.H ? f.wa2[(int64_t)a * f.H + j] : 0.0f;
  return j >= f.H ? f.wv2[j - f.H] : 0.0f;
}

// is gw2[a][j] wanted (branch form: the diagonal blocks only); uniform over a workgroup's
// 16 columns when H % 16 == 0
__device__ __forceinline__ bool fc2_live(const Fc2 &f, int a, int j) {
  return !f.branches || (a < f.A) == (j < f.H);
}

__device__ __forceinline__ void fc2_store_gw(const Fc2 &f, int a, int j, int H2, float v) {
  if (!f.branches) f.gw2[(int64_t)a * H2 + j] = v;
  else if (a < f.A) f.gwa2[(int64_t)a * f.H + j] = v;
  else f.gwv2[j - f.H] = v;
}

__device__ __forceinline__ void fc2_store_gb(const Fc2 &f, int a, float v) {
  if (!f.branches) f.gb2[a] = v;
  else if (a < f.A) f.gba2[a] = v;
  else f.gbv2[0] = v;
}

// NQ sums through the LDS tree at once (one barrier per tree level for all of them): per
// quantity the same additions in the same order as the one-at-a-time loop, so bit-identical;
// the tree stops at `stop` lanes (16 columns, or 1); red holds NQ x kHbThreads floats
template <int NQ>
__device__ __forceinline__ void tree_sums(float *red, const float (&v)[NQ], int tid, int stop) {
#pragma unroll
  for (int q = 0; q < NQ; ++q) red[q * kHbThreads + tid] = v[q];
  __syncthreads();
  for (int st = kHbThreads / 2; st >= stop; st >>= 1) {
    if (tid < st) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) red[q * kHbThreads + tid] = radd(red[q * kHbThreads + tid], red[q * kHbThreads + tid + st]);
    }
    __syncthreads();
  }
}
// batched trees for the small-action variants (MAXA <= 8: 9 / 10 quantities, 36 / 40 KB of LDS)
template <int MAXA, bool BATCH>
constexpr int kHbRedQ = BATCH && MAXA <= 8 ? MAXA + 2 : 1;

template <int MAXA, int RB, bool BATCH = true>
__global__ __launch_bounds__(kHbThreads) void k_heads_backward(const float *__restrict__ dq,
                                                               const float *__restrict__ h, int64_t ldh, Fc2 f,
                                                               int64_t B, int H2, int A1, float *__restrict__ gh,
                                                               float *__restrict__ gb1,
                                                               const float *__restrict__ td_abs,
                                                               float *__restrict__ td_acc) {
  __shared__ float red[kHbThreads * kHbRedQ<MAXA, BATCH>];
  const int tid = threadIdx.x;
  if ((int)blockIdx.x == H2 / kHbCols) {  // gb2 and the |td| mean
    if constexpr (BATCH && MAXA <= 8) {
      float v[MAXA + 1];
#pragma unroll
      for (int a = 0; a <= MAXA; ++a) {
        float s = 0.0f;
        if (a < A1 || (a == A1 && td_abs && td_acc))
          for (int64_t r = tid; r < B; r += kHbThreads) s = radd(s, a < A1 ? dq[r * A1 + a] : td_abs[r]);
        v[a] = s;
      }
      tree_sums<MAXA + 1>(red, v, tid, 1);
      if (tid == 0) {
        for (int a = 0; a < A1; ++a) fc2_store_gb(f, a, red[a * kHbThreads]);
        if (td_abs && td_acc) td_acc[0] = radd(td_acc[0], red[A1 * kHbThreads] / (float)B);
      }
      return;
    }
    for (int a = 0; a <= A1; ++a) {
      if (a == A1 && !(td_abs && td_acc)) break;
      float s = 0.0f;
      for (int64_t r = tid; r < B; r += kHbThreads) s = radd(s, a < A1 ? dq[r * A1 + a] : td_abs[r]);
      red[tid] = s;
      __syncthreads();
      for (int st = kHbThreads / 2; st > 0; st >>= 1) {
        if (tid < st) red[tid] = radd(red[tid], red[tid + st]);
        __syncthreads();
      }
      if (tid == 0) {
        if (a < A1) fc2_store_gb(f, a, red[0]);
        else td_acc[0] = radd(td_acc[0], red[0] / (float)B);  // _err_acc.add_(td.mean())
      }
      __syncthreads();
    }
    return;
  }
  const int c = tid % kHbCols, rg = tid / kHbCols;
  const int j = (int)blockIdx.x * kHbCols + c;
  float wc[MAXA], aw[MAXA];
#pragma unroll
  for (int a = 0; a < MAXA; ++a) {
    wc[a] = a < A1 ? fc2_w(f, a, j, H2) : 0.0f;
    aw[a] = 0.0f;
  }
  float ab = 0.0f;
  for (int64_t r0 = rg; r0 < B; r0 += (int64_t)RB * kHbGroups) {
    float hv[RB], dv[RB][MAXA];
#pragma unroll
    for (int u = 0; u < RB; ++u) {  // all loads of the batch first
      const int64_t r = r0 + (int64_t)u * kHbGroups;
      const int64_t rl = r < B ? r : B - 1;  // unconditional loads (a duplicate row, unused): a load
      hv[u] = h[rl * ldh + j];               // under a branch is waited for before the next one
#pragma unroll
      for (int a = 0; a < MAXA; ++a) dv[u][a] = dq[rl * A1 + (a < A1 ? a : 0)];
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t r = r0 + (int64_t)u * kHbGroups;
      if (r >= B) break;
      float g = 0.0f;
#pragma unroll
      for (int a = 0; a < MAXA; ++a)
        if (a < A1) {
          g = radd(g, rmul(dv[u][a], wc[a]));
          aw[a] = radd(aw[a], rmul(dv[u][a], hv[u]));
        }
      g = hv[u] > 0.0f ? g : 0.0f;  // threshold_backward(g, h, 0)
      gh[r * H2 + j] = g;
      ab = radd(ab, g);
    }
  }
  // fixed-order sums over the row groups: gb1, then each (wanted) row of gw2
  if constexpr (BATCH && MAXA <= 8) {
    float v[MAXA + 1];
    v[0] = ab;
#pragma unroll
    for (int a = 0; a < MAXA; ++a) v[1 + a] = aw[a];
    tree_sums<MAXA + 1>(red, v, tid, kHbCols);
    if (tid < kHbCols) {
      gb1[j] = red[tid];
      for (int a = 0; a < A1; ++a)
        if (fc2_live(f, a, (int)blockIdx.x * kHbCols)) fc2_store_gw(f, a, j, H2, red[(1 + a) * kHbThreads + tid]);
    }
    return;
  }
  for (int a = -1; a < A1; ++a) {
    if (a >= 0 && !fc2_live(f, a, (int)blockIdx.x * kHbCols)) continue;  // uniform
    float v = ab;
#pragma unroll
    for (int k = 0; k < MAXA; ++k)
      if (k == a) v = aw[k];
    red[tid] = v;
    __syncthreads();
    for (int st = kHbThreads / 2; st >= kHbCols; st >>= 1) {  // lanes tid, tid + st: same column
      if (tid < st) red[tid] = radd(red[tid], red[tid + st]);
      __syncthreads();
    }
    if (tid < kHbCols) {
      if (a < 0) gb1[j] = red[tid];
      else fc2_store_gw(f, a, j, H2, red[tid]);
    }
    __syncthreads();
  }
}


// rth_td_huber + k_heads_backward in one launch: every workgroup recomputes the batch's TD rows
// (td_huber_row, the same arithmetic as k_td_huber) into LDS -- d(loss)/d(heads) of all B
// rows, <= kTdHbMaxElems values -- instead of reading them back from a separate launch; the
// last workgroup also writes |td|, the loss (a fixed-order tree) and the |td| mean.
constexpr int kTdHbMaxElems = 16384;

template <int MAXA, int RB, bool BATCH = true>
__global__ __launch_bounds__(kHbThreads) void k_td_heads_backward(
    const float *__restrict__ q0, const float *__restrict__ q1o, const float *__restrict__ q1t,
    const int64_t *__restrict__ act, const float *__restrict__ rew, const float *__restrict__ done,
    const double *__restrict__ isw, int64_t B, int A, float gamma_n, int double_q, const float *__restrict__ h,
    int64_t ldh, Fc2 f, int H2, float *__restrict__ td_abs, float *__restrict__ loss_out,
    float *__restrict__ gh, float *__restrict__ gb1, float *__restrict__ td_acc) {
  extern __shared__ float dqs[];  // B * (A + 1) floats (dynamic: a 16 K-float static array kept
                                  // the kernel off every CU a conv kernel shares)
  __shared__ float red[kHbThreads * kHbRedQ<MAXA, BATCH>];
  const int tid = threadIdx.x, A1 = A + 1;
  const bool tail = (int)blockIdx.x == H2 / kHbCols;  // gb2, |td|, loss, |td| mean
  const float invB = 1.0f / (float)B;
  float lacc = 0.0f, tacc = 0.0f;
  for (int64_t b = tid; b < B; b += kHbThreads) {
    float l;
    const float td = td_huber_row(q0, q1o, q1t, act, rew, done, isw, b, A, 1, gamma_n, double_q, invB, &l,
                                  dqs + b * A1);
    if (tail) {
      td_abs[b] = fabsf(td);
      lacc = radd(lacc, l);
      tacc = radd(tacc, fabsf(td));
    }
  }
  __syncthreads();
  if (tail && BATCH && MAXA <= 8) {  // loss, |td| mean, then gb2: one batched tree
    float v[MAXA + 2];
    v[0] = lacc;
    v[1] = tacc;
#pragma unroll
    for (int a = 0; a < MAXA; ++a) {
      float s = 0.0f;
      if (a < A1)
        for (int64_t r = tid; r < B; r += kHbThreads) s = radd(s, dqs[r * A1 + a]);
      v[2 + a] = s;
    }
    tree_sums<MAXA + 2>(red, v, tid, 1);
    if (tid == 0) {
      loss_out[0] = red[0] * invB;
      if (td_acc) td_acc[0] = radd(td_acc[0], red[kHbThreads] / (float)B);
      for (int a = 0; a < A1; ++a) fc2_store_gb(f, a, red[(2 + a) * kHbThreads]);
    }
    return;
  }
  if (tail) {
    for (int a = -2; a < A1; ++a) {  // loss, |td| mean, then gb2
      float v = a == -2 ? lacc : (a == -1 ? tacc : 0.0f);
      if (a >= 0)
        for (int64_t r = tid; r < B; r += kHbThreads) v = radd(v, dqs[r * A1 + a]);
      red[tid] = v;
      __syncthreads();
      for (int st = kHbThreads / 2; st > 0; st >>= 1) {
        if (tid < st) red[tid] = radd(red[tid], red[tid + st]);
        __syncthreads();
      }
      if (tid == 0) {
        if (a == -2) loss_out[0] = red[0] * invB;
        else if (a == -1) { if (td_acc) td_acc[0] = radd(td_acc[0], red[0] / (float)B); }
        else fc2_store_gb(f, a, red[0]);
      }
      __syncthreads();
    }
    return;
  }
  const int c = tid % kHbCols, rg = tid / kHbCols;
  const int j = (int)blockIdx.x * kHbCols + c;
  float wc[MAXA], aw[MAXA];
#pragma unroll
  for (int a = 0; a < MAXA; ++a) {
    wc[a] = a < A1 ? fc2_w(f, a, j, H2) : 0.0f;
    aw[a] = 0.0f;
  }
  float ab = 0.0f;
  for (int64_t r0 = rg; r0 < B; r0 += (int64_t)RB * kHbGroups) {
    float hv[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t r = r0 + (int64_t)u * kHbGroups;
      hv[u] = h[(r < B ? r : B - 1) * ldh + j];  // unconditional (a duplicate row, unused)
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t r = r0 + (int64_t)u * kHbGroups;
      if (r >= B) break;
      const float *d = dqs + r * A1;
      float g = 0.0f;
#pragma unroll
      for (int a = 0; a < MAXA; ++a)
        if (a < A1) {
          const float da = d[a];
          g = radd(g, rmul(da, wc[a]));
          aw[a] = radd(aw[a], rmul(da, hv[u]));
        }
      g = hv[u] > 0.0f ? g : 0.0f;  // threshold_backward(g, h, 0)
      gh[r * H2 + j] = g;
      ab = radd(ab, g);
    }
  }
  if constexpr (BATCH && MAXA <= 8) {  // gb1, then each (wanted) row of gw2: one batched tree
    float v[MAXA + 1];
    v[0] = ab;
#pragma unroll
    for (int a = 0; a < MAXA; ++a) v[1 + a] = aw[a];
    tree_sums<MAXA + 1>(red, v, tid, kHbCols);
    if (tid < kHbCols) {
      gb1[j] = red[tid];
      for (int a = 0; a < A1; ++a)
        if (fc2_live(f, a, (int)blockIdx.x * kHbCols)) fc2_store_gw(f, a, j, H2, red[(1 + a) * kHbThreads + tid]);
    }
    return;
  }
  for (int a = -1; a < A1; ++a) {
    if (a >= 0 && !fc2_live(f, a, (int)blockIdx.x * kHbCols)) continue;  // uniform
    float v = ab;
#pragma unroll
    for (int k = 0; k < MAXA; ++k)
      if (k == a) v = aw[k];
    red[tid] = v;
    __syncthreads();
    for (int st = kHbThreads / 2; st >= kHbCols; st >>= 1) {
      if (tid < st) red[tid] = radd(red[tid], red[tid + st]);
      __syncthreads();
    }
    if (tid < kHbCols) {
      if (a < 0) gb1[j] = red[tid];
      else fc2_store_gw(f, a, j, H2, red[tid]);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- heads forward, second layer
// heads[r] = (wa2 . h[r, :H] + ba2, wv2 . h[r, H:] + bv2) straight from the reference's four
// parameters (the block-diagonal FC2 without a merged copy).  16 lanes per row (16 rows per
// workgroup): lane l takes columns [l H/16, (l+1) H/16) of each half, all of its h loads
// issued at once, the weights staged in LDS once per workgroup; the A+1 partial dots are
// summed across the 16 lanes by four xor shuffles in a fixed order.  [n, A+1], row stride A+1.
// The staged weights take (A+1) * H * 4 bytes of dynamic LDS: <= 16 KB for Atari's minimal
// action sets (A + 1 <= 8, the k_heads_fc2<8> build), <= 66 KB for the full 18-action set and
// anything up to kMaxActions (k_heads_fc2<kHbMaxA1>).
constexpr int kFc2MaxH = 512;
template <int MAXA1>
__global__ __launch_bounds__(256) void k_heads_fc2(const float *__restrict__ h, int64_t ldh, int64_t n, int H, int A,
                                                   const float *__restrict__ wa2, const float *__restrict__ wv2,
                                                   const float *__restrict__ ba2, const float *__restrict__ bv2,
                                                   float *__restrict__ heads, const int64_t *__restrict__ n_dev,
                                                   float *__restrict__ cache, const int64_t *__restrict__ cache_rows) {
  constexpr int U = kFc2MaxH / 16 / 4;  // float4 per lane and half, at most
  extern __shared__ float4 wl[];         // rows a < A: wa2[a], row A: wv2
  if (n_dev) {                           // device-counted batch: rows >= *n_dev are not computed
    const int64_t nd = *n_dev;
    n = nd < n ? nd : n;
    if ((int64_t)blockIdx.x * 16 >= n) return;  // uniform
  }
  const int l = threadIdx.x & 15;
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t rr = r < n ? r : n - 1;  // tail rows: a duplicate, nothing written
  const int cq = H / 64;                  // float4 per lane and half
  const float4 *ha = reinterpret_cast<const float4 *>(h + rr * ldh) + l * cq;
  const float4 *hv = reinterpret_cast<const float4 *>(h + rr * ldh + H) + l * cq;
  float4 xa[U], xv[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {  // unconditional loads (k >= cq: a duplicate, unused): a load under
    const int kk = k < cq ? k : 0;  // a branch makes the compiler wait for it before the next one
    xa[k] = ha[kk], xv[k] = hv[kk];
  }
  const int A1 = A + 1, H4 = H / 4;
  {  // stage the weights: every load issued before the first LDS write (a load-then-write loop
     // waits for each load in turn)
    constexpr int WPER = (MAXA1 * kFc2MaxH / 4 + 255) / 256;
    const int nw = A1 * H4;
    float4 tw[WPER];
#pragma unroll
    for (int u = 0; u < WPER; ++u) {
      int i = threadIdx.x + u * 256;
      i = i < nw ? i : nw - 1;  // a duplicate, not written
      const int a = i / H4, j4 = i - a * H4;
      tw[u] = reinterpret_cast<const float4 *>(a < A ? wa2 + (int64_t)a * H : wv2)[j4];
    }
#pragma unroll
    for (int u = 0; u < WPER; ++u) {  // out-of-range slots land on the spare slot nw
      const int i = threadIdx.x + u * 256;
      wl[i < nw ? i : nw] = tw[u];
    }
  }
  __syncthreads();
  float acc[MAXA1];
#pragma unroll
  for (int a = 0; a < MAXA1; ++a) {
    acc[a] = 0.0f;
    if (a < A1) {
      const float4 *w = wl + a * H4 + l * cq;
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (k < cq) {
          const float4 x = a < A ? xa[k] : xv[k], ww = w[k];
          acc[a] = radd(radd(radd(radd(acc[a], rmul(x.x, ww.x)), rmul(x.y, ww.y)), rmul(x.z, ww.z)), rmul(x.w, ww.w));
        }
    }
  }
#pragma unroll
  for (int a = 0; a < MAXA1; ++a)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc[a] = radd(acc[a], __shfl_xor(acc[a], o, 64));
  if (l == 0 && r < n) {
    float *out = heads + r * A1;
    float *co = cache ? cache + cache_rows[r] * A1 : nullptr;  // the per-stack heads cache row
#pragma unroll
    for (int a = 0; a < MAXA1; ++a)
      if (a <= A) {
        const float v = radd(acc[a], a < A ? ba2[a] : bv2[0]);
        out[a] = v;
        if (co) co[a] = v;
      }
  }
}

// k_heads_fc2 without LDS and within 64 VGPRs (the default for A + 1 <= 8): the weights are read
// from L2 one float4 column group at a time, so a workgroup fits beside kernels that hold most
// of a CU's LDS and registers (the x9 convs) instead of waiting for a free CU: 0.586 vs 0.589
// ms/step interleaved.  The same lanes, terms and order as k_heads_fc2: bit-identical
template <int MAXA1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_heads_fc2_lean(const float *__restrict__ h, int64_t ldh, int64_t n, int H,
                                                        int A, const float *__restrict__ wa2,
                                                        const float *__restrict__ wv2, const float *__restrict__ ba2,
                                                        const float *__restrict__ bv2, float *__restrict__ heads,
                                                        const int64_t *__restrict__ n_dev, float *__restrict__ cache,
                                                        const int64_t *__restrict__ cache_rows) {
  if (n_dev) {
    const int64_t nd = *n_dev;
    n = nd < n ? nd : n;
    if ((int64_t)blockIdx.x * 16 >= n) return;  // uniform
  }
  const int l = threadIdx.x & 15;
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t rr = r < n ? r : n - 1;  // tail rows: a duplicate, nothing written
  const int cq = H / 64, A1 = A + 1;
  const float4 *ha = reinterpret_cast<const float4 *>(h + rr * ldh) + l * cq;
  const float4 *hv = reinterpret_cast<const float4 *>(h + rr * ldh + H) + l * cq;
  float acc[MAXA1];
#pragma unroll
  for (int a = 0; a < MAXA1; ++a) acc[a] = 0.0f;
#pragma unroll 1
  for (int k = 0; k < cq; ++k) {
    const float4 xa = ha[k], xv = hv[k];
    float4 w[MAXA1];
#pragma unroll
    for (int a = 0; a < MAXA1; ++a) {
      const int ac = a < A1 ? a : A;  // past A: a duplicate row, unused
      w[a] = reinterpret_cast<const float4 *>(ac < A ? wa2 + (int64_t)ac * H : wv2)[l * cq + k];
    }
#pragma unroll
    for (int a = 0; a < MAXA1; ++a)
      if (a < A1) {
        const float4 x = a < A ? xa : xv, ww = w[a];
        acc[a] = radd(radd(radd(radd(acc[a], rmul(x.x, ww.x)), rmul(x.y, ww.y)), rmul(x.z, ww.z)), rmul(x.w, ww.w));
      }
  }
#pragma unroll
  for (int a = 0; a < MAXA1; ++a)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc[a] = radd(acc[a], __shfl_xor(acc[a], o, 64));
  if (l == 0 && r < n) {
    float *out = heads + r * A1;
    float *co = cache ? cache + cache_rows[r] * A1 : nullptr;
#pragma unroll
    for (int a = 0; a < MAXA1; ++a)
      if (a <= A) {
        const float v = radd(acc[a], a < A ? ba2[a] : bv2[0]);
        out[a] = v;
        if (co) co[a] = v;
      }
  }
}


// rows [r0, min(*n_dev, n_max)) of y = relu(x w^T + b), x [*, F] row stride ldx, w [O, F],
// y row stride ldy: the device-counted tail of a batch whose first r0 rows a library GEMM
// covers (the actors' terminal stacks behind the acting rows: none in most steps, so every
// workgroup usually exits at once).  Workgroup = kLrCols output columns; the rows go in
// chunks of kLrRows, each lane a strided float4 slice of F, the partial dots summed by xor
// shuffles and then across the waves in a fixed order (deterministic).
__global__ __launch_bounds__(kLrThreads) void k_linear_relu_rows(const float *__restrict__ x, int64_t ldx, int64_t r0,
                                                                 int64_t n_max, const int64_t *__restrict__ n_dev,
                                                                 const float *__restrict__ w,
                                                                 const float *__restrict__ b, int F, int O,
                                                                 float *__restrict__ y, int64_t ldy) {
  linear_relu_rows_wg((int)blockIdx.x, x, ldx, r0, n_max, n_dev, w, b, F, O, y, ldy);
}

}  // namespace rth

using namespace rth;

extern "C" {

int rth_bias_relu(float *y, const float *bias, int64_t rows, int32_t C, void *stream) {
  RTH_REQUIRE(y && bias, "rth_bias_relu: NULL argument");
  RTH_REQUIRE(C >= 4 && C % 4 == 0 && C <= 4096, "rth_bias_relu: channels %d must be a multiple of 4", C);
  RTH_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0, "rth_bias_relu: activations not 16-byte aligned");
  if (rows <= 0) return RTH_OK;
  const int64_t n4 = rows * C / 4;
  const int64_t want = (n4 + kEpiThreads - 1) / kEpiThreads;
  const int64_t blocks = want < 8192 ? want : 8192;
  hipLaunchKernelGGL(k_bias_relu, dim3((unsigned)blocks), dim3(kEpiThreads), 0, as_stream(stream),
                     reinterpret_cast<float4 *>(y), bias, n4, (int)C);
  RTH_LAUNCHED();
  return RTH_OK;
}

int64_t rth_relu_bias_grad_workspace(int32_t C) { return (int64_t)kGradBlocks * C * 4; }

int rth_relu_bias_grad(const float *g, const float *y, float *gy, float *db, void *workspace, int64_t rows,
                       int32_t C, void *stream) {
  RTH_REQUIRE(g && y && gy && workspace, "rth_relu_bias_grad: NULL argument");
  RTH_REQUIRE(C >= 4 && C % 4 == 0 && C <= kEpiThreads * 4 && kEpiThreads % (C / 4) == 0,
              "rth_relu_bias_grad: channels %d unsupported (multiple of 4 dividing 1024)", C);
  RTH_REQUIRE((C & (C - 1)) == 0 && C <= kEpiThreads, "rth_relu_bias_grad: channels %d must be a power of 2 <= 256", C);
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(gy) |
                reinterpret_cast<uintptr_t>(workspace)) & 15) == 0,
              "rth_relu_bias_grad: buffers not 16-byte aligned");
  if (rows <= 0) return RTH_OK;
  float *part = static_cast<float *>(workspace);
  const int64_t blocks = bias_grad_slabs(rows, C);
  hipLaunchKernelGGL(k_relu_bias_grad, dim3((unsigned)blocks), dim3(kEpiThreads), 0, as_stream(stream),
                     reinterpret_cast<const float4 *>(g), reinterpret_cast<const float4 *>(y),
                     reinterpret_cast<float4 *>(gy), part, rows, (int)C);
  RTH_LAUNCHED();
  if (!db) return RTH_OK;  // deferred: rth_conv_relu_wgrad_ex finishes it
  hipLaunchKernelGGL(k_bias_grad_combine, dim3(1), dim3(kCombThreads), 0, as_stream(stream), part, (int)blocks, (int)C,
                     db);
  RTH_LAUNCHED();
  return RTH_OK;
}


int rth_relu_bias_grad_nchw(const float *g, const float *y, float *gy, float *db, void *workspace, int64_t n,
                            int32_t C, int32_t P, void *stream) {
  RTH_REQUIRE(g && y && gy && workspace && n >= 0, "rth_relu_bias_grad_nchw: NULL argument");
  RTH_REQUIRE(C >= 4 && C <= kEpiThreads && (C & (C - 1)) == 0 && P >= 1 && (int64_t)C * (P + 1) <= kNchwMaxTile,
              "rth_relu_bias_grad_nchw: %d channels x %d positions unsupported", C, P);
  if (n == 0) return RTH_OK;
  float *part = static_cast<float *>(workspace);
  const int64_t blocks = bias_grad_slabs(n * P, C);  // the slab count a deferred job derives from rows = n * P
  hipLaunchKernelGGL(k_relu_bias_grad_nchw, dim3((unsigned)blocks), dim3(kEpiThreads), 0, as_stream(stream), g, y, gy,
                     part, n, (int)C, (int)P);
  RTH_LAUNCHED();
  if (!db) return RTH_OK;
  hipLaunchKernelGGL(k_bias_grad_combine, dim3(1), dim3(kCombThreads), 0, as_stream(stream), part, (int)blocks, (int)C,
                     db);
  RTH_LAUNCHED();
  return RTH_OK;
}


int rth_heads_merge(const float *const *params, int64_t H, int64_t F, int64_t A, int32_t C, int32_t P,
                    float *w1, float *b1, float *w2, float *b2, void *stream) {
  const int fc2_only = C == RTH_HEADS_FC2_ONLY;
  RTH_REQUIRE(params && (fc2_only || (w1 && b1)) && w2 && b2 && H >= 1 && F >= 1 && A >= 1,
              "rth_heads_merge: bad arguments");
  for (int k = fc2_only ? 4 : 0; k < 8; ++k) RTH_REQUIRE(params[k], "rth_heads_merge: parameter %d is NULL", k);
  if (fc2_only) {
    const HeadsDims d{H, F, A, 0, P, 1};
    hipLaunchKernelGGL(k_heads_merge, dim3(1), dim3(256), 0, as_stream(stream), d, params[0], params[1], params[2],
                       params[3], params[4], params[5], params[6], params[7], w1, b1, w2, b2);
    RTH_LAUNCHED();
    return RTH_OK;
  }
  RTH_REQUIRE(C == 0 || (int64_t)C * P == F, "rth_heads_merge: C*P != F");
  const HeadsDims d{H, F, A, C, P, 0};
  RTH_REQUIRE(F <= 12288, "rth_heads_merge: F %lld > 12288 (one row in LDS)", (long long)F);
  RTH_REQUIRE(F % 4 == 0 && C % 4 == 0 && ((reinterpret_cast<uintptr_t>(params[0]) | reinterpret_cast<uintptr_t>(params[1]) |
                                           reinterpret_cast<uintptr_t>(w1)) & 15) == 0,
              "rth_heads_merge: F and C must be multiples of 4, FC1 weights 16-byte aligned");
  const size_t lds = (size_t)(C ? F : 0) * 4;
  hipLaunchKernelGGL(k_heads_merge, dim3((unsigned)(2 * H + 1)), dim3(256), lds, as_stream(stream), d, params[0],
                     params[1], params[2],
                     params[3], params[4], params[5], params[6], params[7], w1, b1, w2, b2);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_heads_split_grad(const float *gw1, const float *gb1, const float *gw2, const float *gb2, int64_t H,
                         int64_t F, int64_t A, int32_t C, int32_t P, float *const *grads, void *stream) {
  const int fc2_only = C == RTH_HEADS_FC2_ONLY;
  RTH_REQUIRE((fc2_only || (gw1 && gb1)) && gw2 && gb2 && grads && H >= 1 && F >= 1 && A >= 1,
              "rth_heads_split_grad: bad arguments");
  for (int k = fc2_only ? 4 : 0; k < 8; ++k) RTH_REQUIRE(grads[k], "rth_heads_split_grad: gradient %d is NULL", k);
  if (fc2_only) {
    const HeadsDims d{H, F, A, 0, P, 1};
    hipLaunchKernelGGL(k_heads_split_grad, dim3(1), dim3(256), 0, as_stream(stream), d, gw1, gb1, gw2, gb2, grads[0],
                       grads[1], grads[2], grads[3], grads[4], grads[5], grads[6], grads[7]);
    RTH_LAUNCHED();
    return RTH_OK;
  }
  RTH_REQUIRE(C == 0 || (int64_t)C * P == F, "rth_heads_split_grad: C*P != F");
  const HeadsDims d{H, F, A, C, P, 0};
  RTH_REQUIRE(F <= 12288, "rth_heads_split_grad: F %lld > 12288 (one row in LDS)", (long long)F);
  RTH_REQUIRE(F % 4 == 0 && C % 4 == 0 && (reinterpret_cast<uintptr_t>(gw1) & 15) == 0,
              "rth_heads_split_grad: F and C must be multiples of 4, gw1 16-byte aligned");
  const size_t lds = (size_t)(C ? F + F / C : 0) * 4;
  hipLaunchKernelGGL(k_heads_split_grad, dim3((unsigned)(2 * H + 1)), dim3(256), lds, as_stream(stream), d, gw1, gb1,
                     gw2, gb2, grads[0],
                     grads[1], grads[2], grads[3], grads[4], grads[5], grads[6], grads[7]);
  RTH_LAUNCHED();
  return RTH_OK;
}

static int heads_backward_impl(const float *dq, const float *h, int64_t ldh, const Fc2 &f, int64_t B, int32_t H2,
                               int32_t A1, float *gh, float *gb1, const float *td_abs, float *td_acc, void *stream) {
  RTH_REQUIRE(B >= 1 && A1 >= 1 && A1 <= kHbMaxA1 && H2 >= kHbCols && H2 % kHbCols == 0 && ldh >= H2,
              "rth_heads_backward: bad shape B=%lld H2=%d A1=%d ldh=%lld", (long long)B, H2, A1, (long long)ldh);
  const dim3 grid((unsigned)(H2 / kHbCols + 1)), block(kHbThreads);
  if (A1 <= 8)  // Atari's minimal action sets (Pong 6, Breakout 4): 4 rows of dq in registers per batch
    hipLaunchKernelGGL((k_heads_backward<8, 4>), grid, block, 0, as_stream(stream), dq, h, ldh, f, B, H2, A1, gh, gb1,
                       td_abs, td_acc);
  else
    hipLaunchKernelGGL((k_heads_backward<kHbMaxA1, 1>), grid, block, 0, as_stream(stream), dq, h, ldh, f, B, H2, A1,
                       gh, gb1, td_abs, td_acc);
  RTH_LAUNCHED();
  return RTH_OK;
}


static int td_heads_backward_impl(const float *q0, const float *q1o, const float *q1t, const int64_t *a,
                                  const float *r, const float *done, const double *isw, int64_t B, int64_t A,
                                  float gamma_n, int32_t double_q, const float *h, int64_t ldh, const Fc2 &f,
                                  int32_t H2, float *td_abs, float *loss_out, float *gh, float *gb1, float *td_acc,
                                  void *stream) {
  RTH_REQUIRE(q0 && q1t && a && r && done && (q1o || !double_q) && h && td_abs && loss_out && gh && gb1,
              "rth_td_heads_backward: NULL argument");
  RTH_REQUIRE(B >= 1 && A >= 1 && A < kHbMaxA1 && B * (A + 1) <= kTdHbMaxElems && H2 >= kHbCols && H2 % kHbCols == 0 &&
                  ldh >= H2,
              "rth_td_heads_backward: bad shape B=%lld A=%lld H2=%d (B * (A + 1) <= %d)", (long long)B, (long long)A,
              H2, kTdHbMaxElems);
  const dim3 grid((unsigned)(H2 / kHbCols + 1)), block(kHbThreads);
  const size_t lds = (size_t)B * (A + 1) * 4;
  if (A + 1 <= 8)
    hipLaunchKernelGGL((k_td_heads_backward<8, 4>), grid, block, lds, as_stream(stream), q0, q1o, q1t, a, r, done, isw,
                       B, (int)A, gamma_n, double_q, h, ldh, f, H2, td_abs, loss_out, gh, gb1, td_acc);
  else if (A + 1 <= 8)
    hipLaunchKernelGGL((k_td_heads_backward<8, 4, false>), grid, block, lds, as_stream(stream), q0, q1o, q1t, a, r,
                       done, isw, B, (int)A, gamma_n, double_q, h, ldh, f, H2, td_abs, loss_out, gh, gb1, td_acc);
  else
    hipLaunchKernelGGL((k_td_heads_backward<kHbMaxA1, 1>), grid, block, lds, as_stream(stream), q0, q1o, q1t, a, r,
                       done, isw, B, (int)A, gamma_n, double_q, h, ldh, f, H2, td_abs, loss_out, gh, gb1, td_acc);
  RTH_LAUNCHED();
  return RTH_OK;
}

static Fc2 fc2_merged(const float *w2, float *gw2, float *gb2) {
  Fc2 f{};
  f.w2 = w2, f.gw2 = gw2, f.gb2 = gb2;
  return f;
}

// params = {wa2, wv2, ...}, grads = {gwa2, gwv2, gba2, gbv2}
static bool fc2_branches(const float *const *params, float *const *grads, int32_t H, int64_t A, Fc2 *f) {
  if (!params || !params[0] || !params[1] || !grads || H < kHbCols || H % kHbCols != 0) return false;
  for (int k = 0; k < 4; ++k)
    if (!grads[k]) return false;
  *f = Fc2{nullptr, nullptr, nullptr, params[0], params[1], grads[0], grads[1], grads[2], grads[3], (int)H, (int)A, 1};
  return true;
}

int rth_heads_backward(const float *dq, const float *h, int64_t ldh, const float *w2, int64_t B, int32_t H2,
                       int32_t A1, float *gh, float *gw2, float *gb2, float *gb1, const float *td_abs, float *td_acc,
                       void *stream) {
  RTH_REQUIRE(dq && h && w2 && gh && gw2 && gb2 && gb1, "rth_heads_backward: NULL argument");
  return heads_backward_impl(dq, h, ldh, fc2_merged(w2, gw2, gb2), B, H2, A1, gh, gb1, td_abs, td_acc, stream);
}

int rth_heads_backward_branches(const float *dq, const float *h, int64_t ldh, const float *const *fc2_params,
                                int32_t H, int64_t B, int64_t A, float *gh, float *const *fc2_grads, float *gb1,
                                const float *td_abs, float *td_acc, void *stream) {
  Fc2 f;
  RTH_REQUIRE(dq && h && gh && gb1 && fc2_branches(fc2_params, fc2_grads, H, A, &f),
              "rth_heads_backward_branches: NULL argument or H %d not a multiple of %d", H, kHbCols);
  return heads_backward_impl(dq, h, ldh, f, B, 2 * H, (int32_t)A + 1, gh, gb1, td_abs, td_acc, stream);
}

int rth_td_heads_backward(const float *q0, const float *q1o, const float *q1t, const int64_t *a, const float *r,
                          const float *done, const double *isw, int64_t B, int64_t A, float gamma_n, int32_t double_q,
                          const float *h, int64_t ldh, const float *w2, int32_t H2, float *td_abs, float *loss_out,
                          float *gh, float *gw2, float *gb2, float *gb1, float *td_acc, void *stream) {
  RTH_REQUIRE(w2 && gw2 && gb2, "rth_td_heads_backward: NULL argument");
  return td_heads_backward_impl(q0, q1o, q1t, a, r, done, isw, B, A, gamma_n, double_q, h, ldh,
                                fc2_merged(w2, gw2, gb2), H2, td_abs, loss_out, gh, gb1, td_acc, stream);
}

int rth_td_heads_backward_branches(const float *q0, const float *q1o, const float *q1t, const int64_t *a,
                                   const float *r, const float *done, const double *isw, int64_t B, int64_t A,
                                   float gamma_n, int32_t double_q, const float *h, int64_t ldh,
                                   const float *const *fc2_params, int32_t H, float *td_abs, float *loss_out, float *gh,
                                   float *const *fc2_grads, float *gb1, float *td_acc, void *stream) {
  Fc2 f;
  RTH_REQUIRE(fc2_branches(fc2_params, fc2_grads, H, A, &f),
              "rth_td_heads_backward_branches: NULL parameter / gradient or H %d not a multiple of %d", H, kHbCols);
  return td_heads_backward_impl(q0, q1o, q1t, a, r, done, isw, B, A, gamma_n, double_q, h, ldh, f, 2 * H, td_abs,
                                loss_out, gh, gb1, td_acc, stream);
}

static int heads_fc2_impl(const float *h, int64_t ldh, int64_t n, int32_t H, int32_t A,
                          const float *const *fc2_params, float *heads, const int64_t *n_dev, float *cache,
                          const int64_t *cache_rows, void *stream) {
  RTH_REQUIRE(h && heads && fc2_params && fc2_params[0] && fc2_params[1] && fc2_params[2] && fc2_params[3],
              "rth_heads_fc2: NULL argument");
  RTH_REQUIRE(n >= 0 && H >= 16 && H % 16 == 0 && A >= 1 && A < kHbMaxA1 && ldh >= 2 * H && ldh % 4 == 0 &&
                  (reinterpret_cast<uintptr_t>(h) & 15) == 0,
              "rth_heads_fc2: bad shape n=%lld H=%d A=%d ldh=%lld (H a multiple of 16, h 16-byte aligned rows)",
              (long long)n, H, A, (long long)ldh);
  if (n == 0) return RTH_OK;
  RTH_REQUIRE(H <= kFc2MaxH && H % 64 == 0,
              "rth_heads_fc2: built for H <= %d, a multiple of 64 (A=%d H=%d)", kFc2MaxH, A, H);
  const dim3 grid((unsigned)((n + 15) / 16)), block(256);
  const size_t lds = (size_t)(A + 1) * H * 4 + 16;  // + the spare slot of the staging writes
  if (A + 1 <= 8)
    hipLaunchKernelGGL((k_heads_fc2_lean<8>), grid, block, 0, as_stream(stream), h, ldh, n, (int)H, (int)A,
                       fc2_params[0], fc2_params[1], fc2_params[2], fc2_params[3], heads, n_dev, cache, cache_rows);
  else if (A + 1 <= 8)
    hipLaunchKernelGGL((k_heads_fc2<8>), grid, block, lds, as_stream(stream), h, ldh, n, (int)H, (int)A, fc2_params[0],
                       fc2_params[1], fc2_params[2], fc2_params[3], heads, n_dev, cache, cache_rows);
  else
    hipLaunchKernelGGL((k_heads_fc2<kHbMaxA1>), grid, block, lds, as_stream(stream), h, ldh, n, (int)H, (int)A,
                       fc2_params[0], fc2_params[1], fc2_params[2], fc2_params[3], heads, n_dev, cache, cache_rows);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_heads_fc2(const float *h, int64_t ldh, int64_t n, int32_t H, int32_t A, const float *const *fc2_params,
                  float *heads, void *stream) {
  return heads_fc2_impl(h, ldh, n, H, A, fc2_params, heads, nullptr, nullptr, nullptr, stream);
}

int rth_heads_fc2_upto(const float *h, int64_t ldh, int64_t n_max, const int64_t *n_dev, int32_t H, int32_t A,
                       const float *const *fc2_params, float *heads, float *cache, const int64_t *cache_rows,
                       void *stream) {
  RTH_REQUIRE(n_dev && (!cache || cache_rows), "rth_heads_fc2_upto: NULL count or cache rows");
  return heads_fc2_impl(h, ldh, n_max, H, A, fc2_params, heads, n_dev, cache, cache_rows, stream);
}

int rth_linear_relu_rows_upto(const float *x, int64_t ldx, int64_t r0, int64_t n_max, const int64_t *n_dev,
                              const float *w, const float *b, int64_t F, int64_t O, float *y, int64_t ldy,
                              void *stream) {
  RTH_REQUIRE(x && n_dev && w && b && y, "rth_linear_relu_rows_upto: NULL argument");
  RTH_REQUIRE(r0 >= 0 && n_max >= r0 && F >= 4 && F % 4 == 0 && O >= 1 && O <= (int64_t)1 << 30 && ldx >= F &&
                  ldx % 4 == 0 && ldy >= O && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w)) & 15) == 0,
              "rth_linear_relu_rows_upto: bad shape r0=%lld n_max=%lld F=%lld O=%lld ldx=%lld ldy=%lld (F, ldx "
              "multiples of 4, x and w 16-byte aligned)",
              (long long)r0, (long long)n_max, (long long)F, (long long)O, (long long)ldx, (long long)ldy);
  if (n_max == r0) return RTH_OK;
  hipLaunchKernelGGL(k_linear_relu_rows, dim3((unsigned)((O + kLrCols - 1) / kLrCols)), dim3(kLrThreads), 0,
                     as_stream(stream), x, ldx, r0, n_max, n_dev, w, b, (int)F, (int)O, y, ldy);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
