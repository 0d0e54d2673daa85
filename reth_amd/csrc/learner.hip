// Learner-side kernel: DQN TD error + Huber loss + its gradient w.r.t. Q(s0), fused.
//
// Reference: reth/reth/algorithm/dqn/dqn_solver.py:68-124.  The Q-network itself stays in
// PyTorch-ROCm (MIOpen/hipBLASLt MFMA GEMMs, fp32); this kernel replaces the chain of
// one_hot / sum / argmax / mul / sub / smooth_l1 / mul / mean / |td|.cpu() ops and their
// autograd backward with one launch, keeps |td| on the device for the priority update, and
// hands autograd d(loss)/d(Q(s0)) directly.
#include <cstdarg>
#include <mutex>

#include "common.hpp"

namespace rth {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

constexpr int kTdThreads = 512;

// One workgroup: B = 512 rows is one row per lane; larger B loops.  The loss mean is a
// fixed-order LDS tree (deterministic run to run).
__global__ __launch_bounds__(kTdThreads) void k_td_huber(
    const float *__restrict__ q0, const float *__restrict__ q1o, const float *__restrict__ q1t,
    const int64_t *__restrict__ act, const float *__restrict__ rew, const float *__restrict__ done,
    const double *__restrict__ isw, int64_t B, int A, float gamma_n, int double_q, int dueling, float *__restrict__ td_out,
    float *__restrict__ td_abs_out, float *__restrict__ loss_elem, float *__restrict__ loss_out,
    float *__restrict__ dq) {
  __shared__ float part[kTdThreads];
  const float invB = 1.0f / (float)B;
  float acc = 0.0f;
  const int ld = A + dueling;  // row length: A values, or A advantages + 1 state value
  for (int64_t b = threadIdx.x; b < B; b += kTdThreads) {
    float l;
    const float td = td_huber_row(q0, q1o, q1t, act, rew, done, isw, b, A, dueling, gamma_n, double_q, invB, &l,
                                  dq ? dq + b * ld : nullptr);
    if (td_out) td_out[b] = td;
    if (td_abs_out) td_abs_out[b] = fabsf(td);  // td_error.detach().cpu().abs() (:109), kept on device
    if (loss_elem) loss_elem[b] = l;
    acc = radd(acc, l);
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kTdThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] = radd(part[threadIdx.x], part[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0 && loss_out) loss_out[0] = part[0] * invB;
}

}  // namespace rth

using namespace rth;

extern "C" {

const char *rth_last_error(void) { return g_last_error.c_str(); }

int rth_version(void) { return 100; }  // 0.1.0

#ifndef RTH_BUILD_ID
#define RTH_BUILD_ID "unknown"
#endif
// the marker lets __graft_entry__.build() read the id from the file without loading it
static const char k_build_id_marker[] __attribute__((used)) = "RTH_BUILD_ID:" RTH_BUILD_ID;
const char *rth_build_id(void) { return k_build_id_marker + 13; }

int rth_graph_upload(void *graph_exec, void *stream) {
  RTH_REQUIRE(graph_exec, "rth_graph_upload: NULL graph");
  const hipError_t e = hipGraphUpload(static_cast<hipGraphExec_t>(graph_exec), as_stream(stream));
  RTH_REQUIRE(e == hipSuccess, "rth_graph_upload: %s", hipGetErrorString(e));
  return RTH_OK;
}

int rth_stream_capture_deps(void *stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const hipGraphNode_t *deps = nullptr;
  size_t n = 0;
  const hipError_t e = hipStreamGetCaptureInfo_v2(as_stream(stream), &st, nullptr, nullptr, &deps, &n);
  RTH_REQUIRE(e == hipSuccess, "rth_stream_capture_deps: %s", hipGetErrorString(e));
  return st == hipStreamCaptureStatusActive ? (int)n : -1;
}

int rth_td_huber(const float *q0, const float *q1o, const float *q1t, const int64_t *a, const float *r,
                 const float *done, const double *isw, int64_t B, int64_t A, float gamma_n, int32_t double_q,
                 int32_t dueling, float *td_out, float *td_abs_out, float *loss_elem, float *loss_out, float *dq,
                 void *stream) {
  RTH_REQUIRE(B >= 1 && A >= 1 && A <= kMaxActions && (dueling == 0 || dueling == 1),
              "rth_td_huber: bad shape B=%lld A=%lld", (long long)B, (long long)A);
  RTH_REQUIRE(q0 && q1t && a && r && done && (q1o || !double_q), "rth_td_huber: NULL input");
  hipLaunchKernelGGL(k_td_huber, dim3(1), dim3(kTdThreads), 0, as_stream(stream), q0, q1o, q1t, a, r, done, isw, B,
                     (int)A, gamma_n, double_q, dueling, td_out, td_abs_out, loss_elem, loss_out, dq);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
