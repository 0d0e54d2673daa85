// Shared helpers for libreth_hip.so (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/reth_hip.h"

// Reference parity needs every f32/f64 product and sum rounded exactly where the reference
// (numpy / numba / torch CPU) rounds it, so nothing in this library may be contracted into
// an FMA.  The pragma covers all code after this point; the build keeps clang's default
// -ffp-contract=fast-honor-pragmas so the ocml math library (pow, exp) keeps the fused
// operations its accuracy depends on.  (The clang HIP header's __fmul_rn & co. are plain
// `x * y` compiled before this pragma, i.e. contractible -- use radd/rsub/rmul instead.)
#pragma clang fp contract(off)

namespace rth {

__host__ __device__ __forceinline__ float radd(float a, float b) { return a + b; }
__host__ __device__ __forceinline__ float rsub(float a, float b) { return a - b; }
__host__ __device__ __forceinline__ float rmul(float a, float b) { return a * b; }
__host__ __device__ __forceinline__ double radd(double a, double b) { return a + b; }
__host__ __device__ __forceinline__ double rsub(double a, double b) { return a - b; }
__host__ __device__ __forceinline__ double rmul(double a, double b) { return a * b; }

// bf16 MFMA operands and the exact three-term bf16 split of fp32 values (conv.hip, wgrad.hip):
// every fp32 v is h1 + h2 + h3 exactly, h1 = rne(v), h2 = rne(v - h1), h3 = rne(v - h1 - h2)
// (8 + 8 + 8 significand bits; each residual is a difference of nearby floats, so exact)
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
__host__ __device__ __forceinline__ uint32_t bf16_rne_bits(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__host__ __device__ __forceinline__ float bf16_bits_f(uint32_t b) { return __uint_as_float(b << 16); }
// the three bf16 terms of 4 fp32 values, packed 2 per dword: out[t] = {t(v0) | t(v1) << 16, ...},
// on the hardware's paired round-to-nearest-even conversion (v_cvt_pk_bf16_f32: the same terms
// as bf16_rne_bits for every finite value, at a quarter of the instructions)
using f32x2v = __attribute__((ext_vector_type(2))) float;
using bf16x2v = __attribute__((ext_vector_type(2))) __bf16;
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t (&t)[3]) {
  f32x2v x = f32x2v{a, b};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const bf16x2v h = __builtin_convertvector(x, bf16x2v);
    t[k] = __builtin_bit_cast(uint32_t, h);
    if (k < 2) x = x - __builtin_convertvector(h, f32x2v);  // exact: h is x's nearest bf16
  }
}
__device__ __forceinline__ void split3_x4(float4 v, uint2 (&out)[3]) {
  uint32_t lo[3], hi[3];
  split3_pair(v.x, v.y, lo);
  split3_pair(v.z, v.w, hi);
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k] = make_uint2(lo[k], hi[k]);
}

// the same split of 8 values: one 16-byte MFMA fragment per term
__device__ __forceinline__ void split3_pk8(const float (&v)[8], bf16x8 (&out)[3]) {
  uint32_t t[4][3];
#pragma unroll
  for (int q = 0; q < 4; ++q) split3_pair(v[2 * q], v[2 * q + 1], t[q]);
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k] = __builtin_bit_cast(bf16x8, u32x4{t[0][k], t[1][k], t[2][k], t[3][k]});
}

// rth_relu_bias_grad's partial-sum slabs: one per workgroup of kBiasThreads lanes, about 8
// row sweeps each, at most kBiasSlabs (shared with the deferred combine in conv.hip)
constexpr int kBiasThreads = 256, kBiasSlabs = 2048;
__host__ __device__ inline int64_t bias_grad_slabs(int64_t rows, int C) {
  const int64_t R = kBiasThreads / (C / 4);  // rows per block sweep
  const int64_t want = (rows + 8 * R - 1) / (8 * R);
  return want < kBiasSlabs ? want : kBiasSlabs;
}

void set_error(const char *fmt, ...);

#define RTH_REQUIRE(cond, ...)          \
  do {                                  \
    if (!(cond)) {                      \
      ::rth::set_error(__VA_ARGS__);    \
      return RTH_ERR_INVALID;           \
    }                                   \
  } while (0)

#define RTH_HIP(call)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::rth::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                       __LINE__);                                                       \
      return RTH_ERR_HIP;                                                               \
    }                                                                                   \
  } while (0)

// check a kernel launch (no sync)
#define RTH_LAUNCHED() RTH_HIP(hipGetLastError())

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline int dtype_size(int32_t t) {
  switch (t) {
    case RTH_U8: return 1;
    case RTH_I32: return 4;
    case RTH_I64: return 8;
    case RTH_F32: return 4;
    case RTH_F64: return 8;
    default: return 0;
  }
}

// ---------------------------------------------------------------- Philox4x32-10
// Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11).  Counter-based, so
// every lane derives its own stream from (seed, counter, lane, stream id) with no state.
// Restated bit-for-bit in oracle/reth_oracle.c (orc_philox4x32) for the parity tests.
constexpr uint32_t STREAM_SAMPLE = 1u, STREAM_EXPLORE = 2u, STREAM_RANDACT = 3u, STREAM_ENV = 4u, STREAM_ATARI = 5u,
                   STREAM_ATARI_RESET = 6u;

__host__ __device__ inline void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int rnd = 0; rnd < 10; ++rnd) {
    if (rnd) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
  }
}

// u in [0, 1) with 53 random bits; same mapping as orc_philox_uniform
__host__ __device__ inline double philox_uniform(uint64_t seed, uint64_t counter, uint32_t lane,
                                                 uint32_t stream) {
  uint32_t c[4] = {lane, (uint32_t)counter, (uint32_t)(counter >> 32), stream};
  philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint64_t bits = ((uint64_t)c[0] | ((uint64_t)c[1] << 32)) >> 11;
  return (double)bits * (1.0 / 9007199254740992.0);
}

// first-maximum argmax with torch semantics (a NaN is the maximum; the first NaN wins)
__device__ inline int argmax_first(const float *q, int A) {
  int best = 0;
  float bv = q[0];
  for (int j = 1; j < A; ++j) {
    const float v = q[j];
    if (bv != bv) break;
    if (v != v || v > bv) {
      bv = v;
      best = j;
    }
  }
  return best;
}

// Q values of one row of network output.  Plain: q_j = row[j].  Dueling heads (row = A
// advantages then the state value, dqn_model.py:185-193): q_j = (v + a_j) - mean(a), with
// torch's mean = sum * (1/A).  A <= kMaxActions.
constexpr int kMaxActions = 32;
__device__ inline void q_row(const float *row, int A, int dueling, float *q) {
  if (!dueling) {
    for (int j = 0; j < A; ++j) q[j] = row[j];
    return;
  }
  float s = 0.0f;
  for (int j = 0; j < A; ++j) s = radd(s, row[j]);
  const float mean = rmul(s, 1.0f / (float)A);
  const float v = row[A];
  for (int j = 0; j < A; ++j) q[j] = rsub(radd(v, row[j]), mean);
}

// The same row arithmetic with each network-output row held in registers: MAXL >= A + dueling
// values loaded unconditionally (indices clamped to the row), so every load of a row is issued
// before any is waited for -- the pointer forms' runtime-length loops load one value per round
// trip.  Identical operations in identical order: the results equal q_row / argmax_first /
// td_huber_row bit for bit.
template <int MAXL>
__device__ inline void load_row(const float *__restrict__ row, int L, float (&v)[MAXL]) {
#pragma unroll
  for (int j = 0; j < MAXL; ++j) v[j] = row[j < L ? j : L - 1];
}

template <int MAXL>
__device__ inline void q_row_reg(const float (&r)[MAXL], int A, int dueling, float (&q)[MAXL]) {
  if (!dueling) {
#pragma unroll
    for (int j = 0; j < MAXL; ++j) q[j] = r[j];
    return;
  }
  float s = 0.0f, v = 0.0f;
#pragma unroll
  for (int j = 0; j < MAXL; ++j) {
    if (j < A) s = radd(s, r[j]);
    if (j == A) v = r[j];
  }
  const float mean = rmul(s, 1.0f / (float)A);
#pragma unroll
  for (int j = 0; j < MAXL; ++j) q[j] = rsub(radd(v, r[j]), mean);
}

template <int MAXL>
__device__ inline int argmax_first_reg(const float (&q)[MAXL], int A) {  // argmax_first's rule
  int best = 0;
  float bv = q[0];
  bool stop = false;
#pragma unroll
  for (int j = 1; j < MAXL; ++j)
    if (j < A && !stop) {
      if (bv != bv) {
        stop = true;
      } else if (q[j] != q[j] || q[j] > bv) {
        bv = q[j];
        best = j;
      }
    }
  return best;
}

template <int MAXL>
__device__ inline float pick(const float (&q)[MAXL], int i) {  // q[i] as a select chain in registers
  float x = q[0];
#pragma unroll
  for (int j = 1; j < MAXL; ++j) {
    float qj = q[j];
    asm volatile("" : "+v"(qj));  // opaque: LLVM would turn the chain back into a scratch array lookup
    x = j == i ? qj : x;
  }
  return x;
}

// td_huber_row for rows given as pointers to their first value (q0r / q1r / q1tr), no dq
template <int MAXL>
__device__ inline float td_huber_row_reg(const float *__restrict__ q0r, const float *__restrict__ q1r,
                                         const float *__restrict__ q1tr, int64_t a, float rw, float dn, float w,
                                         int has_w, int A, int dueling, float gamma_n, int double_q, float *l_out) {
  const int ld = A + dueling;
  float r0[MAXL], r1[MAXL], r2[MAXL];
  load_row(q0r, ld, r0);
  load_row(double_q ? q1r : q1tr, ld, r1);
  load_row(q1tr, ld, r2);
  float qa[MAXL], qs[MAXL];
  q_row_reg(r0, A, dueling, qa);
  const float q = pick(qa, (int)a);  // sum(q * one_hot(a)) (:79-81)
  q_row_reg(r1, A, dueling, qs);
  const int astar = argmax_first_reg(qs, A);  // (:83-94)
  if (double_q) q_row_reg(r2, A, dueling, qs);
  const float nqb = pick(qs, astar);
  float t = rmul(gamma_n, nqb);  // expected = r + (gamma**n * next_q_best) * (1 - done)  (:96)
  t = rmul(t, rsub(1.0f, dn));
  const float y = radd(rw, t);
  const float td = rsub(q, y);  // (:97)
  const float z = fabsf(td);
  float l = z < 1.0f ? rmul(rmul(0.5f, z), z) : rsub(z, 0.5f);  // smooth_l1 (:112) * w (:113-114)
  if (has_w) l = rmul(l, w);
  *l_out = l;
  return td;
}

// One row of DQNSolver._calc_td_error + the IS-weighted smooth-L1 loss (dqn_solver.py:77-114):
// returns td; *l_out = smooth_l1(|td|) * w; dq_row (nullable, A + dueling values) = d(mean
// loss)/d(q row of s0) -- through Q = (V + A) - mean(A) when dueling.  f32, no contraction.
__device__ inline float td_huber_row(const float *__restrict__ q0, const float *__restrict__ q1o,
                                     const float *__restrict__ q1t, const int64_t *__restrict__ act,
                                     const float *__restrict__ rew, const float *__restrict__ done,
                                     const double *__restrict__ isw, int64_t b, int A, int dueling, float gamma_n,
                                     int double_q, float invB, float *l_out, float *dq_row) {
  const int ld = A + dueling;  // row length: A values, or A advantages + 1 state value
  const int64_t a = act[b];
  float qa[kMaxActions], qs[kMaxActions];
  q_row(q0 + b * ld, A, dueling, qa);
  const float q = qa[a];  // sum(q * one_hot(a)) (:79-81)
  q_row((double_q ? q1o : q1t) + b * ld, A, dueling, qs);
  const int astar = argmax_first(qs, A);  // (:83-94)
  if (double_q) q_row(q1t + b * ld, A, dueling, qs);
  const float nqb = qs[astar];
  // expected = r + (gamma**n * next_q_best) * (1 - done)  (:96)
  float t = rmul(gamma_n, nqb);
  t = rmul(t, rsub(1.0f, done[b]));
  const float y = radd(rew[b], t);
  const float td = rsub(q, y);  // (:97)
  const float z = fabsf(td);
  // smooth_l1(beta=1) (:112) * w (:113-114)
  float l = z < 1.0f ? rmul(rmul(0.5f, z), z) : rsub(z, 0.5f);
  const float w = isw ? (float)isw[b] : 1.0f;
  if (isw) l = rmul(l, w);
  *l_out = l;
  if (dq_row) {  // autograd: mean -> mul(w) -> smooth_l1' -> one_hot scatter
    const float g = rmul(invB, w);
    const float d = td <= -1.0f ? -g : (td >= 1.0f ? g : rmul(td, g));
    if (!dueling) {
      for (int j = 0; j < A; ++j) dq_row[j] = rmul(d, j == a ? 1.0f : 0.0f);
    } else {  // through q = (v + adv) - mean(adv): d adv_j = g_j + (-sum g) / A, d v = sum g
      const float dm = (-d) / (float)A;
      for (int j = 0; j < A; ++j) dq_row[j] = radd(j == a ? d : 0.0f, dm);
      dq_row[A] = d;
    }
  }
  return td;
}

// PERSampler._normalize_weights (per_sampler.py:16-17): (w + 1e-6) ** alpha in float32,
// correctly rounded; numpy's `** 0.5` is sqrt (fast_scalar_power), also correctly rounded.
__device__ inline float per_normalize(float w, float alpha) {
  const float x = radd(w, 1e-6f);
  if (alpha == 0.5f) return sqrtf(x);  // NOT __fsqrt_rn: that is __ocml_native_sqrt_f32 (approximate)
  if (alpha == 1.0f) return x;
  return (float)pow((double)x, (double)alpha);
}

// Device-resident service state of a replay shard: every per-step scalar a launch needs is
// read from here, so launches are argument-invariant and a captured HIP graph replays them.
struct ReplayState {
  int64_t tail;        // FIFOPolicy.tail (fifo_policy.py:10)
  int64_t calls;       // sample calls issued (Philox counter)
  int64_t sched_step;  // Schedule.cur_step shared by alpha and beta (per_sampler.py:30-32)
  int64_t pad;
};

// A PER priority update recorded by rth_replay_update_priorities_deferred and applied by the
// next tree-update launch of the shard (merged with an append's), before its keys.
struct UpdPending {
  const int64_t *idx;
  const void *td;
  int32_t dtype;
  int32_t step;  // advance the schedules first (update_priorities(step=True))
  int64_t n;
};

// Schedule.value (schedule.py:29-40, 48-52), python float operation order
__host__ __device__ inline double sched_value(const rth_schedule &s, int64_t step) {
  if (s.method == RTH_SCHED_CONST) return s.start;
  const int64_t k = step < s.max_steps ? step : s.max_steps;
  if (s.method == RTH_SCHED_LINEAR) return s.start + ((s.end - s.start) * (double)k) / (double)s.max_steps;
  return s.end - (s.end - s.start) * exp((double)(-k) / (double)s.max_steps);
}

// the same in float64 (numpy float64 arrays: `** 0.5` is sqrt, other exponents pow)
__device__ inline double per_normalize64(double w, double alpha) {
  const double x = radd(w, 1e-6);
  if (alpha == 0.5) return sqrt(x);
  if (alpha == 1.0) return x;
  return pow(x, alpha);
}

}  // namespace rth
