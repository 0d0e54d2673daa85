// Actor-side kernels: batched epsilon-greedy, per-actor n-step adders, synthetic
// Pong-shaped environment.
//
// Reference: reth/reth/utils/exploration.py:26-31 (RandomExploration.act),
// reth/reth/algorithm/dqn/dqn_solver.py:126-131 (act = argmax Q),
// reth/reth/utils/nstep_adder.py:5-28 (NStepAdder), test/apex-dqn/worker.py:21-61.
#include "common.hpp"

namespace rth {

// ------------------------------------------------------------------ epsilon-greedy
// One lane per actor: A <= 18 for Atari, so the row argmax is a short in-register loop and
// the launch is one wave per 64 actors.
__device__ inline int64_t eps_greedy_one(const float *__restrict__ q, int64_t i, int A, int dueling,
                                         const double *__restrict__ eps, const double *__restrict__ u_in,
                                         const int64_t *__restrict__ ra_in, uint64_t seed, uint64_t counter) {
  const double u = u_in ? u_in[i] : philox_uniform(seed, counter, (uint32_t)i, STREAM_EXPLORE);
  if (u < eps[i]) {
    if (ra_in) return ra_in[i];
    uint32_t c[4] = {(uint32_t)i, (uint32_t)counter, (uint32_t)(counter >> 32), STREAM_RANDACT};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return (int64_t)(((uint64_t)c[0] * (uint64_t)A) >> 32);  // uniform in [0, A)
  }
  float qr[kMaxActions];
  q_row(q + i * (A + dueling), A, dueling, qr);
  return argmax_first(qr, A);
}

__global__ void k_eps_greedy(const float *__restrict__ q, int64_t N, int A, int dueling, const double *__restrict__ eps,
                             const double *__restrict__ u_in, const int64_t *__restrict__ ra_in, uint64_t seed,
                             uint64_t counter, const int64_t *__restrict__ counter_dev, int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  if (counter_dev) counter = (uint64_t)*counter_dev;
  out[i] = eps_greedy_one(q, i, A, dueling, eps, u_in, ra_in, seed, counter);
}

// ------------------------------------------------------------------ n-step adder
// Per actor: a deque of up to n pending rows, position 0 = newest (appendleft), SoA in HBM.
struct NStepState {
  int32_t *count;
  int64_t *s0, *a, *s1;
  float *r, *done;
};

__device__ inline void nstep_push_one(const NStepState &st, int64_t i, int n, double gamma, int mode, int64_t s0,
                                      int64_t a, float rn, int64_t s1n, float done, int32_t *__restrict__ emit,
                                      int64_t *__restrict__ s0_out, int64_t *__restrict__ a_out,
                                      float *__restrict__ r_out, int64_t *__restrict__ s1_out,
                                      float *__restrict__ done_out) {
  const int64_t base = i * n;
  int count = st.count[i];
  int emitted = 0;
  if (count == n) {  // deque full: pop the oldest (nstep_adder.py:13-14)
    const int64_t k = base + count - 1;
    s0_out[i] = st.s0[k];
    a_out[i] = st.a[k];
    r_out[i] = st.r[k];
    s1_out[i] = st.s1[k];
    done_out[i] = st.done[k];
    --count;
    emitted = 1;
  }
  emit[i] = emitted;
  double t_gamma = gamma;
  for (int k = 0; k < count; ++k) {  // newest -> oldest (nstep_adder.py:16-25)
    const int64_t p = base + k;
    if (st.done[p] != 0.0f) break;
    if (mode == 0)  // numpy 1.19: f64 product, += casts back to the f32 row
      st.r[p] = (float)radd((double)st.r[p], rmul(t_gamma, (double)rn));
    else            // numpy 2 / NEP 50: the python float is weak, product stays f32
      st.r[p] = radd(st.r[p], rmul((float)t_gamma, rn));
    t_gamma = rmul(t_gamma, gamma);
    st.s1[p] = s1n;
  }
  for (int k = count; k > 0; --k) {  // appendleft
    const int64_t p = base + k;
    st.s0[p] = st.s0[p - 1];
    st.a[p] = st.a[p - 1];
    st.r[p] = st.r[p - 1];
    st.s1[p] = st.s1[p - 1];
    st.done[p] = st.done[p - 1];
  }
  st.s0[base] = s0;
  st.a[base] = a;
  st.r[base] = rn;
  st.s1[base] = s1n;
  st.done[base] = done;
  st.count[i] = count + 1;
}

__global__ void k_nstep_push(NStepState st, int64_t N, int n, double gamma, int mode,
                             const int64_t *__restrict__ s0, const int64_t *__restrict__ a,
                             const float *__restrict__ r, const int64_t *__restrict__ s1,
                             const float *__restrict__ done, int32_t *__restrict__ emit,
                             int64_t *__restrict__ s0_out, int64_t *__restrict__ a_out,
                             float *__restrict__ r_out, int64_t *__restrict__ s1_out,
                             float *__restrict__ done_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  nstep_push_one(st, i, n, gamma, mode, s0[i], a[i], r[i], s1[i], done[i], emit, s0_out, a_out, r_out, s1_out,
                 done_out);
}

// ------------------------------------------------------------------ synthetic env
constexpr int kFrameBytes = 84 * 84;          // 7,056
constexpr int kFrameVec = kFrameBytes / 16;   // 441 x 16 B
constexpr int kStackVec = 4 * kFrameVec;      // 1,764 x 16 B = 28,224 B
constexpr int kEnvThreads = 256;

__device__ __forceinline__ uint4 env_bytes(uint64_t seed, int64_t actor, int64_t t, int kind, int chunk) {
  uint32_t c[4] = {(uint32_t)chunk | ((uint32_t)kind << 16), (uint32_t)actor, (uint32_t)t,
                   STREAM_ENV | ((uint32_t)(t >> 32) << 8)};
  philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return make_uint4(c[0], c[1], c[2], c[3]);
}

// one actor's synthetic env step by a whole workgroup; returns (in every lane) the reward,
// done flag and the s0 / s1 stack handles; lane 0 writes them and the new cur_slot
struct EnvOut {
  float reward;
  bool done;
  int64_t s0h, s1h;
};

// write_frames = 0: the observation comes from outside (the Atari preprocessing of raw frames,
// rth_atari_env_step, fills the two stacks this step assigns right after this launch)
__device__ inline EnvOut env_step_one(uint8_t *frames, int ring, int64_t t, int64_t i, int64_t *cur_slot, uint64_t seed,
                                      float p_reward, float p_done, float *r_out, float *done_out, int64_t *s0_h,
                                      int64_t *s1_h, int write_frames = 1) {
  const int64_t stack_bytes = 4 * kFrameBytes;
  // reward / done: one Philox block per (actor, t), identical in every lane
  const uint4 rd = env_bytes(seed, i, t, 2, 0);
  const double ur = (double)rd.x * (1.0 / 4294967296.0), ud = (double)rd.y * (1.0 / 4294967296.0);
  const float reward = ur < 0.5 * p_reward ? -1.0f : (ur < p_reward ? 1.0f : 0.0f);
  const bool done = ud < (double)p_done;
  const int64_t cur = cur_slot[i];
  const int64_t nxt = (2 * t) % ring, rst = (2 * t + 1) % ring;
  const uint4 *src = reinterpret_cast<const uint4 *>(frames + (i * ring + cur) * stack_bytes);
  uint4 *dn = reinterpret_cast<uint4 *>(frames + (i * ring + nxt) * stack_bytes);
  uint4 *dr = reinterpret_cast<uint4 *>(frames + (i * ring + rst) * stack_bytes);
  for (int v = threadIdx.x; write_frames && v < kStackVec; v += kEnvThreads) {
    const int f = v / kFrameVec, c = v - f * kFrameVec;
    dn[v] = (f < 3) ? src[v + kFrameVec] : env_bytes(seed, i, t, 0, c);  // FrameStack shift
    if (done) dr[v] = env_bytes(seed, i, t, 1, c);                        // reset: one frame x4
  }
  __syncthreads();  // every lane has read cur_slot[i] before lane 0 rewrites it
  const EnvOut o{reward, done, i * ring + cur, i * ring + nxt};
  if (threadIdx.x == 0) {
    r_out[i] = reward;
    done_out[i] = done ? 1.0f : 0.0f;
    s0_h[i] = o.s0h;
    s1_h[i] = o.s1h;
    cur_slot[i] = done ? rst : nxt;
  }
  return o;
}

__global__ __launch_bounds__(kEnvThreads) void k_env_step(uint8_t *frames, int ring, int64_t t,
                                                          const int64_t *t_dev, int64_t *cur_slot, uint64_t seed,
                                                          float p_reward, float p_done, float *r_out,
                                                          float *done_out, int64_t *s0_h, int64_t *s1_h,
                                                          int write_frames) {
  if (t_dev) t = *t_dev;
  env_step_one(frames, ring, t, blockIdx.x, cur_slot, seed, p_reward, p_done, r_out, done_out, s0_h, s1_h,
               write_frames);
}

// The tail of a fused actor step (VecActors.step_fused), one workgroup per actor i:
// epsilon-greedy on its acting heads, |td| of its previous n-step row from the per-stack heads
// cache (calc_loss, target == online), its env step and its n-step push -- the same device
// functions as k_eps_greedy / k_td_huber / k_env_step / k_nstep_push, one launch instead of
// six (the rows' two heads gathers included).
struct ActorTail {
  const float *q;  // acting heads [N, A + 1]
  const double *eps;
  uint64_t seed;
  const int64_t *t_dev;
  int64_t *action;
  const float *qcache;  // [stacks, A + 1]
  const int64_t *prev_s0, *prev_a, *prev_s1;
  const float *prev_r, *prev_done;
  float gamma_n;
  float *td_abs;
  uint8_t *frames;
  int ring;
  int64_t *cur_slot;
  float p_reward, p_done;
  float *r_out, *done_out;
  int64_t *s0_h, *s1_h;
  NStepState ns;
  int n;
  double gamma;
  int mode;
  int32_t *emit;
  int64_t *row_s0, *row_a, *row_s1;
  float *row_r, *row_done;
  int A;
  int ext_frames;  // the observations come from rth_atari_env_step (no synthetic frame bytes)
};

// MAXL > 0: the heads rows (A + 1 <= MAXL values) are loaded into registers all at once
// (load_row / td_huber_row_reg, the same arithmetic) instead of one value per round trip
template <int MAXL>
__global__ __launch_bounds__(kEnvThreads) void k_actor_tail(ActorTail a) {
  const int64_t i = blockIdx.x;
  const int64_t t = *a.t_dev;
  int64_t act = 0;
  if (threadIdx.x == 0) {
    if constexpr (MAXL > 0) {
      const uint64_t ctr = (uint64_t)t;
      const double u = philox_uniform(a.seed, ctr, (uint32_t)i, STREAM_EXPLORE);
      float r[MAXL], q[MAXL];
      load_row(a.q + i * (a.A + 1), a.A + 1, r);  // issued before the exploration branch
      if (u < a.eps[i]) {
        uint32_t c[4] = {(uint32_t)i, (uint32_t)ctr, (uint32_t)(ctr >> 32), STREAM_RANDACT};
        philox4x32(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
        act = (int64_t)(((uint64_t)c[0] * (uint64_t)a.A) >> 32);
      } else {
        q_row_reg(r, a.A, 1, q);
        act = argmax_first_reg(q, a.A);
      }
    } else {
      act = eps_greedy_one(a.q, i, a.A, 1, a.eps, nullptr, nullptr, a.seed, (uint64_t)t);
    }
    a.action[i] = act;
  } else if (threadIdx.x == 64 && a.td_abs) {  // another wave: the previous row's |td|
    const int A1 = a.A + 1;
    const float *q0 = a.qcache + a.prev_s0[i] * A1, *q1 = a.qcache + a.prev_s1[i] * A1;
    float l, td;
    if constexpr (MAXL > 0)
      td = td_huber_row_reg<MAXL>(q0, q1, q1, a.prev_a[i], a.prev_r[i], a.prev_done[i], 1.0f, 0, a.A, 1, a.gamma_n, 1,
                                  &l);
    else
      td = td_huber_row(q0, q1, q1, a.prev_a + i, a.prev_r + i, a.prev_done + i, nullptr, 0, a.A, 1, a.gamma_n, 1,
                        1.0f, &l, nullptr);
    a.td_abs[i] = fabsf(td);
  }
  const EnvOut e = env_step_one(a.frames, a.ring, t, i, a.cur_slot, a.seed, a.p_reward, a.p_done, a.r_out, a.done_out,
                                a.s0_h, a.s1_h, !a.ext_frames);
  if (threadIdx.x == 0)
    nstep_push_one(a.ns, i, a.n, a.gamma, a.mode, e.s0h, act, e.reward, e.s1h, e.done ? 1.0f : 0.0f, a.emit,
                   a.row_s0, a.row_a, a.row_r, a.row_s1, a.row_done);
}

__global__ __launch_bounds__(kEnvThreads) void k_env_reset(uint8_t *frames, int ring, uint64_t seed,
                                                           int64_t *cur_slot) {
  const int64_t i = blockIdx.x;
  uint4 *dr = reinterpret_cast<uint4 *>(frames + (i * ring + 1) * (int64_t)(4 * kFrameBytes));
  for (int v = threadIdx.x; v < kStackVec; v += kEnvThreads) dr[v] = env_bytes(seed, i, 0, 1, v % kFrameVec);
  if (threadIdx.x == 0) cur_slot[i] = 1;
}


// out[0..k) = vals[i] for the i < n with flag[i] != 0, in order of i; out[k..cap) = fill;
// *count_out = base + k.  One workgroup, per 1024-entry chunk: each wave's flags as a 64-bit
// ballot (a lane's rank among the wave's flagged lanes = the popcount of the lower bits), the
// 16 wave counts prefixed through LDS -- one barrier per chunk instead of a 10-step block scan
// with two barriers a step; the flag and the value of every lane are loaded together.
constexpr int kCompactThreads = 1024;
__global__ __launch_bounds__(kCompactThreads) void k_compact_flagged(const float *__restrict__ flag,
                                                                    const int64_t *__restrict__ vals, int64_t n,
                                                                    int64_t *__restrict__ out, int64_t cap,
                                                                    int64_t fill, int64_t base,
                                                                    int64_t *__restrict__ count_out) {
  constexpr int W = kCompactThreads / 64;
  __shared__ int wcount[2][W];  // double-buffered: chunk c's counts stay readable while c + 1 writes
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t k = 0;
  int buf = 0;
  for (int64_t c0 = 0; c0 < n; c0 += kCompactThreads, buf ^= 1) {
    const int64_t i = c0 + tid, ic = i < n ? i : n - 1;  // past n: a duplicate load, never flagged
    const float fv = flag[ic];
    const int64_t v = vals[ic];
    const bool f = i < n && fv != 0.0f;
    const uint64_t bal = __ballot(f);
    const int below = __popcll(bal & ((uint64_t(1) << lane) - 1));
    if (lane == 0) wcount[buf][wave] = __popcll(bal);
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const int cw = wcount[buf][w];
      before += w < wave ? cw : 0;
      total += cw;
    }
    const int64_t pos = k + before + below;
    if (f && pos < cap) out[pos] = v;
    k += total;
  }
  const int64_t kk = k < cap ? k : cap;
  for (int64_t j = kk + tid; j < cap; j += kCompactThreads) out[j] = fill;
  if (tid == 0) *count_out = base + kk;
}

}  // namespace rth

using namespace rth;

struct rth_nstep {
  int64_t N;
  int32_t n;
  double gamma;
  int32_t mode;
  int device;
  void *mem;
  NStepState st;
};

// the actor step's first launch: the step counter (what ε-greedy and the env step read) and
// the acting stacks' frame-ring rows, rows[i] = i * ring + cur_slot[i] (was two launches)
__global__ __launch_bounds__(256) void k_actor_prologue(int64_t *t, const int64_t *__restrict__ cur_slot, int64_t n,
                                                        int64_t ring, int64_t *__restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) rows[i] = i * ring + cur_slot[i];
  if (i == 0) *t += 1;
}

extern "C" {

int rth_eps_greedy(const float *q, int64_t N, int64_t A, int32_t dueling, const double *eps, const double *u,
                   const int64_t *ra, uint64_t seed, uint64_t counter, const int64_t *counter_dev, int64_t *out,
                   void *stream) {
  RTH_REQUIRE(N >= 0 && A >= 1 && A <= kMaxActions && (dueling == 0 || dueling == 1), "rth_eps_greedy: bad shape");
  if (N == 0) return RTH_OK;
  RTH_REQUIRE(q && eps && out, "rth_eps_greedy: NULL buffer");
  const int bs = 256;
  hipLaunchKernelGGL(k_eps_greedy, dim3((unsigned)((N + bs - 1) / bs)), dim3(bs), 0, as_stream(stream), q, N,
                     (int)A, (int)dueling, eps, u, ra, seed, counter, counter_dev, out);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_nstep_create(int64_t N, int32_t n, double gamma, int32_t mode, int device, rth_nstep **out) {
  RTH_REQUIRE(out && N >= 1 && n >= 1 && n <= 64 && (mode == 0 || mode == 1), "rth_nstep_create: bad arguments");
  RTH_HIP(hipSetDevice(device));
  const size_t slots = (size_t)N * n;
  const size_t bytes = N * sizeof(int32_t) + slots * (3 * sizeof(int64_t) + 2 * sizeof(float)) + 64;
  void *mem = nullptr;
  if (hipMalloc(&mem, bytes) != hipSuccess) {
    set_error("rth_nstep_create: hipMalloc(%zu) failed", bytes);
    return RTH_ERR_NOMEM;
  }
  RTH_HIP(hipMemset(mem, 0, bytes));
  auto *h = new rth_nstep{N, n, gamma, mode, device, mem, {}};
  uint8_t *p = (uint8_t *)mem;
  h->st.s0 = (int64_t *)p;
  p += slots * 8;
  h->st.a = (int64_t *)p;
  p += slots * 8;
  h->st.s1 = (int64_t *)p;
  p += slots * 8;
  h->st.r = (float *)p;
  p += slots * 4;
  h->st.done = (float *)p;
  p += slots * 4;
  h->st.count = (int32_t *)p;
  *out = h;
  return RTH_OK;
}

int rth_nstep_destroy(rth_nstep *h) {
  if (!h) return RTH_OK;
  (void)hipSetDevice(h->device);
  (void)hipFree(h->mem);
  delete h;
  return RTH_OK;
}

int rth_nstep_reset(rth_nstep *h, void *stream) {
  RTH_REQUIRE(h, "rth_nstep_reset: NULL handle");
  RTH_HIP(hipMemsetAsync(h->st.count, 0, h->N * sizeof(int32_t), as_stream(stream)));
  return RTH_OK;
}

int rth_nstep_push(rth_nstep *h, const int64_t *s0, const int64_t *a, const float *r, const int64_t *s1,
                   const float *done, int32_t *emit, int64_t *s0_out, int64_t *a_out, float *r_out, int64_t *s1_out,
                   float *done_out, void *stream) {
  RTH_REQUIRE(h && s0 && a && r && s1 && done && emit && s0_out && a_out && r_out && s1_out && done_out,
              "rth_nstep_push: NULL argument");
  const int bs = 256;
  hipLaunchKernelGGL(k_nstep_push, dim3((unsigned)((h->N + bs - 1) / bs)), dim3(bs), 0, as_stream(stream), h->st,
                     h->N, h->n, h->gamma, h->mode, s0, a, r, s1, done, emit, s0_out, a_out, r_out, s1_out,
                     done_out);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_synth_env_step(uint8_t *frames, int64_t N, int32_t ring, int64_t t, const int64_t *t_dev, int64_t *cur_slot,
                       const int64_t * /*action: the synthetic dynamics ignore it*/, uint64_t seed, float p_reward,
                       float p_done, float *r_out, float *done_out, int64_t *s0_h, int64_t *s1_h, void *stream) {
  RTH_REQUIRE(frames && cur_slot && r_out && done_out && s0_h && s1_h, "rth_synth_env_step: NULL argument");
  RTH_REQUIRE(N >= 1 && N < (int64_t(1) << 31) && ring >= 4 && (t >= 1 || t_dev), "rth_synth_env_step: bad shape");
  hipLaunchKernelGGL(k_env_step, dim3((unsigned)N), dim3(kEnvThreads), 0, as_stream(stream), frames, ring, t, t_dev,
                     cur_slot, seed, p_reward, p_done, r_out, done_out, s0_h, s1_h, 1);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_synth_env_reset(uint8_t *frames, int64_t N, int32_t ring, uint64_t seed, int64_t *cur_slot, void *stream) {
  RTH_REQUIRE(frames && cur_slot && N >= 1 && ring >= 4, "rth_synth_env_reset: bad arguments");
  hipLaunchKernelGGL(k_env_reset, dim3((unsigned)N), dim3(kEnvThreads), 0, as_stream(stream), frames, ring, seed,
                     cur_slot);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_compact_flagged(const float *flag, const int64_t *vals, int64_t n, int64_t *out, int64_t cap, int64_t fill,
                        int64_t base, int64_t *count_out, void *stream) {
  RTH_REQUIRE((n == 0 || (flag && vals)) && (cap == 0 || out) && count_out && n >= 0 && cap >= 0,
              "rth_compact_flagged: bad arguments");
  hipLaunchKernelGGL(k_compact_flagged, dim3(1), dim3(kCompactThreads), 0, as_stream(stream), flag, vals, n, out, cap,
                     fill, base, count_out);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_actor_prologue(int64_t *t_dev, const int64_t *cur_slot, int64_t n, int64_t ring, int64_t *rows_out,
                       void *stream) {
  RTH_REQUIRE(t_dev && cur_slot && rows_out && n >= 1 && ring >= 1, "rth_actor_prologue: bad arguments");
  hipLaunchKernelGGL(k_actor_prologue, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), t_dev,
                     cur_slot, n, ring, rows_out);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_actor_tail(rth_nstep *h, const rth_actor_tail_args *x, int32_t *emit, int64_t *s0_out, int64_t *a_out,
                   float *r_out, int64_t *s1_out, float *done_out, void *stream) {
  RTH_REQUIRE(h && x && emit && s0_out && a_out && r_out && s1_out && done_out, "rth_actor_tail: NULL argument");
  RTH_REQUIRE(x->q && x->eps && x->t_dev && x->action && x->frames && x->cur_slot && x->r_out && x->done_out &&
                  x->s0_h && x->s1_h && (!x->td_abs || (x->qcache && x->prev_s0 && x->prev_a && x->prev_s1 &&
                                                         x->prev_r && x->prev_done)),
              "rth_actor_tail: NULL field");
  RTH_REQUIRE(x->N == h->N && x->N < (int64_t(1) << 31) && x->ring >= 4 && x->A >= 1 && x->A <= kMaxActions,
              "rth_actor_tail: bad shape (N %lld, adder N %lld, ring %d, A %d)", (long long)x->N, (long long)h->N,
              x->ring, x->A);
  ActorTail a{x->q, x->eps, x->seed, x->t_dev, x->action, x->qcache, x->prev_s0, x->prev_a, x->prev_s1,
              x->prev_r, x->prev_done, x->gamma_n, x->td_abs, x->frames, x->ring, x->cur_slot, x->p_reward,
              x->p_done, x->r_out, x->done_out, x->s0_h, x->s1_h, h->st, h->n, h->gamma, h->mode, emit,
              s0_out, a_out, s1_out, r_out, done_out, x->A, x->ext_frames};
  if (x->A + 1 <= 8)  // Atari's minimal action sets (Pong 6, Breakout 4)
    hipLaunchKernelGGL(k_actor_tail<8>, dim3((unsigned)x->N), dim3(kEnvThreads), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(k_actor_tail<0>, dim3((unsigned)x->N), dim3(kEnvThreads), 0, as_stream(stream), a);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
