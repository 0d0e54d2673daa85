/*
 * reth_oracle.c -- CPU restatement of the Reth Ape-X DQN hot path (see reth_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker and the bench's CPU baseline ("port").
 * The product (reth_amd/, libreth_hip.so) never links or calls this.
 *
 * Built with -O2 -ffp-contract=off -fno-fast-math so every f32/f64 operation rounds
 * exactly where the reference's numpy/numba/torch code rounds.
 */
#include "reth_oracle.h"

#include <math.h>
#include <string.h>

/* ------------------------------------------------------------------ sum-tree */

/* reth_buffer/reth_buffer/utils/sumtree.py:5-21 (_numba_maintain_node).
 * sum = val + sum[l] + sum[r] in that order; min seeded with val (or 1 if val == 0);
 * children whose min is 0 (never maintained) are skipped. */
void orc_tree_maintain_node(int64_t cap, double *sum, double *mn, const double *val, int64_t i) {
  int64_t l = 2 * i + 1, r = 2 * i + 2;
  double s = val[i];
  double m = val[i] != 0.0 ? val[i] : 1.0;
  if (l < cap) {
    s += sum[l];
    if (mn[l] != 0.0) m = (mn[l] < m) ? mn[l] : m; /* python min(m, x): keeps m unless x < m */
  }
  if (r < cap) {
    s += sum[r];
    if (mn[r] != 0.0) m = (mn[r] < m) ? mn[r] : m;
  }
  sum[i] = s;
  mn[i] = m;
}

/* sumtree.py:24-31 (_numba_maintain): node, then every ancestor up to the root */
void orc_tree_maintain(int64_t cap, double *sum, double *mn, const double *val, int64_t i) {
  int64_t cur = i;
  for (;;) {
    orc_tree_maintain_node(cap, sum, mn, val, cur);
    if (cur == 0) break;
    cur = (cur - 1) / 2;
  }
}

/* sumtree.py:61-67 (_numba_update): sequential, last writer wins on duplicates */
void orc_tree_update(int64_t cap, double *sum, double *mn, double *val, const int64_t *idx,
                     const double *w, int64_t n) {
  for (int64_t k = 0; k < n; ++k) {
    val[idx[k]] = w[k];
    orc_tree_maintain(cap, sum, mn, val, idx[k]);
  }
}

/* sumtree.py:34-58 (_numba_find_index): in-order descent (left subtree, node, right
 * subtree) with the +1e-5 slack at the node test. */
int64_t orc_tree_find(int64_t cap, const double *sum, const double *val, double weight) {
  int64_t cur = 0;
  for (;;) {
    int64_t l = cur * 2 + 1, r = cur * 2 + 2;
    if (l < cap) {
      if (weight < sum[l]) {
        cur = l;
        continue;
      }
      weight -= sum[l];
    }
    if (weight < val[cur] + 1e-5) return cur;
    weight -= val[cur];
    if (r >= cap) return cur;
    cur = r;
  }
}

/* sumtree.py:70-79 (_numba_sample): seg = sum[0]/B, t_i = (i + U_i) * seg.
 * U is numba's np.random.random_sample stream in the reference; here it is an input. */
void orc_tree_sample(int64_t cap, const double *sum, const double *val, int64_t batch,
                     const double *uniforms, int64_t *idx_out, double *val_out) {
  double seg = sum[0] / (double)batch;
  for (int64_t i = 0; i < batch; ++i) {
    double t = ((double)i + uniforms[i]) * seg;
    int64_t k = orc_tree_find(cap, sum, val, t);
    idx_out[i] = k;
    val_out[i] = val[k];
  }
}

/* sumtree.py:109-110 (NumbaSumTree.min) */
double orc_tree_min(const double *sum, const double *mn) { return sum[0] != 0.0 ? mn[0] : 1.0; }

/* ------------------------------------------------------------------ PER */

/* reth_buffer/reth_buffer/sampler/per_sampler.py:16-17: (w + 1e-6) ** alpha in float32.
 * numpy evaluates `f32_array ** 0.5` as sqrt (fast_scalar_power), correctly rounded on
 * every platform.  For other exponents numpy's own f32 power is platform dependent
 * (glibc powf under the reference's numpy 1.19 pin, SVML under numpy >= 1.22 on AVX512);
 * this restatement and the device kernel both use the correctly rounded f32 power. */
void orc_per_normalize(const float *w, int64_t n, float alpha, float *out) {
  const float eps = 1e-6f;
  for (int64_t k = 0; k < n; ++k) {
    float x = w[k] + eps;
    if (alpha == 0.5f)
      out[k] = sqrtf(x);
    else if (alpha == 1.0f)
      out[k] = x;
    else
      out[k] = (float)pow((double)x, (double)alpha);
  }
}

/* the same on a float64 array: numpy computes in f64 (`** 0.5` -> sqrt) */
void orc_per_normalize64(const double *w, int64_t n, double alpha, double *out) {
  for (int64_t k = 0; k < n; ++k) {
    double x = w[k] + 1e-6;
    out[k] = alpha == 0.5 ? sqrt(x) : (alpha == 1.0 ? x : pow(x, alpha));
  }
}

/* per_sampler.py:24-28: (p / tree.min()) ** (-beta), float64 */
void orc_per_is_weights(const double *p, int64_t n, double tree_min, double beta, double *out) {
  for (int64_t k = 0; k < n; ++k) out[k] = pow(p[k] / tree_min, -beta);
}

/* ------------------------------------------------------------------ Schedule */

/* reth_buffer/reth_buffer/utils/schedule.py:29-40 (the lambdas), python float order:
 * linear: start + (end - start) * step / max_steps  ==  start + (((end-start)*step)/max)
 * exp:    end - (end - start) * exp(-1 * step / max_steps) */
double orc_schedule_value(int method, double start, double end, int64_t max_steps, int64_t step) {
  if (step > max_steps) step = max_steps; /* value(step) clamps; step() stops at max */
  if (method == 0) return start + ((end - start) * (double)step) / (double)max_steps;
  return end - (end - start) * exp((-1.0 * (double)step) / (double)max_steps);
}

/* ------------------------------------------------------------------ FIFO */

/* reth_buffer/reth_buffer/cache_policy/fifo_policy.py:11-18 */
void orc_fifo_indices(int64_t cap, int64_t *tail, int64_t n, int32_t *out) {
  for (int64_t k = 0; k < n; ++k) {
    out[k] = (int32_t)*tail;
    *tail = (*tail + 1) % cap;
  }
}

/* ------------------------------------------------------------------ n-step */

void orc_nstep_init(orc_nstep_state *st, int32_t n) {
  memset(st, 0, sizeof(*st));
  st->n = n;
}

/* reth/reth/utils/nstep_adder.py:11-28.  Position 0 is the newest row (appendleft);
 * the emitted row is the oldest (pop from the right) BEFORE the new reward is folded in. */
int orc_nstep_push(orc_nstep_state *st, double gamma, int mode, int64_t s0, int64_t a, float r,
                   int64_t s1, float done, int64_t *s0_out, int64_t *a_out, float *r_out,
                   int64_t *s1_out, float *done_out) {
  int emitted = 0;
  if (st->count == st->n) {
    int k = st->count - 1;
    *s0_out = st->s0[k];
    *a_out = st->a[k];
    *r_out = st->r[k];
    *s1_out = st->s1[k];
    *done_out = st->done[k];
    st->count--;
    emitted = 1;
  }
  double t_gamma = gamma;
  for (int k = 0; k < st->count; ++k) {
    if (st->done[k] != 0.0f) break;
    if (mode == 0)
      st->r[k] = (float)((double)st->r[k] + t_gamma * (double)r);
    else
      st->r[k] = st->r[k] + (float)t_gamma * r;
    t_gamma *= gamma;
    st->s1[k] = s1;
  }
  for (int k = st->count; k > 0; --k) {
    st->s0[k] = st->s0[k - 1];
    st->a[k] = st->a[k - 1];
    st->r[k] = st->r[k - 1];
    st->s1[k] = st->s1[k - 1];
    st->done[k] = st->done[k - 1];
  }
  st->s0[0] = s0;
  st->a[0] = a;
  st->r[0] = r;
  st->s1[0] = s1;
  st->done[0] = done;
  st->count++;
  return emitted;
}

/* ------------------------------------------------------------------ DQN TD */

int64_t orc_argmax_first(const float *q, int64_t A) {
  int64_t best = 0;
  float bv = q[0];
  for (int64_t j = 1; j < A; ++j) {
    float v = q[j];
    if (isnan(bv)) break;
    if (isnan(v) || v > bv) {
      bv = v;
      best = j;
    }
  }
  return best;
}

/* reth/reth/algorithm/dqn/dqn_solver.py:68-98.
 *   q   = sum(q_s0 * one_hot(a))                        (:79-81)
 *   a*  = argmax(Q_online(s1)) if double_q else argmax(Q_target(s1))   (:83-94)
 *   y   = r + (gamma**n * q_tgt(s1)[a*]) * (1 - done)  (:96; python float gamma**n -> f32)
 *   td  = q - y                                         (:97) */
void orc_td_error(const float *q_s0, const float *q_s1_online, const float *q_s1_target,
                  const int64_t *a, const float *r, const float *done, int64_t B, int64_t A,
                  float gamma_n, int double_q, float *td) {
  for (int64_t b = 0; b < B; ++b) {
    float q = q_s0[b * A + a[b]];
    const float *sel = double_q ? q_s1_online + b * A : q_s1_target + b * A;
    int64_t astar = orc_argmax_first(sel, A);
    float nqb = q_s1_target[b * A + astar];
    float t = gamma_n * nqb;
    t = t * (1.0f - done[b]);
    float y = r[b] + t;
    td[b] = q - y;
  }
}

/* dqn_solver.py:111-115 forward (F.smooth_l1_loss beta=1, *= w, mean) and the autograd
 * backward to q_s0: d/dtd smooth_l1 = x (|x|<1) or sign(x), scaled by w/B, scattered by
 * the one-hot.  torch evaluates x * ((1/B) * w); 1/B is a power of two for the batch
 * sizes used, so the product rounds once either way. */
float orc_td_huber(const float *td, const float *w, const int64_t *a, int64_t B, int64_t A,
                   float *loss_elem, float *dq) {
  float acc = 0.0f;
  const float invB = 1.0f / (float)B;
  for (int64_t b = 0; b < B; ++b) {
    float x = td[b];
    float z = fabsf(x);
    float l = z < 1.0f ? 0.5f * z * z : z - 0.5f;
    float wb = w ? w[b] : 1.0f;
    if (w) l = l * wb;
    if (loss_elem) loss_elem[b] = l;
    acc += l;
    if (dq) {
      float g = invB * wb;
      float d = x <= -1.0f ? -g : (x >= 1.0f ? g : x * g);
      for (int64_t j = 0; j < A; ++j) dq[b * A + j] = d * (j == a[b] ? 1.0f : 0.0f);
    }
  }
  return acc / (float)B;
}

/* ------------------------------------------------------------------ epsilon-greedy */

/* reth/reth/utils/exploration.py:26-31: rand() < eps -> action_space.sample(), else
 * solver.act(state) = argmax Q (dqn_solver.py:126-131). */
void orc_eps_greedy(const float *q, int64_t N, int64_t A, const double *eps, const double *u,
                    const int64_t *rand_action, int64_t *action_out) {
  for (int64_t i = 0; i < N; ++i)
    action_out[i] = (u[i] < eps[i]) ? rand_action[i] : orc_argmax_first(q + i * A, A);
}

/* ------------------------------------------------------------------ Philox4x32-10 */

static inline uint32_t mulhi32(uint32_t a, uint32_t b, uint32_t *lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *lo = (uint32_t)p;
  return (uint32_t)(p >> 32);
}

void orc_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int rnd = 0; rnd < 10; ++rnd) {
    if (rnd) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint32_t lo0, lo1;
    uint32_t hi0 = mulhi32(0xD2511F53u, c0, &lo0);
    uint32_t hi1 = mulhi32(0xCD9E8D57u, c2, &lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* u in [0,1) with 53 random bits: counter = {lane, call lo, call hi, stream}, key = seed */
double orc_philox_uniform(uint64_t seed, uint64_t counter, uint32_t lane, uint32_t stream) {
  uint32_t ctr[4] = {lane, (uint32_t)counter, (uint32_t)(counter >> 32), stream};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  orc_philox4x32(ctr, key, o);
  uint64_t bits = ((uint64_t)o[0] | ((uint64_t)o[1] << 32)) >> 11;
  return (double)bits * (1.0 / 9007199254740992.0);
}
