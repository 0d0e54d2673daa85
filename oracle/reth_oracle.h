/*
 * reth_oracle.h -- CPU restatement of the Reth Ape-X DQN replay/update hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.
 * Parity pinned against golden vectors generated from the reference itself
 * (tests/golden/make_golden.py writes tests/golden/ fixtures).
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * sosp2021/Reth checkout).  Arithmetic follows the reference's operation order and
 * precision exactly (fp64 tree, f32 priorities/TD), compiled without FP contraction.
 */
#ifndef RETH_ORACLE_H
#define RETH_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- in-order heap sum-tree: reth_buffer/reth_buffer/utils/sumtree.py ---- */
void orc_tree_maintain_node(int64_t cap, double *sum, double *mn, const double *val, int64_t i); /* :5-21 */
void orc_tree_maintain(int64_t cap, double *sum, double *mn, const double *val, int64_t i);      /* :24-31 */
void orc_tree_update(int64_t cap, double *sum, double *mn, double *val, const int64_t *idx,
                     const double *w, int64_t n);                                                /* :61-67 */
int64_t orc_tree_find(int64_t cap, const double *sum, const double *val, double weight);         /* :34-58 */
void orc_tree_sample(int64_t cap, const double *sum, const double *val, int64_t batch,
                     const double *uniforms, int64_t *idx_out, double *val_out);                 /* :70-79 */
double orc_tree_min(const double *sum, const double *mn);                                        /* :109-110 */

/* ---- PER sampler: reth_buffer/reth_buffer/sampler/per_sampler.py ---- */
void orc_per_normalize(const float *w, int64_t n, float alpha, float *out);                      /* :16-17 */
void orc_per_normalize64(const double *w, int64_t n, double alpha, double *out);               /* f8 input */
void orc_per_is_weights(const double *p, int64_t n, double tree_min, double beta, double *out);  /* :24-28 */

/* ---- Schedule: reth_buffer/reth_buffer/utils/schedule.py:4-52 (method 0 = linear, 1 = exp) ---- */
double orc_schedule_value(int method, double start, double end, int64_t max_steps, int64_t step);

/* ---- FIFOPolicy.get_indices: reth_buffer/reth_buffer/cache_policy/fifo_policy.py:11-18 ---- */
void orc_fifo_indices(int64_t cap, int64_t *tail, int64_t n, int32_t *out);

/* ---- NStepAdder.push: reth/reth/utils/nstep_adder.py:11-28 ----
 * One adder per actor.  Rows carry integer frame handles for s0/s1 (the frames
 * themselves are referenced, never copied, exactly like the reference's list items).
 * mode 0 = numpy 1.19 scalar promotion (t_gamma*r in f64, cast back to f32 by +=; the
 *          reference's pinned numpy, poetry.lock:249-250)
 * mode 1 = numpy >= 2 / NEP 50 (product stays f32). */
#define ORC_NSTEP_MAX 16
typedef struct {
  int32_t n, count;
  int64_t s0[ORC_NSTEP_MAX], a[ORC_NSTEP_MAX], s1[ORC_NSTEP_MAX];
  float r[ORC_NSTEP_MAX], done[ORC_NSTEP_MAX];
} orc_nstep_state;
void orc_nstep_init(orc_nstep_state *st, int32_t n);
/* returns 1 and fills *_out when a row is emitted (the popped oldest row), else 0 */
int orc_nstep_push(orc_nstep_state *st, double gamma, int mode, int64_t s0, int64_t a, float r,
                   int64_t s1, float done, int64_t *s0_out, int64_t *a_out, float *r_out,
                   int64_t *s1_out, float *done_out);

/* ---- DQN TD error / Huber: reth/reth/algorithm/dqn/dqn_solver.py ---- */
int64_t orc_argmax_first(const float *q, int64_t A);  /* torch.argmax: first max, NaN is max */
/* _calc_td_error :68-98 (q_s1_online ignored when double_q == 0) */
void orc_td_error(const float *q_s0, const float *q_s1_online, const float *q_s1_target,
                  const int64_t *a, const float *r, const float *done, int64_t B, int64_t A,
                  float gamma_n, int double_q, float *td);
/* update :104-124: smooth_l1(td, 0, beta=1) * w, mean; dq = d(loss)/d(q_s0) as autograd
 * forms it (mean -> mul(w) -> smooth_l1 backward -> sum(q*onehot) backward).
 * w may be NULL (no IS weights). Returns the mean loss (fp32, sequential sum). */
float orc_td_huber(const float *td, const float *w, const int64_t *a, int64_t B, int64_t A,
                   float *loss_elem, float *dq);

/* ---- epsilon-greedy: reth/reth/utils/exploration.py:26-31 + dqn_solver.py:126-131 ---- */
void orc_eps_greedy(const float *q, int64_t N, int64_t A, const double *eps, const double *u,
                    const int64_t *rand_action, int64_t *action_out);

/* ---- Philox4x32-10 (Salmon et al., SC'11): the product's device RNG, restated so the
 * device-RNG paths can be checked bit-exactly too. ---- */
void orc_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_philox_uniform(uint64_t seed, uint64_t counter, uint32_t lane, uint32_t stream);
/* stream ids shared with the device code */
#define RTH_STREAM_SAMPLE 1u
#define RTH_STREAM_EXPLORE 2u
#define RTH_STREAM_RANDACT 3u
#define RTH_STREAM_ENV 4u

#ifdef __cplusplus
}
#endif
#endif
