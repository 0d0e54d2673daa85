/*
 * reth_hip.h -- C ABI of libreth_hip.so, the MI355X (gfx950) hot path of Reth's Ape-X DQN
 * rollout -> prioritized replay -> update loop.
 *
 * Conventions
 *   - every call returns int: 0 (RTH_OK) or a negative RTH_ERR_*; rth_last_error() gives the
 *     message of the last failure on the calling thread.
 *   - pointers named *_dev are device (HBM) pointers; everything else is host memory.
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream); all work
 *     is enqueued asynchronously on it, no call synchronises the device.
 *   - handles own their device storage; calls on one handle must be serialised by the
 *     caller (the reference's single-owner sampler process, server/sampler_loop.py:6-42).
 *   - index arrays are int64 (the reference mixes int32 appends, fifo_policy.py:13, and
 *     int64 updates; both widen losslessly).
 *
 * The reference is pure Python (numba/numpy/torch); each entry point names the Python
 * interface it replaces (paths relative to the sosp2021/Reth checkout).  The Python
 * binding (reth_amd/_lib.py, ctypes) re-exposes the reference's own signatures.
 */
#ifndef RETH_HIP_H
#define RETH_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTH_OK 0
#define RTH_ERR_INVALID -1   /* bad argument (the reference's `assert`s) */
#define RTH_ERR_HIP -2       /* a HIP runtime call failed */
#define RTH_ERR_NOMEM -3     /* device allocation failed */

/* element types of replay columns */
#define RTH_U8 0
#define RTH_I32 1
#define RTH_I64 2
#define RTH_F32 3
#define RTH_F64 4
#define RTH_MAX_COLS 8
/* priority "dtype" for the tree/replay update calls: float64 priorities stored as given,
 * without (w + 1e-6) ** alpha (NumbaSumTree.update; reth.buffer.PrioritizedBuffer.append) */
#define RTH_PRIO_RAW 16
/* in_dtype of a frame-stack column of a frame-store replay: each stored row is out_planes
 * int32 frame ids into the replay's frame store (rth_replay_frames_attach); row_elems is the
 * sampled stack (out_planes frames x frame bytes, out_dtype RTH_U8), assembled by the gather */
#define RTH_FRAMES 8

const char *rth_last_error(void);
/* how many tree-update top passes timed out waiting for their subtree workgroups since the
 * library was loaded (the concurrent top workgroup's bounded wait; a timed-out pass leaves the
 * levels above the subtree roots unwritten rather than maintaining them from stale sums).
 * Expected 0; the tests assert it. */
int rth_tree_update_timeouts(int64_t *out);
/* development aid (a library built with -DRTH_CLOCK_STAMPS only; the product build returns an
 * error): per workgroup of the last fp32-MFMA conv launch (k_conv_bias_relu), the shader-clock
 * and 100 MHz wall-clock ticks around wave 0's work -- out[2 i], out[2 i + 1] for workgroups
 * i < slots <= 1024 -- whose ratio is the in-kernel clock */
int rth_debug_conv_clock(unsigned long long *out, int32_t slots);
/* library build/ABI version (major*10000 + minor*100 + patch) */
int rth_version(void);
/* the source tree the library was compiled from: 40 hex digits, the SHA-1 over the lines
 * "<git blob id> <path>\n" of reth_amd/csrc/ and include/reth_hip.h in path order
 * (reth_amd._lib.source_build_id; reproducible from `git ls-tree -r HEAD`) */
const char *rth_build_id(void);
/* hipGraphUpload of a captured graph's executable on `stream` (plumbing for the captured
 * actor / learner blocks, reth_amd.apex.ApexDQN.upload_graphs: a graph's first launch then
 * carries no upload) */
int rth_graph_upload(void *graph_exec, void *stream);
/* The number of nodes the next operation captured on `stream` would depend on (0 at the start
 * of a capture and until something is captured), or -1 when the stream is not capturing:
 * ApexDQN's graph cuts skip a part that would be empty (two boundaries back to back). */
int rth_stream_capture_deps(void *stream);

/* ------------------------------------------------------------------------------------
 * In-order heap sum-tree, fp64, resident in HBM.
 * Replaces reth_buffer/reth_buffer/utils/sumtree.py:82-113 (NumbaSumTree and the numba
 * kernels _numba_maintain_node :5-21, _numba_maintain :24-31, _numba_find_index :34-58,
 * _numba_update :61-67, _numba_sample :70-79).  Bit-exact with the sequential reference.
 * ---------------------------------------------------------------------------------- */
typedef struct rth_sumtree rth_sumtree;
int rth_sumtree_create(int64_t capacity, int device, rth_sumtree **out); /* NumbaSumTree.__init__ :83-87 */
int rth_sumtree_destroy(rth_sumtree *t);
int rth_sumtree_clear(rth_sumtree *t, void *stream);                    /* NumbaSumTree.clear :98-101 */
/* NumbaSumTree.update :103-104 -> _numba_update: val[idx]=w, maintain, in order */
int rth_sumtree_update(rth_sumtree *t, const int64_t *idx_dev, const double *w_dev, int64_t n,
                       void *stream);
/* _numba_find_index :34-58, one target per element */
int rth_sumtree_find(rth_sumtree *t, const double *targets_dev, int64_t n, int64_t *idx_out_dev,
                     double *val_out_dev, void *stream);
/* NumbaSumTree.sample :112-113 -> _numba_sample :70-79.  uniforms_dev (n = batch) replaces
 * numba's internal np.random stream when non-NULL (the parity hook); when NULL the
 * uniforms come from Philox4x32-10(seed, counter). */
int rth_sumtree_sample(rth_sumtree *t, int64_t batch, const double *uniforms_dev, uint64_t seed,
                       uint64_t counter, int64_t *idx_out_dev, double *val_out_dev, void *stream);
/* out2_dev[0] = NumbaSumTree.sum() :106-107, out2_dev[1] = NumbaSumTree.min() :109-110 */
int rth_sumtree_stats(rth_sumtree *t, double *out2_dev, void *stream);
/* the three fp64 arrays of the reference layout (each [capacity], device) */
int rth_sumtree_export(rth_sumtree *t, double *sum_dev, double *min_dev, double *val_dev, void *stream);
int rth_sumtree_import(rth_sumtree *t, const double *sum_dev, const double *min_dev,
                       const double *val_dev, void *stream);
int64_t rth_sumtree_capacity(const rth_sumtree *t);

/* ------------------------------------------------------------------------------------
 * PER sampler on a sum-tree.  Replaces reth_buffer/reth_buffer/sampler/per_sampler.py:5-35.
 * Schedules (alpha/beta, utils/schedule.py) stay on the host; the current values are args.
 * ---------------------------------------------------------------------------------- */
/* PERSampler._normalize_weights :16-17: out = (w + 1e-6) ** alpha  (float32) */
int rth_per_normalize(const float *w_dev, int64_t n, float alpha, float *out_dev, void *stream);
/* PERSampler.update :34-35: tree.update(idx, _normalize_weights(td_abs)) fused in one pass.
 * td_abs_dev is float32 (td_dtype RTH_F32: normalised in f32 with (float)alpha, like numpy
 * on an f4 array) or float64 (RTH_F64: normalised in f64). */
int rth_per_update(rth_sumtree *t, const int64_t *idx_dev, const void *td_abs_dev, int32_t td_dtype,
                   int64_t n, double alpha, void *stream);
/* PERSampler.sample :24-28: (idx, (p / tree.min()) ** -beta) */
int rth_per_sample(rth_sumtree *t, int64_t batch, double beta, const double *uniforms_dev,
                   uint64_t seed, uint64_t counter, int64_t *idx_out_dev, double *isw_out_dev,
                   void *stream);

/* ------------------------------------------------------------------------------------
 * Replay shard in HBM: FIFO slot allocation + column storage + PER tree.
 * Replaces the reth_buffer service: append_loop (server/main_loop.py:21-61: deserialize,
 * FIFOPolicy.get_indices, LMDB put, forward to sampler), sampler_loop
 * (server/sampler_loop.py:6-42), Client.append / update_priorities (client/client.py:21-39)
 * and the loaders' row fetch (client/torch_cuda_loader.py:20-66, numpy_loader.py:27-51).
 * ---------------------------------------------------------------------------------- */
typedef struct {
  int64_t row_elems;  /* elements per row (product of the per-row shape) */
  int32_t in_dtype;   /* storage type == type appended (RTH_U8 ... RTH_F64) */
  int32_t out_dtype;  /* type produced on sample: == in_dtype, or RTH_F32 from RTH_U8 */
  int32_t out_planes; /* 0: same element order; k > 0 (RTH_U8 -> RTH_F32 only): the row is k
                         planes (C,H,W) and is produced channels-last (H,W,C) */
  int32_t reserved;
} rth_col_desc;

/* a column source for an append: rows[i] (or i when rows_dev == NULL) of base_dev, rows
 * row_stride_bytes apart (0 = dense).  src_dtype: element type of the source rows; 0 or the
 * column's storage type = as stored; RTH_F32 into a RTH_U8 column narrows whole-number
 * pixels 0..255 (frames the reference's actors send as float32, test/apex-dqn/worker.py:46-50) */
typedef struct {
  const void *base_dev;
  const int64_t *rows_dev;
  int64_t row_stride_bytes;
  int32_t src_dtype;
  int32_t reserved;
} rth_src;

/* A PERSampler schedule (reth_buffer/reth_buffer/utils/schedule.py:4-52):
 * const: start; linear: start + (end - start) * k / max_steps;
 * exp: end - (end - start) * exp(-k / max_steps); k = steps taken, clamped to max_steps. */
#define RTH_SCHED_CONST 0
#define RTH_SCHED_LINEAR 1
#define RTH_SCHED_EXP 2
typedef struct {
  int32_t method;
  int32_t reserved;
  double start;
  double end;
  int64_t max_steps;
} rth_schedule;

typedef struct rth_replay rth_replay;
/* Samplers of a shard (reth_buffer/reth_buffer/sampler/):
 *   RTH_SAMPLER_PER      PERSampler (per_sampler.py:5-35): sum-tree, IS weights;
 *   RTH_SAMPLER_UNIFORM  UniformSampler (uniform_sampler.py:6-25): updates append their
 *                        indices to a list until it holds `capacity`; a sample draws
 *                        list[floor(u * len)], weights 1;
 *   RTH_SAMPLER_FIFO     FIFOSampler (fifo_sampler.py:8-29): updates push (index, weight)
 *                        into a queue of at most `capacity` (oldest dropped); a sample pops
 *                        the `batch` oldest, weights as pushed. */
#define RTH_SAMPLER_PER 0
#define RTH_SAMPLER_UNIFORM 1
#define RTH_SAMPLER_FIFO 2
/* The shard owns its sampler state (per_sampler.py:5-12): the alpha / beta schedules and
 * the step count, the FIFO tail, the sample-call counter and the uniform list / FIFO queue
 * live in device memory, so every launch below is argument-invariant from step to step
 * (HIP-graph replayable). */
int rth_replay_create(int64_t capacity, int32_t n_cols, const rth_col_desc *cols, int32_t sampler,
                      const rth_schedule *alpha, const rth_schedule *beta, int device, uint64_t seed,
                      rth_replay **out);
int rth_replay_destroy(rth_replay *h);
/* Client.append + append_loop + PERSampler.update: rows go to FIFO slots
 * tail, tail+1, ... mod capacity (FIFOPolicy :11-18), priorities (td_abs + 1e-6)**alpha
 * into the tree.  idx_out_dev (nullable) receives the slots. */
int rth_replay_append(rth_replay *h, const rth_src *srcs, const void *td_abs_dev, int32_t td_dtype,
                      int64_t n, int64_t *idx_out_dev, void *stream);
/* sampler_loop sample + loader gather: PER-sample `batch` rows (uniforms_dev nullable, see
 * rth_sumtree_sample) with the current beta, write IS weights, and gather every column into
 * out_cols_dev[c] ([batch, row] of out_dtype; NULL = no gather) -- TorchCudaLoader.sample's
 * (data, indices, weights).  The sampler's device call counter (the Philox counter of the
 * next sample) is advanced by the gather kernel; with out_cols_dev NULL, by the next
 * rth_replay_gather on this handle, or else by the next sample before it draws. */
int rth_replay_sample(rth_replay *h, int64_t batch, const double *uniforms_dev,
                      void *const *out_cols_dev, int64_t *idx_out_dev, double *isw_out_dev,
                      void *stream);
/* Client.update_priorities :37-39 -> sampler_loop :31-35: step != 0 advances the alpha/beta
 * schedules first (PERSampler.on_step), then PERSampler.update */
int rth_replay_update_priorities(rth_replay *h, const int64_t *idx_dev, const void *td_abs_dev,
                                 int32_t td_dtype, int64_t n, int32_t step, void *stream);
/* The same, deferred (PER shards): the update is recorded and applied by the shard's next
 * tree launch -- merged into the next rth_replay_append's (one launch instead of two), or on
 * its own before a sample / immediate update / rth_replay_flush -- which is the order the
 * reference's sampler applies its messages in.  idx_dev / td_abs_dev must stay valid (and
 * unmodified) until then.  Host counters are updated at once.  Call rth_replay_flush before
 * reading the tree through rth_replay_tree. */
int rth_replay_update_priorities_deferred(rth_replay *h, const int64_t *idx_dev, const void *td_abs_dev,
                                          int32_t td_dtype, int64_t n, int32_t step, void *stream);
int rth_replay_flush(rth_replay *h, void *stream);
/* NumpyLoader row fetch (numpy_loader.py:381-396) for explicit indices */
int rth_replay_gather(rth_replay *h, const int64_t *idx_dev, int64_t n, void *const *out_cols_dev,
                      void *stream);
/* host mirrors of the service counters: rows stored, FIFO tail, sampler cnt (appended +
 * re-prioritised, sampler_loop.py:36), sample calls issued, schedule steps taken, and the
 * sampler's own length (PER: rows stored; uniform: list length; FIFO: queued entries --
 * FIFOSampler.ready_sample is len > batch) */
int rth_replay_info(const rth_replay *h, int64_t *size, int64_t *tail, int64_t *cnt,
                    int64_t *sample_calls, int64_t *sched_steps, int64_t *sampler_len);
/* uniform row draw of NumpyBuffer.sample (reth/reth/buffer/buffer.py:88-90,
 * np.random.choice(size, batch)): idx[i] = floor(u_i * size), u_i = uniforms_dev[i] or
 * Philox(seed, counter (or *counter_dev), i) */
int rth_uniform_indices(int64_t size, int64_t batch, const double *uniforms_dev, uint64_t seed, uint64_t counter,
                        const int64_t *counter_dev, int64_t *idx_out_dev, void *stream);
rth_sumtree *rth_replay_tree(rth_replay *h);
/* Live per-kernel timing (the bench's in-loop HBM rooflines; no reference counterpart):
 * events[2k] / events[2k+1] (hipEvent_t, nullable) are recorded on the launch stream right
 * before / after the next launch of kind k of this handle, once, then disarmed:
 *   RTH_TIMING_TREE_UPDATE  the append's tree launch (k_tree_update_sub: the append's
 *                           priorities + a deferred update_priorities)
 *   RTH_TIMING_SAMPLE       the PER sample (k_tree_sample + IS weights)
 *   RTH_TIMING_GATHER       the gather (k_copy_rows into the learner batch)
 *   RTH_TIMING_INSERT       the append's row copy (k_copy_rows into the FIFO slots)
 * n = number of events given (<= RTH_TIMING_SLOTS); n = 0 disarms all.  fired_out (nullable)
 * receives the bit mask of the slots whose events were recorded since the previous call. */
#define RTH_TIMING_TREE_UPDATE 0
#define RTH_TIMING_SAMPLE 2
#define RTH_TIMING_GATHER 4
#define RTH_TIMING_INSERT 6
#define RTH_TIMING_SLOTS 8
int rth_replay_set_timing(rth_replay *h, void *const *events, int32_t n, int32_t *fired_out);
/* device pointer of column c's storage ([capacity, row] of in_dtype) */
void *rth_replay_column(rth_replay *h, int32_t c);
/* Frame de-duplicated storage (Breakout's 4 M rows are 225.9 GB as full uint8
 * rows, ~30 GB with each frame stored once).  The reference stores every row's two float32
 * stacks (test/apex-dqn/worker.py:44-51); here the RTH_FRAMES columns hold each stack as K
 * frame ids into a frame store of n_frames frames of frame_bytes, owned by the handle, and
 * the gather assembles the same uint8 stacks the full rows would hold.  store_out / head_out
 * (nullable): the store ([n_frames, frame_bytes]) and its device head (frames pushed).  The
 * store is a ring: it must hold every frame a live row references -- a row's oldest frame is
 * at most n + 4 actor steps older than the row, and a row lives capacity / N appends, and a
 * step pushes at most 2 N frames -- so n_frames >= 2 capacity + 2 (n + 16) N with N actors
 * covers every episode-end pattern (reth_amd.apex.ApexDQN.frame_store_frames, "hard").
 * *head_out = the device word holding the next frame id (a second word after it is internal). */
int rth_replay_frames_attach(rth_replay *h, int64_t n_frames, int64_t frame_bytes, void **store_out,
                             int64_t **head_out);
/* One vectorised actor step's frames into the store (VecActors, after the env step):
 * ring_dev = the actors' stack ring [N * ring_slots (+ extra), stack, frame], sid_dev = its
 * stack table ([same stacks, stack] int32 frame ids).  mode 0: stack s1_h[i] is stack s0_h[i]
 * shifted by one frame + a new frame (FrameStack.step, reth/reth/env/util.py:198-204): the new
 * frame enters the store, sid[s1] = sid[s0][1:] + [its id]; where done_dev[i], actor i's reset
 * stack (slot cur_slot_dev[i], one frame `stack` times: FrameStack.reset, :191-196) enters as one
 * frame.  mode 1: every actor's current stack (slot cur_slot_dev[i]) enters as `stack` frames
 * (the initial observations).  Then the device head advances past them. */
int rth_replay_push_frames(rth_replay *h, const uint8_t *ring_dev, int64_t n, int32_t ring_slots, int32_t stack,
                           const int64_t *s0_h_dev, const int64_t *s1_h_dev, const float *done_dev,
                           const int64_t *cur_slot_dev, int32_t *sid_dev, int32_t mode, void *stream);
/* Frames in place (r05): on = 1 makes the gathers (rth_replay_gather / _sample with out_cols)
 * write each frame-stack column's stored id tuple (int32 [n][4], 16-byte aligned output)
 * instead of the assembled stack; rth_conv1_frames_* read the frames from the store by
 * them.  4-frame stacks only.  on = 0 restores the stacks. */
int rth_replay_frames_ids_out(rth_replay *h, int32_t on);

/* ------------------------------------------------------------------------------------
 * Row copy / gather with optional uint8 -> float32 widening (the loaders' pinned copy +
 * H2D, torch_cuda_loader.py:43-62, as one HBM->HBM kernel).  src/dst row index arrays are
 * nullable (identity).  Strides in bytes.  out_planes as in rth_col_desc (channels-last out).
 * ---------------------------------------------------------------------------------- */
int rth_copy_rows(void *dst_dev, int64_t dst_stride, const int64_t *dst_rows_dev, const void *src_dev,
                  int64_t src_stride, const int64_t *src_rows_dev, int64_t n, int64_t row_elems,
                  int32_t in_dtype, int32_t out_dtype, int32_t out_planes, void *stream);

/* ------------------------------------------------------------------------------------
 * Actor side.
 * ---------------------------------------------------------------------------------- */
/* dueling (rth_eps_greedy, rth_td_huber): q rows hold the network's raw heads -- A
 * advantages then the state value -- and Q = (V + A) - mean(A) is formed in-kernel
 * (dqn_model.py:185-193); rth_td_huber's dq is then d(loss)/d(heads) [B, A+1].  A <= 32. */
/* RandomExploration.act (reth/reth/utils/exploration.py:26-31) over N actors:
 * u < eps[i] ? rand_action : argmax_a q[i, a] (first maximum, dqn_solver.py:126-131).
 * u_dev / rand_action_dev nullable -> Philox(seed, counter); counter_dev (nullable) supplies
 * the counter from device memory instead (graph replay). */
int rth_eps_greedy(const float *q_dev, int64_t N, int64_t A, int32_t dueling, const double *eps_dev,
                   const double *u_dev, const int64_t *rand_action_dev, uint64_t seed,
                   uint64_t counter, const int64_t *counter_dev, int64_t *action_out_dev,
                   void *stream);
/* *counter_dev += delta (device-resident step counters) */
int rth_counter_add(int64_t *counter_dev, int64_t delta, void *stream);

/* NStepAdder (reth/reth/utils/nstep_adder.py:5-28), one adder per actor, rows referencing
 * frame handles.  mode 0 = numpy 1.19 promotion (reference pin), 1 = numpy 2 / NEP 50. */
typedef struct rth_nstep rth_nstep;
int rth_nstep_create(int64_t n_actors, int32_t n_step, double gamma, int32_t mode, int device,
                     rth_nstep **out);
int rth_nstep_destroy(rth_nstep *h);
int rth_nstep_reset(rth_nstep *h, void *stream);
/* push one transition per actor; emit_dev[i] = 1 when actor i's oldest row was popped, its
 * fields in the *_out arrays (row i) */
int rth_nstep_push(rth_nstep *h, const int64_t *s0_dev, const int64_t *a_dev, const float *r_dev,
                   const int64_t *s1_dev, const float *done_dev, int32_t *emit_dev,
                   int64_t *s0_out_dev, int64_t *a_out_dev, float *r_out_dev,
                   int64_t *s1_out_dev, float *done_out_dev, void *stream);

/* Synthetic Pong-shaped environment (no ALE on the box): uint8 (4,84,84) frame stacks kept
 * in a per-actor ring of `ring` stacks.  Step t writes the next stack (shift + one fresh
 * frame) into slot (2t) % ring and, on done, a reset stack (one fresh frame x4, FrameStack
 * reset) into slot (2t+1) % ring.  reward in {-1,0,+1}, P(+-1) = p_reward/2 each;
 * done ~ Bernoulli(p_done).  cur_slot_dev is updated in place; s0/s1 handles
 * (actor*ring + slot) are written for the n-step adder.  Actions do not affect it.
 * t_dev (nullable) supplies t from device memory (graph replay). */
int rth_synth_env_step(uint8_t *frames_dev, int64_t n_actors, int32_t ring, int64_t t,
                       const int64_t *t_dev, int64_t *cur_slot_dev, const int64_t *action_dev, uint64_t seed,
                       float p_reward, float p_done, float *r_out_dev, float *done_out_dev,
                       int64_t *s0_handle_dev, int64_t *s1_handle_dev, void *stream);
/* The tail of one fused actor step, one workgroup per actor: rth_eps_greedy (dueling heads,
 * Philox draws at counter *t_dev) on q, the previous n-step rows' |td| (rth_td_huber with
 * target == online, isw = 1) from the per-stack heads cache -- heads of stack h at
 * qcache[h * (A + 1)] --, rth_synth_env_step at t = *t_dev and rth_nstep_push of the new
 * transition into the row outputs; every value equals the one of those separate calls.
 * td_abs (nullable) skips the rows' |td|. */
typedef struct rth_actor_tail_args {
  const float *q;          /* acting heads [N, A + 1] */
  const double *eps;       /* [N] */
  const int64_t *t_dev;    /* env step / Philox counter */
  int64_t *action;         /* out [N] */
  const float *qcache;
  const int64_t *prev_s0, *prev_a, *prev_s1;
  const float *prev_r, *prev_done;
  float *td_abs;           /* out [N] */
  uint8_t *frames;
  int64_t *cur_slot;
  float *r_out, *done_out; /* out [N] */
  int64_t *s0_h, *s1_h;    /* out [N] */
  uint64_t seed;           /* exploration and env seed */
  int64_t N;
  float gamma_n, p_reward, p_done;
  int32_t ring, A;
  int32_t ext_frames;      /* 1: the env step writes no frame bytes -- rth_atari_env_step fills the
                            * step's stacks from raw frames right after (Atari env mode) */
} rth_actor_tail_args;
/* The fused actor step's first launch (reth_amd/actors.py step_fused): *t_dev += 1 (the
 * step counter rth_actor_tail's ε-greedy and env step read) and rows_out[i] = i * ring +
 * cur_slot[i], the acting stacks' frame-ring rows the torso forward reads (i < n). */
int rth_actor_prologue(int64_t *t_dev, const int64_t *cur_slot_dev, int64_t n, int64_t ring, int64_t *rows_out_dev,
                       void *stream);
int rth_actor_tail(rth_nstep *h, const rth_actor_tail_args *args, int32_t *emit_dev, int64_t *s0_out_dev,
                   int64_t *a_out_dev, float *r_out_dev, int64_t *s1_out_dev, float *done_out_dev, void *stream);
/* initial reset of every actor into slot 1 (t = 0) */
int rth_synth_env_reset(uint8_t *frames_dev, int64_t n_actors, int32_t ring, uint64_t seed,
                        int64_t *cur_slot_dev, void *stream);
/* stream compaction for variable-size device batches: out[0..k) = vals[i] for the i < n with
 * flag[i] != 0, in order of i (at most cap of them), out[k..cap) = fill, *count_out = base + k.
 * The actors use it to list the terminal stacks of the episodes that just ended (flag = done,
 * vals = the step's next-observation handles) behind the next acting batch. */
int rth_compact_flagged(const float *flag_dev, const int64_t *vals_dev, int64_t n, int64_t *out_dev, int64_t cap,
                        int64_t fill, int64_t base, int64_t *count_out_dev, void *stream);

/* ------------------------------------------------------------------------------------
 * Learner: DQNSolver TD error + Huber (reth/reth/algorithm/dqn/dqn_solver.py:68-124).
 * td = q_s0[a] - (r + (gamma_n * q_tgt(s1)[a*]) * (1 - done)),  a* = argmax q_online(s1)
 * (double_q) or argmax q_tgt(s1); loss = mean(smooth_l1(td) * w); dq = dloss/dq_s0.
 * Every output pointer is nullable.  isw_dev is the sampler's fp64 IS weight (cast to f32
 * like ensure_tensor, :105-106), nullable = no weights.
 * ---------------------------------------------------------------------------------- */
int rth_td_huber(const float *q_s0_dev, const float *q_s1_online_dev, const float *q_s1_target_dev,
                 const int64_t *a_dev, const float *r_dev, const float *done_dev,
                 const double *isw_dev, int64_t B, int64_t A, float gamma_n, int32_t double_q,
                 int32_t dueling, float *td_out_dev, float *td_abs_out_dev, float *loss_elem_dev,
                 float *loss_out_dev, float *dq_out_dev, void *stream);

/* ------------------------------------------------------------------------------------
 * Q-network conv epilogue (reth/reth/algorithm/dqn/dqn_model.py:14-20: Conv2d -> ReLU),
 * on channels-last (NHWC) contiguous fp32 activations of `rows` = N*H*W rows x C channels.
 * rth_bias_relu: y = relu(y + bias[c]) in place (the convolution runs without bias).
 * rth_relu_bias_grad: gy = (y > 0) ? g : 0 (threshold_backward) and db[c] = sum of gy over
 * the rows, deterministic; `workspace` holds rth_relu_bias_grad_workspace(C) bytes of
 * per-block partial sums (scratch, no initialisation).  C a power of 2 in [4, 256].
 * db = NULL: only the slabs are written (finished by rth_conv_relu_wgrad_ex).
 * ---------------------------------------------------------------------------------- */
int rth_bias_relu(float *y_dev, const float *bias_dev, int64_t rows, int32_t C, void *stream);
int64_t rth_relu_bias_grad_workspace(int32_t C);
/* Merged dueling heads (dqn_model.py:22-43 fc_adv / fc_value): params = {adv.0.weight [H,F],
 * value.0.weight [H,F], adv.0.bias, value.0.bias, adv.2.weight [A,H], value.2.weight [1,H],
 * adv.2.bias [A], value.2.bias [1]} -> w1 [2H,F] (FC1 of both branches; with C > 0 its
 * columns follow the NHWC flatten of a C x P feature map), b1 [2H], w2 [A+1,2H]
 * (block diagonal), b2 [A+1].  rth_heads_split_grad maps the four gradients back onto the
 * eight parameters (grads in the same order).
 * C = RTH_HEADS_FC2_ONLY: only the second layer (w2, b2 / their gradients); w1, b1, gw1, gb1
 * and params / grads 0-3 may be NULL -- for a model whose two FC1 branches are row slices of
 * one merged [2H, F] storage (reth_amd/model.py), which FC1 reads and writes in place. */
#define RTH_HEADS_FC2_ONLY (-1)
int rth_heads_merge(const float *const *params_dev, int64_t H, int64_t F, int64_t A, int32_t C, int32_t P,
                    float *w1_dev, float *b1_dev, float *w2_dev, float *b2_dev, void *stream);
int rth_heads_split_grad(const float *gw1_dev, const float *gb1_dev, const float *gw2_dev, const float *gb2_dev,
                         int64_t H, int64_t F, int64_t A, int32_t C, int32_t P, float *const *grads_dev,
                         void *stream);
int rth_relu_bias_grad(const float *g_dev, const float *y_dev, float *gy_dev, float *db_dev, void *workspace_dev,
                       int64_t rows, int32_t C, void *stream);
/* rth_relu_bias_grad for an NCHW activation (the last conv's output written with
 * RTH_CONV_OUT_NCHW: g and y are [n, C, P]); gy is written channels-last [n, P, C] for the
 * data / weight gradients that follow.  Same workspace and slab layout (a deferred job with
 * rows = n * P finishes it); C a power of 2 in [4, 256], C * (P + 1) <= 3200. */
int rth_relu_bias_grad_nchw(const float *g_dev, const float *y_dev, float *gy_dev, float *db_dev,
                            void *workspace_dev, int64_t n, int32_t C, int32_t P, void *stream);
/* Backward of the merged heads' second layer, heads = h @ w2^T + b2 with h = relu(FC1) [B, H2]
 * (row stride ldh), from d(loss)/d(heads) dq [B, A1] (rth_td_huber, dueling): replaces the
 * addmm backward (two GEMMs + a column sum) and threshold_backward of torch.autograd at
 * dqn_solver.py:116 (loss.backward()).  Writes gh = (h > 0) ? dq @ w2 : 0 [B, H2],
 * gw2 = dq^T @ h [A1, H2], gb2 [A1], gb1 = column sums of gh [H2] (the FC1 bias gradient);
 * deterministic.  td_abs_dev / td_acc_dev (nullable): td_acc[0] += mean(td_abs[0..B)), the
 * Trainer's mean_error accumulator (reth/reth/presets/trainer.py:64-69).  H2 % 16 == 0. */
int rth_heads_backward(const float *dq_dev, const float *h_dev, int64_t ldh, const float *w2_dev, int64_t B,
                       int32_t H2, int32_t A1, float *gh_dev, float *gw2_dev, float *gb2_dev, float *gb1_dev,
                       const float *td_abs_dev, float *td_acc_dev, void *stream);
/* rth_td_huber (dueling heads, want dq) + rth_heads_backward in one launch, for
 * B * (A + 1) <= 16384: writes |td| [B], the loss [1] and the heads' gradients as above;
 * td_acc_dev (nullable) += mean |td|.  |td| and the gradients equal the two-launch path's. */
int rth_td_heads_backward(const float *q_s0_dev, const float *q_s1_online_dev, const float *q_s1_target_dev,
                          const int64_t *a_dev, const float *r_dev, const float *done_dev, const double *isw_dev,
                          int64_t B, int64_t A, float gamma_n, int32_t double_q, const float *h_dev, int64_t ldh,
                          const float *w2_dev, int32_t H2, float *td_abs_dev, float *loss_out_dev, float *gh_dev,
                          float *gw2_dev, float *gb2_dev, float *gb1_dev, float *td_acc_dev, void *stream);
/* The same two kernels with the second layer in the reference's branch form: fc2_params =
 * {adv.2.weight [A, H], value.2.weight [1, H], ...} read in place instead of a merged
 * block-diagonal w2, fc2_grads = {adv.2.weight, value.2.weight, adv.2.bias, value.2.bias}
 * gradients written in place (the off-diagonal blocks of gw2 are not produced); H2 = 2H,
 * H a multiple of 16.  Replaces rth_heads_merge / rth_heads_split_grad for the second layer. */
int rth_heads_backward_branches(const float *dq_dev, const float *h_dev, int64_t ldh, const float *const *fc2_params_dev,
                                int32_t H, int64_t B, int64_t A, float *gh_dev, float *const *fc2_grads_dev,
                                float *gb1_dev, const float *td_abs_dev, float *td_acc_dev, void *stream);
int rth_td_heads_backward_branches(const float *q_s0_dev, const float *q_s1_online_dev, const float *q_s1_target_dev,
                                   const int64_t *a_dev, const float *r_dev, const float *done_dev,
                                   const double *isw_dev, int64_t B, int64_t A, float gamma_n, int32_t double_q,
                                   const float *h_dev, int64_t ldh, const float *const *fc2_params_dev, int32_t H,
                                   float *td_abs_dev, float *loss_out_dev, float *gh_dev,
                                   float *const *fc2_grads_dev, float *gb1_dev, float *td_acc_dev, void *stream);
/* The dueling heads' second layer forward (dqn_model.py:22-43 fc_adv[2] / fc_value[2] on the
 * ReLU'd FC1 output h [n, 2H], row stride ldh): heads [n, A+1] = (adv.2(h[:, :H]),
 * value.2(h[:, H:])), the raw heads the TD / epsilon-greedy kernels consume; fc2_params =
 * {adv.2.weight, value.2.weight, adv.2.bias, value.2.bias} read in place. */
int rth_heads_fc2(const float *h_dev, int64_t ldh, int64_t n, int32_t H, int32_t A, const float *const *fc2_params_dev,
                  float *heads_dev, void *stream);
/* rth_heads_fc2 over a device-counted batch (the actors' acting + terminal stacks,
 * test/apex-dqn/worker.py:46 act and :55-60 calc_loss): only rows r < min(*n_dev, n_max) are
 * computed; cache_dev (nullable) [stacks, A+1] additionally receives row r at cache_rows_dev[r]
 * (the per-stack heads cache the deduplicated calc_loss reads) -- one launch instead of two. */
int rth_heads_fc2_upto(const float *h_dev, int64_t ldh, int64_t n_max, const int64_t *n_dev, int32_t H, int32_t A,
                       const float *const *fc2_params_dev, float *heads_dev, float *cache_dev,
                       const int64_t *cache_rows_dev, void *stream);
/* y[r] = relu(x[r] . w^T + b) for rows r0 <= r < min(*n_dev, n_max) (dqn_model.py:22-43, the
 * heads' first Linear -> ReLU): the device-counted tail of a batch whose first r0 rows a
 * library GEMM covers -- the actors' terminal stacks, absent in most steps (every workgroup
 * exits at once).  x [*, F] row stride ldx, w [O, F], y row stride ldy; F, ldx multiples of 4,
 * x and w 16-byte aligned.  Deterministic (fixed-order sums). */
int rth_linear_relu_rows_upto(const float *x_dev, int64_t ldx, int64_t r0, int64_t n_max, const int64_t *n_dev,
                              const float *w_dev, const float *b_dev, int64_t F, int64_t O, float *y_dev, int64_t ldy,
                              void *stream);

/* ------------------------------------------------------------------------------------
 * Q-network convolution torso forward (reth/reth/algorithm/dqn/dqn_model.py:14-20: each
 * Conv2d -> ReLU of `features`): y = relu(conv2d(x, w) + bias) in one launch, implicit GEMM
 * on the fp32 MFMA, output NHWC fp32 [n, hout, wout, cout].  `packed` is the Conv2d weight
 * in the kernel's fragment order, made by rth_conv_pack from the OHWI weight (a channels_last
 * [cout, cin, kh, kw] parameter) into rth_conv_packed_bytes(shape) bytes -- once per weight
 * version, so every launch stages it into LDS with one coalesced copy.  16-byte aligned.
 *   input RTH_CONV_F32_NHWC: x = [n, hin, win, cin] fp32 (channels-last activations);
 *   input RTH_CONV_U8_CHW:   x = uint8 frame stacks [cin, hin, win] (the reference's float32
 *       frames hold exactly these integers); sample i reads stack rows_dev[i] when rows_dev
 *       is given (replay rows, actor frame-ring handles), else stack i -- no f32 copy of the
 *       observations is made.
 * Built geometries: the Nature-DQN torso on 4 x 84 x 84 stacks (conv1 either input form,
 * conv2 32x20x20 -> 64 k4 s2, conv3 64x9x9 -> 64 k3 s1); rth_conv_supported says whether
 * a shape is one of them.  Replaces MIOpen's forward + the separate rth_bias_relu pass.
 * ---------------------------------------------------------------------------------- */
#define RTH_CONV_F32_NHWC 0
#define RTH_CONV_U8_CHW 1
/* flag OR'ed into `input` of rth_conv_bias_relu(_upto): write y NCHW [n, cout, hout, wout]
 * (the last conv, whose output FC1 reads in the reference's (C, H, W) flatten order); the
 * fp32-MFMA kernels only (not the uint8 conv1, which feeds conv2) */
#define RTH_CONV_OUT_NCHW 16
/* rth_conv_pack_many only: the job packs the flipped data-gradient kernel of this FORWARD
 * shape (rth_conv_dgrad_workspace(shape) bytes) for rth_conv_dgrad_prepacked */
#define RTH_CONV_PACK_DGRAD 32
typedef struct rth_conv_shape {
  int32_t input; /* RTH_CONV_F32_NHWC | RTH_CONV_U8_CHW [| RTH_CONV_OUT_NCHW] */
  int32_t cin, hin, win, cout, kh, kw, stride;
} rth_conv_shape;
int rth_conv_supported(const rth_conv_shape *shape);
/* which kernel rth_conv_bias_relu runs for a shape and n samples (hybrid geometries switch by
 * batch size): RTH_CONV_IMPL_F32 (k_conv_bias_relu, fp32 MFMA), RTH_CONV_IMPL_BF16X3
 * (k_conv1_u8_bf16x3), RTH_CONV_IMPL_X9 (k_conv_x9: both operands split into three exact bf16
 * terms, nine bf16 MFMAs per fp32 product; *nsamp_out = samples per workgroup); 0 = not built.
 * Diagnostics (bench.py's roofline labels), no launch. */
#define RTH_CONV_IMPL_F32 1
#define RTH_CONV_IMPL_BF16X3 2
#define RTH_CONV_IMPL_X9 3
int rth_conv_impl(const rth_conv_shape *shape, int64_t n, int32_t *nsamp_out);
int64_t rth_conv_packed_bytes(const rth_conv_shape *shape);
int rth_conv_pack(const rth_conv_shape *shape, const float *w_ohwi_dev, float *packed_dev, void *stream);
/* rth_conv_pack for n <= 6 layers in one launch (a network's torso, both conv1 forms, and
 * with RTH_CONV_PACK_DGRAD in a job's shape->input the packed data-gradient kernels of the
 * same weights: the learner packs everything its forward and backward read in one launch) */
int rth_conv_pack_many(int32_t n, const rth_conv_shape *shapes, const float *const *w_ohwi_dev,
                       float *const *packed_dev, void *stream);
int rth_conv_bias_relu(const rth_conv_shape *shape, const void *x_dev, const int64_t *rows_dev, int64_t n,
                       const float *packed_dev, const float *bias_dev, float *y_dev, void *stream);
/* rth_conv_bias_relu over the first min(n_max, *n_dev) samples, the count read on the device
 * (graph replay of a variable-size batch: the actors' acting stacks plus the terminal stacks
 * of the episodes that just ended); outputs past the count are left untouched. */
int rth_conv_bias_relu_upto(const rth_conv_shape *shape, const void *x_dev, const int64_t *rows_dev, int64_t n_max,
                            const int64_t *n_dev, const float *packed_dev, const float *bias_dev, float *y_dev,
                            void *stream);
/* Data gradient of conv2d(x, w) (the backward through conv3 / conv2 of the learner's torso,
 * reth/reth/algorithm/dqn/dqn_solver.py:117 loss.backward() on dqn_model.py:14-20; replaces
 * MIOpen's backward-data solver and its zero fill): gx = [n, hin, win, cin] fp32 NHWC from
 * gy = [n, hout, wout, cout] fp32 NHWC and w = the OHWI weight (a channels_last Conv2d
 * parameter, read directly: no packing).  Every element of gx is written exactly once.
 * `shape` is the FORWARD convolution's (input RTH_CONV_F32_NHWC); built: conv2 and conv3 of
 * the Nature-DQN torso (rth_conv_dgrad_supported).  16-byte aligned buffers. */
int rth_conv_dgrad_supported(const rth_conv_shape *shape);
int rth_conv_dgrad(const rth_conv_shape *shape, const float *gy_dev, int64_t n, const float *w_ohwi_dev,
                   float *gx_dev, void *stream);
/* The same with a caller-owned workspace for the flipped kernel the exact-split path packs
 * each launch (rth_conv_dgrad_workspace bytes, 16-byte aligned; 0 bytes: none needed).
 * rth_conv_dgrad uses one internal workspace per device, so two learners in one process whose
 * backward passes run on different streams (or are replayed from different graphs) must each
 * pass their own: the pack and the convolution of one call are stream-ordered, two calls on
 * two streams are not. */
int64_t rth_conv_dgrad_workspace(const rth_conv_shape *shape);
/* rth_conv_dgrad from a kernel packed beforehand: `packed_dev` = the RTH_CONV_PACK_DGRAD job of
 * rth_conv_pack_many for this shape and the weights of the forward (no pack launch here; same
 * result as rth_conv_dgrad_ws on those weights, bit for bit).  Built where
 * rth_conv_dgrad_workspace(shape) > 0. */
int rth_conv_dgrad_prepacked(const rth_conv_shape *shape, const float *gy_dev, int64_t n, const void *packed_dev,
                             float *gx_dev, void *stream);
/* rth_conv_dgrad_prepacked for conv3's geometry (rth_conv_dgrad_relu_supported) with the layer
 * below's ReLU applied in the same launch (r05): gx = the data gradient where y_dev (the layer
 * below's output, [n, 9, 9, 64] NHWC) > 0, else 0 -- what rth_relu_bias_grad makes of the plain
 * data gradient -- and that layer's bias-gradient slab partials written to bias_ws_dev (a
 * rth_relu_bias_grad workspace of C = 64, finished later by a rth_bias_deferred job whose
 * `slabs` is *slabs_out).  Reference: the backward of dqn_model.py:14-20 (Conv2d + ReLU). */
int rth_conv_dgrad_relu_supported(const rth_conv_shape *shape);
int rth_conv_dgrad_relu_prepacked(const rth_conv_shape *shape, const float *gy_dev, int64_t n, const void *packed_dev,
                                  const float *y_dev, float *gx_dev, void *bias_ws_dev, int64_t *slabs_out,
                                  void *stream);
/* FC1 of the dueling heads (the first Linear + ReLU of both branches, dqn_model.py:38-47, as
 * one [N, K] weight) on the exact-split bf16 MFMA: y [M, N] = act(x [M, K] w^T + b), x
 * row-major with row stride ldx, w row-major [N, K] (the Linear weight as stored), act = ReLU
 * when relu != 0, bias may be NULL; M % 64 == 0, N % 128 == 0, K % 32 == 0
 * (rth_fc_x9_supported).  Fixed-order split-K partials in `workspace` (rth_fc_x9_workspace
 * bytes, NULL when that is 0): run-to-run deterministic.  M and N multiples of 128 run on a
 * 128 x 128 workgroup tile (late r05), others on a 64 x 128 tile; the tile and the k splits
 * are fixed functions of (M, N, K), so the workspace size is too.  Replaces the hipBLASLt GEMM
 * + bias + ReLU epilogue (torch._addmm_activation) of every FC1 forward in the loop (r06: the
 * actors', the target pass's and the learner's). */
int rth_fc_x9_supported(int64_t M, int64_t N, int64_t K);
int64_t rth_fc_x9_workspace(int64_t M, int64_t N, int64_t K);
int rth_fc_x9(const float *x_dev, int64_t ldx, int64_t M, const float *w_dev, int64_t N, int64_t K,
              const float *bias_dev, int32_t relu, float *y_dev, void *workspace_dev, void *stream);
/* The actors' counted FC1 (r05): y [n_max, N] rows [0, M) = rth_fc_x9 (ReLU, M % 64 == 0) and
 * rows [M, min(*n_dev, n_max)) = rth_linear_relu_rows_upto (the device-counted terminal stacks),
 * the split-K reduce and the counted rows in one launch; y row stride N; the same bits as
 * those two calls. */
int rth_fc_x9_rows_upto(const float *x_dev, int64_t ldx, int64_t M, int64_t n_max, const int64_t *n_dev,
                        const float *w_dev, int64_t N, int64_t K, const float *bias_dev, float *y_dev,
                        void *workspace_dev, void *stream);
/* FC1 -> FC2 of the dueling heads in two launches (r06; dqn_model.py:38-47, 59-71 forward
 * under dqn_solver.py:77-98 _calc_td_error / the target pass): rth_fc_x9's GEMM into its split-K
 * workspace, then one launch reducing it (+ b1 + ReLU, rth_fc_x9's order) and running the second
 * layer of both branches from the parameters in place (fc2_params = {adv weight [A, H], value
 * weight [1, H], adv bias [A], value bias [1]}, rth_heads_fc2's order): heads [M, A + 1] (raw
 * advantages then value) bit-identical to rth_fc_x9 + rth_heads_fc2; h1_out (nullable) [M, N]
 * receives relu(FC1).  N = 2H <= 512; workspace = rth_fc_x9_workspace(M, N, K) bytes. */
int rth_fc1_heads_supported(int64_t M, int64_t N, int64_t K, int32_t A);
int rth_fc1_heads(const float *x_dev, int64_t ldx, int64_t M, const float *w1_dev, int64_t N, int64_t K,
                  const float *b1_dev, int32_t A, const float *const *fc2_params, float *heads_dev, float *h1_out_dev,
                  void *workspace_dev, void *stream);
/* The same FC1 on the fp32 MFMA with no LDS (r05): the arguments, the workspace protocol and
 * the determinism of rth_fc_x9; any M >= 1 (ragged actor batches), N % 128 == 0, K % 32 == 0
 * (rth_fc_f32_supported).  Not used by the loop (the x9 form is faster there); kept as the
 * fp32-MFMA reference form, tested against it. */
int rth_fc_f32_supported(int64_t M, int64_t N, int64_t K);
int64_t rth_fc_f32_workspace(int64_t M, int64_t N, int64_t K);
int rth_fc_f32(const float *x_dev, int64_t ldx, int64_t M, const float *w_dev, int64_t N, int64_t K,
               const float *bias_dev, int32_t relu, float *y_dev, void *workspace_dev, void *stream);
int rth_conv_dgrad_ws(const rth_conv_shape *shape, const float *gy_dev, int64_t n, const float *w_ohwi_dev,
                      float *gx_dev, void *workspace_dev, void *stream);
/* Weight gradient of conv2d(x, w) for the fp32 channels-last layers (conv2 and conv3 of the
 * torso; the backward of dqn_model.py:14-20 under dqn_solver.py:117 loss.backward(); replaces
 * MIOpen's weight-gradient solver and its zero fill): gw [cout, kh, kw, cin] (OHWI, the
 * channels_last parameter layout) = sum over output pixels of gy[p][co] * x-window[p], from
 * x = [n, hin, win, cin] and gy = [n, hout, wout, cout] (already ReLU-masked), on the fp32
 * MFMA; every sum has a fixed order (deterministic).  `shape` is the forward convolution's
 * (input RTH_CONV_F32_NHWC); workspace = rth_conv_wgrad_f32_workspace(shape) bytes. */
/* The same on the bf16 MFMA with both operands split into three exact bf16 terms (nine
 * products per fp32 product, exact in the fp32 accumulator: the fp32 path's products in
 * another fixed summation order); workspace = rth_conv_wgrad_x9_workspace(shape) bytes. */
int rth_conv_wgrad_x9_supported(const rth_conv_shape *shape);
int64_t rth_conv_wgrad_x9_workspace(const rth_conv_shape *shape);
int rth_conv_wgrad_x9(const rth_conv_shape *shape, const float *x_dev, int64_t n, const float *gy_dev, float *gw_dev,
                      void *workspace_dev, void *stream);
int rth_conv_wgrad_f32_supported(const rth_conv_shape *shape);
int64_t rth_conv_wgrad_f32_workspace(const rth_conv_shape *shape);
int rth_conv_wgrad_f32(const rth_conv_shape *shape, const float *x_dev, int64_t n, const float *gy_dev, float *gw_dev,
                       void *workspace_dev, void *stream);
/* rth_conv_wgrad_f32's partial launch alone (r06): *job_out describes the fixed-order reduce that
 * finishes gw_dev -- handed to conv1's weight-gradient reduce launch (rth_conv_relu_wgrad_ex and
 * its frame-id / norm forms, `wdeferred`), which runs it in its own workgroups; the result is
 * bit-identical to rth_conv_wgrad_f32's. */
typedef struct rth_wgrad_deferred {
  const float *partial; /* the workspace holding the split partials */
  float *gw;            /* OHWI output */
  int32_t splits, elems, nb, K;
} rth_wgrad_deferred;
int rth_conv_wgrad_f32_partials(const rth_conv_shape *shape, const float *x_dev, int64_t n, const float *gy_dev,
                                float *gw_dev, void *workspace_dev, rth_wgrad_deferred *job_out, void *stream);
/* Backward of relu(conv2d(x, w) + b) for the weights and bias, on uint8 stacks (conv1, whose
 * input needs no gradient): gy = (y > 0) ? g : 0, gw = sum over output pixels of gy times the
 * input window (OHWI [cout, kh, kw, cin], the layout of a channels_last weight), gb = sum of
 * gy.  g, y: NHWC fp32 [n, hout, wout, cout] (upstream gradient, forward output).  Summed in
 * a fixed order (deterministic); workspace = rth_conv_wgrad_workspace(shape) bytes.  Built
 * for the uint8 conv1 geometry; replaces rth_relu_bias_grad + MIOpen's weight gradient. */
int64_t rth_conv_wgrad_workspace(const rth_conv_shape *shape);
int rth_conv_relu_wgrad(const rth_conv_shape *shape, const void *x_dev, const int64_t *rows_dev, int64_t n,
                        const float *g_dev, const float *y_dev, float *gw_dev, float *gb_dev, void *workspace_dev,
                        void *stream);
/* rth_conv_relu_wgrad that also finishes up to 4 deferred bias gradients in its reduce launch
 * (one launch fewer per layer): each a rth_relu_bias_grad called with db = NULL on
 * `workspace`, over `rows` rows of C channels, earlier on the same stream; and up to 2 deferred
 * weight gradients (rth_conv_wgrad_f32_partials jobs, earlier on the same stream). */
typedef struct rth_bias_deferred {
  const void *workspace; /* the rth_relu_bias_grad workspace holding the slabs */
  float *db;             /* [C] output */
  int64_t rows;
  int32_t C;
  int32_t slabs; /* the slab count; 0 = rth_relu_bias_grad's for `rows` (rth_conv_dgrad_relu_prepacked
                  * reports its own) */
} rth_bias_deferred;
int rth_conv_relu_wgrad_ex(const rth_conv_shape *shape, const void *x_dev, const int64_t *rows_dev, int64_t n,
                           const float *g_dev, const float *y_dev, float *gw_dev, float *gb_dev, void *workspace_dev,
                           const rth_bias_deferred *deferred, int32_t ndeferred,
                           const rth_wgrad_deferred *wdeferred, int32_t nwdeferred, void *stream);
/* Frames in place (r05): conv1 (4x84x84 uint8 -> 32, k8 s4) forward and weight gradient
 * reading each sample's 4 frames straight from a replay's frame store (the
 * rth_replay_frames_attach store, 84*84-byte frames) by the int32 [n][4] frame ids a
 * rth_replay_frames_ids_out gather wrote (16-byte aligned), instead of from gathered stacks:
 * results bit-identical to rth_conv_bias_relu / rth_conv_relu_wgrad_ex on the stacks
 * rth_replay_gather would have assembled from the same ids, without that copy. */
int rth_conv1_frames_bias_relu(const rth_conv_shape *shape, const uint8_t *store_dev, const int32_t *ids_dev,
                               int64_t n, const float *packed_dev, const float *bias_dev, float *y_dev, void *stream);
int rth_conv1_frames_relu_wgrad_ex(const rth_conv_shape *shape, const uint8_t *store_dev, const int32_t *ids_dev,
                                   int64_t n, const float *g_dev, const float *y_dev, float *gw_dev, float *gb_dev,
                                   void *workspace_dev, const rth_bias_deferred *deferred, int32_t ndeferred,
                                   const rth_wgrad_deferred *wdeferred, int32_t nwdeferred, void *stream);

/* ------------------------------------------------------------------------------------
 * Atari observation preprocessing (reth/reth/env/util.py:121-209, 281-297): per actor, the
 * max of the last two raw RGB frames of the skip window (MaxAndSkipEnv), cv2 RGB2GRAY +
 * INTER_AREA resize to out_h x out_w (WarpFrame; OpenCV's 8-bit algorithms restated, cv2
 * being absent), pushed onto the actor's frame stack (FrameStack, ImageToPyTorch layout).
 *   raw_dev    [n, 2, in_h, in_w, 3] uint8 (for a reset: the reset frame twice)
 *   frames_dev the actors' stack ring [n * ring, stack, out_h, out_w] uint8 (nullable):
 *              slot new_slot[i] <- slot prev_slot[i] shifted by one frame + the new frame,
 *              or the new frame `stack` times when reset_dev[i] != 0 (reset_dev nullable)
 *   out_frame_dev (nullable) [n, out_h, out_w]: the preprocessed frames alone
 * ---------------------------------------------------------------------------------- */
typedef struct rth_atari rth_atari;
int rth_atari_create(int32_t in_h, int32_t in_w, int32_t out_h, int32_t out_w, int device, rth_atari **out);
int rth_atari_destroy(rth_atari *h);
int rth_atari_step(rth_atari *h, const uint8_t *raw_dev, int64_t n, uint8_t *frames_dev, int32_t ring, int32_t stack,
                   const int64_t *prev_slot_dev, const int64_t *new_slot_dev, const uint8_t *reset_dev,
                   uint8_t *out_frame_dev, void *stream);
/* the Ape-X actors' Atari env mode (after rth_actor_tail with ext_frames = 1): per actor i the
 * raw pair raw_dev[i] (MaxAndSkip max, gray, INTER_AREA) becomes the new top frame of stack
 * s1_h[i] = stack s0_h[i] shifted by one (FrameStack.step), and where done_dev[i] != 0 the
 * reset observation -- env.reset()'s screen reset_raw_dev[i] ([n, in_h, in_w, 3], read only
 * where done; MaxAndSkip.reset returns it without a pair max, util.py:129-130), warped, `stack`
 * times (FrameStack.reset, util.py:191-196) -- goes into actor i's slot cur_slot_dev[i].
 * Handles index frames_dev's stacks; slots are per-actor ring slots. */
int rth_atari_env_step(rth_atari *h, const uint8_t *raw_dev, int64_t n, uint8_t *frames_dev, int32_t ring,
                       int32_t stack, const int64_t *s0_h_dev, const int64_t *s1_h_dev, const float *done_dev,
                       const int64_t *cur_slot_dev, const uint8_t *reset_raw_dev, void *stream);
/* synthetic raw emulator screens (the stand-in for ALE's output, ALE being absent): nbytes of
 * device Philox (seed, step *t_dev), 16-byte aligned and a multiple of 16 bytes */
int rth_atari_synth_raw(uint8_t *raw_dev, int64_t nbytes, uint64_t seed, const int64_t *t_dev, void *stream);
/* synthetic reset screens: frame i of reset_raw_dev ([n, frame_bytes]) from device Philox
 * (seed, step *t_dev, its own stream), written only where done_dev[i] != 0 */
int rth_atari_synth_reset(uint8_t *reset_raw_dev, int64_t n, int64_t frame_bytes, uint64_t seed, const int64_t *t_dev,
                          const float *done_dev, void *stream);

/* ------------------------------------------------------------------------------------
 * Learner optimizer step (reth/reth/algorithm/dqn/dqn_solver.py:118-121):
 * torch.nn.utils.clip_grad_norm_(params, max_norm) then torch.optim.Adam.step() over up to
 * RTH_MAX_PARAM_TENSORS fp32 tensors in two launches (norm partials, then the update).
 * max_norm < 0 skips clipping.  step_dev (int64, device) is Adam's step count, incremented on
 * the device; workspace_dev holds rth_clip_adam_workspace() bytes, zero-filled once before the
 * first call; one workspace per optimizer.  total_norm_out_dev (nullable) receives the pre-clip
 * 2-norm (clip_grad_norm_'s return).
 * ---------------------------------------------------------------------------------- */
#define RTH_MAX_PARAM_TENSORS 32
typedef struct rth_param_tensor {
  float *param;
  const float *grad;
  float *exp_avg;    /* Adam state["exp_avg"] */
  float *exp_avg_sq; /* Adam state["exp_avg_sq"] */
  int64_t n;
} rth_param_tensor;
int64_t rth_clip_adam_workspace(void);
int rth_clip_adam(const rth_param_tensor *tensors, int32_t n_tensors, double lr, double beta1, double beta2,
                  double eps, double max_norm, int64_t *step_dev, void *workspace_dev, float *total_norm_out_dev,
                  void *stream);
/* The same step with clip_grad_norm_'s partials produced by the learner's backward (r06, one
 * rank: the gradients are final there).  rth_conv1_relu_wgrad_norm is rth_conv_relu_wgrad_ex
 * (rows_dev != NULL: stacks by row; fids_dev != NULL: rth_conv1_frames_relu_wgrad_ex's frame
 * ids, x_dev the frame store; neither: x_dev the stacks) whose reduce launch also writes the
 * fp64 sum-of-squares partials clip_grad_norm_ reduces: extra workgroups over the gradients of
 * `sq` (every parameter but conv1's weight and bias and the deferred bias and weight gradients,
 * which the launch finishes itself and adds right behind them; only .grad and .n are read), the first of
 * them advancing step_dev and writing the step's bias corrections as rth_clip_adam's first
 * launch does, all into adam_workspace_dev (rth_clip_adam_workspace's layout);
 * *nparts_out = the partial count.  rth_adam_prenormed(..., nparts, ...) is then
 * rth_clip_adam's second launch alone: the same update, the norm summed in partial order. */
int rth_conv1_relu_wgrad_norm(const rth_conv_shape *shape, const void *x_dev, const int64_t *rows_dev,
                              const int32_t *fids_dev, int64_t n, const float *g_dev, const float *y_dev,
                              float *gw_dev, float *gb_dev, void *workspace_dev, const rth_bias_deferred *deferred,
                              int32_t ndeferred, const rth_wgrad_deferred *wdeferred, int32_t nwdeferred,
                              const rth_param_tensor *sq, int32_t n_sq, double lr, double beta1,
                              double beta2, int64_t *step_dev, void *adam_workspace_dev, int32_t *nparts_out,
                              void *stream);
int rth_adam_prenormed(const rth_param_tensor *tensors, int32_t n_tensors, double lr, double beta1, double beta2,
                       double eps, double max_norm, int32_t nparts, int64_t *step_dev, void *workspace_dev,
                       float *total_norm_out_dev, void *stream);

/* ------------------------------------------------------------------------------------
 * Learner -> actor weights: a device-resident latest-wins slot with a device version.
 * Replaces perwez's PUB/SUB CONFLATE weights channel (perwez/perwez/client/socket.py:19-122,
 * 302-328: SendSocket.send / RecvSocket.recv / RecvSocket.empty) as used by
 * test/apex-dqn/trainer.py:38-41 (publish every send_weights_interval updates) and
 * worker.py:37-41 (load when > recv_weights_interval steps passed and a message waits).
 * Segments: the parameter tensors, 4-byte aligned, in a fixed order (<= 64).
 * ---------------------------------------------------------------------------------- */
typedef struct rth_weights rth_weights;
int rth_weights_create(int64_t bytes, int device, rth_weights **out);
int rth_weights_destroy(rth_weights *h);
int64_t rth_weights_bytes(const rth_weights *h);
/* SendSocket.send: copy the n segments into the slot, then version += 1 (stream order) */
int rth_weights_publish(rth_weights *h, int32_t n, const void *const *src_dev, const int64_t *bytes, void *stream);
/* the slot's initial contents without a message (version unchanged): what a subscriber that
 * connects before the first send holds -- the reference's SUB socket delivers nothing until
 * the trainer's first send (test/apex-dqn/trainer.py:38-41) */
int rth_weights_fill(rth_weights *h, int32_t n, const void *const *src_dev, const int64_t *bytes, void *stream);
/* RecvSocket.empty + recv, decided on the device: if version > *seen_dev (and, with a step
 * counter, *step_dev - *prev_dev > interval) copy the slot into the n segments, set
 * *seen_dev = version, *prev_dev = *step_dev and *loaded_dev = 1; else *loaded_dev = 0.
 * step_dev / prev_dev / loaded_dev may be NULL.  Graph-capturable (no host decision). */
int rth_weights_acquire(rth_weights *h, int32_t n, void *const *dst_dev, const int64_t *bytes, int64_t *seen_dev,
                        const int64_t *step_dev, int64_t *prev_dev, int64_t interval, int32_t *loaded_dev,
                        void *stream);
int rth_weights_version(const rth_weights *h, int64_t *out);        /* synchronous read */
int rth_weights_version_ptr(rth_weights *h, int64_t **out_dev);     /* the device counter */

/* ------------------------------------------------------------------------------------
 * LZ4 frames (host code) for compressed wire messages: Client.append(..., compress=True)
 * (reth_buffer/reth_buffer/utils/pack.py:62-84 lz4.frame.compress / :147-164 decompress),
 * what test/apex-dqn/worker.py:60 sends.  Host pointers.
 * ---------------------------------------------------------------------------------- */
int rth_lz4_frame_bound(const uint8_t *src, int64_t n, int64_t *bound);
int rth_lz4_frame_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int64_t *out_len);
int64_t rth_lz4_frame_compress_bound(int64_t n);
int rth_lz4_frame_compress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int64_t *out_len);
uint32_t rth_xxh32(const uint8_t *src, int64_t n, uint32_t seed);

#ifdef __cplusplus
}
#endif
#endif
