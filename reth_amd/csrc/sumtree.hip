// In-order heap sum-tree + PER sampler on gfx950.
//
// Reference semantics: reth_buffer/reth_buffer/utils/sumtree.py (live PER tree) and
// reth_buffer/reth_buffer/sampler/per_sampler.py.  The tree is a heap of `capacity` nodes in
// which EVERY node carries a priority; sum[i] = val[i] + sum[l] + sum[r] (in that order);
// sampling walks left subtree -> node -> right subtree.  All arithmetic is fp64 with the
// reference's operation order, so results are bit-identical to the sequential numba code.
//
// HBM layout: one 32-byte record per node {sum, val, min, pad}, node i at record i + 1, so
// the two children of node i (2i+1, 2i+2) are records 2i+2, 2i+3: one aligned 64-byte pair.
// A descent step therefore needs one 64-byte pair (left {sum,val} + right val), and a
// maintain step reads the pair plus its own record.
//
// Batched update (the reference loops val[idx]=w; maintain(idx) per element):
//   the final state equals "write the last value of every index, then recompute every
//   touched ancestor once, deepest level first, from final children" -- a touched node's
//   last maintenance in the sequential loop happens after every change below it.  Untouched
//   nodes must NOT be recomputed (the min() quirk, sumtree.py:11-19, seeds 1 for a maintained
//   zero node).  One launch, two phases:
//   * k_tree_update_sub: the levels S..maxd (S = 11), one workgroup per group of level-S
//     subtrees (256 workgroups); each sorts its keys by left-aligned leaf position, loads
//     everything its touched nodes need in one parallel pass, runs the level loop in LDS and
//     stores the touched nodes once;
//   * tree_top: the 2^S - 1 nodes above level S, dense in LDS, from the level-S sums the
//     subtree pass wrote through to memory -- run by the subtree pass's last workgroup (a
//     ticket), so the whole update is one launch (k_tree_update_top alone when no key lies
//     below level S).
//   Any partition of the keys by subtree, and any split into launch-ordered rounds, gives the
//   sequential result, so this is bit-identical to _numba_update for every n.
#include <cmath>
#include <cstdlib>

#include "common.hpp"

namespace rth {

struct alignas(32) Node {
  double sum, val, mn, pad;
};

constexpr int64_t kMaxCapacity = int64_t(1) << 40;  // sort key: aligned(41) + depth(6) + slot(10) <= 64

__host__ __device__ __forceinline__ int node_depth(int64_t i) { return 63 - __builtin_clzll((unsigned long long)(i + 1)); }

// _numba_maintain_node (sumtree.py:5-21)
__device__ __forceinline__ void maintain_node(Node *nd, int64_t cap, int64_t i) {
  const int64_t l = 2 * i + 1, r = 2 * i + 2;
  const double v = nd[i + 1].val;
  double s = v;
  double m = (v != 0.0) ? v : 1.0;
  if (l < cap) {
    const Node L = nd[l + 1];
    s = radd(s, L.sum);
    if (L.mn != 0.0) m = (L.mn < m) ? L.mn : m;
  }
  if (r < cap) {
    const Node R = nd[r + 1];
    s = radd(s, R.sum);
    if (R.mn != 0.0) m = (R.mn < m) ? R.mn : m;
  }
  nd[i + 1].sum = s;
  nd[i + 1].mn = m;
}

// _numba_find_index (sumtree.py:34-58).
// The walk is a chain of dependent loads (one per level, ~20 for 1M rows), so it runs
// K levels per memory round trip: at node c it issues the child pairs of c and of its
// descendants down to depth K-1 together (2^K - 1 pairs, all independent), then takes up
// to K steps of the reference's exact comparisons/subtractions on registers.
struct Pair {
  double ls, lv, rv;  // left child {sum, val}, right child val
};

__device__ __forceinline__ Pair load_pair(const Node *__restrict__ nd, int64_t cap, int64_t c) {
  const int64_t l = 2 * c + 1;
  Pair p{0.0, 0.0, 0.0};
  if (l < cap) {
    const double2 L = *reinterpret_cast<const double2 *>(&nd[l + 1]);
    p.ls = L.x;
    p.lv = L.y;
    p.rv = nd[l + 2].val;  // record cap+1 exists (padding), so no bound check needed
  }
  return p;
}

// one level of the reference loop at `cur`; false: `cur` is the answer
__device__ __forceinline__ bool find_step(int64_t &cur, double &cval, double &w, const Pair &p, int64_t cap) {
  const int64_t l = 2 * cur + 1;
  if (l < cap) {
    if (w < p.ls) {
      cur = l;
      cval = p.lv;
      return true;
    }
    w = rsub(w, p.ls);
  }
  if (w < radd(cval, 1e-5)) return false;
  w = rsub(w, cval);
  if (l + 1 >= cap) return false;
  cur = l + 1;  // r < cap implies l < cap: its val came with the pair
  cval = p.rv;
  return true;
}

template <int K>
__device__ __forceinline__ int64_t tree_find_k(const Node *__restrict__ nd, int64_t cap, double w, int64_t cur = 0,
                                               double cval = -1.0) {
  constexpr int NP = (1 << K) - 1;  // pairs per round trip: c's subtree down to depth K-1
  if (cur == 0 && cval < 0.0) cval = nd[1].val;  // from the root (else: resumed below an LDS-staged top)
  for (;;) {
    Pair p[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      // q-th node of the depth-(K-1) heap under cur: depth dq = log2(q+1), offset q+1-2^dq
      const int dq = 31 - __builtin_clz(q + 1);
      const int64_t node = (cur + 1) * (int64_t(1) << dq) - 1 + (q + 1 - (1 << dq));
      p[q] = load_pair(nd, cap, node);
    }
    int q = 0;  // position of `cur` inside the prefetched subtree (heap order)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      Pair pk = p[0];
#pragma unroll
      for (int j = 1; j < NP; ++j)
        if (j == q) pk = p[j];
      const int64_t before = cur;
      if (!find_step(cur, cval, w, pk, cap)) return cur;
      q = 2 * q + 1 + (int)(cur - (2 * before + 1));
    }
  }
}

__device__ __forceinline__ int64_t tree_find(const Node *__restrict__ nd, int64_t cap, double w, int kspec = 2,
                                             int64_t cur = 0, double cval = -1.0) {
  switch (kspec) {
    case 1: return tree_find_k<1>(nd, cap, w, cur, cval);
    case 4: return tree_find_k<4>(nd, cap, w, cur, cval);
    case 3: return tree_find_k<3>(nd, cap, w, cur, cval);
    default: return tree_find_k<2>(nd, cap, w, cur, cval);
  }
}

// The same walk with a group of 2^K lanes per target (K levels per round trip): lane q of
// the group loads the q-th pair of the prefetched subtree -- one 64-byte pair per lane
// instead of 2^K - 1 per lane -- and every lane of the group takes the same K steps on the
// pairs it reads from its group mates (ds_bpermute).  The group's control flow is uniform
// (all its lanes hold the same target), so a shuffle never reads an inactive lane.
template <int K>
__device__ __forceinline__ int64_t tree_find_group(const Node *__restrict__ nd, int64_t cap, double w, int base,
                                                   int sub, int64_t cur = 0, double cval = -1.0) {
  constexpr int NP = (1 << K) - 1;
  if (cur == 0 && cval < 0.0) cval = nd[1].val;  // from the root (else: resumed below an LDS-staged top)
  const int dq = 31 - __builtin_clz(sub + 1);
  const int64_t off = sub + 1 - (1 << dq);
  for (;;) {
    const Pair mine = sub < NP ? load_pair(nd, cap, (cur + 1) * (int64_t(1) << dq) - 1 + off) : Pair{0.0, 0.0, 0.0};
    int q = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const Pair pk{__shfl(mine.ls, base + q, 64), __shfl(mine.lv, base + q, 64), __shfl(mine.rv, base + q, 64)};
      const int64_t before = cur;
      if (!find_step(cur, cval, w, pk, cap)) return cur;
      q = 2 * q + 1 + (int)(cur - (2 * before + 1));
    }
  }
}

// rth_sumtree_find's walk: lane groups of 2^kFindGroupK lanes taking that many levels per
// round trip (one pair per lane); one-lane walks take kFindK levels per round trip
constexpr int kFindGroupK = 4, kFindK = 2, kFindThreads = 64;

__device__ __forceinline__ int64_t tree_find_grouped(const Node *__restrict__ nd, int64_t cap, double w, int gk,
                                                     int base, int sub, int64_t cur = 0, double cval = -1.0) {
  switch (gk) {
    case 3: return tree_find_group<3>(nd, cap, w, base, sub, cur, cval);
    case 5: return tree_find_group<5>(nd, cap, w, base, sub, cur, cval);
    default: return tree_find_group<4>(nd, cap, w, base, sub, cur, cval);
  }
}

// The hot top of the tree staged in LDS (north_star: "LDS-staged segment scans for the tree"):
// every sample workgroup copies {sum, val} of the nodes of the first TL levels (the nodes every
// target's walk passes through; k_tree_sample_deep), then each target walks those levels in
// LDS -- the same find_step comparisons and subtractions -- and only the levels below go to HBM.
// Returns true when the walk must continue below the staged levels (cur / cval / w hold its
// state), false when `cur` is already the answer.
__device__ __forceinline__ bool lds_top_walk(const double2 *__restrict__ top, int64_t cap, int64_t nstaged,
                                             int64_t &cur, double &cval, double &w) {
  cur = 0;
  cval = top[0].y;
  for (;;) {
    const int64_t l = 2 * cur + 1;
    if (l >= nstaged) return l < cap;  // the children are below the staged levels (or absent)
    const Pair p{top[l].x, top[l].y, l + 1 < cap ? top[l + 1].y : 0.0};
    if (!find_step(cur, cval, w, p, cap)) return false;
  }
}

// RTH_TREE_PASSES (read per call): the tree update's subtree passes (tree_update_impl)
static int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}

__device__ __forceinline__ double tree_min(const Node *nd) {  // NumbaSumTree.min :109-110
  const Node root = nd[1];
  return root.sum != 0.0 ? root.mn : 1.0;
}

// ------------------------------------------------------------------ batched update
struct UpdArgs {
  Node *nd;
  int64_t cap;
  int32_t maxd;
  const int64_t *idx;   // nullable: FIFO range (fifo_start + i) % cap
  int64_t fifo_start;
  const double *w64;     // priority as given (NumbaSumTree.update)
  const void *td_abs;    // or PERSampler.update: (td_abs + 1e-6) ** alpha ...
  int32_t td_dtype;      // ... in float32 (RTH_F32) or float64 (RTH_F64), like numpy
  double alpha;
  int64_t n;
  ReplayState *st;        // nullable: a replay shard's device state supplies the FIFO start
  rth_schedule alpha_s;   // and alpha = alpha_s(st->sched_step)
  // a deferred update_priorities merged into this launch, applied before the n keys above
  const int64_t *pidx;
  const void *ptd;
  int32_t pdtype;
  int32_t pre_step;   // st->sched_step += 1 before alpha is read (its step=True on_step)
  int64_t pn;
  int32_t post_tail;  // st->tail += n after every read of it (the append's FIFO advance)
  int32_t fuse_top;   // 1: the subtree pass's last workgroup runs the top pass; 2: an extra
                      // workgroup of the last subtree launch runs it concurrently (r05); 0: its own launch
  // nullable: the subtree pass stages the top pass's key information here (set when it runs):
  // bytes 0 .. 2047 = touched flags of the level-S nodes (each written by the node's owner,
  // no atomics: one line per 128 nodes, not a contended bitmap), stage[kStageFlags + i] =
  // the last key (launch order) on top node i, or -1.  The top pass reads and re-arms it
  // (no scan of the keys).
  int32_t *stage;
};
constexpr int kStageFlags = 512;  // int32 words of touched flags (2^11 level-S nodes, 1 byte each)

// FIFO start and alpha of a launch: both replay-state words loaded together
__device__ __forceinline__ void upd_prologue(const UpdArgs &a, int64_t *fifo_start, double *alpha) {
  if (a.st) {
    const int64_t tail = a.st->tail, step = a.st->sched_step;
    *fifo_start = tail;
    *alpha = sched_value(a.alpha_s, step + a.pre_step);
  } else {
    *fifo_start = a.fifo_start;
    *alpha = a.alpha;
  }
}

__device__ __forceinline__ double prio_value(const void *td, int32_t dt, double alpha, int64_t i) {
  if (dt == RTH_PRIO_RAW) return static_cast<const double *>(td)[i];
  if (dt == RTH_F64) return per_normalize64(static_cast<const double *>(td)[i], alpha);
  return (double)per_normalize(static_cast<const float *>(td)[i], (float)alpha);
}

// key g of the launch: the deferred update's g-th index, then the main segment's
__device__ __forceinline__ int64_t upd_id(const UpdArgs &a, int64_t g, int64_t fifo_start) {
  if (g < a.pn) return a.pidx[g];
  g -= a.pn;
  return a.idx ? a.idx[g] : (fifo_start + g) % a.cap;
}

__device__ __forceinline__ double priority_of(const UpdArgs &a, double alpha, int64_t g) {
  if (g < a.pn) return prio_value(a.ptd, a.pdtype, alpha, g);
  g -= a.pn;
  if (a.w64) return a.w64[g];
  return prio_value(a.td_abs, a.td_dtype, alpha, g);
}

__device__ unsigned long long g_upd_timeouts;  // top-pass waits that timed out (rth_tree_update_timeouts)

// a workgroup barrier that orders LDS only (outstanding global stores are not waited for)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct TopLds;
__device__ __forceinline__ void tree_top(const UpdArgs &a, int S, TopLds &L, unsigned int nsub = 0);

// ---------------------------------------------------------------- subtree pass
// Workgroup w owns the level-S subtrees s with s % gridDim.x == w (consecutive FIFO slots
// sit in consecutive subtrees, so an append spreads over workgroups).  It collects its keys
// in launch order in rounds of <= R keys (rounds in order are the sequential semantics),
// sorts a round by (left-aligned leaf position, depth, slot) -- so every subtree is a
// contiguous run and a node precedes its own subtree -- and lays out one LDS entry per
// touched (node, level): key j owns the levels [lt_j, d_j] of its path that it is the first
// key of (a contiguous range: once an ancestor differs from key j-1's, every deeper one
// does).  All the memory a round needs -- each touched node's val (or its new priority)
// and its children's (sum, min) -- is loaded in one parallel pass; the level loop then runs
// in LDS (each entry pushes its result into its parent's child slot), and the touched
// nodes are stored at the end.  A round whose entries would not fit is re-gathered with
// proportionally fewer keys.
// A leaf key (no children in the tree) gets no entry: its result goes straight into its
// parent's entry, so a contiguous append of 256 leaves fits one round.  LDS (18.2 KB at 320
// entries) fits on a CU beside the learner's conv2 tiles (131 of the 160 KB); 320 entries
// measured faster than 256 (Breakout's 2,048-row append: 4 rounds instead of 5).
constexpr int kSubThreads = 256;
constexpr int kSubKeys = 256;      // keys per round (one per lane; 10 slot bits in the sort key)
constexpr int kSlotBits = 10;
#ifndef SUB_ENTRIES
#define SUB_ENTRIES 320
#endif
constexpr int kSubEntries = SUB_ENTRIES;  // touched (node, level) entries per round
constexpr int kSubGrid = 256;        // workgroups at most
constexpr int kSubGridMin = 64;      // ... and at least
constexpr int kSubKeysPerWg = 12;    // the grid is sized for about this many keys per workgroup
constexpr int kSubSplit = 4;          // the second pass covers S .. S + 3
constexpr int kSubTwoPassDepth = 8;   // two passes when maxd >= S + 8 (trees of >= 2^19 nodes)
constexpr int64_t kTwoPassKeys = 1536;  // ... and the update has at least this many keys (RTH_TREE_PASSES unset)
static_assert(kSubKeys == kSubThreads, "one key per lane in the rank sort / ownership scan");

struct SubEnt {
  double v, ls, lm, rs, rm;  // own val; left / right child (sum, min); ls/lm <- result
};

__device__ __forceinline__ int key_depth(uint64_t k) { return (int)((k >> kSlotBits) & 63); }
__device__ __forceinline__ uint64_t key_aligned(uint64_t k) { return k >> (kSlotBits + 6); }

// exclusive prefix sum over the workgroup (kSubThreads lanes); returns this lane's offset,
// *total = the sum.  Uses wsum[kSubThreads / 64].
__device__ __forceinline__ int wg_scan(int x, int *wsum, int *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  lds_barrier();  // LDS only: a staged top-key atomic (is_mine) is not waited for
  int base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kSubThreads / 64; ++k) {
    const int s = wsum[k];
    if (k < w) base += s;
    tot += s;
  }
  lds_barrier();  // wsum may be reused right away
  *total = tot;
  return base + incl - x;
}

// One pass covers the levels [S, D].  Deep trees take two passes (S1 = S0 + 4): [S1, maxd],
// then [S0, S1 - 1] -- the second pass maps every deeper key to its level-(S1 - 1) ancestor
// as a "valueless" key (its val is kept, its children are final after the first launch), so
// a contiguous FIFO append spreads over many level-S1 subtrees (runs of 2^(d - S1) keys)
// instead of piling into a few level-S0 subtrees and many rounds.
__global__ __launch_bounds__(kSubThreads) void k_tree_update_sub(UpdArgs a, int S, int D, int last_pass) {
  __shared__ uint64_t keys[kSubKeys];
  __shared__ uint64_t scratch[kSubKeys];  // unsorted keys, then ebase[]
  __shared__ int32_t slot_g[kSubKeys];
  __shared__ int8_t elt[kSubKeys];
  __shared__ SubEnt ent[kSubEntries];
  __shared__ int wsum[kSubThreads / 64];
  __shared__ int s_next;
  int32_t *const ebase = reinterpret_cast<int32_t *>(scratch);  // kSubKeys + 1
  const int tid = threadIdx.x;
  const int maxd = a.maxd;
  const int64_t cap = a.cap;
  int64_t fifo_start;
  double alpha;
  upd_prologue(a, &fifo_start, &alpha);
  const int64_t N = a.pn + a.n;
  const int64_t top = (int64_t(1) << S) - 1;  // nodes above level S
  // fuse_top == 2: the last workgroup of the last pass is the top pass, running from the start
  // beside the subtree workgroups (its key scan and its loads of the levels above S overlap
  // them); it waits only for their level-S sums
  const bool early = a.fuse_top == 2 && last_pass;
  const uint32_t G = gridDim.x - (early ? 1u : 0u);
  if (early && blockIdx.x == G) {
    tree_top(a, S, *reinterpret_cast<TopLds *>(ent), G);
    return;
  }
  // key g of this pass: its node (a key below D -> its level-D ancestor, valueless), false
  // when it is not this workgroup's, or a valueless duplicate of the key right before it
  auto is_mine = [&](int64_t g, uint64_t *key, bool *valued) -> bool {
    if (g >= N) return false;
    int64_t id = upd_id(a, g, fifo_start);
    if (id < top) {  // a key above S: the top pass's (workgroup id % G records it, last wins)
      if (last_pass && a.stage && id >= 0 && (uint32_t)(id % G) == blockIdx.x)
        __hip_atomic_fetch_max(&a.stage[kStageFlags + id], (int32_t)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if (id >= cap) return false;
    int d = node_depth(id);
    *valued = d <= D;
    if (d > D) {
      id = ((id + 1) >> (d - D)) - 1;
      d = D;
      if (g > 0) {  // the FIFO run: consecutive keys share their level-D ancestor
        const int64_t pid = upd_id(a, g - 1, fifo_start);
        if (pid >= top && pid < cap) {
          const int pd = node_depth(pid);
          if (pd > D && ((pid + 1) >> (pd - D)) - 1 == id) return false;
        }
      }
    }
    const int64_t sub = ((id + 1) >> (d - S)) - 1 - top;
    const uint64_t al = (uint64_t)(id + 1) << (maxd - d);
    *key = ((al << 6) | (uint64_t)d) << kSlotBits;
    return (uint32_t)(sub % G) == blockIdx.x;
  };
  int64_t scan = 0;
  int R = kSubKeys;
  while (scan < N) {
    // ---- gather the round's keys (launch order) into slots 0..cnt-1; the ids of kGatherU
    // consecutive 256-key windows are loaded together
    constexpr int kGatherU = 4;
    int cnt = 0;
    int64_t pos = scan;
    while (pos < N && cnt < R) {
      bool mine[kGatherU], valued[kGatherU];
      uint64_t kk[kGatherU];  // the sort key's (aligned, depth) part
#pragma unroll
      for (int u = 0; u < kGatherU; ++u) mine[u] = is_mine(pos + u * kSubThreads + tid, &kk[u], &valued[u]);
#pragma unroll
      for (int u = 0; u < kGatherU; ++u) {
        if (pos >= N || cnt >= R) break;  // uniform
        const int64_t g = pos + tid;
        int total;
        const int rank = wg_scan(mine[u] ? 1 : 0, wsum, &total);
        const int take = R - cnt;
        if (tid == 0) s_next = -1;
        lds_barrier();
        if (mine[u] && rank < take) {
          slot_g[cnt + rank] = valued[u] ? (int32_t)g : ~(int32_t)g;  // < 0: valueless
          scratch[cnt + rank] = kk[u] | (uint64_t)(cnt + rank);
        }
        if (mine[u] && rank == take) s_next = (int)(g - pos);  // first key left for the next round
        lds_barrier();
        if (total > take) {
          cnt = R;
          pos += s_next;
        } else {
          cnt += total;
          pos += kSubThreads;
        }
      }
    }
    if (pos > N) pos = N;
    if (cnt == 0) {
      scan = pos;
      continue;
    }
    // ---- sort keys (aligned, depth, slot; built by the gather): rank of each key among the round's
    const int j = tid;
    const uint64_t kmine = j < cnt ? scratch[j] : ~0ull;
    if (j < cnt) {
      int r = 0;
      for (int i = 0; i < cnt; ++i) r += scratch[i] < kmine;
      keys[r] = kmine;
    }
    __syncthreads();  // scratch is reused as ebase / epar below
    // ---- owned level range and entry base of key j
    int own = 0, lf = 0;
    if (j < cnt) {
      const uint64_t kj = keys[j];
      const int dj = key_depth(kj);
      int sh = 0;
      if (j > 0) {
        const uint64_t kp = keys[j - 1];
        const uint64_t x = key_aligned(kj) ^ key_aligned(kp);
        int topl = min(dj, key_depth(kp));
        if (x) topl = min(topl, maxd - (63 - __builtin_clzll(x)) - 1);
        sh = max(0, topl - S + 1);
      }
      elt[j] = (int8_t)(S + sh);
      own = max(0, dj - S + 1 - sh);
      // a leaf below S (no children in the tree) gets no entry: its result (val, val or 1)
      // is known at load time and goes straight into its parent's child slot
      const int64_t nid = (int64_t)(key_aligned(kj) >> (maxd - dj)) - 1;
      lf = own > 0 && dj > S && 2 * nid + 1 >= cap;
    }
    int E;
    const int off = wg_scan(own - lf, wsum, &E);
    if (j < cnt) ebase[j] = off;
    if (E > kSubEntries) {  // uniform: re-gather this round with proportionally fewer keys
      R = max(1, (int)((int64_t)cnt * kSubEntries / E));
      __syncthreads();
      continue;
    }
    __syncthreads();
    const uint64_t k_j = j < cnt ? keys[j] : 0;
    const int lt_j = j < cnt ? elt[j] : 0;
    const int d_j = j < cnt ? key_depth(k_j) : -1;
    const int de_j = d_j - lf;  // the deepest level with an entry
    const int eb_j = j < cnt ? ebase[j] : 0;
    const uint64_t al_j = key_aligned(k_j);
    // ---- parent entry of each key's shallowest owned entry (lower_bound of its owner)
    int ep_j = -1;
    if (j < cnt && own > 0 && lt_j > S) {
      const int L = lt_j - 1;
      const uint64_t al = (al_j >> (maxd - L)) << (maxd - L);
      const uint64_t want = ((al << 6) | (uint64_t)L) << kSlotBits;
      int lo = 0, hi = j;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < want) lo = mid + 1; else hi = mid;
      }
      ep_j = ebase[lo] + (L - elt[lo]);
    }
    // ---- load every entry's inputs (all of a key's levels in flight together; LDS stores
    // cannot alias the loads) and its own node's new priority (the last duplicate's)
    double leaf_v = 0.0;
    if (j < cnt && own > 0) {
      // the node's new val: the last valued duplicate's priority; none -> its val stays
      int32_t g_last = slot_g[k_j & ((1u << kSlotBits) - 1)];
      for (int x = j + 1; x < cnt && (keys[x] >> kSlotBits) == (k_j >> kSlotBits); ++x) {
        const int32_t gx = slot_g[keys[x] & ((1u << kSlotBits) - 1)];
        if (gx >= 0) g_last = gx;
      }
      constexpr int kLoadU = 12;
      for (int L0 = lt_j; L0 <= d_j; L0 += kLoadU) {
        double v[kLoadU], ls[kLoadU], lm[kLoadU], rs[kLoadU], rm[kLoadU];
#pragma unroll
        for (int u = 0; u < kLoadU; ++u) {
          const int L = L0 + u;
          v[u] = ls[u] = lm[u] = rs[u] = rm[u] = 0.0;
          if (L <= d_j) {
            const int64_t node = (int64_t)(al_j >> (maxd - L)) - 1, l = 2 * node + 1;
            if (L < d_j || g_last < 0) v[u] = a.nd[node + 1].val;
            if (l < cap) {
              ls[u] = a.nd[l + 1].sum;
              lm[u] = a.nd[l + 1].mn;
            }
            if (l + 1 < cap) {
              rs[u] = a.nd[l + 2].sum;
              rm[u] = a.nd[l + 2].mn;
            }
          }
        }
        const bool key_val = g_last >= 0 && L0 + kLoadU > d_j;
        const double pv = key_val ? priority_of(a, alpha, g_last) : 0.0;
#pragma unroll
        for (int u = 0; u < kLoadU; ++u) {
          const int L = L0 + u;
          const double vu = L == d_j && key_val ? pv : v[u];
          if (L <= de_j) ent[eb_j + L - lt_j] = SubEnt{vu, ls[u], lm[u], rs[u], rm[u]};
          else if (L == d_j) leaf_v = vu;
        }
      }
    }
    __syncthreads();
    if (lf) {  // _numba_maintain_node of a leaf, pushed into the parent's entry
      const int64_t node = (int64_t)(al_j >> (maxd - d_j)) - 1;
      const int p = d_j > lt_j ? eb_j + (d_j - 1 - lt_j) : ep_j;
      const double mn = (leaf_v != 0.0) ? leaf_v : 1.0;
      if (node & 1) {
        ent[p].ls = leaf_v;
        ent[p].lm = mn;
      } else {
        ent[p].rs = leaf_v;
        ent[p].rm = mn;
      }
    }
    lds_barrier();
    // ---- levels, deepest first (_numba_maintain_node on every touched node, once)
    for (int L = D; L >= S; --L) {
      if (L >= lt_j && L <= de_j) {
        const int e = eb_j + L - lt_j;
        const SubEnt x = ent[e];
        const int64_t node = (int64_t)(al_j >> (maxd - L)) - 1, l = 2 * node + 1;
        double sm = x.v, mn = (x.v != 0.0) ? x.v : 1.0;
        if (l < cap) {
          sm = radd(sm, x.ls);
          if (x.lm != 0.0) mn = (x.lm < mn) ? x.lm : mn;
        }
        if (l + 1 < cap) {
          sm = radd(sm, x.rs);
          if (x.rm != 0.0) mn = (x.rm < mn) ? x.rm : mn;
        }
        ent[e].ls = sm;
        ent[e].lm = mn;
        if (L > S) {
          const int p = L > lt_j ? e - 1 : ep_j;
          if (node & 1) {
            ent[p].ls = sm;
            ent[p].lm = mn;
          } else {
            ent[p].rs = sm;
            ent[p].rm = mn;
          }
        }
      }
      lds_barrier();
    }
    // ---- store the touched nodes (a level-S root write-through: the top pass reads it from
    // another workgroup after the ticket below)
    if (lf) {
      const int64_t node = (int64_t)(al_j >> (maxd - d_j)) - 1;
      a.nd[node + 1].sum = leaf_v;
      a.nd[node + 1].mn = (leaf_v != 0.0) ? leaf_v : 1.0;
      a.nd[node + 1].val = leaf_v;
    }
    if (j < cnt) {
      for (int L = lt_j; L <= de_j; ++L) {
        const SubEnt x = ent[eb_j + L - lt_j];
        const int64_t node = (int64_t)(al_j >> (maxd - L)) - 1;
        if (L == S) {
          __hip_atomic_store(&a.nd[node + 1].sum, x.ls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&a.nd[node + 1].mn, x.lm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (last_pass && a.stage)  // the level-S node was touched (this workgroup owns it)
            __hip_atomic_store(reinterpret_cast<uint8_t *>(a.stage) + (node - top), (uint8_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
          a.nd[node + 1].sum = x.ls;
          a.nd[node + 1].mn = x.lm;
        }
        if (L == d_j) a.nd[node + 1].val = x.v;
      }
    }
    __syncthreads();  // the next round reads these stores (same workgroup)
    scan = pos;
    R = kSubKeys;
  }
  unsigned *const ticket = reinterpret_cast<unsigned *>(&a.nd[0].pad);
  if (early) {  // count this workgroup done once its level-S sums (write-through) have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // ---- ticket: the workgroup that finishes last runs the levels above S (tree_top) in this
  // launch, in the LDS of the entries (no second launch).  The counter lives in the unused
  // record 0 of the node array and is re-armed by that workgroup.
  if (!a.fuse_top || !last_pass) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned tk = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_next = tk == gridDim.x - 1;
    if (s_next) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_next) return;
  if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tree_top(a, S, *reinterpret_cast<TopLds *>(ent));
}

// ---------------------------------------------------------------- top pass
// The levels above S (at most 2^11 - 1 nodes), after the subtree pass, in one 256-lane
// workgroup (small enough to be dispatched beside the learner's kernels).  Lane t owns
// nodes 4t..4t+3 of level S-1, 2t..2t+1 of level S-2 and t of level S-3 (their children
// are its own), and above that the ancestors whose leftmost level-(S-3) descendant is its
// node: node j of level k belongs to lane j << (S-3-k), so a node's left child is on its
// own lane and its right child 2^(S-4-k) lanes up -- a wavefront shuffle below 64 lanes,
// a word in LDS above.  Every record is loaded in one parallel pass; a node is maintained
// iff it is a key or a child was (touched ancestors only -- the min() quirk); last writer
// wins among keys above S.  LDS: the key winners and the touched level-S bitmap (~8.5 KB).
constexpr int kTopS = 11;          // S = max(kTopMinS, min(maxd + 1, kTopS))
constexpr int kTopMinS = 3;        // levels S-1 .. S-3 are lane-local (absent nodes: i >= cap)
constexpr int kTopThreads = 1 << (kTopS - 3);
constexpr int kTopNodes = (1 << kTopS) - 1;
constexpr int kTopRegH = 6;        // shuffle levels h < 6 in registers, the rest (nodes < 7) in LDS

struct TopVal {
  double s, m;
  int t;  // touched
};

__device__ __forceinline__ TopVal top_maintain(double v, bool key, const TopVal &L, const TopVal &R, bool has_l,
                                               bool has_r, double s_old, double m_old) {
  TopVal o{s_old, m_old, 0};
  if (!(key || (has_l && L.t) || (has_r && R.t))) return o;
  double sm = v, mn = (v != 0.0) ? v : 1.0;
  if (has_l) {
    sm = radd(sm, L.s);
    if (L.m != 0.0) mn = (L.m < mn) ? L.m : mn;
  }
  if (has_r) {
    sm = radd(sm, R.s);
    if (R.m != 0.0) mn = (R.m < mn) ? R.m : mn;
  }
  return TopVal{sm, mn, 1};
}

struct TopRec {
  double v, s, m;
};

__device__ __forceinline__ TopRec top_load(const Node *nd, int64_t cap, int64_t i) {
  TopRec r{0.0, 0.0, 0.0};
  if (i < cap) {
    const Node x = nd[i + 1];
    r = TopRec{x.val, x.sum, x.mn};
  }
  return r;
}

// one node: maintain (if touched) and store what changed
__device__ __forceinline__ TopVal top_node(const UpdArgs &a, int64_t i, const TopRec &r, bool key, const TopVal &L,
                                           const TopVal &R) {
  const int64_t l = 2 * i + 1;
  const TopVal o = top_maintain(r.v, key, L, R, l < a.cap, l + 1 < a.cap, r.s, r.m);
  if (key) a.nd[i + 1].val = r.v;
  if (o.t) {
    a.nd[i + 1].sum = o.s;
    a.nd[i + 1].mn = o.m;
  }
  return o;
}

// LDS of the top pass, carved from one buffer: run by its own launch, or by the subtree
// pass's last workgroup in the LDS its level loop no longer needs
struct TopLds {
  int32_t win[kTopNodes];
  uint32_t bot[(kTopNodes + 1) / 32];
  double xs[8], xm[8];
  int xt[8];
  double uv[8], us[8], um[8];  // records of the levels above the register slots
  int ukey[8];
};

// nsub > 0: run as the extra workgroup of a subtree launch (fuse_top == 2): everything that
// does not depend on the subtree pass first (the key scan, the records above level S, the key
// priorities), then wait until its nsub workgroups have counted themselves done (the ticket
// word, re-armed here), then load the level-S sums they wrote
__device__ __forceinline__ void tree_top(const UpdArgs &a, int S, TopLds &L, unsigned int nsub) {
  int32_t *const win = L.win;
  uint32_t *const bot = L.bot;
  double *const xs = L.xs, *const xm = L.xm, *const uv = L.uv, *const us = L.us, *const um = L.um;
  int *const xt = L.xt, *const ukey = L.ukey;
  const int t = threadIdx.x;
  const int64_t cap = a.cap;
  int64_t fifo_start;
  double alpha;
  upd_prologue(a, &fifo_start, &alpha);
  const int64_t N = a.pn + a.n;
  const int ntop = (1 << S) - 1;
  const int n3 = 1 << (S - 3);  // nodes of level S-3 (one per lane)
  const bool lane = t < n3;
  // ---- every record this lane maintains, loads in flight together
  const int64_t b1 = (int64_t)(4 * n3) - 1 + 4 * t;  // level S-1: b1 .. b1+3
  const int64_t b2 = (int64_t)(2 * n3) - 1 + 2 * t;  // level S-2: b2, b2+1
  TopRec r1[4], r2[2], rr[kTopRegH];
  double cs[8], cm[8];  // level S children of the level S-1 nodes
#pragma unroll
  for (int q = 0; q < 4; ++q) r1[q] = top_load(a.nd, lane ? cap : 0, b1 + q);
  auto load_children = [&]() {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int64_t l = 2 * b1 + 1 + c;
      cs[c] = cm[c] = 0.0;
      if (lane && l < cap) {
        cs[c] = a.nd[l + 1].sum;
        cm[c] = a.nd[l + 1].mn;
      }
    }
  };
  if (!nsub) load_children();
#pragma unroll
  for (int q = 0; q < 2; ++q) r2[q] = top_load(a.nd, lane ? cap : 0, b2 + q);
  // shuffle slot h = S-3-k holds level k (lane t owns it when t is a multiple of 2^h):
  // node (2^k - 1) + (t >> h); levels k <= S-3-kTopRegH (nodes < 7) go through LDS
#pragma unroll
  for (int h = 0; h < kTopRegH; ++h) {
    rr[h] = TopRec{0.0, 0.0, 0.0};
    if (h <= S - 3 && lane && (t & ((1 << h) - 1)) == 0) {
      const int k = S - 3 - h;
      rr[h] = top_load(a.nd, cap, ((int64_t)1 << k) - 1 + (t >> h));
    }
  }
  const bool lds_rec = t < 7 && t < cap && node_depth(t) <= S - 3 - kTopRegH;
  if (lds_rec) {
    const TopRec x = top_load(a.nd, cap, t);
    uv[t] = x.v;
    us[t] = x.s;
    um[t] = x.m;
  }
  // ---- keys: the last writer of each node this lane maintains (w1, w2, wr, wu) and the
  // touched flags of its level-S children (mb, 8 bits) -- staged by the subtree pass, or
  // found by a scan of the keys
  const bool staged = a.stage != nullptr;
  int32_t w1[4], w2[2], wr[kTopRegH], wu = -1;
  uint32_t mb = 0;
  uint64_t flags8 = 0;  // staged: the touched flags of this lane's 8 level-S children, one byte each
  auto node_ok = [&](int64_t i) { return lane && i < cap; };
  auto stage_win = [&](int64_t i) -> int32_t {
    return __hip_atomic_load(&a.stage[kStageFlags + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (staged) {  // S == kTopS here: every lane owns a level S-3 node
#pragma unroll
    for (int q = 0; q < 4; ++q) w1[q] = node_ok(b1 + q) ? stage_win(b1 + q) : -1;
#pragma unroll
    for (int q = 0; q < 2; ++q) w2[q] = node_ok(b2 + q) ? stage_win(b2 + q) : -1;
#pragma unroll
    for (int h = 0; h < kTopRegH; ++h) {
      const int64_t i = ((int64_t)1 << (S - 3 - h)) - 1 + (t >> h);
      wr[h] = (h <= S - 3 && (t & ((1 << h) - 1)) == 0 && node_ok(i)) ? stage_win(i) : -1;
    }
    if (lds_rec) wu = stage_win(t);
    flags8 = lane ? __hip_atomic_load(reinterpret_cast<uint64_t *>(a.stage) + t, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT)
                  : 0ull;
#pragma unroll
    for (int c = 0; c < 8; ++c) mb |= (uint32_t)((flags8 >> (8 * c)) & 1u) << c;
  } else {
  for (int i = t; i < ntop; i += kTopThreads) win[i] = -1;
  for (int i = t; i < (kTopNodes + 1) / 32; i += kTopThreads) bot[i] = 0u;
  __syncthreads();
  constexpr int kScanU = 4;
  for (int64_t g0 = 0; g0 < N; g0 += kScanU * kTopThreads) {
    int64_t id[kScanU];
#pragma unroll
    for (int u = 0; u < kScanU; ++u) {
      const int64_t g = g0 + u * kTopThreads + t;
      id[u] = g < N ? upd_id(a, g, fifo_start) : -1;
    }
#pragma unroll
    for (int u = 0; u < kScanU; ++u) {
      if (id[u] < 0 || id[u] >= cap) continue;
      if (id[u] < ntop) {
        atomicMax(&win[id[u]], (int32_t)(g0 + u * kTopThreads + t));
      } else {
        const int d = node_depth(id[u]);
        const int b = (int)(((id[u] + 1) >> (d - S)) - 1 - ntop);
        atomicOr(&bot[b >> 5], 1u << (b & 31));
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) w1[q] = node_ok(b1 + q) ? win[b1 + q] : -1;
#pragma unroll
  for (int q = 0; q < 2; ++q) w2[q] = node_ok(b2 + q) ? win[b2 + q] : -1;
#pragma unroll
  for (int h = 0; h < kTopRegH; ++h) {
    const int64_t i = ((int64_t)1 << (S - 3 - h)) - 1 + (t >> h);
    wr[h] = (h <= S - 3 && (t & ((1 << h) - 1)) == 0 && node_ok(i)) ? win[i] : -1;
  }
  if (lds_rec) wu = win[t];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int b = 8 * t + c;
    if (lane && b < (1 << S)) mb |= ((bot[b >> 5] >> (b & 31)) & 1u) << c;
  }
  }
  // ---- new priorities of this lane's key nodes (before the level loop: it issues no loads,
  // so its stores are never waited for)
  int key1 = 0, key2 = 0, keyr = 0;
  if (lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (w1[q] >= 0) {
        r1[q].v = priority_of(a, alpha, w1[q]);
        key1 |= 1 << q;
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (w2[q] >= 0) {
        r2[q].v = priority_of(a, alpha, w2[q]);
        key2 |= 1 << q;
      }
    }
#pragma unroll
    for (int h = 0; h < kTopRegH; ++h) {
      if (wr[h] >= 0) {
        rr[h].v = priority_of(a, alpha, wr[h]);
        keyr |= 1 << h;
      }
    }
  }
  if (lds_rec) {
    ukey[t] = wu >= 0;
    if (wu >= 0) uv[t] = priority_of(a, alpha, wu);
  }
  __syncthreads();
  // a timed-out wait (never seen: the extra workgroup is dispatched after every subtree
  // workgroup) leaves the levels above S unwritten -- maintaining them from level-S sums not
  // yet written would corrupt them silently -- and is counted (rth_tree_update_timeouts)
  __shared__ int tmo;
  if (nsub) {  // wait for the subtree workgroups (bounded: a timeout is recorded, not hung on)
    if (t == 0) {
      unsigned *const done = reinterpret_cast<unsigned *>(&a.nd[0].pad);
      unsigned spins = 0;
      while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nsub && spins < (1u << 24)) {
        __builtin_amdgcn_s_sleep(2);
        ++spins;
      }
      tmo = spins >= (1u << 24);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // re-arm by subtracting this launch's count (not a store of 0): after a timeout the late
      // workgroups' increments still land and bring the word back to 0
      __hip_atomic_fetch_sub(done, nsub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tmo) atomicAdd(&g_upd_timeouts, 1ull);
    }
    __syncthreads();
    load_children();
  }
  const bool write_top = nsub == 0 || tmo == 0;  // uniform (tmo written before the barrier above)
  // ---- the lane-local levels S-1, S-2, S-3
  TopVal cur{0.0, 0.0, 0};
  if (lane && write_top) {
    TopVal v1[4], v2[2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const TopVal L{cs[2 * q], cm[2 * q], (int)((mb >> (2 * q)) & 1u)};
      const TopVal R{cs[2 * q + 1], cm[2 * q + 1], (int)((mb >> (2 * q + 1)) & 1u)};
      v1[q] = b1 + q < cap ? top_node(a, b1 + q, r1[q], (key1 >> q) & 1, L, R) : TopVal{0.0, 0.0, 0};
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
      v2[q] = b2 + q < cap ? top_node(a, b2 + q, r2[q], (key2 >> q) & 1, v1[2 * q], v1[2 * q + 1])
                           : TopVal{0.0, 0.0, 0};
    const int64_t i3 = (int64_t)n3 - 1 + t;
    if (i3 < cap) cur = top_node(a, i3, rr[0], keyr & 1, v2[0], v2[1]);
  }
  // ---- levels S-4 .. 0 (slot h = S-3-k): left child on this lane, right child 2^(h-1) lanes up
#pragma unroll
  for (int h = 1; h <= kTopS - 3; ++h) {
    if (h <= S - 3 && write_top) {  // uniform
      const int k = S - 3 - h;
      const int d = 1 << (h - 1);
      TopVal R;
      if (d < 64) {
        R.s = __shfl_down(cur.s, d, 64);
        R.m = __shfl_down(cur.m, d, 64);
        R.t = __shfl_down(cur.t, d, 64);
      } else {
        // right children of level k+1 (node ids < 7: k + 1 <= S - 10 <= 1) through LDS;
        // level k+1 is owned by the multiples of d
        if (lane && (t & (d - 1)) == 0 && ((t >> (h - 1)) & 1)) {
          const int node = (1 << (k + 1)) - 1 + (t >> (h - 1));
          xs[node] = cur.s;
          xm[node] = cur.m;
          xt[node] = cur.t;
        }
        lds_barrier();  // LDS only: the level loop's global stores are never waited for
        R = TopVal{0.0, 0.0, 0};
        if (lane && (t & ((1 << h) - 1)) == 0) {
          const int rn = 2 * ((1 << k) - 1 + (t >> h)) + 2;
          R = TopVal{xs[rn], xm[rn], xt[rn]};
        }
        lds_barrier();
      }
      const int64_t i = ((int64_t)1 << k) - 1 + (t >> h);
      if (lane && (t & ((1 << h) - 1)) == 0 && i < cap) {
        const bool reg = h < kTopRegH;
        const int hr = reg ? h : 0;
        const TopRec rec = reg ? rr[hr] : TopRec{uv[i & 7], us[i & 7], um[i & 7]};
        const bool key = reg ? ((keyr >> hr) & 1) : ukey[i & 7] != 0;
        cur = top_node(a, i, rec, key, cur, R);
      }
    }
  }
  if (staged) {  // re-arm what this lane read (its values are consumed: no load is pending)
    auto clear = [&](int64_t i) {
      __hip_atomic_store(&a.stage[kStageFlags + i], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (w1[q] >= 0) clear(b1 + q);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (w2[q] >= 0) clear(b2 + q);
#pragma unroll
    for (int h = 0; h < kTopRegH; ++h)
      if (wr[h] >= 0) clear(((int64_t)1 << (S - 3 - h)) - 1 + (t >> h));
    if (wu >= 0) clear(t);
    if (flags8)
      __hip_atomic_store(reinterpret_cast<uint64_t *>(a.stage) + t, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t == 0) {
    if (a.st) {
      if (a.pre_step) a.st->sched_step += 1;
      if (a.post_tail) a.st->tail = (fifo_start + a.n) % cap;  // every read of tail is done
    }
  }
}

__global__ __launch_bounds__(kTopThreads) void k_tree_update_top(UpdArgs a, int S) {
  __shared__ TopLds lds;
  tree_top(a, S, lds);
}
static_assert(sizeof(TopLds) <= sizeof(SubEnt) * kSubEntries, "the top pass reuses the subtree pass's entry LDS");
static_assert(kTopThreads == kSubThreads, "the subtree pass's last workgroup runs the top pass");

// ------------------------------------------------------------------ find / sample
// target i of a launch with gk > 0 (groups of 2^gk lanes) or gk == 0 (one lane each)
struct FindLane {
  int64_t i;
  int base, sub;
};
__device__ __forceinline__ FindLane find_lane(int gk) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gk == 0) return FindLane{g, 0, 0};
  const int lane = threadIdx.x & 63, sub = lane & ((1 << gk) - 1);
  return FindLane{g >> gk, lane - sub, sub};
}

__global__ void k_tree_find(const Node *__restrict__ nd, int64_t cap, const double *__restrict__ tg,
                            int64_t n, int64_t *__restrict__ idx_out, double *__restrict__ val_out, int kspec,
                            int gk) {
  const FindLane fl = find_lane(gk);
  const int64_t i = fl.i;
  if (i >= n) return;  // uniform over a group
  const int64_t k = gk ? tree_find_grouped(nd, cap, tg[i], gk, fl.base, fl.sub) : tree_find(nd, cap, tg[i], kspec);
  if (fl.sub) return;
  if (idx_out) idx_out[i] = k;
  if (val_out) val_out[i] = nd[k + 1].val;
}

// r05: the sample at its latency floor.  Every workgroup stages the top TL levels of the tree
// ({sum, val} of 2^TL - 1 nodes; 16 KB at TL = 10) with ALL its loads in flight at once -- one
// round trip -- plus the root's min for the IS weights; each lane walks those levels in LDS
// (the reference's comparisons and subtractions, lds_top_walk) and the levels below in round
// trips of K levels: the 2^K - 1 child pairs of the K-deep subtree under its node are loaded
// together, unconditionally (clamped record indices; an absent child is zeroed after the load,
// so no load waits behind a branch), then K steps run on registers.  The sampled node's val
// comes from the walk itself (the val find_step compared against), not from another load.
// Pong's 1 M-row tree (depth 20): 10 levels in LDS + 5 round trips of 2 levels (K = 2).
// Same comparisons in the same order as tree_find: bit-identical indices.
__device__ __forceinline__ Pair load_pair_u(const Node *__restrict__ nd, int64_t cap, int64_t c) {
  const int64_t l = 2 * c + 1;
  const int64_t lc = l < cap ? l : cap - 1;  // record lc + 2 <= cap + 1 exists (padding)
  const double2 L = *reinterpret_cast<const double2 *>(&nd[lc + 1]);
  const double rv = nd[lc + 2].val;
  const bool in = l < cap;
  return Pair{in ? L.x : 0.0, in ? L.y : 0.0, in ? rv : 0.0};
}

template <int K>
__device__ __forceinline__ int64_t tree_find_kv(const Node *__restrict__ nd, int64_t cap, double w, int64_t cur,
                                                double &cval) {
  constexpr int NP = (1 << K) - 1;
  for (;;) {
    Pair p[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int dq = 31 - __builtin_clz(q + 1);
      const int64_t node = (cur + 1) * (int64_t(1) << dq) - 1 + (q + 1 - (1 << dq));
      p[q] = load_pair_u(nd, cap, node);
    }
    int q = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      Pair pk = p[0];
#pragma unroll
      for (int j = 1; j < NP; ++j)
        if (j == q) pk = p[j];
      const int64_t before = cur;
      if (!find_step(cur, cval, w, pk, cap)) return cur;
      q = 2 * q + 1 + (int)(cur - (2 * before + 1));
    }
  }
}

#ifndef DEEP_THREADS
#define DEEP_THREADS 256
#endif
// 256 lanes per workgroup (r05 A/B in the loop, Pong: K = 2 18-19 us, K = 3 23-24, K = 4 37;
// one-wave workgroups (DEEP_THREADS=64) 26-27 / 27-28 / 30 -- eight 16 KB workgroups wait for
// CU slots beside the learner's kernels longer than two do; r04's kernel 27-33)
constexpr int kDeepThreads = DEEP_THREADS;

// TL levels staged (2^TL - 1 nodes x 16 B: 16 KB at TL = 10 -- small enough to be dispatched
// on a CU beside the learner's conv2 workgroup, which holds 128 KB of the 160; 64 KB at TL = 12
// was not, and waited for a free CU in the loop: 41 vs 28 us, r05 A/B)
template <int TL, int K>
__global__ __launch_bounds__(kDeepThreads) void k_tree_sample_deep(
    const Node *__restrict__ nd, int64_t cap, int64_t batch, const double *__restrict__ uniforms, uint64_t seed,
    uint64_t counter, int is_weights, double beta, const ReplayState *st, rth_schedule beta_s,
    int64_t *__restrict__ idx_out, double *__restrict__ out) {
  constexpr int kDeepNodes = (1 << TL) - 1;
  __shared__ double2 topl[kDeepNodes];
  __shared__ double min_sh;
  const int64_t nst = cap < kDeepNodes ? cap : kDeepNodes;
  constexpr int PER = (kDeepNodes + kDeepThreads - 1) / kDeepThreads;
  {
    double2 tmp[PER];  // every staging load in flight before the first LDS write
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int64_t n = threadIdx.x + (int64_t)kDeepThreads * j;
      tmp[j] = *reinterpret_cast<const double2 *>(&nd[(n < nst ? n : nst - 1) + 1]);
    }
    if (threadIdx.x == 0) {
      const Node root = nd[1];
      min_sh = root.sum != 0.0 ? root.mn : 1.0;  // tree_min (NumbaSumTree.min, sumtree.py:109-110)
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // unconditional (a clamped lane rewrites node nst - 1 with its
      const int64_t n = threadIdx.x + (int64_t)kDeepThreads * j;  // own value): no load sinks into a branch
      topl[n < nst ? n : nst - 1] = tmp[j];
    }
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kDeepThreads + threadIdx.x;
  if (i >= batch) return;
  if (st) {
    counter = (uint64_t)st->calls;
    beta = sched_value(beta_s, st->sched_step);
  }
  const double seg = topl[0].x / (double)batch;
  const double u = uniforms ? uniforms[i] : philox_uniform(seed, counter, (uint32_t)i, STREAM_SAMPLE);
  double t = rmul(radd((double)i, u), seg);
  int64_t k;
  double cval;
  if (!lds_top_walk(topl, cap, nst, k, cval, t)) {
    // k is the answer, cval its val
  } else {
    k = tree_find_kv<K>(nd, cap, t, k, cval);
  }
  idx_out[i] = k;
  if (is_weights) {
    out[i] = pow(cval / min_sh, -beta);
  } else if (out) {
    out[i] = cval;
  }
}

__global__ void k_tree_stats(const Node *nd, double *out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = nd[1].sum;
    out[1] = tree_min(nd);
  }
}

__global__ void k_tree_export(const Node *nd, int64_t cap, double *s, double *m, double *v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const Node x = nd[i + 1];
  if (s) s[i] = x.sum;
  if (m) m[i] = x.mn;
  if (v) v[i] = x.val;
}

__global__ void k_tree_import(Node *nd, int64_t cap, const double *s, const double *m, const double *v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  nd[i + 1] = Node{s[i], v[i], m[i], 0.0};
}

__global__ void k_per_normalize(const float *w, int64_t n, float alpha, float *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = per_normalize(w[i], alpha);
}

}  // namespace rth

using namespace rth;

struct rth_sumtree {
  int64_t cap;
  int device;
  int maxd;
  Node *nodes;
  int32_t *stage;  // UpdArgs::stage: behind the nodes in the same allocation, kept re-armed
};

namespace rth {
constexpr size_t kStageInts = kStageFlags + kTopNodes;
}

namespace rth {
int tree_update_impl(rth_sumtree *t, const int64_t *idx, int64_t fifo_start, const double *w64,
                     const void *td_abs, int32_t td_dtype, double alpha, int64_t n, hipStream_t s,
                     ReplayState *st, const rth_schedule *alpha_s, const UpdPending *pend, int post_tail) {
  const bool has_pend = pend && (pend->n > 0 || pend->step);
  if (n <= 0 && !has_pend && !post_tail) return RTH_OK;
  if (n > 0 && !w64 && td_dtype == RTH_PRIO_RAW) w64 = static_cast<const double *>(td_abs);  // stored as given
  RTH_REQUIRE(n <= 0 || w64 || td_dtype == RTH_F32 || td_dtype == RTH_F64,
              "priority dtype must be f32, f64 or raw f64");
  RTH_REQUIRE(!(has_pend || post_tail) || st, "deferred updates and FIFO bumps need a replay state");
  UpdArgs a{t->nodes, t->cap, t->maxd, idx, fifo_start, w64, td_abs, td_dtype, alpha, n > 0 ? n : 0, st,
            alpha_s ? *alpha_s : rth_schedule{}};
  if (has_pend) {
    RTH_REQUIRE(pend->n <= 0 || (pend->idx && pend->td && (pend->dtype == RTH_F32 || pend->dtype == RTH_F64 ||
                                                          pend->dtype == RTH_PRIO_RAW)),
                "deferred update: bad arguments");
    a.pidx = pend->idx;
    a.ptd = pend->td;
    a.pdtype = pend->dtype;
    a.pn = pend->n > 0 ? pend->n : 0;
    a.pre_step = pend->step ? 1 : 0;
  }
  a.post_tail = post_tail;
  // the top pass runs as one more workgroup of the subtree launch (fuse_top 2, r05): its key scan
  // and its loads of the records above level S overlap the subtree pass (Pong 41-42 vs 51-52 us
  // per launch in the loop against the r02-r04 form run by the subtree pass's last workgroup);
  // it is dispatched last, after every subtree workgroup, so its bounded wait never holds a slot
  // they need.  Trees too shallow for a subtree pass run k_tree_update_top alone.
  a.fuse_top = 2;
  RTH_REQUIRE(a.pn + a.n < (int64_t(1) << 31), "tree update: at most 2^31 - 1 keys per call");
  const int S = t->maxd + 1 < kTopMinS ? kTopMinS : (t->maxd + 1 < kTopS ? t->maxd + 1 : kTopS);
  if (t->maxd >= S && a.pn + a.n > 0) {  // levels S..maxd: one workgroup per group of subtrees,
    // deep trees in two passes split at S1 = S + kSubSplit.  RTH_TREE_PASSES: 1 / 2 fixed (read
    // per call: tests drive both shipped forms at every size); unset (0): two passes for large
    // updates -- Breakout's 2,048-row append is one run of leaves, which a single pass hands to
    // the one or two workgroups owning its level-S subtrees (alone 56-57 vs 34-35 us)
    const int passes_env = env_int("RTH_TREE_PASSES", 0);
    const int passes = passes_env > 0 ? passes_env : (a.pn + a.n >= kTwoPassKeys ? 2 : 1);
    // fewer workgroups for small updates: less dispatch and L2 traffic beside the learner
    // stream (Pong's 768 keys: 64 workgroups, 0.617-0.620 vs 0.618-0.625 ms/step with 256;
    // Breakout's 2,560 keys keep 256)
    int grid = kSubGridMin;
    while (grid < kSubGrid && (int64_t)grid * kSubKeysPerWg < a.pn + a.n) grid *= 2;
    const int S1 = S + kSubSplit;
    const bool two = passes >= 2 && t->maxd >= S + kSubTwoPassDepth;
    if (two) {
      const int64_t nsub1 = int64_t(1) << S1;
      hipLaunchKernelGGL(k_tree_update_sub, dim3((unsigned)(nsub1 < grid ? nsub1 : grid)), dim3(kSubThreads), 0, s,
                         a, S1, t->maxd, 0);
      RTH_LAUNCHED();
    }
    const int64_t nsub = int64_t(1) << S;
    const unsigned g_last = (unsigned)(nsub < grid ? nsub : grid);
    // the top pass is the launch's extra last workgroup and scans the keys itself
    a.stage = nullptr;
    hipLaunchKernelGGL(k_tree_update_sub, dim3(g_last + 1u), dim3(kSubThreads), 0, s, a, S, two ? S1 - 1 : t->maxd, 1);
    RTH_LAUNCHED();
    return RTH_OK;
  }
  hipLaunchKernelGGL(k_tree_update_top, dim3(1), dim3(kTopThreads), 0, s, a, S);
  RTH_LAUNCHED();
  return RTH_OK;
}
int tree_sample_impl(rth_sumtree *t, int64_t batch, const double *uniforms, uint64_t seed,
                     uint64_t counter, int is_weights, double beta, int64_t *idx_out, double *out,
                     hipStream_t s, const ReplayState *st, const rth_schedule *beta_s) {
  if (batch <= 0) return RTH_OK;
  // k_tree_sample_deep (r05): the top 10 levels staged per 256-lane workgroup, then 2 levels per
  // HBM round trip below (r04's one-level walk, k_tree_sample: 27-33 vs 17-19 us per Pong launch)
  const Node *nd = t->nodes;
  int64_t cap = t->cap;
  rth_schedule bs_ = beta_s ? *beta_s : rth_schedule{};
  void *args[] = {(void *)&nd, (void *)&cap, (void *)&batch, (void *)&uniforms, (void *)&seed, (void *)&counter,
                  (void *)&is_weights, (void *)&beta, (void *)&st, (void *)&bs_, (void *)&idx_out, (void *)&out};
  RTH_HIP(hipLaunchKernel(reinterpret_cast<const void *>(&k_tree_sample_deep<10, 2>),
                          dim3((unsigned)((batch + kDeepThreads - 1) / kDeepThreads)), dim3(kDeepThreads), args, 0, s));
  return RTH_OK;
}
}  // namespace rth

extern "C" {

int rth_sumtree_create(int64_t capacity, int device, rth_sumtree **out) {
  RTH_REQUIRE(out != nullptr, "rth_sumtree_create: out is NULL");
  RTH_REQUIRE(capacity >= 1 && capacity < kMaxCapacity, "rth_sumtree_create: capacity %lld out of range",
              (long long)capacity);
  RTH_HIP(hipSetDevice(device));
  Node *nodes = nullptr;
  const size_t node_bytes = (size_t)(capacity + 2) * sizeof(Node);
  const size_t bytes = node_bytes + kStageInts * sizeof(int32_t);
  if (hipMalloc(&nodes, bytes) != hipSuccess) {
    set_error("rth_sumtree_create: hipMalloc(%zu) failed", bytes);
    return RTH_ERR_NOMEM;
  }
  RTH_HIP(hipMemset(nodes, 0, node_bytes + kStageFlags * sizeof(int32_t)));  // no touched flag,
  int32_t *stage = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(nodes) + node_bytes);
  RTH_HIP(hipMemset(stage + kStageFlags, 0xff, kTopNodes * sizeof(int32_t)));  // no key (-1) on any top node
  auto *t = new rth_sumtree{capacity, device, node_depth(capacity - 1), nodes, stage};
  *out = t;
  return RTH_OK;
}

int rth_sumtree_destroy(rth_sumtree *t) {
  if (!t) return RTH_OK;
  (void)hipSetDevice(t->device);
  (void)hipFree(t->nodes);
  delete t;
  return RTH_OK;
}

int64_t rth_sumtree_capacity(const rth_sumtree *t) { return t ? t->cap : -1; }

int rth_sumtree_clear(rth_sumtree *t, void *stream) {
  RTH_REQUIRE(t, "rth_sumtree_clear: NULL tree");
  RTH_HIP(hipMemsetAsync(t->nodes, 0, (size_t)(t->cap + 2) * sizeof(Node), as_stream(stream)));
  return RTH_OK;
}

int rth_tree_update_timeouts(int64_t *out) {
  RTH_REQUIRE(out, "rth_tree_update_timeouts: NULL");
  unsigned long long v = 0;
  RTH_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_upd_timeouts), sizeof(v)));
  *out = (int64_t)v;
  return RTH_OK;
}

int rth_sumtree_update(rth_sumtree *t, const int64_t *idx, const double *w, int64_t n, void *stream) {
  RTH_REQUIRE(t && (n == 0 || (idx && w)), "rth_sumtree_update: bad arguments");
  return tree_update_impl(t, idx, 0, w, nullptr, RTH_F64, 0.0, n, as_stream(stream), nullptr, nullptr, nullptr, 0);
}

int rth_sumtree_find(rth_sumtree *t, const double *tg, int64_t n, int64_t *idx_out, double *val_out,
                     void *stream) {
  RTH_REQUIRE(t && (n == 0 || tg), "rth_sumtree_find: bad arguments");
  if (n == 0) return RTH_OK;
  const int64_t lanes = n << kFindGroupK;
  hipLaunchKernelGGL(k_tree_find, dim3((unsigned)((lanes + kFindThreads - 1) / kFindThreads)), dim3(kFindThreads), 0,
                     as_stream(stream), t->nodes, t->cap, tg, n, idx_out, val_out, kFindK, kFindGroupK);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_sumtree_sample(rth_sumtree *t, int64_t batch, const double *uniforms, uint64_t seed,
                       uint64_t counter, int64_t *idx_out, double *val_out, void *stream) {
  RTH_REQUIRE(t && batch > 0 && idx_out, "rth_sumtree_sample: bad arguments");  // assert batch_size > 0 (:73)
  return tree_sample_impl(t, batch, uniforms, seed, counter, 0, 0.0, idx_out, val_out, as_stream(stream), nullptr,
                          nullptr);
}

int rth_sumtree_stats(rth_sumtree *t, double *out2, void *stream) {
  RTH_REQUIRE(t && out2, "rth_sumtree_stats: bad arguments");
  hipLaunchKernelGGL(k_tree_stats, dim3(1), dim3(64), 0, as_stream(stream), t->nodes, out2);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_sumtree_export(rth_sumtree *t, double *s, double *m, double *v, void *stream) {
  RTH_REQUIRE(t, "rth_sumtree_export: NULL tree");
  const int bs = 256;
  hipLaunchKernelGGL(k_tree_export, dim3((unsigned)((t->cap + bs - 1) / bs)), dim3(bs), 0,
                     as_stream(stream), t->nodes, t->cap, s, m, v);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_sumtree_import(rth_sumtree *t, const double *s, const double *m, const double *v, void *stream) {
  RTH_REQUIRE(t && s && m && v, "rth_sumtree_import: bad arguments");
  const int bs = 256;
  hipLaunchKernelGGL(k_tree_import, dim3((unsigned)((t->cap + bs - 1) / bs)), dim3(bs), 0,
                     as_stream(stream), t->nodes, t->cap, s, m, v);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_per_normalize(const float *w, int64_t n, float alpha, float *out, void *stream) {
  RTH_REQUIRE(n == 0 || (w && out), "rth_per_normalize: bad arguments");
  if (n == 0) return RTH_OK;
  const int bs = 256;
  hipLaunchKernelGGL(k_per_normalize, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, as_stream(stream),
                     w, n, alpha, out);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_per_update(rth_sumtree *t, const int64_t *idx, const void *td_abs, int32_t td_dtype, int64_t n,
                   double alpha, void *stream) {
  RTH_REQUIRE(t && (n == 0 || (idx && td_abs)), "rth_per_update: bad arguments");
  return tree_update_impl(t, idx, 0, nullptr, td_abs, td_dtype, alpha, n, as_stream(stream), nullptr, nullptr,
                          nullptr, 0);
}

int rth_per_sample(rth_sumtree *t, int64_t batch, double beta, const double *uniforms, uint64_t seed,
                   uint64_t counter, int64_t *idx_out, double *isw_out, void *stream) {
  RTH_REQUIRE(t && batch > 0 && idx_out && isw_out, "rth_per_sample: bad arguments");
  return tree_sample_impl(t, batch, uniforms, seed, counter, 1, beta, idx_out, isw_out, as_stream(stream), nullptr,
                          nullptr);
}

}  // extern "C"
