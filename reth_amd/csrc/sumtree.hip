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
//   zero node).  Two launches:
//   * k_tree_update_sub: the levels S..maxd (S = 11), one workgroup per group of level-S
//     subtrees (256 workgroups); each sorts its keys by left-aligned leaf position, loads
//     everything its touched nodes need in one parallel pass, runs the level loop in LDS and
//     stores the touched nodes once;
//   * k_tree_update_top: the 2^S - 1 nodes above level S, dense in LDS, from the level-S
//     sums the first launch left in memory.
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
__device__ __forceinline__ int64_t tree_find_k(const Node *__restrict__ nd, int64_t cap, double w) {
  constexpr int NP = (1 << K) - 1;  // pairs per round trip: c's subtree down to depth K-1
  int64_t cur = 0;
  double cval = nd[1].val;
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

__device__ __forceinline__ int64_t tree_find(const Node *__restrict__ nd, int64_t cap, double w, int kspec = 2) {
  switch (kspec) {
    case 1: return tree_find_k<1>(nd, cap, w);
    case 4: return tree_find_k<4>(nd, cap, w);
    case 3: return tree_find_k<3>(nd, cap, w);
    default: return tree_find_k<2>(nd, cap, w);
  }
}

// tuning aids: levels per round trip and sample workgroup size (RTH_FIND_K, RTH_SAMPLE_BS)
static int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}
static int find_k() {
  static const int k = env_int("RTH_FIND_K", 2);
  return k;
}
static int sample_bs() {
  static const int b = env_int("RTH_SAMPLE_BS", 64);
  return b;
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
};

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

// phase timestamps of the last update (wall clock ticks, 100 MHz; development aid, read by
// rth_debug_tree_timing): [0] subtree pass start, [1] its end (workgroup 0), [2] top pass
// start, [3] top pass after its loads and key scan, [4] top pass end
__device__ long long g_upd_clock[8];

// a workgroup barrier that orders LDS only (outstanding global stores are not waited for)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

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
// half the keys.
constexpr int kSubThreads = 256;
constexpr int kSubKeys = 1024;     // keys per round (10 slot bits in the sort key)
constexpr int kSlotBits = 10;
constexpr int kSubEntries = 2560;  // touched (node, level) entries per round
constexpr int kSubGrid = 256;

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
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kSubThreads / 64; ++k) {
    const int s = wsum[k];
    if (k < w) base += s;
    tot += s;
  }
  __syncthreads();  // wsum may be reused right away
  *total = tot;
  return base + incl - x;
}

__global__ __launch_bounds__(kSubThreads) void k_tree_update_sub(UpdArgs a, int S) {
  __shared__ uint64_t keys[kSubKeys];
  __shared__ int32_t slot_g[kSubKeys];
  __shared__ int32_t ebase[kSubKeys + 1];
  __shared__ int32_t epar[kSubKeys];
  __shared__ int8_t elt[kSubKeys];
  __shared__ SubEnt ent[kSubEntries];
  __shared__ int wsum[kSubThreads / 64];
  __shared__ int s_next;
  const int tid = threadIdx.x;
  const int maxd = a.maxd;
  const int64_t cap = a.cap;
  if (tid == 0 && blockIdx.x == 0) g_upd_clock[0] = wall_clock64();
  const int64_t fifo_start = a.st ? a.st->tail : a.fifo_start;
  const double alpha = a.st ? sched_value(a.alpha_s, a.st->sched_step + a.pre_step) : a.alpha;
  const int64_t N = a.pn + a.n;
  const int64_t top = (int64_t(1) << S) - 1;  // nodes above level S
  const uint32_t G = gridDim.x;
  int64_t scan = 0;
  int R = kSubKeys;
  while (scan < N) {
    // ---- gather the round's keys (launch order) into slots 0..cnt-1
    int cnt = 0;
    int64_t pos = scan;
    while (pos < N && cnt < R) {
      const int64_t g = pos + tid;
      bool mine = false;
      if (g < N) {
        const int64_t id = upd_id(a, g, fifo_start);
        if (id >= top && id < cap) {
          const int d = node_depth(id);
          const int64_t sub = ((id + 1) >> (d - S)) - 1 - top;
          mine = (uint32_t)(sub % G) == blockIdx.x;
        }
      }
      int total;
      const int rank = wg_scan(mine ? 1 : 0, wsum, &total);
      const int take = R - cnt;
      if (tid == 0) s_next = -1;
      __syncthreads();
      if (mine && rank < take) slot_g[cnt + rank] = (int32_t)g;
      if (mine && rank == take) s_next = (int)(g - pos);  // first key left for the next round
      __syncthreads();
      if (total > take) {
        cnt = R;
        pos += s_next;
      } else {
        cnt += total;
        pos += kSubThreads;
      }
    }
    if (pos > N) pos = N;
    if (cnt == 0) {
      scan = pos;
      continue;
    }
    // ---- sort keys (aligned, depth, slot)
    int P = 1;
    while (P < cnt) P <<= 1;
    for (int j = tid; j < P; j += kSubThreads) {
      uint64_t k = ~0ull;
      if (j < cnt) {
        const int64_t id = upd_id(a, slot_g[j], fifo_start);
        const int d = node_depth(id);
        const uint64_t al = (uint64_t)(id + 1) << (maxd - d);
        k = (((al << 6) | (uint64_t)d) << kSlotBits) | (uint64_t)j;
      }
      keys[j] = k;
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        for (int i = tid; i < P / 2; i += kSubThreads) {
          const int lo = 2 * jj * (i / jj) + (i % jj), hi = lo + jj;
          const uint64_t x = keys[lo], y = keys[hi];
          const bool up = (lo & k) == 0;
          if ((x > y) == up) {
            keys[lo] = y;
            keys[hi] = x;
          }
        }
        __syncthreads();
      }
    }
    // ---- owned level ranges and entry bases (4 consecutive keys per lane)
    int own[4];
    int csum = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = 4 * tid + u;
      own[u] = 0;
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
        own[u] = max(0, dj - S + 1 - sh);
        csum += own[u];
      }
    }
    int E;
    int off = wg_scan(csum, wsum, &E);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = 4 * tid + u;
      if (j < cnt) ebase[j] = off;
      off += own[u];
    }
    if (E > kSubEntries) {  // uniform: re-gather this round with fewer keys
      R = max(1, cnt / 2);
      __syncthreads();
      continue;
    }
    __syncthreads();
    // ---- parent entry of each key's shallowest owned entry (lower_bound of its owner)
    for (int j = tid; j < cnt; j += kSubThreads) {
      const uint64_t kj = keys[j];
      const int lt = elt[j];
      int p = -1;
      if (ebase[j] != (j + 1 < cnt ? ebase[j + 1] : E) && lt > S) {
        const int L = lt - 1;
        const uint64_t al = (key_aligned(kj) >> (maxd - L)) << (maxd - L);
        const uint64_t want = ((al << 6) | (uint64_t)L) << kSlotBits;
        int lo = 0, hi = j;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (keys[mid] < want) lo = mid + 1; else hi = mid;
        }
        p = ebase[lo] + (L - elt[lo]);
      }
      epar[j] = p;
    }
    // ---- load every entry's inputs (one parallel pass; LDS stores cannot alias the loads)
    for (int j = tid; j < cnt; j += kSubThreads) {
      const uint64_t kj = keys[j];
      const int dj = key_depth(kj), lt = elt[j];
      const uint64_t al = key_aligned(kj);
      const int e0 = ebase[j];
      for (int L0 = lt; L0 <= dj; L0 += 4) {
        double v[4], ls[4], lm[4], rs[4], rm[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int L = L0 + u;
          v[u] = ls[u] = lm[u] = rs[u] = rm[u] = 0.0;
          if (L <= dj) {
            const int64_t node = (int64_t)(al >> (maxd - L)) - 1, l = 2 * node + 1;
            if (L < dj) v[u] = a.nd[node + 1].val;
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
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int L = L0 + u;
          if (L <= dj) ent[e0 + L - lt] = SubEnt{v[u], ls[u], lm[u], rs[u], rm[u]};
        }
      }
      if (e0 + (dj - lt) >= e0 && dj >= lt) {  // j owns its own node: the last duplicate's priority
        int last = j;
        while (last + 1 < cnt && (keys[last + 1] >> kSlotBits) == (kj >> kSlotBits)) ++last;
        ent[e0 + dj - lt].v = priority_of(a, alpha, slot_g[keys[last] & ((1u << kSlotBits) - 1)]);
      }
    }
    __syncthreads();
    if (tid == 0 && blockIdx.x == 0) g_upd_clock[1] = wall_clock64();
    // ---- levels, deepest first (_numba_maintain_node on every touched node, once)
    for (int L = maxd; L >= S; --L) {
      for (int j = tid; j < cnt; j += kSubThreads) {
        const int lt = elt[j];
        const uint64_t kj = keys[j];
        if (L < lt || L > key_depth(kj)) continue;
        const int e = ebase[j] + L - lt;
        const SubEnt x = ent[e];
        const int64_t node = (int64_t)(key_aligned(kj) >> (maxd - L)) - 1, l = 2 * node + 1;
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
          const int p = L > lt ? e - 1 : epar[j];
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
    // ---- store the touched nodes
    for (int j = tid; j < cnt; j += kSubThreads) {
      const uint64_t kj = keys[j];
      const int dj = key_depth(kj), lt = elt[j];
      const uint64_t al = key_aligned(kj);
      for (int L = lt; L <= dj; ++L) {
        const SubEnt x = ent[ebase[j] + L - lt];
        const int64_t node = (int64_t)(al >> (maxd - L)) - 1;
        a.nd[node + 1].sum = x.ls;
        a.nd[node + 1].mn = x.lm;
        if (L == dj) a.nd[node + 1].val = x.v;
      }
    }
    __syncthreads();  // the next round reads these stores (same workgroup)
    scan = pos;
    R = kSubKeys;
  }
  if (tid == 0 && blockIdx.x == 0) g_upd_clock[1] = wall_clock64();
}

// ---------------------------------------------------------------- top pass
// The levels above S (at most 2^11 - 1 nodes) as a dense bottom-up pass in LDS, after the
// subtree pass: every node's (val, sum, min) and level S's (sum, min) are loaded in one
// coalesced sweep; a node is maintained iff it is a key or a child was (touched
// ancestors only -- the min() quirk); last writer wins among keys above S.
constexpr int kTopS = 11;
constexpr int kTopThreads = 1024;
constexpr int kTopNodes = (1 << kTopS) - 1;

__global__ __launch_bounds__(kTopThreads) void k_tree_update_top(UpdArgs a, int S) {
  __shared__ double tv[kTopNodes], tsum[kTopNodes], tmin[kTopNodes];
  __shared__ double bsum[kTopNodes + 1], bmin[kTopNodes + 1];
  __shared__ int32_t win[kTopNodes];
  __shared__ uint8_t ttop[kTopNodes], tbot[kTopNodes + 1];
  const int tid = threadIdx.x;
  const int64_t cap = a.cap;
  if (tid == 0) g_upd_clock[2] = wall_clock64();
  const int64_t fifo_start = a.st ? a.st->tail : a.fifo_start;
  const double alpha = a.st ? sched_value(a.alpha_s, a.st->sched_step + a.pre_step) : a.alpha;
  const int64_t N = a.pn + a.n;
  const int ntop = (1 << S) - 1;
  for (int i = tid; i < ntop; i += kTopThreads) {
    double v = 0.0, s = 0.0, m = 0.0;
    if (i < cap) {
      const Node x = a.nd[i + 1];
      v = x.val;
      s = x.sum;
      m = x.mn;
    }
    tv[i] = v;
    tsum[i] = s;
    tmin[i] = m;
    win[i] = -1;
    ttop[i] = 0;
  }
  for (int k = tid; k <= ntop; k += kTopThreads) {
    const int64_t node = ntop + k;
    double s = 0.0, m = 0.0;
    if (node < cap) {
      s = a.nd[node + 1].sum;
      m = a.nd[node + 1].mn;
    }
    bsum[k] = s;
    bmin[k] = m;
    tbot[k] = 0;
  }
  __syncthreads();
  for (int64_t g = tid; g < N; g += kTopThreads) {
    const int64_t id = upd_id(a, g, fifo_start);
    if (id < 0 || id >= cap) continue;
    if (id < ntop) {
      atomicMax(&win[id], (int32_t)g);
    } else {
      const int d = node_depth(id);
      tbot[((id + 1) >> (d - S)) - 1 - ntop] = 1;
    }
  }
  __syncthreads();
  if (tid == 0) g_upd_clock[3] = wall_clock64();
  for (int i = tid; i < ntop; i += kTopThreads) {
    const int w = win[i];
    if (w >= 0) {
      const double v = priority_of(a, alpha, w);
      tv[i] = v;
      ttop[i] = 1;
      a.nd[i + 1].val = v;
    }
  }
  __syncthreads();
  for (int L = S - 1; L >= 0; --L) {
    const int first = (1 << L) - 1;
    for (int i = first + tid; i < 2 * first + 1 && i < cap; i += kTopThreads) {
      const int64_t l = 2 * (int64_t)i + 1, r = l + 1;
      const bool bottom = (L == S - 1);
      bool t = ttop[i] != 0;
      double ls = 0.0, lm = 0.0, rs = 0.0, rm = 0.0;
      if (l < cap) {
        if (bottom) {
          t |= tbot[l - ntop] != 0;
          ls = bsum[l - ntop];
          lm = bmin[l - ntop];
        } else {
          t |= ttop[l] != 0;
          ls = tsum[l];
          lm = tmin[l];
        }
      }
      if (r < cap) {
        if (bottom) {
          t |= tbot[r - ntop] != 0;
          rs = bsum[r - ntop];
          rm = bmin[r - ntop];
        } else {
          t |= ttop[r] != 0;
          rs = tsum[r];
          rm = tmin[r];
        }
      }
      if (!t) continue;
      const double v = tv[i];
      double sm = v, mn = (v != 0.0) ? v : 1.0;
      if (l < cap) {
        sm = radd(sm, ls);
        if (lm != 0.0) mn = (lm < mn) ? lm : mn;
      }
      if (r < cap) {
        sm = radd(sm, rs);
        if (rm != 0.0) mn = (rm < mn) ? rm : mn;
      }
      tsum[i] = sm;
      tmin[i] = mn;
      ttop[i] = 1;
    }
    lds_barrier();  // LDS only: no wait for global stores inside the level loop
  }
  for (int i = tid; i < ntop && i < cap; i += kTopThreads) {
    if (ttop[i]) {
      a.nd[i + 1].sum = tsum[i];
      a.nd[i + 1].mn = tmin[i];
    }
  }
  if (tid == 0) {
    if (a.st) {
      if (a.pre_step) a.st->sched_step += 1;
      if (a.post_tail) a.st->tail = (fifo_start + a.n) % cap;  // every read of tail is done
    }
    g_upd_clock[4] = wall_clock64();
  }
}

// ------------------------------------------------------------------ find / sample
__global__ void k_tree_find(const Node *__restrict__ nd, int64_t cap, const double *__restrict__ tg,
                            int64_t n, int64_t *__restrict__ idx_out, double *__restrict__ val_out, int kspec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t k = tree_find(nd, cap, tg[i], kspec);
  if (idx_out) idx_out[i] = k;
  if (val_out) val_out[i] = nd[k + 1].val;
}

// _numba_sample (sumtree.py:70-79) and, with is_weights, PERSampler.sample (:24-28)
__global__ void k_tree_sample(const Node *__restrict__ nd, int64_t cap, int64_t batch,
                              const double *__restrict__ uniforms, uint64_t seed, uint64_t counter,
                              int is_weights, double beta, const ReplayState *st, rth_schedule beta_s,
                              int64_t *__restrict__ idx_out, double *__restrict__ out, int kspec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  if (st) {  // a replay shard's device state: call counter and beta_s(sched_step)
    counter = (uint64_t)st->calls;
    beta = sched_value(beta_s, st->sched_step);
  }
  const double total = nd[1].sum;
  const double seg = total / (double)batch;
  const double u = uniforms ? uniforms[i] : philox_uniform(seed, counter, (uint32_t)i, STREAM_SAMPLE);
  const double t = rmul(radd((double)i, u), seg);
  const int64_t k = tree_find(nd, cap, t, kspec);
  const double p = nd[k + 1].val;
  idx_out[i] = k;
  if (is_weights) {
    out[i] = pow(p / tree_min(nd), -beta);
  } else if (out) {
    out[i] = p;
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
};

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
  RTH_REQUIRE(a.pn + a.n < (int64_t(1) << 31), "tree update: at most 2^31 - 1 keys per call");
  const int S = t->maxd + 1 < kTopS ? t->maxd + 1 : kTopS;
  if (t->maxd >= S && a.pn + a.n > 0) {  // levels S..maxd: one workgroup per group of subtrees
    const int64_t nsub = int64_t(1) << S;
    hipLaunchKernelGGL(k_tree_update_sub, dim3((unsigned)(nsub < kSubGrid ? nsub : kSubGrid)), dim3(kSubThreads), 0,
                       s, a, S);
    RTH_LAUNCHED();
  }
  hipLaunchKernelGGL(k_tree_update_top, dim3(1), dim3(kTopThreads), 0, s, a, S);
  RTH_LAUNCHED();
  return RTH_OK;
}
int tree_sample_impl(rth_sumtree *t, int64_t batch, const double *uniforms, uint64_t seed,
                     uint64_t counter, int is_weights, double beta, int64_t *idx_out, double *out,
                     hipStream_t s, const ReplayState *st, const rth_schedule *beta_s) {
  if (batch <= 0) return RTH_OK;
  const int bs = sample_bs();
  hipLaunchKernelGGL(k_tree_sample, dim3((unsigned)((batch + bs - 1) / bs)), dim3(bs), 0, s, t->nodes,
                     t->cap, batch, uniforms, seed, counter, is_weights, beta, st,
                     beta_s ? *beta_s : rth_schedule{}, idx_out, out, find_k());
  RTH_LAUNCHED();
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
  const size_t bytes = (size_t)(capacity + 2) * sizeof(Node);
  if (hipMalloc(&nodes, bytes) != hipSuccess) {
    set_error("rth_sumtree_create: hipMalloc(%zu) failed", bytes);
    return RTH_ERR_NOMEM;
  }
  RTH_HIP(hipMemset(nodes, 0, bytes));
  auto *t = new rth_sumtree{capacity, device, node_depth(capacity - 1), nodes};
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

int rth_debug_tree_timing(long long *out5) {
  RTH_REQUIRE(out5, "rth_debug_tree_timing: NULL");
  RTH_HIP(hipMemcpyFromSymbol(out5, HIP_SYMBOL(g_upd_clock), 5 * sizeof(long long)));
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
  const int bs = sample_bs();
  hipLaunchKernelGGL(k_tree_find, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, as_stream(stream),
                     t->nodes, t->cap, tg, n, idx_out, val_out, find_k());
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
