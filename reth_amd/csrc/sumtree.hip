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
//   zero node).  One workgroup sorts each chunk of <= 4096 (index, position) keys in LDS by
//   the index's left-aligned leaf position, which makes "ancestor at level L" monotone, so
//   each distinct ancestor is maintained exactly once per level by the first key of its run.
//   Chunks run in order, which keeps the sequential semantics for any n.
#include <cmath>
#include <cstdlib>

#include "common.hpp"

namespace rth {

struct alignas(32) Node {
  double sum, val, mn, pad;
};

constexpr int kUpdThreads = 1024;
constexpr int kUpdChunk = 4096;  // keys per LDS chunk (32 KiB)
constexpr int kPosBits = 12;     // log2(kUpdChunk)
constexpr int kDepthBits = 6;
constexpr int64_t kMaxCapacity = int64_t(1) << 40;  // aligned(41) + depth(6) + pos(12) <= 64

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

__device__ __forceinline__ int64_t key_index(uint64_t key, int maxd) {
  const int d = (int)((key >> kPosBits) & ((1u << kDepthBits) - 1));
  const uint64_t aligned = key >> (kPosBits + kDepthBits);
  return (int64_t)(aligned >> (maxd - d)) - 1;
}

// phase timestamps of the last k_tree_update (wall clock ticks; development aid, read by
// rth_debug_tree_timing)
__device__ long long g_upd_clock[8];

// a workgroup barrier that orders LDS only (global stores are not waited for)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ __launch_bounds__(kUpdThreads) void k_tree_update(UpdArgs a) {
  __shared__ uint64_t keys[kUpdChunk];
  __shared__ double res_sum[kUpdChunk], res_min[kUpdChunk];  // an owner's (sum, min) per level
  const int tid = threadIdx.x;
  const int maxd = a.maxd;
  if (tid == 0) g_upd_clock[0] = wall_clock64();
  if (a.pre_step && tid == 0) a.st->sched_step += 1;
  __syncthreads();
  const int64_t fifo_start = a.st ? a.st->tail : a.fifo_start;
  const double alpha = a.st ? sched_value(a.alpha_s, a.st->sched_step) : a.alpha;
  const int64_t N = a.pn + a.n;
  for (int64_t cs = 0; cs < N; cs += kUpdChunk) {
    const int m = (int)min<int64_t>(kUpdChunk, N - cs);
    int P = 2;
    while (P < m) P <<= 1;
    if (P <= kUpdThreads) {
      // One key per lane.  Issue the loads that warm the lines the level loop will touch
      // (the children-pair line of the deepest kPre nodes on the key's path; the top of the
      // tree is hot anyway) and keep them in flight through the sort, which synchronises on
      // LDS only; consume them afterwards.
      constexpr int kPre = 16;
      double pre[kPre];
      const int64_t id = tid < m ? upd_id(a, cs + tid, fifo_start) : -1;
      {
        int64_t x = (id >= 0 && id < a.cap) ? id : -1;
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
          pre[u] = 0.0;
          if (x >= 0) {
            const int64_t c = 2 * x + 1;
            pre[u] = a.nd[(c < a.cap ? c : x) + 1].sum;
            x = x ? (x - 1) / 2 : -1;
          }
        }
      }
      if (tid == 0) g_upd_clock[1] = wall_clock64();
      uint64_t key = ~0ull;
      if (id >= 0 && id < a.cap) {
        const int d = node_depth(id);
        const uint64_t aligned = (uint64_t)(id + 1) << (maxd - d);
        key = (((aligned << kDepthBits) | (uint64_t)d) << kPosBits) | (uint64_t)tid;
      }
      // bitonic sort of the workgroup's 1024 lanes (sentinels sort last): partners within a
      // wave exchange through cross-lane shuffles, wider strides through LDS
      for (int k = 2; k <= kUpdThreads; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          uint64_t y;
          if (jj < 64) {
            y = __shfl_xor(key, jj, 64);
          } else {
            keys[tid] = key;
            lds_barrier();
            y = keys[tid ^ jj];
            lds_barrier();
          }
          const bool up = (tid & k) == 0, lower = (tid & jj) == 0;
          key = (lower == up) ? (key < y ? key : y) : (key < y ? y : key);
        }
      }
      keys[tid] = key;
      uint64_t acc = 0;
#pragma unroll
      for (int u = 0; u < kPre; ++u) acc ^= (uint64_t)__double_as_longlong(pre[u]);
      if (acc == 0x9E3779B97F4A7C15ull) a.nd[0].pad = 1.0;  // record 0 is padding; keeps the loads
      lds_barrier();
    } else {
      // several keys per lane: warm the lines first, then an LDS bitonic sort
      uint64_t acc = 0;
      for (int j = tid; j < m; j += kUpdThreads) {
        int64_t x = upd_id(a, cs + j, fifo_start);
        if (x < 0 || x >= a.cap) continue;
        while (x >= 0) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            v[u] = 0.0;
            if (x >= 0) {
              const int64_t c = 2 * x + 1;
              v[u] = a.nd[(c < a.cap ? c : x) + 1].sum;
              x = x ? (x - 1) / 2 : -1;
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) acc ^= (uint64_t)__double_as_longlong(v[u]);
        }
      }
      if (acc == 0x9E3779B97F4A7C15ull) a.nd[0].pad = 1.0;
      if (tid == 0) g_upd_clock[1] = wall_clock64();
      for (int j = tid; j < P; j += kUpdThreads) {
        uint64_t key = ~0ull;
        if (j < m) {
          const int64_t id = upd_id(a, cs + j, fifo_start);
          if (id >= 0 && id < a.cap) {
            const int d = node_depth(id);
            const uint64_t aligned = (uint64_t)(id + 1) << (maxd - d);
            key = (((aligned << kDepthBits) | (uint64_t)d) << kPosBits) | (uint64_t)j;
          }
        }
        keys[j] = key;
      }
      __syncthreads();
      for (int k = 2; k <= P; k <<= 1) {  // bitonic sort, ascending
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          for (int i = tid; i < P; i += kUpdThreads) {
            const int ixj = i ^ jj;
            if (ixj > i) {
              const uint64_t x = keys[i], y = keys[ixj];
              const bool up = (i & k) == 0;
              if ((x > y) == up) {
                keys[i] = y;
                keys[ixj] = x;
              }
            }
          }
          lds_barrier();
        }
      }
    }
    if (tid == 0) g_upd_clock[2] = wall_clock64();
    // last writer of every index sets val (duplicates sort by position)
    for (int j = tid; j < m; j += kUpdThreads) {
      const uint64_t key = keys[j];
      if (key == ~0ull) continue;
      const int64_t id = key_index(key, maxd);
      const bool last = (j == m - 1) || keys[j + 1] == ~0ull || key_index(keys[j + 1], maxd) != id;
      if (last) {
        const int64_t src = cs + (int64_t)(key & ((1u << kPosBits) - 1));
        a.nd[id + 1].val = priority_of(a, alpha, src);
      }
    }
    __syncthreads();
    if (tid == 0) g_upd_clock[3] = wall_clock64();
    // Touched ancestors, deepest level first; the first key of each ancestor's run maintains
    // it (_numba_maintain_node).  A touched child's (sum, min) comes from LDS -- its owner
    // at the level below stored it in res[owner] -- found by binary search in the sorted
    // keys (the child's subtree is a key range); only untouched children and the node's own
    // val are read from memory (issued before the search), so a level costs one overlapped
    // L2 round trip and an LDS-only barrier instead of store -> barrier -> load.
    for (int L = maxd; L >= 0; --L) {
      for (int j = tid; j < m; j += kUpdThreads) {
        const uint64_t key = keys[j];
        if (key == ~0ull) continue;
        const int d = (int)((key >> kPosBits) & ((1u << kDepthBits) - 1));
        if (d < L) continue;
        const uint64_t aligned = key >> (kPosBits + kDepthBits);
        const uint64_t anc = aligned >> (maxd - L);  // 1-based heap index
        if (j > 0) {
          const uint64_t pk = keys[j - 1];
          const int pd = (int)((pk >> kPosBits) & ((1u << kDepthBits) - 1));
          if (pd >= L && ((pk >> (kPosBits + kDepthBits)) >> (maxd - L)) == anc) continue;
        }
        const int64_t node = (int64_t)anc - 1, l = 2 * node + 1, r = l + 1;
        const double v = a.nd[node + 1].val;
        double ls = 0.0, lm = 0.0, rs = 0.0, rm = 0.0;
        if (l < a.cap) {
          ls = a.nd[l + 1].sum;
          lm = a.nd[l + 1].mn;
        }
        if (r < a.cap) {
          rs = a.nd[r + 1].sum;
          rm = a.nd[r + 1].mn;
        }
        if (L < maxd) {
          // the node's subtree is the key range of aligned values [al, al + 2 half): its own
          // keys first (depth L), then the left child's range, then the right child's; a
          // child's owner at level L + 1 is the first key of its range
          const uint64_t al = anc << (maxd - L), half = uint64_t(1) << (maxd - L - 1);
          constexpr int kSh = kPosBits + kDepthBits;
          int k1 = j;  // skip the node's own keys (duplicates of it)
          while (k1 < m && (keys[k1] >> kSh) == al && (int)((keys[k1] >> kPosBits) & ((1u << kDepthBits) - 1)) == L)
            ++k1;
          if (k1 < m && keys[k1] != ~0ull && (keys[k1] >> kSh) < al + half) {
            ls = res_sum[k1];
            lm = res_min[k1];
          }
          // right child: first key at or after k1 with aligned >= al + half (galloping)
          const uint64_t rc_al = al + half;
          int lo = k1, hi = k1, b = 1;
          while (hi < m && (keys[hi] >> kSh) < rc_al) {
            lo = hi + 1;
            hi = k1 + b;
            b <<= 1;
          }
          if (hi > m) hi = m;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((keys[mid] >> kSh) < rc_al) lo = mid + 1; else hi = mid;
          }
          if (lo < m && keys[lo] != ~0ull && (keys[lo] >> kSh) < al + 2 * half) {
            rs = res_sum[lo];
            rm = res_min[lo];
          }
        }
        double sm = v;  // sum[i] = val[i] + sum[l] + sum[r]; min seeded 1 for a zero val
        double mn = (v != 0.0) ? v : 1.0;
        if (l < a.cap) {
          sm = radd(sm, ls);
          if (lm != 0.0) mn = (lm < mn) ? lm : mn;
        }
        if (r < a.cap) {
          sm = radd(sm, rs);
          if (rm != 0.0) mn = (rm < mn) ? rm : mn;
        }
        a.nd[node + 1].sum = sm;
        a.nd[node + 1].mn = mn;
        res_sum[j] = sm;
        res_min[j] = mn;
      }
      lds_barrier();
    }
    __syncthreads();  // the next chunk reads this chunk's stores from memory
    if (tid == 0) g_upd_clock[4] = wall_clock64();
  }
  if (a.post_tail && tid == 0) a.st->tail = (fifo_start + a.n) % a.cap;  // all reads of tail are done
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
  hipLaunchKernelGGL(k_tree_update, dim3(1), dim3(kUpdThreads), 0, s, a);
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
