// HBM-resident replay shard: FIFO slots + column storage + PER tree, and the row copy /
// gather kernel that replaces the reference's LMDB put/get + pinned copy + H2D.
//
// Reference: reth_buffer/reth_buffer/server/main_loop.py:21-61 (append_loop),
// server/sampler_loop.py:6-42, cache_policy/fifo_policy.py:11-18, client/client.py:21-39,
// client/torch_cuda_loader.py:20-66, client/numpy_loader.py:27-51.
//
// Storage is one dense [capacity, row] array per column (struct of arrays), so a sampled
// row of a frame column is one contiguous 28,224-byte run of uint8: the gather streams it
// with 16-byte loads and widens to float32 on the way out (uint8 -> f32 is exact, so the
// learner receives exactly the f32 frames the reference's actors stored, 4x fewer bytes
// resident and read).
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"

struct rth_sumtree;

namespace rth {
int tree_update_impl(rth_sumtree *t, const int64_t *idx, int64_t fifo_start, const double *w64,
                     const void *td_abs, int32_t td_dtype, double alpha, int64_t n, hipStream_t s,
                     ReplayState *st, const rth_schedule *alpha_s, const UpdPending *pend = nullptr,
                     int post_tail = 0);
int tree_sample_impl(rth_sumtree *t, int64_t batch, const double *uniforms, uint64_t seed,
                     uint64_t counter, int is_weights, double beta, int64_t *idx_out, double *out,
                     hipStream_t s, const ReplayState *st, const rth_schedule *beta_s);

enum Conv : int32_t { CONV_COPY = 0, CONV_U8_F32 = 1, CONV_U8_F32_HWC = 2, CONV_F32_U8 = 3, CONV_STACK = 4 };

// f32 pixel -> u8 (append of frames an actor sends as float32 whole numbers 0..255)
__device__ __forceinline__ uint32_t f32_u8(float v) {
  v = rintf(v);
  return (uint32_t)(v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v));
}

// a float at any byte address (arrays inside a wire-format message body are unaligned)
__device__ __forceinline__ float ld_f32_bytes(const uint8_t *p) {
  const uint32_t u = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
  return __uint_as_float(u);
}

struct CopyCol {
  const uint8_t *src;
  uint8_t *dst;
  const int64_t *src_rows;  // nullable: identity
  const int64_t *dst_rows;  // nullable: identity, or FIFO when CopyArgs::dst_fifo
  int64_t src_stride;       // bytes
  int64_t dst_stride;       // bytes
  int64_t in_bytes;         // bytes of one input row
  int32_t conv;
  int32_t planes;           // CONV_U8_F32_HWC: channel planes per row (CHW in, HWC out)
  // grid layout, filled by launch_copy
  int64_t chunk_in;         // input bytes per chunk
  int64_t chunks;           // chunks per row (0: small column, one lane per row)
  int64_t chunk_px;         // CONV_U8_F32_HWC: pixels per chunk
  int64_t blk0;             // first workgroup of this column
  int32_t vec;              // every row's src/dst 16-byte aligned: vector path
  int32_t pad;
  // CONV_STACK (a frame-stack column of a frame-store replay): the stored row is `planes`
  // int32 frame ids, the output row the `planes` frames of frame_bytes each, read from the
  // frame store (fcap frames); in_bytes is the OUTPUT row size there
  const uint8_t *fstore;
  int64_t frame_bytes;
  int64_t fcap;
};

struct CopyArgs {
  CopyCol col[RTH_MAX_COLS];
  int64_t n;
  int64_t fifo_start;
  int64_t fifo_cap;
  const ReplayState *st;  // nullable: FIFO start = st->tail (device-resident)
  int32_t dst_fifo;
  int32_t ncols;
  ReplayState *bump_st;   // nullable: st->calls += bump_calls here (the sample(s) this gather follows)
  int64_t bump_calls;
};

constexpr int kCopyThreads = 256;
constexpr int kCopyVec = 1;  // COPY: 16-byte vectors per lane (4 KiB chunks: more, smaller workgroups measured faster than 16 KiB)
constexpr int64_t kSmallRow = 64;  // rows up to this many bytes: one lane per row

__device__ __forceinline__ float4 u8x4_to_f4(uint32_t w) {
  return make_float4((float)(w & 0xffu), (float)((w >> 8) & 0xffu), (float)((w >> 16) & 0xffu), (float)(w >> 24));
}

// byte j of each of four words -> one float4 (one pixel's four channel planes)
__device__ __forceinline__ float4 plane_px(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int j) {
  const int s = 8 * j;
  return make_float4((float)((w0 >> s) & 0xffu), (float)((w1 >> s) & 0xffu), (float)((w2 >> s) & 0xffu),
                     (float)((w3 >> s) & 0xffu));
}

// CHW u8 (4 planes of P pixels, P % 4 == 0) -> HWC f32 for pixels [pc, pc + 1024*M): the
// chunk's 4 planes are staged in LDS with coalesced 4-byte loads (M per plane per lane in
// flight), then each lane writes whole pixels, one float4 each: every wave store
// instruction covers 1 KiB of contiguous output.
template <int M>
__device__ __forceinline__ void hwc4_chunk(const uint8_t *__restrict__ src, float *__restrict__ df, int64_t P,
                                           int64_t pc, int tid) {
  constexpr int W = M * kCopyThreads;  // words per plane in the chunk
  extern __shared__ uint32_t stage[];  // 4 * W words, sized at launch
  const int64_t wlim = (P - pc) / 4;   // words of this chunk inside the row
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src + k * P + pc);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int w = j * kCopyThreads + tid;
      if (w < wlim) stage[k * W + w] = s32[w];
    }
  }
  __syncthreads();
  const uint8_t *sb = reinterpret_cast<const uint8_t *>(stage);
  float4 *d4 = reinterpret_cast<float4 *>(df) + pc;
  const int64_t plim = P - pc;
#pragma unroll
  for (int j = 0; j < 4 * M; ++j) {
    const int p = j * kCopyThreads + tid;
    if (p < plim)
      d4[p] = make_float4((float)sb[p], (float)sb[4 * W + p], (float)sb[8 * W + p], (float)sb[12 * W + p]);
  }
}

// Flat 1-D grid.  Column c owns workgroups [blk0, blk0 + nblk); a large column splits each
// row into `chunks` independent chunks of `chunk_in` input bytes (one per workgroup: no LDS,
// no barrier, thousands of workgroups in flight so loads and stores of different chunks
// overlap), a small column (a, r, done: <= 64 B) gives each lane one 4-byte word of a row
// (plain copies) or a whole row (conversions).
//   COPY        16-byte loads and stores (kCopyVec per lane), the row tail vectorised too;
//               chunk = 4 KiB.
//   U8_F32      4-byte loads of 4 pixels become 16-byte stores (1 KiB contiguous per wave
//               instruction), four per lane in flight; chunk = 4 KiB in.
//   U8_F32_HWC  C planes of P pixels (CHW u8) -> P pixels x C floats (HWC f32, channels_last
//               for the Q-net).  C == 4: the chunk's 4 planes x 1024 pixels are staged in
//               4 KiB of LDS, then each lane writes whole pixels (one float4 each, 1 KiB
//               contiguous per wave instruction); chunk = 1024 pixels.
__global__ __launch_bounds__(kCopyThreads) void k_copy_rows(CopyArgs a) {
  const int64_t b = blockIdx.x;
  // the sampler's call counter, read by the sample launch before this one (stream order),
  // advanced here instead of by a launch of its own
  if (a.bump_st && b == 0 && threadIdx.x == 0) a.bump_st->calls += a.bump_calls;
  int c = 0;
  while (c + 1 < a.ncols && b >= a.col[c + 1].blk0) ++c;
  const CopyCol &col = a.col[c];
  const int tid = threadIdx.x;
  int64_t i, chunk = 0;
  int32_t word = -1;
  if (col.chunks == 0 && col.vec) {  // small COPY rows of whole words: one lane per 4-byte word
    const int64_t e = (b - col.blk0) * kCopyThreads + tid, words = col.in_bytes / 4;
    if (e >= a.n * words) return;
    i = e / words;
    word = (int32_t)(e - i * words);
  } else if (col.chunks == 0) {  // small rows
    i = (b - col.blk0) * kCopyThreads + tid;
    if (i >= a.n) return;
  } else {
    const int64_t r = b - col.blk0;
    i = r / col.chunks;
    chunk = r - i * col.chunks;
  }
  const int64_t sr = col.src_rows ? col.src_rows[i] : i;
  int64_t dr;
  if (col.dst_rows)
    dr = col.dst_rows[i];
  else if (a.dst_fifo)
    dr = ((a.st ? a.st->tail : a.fifo_start) + i) % a.fifo_cap;
  else
    dr = i;
  const uint8_t *__restrict__ src = col.src + sr * col.src_stride;
  uint8_t *__restrict__ dst = col.dst + dr * col.dst_stride;
  const int64_t nb = col.in_bytes;
  float *df = reinterpret_cast<float *>(dst);
  if (col.chunks == 0) {
    if (word >= 0) {
      reinterpret_cast<uint32_t *>(dst)[word] = reinterpret_cast<const uint32_t *>(src)[word];
    } else if (col.conv == CONV_COPY) {
      for (int64_t k = 0; k < nb; ++k) dst[k] = src[k];
    } else if (col.conv == CONV_F32_U8) {
      for (int64_t k = 0; k < nb / 4; ++k) dst[k] = (uint8_t)f32_u8(ld_f32_bytes(src + 4 * k));
    } else if (col.conv == CONV_U8_F32) {
      for (int64_t k = 0; k < nb; ++k) df[k] = (float)src[k];
    } else {
      const int C = col.planes;
      const int64_t P = nb / C;
      for (int64_t p = 0; p < P; ++p)
        for (int k = 0; k < C; ++k) df[p * C + k] = (float)src[k * P + p];
    }
    return;
  }
  const bool vec = col.vec != 0;  // alignment checked on the host for every row
  if (col.conv == CONV_U8_F32_HWC) {
    const int C = col.planes;
    const int64_t P = nb / C;
    const int64_t pc = chunk * col.chunk_px;  // first pixel of this chunk
    if (vec && C == 4) {
      switch (col.chunk_px / (4 * kCopyThreads)) {
        case 1: hwc4_chunk<1>(src, df, P, pc, tid); break;
        case 2: hwc4_chunk<2>(src, df, P, pc, tid); break;
        case 4: hwc4_chunk<4>(src, df, P, pc, tid); break;
        default: hwc4_chunk<8>(src, df, P, pc, tid); break;
      }
    } else {
      for (int64_t p = pc + tid; p < pc + col.chunk_px && p < P; p += kCopyThreads)
        for (int k = 0; k < C; ++k) df[p * C + k] = (float)src[k * P + p];
    }
    return;
  }
  const int64_t o = chunk * col.chunk_in;  // first input byte of this chunk
  if (col.conv == CONV_STACK) {  // 16-byte vectors of the stack, each from its frame in the store
    const int32_t *ids = reinterpret_cast<const int32_t *>(src);
    const int64_t off = o + 16 * tid;
    if (off + 16 <= nb) {  // 32-bit index math (a stack row is < 2^31 bytes)
      const uint32_t o32 = (uint32_t)off, fb = (uint32_t)col.frame_bytes;
      const uint32_t f = o32 / fb, in = o32 - f * fb;
      // ids are in [0, fcap) by construction (k_frames_push writes them reduced); an id out of
      // range reads frame 0 rather than past the store
      const uint32_t id = (uint32_t)ids[f];
      const int64_t fid = id < (uint64_t)col.fcap ? (int64_t)id : 0;
      *reinterpret_cast<uint4 *>(dst + off) = *reinterpret_cast<const uint4 *>(col.fstore + fid * col.frame_bytes + in);
    }
    return;
  }
  if (col.conv == CONV_F32_U8) {  // 16-byte loads of 4 pixels -> one 4-byte store
    const float *sf = reinterpret_cast<const float *>(src);
    const int64_t e = o / 4 + 4 * tid;  // first element of this lane
    if (vec && o + col.chunk_in <= nb) {
      const float4 v = *reinterpret_cast<const float4 *>(sf + e);
      *reinterpret_cast<uint32_t *>(dst + e) = f32_u8(v.x) | (f32_u8(v.y) << 8) | (f32_u8(v.z) << 16) | (f32_u8(v.w) << 24);
    } else {
      for (int64_t k = e; k < e + 4 && k < nb / 4; ++k) dst[k] = (uint8_t)f32_u8(ld_f32_bytes(src + 4 * k));
    }
    return;
  }
  if (vec && col.conv == CONV_COPY) {  // lane-contiguous 16-byte loads and stores, kCopyVec in flight
    uint4 v[kCopyVec];
#pragma unroll
    for (int j = 0; j < kCopyVec; ++j) {
      const int64_t off = o + 16 * (j * kCopyThreads + tid);
      if (off + 16 <= nb) v[j] = *reinterpret_cast<const uint4 *>(src + off);
    }
#pragma unroll
    for (int j = 0; j < kCopyVec; ++j) {
      const int64_t off = o + 16 * (j * kCopyThreads + tid);
      if (off + 16 <= nb) *reinterpret_cast<uint4 *>(dst + off) = v[j];
    }
    const int64_t t0 = nb & ~int64_t(15);  // bytes past the row's last whole vector
    if (t0 < nb && t0 >= o && t0 < o + col.chunk_in)
      for (int64_t k = t0 + tid; k < nb; k += kCopyThreads) dst[k] = src[k];
    return;
  }
  if (vec && o + col.chunk_in <= nb) {
    {  // 4-byte loads -> 16-byte stores, 1 KiB contiguous per wave store, 4 in flight
      const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src + o);
      float4 *d4 = reinterpret_cast<float4 *>(df + o);
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = s32[j * kCopyThreads + tid];
#pragma unroll
      for (int j = 0; j < 4; ++j) d4[j * kCopyThreads + tid] = u8x4_to_f4(w[j]);
    }
  } else {
    for (int64_t k = o + tid; k < o + col.chunk_in && k < nb; k += kCopyThreads) {
      if (col.conv == CONV_COPY)
        dst[k] = src[k];
      else
        df[k] = (float)src[k];
    }
  }
}

__global__ void k_fifo_slots(int64_t *out, int64_t n, const ReplayState *st, int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (st->tail + i) % cap;
}

// advance the shard's device state after the launches that read it
__global__ void k_state_bump(ReplayState *st, int64_t dtail, int64_t cap, int64_t dcalls, int64_t dstep) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st->tail = (st->tail + dtail) % cap;
    st->calls += dcalls;
    st->sched_step += dstep;
  }
}

__global__ void k_counter_add(int64_t *c, int64_t d) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *c += d;
}

// ---------------------------------------------------------------- uniform / FIFO samplers
// Device state of the non-PER samplers (one 32-byte record next to the ReplayState).
struct SamplerState {
  int64_t ulen;    // UniformSampler.tail: entries in the index list
  int64_t fhead;   // FIFOSampler deque: ring position of the oldest entry
  int64_t fcount;  // entries queued
  int64_t pad;
};

constexpr int kSampThreads = 256;

// the i-th index of an update: given, or the i-th FIFO slot of an append (before the bump)
__device__ __forceinline__ int64_t upd_index(const int64_t *idx, const ReplayState *st, int64_t cap, int64_t i) {
  return idx ? idx[i] : (st->tail + i) % cap;
}

// UniformSampler.update (uniform_sampler.py:16-21): append while the list is below capacity
__global__ __launch_bounds__(kSampThreads) void k_uniform_push(int64_t *list, SamplerState *ss, int64_t cap,
                                                                const int64_t *idx, const ReplayState *st,
                                                                int64_t n) {
  const int64_t l0 = ss->ulen;
  for (int64_t i = threadIdx.x; i < n && l0 + i < cap; i += kSampThreads) list[l0 + i] = upd_index(idx, st, cap, i);
  __syncthreads();
  if (threadIdx.x == 0) ss->ulen = l0 + n < cap ? l0 + n : cap;
}

// UniformSampler.sample (:12-14): list[choice(len)], weights 1
__global__ void k_uniform_sample(const int64_t *list, const SamplerState *ss, const ReplayState *st, int64_t batch,
                                 const double *uniforms, uint64_t seed, int64_t *idx_out, double *w_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  const int64_t L = ss->ulen;
  const double u = uniforms ? uniforms[i] : philox_uniform(seed, (uint64_t)st->calls, (uint32_t)i, STREAM_SAMPLE);
  int64_t j = (int64_t)(u * (double)L);
  if (j >= L) j = L - 1;
  idx_out[i] = list[j];
  w_out[i] = 1.0;
}

// FIFOSampler.update (fifo_sampler.py:27-29): appendleft((idx, w)) on a deque(maxlen=cap)
__global__ __launch_bounds__(kSampThreads) void k_fifo_push(int64_t *ridx, double *rw, SamplerState *ss, int64_t cap,
                                                             const int64_t *idx, const ReplayState *st,
                                                             const void *w, int32_t wdt, int64_t n) {
  const int64_t head = ss->fhead, cnt = ss->fcount;
  const int64_t keep0 = n > cap ? n - cap : 0;  // only the newest cap entries survive
  for (int64_t i = keep0 + threadIdx.x; i < n; i += kSampThreads) {
    const int64_t pos = (head + cnt + i) % cap;
    ridx[pos] = upd_index(idx, st, cap, i);
    rw[pos] = wdt == RTH_F32 ? (double)static_cast<const float *>(w)[i] : static_cast<const double *>(w)[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t total = cnt + n, drop = total > cap ? total - cap : 0;
    ss->fhead = (head + drop) % cap;
    ss->fcount = total - drop;
  }
}

// FIFOSampler.sample (:19-25): pop() the batch oldest entries
__global__ __launch_bounds__(kSampThreads) void k_fifo_pop(const int64_t *ridx, const double *rw, SamplerState *ss,
                                                            int64_t cap, int64_t batch, int64_t *idx_out,
                                                            double *w_out) {
  const int64_t head = ss->fhead;
  for (int64_t i = threadIdx.x; i < batch; i += kSampThreads) {
    const int64_t pos = (head + i) % cap;
    idx_out[i] = ridx[pos];
    w_out[i] = rw[pos];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ss->fhead = (head + batch) % cap;
    ss->fcount -= batch;
  }
}

// NumpyBuffer.sample (buffer.py:88-90): choice(size, batch)
__global__ void k_uniform_indices(int64_t size, int64_t batch, const double *uniforms, uint64_t seed,
                                  uint64_t counter, const int64_t *counter_dev, int64_t *idx_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  const uint64_t ctr = counter_dev ? (uint64_t)*counter_dev : counter;
  const double u = uniforms ? uniforms[i] : philox_uniform(seed, ctr, (uint32_t)i, STREAM_SAMPLE);
  int64_t j = (int64_t)(u * (double)size);
  idx_out[i] = j < size ? j : size - 1;
}


// lay the columns out on the flat grid (see k_copy_rows)
int launch_copy(CopyArgs &a, hipStream_t s) {
  if (a.n <= 0 || a.ncols <= 0) return RTH_OK;
  int64_t blocks = 0;
  for (int c = 0; c < a.ncols; ++c) {
    CopyCol &col = a.col[c];
    col.blk0 = blocks;
    const int64_t nb = col.in_bytes;
    const uintptr_t al = reinterpret_cast<uintptr_t>(col.src) | reinterpret_cast<uintptr_t>(col.dst) |
                         (uintptr_t)col.src_stride | (uintptr_t)col.dst_stride;
    if (nb <= kSmallRow) {
      col.chunks = 0;
      // plain copies of whole 4-byte words (a, r, done, Q heads): a lane per word
      col.vec = col.conv == CONV_COPY && nb % 4 == 0 && al % 4 == 0;
      blocks += ((col.vec ? a.n * (nb / 4) : a.n) + kCopyThreads - 1) / kCopyThreads;
      continue;
    }
    if (col.conv == CONV_STACK) {
      col.chunk_in = 16 * kCopyThreads;
      col.chunks = (nb + col.chunk_in - 1) / col.chunk_in;
      col.vec = 1;  // frame_bytes % 16 == 0 and 16-byte aligned store / output (checked at attach)
      blocks += a.n * col.chunks;
      continue;
    }
    if (col.conv == CONV_U8_F32_HWC) {
      const int64_t P = nb / col.planes;
      col.chunk_px = 4 * kCopyThreads;  // 1,024 pixels per HWC chunk
      col.chunk_in = col.chunk_px * col.planes;
      col.chunks = (P + col.chunk_px - 1) / col.chunk_px;
      col.vec = (al % 16 == 0) && P % 4 == 0;
    } else {
      col.chunk_in = 16 * kCopyThreads * (col.conv == CONV_COPY ? kCopyVec : 1);
      col.chunks = (nb + col.chunk_in - 1) / col.chunk_in;
      col.vec = al % 16 == 0;
    }
    blocks += a.n * col.chunks;
  }
  RTH_REQUIRE(blocks < (int64_t(1) << 31), "copy: grid too large (%lld workgroups)", (long long)blocks);
  size_t lds = 0;
  for (int c = 0; c < a.ncols; ++c)
    if (a.col[c].conv == CONV_U8_F32_HWC && a.col[c].chunks) lds = (size_t)4 * a.col[c].chunk_px;  // 4 planes x chunk_px bytes
  hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)blocks), dim3(kCopyThreads), lds, s, a);
  RTH_LAUNCHED();
  return RTH_OK;
}

int conv_of(int32_t in_dtype, int32_t out_dtype, int32_t planes, int32_t *conv) {
  if (planes < 0 || planes > 64) {
    set_error("out_planes %d out of range", planes);
    return RTH_ERR_INVALID;
  }
  if (in_dtype == out_dtype && planes == 0) {
    *conv = CONV_COPY;
    return RTH_OK;
  }
  if (in_dtype == RTH_U8 && out_dtype == RTH_F32) {
    *conv = planes ? CONV_U8_F32_HWC : CONV_U8_F32;
    return RTH_OK;
  }
  set_error("unsupported column conversion %d -> %d", in_dtype, out_dtype);
  return RTH_ERR_INVALID;
}

// ---------------------------------------------------------------- frame store
// The actors' new frames enter the store once (rth_replay_push_frames); every stack is a tuple
// of K frame ids in the actors' stack table (sid, one row per frame-ring stack), rows store
// the tuples of their s0 / s1 stacks, and the gather assembles the stacks.  Per actor step:
//   mode 0 (step): actor i's new stack s1_h[i] = its old stack s0_h[i] shifted by one frame +
//     the new frame (FrameStack.step): the new frame (frame K-1 of s1) gets id head + i and
//     sid[s1] = sid[s0][1..K-1] ++ [head + i]; where done[i], the reset stack (slot cur_slot[i])
//     is one frame K times (FrameStack.reset): it gets id head + N + (done actors before i)
//     and sid[reset] = [that id] x K;
//   mode 1 (init): actor i's current stack (slot cur_slot[i]) enters as K new frames
//     head + K i .. head + K i + K - 1.
// One workgroup per actor copies its frame(s) (7,056 bytes each at Atari size, 16-byte
// vectors); the launch's last workgroup (a ticket in fhead[1]) then moves the head past the
// frames of the step -- every workgroup read it at its start, before taking its ticket (r05:
// was a second launch, k_frames_advance).
constexpr int kFrameThreads = 256;

__global__ __launch_bounds__(kFrameThreads) void k_frames_push(const uint8_t *__restrict__ ring, int64_t stack_bytes,
                                                               int64_t frame_bytes, int K, int ring_slots,
                                                               const int64_t *__restrict__ s0_h,
                                                               const int64_t *__restrict__ s1_h,
                                                               const float *__restrict__ done,
                                                               const int64_t *__restrict__ cur_slot,
                                                               int32_t *__restrict__ sid, uint8_t *__restrict__ store,
                                                               int64_t fcap, int64_t *fhead, int64_t n, int mode,
                                                               int ticket) {
  __shared__ int64_t part[kFrameThreads];
  __shared__ int last;
  const int64_t i = blockIdx.x;
  const int64_t head = *fhead;
  // the last workgroup to finish moves the head: N (+ one per done actor in mode 0, K per
  // actor in mode 1).  Relaxed atomics suffice: no data is handed between the workgroups, only
  // the order "every read of the head, then its one write" (the next push reads it after the
  // launch boundary).
  auto advance = [&]() {
    if (!ticket) return;
    __syncthreads();  // every lane's use of head is behind it
    if (threadIdx.x == 0) {
      unsigned int *ticket = reinterpret_cast<unsigned int *>(fhead + 1);
      last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned int)(n - 1);
    }
    __syncthreads();
    if (!last) return;  // workgroup-uniform
    int64_t c = 0;
    if (mode == 0)
      for (int64_t j = threadIdx.x; j < n; j += kFrameThreads) c += done[j] != 0.0f;
    part[threadIdx.x] = c;
    __syncthreads();
    for (int w = kFrameThreads / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      __hip_atomic_store(fhead, head + (mode == 1 ? (int64_t)K * n : n + part[0]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<unsigned int *>(fhead + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  const int64_t vecs = frame_bytes / 16;
  // a frame's vectors, two per lane per round: both loads issued before either store (the
  // one-at-a-time loop waited for each load in turn); the second index clamped, not branched
  auto copy = [&](const uint8_t *src, int64_t fid) {
    uint4 *d = reinterpret_cast<uint4 *>(store + (fid % fcap) * frame_bytes);
    const uint4 *sv = reinterpret_cast<const uint4 *>(src);
    for (int64_t v = threadIdx.x; v < vecs; v += 2 * kFrameThreads) {
      const int64_t v2 = v + kFrameThreads;
      const uint4 x0 = sv[v], x1 = sv[v2 < vecs ? v2 : v];
      d[v] = x0;
      if (v2 < vecs) d[v2] = x1;
    }
  };
  if (mode == 1) {
    const int64_t st = i * ring_slots + cur_slot[i];
    for (int k = 0; k < K; ++k) copy(ring + st * stack_bytes + k * frame_bytes, head + K * i + k);
    if (threadIdx.x < K) sid[st * K + threadIdx.x] = (int32_t)(uint32_t)((head + K * i + threadIdx.x) % fcap);
    advance();
    return;
  }
  const int64_t h0 = s0_h[i], h1 = s1_h[i];
  copy(ring + h1 * stack_bytes + (K - 1) * frame_bytes, head + i);
  if (threadIdx.x < K)  // the shifted tuple: read sid[s0] (another ring slot than s1) before writing s1's
    sid[h1 * K + threadIdx.x] = threadIdx.x + 1 < K ? sid[h0 * K + threadIdx.x + 1]
                                                    : (int32_t)(uint32_t)((head + i) % fcap);
  if (done[i] != 0.0f) {  // workgroup-uniform; rare (p_done), so the rank is a plain count
    int64_t r = 0;
    for (int64_t j = 0; j < i; ++j) r += done[j] != 0.0f;
    const int64_t rs = i * ring_slots + cur_slot[i], fid = head + n + r;
    copy(ring + rs * stack_bytes, fid);
    if (threadIdx.x < K) sid[rs * K + threadIdx.x] = (int32_t)(uint32_t)(fid % fcap);
  }
  advance();
}

}  // namespace rth

using namespace rth;

struct rth_replay {
  int64_t cap;
  int device;
  uint64_t seed;
  int32_t ncols;
  int32_t kind;  // RTH_SAMPLER_*
  rth_col_desc desc[RTH_MAX_COLS];
  uint8_t *store[RTH_MAX_COLS];
  rth_sumtree *tree;   // PER
  int64_t *ulist;      // uniform: index list
  int64_t *fidx;       // FIFO: queue ring (index, weight)
  double *fw;
  rth_schedule alpha, beta;
  ReplayState *st;     // device-resident service state (authoritative)
  SamplerState *ss;    // device-resident uniform / FIFO sampler state
  // host mirrors of the service counters (append_loop / sampler_loop bookkeeping)
  int64_t tail, size, cnt, sample_calls, sched_steps, slen;
  UpdPending pend;  // a deferred PER update, applied by the next tree launch
  int has_pend;
  // sample calls whose st->calls advance is still owed: a sample without out_cols leaves it to
  // the gather that follows (rth_replay_gather), or to the next sample when none does; the
  // advance is stream-ordered after the sample that owes it (owed_stream)
  int64_t calls_owed;
  hipStream_t owed_stream;
  // the last owed-counter advance that ran on a stream other than the one the next sample may
  // use: recorded after it (one event per handle, created on first use), and every sample on
  // another stream waits for it before reading the counter (outside graph capture)
  hipEvent_t bump_ev;
  hipStream_t bump_stream;
  int bump_valid;
  // frame store (rth_replay_frames_attach): the frames the RTH_FRAMES columns' ids point at, a
  // ring of fcap frames of frame_bytes written by rth_replay_push_frames at *fhead
  uint8_t *fstore;
  int64_t fcap, frame_bytes;
  int64_t *fhead;  // device: frames pushed so far (the next frame id)
  // rth_replay_frames_ids_out: gathers write the frame-stack columns' stored id tuples (int32
  // [n][stack]) instead of assembling the stacks; the conv1 kernels read the frames in place
  int32_t ids_out;
  // rth_replay_set_timing: one-shot events recorded around the next launches of each kind
  hipEvent_t timing[RTH_TIMING_SLOTS];
  int32_t timing_fired;  // bit k: slot k's event was recorded since the last arm
};

// bytes of one stored row of column c: a frame-stack column keeps out_planes int32 frame ids
static int64_t stored_row_bytes(const rth_col_desc &d) {
  return d.in_dtype == RTH_FRAMES ? (int64_t)d.out_planes * 4 : d.row_elems * dtype_size(d.in_dtype);
}

// record the one-shot timing event of slot k (if armed) on stream s
static void timing_mark(rth_replay *h, int k, hipStream_t s) {
  if (h->timing[k]) {
    (void)hipEventRecord(h->timing[k], s);
    h->timing[k] = nullptr;
    h->timing_fired |= 1 << k;
  }
}

static int bump(rth_replay *h, int64_t dtail, int64_t dcalls, int64_t dstep, hipStream_t s);

// apply a deferred update on its own (before a sample, an immediate update, a flush)
static int flush_pending(rth_replay *h, hipStream_t s) {
  if (!h->has_pend) return RTH_OK;
  h->has_pend = 0;
  return tree_update_impl(h->tree, nullptr, 0, nullptr, nullptr, RTH_F32, 0.0, 0, s, h->st, &h->alpha, &h->pend, 0);
}

// sampler update for n indices (given, or the FIFO slots of an append when idx == NULL)
static int sampler_update(rth_replay *h, const int64_t *idx, const void *w, int32_t wdt, int64_t n, hipStream_t s) {
  if (n <= 0) return RTH_OK;
  switch (h->kind) {
    case RTH_SAMPLER_PER:
      return tree_update_impl(h->tree, idx, 0, nullptr, w, wdt, 0.0, n, s, h->st, &h->alpha);
    case RTH_SAMPLER_UNIFORM:
      hipLaunchKernelGGL(k_uniform_push, dim3(1), dim3(kSampThreads), 0, s, h->ulist, h->ss, h->cap, idx, h->st, n);
      RTH_LAUNCHED();
      h->slen = h->slen + n < h->cap ? h->slen + n : h->cap;
      return RTH_OK;
    default:
      RTH_REQUIRE(wdt == RTH_F32 || wdt == RTH_F64 || wdt == RTH_PRIO_RAW, "FIFO sampler: weights must be f32/f64");
      hipLaunchKernelGGL(k_fifo_push, dim3(1), dim3(kSampThreads), 0, s, h->fidx, h->fw, h->ss, h->cap, idx, h->st, w,
                         wdt == RTH_F32 ? RTH_F32 : RTH_F64, n);
      RTH_LAUNCHED();
      h->slen = h->slen + n < h->cap ? h->slen + n : h->cap;
      return RTH_OK;
  }
}

static int bump(rth_replay *h, int64_t dtail, int64_t dcalls, int64_t dstep, hipStream_t s) {
  hipLaunchKernelGGL(k_state_bump, dim3(1), dim3(64), 0, s, h->st, dtail, h->cap, dcalls, dstep);
  RTH_LAUNCHED();
  return RTH_OK;
}

static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// the owed seed-counter advance of an earlier sample, on that sample's stream (behind the
// sample kernel that read the counter); remembered so that a sample on any other stream is
// ordered behind it (order_after_bump)
static int bump_owed(rth_replay *h, int64_t owed) {
  int rc = bump(h, 0, owed, 0, h->owed_stream);
  if (rc) return rc;
  if (capturing(h->owed_stream)) return RTH_OK;  // inside a capture the graph's own order holds
  if (!h->bump_ev) RTH_HIP(hipEventCreateWithFlags(&h->bump_ev, hipEventDisableTiming));
  RTH_HIP(hipEventRecord(h->bump_ev, h->owed_stream));
  h->bump_stream = h->owed_stream;
  h->bump_valid = 1;
  return RTH_OK;
}

static int order_after_bump(rth_replay *h, hipStream_t s) {
  if (h->bump_valid && h->bump_stream != s && !capturing(s)) RTH_HIP(hipStreamWaitEvent(s, h->bump_ev, 0));
  return RTH_OK;
}

extern "C" {
int rth_sumtree_create(int64_t capacity, int device, rth_sumtree **out);
int rth_sumtree_destroy(rth_sumtree *t);

int rth_copy_rows(void *dst, int64_t dst_stride, const int64_t *dst_rows, const void *src, int64_t src_stride,
                  const int64_t *src_rows, int64_t n, int64_t row_elems, int32_t in_dtype, int32_t out_dtype,
                  int32_t out_planes, void *stream) {
  RTH_REQUIRE(n == 0 || (dst && src), "rth_copy_rows: NULL buffer");
  RTH_REQUIRE(dtype_size(in_dtype) > 0 && dtype_size(out_dtype) > 0, "rth_copy_rows: bad dtype");
  RTH_REQUIRE(out_planes == 0 || row_elems % out_planes == 0, "rth_copy_rows: row not divisible into planes");
  CopyArgs a{};
  int32_t conv;
  int rc = conv_of(in_dtype, out_dtype, out_planes, &conv);
  if (rc) return rc;
  const int64_t in_bytes = row_elems * dtype_size(in_dtype);
  const int64_t out_bytes = row_elems * dtype_size(out_dtype);
  a.col[0] = CopyCol{(const uint8_t *)src, (uint8_t *)dst, src_rows, dst_rows,
                     src_stride ? src_stride : in_bytes, dst_stride ? dst_stride : out_bytes, in_bytes, conv, out_planes};
  a.n = n;
  a.ncols = 1;
  return launch_copy(a, as_stream(stream));
}

int rth_counter_add(int64_t *c, int64_t d, void *stream) {
  RTH_REQUIRE(c, "rth_counter_add: NULL counter");
  hipLaunchKernelGGL(k_counter_add, dim3(1), dim3(64), 0, as_stream(stream), c, d);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_replay_create(int64_t capacity, int32_t n_cols, const rth_col_desc *cols, int32_t sampler,
                      const rth_schedule *alpha, const rth_schedule *beta, int device, uint64_t seed,
                      rth_replay **out) {
  RTH_REQUIRE(out && cols && alpha && beta, "rth_replay_create: NULL argument");
  RTH_REQUIRE(sampler >= RTH_SAMPLER_PER && sampler <= RTH_SAMPLER_FIFO, "rth_replay_create: bad sampler %d", sampler);
  for (const rth_schedule *sc : {alpha, beta})
    RTH_REQUIRE(sc->method >= RTH_SCHED_CONST && sc->method <= RTH_SCHED_EXP &&
                    (sc->method == RTH_SCHED_CONST || sc->max_steps >= 1),
                "rth_replay_create: bad schedule (method %d, max_steps %lld)", sc->method, (long long)sc->max_steps);
  RTH_REQUIRE(n_cols >= 1 && n_cols <= RTH_MAX_COLS, "rth_replay_create: n_cols=%d not in [1,%d]", n_cols,
              RTH_MAX_COLS);
  RTH_REQUIRE(capacity >= 1, "rth_replay_create: capacity must be >= 1");
  for (int c = 0; c < n_cols; ++c) {
    int32_t conv;
    RTH_REQUIRE(cols[c].row_elems >= 1, "rth_replay_create: column %d has no elements", c);
    RTH_REQUIRE(cols[c].out_planes == 0 || cols[c].row_elems % cols[c].out_planes == 0,
                "rth_replay_create: column %d not divisible into %d planes", c, cols[c].out_planes);
    if (cols[c].in_dtype == RTH_FRAMES) {  // K frame ids -> K frames of row_elems / K bytes
      RTH_REQUIRE(cols[c].out_dtype == RTH_U8 && cols[c].out_planes >= 1 &&
                      (cols[c].row_elems / cols[c].out_planes) % 16 == 0,
                  "rth_replay_create: frame-stack column %d: u8 output of out_planes frames of a multiple of 16 bytes", c);
      continue;
    }
    int rc = conv_of(cols[c].in_dtype, cols[c].out_dtype, cols[c].out_planes, &conv);
    if (rc) return rc;
  }
  RTH_HIP(hipSetDevice(device));
  auto *h = new rth_replay{};
  h->cap = capacity;
  h->device = device;
  h->seed = seed;
  h->ncols = n_cols;
  h->kind = sampler;
  h->alpha = *alpha;
  h->beta = *beta;
  void *state = nullptr;
  if (hipMalloc(&state, sizeof(ReplayState) + sizeof(SamplerState)) != hipSuccess) {
    delete h;
    set_error("rth_replay_create: hipMalloc(state) failed");
    return RTH_ERR_NOMEM;
  }
  h->st = static_cast<ReplayState *>(state);
  h->ss = reinterpret_cast<SamplerState *>(h->st + 1);
  RTH_HIP(hipMemset(state, 0, sizeof(ReplayState) + sizeof(SamplerState)));
  for (int c = 0; c < n_cols; ++c) {
    h->desc[c] = cols[c];
    const size_t bytes = (size_t)capacity * stored_row_bytes(cols[c]);
    if (hipMalloc(&h->store[c], bytes) != hipSuccess) {
      set_error("rth_replay_create: hipMalloc(%zu) for column %d failed", bytes, c);
      for (int k = 0; k < c; ++k) (void)hipFree(h->store[k]);
      delete h;
      return RTH_ERR_NOMEM;
    }
  }
  int rc = RTH_OK;
  if (sampler == RTH_SAMPLER_PER) {
    rc = rth_sumtree_create(capacity, device, &h->tree);
  } else if (sampler == RTH_SAMPLER_UNIFORM) {
    if (hipMalloc(&h->ulist, (size_t)capacity * 8) != hipSuccess) rc = RTH_ERR_NOMEM;
  } else if (hipMalloc(&h->fidx, (size_t)capacity * 8) != hipSuccess ||
             hipMalloc(&h->fw, (size_t)capacity * 8) != hipSuccess) {
    rc = RTH_ERR_NOMEM;
  }
  if (rc) {
    if (rc == RTH_ERR_NOMEM) set_error("rth_replay_create: sampler state allocation failed");
    rth_replay_destroy(h);
    return rc;
  }
  *out = h;
  return RTH_OK;
}

int rth_replay_destroy(rth_replay *h) {
  if (!h) return RTH_OK;
  (void)hipSetDevice(h->device);
  for (int c = 0; c < h->ncols; ++c) (void)hipFree(h->store[c]);
  (void)hipFree(h->st);
  if (h->tree) rth_sumtree_destroy(h->tree);
  for (void *p : {(void *)h->ulist, (void *)h->fidx, (void *)h->fw})
    if (p) (void)hipFree(p);
  if (h->bump_ev) (void)hipEventDestroy(h->bump_ev);
  if (h->fstore) (void)hipFree(h->fstore);
  if (h->fhead) (void)hipFree(h->fhead);
  delete h;
  return RTH_OK;
}

int rth_replay_set_timing(rth_replay *h, void *const *events, int32_t n, int32_t *fired_out) {
  RTH_REQUIRE(h && (n == 0 || events) && n >= 0 && n <= RTH_TIMING_SLOTS, "rth_replay_set_timing: bad arguments");
  if (fired_out) *fired_out = h->timing_fired;
  h->timing_fired = 0;
  for (int k = 0; k < RTH_TIMING_SLOTS; ++k) h->timing[k] = k < n ? static_cast<hipEvent_t>(events[k]) : nullptr;
  return RTH_OK;
}

rth_sumtree *rth_replay_tree(rth_replay *h) { return h ? h->tree : nullptr; }

int rth_replay_frames_attach(rth_replay *h, int64_t n_frames, int64_t frame_bytes, void **store_out,
                             int64_t **head_out) {
  RTH_REQUIRE(h && n_frames >= 1 && frame_bytes >= 16 && frame_bytes % 16 == 0,
              "rth_replay_frames_attach: bad arguments (frames >= 1, frame bytes a multiple of 16)");
  RTH_REQUIRE(n_frames < (int64_t(1) << 31), "rth_replay_frames_attach: %lld frames exceed the int32 frame ids",
              (long long)n_frames);
  RTH_REQUIRE(!h->fstore, "rth_replay_frames_attach: the frame store is already attached");
  bool any = false;
  for (int c = 0; c < h->ncols; ++c)
    if (h->desc[c].in_dtype == RTH_FRAMES) {
      RTH_REQUIRE(h->desc[c].row_elems == h->desc[c].out_planes * frame_bytes,
                  "rth_replay_frames_attach: column %d holds %lld-element stacks of %d frames, not %lld-byte frames", c,
                  (long long)h->desc[c].row_elems, h->desc[c].out_planes, (long long)frame_bytes);
      any = true;
    }
  RTH_REQUIRE(any, "rth_replay_frames_attach: the replay has no frame-stack (RTH_FRAMES) column");
  RTH_HIP(hipSetDevice(h->device));
  if (hipMalloc(&h->fstore, (size_t)n_frames * frame_bytes) != hipSuccess) {
    h->fstore = nullptr;
    set_error("rth_replay_frames_attach: hipMalloc(%lld x %lld) failed", (long long)n_frames, (long long)frame_bytes);
    return RTH_ERR_NOMEM;
  }
  if (hipMalloc(&h->fhead, 16) != hipSuccess) {  // [the next frame id, k_frames_push's ticket]
    (void)hipFree(h->fstore);
    h->fstore = nullptr;
    return RTH_ERR_NOMEM;
  }
  RTH_HIP(hipMemset(h->fstore, 0, (size_t)n_frames * frame_bytes));
  RTH_HIP(hipMemset(h->fhead, 0, 16));
  h->fcap = n_frames;
  h->frame_bytes = frame_bytes;
  if (store_out) *store_out = h->fstore;
  if (head_out) *head_out = h->fhead;
  return RTH_OK;
}

int rth_replay_frames_ids_out(rth_replay *h, int32_t on) {
  RTH_REQUIRE(h && h->fstore, "rth_replay_frames_ids_out: no frame store attached");
  bool stacks4 = true;
  for (int c = 0; c < h->ncols; ++c)
    if (h->desc[c].in_dtype == RTH_FRAMES) stacks4 = stacks4 && h->desc[c].out_planes == 4;
  RTH_REQUIRE(!on || stacks4, "rth_replay_frames_ids_out: id tuples are read as int4 (4-frame stacks only)");
  h->ids_out = on ? 1 : 0;
  return RTH_OK;
}

int rth_replay_push_frames(rth_replay *h, const uint8_t *ring, int64_t n, int32_t ring_slots, int32_t stack,
                           const int64_t *s0_h, const int64_t *s1_h, const float *done, const int64_t *cur_slot,
                           int32_t *sid, int32_t mode, void *stream) {
  RTH_REQUIRE(h && h->fstore, "rth_replay_push_frames: no frame store attached");
  RTH_REQUIRE(ring && sid && cur_slot && n >= 0 && n <= 65535 && ring_slots >= 1 && stack >= 1 && stack <= 64 &&
                  (mode == 1 || (mode == 0 && s0_h && s1_h && done)),
              "rth_replay_push_frames: bad arguments");
  if (n == 0) return RTH_OK;
  const int64_t stack_bytes = (int64_t)stack * h->frame_bytes;
  hipStream_t s = as_stream(stream);
  // the head advance (N + the done count) runs in the push launch's last workgroup
  hipLaunchKernelGGL(k_frames_push, dim3((unsigned)n), dim3(kFrameThreads), 0, s, ring, stack_bytes, h->frame_bytes,
                     (int)stack, (int)ring_slots, s0_h, s1_h, done, cur_slot, sid, h->fstore, h->fcap, h->fhead, n,
                     (int)mode, 1);
  RTH_LAUNCHED();
  return RTH_OK;
}

void *rth_replay_column(rth_replay *h, int32_t c) {
  return (h && c >= 0 && c < h->ncols) ? (void *)h->store[c] : nullptr;
}

int rth_replay_info(const rth_replay *h, int64_t *size, int64_t *tail, int64_t *cnt, int64_t *calls, int64_t *steps,
                    int64_t *sampler_len) {
  RTH_REQUIRE(h, "rth_replay_info: NULL handle");
  if (sampler_len) *sampler_len = h->kind == RTH_SAMPLER_PER ? h->size : h->slen;
  if (size) *size = h->size;
  if (tail) *tail = h->tail;
  if (cnt) *cnt = h->cnt;
  if (calls) *calls = h->sample_calls;
  if (steps) *steps = h->sched_steps;
  return RTH_OK;
}

int rth_replay_append(rth_replay *h, const rth_src *srcs, const void *td_abs, int32_t td_dtype, int64_t n,
                      int64_t *idx_out, void *stream) {
  RTH_REQUIRE(h && srcs, "rth_replay_append: NULL argument");
  RTH_REQUIRE(n >= 0 && n <= h->cap, "rth_replay_append: n=%lld exceeds capacity %lld (fifo_policy.py:12)",
              (long long)n, (long long)h->cap);
  if (n == 0) return RTH_OK;
  RTH_REQUIRE(td_abs, "rth_replay_append: NULL priorities");
  hipStream_t s = as_stream(stream);
  CopyArgs a{};
  for (int c = 0; c < h->ncols; ++c) {
    RTH_REQUIRE(srcs[c].base_dev, "rth_replay_append: column %d source is NULL", c);
    const rth_col_desc &d = h->desc[c];
    const int64_t rb = stored_row_bytes(d);  // frame-stack columns: the K ids (rth_replay_push_frames' table rows)
    int32_t conv = CONV_COPY;
    int64_t ib = rb;  // bytes of one source row
    if (srcs[c].src_dtype != 0 && srcs[c].src_dtype != d.in_dtype) {
      RTH_REQUIRE(srcs[c].src_dtype == RTH_F32 && d.in_dtype == RTH_U8,
                  "rth_replay_append: column %d: source type %d into storage type %d is not supported", c,
                  srcs[c].src_dtype, d.in_dtype);
      conv = CONV_F32_U8;
      ib = d.row_elems * 4;
    }
    a.col[c] = CopyCol{(const uint8_t *)srcs[c].base_dev, h->store[c], srcs[c].rows_dev, nullptr,
                       srcs[c].row_stride_bytes ? srcs[c].row_stride_bytes : ib, rb, ib, conv, 0};
  }
  a.n = n;
  a.ncols = h->ncols;
  a.dst_fifo = 1;
  a.st = h->st;
  a.fifo_cap = h->cap;
  timing_mark(h, RTH_TIMING_INSERT, s);
  int rc = launch_copy(a, s);
  timing_mark(h, RTH_TIMING_INSERT + 1, s);
  if (rc) return rc;
  if (idx_out) {  // FIFO slots for the caller (the append_loop's `indices`)
    hipLaunchKernelGGL(k_fifo_slots, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, idx_out, n, h->st, h->cap);
    RTH_LAUNCHED();
  }
  if (h->kind == RTH_SAMPLER_PER) {
    // one tree launch: a deferred update_priorities (if any), this append's priorities,
    // then the FIFO tail advance -- the sequential order of the reference's messages
    timing_mark(h, RTH_TIMING_TREE_UPDATE, s);
    rc = tree_update_impl(h->tree, nullptr, 0, nullptr, td_abs, td_dtype, 0.0, n, s, h->st, &h->alpha,
                          h->has_pend ? &h->pend : nullptr, 1);
    timing_mark(h, RTH_TIMING_TREE_UPDATE + 1, s);
    h->has_pend = 0;
    if (rc) return rc;
  } else {
    rc = sampler_update(h, nullptr, td_abs, td_dtype, n, s);
    if (rc) return rc;
    rc = bump(h, n, 0, 0, s);
    if (rc) return rc;
  }
  h->tail = (h->tail + n) % h->cap;
  h->size = h->size + n < h->cap ? h->size + n : h->cap;
  h->cnt += n;
  return RTH_OK;
}

static int gather_impl(rth_replay *h, const int64_t *idx, int64_t n, void *const *out_cols, hipStream_t s) {
  RTH_REQUIRE(h && (n == 0 || (idx && out_cols)), "rth_replay_gather: bad arguments");
  CopyArgs a{};
  for (int c = 0; n > 0 && c < h->ncols; ++c) {
    RTH_REQUIRE(out_cols[c], "rth_replay_gather: output column %d is NULL", c);
    const rth_col_desc &d = h->desc[c];
    if (d.in_dtype == RTH_FRAMES && h->ids_out) {  // the stored id tuples (one lane per 4-byte word)
      RTH_REQUIRE((reinterpret_cast<uintptr_t>(out_cols[c]) & 15) == 0, "rth_replay_gather: frame-id column %d not "
                  "16-byte aligned", c);
      const int64_t sb = stored_row_bytes(d);
      a.col[c] = CopyCol{h->store[c], (uint8_t *)out_cols[c], idx, nullptr, sb, sb, sb, CONV_COPY, 0};
      continue;
    }
    if (d.in_dtype == RTH_FRAMES) {  // the stack assembled from the frame store
      RTH_REQUIRE(h->fstore, "rth_replay_gather: frame-stack column %d without a frame store", c);
      const int64_t ob = d.row_elems;
      CopyCol col{h->store[c], (uint8_t *)out_cols[c], idx, nullptr, stored_row_bytes(d), ob, ob, CONV_STACK,
                  d.out_planes};
      col.fstore = h->fstore;
      col.frame_bytes = h->frame_bytes;
      col.fcap = h->fcap;
      RTH_REQUIRE((reinterpret_cast<uintptr_t>(out_cols[c]) & 15) == 0, "rth_replay_gather: output column %d not "
                  "16-byte aligned", c);
      a.col[c] = col;
      continue;
    }
    int32_t conv;
    conv_of(d.in_dtype, d.out_dtype, d.out_planes, &conv);
    const int64_t ib = d.row_elems * dtype_size(d.in_dtype), ob = d.row_elems * dtype_size(d.out_dtype);
    a.col[c] = CopyCol{h->store[c], (uint8_t *)out_cols[c], idx, nullptr, ib, ob, ib, conv, d.out_planes};
  }
  a.n = n;
  a.ncols = h->ncols;
  const int64_t owed = h->calls_owed;
  h->calls_owed = 0;
  if (owed && (n == 0 || s != h->owed_stream)) {
    // on the sample's own stream, behind the sample kernel that reads the counter (a gather
    // on another stream could otherwise advance it first); later samples on other streams
    // wait for it (order_after_bump)
    int rc = bump_owed(h, owed);
    if (rc || n == 0) return rc;
  } else if (owed) {  // same stream: the gather's first lane advances the counter, no launch
    a.bump_st = h->st;
    a.bump_calls = owed;
  }
  if (n == 0) return RTH_OK;
  timing_mark(h, RTH_TIMING_GATHER, s);
  const int rc = launch_copy(a, s);
  timing_mark(h, RTH_TIMING_GATHER + 1, s);
  return rc;
}

int rth_replay_gather(rth_replay *h, const int64_t *idx, int64_t n, void *const *out_cols, void *stream) {
  return gather_impl(h, idx, n, out_cols, as_stream(stream));
}

int rth_replay_sample(rth_replay *h, int64_t batch, const double *uniforms, void *const *out_cols,
                      int64_t *idx_out, double *isw_out, void *stream) {
  RTH_REQUIRE(h && batch > 0 && idx_out && isw_out, "rth_replay_sample: bad arguments");
  hipStream_t s = as_stream(stream);
  int rc = flush_pending(h, s);
  if (rc) return rc;
  if (h->calls_owed) {  // the previous sample was not followed by a gather: its seed advance first
    rc = bump_owed(h, h->calls_owed);
    h->calls_owed = 0;
    if (rc) return rc;
  }
  rc = order_after_bump(h, s);  // this sample reads the counter: behind any advance on another stream
  if (rc) return rc;
  if (h->kind == RTH_SAMPLER_PER) {
    timing_mark(h, RTH_TIMING_SAMPLE, s);
    rc = tree_sample_impl(h->tree, batch, uniforms, h->seed, 0, 1, 0.0, idx_out, isw_out, s, h->st, &h->beta);
    timing_mark(h, RTH_TIMING_SAMPLE + 1, s);
  } else if (h->kind == RTH_SAMPLER_UNIFORM) {
    RTH_REQUIRE(h->slen > 0, "rth_replay_sample: uniform sampler is empty (np.random.choice(0, ...))");
    hipLaunchKernelGGL(k_uniform_sample, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, h->ulist, h->ss, h->st,
                       batch, uniforms, h->seed, idx_out, isw_out);
    RTH_LAUNCHED();
  } else {
    RTH_REQUIRE(h->slen >= batch, "rth_replay_sample: FIFO sampler holds %lld < batch %lld (deque.pop from empty)",
                (long long)h->slen, (long long)batch);
    hipLaunchKernelGGL(k_fifo_pop, dim3(1), dim3(kSampThreads), 0, s, h->fidx, h->fw, h->ss, h->cap, batch, idx_out,
                       isw_out);
    RTH_LAUNCHED();
    h->slen -= batch;
  }
  if (rc) return rc;
  h->sample_calls++;
  h->calls_owed = 1;  // advanced by the gather (this one, or the caller's rth_replay_gather next)
  h->owed_stream = s;
  return out_cols ? gather_impl(h, idx_out, batch, out_cols, s) : RTH_OK;
}

int rth_replay_update_priorities(rth_replay *h, const int64_t *idx, const void *td_abs, int32_t td_dtype, int64_t n,
                                 int32_t step, void *stream) {
  RTH_REQUIRE(h && (n == 0 || (idx && td_abs)), "rth_replay_update_priorities: bad arguments");
  hipStream_t s = as_stream(stream);
  int rc = flush_pending(h, s);
  if (rc) return rc;
  if (step) {  // sampler_loop.py:32-33: on_step() before the update
    rc = bump(h, 0, 0, 1, s);
    if (rc) return rc;
    h->sched_steps++;
  }
  rc = sampler_update(h, idx, td_abs, td_dtype, n, s);
  if (rc) return rc;
  h->cnt += n;
  return RTH_OK;
}

int rth_replay_update_priorities_deferred(rth_replay *h, const int64_t *idx, const void *td_abs, int32_t td_dtype,
                                          int64_t n, int32_t step, void *stream) {
  RTH_REQUIRE(h && n >= 0 && (n == 0 || (idx && td_abs)), "rth_replay_update_priorities_deferred: bad arguments");
  if (h->kind != RTH_SAMPLER_PER) return rth_replay_update_priorities(h, idx, td_abs, td_dtype, n, step, stream);
  RTH_REQUIRE(n == 0 || td_dtype == RTH_F32 || td_dtype == RTH_F64 || td_dtype == RTH_PRIO_RAW,
              "rth_replay_update_priorities_deferred: priority dtype must be f32, f64 or raw f64");
  int rc = flush_pending(h, as_stream(stream));  // at most one update in flight
  if (rc) return rc;
  h->pend = UpdPending{idx, td_abs, td_dtype, step ? 1 : 0, n};
  h->has_pend = 1;
  if (step) h->sched_steps++;
  h->cnt += n;
  return RTH_OK;
}

int rth_replay_flush(rth_replay *h, void *stream) {
  RTH_REQUIRE(h, "rth_replay_flush: NULL handle");
  return flush_pending(h, as_stream(stream));
}

int rth_uniform_indices(int64_t size, int64_t batch, const double *uniforms, uint64_t seed, uint64_t counter,
                        const int64_t *counter_dev, int64_t *idx_out, void *stream) {
  RTH_REQUIRE(size > 0, "rth_uniform_indices: size must be > 0 (np.random.choice(0, ...))");
  RTH_REQUIRE(batch >= 0 && (batch == 0 || idx_out), "rth_uniform_indices: bad arguments");
  if (batch == 0) return RTH_OK;
  hipLaunchKernelGGL(k_uniform_indices, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, as_stream(stream), size,
                     batch, uniforms, seed, counter, counter_dev, idx_out);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
