// FC1 of the dueling heads on the bf16 MFMA with both operands split into three exact bf16
// terms (the x9 scheme of conv.hip's k_conv_x9: every partial product xi * wj has at most 16
// significant bits, so it is exact in the fp32 accumulator -- the products of an fp32 GEMM,
// summed in another fixed order).  Reference: the first Linear of both branches of
// reth/reth/algorithm/dqn/dqn_model.py:38-47 (value / advantage: Linear(3136, 256) + ReLU), run
// by Worker.step -> act, by _calc_td_error's target pass and by the learner's forward
// (dqn_solver.py:68-124); here the two branches' weights are one [512, 3136] storage.
//
//   y[m][n] = act(b[n] + sum_k x[m][k] w[n][k]),  x [M, K] row-major (row stride ldx),
//   w [N, K] row-major (a Linear weight), act = ReLU or identity
//
// Workgroup = 4 waves over a 64 x 128 output tile (wave w: rows 16 w .. 16 w + 15, all 8
// 16-column blocks) and a range of 32-deep k chunks (its split).  Per chunk the workgroup stages
// the 128 weight rows' 32 values split into the three bf16 terms, in fragment order, in LDS
// (double-buffered: one barrier per chunk); each wave loads and splits its own A fragment
// (16 rows x 32 values) in registers and runs 8 x 9 MFMAs.  The next chunk's loads are in flight
// during the MFMAs.  splits > 1: fixed-order partial tiles + k_fc_reduce (bias, activation);
// every sum has a fixed order, so the result is run-to-run deterministic.
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "fc_rows.hpp"

namespace rth {

using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kFcTm = 64, kFcTn = 128, kFcThreads = 256;
__device__ __forceinline__ float fc_relu(float v) { return v < 0.0f ? 0.0f : v; }  // conv.hip's relu_c
constexpr int kFcBUnits = 8 * 3 * 64;  // 16-byte units of one chunk's split weight tile

template <int... I, class F>
__device__ __forceinline__ void static_for(std::integer_sequence<int, I...>, F &&f) {
  (f(std::integral_constant<int, I>{}), ...);
}

// PF: chunks whose global loads are in flight ahead of the one being computed (register ring of
// PF + 1 sets; the LDS weight tile stays double-buffered)
template <int PF>
__global__ __launch_bounds__(kFcThreads) void k_fc_x9(const float *__restrict__ x, int64_t ldx, int M,
                                                      const float *__restrict__ w, int N, int K, int splits,
                                                      const float *__restrict__ bias, int relu,
                                                      float *__restrict__ out) {
  __shared__ uint4 bl[2][kFcBUnits];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = N / kFcTn;
  const int tile = (int)blockIdx.x / splits, split = (int)blockIdx.x % splits;
  const int m0 = (tile / tiles_n) * kFcTm, n0 = (tile % tiles_n) * kFcTn;
  const int chunks = K / 32;
  const int c0 = chunks * split / splits, c1 = chunks * (split + 1) / splits;
  // staging role: weight row n0 + (tid & 127), values 16 (tid >> 7) .. +15 of the chunk
  const int wn = tid & 127, wh = tid >> 7;
  const float *wrow = w + (int64_t)(n0 + wn) * K + 16 * wh;
  const float *xrow = x + (int64_t)(m0 + 16 * wave + r) * ldx + 8 * g;
  constexpr int NR = PF + 1;  // register sets: chunk c's A values + chunks c + 1 .. c + PF in flight
  f32x4 wv[NR][4], xv[NR][2];
  auto load = [&](int c, f32x4 (&wl)[4], f32x4 (&xl)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) wl[j] = *reinterpret_cast<const f32x4 *>(wrow + 32 * c + 4 * j);
#pragma unroll
    for (int j = 0; j < 2; ++j) xl[j] = *reinterpret_cast<const f32x4 *>(xrow + 32 * c + 4 * j);
  };
  // the thread's 16 values = units (nb, t, lane r' + 16 g') for g' = 2 wh, 2 wh + 1
  auto stage = [&](const f32x4 (&wl)[4], uint4 *buf) __attribute__((always_inline)) {
    const int nb = wn >> 4, rr = wn & 15;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float v[8] = {wl[2 * h][0], wl[2 * h][1], wl[2 * h][2], wl[2 * h][3],
                          wl[2 * h + 1][0], wl[2 * h + 1][1], wl[2 * h + 1][2], wl[2 * h + 1][3]};
      bf16x8 tr[3];
      split3_pk8(v, tr);
#pragma unroll
      for (int t = 0; t < 3; ++t) buf[(nb * 3 + t) * 64 + rr + 16 * (2 * wh + h)] = __builtin_bit_cast(uint4, tr[t]);
    }
  };
  f32x4 acc[8];
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const f32x4 (&xl)[2], const uint4 *buf) __attribute__((always_inline)) {
    const float v[8] = {xl[0][0], xl[0][1], xl[0][2], xl[0][3], xl[1][0], xl[1][1], xl[1][2], xl[1][3]};
    bf16x8 af[3];
    split3_pk8(v, af);
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      bf16x8 b[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) b[t] = __builtin_bit_cast(bf16x8, buf[(nb * 3 + t) * 64 + lane]);
      f32x4 a = acc[nb];
      // smallest terms first: (3,3) (3,2) (2,3) (3,1) (2,2) (1,3) (2,1) (1,2) (1,1)
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], b[2], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], b[1], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], b[2], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], b[0], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], b[1], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], b[2], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], b[0], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], b[1], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], b[0], a, 0, 0, 0);
      acc[nb] = a;
    }
  };
  // chunk c = c0 + i: MFMAs from bl[i & 1] with A registers xv[i % NR]; chunk c + 1's weight rows
  // (registers, loaded PF chunks earlier) staged into the other LDS buffer; chunk c + NR loaded
  // into the freed set (past c1 - 1 the loads repeat the range's last chunk: in bounds, unused)
  auto iter = [&](int c, auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;  // (c - c0) mod 2 * NR: the static ring positions
    constexpr int pr = i % NR, pl = i & 1;
    compute(xv[pr], bl[pl]);
    stage(wv[(i + 1) % NR], bl[pl ^ 1]);
    const int cn = c + NR < c1 ? c + NR : c1 - 1;
    load(cn, wv[pr], xv[pr]);
    __syncthreads();
  };
  // before chunk c0 + i: bl[i & 1] = its split weights, xv[i % NR] = its A values, the next PF
  // sets = chunks c + 1 .. c + PF in flight
#pragma unroll
  for (int q = 0; q < NR; ++q) load(c0 + q < c1 ? c0 + q : c1 - 1, wv[q], xv[q]);
  stage(wv[0], bl[0]);
  __syncthreads();
  int c = c0;
  constexpr int U = 2 * NR;  // unroll: both ring positions cycle
  for (; c + U <= c1; c += U)
    static_for(std::make_integer_sequence<int, U>{}, [&](auto ic) __attribute__((always_inline)) {
      iter(c + decltype(ic)::value, ic);
    });
  // the remaining < U chunks, each ring position static
  static_for(std::make_integer_sequence<int, U>{}, [&](auto ic) __attribute__((always_inline)) {
    if (c + decltype(ic)::value < c1) iter(c + decltype(ic)::value, ic);
  });
  // D: lane holds rows 4 g + i of the wave's 16, column r of each 16-column block
  const int mrow = m0 + 16 * wave + 4 * g;
  if (splits == 1) {
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const int n = n0 + 16 * nb + r;
      const float bn = bias ? bias[n] : 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = radd(acc[nb][i], bn);
        out[(int64_t)(mrow + i) * N + n] = relu ? fc_relu(v) : v;
      }
    }
  } else {
    float *part = out + (int64_t)split * M * N;
#pragma unroll
    for (int nb = 0; nb < 8; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(int64_t)(mrow + i) * N + n0 + 16 * nb + r] = acc[nb][i];
  }
}

// The 128 x 128 form (r05; the default where M % 128 == 0, fc_plan): in the 64 x 128 form every 72 MFMAs of a
// wave read 24 split weight fragments from LDS and the wave splits its own 16 activation rows,
// and each weight chunk is split for 64 rows only.  Here BOTH operands of a 32-deep chunk are
// split once per workgroup into LDS fragments (A: 128 rows of x, B: 128 rows of w; 3 bf16 terms
// each, 48 KB per buffer, double-buffered: 96 KB, one barrier per chunk) and each wave owns a
// 64 x (512 / WAVES) block of the tile: 4 x NB output blocks per 12 + 3 NB fragment reads, 36 NB
// MFMAs.  The MFMAs run term-major -- term k of every block before term k + 1 -- so consecutive
// MFMAs never depend on each other; each output's chain is still the 9 terms in the fixed order
// per chunk, chunks in order, splits reduced in order.  Global loads of the next PF chunks are
// in flight in registers while a chunk's MFMAs run.  Measured (r05, profiles/r05/ab_log.txt): 8
// waves beat 4 (2 per SIMD), a ring of 2 chunks in flight and coalesced 8-lanes-per-row staging
// loads do not help; at 512 rows alone the MFMA pipes are 26 % busy (23 us for 5.9 us of bf16
// MFMA work): the waves wait on their loads and the LDS fragments, not on the MFMAs.
constexpr int kFbTile = 128;
// the 9 (A term, B term) pairs, smallest first: (3,3) (3,2) (2,3) (3,1) (2,2) (1,3) (2,1) (1,2) (1,1)
__host__ __device__ constexpr int fc_ta(int k) { return (int)((0x221210100ull >> (4 * (8 - k))) & 15); }
__host__ __device__ constexpr int fc_tb(int k) { return (int)((0x212012010ull >> (4 * (8 - k))) & 15); }
static_assert(fc_ta(0) == 2 && fc_tb(0) == 2 && fc_ta(3) == 2 && fc_tb(3) == 0 && fc_ta(5) == 0 && fc_tb(5) == 2 &&
                  fc_ta(8) == 0 && fc_tb(8) == 0 && fc_ta(6) == 1 && fc_tb(6) == 0,
              "term order");
constexpr int kFbUnits = 8 * 3 * 64;  // 16-byte units of one operand's split chunk (8 blocks x 3 terms)
template <int WAVES, int PF>
__global__ __launch_bounds__(WAVES * 64) void k_fc_x9t(const float *__restrict__ x, int64_t ldx, int M,
                                                      const float *__restrict__ w, int N, int K, int splits,
                                                      const float *__restrict__ bias, int relu,
                                                      float *__restrict__ out) {
  constexpr int T = WAVES * 64, WN = WAVES / 2, NB = 8 / WN;  // waves: 2 along M x WN along N
  constexpr int RH = 2 * 2 * kFbTile / T;                    // row-halves (16 values) staged per thread
  constexpr int NR = PF + 1;                                 // register sets of the load ring
  static_assert(WAVES == 4 || WAVES == 8, "4 or 8 waves");
  __shared__ uint4 sl[2][2][kFbUnits];  // [buffer][A = x, B = w]
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wave & 1, wn = wave >> 1;
  const int tiles_n = N / kFbTile;
  const int tile = (int)blockIdx.x / splits, split = (int)blockIdx.x % splits;
  const int m0 = (tile / tiles_n) * kFbTile, n0 = (tile % tiles_n) * kFbTile;
  const int chunks = K / 32;
  const int c0 = chunks * split / splits, c1 = chunks * (split + 1) / splits;
  // staging role j: row-half u = tid + j T -> operand u >> 8, row u & 127, values 16 ((u >> 7) & 1) ..
  const float *src[RH];
#pragma unroll
  for (int j = 0; j < RH; ++j) {
    const int u = tid + j * T, op = u >> 8, rr = u & 127, h = (u >> 7) & 1;
    src[j] = op == 0 ? x + (int64_t)(m0 + rr) * ldx + 16 * h : w + (int64_t)(n0 + rr) * K + 16 * h;
  }
  f32x4 ring[NR][RH][4];
  auto load = [&](int c, f32x4 (&v)[RH][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < RH; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[j][q] = *reinterpret_cast<const f32x4 *>(src[j] + 32 * c + 4 * q);
  };
  auto stage = [&](const f32x4 (&v)[RH][4], uint4 (*buf)[kFbUnits]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < RH; ++j) {
      const int u = tid + j * T, op = u >> 8, rr = u & 127, h = (u >> 7) & 1;
      const int blk = rr >> 4, rw = rr & 15;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const float vv[8] = {v[j][2 * hh][0], v[j][2 * hh][1], v[j][2 * hh][2], v[j][2 * hh][3],
                             v[j][2 * hh + 1][0], v[j][2 * hh + 1][1], v[j][2 * hh + 1][2], v[j][2 * hh + 1][3]};
        bf16x8 tr[3];
        split3_pk8(vv, tr);
#pragma unroll
        for (int t = 0; t < 3; ++t) buf[op][(blk * 3 + t) * 64 + rw + 16 * (2 * h + hh)] = __builtin_bit_cast(uint4, tr[t]);
      }
    }
  };
  f32x4 acc[4][NB];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](uint4 (*buf)[kFbUnits]) __attribute__((always_inline)) {
    bf16x8 af[4][3], bfr[NB][3];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int t = 0; t < 3; ++t) af[mb][t] = __builtin_bit_cast(bf16x8, buf[0][((4 * wm + mb) * 3 + t) * 64 + lane]);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        bfr[nb][t] = __builtin_bit_cast(bf16x8, buf[1][((NB * wn + nb) * 3 + t) * 64 + lane]);
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mb][fc_ta(k)], bfr[nb][fc_tb(k)], acc[mb][nb], 0, 0, 0);
  };
  // chunk j lives in ring set (j - c0) % NR from its load until it is staged (one iteration
  // before its MFMAs); past c1 - 1 the loads repeat the range's last chunk (in bounds, unused)
  auto clampc = [&](int c) { return c < c1 ? c : c1 - 1; };
#pragma unroll
  for (int q = 0; q < NR; ++q) load(clampc(c0 + q), ring[q]);
  stage(ring[0], sl[0]);
  load(clampc(c0 + NR), ring[0]);
  __syncthreads();
  // iteration i (chunk c0 + i): MFMAs from buffer i & 1; chunk i + 1 staged from its ring set
  // into the other buffer, then chunk i + 1 + NR loaded into that set
  auto iter = [&](int i, auto ic) __attribute__((always_inline)) {
    constexpr int s = decltype(ic)::value;  // i mod 2 NR
    compute(sl[s & 1]);
    stage(ring[(s + 1) % NR], sl[(s + 1) & 1]);
    load(clampc(c0 + i + 1 + NR), ring[(s + 1) % NR]);
    __syncthreads();
  };
  const int n_it = c1 - c0;
  constexpr int U = 2 * NR;
  int i = 0;
  for (; i + U <= n_it; i += U)
    static_for(std::make_integer_sequence<int, U>{}, [&](auto ic) __attribute__((always_inline)) {
      iter(i + decltype(ic)::value, ic);
    });
  static_for(std::make_integer_sequence<int, U>{}, [&](auto ic) __attribute__((always_inline)) {
    if (i + decltype(ic)::value < n_it) iter(i + decltype(ic)::value, ic);
  });
  // D: lane holds rows 4 g + i of each 16-row block, column r of each 16-column block
  float *dst = splits == 1 ? out : out + (int64_t)split * M * N;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = n0 + 16 * (NB * wn + nb) + r;
      const float bn = splits == 1 && bias ? bias[n] : 0.0f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 64 * wm + 16 * mb + 4 * g + e;
        float v = acc[mb][nb][e];
        if (splits == 1) {
          v = radd(v, bn);
          v = relu ? fc_relu(v) : v;
        }
        dst[(int64_t)m * N + n] = v;
      }
    }
}

// FC1 on the fp32 MFMA (v_mfma_f32_16x16x4_f32, the GEMM's own arithmetic) with no LDS (r05,
// hipBLASLt's 512-row tile MT64x16x256 holds 80 KB of LDS per workgroup and runs
// 48 us per launch in the loop against 21-26 alone).  Workgroup = 4 waves over a 64 x 128
// output tile (wave (wm, wn) = rows 32 wm .. +31, columns 64 wn .. +63: 2 x 4 blocks of 16 x 16,
// 8 independent accumulator chains) and one split of the 32-deep k chunks.  Each lane reads its
// fragments straight from global memory (L2): per chunk, 8 consecutive floats (two 16-byte
// loads) of each of its 2 A rows and 4 weight rows -- lane (r, g) holds k = 8 g + 4 h + t of row
// r in register h, element t, and MFMA (h, t) feeds k-slot g with it, for A and B alike, so the
// 8 MFMAs per block cover the chunk's 32 k.  NST chunks are in flight in a register ring.
// Split s runs on blockIdx % splits: with 8 splits, on XCD s (round-robin dispatch), so one
// XCD's L2 holds one K slice of x and w.  Fixed-order partials + k_fc_reduce, as k_fc_x9.
// Rows past M (the ragged actor batches) read row M - 1 and are not written.
constexpr int kFfTm = 64, kFfTn = 128, kFfThreads = 256;
template <int NST>
__global__ __launch_bounds__(kFfThreads) void k_fc_f32(const float *__restrict__ x, int64_t ldx, int M,
                                                       const float *__restrict__ w, int N, int K, int splits,
                                                       const float *__restrict__ bias, int relu,
                                                       float *__restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wave & 1, wn = wave >> 1;
  const int split = (int)blockIdx.x % splits, tile = (int)blockIdx.x / splits;
  const int tiles_n = N / kFfTn;
  const int m0 = (tile / tiles_n) * kFfTm + 32 * wm, n0 = (tile % tiles_n) * kFfTn + 64 * wn;
  const int chunks = K / 32;
  const int c0 = chunks * split / splits, c1 = chunks * (split + 1) / splits;
  // buffer loads: a per-lane row offset (voffset) and the chunk's byte offset as the uniform
  // soffset, so a chunk's 12 loads need no address arithmetic (the host checks both operands
  // are < 2^31 bytes)
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x), 0,
                                                                      (int)(((int64_t)(M - 1) * ldx + K) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(w), 0,
                                                                      (int)((int64_t)N * K * 4), 0x00020000);
  uint32_t xo[2], wo[4];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int row = m0 + 16 * mb + r;
    xo[mb] = (uint32_t)(((int64_t)(row < M ? row : M - 1) * ldx + 8 * g) * 4);
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) wo[nb] = (uint32_t)(((int64_t)(n0 + 16 * nb + r) * K + 8 * g) * 4);
  f32x4 xa[NST][2][2], wb[NST][4][2];
  auto ld = [](__amdgpu_buffer_rsrc_t rs, uint32_t vo, int so) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
  };
  auto load = [&](int c, f32x4 (&a)[2][2], f32x4 (&b)[4][2]) __attribute__((always_inline)) {
    const int so = c * 128;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int h = 0; h < 2; ++h) b[nb][h] = ld(ws, wo[nb] + 16 * h, so);
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int h = 0; h < 2; ++h) a[mb][h] = ld(xs, xo[mb] + 16 * h, so);
  };
  f32x4 acc[2][4];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const f32x4 (&a)[2][2], const f32x4 (&b)[4][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mb][h][t], b[nb][h][t], acc[mb][nb], 0, 0, 0);
  };
  // ring: before chunk c0 + i, set i % NST holds it and the next NST - 1 are in flight; past
  // c1 - 1 the loads repeat the range's last chunk (in bounds, unused)
#pragma unroll
  for (int s = 0; s < NST; ++s) load(c0 + s < c1 ? c0 + s : c1 - 1, xa[s], wb[s]);
  auto iter = [&](int c, auto is) __attribute__((always_inline)) {
    constexpr int s = decltype(is)::value;
    // the fence keeps each set's loads among its own MFMAs (left alone, the compiler moves
    // every MFMA of the unrolled ring ahead of every load and then waits for them in order; a
    // fence on both sides of the MFMAs makes it rotate the accumulators through copies)
    compute(xa[s], wb[s]);
    const int cn = c + NST < c1 ? c + NST : c1 - 1;
    load(cn, xa[s], wb[s]);
    __builtin_amdgcn_sched_barrier(0);
  };
  int c = c0;
  for (; c + NST <= c1; c += NST)
    static_for(std::make_integer_sequence<int, NST>{}, [&](auto is) __attribute__((always_inline)) {
      iter(c + decltype(is)::value, is);
    });
  static_for(std::make_integer_sequence<int, NST>{}, [&](auto is) __attribute__((always_inline)) {
    if (c + decltype(is)::value < c1) compute(xa[decltype(is)::value], wb[decltype(is)::value]);
  });
  // D: lane holds rows 4 g + i of each 16-row block, column r of each 16-column block
  float *dst = splits == 1 ? out : out + (int64_t)split * M * N;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 16 * mb + 4 * g + i;
      if (m < M) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          const int n = n0 + 16 * nb + r;
          float v = acc[mb][nb][i];
          if (splits == 1) {
            v = radd(v, bias ? bias[n] : 0.0f);
            v = relu ? fc_relu(v) : v;
          }
          dst[(int64_t)m * N + n] = v;
        }
      }
    }
}

// y = act(b + sum of the splits' partials, in split order), 4 outputs per thread.  Every partial
// is loaded before the first add (MAXS >= splits loads, unrolled; indices past splits - 1 repeat
// the last partial and are not added): the runtime-count loop waited for each load in turn, 16
// dependent round trips for 16 splits (9.6 / 12.1 us per launch in the loop, r05)
template <int MAXS>
__device__ __forceinline__ void fc_reduce_wg(int blk, const float *__restrict__ part, int splits, int64_t MN, int N,
                                             const float *__restrict__ bias, int relu, float *__restrict__ y,
                                             int64_t ldy) {
  const int64_t e4 = ((int64_t)blk * 256 + threadIdx.x) * 4;
  if (e4 >= MN) return;
  f32x4 v[MAXS];
#pragma unroll
  for (int k = 0; k < MAXS; ++k) v[k] = *reinterpret_cast<const f32x4 *>(part + (int64_t)(k < splits ? k : splits - 1) * MN + e4);
  f32x4 s = v[0];
#pragma unroll
  for (int k = 1; k < MAXS; ++k)
    if (k < splits) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] = radd(s[j], v[k][j]);
    }
  const int64_t m = e4 / N;
  const int n = (int)(e4 - m * N);
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float t = radd(s[j], bias ? bias[n + j] : 0.0f);
    o[j] = relu ? fc_relu(t) : t;
  }
  *reinterpret_cast<f32x4 *>(y + m * ldy + n) = o;
}

template <int MAXS>
__global__ __launch_bounds__(256) void k_fc_reduce(const float *__restrict__ part, int splits, int64_t MN, int N,
                                                   const float *__restrict__ bias, int relu, float *__restrict__ y,
                                                   int64_t ldy) {
  fc_reduce_wg<MAXS>((int)blockIdx.x, part, splits, MN, N, bias, relu, y, ldy);
}

// r06: FC1's split-K reduce (+ bias + ReLU, in k_fc_reduce's order) and FC2 of both dueling
// branches (k_heads_fc2_lean's lanes, terms and order: bit-identical heads) in one launch -- the
// target pass's and the learner's FC1 -> FC2 without the h1 round trip through a second launch.
// Workgroup = kRhRows rows: phase 1, every lane reduces float4 groups of the rows' h1 (all of its
// split loads in flight) into LDS (and h1_out, nullable: the learner's backward reads h1);
// phase 2, 16 lanes per row run FC2 from LDS.  N = 2H <= kRhMaxN.
constexpr int kRhRows = 4, kRhMaxN = 512;
template <int MAXS, int MAXA1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 3))) void k_fc_reduce_heads(const float *__restrict__ part, int splits, int M, int N,
                                                         const float *__restrict__ b1, int A,
                                                         const float *__restrict__ wa2, const float *__restrict__ wv2,
                                                         const float *__restrict__ ba2, const float *__restrict__ bv2,
                                                         float *__restrict__ heads, float *__restrict__ h1_out) {
  __shared__ f32x4 hs[kRhRows * kRhMaxN / 4];
  const int r0 = (int)blockIdx.x * kRhRows, N4 = N / 4;
  const int64_t MN = (int64_t)M * N;
  constexpr int PER = kRhRows * kRhMaxN / 4 / 256;  // float4 groups per lane (at N = kRhMaxN)
  f32x4 v[PER][MAXS];
  // buffer loads: the lane's element as voffset, the split as the uniform soffset -- no address
  // registers per load, so all PER x MAXS loads stay in flight together (the host keeps the
  // partials under 2^31 bytes)
  const __amdgpu_buffer_rsrc_t pr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(part), 0, (int)(splits * MN * 4), 0x00020000);
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = (int)threadIdx.x + 256 * u, rr = i / N4;
    const int row = r0 + rr < M ? r0 + rr : M - 1;  // tail rows: a duplicate, not written
    const uint32_t off = (uint32_t)(((int64_t)row * N + 4 * (i - rr * N4)) * 4);
#pragma unroll
    for (int k = 0; k < MAXS; ++k)
      v[u][k] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, off, (int)((k < splits ? k : splits - 1) * MN * 4), 0));
  }
  __builtin_amdgcn_sched_barrier(0);  // every split load in flight before the first add
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = (int)threadIdx.x + 256 * u, rr = i / N4, c = 4 * (i - rr * N4);
    if (i >= kRhRows * N4) break;
    f32x4 sum = v[u][0];
#pragma unroll
    for (int k = 1; k < MAXS; ++k)
      if (k < splits) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sum[j] = radd(sum[j], v[u][k][j]);
      }
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fc_relu(radd(sum[j], b1[c + j]));
    hs[i] = o;
    if (h1_out && r0 + rr < M) *reinterpret_cast<f32x4 *>(h1_out + (int64_t)(r0 + rr) * N + c) = o;
  }
  __syncthreads();
  if (threadIdx.x >= 16 * kRhRows) return;  // (whole waves past the first)
  const int l = threadIdx.x & 15, rr = threadIdx.x >> 4;
  const int H = N / 2, cq = H / 64, A1 = A + 1;
  const f32x4 *ha = hs + rr * N4 + l * cq, *hv = hs + rr * N4 + H / 4 + l * cq;
  float acc[MAXA1];
#pragma unroll
  for (int a = 0; a < MAXA1; ++a) acc[a] = 0.0f;
#pragma unroll 1
  for (int k = 0; k < cq; ++k) {
    const f32x4 xa = ha[k], xv = hv[k];
    float4 w[MAXA1];
#pragma unroll
    for (int a = 0; a < MAXA1; ++a) {
      const int ac = a < A1 ? a : A;  // past A: a duplicate row, unused
      w[a] = reinterpret_cast<const float4 *>(ac < A ? wa2 + (int64_t)ac * H : wv2)[l * cq + k];
    }
#pragma unroll
    for (int a = 0; a < MAXA1; ++a)
      if (a < A1) {
        const f32x4 x = a < A ? xa : xv;
        const float4 ww = w[a];
        acc[a] = radd(radd(radd(radd(acc[a], rmul(x[0], ww.x)), rmul(x[1], ww.y)), rmul(x[2], ww.z)), rmul(x[3], ww.w));
      }
  }
#pragma unroll
  for (int a = 0; a < MAXA1; ++a)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc[a] = radd(acc[a], __shfl_xor(acc[a], o, 64));
  if (l == 0 && r0 + rr < M) {
    float *out = heads + (int64_t)(r0 + rr) * A1;
#pragma unroll
    for (int a = 0; a < MAXA1; ++a)
      if (a <= A) out[a] = radd(acc[a], a < A ? ba2[a] : bv2[0]);
  }
}

// r05: k_fc_reduce's workgroups (blocks [0, nred)) + the device-counted tail rows behind the M
// fixed rows (k_linear_relu_rows' workgroups, blocks [nred, ...)) in one launch -- the actors'
// counted FC1 (their terminal stacks: none in most steps) without a launch of its own
static_assert(kLrThreads == 256, "k_fc_reduce_rows runs k_linear_relu_rows' workgroups at 256 lanes");
template <int MAXS>
__global__ __launch_bounds__(256) void k_fc_reduce_rows(const float *__restrict__ part, int splits, int64_t MN, int N,
                                                        const float *__restrict__ bias, float *__restrict__ y,
                                                        int64_t ldy, int nred, const float *__restrict__ x,
                                                        int64_t ldx, int64_t r0, int64_t n_max,
                                                        const int64_t *__restrict__ n_dev,
                                                        const float *__restrict__ w, int K) {
  if ((int)blockIdx.x < nred)
    fc_reduce_wg<MAXS>((int)blockIdx.x, part, splits, MN, N, bias, 1, y, ldy);
  else
    linear_relu_rows_wg((int)blockIdx.x - nred, x, ldx, r0, n_max, n_dev, w, bias, K, N, y, ldy);
}

// the reduce launch of `splits` partials: the smallest unrolled instance that holds them
static const void *fc_reduce_fn(int splits, bool rows) {
  if (rows)
    return splits <= 4    ? reinterpret_cast<const void *>(&k_fc_reduce_rows<4>)
           : splits <= 8  ? reinterpret_cast<const void *>(&k_fc_reduce_rows<8>)
           : splits <= 16 ? reinterpret_cast<const void *>(&k_fc_reduce_rows<16>)
                          : reinterpret_cast<const void *>(&k_fc_reduce_rows<32>);
  return splits <= 4    ? reinterpret_cast<const void *>(&k_fc_reduce<4>)
         : splits <= 8  ? reinterpret_cast<const void *>(&k_fc_reduce<8>)
         : splits <= 16 ? reinterpret_cast<const void *>(&k_fc_reduce<16>)
                        : reinterpret_cast<const void *>(&k_fc_reduce<32>);
}
static int launch_fc_reduce(const float *part, int splits, int64_t MN, int N, const float *bias, int relu, float *y,
                            int64_t ldy, hipStream_t s) {
  RTH_REQUIRE(splits >= 1 && splits <= 32, "fc reduce: %d splits", splits);
  void *args[] = {&part, &splits, &MN, &N, &bias, &relu, &y, &ldy};
  RTH_HIP(hipLaunchKernel(fc_reduce_fn(splits, false), dim3((unsigned)((MN / 4 + 255) / 256)), dim3(256), args, 0, s));
  return RTH_OK;
}

// k splits of the 64 x 128 tile: about one workgroup per CU (256) over the output tiles, at
// most 32 and at most the chunk count
static int fc_splits(int M, int N, int K) {
  const int tiles = (M / kFcTm) * (N / kFcTn), chunks = K / 32;
  int s = (256 + tiles - 1) / tiles;
  s = s < 1 ? 1 : (s > 32 ? 32 : s);
  return s < chunks ? s : chunks;
}

// which x9 form runs a shape: the 128 x 128 tile (k_fc_x9t) where M and N are multiples of 128,
// else the 64 x 128 k_fc_x9.  Alone (scripts/bench_fc.py, r05) the 128 tile is faster from 1,024
// rows (37.5 vs 44.1 us; 2,048: 54 vs 72) and slower below (512: 30.6 vs 28.9; 256: 24.6 vs
// 21.8), but in the loop it is the better one at 512 / 256 rows too: 0.521-0.525 vs 0.531-0.533
// ms/step (profiles/r05/ab_log.txt) -- one 96 KB workgroup per CU, a single round of at most 256
// workgroups, where the 64 x 128 form's 256 workgroups of 48 KB share CUs with the other
// stream's kernels.  k splits: about one workgroup per CU, at most 16 (at 512 rows 256
// workgroups; 24 / 32 splits -- two rounds of workgroups -- 0.533-0.539, 8 splits 0.531-0.534),
// never more than the chunk count.  r06: a three-deep LDS ring with the MFMA fragments read one
// chunk ahead (k_fc_x9p, 144 KB per workgroup) was bit-identical and no faster alone (40.4 vs
// 39.3 us at 1,024 rows) and slower in the loop (0.529 vs 0.520 ms/step): removed.
struct FcPlan {
  int big, splits;
};
constexpr int kFcMaxSplits = 16;
static FcPlan fc_plan(int M, int N, int K) {
  if (M % kFbTile || N % kFbTile) return FcPlan{0, fc_splits(M, N, K)};
  const int tiles = (M / kFbTile) * (N / kFbTile), chunks = K / 32;
  int s = (256 + tiles - 1) / tiles;
  s = s > kFcMaxSplits ? kFcMaxSplits : (s < 1 ? 1 : s);
  return FcPlan{1, s < chunks ? s : chunks};
}

// one x9 GEMM launch by plan p into out (y when p.splits == 1, else the partials)
static void fc_x9_launch(const FcPlan &p, const float *x, int64_t ldx, int M, const float *w, int N, int K,
                         const float *bias, int relu, float *out, hipStream_t s) {
  if (!p.big) {  // two chunks of loads in flight (r04: ahead of one)
    const int tiles = (M / kFcTm) * (N / kFcTn);
    hipLaunchKernelGGL(k_fc_x9<2>, dim3((unsigned)(tiles * p.splits)), dim3(kFcThreads), 0, s, x, ldx, M, w, N, K,
                       p.splits, bias, relu, out);
    return;
  }
  const dim3 grid((unsigned)((M / kFbTile) * (N / kFbTile) * p.splits));
  hipLaunchKernelGGL((k_fc_x9t<8, 1>), grid, dim3(512), 0, s, x, ldx, M, w, N, K, p.splits, bias, relu, out);
}

// k_fc_f32's k splits: 8 (one K slice per XCD) while that gives at most 512 workgroups, else
// fewer; never more than the chunk count
static int fcf_splits(int M, int N, int K) {
  const int tiles = ((M + kFfTm - 1) / kFfTm) * (N / kFfTn), chunks = K / 32;
  int s = 8;
  while (s > 1 && tiles * s > 512) s /= 2;
  return s < chunks ? s : chunks;
}

}  // namespace rth

using namespace rth;

extern "C" {

int rth_fc_x9_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && M % kFcTm == 0 && N > 0 && N % kFcTn == 0 && K >= 32 && K % 32 == 0 && M * K < (1ll << 31) &&
                 N * K < (1ll << 31)
             ? 1
             : 0;
}

int64_t rth_fc_x9_workspace(int64_t M, int64_t N, int64_t K) {
  if (!rth_fc_x9_supported(M, N, K)) return 0;
  const int s = fc_plan((int)M, (int)N, (int)K).splits;
  return s > 1 ? (int64_t)s * M * N * 4 : 0;
}

int rth_fc_x9(const float *x, int64_t ldx, int64_t M, const float *w, int64_t N, int64_t K, const float *bias,
              int32_t relu, float *y, void *workspace, void *stream) {
  RTH_REQUIRE(x && w && y, "rth_fc_x9: NULL argument");
  RTH_REQUIRE(rth_fc_x9_supported(M, N, K), "rth_fc_x9: shape %lld x %lld x %lld not built (M %% 64, N %% 128, K %% 32)",
              (long long)M, (long long)N, (long long)K);
  RTH_REQUIRE(ldx >= K && ldx % 4 == 0, "rth_fc_x9: row stride %lld", (long long)ldx);
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) &
               15) == 0,
              "rth_fc_x9: misaligned buffer");
  const FcPlan p = fc_plan((int)M, (int)N, (int)K);
  const int splits = p.splits;
  RTH_REQUIRE(splits == 1 || (workspace && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0),
              "rth_fc_x9: %d splits need the workspace (rth_fc_x9_workspace)", splits);
  hipStream_t s = as_stream(stream);
  float *out = splits == 1 ? y : static_cast<float *>(workspace);
  fc_x9_launch(p, x, ldx, (int)M, w, (int)N, (int)K, bias, (int)relu, out, s);
  RTH_LAUNCHED();
  if (splits > 1) {
    const int64_t MN = M * N;
    const int rc = launch_fc_reduce(static_cast<const float *>(workspace), splits, MN, (int)N, bias, (int)relu, y, N, s);
    if (rc) return rc;
  }
  return RTH_OK;
}

int rth_fc_x9_rows_upto(const float *x, int64_t ldx, int64_t M, int64_t n_max, const int64_t *n_dev, const float *w,
                        int64_t N, int64_t K, const float *bias, float *y, void *workspace, void *stream) {
  RTH_REQUIRE(x && w && y && bias && n_dev, "rth_fc_x9_rows_upto: NULL argument");
  RTH_REQUIRE(rth_fc_x9_supported(M, N, K) && n_max >= M,
              "rth_fc_x9_rows_upto: shape %lld (+ %lld counted) x %lld x %lld not built (M %% 64, N %% 128, K %% 32)",
              (long long)M, (long long)(n_max - M), (long long)N, (long long)K);
  RTH_REQUIRE(ldx >= K && ldx % 4 == 0 &&
                  ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) &
                   15) == 0,
              "rth_fc_x9_rows_upto: row stride %lld or misaligned buffer", (long long)ldx);
  const FcPlan p = fc_plan((int)M, (int)N, (int)K);
  const int splits = p.splits;
  if (splits == 1) {  // no reduce launch to share: the two launches
    int rc = rth_fc_x9(x, ldx, M, w, N, K, bias, 1, y, workspace, stream);
    return rc ? rc : rth_linear_relu_rows_upto(x, ldx, M, n_max, n_dev, w, bias, K, N, y, N, stream);
  }
  RTH_REQUIRE(workspace && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
              "rth_fc_x9_rows_upto: %d splits need the workspace (rth_fc_x9_workspace)", splits);
  hipStream_t s = as_stream(stream);
  float *part = static_cast<float *>(workspace);
  fc_x9_launch(p, x, ldx, (int)M, w, (int)N, (int)K, bias, 1, part, s);
  RTH_LAUNCHED();
  const int64_t MN = M * N;
  const int nred = (int)((MN / 4 + 255) / 256), nrows = n_max > M ? (int)((N + kLrCols - 1) / kLrCols) : 0;
  RTH_REQUIRE(splits <= 32, "rth_fc_x9_rows_upto: %d splits", splits);
  {
    const float *cpart = part;
    int Ni = (int)N, Ki = (int)K;
    int64_t ldy = N, r0 = M;
    void *args[] = {&cpart, const_cast<int *>(&splits), const_cast<int64_t *>(&MN), &Ni, &bias, &y, &ldy,
                    const_cast<int *>(&nred), &x, &ldx, &r0, &n_max, &n_dev, &w, &Ki};
    RTH_HIP(hipLaunchKernel(fc_reduce_fn(splits, true), dim3((unsigned)(nred + nrows)), dim3(256), args, 0, s));
  }
  return RTH_OK;
}

int rth_fc1_heads_supported(int64_t M, int64_t N, int64_t K, int32_t A) {
  if (!rth_fc_x9_supported(M, N, K) || N > kRhMaxN || N % 128 || A < 1 || A + 1 > 8) return 0;
  const int s = fc_plan((int)M, (int)N, (int)K).splits;
  return s >= 2 && s <= 16 ? 1 : 0;
}

int rth_fc1_heads(const float *x, int64_t ldx, int64_t M, const float *w1, int64_t N, int64_t K, const float *b1,
                  int32_t A, const float *const *fc2_params, float *heads, float *h1_out, void *workspace,
                  void *stream) {
  RTH_REQUIRE(x && w1 && b1 && fc2_params && heads && workspace, "rth_fc1_heads: NULL argument");
  RTH_REQUIRE(rth_fc1_heads_supported(M, N, K, A), "rth_fc1_heads: shape %lld x %lld x %lld, A %d not built",
              (long long)M, (long long)N, (long long)K, A);
  RTH_REQUIRE((int64_t)fc_plan((int)M, (int)N, (int)K).splits * M * N * 4 < ((int64_t)1 << 31),
              "rth_fc1_heads: split-K partials past 2 GiB");
  for (int i = 0; i < 4; ++i) RTH_REQUIRE(fc2_params[i], "rth_fc1_heads: NULL FC2 parameter %d", i);
  RTH_REQUIRE(ldx >= K && ldx % 4 == 0 &&
                  ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w1) |
                    reinterpret_cast<uintptr_t>(workspace) | reinterpret_cast<uintptr_t>(h1_out)) &
                   15) == 0,
              "rth_fc1_heads: row stride %lld or misaligned buffer", (long long)ldx);
  const FcPlan p = fc_plan((int)M, (int)N, (int)K);
  hipStream_t s = as_stream(stream);
  float *part = static_cast<float *>(workspace);
  fc_x9_launch(p, x, ldx, (int)M, w1, (int)N, (int)K, b1, 1, part, s);
  RTH_LAUNCHED();
  const dim3 grid((unsigned)((M + kRhRows - 1) / kRhRows));
  if (p.splits <= 8)
    hipLaunchKernelGGL((k_fc_reduce_heads<8, 8>), grid, dim3(256), 0, s, part, p.splits, (int)M, (int)N, b1, (int)A,
                       fc2_params[0], fc2_params[1], fc2_params[2], fc2_params[3], heads, h1_out);
  else
    hipLaunchKernelGGL((k_fc_reduce_heads<16, 8>), grid, dim3(256), 0, s, part, p.splits, (int)M, (int)N, b1, (int)A,
                       fc2_params[0], fc2_params[1], fc2_params[2], fc2_params[3], heads, h1_out);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_fc_f32_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && N % kFfTn == 0 && K >= 32 && K % 32 == 0 && M * K < (1ll << 31) && N * K < (1ll << 31) &&
                 M * N * 32 < (1ll << 31)
             ? 1
             : 0;
}

int64_t rth_fc_f32_workspace(int64_t M, int64_t N, int64_t K) {
  if (!rth_fc_f32_supported(M, N, K)) return 0;
  const int s = fcf_splits((int)M, (int)N, (int)K);
  return s > 1 ? (int64_t)s * M * N * 4 : 0;
}

int rth_fc_f32(const float *x, int64_t ldx, int64_t M, const float *w, int64_t N, int64_t K, const float *bias,
               int32_t relu, float *y, void *workspace, void *stream) {
  RTH_REQUIRE(x && w && y, "rth_fc_f32: NULL argument");
  RTH_REQUIRE(rth_fc_f32_supported(M, N, K), "rth_fc_f32: shape %lld x %lld x %lld not built (N %% 128, K %% 32)",
              (long long)M, (long long)N, (long long)K);
  RTH_REQUIRE(ldx >= K && ldx % 4 == 0 && ((M - 1) * ldx + K) * 4 < (1ll << 31), "rth_fc_f32: row stride %lld",
              (long long)ldx);
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) &
               15) == 0,
              "rth_fc_f32: misaligned buffer");
  const int splits = fcf_splits((int)M, (int)N, (int)K);
  RTH_REQUIRE(splits == 1 || (workspace && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0),
              "rth_fc_f32: %d splits need the workspace (rth_fc_f32_workspace)", splits);
  hipStream_t s = as_stream(stream);
  const int tiles = (int)((M + kFfTm - 1) / kFfTm) * (int)(N / kFfTn);
  float *out = splits == 1 ? y : static_cast<float *>(workspace);
  const void *fn = reinterpret_cast<const void *>(&k_fc_f32<3>);  // 3 chunks in flight (2 / 4: equal or slower, r05)
  int Mi = (int)M, Ni = (int)N, Ki = (int)K, re = (int)relu;
  void *args[] = {&x, &ldx, &Mi, &w, &Ni, &Ki, const_cast<int *>(&splits), &bias, &re, &out};
  RTH_HIP(hipLaunchKernel(fn, dim3((unsigned)(tiles * splits)), dim3(kFfThreads), args, 0, s));
  if (splits > 1) {
    const int64_t MN = M * N;
    const int rc = launch_fc_reduce(static_cast<const float *>(workspace), splits, MN, (int)N, bias, (int)relu, y, N, s);
    if (rc) return rc;
  }
  return RTH_OK;
}

}  // extern "C"
