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

// y = act(b + sum of the splits' partials, in split order), 4 outputs per thread
__device__ __forceinline__ void fc_reduce_wg(int blk, const float *__restrict__ part, int splits, int64_t MN, int N,
                                             const float *__restrict__ bias, int relu, float *__restrict__ y,
                                             int64_t ldy) {
  const int64_t e4 = ((int64_t)blk * 256 + threadIdx.x) * 4;
  if (e4 >= MN) return;
  f32x4 s = *reinterpret_cast<const f32x4 *>(part + e4);
  for (int k = 1; k < splits; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4 *>(part + (int64_t)k * MN + e4);
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = radd(s[j], v[j]);
  }
  const int64_t m = e4 / N;
  const int n = (int)(e4 - m * N);
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float v = radd(s[j], bias ? bias[n + j] : 0.0f);
    o[j] = relu ? fc_relu(v) : v;
  }
  *reinterpret_cast<f32x4 *>(y + m * ldy + n) = o;
}

__global__ __launch_bounds__(256) void k_fc_reduce(const float *__restrict__ part, int splits, int64_t MN, int N,
                                                   const float *__restrict__ bias, int relu, float *__restrict__ y,
                                                   int64_t ldy) {
  fc_reduce_wg((int)blockIdx.x, part, splits, MN, N, bias, relu, y, ldy);
}

// r05: k_fc_reduce's workgroups (blocks [0, nred)) + the device-counted tail rows behind the M
// fixed rows (k_linear_relu_rows' workgroups, blocks [nred, ...)) in one launch -- the actors'
// counted FC1 (their terminal stacks: none in most steps) without a launch of its own
static_assert(kLrThreads == 256, "k_fc_reduce_rows runs k_linear_relu_rows' workgroups at 256 lanes");
__global__ __launch_bounds__(256) void k_fc_reduce_rows(const float *__restrict__ part, int splits, int64_t MN, int N,
                                                        const float *__restrict__ bias, float *__restrict__ y,
                                                        int64_t ldy, int nred, const float *__restrict__ x,
                                                        int64_t ldx, int64_t r0, int64_t n_max,
                                                        const int64_t *__restrict__ n_dev,
                                                        const float *__restrict__ w, int K) {
  if ((int)blockIdx.x < nred)
    fc_reduce_wg((int)blockIdx.x, part, splits, MN, N, bias, 1, y, ldy);
  else
    linear_relu_rows_wg((int)blockIdx.x - nred, x, ldx, r0, n_max, n_dev, w, bias, K, N, y, ldy);
}

// k splits: about one workgroup per CU (256) over the output tiles, at most 16 and at most the
// chunk count; RTH_FC_SPLITS overrides (A/B)
static int fc_splits(int M, int N, int K) {
  static const int env = [] {
    const char *e = getenv("RTH_FC_SPLITS");
    return e ? atoi(e) : 0;
  }();
  const int tiles = (M / kFcTm) * (N / kFcTn), chunks = K / 32;
  int s = env > 0 ? env : (256 + tiles - 1) / tiles;
  s = s < 1 ? 1 : (s > 32 ? 32 : s);
  return s < chunks ? s : chunks;
}

// k_fc_f32's k splits: 8 (one K slice per XCD) while that gives at most 512 workgroups, else
// fewer; RTH_FCF_SPLITS overrides (A/B); never more than the chunk count
static int fcf_splits(int M, int N, int K) {
  static const int env = [] {
    const char *e = getenv("RTH_FCF_SPLITS");
    return e ? atoi(e) : 0;
  }();
  const int tiles = ((M + kFfTm - 1) / kFfTm) * (N / kFfTn), chunks = K / 32;
  int s = env > 0 ? env : 8;
  if (env <= 0)
    while (s > 1 && tiles * s > 512) s /= 2;
  s = s < 1 ? 1 : (s > 32 ? 32 : s);
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
  const int s = fc_splits((int)M, (int)N, (int)K);
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
  const int splits = fc_splits((int)M, (int)N, (int)K);
  RTH_REQUIRE(splits == 1 || (workspace && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0),
              "rth_fc_x9: %d splits need the workspace (rth_fc_x9_workspace)", splits);
  hipStream_t s = as_stream(stream);
  const int tiles = (int)(M / kFcTm) * (int)(N / kFcTn);
  float *out = splits == 1 ? y : static_cast<float *>(workspace);
  static const int pf = [] {  // RTH_FC_PF: chunks of loads in flight (1 or 2)
    const char *e = getenv("RTH_FC_PF");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  if (pf == 1)
    hipLaunchKernelGGL(k_fc_x9<1>, dim3((unsigned)(tiles * splits)), dim3(kFcThreads), 0, s, x, ldx, (int)M, w,
                       (int)N, (int)K, splits, bias, (int)relu, out);
  else
    hipLaunchKernelGGL(k_fc_x9<2>, dim3((unsigned)(tiles * splits)), dim3(kFcThreads), 0, s, x, ldx, (int)M, w,
                       (int)N, (int)K, splits, bias, (int)relu, out);
  RTH_LAUNCHED();
  if (splits > 1) {
    const int64_t MN = M * N;
    hipLaunchKernelGGL(k_fc_reduce, dim3((unsigned)((MN / 4 + 255) / 256)), dim3(256), 0, s,
                       static_cast<const float *>(workspace), splits, MN, (int)N, bias, (int)relu, y, N);
    RTH_LAUNCHED();
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
  const int splits = fc_splits((int)M, (int)N, (int)K);
  if (splits == 1) {  // no reduce launch to share: the two launches
    int rc = rth_fc_x9(x, ldx, M, w, N, K, bias, 1, y, workspace, stream);
    return rc ? rc : rth_linear_relu_rows_upto(x, ldx, M, n_max, n_dev, w, bias, K, N, y, N, stream);
  }
  RTH_REQUIRE(workspace && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
              "rth_fc_x9_rows_upto: %d splits need the workspace (rth_fc_x9_workspace)", splits);
  hipStream_t s = as_stream(stream);
  const int tiles = (int)(M / kFcTm) * (int)(N / kFcTn);
  float *part = static_cast<float *>(workspace);
  hipLaunchKernelGGL(k_fc_x9<2>, dim3((unsigned)(tiles * splits)), dim3(kFcThreads), 0, s, x, ldx, (int)M, w,
                     (int)N, (int)K, splits, bias, 1, part);
  RTH_LAUNCHED();
  const int64_t MN = M * N;
  const int nred = (int)((MN / 4 + 255) / 256), nrows = n_max > M ? (int)((N + kLrCols - 1) / kLrCols) : 0;
  hipLaunchKernelGGL(k_fc_reduce_rows, dim3((unsigned)(nred + nrows)), dim3(256), 0, s, part, splits, MN, (int)N,
                     bias, y, (int64_t)N, nred, x, ldx, M, n_max, n_dev, w, (int)K);
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
  static const int nst = [] {  // RTH_FCF_NST: chunks in flight (2, 3 or 4)
    const char *e = getenv("RTH_FCF_NST");
    const int v = e ? atoi(e) : 3;
    return v == 2 || v == 4 ? v : 3;
  }();
  const void *fn = nst == 2   ? reinterpret_cast<const void *>(&k_fc_f32<2>)
                   : nst == 4 ? reinterpret_cast<const void *>(&k_fc_f32<4>)
                              : reinterpret_cast<const void *>(&k_fc_f32<3>);
  int Mi = (int)M, Ni = (int)N, Ki = (int)K, re = (int)relu;
  void *args[] = {&x, &ldx, &Mi, &w, &Ni, &Ki, const_cast<int *>(&splits), &bias, &re, &out};
  RTH_HIP(hipLaunchKernel(fn, dim3((unsigned)(tiles * splits)), dim3(kFfThreads), args, 0, s));
  if (splits > 1) {
    const int64_t MN = M * N;
    hipLaunchKernelGGL(k_fc_reduce, dim3((unsigned)((MN / 4 + 255) / 256)), dim3(256), 0, s,
                       static_cast<const float *>(workspace), splits, MN, (int)N, bias, (int)relu, y, N);
    RTH_LAUNCHED();
  }
  return RTH_OK;
}

}  // extern "C"
