// Weight gradient of conv2 / conv3 of the Nature-DQN torso on the fp32 MFMA, deterministic
// and without a zero fill (replaces MIOpen's igemm_wrw and its fill).  Reference: the
// backward of reth/reth/algorithm/dqn/dqn_model.py:14-20 under dqn_solver.py:117
// (loss.backward()).
//
//   gw[co][kh][kw][ci] = sum over output pixels p = (b, oy, ox) of
//                        gy[p][co] * x[b][S*oy + kh][S*ox + kw][ci]
//
// x (the layer's input) and gy (the masked upstream gradient) are channels-last fp32; gw is
// the OHWI (channels_last) weight gradient.  GEMM view: rows = co (COUT), columns = kk =
// (kh, kw, ci) in OHWI order (K = KH*KW*CIN), reduction over the pixels.
//
// v_mfma_f32_32x32x2f32: lane (i = lane & 31, h = lane >> 5) supplies A[i][h] = gy[p + h][co]
// and B[h][i] = x-window[p + h][kk] -- both 32 consecutive channels of one NHWC pixel, one
// 128-byte segment per half-wave -- so a wave consumes a pair of pixels per MFMA.  A wave
// holds all COUT = 64 rows (2 blocks) x NB column blocks of 32 (NB*32 consecutive kk, one
// (kh, kw) run of the window when CIN is a multiple of 32) as 2*NB accumulators, and walks
// its pixel range with kPf pairs of loads in flight.  The kWaves waves of a workgroup take
// consecutive pixel sub-ranges of the same column group; their partials are summed in LDS
// in wave order, and the workgroup's partial goes to the workspace; k_wgrad_f32_reduce adds
// the partials of a column group in workgroup order.  Every sum has a fixed order.
#include "common.hpp"

namespace rth {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kWgfWaves = 4;  // waves per workgroup (one per SIMD)
#ifndef WGF_PF
#define WGF_PF 4
#endif
constexpr int kWgfPf = WGF_PF;  // pixel pairs whose loads are in flight ahead of their MFMAs

template <int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN>
struct WgfGeom {
  static constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int K = KH * KW * CIN;
  static_assert(COUT == 64 && CIN % 32 == 0, "64 output channels, input channels in runs of 32");
};

// kk-block kb (32 consecutive kk) -> offset of its first element inside the input window
template <int KW, int CIN, int WIN>
__device__ __forceinline__ int kb_off(int kb) {
  const int kk = kb * 32, khkw = kk / CIN, ci = kk % CIN;
  return ((khkw / KW) * WIN + khkw % KW) * CIN + ci;
}

template <int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN, int NB>
__global__ __launch_bounds__(kWgfWaves * 64) void k_conv_wgrad_f32(const float *__restrict__ x,
                                                                 const float *__restrict__ gy, int64_t n,
                                                                 int splits, float *__restrict__ part) {
  using Gm = WgfGeom<KH, KW, S, CIN, COUT, HIN, WIN>;
  __shared__ float red[2 * NB * 16 * 64];  // one wave's accumulators (lane-major per register)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
  const int group = blockIdx.x / splits, split = blockIdx.x % splits;
  const int64_t P = n * Gm::PIX;
  // this wave's pixel range: split-major, then wave; pair-aligned
  const int64_t units = (int64_t)splits * kWgfWaves, u = (int64_t)split * kWgfWaves + wave;
  const int64_t pairs = (P + 1) / 2;
  const int64_t q0 = pairs * u / units, q1 = pairs * (u + 1) / units;
  int koff[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) koff[nb] = kb_off<KW, CIN, WIN>(group * NB + nb) + i;

  f32x16 acc[2][NB];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][nb][r] = 0.0f;

  // operands of the pairs in launch order from a cursor at pixel 2q + h: (b, oy, ox) advance by
  // two pixels per pair with adds only; a pixel past the range reads the range's last pixel
  // with weight 0
  const int64_t plast = (2 * q1 - 1 < P ? 2 * q1 - 1 : P - 1);  // the range's last live pixel
  const int64_t lb = plast / Gm::PIX;
  const int lpix = (int)(plast - lb * Gm::PIX), loy = lpix / Gm::WOUT, lox = lpix - loy * Gm::WOUT;
  int64_t cp = 2 * q0 + h;
  int64_t cb = cp / Gm::PIX;
  int cpix = (int)(cp - cb * Gm::PIX), coy = cpix / Gm::WOUT, cox = cpix - coy * Gm::WOUT;
  // branch-free: a dead pixel reads the range's last pixel and is weighted 0 (0 * x = 0 for
  // finite x), so pairs past q1 may be multiplied in as well
  auto load = [&](float (&a)[2], float (&b)[NB], bool &lv) {
    const bool live = cp <= plast;
    lv = live;
    const int64_t p = live ? cp : plast, bb = live ? cb : lb;
    const int oy = live ? coy : loy, ox = live ? cox : lox;
    const float *g = gy + p * COUT + i;
    a[0] = g[0];  // weighted 0 at the MFMA when dead (no wait on the load here)
    a[1] = g[32];
    const float *xw = x + ((bb * HIN + S * oy) * WIN + S * ox) * CIN;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) b[nb] = xw[koff[nb]];
    // advance the cursor by one pair (two pixels)
    cp += 2;
    cox += 2;
    const bool wrap = cox >= Gm::WOUT;
    cox = wrap ? cox - Gm::WOUT : cox;
    coy += wrap ? 1 : 0;
    const bool wrap2 = coy == Gm::HOUT;
    coy = wrap2 ? 0 : coy;
    cb += wrap2 ? 1 : 0;
  };
  float av[kWgfPf][2], bv[kWgfPf][NB];
  bool lv[kWgfPf];
#pragma unroll
  for (int d = 0; d < kWgfPf; ++d) load(av[d], bv[d], lv[d]);
#pragma unroll 1
  for (int64_t q = q0; q < q1; q += kWgfPf) {
#pragma unroll
    for (int d = 0; d < kWgfPf; ++d) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float a = lv[d] ? av[d][c] : 0.0f;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[c][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv[d][nb], acc[c][nb], 0, 0, 0);
      }
      // keep the refill of slot d here: the scheduler would otherwise sink these loads down
      // to their use kWgfPf pairs later and expose their latency
      __builtin_amdgcn_sched_barrier(0);
      load(av[d], bv[d], lv[d]);  // the pair kWgfPf ahead (past q1: zero-weighted)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the workgroup's waves in order: wave 0 stores, waves 1..3 add, the last one writes out
  for (int w = 0; w < kWgfWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float &slot = red[((c * NB + nb) * 16 + r) * 64 + lane];
            slot = w == 0 ? acc[c][nb][r] : radd(slot, acc[c][nb][r]);
          }
    }
    __syncthreads();
  }
  // partial [split][COUT][K]: D[row][col] of block (c, nb) -> co = 32c + row, kk = (group*NB + nb)*32 + col;
  // row = (r / 4) * 8 + h' * 4 + r % 4 for the lane (col = l & 31, h' = l >> 5) that held it
  float *out = part + (int64_t)split * COUT * Gm::K;
  for (int e = threadIdx.x; e < 2 * NB * 16 * 64; e += kWgfWaves * 64) {
    const int l = e & 63, r = (e >> 6) & 15, blk = e >> 10, c = blk / NB, nb = blk % NB;
    const int row = (r >> 2) * 8 + (l >> 5) * 4 + (r & 3), col = l & 31;
    out[(int64_t)(32 * c + row) * Gm::K + (group * NB + nb) * 32 + col] = red[e];
  }
}

// gw[e] = sum of the splits' partials (e over COUT * K) in a fixed order: a workgroup takes 64
// consecutive elements; thread (g, e) sums the splits g, g + 4, g + 8, ... of element e with
// all of its loads in flight together, then the 4 group sums are added in group order
constexpr int kWgfRedMax = 64;  // splits per element at most: 16 per thread
__global__ __launch_bounds__(256) void k_conv_wgrad_f32_reduce(const float *__restrict__ part, int splits,
                                                              int64_t elems, float *__restrict__ gw) {
  __shared__ float red[4][64];
  const int el = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + el;
  float v[kWgfRedMax / 4];
#pragma unroll
  for (int u = 0; u < kWgfRedMax / 4; ++u) {
    const int k = grp + 4 * u;
    v[u] = (k < splits && e < elems) ? part[(int64_t)k * elems + e] : 0.0f;
  }
  float s = 0.0f;
#pragma unroll
  for (int u = 0; u < kWgfRedMax / 4; ++u)
    if (grp + 4 * u < splits) s = radd(s, v[u]);
  red[grp][el] = s;
  __syncthreads();
  if (grp == 0 && e < elems) gw[e] = radd(radd(radd(red[0][el], red[1][el]), red[2][el]), red[3][el]);
}

struct WgfLaunch {
  const void *fn;
  int groups;  // column groups (K / (NB * 32))
  int64_t elems;  // COUT * K
};

template <int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN, int NB>
static WgfLaunch wgf_launch() {
  using Gm = WgfGeom<KH, KW, S, CIN, COUT, HIN, WIN>;
  static_assert(Gm::K % (NB * 32) == 0, "column groups tile K");
  return WgfLaunch{reinterpret_cast<const void *>(&k_conv_wgrad_f32<KH, KW, S, CIN, COUT, HIN, WIN, NB>),
                   Gm::K / (NB * 32), (int64_t)COUT * Gm::K};
}

static bool find_wgf(const rth_conv_shape &s, WgfLaunch *out) {
  auto is = [&](int cin, int hin, int win, int cout, int kh, int kw, int st) {
    return s.input == RTH_CONV_F32_NHWC && s.cin == cin && s.hin == hin && s.win == win && s.cout == cout &&
           s.kh == kh && s.kw == kw && s.stride == st;
  };
  if (is(32, 20, 20, 64, 4, 4, 2)) {  // conv2: K = 512 -> 4 groups of 128 columns
    static const WgfLaunch l = wgf_launch<4, 4, 2, 32, 64, 20, 20, 4>();
    *out = l;
  } else if (is(64, 9, 9, 64, 3, 3, 1)) {  // conv3: K = 576 -> 6 groups of 96 columns
    static const WgfLaunch l = wgf_launch<3, 3, 1, 64, 64, 9, 9, 3>();
    *out = l;
  } else {
    return false;
  }
  return true;
}

constexpr int kWgfWorkgroups = 256;  // about one per CU: column groups x pixel splits

static int wgf_splits(const WgfLaunch &l) {
  const int s = kWgfWorkgroups / l.groups;
  return s < kWgfRedMax ? s : kWgfRedMax;
}

// ---------------------------------------------------------------------------------------
// The same weight gradient on the bf16 MFMA with both operands split into three exact bf16
// terms (the x9 scheme of conv.hip's k_conv_x9: every partial product xi * gj has at most 16
// significant bits, so it is exact in the fp32 accumulator -- the same real products as the
// fp32 path, summed in another fixed order).  GEMM view as above, on
// v_mfma_f32_16x16x32_bf16: rows = 16 output channels, columns = 16 kk, reduction = a chunk of
// 32 consecutive output pixels, lane l supplying pixels 8 (l >> 4) + j, j < 8, of row / column
// l & 15 -- 8 scalar loads per operand, each a 64-byte run of channels across 16 lanes.
// Workgroup = 4 waves over one column group of 4 blocks (64 kk) and a range of chunks: wave w
// owns output channels 16w .. 16w + 15 (its A fragments, loaded and split by itself) and
// splits column block w's B fragment for the whole workgroup into LDS (double-buffered, one
// barrier per chunk); every wave then runs 4 blocks x 9 MFMAs per chunk.  Partials per
// workgroup go to the workspace; k_conv_wgrad_f32_reduce adds them in split order.
template <int KH, int KW, int S, int CIN, int HIN, int WIN>
struct WgxGeom {
  static constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int K = KH * KW * CIN, COUT = 64, GROUPS = K / 64;
  static_assert(CIN % 16 == 0 && K % 64 == 0, "16-column blocks inside one tap, 64-column groups");
};

__device__ __forceinline__ void split3_x8(const float (&v)[8], bf16x8 (&out)[3]) {
  uint2 lo[3], hi[3];
  split3_x4(make_float4(v[0], v[1], v[2], v[3]), lo);
  split3_x4(make_float4(v[4], v[5], v[6], v[7]), hi);
#pragma unroll
  for (int t = 0; t < 3; ++t) out[t] = __builtin_bit_cast(bf16x8, u32x4{lo[t].x, lo[t].y, hi[t].x, hi[t].y});
}

#ifndef WGX_PF
#define WGX_PF 1
#endif
template <int KH, int KW, int S, int CIN, int HIN, int WIN>
__global__ __launch_bounds__(256) void k_conv_wgrad_x9(const float *__restrict__ x, const float *__restrict__ gy,
                                                      int64_t n, int splits, float *__restrict__ part) {
  using G = WgxGeom<KH, KW, S, CIN, HIN, WIN>;
  constexpr int COUT = G::COUT, PIX = G::PIX, WOUT = G::WOUT, K = G::K;
  __shared__ bf16x8 bl[2][3][4][64];  // [buffer][term][column block][lane]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const int group = (int)(blockIdx.x / splits), split = (int)(blockIdx.x % splits);
  const int64_t P = n * PIX, chunks = (P + 31) / 32;
  const int64_t c0 = chunks * split / splits, c1 = chunks * (split + 1) / splits;
  const int co = wave * 16 + r;                 // A: this lane's output channel
  const int kk = (group * 4 + wave) * 16 + r;   // B staged by this lane: column kk
  const int tap = kk / CIN, ci = kk % CIN;
  const int xoff = ((tap / KW) * WIN + tap % KW) * CIN + ci;
  // pixel indices fit 32 bits (n * PIX < 2^31 is checked on the host)
  const int Pi = (int)P;
  auto load = [&](int64_t c, float (&a)[8], float (&b)[8]) {
    const int p0 = (int)c * 32 + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = p0 + j;
      const bool live = p < Pi;
      const int bb = p / PIX, pix = p - bb * PIX, oy = pix / WOUT, ox = pix - oy * WOUT;
      a[j] = live ? gy[p * COUT + co] : 0.0f;  // a dead pixel weighs 0
      b[j] = live ? x[((bb * HIN + S * oy) * WIN + S * ox) * CIN + xoff] : 0.0f;
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) acc[kb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  // WGX_PF chunks' raw loads in flight (a register ring; the loop is unrolled by WGX_PF)
  float av[WGX_PF][8], bv[WGX_PF][8];
#pragma unroll
  for (int d = 0; d < WGX_PF; ++d)
    if (c0 + d < c1) load(c0 + d, av[d], bv[d]);
  int buf = 0;
  for (int64_t cb = c0; cb < c1; cb += WGX_PF)
#pragma unroll
  for (int d = 0; d < WGX_PF; ++d) {
    const int64_t c = cb + d;
    if (c >= c1) break;  // uniform
    bf16x8 at[3], bt[3];
    split3_x8(av[d], at);
    split3_x8(bv[d], bt);
#pragma unroll
    for (int t = 0; t < 3; ++t) bl[buf][t][wave][lane] = bt[t];
    if (c + WGX_PF < c1) load(c + WGX_PF, av[d], bv[d]);  // in flight during the next chunks
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const bf16x8 b0 = bl[buf][0][kb][lane], b1 = bl[buf][1][kb][lane], b2 = bl[buf][2][kb][lane];
      f32x4 a = acc[kb];
      // smallest terms first: (3,3) (3,2) (2,3) (3,1) (2,2) (1,3) (2,1) (1,2) (1,1)
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[2], b2, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[2], b1, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[1], b2, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[2], b0, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[1], b1, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[0], b2, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[1], b0, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[0], b1, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[0], b0, a, 0, 0, 0);
      acc[kb] = a;
    }
    buf ^= 1;
  }
  // D: lane holds rows (channels) 16 wave + 4 (l >> 4) + i of column 16 kb + (l & 15)
  float *out = part + (int64_t)split * COUT * K;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      out[(int64_t)(wave * 16 + 4 * g + i) * K + (group * 4 + kb) * 16 + r] = acc[kb][i];
}

struct WgxLaunch {
  const void *fn;
  int groups;
  int64_t elems;
};

template <int KH, int KW, int S, int CIN, int HIN, int WIN>
static WgxLaunch wgx_launch() {
  using G = WgxGeom<KH, KW, S, CIN, HIN, WIN>;
  return WgxLaunch{reinterpret_cast<const void *>(&k_conv_wgrad_x9<KH, KW, S, CIN, HIN, WIN>), G::GROUPS,
                   (int64_t)G::COUT * G::K};
}

static bool find_wgx(const rth_conv_shape &s, WgxLaunch *out) {
  auto is = [&](int cin, int hin, int win, int cout, int kh, int kw, int st) {
    return s.input == RTH_CONV_F32_NHWC && s.cin == cin && s.hin == hin && s.win == win && s.cout == cout &&
           s.kh == kh && s.kw == kw && s.stride == st;
  };
  if (is(32, 20, 20, 64, 4, 4, 2)) {  // conv2: K = 512 -> 8 groups of 64 columns
    static const WgxLaunch l = wgx_launch<4, 4, 2, 32, 20, 20>();
    *out = l;
  } else if (is(64, 9, 9, 64, 3, 3, 1)) {  // conv3: K = 576 -> 9 groups (one tap each)
    static const WgxLaunch l = wgx_launch<3, 3, 1, 64, 9, 9>();
    *out = l;
  } else {
    return false;
  }
  return true;
}

#ifndef WGX_SPLITS
#define WGX_SPLITS 64
#endif
static int wgx_splits() {  // RTH_WGX_SPLITS (A/B), at most kWgfRedMax
  static const int v = [] {
    const char *e = getenv("RTH_WGX_SPLITS");
    int x = e ? atoi(e) : WGX_SPLITS;
    return x < 1 ? 1 : (x > kWgfRedMax ? kWgfRedMax : x);
  }();
  return v;
}

}  // namespace rth

using namespace rth;

extern "C" {

int rth_conv_wgrad_x9_supported(const rth_conv_shape *shape) {
  WgxLaunch l;
  return shape && find_wgx(*shape, &l) ? 1 : 0;
}

int64_t rth_conv_wgrad_x9_workspace(const rth_conv_shape *shape) {
  WgxLaunch l;
  if (!shape || !find_wgx(*shape, &l)) return 0;
  return (int64_t)wgx_splits() * l.elems * 4;
}

int rth_conv_wgrad_x9(const rth_conv_shape *shape, const float *x, int64_t n, const float *gy, float *gw,
                      void *workspace, void *stream) {
  RTH_REQUIRE(shape && x && gy && gw && workspace && n >= 0, "rth_conv_wgrad_x9: NULL argument");
  WgxLaunch l;
  RTH_REQUIRE(find_wgx(*shape, &l), "rth_conv_wgrad_x9: geometry (%d x %d x %d -> %d, k %dx%d, stride %d) not built",
              shape->cin, shape->hin, shape->win, shape->cout, shape->kh, shape->kw, shape->stride);
  if (n == 0) {
    RTH_HIP(hipMemsetAsync(gw, 0, l.elems * 4, as_stream(stream)));
    return RTH_OK;
  }
  RTH_REQUIRE(n * shape->cin * shape->hin * shape->win < ((int64_t)1 << 31), "rth_conv_wgrad_x9: batch too large");
  int splits = wgx_splits();
  float *part = static_cast<float *>(workspace);
  void *args[] = {(void *)&x, (void *)&gy, (void *)&n, (void *)&splits, (void *)&part};
  RTH_HIP(hipLaunchKernel(l.fn, dim3((unsigned)(l.groups * splits)), dim3(256), args, 0, as_stream(stream)));
  hipLaunchKernelGGL(k_conv_wgrad_f32_reduce, dim3((unsigned)((l.elems + 63) / 64)), dim3(256), 0, as_stream(stream),
                     part, splits, l.elems, gw);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_conv_wgrad_f32_supported(const rth_conv_shape *shape) {
  WgfLaunch l;
  return shape && find_wgf(*shape, &l) ? 1 : 0;
}

int64_t rth_conv_wgrad_f32_workspace(const rth_conv_shape *shape) {
  WgfLaunch l;
  if (!shape || !find_wgf(*shape, &l)) return 0;
  return (int64_t)wgf_splits(l) * l.elems * 4;
}

int rth_conv_wgrad_f32(const rth_conv_shape *shape, const float *x, int64_t n, const float *gy, float *gw,
                       void *workspace, void *stream) {
  RTH_REQUIRE(shape && x && gy && gw && workspace && n >= 0, "rth_conv_wgrad_f32: NULL argument");
  WgfLaunch l;
  RTH_REQUIRE(find_wgf(*shape, &l), "rth_conv_wgrad_f32: geometry (%d x %d x %d -> %d, k %dx%d, stride %d) not built",
              shape->cin, shape->hin, shape->win, shape->cout, shape->kh, shape->kw, shape->stride);
  if (n == 0) {
    RTH_HIP(hipMemsetAsync(gw, 0, l.elems * 4, as_stream(stream)));
    return RTH_OK;
  }
  int splits = wgf_splits(l);
  float *part = static_cast<float *>(workspace);
  void *args[] = {(void *)&x, (void *)&gy, (void *)&n, (void *)&splits, (void *)&part};
  RTH_HIP(hipLaunchKernel(l.fn, dim3((unsigned)(l.groups * splits)), dim3(kWgfWaves * 64), args, 0,
                          as_stream(stream)));
  hipLaunchKernelGGL(k_conv_wgrad_f32_reduce, dim3((unsigned)((l.elems + 63) / 64)), dim3(256), 0, as_stream(stream),
                     part, splits, l.elems, gw);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
