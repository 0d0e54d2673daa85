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
#include <type_traits>

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
constexpr int kWgfRedMax = 128;  // splits per element at most: 32 per thread
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
// fp32 path, summed in another fixed order), each operand split ONCE per workgroup.
//
// GEMM view as above on v_mfma_f32_16x16x32_bf16: rows = 16 output channels, columns = 16 kk,
// reduction = a chunk of 32 consecutive output pixels p = (b, oy, ox), lane group g supplying
// pixels 8g .. 8g + 7.  A workgroup owns one kernel row kh (the KW * CIN columns kk = (kh, kw,
// ci), 128 at conv2, 192 at conv3) x all 64 output channels, and a range of chunks (its split).
// Per chunk it stages both operands in LDS already split and transposed to the fragment
// order -- per term, one 64-byte row per output channel (gy) and per column (the im2col x),
// each row the 32 pixels' bf16 values as 4 16-byte units (unit g = pixels 8g .. 8g + 7, XOR-
// placed within the row so that every ds_read_b128 lane group of 16 hits 16 distinct bank
// quads) --, then every wave runs its CPW column blocks x 4 channel blocks x 9 MFMAs from it.
// Staging: 64 threads load gy (float4 = 4 channels of one pixel, 8 pixels each), the next
// XQ * 4 threads the im2col x (float4 = 4 consecutive kk of one pixel, 8 pixels each; the
// pixels' window offsets from a per-chunk table), one chunk ahead in registers; each splits its
// 4 x 8 values into 3 x 4 fragments with v_cvt_pk_bf16_f32.  Partials per workgroup go to the
// workspace; k_conv_wgrad_f32_reduce adds them in split order.
template <int KH, int KW, int S, int CIN, int HIN, int WIN>
struct WgxGeom {
  static constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int K = KH * KW * CIN, COUT = 64, GROUPS = KH;
  static constexpr int NCOL = KW * CIN;     // columns per workgroup (one kernel row)
  static constexpr int NCB = NCOL / 16;     // column blocks
  static constexpr int CPW = NCB / 4;       // column blocks per wave (4 waves)
  static constexpr int XQ = NCOL / 4;       // x column quads
  static constexpr int ROWS = COUT + NCOL;  // LDS rows per term: gy channels, then x columns
  static constexpr int LDS_U4 = 3 * ROWS * 4;
  static_assert(CIN % 4 == 0 && NCB % 4 == 0 && 64 + 4 * XQ <= 256, "column quads, 4 waves of column blocks");
};

// the 16-byte unit of (term, row, pixel group g): rows of 4 units, g XORed with a per-row-quad
// key {0, 2, 3, 1} -- a ds_read_b128 lane group ({0-3, 12-15, 20-27}, ...: rows r and r + 12 of
// one g and rows r + 4 .. r + 11 of the next) then covers all 16 bank quads once
template <int ROWS>
__device__ __forceinline__ int wgx_unit(int t, int row, int g) {
  return (t * ROWS + row) * 4 + (g ^ ((0x78 >> (2 * ((row >> 2) & 3))) & 3));
}

template <int KH, int KW, int S, int CIN, int HIN, int WIN>
__global__ __launch_bounds__(256) void k_conv_wgrad_x9(const float *__restrict__ x, const float *__restrict__ gy,
                                                      int64_t n, int splits, float *__restrict__ part) {
  using G = WgxGeom<KH, KW, S, CIN, HIN, WIN>;
  constexpr int COUT = G::COUT, PIX = G::PIX, WOUT = G::WOUT, K = G::K, ROWS = G::ROWS, CPW = G::CPW;
  constexpr int BUF = G::LDS_U4 + 3 * 4 * 4;  // + a scratch row quad per term (the idle lanes' stores)
  __shared__ uint4 lds[2][BUF];                // double-buffered: chunk c computes while c + 1 is staged
  __shared__ int tbl[2][32];                   // per chunk: each pixel's window origin in x
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = (int)(blockIdx.x / splits), split = (int)(blockIdx.x % splits);
  const int P = (int)(n * PIX);  // < 2^31: checked on the host
  const int chunks = (P + 31) / 32;
  const int c0 = (int)((int64_t)chunks * split / splits), c1 = (int)((int64_t)chunks * (split + 1) / splits);
  if (c0 >= c1) {  // an empty split still owns its partial
    float *out = part + (int64_t)split * COUT * K + kh * G::NCOL;
    for (int e = tid; e < COUT * G::NCOL; e += 256) out[(int64_t)(e / G::NCOL) * K + e % G::NCOL] = 0.f;
    return;
  }
  // staging role, wave-uniform: wave 0 gy (channel quad, pixel group), the next waves the im2col
  // x (column quad, pixel group); lanes past the x tasks repeat one and store into the scratch rows
  const bool is_gy = wave == 0;
  const int u = is_gy ? tid : (tid - 64) % (4 * G::XQ);
  const int quad = is_gy ? (u & 15) : (u % G::XQ), spg = is_gy ? (u >> 4) : (u / G::XQ);
  const int qcol = 4 * quad;
  const int xoff = (kh * WIN + qcol / CIN) * CIN + qcol % CIN;  // (kh, kw, ci0) inside the window
  const int row0 = is_gy ? qcol : (tid - 64 < 4 * G::XQ ? COUT + qcol : ROWS);
  // both operands through buffer resources: a gy pixel past P reads zeros (and weighs 0)
  const __amdgpu_buffer_rsrc_t gy_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(gy), 0, P * COUT * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(x), 0, (int)(n * (int64_t)(HIN * WIN * CIN) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t src_rsrc = is_gy ? gy_rsrc : x_rsrc;  // wave-uniform: one load per element
  auto make_tbl = [&](int c) __attribute__((always_inline)) {  // every lane writes its pixel's entry (lanes 32 apart agree)
    const int p = c * 32 + (tid & 31);
    const int b = p / PIX, pp = p - b * PIX, oy = pp / WOUT, ox = pp - oy * WOUT;
    tbl[c & 1][tid & 31] = p < P ? ((b * HIN + S * oy) * WIN + S * ox) * CIN : 0;  // dead: x's first window
  };
  auto load = [&](int c, f32x4 (&pv)[8]) __attribute__((always_inline)) {
    const int4 *t4 = reinterpret_cast<const int4 *>(&tbl[c & 1][8 * spg]);
    const int4 ta = t4[0], tb = t4[1];
    const int o[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t og = (uint32_t)(((c * 32 + 8 * spg + j) * COUT + qcol) * 4);
      const uint32_t ox4 = (uint32_t)((o[j] + xoff) * 4);
      pv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(src_rsrc, is_gy ? og : ox4, 0, 0));
    }
  };
  auto stage_row = [&](const f32x4 (&pv)[8], auto ec, uint4 *buf) __attribute__((always_inline)) {  // row e of the quad
    constexpr int e = decltype(ec)::value;
    // (clang vectors, not HIP's float4: its union members kept these registers in private memory)
    const float v[8] = {pv[0][e], pv[1][e], pv[2][e], pv[3][e], pv[4][e], pv[5][e], pv[6][e], pv[7][e]};
    bf16x8 tr[3];
    split3_pk8(v, tr);
#pragma unroll
    for (int t = 0; t < 3; ++t) buf[wgx_unit<ROWS + 4>(t, row0 + e, spg)] = __builtin_bit_cast(uint4, tr[t]);
  };
  f32x4 acc[4][CPW];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int kb = 0; kb < CPW; ++kb) acc[cb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // chunk c: its MFMAs from lds[(c - c0) & 1], chunk c + 1's rows (registers ps, loaded one
  // iteration earlier) staged into the other buffer between the channel blocks' MFMAs, chunk
  // c + 2's loads into pl; one barrier per chunk
  auto iter = [&](int c, f32x4 (&ps)[8], f32x4 (&pl)[8]) __attribute__((always_inline)) {
    load(c + 2, pl);
    const uint4 *cur = lds[(c - c0) & 1];
    uint4 *nxt = lds[(c - c0 + 1) & 1];
    bf16x8 bfr[CPW][3];
#pragma unroll
    for (int kb = 0; kb < CPW; ++kb)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        bfr[kb][t] = __builtin_bit_cast(bf16x8, cur[wgx_unit<ROWS + 4>(t, COUT + 16 * (wave * CPW + kb) + r, g)]);
    // the 4 channel blocks as compile-time steps (a runtime cb would index acc / ps dynamically:
    // private memory)
    auto cbstep = [&](auto cbc, const f32x4 (&pst)[8]) __attribute__((always_inline)) {
      constexpr int cb = decltype(cbc)::value;
      bf16x8 af[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) af[t] = __builtin_bit_cast(bf16x8, cur[wgx_unit<ROWS + 4>(t, 16 * cb + r, g)]);
#pragma unroll
      for (int kb = 0; kb < CPW; ++kb) {
        f32x4 a = acc[cb][kb];
        const bf16x8(&b)[3] = bfr[kb];
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
        acc[cb][kb] = a;
      }
      stage_row(pst, cbc, nxt);  // (past c1 - 1: staged into a buffer nobody reads)
    };
    cbstep(std::integral_constant<int, 0>{}, ps);
    cbstep(std::integral_constant<int, 1>{}, ps);
    cbstep(std::integral_constant<int, 2>{}, ps);
    cbstep(std::integral_constant<int, 3>{}, ps);
    make_tbl(c + 3);  // its buffer was last read by load(c + 1)
    __syncthreads();
  };
  f32x4 pa[8], pb[8];
  make_tbl(c0);
  make_tbl(c0 + 1);
  __syncthreads();
  load(c0, pa);
  load(c0 + 1, pb);
  stage_row(pa, std::integral_constant<int, 0>{}, lds[0]);
  stage_row(pa, std::integral_constant<int, 1>{}, lds[0]);
  stage_row(pa, std::integral_constant<int, 2>{}, lds[0]);
  stage_row(pa, std::integral_constant<int, 3>{}, lds[0]);
  make_tbl(c0 + 2);
  __syncthreads();
  int c = c0;
  for (; c + 1 < c1; c += 2) {
    iter(c, pb, pa);
    iter(c + 1, pa, pb);
  }
  if (c < c1) iter(c, pb, pa);
  // D: lane holds channels 16 cb + 4 g + i of column 16 (wave * CPW + kb) + r of this kernel row
  float *out = part + (int64_t)split * COUT * K + kh * G::NCOL;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int kb = 0; kb < CPW; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) out[(int64_t)(16 * cb + 4 * g + i) * K + 16 * (wave * CPW + kb) + r] = acc[cb][kb][i];
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
  if (is(32, 20, 20, 64, 4, 4, 2)) {  // conv2: 4 kernel rows of 128 columns
    static const WgxLaunch l = wgx_launch<4, 4, 2, 32, 20, 20>();
    *out = l;
  } else if (is(64, 9, 9, 64, 3, 3, 1)) {  // conv3: 3 kernel rows of 192 columns
    static const WgxLaunch l = wgx_launch<3, 3, 1, 64, 9, 9>();
    *out = l;
  } else {
    return false;
  }
  return true;
}

// splits per kernel row: about one workgroup per CU over the KH rows, at most kWgfRedMax
static int wgx_splits(const WgxLaunch &l) {
  int x = 256 / l.groups;
  return x < 1 ? 1 : (x > kWgfRedMax ? kWgfRedMax : x);
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
  return (int64_t)wgx_splits(l) * l.elems * 4;
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
  RTH_REQUIRE(n * shape->cin * shape->hin * shape->win < ((int64_t)1 << 31) &&
                  n * ((shape->hin - shape->kh) / shape->stride + 1) * ((shape->win - shape->kw) / shape->stride + 1) *
                          shape->cout * 4 < ((int64_t)1 << 31),
              "rth_conv_wgrad_x9: batch too large");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gy)) & 15) == 0,
              "rth_conv_wgrad_x9: misaligned buffer");
  int splits = wgx_splits(l);
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
