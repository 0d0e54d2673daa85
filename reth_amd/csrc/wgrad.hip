// Weight gradient of conv2 / conv3 of the Nature-DQN torso on the fp32 MFMA, deterministic
// and without a zero fill (replaces MIOpen's igemm_wrw and its fill).  Reference: the
// backward of reth/reth/algorithm/dqn/dqn_model.py:14-20 under dqn_solver.py:117
// (loss.backward()).
//
//   gw[co][kh][kw][ci] = sum over output pixels p = (b, oy, ox) of
//                        gy[p][co] * x[b][S*oy + kh][S*ox + kw][ci]
//
// x (the layer's input) and gy (the masked upstream gradient) are channels-last fp32; gw is
// the OHWI (channels_last) weight gradient.  GEMM view: rows = co (64), columns = kk =
// (kh, kw, ci) in OHWI order (K = KH*KW*CIN), reduction over the output pixels.
//
// r06 form (register-only main loop, no LDS operand staging: it runs beside the actor stream's
// LDS-hungry x9 convolutions).  A workgroup owns one column group -- GN = 32 * NB consecutive
// kk inside one kernel row kh, contiguous in x -- and a range of pixel pairs (its split); each
// of its waves a consecutive part of that range.  v_mfma_f32_32x32x2f32 with the lanes
// (i = lane & 31, h = lane >> 5) of a wave on the pixels 2q + h of pair q:
//   A[i][h] = gy[p][2i + c]             (row block c in {0, 1}: one float2 load per lane)
//   B[h][i] = x-row[p][col0 + NB*i + n] (column block n < NB: NB consecutive floats)
// so a lane's loads are wide and the wave's 2 x NB accumulators (64 x GN outputs) take a pair
// of pixels per 2 * NB MFMAs; PF pairs of loads are in flight ahead of their MFMAs, addressed by
// an incremental cursor (adds and selects only).  The loads go through buffer resources over the
// batch: a pixel past it reads zeros (contributes 0).  The waves' accumulators are added in LDS
// in a fixed tree, one 32x32 block at a time, and wave 0 stores the workgroup's partial in the
// accumulator order; the reduce (wgrad.hpp: k_conv_wgrad_f32_reduce here, or conv1's reduce
// launch for a deferred job) adds the splits' partials in split order and scatters them to
// OHWI.  Every sum has a fixed order: run to run bit-identical.
#include <type_traits>

#include "common.hpp"
#include "wgrad.hpp"

namespace rth {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x3 = __attribute__((ext_vector_type(3))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;

// column groups: GN = 32 * NB consecutive kk per wave (inside one kernel row), NB in {2, 3, 4, 6}
template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NB>
struct WgfGeom {
  static constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int COUT = 64, K = KH * KW * CIN, NCOL = KW * CIN, GN = 32 * NB;
  static constexpr int GROUPS = K / GN;     // column groups
  static constexpr int BLK = 2 * NB;        // 32x32 accumulator blocks per wave
  static constexpr int TILE = BLK * 1024;   // floats of one workgroup's partial (= 64 * GN)
  static_assert(NCOL % GN == 0, "a column group inside one kernel row");
};

template <int NB>
struct XVec;
template <>
struct XVec<2> {
  f32x2 v;
  __device__ __forceinline__ float operator[](int k) const { return v[k]; }
};
template <>
struct XVec<3> {
  f32x3 v;
  __device__ __forceinline__ float operator[](int k) const { return v[k]; }
};
template <>
struct XVec<4> {
  f32x4 v;
  __device__ __forceinline__ float operator[](int k) const { return v[k]; }
};
template <>
struct XVec<6> {
  f32x2 v[3];
  __device__ __forceinline__ float operator[](int k) const { return v[k >> 1][k & 1]; }
};

template <int NB>
__device__ __forceinline__ void load_xvec(XVec<NB> &o, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (NB == 2) {
    o.v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  } else if constexpr (NB == 3) {
    o.v = __builtin_bit_cast(f32x3, __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0));
  } else if constexpr (NB == 4) {
    o.v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  } else {
#pragma unroll
    for (int k = 0; k < 3; ++k)
      o.v[k] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off + 8 * k, 0, 0));
  }
}

// WAVES waves per workgroup take consecutive quarters / eighths of the workgroup's pair range
// and are summed in the fixed tree ((w0 + w1) + (w2 + w3)) + ((w4 + w5) + (w6 + w7)), one 32x32
// block at a time, each tree level in its own LDS slots (WAVES - 1 slots of 4 KB: one barrier
// per level, and a block's slots are free again before the next block writes them)
template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NB, int WAVES, int PF>
__global__ __launch_bounds__(WAVES * 64) void k_conv_wgrad_f32(const float *__restrict__ x,
                                                              const float *__restrict__ gy, int n, int splits,
                                                              float *__restrict__ part) {
  using G = WgfGeom<KH, KW, S, CIN, HIN, WIN, NB>;
  constexpr int PIX = G::PIX, WOUT = G::WOUT, HOUT_ = G::HOUT, LEVELS = WAVES == 8 ? 3 : WAVES == 4 ? 2 : 1;
  static_assert(WAVES == 2 || WAVES == 4 || WAVES == 8, "2, 4 or 8 waves");
  __shared__ float red[WAVES - 1][1024];
  const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // workgroup -> (split, column group): the GROUPS workgroups of a split sit on one XCD
  // (blockIdx % 8 equal) and share its gy pairs through that XCD's L2
  const int b8 = blockIdx.x & 7, rest = blockIdx.x >> 3;
  const int grp = rest % G::GROUPS, split = (rest / G::GROUPS) * 8 + b8;
  const int kk0 = grp * G::GN, kh = kk0 / G::NCOL, col0 = kk0 - kh * G::NCOL;
  const int P = n * PIX, pairs = (P + 1) >> 1;
  const int units = splits * WAVES, u = split * WAVES + wave;
  const int q0 = (int)((int64_t)pairs * u / units), q1 = (int)((int64_t)pairs * (u + 1) / units);

  const __amdgpu_buffer_rsrc_t g_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(gy), 0, P * G::COUT * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x), 0, n * HIN * WIN * CIN * 4, 0x00020000);

  f32x16 acc[2][NB];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][nb][r] = 0.0f;

  f32x2 av[PF];
  XVec<NB> bv[PF];
  // a cursor over this lane's pixels 2q + h: (oy, ox) and both byte offsets advance by one pair
  // per issue with adds and selects only; past the batch both offsets run past the resources'
  // ranges and read 0
  constexpr uint32_t XSTEP = 2 * S * CIN * 4;                         // ox += 2
  constexpr uint32_t XROW = (S * WIN - WOUT * S) * CIN * 4;           // ox wrapped: next output row
  constexpr uint32_t XIMG = (HIN * WIN - HOUT_ * S * WIN) * CIN * 4;  // oy wrapped: next sample
  int cox, coy;
  uint32_t goff, xoff;
  {
    const int p = 2 * q0 + h, b = p / PIX, rem = p - b * PIX;
    coy = rem / WOUT;
    cox = rem - coy * WOUT;
    goff = (uint32_t)p * (G::COUT * 4) + (uint32_t)i * 8;
    xoff = (uint32_t)((((b * HIN + S * coy + kh) * WIN + S * cox) * CIN + col0 + NB * i) * 4);
  }
  auto issue = [&](int d) {
    av[d] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(g_rsrc, goff, 0, 0));
    load_xvec<NB>(bv[d], x_rsrc, xoff);
    goff += 2 * G::COUT * 4;
    cox += 2;
    const bool w1 = cox >= WOUT;
    cox = w1 ? cox - WOUT : cox;
    coy = w1 ? coy + 1 : coy;
    const bool w2 = coy == HOUT_;
    coy = w2 ? 0 : coy;
    xoff += XSTEP + (w1 ? XROW : 0u) + (w2 ? XIMG : 0u);
  };
  auto mfmas = [&](int d) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[c][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[d][c], bv[d][nb], acc[c][nb], 0, 0, 0);
  };

  // the prologue's loads in the loop's order (slot by slot), so the waits the compiler derives
  // at the loop header count the same loads on both edges (else it waits for nearly all)
#pragma unroll
  for (int d = 0; d < PF; ++d) {
    issue(d);
    __builtin_amdgcn_sched_barrier(0);
  }
  int q = q0;
#pragma unroll 1
  for (; q + PF <= q1; q += PF) {
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      mfmas(d);
      // the refill of slot d right behind its MFMAs (the scheduler would sink it to its use
      // PF pairs later)
      __builtin_amdgcn_sched_barrier(0);
      issue(d);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < PF - 1; ++d)
    if (q + d < q1) mfmas(d);  // the last < PF pairs (wave-uniform)

  // the waves' tree sum; wave 0 stores the partial [split][group][block][register][lane]
  float *out = part + ((int64_t)split * G::GROUPS + grp) * G::TILE;
#pragma unroll
  for (int blk = 0; blk < G::BLK; ++blk) {
    f32x16 &v = acc[blk / NB][blk % NB];
    int base = 0;
#pragma unroll
    for (int lv = 0; lv < LEVELS; ++lv) {
      const int span = 1 << lv;  // waves w with w % span == 0 hold the level's inputs
      if (wave % (2 * span) == span) {
        float *s = red[base + (wave >> (lv + 1))];
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r * 64 + lane] = v[r];
      }
      __syncthreads();
      if (wave % (2 * span) == 0) {
        const float *s = red[base + (wave >> (lv + 1))];
        if (lv == LEVELS - 1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) out[(blk * 16 + r) * 64 + lane] = radd(v[r], s[r * 64 + lane]);
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = radd(v[r], s[r * 64 + lane]);
        }
      }
      base += WAVES >> (lv + 1);
    }
  }
}

// gw = the sum of the splits' partials in split order (wgrad.hpp), scattered to OHWI
__global__ __launch_bounds__(kWgfRedElems) void k_conv_wgrad_f32_reduce(WgfJob j) {
  wgf_reduce_wg(j, blockIdx.x);
}

struct WgfLaunch {
  const void *fn;
  int groups;  // column groups (K / (32 * NB))
  int nb;      // column blocks per group
  int K;       // KH * KW * CIN
  int elems;   // 64 * K
  int splits;  // pixel splits (a multiple of 8)
  int threads; // 64 * waves
};

template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NB, int WAVES, int PF>
static WgfLaunch wgf_launch(int splits) {
  using Gm = WgfGeom<KH, KW, S, CIN, HIN, WIN, NB>;
  return WgfLaunch{reinterpret_cast<const void *>(&k_conv_wgrad_f32<KH, KW, S, CIN, HIN, WIN, NB, WAVES, PF>),
                   Gm::GROUPS, NB, Gm::K, Gm::COUT * Gm::K, splits, WAVES * 64};
}

// the launch per geometry, picked in the loop (r06, interleaved A/Bs of the Pong step,
// profiles/r06/wgrad_ab.txt): conv2 on 64-column groups, 8 waves (two per SIMD), 48 splits
// (0.511-0.513 ms/step; 4 waves of 128 columns x 64 splits 0.518-0.520; MIOpen 0.515-0.518);
// conv3 on 96-column groups, 4 waves, 40 splits (its other forms 0.517-0.521)
static bool find_wgf(const rth_conv_shape &s, WgfLaunch *out) {
  auto is = [&](int cin, int hin, int win, int cout, int kh, int kw, int st) {
    return s.input == RTH_CONV_F32_NHWC && s.cin == cin && s.hin == hin && s.win == win && s.cout == cout &&
           s.kh == kh && s.kw == kw && s.stride == st;
  };
  if (is(32, 20, 20, 64, 4, 4, 2)) {  // conv2: 8 groups of 64 columns
    static const WgfLaunch l = wgf_launch<4, 4, 2, 32, 20, 20, 2, 8, 8>(48);
    *out = l;
  } else if (is(64, 9, 9, 64, 3, 3, 1)) {  // conv3: 6 groups of 96 columns
    static const WgfLaunch l = wgf_launch<3, 3, 1, 64, 9, 9, 3, 4, 8>(40);
    *out = l;
  } else {
    return false;
  }
  return true;
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
  const WgfJob job{part, gw, splits, (int)l.elems, 0, 0};
  hipLaunchKernelGGL(k_conv_wgrad_f32_reduce, dim3((unsigned)wgf_reduce_blocks(job)), dim3(kWgfRedElems), 0,
                     as_stream(stream), job);
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
  return (int64_t)l.splits * l.elems * 4;
}

// the partial launch alone; *job = the reduce it needs (rth_conv_wgrad_f32 reduces at once,
// conv1's reduce launch takes it as a deferred job)
static int wgf_partials(const rth_conv_shape *shape, const float *x, int64_t n, const float *gy, float *gw,
                        void *workspace, WgfJob *job, void *stream) {
  RTH_REQUIRE(shape && (n == 0 || (x && gy)) && gw && workspace && n >= 0, "rth_conv_wgrad_f32: NULL argument");
  WgfLaunch l;
  RTH_REQUIRE(find_wgf(*shape, &l), "rth_conv_wgrad_f32: geometry (%d x %d x %d -> %d, k %dx%d, stride %d) not built",
              shape->cin, shape->hin, shape->win, shape->cout, shape->kh, shape->kw, shape->stride);
  // byte offsets of both buffer resources are 32-bit
  RTH_REQUIRE(n * shape->cin * shape->hin * shape->win * 4 < ((int64_t)1 << 31) &&
                  n * ((shape->hin - shape->kh) / shape->stride + 1) * ((shape->win - shape->kw) / shape->stride + 1) *
                          shape->cout * 4 < ((int64_t)1 << 31),
              "rth_conv_wgrad_f32: batch too large");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gy)) & 15) == 0,
              "rth_conv_wgrad_f32: misaligned buffer");
  int ni = (int)n, splits = l.splits;
  float *part = static_cast<float *>(workspace);
  *job = WgfJob{part, gw, n == 0 ? 0 : splits, l.elems, l.nb, l.K};  // no split: the reduce writes zeros
  if (n == 0) return RTH_OK;
  void *args[] = {(void *)&x, (void *)&gy, (void *)&ni, (void *)&splits, (void *)&part};
  RTH_HIP(hipLaunchKernel(l.fn, dim3((unsigned)(l.groups * splits)), dim3(l.threads), args, 0, as_stream(stream)));
  return RTH_OK;
}

int rth_conv_wgrad_f32(const rth_conv_shape *shape, const float *x, int64_t n, const float *gy, float *gw,
                       void *workspace, void *stream) {
  WgfJob job;
  const int rc = wgf_partials(shape, x, n, gy, gw, workspace, &job, stream);
  if (rc != RTH_OK) return rc;
  hipLaunchKernelGGL(k_conv_wgrad_f32_reduce, dim3((unsigned)wgf_reduce_blocks(job)), dim3(kWgfRedElems), 0,
                     as_stream(stream), job);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_conv_wgrad_f32_partials(const rth_conv_shape *shape, const float *x, int64_t n, const float *gy, float *gw,
                                void *workspace, rth_wgrad_deferred *job_out, void *stream) {
  RTH_REQUIRE(job_out, "rth_conv_wgrad_f32_partials: NULL job");
  WgfJob job;
  const int rc = wgf_partials(shape, x, n, gy, gw, workspace, &job, stream);
  if (rc != RTH_OK) return rc;
  *job_out = rth_wgrad_deferred{job.part, job.gw, job.splits, job.elems, job.nb, job.K};
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
