// Nature-DQN convolution torso forward on gfx950: relu(conv2d(x, W) + b) as an implicit GEMM
// on the fp32 MFMA (v_mfma_f32_16x16x4_f32), bias and ReLU applied to the accumulators, NHWC
// fp32 output.  Reference: reth/reth/algorithm/dqn/dqn_model.py:14-20 (Conv2d(4,32,8,4) ->
// ReLU -> Conv2d(32,64,4,2) -> ReLU -> Conv2d(64,64,3,1) -> ReLU).
//
// GEMM view: rows = output pixels (n, oy, ox), columns = output channels, K = (kh, kw, ci).
//   * one wave owns a tile of 16 output pixels x all COUT channels (COUT/16 accumulators of
//     4 registers); the A operand (input window) is read straight from global memory into
//     registers, the B operand (weights) from LDS;
//   * the whole weight tensor is staged once per workgroup in LDS in MFMA fragment order
//     [chunk g][channel block nb][lane][t], so every B read is one conflict-free ds_read_b128
//     feeding four k-steps;
//   * K is walked in chunks of 16 values: lane (m = lane & 15, q = lane >> 4) holds 4
//     consecutive values of the input window (one float4, or 4 uint8 of a CHW stack), k-step
//     t of the chunk multiplies value t -- the k order is a permutation of (kh, kw, ci), the
//     weights are staged in the same permutation.
//
// Input forms:
//   RTH_CONV_F32_NHWC  x = [n, HIN, WIN, CIN] fp32 (the previous layer's output, or the
//                      learner's gathered channels-last batch); K runs are kh rows of
//                      KW*CIN contiguous floats
//   RTH_CONV_U8_CHW    x = uint8 frame stacks [CIN, HIN, WIN] (replay rows / actor frame
//                      ring), optionally addressed through a row index -- the u8 -> f32 cast
//                      happens in registers, no f32 copy of the observation ever exists; K
//                      runs are (ci, kh) rows of KW = 8 contiguous bytes
//
// Numerics: each output is an fp32 fma chain over K in the permuted order above (MFMA f32 is
// a k-ordered fmaf chain), then + bias, then ReLU -- the same operations as conv -> bias ->
// relu, summed in a different order than MIOpen's or the reference's CPU convolution.
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>

#include "common.hpp"
#include "optim.hpp"
#include "wgrad.hpp"

namespace rth {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ float relu_c(float v) { return v < 0.0f ? 0.0f : v; }  // NaN passes, like torch

template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN>
struct ConvGeom {
  static constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int K = KH * KW * CIN, G = K / 16, NB = COUT / 16;
  static constexpr int LDS_F4 = G * NB * 64;  // float4 slots of the staged weights
  // input chunks in flight per wave (f32 input): a divisor of G, at most 8 / MB
  static constexpr int prefetch(int mb) {
    for (int d = 8 / mb; d > 1; --d)
      if (G % d == 0) return d;
    return 1;
  }
  static constexpr int64_t STACK = (int64_t)CIN * HIN * WIN;
  static_assert(K % 16 == 0 && COUT % 16 == 0, "K and COUT must be multiples of 16");
  static_assert(MODE == 0 ? (KW * CIN) % 16 == 0 : (KW == 8 && KH % 2 == 0), "unsupported window");

  // the 4 weights of LDS float4 slot sl = (g * NB + nb) * 64 + lane (t = 0..3) from W in
  // OHWI storage: f32 input -> 4 consecutive ci (one 16-byte read); u8 input -> 4 kw
  __device__ static f32x4 load_slot(const float *__restrict__ w, int sl) {
    const int lane = sl % 64, gn = sl / 64, nb = gn % NB, g = gn / NB;
    const int q = lane >> 4, o = nb * 16 + (lane & 15);
    if (MODE == RTH_CONV_F32_NHWC) {
      constexpr int RC = KW * CIN / 16;
      const int kh = g / RC, r = (g % RC) * 16 + 4 * q;  // r = kw * CIN + ci, ci % 4 == 0
      const float4 v = *reinterpret_cast<const float4 *>(w + (int64_t)o * K + kh * KW * CIN + r);
      return f32x4{v.x, v.y, v.z, v.w};
    } else {
      const int rho = 2 * g + (q >> 1), ci = rho / KH, kh = rho % KH, kw = 4 * (q & 1);
      const float *p = w + (int64_t)o * K + (kh * KW + kw) * CIN + ci;
      return f32x4{p[0], p[CIN], p[2 * CIN], p[3 * CIN]};
    }
  }
};

// In-kernel clock of the fp32-MFMA kernel (a diagnostic build only, -DRTH_CLOCK_STAMPS: the
// shader-clock and 100 MHz wall-clock ticks around wave 0's work of each workgroup, read by
// rth_debug_conv_clock; the product build executes no stamp).  The stamps go to a buffer of
// their own that no kernel reads.
constexpr int kClockSlots = 1024;
__device__ unsigned long long g_conv_clock[kClockSlots][2];

// NS > 1: a wave tile is TP pixels x COUT / NS channels (tile t = pixel tile t / NS, channel
// part t % NS), for more, smaller tiles over the SIMDs; each output keeps its K order.
// PW (r05): the channel part is fixed per workgroup (blockIdx % NS; the grid a multiple of NS)
// and the workgroup stages only that part's weights -- 1 / NS of the LDS, so a workgroup of
// the other stream's kernels (hipBLASLt's FC1 tiles, an x9 conv) fits on the same CU.
// (A dynamic schedule -- waves claiming tiles from a launch-wide atomic counter -- was built
// and measured in r05: 2x slower alone, 108 vs 57 us at 1,024 samples, since every claim is an
// agent-scope atomic on one address from all 8 XCDs; removed.)
template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN, int WAVES, int MB, int NS = 1,
          int PW = 0, int TS = 1>
__global__ __launch_bounds__(WAVES * 64) void k_conv_bias_relu(const void *__restrict__ x,
                                                              const int64_t *__restrict__ rows, int64_t n,
                                                              const int64_t *__restrict__ n_dev,
                                                              const float *__restrict__ w,
                                                              const float *__restrict__ bias,
                                                              float *__restrict__ y, int out_nchw) {
  using Gm = ConvGeom<MODE, KH, KW, S, CIN, COUT, HIN, WIN>;
  constexpr bool F32 = MODE == RTH_CONV_F32_NHWC;
  constexpr int G = Gm::G, NB = Gm::NB, T = WAVES * 64, NBW = NB / NS;
  static_assert(NB % NS == 0, "NS must divide COUT / 16");
  constexpr int TP = 16 * MB;                    // output pixels per wave tile
  constexpr int D = F32 ? Gm::prefetch(MB) : G;  // input chunks in flight per wave
  using Frag = typename std::conditional<F32, f32x4, uint32_t>::type;
  static_assert(!PW || NS > 1, "PW needs channel parts");
  static_assert(TS == 1 || (NS == 1 && !PW && NB % TS == 0), "a split last round needs full-width tiles");
  constexpr int LDSW = PW ? Gm::LDS_F4 / NS : Gm::LDS_F4;  // staged float4 slots
  __shared__ f32x4 wl[LDSW];
  const int part = PW ? (int)(blockIdx.x % NS) : 0;               // PW: this workgroup's channel part
  const int64_t wgs = PW ? gridDim.x / NS : gridDim.x, wgi = PW ? blockIdx.x / NS : blockIdx.x;

  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int q = lane >> 4, mr = lane & 15;
#ifdef RTH_CLOCK_STAMPS
  const unsigned long long clk0 = __builtin_amdgcn_s_memtime(), wall0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (n_dev) {  // a device-side sample count (<= n): rows past it are neither read nor written
    const int64_t m = *n_dev;
    n = m < n ? (m > 0 ? m : 0) : n;
  }
  // PW: tiles are pixel tiles of this workgroup's part; else (pixel tile, part) pairs
  const int64_t P = n * Gm::PIX, tiles = (P + TP - 1) / TP * (PW ? 1 : NS), tstride = wgs * WAVES;
  constexpr int TD = PW ? 1 : NS;  // tile -> pixel tile divisor

  // this lane's window origin in tile t, per M-block (tail lanes read a duplicate pixel)
  auto bases = [&](int64_t t, const uint8_t *(&out)[MB]) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      int64_t p = t * TP + mb * 16 + mr;
      if (p >= P) p = P - 1;
      const int64_t b = p / Gm::PIX;
      const int pp = (int)(p % Gm::PIX), oy = pp / Gm::WOUT, ox = pp % Gm::WOUT;
      if constexpr (F32) {
        out[mb] = reinterpret_cast<const uint8_t *>(static_cast<const float *>(x) +
                                                    ((b * HIN + S * oy) * WIN + S * ox) * CIN + 4 * q);
      } else {
        const int64_t row = rows ? rows[b] : b;
        out[mb] = static_cast<const uint8_t *>(x) + row * Gm::STACK + (int64_t)(S * oy + (q >> 1)) * WIN + S * ox +
                  4 * (q & 1);
      }
    }
  };
  // byte offset of chunk g inside the window: f32 = kh rows of KW*CIN floats in 16-float
  // chunks; u8 = runs 2g, 2g+1 = (ci, kh), (ci, kh+1) with ci = 2g / KH, kh = 2g % KH
  auto chunk_off = [](int g) -> int {
    if constexpr (F32) {
      constexpr int RC = KW * CIN / 16;
      return 4 * ((g / RC) * WIN * CIN + (g % RC) * 16);
    } else {
      return ((2 * g) / KH) * HIN * WIN + ((2 * g) % KH) * WIN;
    }
  };
  auto ld = [](const uint8_t *p) { return *reinterpret_cast<const Frag *>(p); };

  // wave slots are numbered SIMD-major (waves w and w + 4 of a workgroup share a SIMD): the
  // first gridDim.x * 4 slots put one wave on every SIMD, so a partial last round of tiles
  // lands on distinct SIMDs and no SIMD runs more than ceil(tiles / SIMDs) tiles
  const int64_t slot = WAVES % 4 == 0 ? (int64_t)(wave / 4) * wgs * 4 + wgi * 4 + wave % 4 : wgi * WAVES + wave;
  // Units (r05, TS > 1: NS == 1, no PW): the pixel tiles of the whole rounds -- as many as
  // give every SIMD the same count -- run full-width; each pixel tile of the ragged last round
  // is split into TS channel parts (NB / TS blocks each), which the slots continue to take in
  // the same order, so they land on the SIMDs with one tile less: at 1,024 samples the 5,184
  // tiles were 5 or 6 per SIMD, now 5 + at most one quarter.  Same MFMA chain per output.
  const int64_t ptiles = (P + TP - 1) / TP;
  const int64_t per_round = WAVES % 4 == 0 ? wgs * 4 : tstride;  // one slot per SIMD
  const int64_t full = TS > 1 ? ptiles / per_round * per_round : tiles;
  const int64_t total = TS > 1 ? full + (ptiles - full) * TS : tiles;
  auto unit_ptile = [&](int64_t v) -> int64_t { return TS > 1 ? (v < full ? v : full + (v - full) / TS) : v / TD; };
  auto unit_nb0 = [&](int64_t v) -> int {
    if constexpr (TS > 1) return v < full ? 0 : (int)((v - full) % TS) * (NB / TS);
    return PW ? part * NBW : (NS == 1 ? 0 : (int)(v % NS) * NBW);
  };
  // the first tile's leading input chunks are requested before the weights are staged
  int64_t v = slot;
  const uint8_t *cur[MB], *nxt[MB];
  bases(unit_ptile(v < total ? v : total - 1), cur);
  Frag ar[D][MB];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) ar[d][mb] = ld(cur[mb] + chunk_off(d));

  // stage the packed weights (rth_conv_pack: already in fragment order): a coalesced copy,
  // consecutive threads -> consecutive 16-byte LDS slots; all loads first
  {
    constexpr int PER = (LDSW + T - 1) / T;
    const f32x4 *wp = reinterpret_cast<const f32x4 *>(w);
    // PW: LDS slot (g * NBW + nbl) * 64 + lane <- packed slot (g * NB + part * NBW + nbl) * 64 + lane
    auto src = [&](int sl) { return PW ? ((sl / (NBW * 64)) * NB + part * NBW) * 64 + sl % (NBW * 64) : sl; };
    f32x4 tmp[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int sl = threadIdx.x + j * T;
      if (sl < LDSW) tmp[j] = wp[src(sl)];
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int sl = threadIdx.x + j * T;
      if (sl < LDSW) wl[sl] = tmp[j];
    }
  }
  __syncthreads();

  float bl[NBW];  // the full-width units' bias (their channel part is fixed unless NS > 1)
  const int nb_first = unit_nb0(v);
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) bl[nb] = bias[(nb_first + nb) * 16 + mr];
  // this lane's B fragments, offset to the tile's channel part
  const f32x4 *wlane = wl + lane;

  // one unit: NBT channel blocks from nb0 of pixel tile ptile (nxt: the next unit's window)
  auto run = [&](auto nbt, int64_t ptile, int nb0) __attribute__((always_inline)) {
    constexpr int NBT = decltype(nbt)::value;
    const int lb0 = PW ? 0 : nb0;  // its LDS block
    float bt[NBT];
    if constexpr (NBT != NBW || (NS > 1 && !PW)) {
#pragma unroll
      for (int nb = 0; nb < NBT; ++nb) bt[nb] = bias[(nb0 + nb) * 16 + mr];
    } else {
#pragma unroll
      for (int nb = 0; nb < NBT; ++nb) bt[nb] = bl[nb];
    }
    f32x4 acc[MB][NBT];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NBT; ++nb) acc[mb][nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 bcur[NBT], bnxt[NBT];  // B fragments, one chunk ahead
    constexpr int LNB = PW ? NBW : NB;  // channel blocks per chunk in LDS
#pragma unroll
    for (int nb = 0; nb < NBT; ++nb) bcur[nb] = wlane[(lb0 + nb) * 64];

#pragma unroll 1
    for (int g0 = 0; g0 < G; g0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int g = g0 + d;
        const int gb = g + 1 < G ? g + 1 : G - 1;
#pragma unroll
        for (int nb = 0; nb < NBT; ++nb) {
#ifdef RTH_DIAG_NOLDSB  // diagnostic timing builds only (scripts/r05.sh c2diag): wrong results
          bnxt[nb] = bcur[nb];
#else
          bnxt[nb] = wlane[(gb * LNB + lb0 + nb) * 64];
#endif
        }
        // keep the next chunk's B reads here, a whole chunk of MFMAs ahead of their use
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            float a;
            if constexpr (F32) a = ar[d][mb][t];
            else a = (float)((ar[d][mb] >> (8 * t)) & 0xffu);
#pragma unroll
            for (int nb = 0; nb < NBT; ++nb)
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bcur[nb][t], acc[mb][nb], 0, 0, 0);
          }
        const int ga = g + D;
#ifndef RTH_DIAG_NOLOADA
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          ar[d][mb] = ld(ga < G ? cur[mb] + chunk_off(ga) : nxt[mb] + chunk_off(ga - G));
#endif
#pragma unroll
        for (int nb = 0; nb < NBT; ++nb) bcur[nb] = bnxt[nb];
      }
    }
    // C/D: lane holds column mr of rows 4q .. 4q+3 of each M-block; y is NHWC, or NCHW when
    // out_nchw (the last conv feeding FC1 in the reference's (C, H, W) flatten order)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t po = ptile * TP + mb * 16 + 4 * q + i;
#ifdef RTH_DIAG_NOEPI
        if (po < P && acc[mb][0][i] == 12345.678f) {
#else
        if (po < P) {
#endif
          if (out_nchw) {
            const int64_t b = po / Gm::PIX, pp = po - b * Gm::PIX;
#pragma unroll
            for (int nb = 0; nb < NBT; ++nb)
              y[(b * COUT + (nb0 + nb) * 16 + mr) * Gm::PIX + pp] = relu_c(radd(acc[mb][nb][i], bt[nb]));
          } else {
#pragma unroll
            for (int nb = 0; nb < NBT; ++nb)
              y[po * COUT + (nb0 + nb) * 16 + mr] = relu_c(radd(acc[mb][nb][i], bt[nb]));
          }
        }
      }
  };

  for (; v < total;) {
    const int64_t vn = v + tstride;
    // the chunks past the end of this unit are the next unit's leading chunks
    bases(unit_ptile(vn < total ? vn : v), nxt);
    if (TS > 1 && v >= full)
      run(std::integral_constant<int, (TS > 1 ? NB / TS : NBW)>{}, unit_ptile(v), unit_nb0(v));
    else
      run(std::integral_constant<int, NBW>{}, unit_ptile(v), unit_nb0(v));
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) cur[mb] = nxt[mb];
    v = vn;
  }
#ifdef RTH_CLOCK_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < kClockSlots) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), wall1 = __builtin_amdgcn_s_memrealtime();
    g_conv_clock[blockIdx.x][0] = clk1 - clk0;
    g_conv_clock[blockIdx.x][1] = wall1 - wall0;
  }
#endif
}

// ---------------------------------------------------------------------------------------
// conv1 on uint8 stacks on the bf16 MFMA with an exact three-term weight split.
// A byte is exact in bf16, and every fp32 weight is the exact sum w1 + w2 + w3 of three
// bf16 values (w1 = bf16(w), w2 = bf16(w - w1), w3 = w - w1 - w2: 8 + 8 + 8 of the 24
// significand bits), so every product x * wi is exact in fp32 and
//     y = sum_k x_k * w_k = sum_k x_k * w1_k + x_k * w2_k + x_k * w3_k
// is the same sum of exact products as the fp32 path, accumulated in fp32 in a different
// order (3 x K terms instead of K).  Nothing is computed at reduced precision; the rate is
// three bf16 MFMAs per fp32 MFMA's work at 16x the per-clock rate.
// Tile: v_mfma_f32_32x32x16_bf16 with A = the weights (32 output channels x 16 k), B = 32
// output pixels' input windows: lane (r, h) = (lane & 31, lane >> 5) holds k = 8h .. 8h+7 of
// chunk c = run (ci, kh) = 2c + h of pixel r -- 8 consecutive bytes of one stack row -- and
// the same k of output channel r's weights.  A wave keeps all of W (16 chunks x 3 terms,
// 192 VGPRs) in registers for its whole life, so the kernel uses no LDS and leaves the CU's
// LDS to the learner's kernels; it loads the next tile's windows while it multiplies this one.
constexpr int kC1Chunks = 16;                       // K = 256 = 16 chunks of 16
constexpr int kC1PackedBytes = kC1Chunks * 3 * 64 * 16;  // [chunk][term][lane] x 8 bf16
#ifndef C1_NBUF
#define C1_NBUF 3
#endif
constexpr int kC1Buf = C1_NBUF;  // tiles whose windows are in flight (the computed one included)


// term t (0, 1, 2) of the exact split of w
__device__ __forceinline__ uint32_t bf16x3_term(float w, int t) {
  const uint32_t h1 = bf16_rne_bits(w);
  const float r1 = rsub(w, bf16_bits_f(h1));
  const uint32_t h2 = bf16_rne_bits(r1);
  const float r2 = rsub(r1, bf16_bits_f(h2));
  return t == 0 ? h1 : (t == 1 ? h2 : bf16_rne_bits(r2));
}

// packed slot sl = (c * 3 + t) * 64 + lane: the 8 bf16 of lane (r, h) for chunk c, term t
// from W in OHWI storage: k = 8h + j of chunk c is (ci, kh) = run 2c + h, kw = j
__device__ __forceinline__ void pack_conv1_bf16x3(const float *__restrict__ w, u32x4 *__restrict__ packed, int sl) {
  if (sl >= kC1PackedBytes / 16) return;
  const int lane = sl % 64, t = (sl / 64) % 3, c = sl / 192;
  const int co = lane & 31, rho = 2 * c + (lane >> 5), ci = rho >> 3, kh = rho & 7;
  float wv[8];  // every load before the first split (the split's branches kept them one at a time)
#pragma unroll
  for (int j = 0; j < 8; ++j) wv[j] = w[((co * 8 + kh) * 8 + j) * 4 + ci];
  uint32_t e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = bf16x3_term(wv[j], t);
  packed[sl] = u32x4{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
}

// 8 bytes (kw 0..7 of one stack row) -> 8 bf16 (exact: a byte has <= 8 significant bits)
__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint32_t lo, uint32_t hi) {
  auto two = [](uint32_t v, int s) -> uint32_t {
    const uint32_t a = __float_as_uint((float)((v >> s) & 0xffu));
    const uint32_t b = __float_as_uint((float)((v >> (s + 8)) & 0xffu));
    return __builtin_amdgcn_perm(b, a, 0x07060302u);  // {a.hi16, b.hi16}
  };
  return __builtin_bit_cast(bf16x8, (u32x4{two(lo, 0), two(lo, 16), two(hi, 0), two(hi, 16)}));
}

__global__ __launch_bounds__(256) void k_conv1_u8_bf16x3(const void *__restrict__ x, const int64_t *__restrict__ rows,
                                                       int64_t n, const int64_t *__restrict__ n_dev,
                                                       const float *__restrict__ w, const float *__restrict__ bias,
                                                       float *__restrict__ y) {
  constexpr int HIN = 84, WIN = 84, WOUT = 20, PIX = 400, S = 4, COUT = 32;
  constexpr int64_t STACK = 4 * HIN * WIN;
  using f32x16 = __attribute__((ext_vector_type(16))) float;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar tile math
  const int r = lane & 31, h = lane >> 5;
  if (n_dev) {  // a device-side sample count (<= n): rows past it are neither read nor written
    const int64_t m = *n_dev;
    n = m < n ? (m > 0 ? m : 0) : n;
  }
  const int64_t P = n * PIX, tiles = (P + 31) / 32, tstride = (int64_t)gridDim.x * 4;
  int64_t tile = (int64_t)blockIdx.x * 4 + wave;
  if (tile >= tiles) return;  // no barriers below: a wave without tiles just leaves
  const uint8_t *xb = static_cast<const uint8_t *>(x);
  // pixel r of tile t (tail: a duplicate pixel).  A tile spans at most two samples b0, b0+1:
  // their row indices are scalar loads (lgkmcnt), so computing a window never waits for the
  // vector loads of the tiles already in flight
  auto window = [&](int64_t t) -> const uint8_t * {
    const int64_t t32 = t * 32, b0 = t32 / PIX;
    int pp = (int)(t32 - b0 * PIX) + r;
    int64_t b = b0;
    if (pp >= PIX) {
      pp -= PIX;
      b = b0 + 1;
    }
    if (b >= n) {
      b = n - 1;
      pp = PIX - 1;
    }
    int64_t row = b;
    if (rows) {
      const int64_t r0 = rows[b0], r1 = rows[b0 + 1 < n ? b0 + 1 : b0];
      row = b == b0 ? r0 : r1;
    }
    const int oy = pp / WOUT, ox = pp % WOUT;
    return xb + row * STACK + (S * oy) * WIN + S * ox;
  };
  // this lane's run of chunk c: (ci, kh) = (2c + h) >> 3, (2c + h) & 7
  auto run_off = [&](int c) -> int {
    const int rho = 2 * c + h;
    return (rho >> 3) * HIN * WIN + (rho & 7) * WIN;
  };
  const u32x4 *wp = reinterpret_cast<const u32x4 *>(w);
  bf16x8 wf[kC1Chunks][3];
#pragma unroll
  for (int c = 0; c < kC1Chunks; ++c)
#pragma unroll
    for (int t = 0; t < 3; ++t) wf[c][t] = __builtin_bit_cast(bf16x8, wp[(c * 3 + t) * 64 + lane]);
  float bl[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) bl[i] = bias[(i & 3) + 8 * (i >> 2) + 4 * h];

  uint32_t raw[kC1Buf][kC1Chunks][2];  // a ring of tiles in flight
  auto load = [&](uint32_t (&dst)[kC1Chunks][2], int64_t t) {
    const uint8_t *p = window(t);
#pragma unroll
    for (int c = 0; c < kC1Chunks; ++c) {
      const uint8_t *q = p + run_off(c);
      dst[c][0] = *reinterpret_cast<const uint32_t *>(q);
      dst[c][1] = *reinterpret_cast<const uint32_t *>(q + 4);
    }
  };
  auto compute = [&](const uint32_t (&src)[kC1Chunks][2], int64_t t) {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
#pragma unroll
    for (int c = 0; c < kC1Chunks; ++c) {
      const bf16x8 xf = u8x8_to_bf16(src[c][0], src[c][1]);
#pragma unroll
      for (int tm = 0; tm < 3; ++tm) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[c][tm], xf, acc, 0, 0, 0);
    }
    // C/D: lane holds pixel r, channels (i & 3) + 8 (i >> 2) + 4h of register i.  Tail lanes
    // computed the last pixel's window and store the same bytes to it: no branch around the
    // stores, so the compiler can count the loads in flight exactly (no vmcnt(0) per tile)
    int64_t p = t * 32 + r;
    if (p >= P) p = P - 1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 o;
      o.x = relu_c(radd(acc[4 * g + 0], bl[4 * g + 0]));
      o.y = relu_c(radd(acc[4 * g + 1], bl[4 * g + 1]));
      o.z = relu_c(radd(acc[4 * g + 2], bl[4 * g + 2]));
      o.w = relu_c(radd(acc[4 * g + 3], bl[4 * g + 3]));
      *reinterpret_cast<float4 *>(y + p * COUT + 8 * g + 4 * h) = o;
    }
  };
  // loads are unconditional (past the last tile: the last tile again) for the same reason
#pragma unroll
  for (int i = 0; i + 1 < kC1Buf; ++i) load(raw[i], tile + i * tstride < tiles ? tile + i * tstride : tiles - 1);
  for (;;) {
#pragma unroll
    for (int i = 0; i < kC1Buf; ++i) {
      const int64_t ahead = tile + (kC1Buf - 1) * tstride;
      load(raw[(i + kC1Buf - 1) % kC1Buf], ahead < tiles ? ahead : tiles - 1);
      compute(raw[i], tile);
      tile += tstride;
      if (tile >= tiles) return;
    }
  }
}

// conv1 with each stack byte converted once per horizontal window pair (r05).  Horizontally
// adjacent output pixels' windows overlap by half (kernel 8, stride 4): kw 4..7 of pixel ox are
// kw 0..3 of pixel ox + 1.  So a lane loads and converts only the first half (4 bytes) of each
// of its 16 runs and takes the second half, already converted, from the next lane (DPP
// wave_shl:1).  For that the lanes walk VIRTUAL pixels: 21 per output row, the 21st (ox = 20,
// input columns 80..83: inside the 84-wide row) exists only to hand its first halves to ox = 19,
// and each 32-lane tile covers 31 virtual pixels, its lane 31 being the next one, a helper for
// lane 30 (wave_shl:1 moves lane 32 into lane 31: the helper's own second half is garbage, and it
// stores nothing).  Same packed weights, same k order (kw 0..7 of run (ci, kh)), same MFMA
// chain per output as k_conv1_u8_bf16x3: the outputs are bit-identical.  Half the byte loads and
// conversions per tile; 29.5 of 32 lanes produce an output (20 / 21 x 31 / 32).
constexpr int kC1VPix = 21;       // virtual pixels per output row
constexpr int kC1VPerTile = 31;   // virtual pixels a 32-lane tile outputs
#ifndef C1_NBUF_SHARE
#define C1_NBUF_SHARE 2  // r05 A/B: 2 tiles in flight 26.0 us alone at 1,024 samples, 3: 27.3, 1: 30.7
#endif
constexpr int kC1BufShare = C1_NBUF_SHARE;  // tiles in flight (16 dwords each)

// 4 bytes (kw 0..3 of one stack row) -> 4 bf16 in two dwords (exact)
__device__ __forceinline__ void u8x4_to_bf16(uint32_t v, uint32_t &lo, uint32_t &hi) {
  const uint32_t a = __float_as_uint((float)(v & 0xffu)), b = __float_as_uint((float)((v >> 8) & 0xffu));
  const uint32_t c = __float_as_uint((float)((v >> 16) & 0xffu)), d = __float_as_uint((float)(v >> 24));
  lo = __builtin_amdgcn_perm(b, a, 0x07060302u);
  hi = __builtin_amdgcn_perm(d, c, 0x07060302u);
}

__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {  // lane i <- lane i + 1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130 /* wave_shl:1 */, 0xf, 0xf, false);
}

__device__ unsigned char g_conv1_sink[64 * 128];  // stores of lanes without an output (never read)

// FRM (r05): x is a replay's frame store (84 x 84-byte frames) and fids[b] the 4 frame ids of
// sample b's stack (the sampled rows' id tuples, rth_replay_sample_frame_ids): each run
// (ci, kh) is read from frame fids[b][ci] -- the bytes the gather would have assembled, so the
// outputs are bit-identical, without the batch copy of the stacks
constexpr int64_t kC1FrameBytes = 84 * 84;
template <bool FRM = false>
__global__ __launch_bounds__(256) void k_conv1_u8_share(const void *__restrict__ x, const int64_t *__restrict__ rows,
                                                      int64_t n, const int64_t *__restrict__ n_dev,
                                                      const float *__restrict__ w, const float *__restrict__ bias,
                                                      float *__restrict__ y, const int32_t *__restrict__ fids) {
  constexpr int HIN = 84, WIN = 84, WOUT = 20, PIX = 400, S = 4, COUT = 32;
  constexpr int VPS = WOUT * kC1VPix;  // 420 virtual pixels per sample
  constexpr int64_t STACK = 4 * HIN * WIN;
  using f32x16 = __attribute__((ext_vector_type(16))) float;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  if (n_dev) {
    const int64_t m = *n_dev;
    n = m < n ? (m > 0 ? m : 0) : n;
  }
  // 32-bit pixel arithmetic: the launcher requires n * 420 < 2^31
  const int VP = (int)n * VPS, tiles = (VP + kC1VPerTile - 1) / kC1VPerTile, tstride = (int)gridDim.x * 4;
  int tile = (int)blockIdx.x * 4 + wave;
  if (tile >= tiles) return;  // no barriers below
  const uint8_t *xb = static_cast<const uint8_t *>(x);
  // virtual pixel r of tile t: (sample, oy, ox in 0..20); past the end: the last one
  auto vpix = [&](int t, int &b, int &oy, int &ox) {
    int v = t * kC1VPerTile + r;
    if (v >= VP) v = VP - 1;
    b = (int)((unsigned)v / (unsigned)VPS);
    const int rem = v - b * VPS;
    oy = rem / kC1VPix;
    ox = rem - oy * kC1VPix;
  };
  auto window = [&](int t) -> const uint8_t * {
    int b, oy, ox;
    vpix(t, b, oy, ox);
    const int64_t row = rows ? rows[b] : b;
    return xb + row * STACK + ((S * oy) * WIN + S * ox);
  };
  auto run_off = [&](int c) -> int {
    const int rho = 2 * c + h;
    return (rho >> 3) * HIN * WIN + (rho & 7) * WIN;
  };
  const u32x4 *wp = reinterpret_cast<const u32x4 *>(w);
  bf16x8 wf[kC1Chunks][3];
#pragma unroll
  for (int c = 0; c < kC1Chunks; ++c)
#pragma unroll
    for (int t = 0; t < 3; ++t) wf[c][t] = __builtin_bit_cast(bf16x8, wp[(c * 3 + t) * 64 + lane]);
  // (the bias is re-read per tile from L1 / L2 in the epilogue: 16 registers fewer than
  // r04's kernel keeps, which spilled its weights into AGPRs)
  const float4 *bias4 = reinterpret_cast<const float4 *>(bias) + h;

  constexpr int NB = kC1BufShare;
  uint32_t raw[NB][kC1Chunks];  // the first halves of the runs, a ring of tiles in flight
  auto load = [&](uint32_t (&dst)[kC1Chunks], int t) {
    if constexpr (FRM) {
      int b, oy, ox;
      vpix(t, b, oy, ox);
      // a tile's 32 virtual pixels span at most two samples (420 per sample): their id tuples
      // are wave-uniform scalar loads (lgkmcnt: a vector load here would be the newest in the
      // vmcnt queue, and waiting for it would drain the ring of tiles in flight)
      const int tu = __builtin_amdgcn_readfirstlane(t);
      const int v0 = tu * kC1VPerTile, v1 = v0 + kC1VPerTile - 1 < VP ? v0 + kC1VPerTile - 1 : VP - 1;
      const int b0 = (int)((unsigned)v0 / (unsigned)VPS), b1 = (int)((unsigned)v1 / (unsigned)VPS);
      const int4 i0 = reinterpret_cast<const int4 *>(fids)[b0], i1 = reinterpret_cast<const int4 *>(fids)[b1];
      const bool second = b != b0;
      const int4 id = {second ? i1.x : i0.x, second ? i1.y : i0.y, second ? i1.z : i0.z, second ? i1.w : i0.w};
      const int off = (S * oy) * WIN + S * ox;
      const uint8_t *fb[4] = {xb + (int64_t)id.x * kC1FrameBytes + off, xb + (int64_t)id.y * kC1FrameBytes + off,
                              xb + (int64_t)id.z * kC1FrameBytes + off, xb + (int64_t)id.w * kC1FrameBytes + off};
#pragma unroll
      for (int c = 0; c < kC1Chunks; ++c) {
        const int rho = 2 * c + h;  // run (ci, kh) = (rho / 8, rho % 8): h picks the odd / even runs
        dst[c] = *reinterpret_cast<const uint32_t *>(fb[(2 * c) >> 3] + (rho & 7) * WIN);
      }
    } else {
      const uint8_t *p = window(t);
#pragma unroll
      for (int c = 0; c < kC1Chunks; ++c) dst[c] = *reinterpret_cast<const uint32_t *>(p + run_off(c));
    }
  };
  auto compute = [&](const uint32_t (&src)[kC1Chunks], int t) {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
#pragma unroll
    for (int c = 0; c < kC1Chunks; ++c) {
      uint32_t lo, hi;
      u8x4_to_bf16(src[c], lo, hi);
      const uint32_t lo2 = from_next_lane(lo), hi2 = from_next_lane(hi);  // kw 4..7 = the next pixel's kw 0..3
      const bf16x8 xf = __builtin_bit_cast(bf16x8, (u32x4{lo, hi, lo2, hi2}));
#pragma unroll
      for (int tm = 0; tm < 3; ++tm) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[c][tm], xf, acc, 0, 0, 0);
    }
    // lane r holds virtual pixel r's outputs; virtual column 20, the helper lane 31 and lanes
    // past the end store into the sink (no branch around the stores)
    int b, oy, ox;
    vpix(t, b, oy, ox);
    const bool out = r < kC1VPerTile && ox < WOUT && t * kC1VPerTile + r < VP;
    float *dst = out ? y + ((int64_t)b * PIX + oy * WOUT + ox) * COUT
                     : reinterpret_cast<float *>(g_conv1_sink) + lane * 32;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bv = bias4[2 * g];  // channels 8g + 4h .. + 3
      float4 o;
      o.x = relu_c(radd(acc[4 * g + 0], bv.x));
      o.y = relu_c(radd(acc[4 * g + 1], bv.y));
      o.z = relu_c(radd(acc[4 * g + 2], bv.z));
      o.w = relu_c(radd(acc[4 * g + 3], bv.w));
      *reinterpret_cast<float4 *>(dst + 8 * g + 4 * h) = o;
    }
  };
#pragma unroll
  for (int i = 0; i + 1 < NB; ++i) load(raw[i], tile + i * tstride < tiles ? tile + i * tstride : tiles - 1);
  for (;;) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int ahead = tile + (NB - 1) * tstride;
      load(raw[(i + NB - 1) % NB], ahead < tiles ? ahead : tiles - 1);
      compute(raw[i], tile);
      tile += tstride;
      if (tile >= tiles) return;
    }
  }
}

__global__ __launch_bounds__(256) void k_conv1_pack_bf16x3(const float *__restrict__ w, u32x4 *__restrict__ packed) {
  pack_conv1_bf16x3(w, packed, blockIdx.x * 256 + threadIdx.x);
}

// ---------------------------------------------------------------------------------------
// conv2 / conv3 forward (f32 NHWC input) on the bf16 MFMA with an exact 3 x 3-term split of
// BOTH operands.  Every fp32 value v is the exact sum v1 + v2 + v3 of three bf16 values (the
// round-to-nearest split of bf16x3_term: 8 + 8 + 8 of the 24 significand bits, each residual
// exact), so for an input x and a weight w
//     x * w = sum_{i,j in 1..3} xi * wj
// and every partial product xi * wj has at most 16 significant bits: it is exact in the fp32
// accumulator.  The nine bf16 MFMAs per fp32 product therefore sum exactly the same real
// products as the fp32 MFMA's fmaf chain, accumulated in fp32 in a different order (9K terms
// instead of K) -- the difference is summation order, as between any two fp32 GEMM tilings,
// not precision.  (Bounded-exponent caveat: a term below 2^-126 would be a bf16 subnormal;
// activations and weights of the DQN are many orders of magnitude away from that.)  Rate: 9
// v_mfma_f32_16x16x32_bf16 (16 cycles each) do the work of 8 v_mfma_f32_16x16x4_f32 (32
// cycles each): 144 vs 256 matrix-pipe cycles per 16 x 16 x 32 block, 1.78x.
//
// Workgroup = 8 waves over NSAMP (runtime nsamp <= NSAMP) samples: the samples' input is
// split once into the three bf16 planes in LDS ([term][ci / 8][pixel] 16-byte units, pixel
// rows rotated within 16-row blocks against bank conflicts); wave w owns output channels
// 16 (w & 3) .. +15 and K half w >> 2 (its B fragments -- all three weight terms of its K half,
// NCH / 2 chunks x 3 x 8 bf16 -- live in registers for the whole launch); every wave walks all
// M-tiles of 16 output pixels of the workgroup's samples.  The two K halves meet in LDS
// (fixed order: first half + second half, then + bias, ReLU), and the output leaves as one
// contiguous run per workgroup (NHWC, or NCHW for FC1) in 16-byte stores.
template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NSAMP, int ROT, int KS, int COUT_ = 64>
struct X9Geom {
  static constexpr int COUT = COUT_, HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int NCB = COUT / 16;                                   // channel blocks (waves per K part)
  static constexpr int K = KH * KW * CIN, NCH = K / 32, NCHP = NCH / KS;  // 32-deep chunks, per K part
  static constexpr int NT = 64 * NCB * KS;                                // threads: NCB channel blocks x KS
  static constexpr int TILES = (NSAMP * PIX + 15) / 16;                  // 16-pixel M-tiles
  static constexpr int NG = CIN / 8;                                     // 16-byte ci groups
  static constexpr int ROWS = NSAMP * HIN * WIN;                         // staged input pixels
  // ROT = rotation | (shift << 4) | (pad << 8): the staged row r goes to unit (r & ~15) |
  // ((r + (r >> shift) * rotation) & 15) of its plane (shift 0 = 5), planes padded by `pad`
  // units (0 = the r03 rule: 1 at rotation 10) -- scripts/x9_lds_sim.py searches these
  static constexpr int ROTV = ROT & 15, SHV = ((ROT >> 4) & 15) ? ((ROT >> 4) & 15) : 5;
  static constexpr int PADV = (ROT >> 8) ? (ROT >> 8) : (ROT == 10 ? 1 : 0);
  static constexpr int PLANE = (ROWS + 15) / 16 * 16 + PADV;  // 16-B units per (term, cg)
  static_assert(SHV >= 4, "the rotation must be constant over each aligned 16-row block (a permutation)");
  static constexpr int LDS_U4 = 3 * NG * PLANE;                          // LDS in 16-B units
  static constexpr int OUT_F = NSAMP * COUT * PIX;                       // output staging floats
  static constexpr int PACKED_U4 = (COUT / 16) * NCH * 3 * 64;           // packed weight fragments
  static_assert(CIN % 32 == 0 || 32 % CIN == 0, "a 32-deep chunk must stay inside one tap");
  static_assert(CIN % 8 == 0 && NCH % KS == 0 && KS >= 1 && KS <= 4, "K must split into KS parts of 32-deep chunks");
  static_assert(COUT % 16 == 0 && NT <= 1024, "16-channel blocks, at most 16 waves");
  static_assert(OUT_F * 4 <= LDS_U4 * 16, "output staging must fit the input image");
  static_assert(LDS_U4 * 16 <= 163840, "LDS image too large");
  __device__ static int swz(int r) { return (r & ~15) | ((r + (r >> SHV) * ROTV) & 15); }
};

// PAD > 0 (the data gradient, rth_conv_dgrad): the staged HIN x WIN image is the input
// zero-padded by PAD on every side -- x is [n, HIN - 2 PAD, WIN - 2 PAD, CIN], the border reads
// zero through the buffer resource's range check --, and bias == NULL writes the raw sums (no
// bias, no ReLU).  CLS (conv2's data gradient, one launch for the 4 stride-parity classes):
// blockIdx.y = class (py, px), its packed kernel at wpk + class * PACKED_U4, and output pixel
// (jy, jx) of the class goes to pixel (2 jy + py, 2 jx + px) of the [n, 2 HOUT, 2 WOUT, COUT]
// NHWC gradient.
// MASK (r05, the data gradient of conv3 only: PAD > 0, no CLS): the output is the gradient of
// the layer below's ReLU output, passed through that ReLU at once -- y = 0 where ymask (the
// layer below's output, same NHWC index space) is <= 0, threshold_backward -- and each
// workgroup writes the layer below's bias-gradient partial sums (slab blockIdx.x: float4 of
// channels 4q.. per quad q, each lane's float4s in order, then a fixed LDS tree over the lanes of
// a quad -- k_relu_bias_grad's slab layout, finished by the same deferred bias job).  This
// replaces rth_relu_bias_grad's launch between the two data gradients.
template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NSAMP, int ROT, int KS, int PAD = 0, int COUT_ = 64,
          int CLS = 0, int MASK = 0>
__global__ __launch_bounds__(64 * (COUT_ / 16) * KS) void k_conv_x9(const float *__restrict__ x, int64_t n,
                                                                  const int64_t *__restrict__ n_dev, int nsamp,
                                                                  const u32x4 *__restrict__ wpk,
                                                                  const float *__restrict__ bias,
                                                                  float *__restrict__ y, int out_nchw,
                                                                  const float *__restrict__ ymask,
                                                                  float *__restrict__ bpart) {
  static_assert(!MASK || (PAD > 0 && !CLS && (64 * (COUT_ / 16) * KS) % (COUT_ / 4) == 0),
                "the masked epilogue is the NHWC data gradient's; every lane keeps one channel quad");
  using G = X9Geom<KH, KW, S, CIN, HIN, WIN, NSAMP, ROT, KS, COUT_>;
  if constexpr (CLS) wpk += (size_t)blockIdx.y * G::PACKED_U4;
  constexpr int HS = HIN - 2 * PAD, WS = WIN - 2 * PAD;  // the source image
  constexpr int PIX = G::PIX, NCH2 = G::NCHP, NG = G::NG, PLANE = G::PLANE, COUT = G::COUT, NT = G::NT;
  __shared__ uint4 lds[G::LDS_U4];
  if (n_dev) {
    const int64_t m = *n_dev;
    n = m < n ? (m > 0 ? m : 0) : n;
  }
  (void)nsamp;  // == NSAMP: the host launches the instantiation for the samples per workgroup
  const int64_t b0 = (int64_t)blockIdx.x * NSAMP;
  if (b0 >= n) return;  // the whole workgroup leaves: no barrier is reached
  const int ns = (int)(n - b0 < NSAMP ? n - b0 : NSAMP);
  const int nv = ns * PIX;  // valid output pixels
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave % G::NCB, half = wave / G::NCB;  // channel block, K part

  // this wave's B fragments: channels 16 cb + (lane & 15), chunks [half * NCH2, +NCH2), 3 terms
  bf16x8 wf[NCH2][3];
  {
    const u32x4 *wp = wpk + ((size_t)(cb * G::NCH + half * NCH2) * 3) * 64 + lane;
#pragma unroll
    for (int c = 0; c < NCH2; ++c)
#pragma unroll
      for (int t = 0; t < 3; ++t) wf[c][t] = __builtin_bit_cast(bf16x8, wp[(c * 3 + t) * 64]);
  }
  // Staging: the samples' input split into the three bf16 planes, float4 (4 ci of one pixel)
  // -> 8 bytes in each plane, unit (t * NG + ci / 8) * PLANE + swz(pixel), half (ci % 8) / 4.
  // Lane l of a wave-instruction takes pixel 16 k + (l & 15), ci group 4 j + (l >> 4): each
  // 16-lane LDS write group spans 16 pixels of one ci group (distinct banks); each pixel's 64
  // loaded bytes are contiguous in global memory.  Two phases: the first half of the samples is
  // staged, then the second half's loads are issued and the tiles of the first half computed
  // while they are in flight; the second half is written to LDS after them.
  constexpr int CB = CIN / 16;                       // 4-ci groups per lane quarter
  constexpr int NA = NSAMP > 1 ? NSAMP / 2 : NSAMP;  // samples in phase A
  constexpr int RA = NA * HIN * WIN;                 // staged pixels of phase A
  constexpr int SA = (RA + 15) / 16 * CB * 64;       // lane slots of phase A
  constexpr int RB_ = (NSAMP - NA) * HIN * WIN;      // ... of phase B
  constexpr int SB = (RB_ + 15) / 16 * CB * 64;
  constexpr int UA = (SA + NT - 1) / NT, UB = SB > 0 ? (SB + NT - 1) / NT : 1;
  const int rows = ns * HIN * WIN;
  auto slot_of = [&](int i, int r0, int &rr, int &c4) {
    const int l = i & 63, blk = i >> 6;
    rr = r0 + (blk / CB) * 16 + (l & 15);
    c4 = (blk % CB) * 4 + (l >> 4);
  };
  // the staging loads go through a buffer resource over the n samples: a slot past the staged
  // rows gets an offset beyond its range and reads zeros, so no load sits under a branch (a
  // "cond ? load : 0" made the compiler wait for each load before issuing the next: the
  // phase-B loads went out one at a time)
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(x), 0, (int)(n * (int64_t)(HS * WS * CIN) * 4), 0x00020000);
  const uint32_t xb0 = (uint32_t)(b0 * (int64_t)(HS * WS * CIN) * 4);
  auto fetch = [&](int i, int r0, int rend) -> float4 {
    int rr, c4;
    slot_of(i, r0, rr, c4);
    bool ok = rr < rend && rr < rows;
    int src = rr;
    if constexpr (PAD > 0) {  // staged pixel -> source pixel; the border reads zero
      const int s = rr / (HIN * WIN), rem = rr - s * (HIN * WIN), yy = rem / WIN - PAD, xx = rem % WIN - PAD;
      ok = ok && yy >= 0 && yy < HS && xx >= 0 && xx < WS;
      src = (s * HS + yy) * WS + xx;
    }
    const uint32_t off = ok ? xb0 + (uint32_t)((src * (CIN / 4) + c4) * 16) : 0x80000000u;
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(x_rsrc, off, 0, 0));
  };
  auto commit = [&](float4 v, int i, int r0, int rend) {
    int rr, c4;
    slot_of(i, r0, rr, c4);
    if (rr >= rend || rr >= rows) return;
    uint2 tr[3];
    split3_x4(v, tr);
    uint2 *l2 = reinterpret_cast<uint2 *>(lds);
    const int unit = (c4 >> 1) * PLANE + G::swz(rr);
#pragma unroll
    for (int t = 0; t < 3; ++t) l2[(t * NG * PLANE + unit) * 2 + (c4 & 1)] = tr[t];
  };
  {
    float4 va[UA];
#pragma unroll
    for (int u = 0; u < UA; ++u) va[u] = fetch(tid + u * NT, 0, tid + u * NT < SA ? RA : 0);
#pragma unroll
    for (int u = 0; u < UA; ++u)
      if (tid + u * NT < SA) commit(va[u], tid + u * NT, 0, RA);
  }
  float4 vb[UB];
  if constexpr (SB > 0) {
#pragma unroll
    for (int u = 0; u < UB; ++u) vb[u] = fetch(tid + u * NT, RA, tid + u * NT < SB ? RA + RB_ : 0);
  }
  const float bl = bias ? bias[cb * 16 + (lane & 15)] : 0.0f;
  __syncthreads();

  // per chunk of this wave's K half (wave-uniform): the tap's pixel offset and the ci group's
  // plane offset; per tile (per lane): the window origin's staged pixel
  int toff[NCH2], coff[NCH2], rbv[G::TILES];
#pragma unroll
  for (int c = 0; c < NCH2; ++c) {
    const int k0 = (half * NCH2 + c) * 32, tap = k0 / CIN;
    toff[c] = (tap / KW) * WIN + tap % KW;
    coff[c] = ((k0 % CIN) / 8) * PLANE;
  }
  const int g = lane >> 4;
#pragma unroll
  for (int tile = 0; tile < G::TILES; ++tile) {
    int p = tile * 16 + (lane & 15);
    if (p >= nv) p = nv - 1;
    const int s = p / PIX, pp = p - s * PIX, oy = pp / G::WOUT, ox = pp - oy * G::WOUT;
    rbv[tile] = s * (HIN * WIN) + S * oy * WIN + S * ox;
  }
  const uint4 *const lt = lds;
  // the A fragments of step q = tile * NCH2 + c, three LDS buffers: step q + 2 is requested
  // while step q multiplies (a sched barrier keeps the compiler from sinking the reads);
  // phase A's tiles [0, TA) read only phase A's samples
  constexpr int TA = NSAMP > 1 ? (NA * PIX) / 16 : G::TILES;
  auto addr = [&](int q) -> int {
    const int tile = q / NCH2, c = q % NCH2;
    return coff[c] + g * PLANE + G::swz(rbv[tile] + toff[c]);
  };
  constexpr int NQ = G::TILES * NCH2, QA = TA * NCH2;
  bf16x8 xf[3][3];
  auto load = [&](int q) {
    const int u = addr(q);
#pragma unroll
    for (int t = 0; t < 3; ++t) xf[q % 3][t] = __builtin_bit_cast(bf16x8, lt[t * NG * PLANE + u]);
  };
  f32x4 acc[G::TILES];  // every tile's accumulator stays in registers (all loops unrolled)
  auto step = [&](int q, int qend) {
    const int tile = q / NCH2, c = q % NCH2;
    if (q + 2 < qend) load(q + 2);
    __builtin_amdgcn_sched_barrier(0);
    const bf16x8(&xc)[3] = xf[q % 3];
    f32x4 a = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[tile];
    // smallest terms first: (3,3) (3,2) (2,3) (3,1) (2,2) (1,3) (2,1) (1,2) (1,1)
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[2], wf[c][2], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[2], wf[c][1], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[1], wf[c][2], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[2], wf[c][0], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[1], wf[c][1], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[0], wf[c][2], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[1], wf[c][0], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[0], wf[c][1], a, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xc[0], wf[c][0], a, 0, 0, 0);
    acc[tile] = a;
    __builtin_amdgcn_sched_barrier(0);
  };
  load(0);
  if (QA > 1) load(1);
#pragma unroll
  for (int q = 0; q < QA; ++q) step(q, QA);
  if constexpr (QA < NQ) {  // phase B: write the second half's samples, then compute its tiles
    if constexpr (SB > 0) {
#pragma unroll
      for (int u = 0; u < UB; ++u)
        if (tid + u * NT < SB) commit(vb[u], tid + u * NT, RA, RA + RB_);
    }
    __syncthreads();
    load(QA);
    if (QA + 1 < NQ) load(QA + 1);
#pragma unroll
    for (int q = QA; q < NQ; ++q) step(q, NQ);
  }
  // the K halves meet in the (now free) LDS: half 1 stores its partial sums, half 0 adds its
  // own first, then the bias, ReLU; the workgroup's output run leaves in 16-byte stores.
  // C/D: lane holds channel 16 cb + (lane & 15) of pixels 4 (lane >> 4) + i of each tile
  float *F = reinterpret_cast<float *>(lds);
  const int co = cb * 16 + (lane & 15);
  auto fidx = [&](int p) -> int {
    const int s = p / PIX;
    return out_nchw ? (s * COUT + co) * PIX + (p - s * PIX) : p * COUT + co;
  };
  __syncthreads();  // every wave is done reading the input image
  // parts KS-1 .. 1 in turn: the last stores, each earlier one adds its own first
#pragma unroll
  for (int pt = KS - 1; pt >= 1; --pt) {
    if (half == pt) {
#pragma unroll
      for (int tile = 0; tile < G::TILES; ++tile)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = tile * 16 + 4 * g + i;
          if (p < nv) {
            const int f = fidx(p);
            F[f] = pt == KS - 1 ? acc[tile][i] : radd(acc[tile][i], F[f]);
          }
        }
    }
    __syncthreads();
  }
  if (half == 0) {
#pragma unroll
    for (int tile = 0; tile < G::TILES; ++tile)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = tile * 16 + 4 * g + i;
        if (p < nv) {
          const int f = fidx(p);
          F[f] = bias ? relu_c(radd(radd(acc[tile][i], F[f]), bl)) : radd(acc[tile][i], F[f]);
        }
      }
  }
  __syncthreads();
  if constexpr (CLS) {  // the class's pixels scattered into the full gradient, 16-byte stores
    const int py = blockIdx.y >> 1, px = blockIdx.y & 1, total4 = nv * COUT / 4;
    const float4 *Fs = reinterpret_cast<const float4 *>(F);
    for (int i = tid; i < total4; i += NT) {
      const int p = i / (COUT / 4), c4 = i - p * (COUT / 4), s = p / PIX, pp = p - s * PIX;
      const int jy = pp / G::WOUT, jx = pp - jy * G::WOUT;
      const int64_t o = (((b0 + s) * (2 * G::HOUT) + 2 * jy + py) * (2 * G::WOUT) + 2 * jx + px) * COUT + 4 * c4;
      *reinterpret_cast<float4 *>(y + o) = Fs[i];
    }
  } else if constexpr (MASK) {
    const int total4 = nv * COUT / 4;
    float4 *yo = reinterpret_cast<float4 *>(y + b0 * (int64_t)(COUT * PIX));
    const float4 *ym = reinterpret_cast<const float4 *>(ymask + b0 * (int64_t)(COUT * PIX));
    const float4 *Fs = reinterpret_cast<const float4 *>(F);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);  // channel quad tid % (COUT / 4), in i order
    // every mask load of the lane issued before the first use (clamped indices, no load under a
    // branch): the one-at-a-time loop waited for each in turn, ~5 round trips per workgroup
    constexpr int UM = (NSAMP * PIX * (COUT / 4) + NT - 1) / NT;
    float4 mk[UM];
#pragma unroll
    for (int u = 0; u < UM; ++u) {
      const int i = tid + u * NT;
      mk[u] = ym[i < total4 ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < UM; ++u) {
      const int i = tid + u * NT;
      if (i < total4) {
        const float4 g = Fs[i], m = mk[u];
        float4 o;
        o.x = m.x > 0.0f ? g.x : 0.0f;  // threshold_backward(g, y, 0)
        o.y = m.y > 0.0f ? g.y : 0.0f;
        o.z = m.z > 0.0f ? g.z : 0.0f;
        o.w = m.w > 0.0f ? g.w : 0.0f;
        yo[i] = o;
        acc.x = radd(acc.x, o.x);
        acc.y = radd(acc.y, o.y);
        acc.z = radd(acc.z, o.z);
        acc.w = radd(acc.w, o.w);
      }
    }
    __syncthreads();  // every lane is done reading F: its first NT float4 hold the lane sums
    float4 *red = reinterpret_cast<float4 *>(F);
    red[tid] = acc;
    __syncthreads();
    constexpr int Q = COUT / 4;
    for (int st = NT / 2; st >= Q; st >>= 1) {  // lanes tid and tid + st share a quad
      if (tid < st) {
        float4 a = red[tid];
        const float4 o = red[tid + st];
        a.x = radd(a.x, o.x);
        a.y = radd(a.y, o.y);
        a.z = radd(a.z, o.z);
        a.w = radd(a.w, o.w);
        red[tid] = a;
      }
      __syncthreads();
    }
    if (tid < Q) reinterpret_cast<float4 *>(bpart)[(int64_t)blockIdx.x * Q + tid] = red[tid];
  } else {
    const int total4 = nv * COUT / 4;  // the run [b0, b0 + ns) of y is contiguous in both layouts
    float4 *yo = reinterpret_cast<float4 *>(y + b0 * (int64_t)(COUT * PIX));
    const float4 *Fs = reinterpret_cast<const float4 *>(F);
    for (int i = tid; i < total4; i += NT) yo[i] = Fs[i];
  }
}

// OHWI weights -> the B fragments of k_conv_x9: slot ((cb * NCH + c) * 3 + t) * 64 + lane holds
// term t of W[16 cb + (lane & 15)][32 c + 8 (lane >> 4) + j], j = 0..7 (k = (kh, kw, ci), ci fastest)
template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NSAMP, int ROT, int KS>
__device__ __forceinline__ void pack_x9(const float *__restrict__ w, u32x4 *__restrict__ packed, int sl) {
  using G = X9Geom<KH, KW, S, CIN, HIN, WIN, NSAMP, ROT, KS>;
  if (sl >= G::PACKED_U4) return;
  const int lane = sl % 64, t = (sl / 64) % 3, c = (sl / 192) % G::NCH, cb = sl / (192 * G::NCH);
  const int co = cb * 16 + (lane & 15), k0 = c * 32 + 8 * (lane >> 4);
  const float4 *wp = reinterpret_cast<const float4 *>(w + (int64_t)co * G::K + k0);  // 32-byte aligned run
  const float4 w0 = wp[0], w1 = wp[1];  // both loads before the first split
  const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  uint32_t e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = bf16x3_term(wv[j], t);
  packed[sl] = u32x4{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
}

template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NSAMP, int ROT, int KS>
__global__ __launch_bounds__(256) void k_conv_pack_x9(const float *__restrict__ w, u32x4 *__restrict__ packed) {
  pack_x9<KH, KW, S, CIN, HIN, WIN, NSAMP, ROT, KS>(w, packed, blockIdx.x * 256 + threadIdx.x);
}

// The data gradient of a stride-1 KH x KW convolution as a forward one (rth_conv_dgrad, conv3):
//   gx[b, iy, ix, ci] = sum_{kh, kw, co} gy[b, iy - kh, ix - kw, co] W[co, kh, kw, ci]
// = the convolution of gy zero-padded by K - 1 with W' [ci][kh'][kw'][co] = W[co][K-1-kh'][K-1-kw'][ci]
// (the flipped, channel-transposed kernel), run by k_conv_x9 with PAD = K - 1 and no epilogue.
// This packs W' from the forward OHWI weights into the x9 B fragments (slot layout of pack_x9:
// output channel = ci, k' = (kh', kw', co), co fastest).
template <int KH, int KW, int CIN, int COUT, int HIN, int WIN, int NSAMP, int ROT, int KS>
__device__ __forceinline__ void pack_x9_dgrad(const float *__restrict__ w, u32x4 *__restrict__ packed, int sl) {
  using G = X9Geom<KH, KW, 1, COUT, HIN, WIN, NSAMP, ROT, KS>;  // the dgrad's "input" channels = the conv's COUT
  if (sl >= G::PACKED_U4) return;
  const int lane = sl % 64, t = (sl / 64) % 3, c = (sl / 192) % G::NCH, cb = sl / (192 * G::NCH);
  const int ci = cb * 16 + (lane & 15), k0 = c * 32 + 8 * (lane >> 4);
  const int tap = k0 / COUT, co0 = k0 % COUT, kh = KH - 1 - tap / KW, kw = KW - 1 - tap % KW;
  float wv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) wv[j] = w[((int64_t)(co0 + j) * KH * KW + kh * KW + kw) * CIN + ci];  // OHWI
  uint32_t e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = bf16x3_term(wv[j], t);
  packed[sl] = u32x4{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
}
template <int KH, int KW, int CIN, int COUT, int HIN, int WIN, int NSAMP, int ROT, int KS>
__global__ __launch_bounds__(256) void k_conv_pack_x9_dgrad(const float *__restrict__ w, u32x4 *__restrict__ packed) {
  pack_x9_dgrad<KH, KW, CIN, COUT, HIN, WIN, NSAMP, ROT, KS>(w, packed, blockIdx.x * 256 + threadIdx.x);
}

// conv2 (4x4, stride 2) has no single flipped kernel: its data gradient splits by the parity
// (py, px) of the input pixel, iy = 2 jy + py, ix = 2 jx + px.  Only taps kh = py + 2 a,
// kw = px + 2 c reach such a pixel, from output pixel (jy - a, jx - c), so each class is a
// stride-1 2x2 convolution of gy zero-padded by 1 with
//   W'_cls[ci][kh'][kw'][co] = W[co][py + 2 (1 - kh')][px + 2 (1 - kw')][ci]
// (kh' = 1 - a).  The 4 class kernels are packed back to back (class = 2 py + px), the slot
// layout of pack_x9 each (output channel = ci, k' = (kh', kw', co), co fastest).
template <int CIN, int COUT, int NSAMP, int ROT, int KS>
__device__ __forceinline__ void pack_x9_dgrad_cls(const float *__restrict__ w, u32x4 *__restrict__ packed, int slg) {
  using G = X9Geom<2, 2, 1, COUT, 11, 11, NSAMP, ROT, KS, CIN>;
  if (slg >= 4 * G::PACKED_U4) return;
  const int cls = slg / G::PACKED_U4, sl = slg - cls * G::PACKED_U4, py = cls >> 1, px = cls & 1;
  const int lane = sl % 64, t = (sl / 64) % 3, c = (sl / 192) % G::NCH, cb = sl / (192 * G::NCH);
  const int ci = cb * 16 + (lane & 15), k0 = c * 32 + 8 * (lane >> 4);
  const int tap = k0 / COUT, co0 = k0 % COUT, kh = py + 2 * (1 - tap / 2), kw = px + 2 * (1 - tap % 2);
  float wv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) wv[j] = w[((int64_t)(co0 + j) * 16 + kh * 4 + kw) * CIN + ci];  // OHWI, 4x4
  uint32_t e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = bf16x3_term(wv[j], t);
  packed[slg] = u32x4{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
}
template <int CIN, int COUT, int NSAMP, int ROT, int KS>
__global__ __launch_bounds__(256) void k_conv_pack_x9_dgrad_cls(const float *__restrict__ w,
                                                                u32x4 *__restrict__ packed) {
  pack_x9_dgrad_cls<CIN, COUT, NSAMP, ROT, KS>(w, packed, blockIdx.x * 256 + threadIdx.x);
}

// K parts per workgroup (waves = 4 channel blocks x KS): more parts, fewer weight registers per
// wave and more waves per CU
#ifndef X9_CONV2_KS
#define X9_CONV2_KS 2
#endif
#ifndef X9_CONV3_KS
#define X9_CONV3_KS 2
#endif
#define X9_CONV2 4, 4, 2, 32, 20, 20, 2, 10, X9_CONV2_KS
#define X9_CONV3 3, 3, 1, 64, 9, 9, 4, 3, X9_CONV3_KS

// OHWI weights -> MFMA fragment order (the LDS image the conv kernel copies)
template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN>
__global__ __launch_bounds__(256) void k_conv_pack(const float *__restrict__ w, f32x4 *__restrict__ packed) {
  using Gm = ConvGeom<MODE, KH, KW, S, CIN, COUT, HIN, WIN>;
  const int sl = blockIdx.x * 256 + threadIdx.x;
  if (sl < Gm::LDS_F4) packed[sl] = Gm::load_slot(w, sl);
}

// several layers in one launch (a network's torso, and the flipped data-gradient kernels of
// conv2 / conv3 for the backward of the same weights): block ranges per layer
constexpr int kPackMax = 6;
constexpr int kPackDgrad3 = 4, kPackDgrad2 = 5;  // PackJob::geom of the data-gradient packs
struct PackJob {
  int geom[kPackMax];  // index into the built geometries (find_conv order)
  int bf16x3[kPackMax];  // conv1 u8: the bf16x3 kernel's packed form; conv2 / conv3: the x9 form (2: conv3 hybrid)
  const float *w[kPackMax];
  f32x4 *packed[kPackMax];
  int first_block[kPackMax + 1];
  int n;
};

template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN>
__device__ __forceinline__ void pack_one(const float *w, f32x4 *packed, int sl) {
  using Gm = ConvGeom<MODE, KH, KW, S, CIN, COUT, HIN, WIN>;
  if (sl < Gm::LDS_F4) packed[sl] = Gm::load_slot(w, sl);
}

// conv2's packed weights serve both of its kernels: the x9 fragments, then the fp32-MFMA image
// (k_conv_bias_relu runs conv2 above conv2_x9_max() samples, ConvLaunch::big)
using X9Conv2 = X9Geom<X9_CONV2>;
__device__ __forceinline__ void pack_hybrid_conv2(const float *w, f32x4 *packed, int sl) {
  if (sl < X9Conv2::PACKED_U4) pack_x9<X9_CONV2>(w, reinterpret_cast<u32x4 *>(packed), sl);
  else pack_one<RTH_CONV_F32_NHWC, 4, 4, 2, 32, 64, 20, 20>(w, packed + X9Conv2::PACKED_U4, sl - X9Conv2::PACKED_U4);
}
__global__ __launch_bounds__(256) void k_conv_pack_hybrid_conv2(const float *__restrict__ w, f32x4 *__restrict__ packed) {
  pack_hybrid_conv2(w, packed, blockIdx.x * 256 + threadIdx.x);
}
// conv3's: the fp32-MFMA image (small batches), then the x9 fragments (ConvLaunch::big)
using F32Conv3 = ConvGeom<RTH_CONV_F32_NHWC, 3, 3, 1, 64, 64, 9, 9>;
__device__ __forceinline__ void pack_hybrid_conv3(const float *w, f32x4 *packed, int sl) {
  if (sl < F32Conv3::LDS_F4) pack_one<RTH_CONV_F32_NHWC, 3, 3, 1, 64, 64, 9, 9>(w, packed, sl);
  else pack_x9<X9_CONV3>(w, reinterpret_cast<u32x4 *>(packed + F32Conv3::LDS_F4), sl - F32Conv3::LDS_F4);
}
__global__ __launch_bounds__(256) void k_conv_pack_hybrid_conv3(const float *__restrict__ w, f32x4 *__restrict__ packed) {
  pack_hybrid_conv3(w, packed, blockIdx.x * 256 + threadIdx.x);
}

// the data gradients' packed kernels (X9Dgrad3 / X9Dgrad2 below: KS = 2, 1 sample per
// workgroup -- the packed layout does not depend on the samples per workgroup)
#define X9_DGRAD3_KS 2
#ifndef X9_DGRAD2_KS
#define X9_DGRAD2_KS 2
#endif
__device__ __forceinline__ void pack_dgrad3(const float *w, u32x4 *packed, int sl) {
  pack_x9_dgrad<3, 3, 64, 64, 11, 11, 1, 3, X9_DGRAD3_KS>(w, packed, sl);
}
__device__ __forceinline__ void pack_dgrad2(const float *w, u32x4 *packed, int sl) {
  pack_x9_dgrad_cls<32, 64, 1, 3, X9_DGRAD2_KS>(w, packed, sl);
}

__global__ __launch_bounds__(256) void k_conv_pack_many(PackJob job) {
  int l = 0;
  while (l + 1 < job.n && (int)blockIdx.x >= job.first_block[l + 1]) ++l;
  const int sl = ((int)blockIdx.x - job.first_block[l]) * 256 + threadIdx.x;
  switch (job.geom[l]) {
    case 0:
      if (job.bf16x3[l]) pack_conv1_bf16x3(job.w[l], reinterpret_cast<u32x4 *>(job.packed[l]), sl);
      else pack_one<RTH_CONV_U8_CHW, 8, 8, 4, 4, 32, 84, 84>(job.w[l], job.packed[l], sl);
      break;
    case 1: pack_one<RTH_CONV_F32_NHWC, 8, 8, 4, 4, 32, 84, 84>(job.w[l], job.packed[l], sl); break;
    case 2:
      if (job.bf16x3[l]) pack_hybrid_conv2(job.w[l], job.packed[l], sl);
      else pack_one<RTH_CONV_F32_NHWC, 4, 4, 2, 32, 64, 20, 20>(job.w[l], job.packed[l], sl);
      break;
    case kPackDgrad3: pack_dgrad3(job.w[l], reinterpret_cast<u32x4 *>(job.packed[l]), sl); break;
    case kPackDgrad2: pack_dgrad2(job.w[l], reinterpret_cast<u32x4 *>(job.packed[l]), sl); break;
    default:
      if (job.bf16x3[l] == 2) pack_hybrid_conv3(job.w[l], job.packed[l], sl);
      else if (job.bf16x3[l]) pack_x9<X9_CONV3>(job.w[l], reinterpret_cast<u32x4 *>(job.packed[l]), sl);
      else pack_one<RTH_CONV_F32_NHWC, 3, 3, 1, 64, 64, 9, 9>(job.w[l], job.packed[l], sl);
      break;
  }
}

struct ConvLaunch {
  const void *fn, *pack;
  int waves;
  int lds_bytes;  // packed weight bytes
  int per_cu;  // resident workgroups per CU (occupancy query, cached)
  int tile_px;  // output pixels per wave tile
  int bf16x3;   // conv1 on uint8 stacks, exact-split bf16 MFMA: 1 = k_conv1_u8_bf16x3, 2 = k_conv1_u8_share
  int nsplit;   // wave tiles per pixel tile (channel parts; 0 = 1)
  int x9;       // k_conv_x9: samples per workgroup at most (0 = not an x9 kernel)
  const void *x9fn[5];  // k_conv_x9 by samples per workgroup (nullptr: not built)
  // hybrid geometries: above `big_above` samples the fp32-MFMA kernel *big runs instead, its
  // packed weights behind the x9 ones (at byte `big_off`; lds_bytes counts both)
  const struct ConvLaunch *big;
  int64_t big_above;
  int big_off;
  int pw;   // k_conv_bias_relu PW: channel part per workgroup (the grid a multiple of nsplit)
  // the same kernel with its ragged last round split into channel parts (TS > 1), launched
  // instead of fn when a launch has at least tsfn_rounds whole rounds of tiles (nullptr: never)
  const void *tsfn = nullptr;
  int tsfn_rounds = 0;
};

template <int KH, int KW, int S, int CIN, int HIN, int WIN, int NSAMP, int ROT, int KS>
static ConvLaunch x9_launch() {
  using G = X9Geom<KH, KW, S, CIN, HIN, WIN, NSAMP, ROT, KS>;
  ConvLaunch l{reinterpret_cast<const void *>(&k_conv_x9<KH, KW, S, CIN, HIN, WIN, NSAMP, ROT, KS>),
               reinterpret_cast<const void *>(&k_conv_pack_x9<KH, KW, S, CIN, HIN, WIN, NSAMP, ROT, KS>), 4 * KS,
               G::PACKED_U4 * 16, 1, 16, 0, 0, NSAMP, {}, nullptr, 0, 0};
  l.x9fn[1] = reinterpret_cast<const void *>(&k_conv_x9<KH, KW, S, CIN, HIN, WIN, 1, ROT, KS>);
  if (NSAMP >= 2) l.x9fn[2] = reinterpret_cast<const void *>(&k_conv_x9<KH, KW, S, CIN, HIN, WIN, (NSAMP >= 2 ? 2 : 1), ROT, KS>);
  if (NSAMP >= 3) l.x9fn[3] = reinterpret_cast<const void *>(&k_conv_x9<KH, KW, S, CIN, HIN, WIN, (NSAMP >= 3 ? 3 : 1), ROT, KS>);
  if (NSAMP >= 4) l.x9fn[4] = reinterpret_cast<const void *>(&k_conv_x9<KH, KW, S, CIN, HIN, WIN, (NSAMP >= 4 ? 4 : 1), ROT, KS>);
  return l;
}

template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN, int WAVES, int MB, int NS = 1,
          int PW = 0, int TS = 1>
static ConvLaunch conv_launch() {
  using Gm = ConvGeom<MODE, KH, KW, S, CIN, COUT, HIN, WIN>;
  ConvLaunch l{reinterpret_cast<const void *>(&k_conv_bias_relu<MODE, KH, KW, S, CIN, COUT, HIN, WIN, WAVES, MB, NS, PW, TS>),
               reinterpret_cast<const void *>(&k_conv_pack<MODE, KH, KW, S, CIN, COUT, HIN, WIN>), WAVES,
               Gm::LDS_F4 * 16, 0, 16 * MB, 0, NS, 0, {}, nullptr, 0, 0, PW};
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, l.fn, WAVES * 64, 0) != hipSuccess || blocks < 1)
    blocks = 1;
  l.per_cu = blocks;
  return l;
}

// conv1 on the uint8 stacks: k_conv1_u8_share (r05: each lane converts half of its window and
// takes the other half from its neighbour by DPP; bit-identical to r04's k_conv1_u8_bf16x3)
static ConvLaunch conv1_bf16x3_launch() {
  ConvLaunch l{reinterpret_cast<const void *>(&k_conv1_u8_share<false>),
               reinterpret_cast<const void *>(&k_conv1_pack_bf16x3), 4, kC1PackedBytes, 0, 32, 2, 0, 0,
               {}, nullptr, 0, 0};
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, l.fn, 256, 0) != hipSuccess || blocks < 1) blocks = 1;
  l.per_cu = blocks;
  return l;
}

#ifndef CONV1_MB
#define CONV1_MB 1
#endif
#ifndef CONV2_MB
#define CONV2_MB 1
#endif
#ifndef CONV2_NS
#define CONV2_NS 1
#endif
#ifndef CONV3_MB
#define CONV3_MB 1
#endif
#ifndef CONV3_WAVES
#define CONV3_WAVES 8
#endif
#ifndef CONV3_NS
#define CONV3_NS 1
#endif

#ifndef CONV2_X9_MAX
#define CONV2_X9_MAX 0
#endif
#ifndef CONV3_X9_MIN
#define CONV3_X9_MIN 0
#endif
// hybrid switch points (samples; build-time options of variant libraries): conv2 runs x9 up to
// CONV2_X9_MAX samples (0: never -- its 77-154 KB of LDS per workgroup crowds the other stream's
// kernels out of the CUs in the loop), conv3 runs x9 above CONV3_X9_MIN (0: always)
constexpr int64_t conv2_x9_max() { return CONV2_X9_MAX; }
constexpr int64_t conv3_x9_min() { return CONV3_X9_MIN; }
// x9 samples per workgroup = n / CUs, rounded down to a built instantiation
constexpr int64_t x9_wg_per_cu() { return 1; }

// the supported geometries (the Nature-DQN torso on 4 x 84 x 84 stacks)
static bool find_conv(const rth_conv_shape &s, ConvLaunch *out, int *geom = nullptr) {
  auto is = [&](int mode, int cin, int hin, int win, int cout, int kh, int kw, int st) {
    return (s.input & ~RTH_CONV_OUT_NCHW) == mode && s.cin == cin && s.hin == hin && s.win == win && s.cout == cout && s.kh == kh &&
           s.kw == kw && s.stride == st;
  };
  if (is(RTH_CONV_U8_CHW, 4, 84, 84, 32, 8, 8, 4)) {
    static const ConvLaunch l = conv1_bf16x3_launch();
    *out = l;
    if (geom) *geom = 0;
  } else if (is(RTH_CONV_F32_NHWC, 4, 84, 84, 32, 8, 8, 4)) {
    static const ConvLaunch l = conv_launch<RTH_CONV_F32_NHWC, 8, 8, 4, 4, 32, 84, 84, 4, CONV1_MB>();
    *out = l;
    if (geom) *geom = 1;
  } else if (is(RTH_CONV_F32_NHWC, 32, 20, 20, 64, 4, 4, 2)) {
    // x9 up to conv2_x9_max() samples, the fp32-MFMA kernel above.  Default 0 (fp32 only):
    // standalone the x9 kernel wins below ~400 samples (16 vs 22 us at 256), but in the Ape-X
    // loop its 77-154 KB of LDS per workgroup crowds the concurrent stream's kernels out of the
    // CUs, and the loop ran 0.5-1 % slower with it
    // the tile schedule (r05 A/B, profiles/r05/ab_log.txt): 16-pixel x 64-channel wave tiles
    // round-robin, the ragged last round split into quarter-width units for launches of >= 4
    // whole rounds of tiles (the learner's 1,024 samples: 53.1 vs 57.9 us alone; whole tiles
    // below) -- the same outputs, bit for bit
    static const ConvLaunch f32 = [] {
      ConvLaunch l = conv_launch<RTH_CONV_F32_NHWC, 4, 4, 2, 32, 64, 20, 20, 8, CONV2_MB, 1>();
      l.tsfn = conv_launch<RTH_CONV_F32_NHWC, 4, 4, 2, 32, 64, 20, 20, 8, CONV2_MB, 1, 0, 4>().fn;
      l.tsfn_rounds = 4;
      return l;
    }();
    static const ConvLaunch l = [] {
      if (conv2_x9_max() <= 0) return f32;
      ConvLaunch h = x9_launch<X9_CONV2>();
      h.big = &f32;
      h.big_above = conv2_x9_max();
      h.big_off = h.lds_bytes;
      h.lds_bytes += f32.lds_bytes;
      h.pack = reinterpret_cast<const void *>(&k_conv_pack_hybrid_conv2);
      return h;
    }();
    *out = l;
    if (geom) *geom = 2;
  } else if (is(RTH_CONV_F32_NHWC, 64, 9, 9, 64, 3, 3, 1)) {
    // the fp32-MFMA kernel up to conv3_x9_min() samples, x9 above (packed: fp32 image, then x9)
    static const ConvLaunch x9 = x9_launch<X9_CONV3>();
    static const ConvLaunch l = [] {
      ConvLaunch f = conv_launch<RTH_CONV_F32_NHWC, 3, 3, 1, 64, 64, 9, 9, CONV3_WAVES, CONV3_MB, CONV3_NS>();
      if (conv3_x9_min() <= 0) return x9;
      f.big = &x9;
      f.big_above = conv3_x9_min();
      f.big_off = f.lds_bytes;
      f.lds_bytes += x9.lds_bytes;
      f.pack = reinterpret_cast<const void *>(&k_conv_pack_hybrid_conv3);
      f.x9 = 0;
      return f;
    }();
    *out = l;
    if (geom) *geom = 3;
  } else {
    return false;
  }
  return true;
}

static int cu_count() {
  static int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  return cus;
}

// ---------------------------------------------------------------------------------------
// conv data gradient (the learner's backward through conv3 / conv2): gx = the transposed
// convolution of gy with W, as an implicit GEMM per stride-parity class on the fp32 MFMA.
// Input pixel (iy, ix) = (S*jy + py, S*jx + px) of class (py, px) only meets the taps
// kh = py + S*dy, kw = px + S*dx (dy < KH/S, dx < KW/S), at output pixel (jy - dy, jx - dx):
//   gx[b, iy, ix, ci] = sum_{dy, dx, co} gy[b, jy - dy, jx - dx, co] * W[co, kh, kw, ci]
// (taps falling outside gy read zero).  Rows = the class's pixels (b, jy, jx), columns = ci,
// K = (tap, co): every input pixel belongs to exactly one class and is written once, so
// there is no zero fill and no atomic.  A workgroup serves one class and stages that class's
// taps of W in LDS in MFMA fragment order (lane (n, q) holds co = 4q .. 4q+3 of column n);
// the A operand is a float4 of gy's channels-last row, read straight from global memory.
#ifndef DGRAD_WAVES
#define DGRAD_WAVES 8
#endif
#ifndef DGRAD_D
#define DGRAD_D 4  // input chunks in flight per wave, at most (the largest divisor of the chunk count)
#endif

template <int KH, int KW, int S, int CI, int CO, int HI, int WI>
struct DgradGeom {
  static constexpr int HO = (HI - KH) / S + 1, WO = (WI - KW) / S + 1;
  static constexpr int TH = KH / S, TW = KW / S, TAPS = TH * TW, JH = HI / S, JW = WI / S;
  static constexpr int CPT = CO / 16, G = TAPS * CPT, NB = CI / 16, LDS_F4 = G * NB * 64;
  static_assert(KH % S == 0 && KW % S == 0 && HI % S == 0 && WI % S == 0, "stride must tile kernel and input");
  static_assert(CI % 16 == 0 && CO % 16 == 0, "channels must be multiples of 16");
  static constexpr int D = [] {  // input chunks in flight: the largest divisor of G <= DGRAD_D
    int d = DGRAD_D;
    while (G % d) --d;
    return d;
  }();
};

// XCD-aware workgroup -> (class, tile range) map (xcd != 0; the grid a multiple of 8 x NCLS):
// consecutive workgroups land on consecutive XCDs (blockIdx % 8), each with its own L2, so
// XCD x serves all classes of one contiguous eighth of the class tiles -- the 4 classes and
// the neighbouring tiles that read the same gy rows share that XCD's L2 instead of fetching
// them from HBM up to 8 times.  xcd == 0: the plain interleave (class = blockIdx % NCLS).
template <int KH, int KW, int S, int CI, int CO, int HI, int WI, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_conv_dgrad(const float *__restrict__ gy, int64_t n,
                                                          const float *__restrict__ w, float *__restrict__ gx,
                                                          int xcd) {
  using Gm = DgradGeom<KH, KW, S, CI, CO, HI, WI>;
  constexpr int HO = Gm::HO, WO = Gm::WO, TW = Gm::TW, CPT = Gm::CPT, NB = Gm::NB;
  constexpr int T = WAVES * 64, NCLS = S * S;
  __shared__ f32x4 wl[Gm::LDS_F4];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64, q = lane >> 4, mr = lane & 15;
  const int64_t PC = n * Gm::JH * Gm::JW, tiles = (PC + 15) / 16;
  int cls;
  int64_t wg, nwg, tile_lo = 0, tile_hi = tiles;
  if (xcd) {
    const int x = (int)(blockIdx.x % 8), slot = (int)(blockIdx.x / 8);
    cls = slot % NCLS;
    wg = slot / NCLS;
    nwg = gridDim.x / (8 * NCLS);
    const int64_t per = (tiles + 7) / 8;
    tile_lo = x * per;
    tile_hi = tile_lo + per < tiles ? tile_lo + per : tiles;
  } else {
    cls = blockIdx.x % NCLS;
    wg = blockIdx.x / NCLS;
    nwg = gridDim.x / NCLS;
  }
  const int py = cls / S, px = cls % S;
  // gy as a buffer resource (kernel arguments only: wave-uniform), its range the n samples
  const __amdgpu_buffer_rsrc_t gy_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float *>(gy), 0, (int)(n * (HO * WO * CO) * 4), 0x00020000);

  // stage this class's taps: slot (g * NB + nb) * 64 + lane, chunk g = (tap, 16 co)
  for (int sl = threadIdx.x; sl < Gm::LDS_F4; sl += T) {
    const int ln = sl % 64, gn = sl / 64, nb = gn % NB, g = gn / NB;
    const int t = g / CPT, co = (g % CPT) * 16 + 4 * (ln >> 4), ci = nb * 16 + (ln & 15);
    const int kh = py + S * (t / TW), kw = px + S * (t % TW);
    const float *src = w + ((int64_t)co * KH * KW + kh * KW + kw) * CI + ci;
    constexpr int CS = KH * KW * CI;  // OHWI stride between consecutive co
    wl[sl] = f32x4{src[0], src[CS], src[2 * CS], src[3 * CS]};
  }
  __syncthreads();

  const f32x4 *wlane = wl + lane;
  for (int64_t tile = tile_lo + wg * WAVES + wave; tile < tile_hi; tile += nwg * WAVES) {
    int64_t p = tile * 16 + mr;
    if (p >= PC) p = PC - 1;  // tail lanes compute a duplicate pixel, never stored
    const int64_t b = p / (Gm::JH * Gm::JW);
    const int r = (int)(p % (Gm::JH * Gm::JW)), jy = r / Gm::JW, jx = r % Gm::JW;
    const uint32_t gyb = (uint32_t)((b * (HO * WO * CO) + 4 * q) * 4);  // byte offset (host: gy < 2 GiB)
    // chunk g = (tap g / CPT, 16 co from (g % CPT) * 16): this lane's float4 of gy, zero off the
    // edge -- a buffer load whose offset lies past the descriptor's range returns zeros, so
    // every load is unconditional (a load under a branch made the compiler wait for ALL loads
    // in flight, vmcnt(0), before each group's first MFMA: no prefetch left)
    auto aload = [&](int g) {  // g >= G: past the tile (zeros, no memory access), keeps the count static
      const int t = g / CPT, oy = jy - t / TW, ox = jx - t % TW;
      const bool in = g < Gm::G && oy >= 0 && oy < HO && ox >= 0 && ox < WO;
      const uint32_t off = in ? gyb + (uint32_t)(((oy * WO + ox) * CO + (g % CPT) * 16) * 4) : 0x80000000u;
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(gy_rsrc, off, 0, 0));
    };
    f32x4 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int D = Gm::D;
    f32x4 ar[D];  // input chunks in flight
#pragma unroll
    for (int d = 0; d < D; ++d) ar[d] = aload(d);
#pragma unroll 1
    for (int g0 = 0; g0 < Gm::G; g0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int g = g0 + d;
        f32x4 bf[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) bf[nb] = wlane[(g * NB + nb) * 64];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[d][tt], bf[nb][tt], acc[nb], 0, 0, 0);
        ar[d] = aload(g + D);  // unconditional: the compiler keeps D - 1 loads in flight
      }
    }
    // C/D: lane holds column mr of rows 4q .. 4q+3
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t po = tile * 16 + 4 * q + i;
      if (po < PC) {
        const int64_t bo = po / (Gm::JH * Gm::JW);
        const int ro = (int)(po % (Gm::JH * Gm::JW)), iy = S * (ro / Gm::JW) + py, ix = S * (ro % Gm::JW) + px;
        float *dst = gx + ((bo * HI + iy) * WI + ix) * CI + mr;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) dst[nb * 16] = acc[nb][i];
      }
    }
  }
}

constexpr int dgrad_xcd() { return 1; }  // the XCD-aware class interleave (neutral, r03)

struct DgradLaunch {
  const void *fn;
  int waves, classes, per_cu, lds_bytes;
  int jh, jw;
};

template <int KH, int KW, int S, int CI, int CO, int HI, int WI, int WAVES>
static DgradLaunch dgrad_launch() {
  using Gm = DgradGeom<KH, KW, S, CI, CO, HI, WI>;
  DgradLaunch l{reinterpret_cast<const void *>(&k_conv_dgrad<KH, KW, S, CI, CO, HI, WI, WAVES>), WAVES, S * S, 1,
                Gm::LDS_F4 * 16, Gm::JH, Gm::JW};
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, l.fn, WAVES * 64, 0) == hipSuccess && blocks >= 1)
    l.per_cu = blocks;
  return l;
}


static bool find_dgrad(const rth_conv_shape &s, DgradLaunch *out) {
  auto is = [&](int cin, int hin, int win, int cout, int kh, int kw, int st) {
    return s.input == RTH_CONV_F32_NHWC && s.cin == cin && s.hin == hin && s.win == win && s.cout == cout &&
           s.kh == kh && s.kw == kw && s.stride == st;
  };
  if (is(32, 20, 20, 64, 4, 4, 2)) {
    static const DgradLaunch l = dgrad_launch<4, 4, 2, 32, 64, 20, 20, DGRAD_WAVES>();
    *out = l;
  } else if (is(64, 9, 9, 64, 3, 3, 1)) {
    static const DgradLaunch l = dgrad_launch<3, 3, 1, 64, 64, 9, 9, DGRAD_WAVES>();
    *out = l;
  } else {
    return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------
// conv1 backward on uint8 stacks: gy = (y > 0) ? g : 0 (ReLU backward), gw = sum over output
// pixels of gy (x) im2col(x), gb = sum of gy -- one pass over g, y and the stacks, MFMA
// 32x32x2 f32 with the reduction over pixels (2 per MFMA).  The 32 x 256 weight gradient is
// held as KW = 8 accumulator tiles per wave: tile kw, column j = (ci, kh) (32 of them), so a
// lane's 8 B-operand values of one pixel are 8 contiguous bytes of one input row (two dword
// loads).  Pixel pairs are loaded one group of kWgU pairs ahead.  Workgroup w sums a
// contiguous pixel range and writes its partial; k_wgrad_reduce adds the partials in
// workgroup order (deterministic).
#ifndef CONV_WG_BLOCKS
#define CONV_WG_BLOCKS 256
#endif
#ifndef CONV_WG_U
#define CONV_WG_U 4
#endif
constexpr int kWgWaves = 8, kWgBlocks = CONV_WG_BLOCKS, kWgU = CONV_WG_U;

template <int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN>
__global__ __launch_bounds__(kWgWaves * 64) void k_conv_wgrad_u8(const uint8_t *__restrict__ x,
                                                                const int64_t *__restrict__ rows, int64_t n,
                                                                const float *__restrict__ g,
                                                                const float *__restrict__ y,
                                                                float *__restrict__ partial) {
  constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  constexpr int K = CIN * KH * KW, STACK = CIN * HIN * WIN;
  static_assert(COUT == 32 && CIN * KH == 32 && KW == 8 && S % 4 == 0, "conv1 layout");
  __shared__ float red[kWgWaves][32];
  __shared__ float tile[kWgWaves][32 * 32];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64, o = lane & 31, h = lane >> 5;
  const int64_t P = n * PIX;
  constexpr int STEP = 2 * kWgWaves;  // pixels per round over the workgroup's waves
  const int64_t chunk = ((P + gridDim.x - 1) / gridDim.x + STEP * kWgU - 1) / (STEP * kWgU) * (STEP * kWgU);
  const int64_t p_begin = (int64_t)blockIdx.x * chunk, p_end = p_begin + chunk < P ? p_begin + chunk : P;
  // B column j = o = (ci, kh): its input row inside the window
  const int row_off = (o / KH) * HIN * WIN + (o % KH) * WIN;
  struct Pair {
    float a;
    uint32_t lo, hi;
  };
  auto load = [&](int64_t p0) {  // pixel p0 + h of this wave's pair
    const int64_t p = p0 + h;
    const bool live = p < p_end;
    const int64_t pc = live ? p : (p_begin < P ? p_begin : 0);
    const int64_t b = pc / PIX;
    const int pp = (int)(pc % PIX), oy = pp / WOUT, ox = pp % WOUT;
    const uint8_t *src = x + (rows ? rows[b] : b) * (int64_t)STACK + row_off + (S * oy) * WIN + S * ox;
    const float gv = g[pc * COUT + o], yv = y[pc * COUT + o];
    Pair r;
    r.a = (live && yv > 0.0f) ? gv : 0.0f;
    r.lo = *reinterpret_cast<const uint32_t *>(src);
    r.hi = *reinterpret_cast<const uint32_t *>(src + 4);
    return r;
  };
  f32x16 acc[KW];
#pragma unroll
  for (int t = 0; t < KW; ++t) acc[t] = f32x16{};
  float db = 0.0f;
  Pair cur[kWgU], nxt[kWgU];
  int64_t p0 = p_begin + 2 * wave;
#pragma unroll
  for (int u = 0; u < kWgU; ++u) cur[u] = load(p0 + u * STEP);
  for (; p0 < p_end; p0 += kWgU * STEP) {
#pragma unroll
    for (int u = 0; u < kWgU; ++u) nxt[u] = load(p0 + (kWgU + u) * STEP);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kWgU; ++u) {
      db = radd(db, cur[u].a);
#pragma unroll
      for (int t = 0; t < KW; ++t) {
        const uint32_t wv = t < 4 ? cur[u].lo : cur[u].hi;
        const float bx = (float)((wv >> (8 * (t % 4))) & 0xffu);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[u].a, bx, acc[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < kWgU; ++u) cur[u] = nxt[u];
  }
  // bias: lanes o and o + 32 of every wave
  db = radd(db, __shfl_down(db, 32));
  if (h == 0) red[wave][o] = db;
  // the weight tiles: sum the waves through LDS, tile by tile (C/D: lane -> column o of the
  // tile, register r -> row i = 8 (r / 4) + 4 h + r % 4 = output channel)
  float *out = partial + (int64_t)blockIdx.x * (COUT * K + COUT);
#pragma unroll
  for (int t = 0; t < KW; ++t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[wave][(8 * (r / 4) + 4 * h + r % 4) * 32 + o] = acc[t][r];
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * 32; e += kWgWaves * 64) {
      float v = tile[0][e];
#pragma unroll
      for (int w = 1; w < kWgWaves; ++w) v = radd(v, tile[w][e]);
      out[(e / 32) * K + t * 32 + e % 32] = v;  // [o][kk = kw * 32 + (ci, kh)]
    }
    __syncthreads();
  }
  if (threadIdx.x < 32) {
    float v = red[0][threadIdx.x];
    for (int w = 1; w < kWgWaves; ++w) v = radd(v, red[w][threadIdx.x]);
    out[COUT * K + threadIdx.x] = v;
  }
}

// conv1 weight gradient on uint8 stacks on the bf16 MFMA, the upstream gradient split into
// three exact bf16 terms (truncation split: a = hi + mid + lo, 8 significand bits each, so
// every product with a byte is exact in fp32): the same partials as k_conv_wgrad_u8 --
// D[co][(ci, kh)] per kw over this workgroup's pixels -- summed in a different order.
// One v_mfma_f32_32x32x16_bf16 takes 16 pixels as two "slots" of 8 consecutive output
// pixels of one output row (ox 0-7, 8-15, 16-19 + 4 masked: 3 slots per row, 60 per
// stack); lane (r, h) holds slot h: as A the masked gradient of channel r (3 terms), as B
// byte kw of run (ci, kh) = r of each pixel's window.  The 8 windows of a slot overlap: run r
// of all of them is one 36-byte span of stack row (ci, 4 oy + kh) (20 bytes for the last
// slot of a row), loaded as 2 x dwordx4 + dword; v_cvt_f32_ubyteN picks byte kw of pixel j
// (byte 4j + kw of the span), so the 8x8 byte transpose is free.  The tile / partial
// layout and the cross-wave LDS sum are k_conv_wgrad_u8's.
__device__ __forceinline__ void split3_trunc(float a, uint32_t &t0, uint32_t &t1, uint32_t &t2) {
  const uint32_t u = __float_as_uint(a);
  t0 = u & 0xffff0000u;
  const float r1 = rsub(a, __uint_as_float(t0));
  t1 = __float_as_uint(r1) & 0xffff0000u;
  t2 = __float_as_uint(rsub(r1, __uint_as_float(t1)));  // <= 8 significand bits: exact in bf16
}

// MODE 0: x holds the n stacks; 1: rows[b] indexes x's stacks; 2 (r05): x is a replay's frame
// store and rows the int32 [n][4] frame ids of the stacks (k_conv1_u8_share<true>'s input)
template <int MODE>
__global__ __launch_bounds__(kWgWaves * 64) void k_conv1_wgrad_bf16x3(const uint8_t *__restrict__ x,
                                                                     const int64_t *__restrict__ rows, int64_t n,
                                                                     const float *__restrict__ g,
                                                                     const float *__restrict__ y,
                                                                     float *__restrict__ partial) {
  constexpr int HIN = 84, WIN = 84, WOUT = 20, PIX = 400, KH = 8, KW = 8, S = 4, COUT = 32;
  constexpr int K = 4 * KH * KW, STACK = 4 * HIN * WIN, SLOTS = 3 * 20;  // slots per stack
  using f32x16 = __attribute__((ext_vector_type(16))) float;
  __shared__ float red[kWgWaves][32];
  __shared__ float tile[kWgWaves][32 * 32];
  const int lane = threadIdx.x % 64, o = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const int64_t NS = n * SLOTS, NG = (NS + 1) / 2;  // slots, 2-slot groups
  const int64_t chunk = ((NG + gridDim.x - 1) / gridDim.x + kWgWaves - 1) / kWgWaves * kWgWaves;
  const int64_t g_begin = (int64_t)blockIdx.x * chunk, g_end = g_begin + chunk < NG ? g_begin + chunk : NG;
  const int row_off = (o / KH) * HIN * WIN + (o % KH) * WIN;  // run (ci, kh) = o
  struct Raw {
    float gv[8], yv[8];
    uint32_t sp[9];  // the 36-byte span
    int nv;          // valid pixels of the slot (0: past the end)
  };
  // no branches around loads (the compiler then counts the loads in flight exactly instead of
  // waiting for all of them): the two slots' samples and row indices are scalar
  auto load = [&](int64_t gq, Raw &rw) {
    const bool live = gq < g_end;
    const int64_t gi = live ? gq : g_end - 1;
    const int64_t s0 = 2 * gi, s1 = s0 + 1 < NS ? s0 + 1 : NS - 1;  // wave-uniform
    const int64_t b0 = s0 / SLOTS, b1 = s1 / SLOTS;
    const int64_t rw0 = MODE == 1 ? rows[b0] : b0, rw1 = MODE == 1 ? rows[b1] : b1;
    const int64_t sl = h ? s1 : s0, b = h ? b1 : b0, row = h ? rw1 : rw0;
    const int rem = (int)(sl - b * SLOTS), oy = rem / 3, seg = rem % 3;
    rw.nv = live && 2 * gi + h < NS ? (seg == 2 ? 4 : 8) : 0;
    const uint8_t *src;
    if constexpr (MODE == 2) {  // run (ci, kh) = (o / KH, o % KH) from frame ids[b][ci]
      // the two slots' id tuples as wave-uniform scalar loads (not in the vmcnt queue)
      const int4 i0 = reinterpret_cast<const int4 *>(rows)[b0], i1 = reinterpret_cast<const int4 *>(rows)[b1];
      const int4 iv = h ? i1 : i0;
      const int ci = o / KH;
      const int64_t fid = ci == 0 ? iv.x : ci == 1 ? iv.y : ci == 2 ? iv.z : iv.w;
      src = x + fid * (int64_t)(HIN * WIN) + (o % KH) * WIN + (S * oy) * WIN + S * 8 * seg;
    } else {
      src = x + row * (int64_t)STACK + row_off + (S * oy) * WIN + S * 8 * seg;
    }
    const u32x4 v0 = *reinterpret_cast<const u32x4 *>(src);
    const uint32_t v4 = *reinterpret_cast<const uint32_t *>(src + 16);
    // the last slot's span ends the row: its unused upper part re-reads the lower
    const u32x4 v1 = *reinterpret_cast<const u32x4 *>(src + (seg < 2 ? 20 : 0));
    rw.sp[0] = v0[0], rw.sp[1] = v0[1], rw.sp[2] = v0[2], rw.sp[3] = v0[3], rw.sp[4] = v4;
    rw.sp[5] = v1[0], rw.sp[6] = v1[1], rw.sp[7] = v1[2], rw.sp[8] = v1[3];
    const int64_t q0 = b * PIX + oy * WOUT + 8 * seg;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t q = q0 + (j < 4 || seg < 2 ? j : 0);  // masked pixels re-read pixel 0
      rw.gv[j] = g[q * COUT + o];
      rw.yv[j] = y[q * COUT + o];
    }
  };
  f32x16 acc[KW];
#pragma unroll
  for (int t = 0; t < KW; ++t) acc[t] = f32x16{};
  float db = 0.0f;
  auto compute = [&](const Raw &rw) {
    uint32_t tm[3][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = (j < rw.nv && rw.yv[j] > 0.0f) ? rw.gv[j] : 0.0f;
      db = radd(db, a);
      split3_trunc(a, tm[0][j], tm[1][j], tm[2][j]);
    }
    bf16x8 af[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
      af[t] = __builtin_bit_cast(bf16x8, (u32x4{__builtin_amdgcn_perm(tm[t][1], tm[t][0], 0x07060302u),
                                                 __builtin_amdgcn_perm(tm[t][3], tm[t][2], 0x07060302u),
                                                 __builtin_amdgcn_perm(tm[t][5], tm[t][4], 0x07060302u),
                                                 __builtin_amdgcn_perm(tm[t][7], tm[t][6], 0x07060302u)}));
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) {
      uint32_t f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // byte 4j + kw of the span
        const uint32_t wv = rw.sp[j + kw / 4];
        f[j] = __float_as_uint((float)((wv >> (8 * (kw % 4))) & 0xffu));
      }
      const bf16x8 bf = __builtin_bit_cast(bf16x8, (u32x4{__builtin_amdgcn_perm(f[1], f[0], 0x07060302u),
                                                         __builtin_amdgcn_perm(f[3], f[2], 0x07060302u),
                                                         __builtin_amdgcn_perm(f[5], f[4], 0x07060302u),
                                                         __builtin_amdgcn_perm(f[7], f[6], 0x07060302u)}));
#pragma unroll
      for (int t = 0; t < 3; ++t) acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t], bf, acc[kw], 0, 0, 0);
    }
  };
  // this wave's groups g_begin + wave + k * waves, k < ng, two per trip (a group past the end
  // loads a valid one, masked): no branch but the loop's own, and the next group's loads are
  // issued before this group's math
  const int64_t gi0 = g_begin + wave;
  const int64_t ng = gi0 < g_end ? (g_end - gi0 + kWgWaves - 1) / kWgWaves : 0;
  if (ng > 0) {
    Raw ra, rb;
    load(gi0, ra);
    for (int64_t k = 0; k < ng; k += 2) {
      load(gi0 + (k + 1) * kWgWaves, rb);
      __builtin_amdgcn_sched_barrier(0);
      compute(ra);
      load(gi0 + (k + 2) * kWgWaves, ra);
      __builtin_amdgcn_sched_barrier(0);
      compute(rb);
    }
  }
  // bias: lanes o and o + 32 of every wave
  db = radd(db, __shfl_down(db, 32));
  if (h == 0) red[wave][o] = db;
  // the weight tiles: sum the waves through LDS, tile by tile (C/D: lane -> column o of the
  // tile, register r -> row i = 8 (r / 4) + 4 h + r % 4 = output channel)
  float *out = partial + (int64_t)blockIdx.x * (COUT * K + COUT);
#pragma unroll
  for (int t = 0; t < KW; ++t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[wave][(8 * (r / 4) + 4 * h + r % 4) * 32 + o] = acc[t][r];
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * 32; e += kWgWaves * 64) {
      float v = tile[0][e];
#pragma unroll
      for (int w = 1; w < kWgWaves; ++w) v = radd(v, tile[w][e]);
      out[(e / 32) * K + t * 32 + e % 32] = v;  // [o][kk = kw * 32 + (ci, kh)]
    }
    __syncthreads();
  }
  if (threadIdx.x < 32) {
    float v = red[0][threadIdx.x];
    for (int w = 1; w < kWgWaves; ++w) v = radd(v, red[w][threadIdx.x]);
    out[COUT * K + threadIdx.x] = v;
  }
}

// partials [blocks][COUT * K + COUT] (kk = kw * 32 + ci * KH + kh) -> gw OHWI, gb: 64
// elements per workgroup, 4 groups of 64 lanes each summing a quarter of the partials
// (coalesced rows), then the 4 group sums in fixed order
// deferred bias gradients (rth_relu_bias_grad with db = NULL) finished by the extra
// workgroups of this launch, in exactly k_bias_grad_combine's order (qnet.hip: 1024 lanes,
// G = 1024 / C lanes per channel striding the slabs, then a fixed LDS tree): each of the 256
// threads plays 4 of those virtual lanes, so the result is bit-identical to the two-launch form
constexpr int kBiasJobsMax = 4;
constexpr int kBiasVLanes = 1024;  // = qnet.hip's kCombThreads
struct BiasJobs {
  const float *part[kBiasJobsMax];
  float *db[kBiasJobsMax];
  int slabs[kBiasJobsMax], C[kBiasJobsMax];
  int n;
};

// sq (nullable): the fp64 sum of squares of the finished db (clip_grad_norm_'s partial, r06)
__device__ void bias_job(const BiasJobs &bj, int j, double *sq = nullptr) {
  __shared__ float red[kBiasVLanes];
  constexpr int Q = kBiasVLanes / 256, U = 16;
  const int C = bj.C[j], G = kBiasVLanes / C, tid = threadIdx.x, slabs = bj.slabs[j];
  const float *part = bj.part[j];
  // virtual lane vt = tid + 256 q sums slabs vt / C, + G, + 2 G, ... in that order (the order of
  // k_bias_grad_combine's lane vt); the loads of all Q lanes, U slabs each, are in flight together
  // (one round trip per U * G slabs -- 2 for conv2's 324 slabs, where a lane-by-lane loop of
  // 8-load batches took 12); the slabs past the end add +0 (the clamped load is replaced), which
  // leaves every sum unchanged
  float acc[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) acc[q] = 0.0f;
  for (int base = 0; base < slabs; base += U * G) {
    float v[Q][U];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int vt = tid + 256 * q, c = vt % C, k0 = vt / C + base;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k0 + u * G;
        v[q][u] = part[(int64_t)(kk < slabs ? kk : slabs - 1) * C + c];
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int k0 = (tid + 256 * q) / C + base;
#pragma unroll
      for (int u = 0; u < U; ++u) acc[q] = radd(acc[q], k0 + u * G < slabs ? v[q][u] : 0.0f);
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) red[tid + 256 * q] = acc[q];
  __syncthreads();
  for (int st = kBiasVLanes / 2; st >= C; st >>= 1) {
    for (int i = tid; i < st; i += 256) red[i] = radd(red[i], red[i + st]);
    __syncthreads();
  }
  if (tid < C) bj.db[j][tid] = red[tid];
  if (sq) {
    __shared__ double red4[4];
    const double d = tid < C ? (double)red[tid] : 0.0;
    const double t = block_sum(rmul(d, d), red4);
    if (tid == 0) *sq = t;
  }
}

// deferred conv2 / conv3 weight gradients (rth_conv_wgrad_f32_partials): their reduce
// workgroups follow the bias jobs' (r06)
constexpr int kWgradJobsMax = 2;
struct WgradJobs {
  WgfJob j[kWgradJobsMax];
  int n;
};

// workgroup blk of conv1's weight-gradient reduce: 64 of its E outputs, or (blk >= RB) a
// deferred bias gradient, or (past those) a reduce workgroup of a deferred weight gradient.
// sq (nullable): the fp64 sum of squares of what the workgroup finished goes to sq[blk] (r06:
// clip_grad_norm_'s partials from the backward)
template <int KH, int KW, int CIN, int COUT>
__device__ __forceinline__ void wgrad_reduce_wg(int blk, const float *__restrict__ partial, int blocks,
                                                float *__restrict__ gw, float *__restrict__ gb, const BiasJobs &bj,
                                                const WgradJobs &wj, double *__restrict__ sq) {
  constexpr int K = CIN * KH * KW, E = COUT * K + COUT, RB = (E + 63) / 64;
  __shared__ float part[4][64];
  if (blk >= RB + bj.n) {  // a deferred weight gradient
    int b = blk - RB - bj.n, j = 0;
    while (j + 1 < wj.n && b >= wgf_reduce_blocks(wj.j[j])) b -= wgf_reduce_blocks(wj.j[j++]);
    const float v = wgf_reduce_wg(wj.j[j], b);
    if (sq) {
      __shared__ double red4[4];
      const double t = block_sum(rmul((double)v, (double)v), red4);
      if (threadIdx.x == 0) sq[blk] = t;
    }
    return;
  }
  if (blk >= RB) {  // a deferred bias gradient
    bias_job(bj, blk - RB, sq ? sq + blk : nullptr);
    return;
  }
  const int grp = threadIdx.x / 64, l = threadIdx.x % 64;
  const int e = blk * 64 + l;
  const int per = (blocks + 3) / 4, w0 = grp * per, w1 = w0 + per < blocks ? w0 + per : blocks;
  float v = 0.0f;
  if (e < E) {
    int w = w0;
    for (; w + 32 <= w1; w += 32) {  // 32 loads in flight per round trip; the sum stays in w order
      float t[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) t[u] = partial[(int64_t)(w + u) * E + e];
#pragma unroll
      for (int u = 0; u < 32; ++u) v = radd(v, t[u]);
    }
    for (; w + 16 <= w1; w += 16) {
      float t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = partial[(int64_t)(w + u) * E + e];
#pragma unroll
      for (int u = 0; u < 16; ++u) v = radd(v, t[u]);
    }
    for (; w + 8 <= w1; w += 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = partial[(int64_t)(w + u) * E + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) v = radd(v, t[u]);
    }
    for (; w < w1; ++w) v = radd(v, partial[(int64_t)w * E + e]);
  }
  part[grp][l] = v;
  __syncthreads();
  if (grp != 0) return;  // (wave-uniform)
  v = radd(radd(radd(part[0][l], part[1][l]), part[2][l]), part[3][l]);
  if (sq) {  // wave 0's 64 outputs, a fixed shuffle tree
    double d = e < E ? rmul((double)v, (double)v) : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = radd(d, __shfl_down(d, o, 64));
    if (l == 0) sq[blk] = d;
  }
  if (e >= E) return;
  if (e >= COUT * K) {
    gb[e - COUT * K] = v;
    return;
  }
  const int oi = e / K, kk = e % K, kw = kk / 32, ci = (kk % 32) / KH, kh = kk % KH;
  gw[((oi * KH + kh) * KW + kw) * CIN + ci] = v;
}

template <int KH, int KW, int CIN, int COUT>
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float *__restrict__ partial, int blocks,
                                                      float *__restrict__ gw, float *__restrict__ gb, BiasJobs bj,
                                                      WgradJobs wj) {
  wgrad_reduce_wg<KH, KW, CIN, COUT>(blockIdx.x, partial, blocks, gw, gb, bj, wj, nullptr);
}

// the same reduce launch with clip_grad_norm_'s partials (r06, one rank): workgroups [0, nsq)
// are norm-partial workgroups over the gradients final before it (optim.hpp's grad_sqsum_wg,
// workgroup 0 advancing Adam's step count), the rest the reduce's, each writing the sum of
// squares of the gradients it finishes -- conv1's weight and bias, the deferred bias and weight
// gradients -- right behind them: rth_adam_prenormed then runs the update alone
template <int KH, int KW, int CIN, int COUT>
__global__ __launch_bounds__(256) void k_wgrad_reduce_norm(const float *__restrict__ partial, int blocks,
                                                           float *__restrict__ gw, float *__restrict__ gb, BiasJobs bj,
                                                           WgradJobs wj, OptArgs na, int nsq, double *__restrict__ npart,
                                                           SqStep st, int nlong) {
  // dispatch order (r06): the long workgroups first -- the deferred bias and weight-gradient
  // reduces (nlong of them: hundreds of dependent-ish loads each) -- then conv1's reduce, then the
  // norm partials of the finished gradients; every workgroup keeps its partial slot (nsq + the
  // reduce's block, or the norm block), so the sums are the same (0.504 vs 0.506 ms/step with the
  // norm workgroups first, interleaved)
  constexpr int RB = (COUT * CIN * KH * KW + COUT + 63) / 64;
  const int b = (int)blockIdx.x;
  if (b < nlong) {
    wgrad_reduce_wg<KH, KW, CIN, COUT>(RB + b, partial, blocks, gw, gb, bj, wj, npart + nsq);
  } else if (b < nlong + RB) {
    wgrad_reduce_wg<KH, KW, CIN, COUT>(b - nlong, partial, blocks, gw, gb, bj, wj, npart + nsq);
  } else {
    grad_sqsum_wg(na, b - nlong - RB, npart, st);
  }
}

constexpr int wg_per_cu() { return 2; }

}  // namespace rth

using namespace rth;

// conv3's and conv2's data gradients on the exact-split bf16 MFMA (k_conv_x9 with PAD = K - 1
// and no epilogue; conv2 as its 4 stride-parity classes, one launch, blockIdx.y = class), the
// flipped kernels packed into a per-device workspace each launch (the fp32-MFMA k_conv_dgrad
// serves the other geometries)
template <int NS>
using X9Dgrad3 = X9Geom<3, 3, 1, 64, 11, 11, NS, 3, X9_DGRAD3_KS>;
template <int NS>
using X9Dgrad2 = X9Geom<2, 2, 1, 64, 11, 11, NS, 3, X9_DGRAD2_KS, 32>;
constexpr bool dgrad3_x9() { return true; }
constexpr bool dgrad2_x9() { return true; }  // 37.8 vs 43 us alone, 0.571-0.573 vs 0.574-0.575 ms/step (r04)

static bool is_dgrad3_x9(const rth_conv_shape *shape) {
  return dgrad3_x9() && shape->input == RTH_CONV_F32_NHWC && shape->cin == 64 && shape->hin == 9 && shape->win == 9 &&
         shape->cout == 64 && shape->kh == 3 && shape->kw == 3 && shape->stride == 1;
}
static bool is_dgrad2_x9(const rth_conv_shape *shape) {
  return dgrad2_x9() && shape->input == RTH_CONV_F32_NHWC && shape->cin == 32 && shape->hin == 20 &&
         shape->win == 20 && shape->cout == 64 && shape->kh == 4 && shape->kw == 4 && shape->stride == 2;
}

// the per-device packed-kernel workspace of one dgrad geometry (allocated on first use, which
// must not be inside a graph capture; the allocation is serialised across host threads).  It is
// shared by every caller of the NULL-workspace form on that device: that form is for one stream
// at a time (include/reth_hip.h, rth_conv_dgrad); concurrent learners pass their own workspace.
static int dgrad_workspace(u32x4 **ws, size_t bytes, hipStream_t st, u32x4 **out) {
  static std::mutex mu;
  int dev = 0;
  RTH_HIP(hipGetDevice(&dev));
  RTH_REQUIRE(dev >= 0 && dev < 64, "rth_conv_dgrad: device %d out of range", dev);
  std::lock_guard<std::mutex> lock(mu);
  if (!ws[dev]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    RTH_REQUIRE(hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone,
                "rth_conv_dgrad: the first data gradient of a geometry on a device must run outside graph capture");
    RTH_HIP(hipMalloc(&ws[dev], bytes));
  }
  *out = ws[dev];
  return RTH_OK;
}

// samples per workgroup (1 .. 3): the cost model of select_launch, `classes` workgroups per
// group, with each instantiation's resident workgroups per CU from the occupancy query (the
// LDS image: 1 - 3 per CU)
static int64_t dgrad_x9_nsamp(int64_t n, int classes, const void *const *fn, int threads, int cap) {
  int64_t ns = 0;
  double best = 0.0;
  for (int64_t k = 1; k <= 3; ++k) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn[k], threads, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    const int64_t slots = (int64_t)cu_count() * (per_cu < cap ? per_cu : cap);
    const int64_t rounds = (classes * ((n + k - 1) / k) + slots - 1) / slots;
    const double cost = (double)rounds * ((double)k + 0.5);
    if (ns == 0 || cost < best) best = cost, ns = k;
  }
  return ns;
}

static int launch_dgrad_x9(const void *fn, const float *gy, int64_t n, int64_t ns, int classes, int threads,
                           const u32x4 *wpk, float *gx, hipStream_t st, const float *ymask = nullptr,
                           float *bpart = nullptr) {
  const int nsi = (int)ns;
  const int64_t grid = (n + ns - 1) / ns;
  const int64_t *n_dev = nullptr;
  const float *bias = nullptr;
  int out_nchw = 0;
  void *args[] = {(void *)&gy,  (void *)&n,  (void *)&n_dev,    (void *)&nsi,   (void *)&wpk,
                  (void *)&bias, (void *)&gx, (void *)&out_nchw, (void *)&ymask, (void *)&bpart};
  RTH_HIP(hipLaunchKernel(fn, dim3((unsigned)grid, (unsigned)classes), dim3(threads), args, 0, st));
  return RTH_OK;
}

// w == NULL: user_ws already holds the packed kernel (rth_conv_pack_many's data-gradient job)
// the samples per workgroup of conv3's data gradient at n samples (= its grid's divisor)
static int64_t dgrad3_nsamp(int64_t n, bool mask) {
  const void *fn[4] = {nullptr, reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 1, 3, X9_DGRAD3_KS, 2>),
                       reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 2, 3, X9_DGRAD3_KS, 2>),
                       reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 3, 3, X9_DGRAD3_KS, 2>)};
  const void *fm[4] = {
      nullptr, reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 1, 3, X9_DGRAD3_KS, 2, 64, 0, 1>),
      reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 2, 3, X9_DGRAD3_KS, 2, 64, 0, 1>),
      reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 3, 3, X9_DGRAD3_KS, 2, 64, 0, 1>)};
  return dgrad_x9_nsamp(n, 1, mask ? fm : fn, X9Dgrad3<1>::NT, (int)x9_wg_per_cu());
}
static const void *dgrad3_fn(int64_t ns, bool mask) {
  const void *fn[4] = {nullptr, reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 1, 3, X9_DGRAD3_KS, 2>),
                       reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 2, 3, X9_DGRAD3_KS, 2>),
                       reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 3, 3, X9_DGRAD3_KS, 2>)};
  const void *fm[4] = {
      nullptr, reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 1, 3, X9_DGRAD3_KS, 2, 64, 0, 1>),
      reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 2, 3, X9_DGRAD3_KS, 2, 64, 0, 1>),
      reinterpret_cast<const void *>(&k_conv_x9<3, 3, 1, 64, 11, 11, 3, 3, X9_DGRAD3_KS, 2, 64, 0, 1>)};
  return mask ? fm[ns] : fn[ns];
}
static int conv_dgrad_x9_conv3(const float *gy, int64_t n, const float *w, float *gx, void *user_ws, hipStream_t st,
                               const float *ymask = nullptr, float *bpart = nullptr) {
  static u32x4 *ws[64] = {};
  constexpr int PK = X9Dgrad3<1>::PACKED_U4;
  u32x4 *wpk = static_cast<u32x4 *>(user_ws);
  if (!wpk)
    if (const int rc = dgrad_workspace(ws, (size_t)PK * 16, st, &wpk)) return rc;
  RTH_REQUIRE(n * 49 * 64 * 4 < ((int64_t)1 << 31), "rth_conv_dgrad: gy of %lld samples exceeds 2 GiB", (long long)n);
  if (w) {
    hipLaunchKernelGGL((k_conv_pack_x9_dgrad<3, 3, 64, 64, 11, 11, 1, 3, X9_DGRAD3_KS>), dim3((PK + 255) / 256),
                       dim3(256), 0, st, w, wpk);
    RTH_LAUNCHED();
  }
  const bool mask = ymask != nullptr;
  const int64_t ns = dgrad3_nsamp(n, mask);
  return launch_dgrad_x9(dgrad3_fn(ns, mask), gy, n, ns, 1, X9Dgrad3<1>::NT, wpk, gx, st, ymask, bpart);
}

// conv2: gy [n, 9, 9, 64] -> gx [n, 20, 20, 32]; each class reads gy padded to 11 x 11 and
// writes its 10 x 10 pixels
static int conv_dgrad_x9_conv2(const float *gy, int64_t n, const float *w, float *gx, void *user_ws, hipStream_t st) {
  // (w == NULL: user_ws holds the 4 packed class kernels already)
  static u32x4 *ws[64] = {};
  constexpr int PK = X9Dgrad2<1>::PACKED_U4;
  u32x4 *wpk = static_cast<u32x4 *>(user_ws);
  if (!wpk)
    if (const int rc = dgrad_workspace(ws, (size_t)4 * PK * 16, st, &wpk)) return rc;
  RTH_REQUIRE(n * 400 * 32 * 4 < ((int64_t)1 << 31), "rth_conv_dgrad: gx of %lld samples exceeds 2 GiB", (long long)n);
  if (w) {
    hipLaunchKernelGGL((k_conv_pack_x9_dgrad_cls<32, 64, 1, 3, X9_DGRAD2_KS>), dim3((4 * PK + 255) / 256), dim3(256),
                       0, st, w, wpk);
    RTH_LAUNCHED();
  }
  const void *fn[4] = {
      nullptr, reinterpret_cast<const void *>(&k_conv_x9<2, 2, 1, 64, 11, 11, 1, 3, X9_DGRAD2_KS, 1, 32, 1>),
      reinterpret_cast<const void *>(&k_conv_x9<2, 2, 1, 64, 11, 11, 2, 3, X9_DGRAD2_KS, 1, 32, 1>),
      reinterpret_cast<const void *>(&k_conv_x9<2, 2, 1, 64, 11, 11, 3, 3, X9_DGRAD2_KS, 1, 32, 1>)};
  // (4 waves per workgroup at COUT = 32: as many resident as the LDS image allows)
  const int64_t ns = dgrad_x9_nsamp(n, 4, fn, X9Dgrad2<1>::NT, 4);
  return launch_dgrad_x9(fn[ns], gy, n, ns, 4, X9Dgrad2<1>::NT, wpk, gx, st);
}

extern "C" {

int rth_conv_supported(const rth_conv_shape *shape) {
  ConvLaunch l;
  if (!shape || !find_conv(*shape, &l)) return 0;
  return (shape->input & RTH_CONV_OUT_NCHW) && l.bf16x3 ? 0 : 1;  // NCHW output: not the conv1 u8 kernel
}

static void select_launch(ConvLaunch *l, int64_t n, int64_t *w_off, int64_t *nsamp);

int rth_conv_impl(const rth_conv_shape *shape, int64_t n, int32_t *nsamp_out) {
  ConvLaunch l;
  if (nsamp_out) *nsamp_out = 0;
  if (!shape || n < 1 || !find_conv(*shape, &l)) return 0;
  int64_t w_off = 0, nsamp = 0;
  select_launch(&l, n, &w_off, &nsamp);
  if (nsamp_out) *nsamp_out = (int32_t)nsamp;
  return l.x9 ? RTH_CONV_IMPL_X9 : (l.bf16x3 ? RTH_CONV_IMPL_BF16X3 : RTH_CONV_IMPL_F32);
}

int64_t rth_conv_packed_bytes(const rth_conv_shape *shape) {
  ConvLaunch l;
  return shape && find_conv(*shape, &l) ? (int64_t)l.lds_bytes : 0;
}

int rth_conv_pack(const rth_conv_shape *shape, const float *w, float *packed, void *stream) {
  RTH_REQUIRE(shape && w && packed, "rth_conv_pack: NULL argument");
  ConvLaunch l;
  RTH_REQUIRE(find_conv(*shape, &l), "rth_conv_pack: geometry not built");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(packed)) & 15) == 0,
              "rth_conv_pack: misaligned buffer");
  void *args[] = {(void *)&w, (void *)&packed};
  const int slots = l.lds_bytes / 16;
  RTH_HIP(hipLaunchKernel(l.pack, dim3((unsigned)((slots + 255) / 256)), dim3(256), args, 0, as_stream(stream)));
  return RTH_OK;
}

int rth_conv_pack_many(int32_t n, const rth_conv_shape *shapes, const float *const *w, float *const *packed,
                       void *stream) {
  RTH_REQUIRE(n >= 0 && n <= kPackMax && (n == 0 || (shapes && w && packed)), "rth_conv_pack_many: bad arguments");
  PackJob job{};
  job.n = n;
  int blocks = 0;
  for (int l = 0; l < n; ++l) {
    if (shapes[l].input & RTH_CONV_PACK_DGRAD) {  // the flipped data-gradient kernel of this forward shape
      rth_conv_shape fw = shapes[l];
      fw.input &= ~RTH_CONV_PACK_DGRAD;
      const bool d3 = is_dgrad3_x9(&fw), d2 = is_dgrad2_x9(&fw);
      RTH_REQUIRE(d3 || d2, "rth_conv_pack_many: job %d: no packed data-gradient kernel for this geometry", l);
      RTH_REQUIRE(w[l] && packed[l] && ((reinterpret_cast<uintptr_t>(w[l]) | reinterpret_cast<uintptr_t>(packed[l])) &
                                        15) == 0,
                  "rth_conv_pack_many: layer %d buffer NULL or misaligned", l);
      job.geom[l] = d3 ? kPackDgrad3 : kPackDgrad2;
      job.w[l] = w[l];
      job.packed[l] = reinterpret_cast<f32x4 *>(packed[l]);
      job.first_block[l] = blocks;
      blocks += (int)((rth_conv_dgrad_workspace(&fw) / 16 + 255) / 256);
      continue;
    }
    ConvLaunch cl;
    RTH_REQUIRE(find_conv(shapes[l], &cl, &job.geom[l]), "rth_conv_pack_many: layer %d geometry not built", l);
    RTH_REQUIRE(w[l] && packed[l] && ((reinterpret_cast<uintptr_t>(w[l]) | reinterpret_cast<uintptr_t>(packed[l])) &
                                      15) == 0,
                "rth_conv_pack_many: layer %d buffer NULL or misaligned", l);
    job.w[l] = w[l];
    job.packed[l] = reinterpret_cast<f32x4 *>(packed[l]);
    // packed form: 1 = the bf16x3 / x9 (or conv2's x9-first hybrid) image, 2 = conv3's
    // fp32-first hybrid
    job.bf16x3[l] = (cl.big && !cl.x9) ? 2 : (cl.bf16x3 || cl.x9) ? 1 : 0;
    job.first_block[l] = blocks;
    blocks += (cl.lds_bytes / 16 + 255) / 256;
  }
  job.first_block[n] = blocks;
  if (n == 0) return RTH_OK;
  hipLaunchKernelGGL(k_conv_pack_many, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), job);
  RTH_LAUNCHED();
  return RTH_OK;
}

static bool is_conv1_u8(const rth_conv_shape *s) {
  return s && s->input == RTH_CONV_U8_CHW && s->cin == 4 && s->hin == 84 && s->win == 84 && s->cout == 32 &&
         s->kh == 8 && s->kw == 8 && s->stride == 4;
}

int64_t rth_conv_wgrad_workspace(const rth_conv_shape *shape) {
  return is_conv1_u8(shape) ? (int64_t)kWgBlocks * (32 * 256 + 32) * 4 : 0;
}

// (norm: clip_grad_norm_'s partials in the reduce launch, rth_conv1_relu_wgrad_norm)
struct NormJob {
  const rth_param_tensor *sq;
  int32_t n_sq;
  double lr, beta1, beta2;
  int64_t *step;
  void *adam_ws;
  int32_t *nparts_out;
};
static int conv1_relu_wgrad(const rth_conv_shape *shape, const void *x, const int64_t *rows, const int32_t *fids,
                            int64_t n, const float *g, const float *y, float *gw, float *gb, void *workspace,
                            const rth_bias_deferred *deferred, int32_t ndeferred, const rth_wgrad_deferred *wdeferred,
                            int32_t nwdeferred, void *stream, const NormJob *norm = nullptr);

int rth_conv_relu_wgrad_ex(const rth_conv_shape *shape, const void *x, const int64_t *rows, int64_t n, const float *g,
                           const float *y, float *gw, float *gb, void *workspace, const rth_bias_deferred *deferred,
                           int32_t ndeferred, const rth_wgrad_deferred *wdeferred, int32_t nwdeferred, void *stream) {
  return conv1_relu_wgrad(shape, x, rows, nullptr, n, g, y, gw, gb, workspace, deferred, ndeferred, wdeferred,
                          nwdeferred, stream);
}

int rth_conv1_frames_relu_wgrad_ex(const rth_conv_shape *shape, const uint8_t *store, const int32_t *ids, int64_t n,
                                   const float *g, const float *y, float *gw, float *gb, void *workspace,
                                   const rth_bias_deferred *deferred, int32_t ndeferred,
                                   const rth_wgrad_deferred *wdeferred, int32_t nwdeferred, void *stream) {
  RTH_REQUIRE(store && ids && (reinterpret_cast<uintptr_t>(ids) & 15) == 0,
              "rth_conv1_frames_relu_wgrad_ex: NULL / misaligned frame store or ids");
  return conv1_relu_wgrad(shape, store, nullptr, ids, n, g, y, gw, gb, workspace, deferred, ndeferred, wdeferred,
                          nwdeferred, stream);
}

int rth_conv1_relu_wgrad_norm(const rth_conv_shape *shape, const void *x, const int64_t *rows, const int32_t *fids,
                              int64_t n, const float *g, const float *y, float *gw, float *gb, void *workspace,
                              const rth_bias_deferred *deferred, int32_t ndeferred, const rth_wgrad_deferred *wdeferred,
                              int32_t nwdeferred, const rth_param_tensor *sq, int32_t n_sq, double lr, double beta1,
                              double beta2, int64_t *step_dev,
                              void *adam_workspace_dev, int32_t *nparts_out, void *stream) {
  RTH_REQUIRE(!(rows && fids) && sq && n_sq >= 1 && n_sq <= RTH_MAX_PARAM_TENSORS && step_dev && adam_workspace_dev &&
                  nparts_out && n > 0,
              "rth_conv1_relu_wgrad_norm: bad arguments (rows and fids, %d tensors, a batch of %lld)", n_sq,
              (long long)n);
  for (int i = 0; i < n_sq; ++i)
    RTH_REQUIRE(sq[i].grad && sq[i].n >= 1, "rth_conv1_relu_wgrad_norm: tensor %d incomplete", i);
  if (fids)
    RTH_REQUIRE((reinterpret_cast<uintptr_t>(fids) & 15) == 0, "rth_conv1_relu_wgrad_norm: misaligned frame ids");
  const NormJob nj{sq, n_sq, lr, beta1, beta2, step_dev, adam_workspace_dev, nparts_out};
  return conv1_relu_wgrad(shape, x, rows, fids, n, g, y, gw, gb, workspace, deferred, ndeferred, wdeferred, nwdeferred,
                          stream, &nj);
}

static int conv1_relu_wgrad(const rth_conv_shape *shape, const void *x, const int64_t *rows, const int32_t *fids,
                            int64_t n, const float *g, const float *y, float *gw, float *gb, void *workspace,
                            const rth_bias_deferred *deferred, int32_t ndeferred, const rth_wgrad_deferred *wdeferred,
                            int32_t nwdeferred, void *stream, const NormJob *norm) {
  RTH_REQUIRE(shape && x && g && y && gw && gb && workspace && n >= 0, "rth_conv_relu_wgrad: NULL argument");
  RTH_REQUIRE(nwdeferred >= 0 && nwdeferred <= kWgradJobsMax && (nwdeferred == 0 || wdeferred),
              "rth_conv_relu_wgrad_ex: %d deferred weight gradients (at most %d)", nwdeferred, kWgradJobsMax);
  WgradJobs wj{};
  wj.n = nwdeferred;
  int wblocks = 0;
  for (int j = 0; j < nwdeferred; ++j) {
    const rth_wgrad_deferred &d = wdeferred[j];
    RTH_REQUIRE(d.gw && (d.splits == 0 || d.partial) && d.splits >= 0 && d.splits <= kWgfRedMax && d.elems > 0 &&
                    d.nb >= 0 && d.K > 0,
                "rth_conv_relu_wgrad_ex: deferred weight gradient %d malformed", j);
    wj.j[j] = WgfJob{d.partial, d.gw, d.splits, d.elems, d.nb, d.K};
    wblocks += wgf_reduce_blocks(wj.j[j]);
  }
  RTH_REQUIRE(ndeferred >= 0 && ndeferred <= kBiasJobsMax && (ndeferred == 0 || deferred),
              "rth_conv_relu_wgrad_ex: %d deferred bias gradients (at most %d)", ndeferred, kBiasJobsMax);
  BiasJobs bj{};
  bj.n = ndeferred;
  for (int j = 0; j < ndeferred; ++j) {
    const rth_bias_deferred &d = deferred[j];
    RTH_REQUIRE(d.workspace && d.db && d.C >= 4 && d.C <= 256 && (d.C & (d.C - 1)) == 0 && d.rows >= 0 &&
                    d.slabs >= 0 && d.slabs <= kBiasSlabs,
                "rth_conv_relu_wgrad_ex: deferred bias gradient %d malformed", j);
    bj.part[j] = static_cast<const float *>(d.workspace);
    bj.db[j] = d.db;
    bj.C[j] = d.C;
    bj.slabs[j] = d.slabs > 0 ? d.slabs : (int)bias_grad_slabs(d.rows, d.C);
  }
  RTH_REQUIRE(is_conv1_u8(shape), "rth_conv_relu_wgrad: only the uint8 conv1 geometry (4x84x84 -> 32, k8 s4) is built");
  float *part = static_cast<float *>(workspace);
  if (n == 0) {
    RTH_HIP(hipMemsetAsync(gw, 0, 32 * 256 * 4, as_stream(stream)));
    RTH_HIP(hipMemsetAsync(gb, 0, 32 * 4, as_stream(stream)));
    for (int j = 0; j < ndeferred; ++j)  // an empty batch: every layer's slabs are empty too
      RTH_HIP(hipMemsetAsync(deferred[j].db, 0, deferred[j].C * 4, as_stream(stream)));
    for (int j = 0; j < nwdeferred; ++j)
      RTH_HIP(hipMemsetAsync(wdeferred[j].gw, 0, (size_t)wdeferred[j].elems * 4, as_stream(stream)));
    return RTH_OK;
  }
  hipLaunchKernelGGL(fids ? k_conv1_wgrad_bf16x3<2> : (rows ? k_conv1_wgrad_bf16x3<1> : k_conv1_wgrad_bf16x3<0>),
                     dim3(kWgBlocks), dim3(kWgWaves * 64), 0, as_stream(stream), static_cast<const uint8_t *>(x),
                     fids ? reinterpret_cast<const int64_t *>(fids) : rows, n, g, y, part);
  RTH_LAUNCHED();
  constexpr int RB = (32 * 256 + 32 + 63) / 64;
  if (!norm) {
    hipLaunchKernelGGL((k_wgrad_reduce<8, 8, 4, 32>), dim3(RB + ndeferred + wblocks), dim3(256), 0, as_stream(stream),
                       part, kWgBlocks, gw, gb, bj, wj);
    RTH_LAUNCHED();
    return RTH_OK;
  }
  OptArgs na{};
  const int64_t nsq = opt_segments(norm->sq, norm->n_sq, kOptChunk, &na);
  const int64_t nparts = nsq + RB + ndeferred + wblocks;
  RTH_REQUIRE(nparts <= kMaxPartials, "rth_conv1_relu_wgrad_norm: %lld norm partials (at most %d)",
              (long long)nparts, kMaxPartials);
  auto *npart = static_cast<double *>(norm->adam_ws);  // rth_clip_adam_workspace's layout (optim.hip)
  auto *bc = reinterpret_cast<BiasCorr *>(static_cast<uint8_t *>(norm->adam_ws) + (int64_t)kMaxPartials * 8 + 16);
  const SqStep st{norm->step, bc, norm->lr, norm->beta1, norm->beta2};
  hipLaunchKernelGGL((k_wgrad_reduce_norm<8, 8, 4, 32>), dim3((unsigned)nparts), dim3(256), 0, as_stream(stream), part,
                     kWgBlocks, gw, gb, bj, wj, na, (int)nsq, npart, st, (int)(ndeferred + wblocks));
  RTH_LAUNCHED();
  *norm->nparts_out = (int32_t)nparts;
  return RTH_OK;
}

int rth_conv_relu_wgrad(const rth_conv_shape *shape, const void *x, const int64_t *rows, int64_t n, const float *g,
                        const float *y, float *gw, float *gb, void *workspace, void *stream) {
  return rth_conv_relu_wgrad_ex(shape, x, rows, n, g, y, gw, gb, workspace, nullptr, 0, nullptr, 0, stream);
}

// the kernel a hybrid geometry runs for n samples (*l becomes it; its packed weights start at
// byte *w_off) and, for the x9 kernels, the samples per workgroup: the built instantiation with
// the least estimated time, rounds x per-round time, where one workgroup is resident per CU (the
// kernel's ~160-220 VGPRs) and a round of s-sample workgroups takes ~(s + 0.5) single-sample
// times (microbench: conv3 12.3 / 20.6 / 37.2 us for s = 1 / 2 / 4 on 256 CUs, conv2 15.8 / 31 us)
static void select_launch(ConvLaunch *l, int64_t n, int64_t *w_off, int64_t *nsamp) {
  *w_off = 0;
  *nsamp = 0;
  if (l->big && n > l->big_above) {
    *w_off = l->big_off;
    *l = *l->big;
  }
  if (!l->x9) return;
  const int64_t slots = (int64_t)cu_count() * x9_wg_per_cu();
  double best = 0.0;
  for (int64_t s = 1; s <= l->x9; ++s) {
    if (!l->x9fn[s]) continue;
    const int64_t rounds = ((n + s - 1) / s + slots - 1) / slots;
    const double cost = (double)rounds * ((double)s + 0.5);
    if (*nsamp == 0 || cost < best) best = cost, *nsamp = s;
  }
}

static int conv_bias_relu(const rth_conv_shape *shape, const void *x, const int64_t *rows, int64_t n,
                          const int64_t *n_dev, const float *w, const float *bias, float *y, void *stream,
                          const int32_t *fids = nullptr) {
  RTH_REQUIRE(shape && x && w && bias && y && n >= 0, "rth_conv_bias_relu: NULL argument");
  ConvLaunch l;
  RTH_REQUIRE(find_conv(*shape, &l),
              "rth_conv_bias_relu: geometry (input %d, %d x %d x %d -> %d, k %dx%d, stride %d) not built", shape->input,
              shape->cin, shape->hin, shape->win, shape->cout, shape->kh, shape->kw, shape->stride);
  const int input = shape->input & ~RTH_CONV_OUT_NCHW, out_nchw = (shape->input & RTH_CONV_OUT_NCHW) ? 1 : 0;
  RTH_REQUIRE(!rows || input == RTH_CONV_U8_CHW, "rth_conv_bias_relu: row index needs uint8 stacks");
  RTH_REQUIRE(!out_nchw || !l.bf16x3, "rth_conv_bias_relu: NCHW output is not built for conv1 on uint8 stacks");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) & 15) == 0 &&
                  (input == RTH_CONV_U8_CHW ? (reinterpret_cast<uintptr_t>(x) & 3) == 0
                                                   : (reinterpret_cast<uintptr_t>(x) & 15) == 0),
              "rth_conv_bias_relu: misaligned buffer");
  if (n == 0) return RTH_OK;
  int64_t w_off = 0, nsamp = 0;
  select_launch(&l, n, &w_off, &nsamp);
  w = reinterpret_cast<const float *>(reinterpret_cast<const uint8_t *>(w) + w_off);
  if (l.x9) {  // one workgroup per nsamp samples
    RTH_REQUIRE(input == RTH_CONV_F32_NHWC, "rth_conv_bias_relu: the x9 kernels read f32 NHWC input");
    RTH_REQUIRE(n * (int64_t)shape->hin * shape->win * shape->cin * 4 < ((int64_t)1 << 31),
                "rth_conv_bias_relu: %lld input samples exceed the x9 kernels' 2 GiB buffer range", (long long)n);
    const int ns = (int)nsamp;
    const int64_t grid = (n + nsamp - 1) / nsamp;
    const float *xf = static_cast<const float *>(x);
    const float *no_mask = nullptr;
    float *no_part = nullptr;
    void *args[] = {(void *)&xf, (void *)&n, (void *)&n_dev, (void *)&ns, (void *)&w, (void *)&bias, (void *)&y,
                    (void *)&out_nchw, (void *)&no_mask, (void *)&no_part};
    RTH_HIP(hipLaunchKernel(l.x9fn[nsamp], dim3((unsigned)grid), dim3(l.waves * 64), args, 0, as_stream(stream)));
    return RTH_OK;
  }
  const int hout = (shape->hin - shape->kh) / shape->stride + 1, wout = (shape->win - shape->kw) / shape->stride + 1;
  // (k_conv1_u8_share, bf16x3 == 2: 31 virtual pixels of 21 per output row per tile)
  RTH_REQUIRE(l.bf16x3 != 2 || n * hout * kC1VPix < ((int64_t)1 << 31),
              "rth_conv_bias_relu: %lld conv1 samples exceed the kernel's 32-bit pixel index", (long long)n);
  const int64_t tiles = l.bf16x3 == 2 ? (n * hout * kC1VPix + kC1VPerTile - 1) / kC1VPerTile
                                      : (n * hout * wout + l.tile_px - 1) / l.tile_px * (l.nsplit > 1 ? l.nsplit : 1);
  int64_t grid = (tiles + l.waves - 1) / l.waves;
  // persistent: at most wg_per_cu() workgroups per CU (each stages the weights once)
  const int cap = wg_per_cu();
  const int64_t resident = (int64_t)cu_count() * (l.per_cu < cap ? l.per_cu : cap);
  if (grid > resident) grid = resident;
  if (l.pw) {  // every channel part gets grid / nsplit workgroups
    const int64_t ns = l.nsplit;
    grid = grid / ns * ns;
    if (grid < ns) grid = ns;
  }
  RTH_REQUIRE(!fids || (l.bf16x3 == 2 && !rows), "rth_conv1_frames_bias_relu: needs k_conv1_u8_share (not RTH_CONV1_NOSHARE)");
  void *args[] = {(void *)&x, (void *)&rows, (void *)&n, (void *)&n_dev, (void *)&w, (void *)&bias, (void *)&y,
                  l.bf16x3 == 2 ? (void *)&fids : (void *)&out_nchw};  // (k_conv1_u8_bf16x3 takes the first seven)
  // whole rounds of pixel tiles over one wave slot per SIMD (the kernel's own split rule)
  const bool ts = l.tsfn && l.waves % 4 == 0 && tiles / (grid * 4) >= l.tsfn_rounds;
  const void *fn = fids ? reinterpret_cast<const void *>(&k_conv1_u8_share<true>) : (ts ? l.tsfn : l.fn);
  RTH_HIP(hipLaunchKernel(fn, dim3((unsigned)grid), dim3(l.waves * 64), args, 0, as_stream(stream)));
  return RTH_OK;
}

int rth_conv_dgrad_supported(const rth_conv_shape *shape) {
  DgradLaunch l;
  return shape && find_dgrad(*shape, &l) ? 1 : 0;
}


int64_t rth_conv_dgrad_workspace(const rth_conv_shape *shape) {
  if (!shape) return 0;
  if (is_dgrad3_x9(shape)) return (int64_t)X9Dgrad3<1>::PACKED_U4 * 16;
  if (is_dgrad2_x9(shape)) return (int64_t)4 * X9Dgrad2<1>::PACKED_U4 * 16;
  return 0;
}

int rth_debug_conv_clock(unsigned long long *out, int32_t slots) {
  RTH_REQUIRE(out && slots >= 1 && slots <= kClockSlots, "rth_debug_conv_clock: bad arguments");
#ifdef RTH_CLOCK_STAMPS
  RTH_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_conv_clock), (size_t)slots * 2 * sizeof(unsigned long long)));
  return RTH_OK;
#else
  RTH_REQUIRE(false, "rth_debug_conv_clock: not a clock-stamp build (-DRTH_CLOCK_STAMPS)");
  return RTH_OK;
#endif
}

int rth_conv_dgrad(const rth_conv_shape *shape, const float *gy, int64_t n, const float *w, float *gx, void *stream) {
  return rth_conv_dgrad_ws(shape, gy, n, w, gx, nullptr, stream);
}

int rth_conv_dgrad_prepacked(const rth_conv_shape *shape, const float *gy, int64_t n, const void *packed, float *gx,
                             void *stream) {
  RTH_REQUIRE(shape && gy && packed && gx && n >= 0, "rth_conv_dgrad_prepacked: NULL argument");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(packed) | reinterpret_cast<uintptr_t>(gx)) &
               15) == 0,
              "rth_conv_dgrad_prepacked: misaligned buffer");
  const bool d3 = is_dgrad3_x9(shape), d2 = is_dgrad2_x9(shape);
  RTH_REQUIRE(d3 || d2, "rth_conv_dgrad_prepacked: no packed data-gradient kernel for this geometry");
  if (n == 0) return RTH_OK;
  void *ws = const_cast<void *>(packed);
  return d3 ? conv_dgrad_x9_conv3(gy, n, nullptr, gx, ws, as_stream(stream))
            : conv_dgrad_x9_conv2(gy, n, nullptr, gx, ws, as_stream(stream));
}

int rth_conv_dgrad_relu_supported(const rth_conv_shape *shape) { return shape && is_dgrad3_x9(shape) ? 1 : 0; }

int rth_conv_dgrad_relu_prepacked(const rth_conv_shape *shape, const float *gy, int64_t n, const void *packed,
                                  const float *y, float *gx, void *bias_ws, int64_t *slabs_out, void *stream) {
  RTH_REQUIRE(shape && gy && packed && y && gx && bias_ws && slabs_out && n >= 0,
              "rth_conv_dgrad_relu_prepacked: NULL argument");
  RTH_REQUIRE(is_dgrad3_x9(shape), "rth_conv_dgrad_relu_prepacked: only conv3's geometry (64x9x9, k3 s1) is built");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(packed) | reinterpret_cast<uintptr_t>(gx) |
                reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(bias_ws)) &
               15) == 0,
              "rth_conv_dgrad_relu_prepacked: misaligned buffer");
  *slabs_out = 0;
  if (n == 0) return RTH_OK;
  const int64_t slabs = (n + dgrad3_nsamp(n, true) - 1) / dgrad3_nsamp(n, true);
  RTH_REQUIRE(slabs <= kBiasSlabs, "rth_conv_dgrad_relu_prepacked: %lld samples need %lld bias slabs (at most %d)",
              (long long)n, (long long)slabs, kBiasSlabs);
  *slabs_out = slabs;
  return conv_dgrad_x9_conv3(gy, n, nullptr, gx, const_cast<void *>(packed), as_stream(stream), y,
                             static_cast<float *>(bias_ws));
}

int rth_conv_dgrad_ws(const rth_conv_shape *shape, const float *gy, int64_t n, const float *w, float *gx,
                      void *workspace, void *stream) {
  RTH_REQUIRE(shape && gy && w && gx && n >= 0, "rth_conv_dgrad: NULL argument");
  RTH_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "rth_conv_dgrad: misaligned workspace");
  if (is_dgrad3_x9(shape)) {
    RTH_REQUIRE(((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(gx)) &
                 15) == 0,
                "rth_conv_dgrad: misaligned buffer");
    if (n == 0) return RTH_OK;
    return conv_dgrad_x9_conv3(gy, n, w, gx, workspace, as_stream(stream));
  }
  if (is_dgrad2_x9(shape)) {
    RTH_REQUIRE(((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(gx)) &
                 15) == 0,
                "rth_conv_dgrad: misaligned buffer");
    if (n == 0) return RTH_OK;
    return conv_dgrad_x9_conv2(gy, n, w, gx, workspace, as_stream(stream));
  }
  DgradLaunch l;
  RTH_REQUIRE(find_dgrad(*shape, &l), "rth_conv_dgrad: geometry (%d x %d x %d -> %d, k %dx%d, stride %d) not built",
              shape->cin, shape->hin, shape->win, shape->cout, shape->kh, shape->kw, shape->stride);
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(gx)) &
               15) == 0,
              "rth_conv_dgrad: misaligned buffer");
  if (n == 0) return RTH_OK;
  RTH_REQUIRE(n * (int64_t)shape->cout * ((shape->hin - shape->kh) / shape->stride + 1) *
                      ((shape->win - shape->kw) / shape->stride + 1) * 4 < ((int64_t)1 << 31),
              "rth_conv_dgrad: gy of %lld samples exceeds the 2 GiB buffer range", (long long)n);
  const int64_t tiles = (n * l.jh * l.jw + 15) / 16;
  int64_t per_class = (tiles + l.waves - 1) / l.waves;
  const int64_t resident = (int64_t)cu_count() * l.per_cu / l.classes;
  if (per_class > resident) per_class = resident > 0 ? resident : 1;
  const int xcd = dgrad_xcd();
  if (xcd) per_class = (per_class + 7) / 8 * 8;  // whole XCD groups (spare workgroups find no tile)
  const int64_t grid = per_class * l.classes;
  void *args[] = {(void *)&gy, (void *)&n, (void *)&w, (void *)&gx, (void *)&xcd};
  RTH_HIP(hipLaunchKernel(l.fn, dim3((unsigned)grid), dim3(l.waves * 64), args, 0, as_stream(stream)));
  return RTH_OK;
}

int rth_conv_bias_relu(const rth_conv_shape *shape, const void *x, const int64_t *rows, int64_t n, const float *w,
                       const float *bias, float *y, void *stream) {
  return conv_bias_relu(shape, x, rows, n, nullptr, w, bias, y, stream);
}

int rth_conv1_frames_bias_relu(const rth_conv_shape *shape, const uint8_t *store, const int32_t *ids, int64_t n,
                               const float *w, const float *bias, float *y, void *stream) {
  RTH_REQUIRE(store && ids && (reinterpret_cast<uintptr_t>(ids) & 15) == 0,
              "rth_conv1_frames_bias_relu: NULL / misaligned frame store or ids");
  RTH_REQUIRE(shape && is_conv1_u8(shape) && !(shape->input & RTH_CONV_OUT_NCHW),
              "rth_conv1_frames_bias_relu: only the uint8 conv1 geometry (4x84x84 -> 32, k8 s4) is built");
  return conv_bias_relu(shape, store, nullptr, n, nullptr, w, bias, y, stream, ids);
}

int rth_conv_bias_relu_upto(const rth_conv_shape *shape, const void *x, const int64_t *rows, int64_t n_max,
                            const int64_t *n_dev, const float *w, const float *bias, float *y, void *stream) {
  RTH_REQUIRE(n_dev, "rth_conv_bias_relu_upto: NULL count");
  return conv_bias_relu(shape, x, rows, n_max, n_dev, w, bias, y, stream);
}

}  // extern "C"
