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
#include "common.hpp"

namespace rth {

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ float relu_c(float v) { return v < 0.0f ? 0.0f : v; }  // NaN passes, like torch

template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN>
struct ConvGeom {
  static constexpr int HOUT = (HIN - KH) / S + 1, WOUT = (WIN - KW) / S + 1, PIX = HOUT * WOUT;
  static constexpr int K = KH * KW * CIN, G = K / 16, NB = COUT / 16;
  static constexpr int LDS_F4 = G * NB * 64;  // float4 slots of the staged weights
  // input chunks in flight per wave (f32 input): a divisor of G, at most 12
  static constexpr int PREFETCH = G % 8 == 0 ? 8 : (G % 12 == 0 ? 12 : (G % 6 == 0 ? 6 : (G % 4 == 0 ? 4 : 1)));
  static constexpr int64_t STACK = (int64_t)CIN * HIN * WIN;
  static_assert(K % 16 == 0 && COUT % 16 == 0, "K and COUT must be multiples of 16");
  static_assert(MODE == 0 ? (KW * CIN) % 16 == 0 : (KW == 8 && KH % 2 == 0), "unsupported window");

  // LDS float index of weight W[o][kh][kw][ci] (OHWI storage order)
  __device__ static int lds_index(int o, int kh, int kw, int ci) {
    int g, q, t;
    if (MODE == RTH_CONV_F32_NHWC) {
      const int r = kw * CIN + ci;  // position inside the kh row
      g = kh * (KW * CIN / 16) + r / 16;
      q = (r % 16) / 4;
      t = r % 4;
    } else {
      const int rho = ci * KH + kh;  // (ci, kh) byte run
      g = rho / 2;
      q = (rho % 2) * 2 + kw / 4;
      t = kw % 4;
    }
    const int nb = o / 16, lane = q * 16 + o % 16;
    return ((g * NB + nb) * 64 + lane) * 4 + t;
  }
};

template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_conv_bias_relu(const void *__restrict__ x,
                                                              const int64_t *__restrict__ rows, int64_t n,
                                                              const float *__restrict__ w,
                                                              const float *__restrict__ bias,
                                                              float *__restrict__ y) {
  using Gm = ConvGeom<MODE, KH, KW, S, CIN, COUT, HIN, WIN>;
  constexpr int G = Gm::G, NB = Gm::NB, K = Gm::K;
  __shared__ f32x4 wl[Gm::LDS_F4];
  float *wf = reinterpret_cast<float *>(wl);

  // stage W (OHWI, contiguous) into fragment order: coalesced float4 reads
  for (int i = threadIdx.x; i < COUT * K / 4; i += WAVES * 64) {
    const float4 v = reinterpret_cast<const float4 *>(w)[i];
    const int e = 4 * i, o = e / K, rem = e % K;
    const int kh = rem / (KW * CIN), r = rem % (KW * CIN), kw = r / CIN, ci = r % CIN;
    if (MODE == RTH_CONV_F32_NHWC) {  // 4 consecutive ci -> 4 consecutive t: one LDS float4
      wl[Gm::lds_index(o, kh, kw, ci) / 4] = f32x4{v.x, v.y, v.z, v.w};
    } else {
      wf[Gm::lds_index(o, kh, kw, ci)] = v.x;
      wf[Gm::lds_index(o, kh, kw, ci + 1)] = v.y;
      wf[Gm::lds_index(o, kh, kw, ci + 2)] = v.z;
      wf[Gm::lds_index(o, kh, kw, ci + 3)] = v.w;
    }
  }
  __syncthreads();

  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int q = lane >> 4, mr = lane & 15;
  const int64_t P = n * Gm::PIX, tiles = (P + 15) / 16;
  float bl[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) bl[nb] = bias[nb * 16 + mr];

  for (int64_t tile = (int64_t)blockIdx.x * WAVES + wave; tile < tiles; tile += (int64_t)gridDim.x * WAVES) {
    int64_t p = tile * 16 + mr;
    if (p >= P) p = P - 1;  // tail lanes compute a duplicate, never stored
    const int64_t b = p / Gm::PIX;
    const int pp = (int)(p % Gm::PIX), oy = pp / Gm::WOUT, ox = pp % Gm::WOUT;
    f32x4 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    if constexpr (MODE == RTH_CONV_F32_NHWC) {
      const float *base =
          static_cast<const float *>(x) + ((b * HIN + S * oy) * WIN + S * ox) * CIN + 4 * q;
      constexpr int RC = KW * CIN / 16;  // chunks per kh row
      auto a_at = [&](int g) {
        return *reinterpret_cast<const f32x4 *>(base + (g / RC) * WIN * CIN + (g % RC) * 16);
      };
      // A ring: chunk g + D is requested while chunk g is multiplied (D chunks in flight)
      constexpr int D = Gm::PREFETCH;
      f32x4 ar[D];
#pragma unroll
      for (int d = 0; d < D; ++d) ar[d] = a_at(d);
#pragma unroll 1
      for (int g0 = 0; g0 < G; g0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int g = g0 + d;
          const f32x4 a = ar[d];
          if (g + D < G) ar[d] = a_at(g + D);
          f32x4 bv[NB];
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) bv[nb] = wl[(g * NB + nb) * 64 + lane];
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
              acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], bv[nb][t], acc[nb], 0, 0, 0);
        }
      }
    } else {
      const int64_t row = rows ? rows[b] : b;
      const uint8_t *base = static_cast<const uint8_t *>(x) + row * Gm::STACK + (int64_t)(S * oy + (q >> 1)) * WIN +
                            S * ox + 4 * (q & 1);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        // runs 2g, 2g+1 = (ci, kh), (ci, kh+1) with ci = 2g / KH, kh = 2g % KH
        const uint32_t v =
            *reinterpret_cast<const uint32_t *>(base + ((2 * g) / KH) * HIN * WIN + ((2 * g) % KH) * WIN);
        f32x4 bv[NB];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) bv[nb] = wl[(g * NB + nb) * 64 + lane];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float a = (float)((v >> (8 * t)) & 0xffu);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[nb][t], acc[nb], 0, 0, 0);
        }
      }
    }
    // C/D: lane holds column mr of rows 4q .. 4q+3
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t po = tile * 16 + 4 * q + i;
      if (po < P) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) y[po * COUT + nb * 16 + mr] = relu_c(radd(acc[nb][i], bl[nb]));
      }
    }
  }
}

struct ConvLaunch {
  const void *fn;
  int waves;
  int lds_bytes;
  int per_cu;  // resident workgroups per CU (occupancy query, cached)
};

template <int MODE, int KH, int KW, int S, int CIN, int COUT, int HIN, int WIN, int WAVES>
static ConvLaunch conv_launch() {
  using Gm = ConvGeom<MODE, KH, KW, S, CIN, COUT, HIN, WIN>;
  ConvLaunch l{reinterpret_cast<const void *>(&k_conv_bias_relu<MODE, KH, KW, S, CIN, COUT, HIN, WIN, WAVES>), WAVES,
               Gm::LDS_F4 * 16, 0};
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, l.fn, WAVES * 64, 0) != hipSuccess || blocks < 1)
    blocks = 1;
  l.per_cu = blocks;
  return l;
}

// the supported geometries (the Nature-DQN torso on 4 x 84 x 84 stacks)
static bool find_conv(const rth_conv_shape &s, ConvLaunch *out) {
  auto is = [&](int mode, int cin, int hin, int win, int cout, int kh, int kw, int st) {
    return s.input == mode && s.cin == cin && s.hin == hin && s.win == win && s.cout == cout && s.kh == kh &&
           s.kw == kw && s.stride == st;
  };
  if (is(RTH_CONV_U8_CHW, 4, 84, 84, 32, 8, 8, 4)) {
    static const ConvLaunch l = conv_launch<RTH_CONV_U8_CHW, 8, 8, 4, 4, 32, 84, 84, 4>();
    *out = l;
  } else if (is(RTH_CONV_F32_NHWC, 4, 84, 84, 32, 8, 8, 4)) {
    static const ConvLaunch l = conv_launch<RTH_CONV_F32_NHWC, 8, 8, 4, 4, 32, 84, 84, 4>();
    *out = l;
  } else if (is(RTH_CONV_F32_NHWC, 32, 20, 20, 64, 4, 4, 2)) {
    static const ConvLaunch l = conv_launch<RTH_CONV_F32_NHWC, 4, 4, 2, 32, 64, 20, 20, 8>();
    *out = l;
  } else if (is(RTH_CONV_F32_NHWC, 64, 9, 9, 64, 3, 3, 1)) {
    static const ConvLaunch l = conv_launch<RTH_CONV_F32_NHWC, 3, 3, 1, 64, 64, 9, 9, 8>();
    *out = l;
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

}  // namespace rth

using namespace rth;

extern "C" {

int rth_conv_supported(const rth_conv_shape *shape) {
  ConvLaunch l;
  return shape && find_conv(*shape, &l) ? 1 : 0;
}

int rth_conv_bias_relu(const rth_conv_shape *shape, const void *x, const int64_t *rows, int64_t n, const float *w,
                       const float *bias, float *y, void *stream) {
  RTH_REQUIRE(shape && x && w && bias && y && n >= 0, "rth_conv_bias_relu: NULL argument");
  ConvLaunch l;
  RTH_REQUIRE(find_conv(*shape, &l),
              "rth_conv_bias_relu: geometry (input %d, %d x %d x %d -> %d, k %dx%d, stride %d) not built", shape->input,
              shape->cin, shape->hin, shape->win, shape->cout, shape->kh, shape->kw, shape->stride);
  RTH_REQUIRE(!rows || shape->input == RTH_CONV_U8_CHW, "rth_conv_bias_relu: row index needs uint8 stacks");
  RTH_REQUIRE(((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y)) & 15) == 0 &&
                  (shape->input == RTH_CONV_U8_CHW ? (reinterpret_cast<uintptr_t>(x) & 3) == 0
                                                   : (reinterpret_cast<uintptr_t>(x) & 15) == 0),
              "rth_conv_bias_relu: misaligned buffer");
  if (n == 0) return RTH_OK;
  const int hout = (shape->hin - shape->kh) / shape->stride + 1, wout = (shape->win - shape->kw) / shape->stride + 1;
  const int64_t tiles = (n * hout * wout + 15) / 16;
  int64_t grid = (tiles + l.waves - 1) / l.waves;
  const int64_t resident = (int64_t)cu_count() * l.per_cu;
  if (grid > resident) grid = resident;  // persistent: each workgroup stages W once
  void *args[] = {(void *)&x, (void *)&rows, (void *)&n, (void *)&w, (void *)&bias, (void *)&y};
  RTH_HIP(hipLaunchKernel(l.fn, dim3((unsigned)grid), dim3(l.waves * 64), args, 0, as_stream(stream)));
  return RTH_OK;
}

}  // extern "C"
