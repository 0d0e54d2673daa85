// Atari observation preprocessing on gfx950: MaxAndSkip max-pool + WarpFrame (gray, 84x84
// INTER_AREA) + FrameStack, one launch for every actor, writing uint8 stacks straight into
// the actors' frame ring in HBM (no host cv2, no float32 frames).
//
// Reference: reth/reth/env/util.py:121-149 (MaxAndSkipEnv: max over the last two raw
// frames of the skip window), :161-176 (WarpFrame: cv2.cvtColor(RGB2GRAY) then
// cv2.resize(84x84, INTER_AREA)), :179-209 (FrameStack, k = 4) and :281-297
// (ImageToPyTorch: the stack as (k, 84, 84), oldest frame first).
//
// cv2 is a third-party dependency absent from this image; its published 8-bit algorithms
// are restated (OpenCV imgproc color / resize):
//   gray  = (R*4899 + G*9617 + B*1868 + 8192) >> 14       (fixed point, yuv_shift 14)
//   area  non-integer scale: per output pixel the source rows/columns it covers with
//         fractional weights (computeResizeAreaTab: alpha = overlap / cell size, float),
//         buf = sum_x S*alpha_x (in table order), sum = sum_y beta_y*buf (float), then
//         saturate_cast<uchar> (round half to even, clamp).
// The oracle (oracle/oracle.py: warp_frame) restates the same float32 operation order.
#include <cmath>
#include <vector>

#include "common.hpp"

namespace rth {

constexpr int kMaxTaps = 8;  // source rows / columns one output pixel may touch

struct AreaTab {  // per output coordinate: taps [first, first + count) of (src index, weight)
  int first, count;
};

__device__ __forceinline__ uint32_t gray_u8(uint32_t r, uint32_t g, uint32_t b) {
  return (r * 4899u + g * 9617u + b * 1868u + 8192u) >> 14;
}

// one workgroup per (actor, output row); lane = output column
__global__ void k_atari_step(const uint8_t *__restrict__ raw, int64_t n, int H, int W, int OH, int OW, int K,
                             const AreaTab *__restrict__ xt, const int *__restrict__ xsrc,
                             const float *__restrict__ xw, const AreaTab *__restrict__ yt,
                             const int *__restrict__ ysrc, const float *__restrict__ yw, uint8_t *__restrict__ frames,
                             int ring, const int64_t *__restrict__ prev_slot, const int64_t *__restrict__ new_slot,
                             const uint8_t *__restrict__ reset, uint8_t *__restrict__ out_frame) {
  const int64_t i = blockIdx.x / OH;
  const int dy = blockIdx.x % OH;
  const int dx = threadIdx.x;
  if (i >= n || dx >= OW) return;
  const int64_t plane = (int64_t)H * W * 3;
  const uint8_t *f0 = raw + i * 2 * plane, *f1 = f0 + plane;
  const AreaTab ty = yt[dy], tx = xt[dx];
  float sum = 0.0f;
  for (int j = 0; j < ty.count; ++j) {
    const int sy = ysrc[ty.first + j];
    const float beta = yw[ty.first + j];
    float buf = 0.0f;
    for (int k = 0; k < tx.count; ++k) {
      const int64_t o = ((int64_t)sy * W + xsrc[tx.first + k]) * 3;
      const uint32_t r = max(f0[o], f1[o]), g = max(f0[o + 1], f1[o + 1]), b = max(f0[o + 2], f1[o + 2]);
      buf = radd(buf, rmul((float)gray_u8(r, g, b), xw[tx.first + k]));
    }
    sum = j == 0 ? rmul(beta, buf) : radd(sum, rmul(beta, buf));
  }
  float v = rintf(sum);  // saturate_cast<uchar>: cvRound, then clamp
  const uint8_t px = (uint8_t)(v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v));
  const int64_t pix = (int64_t)dy * OW + dx, pl = (int64_t)OH * OW;
  if (out_frame) out_frame[i * pl + pix] = px;
  if (!frames) return;
  uint8_t *dst = frames + (i * ring + new_slot[i]) * K * pl;
  if (reset && reset[i]) {  // FrameStack.reset: the first observation k times
    for (int p = 0; p < K; ++p) dst[p * pl + pix] = px;
    return;
  }
  const uint8_t *src = frames + (i * ring + prev_slot[i]) * K * pl;
  for (int p = 0; p + 1 < K; ++p) dst[p * pl + pix] = src[(p + 1) * pl + pix];  // deque drops the oldest
  dst[(K - 1) * pl + pix] = px;
}

// WarpFrame of one output pixel (dy, dx) from the max of two raw RGB frames (f0 == f1: one
// frame, no pair max -- MaxAndSkip.reset returns the reset screen itself, util.py:129-130)
__device__ __forceinline__ uint8_t warp_pixel(const uint8_t *__restrict__ f0, const uint8_t *__restrict__ f1, int W,
                                              const AreaTab ty, const AreaTab tx, const int *__restrict__ xsrc,
                                              const float *__restrict__ xw, const int *__restrict__ ysrc,
                                              const float *__restrict__ yw) {
  float sum = 0.0f;
  for (int j = 0; j < ty.count; ++j) {
    const int sy = ysrc[ty.first + j];
    const float beta = yw[ty.first + j];
    float buf = 0.0f;
    for (int k = 0; k < tx.count; ++k) {
      const int64_t o = ((int64_t)sy * W + xsrc[tx.first + k]) * 3;
      const uint32_t r = max(f0[o], f1[o]), g = max(f0[o + 1], f1[o + 1]), b = max(f0[o + 2], f1[o + 2]);
      buf = radd(buf, rmul((float)gray_u8(r, g, b), xw[tx.first + k]));
    }
    sum = j == 0 ? rmul(beta, buf) : radd(sum, rmul(beta, buf));
  }
  const float v = rintf(sum);  // saturate_cast<uchar>: cvRound, then clamp
  return (uint8_t)(v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v));
}

// The Ape-X actors' Atari env mode (reth_amd/actors.py env="atari"): after the actor tail
// assigned this step's stack handles (s0_h = the observation acted on, s1_h = the next one;
// cur_slot = where the next observation lives: s1's slot, or a reset slot after done), the
// raw frame pair of each actor becomes the new top frame of s1 (FrameStack shift of s0), and
// -- done -- the reset observation goes into cur_slot: Worker.step calls env.reset()
// (presets/worker.py:146-148), whose MaxAndSkip.reset returns the emulator's fresh reset
// screen (util.py:129-130, no pair max), warped, k times (FrameStack.reset, util.py:191-196).
__global__ void k_atari_env(const uint8_t *__restrict__ raw, int64_t n, int H, int W, int OH, int OW, int K,
                            const AreaTab *__restrict__ xt, const int *__restrict__ xsrc, const float *__restrict__ xw,
                            const AreaTab *__restrict__ yt, const int *__restrict__ ysrc, const float *__restrict__ yw,
                            uint8_t *__restrict__ frames, int ring, const int64_t *__restrict__ s0_h,
                            const int64_t *__restrict__ s1_h, const float *__restrict__ done,
                            const int64_t *__restrict__ cur_slot, const uint8_t *__restrict__ reset_raw) {
  const int64_t i = blockIdx.x / OH;
  const int dy = blockIdx.x % OH;
  const int dx = threadIdx.x;
  if (i >= n || dx >= OW) return;
  const int64_t plane = (int64_t)H * W * 3;
  const uint8_t *f0 = raw + i * 2 * plane, *f1 = f0 + plane;
  const AreaTab ty = yt[dy], tx = xt[dx];
  const uint8_t px = warp_pixel(f0, f1, W, ty, tx, xsrc, xw, ysrc, yw);
  const int64_t pix = (int64_t)dy * OW + dx, pl = (int64_t)OH * OW;
  uint8_t *dst = frames + s1_h[i] * K * pl;
  const uint8_t *src = frames + s0_h[i] * K * pl;
  for (int p = 0; p + 1 < K; ++p) dst[p * pl + pix] = src[(p + 1) * pl + pix];
  dst[(K - 1) * pl + pix] = px;
  if (done[i] != 0.0f) {  // workgroup-uniform (one actor per workgroup)
    const uint8_t *fr = reset_raw + i * plane;
    const uint8_t rpx = warp_pixel(fr, fr, W, ty, tx, xsrc, xw, ysrc, yw);
    uint8_t *rs = frames + (i * ring + cur_slot[i]) * K * pl;
    for (int p = 0; p < K; ++p) rs[p * pl + pix] = rpx;
  }
}

// the synthetic reset screens (the stand-in for the emulator's reset output): actor i's frame
// of device Philox (seed, step *t_dev, stream STREAM_ATARI_RESET), generated only where
// done[i] != 0 -- the only rows k_atari_env reads it for.  grid (vector chunks, actors)
__global__ __launch_bounds__(256) void k_atari_synth_reset(uint4 *__restrict__ raw, int64_t vec_per_frame, uint64_t seed,
                                                           const int64_t *__restrict__ t_dev,
                                                           const float *__restrict__ done) {
  const int64_t i = blockIdx.y;
  if (done[i] == 0.0f) return;
  const int64_t t = *t_dev;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < vec_per_frame; v += (int64_t)gridDim.x * 256) {
    const int64_t g = i * vec_per_frame + v;
    uint32_t c[4] = {(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)t, STREAM_ATARI_RESET | ((uint32_t)(t >> 32) << 8)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    raw[g] = make_uint4(c[0], c[1], c[2], c[3]);
  }
}

// raw emulator frames from device Philox (the synthetic stand-in for ALE's screen output):
// 16 bytes per counter, counter = (vector index, step t), stream STREAM_ATARI
__global__ __launch_bounds__(256) void k_atari_synth_raw(uint4 *__restrict__ raw, int64_t nvec, uint64_t seed,
                                                         const int64_t *__restrict__ t_dev) {
  const int64_t t = *t_dev;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    uint32_t c[4] = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)t, STREAM_ATARI | ((uint32_t)(t >> 32) << 8)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    raw[v] = make_uint4(c[0], c[1], c[2], c[3]);
  }
}

// computeResizeAreaTab for one axis: entries (dst, src, weight) in OpenCV's order
static void area_tab(int ssize, int dsize, double scale, std::vector<AreaTab> &tab, std::vector<int> &src,
                     std::vector<float> &w) {
  tab.assign(dsize, AreaTab{0, 0});
  for (int dx = 0; dx < dsize; ++dx) {
    const double f1 = dx * scale, f2 = f1 + scale;
    const double cell = std::min(scale, ssize - f1);
    int s1 = (int)std::ceil(f1), s2 = (int)std::floor(f2);
    s2 = std::min(s2, ssize - 1);
    s1 = std::min(s1, s2);
    tab[dx].first = (int)src.size();
    if (s1 - f1 > 1e-3) {
      src.push_back(s1 - 1);
      w.push_back((float)((s1 - f1) / cell));
    }
    for (int s = s1; s < s2; ++s) {
      src.push_back(s);
      w.push_back((float)(1.0 / cell));
    }
    if (f2 - s2 > 1e-3) {
      src.push_back(s2);
      w.push_back((float)(std::min(std::min(f2 - s2, 1.0), cell) / cell));
    }
    tab[dx].count = (int)src.size() - tab[dx].first;
  }
}

}  // namespace rth

using namespace rth;

struct rth_atari {
  int H, W, OH, OW, device;
  AreaTab *xt, *yt;
  int *xsrc, *ysrc;
  float *xw, *yw;
};

extern "C" {

int rth_atari_destroy(rth_atari *h) {
  if (!h) return RTH_OK;
  (void)hipSetDevice(h->device);
  for (void *p : {(void *)h->xt, (void *)h->yt, (void *)h->xsrc, (void *)h->ysrc, (void *)h->xw, (void *)h->yw})
    if (p) (void)hipFree(p);
  delete h;
  return RTH_OK;
}

int rth_atari_create(int32_t in_h, int32_t in_w, int32_t out_h, int32_t out_w, int device, rth_atari **out) {
  RTH_REQUIRE(out, "rth_atari_create: NULL out");
  RTH_REQUIRE(in_h >= out_h && in_w >= out_w && out_h >= 1 && out_w >= 1 && out_w <= 1024,
              "rth_atari_create: only downscaling to <= 1024 columns (INTER_AREA), got %dx%d -> %dx%d", in_h, in_w,
              out_h, out_w);
  // cv::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale
  const double sx = 1.0 / ((double)out_w / in_w), sy = 1.0 / ((double)out_h / in_h);
  RTH_REQUIRE(!(sx == std::floor(sx) && sy == std::floor(sy)),
              "rth_atari_create: integer scale factors take OpenCV's resizeAreaFast path, not restated");
  std::vector<AreaTab> xt, yt;
  std::vector<int> xs, ys;
  std::vector<float> xw, yw;
  area_tab(in_w, out_w, sx, xt, xs, xw);
  area_tab(in_h, out_h, sy, yt, ys, yw);
  for (const auto &t : xt) RTH_REQUIRE(t.count <= kMaxTaps, "rth_atari_create: too many taps");
  for (const auto &t : yt) RTH_REQUIRE(t.count <= kMaxTaps, "rth_atari_create: too many taps");
  RTH_HIP(hipSetDevice(device));
  auto *h = new rth_atari{in_h, in_w, out_h, out_w, device, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  auto up = [&](void **dst, const void *src, size_t bytes) {
    if (hipMalloc(dst, bytes) != hipSuccess) return false;
    return hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  const bool ok = up((void **)&h->xt, xt.data(), xt.size() * sizeof(AreaTab)) &&
                  up((void **)&h->yt, yt.data(), yt.size() * sizeof(AreaTab)) &&
                  up((void **)&h->xsrc, xs.data(), xs.size() * 4) && up((void **)&h->ysrc, ys.data(), ys.size() * 4) &&
                  up((void **)&h->xw, xw.data(), xw.size() * 4) && up((void **)&h->yw, yw.data(), yw.size() * 4);
  if (!ok) {
    rth_atari_destroy(h);
    set_error("rth_atari_create: device table upload failed");
    return RTH_ERR_NOMEM;
  }
  *out = h;
  return RTH_OK;
}

int rth_atari_step(rth_atari *h, const uint8_t *raw, int64_t n, uint8_t *frames, int32_t ring, int32_t stack,
                   const int64_t *prev_slot, const int64_t *new_slot, const uint8_t *reset, uint8_t *out_frame,
                   void *stream) {
  RTH_REQUIRE(h && raw && n >= 0, "rth_atari_step: bad arguments");
  RTH_REQUIRE(frames || out_frame, "rth_atari_step: nothing to write");
  RTH_REQUIRE(!frames || (ring >= 2 && stack >= 1 && new_slot && prev_slot),
              "rth_atari_step: frame-ring arguments incomplete");
  if (n == 0) return RTH_OK;
  const int threads = (h->OW + 63) / 64 * 64;
  hipLaunchKernelGGL(k_atari_step, dim3((unsigned)(n * h->OH)), dim3(threads), 0, as_stream(stream), raw, n, h->H,
                     h->W, h->OH, h->OW, stack, h->xt, h->xsrc, h->xw, h->yt, h->ysrc, h->yw, frames, ring, prev_slot,
                     new_slot, reset, out_frame);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_atari_env_step(rth_atari *h, const uint8_t *raw, int64_t n, uint8_t *frames, int32_t ring, int32_t stack,
                       const int64_t *s0_h, const int64_t *s1_h, const float *done, const int64_t *cur_slot,
                       const uint8_t *reset_raw, void *stream) {
  RTH_REQUIRE(h && raw && frames && s0_h && s1_h && done && cur_slot && reset_raw && n >= 0 && ring >= 2 && stack >= 1,
              "rth_atari_env_step: bad arguments");
  if (n == 0) return RTH_OK;
  const int threads = (h->OW + 63) / 64 * 64;
  hipLaunchKernelGGL(k_atari_env, dim3((unsigned)(n * h->OH)), dim3(threads), 0, as_stream(stream), raw, n, h->H,
                     h->W, h->OH, h->OW, stack, h->xt, h->xsrc, h->xw, h->yt, h->ysrc, h->yw, frames, ring, s0_h, s1_h,
                     done, cur_slot, reset_raw);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_atari_synth_reset(uint8_t *reset_raw, int64_t n, int64_t frame_bytes, uint64_t seed, const int64_t *t_dev,
                          const float *done, void *stream) {
  RTH_REQUIRE(reset_raw && t_dev && done && n >= 0 && frame_bytes > 0 && frame_bytes % 16 == 0 &&
                  (reinterpret_cast<uintptr_t>(reset_raw) & 15) == 0 && n <= 65535,
              "rth_atari_synth_reset: bad arguments (16-byte aligned frames, a multiple of 16 bytes, n <= 65535)");
  if (n == 0) return RTH_OK;
  const int64_t vec = frame_bytes / 16, chunks = (vec + 255) / 256;
  hipLaunchKernelGGL(k_atari_synth_reset, dim3((unsigned)(chunks < 64 ? chunks : 64), (unsigned)n), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<uint4 *>(reset_raw), vec, seed, t_dev, done);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_atari_synth_raw(uint8_t *raw, int64_t nbytes, uint64_t seed, const int64_t *t_dev, void *stream) {
  RTH_REQUIRE(raw && t_dev && nbytes >= 0 && nbytes % 16 == 0 && (reinterpret_cast<uintptr_t>(raw) & 15) == 0,
              "rth_atari_synth_raw: bad arguments (16-byte aligned, a multiple of 16 bytes)");
  const int64_t nvec = nbytes / 16;
  if (nvec == 0) return RTH_OK;
  const int64_t want = (nvec + 255) / 256;
  hipLaunchKernelGGL(k_atari_synth_raw, dim3((unsigned)(want < 4096 ? want : 4096)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<uint4 *>(raw), nvec, seed, t_dev);
  RTH_LAUNCHED();
  return RTH_OK;
}

}  // extern "C"
