// Shared by wgrad.hip (rth_conv_wgrad_f32 / _x9) and conv.hip (conv1's weight-gradient reduce
// launch, which also finishes deferred conv2 / conv3 weight gradients, r06): the fixed-order
// reduce of a weight gradient's split partials.  Reference: the weight gradients of
// reth/reth/algorithm/dqn/dqn_model.py:14-20 under dqn_solver.py:117 (loss.backward()).
#pragma once

#include "common.hpp"

namespace rth {

constexpr int kWgfRedMax = 128;  // splits per element at most
constexpr int kWgfRedElems = 256;  // elements per reduce workgroup (one per lane)

// one weight gradient's partials [splits][elems]; nb > 0: the elements are in k_conv_wgrad_f32's
// accumulator order (column groups of 32 * nb kk, 32x32 blocks, register, lane) and scatter to
// OHWI gw[co * K + kk]; nb == 0: already OHWI (k_conv_wgrad_x9)
struct WgfJob {
  const float *part;
  float *gw;
  int splits, elems, nb, K;
};

__host__ __device__ inline int wgf_reduce_blocks(const WgfJob &j) {
  return (j.elems + kWgfRedElems - 1) / kWgfRedElems;
}

// reduce workgroup blk of job j: lane t sums the splits of element blk * 256 + t in split
// order (32 loads in flight per round trip) and writes it to gw; returns the sum (0 past elems)
__device__ __forceinline__ float wgf_reduce_wg(const WgfJob &j, int blk) {
  const int e = blk * kWgfRedElems + (int)threadIdx.x;
  if (e >= j.elems) return 0.0f;
  float s = 0.0f;
  int k = 0;
  for (; k + 32 <= j.splits; k += 32) {
    float t[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) t[u] = j.part[(int64_t)(k + u) * j.elems + e];
#pragma unroll
    for (int u = 0; u < 32; ++u) s = radd(s, t[u]);
  }
  for (; k + 8 <= j.splits; k += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = j.part[(int64_t)(k + u) * j.elems + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = radd(s, t[u]);
  }
  for (; k < j.splits; ++k) s = radd(s, j.part[(int64_t)k * j.elems + e]);
  if (j.nb == 0) {
    j.gw[e] = s;
    return s;
  }
  // e = ((g * 2 * nb + blk) * 16 + r) * 64 + lane, blk = c * nb + n', g the column group of
  // 32 * nb columns; D[row][col] of the 32x32 block: col = lane & 31,
  // row = (r / 4) * 8 + (lane / 32) * 4 + r % 4; co = 2 row + c, kk = 32 nb g + nb col + n'
  const int nb = j.nb, tile = 2 * nb * 1024, g = e / tile, t = e - g * tile;
  const int b = t >> 10, r = (t >> 6) & 15, l = t & 63;
  const int c = b / nb, n2 = b - c * nb;
  const int row = (r >> 2) * 8 + (l >> 5) * 4 + (r & 3), col = l & 31;
  j.gw[(2 * row + c) * j.K + g * nb * 32 + nb * col + n2] = s;
  return s;
}

}  // namespace rth
