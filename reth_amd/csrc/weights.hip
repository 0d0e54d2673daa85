// Learner -> actor weights as a device-resident latest-wins slot with a device version.
//
// Reference contract: perwez PUB/SUB with CONFLATE (perwez/perwez/client/socket.py:19-122,
// 302-328): the trainer publishes every send_weights_interval updates
// (test/apex-dqn/trainer.py:38-41), an actor loads when more than recv_weights_interval
// steps passed since its last load and a message is waiting (worker.py:37-41), and only the
// newest message survives.  Learner and actors of a GPU share its HBM, so the message is
// the parameters themselves: publish gathers the parameter tensors into the slot and then
// bumps the version (stream order puts the bump after the copy); acquire takes its load
// decision on the device -- version > the consumer's seen version, and (optionally) its
// step counter more than `interval` past its previous load -- so a captured actor graph
// replays it without a host branch, and copies the slot out only when it decided to.
// Several publishes before one acquire leave the last one (conflation = overwrite).
#include "common.hpp"

namespace rth {

constexpr int kWSegMax = 64;
constexpr int kWThreads = 256;

struct WSegs {
  void *ptr[kWSegMax];     // the parameter tensors (publish: sources, acquire: destinations)
  int64_t off[kWSegMax + 1];  // their dword offsets in the slot (prefix sums)
  int32_t n;
};

__device__ __forceinline__ int seg_of(const WSegs &s, int64_t w) {
  int lo = 0, hi = s.n - 1;
  while (lo < hi) {  // last segment whose offset <= w
    const int mid = (lo + hi + 1) >> 1;
    if (s.off[mid] <= w) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// dir 0: tensors -> slot (publish); dir 1: slot -> tensors (acquire, if *go)
__global__ __launch_bounds__(kWThreads) void k_weights_copy(WSegs s, uint32_t *__restrict__ slot, int dir,
                                                            const int32_t *__restrict__ go) {
  if (go && *go == 0) return;
  const int64_t total = s.off[s.n];
  for (int64_t w = (int64_t)blockIdx.x * kWThreads + threadIdx.x; w < total; w += (int64_t)gridDim.x * kWThreads) {
    const int k = seg_of(s, w);
    uint32_t *t = static_cast<uint32_t *>(s.ptr[k]) + (w - s.off[k]);
    if (dir == 0) slot[w] = *t;
    else *t = slot[w];
  }
}

__global__ void k_weights_bump(int64_t *ver) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *ver += 1;
}

// the consumer's decision (worker.py:37-41): newer version and, with a step counter, more
// than `interval` steps since the previous load; commits seen / prev and raises *go
__global__ void k_weights_gate(const int64_t *__restrict__ ver, int64_t *__restrict__ seen,
                               const int64_t *__restrict__ step, int64_t *__restrict__ prev, int64_t interval,
                               int32_t *__restrict__ go) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t v = *ver;
  bool load = v > *seen;
  if (step) load = load && (*step - *prev > interval);
  if (load) {
    *seen = v;
    if (step) *prev = *step;
  }
  *go = load ? 1 : 0;
}

}  // namespace rth

using namespace rth;

struct rth_weights {
  int64_t bytes;
  int device;
  uint32_t *slot;
  int64_t *ver;   // device version counter
  int32_t *go;    // device scratch flag when the caller passes none
};

static int make_segs(const rth_weights *h, int32_t n, void *const *ptrs, const int64_t *bytes, WSegs *s) {
  RTH_REQUIRE(n >= 1 && n <= kWSegMax && ptrs && bytes, "rth_weights: 1..%d segments expected, got %d", kWSegMax, n);
  s->n = n;
  s->off[0] = 0;
  for (int k = 0; k < n; ++k) {
    RTH_REQUIRE(ptrs[k] && bytes[k] >= 0 && bytes[k] % 4 == 0 && (reinterpret_cast<uintptr_t>(ptrs[k]) & 3) == 0,
                "rth_weights: segment %d must be a 4-byte aligned device buffer of a multiple of 4 bytes", k);
    s->ptr[k] = ptrs[k];
    s->off[k + 1] = s->off[k] + bytes[k] / 4;
  }
  RTH_REQUIRE(s->off[n] * 4 == h->bytes, "rth_weights: segments hold %lld bytes, the slot %lld",
              (long long)(s->off[n] * 4), (long long)h->bytes);
  return RTH_OK;
}

static unsigned copy_grid(int64_t dwords) {
  const int64_t b = (dwords + kWThreads - 1) / kWThreads;
  return (unsigned)(b < 1024 ? (b > 0 ? b : 1) : 1024);
}

extern "C" {

int rth_weights_create(int64_t bytes, int device, rth_weights **out) {
  RTH_REQUIRE(out && bytes > 0 && bytes % 4 == 0, "rth_weights_create: bytes must be a positive multiple of 4");
  RTH_HIP(hipSetDevice(device));
  auto *h = new rth_weights{bytes, device, nullptr, nullptr, nullptr};
  if (hipMalloc(&h->slot, (size_t)bytes) != hipSuccess || hipMalloc(&h->ver, 16) != hipSuccess) {
    (void)hipFree(h->slot);
    delete h;
    set_error("rth_weights_create: hipMalloc(%lld) failed", (long long)bytes);
    return RTH_ERR_NOMEM;
  }
  h->go = reinterpret_cast<int32_t *>(h->ver + 1);
  RTH_HIP(hipMemset(h->ver, 0, 16));
  RTH_HIP(hipMemset(h->slot, 0, (size_t)bytes));
  *out = h;
  return RTH_OK;
}

int rth_weights_destroy(rth_weights *h) {
  if (!h) return RTH_OK;
  (void)hipSetDevice(h->device);
  (void)hipFree(h->slot);
  (void)hipFree(h->ver);
  delete h;
  return RTH_OK;
}

static int weights_put(rth_weights *h, int32_t n, const void *const *src, const int64_t *bytes, void *stream,
                       int bump) {
  RTH_REQUIRE(h, "rth_weights_publish: NULL handle");
  WSegs s;
  int rc = make_segs(h, n, const_cast<void *const *>(src), bytes, &s);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_weights_copy, dim3(copy_grid(s.off[n])), dim3(kWThreads), 0, st, s, h->slot, 0, nullptr);
  RTH_LAUNCHED();
  if (!bump) return RTH_OK;
  hipLaunchKernelGGL(k_weights_bump, dim3(1), dim3(64), 0, st, h->ver);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_weights_publish(rth_weights *h, int32_t n, const void *const *src, const int64_t *bytes, void *stream) {
  return weights_put(h, n, src, bytes, stream, 1);
}

int rth_weights_fill(rth_weights *h, int32_t n, const void *const *src, const int64_t *bytes, void *stream) {
  return weights_put(h, n, src, bytes, stream, 0);
}

int rth_weights_acquire(rth_weights *h, int32_t n, void *const *dst, const int64_t *bytes, int64_t *seen_dev,
                        const int64_t *step_dev, int64_t *prev_dev, int64_t interval, int32_t *loaded_dev,
                        void *stream) {
  RTH_REQUIRE(h && seen_dev && (!step_dev || prev_dev), "rth_weights_acquire: bad arguments");
  WSegs s;
  int rc = make_segs(h, n, dst, bytes, &s);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  int32_t *go = loaded_dev ? loaded_dev : h->go;
  hipLaunchKernelGGL(k_weights_gate, dim3(1), dim3(64), 0, st, h->ver, seen_dev, step_dev, prev_dev, interval, go);
  RTH_LAUNCHED();
  hipLaunchKernelGGL(k_weights_copy, dim3(copy_grid(s.off[n])), dim3(kWThreads), 0, st, s, h->slot, 1, go);
  RTH_LAUNCHED();
  return RTH_OK;
}

int rth_weights_version(const rth_weights *h, int64_t *out) {
  RTH_REQUIRE(h && out, "rth_weights_version: bad arguments");
  RTH_HIP(hipMemcpy(out, h->ver, 8, hipMemcpyDeviceToHost));
  return RTH_OK;
}

int64_t rth_weights_bytes(const rth_weights *h) { return h ? h->bytes : -1; }

int rth_weights_version_ptr(rth_weights *h, int64_t **out_dev) {
  RTH_REQUIRE(h && out_dev, "rth_weights_version_ptr: bad arguments");
  *out_dev = h->ver;
  return RTH_OK;
}

}  // extern "C"
