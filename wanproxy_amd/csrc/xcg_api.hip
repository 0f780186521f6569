// Host side of the C ABI declared in include/xcgpu.h.
//
// A context pins a device and the encoder configuration the reference keeps
// in XCodecEncoder / XCodecCache (stream_ = !cache_->out_of_band(),
// xcodec/xcodec_encoder.cc:40-46).  All work is enqueued on the caller's
// stream; nothing here allocates or synchronises inside xcg_encode_batch, so a
// caller may capture it into a hipGraph.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/xcgpu.h"

extern "C" int xcg_launch_encode_independent(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint32_t,
                                             uint32_t, uint8_t*, const uint64_t*, uint64_t*, uint32_t*, int32_t*,
                                             hipStream_t);
extern "C" int xcg_launch_window_hashes(const uint8_t*, uint64_t, uint64_t*, hipStream_t);
extern "C" int xcg_launch_segment_hashes(const uint8_t*, uint64_t, uint64_t*, hipStream_t);

struct xcg_ctx {
  int device;
  uint32_t flags;
  int32_t* d_status;   // sticky internal-overflow word
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

const char* xcg_version(void) { return "xcgpu 0.1 gfx950"; }

const char* xcg_strerror(int status) {
  switch (status) {
    case XCG_OK: return "ok";
    case XCG_EHIP: return "HIP runtime error";
    case XCG_ENOMEM: return "out of device memory";
    case XCG_EINVAL: return "invalid argument";
    case XCG_EOVERFLOW: return "internal table overflow";
    case XCG_ENOTSUP: return "not supported";
    default: return "unknown status";
  }
}

uint64_t xcg_encode_bound(uint32_t len) { return 2ull * len + 16ull; }

int xcg_ctx_create(int device, uint32_t flags, xcg_ctx** out) {
  if (!out) return XCG_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return XCG_EINVAL;
  if (flags & ~(XCG_FLAG_OOB | XCG_FLAG_NULLCACHE)) return XCG_EINVAL;
  DeviceGuard g(device);
  xcg_ctx* c = new xcg_ctx{device, flags, nullptr};
  if (hipMalloc(&c->d_status, 16) != hipSuccess) {
    delete c;
    return XCG_ENOMEM;
  }
  if (hipMemset(c->d_status, 0, 16) != hipSuccess) {
    (void)hipFree(c->d_status);
    delete c;
    return XCG_EHIP;
  }
  *out = c;
  return XCG_OK;
}

void xcg_ctx_destroy(xcg_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  (void)hipFree(c->d_status);
  delete c;
}

int xcg_ctx_status(xcg_ctx* c) {
  if (!c) return XCG_EINVAL;
  DeviceGuard g(c->device);
  int32_t st = 0;
  if (hipDeviceSynchronize() != hipSuccess) return XCG_EHIP;
  if (hipMemcpy(&st, c->d_status, sizeof st, hipMemcpyDeviceToHost) != hipSuccess) return XCG_EHIP;
  return st ? XCG_EOVERFLOW : XCG_OK;
}

int xcg_encode_batch(xcg_ctx* c, int semantics, const uint8_t* d_in, const uint64_t* d_chunk_off,
                     const uint32_t* d_chunk_len, uint32_t n, uint32_t max_chunk_len, uint8_t* d_out,
                     const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_stats, void* stream) {
  if (!c) return XCG_EINVAL;
  if (n == 0) return XCG_OK;
  if (!d_in || !d_chunk_off || !d_chunk_len || !d_out || !d_out_off || !d_out_len) return XCG_EINVAL;
  if (semantics != XCG_SEM_INDEPENDENT) return XCG_ENOTSUP;
  if (max_chunk_len > (1u << 19)) return XCG_EINVAL;
  DeviceGuard g(c->device);
  int rc = xcg_launch_encode_independent(d_in, d_chunk_off, d_chunk_len, n, max_chunk_len, c->flags, d_out,
                                         d_out_off, d_out_len, d_stats, c->d_status, (hipStream_t)stream);
  return rc == 0 ? XCG_OK : (rc == -22 ? XCG_EINVAL : XCG_EHIP);
}

int xcg_encode_host(xcg_ctx* c, int semantics, const uint8_t* h_in, uint64_t in_len, const uint64_t* h_chunk_off,
                    const uint32_t* h_chunk_len, uint32_t n, uint8_t* h_out, uint64_t out_cap,
                    const uint64_t* h_out_off, uint64_t* h_out_len) {
  if (!c || (n && (!h_in || !h_chunk_off || !h_chunk_len || !h_out || !h_out_off || !h_out_len))) return XCG_EINVAL;
  if (n == 0) return XCG_OK;
  uint32_t maxlen = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (h_chunk_off[i] + h_chunk_len[i] > in_len) return XCG_EINVAL;
    if (h_out_off[i] + xcg_encode_bound(h_chunk_len[i]) > out_cap) return XCG_EINVAL;
    if (h_chunk_len[i] > maxlen) maxlen = h_chunk_len[i];
  }
  DeviceGuard g(c->device);
  uint8_t *d_in = nullptr, *d_out = nullptr;
  uint64_t *d_off = nullptr, *d_oo = nullptr, *d_ol = nullptr;
  uint32_t* d_len = nullptr;
  int rc = XCG_OK;
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return XCG_EHIP;
  do {
    if (hipMalloc(&d_in, in_len ? in_len : 1) != hipSuccess || hipMalloc(&d_out, out_cap ? out_cap : 1) != hipSuccess ||
        hipMalloc(&d_off, 8ull * n) != hipSuccess || hipMalloc(&d_oo, 8ull * n) != hipSuccess ||
        hipMalloc(&d_ol, 8ull * n) != hipSuccess || hipMalloc(&d_len, 4ull * n) != hipSuccess) {
      rc = XCG_ENOMEM;
      break;
    }
    if (hipMemcpyAsync(d_in, h_in, in_len, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_off, h_chunk_off, 8ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_oo, h_out_off, 8ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_len, h_chunk_len, 4ull * n, hipMemcpyHostToDevice, st) != hipSuccess) {
      rc = XCG_EHIP;
      break;
    }
    rc = xcg_encode_batch(c, semantics, d_in, d_off, d_len, n, maxlen, d_out, d_oo, d_ol, nullptr, st);
    if (rc != XCG_OK) break;
    std::vector<uint64_t> ol(n);
    if (hipMemcpyAsync(ol.data(), d_ol, 8ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      rc = XCG_EHIP;
      break;
    }
    // Copy back only the bytes each slot actually holds.
    for (uint32_t i = 0; i < n; ++i) {
      h_out_len[i] = ol[i];
      if (ol[i] && hipMemcpyAsync(h_out + h_out_off[i], d_out + h_out_off[i], ol[i], hipMemcpyDeviceToHost, st) !=
                       hipSuccess) {
        rc = XCG_EHIP;
        break;
      }
    }
    if (rc == XCG_OK && hipStreamSynchronize(st) != hipSuccess) rc = XCG_EHIP;
    int32_t status = 0;
    if (rc == XCG_OK && hipMemcpy(&status, c->d_status, 4, hipMemcpyDeviceToHost) != hipSuccess) rc = XCG_EHIP;
    if (rc == XCG_OK && status) rc = XCG_EOVERFLOW;
  } while (0);
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  (void)hipFree(d_off);
  (void)hipFree(d_oo);
  (void)hipFree(d_ol);
  (void)hipFree(d_len);
  (void)hipStreamDestroy(st);
  return rc;
}

int xcg_window_hashes(xcg_ctx* c, const uint8_t* d_x, uint64_t len, uint64_t* d_hash, void* stream) {
  if (!c || (len && (!d_x || !d_hash))) return XCG_EINVAL;
  DeviceGuard g(c->device);
  return xcg_launch_window_hashes(d_x, len, d_hash, (hipStream_t)stream) == 0 ? XCG_OK : XCG_EHIP;
}

int xcg_segment_hashes(xcg_ctx* c, const uint8_t* d_x, uint64_t len, uint64_t* d_hash_be, void* stream) {
  if (!c || (len && (!d_x || !d_hash_be))) return XCG_EINVAL;
  DeviceGuard g(c->device);
  return xcg_launch_segment_hashes(d_x, len, d_hash_be, (hipStream_t)stream) == 0 ? XCG_OK : XCG_EHIP;
}

}  // extern "C"
