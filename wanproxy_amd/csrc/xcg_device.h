// Device-side building blocks shared by the XCodec encode/decode kernels.
// gfx950 (CDNA4), wave64.  No host code here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xcg {

constexpr int SEG = 2048;                // XCODEC_SEGMENT_LENGTH, xcodec/xcodec.h:87
constexpr uint32_t MAGIC = 0xF1u;        // XCODEC_MAGIC, xcodec/xcodec.h:30
constexpr uint32_t OP_ESCAPE = 0x00u;    // xcodec/xcodec.h:42
constexpr uint32_t OP_EXTRACT = 0x01u;   // xcodec/xcodec.h:60
constexpr uint32_t OP_REF = 0x02u;       // xcodec/xcodec.h:75
constexpr uint32_t OP_BACKREF = 0x03u;   // xcodec/xcodec.h:85

// Low word of XCodecHash::mix (xcodec/xcodec_hash.h:155-164) in terms of the
// raw-byte window sums X1 = sum(x), X2 = sum((2048-k) x):
//   bytes_hash = (s1 << 20) + s2, s1 = X1 + 2048, s2 = X2 + 2048*2049/2
//             = (X1 << 20) + X2 + CLO   (mod 2^32)
// The high word is (bits_hash << 4) with bits_hash = (F1 << 16) + F2 over
// f = ffs(byte); mix()'s `<< 36` keeps bits_hash bits 0..27 only.
constexpr uint32_t CLO = 0x80200400u;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;   // unaligned 16-B global access
typedef uint32_t __attribute__((aligned(1))) u32_u;
typedef uint16_t __attribute__((aligned(1))) u16_u;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// A copy of v the optimiser cannot see through: values derived from it are
// recomputed where used instead of being hoisted and held live across a big
// loop (register pressure control).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint32_t readfirst(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)readlane((uint32_t)(v >> 32), l) << 32) | readlane((uint32_t)v, l);
}

// v_ffbl_b32: index of the lowest set bit, 0xFFFFFFFF for 0.  So
// ffbl(x) + 1 == POSIX ffs(x) for every x, which is what XCodecHash::add /
// roll feed the bits_ RollingHash (xcodec_hash.h:95,124).
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// Inclusive wave64 prefix sum (u32, wrapping).  Rows of 16 by DPP row_shr,
// then the row carries by DPP row_bcast:15 (rows 1, 3 += lane 15 of the row
// before) and row_bcast:31 (rows 2, 3 += lane 31); disabled rows add 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return readlane(wave_incl_scan(v), 63); }

// Number of bytes equal to 0xF1 in a dword (exact zero-byte count of d^F1F1F1F1).
__device__ __forceinline__ uint32_t count_magic(uint32_t d) {
  uint32_t v = d ^ 0xF1F1F1F1u;
  uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  t = ~(t | v | 0x7F7F7F7Fu);
  return __builtin_popcount(t);
}

__device__ __forceinline__ uint32_t byte_of(uint32_t d, int k) { return (d >> (8 * k)) & 0xFFu; }

// Load 16 bytes of chunk position q (relative to x, may be outside [0, len)):
// bytes outside the chunk read as 0.  Fast path is one (possibly unaligned)
// dwordx4 load.
__device__ __forceinline__ u32x4 load16_guarded(const uint8_t* x, int64_t q, int64_t len) {
  if (q >= 0 && q + 16 <= len) return *(const u32x4_u*)(x + q);
  u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int64_t i = q + k;
    uint32_t b = (i >= 0 && i < len) ? (uint32_t)x[i] : 0u;
    r[k >> 2] |= b << (8 * (k & 3));
  }
  return r;
}

// 16 bytes at chunk position q where x + q is 16-byte aligned.  A 16-byte
// aligned block that overlaps [0, len) lies inside one page of the caller's
// buffer, so it is loaded whole; blocks wholly outside read as 0.  Bytes
// outside the chunk only ever enter windows of non-positions (s > len-2048 or
// s < 0), and a rolling sum removes exactly what it added, so their values
// never reach a valid window hash.
__device__ __forceinline__ u32x4 load16_aligned_safe(const uint8_t* x, int q, int len) {
  u32x4 r = {0u, 0u, 0u, 0u};
  if (q > -16 && q < len) r = *(const u32x4*)(x + q);
  return r;
}
// The same as a streaming (non-temporal) load: a chunk's bytes are read once,
// and marking them so keeps them from evicting the L2-resident probe tables
// (lane filter, fingerprint buckets, hash tables) that every position reads.
__device__ __forceinline__ u32x4 load16_stream(const uint8_t* p) {
  return __builtin_nontemporal_load((const u32x4*)p);
}
__device__ __forceinline__ u32x4 load16_aligned_safe_stream(const uint8_t* x, int q, int len) {
  u32x4 r = {0u, 0u, 0u, 0u};
  if (q > -16 && q < len) r = load16_stream(x + q);
  return r;
}

}  // namespace xcg
