// GPU-resident XCodec segment cache (XCodecMemoryCache, xcodec/xcodec_cache.h:
// 245-365, unbounded variant) and the per-batch declaration table used by the
// stream-semantics encoder.  Device views are plain structs of pointers.
//
// Layout in HBM (see DESIGN.md "Data layout"):
//   keys[cap]  u64   XCodecHash of the segment; EMPTY = all ones (a real hash
//                    always has bits 32..35 clear: mix() shifts bits_hash by 36)
//   vals[cap]  u64   G: segment index into pool;  B: (chunk << 32) | position
//   pool[nseg_cap * 2048]  segment bytes (G only)
//   ftab[fbuckets * 4] u32  lane-probe fingerprint buckets of 16 B: seven 16-bit
//                    fingerprints of K + an overflow flag, one 16-byte load per
//                    probe; ~2 keys per bucket at capacity, so the table (2 MiB
//                    per 2^18 segments) stays in an XCD's L2
//   filt[FILT_BITS / 32] u32  the bitmap a workgroup loads into LDS (bit K mod 2^19)
#pragma once
#include "xcg_device.h"

namespace xcg {

constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr int FILT_LOG2 = 19;                       // 2^19 bits = 64 KiB of LDS
constexpr uint32_t FILT_WORDS = (1u << FILT_LOG2) / 32;
// A round's LDS lane filter comes in PREFIX_FILTERS slices: slice j holds the
// cache and the batch declarations of chunks < (j + 1) * pfdiv, so a workgroup
// whose chunks all lie below that copies slice j -- on average half the
// batch's keys, and far fewer for the first chunks (xcg_encode.hip
// filt_prefix_kernel).
constexpr uint32_t PREFIX_FILTERS = 16;
constexpr uint32_t FOVF16 = 2u;                     // bucket-overflow flag in slot 7 (even: never a fingerprint)

// Bounded (LRU) cache: kinds of the cache references a stream chunk records
// (bits 30..31 of an event's .w; the low 30 bits are the declaration index of
// an ENTER or the pool slot of a GHIT / GMISS).
//   ENTER  encode_declaration's enter() (xcodec_encoder.cc:284-286)
//   HIT    a lookup that found a declaration of this batch
//   GHIT   a lookup that found a persistent entry (lookup() refreshes it)
//   GMISS  a lookup of a persistent entry the LRU had evicted by then
constexpr uint32_t EV_ENTER = 0, EV_HIT = 1, EV_GHIT = 2, EV_GMISS = 3;
constexpr uint32_t EV_REF_MASK = (1u << 30) - 1u;

struct HashTab {      // exact open-addressed map u64 -> u64
  uint64_t* keys;
  uint64_t* vals;
  uint32_t mask;      // cap - 1
};

struct LaneFilter {   // what a lane probes: LDS bitmap (copied from filt) or the global
                      // filter gfilt, then the fingerprint buckets
  const uint32_t* filt;
  const u32x4* ftab;
  uint32_t fmask;     // fbuckets - 1
  const uint32_t* gfilt;
  uint32_t gmask;     // gfilt words - 1
  uint32_t pfdiv = 0; // filt is PREFIX_FILTERS slices of pfdiv chunks each (0: one filter)
};

// Every filter kept over a set of hashes (the persistent cache's, or a round's
// copy extended by the batch declarations).
struct FiltSet {
  uint32_t* filt;     // FILT_WORDS: the 64 KiB LDS lane filter
  uint32_t* ftab;     // (fmask + 1) * 4: fingerprint buckets
  uint32_t fmask;
  uint32_t* gfilt;    // (gmask + 1): the global lane filter (large caches)
  uint32_t gmask;
};

__device__ __forceinline__ uint32_t mix32(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}

// Exact-table slot of a hash (lo = bytes_hash word, hi = bits_hash << 4).
__device__ __forceinline__ uint32_t tab_slot(uint32_t lo, uint32_t hi, uint32_t mask) {
  return mix32(lo, hi) & mask;
}

// Lane-probe key of a hash: K = -lo (mod 2^32).  The encoder's rolling loop
// keeps negated sums (NX1 = -X1, NX2 = -(X2 + CLO)), so K = (NX1 << 20) + NX2
// costs one instruction per position, and every table the lanes probe (the
// per-wave declaration table, the LDS filter, the fingerprint buckets) is
// keyed by K.  The F (bits_hash) half of the hash is only needed after a K
// match, by the exact re-check.
__device__ __forceinline__ uint32_t probe_key(uint32_t lo) { return 0u - lo; }
// Lane filter = blocked Bloom filter, two bits per key in one 32-bit word
// (FP rate ~5 % at 65 k keys instead of ~12 % for one bit): word = bits 2..15
// of K (so the LDS byte offset is K & 0xFFFC), bits = K bits 16..20 and
// 24..28 (v_lshrrev takes the shift amount mod 32).
__device__ __forceinline__ uint32_t filt_word_ofs(uint32_t k) { return k & ((FILT_WORDS - 1u) << 2); }
__device__ __forceinline__ uint32_t filt_mask(uint32_t k) {
  return (1u << ((k >> 16) & 31u)) | (1u << ((k >> 24) & 31u));
}
__device__ __forceinline__ uint32_t filt_test(uint32_t w, uint32_t k) {
  return (w >> ((k >> 16) & 31u)) & (w >> ((k >> 24) & 31u)) & 1u;
}
// Global lane filter (caches too large for 64 KiB: >~100 k keys, where the
// LDS filter saturates): the same two-bits-per-word blocked Bloom filter,
// ~1 key per word (2 MiB at 2^19 keys, so it stays in an XCD's 4 MiB L2 --
// random loads run at ~270 G/s from L2-resident tables vs ~60 G/s beyond).
// word = K bits 10.., bits = K bits 0..4 and 5..9.
__device__ __forceinline__ uint32_t gfilt_word(uint32_t k, uint32_t gmask) { return (k >> 10) & gmask; }
__device__ __forceinline__ uint32_t gfilt_mask(uint32_t k) { return (1u << (k & 31u)) | (1u << ((k >> 5) & 31u)); }
__device__ __forceinline__ uint32_t gfilt_test(uint32_t w, uint32_t k) {
  return (w >> (k & 31u)) & (w >> ((k >> 5) & 31u)) & 1u;
}
// Fingerprint bucket = K bits 13.. (K is a sum-based hash; its high bits are
// well spread), fingerprint = top 16 bits of K * golden ratio: two keys of
// one bucket differ in bits 0..12, and their products' top halves then agree
// with probability ~2^-16.  (Two cheap ops each instead of a full mix.)
__device__ __forceinline__ uint32_t fbucket(uint32_t k, uint32_t fmask) { return (k >> 13) & fmask; }

// Wave-uniform 64-bit value (readfirstlane per 32-bit half; no sign extension).
__device__ __forceinline__ uint64_t readfirst64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Uniform (wave-level) exact lookup: value or ~0 when absent.
__device__ __forceinline__ uint64_t tab_lookup(const HashTab& t, uint32_t lo, uint32_t hi) {
  const uint64_t key = ((uint64_t)hi << 32) | lo;
  uint32_t i = tab_slot(lo, hi, t.mask);
  for (uint32_t n = 0; n <= t.mask; ++n) {
    const uint64_t k = readfirst64(t.keys[i]);
    if (k == key) return readfirst64(t.vals[i]);
    if (k == EMPTY_KEY) break;
    i = (i + 1) & t.mask;
  }
  return ~0ull;
}

// Uniform lookup of one key in two tables at once: the first probe slot of
// each (key and value words) is loaded together, so the common case (found
// there, or an empty slot) costs one memory round trip instead of four.
__device__ __forceinline__ uint64_t tab_probe_rest(const HashTab& t, uint64_t key, uint32_t i) {
  for (uint32_t n = 1; n <= t.mask; ++n) {
    i = (i + 1) & t.mask;
    const uint64_t k = readfirst64(t.keys[i]);
    if (k == key) return readfirst64(t.vals[i]);
    if (k == EMPTY_KEY) break;
  }
  return ~0ull;
}
__device__ __forceinline__ void tab_lookup2(const HashTab& a, const HashTab& b, uint32_t lo, uint32_t hi,
                                            uint64_t& va, uint64_t& vb) {
  const uint64_t key = ((uint64_t)hi << 32) | lo;
  const uint32_t ia = tab_slot(lo, hi, a.mask), ib = tab_slot(lo, hi, b.mask);
  const uint64_t ka = a.keys[ia], xa = a.vals[ia], kb = b.keys[ib], xb = b.vals[ib];
  const uint64_t ua = readfirst64(ka), ub = readfirst64(kb);
  va = ua == key ? readfirst64(xa) : (ua == EMPTY_KEY ? ~0ull : tab_probe_rest(a, key, ia));
  vb = ub == key ? readfirst64(xb) : (ub == EMPTY_KEY ? ~0ull : tab_probe_rest(b, key, ib));
}

// Per-thread probe on from slot i (whose key was neither `key` nor empty).
__device__ __forceinline__ uint64_t tab_probe_rest_t(const HashTab& t, uint64_t key, uint32_t i) {
  for (uint32_t n = 1; n <= t.mask; ++n) {
    i = (i + 1) & t.mask;
    const uint64_t k = t.keys[i];
    if (k == key) return t.vals[i];
    if (k == EMPTY_KEY) break;
  }
  return ~0ull;
}

// Per-thread exact lookup (each lane its own key): value or ~0 when absent.
__device__ __forceinline__ uint64_t tab_lookup_t(const HashTab& t, uint32_t lo, uint32_t hi) {
  const uint64_t key = ((uint64_t)hi << 32) | lo;
  uint32_t i = tab_slot(lo, hi, t.mask);
  for (uint32_t n = 0; n <= t.mask; ++n) {
    const uint64_t k = t.keys[i];
    if (k == key) return t.vals[i];
    if (k == EMPTY_KEY) break;
    i = (i + 1) & t.mask;
  }
  return ~0ull;
}

// Segment numbers for a block's new entries without a per-entry global
// atomic (65 k lane-0 atomicAdds on one counter serialise at ~11 ns each):
// a block-wide count, one atomicAdd per block.  Returns this thread's
// segment (valid where `need`), uniform within the block.
__device__ __forceinline__ uint32_t block_alloc_segs(bool need, uint32_t* nseg, uint32_t* s_cnt, uint32_t* s_base) {
  if (threadIdx.x == 0) *s_cnt = 0;
  __syncthreads();
  uint32_t mine = 0;
  // wave-aggregated: one LDS atomic per wave
  const uint64_t m = __ballot(need);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  uint32_t wbase = 0;
  if (__lane_id() == 0 && m) wbase = atomicAdd(s_cnt, (uint32_t)__builtin_popcountll(m));
  wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)wbase);
  mine = wbase + below;
  __syncthreads();
  if (threadIdx.x == 0) *s_base = *s_cnt ? atomicAdd(nseg, *s_cnt) : 0u;
  __syncthreads();
  return *s_base + mine;
}

// Per-thread insert (keys unique per call site).  For B, `val` is combined with
// atomicMin so the earliest (chunk, position) declaring a hash wins.
__device__ __forceinline__ bool tab_insert_min(HashTab t, uint32_t lo, uint32_t hi, uint64_t val) {
  const uint64_t key = ((uint64_t)hi << 32) | lo;
  uint32_t i = tab_slot(lo, hi, t.mask);
  for (uint32_t n = 0; n <= t.mask; ++n) {
    const uint64_t prev = atomicCAS((unsigned long long*)&t.keys[i], (unsigned long long)EMPTY_KEY,
                                    (unsigned long long)key);
    if (prev == EMPTY_KEY || prev == key) {
      atomicMin((unsigned long long*)&t.vals[i], (unsigned long long)val);
      return true;
    }
    i = (i + 1) & t.mask;
  }
  return false;
}

// 16-bit fingerprint of a probe key (odd, so never 0 = empty or FOVF16).
__device__ __forceinline__ uint32_t fp16_of(uint32_t k) { return ((k * 0x9E3779B1u) >> 16) | 1u; }

// Fingerprint bucket insert: first free of the 7 slots, else set the bucket's
// overflow flag (a probe of that bucket then reports an event and the
// resolver decides exactly).
__device__ __forceinline__ void ftab_insert(uint32_t* ftab, uint32_t fmask, uint32_t lo, uint32_t hi) {
  (void)hi;
  const uint32_t k = probe_key(lo), fp = fp16_of(k);
  uint32_t* s = ftab + 4 * fbucket(k, fmask);
  for (int w = 0; w < 4; ++w) {
    uint32_t old = s[w];
    for (;;) {
      const uint32_t a = old & 0xFFFFu, b = old >> 16;
      if (a == fp || (w < 3 && b == fp)) return;      // already there
      uint32_t nw;
      if (a == 0u) nw = old | fp;
      else if (w < 3 && b == 0u) nw = old | (fp << 16);
      else break;                                      // word full (slot 7 is the flag)
      const uint32_t got = atomicCAS(s + w, old, nw);
      if (got == old) return;
      old = got;
    }
  }
  atomicOr(s + 3, FOVF16 << 16);
}

// Does the bucket q hold key k (or overflow)?
__device__ __forceinline__ bool ftab_match(const u32x4 q, uint32_t k) {
  const uint32_t t = fp16_of(k) * 0x10001u;
  bool m = (q[3] >> 16) == FOVF16;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t d = q[w] ^ t;
    m = m || (d & 0xFFFFu) == 0u || (d >> 16) == 0u;
  }
  return m;
}

__device__ __forceinline__ void filt_insert(const FiltSet& f, uint32_t lo, uint32_t hi) {
  const uint32_t k = probe_key(lo);
  atomicOr(f.filt + (filt_word_ofs(k) >> 2), filt_mask(k));
  atomicOr(f.gfilt + gfilt_word(k, f.gmask), gfilt_mask(k));
  ftab_insert(f.ftab, f.fmask, lo, hi);
}

// tab_insert_min + filt_insert with a shorter chain of memory round trips (a
// thread per key, e.g. a batch table build or a commit): the fingerprint
// bucket is loaded together with the table's first CAS, the value's atomicMin
// and the filter ORs return nothing, and the bucket is updated from the loaded
// copy -- on gfx9 each returning atomic waits for every older memory operation
// of the wave, so the plain sequence cost about four round trips, this two.
__device__ __forceinline__ bool tab_insert_min_filt(HashTab t, const FiltSet& f, uint32_t lo, uint32_t hi,
                                                    uint64_t val) {
  const uint32_t k = probe_key(lo), fp = fp16_of(k);
  uint32_t* s = f.ftab + 4 * fbucket(k, f.fmask);
  const u32x4 q = *(const u32x4*)s;
  const uint64_t key = ((uint64_t)hi << 32) | lo;
  uint32_t i = tab_slot(lo, hi, t.mask);
  bool ok = false;
  for (uint32_t n = 0; n <= t.mask; ++n) {
    const uint64_t prev = atomicCAS((unsigned long long*)&t.keys[i], (unsigned long long)EMPTY_KEY,
                                    (unsigned long long)key);
    if (prev == EMPTY_KEY || prev == key) {
      (void)atomicMin((unsigned long long*)&t.vals[i], (unsigned long long)val);
      ok = true;
      break;
    }
    i = (i + 1) & t.mask;
  }
  atomicOr(f.filt + (filt_word_ofs(k) >> 2), filt_mask(k));
  atomicOr(f.gfilt + gfilt_word(k, f.gmask), gfilt_mask(k));
  // the bucket, as ftab_insert, starting from the loaded copy
  for (int w = 0; w < 4; ++w) {
    uint32_t old = q[w];
    for (;;) {
      const uint32_t a = old & 0xFFFFu, b = old >> 16;
      if (a == fp || (w < 3 && b == fp)) return ok;
      uint32_t nw;
      if (a == 0u) nw = old | fp;
      else if (w < 3 && b == 0u) nw = old | (fp << 16);
      else break;
      const uint32_t got = atomicCAS(s + w, old, nw);
      if (got == old) return ok;
      old = got;
    }
  }
  atomicOr(s + 3, FOVF16 << 16);
  return ok;
}

}  // namespace xcg
