// XCodec encoder, MI355X (gfx950) HIP kernels.
//
// Restates XCodecEncoder::encode (xcodec/xcodec_encoder.cc:74-274) for a batch
// of independent encode() calls: one wave64 per chunk, so a 64 KiB chunk (the
// unit tack and wanproxy hand to encode(), programs/tack/tack.cc:308-321,
// io/io_system_handle.cc:39) is parsed by 64 lanes with no inter-wave sync.
//
// The reference walks every byte offset sequentially: roll the 2048-byte
// XCodecHash (xcodec_hash.h:93-163), probe the cache (find_reference,
// xcodec_encoder.cc:374-416), and run a greedy candidate / declare / reference
// state machine (:183-248).  Here a chunk is parsed in PIECES of 2048 window
// positions:
//
//   1. vector phase: lane i rolls the hash over the 32 positions
//      [p + 32 i, p + 32 i + 32) -- its start sums come from wave prefix scans
//      over 32-byte segment sums -- and probes a per-wave LDS fingerprint table
//      of the declarations made so far, producing a 32-bit event mask;
//   2. resolve phase (wave-uniform): the state machine jumps from event to
//      event through those masks.  Within 2048 positions of the parse point at
//      most ONE declaration can become visible (the candidate pending at piece
//      start, visible from cand + 2048), which the vector phase covers with a
//      gated compare, so every event the masks miss is a true miss.
//
// Events are re-checked exactly (full 64-bit hash, then byte compare against
// the declared segment) before a REF or a collision skip is emitted, so the
// fingerprint table can be approximate without affecting output.  Output ops
// (ESCAPE / EXTRACT / REF, xcodec_encoder.cc:276-372) are written by the whole
// wave as they are resolved, into the chunk's output slot.
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "xcg_cache.h"
#include "xcg_args.h"
#include "../../include/xcgpu.h"

namespace xcg {

// A chunk's piece loads.  Independent chunks read theirs as streaming
// (non-temporal) loads: each byte is read once, and the headline launch runs
// ~5 % faster so (the stream kernel, whose probes read L2-resident tables,
// measured no gain: C4 654 vs 636 us, C2-S2 294 vs 297).
#ifndef XCG_STREAM_NT
#define XCG_STREAM_NT 0
#endif
template <bool STREAM>
__device__ __forceinline__ u32x4 piece_ld_safe(const uint8_t* x, int q, int len) {
  if constexpr (STREAM && !XCG_STREAM_NT) return load16_aligned_safe(x, q, len);
  else return load16_aligned_safe_stream(x, q, len);
}
template <bool STREAM>
__device__ __forceinline__ u32x4 piece_ld(const uint8_t* p) {
  if constexpr (STREAM && !XCG_STREAM_NT) return *(const u32x4*)p;
  else return load16_stream(p);
}

// Per-wave LDS state of one encode() call's XCodecMemoryCache
// (xcodec_cache.h:245-365): a 2-slot-bucket table of probe keys K = -lo over
// the chunk's declarations -- bucket = bits 3.. of K; an empty slot of bucket b
// holds kempty(b), whose bucket bits are ~b, so it never equals a K probed
// there -- plus the exact records the slots point to.  The key tables of a
// block's waves sit first in LDS, 8 << LOGNB bytes each, so a lane's probe
// address is a single and-or of K.
// Overflow keys a chunk's table holds: 8, or 32 for frames of up to 512 KiB
// (~256 declarations in 1024 buckets: a tail of 9+ three-key buckets happens).
// Independent chunks' direct-mapped tables (DMV, roll_probe_dm): 32, a key
// overflowing as soon as its slot is taken.
template <int MAXD, bool DMV = false>
constexpr int ovf_cap() { return MAXD > 72 || DMV ? 32 : 8; }

template <int LOGNB, int MAXD, bool DMV = false>
struct WaveRecs {
  static constexpr int NB = 1 << LOGNB;
  uint32_t rlo[MAXD], rhi[MAXD], rc[MAXD];  // exact hash + chunk position
  uint32_t ovf_k[ovf_cap<MAXD, DMV>()];     // keys whose bucket was full
};

template <int LOGNB>
__device__ __forceinline__ uint32_t kbucket(uint32_t k) { return (k >> 3) & ((1u << LOGNB) - 1u); }
template <int LOGNB>
__device__ __forceinline__ uint32_t kempty(uint32_t b) { return (~b & ((1u << LOGNB) - 1u)) << 3; }

template <int LOGNB, int MAXD, int W>
struct IndepLDS {
  uint32_t key[W][2 << LOGNB];
  WaveRecs<LOGNB, MAXD, (MAXD <= 72)> rec[W];
};
constexpr int GSLOTS_DECL = 8;   // = GSLOTS (pass-1 queue depth per lane)
template <int LOGNB, int MAXD, int W>
struct StreamLDS {
  uint32_t key[W][2 << LOGNB];               // offset 0, as in IndepLDS
  uint32_t lfilt[FILT_WORDS];                // the lane filter (64 KiB)
  uint32_t scr[W][GSLOTS_DECL + 1][64];      // pass-1 queues (+ a garbage slot)
  WaveRecs<LOGNB, MAXD> rec[W];
  uint32_t ro[W][MAXD];                      // output length after each declaration's op (restart points)
  uint32_t rsv[W][8];                        // restart state (kept out of registers)
  uint32_t cmax;                             // the workgroup's highest chunk (prefix filter slice)
};

// Re-parse restart (bounded / pair passes after the first; the driver backs up
// the previous pass's rows of each flagged chunk, xcg_restart_backup_kernel).
struct RestartArgs {
  const uint32_t* bad_t;   // [n] in-chunk time of the chunk's earliest contradicted lookup (~0: none)
  const uint32_t* bad_hi;  // [n] ... and of its latest
  const uint32_t* bslot;   // [n] backup slot of the chunk's previous pass (~0: none)
  const uint4* b_ev;       // [slots * maxe] its reference rows
  const uint32_t* b_eo;    // [slots * maxe] their REF output lengths
  const uint64_t* b_hits;  // [slots * maxh] its batch hits
  const uint32_t* b_cnt;   // [slots * 4] its nev, nhits, output length, ndecl
  uint4* splice;           // [n] {new offset, old offset, old end, 1}: the old tail to append
};

struct EncParams {
  const uint8_t* in;
  const uint64_t* chunk_off;
  const uint32_t* chunk_len;
  uint32_t n;
  uint32_t flags;
  uint8_t* out;
  const uint64_t* out_off;
  uint64_t* out_len;
  uint32_t* stats;     // optional: per chunk {n_extract, n_ref, n_collision, n_pieces}
  int32_t* status;     // optional: nonzero on internal overflow
  // ---- stream semantics (XCG_SEM_STREAM) only
  HashTab g;           // the persistent cache: hash -> segment index
  const uint8_t* pool; // its segment bytes
  HashTab b;           // this batch's declarations (earlier rounds): hash -> (chunk << 32 | pos)
  bool use_b;
  LaneFilter lf;       // lane probe filter over g + b
  uint4* decl;         // [n * maxd] (lo, hi, pos, 0) declarations of the chunk, this round
  uint32_t* ndecl;     // [n]
  uint32_t maxd;
  uint32_t* changed;   // lowest chunk whose declaration list differs from the last round (~0: none)
  uint32_t lds_filter_keys;  // LDS lane filter up to this many keys, else the global one
  uint32_t lds_prefilter_keys;  // up to this many: the LDS filter in front of the global one (fmode 3)
  const uint32_t* nseg;    // segments in the persistent cache
  const uint32_t* bcount;  // [64] partial counts of the batch table's declarations (use_b)
  uint32_t skip_below; // chunks below this keep their last parse (their batch input is unchanged)
  const uint32_t* need;  // (verification rounds) parse only chunks with need[c] != 0
  uint64_t* hits;      // [n * maxh] hashes the chunk found among the batch declarations (REF or collision)
  uint32_t* nhits;     // [n] (> maxh: overflowed, always re-parsed)
  uint32_t maxh;
  uint32_t max_len;    // the caller's bound on every chunk length (sizes LDS records and declaration rows)
  // ---- bounded (LRU) cache only (xcg_lru.hip); null otherwise
  const uint64_t* ptime;  // [pool slot] batch time from which the entry is evicted (~0: never)
  uint4* ev;           // [n * maxe] the chunk's cache references in order (lo, hi, time, kind << 30 | ref)
  uint32_t* nev;       // [n] (> maxe: overflowed)
  uint32_t maxe;
  uint32_t* eo;        // [n * maxe] output length after the REF a lookup made (~0: it made none)
  RestartArgs rs;      // re-parse from the previous pass's rows (bslot null: off)
  // ---- (stream) parse only the chunks of a work list: work[0] = count, work[1..] chunks (null: all)
  const uint32_t* work;
};

// ------------------------------------------------------------------ emission

// Copy n bytes src -> dst (any alignment), whole wave.
__device__ __noinline__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n) {
  const int l = lane_id();
  for (uint32_t base = 0; base < n; base += 1024) {
    uint32_t off = base + 16u * l;
    if (off + 16 <= n) {
      *(u32x4_u*)(dst + off) = *(const u32x4_u*)(src + off);
    } else if (off < n) {
      for (uint32_t k = off; k < n; ++k) dst[k] = src[k];
    }
  }
}

// encode_escape (xcodec_encoder.cc:315-340): x[a..b) with F1 -> F1 00.
// Returns bytes written (uniform).
__device__ __noinline__ uint32_t wave_escape(uint8_t* dst, const uint8_t* x, uint32_t a, uint32_t b) {
  const int l = lane_id();
  const uint32_t n = b - a;
  uint32_t written = 0;
  for (uint32_t base = 0; base < n; base += 1024) {
    uint32_t off = base + 16u * l;
    uint32_t cnt = off < n ? min(16u, n - off) : 0u;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (cnt == 16) {
      v = *(const u32x4_u*)(x + a + off);
    } else {
      for (uint32_t k = 0; k < cnt; ++k) v[k >> 2] |= (uint32_t)x[a + off + k] << (8 * (k & 3));
    }
    uint32_t nm = count_magic(v[0]) + count_magic(v[1]) + count_magic(v[2]) + count_magic(v[3]);
    if (cnt < 16) {
      // padding bytes are 0 (never magic) unless the chunk byte was; recount exactly
      nm = 0;
      for (uint32_t k = 0; k < cnt; ++k) nm += byte_of(v[k >> 2], k & 3) == MAGIC;
    }
    uint32_t olen = cnt + nm;
    uint32_t incl = wave_incl_scan(olen);
    uint32_t pos = written + incl - olen;
    if (nm == 0) {
      if (cnt == 16) {
        *(u32x4_u*)(dst + pos) = v;
      } else {
        for (uint32_t k = 0; k < cnt; ++k) dst[pos + k] = (uint8_t)byte_of(v[k >> 2], k & 3);
      }
    } else {
      uint32_t o = pos;
      for (uint32_t k = 0; k < cnt; ++k) {
        uint32_t c = byte_of(v[k >> 2], k & 3);
        dst[o++] = (uint8_t)c;
        if (c == MAGIC) dst[o++] = (uint8_t)OP_ESCAPE;
      }
    }
    written += readlane(incl, 63);
  }
  return written;
}

// F1 02 BE64(hash): encode_reference, xcodec_encoder.cc:357-360.
__device__ __forceinline__ void wave_put_ref(uint8_t* dst, uint32_t lo, uint32_t hi) {
  const int l = lane_id();
  if (l < 10) {
    uint32_t v;
    if (l == 0) v = MAGIC;
    else if (l == 1) v = OP_REF;
    else if (l < 6) v = hi >> (8 * (5 - l));
    else v = lo >> (8 * (9 - l));
    dst[l] = (uint8_t)v;
  }
}

// ------------------------------------------------------------ exact checks

// XCodecHash::hash of the 2048-byte window at w (xcodec_hash.h:166-174),
// whole wave: lane l sums bytes [16l, 16l+16) and [1024+16l, +16).  z = the
// window's direct-mapped probe key -(X2 + CLO) (independent chunks, see
// roll_probe_dm).
__device__ __noinline__ uint3 wave_window_hash(const uint8_t* w) {
  const int l = lane_id();
  uint32_t X1 = 0, X2 = 0, F1 = 0, F2 = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t k0 = 1024u * h + 16u * l;
    u32x4 v = *(const u32x4_u*)(w + k0);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      uint32_t x = byte_of(v[k >> 2], k & 3);
      uint32_t f = ffbl(x) + 1u;
      uint32_t wt = 2048u - (k0 + k);
      X1 += x; X2 += wt * x; F1 += f; F2 += wt * f;
    }
  }
  X1 = wave_sum(X1); X2 = wave_sum(X2); F1 = wave_sum(F1); F2 = wave_sum(F2);
  return make_uint3((X1 << 20) + X2 + CLO, ((F1 << 16) + F2) << 4, 0u - (X2 + CLO));
}

// Byte-equality of two 2048-byte segments (BufferSegment::equal in
// find_reference, xcodec_encoder.cc:383-390), whole wave.
__device__ __noinline__ bool wave_equal2048(const uint8_t* a, const uint8_t* b) {
  const int l = lane_id();
  bool ok = true;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t k0 = 1024u * h + 16u * l;
    u32x4 va = *(const u32x4_u*)(a + k0);
    u32x4 vb = *(const u32x4_u*)(b + k0);
    ok = ok && va[0] == vb[0] && va[1] == vb[1] && va[2] == vb[2] && va[3] == vb[3];
  }
  return ballot(!ok) == 0;
}

// Call-site wrappers: a non-inlined call returns in VGPRs, which hipcc must
// treat as divergent; these values are wave-uniform, and saying so keeps the
// whole parse state machine in SGPRs / scalar branches.
__device__ __forceinline__ uint32_t escape_u(uint8_t* dst, const uint8_t* x, uint32_t a, uint32_t b) {
  return readfirst(wave_escape(dst, x, a, b));
}
__device__ __forceinline__ uint3 window_hash_u(const uint8_t* w) {
  const uint3 h = wave_window_hash(w);
  return make_uint3(readfirst(h.x), readfirst(h.y), readfirst(h.z));
}
__device__ __forceinline__ bool equal2048_u(const uint8_t* a, const uint8_t* b) {
  return readfirst((uint32_t)wave_equal2048(a, b)) != 0u;
}
// The same compare when the window is a piece start: its bytes are the A
// registers (lane l holds [32 l, 32 l + 32)), so only the other side is read.
__device__ __forceinline__ bool equal2048_regs(const uint8_t* a, const u32x4& w0, const u32x4& w1) {
  const uint32_t o = 32u * (uint32_t)lane_id();
  const u32x4 v0 = *(const u32x4_u*)(a + o), v1 = *(const u32x4_u*)(a + o + 16);
  const bool ok = v0[0] == w0[0] && v0[1] == w0[1] && v0[2] == w0[2] && v0[3] == w0[3] && v1[0] == w1[0] &&
                  v1[1] == w1[1] && v1[2] == w1[2] && v1[3] == w1[3];
  return ballot(!ok) == 0;
}

// ------------------------------------------------------------ vector phase

// Make the registers of v live here (the compiler waits for their load first).
__device__ __forceinline__ void vuse(const u32x4& v) {
  asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
}

struct Piece {
  u32x4 a0, a1;   // bytes [q0, q0+32): the windows' leaving bytes
  u32x4 b0, b1;   // bytes [q0+2048, q0+2080): the entering bytes
  // byte sums of the A and B segments: plain and weighted by j (offset in it)
  uint32_t sxa, sqxa;
  uint32_t sxb, sqxb;
};

__device__ __forceinline__ void seg_sums(const u32x4 d0, const u32x4 d1, uint32_t& sx, uint32_t& sqx) {
  const uint32_t d[8] = {d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
  sx = 0; sqx = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t wts = (4u * k) | ((4u * k + 1) << 8) | ((4u * k + 2) << 16) | ((4u * k + 3) << 24);
    sx = __builtin_amdgcn_udot4(d[k], 0x01010101u, sx, false);
    sqx = __builtin_amdgcn_udot4(d[k], wts, sqx, false);
  }
}

// bits_hash half of the hash of the window that starts at lane L's first
// position (bytes A of lanes >= L, then B of lanes < L), from the registers:
// hi = ((F1 << 16) + F2) << 4 with F1 = sum ffs(x), F2 = sum (2048 - k) ffs(x_k)
// (XCodecHash, xcodec_hash.h:93-174).  Only candidates need it.
__device__ __forceinline__ uint32_t lane_window_hi(const Piece& P, int L) {
  const int l = lane_id();
  const bool useA = l >= L;
  const uint32_t d[8] = {useA ? P.a0[0] : P.b0[0], useA ? P.a0[1] : P.b0[1], useA ? P.a0[2] : P.b0[2],
                         useA ? P.a0[3] : P.b0[3], useA ? P.a1[0] : P.b1[0], useA ? P.a1[1] : P.b1[1],
                         useA ? P.a1[2] : P.b1[2], useA ? P.a1[3] : P.b1[3]};
  uint32_t sf = 0, sqf = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t f = ffbl(byte_of(d[k], b)) + 1u;
      sf += f;
      sqf += (4u * k + b) * f;
    }
  }
  const uint32_t o = 32u * (uint32_t)((l - L) & 63);   // lane's offset in the window
  const uint32_t F1 = wave_sum(sf), F2 = wave_sum((2048u - o) * sf - sqf);
  return ((F1 << 16) + F2) << 4;
}

// Lane mask of a == b, straight from v_cmp (a bool would be materialised
// in a VGPR and compared again before any ballot).
__device__ __forceinline__ uint64_t lanes_eq(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 32); }

// ev = 2 ev + (this lane's bit of m) in one v_addc, m being the carry-in: no
// per-position bit constants, which VOP3 cannot encode as literals on gfx9.
__device__ __forceinline__ uint32_t shift_in(uint32_t ev, uint64_t m) {
  uint32_t r;
  uint64_t co;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(ev), "s"(readfirst64(m)));
  return r;
}

// Stream-semantics probe of the persistent cache + batch declarations.
// Pass 1 (inside the roll): the key's lane-filter word -- the blocked-Bloom
// LDS filter (xcg_cache.h filt_*) or, for large caches, the global one
// (gfilt_*); a passing key is queued in the wave's LDS scratch, slot
// min(passes, GSLOTS) of the lane (slot-major, so a wave's 64 stores are
// consecutive dwords), and its position bit set in pm.  Pass 2 (glb_flush,
// after each half of the lane's 32 positions) checks the queued keys against
// the 16-bit fingerprint buckets (an L2-resident table), all of a lane's
// loads in flight together instead of one round trip per group of positions.
// Passes beyond GSLOTS in one half are reported as events unchecked.
// FM 3 (caches past the LDS filter's ~220 k keys): the global filter mode is
// bound by L2 requests, one per window position (rocprofv3 TCC_READ ~430 M per
// 512 MiB C5 sub-batch at a 97 % L2 hit rate, profiles/r06_l2_*), so the
// saturated LDS filter (FP ~0.4 at 260 k keys, ~0.7 at 470 k) goes first and
// only the lanes it passes load their global word (exec-masked: the other
// lanes send no request).
constexpr int GSLOTS = 8;
// (with the prefix slices; measured on C2-S2 / C5, profiles/r06_filter_modes.txt:
// the two-level mode beats the LDS filter alone beyond ~150 k keys)
constexpr uint32_t LDS_FILTER_KEYS_DEFAULT = 150000;
constexpr uint32_t LDS_PREFILTER_KEYS_DEFAULT = 700000;
struct GlbQ {
  char* lds;        // LDS base of the workgroup's struct (offset 0)
  uint32_t lfo;     // byte offset of the lane filter (FM 1)
  const uint32_t* gf;   // global lane filter (FM 2)
  uint32_t gmask;
  const u32x4* ftab;    // fingerprint buckets
  uint32_t fmask;
  uint32_t sa0;     // this lane's scratch slot 0 (absolute LDS byte address)
  uint32_t sa;      // its next slot
  uint32_t salim;   // its garbage slot (slot GSLOTS)
  uint32_t pm;      // filter passes of the current half, bit j = position j
  uint32_t gev;     // verified cache / batch hits, bit j = position j
};

// Pass 2 over the queued keys of the current half; resets the queue.
__device__ __forceinline__ void glb_flush(GlbQ& gq) {
#ifdef XCG_EXP_NOPASS2   // (timing experiment only: output is wrong)
  gq.pm = 0;
  gq.sa = gq.sa0;
  return;
#endif
  const uint32_t cnt = (gq.sa - gq.sa0) >> 8;
  uint32_t rem = gq.pm;
#pragma unroll
  for (int i0 = 0; i0 < GSLOTS; i0 += 4) {
    if (ballot(cnt > (uint32_t)i0) == 0) break;
    uint32_t kk[4];
    u32x4 q[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) kk[t] = *(const uint32_t*)(gq.lds + gq.sa0 + 256u * (i0 + t));
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      q[t] = u32x4{0u, 0u, 0u, 0u};
      if ((uint32_t)(i0 + t) < cnt) q[t] = gq.ftab[fbucket(kk[t], gq.fmask)];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if ((uint32_t)(i0 + t) < cnt) {
        const uint32_t j = (uint32_t)__builtin_ctz(rem);
        rem &= rem - 1u;
        gq.gev |= (uint32_t)ftab_match(q[t], kk[t]) << j;
      }
    }
  }
  gq.gev |= rem;
  gq.pm = 0;
  gq.sa = gq.sa0;
}

// Roll the probe key over the lane's 32 positions; bit j of the result is set
// when position q0 + j is a possible cache hit.  NX1 = -X1, NX2 = -(X2 + CLO)
// at q0 (RollingHash::roll, xcodec_hash.h:57-70, negated), so K = -lo costs one
// instruction.  C0: the pending candidate (key c0k) is not in the table yet and
// becomes visible at piece offset rvis (position p + rvis).  OVF: also compare the (rare) overflow
// keys ovk[NOVF].  FM: also run pass 1 of the persistent cache / batch probe (gq)
// through the LDS lane filter (1) or the global one (2); 0: no such probe.
template <int LOGNB, bool C0, int NOVF, int FM>
__device__ __forceinline__ uint32_t roll_probe(const Piece& P, uint32_t NX1, uint32_t NX2, const char* kblk,
                                               uint32_t kofs, uint32_t c0k, int rvis, const uint32_t* ovk,
                                               GlbQ& gq) {
  constexpr bool GLB = FM != 0;
  // bucket mask in a VGPR so that (K & KM) | kofs is one v_and_or_b32 (VOP3
  // takes no literal and one SGPR on gfx9)
  const uint32_t KM = (uint32_t)opaque((int)(((1u << LOGNB) - 1u) << 3));
  const uint32_t xa[8] = {P.a0[0], P.a0[1], P.a0[2], P.a0[3], P.a1[0], P.a1[1], P.a1[2], P.a1[3]};
  const uint32_t xb[8] = {P.b0[0], P.b0[1], P.b0[2], P.b0[3], P.b1[0], P.b1[1], P.b1[2], P.b1[3]};
  uint32_t o[NOVF > 0 ? NOVF : 1];
#pragma unroll
  for (int k = 0; k < NOVF; ++k) o[k] = ovk[k];
  // C0 visibility: lanes l with 32 l + j >= rvis.  With rvis = 32 A + B that is
  // l >= A + 1 for j < B and l >= A for j >= B -- two masks per piece.
  uint64_t vis_hi = 0, vis_lo = 0;
  int vB = 0;
  if (C0) {
    const int A = rvis >> 5;
    vB = rvis & 31;
    auto from_lane = [](int t) -> uint64_t { return t <= 0 ? ~0ull : (t >= 64 ? 0ull : (~0ull << t)); };
    vis_hi = from_lane(A + 1);
    vis_lo = from_lane(A);
  }
  uint32_t ev = 0;
  // Groups of 4 positions, software-pipelined: group g+1's keys are rolled and
  // its 4 LDS probes issued before group g's probes are compared, so each
  // group's LDS latency overlaps the next group's arithmetic.  The
  // sched_barrier keeps hipcc from hoisting more than that (VGPRs).
  auto roll4 = [&](int g, uint32_t (&kv)[4], uint2 (&e)[4], uint32_t (&fw)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 4 * g + t;
      kv[t] = (NX1 << 20) + NX2;
      if (j < 31) {
        const uint32_t xo = byte_of(xa[j >> 2], j & 3);
        const uint32_t xn = byte_of(xb[j >> 2], j & 3);
        NX1 += xo - xn;
        NX2 += NX1 + (xo << 11);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) e[t] = *(const uint2*)(kblk + ((kv[t] & KM) | kofs));
    if (FM == 1 || FM == 3) {
#pragma unroll
      for (int t = 0; t < 4; ++t) fw[t] = *(const uint32_t*)(gq.lds + gq.lfo + filt_word_ofs(kv[t]));
    } else if (FM == 2) {
#pragma unroll
      for (int t = 0; t < 4; ++t) fw[t] = gq.gf[gfilt_word(kv[t], gq.gmask)];
    }
    if (FM == 3) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t w = filt_test(fw[t], kv[t]) ? gq.gf[gfilt_word(kv[t], gq.gmask)] : 0u;
        fw[t] = w;
      }
    }
  };
  uint32_t kc[4], fc[4];
  uint2 ec[4];
  roll4(0, kc, ec, fc);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    uint32_t kn[4], fn[4];
    uint2 en[4];
    if (g < 7) roll4(g + 1, kn, en, fn);
    if (GLB) {
      // Persistent cache + batch declarations, pass 1: queue filter passes.
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t p = FM == 1 ? filt_test(fc[t], kc[t]) : gfilt_test(fc[t], kc[t]);   // (FM 3: 0 if the LDS one failed)
        *(uint32_t*)(gq.lds + gq.sa) = kc[t];
        gq.sa = min(gq.sa + (p << 8), gq.salim);
        gq.pm |= p << (4 * g + t);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 4 * g + t;
      uint64_t hit = lanes_eq(ec[t].x, kc[t]) | lanes_eq(ec[t].y, kc[t]);
      if (C0) hit |= lanes_eq(kc[t], c0k) & (j < vB ? vis_hi : vis_lo);
#pragma unroll
      for (int k = 0; k < NOVF; ++k) hit |= lanes_eq(o[k], kc[t]);
      ev = shift_in(ev, hit);
    }
    asm volatile("" : "+v"(ev));   // materialise this group's bits before the next group
    __builtin_amdgcn_sched_barrier(0);
    if (GLB && (g == 3 || g == 7)) glb_flush(gq);
    if (g < 7) {
#pragma unroll
      for (int t = 0; t < 4; ++t) { kc[t] = kn[t]; ec[t] = en[t]; fc[t] = fn[t]; }
    }
  }
  return __builtin_bitreverse32(ev) | (GLB ? gq.gev : 0u);   // ev: position j was shifted in at bit 31 - j
}

// Independent chunks of up to 128 KiB (the headline path): the wave's table
// holds only its own chunk's declarations (at most 63), so its probe key need
// not be -lo, which the persistent cache's filters are built on.  It is NX2 =
// -(X2 + CLO), the rolled weighted sum itself (no key instruction), in a
// direct-mapped table of 2 << LOGNB slots (slot = bits 2.. of the key; one
// compare; a key whose slot is taken is an overflow key).  EVW false: return
// only the lanes with a possible hit (per lane, the minimum of slot ^ key over
// its positions is 0), no per-position event bit -- in independent chunks
// almost every piece has none, and a piece that has one is rolled again with
// EVW true for its event word.  Per position: 4 VALU to roll, 1 for the LDS
// address, 1.5 for the xor / min3 (vs 9 for roll_probe's event word).
template <int LOGNB>
__device__ __forceinline__ uint32_t dm_slot_mask() { return ((2u << LOGNB) - 1u) << 2; }
template <int LOGNB>
__device__ __forceinline__ uint32_t dm_empty(uint32_t slot) { return (~slot & ((2u << LOGNB) - 1u)) << 2; }

template <int LOGNB, bool C0, int NOVF, bool EVW>
__device__ __forceinline__ uint64_t roll_probe_dm(const Piece& P, uint32_t NX1, uint32_t NX2, const char* kblk,
                                                  uint32_t kofs, uint32_t c0k, int rvis, const uint32_t* ovp,
                                                  uint32_t novf) {
  const uint32_t KM = (uint32_t)opaque((int)dm_slot_mask<LOGNB>());
  const uint32_t xa[8] = {P.a0[0], P.a0[1], P.a0[2], P.a0[3], P.a1[0], P.a1[1], P.a1[2], P.a1[3]};
  const uint32_t xb[8] = {P.b0[0], P.b0[1], P.b0[2], P.b0[3], P.b1[0], P.b1[1], P.b1[2], P.b1[3]};
  // (unused overflow slots repeat a real overflow key)
  uint32_t o[NOVF > 0 ? NOVF : 1];
#pragma unroll
  for (int k = 0; k < NOVF; ++k) o[k] = readfirst(ovp[(uint32_t)k < novf ? k : 0]);
  uint64_t vis_hi = 0, vis_lo = 0;
  int vB = 0;
  if (C0) {
    const int A = rvis >> 5;
    vB = rvis & 31;
    auto from_lane = [](int t) -> uint64_t { return t <= 0 ? ~0ull : (t >= 64 ? 0ull : (~0ull << t)); };
    vis_hi = from_lane(A + 1);
    vis_lo = from_lane(A);
  }
  static_assert(EVW || !C0, "a piece with a pending candidate takes the event word directly");
  uint32_t ev = 0, amin = ~0u;
  auto roll4 = [&](int g, uint32_t (&kv)[4], uint32_t (&e)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 4 * g + t;
      kv[t] = NX2;
      if (j < 31) {
        const uint32_t xo = byte_of(xa[j >> 2], j & 3);
        const uint32_t xn = byte_of(xb[j >> 2], j & 3);
        NX1 += xo - xn;
        NX2 += NX1 + (xo << 11);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) e[t] = *(const uint32_t*)(kblk + ((kv[t] & KM) | kofs));
  };
  uint32_t kc[4], ec[4];
  roll4(0, kc, ec);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    uint32_t kn[4], en[4];
    if (g < 7) roll4(g + 1, kn, en);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = 4 * g + t;
      if (EVW) {
        uint64_t hit = lanes_eq(ec[t], kc[t]);
        if (C0) hit |= lanes_eq(kc[t], c0k) & (j < vB ? vis_hi : vis_lo);
#pragma unroll
        for (int k = 0; k < NOVF; ++k) hit |= lanes_eq(o[k], kc[t]);
        ev = shift_in(ev, hit);
      }
    }
    if (!EVW) {
      // per lane: the minimum of (slot ^ key) over the positions is 0 iff one
      // matched -- xor + half a min3 per position, no SGPR round trip
      uint32_t xx[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) xx[t] = ec[t] ^ kc[t];
      amin = min(amin, min(xx[0], xx[1]));
      amin = min(amin, min(xx[2], xx[3]));
#pragma unroll
      for (int k = 0; k < NOVF; ++k) {
#pragma unroll
        for (int t = 0; t < 4; t += 2) amin = min(amin, min(o[k] ^ kc[t], o[k] ^ kc[t + 1]));
      }
    }
    if (EVW) asm volatile("" : "+v"(ev));
    __builtin_amdgcn_sched_barrier(0);
    if (g < 7) {
#pragma unroll
      for (int t = 0; t < 4; ++t) { kc[t] = kn[t]; ec[t] = en[t]; }
    }
  }
  return EVW ? (uint64_t)__builtin_bitreverse32(ev) : ballot(amin == 0u);
}

// ------------------------------------------------------------------ kernel

// Waves sharing a SIMD issue by priority, then age: with equal priorities the
// oldest of the four chunk-waves runs ahead and the youngest finishes alone,
// leaving its SIMD under-used.  A wave's priority falls as it parses its
// chunk (bands 1/2, 3/4, 15/16: a wave that reaches a band boundary first
// yields until the others catch up), so the four finish nearly together;
// only the last 1/16 is age-ordered.
__device__ __forceinline__ void progress_priority(int s, int L) {
  const int s16 = 16 * s;                          // sixteenths of the chunk parsed: 16 s / L (no division)
  if (s16 < 8 * L) __builtin_amdgcn_s_setprio(3);
  else if (s16 < 12 * L) __builtin_amdgcn_s_setprio(2);
  else if (s16 < 15 * L) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// One wave encodes chunk `chunk` (one XCodecEncoder::encode call).  Its key
// table is kblk + kofs (LDS), its records T.  STREAM: the cache also holds the
// persistent GPU cache g and the batch declarations b of chunks < chunk,
// probed through the workgroup's LDS filter lfilt.
// What a stream wave probes besides its own table: the workgroup's LDS (base
// = offset 0), where the lane filter sits (lfo), the wave's pass-1 scratch
// (sofs), and which filter pass 1 reads (fmode; 0 = the filter holds nothing).
struct GlbView {
  char* lds;
  uint32_t lfo;
  uint32_t sofs;
  int fmode;   // 0: no probe, 1: LDS lane filter, 2: global lane filter, 3: LDS filter, then global
  uint32_t* ro;   // (stream) the wave's per-declaration output lengths, LDS
  uint32_t* rsv;  // (stream) the wave's restart state, LDS: slot, old nev, nhits, olen, ndecl, restart ndecl
};

template <int LOGNB, int MAXD, bool STREAM, bool LRU = false>
__device__ __forceinline__ void encode_chunk(const EncParams& prm, char* kblk, const uint32_t kofs,
                                             WaveRecs<LOGNB, MAXD, (!STREAM && MAXD <= 72)>& T, const uint32_t chunk,
                                             const GlbView gs) {
  constexpr int NB = 1 << LOGNB;
  // independent chunks of up to 128 KiB: direct-mapped NX2 keys (roll_probe_dm)
  constexpr bool DM = !STREAM && MAXD <= 72;
  const int l = lane_id();

  const uint8_t* x = prm.in + prm.chunk_off[chunk];
  const int L = (int)prm.chunk_len[chunk];
  uint8_t* const out = prm.out + prm.out_off[chunk];
  const bool oob = (prm.flags & XCG_FLAG_OOB) != 0;
  const bool nullcache = (prm.flags & XCG_FLAG_NULLCACHE) != 0;
  uint32_t olen = 0;
  uint32_t n_extract = 0, n_ref = 0, n_coll = 0, n_pieces = 0;

#if defined(XCG_TIMING) || defined(XCG_PHASES)
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef XCG_PHASES
#ifndef XCG_PHASES_SLOT1
#define XCG_PHASES_SLOT1 0   // stats word 1: 0 exact-event time, 1 piece setup time, 2 prefetch wait
#endif
  // diagnostics build: time in the vector phase and in REF-chaining probes
  uint64_t ph_vec = 0, ph_chain = 0, ph_ev = 0, ph_setup = 0, ph_wait = 0;
  uint32_t ph_nev = 0;
#endif
  // A chunk longer than the launch's bound would overrun the records sized
  // for it: refuse it loudly (status bit 3) instead.
  if ((uint32_t)L > prm.max_len || (uint32_t)L / SEG >= (uint32_t)MAXD) {
    if (l == 0) {
      prm.out_len[chunk] = 0;
      if (prm.status) atomicOr(prm.status, 8);
      if (LRU) prm.nev[chunk] = 0;
    }
    return;
  }
  if (L < SEG) {                                   // xcodec_encoder.cc:77-83
    if (L > 0) olen = escape_u(out, x, 0, (uint32_t)L);
    if (l == 0) {
      prm.out_len[chunk] = olen;
      if (LRU) prm.nev[chunk] = 0;                 // (no cache reference; the list is scratch)
    }
    return;
  }

  uint32_t* const keyt = (uint32_t*)(kblk + kofs);
  for (int k = l; k < 2 * NB; k += 64) keyt[k] = DM ? dm_empty<LOGNB>((uint32_t)k) : kempty<LOGNB>((uint32_t)k >> 1);
  uint32_t ndecl = 0, novf = 0;
  // (stream) the own key table overflowed: this parse may have missed one of
  // its own declarations.  The chunk's hit count becomes maxh + 1, which the
  // verification treats as "always re-parse" (structured data can put a
  // transient round's many declarations into few buckets; the re-parse sees the
  // round's lists); a result no verification follows is checked by the driver.
  bool own_ovf = false;

  const int last = L - SEG;                        // last window start
  const int mis = (int)(reinterpret_cast<uintptr_t>(x) & 15u);
  int s = 0, base = 0;
  bool have_cand = false;
  int cand = 0;
  uint32_t cand_lo = 0, cand_hi = 0;
  uint32_t cand_k = 0;                             // (DM) the candidate's probe key
  // In-band independent encoding never outputs a declared hash, and its hi half
  // only matters when a later window matches the declaration's lo: then it is
  // computed from the declared bytes (lookup).  HI_LAZY (odd) marks "not yet";
  // a real hi has its low 4 bits clear (mix(), xcodec_hash.h:155-164).
  constexpr uint32_t HI_LAZY = 1u;
  const bool lazy_hi = !STREAM && !oob;
  bool c0_in_table = true;                         // pending candidate already inserted?

  Piece P;
  int p_prev = INT32_MIN;
  // Registers that already hold window bytes: the previous piece's A half
  // (bytes [p_prev, p_prev + 2048) across the wave) and the next piece's
  // prefetched B half.
  u32x4 nb0 = {0u, 0u, 0u, 0u}, nb1 = nb0;
  int nb_start = INT32_MIN;
  // A candidate set at the piece start has its whole segment in the wave's A
  // registers; its EXTRACT body is written to the output right then, at the
  // offset the declaration will have if nothing cancels it (spec_olen).
  int spec_cand = -1;
  uint32_t spec_olen = 0;
  uint32_t totXA = 0, totTA = 0;                   // sums over the A half (carried)

  // Insert a declaration into the LDS table (XCodecMemoryCache::enter,
  // xcodec_cache.h:303-325) -- by lane 0, visible to later LDS reads of the
  // wave (LDS ops of one wave complete in order).
  // (DM) enter into slot sl of the direct-mapped table, whose word s0 the
  // caller has read
  auto insert_dm = [&](uint32_t lo, uint32_t hi, uint32_t c, uint32_t k2, uint32_t sl, uint32_t s0) {
    const uint32_t d = ndecl++, ke = dm_empty<LOGNB>(sl);
    if (l == 0) {
      T.rlo[d] = lo; T.rhi[d] = hi; T.rc[d] = c;
      if (s0 == ke) keyt[sl] = k2;
      else if (novf < (uint32_t)ovf_cap<MAXD, DM>()) T.ovf_k[novf] = k2;
    }
    if (s0 != ke) {
      if (novf < (uint32_t)ovf_cap<MAXD, DM>()) ++novf;
      else if (l == 0 && prm.status) atomicOr(prm.status, 1);
    }
    __builtin_amdgcn_wave_barrier();
  };
  auto insert = [&](uint32_t lo, uint32_t hi, uint32_t c, uint32_t k2) {
    if (DM) {
      const uint32_t sl = (k2 >> 2) & ((2u << LOGNB) - 1u);
      insert_dm(lo, hi, c, k2, sl, readfirst(keyt[sl]));
      return;
    }
    const uint32_t d = ndecl++;
    const uint32_t k = probe_key(lo);
    const uint32_t b = kbucket<LOGNB>(k), ke = kempty<LOGNB>(b);
    const uint32_t s0 = readfirst(keyt[2 * b]), s1 = readfirst(keyt[2 * b + 1]);
    if (l == 0) {
      T.rlo[d] = lo; T.rhi[d] = hi; T.rc[d] = c;
      if (s0 == ke) keyt[2 * b] = k;
      else if (s1 == ke) keyt[2 * b + 1] = k;
      else if (novf < (uint32_t)ovf_cap<MAXD>()) T.ovf_k[novf] = k;
    }
    if (s0 != ke && s1 != ke) {
      if (novf < (uint32_t)ovf_cap<MAXD>()) ++novf;
      else if (STREAM) own_ovf = true;
      else if (l == 0 && prm.status) atomicOr(prm.status, 1);
#ifdef XCG_DEBUG_OVF
      if (l == 0 && novf >= (uint32_t)ovf_cap<MAXD>())
        printf("ovf chunk %u decl %u lo %08x hi %08x at %u bucket %u\n", chunk, d, lo, hi, c, b);
#endif
    }
    __builtin_amdgcn_wave_barrier();
  };

  // Exact lookup: declaration index whose hash is (lo, hi), or -1; or -2 - d
  // when record d matches lo but its hi has not been computed yet.
  auto rec_matches = [&](uint32_t d, uint32_t lo, uint32_t hi, int& found) {
    if (readfirst(T.rlo[d]) != lo) return;
    const uint32_t rh = readfirst(T.rhi[d]);
    if (rh == HI_LAZY) found = -2 - (int)d;
    else if (rh == hi) found = (int)d;
  };
  auto lookup = [&](uint32_t lo, uint32_t hi) -> int {
    // records whose lo matches, by a wave ballot (at most MAXD of them)
    int found = -1;
    for (uint32_t base = 0; base < ndecl && found == -1; base += 64) {
      const uint32_t d = base + (uint32_t)l;
      uint64_t m = ballot(d < ndecl && T.rlo[d] == lo);
      while (m && found == -1) {
        rec_matches(base + (uint32_t)__builtin_ctzll(m), lo, hi, found);
        m &= m - 1;
      }
    }
    return found;
  };

  // Segment bytes of a hash in the persistent cache or, declared by an
  // earlier chunk of the batch, in the batch input (nullptr if neither).
  // A batch hit is recorded: the verification after the round re-parses the
  // chunk if that declaration's visibility or bytes change (xcg_verify_*).
  uint32_t nh = 0;
  // Bounded cache: every reference the chunk makes to the cache, in order --
  // enter (declaration d), lookup hit (XCodecMemoryCache::lookup refreshes the
  // entry's recency whether or not the bytes then match, xcodec_cache.h:348-364),
  // and a lookup of a persistent entry the LRU has evicted by then.  The
  // LRU pass (xcg_lru.hip) derives the eviction times from these.
  uint32_t ne = 0;
  auto record = [&](uint32_t lo, uint32_t hi, uint32_t t, uint32_t kind, uint32_t ref) {
    if (ne < prm.maxe && l == 0) {
      prm.ev[(uint64_t)chunk * prm.maxe + ne] = make_uint4(lo, hi, t, (kind << 30) | ref);
      if (prm.eo) prm.eo[(uint64_t)chunk * prm.maxe + ne] = ~0u;
    }
    ++ne;
  };
  // (after a REF: the output length, at the lookup that made it)
  auto ref_made = [&]() {
    if (LRU && prm.eo && l == 0 && ne > 0 && ne - 1 < prm.maxe) prm.eo[(uint64_t)chunk * prm.maxe + ne - 1] = olen;
  };
  auto cache_src = [&](uint32_t lo, uint32_t hi, int at) -> const uint8_t* {
    uint64_t gv, bv;                               // (both tables probed in one round trip)
    tab_lookup2(prm.g, prm.use_b ? prm.b : prm.g, lo, hi, gv, bv);
    if (gv != ~0ull) {
      if (!LRU) return prm.pool + gv * (uint64_t)SEG;
      const uint32_t t = 2u * (uint32_t)at + 1u;
      if ((((uint64_t)chunk << 21) | t) < prm.ptime[gv]) {
        record(lo, hi, t, EV_GHIT, (uint32_t)gv);
        return prm.pool + gv * (uint64_t)SEG;
      }
      record(lo, hi, t, EV_GMISS, (uint32_t)gv);   // evicted earlier in the batch
    }
    if (prm.use_b) {
      if (bv != ~0ull && (uint32_t)(bv >> 32) < chunk) {
        if (nh < prm.maxh && l == 0) prm.hits[(uint64_t)chunk * prm.maxh + nh] = ((uint64_t)hi << 32) | lo;
        ++nh;
        if (LRU) record(lo, hi, 2u * (uint32_t)at + 1u, EV_HIT, 1u);   // (ref 1: a batch hit, listed in hits)
        return prm.in + prm.chunk_off[bv >> 32] + (uint32_t)bv;
      }
    }
    return nullptr;
  };
  // Could the cache or the batch hold probe key k?  (the LDS lane filter, no
  // false negatives; the global-filter mode goes to the exact tables)
  auto glb_pass = [&](uint32_t k) -> bool {
    if (gs.fmode == 0) return false;
    if (gs.fmode == 2) return true;   // (1 and 3: the LDS filter)
    return readfirst(filt_test(*(const uint32_t*)(gs.lds + gs.lfo + filt_word_ofs(k)), k)) != 0u;
  };
  bool chain = false;                              // the last op was a REF

  // encode_declaration (xcodec_encoder.cc:276-313), made while examining
  // window `at` (the enter precedes that window's lookup).
  auto declare = [&](int at) {
    if (LRU) record(cand_lo, cand_hi, 2u * (uint32_t)at, EV_ENTER, n_extract);
    if (cand > base) olen += escape_u(out + olen, x, (uint32_t)base, (uint32_t)cand);
    if (!nullcache && !c0_in_table) insert(cand_lo, cand_hi, (uint32_t)cand, cand_k);
    if (oob) {
      wave_put_ref(out + olen, cand_lo, cand_hi);           // :288-295
      olen += 10;
    } else {
      if (l < 2) out[olen + l] = (uint8_t)(l == 0 ? MAGIC : OP_EXTRACT);   // :300-302
      if (!(cand == spec_cand && olen == spec_olen)) wave_copy(out + olen + 2, x + cand, SEG);
      olen += 2 + SEG;
    }
    ++n_extract;
    if (STREAM && gs.ro && !nullcache && l == 0 && ndecl > 0) gs.ro[ndecl - 1] = olen;   // (the candidate's record)
    base = cand + SEG;
    have_cand = false;
    c0_in_table = true;
  };

  // ---- Re-parse restart (bounded / pair passes after the first, xcg_lru.hip /
  // xcg_pair.hip).  The previous pass's parse of this chunk stands up to its
  // first lookup the new eviction times contradict (in-chunk time bad_t).
  // Resume at its last clean point before that -- right after a declaration or
  // a REF: parse point = base, nothing pending, about to look that window up
  // (xcodec_encoder.cc:183-208) -- from the state its rows give, and stop as
  // soon as the new parse reaches a clean point the old one also passed
  // through, with the same own declarations as far as the old remainder looks
  // them up: the old remainder is then appended (rows here, output bytes by
  // xcg_splice_kernel after the launch).  The rows of a chunk are in time
  // order, so everything before the restart point is still in place.
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  int rs_q = -1;
  uint32_t rs_hi = 0;                              // in-chunk time of the latest contradicted lookup
  bool spliced = false;
  if (LRU && STREAM && prm.rs.bslot && prm.eo && gs.ro && gs.rsv && !nullcache) {
    const uint32_t rs_slot = readfirst(prm.rs.bslot[chunk]);
    const uint32_t tb = readfirst(prm.rs.bad_t[chunk]);
    rs_hi = readfirst(prm.rs.bad_hi[chunk]);
    if (rs_slot != NONE && tb != NONE) {
      const uint4* const odl = prm.decl + (uint64_t)chunk * prm.maxd;   // old rows (in place until the end)
      const uint4* oev = prm.rs.b_ev + (uint64_t)rs_slot * prm.maxe;
      const uint32_t* oeo = prm.rs.b_eo + (uint64_t)rs_slot * prm.maxe;
      const uint32_t o_nev = min(readfirst(prm.rs.b_cnt[4 * rs_slot]), prm.maxe);
      const uint32_t o_nd = readfirst(prm.rs.b_cnt[4 * rs_slot + 3]);
      // the latest clean point q (a window, <= last) with 2q + 1 <= tb
      int best = -1;
      uint32_t best_olen = 0;
      for (uint32_t i0 = 0; i0 < o_nev; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)l;
        int q = -1;
        uint32_t ol = 0;
        if (i < o_nev) {
          const uint4 e = oev[i];
          if ((e.w >> 30) == EV_ENTER) {               // declared while examining window e.z / 2
            const uint32_t d = e.w & EV_REF_MASK;
            if (d < o_nd) { q = (int)(e.z >> 1); ol = odl[d].w; }
          } else if (oeo[i] != NONE) {                  // a REF at window (e.z - 1) / 2
            q = (int)((e.z - 1u) >> 1) + SEG;
            ol = oeo[i];
          }
          if (q > last || (q >= 0 && 2u * (uint32_t)q + 1u > tb)) q = -1;
        }
        int mq = q;
        for (int off = 32; off >= 1; off >>= 1) mq = max(mq, __shfl_xor(mq, off));
        mq = readfirst(mq);
        if (mq > best) {
          const uint64_t bl = ballot(q == mq);
          best = mq;
          best_olen = readlane(ol, (int)__builtin_ctzll(bl));
        }
      }
      if (best >= 0) {
        rs_q = best;
        uint32_t ne_r = 0, nd_r = 0, nh_r = 0, nref_r = 0;
        for (uint32_t i0 = 0; i0 < o_nev; i0 += 64) {
          const uint32_t i = i0 + (uint32_t)l;
          bool in = false, ent = false, bh = false, rf = false;
          if (i < o_nev) {
            const uint4 e = oev[i];
            in = e.z < 2u * (uint32_t)best + 1u;
            ent = in && (e.w >> 30) == EV_ENTER;
            bh = in && (e.w >> 30) == EV_HIT && (e.w & EV_REF_MASK) == 1u;
            rf = in && oeo[i] != NONE;
          }
          ne_r += (uint32_t)__builtin_popcountll(ballot(in));
          nd_r += (uint32_t)__builtin_popcountll(ballot(ent));
          nh_r += (uint32_t)__builtin_popcountll(ballot(bh));
          nref_r += (uint32_t)__builtin_popcountll(ballot(rf));
        }
        for (uint32_t d = 0; d < nd_r; ++d) {           // the own records and key table so far
          const uint4 r = odl[d];
          insert(readfirst(r.x), readfirst(r.y), readfirst(r.z), 0u);   // (stream: keyed by lo)
          if (l == 0) gs.ro[d] = r.w;
        }
        if (l == 0) {
          gs.rsv[0] = rs_slot;
          gs.rsv[1] = o_nev;
          gs.rsv[2] = readfirst(prm.rs.b_cnt[4 * rs_slot + 1]);
          gs.rsv[3] = readfirst(prm.rs.b_cnt[4 * rs_slot + 2]);
          gs.rsv[4] = o_nd;
          gs.rsv[5] = nd_r;
        }
        __builtin_amdgcn_wave_barrier();
        ne = ne_r;
        nh = nh_r;
        olen = best_olen;
        n_extract = nd_r;
        n_ref = nref_r;
        s = base = best;
        chain = true;
      }
    }
  }
  // Splice at clean point s (the new parse is about to look window s up, with
  // nothing pending): true when the old parse had the same state there.
  auto try_splice = [&]() -> bool {
    const uint32_t rs_slot = readfirst(gs.rsv[0]), o_nev = readfirst(gs.rsv[1]), o_nh = readfirst(gs.rsv[2]);
    const uint32_t o_olen = readfirst(gs.rsv[3]), o_nd = readfirst(gs.rsv[4]), rs_nd = readfirst(gs.rsv[5]);
    const uint4* const odl = prm.decl + (uint64_t)chunk * prm.maxd;
    const uint4* const oev = prm.rs.b_ev + (uint64_t)rs_slot * prm.maxe;
    const uint32_t* const oeo = prm.rs.b_eo + (uint64_t)rs_slot * prm.maxe;
    // the old clean point at s: a declaration made at window s, or a REF at s - 2048
    int it = -1, dt = -1;
    uint32_t ol_old = 0;
    for (uint32_t i0 = 0; i0 < o_nev && it < 0; i0 += 64) {
      const uint32_t i = i0 + (uint32_t)l;
      bool hit = false;
      if (i < o_nev) {
        const uint4 e = oev[i];
        hit = ((e.w >> 30) == EV_ENTER && e.z == 2u * (uint32_t)s) ||
              (oeo[i] != NONE && s >= SEG && e.z == 2u * (uint32_t)(s - SEG) + 1u);
      }
      const uint64_t bl = ballot(hit);
      if (bl) it = (int)(i0 + (uint32_t)__builtin_ctzll(bl));
    }
    if (it < 0) return false;
    {
      const uint4 e = oev[it];
      if ((e.w >> 30) == EV_ENTER) {
        dt = (int)(e.w & EV_REF_MASK) + 1;
        ol_old = readfirst(odl[dt - 1].w);
      } else {
        ol_old = readfirst(oeo[it]);
        uint32_t c = 0;                                  // declarations before the REF
        for (uint32_t i0 = 0; i0 < (uint32_t)it; i0 += 64) {
          const uint32_t i = i0 + (uint32_t)l;
          c += (uint32_t)__builtin_popcountll(ballot(i < (uint32_t)it && (oev[i].w >> 30) == EV_ENTER));
        }
        dt = (int)c;
      }
    }
    ++it;                                                // the old remainder's first reference
    if ((uint32_t)dt < rs_nd || (uint32_t)dt > o_nd) return false;
    // own declarations that differ: the new ones since the restart vs the old ones
    const uint32_t nn = ndecl - rs_nd, no = (uint32_t)dt - rs_nd;
    if (nn > 32 || no > 32) return false;
    uint32_t hlo = 0, hhi = 0;
    if ((uint32_t)l < nn) { hlo = T.rlo[rs_nd + l]; hhi = T.rhi[rs_nd + l]; }
    else if ((uint32_t)l >= 32 && (uint32_t)l - 32 < no) { const uint4 r = odl[rs_nd + l - 32]; hlo = r.x; hhi = r.y; }
    const bool is_new = (uint32_t)l < nn, is_old = (uint32_t)l >= 32 && (uint32_t)l - 32 < no;
    bool inD = is_new || is_old;
    for (uint32_t j = 0; j < (nn > no ? nn : no); ++j) {   // (uniform: readlane of lanes j and 32 + j)
      const uint32_t nlo = readlane(hlo, (int)j), nhi = readlane(hhi, (int)j);
      const uint32_t olo = readlane(hlo, (int)(32 + j)), ohi = readlane(hhi, (int)(32 + j));
      if (is_old && j < nn && hlo == nlo && hhi == nhi) inD = false;
      if (is_new && j < no && hlo == olo && hhi == ohi) inD = false;
    }
    const uint64_t dm = ballot(inD);
    // The old remainder's lookups of these are in its rows only where the old
    // parse found the hash: as its own record (the old ones), in the
    // persistent table, or in the batch table visible to this chunk.  A new
    // declaration found nowhere else may have been missed there unrecorded
    // (an in-chunk repeat): no splice then.
    bool unknown = false;
    if (is_new && inD) {
      bool known = tab_lookup_t(prm.g, hlo, hhi) != ~0ull;
      if (!known && prm.use_b) {
        const uint64_t bv = tab_lookup_t(prm.b, hlo, hhi);
        known = bv != ~0ull && (uint32_t)(bv >> 32) < chunk;
      }
      unknown = !known;
    }
    if (ballot(unknown)) return false;
    // the old remainder must not look any of them up (or declare one)
    for (uint32_t i0 = (uint32_t)it; i0 < o_nev; i0 += 64) {
      const uint32_t i = i0 + (uint32_t)l;
      const uint4 e = i < o_nev ? oev[i] : make_uint4(0u, 0u, 0u, 0u);
      bool clash = false;
      uint64_t m = dm;
      while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        clash |= i < o_nev && e.x == (uint32_t)readlane(hlo, j) && e.y == (uint32_t)readlane(hhi, j);
      }
      if (ballot(clash)) return false;
    }
    // splice: the old remainder's declarations, references and batch hits follow
    const uint32_t delta = olen - ol_old;                // (mod 2^32: offsets shift by it)
    const uint32_t nd0 = ndecl;
    for (uint32_t d = (uint32_t)dt; d < o_nd && ndecl < (uint32_t)MAXD; ++d) {
      const uint4 r = odl[d];
      if (l == 0) {
        T.rlo[ndecl] = r.x; T.rhi[ndecl] = r.y; T.rc[ndecl] = r.z;
        gs.ro[ndecl] = r.w + delta;
      }
      ++ndecl;
    }
    uint32_t hb = 0;                                     // batch hits before the old remainder
    for (uint32_t i0 = 0; i0 < (uint32_t)it; i0 += 64) {
      const uint32_t i = i0 + (uint32_t)l;
      hb += (uint32_t)__builtin_popcountll(
          ballot(i < (uint32_t)it && (oev[i].w >> 30) == EV_HIT && (oev[i].w & EV_REF_MASK) == 1u));
    }
    uint32_t nref_t = 0;
    for (uint32_t i0 = (uint32_t)it; i0 < o_nev; i0 += 64) {
      const uint32_t i = i0 + (uint32_t)l;
      if (i < o_nev) {
        uint4 e = oev[i];
        if ((e.w >> 30) == EV_ENTER) e.w = (EV_ENTER << 30) | ((e.w & EV_REF_MASK) - (uint32_t)dt + nd0);
        const uint32_t o = oeo[i];
        const uint32_t k = ne + (i - (uint32_t)it);
        if (k < prm.maxe) {
          prm.ev[(uint64_t)chunk * prm.maxe + k] = e;
          prm.eo[(uint64_t)chunk * prm.maxe + k] = o == NONE ? NONE : o + delta;
        }
      }
      nref_t += (uint32_t)__builtin_popcountll(ballot(i < o_nev && oeo[i] != NONE));
    }
    ne += o_nev - (uint32_t)it;
    const uint64_t* oh = prm.rs.b_hits + (uint64_t)rs_slot * prm.maxh;
    for (uint32_t j = hb + (uint32_t)l; j < o_nh && j < prm.maxh; j += 64) {
      const uint32_t k = nh + (j - hb);
      if (k < prm.maxh) prm.hits[(uint64_t)chunk * prm.maxh + k] = oh[j];
    }
    nh += o_nh > hb ? o_nh - hb : 0u;
    n_ref += nref_t;
    n_extract += o_nd - (uint32_t)dt;
    if (l == 0) prm.rs.splice[chunk] = make_uint4(olen, ol_old, o_olen, 1u);
    olen += o_olen - ol_old;
    return true;
  };

  while (s <= last) {
#ifdef XCG_PHASES
    const uint64_t tp0 = __builtin_amdgcn_s_memrealtime();
#endif
    // ---- piece geometry: q0 = p + 32 lane, loads 16-byte aligned in memory
    const int p = s - (int)(((uint32_t)mis + (uint32_t)s) & 15u);
    const int l = opaque(lane_id());
    const int q0 = p + 32 * l;
    const bool contig = (p == p_prev + SEG);
    ++n_pieces;
    progress_priority(s, L);
    // vmcnt counts loads and stores together, in order (gfx9): every wait on
    // a load also waits for all older stores.  So fresh loads are waited for
    // here, inside their branch, and the prefetch below is waited for after
    // the vector phase -- never right behind its own issue.
    // (contig implies nb_start == p: the previous piece prefetched this B.)
    if (contig) {
      P.a0 = P.b0; P.a1 = P.b1;
      P.sxa = P.sxb; P.sqxa = P.sqxb;
      P.b0 = nb0; P.b1 = nb1;
    } else {
      P.a0 = piece_ld_safe<STREAM>(x, q0, L);
      P.a1 = piece_ld_safe<STREAM>(x, q0 + 16, L);
      P.b0 = piece_ld_safe<STREAM>(x, q0 + SEG, L);
      P.b1 = piece_ld_safe<STREAM>(x, q0 + SEG + 16, L);
      vuse(P.a0); vuse(P.a1); vuse(P.b0); vuse(P.b1);
      seg_sums(P.a0, P.a1, P.sxa, P.sqxa);
    }
    seg_sums(P.b0, P.b1, P.sxb, P.sqxb);
    p_prev = p;

    // ---- start sums of lane l's first window (positions relative to p)
    const uint32_t qa = 32u * (uint32_t)l, qb = 2048u + 32u * (uint32_t)l;
    const uint32_t ta = qa * P.sxa + P.sqxa, tb = qb * P.sxb + P.sqxb;
    if (!contig) {
      totXA = wave_sum(P.sxa); totTA = wave_sum(ta);
    }
    const uint32_t dx = P.sxb - P.sxa, dt = tb - ta;
    const uint32_t ix = wave_incl_scan(dx), it = wave_incl_scan(dt);
    const uint32_t X1 = totXA + ix - dx;
    const uint32_t TT = totTA + it - dt;
    const uint32_t X2c = (2048u + qa) * X1 - TT + CLO;
    // Next piece's A half (if contiguous) is this B half, shifted by 2048.
    const uint32_t totXB = totXA + readlane(ix, 63);
    const uint32_t totTB = totTA + readlane(it, 63) - 2048u * totXB;
    // probe key of the lane's first window
    const uint32_t NX1 = 0u - X1, NX2 = 0u - X2c;
    const uint32_t k0 = (NX1 << 20) + NX2;

    // Prefetch the next contiguous piece's entering bytes; they land while
    // this piece rolls (issued after every use of this piece's loads).
    nb_start = p + SEG;
    if (nb_start < last) {                         // (nb_start == last: decided as this piece's tail1 window)
      if (p + 3 * SEG <= L) {                      // (uniform) every lane's 32 bytes inside the chunk: no guards
        nb0 = piece_ld<STREAM>(x + q0 + 2 * SEG);
        nb1 = piece_ld<STREAM>(x + q0 + 2 * SEG + 16);
      } else {
        nb0 = piece_ld_safe<STREAM>(x, q0 + 2 * SEG, L);
        nb1 = piece_ld_safe<STREAM>(x, q0 + 2 * SEG + 16, L);
      }
    }

    // ---- REF chaining (stream semantics).  The previous piece ended with a
    // REF, so this piece starts at the parse point with no candidate pending;
    // in REF-dense streams (warm caches, duplicated runs) the window there is
    // usually the next REF.  Probe it exactly (lookup, find_reference
    // xcodec_encoder.cc:374-416) before rolling 2048 positions; a miss goes
    // through the filters only, and a miss or a collision falls through to
    // the ordinary vector phase, which decides position s itself.
    // The same holds right after a declaration: a candidate that survived its
    // 2048 windows is declared here, at window s = cand + 2048, before that
    // window's lookup (:183-196) -- and when the data repeats in 2 KiB blocks
    // the window at the end of a new block is often the next REF.
    int chain_miss = -1;
    if (STREAM && !nullcache && !chain && have_cand && cand + SEG == s) {
      declare(s);
      chain = true;
    }
    // a clean point past every contradicted lookup: rejoin the old parse?
    if (LRU && rs_q >= 0 && chain && s > rs_q && 2u * (uint32_t)s + 1u > rs_hi && try_splice()) {
      spliced = true;
      break;
    }
    if (STREAM && chain && !nullcache) {
#ifdef XCG_PHASES
      const uint64_t tc0 = __builtin_amdgcn_s_memrealtime();
#endif
      chain = false;
      uint32_t lo, hi;
      if (s == p) {
        lo = 0u - readfirst(k0);
        hi = readfirst(lane_window_hi(P, 0));
      } else {
        const uint3 h = window_hash_u(x + s);
        lo = h.x; hi = h.y;
      }
      const int d = lookup(lo, hi);                 // stream records carry their hi
      const uint8_t* src = d >= 0 ? x + readfirst(T.rc[d]) : nullptr;
      if (LRU && d >= 0) record(lo, hi, 2u * (uint32_t)s + 1u, EV_HIT, 0u);
      // (straight to the exact tables after the LDS lane filter: a chain probe
      // hits often, and both tables cost one round trip together)
      if (src == nullptr && glb_pass(probe_key(lo))) src = cache_src(lo, hi, s);
      if (src != nullptr && (s == p ? equal2048_regs(src, P.a0, P.a1) : equal2048_u(src, x + s))) {
        wave_put_ref(out + olen, lo, hi);           // encode_reference :342-372
        olen += 10;
        ref_made();
        ++n_ref;
        base = s + SEG;
        s = base;
        chain = true;
        totXA = totXB; totTA = totTB;               // (as at the end of a piece)
#ifdef XCG_PHASES
        ph_chain += __builtin_amdgcn_s_memrealtime() - tc0;
#endif
        continue;
      }
      if (src == nullptr) chain_miss = s;          // an exact miss: the vector phase's event at s is moot
#ifdef XCG_PHASES
      ph_chain += __builtin_amdgcn_s_memrealtime() - tc0;
#endif
    }

    // ---- vector phase
#ifdef XCG_PHASES
    const uint64_t tv0 = __builtin_amdgcn_s_memrealtime();
    ph_setup += tv0 - tp0;
#endif
    uint32_t ev = 0;
    bool quiet = false;                            // (DM) no lane has a possible hit in this piece
    const int pe = min(p + SEG, last + 1);         // piece end (exclusive)
    if (!nullcache) {
      // c0 = the pending candidate; once it is visible from the piece start on,
      // it goes straight into the table (a REF can no longer cancel it).
      if (have_cand && !c0_in_table && cand + SEG <= p) {
        insert(cand_lo, cand_hi, (uint32_t)cand, cand_k);
        c0_in_table = true;
      }
      if (pe - s <= 2) {
        // One or two positions left (every chunk of 2048 k bytes ends with a
        // one-position piece): decide them exactly, as events, instead of
        // rolling 2048 positions for them.
        ev = lane_id() == 0 ? ((1u << (uint32_t)(pe - s)) - 1u) << (uint32_t)(s - p) : 0u;
      } else {
        const bool c0 = have_cand && !c0_in_table;
        const int vis = cand + SEG;
        const int rvis = vis - p;
        const uint32_t c0k = DM ? cand_k : probe_key(cand_lo);
        // Bucket overflows are rare (three of a chunk's keys in one 2-slot
        // bucket); one overflow key costs one compare, more cost eight (32
        // beyond eight, in frames of up to 512 KiB).
        constexpr int OC = ovf_cap<MAXD, DM>();
        uint32_t ovk[OC];
  #pragma unroll
        for (int k = 0; k < (DM ? 1 : OC); ++k) ovk[k] = novf ? readfirst(T.ovf_k[(uint32_t)k < novf ? k : 0]) : 0u;
        const uint32_t sa0 = gs.sofs + 4u * (uint32_t)lane_id();
        GlbQ gq{gs.lds, gs.lfo, prm.lf.gfilt, prm.lf.gmask, prm.lf.ftab, prm.lf.fmask, sa0, sa0, sa0 + 256u * GSLOTS,
                0u, 0u};
        // G = probe the persistent cache / batch declarations too
        auto roll = [&](auto c0t, auto novft, auto glbt) {
          return roll_probe<LOGNB, decltype(c0t)::value, decltype(novft)::value, decltype(glbt)::value>(
              P, NX1, NX2, kblk, kofs, c0k, rvis, ovk, gq);
        };
        using T0 = std::integral_constant<bool, false>;
        using T1 = std::integral_constant<bool, true>;
        using N0 = std::integral_constant<int, 0>;
        using N1 = std::integral_constant<int, 1>;
        using N8 = std::integral_constant<int, 8>;
        using NC = std::integral_constant<int, OC>;
        auto by_novf = [&](auto glbt) {
          if (novf == 0) return c0 ? roll(T1{}, N0{}, glbt) : roll(T0{}, N0{}, glbt);
          if (novf == 1) return c0 ? roll(T1{}, N1{}, glbt) : roll(T0{}, N1{}, glbt);
          // duplicates of a real overflow key pad the unused slots
          if (OC == 8 || novf <= 8) return c0 ? roll(T1{}, N8{}, glbt) : roll(T0{}, N8{}, glbt);
          return c0 ? roll(T1{}, NC{}, glbt) : roll(T0{}, NC{}, glbt);
        };
        if constexpr (DM) {
          // the lane mask of possible hits first; the event word only if any
          auto rolld = [&](auto c0t, auto novft, auto evwt) -> uint64_t {
            return roll_probe_dm<LOGNB, decltype(c0t)::value, decltype(novft)::value, decltype(evwt)::value>(
                P, NX1, NX2, kblk, kofs, c0k, rvis, T.ovf_k, novf);
          };
          auto by_novf_dm = [&](auto evwt) -> uint64_t {
            if (novf == 0) return rolld(T0{}, N0{}, evwt);
            if (novf == 1) return rolld(T0{}, N1{}, evwt);
            return rolld(T0{}, N8{}, evwt);
          };
#ifdef XCG_EXP_NOVEC   // (timing experiment only: output is wrong)
          if (true) {
            ev = 0;
          } else
#endif
          if (c0 || novf > 8) {   // (rare: the event word straight away)
            if (novf == 0) ev = (uint32_t)rolld(T1{}, N0{}, T1{});
            else if (novf == 1) ev = (uint32_t)rolld(T1{}, N1{}, T1{});
            else if (novf <= 8) ev = (uint32_t)rolld(T1{}, N8{}, T1{});
            else ev = (uint32_t)(c0 ? rolld(T1{}, NC{}, T1{}) : rolld(T0{}, NC{}, T1{}));
          } else {
            quiet = by_novf_dm(T0{}) == 0;
            ev = quiet ? 0u : (uint32_t)by_novf_dm(T1{});
          }
        } else if (STREAM && gs.fmode == 1) {
          ev = by_novf(std::integral_constant<int, STREAM ? 1 : 0>{});
        } else if (STREAM && gs.fmode == 2) {
          ev = by_novf(std::integral_constant<int, STREAM ? 2 : 0>{});
        } else if (STREAM && gs.fmode == 3) {
          ev = by_novf(std::integral_constant<int, STREAM ? 3 : 0>{});
        } else {
          ev = by_novf(std::integral_constant<int, 0>{});
        }
        // positions past the last window are not positions (branch-free mask)
        const int nvalid = pe - q0;
        const uint32_t vm = nvalid >= 32 ? 0xFFFFFFFFu : ((1u << (uint32_t)max(nvalid, 0)) - 1u);
        ev &= vm;
        if (STREAM && chain_miss >= 0) {         // (chain_miss == s: decided by the chain probe)
          const int rel = chain_miss - p;
          if (lane_id() == (rel >> 5)) ev &= ~(1u << (rel & 31));
        }
      }
    }
    // The prefetch has had the vector phase to land; take it before the
    // resolve phase issues this piece's stores.
#ifdef XCG_PHASES
    const uint64_t tw0 = __builtin_amdgcn_s_memrealtime();
#endif
    vuse(nb0); vuse(nb1);                          // (unconditional: so the compiler sees them waited)
#ifdef XCG_PHASES
    ph_wait += __builtin_amdgcn_s_memrealtime() - tw0;
#endif

#ifdef XCG_PHASES
    ph_vec += __builtin_amdgcn_s_memrealtime() - tv0;
#endif
    // ---- resolve phase (wave-uniform)
    // A chunk whose last window is one past a full piece (every chunk of
    // 2048 k + 2048 bytes: C2's 64 KiB, C4's 4 KiB) decides that window here,
    // as an event (hashed by the one window-hash call site), instead of in a
    // piece of its own.
    const bool tail1 = pe == p + SEG && last == pe;
    const int pe_x = tail1 ? pe + 1 : pe;
    auto next_event = [&](int from) -> int {
      if (tail1 && from == pe) return from;
      const int rel = from - p;
      const int ls = rel >> 5, bs = rel & 31;
      uint32_t m = l < ls ? 0u : (l == ls ? (ev & (0xFFFFFFFFu << bs)) : ev);
      const uint64_t bal = ballot(m != 0u);
      if (bal == 0) return INT32_MAX;
      const int lw = __builtin_ctzll(bal);
      const uint32_t mm = readlane(m, lw);
      return p + 32 * lw + __builtin_ctz(mm);
    };
    auto hash_at = [&](int pos, uint32_t& lo, uint32_t& hi, uint32_t& k2) {
      const int rel = pos - p;
      if ((rel & 31) == 0 && rel < SEG) {
        lo = 0u - readlane(k0, rel >> 5);
        hi = lazy_hi ? HI_LAZY : readfirst(lane_window_hi(P, rel >> 5));
        k2 = DM ? readlane(NX2, rel >> 5) : 0u;
      } else {
        const uint3 h = window_hash_u(x + pos);
        lo = h.x; hi = h.y; k2 = h.z;
      }
    };

#ifdef XCG_EXP_NORESOLVE   // (timing experiment only: output is wrong)
    s = pe;
#endif
    // Independent chunks' steady state: the candidate set at the previous
    // piece's start is declared here (its key went into the table before the
    // vector phase, its body was stored from registers), nothing matched, and
    // the next candidate is this piece's first window -- the resolve loop
    // below would do exactly this, through two event searches.
    // The new candidate can no longer be cancelled: positions before its
    // declaration point (the next piece's start) are all in this quiet piece.
    // So it enters the table now (XCodecMemoryCache::enter at its declaration,
    // visible from the next piece on), its slot read overlapping the stores.
    if (DM && quiet && !oob && !nullcache && have_cand && c0_in_table && cand + SEG == s && s == p && base == cand &&
        spec_cand == cand && spec_olen == olen && pe == p + SEG) {
      const uint32_t k2 = readlane(NX2, 0);
      const uint32_t sl = (k2 >> 2) & ((2u << LOGNB) - 1u);
      const uint32_t s0v = keyt[sl];
      if (l < 2) out[olen + l] = (uint8_t)(l == 0 ? MAGIC : OP_EXTRACT);   // encode_declaration :300-302
      olen += 2 + SEG;
      ++n_extract;
      base = s;
      cand = s;                                     // :246-248, the hash from registers
      cand_lo = 0u - readlane(k0, 0);
      cand_hi = lazy_hi ? HI_LAZY : readfirst(lane_window_hi(P, 0));
      cand_k = k2;
      uint8_t* dst = out + olen + 2 + 32 * lane_id();
      *(u32x4_u*)dst = P.a0;
      *(u32x4_u*)(dst + 16) = P.a1;
      spec_cand = s;
      spec_olen = olen;
      s = pe;
      insert_dm(cand_lo, cand_hi, (uint32_t)cand, k2, sl, readfirst(s0v));   // (its slot already read)
      c0_in_table = true;
    }
    while (s < pe_x) {
      if (have_cand && cand + SEG <= s) declare(s);           // :183-190
      const int e = nullcache ? INT32_MAX : next_event(s);
      if (e == s) {
#ifdef XCG_PHASES
        const uint64_t te0 = __builtin_amdgcn_s_memrealtime();
        ++ph_nev;
        struct PhEv {
          uint64_t t0; uint64_t& acc;
          __device__ ~PhEv() { acc += __builtin_amdgcn_s_memrealtime() - t0; }
        } ph_guard{te0, ph_ev};
#endif
        // Exact re-check of the probe (find_reference, :374-416).  A record
        // still missing its hi gets it from the same (single) hash call site,
        // then the window is hashed again.
        uint32_t lo = 0, hi = 0;
        int d = -1, fill = -1;
        uint3 hh;
        for (;;) {
          if (fill < 0 && ((s - p) & 31) == 0 && s - p < SEG) {   // a lane's first window: the hash from registers
            hh.x = 0u - readlane(k0, (s - p) >> 5);
            hh.y = readfirst(lane_window_hi(P, (s - p) >> 5));
            hh.z = DM ? readlane(NX2, (s - p) >> 5) : 0u;
          } else {
            hh = window_hash_u(fill >= 0 ? x + readfirst(T.rc[fill]) : x + s);
          }
          if (fill >= 0) {
            if (l == 0) T.rhi[fill] = hh.y;
            __builtin_amdgcn_wave_barrier();
            fill = -1;
            continue;
          }
          lo = hh.x; hi = hh.y;
          d = lookup(lo, hi);
          if (d >= -1) break;
          fill = -2 - d;
        }
        // Where the hash is declared: this chunk (d), the persistent cache, or
        // an earlier chunk of the batch.  src = that segment's bytes.
        const uint8_t* src = d >= 0 ? x + readfirst(T.rc[d]) : nullptr;
        if (LRU && d >= 0) record(lo, hi, 2u * (uint32_t)s + 1u, EV_HIT, 0u);
        // (through the lane filter first: the forced events of a chunk's last
        // one or two windows and own-table false positives have not passed it)
        if (STREAM && src == nullptr && glb_pass(probe_key(lo))) src = cache_src(lo, hi, s);
        if (src != nullptr) {
          if (s == p ? equal2048_regs(src, P.a0, P.a1) : equal2048_u(src, x + s)) {
            if (spec_cand >= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // speculative body lands first
            if (s > base) olen += escape_u(out + olen, x, (uint32_t)base, (uint32_t)s);
            wave_put_ref(out + olen, lo, hi);                 // encode_reference :342-372
            olen += 10;
            ref_made();
            ++n_ref;
            base = s + SEG;
            s = base;
            have_cand = false;                                // :208
            c0_in_table = true;
            chain = true;
            continue;
          }
          ++n_coll;                                           // collision, :390-406 / :215-216
          ++s;
          continue;
        }
        // fingerprint false positive: an ordinary miss
        if (!have_cand) {
          have_cand = true; cand = s; cand_lo = lo; cand_hi = hi; cand_k = hh.z; c0_in_table = false;
        }
        ++s;
        continue;
      }
      if (!have_cand) {                                       // :246-248
        hash_at(s, cand_lo, cand_hi, cand_k);
        have_cand = true;
        cand = s;
        c0_in_table = false;
        if (s == p && base == s && !oob) {
          // Declaration body = bytes [p, p + 2048) = the A registers.
          uint8_t* dst = out + olen + 2 + 32 * lane_id();
#if defined(XCG_EXP_ALIGNSTORE)   // (timing experiments only: output is wrong)
          dst = out + ((olen + 2) & ~15u) + 32 * lane_id();
#endif
#ifndef XCG_EXP_NOSTORE
          *(u32x4_u*)dst = P.a0;
          *(u32x4_u*)(dst + 16) = P.a1;
#endif
          spec_cand = s;
          spec_olen = olen;
        }
        ++s;
        continue;
      }
      // Non-event positions before the next milestone change nothing.
      s = min(min(e, cand + SEG), pe);
    }
    // The table holds every declaration once the piece is done; a still
    // pending candidate stays out of it until declared.
    totXA = totXB; totTA = totTB;
  }

  if (!spliced) {
    if (have_cand) declare(last + 1);                         // :257-261 (after every lookup)
    if (base < L) olen += escape_u(out + olen, x, (uint32_t)base, (uint32_t)L);   // :267-269
  }
  if (STREAM) {
    // This round's declarations; flag a change against the previous round's.
    const uint32_t nold = prm.ndecl[chunk];
    bool diff = nold != ndecl;
    uint4* dl = prm.decl + (uint64_t)chunk * prm.maxd;
    for (uint32_t k = l; k < ndecl; k += 64) {
      const uint4 nv = make_uint4(T.rlo[k], T.rhi[k], T.rc[k], gs.ro ? gs.ro[k] : 0u);
      if (k < nold) {
        const uint4 ov = dl[k];
        diff |= ov.x != nv.x || ov.y != nv.y || ov.z != nv.z;
      }
      dl[k] = nv;
    }
    if (ballot(diff) != 0 && l == 0) atomicMin(prm.changed, chunk);
    if (l == 0) {
      prm.ndecl[chunk] = ndecl;
      prm.nhits[chunk] = own_ovf ? prm.maxh + 1u : nh;
      if (LRU) prm.nev[chunk] = ne;
    }
  }
  if (l == 0) {
    prm.out_len[chunk] = olen;
    if (prm.stats) {
#if defined(XCG_PHASES)
      // diagnostics build: {vector phase, REF-chaining probes, whole chunk} (100 MHz ticks), pieces
      prm.stats[4 * chunk + 0] = (uint32_t)ph_vec;
      prm.stats[4 * chunk + 1] = (uint32_t)(XCG_PHASES_SLOT1 == 2 ? ph_wait : XCG_PHASES_SLOT1 ? ph_setup : ph_ev);
      prm.stats[4 * chunk + 2] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_start);
      prm.stats[4 * chunk + 3] = (ph_nev << 16) | n_pieces;
      (void)ph_chain; (void)ph_setup; (void)ph_ev; (void)ph_wait;
      (void)n_extract; (void)n_ref; (void)n_coll;
#elif defined(XCG_TIMING)
      // diagnostics build: {start, end} (100 MHz realtime, low words), HW_ID, XCC_ID
      const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
      prm.stats[4 * chunk + 0] = (uint32_t)t_start;
      prm.stats[4 * chunk + 1] = (uint32_t)t_end;
      prm.stats[4 * chunk + 2] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
      prm.stats[4 * chunk + 3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));   // HW_REG_XCC_ID
      (void)n_extract; (void)n_ref; (void)n_coll; (void)n_pieces;
#else
      prm.stats[4 * chunk + 0] = n_extract;
      prm.stats[4 * chunk + 1] = n_ref;
      prm.stats[4 * chunk + 2] = n_coll;
      prm.stats[4 * chunk + 3] = n_pieces;
#endif
    }
  }
}


#ifndef XCG_INDEP_OCC
#define XCG_INDEP_OCC 4
#endif
#ifndef XCG_INDEP_LOGNB
#define XCG_INDEP_LOGNB 10
#endif
#ifndef XCG_INDEP_W
#define XCG_INDEP_W 4         // chunk-waves per workgroup
#endif
template <int LOGNB, int MAXD>
__global__ __launch_bounds__(64 * XCG_INDEP_W, XCG_INDEP_OCC) void encode_independent_kernel(EncParams prm) {
  __shared__ IndepLDS<LOGNB, MAXD, XCG_INDEP_W> S;
  const int wv = (int)readfirst(threadIdx.x >> 6);   // wave-uniform: keeps the parse state in SGPRs
  const uint32_t chunk = blockIdx.x * (uint32_t)XCG_INDEP_W + (uint32_t)wv;
  if (chunk >= prm.n) return;
  encode_chunk<LOGNB, MAXD, false>(prm, (char*)S.key, (uint32_t)wv << (LOGNB + 3), S.rec[wv], chunk,
                                   GlbView{nullptr, 0u, 0u, 0, nullptr, nullptr});
}

// Stream semantics: persistent workgroups of SW waves share one LDS copy of
// the lane filter; each wave walks chunks wave_id, wave_id + total_waves, ...
template <int LOGNB, int MAXD, int SW, bool LRU>
__global__ __launch_bounds__(64 * SW) void encode_stream_kernel(EncParams prm) {
  using L = StreamLDS<LOGNB, MAXD, SW>;
  __shared__ L S;
  // Which lane filter the cache + batch declarations fit: the 64 KiB LDS one
  // up to LDS_FILTER_KEYS keys (FP <~10 %), else the global one.
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t stride = gridDim.x * SW;
  const uint32_t items = prm.work ? readfirst(prm.work[0]) : prm.n;
  // Prefix slices of the round's LDS filter (xcg_cache.h PREFIX_FILTERS): the
  // slice that covers the workgroup's highest chunk holds every batch key its
  // chunks can see.  (The cache's and the batch's key counts pick the mode.)
  uint32_t slice = 0, bkeys = prm.use_b ? readfirst(wave_sum(prm.bcount[lane_id()])) : 0u;
  if (prm.lf.pfdiv) {
    uint32_t cmax = 0;
    for (uint32_t i = blockIdx.x * SW + (uint32_t)wv; i < items; i += stride)
      cmax = max(cmax, prm.work ? readfirst(prm.work[1 + i]) : i);
    if (threadIdx.x == 0) S.cmax = 0u;
    __syncthreads();
    if (lane_id() == 0) atomicMax(&S.cmax, cmax);
    __syncthreads();
    slice = min(readfirst(S.cmax) / prm.lf.pfdiv, PREFIX_FILTERS - 1u);
    // (batch keys below the slice's end, taken as spread evenly over the chunks)
    const uint32_t cend = min(prm.n, (slice + 1u) * prm.lf.pfdiv);
    bkeys = (uint32_t)((uint64_t)bkeys * cend / max(prm.n, 1u));
  }
  const uint32_t keys = readfirst(*prm.nseg) + bkeys;
  const int fmode = keys == 0 ? 0 : (keys <= prm.lds_filter_keys ? 1 : (keys <= prm.lds_prefilter_keys ? 3 : 2));
  if (fmode == 1 || fmode == 3) {
    const u32x4* src = (const u32x4*)(prm.lf.filt + (uint64_t)slice * FILT_WORDS);
    for (uint32_t i = threadIdx.x; i < FILT_WORDS / 4; i += blockDim.x) ((u32x4*)S.lfilt)[i] = src[i];
  }
  __syncthreads();
  const GlbView gs{(char*)&S, (uint32_t)offsetof(L, lfilt),
                   (uint32_t)(offsetof(L, scr) + (size_t)wv * sizeof(S.scr[0])), fmode, S.ro[wv], S.rsv[wv]};
  // The batch's first chunk sees no batch declaration: on an empty cache it
  // probes nothing.  (The filter holds every chunk's keys; in a seeded round
  // of REF-dense data the first chunk's windows match thousands of later
  // chunks' tiles, each an exact lookup that finds nothing visible.)
  const bool g_empty = readfirst(*prm.nseg) == 0u;
  for (uint32_t i = blockIdx.x * SW + (uint32_t)wv; i < items; i += stride) {
    const uint32_t chunk = prm.work ? readfirst(prm.work[1 + i]) : i;
    if (chunk < prm.skip_below) continue;      // input unchanged since its last parse
    if (prm.need && readfirst(prm.need[chunk]) == 0u) continue;   // verified: its parse stands
    GlbView gv = gs;
    if (chunk == 0 && g_empty) gv.fmode = 0;
    encode_chunk<LOGNB, MAXD, true, LRU>(prm, (char*)S.key, (uint32_t)wv << (LOGNB + 3), S.rec[wv], chunk, gv);
  }
}

// ------------------------------------------------------------ quiet-chunk screen
//
// Small stream chunks (C4's 4 KiB packets: 2049 window positions each, a wave
// per packet, sixteen packets in turn per wave) spend their parse mostly in
// per-chunk round trips, and in hash-bound traffic (few repeats) almost every
// one of them ends as the cold parse: the 2048-byte tiling, with no lookup
// finding anything ("the cold parse of unique data is an exact
// 2048-aligned tiling").  That outcome is decided without the state machine:
// when no window of the chunk can be found -- in the persistent cache, among
// the batch's declarations, or among the chunk's own tiles declared before it
// (a tile at t is declared while examining window t + 2048, xcodec_encoder.cc:
// 183-190, so it is visible to the windows of every later piece) -- every lookup
// misses, and encode() declares exactly the tiles (:222-261) and escapes the
// tail (:267-269).
//
// stream_screen_kernel rolls every window of a chunk through the round's
// filters (a 128 KiB LDS fold of the global lane filter, then the global filter
// and the fingerprint buckets for what passes) and compares it with the
// chunk's earlier tiles; it writes the chunk's tiling output and stages its
// rows, with no dependent lookups, the next chunk's loads in flight meanwhile.
// screen_finish_kernel (a thread per chunk) checks each tile's own window
// exactly -- a tile is in the batch table as this chunk's own declaration;
// anything else there or in the persistent cache is a possible hit -- and
// either commits the staged rows and counters or puts the chunk on the work
// list encode_stream_kernel parses as always (any possible hit, an unaligned
// start, more than SCREEN_MAXD tiles).  Either way the output is the
// sequential encoder's: the screen only skips parses whose every lookup misses.
constexpr int SCREEN_MAXD = 4;                       // chunks shorter than 4 tiles (< 8 KiB)
constexpr uint32_t SCREEN_FOLD_WORDS = 32768;        // 128 KiB of LDS
constexpr int SCREEN_W = 12;                         // waves per workgroup (one workgroup per CU; 16: 3 % slower)
constexpr uint32_t SCR_NEEDY = 1u << 31, SCR_SKIP = 1u << 30;   // s_info flags
__device__ __forceinline__ uint32_t fold_word_of(uint32_t k, uint32_t fwm) { return (k >> 10) & fwm; }

// The LDS fold of the global lane filter: word j of the fold = OR of the global
// words j, j + F, j + 2F, ... (gfilt_word = K bits 10..; the fold keeps the
// low bits of that index), so a key's two bits are set in the fold whenever
// they are in its global word: no false negatives.
__global__ __launch_bounds__(256) void screen_fold_kernel(const uint32_t* gf, uint32_t gwords, uint32_t* fold,
                                                          uint32_t fwords) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= fwords) return;
  uint32_t w = 0;
  for (uint32_t j = i; j < gwords; j += fwords) w |= gf[j];
  fold[i] = w;
}

// What the screen stages: per chunk s_info = flags | tiles << 16 | output
// length, its tiles' rows (lo, hi, position, output length after it), and the
// keys of its windows that passed the LDS fold (qcnt of them), for the probe.
constexpr uint32_t SCREEN_QCAP = 1024;               // fold passes kept per chunk (more: the parse)
struct ScreenStage {
  uint32_t* info;      // [n]
  uint4* rows;         // [n * SCREEN_MAXD]
  uint32_t* qcnt;      // [n]
  uint32_t* qkeys;     // [n * SCREEN_QCAP]
};

// What the screen reads (a slim copy of EncParams: kernel arguments live in
// SGPRs, and the screen needs few of them).
struct ScreenParams {
  const uint8_t* in;
  const uint64_t* chunk_off;
  const uint32_t* chunk_len;
  const uint64_t* out_off;
  uint8_t* out;
  const uint4* decl;
  const uint32_t* ndecl;
  uint32_t* changed;
  const uint32_t* need;
  uint32_t n, skip_below, max_len, maxd;
};

// The lanes' chunk metadata for chunks base + k * stride (lane k).
struct ScreenMeta {
  uint64_t off, oo;
  uint32_t len, nold, go;
};

__device__ __forceinline__ ScreenMeta screen_meta(const ScreenParams& prm, uint32_t ck) {
  ScreenMeta m{0ull, 0ull, 0u, 0u, 0u};
  if (ck < prm.n && ck >= prm.skip_below && (!prm.need || prm.need[ck] != 0u)) {
    m.go = 1u;
    m.off = prm.chunk_off[ck];
    m.oo = prm.out_off[ck];
    m.len = prm.chunk_len[ck];
    m.nold = prm.ndecl[ck];
  }
  return m;
}

// Where a chunk is (wave-uniform, read from the lanes that loaded it: no
// memory wait inside the chunk loop), its first piece's A and B halves and
// its old rows (lane i: row i), all loaded while the chunk before it rolls.
struct ScreenLoad {
  uint64_t off, oo;    // input offset, output offset
  int L;
  uint32_t nold;       // its rows of the last round
  bool go;             // screened (not skipped by the round)
  u32x4 a0, a1, b0, b1;
  uint4 ov;
};

__device__ __forceinline__ bool screen_shape(int L, uint64_t off, const uint8_t* in) {
  return L >= SEG && !(L & (SEG - 1)) && L / SEG < SCREEN_MAXD && !(off & 15u) && !((uintptr_t)in & 15u);
}

__device__ __forceinline__ void screen_issue(const ScreenParams& prm, const ScreenMeta& m, int k, uint32_t chunk,
                                             ScreenLoad& s) {
  const int l = lane_id();
  s.go = readlane(m.go, k) != 0u;
  s.off = readlane64(m.off, k);
  s.oo = readlane64(m.oo, k);
  s.L = (int)readlane(m.len, k);
  s.nold = readlane(m.nold, k);
  s.a0 = s.a1 = s.b0 = s.b1 = u32x4{0u, 0u, 0u, 0u};
  s.ov = make_uint4(0u, 0u, 0u, 0u);
  if (!s.go || !screen_shape(s.L, s.off, prm.in)) return;
  const uint8_t* x = prm.in + s.off;
  const int q0 = 32 * l;
  s.a0 = load16_stream(x + q0);
  s.a1 = load16_stream(x + q0 + 16);
  if (s.L > SEG + 1) {
    s.b0 = load16_stream(x + q0 + SEG);
    s.b1 = load16_stream(x + q0 + SEG + 16);
  }
  if ((uint32_t)l < s.nold && l < SCREEN_MAXD) s.ov = prm.decl[(uint64_t)chunk * prm.maxd + l];
}

// Pass 1 of one chunk whose loads `cur` issued: every window rolled through
// the LDS fold; the passes queued for the probe, the tiling written, the rows
// staged.  No memory wait but the loads `cur` made (the next chunk's go out
// here).
__device__ __forceinline__ void screen_chunk(const ScreenParams& prm, const uint32_t* F, uint32_t fwm, uint32_t chunk,
                                             const ScreenLoad& cur, ScreenStage st, ScreenLoad& nxt,
                                             const ScreenMeta& meta, int knext, uint32_t next_chunk) {
  const int l = lane_id();
  const int L = cur.L;
  const uint8_t* x = prm.in + cur.off;
  uint8_t* const out = prm.out + cur.oo;
  const uint4 ov = cur.ov;
  Piece P;
  P.a0 = cur.a0; P.a1 = cur.a1; P.b0 = cur.b0; P.b1 = cur.b1;
  if (knext < 64) screen_issue(prm, meta, knext, next_chunk, nxt);
  else nxt.go = false;
  auto verdict = [&](uint32_t v) {
    if (l == 0) st.info[chunk] = v;
  };
  // Longer than the launch's bound, shorter than a window (only an escape,
  // xcodec_encoder.cc:77-83), a tail after the tiles (escaped by the parse),
  // or an unaligned start (pieces = tiles needs an aligned one): the parse.
  if ((uint32_t)L > prm.max_len || L / SEG >= (int)prm.maxd || !screen_shape(L, cur.off, prm.in)) {
    verdict(SCR_NEEDY);
    return;
  }
  const uint32_t nold = cur.nold;
  const int last = L - SEG;                        // last window start
  const int nt = L / SEG;                          // tiles = pieces
  uint32_t tlo[SCREEN_MAXD] = {0u, 0u, 0u, 0u}, thi[SCREEN_MAXD] = {0u, 0u, 0u, 0u};
  uint32_t tk[SCREEN_MAXD] = {0u, 0u, 0u, 0u};
  P.sxb = 0u; P.sqxb = 0u;
  uint32_t totXA = 0, totTA = 0;
  uint32_t qn = 0;                                 // passes queued so far
  uint32_t* const q = st.qkeys + (uint64_t)chunk * SCREEN_QCAP;
  bool needy = false;
  // the old rows are the tiling (the seeded round): their hi halves stand
  const bool rows_tiling = nold == (uint32_t)nt;
#pragma unroll 1
  for (int i = 0; i < nt && !needy; ++i) {
    const int p = SEG * i;
    const int q0 = p + 32 * l;
    const int pe = min(p + SEG, last + 1);         // piece end (exclusive)
    const bool one = pe - p == 1;                  // (a chunk of 2048 k bytes ends with a one-window piece)
    if (i == 0) {
      seg_sums(P.a0, P.a1, P.sxa, P.sqxa);
    } else {
      P.a0 = P.b0; P.a1 = P.b1;
      P.sxa = P.sxb; P.sqxa = P.sqxb;
      if (!one) {
        P.b0 = load16_stream(x + q0 + SEG);
        P.b1 = load16_stream(x + q0 + SEG + 16);
      }
    }
    // start sums of the lane's first window (encode_chunk's piece setup); a
    // one-window piece needs only lane 0's, which are the carried totals
    uint32_t tki;
    uint32_t NX1 = 0, NX2 = 0, totXB = 0, totTB = 0;
    const uint32_t qa = 32u * (uint32_t)l;
    if (i == 0) {
      totXA = wave_sum(P.sxa);
      totTA = wave_sum(qa * P.sxa + P.sqxa);
    }
    if (one) {
      tki = (0u - totXA) * (1u << 20) + (0u - (2048u * totXA - totTA + CLO));
    } else {
      seg_sums(P.b0, P.b1, P.sxb, P.sqxb);
      const uint32_t qb = 2048u + qa;
      const uint32_t ta = qa * P.sxa + P.sqxa, tb = qb * P.sxb + P.sqxb;
      const uint32_t dx = P.sxb - P.sxa, dt = tb - ta;
      const uint32_t ix = wave_incl_scan(dx), it = wave_incl_scan(dt);
      const uint32_t X1 = totXA + ix - dx;
      const uint32_t TT = totTA + it - dt;
      const uint32_t X2c = (2048u + qa) * X1 - TT + CLO;
      totXB = totXA + readlane(ix, 63);
      totTB = totTA + readlane(it, 63) - 2048u * totXB;
      NX1 = 0u - X1;
      NX2 = 0u - X2c;
      tki = readfirst((NX1 << 20) + NX2);
    }
    // the tile at the piece start: its hash (the old row's hi when the row is
    // this tile), and its EXTRACT (encode_declaration :300-302; the body is
    // this piece's A half)
    const uint32_t oz = readlane(ov.z, i), ox = readlane(ov.x, i), oy = readlane(ov.y, i);
    const uint32_t thii = rows_tiling && oz == (uint32_t)p && ox == 0u - tki ? oy : readfirst(lane_window_hi(P, 0));
    bool own = false;
#pragma unroll
    for (int u = 0; u < SCREEN_MAXD; ++u) {
      if (u < i) own |= tki == tk[u];
      if (u == i) { tk[u] = tki; tlo[u] = 0u - tki; thi[u] = thii; }
    }
    {
      uint8_t* dst = out + (uint32_t)(2 + SEG) * (uint32_t)i;
      if (l < 2) dst[l] = (uint8_t)(l == 0 ? MAGIC : OP_EXTRACT);
      *(u32x4_u*)(dst + 2 + 32 * l) = P.a0;
      *(u32x4_u*)(dst + 2 + 32 * l + 16) = P.a1;
    }
    if (own) {                                     // the tile's own window = an earlier tile
      needy = true;
      break;
    }
    if (one) continue;
    // every other window of the piece: the round's filters, the earlier tiles
    const uint32_t xa[8] = {P.a0[0], P.a0[1], P.a0[2], P.a0[3], P.a1[0], P.a1[1], P.a1[2], P.a1[3]};
    const uint32_t xb[8] = {P.b0[0], P.b0[1], P.b0[2], P.b0[3], P.b1[0], P.b1[1], P.b1[2], P.b1[3]};
    // positions past the last window are not positions; the piece start is the
    // tile itself (checked exactly by the probe).  (A window past the last one
    // that equals an earlier tile only costs the screen this chunk.)
    const int nvalid = pe - q0;
    uint32_t vm = nvalid >= 32 ? 0xFFFFFFFFu : ((1u << (uint32_t)max(nvalid, 0)) - 1u);
    if (l == 0) vm &= ~1u;
    // own earlier tiles: only a full piece after the first has one (chunks are
    // 2, 4 or 6 KiB; the last piece of each is one window), tile 0
    const uint32_t ko = tk[0];
    const uint32_t fbm = fwm << 2;                 // fold byte offset = K bits 10.. as a word index
    const char* const Fb = (const char*)F;
    uint32_t kk[32];
    uint32_t pass = 0u;
    uint64_t ownl = 0;   // lanes with a window equal to an earlier tile (lane masks: no VGPRs)
    // groups of 4 positions, one group's LDS reads in flight while the next
    // group rolls (as roll_probe; the sched_barrier bounds what is hoisted)
    uint32_t fwc[4], fwn[4];
    auto roll4 = [&](int g, uint32_t (&fw)[4]) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = 4 * g + t;
        kk[j] = (NX1 << 20) + NX2;
        if (j < 31) {
          const uint32_t xo = byte_of(xa[j >> 2], j & 3);
          const uint32_t xn = byte_of(xb[j >> 2], j & 3);
          NX1 += xo - xn;
          NX2 += NX1 + (xo << 11);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) fw[t] = *(const uint32_t*)(Fb + ((kk[4 * g + t] >> 8) & fbm));
    };
    auto roll = [&](auto own_t) {
      constexpr bool OWN = decltype(own_t)::value;
      roll4(0, fwc);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        if (g < 7) roll4(g + 1, fwn);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = 4 * g + t;
          // gfilt_test as two bit extracts (v_bfe takes the offset mod 32)
          const uint32_t b = __builtin_amdgcn_ubfe(fwc[t], kk[j], 1u) & __builtin_amdgcn_ubfe(fwc[t], kk[j] >> 5, 1u);
          pass |= b << j;
          if (OWN) ownl |= lanes_eq(kk[j], ko);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (g < 7) {
#pragma unroll
          for (int t = 0; t < 4; ++t) fwc[t] = fwn[t];
        }
      }
    };
    if (i > 0) roll(std::integral_constant<bool, true>{});
    else roll(std::integral_constant<bool, false>{});
    pass &= vm;
    if (ownl) {
      needy = true;
      break;
    }
    // the fold's passes, queued for the probe (stores only: nothing waits)
    const uint32_t cnt = (uint32_t)__builtin_popcount(pass);
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t tot = readlane(incl, 63);
    if (qn + tot > SCREEN_QCAP) {
      needy = true;
      break;
    }
    uint32_t* const ql = q + qn + incl - cnt;
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if ((pass >> j) & 1u) ql[__builtin_popcount(pass & ((1u << j) - 1u))] = kk[j];
    qn += tot;
    totXA = totXB; totTA = totTB;
  }
  if (needy) {
    verdict(SCR_NEEDY);
    return;
  }
  // the cold parse: the tiles (written above), no tail
  const uint32_t olen = (uint32_t)(2 + SEG) * (uint32_t)nt;
  // its rows, staged; against the round's old ones (a change flagged now is
  // conservative: the chunk may still go to the parse)
  bool diff = nold != (uint32_t)nt;
  uint4 nv = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int u = 0; u < SCREEN_MAXD; ++u)
    if (l == u) nv = make_uint4(tlo[u], thi[u], (uint32_t)(SEG * u), (uint32_t)(2 + SEG) * (uint32_t)(u + 1));
  if (l < nt) {
    if ((uint32_t)l < nold) diff |= ov.x != nv.x || ov.y != nv.y || ov.z != nv.z;
    st.rows[(uint64_t)chunk * SCREEN_MAXD + l] = nv;
  }
  if (ballot(diff) != 0 && l == 0) atomicMin(prm.changed, chunk);
  if (l == 0) st.qcnt[chunk] = qn;
  verdict(((uint32_t)nt << 16) | olen);
}

// Pass 1: persistent workgroups of W waves over the chunks; a wave's
// chunks chunk0, chunk0 + stride, ... in groups of 64 whose metadata lane k
// holds.
template <int W>
__global__ __launch_bounds__(64 * W) void stream_screen_kernel(ScreenParams prm, const uint32_t* fold,
                                                               uint32_t fwords, ScreenStage st) {
  __shared__ uint32_t F[SCREEN_FOLD_WORDS];
  for (uint32_t i = threadIdx.x; i < fwords / 4; i += blockDim.x) ((u32x4*)F)[i] = ((const u32x4*)fold)[i];
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t stride = gridDim.x * W;
  __syncthreads();
  for (uint32_t base = blockIdx.x * W + (uint32_t)wv; base < prm.n; base += 64u * stride) {
    const ScreenMeta meta = screen_meta(prm, base + (uint32_t)lane_id() * stride);
    ScreenLoad cur, nxt;
    screen_issue(prm, meta, 0, base, cur);
    for (int k = 0; k < 64; ++k) {
      const uint32_t chunk = base + (uint32_t)k * stride;
      if (chunk >= prm.n) break;
      if (!cur.go) {
        if (lane_id() == 0) st.info[chunk] = SCR_SKIP;
        if (k + 1 < 64) screen_issue(prm, meta, k + 1, chunk + stride, nxt);
        else nxt.go = false;
      } else {
        screen_chunk(prm, F, fwords - 1u, chunk, cur, st, nxt, meta, k + 1, chunk + stride);
      }
      cur = nxt;
    }
  }
}

// Pass 2, a wave per chunk: the queued fold passes through the global lane
// filter and the fingerprint buckets, the tiles' own windows exactly (the
// persistent cache; the batch table, where a tile is this chunk's own
// declaration and anything else a possible hit); then either the staged rows
// and counters go in, or the chunk joins the work list (work[0] counts it).
__global__ __launch_bounds__(256) void screen_finish_kernel(EncParams prm, ScreenStage st, uint32_t* work) {
  const uint32_t c = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  const int l = lane_id();
  if (c >= prm.n) return;
  // One round trip for the verdict and what a screened chunk's check starts
  // from (the staged count and rows are read whatever the verdict; a skipped
  // or needy chunk ignores them).
  const uint32_t info0 = st.info[c];
  const uint32_t qn0 = st.qcnt[c];
  const uint4 r0 = l < SCREEN_MAXD ? st.rows[(uint64_t)c * SCREEN_MAXD + l] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t ns0 = *prm.nseg;
  const uint32_t info = readfirst(info0);
  if (info & SCR_SKIP) return;
  bool needy = (info & SCR_NEEDY) != 0u;
  const uint32_t nt = (info >> 16) & 0xFFu;
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  if (!needy) {
    const uint32_t qn = readfirst(qn0);
    const uint32_t* const q = st.qkeys + (uint64_t)c * SCREEN_QCAP;
    const bool tile = (uint32_t)l < nt;
    if (tile) r = r0;
    // the tiles' own windows: their first probe slots in the persistent cache
    // and the batch table load with the first keys (a second round trip, not
    // a chain of them after the keys')
    const uint64_t key = ((uint64_t)r.y << 32) | r.x;
    const bool gl = tile && readfirst(ns0) != 0u, bl = tile && prm.use_b;
    const uint32_t ig = tab_slot(r.x, r.y, prm.g.mask), ib = prm.use_b ? tab_slot(r.x, r.y, prm.b.mask) : 0u;
    uint64_t kg = EMPTY_KEY, vg = 0ull, kb = EMPTY_KEY, vb = 0ull;
    if (gl) { kg = prm.g.keys[ig]; vg = prm.g.vals[ig]; }
    if (bl) { kb = prm.b.keys[ib]; vb = prm.b.vals[ib]; }
    bool hit = false;
    // up to 8 keys per lane in flight: their filter words, then (rarely) buckets
    for (uint32_t j0 = 0; j0 < qn; j0 += 512) {
      uint32_t k[8], w[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t j = j0 + 64u * t + (uint32_t)l;
        k[t] = j < qn ? q[j] : 0u;
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t j = j0 + 64u * t + (uint32_t)l;
        w[t] = j < qn ? prm.lf.gfilt[gfilt_word(k[t], prm.lf.gmask)] : 0u;
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t j = j0 + 64u * t + (uint32_t)l;
        if (j < qn && gfilt_test(w[t], k[t])) hit |= ftab_match(prm.lf.ftab[fbucket(k[t], prm.lf.fmask)], k[t]);
      }
    }
    // (a tile is in the batch table as this chunk's own declaration; anything
    // else there or in the persistent cache is a possible hit)
    if (gl && (kg == key ? vg : (kg == EMPTY_KEY ? ~0ull : tab_probe_rest_t(prm.g, key, ig))) != ~0ull) hit = true;
    if (bl) {
      const uint64_t bv = kb == key ? vb : (kb == EMPTY_KEY ? ~0ull : tab_probe_rest_t(prm.b, key, ib));
      if (bv != ~0ull && ((uint32_t)(bv >> 32) < c || ((uint32_t)(bv >> 32) == c && (uint32_t)bv != r.z))) hit = true;
    }
    needy = ballot(hit) != 0;
  }
  if (needy) {
    if (l == 0) work[1 + atomicAdd(work, 1u)] = c;
    return;
  }
  if ((uint32_t)l < nt) prm.decl[(uint64_t)c * prm.maxd + l] = r;
  if (l == 0) {
    prm.ndecl[c] = nt;
    prm.nhits[c] = 0u;
    prm.out_len[c] = info & 0xFFFFu;
    if (prm.stats) {
      prm.stats[4 * c + 0] = nt; prm.stats[4 * c + 1] = 0u;
      prm.stats[4 * c + 2] = 0u; prm.stats[4 * c + 3] = nt;
    }
  }
}

template __global__ void encode_independent_kernel<XCG_INDEP_LOGNB, 72>(EncParams);
template __global__ void encode_independent_kernel<11, 264>(EncParams);
template __global__ void encode_stream_kernel<8, 72, 16, false>(EncParams);
template __global__ void encode_stream_kernel<8, 72, 8, false>(EncParams);
template __global__ void encode_stream_kernel<8, 72, 4, false>(EncParams);
template __global__ void encode_stream_kernel<10, 264, 6, false>(EncParams);
template __global__ void encode_stream_kernel<10, 264, 2, false>(EncParams);
template __global__ void encode_stream_kernel<8, 72, 16, true>(EncParams);
template __global__ void encode_stream_kernel<8, 72, 8, true>(EncParams);
template __global__ void encode_stream_kernel<8, 72, 4, true>(EncParams);
template __global__ void encode_stream_kernel<10, 264, 6, true>(EncParams);
template __global__ void encode_stream_kernel<10, 264, 2, true>(EncParams);

}  // namespace xcg

extern "C" int xcg_launch_encode_independent(const uint8_t* d_in, const uint64_t* d_chunk_off,
                                             const uint32_t* d_chunk_len, uint32_t n, uint32_t max_chunk_len,
                                             uint32_t flags, uint8_t* d_out, const uint64_t* d_out_off,
                                             uint64_t* d_out_len, uint32_t* d_stats, int32_t* d_status,
                                             hipStream_t stream) {
  if (n == 0) return 0;
  xcg::EncParams prm{d_in, d_chunk_off, d_chunk_len, n, flags, d_out, d_out_off, d_out_len, d_stats, d_status};
  prm.max_len = max_chunk_len;
  dim3 grid((n + XCG_INDEP_W - 1) / XCG_INDEP_W), block(64 * XCG_INDEP_W);
  if (max_chunk_len <= (1u << 17)) {
    hipLaunchKernelGGL((xcg::encode_independent_kernel<XCG_INDEP_LOGNB, 72>), grid, block, 0, stream, prm);
  } else if (max_chunk_len <= (1u << 19)) {
    hipLaunchKernelGGL((xcg::encode_independent_kernel<11, 264>), grid, block, 0, stream, prm);
  } else {
    return -22;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ------------------------------------------------------------ stream rounds

namespace xcg {

// B <- every declaration of this round (earliest chunk wins per hash), and the
// round's lane filter = the persistent cache's filter + B.  One thread per
// (chunk, declaration).
constexpr uint32_t PREP_TABLE = 1, PREP_FILTERS = 2;   // (what a round's prep / build covers)

// The round's LDS-filter slices (xcg_cache.h PREFIX_FILTERS): a batch key of
// chunk c goes into slice c / pfdiv, then every slice is ORed into the ones
// above it, so slice j = the cache + the keys of chunks < (j + 1) pfdiv.
__device__ __forceinline__ FiltSet prefix_slice(FiltSet f, uint32_t c, uint32_t pfdiv) {
  if (pfdiv) f.filt += (uint64_t)min(c / pfdiv, PREFIX_FILTERS - 1u) * FILT_WORDS;
  return f;
}
__global__ __launch_bounds__(256) void filt_prefix_kernel(uint32_t* f) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  uint32_t w = 0;
#pragma unroll
  for (uint32_t j = 0; j < PREFIX_FILTERS; ++j) {
    w |= f[(uint64_t)j * FILT_WORDS + i];
    f[(uint64_t)j * FILT_WORDS + i] = w;
  }
}

// what: PREP_TABLE (the table and the counters), PREP_FILTERS, or both.  A
// verification builds the table alone: the filters of its declarations are
// only needed if a re-parse follows (then a filters-only pass adds them).
__global__ __launch_bounds__(256) void build_batch_table_kernel(const uint4* decl, const uint32_t* ndecl, uint32_t n,
                                                                uint32_t maxd, HashTab b, FiltSet fs, uint32_t* bcount,
                                                                int32_t* status, uint32_t what, uint32_t pfdiv) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (uint32_t)(i / maxd), k = (uint32_t)(i % maxd);
  const bool have = c < n && k < ndecl[c];
  const uint64_t m = ballot(have);
  if ((what & PREP_TABLE) && lane_id() == 0 && m) atomicAdd(bcount + ((i >> 6) & 63u), (uint32_t)__builtin_popcountll(m));
  if (!have) return;
  const uint4 d = decl[i];
  if (what == (PREP_TABLE | PREP_FILTERS)) {
    if (!tab_insert_min_filt(b, prefix_slice(fs, c, pfdiv), d.x, d.y, ((uint64_t)c << 32) | d.z)) atomicOr(status, 2);
  } else if (what == PREP_TABLE) {
    if (!tab_insert_min(b, d.x, d.y, ((uint64_t)c << 32) | d.z)) atomicOr(status, 2);
  } else {
    filt_insert(prefix_slice(fs, c, pfdiv), d.x, d.y);
  }
}

// Restart backup (before a re-parse round that may resume chunks from their
// rows): every flagged chunk with a contradicted-lookup time gets a backup
// slot (while slots last) holding its previous pass's reference rows, REF
// output lengths, batch hits, counts and output bytes.  One workgroup per chunk.
__global__ __launch_bounds__(256) void restart_backup_kernel(uint32_t n, const uint32_t* need, const uint32_t* bad_t,
                                                             uint32_t* bslot, uint32_t* b_count, uint32_t slots,
                                                             const uint8_t* out, const uint64_t* out_off,
                                                             const uint64_t* out_len, uint8_t* b_out, uint64_t stride,
                                                             const uint4* ev, const uint32_t* eo, const uint32_t* nev,
                                                             uint32_t maxe, const uint64_t* hits, const uint32_t* nhits,
                                                             uint32_t maxh, const uint32_t* ndecl, uint4* b_ev,
                                                             uint32_t* b_eo, uint64_t* b_hits, uint32_t* b_cnt) {
  __shared__ uint32_t sk;
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  if (c >= n) return;
  if (t == 0) {
    uint32_t k = ~0u;
    // (overflowed rows are incomplete: such a chunk re-parses from the start,
    // like one flagged with bad_t 0 or ~0)
    if (need[c] && bad_t[c] != ~0u && bad_t[c] != 0u && nev[c] <= maxe && nhits[c] <= maxh) {
      const uint32_t j = atomicAdd(b_count, 1u);
      if (j < slots) {
        k = j;
        atomicAdd(b_count + 2, 1u);                  // (cumulative: chunks resumed from their rows)
      }
    }
    bslot[c] = k;
    sk = k;
  }
  __syncthreads();
  const uint32_t k = sk;
  if (k == ~0u) return;
  const uint32_t ne = nev[c], nh = nhits[c];
  const uint64_t ol = out_len[c];
  if (t == 0) {
    b_cnt[4 * k] = ne;
    b_cnt[4 * k + 1] = nh;
    b_cnt[4 * k + 2] = (uint32_t)ol;
    b_cnt[4 * k + 3] = ndecl[c];
  }
  for (uint32_t i = t; i < ne; i += 256) {
    b_ev[(uint64_t)k * maxe + i] = ev[(uint64_t)c * maxe + i];
    b_eo[(uint64_t)k * maxe + i] = eo[(uint64_t)c * maxe + i];
  }
  for (uint32_t i = t; i < nh; i += 256) b_hits[(uint64_t)k * maxh + i] = hits[(uint64_t)c * maxh + i];
  const uint8_t* src = out + out_off[c];
  uint8_t* dst = b_out + (uint64_t)k * stride;
  for (uint64_t i = 16ull * t; i < ol; i += 16ull * 256) {
    if (i + 16 <= ol) *(u32x4_u*)(dst + i) = *(const u32x4_u*)(src + i);
    else for (uint64_t j = i; j < ol; ++j) dst[j] = src[j];
  }
}

// After that round: the old output tail of every spliced chunk (its previous
// pass's bytes from the rejoin point on) to its place behind the new part.
__global__ __launch_bounds__(256) void restart_splice_kernel(uint32_t n, uint4* splice, const uint32_t* bslot,
                                                             const uint8_t* b_out, uint64_t stride, uint8_t* out,
                                                             const uint64_t* out_off, uint32_t* b_count) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  if (c >= n) return;
  const uint4 sp = splice[c];
  if (sp.w == 0u) return;
  if (t == 0) atomicAdd(b_count + 3, 1u);          // (cumulative: chunks that rejoined their old parse)
  const uint8_t* src = b_out + (uint64_t)bslot[c] * stride + sp.y;
  uint8_t* dst = out + out_off[c] + sp.x;
  const uint64_t len = sp.z - sp.y;
  for (uint64_t i = 16ull * t; i < len; i += 16ull * 256) {
    if (i + 16 <= len) *(u32x4_u*)(dst + i) = *(const u32x4_u*)(src + i);
    else for (uint64_t j = i; j < len; ++j) dst[j] = src[j];
  }
  __syncthreads();
  if (t == 0) splice[c].w = 0u;
}

// Seed for the rounds instead of round 0: a chunk's cold parse (nothing
// cached, no repeat inside the chunk) declares exactly the 2048-byte tiling
// 0, 2048, ... ("the cold parse of unique data is an exact
// 2048-aligned tiling").  Round 1 then parses every chunk against the
// tiling of the chunks before it; the verification flags every chunk the
// guess misled, so the result is exact whatever the data.  One wave per
// (chunk, tile): a hash pass over the batch instead of a full parse.
// SEED_TILES tiles per wave (several waves per chunk): all of a wave's loads
// are in flight together, and the batch's ~32 k waves hide HBM latency (one
// wave per chunk walking its tiles four at a time left each wave waiting).
constexpr uint32_t SEED_TILES = 8;
// With b.keys set, the kernel also builds round 1's batch table and filters
// from the tiles (what build_batch_table_kernel does from the lists): lane 0
// of each wave inserts its tiles' hashes as they are made, so the table's
// atomics overlap the other waves' hashing instead of a second pass.
__global__ __launch_bounds__(256) void seed_tiling_kernel(const uint8_t* in, const uint64_t* chunk_off,
                                                          const uint32_t* chunk_len, uint32_t n, uint32_t maxd,
                                                          uint4* decl, uint32_t* ndecl, uint32_t* nhits,
                                                          uint32_t* changed, HashTab b, FiltSet fs, uint32_t* bcount,
                                                          int32_t* status, uint32_t pfdiv) {
  const uint32_t wpc = (maxd + SEED_TILES - 1) / SEED_TILES;       // waves per chunk
  const uint32_t w = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  const uint32_t c = w / wpc, k0 = (w % wpc) * SEED_TILES;
  if (w == 0 && threadIdx.x == 0) *changed = ~0u;
  if (c >= n) return;
  const int l = lane_id();
  const uint32_t m = min(chunk_len[c] / SEG, maxd);    // (an over-long chunk is refused by the round)
  const uint8_t* x = in + chunk_off[c];
  if (l == 0 && k0 == 0) {
    ndecl[c] = m;
    nhits[c] = 0u;
  }
  if (k0 >= m) return;
  // lane l sums bytes [16 l, 16 l + 16) and [1024 + 16 l, ...) of each tile
  u32x4 v[SEED_TILES][2];
  uint32_t mlo = 0, mhi = 0;
#pragma unroll
  for (uint32_t t = 0; t < SEED_TILES; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      v[t][h] = k0 + t < m ? *(const u32x4_u*)(x + (uint64_t)(k0 + t) * SEG + 1024u * h + 16u * l)
                           : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t t = 0; t < SEED_TILES; ++t) {
    if (k0 + t >= m) break;
    // Per 16-byte group h (offset q0 = 1024 h + 16 l in the tile): plain and
    // k-weighted sums of the bytes (v_dot4) and of ffs = ffbl + 1 (ffbl of a
    // zero byte is -1, so ffs sums are the ffbl sums + 16 and + 0 + ... + 15);
    // then X2 = sum (2048 - q0) S - W per group, and the same for F.
    uint32_t X1 = 0, X2 = 0, F1 = 0, F2 = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t q0 = 1024u * h + 16u * l;
      uint32_t sx = 0, wx = 0;
      int sf = 0, wf = 0;
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const uint32_t d = v[t][h][w4];
        const uint32_t wts = (4u * w4) | ((4u * w4 + 1) << 8) | ((4u * w4 + 2) << 16) | ((4u * w4 + 3) << 24);
        sx = __builtin_amdgcn_udot4(d, 0x01010101u, sx, false);
        wx = __builtin_amdgcn_udot4(d, wts, wx, false);
        // the four bytes' ffbl (-1 for a zero byte) packed as signed bytes, then
        // summed plain and k-weighted by v_dot4_i32_i8 (8 VALU per word, not 12)
        auto fb = [d](int b) {   // (the compiler's ffbl reads the byte in place: v_ffbl_b32_sdwa)
          return (uint32_t)(__builtin_ffs((int)__builtin_amdgcn_ubfe(d, 8u * b, 8u)) - 1);
        };
        const uint32_t p = __builtin_amdgcn_perm(fb(1), fb(0), 0x0c0c0400u) |
                           __builtin_amdgcn_perm(fb(3), fb(2), 0x04000c0cu);
        sf = __builtin_amdgcn_sdot4((int)p, 0x01010101, sf, false);
        wf = __builtin_amdgcn_sdot4((int)p, (int)wts, wf, false);
      }
      sf += 16;
      wf += 120;
      X1 += sx; X2 += (2048u - q0) * sx - wx;
      F1 += sf; F2 += (2048u - q0) * sf - wf;
    }
    X1 = wave_sum(X1); X2 = wave_sum(X2); F1 = wave_sum(F1); F2 = wave_sum(F2);
    if ((uint32_t)l == t) {                        // lane t keeps tile t's hash
      mlo = (X1 << 20) + X2 + CLO;
      mhi = ((F1 << 16) + F2) << 4;
    }
  }
  // lanes 0 .. tiles-1: the declaration records and, with a table, its inserts
  // (all of the wave's tiles in one chain of round trips)
  const uint32_t tiles = min(SEED_TILES, m - k0);
  if ((uint32_t)l < tiles) {
    const uint32_t k = k0 + (uint32_t)l;
    decl[(uint64_t)c * maxd + k] = make_uint4(mlo, mhi, k * SEG, 0u);
    if (b.keys && !tab_insert_min_filt(b, prefix_slice(fs, c, pfdiv), mlo, mhi, ((uint64_t)c << 32) | (k * SEG)))
      atomicOr(status, 2);
  }
  if (b.keys && l == 0 && k0 == 0) atomicAdd(bcount + (c & 63u), m);   // (the chunk's count, once)
}

// Everything a round clears or copies before its batch table is built, in
// one launch (six separate memset / copy calls cost ~7 us each in launch
// gaps): the table, the round's filters (copies of the cache's, or zero while
// the cache is empty), the key counters, the changed word and, for a
// verification, the changed-hash table and its flags.
struct RoundPrep {
  HashTab tab;
  uint32_t* r_filt; const uint32_t* g_filt;
  u32x4* r_ftab; const u32x4* g_ftab; uint32_t ftab_n;      // 16-byte units
  uint32_t* r_gfilt; const uint32_t* g_gfilt; uint32_t gfilt_n;
  const uint32_t* nseg;
  uint32_t* bcount;
  uint32_t* changed;
  HashTab rt;           // keys == nullptr: not a verification round
  uint32_t* vflags;
  HashTab at;           // (keys == nullptr: no (a)-probe) newly visible hashes
  uint32_t* abits;
  uint32_t n;           // verification: need[0..n) cleared, bad_t / bad_hi (nullable) reset
  uint32_t* need;
  uint32_t* bad_t;
  uint32_t* bad_hi;
  uint32_t what;        // PREP_TABLE: the table, counters and verification state; PREP_FILTERS: the filters
};
__global__ __launch_bounds__(256) void round_prep_kernel(RoundPrep a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool g_empty = *a.nseg == 0u;
  if (a.what & PREP_FILTERS) {
    // slice 0 starts as the cache's filter, the others empty (filt_prefix_kernel
    // ORs each slice into the ones above it once the batch keys are in)
    for (uint64_t i = i0; i < (uint64_t)FILT_WORDS * PREFIX_FILTERS; i += stride)
      a.r_filt[i] = (g_empty || i >= FILT_WORDS) ? 0u : a.g_filt[i];
    for (uint64_t i = i0; i < a.ftab_n; i += stride) a.r_ftab[i] = g_empty ? u32x4{0u, 0u, 0u, 0u} : a.g_ftab[i];
    for (uint64_t i = i0; i < a.gfilt_n; i += stride) a.r_gfilt[i] = g_empty ? 0u : a.g_gfilt[i];
  }
  if (!(a.what & PREP_TABLE)) return;
  for (uint64_t i = i0; i <= a.tab.mask; i += stride) { a.tab.keys[i] = EMPTY_KEY; a.tab.vals[i] = ~0ull; }
  if (a.rt.keys)
    for (uint64_t i = i0; i <= a.rt.mask; i += stride) { a.rt.keys[i] = EMPTY_KEY; a.rt.vals[i] = ~0ull; }
  if (a.rt.keys && a.need)
    for (uint64_t i = i0; i < a.n; i += stride) {
      a.need[i] = 0u;
      if (a.bad_t) { a.bad_t[i] = ~0u; a.bad_hi[i] = 0u; }
    }
  if (a.rt.keys && a.at.keys) {
    for (uint64_t i = i0; i <= a.at.mask; i += stride) { a.at.keys[i] = EMPTY_KEY; a.at.vals[i] = ~0ull; }
    for (uint64_t i = i0; i < XCG_VERIFY_A_WORDS; i += stride) a.abits[i] = 0u;
  }
  if (i0 < 64) a.bcount[i0] = 0u;
  if (i0 == 0) {
    *a.changed = ~0u;
    if (a.rt.keys) { a.vflags[0] = ~0u; a.vflags[1] = 0u; a.vflags[3] = 0u; }
  }
}

// ------------------------------------------------ verification of a round
//
// Round r parsed chunk k against V = the batch table of round r-1's
// declarations; T = the table of round r's.  k's parse depends on the batch
// only through its lookups, so it stands under T unless, for some hash h,
// (a) h becomes visible to k (earliest declaring chunk c_T < k <= c_V: a miss
//     may turn into a hit) and one of k's windows has hash h
//     (verify_probe_kernel; with more than XCG_VERIFY_A_LIMIT such hashes,
//     conservatively every k > c_T); or
// (b) k found h in V (a recorded hit) and under T h is invisible to k, or its
//     earliest declaration has other bytes.
// The fixed point is reached when no chunk is flagged.
__device__ __forceinline__ bool v4_ne(u32x4 a, u32x4 b) { return a[0] != b[0] || a[1] != b[1] || a[2] != b[2] || a[3] != b[3]; }
__device__ __forceinline__ bool seg_equal_t(const uint8_t* a, const uint8_t* b) {   // one thread, 2048 bytes
  for (int i = 0; i < SEG; i += 16)
    if (v4_ne(*(const u32x4_u*)(a + i), *(const u32x4_u*)(b + i))) return false;
  return true;
}

// The newly visible hashes' blocked Bloom filter: one word, two bits.
__device__ __forceinline__ uint32_t abits_word(uint32_t lo, uint32_t hi) {
  return (lo ^ (hi >> 4)) & (XCG_VERIFY_A_WORDS - 1u);
}
__device__ __forceinline__ uint32_t abits_mask(uint32_t lo, uint32_t hi) {
  return (1u << ((lo >> 13) & 31u)) | (1u << ((hi >> 21) & 31u));
}

__global__ __launch_bounds__(256) void verify_diff_kernel(HashTab tv, HashTab tt, const uint8_t* in,
                                                          const uint64_t* chunk_off, HashTab rt, uint32_t* a_first,
                                                          HashTab at, uint32_t* abits, int32_t* status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)tt.mask + 1, nv = (uint64_t)tv.mask + 1;
  uint64_t h, vt, vv;
  if (i < nt) {
    h = tt.keys[i];
    if (h == EMPTY_KEY) return;
    vt = tt.vals[i];
    vv = tab_lookup_t(tv, (uint32_t)h, (uint32_t)(h >> 32));
  } else if (i < nt + nv) {
    h = tv.keys[i - nt];
    if (h == EMPTY_KEY) return;
    if (tab_lookup_t(tt, (uint32_t)h, (uint32_t)(h >> 32)) != ~0ull) return;   // seen from T's side
    vt = ~0ull;
    vv = tv.vals[i - nt];
  } else {
    return;
  }
  if (vt == vv) return;
  const uint32_t INF = 0xFFFFFFFFu;
  const uint32_t ct = vt == ~0ull ? INF : (uint32_t)(vt >> 32), cv = vv == ~0ull ? INF : (uint32_t)(vv >> 32);
  uint32_t rlo = INF, rhi = 0;
  if (ct < cv) {                                                             // (a)
    atomicMin(a_first, ct + 1);
    if (at.keys) {                  // chunks (ct, cv] newly see h (a_first[3]: how many such h)
      const uint32_t j = atomicAdd(a_first + 3, 1u);
      if (j < XCG_VERIFY_A_LIMIT) {
        const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
        if (!tab_insert_min(at, lo, hi, ((uint64_t)(ct + 1) << 32) | (cv == INF ? INF - 1 : cv)))
          atomicOr(a_first + 3, 0x80000000u);                                 // (conservative then)
        atomicOr(abits + abits_word(lo, hi), abits_mask(lo, hi));
      }
    }
  }
  bool same = false;
  if (vt != ~0ull && vv != ~0ull)
    same = seg_equal_t(in + chunk_off[ct] + (uint32_t)vt, in + chunk_off[cv] + (uint32_t)vv);
  // (b): chunks in (cv, ct] lose h; with other bytes, every chunk > min(cv, ct) that found h
  if (cv < ct) { rlo = min(rlo, cv + 1); rhi = max(rhi, ct == INF ? INF - 1 : ct); }
  if (!same && ct != INF && cv != INF) { rlo = min(rlo, min(ct, cv) + 1); rhi = INF - 1; }
  if (rlo <= rhi && !tab_insert_min(rt, (uint32_t)h, (uint32_t)(h >> 32), ((uint64_t)rlo << 32) | rhi))
    atomicOr(status, 2);
}

__global__ __launch_bounds__(256) void own_ovf_check_kernel(const uint32_t* nhits, uint32_t n, uint32_t maxh,
                                                            int32_t* status) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n && nhits[c] == maxh + 1u && status) atomicOr(status, 1);
}

// need[k] for every chunk: the conservative (a) (no probe, or too many newly
// visible hashes) or overflowed hit / reference lists -- such a chunk re-parses
// from its start (bad_t 0); then (a) by the probe and (b), which also give
// the times of the first and last affected lookup (bad_t / bad_hi, for the
// re-parse restart; ~0 / 0 until then).
__device__ __forceinline__ void verify_check_body(uint32_t bid, uint32_t n, const uint32_t* nhits, uint32_t maxh,
                                                  const uint32_t* nev, uint32_t maxe, bool probe,
                                                  const uint32_t* vflags, uint32_t* need, uint32_t* any,
                                                  uint32_t* bad_t, uint32_t* bad_hi) {
  const uint32_t k = bid * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const bool conservative = !probe || vflags[3] > XCG_VERIFY_A_LIMIT;
  const bool f = (k >= vflags[0] && conservative) || nhits[k] > maxh || (nev && nev[k] > maxe);
  if (f) {                                       // (need / bad_t / bad_hi start cleared: round_prep)
    need[k] = 1u;
    if (bad_t) {
      bad_t[k] = 0u;
      bad_hi[k] = ~1u;
    }
  }
  if (ballot(f) != 0 && lane_id() == 0) atomicOr(any, 1u);
}

// Flag chunk k with the in-chunk times [lo, hi] of affected lookups.
__device__ __forceinline__ void flag_chunk(uint32_t k, uint32_t lo, uint32_t hi, uint32_t* need, uint32_t* any,
                                           uint32_t* bad_t, uint32_t* bad_hi) {
  for (int off = 32; off >= 1; off >>= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, off));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, off));
  }
  if (lane_id() == 0 && lo != ~0u) {
    need[k] = 1u;
    atomicOr(any, 1u);
    if (bad_t) {
      atomicMin(bad_t + k, lo);
      atomicMax(bad_hi + k, hi);
    }
  }
}

// (a) exactly: every window of every chunk >= a_first, hashed like
// window_hashes_kernel (one wave per 2048 positions, 32 per lane), tested
// against the newly visible hashes' Bloom filter in LDS, then exactly; a
// window of chunk k whose hash became visible to k flags k at that window's
// lookup time 2 s + 1.  Blocks loop over the (chunk, span) items.
__device__ __forceinline__ void verify_probe_body(uint32_t bid, uint32_t nblk, uint32_t* sb, const uint8_t* in,
                                                  const uint64_t* chunk_off, const uint32_t* chunk_len, uint32_t n,
                                                  uint32_t spc, const uint32_t* vflags, HashTab at,
                                                  const uint32_t* abits, uint32_t* need, uint32_t* any,
                                                  uint32_t* bad_t, uint32_t* bad_hi) {
  const uint32_t a_first = vflags[0], acount = vflags[3];
  if (acount == 0u || acount > XCG_VERIFY_A_LIMIT || a_first >= n) return;
  for (uint32_t i = threadIdx.x; i < XCG_VERIFY_A_WORDS / 4; i += blockDim.x)
    ((u32x4*)sb)[i] = ((const u32x4*)abits)[i];
  __syncthreads();
  const int l = lane_id();
  const uint64_t items = (uint64_t)(n - a_first) * spc, nw = (uint64_t)nblk * 4u;
  for (uint64_t it = (uint64_t)bid * 4u + readfirst(threadIdx.x >> 6); it < items; it += nw) {
    const uint32_t k = a_first + (uint32_t)(it / spc);
    const int64_t len = chunk_len[k], npos = len - SEG + 1, p = (int64_t)(it % spc) * SEG;
    if (p >= npos) continue;
    const uint8_t* x = in + chunk_off[k];
    const int64_t q0 = p + 32 * l;
    const u32x4 a0 = load16_guarded(x, q0, len), a1 = load16_guarded(x, q0 + 16, len);
    const u32x4 b0 = load16_guarded(x, q0 + SEG, len), b1 = load16_guarded(x, q0 + SEG + 16, len);
    const uint32_t xa[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    const uint32_t xb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    uint32_t sxa = 0, sqxa = 0, sfa = 0, sqfa = 0, sxb = 0, sqxb = 0, sfb = 0, sqfb = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint32_t va = byte_of(xa[j >> 2], j & 3), vb = byte_of(xb[j >> 2], j & 3);
      const uint32_t fa = ffbl(va) + 1u, fb = ffbl(vb) + 1u;
      sxa += va; sqxa += j * va; sfa += fa; sqfa += j * fa;
      sxb += vb; sqxb += j * vb; sfb += fb; sqfb += j * fb;
    }
    const uint32_t qa = 32u * l, qb = 2048u + 32u * l;
    const uint32_t ta = qa * sxa + sqxa, tb = qb * sxb + sqxb;
    const uint32_t tfa = qa * sfa + sqfa, tfb = qb * sfb + sqfb;
    const uint32_t dx = sxb - sxa, dt = tb - ta, df = sfb - sfa, dtf = tfb - tfa;
    uint32_t X1 = wave_sum(sxa) + wave_incl_scan(dx) - dx;
    const uint32_t TT = wave_sum(ta) + wave_incl_scan(dt) - dt;
    uint32_t F1 = wave_sum(sfa) + wave_incl_scan(df) - df;
    const uint32_t TF = wave_sum(tfa) + wave_incl_scan(dtf) - dtf;
    uint32_t X2c = (2048u + qa) * X1 - TT + CLO;
    uint32_t F2 = (2048u + qa) * F1 - TF;
    uint32_t tlo = ~0u, thi = 0u;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int64_t s = q0 + j;
      const uint32_t lo = (X1 << 20) + X2c, hi = ((F1 << 16) + F2) << 4;
      const uint32_t w = sb[abits_word(lo, hi)], m = abits_mask(lo, hi);
      if (s < npos && (w & m) == m) {
        const uint64_t v = tab_lookup_t(at, lo, hi);
        if (v != ~0ull && k >= (uint32_t)(v >> 32) && k <= (uint32_t)v) {
          tlo = min(tlo, 2u * (uint32_t)s + 1u);
          thi = max(thi, 2u * (uint32_t)s + 1u);
        }
      }
      const uint32_t xo = byte_of(xa[j >> 2], j & 3), xn = byte_of(xb[j >> 2], j & 3);
      const uint32_t ro = ffbl(xo), rn = ffbl(xn);
      X1 = X1 + xn - xo;
      X2c = X2c + X1 - (xo << 11);
      F1 = F1 + rn - ro;
      F2 = F2 + F1 - (ro << 11) - 2048u;
    }
    flag_chunk(k, tlo, thi, need, any, bad_t, bad_hi);
  }
}

// (b) from the reference rows (bounded caches: batch hits carry their lookup
// times), one wave per chunk; the hit lists' verify_hits_kernel otherwise.
__device__ __forceinline__ void verify_hit_events_body(uint32_t bid, uint32_t n, const uint4* ev, const uint32_t* nev,
                                                       uint32_t maxe, HashTab rt, uint32_t* need, uint32_t* any,
                                                       uint32_t* bad_t, uint32_t* bad_hi) {
  const uint32_t k = bid * 4u + readfirst(threadIdx.x >> 6);
  if (k >= n) return;
  const uint32_t cnt = min(nev[k], maxe);
  uint32_t lo = ~0u, hi = 0u;
  for (uint32_t i = lane_id(); i < cnt; i += 64) {
    const uint4 e = ev[(uint64_t)k * maxe + i];
    if ((e.w >> 30) == EV_HIT && (e.w & EV_REF_MASK) == 1u) {
      const uint64_t r = tab_lookup_t(rt, e.x, e.y);
      if (r != ~0ull && k >= (uint32_t)(r >> 32) && k <= (uint32_t)r) { lo = min(lo, e.z); hi = max(hi, e.z); }
    }
  }
  flag_chunk(k, lo, hi, need, any, bad_t, bad_hi);
}
__device__ __forceinline__ void verify_hits_body(uint32_t bid, uint32_t n, const uint64_t* hits, const uint32_t* nhits,
                                                 uint32_t maxh, HashTab rt, uint32_t* need, uint32_t* any) {
  const uint64_t j = (uint64_t)bid * blockDim.x + threadIdx.x;
  const uint32_t k = (uint32_t)(j / maxh), i = (uint32_t)(j % maxh);
  bool f = false;
  if (k < n && i < nhits[k]) {
    const uint64_t h = hits[j];
    const uint64_t r = tab_lookup_t(rt, (uint32_t)h, (uint32_t)(h >> 32));
    f = r != ~0ull && k >= (uint32_t)(r >> 32) && k <= (uint32_t)r;
    if (f) need[k] = 1u;
  }
  if (ballot(f) != 0 && lane_id() == 0) atomicOr(any, 1u);
}

// The verification's flagging passes in one launch (they only set flags, so
// their order does not matter; round_prep cleared need / bad_t / bad_hi):
// blocks [0, bc) the per-chunk check (block 0 also sums the declaration
// counters into vflags[2]), [bc, bc + bp) the (a)-probe, the rest the (b)
// hit check -- four launches' gaps fewer per round.
struct VerifyFlags {
  uint32_t n, bc, bp, bh;
  const uint32_t* nhits; uint32_t maxh; const uint64_t* hits;
  const uint32_t* nev; uint32_t maxe; const uint4* ev;
  bool probe; uint32_t* vflags; uint32_t* need; uint32_t* bad_t; uint32_t* bad_hi;
  const uint8_t* in; const uint64_t* chunk_off; const uint32_t* chunk_len; uint32_t spc;
  HashTab at; const uint32_t* abits; HashTab rt; const uint32_t* bcount;
};
__global__ __launch_bounds__(256) void verify_flags_kernel(VerifyFlags v) {
  __shared__ uint32_t sb[XCG_VERIFY_A_WORDS];
  const uint32_t b = blockIdx.x;
  uint32_t* any = v.vflags + 1;
  if (b < v.bc) {
    if (b == 0 && threadIdx.x < 64) {
      const uint32_t t = wave_sum(v.bcount[lane_id()]);
      if (lane_id() == 0) v.vflags[2] = t;
    }
    verify_check_body(b, v.n, v.nhits, v.maxh, v.nev, v.maxe, v.probe, v.vflags, v.need, any, v.bad_t, v.bad_hi);
  } else if (b < v.bc + v.bp) {
    verify_probe_body(b - v.bc, v.bp, sb, v.in, v.chunk_off, v.chunk_len, v.n, v.spc, v.vflags, v.at, v.abits, v.need,
                      any, v.bad_t, v.bad_hi);
  } else if (v.ev) {
    verify_hit_events_body(b - v.bc - v.bp, v.n, v.ev, v.nev, v.maxe, v.rt, v.need, any, v.bad_t, v.bad_hi);
  } else {
    verify_hits_body(b - v.bc - v.bp, v.n, v.hits, v.nhits, v.maxh, v.rt, v.need, any);
  }
}

// Segment numbers of the committed declarations: seg_base[c] = nseg + the
// declarations of chunks < c (exclusive scan, one workgroup), and nseg
// advanced by the total -- no per-block atomic on one counter (16 k of those
// serialised to ~190 us for a batch of 4 KiB packets).
// gate (nullable): run only if *gate == 0 -- the commit is queued right
// behind a verification and does nothing if that verification flagged chunks.
__global__ __launch_bounds__(1024) void commit_scan_kernel(const uint32_t* ndecl, uint32_t n, uint32_t* seg_base,
                                                           uint32_t* nseg, const uint32_t* gate) {
  // tiles of 1024 x 8 counts: each thread loads its 8 consecutive counts as
  // two 16-byte loads (coalesced across the wave), the block scans the 1024
  // thread sums (wave scans + the 16 wave totals: two barriers a tile, where a
  // Hillis-Steele pass per 4096 counts took twenty -- 54 us at 65 k chunks)
  constexpr uint32_t PER = 8;
  __shared__ uint32_t wtot[16];
  const uint32_t t = threadIdx.x, wv = t >> 6;
  if (gate && *gate) return;
  uint32_t carry = *nseg;
  for (uint32_t base = 0; base < n; base += 1024 * PER) {
    const uint32_t i0 = base + PER * t;
    uint32_t v[PER];
    if (i0 + PER <= n) {
      const uint4 a0 = *(const uint4*)(ndecl + i0), a1 = *(const uint4*)(ndecl + i0 + 4);
      v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
    } else {
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k) v[k] = i0 + k < n ? ndecl[i0 + k] : 0u;
    }
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) sum += v[k];
    const uint32_t incl = wave_incl_scan(sum);
    if (lane_id() == 63) wtot[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) {
      const uint32_t x = wtot[q];
      before += q < wv ? x : 0u;
      total += x;
    }
    uint32_t o[PER];
    uint32_t run = carry + before + incl - sum;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      o[k] = run;
      run += v[k];
    }
    if (i0 + PER <= n) {
      *(uint4*)(seg_base + i0) = make_uint4(o[0], o[1], o[2], o[3]);
      *(uint4*)(seg_base + i0 + 4) = make_uint4(o[4], o[5], o[6], o[7]);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k)
        if (i0 + k < n) seg_base[i0 + k] = o[k];
    }
    carry += total;
    __syncthreads();                                   // (wtot is reused)
  }
  if (t == 0) *nseg = carry;
}

// Commit the converged declarations into the persistent cache
// (XCodecMemoryCache::enter, xcodec_cache.h:303-325).  Block (chunk c, part q)
// takes declarations q*256 .. q*256+255 of chunk c, whose segments are
// seg_base[c] + q*256 + j in declaration order.  Each wave first copies four
// 2048-byte segments at a time into the pool with all eight 16-byte loads per
// lane in flight together (the input offsets staged in LDS), then each thread
// inserts its declaration's hash.  The copy is issued
// before the inserts: on gfx9 an atomic's return waits on every older memory
// operation of the wave, so inserts first serialised each segment copy behind
// the insert chain (70 -> 44 us for C2-S2's ~66 k declarations).
__global__ __launch_bounds__(256) void commit_kernel(const uint4* decl, const uint32_t* ndecl, uint32_t n,
                                                     uint32_t maxd, const uint8_t* in, const uint64_t* chunk_off,
                                                     HashTab g, uint8_t* pool, const uint32_t* seg_base,
                                                     uint32_t seg_cap, FiltSet fs, int32_t* status,
                                                     const uint32_t* gate) {
  if (gate && *gate) return;
  const uint32_t parts = (maxd + 255) / 256;
  const uint32_t c = blockIdx.x / parts, k0 = (blockIdx.x % parts) * 256u;
  const uint32_t nd = c < n ? ndecl[c] : 0u;
  const uint32_t cnt = nd > k0 ? min(256u, nd - k0) : 0u;
  if (cnt == 0) return;                            // uniform over the block
  const uint32_t s_base = seg_base[c] + k0;
  const uint32_t k = k0 + threadIdx.x;
  const bool have = k < nd;
  __shared__ uint32_t zoff[256];                   // the declarations' input offsets
  uint4 d = make_uint4(0u, 0u, 0u, 0u);
  if (have) d = decl[(uint64_t)c * maxd + k];
  zoff[threadIdx.x] = d.z;
  __syncthreads();
  const int l = lane_id();
  const uint32_t wv = readfirst(threadIdx.x >> 6);
  const uint8_t* x = in + chunk_off[c];
  for (uint32_t j0 = 4u * wv; j0 < cnt; j0 += 16u) {
    u32x4 v[8];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      if (j0 + j < cnt) {
        const uint8_t* src = x + readfirst(zoff[j0 + j]);
        v[2 * j] = *(const u32x4_u*)(src + 32 * l);
        v[2 * j + 1] = *(const u32x4_u*)(src + 32 * l + 16);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t sg = s_base + j0 + j;
      if (j0 + j < cnt && sg < seg_cap) {
        uint8_t* dst = pool + (uint64_t)sg * SEG;
        *(u32x4_u*)(dst + 32 * l) = v[2 * j];
        *(u32x4_u*)(dst + 32 * l + 16) = v[2 * j + 1];
      }
    }
  }
  if (have) {
    const uint32_t seg = s_base + threadIdx.x;
    if (seg >= seg_cap) {
      atomicOr(status, 4);
    } else {
      if (!tab_insert_min_filt(g, fs, d.x, d.y, seg)) atomicOr(status, 2);
    }
  }
}

}  // namespace xcg



// LDS / global lane filter threshold (keys): XCG_LDS_FILTER_KEYS at load
// time, or xcg_debug_set_lds_filter_keys (tests force either mode with it).
// Default (LFK_AUTO): per cache -- LDS_FILTER_KEYS_DEFAULT while its fingerprint
// buckets fit 2 MiB of L2, else 0: with a larger bucket table (unbounded caches
// of 2^19+ segments, pairs) an LDS-filter pass costs fewer HBM misses as a
// probe of the L2-resident global filter than as a bucket load (C5 308 -> 316
// GiB/s; C2-S2 and the LRU cache, 2 MiB of buckets, lose with 0:
// profiles/r06_s3_lfk.txt).
constexpr uint32_t LFK_AUTO = ~0u;
static uint32_t g_lds_filter_keys = [] {
  const char* e = getenv("XCG_LDS_FILTER_KEYS");
  return e ? (uint32_t)strtoul(e, nullptr, 10) : LFK_AUTO;
}();
static uint32_t xcg_lds_filter_keys() { return __atomic_load_n(&g_lds_filter_keys, __ATOMIC_RELAXED); }
extern "C" uint32_t xcg_debug_set_lds_filter_keys(uint32_t keys) {
  return __atomic_exchange_n(&g_lds_filter_keys, keys, __ATOMIC_RELAXED);
}
// Past that, the LDS filter still screens the global one's loads up to this
// many keys (XCG_LDS_PREFILTER_KEYS, xcg_debug_set_lds_prefilter_keys).
static uint32_t g_lds_prefilter_keys = [] {
  const char* e = getenv("XCG_LDS_PREFILTER_KEYS");
  return e ? (uint32_t)strtoul(e, nullptr, 10) : xcg::LDS_PREFILTER_KEYS_DEFAULT;
}();
extern "C" uint32_t xcg_debug_set_lds_prefilter_keys(uint32_t keys) {
  return __atomic_exchange_n(&g_lds_prefilter_keys, keys, __ATOMIC_RELAXED);
}

// The tiling seed alone (decl / ndecl / nhits / changed), for a caller that
// looks at it before the rounds (the bounded cache's first eviction guess);
// then xcg_launch_encode_stream with keep_decls.
extern "C" int xcg_launch_seed_tiling(const XcgStreamArgs* a, hipStream_t stream) {
  if (a->n == 0) return 0;
  const uint32_t seed_waves = a->n * ((a->maxd + xcg::SEED_TILES - 1) / xcg::SEED_TILES);
  hipLaunchKernelGGL(xcg::seed_tiling_kernel, dim3((seed_waves + 3) / 4), dim3(256), 0, stream, a->in, a->chunk_off,
                     a->chunk_len, a->n, a->maxd, (uint4*)a->decl, a->ndecl, a->nhits, a->changed,
                     xcg::HashTab{nullptr, nullptr, 0u}, xcg::FiltSet{}, nullptr, nullptr, 0u);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The quiet-chunk screen on (default) / off: XCG_SCREEN=0, or
// xcg_debug_set_screen (tests run both ways).
static int g_screen = [] {
  const char* e = getenv("XCG_SCREEN");
  return e ? atoi(e) : 1;
}();
static bool xcg_screen_on() { return __atomic_load_n(&g_screen, __ATOMIC_RELAXED) != 0; }
// (2: on, and count what the screen sees -- a host sync per screened launch)
static bool xcg_screen_counting() { return __atomic_load_n(&g_screen, __ATOMIC_RELAXED) == 2; }
extern "C" int xcg_debug_set_screen(int mode) {
  return __atomic_exchange_n(&g_screen, mode < 0 ? 0 : (mode > 2 ? 2 : mode), __ATOMIC_RELAXED);
}
static uint64_t g_screen_seen = 0, g_screen_parsed = 0;
extern "C" int xcg_debug_screen_counts(uint64_t* seen, uint64_t* parsed) {
  if (seen) *seen = __atomic_exchange_n(&g_screen_seen, 0ull, __ATOMIC_RELAXED);
  if (parsed) *parsed = __atomic_exchange_n(&g_screen_parsed, 0ull, __ATOMIC_RELAXED);
  return 0;
}

static bool stream_debug() {
  static const bool on = getenv("XCG_STREAM_DEBUG") != nullptr;
  return on;
}

// Live timing of the stream-parse kernel for bench.py's roofline: while on,
// every encode_stream_kernel launch is bracketed by HIP events on its own
// launch stream; xcg_debug_stream_kernel_time sums them (process-wide).
namespace {
std::mutex g_ktime_mu;
bool g_ktime_on = false;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_ktime_ev;
}  // namespace
extern "C" int xcg_debug_stream_kernel_timing(int on) {
  std::lock_guard<std::mutex> g(g_ktime_mu);
  const int old = g_ktime_on;
  g_ktime_on = on != 0;
  return old;
}
extern "C" int xcg_debug_stream_kernel_time(double* ms, uint32_t* launches) {
  std::lock_guard<std::mutex> g(g_ktime_mu);
  double tot = 0;
  int rc = 0;
  for (auto& e : g_ktime_ev) {
    float t = 0;
    if (hipEventSynchronize(e.second) != hipSuccess || hipEventElapsedTime(&t, e.first, e.second) != hipSuccess)
      rc = -5;
    tot += t;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (ms) *ms = tot;
  if (launches) *launches = (uint32_t)g_ktime_ev.size();
  g_ktime_ev.clear();
  return rc;
}
static hipEvent_t ktime_begin(hipStream_t s) {
  std::lock_guard<std::mutex> g(g_ktime_mu);
  hipEvent_t e = nullptr;
  if (!g_ktime_on || hipEventCreate(&e) != hipSuccess) return nullptr;
  (void)hipEventRecord(e, s);
  return e;
}
static void ktime_end(hipEvent_t e0, hipStream_t s) {
  if (!e0) return;
  std::lock_guard<std::mutex> g(g_ktime_mu);
  hipEvent_t e1 = nullptr;
  if (hipEventCreate(&e1) != hipSuccess) return;
  (void)hipEventRecord(e1, s);
  g_ktime_ev.emplace_back(e0, e1);
}

// The event behind the verification flags' copy: the context's (destroyed with
// it), or one made for this call when the caller passes none.
struct FlagsEvent {
  hipEvent_t ev = nullptr;
  bool own = false;
  explicit FlagsEvent(void* given) {
    if (given) {
      ev = (hipEvent_t)given;
    } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
      own = true;
    } else {
      ev = nullptr;
    }
  }
  ~FlagsEvent() {
    if (own) (void)hipEventDestroy(ev);
  }
};

extern "C" int xcg_launch_encode_stream(const XcgStreamArgs* a, int* rounds_out, hipStream_t stream) {
  using namespace xcg;

  const uint32_t n = a->n;
  if (n == 0) return 0;
  EncParams prm{a->in, a->chunk_off, a->chunk_len, n, a->flags, a->out, a->out_off, a->out_len, a->stats, a->status};
  prm.max_len = (a->maxd - 1) * SEG + (SEG - 1);     // maxd = max_chunk_len / 2048 + 1
  prm.g = HashTab{a->g_keys, a->g_vals, a->g_mask};
  prm.pool = a->pool;
  prm.b = HashTab{a->b_keys, a->b_vals, a->b_mask};
  prm.decl = (uint4*)a->decl;
  prm.ndecl = a->ndecl;
  prm.maxd = a->maxd;
  prm.changed = a->changed;
  prm.nseg = a->nseg;
  prm.bcount = a->bcount;
  prm.lds_filter_keys = xcg_lds_filter_keys();
  if (prm.lds_filter_keys == LFK_AUTO)
    prm.lds_filter_keys = 16ull * ((uint64_t)a->fmask + 1) > (2ull << 20) ? 0u : xcg::LDS_FILTER_KEYS_DEFAULT;
  prm.lds_prefilter_keys = __atomic_load_n(&g_lds_prefilter_keys, __ATOMIC_RELAXED);
  prm.ptime = a->ptime;
  prm.ev = (uint4*)a->ev;
  prm.nev = a->nev;
  prm.maxe = a->maxe;
  prm.eo = a->ev ? a->eo : nullptr;
  prm.rs = RestartArgs{};
  const size_t tbytes = ((size_t)a->fmask + 1) * 16;
  const size_t gbytes = ((size_t)a->gmask + 1) * 4;
  FlagsEvent flags_ev(a->flags_ev);
  int dev = 0;
  int cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -5;
  const uint32_t wgs = (uint32_t)cus;
  const bool big = a->maxd > 72;                     // chunks > 128 KiB (<= 512 KiB frames): 264 records
  // One workgroup per CU (LDS): SW chunk-waves each.  A batch too small to
  // give every CU a full workgroup spreads over more CUs with fewer waves
  // (a wave alone on its SIMD parses faster than four sharing it).
  const uint32_t SW = big ? (n <= 2 * wgs ? 2u : 6u) : (n <= 4 * wgs ? 4u : (n <= 8 * wgs ? 8u : 16u));
  const dim3 sgrid(min(wgs, (n + SW - 1) / SW)), sblock(64 * SW);
  auto launch_sw = [&](auto lru) {
    constexpr bool R = decltype(lru)::value;
    if (big) {
      if (SW == 2) hipLaunchKernelGGL((encode_stream_kernel<10, 264, 2, R>), sgrid, sblock, 0, stream, prm);
      else hipLaunchKernelGGL((encode_stream_kernel<10, 264, 6, R>), sgrid, sblock, 0, stream, prm);
    } else if (SW == 4) {
      hipLaunchKernelGGL((encode_stream_kernel<8, 72, 4, R>), sgrid, sblock, 0, stream, prm);
    } else if (SW == 8) {
      hipLaunchKernelGGL((encode_stream_kernel<8, 72, 8, R>), sgrid, sblock, 0, stream, prm);
    } else {
      hipLaunchKernelGGL((encode_stream_kernel<8, 72, 16, R>), sgrid, sblock, 0, stream, prm);
    }
  };
  // The quiet-chunk screen (stream_screen_kernel) in front of the parse: small
  // chunks, in-band, not the bounded / pair variants (which record references).
  const bool screen = a->s_fold && a->s_work && a->s_info && a->s_rows && a->s_qcnt && a->s_qkeys && !a->ev && !(a->flags & (XCG_FLAG_OOB | XCG_FLAG_NULLCACHE)) &&
                      a->maxd <= (uint32_t)SCREEN_MAXD && xcg_screen_on();
  // bounded cache: the variant that records the chunks' cache references (xcg_lru.hip)
  auto launch = [&]() {
    if (screen) {
      const uint32_t gwords = prm.lf.gmask + 1u;
      const uint32_t fwords = gwords < SCREEN_FOLD_WORDS ? gwords : SCREEN_FOLD_WORDS;
      hipLaunchKernelGGL(screen_fold_kernel, dim3((fwords + 255) / 256), dim3(256), 0, stream, prm.lf.gfilt, gwords,
                         a->s_fold, fwords);
      (void)hipMemsetAsync(a->s_work, 0, 4, stream);
      const ScreenStage sst{a->s_info, (uint4*)a->s_rows, a->s_qcnt, a->s_qkeys};
      const ScreenParams sp{prm.in, prm.chunk_off, prm.chunk_len, prm.out_off, prm.out, prm.decl, prm.ndecl,
                            prm.changed, prm.need, prm.n, prm.skip_below, prm.max_len, prm.maxd};
      hipLaunchKernelGGL(stream_screen_kernel<SCREEN_W>, dim3(wgs), dim3(64 * SCREEN_W), 0, stream, sp,
                         (const uint32_t*)a->s_fold, fwords, sst);
      hipLaunchKernelGGL(screen_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, prm, sst, a->s_work);
      prm.work = a->s_work;
      if (xcg_screen_counting()) {
        uint32_t w = 0;
        (void)hipMemcpyAsync(&w, a->s_work, 4, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        uint32_t seen = n;
        if (prm.need) {
          std::vector<uint32_t> h(n);
          (void)hipMemcpy(h.data(), prm.need, 4ull * n, hipMemcpyDeviceToHost);
          seen = 0;
          for (uint32_t v : h) seen += v != 0;
        }
        __atomic_add_fetch(&g_screen_seen, (uint64_t)(seen - (prm.skip_below < seen ? prm.skip_below : 0u)),
                           __ATOMIC_RELAXED);
        __atomic_add_fetch(&g_screen_parsed, (uint64_t)w, __ATOMIC_RELAXED);
      }
    }
    if (stream_debug()) {
      uint32_t cnt = n;
      if (prm.need) {
        std::vector<uint32_t> h(n);
        (void)hipMemcpyAsync(h.data(), prm.need, 4ull * n, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        cnt = 0;
        for (uint32_t v : h) cnt += v != 0;
      }
      fprintf(stderr, "stream: launch over %u of %u chunks (skip below %u)\n", cnt, n, prm.skip_below);
    }
    hipEvent_t e0 = ktime_begin(stream);
    if (prm.ev) launch_sw(std::integral_constant<bool, true>{});
    else launch_sw(std::integral_constant<bool, false>{});
    ktime_end(e0, stream);
    prm.work = nullptr;
  };
  // lowest chunk whose declaration list changed in the round just run (~0u: none)
  auto changed_after = [&](uint32_t& fc) -> bool {
    if (hipMemcpyAsync(a->h_changed, a->changed, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return false;
    fc = *a->h_changed;
    return true;
  };
  const bool keep = a->keep_decls && n > 1;
  const bool seeded = (a->seed || keep) && n > 1;
  if (!seeded && (hipMemsetAsync(a->ndecl, 0, 4ull * n, stream) != hipSuccess ||
                  hipMemsetAsync(a->nhits, 0, 4ull * n, stream) != hipSuccess ||
                  hipMemsetAsync(a->changed, 0xFF, 4, stream) != hipSuccess))
    return -5;                                       // (the seed kernel initialises these itself)
  if (a->decls_out) *a->decls_out = ~0u;
  prm.need = nullptr;
  prm.hits = a->hits;                              // every stream round writes nhits[chunk]
  prm.nhits = a->nhits;
  prm.maxh = a->maxh;
  // Round 0: every chunk against the persistent cache + its own declarations.
  prm.use_b = false;
  prm.skip_below = 0;
  prm.lf = LaneFilter{a->g_filt, (const u32x4*)a->g_ftab, a->fmask, a->g_gfilt, a->gmask};
  HashTab tabs[2] = {HashTab{a->b_keys, a->b_vals, a->b_mask}, HashTab{a->b2_keys, a->b2_vals, a->b_mask}};
  const HashTab rt{a->r_keys, a->r_vals, a->r_mask};
  // (a) by probing the windows (a_bits null: the conservative flag)
  const bool probe = a->a_bits && a->a_keys;
  const HashTab at = probe ? HashTab{a->a_keys, a->a_vals, XCG_VERIFY_A_CAP - 1} : HashTab{nullptr, nullptr, 0u};
  int cur = 0;
  int dev_cus = (int)wgs;
  // A round's batch table, filters and counters cleared / copied from the cache's.
  // later rounds resume flagged chunks too (bounded / pair: the verification
  // gives the affected lookups' times)
  const bool rs_rounds = a->ev && a->restart && a->bslot && prm.eo && a->bad_t;
  static const bool pf_off = getenv("XCG_NO_PREFIX_FILTERS") != nullptr;   // (A/B runs: one slice)
  const uint32_t pfdiv = pf_off ? 0u : (n + PREFIX_FILTERS - 1) / PREFIX_FILTERS;   // chunks per slice of the round's LDS filter
  auto prep = [&](int t, bool verify, uint32_t what) -> bool {
    RoundPrep rp{tabs[t], a->r_filt, a->g_filt, (u32x4*)a->r_ftab, (const u32x4*)a->g_ftab, (uint32_t)(tbytes / 16),
                 a->r_gfilt, a->g_gfilt, (uint32_t)(gbytes / 4), a->nseg, a->bcount, a->changed,
                 verify ? rt : HashTab{nullptr, nullptr, 0u}, a->vflags, at, a->a_bits, n, a->need,
                 rs_rounds ? a->bad_t : nullptr, rs_rounds ? a->bad_hi : nullptr, what};
    hipLaunchKernelGGL(round_prep_kernel, dim3(4 * dev_cus), dim3(256), 0, stream, rp);
    return hipGetLastError() == hipSuccess;
  };
  bool seed_built = false;
  int rounds = 0;
  uint32_t fc = 0;
  if (keep) {
    // the previous pass's declaration lists seed round 1 (a bounded cache's
    // eviction times changed under them)
  } else if (seeded) {
    // Round 1's table and filters are built by the seed itself (after the
    // round's prep has cleared them) when its waves hash full groups of tiles;
    // with small chunks (a wave per chunk of one or two tiles) the waves would
    // sit on their inserts at low occupancy (C4's 4 KiB packets: seed 66 ->
    // 342 us), so the separate build keeps them.
    const bool fuse = a->maxd > SEED_TILES;
    if (fuse && !prep(cur, false, PREP_TABLE | PREP_FILTERS)) return -5;
    const uint32_t seed_waves = n * ((a->maxd + SEED_TILES - 1) / SEED_TILES);
    hipLaunchKernelGGL(seed_tiling_kernel, dim3((seed_waves + 3) / 4), dim3(256), 0, stream, a->in, a->chunk_off,
                       a->chunk_len, n, a->maxd, (uint4*)a->decl, a->ndecl, a->nhits, a->changed,
                       fuse ? tabs[cur] : HashTab{nullptr, nullptr, 0u},
                       FiltSet{a->r_filt, a->r_ftab, a->fmask, a->r_gfilt, a->gmask}, a->bcount, a->status, pfdiv);
    if (fuse) hipLaunchKernelGGL(filt_prefix_kernel, dim3(FILT_WORDS / 256), dim3(256), 0, stream, a->r_filt);
    seed_built = fuse;
  } else {
    launch();
    rounds = 1;
    // (one chunk: no round follows, so no need to learn what it declared)
    if (n > 1 && !changed_after(fc)) return -5;
    if (n > 1 && fc == ~0u && a->decls_out) *a->decls_out = 0;   // round 0 declared nothing
  }
  // Jacobi rounds: chunk k re-parses against the declarations chunks < k made
  // in the previous round.  Chunk 0 is exact after round 0 and, inductively,
  // chunk k after round k.  Round 1 re-parses every chunk after the first
  // that declared anything in round 0 (those before it saw an empty batch);
  // after each later round the verification (verify_*_kernel) compares the
  // round's batch table with the one the round parsed against and flags the
  // chunks whose lookups could change; only those are re-parsed.  No flag =
  // the fixed point, which is the sequential result.

  // Commit the declaration lists into the persistent cache; with a gate, only
  // if the verification that precedes it in the stream flagged nothing.
  bool committed = false;
  auto commit = [&](const uint32_t* gate) {
    if (a->no_commit) return;
    const uint32_t parts = (a->maxd + 255) / 256;
    uint32_t* seg_base = (uint32_t*)a->hits;       // (free once the rounds are over: n words)
    hipLaunchKernelGGL(commit_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint32_t*)a->ndecl, n, seg_base,
                       a->nseg, gate);
    hipLaunchKernelGGL(commit_kernel, dim3(n * parts), dim3(256), 0, stream, (const uint4*)a->decl,
                       (const uint32_t*)a->ndecl, n, a->maxd, a->in, a->chunk_off, prm.g, a->pool,
                       (const uint32_t*)seg_base, a->seg_cap,
                       FiltSet{a->g_filt, a->g_ftab, a->fmask, a->g_gfilt, a->gmask}, a->status, gate);
  };
  auto build = [&](int t, bool verify, uint32_t what) -> bool {
    if (!prep(t, verify, what)) return false;
    const uint64_t nthreads = (uint64_t)n * a->maxd;
    hipLaunchKernelGGL(build_batch_table_kernel, dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, stream,
                       (const uint4*)a->decl, (const uint32_t*)a->ndecl, n, a->maxd, tabs[t],
                       FiltSet{a->r_filt, a->r_ftab, a->fmask, a->r_gfilt, a->gmask}, a->bcount, a->status, what,
                       pfdiv);
    if (what & PREP_FILTERS)
      hipLaunchKernelGGL(filt_prefix_kernel, dim3(FILT_WORDS / 256), dim3(256), 0, stream, a->r_filt);
    return hipGetLastError() == hipSuccess;
  };
  // A re-parse round whose flagged chunks (their first contradicted lookup in
  // bad_t) resume from their rows (encode_chunk, "Re-parse restart"): back
  // the rows up, parse, splice the rejoined tails' bytes.
  auto run_restarted = [&]() {
    (void)hipMemsetAsync(a->b_count, 0, 4, stream);
    hipLaunchKernelGGL(restart_backup_kernel, dim3(n), dim3(256), 0, stream, n, (const uint32_t*)a->need,
                       (const uint32_t*)a->bad_t, a->bslot, a->b_count, a->b_slots, (const uint8_t*)a->out,
                       a->out_off, (const uint64_t*)a->out_len, a->b_out, a->b_stride, (const uint4*)a->ev,
                       (const uint32_t*)a->eo, (const uint32_t*)a->nev, a->maxe, (const uint64_t*)a->hits,
                       (const uint32_t*)a->nhits, a->maxh, (const uint32_t*)a->ndecl, (uint4*)a->b_ev, a->b_eo,
                       a->b_hits, a->b_cnt);
    prm.rs = RestartArgs{a->bad_t, a->bad_hi, a->bslot, (const uint4*)a->b_ev, a->b_eo, a->b_hits, a->b_cnt,
                         (uint4*)a->splice};
    launch();
    hipLaunchKernelGGL(restart_splice_kernel, dim3(n), dim3(256), 0, stream, n, (uint4*)a->splice,
                       (const uint32_t*)a->bslot, (const uint8_t*)a->b_out, a->b_stride, a->out, a->out_off,
                       a->b_count);
    prm.rs = RestartArgs{};
    if (stream_debug()) {
      uint32_t bc[4] = {0, 0, 0, 0};
      (void)hipMemcpyAsync(bc, a->b_count, 16, hipMemcpyDeviceToHost, stream);
      (void)hipStreamSynchronize(stream);
      fprintf(stderr, "stream: restart slots %u, cumulative resumed %u rejoined %u\n", bc[0], bc[2], bc[3]);
    }
  };
  if (n > 1 && fc != ~0u) {
    if (!seed_built && !build(cur, false, PREP_TABLE | PREP_FILTERS)) return -5;
    prm.use_b = true;
    prm.b = tabs[cur];
    prm.skip_below = seeded ? 0 : fc + 1;            // (seeded: round 1 parses every chunk)
    prm.lf = LaneFilter{a->r_filt, (const u32x4*)a->r_ftab, a->fmask, a->r_gfilt, a->gmask, pfdiv};
    if (keep && a->need_given) prm.need = a->need;   // the rest stand under the kept lists
    const bool rs = keep && a->need_given && a->restart && a->bslot && prm.eo;
    if (rs) run_restarted();
    else launch();
    ++rounds;
    prm.skip_below = 0;
    // (no host sync here: the verification's own sync tells whether round 1
    // changed anything that matters)
    // Each round fixes at least the first flagged chunk (every chunk before
    // it already stands under the final lists), so n rounds always suffice.
    bool converged = false;
    for (uint32_t r = 2; r <= n + 1; ++r) {
      // verify round r-1 (parsed against tabs[cur]) against its own declarations
      const int nxt = cur ^ 1;
      if (!build(nxt, true, PREP_TABLE)) return -5;   // (filters only if a re-parse follows)
      const uint64_t slots = 2ull * (a->b_mask + 1);
      hipLaunchKernelGGL(verify_diff_kernel, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, stream, tabs[cur],
                         tabs[nxt], a->in, a->chunk_off, rt, a->vflags, at, a->a_bits, a->status);
      uint32_t* vbad_t = rs_rounds ? a->bad_t : nullptr;
      uint32_t* vbad_hi = rs_rounds ? a->bad_hi : nullptr;
      {
        VerifyFlags v{};
        v.n = n;
        v.bc = (n + 255) / 256;
        if (probe) {
          const uint64_t items = (uint64_t)n * a->maxd;   // (chunk, 2048-position span) pairs, maxd per chunk
          const uint64_t blocks = (items + 3) / 4, cap = 5ull * (uint64_t)dev_cus;   // (32 KiB of LDS each)
          v.bp = (uint32_t)(blocks < cap ? blocks : cap);
        }
        v.bh = a->ev ? (n + 3) / 4 : (uint32_t)(((uint64_t)n * a->maxh + 255) / 256);
        v.nhits = (const uint32_t*)a->nhits; v.maxh = a->maxh; v.hits = (const uint64_t*)a->hits;
        v.nev = (const uint32_t*)(a->ev ? a->nev : nullptr); v.maxe = a->maxe; v.ev = (const uint4*)a->ev;
        v.probe = probe; v.vflags = a->vflags; v.need = a->need; v.bad_t = vbad_t; v.bad_hi = vbad_hi;
        v.in = a->in; v.chunk_off = a->chunk_off; v.chunk_len = a->chunk_len; v.spc = a->maxd;
        v.at = at; v.abits = (const uint32_t*)a->a_bits; v.rt = rt; v.bcount = (const uint32_t*)a->bcount;
        hipLaunchKernelGGL(verify_flags_kernel, dim3(v.bc + v.bp + v.bh), dim3(256), 0, stream, v);
      }
      if (hipMemcpyAsync(a->h_vflags, a->vflags, 16, hipMemcpyDeviceToHost, stream) != hipSuccess) return -5;
      // The host waits for the flags alone: the commit (a no-op if anything was
      // flagged) runs on the device while the host returns and queues the next
      // batch behind it, so the device does not idle through the host's turn.
      const hipEvent_t vev = flags_ev.ev;
      if (!vev || hipEventRecord(vev, stream) != hipSuccess) return -5;
      commit(a->vflags + 1);
      if (a->post_verify && a->post_verify(a->post_user, a->vflags + 1, stream)) return -5;
      if (hipEventSynchronize(vev) != hipSuccess) return -5;
      if (a->decls_out) *a->decls_out = a->h_vflags[2];
      if (stream_debug())
        fprintf(stderr, "stream: n %u round %u first (a)-flag %d any %u newly visible %u\n", n, r,
                (int)a->h_vflags[0], a->h_vflags[1], a->h_vflags[3]);
      if (a->h_vflags[1] == 0) {                       // nothing flagged: fixed point (already committed)
        converged = true;
        committed = true;
        break;
      }
      if (hipMemsetAsync(a->changed, 0xFF, 4, stream) != hipSuccess) return -5;
      if (!build(nxt, false, PREP_FILTERS)) return -5;   // the re-parse's filters: cache + round r-1's lists
      cur = nxt;
      prm.b = tabs[cur];
      prm.need = a->need;
      if (rs_rounds) run_restarted();                // (resumed before the first affected lookup)
      else launch();                                 // (flagged by the verification: from the start)
      ++rounds;
    }
    if (!converged) return -75;
  }
  // A result no verification passed over (one chunk, or round 0 declared
  // nothing): an own-table overflow in it is reported (status bit 0).
  if (!committed) hipLaunchKernelGGL(own_ovf_check_kernel, dim3((n + 255) / 256), dim3(256), 0, stream,
                                     (const uint32_t*)a->nhits, n, a->maxh, a->status);
  if (!committed) commit(nullptr);
  if (rounds_out) *rounds_out = rounds;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
