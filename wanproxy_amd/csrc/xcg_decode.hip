// XCodec decoder, MI355X (gfx950) HIP kernels.
//
// Restates XCodecDecoder::decode (xcodec/xcodec_decoder.cc:66-188) for a batch
// of encoded chunks that form ONE stream (successive decode() calls on one
// decoder and cache, e.g. tack -d, programs/tack/tack.cc:329-359, or the
// frames of one XCodecPipePair, xcodec/xcodec_pipe_pair.cc:425-483).
//
//   scan   (one wave per chunk): walk the op stream.  Literal runs are found
//          1 KiB at a time with a wave ballot over the bytes: an 0xF1 followed
//          by 0x00 is an ESCAPE inside the run, any other 0xF1 starts an op.
//          EXTRACT payloads are hashed (XCodecHash::hash, :106) and entered in
//          the batch table X: hash -> earliest / latest stream position.
//   size   exclusive scan of the decoded lengths -> output offsets.
//   emit   (one wave per chunk): walk again and write: literal runs with
//          F1 00 -> F1, EXTRACT payloads, REF segments gathered from the
//          earliest earlier EXTRACT in the batch or from the persistent cache
//          (the cache state at that point of the stream, :151-162).  A REF
//          that neither resolves blocks the stream there (:151-156).
//   commit EXTRACTs before the blocking point enter the cache
//          (XCodecMemoryCache::enter / replace, :120-136).
//
// BACKREF (:165-181) reads the decoder's XCodecWindow (xcodec/xcodec_window.h):
// every EXTRACT and resolved REF declares its hash into slot k mod 256 (k =
// declares made by this decoder so far), emptying the slot that held the same
// hash before (:68-100).  Slot c at declare count G therefore holds the latest
// declare g < G with g = c (mod 256) unless that hash was declared again in
// (g, G).  The scan counts declares per chunk; an exclusive scan numbers them;
// `decl_record` writes (hash, bytes) records of the declares a BACKREF or the
// window update can reach; an invalid BACKREF stops the stream like an unknown
// REF (decode() returns false there, :172-176); `window_update` carries the
// 256 slots (hash + an owned copy of the bytes) into the next batch.
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <utility>
#include <vector>

#include "xcg_cache.h"
#include "xcg_args.h"

namespace xcg {

struct DecParams {
  const uint8_t* in;           // encoded chunks
  const uint64_t* chunk_off;
  const uint32_t* chunk_len;
  uint32_t n;
  HashTab g;                   // persistent cache
  const uint8_t* pool;
  HashTab x;                   // batch EXTRACT table: hash -> (earliest, latest) packed positions
  uint64_t* x_latest;          // parallel to x.vals: latest position (atomicMax)
  uint64_t* out_len;           // scan: tentative decoded length; emit: final
  const uint64_t* out_off;     // emit: exclusive scan of scan's out_len
  uint8_t* out;
  int32_t* chunk_status;       // 0 ok, 1 blocked (unknown REF), 2 not reached, 3 partial op at end, <0 error
  uint64_t* consumed;          // input bytes fully parsed per chunk
  uint64_t* unknown;           // emit: unresolvable REFs (hash), with their positions
  uint64_t* unknown_pos;
  uint32_t* nunknown;
  uint32_t unknown_cap;
  uint64_t* block_pos;         // min stream position of an unresolvable REF (atomicMin)
  int32_t* status;             // bit 9: EXTRACT name reuse inside the batch
  // ---- BACKREF window
  uint64_t* berr_pos;          // min stream position of a BACKREF to an empty slot (atomicMin)
  uint64_t* n_decl;            // scan: declares (EXTRACT + REF) per chunk
  uint64_t* n_bref;            // scan: BACKREFs per chunk
  const uint64_t* decl_base;   // exclusive scan of n_decl: batch index of the chunk's first declare
  uint64_t* n_decl_emit;       // emit: declares made before the chunk stopped
  uint64_t* t_end;             // declares of the batch before the stop point
  uint4* D;                    // declare records (lo, hi, src lo, src hi), batch indices [D_lo, ...)
  uint64_t D_lo;               // (tail mode: D_lo = max(t_end - 256, 0), read from *t_end)
  bool D_tail;
  // (emit, no stop point) the window's tail records written by the emit pass
  // itself: declares [tail_lo, tail_hi) into tail_D (null: decl_record_kernel)
  uint4* tail_D;
  uint64_t tail_lo, tail_hi;
  uint64_t* win_hash;          // the decoder's window: 256 hashes (0 = empty slot)
  uint8_t* win_seg;            //   and the bytes of each slot
  uint64_t win_count;          // declares made before this batch
  // ---- bounded cache (xcg_lru.hip): a persistent entry serves a lookup at
  // stream time (chunk << 21 | op offset) only before ptime[slot]
  const uint64_t* ptime;
  uint64_t* u_keys;            // unknown-hash set (EMPTY_KEY = free)
  uint32_t u_mask;
};

// Insert h into an open-addressed set; true if it was not there.  A full set
// reports every hash as new (the caller then overflows its cap).
__device__ __forceinline__ bool uset_insert(uint64_t* keys, uint32_t mask, uint64_t h) {
  uint32_t i = tab_slot((uint32_t)h, (uint32_t)(h >> 32), mask);
  for (uint32_t n = 0; n <= mask; ++n) {
    const uint64_t prev = atomicCAS((unsigned long long*)&keys[i], (unsigned long long)EMPTY_KEY,
                                    (unsigned long long)h);
    if (prev == EMPTY_KEY) return true;
    if (prev == h) return false;
    i = (i + 1) & mask;
  }
  return true;
}

// Is persistent slot gv live for a lookup at stream position `here`?
__device__ __forceinline__ bool g_live(const DecParams& prm, uint64_t gv, uint64_t here) {
  if (gv == ~0ull) return false;
  if (!prm.ptime) return true;
  return ((here >> 32 << 21) | (uint32_t)here) < prm.ptime[gv];
}

__device__ __forceinline__ uint64_t spos(uint32_t chunk, uint32_t off) { return ((uint64_t)chunk << 32) | off; }

// Next real op at or after i in x[0..len): an 0xF1 not followed by 0x00.
// Returns its position (or len) and the number of ESCAPE pairs before it.
// (P: a generic pointer, or an LDS-qualified one for input staged in LDS -- then
// the walk's loads wait on LDS alone, not on the global stores queued behind them)
template <typename P>
__device__ __forceinline__ uint32_t next_op(P x, uint32_t i, uint32_t len, uint32_t& nesc) {
  const int l = lane_id();
  nesc = 0;
  // Fast path: the op follows immediately (EXTRACT/REF-dense streams).
  if (i < len && x[i] == MAGIC && (i + 1 >= len || x[i + 1] != 0u)) return i;
  for (uint32_t base = i; base < len; base += 1024) {
    const uint32_t off = base + 16u * l;
    uint32_t opmask = 0, escmask = 0;
    if (off < len) {
      const uint32_t cnt = min(16u, len - off);
      uint32_t b[17];
#pragma unroll
      for (int k = 0; k < 17; ++k) b[k] = (off + k < len) ? (uint32_t)x[off + k] : 0x100u;  // 0x100: past the end
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if ((uint32_t)k < cnt && b[k] == MAGIC) {
          if (b[k + 1] == 0u) escmask |= 1u << k;
          else opmask |= 1u << k;
        }
      }
    }
    // An ESCAPE's 0x00 is never itself scanned as a byte that matters (it is
    // not 0xF1), so the masks are exact.  First op in this window:
    const uint64_t bal = ballot(opmask != 0u);
    if (bal) {
      const int lw = __builtin_ctzll(bal);
      const uint32_t om = readlane(opmask, lw);
      const uint32_t pos = base + 16u * lw + __builtin_ctz(om);
      // escapes strictly before pos
      uint32_t e = (uint32_t)l < (uint32_t)lw ? __builtin_popcount(escmask)
                   : ((uint32_t)l == (uint32_t)lw ? __builtin_popcount(escmask & ((1u << __builtin_ctz(om)) - 1u)) : 0u);
      nesc += wave_sum(e);
      return pos;
    }
    nesc += wave_sum(__builtin_popcount(escmask));
  }
  return len;
}

// Copy the literal run x[a..b) (which contains only ESCAPE pairs) to dst with
// F1 00 -> F1.  Returns bytes written.
__device__ __noinline__ uint32_t wave_unescape(uint8_t* dst, const uint8_t* x, uint32_t a, uint32_t b) {
  const int l = lane_id();
  uint32_t written = 0;
  // An escape pair never straddles 16-byte lanes ambiguously: a 0x00 is an
  // escape zero iff the byte before it is 0xF1 (runs hold no other 0xF1).
  for (uint32_t base = a; base < b; base += 1024) {
    const uint32_t off = base + 16u * l;
    uint32_t cnt = off < b ? min(16u, b - off) : 0u;
    uint32_t v[16];
    uint32_t prev = (off > a && off - 1 < b) ? (uint32_t)x[off - 1] : 0u;
    uint32_t keep = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      v[k] = ((uint32_t)k < cnt) ? (uint32_t)x[off + k] : 0u;
      const bool drop = (uint32_t)k < cnt && v[k] == 0u && prev == MAGIC;
      if ((uint32_t)k < cnt && !drop) keep |= 1u << k;
      prev = drop ? 0u : v[k];   // F1 00 F1 00: the 00 resets
    }
    const uint32_t nk = __builtin_popcount(keep);
    const uint32_t incl = wave_incl_scan(nk);
    uint32_t o = written + incl - nk;
    if (nk == 16u && cnt == 16u) {
      u32x4 w;
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = v[4 * q] | (v[4 * q + 1] << 8) | (v[4 * q + 2] << 16) | (v[4 * q + 3] << 24);
      *(u32x4_u*)(dst + o) = w;
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if ((keep >> k) & 1u) dst[o++] = (uint8_t)v[k];
    }
    written += readlane(incl, 63);
  }
  return written;
}

// 16 bytes at any alignment, from global memory or from LDS
typedef const __attribute__((address_space(3))) uint8_t* lds_u8p;
typedef const __attribute__((address_space(3))) u32x4_u* lds_u32x4p;
__device__ __forceinline__ u32x4 load16(const uint8_t* p) { return *(const u32x4_u*)p; }
__device__ __forceinline__ u32x4 load16(lds_u8p p) { return *(lds_u32x4p)p; }

template <typename P>
__device__ __noinline__ uint2 dec_window_hash(P w) {
  const int l = lane_id();
  uint32_t X1 = 0, X2 = 0, F1 = 0, F2 = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t k0 = 1024u * h + 16u * l;
    const u32x4 v = load16(w + k0);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t c = byte_of(v[k >> 2], k & 3);
      const uint32_t f = ffbl(c) + 1u;
      const uint32_t wt = 2048u - (k0 + k);
      X1 += c; X2 += wt * c; F1 += f; F2 += wt * f;
    }
  }
  X1 = wave_sum(X1); X2 = wave_sum(X2); F1 = wave_sum(F1); F2 = wave_sum(F2);
  return make_uint2((X1 << 20) + X2 + CLO, ((F1 << 16) + F2) << 4);
}

__device__ __forceinline__ void wave_copy2048(uint8_t* dst, const uint8_t* src) {
  const int l = lane_id();
  *(u32x4_u*)(dst + 32 * l) = *(const u32x4_u*)(src + 32 * l);
  *(u32x4_u*)(dst + 32 * l + 16) = *(const u32x4_u*)(src + 32 * l + 16);
}

__device__ __noinline__ bool dec_equal2048(const uint8_t* a, const uint8_t* b) {
  const int l = lane_id();
  const u32x4 a0 = *(const u32x4_u*)(a + 32 * l), a1 = *(const u32x4_u*)(a + 32 * l + 16);
  const u32x4 b0 = *(const u32x4_u*)(b + 32 * l), b1 = *(const u32x4_u*)(b + 32 * l + 16);
  const bool ok = a0[0] == b0[0] && a0[1] == b0[1] && a0[2] == b0[2] && a0[3] == b0[3] && a1[0] == b1[0] &&
                  a1[1] == b1[1] && a1[2] == b1[2] && a1[3] == b1[3];
  return ballot(!ok) == 0;
}

template <typename P>
__device__ __forceinline__ uint64_t be64(P p) {
  uint64_t h = 0;
  for (int k = 0; k < 8; ++k) h = (h << 8) | p[k];
  return h;
}

// Batch table insert with earliest (vals, atomicMin) and latest (atomicMax).
__device__ __forceinline__ bool xtab_insert(HashTab t, uint64_t* latest, uint32_t lo, uint32_t hi, uint64_t pos,
                                            bool& existed) {
  const uint64_t key = ((uint64_t)hi << 32) | lo;
  uint32_t i = tab_slot(lo, hi, t.mask);
  for (uint32_t n = 0; n <= t.mask; ++n) {
    const uint64_t prev = atomicCAS((unsigned long long*)&t.keys[i], (unsigned long long)EMPTY_KEY,
                                    (unsigned long long)key);
    if (prev == EMPTY_KEY || prev == key) {
      existed = prev == key;
      atomicMin((unsigned long long*)&t.vals[i], (unsigned long long)pos);
      atomicMax((unsigned long long*)&latest[i], (unsigned long long)pos);
      return true;
    }
    i = (i + 1) & t.mask;
  }
  return false;
}

// ------------------------------------------------------------------ window

__device__ __forceinline__ uint64_t d_lo_of(const DecParams& prm) {
  if (!prm.D_tail) return prm.D_lo;
  const uint64_t te = readfirst64(*prm.t_end);
  return te > 256u ? te - 256u : 0u;
}

// XCodecWindow::dereference(c) (xcodec/xcodec_window.h:102-111) after T
// declares of this batch: false if the slot is empty, else the slot's hash
// and bytes.  Wave-uniform.  `gd` receives the global declare index.
__device__ bool window_slot(const DecParams& prm, uint64_t T, uint32_t c, uint64_t& h, const uint8_t*& src,
                            uint64_t& gd) {
  const uint64_t W = prm.win_count, G = W + T, DL = d_lo_of(prm);
  if (G == 0) return false;
  const uint64_t r = (G - 1u - c) & 255u;
  if (r > G - 1u) return false;                              // slot never written
  const uint64_t g = G - 1u - r;                              // latest declare with g = c (mod 256)
  gd = g;
  if (g < W) {                                               // made before this batch: the window holds it
    h = readfirst64(prm.win_hash[c]);
    if (h == 0) return false;                                // emptied by a re-declare (:79-83)
    src = prm.win_seg + (uint64_t)c * SEG;
  } else {
    const uint4 rec = prm.D[g - W - DL];
    h = ((uint64_t)readfirst(rec.y) << 32) | readfirst(rec.x);
    src = (const uint8_t*)(((uint64_t)readfirst(rec.w) << 32) | readfirst(rec.z));
  }
  // declared again after g (batch declares only; the window state covers the rest)?
  const uint64_t a = (g + 1u > W ? g + 1u - W : 0u), b = T;
  bool dup = false;
  for (uint64_t t = a + lane_id(); t < b; t += 64) {
    const uint4 e = prm.D[t - DL];
    dup |= e.x == (uint32_t)h && e.y == (uint32_t)(h >> 32);
  }
  return ballot(dup) == 0;
}

// REF source: the earliest EXTRACT of h in the batch before `here`, else the
// persistent cache (the cache state at that point of the stream).
__device__ __forceinline__ const uint8_t* ref_source(const DecParams& prm, uint32_t lo, uint32_t hi, uint64_t here) {
  const uint64_t e = tab_lookup(prm.x, lo, hi);
  if (e != ~0ull && e < here) return prm.in + prm.chunk_off[e >> 32] + (uint32_t)e;
  const uint64_t gv = tab_lookup(prm.g, lo, hi);
  if (g_live(prm, gv, here)) return prm.pool + gv * (uint64_t)SEG;
  return nullptr;
}

// Per-lane REF source (the same rule as ref_source, each lane its own hash).
__device__ __forceinline__ const uint8_t* ref_source_t(const DecParams& prm, uint32_t lo, uint32_t hi, uint64_t here) {
  const uint64_t e = tab_lookup_t(prm.x, lo, hi);
  if (e != ~0ull && e < here) return prm.in + prm.chunk_off[e >> 32] + (uint32_t)e;
  const uint64_t gv = tab_lookup_t(prm.g, lo, hi);
  if (g_live(prm, gv, here)) return prm.pool + gv * (uint64_t)SEG;
  return nullptr;
}

// A run of consecutive REF ops from offset i (the op at i is a whole REF
// before `limit`): lane l takes the l-th REF, at i + 10 l, while every op
// before it is a REF too (a REF is 10 bytes, so that is where the next op
// starts).  REF-dense streams (warm caches: one REF per 2 KiB) then pay one
// round of lane-parallel table lookups per 64 REFs instead of one dependent
// chain per REF.  Returns the run length (1..64, uniform); lanes < run get
// their hash and stream position.
template <typename P>
__device__ __forceinline__ uint32_t ref_run(P x, uint32_t i, uint32_t len, uint32_t chunk,
                                            uint64_t limit, uint64_t& h, uint64_t& here) {
  const uint32_t l = (uint32_t)lane_id();
  const uint32_t o = i + 10u * l;
  here = spos(chunk, o);
  bool isref = o + 10u <= len && here < limit;
  if (isref) isref = x[o] == MAGIC && x[o + 1] == OP_REF;
  const uint64_t bad = ballot(!isref);
  const uint32_t r = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
  h = 0;
  if (l < r) h = be64(x + o + 2);
  return r;
}

// Copy k segments (pointers held by lanes 0..k-1) to dst, consecutively; the
// loads of four segments are in flight together.
__device__ __forceinline__ void copy_segments(uint8_t* dst, const uint8_t* src_lane, uint32_t k) {
  const int l = lane_id();
  for (uint32_t a = 0; a < k; a += 4) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (a + j < k) {
        const uint64_t sp = readlane64((uint64_t)src_lane, (int)(a + j));
        const uint8_t* sj = (const uint8_t*)sp;
        v[2 * j] = *(const u32x4_u*)(sj + 32 * l);
        v[2 * j + 1] = *(const u32x4_u*)(sj + 32 * l + 16);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (a + j < k) {
        uint8_t* d = dst + (uint64_t)(a + j) * SEG;
        *(u32x4_u*)(d + 32 * l) = v[2 * j];
        *(u32x4_u*)(d + 32 * l + 16) = v[2 * j + 1];
      }
    }
  }
}

// ------------------------------------------------------------------ kernels

template <bool EMIT>
__global__ __launch_bounds__(256) void decode_kernel(DecParams prm) {
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t chunk = blockIdx.x * 4u + (uint32_t)wv;
  if (chunk >= prm.n) return;
  const int l = lane_id();
  const uint8_t* x = prm.in + prm.chunk_off[chunk];
  const uint32_t len = prm.chunk_len[chunk];
  uint8_t* out = EMIT ? prm.out + prm.out_off[chunk] : nullptr;
  uint64_t olen = 0;
  int32_t st = 0;
  uint32_t i = 0;
  uint64_t ndecl = 0, nbref = 0;
  const uint64_t blockp = EMIT ? min(readfirst64(*prm.block_pos), readfirst64(*prm.berr_pos)) : ~0ull;
  if (EMIT && spos(chunk, 0) > blockp) {      // after the stop point: decode() never got here
    if (l == 0) {
      prm.out_len[chunk] = 0;
      prm.chunk_status[chunk] = 2;
      prm.consumed[chunk] = 0;
      prm.n_decl_emit[chunk] = 0;
    }
    return;
  }
  const uint64_t dbase = EMIT ? prm.decl_base[chunk] : 0;

  while (i < len) {
    uint32_t nesc = 0;
    const uint32_t m = next_op(x, i, len, nesc);
    // literal run [i, m) with nesc escape pairs (:71-81 and OP_ESCAPE :91-94)
    if (m > i) {
      if (EMIT) olen += readfirst(wave_unescape(out + olen, x, i, m));
      else olen += (m - i) - nesc;
    }
    i = m;
    if (i >= len) break;
    if (len - i == 1) { st = 3; break; }                     // :87-88 need the op byte
    const uint32_t op = x[i + 1];
    if (op == OP_EXTRACT) {                                  // :96-140
      if (len - i < 2u + SEG) { st = 3; break; }
      const uint8_t* seg = x + i + 2;
      if (EMIT) {
        wave_copy2048(out + olen, seg);
        const uint64_t t = dbase + ndecl;
        if (prm.tail_D && t >= prm.tail_lo && t < prm.tail_hi) {   // (the window's tail: its hash here)
          const uint2 h = dec_window_hash(seg);
          const uint64_t src = (uint64_t)seg;
          if (l == 0) prm.tail_D[t - prm.tail_lo] = make_uint4(readfirst(h.x), readfirst(h.y), (uint32_t)src,
                                                               (uint32_t)(src >> 32));
        }
      } else {
        const uint2 h = dec_window_hash(seg);
        bool existed = false;
        if (l == 0 && !xtab_insert(prm.x, prm.x_latest, readfirst(h.x), readfirst(h.y), spos(chunk, i + 2),
                                   existed))
          atomicOr(prm.status, 1 << 10);
        (void)existed;
      }
      olen += SEG;
      i += 2 + SEG;
      ++ndecl;                                               // window_.declare, :137
    } else if (op == OP_REF) {                               // :141-163
      if (len - i < 10u) { st = 3; break; }
      if (EMIT && spos(chunk, i) >= blockp) { st = 1; break; }   // blocked at or before this op
      // Resolvability (an earlier EXTRACT of h in the batch, or the cache)
      // is checked after the scan (decode_refcheck_kernel), once the batch
      // table is complete; emit resolves a whole run of REFs at a time.
      uint64_t h, here;
      uint32_t r = ref_run(x, i, len, chunk, blockp, h, here);
      bool stop = false;
      if (EMIT) {
        const uint8_t* src = nullptr;
        if ((uint32_t)l < r) src = ref_source_t(prm, (uint32_t)h, (uint32_t)(h >> 32), here);
        const uint64_t miss = ballot((uint32_t)l < r && src == nullptr);
        if (miss) {                                          // cannot happen: refcheck found all
          r = (uint32_t)__builtin_ctzll(miss);
          stop = true;
        }
        copy_segments(out + olen, src, r);
        const uint64_t tl = dbase + ndecl + (uint64_t)l;
        if (prm.tail_D && (uint32_t)l < r && tl >= prm.tail_lo && tl < prm.tail_hi)
          prm.tail_D[tl - prm.tail_lo] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(uint64_t)src,
                                                    (uint32_t)((uint64_t)src >> 32));
      }
      olen += (uint64_t)SEG * r;
      i += 10u * r;
      ndecl += r;                                            // window_.declare, :160
      if (stop) { st = 1; break; }
    } else if (op == OP_BACKREF) {                           // :165-181
      if (len - i < 3u) { st = 3; break; }
      if (EMIT) {
        if (spos(chunk, i) >= blockp) { st = -1; i += 3; break; }   // empty slot: moveout precedes the check
        uint64_t h = 0, gd = 0;
        const uint8_t* src = nullptr;
        if (!window_slot(prm, dbase + ndecl, x[i + 2], h, src, gd)) { st = -1; i += 3; break; }
        wave_copy2048(out + olen, src);
      }
      ++nbref;
      olen += SEG;
      i += 3;
    } else {
      st = -1;                                               // :183-184 unsupported opcode
      break;
    }
  }
  if (l == 0) {
    prm.out_len[chunk] = olen;
    if (EMIT) {
      prm.chunk_status[chunk] = st;
      prm.consumed[chunk] = i;
      prm.n_decl_emit[chunk] = ndecl;
    } else {
      prm.n_decl[chunk] = ndecl;
      prm.n_bref[chunk] = nbref;
    }
  }
}

// Declare records for batch indices [lo_t, hi_t): full (every declare, when
// the batch holds BACKREFs) or tail (the 256 before the stop point, for the
// window update).  One wave per chunk.
__global__ __launch_bounds__(256) void decl_record_kernel(DecParams prm, uint64_t total) {
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t chunk = blockIdx.x * 4u + (uint32_t)wv;
  if (chunk >= prm.n) return;
  const uint64_t hi_t = prm.D_tail ? readfirst64(*prm.t_end) : total, lo_t = d_lo_of(prm);
  const uint64_t base = prm.decl_base[chunk], cnt = prm.n_decl[chunk];
  if (base >= hi_t || base + cnt <= lo_t) return;
  const uint8_t* x = prm.in + prm.chunk_off[chunk];
  const uint32_t len = prm.chunk_len[chunk];
  uint64_t t = base;
  uint32_t i = 0;
  while (i < len && t < hi_t) {
    uint32_t nesc = 0;
    i = next_op(x, i, len, nesc);
    if (i + 1 >= len) break;
    const uint32_t op = x[i + 1];
    if (op == OP_EXTRACT) {
      if (len - i < 2u + SEG) break;
      if (t >= lo_t) {
        const uint2 h = dec_window_hash(x + i + 2);
        const uint64_t src = (uint64_t)(x + i + 2);
        if (lane_id() == 0) prm.D[t - lo_t] = make_uint4(readfirst(h.x), readfirst(h.y), (uint32_t)src, (uint32_t)(src >> 32));
      }
      ++t;
      i += 2 + SEG;
    } else if (op == OP_REF) {
      if (len - i < 10u) break;
      uint64_t h, here;
      const uint32_t r = ref_run(x, i, len, chunk, ~0ull, h, here);
      const uint64_t tl = t + (uint64_t)lane_id();
      if ((uint32_t)lane_id() < r && tl >= lo_t && tl < hi_t) {
        const uint64_t src = (uint64_t)ref_source_t(prm, (uint32_t)h, (uint32_t)(h >> 32), here);
        prm.D[tl - lo_t] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)src, (uint32_t)(src >> 32));
      }
      t += r;
      i += 10u * r;
    } else if (op == OP_BACKREF) {
      if (len - i < 3u) break;
      i += 3;
    } else {
      break;
    }
  }
}

// Invalid BACKREFs (empty window slot): the first one stops the stream.
__global__ __launch_bounds__(256) void decode_brefcheck_kernel(DecParams prm) {
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t chunk = blockIdx.x * 4u + (uint32_t)wv;
  if (chunk >= prm.n || prm.n_bref[chunk] == 0) return;
  const uint8_t* x = prm.in + prm.chunk_off[chunk];
  const uint32_t len = prm.chunk_len[chunk];
  uint64_t t = prm.decl_base[chunk];
  uint32_t i = 0;
  while (i < len) {
    uint32_t nesc = 0;
    i = next_op(x, i, len, nesc);
    if (i + 1 >= len) break;
    const uint32_t op = x[i + 1];
    if (op == OP_EXTRACT) {
      if (len - i < 2u + SEG) break;
      ++t;
      i += 2 + SEG;
    } else if (op == OP_REF) {
      if (len - i < 10u) break;
      ++t;
      i += 10;
    } else if (op == OP_BACKREF) {
      if (len - i < 3u) break;
      uint64_t h = 0, gd = 0;
      const uint8_t* src = nullptr;
      if (!window_slot(prm, t, x[i + 2], h, src, gd)) {
        if (lane_id() == 0) atomicMin((unsigned long long*)prm.berr_pos, (unsigned long long)spos(chunk, i));
        break;
      }
      i += 3;
    } else {
      break;
    }
  }
}

// Declares before the stop point (the first unknown REF or invalid BACKREF).
__global__ void decode_tend_kernel(DecParams prm, uint64_t total) {
  const uint64_t stop = min(*prm.block_pos, *prm.berr_pos);
  *prm.t_end = stop == ~0ull ? total : prm.decl_base[stop >> 32] + prm.n_decl_emit[stop >> 32];
}

// The window after the batch: slot c as window_slot() sees it at t_end, with
// the bytes copied in (the window holds its own reference to them).  One wave
// per slot; every source is batch input or pool, never another slot.
__global__ __launch_bounds__(256) void window_update_kernel(DecParams prm) {
  const uint32_t c = blockIdx.x * 4u + (uint32_t)readfirst(threadIdx.x >> 6);
  if (c >= 256u) return;
  const uint64_t T = readfirst64(*prm.t_end);
  if (T == 0) return;
  uint64_t h = 0, gd = 0;
  const uint8_t* src = nullptr;
  const bool ok = window_slot(prm, T, c, h, src, gd);
  const uint64_t G = prm.win_count + T;
  const bool written = ((G - 1u - c) & 255u) <= G - 1u;
  if (!written) return;
  if (!ok) {
    if (lane_id() == 0) prm.win_hash[c] = 0;
    return;
  }
  if (gd >= prm.win_count) wave_copy2048(prm.win_seg + (uint64_t)c * SEG, src);
  if (lane_id() == 0) prm.win_hash[c] = h;
}

// Between scan and emit: find unresolvable REFs (no earlier EXTRACT of the
// hash in the batch, not in the cache) and the first such stream position.
// One wave per chunk; walks only the op headers.
__global__ __launch_bounds__(256) void decode_refcheck_kernel(DecParams prm) {
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t chunk = blockIdx.x * 4u + (uint32_t)wv;
  if (chunk >= prm.n) return;
  const uint8_t* x = prm.in + prm.chunk_off[chunk];
  const uint32_t len = prm.chunk_len[chunk];
  uint32_t i = 0;
  while (i < len) {
    uint32_t nesc = 0;
    i = next_op(x, i, len, nesc);
    if (i + 1 >= len) break;
    const uint32_t op = x[i + 1];
    if (op == OP_EXTRACT) {
      if (len - i < 2u + SEG) break;
      i += 2 + SEG;
    } else if (op == OP_REF) {
      if (len - i < 10u) break;
      uint64_t h, here;
      const uint32_t r = ref_run(x, i, len, chunk, ~0ull, h, here);
      if ((uint32_t)lane_id() < r) {
        const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
        const uint64_t e = tab_lookup_t(prm.x, lo, hi);
        bool ok = e != ~0ull && e < here;
        if (!ok) ok = g_live(prm, tab_lookup_t(prm.g, lo, hi), here);
        if (!ok) {
          atomicMin((unsigned long long*)prm.block_pos, (unsigned long long)here);
          // decode_skim's set (xcodec_decoder.cc:196-272): each unknown hash once
          // (u: open-addressed set of 2 * unknown_cap slots); past the cap the
          // count keeps growing and xcg_decode_batch reports XCG_EOVERFLOW.
          if (uset_insert(prm.u_keys, prm.u_mask, h)) {
            const uint32_t k = atomicAdd(prm.nunknown, 1u);
            if (k < prm.unknown_cap) {
              prm.unknown[k] = h;
              prm.unknown_pos[k] = here;
            }
          }
        }
      }
      i += 10u * r;
    } else if (op == OP_BACKREF) {
      if (len - i < 3u) break;
      i += 3;
    } else {
      break;
    }
  }
}

// Exclusive scan of n u64 lengths (single workgroup).  Tiles of 4096: each
// thread loads four consecutive lengths (coalesced), scans them, the block
// scans the 1024 partial sums in LDS, and a running carry joins the tiles --
// a handful of load round trips instead of one per element per thread.
__global__ __launch_bounds__(1024) void exclusive_scan_kernel(const uint64_t* len, uint64_t* off, uint32_t n,
                                                             uint64_t* total) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  uint64_t carry = 0;
  for (uint32_t base = 0; base < n; base += 4096) {
    const uint32_t i0 = base + 4 * t;
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i0 + k < n ? len[i0 + k] : 0u;
    const uint64_t s = v[0] + v[1] + v[2] + v[3];
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
      const uint64_t u = t >= d ? part[t - d] : 0u;
      __syncthreads();
      part[t] += u;
      __syncthreads();
    }
    uint64_t run = carry + part[t] - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < n) off[i0 + k] = run;
      run += v[k];
    }
    carry += part[1023];
    __syncthreads();
  }
  if (t == 0) *total = carry;
}

// Commit: every batch EXTRACT hash whose latest occurrence precedes the
// blocking point enters the cache (enter, or replace on name reuse).
// A block takes 256 batch-table slots: one thread per slot decides (enter /
// replace / skip), new segments are numbered by a block count (one global
// atomic per block), then the block's waves copy the segments.
__global__ __launch_bounds__(256) void decode_commit_kernel(DecParams prm, uint8_t* pool, uint32_t* nseg,
                                                            uint32_t seg_cap, FiltSet fs) {
  __shared__ uint32_t s_cnt, s_base, s_njob, s_rest;
  __shared__ uint4 s_job[256];   // (slot, destination segment, kind, -)
  const uint64_t w = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint64_t blockp = min(*prm.block_pos, *prm.berr_pos);
  int kind = 0;                  // 0 none, 1 enter, 2 replace
  uint64_t gv = ~0ull;
  uint64_t key = EMPTY_KEY;
  if (w <= prm.x.mask) {
    key = prm.x.keys[w];
    if (key != EMPTY_KEY) {
      const uint64_t first = prm.x.vals[w], last = prm.x_latest[w];
      if (first < blockp) {                      // else never reached
        if (last >= blockp && last != first) {   // several EXTRACTs straddle the block: not modelled
          atomicOr(prm.status, 1 << 9);
        } else {
          gv = tab_lookup_t(prm.g, (uint32_t)key, (uint32_t)(key >> 32));
          kind = gv != ~0ull ? 2 : 1;
        }
      }
    }
  }
  const uint32_t seg = block_alloc_segs(kind == 1, nseg, &s_cnt, &s_base);
  if (threadIdx.x == 0) { s_njob = 0; s_rest = 0; }
  __syncthreads();
  if (kind == 1 && seg >= seg_cap) {
    atomicOr(prm.status, 4);
    kind = 0;
  }
  if (kind == 1) {
    const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
    if (!tab_insert_min(prm.g, lo, hi, seg)) atomicOr(prm.status, 2);
    filt_insert(fs, lo, hi);
  }
  if (kind) {
    const uint32_t j = atomicAdd(&s_njob, 1u);
    s_job[j] = make_uint4((uint32_t)w, kind == 1 ? seg : (uint32_t)gv, (uint32_t)kind, 0u);
  }
  __syncthreads();
  const uint32_t njob = s_njob;
  const uint32_t wv = readfirst(threadIdx.x >> 6);
  const int l = lane_id();
  // Plain enters (one EXTRACT of the hash, not cached): four of the wave's
  // segments loaded together, then stored (one round trip per four copies
  // instead of one per copy); everything else one job at a time below.
  bool rest = false;
  for (uint32_t j0 = 4u * wv; j0 < njob; j0 += 16u) {
    u32x4 v[4][2];
    uint8_t* dst[4];
    bool plain[4];
    uint64_t first[4], last[4], coff[4];
    uint4 jb[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {                  // (the four jobs' table reads in flight together)
      const uint32_t j = min(j0 + (uint32_t)t, njob - 1u);
      jb[t] = s_job[j];
      const uint32_t slot = readfirst(jb[t].x);
      first[t] = prm.x.vals[slot];
      last[t] = prm.x_latest[slot];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) coff[t] = prm.chunk_off[readfirst64(last[t]) >> 32];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint64_t f = readfirst64(first[t]), la = readfirst64(last[t]);
      plain[t] = j0 + (uint32_t)t < njob && readfirst(jb[t].z) == 1u && la == f;
      if (j0 + (uint32_t)t < njob && !plain[t]) rest = true;
      dst[t] = pool + (uint64_t)readfirst(jb[t].y) * SEG;
      const uint8_t* src = prm.in + readfirst64(coff[t]) + (uint32_t)la;
      if (plain[t]) {
        v[t][0] = *(const u32x4_u*)(src + 32 * l);
        v[t][1] = *(const u32x4_u*)(src + 32 * l + 16);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (plain[t]) {
        *(u32x4_u*)(dst[t] + 32 * l) = v[t][0];
        *(u32x4_u*)(dst[t] + 32 * l + 16) = v[t][1];
      }
  }
  if (rest && l == 0) s_rest = 1u;
  __syncthreads();
  if (s_rest == 0u) return;
  for (uint32_t j = wv; j < njob; j += 4) {
    const uint4 jb = s_job[j];
    const uint32_t slot = readfirst(jb.x), dseg = readfirst(jb.y), jkind = readfirst(jb.z);
    const uint64_t first = readfirst64(prm.x.vals[slot]), last = readfirst64(prm.x_latest[slot]);
    if (jkind == 1u && last == first) continue;   // (copied above)
    const uint8_t* src = prm.in + prm.chunk_off[last >> 32] + (uint32_t)last;
    if (last != first) {
      // name reuse inside the batch with different bytes would need per-REF
      // resolution of the latest EXTRACT; the emit pass used the earliest.
      const uint8_t* s0 = prm.in + prm.chunk_off[first >> 32] + (uint32_t)first;
      if (!readfirst((uint32_t)dec_equal2048(s0, src)) && lane_id() == 0) atomicOr(prm.status, 1 << 9);
    }
    uint8_t* dst = pool + (uint64_t)dseg * SEG;
    if (jkind == 1 || !readfirst((uint32_t)dec_equal2048(dst, src))) wave_copy2048(dst, src);   // enter / replace (:130)
  }
}

// ------------------------------------------------ bounded cache (xcg_lru.hip)

// Every EXTRACT / REF op of the batch as (lo, hi, op offset, op), packed by
// chunk at decl_base[c] (the scan's declare numbering).  One wave per chunk.
__global__ __launch_bounds__(256) void dec_ops_kernel(DecParams prm, uint4* raw) {
  const int wv = (int)readfirst(threadIdx.x >> 6);
  const uint32_t chunk = blockIdx.x * 4u + (uint32_t)wv;
  if (chunk >= prm.n) return;
  const uint8_t* x = prm.in + prm.chunk_off[chunk];
  const uint32_t len = prm.chunk_len[chunk];
  uint64_t t = prm.decl_base[chunk];
  uint32_t i = 0;
  while (i < len) {
    uint32_t nesc = 0;
    i = next_op(x, i, len, nesc);
    if (i + 1 >= len) break;
    const uint32_t op = x[i + 1];
    if (op == OP_EXTRACT) {
      if (len - i < 2u + SEG) break;
      const uint2 h = dec_window_hash(x + i + 2);
      if (lane_id() == 0) raw[t] = make_uint4(readfirst(h.x), readfirst(h.y), i, OP_EXTRACT);
      ++t;
      i += 2 + SEG;
    } else if (op == OP_REF) {
      if (len - i < 10u) break;
      uint64_t h, here;
      const uint32_t r = ref_run(x, i, len, chunk, ~0ull, h, here);
      if ((uint32_t)lane_id() < r) raw[t + lane_id()] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)here, OP_REF);
      t += r;
      i += 10u * r;
    } else if (op == OP_BACKREF) {
      if (len - i < 3u) break;
      i += 3;
    } else {
      break;
    }
  }
}

// What each op does to the bounded cache, given the eviction times (ptime)
// and the stop point of the last pass (blockp): an EXTRACT looks its hash up
// (xcodec_decoder.cc:106-136): an earlier EXTRACT of the batch (HIT), a live
// persistent entry (GHIT: use, replace if the bytes differ) or an ENTER; a
// REF (:141-163) hits likewise or is unknown -- the stream stops at the first
// one.  After the stop point decode_skim (:196-272) still looks up every REF
// (a hit refreshes the entry) against the cache as it stands there.
// ev[decl_base[c] + k]: (lo, hi, op offset, kind << 30 | ref) with GMISS =
// no cache effect; ENTERs also as declaration rows.  One wave per chunk.
//
// PAIR (XCodecCachePair, xcg_pair.hip): ptime is the time a hash leaves both
// levels.  A skim lookup can promote a disk-only hash and so evict another
// (xcodec_cache.h:223-227), so each skim lookup sees the pair at its own time,
// not at the stop.  An EXTRACT whose cached bytes differ is a REPLACE (op
// offset | 1 << 31, GHIT): it takes a declaration row like an ENTER (the new
// bytes' source), numbered with the ENTERs in op order.
template <bool PAIR>
__global__ __launch_bounds__(256) void dec_classify_kernel(DecParams prm, const uint4* raw, uint4* ev, uint32_t* nev,
                                                           uint4* drow, uint32_t* ndecl, uint32_t maxd,
                                                           uint64_t blockp, uint64_t* block_new, uint32_t* changes,
                                                           int first) {
  const uint32_t c = blockIdx.x * 4u + (uint32_t)readfirst(threadIdx.x >> 6);
  if (c >= prm.n) return;
  const uint32_t cnt = (uint32_t)prm.n_decl[c];
  const uint64_t base = prm.decl_base[c];
  const uint64_t tb = blockp == ~0ull ? ~0ull : ((blockp >> 32 << 21) | (uint32_t)blockp);
  const uint8_t* x = prm.in + prm.chunk_off[c];
  uint32_t nd = 0;
  bool chg = false;
  for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
    const uint32_t k = k0 + (uint32_t)lane_id();
    const bool valid = k < cnt;
    uint4 r = valid ? raw[base + k] : make_uint4(0u, 0u, 0u, 0u);
    const uint64_t here = spos(c, r.z), t = ((uint64_t)c << 21) | r.z;
    uint32_t kind = EV_GMISS, ref = 0, zflag = 0;
    bool enter = false;
    if (valid) {
      const uint64_t e = tab_lookup_t(prm.x, r.x, r.y);
      if (here <= blockp) {                           // (the op at the stop point is looked at again)
        if (e != ~0ull && e < here) {
          kind = EV_HIT;
        } else {
          const uint64_t gv = tab_lookup_t(prm.g, r.x, r.y);
          if (gv != ~0ull && t < prm.ptime[gv]) {
            kind = EV_GHIT;
            ref = (uint32_t)gv;
            if (PAIR && r.w == OP_EXTRACT) {          // name reuse: the cached bytes differ
              const u32x4_u* a = (const u32x4_u*)(x + r.z + 2);
              const u32x4_u* b = (const u32x4_u*)(prm.pool + gv * (uint64_t)SEG);
              bool same = true;
              for (uint32_t q = 0; q < SEG / 16 && same; ++q) {
                const u32x4 va = a[q], vb = b[q];
                same = va[0] == vb[0] && va[1] == vb[1] && va[2] == vb[2] && va[3] == vb[3];
              }
              if (!same) {
                zflag = 1u << 31;
                enter = true;                         // (a declaration row; the kind stays GHIT)
              }
            }
          } else if (r.w == OP_EXTRACT) {
            enter = true;
          } else {
            atomicMin((unsigned long long*)block_new, (unsigned long long)here);   // unknown REF
          }
        }
      } else if (r.w == OP_REF) {                     // decode_skim's lookup
        if (e != ~0ull && e < blockp) {
          kind = EV_HIT;
        } else {
          const uint64_t gv = tab_lookup_t(prm.g, r.x, r.y);
          if (gv != ~0ull && (PAIR ? t : tb) < prm.ptime[gv]) {
            kind = EV_GHIT;
            ref = (uint32_t)gv;
          }
        }
      }
    }
    const uint64_t m = ballot(enter);
    if (enter) {
      const uint32_t d = nd + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (!zflag) {
        kind = EV_ENTER;
        ref = d;
      }
      if (d < maxd) drow[(uint64_t)c * maxd + d] = make_uint4(r.x, r.y, r.z + 2u, 0u);
    }
    nd += (uint32_t)__builtin_popcountll(m);
    if (valid) {
      const uint32_t w = (kind << 30) | ref;
      const uint4 old = ev[base + k];
      chg |= first || old.w != w || old.z != (r.z | zflag);
      ev[base + k] = make_uint4(r.x, r.y, r.z | zflag, w);
    }
  }
  if (ballot(chg) != 0 && lane_id() == 0) atomicAdd(changes, 1u);
  if (lane_id() == 0) {
    nev[c] = cnt;
    ndecl[c] = nd;
    if (nd > maxd) atomicOr(prm.status, 1 << 11);
  }
}

// EXTRACTs that looked up a live entry: replace its bytes if they differ
// (XCodecMemoryCache::replace, :130); a second EXTRACT of a hash in the batch
// with other bytes is the name reuse the batch decoder does not model (bit 9).
__global__ __launch_bounds__(256) void dec_replace_kernel(DecParams prm, const uint4* raw, const uint4* ev,
                                                          uint8_t* pool) {
  const uint32_t c = blockIdx.x * 4u + (uint32_t)readfirst(threadIdx.x >> 6);
  if (c >= prm.n) return;
  const uint32_t cnt = (uint32_t)prm.n_decl[c];
  const uint64_t base = prm.decl_base[c];
  const uint8_t* x = prm.in + prm.chunk_off[c];
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint4 e = ev[base + k];
    const uint32_t kind = readfirst(e.w) >> 30;
    if (readfirst(raw[base + k].w) != OP_EXTRACT || (kind != EV_GHIT && kind != EV_HIT)) continue;
    const uint8_t* src = x + readfirst(e.z) + 2;
    if (kind == EV_GHIT) {
      uint8_t* dst = pool + (uint64_t)(readfirst(e.w) & EV_REF_MASK) * SEG;
      if (!dec_equal2048(dst, src)) wave_copy2048(dst, src);
    } else {
      const uint64_t first = tab_lookup(prm.x, readfirst(e.x), readfirst(e.y));
      const uint8_t* s0 = prm.in + prm.chunk_off[first >> 32] + (uint32_t)first;
      if (!dec_equal2048(s0, src) && lane_id() == 0) atomicOr(prm.status, 1 << 9);
    }
  }
}

// Before anything is emitted or committed: batch EXTRACTs of one hash that
// the batch decoder cannot model -- a second EXTRACT with other bytes (name
// reuse; REFs between them would need the latest bytes, the emit pass uses the
// earliest), or EXTRACTs on both sides of the stop point.  Status bit 9 makes
// xcg_decode_batch refuse the batch (XCG_ENOTSUP) with the cache, window and
// outputs untouched.  One thread per batch-table slot; the byte compare is rare.
__global__ __launch_bounds__(256) void dec_precheck_kernel(DecParams prm) {
  const uint64_t w = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (w > prm.x.mask) return;
  const uint64_t key = prm.x.keys[w];
  if (key == EMPTY_KEY) return;
  const uint64_t first = prm.x.vals[w], last = prm.x_latest[w];
  const uint64_t blockp = min(*prm.block_pos, *prm.berr_pos);
  if (first >= blockp || last == first) return;
  bool bad = last >= blockp;
  if (!bad) {
    const uint8_t* a = prm.in + prm.chunk_off[first >> 32] + (uint32_t)first;
    const uint8_t* b = prm.in + prm.chunk_off[last >> 32] + (uint32_t)last;
    for (uint32_t k = 0; k < SEG && !bad; ++k) bad = a[k] != b[k];
  }
  if (bad) atomicOr(prm.status, 1 << 9);
}

// Pack per-chunk output slots into one contiguous buffer (one wave per chunk).
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                                                   const uint64_t* dst_off, uint8_t* dst, uint32_t n) {
  const uint32_t c = blockIdx.x * 4u + (uint32_t)readfirst(threadIdx.x >> 6);
  if (c >= n) return;
  const uint8_t* s = src + src_off[c];
  uint8_t* d = dst + dst_off[c];
  const uint64_t m = len[c];
  const int l = lane_id();
  for (uint64_t base = 0; base < m; base += 1024) {
    const uint64_t off = base + 16u * l;
    if (off + 16 <= m) *(u32x4_u*)(d + off) = *(const u32x4_u*)(s + off);
    else for (uint64_t k = off; k < m; ++k) d[k] = s[k];
  }
}

// ---------------------------------------- one decode() call, one workgroup
//
// XCodecDecoder::decode (xcodec/xcodec_decoder.cc:66-272) of ONE call's input
// on an unbounded cache, as the drop-in adapter issues it (tack -d: one call
// per 64 KiB read, programs/tack/tack.cc:329-359; XCodecPipePair: the buffered
// frames, xcodec_pipe_pair.cc:425-446) -- the passes of the batch decoder
// (scan, hash, resolve, emit, window, commit) in one launch, with __syncthreads
// between them instead of kernel boundaries and host synchronisations.
// Wave 0 walks the ops and lists them (literal runs, EXTRACT, REF) with their
// output offsets and declare numbers; all waves hash the EXTRACTs into an LDS
// table (earliest / latest position), resolve every REF (an earlier EXTRACT
// of the call, else the cache; else it is unknown -- the first one is the stop
// point and the rest form decode_skim's set), then copy every op before the
// stop to its output offset, update the BACKREF window (window_slot over the
// call's declare records) and commit the EXTRACTs before the stop.  Anything
// the batch decoder refuses or this pass does not cover -- a BACKREF op, name
// reuse inside the call, EXTRACTs on both sides of the stop, more than
// SD_XSLOTS / 2 EXTRACTs or SD_UMAX unknown hashes -- sets `fallback` before
// anything is written; the host then takes the batch path.
constexpr uint32_t SD_XSLOTS = 2048, SD_USLOTS = 4096, SD_UMAX = 2048, SD_EMAX = 1024;
// A call's input up to this size is staged in LDS first (with the tables:
// 80 KiB + 78 KiB of the 160 KiB): the op walk is a chain of dependent reads,
// one per op, that would each wait on HBM.
constexpr uint32_t SD_LDS_IN = 76000;
constexpr uint32_t SD_LIT = 0, SD_EXT = 1, SD_REF = 2;

struct SmallDec {
  const uint8_t* in;
  uint32_t len;
  HashTab g;
  uint8_t* pool;
  uint32_t* nseg;
  uint32_t seg_cap;
  FiltSet fs;
  int32_t* status;             // the context's sticky word
  uint4* ops;                  // (type, in_off, out_off, declare number | nesc)
  uint64_t* opv;               // EXTRACT / REF hash
  uint4* D;                    // declare records (lo, hi, src lo, src hi)
  uint32_t ops_cap;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* win_hash;
  uint8_t* win_seg;
  uint64_t win_count;
  uint64_t* res;               // [0] out_len [1] consumed [2] status [3] declares before the stop
                               // [4] unknowns [5] fallback [6] EXTRACTs before the stop [7] decoded size
                               // then SD_UMAX unknown hashes, then SD_EMAX EXTRACT hashes (op order),
                               // then the context's sticky word
  uint64_t* tim;               // (diagnostics, nullable) SD_PHASES clock stamps at the phase boundaries
  uint32_t* flag;              // (nullable) completion word in host memory: seq is stored there last
  uint32_t seq;
};
constexpr uint32_t SD_PHASES = 11;
#define SD_STAMP(k) do { if (a.tim && threadIdx.x == 0) a.tim[k] = __builtin_amdgcn_s_memrealtime(); } while (0)

__device__ __forceinline__ void decode_small_body(const SmallDec& a) {
  __shared__ uint64_t xk[SD_XSLOTS], xf[SD_XSLOTS], xl[SD_XSLOTS];
  __shared__ uint64_t uk[SD_USLOTS];
  __shared__ uint32_t s_nops, s_ndecl, s_next, s_nunk, s_fb, s_walk_st, s_walk_end;
  __shared__ uint64_t s_stop;  // (position << 32) | declare number of the first unknown REF
  __shared__ uint64_t s_olen;
  __shared__ uint4 xin[SD_LDS_IN / 16];
  __shared__ uint16_t xlist[SD_XSLOTS / 2];                  // the occupied EXTRACT slots
  __shared__ uint16_t wcopy[256];                            // window slots that take a new segment
  __shared__ uint32_t s_nx, s_nw;
  const uint32_t t = threadIdx.x, w = t >> 6;
  const int l = lane_id();
  const uint32_t len = a.len;
  const uint8_t* x = a.in;
  SD_STAMP(0);
  const bool staged = len <= SD_LDS_IN;
  constexpr uint32_t SV = (SD_LDS_IN / 16 + 1023) / 1024;    // 16-byte loads per thread
  if (staged) {                                              // stage the input (all loads in flight together)
    const uint32_t nv = len / 16;
    uint4 v[SV];
#pragma unroll
    for (uint32_t j = 0; j < SV; ++j)
      if (t + 1024u * j < nv) v[j] = ((const uint4*)a.in)[t + 1024u * j];
#pragma unroll
    for (uint32_t j = 0; j < SV; ++j)
      if (t + 1024u * j < nv) xin[t + 1024u * j] = v[j];
    uint8_t* xb = (uint8_t*)xin;
    for (uint32_t i = nv * 16 + t; i < len; i += 1024) xb[i] = a.in[i];
    x = xb;
  }
  const lds_u8p xs = (lds_u8p)(const uint8_t*)xin;
  for (uint32_t i = t; i < SD_XSLOTS; i += 1024) { xk[i] = EMPTY_KEY; xf[i] = ~0ull; xl[i] = 0; }
  for (uint32_t i = t; i < SD_USLOTS; i += 1024) uk[i] = EMPTY_KEY;
  if (t == 0) {
    s_nunk = 0; s_fb = 0; s_stop = ~0ull; s_next = 0;
    a.res[8 + SD_UMAX + SD_EMAX] = (uint64_t)(uint32_t)*a.status;   // (the paths that return early)
  }
  // (wave 0's walk reads input bytes every wave staged)
  __syncthreads();
  SD_STAMP(1);
  // ---- walk (wave 0): op list, output offsets, declare numbers
  auto walk = [&](auto xp) {
    uint32_t i = 0, k = 0, dn = 0, st = 0, fb = 0;
    uint64_t olen = 0;
    while (i < len) {
      uint32_t nesc = 0;
      const uint32_t m = next_op(xp, i, len, nesc);
      if (m > i) {                                           // literal run (:71-81, ESCAPE :91-94)
        if (k >= a.ops_cap) { fb = 1; break; }
        if (l == 0) a.ops[k] = make_uint4(SD_LIT, i, (uint32_t)olen, m - i);
        ++k;
        olen += (m - i) - nesc;
      }
      i = m;
      if (i >= len) break;
      if (len - i == 1) { st = 3; break; }
      const uint32_t op = xp[i + 1];
      if (op == OP_EXTRACT) {
        if (len - i < 2u + SEG) { st = 3; break; }
        if (k >= a.ops_cap) { fb = 1; break; }
        if (l == 0) a.ops[k] = make_uint4(SD_EXT, i, (uint32_t)olen, dn);
        ++k; ++dn;
        olen += SEG;
        i += 2 + SEG;
      } else if (op == OP_REF) {
        if (len - i < 10u) { st = 3; break; }
        uint64_t h, here;
        const uint32_t r = ref_run(xp, i, len, 0, ~0ull, h, here);
        if (k + r > a.ops_cap) { fb = 1; break; }
        if ((uint32_t)l < r) {
          a.ops[k + l] = make_uint4(SD_REF, i + 10u * l, (uint32_t)(olen + (uint64_t)SEG * l), dn + l);
          a.opv[k + l] = h;
        }
        k += r; dn += r;
        olen += (uint64_t)SEG * r;
        i += 10u * r;
      } else if (op == OP_BACKREF) {
        fb = 1;                                              // (the batch path models the window's BACKREFs)
        break;
      } else {
        st = (uint32_t)-1;                                   // :183-184 unsupported opcode
        break;
      }
    }
    if (olen >= (1ull << 32)) fb = 1;
    if (l == 0) {
      s_nops = k; s_ndecl = dn; s_walk_st = st; s_walk_end = i; s_olen = olen;
      if (fb) s_fb = 1;
    }
  };
  if (w == 0) {
    if (staged) walk(xs);
    else walk(a.in);
  }
  __syncthreads();
  SD_STAMP(2);
  const uint32_t nops = s_nops;
  if (s_fb) {
    if (t == 0) a.res[5] = 1;
    return;
  }
  // ---- EXTRACT hashes (a wave per EXTRACT) into the LDS table
  for (uint32_t k = w; k < nops; k += 16) {
    const uint4 o = a.ops[k];
    if (readfirst(o.x) != SD_EXT) continue;
    const uint32_t pos = readfirst(o.y) + 2u;
    const uint2 h = staged ? dec_window_hash(xs + pos) : dec_window_hash(x + pos);
    const uint64_t key = ((uint64_t)readfirst(h.y) << 32) | readfirst(h.x);
    if (l == 0) {
      a.opv[k] = key;
      uint32_t i = mix32((uint32_t)key, (uint32_t)(key >> 32)) & (SD_XSLOTS - 1);
      for (uint32_t n = 0; n < SD_XSLOTS; ++n) {
        const uint64_t prev = atomicCAS((unsigned long long*)&xk[i], (unsigned long long)EMPTY_KEY, (unsigned long long)key);
        if (prev == EMPTY_KEY || prev == key) {
          atomicMin((unsigned long long*)&xf[i], (unsigned long long)pos);
          atomicMax((unsigned long long*)&xl[i], (unsigned long long)pos);
          break;
        }
        i = (i + 1) & (SD_XSLOTS - 1);
      }
      atomicAdd(&s_next, 1u);
    }
  }
  if (t == 0) { s_nx = 0; s_nw = 0; }
  __syncthreads();
  SD_STAMP(3);
  if (s_next > SD_XSLOTS / 2) {
    if (t == 0) a.res[5] = 1;
    return;
  }
  // occupied slots of the EXTRACT table, once (the precheck and the commit walk
  // only these instead of all SD_XSLOTS)
  for (uint32_t i = t; i < SD_XSLOTS; i += 1024)
    if (xk[i] != EMPTY_KEY) xlist[atomicAdd(&s_nx, 1u)] = (uint16_t)i;
  // ---- resolve every REF (a thread per op): an earlier EXTRACT of the call,
  // else the cache; else unknown (:151-156; decode_skim's set, :196-272)
  for (uint32_t k = t; k < nops; k += 1024) {
    const uint4 o = a.ops[k];
    uint64_t src = 0, key = 0;
    if (o.x == SD_EXT) {
      key = a.opv[k];
      src = (uint64_t)(x + o.y + 2);
    } else if (o.x == SD_REF) {
      key = a.opv[k];
      const uint64_t here = o.y;
      uint32_t i = mix32((uint32_t)key, (uint32_t)(key >> 32)) & (SD_XSLOTS - 1);
      uint64_t e = ~0ull;
      for (uint32_t n = 0; n < SD_XSLOTS; ++n) {
        const uint64_t kk = xk[i];
        if (kk == key) { e = xf[i]; break; }
        if (kk == EMPTY_KEY) break;
        i = (i + 1) & (SD_XSLOTS - 1);
      }
      if (e != ~0ull && e < here) {
        src = (uint64_t)(x + e);
      } else {
        const uint64_t gv = tab_lookup_t(a.g, (uint32_t)key, (uint32_t)(key >> 32));
        if (gv != ~0ull) {
          src = (uint64_t)(a.pool + gv * (uint64_t)SEG);
        } else {
          atomicMin((unsigned long long*)&s_stop, (unsigned long long)((here << 32) | o.w));
          uint32_t j = mix32((uint32_t)key, (uint32_t)(key >> 32)) & (SD_USLOTS - 1);
          for (uint32_t n = 0; n < SD_USLOTS; ++n) {
            const uint64_t prev = atomicCAS((unsigned long long*)&uk[j], (unsigned long long)EMPTY_KEY,
                                            (unsigned long long)key);
            if (prev == EMPTY_KEY) {
              const uint32_t u = atomicAdd(&s_nunk, 1u);
              if (u < SD_UMAX) a.res[8 + u] = key;
              break;
            }
            if (prev == key) break;
            j = (j + 1) & (SD_USLOTS - 1);
          }
        }
      }
    }
    if (o.x != SD_LIT) a.D[o.w] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), (uint32_t)src, (uint32_t)(src >> 32));
  }
  __syncthreads();
  SD_STAMP(4);
  const uint64_t stop = s_stop;
  const uint32_t stop_pos = stop == ~0ull ? ~0u : (uint32_t)(stop >> 32);
  const uint32_t T = stop == ~0ull ? s_ndecl : (uint32_t)stop;   // declares before the stop
  if (s_nunk > SD_UMAX) {
    if (t == 0) a.res[5] = 1;
    return;
  }
  // ---- what the batch decoder refuses (dec_precheck_kernel): several EXTRACTs
  // of one hash before the stop with other bytes, or on both sides of it
  const uint32_t nx = s_nx;
  for (uint32_t q = w; q < nx; q += 16) {
    const uint32_t i = xlist[q];
    const uint64_t f = xf[i], z = xl[i];
    if (f >= stop_pos || z == f) continue;
    bool bad = z >= stop_pos;
    if (!bad) bad = !dec_equal2048(x + f, x + z);
    if (bad && l == 0) atomicOr(&s_fb, 1u);
  }
  __syncthreads();
  SD_STAMP(5);
  if (s_fb) {
    if (t == 0) a.res[5] = 1;
    return;
  }
  // ---- output: every op before the stop at its offset (a wave per op); the
  // output ends at the stop REF's offset
  if (stop != ~0ull)
    for (uint32_t k = t; k < nops; k += 1024) {
      const uint4 o = a.ops[k];
      if (o.x == SD_REF && o.y == stop_pos) s_olen = o.z;
    }
  __syncthreads();
  SD_STAMP(6);
  const uint64_t out_len = s_olen;
  if (out_len > a.out_cap) {
    if (t == 0) { a.res[5] = 2; a.res[7] = out_len; }      // (more room needed; nothing written)
    return;
  }
  for (uint32_t k = w; k < nops; k += 16) {
    const uint4 o = a.ops[k];
    const uint32_t ty = readfirst(o.x), io = readfirst(o.y), oo = readfirst(o.z);
    if (io >= stop_pos) continue;
    if (ty == SD_LIT) {
      (void)wave_unescape(a.out + oo, x, io, io + readfirst(o.w));
    } else {
      const uint4 d = a.D[readfirst(o.w)];
      const uint8_t* src = (const uint8_t*)(((uint64_t)readfirst(d.w) << 32) | readfirst(d.z));
      wave_copy2048(a.out + oo, src);
    }
  }
  if (a.tim) {
    __syncthreads();
    SD_STAMP(7);
  }
  // ---- the BACKREF window after the call's declares (before the commit
  // overwrites any pool bytes a REF's declare reads).  Up to 256 declares: a
  // thread per slot against the call's declared hashes in LDS (uk is free
  // again); only slots this call declares into take a segment; an older slot
  // whose hash the call declares again is emptied (XCodecWindow::declare,
  // xcodec_window.h:68-90).  More declares: window_slot per slot.
  if (T > 0 && T <= 256) {
    for (uint32_t i = t; i < T; i += 1024) {
      const uint4 d = a.D[i];
      uk[i] = ((uint64_t)d.y << 32) | d.x;
    }
    __syncthreads();
    if (t < 256) {
      const uint32_t c = t;
      const uint64_t W = a.win_count, G = W + T;
      const uint64_t r = (G - 1u - c) & 255u;
      if (r <= G - 1u) {                                     // (else never written)
        const uint64_t g = G - 1u - r;
        if (g >= W) {
          const uint32_t tl = (uint32_t)(g - W);
          const uint64_t h = uk[tl];
          bool dup = false;
          for (uint32_t k = tl + 1; k < T; ++k) dup |= uk[k] == h;
          if (dup) {
            a.win_hash[c] = 0;
          } else {
            a.win_hash[c] = h;
            wcopy[atomicAdd(&s_nw, 1u)] = (uint16_t)(c | (tl << 8));   // (tl < 256)
          }
        } else {
          const uint64_t h = a.win_hash[c];
          if (h != 0) {
            bool dup = false;
            for (uint32_t k = 0; k < T; ++k) dup |= uk[k] == h;
            if (dup) a.win_hash[c] = 0;
          }
        }
      }
    }
    __syncthreads();
    for (uint32_t q = w; q < s_nw; q += 16) {
      const uint32_t e = wcopy[q], c = e & 255u, tl = e >> 8;
      const uint4 d = a.D[tl];
      wave_copy2048(a.win_seg + (uint64_t)c * SEG, (const uint8_t*)(((uint64_t)d.w << 32) | d.z));
    }
  } else {
    DecParams prm{};
    prm.D = a.D;
    prm.D_lo = 0;
    prm.D_tail = false;
    prm.win_hash = a.win_hash;
    prm.win_seg = a.win_seg;
    prm.win_count = a.win_count;
    const uint64_t G = a.win_count + T;
    for (uint32_t c = w; c < 256u && T > 0; c += 16) {
      uint64_t h = 0, gd = 0;
      const uint8_t* src = nullptr;
      const bool ok = window_slot(prm, T, c, h, src, gd);
      if (((G - 1u - c) & 255u) > G - 1u) continue;          // never written
      if (!ok) {
        if (l == 0) a.win_hash[c] = 0;
        continue;
      }
      if (gd >= a.win_count) wave_copy2048(a.win_seg + (uint64_t)c * SEG, src);
      if (l == 0) a.win_hash[c] = h;
    }
  }
  __syncthreads();
  SD_STAMP(8);
  // ---- commit: EXTRACTs before the stop enter the cache, or replace a cached
  // segment's bytes (name reuse, :106-136)
  for (uint32_t q = w; q < nx; q += 16) {
    const uint32_t i = xlist[q];
    const uint64_t key = xk[i];
    const uint64_t f = xf[i];
    if (f >= stop_pos) continue;
    const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
    const uint64_t gv = tab_lookup(a.g, lo, hi);
    const uint8_t* src = x + f;
    if (gv != ~0ull) {
      uint8_t* dst = a.pool + gv * (uint64_t)SEG;
      if (!dec_equal2048(dst, src)) wave_copy2048(dst, src);
      continue;
    }
    uint32_t sg = 0;
    if (l == 0) sg = atomicAdd(a.nseg, 1u);
    sg = readfirst(sg);
    if (sg >= a.seg_cap) {
      if (l == 0) atomicOr(a.status, 4);
      continue;
    }
    wave_copy2048(a.pool + (uint64_t)sg * SEG, src);
    if (l == 0) {
      if (!tab_insert_min(a.g, lo, hi, sg)) atomicOr(a.status, 2);
      filt_insert(a.fs, lo, hi);
    }
  }
  if (a.tim) {
    __syncthreads();
    SD_STAMP(9);
  }
  // ---- results: the EXTRACTs before the stop in op order (the host cache's
  // mirror enters them without hashing again)
  if (w == 0) {
    uint32_t ne = 0;
    for (uint32_t k0 = 0; k0 < nops; k0 += 64) {
      const uint32_t k = k0 + (uint32_t)l;
      bool is = false;
      uint64_t key = 0;
      if (k < nops) {
        const uint4 o = a.ops[k];
        is = o.x == SD_EXT && o.y < stop_pos;
        if (is) key = a.opv[k];
      }
      const uint64_t m = ballot(is);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (is && ne + below < SD_EMAX) a.res[8 + SD_UMAX + ne + below] = key;
      ne += (uint32_t)__builtin_popcountll(m);
    }
    if (l == 0) {
      const int32_t wst = (int32_t)s_walk_st;
      a.res[8 + SD_UMAX + SD_EMAX] = (uint64_t)(uint32_t)*a.status;
      a.res[0] = out_len;
      a.res[1] = stop != ~0ull ? stop_pos : s_walk_end;
      a.res[2] = (uint64_t)(int64_t)(stop != ~0ull ? 1 : wst);
      a.res[3] = T;
      a.res[4] = s_nunk;
      a.res[5] = 0;
      a.res[6] = ne;
      a.res[7] = out_len;
    }
  }
  SD_STAMP(10);
}

// The call's input, output and results may live in host memory (the
// zero-copy call path: the input is staged into LDS first, the output and
// results cross PCIe as posted writes); the host then waits on `flag`,
// stored after every other write of the block is visible system-wide.
__global__ __launch_bounds__(1024) void decode_small_kernel(SmallDec a) {
  decode_small_body(a);
  if (a.flag) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Host-driven cache access (one wave): look a hash up and copy its segment
// out, or enter a segment under a hash (XCodecCache::lookup / enter /
// replace, xcodec/xcodec_cache.h:83-89).
__global__ __launch_bounds__(64) void cache_lookup_kernel(HashTab g, const uint8_t* pool, uint64_t key, uint8_t* seg_out,
                                                          int32_t* found) {
  const uint64_t v = tab_lookup(g, (uint32_t)key, (uint32_t)(key >> 32));
  if (v == ~0ull) {
    if (lane_id() == 0) *found = 0;
    return;
  }
  wave_copy2048(seg_out, pool + v * (uint64_t)SEG);
  if (lane_id() == 0) *found = 1;
}

__global__ __launch_bounds__(64) void cache_enter_kernel(HashTab g, uint8_t* pool, uint32_t* nseg, uint32_t seg_cap,
                                                         FiltSet fs, uint64_t key, const uint8_t* seg,
                                                         int replace_only, int32_t* result) {
  const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
  const uint64_t v = tab_lookup(g, lo, hi);
  if (v != ~0ull) {                          // present: replace the bytes
    wave_copy2048(pool + v * (uint64_t)SEG, seg);
    if (lane_id() == 0) *result = 1;
    return;
  }
  if (replace_only) {
    if (lane_id() == 0) *result = -1;
    return;
  }
  uint32_t s = 0;
  if (lane_id() == 0) s = atomicAdd(nseg, 1u);   // single-segment host call: one atomic
  s = readfirst(s);
  if (s >= seg_cap) {
    if (lane_id() == 0) *result = -2;
    return;
  }
  wave_copy2048(pool + (uint64_t)s * SEG, seg);
  if (lane_id() == 0) {
    tab_insert_min(g, lo, hi, s);
    filt_insert(fs, lo, hi);
    *result = 0;
  }
}

}  // namespace xcg

extern "C" int xcg_launch_cache_lookup(uint64_t* keys, uint64_t* vals, uint32_t mask, const uint8_t* pool, uint64_t key,
                                       uint8_t* seg_out, int32_t* found, hipStream_t s) {
  hipLaunchKernelGGL(xcg::cache_lookup_kernel, dim3(1), dim3(64), 0, s, xcg::HashTab{keys, vals, mask}, pool, key,
                     seg_out, found);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int xcg_launch_cache_enter(uint64_t* keys, uint64_t* vals, uint32_t mask, uint8_t* pool, uint32_t* nseg,
                                      uint32_t seg_cap, uint32_t* filt, uint32_t* ftab, uint32_t fmask, uint32_t* gfilt,
                                      uint32_t gmask, uint64_t key, const uint8_t* seg, int replace_only,
                                      int32_t* result, hipStream_t s) {
  hipLaunchKernelGGL(xcg::cache_enter_kernel, dim3(1), dim3(64), 0, s, xcg::HashTab{keys, vals, mask}, pool, nseg,
                     seg_cap, xcg::FiltSet{filt, ftab, fmask, gfilt, gmask}, key, seg, replace_only, result);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int xcg_launch_pack(const uint8_t* src, const uint64_t* src_off, const uint64_t* len, uint32_t n,
                               uint8_t* dst, uint64_t* dst_off, uint64_t* d_total, hipStream_t stream) {
  using namespace xcg;
  if (n == 0) return 0;
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(1024), 0, stream, len, dst_off, n, d_total);
  hipLaunchKernelGGL(pack_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, src, src_off, len, (const uint64_t*)dst_off,
                     dst, n);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

struct XcgDecodeArgs {
  const uint8_t* in;
  const uint64_t* chunk_off;
  const uint32_t* chunk_len;
  uint32_t n;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* out_off;
  uint64_t* out_len;
  int32_t* chunk_status;
  uint64_t* consumed;
  int32_t* status;
  uint64_t* g_keys;
  uint64_t* g_vals;
  uint32_t g_mask;
  uint8_t* pool;
  uint32_t* nseg;
  uint32_t seg_cap;
  uint32_t* g_filt;
  uint32_t* g_ftab;
  uint32_t fmask;
  uint32_t* g_gfilt;
  uint32_t gmask;
  uint64_t* x_keys;
  uint64_t* x_vals;
  uint64_t* x_latest;
  uint32_t x_mask;
  uint64_t* u_keys;      // unknown-hash set, 2 * unknown_cap slots
  uint64_t* unknown;
  uint64_t* unknown_pos;
  uint32_t* nunknown;
  uint32_t unknown_cap;
  uint64_t* scratch;     // [0] total out, [1] REF block, [2] BACKREF error, [3] declares, [4] BACKREFs, [5] t_end
  uint64_t* h_scratch;   // pinned copy of scratch[0..5], [6] nunknown
  uint64_t* chunk_tmp;   // 4 * n u64: n_decl, n_bref, decl_base, n_decl_emit
  uint4* d_tail;         // 256 declare records
  uint64_t* win_hash;    // the decoder's BACKREF window
  uint8_t* win_seg;
  uint64_t win_count;
  XcgLruState* lru;      // bounded cache (null: unbounded)
  uint32_t maxd;         // EXTRACTs a chunk can hold (bounded: declaration rows per chunk)
  XcgPairState* pair;    // XCodecCachePair (null: not a pair)
  int no_window;         // the BACKREF window is left alone (<LEARN>, single-segment host calls)
};

// Returns 0, -75 (output too small) or -5.  Outputs: total decoded bytes, the
// REF block and BACKREF error positions (~0 = none), unknown-REF count.
// Diagnostics (bench.py's decode roofline): HIP events bracket the batch
// decode's three device segments on its stream -- scan, refcheck / sizing,
// emit + commit (the host's two readbacks between them are not device time)
// -- and the emit kernel alone; xcg_debug_decode_kernel_time sums them.
namespace {
std::mutex g_dt_mu;
bool g_dt_on = false;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_dt_step, g_dt_emit;
struct DecTimer {
  hipStream_t s;
  hipEvent_t e0 = nullptr;
  std::vector<std::pair<hipEvent_t, hipEvent_t>>* dst;
  DecTimer(hipStream_t st, std::vector<std::pair<hipEvent_t, hipEvent_t>>* d) : s(st), dst(d) {
    std::lock_guard<std::mutex> g(g_dt_mu);
    if (g_dt_on && hipEventCreate(&e0) == hipSuccess) (void)hipEventRecord(e0, s);
  }
  ~DecTimer() {
    if (e0) (void)hipEventDestroy(e0);   // (a path that did not reach its end: not counted)
  }
  void end() {
    if (!e0) return;
    std::lock_guard<std::mutex> g(g_dt_mu);
    hipEvent_t e1 = nullptr;
    if (hipEventCreate(&e1) == hipSuccess && hipEventRecord(e1, s) == hipSuccess) dst->emplace_back(e0, e1);
    e0 = nullptr;
  }
};
double dt_sum(std::vector<std::pair<hipEvent_t, hipEvent_t>>& v) {
  double tot = 0;
  for (auto& e : v) {
    float t = 0;
    if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&t, e.first, e.second) == hipSuccess)
      tot += t;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  v.clear();
  return tot;
}
}  // namespace
extern "C" int xcg_debug_decode_kernel_timing(int on) {
  std::lock_guard<std::mutex> g(g_dt_mu);
  const int old = g_dt_on;
  g_dt_on = on != 0;
  return old;
}
extern "C" int xcg_debug_decode_kernel_time(double* step_ms, double* emit_ms, uint32_t* segments) {
  std::lock_guard<std::mutex> g(g_dt_mu);
  if (segments) *segments = (uint32_t)g_dt_step.size();
  const double s = dt_sum(g_dt_step), e = dt_sum(g_dt_emit);
  if (step_ms) *step_ms = s;
  if (emit_ms) *emit_ms = e;
  return 0;
}

extern "C" int xcg_launch_decode(const XcgDecodeArgs* a, uint64_t* total_out, uint64_t* block_pos_out,
                                 uint64_t* berr_pos_out, uint32_t* nunknown_out, hipStream_t stream) {
  using namespace xcg;
  const uint32_t n = a->n;
  DecParams p{};
  p.in = a->in;
  p.chunk_off = a->chunk_off;
  p.chunk_len = a->chunk_len;
  p.n = n;
  p.g = HashTab{a->g_keys, a->g_vals, a->g_mask};
  p.pool = a->pool;
  p.x = HashTab{a->x_keys, a->x_vals, a->x_mask};
  p.x_latest = a->x_latest;
  p.out_len = a->out_len;
  p.out_off = a->out_off;
  p.out = a->out;
  p.chunk_status = a->chunk_status;
  p.consumed = a->consumed;
  p.unknown = a->unknown;
  p.unknown_pos = a->unknown_pos;
  p.nunknown = a->nunknown;
  p.unknown_cap = a->unknown_cap;
  p.u_keys = a->u_keys;
  p.u_mask = 2 * a->unknown_cap - 1;
  p.block_pos = a->scratch + 1;
  p.berr_pos = a->scratch + 2;
  p.t_end = a->scratch + 5;
  p.status = a->status;
  p.n_decl = a->chunk_tmp;
  p.n_bref = a->chunk_tmp + n;
  p.decl_base = a->chunk_tmp + 2ull * n;
  p.n_decl_emit = a->chunk_tmp + 3ull * n;
  p.win_hash = a->win_hash;
  p.win_seg = a->win_seg;
  p.win_count = a->win_count;
  const dim3 grid((n + 3) / 4), block(256);
  DecTimer seg1(stream, &g_dt_step);
  if (hipMemsetAsync(a->x_keys, 0xFF, 8ull * (a->x_mask + 1), stream) != hipSuccess ||
      hipMemsetAsync(a->x_vals, 0xFF, 8ull * (a->x_mask + 1), stream) != hipSuccess ||
      hipMemsetAsync(a->x_latest, 0, 8ull * (a->x_mask + 1), stream) != hipSuccess ||
      hipMemsetAsync(a->scratch + 1, 0xFF, 16, stream) != hipSuccess ||
      hipMemsetAsync(a->nunknown, 0, 4, stream) != hipSuccess ||
      hipMemsetAsync(a->u_keys, 0xFF, 16ull * a->unknown_cap, stream) != hipSuccess)
    return -5;
  // scan, then number the declares
  hipLaunchKernelGGL(decode_kernel<false>, grid, block, 0, stream, p);
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint64_t*)p.n_decl,
                     (uint64_t*)p.decl_base, n, a->scratch + 3);
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint64_t*)p.n_bref,
                     p.n_decl_emit, n, a->scratch + 4);          // (n_decl_emit: scratch output here)
  seg1.end();
  if (hipMemcpyAsync(a->h_scratch + 3, a->scratch + 3, 16, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return -5;
  const uint64_t ndecl = a->h_scratch[3], nbref = a->h_scratch[4];
  // Bounded cache: classify every op against the eviction times until they
  // agree (xcg_lru.hip); the passes below then see the cache as it evolves.
  uint8_t* lru_mem = nullptr;
  LruBatch lb{};
  uint4 *raw = nullptr, *evs = nullptr;
  if (a->lru) {
    if (nbref > 0) return -95;                       // (BACKREF stop points are not modelled on a bounded cache)
    XcgLruState* L = a->lru;
    const uint64_t m = ndecl ? ndecl : 1;
    // raw ops, classified ops, declaration rows | evtime | evslot, per-chunk
    // counts, bases, flags
    const uint64_t bytes = 32 * m + 16ull * n * a->maxd + 8 * m + 4 * m + 20ull * (n + 1) + 64;
    if (hipMallocAsync((void**)&lru_mem, bytes, stream) != hipSuccess) return -5;
    raw = (uint4*)lru_mem;
    evs = raw + m;
    uint4* drow = evs + m;
    L->evtime = (uint64_t*)(drow + (uint64_t)n * a->maxd);
    L->evslot = (uint32_t*)(L->evtime + m);
    uint32_t* nev32 = L->evslot + m;
    uint32_t* nd32 = nev32 + (n + 1);
    uint32_t* need = nd32 + (n + 1);
    L->ev_base = need + (n + 1);
    L->enter_base = L->ev_base + (n + 1);
    uint64_t* blk = (uint64_t*)(((uintptr_t)(L->enter_base + n + 1) + 15) & ~(uintptr_t)15);
    uint32_t* changes = (uint32_t*)(blk + 1);
    lb = LruBatch{n, a->in, a->chunk_off, drow, nd32, a->maxd, evs, nev32, 0xFFFFFFFFu, 1, need,
                  a->g_keys, a->g_vals, a->g_mask, a->pool, a->nseg, a->g_filt, a->g_ftab, a->fmask,
                  a->g_gfilt, a->gmask, a->status, m};
    auto fail = [&](int rc) {
      (void)hipFreeAsync(lru_mem, stream);
      return rc;
    };
    hipLaunchKernelGGL(dec_ops_kernel, grid, block, 0, stream, p, raw);
    if (xcg_lru_reset_times(L, stream)) return fail(-5);
    p.ptime = L->ptime;
    uint64_t blockp = ~0ull;
    bool agreed = false;
    for (int pass = 0; pass < 64 && !agreed; ++pass) {
      if (hipMemsetAsync(blk, 0xFF, 8, stream) != hipSuccess || hipMemsetAsync(changes, 0, 4, stream) != hipSuccess)
        return fail(-5);
      hipLaunchKernelGGL(dec_classify_kernel<false>, grid, block, 0, stream, p, (const uint4*)raw, evs, nev32, drow, nd32,
                         a->maxd, blockp, blk, changes, pass == 0 ? 1 : 0);
      if (xcg_lru_times(&lb, L, stream)) return fail(-5);   // (synchronises)
      if (hipMemcpyAsync(a->h_scratch + 8, blk, 16, hipMemcpyDeviceToHost, stream) != hipSuccess ||
          hipStreamSynchronize(stream) != hipSuccess)
        return fail(-5);
      const uint64_t nb = a->h_scratch[8];
      const uint32_t nchg = (uint32_t)a->h_scratch[9];
      if ((uint64_t)L->h_tot[1] + L->h_tot[8] > L->C) return fail(-95);   // enters + persistent lookups > limit
      if (getenv("XCG_LRU_DEBUG"))
        fprintf(stderr, "lru-dec: n %u pass %d enters %u evict %u live %u hits %u changes %u block %llx -> %llx\n", n,
                pass, L->h_tot[1], L->h_tot[2], L->h_tot[3], L->h_tot[8], nchg, (unsigned long long)blockp,
                (unsigned long long)nb);
      agreed = nchg == 0 && nb == blockp;
      blockp = nb;
    }
    if (!agreed) return fail(-75);
  }
  // Pair: classify every op against ptime (the time a hash leaves both
  // levels), replay the classified ops through the pair's policy on the host
  // (xcg_pair.hip), and repeat until the departure times the replay computes
  // are the ones the classification used.
  uint8_t* pair_mem = nullptr;
  uint4* prow = nullptr;
  if (a->pair) {
    if (nbref > 0) return -95;                       // (BACKREF stop points are not modelled on a pair)
    if (xcg_pair_decode_begin(a->pair, stream)) return -5;
    const uint64_t m = ndecl ? ndecl : 1;
    const uint64_t bytes = 32 * m + 16ull * n * a->maxd + 8ull * (n + 1) + 64;
    if (hipMallocAsync((void**)&pair_mem, bytes, stream) != hipSuccess) return -5;
    auto fail = [&](int rc) {
      (void)hipFreeAsync(pair_mem, stream);
      return rc;
    };
    raw = (uint4*)pair_mem;
    evs = raw + m;
    prow = evs + m;
    uint32_t* nev32 = (uint32_t*)(prow + (uint64_t)n * a->maxd);
    uint32_t* nd32 = nev32 + (n + 1);
    uint64_t* blk = (uint64_t*)(((uintptr_t)(nd32 + n + 1) + 15) & ~(uintptr_t)15);
    uint32_t* changes = (uint32_t*)(blk + 1);
    hipLaunchKernelGGL(dec_ops_kernel, grid, block, 0, stream, p, raw);
    p.ptime = xcg_pair_state_ptime(a->pair);
    uint64_t blockp = ~0ull;
    bool agreed = false;
    for (int pass = 0; pass < 64 && !agreed; ++pass) {
      if (hipMemsetAsync(blk, 0xFF, 8, stream) != hipSuccess || hipMemsetAsync(changes, 0, 4, stream) != hipSuccess)
        return fail(-5);
      hipLaunchKernelGGL(dec_classify_kernel<true>, grid, block, 0, stream, p, (const uint4*)raw, evs, nev32, prow, nd32,
                         a->maxd, blockp, blk, changes, 1);
      if (hipMemcpyAsync(a->h_scratch + 8, blk, 8, hipMemcpyDeviceToHost, stream) != hipSuccess) return fail(-5);
      int same = 0;
      const PairGpu G{a->in, a->chunk_off, prow, a->maxd, a->pool, a->g_keys, a->g_vals, a->g_mask,
                      a->g_filt, a->g_ftab, a->fmask, a->g_gfilt, a->gmask, a->nseg, a->status};
      const int prc = xcg_pair_decode_pass(a->pair, &G, evs, p.decl_base, p.n_decl, n, ndecl, a->maxd, &same, stream);
      if (prc) return fail(prc);
      const uint64_t nb = a->h_scratch[8];
      if (getenv("XCG_PAIR_DEBUG"))
        fprintf(stderr, "pair-dec: n %u pass %d same %d block %llx -> %llx\n", n, pass, same,
                (unsigned long long)blockp, (unsigned long long)nb);
      agreed = same && nb == blockp;
      blockp = nb;
    }
    if (!agreed) return fail(-75);
  }
  uint4* dfull = nullptr;
  if (nbref > 0 && ndecl > 0) {
    // BACKREFs present: records of every declare (rare; never made by XCodecEncoder)
    if (hipMallocAsync((void**)&dfull, 16ull * ndecl, stream) != hipSuccess) return -5;
    p.D = dfull;
    p.D_lo = 0;
    p.D_tail = false;
    hipLaunchKernelGGL(decl_record_kernel, grid, block, 0, stream, p, ndecl);
  }
  DecTimer seg2(stream, &g_dt_step);
  hipLaunchKernelGGL(decode_refcheck_kernel, grid, block, 0, stream, p);
  if (nbref > 0) hipLaunchKernelGGL(decode_brefcheck_kernel, grid, block, 0, stream, p);
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint64_t*)a->out_len, a->out_off,
                     n, a->scratch);
  hipLaunchKernelGGL(dec_precheck_kernel, dim3((unsigned)(((uint64_t)a->x_mask + 256) / 256)), dim3(256), 0, stream,
                     p);
  seg2.end();
  a->h_scratch[10] = 0;
  if (hipMemcpyAsync(a->h_scratch, a->scratch, 24, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipMemcpyAsync(a->h_scratch + 6, a->nunknown, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipMemcpyAsync(a->h_scratch + 10, a->status, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess) {
    if (dfull) (void)hipFreeAsync(dfull, stream);
    return -5;
  }
  if (a->h_scratch[10] & (1u << 9)) {
    // refused before any output, cache or window change (dec_precheck_kernel)
    a->h_scratch[11] = a->h_scratch[10] & ~(uint64_t)(1u << 9);
    (void)hipMemcpyAsync(a->status, a->h_scratch + 11, 4, hipMemcpyHostToDevice, stream);
    (void)hipStreamSynchronize(stream);
    if (dfull) (void)hipFreeAsync(dfull, stream);
    if (lru_mem) (void)hipFreeAsync(lru_mem, stream);
    if (pair_mem) (void)hipFreeAsync(pair_mem, stream);
    return -95;
  }
  *total_out = a->h_scratch[0];
  *block_pos_out = a->h_scratch[1];
  *berr_pos_out = a->h_scratch[2];
  *nunknown_out = (uint32_t)(a->h_scratch[6] & 0xFFFFFFFFu);
  if (*total_out > a->out_cap) {
    if (dfull) (void)hipFreeAsync(dfull, stream);
    if (lru_mem) (void)hipFreeAsync(lru_mem, stream);
    if (pair_mem) (void)hipFreeAsync(pair_mem, stream);
    return -75;
  }
  DecTimer seg3(stream, &g_dt_step), emit(stream, &g_dt_emit);
  // No stop point: the declares end at ndecl, so the window's tail is known
  // now and the emit pass records it (no second walk over the ops).
  const bool fuse_tail = !a->no_window && !dfull && *block_pos_out == ~0ull && *berr_pos_out == ~0ull;
  if (fuse_tail) {
    p.tail_D = a->d_tail;
    p.tail_hi = ndecl;
    p.tail_lo = ndecl > 256u ? ndecl - 256u : 0u;
  }
  hipLaunchKernelGGL(decode_kernel<true>, grid, block, 0, stream, p);
  emit.end();
  p.tail_D = nullptr;
  hipLaunchKernelGGL(decode_tend_kernel, dim3(1), dim3(1), 0, stream, p, ndecl);
  if (!a->no_window) {
    if (!dfull) {
      p.D = a->d_tail;
      p.D_tail = true;
      if (!fuse_tail) hipLaunchKernelGGL(decl_record_kernel, grid, block, 0, stream, p, ndecl);
    }
    hipLaunchKernelGGL(window_update_kernel, dim3(64), dim3(256), 0, stream, p);
  }
  if (a->pair) {
    // the classification's declaration rows give each new entry's bytes
    const PairGpu G{a->in, a->chunk_off, prow, a->maxd, a->pool, a->g_keys, a->g_vals, a->g_mask,
                    a->g_filt, a->g_ftab, a->fmask, a->g_gfilt, a->gmask, a->nseg, a->status};
    const int crc = xcg_pair_decode_commit(a->pair, &G, stream);
    (void)hipFreeAsync(pair_mem, stream);
    if (dfull) (void)hipFreeAsync(dfull, stream);
    if (crc) return crc;
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
  if (a->lru) {
    hipLaunchKernelGGL(dec_replace_kernel, grid, block, 0, stream, p, (const uint4*)raw, (const uint4*)evs, a->pool);
    const int crc = xcg_lru_commit(&lb, a->lru, stream);
    (void)hipFreeAsync(lru_mem, stream);
    if (crc) return crc;
  } else {
    const uint64_t slots = (uint64_t)a->x_mask + 1;
    hipLaunchKernelGGL(decode_commit_kernel, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, stream, p,
                       a->pool, a->nseg, a->seg_cap, FiltSet{a->g_filt, a->g_ftab, a->fmask, a->g_gfilt, a->gmask});
    seg3.end();
  }
  if (dfull) (void)hipFreeAsync(dfull, stream);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// One decode() call on an unbounded cache in one launch (decode_small_kernel).
extern "C" int xcg_launch_decode_small(const uint8_t* in, uint32_t len, uint64_t* g_keys, uint64_t* g_vals,
                                       uint32_t g_mask, uint8_t* pool, uint32_t* nseg, uint32_t seg_cap,
                                       uint32_t* filt, uint32_t* ftab, uint32_t fmask, uint32_t* gfilt, uint32_t gmask,
                                       int32_t* status, void* scratch, uint32_t ops_cap, uint8_t* out, uint64_t out_cap,
                                       uint64_t* win_hash, uint8_t* win_seg, uint64_t win_count, uint64_t* res,
                                       uint64_t* tim, uint32_t* flag, uint32_t seq, hipStream_t stream) {
  using namespace xcg;
  SmallDec a;
  a.in = in;
  a.len = len;
  a.g = HashTab{g_keys, g_vals, g_mask};
  a.pool = pool;
  a.nseg = nseg;
  a.seg_cap = seg_cap;
  a.fs = FiltSet{filt, ftab, fmask, gfilt, gmask};
  a.status = status;
  a.ops = (uint4*)scratch;
  a.opv = (uint64_t*)(a.ops + ops_cap);
  a.D = (uint4*)(a.opv + ops_cap);
  a.ops_cap = ops_cap;
  a.out = out;
  a.out_cap = out_cap;
  a.win_hash = win_hash;
  a.win_seg = win_seg;
  a.win_count = win_count;
  a.res = res;
  a.tim = tim;
  a.flag = flag;
  a.seq = seq;
  hipLaunchKernelGGL(decode_small_kernel, dim3(1), dim3(1024), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" uint64_t xcg_decode_small_scratch(uint32_t ops_cap) { return 40ull * ops_cap; }
extern "C" uint32_t xcg_decode_small_res_words(void) { return 8 + xcg::SD_UMAX + xcg::SD_EMAX + 1; }
extern "C" uint32_t xcg_decode_small_phases(void) { return xcg::SD_PHASES; }
extern "C" uint32_t xcg_decode_small_lds_in(void) { return xcg::SD_LDS_IN; }
