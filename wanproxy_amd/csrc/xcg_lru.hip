// Bounded persistent cache: XCodecMemoryCache with memory_cache_limit_ != 0
// (xcodec/xcodec_cache.h:277-364) -- at the limit, enter() first evicts the
// least recently used entry; lookup() and replace() refresh an entry
// (XCodecLRU, xcodec/xcodec_lru.h:30-104).  Stream-semantics encode batches,
// decode batches and single-segment host calls stay bit-exact with the
// sequential XCodecEncoder / XCodecDecoder on such a cache.
//
// LRU state in HBM (C = limit in segments = pool slots):
//   skey[C]     key of the entry in pool slot s
//   lastref[C]  LRU time of its last enter / lookup (a 64-bit clock: batch
//               base + (chunk << 21 | 2 * window + 1 for a lookup, 2 * window
//               for an enter)) -- the order XCodecLRU's counters give
//   queue[A]    the A live slots, least recently used first
//
// Within one batch whose enters N plus persistent entries looked up H stay
// within C, the entries evicted are persistent ones that the batch does not
// look up: enter number C - A + j (in stream order) evicts the j-th least
// recently used persistent entry not looked up before that point, and the
// N + A - C <= A - H evictions never reach an entry the batch itself made or
// refreshed (those sit above every persistent entry in the LRU order).  For
// a persistent entry of LRU rank r, with S(r) entries below it that the batch
// looks up, that is eviction j = r - S(r) at tau[j], unless the batch looks it
// up first.  The parse takes these eviction times (ptime) as given; the pass
// below recomputes
// them from the references the parse made and checks every recorded lookup of
// a persistent entry against them -- a hit must come before the entry's
// eviction, a miss (GMISS) after it.  All checks passing means the parse is
// the sequential one (by induction over stream time: every lookup result then
// equals the LRU state the sequential encoder has at that point); otherwise
// the chunks with an inconsistent lookup are parsed again with the new times.
// (The decoder's references follow from the stream, so xcg_decode.hip only
// alternates classification and these times; see dec_classify_kernel.)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>

#include "xcg_cache.h"
#include "xcg_args.h"

namespace xcg {

constexpr uint64_t NEVER = ~0ull;
enum : uint32_t { T_E = 0, T_N, T_P, T_A, T_BAD, T_OVF, T_A2, T_NFREE, T_H, T_GATE = 15, T_WORDS = 16 };

// Ordered scan by one 1024-thread workgroup over i in [0, n): emit(i, p, v)
// with p = carry + sum of val(j) for j < i.  Returns carry + the total.
template <class V, class E>
__device__ uint32_t wg_scan(uint32_t n, uint32_t carry, V val, E emit) {
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x, w = t >> 6;
  for (uint32_t base = 0; base < n; base += 4096) {
    const uint32_t i0 = base + 4 * t;
    uint32_t x[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[k] = i0 + k < n ? val(i0 + k) : 0u;
      sum += x[k];
    }
    const uint32_t inc = wave_incl_scan(sum);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t s = wsum[j];
      if (j < w) wpre += s;
      tot += s;
    }
    uint32_t run = carry + wpre + inc - sum;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < n) emit(i0 + k, run, x[k]);
      run += x[k];
    }
    carry += tot;
    __syncthreads();
  }
  return carry;
}

__device__ __forceinline__ uint64_t ev_time(uint32_t c, uint4 e) { return ((uint64_t)c << 21) | e.z; }

__global__ __launch_bounds__(256) void lru_fill64_kernel(uint64_t* p, uint32_t n, uint64_t v) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}
// Several fills in one launch (each launch costs ~4 us of the sub-batch).
struct Fill64 {
  uint64_t* p;
  uint32_t n;
  uint64_t v;
};
__global__ __launch_bounds__(256) void lru_fill64x4_kernel(Fill64 f0, Fill64 f1, Fill64 f2, Fill64 f3,
                                                           const uint32_t* skip) {
  if (skip && *skip) return;
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, step = gridDim.x * blockDim.x;
  for (uint32_t i = i0; i < f0.n; i += step) f0.p[i] = f0.v;
  for (uint32_t i = i0; i < f1.n; i += step) f1.p[i] = f1.v;
  for (uint32_t i = i0; i < f2.n; i += step) f2.p[i] = f2.v;
  for (uint32_t i = i0; i < f3.n; i += step) f3.p[i] = f3.v;
}
__global__ __launch_bounds__(256) void lru_fill32_kernel(uint32_t* p, uint32_t n, uint32_t v) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

// Per-chunk reference / enter bases, batch totals, the eviction count.
__global__ __launch_bounds__(1024) void lru_prep_kernel(uint32_t n, const uint32_t* nev, const uint32_t* ndecl,
                                                        uint32_t maxe, uint32_t C, const uint32_t* nseg,
                                                        uint32_t* ev_base, uint32_t* enter_base, uint32_t* need,
                                                        uint32_t* tot, const uint32_t* skip) {
  if (skip && *skip) return;
  if (threadIdx.x == 0) tot[T_OVF] = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) need[i] = 0u;
  __syncthreads();
  const uint32_t e = wg_scan(
      n, 0u,
      [&](uint32_t i) {
        const uint32_t v = nev[i];
        if (v > maxe) atomicOr(&tot[T_OVF], 1u);
        return v < maxe ? v : maxe;
      },
      [&](uint32_t i, uint32_t p, uint32_t) { ev_base[i] = p; });
  const uint32_t ne = wg_scan(n, 0u, [&](uint32_t i) { return ndecl[i]; },
                              [&](uint32_t i, uint32_t p, uint32_t) { enter_base[i] = p; });
  if (threadIdx.x == 0) {
    ev_base[n] = e;
    enter_base[n] = ne;
    const uint32_t A = *nseg;
    tot[T_E] = e;
    tot[T_N] = ne;
    tot[T_A] = A;
    tot[T_P] = A + ne > C ? A + ne - C : 0u;
    tot[T_BAD] = 0;
  }
}

// tau[j] = time of the enter that makes eviction j; hmin[s] = first lookup hit
// of persistent slot s.
// Reference lists: chunk c's k-th reference is ev[row(c) + k], k < nev[c]
// (capped at maxe); row(c) = c * maxe (the encoder's fixed rows) or, dense,
// ev_base[c] (the decoder's, packed by op).  One wave per chunk.
struct EvRows {
  const uint4* ev;
  const uint32_t* nev;
  const uint32_t* ev_base;
  uint32_t maxe;
  bool dense;
  __device__ uint64_t row(uint32_t c) const { return dense ? (uint64_t)ev_base[c] : (uint64_t)c * maxe; }
  __device__ uint32_t count(uint32_t c) const { return min(nev[c], maxe); }
};
__device__ __forceinline__ uint32_t wave_chunk() { return blockIdx.x * 4u + readfirst(threadIdx.x >> 6); }

__global__ __launch_bounds__(256) void lru_events_kernel(uint32_t n, EvRows R, const uint32_t* enter_base,
                                                         const uint32_t* tot, uint32_t C, uint64_t* hmin,
                                                         uint64_t* tau, const uint32_t* skip) {
  const uint32_t c = wave_chunk();
  if ((skip && readfirst(*skip)) || c >= n) return;
  const uint64_t r0 = R.row(c);
  const uint32_t cnt = R.count(c);
  for (uint32_t k = lane_id(); k < cnt; k += 64) {
    const uint4 e = R.ev[r0 + k];
    const uint32_t kind = e.w >> 30, ref = e.w & EV_REF_MASK;
    if (kind == EV_ENTER) {
      const uint32_t ge = enter_base[c] + ref, thr = C - tot[T_A];
      if (ge >= thr) tau[ge - thr] = ev_time(c, e);
    } else if (kind == EV_GHIT) {
      atomicMin((unsigned long long*)&hmin[ref], (unsigned long long)ev_time(c, e));
    }
  }
}

// First guess of a sub-batch's evictions, before any parse: every chunk
// parses as its 2048-byte tiling (the seed), a tile found in the persistent
// cache being a REF there (a lookup hit), a tile equal to an earlier tile of
// the batch a REF too, and every other tile a declaration.  Enter times as
// the sequential encoder makes them: tile p is declared while examining window
// p + 2048, or after the last window.  One wave per chunk; pass 0 counts the
// chunk's enters (cnt) and records the hits, pass 1 places the enters in tau.
// With ptime (the eviction times the previous guess implies): a cached tile
// looked up at or after its entry's eviction is a miss and a declaration, as
// the parse makes it (and a later tile of that hash whose earliest tile in the
// batch was such a hit before the eviction declares it again).  The guess is
// iterated so the first parse already sees the evictions its own declarations
// cause (lru_seed_guess).
__global__ __launch_bounds__(256) void lru_seed_classify_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                                uint32_t maxd, const uint32_t* chunk_len, HashTab g,
                                                                HashTab b, uint32_t* cnt, const uint32_t* enter_base,
                                                                const uint32_t* tot, uint32_t C, uint64_t* hmin,
                                                                uint64_t* tau, int pass, const uint64_t* ptime) {
  const uint32_t c = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (c >= n) return;
  const uint32_t nd = ndecl[c], last = chunk_len[c] - SEG;
  uint32_t ne = 0;
  for (uint32_t d0 = 0; d0 < nd; d0 += 64) {
    const uint32_t d = d0 + (uint32_t)lane_id();
    bool enter = false;
    uint4 dd = make_uint4(0u, 0u, 0u, 0u);
    if (d < nd) {
      dd = decl[(uint64_t)c * maxd + d];
      const uint64_t gv = tab_lookup_t(g, dd.x, dd.y);
      const uint64_t th = ((uint64_t)c << 21) | (2u * dd.z + 1u);
      if (gv != ~0ull && (!ptime || th < ptime[gv])) {
        if (pass == 0) atomicMin((unsigned long long*)&hmin[gv], (unsigned long long)th);
      } else {
        const uint64_t e = tab_lookup_t(b, dd.x, dd.y);
        enter = e == (((uint64_t)c << 32) | dd.z);     // the earliest tile with this hash
        if (!enter && gv != ~0ull)                     // the earliest was a hit on the entry, before its eviction
          enter = ((((e >> 32) << 21) | (2u * (uint32_t)e + 1u)) < ptime[gv]);
      }
    }
    const uint64_t m = ballot(enter);
    if (pass == 1 && enter) {
      const uint32_t o = ne + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const uint32_t t = dd.z + SEG <= last ? 2u * (dd.z + SEG) : 2u * (last + 1u);
      const uint32_t ge = enter_base[c] + o, thr = C - tot[T_A];
      if (ge >= thr) tau[ge - thr] = ((uint64_t)c << 21) | t;
    }
    ne += (uint32_t)__builtin_popcountll(m);
  }
  if (pass == 0 && lane_id() == 0) cnt[c] = ne;
}

// The batch's tiles in a scratch table: hash -> earliest (chunk << 32 | position).
__global__ __launch_bounds__(256) void lru_seed_table_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                             uint32_t maxd, HashTab b, int32_t* status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (uint32_t)(i / maxd), d = (uint32_t)(i % maxd);
  if (c >= n || d >= ndecl[c]) return;
  const uint4 dd = decl[i];
  if (!tab_insert_min(b, dd.x, dd.y, ((uint64_t)c << 32) | dd.z)) atomicOr(status, 2);
}


// Every recorded lookup of a persistent entry against the recomputed times.
// The in-chunk times of the first and last inconsistent lookup go to bad_t /
// bad_hi (the re-parse resumes before the first and may rejoin its old parse
// after the last, encode_chunk "Re-parse restart").
__global__ __launch_bounds__(256) void lru_check_kernel(uint32_t n, EvRows R, const uint64_t* hmin,
                                                        const uint64_t* wpop, uint32_t* need, uint32_t* tot,
                                                        uint32_t* bad_t, uint32_t* bad_hi, const uint32_t* skip) {
  const uint32_t c = wave_chunk();
  if ((skip && readfirst(*skip)) || c >= n) return;
  const uint64_t r0 = R.row(c);
  const uint32_t cnt = R.count(c);
  uint32_t lo = ~0u, hi = 0u;
  for (uint32_t k = lane_id(); k < cnt; k += 64) {
    const uint4 e = R.ev[r0 + k];
    const uint32_t kind = e.w >> 30, ref = e.w & EV_REF_MASK;
    const uint64_t t = ev_time(c, e);
    bool bad = false;
    if (kind == EV_GHIT) bad = t == hmin[ref] && !(t < wpop[ref]);        // hit after its eviction
    else if (kind == EV_GMISS) bad = !(hmin[ref] == NEVER && t >= wpop[ref]);   // missed a live entry
    if (bad) { lo = min(lo, e.z); hi = max(hi, e.z); }
  }
  for (int off = 32; off >= 1; off >>= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, off));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, off));
  }
  if (lane_id() == 0) {
    if (bad_t) { bad_t[c] = lo; bad_hi[c] = hi; }
    if (lo != ~0u) {
      need[c] = 1u;                                   // the next pass re-parses chunk c
      atomicAdd(&tot[T_BAD], 1u);
    }
  }
}

// The batch stands (no overflow, within the bound, no inconsistent lookup):
// tot[T_GATE] = 0, which lets a commit queued behind it act.
// (skip set: the pass itself was skipped -- the Jacobi round it followed did
// not converge -- so nothing stands)
__global__ void lru_gate_kernel(uint32_t* tot, uint32_t C, const uint32_t* skip) {
  if (threadIdx.x == 0)
    tot[T_GATE] = !(skip && *skip) && tot[T_OVF] == 0u && (uint64_t)tot[T_N] + tot[T_H] <= C && tot[T_BAD] == 0u
                      ? 0u : 1u;
}

// ---- ordered scans over many workgroups (rank walk, free list, new LRU order)
//
// Two launches instead of one workgroup walking everything (whose dependent
// random loads per 4096-element tile made it ~100 us at C = 65536): pass 0
// counts each 1024-element tile's flags into part[tile]; pass 1 adds the counts
// of the tiles before it and emits.
enum : int { SK_RANK = 0, SK_QUEUE = 1, SK_FREE = 2 };
struct ScanArgs {
  uint32_t* tot;
  const uint32_t* queue;
  const uint64_t* hmin;
  const uint64_t* tau;
  uint64_t* wpop;
  uint64_t* ptime;
  const uint32_t* alive;
  const uint64_t* lastref;
  uint64_t clock;
  const uint32_t* evslot;
  const uint64_t* evtime;
  uint32_t* queue2;
  uint32_t* nseg;
  uint32_t C;
  uint32_t* freel;
  uint32_t* part;
  uint64_t* hmin_reset;                            // (SK_RANK) reset hmin behind the scan: the next guess's atomics
  const uint32_t* gate;                            // (commit scans) nonzero: the commit does nothing
};

template <int K>
__device__ __forceinline__ uint32_t scan_n(const ScanArgs& a) {
  if (K == SK_RANK) return a.tot[T_A];
  if (K == SK_QUEUE) return a.tot[T_A] + a.tot[T_E];
  return a.C;
}

// flag of element i (and the value a compaction writes)
template <int K>
__device__ __forceinline__ uint32_t scan_flag(const ScanArgs& a, uint32_t i, uint32_t& v) {
  if (K == SK_RANK) {
    v = a.queue[i];
    return a.hmin[v] != NEVER ? 1u : 0u;
  }
  if (K == SK_QUEUE) {
    const uint32_t A = a.tot[T_A];
    if (i < A) {                                   // persistent entries the batch left alone, old order
      v = a.queue[i];
      return a.alive[v] && a.lastref[v] < a.clock ? 1u : 0u;
    }
    v = a.evslot[i - A];                           // then each entry's last reference, in stream order
    return v != ~0u && a.lastref[v] == a.evtime[i - A] ? 1u : 0u;
  }
  v = i;
  return a.alive[i] ? 0u : 1u;
}

template <int K>
__device__ __forceinline__ void scan_emit(const ScanArgs& a, uint32_t i, uint32_t p, uint32_t f, uint32_t v) {
  if (K == SK_RANK) {                              // p = S(r): looked-up entries below rank i
    const uint32_t j = i - p, P = a.tot[T_P];
    const uint64_t w = j < P ? a.tau[j] : NEVER;
    a.wpop[v] = w;
    a.ptime[v] = f && a.hmin[v] < w ? NEVER : w;   // (a hit after the eviction did not happen)
    if (a.hmin_reset) a.hmin_reset[v] = NEVER;
  } else if (K == SK_QUEUE) {
    if (f) a.queue2[p] = v;
  } else {
    if (f) a.freel[p] = v;
  }
}

template <int K>
__device__ __forceinline__ void scan_total(const ScanArgs& a, uint32_t total) {
  if (K == SK_RANK) a.tot[T_H] = total;
  else if (K == SK_QUEUE) { *a.nseg = total; a.tot[T_A2] = total; }
  else a.tot[T_NFREE] = total;
}

template <int K>
__global__ __launch_bounds__(256) void scan_count_kernel(ScanArgs a) {
  __shared__ uint32_t ws[4];
  if (a.gate && *a.gate) return;
  const uint32_t n = scan_n<K>(a), i0 = blockIdx.x * 1024u + 4u * threadIdx.x;
  if (blockIdx.x * 1024u >= n && blockIdx.x != 0) return;
  uint32_t c = 0, v;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i0 + k < n) c += scan_flag<K>(a, i0 + k, v);
  c = wave_sum(c);
  if (lane_id() == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) a.part[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

template <int K>
__global__ __launch_bounds__(256) void scan_emit_kernel(ScanArgs a) {
  __shared__ uint32_t ws[4], s_base;
  if (a.gate && *a.gate) return;
  const uint32_t n = scan_n<K>(a), ntiles = (n + 1023u) / 1024u, tile = blockIdx.x;
  if (tile >= ntiles && !(tile == 0 && n == 0)) return;
  // base = counts of the tiles before this one
  uint32_t b = 0;
  for (uint32_t t = threadIdx.x; t < tile; t += 256) b += a.part[t];
  b = wave_sum(b);
  if (lane_id() == 0) ws[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) s_base = ws[0] + ws[1] + ws[2] + ws[3];
  __syncthreads();
  const uint32_t base = s_base;
  __syncthreads();
  const uint32_t i0 = tile * 1024u + 4u * threadIdx.x;
  uint32_t f[4], v[4], c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[k] = i0 + k < n ? scan_flag<K>(a, i0 + k, v[k]) : 0u;
    c += f[k];
  }
  const uint32_t inc = wave_incl_scan(c);
  if (lane_id() == 63) ws[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t wpre = 0, tt = 0;
  for (uint32_t w = 0; w < 4; ++w) {
    const uint32_t x = ws[w];
    if (w < (threadIdx.x >> 6)) wpre += x;
    tt += x;
  }
  uint32_t run = base + wpre + inc - c;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (i0 + k < n) scan_emit<K>(a, i0 + k, run, f[k], v[k]);
    run += f[k];
  }
  if (threadIdx.x == 0 && (tile + 1 >= ntiles)) scan_total<K>(a, base + tt);
}

// ---- commit

// (commit kernels: gate nonzero = the eviction pass found the batch
// inconsistent; the commit, queued before the host has read that, does nothing)
__global__ __launch_bounds__(256) void lru_unmark_kernel(uint32_t* alive, uint32_t n, const uint32_t* gate) {
  if (gate && *gate) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) alive[i] = 0u;
}
__global__ __launch_bounds__(256) void lru_mark_kernel(const uint32_t* tot, const uint32_t* queue,
                                                       const uint64_t* hmin, const uint64_t* wpop, uint32_t* alive,
                                                       const uint32_t* gate) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if ((gate && *gate) || r >= tot[T_A]) return;
  const uint32_t s = queue[r];
  alive[s] = (hmin[s] == NEVER && wpop[s] != NEVER) ? 0u : 1u;   // evicted in the batch
}


struct Wipe {
  HashTab g;
  uint32_t* filt;
  u32x4* ftab; uint32_t ftab_n;
  uint32_t* gfilt; uint32_t gfilt_n;
};
__global__ __launch_bounds__(256) void lru_wipe_kernel(Wipe w, const uint32_t* gate) {
  if (gate && *gate) return;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = i0; i <= w.g.mask; i += stride) { w.g.keys[i] = EMPTY_KEY; w.g.vals[i] = ~0ull; }
  for (uint64_t i = i0; i < FILT_WORDS; i += stride) w.filt[i] = 0u;
  for (uint64_t i = i0; i < w.ftab_n; i += stride) w.ftab[i] = u32x4{0u, 0u, 0u, 0u};
  for (uint64_t i = i0; i < w.gfilt_n; i += stride) w.gfilt[i] = 0u;
}

__global__ __launch_bounds__(256) void lru_insert_alive_kernel(uint32_t C, const uint32_t* alive,
                                                               const uint64_t* skey, HashTab g, FiltSet fs,
                                                               int32_t* status, const uint32_t* gate) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if ((gate && *gate) || s >= C || !alive[s]) return;
  const uint64_t k = skey[s];
  // (table + filters with the short chain of returning atomics, xcg_cache.h)
  if (!tab_insert_min_filt(g, fs, (uint32_t)k, (uint32_t)(k >> 32), s)) atomicOr(status, 2);
}

// One wave per declaration: its pool slot from the free list, key, table,
// filters, and the 2048 bytes.
__global__ __launch_bounds__(256) void lru_insert_new_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                             uint32_t maxd, const uint32_t* enter_base,
                                                             const uint32_t* freel, const uint8_t* in,
                                                             const uint64_t* chunk_off, uint64_t* skey,
                                                             uint32_t* alive, HashTab g, uint8_t* pool, FiltSet fs,
                                                             int32_t* status, const uint32_t* gate) {
  const uint64_t w = (uint64_t)blockIdx.x * 4 + readfirst(threadIdx.x >> 6);
  const uint32_t c = (uint32_t)(w / maxd), d = (uint32_t)(w % maxd);
  if ((gate && readfirst(*gate)) || c >= n || d >= ndecl[c]) return;
  const uint4 dd = decl[(uint64_t)c * maxd + d];
  // the segment's loads first: a returning atomic (the table insert) waits for
  // every older memory operation of the wave on gfx9, so loads issued after it
  // would add their latency to the insert's
  const uint8_t* src = in + chunk_off[c] + dd.z;
  const int l = lane_id();
  const u32x4 v0 = *(const u32x4_u*)(src + 32 * l), v1 = *(const u32x4_u*)(src + 32 * l + 16);
  const uint32_t s = freel[enter_base[c] + d];
  if (l == 0) {
    skey[s] = ((uint64_t)dd.y << 32) | dd.x;
    alive[s] = 1u;
    if (!tab_insert_min_filt(g, fs, dd.x, dd.y, s)) atomicOr(status, 2);
  }
  uint8_t* dst = pool + (uint64_t)s * SEG;
  *(u32x4_u*)(dst + 32 * l) = v0;
  *(u32x4_u*)(dst + 32 * l + 16) = v1;
}

// Every reference's slot (evslot, in stream order) and time; lastref = the
// latest reference of each slot.
__global__ __launch_bounds__(256) void lru_lastref_kernel(uint32_t n, EvRows R, const uint32_t* enter_base,
                                                          const uint32_t* freel, HashTab g, uint64_t clock,
                                                          uint64_t* lastref, uint32_t* evslot, uint64_t* evtime,
                                                          const uint32_t* gate) {
  const uint32_t c = wave_chunk();
  if ((gate && readfirst(*gate)) || c >= n) return;
  const uint64_t r0 = R.row(c);
  const uint32_t cnt = R.count(c);
  for (uint32_t k = lane_id(); k < cnt; k += 64) {
    const uint4 e = R.ev[r0 + k];
    const uint32_t kind = e.w >> 30, ref = e.w & EV_REF_MASK;
    uint32_t s = ~0u;
    if (kind == EV_ENTER) s = freel[enter_base[c] + ref];
    else if (kind == EV_GHIT) s = ref;
    else if (kind == EV_HIT) s = (uint32_t)tab_lookup_t(g, e.x, e.y);
    const uint64_t t = clock + ev_time(c, e);
    const uint32_t gi = R.ev_base[c] + k;
    evslot[gi] = s;
    evtime[gi] = t;
    if (s != ~0u) atomicMax((unsigned long long*)&lastref[s], (unsigned long long)t);
  }
}


}  // namespace xcg

namespace {

bool lru_debug() {
  static const bool on = getenv("XCG_LRU_DEBUG") != nullptr;
  return on;
}

unsigned grid_for(uint64_t threads) { return (unsigned)((threads + 255) / 256); }

// One multi-workgroup ordered scan over at most max_n elements.
template <int K>
int run_scan(XcgLruState* L, xcg::ScanArgs a, uint64_t max_n, hipStream_t st) {
  const uint32_t tiles = (uint32_t)((max_n + 1023) / 1024) + 1;
  if (tiles > L->part_cap) {
    (void)hipFree(L->part);
    L->part = nullptr;
    L->part_cap = 0;
    if (hipMalloc(&L->part, 4ull * tiles * 2) != hipSuccess) return -5;
    L->part_cap = tiles * 2;
  }
  a.part = L->part;
  hipLaunchKernelGGL(xcg::scan_count_kernel<K>, dim3(tiles), dim3(256), 0, st, a);
  hipLaunchKernelGGL(xcg::scan_emit_kernel<K>, dim3(tiles), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

xcg::ScanArgs scan_args(XcgLruState* L, uint32_t* nseg) {
  xcg::ScanArgs a{};
  a.tot = L->tot;
  a.queue = L->queue;
  a.hmin = L->hmin;
  a.tau = L->tau;
  a.wpop = L->wpop;
  a.ptime = L->ptime;
  a.alive = L->alive;
  a.lastref = L->lastref;
  a.clock = L->clock;
  a.evslot = L->evslot;
  a.evtime = L->evtime;
  a.queue2 = L->queue2;
  a.nseg = nseg;
  a.C = L->C;
  a.freel = L->freel;
  return a;
}

LruBatch batch_of(const XcgStreamArgs& a) {
  return LruBatch{a.n, a.in, a.chunk_off, a.decl, a.ndecl, a.maxd, a.ev, a.nev, a.maxe, 0, a.need,
                  a.g_keys, a.g_vals, a.g_mask, a.pool, a.nseg, a.g_filt, a.g_ftab, a.fmask, a.g_gfilt, a.gmask,
                  a.status, (uint64_t)a.n * a.maxe, a.bad_t, a.bad_hi};
}

// Eviction times from a batch's references: tau, first hits, the LRU-order
// scan (ptime, wpop), and -- check != 0 -- every recorded persistent lookup
// against them.  h_tot gets the totals.  Synchronises `st`.
// skip (nullable, !sync only): a device word that, nonzero, makes the whole
// pass do nothing (and the gate refuse the commit).
int lru_times(const LruBatch& b, XcgLruState* L, bool check, hipStream_t st, bool sync = true,
              const uint32_t* skip = nullptr) {
  using namespace xcg;
  const uint32_t n = b.n;
  hipLaunchKernelGGL(lru_prep_kernel, dim3(1), dim3(1024), 0, st, n, b.nev, b.ndecl, b.maxe, L->C,
                     (const uint32_t*)b.nseg, L->ev_base, L->enter_base, b.need, L->tot, skip);
  const unsigned cg = grid_for(L->C) < 1024 ? grid_for(L->C) : 1024;
  hipLaunchKernelGGL(lru_fill64x4_kernel, dim3(cg), dim3(256), 0, st, Fill64{L->hmin, L->C, NEVER},
                     Fill64{L->tau, L->C, NEVER}, Fill64{nullptr, 0u, 0ull}, Fill64{nullptr, 0u, 0ull}, skip);
  const EvRows R{(const uint4*)b.ev, b.nev, (const uint32_t*)L->ev_base, b.maxe, b.dense != 0};
  const dim3 wgrid((n + 3) / 4);
  hipLaunchKernelGGL(lru_events_kernel, wgrid, dim3(256), 0, st, n, R, (const uint32_t*)L->enter_base,
                     (const uint32_t*)L->tot, L->C, L->hmin, L->tau, skip);
  ScanArgs ra = scan_args(L, nullptr);
  ra.gate = skip;
  if (run_scan<SK_RANK>(L, ra, L->C, st)) return -5;
  if (check)
    hipLaunchKernelGGL(lru_check_kernel, wgrid, dim3(256), 0, st, n, R, (const uint64_t*)L->hmin,
                       (const uint64_t*)L->wpop, b.need, L->tot, b.bad_t, b.bad_hi, skip);
  if (!sync) {                                     // (the caller waits on L->tev after queueing more)
    hipLaunchKernelGGL(lru_gate_kernel, dim3(1), dim3(64), 0, st, L->tot, L->C, skip);
    if (!L->tev && hipEventCreateWithFlags((hipEvent_t*)&L->tev, hipEventDisableTiming) != hipSuccess) return -5;
    if (hipMemcpyAsync(L->h_tot, L->tot, 4 * T_WORDS, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipEventRecord((hipEvent_t)L->tev, st) != hipSuccess)
      return -5;
    return 0;
  }
  if (hipMemcpyAsync(L->h_tot, L->tot, 4 * T_WORDS, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return -5;
  return 0;
}

// Guesses of the seed's evictions (XCG_LRU_SEED_ITERS, default 3; 1 = the
// round-4 single guess).
int seed_iters() {                                // (read per sub-batch: tests switch it)
  const char* e = getenv("XCG_LRU_SEED_ITERS");
  const int k = e ? atoi(e) : 3;
  return k < 1 ? 1 : (k > 8 ? 8 : k);
}

// ptime from the tiling seed (lru_seed_classify_kernel).  Asynchronous.
int lru_seed_guess(const XcgStreamArgs& a, XcgLruState* L, hipStream_t st) {
  using namespace xcg;
  const uint32_t n = a.n;
  const unsigned cg = grid_for(L->C) < 1024 ? grid_for(L->C) : 1024;
  const HashTab g{a.g_keys, a.g_vals, a.g_mask}, b{a.b_keys, a.b_vals, a.b_mask};   // (b: the rounds rebuild it)
  (void)cg;
  hipLaunchKernelGGL(lru_fill64x4_kernel, dim3(1024), dim3(256), 0, st, Fill64{b.keys, b.mask + 1, EMPTY_KEY},
                     Fill64{b.vals, b.mask + 1, ~0ull}, Fill64{L->hmin, L->C, NEVER}, Fill64{L->tau, L->C, NEVER},
                     nullptr);
  hipLaunchKernelGGL(lru_seed_table_kernel, dim3(grid_for((uint64_t)n * a.maxd)), dim3(256), 0, st, n,
                     (const uint4*)a.decl, (const uint32_t*)a.ndecl, a.maxd, b, a.status);
  uint32_t* cnt = a.nhits;                         // (scratch until the rounds: round 1 rewrites it)
  const dim3 wgrid((n + 3) / 4);
  // guess 0 takes every cached tile for a hit; each further guess classifies
  // against the evictions the one before implies (lru_seed_classify_kernel)
  // (hmin: reset behind each scan but the last; tau needs no reset: the scan
  // reads tau[j] for j below the eviction count only, and a guess's enters
  // write every one of those)
  const int iters = seed_iters();
  for (int it = 0; it < iters; ++it) {
    const uint64_t* pt = it ? (const uint64_t*)L->ptime : nullptr;
    hipLaunchKernelGGL(lru_seed_classify_kernel, wgrid, dim3(256), 0, st, n, (const uint4*)a.decl,
                       (const uint32_t*)a.ndecl, a.maxd, a.chunk_len, g, b, cnt, (const uint32_t*)L->enter_base,
                       (const uint32_t*)L->tot, L->C, L->hmin, L->tau, 0, pt);
    hipLaunchKernelGGL(lru_prep_kernel, dim3(1), dim3(1024), 0, st, n, (const uint32_t*)a.nev, (const uint32_t*)cnt,
                       a.maxe, L->C, (const uint32_t*)a.nseg, L->ev_base, L->enter_base, a.need, L->tot,
                       (const uint32_t*)nullptr);
    hipLaunchKernelGGL(lru_seed_classify_kernel, wgrid, dim3(256), 0, st, n, (const uint4*)a.decl,
                       (const uint32_t*)a.ndecl, a.maxd, a.chunk_len, g, b, cnt, (const uint32_t*)L->enter_base,
                       (const uint32_t*)L->tot, L->C, L->hmin, L->tau, 1, pt);
    ScanArgs sa = scan_args(L, nullptr);
    if (it + 1 < iters) sa.hmin_reset = L->hmin;
    if (run_scan<SK_RANK>(L, sa, L->C, st)) return -5;
  }
  return 0;
}

}  // namespace

// Commit a consistent batch (its references as lru_times last saw them):
// evict, number the new entries, rebuild table + probe structures, new LRU
// order.  Asynchronous.
namespace {
// The device part of a commit; gate (nullable): a device word that, nonzero,
// makes every kernel of it do nothing.
int lru_commit_dev(const LruBatch* bp, XcgLruState* L, const uint32_t* gate, hipStream_t st) {
  using namespace xcg;
  const LruBatch& b = *bp;
  const uint32_t n = b.n, C = L->C;
  const unsigned cg = grid_for(C) < 1024 ? grid_for(C) : 1024;
  hipLaunchKernelGGL(lru_unmark_kernel, dim3(cg), dim3(256), 0, st, L->alive, C, gate);
  hipLaunchKernelGGL(lru_mark_kernel, dim3(grid_for(C)), dim3(256), 0, st, (const uint32_t*)L->tot,
                     (const uint32_t*)L->queue, (const uint64_t*)L->hmin, (const uint64_t*)L->wpop, L->alive, gate);
  ScanArgs fa = scan_args(L, nullptr);
  fa.gate = gate;
  if (run_scan<SK_FREE>(L, fa, C, st)) return -5;
  const HashTab g{b.g_keys, b.g_vals, b.g_mask};
  const FiltSet fs{b.g_filt, b.g_ftab, b.fmask, b.g_gfilt, b.gmask};
  Wipe w{g, b.g_filt, (u32x4*)b.g_ftab, b.fmask + 1, b.g_gfilt, b.gmask + 1};
  hipLaunchKernelGGL(lru_wipe_kernel, dim3(1024), dim3(256), 0, st, w, gate);
  hipLaunchKernelGGL(lru_insert_alive_kernel, dim3(grid_for(C)), dim3(256), 0, st, C, (const uint32_t*)L->alive,
                     (const uint64_t*)L->skey, g, fs, b.status, gate);
  const uint64_t waves = (uint64_t)n * b.maxd;
  hipLaunchKernelGGL(lru_insert_new_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, n,
                     (const uint4*)b.decl, b.ndecl, b.maxd, (const uint32_t*)L->enter_base,
                     (const uint32_t*)L->freel, b.in, b.chunk_off, L->skey, L->alive, g, b.pool, fs, b.status, gate);
  const EvRows R{(const uint4*)b.ev, b.nev, (const uint32_t*)L->ev_base, b.maxe, b.dense != 0};
  hipLaunchKernelGGL(lru_lastref_kernel, dim3((n + 3) / 4), dim3(256), 0, st, n, R, (const uint32_t*)L->enter_base,
                     (const uint32_t*)L->freel, g, L->clock, L->lastref, L->evslot, L->evtime, gate);
  {
    ScanArgs qa = scan_args(L, b.nseg);
    qa.gate = gate;
    if (run_scan<SK_QUEUE>(L, qa, (uint64_t)C + b.ev_bound, st)) return -5;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The host side of a commit that happened: the new LRU order, the clock.
void lru_commit_host(XcgLruState* L, uint32_t n) {
  uint32_t* q = L->queue;
  L->queue = L->queue2;
  L->queue2 = q;
  L->clock += ((uint64_t)n << 21) + 4;
}
}  // namespace

extern "C" int xcg_lru_commit(const LruBatch* bp, XcgLruState* L, hipStream_t st) {
  if (lru_commit_dev(bp, L, nullptr, st)) return -5;
  lru_commit_host(L, bp->n);
  return 0;
}


// Eviction times of a batch whose references are already classified (the
// decoder's: fixed by the stream).  h_tot: totals.  Synchronises.
extern "C" int xcg_lru_times(const LruBatch* b, XcgLruState* L, hipStream_t st) { return lru_times(*b, L, false, st); }

extern "C" int xcg_lru_reset_times(XcgLruState* L, hipStream_t st) {
  using namespace xcg;
  const unsigned cg = grid_for(L->C) < 1024 ? grid_for(L->C) : 1024;
  hipLaunchKernelGGL(lru_fill64_kernel, dim3(cg), dim3(256), 0, st, L->ptime, L->C, NEVER);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Stream-semantics encode of a batch on a bounded cache.  The batch is cut
// into sub-batches with N + H <= C (the bound the eviction rule above needs; a
// sub-batch that exceeds it is halved); each is parsed
// (xcg_launch_encode_stream, commit off) until its eviction times are
// consistent, then committed.  Returns 0, -75 (no fixed point / reference
// list overflow), -95 (one chunk alone exceeds the bound), -5.
extern "C" int xcg_lru_encode_stream(const XcgStreamArgs* a0, XcgLruState* L, int* rounds_out, hipStream_t st) {
  using namespace xcg;
  const uint32_t n = a0->n, C = L->C;
  int rounds = 0;
  // chunks per sub-batch: from the bound (a chunk declares or REFs each
  // 2048 bytes at most once; collision lookups aside), then from what the last
  // sub-batch used
  uint32_t per = C / a0->maxd ? C / a0->maxd : 1u;
  if (L->fit_hint >= a0->maxd) {                   // equal parts at what the last sub-batches held
    const uint32_t hint = L->fit_hint / a0->maxd;
    const uint32_t k = (n + hint - 1) / hint;
    per = (n + k - 1) / k;
  }
  constexpr int MAX_PASSES = 12;
  uint32_t i0 = 0;
  while (i0 < n) {
    const uint32_t m = per < n - i0 ? per : n - i0;
    XcgStreamArgs a = *a0;
    a.n = m;
    a.chunk_off += i0;
    a.chunk_len += i0;
    a.out_off += i0;
    a.out_len += i0;
    if (a.stats) a.stats += 4ull * i0;
    a.ptime = L->ptime;
    a.no_commit = 1;
    // Behind each Jacobi verification, before the host has read its flags: the
    // eviction pass and the gated commit, both doing nothing unless the round
    // converged (vflags[1] == 0).  The host then waits once, on the totals.
    struct Hook {
      XcgLruState* L;
      const XcgStreamArgs* a;
      bool fired;
    } hook{L, &a, false};
    a.post_user = &hook;
    a.post_verify = [](void* u, const uint32_t* vbusy, hipStream_t s) -> int {
      Hook* h = (Hook*)u;
      const LruBatch b = batch_of(*h->a);
      h->fired = true;
      if (lru_times(b, h->L, true, s, false, vbusy)) return -5;
      return lru_commit_dev(&b, h->L, h->L->tot + T_GATE, s);
    };
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    auto dsync = [&]() { if (lru_debug()) (void)hipStreamSynchronize(st); return clk::now(); };
    const clk::time_point t0 = dsync();
    // Pass 0 starts from the tiling seed, with the evictions it implies.
    if (xcg_launch_seed_tiling(&a, st)) return -5;
    if (lru_seed_guess(a, L, st)) return -5;
    const clk::time_point t1 = dsync();
    bool done = false, split = false;
    for (int pass = 0; pass < MAX_PASSES && !done && !split; ++pass) {
      a.keep_decls = 1;
      a.need_given = pass > 0;                       // re-parse the chunks with an inconsistent lookup
      int r = 0;
      const clk::time_point q0 = dsync();
      hook.fired = false;
      const int rc = xcg_launch_encode_stream(&a, &r, st);
      rounds += r;
      if (rc) return rc;
      const clk::time_point q1 = dsync();
      // The commit is queued behind the eviction pass, gated on its verdict
      // (tot[T_GATE]), before the host has read the totals: it runs in the
      // time the host waits for them.
      if (!hook.fired) {                             // (no verification ran: one chunk, or nothing declared)
        const LruBatch b = batch_of(a);
        if (lru_times(b, L, true, st, false)) return -5;
        if (lru_commit_dev(&b, L, L->tot + T_GATE, st)) return -5;
      }
      if (hipEventSynchronize((hipEvent_t)L->tev) != hipSuccess) return -5;
      const clk::time_point q2 = dsync();
      if (lru_debug()) {
        int32_t stw = 0;
        (void)hipMemcpy(&stw, a.status, 4, hipMemcpyDeviceToHost);
        fprintf(stderr, "lru: chunks %u+%u pass %d rounds %d refs %u enters %u evict %u live %u bad %u ovf %u status %x"
                " | ms seed %.3f parse %.3f times %.3f\n",
                i0, m, pass, r, L->h_tot[T_E], L->h_tot[T_N], L->h_tot[T_P], L->h_tot[T_A], L->h_tot[T_BAD],
                L->h_tot[T_OVF], stw, pass == 0 ? ms(t0, t1) : 0.0, ms(q0, q1), ms(q1, q2));
      }
      if (L->h_tot[T_OVF]) return -75;
      if ((uint64_t)L->h_tot[T_N] + L->h_tot[T_H] > C) split = true;
      else if (L->h_tot[T_BAD] == 0) done = true;
    }
    if (!done) {
      if (m == 1) return split ? -95 : -75;
      per = m / 2;                                   // redo this part in halves
      continue;
    }
    lru_commit_host(L, m);
    L->last_base = i0;
    i0 += m;
    // (a sub-batch that started below the limit saw fewer cached entries to
    // look up than the next will: size the next one more cautiously)
    const uint64_t used = (uint64_t)L->h_tot[T_N] + L->h_tot[T_H];
    // The most chunks that fit under 95 % of the bound at this sub-batch's use
    // per chunk (75 % while the cache is still filling: a sub-batch that
    // started below the limit saw fewer cached entries to look up than the
    // next will), then what is left in equal parts of that size or less: a
    // launch costs about one chunk's serial parse however few chunks it holds,
    // so the count of sub-batches is what matters.
    const uint64_t rest = n - i0;
    uint64_t want = (uint64_t)n;
    if (used) {
      const uint64_t pct = L->h_tot[T_A] < C ? 75 : 95;
      uint64_t fit = (uint64_t)C * pct / 100 * m / used;
      if (fit < 1) fit = 1;
      L->fit_hint = pct == 95 ? (uint32_t)std::min<uint64_t>(fit * a0->maxd, 1u << 31) : 0u;
      const uint64_t k = rest ? (rest + fit - 1) / fit : 1;
      want = rest ? (rest + k - 1) / k : fit;
    }
    per = (uint32_t)(want < 1 ? 1 : (want > n ? n : want));
  }
  if (rounds_out) *rounds_out = rounds;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
