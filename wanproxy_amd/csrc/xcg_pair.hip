// XCodecCachePair (xcodec/xcodec_cache.h:140-237) of a bounded
// XCodecMemoryCache primary (:245-365, XCodecLRU xcodec/xcodec_lru.h) and an
// XCodecDisk secondary (xcodec/xcodec_cache_disk.{h,cc}): wanproxy.conf's
// cache, `memory` + `disk` under a `pair` (programs/wanproxy/wanproxy.conf:
// 8-26).  Stream-semantics encode and decode batches stay bit-exact with the
// sequential XCodecEncoder / XCodecDecoder on such a pair.  Everything --
// the pair's state and its policy -- lives on the GPU.
//
// Semantics (restated from the reference):
//   lookup(h)  primary hit: LRU use, then the disk's touch -- re-enter h if
//              the disk index lost it (:217-221, xcodec_cache_disk.cc:813-823);
//              else disk hit: enter h into the primary, evicting its LRU entry
//              at the limit (:223-227); else miss.
//   enter(h)   primary enter (may evict) and disk enter (:163-185).
//   disk       FIFO: entry number e goes to data block e mod nb*204; when an
//              index block of 204 entries fills, the write head moves to the
//              next one and the entries written there one lap earlier leave the
//              index (xcodec_cache_disk.cc:694-741, :327-382).
// A hash is visible while it is in either level.
//
// State in HBM.  Per front (one XCodecCache object): the primary's slots
// (pkey: hash, pdisk: the number of the same hash's disk entry) and its LRU
// order (lru[0 .. pcount), least recent first).  Per disk (shared by the fronts
// on it, as XCodecDisk is by its XCodecDiskCache front-ends): per data block
// the hash, the entry number written there (dent, NOENT when removed) and the
// writing front's xuid.  An entry's index block is invalidated when the write
// clock reaches 204 * (e / 204 + nb) (the write head entering that block one lap
// on), so liveness is a function of the clock and nothing is swept.  The pool
// holds C primary segments and the disk's data blocks; with HIP virtual memory
// the disk's blocks are ONE physical allocation mapped behind every front's
// primary, so `pool + id * 2048` addresses both and N fronts cost one disk.
//
// Division of work.  The parse (encode_stream_kernel, the same rounds as every
// stream batch) runs against G = one table over both levels (id s < C = primary
// slot s, id C + i = disk block i; a hash in both maps to its primary slot),
// takes per id the batch time from which the hash is gone from both levels
// (ptime) as given, and records every cache reference it makes (ENTER / HIT /
// GHIT / GMISS, xcg_cache.h).  The replay below recomputes the pair's state
// along those references with data-parallel passes instead of a sequential
// walk (tests/pair_model.py states the formulation and checks it against a
// sequential replay of the reference's policy):
//  * primary residency at a reference is an LRU stack distance: the entity of
//    reference j (previous reference p) is still in the primary iff fewer than
//    C distinct entities were referenced in (p, j), i.e. fewer than C
//    references k in (p, j) have their own previous reference before p.  The
//    primary's content at the start is a prefix of pseudo references in LRU
//    order.  Short gaps are decided by a prefix count; long ones by a block
//    table of 2-D prefix counts plus two partial block scans;
//  * evictions: the i-th miss of a full primary evicts the entity of the i-th
//    *terminal* reference (an entity's last reference before a miss of it, or
//    its last) in sequence order;
//  * the disk clock is the prefix count of appends (every enter, and every
//    primary hit on an entity whose disk entry has died: XCodecDisk::touch);
//    touches depend on the clock through the deaths, so the clock is the least
//    fixed point of "touches under this clock", reached by monotone rounds;
//  * presence at a lookup = primary residency or a live disk entry; a recorded
//    lookup that contradicts it flags its chunk, and the time each cached entity
//    leaves both levels becomes ptime for the re-parse.
// All consistent = the sequential encoder's result (by induction over stream
// time); otherwise the flagged chunks are parsed again under the new ptime.  An
// entry a sub-batch made must not leave both levels within it (the parse sees
// the batch's declarations to its end): a sub-batch writes less than a disk lap,
// which guarantees that.  The commit then places the final primary residents,
// writes the appended disk blocks and rebuilds G -- all on the device.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_radix_sort_config.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "xcg_cache.h"
#include "xcg_args.h"

namespace xcg {

constexpr uint32_t DISK_ENTRIES = 204;   // XCDFS_ENTRIES_PER_INDEX_BLOCK, xcodec_cache_disk.cc:87
constexpr uint64_t NOENT = ~0ull;        // no disk entry
constexpr uint64_t NOKEY = ~0ull;
constexpr uint64_t NEVERT = ~0ull;       // ptime: visible to the end
constexpr uint32_t NIL = 0xFFFFFFFFu;

// Position kinds.  A position is a pseudo reference (the primary at the start,
// LRU order) or a recorded row.
enum : uint8_t { K_PSEUDO = 0, K_ENTER = 1, K_LOOKUP = 2, K_GMISS = 3, K_SKIP = 4, K_REPL = 5 };

struct PairCnt {                          // device counters of one pass
  uint32_t split;                         // a row list overflowed: a smaller sub-batch
  uint32_t nbad;                          // recorded lookups the replay contradicts
  uint32_t unsorted;                      // a chunk's rows out of time order
  uint32_t changed;                       // touches moved (fixed-point round) / ptime moved (decode)
  uint32_t nslow;                         // stack-distance queries for the block table
  uint32_t nmove, nstage, nomiss;         // commit moves, staged moves
  uint32_t nohit;                         // (decode) a HIT with no earlier definer
  uint32_t pad[7];
};

struct PairDev {
  // the front
  uint32_t C, xuid, P;                    // limit, front id, primary entries at the start
  uint64_t* pkey;                         // [C]
  uint64_t* pdisk;                        // [C] number of the same hash's disk entry (NOENT)
  const uint32_t* lru;                    // [P] slots, least recent first
  uint64_t* ptime;                        // [C + D]
  // the disk
  uint32_t D, nb;
  uint64_t dclock0;
  uint64_t* dkey;                         // [D]
  uint64_t* dent;                         // [D]
  uint32_t* dxuid;                        // [D]
  // rows
  int dec;                                // decode rows (packed, REPLACE flags) vs encode rows
  uint32_t n, maxd, maxe;
  const uint4* ev;
  const uint32_t* nev;                    // encode: rows per chunk
  const uint64_t* base64;                 // decode: row base per chunk
  const uint64_t* cnt64;                  // decode: rows per chunk
  uint32_t* pbase;                        // encode: position base per chunk (exclusive scan) [n + 1]
  uint32_t* pcnt;                         // encode: rows per chunk [n + 1]
  // positions [np)
  uint32_t newb, etot, np;
  uint32_t* ent;                          // entity (decode REPL rows: the replaced entity)
  uint32_t* yent;                         // decode REPL rows: the new entity (else NIL)
  uint8_t* kind;
  uint64_t* tim;                          // stream time (chunk << 21 | t)
  uint64_t* hsh;
  uint32_t* skey;                         // sort input keys (entity, etot = none) / values (position)
  uint32_t* sval;
  uint32_t* sk;                           // sorted
  uint32_t* sv;
  int32_t* prv;                           // previous reference of the same entity (-1)
  int32_t* nxt;                           // next reference (-1)
  uint32_t* isr;                          // 1: a reference [np + 1]
  uint32_t* rc;                           // exclusive prefix of isr [np + 1]
  uint8_t* phit;                          // primary hit (a lookup / GMISS whose entity is resident)
  uint32_t* app;                          // appends at the position [np + 1]
  uint32_t* clk;                          // exclusive prefix of app [np + 1]
  uint32_t* elast;                        // [etot] position of the entity's last append (NIL)
  uint8_t* tflag;                         // [np] a touch at the position
  uint64_t* ddeath;                       // [np] death clock of the entity's disk entry current at the row
  uint32_t* erep;                         // [newb] (decode) position of the REPLACE that ends it (NIL)
  uint32_t* erun;                         // [etot] sorted index of the entity's first element (NIL)
  uint32_t* erend;                        // [etot] one past its last element
  uint64_t* einit;                        // [etot] disk entry current before the entity's first element
  uint32_t* ecov;                         // [etot] (leave) initial coverage end (NIL: to the end)
  uint32_t* egap;                         // [etot] (leave) first uncovered position found at a span start
  uint32_t* etail;                        // [etot] (leave) coverage end after the entity's last element
  uint64_t* sa;                           // [np + 1] segmented-scan input / output
  uint64_t* sb;
  uint32_t* nq;                           // [np + 1] next element of the run that can touch (NIL)
  uint8_t* tnew;                          // [np + 1] touches of the running round
  uint32_t* slow;                         // positions for the block table
  uint32_t* tab;                          // [nbk * (nbk + 1)] 2-D prefix counts
  uint32_t bsh, nbk;                      // table block = 1 << bsh positions
  uint32_t* f1;                           // misses / final residents [np + 1]
  uint32_t* f2;                           // terminals / new residents [np + 1]
  uint32_t* r1;                           // exclusive prefixes [np + 1]
  uint32_t* r2;
  uint32_t* missrow;                      // position of the i-th miss
  uint32_t* occ;                          // [C] slot kept / free list
  uint32_t* freel;                        // [C]
  uint32_t* lru2;                         // [C] the next LRU order
  uint4* moves;                           // commit moves
  PairCnt* cnt;
  HashTab bm;                             // hash -> ENTER position (encode)
  HashTab g;                              // the front's G (leave: which disk blocks are entities)
  uint32_t* need;                         // per chunk: flagged; earliest / latest contradicted time
  uint32_t* bad_t;
  uint32_t* bad_hi;
};

__device__ __forceinline__ uint64_t death_of(uint64_t e, uint32_t nb) {
  return e == NOENT ? 0ull : (uint64_t)DISK_ENTRIES * (e / DISK_ENTRIES + nb);
}

// The live disk entry an initial entity (id < newb) had at the pass start.
__device__ __forceinline__ uint64_t e0_of(const PairDev& d, uint32_t x) {
  uint64_t e;
  if (x < d.C) {
    e = d.pdisk[x];
  } else {
    const uint32_t i = x - d.C;
    if (d.dxuid[i] != d.xuid) return NOENT;
    e = d.dent[i];
  }
  if (e == NOENT || d.dent[e % d.D] != e || d.dclock0 >= death_of(e, d.nb)) return NOENT;
  return e;
}

__device__ __forceinline__ void mark_bad(const PairDev& d, uint64_t tm) {
  const uint32_t c = (uint32_t)(tm >> 21), t = (uint32_t)tm & 0x1FFFFFu;
  d.need[c] = 1u;
  atomicMin(d.bad_t + c, t);
  atomicMax(d.bad_hi + c, t);
  atomicAdd(&d.cnt->nbad, 1u);
}

__global__ __launch_bounds__(256) void pr_fill64_kernel(uint64_t* p, uint64_t n, uint64_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ __launch_bounds__(256) void pr_fill32_kernel(uint32_t* p, uint64_t n, uint32_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ __launch_bounds__(256) void pr_iota_kernel(uint32_t* p, uint32_t n, uint32_t base) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = base + i;
}

constexpr uint32_t HITMARK = 0xFFFFFFFEu;   // yent of a decode HIT row (resolved by hash)

// Encode: rows per chunk (a chunk whose list overflowed splits the sub-batch).
__global__ __launch_bounds__(256) void pr_count_kernel(PairDev d) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > d.n) return;
  if (c == d.n) { d.pcnt[c] = 0u; return; }
  const uint32_t m = d.nev[c];
  if (m > d.maxe) atomicOr(&d.cnt->split, 1u);
  d.pcnt[c] = m < d.maxe ? m : d.maxe;
}

// Pseudo references: the primary at the start, least recent first.
__global__ __launch_bounds__(256) void pr_pseudo_kernel(PairDev d) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= d.P) return;
  const uint32_t s = d.lru[r];
  d.ent[r] = s;
  d.yent[r] = NIL;
  d.kind[r] = K_PSEUDO;
  d.tim[r] = 0;
  d.hsh[r] = d.pkey[s];
  d.app[r] = 0u;
}

// Rows -> positions, one wave per chunk.  ENTER: a new entity numbered by its
// declaration row; GHIT / GMISS: the G id it found; HIT: resolved afterwards.
// Decode rows: a GHIT with the REPLACE flag (name reuse, xcodec_decoder.cc:
// 110-133) makes a new entity from the declaration row numbered with the
// ENTERs in op order; GMISS rows have no cache effect.
__global__ __launch_bounds__(256) void pr_rows_kernel(PairDev d) {
  const uint32_t c = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (c >= d.n) return;
  uint32_t m;
  uint64_t rb, pb;
  if (d.dec) {
    m = (uint32_t)d.cnt64[c];
    rb = d.base64[c];
    pb = d.P + d.base64[c];
  } else {
    m = min(d.nev[c], d.maxe);
    rb = (uint64_t)c * d.maxe;
    pb = d.P + d.pbase[c];
  }
  uint32_t ndecl = 0;
  for (uint32_t k0 = 0; k0 < m; k0 += 64) {
    const uint32_t k = k0 + (uint32_t)lane_id();
    const bool valid = k < m;
    const uint4 e = valid ? d.ev[rb + k] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t kd = e.w >> 30, ref = e.w & EV_REF_MASK;
    const bool rep = d.dec && (e.z >> 31) != 0u;
    const uint32_t t = d.dec ? (e.z & 0x7FFFFFFFu) : e.z;
    const bool isdecl = valid && d.dec && (kd == EV_ENTER || (kd == EV_GHIT && rep));
    const uint64_t dm = ballot(isdecl);
    const uint32_t dnum = ndecl + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
    ndecl += (uint32_t)__builtin_popcountll(dm);
    if (!valid) continue;
    if (k > 0 && (d.dec ? (d.ev[rb + k - 1].z & 0x7FFFFFFFu) : d.ev[rb + k - 1].z) > t) atomicOr(&d.cnt->unsorted, 1u);
    const uint64_t pos = pb + k;
    const uint64_t tm = ((uint64_t)c << 21) | t;
    d.tim[pos] = tm;
    d.hsh[pos] = ((uint64_t)e.y << 32) | e.x;
    d.yent[pos] = NIL;
    uint32_t x = NIL;
    uint8_t kk = K_SKIP;
    uint32_t a = 0u;
    if (kd == EV_ENTER) {
      if (ref < d.maxd) {
        x = d.newb + c * d.maxd + ref;
        kk = K_ENTER;
        a = 1u;
        if (!d.dec && !tab_insert_min(d.bm, e.x, e.y, pos)) atomicOr(&d.cnt->split, 2u);
      } else {
        atomicOr(&d.cnt->split, 4u);
      }
    } else if (kd == EV_HIT) {
      kk = K_LOOKUP;                                 // (entity resolved by pr_resolve_kernel)
      if (d.dec) d.yent[pos] = HITMARK;
    } else if (kd == EV_GHIT) {
      if (ref < d.newb) {
        x = ref;
        kk = K_LOOKUP;
        if (rep) {
          if (dnum < d.maxd) {
            kk = K_REPL;
            d.yent[pos] = d.newb + c * d.maxd + dnum;
            d.erep[ref] = (uint32_t)pos;
            a = 1u;
          } else {
            atomicOr(&d.cnt->split, 4u);
          }
        }
      } else if (!d.dec) {
        mark_bad(d, tm);
      }
    } else {                                         // EV_GMISS
      if (d.dec) {
        kk = K_SKIP;                                 // (decode: no cache effect)
      } else if (ref < d.newb) {
        x = ref;
        kk = K_GMISS;
      } else {
        mark_bad(d, tm);
      }
    }
    d.ent[pos] = x;
    d.kind[pos] = kk;
    d.app[pos] = a;
  }
}

// Decode definers of a hash for HIT resolution: ENTER / REPL rows (the entity
// they make) and GHIT rows (the cached entity); bm maps hash -> a chain head.
// A decode HIT resolves to the latest ENTER / REPL of its hash before it, else
// the first GHIT before it (XcgPairState's bmap: a GHIT puts only when absent,
// xcodec_decoder.cc's lookups).  Done by sorting (hash, position) pairs: see
// pr_dec_hits_kernel.
//
// Encode HIT resolution: the ENTER of the hash (the table holds the earliest;
// a second ENTER of a hash present in the sub-batch contradicts the replay).
__global__ __launch_bounds__(256) void pr_resolve_kernel(PairDev d) {
  const uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= d.np) return;
  uint8_t kk = d.kind[pos];
  if (pos >= d.P && !d.dec) {
    const uint64_t h = d.hsh[pos];
    if (kk == K_LOOKUP && d.ent[pos] == NIL) {
      const uint64_t v = tab_lookup_t(d.bm, (uint32_t)h, (uint32_t)(h >> 32));
      if (v != ~0ull && v < pos) {
        d.ent[pos] = d.ent[v];
      } else {
        kk = K_SKIP;
        d.kind[pos] = kk;
        mark_bad(d, d.tim[pos]);
      }
    } else if (kk == K_ENTER) {
      const uint64_t v = tab_lookup_t(d.bm, (uint32_t)h, (uint32_t)(h >> 32));
      if (v != pos) {                                // a second ENTER of a hash the sub-batch holds
        kk = K_SKIP;
        d.kind[pos] = kk;
        d.app[pos] = 0u;
        mark_bad(d, d.tim[pos]);
      }
    }
  }
  if (kk != K_SKIP && d.ent[pos] >= d.etot) {        // (a decode HIT with no definer: the pass returns -95)
    kk = K_SKIP;
    d.kind[pos] = kk;
  }
  const bool r = kk != K_SKIP && kk != K_GMISS;
  d.skey[pos] = kk == K_SKIP ? d.etot : d.ent[pos];
  d.sval[pos] = pos;
  d.isr[pos] = r ? 1u : 0u;
  if (pos == 0) { d.isr[d.np] = 0u; d.app[d.np] = 0u; }
}

// Segmented scans.  Runs (an entity's elements in the entity-sorted order, a
// hash's in the hash-sorted one) are numbered in ascending order, so a max-scan
// of (run << 32 | v) never carries a value across runs: an element's scan value
// belongs to its own run iff its upper half is the run's number.  v = 0 is
// "none"; indices and positions are stored + 1.
__device__ __forceinline__ uint64_t pk(uint32_t run, uint32_t v) { return ((uint64_t)run << 32) | v; }
__device__ __forceinline__ uint32_t in_run(uint64_t s, uint32_t run) { return (uint32_t)(s >> 32) == run ? (uint32_t)s : 0u; }

// Decode HIT resolution over rows sorted by (hash, position) (hk / hv, m rows):
// a HIT resolves to the latest ENTER / REPL of its hash before it, else to the
// first GHIT of the hash before it.  Step 1: run heads (-> run numbers by a
// scan); step 2: per run the first GHIT (atomicMin) and per row the packed
// latest-definer value (-> max-scan); step 3: the resolution.
__global__ __launch_bounds__(256) void pr_dh_heads_kernel(const uint64_t* hk, uint32_t m, uint32_t* head) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= m) head[i] = (i < m && (i == 0 || hk[i - 1] != hk[i])) ? 1u : 0u;
}
__global__ __launch_bounds__(256) void pr_dh_vals_kernel(PairDev d, const uint32_t* hv, uint32_t m, const uint32_t* head,
                                                         const uint32_t* hrank, uint32_t* fg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t r = hrank[i] + head[i] - 1u;        // this row's run
  const uint32_t q = hv[i];
  const uint8_t kq = d.kind[q];
  if (kq == K_LOOKUP && d.ent[q] != NIL && d.ent[q] < d.newb) atomicMin(fg + r, i);
  d.sa[i] = pk(r, (kq == K_ENTER || kq == K_REPL) ? i + 1u : 0u);
}
__global__ __launch_bounds__(256) void pr_dec_hits_kernel(PairDev d, const uint32_t* hv, uint32_t m, const uint32_t* head,
                                                          const uint32_t* hrank, const uint32_t* fg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t pos = hv[i];
  if (d.kind[pos] != K_LOOKUP || d.ent[pos] != NIL) return;
  const uint32_t r = hrank[i] + head[i] - 1u;
  const uint32_t v = in_run(d.sb[i], r);
  uint32_t x = NIL;
  if (v) {
    const uint32_t q = hv[v - 1u];
    x = d.kind[q] == K_ENTER ? d.ent[q] : d.yent[q];
  } else if (fg[r] < i) {
    x = d.ent[hv[fg[r]]];
  }
  if (x == NIL) {
    atomicOr(&d.cnt->nohit, 1u);
    return;
  }
  d.ent[pos] = x;
}

// Per sorted element: the entity's previous / next reference (GMISS rows are
// not references) and the bounds of each entity's run.  prv = the latest
// non-GMISS element before it in the run (an exclusive max-scan); each
// reference's successor is written by that successor (nxt starts at -1).
__global__ __launch_bounds__(256) void pr_link_vals_kernel(PairDev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint32_t e = d.sk[i];
  if (e >= d.etot) { d.sa[i] = pk(d.etot, 0u); return; }
  if (i == 0 || d.sk[i - 1] != e) d.erun[e] = i;
  if (i + 1 == d.np || d.sk[i + 1] != e) d.erend[e] = i + 1;
  d.sa[i] = pk(e, d.kind[d.sv[i]] != K_GMISS ? i + 1u : 0u);
}
__global__ __launch_bounds__(256) void pr_links_kernel(PairDev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint32_t e = d.sk[i];
  if (e >= d.etot) return;
  const uint32_t pos = d.sv[i];
  const uint32_t v = in_run(d.sb[i], e);
  const int32_t p = v ? (int32_t)d.sv[v - 1u] : -1;
  d.prv[pos] = p;
  if (p >= 0 && d.kind[pos] != K_GMISS) d.nxt[p] = (int32_t)pos;
}

// Decode REPLACE rows: the new entity continues the replaced one's place in
// the primary (the slot keeps its LRU position, xcodec_cache.h:187-196), so
// for the stack distance the replaced entity's references and the new one's
// form one chain through the REPLACE row.
__global__ __launch_bounds__(256) void pr_repl_links_kernel(PairDev d) {
  const uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= d.np || d.kind[pos] != K_REPL) return;
  const uint32_t y = d.yent[pos];
  const uint32_t i = d.erun[y];
  if (i == NIL) { d.nxt[pos] = -1; return; }
  // y's first reference (its run holds only references: HITs)
  const uint32_t q = d.sv[i];
  d.nxt[pos] = (int32_t)q;
  d.prv[q] = (int32_t)pos;
}

// Primary hits from the stack distance: short gaps by the reference count
// alone, the rest queued for the block table.
__global__ __launch_bounds__(256) void pr_hits_kernel(PairDev d) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d.np || j < d.P) return;
  const uint8_t kk = d.kind[j];
  uint8_t h = 0;
  if (kk == K_LOOKUP || kk == K_GMISS || kk == K_REPL) {
    const int32_t p = d.prv[j];
    if (p >= 0) {
      const uint32_t between = d.rc[j] - d.rc[p + 1];
      if (between < d.C) h = 1;
      else d.slow[atomicAdd(&d.cnt->nslow, 1u)] = j;
    }
  }
  d.phit[j] = h;
}

// Block table: H[b][v] = references k in block b whose previous reference is
// in block v - 1 (v = 0: none).
__global__ __launch_bounds__(256) void pr_tab_hist_kernel(PairDev d) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= d.np || !d.isr[k]) return;
  const int32_t p = d.prv[k];
  const uint32_t v = p < 0 ? 0u : ((uint32_t)p >> d.bsh) + 1u;
  atomicAdd(d.tab + (uint64_t)(k >> d.bsh) * (d.nbk + 1) + v, 1u);
}
// Row prefix over v (inclusive), one wave per row.
__global__ __launch_bounds__(256) void pr_tab_rows_kernel(PairDev d) {
  const uint32_t b = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (b >= d.nbk) return;
  uint32_t* row = d.tab + (uint64_t)b * (d.nbk + 1);
  uint32_t carry = 0;
  for (uint32_t v0 = 0; v0 <= d.nbk; v0 += 64) {
    const uint32_t v = v0 + (uint32_t)lane_id();
    const uint32_t x = v <= d.nbk ? row[v] : 0u;
    const uint32_t s = wave_incl_scan(x) + carry;
    if (v <= d.nbk) row[v] = s;
    carry = readlane(s, 63);
  }
}
// Column prefix over b (exclusive) in 32 segments: segment sums, their prefix,
// then each segment's rows.
constexpr uint32_t TSEG = 32;
__global__ __launch_bounds__(256) void pr_tab_cols_kernel(PairDev d, uint32_t* segsum, int phase) {
  const uint32_t w = d.nbk + 1;
  const uint32_t per = (d.nbk + TSEG - 1) / TSEG;
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (phase == 1) {                                  // prefix over the segments, per column
    if (id >= w) return;
    uint32_t acc = 0;
    for (uint32_t s = 0; s < TSEG; ++s) {
      const uint32_t x = segsum[(uint64_t)s * w + id];
      segsum[(uint64_t)s * w + id] = acc;
      acc += x;
    }
    return;
  }
  if (id >= (uint64_t)w * TSEG) return;
  const uint32_t v = (uint32_t)(id % w), s = (uint32_t)(id / w);
  const uint32_t b0 = s * per, b1 = min(d.nbk, b0 + per);
  if (phase == 0) {
    uint32_t acc = 0;
    for (uint32_t b = b0; b < b1; ++b) acc += d.tab[(uint64_t)b * w + v];
    segsum[(uint64_t)s * w + v] = acc;
  } else {
    uint32_t acc = segsum[(uint64_t)s * w + v];
    for (uint32_t b = b0; b < b1; ++b) {
      const uint32_t x = d.tab[(uint64_t)b * w + v];
      d.tab[(uint64_t)b * w + v] = acc;
      acc += x;
    }
  }
}
// One wave per queued position j (previous reference p):
//   count = T[jb][pb] + #{m in [pb*B, p): nxt(m) < jb*B} + #{k in [jb*B, j): prv(k) < p} - rc[p + 1]
// = distinct entities referenced in (p, j); a hit iff < C.
__global__ __launch_bounds__(256) void pr_tab_query_kernel(PairDev d) {
  const uint32_t q = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (q >= d.cnt->nslow) return;
  const uint32_t j = d.slow[q];
  const uint32_t p = (uint32_t)d.prv[j];
  const uint32_t jb = j >> d.bsh, pb = p >> d.bsh;
  uint32_t cnt = d.tab[(uint64_t)jb * (d.nbk + 1) + pb];
  const uint32_t lim1 = jb << d.bsh;
  for (uint32_t m = (pb << d.bsh) + (uint32_t)lane_id(); m < p + 63u; m += 64) {
    const bool ok = m < p && d.isr[m] && d.nxt[m] >= 0 && (uint32_t)d.nxt[m] < lim1;
    cnt += (uint32_t)__builtin_popcountll(ballot(ok));
  }
  for (uint32_t k = lim1 + (uint32_t)lane_id(); k < j + 63u; k += 64) {
    const bool ok = k < j && d.isr[k] && d.prv[k] < (int32_t)p;
    cnt += (uint32_t)__builtin_popcountll(ballot(ok));
  }
  cnt -= d.rc[p + 1];
  if (lane_id() == 0) d.phit[j] = cnt < d.C ? 1 : 0;
}

// The disk entry a REPLACE-made entity starts with: the REPLACE row's append
// (after the replaced entity's touch there, if any).
__device__ __forceinline__ uint64_t repl_entry(const PairDev& d, uint32_t rp) {
  return d.dclock0 + d.clk[rp] + d.tflag[rp];
}

// One fixed-point round of the disk clock.  Per entity, in stream order: the
// entity's current disk entry (the initial one, its ENTER's, or its last
// touch's) and, at every primary hit, a touch if that entry has died by the
// row's clock (XCodecDisk::touch re-enters the hash; an entry can die and be
// re-entered more than once when the sub-batch laps a small disk).  Each row
// also records the death clock of the entry current at it (presence checks).
//
// Without walking a run: the touches of an entity are a chain -- from the
// current entry (clock c), the next touch is the first element that can touch
// (nq: a primary-hit lookup / REPLACE) at or after the first element whose clock
// reaches death(c) (a binary search: clocks grow along the run).  A chain is as
// long as the entity's entries die, at most a few per sub-batch.  Then every
// row's current entry is its run's latest setter (ENTER / touch) before it: an
// exclusive max-scan (pr_touch_rows_kernel).
__global__ __launch_bounds__(256) void pr_nq_vals_kernel(PairDev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint32_t e = min(d.sk[i], d.etot);
  const uint32_t pos = d.sv[i];
  const uint8_t kk = d.kind[pos];
  const bool can = e < d.etot && pos >= d.P && (kk == K_LOOKUP || kk == K_REPL) && d.phit[pos];
  d.sa[d.np - 1u - i] = pk(e, can ? i : NIL);        // (reversed: a min-scan finds the next one)
}
__global__ __launch_bounds__(256) void pr_nq_kernel(PairDev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint64_t s = d.sb[d.np - 1u - i];
  d.nq[i] = (uint32_t)(s >> 32) == d.sk[i] ? (uint32_t)s : NIL;
}
__global__ __launch_bounds__(256) void pr_touch_chain_kernel(PairDev d) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.etot) return;
  const uint32_t i0 = d.erun[e];
  if (i0 == NIL) return;
  const uint32_t i1 = d.erend[e];
  uint64_t cur = NOENT;
  uint32_t last = NIL, start = i0;
  if (e < d.newb) {
    cur = e0_of(d, e);
  } else {
    const uint32_t p0 = d.sv[i0];
    if (d.kind[p0] == K_ENTER) {
      last = p0;
      start = i0 + 1u;
    } else {                                         // a REPLACE-made entity: its first row is a HIT
      const int32_t rp = d.prv[p0];
      if (rp >= 0 && d.kind[rp] == K_REPL) cur = repl_entry(d, (uint32_t)rp);
    }
  }
  d.einit[e] = cur;
  if (last != NIL) cur = d.dclock0 + d.clk[last];
  for (int guard = 0; guard < (1 << 20) && start < i1; ++guard) {
    const uint64_t dth = death_of(cur, d.nb);
    uint32_t lo = start, hi = i1;                    // first element whose clock reaches dth
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (d.dclock0 + d.clk[d.sv[mid]] >= dth) hi = mid; else lo = mid + 1u;
    }
    if (lo >= i1) break;
    const uint32_t j = d.nq[lo];
    if (j == NIL || j >= i1) break;
    const uint32_t pos = d.sv[j];
    d.tnew[pos] = 1u;
    cur = d.dclock0 + d.clk[pos];
    last = pos;
    start = j + 1u;
  }
  d.elast[e] = last;
}
__global__ __launch_bounds__(256) void pr_setter_vals_kernel(PairDev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint32_t e = min(d.sk[i], d.etot);
  const uint32_t pos = d.sv[i];
  const bool set = e < d.etot && pos >= d.P && (d.kind[pos] == K_ENTER || d.tnew[pos]);
  d.sa[i] = pk(e, set ? d.clk[pos] + 1u : 0u);
}
__global__ __launch_bounds__(256) void pr_touch_rows_kernel(PairDev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t chg = 0;
  if (i < d.np) {
    const uint32_t e = d.sk[i], pos = d.sv[i];
    if (e < d.etot && pos >= d.P) {
      const uint32_t v = in_run(d.sb[i], e);
      const uint64_t cur = v ? d.dclock0 + (v - 1u) : d.einit[e];
      d.ddeath[pos] = death_of(cur, d.nb);
      const uint8_t t = d.tnew[pos];
      d.tnew[pos] = 0u;
      if (d.tflag[pos] != t) {
        d.tflag[pos] = t;
        chg = 1u;
      }
      const uint8_t kk = d.kind[pos];
      d.app[pos] = ((kk == K_ENTER || kk == K_REPL) ? 1u : 0u) + t;
    }
  }
  const uint64_t m = ballot(chg != 0u);
  if (lane_id() == 0 && m) atomicAdd(&d.cnt->changed, (uint32_t)__builtin_popcountll(m));
}

// Presence at every recorded lookup: primary residency or a live disk entry.
// Encode: a lookup the parse recorded the other way flags its chunk; a lookup
// of an entity the sub-batch made and lost again splits the sub-batch (the
// parse sees the batch's declarations to its end).  Decode: HITs only.
__global__ __launch_bounds__(256) void pr_check_kernel(PairDev d) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d.np || j < d.P) return;
  const uint8_t kk = d.kind[j];
  if (kk != K_LOOKUP && kk != K_GMISS) return;
  if (d.dec && d.yent[j] != HITMARK) return;
  const uint32_t x = d.ent[j];
  const bool present = d.phit[j] || d.dclock0 + d.clk[j] < d.ddeath[j];
  if (d.dec || x >= d.newb) {
    if (!present) atomicOr(&d.cnt->split, 8u);
  } else if (present != (kk == K_LOOKUP)) {
    mark_bad(d, d.tim[j]);
  }
}

// Misses (references that enter the primary) and terminal references (the
// last before a miss of the same entity, or the last).
__global__ __launch_bounds__(256) void pr_missterm_kernel(PairDev d) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > d.np) return;
  uint32_t miss = 0, term = 0;
  if (k < d.np && d.isr[k]) {
    miss = k >= d.P && !d.phit[k] ? 1u : 0u;
    const int32_t nx = d.nxt[k];
    term = (nx < 0 || !d.phit[nx]) ? 1u : 0u;
  }
  d.f1[k] = miss;
  d.f2[k] = term;
}
__global__ __launch_bounds__(256) void pr_missrow_kernel(PairDev d) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < d.np && d.f1[k]) d.missrow[d.r1[k]] = k;
}

// Position at which the entity of terminal reference k is evicted (NIL: not
// in this sub-batch).  M misses, the i-th (1-based) evicts once i > C - P.
__device__ __forceinline__ uint32_t evict_pos(const PairDev& d, uint32_t k, uint32_t M) {
  const int64_t i = (int64_t)d.r2[k] + 1 + ((int64_t)d.C - (int64_t)d.P);
  return (i >= 1 && i <= (int64_t)M) ? d.missrow[i - 1] : NIL;
}

// The position whose append brings the clock to `death` (the entry is dead
// after it), or NIL when the sub-batch does not get there.
__device__ __forceinline__ uint32_t death_row(const PairDev& d, uint64_t death) {
  if (d.dclock0 + d.clk[d.np] < death) return NIL;
  uint32_t lo = d.P, hi = d.np - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (d.dclock0 + d.clk[mid + 1] >= death) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// ptime for the next parse: per id, the batch time from which the hash is in
// neither level (NEVERT: not within the sub-batch; 0: gone at its start) = the
// first position no primary span [reference, its exit) and no disk span
// [append, death) covers.  Decode: also whether anything moved (the
// classification repeats until not).
//
// Spans start at the entity's elements, which are in position order, so the
// first uncovered position is found with a max-scan instead of a walk: X(k) =
// max(P, initial coverage, ends of the spans of elements before k); the first
// element k starting past X(k) leaves a gap at X(k); without one the coverage
// ends at X after the last element.
__global__ __launch_bounds__(256) void pr_cover_kernel(PairDev d) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= d.newb) return;
  const uint64_t e0 = e0_of(d, id);
  d.ecov[id] = e0 == NOENT ? d.P : death_row(d, death_of(e0, d.nb));
  d.egap[id] = NIL;
  d.etail[id] = NIL;
}
// encoded span end: 0 none, NIL to the end, else end + 1
__device__ __forceinline__ uint32_t span_end(const PairDev& d, uint32_t pos, uint8_t kk, uint32_t M) {
  if (kk == K_GMISS) return 0u;
  if (kk == K_REPL) return NIL;                      // (gone at the REPLACE: pr_leave_kernel)
  const int32_t nx = d.nxt[pos];
  const uint32_t b = (nx >= 0 && d.phit[nx]) ? (uint32_t)nx : evict_pos(d, pos, M);
  uint32_t end = b == NIL ? NIL : b + 1u;
  if (pos >= d.P && d.tflag[pos]) {                  // a touch's disk span [touch, death)
    const uint32_t t = death_row(d, death_of(d.dclock0 + d.clk[pos], d.nb));
    end = max(end, t == NIL ? NIL : t + 1u);
  }
  return end;
}
__global__ __launch_bounds__(256) void pr_span_vals_kernel(PairDev d, uint32_t M) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint32_t e = min(d.sk[i], d.etot);
  d.sa[i] = pk(e, e < d.newb ? span_end(d, d.sv[i], d.kind[d.sv[i]], M) : 0u);
}
__global__ __launch_bounds__(256) void pr_gaps_kernel(PairDev d, uint32_t M) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.np) return;
  const uint32_t e = d.sk[i];
  if (e >= d.newb) return;
  const uint32_t pos = d.sv[i];
  const uint32_t v = in_run(d.sb[i], e);
  uint32_t x = max(d.ecov[e], d.P);                  // (NIL: covered to the end)
  if (v) x = max(x, v == NIL ? NIL : v - 1u);
  const uint32_t own = (uint32_t)d.sa[i];            // (this element's encoded end)
  if (own && x != NIL && pos > x) atomicMin(d.egap + e, x);
  if (i + 1u == d.erend[e]) d.etail[e] = (own == 0u || x == NIL) ? x : max(x, own == NIL ? NIL : own - 1u);
}
__global__ __launch_bounds__(256) void pr_leave_kernel(PairDev d) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= d.newb) return;
  uint64_t pt = NEVERT;
  bool entity;
  if (id < d.C) {
    entity = d.pkey[id] != NOKEY;
  } else {
    const uint32_t i = id - d.C;
    const uint64_t k = d.dkey[i];
    entity = d.dxuid[i] == d.xuid && d.dent[i] != NOENT && k != NOKEY &&
             tab_lookup_t(d.g, (uint32_t)k, (uint32_t)(k >> 32)) == id;
  }
  if (entity) {
    const bool present_at_start = id < d.C || e0_of(d, id) != NOENT;
    if (!present_at_start) {
      pt = 0;
    } else {
      uint32_t lv = d.egap[id];
      if (lv == NIL) {
        const uint32_t x = d.erun[id] == NIL ? max(d.ecov[id], d.P) : d.etail[id];
        lv = x < d.np ? x : NIL;
      }
      const uint32_t rp = d.dec ? d.erep[id] : NIL;  // replaced: gone right after its own lookup
      if (rp != NIL && (lv == NIL || lv > rp)) pt = d.tim[rp] + 1;
      else if (lv != NIL) pt = d.tim[lv];
    }
  }
  if (d.ptime[id] != pt) {
    d.ptime[id] = pt;
    atomicOr(&d.cnt->changed, 1u);
  }
}

// Commit, step 1: the final primary residents -- last references that are
// terminal and not evicted -- and the slots initial residents keep.
// E = P + M - C primary evictions, M (the misses) read on the device: the
// commit needs no readback before it.
__global__ __launch_bounds__(256) void pr_final_kernel(PairDev d, const uint32_t* Mp) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > d.np) return;
  const int64_t e64 = (int64_t)d.P + (int64_t)*Mp - (int64_t)d.C;
  const uint32_t E = e64 > 0 ? (uint32_t)e64 : 0u;
  uint32_t fin = 0, nw = 0;
  if (k < d.np && d.isr[k] && d.nxt[k] < 0 && d.r2[k] >= E) {
    const uint32_t x = d.kind[k] == K_REPL ? d.yent[k] : d.ent[k];
    fin = 1u;
    if (x < d.C) d.occ[x] = 1u;
    else nw = 1u;
  }
  d.f1[k] = fin;
  d.f2[k] = nw;
}
// step 2: free slots (never used, or an initial resident's that left)
__global__ __launch_bounds__(256) void pr_free_kernel(PairDev d, const uint32_t* frank) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= d.C) return;
  if (!d.occ[s]) {
    d.freel[frank[s]] = s;
    d.pkey[s] = NOKEY;
    d.pdisk[s] = NOENT;
  }
}

__device__ __forceinline__ void add_move(const PairDev& d, uint32_t dest, uint32_t x) {
  const uint32_t j = atomicAdd(&d.cnt->nmove, 1u);
  if (x >= d.newb) {
    const uint32_t r = x - d.newb;
    d.moves[j] = make_uint4(dest, 0u, r / d.maxd, r % d.maxd);
  } else {
    d.moves[j] = make_uint4(dest, 1u, x, atomicAdd(&d.cnt->nstage, 1u));
  }
}

// The disk entry an entity holds at the end of the sub-batch (NOENT: none).
__device__ __forceinline__ uint64_t final_disk(const PairDev& d, uint32_t x, uint64_t dend) {
  uint64_t e = NOENT;
  const uint32_t la = d.elast[x];
  if (la != NIL) {
    e = d.dclock0 + d.clk[la];                       // (an ENTER's or a touch's: the row's first append)
  } else if (x >= d.newb) {                          // a REPLACE-made entity never touched
    const uint32_t i = d.erun[x];
    if (i != NIL) {
      const int32_t rp = d.prv[d.sv[i]];
      if (rp >= 0 && d.kind[rp] == K_REPL) e = repl_entry(d, (uint32_t)rp);
    }
  } else {
    e = e0_of(d, x);
  }
  return (e != NOENT && dend < death_of(e, d.nb)) ? e : NOENT;
}

// step 3: place every final resident (new LRU order; new slots from the free
// list), with its key, disk link and, for a new slot, a byte move.
__global__ __launch_bounds__(256) void pr_place_kernel(PairDev d, uint64_t dend) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= d.np || !d.f1[k]) return;
  const uint32_t x = d.kind[k] == K_REPL ? d.yent[k] : d.ent[k];
  uint32_t s;
  if (x < d.C) {
    s = x;
  } else {
    s = d.freel[d.r2[k]];
    add_move(d, s, x);
  }
  d.lru2[d.r1[k]] = s;
  d.pkey[s] = d.hsh[k];
  uint64_t fd = NOENT;
  if (x == NIL) return;
  if (d.kind[k] == K_REPL && x == d.yent[k]) {
    // new bytes under the replaced name: the append at this row after the touch (if any)
    fd = repl_entry(d, k);
    if (dend >= death_of(fd, d.nb)) fd = NOENT;
  } else {
    fd = final_disk(d, x, dend);
  }
  d.pdisk[s] = fd;
}

// step 4: the disk appends: per appending position the entry number, the data
// block, its key and owner, and a byte move -- for the last write into each
// block only (a small disk can be lapped within a sub-batch).  A REPLACE row
// appends the new entity after the replaced one's touch; the replaced entity's
// current entry leaves the index (XCodecDisk::remove).
__device__ __forceinline__ void disk_write(const PairDev& d, uint64_t e, uint64_t dend, uint64_t key, uint32_t x,
                                           bool removed) {
  if (e + d.D < dend) return;                        // (written over later in this sub-batch)
  const uint32_t i = (uint32_t)(e % d.D);
  d.dkey[i] = key;                                   // (the volume's index entry, even when removed)
  d.dent[i] = removed ? NOENT : e;
  d.dxuid[i] = d.xuid;
  if (!removed) add_move(d, d.C + i, x);
}
__global__ __launch_bounds__(256) void pr_append_kernel(PairDev d, uint64_t dend) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d.np || j < d.P || !d.app[j]) return;
  const uint8_t kk = d.kind[j];
  uint64_t e = d.dclock0 + d.clk[j];
  const uint32_t x = d.ent[j];
  if (d.tflag[j]) {                                  // a touch of x
    const bool removed = kk == K_REPL || (d.dec && x < d.newb && d.erep[x] != NIL && d.elast[x] == j);
    disk_write(d, e, dend, d.hsh[j], x, removed);
    ++e;
  }
  if (kk == K_ENTER) disk_write(d, e, dend, d.hsh[j], x, false);
  if (kk == K_REPL) disk_write(d, e, dend, d.hsh[j], d.yent[j], false);
}

// Decode REPLACE of an entity that appended nothing in this batch: its
// initial entry leaves the index (unless this batch wrote over that block).
__global__ __launch_bounds__(256) void pr_remove_kernel(PairDev d, uint64_t dend) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d.np || d.kind[j] != K_REPL) return;
  const uint32_t x = d.ent[j];
  if (x >= d.newb || d.elast[x] != NIL) return;
  const uint64_t e0 = e0_of(d, x);
  if (e0 == NOENT || e0 + d.D < dend) return;
  const uint32_t i = (uint32_t)(e0 % d.D);
  d.dent[i] = NOENT;                                 // (XCodecDisk::remove leaves the volume's index block as it is)
}

// Commit moves: w = (destination pool index, kind, a, b); kind 0: the bytes of
// declaration b of chunk a (input), kind 1: the pre-batch bytes of pool index a
// (staged first into staging slot b, so no move reads what another overwrote).
__global__ __launch_bounds__(256) void pair_stage_kernel(const uint4* w, const PairCnt* cnt, const uint8_t* pool,
                                                         uint8_t* staging) {
  const uint32_t j = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (j >= cnt->nmove) return;
  const uint4 m = w[j];
  if (m.y != 1u) return;
  const uint8_t* src = pool + (uint64_t)m.z * SEG;
  uint8_t* dst = staging + (uint64_t)m.w * SEG;
  const int l = lane_id();
  *(u32x4_u*)(dst + 32 * l) = *(const u32x4_u*)(src + 32 * l);
  *(u32x4_u*)(dst + 32 * l + 16) = *(const u32x4_u*)(src + 32 * l + 16);
}

// Four moves per wave (MOVES_PER_WAVE): their job words, then their source
// addresses, then all eight 16-byte loads per lane are in flight before the
// first store -- one chain of round trips per four 2 KiB copies instead of one
// per copy (the commit's largest kernel: ~2 GB per GiB of C5).
constexpr uint32_t MOVES_PER_WAVE = 4;
__global__ __launch_bounds__(256) void pair_move_kernel(const uint4* w, const PairCnt* cnt, const uint8_t* in,
                                                        const uint64_t* chunk_off, const uint4* decl, uint32_t maxd,
                                                        const uint8_t* staging, uint8_t* pool) {
  const uint32_t j0 = (blockIdx.x * 4u + readfirst(threadIdx.x >> 6)) * MOVES_PER_WAVE;
  const uint32_t nm = readfirst(cnt->nmove);
  if (j0 >= nm) return;
  const int l = lane_id();
  uint4 m[MOVES_PER_WAVE];
#pragma unroll
  for (int t = 0; t < (int)MOVES_PER_WAVE; ++t) m[t] = w[min(j0 + (uint32_t)t, nm - 1u)];
  uint64_t co[MOVES_PER_WAVE];
  uint32_t dz[MOVES_PER_WAVE];
#pragma unroll
  for (int t = 0; t < (int)MOVES_PER_WAVE; ++t) {     // (kind 0: where the declaration's bytes are)
    co[t] = 0ull;
    dz[t] = 0u;
    if (m[t].y == 0u) {
      co[t] = chunk_off[m[t].z];
      dz[t] = decl[(uint64_t)m[t].z * maxd + m[t].w].z;
    }
  }
  u32x4 v[MOVES_PER_WAVE][2];
#pragma unroll
  for (int t = 0; t < (int)MOVES_PER_WAVE; ++t) {
    const uint8_t* src = m[t].y == 0u ? in + co[t] + dz[t] : staging + (uint64_t)m[t].w * SEG;
    v[t][0] = *(const u32x4_u*)(src + 32 * l);
    v[t][1] = *(const u32x4_u*)(src + 32 * l + 16);
  }
#pragma unroll
  for (int t = 0; t < (int)MOVES_PER_WAVE; ++t) {
    if (j0 + (uint32_t)t >= nm) break;
    uint8_t* dst = pool + (uint64_t)m[t].x * SEG;
    *(u32x4_u*)(dst + 32 * l) = v[t][0];
    *(u32x4_u*)(dst + 32 * l + 16) = v[t][1];
  }
}

struct PairWipe {
  HashTab g;
  uint32_t* filt;
  u32x4* ftab; uint32_t ftab_n;
  uint32_t* gfilt; uint32_t gfilt_n;
  uint32_t* nseg;
};
__global__ __launch_bounds__(256) void pair_wipe_kernel(PairWipe w) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = i0; i <= w.g.mask; i += stride) { w.g.keys[i] = EMPTY_KEY; w.g.vals[i] = ~0ull; }
  for (uint64_t i = i0; i < FILT_WORDS; i += stride) w.filt[i] = 0u;
  for (uint64_t i = i0; i < w.ftab_n; i += stride) w.ftab[i] = u32x4{0u, 0u, 0u, 0u};
  for (uint64_t i = i0; i < w.gfilt_n; i += stride) w.gfilt[i] = 0u;
  if (i0 == 0) *w.nseg = 0u;
}

// G from the state: every primary slot with a hash, and every live disk entry
// of this front (a hash in both levels maps to its primary slot: the smaller id).
__global__ __launch_bounds__(256) void pair_rebuild_kernel(const uint64_t* pkey, uint32_t C, const uint64_t* dkey,
                                                           const uint64_t* dent, const uint32_t* dxuid, uint32_t D,
                                                           uint32_t nb, uint32_t xuid, uint64_t dclock, HashTab g,
                                                           FiltSet fs, uint32_t* nseg, int32_t* status) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t k = EMPTY_KEY;
  if (id < C) {
    k = pkey[id];
  } else if (id < C + D) {
    const uint32_t i = id - C;
    const uint64_t e = dent[i];
    if (dxuid[i] == xuid && e != NOENT && dclock < death_of(e, nb)) k = dkey[i];
  }
  const bool have = k != EMPTY_KEY;
  // (the table insert and the three filters with the short chain of returning
  // atomics: two round trips per key instead of about four)
  if (have && !tab_insert_min_filt(g, fs, (uint32_t)k, (uint32_t)(k >> 32), id)) atomicOr(status, 2);
  const uint64_t m = ballot(have);
  if (lane_id() == 0 && m) atomicAdd(nseg, (uint32_t)__builtin_popcountll(m));
}

// First guess of a sub-batch's references, before any parse: every chunk
// parses as its 2048-byte tiling (its cold parse), a tile found in G being a
// lookup hit, a repeat of an earlier tile of the batch a hit on that
// declaration, and every other tile a declaration, entered while the window
// 2048 bytes on (or after the last window) is examined.  One event per tile,
// in the same row format the parse records.
__global__ __launch_bounds__(256) void pair_seed_table_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                              uint32_t maxd, HashTab b, int32_t* status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (uint32_t)(i / maxd), dd = (uint32_t)(i % maxd);
  if (c >= n || dd >= ndecl[c]) return;
  const uint4 r = decl[i];
  if (!tab_insert_min(b, r.x, r.y, ((uint64_t)c << 32) | r.z)) atomicOr(status, 2);
}
__global__ __launch_bounds__(256) void pair_seed_events_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                               uint32_t maxd, const uint32_t* chunk_len, HashTab g,
                                                               HashTab b, uint4* ev, uint32_t* nev, uint32_t maxe,
                                                               const uint64_t* ptime) {
  const uint32_t c = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (c >= n) return;
  const uint32_t nd = min(ndecl[c], maxe / 2u), last = chunk_len[c] - SEG;
  uint32_t row = 0;
  for (uint32_t k0 = 0; k0 < nd; k0 += 64) {
    const uint32_t k = k0 + (uint32_t)lane_id();
    uint4 r0 = make_uint4(0u, 0u, 0u, 0u), r1 = r0;
    uint32_t nr = 0;
    if (k < nd) {
      const uint4 dd = decl[(uint64_t)c * maxd + k];
      const uint64_t gv = tab_lookup_t(g, dd.x, dd.y);
      const uint32_t th = 2u * dd.z + 1u, te = dd.z + SEG <= last ? 2u * (dd.z + SEG) : 2u * (last + 1u);
      if (gv != ~0ull && (!ptime || ((((uint64_t)c << 21) | th) < ptime[gv]))) {
        r0 = make_uint4(dd.x, dd.y, th, (EV_GHIT << 30) | (uint32_t)gv);
        nr = 1;
      } else {
        // gone from both levels by now (with ptime: the guess before this one)
        // or never cached: a declaration if it is the batch's earliest tile of
        // the hash, or if that earliest tile found the entry before it left
        const uint64_t e = tab_lookup_t(b, dd.x, dd.y);
        bool enter = e == (((uint64_t)c << 32) | dd.z);
        if (!enter && gv != ~0ull)
          enter = ((((e >> 32) << 21) | (2u * (uint32_t)e + 1u)) < ptime[gv]);
        if (gv != ~0ull) r0 = make_uint4(dd.x, dd.y, th, (EV_GMISS << 30) | (uint32_t)gv);
        const uint4 second = enter ? make_uint4(dd.x, dd.y, te, (EV_ENTER << 30) | k)
                                   : make_uint4(dd.x, dd.y, th, EV_HIT << 30);
        if (gv != ~0ull) { r1 = second; nr = 2; }
        else { r0 = second; nr = 1; }
      }
    }
    // rows in tile order (a GMISS precedes its tile's ENTER; an ENTER at window
    // + 2048 precedes the next tile's lookup one position later)
    const uint32_t inc = wave_incl_scan(nr);
    const uint32_t o = row + inc - nr;
    if (nr > 0) ev[(uint64_t)c * maxe + o] = r0;
    if (nr > 1) ev[(uint64_t)c * maxe + o + 1] = r1;
    row += readlane(inc, 63);
  }
  if (lane_id() == 0) nev[c] = row;
}

// Statistics: this front's live disk entries (xuid) or every live entry (xuid ~0).
__global__ __launch_bounds__(256) void pair_count_live_kernel(const uint64_t* dent, const uint32_t* dxuid, uint32_t D,
                                                              uint32_t nb, uint64_t dclock, uint32_t xuid,
                                                              uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool live = false;
  if (i < D) {
    const uint64_t e = dent[i];
    live = e != NOENT && dclock < death_of(e, nb) && (xuid == NIL || dxuid[i] == xuid);
  }
  const uint64_t m = ballot(live);
  if (lane_id() == 0 && m) atomicAdd(out, (uint32_t)__builtin_popcountll(m));
}

// A front goes away or is cleared: its disk entries leave the index (the
// volume's index blocks keep them unless the whole volume is reset).
__global__ __launch_bounds__(256) void pair_drop_front_kernel(uint64_t* dkey, uint64_t* dent, const uint32_t* dxuid,
                                                              uint32_t D, uint32_t xuid) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < D && (xuid == NIL || dxuid[i] == xuid)) {
    dent[i] = NOENT;
    if (xuid == NIL) dkey[i] = NOKEY;
  }
}

}  // namespace xcg

// ---------------------------------------------------------------------------
// Host side: the state objects and the passes' drivers.

struct XcgPairState;

// One XCodecDisk: the ring's blocks (device arrays) and the fronts on it.
struct XcgDiskState {
  uint64_t nb = 0;                 // index blocks
  uint32_t D = 0;                  // nb * 204 data blocks
  uint64_t dclock = 0;             // entries written to the disk (every front)
  int device = -1;                 // bound by the first front
  uint64_t* dkey = nullptr;
  uint64_t* dent = nullptr;
  uint32_t* dxuid = nullptr;
  // the data blocks' bytes: one physical allocation mapped behind every front's primary
  uint32_t flags = 0;              // XCG_DISK_* (xcgpu.h)
  int tier = -1;                   // where the blocks live: 0 HBM, 1 pinned host memory (-1: not yet)
  bool vmm = false;
  hipMemGenericAllocationHandle_t pool_h{};
  size_t pool_bytes = 0;
  void* dva = nullptr;             // the disk's own mapping of pool_h, for its whole life (xcg_disk_save)
  std::vector<XcgPairState*> fronts;   // by xuid (nullptr: free)
  // the volume (xcodec_cache_disk.cc:72-101): its size, per index block the
  // counter it was last written with, the counter of the block being filled,
  // the registry's blocks and the UUID each xuid has there
  uint64_t bytes = 0;
  std::vector<uint64_t> ctr;
  uint64_t ibc = 1;
  std::vector<uint8_t> reg;
  std::vector<std::string> uuid;
  // a reopened volume's ring, waiting for the first front's device
  bool pending = false;
  bool ring_loaded = false;
  bool zeroed = false;             // a fresh volume's blocks read as zeros (as the reference's ftruncate'd file)
  std::vector<uint64_t> h_key, h_ent;
  std::vector<uint32_t> h_xuid;
  std::vector<uint8_t> h_data;
  // without HIP virtual memory every front has its own copy of the blocks: a
  // front that goes away leaves the blocks it wrote here (shadow_ok: per block)
  std::vector<uint8_t> shadow, shadow_ok;
  int refs = 1;                    // the creator's reference + one per front
};

struct XcgPairState {
  uint32_t C = 0;                  // primary limit in segments
  // XCodecCachePair over an unbounded XCodecMemoryCache (limit 0: enter never
  // evicts, xcodec_cache.h:303-318): C is then only the primary's capacity,
  // and a commit that would evict fails (XCG_EOVERFLOW) instead
  bool unbounded = false;
  uint32_t D = 0, nb = 0;
  XcgDiskState* disk = nullptr;
  uint16_t xuid = 0;
  uint32_t pcount = 0;             // primary entries
  uint64_t gclock = 0;             // disk clock when G was last rebuilt
  bool gstale = false;
  // device state
  uint64_t* pkey = nullptr;        // [C]
  uint64_t* pdisk = nullptr;       // [C]
  uint32_t* lru = nullptr;         // [C]
  uint32_t* lru2 = nullptr;        // [C]
  uint64_t* ptime = nullptr;       // [C + D]
  // the pool (C primary segments, then the disk's blocks)
  uint8_t* pool = nullptr;
  bool pool_vmm = false;
  void* va = nullptr;
  size_t va_bytes = 0, prim_bytes = 0;
  hipMemGenericAllocationHandle_t prim_h{};
  // pass scratch, grown on demand
  uint64_t np_cap = 0, n_cap = 0, et_cap = 0, tab_cap = 0, stg_cap = 0, tmp_cap = 0, bm_cap = 0, hk_cap = 0;
  uint32_t* ent = nullptr; uint32_t* yent = nullptr; uint8_t* kind = nullptr; uint64_t* tim = nullptr;
  uint64_t* hsh = nullptr; uint32_t* skey = nullptr; uint32_t* sval = nullptr; uint32_t* sk = nullptr;
  uint32_t* sv = nullptr; int32_t* prv = nullptr; int32_t* nxt = nullptr; uint32_t* isr = nullptr;
  uint32_t* rc = nullptr; uint8_t* phit = nullptr; uint32_t* app = nullptr; uint32_t* clk = nullptr;
  uint32_t* slow = nullptr; uint32_t* f1 = nullptr; uint32_t* f2 = nullptr; uint32_t* r1 = nullptr;
  uint32_t* r2 = nullptr; uint32_t* missrow = nullptr; uint4* moves = nullptr;
  uint32_t* pbase = nullptr;       // [n + 1]
  uint32_t* pcnt = nullptr;        // [n + 1]
  uint32_t* elast = nullptr;       // [etot]
  uint64_t el_cap = 0;
  uint8_t* tflag = nullptr;        // [np]
  uint64_t* ddeath = nullptr;      // [np]
  uint32_t* erep = nullptr;        // [C + D]
  uint32_t* erun = nullptr;        // [etot]
  uint32_t* erend = nullptr;       // [etot]
  uint64_t* einit = nullptr;       // [etot]
  uint32_t* ecov = nullptr; uint32_t* egap = nullptr; uint32_t* etail = nullptr;   // [etot]
  uint64_t* sa = nullptr; uint64_t* sb = nullptr;   // [np + 1] segmented scans
  uint32_t* nq = nullptr;          // [np + 1]
  uint8_t* tnew = nullptr;         // [np + 1]
  uint64_t ex_cap = 0;
  uint32_t* tab = nullptr;         // block table + its segment sums
  uint32_t* occ = nullptr; uint32_t* freel = nullptr; uint32_t* ofl = nullptr; uint32_t* ofr = nullptr;
  uint64_t* hk = nullptr; uint64_t* hk2 = nullptr; uint32_t* hv = nullptr; uint32_t* hv2 = nullptr;
  uint64_t* bm_keys = nullptr; uint64_t* bm_vals = nullptr;
  uint8_t* staging = nullptr;
  void* tmp = nullptr;
  xcg::PairCnt* cnt = nullptr;
  uint32_t* h_small = nullptr;     // pinned: small readbacks
  xcg::PairCnt* h_cnt = nullptr;   // pinned
  // the last pass (kept for the commit)
  xcg::PairDev last{};
  uint32_t last_M = 0;
  bool last_ranked = false;
  uint64_t last_appends = 0;
  // sub-batch bookkeeping
  uint64_t appends = 0;            // disk blocks the last committed sub-batch wrote
  uint32_t last_base = 0;
  int prev_passes = 1;
  // chunks per sub-batch the last committed sub-batch's disk writes imply (90 %
  // of a lap at its rate; 0: none yet); the next call starts from it
  uint32_t fit_per = 0;
};

namespace {

using namespace xcg;

// The replay's sorts (a few hundred thousand rows of 20-bit entity keys, or
// 64-bit hashes) as rocPRIM's Onesweep radix sort: a histogram, a scan and one
// pass per 8 bits.  The default config takes merge sort up to 2^20 items, ~20
// launches of block merges for a C5 sub-batch (profiles/r06_s3_*).  Both are
// stable, which the entity runs need (positions stay in order).
using PairSortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                               rocprim::default_config, 0>;

bool pair_debug() {
  static const bool on = getenv("XCG_PAIR_DEBUG") != nullptr;
  return on;
}

unsigned grid_for(uint64_t threads) { return (unsigned)((threads + 255) / 256); }

// Guesses of a sub-batch's tiling seed replayed before its first parse
// (read per sub-batch).  Default 1: on C5-PAIR-LAPS three guesses save two of
// fifteen parse passes but each costs a replay with departures (~1.2 ms per
// 2000 chunks there), 49.7 -> 46.9 GiB/s.
int pair_seed_iters() {
  const char* e = getenv("XCG_PAIR_SEED_ITERS");
  const int k = e ? atoi(e) : 1;
  return k < 1 ? 1 : (k > 8 ? 8 : k);
}

template <class T>
bool grow(T** p, uint64_t* cap, uint64_t want) {
  if (*cap >= want) return true;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, want * sizeof(T)) != hipSuccess) return false;
  *cap = want;
  return true;
}

// Pass scratch for np positions, n chunks, etot entities.
int ensure_scratch(XcgPairState* P, uint64_t np, uint64_t n, uint64_t etot) {
  if (np + 1 > P->np_cap) {
    const uint64_t cap = std::max<uint64_t>(np + 1, P->np_cap + P->np_cap / 2);
    void** arrs[] = {(void**)&P->ent, (void**)&P->yent, (void**)&P->kind, (void**)&P->tim, (void**)&P->hsh,
                     (void**)&P->skey, (void**)&P->sval, (void**)&P->sk, (void**)&P->sv, (void**)&P->prv,
                     (void**)&P->nxt, (void**)&P->isr, (void**)&P->rc, (void**)&P->phit, (void**)&P->app,
                     (void**)&P->clk, (void**)&P->slow, (void**)&P->f1, (void**)&P->f2, (void**)&P->r1,
                     (void**)&P->r2, (void**)&P->missrow, (void**)&P->moves, (void**)&P->tflag,
                     (void**)&P->ddeath, (void**)&P->sa, (void**)&P->sb, (void**)&P->nq, (void**)&P->tnew};
    const size_t sz[] = {4, 4, 1, 8, 8, 4, 4, 4, 4, 4, 4, 4, 4, 1, 4, 4, 4, 4, 4, 4, 4, 4, 32, 1, 8, 8, 8, 4, 1};
    for (size_t k = 0; k < sizeof(sz) / sizeof(sz[0]); ++k) {
      (void)hipFree(*arrs[k]);
      *arrs[k] = nullptr;
    }
    P->np_cap = 0;
    for (size_t k = 0; k < sizeof(sz) / sizeof(sz[0]); ++k)
      if (hipMalloc(arrs[k], (cap + 1) * sz[k]) != hipSuccess) return -5;
    P->np_cap = cap;
  }
  if (n + 1 > P->n_cap) {
    (void)hipFree(P->pbase);
    (void)hipFree(P->pcnt);
    P->pbase = P->pcnt = nullptr;
    P->n_cap = 0;
    if (hipMalloc(&P->pbase, 4 * (n + 1)) != hipSuccess || hipMalloc(&P->pcnt, 4 * (n + 1)) != hipSuccess) return -5;
    P->n_cap = n + 1;
  }
  uint64_t ec = P->et_cap, lc = P->el_cap;
  if (!grow(&P->erun, &ec, etot) || !grow(&P->elast, &lc, etot)) return -5;
  P->et_cap = ec;
  P->el_cap = lc;
  if (etot > P->ex_cap) {
    void** arrs[] = {(void**)&P->erend, (void**)&P->einit, (void**)&P->ecov, (void**)&P->egap, (void**)&P->etail};
    const size_t sz[] = {4, 8, 4, 4, 4};
    P->ex_cap = 0;
    for (size_t k = 0; k < 5; ++k) {
      (void)hipFree(*arrs[k]);
      *arrs[k] = nullptr;
    }
    for (size_t k = 0; k < 5; ++k)
      if (hipMalloc(arrs[k], etot * sz[k] + 8) != hipSuccess) return -5;
    P->ex_cap = etot;
  }
  // rocprim temporary storage for the largest sort / scan of this size
  size_t a = 0, b = 0, c = 0;
  (void)rocprim::radix_sort_pairs<PairSortCfg>(nullptr, a, P->skey, P->sk, P->sval, P->sv, (uint32_t)np, 0, 32);
  // (the commit also scans the primary's C + 1 free-slot flags, pair_commit)
  (void)rocprim::exclusive_scan(nullptr, b, P->isr, P->rc, 0u,
                                (size_t)std::max<uint64_t>(std::max<uint64_t>(np, n), P->C) + 1,
                                rocprim::plus<uint32_t>());
  (void)rocprim::radix_sort_pairs<PairSortCfg>(nullptr, c, P->hk, P->hk2, P->hv, P->hv2, (uint32_t)np, 0, 64);
  size_t e1 = 0, e2 = 0, e3 = 0;
  (void)rocprim::exclusive_scan(nullptr, e1, P->sa, P->sb, (uint64_t)0, (size_t)np + 1, rocprim::maximum<uint64_t>());
  (void)rocprim::inclusive_scan(nullptr, e2, P->sa, P->sb, (size_t)np + 1, rocprim::maximum<uint64_t>());
  (void)rocprim::inclusive_scan(nullptr, e3, P->sa, P->sb, (size_t)np + 1, rocprim::minimum<uint64_t>());
  const uint64_t want = std::max(std::max(std::max(a, b), c), std::max(std::max(e1, e2), e3)) + 256;
  if (want > P->tmp_cap) {
    (void)hipFree(P->tmp);
    P->tmp = nullptr;
    P->tmp_cap = 0;
    if (hipMalloc(&P->tmp, want) != hipSuccess) return -5;
    P->tmp_cap = want;
  }
  return 0;
}

int scan_u32(XcgPairState* P, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t st) {
  size_t tb = P->tmp_cap;
  return rocprim::exclusive_scan(P->tmp, tb, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), st) == hipSuccess
             ? 0 : -5;
}

// Segmented max / min scans of the packed (run << 32 | v) values (sa -> sb).
int scan_max_excl(XcgPairState* P, uint64_t n, hipStream_t st) {
  size_t tb = P->tmp_cap;
  return rocprim::exclusive_scan(P->tmp, tb, P->sa, P->sb, (uint64_t)0, (size_t)n, rocprim::maximum<uint64_t>(),
                                 st) == hipSuccess ? 0 : -5;
}
int scan_max_incl(XcgPairState* P, uint64_t n, hipStream_t st) {
  size_t tb = P->tmp_cap;
  return rocprim::inclusive_scan(P->tmp, tb, P->sa, P->sb, (size_t)n, rocprim::maximum<uint64_t>(), st) == hipSuccess
             ? 0 : -5;
}
int scan_min_incl(XcgPairState* P, uint64_t n, hipStream_t st) {
  size_t tb = P->tmp_cap;
  return rocprim::inclusive_scan(P->tmp, tb, P->sa, P->sb, (size_t)n, rocprim::minimum<uint64_t>(), st) == hipSuccess
             ? 0 : -5;
}

int read_small(XcgPairState* P, const void* src, size_t bytes, hipStream_t st) {
  return hipMemcpyAsync(P->h_small, src, bytes, hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipStreamSynchronize(st) == hipSuccess
             ? 0 : -5;
}
int read_cnt(XcgPairState* P, hipStream_t st) {
  return hipMemcpyAsync(P->h_cnt, P->cnt, sizeof(PairCnt), hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipStreamSynchronize(st) == hipSuccess
             ? 0 : -5;
}

// Where the rows of a pass come from.
struct RowSrc {
  int dec;
  uint32_t n, maxd;
  const uint4* ev;
  const uint32_t* nev;             // encode
  uint32_t maxe;
  const uint64_t* base64;          // decode
  const uint64_t* cnt64;
  uint64_t rows;                   // decode: rows in all
  uint32_t* need;                  // encode: per chunk flags / contradicted times
  uint32_t* bad_t;
  uint32_t* bad_hi;
};

struct PassOut {
  uint32_t nbad = 0;
  bool split = false;
  bool changed = false;            // (want_leave) ptime moved
  uint64_t appends = 0;
};

// One replay pass (see the top of this file).  want_leave: compute ptime from
// the departures even if every lookup agrees (decode, seed guesses).
int replay(XcgPairState* P, const RowSrc& rs, const HashTab& g, bool want_leave, PassOut* out, hipStream_t st) {
  XcgDiskState* K = P->disk;
  const uint32_t n = rs.n;
  const uint32_t newb = P->C + P->D;
  const uint64_t etot64 = (uint64_t)newb + (uint64_t)n * rs.maxd;
  if (etot64 >= (1ull << 31)) return -95;
  const uint32_t etot = (uint32_t)etot64;
  if (!P->cnt) {
    if (hipMalloc(&P->cnt, sizeof(PairCnt)) != hipSuccess || hipHostMalloc(&P->h_cnt, sizeof(PairCnt)) != hipSuccess ||
        hipHostMalloc(&P->h_small, 256) != hipSuccess)
      return -5;
  }
  if (hipMemsetAsync(P->cnt, 0, sizeof(PairCnt), st) != hipSuccess) return -5;
  PairDev d{};
  d.C = P->C; d.xuid = P->xuid; d.P = P->pcount;
  d.pkey = P->pkey; d.pdisk = P->pdisk; d.lru = P->lru; d.ptime = P->ptime;
  d.D = P->D; d.nb = P->nb; d.dclock0 = K->dclock;
  d.dkey = K->dkey; d.dent = K->dent; d.dxuid = K->dxuid;
  d.dec = rs.dec; d.n = n; d.maxd = rs.maxd; d.maxe = rs.maxe; d.ev = rs.ev; d.nev = rs.nev;
  d.base64 = rs.base64; d.cnt64 = rs.cnt64;
  d.newb = newb; d.etot = etot;
  d.need = rs.need; d.bad_t = rs.bad_t; d.bad_hi = rs.bad_hi;
  d.g = g;
  // rows per chunk -> positions
  uint64_t R;
  if (ensure_scratch(P, (uint64_t)P->pcount + 1, n, etot)) return -5;
  if (!rs.dec) {
    d.pbase = P->pbase;
    d.pcnt = P->pcnt;
    d.cnt = P->cnt;
    hipLaunchKernelGGL(pr_count_kernel, dim3(grid_for(n + 1)), dim3(256), 0, st, d);
    if (scan_u32(P, P->pcnt, P->pbase, (uint64_t)n + 1, st) || read_small(P, P->pbase + n, 4, st)) return -5;
    R = P->h_small[0];
  } else {
    R = rs.rows;
  }
  const uint64_t np = (uint64_t)P->pcount + R;
  if (np >= (1ull << 31)) return -95;
  if (ensure_scratch(P, np, n, etot)) return -5;
  d.np = (uint32_t)np;
  d.ent = P->ent; d.yent = P->yent; d.kind = P->kind; d.tim = P->tim; d.hsh = P->hsh;
  d.skey = P->skey; d.sval = P->sval; d.sk = P->sk; d.sv = P->sv; d.prv = P->prv; d.nxt = P->nxt;
  d.isr = P->isr; d.rc = P->rc; d.phit = P->phit; d.app = P->app; d.clk = P->clk; d.slow = P->slow;
  d.f1 = P->f1; d.f2 = P->f2; d.r1 = P->r1; d.r2 = P->r2; d.missrow = P->missrow; d.moves = P->moves;
  d.pbase = P->pbase; d.pcnt = P->pcnt; d.cnt = P->cnt; d.elast = P->elast; d.tflag = P->tflag; d.ddeath = P->ddeath; d.erep = P->erep; d.erun = P->erun;
  d.lru2 = P->lru2; d.occ = P->occ; d.freel = P->freel;
  d.erend = P->erend; d.einit = P->einit; d.ecov = P->ecov; d.egap = P->egap; d.etail = P->etail;
  d.sa = P->sa; d.sb = P->sb; d.nq = P->nq; d.tnew = P->tnew;
  // encode: hash -> ENTER position
  if (!rs.dec) {
    const uint64_t want = std::max<uint64_t>(1024, 2ull << (64 - __builtin_clzll(R + 1)));
    uint64_t kc = P->bm_cap, vc = P->bm_cap;
    if (!grow(&P->bm_keys, &kc, want) || !grow(&P->bm_vals, &vc, want)) return -5;
    P->bm_cap = std::min(kc, vc);
    d.bm = HashTab{P->bm_keys, P->bm_vals, (uint32_t)(want - 1)};
    hipLaunchKernelGGL(pr_fill64_kernel, dim3(grid_for(want)), dim3(256), 0, st, P->bm_keys, want, EMPTY_KEY);
    hipLaunchKernelGGL(pr_fill64_kernel, dim3(grid_for(want)), dim3(256), 0, st, P->bm_vals, want, ~0ull);
  }
  if (hipMemsetAsync(P->tflag, 0, np + 1, st) != hipSuccess) return -5;
  if (rs.dec) hipLaunchKernelGGL(pr_fill32_kernel, dim3(grid_for(newb)), dim3(256), 0, st, P->erep, (uint64_t)newb, NIL);
  hipLaunchKernelGGL(pr_fill32_kernel, dim3(grid_for(etot)), dim3(256), 0, st, P->erun, (uint64_t)etot, NIL);
  if (P->pcount) hipLaunchKernelGGL(pr_pseudo_kernel, dim3(grid_for(P->pcount)), dim3(256), 0, st, d);
  if (n) hipLaunchKernelGGL(pr_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, st, d);
  if (rs.dec && R) {                               // decode HITs: latest definer of the hash
    uint64_t c1 = P->hk_cap, c2 = P->hk_cap, c3 = P->hk_cap, c4 = P->hk_cap;
    if (!grow(&P->hk, &c1, R) || !grow(&P->hk2, &c2, R) || !grow(&P->hv, &c3, R) || !grow(&P->hv2, &c4, R))
      return -5;
    P->hk_cap = std::min(std::min(c1, c2), std::min(c3, c4));
    if (hipMemcpyAsync(P->hk, P->hsh + P->pcount, 8 * R, hipMemcpyDeviceToDevice, st) != hipSuccess) return -5;
    // values: positions P .. np-1
    hipLaunchKernelGGL(pr_iota_kernel, dim3(grid_for(R)), dim3(256), 0, st, P->hv, (uint32_t)R, P->pcount);
    size_t tb = P->tmp_cap;
    if (rocprim::radix_sort_pairs<PairSortCfg>(P->tmp, tb, P->hk, P->hk2, P->hv, P->hv2, (uint32_t)R, 0, 64, st) != hipSuccess)
      return -5;
    // latest definer / first GHIT per hash run by scans (f1: run heads, f2: their prefix, r1: first GHIT)
    hipLaunchKernelGGL(pr_dh_heads_kernel, dim3(grid_for(R + 1)), dim3(256), 0, st, (const uint64_t*)P->hk2,
                       (uint32_t)R, P->f1);
    if (scan_u32(P, P->f1, P->f2, R + 1, st)) return -5;
    hipLaunchKernelGGL(pr_fill32_kernel, dim3(grid_for(R)), dim3(256), 0, st, P->r1, R, NIL);
    hipLaunchKernelGGL(pr_dh_vals_kernel, dim3(grid_for(R)), dim3(256), 0, st, d, (const uint32_t*)P->hv2,
                       (uint32_t)R, (const uint32_t*)P->f1, (const uint32_t*)P->f2, P->r1);
    if (scan_max_incl(P, R, st)) return -5;
    hipLaunchKernelGGL(pr_dec_hits_kernel, dim3(grid_for(R)), dim3(256), 0, st, d, (const uint32_t*)P->hv2,
                       (uint32_t)R, (const uint32_t*)P->f1, (const uint32_t*)P->f2, (const uint32_t*)P->r1);
  }
  hipLaunchKernelGGL(pr_resolve_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  // entity runs: sort positions by entity (stable: positions stay in order)
  {
    const uint32_t bits = 32 - __builtin_clz(etot | 1u);
    size_t tb = P->tmp_cap;
    if (rocprim::radix_sort_pairs<PairSortCfg>(P->tmp, tb, P->skey, P->sk, P->sval, P->sv, (uint32_t)np, 0, bits, st) !=
        hipSuccess)
      return -5;
  }
  hipLaunchKernelGGL(pr_fill32_kernel, dim3(grid_for(np)), dim3(256), 0, st, (uint32_t*)P->nxt, np, NIL);
  hipLaunchKernelGGL(pr_link_vals_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (scan_max_excl(P, np, st)) return -5;
  hipLaunchKernelGGL(pr_links_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (rs.dec) hipLaunchKernelGGL(pr_repl_links_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (scan_u32(P, P->isr, P->rc, np + 1, st)) return -5;
  hipLaunchKernelGGL(pr_hits_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (read_cnt(P, st)) return -5;
  const uint32_t nslow = P->h_cnt->nslow;
  if (P->h_cnt->nohit) return -95;
  if (nslow) {                                     // the block table for long gaps
    uint32_t bsh = 8;
    while ((np >> bsh) > 1024) ++bsh;
    const uint32_t nbk = (uint32_t)((np + (1ull << bsh) - 1) >> bsh);
    const uint64_t w = (uint64_t)nbk + 1;
    const uint64_t cells = (uint64_t)nbk * w + TSEG * w;
    uint64_t tc = P->tab_cap;
    if (!grow(&P->tab, &tc, cells)) return -5;
    P->tab_cap = tc;
    d.tab = P->tab;
    d.bsh = bsh;
    d.nbk = nbk;
    if (hipMemsetAsync(P->tab, 0, 4 * (uint64_t)nbk * w, st) != hipSuccess) return -5;
    hipLaunchKernelGGL(pr_tab_hist_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
    hipLaunchKernelGGL(pr_tab_rows_kernel, dim3((nbk + 3) / 4), dim3(256), 0, st, d);
    uint32_t* segsum = P->tab + (uint64_t)nbk * w;
    hipLaunchKernelGGL(pr_tab_cols_kernel, dim3(grid_for(w * TSEG)), dim3(256), 0, st, d, segsum, 0);
    hipLaunchKernelGGL(pr_tab_cols_kernel, dim3(grid_for(w)), dim3(256), 0, st, d, segsum, 1);
    hipLaunchKernelGGL(pr_tab_cols_kernel, dim3(grid_for(w * TSEG)), dim3(256), 0, st, d, segsum, 2);
    hipLaunchKernelGGL(pr_tab_query_kernel, dim3((nslow + 3) / 4), dim3(256), 0, st, d);
  }
  // the disk clock: monotone rounds to the least fixed point
  hipLaunchKernelGGL(pr_nq_vals_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (scan_min_incl(P, np, st)) return -5;
  hipLaunchKernelGGL(pr_nq_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (hipMemsetAsync(P->tnew, 0, np + 1, st) != hipSuccess) return -5;
  int rounds = 0;
  for (;; ++rounds) {
    if (scan_u32(P, P->app, P->clk, np + 1, st)) return -5;
    if (rounds >= 64) return -75;
    if (hipMemsetAsync(&P->cnt->changed, 0, 4, st) != hipSuccess) return -5;
    hipLaunchKernelGGL(pr_touch_chain_kernel, dim3(grid_for(etot)), dim3(256), 0, st, d);
    hipLaunchKernelGGL(pr_setter_vals_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
    if (scan_max_excl(P, np, st)) return -5;
    hipLaunchKernelGGL(pr_touch_rows_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
    if (read_cnt(P, st)) return -5;
    if (P->h_cnt->changed == 0) break;
  }
  hipLaunchKernelGGL(pr_check_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
  if (hipMemcpyAsync(P->h_small, P->clk + np, 4, hipMemcpyDeviceToHost, st) != hipSuccess || read_cnt(P, st))
    return -5;
  out->appends = P->h_small[0];
  out->nbad = P->h_cnt->nbad;
  out->split = P->h_cnt->split != 0 || P->h_cnt->unsorted != 0;
  P->last = d;
  P->last_ranked = false;
  P->last_appends = out->appends;
  if (pair_debug())
    fprintf(stderr, "pair-replay: dec %d n %u rows %llu P %u slow %u touch-rounds %d appends %llu bad %u split %u "
                    "unsorted %u\n", rs.dec, n, (unsigned long long)R, P->pcount, nslow, rounds,
            (unsigned long long)out->appends, out->nbad, P->h_cnt->split, P->h_cnt->unsorted);
  if (out->split) return 0;
  if (want_leave || out->nbad) {
    hipLaunchKernelGGL(pr_missterm_kernel, dim3(grid_for(np + 1)), dim3(256), 0, st, d);
    if (scan_u32(P, P->f1, P->r1, np + 1, st) || scan_u32(P, P->f2, P->r2, np + 1, st)) return -5;
    hipLaunchKernelGGL(pr_missrow_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
    if (read_small(P, P->r1 + np, 4, st)) return -5;
    P->last_M = P->h_small[0];
    P->last_ranked = true;
    if (hipMemsetAsync(&P->cnt->changed, 0, 4, st) != hipSuccess) return -5;
    hipLaunchKernelGGL(pr_cover_kernel, dim3(grid_for(newb)), dim3(256), 0, st, d);
    hipLaunchKernelGGL(pr_span_vals_kernel, dim3(grid_for(np)), dim3(256), 0, st, d, P->last_M);
    if (scan_max_excl(P, np, st)) return -5;
    hipLaunchKernelGGL(pr_gaps_kernel, dim3(grid_for(np)), dim3(256), 0, st, d, P->last_M);
    hipLaunchKernelGGL(pr_leave_kernel, dim3(grid_for(newb)), dim3(256), 0, st, d);
    if (read_cnt(P, st)) return -5;
    out->changed = P->h_cnt->changed != 0;
  }
  return 0;
}

// The primary's arrays must outlive one replay; the commit's slot arrays too.
int ensure_front_arrays(XcgPairState* P) {
  if (P->occ) return 0;
  if (hipMalloc(&P->occ, 4ull * P->C) != hipSuccess || hipMalloc(&P->freel, 4ull * P->C) != hipSuccess ||
      hipMalloc(&P->ofl, 4ull * (P->C + 1)) != hipSuccess || hipMalloc(&P->ofr, 4ull * (P->C + 1)) != hipSuccess)
    return -5;
  return 0;
}

// G from the state: wipe, then every primary slot and live own disk block.
void pair_rebuild(XcgPairState* P, const PairGpu& G, hipStream_t st) {
  const HashTab g{G.g_keys, G.g_vals, G.g_mask};
  const FiltSet fs{G.g_filt, G.g_ftab, G.fmask, G.g_gfilt, G.gmask};
  PairWipe wp{g, G.g_filt, (u32x4*)G.g_ftab, G.fmask + 1, G.g_gfilt, G.gmask + 1, G.nseg};
  hipLaunchKernelGGL(pair_wipe_kernel, dim3(1024), dim3(256), 0, st, wp);
  XcgDiskState* K = P->disk;
  hipLaunchKernelGGL(pair_rebuild_kernel, dim3(grid_for((uint64_t)P->C + P->D)), dim3(256), 0, st,
                     (const uint64_t*)P->pkey, P->C, (const uint64_t*)K->dkey, (const uint64_t*)K->dent,
                     (const uint32_t*)K->dxuid, P->D, P->nb, (uint32_t)P->xuid, K->dclock, g, fs, G.nseg, G.status);
  P->gclock = K->dclock;
  P->gstale = false;
}

__global__ __launch_bounds__(256) void pr_notocc_kernel(const uint32_t* occ, uint32_t C, uint32_t* fl) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s <= C) fl[s] = s < C && !occ[s] ? 1u : 0u;
}

// Commit the last (consistent) pass: final primary, disk appends, bytes, G.
int pair_commit(XcgPairState* P, const PairGpu& G, hipStream_t st) {
  XcgDiskState* K = P->disk;
  PairDev d = P->last;
  const uint64_t np = d.np;
  if (ensure_front_arrays(P)) return -5;
  d.occ = P->occ; d.freel = P->freel; d.lru2 = P->lru2;
  if (!P->last_ranked) {
    hipLaunchKernelGGL(pr_missterm_kernel, dim3(grid_for(np + 1)), dim3(256), 0, st, d);
    if (scan_u32(P, P->f1, P->r1, np + 1, st) || scan_u32(P, P->f2, P->r2, np + 1, st)) return -5;
    hipLaunchKernelGGL(pr_missrow_kernel, dim3(grid_for(np)), dim3(256), 0, st, d);
    if (P->unbounded) {                            // (only this check needs M on the host)
      if (read_small(P, P->r1 + np, 4, st)) return -5;
      P->last_M = P->h_small[0];
    }
  }
  // the primary never evicts: its capacity is exceeded
  if (P->unbounded && (int64_t)d.P + (int64_t)P->last_M - (int64_t)P->C > 0) return -75;
  const uint64_t dend = K->dclock + P->last_appends;
  if (hipMemsetAsync(P->occ, 0, 4ull * P->C, st) != hipSuccess ||
      hipMemsetAsync(&P->cnt->nmove, 0, 8, st) != hipSuccess)
    return -5;
  // (terminal ranks r2 are consumed by pr_final before f1 / f2 / r1 / r2 are reused)
  hipLaunchKernelGGL(pr_final_kernel, dim3(grid_for(np + 1)), dim3(256), 0, st, d, (const uint32_t*)P->r1 + np);
  if (scan_u32(P, P->f1, P->r1, np + 1, st) || scan_u32(P, P->f2, P->r2, np + 1, st)) return -5;
  hipLaunchKernelGGL(pr_notocc_kernel, dim3(grid_for(P->C + 1)), dim3(256), 0, st, (const uint32_t*)P->occ, P->C,
                     P->ofl);
  if (scan_u32(P, P->ofl, P->ofr, (uint64_t)P->C + 1, st)) return -5;
  hipLaunchKernelGGL(pr_free_kernel, dim3(grid_for(P->C)), dim3(256), 0, st, d, (const uint32_t*)P->ofr);
  hipLaunchKernelGGL(pr_place_kernel, dim3(grid_for(np)), dim3(256), 0, st, d, dend);
  if (d.dec) hipLaunchKernelGGL(pr_remove_kernel, dim3(grid_for(np)), dim3(256), 0, st, d, dend);
  hipLaunchKernelGGL(pr_append_kernel, dim3(grid_for(np)), dim3(256), 0, st, d, dend);
  if (hipMemcpyAsync(P->h_small, P->r1 + np, 4, hipMemcpyDeviceToHost, st) != hipSuccess || read_cnt(P, st))
    return -5;
  const uint32_t pc = P->h_small[0], nmove = P->h_cnt->nmove, nstage = P->h_cnt->nstage;
  if (pc > P->C) return -5;
  uint64_t sc = P->stg_cap;
  if (!grow(&P->staging, &sc, (uint64_t)std::max<uint32_t>(nstage, 1) * SEG)) return -5;
  P->stg_cap = sc;
  if (nmove) {
    hipLaunchKernelGGL(pair_stage_kernel, dim3((nmove + 3) / 4), dim3(256), 0, st, (const uint4*)P->moves,
                       (const PairCnt*)P->cnt, (const uint8_t*)G.pool, P->staging);
    hipLaunchKernelGGL(pair_move_kernel, dim3((nmove + 4 * MOVES_PER_WAVE - 1) / (4 * MOVES_PER_WAVE)), dim3(256), 0, st,
                       (const uint4*)P->moves,
                       (const PairCnt*)P->cnt, G.in, G.chunk_off, (const uint4*)G.decl, G.maxd,
                       (const uint8_t*)P->staging, G.pool);
  }
  std::swap(P->lru, P->lru2);
  P->pcount = pc;
  // index blocks filled by this commit are written with the running counter
  // (XCodecDisk::enter, xcodec_cache_disk.cc:708-738; 0 means unused)
  for (uint64_t m = K->dclock / DISK_ENTRIES + 1; m <= dend / DISK_ENTRIES; ++m) {
    K->ctr[(m - 1) % K->nb] = K->ibc;
    if (++K->ibc == 0) K->ibc = 1;
  }
  K->dclock = dend;
  P->appends = P->last_appends;
  pair_rebuild(P, G, st);
  return hipStreamSynchronize(st) == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -5;
}

int fill_ptime(XcgPairState* P, hipStream_t st) {
  hipLaunchKernelGGL(pr_fill64_kernel, dim3(1024), dim3(256), 0, st, P->ptime, (uint64_t)P->C + P->D, NEVERT);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Entries another front's writes retired (the clock crossed an index block
// since G was built): rebuild G before this front looks anything up.
int pair_sync_front(XcgPairState* P, const PairGpu& G, hipStream_t st) {
  XcgDiskState* K = P->disk;
  if (!P->gstale && K->dclock / DISK_ENTRIES == P->gclock / DISK_ENTRIES) return 0;
  pair_rebuild(P, G, st);
  return hipStreamSynchronize(st) == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -5;
}

PairGpu gpu_of(const XcgStreamArgs& a) {
  return PairGpu{a.in, a.chunk_off, a.decl, a.maxd, a.pool, a.g_keys, a.g_vals, a.g_mask,
                 a.g_filt, a.g_ftab, a.fmask, a.g_gfilt, a.gmask, a.nseg, a.status};
}

// The disk's device arrays, on the first front's device.
int disk_bind(XcgDiskState* K, int device) {
  if (K->device >= 0) return K->device == device ? 0 : -22;
  const uint64_t D = K->D;
  if (hipMalloc(&K->dkey, 8 * D) != hipSuccess || hipMalloc(&K->dent, 8 * D) != hipSuccess ||
      hipMalloc(&K->dxuid, 4 * D) != hipSuccess || hipMemset(K->dkey, 0xFF, 8 * D) != hipSuccess ||
      hipMemset(K->dent, 0xFF, 8 * D) != hipSuccess || hipMemset(K->dxuid, 0xFF, 4 * D) != hipSuccess) {
    (void)hipFree(K->dkey); (void)hipFree(K->dent); (void)hipFree(K->dxuid);
    K->dkey = K->dent = nullptr;
    K->dxuid = nullptr;
    return -12;
  }
  K->device = device;
  return 0;
}

size_t round_up(size_t v, size_t g) { return (v + g - 1) / g * g; }

// The front's pool: C primary segments followed by the disk's D blocks at
// pool + (C + i) * 2048.  HIP virtual memory maps the disk's one physical
// allocation behind every front; without it each front allocates its own copy
// (a front reads only the blocks it wrote itself, so that is correct too).
int map_pool(XcgPairState* P, int device) {
  XcgDiskState* K = P->disk;
  if (!getenv("XCG_NO_VMM")) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    bool ok = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) == hipSuccess &&
              gran > 0;
    if (ok && !K->vmm && K->pool_bytes == 0) {
      // The disk's blocks: HBM, unless the volume does not fit beside what the
      // device already holds (keep 4 GiB free) or the caller asks for the host
      // tier -- then pinned host memory behind the same addresses, which the
      // kernels read and write over PCIe (a spill level below HBM).
      const size_t sd = round_up((size_t)K->D * SEG + 256, gran);
      size_t fr = 0, tot = 0;
      const bool fits = hipMemGetInfo(&fr, &tot) == hipSuccess && fr > sd + (4ull << 30);
      const bool want_host = (K->flags & 1u) != 0 || (!(K->flags & 2u) && !fits);
      if (!want_host && hipMemCreate(&K->pool_h, sd, &prop, 0) == hipSuccess) {
        K->pool_bytes = sd;
        K->vmm = true;
        K->tier = 0;
      } else if (!(K->flags & 2u)) {
        (void)hipGetLastError();
        hipMemAllocationProp hp{};
        hp.type = hipMemAllocationTypePinned;
        hp.location.type = hipMemLocationTypeHost;
        hp.location.id = 0;
        size_t hg = 0;
        const hipError_t e1 = hipMemGetAllocationGranularity(&hg, &hp, hipMemAllocationGranularityMinimum);
        const hipError_t e2 = e1 == hipSuccess && hg && gran % hg == 0 ? hipMemCreate(&K->pool_h, sd, &hp, 0)
                                                                        : hipErrorInvalidValue;
        if (e2 == hipSuccess) {
          K->pool_bytes = sd;
          K->vmm = true;
          K->tier = 1;
        } else {
          // (host-located VMM needs a runtime that has it: ROCm 7.2's does, the
          // 7.0 runtime PyTorch bundles refuses it) -- stay on the device
          if (pair_debug())
            fprintf(stderr, "pair: host tier not available (granularity %s %zu, create %s)\n", hipGetErrorString(e1),
                    hg, hipGetErrorString(e2));
          (void)hipGetLastError();
          if (hipMemCreate(&K->pool_h, sd, &prop, 0) == hipSuccess) {
            K->pool_bytes = sd;
            K->vmm = true;
            K->tier = 0;
          }
        }
      }
    }
    ok = ok && K->vmm;
    if (ok && !K->dva) {
      // The disk's own mapping of its blocks, held until the disk goes: the
      // volume can be saved after every front is gone, and the allocation
      // always has a mapping until it is released (fronts come and go).
      void* va = nullptr;
      hipMemAccessDesc acc{};
      acc.location = prop.location;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      bool m = false;
      bool dok = hipMemAddressReserve(&va, K->pool_bytes, 0, nullptr, 0) == hipSuccess;
      dok = dok && (m = hipMemMap(va, K->pool_bytes, 0, K->pool_h, 0) == hipSuccess);
      dok = dok && hipMemSetAccess(va, K->pool_bytes, &acc, 1) == hipSuccess;
      if (dok) {
        K->dva = va;
      } else {
        if (m) (void)hipMemUnmap(va, K->pool_bytes);
        if (va) (void)hipMemAddressFree(va, K->pool_bytes);
        (void)hipGetLastError();
      }
    }
    const size_t sp = round_up((size_t)P->C * SEG, gran ? gran : 1);
    bool prim = false, reserved = false, m1 = false, m2 = false;
    if (ok) prim = ok = hipMemCreate(&P->prim_h, sp, &prop, 0) == hipSuccess;
    if (ok) reserved = ok = hipMemAddressReserve(&P->va, sp + K->pool_bytes, 0, nullptr, 0) == hipSuccess;
    if (ok) m1 = ok = hipMemMap(P->va, sp, 0, P->prim_h, 0) == hipSuccess;
    if (ok) m2 = ok = hipMemMap((char*)P->va + sp, K->pool_bytes, 0, K->pool_h, 0) == hipSuccess;
    if (ok) {
      hipMemAccessDesc acc{};
      acc.location = prop.location;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      ok = hipMemSetAccess(P->va, sp + K->pool_bytes, &acc, 1) == hipSuccess;
    }
    if (!ok && pair_debug())
      fprintf(stderr, "pair: pool mapping failed (prim %d reserved %d map %d/%d tier %d): %s\n", (int)prim, (int)reserved,
              (int)m1, (int)m2, K->tier, hipGetErrorString(hipGetLastError()));
    if (ok) {
      P->pool_vmm = true;
      P->prim_bytes = sp;
      P->va_bytes = sp + K->pool_bytes;
      P->pool = (uint8_t*)P->va + sp - (size_t)P->C * SEG;
      return 0;
    }
    if (m2) (void)hipMemUnmap((char*)P->va + sp, K->pool_bytes);
    if (m1) (void)hipMemUnmap(P->va, sp);
    if (reserved) (void)hipMemAddressFree(P->va, sp + K->pool_bytes);
    if (prim) (void)hipMemRelease(P->prim_h);
    P->va = nullptr;
    (void)hipGetLastError();
  }
  if (hipMalloc(&P->pool, ((uint64_t)P->C + P->D) * SEG + 256) != hipSuccess) return -12;
  P->pool_vmm = false;
  return 0;
}

void unmap_pool(XcgPairState* P) {
  if (P->pool_vmm) {
    (void)hipDeviceSynchronize();
    (void)hipMemUnmap((char*)P->va + P->prim_bytes, P->va_bytes - P->prim_bytes);
    (void)hipMemUnmap(P->va, P->prim_bytes);
    (void)hipMemAddressFree(P->va, P->va_bytes);
    (void)hipMemRelease(P->prim_h);
  } else {
    (void)hipFree(P->pool);
  }
  P->pool = nullptr;
}

void free_scratch(XcgPairState* P) {
  void* arrs[] = {P->ent, P->yent, P->kind, P->tim, P->hsh, P->skey, P->sval, P->sk, P->sv, P->prv, P->nxt,
                  P->isr, P->rc, P->phit, P->app, P->clk, P->slow, P->f1, P->f2, P->r1, P->r2, P->missrow,
                  P->moves, P->pbase, P->pcnt, P->elast, P->tflag, P->ddeath, P->erep, P->erun, P->erend, P->einit, P->ecov, P->egap, P->etail, P->sa, P->sb, P->nq, P->tnew, P->tab, P->occ, P->freel, P->ofl, P->ofr, P->hk, P->hk2,
                  P->hv, P->hv2, P->bm_keys, P->bm_vals, P->staging, P->tmp, P->cnt};
  for (void* p : arrs) (void)hipFree(p);
  if (P->h_small) (void)hipHostFree(P->h_small);
  if (P->h_cnt) (void)hipHostFree(P->h_cnt);
}

// XCodecHash::hash of one segment (xcodec/xcodec_hash.h:166-174), host side:
// the reload's check of an index entry against its data block.
uint64_t host_hash(const uint8_t* w) {
  uint32_t s1 = 0, s2 = 0, b1 = 0, b2 = 0;
  for (int k = 0; k < SEG; ++k) {
    s1 += (uint32_t)w[k] + 1u;
    s2 += s1;
    b1 += w[k] ? (uint32_t)__builtin_ctz(w[k]) + 1u : 0u;
    b2 += b1;
  }
  const uint32_t bits = (b1 << 16) + b2, bytes = (s1 << 20) + s2;
  return ((uint64_t)bits << 36) + (uint64_t)bytes;
}

constexpr uint32_t REG_BLOCKS = 18, REG_ENTRIES = 2048 / 36, CHECK_BOUNDARY = 80, XUIDS = 1024;

// XCodecDisk::registry_write (xcodec_cache_disk.cc:603-627): the xuid's
// registry block with the UUID patched in, written back to block 0 (as the
// reference does).
void registry_write(XcgDiskState* K, uint32_t xuid, const char* u36) {
  uint8_t blk[2048];
  memcpy(blk, &K->reg[(xuid / REG_ENTRIES) * 2048], 2048);
  memcpy(&blk[(xuid % REG_ENTRIES) * 36], u36, 36);
  memcpy(&K->reg[0], blk, 2048);
}

// uuid_parse's format (common/uuid/uuid_libuuid.cc UUID::decode): 8-4-4-4-12 hex.
bool uuid_ok(const uint8_t* u) {
  for (int i = 0; i < 36; ++i) {
    if (i == 8 || i == 13 || i == 18 || i == 23) {
      if (u[i] != '-') return false;
    } else if (!isxdigit(u[i])) {
      return false;
    }
  }
  return true;
}

// A reopened volume (XCodecDisk::XCodecDisk, xcodec_cache_disk.cc:107-237):
// the registry gives the fronts; index blocks are scanned in block order up
// to the first free one (counter 0); the lowest counter is the write head and
// is not loaded; the rest load in counter order, a later entry of a hash
// replacing an earlier one, the first and last 80 checked against their data
// blocks (index_load_entries :408-478); fronts left without entries leave the
// registry (registry_collect :496-528).  In the engine's clock model the write
// head's entry 0 is clock 204 * (nb + head), and a block b loaded from the last
// lap holds entries numbered from 204 * (nb + head - ((head - b) mod nb)): each
// dies when the head reaches b again, as the reference invalidates it.
//
// Whole-range file I/O: one read()/write() moves at most 0x7ffff000 bytes on
// Linux, so a volume past 2 GiB takes several.  A read that meets the end of
// the file leaves the rest zero (the reference's ftruncate'd volume reads as
// zeros there, xcodec_cache_disk.cc:853-860).
bool pread_all(int fd, uint8_t* p, size_t n, off_t off) {
  while (n > 0) {
    const ssize_t r = pread(fd, p, n, off);
    if (r < 0 && errno == EINTR) continue;
    if (r < 0) return false;
    if (r == 0) {
      memset(p, 0, n);
      return true;
    }
    p += r;
    n -= (size_t)r;
    off += r;
  }
  return true;
}

bool pwrite_all(int fd, const uint8_t* p, size_t n, off_t off) {
  while (n > 0) {
    const ssize_t r = pwrite(fd, p, n, off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
    off += r;
  }
  return true;
}

// UUID::generate (common/uuid/uuid_libuuid.cc: uuid_generate + uuid_unparse):
// a random (version 4) UUID in its 36-character lower-case form.
bool gen_uuid(char out[37]) {
  uint8_t b[16];
  const int fd = ::open("/dev/urandom", O_RDONLY);
  const bool ok = fd != -1 && pread_all(fd, b, 16, 0);
  if (fd != -1) close(fd);
  if (!ok) return false;
  b[6] = (uint8_t)((b[6] & 0x0F) | 0x40);
  b[8] = (uint8_t)((b[8] & 0x3F) | 0x80);
  snprintf(out, 37, "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[0], b[1], b[2], b[3],
           b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
  return true;
}

int load_volume(XcgDiskState* K, int fd) {
  const uint64_t nb = K->nb, D = K->D;
  // the registry and index blocks; the data blocks go straight to h_data
  std::vector<uint8_t> vol((REG_BLOCKS + nb) * 2048);
  K->h_data.assign((size_t)D * SEG, 0);
  if (!pread_all(fd, vol.data(), vol.size(), 0) ||
      !pread_all(fd, K->h_data.data(), K->h_data.size(), (off_t)vol.size())) {
    std::vector<uint8_t>().swap(K->h_data);
    return -2;
  }
  memcpy(&K->reg[0], &vol[0], K->reg.size());
  std::unordered_map<std::string, uint32_t> seen;
  for (uint32_t x = 0; x < REG_BLOCKS * REG_ENTRIES && x < XUIDS; ++x) {
    const uint8_t* u = &K->reg[(x / REG_ENTRIES) * 2048 + (x % REG_ENTRIES) * 36];
    bool zero = true;
    for (int i = 0; i < 36; ++i) zero &= u[i] == 0;
    if (zero || !uuid_ok(u)) continue;
    const std::string us((const char*)u, 36);
    if (seen.count(us)) continue;
    seen[us] = x;
    K->uuid[x] = us;
  }
  if (seen.empty()) {                                       // registry_load: a local UUID (:575-596)
    char u[37];
    if (!gen_uuid(u)) return -2;
    K->uuid[0] = std::string(u, 36);
    registry_write(K, 0, u);
  }
  std::map<uint64_t, uint64_t> cmap;
  uint64_t ibc = 0;
  for (uint64_t o = 0; o < nb; ++o) {
    uint64_t counter;
    memcpy(&counter, &vol[(REG_BLOCKS + o) * 2048], 8);
    if (counter == 0) {
      cmap[0] = o;
      break;
    }
    if (counter > ibc) ibc = counter + 1;
    cmap[counter] = o;
  }
  uint64_t cib = 0;
  if (!cmap.empty()) {
    cib = cmap.begin()->second;
    cmap.erase(cmap.begin());
  }
  K->h_key.assign(D, NOKEY);
  K->h_ent.assign(D, NOENT);
  K->h_xuid.assign(D, 0xFFFFFFFFu);
  for (uint64_t o = 0; o < nb; ++o) {
    memcpy(&K->ctr[o], &vol[(REG_BLOCKS + o) * 2048], 8);
    const uint8_t* q = &vol[(REG_BLOCKS + o) * 2048 + 8];
    for (uint64_t j = 0; j < DISK_ENTRIES; ++j, q += 10) {
      uint16_t xu;
      uint64_t h;
      memcpy(&xu, q, 2);
      memcpy(&h, q + 2, 8);
      if (h == 0) continue;
      K->h_key[o * DISK_ENTRIES + j] = h;
      K->h_xuid[o * DISK_ENTRIES + j] = xu;
    }
  }
  std::vector<std::unordered_map<uint64_t, uint64_t>> index(XUIDS);   // per xuid: hash -> slot
  auto invalidate = [&](uint64_t b) {
    if (K->ctr[b] == 0) return;
    for (uint64_t i = b * DISK_ENTRIES; i < (b + 1) * DISK_ENTRIES; ++i) {
      const uint32_t xu = K->h_xuid[i];
      if (K->h_key[i] == NOKEY || xu >= XUIDS || K->uuid[xu].empty()) continue;
      auto it = index[xu].find(K->h_key[i]);
      if (it != index[xu].end() && it->second == i) index[xu].erase(it);
    }
  };
  unsigned leading = CHECK_BOUNDARY;
  while (!cmap.empty()) {
    bool check;
    if (leading != 0) {
      check = true;
      --leading;
    } else {
      check = cmap.size() <= CHECK_BOUNDARY;
    }
    const uint64_t b = cmap.begin()->second;
    cmap.erase(cmap.begin());
    for (uint64_t j = 0; j < DISK_ENTRIES; ++j) {
      const uint64_t slot = b * DISK_ENTRIES + j;
      const uint64_t h = K->h_key[slot];
      const uint32_t xu = K->h_xuid[slot];
      if (h == NOKEY || xu >= XUIDS || K->uuid[xu].empty()) continue;
      index[xu].erase(h);                                   // ("Replacing previous cache entry.")
      if (check && host_hash(&K->h_data[slot * SEG]) != h) {
        if (cib > b) {                                      // rewrite the block with errors
          invalidate(b);
          cib = b;
          break;
        }
        continue;
      }
      index[xu][h] = slot;
    }
  }
  for (uint32_t x = 1; x < XUIDS; ++x) {                    // registry_collect
    if (K->uuid[x].empty() || !index[x].empty()) continue;
    static const char zero36[36] = {0};
    registry_write(K, x, zero36);
    K->uuid[x].clear();
  }
  for (uint32_t x = 0; x < XUIDS; ++x)
    for (const auto& kv : index[x]) {
      const uint64_t slot = kv.second, b = slot / DISK_ENTRIES;
      const uint64_t bn = nb + cib - ((cib + nb - b) % nb);
      K->h_ent[slot] = DISK_ENTRIES * bn + slot % DISK_ENTRIES;
    }
  K->ibc = ibc == 0 ? 1 : ibc;
  K->dclock = DISK_ENTRIES * (nb + cib);
  K->pending = true;
  return 0;
}

}  // namespace

extern "C" {

int xcg_disk_state_create(uint64_t disk_bytes, uint32_t flags, XcgDiskState** out) {
  const uint64_t blocks = disk_bytes / SEG;
  if (blocks <= 18) return -22;
  const uint64_t nb = (blocks - 18) / (1 + DISK_ENTRIES);   // xcodec_cache_disk.cc:110-111
  if (nb == 0 || nb * DISK_ENTRIES >= (1ull << 29)) return -22;
  XcgDiskState* K = new XcgDiskState;
  K->nb = nb;
  K->D = (uint32_t)(nb * DISK_ENTRIES);
  K->flags = flags;
  K->bytes = disk_bytes;
  K->ctr.assign(nb, 0);
  K->reg.assign(18 * 2048, 0);
  K->uuid.assign(1024, std::string());
  *out = K;
  return 0;
}

void xcg_disk_state_release(XcgDiskState* K) {
  if (!K || --K->refs > 0) return;
  (void)hipFree(K->dkey); (void)hipFree(K->dent); (void)hipFree(K->dxuid);
  if (K->dva) {
    (void)hipDeviceSynchronize();
    (void)hipMemUnmap(K->dva, K->pool_bytes);
    (void)hipMemAddressFree(K->dva, K->pool_bytes);
  }
  if (K->vmm) (void)hipMemRelease(K->pool_h);
  delete K;
}

void xcg_disk_state_stats(const XcgDiskState* K, uint64_t* st) {
  uint64_t live = 0, fronts = 0;
  for (const XcgPairState* f : K->fronts) fronts += f != nullptr;
  if (K->device >= 0) {
    uint32_t* d = nullptr;
    uint32_t h = 0;
    if (hipMalloc(&d, 4) == hipSuccess && hipMemset(d, 0, 4) == hipSuccess) {
      hipLaunchKernelGGL(pair_count_live_kernel, dim3(grid_for(K->D)), dim3(256), 0, nullptr,
                         (const uint64_t*)K->dent, (const uint32_t*)K->dxuid, K->D, (uint32_t)K->nb, K->dclock, NIL, d);
      if (hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost) == hipSuccess) live = h;
    }
    (void)hipFree(d);
  }
  st[0] = live;
  st[1] = K->dclock;
  st[2] = K->nb;
  st[3] = fronts;
}

// A pair front on disk K, on the current device.  Which front (xuid):
//  * want_xuid >= 0: that one -- a host XCodecDiskCache's own xuid_, so the
//    engine's fronts are the host disk's whatever order they bind in; uuid36,
//    when given, must be registered there or nowhere;
//  * uuid36: XCodecDisk::connect (xcodec_cache_disk.cc:640-690), the uuid's
//    registered xuid, else the lowest xuid nothing holds (no registry entry, no
//    front);
//  * neither: XCodecDisk::local (:635-641), xuid 0 when it is registered and
//    free (a reopened volume's local front), else the lowest free xuid under a
//    generated UUID (registry_load's local UUID on a fresh volume, :575-596).
// The registry entry is written once the front exists.
void xcg_pair_state_set_unbounded(XcgPairState* P) { P->unbounded = true; }
int xcg_pair_state_unbounded(const XcgPairState* P) { return P && P->unbounded ? 1 : 0; }

int xcg_pair_state_create(uint32_t C, XcgDiskState* K, const char* uuid36, int want_xuid, XcgPairState** out) {
  if (C == 0 || !K || (uint64_t)K->D + C >= (1ull << 30)) return -22;
  if (uuid36 && (strlen(uuid36) != 36 || !uuid_ok((const uint8_t*)uuid36))) return -22;
  if (want_xuid >= (int)XUIDS) return -22;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return -5;
  auto bound = [&](uint32_t x) { return x < K->fronts.size() && K->fronts[x] != nullptr; };
  uint32_t xuid = XUIDS;
  if (uuid36)
    for (uint32_t x = 0; x < XUIDS; ++x)
      if (K->uuid[x] == uuid36) { xuid = x; break; }
  if (want_xuid >= 0) {
    if (xuid < XUIDS && xuid != (uint32_t)want_xuid) return -22;
    xuid = (uint32_t)want_xuid;
  } else if (!uuid36 && !K->uuid[0].empty() && !bound(0)) {
    xuid = 0;
  }
  if (xuid < XUIDS && bound(xuid)) return -22;               // (one engine front per disk front)
  if (xuid >= XUIDS)
    for (xuid = 0; xuid < XUIDS && (bound(xuid) || !K->uuid[xuid].empty()); ++xuid) {
    }
  if (xuid >= XUIDS) return -22;                            // XCDFS_XUID_COUNT
  char gen[37];
  const char* name = uuid36;
  if (!name && K->uuid[xuid].empty()) {
    if (!gen_uuid(gen)) return -5;
    name = gen;
  }
  const int brc = disk_bind(K, device);
  if (brc) return brc;
  XcgPairState* P = new XcgPairState;
  P->C = C;
  P->nb = (uint32_t)K->nb;
  P->D = K->D;
  P->disk = K;
  P->xuid = (uint16_t)xuid;
  P->gclock = K->dclock;
  const uint64_t ids = (uint64_t)C + P->D;
  auto fail = [&](int rc) {
    unmap_pool(P);
    (void)hipFree(P->pkey); (void)hipFree(P->pdisk); (void)hipFree(P->lru); (void)hipFree(P->lru2);
    (void)hipFree(P->ptime);
    free_scratch(P);
    delete P;
    return rc;
  };
  if (hipMalloc(&P->pkey, 8ull * C) != hipSuccess || hipMalloc(&P->pdisk, 8ull * C) != hipSuccess ||
      hipMalloc(&P->lru, 4ull * C) != hipSuccess || hipMalloc(&P->lru2, 4ull * C) != hipSuccess ||
      hipMalloc(&P->ptime, 8 * ids) != hipSuccess ||
      hipMalloc(&P->erep, 4 * ids) != hipSuccess ||
      hipMemset(P->pkey, 0xFF, 8ull * C) != hipSuccess || hipMemset(P->pdisk, 0xFF, 8ull * C) != hipSuccess ||
      hipMemset(P->ptime, 0xFF, 8 * ids) != hipSuccess || ensure_front_arrays(P) != 0 || map_pool(P, device) != 0)
    return fail(-12);
  uint8_t* blocks = P->pool + (uint64_t)C * SEG;
  const uint64_t D = K->D;
  if (!K->pending && !K->zeroed) {
    if (hipMemset(blocks, 0, D * SEG) != hipSuccess) return fail(-5);
    K->zeroed = K->vmm;
  }
  if (K->pending) {                                         // a reopened volume's ring and blocks
    if (!K->ring_loaded &&
        (hipMemcpy(K->dkey, K->h_key.data(), 8 * D, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(K->dent, K->h_ent.data(), 8 * D, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(K->dxuid, K->h_xuid.data(), 4 * D, hipMemcpyHostToDevice) != hipSuccess))
      return fail(-5);
    K->ring_loaded = true;
    if (hipMemcpy(blocks, K->h_data.data(), D * SEG, hipMemcpyHostToDevice) != hipSuccess) return fail(-5);
  }
  if (!P->pool_vmm && !K->shadow_ok.empty()) {               // blocks of fronts that went away
    for (uint64_t i = 0; i < D; ++i)
      if (K->shadow_ok[i] &&
          hipMemcpy(blocks + i * SEG, &K->shadow[i * SEG], SEG, hipMemcpyHostToDevice) != hipSuccess)
        return fail(-5);
  }
  if (K->pending && K->vmm) {                                // (one copy serves every front)
    K->pending = false;
    K->zeroed = true;                                        // (the blocks hold the volume's bytes)
    std::vector<uint64_t>().swap(K->h_key);
    std::vector<uint64_t>().swap(K->h_ent);
    std::vector<uint32_t>().swap(K->h_xuid);
    std::vector<uint8_t>().swap(K->h_data);
  }
  if (name && K->uuid[xuid] != name) {
    K->uuid[xuid] = std::string(name, 36);
    registry_write(K, xuid, name);
  }
  P->gstale = true;                                          // (G from the disk's entries at the first call)
  if (xuid >= K->fronts.size()) K->fronts.resize(xuid + 1, nullptr);
  K->fronts[xuid] = P;
  ++K->refs;
  *out = P;
  return 0;
}

// Where the write head is: XCodecDisk's current_index_block_ and
// index_block_next_ (xcodec_cache_disk.cc:701-727).
void xcg_disk_state_head(const XcgDiskState* K, uint64_t* index_block, uint64_t* next) {
  *index_block = (K->dclock / DISK_ENTRIES) % K->nb;
  *next = K->dclock % DISK_ENTRIES;
}

uint32_t xcg_pair_state_xuid(const XcgPairState* P) { return P->xuid; }

// Write the volume as the reference's file stands now (registry, every
// written index block with its counter and entries, the data blocks).
namespace {

struct OnDevice {                 // run on `dev`, restore the caller's device after
  int prev = -1;
  explicit OnDevice(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && prev != dev) (void)hipSetDevice(dev);
  }
  ~OnDevice() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// The disk's blocks through its own mapping of the physical allocation: the
// bytes are there whether or not any front still maps them.
int read_disk_blocks(const XcgDiskState* K, uint8_t* dst) {
  const uint8_t* src = (const uint8_t*)K->dva;
  for (const XcgPairState* f : K->fronts)            // (no mapping of its own: a live front's)
    if (!src && f) src = f->pool + (uint64_t)f->C * SEG;
  if (!src) return -5;
  return hipMemcpy(dst, src, (size_t)K->D * SEG, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -5;
}

}  // namespace

int xcg_disk_state_save(XcgDiskState* K, const char* path) {
  const uint64_t nb = K->nb, D = K->D;
  std::vector<uint64_t> key(D, NOKEY);
  std::vector<uint32_t> xu(D, 0xFFFFFFFFu);
  std::vector<uint8_t> data((size_t)D * SEG, 0);
  if (K->pending && !K->ring_loaded) {
    key = K->h_key;
    xu = K->h_xuid;
    data = K->h_data;
  } else if (K->device >= 0) {
    OnDevice on(K->device);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(key.data(), K->dkey, 8 * D, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(xu.data(), K->dxuid, 4 * D, hipMemcpyDeviceToHost) != hipSuccess)
      return -5;
    if (K->vmm) {
      if (read_disk_blocks(K, data.data())) return -5;
    } else {
      // per-front copies: a block comes from the live front that wrote it,
      // else from what a front that went away left, else from the volume
      if (!K->h_data.empty()) data = K->h_data;
      for (uint64_t i = 0; i < D && !K->shadow_ok.empty(); ++i)
        if (K->shadow_ok[i]) memcpy(&data[i * SEG], &K->shadow[i * SEG], SEG);
      std::vector<uint8_t> tmp((size_t)D * SEG);
      for (XcgPairState* f : K->fronts) {
        if (!f) continue;
        if (hipMemcpy(tmp.data(), f->pool + (uint64_t)f->C * SEG, D * SEG, hipMemcpyDeviceToHost) != hipSuccess)
          return -5;
        for (uint64_t i = 0; i < D; ++i)
          if (xu[i] == f->xuid) memcpy(&data[i * SEG], &tmp[i * SEG], SEG);
      }
    }
  }
  const int fd = ::open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
  if (fd == -1) return -2;
  bool ok = ftruncate(fd, (off_t)K->bytes) == 0;
  ok = ok && pwrite_all(fd, K->reg.data(), K->reg.size(), 0);
  std::vector<uint8_t> ib(2048);
  for (uint64_t b = 0; ok && b < nb; ++b) {
    memset(ib.data(), 0, ib.size());
    if (K->ctr[b] != 0) {
      uint8_t* q = ib.data();
      memcpy(q, &K->ctr[b], 8);
      q += 8;
      for (uint64_t j = 0; j < DISK_ENTRIES; ++j, q += 10) {
        const uint64_t i = b * DISK_ENTRIES + j;
        const uint64_t h = key[i] == NOKEY ? 0 : key[i];
        const uint16_t x = h == 0 ? 0 : (uint16_t)xu[i];
        memcpy(q, &x, 2);
        memcpy(q + 2, &h, 8);
      }
    }
    ok = pwrite_all(fd, ib.data(), 2048, (off_t)((REG_BLOCKS + b) * 2048));
  }
  ok = ok && pwrite_all(fd, data.data(), data.size(), (off_t)((REG_BLOCKS + nb) * 2048));
  close(fd);
  return ok ? 0 : -5;
}

// A volume read through an open descriptor (the reference's XCodecDisk keeps
// its file open as fd_, xcodec_cache_disk.cc:840-871): reloaded when it holds
// one (a non-empty file), else a fresh disk.
int xcg_disk_state_open_fd(int fd, uint64_t disk_bytes, uint32_t flags, XcgDiskState** out) {
  XcgDiskState* K = nullptr;
  const int rc = xcg_disk_state_create(disk_bytes, flags, &K);
  if (rc) return rc;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    delete K;
    return -2;
  }
  if (st.st_size > 0 && load_volume(K, fd) != 0) {
    delete K;
    return -2;
  }
  *out = K;
  return 0;
}

// Open a volume file: reloaded when it holds one, else a fresh disk.
int xcg_disk_state_open(const char* path, uint64_t disk_bytes, uint32_t flags, XcgDiskState** out) {
  const int fd = ::open(path, O_RDONLY);
  if (fd == -1) {
    if (errno == ENOENT) return xcg_disk_state_create(disk_bytes, flags, out);
    return -2;
  }
  const int rc = xcg_disk_state_open_fd(fd, disk_bytes, flags, out);
  close(fd);
  return rc;
}

uint8_t* xcg_pair_state_pool(const XcgPairState* P) { return P->pool; }
int xcg_disk_state_tier(const XcgDiskState* K) { return K->tier; }

// A front goes away (its XCodecCache is deleted): its entries leave the ring's
// index (XCodecDisk::disconnect).
void xcg_pair_state_destroy(XcgPairState* P) {
  if (!P) return;
  XcgDiskState* K = P->disk;
  (void)hipDeviceSynchronize();
  if (K && K->dent && !P->pool_vmm) {                        // keep the blocks this front wrote
    const uint64_t D = K->D;
    std::vector<uint32_t> xu(D);
    std::vector<uint8_t> tmp((size_t)D * SEG);
    if (hipMemcpy(xu.data(), K->dxuid, 4 * D, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(tmp.data(), P->pool + (uint64_t)P->C * SEG, D * SEG, hipMemcpyDeviceToHost) == hipSuccess) {
      if (K->shadow_ok.empty()) {
        K->shadow.assign((size_t)D * SEG, 0);
        K->shadow_ok.assign(D, 0);
      }
      for (uint64_t i = 0; i < D; ++i)
        if (xu[i] == P->xuid) {
          memcpy(&K->shadow[i * SEG], &tmp[i * SEG], SEG);
          K->shadow_ok[i] = 1;
        }
    }
  }
  if (K && K->dent)
    hipLaunchKernelGGL(pair_drop_front_kernel, dim3(grid_for(K->D)), dim3(256), 0, nullptr, K->dkey, K->dent,
                       (const uint32_t*)K->dxuid, K->D, (uint32_t)P->xuid);
  (void)hipDeviceSynchronize();
  unmap_pool(P);
  (void)hipFree(P->pkey); (void)hipFree(P->pdisk); (void)hipFree(P->lru); (void)hipFree(P->lru2);
  (void)hipFree(P->ptime);
  free_scratch(P);
  if (K) {
    K->fronts[P->xuid] = nullptr;
    xcg_disk_state_release(K);
  }
  delete P;
}

// Drop everything this front holds (XCodecCache objects have no clear: this is
// a fresh front; on a disk of its own, a fresh volume).  The caller wipes G.
int xcg_pair_state_clear(XcgPairState* P) {
  XcgDiskState* K = P->disk;
  uint64_t others = 0;
  for (const XcgPairState* f : K->fronts) others += f && f != P;
  if (hipMemset(P->pkey, 0xFF, 8ull * P->C) != hipSuccess || hipMemset(P->pdisk, 0xFF, 8ull * P->C) != hipSuccess)
    return -5;
  hipLaunchKernelGGL(pair_drop_front_kernel, dim3(grid_for(K->D)), dim3(256), 0, nullptr, K->dkey, K->dent,
                     (const uint32_t*)K->dxuid, K->D, others ? (uint32_t)P->xuid : NIL);
  if (!others) {                                             // a fresh volume
    K->dclock = 0;
    K->ctr.assign(K->nb, 0);
    K->ibc = 1;
  }
  P->pcount = 0;
  P->gclock = K->dclock;
  P->gstale = false;
  P->prev_passes = 1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -5;
}

void xcg_pair_state_stats(const XcgPairState* P, uint64_t* st) {
  const XcgDiskState* K = P->disk;
  uint32_t h = 0;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 4) == hipSuccess && hipMemset(d, 0, 4) == hipSuccess) {
    hipLaunchKernelGGL(pair_count_live_kernel, dim3(grid_for(K->D)), dim3(256), 0, nullptr, (const uint64_t*)K->dent,
                       (const uint32_t*)K->dxuid, K->D, (uint32_t)K->nb, K->dclock, (uint32_t)P->xuid, d);
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  }
  (void)hipFree(d);
  st[0] = P->pcount;
  st[1] = h;
  st[2] = K->dclock;
  st[3] = P->nb;
}

uint32_t xcg_pair_state_last_base(const XcgPairState* P) { return P->last_base; }
uint32_t xcg_pair_state_limit(const XcgPairState* P) { return P->C; }
uint32_t xcg_pair_state_disk_blocks(const XcgPairState* P) { return P->D; }
XcgDiskState* xcg_pair_state_disk(const XcgPairState* P) { return P->disk; }
const uint64_t* xcg_pair_state_ptime(const XcgPairState* P) { return P->ptime; }

int xcg_pair_sync(XcgPairState* P, const PairGpu* G, hipStream_t st) { return pair_sync_front(P, *G, st); }

// Decode on the pair, first step: ptime NEVER everywhere.
int xcg_pair_decode_begin(XcgPairState* P, hipStream_t st) { return fill_ptime(P, st); }

// One replay of a decode batch's classified ops (rows packed per chunk at
// d_base[c], d_cnt[c] of them; `rows` total).  *same = the departure times it
// computes equal those the classification used (then it was the sequential
// decoder's).  Otherwise ptime is updated for the next classification.
// Returns 0, -95 (a batch the pair model declines: a hash this batch named
// gone before a later lookup, more than a disk lap of writes), -5.
int xcg_pair_decode_pass(XcgPairState* P, const PairGpu* G, const void* d_rows, const uint64_t* d_base,
                         const uint64_t* d_cnt, uint32_t n, uint64_t rows, uint32_t maxd, int* same, hipStream_t st) {
  RowSrc rs{1, n, maxd, (const uint4*)d_rows, nullptr, 0u, d_base, d_cnt, rows, nullptr, nullptr, nullptr};
  PassOut o;
  const HashTab g{G->g_keys, G->g_vals, G->g_mask};
  const int rc = replay(P, rs, g, true, &o, st);
  if (rc) return rc;
  if (o.split) return -95;
  *same = !o.changed;
  return 0;
}

// Keep the last decode replay and commit it (bytes from the batch input at the
// declaration rows: G.decl[c * maxd + d].z = the EXTRACT payload's offset).
int xcg_pair_decode_commit(XcgPairState* P, const PairGpu* G, hipStream_t st) {
  const int rc = pair_commit(P, *G, st);
  if (fill_ptime(P, st)) return -5;
  return rc;
}

// Stream-semantics encode of a batch on the pair, in sub-batches (see the top
// of this file).  Returns 0, -75 (no consistent pass / overflow), -95 (one
// chunk alone exceeds what a sub-batch may hold), -5.
int xcg_pair_encode_stream(const XcgStreamArgs* a0, XcgPairState* P, int* rounds_out, hipStream_t st) {
  const uint32_t n = a0->n;
  int rounds = 0;
  if (pair_sync_front(P, gpu_of(*a0), st)) return -5;
  // A sub-batch is bounded by the disk only: while it writes fewer than a lap
  // of disk blocks, nothing it declared can leave both levels within it (a
  // chunk writes at most maxd declarations plus its touches).
  const uint64_t lap = P->D > 2 * DISK_ENTRIES ? P->D - 2 * DISK_ENTRIES : 1;
  // (maxd writes per chunk at most; the rate a previous sub-batch measured is
  // used when it allows more -- a sub-batch that still laps the disk is split)
  uint32_t per = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, std::max<uint64_t>(lap / a0->maxd, P->fit_per)));
  constexpr int MAX_PASSES = 12;
  uint32_t i0 = 0;
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const HashTab g{a0->g_keys, a0->g_vals, a0->g_mask};
  while (i0 < n) {
    const clk::time_point t0 = clk::now();
    // what is left in equal parts of at most `per` chunks (no short tail
    // sub-batch: each costs a replay and a commit whatever its size)
    const uint32_t rem = n - i0, parts = (rem + per - 1) / per;
    const uint32_t m = (rem + parts - 1) / parts;
    XcgStreamArgs a = *a0;
    a.n = m;
    a.chunk_off += i0;
    a.chunk_len += i0;
    a.out_off += i0;
    a.out_len += i0;
    if (a.stats) a.stats += 4ull * i0;
    a.ptime = P->ptime;
    a.no_commit = 1;
    RowSrc rs{0, m, a.maxd, (const uint4*)a.ev, a.nev, a.maxe, nullptr, nullptr, 0, a.need, a.bad_t, a.bad_hi};
    auto clear_flags = [&]() {
      return hipMemsetAsync(a.need, 0, 4ull * m, st) == hipSuccess &&
             (!a.bad_t || (hipMemsetAsync(a.bad_t, 0xFF, 4ull * m, st) == hipSuccess &&
                           hipMemsetAsync(a.bad_hi, 0, 4ull * m, st) == hipSuccess));
    };
    uint32_t* scratch_flags = nullptr;
    if (!a.bad_t) {                                  // (no restart arrays: flags into scratch)
      if (hipMallocAsync((void**)&scratch_flags, 8ull * m, st) != hipSuccess) return -5;
      rs.bad_t = scratch_flags;
      rs.bad_hi = scratch_flags + m;
    }
    auto done_scratch = [&]() {
      if (scratch_flags) (void)hipFreeAsync(scratch_flags, st);
    };
    // The rounds start from each chunk's tiling (its cold parse).  ptime is
    // NEVER (no cached entry leaves) unless the last sub-batch needed more than
    // one pass: then the first guess is the tiling seed's own references,
    // replayed (a cached tile is a lookup hit, a repeat of an earlier tile a hit
    // on its declaration, every other tile a declaration).
    if (xcg_launch_seed_tiling(&a, st)) { done_scratch(); return -5; }
    const clk::time_point t1 = clk::now();
    if (P->prev_passes > 1) {
      const HashTab b{a.b_keys, a.b_vals, a.b_mask};
      hipLaunchKernelGGL(pr_fill64_kernel, dim3(1024), dim3(256), 0, st, b.keys, (uint64_t)b.mask + 1, EMPTY_KEY);
      hipLaunchKernelGGL(pr_fill64_kernel, dim3(1024), dim3(256), 0, st, b.vals, (uint64_t)b.mask + 1, ~0ull);
      hipLaunchKernelGGL(pair_seed_table_kernel, dim3(grid_for((uint64_t)m * a.maxd)), dim3(256), 0, st, m,
                         (const uint4*)a.decl, (const uint32_t*)a.ndecl, a.maxd, b, a.status);
      // guess 0 takes every cached tile for a hit; each further guess
      // classifies against the departure times the one before implies
      // (XCG_PAIR_SEED_ITERS)
      const int iters = pair_seed_iters();
      for (int it = 0; it < iters; ++it) {
        hipLaunchKernelGGL(pair_seed_events_kernel, dim3((m + 3) / 4), dim3(256), 0, st, m, (const uint4*)a.decl,
                           (const uint32_t*)a.ndecl, a.maxd, a.chunk_len, g, b, (uint4*)a.ev, a.nev, a.maxe,
                           it ? (const uint64_t*)P->ptime : nullptr);
        if (!clear_flags()) { done_scratch(); return -5; }
        PassOut o;
        const int rc = replay(P, rs, g, true, &o, st);
        if (rc) { done_scratch(); return rc; }
        if (o.split) break;                        // (a guess the replay declines: keep the last times)
      }
    }
    const clk::time_point t2 = clk::now();
    double t_parse = 0, t_replay = 0;
    bool done = false, split = false;
    int passes = 0;
    for (int pass = 0; pass < MAX_PASSES && !done && !split; ++pass) {
      ++passes;
      a.keep_decls = 1;
      a.need_given = pass > 0;
      int r = 0;
      const clk::time_point q0 = clk::now();
      const int rc = xcg_launch_encode_stream(&a, &r, st);
      rounds += r;
      if (rc) { done_scratch(); return rc; }
      if (pair_debug()) (void)hipStreamSynchronize(st);
      const clk::time_point q1 = clk::now();
      if (!clear_flags()) { done_scratch(); return -5; }
      PassOut o;
      const int prc = replay(P, rs, g, false, &o, st);
      if (prc == -75) { split = true; break; }
      if (prc) { done_scratch(); return prc; }
      const clk::time_point q2 = clk::now();
      t_parse += ms(q0, q1);
      t_replay += ms(q1, q2);
      if (pair_debug())
        fprintf(stderr, "pair: chunks %u+%u pass %d rounds %d appends %llu bad %u split %d\n", i0, m, pass, r,
                (unsigned long long)o.appends, o.nbad, (int)o.split);
      if (o.split) split = true;
      else if (o.nbad == 0) done = true;
      // else: the replay flagged the chunks (need / bad_t / bad_hi) and set ptime
    }
    if (!done) {
      done_scratch();
      if (m == 1) return split ? -95 : -75;
      per = m / 2;                                 // redo this part in halves
      P->fit_per = 0;                              // (and size the next call from the worst case again)
      P->prev_passes = MAX_PASSES;
      if (fill_ptime(P, st)) return -5;
      continue;
    }
    const clk::time_point t3 = clk::now();
    const PairGpu G = gpu_of(a);
    if (const int crc = pair_commit(P, G, st)) { done_scratch(); return crc == -75 ? -75 : -5; }
    done_scratch();
    if (pair_debug())
      fprintf(stderr, "pair: ms seed %.2f seed-replay %.2f parse %.2f replay %.2f commit %.2f (primary %u, clock %llu)\n",
              ms(t0, t1), ms(t1, t2), t_parse, t_replay, ms(t3, clk::now()), P->pcount,
              (unsigned long long)P->disk->dclock);
    // the next sub-batch starts with every hash visible to its end
    if (fill_ptime(P, st)) return -5;
    P->last_base = i0;
    P->prev_passes = passes;
    i0 += m;
    // size the next sub-batch from the disk blocks this one wrote
    const uint64_t useD = P->appends;
    uint64_t want = (uint64_t)n;
    if (useD) {
      want = std::min<uint64_t>(want, lap * 9 / 10 * m / useD);
      P->fit_per = (uint32_t)std::min<uint64_t>(lap * 9 / 10 * m / useD, 1u << 30);
    }
    per = (uint32_t)(want < 1 ? 1 : (want > n ? n : want));
  }
  if (rounds_out) *rounds_out = rounds;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
