// XCodecCachePair (xcodec/xcodec_cache.h:140-237) of a bounded
// XCodecMemoryCache primary (:245-365, XCodecLRU xcodec/xcodec_lru.h) and an
// XCodecDisk secondary (xcodec/xcodec_cache_disk.{h,cc}): wanproxy.conf's
// cache, `memory` + `disk` under a `pair` (programs/wanproxy/wanproxy.conf:
// 8-26).  Stream-semantics encode batches stay bit-exact with the sequential
// XCodecEncoder on such a pair.
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
// Division of work.  The GPU parses (encode_stream_kernel, the same rounds as
// every stream batch) against G = one table over the union of both levels:
// id s < C = primary slot s, id C + i = disk data block i (a hash in both maps
// to its primary slot); the pool holds C + nb*204 segments, so `pool + id *
// 2048` is the hash's bytes either way.  The parse takes, per id, the batch
// time from which the hash is gone from both levels (ptime) as given and
// records every cache reference it makes, in order (ENTER / HIT / GHIT /
// GMISS, xcg_cache.h).  The host replays those references through the pair's
// exact policy over metadata only (XcgPairState below: the primary's LRU list, the
// disk ring, the links between them) -- a sequential walk over a few tens of
// thousands of references -- and checks every recorded lookup against it.
// All consistent = the sequential encoder's result (by induction over stream
// time); otherwise the inconsistent chunks are parsed again under the replay's
// ptime.  An entry a sub-batch made must not leave both levels and then be
// looked up within it (the parse sees the batch's declarations to its end);
// the replay detects that and the sub-batch is halved.  The commit then moves bytes on the GPU (input ->
// new primary / disk slots, disk -> promoted primary slots, primary -> touched
// disk slots, through a staging copy) and rebuilds G and its probe filters.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "xcg_cache.h"
#include "xcg_args.h"

namespace xcg {

constexpr uint32_t DISK_ENTRIES = 204;   // XCDFS_ENTRIES_PER_INDEX_BLOCK, xcodec_cache_disk.cc:87

__global__ __launch_bounds__(256) void pair_fill64_kernel(uint64_t* p, uint64_t n, uint64_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// dst[kv[2j]] = kv[2j + 1]
__global__ __launch_bounds__(256) void pair_scatter64_kernel(uint64_t* dst, const uint64_t* kv, uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) dst[kv[2 * j]] = kv[2 * j + 1];
}

// Seed tiles in a batch table: hash -> earliest (chunk << 32 | position).
__global__ __launch_bounds__(256) void pair_seed_table_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                              uint32_t maxd, HashTab b, int32_t* status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (uint32_t)(i / maxd), d = (uint32_t)(i % maxd);
  if (c >= n || d >= ndecl[c]) return;
  const uint4 dd = decl[i];
  if (!tab_insert_min(b, dd.x, dd.y, ((uint64_t)c << 32) | dd.z)) atomicOr(status, 2);
}

// First guess of a sub-batch's references, before any parse: every chunk
// parses as its 2048-byte tiling (its cold parse), a tile found in G being a
// lookup hit, a repeat of an earlier tile of the batch a hit on that
// declaration, and every other tile a declaration, entered while the window
// 2048 bytes on (or after the last window) is examined.  One event per tile,
// in the same row format the parse records.
__global__ __launch_bounds__(256) void pair_seed_events_kernel(uint32_t n, const uint4* decl, const uint32_t* ndecl,
                                                               uint32_t maxd, const uint32_t* chunk_len, HashTab g,
                                                               HashTab b, uint4* ev, uint32_t* nev, uint32_t maxe) {
  const uint32_t c = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (c >= n) return;
  const uint32_t nd = min(ndecl[c], maxe), last = chunk_len[c] - SEG;
  for (uint32_t d = (uint32_t)lane_id(); d < nd; d += 64) {
    const uint4 dd = decl[(uint64_t)c * maxd + d];
    const uint64_t gv = tab_lookup_t(g, dd.x, dd.y);
    uint4 e;
    if (gv != ~0ull) {
      e = make_uint4(dd.x, dd.y, 2u * dd.z + 1u, (EV_GHIT << 30) | (uint32_t)gv);
    } else if (tab_lookup_t(b, dd.x, dd.y) == (((uint64_t)c << 32) | dd.z)) {
      const uint32_t t = dd.z + SEG <= last ? 2u * (dd.z + SEG) : 2u * (last + 1u);
      e = make_uint4(dd.x, dd.y, t, (EV_ENTER << 30) | d);
    } else {
      e = make_uint4(dd.x, dd.y, 2u * dd.z + 1u, EV_HIT << 30);
    }
    ev[(uint64_t)c * maxe + d] = e;
  }
  if (lane_id() == 0) nev[c] = nd;
}

// Commit moves: w = (destination pool index, kind, a, b); kind 0: the bytes of
// declaration b of chunk a (input), kind 1: the pre-batch bytes of pool index a
// (staged first into staging slot b, so no move reads what another overwrote).
__global__ __launch_bounds__(256) void pair_stage_kernel(const uint4* w, uint32_t nw, const uint8_t* pool,
                                                         uint8_t* staging) {
  const uint32_t j = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (j >= nw) return;
  const uint4 m = w[j];
  if (m.y != 1u) return;
  const uint8_t* src = pool + (uint64_t)m.z * SEG;
  uint8_t* dst = staging + (uint64_t)m.w * SEG;
  const int l = lane_id();
  *(u32x4_u*)(dst + 32 * l) = *(const u32x4_u*)(src + 32 * l);
  *(u32x4_u*)(dst + 32 * l + 16) = *(const u32x4_u*)(src + 32 * l + 16);
}

__global__ __launch_bounds__(256) void pair_move_kernel(const uint4* w, uint32_t nw, const uint8_t* in,
                                                        const uint64_t* chunk_off, const uint4* decl, uint32_t maxd,
                                                        const uint8_t* staging, uint8_t* pool) {
  const uint32_t j = blockIdx.x * 4u + readfirst(threadIdx.x >> 6);
  if (j >= nw) return;
  const uint4 m = w[j];
  const uint8_t* src = m.y == 0u ? in + chunk_off[m.z] + decl[(uint64_t)m.z * maxd + m.w].z
                                 : staging + (uint64_t)m.w * SEG;
  uint8_t* dst = pool + (uint64_t)m.x * SEG;
  const int l = lane_id();
  *(u32x4_u*)(dst + 32 * l) = *(const u32x4_u*)(src + 32 * l);
  *(u32x4_u*)(dst + 32 * l + 16) = *(const u32x4_u*)(src + 32 * l + 16);
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

// G from the per-id keys (EMPTY_KEY: no hash there, or a disk block whose hash
// also sits in the primary), plus the probe filters and the key count.
__global__ __launch_bounds__(256) void pair_rebuild_kernel(const uint64_t* keyg, uint32_t n, HashTab g, FiltSet fs,
                                                           uint32_t* nseg, int32_t* status) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t k = id < n ? keyg[id] : EMPTY_KEY;
  const bool have = k != EMPTY_KEY;
  if (have) {
    if (!tab_insert_min(g, (uint32_t)k, (uint32_t)(k >> 32), id)) atomicOr(status, 2);
    filt_insert(fs, (uint32_t)k, (uint32_t)(k >> 32));
  }
  const uint64_t m = ballot(have);
  if (lane_id() == 0 && m) atomicAdd(nseg, (uint32_t)__builtin_popcountll(m));
}

}  // namespace xcg

namespace {

using namespace xcg;
constexpr uint32_t NIL = 0xFFFFFFFFu;
constexpr uint64_t NEVER = ~0ull;
constexpr uint64_t NOKEY = ~0ull;

bool pair_debug() {
  static const bool on = getenv("XCG_PAIR_DEBUG") != nullptr;
  return on;
}

// Open-addressed u64 -> u32 map whose slots are tagged with an epoch, so a
// new pass clears it in O(1); one 16-byte slot per probe.
struct EpochMap {
  struct Slot {
    uint64_t key;
    uint32_t val, tag;
  };
  std::vector<Slot> t;
  uint64_t mask = 0;
  uint32_t epoch = 0;
  void reset(uint64_t want) {
    uint64_t cap = 1024;
    while (cap < 2 * want + 16) cap <<= 1;
    if (cap > t.size()) {
      t.assign(cap, Slot{0, 0, 0});
      epoch = 0;
    }
    mask = t.size() - 1;
    if (++epoch == 0) {
      for (Slot& q : t) q.tag = 0;
      epoch = 1;
    }
  }
  static uint64_t mixk(uint64_t k) {
    k ^= k >> 31;
    k *= 0x9E3779B97F4A7C15ull;
    return k ^ (k >> 29);
  }
  void prefetch(uint64_t k) const { __builtin_prefetch(&t[mixk(k) & mask]); }
  uint32_t find(uint64_t k) const {
    for (uint64_t i = mixk(k) & mask;; i = (i + 1) & mask) {
      const Slot& q = t[i];
      if (q.tag != epoch) return NIL;
      if (q.key == k) return q.val;
    }
  }
  void put(uint64_t k, uint32_t v) {
    for (uint64_t i = mixk(k) & mask;; i = (i + 1) & mask) {
      Slot& q = t[i];
      if (q.tag != epoch || q.key == k) {
        q.tag = epoch;
        q.key = k;
        q.val = v;
        return;
      }
    }
  }
};

}  // namespace

// The pair's metadata (host, authoritative) and one replay pass over a
// sub-batch's references.  Slots: primary s in [0, C), disk data block i in
// [0, D).  Entities: the hash in primary slot s at the sub-batch start is
// entity s, a hash only on disk at the start is entity C + i, the pass's own
// declarations are C + D + k.  A pass never writes the committed arrays: it
// works on epoch-tagged copies of the slots it touches, which the commit
// copies back (so an inconsistent pass is dropped for free).
// One primary slot / disk block / entity record each in one cache line:
// the committed fields, then the pass's copy (valid while ep == the pass's
// epoch).
//
// The disk is shared.  XCodecDisk is one FIFO for every XCodecDiskCache
// front-end on it (xcodec/xcodec_cache_disk.h:33-69): the local cache and each
// peer cache XCodecCache::connect makes (XCodecDisk::connect, xcodec_cache_
// disk.cc:640-690) append to the same ring, index entries carry the front's
// xuid, and when the write head enters an index block every front loses the
// entries it still had there (index_invalidate_entries, :327-382, walking
// xuid_cache_map_).  So the ring (XcgDiskState: blocks, their owner xuid, the
// write clock) is one object; each pair context is a front (its xuid, its
// primary, its hash index = the live blocks it owns).  A front's pass may
// invalidate another front's entries: they are applied to that front when the
// pass is kept, and reach its GPU table at its next call (pending list).
struct PSlot {
  uint64_t key, okey;              // hash (NOKEY: free)
  uint32_t prev, next, pd;         // LRU links; the hash's disk block (NIL: not on disk)
  uint32_t oprev, onext, opd, owner, ep;
};
struct DSlot {
  uint64_t key, okey;
  uint32_t dp, odp;                // the hash's primary slot in its owner front (NIL: disk only)
  uint32_t owner, ep;              // (owner: entity of the pass's front, FOREIGN for another front's entry)
  uint16_t xuid, oxuid;            // the front whose index entry this is (XCodecDisk index entry xuid)
  uint8_t live, olive;             // the disk index's entry for its hash
};
struct Ent {                       // a hash cached at the sub-batch start
  uint64_t leave;                  // time it left both levels (NEVER)
  uint32_t ep, p, d;
  uint8_t ref;
};
struct NewEnt {                    // a declaration of the pass
  uint64_t key;
  uint32_t p, d, chunk, decl;
};
constexpr uint32_t FOREIGN = 0xFFFFFFFEu;

struct XcgPairState;

// One XCodecDisk: the ring and the fronts on it.
struct XcgDiskState {
  uint64_t nb = 0;                 // index blocks
  uint32_t D = 0;                  // nb * 204 data blocks
  uint64_t dclock = 0;             // entries written to the disk (every front)
  uint32_t epoch = 0;              // pass epochs, unique across the fronts
  std::vector<DSlot> ds;
  std::vector<XcgPairState*> fronts;   // by xuid (nullptr: free)
  int refs = 1;                    // the creator's reference + one per front
};

struct XcgPairState {
  uint32_t C = 0;                  // primary limit in segments
  uint64_t nb = 0;                 // disk index blocks
  uint32_t D = 0;                  // nb * 204 disk data blocks
  XcgDiskState* disk = nullptr;
  uint16_t xuid = 0;
  // committed scalars
  uint32_t head = NIL, tail = NIL, pcount = 0, ftop = 0;
  std::vector<uint32_t> pfree;     // free primary slots, pfree[0 .. ftop)
  uint64_t dlive = 0;              // this front's live disk index entries
  std::vector<PSlot> ps;
  std::vector<DSlot>* dsp = nullptr;
  // another front's kept pass took index entries of ours: ids to clear in keyg
  std::vector<uint64_t> pending;
  // pass state
  uint32_t epoch = 0;
  std::vector<uint32_t> touchedP, touchedD;
  uint32_t s_head, s_tail, s_pcount, s_ftop;
  uint64_t s_dclock, s_dlive;
  std::vector<Ent> es;
  std::vector<uint32_t> touchedE;
  std::vector<NewEnt> ns;
  EpochMap bmap;                   // hash -> the pass's declaration (decode: any entity of the hash)
  // pass results
  bool split = false;
  std::vector<uint8_t> bad;        // per chunk: a recorded lookup the replay contradicts
  std::vector<uint32_t> blo, bhi;  // ... the in-chunk times of the first and last such lookup
  std::vector<uint4> writes;       // commit moves (dest, kind, a, b)
  uint32_t nstaged = 0;
  uint64_t enters = 0, refs = 0, appends = 0;
  std::vector<uint64_t> leaves;    // decode: the (id, leave time) list ptime was last built from
  // device
  uint64_t* d_keyg = nullptr;      // [C + D]
  uint64_t* d_ptime = nullptr;     // [C + D]
  uint8_t* d_staging = nullptr;
  uint64_t staging_cap = 0;
  uint8_t* d_xfer = nullptr;       // upload area (moves, key updates, ptime list)
  uint64_t xfer_cap = 0;
  uint8_t* h_xfer = nullptr;       // pinned
  uint64_t h_xfer_cap = 0;
  uint4* h_ev = nullptr;           // pinned copy of the reference rows
  uint64_t h_ev_cap = 0;
  uint32_t* h_nev = nullptr;
  uint32_t h_nev_cap = 0;
  uint32_t* h_need = nullptr;
  uint64_t* h_base = nullptr;      // decode: per-chunk row base and count (pinned)
  uint32_t h_base_cap = 0;
  uint32_t last_base = 0;
  int prev_passes = 1;             // passes the last sub-batch needed

  uint32_t ids() const { return C + D; }
  std::vector<DSlot>& ds() { return *dsp; }
  const std::vector<DSlot>& ds() const { return *dsp; }

  // ---- the pass's view of a slot / block / entity (copied on first use)
  PSlot& P(uint32_t s) {
    PSlot& q = ps[s];
    if (q.ep != epoch) {
      q.ep = epoch;
      q.okey = q.key; q.oprev = q.prev; q.onext = q.next; q.opd = q.pd;
      q.owner = q.key != NOKEY ? s : NIL;
      touchedP.push_back(s);
    }
    return q;
  }
  DSlot& Dk(uint32_t i) {
    DSlot& q = ds()[i];
    if (q.ep != epoch) {
      q.ep = epoch;
      q.okey = q.key; q.olive = q.live; q.odp = q.dp; q.oxuid = q.xuid;
      q.owner = !q.live ? NIL : (q.xuid != xuid ? FOREIGN : (q.dp != NIL ? q.dp : C + i));
      touchedD.push_back(i);
    }
    return q;
  }
  Ent& E(uint32_t x) {
    Ent& e = es[x];
    if (e.ep != epoch) {
      e.ep = epoch;
      if (x < C) {
        const PSlot& q = ps[x];              // committed fields: the sub-batch start
        e.p = q.key != NOKEY ? x : NIL;
        e.d = e.p != NIL ? q.pd : NIL;
      } else {
        const DSlot& q = ds()[x - C];
        e.p = NIL;
        e.d = q.live && q.xuid == xuid && q.dp == NIL ? x - C : NIL;
      }
      e.ref = 0;
      e.leave = NEVER;
      touchedE.push_back(x);
    }
    return e;
  }
  bool is_new(uint32_t x) const { return x >= C + D; }
  // (XCG_PAIR_DEBUG) a recorded lookup the replay contradicts
  void bad_row(uint32_t kind, uint32_t x, uint64_t h, uint64_t t) {
    fprintf(stderr, "pair bad: xuid %u kind %u id %u%s t %llx hash %016llx key %016llx p %d d %d", xuid, kind, x,
            is_new(x) ? " (new)" : "", (unsigned long long)t, (unsigned long long)h, (unsigned long long)ekey(x),
            (int)ep(x), (int)ed(x));
    if (x >= C && !is_new(x)) {
      const DSlot& q = ds()[x - C];
      fprintf(stderr, " | block live %u xuid %u dp %d olive %u oxuid %u odp %d ep %u/%u", q.live, q.xuid, (int)q.dp,
              q.olive, q.oxuid, (int)q.odp, q.ep, epoch);
    } else if (x < C) {
      const PSlot& q = ps[x];
      fprintf(stderr, " | slot key %016llx pd %d okey %016llx opd %d ep %u/%u", (unsigned long long)q.key, (int)q.pd,
              (unsigned long long)q.okey, (int)q.opd, q.ep, epoch);
    }
    fprintf(stderr, "\n");
  }
  void mark_bad(uint32_t c, uint32_t t) {
    bad[c] = 1;
    blo[c] = t < blo[c] ? t : blo[c];
    bhi[c] = t > bhi[c] ? t : bhi[c];
  }
  // an entity's current primary slot / disk block
  uint32_t& ep(uint32_t x) { return is_new(x) ? ns[x - C - D].p : E(x).p; }
  uint32_t& ed(uint32_t x) { return is_new(x) ? ns[x - C - D].d : E(x).d; }
  uint64_t ekey(uint32_t x) const {
    return is_new(x) ? ns[x - C - D].key : (x < C ? ps[x].key : ds()[x - C].key);
  }
  bool present(uint32_t x) { return ep(x) != NIL || ed(x) != NIL; }
  // commit move of entity x's bytes to pool index `dest`
  void move_to(uint32_t dest, uint32_t x) {
    if (is_new(x)) writes.push_back(make_uint4(dest, 0u, ns[x - C - D].chunk, ns[x - C - D].decl));
    else writes.push_back(make_uint4(dest, 1u, x, nstaged++));
  }
  // x is in neither level from time t on.  A cached entry's departure becomes
  // its ptime; one this sub-batch made has no ptime (the parse sees the batch's
  // declarations to its end), so a later lookup of it splits the sub-batch.
  void left(uint32_t x, uint64_t t) {
    if (!is_new(x)) E(x).leave = t;
  }

  // ---- the primary's LRU list (xcodec_lru.h: enter / use move to the tail, evict takes the head)
  void unlink(PSlot& q) {
    const uint32_t p = q.oprev, n = q.onext;
    if (p != NIL) P(p).onext = n; else s_head = n;
    if (n != NIL) P(n).oprev = p; else s_tail = p;
  }
  void append(uint32_t s, PSlot& q) {
    q.oprev = s_tail;
    q.onext = NIL;
    if (s_tail != NIL) P(s_tail).onext = s; else s_head = s;
    s_tail = s;
  }

  // XCodecMemoryCache::enter (xcodec_cache.h:303-325)
  void p_enter(uint32_t x, uint64_t t) {
    uint32_t s;
    if (s_pcount == C) {
      s = s_head;
      PSlot& q = P(s);
      const uint32_t y = q.owner;
      unlink(q);
      --s_pcount;
      ep(y) = NIL;
      if (q.opd != NIL) Dk(q.opd).odp = NIL;      // now on disk only
      else left(y, t);
    } else {
      s = pfree[--s_ftop];
    }
    PSlot& q = P(s);
    if (s_head != NIL) {                           // the next victim and what it links to
      const PSlot& h = ps[s_head];
      __builtin_prefetch(&es[s_head < C ? s_head : 0]);
      if (h.onext != NIL && h.ep == epoch) __builtin_prefetch(&ps[h.onext]);
      else if (h.next != NIL) __builtin_prefetch(&ps[h.next]);
      const uint32_t hd = h.ep == epoch ? h.opd : h.pd;
      if (hd != NIL) __builtin_prefetch(&ds()[hd]);
    }
    q.okey = ekey(x);
    q.owner = x;
    ep(x) = s;
    append(s, q);
    ++s_pcount;
    const uint32_t dj = ed(x);
    q.opd = dj;
    if (dj != NIL) Dk(dj).odp = s;
    move_to(s, x);
    ++enters;
  }

  // XCodecDisk::enter (xcodec_cache_disk.cc:694-741): the shared write head
  void d_append(uint32_t x, uint64_t t) {
    const uint32_t i = (uint32_t)(s_dclock % D);
    DSlot& q = Dk(i);
    q.okey = ekey(x);
    q.olive = 1;
    q.oxuid = xuid;
    q.owner = x;
    const uint32_t p = ep(x);
    q.odp = p;
    if (p != NIL) P(p).opd = i;
    ed(x) = i;
    move_to(C + i, x);
    ++s_dlive;
    ++appends;
    if (++s_dclock % DISK_ENTRIES == 0) {          // the write head moves on: index_invalidate_entries
      const uint64_t b = (s_dclock / DISK_ENTRIES) % nb;
      for (uint32_t j = (uint32_t)(b * DISK_ENTRIES); j < (uint32_t)((b + 1) * DISK_ENTRIES); ++j) {
        DSlot& r = Dk(j);
        if (!r.olive) continue;
        const uint32_t y = r.owner;
        r.olive = 0;
        r.owner = NIL;
        if (y == FOREIGN) continue;                // another front's entry: applied to it at keep()
        --s_dlive;
        ed(y) = NIL;
        if (r.odp != NIL) P(r.odp).opd = NIL;      // now in the primary only
        else left(y, t);
      }
    }
  }

  // XCodecCachePair::lookup on a hash present in a level (:208-230)
  void lookup(uint32_t x, uint64_t t) {
    if (!is_new(x)) {
      Ent& e = E(x);
      if (!e.ref) {
        e.ref = 1;
        ++refs;                                    // distinct cached entries referenced
      }
    }
    const uint32_t p = ep(x);
    if (p != NIL) {
      PSlot& q = P(p);
      if (s_tail != p) {                           // XCodecLRU::use
        unlink(q);
        append(p, q);
      }
      if (ed(x) == NIL) d_append(x, t);            // XCodecDisk::touch
    } else {
      p_enter(x, t);                               // promotion
    }
  }

  // XCodecCachePair::replace (xcodec_cache.h:187-196) right after a lookup of
  // x found other bytes (the decoder's name reuse, xcodec_decoder.cc:110-133;
  // <LEARN>, xcodec_pipe_pair.cc:311-327): the primary keeps the slot (an LRU
  // use: x is at the tail already) with the new bytes; the disk removes the
  // hash and enters it again (XCodecDiskCache::replace, xcodec_cache_disk.h).
  // The new bytes are a new entity y in x's place; x has left.
  void replace(uint32_t x, uint64_t h, uint32_t c, uint32_t d, uint64_t t) {
    const uint32_t y = C + D + (uint32_t)ns.size();
    ns.push_back(NewEnt{h, NIL, NIL, c, d});
    const uint32_t p = ep(x);                      // (the lookup made x primary-resident)
    PSlot& q = P(p);
    q.owner = y;
    ep(y) = p;
    ep(x) = NIL;
    const uint32_t di = ed(x);
    if (di != NIL) {                               // XCodecDisk::remove
      DSlot& r = Dk(di);
      r.olive = 0;
      r.owner = NIL;
      r.odp = NIL;
      --s_dlive;
      ed(x) = NIL;
    }
    q.opd = NIL;
    move_to(p, y);
    left(x, t + 1);                                // (x served this op's own lookup at t)
    bmap.put(h, y);
    d_append(y, t);
  }

  void begin_pass(uint32_t n, uint64_t decls) {
    epoch = ++disk->epoch;
    if (epoch == 0) {                              // (2^32 passes: re-tag everything)
      for (XcgPairState* f : disk->fronts) {
        if (!f) continue;
        for (PSlot& q : f->ps) q.ep = 0;
        for (Ent& e : f->es) e.ep = 0;
      }
      for (DSlot& q : ds()) q.ep = 0;
      epoch = disk->epoch = 1;
    }
    touchedP.clear();
    touchedD.clear();
    touchedE.clear();
    ns.clear();
    bmap.reset(decls);
    writes.clear();
    writes.reserve((size_t)decls * 2);
    ns.reserve((size_t)decls);
    nstaged = 0;
    enters = refs = appends = 0;
    split = false;
    bad.assign(n, 0);
    blo.assign(n, ~0u);
    bhi.assign(n, 0u);
    s_head = head; s_tail = tail; s_pcount = pcount; s_ftop = ftop; s_dclock = disk->dclock; s_dlive = dlive;
  }

  // One replay pass over chunks [0, n) of the sub-batch: rows ev[c * maxe ..],
  // nev[c].  Returns false if the pass is not the sequential one (bad[] and
  // split tell why).
  bool replay(uint32_t n, const uint4* ev, const uint32_t* nev, uint32_t maxe, uint32_t maxd) {
    begin_pass(n, (uint64_t)n * maxd);
    std::vector<uint32_t> order;
    bool ok = true;
    for (uint32_t c = 0; c < n && !split; ++c) {
      const uint32_t cnt = nev[c];
      if (cnt > maxe) { split = true; break; }     // (reference list overflow: a smaller sub-batch)
      const uint4* r = ev + (uint64_t)c * maxe;
      // rows are in stream order; a stable sort by time guards it
      bool sorted = true;
      for (uint32_t k = 1; k < cnt; ++k) sorted &= r[k - 1].z <= r[k].z;
      if (!sorted) {
        order.resize(cnt);
        for (uint32_t k = 0; k < cnt; ++k) order[k] = k;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return r[a].z < r[b].z; });
      }
      for (uint32_t k = 0; k < cnt && !split; ++k) {
        if (k + 8 < cnt) {                         // memory-level parallelism: touch ahead
          const uint4 f = r[sorted ? k + 8 : order[k + 8]];
          const uint32_t fk = f.w >> 30, fr = f.w & EV_REF_MASK;
          if (fk == EV_GHIT || fk == EV_GMISS) {
            if (fr < C + D) {
              __builtin_prefetch(&es[fr]);
              if (fr < C) __builtin_prefetch(&ps[fr]);
              else __builtin_prefetch(&ds()[fr - C]);
            }
          } else {
            bmap.prefetch(((uint64_t)f.y << 32) | f.x);
          }
        }
        const uint4 e = r[sorted ? k : order[k]];
        const uint32_t kind = e.w >> 30, ref = e.w & EV_REF_MASK;
        const uint64_t t = ((uint64_t)c << 21) | e.z;
        const uint64_t h = ((uint64_t)e.y << 32) | e.x;
        if (kind == EV_GHIT || kind == EV_GMISS) {
          if (ref >= C + D) { mark_bad(c, e.z); ok = false; continue; }
          const bool pr = present(ref);
          if (pr != (kind == EV_GHIT)) {
            mark_bad(c, e.z);
            ok = false;
            if (pair_debug()) bad_row(kind, ref, h, t);
          }
          if (pr) lookup(ref, t);
        } else if (kind == EV_HIT) {
          const uint32_t x = bmap.find(h);
          if (x == NIL) { mark_bad(c, e.z); ok = false; continue; }
          if (!present(x)) { split = true; break; }   // made here, gone already
          lookup(x, t);
        } else {                                   // EV_ENTER: encode_declaration's enter (:284-286)
          const uint32_t x0 = bmap.find(h);
          if (x0 != NIL && present(x0)) {
            mark_bad(c, e.z);
            ok = false;
            if (pair_debug()) bad_row(kind, x0, h, t);
            continue;
          }
          const uint32_t x = C + D + (uint32_t)ns.size();
          ns.push_back(NewEnt{h, NIL, NIL, c, ref});
          bmap.put(h, x);
          p_enter(x, t);
          d_append(x, t);
        }
      }
    }
    return ok && !split;
  }

  // One replay pass over a decode batch's classified ops (dec_classify_kernel
  // in pair mode): chunk c's rows are rows[base[c] .. base[c] + cnt[c]) in op
  // order, (lo, hi, op offset | REPLACE << 31, kind << 30 | ref).  ENTER (ref =
  // declaration row) = an EXTRACT whose hash no level holds: enter both
  // levels; HIT = a lookup of a hash an earlier EXTRACT of the batch named;
  // GHIT (ref = id) = a lookup of a cached hash, REPLACE when an EXTRACT's
  // bytes differ; GMISS = no cache effect.  A decode's references are fixed by
  // the stream except for presence, which this pass computes (ptime); the
  // caller classifies again under it until nothing changes.  Returns false
  // when a lookup would find a hash the batch entered already gone from both
  // levels (the stream then blocks or re-enters there: not modelled -- split).
  bool replay_decode(uint32_t n, const uint4* rows, const uint64_t* base, const uint64_t* cnt, uint64_t decls) {
    begin_pass(n, decls);
    for (uint32_t c = 0; c < n; ++c) {
      const uint4* r = rows + base[c];
      const uint32_t m = (uint32_t)cnt[c];
      uint32_t d_next = 0;                         // declaration rows in op order: ENTERs and REPLACEs
      for (uint32_t k = 0; k < m; ++k) {
        const uint4 e = r[k];
        const uint32_t kind = e.w >> 30, ref = e.w & EV_REF_MASK;
        const bool rep = (e.z >> 31) != 0;
        const uint64_t t = ((uint64_t)c << 21) | (e.z & 0x7FFFFFFFu);
        const uint64_t h = ((uint64_t)e.y << 32) | e.x;
        if (kind == EV_ENTER) {
          const uint32_t x = C + D + (uint32_t)ns.size();
          ns.push_back(NewEnt{h, NIL, NIL, c, ref});
          d_next = ref + 1;
          bmap.put(h, x);
          p_enter(x, t);
          d_append(x, t);
        } else if (kind == EV_HIT) {
          const uint32_t x = bmap.find(h);
          if (x == NIL || !present(x)) { split = true; return false; }
          lookup(x, t);
        } else if (kind == EV_GHIT) {
          if (ref >= C + D) { split = true; return false; }
          if (bmap.find(h) == NIL) bmap.put(h, ref);
          if (!present(ref)) continue;             // (classified under an older ptime: the next pass sees it)
          lookup(ref, t);
          if (rep) replace(ref, h, c, d_next++, t);
        }
      }
    }
    return true;
  }

  // Keep the pass: its copies -> committed; another front's entries the pass
  // invalidated leave that front.
  void keep() {
    for (uint32_t s : touchedP) {
      PSlot& q = ps[s];
      q.key = q.okey; q.prev = q.oprev; q.next = q.onext; q.pd = q.opd;
    }
    for (uint32_t i : touchedD) {
      DSlot& q = ds()[i];
      // another front's index entry went: invalidated, and maybe rewritten with
      // one of this front's entries since (only this front writes in its pass)
      if (q.live && q.xuid != xuid && (!q.olive || q.oxuid != q.xuid)) {
        XcgPairState* f = q.xuid < disk->fronts.size() ? disk->fronts[q.xuid] : nullptr;
        if (f) {
          --f->dlive;
          if (q.dp != NIL) f->ps[q.dp].pd = NIL;   // in its primary only now
          else f->pending.push_back((uint64_t)f->C + i);
        }
      }
      q.key = q.okey; q.live = q.olive; q.dp = q.odp; q.xuid = q.oxuid;
    }
    head = s_head; tail = s_tail; pcount = s_pcount; ftop = s_ftop; disk->dclock = s_dclock; dlive = s_dlive;
  }
};

namespace {

unsigned grid_for(uint64_t threads) { return (unsigned)((threads + 255) / 256); }

int ensure_dev(uint8_t** p, uint64_t* cap, uint64_t want) {
  if (*cap >= want) return 0;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, want) != hipSuccess) return -5;
  *cap = want;
  return 0;
}
int ensure_pinned(uint8_t** p, uint64_t* cap, uint64_t want) {
  if (*cap >= want) return 0;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipHostMalloc(p, want) != hipSuccess) return -5;
  *cap = want;
  return 0;
}

// Upload `bytes` from the pinned transfer area to the device one (offset o).
int upload(XcgPairState* P, uint64_t o, uint64_t bytes, hipStream_t st) {
  if (!bytes) return 0;
  return hipMemcpyAsync(P->d_xfer + o, P->h_xfer + o, bytes, hipMemcpyHostToDevice, st) == hipSuccess ? 0 : -5;
}

// ptime for the next parse: NEVER everywhere, then the replay's departures.
int upload_ptime(XcgPairState* P, hipStream_t st) {
  const uint32_t ids = P->ids();
  hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, P->d_ptime, (uint64_t)ids, NEVER);
  uint64_t* kv = (uint64_t*)P->h_xfer;
  uint32_t m = 0;
  for (uint32_t x : P->touchedE)
    if (P->es[x].leave != NEVER) {
      kv[2 * m] = x;
      kv[2 * m + 1] = P->es[x].leave;
      ++m;
    }
  if (m) {
    if (upload(P, 0, 16ull * m, st)) return -5;
    hipLaunchKernelGGL(pair_scatter64_kernel, dim3(grid_for(m)), dim3(256), 0, st, P->d_ptime,
                       (const uint64_t*)P->d_xfer, m);
  }
  // (the pinned area is reused by the next upload only after a stream sync)
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -5;
}

// The reference rows of a sub-batch, to the host.
int download_refs(XcgPairState* P, const XcgStreamArgs& a, hipStream_t st) {
  const uint64_t rows = (uint64_t)a.n * a.maxe;
  if (P->h_ev_cap < rows) {
    if (P->h_ev) (void)hipHostFree(P->h_ev);
    P->h_ev = nullptr;
    P->h_ev_cap = 0;
    if (hipHostMalloc(&P->h_ev, 16 * rows) != hipSuccess) return -5;
    P->h_ev_cap = rows;
  }
  if (P->h_nev_cap < a.n) {
    if (P->h_nev) (void)hipHostFree(P->h_nev);
    if (P->h_need) (void)hipHostFree(P->h_need);
    P->h_nev = P->h_need = nullptr;
    P->h_nev_cap = 0;
    if (hipHostMalloc(&P->h_nev, 4ull * a.n) != hipSuccess || hipHostMalloc(&P->h_need, 12ull * a.n) != hipSuccess)
      return -5;
    P->h_nev_cap = a.n;
  }
  if (hipMemcpyAsync(P->h_nev, a.nev, 4ull * a.n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(P->h_ev, a.ev, 16 * rows, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return -5;
  return 0;
}

// XCodecHash::hash of one segment (xcodec/xcodec_hash.h:166-174), host side,
// for the XCG_PAIR_VERIFY diagnostics.
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

// Diagnostics (XCG_PAIR_VERIFY): every primary slot and live disk block holds
// bytes of its hash, and G finds every level entry.
void pair_verify(XcgPairState* P, const uint8_t* d_pool, hipStream_t st) {
  const uint64_t ids = P->ids();
  std::vector<uint8_t> pool(ids * SEG);
  std::vector<uint64_t> keyg(ids);
  (void)hipStreamSynchronize(st);
  (void)hipMemcpy(pool.data(), d_pool, ids * SEG, hipMemcpyDeviceToHost);
  (void)hipMemcpy(keyg.data(), P->d_keyg, 8 * ids, hipMemcpyDeviceToHost);
  uint32_t bad = 0;
  for (uint32_t s = 0; s < P->C; ++s) {
    const PSlot& q = P->ps[s];
    if (q.key == NOKEY) continue;
    if (host_hash(&pool[(uint64_t)s * SEG]) != q.key && bad++ < 5)
      fprintf(stderr, "pair verify: primary slot %u bytes do not hash to its key\n", s);
    if (keyg[s] != q.key && bad++ < 5) fprintf(stderr, "pair verify: keyg[%u] stale\n", s);
    if (q.pd != NIL && (P->ds()[q.pd].key != q.key || !P->ds()[q.pd].live || P->ds()[q.pd].xuid != P->xuid) &&
        bad++ < 5)
      fprintf(stderr, "pair verify: slot %u links disk block %u of another hash\n", s, q.pd);
  }
  uint64_t mine = 0;
  for (uint32_t i = 0; i < P->D; ++i) {
    const DSlot& q = P->ds()[i];
    const bool own = q.live && q.xuid == P->xuid;
    mine += own;
    const uint64_t want = own && q.dp == NIL ? q.key : NOKEY;
    if (keyg[P->C + i] != want && bad++ < 5) fprintf(stderr, "pair verify: keyg[C+%u] stale\n", i);
    if (!own) continue;
    if (host_hash(&pool[((uint64_t)P->C + i) * SEG]) != q.key && bad++ < 5)
      fprintf(stderr, "pair verify: disk block %u bytes do not hash to its key\n", i);
    if (q.dp != NIL && P->ps[q.dp].key != q.key && bad++ < 5)
      fprintf(stderr, "pair verify: disk block %u links slot %u of another hash\n", i, q.dp);
  }
  if (mine != P->dlive && bad++ < 5) fprintf(stderr, "pair verify: %llu own disk entries, count says %llu\n",
                                             (unsigned long long)mine, (unsigned long long)P->dlive);
  fprintf(stderr, "pair verify: %u problems (primary %u, disk live %llu)\n", bad, P->pcount,
          (unsigned long long)P->dlive);
}

// G from scratch: wipe, then every id whose keyg holds a hash.
void pair_rebuild(XcgPairState* P, const PairGpu& G, hipStream_t st) {
  const HashTab g{G.g_keys, G.g_vals, G.g_mask};
  const FiltSet fs{G.g_filt, G.g_ftab, G.fmask, G.g_gfilt, G.gmask};
  PairWipe wp{g, G.g_filt, (u32x4*)G.g_ftab, G.fmask + 1, G.g_gfilt, G.gmask + 1, G.nseg};
  hipLaunchKernelGGL(pair_wipe_kernel, dim3(1024), dim3(256), 0, st, wp);
  const uint32_t ids = P->ids();
  hipLaunchKernelGGL(pair_rebuild_kernel, dim3(grid_for(ids)), dim3(256), 0, st, (const uint64_t*)P->d_keyg, ids,
                     g, fs, G.nseg, G.status);
}

// Commit a kept pass on the GPU: bytes, per-id keys, G and its filters.
int pair_commit(XcgPairState* P, const PairGpu& G, hipStream_t st) {
  // A primary slot can change hands more than once in a sub-batch (an entry
  // evicted to disk frees it again), and a small disk can lap within one:
  // only the last move into each destination stays.  (Sources are the input or
  // pre-sub-batch bytes, staged before any move.)
  {
    std::vector<uint4>& w = P->writes;
    std::vector<uint8_t> seen(P->ids(), 0);
    size_t k = w.size();
    for (size_t j = w.size(); j-- > 0;) {
      if (seen[w[j].x]) continue;
      seen[w[j].x] = 1;
      w[--k] = w[j];
    }
    w.erase(w.begin(), w.begin() + (ptrdiff_t)k);
  }
  const uint32_t nw = (uint32_t)P->writes.size();
  // per-id key updates for every slot the pass touched (a disk block counts
  // for this front only while its live index entry is this front's)
  std::vector<uint64_t> kv;
  kv.reserve(2 * (P->touchedP.size() + P->touchedD.size() + P->pending.size()));
  for (uint32_t s : P->touchedP) {
    kv.push_back(s);
    kv.push_back(P->ps[s].key);
  }
  for (uint32_t i : P->touchedD) {
    const DSlot& q = P->ds()[i];
    kv.push_back((uint64_t)P->C + i);
    kv.push_back(q.live && q.xuid == P->xuid && q.dp == NIL ? q.key : NOKEY);
  }
  const uint32_t nk = (uint32_t)(kv.size() / 2);
  const uint64_t wbytes = 16ull * nw, kbytes = 8ull * kv.size();
  if (ensure_pinned(&P->h_xfer, &P->h_xfer_cap, wbytes + kbytes + 16) ||
      ensure_dev(&P->d_xfer, &P->xfer_cap, wbytes + kbytes + 16) ||
      ensure_dev(&P->d_staging, &P->staging_cap, (uint64_t)(P->nstaged ? P->nstaged : 1) * SEG))
    return -5;
  memcpy(P->h_xfer, P->writes.data(), wbytes);
  memcpy(P->h_xfer + wbytes, kv.data(), kbytes);
  if (upload(P, 0, wbytes + kbytes, st)) return -5;
  const uint4* w = (const uint4*)P->d_xfer;
  if (nw) {
    hipLaunchKernelGGL(pair_stage_kernel, dim3((nw + 3) / 4), dim3(256), 0, st, w, nw, (const uint8_t*)G.pool,
                       P->d_staging);
    hipLaunchKernelGGL(pair_move_kernel, dim3((nw + 3) / 4), dim3(256), 0, st, w, nw, G.in, G.chunk_off,
                       (const uint4*)G.decl, G.maxd, (const uint8_t*)P->d_staging, G.pool);
  }
  if (nk)
    hipLaunchKernelGGL(pair_scatter64_kernel, dim3(grid_for(nk)), dim3(256), 0, st, P->d_keyg,
                       (const uint64_t*)(P->d_xfer + wbytes), nk);
  pair_rebuild(P, G, st);
  // (the pinned transfer area is free again once the stream passes here)
  return hipStreamSynchronize(st) == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -5;
}

// Index entries another front's kept pass took from this one (the shared
// ring's invalidations): clear their ids and rebuild G before this front's
// next batch looks anything up.
int pair_sync_pending(XcgPairState* P, const PairGpu& G, hipStream_t st) {
  if (P->pending.empty()) return 0;
  const uint32_t m = (uint32_t)P->pending.size();
  std::vector<uint64_t> kv(2ull * m);
  for (uint32_t j = 0; j < m; ++j) {
    kv[2 * j] = P->pending[j];
    kv[2 * j + 1] = NOKEY;
  }
  P->pending.clear();
  if (ensure_pinned(&P->h_xfer, &P->h_xfer_cap, 16ull * m) || ensure_dev(&P->d_xfer, &P->xfer_cap, 16ull * m))
    return -5;
  memcpy(P->h_xfer, kv.data(), 16ull * m);
  if (upload(P, 0, 16ull * m, st)) return -5;
  hipLaunchKernelGGL(pair_scatter64_kernel, dim3(grid_for(m)), dim3(256), 0, st, P->d_keyg,
                     (const uint64_t*)P->d_xfer, m);
  pair_rebuild(P, G, st);
  return hipStreamSynchronize(st) == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -5;
}

PairGpu gpu_of(const XcgStreamArgs& a) {
  return PairGpu{a.in, a.chunk_off, a.decl, a.maxd, a.pool, a.g_keys, a.g_vals, a.g_mask,
                 a.g_filt, a.g_ftab, a.fmask, a.g_gfilt, a.gmask, a.nseg, a.status};
}

}  // namespace

extern "C" {

int xcg_disk_state_create(uint64_t disk_bytes, XcgDiskState** out) {
  const uint64_t blocks = disk_bytes / SEG;
  if (blocks <= 18) return -22;
  const uint64_t nb = (blocks - 18) / (1 + DISK_ENTRIES);   // xcodec_cache_disk.cc:110-111
  if (nb == 0 || nb * DISK_ENTRIES >= (1ull << 29)) return -22;
  XcgDiskState* K = new XcgDiskState;
  K->nb = nb;
  K->D = (uint32_t)(nb * DISK_ENTRIES);
  K->ds.assign(K->D, DSlot{NOKEY, NOKEY, NIL, NIL, NIL, 0, 0, 0, 0, 0});
  *out = K;
  return 0;
}

void xcg_disk_state_release(XcgDiskState* K) {
  if (K && --K->refs == 0) delete K;
}

void xcg_disk_state_stats(const XcgDiskState* K, uint64_t* st) {
  uint64_t live = 0, fronts = 0;
  for (const DSlot& q : K->ds) live += q.live;
  for (const XcgPairState* f : K->fronts) fronts += f != nullptr;
  st[0] = live;
  st[1] = K->dclock;
  st[2] = K->nb;
  st[3] = fronts;
}

// A pair front on disk K (XCodecDisk::local for the first, ::connect for the
// others: the lowest free xuid, xcodec_cache_disk.cc:640-690).
int xcg_pair_state_create(uint32_t C, XcgDiskState* K, XcgPairState** out) {
  if (C == 0 || !K || (uint64_t)K->D + C >= (1ull << 30)) return -22;
  uint32_t xuid = 0;
  while (xuid < K->fronts.size() && K->fronts[xuid]) ++xuid;
  if (xuid >= 1024) return -22;                             // XCDFS_XUID_COUNT
  XcgPairState* P = new XcgPairState;
  P->C = C;
  P->nb = K->nb;
  P->D = K->D;
  P->disk = K;
  P->dsp = &K->ds;
  P->xuid = (uint16_t)xuid;
  const uint32_t D = P->D, ids = C + D;
  P->ps.assign(C, PSlot{NOKEY, NOKEY, NIL, NIL, NIL, NIL, NIL, NIL, NIL, 0});
  P->es.assign(ids, Ent{NEVER, 0, NIL, NIL, 0});
  P->pfree.resize(C);
  for (uint32_t s = 0; s < C; ++s) P->pfree[s] = C - 1 - s;   // slot 0 first
  P->ftop = C;
  if (hipMalloc(&P->d_keyg, 8ull * ids) != hipSuccess || hipMalloc(&P->d_ptime, 8ull * ids) != hipSuccess ||
      hipMemset(P->d_keyg, 0xFF, 8ull * ids) != hipSuccess || hipMemset(P->d_ptime, 0xFF, 8ull * ids) != hipSuccess) {
    (void)hipFree(P->d_keyg);
    (void)hipFree(P->d_ptime);
    delete P;
    return -12;
  }
  if (xuid >= K->fronts.size()) K->fronts.resize(xuid + 1, nullptr);
  K->fronts[xuid] = P;
  ++K->refs;
  *out = P;
  return 0;
}

// A front goes away (its XCodecCache is deleted): its entries stay in the
// ring as entries of no live front (index_invalidate_entries skips an xuid
// with no cache, xcodec_cache_disk.cc:360-364).
void xcg_pair_state_destroy(XcgPairState* P) {
  if (!P) return;
  (void)hipFree(P->d_keyg); (void)hipFree(P->d_ptime); (void)hipFree(P->d_staging); (void)hipFree(P->d_xfer);
  if (P->h_xfer) (void)hipHostFree(P->h_xfer);
  if (P->h_ev) (void)hipHostFree(P->h_ev);
  if (P->h_nev) (void)hipHostFree(P->h_nev);
  if (P->h_need) (void)hipHostFree(P->h_need);
  if (P->h_base) (void)hipHostFree(P->h_base);
  XcgDiskState* K = P->disk;
  if (K) {
    for (DSlot& q : K->ds)
      if (q.live && q.xuid == P->xuid) q.live = 0;
    K->fronts[P->xuid] = nullptr;
    xcg_disk_state_release(K);
  }
  delete P;
}

// Drop everything this front holds (XCodecCache objects have no clear: this is
// a fresh front; on a disk of its own, a fresh volume).  The caller wipes G.
int xcg_pair_state_clear(XcgPairState* P) {
  XcgDiskState* K = P->disk;
  P->ps.assign(P->C, PSlot{NOKEY, NOKEY, NIL, NIL, NIL, NIL, NIL, NIL, NIL, 0});
  uint64_t others = 0;
  for (const XcgPairState* f : K->fronts) others += f && f != P;
  for (DSlot& q : K->ds) {
    if (q.live && q.xuid == P->xuid) q.live = 0;
    q.dp = q.xuid == P->xuid ? NIL : q.dp;
  }
  if (others == 0) {
    K->ds.assign(K->D, DSlot{NOKEY, NOKEY, NIL, NIL, NIL, 0, 0, 0, 0, 0});
    K->dclock = 0;
  }
  for (Ent& e : P->es) e.ep = 0;
  for (uint32_t s = 0; s < P->C; ++s) P->pfree[s] = P->C - 1 - s;
  P->ftop = P->C;
  P->head = P->tail = NIL;
  P->pcount = 0;
  P->dlive = 0;
  P->pending.clear();
  return hipMemset(P->d_keyg, 0xFF, 8ull * P->ids()) == hipSuccess ? 0 : -5;
}

void xcg_pair_state_stats(const XcgPairState* P, uint64_t* st) {
  st[0] = P->pcount;
  st[1] = P->dlive;
  st[2] = P->disk->dclock;
  st[3] = P->nb;
}

uint32_t xcg_pair_state_last_base(const XcgPairState* P) { return P->last_base; }
uint32_t xcg_pair_state_limit(const XcgPairState* P) { return P->C; }
uint32_t xcg_pair_state_disk_blocks(const XcgPairState* P) { return P->D; }
const uint64_t* xcg_pair_state_ptime(const XcgPairState* P) { return P->d_ptime; }

int xcg_pair_sync(XcgPairState* P, const PairGpu* G, hipStream_t st) { return pair_sync_pending(P, *G, st); }

// Decode on the pair, first step: ptime NEVER everywhere.
int xcg_pair_decode_begin(XcgPairState* P, hipStream_t st) {
  P->leaves.clear();
  hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, P->d_ptime, (uint64_t)P->ids(), NEVER);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// One replay of a decode batch's classified ops (rows packed per chunk at
// d_base[c], d_cnt[c] of them; `rows` total).  *same = the departure times it
// computes equal those the classification used (then it was the sequential
// decoder's).  Otherwise ptime is updated for the next classification.
// Returns 0, -95 (a hash this batch entered is gone before a later lookup),
// -5.
int xcg_pair_decode_pass(XcgPairState* P, const void* d_rows, const uint64_t* d_base, const uint64_t* d_cnt,
                         uint32_t n, uint64_t rows, uint64_t decls, int* same, hipStream_t st) {
  if (P->h_ev_cap < rows + 1) {
    if (P->h_ev) (void)hipHostFree(P->h_ev);
    P->h_ev = nullptr;
    P->h_ev_cap = 0;
    if (hipHostMalloc(&P->h_ev, 16 * (rows + 1)) != hipSuccess) return -5;
    P->h_ev_cap = rows + 1;
  }
  if (P->h_base_cap < n) {
    if (P->h_base) (void)hipHostFree(P->h_base);
    P->h_base = nullptr;
    P->h_base_cap = 0;
    if (hipHostMalloc(&P->h_base, 16ull * n) != hipSuccess) return -5;
    P->h_base_cap = n;
  }
  if ((rows && hipMemcpyAsync(P->h_ev, d_rows, 16 * rows, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      hipMemcpyAsync(P->h_base, d_base, 8ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(P->h_base + n, d_cnt, 8ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return -5;
  if (!P->replay_decode(n, P->h_ev, P->h_base, P->h_base + n, decls)) return -95;
  std::vector<uint64_t> lv;
  for (uint32_t x : P->touchedE)
    if (P->es[x].leave != NEVER) {
      lv.push_back(x);
      lv.push_back(P->es[x].leave);
    }
  {
    std::vector<std::pair<uint64_t, uint64_t>> pr(lv.size() / 2);
    for (size_t j = 0; j < pr.size(); ++j) pr[j] = {lv[2 * j], lv[2 * j + 1]};
    std::sort(pr.begin(), pr.end());
    for (size_t j = 0; j < pr.size(); ++j) {
      lv[2 * j] = pr[j].first;
      lv[2 * j + 1] = pr[j].second;
    }
  }
  *same = lv == P->leaves;
  if (*same) return 0;
  P->leaves = lv;
  hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, P->d_ptime, (uint64_t)P->ids(), NEVER);
  const uint32_t m = (uint32_t)(lv.size() / 2);
  if (m) {
    if (ensure_pinned(&P->h_xfer, &P->h_xfer_cap, 16ull * m) || ensure_dev(&P->d_xfer, &P->xfer_cap, 16ull * m))
      return -5;
    memcpy(P->h_xfer, lv.data(), 16ull * m);
    if (upload(P, 0, 16ull * m, st)) return -5;
    hipLaunchKernelGGL(pair_scatter64_kernel, dim3(grid_for(m)), dim3(256), 0, st, P->d_ptime,
                       (const uint64_t*)P->d_xfer, m);
  }
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -5;
}

// Keep the last decode replay and commit it (bytes from the batch input at the
// declaration rows: G.decl[c * maxd + d].z = the EXTRACT payload's offset).
int xcg_pair_decode_commit(XcgPairState* P, const PairGpu* G, hipStream_t st) {
  P->keep();
  const int rc = pair_commit(P, *G, st);
  if (getenv("XCG_PAIR_VERIFY")) pair_verify(P, G->pool, st);
  P->leaves.clear();
  hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, P->d_ptime, (uint64_t)P->ids(), NEVER);
  return rc;
}

// Stream-semantics encode of a batch on the pair, in sub-batches (see the top
// of this file).  Returns 0, -75 (no consistent pass / overflow), -95 (one
// chunk alone exceeds what a sub-batch may hold), -5.
int xcg_pair_encode_stream(const XcgStreamArgs* a0, XcgPairState* P, int* rounds_out, hipStream_t st) {
  const uint32_t n = a0->n;
  int rounds = 0;
  if (pair_sync_pending(P, gpu_of(*a0), st)) return -5;
  // A sub-batch is bounded by the disk only: while it writes fewer than a lap
  // of disk blocks, nothing it declared can leave both levels within it (a
  // chunk writes at most maxd declarations plus its touches).
  const uint64_t lap = P->D > 2 * DISK_ENTRIES ? P->D - 2 * DISK_ENTRIES : 1;
  uint32_t per = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, lap / a0->maxd));
  constexpr int MAX_PASSES = 12;
  uint32_t i0 = 0;
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  while (i0 < n) {
    const clk::time_point t0 = clk::now();
    const uint32_t m = per < n - i0 ? per : n - i0;
    XcgStreamArgs a = *a0;
    a.n = m;
    a.chunk_off += i0;
    a.chunk_len += i0;
    a.out_off += i0;
    a.out_len += i0;
    if (a.stats) a.stats += 4ull * i0;
    a.ptime = P->d_ptime;
    a.no_commit = 1;
    // The rounds start from each chunk's tiling (its cold parse).  ptime is
    // NEVER (no cached entry leaves) unless the last sub-batch needed more than
    // one pass: then the first guess is the tiling seed's own references,
    // replayed (a cached tile is a lookup hit, a repeat of an earlier tile a hit
    // on its declaration, every other tile a declaration).
    if (xcg_launch_seed_tiling(&a, st)) return -5;
    const clk::time_point t1 = clk::now();
    if (P->prev_passes > 1) {
      const HashTab g{a.g_keys, a.g_vals, a.g_mask}, b{a.b_keys, a.b_vals, a.b_mask};
      hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, b.keys, (uint64_t)b.mask + 1, NOKEY);
      hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, b.vals, (uint64_t)b.mask + 1, ~0ull);
      hipLaunchKernelGGL(pair_seed_table_kernel, dim3(grid_for((uint64_t)m * a.maxd)), dim3(256), 0, st, m,
                         (const uint4*)a.decl, (const uint32_t*)a.ndecl, a.maxd, b, a.status);
      hipLaunchKernelGGL(pair_seed_events_kernel, dim3((m + 3) / 4), dim3(256), 0, st, m, (const uint4*)a.decl,
                         (const uint32_t*)a.ndecl, a.maxd, a.chunk_len, g, b, (uint4*)a.ev, a.nev, a.maxe);
      if (download_refs(P, a, st)) return -5;
      (void)P->replay(m, P->h_ev, P->h_nev, a.maxe, a.maxd);
      if (ensure_pinned(&P->h_xfer, &P->h_xfer_cap, 16ull * (P->touchedE.size() + 1)) ||
          ensure_dev(&P->d_xfer, &P->xfer_cap, 16ull * (P->touchedE.size() + 1)) || upload_ptime(P, st))
        return -5;
    }
    const clk::time_point t2 = clk::now();
    double t_parse = 0, t_dl = 0, t_replay = 0;
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
      if (rc) return rc;
      if (pair_debug()) (void)hipStreamSynchronize(st);
      const clk::time_point q1 = clk::now();
      if (download_refs(P, a, st)) return -5;
      const clk::time_point q2 = clk::now();
      const bool ok = P->replay(m, P->h_ev, P->h_nev, a.maxe, a.maxd);
      const clk::time_point q3 = clk::now();
      t_parse += ms(q0, q1);
      t_dl += ms(q1, q2);
      t_replay += ms(q2, q3);
      uint32_t nbad = 0;
      for (uint32_t c = 0; c < m; ++c) nbad += P->bad[c];
      if (pair_debug())
        fprintf(stderr, "pair: chunks %u+%u pass %d rounds %d enters %llu refs %llu appends %llu bad %u split %d\n",
                i0, m, pass, r, (unsigned long long)P->enters, (unsigned long long)P->refs,
                (unsigned long long)P->appends, nbad, (int)P->split);
      if (P->split) split = true;
      else if (ok) done = true;
      else {
        for (uint32_t c = 0; c < m; ++c) {
          P->h_need[c] = P->bad[c];
          P->h_need[m + c] = P->blo[c];
          P->h_need[2 * m + c] = P->bhi[c];
        }
        if (hipMemcpyAsync(a.need, P->h_need, 4ull * m, hipMemcpyHostToDevice, st) != hipSuccess) return -5;
        if (a.bad_t && (hipMemcpyAsync(a.bad_t, P->h_need + m, 4ull * m, hipMemcpyHostToDevice, st) != hipSuccess ||
                        hipMemcpyAsync(a.bad_hi, P->h_need + 2 * m, 4ull * m, hipMemcpyHostToDevice, st) != hipSuccess))
          return -5;
        if (ensure_pinned(&P->h_xfer, &P->h_xfer_cap, 16ull * (P->touchedE.size() + 1)) ||
            ensure_dev(&P->d_xfer, &P->xfer_cap, 16ull * (P->touchedE.size() + 1)) || upload_ptime(P, st))
          return -5;
      }
    }
    if (!done) {
      if (m == 1) return split ? -95 : -75;
      per = m / 2;                                 // redo this part in halves
      P->prev_passes = MAX_PASSES;
      continue;
    }
    const clk::time_point t3 = clk::now();
    P->keep();
    if (pair_commit(P, gpu_of(a), st)) return -5;
    if (pair_debug())
      fprintf(stderr, "pair: ms seed %.2f seed-replay %.2f parse %.2f download %.2f replay %.2f commit %.2f\n",
              ms(t0, t1), ms(t1, t2), t_parse, t_dl, t_replay, ms(t3, clk::now()));
    if (getenv("XCG_PAIR_VERIFY")) pair_verify(P, a.pool, st);
    // the next sub-batch starts with every hash visible to its end
    hipLaunchKernelGGL(pair_fill64_kernel, dim3(1024), dim3(256), 0, st, P->d_ptime, (uint64_t)P->ids(), NEVER);
    P->last_base = i0;
    P->prev_passes = passes;
    i0 += m;
    // size the next sub-batch from the disk blocks this one wrote
    const uint64_t useD = P->appends;
    uint64_t want = (uint64_t)n;
    if (useD) want = std::min<uint64_t>(want, lap * 9 / 10 * m / useD);
    per = (uint32_t)(want < 1 ? 1 : (want > n ? n : want));
  }
  if (rounds_out) *rounds_out = rounds;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
