// Arguments of the stream-semantics encode driver (xcg_launch_encode_stream),
// shared by xcg_api.hip (the caller) and xcg_lru.hip (the bounded-cache pass).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct XcgStreamArgs {
  const uint8_t* in;
  const uint64_t* chunk_off;
  const uint32_t* chunk_len;
  uint32_t n;
  uint32_t flags;
  uint8_t* out;
  const uint64_t* out_off;
  uint64_t* out_len;
  uint32_t* stats;
  int32_t* status;
  // persistent cache
  uint64_t* g_keys;
  uint64_t* g_vals;
  uint32_t g_mask;
  uint8_t* pool;
  uint32_t* nseg;
  uint32_t seg_cap;
  uint32_t* g_filt;
  uint32_t* g_ftab;
  uint32_t fmask;
  // batch scratch
  uint64_t* b_keys;
  uint64_t* b_vals;
  uint32_t b_mask;
  uint32_t* r_filt;
  uint32_t* r_ftab;
  void* decl;             // uint4 rows
  uint32_t* ndecl;
  uint32_t maxd;
  uint32_t* changed;
  uint32_t* h_changed;   // pinned host word
  uint32_t* g_gfilt;     // global lane filters: the cache's and the round's copy
  uint32_t* r_gfilt;
  uint32_t gmask;
  uint32_t* bcount;      // [64]
  // verification: a second batch table (tables alternate between rounds), the
  // changed-hash table, per-chunk batch hits, flags
  uint64_t* b2_keys;
  uint64_t* b2_vals;
  uint64_t* r_keys;
  uint64_t* r_vals;
  uint32_t r_mask;
  uint64_t* hits;
  uint32_t* nhits;
  uint32_t maxh;
  uint32_t* need;
  uint32_t* vflags;      // [0] a_first, [1] any, [2] declarations in the last table built
  uint32_t* h_vflags;    // pinned
  int seed;              // start from the tiling seed instead of round 0
  uint32_t* decls_out;   // (host) declarations the batch made, ~0 if unknown
  // bounded (LRU) cache: eviction times per pool slot, the reference lists,
  // and whether the driver commits (the LRU pass commits itself)
  const uint64_t* ptime;
  void* ev;
  uint32_t* nev;
  uint32_t maxe;
  int no_commit;
  int keep_decls;        // start from the declaration lists already in decl/ndecl
  int need_given;        // (keep_decls) round 1 parses only the chunks flagged in need[]
  // re-parse restart (bounded / pair): output length after each REF-making
  // lookup, per chunk the earliest / latest contradicted lookup time, and the
  // backup of the previous pass's rows of the flagged chunks
  uint32_t* eo;          // [n * maxe]
  uint32_t* bad_t;       // [n] (~0: none)
  uint32_t* bad_hi;      // [n]
  int restart;           // (need_given) round 1 resumes flagged chunks from their rows
  uint32_t* bslot;       // [n]
  uint32_t* b_count;     // [1]
  uint32_t b_slots;
  void* b_ev;            // [b_slots * maxe] uint4
  uint32_t* b_eo;        // [b_slots * maxe]
  uint64_t* b_hits;      // [b_slots * maxh]
  uint32_t* b_cnt;       // [b_slots * 4]
  uint8_t* b_out;        // [b_slots * b_stride]
  uint64_t b_stride;
  void* splice;          // [n] uint4
  // verification (a), exactly (verify_probe_kernel): the hashes that became
  // visible to more chunks -> that chunk range, and their Bloom words
  uint64_t* a_keys;      // [XCG_VERIFY_A_CAP]
  uint64_t* a_vals;
  uint32_t* a_bits;      // [XCG_VERIFY_A_WORDS]
  // the context's event behind the verification flags' copy (hipEvent_t; null:
  // the driver makes one for the call)
  void* flags_ev;
  // the quiet-chunk screen (small chunks): the 128 KiB LDS fold of the round's
  // global lane filter, and the work list of chunks it sends to the parse
  // ([0] count, [1..n] chunks); null: no screen
  uint32_t* s_fold = nullptr;
  uint32_t* s_work = nullptr;
  uint32_t* s_info = nullptr;    // [n] the screen's verdict per chunk
  void* s_rows = nullptr;        // [n * 4] uint4: its staged rows
  uint32_t* s_qcnt = nullptr;    // [n] and [n * 1024]: the windows it queues for the probe
  uint32_t* s_qkeys = nullptr;
  // (bounded cache) called behind each Jacobi verification, before the host
  // reads its flags: queues work gated on vflags[1] == 0 (the round converged)
  int (*post_verify)(void* user, const uint32_t* vbusy, hipStream_t st) = nullptr;
  void* post_user = nullptr;
};

// (a)-probe sizes: at most A_LIMIT newly visible hashes per verification (more:
// the conservative flag), a table of twice that, a 32 KiB blocked Bloom filter.
constexpr uint32_t XCG_VERIFY_A_LIMIT = 8192, XCG_VERIFY_A_CAP = 16384, XCG_VERIFY_A_WORDS = 8192;

// Bounded cache (xcg_lru.hip): device LRU state of a context.
struct XcgLruState {
  uint32_t C;             // memory_cache_limit_ in segments (= pool slots)
  uint64_t* skey;         // [C] key of the entry in pool slot s
  uint64_t* lastref;      // [C] LRU time of its last enter / lookup
  uint32_t* queue;        // [C] live slots, least recently used first
  uint32_t* queue2;
  uint64_t* ptime;        // [C] batch time from which slot s is evicted (~0: never)
  uint64_t* hmin;
  uint64_t* wpop;
  uint64_t* tau;
  uint32_t* alive;
  uint32_t* freel;
  uint32_t* evslot;       // per reference of the batch (scratch)
  uint64_t* evtime;
  uint32_t* ev_base;      // [n + 1]
  uint32_t* enter_base;   // [n + 1]
  uint32_t* tot;          // [16]
  uint32_t* h_tot;        // pinned [16]
  uint64_t clock;         // LRU time base of the next batch (host)
  uint32_t* part;         // per-tile counts of the multi-workgroup scans (grown on demand)
  uint32_t part_cap;
  uint32_t last_base;     // first chunk of the last committed sub-batch (its rows stay in the scratch)
  uint32_t fit_hint;      // chunks x maxd a full-cache sub-batch held last (0: none yet)
  void* tev;              // hipEvent_t behind the eviction times' totals (lazily made)
};

// A batch's cache references for the LRU pass: enters as declaration rows
// decl[c * maxd + d] = (lo, hi, position, -), d < ndecl[c]; references as
// ev[row(c) + k], k < nev[c] (row = c * maxe, or packed when dense).
struct LruBatch {
  uint32_t n;
  const uint8_t* in;
  const uint64_t* chunk_off;
  const void* decl;
  const uint32_t* ndecl;
  uint32_t maxd;
  const void* ev;
  const uint32_t* nev;
  uint32_t maxe;
  int dense;
  uint32_t* need;         // (encoder) chunks with an inconsistent lookup; may be scratch
  uint64_t* g_keys;
  uint64_t* g_vals;
  uint32_t g_mask;
  uint8_t* pool;
  uint32_t* nseg;
  uint32_t* g_filt;
  uint32_t* g_ftab;
  uint32_t fmask;
  uint32_t* g_gfilt;
  uint32_t gmask;
  int32_t* status;
  uint64_t ev_bound;      // upper bound of the batch's references (sizes the scans)
  uint32_t* bad_t;        // (encoder, optional) per chunk earliest / latest contradicted lookup time
  uint32_t* bad_hi;
};

// XCodecCachePair of a bounded memory primary and a disk secondary (xcg_pair.hip).
// The disk (XcgDiskState) is shared by every pair front on it, as XCodecDisk is
// by its XCodecDiskCache front-ends.
struct XcgDiskState;
struct XcgPairState;
// What a pair commit / table rebuild touches on the GPU: the batch input and
// its declaration rows (bytes of new entries), the pool, G and its filters.
struct PairGpu {
  const uint8_t* in;
  const uint64_t* chunk_off;
  const void* decl;       // uint4 rows: decl[c * maxd + d].z = the segment's offset in chunk c
  uint32_t maxd;
  uint8_t* pool;
  uint64_t* g_keys;
  uint64_t* g_vals;
  uint32_t g_mask;
  uint32_t* g_filt;
  uint32_t* g_ftab;
  uint32_t fmask;
  uint32_t* g_gfilt;
  uint32_t gmask;
  uint32_t* nseg;
  int32_t* status;
};
extern "C" int xcg_disk_state_create(uint64_t disk_bytes, uint32_t flags, XcgDiskState** out);
extern "C" int xcg_disk_state_tier(const XcgDiskState* K);
extern "C" void xcg_disk_state_release(XcgDiskState* K);
extern "C" void xcg_disk_state_stats(const XcgDiskState* K, uint64_t* st);
extern "C" int xcg_pair_state_create(uint32_t C, XcgDiskState* K, const char* uuid36, int want_xuid,
                                     XcgPairState** out);
extern "C" int xcg_disk_state_save(XcgDiskState* K, const char* path);
extern "C" int xcg_disk_state_open(const char* path, uint64_t disk_bytes, uint32_t flags, XcgDiskState** out);
extern "C" int xcg_disk_state_open_fd(int fd, uint64_t disk_bytes, uint32_t flags, XcgDiskState** out);
extern "C" void xcg_disk_state_head(const XcgDiskState* K, uint64_t* index_block, uint64_t* next);
extern "C" uint32_t xcg_pair_state_xuid(const XcgPairState* P);
extern "C" void xcg_pair_state_set_unbounded(XcgPairState* P);
extern "C" int xcg_pair_state_unbounded(const XcgPairState* P);
extern "C" void xcg_pair_state_destroy(XcgPairState* P);
extern "C" int xcg_pair_state_clear(XcgPairState* P);
extern "C" void xcg_pair_state_stats(const XcgPairState* P, uint64_t* st);
extern "C" uint32_t xcg_pair_state_last_base(const XcgPairState* P);
extern "C" uint32_t xcg_pair_state_limit(const XcgPairState* P);
extern "C" uint32_t xcg_pair_state_disk_blocks(const XcgPairState* P);
extern "C" XcgDiskState* xcg_pair_state_disk(const XcgPairState* P);
extern "C" const uint64_t* xcg_pair_state_ptime(const XcgPairState* P);
extern "C" int xcg_pair_sync(XcgPairState* P, const PairGpu* G, hipStream_t st);
extern "C" int xcg_pair_encode_stream(const XcgStreamArgs* a, XcgPairState* P, int* rounds_out, hipStream_t st);
extern "C" int xcg_pair_decode_begin(XcgPairState* P, hipStream_t st);
extern "C" int xcg_pair_decode_pass(XcgPairState* P, const PairGpu* G, const void* d_rows, const uint64_t* d_base,
                                    const uint64_t* d_cnt, uint32_t n, uint64_t rows, uint32_t maxd, int* same,
                                    hipStream_t st);
extern "C" uint8_t* xcg_pair_state_pool(const XcgPairState* P);
extern "C" int xcg_pair_decode_commit(XcgPairState* P, const PairGpu* G, hipStream_t st);

extern "C" int xcg_launch_encode_stream(const XcgStreamArgs* a, int* rounds_out, hipStream_t stream);
extern "C" int xcg_lru_encode_stream(const XcgStreamArgs* a, XcgLruState* L, int* rounds_out, hipStream_t st);
extern "C" int xcg_lru_times(const LruBatch* b, XcgLruState* L, hipStream_t st);
extern "C" int xcg_lru_commit(const LruBatch* b, XcgLruState* L, hipStream_t st);
extern "C" int xcg_lru_reset_times(XcgLruState* L, hipStream_t st);
extern "C" int xcg_launch_seed_tiling(const XcgStreamArgs* a, hipStream_t stream);
