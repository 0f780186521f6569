// Host side of the C ABI declared in include/xcgpu.h.
//
// A context pins a device and the encoder configuration the reference keeps
// in XCodecEncoder / XCodecCache (stream_ = !cache_->out_of_band(),
// xcodec/xcodec_encoder.cc:40-46).  All work is enqueued on the caller's
// stream; nothing here allocates or synchronises inside xcg_encode_batch, so a
// caller may capture it into a hipGraph.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <ctype.h>

#include <algorithm>
#include <chrono>
#include <iterator>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/xcgpu.h"
#include "xcg_args.h"

extern "C" int xcg_launch_encode_independent(const uint8_t*, const uint64_t*, const uint32_t*, uint32_t, uint32_t,
                                             uint32_t, uint8_t*, const uint64_t*, uint64_t*, uint32_t*, int32_t*,
                                             hipStream_t);
extern "C" int xcg_launch_window_hashes(const uint8_t*, uint64_t, uint64_t*, hipStream_t);


extern "C" int xcg_launch_segment_hashes(const uint8_t*, uint64_t, uint64_t*, hipStream_t);

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
  uint64_t* u_keys;
  uint64_t* unknown;
  uint64_t* unknown_pos;
  uint32_t* nunknown;
  uint32_t unknown_cap;
  uint64_t* scratch;
  uint64_t* h_scratch;
  uint64_t* chunk_tmp;
  uint4* d_tail;
  uint64_t* win_hash;
  uint8_t* win_seg;
  uint64_t win_count;
  XcgLruState* lru;      // bounded cache (null: unbounded)
  uint32_t maxd;         // EXTRACTs a chunk can hold (bounded: declaration rows per chunk)
  XcgPairState* pair;    // XCodecCachePair (null: not a pair)
  int no_window;         // the BACKREF window is left alone (<LEARN>, single-segment host calls)
};
extern "C" int xcg_launch_pack(const uint8_t*, const uint64_t*, const uint64_t*, uint32_t, uint8_t*, uint64_t*,
                               uint64_t*, hipStream_t);
extern "C" int xcg_launch_cache_lookup(uint64_t*, uint64_t*, uint32_t, const uint8_t*, uint64_t, uint8_t*, int32_t*,
                                       hipStream_t);
extern "C" int xcg_launch_cache_enter(uint64_t*, uint64_t*, uint32_t, uint8_t*, uint32_t*, uint32_t, uint32_t*,
                                      uint32_t*, uint32_t, uint32_t*, uint32_t, uint64_t, const uint8_t*, int, int32_t*,
                                      hipStream_t);
extern "C" int xcg_launch_decode(const XcgDecodeArgs*, uint64_t*, uint64_t*, uint64_t*, uint32_t*, hipStream_t);

// The persistent segment cache of a context: XCodecMemoryCache's
// hash_map<Tag64, BufferSegment*> (xcodec/xcodec_cache.h:270) as an
// open-addressed table in HBM plus a segment pool, and the two lane-probe
// filters over it (see xcg_cache.h).
struct GpuCache {
  uint64_t* keys = nullptr;
  uint64_t* vals = nullptr;
  uint32_t mask = 0;
  uint8_t* pool = nullptr;
  uint32_t seg_cap = 0;
  uint32_t* nseg = nullptr;     // device counter
  uint32_t* filt = nullptr;     // FILT_WORDS
  uint32_t* ftab = nullptr;     // fbuckets * 4
  uint32_t fmask = 0;
  uint32_t* gfilt = nullptr;    // global lane filter: gmask + 1 words (~1 per segment)
  uint32_t gmask = 0;
  bool pool_borrowed = false;   // (a pair front's pool: owned by its XcgPairState)
};

struct BatchScratch {
  uint32_t n_cap = 0, maxd = 0;
  uint64_t* b_keys = nullptr;
  uint64_t* b_vals = nullptr;
  uint32_t b_mask = 0;
  uint32_t* r_filt = nullptr;
  uint32_t* r_ftab = nullptr;
  void* decl = nullptr;
  uint32_t* ndecl = nullptr;
  uint32_t* changed = nullptr;
  uint32_t* h_changed = nullptr;   // pinned
  uint32_t* r_gfilt = nullptr;
  uint32_t* bcount = nullptr;
  // verification between rounds
  uint64_t* b2_keys = nullptr;     // second batch table (same mask)
  uint64_t* b2_vals = nullptr;
  uint64_t* r_keys = nullptr;      // changed hashes -> chunk range
  uint64_t* r_vals = nullptr;
  uint32_t r_mask = 0;
  uint64_t* hits = nullptr;        // n_cap * maxh batch hits
  uint32_t* nhits = nullptr;
  uint32_t maxh = 0;
  uint32_t* need = nullptr;
  uint32_t* vflags = nullptr;
  uint32_t* h_vflags = nullptr;    // pinned
  uint64_t* a_keys = nullptr;      // newly visible hashes -> chunk range (verification (a))
  uint64_t* a_vals = nullptr;
  uint32_t* a_bits = nullptr;
  uint32_t* s_fold = nullptr;      // quiet-chunk screen: LDS fold of the lane filter
  uint32_t* s_work = nullptr;      // [n + 1] its work list
  uint32_t* s_info = nullptr;      // [n] its verdicts
  uint32_t* s_rows = nullptr;      // [n * 4] uint4: its staged rows
  uint32_t* s_qcnt = nullptr;      // [n], [n * 1024]: its queued windows
  uint32_t* s_qkeys = nullptr;
  uint32_t last_maxd = 0;          // declaration stride of the last stream batch
  // bounded cache: every chunk's cache references (xcg_lru.hip)
  void* ev = nullptr;              // n_cap * maxe uint4
  uint32_t* nev = nullptr;
  uint32_t maxe = 0;
  uint32_t* ev_base = nullptr;     // n_cap + 1
  uint32_t* enter_base = nullptr;  // n_cap + 1
  uint32_t* ev_slot = nullptr;     // n_cap * maxe: each reference's pool slot / LRU time
  uint64_t* ev_time = nullptr;
  // re-parse restart (xcg_encode.hip RestartArgs): REF output lengths, the
  // contradicted-lookup times, and a backup of the flagged chunks' rows
  uint32_t* eo = nullptr;          // n_cap * maxe
  uint32_t* bad_t = nullptr;       // n_cap
  uint32_t* bad_hi = nullptr;      // n_cap
  uint32_t* bslot = nullptr;       // n_cap
  uint32_t* b_count = nullptr;
  uint32_t b_slots = 0;
  void* b_ev = nullptr;            // b_slots * maxe uint4
  uint32_t* b_eo = nullptr;
  uint64_t* b_hits = nullptr;      // b_slots * maxh
  uint32_t* b_cnt = nullptr;       // b_slots * 4
  uint8_t* b_out = nullptr;        // b_slots * b_stride
  uint64_t b_stride = 0;
  void* splice = nullptr;          // n_cap uint4
};

struct DecodeScratch {
  uint32_t x_cap = 0;
  uint64_t* x_keys = nullptr;
  uint64_t* x_vals = nullptr;
  uint64_t* x_latest = nullptr;
  uint64_t* u_keys = nullptr;      // unknown-hash set (2 * UNKNOWN_CAP)
  uint64_t* unknown = nullptr;
  uint64_t* unknown_pos = nullptr;
  uint32_t* nunknown = nullptr;
  uint64_t* scratch = nullptr;
  uint64_t* h_scratch = nullptr;   // pinned
  uint32_t chunk_cap = 0;
  uint64_t* chunk_tmp = nullptr;   // 4 u64 per chunk (declare counts / bases)
  uint4* d_tail = nullptr;         // 256 declare records (window update)
};

// A decoder's BACKREF window (XCodecWindow, xcodec/xcodec_window.h): 256 slots
// of (hash, owned 2048-byte copy) and the number of declares made so far
// (cursor = count mod 256).  One per XCodecDecoder; a context has a default.
struct xcg_window {
  int device = 0;
  uint64_t* hash = nullptr;
  uint8_t* seg = nullptr;
  uint64_t count = 0;
};
constexpr uint32_t UNKNOWN_CAP = 1u << 16;

struct xcg_ctx {
  int device;
  uint32_t flags;
  int32_t* d_status;   // sticky internal-overflow word
  uint64_t cache_segments;
  GpuCache g;
  BatchScratch bs;
  int last_rounds;
  DecodeScratch ds;
  xcg_window* own_win = nullptr;   // default window (lazily allocated)
  xcg_window* cur_win = nullptr;   // window used by decodes (own_win unless set)
  int32_t* h_status = nullptr;     // pinned copy of d_status
  // seed the next stream batch with the chunks' tilings: a fresh cache is cold (every
  // first batch declares), and later the last batch declared something
  bool seed_next = true;
  bool bounded = false;            // XCodecMemoryCache with a limit: LRU eviction (xcg_lru.hip)
  XcgLruState lru{};
  // Completion of the context's last enqueued work (recorded on the caller's
  // stream): the cache-inspection calls wait for this event only, never for
  // the whole device, so other contexts and streams keep running.
  hipEvent_t done_ev = nullptr;
  hipEvent_t flags_ev = nullptr;   // stream batches: behind the verification flags' copy (xcg_encode.hip)
  XcgPairState* pair = nullptr;   // XCodecCachePair(memory, disk) (xcg_pair.hip): a front of a disk
  uint32_t pair_C = 0;             // its primary limit in segments
  bool no_window = false;          // (single-segment host calls: decodes that leave the window alone)
  // Host-call staging (xcg_encode_call / xcg_encode_host): kept across calls,
  // so a per-call encode() allocates nothing and synchronises once.
  uint8_t* stage_h = nullptr;      // pinned
  uint8_t* stage_d = nullptr;
  size_t stage_h_cap = 0, stage_d_cap = 0;
  hipStream_t call_st = nullptr;
  hipStream_t last_mark = nullptr; // stream of the last ctx_mark (ctx_order on it needs no wait)
  bool marked = false;
  bool mark_pending = false;       // done_ev not yet recorded behind the last call (ctx_flush_mark)
  // zero-copy staging of the one-launch decode() (coherent pinned host memory
  // the kernel reads and writes directly): [flag 256][input][output][results]
  uint8_t* zc_h = nullptr;
  size_t zc_cap = 0;
  uint32_t zc_seq = 0;
};

namespace {

// Stream-round seeding: -1 automatic, 0 never, 1 always (tests exercise both).
int g_stream_seed = -1;

// XCodecCache's process-wide UUID map (xcodec/xcodec_cache.h:101-127):
// lowercase UUID -> context, and whether the registry made (owns) it.
struct RegEntry {
  xcg_ctx* ctx;
  bool owned;
};
std::mutex g_reg_mu;
std::map<std::string, RegEntry> g_reg;
// A pipe that connected a registry context at <HELLO> holds it until the pipe
// is destroyed (xcg_pipe.cpp); clearing the registry destroys a held context
// only when its last holder lets go (g_deferred), never under a live pipe.
std::map<xcg_ctx*, int> g_holds;
std::set<xcg_ctx*> g_deferred;

bool uuid_key(const char* u, std::string* key) {     // the 8-4-4-4-12 form UUID::decode takes
  if (!u) return false;
  std::string k(36, ' ');
  for (int i = 0; i < 36; ++i) {
    const char c = u[i];
    const bool dash = i == 8 || i == 13 || i == 18 || i == 23;
    if (dash ? c != '-' : !isxdigit((unsigned char)c)) return false;
    k[i] = (char)tolower((unsigned char)c);
  }
  *key = k;
  return true;
}

void registry_forget(xcg_ctx* c) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (auto it = g_reg.begin(); it != g_reg.end();) it = it->second.ctx == c ? g_reg.erase(it) : std::next(it);
}

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

constexpr uint32_t FILT_WORDS = (1u << 19) / 32;   // xcg_cache.h FILT_LOG2
constexpr uint32_t PREFIX_FILTERS = 16;             // xcg_cache.h: slices of a round's LDS filter

// The context's last call was enqueued on last_mark; done_ev is recorded
// behind it only when another stream or a host wait needs it.  Recording it
// later on the same stream marks the same point or a later one (never an
// earlier one), and back-to-back calls on one stream -- the batched encode's
// steady state -- enqueue nothing but their kernels (a marker per call cost
// the headline launch ~5-10 us of gap).
void ctx_flush_mark(xcg_ctx* c) {
  if (c->mark_pending && c->done_ev) (void)hipEventRecord(c->done_ev, c->last_mark);
  c->mark_pending = false;
}
// The context's work so far is complete (its last call's stream reached the
// event) -- the per-context replacement for a device-wide synchronise.
int ctx_wait(xcg_ctx* c) {
  ctx_flush_mark(c);
  return c->done_ev && hipEventSynchronize(c->done_ev) != hipSuccess ? XCG_EHIP : XCG_OK;
}
void ctx_mark(xcg_ctx* c, hipStream_t st) {
  c->last_mark = st;
  c->marked = true;
  c->mark_pending = true;
}
// Work enqueued on `st` starts after the context's last enqueued work (a cache
// clear on another stream, the previous call of another stream): the
// reference's calls on one cache are serialised, and so are these.
void ctx_order(xcg_ctx* c, hipStream_t st) {
  if (c->marked && c->last_mark == st && st != nullptr) return;   // (in stream order already)
  ctx_flush_mark(c);
  if (c->done_ev) (void)hipStreamWaitEvent(st, c->done_ev, 0);
}

uint32_t pow2_at_least(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return (uint32_t)p;
}

void free_cache(GpuCache& g) {
  (void)hipFree(g.keys); (void)hipFree(g.vals); (void)hipFree(g.nseg);
  if (!g.pool_borrowed) (void)hipFree(g.pool);
  (void)hipFree(g.filt); (void)hipFree(g.ftab); (void)hipFree(g.gfilt);
  g = GpuCache{};
}

void free_lru(XcgLruState& L) {
  (void)hipFree(L.skey); (void)hipFree(L.lastref); (void)hipFree(L.queue); (void)hipFree(L.queue2);
  (void)hipFree(L.ptime); (void)hipFree(L.hmin); (void)hipFree(L.wpop); (void)hipFree(L.tau);
  (void)hipFree(L.alive); (void)hipFree(L.freel); (void)hipFree(L.part);
  (void)hipFree(L.tot);
  if (L.h_tot) (void)hipHostFree(L.h_tot);
  if (L.tev) (void)hipEventDestroy((hipEvent_t)L.tev);
  const uint32_t C = L.C;
  L = XcgLruState{};
  L.C = C;
}

int alloc_lru(XcgLruState& L) {
  const uint64_t C = L.C;
  if (hipMalloc(&L.skey, 8 * C) != hipSuccess || hipMalloc(&L.lastref, 8 * C) != hipSuccess ||
      hipMalloc(&L.queue, 4 * C) != hipSuccess || hipMalloc(&L.queue2, 4 * C) != hipSuccess ||
      hipMalloc(&L.ptime, 8 * C) != hipSuccess || hipMalloc(&L.hmin, 8 * C) != hipSuccess ||
      hipMalloc(&L.wpop, 8 * C) != hipSuccess || hipMalloc(&L.tau, 8 * C) != hipSuccess ||
      hipMalloc(&L.alive, 4 * C) != hipSuccess || hipMalloc(&L.freel, 4 * C) != hipSuccess ||
      hipMalloc(&L.tot, 64) != hipSuccess || hipHostMalloc(&L.h_tot, 64) != hipSuccess ||
      hipMemset(L.lastref, 0, 8 * C) != hipSuccess) {
    free_lru(L);
    return XCG_ENOMEM;
  }
  L.clock = 1;
  return XCG_OK;
}

void free_scratch(BatchScratch& b) {
  (void)hipFree(b.b_keys); (void)hipFree(b.b_vals); (void)hipFree(b.r_filt); (void)hipFree(b.r_ftab);
  (void)hipFree(b.decl); (void)hipFree(b.ndecl); (void)hipFree(b.changed); (void)hipFree(b.r_gfilt);
  (void)hipFree(b.bcount);
  (void)hipFree(b.b2_keys); (void)hipFree(b.b2_vals); (void)hipFree(b.r_keys); (void)hipFree(b.r_vals);
  (void)hipFree(b.hits); (void)hipFree(b.nhits); (void)hipFree(b.need); (void)hipFree(b.vflags);
  if (b.h_vflags) (void)hipHostFree(b.h_vflags);
  if (b.h_changed) (void)hipHostFree(b.h_changed);
  (void)hipFree(b.ev); (void)hipFree(b.nev); (void)hipFree(b.ev_base); (void)hipFree(b.enter_base);
  (void)hipFree(b.ev_slot); (void)hipFree(b.ev_time);
  (void)hipFree(b.eo); (void)hipFree(b.bad_t); (void)hipFree(b.bad_hi); (void)hipFree(b.bslot);
  (void)hipFree(b.b_count); (void)hipFree(b.b_ev); (void)hipFree(b.b_eo); (void)hipFree(b.b_hits);
  (void)hipFree(b.b_cnt); (void)hipFree(b.b_out); (void)hipFree(b.splice);
  (void)hipFree(b.a_keys); (void)hipFree(b.a_vals); (void)hipFree(b.a_bits);
  (void)hipFree(b.s_fold); (void)hipFree(b.s_work); (void)hipFree(b.s_info); (void)hipFree(b.s_rows);
  (void)hipFree(b.s_qcnt); (void)hipFree(b.s_qkeys);
  b = BatchScratch{};
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// The context's host-call staging: pinned host and device blocks of at least
// the given sizes, and its own stream.
int ensure_stage(xcg_ctx* c, size_t dbytes, size_t hbytes) {
  if (!c->call_st && hipStreamCreateWithFlags(&c->call_st, hipStreamNonBlocking) != hipSuccess) return XCG_EHIP;
  if (dbytes > c->stage_d_cap) {
    if (c->stage_d) { (void)hipStreamSynchronize(c->call_st); (void)hipFree(c->stage_d); }
    c->stage_d = nullptr;
    c->stage_d_cap = 0;
    const size_t want = dbytes < (1u << 20) ? (1u << 20) : dbytes;
    if (hipMalloc(&c->stage_d, want) != hipSuccess) return XCG_ENOMEM;
    c->stage_d_cap = want;
  }
  if (hbytes > c->stage_h_cap) {
    if (c->stage_h) { (void)hipStreamSynchronize(c->call_st); (void)hipHostFree(c->stage_h); }
    c->stage_h = nullptr;
    c->stage_h_cap = 0;
    const size_t want = hbytes < (1u << 20) ? (1u << 20) : hbytes;
    if (hipHostMalloc(&c->stage_h, want, hipHostMallocDefault) != hipSuccess) return XCG_ENOMEM;
    c->stage_h_cap = want;
  }
  return XCG_OK;
}

// Every array of an empty cache in one launch: the table (all ones), the
// segment count and the three probe filters (zero).
__global__ __launch_bounds__(256) void cache_wipe_kernel(uint4* kv, uint64_t kv_n, uint32_t* nseg, uint4* filt,
                                                         uint32_t filt_n, uint4* ftab, uint64_t ftab_n, uint4* gfilt,
                                                         uint64_t gfilt_n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u), zero = make_uint4(0u, 0u, 0u, 0u);
  for (uint64_t i = i0; i < kv_n; i += stride) kv[i] = ones;
  for (uint64_t i = i0; i < filt_n; i += stride) filt[i] = zero;
  for (uint64_t i = i0; i < ftab_n; i += stride) ftab[i] = zero;
  for (uint64_t i = i0; i < gfilt_n; i += stride) gfilt[i] = zero;
  if (i0 == 0) *nseg = 0u;
}

int clear_cache(GpuCache& g, bool sync = true) {
  // keys and vals are separate allocations of (mask + 1) u64 each (>= 1024)
  const uint64_t half = (uint64_t)(g.mask + 1) / 2;   // uint4 per array
  hipLaunchKernelGGL(cache_wipe_kernel, dim3(1024), dim3(256), 0, nullptr, (uint4*)g.keys, half, g.nseg,
                     (uint4*)g.filt, FILT_WORDS / 4, (uint4*)g.ftab, (uint64_t)g.fmask + 1, (uint4*)g.gfilt,
                     ((uint64_t)g.gmask + 1) / 4);
  hipLaunchKernelGGL(cache_wipe_kernel, dim3(256), dim3(256), 0, nullptr, (uint4*)g.vals, half, g.nseg,
                     (uint4*)nullptr, 0u, (uint4*)nullptr, 0ull, (uint4*)nullptr, 0ull);
  if (hipGetLastError() != hipSuccess || (sync && hipStreamSynchronize(nullptr) != hipSuccess)) return XCG_EHIP;
  return XCG_OK;
}

// Lazily allocate the persistent cache (segments * 2 KiB of pool).
int ensure_cache(xcg_ctx* c) {
  if (c->g.keys) return XCG_OK;
  GpuCache& g = c->g;
  const uint64_t segs = c->cache_segments;
  g.seg_cap = (uint32_t)segs;
  const uint32_t cap = pow2_at_least(2 * segs + 1024);
  g.mask = cap - 1;
  // ~2 keys per bucket at capacity.  A bounded cache is always full and a
  // batch's declarations (up to the limit again) share the round's copy, so
  // it gets ~1 bucket per key (a bucket past 7 fingerprints sends every probe
  // into an exact check).
  const uint64_t fkeys = c->bounded ? 4 * segs : (c->pair ? segs + 2ull * c->pair_C : segs);
  const uint32_t fb = pow2_at_least(fkeys < 65536 ? 32768 : fkeys / 2);
  g.fmask = fb - 1;
  const uint32_t gw = pow2_at_least(fkeys < 131072 ? 65536 : fkeys / 2);
  g.gmask = gw - 1;
  // A pair front's pool is its primary followed by the disk's blocks, mapped
  // by the pair state (one physical disk behind every front, xcg_pair.hip).
  g.pool_borrowed = c->pair != nullptr;
  if (c->pair) g.pool = xcg_pair_state_pool(c->pair);
  if (hipMalloc(&g.keys, 8ull * cap) != hipSuccess || hipMalloc(&g.vals, 8ull * cap) != hipSuccess ||
      (!c->pair && hipMalloc(&g.pool, segs * (uint64_t)XCG_SEGMENT_LENGTH + 16) != hipSuccess) ||
      hipMalloc(&g.nseg, 16) != hipSuccess || hipMalloc(&g.filt, 4ull * FILT_WORDS) != hipSuccess ||
      hipMalloc(&g.ftab, 16ull * fb) != hipSuccess || hipMalloc(&g.gfilt, 4ull * gw) != hipSuccess) {
    free_cache(g);
    return XCG_ENOMEM;
  }
  int rc = clear_cache(g);
  if (rc == XCG_OK && c->bounded) rc = alloc_lru(c->lru);
  if (rc) free_cache(g);
  return rc;
}

// The quiet-chunk screen's key queues (small-chunk calls, maxd <= 4): 4 KiB
// per chunk of the scratch's capacity (SCREEN_QCAP keys; ~ the input's size
// for 4 KiB packets), allocated by the first such call on the context --
// whatever size of chunks grew the scratch before it -- and kept with it.
int ensure_screen_queues(BatchScratch& b, uint32_t maxd) {
  if (maxd > 4 || (b.s_qcnt && b.s_qkeys)) return XCG_OK;
  if (hipMalloc(&b.s_qcnt, 4ull * b.n_cap) != hipSuccess || hipMalloc(&b.s_qkeys, 4096ull * b.n_cap) != hipSuccess) {
    (void)hipFree(b.s_qcnt); (void)hipFree(b.s_qkeys);
    b.s_qcnt = nullptr; b.s_qkeys = nullptr;      // (the screen stays off; the parse decides alone)
  }
  return XCG_OK;
}

int ensure_scratch(xcg_ctx* c, uint32_t n, uint32_t maxd) {
  BatchScratch& b = c->bs;
  if (b.decl && n <= b.n_cap && maxd <= b.maxd) return ensure_screen_queues(b, maxd);
  free_scratch(b);
  b.n_cap = n;
  b.maxd = maxd;
  const uint32_t cap = pow2_at_least(2ull * n * maxd + 1024);
  b.b_mask = cap - 1;
  b.r_mask = 2 * cap - 1;          // union of two rounds' hashes
  b.maxh = maxd + 8;
  if (hipMalloc(&b.b_keys, 8ull * cap) != hipSuccess || hipMalloc(&b.b_vals, 8ull * cap) != hipSuccess ||
      hipMalloc(&b.r_filt, 4ull * FILT_WORDS * PREFIX_FILTERS) != hipSuccess ||
      hipMalloc(&b.r_ftab, 16ull * (c->g.fmask + 1)) != hipSuccess ||
      hipMalloc(&b.decl, 16ull * n * maxd) != hipSuccess || hipMalloc(&b.ndecl, 4ull * n) != hipSuccess ||
      hipMalloc(&b.changed, 16) != hipSuccess || hipHostMalloc(&b.h_changed, 16) != hipSuccess ||
      hipMalloc(&b.r_gfilt, 4ull * (c->g.gmask + 1)) != hipSuccess || hipMalloc(&b.bcount, 4 * 64) != hipSuccess ||
      hipMalloc(&b.b2_keys, 8ull * cap) != hipSuccess || hipMalloc(&b.b2_vals, 8ull * cap) != hipSuccess ||
      hipMalloc(&b.r_keys, 16ull * cap) != hipSuccess || hipMalloc(&b.r_vals, 16ull * cap) != hipSuccess ||
      hipMalloc(&b.hits, 8ull * n * (maxd + 8)) != hipSuccess || hipMalloc(&b.nhits, 4ull * n) != hipSuccess ||
      hipMalloc(&b.need, 4ull * n) != hipSuccess || hipMalloc(&b.vflags, 16) != hipSuccess ||
      hipHostMalloc(&b.h_vflags, 16) != hipSuccess || hipMalloc(&b.a_keys, 8ull * XCG_VERIFY_A_CAP) != hipSuccess ||
      hipMalloc(&b.a_vals, 8ull * XCG_VERIFY_A_CAP) != hipSuccess ||
      hipMalloc(&b.a_bits, 4ull * XCG_VERIFY_A_WORDS) != hipSuccess ||
      hipMalloc(&b.s_fold, 4ull * 32768) != hipSuccess || hipMalloc(&b.s_work, 4ull * (n + 1)) != hipSuccess ||
      hipMalloc(&b.s_info, 4ull * n) != hipSuccess || hipMalloc(&b.s_rows, 64ull * n) != hipSuccess) {
    free_scratch(b);
    return XCG_ENOMEM;
  }
  ensure_screen_queues(b, maxd);
  if (c->bounded || c->pair) {
    b.maxe = 2 * maxd + 64;        // declarations + REFs + collision lookups of one chunk
    if (hipMalloc(&b.ev, 16ull * n * b.maxe) != hipSuccess || hipMalloc(&b.nev, 4ull * n) != hipSuccess ||
        hipMalloc(&b.ev_base, 4ull * (n + 1)) != hipSuccess || hipMalloc(&b.enter_base, 4ull * (n + 1)) != hipSuccess ||
        hipMalloc(&b.ev_slot, 4ull * n * b.maxe) != hipSuccess || hipMalloc(&b.ev_time, 8ull * n * b.maxe) != hipSuccess) {
      free_scratch(b);
      return XCG_ENOMEM;
    }
    // restart backups for up to b_slots flagged chunks per pass (more re-parse from the start)
    b.b_slots = n < 256 ? n : 256;
    b.b_stride = (2ull * maxd * XCG_SEGMENT_LENGTH + 16 + 255) & ~255ull;   // >= xcg_encode_bound(max chunk)
    if (hipMalloc(&b.eo, 4ull * n * b.maxe) != hipSuccess || hipMalloc(&b.bad_t, 4ull * n) != hipSuccess ||
        hipMalloc(&b.bad_hi, 4ull * n) != hipSuccess || hipMalloc(&b.bslot, 4ull * n) != hipSuccess ||
        hipMalloc(&b.b_count, 16) != hipSuccess || hipMalloc(&b.b_ev, 16ull * b.b_slots * b.maxe) != hipSuccess ||
        hipMalloc(&b.b_eo, 4ull * b.b_slots * b.maxe) != hipSuccess ||
        hipMalloc(&b.b_hits, 8ull * b.b_slots * b.maxh) != hipSuccess ||
        hipMalloc(&b.b_cnt, 16ull * b.b_slots) != hipSuccess ||
        hipMalloc(&b.b_out, b.b_stride * b.b_slots) != hipSuccess || hipMalloc(&b.splice, 16ull * n) != hipSuccess ||
        hipMemset(b.splice, 0, 16ull * n) != hipSuccess || hipMemset(b.bad_t, 0xFF, 4ull * n) != hipSuccess ||
        hipMemset(b.bad_hi, 0, 4ull * n) != hipSuccess || hipMemset(b.b_count, 0, 16) != hipSuccess) {
      free_scratch(b);
      return XCG_ENOMEM;
    }
  }
  return XCG_OK;
}

void free_dscratch(DecodeScratch& d) {
  (void)hipFree(d.x_keys); (void)hipFree(d.x_vals); (void)hipFree(d.x_latest); (void)hipFree(d.unknown);
  (void)hipFree(d.u_keys);
  (void)hipFree(d.unknown_pos); (void)hipFree(d.nunknown); (void)hipFree(d.scratch);
  (void)hipFree(d.chunk_tmp); (void)hipFree(d.d_tail);
  if (d.h_scratch) (void)hipHostFree(d.h_scratch);
  d = DecodeScratch{};
}

int ensure_dchunks(xcg_ctx* c, uint32_t n) {
  DecodeScratch& d = c->ds;
  if (!d.d_tail && hipMalloc(&d.d_tail, 16ull * 256) != hipSuccess) return XCG_ENOMEM;
  if (d.chunk_tmp && n <= d.chunk_cap) return XCG_OK;
  (void)hipFree(d.chunk_tmp);
  d.chunk_tmp = nullptr;
  d.chunk_cap = n < 1024 ? 1024 : n;
  if (hipMalloc(&d.chunk_tmp, 32ull * d.chunk_cap) != hipSuccess) {
    d.chunk_cap = 0;
    return XCG_ENOMEM;
  }
  return XCG_OK;
}

int window_alloc(int device, xcg_window** out) {
  xcg_window* w = new xcg_window;
  w->device = device;
  if (hipMalloc(&w->hash, 8ull * 256) != hipSuccess || hipMalloc(&w->seg, 256ull * 2048) != hipSuccess ||
      hipMemset(w->hash, 0, 8ull * 256) != hipSuccess) {
    (void)hipFree(w->hash); (void)hipFree(w->seg);
    delete w;
    return XCG_ENOMEM;
  }
  *out = w;
  return XCG_OK;
}

void window_free(xcg_window* w) {
  if (!w) return;
  (void)hipFree(w->hash); (void)hipFree(w->seg);
  delete w;
}

int ensure_dscratch(xcg_ctx* c, uint64_t max_extracts) {
  DecodeScratch& d = c->ds;
  const uint32_t cap = pow2_at_least(2 * max_extracts + 1024);
  if (d.x_keys && cap <= d.x_cap) return XCG_OK;
  free_dscratch(d);
  d.x_cap = cap;
  if (hipMalloc(&d.x_keys, 8ull * cap) != hipSuccess || hipMalloc(&d.x_vals, 8ull * cap) != hipSuccess ||
      hipMalloc(&d.x_latest, 8ull * cap) != hipSuccess || hipMalloc(&d.unknown, 8ull * UNKNOWN_CAP) != hipSuccess ||
      hipMalloc(&d.u_keys, 16ull * UNKNOWN_CAP) != hipSuccess ||
      hipMalloc(&d.unknown_pos, 8ull * UNKNOWN_CAP) != hipSuccess || hipMalloc(&d.nunknown, 16) != hipSuccess ||
      hipMalloc(&d.scratch, 64) != hipSuccess || hipHostMalloc(&d.h_scratch, 128) != hipSuccess) {
    free_dscratch(d);
    return XCG_ENOMEM;
  }
  return XCG_OK;
}

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
    case XCG_ENOENT: return "no such segment";
    case XCG_EPROTO: return "pipe protocol error";
    case XCG_EEXIST: return "already registered";
    default: return "unknown status";
  }
}

uint64_t xcg_encode_bound(uint32_t len) { return 2ull * len + 16ull; }

int xcg_debug_set_stream_seed(int mode) {
  return __atomic_exchange_n(&g_stream_seed, mode < 0 ? -1 : (mode ? 1 : 0), __ATOMIC_RELAXED);
}

int xcg_ctx_create(int device, uint32_t flags, xcg_ctx** out) {
  return xcg_ctx_create_ex(device, flags, XCG_DEFAULT_CACHE_SEGMENTS, out);
}

int xcg_ctx_create_bounded(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_ctx** out) {
  if (!out || memory_cache_limit_bytes == 0) return XCG_EINVAL;
  // memory_cache_limit_ = bytes / XCODEC_SEGMENT_LENGTH, at least 1 (xcodec_cache.h:277-288)
  uint64_t segs = memory_cache_limit_bytes / XCG_SEGMENT_LENGTH;
  if (segs == 0) segs = 1;
  if (segs > (1ull << 29) || (flags & XCG_FLAG_NULLCACHE)) return XCG_EINVAL;
  const int rc = xcg_ctx_create_ex(device, flags, segs, out);
  if (rc != XCG_OK) return rc;
  (*out)->bounded = true;
  (*out)->lru.C = (uint32_t)segs;
  return XCG_OK;
}

int xcg_disk_create(uint64_t disk_bytes, xcg_disk** out) { return xcg_disk_create_ex(disk_bytes, 0, out); }

int xcg_disk_create_ex(uint64_t disk_bytes, uint32_t flags, xcg_disk** out) {
  if (!out || (flags & ~(XCG_DISK_HOST | XCG_DISK_DEVICE)) || flags == (XCG_DISK_HOST | XCG_DISK_DEVICE))
    return XCG_EINVAL;
  *out = nullptr;
  XcgDiskState* K = nullptr;
  const int rc = xcg_disk_state_create(disk_bytes, flags, &K);
  if (rc) return rc == -22 ? XCG_EINVAL : XCG_ENOMEM;
  *out = (xcg_disk*)K;
  return XCG_OK;
}

void xcg_disk_destroy(xcg_disk* d) { xcg_disk_state_release((XcgDiskState*)d); }

int xcg_disk_open(const char* path, uint64_t disk_bytes, uint32_t flags, xcg_disk** out) {
  if (!out || !path || (flags & ~(XCG_DISK_HOST | XCG_DISK_DEVICE)) || flags == (XCG_DISK_HOST | XCG_DISK_DEVICE))
    return XCG_EINVAL;
  *out = nullptr;
  XcgDiskState* K = nullptr;
  const int rc = xcg_disk_state_open(path, disk_bytes, flags, &K);
  if (rc) return rc == -22 ? XCG_EINVAL : (rc == -2 ? XCG_ENOENT : XCG_ENOMEM);
  *out = (xcg_disk*)K;
  return XCG_OK;
}

int xcg_disk_open_fd(int fd, uint64_t disk_bytes, uint32_t flags, xcg_disk** out) {
  if (!out || fd < 0 || (flags & ~(XCG_DISK_HOST | XCG_DISK_DEVICE)) ||
      flags == (XCG_DISK_HOST | XCG_DISK_DEVICE))
    return XCG_EINVAL;
  *out = nullptr;
  XcgDiskState* K = nullptr;
  const int rc = xcg_disk_state_open_fd(fd, disk_bytes, flags, &K);
  if (rc) return rc == -22 ? XCG_EINVAL : (rc == -2 ? XCG_ENOENT : XCG_ENOMEM);
  *out = (xcg_disk*)K;
  return XCG_OK;
}

int xcg_disk_head(const xcg_disk* d, uint64_t* index_block, uint64_t* next_entry) {
  if (!d || !index_block || !next_entry) return XCG_EINVAL;
  xcg_disk_state_head((const XcgDiskState*)d, index_block, next_entry);
  return XCG_OK;
}

int xcg_pair_xuid(const xcg_ctx* c) { return c && c->pair ? (int)xcg_pair_state_xuid(c->pair) : XCG_EINVAL; }

int xcg_disk_save(xcg_disk* d, const char* path) {
  if (!d || !path) return XCG_EINVAL;
  const int rc = xcg_disk_state_save((XcgDiskState*)d, path);
  return rc == 0 ? XCG_OK : (rc == -2 ? XCG_ENOENT : XCG_EHIP);
}

int xcg_disk_tier(const xcg_disk* d) { return d ? xcg_disk_state_tier((const XcgDiskState*)d) : XCG_EINVAL; }

int xcg_disk_stats(const xcg_disk* d, uint64_t* st) {
  if (!d || !st) return XCG_EINVAL;
  xcg_disk_state_stats((const XcgDiskState*)d, st);
  return XCG_OK;
}

int xcg_ctx_create_pair_on(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_disk* disk,
                           xcg_ctx** out) {
  return xcg_ctx_create_pair_uuid(device, flags, memory_cache_limit_bytes, disk, nullptr, out);
}

int xcg_ctx_create_pair_uuid(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_disk* disk,
                             const char* uuid36, xcg_ctx** out) {
  return xcg_ctx_create_pair_xuid(device, flags, memory_cache_limit_bytes, disk, uuid36, -1, out);
}

int xcg_ctx_create_pair_xuid(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_disk* disk,
                             const char* uuid36, int xuid, xcg_ctx** out) {
  if (!out || !disk || memory_cache_limit_bytes == 0 || (flags & (XCG_FLAG_OOB | XCG_FLAG_NULLCACHE)) || xuid < -1)
    return XCG_EINVAL;
  *out = nullptr;
  uint64_t C = memory_cache_limit_bytes / XCG_SEGMENT_LENGTH;   // xcodec_cache.h:283-287
  if (C == 0) C = 1;
  if (C > (1ull << 28)) return XCG_EINVAL;
  XcgPairState* P = nullptr;
  {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return XCG_EINVAL;
    DeviceGuard g(device);
    const int prc = xcg_pair_state_create((uint32_t)C, (XcgDiskState*)disk, uuid36, xuid, &P);
    if (prc == -22) return XCG_EINVAL;
    if (prc) return XCG_ENOMEM;
  }
  const int rc = xcg_ctx_create_ex(device, flags, C + xcg_pair_state_disk_blocks(P), out);
  if (rc != XCG_OK) {
    DeviceGuard g(device);
    xcg_pair_state_destroy(P);
    return rc;
  }
  (*out)->pair = P;
  (*out)->pair_C = (uint32_t)C;
  return XCG_OK;
}

int xcg_ctx_create_pair_unbounded(int device, uint32_t flags, uint64_t capacity_segments, xcg_disk* disk,
                                  const char* uuid36, int xuid, xcg_ctx** out) {
  if (capacity_segments == 0) capacity_segments = XCG_DEFAULT_CACHE_SEGMENTS;
  if (capacity_segments > (1ull << 28)) return XCG_EINVAL;
  const int rc = xcg_ctx_create_pair_xuid(device, flags, capacity_segments * XCG_SEGMENT_LENGTH, disk, uuid36, xuid,
                                          out);
  if (rc == XCG_OK) xcg_pair_state_set_unbounded((*out)->pair);
  return rc;
}

int xcg_ctx_create_pair(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, uint64_t disk_bytes,
                        xcg_ctx** out) {
  if (!out) return XCG_EINVAL;
  xcg_disk* d = nullptr;
  int rc = xcg_disk_create(disk_bytes, &d);
  if (rc != XCG_OK) return rc;
  rc = xcg_ctx_create_pair_on(device, flags, memory_cache_limit_bytes, d, out);
  xcg_disk_destroy(d);                 // (the front holds the disk from here)
  return rc;
}

// XCodecCache::connect(uuid, parent) (xcodec/xcodec_cache.h:101-111) with
// the parent's connect: XCodecMemoryCache::connect (:340-346, an empty cache
// of the same limit), XCodecCachePair::connect (:158-161: the primary's connect
// over XCodecDisk::connect(uuid), xcodec_cache_disk.cc:640-690).
int xcg_ctx_connect(xcg_ctx* parent, const char* uuid36, xcg_ctx** out) {
  std::string key;
  if (!parent || !out || !uuid_key(uuid36, &key)) return XCG_EINVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(key);
  if (it != g_reg.end()) {
    *out = it->second.ctx;
    return XCG_OK;
  }
  xcg_ctx* c = nullptr;
  int rc;
  if (parent->pair && xcg_pair_state_unbounded(parent->pair))
    rc = xcg_ctx_create_pair_unbounded(parent->device, parent->flags, parent->pair_C,
                                       (xcg_disk*)xcg_pair_state_disk(parent->pair), key.c_str(), -1, &c);
  else if (parent->pair)
    rc = xcg_ctx_create_pair_uuid(parent->device, parent->flags, (uint64_t)parent->pair_C * XCG_SEGMENT_LENGTH,
                                  (xcg_disk*)xcg_pair_state_disk(parent->pair), key.c_str(), &c);
  else if (parent->bounded)
    rc = xcg_ctx_create_bounded(parent->device, parent->flags, (uint64_t)parent->lru.C * XCG_SEGMENT_LENGTH, &c);
  else
    rc = xcg_ctx_create_ex(parent->device, parent->flags, parent->cache_segments, &c);
  if (rc != XCG_OK) return rc;
  g_reg[key] = RegEntry{c, true};
  *out = c;
  return XCG_OK;
}

// XCodecCache::enter(uuid, cache) (:113-117): a context the caller keeps.
int xcg_ctx_register(xcg_ctx* c, const char* uuid36) {
  std::string key;
  if (!c || !uuid_key(uuid36, &key)) return XCG_EINVAL;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  if (g_reg.count(key)) return XCG_EEXIST;
  g_reg[key] = RegEntry{c, false};
  return XCG_OK;
}

xcg_ctx* xcg_ctx_lookup(const char* uuid36) {
  std::string key;
  if (!uuid_key(uuid36, &key)) return nullptr;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(key);
  return it == g_reg.end() ? nullptr : it->second.ctx;
}

void xcg_connect_registry_clear(void) {
  std::vector<xcg_ctx*> owned;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (auto& e : g_reg) {
      if (!e.second.owned) continue;
      if (g_holds.count(e.second.ctx)) g_deferred.insert(e.second.ctx);   // (a pipe still uses it)
      else owned.push_back(e.second.ctx);
    }
    g_reg.clear();
  }
  for (xcg_ctx* c : owned) xcg_ctx_destroy(c);
}

// (xcg_pipe.cpp, not part of the ABI) a connecting pipe takes and drops its context
extern "C" void xcg_registry_hold(xcg_ctx* c) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  ++g_holds[c];
}
extern "C" void xcg_registry_release(xcg_ctx* c) {
  bool destroy = false;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_holds.find(c);
    if (it == g_holds.end()) return;
    if (--it->second == 0) {
      g_holds.erase(it);
      destroy = g_deferred.erase(c) != 0;
    }
  }
  if (destroy) xcg_ctx_destroy(c);
}

int xcg_pair_stats(xcg_ctx* c, uint64_t* st) {
  if (!c || !c->pair || !st) return XCG_EINVAL;
  xcg_pair_state_stats(c->pair, st);
  return XCG_OK;
}

int xcg_ctx_create_ex(int device, uint32_t flags, uint64_t cache_segments, xcg_ctx** out) {
  if (!out || cache_segments == 0 || cache_segments > (1ull << 30)) return XCG_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return XCG_EINVAL;
  if (flags & ~(XCG_FLAG_OOB | XCG_FLAG_NULLCACHE)) return XCG_EINVAL;
  DeviceGuard g(device);
  xcg_ctx* c = new xcg_ctx{device, flags, nullptr, cache_segments, GpuCache{}, BatchScratch{}, 0, DecodeScratch{}};
  if (hipMalloc(&c->d_status, 16) != hipSuccess || hipHostMalloc(&c->h_status, 16) != hipSuccess) {
    (void)hipFree(c->d_status);
    delete c;
    return XCG_ENOMEM;
  }
  if (hipMemset(c->d_status, 0, 16) != hipSuccess ||
      hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->flags_ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipFree(c->d_status);
    if (c->done_ev) (void)hipEventDestroy(c->done_ev);
    delete c;
    return XCG_EHIP;
  }
  *out = c;
  return XCG_OK;
}

void xcg_ctx_destroy(xcg_ctx* c) {
  if (!c) return;
  registry_forget(c);
  DeviceGuard g(c->device);
  (void)hipFree(c->d_status);
  if (c->h_status) (void)hipHostFree(c->h_status);
  free_cache(c->g);
  free_lru(c->lru);
  free_scratch(c->bs);
  free_dscratch(c->ds);
  window_free(c->own_win);
  if (c->done_ev) (void)hipEventDestroy(c->done_ev);
  if (c->flags_ev) (void)hipEventDestroy(c->flags_ev);
  xcg_pair_state_destroy(c->pair);
  if (c->stage_h) (void)hipHostFree(c->stage_h);
  if (c->zc_h) (void)hipHostFree(c->zc_h);
  (void)hipFree(c->stage_d);
  if (c->call_st) (void)hipStreamDestroy(c->call_st);
  delete c;
}

uint64_t xcg_cache_size(xcg_ctx* c) {
  if (!c || !c->g.keys) return 0;
  DeviceGuard g(c->device);
  uint32_t n = 0;
  if (ctx_wait(c) != XCG_OK || hipMemcpy(&n, c->g.nseg, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return n < c->g.seg_cap ? n : c->g.seg_cap;
}

int xcg_cache_clear(xcg_ctx* c) {
  if (!c) return XCG_EINVAL;
  if (!c->g.keys) return XCG_OK;
  DeviceGuard g(c->device);
  // The wipe is ordered behind the context's last work on the device; only a
  // pair, whose metadata lives on the host, waits for that work here.
  if (c->pair && ctx_wait(c) != XCG_OK) return XCG_EHIP;
  ctx_order(c, nullptr);
  // (the LRU clock keeps running: slots keep their last-reference times, which
  // must stay below every later batch's)
  if (c->pair && xcg_pair_state_clear(c->pair) != 0) return XCG_EHIP;
  // asynchronous: the context's later work waits for the wipe on the device
  // (ctx_order), host inspection calls wait for it (ctx_wait)
  const int rc = clear_cache(c->g, c->done_ev == nullptr);
  ctx_mark(c, nullptr);
  return rc;
}

int xcg_last_rounds(xcg_ctx* c) { return c ? c->last_rounds : -1; }

int xcg_ctx_flags(const xcg_ctx* c, uint32_t* flags) {
  if (!c || !flags) return XCG_EINVAL;
  *flags = c->flags;
  return XCG_OK;
}

namespace {
// A small pinned + device staging area for single-segment host calls.
int host_seg_call(xcg_ctx* c, uint64_t hash, const uint8_t* in_seg, uint8_t* out_seg, int mode, int32_t* res) {
  DeviceGuard g(c->device);
  int rc = ensure_cache(c);
  if (rc != XCG_OK) return rc;
  uint8_t* d_seg = nullptr;
  int32_t* d_res = nullptr;
  if (hipMalloc(&d_seg, XCG_SEGMENT_LENGTH) != hipSuccess || hipMalloc(&d_res, 4) != hipSuccess) {
    (void)hipFree(d_seg);
    return XCG_ENOMEM;
  }
  rc = XCG_OK;
  if (mode == 0) {   // lookup
    if (xcg_launch_cache_lookup(c->g.keys, c->g.vals, c->g.mask, c->g.pool, hash, d_seg, d_res, nullptr) != 0 ||
        hipMemcpy(res, d_res, 4, hipMemcpyDeviceToHost) != hipSuccess ||
        (*res && hipMemcpy(out_seg, d_seg, XCG_SEGMENT_LENGTH, hipMemcpyDeviceToHost) != hipSuccess))
      rc = XCG_EHIP;
  } else {           // enter (1) / replace (2)
    if (hipMemcpy(d_seg, in_seg, XCG_SEGMENT_LENGTH, hipMemcpyHostToDevice) != hipSuccess ||
        xcg_launch_cache_enter(c->g.keys, c->g.vals, c->g.mask, c->g.pool, c->g.nseg, c->g.seg_cap, c->g.filt,
                               c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask, hash, d_seg, mode == 2, d_res,
                               nullptr) != 0 ||
        hipMemcpy(res, d_res, 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = XCG_EHIP;
  }
  (void)hipFree(d_seg);
  (void)hipFree(d_res);
  return rc;
}
}  // namespace

namespace {
// Single-segment host calls on a bounded cache: lookup (a hit refreshes the
// entry, xcodec_cache.h:348-364) and enter (XCodecPipePair's <LEARN>:
// lookup, then replace if the bytes differ or enter, evicting at the limit,
// xcodec_pipe_pair.cc:311-327) -- as a one-reference batch through the LRU
// pass and commit (xcg_lru.hip).
int lru_host_call(xcg_ctx* c, uint64_t hash, const uint8_t* in_seg, uint8_t* out_seg, int enter, int32_t* found) {
  DeviceGuard g(c->device);
  int rc = ensure_cache(c);
  if (rc != XCG_OK) return rc;
  // device scratch: [0, 2048) new bytes, [2048, 4096) old bytes, then the batch
  uint8_t* m = nullptr;
  if (hipMalloc(&m, 8192) != hipSuccess) return XCG_ENOMEM;
  uint8_t* d_new = m;
  uint8_t* d_old = m + 2048;
  int32_t* d_res = (int32_t*)(m + 4096);
  rc = XCG_OK;
  do {
    if (xcg_launch_cache_lookup(c->g.keys, c->g.vals, c->g.mask, c->g.pool, hash, d_old, d_res, nullptr) != 0 ||
        hipMemcpy(found, d_res, 4, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = XCG_EHIP;
      break;
    }
    if (*found && out_seg && hipMemcpy(out_seg, d_old, XCG_SEGMENT_LENGTH, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = XCG_EHIP;
      break;
    }
    if (!*found && !enter) break;                   // a miss changes nothing
    if (enter && hipMemcpy(d_new, in_seg, XCG_SEGMENT_LENGTH, hipMemcpyHostToDevice) != hipSuccess) {
      rc = XCG_EHIP;
      break;
    }
    int32_t res = 0;
    if (enter && *found &&                          // replace (the table entry stays)
        (xcg_launch_cache_enter(c->g.keys, c->g.vals, c->g.mask, c->g.pool, c->g.nseg, c->g.seg_cap, c->g.filt,
                                c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask, hash, d_new, 1, d_res, nullptr) != 0 ||
         hipMemcpy(&res, d_res, 4, hipMemcpyDeviceToHost) != hipSuccess)) {
      rc = XCG_EHIP;
      break;
    }
    // the one-reference batch: chunk 0 = the new bytes; an ENTER (declaration
    // row 0) or a HIT at time 1
    struct {
      uint64_t chunk_off;
      uint32_t ev[4], decl[4];
      uint32_t nev, ndecl, need, pad;
      uint32_t ev_base[2], enter_base[2];
      uint32_t evslot[2];
      uint64_t evtime[2];
    } h{};
    const uint32_t lo = (uint32_t)hash, hi = (uint32_t)(hash >> 32);
    h.ev[0] = lo; h.ev[1] = hi;
    h.ev[2] = *found ? 1u : 0u;
    h.ev[3] = *found ? (1u << 30) : 0u;             // EV_HIT / EV_ENTER d = 0
    h.decl[0] = lo; h.decl[1] = hi;
    h.nev = 1;
    h.ndecl = *found ? 0u : 1u;
    uint8_t* d_h = m + 4608;
    if (hipMemcpy(d_h, &h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) {
      rc = XCG_EHIP;
      break;
    }
    auto at = [&](const void* field) { return d_h + ((const uint8_t*)field - (const uint8_t*)&h); };
    XcgLruState& L = c->lru;
    L.ev_base = (uint32_t*)at(h.ev_base);
    L.enter_base = (uint32_t*)at(h.enter_base);
    L.evslot = (uint32_t*)at(h.evslot);
    L.evtime = (uint64_t*)at(h.evtime);
    const LruBatch b{1u, d_new, (const uint64_t*)at(&h.chunk_off), at(h.decl), (const uint32_t*)at(&h.ndecl), 1u,
                     at(h.ev), (const uint32_t*)at(&h.nev), 1u, 0, (uint32_t*)at(&h.need), c->g.keys, c->g.vals,
                     c->g.mask, c->g.pool, c->g.nseg, c->g.filt, c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask,
                     c->d_status, 1u};
    if (xcg_lru_times(&b, &L, nullptr) != 0 || xcg_lru_commit(&b, &L, nullptr) != 0 ||
        hipStreamSynchronize(nullptr) != hipSuccess)
      rc = XCG_EHIP;
  } while (0);
  (void)hipFree(m);
  return rc;
}
}  // namespace

namespace {
uint64_t host_seg_hash(const uint8_t* w) {   // XCodecHash::hash, xcodec/xcodec_hash.h:166-174
  uint32_t s1 = 0, s2 = 0, b1 = 0, b2 = 0;
  for (uint32_t k = 0; k < XCG_SEGMENT_LENGTH; ++k) {
    s1 += (uint32_t)w[k] + 1u;
    s2 += s1;
    b1 += w[k] ? (uint32_t)__builtin_ctz(w[k]) + 1u : 0u;
    b2 += b1;
  }
  return ((uint64_t)((b1 << 16) + b2) << 36) + (uint64_t)((s1 << 20) + s2);
}

// Single-segment host calls on a pair: a one-op decode batch that leaves the
// BACKREF window alone.  A lookup is <REF hash> (XCodecCachePair::lookup, with
// its LRU use / disk touch / promotion, xcodec_cache.h:208-230); an enter is
// <EXTRACT seg> -- lookup, then nothing (same bytes), replace (other bytes) or
// enter (absent), exactly <LEARN>'s sequence (xcodec_pipe_pair.cc:311-327).
int pair_host_call(xcg_ctx* c, uint64_t hash, const uint8_t* in_seg, uint8_t* out_seg, int32_t* found) {
  uint8_t op[2 + XCG_SEGMENT_LENGTH];
  uint32_t len;
  op[0] = 0xF1;
  if (in_seg) {
    op[1] = 0x01;
    memcpy(op + 2, in_seg, XCG_SEGMENT_LENGTH);
    len = 2 + XCG_SEGMENT_LENGTH;
  } else {
    op[1] = 0x02;
    for (int k = 0; k < 8; ++k) op[2 + k] = (uint8_t)(hash >> (56 - 8 * k));
    len = 10;
  }
  const uint64_t off = 0;
  uint64_t ooff = 0, olen = 0, cons = 0, unk = 0;
  int32_t st = 0;
  uint32_t nunk = 0;
  uint8_t out[XCG_SEGMENT_LENGTH];
  c->no_window = true;
  const int rc = xcg_decode_host(c, op, len, &off, &len, 1, out, sizeof out, &ooff, &olen, &st, &cons, &unk, 1, &nunk);
  c->no_window = false;
  if (rc != XCG_OK) return rc;
  if (st < 0) return XCG_EHIP;
  *found = st == 0 && olen == XCG_SEGMENT_LENGTH;
  if (*found && out_seg) memcpy(out_seg, out, XCG_SEGMENT_LENGTH);
  return XCG_OK;
}
}  // namespace

int xcg_cache_lookup_host(xcg_ctx* c, uint64_t hash, uint8_t* seg_out) {
  if (!c || !seg_out) return XCG_EINVAL;
  if (c->pair) {
    int32_t found = 0;
    const int rc = pair_host_call(c, hash, nullptr, seg_out, &found);
    return rc != XCG_OK ? rc : (found ? XCG_OK : XCG_ENOENT);
  }
  if (c->bounded) {
    int32_t found = 0;
    const int rc = lru_host_call(c, hash, nullptr, seg_out, 0, &found);
    return rc != XCG_OK ? rc : (found ? XCG_OK : XCG_ENOENT);
  }
  int32_t found = 0;
  const int rc = host_seg_call(c, hash, nullptr, seg_out, 0, &found);
  if (rc != XCG_OK) return rc;
  return found ? XCG_OK : XCG_ENOENT;
}

int xcg_cache_enter_host(xcg_ctx* c, uint64_t hash, const uint8_t* seg) {
  if (!c || !seg) return XCG_EINVAL;
  if (c->pair) {
    if (host_seg_hash(seg) != hash) return XCG_EINVAL;   // (a pair names a segment by its own hash)
    int32_t found = 0;
    return pair_host_call(c, hash, seg, nullptr, &found);
  }
  if (c->bounded) {
    int32_t found = 0;
    return lru_host_call(c, hash, seg, nullptr, 1, &found);
  }
  int32_t res = 0;
  const int rc = host_seg_call(c, hash, seg, nullptr, 1, &res);
  if (rc != XCG_OK) return rc;
  return res == -2 ? XCG_EOVERFLOW : XCG_OK;
}

int xcg_last_declarations(xcg_ctx* c, uint32_t chunk, uint64_t* h_hash, uint32_t* h_pos, uint32_t cap,
                          uint32_t* h_count) {
  if (!c || !h_count || !c->bs.decl) return XCG_EINVAL;
  if (c->bounded || c->pair) {                         // rows of the last sub-batch only
    const uint32_t base = c->pair ? xcg_pair_state_last_base(c->pair) : c->lru.last_base;
    if (chunk < base) return XCG_ENOTSUP;
    chunk -= base;
  }
  if (chunk >= c->bs.n_cap) return XCG_EINVAL;
  DeviceGuard g(c->device);
  uint32_t nd = 0;
  if (ctx_wait(c) != XCG_OK ||
      hipMemcpy(&nd, c->bs.ndecl + chunk, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return XCG_EHIP;
  *h_count = nd;
  const uint32_t k = nd < cap ? nd : cap;
  if (k == 0) return XCG_OK;
  std::vector<uint32_t> buf(4ull * k);
  if (hipMemcpy(buf.data(), (const uint8_t*)c->bs.decl + 16ull * chunk * c->bs.last_maxd, 16ull * k,
                hipMemcpyDeviceToHost) != hipSuccess)
    return XCG_EHIP;
  for (uint32_t i = 0; i < k; ++i) {
    if (h_hash) h_hash[i] = ((uint64_t)buf[4 * i + 1] << 32) | buf[4 * i];
    if (h_pos) h_pos[i] = buf[4 * i + 2];
  }
  return XCG_OK;
}

int xcg_last_references(xcg_ctx* c, uint32_t chunk, uint64_t* h_hash, uint32_t* h_kind, uint32_t* h_ref,
                        uint32_t cap, uint32_t* h_count) {
  if (!c || !h_count) return XCG_EINVAL;
  if (!(c->bounded || c->pair) || !c->bs.ev) return XCG_ENOTSUP;
  const uint32_t base = c->pair ? xcg_pair_state_last_base(c->pair) : c->lru.last_base;
  if (chunk < base) return XCG_ENOTSUP;
  chunk -= base;
  if (chunk >= c->bs.n_cap) return XCG_EINVAL;
  DeviceGuard g(c->device);
  uint32_t ne = 0;
  if (ctx_wait(c) != XCG_OK || hipMemcpy(&ne, c->bs.nev + chunk, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return XCG_EHIP;
  if (ne > c->bs.maxe) return XCG_EOVERFLOW;
  *h_count = ne;
  std::vector<uint32_t> buf(4ull * ne);
  if (ne && hipMemcpy(buf.data(), (const uint8_t*)c->bs.ev + 16ull * chunk * c->bs.maxe, 16ull * ne,
                      hipMemcpyDeviceToHost) != hipSuccess)
    return XCG_EHIP;
  std::vector<uint32_t> order(ne);
  for (uint32_t i = 0; i < ne; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return buf[4 * a + 2] < buf[4 * b + 2]; });
  const uint32_t k = ne < cap ? ne : cap;
  for (uint32_t j = 0; j < k; ++j) {
    const uint32_t* e = &buf[4ull * order[j]];
    if (h_hash) h_hash[j] = ((uint64_t)e[1] << 32) | e[0];
    if (h_kind) h_kind[j] = e[3] >> 30;          // EV_ENTER 0, EV_HIT 1, EV_GHIT 2, EV_GMISS 3 (xcg_cache.h)
    if (h_ref) h_ref[j] = e[3] & ((1u << 30) - 1u);
  }
  return XCG_OK;
}

int xcg_debug_restart_counts(xcg_ctx* c, uint64_t* resumed, uint64_t* spliced) {
  if (!c || !resumed || !spliced) return XCG_EINVAL;
  *resumed = *spliced = 0;
  if (!c->bs.b_count) return XCG_OK;
  DeviceGuard g(c->device);
  uint32_t v[4] = {0, 0, 0, 0};
  if (ctx_wait(c) != XCG_OK || hipMemcpy(v, c->bs.b_count, 16, hipMemcpyDeviceToHost) != hipSuccess) return XCG_EHIP;
  *resumed = v[2];
  *spliced = v[3];
  return XCG_OK;
}

int xcg_debug_cache_dump(xcg_ctx* c, uint32_t* h_filt, uint32_t* h_ftab, uint64_t ftab_words, uint32_t* h_fmask) {
  if (!c || !c->g.keys) return XCG_EINVAL;
  DeviceGuard g(c->device);
  *h_fmask = c->g.fmask;
  if (ctx_wait(c) != XCG_OK) return XCG_EHIP;
  if (h_filt && hipMemcpy(h_filt, c->g.filt, 4ull * FILT_WORDS, hipMemcpyDeviceToHost) != hipSuccess) return XCG_EHIP;
  const uint64_t tw = 4ull * (c->g.fmask + 1);
  if (h_ftab && hipMemcpy(h_ftab, c->g.ftab, 4ull * (ftab_words < tw ? ftab_words : tw), hipMemcpyDeviceToHost) !=
                    hipSuccess)
    return XCG_EHIP;
  return XCG_OK;
}

int xcg_ctx_status(xcg_ctx* c) {
  if (!c) return XCG_EINVAL;
  DeviceGuard g(c->device);
  int32_t st = 0;
  if (ctx_wait(c) != XCG_OK ||
      hipMemcpyAsync(c->h_status, c->d_status, sizeof st, hipMemcpyDeviceToHost, nullptr) != hipSuccess ||
      hipStreamSynchronize(nullptr) != hipSuccess)
    return XCG_EHIP;
  st = *c->h_status;
  if (st && getenv("XCG_STATUS_DEBUG")) fprintf(stderr, "xcg: context status word %#x\n", (unsigned)st);
  return st ? XCG_EOVERFLOW : XCG_OK;
}

}  // extern "C"

namespace {
int encode_batch_impl(xcg_ctx* c, int semantics, const uint8_t* d_in, const uint64_t* d_chunk_off,
                      const uint32_t* d_chunk_len, uint32_t n, uint32_t max_chunk_len, uint8_t* d_out,
                      const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_stats, void* stream) {
  if (!c) return XCG_EINVAL;
  if (n == 0) return XCG_OK;
  if (!d_in || !d_chunk_off || !d_chunk_len || !d_out || !d_out_off || !d_out_len) return XCG_EINVAL;
  if (semantics != XCG_SEM_INDEPENDENT && semantics != XCG_SEM_STREAM) return XCG_EINVAL;
  if (max_chunk_len > (1u << 19)) return XCG_EINVAL;
  DeviceGuard g(c->device);
  ctx_order(c, (hipStream_t)stream);
  // A null cache has no state to carry: both semantics are the same pass.
  if (semantics == XCG_SEM_STREAM && !(c->flags & XCG_FLAG_NULLCACHE)) {
    // declaration slots per chunk: a chunk of L bytes declares at most L / 2048
    const uint32_t maxd = max_chunk_len / XCG_SEGMENT_LENGTH + 1;
    int rc = ensure_cache(c);
    if (rc == XCG_OK) rc = ensure_scratch(c, n, maxd);
    if (rc != XCG_OK) return rc;
    c->bs.last_maxd = maxd;
    XcgStreamArgs a{d_in, d_chunk_off, d_chunk_len, n, c->flags, d_out, d_out_off, d_out_len, d_stats,
                    c->d_status, c->g.keys, c->g.vals, c->g.mask, c->g.pool, c->g.nseg, c->g.seg_cap,
                    c->g.filt, c->g.ftab, c->g.fmask, c->bs.b_keys, c->bs.b_vals, c->bs.b_mask,
                    c->bs.r_filt, c->bs.r_ftab, c->bs.decl, c->bs.ndecl, maxd, c->bs.changed, c->bs.h_changed,
                    c->g.gfilt, c->bs.r_gfilt, c->g.gmask, c->bs.bcount, c->bs.b2_keys, c->bs.b2_vals,
                    c->bs.r_keys, c->bs.r_vals, c->bs.r_mask, c->bs.hits, c->bs.nhits, c->bs.maxh, c->bs.need,
                    c->bs.vflags, c->bs.h_vflags, 0, nullptr, nullptr, nullptr, nullptr, 0u, 0, 0, 0};
    // Seed the rounds with the chunks' 2048-byte tilings instead of a parse
    // round 0 when the last batch declared segments (cold / growing caches);
    // a warm cache's all-REF batches keep round 0, which then is all they need.
    const int mode = __atomic_load_n(&g_stream_seed, __ATOMIC_RELAXED);
    a.seed = mode < 0 ? (c->seed_next ? 1 : 0) : mode;
    uint32_t decls = ~0u;
    a.decls_out = &decls;
    int rounds = 0;
    a.a_keys = c->bs.a_keys;
    a.a_vals = c->bs.a_vals;
    a.a_bits = getenv("XCG_NO_APROBE") ? nullptr : c->bs.a_bits;
    a.flags_ev = c->flags_ev;
    a.s_fold = c->bs.s_fold;
    a.s_work = c->bs.s_work;
    a.s_info = c->bs.s_info;
    a.s_rows = c->bs.s_rows;
    a.s_qcnt = c->bs.s_qcnt;
    a.s_qkeys = c->bs.s_qkeys;
    if (c->pair || c->bounded) {
      BatchScratch& b = c->bs;
      a.eo = b.eo; a.bad_t = b.bad_t; a.bad_hi = b.bad_hi; a.bslot = b.bslot; a.b_count = b.b_count;
      a.b_slots = b.b_slots; a.b_ev = b.b_ev; a.b_eo = b.b_eo; a.b_hits = b.b_hits; a.b_cnt = b.b_cnt;
      a.b_out = b.b_out; a.b_stride = b.b_stride; a.splice = b.splice;
      a.restart = getenv("XCG_NO_RESTART") ? 0 : 1;
    }
    if (c->pair) {
      a.ev = c->bs.ev;
      a.nev = c->bs.nev;
      a.maxe = c->bs.maxe;
      rc = xcg_pair_encode_stream(&a, c->pair, &rounds, (hipStream_t)stream);
      c->last_rounds = rounds;
      return rc == 0 ? XCG_OK : (rc == -75 ? XCG_EOVERFLOW : (rc == -95 ? XCG_ENOTSUP : XCG_EHIP));
    }
    if (c->bounded) {
      a.ev = c->bs.ev;
      a.nev = c->bs.nev;
      a.maxe = c->bs.maxe;
      c->lru.ev_base = c->bs.ev_base;
      c->lru.enter_base = c->bs.enter_base;
      c->lru.evslot = c->bs.ev_slot;
      c->lru.evtime = c->bs.ev_time;
      rc = xcg_lru_encode_stream(&a, &c->lru, &rounds, (hipStream_t)stream);
      c->last_rounds = rounds;
      return rc == 0 ? XCG_OK : (rc == -75 ? XCG_EOVERFLOW : (rc == -95 ? XCG_ENOTSUP : XCG_EHIP));
    }
    rc = xcg_launch_encode_stream(&a, &rounds, (hipStream_t)stream);
    if (decls != ~0u) c->seed_next = decls > 0;
    c->last_rounds = rounds;
    return rc == 0 ? XCG_OK : (rc == -75 ? XCG_EOVERFLOW : XCG_EHIP);
  }
  // A fresh bounded cache per chunk evicts nothing while the chunk's
  // declarations fit the limit (at most max_chunk_len / 2048 of them).
  if (c->bounded && max_chunk_len / XCG_SEGMENT_LENGTH > c->lru.C) return XCG_ENOTSUP;
  if (c->pair && max_chunk_len / XCG_SEGMENT_LENGTH > c->pair_C) return XCG_ENOTSUP;
  int rc = xcg_launch_encode_independent(d_in, d_chunk_off, d_chunk_len, n, max_chunk_len, c->flags, d_out,
                                         d_out_off, d_out_len, d_stats, c->d_status, (hipStream_t)stream);
  return rc == 0 ? XCG_OK : (rc == -22 ? XCG_EINVAL : XCG_EHIP);
}
}  // namespace

extern "C" {

int xcg_encode_batch(xcg_ctx* c, int semantics, const uint8_t* d_in, const uint64_t* d_chunk_off,
                     const uint32_t* d_chunk_len, uint32_t n, uint32_t max_chunk_len, uint8_t* d_out,
                     const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_stats, void* stream) {
  const int rc = encode_batch_impl(c, semantics, d_in, d_chunk_off, d_chunk_len, n, max_chunk_len, d_out, d_out_off,
                                   d_out_len, d_stats, stream);
  if (c) {
    DeviceGuard g(c->device);
    ctx_mark(c, (hipStream_t)stream);
  }
  return rc;
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
  // staging (kept by the context): [off n][oo n][ol n][len n] | input | output slots
  const size_t meta = align256(28ull * n), inb = align256(in_len ? in_len : 1), outb = align256(out_cap ? out_cap : 1);
  int rc = ensure_stage(c, meta + inb + outb, meta + inb + outb);
  if (rc != XCG_OK) return rc;
  uint8_t* hm = c->stage_h;
  uint8_t* dm = c->stage_d;
  memcpy(hm, h_chunk_off, 8ull * n);
  memcpy(hm + 8ull * n, h_out_off, 8ull * n);
  memcpy(hm + 24ull * n, h_chunk_len, 4ull * n);
  memcpy(hm + meta, h_in, in_len);
  const hipStream_t st = c->call_st;
  const uint64_t* d_off = (const uint64_t*)dm;
  const uint64_t* d_oo = (const uint64_t*)(dm + 8ull * n);
  uint64_t* d_ol = (uint64_t*)(dm + 16ull * n);
  const uint32_t* d_len = (const uint32_t*)(dm + 24ull * n);
  uint8_t* d_out = dm + meta + inb;
  if (hipMemcpyAsync(dm, hm, meta + in_len, hipMemcpyHostToDevice, st) != hipSuccess) return XCG_EHIP;
  rc = xcg_encode_batch(c, semantics, dm + meta, d_off, d_len, n, maxlen, d_out, d_oo, d_ol, nullptr, st);
  if (rc != XCG_OK) return rc;
  uint64_t* ol = (uint64_t*)(hm + 16ull * n);
  if (hipMemcpyAsync(ol, d_ol, 8ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(c->h_status, c->d_status, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return XCG_EHIP;
  if (*c->h_status) return XCG_EOVERFLOW;
  // only the bytes each slot holds come back
  uint8_t* ho = hm + meta + inb;
  for (uint32_t i = 0; i < n; ++i) {
    h_out_len[i] = ol[i];
    if (ol[i] && hipMemcpyAsync(ho + h_out_off[i], d_out + h_out_off[i], ol[i], hipMemcpyDeviceToHost, st) != hipSuccess)
      return XCG_EHIP;
  }
  if (hipStreamSynchronize(st) != hipSuccess) return XCG_EHIP;
  for (uint32_t i = 0; i < n; ++i)
    if (ol[i]) memcpy(h_out + h_out_off[i], ho + h_out_off[i], ol[i]);
  return XCG_OK;
}

int xcg_encode_call(xcg_ctx* c, const uint8_t* h_in, uint32_t len, uint8_t* h_out, uint64_t out_cap,
                    uint64_t* h_out_len, uint64_t* h_decl_hash, uint32_t* h_decl_pos, uint32_t decl_cap,
                    uint32_t* h_ndecl, uint64_t* h_ref_hash, uint32_t* h_ref_kind, uint32_t* h_ref_idx, uint32_t ref_cap,
                    uint32_t* h_nref) {
  if (!c || !h_out_len || !h_ndecl || !h_nref || (len && (!h_in || !h_out))) return XCG_EINVAL;
  *h_out_len = 0;
  *h_ndecl = 0;
  *h_nref = (c->bounded || c->pair) ? 0u : XCG_NO_REFERENCES;
  if (len == 0) return XCG_OK;
  if (out_cap < xcg_encode_bound(len) || len > (1u << 19)) return XCG_EINVAL;
  DeviceGuard g(c->device);
  const bool nullc = (c->flags & XCG_FLAG_NULLCACHE) != 0;
  const bool refs = (c->bounded || c->pair) && !nullc;
  const uint32_t maxd = len / XCG_SEGMENT_LENGTH + 1;
  // staging: device [off 8][oo 8][ol 8][len 4] | input | output slot;
  //          host   the same head, then [ndecl 4][nev 4] | decl rows | event rows | output
  const uint64_t bound = xcg_encode_bound(len);
  const size_t inb = align256(len), outb = align256(bound);
  const size_t rows_d = align256(16ull * maxd);
  size_t rows_e = 0;
  if (refs) {
    int rc0 = ensure_cache(c);
    if (rc0 == XCG_OK) rc0 = ensure_scratch(c, 1, maxd);
    if (rc0 != XCG_OK) return rc0;
    rows_e = align256(16ull * c->bs.maxe);
  }
  int rc = ensure_stage(c, 256 + inb + outb, 256 + inb + 256 + rows_d + rows_e + outb);
  if (rc != XCG_OK) return rc;
  uint8_t* hm = c->stage_h;
  uint8_t* dm = c->stage_d;
  uint64_t* hmeta = (uint64_t*)hm;
  hmeta[0] = 0;                                      // chunk offset
  hmeta[1] = 0;                                      // output slot offset
  hmeta[2] = 0;
  *(uint32_t*)(hm + 24) = len;
  memcpy(hm + 256, h_in, len);
  const hipStream_t st = c->call_st;
  uint8_t* d_out = dm + 256 + inb;
  if (hipMemcpyAsync(dm, hm, 256 + len, hipMemcpyHostToDevice, st) != hipSuccess) return XCG_EHIP;
  rc = xcg_encode_batch(c, XCG_SEM_STREAM, dm + 256, (const uint64_t*)dm, (const uint32_t*)(dm + 24), 1, len, d_out,
                        (const uint64_t*)(dm + 8), (uint64_t*)(dm + 16), nullptr, st);
  if (rc != XCG_OK) return rc;
  // everything the call produced, back in one synchronisation
  uint8_t* hres = hm + 256 + inb;
  uint32_t* hcnt = (uint32_t*)hres;                  // [0] ndecl, [1] nev
  uint8_t* hdecl = hres + 256;
  uint8_t* hev = hdecl + rows_d;
  uint8_t* hout = hev + rows_e;
  const bool stream_rows = !nullc;                   // (a null cache parses without declaration rows)
  if (hipMemcpyAsync(hm + 16, dm + 16, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(c->h_status, c->d_status, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(hout, d_out, bound, hipMemcpyDeviceToHost, st) != hipSuccess)
    return XCG_EHIP;
  if (stream_rows && (hipMemcpyAsync(hcnt, c->bs.ndecl, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                      hipMemcpyAsync(hdecl, c->bs.decl, 16ull * maxd, hipMemcpyDeviceToHost, st) != hipSuccess))
    return XCG_EHIP;
  if (refs && (hipMemcpyAsync(hcnt + 1, c->bs.nev, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipMemcpyAsync(hev, c->bs.ev, 16ull * c->bs.maxe, hipMemcpyDeviceToHost, st) != hipSuccess))
    return XCG_EHIP;
  if (hipStreamSynchronize(st) != hipSuccess) return XCG_EHIP;
  if (*c->h_status) return XCG_EOVERFLOW;
  const uint64_t olen = hmeta[2];
  if (olen > bound) return XCG_EHIP;
  memcpy(h_out, hout, olen);
  *h_out_len = olen;
  if (stream_rows) {
    const uint32_t nd = hcnt[0];
    *h_ndecl = nd;
    const uint32_t k = nd < decl_cap ? nd : decl_cap;
    const uint32_t* r = (const uint32_t*)hdecl;
    for (uint32_t i = 0; i < k; ++i) {
      if (h_decl_hash) h_decl_hash[i] = ((uint64_t)r[4 * i + 1] << 32) | r[4 * i];
      if (h_decl_pos) h_decl_pos[i] = r[4 * i + 2];
    }
  }
  if (refs) {
    const uint32_t ne = hcnt[1];
    if (ne > c->bs.maxe) return XCG_EOVERFLOW;
    *h_nref = ne;
    const uint32_t* e = (const uint32_t*)hev;
    std::vector<uint32_t> order(ne);
    for (uint32_t i = 0; i < ne; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return e[4 * a + 2] < e[4 * b + 2]; });
    const uint32_t k = ne < ref_cap ? ne : ref_cap;
    for (uint32_t j = 0; j < k; ++j) {
      const uint32_t* v = e + 4ull * order[j];
      if (h_ref_hash) h_ref_hash[j] = ((uint64_t)v[1] << 32) | v[0];
      if (h_ref_kind) h_ref_kind[j] = v[3] >> 30;
      if (h_ref_idx) h_ref_idx[j] = v[3] & ((1u << 30) - 1u);
    }
  }
  return XCG_OK;
}

}  // extern "C"

namespace {
int decode_batch_impl(xcg_ctx* c, const uint8_t* d_enc, const uint64_t* d_chunk_off, const uint32_t* d_chunk_len,
                      uint32_t n, uint32_t max_chunk_len, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off,
                      uint64_t* d_out_len, int32_t* d_chunk_status, uint64_t* d_consumed, uint64_t* h_unknown,
                      uint32_t unknown_cap, uint32_t* h_nunknown, uint64_t* h_total_out, void* stream) {
  if (!c || (n && (!d_enc || !d_chunk_off || !d_chunk_len || !d_out_off || !d_out_len || !d_chunk_status ||
                   !d_consumed)))
    return XCG_EINVAL;
  if (h_nunknown) *h_nunknown = 0;
  if (h_total_out) *h_total_out = 0;
  if (n == 0) return XCG_OK;
  // a bounded or pair batch numbers its ops by (chunk << 21 | offset)
  if ((c->bounded || c->pair) && max_chunk_len >= (1u << 21)) return XCG_EINVAL;
  DeviceGuard g(c->device);
  ctx_order(c, (hipStream_t)stream);
  int rc = ensure_cache(c);
  if (rc == XCG_OK) rc = ensure_dscratch(c, (uint64_t)n * (max_chunk_len / 2050 + 1));
  if (rc == XCG_OK) rc = ensure_dchunks(c, n);
  if (rc == XCG_OK && !c->cur_win) {
    rc = window_alloc(c->device, &c->own_win);
    c->cur_win = c->own_win;
  }
  if (rc != XCG_OK) return rc;
  xcg_window* w = c->cur_win;
  XcgDecodeArgs a{d_enc, d_chunk_off, d_chunk_len, n, d_out, out_cap, d_out_off, d_out_len, d_chunk_status,
                  d_consumed, c->d_status, c->g.keys, c->g.vals, c->g.mask, c->g.pool, c->g.nseg, c->g.seg_cap,
                  c->g.filt, c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask, c->ds.x_keys, c->ds.x_vals, c->ds.x_latest, c->ds.x_cap - 1,
                  c->ds.u_keys, c->ds.unknown, c->ds.unknown_pos, c->ds.nunknown, UNKNOWN_CAP, c->ds.scratch, c->ds.h_scratch,
                  c->ds.chunk_tmp, c->ds.d_tail, w->hash, w->seg, w->count, c->bounded ? &c->lru : nullptr,
                  max_chunk_len / 2050 + 1, c->pair, c->no_window ? 1 : 0};
  if (c->pair) {
    const PairGpu G{d_enc, d_chunk_off, nullptr, 0u, c->g.pool, c->g.keys, c->g.vals, c->g.mask, c->g.filt,
                    c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask, c->g.nseg, c->d_status};
    if (xcg_pair_sync(c->pair, &G, (hipStream_t)stream)) return XCG_EHIP;
  }
  uint64_t total = 0, blockp = 0, berr = 0;
  uint32_t nunk = 0;
  const int lrc = xcg_launch_decode(&a, &total, &blockp, &berr, &nunk, (hipStream_t)stream);
  if (h_total_out) *h_total_out = total;
  if (lrc == -75) return XCG_EOVERFLOW;
  if (lrc == -95) return XCG_ENOTSUP;
  if (lrc != 0) return XCG_EHIP;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return XCG_EHIP;
  // status word and the declare count, by async copies into pinned memory
  // (a synchronous 4-byte hipMemcpy costs milliseconds here)
  if (hipMemcpyAsync(c->h_status, c->d_status, 4, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
      hipMemcpyAsync(c->ds.h_scratch + 7, c->ds.scratch + 5, 8, hipMemcpyDeviceToHost, (hipStream_t)stream) !=
          hipSuccess ||
      hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
    return XCG_EHIP;
  const int32_t st = *c->h_status;
  const uint64_t t_end = c->ds.h_scratch[7];
  if (!c->no_window) w->count += t_end;               // declares made: the window cursor advances
  if (st & (1 << 9)) {
    (void)hipMemsetAsync(c->d_status, 0, 4, (hipStream_t)stream);
    return XCG_ENOTSUP;
  }
  if (nunk > UNKNOWN_CAP) return XCG_EOVERFLOW;     // more distinct unknown hashes than the set holds
  if (nunk && blockp < berr) {
    // XCodecDecoder::decode_skim (xcodec/xcodec_decoder.cc:196-272): every REF
    // from the blocking point on that cannot resolve, as a sorted set.  The
    // batch's frames are one buffered stream (a pipe pair appends each FRAME
    // to the decoder's input, xcodec/xcodec_pipe_pair.cc:425-483), so the skim
    // runs to the end of the batch.  (A BACKREF error first: decode() is false,
    // no ASK.)
    const uint32_t m = nunk < UNKNOWN_CAP ? nunk : UNKNOWN_CAP;
    std::vector<uint64_t> hs(m);
    if (hipMemcpyAsync(hs.data(), c->ds.unknown, 8ull * m, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
      return XCG_EHIP;
    std::sort(hs.begin(), hs.end());
    hs.erase(std::unique(hs.begin(), hs.end()), hs.end());
    const uint32_t k = (uint32_t)hs.size() < unknown_cap ? (uint32_t)hs.size() : unknown_cap;
    if (h_unknown) memcpy(h_unknown, hs.data(), 8ull * k);
    if (h_nunknown) *h_nunknown = k;
  }
  return XCG_OK;
}
}  // namespace

extern "C" {

int xcg_decode_batch(xcg_ctx* c, const uint8_t* d_enc, const uint64_t* d_chunk_off, const uint32_t* d_chunk_len,
                     uint32_t n, uint32_t max_chunk_len, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off,
                     uint64_t* d_out_len, int32_t* d_chunk_status, uint64_t* d_consumed, uint64_t* h_unknown,
                     uint32_t unknown_cap, uint32_t* h_nunknown, uint64_t* h_total_out, void* stream) {
  const int rc = decode_batch_impl(c, d_enc, d_chunk_off, d_chunk_len, n, max_chunk_len, d_out, out_cap, d_out_off,
                                   d_out_len, d_chunk_status, d_consumed, h_unknown, unknown_cap, h_nunknown,
                                   h_total_out, stream);
  if (c) {
    DeviceGuard g(c->device);
    ctx_mark(c, (hipStream_t)stream);
  }
  return rc;
}

int xcg_window_create(xcg_ctx* c, xcg_window** out) {
  if (!c || !out) return XCG_EINVAL;
  DeviceGuard g(c->device);
  return window_alloc(c->device, out);
}

void xcg_window_destroy(xcg_window* w) {
  if (!w) return;
  DeviceGuard g(w->device);
  window_free(w);
}

int xcg_decode_set_window(xcg_ctx* c, xcg_window* w) {
  if (!c) return XCG_EINVAL;
  c->cur_win = w ? w : c->own_win;
  return XCG_OK;
}

int xcg_decode_host(xcg_ctx* c, const uint8_t* h_enc, uint64_t enc_len, const uint64_t* h_chunk_off,
                    const uint32_t* h_chunk_len, uint32_t n, uint8_t* h_out, uint64_t out_cap, uint64_t* h_out_off,
                    uint64_t* h_out_len, int32_t* h_chunk_status, uint64_t* h_consumed, uint64_t* h_unknown,
                    uint32_t unknown_cap, uint32_t* h_nunknown) {
  if (!c || (n && (!h_enc || !h_chunk_off || !h_chunk_len || !h_out_off || !h_out_len || !h_chunk_status ||
                   !h_consumed)))
    return XCG_EINVAL;
  if (n == 0) return XCG_OK;
  uint32_t maxlen = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (h_chunk_off[i] + h_chunk_len[i] > enc_len) return XCG_EINVAL;
    if (h_chunk_len[i] > maxlen) maxlen = h_chunk_len[i];
  }
  DeviceGuard g(c->device);
  // staging (kept by the context): [off n][oo n][ol n][cons n][len n][status n] | input | output
  const size_t meta = align256(40ull * n), inb = align256(enc_len ? enc_len : 1), outb = align256(out_cap ? out_cap : 1);
  int rc = ensure_stage(c, meta + inb + outb, meta + inb + outb);
  if (rc != XCG_OK) return rc;
  uint8_t* hm = c->stage_h;
  uint8_t* dm = c->stage_d;
  memcpy(hm, h_chunk_off, 8ull * n);
  memcpy(hm + 32ull * n, h_chunk_len, 4ull * n);
  memcpy(hm + meta, h_enc, enc_len);
  const hipStream_t st = c->call_st;
  uint64_t* d_oo = (uint64_t*)(dm + 8ull * n);
  uint64_t* d_ol = (uint64_t*)(dm + 16ull * n);
  uint64_t* d_cons = (uint64_t*)(dm + 24ull * n);
  int32_t* d_st = (int32_t*)(dm + 36ull * n);
  uint8_t* d_out = dm + meta + inb;
  if (hipMemcpyAsync(dm, hm, meta + enc_len, hipMemcpyHostToDevice, st) != hipSuccess) return XCG_EHIP;
  uint64_t total = 0;
  rc = xcg_decode_batch(c, dm + meta, (const uint64_t*)dm, (const uint32_t*)(dm + 32ull * n), n, maxlen, d_out,
                        out_cap, d_oo, d_ol, d_st, d_cons, h_unknown, unknown_cap, h_nunknown, &total, st);
  if (rc != XCG_OK) return rc;
  uint8_t* ho = hm + meta + inb;
  const uint64_t nout = total < out_cap ? total : out_cap;
  if (hipMemcpyAsync(hm + 8ull * n, dm + 8ull * n, 24ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(hm + 36ull * n, d_st, 4ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      (nout && hipMemcpyAsync(ho, d_out, nout, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess)
    return XCG_EHIP;
  memcpy(h_out_off, hm + 8ull * n, 8ull * n);
  memcpy(h_out_len, hm + 16ull * n, 8ull * n);
  memcpy(h_consumed, hm + 24ull * n, 8ull * n);
  memcpy(h_chunk_status, hm + 36ull * n, 4ull * n);
  if (nout) memcpy(h_out, ho, nout);
  return XCG_OK;
}

}  // extern "C"

extern "C" int xcg_launch_decode_small(const uint8_t*, uint32_t, uint64_t*, uint64_t*, uint32_t, uint8_t*, uint32_t*,
                                       uint32_t, uint32_t*, uint32_t*, uint32_t, uint32_t*, uint32_t, int32_t*, void*,
                                       uint32_t, uint8_t*, uint64_t, uint64_t*, uint8_t*, uint64_t, uint64_t*,
                                       uint64_t*, uint32_t*, uint32_t, hipStream_t);
extern "C" uint64_t xcg_decode_small_scratch(uint32_t ops_cap);
extern "C" uint32_t xcg_decode_small_lds_in(void);
extern "C" uint32_t xcg_decode_small_res_words(void);
extern "C" uint32_t xcg_decode_small_phases(void);

// Diagnostics: with XCG_DECODE_PHASES set, every one-launch decode() records
// clock stamps at its phase boundaries (decode_small_kernel); the sums of the
// phase durations and the call count come back through
// xcg_debug_decode_phases.  (Costs a synchronous copy per call.)
namespace {
std::mutex g_dph_mu;
std::vector<double> g_dph_sum;
uint32_t g_dph_calls = 0;
bool dphase_on() {
  static const bool on = getenv("XCG_DECODE_PHASES") != nullptr;
  return on;
}
}  // namespace

namespace {
bool getenv_flag_no_zc() {
  static const bool off = getenv("XCG_NO_ZEROCOPY") != nullptr;
  return off;
}

// The results words of one decode_small_kernel launch -> the call's outputs.
// XCG_ENOTSUP: the kernel declined (fallback); nothing was written.
int decode_call_results(xcg_window* w, const uint64_t* h_res, uint32_t rw, const uint8_t* h_o, uint8_t* h_out,
                        uint64_t* h_out_len, uint64_t* h_consumed, int32_t* h_status, uint64_t* h_unknown,
                        uint32_t unknown_cap, uint32_t* h_nunknown, uint64_t* h_extract_hash, uint32_t extract_cap,
                        uint32_t* h_nextract) {
  if ((uint32_t)h_res[rw - 1]) return XCG_EOVERFLOW;   // (cache capacity: the sticky word)
  if (h_res[5] == 2) {
    *h_out_len = h_res[7];
    return XCG_EOVERFLOW;
  }
  if (h_res[5] != 0) return XCG_ENOTSUP;
  const uint64_t ol = h_res[0];
  memcpy(h_out, h_o, ol);
  *h_out_len = ol;
  *h_consumed = h_res[1];
  *h_status = (int32_t)(int64_t)h_res[2];
  w->count += h_res[3];
  const uint32_t nu = (uint32_t)h_res[4];
  uint64_t* u = (uint64_t*)alloca(8ull * (nu ? nu : 1));
  memcpy(u, h_res + 8, 8ull * nu);
  std::sort(u, u + nu);
  const uint32_t ku = nu < unknown_cap ? nu : unknown_cap;
  if (h_unknown && ku) memcpy(h_unknown, u, 8ull * ku);
  *h_nunknown = ku;
  const uint32_t ne = (uint32_t)h_res[6];
  if (ne <= extract_cap && ne <= 1024) {
    if (ne && h_extract_hash) memcpy(h_extract_hash, h_res + 8 + 2048, 8ull * ne);
    *h_nextract = ne;
  }
  return XCG_OK;
}

// One decode() in one launch with no copies: the kernel reads the input from,
// and writes the output and results to, coherent pinned host memory, then
// stores the call's sequence number there; the host waits on that word (a
// launch + poll is ~11 us on this box against ~29 us for copy in, launch, copy
// out and a stream synchronisation).  Input up to the kernel's LDS staging size.
int decode_call_zc(xcg_ctx* c, const uint8_t* h_in, uint32_t len, uint8_t* h_out, uint64_t out_cap, uint32_t ops_cap,
                   uint32_t rw, uint64_t* h_out_len, uint64_t* h_consumed, int32_t* h_status, uint64_t* h_unknown,
                   uint32_t unknown_cap, uint32_t* h_nunknown, uint64_t* h_extract_hash, uint32_t extract_cap,
                   uint32_t* h_nextract) {
  const size_t inb = align256(len), outb = align256(out_cap ? out_cap : 1), resb = align256(8ull * rw);
  const size_t need = 256 + inb + outb + resb;
  if (need > c->zc_cap) {
    if (c->zc_h) {
      (void)hipStreamSynchronize(c->call_st);
      (void)hipHostFree(c->zc_h);
    }
    c->zc_h = nullptr;
    c->zc_cap = 0;
    const size_t want = need + need / 2;
    if (hipHostMalloc(&c->zc_h, want, hipHostMallocCoherent) != hipSuccess) return XCG_ENOMEM;
    c->zc_cap = want;
    memset(c->zc_h, 0, 256);
  }
  const size_t scr = align256(xcg_decode_small_scratch(ops_cap));
  int rc = ensure_stage(c, scr, 0);                  // (device scratch: the op lists)
  if (rc != XCG_OK) return rc;
  uint8_t* hz = c->zc_h;
  void* dz = nullptr;
  if (hipHostGetDevicePointer(&dz, hz, 0) != hipSuccess) return XCG_EHIP;
  uint8_t* dzb = (uint8_t*)dz;
  volatile uint32_t* flag = (volatile uint32_t*)hz;
  uint8_t* h_o = hz + 256 + inb;
  const uint64_t* h_res = (const uint64_t*)(hz + 256 + inb + outb);
  memcpy(hz + 256, h_in, len);
  const uint32_t seq = ++c->zc_seq ? c->zc_seq : ++c->zc_seq;   // (never 0: the word's initial value)
  const hipStream_t st = c->call_st;
  ctx_order(c, st);
  xcg_window* w = c->cur_win;
  if (xcg_launch_decode_small(dzb + 256, len, c->g.keys, c->g.vals, c->g.mask, c->g.pool, c->g.nseg, c->g.seg_cap,
                              c->g.filt, c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask, c->d_status, c->stage_d,
                              ops_cap, dzb + 256 + inb, out_cap, w->hash, w->seg, w->count,
                              (uint64_t*)(dzb + 256 + inb + outb), nullptr, (uint32_t*)dzb, seq, st) != 0)
    return XCG_EHIP;
  ctx_mark(c, st);
  // Spin (with a pause per poll, so a sibling hyperthread keeps its share) for
  // about the kernel's expected time; past ZC_SPIN_NS block in the runtime
  // instead, which sleeps -- so a slow or stuck kernel costs the caller's
  // event-loop thread no more than that much busy time.
  constexpr int64_t ZC_SPIN_NS = 2000000;
  const auto t_spin = std::chrono::steady_clock::now();
  for (uint64_t n = 1;; ++n) {
    if (__atomic_load_n((const uint32_t*)flag, __ATOMIC_ACQUIRE) == seq) break;
    __builtin_ia32_pause();
    if ((n & 1023) == 0) {
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) {
        if (__atomic_load_n((const uint32_t*)flag, __ATOMIC_ACQUIRE) == seq) break;
        return XCG_EHIP;                             // (finished without storing the word)
      }
      if (e != hipErrorNotReady) return XCG_EHIP;
      if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_spin).count() >
          ZC_SPIN_NS) {
        if (hipStreamSynchronize(st) != hipSuccess) return XCG_EHIP;
        if (__atomic_load_n((const uint32_t*)flag, __ATOMIC_ACQUIRE) != seq) return XCG_EHIP;
        break;
      }
    }
  }
  return decode_call_results(w, h_res, rw, h_o, h_out, h_out_len, h_consumed, h_status, h_unknown, unknown_cap,
                             h_nunknown, h_extract_hash, extract_cap, h_nextract);
}
}  // namespace

extern "C" {

int xcg_decode_call(xcg_ctx* c, const uint8_t* h_in, uint32_t len, uint8_t* h_out, uint64_t out_cap,
                    uint64_t* h_out_len, uint64_t* h_consumed, int32_t* h_status, uint64_t* h_unknown,
                    uint32_t unknown_cap, uint32_t* h_nunknown, uint64_t* h_extract_hash, uint32_t extract_cap,
                    uint32_t* h_nextract) {
  if (!c || !h_out_len || !h_consumed || !h_status || !h_nunknown || !h_nextract || (len && !h_in) ||
      (out_cap && !h_out))
    return XCG_EINVAL;
  *h_out_len = *h_consumed = 0;
  *h_status = 0;
  *h_nunknown = 0;
  *h_nextract = XCG_NO_REFERENCES;
  if (len == 0) return XCG_OK;
  DeviceGuard g(c->device);
  const bool fast = !c->bounded && !c->pair && !(c->flags & XCG_FLAG_NULLCACHE) && len <= (1u << 20);
  if (fast) {
    int rc = ensure_cache(c);
    if (rc == XCG_OK && !c->cur_win) {
      rc = window_alloc(c->device, &c->own_win);
      c->cur_win = c->own_win;
    }
    if (rc != XCG_OK) return rc;
    const uint32_t ops_cap = len / 4 + 64;
    const uint32_t rw = xcg_decode_small_res_words();
    if (len <= xcg_decode_small_lds_in() && !dphase_on() && !getenv_flag_no_zc()) {
      rc = decode_call_zc(c, h_in, len, h_out, out_cap, ops_cap, rw, h_out_len, h_consumed, h_status, h_unknown,
                          unknown_cap, h_nunknown, h_extract_hash, extract_cap, h_nextract);
      if (rc != XCG_ENOTSUP) return rc;
      // (fallback: the batch decoder takes it; nothing was written)
      const uint64_t off = 0;
      uint64_t ooff = 0;
      return xcg_decode_host(c, h_in, len, &off, &len, 1, h_out, out_cap, &ooff, h_out_len, h_status, h_consumed,
                             h_unknown, unknown_cap, h_nunknown);
    }
    // device: input | output | results | op lists;  host: input | output | results (one D2H brings
    // both back; the results' last word is the context's sticky word)
    const size_t inb = align256(len), outb = align256(out_cap ? out_cap : 1), resb = align256(8ull * rw);
    const size_t scr = align256(xcg_decode_small_scratch(ops_cap));
    const uint32_t nph = xcg_decode_small_phases();
    const size_t timb = dphase_on() ? align256(8ull * nph) : 0;
    rc = ensure_stage(c, inb + outb + resb + scr + timb, inb + outb + resb);
    if (rc != XCG_OK) return rc;
    uint8_t* dm = c->stage_d;
    uint8_t* hm = c->stage_h;
    uint64_t* d_res = (uint64_t*)(dm + inb + outb);
    uint64_t* h_res = (uint64_t*)(hm + inb + outb);
    uint8_t* h_o = hm + inb;
    const hipStream_t st = c->call_st;
    memcpy(hm, h_in, len);
    ctx_order(c, st);
    xcg_window* w = c->cur_win;
    if (hipMemcpyAsync(dm, hm, len, hipMemcpyHostToDevice, st) != hipSuccess ||
        xcg_launch_decode_small(dm, len, c->g.keys, c->g.vals, c->g.mask, c->g.pool, c->g.nseg, c->g.seg_cap,
                                c->g.filt, c->g.ftab, c->g.fmask, c->g.gfilt, c->g.gmask, c->d_status,
                                dm + inb + outb + resb, ops_cap, dm + inb, out_cap, w->hash, w->seg, w->count,
                                d_res, timb ? (uint64_t*)(dm + inb + outb + resb + scr) : nullptr, nullptr, 0u,
                                st) != 0 ||
        hipMemcpyAsync(h_o, dm + inb, outb + 8ull * rw, hipMemcpyDeviceToHost, st) != hipSuccess)
      return XCG_EHIP;
    ctx_mark(c, st);
    if (hipStreamSynchronize(st) != hipSuccess) return XCG_EHIP;
    if (timb) {
      std::vector<uint64_t> tm(nph, 0);
      if (hipMemcpy(tm.data(), dm + inb + outb + resb + scr, 8ull * nph, hipMemcpyDeviceToHost) == hipSuccess &&
          h_res[5] == 0) {
        std::lock_guard<std::mutex> g(g_dph_mu);
        g_dph_sum.resize(nph, 0.0);
        for (uint32_t k = 1; k < nph; ++k)
          if (tm[k] >= tm[k - 1]) g_dph_sum[k] += (double)(tm[k] - tm[k - 1]) * 0.01;   // 100 MHz clock
        g_dph_sum[0] += (double)(tm[nph - 1] - tm[0]) * 0.01;
        ++g_dph_calls;
      }
    }
    const int r2 = decode_call_results(w, h_res, rw, h_o, h_out, h_out_len, h_consumed, h_status, h_unknown,
                                       unknown_cap, h_nunknown, h_extract_hash, extract_cap, h_nextract);
    if (r2 != XCG_ENOTSUP) return r2;
    // (fallback: the batch decoder takes it; nothing was written)
  }
  const uint64_t off = 0;
  uint64_t ooff = 0;
  const int rc = xcg_decode_host(c, h_in, len, &off, &len, 1, h_out, out_cap, &ooff, h_out_len, h_status, h_consumed,
                                 h_unknown, unknown_cap, h_nunknown);
  return rc;
}

uint32_t xcg_debug_decode_phases(double* us, uint32_t n) {
  std::lock_guard<std::mutex> g(g_dph_mu);
  for (uint32_t k = 0; k < n; ++k) us[k] = k < g_dph_sum.size() ? g_dph_sum[k] : 0.0;
  const uint32_t calls = g_dph_calls;
  g_dph_sum.assign(g_dph_sum.size(), 0.0);
  g_dph_calls = 0;
  return calls;
}

int xcg_pack_outputs(xcg_ctx* c, const uint8_t* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                     uint32_t n, uint8_t* d_packed, uint64_t* d_packed_off, uint64_t* d_total, void* stream) {
  if (!c || (n && (!d_out || !d_out_off || !d_out_len || !d_packed || !d_packed_off || !d_total))) return XCG_EINVAL;
  DeviceGuard g(c->device);
  const int rc = xcg_launch_pack(d_out, d_out_off, d_out_len, n, d_packed, d_packed_off, d_total, (hipStream_t)stream);
  ctx_mark(c, (hipStream_t)stream);
  return rc == 0 ? XCG_OK : XCG_EHIP;
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
