/*
 * xcgpu.h -- C ABI of the MI355X-native XCodec engine (libxcgpu.so).
 *
 * Plain pointers and sizes only.  Every `d_` pointer is device memory (HBM)
 * of the context's device; `stream` is a hipStream_t passed as void* (NULL =
 * the default stream).  Functions return 0 (XCG_OK) or a negative XCG_E*
 * status; no exceptions cross the ABI.  One context per host thread, or
 * external locking -- the reference calls its codec under
 * XCodecPipePair::mtx_ (xcodec/xcodec_pipe_pair.h:45) from one EventThread.
 *
 * Reference interfaces replaced (paths relative to wanproxy's tree):
 *   xcg_ctx_create / xcg_ctx_destroy
 *       XCodecEncoder::XCodecEncoder(XCodecCache *)   xcodec/xcodec_encoder.cc:40-46
 *       XCodecMemoryCache(const UUID&, size_t)         xcodec/xcodec_cache.h:277-288
 *       XCodecCache::out_of_band()                     xcodec/xcodec_cache.h:89
 *   xcg_encode_batch / xcg_encode_host
 *       void XCodecEncoder::encode(Buffer *output, Buffer *input,
 *                                  std::map<uint64_t, BufferSegment *> *refmap)
 *                                                      xcodec/xcodec_encoder.h:42,
 *                                                      xcodec/xcodec_encoder.cc:74-274
 *       (one encode() call per chunk, exactly as tack / XCodecPipePair issue
 *        them: programs/tack/tack.cc:308-321, xcodec/xcodec_pipe_pair.cc:596-630)
 *   xcg_decode_batch / xcg_decode_host / xcg_window_*
 *       bool XCodecDecoder::decode(Buffer *output, Buffer *input,
 *                                  std::set<uint64_t>& unknown_hashes)
 *                                                      xcodec/xcodec_decoder.h:44,
 *                                                      xcodec/xcodec_decoder.cc:66-272
 *   xcg_window_hashes
 *       XCodecHash::{add,roll,mix}                     xcodec/xcodec_hash.h:93-164
 *   xcg_segment_hashes
 *       XCodecHash::hash per 2048-byte segment          xcodec/xcodec_hash.h:166-174
 *       (tack -h, programs/tack/tack.cc:368-414)
 *   xcg_zdeflate_*
 *       DeflatePipe::DeflatePipe(int level) / consume(Buffer *)
 *                                                      zlib/deflate_pipe.h:33-42,
 *                                                      zlib/deflate_pipe.cc:36-115
 *   xcg_zinflate_*
 *       InflatePipe::InflatePipe() / consume(Buffer *) zlib/inflate_pipe.h:33-42,
 *                                                      zlib/inflate_pipe.cc:33-139
 */
#ifndef XCGPU_H
#define XCGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XCG_SEGMENT_LENGTH 2048u   /* XCODEC_SEGMENT_LENGTH, xcodec/xcodec.h:87 */

/* Context / call flags. */
#define XCG_FLAG_OOB 0x1u          /* out-of-band declarations (F1 02 BE64 instead of
                                      F1 01 + data): XCodecCache::out_of_band() == true,
                                      xcodec/xcodec_encoder.cc:44,288-295 */
#define XCG_FLAG_NULLCACHE 0x2u    /* lookups always miss, enter is a no-op: tack -N's
                                      TackNullCache, programs/tack/tack.cc:70-101 */

/* Batch semantics. */
#define XCG_SEM_INDEPENDENT 0      /* chunk i = one encode() with a fresh, empty
                                      XCodecMemoryCache (no cross-chunk state) */
#define XCG_SEM_STREAM 1           /* chunks 0..n-1 = successive encode() calls of ONE
                                      XCodecEncoder on the context's persistent cache
                                      (tack's loop, programs/tack/tack.cc:308-321); the
                                      batch's declarations are committed to the cache */

#define XCG_DEFAULT_CACHE_SEGMENTS (1u << 19)   /* 1 GiB of segments */

/* Status codes. */
#define XCG_OK 0
#define XCG_ENOENT (-2)            /* hash not in the cache */
#define XCG_EHIP (-5)              /* a HIP runtime call failed */
#define XCG_ENOMEM (-12)
#define XCG_EINVAL (-22)
#define XCG_EOVERFLOW (-75)        /* internal table overflow (reported, never silent) */
#define XCG_EPROTO (-71)           /* pipe protocol error (XCodecPipePair::decoder_error) */
#define XCG_ENOTSUP (-95)
#define XCG_EEXIST (-17)           /* (registry) the UUID is registered already */

typedef struct xcg_ctx xcg_ctx;

/* Library build / version string. */
const char *xcg_version(void);
const char *xcg_strerror(int status);

/* Worst-case encoded size of one encode() call over `len` input bytes:
 * every byte literal and 0xF1 (each escaped to two bytes). */
uint64_t xcg_encode_bound(uint32_t len);

int xcg_ctx_create(int device, uint32_t flags, xcg_ctx **out);
/* As xcg_ctx_create with an explicit persistent-cache capacity in 2 KiB
 * segments (XCodecMemoryCache(uuid, limit), xcodec/xcodec_cache.h:277; here
 * exceeding it is an error, XCG_EOVERFLOW, not an LRU eviction). */
int xcg_ctx_create_ex(int device, uint32_t flags, uint64_t cache_segments, xcg_ctx **out);
/* A context whose persistent cache is the BOUNDED XCodecMemoryCache(uuid,
 * memory_cache_limit_bytes) (xcodec/xcodec_cache.h:277-364; wanproxy.conf's
 * `set <cache>.size`, programs/wanproxy/wanproxy_config_class_cache.cc:66):
 * limit = bytes / 2048 segments (at least 1); entering at the limit evicts the
 * least recently entered-or-looked-up segment (XCodecLRU, xcodec/xcodec_lru.h).
 * XCG_SEM_STREAM batches, decode batches and the single-segment host calls
 * stay bit-exact with the sequential XCodecEncoder / XCodecDecoder on such a
 * cache.  XCG_ENOTSUP (never a different result): an encode chunk, or a decode
 * call, whose own enters + persistent-entry lookups exceed the limit (encode
 * batches are cut into sub-batches that fit); XCG_SEM_INDEPENDENT with chunks of
 * more than limit * 2048 bytes; BACKREF ops in a decode on a bounded cache. */
int xcg_ctx_create_bounded(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_ctx **out);
/* A context whose persistent cache is wanproxy.conf's XCodecCachePair
 * (xcodec/xcodec_cache.h:140-237, programs/wanproxy/wanproxy.conf:8-26): a
 * bounded XCodecMemoryCache(uuid, memory_cache_limit_bytes) primary (LRU, as
 * xcg_ctx_create_bounded) over the local XCodecDiskCache of a fresh volume of
 * disk_bytes (xcodec/xcodec_cache_disk.cc: FIFO data blocks in index blocks
 * of 204 entries, (disk_bytes / 2048 - 18) / 205 index blocks).  A lookup
 * that misses the primary and hits the disk enters the hash into the primary;
 * a primary hit re-enters a hash the disk index lost.  XCG_SEM_STREAM batches,
 * decode batches and the single-segment host calls are bit-exact with the
 * sequential XCodecEncoder / XCodecDecoder on such a pair; the disk level lives
 * on the device (its index as GPU arrays, its bytes in HBM or, past free HBM,
 * in pinned host memory: xcg_disk_create_ex).  In-band only (XCG_EINVAL
 * with XCG_FLAG_OOB / XCG_FLAG_NULLCACHE, or a volume without one index
 * block).  XCG_ENOTSUP (never a different result): a decode batch in which a
 * hash it EXTRACTed leaves both levels before a later op names it (decode it
 * in smaller batches), BACKREF ops.  Decode chunks of a bounded or pair
 * context are < 2 MiB each (XCG_EINVAL). */
int xcg_ctx_create_pair(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, uint64_t disk_bytes,
                        xcg_ctx **out);
/* One XCodecDisk shared by several pairs (xcodec/xcodec_cache_disk.h:33-69):
 * its FIFO ring is common to every XCodecDiskCache front-end on it -- the
 * local cache (XCodecDisk::local) and each peer cache XCodecCache::connect
 * makes on it (XCodecDisk::connect, xcodec_cache_disk.cc:640-690) -- and when
 * the write head enters an index block, every front loses its entries there
 * (index_invalidate_entries, :327-382).  xcg_ctx_create_pair_on makes a pair
 * context whose secondary is the next front (xuid) of `disk`; its cache
 * references then interleave with the other fronts' in one ring, in the order
 * the calls are made (the reference serialises them on its event thread).
 * The disk lives until its last front and xcg_disk_destroy are gone.
 * xcg_disk_stats: st[0] live index entries (all fronts), st[1] entries
 * written, st[2] index blocks, st[3] fronts. */
typedef struct xcg_disk xcg_disk;
int xcg_disk_create(uint64_t disk_bytes, xcg_disk **out);
/* The disk's data blocks are one allocation mapped (HIP virtual memory) behind
 * the primary of every front on the disk, so N fronts cost one disk.  Where
 * the blocks live: HBM when the volume fits beside what the device already
 * holds (4 GiB kept free), otherwise pinned host memory behind the same device
 * addresses -- a spill level below HBM that the kernels read and write over
 * PCIe.  XCG_DISK_HOST / XCG_DISK_DEVICE force one tier (DEVICE: fail rather
 * than spill).  xcg_disk_tier: 0 HBM, 1 host memory, -1 before the first
 * front (the tier is chosen when the first front binds the disk to a device). */
#define XCG_DISK_HOST 1u
#define XCG_DISK_DEVICE 2u
int xcg_disk_create_ex(uint64_t disk_bytes, uint32_t flags, xcg_disk **out);
int xcg_disk_tier(const xcg_disk *disk);
/* The volume file (XCodecDisk::open, xcodec/xcodec_cache_disk.cc:824-871; its
 * layout :72-101: 18 registry blocks of 36-byte UUIDs, nb index blocks of a
 * u64 counter and 204 (u16 xuid, u64 hash) entries, the data blocks).
 * xcg_disk_open reopens a volume a previous process saved -- the reference's
 * reload (:107-237): registered fronts, the write head at the lowest counter,
 * the other index blocks loaded in counter order with the first and last 80
 * checked against their data -- or starts a fresh one when `path` is absent
 * or empty.  xcg_disk_save writes the volume as the reference's file stands at
 * that moment (data blocks written at every enter, an index block when it
 * fills).  Fronts find their entries again by UUID: xcg_ctx_create_pair_uuid
 * makes the front of a 36-character UUID string (XCodecDisk::connect: the
 * registered xuid, else the lowest free one, registered); the local front is
 * the first one made on a fresh volume (xuid 0).  A front made without a UUID
 * is XCodecDisk::local (:635-641): xuid 0 when the volume registered it and no
 * front holds it, else the lowest free xuid under a generated UUID (on a fresh
 * volume that is xuid 0, as registry_load's local UUID, :575-596).  A volume
 * whose registry is empty gets a local UUID at open, as registry_load does.
 * xcg_disk_save writes the data blocks whether or not any front is left. */
int xcg_disk_open(const char *path, uint64_t disk_bytes, uint32_t flags, xcg_disk **out);
int xcg_disk_save(xcg_disk *disk, const char *path);
int xcg_ctx_create_pair_uuid(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_disk *disk,
                             const char *uuid36, xcg_ctx **out);
/* The drop-in's disk (integration/xcgpu_binding.cc): the engine disk of a host
 * XCodecDisk is read from the descriptor the host object keeps its volume open
 * on (XCodecDisk::fd_, xcodec_cache_disk.h:38; the file as the host's reload
 * left it, :107-237), with the reference's reload semantics; a descriptor of an
 * empty file gives a fresh disk.  xcg_ctx_create_pair_xuid binds the front a
 * host XCodecDiskCache already is (its xuid_, xcodec_cache_disk.h:106; uuid36
 * its UUID, or NULL), so the engine's fronts are the host disk's whatever
 * order they are bound in (xuid -1: as xcg_ctx_create_pair_uuid).  XCG_EINVAL
 * when that xuid is held by another front or the UUID is registered at
 * another xuid.  xcg_disk_head: the write head as XCodecDisk keeps it
 * (current_index_block_, index_block_next_, :701-727) -- after a reload, the
 * host object's and the engine's agree.  xcg_pair_xuid: a pair context's
 * front. */
int xcg_disk_open_fd(int fd, uint64_t disk_bytes, uint32_t flags, xcg_disk **out);
int xcg_ctx_create_pair_xuid(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_disk *disk,
                             const char *uuid36, int xuid, xcg_ctx **out);
int xcg_disk_head(const xcg_disk *disk, uint64_t *index_block, uint64_t *next_entry);
int xcg_pair_xuid(const xcg_ctx *ctx);
/* XCodecCachePair over an UNBOUNDED XCodecMemoryCache (a memory cache without
 * a size: XCodecMemoryCache(uuid, 0) never evicts, xcodec/xcodec_cache.h:
 * 303-318) and `disk`: the pair's policy as above -- a primary miss goes to the
 * disk, a disk hit is promoted, a primary hit touches the disk (:208-237) --
 * over a primary that holds up to capacity_segments (0: XCG_DEFAULT_CACHE_
 * SEGMENTS); a batch that would need more fails with XCG_EOVERFLOW instead of
 * evicting.  uuid36 / xuid as for xcg_ctx_create_pair_xuid.  A connect
 * (xcg_ctx_connect) on such a context makes another one. */
int xcg_ctx_create_pair_unbounded(int device, uint32_t flags, uint64_t capacity_segments, xcg_disk *disk,
                                  const char *uuid36, int xuid, xcg_ctx **out);
void xcg_disk_destroy(xcg_disk *disk);
int xcg_disk_stats(const xcg_disk *disk, uint64_t *st);
int xcg_ctx_create_pair_on(int device, uint32_t flags, uint64_t memory_cache_limit_bytes, xcg_disk *disk,
                           xcg_ctx **out);
/* Pair context counters: st[0] primary entries, st[1] this front's disk index
 * entries, st[2] disk entries written so far (all fronts), st[3] disk index
 * blocks. */
int xcg_pair_stats(xcg_ctx *ctx, uint64_t *st);
void xcg_ctx_destroy(xcg_ctx *ctx);
/* The XCG_FLAG_* the context was created with. */
int xcg_ctx_flags(const xcg_ctx *ctx, uint32_t *flags);

/* Persistent cache: number of segments held / drop everything. */
uint64_t xcg_cache_size(xcg_ctx *ctx);
int xcg_cache_clear(xcg_ctx *ctx);
/* Rounds the last XCG_SEM_STREAM batch needed to reach its fixed point. */
int xcg_last_rounds(xcg_ctx *ctx);
/* Single-segment host access to the persistent cache, for host adapters:
 * XCodecCache::lookup (xcodec/xcodec_cache.h:86) copies the 2048 bytes out
 * (XCG_ENOENT if absent); XCodecCache::enter/replace (:84-85) -- an existing
 * hash has its bytes replaced.  On bounded and pair caches these are the
 * reference's calls with their side effects (LRU use; a pair's disk touch or
 * promotion), and enter is <LEARN>'s lookup-then-replace-or-enter
 * (xcodec/xcodec_pipe_pair.cc:311-327); on a pair, `hash` must be the
 * segment's XCodecHash (XCG_EINVAL otherwise). */
int xcg_cache_lookup_host(xcg_ctx *ctx, uint64_t hash, uint8_t *seg_out);
int xcg_cache_enter_host(xcg_ctx *ctx, uint64_t hash, const uint8_t *seg);
/* Declarations (hash, position in the chunk) chunk `chunk` of the last
 * XCG_SEM_STREAM batch made, in order: what XCodecEncoder::encode_declaration
 * entered into the cache (xcodec/xcodec_encoder.cc:276-313).  On a bounded
 * cache only the chunks of the batch's last sub-batch are kept (XCG_ENOTSUP
 * for earlier ones; a single-chunk batch is always one sub-batch). */
int xcg_last_declarations(xcg_ctx *ctx, uint32_t chunk, uint64_t *h_hash, uint32_t *h_pos, uint32_t cap,
                          uint32_t *h_count);
/* The cache references chunk `chunk` of the last XCG_SEM_STREAM batch made on
 * a bounded or pair cache, in stream order: every lookup that found the hash
 * in a level at some point of the batch (XCodecCache::lookup refreshes an LRU
 * entry, and a pair promotes or re-enters it, xcodec/xcodec_cache.h:208-230,
 * :348-364 -- whether or not the bytes then match) and every declaration's
 * enter (xcodec/xcodec_encoder.cc:284-286).  h_kind[i]: 0 enter (h_ref[i] =
 * declaration index, as xcg_last_declarations numbers them), 1 lookup of a
 * hash this batch declared, 2 lookup of a cached hash, 3 lookup of a cached
 * hash already gone (a miss).  A host mirror of the cache that replays them
 * in order -- lookup for kinds 1-3, enter for 0 -- holds what the engine's
 * cache holds.  XCG_ENOTSUP on an unbounded cache (its lookups change
 * nothing) and for chunks before the last sub-batch. */
int xcg_last_references(xcg_ctx *ctx, uint32_t chunk, uint64_t *h_hash, uint32_t *h_kind, uint32_t *h_ref,
                        uint32_t cap, uint32_t *h_count);
/* Diagnostics: copy the persistent cache's lane filters to host memory
 * (h_filt: 2^19 bits; h_ftab: up to ftab_words u32; *h_fmask = buckets - 1). */
int xcg_debug_cache_dump(xcg_ctx *ctx, uint32_t *h_filt, uint32_t *h_ftab, uint64_t ftab_words, uint32_t *h_fmask);

/*
 * Encode n chunks in one launch.  Chunk i is d_in[d_chunk_off[i] ..
 * d_chunk_off[i] + d_chunk_len[i]); its encoding (bit-exact with one
 * XCodecEncoder::encode call over it) is written to d_out + d_out_off[i], which
 * must have room for xcg_encode_bound(d_chunk_len[i]) bytes; its length goes to
 * d_out_len[i].  max_chunk_len bounds every d_chunk_len[i] (<= 512 KiB, the
 * XCodecPipePair frame cap, xcodec/xcodec_pipe_pair.cc:596-604).
 * d_stats (nullable): 4 u32 per chunk {EXTRACT or OOB declarations, REFs,
 * hash collisions, pieces}.  XCG_SEM_INDEPENDENT is asynchronous on `stream`;
 * XCG_SEM_STREAM synchronises `stream` once per round.
 */
int xcg_encode_batch(xcg_ctx *ctx, int semantics, const uint8_t *d_in, const uint64_t *d_chunk_off,
                     const uint32_t *d_chunk_len, uint32_t n, uint32_t max_chunk_len, uint8_t *d_out,
                     const uint64_t *d_out_off, uint64_t *d_out_len, uint32_t *d_stats, void *stream);

/* Synchronous host-memory convenience over xcg_encode_batch (copies in, encodes,
 * copies out, checks the internal status word).  h_out_off[i] slots as above. */
int xcg_encode_host(xcg_ctx *ctx, int semantics, const uint8_t *h_in, uint64_t in_len,
                    const uint64_t *h_chunk_off, const uint32_t *h_chunk_len, uint32_t n, uint8_t *h_out,
                    uint64_t out_cap, const uint64_t *h_out_off, uint64_t *h_out_len);

/* *h_nref of xcg_encode_call on a cache whose lookups change nothing (an
 * unbounded memory cache, the null cache): no reference list is kept. */
#define XCG_NO_REFERENCES 0xFFFFFFFFu

/* One XCodecEncoder::encode(output, input) call from host memory, the way tack
 * (programs/tack/tack.cc:308-321, one call per <= 64 KiB read) and
 * XCodecPipePair (xcodec/xcodec_pipe_pair.cc:596-618, per <= 512 KiB frame)
 * make it -- stream semantics on the context's persistent cache.  h_in[0 .. len)
 * is encoded into h_out (out_cap >= xcg_encode_bound(len)); the call's
 * declarations come back in order (hash and input offset, encode_declaration
 * xcodec_encoder.cc:276-313) and, on a bounded or pair cache, its cache
 * references in stream order (kind: 0 enter, 1 hit on a declaration of the
 * call, 2 hit on a cached entry, 3 lookup of an entry evicted earlier in the
 * call; idx: the declaration number of an enter), else *h_nref =
 * XCG_NO_REFERENCES.  The reference-class adapters (integration/) replay these
 * into the host XCodecCache.  The context keeps its staging buffers and stream,
 * so a call allocates nothing and synchronises once (unbounded caches).
 * *h_ndecl / *h_nref may exceed the caps (then only the first cap are written). */
int xcg_encode_call(xcg_ctx *ctx, const uint8_t *h_in, uint32_t len, uint8_t *h_out, uint64_t out_cap,
                    uint64_t *h_out_len, uint64_t *h_decl_hash, uint32_t *h_decl_pos, uint32_t decl_cap,
                    uint32_t *h_ndecl, uint64_t *h_ref_hash, uint32_t *h_ref_kind, uint32_t *h_ref_idx,
                    uint32_t ref_cap, uint32_t *h_nref);

/*
 * Decode n encoded chunks that form ONE stream (successive
 * XCodecDecoder::decode calls on one decoder whose cache is the context's
 * persistent cache), xcodec/xcodec_decoder.cc:66-188.  Each chunk should be a
 * whole encode() output (an XCodecPipePair frame); an op cut at a chunk's end
 * stops that chunk with status 3 and d_consumed[i] < d_chunk_len[i], as decode()
 * leaves a partial op in its input.  Decoded bytes are packed contiguously in
 * d_out (offsets in d_out_off); *h_total_out is the size needed -- if it exceeds
 * out_cap nothing is written and XCG_EOVERFLOW is returned.
 * d_chunk_status[i]: 0 decoded, 1 blocked on an unknown REF (decode() returned
 * true with unknown hashes; later chunks get 2 = not reached), 3 partial op,
 * -1 bad opcode or BACKREF to an empty window slot (decode() returned false;
 * later chunks get 2).  h_unknown receives the sorted unknown hashes from the
 * blocking point to the end of the batch (decode_skim, :196-272, over the
 * frames a pipe pair has buffered) for the ASK/LEARN protocol.
 * EXTRACTs decoded before the stop point enter the persistent cache
 * (enter / replace, :106-136) and every EXTRACT / REF declares into the
 * decoder's BACKREF window.  Synchronises `stream`.
 */
int xcg_decode_batch(xcg_ctx *ctx, const uint8_t *d_enc, const uint64_t *d_chunk_off, const uint32_t *d_chunk_len,
                     uint32_t n, uint32_t max_chunk_len, uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off,
                     uint64_t *d_out_len, int32_t *d_chunk_status, uint64_t *d_consumed, uint64_t *h_unknown,
                     uint32_t unknown_cap, uint32_t *h_nunknown, uint64_t *h_total_out, void *stream);

/* A decoder's BACKREF window (XCodecWindow, xcodec/xcodec_window.h:40-125):
 * 256 slots of (hash, segment) that EXTRACT and REF declare into and
 * <BACKREF> index reads (xcodec/xcodec_decoder.cc:137,160,165-181).  It lives
 * as long as the decoder: one per XCodecDecoder (the cache may be shared).
 * Decodes use the context's own window unless xcg_decode_set_window selected
 * another (NULL = back to the context's own). */
typedef struct xcg_window xcg_window;
int xcg_window_create(xcg_ctx *ctx, xcg_window **out);
void xcg_window_destroy(xcg_window *win);
int xcg_decode_set_window(xcg_ctx *ctx, xcg_window *win);

/* Host-memory convenience over xcg_decode_batch. */
int xcg_decode_host(xcg_ctx *ctx, const uint8_t *h_enc, uint64_t enc_len, const uint64_t *h_chunk_off,
                    const uint32_t *h_chunk_len, uint32_t n, uint8_t *h_out, uint64_t out_cap, uint64_t *h_out_off,
                    uint64_t *h_out_len, int32_t *h_chunk_status, uint64_t *h_consumed, uint64_t *h_unknown,
                    uint32_t unknown_cap, uint32_t *h_nunknown);

/* One XCodecDecoder::decode(output, input, unknown_hashes) call from host
 * memory (xcodec/xcodec_decoder.cc:66-272), the way tack (-d, one call per
 * 64 KiB read, programs/tack/tack.cc:329-359) and XCodecPipePair
 * (xcodec_pipe_pair.cc:425-446) make it: h_in[0 .. len) continues the
 * context's stream (cache, current window).  *h_status / *h_consumed as
 * xcg_decode_batch's for one chunk; decode_skim's unknown hashes sorted in
 * h_unknown.  On an unbounded cache an input of <= 1 MiB is decoded in ONE
 * launch and one synchronisation on the context's staging and stream, and the
 * XCodecHash of every EXTRACT before the stop comes back in op order
 * (h_extract_hash, *h_nextract; XCG_NO_REFERENCES when not provided: other
 * caches, larger inputs, BACKREF ops -- those take the batch decoder), so a
 * host cache mirror needs no hashing.  XCG_EOVERFLOW if out_cap is too small
 * (*h_out_len = the size needed; nothing is committed). */
int xcg_decode_call(xcg_ctx *ctx, const uint8_t *h_in, uint32_t len, uint8_t *h_out, uint64_t out_cap,
                    uint64_t *h_out_len, uint64_t *h_consumed, int32_t *h_status, uint64_t *h_unknown,
                    uint32_t unknown_cap, uint32_t *h_nunknown, uint64_t *h_extract_hash, uint32_t extract_cap,
                    uint32_t *h_nextract);

/* Pack n output slots (d_out + d_out_off[i], d_out_len[i] bytes) back to back
 * into d_packed; d_packed_off[i] receives each chunk's offset and *d_total
 * (device) the packed size.  Asynchronous on `stream`. */
int xcg_pack_outputs(xcg_ctx *ctx, const uint8_t *d_out, const uint64_t *d_out_off, const uint64_t *d_out_len,
                     uint32_t n, uint8_t *d_packed, uint64_t *d_packed_off, uint64_t *d_total, void *stream);

/* Status word of the context (sticky; nonzero = an internal overflow happened
 * in an earlier asynchronous call).  Synchronises the context's device. */
int xcg_ctx_status(xcg_ctx *ctx);

/*
 * XCodecPipePair protocol layer (xcodec/xcodec_pipe_pair.cc,
 * xcodec/xcodec_pipe_protocol.h), host side over the functions above:
 * <HELLO>, <FRAME> (one encode() per <= 512 KiB of input), <ASK>/<LEARN>,
 * <ADVANCE>, <EOS>/<EOS_ACK>.  `enc` is the codec's encoder context (its cache
 * is shared by every pipe of the codec, xcodec/xcodec.h:91-107); `dec` the
 * decoder context of the peer's cache (XCodecCache::connect(uuid), one per
 * peer); `uuid` the 36-character UUID string this side sends in <HELLO>.
 * Each call returns what XCodecPipePair would produce: bytes for the peer
 * (encoder_produce) and decoded bytes for the local side (decoder_produce),
 * plus the two EOS signals.  Output buffers belong to the pipe and stay valid
 * until its next call.  XCG_EPROTO = decoder_error().
 *   encoder_consume  = XCodecPipePair::encoder_consume (:549-642); len 0 = EOS
 *   decoder_consume  = XCodecPipePair::decoder_consume (:68-166);  len 0 = EOS
 *   encoder_consume_many: n pipes sharing one `enc`, their frames encoded in
 *   ONE GPU batch in the given order (the order one event thread serves them).
 */
typedef struct xcg_pipe xcg_pipe;
typedef struct xcg_pipe_out {
  const uint8_t *to_peer;
  uint64_t to_peer_len;
  const uint8_t *to_local;
  uint64_t to_local_len;
  int local_eos;                 /* decoder_produce_eos */
  int peer_eos;                  /* encoder_produce_eos */
} xcg_pipe_out;
int xcg_pipe_create(xcg_ctx *enc, xcg_ctx *dec, const uint8_t *uuid, xcg_pipe **out);
/* As xcg_pipe_create, with the decoder's cache connected when the peer's
 * <HELLO> arrives, as XCodecPipePair::decoder_decode does
 * (decoder_cache_ = XCodecCache::connect(uuid, codec_->cache()),
 * xcodec/xcodec_pipe_pair.cc:182-203): xcg_ctx_connect(parent, <HELLO>'s UUID).
 * Pipes whose peers send the same UUID decode on one context. */
int xcg_pipe_create_connect(xcg_ctx *enc, xcg_ctx *parent, const uint8_t *uuid, xcg_pipe **out);
/* The decoder context a pipe decodes on (NULL before a connecting pipe's <HELLO>). */
xcg_ctx *xcg_pipe_decoder_ctx(const xcg_pipe *p);
void xcg_pipe_destroy(xcg_pipe *p);
int xcg_pipe_encoder_consume(xcg_pipe *p, const uint8_t *data, uint64_t len, xcg_pipe_out *out);
int xcg_pipe_encoder_consume_many(xcg_pipe *const *pipes, const uint8_t *const *data, const uint64_t *len, uint32_t n,
                                  xcg_pipe_out *out);
int xcg_pipe_decoder_consume(xcg_pipe *p, const uint8_t *data, uint64_t len, xcg_pipe_out *out);
/* Frames whose REF segments the encoder still keeps for <ASK> (not yet <ADVANCE>d). */
uint32_t xcg_pipe_pending_frames(const xcg_pipe *p);

/*
 * The process-wide cache registry of XCodecCache::connect / enter / lookup
 * (xcodec/xcodec_cache.h:101-127, one std::map<UUID, XCodecCache*> per
 * process).  xcg_ctx_connect returns the context registered under `uuid36`,
 * else makes one with the parent's connect -- XCodecMemoryCache::connect: an
 * empty cache of the parent's limit (unbounded or bounded, same flags);
 * XCodecCachePair::connect: a new pair whose primary is such a cache and whose
 * secondary is the front XCodecDisk::connect gives that UUID on the parent's
 * disk (xcodec_cache_disk.cc:640-690) -- and registers it.  The registry owns
 * what it made; xcg_ctx_register enters a caller's context (wanproxy registers
 * its own codec cache under the local UUID) without taking it.
 * xcg_connect_registry_clear destroys the contexts the registry made and
 * forgets every entry (the reference never does; for tests and shutdown).
 * XCG_EEXIST: the UUID is registered already.
 */
int xcg_ctx_connect(xcg_ctx *parent, const char *uuid36, xcg_ctx **out);
int xcg_ctx_register(xcg_ctx *c, const char *uuid36);
xcg_ctx *xcg_ctx_lookup(const char *uuid36);
void xcg_connect_registry_clear(void);

/* ------------------------------------------------------------------------
 * zlib stage: wanproxy's DeflatePipe after the XCodec encoder
 * (programs/wanproxy/wanproxy_codec_pipe_pair.cc:97-106,148-157; set
 * codecN.compressor zlib / compressor_level N, wanproxy.conf:32-41).
 * A context holds `nstreams` DeflatePipe(level) instances
 * (zlib/deflate_pipe.cc:36-50: deflateInit(level), windowBits 15, memLevel 8)
 * in HBM.  Output is bit-exact with zlib 1.2.11 driven by DeflatePipe::consume at
 * every level: 4-9 deflate_slow, 1-3 deflate_fast, 0 deflate_stored.
 *   xcg_zdeflate_batch: one DeflatePipe::consume() per listed stream (a stream
 *   at most once per batch; successive batches continue the streams):
 *   h_len[i] > 0 bytes at d_in + h_in_off[i] = every segment through
 *   deflate(Z_NO_FLUSH), then ONE deflate(Z_SYNC_FLUSH) into the pipe's
 *   64 KiB buffer (deflate_pipe.cc:57-115); h_len[i] == 0 = EOS:
 *   deflate(Z_FINISH) (zlib trailer; the stream is done).
 *   d_out + h_out_off[i] (4-byte aligned, room for xcg_zdeflate_bound(h_len[i]))
 *   receives the call's new stream bytes, d_out_len[i] of them; d_deliver[i]
 *   is how many bytes the consume produce()s: the stream's not yet delivered
 *   bytes followed by these new ones, cut at d_deliver[i].  The pipe's flush
 *   call ends when its 64 KiB buffer fills, so a consume can produce less
 *   than it made (zlib keeps the rest pending; a stop at a block flush also
 *   leaves out the sync marker and parses the last < 262 positions with the
 *   next consume's bytes).  The caller keeps the undelivered bytes (at most
 *   ~64 KiB per stream) and delivers them first next time.  Metadata arrays
 *   are host memory; the call is asynchronous on `stream`.
 *   xcg_zdeflate_reset: the slot becomes a fresh DeflatePipe.
 */
typedef struct xcg_zdeflate xcg_zdeflate;
uint64_t xcg_zdeflate_bound(uint32_t len);
int xcg_zdeflate_create(int device, int level, uint32_t nstreams, xcg_zdeflate **out);
void xcg_zdeflate_destroy(xcg_zdeflate *z);
int xcg_zdeflate_reset(xcg_zdeflate *z, uint32_t stream);
int xcg_zdeflate_batch(xcg_zdeflate *z, const uint8_t *d_in, const uint64_t *h_in_off, const uint32_t *h_len,
                       const uint32_t *h_stream, uint32_t n, uint8_t *d_out, const uint64_t *h_out_off,
                       uint32_t *d_out_len, uint64_t *d_deliver, void *stream);
/* The same with the Buffer's segments: call i's bytes are cut into h_nseg[i]
 * segments whose lengths follow in h_seg (all calls' lists concatenated).
 * Level 0's stored blocks follow the segments (deflate_stored copies what
 * each deflate() call is given); levels 1-9 do not depend on them.
 * xcg_zdeflate_batch cuts every call into 2048-byte segments (BUFFER_SEGMENT_SIZE,
 * common/buffer.h:52: a Buffer filled by append). */
int xcg_zdeflate_batch_seg(xcg_zdeflate *z, const uint8_t *d_in, const uint64_t *h_in_off, const uint32_t *h_len,
                           const uint32_t *h_stream, uint32_t n, const uint32_t *h_seg, const uint32_t *h_nseg,
                           uint8_t *d_out, const uint64_t *h_out_off, uint32_t *d_out_len, uint64_t *d_deliver,
                           void *stream);
/* Host buffers, synchronous; segments as in xcg_zdeflate_batch_seg (h_seg NULL: 2048-byte cuts). */
int xcg_zdeflate_host(xcg_zdeflate *z, const uint8_t *h_in, const uint64_t *h_in_off, const uint32_t *h_len,
                      const uint32_t *h_stream, uint32_t n, const uint32_t *h_seg, const uint32_t *h_nseg,
                      uint8_t *h_out, const uint64_t *h_out_off, uint32_t *h_out_len, uint64_t *h_deliver);

/* Diagnostics: parse rounds the last levels 1-3 batch took (deflate_fast's
 * hashed positions guessed, then reproduced; 0 for other levels). */
uint32_t xcg_debug_zdeflate_rounds(const xcg_zdeflate *z);

/* Receiving side: `nstreams` InflatePipe instances (zlib/inflate_pipe.cc:33-46,
 * inflateInit) in HBM.  xcg_zinflate_batch: one InflatePipe::consume() per
 * listed stream (at most once per batch): h_len[i] bytes at d_in + h_in_off[i]
 * are the next cut of the peer's zlib stream (any cut: inside a symbol or a
 * block header is fine); every byte they let inflate() produce goes to
 * d_out + h_out_off[i] (at most h_out_cap[i] bytes), its count to
 * d_out_len[i].  d_status[i]: 0 ok, 1 the stream's end was reached (with
 * h_len 0 = EOS: InflatePipe's produce_eos), -1 Z_DATA_ERROR (bad header,
 * code, distance, adler32, or bytes after the end: produce_error), -2 h_out_cap
 * too small (nothing committed: the call may be repeated with more room). */
typedef struct xcg_zinflate xcg_zinflate;
int xcg_zinflate_create(int device, uint32_t nstreams, xcg_zinflate **out);
void xcg_zinflate_destroy(xcg_zinflate *z);
/* The slot becomes a fresh InflatePipe (inflateInit): every InflatePipe
 * construction on a reused slot calls it, as DeflatePipe does xcg_zdeflate_reset. */
int xcg_zinflate_reset(xcg_zinflate *z, uint32_t stream);
int xcg_zinflate_batch(xcg_zinflate *z, const uint8_t *d_in, const uint64_t *h_in_off, const uint32_t *h_len,
                       const uint32_t *h_stream, uint32_t n, uint8_t *d_out, const uint64_t *h_out_off,
                       const uint32_t *h_out_cap, uint32_t *d_out_len, int32_t *d_status, void *stream);
/* The same on host buffers (synchronous); lengths / statuses to host arrays. */
int xcg_zinflate_host(xcg_zinflate *z, const uint8_t *h_in, const uint64_t *h_in_off, const uint32_t *h_len,
                      const uint32_t *h_stream, uint32_t n, uint8_t *h_out, const uint64_t *h_out_off,
                      const uint32_t *h_out_cap, uint32_t *h_out_len, int32_t *h_status);
/* Tests / A-B: which inflate kernel runs -- 0 by batch size (a 1024-thread
 * workgroup per call up to 256 calls, 256 threads up to 4096, a wave per call
 * beyond), 1 always a wave per call, 2 always a 1024-thread workgroup per call,
 * 3 always a 256-thread workgroup per call. */
int xcg_debug_set_zinflate_mode(int mode);
/* Workgroup-kernel regions since the last call (then reset): regions,
 * fixed-point iterations, bytes committed, resolve rounds. */
int xcg_debug_zinflate_regions(uint64_t *out);

/* Diagnostics / tests: stream-semantics batches probe the cache through a
 * 64 KiB LDS lane filter while the cache + batch hold at most this many keys,
 * else through a global (L2-resident) one; both give the same output.
 * Returns the previous threshold (default ~0u = automatic: 150000, or 0 for a
 * cache whose fingerprint buckets exceed 2 MiB; or XCG_LDS_FILTER_KEYS). */
uint32_t xcg_debug_set_lds_filter_keys(uint32_t keys);
/* Diagnostics / tests: past that threshold, and while the cache + batch hold at
 * most this many keys, the LDS filter still goes first and only the positions
 * it passes load the global filter (fewer L2 requests); beyond it the global
 * filter alone.  Same output either way.  Returns the previous threshold
 * (default 700000, or XCG_LDS_PREFILTER_KEYS). */
uint32_t xcg_debug_set_lds_prefilter_keys(uint32_t keys);
/* Diagnostics (bench.py's decode roofline): while on, every xcg_decode_batch on
 * an unbounded cache brackets its device work with HIP events on its stream --
 * the scan, the reference check / sizing, and the emit + commit segments (the
 * host's two readbacks between them excluded) -- and the emit kernel alone.
 * xcg_debug_decode_kernel_time returns the sums in ms since the last call and
 * the number of segments, and resets them.  Returns the previous setting. */
int xcg_debug_decode_kernel_timing(int on);
int xcg_debug_decode_kernel_time(double *step_ms, double *emit_ms, uint32_t *segments);
/* Diagnostics / tests: stream batches start either with a parse round against
 * the cache alone, or -- automatically when the context's previous batch
 * declared segments -- from each chunk's 2048-byte tiling (its cold parse),
 * corrected by the verification.  Same output either way.  mode: -1
 * automatic (default), 0 never seed, 1 always seed.  Returns the previous mode. */
int xcg_debug_set_stream_seed(int mode);
/* Diagnostics / tests: stream batches of small chunks (< 8 KiB) pass a screen
 * first that gives every chunk none of whose windows can be found (nothing in
 * the cache, the batch or its own earlier tiles) its cold parse -- the
 * 2048-byte tiling -- and sends the rest to the parse; same output either way.
 * mode 0 off, 1 on (default; env XCG_SCREEN), 2 on and counting:
 * xcg_debug_screen_counts returns (and resets) the chunks screened and those
 * sent on to the parse.  Returns the previous mode. */
int xcg_debug_set_screen(int mode);
int xcg_debug_screen_counts(uint64_t *screened, uint64_t *parsed);
/* Diagnostics / bench: while on, every stream-parse kernel launch
 * (encode_stream_kernel) is bracketed by HIP events on its launch stream;
 * xcg_debug_stream_kernel_time returns (and resets) the summed milliseconds
 * and the launch count.  Process-wide.  Returns the previous setting. */
int xcg_debug_stream_kernel_timing(int on);
/* Diagnostics / tests: on a bounded or pair context, how many re-parsed chunks
 * so far resumed from their previous pass's rows, and how many of those rejoined
 * their old parse (DESIGN.md 3.6 "Re-parse restart"); env XCG_NO_RESTART turns
 * resuming off (same output). */
int xcg_debug_restart_counts(xcg_ctx *ctx, uint64_t *resumed, uint64_t *spliced);
int xcg_debug_stream_kernel_time(double *ms, uint32_t *launches);
/* Diagnostics: with env XCG_DECODE_PHASES set, each one-launch decode()
 * (xcg_decode_call) records clock stamps at its kernel's phase boundaries;
 * us[0] = summed kernel time, us[k] = summed duration of phase k (1 stage,
 * 2 walk, 3 EXTRACT hashes, 4 resolve, 5 precheck, 6 output size, 7 output
 * copy, 8 window, 9 commit, 10 results), microseconds.  Returns (and resets)
 * the call count. */
uint32_t xcg_debug_decode_phases(double *us, uint32_t n);

/* Every window hash: d_hash[s] = XCodecHash over d_x[s .. s+2048) for
 * s in [0, len - 2048]. */
int xcg_window_hashes(xcg_ctx *ctx, const uint8_t *d_x, uint64_t len, uint64_t *d_hash, void *stream);

/* tack -h: XCodecHash::hash of each whole 2048-byte segment, big-endian u64. */
int xcg_segment_hashes(xcg_ctx *ctx, const uint8_t *d_x, uint64_t len, uint64_t *d_hash_be, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* XCGPU_H */
