/*
 * xcgpu_binding.h -- how wanproxy's XCodec classes reach the MI355X engine.
 *
 * One xcg_ctx (device memory: the GPU-resident segment cache) per reference
 * XCodecCache object.  The reference shares one cache among every encoder and
 * decoder of a codec (programs/wanproxy/wanproxy_config_class_codec.cc:71-79,
 * xcodec/test/xcodec-encode-decode1.cc:59-82), so the binding is keyed by the
 * cache pointer and the GPU cache is shared the same way.  The host-side
 * XCodecCache is kept as a mirror of every entry the engine makes, so the rest
 * of wanproxy (ASK/LEARN in xcodec_pipe_pair.cc, other caches) sees exactly the
 * reference's cache contents.
 *
 * The GPU mirror takes its geometry from the cache object itself
 * (xcgpu_binding.cc), whoever made it: wanproxy's cache config, or
 * XCodecCache::connect on the decoding side of a pipe pair
 * (xcodec/xcodec_pipe_pair.cc:203 -> xcodec/xcodec_cache.h:101-111), which
 * makes a bounded XCodecMemoryCache of its parent's limit (:297-301) or a new
 * XCodecCachePair of connected levels (:158-161).  No registration call is
 * needed anywhere.  Pairs whose disk levels are front-ends of one XCodecDisk
 * share one engine disk (xcg_disk): one FIFO ring, as the reference's.
 */
#ifndef XCGPU_BINDING_H
#define XCGPU_BINDING_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <map>
#include <string>

#include "../include/xcgpu.h"

/* Largest input of one encode() call (XCodecPipePair frames are at most
 * XCODEC_PIPE_MAX_FRAME / 2 = 512 KiB, xcodec/xcodec_pipe_pair.cc:596-604;
 * tack reads 64 KiB, programs/tack/tack.cc:419). */
#define XCGPU_MAX_ENCODE (512u * 1024u)

class XCodecCache;

namespace xcgpu_binding {

/* What a cache object is, read from the object (xcgpu_binding.cc). */
enum CacheKind {
	KIND_UNSUPPORTED = 0,	/* a cache class the engine does not mirror */
	KIND_NULL,		/* tack's TackNullCache: lookups miss (programs/tack/tack.cc:70-101) */
	KIND_MEMORY,		/* XCodecMemoryCache, no limit (xcodec/xcodec_cache.h:245-365) */
	KIND_BOUNDED,		/* XCodecMemoryCache with a limit: LRU eviction */
	KIND_PAIR		/* XCodecCachePair(memory -- bounded, or unbounded: limit_bytes 0 --, disk front-end) (:140-237) */
};

/* The disk level of a pair: the XCodecDisk under it and which front it is. */
struct DiskInfo {
	const void *disk;	/* identity of the XCodecDisk under the disk level */
	uint64_t bytes;		/* its volume size */
	int xuid;		/* the front's xuid on it (XCodecDiskCache::xuid_), -1 unknown */
	std::string uuid;	/* the front's UUID (XCodecCache::get_uuid) */
	/* asked for only when the engine disk is made (want_volume): */
	int fd;			/* the volume's descriptor (XCodecDisk::fd_), -1 none: a fresh disk */
	bool close_fd;		/* the resolver opened fd for this call: the binding closes it */
	bool head_known;	/* the host disk's write head (current_index_block_, index_block_next_) */
	uint64_t head_block, head_next;

	DiskInfo() : disk(NULL), bytes(0), xuid(-1), uuid(), fd(-1), close_fd(false), head_known(false),
	             head_block(0), head_next(0) { }
};

struct Geometry {
	CacheKind kind;
	uint64_t limit_bytes;	/* the memory (primary) limit, bytes */
	DiskInfo disk;		/* KIND_PAIR: the disk level */
	const char *why;	/* KIND_UNSUPPORTED: what is not mirrored */
};

Geometry geometry_of(XCodecCache *cache);

/*
 * A disk level class other than XCodecDiskCache (e.g. a test harness's
 * restatement of XCodecDisk) can be resolved to its disk by a resolver; return
 * false for objects it does not know.  With want_volume it also gives a
 * descriptor its volume file can be read from, as the file stands now, and the
 * host disk's write head.
 */
typedef bool (*DiskResolver)(XCodecCache *level, DiskInfo *info, bool want_volume);
void set_disk_resolver(DiskResolver fn);

/* The GPU mirror of `cache`, created on first use; NULL if it cannot be made
 * -- why_not() then says why (the adapters HALT with it). */
xcg_ctx *ctx_for(XCodecCache *cache, bool out_of_band);
const char *why_not(XCodecCache *cache);

/* The GPU mirror lives as long as the cache object.  wanproxy and tack keep
 * their caches for the life of the process (XCodecCache::connect's registry
 * never deletes one); a caller that deletes a cache calls forget() first. */
void forget(XCodecCache *cache);

inline bool is_null_cache(XCodecCache *cache)
{
	return geometry_of(cache).kind == KIND_NULL;
}

/* One BACKREF window per XCodecDecoder object (the reference's
 * XCodecDecoder::window_ member, xcodec/xcodec_decoder.h:37); the header's
 * members are unchanged, so the handle is kept beside the object. */
inline std::map<const void *, xcg_window *>& window_map()
{
	static std::map<const void *, xcg_window *> wins;
	return wins;
}

inline xcg_window *window_for(const void *decoder, xcg_ctx *ctx)
{
	std::map<const void *, xcg_window *>::iterator it = window_map().find(decoder);
	if (it != window_map().end())
		return it->second;
	xcg_window *w = NULL;
	if (xcg_window_create(ctx, &w) != XCG_OK)
		return NULL;
	window_map()[decoder] = w;
	return w;
}

inline void forget_window(const void *decoder)
{
	std::map<const void *, xcg_window *>::iterator it = window_map().find(decoder);
	if (it == window_map().end())
		return;
	xcg_window_destroy(it->second);
	window_map().erase(it);
}

}  // namespace xcgpu_binding

#endif /* !XCGPU_BINDING_H */
