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
 */
#ifndef XCGPU_BINDING_H
#define XCGPU_BINDING_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <typeinfo>
#include <map>

#include "../include/xcgpu.h"

/* Largest input of one encode() call (XCodecPipePair frames are at most
 * XCODEC_PIPE_MAX_FRAME / 2 = 512 KiB, xcodec/xcodec_pipe_pair.cc:596-604;
 * tack reads 64 KiB, programs/tack/tack.cc:419). */
#define XCGPU_MAX_ENCODE (512u * 1024u)

class XCodecCache;

namespace xcgpu_binding {

/* Cache kinds the engine mirrors exactly: XCodecMemoryCache (unbounded, or
 * bounded via set_cache_limit), XCodecCachePair of a bounded memory cache and
 * the local disk cache (via set_pair_geometry), and tack's TackNullCache
 * (lookups miss). */
inline bool is_null_cache(XCodecCache *cache)
{
	return strstr(typeid(*cache).name(), "NullCache") != NULL;
}

inline std::map<XCodecCache *, xcg_ctx *>& ctx_map()
{
	static std::map<XCodecCache *, xcg_ctx *> ctxs;
	return ctxs;
}

inline std::map<XCodecCache *, uint64_t>& limit_map();
struct PairGeometry;
inline std::map<XCodecCache *, PairGeometry>& pair_map();

/* The GPU mirror lives as long as the cache object.  wanproxy and tack keep
 * their caches for the life of the process; a caller that deletes a cache
 * must call forget() first (the reference caches have no hook for it). */
inline void forget(XCodecCache *cache)
{
	std::map<XCodecCache *, xcg_ctx *>::iterator it = ctx_map().find(cache);
	if (it == ctx_map().end())
		return;
	xcg_ctx_destroy(it->second);
	ctx_map().erase(it);
	limit_map().erase(cache);
	pair_map().erase(cache);
}

/* Bounded memory caches: XCodecMemoryCache keeps memory_cache_limit_
 * private (xcodec/xcodec_cache.h:272-288), so the code that makes one with a
 * size (programs/wanproxy/wanproxy_config_class_cache.cc:66) tells the binding:
 * its GPU mirror is then created with xcg_ctx_create_bounded (LRU eviction). */
inline std::map<XCodecCache *, uint64_t>& limit_map()
{
	static std::map<XCodecCache *, uint64_t> limits;
	return limits;
}

inline void set_cache_limit(XCodecCache *cache, uint64_t memory_cache_limit_bytes)
{
	if (memory_cache_limit_bytes != 0)
		limit_map()[cache] = memory_cache_limit_bytes;
}

/* wanproxy.conf's cache pair (XCodecCachePair of a bounded XCodecMemoryCache
 * and the local XCodecDiskCache, programs/wanproxy/wanproxy.conf:8-26): the
 * pair keeps its levels private (xcodec/xcodec_cache.h:140-153), so the code
 * that builds it (wanproxy_config_class_cache.cc) tells the binding the two
 * sizes; the GPU mirror is then an xcg_ctx_create_pair context. */
struct PairGeometry {
	uint64_t memory_limit_bytes;
	uint64_t disk_bytes;
};

inline std::map<XCodecCache *, PairGeometry>& pair_map()
{
	static std::map<XCodecCache *, PairGeometry> pairs;
	return pairs;
}

inline void set_pair_geometry(XCodecCache *cache, uint64_t memory_limit_bytes, uint64_t disk_bytes)
{
	PairGeometry g = { memory_limit_bytes, disk_bytes };
	pair_map()[cache] = g;
}

inline bool is_pair(XCodecCache *cache)
{
	return pair_map().find(cache) != pair_map().end();
}

inline xcg_ctx *ctx_for(XCodecCache *cache, bool out_of_band)
{
	std::map<XCodecCache *, xcg_ctx *>& ctxs = ctx_map();
	std::map<XCodecCache *, xcg_ctx *>::iterator it = ctxs.find(cache);
	if (it != ctxs.end())
		return it->second;
	/* a pair the binding was not told about (e.g. made by XCodecCachePair::
	 * connect) cannot be mirrored: refuse rather than diverge */
	if (strstr(typeid(*cache).name(), "XCodecCachePair") != NULL && !is_pair(cache))
		return NULL;
	uint32_t flags = out_of_band ? XCG_FLAG_OOB : 0;
	if (is_null_cache(cache))
		flags |= XCG_FLAG_NULLCACHE;
	xcg_ctx *ctx = NULL;
	int device = 0;
	const char *dev = getenv("XCGPU_DEVICE");
	if (dev != NULL)
		device = atoi(dev);
	std::map<XCodecCache *, uint64_t>::const_iterator lim = limit_map().find(cache);
	std::map<XCodecCache *, PairGeometry>::const_iterator pg = pair_map().find(cache);
	int rc;
	if (pg != pair_map().end())
		rc = xcg_ctx_create_pair(device, flags, pg->second.memory_limit_bytes, pg->second.disk_bytes, &ctx);
	else if (lim != limit_map().end())
		rc = xcg_ctx_create_bounded(device, flags, lim->second, &ctx);
	else
		rc = xcg_ctx_create(device, flags, &ctx);
	if (rc != XCG_OK)
		return NULL;
	ctxs[cache] = ctx;
	return ctx;
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
