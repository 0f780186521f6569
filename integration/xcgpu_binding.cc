/*
 * xcgpu_binding.cc -- the GPU mirror of a reference XCodecCache object, with
 * the geometry read from the object itself.
 *
 * The cache classes keep their configuration private: XCodecMemoryCache's
 * memory_cache_limit_ (xcodec/xcodec_cache.h:276), XCodecCachePair's levels
 * (:141-142), XCodecDiskCache's disk (xcodec/xcodec_cache_disk.h:94-99) and
 * XCodecDisk's volume size (:38).  The reference headers are unchanged, so the
 * binding reads those members through explicit template instantiations --
 * the one place C++ waives access checking ([temp.explicit]) -- instead of
 * asking wanproxy's config code to repeat them.  That is what makes caches
 * created by XCodecCache::connect (xcodec/xcodec_cache.h:101-111: a bounded
 * memory cache of the parent's limit, :297-301; a pair of connected levels,
 * :158-161) mirror with their real geometry: the decoding side of every pipe
 * pair (xcodec/xcodec_pipe_pair.cc:203) gets its caches that way.
 */
#include <string.h>
#include <unistd.h>

#include <map>
#include <string>
#include <typeinfo>

#include <common/buffer.h>

#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_cache_disk.h>

#include "xcgpu_binding.h"

namespace {

/* Member<Tag, &Class::member> defines member_of(Tag) returning the member
 * pointer; the explicit instantiations below name the private members. */
template <typename Tag, typename Tag::type M>
struct Member {
	friend typename Tag::type member_of(Tag) { return M; }
};

struct MemoryLimit {
	typedef size_t XCodecMemoryCache::*type;
	friend type member_of(MemoryLimit);
};
struct PairPrimary {
	typedef XCodecCache *XCodecCachePair::*type;
	friend type member_of(PairPrimary);
};
struct PairSecondary {
	typedef XCodecCache *XCodecCachePair::*type;
	friend type member_of(PairSecondary);
};
struct DiskOf {
	typedef XCodecDisk *XCodecDiskCache::*type;
	friend type member_of(DiskOf);
};
struct DiskBlocks {
	typedef uint64_t XCodecDisk::*type;
	friend type member_of(DiskBlocks);
};
struct DiskFd {
	typedef int XCodecDisk::*type;
	friend type member_of(DiskFd);
};
struct DiskHeadBlock {
	typedef uint64_t XCodecDisk::*type;
	friend type member_of(DiskHeadBlock);
};
struct DiskHeadNext {
	typedef size_t XCodecDisk::*type;
	friend type member_of(DiskHeadNext);
};
struct FrontXuid {
	typedef uint16_t XCodecDiskCache::*type;
	friend type member_of(FrontXuid);
};

template struct Member<MemoryLimit, &XCodecMemoryCache::memory_cache_limit_>;
template struct Member<PairPrimary, &XCodecCachePair::primary_>;
template struct Member<PairSecondary, &XCodecCachePair::secondary_>;
template struct Member<DiskOf, &XCodecDiskCache::disk_>;
template struct Member<DiskBlocks, &XCodecDisk::disk_blocks_>;
template struct Member<DiskFd, &XCodecDisk::fd_>;
template struct Member<DiskHeadBlock, &XCodecDisk::current_index_block_>;
template struct Member<DiskHeadNext, &XCodecDisk::index_block_next_>;
template struct Member<FrontXuid, &XCodecDiskCache::xuid_>;

xcgpu_binding::DiskResolver& resolver()
{
	static xcgpu_binding::DiskResolver fn = NULL;
	return fn;
}

std::map<XCodecCache *, xcg_ctx *>& ctx_map()
{
	static std::map<XCodecCache *, xcg_ctx *> ctxs;
	return ctxs;
}

std::map<XCodecCache *, std::string>& refusals()
{
	static std::map<XCodecCache *, std::string> r;
	return r;
}

/* One engine disk per XCodecDisk (XCodecDisk::open shares one disk per path,
 * xcodec_cache_disk.cc:826-838); kept for the life of the process, as the
 * reference's disk_map keeps its disks. */
std::map<const void *, xcg_disk *>& disk_map()
{
	static std::map<const void *, xcg_disk *> disks;
	return disks;
}

/* The XCodecDisk under a disk level, its volume size and the front's xuid and
 * UUID; with want_volume also the descriptor the XCodecDisk keeps its volume
 * open on (XCodecDisk::open, xcodec_cache_disk.cc:840-871) and its write
 * head. */
bool disk_of(XCodecCache *level, xcgpu_binding::DiskInfo *info, bool want_volume)
{
	if (resolver() != NULL && resolver()(level, info, want_volume))
		return true;
	XCodecDiskCache *front = dynamic_cast<XCodecDiskCache *>(level);
	if (front == NULL)
		return false;
	XCodecDisk *d = front->*member_of(DiskOf());
	info->disk = d;
	info->bytes = (d->*member_of(DiskBlocks())) * (uint64_t)XCG_SEGMENT_LENGTH;
	info->xuid = front->*member_of(FrontXuid());
	info->uuid = front->get_uuid().string_;
	if (want_volume) {
		info->fd = d->*member_of(DiskFd());
		info->close_fd = false;
		info->head_known = true;
		info->head_block = d->*member_of(DiskHeadBlock());
		info->head_next = d->*member_of(DiskHeadNext());
	}
	return true;
}

/* The engine disk under a pair's disk level: one per XCodecDisk, read from the
 * volume the host object reloaded (XCodecDisk::XCodecDisk,
 * xcodec_cache_disk.cc:107-237 -- the engine applies the same reload to the
 * same file, so both start from the same index, registry and write head). */
int engine_disk(XCodecCache *level, const xcgpu_binding::DiskInfo& g, xcg_disk **out, std::string *why)
{
	xcg_disk *&disk = disk_map()[g.disk];
	if (disk != NULL) {
		*out = disk;
		return XCG_OK;
	}
	xcgpu_binding::DiskInfo v;
	if (!disk_of(level, &v, true))
		return XCG_EINVAL;
	int rc = v.fd >= 0 ? xcg_disk_open_fd(v.fd, v.bytes, 0, &disk) : xcg_disk_create(v.bytes, &disk);
	if (v.close_fd && v.fd >= 0)
		close(v.fd);
	if (rc != XCG_OK) {
		disk = NULL;
		return rc;
	}
	uint64_t hb = 0, hn = 0;
	if (v.head_known && (xcg_disk_head(disk, &hb, &hn) != XCG_OK || hb != v.head_block || hn != v.head_next)) {
		*why = "the disk volume's reload put the engine's write head at index block " + std::to_string(hb) +
		       " entry " + std::to_string(hn) + ", the host XCodecDisk's is at " + std::to_string(v.head_block) +
		       " entry " + std::to_string(v.head_next) + " (the host disk was written to before its first pair "
		       "reached the engine)";
		xcg_disk_destroy(disk);
		disk = NULL;
		return XCG_EINVAL;
	}
	*out = disk;
	return XCG_OK;
}

}  // namespace

namespace xcgpu_binding {

void set_disk_resolver(DiskResolver fn)
{
	resolver() = fn;
}

Geometry geometry_of(XCodecCache *cache)
{
	Geometry g;
	g.kind = KIND_UNSUPPORTED;
	g.limit_bytes = 0;
	g.why = "a cache class the MI355X engine does not mirror";
	if (strstr(typeid(*cache).name(), "NullCache") != NULL) {
		g.kind = KIND_NULL;
		return g;
	}
	XCodecMemoryCache *m = dynamic_cast<XCodecMemoryCache *>(cache);
	if (m != NULL) {
		const size_t limit = m->*member_of(MemoryLimit());
		g.kind = limit != 0 ? KIND_BOUNDED : KIND_MEMORY;
		g.limit_bytes = (uint64_t)limit * XCG_SEGMENT_LENGTH;
		return g;
	}
	XCodecCachePair *p = dynamic_cast<XCodecCachePair *>(cache);
	if (p == NULL)
		return g;
	XCodecMemoryCache *primary = dynamic_cast<XCodecMemoryCache *>(p->*member_of(PairPrimary()));
	if (primary == NULL) {
		g.why = "an XCodecCachePair whose primary is not an XCodecMemoryCache";
		return g;
	}
	const size_t limit = primary->*member_of(MemoryLimit());
	if (!disk_of(p->*member_of(PairSecondary()), &g.disk, false)) {
		g.why = "an XCodecCachePair whose secondary is not a disk cache";
		return g;
	}
	/* An unbounded primary (limit 0) never evicts; the pair is still a pair:
	 * a primary miss goes to the disk, which may hold what an earlier pair on
	 * the same front entered (XCodecDisk::connect returns its existing front)
	 * or what a reloaded volume held, and a disk hit is promoted
	 * (xcodec_cache.h:208-230).  The engine runs it as a pair whose primary
	 * never evicts (xcg_ctx_create_pair_unbounded, limit_bytes 0 here). */
	g.kind = KIND_PAIR;
	g.limit_bytes = (uint64_t)limit * XCG_SEGMENT_LENGTH;
	return g;
}

xcg_ctx *ctx_for(XCodecCache *cache, bool out_of_band)
{
	std::map<XCodecCache *, xcg_ctx *>::iterator it = ctx_map().find(cache);
	if (it != ctx_map().end())
		return it->second;
	const Geometry g = geometry_of(cache);
	if (g.kind == KIND_UNSUPPORTED) {
		refusals()[cache] = std::string("cache is ") + g.why;
		return NULL;
	}
	uint32_t flags = out_of_band ? XCG_FLAG_OOB : 0;
	int device = 0;
	const char *dev = getenv("XCGPU_DEVICE");
	if (dev != NULL)
		device = atoi(dev);
	xcg_ctx *ctx = NULL;
	std::string why;
	int rc;
	switch (g.kind) {
	case KIND_NULL:
		rc = xcg_ctx_create(device, flags | XCG_FLAG_NULLCACHE, &ctx);
		break;
	case KIND_BOUNDED:
		rc = xcg_ctx_create_bounded(device, flags, g.limit_bytes, &ctx);
		break;
	case KIND_PAIR: {
		/* the pair's disk level is the host front of xuid g.disk.xuid: the
		 * engine binds the same front of the same (reloaded) disk */
		XCodecCache *level = dynamic_cast<XCodecCachePair *>(cache)->*member_of(PairSecondary());
		xcg_disk *disk = NULL;
		rc = engine_disk(level, g.disk, &disk, &why);
		if (rc == XCG_OK)
			rc = g.limit_bytes == 0 ?
			     xcg_ctx_create_pair_unbounded(device, flags, 0, disk,
			                                   g.disk.uuid.length() == 36 ? g.disk.uuid.c_str() : NULL, g.disk.xuid,
			                                   &ctx) :
			     xcg_ctx_create_pair_xuid(device, flags, g.limit_bytes, disk,
			                              g.disk.uuid.length() == 36 ? g.disk.uuid.c_str() : NULL, g.disk.xuid,
			                              &ctx);
		break;
	}
	default:
		rc = xcg_ctx_create(device, flags, &ctx);
		break;
	}
	if (rc != XCG_OK) {
		refusals()[cache] = std::string("MI355X engine: ") + (why.empty() ? xcg_strerror(rc) : why.c_str()) +
		                    " (XCGPU_DEVICE " + std::to_string(device) + ")";
		return NULL;
	}
	ctx_map()[cache] = ctx;
	refusals().erase(cache);
	return ctx;
}

const char *why_not(XCodecCache *cache)
{
	std::map<XCodecCache *, std::string>::const_iterator it = refusals().find(cache);
	return it == refusals().end() ? "no MI355X device for the XCodec engine" : it->second.c_str();
}

void forget(XCodecCache *cache)
{
	std::map<XCodecCache *, xcg_ctx *>::iterator it = ctx_map().find(cache);
	if (it == ctx_map().end())
		return;
	xcg_ctx_destroy(it->second);
	ctx_map().erase(it);
}

}  // namespace xcgpu_binding
