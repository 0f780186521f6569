/*
 * Drop-in bodies for wanproxy's zlib stage on the MI355X engine: DeflatePipe
 * and InflatePipe with their reference headers unchanged (zlib/deflate_pipe.h,
 * zlib/inflate_pipe.h); this file replaces zlib/deflate_pipe.cc and
 * zlib/inflate_pipe.cc in zlib/lib.mk.  Every pipe is a slot
 * of a process-wide pool of GPU contexts per direction (and level; device
 * XCGPU_DEVICE, default 0): a DeflatePipe(level) consume() is one xcg_zdeflate
 * call on its slot, an InflatePipe consume() one xcg_zinflate call.  Output
 * bytes equal zlib 1.2.11's driven by the reference loop at every level 0-9
 * (wanproxy.conf uses 6), including where that loop's single Z_SYNC_FLUSH call
 * into its 64 KiB buffer stops early (the held-back bytes are produced first
 * by the next consume).  The z_stream member the headers declare is left
 * unused.
 *
 * Reference behaviour kept (zlib/deflate_pipe.cc:57-115,
 * zlib/inflate_pipe.cc:54-139): a non-empty consume produces the bytes after
 * Z_SYNC_FLUSH; an empty one is EOS (Z_FINISH -> produce_eos).  The inflate
 * side produces what the input so far decodes to, produce_eos on EOS after the
 * stream's end, produce_error on a data error or bytes after the end.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <vector>

#include <common/buffer.h>
#include <common/thread/mutex.h>
#include <event/event_callback.h>
#include <io/pipe/pipe.h>

#include <zlib/deflate_pipe.h>
#include <zlib/inflate_pipe.h>

#include "../include/xcgpu.h"

namespace {

/*
 * Slots: a GPU context holds XCGPU_ZLIB_SLOTS pipes; a pool grows by another
 * context when every slot is taken (no limit on live pipes beyond device
 * memory), and a destroyed pipe's slot is reused (after a reset: the fresh
 * z_stream the reference's constructor makes).
 */
const uint32_t XCGPU_ZLIB_SLOTS = 4096;

int xcgpu_device(void)
{
	const char *dev = getenv("XCGPU_DEVICE");	/* as the XCodec binding (xcgpu_binding.cc) */
	return dev != NULL ? atoi(dev) : 0;
}

struct Slot {
	uint32_t ctx, slot;
};

struct DeflatePool {
	int level;
	std::vector<xcg_zdeflate *> ctx;
	std::vector<Slot> free_slots;
	std::map<const void *, Slot> slot_of;
	/* bytes a consume made but did not produce: zlib's pending output past
	 * the pipe's 64 KiB buffer (deflate_pipe.cc:34,86-105) */
	std::map<const void *, std::vector<uint8_t> > held;

	int grow(void)
	{
		xcg_zdeflate *z = NULL;
		int rc = xcg_zdeflate_create(xcgpu_device(), level, XCGPU_ZLIB_SLOTS, &z);
		if (rc != XCG_OK)
			return rc;
		ctx.push_back(z);
		for (uint32_t i = XCGPU_ZLIB_SLOTS; i > 0; i--) {
			Slot s = { (uint32_t)ctx.size() - 1, i - 1 };
			free_slots.push_back(s);
		}
		return XCG_OK;
	}
};

struct InflatePool {
	std::vector<xcg_zinflate *> ctx;
	std::vector<Slot> free_slots;
	std::map<const void *, Slot> slot_of;

	int grow(void)
	{
		xcg_zinflate *z = NULL;
		int rc = xcg_zinflate_create(xcgpu_device(), XCGPU_ZLIB_SLOTS, &z);
		if (rc != XCG_OK)
			return rc;
		ctx.push_back(z);
		for (uint32_t i = XCGPU_ZLIB_SLOTS; i > 0; i--) {
			Slot s = { (uint32_t)ctx.size() - 1, i - 1 };
			free_slots.push_back(s);
		}
		return XCG_OK;
	}
};

DeflatePool *deflate_pool(int level)
{
	static std::map<int, DeflatePool *> pools;
	std::map<int, DeflatePool *>::iterator it = pools.find(level);
	if (it != pools.end())
		return it->second;
	DeflatePool *p = new DeflatePool();
	p->level = level;
	pools[level] = p;
	return p;
}

InflatePool *inflate_pool(void)
{
	static InflatePool *p;
	if (p == NULL)
		p = new InflatePool();
	return p;
}

std::map<const void *, int>& deflate_levels()
{
	static std::map<const void *, int> levels;
	return levels;
}

void take_all(Buffer *in, std::vector<uint8_t>& bytes)
{
	bytes.resize(in->length());
	if (!bytes.empty()) {
		in->copyout(&bytes[0], bytes.size());
		in->skip(bytes.size());
	}
}

}  // namespace

DeflatePipe::DeflatePipe(int level)
: PipeProducer("/zlib/deflate_pipe", &mtx_),
  mtx_("DeflatePipe"),
  stream_()
{
	DeflatePool *p = deflate_pool(level);
	int rc = p->free_slots.empty() ? p->grow() : XCG_OK;
	if (rc != XCG_OK)	/* deflateInit's failure (bad level, no device / memory) */
		HALT(log_) << "Could not initialize deflate stream: " << xcg_strerror(rc);
	Slot slot = p->free_slots.back();
	p->free_slots.pop_back();
	if (xcg_zdeflate_reset(p->ctx[slot.ctx], slot.slot) != XCG_OK)
		HALT(log_) << "Could not initialize deflate stream.";
	p->slot_of[this] = slot;
	deflate_levels()[this] = level;
}

DeflatePipe::~DeflatePipe()
{
	int level = deflate_levels()[this];
	DeflatePool *p = deflate_pool(level);
	p->free_slots.push_back(p->slot_of[this]);
	p->slot_of.erase(this);
	p->held.erase(this);
	deflate_levels().erase(this);
}

void
DeflatePipe::consume(Buffer *in)
{
	DeflatePool *p = deflate_pool(deflate_levels()[this]);
	Slot slot = p->slot_of[this];
	/* the Buffer's segments: deflate() gets one per call (deflate_pipe.cc:66-84),
	 * which level 0's stored blocks follow */
	std::vector<uint32_t> segs;
	for (Buffer::SegmentIterator it = in->segments(); !it.end(); it.next())
		segs.push_back((*it)->length());
	std::vector<uint8_t> bytes;
	take_all(in, bytes);
	uint32_t len = bytes.size();
	uint32_t nseg = segs.size();
	uint64_t in_off = 0, out_off = 0;
	uint32_t out_len = 0;
	uint64_t deliver = 0;
	std::vector<uint8_t> obuf(xcg_zdeflate_bound(len));
	int rc = xcg_zdeflate_host(p->ctx[slot.ctx], bytes.empty() ? NULL : &bytes[0], &in_off, &len, &slot.slot, 1,
				   segs.empty() ? NULL : &segs[0], &nseg, &obuf[0], &out_off, &out_len, &deliver);
	if (rc != XCG_OK)
		HALT(log_) << "xcgpu deflate: " << xcg_strerror(rc);
	/* produce the held bytes and the new ones up to `deliver`; keep the rest */
	std::vector<uint8_t>& q = p->held[this];
	q.insert(q.end(), obuf.begin(), obuf.begin() + out_len);
	if (deliver > q.size())
		HALT(log_) << "xcgpu deflate: delivers more than it made";
	Buffer out;
	if (deliver)
		out.append(&q[0], deliver);
	q.erase(q.begin(), q.begin() + deliver);
	if (len == 0) {			/* Z_FINISH */
		produce_eos(&out);
		return;
	}
	if (!out.empty())
		produce(&out);
}

InflatePipe::InflatePipe(void)
: PipeProducer("/zlib/inflate_pipe", &mtx_),
  mtx_("InflatePipe"),
  stream_()
{
	InflatePool *p = inflate_pool();
	int rc = p->free_slots.empty() ? p->grow() : XCG_OK;
	if (rc != XCG_OK)
		HALT(log_) << "Could not initialize inflate stream: " << xcg_strerror(rc);
	Slot slot = p->free_slots.back();
	p->free_slots.pop_back();
	/* a reused slot still holds its last stream: inflateInit (inflate_pipe.cc:38-50) */
	if (xcg_zinflate_reset(p->ctx[slot.ctx], slot.slot) != XCG_OK)
		HALT(log_) << "Could not initialize inflate stream.";
	p->slot_of[this] = slot;
}

InflatePipe::~InflatePipe()
{
	InflatePool *p = inflate_pool();
	p->free_slots.push_back(p->slot_of[this]);
	p->slot_of.erase(this);
}

void
InflatePipe::consume(Buffer *in)
{
	InflatePool *p = inflate_pool();
	Slot slot = p->slot_of[this];
	std::vector<uint8_t> bytes;
	take_all(in, bytes);
	uint32_t len = bytes.size();
	uint64_t in_off = 0, out_off = 0;
	uint32_t cap = 8 * len + 65536, out_len = 0;
	int32_t status = 0;
	std::vector<uint8_t> obuf;
	for (;;) {		/* -2: more output room, nothing was committed */
		obuf.resize(cap);
		int rc = xcg_zinflate_host(p->ctx[slot.ctx], bytes.empty() ? NULL : &bytes[0], &in_off, &len, &slot.slot, 1,
					   &obuf[0], &out_off, &cap, &out_len, &status);
		if (rc != XCG_OK)
			HALT(log_) << "xcgpu inflate: " << xcg_strerror(rc);
		if (status != -2)
			break;
		cap *= 4;
	}
	if (status == -1) {
		ERROR(log_) << "inflate(): data error";
		produce_error();
		return;
	}
	Buffer out;
	if (out_len)
		out.append(&obuf[0], out_len);
	if (len == 0 && status == 1) {	/* Z_FINISH after the stream's end */
		produce_eos(&out);
		return;
	}
	if (!out.empty())
		produce(&out);
}
