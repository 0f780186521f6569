/*
 * ref_driver.cc -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A thin extern "C" harness around the REAL reference classes, compiled by
 * oracle/Makefile directly from the reference sources where they lie under
 * /root/reference (xcodec/xcodec_encoder.cc, xcodec/xcodec_decoder.cc,
 * xcodec/xcodec_cache.cc, common/buffer.cc, common/log.cc).  No reference
 * source is copied into this repository; the build output goes only to
 * oracle/_ref/.  This file plays the role of the reference's own drivers
 * (programs/tack/tack.cc:298-359, xcodec/test/xcodec-encode-decode1).
 */
#include <common/buffer.h>
#include <common/endian.h>
#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_decoder.h>
#include <xcodec/xcodec_encoder.h>
#include <xcodec/xcodec_hash.h>

#include <string.h>

#include <map>
#include <vector>

#ifdef XCGPU_DROPIN
#include "../integration/xcgpu_binding.h"
#define RELEASE_CACHE(c) xcgpu_binding::forget(c)
#else
#define RELEASE_CACHE(c) do { } while (0)
#endif

/* Out-of-band null cache: the same contract as tack's TackNullCache
 * (programs/tack/tack.cc:70-101): lookups miss, enter is a no-op. */
class RefNullCache : public XCodecCache {
public:
	RefNullCache(const UUID& uuid) : XCodecCache(uuid) { }
	XCodecCache *connect(const UUID&) { return NULL; }
	void enter(const uint64_t&, BufferSegment *) { }
	void replace(const uint64_t&, BufferSegment *) { }
	BufferSegment *lookup(const uint64_t&) { return NULL; }
	bool out_of_band(void) const { return true; }
};

/*
 * The disk secondary of wanproxy.conf's cache pair.  XCodecDisk /
 * XCodecDiskCache (xcodec/xcodec_cache_disk.{h,cc}) cannot be compiled here:
 * it needs UUID::generate / UUID::decode from common/uuid/uuid_libuuid.cc,
 * whose libuuid header the image lacks (no stand-in is written).  This class
 * RESTATES its in-memory behaviour for the local namespace, so the REAL
 * XCodecCachePair (xcodec/xcodec_cache.h:140-237) and the real encoder /
 * decoder run over it: FIFO data blocks in index blocks of 204 entries
 * (:72-101, :694-741), the next index block's entries leave the index when the
 * write head reaches it (:327-382), lookup re-hashes (:743-771), touch
 * re-enters a lost hash (:813-823), replace = remove + enter
 * (xcodec_cache_disk.h:130-134).  The bytes live in memory, not in a file.
 */
class RefDiskCache : public XCodecCache {
	uint64_t nb_, slots_, clock_;
	std::vector<uint64_t> key_;
	std::vector<uint8_t> alive_;
	std::vector<uint8_t> data_;
	std::map<uint64_t, uint64_t> index_;
public:
	RefDiskCache(const UUID& uuid, uint64_t disk_bytes)
	: XCodecCache(uuid),
	  nb_(((disk_bytes / XCODEC_SEGMENT_LENGTH) - 18) / 205),
	  slots_(nb_ * 204),
	  clock_(0),
	  key_(slots_),
	  alive_(slots_),
	  data_(slots_ * XCODEC_SEGMENT_LENGTH),
	  index_()
	{ }

	XCodecCache *connect(const UUID&) { return NULL; }

	void enter(const uint64_t& hash, BufferSegment *seg)
	{
		ASSERT("/ref/disk", index_.find(hash) == index_.end());
		uint64_t slot = clock_ % slots_;
		seg->copyout(&data_[slot * XCODEC_SEGMENT_LENGTH], 0, XCODEC_SEGMENT_LENGTH);
		key_[slot] = hash;
		alive_[slot] = 1;
		index_[hash] = slot;
		if (++clock_ % 204 == 0) {
			uint64_t b = (clock_ / 204) % nb_;
			for (uint64_t i = b * 204; i < (b + 1) * 204; i++) {
				if (!alive_[i])
					continue;
				index_.erase(key_[i]);
				alive_[i] = 0;
			}
		}
	}

	void remove(const uint64_t& hash)
	{
		std::map<uint64_t, uint64_t>::iterator it = index_.find(hash);
		if (it == index_.end())
			return;
		alive_[it->second] = 0;
		index_.erase(it);
	}

	void replace(const uint64_t& hash, BufferSegment *seg)
	{
		remove(hash);
		enter(hash, seg);
	}

	BufferSegment *lookup(const uint64_t& hash)
	{
		std::map<uint64_t, uint64_t>::iterator it = index_.find(hash);
		if (it == index_.end())
			return NULL;
		BufferSegment *seg = BufferSegment::create();
		memcpy(seg->head(), &data_[it->second * XCODEC_SEGMENT_LENGTH], XCODEC_SEGMENT_LENGTH);
		seg->set_length(XCODEC_SEGMENT_LENGTH);
		if (XCodecHash::hash(seg->data()) != hash) {
			seg->unref();
			alive_[it->second] = 0;
			index_.erase(it);
			return NULL;
		}
		return seg;
	}

	void touch(const uint64_t& hash, BufferSegment *seg)
	{
		if (index_.find(hash) == index_.end())
			enter(hash, seg);
	}

	bool out_of_band(void) const { return false; }

	uint64_t entries(void) const { return index_.size(); }
	uint64_t written(void) const { return clock_; }
};

static std::map<void *, std::pair<XCodecCache *, XCodecCache *> >& pair_levels()
{
	static std::map<void *, std::pair<XCodecCache *, XCodecCache *> > m;
	return m;
}

static uint64_t drain(Buffer *b, uint8_t *out, uint64_t cap)
{
	uint64_t n = b->length();
	if (n > cap)
		return ~(uint64_t)0;
	b->copyout(out, n);
	b->clear();
	return n;
}

extern "C" {

uint64_t xcr_hash(const uint8_t *data)
{
	return XCodecHash::hash(data);
}

/* Per-window XCodecHash values exactly as the encoder's rolling loop sees
 * them (add() x 2048 then roll()), xcodec_encoder.cc:126-176. */
void xcr_window_hashes(const uint8_t *x, uint64_t len, uint64_t *out)
{
	if (len < XCODEC_SEGMENT_LENGTH)
		return;
	XCodecHash h;
	for (unsigned i = 0; i < XCODEC_SEGMENT_LENGTH; i++)
		h.add(x[i]);
	for (uint64_t s = 0;; s++) {
		out[s] = h.mix();
		if (s + XCODEC_SEGMENT_LENGTH >= len)
			break;
		h.roll(x[s + XCODEC_SEGMENT_LENGTH]);
	}
}

void *xcr_cache_new(void)
{
	UUID uuid;
	return new XCodecMemoryCache(uuid);
}

/* XCodecMemoryCache(uuid, memory_cache_limit_bytes): the bounded, LRU-evicting
 * variant (xcodec/xcodec_cache.h:277-288, xcodec/xcodec_lru.h). */
void *xcr_cache_new_limited(uint64_t limit_bytes)
{
	UUID uuid;
	XCodecCache *c = new XCodecMemoryCache(uuid, (size_t)limit_bytes);
#ifdef XCGPU_DROPIN
	xcgpu_binding::set_cache_limit(c, limit_bytes);   /* as wanproxy_config_class_cache.cc would */
#endif
	return c;
}

/* XCodecCachePair(XCodecMemoryCache(uuid, memory_limit_bytes), disk of
 * disk_bytes): wanproxy.conf's memory + disk pair
 * (programs/wanproxy/wanproxy.conf:8-26, wanproxy_config_class_cache.cc). */
void *xcr_cache_new_pair(uint64_t memory_limit_bytes, uint64_t disk_bytes)
{
	UUID uuid;
	XCodecCache *primary = new XCodecMemoryCache(uuid, (size_t)memory_limit_bytes);
	XCodecCache *secondary = new RefDiskCache(uuid, disk_bytes);
	XCodecCache *pair = new XCodecCachePair(primary, secondary);
	pair_levels()[pair] = std::make_pair(primary, secondary);
#ifdef XCGPU_DROPIN
	xcgpu_binding::set_pair_geometry(pair, memory_limit_bytes, disk_bytes);
#endif
	return pair;
}

void xcr_cache_free(void *c)
{
	RELEASE_CACHE((XCodecCache *)c);
	std::map<void *, std::pair<XCodecCache *, XCodecCache *> >::iterator it = pair_levels().find(c);
	if (it != pair_levels().end()) {       /* the pair does not own its levels */
		delete it->second.first;
		delete it->second.second;
		pair_levels().erase(it);
	}
	delete (XCodecCache *)c;
}

/* Diagnostics of a pair made by xcr_cache_new_pair: [0] disk index entries,
 * [1] disk entries written. */
void xcr_pair_stats(void *c, uint64_t *st)
{
	RefDiskCache *d = (RefDiskCache *)pair_levels()[c].second;
	st[0] = d->entries();
	st[1] = d->written();
}

/* mode 0: fresh XCodecMemoryCache per chunk; mode 1: one cache + one encoder
 * for the whole batch (tack's loop); mode 2: RefNullCache (tack -N).
 * cache may carry a pre-state for mode 1 (NULL = a fresh one). */
int xcr_encode_batch(void *cache, const uint8_t *in, const uint64_t *off, const uint32_t *len, uint32_t n,
                     int mode, uint8_t *out, const uint64_t *out_off, uint64_t *out_len)
{
	UUID uuid;
	XCodecCache *stream_cache = (XCodecCache *)cache;
	bool own = false;
	if (mode == 1 && stream_cache == NULL) {
		stream_cache = new XCodecMemoryCache(uuid);
		own = true;
	}
	if (mode == 2)
		stream_cache = new RefNullCache(uuid);
	XCodecEncoder *stream_enc = (mode != 0) ? new XCodecEncoder(stream_cache) : NULL;
	int rc = 0;
	for (uint32_t i = 0; i < n; i++) {
		Buffer input, output;
		input.append(in + off[i], len[i]);
		if (mode == 0) {
			XCodecMemoryCache c(uuid);
			XCodecEncoder e(&c);
			e.encode(&output, &input);
			RELEASE_CACHE(&c);
		} else {
			stream_enc->encode(&output, &input);
		}
		uint64_t r = drain(&output, out + out_off[i], 2 * (uint64_t)len[i] + 16);
		if (r == ~(uint64_t)0) {
			rc = -1;
			break;
		}
		out_len[i] = r;
	}
	delete stream_enc;
	if (own || mode == 2) {
		RELEASE_CACHE(stream_cache);
		delete stream_cache;
	}
	return rc;
}

/* One XCodecEncoder::encode call with a refmap (the XCodecPipePair caller,
 * xcodec/xcodec_pipe_pair.cc:610-618), on a persistent encoder made by
 * xcr_encoder_new.  Returns the output and the refmap: hashes in map order and
 * their segments.  Returns 0, or -1 on overflow. */
void *xcr_encoder_new(void *cache) { return new XCodecEncoder((XCodecCache *)cache); }
void xcr_encoder_free(void *enc) { delete (XCodecEncoder *)enc; }

int xcr_encode_refmap(void *enc, const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *out_len,
                      uint64_t *hashes, uint8_t *segs, uint64_t max, uint64_t *nref)
{
	Buffer input, output;
	input.append(in, len);
	std::map<uint64_t, BufferSegment *> refmap;
	((XCodecEncoder *)enc)->encode(&output, &input, &refmap);
	uint64_t r = drain(&output, out, cap);
	*nref = 0;
	for (std::map<uint64_t, BufferSegment *>::iterator it = refmap.begin(); it != refmap.end(); ++it) {
		if (*nref < max) {
			hashes[*nref] = it->first;
			it->second->copyout(segs + *nref * XCODEC_SEGMENT_LENGTH, 0, XCODEC_SEGMENT_LENGTH);
			(*nref)++;
		}
		it->second->unref();
	}
	if (r == ~(uint64_t)0)
		return -1;
	*out_len = r;
	return 0;
}

/* One XCodecDecoder::decode over a whole buffer with cache `cache`
 * (tack -d, programs/tack/tack.cc:329-359).  Returns 1/0 like decode(),
 * -1 on overflow; *consumed = bytes parsed; *nunk = unknown hashes. */
/* A persistent XCodecDecoder (its BACKREF window lives across calls). */
void *xcr_decoder_new(void *cache) { return new XCodecDecoder((XCodecCache *)cache); }
void xcr_decoder_free(void *dec) { delete (XCodecDecoder *)dec; }

int xcr_decoder_decode(void *dec, const uint8_t *x, uint64_t len, uint8_t *out, uint64_t cap,
                       uint64_t *out_len, uint64_t *consumed, uint64_t *unk, uint64_t *nunk, uint64_t unk_max)
{
	Buffer input, output;
	input.append(x, len);
	std::set<uint64_t> unknown;
	bool ok = ((XCodecDecoder *)dec)->decode(&output, &input, unknown);
	*consumed = len - input.length();
	*nunk = 0;
	for (std::set<uint64_t>::const_iterator it = unknown.begin(); it != unknown.end() && *nunk < unk_max; ++it)
		unk[(*nunk)++] = *it;
	uint64_t r = drain(&output, out, cap);
	if (r == ~(uint64_t)0)
		return -1;
	*out_len = r;
	return ok ? 1 : 0;
}

int xcr_decode(void *cache, const uint8_t *x, uint64_t len, uint8_t *out, uint64_t cap,
               uint64_t *out_len, uint64_t *consumed, uint64_t *unk, uint64_t *nunk, uint64_t unk_max)
{
	XCodecDecoder d((XCodecCache *)cache);
	Buffer input, output;
	input.append(x, len);
	std::set<uint64_t> unknown;
	bool ok = d.decode(&output, &input, unknown);
	*consumed = len - input.length();
	*nunk = 0;
	for (std::set<uint64_t>::const_iterator it = unknown.begin(); it != unknown.end() && *nunk < unk_max; ++it)
		unk[(*nunk)++] = *it;
	uint64_t r = drain(&output, out, cap);
	if (r == ~(uint64_t)0)
		return -1;
	*out_len = r;
	return ok ? 1 : 0;
}

}
