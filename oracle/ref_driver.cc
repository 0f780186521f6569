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

#include <ctype.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

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
 * whose libuuid header the image lacks (no stand-in is written).  RefDisk and
 * RefDiskCache RESTATE their in-memory behaviour, so the REAL XCodecCachePair
 * (xcodec/xcodec_cache.h:140-237) and the real encoder / decoder run over it:
 * one FIFO of data blocks in index blocks of 204 entries shared by every
 * front-end (xuid) on the disk (:72-101, :694-741); when the write head enters
 * an index block, each front loses the entries it still has there -- the
 * index entry names the front, and a front's hash counts only if its index
 * still points at that block (index_invalidate_entries, :327-382); lookup
 * re-hashes (:743-771), touch re-enters a lost hash (:813-823), replace =
 * remove + enter (xcodec_cache_disk.h:130-134); connect(uuid) gives the uuid's
 * front, a new one on the lowest free xuid (XCodecDisk::connect, :640-690).
 * The bytes live in memory; save() / the path constructor write and reload
 * the reference's volume file (below).
 */
class RefDisk;

class RefDiskCache : public XCodecCache {
	friend class RefDisk;
	RefDisk *disk_;
	uint16_t xuid_;
	std::map<uint64_t, uint64_t> index_;   /* hash -> data block (XCodecDiskCache::hash_cache_) */
	RefDiskCache(const UUID& uuid, RefDisk *disk, uint16_t xuid)
	: XCodecCache(uuid), disk_(disk), xuid_(xuid), index_()
	{ }
public:
	XCodecCache *connect(const UUID& uuid);
	void enter(const uint64_t& hash, BufferSegment *seg);
	void replace(const uint64_t& hash, BufferSegment *seg);
	BufferSegment *lookup(const uint64_t& hash);
	void touch(const uint64_t& hash, BufferSegment *seg);
	bool out_of_band(void) const { return false; }
	uint64_t entries(void) const { return index_.size(); }
	uint64_t written(void) const;
	RefDisk *disk(void) const { return disk_; }
	uint16_t xuid(void) const { return xuid_; }
};

/*
 * The volume file (xcodec_cache_disk.cc:72-101): 18 registry blocks of
 * 36-byte UUID strings (56 per block, 1024 xuids), nb index blocks (a u64
 * counter, then 204 x (u16 xuid, u64 hash)), nb * 204 data blocks
 * (data_block_address :305-311).  The reference writes a data block at every
 * enter and an index block when it fills (:694-741); save() writes what such a
 * volume holds at that moment.  Reopening restates XCodecDisk::XCodecDisk
 * (:107-237): the registry gives the fronts, index blocks are scanned in order
 * up to the first free one (counter 0), the lowest counter is the write head
 * and is not loaded, the others load in counter order (a later entry of a hash
 * replaces an earlier one), the first and last 80 are checked against their
 * data blocks' hashes (index_load_entries :408-478), fronts without entries
 * leave the registry (registry_collect :496-528).
 */
static const unsigned REG_BLOCKS = 18, REG_ENTRIES = 2048 / 36, CHECK_BOUNDARY = 80;

static bool uuid_string_ok(const uint8_t *u)	/* uuid_parse's format: 8-4-4-4-12 hex digits */
{
	for (unsigned i = 0; i < 36; i++) {
		if (i == 8 || i == 13 || i == 18 || i == 23) {
			if (u[i] != '-')
				return false;
		} else if (!isxdigit(u[i])) {
			return false;
		}
	}
	return true;
}

class RefDisk {
	uint64_t nb_, slots_, clock_;
	std::vector<uint64_t> key_;
	std::vector<uint16_t> xuid_;
	std::vector<uint8_t> used_;
	std::vector<uint8_t> data_;
	std::map<uint16_t, RefDiskCache *> fronts_;
	std::map<std::string, uint16_t> uuid_xuid_;
	std::vector<uint64_t> ctr_;	/* per index block: the counter it was last written with (0: never) */
	uint64_t ibc_;			/* index_block_counter_: the counter of the block being filled */
	std::vector<uint8_t> reg_;	/* the registry blocks */
public:
	const uint64_t bytes_;

	RefDisk(uint64_t disk_bytes)
	: nb_(((disk_bytes / XCODEC_SEGMENT_LENGTH) - 18) / 205),
	  slots_(nb_ * 204),
	  clock_(0),
	  key_(slots_),
	  xuid_(slots_),
	  used_(slots_),
	  data_(slots_ * XCODEC_SEGMENT_LENGTH),
	  fronts_(),
	  uuid_xuid_(),
	  ctr_(nb_, 0),
	  ibc_(1),
	  reg_(REG_BLOCKS * 2048, 0),
	  bytes_(disk_bytes)
	{ }

	/* XCodecDisk::registry_write (:603-627): reads the xuid's registry block,
	 * patches the UUID in, and writes the block back to block 0 (sic). */
	void registry_write(uint16_t xuid, const uint8_t *u36)
	{
		uint8_t blk[2048];
		memcpy(blk, &reg_[(xuid / REG_ENTRIES) * 2048], 2048);
		memcpy(&blk[(xuid % REG_ENTRIES) * 36], u36, 36);
		memcpy(&reg_[0], blk, 2048);
	}

	/* XCodecDisk::local: the front of xuid 0 (registry_load establishes it;
	 * a reopened volume's local front keeps its registered UUID). */
	RefDiskCache *local(const UUID& uuid)
	{
		if (fronts_.find(0) == fronts_.end()) {
			fronts_[0] = new RefDiskCache(uuid, this, 0);
			uuid_xuid_[uuid.string_] = 0;
			if (uuid.string_.length() == 36)
				registry_write(0, (const uint8_t *)uuid.string_.data());
		}
		return fronts_[0];
	}

	/* Write the volume as the reference's would stand now. */
	bool save(const char *path) const
	{
		int fd = ::open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
		if (fd == -1)
			return false;
		bool ok = save_fd(fd);
		close(fd);
		return ok;
	}

	/* The volume file as it stands now, in an anonymous file (the descriptor
	 * the reference's XCodecDisk keeps as fd_). */
	int image_fd(void) const
	{
		int fd = memfd_create("refdisk", 0);
		if (fd == -1)
			return -1;
		if (!save_fd(fd)) {
			close(fd);
			return -1;
		}
		return fd;
	}

	/* The write head (current_index_block_, index_block_next_). */
	uint64_t head_block(void) const { return (clock_ / 204) % nb_; }
	uint64_t head_next(void) const { return clock_ % 204; }

	bool save_fd(int fd) const
	{
		bool ok = ftruncate(fd, (off_t)bytes_) == 0;
		ok = ok && pwrite(fd, &reg_[0], reg_.size(), 0) == (ssize_t)reg_.size();
		std::vector<uint8_t> ib(2048);
		for (uint64_t b = 0; ok && b < nb_; b++) {
			memset(&ib[0], 0, ib.size());
			if (ctr_[b] != 0) {
				uint8_t *q = &ib[0];
				memcpy(q, &ctr_[b], 8);
				q += 8;
				for (uint64_t j = 0; j < 204; j++, q += 10) {
					memcpy(q, &xuid_[b * 204 + j], 2);
					memcpy(q + 2, &key_[b * 204 + j], 8);
				}
			}
			ok = pwrite(fd, &ib[0], 2048, (off_t)((REG_BLOCKS + b) * 2048)) == 2048;
		}
		ok = ok && pwrite(fd, &data_[0], data_.size(), (off_t)((REG_BLOCKS + nb_) * 2048)) == (ssize_t)data_.size();
		return ok;
	}

	/* Reopen a volume (XCodecDisk::XCodecDisk, :107-237). */
	bool load(const char *path, const UUID& local_uuid)
	{
		int fd = ::open(path, O_RDONLY);
		if (fd == -1)
			return false;
		std::vector<uint8_t> vol(bytes_, 0);
		ssize_t got = pread(fd, &vol[0], vol.size(), 0);
		close(fd);
		if (got < 0)
			return false;
		memcpy(&reg_[0], &vol[0], reg_.size());
		/* registry_load (:556-601) */
		for (uint16_t xuid = 0; xuid < REG_BLOCKS * REG_ENTRIES && xuid < 1024; xuid++) {
			const uint8_t *u = &reg_[(xuid / REG_ENTRIES) * 2048 + (xuid % REG_ENTRIES) * 36];
			bool zero = true;
			for (unsigned i = 0; i < 36; i++)
				zero &= u[i] == 0;
			if (zero || !uuid_string_ok(u))
				continue;
			UUID uuid;
			uuid.string_ = std::string((const char *)u, 36);
			if (uuid_xuid_.find(uuid.string_) != uuid_xuid_.end())
				continue;
			fronts_[xuid] = new RefDiskCache(uuid, this, xuid);
			uuid_xuid_[uuid.string_] = xuid;
		}
		if (fronts_.empty())
			local(local_uuid);
		/* the index blocks' counters, in block order, to the first free one */
		std::map<uint64_t, uint64_t> cmap;
		uint64_t ibc = 0;
		for (uint64_t o = 0; o < nb_; o++) {
			uint64_t counter;
			memcpy(&counter, &vol[(REG_BLOCKS + o) * 2048], 8);
			if (counter == 0) {
				cmap[0] = o;
				break;
			}
			if (counter > ibc)
				ibc = counter + 1;
			cmap[counter] = o;
		}
		uint64_t cib = 0;
		if (!cmap.empty()) {
			cib = cmap.begin()->second;
			cmap.erase(cmap.begin());
		}
		for (uint64_t o = 0; o < nb_; o++)
			memcpy(&ctr_[o], &vol[(REG_BLOCKS + o) * 2048], 8);
		memcpy(&data_[0], &vol[(REG_BLOCKS + nb_) * 2048], data_.size());
		for (uint64_t o = 0; o < nb_; o++) {	/* the ring's slots as the file holds them */
			const uint8_t *q = &vol[(REG_BLOCKS + o) * 2048 + 8];
			for (uint64_t j = 0; j < 204; j++, q += 10) {
				memcpy(&xuid_[o * 204 + j], q, 2);
				memcpy(&key_[o * 204 + j], q + 2, 8);
				used_[o * 204 + j] = key_[o * 204 + j] != 0;
			}
		}
		unsigned leading = CHECK_BOUNDARY;
		while (!cmap.empty()) {
			bool check;
			if (leading != 0) {
				check = true;
				leading--;
			} else {
				check = cmap.size() <= CHECK_BOUNDARY;
			}
			load_entries(cmap.begin()->second, check, &cib);
			cmap.erase(cmap.begin());
		}
		/* registry_collect (:496-528) */
		for (std::map<uint16_t, RefDiskCache *>::iterator f = fronts_.begin(); f != fronts_.end();) {
			if (!f->second->index_.empty() || f->first == 0) {
				++f;
				continue;
			}
			static const uint8_t zero36[36] = {0};
			registry_write(f->first, zero36);
			uuid_xuid_.erase(f->second->get_uuid().string_);
			delete f->second;
			fronts_.erase(f++);
		}
		ibc_ = ibc == 0 ? 1 : ibc;
		clock_ = cib * 204;			/* the write head: entry 0 of block cib */
		return true;
	}

	/* XCodecDisk::index_load_entries (:408-478) on the file's image. */
	void load_entries(uint64_t b, bool check, uint64_t *cib)
	{
		for (uint64_t j = 0; j < 204; j++) {
			const uint64_t slot = b * 204 + j;
			const uint64_t hash = key_[slot];
			if (hash == 0)
				continue;
			std::map<uint16_t, RefDiskCache *>::iterator f = fronts_.find(xuid_[slot]);
			if (f == fronts_.end())
				continue;
			f->second->index_.erase(hash);		/* ("Replacing previous cache entry.") */
			if (check && XCodecHash::hash(&data_[slot * XCODEC_SEGMENT_LENGTH]) != hash) {
				if (*cib > b) {			/* rewrite the block with errors */
					invalidate(b);
					*cib = b;
					return;
				}
				continue;
			}
			f->second->index_[hash] = slot;
		}
	}

	/* XCodecDisk::index_invalidate_entries (:327-382) for block b. */
	void invalidate(uint64_t b)
	{
		if (ctr_[b] == 0)
			return;
		for (uint64_t i = b * 204; i < (b + 1) * 204; i++) {
			if (!used_[i])
				continue;
			std::map<uint16_t, RefDiskCache *>::iterator f = fronts_.find(xuid_[i]);
			if (f == fronts_.end())
				continue;
			std::map<uint64_t, uint64_t>::iterator it = f->second->index_.find(key_[i]);
			if (it == f->second->index_.end() || it->second != i)
				continue;
			f->second->index_.erase(it);
		}
	}

	RefDiskCache *connect(const UUID& uuid)
	{
		std::map<std::string, uint16_t>::const_iterator it = uuid_xuid_.find(uuid.string_);
		if (it != uuid_xuid_.end())
			return fronts_[it->second];
		uint16_t xuid;
		for (xuid = 0; xuid < 1024; xuid++)
			if (fronts_.find(xuid) == fronts_.end())
				break;
		if (xuid == 1024)
			return NULL;
		RefDiskCache *c = new RefDiskCache(uuid, this, xuid);
		fronts_[xuid] = c;
		uuid_xuid_[uuid.string_] = xuid;
		if (uuid.string_.length() == 36)
			registry_write(xuid, (const uint8_t *)uuid.string_.data());
		return c;
	}

	void enter(RefDiskCache *c, uint64_t hash, BufferSegment *seg)
	{
		ASSERT("/ref/disk", c->index_.find(hash) == c->index_.end());
		uint64_t slot = clock_ % slots_;
		seg->copyout(&data_[slot * XCODEC_SEGMENT_LENGTH], 0, XCODEC_SEGMENT_LENGTH);
		key_[slot] = hash;
		xuid_[slot] = c->xuid_;
		used_[slot] = 1;
		c->index_[hash] = slot;
		if (++clock_ % 204 == 0) {
			ctr_[(clock_ / 204 - 1) % nb_] = ibc_;	/* the filled index block is written (:708-734) */
			if (++ibc_ == 0)
				ibc_ = 1;
			uint64_t b = (clock_ / 204) % nb_;
			for (uint64_t i = b * 204; i < (b + 1) * 204; i++) {
				if (!used_[i])
					continue;
				std::map<uint16_t, RefDiskCache *>::iterator f = fronts_.find(xuid_[i]);
				if (f == fronts_.end())
					continue;
				std::map<uint64_t, uint64_t>::iterator it = f->second->index_.find(key_[i]);
				if (it == f->second->index_.end() || it->second != i)
					continue;	/* absent, or the hash lives in a newer block */
				f->second->index_.erase(it);
			}
		}
	}

	void remove(RefDiskCache *c, uint64_t hash)
	{
		c->index_.erase(hash);
	}

	BufferSegment *lookup(RefDiskCache *c, uint64_t hash)
	{
		std::map<uint64_t, uint64_t>::iterator it = c->index_.find(hash);
		if (it == c->index_.end())
			return NULL;
		BufferSegment *seg = BufferSegment::create();
		memcpy(seg->head(), &data_[it->second * XCODEC_SEGMENT_LENGTH], XCODEC_SEGMENT_LENGTH);
		seg->set_length(XCODEC_SEGMENT_LENGTH);
		if (XCodecHash::hash(seg->data()) != hash) {
			seg->unref();
			c->index_.erase(it);
			return NULL;
		}
		return seg;
	}

	uint64_t written(void) const { return clock_; }
	uint64_t live(void) const
	{
		uint64_t n = 0;
		for (std::map<uint16_t, RefDiskCache *>::const_iterator f = fronts_.begin(); f != fronts_.end(); ++f)
			n += f->second->entries();
		return n;
	}
};

XCodecCache *RefDiskCache::connect(const UUID& uuid) { return disk_->connect(uuid); }
void RefDiskCache::enter(const uint64_t& hash, BufferSegment *seg) { disk_->enter(this, hash, seg); }
void RefDiskCache::replace(const uint64_t& hash, BufferSegment *seg)
{
	disk_->remove(this, hash);
	disk_->enter(this, hash, seg);
}
BufferSegment *RefDiskCache::lookup(const uint64_t& hash) { return disk_->lookup(this, hash); }
void RefDiskCache::touch(const uint64_t& hash, BufferSegment *seg)
{
	if (index_.find(hash) == index_.end())
		disk_->enter(this, hash, seg);
}
uint64_t RefDiskCache::written(void) const { return disk_->written(); }

#ifdef XCGPU_DROPIN
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
/* Diagnostics: XCG_SEGV_TRACE=1 prints the native stack of a fatal signal. */
static void segv_trace(int sig)
{
	void *fr[64];
	int n = backtrace(fr, 64);
	backtrace_symbols_fd(fr, n, 2);
	signal(sig, SIG_DFL);
	raise(sig);
}
static const bool segv_trace_set = getenv("XCG_SEGV_TRACE") != NULL &&
    (signal(SIGSEGV, segv_trace), signal(SIGABRT, segv_trace), true);

/* The binding finds the XCodecDisk under an XCodecDiskCache by itself; this
 * harness's restated disk level is resolved here: the front's xuid and UUID,
 * and -- when the engine disk is made -- the volume file as it stands now (the
 * reference's XCodecDisk has it on disk, written block by block; RefDisk keeps
 * it in memory and writes the same image) and the write head. */
static bool ref_disk_resolver(XCodecCache *level, xcgpu_binding::DiskInfo *info, bool want_volume)
{
	RefDiskCache *front = dynamic_cast<RefDiskCache *>(level);
	if (front == NULL)
		return false;
	info->disk = front->disk();
	info->bytes = front->disk()->bytes_;
	info->xuid = front->xuid();
	info->uuid = front->get_uuid().string_;
	if (want_volume) {
		info->fd = front->disk()->image_fd();
		info->close_fd = true;
		info->head_known = true;
		info->head_block = front->disk()->head_block();
		info->head_next = front->disk()->head_next();
		if (info->fd == -1)
			return false;
	}
	return true;
}
static const bool ref_disk_resolver_set = (xcgpu_binding::set_disk_resolver(ref_disk_resolver), true);
#endif

static std::map<void *, std::pair<XCodecCache *, XCodecCache *> >& pair_levels()
{
	static std::map<void *, std::pair<XCodecCache *, XCodecCache *> > m;
	return m;
}

/* the disk front under each pair the harness made or connected */
static std::map<void *, RefDiskCache *>& pair_fronts()
{
	static std::map<void *, RefDiskCache *> m;
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
	return new XCodecMemoryCache(uuid, (size_t)limit_bytes);
}

/* XCodecCachePair(XCodecMemoryCache(uuid, memory_limit_bytes), the local front
 * of a disk of disk_bytes): wanproxy.conf's memory + disk pair
 * (programs/wanproxy/wanproxy.conf:8-26, wanproxy_config_class_cache.cc). */
void *xcr_cache_new_pair(uint64_t memory_limit_bytes, uint64_t disk_bytes)
{
	UUID uuid;
	XCodecCache *primary = new XCodecMemoryCache(uuid, (size_t)memory_limit_bytes);
	RefDisk *disk = new RefDisk(disk_bytes);
	RefDiskCache *secondary = disk->local(uuid);
	XCodecCache *pair = new XCodecCachePair(primary, secondary);
	pair_levels()[pair] = std::make_pair(primary, (XCodecCache *)NULL);
	pair_fronts()[pair] = secondary;
	return pair;
}

/* XCodecCache::connect(uuid, parent) (xcodec/xcodec_cache.h:101-111), as the
 * decoding side of XCodecPipePair makes its cache on <HELLO>
 * (xcodec/xcodec_pipe_pair.cc:203): the registered cache of that uuid, else
 * parent->connect(uuid) -- a bounded memory cache of the parent's limit, or a
 * pair of connected levels (the disk level: the uuid's front on the same
 * disk).  Such caches live for the process, as in the reference. */
void *xcr_cache_connect(void *parent, const char *uuid_string)
{
	UUID uuid;
	uuid.string_ = uuid_string;
	XCodecCache *c = XCodecCache::connect(uuid, (XCodecCache *)parent);
	std::map<void *, RefDiskCache *>::iterator f = pair_fronts().find(parent);
	if (c != NULL && f != pair_fronts().end())
		pair_fronts()[c] = f->second->disk()->connect(uuid);   /* (the front the pair's connect made) */
	return c;
}

/* wanproxy.conf's pair over a disk volume at `path` (XCodecDisk::open,
 * :824-871): reopened when the file holds one, else fresh; the local front
 * registers local_uuid on a fresh volume. */
void *xcr_cache_open_pair(uint64_t memory_limit_bytes, uint64_t disk_bytes, const char *path, const char *local_uuid)
{
	UUID uuid;
	uuid.string_ = local_uuid;
	XCodecCache *primary = new XCodecMemoryCache(uuid, (size_t)memory_limit_bytes);
	RefDisk *disk = new RefDisk(disk_bytes);
	struct stat st;
	if (::stat(path, &st) == 0 && st.st_size > 0 && !disk->load(path, uuid))
		return NULL;
	RefDiskCache *secondary = disk->local(uuid);
	XCodecCache *pair = new XCodecCachePair(primary, secondary);
	pair_levels()[pair] = std::make_pair(primary, (XCodecCache *)NULL);
	pair_fronts()[pair] = secondary;
	return pair;
}

/* A new pair (fresh bounded memory cache) over the front of `uuid` on the disk
 * under `pair` -- what a restarted process's connect(uuid) builds on a
 * reopened volume; made directly, so this process's registry of caches by
 * UUID (XCodecCache::connect's first step) does not hand back the pair an
 * earlier connect made. */
void *xcr_cache_pair_front(void *pair, const char *uuid_string, uint64_t memory_limit_bytes)
{
	std::map<void *, RefDiskCache *>::iterator f = pair_fronts().find(pair);
	if (f == pair_fronts().end())
		return NULL;
	UUID uuid;
	uuid.string_ = uuid_string;
	RefDiskCache *front = f->second->disk()->connect(uuid);
	if (front == NULL)
		return NULL;
	XCodecCache *primary = new XCodecMemoryCache(uuid, (size_t)memory_limit_bytes);
	XCodecCache *c = new XCodecCachePair(primary, front);
	pair_levels()[c] = std::make_pair(primary, (XCodecCache *)NULL);
	pair_fronts()[c] = front;
	return c;
}

/* Write the volume under a pair (the reference's file at this moment). */
int xcr_disk_save(void *pair, const char *path)
{
	std::map<void *, RefDiskCache *>::iterator f = pair_fronts().find(pair);
	if (f == pair_fronts().end())
		return -1;
	return f->second->disk()->save(path) ? 0 : -1;
}

void xcr_cache_free(void *c)
{
	RELEASE_CACHE((XCodecCache *)c);
	std::map<void *, std::pair<XCodecCache *, XCodecCache *> >::iterator it = pair_levels().find(c);
	if (it != pair_levels().end()) {       /* the pair does not own its levels (the disk stays) */
		delete it->second.first;
		pair_levels().erase(it);
	}
	pair_fronts().erase(c);
	delete (XCodecCache *)c;
}

/* XCodecPipePair's <LEARN> of one segment into a (peer) cache
 * (xcodec/xcodec_pipe_pair.cc:296-327): lookup, then replace if the bytes
 * differ, enter if absent. */
void xcr_cache_learn(void *c, const uint8_t *bytes)
{
	XCodecCache *cache = (XCodecCache *)c;
	Buffer b(bytes, XCODEC_SEGMENT_LENGTH);
	BufferSegment *seg;
	b.copyout(&seg, XCODEC_SEGMENT_LENGTH);
	uint64_t hash = XCodecHash::hash(seg->data());
	BufferSegment *oseg = cache->lookup(hash);
	if (oseg != NULL) {
		if (!oseg->equal(seg))
			cache->replace(hash, seg);
		oseg->unref();
	} else {
		cache->enter(hash, seg);
	}
	seg->unref();
}

/* Diagnostics of a pair: [0] disk index entries of its disk front, [1] disk
 * entries written (the whole disk), [2] index entries of every front. */
void xcr_pair_stats(void *c, uint64_t *st)
{
	RefDiskCache *d = pair_fronts()[c];
	st[0] = d->entries();
	st[1] = d->written();
	st[2] = d->disk()->live();
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
