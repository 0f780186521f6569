/*
 * xcodec_encoder_xcgpu.cc -- XCodecEncoder (xcodec/xcodec_encoder.h:35-49)
 * implemented on the MI355X engine.  Drop-in replacement for
 * xcodec/xcodec_encoder.cc: same class, same header, same callers
 * (programs/tack/tack.cc:301-313, xcodec/xcodec_pipe_pair.cc:574-618).
 *
 * encode() flattens the input Buffer, runs one XCG_SEM_STREAM encode() on the
 * GPU against the cache's GPU mirror, appends the bytes, then reproduces the
 * reference's side effects on the host objects: the call's cache references
 * are replayed into the XCodecCache in stream order (enters,
 * encode_declaration :284-286, and -- on a bounded or pair cache, where they
 * change the cache -- lookups, find_reference :374-416), and every REF target
 * enters the refmap once, its segment taken from the input at the REF
 * (encode_reference, :364-371).
 */
#include <set>
#include <vector>

#include <common/buffer.h>
#include <common/endian.h>

#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_encoder.h>
#include <xcodec/xcodec_hash.h>

#include "xcgpu_binding.h"

XCodecEncoder::XCodecEncoder(XCodecCache *cache)
: log_("/xcodec/encoder"),
  cache_(cache),
  window_(),
  stream_(!cache_->out_of_band())
{ }

XCodecEncoder::~XCodecEncoder()
{ }

static BufferSegment *
segment_of(const uint8_t *p)
{
	Buffer tmp(p, XCODEC_SEGMENT_LENGTH);
	BufferSegment *seg;
	tmp.copyout(&seg, XCODEC_SEGMENT_LENGTH);
	return (seg);
}

void
XCodecEncoder::encode(Buffer *output, Buffer *input, std::map<uint64_t, BufferSegment *> *refmap)
{
	if (input->empty())
		return;

	xcg_ctx *ctx = xcgpu_binding::ctx_for(cache_, !stream_);
	if (ctx == NULL)
		HALT(log_) << "xcgpu: " << xcgpu_binding::why_not(cache_) << ".";

	const uint32_t len = input->length();
	if (len > XCGPU_MAX_ENCODE)
		HALT(log_) << "xcgpu encode: " << len << " bytes in one encode() call; the engine takes at most "
		           << XCGPU_MAX_ENCODE << " (XCodecPipePair frames are <= 512 KiB, tack reads 64 KiB).";
	std::vector<uint8_t> in(len);
	input->moveout(&in[0], len);

	/*
	 * One engine call: the output, the call's declarations in order
	 * (encode_declaration, :276-313) and, on a bounded or pair cache, its
	 * cache references in stream order -- one host synchronisation.
	 */
	uint64_t olen = 0;
	std::vector<uint8_t> out(xcg_encode_bound(len));
	uint32_t ndecl = 0, nref = 0;
	std::vector<uint64_t> dh(len / XCODEC_SEGMENT_LENGTH + 1);
	std::vector<uint32_t> dp(dh.size());
	std::vector<uint64_t> rh(2 * dh.size() + 64);
	std::vector<uint32_t> rk(rh.size()), rr(rh.size());
	int rc = xcg_encode_call(ctx, &in[0], len, &out[0], out.size(), &olen, &dh[0], &dp[0], dh.size(), &ndecl,
	                         &rh[0], &rk[0], &rr[0], rh.size(), &nref);
	if (rc != XCG_OK)
		HALT(log_) << "xcgpu encode failed: " << xcg_strerror(rc);
	if (ndecl > dh.size())
		HALT(log_) << "xcgpu declarations: list overflow.";
	output->append(&out[0], olen);

	/*
	 * The host cache mirror.  On a bounded or pair cache every lookup that
	 * found its hash changed the cache (LRU refresh, promotion, disk
	 * re-enter, xcodec/xcodec_cache.h:208-230, :348-364), so the call's cache
	 * references are replayed in stream order; on an unbounded memory cache
	 * only the enters matter.
	 */
	if (xcgpu_binding::is_null_cache(cache_)) {
		/* TackNullCache: nothing to keep. */
	} else if (nref != XCG_NO_REFERENCES) {
		if (nref > rh.size())
			HALT(log_) << "xcgpu references: list overflow.";
		for (uint32_t i = 0; i < nref; i++) {
			if (rk[i] == 0) {
				if (rr[i] >= ndecl)
					HALT(log_) << "xcgpu references: unknown declaration.";
				BufferSegment *seg = segment_of(&in[dp[rr[i]]]);
				cache_->enter(dh[rr[i]], seg);
				seg->unref();
			} else {
				BufferSegment *seg = cache_->lookup(rh[i]);
				if (seg != NULL)
					seg->unref();
			}
		}
	} else {
		for (uint32_t i = 0; i < ndecl; i++) {
			BufferSegment *seg = segment_of(&in[dp[i]]);
			cache_->enter(dh[i], seg);
			seg->unref();
		}
	}

	if (refmap == NULL)
		return;
	/*
	 * REF ops of the output, each with the input offset it stands for: the
	 * refmap segment is the input there (a REF is only emitted on byte
	 * equality, xcodec_encoder.cc:382-390), entered once per hash
	 * (encode_reference, :364-371).  An out-of-band declaration is written as
	 * F1 02 too, but encode_declaration passes no refmap (:288-295): those
	 * (offset, hash) pairs are skipped.
	 */
	std::set<std::pair<uint64_t, uint64_t> > declared;
	if (!stream_)
		for (uint32_t i = 0; i < ndecl; i++)
			declared.insert(std::make_pair((uint64_t)dp[i], dh[i]));
	uint64_t i = 0, pos = 0;
	while (i < olen) {
		if (out[i] != XCODEC_MAGIC) {
			i++;
			pos++;
			continue;
		}
		const uint8_t op = out[i + 1];
		if (op == XCODEC_OP_ESCAPE) {
			i += 2;
			pos++;
		} else if (op == XCODEC_OP_EXTRACT) {
			i += 2 + XCODEC_SEGMENT_LENGTH;
			pos += XCODEC_SEGMENT_LENGTH;
		} else {
			uint64_t behash;
			memcpy(&behash, &out[i + 2], sizeof behash);
			const uint64_t hash = BigEndian::decode(behash);
			const uint64_t at = pos;
			i += 10;
			pos += XCODEC_SEGMENT_LENGTH;
			if (declared.count(std::make_pair(at, hash)) != 0)
				continue;
			if (refmap->find(hash) != refmap->end())
				continue;
			refmap->insert(std::map<uint64_t, BufferSegment *>::value_type(hash, segment_of(&in[at])));
		}
	}
}
