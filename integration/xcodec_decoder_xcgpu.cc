/*
 * xcodec_decoder_xcgpu.cc -- XCodecDecoder (xcodec/xcodec_decoder.h:35-45)
 * implemented on the MI355X engine.  Drop-in replacement for
 * xcodec/xcodec_decoder.cc.
 *
 * decode() runs the GPU decoder over the whole input.  Hashes the GPU cache
 * does not know but the host cache does (entered by ASK/LEARN,
 * xcodec/xcodec_pipe_pair.cc:274-333) are pushed to the GPU and the call is
 * retried; what remains unknown is returned like decode_skim (:196-272).
 * The call's cache references are mirrored into the host cache in stream
 * order: EXTRACT lookup + enter / replace (:106-136), REF lookups (:151-162)
 * and, when blocked, decode_skim's lookups (:196-272) -- on a bounded cache
 * each lookup that finds its hash refreshes it, so the host cache then holds
 * what the engine's does.
 */
#include <string.h>

#include <set>
#include <vector>

#include <common/buffer.h>
#include <common/endian.h>

#include <xcodec/xcodec.h>
#include <xcodec/xcodec_cache.h>
#include <xcodec/xcodec_decoder.h>
#include <xcodec/xcodec_hash.h>

#include "xcgpu_binding.h"

XCodecDecoder::XCodecDecoder(XCodecCache *cache)
: log_("/xcodec/decoder"),
  cache_(cache),
  window_()
{ }

XCodecDecoder::~XCodecDecoder()
{
	xcgpu_binding::forget_window(this);
}

/* Host cache mirror of the EXTRACTs in in[a..b) (enter / replace, :106-136). */
static void
mirror_extracts(XCodecCache *cache, const std::vector<uint8_t>& in, uint64_t a, uint64_t b)
{
	uint64_t i = a;
	while (i + 1 < b) {
		if (in[i] != XCODEC_MAGIC) {
			i++;
			continue;
		}
		const uint8_t op = in[i + 1];
		if (op == XCODEC_OP_EXTRACT) {
			const uint8_t *p = &in[i + 2];
			const uint64_t hash = XCodecHash::hash(p);
			Buffer tmp(p, XCODEC_SEGMENT_LENGTH);
			BufferSegment *seg;
			tmp.copyout(&seg, XCODEC_SEGMENT_LENGTH);
			BufferSegment *oseg = cache->lookup(hash);
			if (oseg == NULL) {
				cache->enter(hash, seg);
			} else {
				if (!oseg->equal(seg))
					cache->replace(hash, seg);
				oseg->unref();
			}
			seg->unref();
			i += 2 + XCODEC_SEGMENT_LENGTH;
		} else if (op == XCODEC_OP_REF) {
			/* :151-162: the REF's lookup refreshes a bounded cache's entry */
			uint64_t behash;
			memcpy(&behash, &in[i + 2], sizeof behash);
			BufferSegment *oseg = cache->lookup(BigEndian::decode(behash));
			if (oseg != NULL)
				oseg->unref();
			i += 10;
		} else if (op == XCODEC_OP_BACKREF) {
			i += 3;
		} else {
			i += 2;
		}
	}
}

/* decode_skim's lookups (:196-272) of the REFs from the blocking point on. */
static void
mirror_skim(XCodecCache *cache, const std::vector<uint8_t>& in, uint64_t a)
{
	uint64_t i = a;
	const uint64_t b = in.size();
	while (i + 1 < b) {
		if (in[i] != XCODEC_MAGIC) {
			i++;
			continue;
		}
		const uint8_t op = in[i + 1];
		if (op == XCODEC_OP_ESCAPE) {
			i += 2;
		} else if (op == XCODEC_OP_EXTRACT) {
			if (b - i < 2 + XCODEC_SEGMENT_LENGTH)
				return;
			i += 2 + XCODEC_SEGMENT_LENGTH;
		} else if (op == XCODEC_OP_REF) {
			if (b - i < 10)
				return;
			uint64_t behash;
			memcpy(&behash, &in[i + 2], sizeof behash);
			BufferSegment *oseg = cache->lookup(BigEndian::decode(behash));
			if (oseg != NULL)
				oseg->unref();
			i += 10;
		} else if (op == XCODEC_OP_BACKREF) {
			if (b - i < 3)
				return;
			i += 3;
		} else {
			return;
		}
	}
}

/* Decoded size of in[a..) if every op resolves: literal and escaped bytes one
 * each, EXTRACT / REF / BACKREF one segment each (:73-185). */
static uint64_t
decoded_bound(const std::vector<uint8_t>& in, uint64_t a)
{
	uint64_t i = a, n = 0;
	const uint64_t b = in.size();
	while (i < b) {
		const uint8_t *m = (const uint8_t *)memchr(&in[i], XCODEC_MAGIC, b - i);
		if (m == NULL)
			return n + (b - i);
		const uint64_t at = (uint64_t)(m - &in[0]);
		n += at - i;
		i = at;
		if (i + 1 >= b)
			return n;
		const uint8_t op = in[i + 1];
		if (op == XCODEC_OP_ESCAPE) {
			n += 1;
			i += 2;
		} else if (op == XCODEC_OP_EXTRACT) {
			n += XCODEC_SEGMENT_LENGTH;
			i += 2 + XCODEC_SEGMENT_LENGTH;
		} else if (op == XCODEC_OP_REF) {
			n += XCODEC_SEGMENT_LENGTH;
			i += 10;
		} else if (op == XCODEC_OP_BACKREF) {
			n += XCODEC_SEGMENT_LENGTH;
			i += 3;
		} else {
			return n;
		}
	}
	return n;
}

bool
XCodecDecoder::decode(Buffer *output, Buffer *input, std::set<uint64_t>& unknown_hashes)
{
	if (input->empty())
		return (true);
	xcg_ctx *ctx = xcgpu_binding::ctx_for(cache_, cache_->out_of_band());
	if (ctx == NULL)
		HALT(log_) << "No MI355X device for the XCodec engine.";
	xcg_window *win = xcgpu_binding::window_for(this, ctx);
	if (win == NULL)
		HALT(log_) << "No device memory for the XCodec window.";

	const uint32_t len = input->length();
	std::vector<uint8_t> in(len);
	input->copyout(&in[0], len);
	std::vector<uint8_t> out;
	std::vector<uint64_t> unk(1u << 16);
	uint64_t pos = 0;
	int32_t status = 0;
	uint32_t nunk = 0;
	xcg_decode_set_window(ctx, win);
	/*
	 * The GPU decodes from pos until the end, a bad op, or a REF its cache
	 * does not hold.  In the last case the hashes the host cache learned
	 * (ASK/LEARN, xcodec/xcodec_pipe_pair.cc:274-333) go to the GPU and the
	 * decode continues from the blocking REF, as decode() itself would with
	 * those hashes in its cache; what stays unknown is returned like
	 * decode_skim (:196-272).
	 */
	for (;;) {
		const uint64_t off = 0;
		const uint32_t rest = (uint32_t)(len - pos);
		uint64_t ooff = 0, olen = 0, consumed = 0;
		out.resize(decoded_bound(in, pos) + 1);
		int rc = xcg_decode_host(ctx, &in[pos], rest, &off, &rest, 1, &out[0], out.size(), &ooff, &olen, &status,
		                         &consumed, &unk[0], unk.size(), &nunk);
		if (rc != XCG_OK) {
			xcg_decode_set_window(ctx, NULL);
			HALT(log_) << "xcgpu decode failed: " << xcg_strerror(rc);
		}
		mirror_extracts(cache_, in, pos, pos + consumed);
		output->append(&out[0], olen);
		pos += consumed;
		if (status != 1 || pos >= len)
			break;
		unsigned pushed = 0;
		for (uint32_t k = 0; k < nunk; k++) {
			BufferSegment *seg = cache_->lookup(unk[k]);
			if (seg == NULL)
				continue;
			xcg_cache_enter_host(ctx, unk[k], seg->data());
			seg->unref();
			pushed++;
		}
		if (pushed == 0)
			break;
	}
	xcg_decode_set_window(ctx, NULL);

	input->skip(pos);
	if (status == 1) {
		mirror_skim(cache_, in, pos);
		for (uint32_t k = 0; k < nunk; k++) {
			BufferSegment *seg = cache_->lookup(unk[k]);
			if (seg != NULL) {
				seg->unref();
				continue;
			}
			unknown_hashes.insert(unk[k]);
		}
		return (true);
	}
	return (status >= 0);
}
