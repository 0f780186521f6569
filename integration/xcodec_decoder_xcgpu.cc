/*
 * xcodec_decoder_xcgpu.cc -- XCodecDecoder (xcodec/xcodec_decoder.h:35-45)
 * implemented on the MI355X engine.  Drop-in replacement for
 * xcodec/xcodec_decoder.cc.
 *
 * decode() runs the GPU decoder over the whole input.  Hashes the GPU cache
 * does not know but the host cache does (entered by ASK/LEARN,
 * xcodec/xcodec_pipe_pair.cc:274-333) are pushed to the GPU and the call is
 * retried; what remains unknown is returned like decode_skim (:196-272).
 * EXTRACTs are mirrored into the host cache (enter / replace, :106-136).
 */
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
{ }

bool
XCodecDecoder::decode(Buffer *output, Buffer *input, std::set<uint64_t>& unknown_hashes)
{
	if (input->empty())
		return (true);
	xcg_ctx *ctx = xcgpu_binding::ctx_for(cache_, cache_->out_of_band());
	if (ctx == NULL)
		HALT(log_) << "No MI355X device for the XCodec engine.";

	const uint32_t len = input->length();
	std::vector<uint8_t> in(len);
	input->copyout(&in[0], len);
	const uint64_t off = 0;
	uint64_t ooff = 0, olen = 0, consumed = 0;
	int32_t status = 0;
	std::vector<uint8_t> out((uint64_t)len * 205 + 4096);
	std::vector<uint64_t> unk(1u << 16);
	uint32_t nunk = 0;
	for (;;) {
		int rc = xcg_decode_host(ctx, &in[0], len, &off, &len, 1, &out[0], out.size(), &ooff, &olen, &status,
		                         &consumed, &unk[0], unk.size(), &nunk);
		if (rc != XCG_OK)
			HALT(log_) << "xcgpu decode failed: " << xcg_strerror(rc);
		if (status != 1)
			break;
		/* Blocked: anything the host cache learned since goes to the GPU. */
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

	/* Mirror the consumed EXTRACTs into the host cache. */
	uint64_t i = 0;
	while (i + 1 < consumed) {
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
			BufferSegment *oseg = cache_->lookup(hash);
			if (oseg == NULL) {
				cache_->enter(hash, seg);
			} else {
				if (!oseg->equal(seg))
					cache_->replace(hash, seg);
				oseg->unref();
			}
			window_.declare(hash, seg);
			seg->unref();
			i += 2 + XCODEC_SEGMENT_LENGTH;
		} else if (op == XCODEC_OP_REF) {
			i += 10;
		} else if (op == XCODEC_OP_BACKREF) {
			i += 3;
		} else {
			i += 2;
		}
	}

	output->append(&out[0], olen);
	input->skip(consumed);
	if (status == 1) {
		for (uint32_t k = 0; k < nunk; k++)
			unknown_hashes.insert(unk[k]);
		return (true);
	}
	return (status >= 0);
}
