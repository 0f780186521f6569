/*
 * xcodec_encoder_xcgpu.cc -- XCodecEncoder (xcodec/xcodec_encoder.h:35-49)
 * implemented on the MI355X engine.  Drop-in replacement for
 * xcodec/xcodec_encoder.cc: same class, same header, same callers
 * (programs/tack/tack.cc:301-313, xcodec/xcodec_pipe_pair.cc:574-618).
 *
 * encode() flattens the input Buffer, runs one XCG_SEM_STREAM encode() on the
 * GPU against the cache's GPU mirror, appends the bytes, then reproduces the
 * reference's side effects on the host objects: the declarations enter the
 * XCodecCache (encode_declaration, :284-286) and every REF target enters the
 * refmap once (encode_reference, :364-371).
 */
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
		HALT(log_) << "No MI355X device for the XCodec engine.";

	const uint32_t len = input->length();
	std::vector<uint8_t> in(len);
	input->moveout(&in[0], len);

	const uint64_t off = 0;
	const uint64_t ooff = 0;
	uint64_t olen = 0;
	std::vector<uint8_t> out(xcg_encode_bound(len));
	int rc = xcg_encode_host(ctx, XCG_SEM_STREAM, &in[0], len, &off, &len, 1, &out[0], out.size(), &ooff, &olen);
	if (rc != XCG_OK)
		HALT(log_) << "xcgpu encode failed: " << xcg_strerror(rc);
	output->append(&out[0], olen);

	/* Declarations made by this call, mirrored into the host cache. */
	uint32_t ndecl = 0;
	std::vector<uint64_t> dh(len / XCODEC_SEGMENT_LENGTH + 1);
	std::vector<uint32_t> dp(dh.size());
	if (!xcgpu_binding::is_null_cache(cache_)) {
		rc = xcg_last_declarations(ctx, 0, &dh[0], &dp[0], dh.size(), &ndecl);
		if (rc != XCG_OK)
			HALT(log_) << "xcgpu declarations: " << xcg_strerror(rc);
	}
	std::map<uint64_t, unsigned> declared;
	for (uint32_t i = 0; i < ndecl; i++) {
		BufferSegment *seg = segment_of(&in[dp[i]]);
		cache_->enter(dh[i], seg);
		seg->unref();
		declared[dh[i]] = dp[i];
	}

	if (refmap == NULL)
		return;
	/* REF ops of the output.  An out-of-band declaration looks like a REF and
	 * comes first in the output for its hash (a REF to it can only follow);
	 * encode_declaration passes no refmap (xcodec_encoder.cc:288-295), so that
	 * first occurrence is skipped, later ones are REFs. */
	uint64_t i = 0;
	while (i < olen) {
		if (out[i] != XCODEC_MAGIC) {
			i++;
			continue;
		}
		const uint8_t op = out[i + 1];
		if (op == XCODEC_OP_ESCAPE) {
			i += 2;
		} else if (op == XCODEC_OP_EXTRACT) {
			i += 2 + XCODEC_SEGMENT_LENGTH;
		} else {
			uint64_t behash;
			memcpy(&behash, &out[i + 2], sizeof behash);
			const uint64_t hash = BigEndian::decode(behash);
			i += 10;
			if (!stream_) {
				std::map<uint64_t, unsigned>::iterator dit = declared.find(hash);
				if (dit != declared.end()) {
					declared.erase(dit);
					continue;
				}
			}
			if (refmap->find(hash) != refmap->end())
				continue;
			BufferSegment *seg = cache_->lookup(hash);
			if (seg == NULL)
				HALT(log_) << "REF target missing from the cache mirror.";
			refmap->insert(std::map<uint64_t, BufferSegment *>::value_type(hash, seg));
		}
	}
}
