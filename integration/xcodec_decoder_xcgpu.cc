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

#ifdef XCGPU_ADAPTER_TIMING
/* (diagnostics build only: per-section host time of decode(), medians over the
 * calls, printed at exit) */
#include <stdio.h>
#include <time.h>
#include <algorithm>
namespace {
struct AdapterTiming {
	double cur[8] = {0};
	std::vector<double> t[8];
	~AdapterTiming() {
		static const char *nm[8] = {"total", "copyin", "cut", "bound", "engine", "append", "mirror", "other"};
		if (t[0].empty())
			return;
		fprintf(stderr, "decode adapter, median us per call over %zu calls:", t[0].size());
		for (int k = 0; k < 7; k++) {
			std::sort(t[k].begin(), t[k].end());
			fprintf(stderr, " %s %.2f", nm[k], t[k][t[k].size() / 2]);
		}
		fprintf(stderr, "\n");
	}
} g_at;
inline double at_now() { timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3; }
inline void at_end(double v) {
	g_at.cur[0] = v;
	for (int k = 0; k < 7; k++) {
		g_at.t[k].push_back(g_at.cur[k]);
		g_at.cur[k] = 0;
	}
}
}
#define AT_MARK(v) const double v = at_now()
#define AT_ADD(k, a, b) ((k) == 0 ? at_end((b) - (a)) : (void)(g_at.cur[k] += (b) - (a)))
#define AT_CALL() do { } while (0)
#else
#define AT_MARK(v) do { } while (0)
#define AT_ADD(k, a, b) do { } while (0)
#define AT_CALL() do { } while (0)
#endif

XCodecDecoder::XCodecDecoder(XCodecCache *cache)
: log_("/xcodec/decoder"),
  cache_(cache),
  window_()
{ }

XCodecDecoder::~XCodecDecoder()
{
	xcgpu_binding::forget_window(this);
}

/* Host cache mirror of the EXTRACTs in in[a..b) (enter / replace, :106-136).
 * hashes: their XCodecHash in op order when the engine returned them (nh of
 * them), else NULL and they are computed here. */
static void
mirror_extracts(XCodecCache *cache, const std::vector<uint8_t>& in, uint64_t a, uint64_t b,
                const uint64_t *hashes = NULL, uint32_t nh = 0)
{
	uint64_t i = a;
	uint32_t e = 0;
	while (i + 1 < b) {
		if (in[i] != XCODEC_MAGIC) {
			/* (literal bytes up to the next op: memchr, not a byte loop) */
			const uint8_t *m = (const uint8_t *)memchr(&in[i], XCODEC_MAGIC, b - i);
			if (m == NULL)
				break;
			i = (uint64_t)(m - &in[0]);
			continue;
		}
		const uint8_t op = in[i + 1];
		if (op == XCODEC_OP_EXTRACT) {
			const uint8_t *p = &in[i + 2];
			const uint64_t hash = hashes != NULL && e < nh ? hashes[e] : XCodecHash::hash(p);
			e++;
			/* one segment made straight from the input (as Buffer + copyout
			 * would, without the Buffer around it) */
			BufferSegment *seg = BufferSegment::create(p, XCODEC_SEGMENT_LENGTH);
			BufferSegment *oseg = cache->lookup(hash);
			if (oseg == NULL) {
				cache->enter(hash, seg);
			} else {
				if (!oseg->equal(seg)) {
					cache->replace(hash, seg);
					/*
					 * XCodecMemoryCache::replace stores the new entry with
					 * CacheEntry's implicit copy assignment (xcodec_cache.h:
					 * 246-269, :333-336), which takes no reference: the cache
					 * keeps a pointer the reference decoder's window and output
					 * keep alive (:137-139).  The host mirror has neither, so
					 * it keeps one reference itself (a 2 KiB segment per name
					 * reuse, never freed) rather than leave the cache dangling.
					 */
					seg->ref();
				}
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
decoded_bound(const std::vector<uint8_t>& in, uint64_t a, uint64_t b)
{
	uint64_t i = a, n = 0;
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

/*
 * Cut in[a..) into pieces of whole ops of at most XCGPU_DECODE_PIECE bytes
 * each (a bounded or pair decode batch numbers ops within 2 MiB chunks); the
 * pieces of one call form one stream, so the cut changes nothing.  piece[k] is
 * the start of piece k; the last entry is in.size().
 */
#define XCGPU_DECODE_PIECE (1u << 20)

static void
cut_pieces(const std::vector<uint8_t>& in, uint64_t a, std::vector<uint64_t>& piece)
{
	piece.clear();
	piece.push_back(a);
	uint64_t i = a;
	const uint64_t b = in.size();
	while (i < b) {
		const uint8_t *m = (const uint8_t *)memchr(&in[i], XCODEC_MAGIC, b - i);
		uint64_t at = m == NULL ? b : (uint64_t)(m - &in[0]);
		uint64_t next = at;
		if (at + 1 < b) {
			const uint8_t op = in[at + 1];
			next = at + (op == XCODEC_OP_EXTRACT ? 2 + XCODEC_SEGMENT_LENGTH :
				     op == XCODEC_OP_REF ? 10 : op == XCODEC_OP_BACKREF ? 3 : 2);
		} else {
			next = b;
		}
		if (next > b)
			next = b;
		/*
		 * Literal bytes may be cut anywhere outside an op.  The cut lies in
		 * [i, at]: i is where the last op ended, and the run [i, at) holds no
		 * 0xF1 (at is the first at or after i; an ESCAPE is an op at `at`), so
		 * every such cut is on an op boundary as it stands.
		 */
		while (at - piece.back() >= XCGPU_DECODE_PIECE)
			piece.push_back(piece.back() + XCGPU_DECODE_PIECE);
		if (next - piece.back() > XCGPU_DECODE_PIECE && at > piece.back())
			piece.push_back(at);
		i = next;
	}
	piece.push_back(b);
}

/* A cut point strictly inside piece [lo, hi) at an op boundary, or 0. */
static uint64_t
split_point(const std::vector<uint8_t>& in, uint64_t lo, uint64_t hi)
{
	const uint64_t mid = lo + (hi - lo) / 2;
	uint64_t i = lo, best = 0;
	while (i < hi) {
		const uint8_t *m = (const uint8_t *)memchr(&in[i], XCODEC_MAGIC, hi - i);
		if (m == NULL)
			break;
		const uint64_t at = (uint64_t)(m - &in[0]);
		if (at > lo && (best == 0 || at <= mid))
			best = at;
		if (at > mid && best != 0)
			break;
		if (at + 1 >= hi)
			break;
		const uint8_t op = in[at + 1];
		i = at + (op == XCODEC_OP_EXTRACT ? 2 + XCODEC_SEGMENT_LENGTH : op == XCODEC_OP_REF ? 10 :
			  op == XCODEC_OP_BACKREF ? 3 : 2);
	}
	return best;
}

bool
XCodecDecoder::decode(Buffer *output, Buffer *input, std::set<uint64_t>& unknown_hashes)
{
	if (input->empty())
		return (true);
	AT_MARK(at0);
	AT_CALL();
	xcg_ctx *ctx = xcgpu_binding::ctx_for(cache_, cache_->out_of_band());
	if (ctx == NULL)
		HALT(log_) << "xcgpu: " << xcgpu_binding::why_not(cache_) << ".";
	xcg_window *win = xcgpu_binding::window_for(this, ctx);
	if (win == NULL)
		HALT(log_) << "No device memory for the XCodec window.";

	/* call scratch kept across calls (a std::vector zero-fills what it grows:
	 * per call that was 512 KiB of unknown-hash room alone) */
	static thread_local std::vector<uint8_t> in, out;
	static thread_local std::vector<uint64_t> unk, ext;
	const uint64_t len = input->length();
	in.resize(len);			/* (shrinking keeps the storage; growing fills only the new tail) */
	AT_MARK(at1);
	input->copyout(&in[0], len);
	AT_MARK(at2);
	AT_ADD(1, at1, at2);
	if (unk.size() < (1u << 16)) {
		unk.resize(1u << 16);
		ext.resize(1024);
	}
	std::vector<uint64_t> piece, coff, ooff, olen, cons;
	std::vector<uint32_t> clen;
	std::vector<int32_t> cst;
	uint64_t pos = 0, batch_end = 0;
	int32_t status = 0;
	uint32_t nunk = 0;
	xcg_decode_set_window(ctx, win);
	AT_MARK(at3);
	/*
	 * The GPU decodes from pos until the end, a bad op, or a REF its cache
	 * does not hold.  In the last case the hashes the host cache learned
	 * (ASK/LEARN, xcodec/xcodec_pipe_pair.cc:274-333) go to the GPU and the
	 * decode continues from the blocking REF, as decode() itself would with
	 * those hashes in its cache; what stays unknown is returned like
	 * decode_skim (:196-272).  A batch the engine declines (XCG_ENOTSUP: on a
	 * bounded or pair cache, more cache references than one batch models) is
	 * decoded as successive smaller batches -- the same stream, so the same
	 * result.
	 */
	cut_pieces(in, pos, piece);
	AT_MARK(at4);
	AT_ADD(2, at3, at4);
	size_t k0 = 0, per = piece.size() - 1;
	for (;;) {
		const size_t k1 = k0 + per < piece.size() - 1 ? k0 + per : piece.size() - 1;
		const uint32_t n = (uint32_t)(k1 - k0);
		coff.resize(n); clen.resize(n); ooff.resize(n); olen.resize(n); cons.resize(n); cst.resize(n);
		for (uint32_t j = 0; j < n; j++) {
			coff[j] = piece[k0 + j] - pos;
			clen[j] = (uint32_t)(piece[k0 + j + 1] - piece[k0 + j]);
		}
		const uint64_t span = piece[k1] - pos;
		AT_MARK(at5);
		out.resize(decoded_bound(in, pos, piece[k1]) + 1);
		AT_MARK(at6);
		AT_ADD(3, at5, at6);
		nunk = 0;
		int rc;
		uint32_t next = XCG_NO_REFERENCES;
		if (n == 1) {		/* one launch, one synchronisation (xcg_decode_call) */
			ooff[0] = 0;
			rc = xcg_decode_call(ctx, &in[pos], clen[0], &out[0], out.size(), &olen[0], &cons[0], &cst[0],
			                     &unk[0], unk.size(), &nunk, &ext[0], ext.size(), &next);
		} else {
			rc = xcg_decode_host(ctx, &in[pos], span, &coff[0], &clen[0], n, &out[0], out.size(), &ooff[0],
			                     &olen[0], &cst[0], &cons[0], &unk[0], unk.size(), &nunk);
		}
		AT_MARK(at7);
		AT_ADD(4, at6, at7);
		if (rc == XCG_ENOTSUP) {
			if (n > 1) {
				per = n / 2;
				continue;
			}
			const uint64_t c = split_point(in, piece[k0], piece[k0 + 1]);
			if (c == 0) {
				xcg_decode_set_window(ctx, NULL);
				HALT(log_) << "xcgpu decode: " << xcg_strerror(rc) << " (an op the engine does not model on "
				           << "this cache).";
			}
			piece.insert(piece.begin() + k0 + 1, c);
			per = 1;
			continue;
		}
		if (rc != XCG_OK) {
			xcg_decode_set_window(ctx, NULL);
			HALT(log_) << "xcgpu decode failed: " << xcg_strerror(rc);
		}
		batch_end = piece[k1];
		/* the pieces decoded, in order, up to the first that stopped */
		uint64_t consumed = 0;
		status = 0;
		for (uint32_t j = 0; j < n; j++) {
			if (cst[j] == 2)
				break;
			if (olen[j])
				output->append(&out[ooff[j]], olen[j]);
			consumed += cons[j];
			if (cst[j] != 0) {
				status = cst[j];
				break;
			}
		}
		AT_MARK(at8);
		AT_ADD(5, at7, at8);
		mirror_extracts(cache_, in, pos, pos + consumed, next == XCG_NO_REFERENCES ? NULL : &ext[0],
		                next == XCG_NO_REFERENCES ? 0 : next);
		AT_MARK(at9);
		AT_ADD(6, at8, at9);
		pos += consumed;
		if (status == 0 && k1 < piece.size() - 1) {	/* more batches of this call */
			k0 = k1;
			continue;
		}
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
		cut_pieces(in, pos, piece);
		k0 = 0;
		per = piece.size() - 1;
	}
	if (status == 1 && batch_end < len) {
		/*
		 * The stop fell in a batch that ended before the input did: the
		 * engine skimmed up to batch_end.  decode_skim's lookups go on to the
		 * end (:196-272), so the rest is decoded behind a REF no cache can
		 * hold -- bits 32..35 of a real XCodecHash are always clear (mix()
		 * shifts bits_hash by 36) -- which stops the batch at its first op and
		 * leaves only the skim.
		 */
		std::vector<uint8_t> rest(10 + (len - batch_end));
		static const uint64_t NOHASH = 0x0000000F00000000ull;
		rest[0] = XCODEC_MAGIC;
		rest[1] = XCODEC_OP_REF;
		for (int b = 0; b < 8; b++)
			rest[2 + b] = (uint8_t)(NOHASH >> (56 - 8 * b));
		memcpy(&rest[10], &in[batch_end], len - batch_end);
		cut_pieces(rest, 0, piece);
		const uint32_t n = (uint32_t)(piece.size() - 1);
		coff.resize(n); clen.resize(n); ooff.resize(n); olen.resize(n); cons.resize(n); cst.resize(n);
		for (uint32_t j = 0; j < n; j++) {
			coff[j] = piece[j];
			clen[j] = (uint32_t)(piece[j + 1] - piece[j]);
		}
		std::vector<uint64_t> unk2(unk.size());
		uint32_t nunk2 = 0;
		uint8_t dummy[16];
		int rc = xcg_decode_host(ctx, &rest[0], rest.size(), &coff[0], &clen[0], n, dummy, sizeof dummy, &ooff[0],
		                         &olen[0], &cst[0], &cons[0], &unk2[0], unk2.size(), &nunk2);
		if (rc != XCG_OK || cst[0] != 1) {
			xcg_decode_set_window(ctx, NULL);
			HALT(log_) << "xcgpu decode: skim of the rest failed: " << xcg_strerror(rc);
		}
		for (uint32_t k = 0; k < nunk2 && nunk < unk.size(); k++)
			if (unk2[k] != NOHASH)
				unk[nunk++] = unk2[k];
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
	AT_MARK(at10);
	AT_ADD(0, at0, at10);
	return (status >= 0);
}
