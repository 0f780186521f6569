/*
 * DeflatePipe's call pattern over the SYSTEM zlib -- TEST INFRASTRUCTURE ONLY
 * (the checker tests/ and bench.py compare against; nothing in wanproxy_amd/
 * links it).
 *
 * zlib is a third-party dependency /root/reference does not vendor; this image
 * and the GPU box carry zlib 1.2.11.  What the reference adds on top of it is
 * the call pattern, and that pattern is part of the output: DeflatePipe::
 * consume (zlib/deflate_pipe.cc:57-115) runs every Buffer segment (at most
 * BUFFER_SEGMENT_SIZE = 2048 bytes, common/buffer.h:52) through
 * deflate(Z_NO_FLUSH) and then calls deflate(Z_SYNC_FLUSH) ONCE into a 64 KiB
 * stack buffer (DEFLATE_CHUNK_SIZE, :34): a Z_OK return ends the consume
 * (:101-105) even when zlib stopped because that buffer was full.  zlib then
 * keeps the rest of its output pending, and when the stop came from a block
 * flush (FLUSH_BLOCK's need_more) the sync marker is never written and the
 * positions not yet processed wait for the next consume's data.  So a consume
 * whose output crosses a 64 KiB boundary of its buffer during the flush call
 * (every 64 KiB consume of incompressible bytes) produces exactly up to that
 * boundary, and the stream goes on without a marker there.  This file restates
 * the loop (:57-115) so the real zlib runs in exactly that pattern; Python's
 * zlib module (unbounded output per call) draws other call boundaries.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define CHUNK 65536u              /* DEFLATE_CHUNK_SIZE (deflate_pipe.cc:34) */
#define SEGMENT 2048u             /* BUFFER_SEGMENT_SIZE (common/buffer.h:52) */

typedef struct { z_stream z; int done; } dpr;

dpr *dpr_create(int level) {                                  /* DeflatePipe(level), :36-48 */
    dpr *d = calloc(1, sizeof(dpr));
    if (!d) return NULL;
    if (deflateInit(&d->z, level) != Z_OK) { free(d); return NULL; }
    return d;
}

void dpr_free(dpr *d) {
    if (!d) return;
    deflateEnd(&d->z);
    free(d);
}

/* One DeflatePipe::consume of in[0..n), the Buffer's segments being seg[0..nseg)
 * (seg == NULL: SEGMENT-byte cuts).  Returns the bytes produce()d (n == 0:
 * produce_eos, Z_FINISH), or -1 (cap too small, segments not covering n, a zlib
 * error). */
int64_t dpr_consume(dpr *d, const uint8_t *in, uint64_t n, const uint32_t *seg, uint32_t nseg, uint8_t *out,
                    uint64_t cap) {
    uint8_t buf[CHUNK];
    uint64_t o = 0, pos = 0, soff = 0;
    uint32_t si = 0;
    int first = 1, err = 0;
    if (d->done) return 0;
    if (seg) {
        uint64_t t = 0;
        for (uint32_t i = 0; i < nseg; i++) t += seg[i];
        if (t != n) return -1;
    }
    d->z.avail_out = CHUNK;                                   /* :63-64 */
    d->z.next_out = buf;
    for (;;) {
        int flush;
        uint64_t slen = 0;
        if (pos == n) {                                       /* :71-77: no segment left */
            flush = first ? Z_FINISH : Z_SYNC_FLUSH;
            d->z.avail_in = 0;
            d->z.next_in = Z_NULL;
        } else {                                              /* :78-84: the first segment */
            if (seg) {
                while (seg[si] == soff) { si++; soff = 0; }  /* (empty segments) */
                slen = seg[si] - soff;
            } else {
                slen = n - pos < SEGMENT ? n - pos : SEGMENT;
            }
            flush = Z_NO_FLUSH;
            first = 0;
            d->z.avail_in = (uInt)slen;
            d->z.next_in = (Bytef *)(uintptr_t)(in + pos);
        }
        for (;;) {                                            /* :86-111 */
            int e = deflate(&d->z, flush);
            if (e == Z_OK && d->z.avail_out > 0 && flush == Z_NO_FLUSH) break;
            const uint64_t k = CHUNK - d->z.avail_out;
            if (o + k > cap) err = 1;
            else memcpy(out + o, buf, k);
            o += k;
            d->z.avail_out = CHUNK;
            d->z.next_out = buf;
            if (flush == Z_NO_FLUSH) break;
            if (flush == Z_SYNC_FLUSH && e == Z_OK) return err ? -1 : (int64_t)o;
            if (flush == Z_FINISH && e == Z_STREAM_END) {
                d->done = 1;
                return err ? -1 : (int64_t)o;
            }
            if (e != Z_OK && e != Z_BUF_ERROR) return -1;
        }
        if (slen) {                                           /* :113-114: in->skip(consumed) */
            const uint64_t used = slen - d->z.avail_in;
            pos += used;
            soff += used;
            if (seg && soff == seg[si]) { si++; soff = 0; }
        }
    }
}
