/*
 * zlib stage oracle -- TEST INFRASTRUCTURE ONLY (tests/, smoke() and bench.py's
 * cpu_baseline may use it; nothing in wanproxy_amd/ links it).
 *
 * What it restates.  wanproxy chains a DeflatePipe after the XCodec encoder
 * (programs/wanproxy/wanproxy_codec_pipe_pair.cc:97-106,148-157).  Its
 * consume() (zlib/deflate_pipe.cc:57-115) feeds every input segment to
 * deflate(Z_NO_FLUSH) and then calls deflate(Z_SYNC_FLUSH) -- or deflate(
 * Z_FINISH) when the consumed buffer is empty (EOS).  The compressor itself is
 * zlib, a third-party dependency that /root/reference does not vendor; this
 * image (and the GPU box) carries zlib 1.2.11, the pinned version checked
 * here.  This file restates zlib 1.2.11's deflate for windowBits 15, memLevel
 * 8, Z_DEFAULT_STRATEGY, levels 4-9 (deflateInit(level), deflate_pipe.cc:45;
 * levels 1-3 run deflate_fast, whose hash insertion depends on the parse, and
 * level 0 deflate_stored -- neither is restated):
 *   - deflate.c: configuration_table, deflate() header / flush / trailer,
 *     fill_window() (window slides), longest_match(),
 *     deflate_slow() (levels 4-9: lazy matching; wanproxy.conf sets 6)
 *   - trees.c: _tr_tally, _tr_flush_block (stored / static / dynamic choice),
 *     build_tree / gen_bitlen / gen_codes, scan_tree / send_tree,
 *     build_bl_tree, send_all_trees, compress_block, _tr_stored_block.
 * It is written in the formulation the GPU kernels use (wanproxy_amd/csrc/
 * xcg_deflate.hip): a call's bytes are hashed at every position, every
 * position's hash chain is walked up front ("match table": best length and
 * first position reaching it, for the full and the quartered chain budget),
 * and a sequential scan then replays deflate_slow's decisions over that
 * table.  zlib's 64 KiB window itself is never materialised: only its slides
 * (which make coord 0 NIL and decide whether a block can still be stored) are
 * tracked, and what longest_match reads past the data cannot change its
 * result (walk()).  Per stream only the last 32 KiB of input persist.  Why the input's
 * segmentation into deflate(Z_NO_FLUSH) calls cannot change the output: every
 * position deflate processes under Z_NO_FLUSH has >= MIN_LOOKAHEAD bytes of
 * lookahead and the window slides at the first loop top past strstart 65274
 * whatever the segment sizes (checked against zlib with random segmentations
 * in tests/test_zlib_oracle.py).
 *
 * Pinning: tests/test_zlib_oracle.py compares every call's output with the
 * system zlib 1.2.11 driven in DeflatePipe's call pattern
 * (oracle/zlib_pipe.py), and with fixtures it produced (tests/golden/zlib.json).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define WSIZE 32768u
#define WINSZ 65536u
#define MIN_MATCH 3
#define MAX_MATCH 258
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1)   /* deflate.h */
#define MAX_DIST (WSIZE - MIN_LOOKAHEAD)             /* 32506 */
#define TOO_FAR 4096
#define LIT_BUFSIZE 16384u                           /* 1 << (memLevel + 6) */
#define NONE UINT64_MAX

#define L_CODES 286
#define D_CODES 30
#define BL_CODES 19
#define HEAP_SIZE (2 * L_CODES + 1)
#define MAX_BITS 15
#define END_BLOCK 256

/* configuration_table (deflate.c): good, lazy, nice, chain */
static const int CFG[10][4] = {
    {0, 0, 0, 0},        {4, 4, 8, 4},         {4, 5, 16, 8},       {4, 6, 32, 32},
    {4, 4, 16, 16},      {8, 16, 32, 32},      {8, 16, 128, 128},   {8, 32, 128, 256},
    {32, 128, 258, 1024}, {32, 258, 258, 4096}};

static const int XLB[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const int XDB[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const int XBB[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t BL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static uint8_t len_code[256], dist_code[512];
static int base_len[29], base_dist[30];
static uint16_t st_lcode[288], st_llen[288], st_dcode[30];
static int tables_ready;

static unsigned bitrev(unsigned c, int n) {
    unsigned r = 0;
    while (n-- > 0) { r = (r << 1) | (c & 1); c >>= 1; }
    return r;
}

/* trees.c tr_static_init: length / distance code maps and the fixed trees */
static void init_tables(void) {
    if (tables_ready) return;
    int l = 0, code;
    for (code = 0; code < 28; code++) {
        base_len[code] = l;
        for (int n = 0; n < (1 << XLB[code]); n++) len_code[l++] = (uint8_t)code;
    }
    len_code[255] = 28;              /* length 258: code 285, no extra bits */
    base_len[28] = 0;
    int d = 0;
    for (code = 0; code < 16; code++) {
        base_dist[code] = d;
        for (int n = 0; n < (1 << XDB[code]); n++) dist_code[d++] = (uint8_t)code;
    }
    d >>= 7;
    for (; code < D_CODES; code++) {
        base_dist[code] = d << 7;
        for (int n = 0; n < (1 << (XDB[code] - 7)); n++) dist_code[256 + d++] = (uint8_t)code;
    }
    int cnt[MAX_BITS + 1] = {0};
    for (int n = 0; n < 288; n++) {
        st_llen[n] = n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8;
        cnt[st_llen[n]]++;
    }
    unsigned next[MAX_BITS + 1], c = 0;
    for (int b = 1; b <= MAX_BITS; b++) { c = (c + cnt[b - 1]) << 1; next[b] = c; }
    for (int n = 0; n < 288; n++) st_lcode[n] = (uint16_t)bitrev(next[st_llen[n]]++, st_llen[n]);
    for (int n = 0; n < D_CODES; n++) st_dcode[n] = (uint16_t)bitrev(n, 5);
    tables_ready = 1;
}

static int d_code(unsigned dist) { return dist < 256 ? dist_code[dist] : dist_code[256 + (dist >> 7)]; }

/* ------------------------------------------------------------------ bits */
typedef struct { uint8_t *p; uint64_t n, cap; uint64_t acc; int nb; int err; } Bits;

static void put_byte(Bits *b, uint8_t v) {
    if (b->n < b->cap) b->p[b->n] = v; else b->err = 1;
    b->n++;
}
static void put_bits(Bits *b, unsigned v, int n) {      /* LSB first, as send_bits */
    b->acc |= (uint64_t)v << b->nb;
    b->nb += n;
    while (b->nb >= 8) { put_byte(b, (uint8_t)b->acc); b->acc >>= 8; b->nb -= 8; }
}
static void windup(Bits *b) {                           /* bi_windup */
    if (b->nb > 0) put_byte(b, (uint8_t)b->acc);
    b->acc = 0; b->nb = 0;
}

/* ------------------------------------------------------------------ trees */
typedef struct { uint16_t fc; uint16_t dl; } ct;         /* Freq|Code, Dad|Len */

typedef struct {
    ct lt[HEAP_SIZE], dt[2 * D_CODES + 1], bt[2 * BL_CODES + 1];
    int heap[2 * L_CODES + 1], heap_len, heap_max;
    uint8_t depth[2 * L_CODES + 1];
    int bl_count[MAX_BITS + 1];
    uint64_t opt_len, static_len;
    int lmax, dmax;
} Trees;

#define SMALLER(t, n, m, dep) ((t)[n].fc < (t)[m].fc || ((t)[n].fc == (t)[m].fc && (dep)[n] <= (dep)[m]))

static void downheap(Trees *s, ct *t, int k) {
    int v = s->heap[k], j = k << 1;
    while (j <= s->heap_len) {
        if (j < s->heap_len && SMALLER(t, s->heap[j + 1], s->heap[j], s->depth)) j++;
        if (SMALLER(t, v, s->heap[j], s->depth)) break;
        s->heap[k] = s->heap[j]; k = j; j <<= 1;
    }
    s->heap[k] = v;
}

/* build_tree + gen_bitlen + gen_codes (trees.c).  stl: static lengths or NULL. */
static int build_tree(Trees *s, ct *t, int elems, const uint16_t *stl, const int *extra, int xbase, int maxlen) {
    int n, m, max_code = -1, node;
    s->heap_len = 0; s->heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (t[n].fc) { s->heap[++s->heap_len] = max_code = n; s->depth[n] = 0; }
        else t[n].dl = 0;
    }
    while (s->heap_len < 2) {
        node = s->heap[++s->heap_len] = (max_code < 2 ? ++max_code : 0);
        t[node].fc = 1; s->depth[node] = 0;
        s->opt_len--; if (stl) s->static_len -= stl[node];
    }
    for (n = s->heap_len / 2; n >= 1; n--) downheap(s, t, n);
    node = elems;
    do {
        n = s->heap[1]; s->heap[1] = s->heap[s->heap_len--]; downheap(s, t, 1);
        m = s->heap[1];
        s->heap[--s->heap_max] = n; s->heap[--s->heap_max] = m;
        t[node].fc = (uint16_t)(t[n].fc + t[m].fc);
        s->depth[node] = (uint8_t)((s->depth[n] >= s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
        t[n].dl = t[m].dl = (uint16_t)node;
        s->heap[1] = node++;
        downheap(s, t, 1);
    } while (s->heap_len >= 2);
    s->heap[--s->heap_max] = s->heap[1];

    /* gen_bitlen */
    int h, bits, overflow = 0;
    for (bits = 0; bits <= MAX_BITS; bits++) s->bl_count[bits] = 0;
    t[s->heap[s->heap_max]].dl = 0;
    for (h = s->heap_max + 1; h < HEAP_SIZE; h++) {
        n = s->heap[h];
        bits = t[t[n].dl].dl + 1;
        if (bits > maxlen) { bits = maxlen; overflow++; }
        t[n].dl = (uint16_t)bits;
        if (n > max_code) continue;
        s->bl_count[bits]++;
        int xb = n >= xbase ? extra[n - xbase] : 0;
        s->opt_len += (uint64_t)t[n].fc * (unsigned)(bits + xb);
        if (stl) s->static_len += (uint64_t)t[n].fc * (unsigned)(stl[n] + xb);
    }
    if (overflow) {
        do {
            bits = maxlen - 1;
            while (s->bl_count[bits] == 0) bits--;
            s->bl_count[bits]--; s->bl_count[bits + 1] += 2; s->bl_count[maxlen]--;
            overflow -= 2;
        } while (overflow > 0);
        for (bits = maxlen; bits != 0; bits--) {
            n = s->bl_count[bits];
            while (n != 0) {
                m = s->heap[--h];
                if (m > max_code) continue;
                if (t[m].dl != (unsigned)bits) {
                    s->opt_len += ((uint64_t)bits - t[m].dl) * t[m].fc;
                    t[m].dl = (uint16_t)bits;
                }
                n--;
            }
        }
    }
    /* gen_codes */
    unsigned next[MAX_BITS + 1], code = 0;
    for (bits = 1; bits <= MAX_BITS; bits++) { code = (code + s->bl_count[bits - 1]) << 1; next[bits] = code; }
    for (n = 0; n <= max_code; n++) {
        int len = t[n].dl;
        if (len) t[n].fc = (uint16_t)bitrev(next[len]++, len);
    }
    return max_code;
}

/* scan_tree (count) when b == NULL, send_tree (emit) otherwise */
static void scan_send_tree(Trees *s, ct *t, int max_code, Bits *b) {
    int prevlen = -1, curlen, nextlen = t[0].dl, count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    if (!b) t[max_code + 1].dl = 0xffff;                  /* guard */
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen; nextlen = t[n + 1].dl;
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) {
            if (!b) s->bt[curlen].fc += count;
            else do { put_bits(b, s->bt[curlen].fc, s->bt[curlen].dl); } while (--count != 0);
        } else if (curlen != 0) {
            if (!b) { if (curlen != prevlen) s->bt[curlen].fc++; s->bt[16].fc++; }
            else {
                if (curlen != prevlen) { put_bits(b, s->bt[curlen].fc, s->bt[curlen].dl); count--; }
                put_bits(b, s->bt[16].fc, s->bt[16].dl); put_bits(b, count - 3, 2);
            }
        } else if (count <= 10) {
            if (!b) s->bt[17].fc++;
            else { put_bits(b, s->bt[17].fc, s->bt[17].dl); put_bits(b, count - 3, 3); }
        } else {
            if (!b) s->bt[18].fc++;
            else { put_bits(b, s->bt[18].fc, s->bt[18].dl); put_bits(b, count - 11, 7); }
        }
        count = 0; prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

/* one block's symbols: lit[i] = literal or length-3, dist[i] = 0 or distance */
typedef struct { uint8_t lit[LIT_BUFSIZE]; uint16_t dist[LIT_BUFSIZE]; uint32_t n; } Syms;

static void compress_block(Bits *b, const Syms *sy, const ct *lt, const ct *dt) {
    for (uint32_t i = 0; i < sy->n; i++) {
        unsigned lc = sy->lit[i], dist = sy->dist[i];
        if (dist == 0) { put_bits(b, lt[lc].fc, lt[lc].dl); continue; }
        int code = len_code[lc];
        put_bits(b, lt[code + 257].fc, lt[code + 257].dl);
        if (XLB[code]) put_bits(b, lc - base_len[code], XLB[code]);
        dist--;
        code = d_code(dist);
        put_bits(b, dt[code].fc, dt[code].dl);
        if (XDB[code]) put_bits(b, dist - base_dist[code], XDB[code]);
    }
    put_bits(b, lt[END_BLOCK].fc, lt[END_BLOCK].dl);
}

static void stored_block(Bits *b, const uint8_t *buf, uint32_t len, int last) {   /* _tr_stored_block */
    put_bits(b, (0 << 1) + last, 3);
    windup(b);
    put_byte(b, len & 0xff); put_byte(b, (len >> 8) & 0xff);
    put_byte(b, ~len & 0xff); put_byte(b, (~len >> 8) & 0xff);
    for (uint32_t i = 0; i < len; i++) put_byte(b, buf[i]);
}

/* _tr_flush_block: buf == NULL when the block's bytes left the window */
static void flush_block(Bits *b, const Syms *sy, const uint8_t *buf, uint64_t stored_len, int last) {
    static ct slt[288], sdt[30];
    Trees *s = calloc(1, sizeof(Trees));
    for (uint32_t i = 0; i < sy->n; i++) {
        if (sy->dist[i] == 0) s->lt[sy->lit[i]].fc++;
        else { s->lt[len_code[sy->lit[i]] + 257].fc++; s->dt[d_code(sy->dist[i] - 1u)].fc++; }
    }
    s->lt[END_BLOCK].fc = 1;
    s->lmax = build_tree(s, s->lt, L_CODES, st_llen, XLB, 257, MAX_BITS);
    static uint16_t st_dlen[30];
    for (int i = 0; i < 30; i++) st_dlen[i] = 5;
    s->dmax = build_tree(s, s->dt, D_CODES, st_dlen, XDB, 0, MAX_BITS);
    scan_send_tree(s, s->lt, s->lmax, NULL);
    scan_send_tree(s, s->dt, s->dmax, NULL);
    build_tree(s, s->bt, BL_CODES, NULL, XBB, 0, 7);
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s->bt[BL_ORDER[max_blindex]].dl != 0) break;
    s->opt_len += 3 * ((uint64_t)max_blindex + 1) + 5 + 5 + 4;
    uint64_t opt_lenb = (s->opt_len + 3 + 7) >> 3, static_lenb = (s->static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if (stored_len + 4 <= opt_lenb && buf) {
        stored_block(b, buf, (uint32_t)stored_len, last);
    } else if (static_lenb == opt_lenb) {
        for (int i = 0; i < 288; i++) { slt[i].fc = st_lcode[i]; slt[i].dl = st_llen[i]; }
        for (int i = 0; i < 30; i++) { sdt[i].fc = st_dcode[i]; sdt[i].dl = 5; }
        put_bits(b, (1 << 1) + last, 3);
        compress_block(b, sy, slt, sdt);
    } else {
        put_bits(b, (2 << 1) + last, 3);
        int lcodes = s->lmax + 1, dcodes = s->dmax + 1, blcodes = max_blindex + 1;
        put_bits(b, lcodes - 257, 5); put_bits(b, dcodes - 1, 5); put_bits(b, blcodes - 4, 4);
        for (int r = 0; r < blcodes; r++) put_bits(b, s->bt[BL_ORDER[r]].dl, 3);
        scan_send_tree(s, s->lt, lcodes - 1, b);
        scan_send_tree(s, s->dt, dcodes - 1, b);
        compress_block(b, sy, s->lt, s->dt);
    }
    if (last) windup(b);
    free(s);
}

/* ------------------------------------------------------------------ stream */
typedef struct zr_stream {
    int level, good, lazy, nice, chain;
    uint8_t hist[WSIZE];          /* hist[i] = byte at stream position total - WSIZE + i */
    uint64_t base;                /* stream position of zlib's window coord 0 (moves by WSIZE per slide) */
    uint64_t total;               /* bytes consumed so far */
    int started, finished;
    uint32_t adler;
    uint64_t match_start;
    uint64_t block_start;         /* stream position */
    uint64_t strstart;            /* next loop top; < total when a flush call stopped early */
    int avail, mlen;              /* deflate_slow's match_available / match_length across such a stop */
    int ins;                      /* deflate_fast: s->insert, positions before strstart still to hash */
    uint64_t acc; int nb;         /* bits of the last incomplete output byte (bi_buf after flush_pending) */
    uint8_t *q; uint64_t qn, qcap;/* produced but not yet delivered: zlib's pending past the pipe's buffer */
    uint64_t *fhead, *fprev;      /* deflate_fast: zlib's head[] / prev[] by stream position (NONE: NIL) */
    Syms sy;
    /* per-call scratch */
    uint64_t lo;                  /* stream position of x[0] */
    uint8_t *x; uint32_t *prv;    /* bytes [lo, end) and their hash-chain links (index or UINT32_MAX) */
    uint16_t *mfull, *mquar; uint32_t *sfull, *squar;
} zr_stream;

zr_stream *zr_create(int level) {
    if (level < 1 || level > 9) return NULL;   /* deflate_fast 1-3, deflate_slow 4-9 (wanproxy.conf: 6) */
    init_tables();
    zr_stream *s = calloc(1, sizeof(zr_stream));
    s->level = level;
    s->good = CFG[level][0]; s->lazy = CFG[level][1]; s->nice = CFG[level][2]; s->chain = CFG[level][3];
    s->adler = 1;
    s->mlen = MIN_MATCH - 1;
    if (level < 4) {
        s->fhead = malloc(sizeof(uint64_t) * 32768);
        s->fprev = malloc(sizeof(uint64_t) * WSIZE);
        for (int i = 0; i < 32768; i++) s->fhead[i] = NONE;
        for (unsigned i = 0; i < WSIZE; i++) s->fprev[i] = NONE;
    }
    return s;
}

void zr_free(zr_stream *s) {
    if (!s) return;
    free(s->q); free(s->fhead); free(s->fprev);
    free(s);
}

static uint32_t adler32(uint32_t a, const uint8_t *p, uint64_t n) {
    uint32_t s1 = a & 0xffff, s2 = a >> 16;
    for (uint64_t i = 0; i < n; i++) { s1 = (s1 + p[i]) % 65521; s2 = (s2 + s1) % 65521; }
    return (s2 << 16) | s1;
}

static inline uint8_t X(const zr_stream *s, uint64_t pos) { return s->x[pos - s->lo]; }
static inline uint32_t hash3(const zr_stream *s, uint64_t q) {   /* UPDATE_HASH x3, hash_shift 5, 15 bits */
    return (((uint32_t)X(s, q) << 10) ^ ((uint32_t)X(s, q + 1) << 5) ^ X(s, q + 2)) & 0x7fff;
}
static inline uint64_t prevlink(const zr_stream *s, uint64_t q) {
    uint32_t v = s->prv[q - s->lo];
    return v == UINT32_MAX ? NONE : s->lo + v;
}

/* longest_match's inner compare over the data only: bytes 0, 1, then 3.. (2
 * is equal by the hash), at most `cap` = min(MAX_MATCH, lookahead) bytes */
static int lcp(const zr_stream *s, uint64_t p, uint64_t c, int cap) {
    if (X(s, p) != X(s, c) || X(s, p + 1) != X(s, c + 1)) return 0;
    int len = 3;
    while (len < cap && X(s, p + len) == X(s, c + len)) len++;
    return len;
}

/* Match table entry for position p with lookahead la = end - p >= MIN_MATCH:
 * longest_match's walk from the chain head with `budget` candidates, giving
 * M = the best length (0: none reaches MIN_MATCH), S = the first candidate
 * reaching it.  Independent of the threshold prev_length: longest_match keeps
 * the first candidate of maximal length, and its nice break (the first
 * candidate with len >= nice) does not depend on it.
 * Bytes past the data: longest_match may compare into the stale window past
 * the lookahead, but that never changes its result.  nice is clipped to the
 * lookahead; if la <= nice, the first candidate matching all la data bytes is
 * the break candidate (every earlier one mismatched inside the data), and if
 * la > nice, len >= nice is decided inside the data.  So lengths are capped
 * at la, and the scan clips the threshold to la as longest_match's return
 * does. */
static void walk(const zr_stream *s, uint64_t p, uint64_t end, int budget, int nice, uint16_t *M, uint32_t *S) {
    int cap = end - p < MAX_MATCH ? (int)(end - p) : MAX_MATCH;
    if (nice > cap) nice = cap;
    uint64_t cur = prevlink(s, p), limit = p > MAX_DIST ? p - MAX_DIST : 0;
    int best = 0; uint64_t bs = 0;
    while (cur != NONE) {
        int len = lcp(s, p, cur, cap);
        if (len > best) { best = len; bs = cur; if (len >= nice) break; }
        cur = prevlink(s, cur);
        if (cur == NONE || cur <= limit || --budget == 0) break;
    }
    *M = (uint16_t)best; *S = (uint32_t)(bs - s->lo);
}
typedef struct { uint64_t rd, end; } Feed;   /* stream positions read into zlib's window / available */

/* deflate_fast's INSERT_STRING at q: the old head (zlib's hash_head), q becomes the head */
static uint64_t fast_insert(zr_stream *s, uint64_t q) {
    uint32_t h = hash3(s, q);
    uint64_t hh = s->fhead[h];
    s->fprev[q & (WSIZE - 1)] = hh;
    s->fhead[h] = q;
    return hh;
}

/* fill_window's effect on positions: slide (base += WSIZE) when strstart >=
 * WSIZE + MAX_DIST, then read what fits; deflate_fast also hashes the
 * positions s->insert names once their bytes exist.  The window's bytes
 * themselves are not needed (see walk()). */
static void fill_window(zr_stream *s, uint64_t strstart, Feed *f) {
    do {
        uint64_t more = WINSZ - (f->rd - s->base);
        if (strstart - s->base >= WSIZE + MAX_DIST) { s->base += WSIZE; more += WSIZE; }
        if (f->rd == f->end) break;
        uint64_t n = f->end - f->rd; if (n > more) n = more;
        f->rd += n;
        if (s->fhead && f->rd - strstart + s->ins >= MIN_MATCH) {
            uint64_t str = strstart - (uint64_t)s->ins;
            while (s->ins) {
                fast_insert(s, str);
                str++;
                s->ins--;
                if (f->rd - strstart + s->ins < MIN_MATCH) break;
            }
        }
    } while (f->rd - strstart < MIN_LOOKAHEAD && f->rd < f->end);
}

static int tally(zr_stream *s, unsigned lc, unsigned dist) {
    s->sy.lit[s->sy.n] = (uint8_t)lc; s->sy.dist[s->sy.n] = (uint16_t)dist; s->sy.n++;
    return s->sy.n == LIT_BUFSIZE - 1;
}

static void flush(zr_stream *s, Bits *b, uint64_t strstart, int last) {   /* FLUSH_BLOCK_ONLY */
    /* the block's bytes are still in zlib's window unless a slide passed block_start */
    const uint8_t *buf = s->block_start >= s->base ? s->x + (s->block_start - s->lo) : NULL;
    flush_block(b, &s->sy, buf, strstart - s->block_start, last);
    s->sy.n = 0;
    s->block_start = strstart;
}

/* the eligible chain head at loop top p (hash_head != NIL && within MAX_DIST) */
static uint64_t head_of(const zr_stream *s, uint64_t p, uint32_t lookahead) {
    if (lookahead < MIN_MATCH) return NONE;
    uint64_t h = prevlink(s, p);
    if (h == NONE || h <= s->base || p - h > MAX_DIST) return NONE;   /* coord 0 is NIL */
    return h;
}

/* DeflatePipe's buffer (deflate_pipe.cc:57-115).  Output reaches the pipe at
 * flush_pending, i.e. after every block flush (b->n = bytes complete).  Under
 * Z_NO_FLUSH (loop tops with >= MIN_LOOKAHEAD bytes of lookahead) the pipe
 * takes everything, emptying its 64 KiB buffer whenever it fills, so when the
 * Z_SYNC_FLUSH call begins the buffer holds n mod 65536 bytes, n = the bytes
 * the consume took so far.  That call ends at the first block flush that
 * leaves the buffer full (FLUSH_BLOCK's need_more): the consume delivers up
 * to the boundary L = 65536 * (n / 65536 + 1) and the stream goes on from
 * there at the next consume, without a sync marker. */
typedef struct { uint64_t n; int stopped; } Pipe;

static int flushed(Pipe *pp, const Bits *b, uint64_t la) {   /* 1: the flush call stops here */
    if (la >= MIN_LOOKAHEAD) { pp->n = b->n; return 0; }
    if (b->n >= 65536 * (pp->n / 65536 + 1)) { pp->stopped = 1; return 1; }
    return 0;
}

/* deflate_slow (levels 4-9) over the match table from s->strstart.  Returns 1
 * if the flush call stopped at a block flush (state saved for the next call). */
static int scan_slow(zr_stream *s, Bits *b, Feed *f, Pipe *pp, int finishing) {
    uint64_t p = s->strstart, lo = s->lo;
    int match_length = s->mlen, match_available = s->avail;
    for (;;) {
        if (f->rd - p < MIN_LOOKAHEAD) {
            fill_window(s, p, f);
            if (f->rd - p == 0) break;
        }
        uint32_t lookahead = (uint32_t)(f->rd - p);
        uint64_t head = head_of(s, p, lookahead);
        int prev_length = match_length;
        uint64_t prev_match = s->match_start;
        match_length = MIN_MATCH - 1;
        if (head != NONE && prev_length < s->lazy) {
            uint64_t i = p - lo;
            int quar = prev_length >= s->good;
            int M = quar ? s->mquar[i] : s->mfull[i];
            if (M > prev_length) {
                match_length = M;
                s->match_start = lo + (quar ? s->squar[i] : s->sfull[i]);
            } else {
                match_length = (uint32_t)prev_length <= lookahead ? prev_length : (int)lookahead;
            }
            if (match_length <= 5 && match_length == MIN_MATCH && p - s->match_start > TOO_FAR)
                match_length = MIN_MATCH - 1;
        }
        if (prev_length >= MIN_MATCH && match_length <= prev_length) {
            int bf = tally(s, (unsigned)(prev_length - MIN_MATCH), (unsigned)(p - 1 - prev_match));
            p += (uint64_t)prev_length - 1;
            match_available = 0;
            match_length = MIN_MATCH - 1;
            if (bf) {                                     /* FLUSH_BLOCK */
                flush(s, b, p, 0);
                if (!finishing && flushed(pp, b, lookahead)) goto stop;
            }
        } else if (match_available) {
            int bf = tally(s, X(s, p - 1), 0);
            if (bf) flush(s, b, p, 0);                    /* FLUSH_BLOCK_ONLY */
            p++;
            if (bf && !finishing && flushed(pp, b, lookahead)) goto stop;   /* avail_out == 0: need_more */
        } else {
            match_available = 1;
            p++;
        }
    }
    if (match_available) tally(s, X(s, p - 1), 0);
    s->strstart = p;
    s->avail = 0;
    s->mlen = MIN_MATCH - 1;
    return 0;
stop:
    s->strstart = p;
    s->avail = match_available;
    s->mlen = match_length;
    return 1;
}

/* deflate_fast (levels 1-3): zlib's own chains (only the positions the parse
 * hashes: loop tops, and the inside of matches no longer than max_lazy).
 * Returns 1 if the flush call stopped at a block flush. */
static int scan_fast(zr_stream *s, Bits *b, Feed *f, Pipe *pp, int finishing) {
    uint64_t p = s->strstart;
    const int max_insert = s->lazy;
    for (;;) {
        if (f->rd - p < MIN_LOOKAHEAD) {
            fill_window(s, p, f);
            if (f->rd - p == 0) break;
        }
        const uint64_t lookahead = f->rd - p;
        uint64_t hh = NONE;
        if (lookahead >= MIN_MATCH) hh = fast_insert(s, p);
        int ml = 0;
        uint64_t ms = 0;
        if (hh != NONE && hh > s->base && p - hh <= MAX_DIST) {   /* longest_match from hash_head */
            int cap = lookahead < MAX_MATCH ? (int)lookahead : MAX_MATCH;
            int nice = s->nice < cap ? s->nice : cap, chain = s->chain, best = MIN_MATCH - 1;
            uint64_t cur = hh, limit = p > MAX_DIST ? p - MAX_DIST : 0;
            for (;;) {
                int len = lcp(s, p, cur, cap);
                if (len > best) { best = len; ms = cur; if (len >= nice) break; }
                cur = s->fprev[cur & (WSIZE - 1)];
                if (cur == NONE || cur <= limit || --chain == 0) break;
            }
            if (best >= MIN_MATCH) ml = best;
        }
        int bf;
        if (ml >= MIN_MATCH) {
            bf = tally(s, (unsigned)(ml - MIN_MATCH), (unsigned)(p - ms));
            if ((uint64_t)ml <= (uint64_t)max_insert && lookahead - (uint64_t)ml >= MIN_MATCH) {
                for (int k = 1; k < ml; k++) fast_insert(s, p + (uint64_t)k);
            }
            p += (uint64_t)ml;
        } else {
            bf = tally(s, X(s, p), 0);
            p++;
        }
        if (bf) {                                         /* FLUSH_BLOCK */
            flush(s, b, p, 0);
            if (!finishing && flushed(pp, b, lookahead)) { s->strstart = p; return 1; }
        }
    }
    s->strstart = p;
    s->ins = p - s->base < MIN_MATCH - 1 ? (int)(p - s->base) : MIN_MATCH - 1;
    return 0;
}

static void grow(zr_stream *s, uint64_t want) {
    if (s->qcap >= want) return;
    uint64_t c = s->qcap ? s->qcap : 65536;
    while (c < want) c *= 2;
    s->q = realloc(s->q, c);
    s->qcap = c;
}

/* One DeflatePipe::consume(): n > 0 bytes, then Z_SYNC_FLUSH; n == 0: Z_FINISH.
 * Returns the bytes the pipe produces (written to out), or -1 if cap was too small. */
int64_t zr_consume(zr_stream *s, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap) {
    if (s->finished) return 0;
    const uint64_t p0 = s->strstart, end = s->total + n;
    grow(s, s->qn + 2 * (n + (s->total - p0)) + 4096);
    Bits b = {s->q, s->qn, s->qcap, s->acc, s->nb, 0};
    if (!s->started) {
        unsigned lf = s->level < 2 ? 0 : s->level < 6 ? 1 : s->level == 6 ? 2 : 3;
        unsigned header = ((8 + (7 << 4)) << 8) | (lf << 6);
        header += 31 - (header % 31);
        put_byte(&b, header >> 8); put_byte(&b, header & 0xff);
        s->started = 1;
    }
    /* history the chains can reach + this call's bytes, by stream position */
    uint64_t lo = s->total > WSIZE ? s->total - WSIZE : 0;
    if (lo < s->base) lo = s->base;
    s->lo = lo;
    uint64_t span = end - lo;
    s->x = malloc(span + MAX_MATCH + 8);
    memcpy(s->x, s->hist + (lo + WSIZE - s->total), s->total - lo);
    memcpy(s->x + (s->total - lo), in, n);
    memset(s->x + span, 0, MAX_MATCH + 8);
    s->adler = adler32(s->adler, in, n);
    s->prv = NULL;
    s->mfull = s->mquar = NULL;
    s->sfull = s->squar = NULL;

    if (!s->fhead) {
        /* phase A: hash chains (prev links) over [lo, end - 2) */
        s->prv = malloc(sizeof(uint32_t) * (span + 1));
        uint32_t *headt = malloc(sizeof(uint32_t) * 32768);
        for (int i = 0; i < 32768; i++) headt[i] = UINT32_MAX;
        for (uint64_t q = lo; q < end; q++) {
            if (q + 2 < end) {
                uint32_t h = hash3(s, q);
                s->prv[q - lo] = headt[h];
                headt[h] = (uint32_t)(q - lo);
            } else s->prv[q - lo] = UINT32_MAX;
        }
        free(headt);
        /* phase B: match table for every position with >= MIN_MATCH lookahead */
        s->mfull = calloc(span, 2); s->mquar = calloc(span, 2);
        s->sfull = calloc(span, 4); s->squar = calloc(span, 4);
        for (uint64_t q = p0; q + 2 < end; q++) {
            uint64_t i = q - lo;
            if (prevlink(s, q) == NONE) continue;
            walk(s, q, end, s->chain, s->nice, &s->mfull[i], &s->sfull[i]);
            walk(s, q, end, s->chain >> 2, s->nice, &s->mquar[i], &s->squar[i]);
        }
    }

    /* phase C: the parse; a flush call may stop at a block flush */
    Feed f = {s->total, end};
    Pipe pp = {s->qn, 0};
    const int finishing = n == 0;
    int stopped = s->fhead ? scan_fast(s, &b, &f, &pp, finishing) : scan_slow(s, &b, &f, &pp, finishing);
    uint64_t deliver;
    if (finishing) {
        flush(s, &b, s->strstart, 1);
        put_byte(&b, s->adler >> 24); put_byte(&b, (s->adler >> 16) & 0xff);
        put_byte(&b, (s->adler >> 8) & 0xff); put_byte(&b, s->adler & 0xff);
        s->finished = 1;
        deliver = b.n;
    } else {
        if (!stopped && s->sy.n) {                         /* deflate_*'s last FLUSH_BLOCK(s, 0) */
            flush(s, &b, s->strstart, 0);
            stopped = flushed(&pp, &b, 0);
        }
        if (!stopped) stored_block(&b, NULL, 0, 0);       /* Z_SYNC_FLUSH marker */
        const uint64_t lim = 65536 * (pp.n / 65536 + 1);
        deliver = b.n < lim ? b.n : lim;
    }
    /* keep the last WSIZE bytes: the next call's chains reach back MAX_DIST */
    uint64_t keep = end - lo < WSIZE ? end - lo : WSIZE;
    memcpy(s->hist + WSIZE - keep, s->x + (end - keep - lo), keep);
    s->total = end;
    free(s->x); free(s->prv); free(s->mfull); free(s->mquar); free(s->sfull); free(s->squar);
    s->x = NULL;
    s->acc = b.acc; s->nb = b.nb;
    if (b.err) return -1;
    if (deliver > cap) return -1;
    memcpy(out, s->q, deliver);
    memmove(s->q, s->q + deliver, b.n - deliver);
    s->qn = b.n - deliver;
    return (int64_t)deliver;
}

uint64_t zr_bound(uint64_t n) { return 2 * n + 4 * 65536 + 1024; }

/* Test hook: positions the last flush call left for the next consume (a stop
 * inside the flush call's tail), and bytes produced but not yet delivered. */
void zr_carry(const zr_stream *s, uint64_t *deferred, uint64_t *pending) {
    *deferred = s->total - s->strstart;
    *pending = s->qn;
}
