// wanproxy's zlib stage on the GPU: DeflatePipe (zlib/deflate_pipe.cc:57-115)
// for many streams at once, bit-exact with zlib 1.2.11's deflate at levels 4-9
// (deflate_slow; wanproxy.conf sets level 6).  gfx950, wave64.
//
// A DeflatePipe::consume() of n bytes is deflate(Z_NO_FLUSH) over its
// segments then deflate(Z_SYNC_FLUSH); an empty consume is deflate(Z_FINISH).
// The output does not depend on the segmentation (every position zlib
// processes under Z_NO_FLUSH has >= MIN_LOOKAHEAD bytes of lookahead), so a
// call is its bytes plus a flush.  Per call, in HBM:
//
//   X      the stream's last 32 KiB (history) ++ the call's bytes.  X index j
//          is stream position total - 32768 + j.
//   d16    hash-chain links: j - prev(j), prev(j) = the latest earlier position
//          with the same 3-byte hash (zlib's head/prev, deflate.c INSERT_STRING:
//          deflate_slow inserts every position once its 3 bytes exist, in
//          order), 0 = none / farther than 32767.          zd_chain_kernel
//   tf/tq  per position: longest_match's walk from the chain head with the full
//          and the quartered (prev_length >= good_match) chain budget: best
//          length and the distance of the first candidate reaching it.  The
//          threshold prev_length cannot change which candidate wins (first of
//          maximal length) nor where the nice-length break falls, so one walk
//          serves every prev_length.  Bytes past the lookahead never change
//          longest_match's result (nice is clipped to the lookahead), so lengths
//          are capped there and zlib's 64 KiB window is never materialised.
//                                                          zd_match_kernel
//   sym    the lazy-matching scan (deflate_slow) over that table, one wave per
//          call, sequential but cheap per position; runs of positions where no
//          match can start are emitted 64 at a time.  Window slides are
//          tracked (coord 0 is NIL; a block whose start slid out cannot be
//          stored).  Blocks end every 16383 symbols (lit_bufsize - 1).
//                                                          zd_scan_kernel
//   trees  per block (one wave): symbol histogram, zlib's build_tree /
//          gen_bitlen / gen_codes, bit-length tree, the stored / static /
//          dynamic choice of _tr_flush_block.              zd_trees_kernel
//   out    layout (block bit offsets, zeroed output), then every block's bits
//          in parallel (atomicOr into the zeroed words).   zd_layout / zd_emit
//
// The reference interface replaced is DeflatePipe(level) / consume(Buffer*)
// (zlib/deflate_pipe.h:33-42, deflate_pipe.cc:36-115).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/xcgpu.h"
#include "xcg_device.h"
#include "xcg_stored_plan.h"

namespace xcg {
namespace zd {

constexpr int WSIZE = 32768;
constexpr int WINSZ = 65536;
constexpr int MIN_MATCH = 3;
constexpr int MAX_MATCH = 258;
constexpr int MIN_LOOKAHEAD = MAX_MATCH + MIN_MATCH + 1;   // 262
constexpr int MAX_DIST = WSIZE - MIN_LOOKAHEAD;            // 32506
constexpr int TOO_FAR = 4096;
constexpr uint32_t SYMS_PER_BLOCK = 16383;                 // lit_bufsize - 1
constexpr int L_CODES = 286, D_CODES = 30, BL_CODES = 19, HEAP_SIZE = 2 * L_CODES + 1;
constexpr int MAX_BITS = 15;
constexpr int XPAD = 272;                                  // zeroed bytes after a call's data in X
constexpr int TAB_WORDS = L_CODES + D_CODES + BL_CODES;    // per block: code | len << 16
constexpr int DMAX = 264;            // >= MIN_LOOKAHEAD - 1: positions a stopped flush call can leave
constexpr uint32_t PIPE_CHUNK = 65536;   // DeflatePipe's output buffer (DEFLATE_CHUNK_SIZE, deflate_pipe.cc:34)

// configuration_table (deflate.c): good, lazy, nice, chain
__constant__ int CFG[10][4] = {{0, 0, 0, 0},        {4, 4, 8, 4},     {4, 5, 16, 8},      {4, 6, 32, 32},
                               {4, 4, 16, 16},      {8, 16, 32, 32},  {8, 16, 128, 128},  {8, 32, 128, 256},
                               {32, 128, 258, 1024}, {32, 258, 258, 4096}};
__constant__ uint8_t XLB[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint8_t XDB[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t XBB[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
__constant__ uint8_t BL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
__constant__ uint16_t BASE_LEN[29] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 0};
__constant__ uint16_t BASE_DIST[30] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512, 768,
                                       1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 24576};

// length - 3 (0..255) -> length code 0..28 (trees.c _length_code; 255 -> 28)
__device__ __forceinline__ int len_code(uint32_t lc) {
  if (lc >= 255) return 28;
  if (lc < 8) return (int)lc;
  int b = 31 - __clz(lc);                       // 3..7
  return 4 * (b - 1) + (int)((lc >> (b - 2)) & 3);
}
// distance - 1 (0..32767) -> distance code 0..29 (trees.c d_code)
__device__ __forceinline__ int dist_code(uint32_t d) {
  if (d < 4) return (int)d;
  int b = 31 - __clz(d);                        // 2..14
  return 2 * b + (int)((d >> (b - 1)) & 1);
}
__device__ __forceinline__ uint32_t bitrev(uint32_t c, int n) { return __brev(c) >> (32 - n); }

struct ZState {          // one DeflatePipe's z_stream, reduced to what the output depends on
  uint64_t total;        // bytes consumed
  uint64_t base;         // stream position of zlib's window coord 0 (slides by WSIZE)
  uint32_t adler;        // adler32 of everything consumed (the Z_FINISH trailer)
  uint32_t flags;        // 1: header written, 2: finished (Z_STREAM_END)
  // What a flush call that stopped at a full pipe buffer leaves (see zd_layout_kernel):
  uint64_t pend;         // bytes produced but not delivered yet (zlib's pending past the buffer)
  uint64_t block_start;  // stream position of the open block's start
  uint64_t mstart;       // match_start (stream position)
  uint32_t dlen;         // positions before `total` not parsed yet (strstart = total - dlen)
  uint32_t avail, mlen;  // deflate_slow's match_available, match_length at strstart
  uint32_t cbits, cnb;   // the last incomplete output byte: its cnb < 8 low bits
  uint32_t pad;
};

struct ZCall {           // host-built, one per consume()
  uint64_t in_off, out_off;   // into d_in / d_out (out_off % 4 == 0)
  uint64_t x_off;             // X (and d16 at 2 * x_off) in the scratch
  uint64_t t_off;             // tf / tq / sym: call-relative position 0
  uint32_t len, stream;
  uint32_t blk_off, blk_cap;  // block records
  uint64_t m_off;             // deflate_fast: the call's hashed-position masks (words; bit j = X index j)
};

struct ZBlock {
  uint32_t sym_begin, sym_end;
  uint32_t start;        // X index of block_start
  uint32_t stored_len;
  uint32_t flags;        // 1 storable (block_start not slid out), 2 last, 4 flushed in the flush call
                         // (a loop top with lookahead < MIN_LOOKAHEAD, or the call's final flush)
  uint32_t type;         // 0 stored, 1 static, 2 dynamic
  uint32_t lcodes, dcodes, blcodes, pad;
  uint64_t bits;         // Huffman blocks: 3 + trees + symbols + end-of-block
  uint64_t bit_off;      // start of the block in the call's output
  // the parse state right after this flush (where a stopped flush call resumes)
  int64_t bidx;          // X index of window coord 0
  uint32_t p_after, ms;  // X indices: strstart, match_start
  uint32_t avail, ml;
};

struct ZCallRes {
  uint32_t nblocks;      // blocks emitted (a stopped flush call drops the ones after the stop)
  uint32_t nsym;
  uint64_t base_end;     // stream position of coord 0 after the call
  uint32_t adler;        // adler32 after the call
  uint32_t out_len;      // output bytes the emit may touch (incl. a stop's incomplete last byte)
  uint64_t end_bit;      // bit offset after the last emitted block
  uint32_t stop;         // 0 none, else 1 + the block the flush call stopped at
  uint32_t out_bytes;    // complete new bytes (what the caller appends to the undelivered ones)
  uint64_t deliver;      // bytes DeflatePipe::consume produces now
  uint32_t scan_end;     // X index the parse reached (all positions, unless stopped)
  uint32_t pad;
};

struct ZArgs {
  const ZCall* calls;
  ZState* st;
  uint8_t* hist;         // nstreams x WSIZE
  const uint8_t* in;
  uint8_t* out;
  uint8_t* X;
  uint16_t* d16;
  uint32_t* pk;          // packed hashes (zd_hashes_kernel), indexed like X
  uint32_t* tf;
  uint32_t* tq;
  uint32_t* sym;
  ZBlock* blk;
  uint32_t* tabs;        // blk index * TAB_WORDS
  ZCallRes* res;
  uint32_t* out_len;     // caller's d_out_len
  uint64_t* deliver;     // caller's d_deliver
  uint32_t n;                  // calls
  const uint32_t* mstart;      // first 256-position match tile of each call (n + 1, prefix)
  const uint32_t* gstart;      // first 64-position hash group of each call (n + 1, prefix)
  const uint32_t* bstart;      // first block record of each call (n + 1, prefix)
  int level;
  // deflate_fast (levels 1-3): which positions zlib hashes depends on its parse.
  // mcur: this round's guess (X index >= strstart; earlier ones from `ring`),
  // mnext: the positions the round's parse hashes, ring: per stream, bit
  // (position mod 32768) of the last 32 KiB, changed: per call, mnext != mcur.
  int fast;
  uint32_t* mcur;
  uint32_t* mnext;
  uint32_t* ring;
  uint32_t* changed;
};

// ------------------------------------------------------------------- prep
// X = history ++ data ++ zero pad, 16 bytes per thread (X and the history are
// 256-byte aligned; WSIZE and XPAD are multiples of 16, so only the vector at
// the data's end is assembled bytewise).  Grid: (tiles of 4 KiB, calls).
__global__ __launch_bounds__(256) void zd_prep_kernel(ZArgs a) {
  const ZCall c = a.calls[blockIdx.y];
  const uint64_t dend = (uint64_t)WSIZE + c.len, nv = (dend + XPAD + 15) / 16;
  uint8_t* X = a.X + c.x_off;
  const uint8_t* h = a.hist + (uint64_t)c.stream * WSIZE;
  const uint8_t* d = a.in + c.in_off;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * 256) {
    const uint64_t q = 16 * v;
    u32x4 r = {0u, 0u, 0u, 0u};
    if (q < WSIZE) {
      r = *(const u32x4*)(h + q);
    } else if (q + 16 <= dend) {
      r = *(const u32x4_u*)(d + (q - WSIZE));
    } else if (q < dend) {
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      for (uint64_t k = 0; q + k < dend; k++) w[k >> 2] |= (uint32_t)d[q + k - WSIZE] << (8 * (k & 3));
      r = u32x4{w[0], w[1], w[2], w[3]};
    }
    *(u32x4*)(X + q) = r;
  }
}

// adler32 of the call's bytes, combined with the stream's.  Four waves per
// call read consecutive 4-byte words (coalesced); per thread sum d_i and
// sum i * d_i (i < len <= 2^24: both fit 64 bits), reduced through LDS.
__global__ __launch_bounds__(256) void zd_adler_kernel(ZArgs a) {
  __shared__ uint64_t red[2][4];
  const ZCall c = a.calls[blockIdx.x];
  const uint8_t* d = a.in + c.in_off;
  const int t = threadIdx.x;
  uint64_t A = 0, B = 0;
  const uint32_t words = c.len / 4;
#pragma unroll 4
  for (uint32_t w = t; w < words; w += 256) {
    const uint32_t v = *(const u32_u*)(d + 4ull * w);
    const uint32_t s = (v & 0xff) + ((v >> 8) & 0xff) + ((v >> 16) & 0xff) + (v >> 24);
    const uint32_t wsum = ((v >> 8) & 0xff) + 2 * ((v >> 16) & 0xff) + 3 * (v >> 24);   // in-word offsets
    A += s;
    B += (uint64_t)(4ull * w) * s + wsum;
  }
  for (uint32_t i = 4 * words + t; i < c.len; i += 256) {
    const uint32_t v = d[i];
    A += v;
    B += (uint64_t)i * v;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    A += __shfl_xor(A, o);
    B += __shfl_xor(B, o);
  }
  if ((t & 63) == 0) {
    red[0][t >> 6] = A;
    red[1][t >> 6] = B;
  }
  __syncthreads();
  if (t == 0) {
    A = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) % 65521u;
    B = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) % 65521u;
    uint32_t old = a.st[c.stream].adler;
    uint64_t s1 = old & 0xffff, s2 = old >> 16, n = c.len % 65521u;
    uint64_t ns1 = (s1 + A) % 65521u;
    uint64_t ns2 = (s2 + n * s1 + n * A + 65521u - B) % 65521u;
    a.res[blockIdx.x].adler = (uint32_t)((ns2 << 16) | ns1);
  }
}

// ------------------------------------------------------------------- chains
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *(const u32_u*)p; }

// Hash-chain links in two passes.  Groups of 64 consecutive positions start at
// the call's first valid position jlo (max(base, total - WSIZE) as an X index).
//
// zd_hashes_kernel (every group of every call in parallel): a position's 3-byte
// hash (UPDATE_HASH x3, hash_shift 5) and its nearest lower lane with the same
// hash inside the group (lanes with an equal hash found by 15 ballots, one per
// hash bit), and whether it is the group's last with that hash; packed as
// h | pred_delta << 15 | last << 21 | valid << 22.
__device__ __forceinline__ uint32_t call_of(const uint32_t* starts, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;   // last call with starts[call] <= x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (starts[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t first_valid(const ZState& s) {
  return (s.total - s.base >= (uint64_t)WSIZE) ? 0 : (int64_t)WSIZE - (int64_t)(s.total - s.base);
}
// call of x in a prefix array (starts[0] = 0), searched 64 entries per step by
// the whole wave: two dependent loads for n <= 4096 instead of a 12-step chain
__device__ __forceinline__ uint32_t call_of_wave(const uint32_t* starts, uint32_t n, uint32_t x, int lane) {
  uint32_t lo = 0, span = n;   // answer in [lo, lo + span), starts[lo] <= x
  while (span > 1) {
    const uint32_t step = (span + 63) / 64;
    const uint32_t idx = lo + (uint32_t)lane * step;
    const uint64_t b = ballot(idx < lo + span && starts[idx] <= x);
    const uint32_t nlo = lo + (uint32_t)(__popcll(b) - 1) * step;
    span = std::min(step, lo + span - nlo);
    lo = nlo;
  }
  return lo;
}

constexpr uint32_t HGROUPS = 8;    // hash groups per wave (a call has > 512 groups: at most two calls)
__global__ __launch_bounds__(256) void zd_hashes_kernel(ZArgs a, uint32_t n, const uint32_t* gstart) {
  const uint32_t g0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * HGROUPS;   // this wave's first group
  const uint32_t total = gstart[n];
  if (g0 >= total) return;
  const int lane = threadIdx.x & 63;
  const uint32_t c0 = call_of_wave(gstart, n, g0, lane);
  const uint32_t s0 = gstart[c0], split = gstart[c0 + 1];
  const ZCall cA = a.calls[c0];
  const ZCall cB = (split < g0 + HGROUPS && c0 + 1 < n) ? a.calls[c0 + 1] : cA;
  const ZState sA = a.st[cA.stream], sB = a.st[cB.stream];
  const int64_t jloA = first_valid(sA), jloB = first_valid(sB);
  // deflate_fast: is X index j of a call hashed (zlib's INSERT_STRING)?
  auto hashed = [&](bool B, int32_t j) -> bool {
    const ZCall& c = B ? cB : cA;
    const ZState& st = B ? sB : sA;
    if (j >= WSIZE - (int32_t)st.dlen) return (a.mcur[c.m_off + (uint32_t)(j >> 5)] >> (j & 31)) & 1u;
    const uint64_t q = st.total - WSIZE + (uint64_t)j;
    return (a.ring[(uint64_t)c.stream * (WSIZE / 32) + ((q & (WSIZE - 1)) >> 5)] >> (q & 31)) & 1u;
  };
  // per group (wave-uniform): the call's X base, the group's first position, the call's end
  auto group = [&](uint32_t k, const uint8_t*& x, int32_t& g, int32_t& jend) {
    const uint32_t gid = g0 + k;
    const bool B = gid >= split;
    x = a.X + (B ? cB.x_off : cA.x_off);
    g = (int32_t)((B ? jloB : jloA) + 64ll * (gid - (B ? split : s0)));
    jend = gid < total ? WSIZE + (int32_t)(B ? cB.len : cA.len) : 0;
  };
  uint32_t w[HGROUPS];
#pragma unroll
  for (uint32_t k = 0; k < HGROUPS; k++) {   // all loads first
    const uint8_t* x;
    int32_t g, jend;
    group(k, x, g, jend);
    const int32_t j = g + lane;
    w[k] = j + 2 < jend ? *(const u32_u*)(x + j) : 0u;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
  for (uint32_t k = 0; k < HGROUPS; k++) {
    const uint8_t* x;
    int32_t g, jend;
    group(k, x, g, jend);
    const int32_t j = g + lane;
    bool valid = j + 2 < jend;
    if (a.fast && valid) valid = hashed(g0 + k >= split, j);   // a position zlib never hashes: no link, not a head
    uint32_t h = 0x8000u;    // invalid lanes form their own class
    if (valid) h = (((w[k] & 0xff) << 10) ^ (((w[k] >> 8) & 0xff) << 5) ^ ((w[k] >> 16) & 0xff)) & 0x7fffu;
    uint64_t m = ballot(valid);
#pragma unroll
    for (int b = 0; b < 15; b++) {
      const bool bit = (h >> b) & 1;
      const uint64_t bl = ballot(bit);
      m &= bit ? bl : ~bl;
    }
    const uint64_t lower = m & below;
    const uint32_t pd = lower ? (uint32_t)(lane - (63 - __clzll(lower))) : 0u;
    const uint32_t last = (m >> lane) == 1ull ? 1u : 0u;
    if (j < jend)
      a.pk[(uint64_t)(x - a.X) + j] = (h & 0x7fffu) | (pd << 15) | (last << 21) | ((valid ? 1u : 0u) << 22);
  }
}

// zd_chain_kernel (one wave per call, groups in order): a position's previous
// occurrence is its in-group predecessor, else the LDS head table; the last of
// each hash in the group becomes the head.  The head table keeps the low 16
// bits of positions (64 KiB); an entry's age is (j - v) mod 2^16, valid for
// 1..32767 (farther links are 0 anyway).  Every 32768 positions entries aged
// 0 or above 32767 are expired (set to age 32768), so between expiries every
// live entry's true age stays below 65536 and its 16-bit age is exact.  The
// packed hashes of the next 1024 positions are loaded into registers while
// the current ones are linked, and the links leave from registers: the group
// loop touches LDS only.
constexpr int CG = 16;   // groups per tile
__global__ __launch_bounds__(64) void zd_chain_kernel(ZArgs a) {
  __shared__ uint16_t head[32768];
  const ZCall c = a.calls[blockIdx.x];
  const ZState s = a.st[c.stream];
  const int lane = threadIdx.x;
  uint16_t* d16 = a.d16 + c.x_off;
  const uint32_t* pk = a.pk + c.x_off;
  const int64_t jlo = first_valid(s);
  const uint16_t empty = (uint16_t)(jlo + 32768);   // age 32768 at jlo, expired again at jlo + 32768
  for (int i = lane; i < 32768; i += 64) head[i] = empty;
  __syncthreads();
  const int64_t jend = (int64_t)WSIZE + c.len;
  int64_t next_expiry = jlo + 32768;   // tiles are 1024 positions from jlo: expiry falls on a tile start
  uint32_t cur[CG], nxt[CG];
#pragma unroll
  for (int k = 0; k < CG; k++) {
    const int64_t q = jlo + 64 * k + lane;
    cur[k] = q < jend ? pk[q] : 0u;
  }
  for (int64_t t0 = jlo; t0 < jend; t0 += 64 * CG) {
#pragma unroll
    for (int k = 0; k < CG; k++) {
      const int64_t q = t0 + 64 * (CG + k) + lane;
      nxt[k] = q < jend ? pk[q] : 0u;
    }
    if (t0 == next_expiry) {
      next_expiry += 32768;
      const uint32_t far = (uint16_t)(t0 + 32768);
      uint64_t* h64 = (uint64_t*)head;
#pragma unroll 8
      for (int i = lane; i < 8192; i += 64) {
        const uint64_t v = h64[i];
        uint64_t r = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint16_t e = (uint16_t)(v >> (16 * b));
          const uint16_t age = (uint16_t)((uint16_t)t0 - e);
          r |= (uint64_t)((age == 0 || age > 32767) ? (uint16_t)far : e) << (16 * b);
        }
        if (r != v) h64[i] = r;
      }
      __syncthreads();
    }
    uint16_t lk[CG];
#pragma unroll
    for (int k = 0; k < CG; k++) {
      const uint32_t e = cur[k];
      const int64_t j = t0 + 64 * k + lane;
      const uint32_t h = e & 0x7fffu, pd = (e >> 15) & 63u;
      int32_t age = 0;
      if (e >> 22) age = pd ? (int32_t)pd : (int32_t)(uint16_t)((uint16_t)j - head[h]);
      lk[k] = (age > 0 && age <= 32767) ? (uint16_t)age : 0;
      if ((e >> 22) && ((e >> 21) & 1)) head[h] = (uint16_t)j;
    }
#pragma unroll
    for (int k = 0; k < CG; k++) {
      const int64_t q = t0 + 64 * k + lane;
      if (q < jend) d16[q] = lk[k];
      cur[k] = nxt[k];
    }
  }
}

// ------------------------------------------------------------------- match table

// Entry: M (9 bits) | distance of the first candidate reaching M (15 bits) << 9
// | ELIG << 31 (chain head exists, within MAX_DIST, lookahead >= 3).  The scan
// also rejects a head at zlib's window coord 0 (NIL).
// Entries are indexed t = X index - WSIZE + DMAX: positions a stopped flush
// call left (the last s.dlen before the call's bytes) are parsed again now,
// with this call's bytes as their lookahead.
__global__ __launch_bounds__(256) void zd_match_kernel(ZArgs a) {
  const uint32_t ci = call_of(a.mstart, a.n, blockIdx.x);
  const ZCall c = a.calls[ci];
  const uint32_t t = (blockIdx.x - a.mstart[ci]) * 256u + threadIdx.x;
  const ZState s = a.st[c.stream];
  if (t < (uint32_t)DMAX - s.dlen || t >= (uint32_t)DMAX + c.len) return;
  const int64_t rel = (int64_t)t - DMAX;
  const uint8_t* X = a.X + c.x_off;
  const uint16_t* d16 = a.d16 + c.x_off;
  const int64_t j = (int64_t)WSIZE + rel;
  const int64_t la = (int64_t)c.len - rel;
  uint32_t ef = 0, eq = 0;
  uint32_t d = la >= MIN_MATCH ? d16[j] : 0;
  if (d != 0 && d <= (uint32_t)MAX_DIST) {
    const int budget = CFG[a.level][3], qb = budget >> 2;
    const int cap = la < MAX_MATCH ? (int)la : MAX_MATCH;
    const int nice = CFG[a.level][2] < cap ? CFG[a.level][2] : cap;
    // chain continues while cur > max(p - MAX_DIST, stream position 0)
    int64_t limit = j - MAX_DIST;
    int64_t zero = (int64_t)WSIZE - (int64_t)s.total;
    if (zero > limit) limit = zero;
    int64_t cur = j - d;
    int best = 0, bq = -1;
    int64_t bs = 0, bsq = 0;
    const uint32_t x01 = *(const u16_u*)(X + j);
    int count = 0;
    for (;;) {
      // the next link is loaded with the candidate's bytes (both depend on cur only)
      const uint32_t dd = d16[cur];
      // longest_match: reject on bytes 0, 1 (and at best_len), then compare
      if (*(const u16_u*)(X + cur) == x01 && (best < 3 || X[cur + best] == X[j + best])) {
        int len = 2;
        while (len < cap) {
          uint32_t w = ld32(X + cur + len) ^ ld32(X + j + len);
          if (w) {
            len += __builtin_ctz(w) >> 3;
            break;
          }
          len += 4;
        }
        if (len > cap) len = cap;
        if (len >= MIN_MATCH && len > best) {
          best = len;
          bs = cur;
          if (len >= nice) break;
        }
      }
      if (++count == qb) {
        bq = best;
        bsq = bs;
      }
      if (count >= budget) break;
      if (dd == 0) break;
      cur -= dd;
      if (cur <= limit) break;
    }
    if (bq < 0) {
      bq = best;
      bsq = bs;
    }
    ef = 0x80000000u | (uint32_t)best | (best ? (uint32_t)(j - bs) << 9 : 0);
    eq = 0x80000000u | (uint32_t)bq | (bq ? (uint32_t)(j - bsq) << 9 : 0);
  }
  a.tf[c.t_off + t] = ef;
  a.tq[c.t_off + t] = eq;
}

#ifdef XCG_ZD_TIMING
// diagnostics build: wave cycles per phase summed over blocks (trees: histogram,
// literal tree, distance + bit-length trees, bit count, tables; emit: tables and
// header, sizing pass, packing pass; scan: loop tops, literal runs and their positions,
// cycles) and block / call counts
__device__ unsigned long long g_zd_t[16];
#define ZD_NOW() __builtin_readcyclecounter()
#define ZD_ADD(i, t0)                                                         \
  do {                                                                        \
    uint64_t t1_ = ZD_NOW();                                                  \
    if (threadIdx.x == 0) atomicAdd(&g_zd_t[i], (unsigned long long)(t1_ - (t0))); \
    t0 = t1_;                                                                 \
  } while (0)
#else
#define ZD_NOW() 0ull
#define ZD_ADD(i, t0) (void)(t0)
#endif
// ------------------------------------------------------------------- lazy scan
struct ScanWin {
  uint32_t tf, tq, x;   // lane l: entries of position w + l, X byte w - 1 + l
  uint32_t d;
};

__device__ __forceinline__ void load_win(ScanWin& W, const ZArgs& a, const ZCall& c, int64_t w, int64_t p0) {
  const int lane = threadIdx.x;
  int64_t rel = w - WSIZE + lane;
  W.tf = 0;
  W.tq = 0;
  W.d = 0;
  if (w + lane >= p0 && rel < (int64_t)c.len) {
    W.tf = a.tf[c.t_off + rel + DMAX];
    W.tq = a.tq[c.t_off + rel + DMAX];
    W.d = a.d16[c.x_off + w + lane];
  }
  W.x = (rel - 1 < (int64_t)c.len) ? a.X[c.x_off + w - 1 + lane] : 0;
}

// deflate_slow (deflate.c) over the match table; one wave per call.
__global__ __launch_bounds__(64) void zd_scan_kernel(ZArgs a) {
  const uint32_t ci = blockIdx.x;
  const ZCall c = a.calls[ci];
  const ZState s = a.st[c.stream];
  const int lane = threadIdx.x;
  const int good = CFG[a.level][0], lazy = CFG[a.level][1];
  uint32_t* sym = a.sym + c.t_off;
  ZBlock* blk = a.blk + c.blk_off;
  const bool finish = c.len == 0;
  // positions are X indices; bidx = X index of zlib's window coord 0.  The
  // parse resumes where the last call's left it (strstart = total - dlen, with
  // its lazy-match state); data was read up to `total`.
  int64_t bidx = (int64_t)s.base - (int64_t)s.total + WSIZE;
  const int64_t end = (int64_t)WSIZE + c.len;
  const int64_t p0 = (int64_t)WSIZE - s.dlen;
  int64_t p = p0, rd = WSIZE;
  uint32_t nsym = 0, symbase = 0, nblk = 0;
  int64_t block_start = (int64_t)s.block_start - (int64_t)s.total + WSIZE;
  int ml = (int)s.mlen, avail = (int)s.avail;
  int64_t ms = (int64_t)s.mstart - (int64_t)s.total + WSIZE;
  ScanWin W, N;   // entries of [w, w + 64) and, loaded ahead, [w + 64, w + 128)
  int64_t w = p;
  load_win(W, a, c, w, p0);
  load_win(N, a, c, w + 64, p0);
#ifdef XCG_ZD_TIMING
  uint64_t n_fast = 0, n_slow = 0, n_fastpos = 0, t_scan = ZD_NOW();
#endif

  // FLUSH_BLOCK at strstart q; `tail`: inside the flush call (loop-top
  // lookahead < MIN_LOOKAHEAD, or the final flush); the parse then stands at
  // (pa, va, mla) -- where a consume that stops at this flush resumes
  auto flush = [&](int64_t q, bool last, bool tail, int64_t pa, int va, int mla) {
    if (lane == 0) {
      ZBlock b;
      b.sym_begin = symbase;
      b.sym_end = symbase + nsym;
      b.start = (uint32_t)block_start;
      b.stored_len = (uint32_t)(q - block_start);
      b.flags = (block_start >= bidx ? 1u : 0u) | (last ? 2u : 0u) | (tail ? 4u : 0u);
      b.type = 0;
      b.lcodes = b.dcodes = b.blcodes = b.pad = 0;
      b.bits = 0;
      b.bit_off = 0;
      b.bidx = bidx;
      b.p_after = (uint32_t)pa;
      b.ms = (uint32_t)ms;
      b.avail = (uint32_t)va;
      b.ml = (uint32_t)mla;
      blk[nblk] = b;
    }
    nblk++;
    symbase += nsym;
    nsym = 0;
    block_start = q;
  };
  // Symbols are staged in LDS and written out 2048 at a time (coalesced): a
  // store per symbol would make every window load wait for all earlier
  // stores (gfx9 counts both in vmcnt).
  __shared__ uint32_t sbuf[2048 + 64];
  uint32_t sb_n = 0, sb_base = 0;
  auto sflush = [&]() {
    for (uint32_t i = lane; i < sb_n; i += 64) sym[sb_base + i] = sbuf[i];
    sb_base += sb_n;
    sb_n = 0;
  };
  auto put = [&](uint32_t v) {
    if (lane == 0) sbuf[sb_n] = v;
    sb_n++;
    nsym++;
    if (sb_n >= 2048) sflush();
  };

  for (;;) {
    if (rd - p < MIN_LOOKAHEAD) {   // fill_window: slide, then read what fits
      do {
        int64_t more = WINSZ - (rd - bidx);
        if (p - bidx >= WSIZE + MAX_DIST) {
          bidx += WSIZE;
          more += WSIZE;
        }
        if (rd == end) break;
        int64_t nrd = end - rd;
        if (nrd > more) nrd = more;
        rd += nrd;
      } while (rd - p < MIN_LOOKAHEAD && rd < end);
      if (rd == p) break;
    }
    if (p >= w + 64) {
      if (p < w + 128) {
        W = N;
        w += 64;
      } else {
        w = p;
        load_win(W, a, c, w, p0);
      }
      load_win(N, a, c, w + 64, p0);
    }
    const int li = (int)(p - w);
    if (avail && ml == MIN_MATCH - 1) {
      // literal run: positions where no match can start emit the previous byte
      int64_t lim = w + 64;
      if (rd - (MIN_LOOKAHEAD - 1) < lim) lim = rd - (MIN_LOOKAHEAD - 1);
      int64_t room = SYMS_PER_BLOCK - nsym;
      if (p + room < lim) lim = p + room;
      if (lim > p) {
        uint32_t M = W.tf & 511u, dist = (W.tf >> 9) & 0x7fffu;
        int64_t pos = w + lane;
        bool elig = (W.tf >> 31) && pos - (int64_t)W.d != bidx && M >= MIN_MATCH && !(M == MIN_MATCH && dist > TOO_FAR);
        uint64_t m = ballot(elig && pos >= p && pos < lim);
        int64_t stop = m ? w + (int64_t)__builtin_ctzll(m) : lim;
        int64_t k = stop - p;
        if (k > 0) {
          if (lane >= li && lane < li + k) sbuf[sb_n + (lane - li)] = W.x;
          sb_n += (uint32_t)k;
          nsym += (uint32_t)k;
          if (sb_n >= 2048) sflush();
          p = stop;
#ifdef XCG_ZD_TIMING
          n_fast++;
          n_fastpos += (uint64_t)k;
#endif
          if (nsym == SYMS_PER_BLOCK) flush(p - 1, false, false, p, 1, MIN_MATCH - 1);
          continue;
        }
      }
    }
    // one loop top of deflate_slow at p
#ifdef XCG_ZD_TIMING
    n_slow++;
#endif
    const uint32_t ef = readlane(W.tf, li), dd = readlane(W.d, li);
    const int64_t la = rd - p;
    int prev_length = ml;
    int64_t prev_match = ms;
    ml = MIN_MATCH - 1;
    bool head_ok = la >= MIN_MATCH && (ef >> 31) && (p - (int64_t)dd != bidx);
    if (head_ok && prev_length < lazy) {
      uint32_t e = prev_length >= good ? readlane(W.tq, li) : ef;
      int M = (int)(e & 511u);
      if (M > prev_length) {
        ml = M;
        ms = p - (int64_t)((e >> 9) & 0x7fffu);
      } else {
        ml = (int64_t)prev_length <= la ? prev_length : (int)la;
      }
      if (ml == MIN_MATCH && p - ms > TOO_FAR) ml = MIN_MATCH - 1;
    }
    if (prev_length >= MIN_MATCH && ml <= prev_length) {
      put((uint32_t)(prev_length - MIN_MATCH) | ((uint32_t)(p - 1 - prev_match) << 8));
      p += prev_length - 1;
      avail = 0;
      ml = MIN_MATCH - 1;
      if (nsym == SYMS_PER_BLOCK) flush(p, false, la < MIN_LOOKAHEAD, p, 0, MIN_MATCH - 1);
    } else if (avail) {
      put(readlane(W.x, li));
      if (nsym == SYMS_PER_BLOCK) flush(p, false, la < MIN_LOOKAHEAD, p + 1, 1, ml);
      p++;
    } else {
      avail = 1;
      p++;
    }
  }
  if (avail) put(a.X[c.x_off + p - 1]);
  sflush();
#ifdef XCG_ZD_TIMING
  if (lane == 0) {
    atomicAdd(&g_zd_t[5], (unsigned long long)n_slow);
    atomicAdd(&g_zd_t[6], (unsigned long long)n_fast);
    atomicAdd(&g_zd_t[7], (unsigned long long)n_fastpos);
    atomicAdd(&g_zd_t[11], (unsigned long long)(ZD_NOW() - t_scan));
    atomicAdd(&g_zd_t[12], 1ull);
  }
#endif
  if (finish) flush(p, true, true, p, 0, MIN_MATCH - 1);
  else if (nsym) flush(p, false, true, p, 0, MIN_MATCH - 1);
  if (lane == 0) {
    ZCallRes r = a.res[ci];
    r.nblocks = nblk;
    r.nsym = symbase;
    r.base_end = (uint64_t)((int64_t)s.total - WSIZE + bidx);
    r.scan_end = (uint32_t)p;
    a.res[ci] = r;
  }
}

// ------------------------------------------------------------------- deflate_fast
// deflate_fast (deflate.c, levels 1-3) over the match table built from this
// round's hashed-position guess (ZArgs::mcur); one wave per call.  zlib hashes
// every loop top with >= MIN_MATCH bytes of lookahead and the inside of a match
// only when it is at most max_lazy (= max_insert_length) long and leaves >=
// MIN_MATCH bytes of lookahead; the positions this parse hashes go to mnext.
// When mnext == mcur the table was zlib's (by induction over positions: a
// loop top's chain holds exactly the positions hashed before it) and so is
// the parse.
__device__ __forceinline__ void mark_range(uint32_t* mk, int64_t lo, int64_t hi, int lane) {
  if (hi <= lo) return;
  const int64_t w0 = lo >> 5, w1 = (hi - 1) >> 5;
  for (int64_t wd = w0 + lane; wd <= w1; wd += 64) {
    const int64_t b0 = wd * 32, a0 = lo > b0 ? lo - b0 : 0, a1 = hi < b0 + 32 ? hi - b0 : 32;
    const uint32_t m = (a1 - a0 == 32) ? ~0u : (((1u << (a1 - a0)) - 1u) << a0);
    atomicOr(mk + wd, m);
  }
}

__global__ __launch_bounds__(64) void zd_fscan_kernel(ZArgs a) {
  const uint32_t ci = blockIdx.x;
  const ZCall c = a.calls[ci];
  const ZState s = a.st[c.stream];
  const int lane = threadIdx.x;
  const int max_insert = CFG[a.level][1];
  uint32_t* sym = a.sym + c.t_off;
  ZBlock* blk = a.blk + c.blk_off;
  uint32_t* mk = a.mnext + c.m_off;
  const bool finish = c.len == 0;
  int64_t bidx = (int64_t)s.base - (int64_t)s.total + WSIZE;
  const int64_t end = (int64_t)WSIZE + c.len;
  const int64_t p0 = (int64_t)WSIZE - s.dlen;
  int64_t p = p0, rd = WSIZE;
  uint32_t nsym = 0, symbase = 0, nblk = 0;
  int64_t block_start = (int64_t)s.block_start - (int64_t)s.total + WSIZE;
  ScanWin W, N;
  int64_t w = p;
  load_win(W, a, c, w, p0);
  load_win(N, a, c, w + 64, p0);
  auto flush = [&](int64_t q, bool last, bool tail) {   // FLUSH_BLOCK at strstart q (after its symbol)
    if (lane == 0) {
      ZBlock b;
      b.sym_begin = symbase;
      b.sym_end = symbase + nsym;
      b.start = (uint32_t)block_start;
      b.stored_len = (uint32_t)(q - block_start);
      b.flags = (block_start >= bidx ? 1u : 0u) | (last ? 2u : 0u) | (tail ? 4u : 0u);
      b.type = 0;
      b.lcodes = b.dcodes = b.blcodes = b.pad = 0;
      b.bits = 0;
      b.bit_off = 0;
      b.bidx = bidx;
      b.p_after = (uint32_t)q;
      b.ms = 0;
      b.avail = 0;
      b.ml = MIN_MATCH - 1;
      blk[nblk] = b;
    }
    nblk++;
    symbase += nsym;
    nsym = 0;
    block_start = q;
  };
  __shared__ uint32_t sbuf[2048 + 64];
  uint32_t sb_n = 0, sb_base = 0;
  auto sflush = [&]() {
    for (uint32_t i = lane; i < sb_n; i += 64) sym[sb_base + i] = sbuf[i];
    sb_base += sb_n;
    sb_n = 0;
  };
  auto put = [&](uint32_t v) {
    if (lane == 0) sbuf[sb_n] = v;
    sb_n++;
    nsym++;
    if (sb_n >= 2048) sflush();
  };
  for (;;) {
    if (rd - p < MIN_LOOKAHEAD) {   // fill_window: slide, then read what fits
      do {
        int64_t more = WINSZ - (rd - bidx);
        if (p - bidx >= WSIZE + MAX_DIST) {
          bidx += WSIZE;
          more += WSIZE;
        }
        if (rd == end) break;
        int64_t nrd = end - rd;
        if (nrd > more) nrd = more;
        rd += nrd;
      } while (rd - p < MIN_LOOKAHEAD && rd < end);
      if (rd == p) break;
    }
    if (p >= w + 64) {
      if (p < w + 128) {
        W = N;
        w += 64;
      } else {
        w = p;
        load_win(W, a, c, w, p0);
      }
      load_win(N, a, c, w + 64, p0);
    }
    const int li = (int)(p - w);
    // X[w + lane] (W.x holds X[w - 1 + lane])
    uint32_t xs = __shfl(W.x, (lane + 1) & 63);
    const uint32_t nx0 = readlane(N.x, 0);
    if (lane == 63) xs = nx0;
    {
      // literal run: loop tops where no match starts (all hashed, lookahead >= MIN_LOOKAHEAD)
      int64_t lim = w + 64;
      if (rd - (MIN_LOOKAHEAD - 1) < lim) lim = rd - (MIN_LOOKAHEAD - 1);
      const int64_t room = SYMS_PER_BLOCK - nsym;
      if (p + room < lim) lim = p + room;
      if (lim > p) {
        const int64_t pos = w + lane;
        const bool elig = (W.tf >> 31) && pos - (int64_t)W.d != bidx && (W.tf & 511u) >= MIN_MATCH;
        const uint64_t m = ballot(elig && pos >= p && pos < lim);
        const int64_t stop = m ? w + (int64_t)__builtin_ctzll(m) : lim;
        const int64_t k = stop - p;
        if (k > 0) {
          if (lane >= li && lane < li + k) sbuf[sb_n + (lane - li)] = xs;
          sb_n += (uint32_t)k;
          nsym += (uint32_t)k;
          if (sb_n >= 2048) sflush();
          mark_range(mk, p, stop, lane);
          p = stop;
          if (nsym == SYMS_PER_BLOCK) flush(p, false, false);
          continue;
        }
      }
    }
    // one loop top of deflate_fast at p
    const uint32_t ef = readlane(W.tf, li), dd = readlane(W.d, li);
    const int64_t la = rd - p;
    if (la >= MIN_MATCH && lane == 0) atomicOr(mk + (p >> 5), 1u << (p & 31));   // INSERT_STRING
    const bool head_ok = la >= MIN_MATCH && (ef >> 31) && (p - (int64_t)dd != bidx);
    const int ml = head_ok ? (int)(ef & 511u) : 0;
    if (ml >= MIN_MATCH) {
      put((uint32_t)(ml - MIN_MATCH) | (((ef >> 9) & 0x7fffu) << 8));
      if (ml <= max_insert && la - ml >= MIN_MATCH) mark_range(mk, p + 1, p + ml, lane);
      p += ml;
    } else {
      put(readlane(xs, li));
      p++;
    }
    if (nsym == SYMS_PER_BLOCK) flush(p, false, la < MIN_LOOKAHEAD);
  }
  sflush();
  // s->insert = min(strstart, MIN_MATCH - 1): the last positions are hashed once their bytes exist
  const int64_t ins = p - bidx < MIN_MATCH - 1 ? p - bidx : MIN_MATCH - 1;
  mark_range(mk, p - ins, p, lane);
  if (finish) flush(p, true, true);
  else if (nsym) flush(p, false, true);
  if (lane == 0) {
    ZCallRes r = a.res[ci];
    r.nblocks = nblk;
    r.nsym = symbase;
    r.base_end = (uint64_t)((int64_t)s.total - WSIZE + bidx);
    r.scan_end = (uint32_t)p;
    a.res[ci] = r;
  }
}

// mnext == mcur over the positions the call parses? (changed[ci] = 1 if not)
__global__ __launch_bounds__(256) void zd_mcmp_kernel(ZArgs a) {
  const uint32_t ci = blockIdx.x;
  const ZCall c = a.calls[ci];
  const ZState s = a.st[c.stream];
  const int64_t lo = (int64_t)WSIZE - s.dlen, hi = (int64_t)WSIZE + c.len;
  bool diff = false;
  for (int64_t wd = (lo >> 5) + threadIdx.x; wd <= ((hi - 1) >> 5); wd += 256) {
    const int64_t b0 = wd * 32, a0 = lo > b0 ? lo - b0 : 0, a1 = hi < b0 + 32 ? hi - b0 : 32;
    const uint32_t m = (a1 - a0 == 32) ? ~0u : (((1u << (a1 - a0)) - 1u) << a0);
    if ((a.mcur[c.m_off + wd] ^ a.mnext[c.m_off + wd]) & m) diff = true;
  }
  if (__syncthreads_or(diff) && threadIdx.x == 0) a.changed[ci] = 1u;
}

// Round 0's guess: every position hashed.  Also clears mnext.
__global__ __launch_bounds__(256) void zd_mfill_kernel(uint32_t* m, uint32_t* mn, uint64_t words) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256) {
    m[i] = ~0u;
    mn[i] = 0u;
  }
}
__global__ __launch_bounds__(256) void zd_mzero_kernel(uint32_t* m, uint64_t words) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256) m[i] = 0u;
}

// The stream's ring of hashed positions after the call: bit (q mod 32768) for
// the last 32 KiB; positions from strstart on come from the final mask.
__global__ __launch_bounds__(256) void zd_ring_kernel(ZArgs a) {
  const uint32_t ci = blockIdx.x;
  const ZCall c = a.calls[ci];
  const ZState s = a.st[c.stream];
  const uint64_t hi = s.total + c.len, p0 = s.total - s.dlen;
  const uint64_t lo = hi > (uint64_t)WSIZE ? hi - WSIZE : 0;
  const uint64_t from = p0 > lo ? p0 : lo;
  uint32_t* ring = a.ring + (uint64_t)c.stream * (WSIZE / 32);
  const uint32_t* mk = a.mcur + c.m_off;
  for (uint32_t r = threadIdx.x; r < (uint32_t)WSIZE / 32; r += 256) {
    uint32_t v = ring[r];
    for (int b = 0; b < 32; b++) {
      const uint64_t slot = (uint64_t)r * 32 + b;
      if (hi < (uint64_t)WSIZE && slot >= hi) continue;   // (no such position yet)
      const uint64_t q = hi - WSIZE + ((slot - hi) & (WSIZE - 1));   // the position in [hi - 32768, hi) on this slot
      if (q < from) continue;
      const uint64_t j = q - (s.total - WSIZE);
      const uint32_t bit = (mk[j >> 5] >> (j & 31)) & 1u;
      v = (v & ~(1u << b)) | (bit << b);
    }
    ring[r] = v;
  }
}

// ------------------------------------------------------------------- trees
// Heap entries are freq << 15 | depth << 10 | node: trees.c's smaller(n, m)
// (freq, then depth <=) is `key(n) <= key(m)` on key = entry >> 10, so a
// downheap step is one 8-byte LDS read of both children.  A block holds at
// most 16383 symbols + END_BLOCK (+2 forced), so freq < 2^17, and a Huffman
// tree over that total weight is at most ~21 deep (Fibonacci bound): depth
// fits 5 bits, nodes (< 573) 10.
struct TreeLds {
  uint32_t heap[HEAP_SIZE + 1];
  uint16_t dl[HEAP_SIZE + 1];  // Dad | Len
  uint16_t fc[L_CODES];        // leaf Freq | Code
  uint16_t dfc[D_CODES], ddl[2 * D_CODES + 1];
  uint16_t bfc[BL_CODES], bdl[2 * BL_CODES + 1];
  uint16_t lfreq[L_CODES], dfreq[D_CODES], bfreq[BL_CODES + 1];   // real counts (forced codes excluded)
  uint16_t bl_count[MAX_BITS + 1];
  uint32_t next_code[MAX_BITS + 1];
  int64_t opt_len, static_len;
};
// one TreeLds per lane-owned block, at a stride of 4 mod 64 words (16-byte aligned, no bank conflicts
// between the TB lanes)
constexpr int TB_BATCH = 2;   // blocks per wave in batches (one per wave when few blocks)
constexpr uint32_t TSTRIDE = ((sizeof(TreeLds) + 255) / 256) * 256 + 16;

__device__ __forceinline__ uint32_t hkey(uint32_t e) { return e >> 10; }
// Two levels per LDS round trip: the children pair and the four grandchildren
// are read together (stores along the path go to indices below both).
__device__ void downheap(TreeLds& s, int k, int len) {
  const uint32_t v = s.heap[k], kv = hkey(v);
  int j = k << 1;
  while (j <= len) {
    const uint2 p = *(const uint2*)&s.heap[j];   // j even
    uint4 g = make_uint4(0, 0, 0, 0);
    if (2 * j <= len) g = *(const uint4*)&s.heap[2 * j];   // 2j % 4 == 0
    uint32_t e = p.x;
    if (j < len && hkey(p.y) <= hkey(p.x)) {
      e = p.y;
      j++;
    }
    if (kv <= hkey(e)) break;
    s.heap[k] = e;
    k = j;
    const bool right = j & 1;
    j <<= 1;
    if (j > len) break;
    const uint32_t e0 = right ? g.z : g.x, e1 = right ? g.w : g.y;
    e = e0;
    if (j < len && hkey(e1) <= hkey(e0)) {
      e = e1;
      j++;
    }
    if (kv <= hkey(e)) break;
    s.heap[k] = e;
    k = j;
    j <<= 1;
  }
  s.heap[k] = v;
}
__device__ __forceinline__ int static_llen(int n) { return n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8; }

// trees.c build_tree + gen_bitlen + gen_codes.  kind: 0 literal/length, 1 distance, 2 bit length.
__device__ int build_tree(TreeLds& s, uint16_t* fc, uint16_t* dl, int elems, int kind) {
  const int maxlen = kind == 2 ? 7 : MAX_BITS;
  int n, m, max_code = -1, node;
  int len = 0, hmax = HEAP_SIZE;
  for (n = 0; n < elems; n++) {
    if (fc[n]) {
      s.heap[++len] = ((uint32_t)fc[n] << 15) | (uint32_t)n;
      max_code = n;
    } else {
      dl[n] = 0;
    }
  }
  while (len < 2) {
    node = max_code < 2 ? ++max_code : 0;
    s.heap[++len] = (1u << 15) | (uint32_t)node;
    fc[node] = 1;
    s.opt_len--;
    if (kind == 0) s.static_len -= static_llen(node);
    else if (kind == 1) s.static_len -= 5;
  }
  for (n = len / 2; n >= 1; n--) downheap(s, n, len);
  node = elems;
  do {
    const uint32_t en = s.heap[1];
    s.heap[1] = s.heap[len--];
    downheap(s, 1, len);
    const uint32_t em = s.heap[1];
    s.heap[--hmax] = en;
    s.heap[--hmax] = em;
    const uint32_t dn = (en >> 10) & 31, dm = (em >> 10) & 31;
    const uint32_t f = (en >> 15) + (em >> 15), d = (dn >= dm ? dn : dm) + 1;
    dl[en & 1023] = dl[em & 1023] = (uint16_t)node;
    s.heap[1] = (f << 15) | (d << 10) | (uint32_t)node++;
    downheap(s, 1, len);
  } while (len >= 2);
  s.heap[--hmax] = s.heap[1];

  int h, bits, overflow = 0;
  for (bits = 0; bits <= MAX_BITS; bits++) s.bl_count[bits] = 0;
  dl[s.heap[hmax] & 1023] = 0;
  for (h = hmax + 1; h < HEAP_SIZE; h++) {
    n = s.heap[h] & 1023;
    bits = dl[dl[n]] + 1;
    if (bits > maxlen) {
      bits = maxlen;
      overflow++;
    }
    dl[n] = (uint16_t)bits;
    if (n > max_code) continue;
    s.bl_count[bits]++;
    int xb = 0;
    if (kind == 0 && n >= 257) xb = XLB[n - 257];
    else if (kind == 1) xb = XDB[n];
    else if (kind == 2) xb = XBB[n];
    s.opt_len += (int64_t)fc[n] * (bits + xb);
    if (kind == 0) s.static_len += (int64_t)fc[n] * (static_llen(n) + xb);
    else if (kind == 1) s.static_len += (int64_t)fc[n] * (5 + xb);
  }
  if (overflow) {
    do {
      bits = maxlen - 1;
      while (s.bl_count[bits] == 0) bits--;
      s.bl_count[bits]--;
      s.bl_count[bits + 1] += 2;
      s.bl_count[maxlen]--;
      overflow -= 2;
    } while (overflow > 0);
    for (bits = maxlen; bits != 0; bits--) {
      n = s.bl_count[bits];
      while (n != 0) {
        m = s.heap[--h] & 1023;
        if (m > max_code) continue;
        if (dl[m] != (unsigned)bits) {
          s.opt_len += ((int64_t)bits - dl[m]) * fc[m];
          dl[m] = (uint16_t)bits;
        }
        n--;
      }
    }
  }
  uint32_t code = 0;
  for (bits = 1; bits <= MAX_BITS; bits++) {
    code = (code + s.bl_count[bits - 1]) << 1;
    s.next_code[bits] = code;
  }
  for (n = 0; n <= max_code; n++) {
    const int l = dl[n];
    if (l) fc[n] = (uint16_t)bitrev(s.next_code[l]++, l);
  }
  return max_code;
}

// scan_tree: bit-length code frequencies of one tree's lengths (guard: 0xffff)
__device__ void scan_tree(TreeLds& s, const uint16_t* dl, int max_code) {
  int prevlen = -1, curlen, nextlen = dl[0], count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) {
    max_count = 138;
    min_count = 3;
  }
  for (int n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = n + 1 <= max_code ? dl[n + 1] : 0xffff;
    if (++count < max_count && curlen == nextlen) continue;
    if (count < min_count) s.bfreq[curlen] += count;
    else if (curlen != 0) {
      if (curlen != prevlen) s.bfreq[curlen]++;
      s.bfreq[16]++;
    } else if (count <= 10) s.bfreq[17]++;
    else s.bfreq[18]++;
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) {
      max_count = 138;
      min_count = 3;
    } else if (curlen == nextlen) {
      max_count = 6;
      min_count = 3;
    } else {
      max_count = 7;
      min_count = 4;
    }
  }
}

// One wave per block: histogram, trees, the _tr_flush_block decision and the
// block's exact bit count; code tables to `tabs`.
// TB blocks per wave: the wave builds each block's symbol histogram in turn,
// then lane t runs block t's trees (the heap work is a serial chain per
// block; one lane per block spends the wave's VALU issue slots on TB chains
// instead of one), then the code tables leave with the whole wave.
template <int TB>
__global__ __launch_bounds__(64) void zd_trees_kernel(ZArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[TB * TSTRIDE];
  __shared__ int ttype[TB];
  const int lane = threadIdx.x;
  const uint32_t nrec = a.bstart[a.n];
  uint64_t tz = ZD_NOW();
  for (int t = 0; t < TB; t++) {
    const uint32_t bi = blockIdx.x * TB + t;
    if (lane == 0) ttype[t] = -1;
    if (bi >= nrec) continue;
    const uint32_t ci = call_of(a.bstart, a.n, bi);
    const ZCall c = a.calls[ci];
    if (bi - c.blk_off >= a.res[ci].nblocks) continue;
    TreeLds& s = *(TreeLds*)(raw + t * TSTRIDE);
    uint32_t* hist = s.heap;   // the symbol counts live in the block's heap until build_tree
    for (int i = lane; i < L_CODES + D_CODES; i += 64) hist[i] = 0;
    __syncthreads();
    const ZBlock* B = a.blk + bi;
    const uint32_t* sym = a.sym + c.t_off;
    const uint32_t sb = B->sym_begin, se = B->sym_end;
    for (uint32_t i0 = sb; i0 < se; i0 += 64 * 8) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const uint32_t i = i0 + 64 * q + lane;
        v[q] = i < se ? sym[i] : 0xffffffffu;
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {
        if (v[q] == 0xffffffffu) continue;
        const uint32_t dist = v[q] >> 8;
        if (dist == 0) atomicAdd(&hist[v[q] & 255], 1u);
        else {
          atomicAdd(&hist[257 + len_code(v[q] & 255)], 1u);
          atomicAdd(&hist[L_CODES + dist_code(dist - 1)], 1u);
        }
      }
    }
    __syncthreads();
    for (int i = lane; i < L_CODES; i += 64) {
      const uint16_t f = i == 256 ? 1 : (uint16_t)hist[i];
      s.lfreq[i] = f;
      s.fc[i] = f;
    }
    if (lane < D_CODES) s.dfreq[lane] = s.dfc[lane] = (uint16_t)hist[L_CODES + lane];
    if (lane <= BL_CODES) s.bfreq[lane] = 0;
    if (lane == 0) ttype[t] = 0;
    __syncthreads();
  }
  ZD_ADD(0, tz);
  if (lane < TB && ttype[lane] >= 0) {
    TreeLds& s = *(TreeLds*)(raw + lane * TSTRIDE);
    ZBlock* B = a.blk + blockIdx.x * TB + lane;
    s.opt_len = s.static_len = 0;
    int lmax = build_tree(s, s.fc, s.dl, L_CODES, 0);
    ZD_ADD(1, tz);
    int dmax = build_tree(s, s.dfc, s.ddl, D_CODES, 1);
    scan_tree(s, s.dl, lmax);
    scan_tree(s, s.ddl, dmax);
    for (int i = 0; i < BL_CODES; i++) s.bfc[i] = s.bfreq[i];
    build_tree(s, s.bfc, s.bdl, BL_CODES, 2);
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
      if (s.bdl[BL_ORDER[max_blindex]] != 0) break;
    s.opt_len += 3 * ((int64_t)max_blindex + 1) + 5 + 5 + 4;
    ZD_ADD(2, tz);
    int64_t opt_lenb = (s.opt_len + 3 + 7) >> 3, static_lenb = (s.static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    uint32_t type;
    if ((int64_t)B->stored_len + 4 <= opt_lenb && (B->flags & 1)) type = 0;
    else if (static_lenb == opt_lenb) type = 1;
    else type = 2;
    // exact bits of a Huffman block (real symbol counts; forced codes emit nothing)
    uint64_t bits = 3;
    if (type == 1) {
      for (int i = 0; i < L_CODES; i++)
        bits += (uint64_t)s.lfreq[i] * (static_llen(i) + (i >= 257 ? XLB[i - 257] : 0));
      for (int i = 0; i < D_CODES; i++) bits += (uint64_t)s.dfreq[i] * (5 + XDB[i]);
    } else if (type == 2) {
      bits += 14 + 3 * (uint64_t)(max_blindex + 1);
      for (int i = 0; i < BL_CODES; i++) bits += (uint64_t)s.bfreq[i] * (s.bdl[i] + XBB[i]);
      for (int i = 0; i < L_CODES; i++) bits += (uint64_t)s.lfreq[i] * (s.dl[i] + (i >= 257 ? XLB[i - 257] : 0));
      for (int i = 0; i < D_CODES; i++) bits += (uint64_t)s.dfreq[i] * (s.ddl[i] + XDB[i]);
    }
    B->type = type;
    B->bits = bits;
    B->lcodes = lmax + 1;
    B->dcodes = dmax + 1;
    B->blcodes = max_blindex + 1;
    ttype[lane] = (int)type;
    ZD_ADD(3, tz);
  }
  __syncthreads();
  for (int t = 0; t < TB; t++) {
    if (ttype[t] != 2) continue;
    const TreeLds& s = *(const TreeLds*)(raw + t * TSTRIDE);
    uint32_t* tab = a.tabs + (uint64_t)(blockIdx.x * TB + t) * TAB_WORDS;
    for (int i = lane; i < L_CODES; i += 64) tab[i] = s.fc[i] | ((uint32_t)s.dl[i] << 16);
    if (lane < D_CODES) tab[L_CODES + lane] = s.dfc[lane] | ((uint32_t)s.ddl[lane] << 16);
    if (lane < BL_CODES) tab[L_CODES + D_CODES + lane] = s.bfc[lane] | ((uint32_t)s.bdl[lane] << 16);
  }
  ZD_ADD(4, tz);
#ifdef XCG_ZD_TIMING
  if (lane == 0) atomicAdd(&g_zd_t[14], 1ull);
#endif
}

// ------------------------------------------------------------------- layout
// One wave per call: block bit offsets, the call's length, zeroed output, and
// where DeflatePipe::consume (zlib/deflate_pipe.cc:57-115) stops.  Output
// reaches the pipe at every block flush (flush_pending: the complete bytes).
// Under Z_NO_FLUSH the pipe takes all of it, emptying its 64 KiB buffer as it
// fills, so the one deflate(Z_SYNC_FLUSH) call starts with n mod 65536 bytes
// in the buffer (n = the bytes the consume took so far, the ones zlib still
// held from the last consume included) and returns at the first block flush
// that leaves the buffer full (FLUSH_BLOCK's need_more): the consume produces
// up to L = 65536 * (n / 65536 + 1), the rest stays pending, no sync marker
// is written, and positions after that flush are parsed with the next
// consume's bytes.  Otherwise the marker follows and the consume produces
// min(all, L).  Bits of an incomplete last byte carry into the next call
// (the call's output starts with them).
__global__ __launch_bounds__(64) void zd_layout_kernel(ZArgs a) {
  const uint32_t ci = blockIdx.x;
  const ZCall c = a.calls[ci];
  const ZState s = a.st[c.stream];
  const int lane = threadIdx.x;
  __shared__ uint32_t total_bytes;
  if (lane == 0) {
    uint64_t off = (s.flags & 1) ? s.cnb : 16;   // carried bits, or the zlib header on the first call
    const uint32_t nb = a.res[ci].nblocks;
    const bool finish = c.len == 0;
    bool last = false;
    uint32_t stop = 0, nemit = nb;
    uint64_t n = s.pend;                          // bytes the consume took before its flush call
    for (uint32_t k = 0; k < nb; k++) {
      ZBlock* B = a.blk + c.blk_off + k;
      B->bit_off = off;
      if (B->type == 0) off = (((off + 3 + 7) >> 3) + 4 + B->stored_len) * 8;
      else off += B->bits;
      if (B->flags & 2) {
        off = (off + 7) & ~7ull;   // bi_windup after the last block
        last = true;
      }
      if (finish) continue;
      const uint64_t avail = s.pend + (off >> 3);
      if (!(B->flags & 4)) {
        n = avail;
      } else if (avail >= (uint64_t)PIPE_CHUNK * (n / PIPE_CHUNK + 1)) {
        stop = k + 1;
        nemit = k + 1;
        break;
      }
    }
    ZCallRes& r = a.res[ci];
    r.end_bit = off;
    r.nblocks = nemit;
    r.stop = stop;
    uint64_t bytes, room;
    if (last) bytes = room = off / 8 + 4;                           // adler32 trailer
    else if (stop) { bytes = off >> 3; room = (off + 7) >> 3; }     // no marker; the partial byte carries
    else bytes = room = ((off + 3 + 7) >> 3) + 4;                   // Z_SYNC_FLUSH: empty stored block
    const uint64_t lim = (uint64_t)PIPE_CHUNK * (n / PIPE_CHUNK + 1), all = s.pend + bytes;
    r.deliver = finish ? all : (all < lim ? all : lim);
    r.out_bytes = (uint32_t)bytes;
    total_bytes = (uint32_t)room;
    r.out_len = (uint32_t)room;
    a.out_len[ci] = (uint32_t)bytes;
    a.deliver[ci] = r.deliver;
  }
  __syncthreads();
  uint32_t* o = (uint32_t*)(a.out + c.out_off);
  uint32_t words = (total_bytes + 3) / 4;
  for (uint32_t i = lane; i < words; i += 64) o[i] = 0;
  __syncthreads();
  if (lane == 0 && (s.flags & 1) && s.cnb) o[0] |= s.cbits;   // (the header call starts byte-aligned)
}

// ------------------------------------------------------------------- emit
// Output words of one call: writes past its computed length are dropped (they
// cannot happen when the layout is right; the guard keeps a bug from touching
// another call's output).
struct OutW {
  uint32_t* o;
  uint64_t nwords;
};
__device__ __forceinline__ void or_word(OutW o, uint64_t wi, uint32_t v) {
  if (v && wi < o.nwords) atomicOr(o.o + wi, v);
}
__device__ __forceinline__ void or_bits(OutW o, uint64_t pos, uint64_t v, int nb) {
  // v < 2^nb, nb <= 48: spans at most three words
  if (nb == 0) return;
  uint64_t wi = pos >> 5;
  int sh = (int)(pos & 31);
  uint64_t lo = v << sh;                     // bits [sh, sh + nb) of a 96-bit window
  or_word(o, wi, (uint32_t)lo);
  or_word(o, wi + 1, (uint32_t)(lo >> 32));
  if (sh) or_word(o, wi + 2, (uint32_t)(v >> (64 - sh)));
}
__device__ __forceinline__ void or_byte(OutW o, uint64_t byte, uint32_t v) {
  or_word(o, byte >> 2, v << (8 * (byte & 3)));
}

// Huffman blocks are packed through an LDS ring of output words: absolute
// word w of the call's output lives in ring[w % RING] until it is complete.
constexpr int RING = 512;
struct RingW {          // lane-0 sequential writer (block header, tree description)
  uint32_t* ring;
  uint64_t pos;
  __device__ void put(uint32_t v, int n) {   // v < 2^n, n <= 16
    const uint64_t x = (uint64_t)v << (pos & 31);
    const uint64_t w = pos >> 5;
    if ((uint32_t)x) atomicOr(&ring[w % RING], (uint32_t)x);
    if (x >> 32) atomicOr(&ring[(w + 1) % RING], (uint32_t)(x >> 32));
    pos += n;
  }
};

__device__ void send_tree(RingW& bw, const uint32_t* tab, int max_code, const uint32_t* btab) {
  int prevlen = -1, curlen, nextlen = tab[0] >> 16, count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) {
    max_count = 138;
    min_count = 3;
  }
  auto code = [&](int c) { bw.put(btab[c] & 0xffff, btab[c] >> 16); };
  for (int n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = n + 1 <= max_code ? (int)(tab[n + 1] >> 16) : 0xffff;
    if (++count < max_count && curlen == nextlen) continue;
    if (count < min_count) {
      do code(curlen);
      while (--count != 0);
    } else if (curlen != 0) {
      if (curlen != prevlen) {
        code(curlen);
        count--;
      }
      code(16);
      bw.put(count - 3, 2);
    } else if (count <= 10) {
      code(17);
      bw.put(count - 3, 3);
    } else {
      code(18);
      bw.put(count - 11, 7);
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) {
      max_count = 138;
      min_count = 3;
    } else if (curlen == nextlen) {
      max_count = 6;
      min_count = 3;
    } else {
      max_count = 7;
      min_count = 4;
    }
  }
}

__device__ __forceinline__ uint32_t static_lcode(int n) {   // fixed literal/length tree (code | len << 16)
  uint32_t len, code;
  if (n < 144) { len = 8; code = 0x30 + n; }
  else if (n < 256) { len = 9; code = 0x190 + (n - 144); }
  else if (n < 280) { len = 7; code = n - 256; }
  else { len = 8; code = 0xc0 + (n - 280); }
  return bitrev(code, len) | (len << 16);
}

// One wave per block.  Huffman blocks: per-block LDS tables give every symbol
// its bits with the extra bits merged (literal: code; length: code + extra;
// distance: code + extra), 64 symbols per step are loaded coalesced (prefetched
// a step ahead), a wave scan places them, they are OR-ed into the LDS ring, and
// completed words leave with coalesced stores -- the block's first and last
// words (shared with its neighbours) with atomicOr.
constexpr int EBATCH = 4;   // 64-symbol steps per prefetch
__global__ __launch_bounds__(64) void zd_emit_kernel(ZArgs a) {
  __shared__ uint32_t litx[256], lenx[256], dtx[D_CODES];   // bits | nbits << 24 (dist: code | nbits << 16)
  __shared__ uint32_t stab[TAB_WORDS];
  __shared__ uint32_t ring[RING];
  const uint32_t bi = blockIdx.x;
  const uint32_t ci = call_of(a.bstart, a.n, bi);
  const ZCall c = a.calls[ci];
  const uint32_t k = bi - c.blk_off;
  const ZCallRes r = a.res[ci];
  if (k >= r.nblocks) return;
  const ZBlock B = a.blk[bi];
  const ZState s = a.st[c.stream];
  const int lane = threadIdx.x;
  uint64_t tz = ZD_NOW();
  const OutW o{(uint32_t*)(a.out + c.out_off), (r.out_len + 3ull) / 4};
  const OutW ob = o;
  const bool last = B.flags & 2;
  if (k == 0 && lane == 0 && !(s.flags & 1)) {   // zlib header (deflate.c: 0x78, level flags)
    int lf = a.level < 2 ? 0 : a.level < 6 ? 1 : a.level == 6 ? 2 : 3;
    uint32_t hdr = ((8 + (7 << 4)) << 8) | (lf << 6);
    hdr += 31 - (hdr % 31);
    or_byte(ob, 0, hdr >> 8);
    or_byte(ob, 1, hdr & 0xff);
  }
  if (B.type == 0) {   // _tr_stored_block
    if (lane == 0) {
      or_bits(o, B.bit_off, last ? 1 : 0, 3);
      uint64_t db = (B.bit_off + 3 + 7) >> 3;
      uint32_t L = B.stored_len;
      or_byte(ob, db, L & 0xff);
      or_byte(ob, db + 1, (L >> 8) & 0xff);
      or_byte(ob, db + 2, ~L & 0xff);
      or_byte(ob, db + 3, (~L >> 8) & 0xff);
    }
    const uint8_t* X = a.X + c.x_off + B.start;
    uint64_t db = ((B.bit_off + 3 + 7) >> 3) + 4;
    // whole words inside [db, db + L) by plain stores, the edge words by atomicOr
    uint64_t w0 = (db + 3) >> 2, w1 = (db + B.stored_len) >> 2;
    for (uint64_t wi = w0 + lane; wi < w1 && wi < o.nwords; wi += 64) {
      uint64_t b = wi * 4 - db;
      o.o[wi] = ld32(X + b);
    }
    for (uint64_t i = lane; i < B.stored_len; i += 64) {
      uint64_t byte = db + i;
      if ((byte >> 2) < w0 || (byte >> 2) >= w1) or_byte(ob, byte, X[i]);
    }
  } else {
    const bool dyn = B.type == 2;
    const uint32_t* tab = a.tabs + (uint64_t)bi * TAB_WORDS;
    if (dyn)
      for (int i = lane; i < TAB_WORDS; i += 64) stab[i] = tab[i];
    for (int i = lane; i < RING; i += 64) ring[i] = 0;
    __syncthreads();
    auto lcode = [&](int n) { return dyn ? stab[n] : static_lcode(n); };
    for (int i = lane; i < 256; i += 64) {
      const uint32_t t = lcode(i);
      litx[i] = (t & 0xffff) | ((t >> 16) << 24);
      const int code = len_code(i), xl = XLB[code];
      const uint32_t u = lcode(257 + code), hl = u >> 16;
      lenx[i] = ((u & 0xffff) | (xl ? (uint32_t)(i - BASE_LEN[code]) << hl : 0u)) | ((hl + xl) << 24);
    }
    if (lane < D_CODES) dtx[lane] = dyn ? stab[L_CODES + lane] : (bitrev(lane, 5) | (5u << 16));
    const uint32_t eob = lcode(256);
    uint64_t pos = B.bit_off;
    __syncthreads();
    if (lane == 0) {
      RingW bw{ring, pos};
      bw.put((B.type << 1) | (last ? 1 : 0), 3);
      if (dyn) {
        const uint32_t* btab = stab + L_CODES + D_CODES;
        bw.put(B.lcodes - 257, 5);
        bw.put(B.dcodes - 1, 5);
        bw.put(B.blcodes - 4, 4);
        for (uint32_t rk = 0; rk < B.blcodes; rk++) bw.put(btab[BL_ORDER[rk]] >> 16, 3);
        send_tree(bw, stab, B.lcodes - 1, btab);
        send_tree(bw, stab + L_CODES, B.dcodes - 1, btab);
      }
      pos = bw.pos;
    }
    pos = readlane64(pos, 0);
    __syncthreads();
    ZD_ADD(8, tz);
    const uint64_t wfirst = B.bit_off >> 5;
    uint64_t flushed = wfirst;
    auto flush = [&](uint64_t upto) {   // words [flushed, upto) are complete
      for (uint64_t w = flushed + lane; w < upto; w += 64) {
        const uint32_t v = ring[w % RING];
        ring[w % RING] = 0;
        if (w == wfirst) or_word(o, w, v);
        else if (w < o.nwords) o.o[w] = v;
      }
      flushed = upto;
    };
    const uint32_t* sym = a.sym + c.t_off;
    const uint32_t sb = B.sym_begin, se = B.sym_end;
    uint32_t cur[EBATCH], nxt[EBATCH];
#pragma unroll
    for (int q = 0; q < EBATCH; q++) {
      const uint32_t i = sb + 64 * q + lane;
      cur[q] = i < se ? sym[i] : 0xffffffffu;
    }
    for (uint32_t b0 = sb; b0 < se; b0 += 64 * EBATCH) {
#pragma unroll
      for (int q = 0; q < EBATCH; q++) {
        const uint32_t i = b0 + 64 * (EBATCH + q) + lane;
        nxt[q] = i < se ? sym[i] : 0xffffffffu;
      }
#pragma unroll
      for (int q = 0; q < EBATCH; q++) {
        if (b0 + 64 * q >= se) break;
        const uint32_t e = cur[q];
        uint64_t v = 0;
        uint32_t nb = 0;
        if (e != 0xffffffffu) {
          const uint32_t dist = e >> 8;
          if (dist == 0) {
            const uint32_t t = litx[e & 255];
            v = t & 0xffffff;
            nb = t >> 24;
          } else {
            const uint32_t t = lenx[e & 255];
            const uint32_t d = dist - 1;
            const int dc = dist_code(d);
            const uint32_t td = dtx[dc], hd = td >> 16;
            const uint32_t xd = d < 4 ? 0u : (uint32_t)(31 - __clz(d)) - 1u;   // XDB[dc]
            const uint32_t v1 = (td & 0xffff) | ((d & ((1u << xd) - 1u)) << hd);
            const uint32_t n0 = t >> 24;
            v = (uint64_t)(t & 0xffffff) | ((uint64_t)v1 << n0);
            nb = n0 + hd + xd;
          }
        }
        const uint32_t incl = wave_incl_scan(nb);
        if (nb) {
          const uint64_t P = pos + incl - nb;
          const uint64_t w = P >> 5;
          const uint32_t sh = (uint32_t)(P & 31);
          const uint64_t lo = v << sh;
          if ((uint32_t)lo) atomicOr(&ring[w % RING], (uint32_t)lo);
          if (lo >> 32) atomicOr(&ring[(w + 1) % RING], (uint32_t)(lo >> 32));
          if (sh && (v >> (64 - sh))) atomicOr(&ring[(w + 2) % RING], (uint32_t)(v >> (64 - sh)));
        }
        pos += readlane(incl, 63);
        flush(pos >> 5);
      }
#pragma unroll
      for (int q = 0; q < EBATCH; q++) cur[q] = nxt[q];
    }
    ZD_ADD(9, tz);
    if (lane == 0) {
      RingW bw{ring, pos};
      bw.put(eob & 0xffff, eob >> 16);
      pos = bw.pos;
    }
    pos = readlane64(pos, 0);
    // the last (partial) word is shared with the next block
    const uint64_t wend = (pos + 31) >> 5;
    for (uint64_t w = flushed + lane; w < wend; w += 64) {
      const uint32_t v = ring[w % RING];
      if (w == wfirst || w == wend - 1) or_word(o, w, v);
      else if (w < o.nwords) o.o[w] = v;
    }
    ZD_ADD(10, tz);
  }
#ifdef XCG_ZD_TIMING
  if (lane == 0) atomicAdd(&g_zd_t[15], 1ull);
#endif
  if (k == r.nblocks - 1 && lane == 0 && !r.stop) {
    if (last) {   // Z_FINISH: adler32 trailer, big-endian (putShortMSB x2)
      uint64_t b = r.end_bit >> 3;
      uint32_t ad = s.adler;
      or_byte(ob, b, ad >> 24);
      or_byte(ob, b + 1, (ad >> 16) & 0xff);
      or_byte(ob, b + 2, (ad >> 8) & 0xff);
      or_byte(ob, b + 3, ad & 0xff);
    } else {      // Z_SYNC_FLUSH: empty stored block, 000 + align + 00 00 FF FF
      uint64_t b = (r.end_bit + 3 + 7) >> 3;
      or_byte(ob, b + 2, 0xff);
      or_byte(ob, b + 3, 0xff);
    }
  }
}

// ------------------------------------------------------------------- commit
// Stream state after the call: history = the last 32 KiB of X, position,
// window base, adler, flags.  Grid: (8 tiles, calls).
__global__ __launch_bounds__(256) void zd_commit_kernel(ZArgs a) {
  const uint32_t ci = blockIdx.y;
  const ZCall c = a.calls[ci];
  const uint8_t* X = a.X + c.x_off + c.len;   // X[len .. len + WSIZE) = the last WSIZE positions
  uint8_t* h = a.hist + (uint64_t)c.stream * WSIZE;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < (uint32_t)WSIZE / 4; i += gridDim.x * 256) {
    const uint8_t* q = X + 4 * i;
    *(uint32_t*)(h + 4 * i) = q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ZState s = a.st[c.stream];
    const ZCallRes& r = a.res[ci];
    const int64_t x2s = (int64_t)s.total - WSIZE;   // X index -> stream position
    if (r.stop) {   // resume right after the block the flush call stopped at
      const ZBlock& B = a.blk[c.blk_off + r.stop - 1];
      s.base = (uint64_t)(x2s + B.bidx);
      s.dlen = (uint32_t)((int64_t)WSIZE + c.len - (int64_t)B.p_after);
      s.block_start = (uint64_t)(x2s + (int64_t)B.start + B.stored_len);
      s.mstart = (uint64_t)(x2s + (int64_t)B.ms);
      s.avail = B.avail;
      s.mlen = B.ml;
      const uint64_t e = r.end_bit;
      s.cnb = (uint32_t)(e & 7);
      s.cbits = s.cnb ? a.out[c.out_off + (e >> 3)] & ((1u << s.cnb) - 1u) : 0u;
    } else {
      s.base = r.base_end;
      s.dlen = 0;
      s.block_start = (uint64_t)((int64_t)s.total + c.len);
      s.avail = 0;
      s.mlen = MIN_MATCH - 1;
      s.cnb = 0;
      s.cbits = 0;
    }
    s.pend = s.pend + r.out_bytes - r.deliver;
    s.total += c.len;
    s.adler = c.len ? r.adler : s.adler;
    s.flags |= 1u;
    if (c.len == 0) s.flags |= 2u;
    a.st[c.stream] = s;
  }
}

// ------------------------------------------------------------------- level 0
// deflate_stored (deflate.c, zlib 1.2.11) writes no Huffman codes: a stream
// is stored blocks (5 header bytes + raw bytes) whose sizes follow zlib's
// control flow over avail_in (the Buffer's segments, <= 2048 bytes each) and
// avail_out (DeflatePipe's 64 KiB buffer, deflate_pipe.cc:57-115): it copies
// blocks straight to next_out while they are >= 32 KiB (or flush everything),
// and otherwise collects input in its 64 KiB window and emits from there.
// The host replays that control flow over lengths only (StoredPlan) and the
// GPU moves the bytes (zs_copy_kernel): every piece of a call's output is a
// header, a range of the stream (this call's input, or earlier bytes from the
// stream's 64 KiB ring) or the adler32 trailer.
__global__ __launch_bounds__(256) void zs_copy_kernel(const ZPiece* pc, const ZCall* calls, const ZState* st,
                                                      const uint8_t* in, const uint8_t* ring, uint8_t* out) {
  const ZPiece p = pc[blockIdx.x];
  const ZCall c = calls[p.call];
  uint8_t* o = out + c.out_off + p.out;
  if (p.kind == 0) {
    if (threadIdx.x < p.len) o[threadIdx.x] = (uint8_t)(p.src >> (8 * threadIdx.x));
    return;
  }
  if (p.kind == 2) {
    const uint32_t ad = st[c.stream].adler;
    if (threadIdx.x < 4) o[threadIdx.x] = (uint8_t)(ad >> (24 - 8 * threadIdx.x));
    return;
  }
  const uint64_t total = st[c.stream].total;           // stream position of this call's first byte
  const uint8_t* r = ring + (uint64_t)c.stream * (2 * WSIZE);
  for (uint32_t i = threadIdx.x; i < p.len; i += 256) {
    const uint64_t q = p.src + i;
    o[i] = q >= total ? in[c.in_off + (q - total)] : r[q & (2 * WSIZE - 1)];
  }
}

// The stream's last 64 KiB (ring by position) after the call; adler, position.
__global__ __launch_bounds__(256) void zs_commit_kernel(ZArgs a) {
  const ZCall c = a.calls[blockIdx.x];
  const ZState s0 = a.st[c.stream];
  uint8_t* r = a.hist + (uint64_t)c.stream * (2 * WSIZE);
  const uint32_t keep = c.len < 2u * WSIZE ? c.len : 2u * WSIZE;
  for (uint32_t i = threadIdx.x; i < keep; i += 256) {
    const uint64_t q = s0.total + c.len - keep + i;
    r[q & (2 * WSIZE - 1)] = a.in[c.in_off + (c.len - keep + i)];
  }
  if (threadIdx.x == 0) {
    ZState s = s0;
    s.total += c.len;
    s.adler = c.len ? a.res[blockIdx.x].adler : s.adler;
    s.flags |= 1u;
    if (c.len == 0) s.flags |= 2u;
    a.st[c.stream] = s;
  }
}


}  // namespace zd
}  // namespace xcg

using namespace xcg::zd;

struct xcg_zdeflate {
  int device = 0, level = 6;
  uint32_t nstreams = 0;
  ZState* st = nullptr;
  uint8_t* hist = nullptr;
  std::vector<ZState> h_init;
  // scratch (grow-only)
  uint8_t* scratch = nullptr;
  size_t scratch_cap = 0;
  void* meta = nullptr;       // ZCall[] + tile maps + block maps (device)
  size_t meta_cap = 0;
  void* h_meta = nullptr;     // pinned staging for meta
  size_t h_meta_cap = 0;
  hipEvent_t done = nullptr;
  uint32_t* ring = nullptr;   // deflate_fast: per stream, the hashed positions of the last 32 KiB
  uint32_t* h_changed = nullptr;   // pinned, per call (deflate_fast rounds)
  size_t h_changed_cap = 0;
  uint32_t last_rounds = 0;
  std::vector<StoredPlan> splan;   // level 0: zlib's control state per stream (host, lengths only)
  // host-buffer calls (xcg_zdeflate_host: the drop-in DeflatePipe::consume):
  // kept staging and a private stream, one synchronisation per call
  hipStream_t hst = nullptr;
  uint8_t* hs_h = nullptr;         // pinned
  uint8_t* hs_d = nullptr;
  size_t hs_hcap = 0, hs_dcap = 0;
};

namespace {
int grow(void** p, size_t* cap, size_t want, bool pinned) {
  if (*cap >= want) return XCG_OK;
  size_t n = std::max(want, *cap * 3 / 2);
  if (*p) {
    if (pinned) (void)hipHostFree(*p);
    else (void)hipFree(*p);
    *p = nullptr;
  }
  hipError_t e = pinned ? hipHostMalloc(p, n) : hipMalloc(p, n);
  if (e != hipSuccess) {
    *cap = 0;
    *p = nullptr;
    return XCG_ENOMEM;
  }
  *cap = n;
  return XCG_OK;
}
inline size_t al(size_t v, size_t a) { return (v + a - 1) / a * a; }
ZState fresh_state() {   // deflateInit
  ZState s;
  memset(&s, 0, sizeof s);
  s.adler = 1u;
  s.mlen = MIN_MATCH - 1;
  return s;
}
}  // namespace

extern "C" {

uint64_t xcg_zdeflate_bound(uint32_t len) { return (uint64_t)len + (len >> 1) + 2 * DMAX + 128; }

int xcg_zdeflate_create(int device, int level, uint32_t nstreams, xcg_zdeflate** out) {
  if (!out || level < 0 || level > 9 || nstreams == 0) return XCG_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return XCG_EHIP;
  xcg_zdeflate* z = new xcg_zdeflate();
  z->device = device;
  z->level = level;
  z->nstreams = nstreams;
  if (hipMalloc(&z->st, sizeof(ZState) * nstreams) != hipSuccess ||
      hipMalloc(&z->hist, (size_t)WSIZE * (level == 0 ? 2 : 1) * nstreams) != hipSuccess ||
      hipEventCreateWithFlags(&z->done, hipEventDisableTiming) != hipSuccess ||
      (level < 4 && (hipMalloc(&z->ring, (size_t)WSIZE / 8 * nstreams) != hipSuccess ||
                     hipMemset(z->ring, 0, (size_t)WSIZE / 8 * nstreams) != hipSuccess))) {
    delete z;
    return XCG_ENOMEM;
  }
  z->h_init.assign(nstreams, fresh_state());
  if (level == 0) z->splan.assign(nstreams, StoredPlan());
  if (hipMemcpy(z->st, z->h_init.data(), sizeof(ZState) * nstreams, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(z->hist, 0, (size_t)WSIZE * nstreams) != hipSuccess) {
    delete z;
    return XCG_EHIP;
  }
  *out = z;
  return XCG_OK;
}

void xcg_zdeflate_destroy(xcg_zdeflate* z) {
  if (!z) return;
  (void)hipSetDevice(z->device);
  if (z->done) (void)hipEventSynchronize(z->done);
  (void)hipFree(z->st);
  (void)hipFree(z->hist);
  (void)hipFree(z->ring);
  if (z->h_changed) (void)hipHostFree(z->h_changed);
  if (z->hs_h) (void)hipHostFree(z->hs_h);
  (void)hipFree(z->hs_d);
  if (z->hst) (void)hipStreamDestroy(z->hst);
  (void)hipFree(z->scratch);
  (void)hipFree(z->meta);
  if (z->h_meta) (void)hipHostFree(z->h_meta);
  if (z->done) (void)hipEventDestroy(z->done);
  delete z;
}

int xcg_zdeflate_reset(xcg_zdeflate* z, uint32_t stream) {
  if (!z || stream >= z->nstreams) return XCG_EINVAL;
  (void)hipSetDevice(z->device);
  if (hipEventSynchronize(z->done) != hipSuccess) return XCG_EHIP;
  const ZState s0 = fresh_state();
  if (hipMemcpy(z->st + stream, &s0, sizeof s0, hipMemcpyHostToDevice) != hipSuccess) return XCG_EHIP;
  if (z->ring && hipMemset(z->ring + (size_t)stream * (WSIZE / 32), 0, WSIZE / 8) != hipSuccess) return XCG_EHIP;
  if (!z->splan.empty()) z->splan[stream] = StoredPlan();
  return XCG_OK;
}

}  // extern "C"

namespace {
// Level 0: the host replays zlib's control flow per consume (StoredPlan), the
// GPU computes adler32, moves the pieces and keeps each stream's last 64 KiB.
int stored_batch(xcg_zdeflate* z, const uint8_t* d_in, const uint64_t* h_in_off, const uint32_t* h_len,
                 const uint32_t* h_stream, uint32_t n, const uint32_t* h_seg, const uint32_t* h_nseg, uint8_t* d_out,
                 const uint64_t* h_out_off, uint32_t* d_out_len, uint64_t* d_deliver, hipStream_t st) {
  std::vector<ZCall> calls(n);
  std::vector<ZPiece> pieces;
  std::vector<uint32_t> made32(n);
  std::vector<uint64_t> deliver(n);
  std::vector<uint8_t> seen(z->nstreams, 0);
  uint64_t so = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (h_stream[i] >= z->nstreams || seen[h_stream[i]] || (h_out_off[i] & 3) || h_len[i] > (1u << 24))
      return XCG_EINVAL;
    seen[h_stream[i]] = 1;
  }
  // the plan mutates the streams' host state: check everything first, then plan
  for (uint32_t i = 0; i < n; i++) {
    ZCall& c = calls[i];
    memset(&c, 0, sizeof c);
    c.in_off = h_in_off[i];
    c.out_off = h_out_off[i];
    c.len = h_len[i];
    c.stream = h_stream[i];
    const size_t first = pieces.size();
    uint64_t made = 0;
    const uint32_t ns = h_nseg ? h_nseg[i] : 0;
    if (!z->splan[c.stream].consume(c.len, h_seg ? h_seg + so : nullptr, ns, pieces, &made, &deliver[i]))
      return XCG_EINVAL;
    so += ns;
    if (made > xcg_zdeflate_bound(c.len)) return XCG_EOVERFLOW;
    made32[i] = (uint32_t)made;
    for (size_t k = first; k < pieces.size(); k++) pieces[k].call = i;
  }
  size_t m_calls = 0, m_pc = al(sizeof(ZCall) * n, 256), m_len = al(m_pc + sizeof(ZPiece) * pieces.size(), 256),
         m_dl = al(m_len + 4ull * n, 256), m_end = al(m_dl + 8ull * n, 256);
  if (hipEventSynchronize(z->done) != hipSuccess) return XCG_EHIP;
  const size_t r_res = sizeof(ZCallRes) * n;
  if (grow((void**)&z->scratch, &z->scratch_cap, al(r_res, 256), false)) return XCG_ENOMEM;
  if (grow(&z->meta, &z->meta_cap, m_end, false) || grow(&z->h_meta, &z->h_meta_cap, m_end, true)) return XCG_ENOMEM;
  uint8_t* hm = (uint8_t*)z->h_meta;
  memcpy(hm + m_calls, calls.data(), sizeof(ZCall) * n);
  if (!pieces.empty()) memcpy(hm + m_pc, pieces.data(), sizeof(ZPiece) * pieces.size());
  memcpy(hm + m_len, made32.data(), 4ull * n);
  memcpy(hm + m_dl, deliver.data(), 8ull * n);
  if (hipMemcpyAsync(z->meta, hm, m_end, hipMemcpyHostToDevice, st) != hipSuccess) return XCG_EHIP;
  uint8_t* dm = (uint8_t*)z->meta;
  if (hipMemcpyAsync(d_out_len, dm + m_len, 4ull * n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipMemcpyAsync(d_deliver, dm + m_dl, 8ull * n, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return XCG_EHIP;
  ZArgs a;
  memset(&a, 0, sizeof a);
  a.calls = (const ZCall*)(dm + m_calls);
  a.st = z->st;
  a.hist = z->hist;
  a.in = d_in;
  a.out = d_out;
  a.res = (ZCallRes*)z->scratch;
  a.n = n;
  a.level = 0;
  hipLaunchKernelGGL(zd_adler_kernel, dim3(n), dim3(256), 0, st, a);
  if (!pieces.empty())
    hipLaunchKernelGGL(zs_copy_kernel, dim3((unsigned)pieces.size()), dim3(256), 0, st, (const ZPiece*)(dm + m_pc),
                       a.calls, (const ZState*)z->st, d_in, (const uint8_t*)z->hist, d_out);
  hipLaunchKernelGGL(zs_commit_kernel, dim3(n), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return XCG_EHIP;
  if (hipEventRecord(z->done, st) != hipSuccess) return XCG_EHIP;
  return XCG_OK;
}
}  // namespace

extern "C" {

int xcg_zdeflate_batch_seg(xcg_zdeflate* z, const uint8_t* d_in, const uint64_t* h_in_off, const uint32_t* h_len,
                           const uint32_t* h_stream, uint32_t n, const uint32_t* h_seg, const uint32_t* h_nseg,
                           uint8_t* d_out, const uint64_t* h_out_off, uint32_t* d_out_len, uint64_t* d_deliver,
                           void* stream) {
  if (!z || n == 0 || !h_in_off || !h_len || !h_stream || !h_out_off || !d_out || !d_out_len || !d_deliver ||
      (h_seg && !h_nseg))
    return XCG_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  (void)hipSetDevice(z->device);
  if (z->level == 0)
    return stored_batch(z, d_in, h_in_off, h_len, h_stream, n, h_seg, h_nseg, d_out, h_out_off, d_out_len, d_deliver,
                        st);
  // host plan: scratch offsets, tiles, block maps
  std::vector<ZCall> calls(n);
  std::vector<uint32_t> mstart(n + 1), gstart(n + 1), bstart(n + 1);
  std::vector<uint8_t> seen(z->nstreams, 0);
  size_t xo = 0, to = 0, mo = 0;
  uint32_t bo = 0;
  const bool fast = z->level < 4;
  for (uint32_t i = 0; i < n; i++) {
    if (h_stream[i] >= z->nstreams || seen[h_stream[i]] || (h_out_off[i] & 3) || h_len[i] > (1u << 24))
      return XCG_EINVAL;
    seen[h_stream[i]] = 1;
    ZCall& c = calls[i];
    c.in_off = h_in_off[i];
    c.out_off = h_out_off[i];
    c.len = h_len[i];
    c.stream = h_stream[i];
    c.x_off = xo;
    xo += al((size_t)WSIZE + c.len + XPAD, 256);
    c.m_off = mo;                                 // (deflate_fast masks: one bit per X index)
    mo += fast ? al(((size_t)WSIZE + c.len + 64) / 32 + 1, 64) : 0;
    c.t_off = to;                                 // (parsed positions: up to DMAX left by the last call)
    to += al((size_t)c.len + DMAX + 1, 64);
    c.blk_off = bo;
    c.blk_cap = (c.len + DMAX) / SYMS_PER_BLOCK + 2;
    bstart[i] = bo;
    bo += c.blk_cap;
    mstart[i + 1] = mstart[i] + (c.len + DMAX + 255) / 256;
    gstart[i + 1] = gstart[i] + ((uint32_t)WSIZE + c.len + 63) / 64 + 1;
  }
  bstart[n] = bo;
  const uint32_t mtiles = mstart[n], groups = gstart[n];
  // scratch layout
  size_t o_X = 0, o_d16 = al(o_X + xo, 256), o_pk = al(o_d16 + 2 * xo, 256), o_tf = al(o_pk + 4 * xo, 256),
         o_tq = al(o_tf + 4 * to, 256),
         o_sym = al(o_tq + 4 * to, 256), o_blk = al(o_sym + 4 * to, 256),
         o_tab = al(o_blk + sizeof(ZBlock) * bo, 256), o_res = al(o_tab + 4ull * TAB_WORDS * bo, 256),
         o_ma = al(o_res + sizeof(ZCallRes) * n, 256), o_mb = al(o_ma + 4 * mo, 256), o_chg = al(o_mb + 4 * mo, 256),
         o_end = al(o_chg + 4ull * n, 256);
  // the previous batch may still read the scratch
  if (hipEventSynchronize(z->done) != hipSuccess) return XCG_EHIP;
  if (grow((void**)&z->scratch, &z->scratch_cap, o_end, false)) return XCG_ENOMEM;
  size_t m_calls = 0, m_ms = al(sizeof(ZCall) * n, 256), m_gs = al(m_ms + 4ull * (n + 1), 256),
         m_bs = al(m_gs + 4ull * (n + 1), 256), m_end = al(m_bs + 4ull * (n + 1), 256);
  if (grow(&z->meta, &z->meta_cap, m_end, false) || grow(&z->h_meta, &z->h_meta_cap, m_end, true)) return XCG_ENOMEM;
  uint8_t* hm = (uint8_t*)z->h_meta;
  memcpy(hm + m_calls, calls.data(), sizeof(ZCall) * n);
  memcpy(hm + m_ms, mstart.data(), 4ull * (n + 1));
  memcpy(hm + m_gs, gstart.data(), 4ull * (n + 1));
  memcpy(hm + m_bs, bstart.data(), 4ull * (n + 1));
  if (hipMemcpyAsync(z->meta, hm, m_end, hipMemcpyHostToDevice, st) != hipSuccess) return XCG_EHIP;
  uint8_t* dm = (uint8_t*)z->meta;
  ZArgs a;
  a.calls = (const ZCall*)(dm + m_calls);
  a.st = z->st;
  a.hist = z->hist;
  a.in = d_in;
  a.out = d_out;
  a.X = z->scratch + o_X;
  a.d16 = (uint16_t*)(z->scratch + o_d16);
  a.pk = (uint32_t*)(z->scratch + o_pk);
  a.tf = (uint32_t*)(z->scratch + o_tf);
  a.tq = (uint32_t*)(z->scratch + o_tq);
  a.sym = (uint32_t*)(z->scratch + o_sym);
  a.blk = (ZBlock*)(z->scratch + o_blk);
  a.tabs = (uint32_t*)(z->scratch + o_tab);
  a.res = (ZCallRes*)(z->scratch + o_res);
  a.out_len = d_out_len;
  a.deliver = d_deliver;
  a.n = n;
  a.mstart = (const uint32_t*)(dm + m_ms);
  a.gstart = (const uint32_t*)(dm + m_gs);
  a.bstart = (const uint32_t*)(dm + m_bs);
  a.level = z->level;
  a.fast = fast ? 1 : 0;
  uint32_t* mA = (uint32_t*)(z->scratch + o_ma);
  uint32_t* mB = (uint32_t*)(z->scratch + o_mb);
  a.mcur = mA;
  a.mnext = mB;
  a.ring = z->ring;
  a.changed = (uint32_t*)(z->scratch + o_chg);
  uint32_t maxlen = 0;
  for (uint32_t i = 0; i < n; i++) maxlen = std::max(maxlen, h_len[i]);
  uint32_t prep_tiles = std::min<uint32_t>(64, ((uint32_t)WSIZE + maxlen + XPAD + 4095) / 4096);
  hipLaunchKernelGGL(zd_prep_kernel, dim3(prep_tiles, n), dim3(256), 0, st, a);
  hipLaunchKernelGGL(zd_adler_kernel, dim3(n), dim3(256), 0, st, a);
  const unsigned hgrid = (groups + 4 * HGROUPS - 1) / (4 * HGROUPS);
  if (!fast) {
    hipLaunchKernelGGL(zd_hashes_kernel, dim3(hgrid), dim3(256), 0, st, a, n, a.gstart);
    hipLaunchKernelGGL(zd_chain_kernel, dim3(n), dim3(64), 0, st, a);
    if (mtiles) hipLaunchKernelGGL(zd_match_kernel, dim3(mtiles), dim3(256), 0, st, a);
    hipLaunchKernelGGL(zd_scan_kernel, dim3(n), dim3(64), 0, st, a);
  } else {
    // deflate_fast: which positions zlib hashes depends on its own parse.  Guess
    // (round 0: all), build the chains and the match table from the guess, parse,
    // and repeat with the parse's hashed positions until they reproduce the guess
    // (the correct prefix grows every round, so this ends).
    if (grow((void**)&z->h_changed, &z->h_changed_cap, 4ull * n, true)) return XCG_ENOMEM;
    const unsigned mgrid = (unsigned)std::min<size_t>(4096, (mo + 255) / 256 + 1);
    hipLaunchKernelGGL(zd_mfill_kernel, dim3(mgrid), dim3(256), 0, st, mA, mB, (uint64_t)mo);
    uint32_t rounds = 0;
    for (;;) {
      rounds++;
      if (hipMemsetAsync(a.changed, 0, 4ull * n, st) != hipSuccess) return XCG_EHIP;
      hipLaunchKernelGGL(zd_hashes_kernel, dim3(hgrid), dim3(256), 0, st, a, n, a.gstart);
      hipLaunchKernelGGL(zd_chain_kernel, dim3(n), dim3(64), 0, st, a);
      if (mtiles) hipLaunchKernelGGL(zd_match_kernel, dim3(mtiles), dim3(256), 0, st, a);
      hipLaunchKernelGGL(zd_fscan_kernel, dim3(n), dim3(64), 0, st, a);
      hipLaunchKernelGGL(zd_mcmp_kernel, dim3(n), dim3(256), 0, st, a);
      if (hipMemcpyAsync(z->h_changed, a.changed, 4ull * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return XCG_EHIP;
      bool any = false;
      for (uint32_t i = 0; i < n && !any; i++) any = z->h_changed[i] != 0;
      std::swap(a.mcur, a.mnext);   // the parse's positions are the next guess (and, when equal, final)
      if (!any) break;
      if (rounds > 100000) return XCG_EOVERFLOW;
      hipLaunchKernelGGL(zd_mzero_kernel, dim3(mgrid), dim3(256), 0, st, a.mnext,
                         (uint64_t)mo);
    }
    z->last_rounds = rounds;
  }
  // few blocks (one consume at a time): a wave per block, whose heap chains
  // then run without a second lane's diverging beside them; many: two per wave
  if (bo <= 64) hipLaunchKernelGGL(zd_trees_kernel<1>, dim3(bo), dim3(64), 0, st, a);
  else hipLaunchKernelGGL(zd_trees_kernel<TB_BATCH>, dim3((bo + TB_BATCH - 1) / TB_BATCH), dim3(64), 0, st, a);
  hipLaunchKernelGGL(zd_layout_kernel, dim3(n), dim3(64), 0, st, a);
  hipLaunchKernelGGL(zd_emit_kernel, dim3(bo), dim3(64), 0, st, a);
  if (fast) hipLaunchKernelGGL(zd_ring_kernel, dim3(n), dim3(256), 0, st, a);   // (before commit moves the state)
  hipLaunchKernelGGL(zd_commit_kernel, dim3(8, n), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return XCG_EHIP;
  if (hipEventRecord(z->done, st) != hipSuccess) return XCG_EHIP;
  return XCG_OK;
}

int xcg_zdeflate_batch(xcg_zdeflate* z, const uint8_t* d_in, const uint64_t* h_in_off, const uint32_t* h_len,
                       const uint32_t* h_stream, uint32_t n, uint8_t* d_out, const uint64_t* h_out_off,
                       uint32_t* d_out_len, uint64_t* d_deliver, void* stream) {
  return xcg_zdeflate_batch_seg(z, d_in, h_in_off, h_len, h_stream, n, nullptr, nullptr, d_out, h_out_off, d_out_len,
                                d_deliver, stream);
}

// Host buffers: one consume() per listed stream, inputs concatenated in h_in
// at h_in_off, outputs to h_out at h_out_off (room for xcg_zdeflate_bound);
// lengths to h_out_len.  Synchronous.
int xcg_zdeflate_host(xcg_zdeflate* z, const uint8_t* h_in, const uint64_t* h_in_off, const uint32_t* h_len,
                      const uint32_t* h_stream, uint32_t n, const uint32_t* h_seg, const uint32_t* h_nseg,
                      uint8_t* h_out, const uint64_t* h_out_off, uint32_t* h_out_len, uint64_t* h_deliver) {
  if (!z || n == 0 || !h_deliver || !h_out_len || !h_in_off || !h_len) return XCG_EINVAL;
  (void)hipSetDevice(z->device);
  if (!z->hst && hipStreamCreateWithFlags(&z->hst, hipStreamNonBlocking) != hipSuccess) return XCG_EHIP;
  uint64_t in_end = 0, out_end = 0;
  std::vector<uint64_t> doff(n);
  for (uint32_t i = 0; i < n; i++) {
    in_end = std::max(in_end, h_in_off[i] + h_len[i]);
    doff[i] = out_end;
    out_end += al(xcg_zdeflate_bound(h_len[i]), 4);
  }
  // staging: [in][out][out_len n][deliver n]
  const size_t o_out = al(in_end + 1, 256), o_len = al(o_out + out_end, 256), o_dl = al(o_len + 4ull * n, 256),
               o_end = al(o_dl + 8ull * n, 256);
  if (grow((void**)&z->hs_h, &z->hs_hcap, o_end, true) || grow((void**)&z->hs_d, &z->hs_dcap, o_end, false))
    return XCG_ENOMEM;
  if (in_end) memcpy(z->hs_h, h_in, in_end);
  if (in_end && hipMemcpyAsync(z->hs_d, z->hs_h, in_end, hipMemcpyHostToDevice, z->hst) != hipSuccess) return XCG_EHIP;
  int rc = xcg_zdeflate_batch_seg(z, z->hs_d, h_in_off, h_len, h_stream, n, h_seg, h_nseg, z->hs_d + o_out,
                                  doff.data(), (uint32_t*)(z->hs_d + o_len), (uint64_t*)(z->hs_d + o_dl), z->hst);
  if (rc != XCG_OK) return rc;
  // the outputs' room (<= 1.5x the input) comes back with the lengths: one synchronisation
  if (hipMemcpyAsync(z->hs_h + o_out, z->hs_d + o_out, o_end - o_out, hipMemcpyDeviceToHost, z->hst) != hipSuccess ||
      hipStreamSynchronize(z->hst) != hipSuccess)
    return XCG_EHIP;
  memcpy(h_out_len, z->hs_h + o_len, 4ull * n);
  memcpy(h_deliver, z->hs_h + o_dl, 8ull * n);
  for (uint32_t i = 0; i < n; i++) memcpy(h_out + h_out_off[i], z->hs_h + o_out + doff[i], h_out_len[i]);
  return XCG_OK;
}

uint32_t xcg_debug_zdeflate_rounds(const xcg_zdeflate* z) { return z ? z->last_rounds : 0; }

#ifdef XCG_ZD_TIMING
int xcg_debug_zd_times(uint64_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zd_t), 8 * 16) != hipSuccess) return XCG_EHIP;
  uint64_t z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_zd_t), z, sizeof z) == hipSuccess ? XCG_OK : XCG_EHIP;
}
#endif

}  // extern "C"
