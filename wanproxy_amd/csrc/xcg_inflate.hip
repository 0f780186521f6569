// wanproxy's zlib stage, receiving side: InflatePipe (zlib/inflate_pipe.cc:
// 54-139) for many streams at once.  Each consume() gets an arbitrary cut of
// the peer's zlib stream (the network splits it anywhere) and produces every
// byte the input so far lets inflate() produce.  gfx950, wave64.
//
// One wave per call; the decoder's control state is wave-uniform (every lane
// runs it, values come from readlane), lanes split the byte copies.  The last
// 8 KiB of output live in an LDS ring: a match up to 4 KiB back copies LDS ->
// LDS (the modular source index handles overlapping copies); a farther one
// reads HBM -- this call's output, flushed to the caller's buffer every 2 KiB
// (a fence after each flush makes it readable), or the stream's 32 KiB history.
// ~16 KiB of LDS per stream: ten streams per CU, where a 32 KiB window ring
// allowed four, and the serial decode is latency-bound per stream.  Input bits come from a 256-byte register window.  Huffman
// decoding: a 512-entry primary table per tree in LDS, longer codes by
// canonical decoding; the decoder's wave-uniform control runs on the SALU.  Every field is read under a bounds check; when the
// input ends inside a symbol or a block header, the call stops at the symbol /
// header start and carries the unread bytes (at most a dynamic block header)
// into the next call.  The adler32 trailer is checked (inflate()'s
// Z_DATA_ERROR on a mismatch).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/xcgpu.h"
#include "xcg_device.h"

namespace xcg {
namespace zi {

constexpr int WSIZE = 32768;
constexpr uint32_t RMASK = 4095;    // LDS ring of the last 4 KiB of output
constexpr uint32_t NEAR = 2048;     // matches up to this distance copy inside the ring
constexpr uint32_t FLUSH_AT = 1024; // output is flushed to HBM every 1 KiB
constexpr int PEND_CAP = 1024;
constexpr int PRI = 9;              // primary table bits
constexpr int IPAD = 512;           // zero bytes after a call's input in the scratch

enum Mode : uint32_t { M_HEADER = 0, M_BLOCK = 1, M_STORED = 2, M_HUFF = 3, M_TRAILER = 4, M_DONE = 5, M_ERROR = 6 };

__constant__ uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                   1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t CL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct IState {             // one InflatePipe's z_stream
  uint64_t total_out;       // bytes produced so far
  uint32_t mode, last, stored_left, btype;
  uint32_t nlen, ndist;     // dynamic block: code counts (lengths in `lens`)
  uint32_t npend, pend_bit; // carried input bytes, first unread bit in them
  uint32_t adler;           // adler32 of the output so far
  uint32_t pad;
  uint8_t lens[320];
  uint8_t pend[PEND_CAP];
};

struct ICall {
  uint64_t in_off, out_off;
  uint64_t i_off;           // scratch: carried + new input
  uint32_t len, stream, out_cap, pad;
};

struct IRes {
  uint32_t out_len;
  int32_t status;           // 0 ok, 1 stream end reached, -1 data error, -2 output capacity exceeded
  uint32_t trailer;         // the stream's adler32 trailer (when it was read in this call)
  uint32_t have_trailer;
};

struct IArgs {
  const ICall* calls;
  IState* st;
  uint8_t* hist;            // nstreams x WSIZE: the last 32 KiB of output
  const uint8_t* in;
  uint8_t* out;
  uint8_t* I;
  IRes* res;
  uint32_t* out_len;
  int32_t* status;
};

// carried bytes ++ new input into the scratch, 16 bytes per thread (the
// scratch slot is 256-byte aligned; vectors straddling the carried / new /
// pad boundaries are assembled bytewise).  Grid: (tiles, calls).
__global__ __launch_bounds__(256) void zi_prep_kernel(IArgs a) {
  const ICall c = a.calls[blockIdx.y];
  const IState* s = a.st + c.stream;
  const uint64_t np = s->npend, dend = np + c.len;
  uint8_t* I = a.I + c.i_off;
  const uint8_t* d = a.in + c.in_off;
  const uint64_t nv = (dend + IPAD + 15) / 16;
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * 256) {
    const uint64_t q = 16 * v;
    u32x4 r = {0u, 0u, 0u, 0u};
    if (q >= np && q + 16 <= dend) {
      r = *(const u32x4_u*)(d + (q - np));
    } else if (q < dend) {
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      for (uint64_t k = 0; k < 16 && q + k < dend; k++) {
        const uint64_t x = q + k;
        w[k >> 2] |= (uint32_t)(x < np ? s->pend[x] : d[x - np]) << (8 * (k & 3));
      }
      r = u32x4{w[0], w[1], w[2], w[3]};
    }
    *(u32x4*)(I + q) = r;
  }
}

template <int B, int NS>
struct TreeT {
  static constexpr int BITS = B;
  uint16_t pri[1 << B];     // (sym << 4) | len; 0: a code longer than B bits
  uint16_t cnt[16];
  uint16_t sym[NS];         // symbols in canonical order (by length, then value)
};
// literal/length codes of skewed blocks run to 10-12 bits: a 10-bit primary
// table keeps most of them off the canonical path while a stream's LDS stays at
// ~9.5 KiB (16 streams per CU, all 4096 of a batch resident at once)
typedef TreeT<10, 288> LTree;
typedef TreeT<PRI, 32> DTree;
typedef TreeT<7, 20> CTree;

struct Lds {
  uint8_t ring[RMASK + 1];
  LTree lt;
  DTree dt;
  CTree ct;                 // literal/length, distance, code-length trees
  uint8_t lens[320];        // fixed / code-length tree lengths
  uint8_t dlens[320];       // the dynamic block's literal/length + distance lengths
  uint16_t codes[320];
  int ok;
};

// Canonical decoder from code lengths (inflate_table's rules: over-subscribed
// sets are errors, incomplete ones too unless the only code has length 1).
template <class Tree>
__device__ bool build(Lds& L, Tree& T, const uint8_t* lens, int n) {
  constexpr int PB = Tree::BITS;
  const int lane = threadIdx.x;
  for (int i = lane; i < (1 << PB); i += 64) T.pri[i] = 0;
  if (lane == 0) {
    for (int l = 0; l < 16; l++) T.cnt[l] = 0;
    for (int i = 0; i < n; i++) T.cnt[lens[i]]++;
    T.cnt[0] = 0;
    int left = 1, maxl = 0;
    bool ok = true;
    for (int l = 1; l < 16; l++) {
      left = (left << 1) - T.cnt[l];
      if (left < 0) ok = false;
      if (T.cnt[l]) maxl = l;
    }
    if (ok && left > 0 && maxl != 1) ok = false;
    uint16_t offs[16], next[16];
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + T.cnt[l];
    uint32_t code = 0;   // first code of each length (RFC 1951 3.2.2)
    for (int l = 1; l < 16; l++) {
      code = (code + T.cnt[l - 1]) << 1;
      next[l] = (uint16_t)code;
    }
    for (int i = 0; i < n; i++) {
      int l = lens[i];
      if (!l) continue;
      T.sym[offs[l]++] = (uint16_t)i;
      L.codes[i] = next[l]++;
    }
    L.ok = ok;
  }
  __syncthreads();
  for (int i = lane; i < n; i += 64) {
    int l = lens[i];
    if (!l || l > PB) continue;
    uint32_t r = __brev((uint32_t)L.codes[i]) >> (32 - l);
    for (uint32_t k = r; k < (1u << PB); k += 1u << l) T.pri[k] = (uint16_t)((i << 4) | l);
  }
  __syncthreads();
  return L.ok;
}

// bits [q, q + 64) of the call's input (zero past its end)
struct Reader {
  const uint8_t* I;
  uint64_t wb;       // byte offset of the window (multiple of 4)
  uint32_t win;      // lane l: bytes wb + 4l .. wb + 4l + 3
  __device__ void load(uint64_t byte) {
    wb = byte & ~3ull;
    win = *(const uint32_t*)(I + wb + 4 * threadIdx.x);
  }
  __device__ uint64_t get(uint64_t q) {
    uint64_t k = (q >> 5) - (wb >> 2);
    if (k > 60) {
      load(q >> 3);
      k = (q >> 5) - (wb >> 2);
    }
    uint32_t sh = q & 31;
    uint64_t lo = readlane(win, (int)k) | ((uint64_t)readlane(win, (int)k + 1) << 32);
    uint64_t hi = readlane(win, (int)k + 2);
    uint64_t r = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    return ((uint64_t)readfirst((uint32_t)(r >> 32)) << 32) | readfirst((uint32_t)r);
  }
};

// A wave-uniform LDS value into a scalar register: the decoder's control runs
// on the SALU instead of as 64-lane vector ops.
__device__ __forceinline__ uint32_t su(uint32_t v) { return readfirst(v); }

// the primary-table entry for the bits in v ((sym << 4) | len; len 0: longer code)
template <class Tree>
__device__ __forceinline__ uint32_t decode_pri(const Tree& T, uint64_t v) {
  return su(T.pri[v & ((1u << Tree::BITS) - 1)]);
}

// Huffman decode of the bits in v: returns (sym << 4) | len, 0 if no code matches
template <class Tree>
__device__ __forceinline__ uint32_t decode(const Tree& T, uint64_t v) {
  uint32_t e = su(T.pri[v & ((1u << Tree::BITS) - 1)]);
  if (e & 15) return e;
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    code |= (int)((v >> (l - 1)) & 1);
    int count = (int)su(T.cnt[l]);
    if (code - first < count) return (su(T.sym[index + code - first]) << 4) | (uint32_t)l;
    index += count;
    first = (first + count) << 1;
    code <<= 1;
  }
  return 0;
}

#ifdef XCG_ZI_TIMING
// diagnostics build: cycles per phase, summed over calls (setup, fast literals,
// fast matches, careful path, flushes, stored copies, tail) and symbol counts
__device__ unsigned long long g_zi_t[10];
#define ZT_NOW() __builtin_readcyclecounter()
#define ZT_ADD(i, t0)                                                         \
  do {                                                                        \
    uint64_t t1_ = ZT_NOW();                                                  \
    if (threadIdx.x == 0) zt[i] += t1_ - (t0);                                \
    t0 = t1_;                                                                 \
  } while (0)
#else
#define ZT_NOW() 0ull
#define ZT_ADD(i, t0) (void)(t0)
#endif

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void zi_inflate_kernel(IArgs a) {
#ifdef XCG_ZI_TIMING
  uint64_t zt[10] = {0};
#endif
  uint64_t tz = ZT_NOW();
  __shared__ Lds L;
  const uint32_t ci = blockIdx.x;
  const ICall c = a.calls[ci];
  const int lane = threadIdx.x;
  IState* sp = a.st + c.stream;
  uint32_t mode = sp->mode, last = sp->last, stored_left = sp->stored_left, btype = sp->btype;
  uint32_t nlen = sp->nlen, ndist = sp->ndist;
  const uint64_t total0 = sp->total_out;
  const uint32_t npend = sp->npend;
  const uint64_t qend = 8ull * (npend + c.len);
  uint64_t q = sp->pend_bit;
  Reader R{a.I + c.i_off, 0, 0};
  R.load(0);
  // history -> ring
  const uint8_t* hist = a.hist + (uint64_t)c.stream * WSIZE;
  const uint64_t hn = total0 < (uint64_t)(RMASK + 1) ? total0 : (uint64_t)(RMASK + 1);
  for (uint64_t i = lane; i < hn; i += 64) {
    uint64_t pos = total0 - hn + i;
    L.ring[pos & RMASK] = hist[WSIZE - hn + i];
  }
  uint64_t pos = total0, flushed = total0;
  int32_t status = 0;
  uint32_t trailer = 0, have_trailer = 0;
  uint8_t* out = a.out + c.out_off;
  auto flush = [&]() {
    __syncthreads();
    for (uint64_t p = flushed + lane; p < pos; p += 64) out[p - total0] = L.ring[p & RMASK];
    flushed = pos;
    __threadfence();   // the flushed bytes are read back by far matches
  };
  // a match of `length` bytes from `dist` back, at pos
  auto copy_match = [&](uint32_t dist, uint32_t length) {
    if (dist >= length && dist <= NEAR) {
      for (uint32_t i = lane; i < length; i += 64) L.ring[(pos + i) & RMASK] = L.ring[(pos - dist + i) & RMASK];
    } else if (dist <= NEAR) {   // overlapping: byte i repeats source byte i mod dist
      uint32_t r = lane % dist;
      const uint32_t step = 64 % dist;
      for (uint32_t i = lane; i < length; i += 64) {
        L.ring[(pos + i) & RMASK] = L.ring[(pos - dist + r) & RMASK];
        r += step;
        if (r >= dist) r -= dist;
      }
    } else {                     // far: every source byte is in HBM already (pos - dist + 258 < flushed)
      for (uint32_t i = lane; i < length; i += 64) {
        const uint64_t x = pos - dist + i;
        L.ring[(pos + i) & RMASK] = x >= total0 ? out[x - total0] : hist[WSIZE - (total0 - x)];
      }
    }
  };
  auto tables_for_block = [&]() -> bool {   // (re)build the block's trees
    if (btype == 1) {
      for (int i = lane; i < 288; i += 64) L.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
      __syncthreads();
      build(L, L.lt, L.lens, 288);
      for (int i = lane; i < 30; i += 64) L.lens[i] = 5;
      __syncthreads();
      build(L, L.dt, L.lens, 30);
      return true;
    }
    bool ok = build(L, L.lt, L.dlens, nlen);
    ok = build(L, L.dt, L.dlens + nlen, ndist) && ok;
    return ok;
  };
  ZT_ADD(0, tz);
  if (mode == M_HUFF) {   // resume inside a block: rebuild its trees
    for (int i = lane; i < 320; i += 64) L.dlens[i] = sp->lens[i];
    __syncthreads();
    if (!tables_for_block()) mode = M_ERROR;
  }
  __syncthreads();
  bool stall = false;
  while (!stall && mode != M_ERROR && mode != M_DONE) {
    if (mode == M_HEADER) {   // zlib header: CMF FLG (RFC 1950)
      if (q + 16 > qend) { stall = true; break; }
      uint64_t v = R.get(q);
      uint32_t cmf = v & 0xff, flg = (v >> 8) & 0xff;
      if (((cmf << 8) | flg) % 31 != 0 || (cmf & 15) != 8 || (cmf >> 4) > 7 || (flg & 0x20)) { mode = M_ERROR; break; }
      q += 16;
      mode = M_BLOCK;
    } else if (mode == M_BLOCK) {
      const uint64_t q0 = q;
      if (q + 3 > qend) { stall = true; break; }
      uint64_t v = R.get(q);
      last = v & 1;
      btype = (v >> 1) & 3;
      q += 3;
      if (btype == 0) {
        q = (q + 7) & ~7ull;
        if (q + 32 > qend) { q = q0; stall = true; break; }
        v = R.get(q);
        uint32_t len = v & 0xffff, nl = (v >> 16) & 0xffff;
        if ((len ^ 0xffff) != nl) { mode = M_ERROR; break; }
        q += 32;
        stored_left = len;
        mode = M_STORED;
      } else if (btype == 1) {
        tables_for_block();
        mode = M_HUFF;
      } else if (btype == 2) {
        if (q + 14 > qend) { q = q0; stall = true; break; }
        v = R.get(q);
        nlen = (v & 31) + 257;
        ndist = ((v >> 5) & 31) + 1;
        uint32_t ncl = ((v >> 10) & 15) + 4;
        q += 14;
        if (nlen > 286 || ndist > 30) { mode = M_ERROR; break; }
        if (q + 3 * ncl > qend) { q = q0; stall = true; break; }
        if (lane < 19) L.lens[lane] = 0;
        __syncthreads();
        for (uint32_t i = 0; i < ncl; i++) {
          uint32_t l = (R.get(q) & 7);
          if (lane == 0) L.lens[CL_ORDER[i]] = (uint8_t)l;
          q += 3;
        }
        __syncthreads();
        if (!build(L, L.ct, L.lens, 19)) { mode = M_ERROR; break; }
        // the literal/length and distance code lengths, with repeats
        uint32_t n = 0;
        bool bad = false;
        while (n < nlen + ndist) {
          if (q >= qend) { stall = true; break; }
          uint64_t b = R.get(q);
          uint32_t e = decode(L.ct, b);
          uint32_t cl = e & 15, sym = e >> 4;
          if (!e || q + cl > qend) { if (!e) bad = true; else stall = true; break; }
          if (sym < 16) {
            q += cl;
            if (lane == 0) L.dlens[n] = (uint8_t)sym;
            n++;
            continue;
          }
          uint32_t rep, val = 0, xb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
          if (q + cl + xb > qend) { stall = true; break; }
          uint32_t x = (uint32_t)(b >> cl) & ((1u << xb) - 1);
          if (sym == 16) {
            if (n == 0) { bad = true; break; }
            __syncthreads();
            val = L.dlens[n - 1];
            rep = 3 + x;
          } else rep = (sym == 17 ? 3 : 11) + x;
          if (n + rep > nlen + ndist) { bad = true; break; }
          if (lane == 0) for (uint32_t r = 0; r < rep; r++) L.dlens[n + r] = (uint8_t)val;
          n += rep;
          q += cl + xb;
        }
        if (bad) { mode = M_ERROR; break; }
        if (stall) { q = q0; break; }
        __syncthreads();
        if (L.dlens[256] == 0 || !tables_for_block()) { mode = M_ERROR; break; }
        mode = M_HUFF;   // (its lengths reach sp->lens only when the call commits)
      } else {
        mode = M_ERROR;
        break;
      }
    } else if (mode == M_STORED) {
      uint64_t avail = (qend - q) >> 3;   // q is byte aligned here
      uint64_t n = stored_left < avail ? stored_left : avail;
      if (pos + n - total0 > c.out_cap) { status = -2; break; }
      // straight to the output (HBM), the ring's earlier bytes flushed first;
      // then the last 8 KiB also into the ring for later near matches
      flush();
      const uint8_t* src = R.I + (q >> 3);
      uint8_t* dst = out + (pos - total0);
      for (uint64_t i = lane; i < n; i += 64) dst[i] = src[i];
      const uint64_t keep = n < (uint64_t)(RMASK + 1) ? n : (uint64_t)(RMASK + 1);
      for (uint64_t i = lane; i < keep; i += 64) L.ring[(pos + n - keep + i) & RMASK] = src[n - keep + i];
      pos += n;
      flushed = pos;
      __threadfence();   // readable by far matches
      __syncthreads();
      q += 8 * n;
      ZT_ADD(5, tz);
      stored_left -= (uint32_t)n;
      if (stored_left) { stall = true; break; }
      mode = last ? M_TRAILER : M_BLOCK;
      R.load(q >> 3);
    } else if (mode == M_HUFF) {
      for (;;) {
        // fast path (as zlib's inflate_fast): while 128 input bits, 516 bytes of
        // output room and the ring before its next flush are guaranteed, decode
        // without per-field checks; literals straight from a 64-bit bit buffer
        // (one window fetch per run of literals)
        {
          const uint64_t qlim = qend > 128 ? qend - 128 : 0;
          const uint64_t pcap = total0 + c.out_cap > 516 ? total0 + c.out_cap - 516 : 0;
          while (q < qlim) {
            const uint64_t plim = flushed + FLUSH_AT < pcap ? flushed + FLUSH_AT : pcap;
            if (pos >= plim) break;
            uint64_t v = R.get(q);
            int vb = 64;
            uint32_t e = 0;
            ZT_ADD(3, tz);
            for (;;) {   // literals while the buffer surely holds a primary code
              e = decode_pri(L.lt, v);
              if ((e & 15) == 0 || (e >> 4) >= 256 || vb < LTree::BITS || pos >= plim) break;
              if (lane == 0) L.ring[pos & RMASK] = (uint8_t)(e >> 4);
              const uint32_t l1 = e & 15;
              pos++;
              v >>= l1;
              vb -= (int)l1;
              q += l1;
            }
            ZT_ADD(1, tz);
            if (pos >= plim) break;
            if (vb < LTree::BITS) continue;                // refill
            const uint32_t l1 = e & 15, sym = e >> 4;
            if (!l1 || sym == 256 || sym > 285) break;     // long code / end of block: the careful path
            const uint64_t vv = R.get(q);
            const uint32_t li = sym - 257, xl = LEXT[li];
            const uint32_t length = LBASE[li] + ((uint32_t)(vv >> l1) & ((1u << xl) - 1));
            const uint64_t qd = q + l1 + xl;
            const uint64_t vd = R.get(qd);
            const uint32_t ed = decode_pri(L.dt, vd);
            const uint32_t l2 = ed & 15, dsym = ed >> 4;
            if (!l2 || dsym > 29) break;
            const uint32_t xd = DEXT[dsym];
            const uint32_t dist = DBASE[dsym] + ((uint32_t)(vd >> l2) & ((1u << xd) - 1));
            if (dist > pos || dist > (uint32_t)WSIZE) break;
            // One wave: its LDS accesses are ordered, and every byte read lies
            // before pos, so no barrier is needed around the copy.
            copy_match(dist, length);
            pos += length;
            q = qd + l2 + xd;
            ZT_ADD(2, tz);
          }
        }
        ZT_ADD(3, tz);
        if (pos - flushed >= FLUSH_AT) { flush(); ZT_ADD(4, tz); }   // (the fast path's limit)
        uint64_t v = R.get(q);
        uint32_t e = decode(L.lt, v);
        uint32_t l1 = e & 15, sym = e >> 4;
        if (!e) { mode = (q + 15 <= qend) ? M_ERROR : mode; stall = mode != M_ERROR; break; }
        if (q + l1 > qend) { stall = true; break; }
        if (sym < 256) {
          if (pos + 1 - total0 > c.out_cap) { status = -2; break; }
          if (lane == 0) L.ring[pos & RMASK] = (uint8_t)sym;
          pos++;
          q += l1;
          continue;
        }
        if (sym == 256) {
          q += l1;
          mode = last ? M_TRAILER : M_BLOCK;
          break;
        }
        if (sym > 285) { mode = M_ERROR; break; }
        uint32_t li = sym - 257, xl = LEXT[li];
        if (q + l1 + xl > qend) { stall = true; break; }
        uint32_t length = LBASE[li] + ((uint32_t)(v >> l1) & ((1u << xl) - 1));
        uint64_t qd = q + l1 + xl;
        uint64_t vd = R.get(qd);
        uint32_t ed = decode(L.dt, vd);
        uint32_t l2 = ed & 15, dsym = ed >> 4;
        if (!ed) { mode = (qd + 15 <= qend) ? M_ERROR : mode; stall = mode != M_ERROR; break; }
        if (dsym > 29) { mode = M_ERROR; break; }
        uint32_t xd = DEXT[dsym];
        if (qd + l2 + xd > qend) { stall = true; break; }
        uint32_t dist = DBASE[dsym] + ((uint32_t)(vd >> l2) & ((1u << xd) - 1));
        if (dist > pos || dist > (uint32_t)WSIZE) { mode = M_ERROR; break; }   // too far back
        if (pos + length - total0 > c.out_cap) { status = -2; break; }
        __syncthreads();
        copy_match(dist, length);
        __syncthreads();
        pos += length;
        q = qd + l2 + xd;
      }
      if (status) break;
    } else if (mode == M_TRAILER) {
      q = (q + 7) & ~7ull;
      if (q + 32 > qend) { stall = true; break; }
      uint64_t v = R.get(q);
      uint32_t t = (uint32_t)v;
      trailer = __builtin_bswap32(t);
      have_trailer = 1;
      q += 32;
      mode = M_DONE;
    }
  }
  ZT_ADD(3, tz);
  if (status == 0 && mode == M_ERROR) status = -1;
  // InflatePipe: bytes after the stream's end are an error ("Stream ended but more data follows")
  if (status == 0 && mode == M_DONE && q < qend && c.len) status = -1;
  if (status == 0 && mode == M_DONE) status = 1;
  flush();
  __syncthreads();
  if (status == -1 && lane == 0) sp->mode = M_ERROR;   // InflatePipe::produce_error: the pipe is done
  if (status >= 0) {
    // the carried input for the next call
    uint64_t qb = q >> 3;
    uint64_t np = (qend >> 3) - qb;
    if (mode == M_DONE) np = 0;
    if (np > PEND_CAP) status = -1;
    else {
      for (uint64_t i = lane; i < np; i += 64) sp->pend[i] = R.I[qb + i];
      // A call that ends inside a dynamic block carries that block's code
      // lengths for the next call's resume.  Written here, with the rest of
      // the committed state, never while parsing: a call that ends in -2 (no
      // room) must leave the stream exactly as it found it, and the block it
      // resumes in is then still the one sp->lens describes.
      if (mode == M_HUFF && btype == 2)
        for (uint32_t i = lane; i < nlen + ndist; i += 64) sp->lens[i] = L.dlens[i];
      // history = the last 32 KiB of output: the old history moved down by this
      // call's output length (ascending, so no lane reads what another wrote),
      // then the output itself (flushed and fenced above)
      const uint64_t ol = pos - total0;
      uint8_t* h = a.hist + (uint64_t)c.stream * WSIZE;
      if (ol < (uint64_t)WSIZE) {
        for (uint64_t i0 = 0; ol && i0 < WSIZE - ol; i0 += 64) {
          const uint64_t i = i0 + lane;
          const uint8_t b = i < WSIZE - ol ? h[i + ol] : 0;
          __syncthreads();
          if (i < WSIZE - ol) h[i] = b;
        }
        for (uint64_t i = lane; i < ol; i += 64) h[WSIZE - ol + i] = out[i];
      } else {
        for (uint64_t i = lane; i < (uint64_t)WSIZE; i += 64) h[i] = out[ol - WSIZE + i];
      }
      if (lane == 0) {
        sp->total_out = pos;
        sp->mode = mode;
        sp->last = last;
        sp->stored_left = stored_left;
        sp->btype = btype;
        sp->nlen = nlen;
        sp->ndist = ndist;
        sp->npend = (uint32_t)np;
        sp->pend_bit = (uint32_t)(q & 7);
      }
    }
  }
  ZT_ADD(6, tz);
#ifdef XCG_ZI_TIMING
  if (lane == 0)
    for (int i = 0; i < 7; i++) atomicAdd(&g_zi_t[i], (unsigned long long)zt[i]);
#endif
  if (lane == 0) {
    IRes r;
    r.out_len = (uint32_t)(pos - total0);
    r.status = status;
    r.trailer = trailer;
    r.have_trailer = have_trailer;
    a.res[ci] = r;
  }
}

// adler32 of each call's output, combined into the stream's; the trailer
// check (one wave per call)
// adler32 of the call's output (four waves per call, consecutive 4-byte words:
// coalesced), combined with the stream's, checked against a trailer.
__global__ __launch_bounds__(256) void zi_adler_kernel(IArgs a) {
  __shared__ uint64_t red[2][4];
  const uint32_t ci = blockIdx.x;
  const ICall c = a.calls[ci];
  IRes r = a.res[ci];
  const int t = threadIdx.x, lane = t & 63;
  IState* sp = a.st + c.stream;
  if (r.status >= 0) {
    const uint8_t* d = a.out + c.out_off;
    const uint64_t n = r.out_len;
    uint64_t A = 0, B = 0;   // sum d_i, sum i * d_i, reduced mod 65521 every 4096 words
    const uint64_t words = n / 4;
    uint32_t since = 0;
#pragma unroll 4
    for (uint64_t w = t; w < words; w += 256) {
      const uint32_t v = *(const u32_u*)(d + 4 * w);
      const uint32_t s = (v & 0xff) + ((v >> 8) & 0xff) + ((v >> 16) & 0xff) + (v >> 24);
      A += s;
      B += (4 * w) * s + ((v >> 8) & 0xff) + 2 * ((v >> 16) & 0xff) + 3 * (v >> 24);
      if (++since == 4096) {
        A %= 65521u;
        B %= 65521u;
        since = 0;
      }
    }
    for (uint64_t i = 4 * words + t; i < n; i += 256) {
      const uint32_t v = d[i];
      A += v;
      B += i * v;
    }
    A %= 65521u;
    B %= 65521u;
    for (int o = 32; o >= 1; o >>= 1) {
      A += __shfl_xor(A, o);
      B += __shfl_xor(B, o);
    }
    if (lane == 0) {
      red[0][t >> 6] = A;
      red[1][t >> 6] = B;
    }
  }
  __syncthreads();
  if (t == 0 && r.status >= 0) {
    const uint64_t n = r.out_len;
    uint64_t A = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) % 65521u;
    uint64_t B = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) % 65521u;
    {
      uint32_t old = sp->adler;
      uint64_t s1 = old & 0xffff, s2 = old >> 16, nn = n % 65521u;
      uint64_t ns1 = (s1 + A) % 65521u;
      uint64_t ns2 = (s2 + nn * s1 + nn * A + 65521u - B) % 65521u;
      uint32_t ad = (uint32_t)((ns2 << 16) | ns1);
      sp->adler = ad;
      if (r.have_trailer && r.trailer != ad) {
        r.status = -1;
        sp->mode = M_ERROR;
      }
    }
  }
  if (t == 0) {
    a.res[ci] = r;
    a.out_len[ci] = r.out_len;
    a.status[ci] = r.status;
  }
}

}  // namespace zi
}  // namespace xcg

using namespace xcg::zi;

struct xcg_zinflate {
  int device = 0;
  uint32_t nstreams = 0;
  IState* st = nullptr;
  uint8_t* hist = nullptr;
  uint8_t* scratch = nullptr;
  size_t scratch_cap = 0;
  void* meta = nullptr;
  size_t meta_cap = 0;
  void* h_meta = nullptr;
  size_t h_meta_cap = 0;
  hipEvent_t done = nullptr;
  // host-buffer calls (xcg_zinflate_host: the drop-in InflatePipe::consume):
  // kept staging and a private stream
  hipStream_t hst = nullptr;
  uint8_t* hs_h = nullptr;         // pinned
  uint8_t* hs_d = nullptr;
  size_t hs_hcap = 0, hs_dcap = 0;
};

namespace {
int igrow(void** p, size_t* cap, size_t want, bool pinned) {
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
inline size_t ial(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

extern "C" {

int xcg_zinflate_create(int device, uint32_t nstreams, xcg_zinflate** out) {
  if (!out || nstreams == 0) return XCG_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return XCG_EHIP;
  xcg_zinflate* z = new xcg_zinflate();
  z->device = device;
  z->nstreams = nstreams;
  if (hipMalloc(&z->st, sizeof(IState) * nstreams) != hipSuccess ||
      hipMalloc(&z->hist, (size_t)WSIZE * nstreams) != hipSuccess ||
      hipEventCreateWithFlags(&z->done, hipEventDisableTiming) != hipSuccess) {
    delete z;
    return XCG_ENOMEM;
  }
  std::vector<IState> init(nstreams);
  memset(init.data(), 0, sizeof(IState) * nstreams);
  for (auto& s : init) s.adler = 1;
  if (hipMemcpy(z->st, init.data(), sizeof(IState) * nstreams, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(z->hist, 0, (size_t)WSIZE * nstreams) != hipSuccess) {
    delete z;
    return XCG_EHIP;
  }
  *out = z;
  return XCG_OK;
}

void xcg_zinflate_destroy(xcg_zinflate* z) {
  if (!z) return;
  (void)hipSetDevice(z->device);
  if (z->done) (void)hipEventSynchronize(z->done);
  (void)hipFree(z->st);
  (void)hipFree(z->hist);
  (void)hipFree(z->scratch);
  (void)hipFree(z->meta);
  if (z->h_meta) (void)hipHostFree(z->h_meta);
  if (z->done) (void)hipEventDestroy(z->done);
  if (z->hs_h) (void)hipHostFree(z->hs_h);
  (void)hipFree(z->hs_d);
  if (z->hst) (void)hipStreamDestroy(z->hst);
  delete z;
}

int xcg_zinflate_batch(xcg_zinflate* z, const uint8_t* d_in, const uint64_t* h_in_off, const uint32_t* h_len,
                       const uint32_t* h_stream, uint32_t n, uint8_t* d_out, const uint64_t* h_out_off,
                       const uint32_t* h_out_cap, uint32_t* d_out_len, int32_t* d_status, void* stream) {
  if (!z || n == 0 || !h_in_off || !h_len || !h_stream || !h_out_off || !h_out_cap || !d_out_len || !d_status)
    return XCG_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  (void)hipSetDevice(z->device);
  std::vector<ICall> calls(n);
  std::vector<uint8_t> seen(z->nstreams, 0);
  size_t io = 0;
  uint32_t maxlen = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (h_stream[i] >= z->nstreams || seen[h_stream[i]] || h_len[i] > (1u << 26)) return XCG_EINVAL;
    seen[h_stream[i]] = 1;
    ICall& c = calls[i];
    c.in_off = h_in_off[i];
    c.out_off = h_out_off[i];
    c.len = h_len[i];
    c.stream = h_stream[i];
    c.out_cap = h_out_cap[i];
    c.i_off = io;
    io += ial((size_t)PEND_CAP + c.len + IPAD, 256);
    maxlen = std::max(maxlen, c.len);
  }
  size_t o_I = 0, o_res = ial(io, 256), o_end = ial(o_res + sizeof(IRes) * n, 256);
  if (hipEventSynchronize(z->done) != hipSuccess) return XCG_EHIP;
  if (igrow((void**)&z->scratch, &z->scratch_cap, o_end, false)) return XCG_ENOMEM;
  size_t m_end = ial(sizeof(ICall) * n, 256);
  if (igrow(&z->meta, &z->meta_cap, m_end, false) || igrow(&z->h_meta, &z->h_meta_cap, m_end, true)) return XCG_ENOMEM;
  memcpy(z->h_meta, calls.data(), sizeof(ICall) * n);
  if (hipMemcpyAsync(z->meta, z->h_meta, m_end, hipMemcpyHostToDevice, st) != hipSuccess) return XCG_EHIP;
  IArgs a;
  a.calls = (const ICall*)z->meta;
  a.st = z->st;
  a.hist = z->hist;
  a.in = d_in;
  a.out = d_out;
  a.I = z->scratch + o_I;
  a.res = (IRes*)(z->scratch + o_res);
  a.out_len = d_out_len;
  a.status = d_status;
  uint32_t tiles = std::min<uint32_t>(64, (PEND_CAP + maxlen + IPAD + 4095) / 4096);   // 4 KiB per block
  hipLaunchKernelGGL(zi_prep_kernel, dim3(tiles, n), dim3(256), 0, st, a);
  hipLaunchKernelGGL(zi_inflate_kernel, dim3(n), dim3(64), 0, st, a);
  hipLaunchKernelGGL(zi_adler_kernel, dim3(n), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) return XCG_EHIP;
  if (hipEventRecord(z->done, st) != hipSuccess) return XCG_EHIP;
  return XCG_OK;
}

// A fresh InflatePipe on slot `stream` (inflateInit, zlib/inflate_pipe.cc:38-50):
// nothing of the slot's previous stream -- mode, totals, carried input,
// history, adler32 -- survives.
int xcg_zinflate_reset(xcg_zinflate* z, uint32_t stream) {
  if (!z || stream >= z->nstreams) return XCG_EINVAL;
  (void)hipSetDevice(z->device);
  if (hipEventSynchronize(z->done) != hipSuccess) return XCG_EHIP;
  IState s0;
  memset(&s0, 0, sizeof s0);
  s0.adler = 1;
  if (hipMemcpy(z->st + stream, &s0, sizeof s0, hipMemcpyHostToDevice) != hipSuccess) return XCG_EHIP;
  return XCG_OK;
}

// Host buffers, synchronous: inputs at h_in + h_in_off[i], outputs to h_out +
// h_out_off[i] (room h_out_cap[i]); lengths and statuses to host arrays.
int xcg_zinflate_host(xcg_zinflate* z, const uint8_t* h_in, const uint64_t* h_in_off, const uint32_t* h_len,
                      const uint32_t* h_stream, uint32_t n, uint8_t* h_out, const uint64_t* h_out_off,
                      const uint32_t* h_out_cap, uint32_t* h_out_len, int32_t* h_status) {
  if (!z || n == 0 || !h_in_off || !h_len || !h_out_cap || !h_out_len || !h_status) return XCG_EINVAL;
  (void)hipSetDevice(z->device);
  if (!z->hst && hipStreamCreateWithFlags(&z->hst, hipStreamNonBlocking) != hipSuccess) return XCG_EHIP;
  uint64_t in_end = 0, out_end = 0;
  std::vector<uint64_t> doff(n);
  for (uint32_t i = 0; i < n; i++) {
    in_end = std::max(in_end, h_in_off[i] + h_len[i]);
    doff[i] = out_end;
    out_end += ial(h_out_cap[i] ? h_out_cap[i] : 1, 4);
  }
  // staging: [len n][status n][in][out]
  const size_t o_st = ial(4ull * n, 256), o_in = ial(o_st + 4ull * n, 256), o_out = ial(o_in + in_end + 1, 256),
               o_end = ial(o_out + out_end, 256);
  if (igrow((void**)&z->hs_h, &z->hs_hcap, o_end, true) || igrow((void**)&z->hs_d, &z->hs_dcap, o_end, false))
    return XCG_ENOMEM;
  if (in_end) memcpy(z->hs_h + o_in, h_in, in_end);
  if (in_end && hipMemcpyAsync(z->hs_d + o_in, z->hs_h + o_in, in_end, hipMemcpyHostToDevice, z->hst) != hipSuccess)
    return XCG_EHIP;
  int rc = xcg_zinflate_batch(z, z->hs_d + o_in, h_in_off, h_len, h_stream, n, z->hs_d + o_out, doff.data(), h_out_cap,
                              (uint32_t*)z->hs_d, (int32_t*)(z->hs_d + o_st), z->hst);
  if (rc != XCG_OK) return rc;
  if (hipMemcpyAsync(z->hs_h, z->hs_d, o_in, hipMemcpyDeviceToHost, z->hst) != hipSuccess ||
      hipStreamSynchronize(z->hst) != hipSuccess)
    return XCG_EHIP;
  memcpy(h_out_len, z->hs_h, 4ull * n);
  memcpy(h_status, z->hs_h + o_st, 4ull * n);
  // the outputs: only what was produced (the room is up to 8x the input)
  for (uint32_t i = 0; i < n; i++)
    if (h_out_len[i] && hipMemcpyAsync(z->hs_h + o_out + doff[i], z->hs_d + o_out + doff[i], h_out_len[i],
                                       hipMemcpyDeviceToHost, z->hst) != hipSuccess)
      return XCG_EHIP;
  if (hipStreamSynchronize(z->hst) != hipSuccess) return XCG_EHIP;
  for (uint32_t i = 0; i < n; i++)
    if (h_out_len[i]) memcpy(h_out + h_out_off[i], z->hs_h + o_out + doff[i], h_out_len[i]);
  return XCG_OK;
}

#ifdef XCG_ZI_TIMING
int xcg_debug_zi_times(uint64_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zi_t), 8 * 10) != hipSuccess) return XCG_EHIP;
  uint64_t z[10] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_zi_t), z, sizeof z) == hipSuccess ? XCG_OK : XCG_EHIP;
}
#endif

}  // extern "C"
