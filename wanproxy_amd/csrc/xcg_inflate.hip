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
  uint32_t* pres;           // NW > 1: RES_CAP resolve slots per call
  uint32_t warm, maxthr;    // NW > 1: warm-up bits, threads per region (A/B: XCG_ZI_WARM, XCG_ZI_THREADS)
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
  uint16_t bfirst[16], boffs[16];   // build(): first code, first symbol slot of each length
};

// The decoder's own barrier: the whole workgroup for the one-wave kernel; for
// the many-wave kernel the decoder's control runs in wave 0 alone, so its
// barriers order that wave's LDS traffic only (the other waves wait in
// helper_loop until wave 0 hands them a region).
template <int NW>
__device__ __forceinline__ void wsync() {
  if constexpr (NW == 1) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

// Canonical decoder from code lengths (inflate_table's rules: over-subscribed
// sets are errors, incomplete ones too unless the only code has length 1).
// One wave, no serial loop over the symbols: per-length counts and each
// symbol's rank among the symbols of its length come from ballots over chunks
// of 64 symbols (canonical codes are assigned in symbol order within a
// length), the first code and table offset of each length from the counts.
template <int NW, class Tree>
__device__ bool build(Lds& L, Tree& T, const uint8_t* lens, int n) {
  constexpr int PB = Tree::BITS;
  const int lane = threadIdx.x;
  for (int i = lane; i < (1 << PB); i += 64) T.pri[i] = 0;
  const int nch = (n + 63) >> 6;
  uint32_t cnt = 0;                  // lane l in 1..15: codes of length l
  for (int ch = 0; ch < nch; ch++) {
    const int i = (ch << 6) + lane;
    const int l = i < n ? lens[i] : 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
      const uint32_t c = (uint32_t)__popcll(ballot(l == k));
      if (lane == k) cnt += c;
    }
  }
  // Kraft check, first code and symbol offset of each length (lane l)
  int left = 1, maxl = 0;
  bool ok = true;
  uint32_t first = 0, offs = 0;
#pragma unroll
  for (int k = 1; k < 16; k++) {
    const uint32_t ck = readlane(cnt, k);
    left = (left << 1) - (int)ck;
    if (left < 0) ok = false;
    if (ck) maxl = k;
    if (k < lane) {
      first += ck << (lane - k);   // RFC 1951 3.2.2: code(l) = (code(l-1) + count(l-1)) << 1
      offs += ck;
    }
  }
  if (ok && left > 0 && maxl != 1) ok = false;
  if (lane < 16) {
    T.cnt[lane] = (uint16_t)(lane ? cnt : 0);
    L.bfirst[lane] = (uint16_t)first;
    L.boffs[lane] = (uint16_t)offs;
  }
  wsync<NW>();
  uint32_t run = 0;                  // lane l: symbols of length l placed so far
  const uint64_t below = (1ull << lane) - 1;
  for (int ch = 0; ch < nch; ch++) {
    const int i = (ch << 6) + lane;
    const int l = i < n ? lens[i] : 0;
    uint32_t rank = 0, add = 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
      const uint64_t b = ballot(l == k);
      const uint32_t base = readlane(run, k);
      if (l == k) rank = base + (uint32_t)__popcll(b & below);
      if (lane == k) add = (uint32_t)__popcll(b);
    }
    run += add;
    if (l) {
      T.sym[L.boffs[l] + rank] = (uint16_t)i;
      L.codes[i] = (uint16_t)(L.bfirst[l] + rank);
    }
  }
  wsync<NW>();
  for (int i = lane; i < n; i += 64) {
    int l = lens[i];
    if (!l || l > PB) continue;
    uint32_t r = __brev((uint32_t)L.codes[i]) >> (32 - l);
    for (uint32_t k = r; k < (1u << PB); k += 1u << l) T.pri[k] = (uint16_t)((i << 4) | l);
  }
  wsync<NW>();
  return ok;
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

// A dynamic block's literal/length and distance code lengths, with repeats
// (RFC 1951 3.2.7), into L.dlens: the serial loop of the decoder, in a function
// of its own so that its few live values stay in registers (the decoder around
// it spills SGPRs into VGPR lanes).  The bits come from a 64-bit buffer
// refilled when fewer than a code (7) and its extra bits (7) remain; the code-
// length code's 128-entry table sits in `ctw`, two entries per lane.  Returns
// 0 with q past the sequence, 1 when the input ends inside it, 2 on bad data.
__device__ __attribute__((noinline)) int cl_sequence(Lds& L, const uint8_t* I, uint64_t& q_io, uint64_t qend_in,
                                                     uint32_t N, uint32_t ctw) {
  const int lane = threadIdx.x;
  uint64_t q = ((uint64_t)readfirst((uint32_t)(q_io >> 32)) << 32) | readfirst((uint32_t)q_io);
  const uint64_t qend = ((uint64_t)readfirst((uint32_t)(qend_in >> 32)) << 32) | readfirst((uint32_t)qend_in);
  N = readfirst(N);
  Reader R{I, 0, 0};
  R.load(q >> 3);
  uint32_t n = 0, prev = 0;
  int rc = 0;
  uint64_t b = 0;
  uint32_t bb = 0;
  while (n < N) {
    if (q >= qend) { rc = 1; break; }
    if (bb < 14) {
      b = R.get(q);
      bb = 64;
    }
    const uint32_t ci = (uint32_t)b & 127;
    const uint32_t e = (readlane(ctw, (int)(ci >> 1)) >> (16 * (ci & 1))) & 0xffff;
    const uint32_t cl = e & 15, sym = e >> 4;
    if (!e) { rc = 2; break; }
    if (q + cl > qend) { rc = 1; break; }
    if (sym < 16) {
      q += cl;
      b >>= cl;
      bb -= cl;
      if (lane == 0) L.dlens[n] = (uint8_t)sym;
      prev = sym;
      n++;
      continue;
    }
    uint32_t rep, val = 0;
    const uint32_t xb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
    if (q + cl + xb > qend) { rc = 1; break; }
    const uint32_t x = (uint32_t)(b >> cl) & ((1u << xb) - 1);
    if (sym == 16) {
      if (n == 0) { rc = 2; break; }
      val = prev;
      rep = 3 + x;
    } else rep = (sym == 17 ? 3 : 11) + x;
    if (n + rep > N) { rc = 2; break; }
    for (uint32_t r = lane; r < rep; r += 64) L.dlens[n + r] = (uint8_t)val;
    prev = val;
    n += rep;
    q += cl + xb;
    b >>= cl + xb;
    bb -= cl + xb;
  }
  q_io = q;
  return rc;
}

// The same sequence decoded speculatively by wave 0's 64 lanes (the
// workgroup kernels): lane l owns bits [36 l, 36 l + 36) of the next 2304 (more
// than the longest sequence, 316 lengths x 7 bits).  It decodes the 48 bits
// before its range to fall onto the true symbol starts, decodes its range,
// and the lanes move to their predecessors' ends until the starts are fixed
// up to the lane that completes the nlen + ndist lengths (or stops).  A scan of
// the lanes' repeat counts places them; each lane then writes its lengths and
// checks the serial loop's conditions in its order, and the first lane with an
// event decides.  Returns 0 (q past the sequence), 1 (input ends inside it),
// 2 (bad data), or 3 to leave it to cl_sequence.
constexpr uint32_t CL_LANE_BITS = 36, CL_WARM = 48, CL_INV = 0xffffffffu;

__device__ __forceinline__ uint32_t cl_at(const Lds& L, const uint32_t* bits, uint32_t sh0, uint32_t j) {
  const uint32_t bp = sh0 + j, w = bp >> 5;
  const uint64_t v = (((uint64_t)bits[w + 1] << 32) | bits[w]) >> (bp & 31);
  const uint32_t e = L.ct.pri[v & 127];
  if (!(e & 15)) return CL_INV;
  const uint32_t cl = e & 15, sym = e >> 4;
  const uint32_t xb = sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0;
  const uint32_t x = (uint32_t)(v >> cl) & ((1u << xb) - 1);
  const uint32_t rep = sym < 16 ? 1 : sym == 18 ? 11 + x : 3 + x;
  return sym | (rep << 8) | (cl << 16) | (xb << 20);
}

// decode from s while s < lim: the end; cnt = lengths produced; fl: stopped at
// an invalid code; lv / hv: value of the last non-16 symbol, and whether any
__device__ __forceinline__ uint32_t cl_run(const Lds& L, const uint32_t* bits, uint32_t sh0, uint32_t s, uint32_t lim,
                                           uint32_t& cnt, uint32_t& fl, uint32_t& lv, uint32_t& hv) {
  cnt = 0;
  fl = 0;
  lv = 0;
  hv = 0;
  while (s < lim) {
    const uint32_t in = cl_at(L, bits, sh0, s);
    if (in == CL_INV) {
      fl = 1;
      break;
    }
    const uint32_t sym = in & 255;
    cnt += (in >> 8) & 255;
    if (sym != 16) {
      lv = sym < 16 ? sym : 0;
      hv = 1;
    }
    s += ((in >> 16) & 15) + ((in >> 20) & 15);
  }
  return s;
}

template <int NW>
__device__ __attribute__((noinline)) int cl_spec(Lds& L, uint32_t* bits, const uint8_t* I, uint64_t& q_io,
                                                 uint64_t qend_in, uint32_t N) {
  const int lane = threadIdx.x;
  const uint64_t q = ((uint64_t)readfirst((uint32_t)(q_io >> 32)) << 32) | readfirst((uint32_t)q_io);
  const uint64_t qend = ((uint64_t)readfirst((uint32_t)(qend_in >> 32)) << 32) | readfirst((uint32_t)qend_in);
  N = readfirst(N);
  const uint64_t qw = q >> 5;
  for (int k = lane; k < 80; k += 64) bits[k] = ((const uint32_t*)I)[qw + k];
  wsync<NW>();
  const uint32_t sh0 = (uint32_t)(q & 31);
  const uint32_t c0 = (uint32_t)lane * CL_LANE_BITS, c1 = c0 + CL_LANE_BITS;
  uint32_t s = c0, cnt, fl, lv, hv;
  if (lane > 0) {
    uint32_t wc, wf, wl, wh;
    const uint32_t we = cl_run(L, bits, sh0, c0 > CL_WARM ? c0 - CL_WARM : 0, c0, wc, wf, wl, wh);
    if (!wf) s = we;
  }
  uint32_t e = cl_run(L, bits, sh0, s, c1, cnt, fl, lv, hv);
  for (int it = 0; it < 64; it++) {   // fixed point of the lanes' starts
    const uint32_t pe = __shfl_up(e, 1), pf = __shfl_up(fl, 1);
    const bool mv = lane > 0 && !pf && pe != s;
    const uint64_t bm = ballot(mv);
    if (!bm) break;
    const uint32_t incl = wave_incl_scan(cnt);
    const uint64_t bt = ballot(incl >= N) | ballot(fl != 0);
    if (bt && __builtin_ctzll(bt) < __builtin_ctzll(bm)) break;   // every start up to the deciding lane is final
    if (mv) {
      s = pe;
      e = cl_run(L, bits, sh0, s, c1, cnt, fl, lv, hv);
    }
  }
  const uint32_t incl = wave_incl_scan(cnt);
  const uint32_t base = incl - cnt;
  // the value of the last non-16 symbol below this lane (the "previous length" a 16 repeats)
  uint32_t tag = hv ? (uint32_t)lane + 1 : 0u;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(tag, o);
    if (lane >= o) tag = max(tag, y);
  }
  uint32_t ex = __shfl_up(tag, 1);
  if (lane == 0) ex = 0;
  const uint32_t pv = __shfl(lv, ex ? (int)ex - 1 : 0);
  uint32_t prev = ex ? pv : 0;
  // write and check, in stream order within the lane
  uint32_t ev = 0, evbits = 0;   // 1 stall, 2 bad, 3 complete (evbits: bits consumed)
  if (base < N) {
    uint32_t r = s, o = base;
    while (r < c1) {
      const uint64_t pos = q + r;
      if (pos >= qend) { ev = 1; break; }
      const uint32_t in = cl_at(L, bits, sh0, r);
      if (in == CL_INV) { ev = 2; break; }
      const uint32_t sym = in & 255, rep = (in >> 8) & 255, cl = (in >> 16) & 15, xb = (in >> 20) & 15;
      if (pos + cl > qend) { ev = 1; break; }
      if (sym >= 16 && pos + cl + xb > qend) { ev = 1; break; }
      if (sym == 16 && o == 0) { ev = 2; break; }
      if (o + rep > N) { ev = 2; break; }
      const uint32_t val = sym < 16 ? sym : sym == 16 ? prev : 0;
      for (uint32_t k = 0; k < rep; k++) L.dlens[o + k] = (uint8_t)val;
      prev = val;
      o += rep;
      r += cl + xb;
      if (o == N) {
        ev = 3;
        evbits = r;
        break;
      }
    }
  }
  const uint64_t bev = ballot(ev != 0);
  wsync<NW>();
  if (!bev) return 3;
  const int dl = __builtin_ctzll(bev);
  const uint32_t dev = readlane(ev, dl), dbits = readlane(evbits, dl);
  if (dev == 3) {
    q_io = q + dbits;
    return 0;
  }
  return (int)dev;
}

// ---------------------------------------------------------------------------
// One call on a whole workgroup (the per-call path: a consume() with few
// others in its batch).  Wave 0 runs the decoder above; inside a Huffman block
// it hands the workgroup a region of the block's input (up to IN_CAP bytes,
// ending 128 bits before the call's input end, where the careful path takes
// over).  The region is cut into equal bit ranges, one per thread; thread t
// decodes from its range start as if a symbol began there (Huffman codes
// resynchronise within a few symbols) and ends at the first symbol boundary
// past its range.  Thread t's start is then replaced by thread t-1's end and
// the changed threads decode again until no start moves (a fixed point:
// thread 0 starts on a true boundary, so by induction every start is one).
// The threads before the first one that met an end of block or an invalid
// code commit: a scan of their byte counts places them, a second decode
// writes literal bytes and, for every match byte, the position it copies
// (dist back, modulo dist inside an overlapping match, so each points before
// its own match); pointer jumping over those resolves every byte (log of the
// match-on-match depth rounds).  Wave 0 resumes from the first uncommitted
// thread's start -- its end of block, its error, its input end -- exactly as
// the one-wave decoder would have reached it.
constexpr uint32_t IN_CAP = 32768;    // region input bytes
constexpr uint32_t SMIN = 128;        // bits per thread at least (> a 48-bit symbol)
constexpr uint32_t RES_CAP = 65536;   // region output bytes (the call's u32 resolve slots: 256 KiB)
constexpr uint32_t RES_FLAG = 0x80000000u;
constexpr uint32_t PBIAS = 1u << 20;  // resolve slot: PBIAS + source index (may be < 0: before the region)
constexpr uint32_t F_STOP = 1, F_BAD = 2;
constexpr uint64_t PAR_MIN_BITS = 8 * 2048;
constexpr uint32_t WARM_DEFAULT = 128;   // bits decoded before a thread's range to find the true path

template <int NW>
struct ParT {
  static constexpr int NT = 64 * NW;
  static constexpr uint32_t INC = NW >= 8 ? IN_CAP : IN_CAP * NW / 8;   // (smaller workgroups: more per CU by LDS)
  uint64_t stg[INC / 8 + 8];          // the region's input, 8-byte words from byte b0
  uint32_t st[NT], nst[NT];           // thread t's start, and the one it moves to
  uint32_t endp[NT];                  // bit where thread t's decode ended
  uint32_t cnt[NT];                   // ... the bytes it produced
  uint16_t list[NT];                  // threads whose start moves in this pass
  uint32_t nd;
  uint8_t flag[NT];                   // ... and whether at an end of block / invalid code
  uint32_t incl[NT];                  // inclusive scan of the committed threads' byte counts
  uint32_t flt[1 << 10], fdt[1 << PRI];   // the block's primary tables as lfast / dfast entries
  uint32_t wsum[NW];
  uint32_t any[2], f, f2, f3;
  uint32_t chg[2], fm[2];             // fixed point: first thread whose start moved / that stopped
  uint32_t cmd;                       // 0 done, 1 Huffman region, 2 stored copy
  uint64_t q0, qlim, pos0, room, n, soff;
  uint32_t R, stopped;
  uint64_t qn;
  uint64_t t_ol;                      // the tail's history update: output length, and whether to do it
  uint32_t t_do;
};
template <>
struct ParT<1> {};

__device__ __forceinline__ uint32_t ld_ws(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_ws(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// bits [r, r + 64) of the staged region
__device__ __forceinline__ uint64_t get64(const uint64_t* stg, uint32_t r) {
  const uint32_t w = r >> 6, sh = r & 63;
  const uint64_t lo = stg[w], hi = stg[w + 1];
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

// one lane's Huffman decode (as decode(), per lane)
template <class Tree>
__device__ __forceinline__ uint32_t ldec(const Tree& T, uint64_t v) {
  const uint32_t e = T.pri[v & ((1u << Tree::BITS) - 1)];
  if (e & 15) return e;
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    code |= (int)((v >> (l - 1)) & 1);
    const int count = (int)T.cnt[l];
    if (code - first < count) return ((uint32_t)T.sym[index + code - first] << 4) | (uint32_t)l;
    index += count;
    first = (first + count) << 1;
    code <<= 1;
  }
  return 0;
}

// Region tables (ParT::flt / fdt), 32 bits per primary entry: code length in
// bits 0-3 (0: a longer code), FT_STOP for an end of block / invalid symbol,
// FT_MATCH for a length.  Literal: byte in bits 8-15; length: base in bits
// 8-16, extra bits in 20-23; distance: base in bits 8-23, extra bits in 24-27.
constexpr uint32_t FT_MATCH = 16, FT_STOP = 32;
__device__ __forceinline__ uint32_t lfast(uint32_t e) {   // e: (sym << 4) | len, 0: no code
  const uint32_t len = e & 15, sym = e >> 4;
  if (!e) return FT_STOP | 1;
  if (sym < 256) return len | (sym << 8);
  if (sym == 256 || sym > 285) return len | FT_STOP;
  return len | FT_MATCH | ((uint32_t)LBASE[sym - 257] << 8) | ((uint32_t)LEXT[sym - 257] << 20);
}
__device__ __forceinline__ uint32_t dfast(uint32_t e) {
  const uint32_t len = e & 15, sym = e >> 4;
  if (!e || sym > 29) return FT_STOP | 1;
  return len | ((uint32_t)DBASE[sym] << 8) | ((uint32_t)DEXT[sym] << 24);
}

// Decode from bit r while r < lim: e = the bit after the last symbol, n = the
// bytes produced, fl = F_STOP at an end of block / invalid code (e = its
// start), F_BAD (WRITE) at a distance past the stream's start.  WRITE: slot
// o + i of res gets byte i (RES_FLAG | byte) or its source (PBIAS + index).
template <bool WRITE, int NW>
__device__ __forceinline__ void spec(const Lds& L, const ParT<NW>& P, uint32_t r, const uint32_t lim, uint32_t& e,
                                     uint32_t& n, uint32_t& fl, uint32_t* res, uint32_t o, uint64_t pos0) {
  n = 0;
  fl = 0;
  // a 64-bit buffer of the bits from r, refilled from LDS when fewer than the
  // 48 a length/distance pair may take remain (every ~5 literals)
  uint64_t v = 0;
  uint32_t vb = 0;
  while (r < lim) {
    if (vb < 48) {
      v = get64(P.stg, r);
      vb = 64;
    }
    // the region's 32-bit tables: one lookup gives a literal, or a length's
    // base and extra bits (a distance likewise); codes past the primary bits
    // go the canonical way
    uint32_t fe = P.flt[v & ((1u << LTree::BITS) - 1)];
    if (!(fe & 15)) fe = lfast(ldec(L.lt, v));
    const uint32_t l1 = fe & 15;
    if (!(fe & (FT_MATCH | FT_STOP))) {
      if (WRITE) st_ws(res + o + n, RES_FLAG | ((fe >> 8) & 255));
      n++;
      r += l1;
      v >>= l1;
      vb -= l1;
      continue;
    }
    if (fe & FT_STOP) { fl = F_STOP; break; }
    const uint32_t xl = (fe >> 20) & 15;
    const uint32_t length = ((fe >> 8) & 511) + ((uint32_t)(v >> l1) & ((1u << xl) - 1));
    const uint64_t v2 = v >> (l1 + xl);
    uint32_t fd = P.fdt[v2 & ((1u << DTree::BITS) - 1)];
    if (!(fd & 15)) fd = dfast(ldec(L.dt, v2));
    if (fd & FT_STOP) { fl = F_STOP; break; }
    const uint32_t l2 = fd & 15, xd = (fd >> 24) & 15;
    const uint32_t dist = ((fd >> 8) & 0xffff) + ((uint32_t)(v2 >> l2) & ((1u << xd) - 1));
    if (WRITE) {
      const uint32_t at = o + n;
      if ((uint64_t)dist > pos0 + at) { fl = F_BAD; break; }   // too far back (inflate's "invalid distance")
      const uint32_t sb = at + PBIAS - dist;
      uint32_t k = 0;
      for (uint32_t j = 0; j < length; j++) {
        st_ws(res + at + j, sb + k);
        if (++k == dist) k = 0;
      }
    }
    n += length;
    const uint32_t used = l1 + xl + l2 + xd;
    r += used;
    v >>= used;
    vb -= used;
  }
  e = r;
}

// A Huffman region: P.q0 (a symbol start, bits into the call's input) ..
// P.qlim; output from P.pos0 (absolute), at most P.room bytes.  Every thread
// of the workgroup calls it; results in P.R (bytes) and P.qn (next symbol).
#ifdef XCG_ZI_TIMING
// diagnostics build: cycles per phase, summed over calls (setup, fast literals,
// fast matches, careful path, flushes, stored copies, tail) and symbol counts
__device__ unsigned long long g_zi_t[16];   // 0-8 decoder phases, 10-15 region phases
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
#ifdef XCG_ZI_TIMING
#define RT_ADD(i, t0)                                                         \
  do {                                                                        \
    uint64_t t1_ = ZT_NOW();                                                  \
    if (threadIdx.x == 0) atomicAdd(&g_zi_t[10 + (i)], (unsigned long long)(t1_ - (t0))); \
    t0 = t1_;                                                                 \
  } while (0)
#else
#define RT_ADD(i, t0) (void)(t0)
#endif

// region statistics (xcg_debug_zinflate_regions): regions, fixed-point
// iterations, bytes committed, resolve rounds
__device__ unsigned long long g_zi_reg[4];

template <int NW>
__device__ void region(Lds& L, ParT<NW>& P, const uint8_t* I, uint8_t* out, const uint8_t* hist, uint64_t total0,
                       uint32_t* res, const uint32_t WARM, const uint32_t maxthr) {
  constexpr int NT = 64 * NW;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint64_t rt = ZT_NOW();
  const uint64_t q0 = P.q0, pos0 = P.pos0;
  const uint64_t b0 = (q0 >> 3) & ~7ull;
  const uint32_t r0 = (uint32_t)(q0 - 8 * b0), rl = (uint32_t)(P.qlim - 8 * b0);
  const uint32_t nwd = (rl >> 6) + 4;
  for (uint32_t k = t; k < nwd; k += NT) P.stg[k] = *(const uint64_t*)(I + b0 + 8ull * k);
  for (int i = t; i < (1 << LTree::BITS); i += NT) {
    const uint32_t e = L.lt.pri[i];
    P.flt[i] = (e & 15) ? lfast(e) : 0;
  }
  for (int i = t; i < (1 << DTree::BITS); i += NT) {
    const uint32_t e = L.dt.pri[i];
    P.fdt[i] = (e & 15) ? dfast(e) : 0;
  }
  const uint32_t span = rl - r0;
  const uint32_t nact = max(1u, min(min((uint32_t)NT, maxthr), span / SMIN));
  const uint32_t S = span / nact;
  if (t == 0) {
    P.any[0] = P.any[1] = 0;
    P.f = nact;
    P.f2 = P.f3 = 0xffffffffu;
  }
  __syncthreads();
  const bool act = (uint32_t)t < nact;
  const uint32_t lim = (uint32_t)t + 1 == nact ? rl : r0 + ((uint32_t)t + 1) * S;
  uint32_t s = r0 + (uint32_t)t * S, e = 0, n = 0, fl = 0;
  RT_ADD(0, rt);
  // Warm-up: a thread first decodes the WARM bits before its range and starts
  // at the first symbol boundary that decode reaches inside its range.  A
  // decode from a wrong bit usually falls onto the true symbol boundaries
  // within ~100 bits, so most threads start on the true path at once.
  if (act) {
    if (t > 0) {
      const uint32_t ws = s - r0 > WARM ? s - WARM : r0;
      spec<false, NW>(L, P, ws, s, e, n, fl, nullptr, 0, 0);
      if (!fl) s = e;
    }
    spec<false, NW>(L, P, s, lim, e, n, fl, nullptr, 0, 0);
    P.st[t] = s;
    P.endp[t] = e;
    P.cnt[t] = n;
    P.flag[t] = (uint8_t)fl;
  }
  // Fixed point of the starts: a thread whose predecessor's end differs from
  // its start decodes again from that end.  The (few) threads that move are
  // listed and re-decoded by the first threads of the workgroup, so a pass
  // costs the waves it needs, not all sixteen.
  int iters = 1;
  for (int it = 0;; it++) {
    if (t == 0) {
      P.nd = 0;
      P.chg[it & 1] = NT;
      P.fm[it & 1] = NT;
    }
    __syncthreads();
    // a thread behind a stopped one keeps its start: if the stop is real (an
    // end of block on the true path) nothing after it commits, and if not,
    // the stopped thread's own start moves and it reports a new end later
    // (without this an end of block would walk one thread per pass)
    if (act && t > 0 && !P.flag[t - 1]) {
      const uint32_t ns = P.endp[t - 1];
      if (ns != P.st[t]) {
        P.nst[t] = ns;
        P.list[atomicAdd(&P.nd, 1u)] = (uint16_t)t;
        atomicMin(&P.chg[it & 1], (uint32_t)t);
      }
    }
    if (act && P.flag[t]) atomicMin(&P.fm[it & 1], (uint32_t)t);
    __syncthreads();
    // done when no start moved, or when the first stopped thread lies before
    // the first moved one (every start up to it is final; what follows it
    // never commits)
    const uint32_t chg = P.chg[it & 1], fm = P.fm[it & 1];
    if (chg >= (uint32_t)NT || fm < chg) break;
    iters++;
    const uint32_t nd = P.nd;
    for (uint32_t k = t; k < nd; k += NT) {
      const uint32_t u = P.list[k];
      const uint32_t su0 = P.nst[u], lu = u + 1 == nact ? rl : r0 + (u + 1) * S;
      uint32_t eu, nu, fu;
      spec<false, NW>(L, P, su0, lu, eu, nu, fu, nullptr, 0, 0);
      P.st[u] = su0;
      P.endp[u] = eu;
      P.cnt[u] = nu;
      P.flag[u] = (uint8_t)fu;
    }
    __syncthreads();
  }
  RT_ADD(1, rt);
  if (t == 0) {
    atomicAdd(&g_zi_reg[0], 1ull);
    atomicAdd(&g_zi_reg[1], (unsigned long long)iters);
  }
  // Threads before the first stopped one commit, and that one too up to its
  // stop (an end of block or an invalid code on the true path: its bytes
  // before it are the decoder's): wave 0 resumes at the stopping symbol.
  const uint32_t fstop = min(P.fm[(iters - 1) & 1], nact);
  uint32_t f = fstop < nact ? fstop + 1 : nact;
  if (act) {
    s = P.st[t];
    n = P.cnt[t];
  }
  // exclusive offsets of the committed threads' bytes
  const uint32_t v = (uint32_t)t < f ? n : 0;
  uint32_t x = wave_incl_scan(v);
  if (lane == 63) P.wsum[wid] = x;
  __syncthreads();
  for (int w = 0; w < wid; w++) x += P.wsum[w];
  P.incl[t] = x;
  const uint64_t cap = P.room < RES_CAP ? P.room : RES_CAP;
  if ((uint32_t)t < f && x > cap) atomicMin(&P.f2, (uint32_t)t);
  __syncthreads();
  f = min(f, P.f2);
  RT_ADD(2, rt);
  if ((uint32_t)t < f) {
    uint32_t e2, n2, fl2;
    spec<true, NW>(L, P, s, lim, e2, n2, fl2, res, x - v, pos0);
    if (fl2 & F_BAD) atomicMin(&P.f3, (uint32_t)t);
  }
  __syncthreads();
  f = min(f, P.f3);
  RT_ADD(3, rt);
  const uint32_t R = f ? P.incl[f - 1] : 0;
  const uint32_t qn = f ? P.endp[f - 1] : r0;
  // resolve: every slot to its byte (pointer jumping; sources lie before the slot)
  for (int it = 0;; it++) {
    if (t == 0) P.any[it & 1] = 0;
    __syncthreads();
    bool more = false;
    for (uint32_t i = t; i < R; i += NT) {
      const uint32_t y = ld_ws(res + i);
      if (y & RES_FLAG) continue;
      const int32_t src = (int32_t)(y - PBIAS);
      uint32_t w;
      if (src < 0) {
        const uint64_t ab = pos0 - (uint64_t)(-(int64_t)src);
        w = RES_FLAG | (ab >= total0 ? out[ab - total0] : hist[WSIZE - (total0 - ab)]);
      } else {
        w = ld_ws(res + src);
        more |= !(w & RES_FLAG);
      }
      st_ws(res + i, w);
    }
    if (more) P.any[it & 1] = 1;
    __syncthreads();
    if (t == 0) atomicAdd(&g_zi_reg[3], 1ull);
    if (!P.any[it & 1]) break;
  }
  RT_ADD(4, rt);
  if (t == 0) atomicAdd(&g_zi_reg[2], (unsigned long long)R);
  const uint64_t pos1 = pos0 + R;
  uint8_t* o = out + (pos0 - total0);
  for (uint32_t i = t; i < R; i += NT) o[i] = (uint8_t)ld_ws(res + i);
  const uint64_t lo = pos1 - pos0 > RMASK + 1 ? pos1 - (RMASK + 1) : pos0;
  for (uint64_t p = lo + t; p < pos1; p += NT) L.ring[p & RMASK] = (uint8_t)ld_ws(res + (p - pos0));
  if (t == 0) {
    P.R = R;
    P.qn = 8 * b0 + qn;
    P.stopped = fstop < nact && f > fstop;   // resumes at the stopping symbol
  }
  __threadfence();   // the region's bytes are read back by later far matches
  __syncthreads();
  RT_ADD(5, rt);
}

// A stored block's bytes straight to the output, the last 4 KiB also into the ring.
template <int NW>
__device__ void stored_copy(Lds& L, ParT<NW>& P, const uint8_t* I, uint8_t* out, uint64_t total0) {
  constexpr int NT = 64 * NW;
  const int t = threadIdx.x;
  const uint64_t n = P.n, pos = P.pos0;
  const uint8_t* src = I + P.soff;
  uint8_t* dst = out + (pos - total0);
  // 16 bytes per thread and step (unaligned vector access), the tail bytewise
  const uint64_t nv = n / 16;
  for (uint64_t i = t; i < nv; i += NT) *(u32x4_u*)(dst + 16 * i) = *(const u32x4_u*)(src + 16 * i);
  for (uint64_t i = 16 * nv + t; i < n; i += NT) dst[i] = src[i];
  const uint64_t keep = n < (uint64_t)(RMASK + 1) ? n : (uint64_t)(RMASK + 1);
  for (uint64_t i = t; i < keep; i += NT) L.ring[(pos + n - keep + i) & RMASK] = src[n - keep + i];
  __threadfence();
  __syncthreads();
}


// NW = 1: one wave per call (batches of many streams).  NW > 1: one workgroup
// per call, wave 0 decoding, the workgroup on Huffman regions and stored
// copies (region(), stored_copy()) -- the per-call path.
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4))) void zi_inflate_kernel(IArgs a) {
#ifdef XCG_ZI_TIMING
  uint64_t zt[10] = {0};
#endif
  uint64_t tz = ZT_NOW();
  __shared__ Lds L;
  __shared__ ParT<NW> P;
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
  const uint8_t* hist = a.hist + (uint64_t)c.stream * WSIZE;
  uint64_t pos = total0, flushed = total0;
  int32_t status = 0;
  uint32_t trailer = 0, have_trailer = 0;
  uint8_t* out = a.out + c.out_off;
  uint32_t* res = NW > 1 ? a.pres + (uint64_t)ci * RES_CAP : nullptr;
  bool do_hist = false;
  uint64_t ol = 0;
  if (NW > 1 && threadIdx.x >= 64) {   // helper waves: regions and copies until wave 0 is done
    if constexpr (NW > 1) {
      for (;;) {
        __syncthreads();
        const uint32_t cmd = P.cmd;
        if (cmd == 0) break;
        if (cmd == 1) region<NW>(L, P, R.I, out, hist, total0, res, a.warm, a.maxthr);
        else stored_copy<NW>(L, P, R.I, out, total0);
      }
    }
  } else {
  R.load(0);
  // history -> ring
  // (16 bytes per lane and step, every step's load issued before its stores:
  // one memory latency per 1 KiB instead of one per 64 bytes)
  const uint64_t hn = total0 < (uint64_t)(RMASK + 1) ? total0 : (uint64_t)(RMASK + 1);
  for (uint64_t i0 = 0; i0 < hn; i0 += 1024) {
    const uint64_t i = i0 + 16 * (uint64_t)lane;
    const uint8_t* src = hist + (WSIZE - hn + i);
    if (i + 16 <= hn) {
      const u32x4 w = *(const u32x4_u*)src;
      const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 16; k++) L.ring[(total0 - hn + i + k) & RMASK] = (uint8_t)(ww[k >> 2] >> (8 * (k & 3)));
    } else {
      for (uint64_t k = i; k < hn; k++) L.ring[(total0 - hn + k) & RMASK] = hist[WSIZE - hn + k];
    }
  }
  auto flush = [&]() {
    wsync<NW>();
    for (uint64_t p = flushed + lane; p < pos; p += 64) out[p - total0] = L.ring[p & RMASK];
    flushed = pos;
    __threadfence();   // the flushed bytes are read back by far matches
  };
  // the workgroup's turn (NW > 1): P's parameters set by lane 0, then every
  // wave runs the command
  auto help = [&](uint32_t cmd) {
    if constexpr (NW > 1) {
      if (lane == 0) P.cmd = cmd;
      __syncthreads();
      if (cmd == 1) region<NW>(L, P, R.I, out, hist, total0, res, a.warm, a.maxthr);
      else stored_copy<NW>(L, P, R.I, out, total0);
    }
  };
  bool par_ok = true;   // a region may help in this Huffman block
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
      wsync<NW>();
      build<NW>(L, L.lt, L.lens, 288);
      for (int i = lane; i < 30; i += 64) L.lens[i] = 5;
      wsync<NW>();
      build<NW>(L, L.dt, L.lens, 30);
      return true;
    }
    bool ok = build<NW>(L, L.lt, L.dlens, nlen);
    ok = build<NW>(L, L.dt, L.dlens + nlen, ndist) && ok;
    return ok;
  };
  ZT_ADD(0, tz);
  if (mode == M_HUFF) {   // resume inside a block: rebuild its trees
    for (int i = lane; i < 320; i += 64) L.dlens[i] = sp->lens[i];
    wsync<NW>();
    if (!tables_for_block()) mode = M_ERROR;
  }
  wsync<NW>();
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
      ZT_ADD(3, tz);
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
        par_ok = true;
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
        wsync<NW>();
        {   // 3 bits per code-length code length, all 19 within one 64-bit read
          const uint64_t cv = R.get(q);
          if (lane < (int)ncl) L.lens[CL_ORDER[lane]] = (uint8_t)((cv >> (3 * lane)) & 7);
          q += 3 * ncl;
        }
        wsync<NW>();
        if (!build<NW>(L, L.ct, L.lens, 19)) { mode = M_ERROR; break; }
        // the code-length code's 128-entry table (codes of at most 7 bits: no
        // canonical path) in one register, two entries per lane, read with
        // v_readlane instead of an LDS round trip per symbol
        const uint32_t ctw = ((uint32_t)L.ct.pri[2 * lane + 1] << 16) | L.ct.pri[2 * lane];
        ZT_ADD(7, tz);
        // the literal/length and distance code lengths, with repeats; the bits
        // come from a 64-bit buffer refilled when fewer than a code (7) and
        // its extra bits (7) remain
        bool bad = false;
        if constexpr (NW > 1) {   // (the one-wave kernel keeps it inline: the call costs it 20 %)
          int cr = cl_spec<NW>(L, (uint32_t*)P.stg, R.I, q, qend, nlen + ndist);
          if (cr == 3) cr = cl_sequence(L, R.I, q, qend, nlen + ndist, ctw);
          if (cr == 2) bad = true;
          else if (cr == 1) stall = true;
        } else {
          uint32_t n = 0, prev = 0;
          uint64_t b = 0;
          uint32_t bb = 0;
          while (n < nlen + ndist) {
            if (q >= qend) { stall = true; break; }
            if (bb < 14) {
              b = R.get(q);
              bb = 64;
            }
            const uint32_t ci = (uint32_t)b & 127;
            const uint32_t e = (readlane(ctw, (int)(ci >> 1)) >> (16 * (ci & 1))) & 0xffff;
            uint32_t cl = e & 15, sym = e >> 4;
            if (!e || q + cl > qend) { if (!e) bad = true; else stall = true; break; }
            if (sym < 16) {
              q += cl;
              b >>= cl;
              bb -= cl;
              if (lane == 0) L.dlens[n] = (uint8_t)sym;
              prev = sym;
              n++;
              continue;
            }
            uint32_t rep, val = 0, xb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
            if (q + cl + xb > qend) { stall = true; break; }
            uint32_t x = (uint32_t)(b >> cl) & ((1u << xb) - 1);
            if (sym == 16) {
              if (n == 0) { bad = true; break; }
              val = prev;
              rep = 3 + x;
            } else rep = (sym == 17 ? 3 : 11) + x;
            if (n + rep > nlen + ndist) { bad = true; break; }
            for (uint32_t r = lane; r < rep; r += 64) L.dlens[n + r] = (uint8_t)val;
            prev = val;
            n += rep;
            q += cl + xb;
            b >>= cl + xb;
            bb -= cl + xb;
          }
        }
        ZT_ADD(9, tz);
        if (bad) { mode = M_ERROR; break; }
        if (stall) { q = q0; break; }
        wsync<NW>();
        if (L.dlens[256] == 0 || !tables_for_block()) { mode = M_ERROR; break; }
        mode = M_HUFF;   // (its lengths reach sp->lens only when the call commits)
        par_ok = true;
        ZT_ADD(7, tz);
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
      if constexpr (NW > 1) {
        if (lane == 0) {
          P.n = n;
          P.pos0 = pos;
          P.soff = q >> 3;
        }
        help(2);
      } else {
        const uint8_t* src = R.I + (q >> 3);
        uint8_t* dst = out + (pos - total0);
        for (uint64_t i = lane; i < n; i += 64) dst[i] = src[i];
        const uint64_t keep = n < (uint64_t)(RMASK + 1) ? n : (uint64_t)(RMASK + 1);
        for (uint64_t i = lane; i < keep; i += 64) L.ring[(pos + n - keep + i) & RMASK] = src[n - keep + i];
      }
      pos += n;
      flushed = pos;
      __threadfence();   // readable by far matches
      wsync<NW>();
      q += 8 * n;
      ZT_ADD(5, tz);
      stored_left -= (uint32_t)n;
      if (stored_left) { stall = true; break; }
      mode = last ? M_TRAILER : M_BLOCK;
      R.load(q >> 3);
    } else if (mode == M_HUFF) {
      for (;;) {
        if constexpr (NW > 1) {   // the workgroup on the block's middle
          const uint64_t qlim = qend > 128 ? qend - 128 : 0;
          if (par_ok && q + PAR_MIN_BITS <= qlim && pos - total0 < c.out_cap) {
            ZT_ADD(3, tz);
            flush();
            if (lane == 0) {
              P.q0 = q;
              P.qlim = qlim - q > 8ull * ParT<NW>::INC ? q + 8ull * ParT<NW>::INC : qlim;
              P.pos0 = pos;
              P.room = c.out_cap - (pos - total0);
            }
            help(1);
            const uint32_t rn = su(P.R);
            const uint64_t qn = ((uint64_t)su((uint32_t)(P.qn >> 32)) << 32) | su((uint32_t)P.qn);
            ZT_ADD(8, tz);
            // the block ends (or fails) at the region's end, or within its first
            // thread's range: the careful path takes it from here
            if (!rn || su(P.stopped)) par_ok = false;
            pos += rn;
            flushed = pos;
            q = qn;
            R.load(q >> 3);
            continue;
          }
        }
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
        wsync<NW>();
        copy_match(dist, length);
        wsync<NW>();
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
  wsync<NW>();
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
      do_hist = true;
      ol = pos - total0;
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
  if constexpr (NW > 1) {   // release the helper waves for the history update
    if (lane == 0) {
      P.t_do = do_hist;
      P.t_ol = ol;
      P.cmd = 0;
    }
    __syncthreads();
  }
  }   // wave 0 (every wave when NW == 1)
  // history = the last 32 KiB of output: the old history moved down by this
  // call's output length, then the output itself (flushed and fenced above)
  {
    constexpr int NT = 64 * NW;
    const int t = threadIdx.x;
    if constexpr (NW > 1) {
      do_hist = P.t_do;
      ol = P.t_ol;
    }
    uint8_t* h = a.hist + (uint64_t)c.stream * WSIZE;
    if (do_hist) {
      if (ol < (uint64_t)WSIZE) {
        constexpr int PER = NW > 1 ? WSIZE / NT : 16;   // bytes per thread and pass: read, then write
        for (uint64_t i0 = 0; ol && i0 < WSIZE - ol; i0 += (uint64_t)NT * PER) {
          uint8_t b[PER];
#pragma unroll
          for (int k = 0; k < PER; k++) {
            const uint64_t i = i0 + (uint64_t)k * NT + t;
            b[k] = i < WSIZE - ol ? h[i + ol] : 0;
          }
          __syncthreads();
#pragma unroll
          for (int k = 0; k < PER; k++) {
            const uint64_t i = i0 + (uint64_t)k * NT + t;
            if (i < WSIZE - ol) h[i] = b[k];
          }
        }
        for (uint64_t i = t; i < ol; i += NT) h[WSIZE - ol + i] = out[i];
      } else {
        for (uint64_t i = t; i < (uint64_t)WSIZE; i += NT) h[i] = out[ol - WSIZE + i];
      }
    }
  }
  ZT_ADD(6, tz);
#ifdef XCG_ZI_TIMING
  if (lane == 0)
    for (int i = 0; i < 10; i++) atomicAdd(&g_zi_t[i], (unsigned long long)zt[i]);
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
template <int AW>
__global__ __launch_bounds__(64 * AW) void zi_adler_kernel(IArgs a) {
  constexpr int AT = 64 * AW;
  __shared__ uint64_t red[2][AW];
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
    for (uint64_t w = t; w < words; w += AT) {
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
    for (uint64_t i = 4 * words + t; i < n; i += AT) {
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
    uint64_t A = 0, B = 0;
    for (int w = 0; w < AW; w++) {
      A += red[0][w];
      B += red[1][w];
    }
    A %= 65521u;
    B %= 65521u;
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
int g_zi_par = 0;                    // 0: by batch size, 1: a wave per call, 2: a workgroup per call
uint32_t g_zi_warm = xcg::zi::WARM_DEFAULT, g_zi_threads = 1024;   // region shape (A/B runs)
// A workgroup per call up to this many calls: per call (1024 threads) it is
// 13x faster on Huffman data; batched (256 threads, four calls per CU), 2.6x on
// text and 1.8x on stored blocks (profiles/r06_zinflate_modes.txt).  Beyond it
// the 256 KiB of resolve scratch per call is not worth holding.
constexpr uint32_t ZI_PAR_CALLS = 4096;
constexpr uint32_t ZI_QUARTER_CALLS = 256;
}  // namespace

extern "C" {

int xcg_zinflate_create(int device, uint32_t nstreams, xcg_zinflate** out) {
  if (!out || nstreams == 0) return XCG_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return XCG_EHIP;
  if (const char* m = getenv("XCG_ZINFLATE_MODE")) g_zi_par = atoi(m) & 3;   // A/B runs (xcg_debug_set_zinflate_mode)
  if (const char* m = getenv("XCG_ZI_WARM")) g_zi_warm = (uint32_t)atoi(m);
  if (const char* m = getenv("XCG_ZI_THREADS")) g_zi_threads = std::max(64, std::min(1024, atoi(m)));
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
  // few calls: a workgroup per call (zi_inflate_kernel<16>) with RES_CAP
  // resolve slots each; many: a wave per call
  const bool par = g_zi_par >= 2 || (g_zi_par == 0 && n <= ZI_PAR_CALLS);
  // quarter workgroups (four calls per CU: one call's serial stretches overlap
  // the others') once the batch fills the CUs
  const bool quarter = g_zi_par == 3 || (g_zi_par == 0 && n > ZI_QUARTER_CALLS);
  size_t o_I = 0, o_res = ial(io, 256), o_pres = ial(o_res + sizeof(IRes) * n, 256),
         o_end = par ? o_pres + 4ull * RES_CAP * n : o_pres;
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
  a.pres = par ? (uint32_t*)(z->scratch + o_pres) : nullptr;
  a.warm = g_zi_warm;
  a.maxthr = g_zi_threads;
  uint32_t tiles = std::min<uint32_t>(64, (PEND_CAP + maxlen + IPAD + 4095) / 4096);   // 4 KiB per block
  hipLaunchKernelGGL(zi_prep_kernel, dim3(tiles, n), dim3(256), 0, st, a);
  if (par && quarter) hipLaunchKernelGGL(zi_inflate_kernel<4>, dim3(n), dim3(256), 0, st, a);
  else if (par) hipLaunchKernelGGL(zi_inflate_kernel<16>, dim3(n), dim3(1024), 0, st, a);
  else hipLaunchKernelGGL(zi_inflate_kernel<1>, dim3(n), dim3(64), 0, st, a);
  if (par) hipLaunchKernelGGL(zi_adler_kernel<16>, dim3(n), dim3(1024), 0, st, a);
  else hipLaunchKernelGGL(zi_adler_kernel<4>, dim3(n), dim3(256), 0, st, a);
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

int xcg_debug_zinflate_regions(uint64_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zi_reg), 8 * 4) != hipSuccess) return XCG_EHIP;
  uint64_t z[4] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_zi_reg), z, sizeof z) == hipSuccess ? XCG_OK : XCG_EHIP;
}

int xcg_debug_set_zinflate_mode(int mode) {
  if (mode < 0 || mode > 3) return XCG_EINVAL;
  g_zi_par = mode;
  return XCG_OK;
}

#ifdef XCG_ZI_TIMING
int xcg_debug_zi_times(uint64_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_zi_t), 8 * 16) != hipSuccess) return XCG_EHIP;
  uint64_t z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_zi_t), z, sizeof z) == hipSuccess ? XCG_OK : XCG_EHIP;
}
#endif

}  // extern "C"
