// Level 0 of wanproxy's zlib stage: zlib 1.2.11's deflate() + deflate_stored
// control flow in DeflatePipe::consume's call pattern (zlib/deflate_pipe.cc:
// 57-115), over lengths only.  Host code shared by the engine
// (xcg_deflate.hip: the GPU moves the bytes the plan names) and its CPU test
// (tests/test_zlib_oracle.py runs the plan through oracle/stored_plan_harness.cc
// and checks it against the system zlib).
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

namespace xcg {
namespace zd {

struct ZPiece {
  uint64_t out;          // offset in the call's output
  uint64_t src;          // kind 1: stream position; kind 0: the header bytes (little-endian, <= 5)
  uint32_t len, kind;    // kind 0 literal bytes, 1 stream bytes, 2 adler32 trailer (big-endian)
  uint32_t call, pad;
};

// zlib's z_stream + deflate_state at level 0, lengths only.
struct StoredPlan {
  enum { INIT = 0, BUSY = 1, FINISHED = 2 };
  enum { NEED_MORE, BLOCK_DONE, FINISH_STARTED, FINISH_DONE };
  int status = INIT, last_flush = 0;   // (deflateReset: last_flush = Z_NO_FLUSH)
  bool trailer = false;                // wrap < 0: the trailer was written
  uint32_t strstart = 0, block_start = 0;   // window coordinates
  uint64_t wbase = 0;                  // stream position of window coordinate 0
  uint64_t pend = 0;                   // bytes zlib holds in its pending buffer
  // the current deflate() call
  uint64_t next_in = 0;                // stream position of next_in
  uint32_t avail_in = 0, avail_out = 0;
  // the current consume's output
  std::vector<ZPiece>* pieces = nullptr;
  uint64_t produced = 0;               // stream bytes this consume made
  uint64_t copied = 0;                 // bytes copied to the pipe's buffer (delivered)

  static int rank(int f) { return f * 2 - (f > 4 ? 9 : 0); }
  void emit_lit(uint64_t v, uint32_t n) {
    pieces->push_back(ZPiece{produced, v, n, 0u, 0u, 0u});
    produced += n;
  }
  void emit_stream(uint64_t pos, uint32_t n) {
    if (n) pieces->push_back(ZPiece{produced, pos, n, 1u, 0u, 0u});
    produced += n;
  }
  void flush_pending() {
    const uint64_t k = pend < avail_out ? pend : avail_out;
    pend -= k;
    avail_out -= (uint32_t)k;
    copied += k;
  }
  void stored_header(uint32_t len, bool last) {   // _tr_stored_block's 3 bits + windup + LEN / NLEN
    const uint32_t nlen = ~len & 0xffffu;
    emit_lit((last ? 1u : 0u) | (uint64_t)(len & 0xffff) << 8 | (uint64_t)nlen << 24, 5);
  }
  // deflate_stored (zlib 1.2.11)
  int stored(int flush) {
    const uint32_t MAX_STORED = 65535, w_size = 32768u, window_size = 2 * 32768u;
    uint32_t min_block = std::min<uint32_t>(65536 - 5, w_size);
    uint32_t len, left, have;
    bool last = false;
    uint32_t used = avail_in;
    do {
      len = MAX_STORED;
      have = 5;                                          // (bi_valid + 42) >> 3; bi_valid is 0 at level 0
      if (avail_out < have) break;
      have = avail_out - have;
      left = strstart - block_start;
      if ((uint64_t)len > (uint64_t)left + avail_in) len = left + avail_in;
      if (len > have) len = have;
      if (len < min_block && ((len == 0 && flush != 4) || flush == 0 || len != left + avail_in)) break;
      last = flush == 4 && len == left + avail_in;
      stored_header(len, last);                          // into pending, then flushed (pending was empty)
      pend += 5;
      flush_pending();
      if (left) {                                        // from the window, straight to next_out
        if (left > len) left = len;
        emit_stream(wbase + block_start, left);
        avail_out -= left;
        copied += left;
        block_start += left;
        len -= left;
      }
      if (len) {                                         // straight from next_in
        emit_stream(next_in, len);
        next_in += len;
        avail_in -= len;
        avail_out -= len;
        copied += len;
      }
    } while (!last);
    used -= avail_in;
    if (used) {                                          // the window keeps the copied data
      if (used >= w_size) {
        wbase = next_in - w_size;
        strstart = w_size;
      } else {
        if (window_size - strstart <= used) {
          strstart -= w_size;
          wbase += w_size;
        }
        strstart += used;
      }
      block_start = strstart;
    }
    if (last) return FINISH_DONE;
    if (flush != 0 && flush != 4 && avail_in == 0 && strstart == block_start) return BLOCK_DONE;
    have = window_size - strstart - 1;                   // fill the window with the rest of the input
    if (avail_in > have && block_start >= w_size) {
      block_start -= w_size;
      strstart -= w_size;
      wbase += w_size;
      have += w_size;
    }
    if (have > avail_in) have = avail_in;
    if (have) {
      next_in += have;
      avail_in -= have;
      strstart += have;
    }
    have = std::min<uint32_t>(65536 - 5, MAX_STORED);    // a stored block in the pending buffer
    min_block = std::min<uint32_t>(have, w_size);
    left = strstart - block_start;
    if (left >= min_block || ((left || flush == 4) && flush != 0 && avail_in == 0 && left <= have)) {
      len = left < have ? left : have;
      last = flush == 4 && avail_in == 0 && len == left;
      stored_header(len, last);
      emit_stream(wbase + block_start, len);
      pend += 5 + len;
      block_start += len;
      flush_pending();
    }
    return last ? FINISH_STARTED : NEED_MORE;
  }
  // deflate() (zlib 1.2.11) at level 0, zlib wrapper; flush 0 NO_FLUSH, 2 SYNC_FLUSH, 4 FINISH.
  // Returns 0 Z_OK, 1 Z_STREAM_END, -5 Z_BUF_ERROR.
  int deflate(int flush) {
    if (avail_out == 0) return -5;
    const int old_flush = last_flush;
    last_flush = flush;
    if (pend) {
      flush_pending();
      if (avail_out == 0) {
        last_flush = -1;
        return 0;
      }
    } else if (avail_in == 0 && rank(flush) <= rank(old_flush) && flush != 4) {
      return -5;
    }
    if (status == FINISHED && avail_in != 0) return -5;
    if (status == INIT) {                                // zlib header, level_flags 0
      uint32_t header = (8 + (7 << 4)) << 8;
      header += 31 - (header % 31);
      emit_lit((header >> 8) | (header & 0xff) << 8, 2);
      pend += 2;
      status = BUSY;
      flush_pending();
      if (pend) {
        last_flush = -1;
        return 0;
      }
    }
    if (avail_in != 0 || (flush != 0 && status != FINISHED)) {
      const int b = stored(flush);
      if (b == FINISH_STARTED || b == FINISH_DONE) status = FINISHED;
      if (b == NEED_MORE || b == FINISH_STARTED) {
        if (avail_out == 0) last_flush = -1;
        return 0;
      }
      if (b == BLOCK_DONE) {                            // Z_SYNC_FLUSH: the empty stored block
        stored_header(0, false);
        pend += 5;
        flush_pending();
        if (avail_out == 0) {
          last_flush = -1;
          return 0;
        }
      }
    }
    if (flush != 4) return 0;
    if (trailer) return 1;
    pieces->push_back(ZPiece{produced, 0, 4, 2u, 0u, 0u});   // adler32, big-endian
    produced += 4;
    pend += 4;
    flush_pending();
    trailer = true;
    return pend ? 0 : 1;
  }
  // DeflatePipe::consume (deflate_pipe.cc:57-115) of n bytes cut into seg[0..nseg)
  // (n == 0: EOS).  Appends the call's pieces; returns false on a zlib error.
  bool consume(uint64_t n, const uint32_t* seg, uint32_t nseg, std::vector<ZPiece>& out, uint64_t* made,
               uint64_t* deliver) {
    pieces = &out;
    produced = copied = 0;
    if (status == FINISHED) return false;                // (a consume after EOS: zlib refuses more input)
    uint64_t done_in = 0, soff = 0;
    uint32_t si = 0, stalls = 0;
    bool first = true;
    avail_out = 65536;
    for (;;) {
      int flush;
      uint64_t slen = 0;
      if (done_in == n) {
        flush = first ? 4 : 2;
        avail_in = 0;
      } else {
        if (seg) {
          while (si < nseg && seg[si] == soff) { si++; soff = 0; }
          if (si == nseg) return false;
          slen = seg[si] - soff;
        } else {
          slen = n - done_in < 2048 ? n - done_in : 2048;
        }
        flush = 0;
        first = false;
        avail_in = (uint32_t)slen;
      }
      for (;;) {
        const int e = deflate(flush);
        if (e == 0 && avail_out > 0 && flush == 0) break;
        avail_out = 65536;                               // out.append(outbuf, ...), fresh buffer
        if (flush == 0) break;
        if ((flush == 2 && e == 0) || (flush == 4 && e == 1)) {
          *made = produced;
          *deliver = copied;
          return true;
        }
        if (e != 0 && e != -5) return false;
      }
      if (slen) {
        const uint64_t used = slen - avail_in;
        if (used == 0 && ++stalls > 2) return false;     // (no progress: not a state zlib reaches)
        done_in += used;
        soff += used;
        if (seg && soff == seg[si]) { si++; soff = 0; }
      }
    }
  }
};

}  // namespace zd
}  // namespace xcg
