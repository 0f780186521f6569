// TEST INFRASTRUCTURE ONLY: runs the engine's level-0 planner
// (wanproxy_amd/csrc/xcg_stored_plan.h, host code the GPU path executes) on
// the CPU and assembles the bytes its pieces name, so tests/test_zlib_oracle.py
// can compare it with the system zlib in DeflatePipe's call pattern
// (oracle/deflate_pipe_ref.c) without a GPU.  The GPU path moves the same
// pieces with zs_copy_kernel.
#include <zlib.h>

#include <deque>

#include "../wanproxy_amd/csrc/xcg_stored_plan.h"

using xcg::zd::StoredPlan;
using xcg::zd::ZPiece;

struct sp_stream {
  StoredPlan plan;
  std::vector<uint8_t> hist;   // the whole stream so far (tests are small)
  uint32_t adler = 1;
  std::deque<uint8_t> held;    // made, not delivered yet
};

extern "C" {

sp_stream* sp_new(void) { return new sp_stream(); }
void sp_free(sp_stream* s) { delete s; }

// One consume: returns the delivered bytes (to out), -1 on error.
int64_t sp_consume(sp_stream* s, const uint8_t* in, uint64_t n, const uint32_t* seg, uint32_t nseg, uint8_t* out,
                   uint64_t cap) {
  std::vector<ZPiece> pieces;
  uint64_t made = 0, deliver = 0;
  const uint64_t total = s->hist.size();
  if (!s->plan.consume(n, seg, nseg, pieces, &made, &deliver)) return -1;
  std::vector<uint8_t> bytes(made);
  s->hist.insert(s->hist.end(), in, in + n);
  if (n) s->adler = (uint32_t)adler32(s->adler, in, (uInt)n);
  for (const ZPiece& p : pieces) {
    if (p.kind == 0) {
      for (uint32_t i = 0; i < p.len; i++) bytes[p.out + i] = (uint8_t)(p.src >> (8 * i));
    } else if (p.kind == 2) {
      for (uint32_t i = 0; i < 4; i++) bytes[p.out + i] = (uint8_t)(s->adler >> (24 - 8 * i));
    } else {
      if (p.src + p.len > s->hist.size() || (total > 65536 && p.src < total - 65536)) return -1;  // (the GPU keeps 64 KiB)
      memcpy(&bytes[p.out], &s->hist[p.src], p.len);
    }
  }
  s->held.insert(s->held.end(), bytes.begin(), bytes.end());
  if (deliver > s->held.size() || deliver > cap) return -1;
  for (uint64_t i = 0; i < deliver; i++) {
    out[i] = s->held.front();
    s->held.pop_front();
  }
  return (int64_t)deliver;
}

}  // extern "C"
