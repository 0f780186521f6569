// TEST INFRASTRUCTURE ONLY: a C driver around wanproxy's zlib pipes, built two
// ways by oracle/Makefile from the reference's own sources:
//   _ref/libzpref.so     zlib/deflate_pipe.cc + zlib/inflate_pipe.cc (the real
//                        reference over the system zlib 1.2.11)
//   _ref/libzpdropin.so  integration/zlib_pipes_xcgpu.cc (the MI355X drop-in
//                        bodies of the same classes, over libxcgpu.so)
// Both link the reference's PipeProducer (io/pipe/pipe_producer.cc) and Buffer.
// consume() is private in DeflatePipe / InflatePipe and produce() parks bytes
// in PipeProducer's private output_buffer_; this harness opens both up to call
// the pipe directly (Pipe::input would need the event system's scheduler).
#include <stdint.h>
#include <string.h>

#include <common/buffer.h>
#include <common/thread/mutex.h>
#include <event/event_callback.h>
#include <io/pipe/pipe.h>
#define private public
#define protected public
#include <io/pipe/pipe_producer.h>
#include <zlib/deflate_pipe.h>
#include <zlib/inflate_pipe.h>
#undef private
#undef protected

extern "C" {

void* zp_new(int kind, int level) {
  if (kind == 0) return static_cast<PipeProducer*>(new DeflatePipe(level));
  return static_cast<PipeProducer*>(new InflatePipe());
}

void zp_free(void* h, int kind) {
  PipeProducer* p = static_cast<PipeProducer*>(h);
  if (kind == 0) delete static_cast<DeflatePipe*>(p);
  else delete static_cast<InflatePipe*>(p);
}

// One consume() of in[0..n) as a Buffer of the given segments (seg NULL:
// Buffer::append's 2048-byte segments).  Returns the bytes produce()d so far
// (moved to out), or -1 if cap is too small; *status: 1 after produce_eos,
// -1 after produce_error, else 0.
int64_t zp_consume(void* h, int kind, const uint8_t* in, uint64_t n, const uint32_t* seg, uint32_t nseg, uint8_t* out,
                   uint64_t cap, int* status) {
  PipeProducer* p = static_cast<PipeProducer*>(h);
  Buffer b;
  if (seg) {
    uint64_t o = 0;
    for (uint32_t i = 0; i < nseg; i++) {
      if (!seg[i]) continue;
      BufferSegment* s = BufferSegment::create(in + o, seg[i]);
      b.append(s);
      s->unref();
      o += seg[i];
    }
  } else if (n) {
    b.append(in, n);
  }
  if (kind == 0) static_cast<DeflatePipe*>(p)->consume(&b);
  else static_cast<InflatePipe*>(p)->consume(&b);
  *status = p->error_ ? -1 : (p->output_eos_ ? 1 : 0);
  const uint64_t len = p->output_buffer_.length();
  if (len > cap) return -1;
  if (len) {
    p->output_buffer_.copyout(out, len);
    p->output_buffer_.clear();
  }
  return (int64_t)len;
}

}  // extern "C"
