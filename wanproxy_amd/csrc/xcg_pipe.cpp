// XCodecPipePair protocol layer on the MI355X engine (host C++ over the C ABI).
//
// Restates xcodec/xcodec_pipe_pair.cc (encoder_consume :549-642,
// decoder_consume :68-166, decoder_decode :168-433, decoder_decode_data
// :435-547) and the wire ops of xcodec/xcodec_pipe_protocol.h:
//   <HELLO> 0xFF len[u8] uuid[len]     <FRAME> 0x02 len[BE32] data[len]
//   <ASK>   0xF0 count[BE16] hash[BE64 x count]
//   <LEARN> 0xF1 count[BE16] segment[2048 x count]
//   <ADVANCE> 0x01 count[BE32]   <EOS> 0xFC   <EOS_ACK> 0xFB
// Frames carry one XCodecEncoder::encode() call over <= XCODEC_PIPE_MAX_FRAME/2
// input bytes; the encoder keeps, per unacknowledged frame, the segments its
// REFs name (its refmap) to answer <ASK> with <LEARN>; the decoder decodes the
// concatenated frame bytes, asks for unknown hashes, and acknowledges
// finished frames with <ADVANCE>.  The codec work -- every encode and decode --
// runs on the GPU through xcg_encode_host / xcg_decode_host; pipes that share
// an encoder context (one codec, one cache) can be encoded in one GPU batch
// (xcg_pipe_encoder_consume_many), in the order the reference's single event
// thread would have served them.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <memory>
#include <set>
#include <unordered_map>
#include <vector>

#include "../../include/xcgpu.h"

namespace {

constexpr uint8_t OP_HELLO = 0xff, OP_LEARN = 0xf1, OP_ASK = 0xf0, OP_EOS = 0xfc, OP_EOS_ACK = 0xfb,
                  OP_FRAME = 0x02, OP_ADVANCE = 0x01;            // xcodec_pipe_protocol.h:39-118
constexpr uint32_t MAX_FRAME = 1024 * 1024;                     // XCODEC_PIPE_MAX_FRAME, :61
constexpr uint32_t ASK_MAX = 512;                               // XCODEC_PIPE_ASK_MAX, :66
constexpr uint32_t SEG = XCG_SEGMENT_LENGTH;
constexpr uint32_t UUID_LEN = 36;                               // UUID_SIZE, common/uuid/uuid.h:33

void put_be16(std::vector<uint8_t>& o, uint16_t v) { o.push_back(v >> 8); o.push_back(v & 0xff); }
void put_be32(std::vector<uint8_t>& o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o.push_back((v >> s) & 0xff);
}
void put_be64(std::vector<uint8_t>& o, uint64_t v) {
  for (int s = 56; s >= 0; s -= 8) o.push_back((v >> s) & 0xff);
}
uint64_t get_be(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; ++i) v = (v << 8) | p[i];
  return v;
}

// XCodecHash::hash (xcodec/xcodec_hash.h:155-174) of a 2048-byte segment: a
// <LEARN> names no hash, the decoder derives it (xcodec_pipe_pair.cc:306).
uint64_t seg_hash(const uint8_t* d) {
  uint32_t s1 = 0, s2 = 0, b1 = 0, b2 = 0;
  for (uint32_t i = 0; i < SEG; ++i) {
    const uint32_t w = d[i] + 1u, f = d[i] ? (uint32_t)__builtin_ffs(d[i]) : 0u;
    s1 += w; s2 += (SEG - i) * w;
    b1 += f; b2 += (SEG - i) * f;
  }
  const uint64_t bits = (uint32_t)((b1 << 16) + b2), bytes = (uint32_t)((s1 << 20) + s2);
  return (bits << 36) + bytes;
}

bool uuid_ok(const uint8_t* u) {   // the string form UUID::decode accepts (8-4-4-4-12 hex)
  for (uint32_t i = 0; i < UUID_LEN; ++i) {
    const bool dash = i == 8 || i == 13 || i == 18 || i == 23;
    const uint8_t c = u[i];
    if (dash ? c != '-' : !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F')))
      return false;
  }
  return true;
}

// Walk one encoded frame, recording the input offset of every REF: the window
// there equals the segment the REF names (find_reference only emits a REF on
// byte equality, xcodec_encoder.cc:382-390), so the refmap's segments come
// from the frame's own input.
// An out-of-band declaration is written as F1 02 BE64 too (xcodec_encoder.cc:
// 288-295), but encode_declaration passes no refmap: those (hash, input offset)
// pairs -- `decl`, sorted -- are skipped, so an <ASK> for such a hash is a
// protocol error as in the reference (xcodec_pipe_pair.cc:265-267).
void frame_refs(const uint8_t* enc, uint64_t n, const uint8_t* in,
                const std::vector<std::pair<uint64_t, uint64_t>>& decl,
                std::unordered_map<uint64_t, std::vector<uint8_t>>& refmap) {
  uint64_t i = 0, pos = 0;
  while (i < n) {
    if (enc[i] != 0xF1) { ++i; ++pos; continue; }
    const uint8_t op = enc[i + 1];
    if (op == 0x00) { i += 2; ++pos; }                      // escaped 0xF1
    else if (op == 0x01) { i += 2 + SEG; pos += SEG; }      // EXTRACT
    else {                                                  // REF (or out-of-band declaration)
      const uint64_t h = get_be(enc + i + 2, 8);
      const bool is_decl = std::binary_search(decl.begin(), decl.end(), std::make_pair(pos, h));
      if (!is_decl && !refmap.count(h)) refmap.emplace(h, std::vector<uint8_t>(in + pos, in + pos + SEG));
      i += 10;
      pos += SEG;
    }
  }
}

// Decoded size of enc[0..n) if every op resolves (xcodec_decoder.cc:73-185):
// literal and escaped bytes one each, EXTRACT / REF / BACKREF one segment
// each; the walk stops at an incomplete or unknown op, as the decoder does.
uint64_t decoded_bound(const uint8_t* enc, uint64_t n) {
  uint64_t i = 0, out = 0;
  while (i < n) {
    const uint8_t* m = (const uint8_t*)memchr(enc + i, 0xF1, n - i);
    if (!m) return out + (n - i);
    const uint64_t at = (uint64_t)(m - enc);
    out += at - i;
    i = at;
    if (i + 1 >= n) return out;
    const uint8_t op = enc[i + 1];
    if (op == 0x00) { out += 1; i += 2; }                       // escaped 0xF1
    else if (op == 0x01) { out += SEG; i += 2 + SEG; }          // EXTRACT
    else if (op == 0x02) { out += SEG; i += 10; }               // REF
    else if (op == 0x03) { out += SEG; i += 3; }                // BACKREF
    else return out;
  }
  return out;
}

}  // namespace

// (xcg_api.hip) registry contexts a connecting pipe holds while it lives
extern "C" void xcg_registry_hold(xcg_ctx* c);
extern "C" void xcg_registry_release(xcg_ctx* c);

struct xcg_pipe {
  xcg_ctx* enc;
  xcg_ctx* dec;                    // (connecting pipes: set at <HELLO>)
  xcg_ctx* parent = nullptr;       // codec_->cache() of a connecting pipe
  xcg_window* win;                 // the decoder's BACKREF window (one per XCodecDecoder)
  uint8_t uuid[UUID_LEN];
  // encoder side
  bool encoder = false;            // encoder_ != NULL: <HELLO> sent
  bool encoder_sent_eos = false, encoder_sent_eos_ack = false, encoder_produced_eos = false;
  std::deque<std::unordered_map<uint64_t, std::vector<uint8_t>>> ref_frames;   // encoder_reference_frames_
  // decoder side
  bool decoder = false;            // decoder_ != NULL: <HELLO> received
  bool decoder_received_eos = false, decoder_sent_eos = false, decoder_received_eos_ack = false;
  std::vector<uint8_t> dbuf;       // decoder_buffer_
  std::vector<uint8_t> fbuf;       // decoder_frame_buffer_
  std::deque<uint32_t> flens;      // decoder_frame_lengths_
  std::set<uint64_t> unknown;      // decoder_unknown_hashes_
  // this call's outputs
  std::vector<uint8_t> to_peer, to_local;
  int local_eos = 0, peer_eos = 0;

  void begin() {
    to_peer.clear();
    to_local.clear();
    local_eos = peer_eos = 0;
  }
  void finish(xcg_pipe_out* o) const {
    if (!o) return;
    o->to_peer = to_peer.data();
    o->to_peer_len = to_peer.size();
    o->to_local = to_local.data();
    o->to_local_len = to_local.size();
    o->local_eos = local_eos;
    o->peer_eos = peer_eos;
  }
  int decode_ops();
  int decode_data();
};

// decoder_decode (:168-433): process pipe ops until the buffer is empty or an
// op is incomplete.  XCG_EPROTO = decoder_error().
int xcg_pipe::decode_ops() {
  size_t i = 0;
  int rc = XCG_OK;
  while (i < dbuf.size()) {
    const uint8_t* b = dbuf.data() + i;
    const size_t avail = dbuf.size() - i;
    const uint8_t op = b[0];
    if (op == OP_HELLO) {
      if (decoder) { rc = XCG_EPROTO; break; }                       // <HELLO> twice
      if (avail < 2) break;
      const uint8_t len = b[1];
      if (avail < 2u + len) break;
      if (len != UUID_LEN || !uuid_ok(b + 2)) { rc = XCG_EPROTO; break; }
      if (parent) {                                                  // XCodecCache::connect(uuid, codec cache)
        char u[UUID_LEN + 1];
        memcpy(u, b + 2, UUID_LEN);
        u[UUID_LEN] = 0;
        xcg_ctx* c = nullptr;
        rc = xcg_ctx_connect(parent, u, &c);
        if (rc == XCG_OK) rc = xcg_window_create(c, &win);
        if (rc != XCG_OK) break;
        xcg_registry_hold(c);                                        // (until xcg_pipe_destroy)
        dec = c;
      }
      decoder = true;
      i += 2 + len;
    } else if (op == OP_ASK) {
      if (!encoder) { rc = XCG_EPROTO; break; }
      if (avail < 3) break;
      const uint32_t count = (uint32_t)get_be(b + 1, 2);
      if (count == 0 || count > ASK_MAX) { rc = XCG_EPROTO; break; }
      if (avail < 3 + 8ull * count) break;
      std::vector<uint8_t> learn;
      learn.push_back(OP_LEARN);
      put_be16(learn, (uint16_t)count);
      for (uint32_t k = 0; k < count && rc == XCG_OK; ++k) {
        const uint64_t h = get_be(b + 3 + 8 * k, 8);
        if (ref_frames.empty()) { rc = XCG_EPROTO; break; }          // all frames advanced
        bool found = false;
        for (const auto& rm : ref_frames) {
          auto it = rm.find(h);
          if (it == rm.end()) continue;
          learn.insert(learn.end(), it->second.begin(), it->second.end());
          found = true;
          break;
        }
        if (!found) rc = XCG_EPROTO;                                  // in no reference frame
      }
      if (rc != XCG_OK) break;
      to_peer.insert(to_peer.end(), learn.begin(), learn.end());
      i += 3 + 8ull * count;
    } else if (op == OP_LEARN) {
      if (!decoder) { rc = XCG_EPROTO; break; }
      if (avail < 3) break;
      const uint32_t count = (uint32_t)get_be(b + 1, 2);
      if (count == 0 || count > ASK_MAX) { rc = XCG_EPROTO; break; }
      if (avail < 3 + (size_t)SEG * count) break;
      for (uint32_t k = 0; k < count; ++k) {
        const uint8_t* seg = b + 3 + (size_t)SEG * k;
        const uint64_t h = seg_hash(seg);
        if (!unknown.erase(h)) { rc = XCG_EPROTO; break; }           // gratuitous <LEARN>
        // lookup: equal -> redundant; else replace / enter (:311-327)
        const int e = xcg_cache_enter_host(dec, h, seg);
        if (e != XCG_OK) { rc = e; break; }
      }
      if (rc != XCG_OK) break;
      i += 3 + (size_t)SEG * count;
    } else if (op == OP_EOS) {
      if (decoder_received_eos) { rc = XCG_EPROTO; break; }
      decoder_received_eos = true;
      i += 1;
    } else if (op == OP_EOS_ACK) {
      if (!encoder_sent_eos || decoder_received_eos_ack) { rc = XCG_EPROTO; break; }
      decoder_received_eos_ack = true;
      i += 1;
    } else if (op == OP_FRAME) {
      if (!decoder) { rc = XCG_EPROTO; break; }
      if (avail < 5) break;
      const uint32_t len = (uint32_t)get_be(b + 1, 4);
      if (len == 0 || len > MAX_FRAME) { rc = XCG_EPROTO; break; }
      if (avail < 5ull + len) break;
      fbuf.insert(fbuf.end(), b + 5, b + 5 + len);
      flens.push_back(len);
      i += 5ull + len;
    } else if (op == OP_ADVANCE) {
      if (!encoder) { rc = XCG_EPROTO; break; }
      if (avail < 5) break;
      const uint32_t count = (uint32_t)get_be(b + 1, 4);
      if (count == 0 || count > ref_frames.size()) { rc = XCG_EPROTO; break; }
      for (uint32_t k = 0; k < count; ++k) ref_frames.pop_front();   // encoder_reference_frame_advance
      i += 5;
    } else {
      rc = XCG_EPROTO;                                               // unsupported operation
      break;
    }
  }
  dbuf.erase(dbuf.begin(), dbuf.begin() + (ptrdiff_t)i);
  return rc;
}

// decoder_decode_data (:435-547): decode the buffered frame bytes on the GPU.
int xcg_pipe::decode_data() {
  if (fbuf.empty()) {
    if (decoder_received_eos && !encoder_sent_eos_ack) {
      to_peer.push_back(OP_EOS_ACK);
      encoder_sent_eos_ack = true;
    }
    return XCG_OK;
  }
  // One decode() call over everything buffered, into an output sized from
  // the ops themselves (not filled: the decode writes what it returns).
  const uint64_t off = 0;
  const uint32_t len = (uint32_t)fbuf.size();
  uint64_t oo = 0, ol = 0, cons = 0;
  int32_t st = 0;
  std::vector<uint64_t> unk(1u << 16);
  uint32_t nunk = 0;
  const uint64_t cap = decoded_bound(fbuf.data(), len) + 4096;
  std::unique_ptr<uint8_t[]> out(new uint8_t[cap]);
  int rc = xcg_decode_set_window(dec, win);
  if (rc == XCG_OK)
    rc = xcg_decode_host(dec, fbuf.data(), len, &off, &len, 1, out.get(), cap, &oo, &ol, &st, &cons,
                         unk.data(), (uint32_t)unk.size(), &nunk);
  xcg_decode_set_window(dec, nullptr);
  if (rc != XCG_OK) return rc;
  if (st < 0) return XCG_EPROTO;                                     // decode() returned false
  // <ADVANCE> for every frame consumed in full (:460-490)
  uint64_t consumed = cons;
  if (consumed) {
    uint32_t adv = 0;
    while (consumed) {
      const uint32_t first = flens.front();
      if (consumed < first) {
        flens.front() = first - (uint32_t)consumed;
        break;
      }
      consumed -= first;
      ++adv;
      flens.pop_front();
    }
    if (adv) {
      to_peer.push_back(OP_ADVANCE);
      put_be32(to_peer, adv);
    }
    fbuf.erase(fbuf.begin(), fbuf.begin() + (ptrdiff_t)cons);
  }
  to_local.insert(to_local.end(), out.get() + oo, out.get() + oo + ol);
  for (uint32_t k = 0; k < nunk; ++k) unknown.insert(unk[k]);
  // <ASK>s in groups of ASK_MAX (:510-545)
  std::vector<uint64_t> hs(unknown.begin(), unknown.end());
  for (size_t a = 0; a < hs.size(); a += ASK_MAX) {
    const size_t c = std::min<size_t>(ASK_MAX, hs.size() - a);
    to_peer.push_back(OP_ASK);
    put_be16(to_peer, (uint16_t)c);
    for (size_t k = 0; k < c; ++k) put_be64(to_peer, hs[a + k]);
  }
  return XCG_OK;
}

extern "C" {

int xcg_pipe_create(xcg_ctx* enc, xcg_ctx* dec, const uint8_t* uuid, xcg_pipe** out) {
  if (!enc || !dec || !uuid || !out || !uuid_ok(uuid)) return XCG_EINVAL;
  *out = nullptr;
  xcg_window* w = nullptr;
  const int rc = xcg_window_create(dec, &w);
  if (rc != XCG_OK) return rc;
  xcg_pipe* p = new xcg_pipe;
  p->enc = enc;
  p->dec = dec;
  p->win = w;
  memcpy(p->uuid, uuid, UUID_LEN);
  *out = p;
  return XCG_OK;
}

int xcg_pipe_create_connect(xcg_ctx* enc, xcg_ctx* parent, const uint8_t* uuid, xcg_pipe** out) {
  if (!enc || !parent || !uuid || !out || !uuid_ok(uuid)) return XCG_EINVAL;
  xcg_pipe* p = new xcg_pipe;
  p->enc = enc;
  p->dec = nullptr;
  p->parent = parent;
  p->win = nullptr;
  memcpy(p->uuid, uuid, UUID_LEN);
  *out = p;
  return XCG_OK;
}

xcg_ctx* xcg_pipe_decoder_ctx(const xcg_pipe* p) { return p ? p->dec : nullptr; }

void xcg_pipe_destroy(xcg_pipe* p) {
  if (!p) return;
  if (p->win) xcg_window_destroy(p->win);
  if (p->parent && p->dec) xcg_registry_release(p->dec);   // (a cleared registry's context goes now)
  delete p;
}

int xcg_pipe_encoder_consume_many(xcg_pipe* const* pipes, const uint8_t* const* data, const uint64_t* len,
                                  uint32_t n, xcg_pipe_out* out) {
  if (n == 0) return XCG_OK;
  if (!pipes || !data || !len) return XCG_EINVAL;
  xcg_ctx* enc = pipes[0]->enc;
  // Frames of every pipe's input, in order: <= MAX_FRAME / 2 bytes each
  // (:585-600), so a frame's encoding never exceeds MAX_FRAME.
  struct Frame { uint32_t pipe; uint64_t in_off; uint32_t len; };
  std::vector<Frame> frames;
  std::vector<uint64_t> base(n);
  uint64_t total = 0;
  for (uint32_t k = 0; k < n; ++k) {
    xcg_pipe* p = pipes[k];
    if (!p || p->enc != enc || p->encoder_sent_eos || (len[k] && !data[k])) return XCG_EINVAL;
    base[k] = total;
    for (uint64_t a = 0; a < len[k]; a += MAX_FRAME / 2)
      frames.push_back({k, total + a, (uint32_t)std::min<uint64_t>(MAX_FRAME / 2, len[k] - a)});
    total += len[k];
  }
  std::vector<uint8_t> in(total ? total : 1);
  for (uint32_t k = 0; k < n; ++k)
    if (len[k]) memcpy(in.data() + base[k], data[k], len[k]);
  const uint32_t nf = (uint32_t)frames.size();
  std::vector<uint64_t> off(nf), oo(nf), ol(nf);
  std::vector<uint32_t> fl(nf);
  uint64_t cap = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    off[f] = frames[f].in_off;
    fl[f] = frames[f].len;
    oo[f] = cap;
    cap += xcg_encode_bound(frames[f].len);
  }
  std::vector<uint8_t> enc_out(cap ? cap : 1);
  // one GPU batch: successive encode() calls of one XCodecEncoder cache
  if (nf) {
    const int rc = xcg_encode_host(enc, XCG_SEM_STREAM, in.data(), total, off.data(), fl.data(), nf, enc_out.data(),
                                   enc_out.size(), oo.data(), ol.data());
    if (rc != XCG_OK) return rc;
  }
  for (uint32_t k = 0; k < n; ++k) pipes[k]->begin();
  uint32_t eflags = 0;
  if (xcg_ctx_flags(enc, &eflags) != XCG_OK) return XCG_EINVAL;
  const bool oob = (eflags & XCG_FLAG_OOB) != 0, nullc = (eflags & XCG_FLAG_NULLCACHE) != 0;
  uint32_t f = 0;
  for (uint32_t k = 0; k < n; ++k) {
    xcg_pipe* p = pipes[k];
    if (!p->encoder) {                                   // <HELLO> (:557-573)
      p->to_peer.push_back(OP_HELLO);
      p->to_peer.push_back((uint8_t)UUID_LEN);
      p->to_peer.insert(p->to_peer.end(), p->uuid, p->uuid + UUID_LEN);
      p->encoder = true;
    }
    if (len[k] == 0) {                                   // <EOS> (:632-636)
      p->to_peer.push_back(OP_EOS);
      p->encoder_sent_eos = true;
    }
    for (; f < nf && frames[f].pipe == k; ++f) {
      std::unordered_map<uint64_t, std::vector<uint8_t>> rm;
      std::vector<std::pair<uint64_t, uint64_t>> decl;   // (input offset, hash) of out-of-band declarations
      if (nullc) {
        // TackNullCache: every F1 02 is a declaration (lookups always miss)
      } else if (oob) {
        std::vector<uint64_t> dh(fl[f] / SEG + 1);
        std::vector<uint32_t> dp(dh.size());
        uint32_t nd = 0;
        const int rc = xcg_last_declarations(enc, f, dh.data(), dp.data(), (uint32_t)dh.size(), &nd);
        if (rc != XCG_OK) return rc;
        for (uint32_t d = 0; d < nd && d < dh.size(); ++d) decl.emplace_back(dp[d], dh[d]);
        std::sort(decl.begin(), decl.end());
      }
      if (!nullc) frame_refs(enc_out.data() + oo[f], ol[f], in.data() + off[f], decl, rm);
      p->ref_frames.push_back(std::move(rm));
      p->to_peer.push_back(OP_FRAME);                    // (:620-628)
      put_be32(p->to_peer, (uint32_t)ol[f]);
      p->to_peer.insert(p->to_peer.end(), enc_out.begin() + (ptrdiff_t)oo[f],
                        enc_out.begin() + (ptrdiff_t)(oo[f] + ol[f]));
    }
    if (out) p->finish(out + k);
  }
  return XCG_OK;
}

int xcg_pipe_encoder_consume(xcg_pipe* p, const uint8_t* data, uint64_t len, xcg_pipe_out* out) {
  if (!p) return XCG_EINVAL;
  return xcg_pipe_encoder_consume_many(&p, &data, &len, 1, out);
}

int xcg_pipe_decoder_consume(xcg_pipe* p, const uint8_t* data, uint64_t len, xcg_pipe_out* out) {
  if (!p || (len && !data)) return XCG_EINVAL;
  p->begin();
  int rc = XCG_OK;
  if (len == 0) {                                        // peer closed (:72-87)
    if (!p->decoder_sent_eos) {
      p->decoder_sent_eos = true;
      p->local_eos = 1;
    }
    p->finish(out);
    return XCG_OK;
  }
  p->dbuf.insert(p->dbuf.end(), data, data + len);
  rc = p->decode_ops();
  if (rc == XCG_OK && p->unknown.empty()) rc = p->decode_data();
  if (rc == XCG_OK && p->dbuf.empty() && p->fbuf.empty()) {
    if (p->decoder_received_eos && !p->decoder_sent_eos && p->unknown.empty()) {
      p->local_eos = 1;                                  // decoder_produce_eos (:125-138)
      p->decoder_sent_eos = true;
    }
    if (p->encoder_sent_eos_ack && p->decoder_received_eos_ack && !p->encoder_produced_eos) {
      p->peer_eos = 1;                                   // encoder_produce_eos (:150-159)
      p->encoder_produced_eos = true;
    }
  }
  p->finish(out);
  return rc;
}

uint32_t xcg_pipe_pending_frames(const xcg_pipe* p) { return p ? (uint32_t)p->ref_frames.size() : 0u; }

}  // extern "C"
