// Host-only timing of the pair replay (XcgPairState::replay) on a synthetic
// C5-like reference stream: build with
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/prb scripts/dev/pair_replay_bench.cpp
// and run /tmp/prb (no GPU needed: no HIP call is made).
#include "../../wanproxy_amd/csrc/xcg_pair.hip"

#include <chrono>
#include <random>

int main(int argc, char** argv) {
  const uint32_t C = 65536, nb = 2557, D = nb * 204, ids = C + D;
  XcgPairState* P = new XcgPairState;
  P->C = C; P->nb = nb; P->D = D;
  P->ps.assign(C, PSlot{NOKEY, NOKEY, NIL, NIL, NIL, NIL, NIL, NIL, NIL, 0});
  XcgDiskState* K = new XcgDiskState;
  K->nb = nb; K->D = D;
  K->ds.assign(D, DSlot{NOKEY, NOKEY, NIL, NIL, NIL, 0, 0, 0, 0, 0});
  K->fronts.push_back(P);
  P->disk = K; P->dsp = &K->ds; P->xuid = 0;
  P->es.assign(ids, Ent{NEVER, 0, NIL, NIL, 0});
  P->pfree.resize(C);
  for (uint32_t s = 0; s < C; ++s) P->pfree[s] = C - 1 - s;
  P->ftop = C;
  const uint32_t n = 4096, maxd = 65, maxe = 2 * maxd + 64;
  std::vector<uint4> ev((size_t)n * maxe);
  std::vector<uint32_t> nev(n);
  std::mt19937_64 rng(1);
  uint64_t hseq = 1;
  for (int batch = 0; batch < 3; ++batch) {
    // chunk c: ~52 declarations, ~8 lookups of cached hashes (the sub-batch start state)
    std::vector<uint32_t> live;
    for (uint32_t s = 0; s < C; ++s) if (P->ps[s].key != NOKEY) live.push_back(s);
    for (uint32_t i = 0; i < D; ++i) if (P->ds()[i].live && P->ds()[i].dp == NIL) live.push_back(C + i);
    for (uint32_t c = 0; c < n; ++c) {
      uint32_t k = 0, d = 0;
      for (uint32_t w = 0; w < 60; ++w) {
        const uint32_t t = 2 * (w * 2048);
        if (!live.empty() && rng() % 100 < 13) {
          const uint32_t id = live[rng() % live.size()];
          ev[(size_t)c * maxe + k++] = make_uint4(0, 0, t + 1, (EV_GHIT << 30) | id);
        } else {
          const uint64_t h = (hseq++) * 0x9E3779B97F4A7C15ull >> 4;
          ev[(size_t)c * maxe + k++] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), t + 2, (EV_ENTER << 30) | d++);
        }
      }
      nev[c] = k;
    }
    for (int rep = 0; rep < 2; ++rep) {            // (the pass copies make a replay repeatable)
      const auto r0 = std::chrono::steady_clock::now();
      P->replay(n, ev.data(), nev.data(), maxe, maxd);
      printf("  dry replay %.2f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - r0).count());
    }
    const auto t0 = std::chrono::steady_clock::now();
    const bool ok = P->replay(n, ev.data(), nev.data(), maxe, maxd);
    const auto t1 = std::chrono::steady_clock::now();
    P->keep();
    const auto t2 = std::chrono::steady_clock::now();
    printf("batch %d ok %d enters %llu refs %llu appends %llu: replay %.2f ms keep %.2f ms (%.1f ns/event)\n", batch,
           ok, (unsigned long long)P->enters, (unsigned long long)P->refs, (unsigned long long)P->appends,
           std::chrono::duration<double, std::milli>(t1 - t0).count(),
           std::chrono::duration<double, std::milli>(t2 - t1).count(),
           std::chrono::duration<double, std::nano>(t1 - t0).count() / (n * 60.0));
  }
  return 0;
}

// (the stream driver is not linked in this host-only harness)
extern "C" int xcg_launch_seed_tiling(const XcgStreamArgs*, hipStream_t) { return -5; }
extern "C" int xcg_launch_encode_stream(const XcgStreamArgs*, int*, hipStream_t) { return -5; }
