/* The survey's synthetic workload generator (BASELINE.md "Generator for
 * kat_a/b/c") in C, for bench and test inputs of many GiB:
 * bytes [lo, hi) of stream(seed, dup, magic) without materialising the
 * prefix.  Bit-exact with wanproxy_amd/synth.py (tests/test_synth.py).
 *
 * stream: splitmix64 draws; per 2048-byte block, once a fresh block exists,
 * draw r and if r % 100 < dup copy fresh block (next() % nfresh); otherwise a
 * fresh block = 256 little-endian draws, then with magic one draw per byte
 * forcing it to 0xF1 when draw % 100 < magic.  Not product code: no GPU path
 * calls it. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t sm_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* 0 ok, -1 out of memory */
int xcs_stream_range(uint64_t seed, uint32_t dup, uint32_t magic, uint64_t lo, uint64_t hi, uint8_t *out) {
  if (hi <= lo) return 0;
  const uint64_t SEG = 2048, b0 = lo / SEG, b1 = (hi + SEG - 1) / SEG;
  const uint64_t per_fresh = 256 + (magic ? SEG : 0);
  uint64_t cap = 1024, nfresh = 0, pos = 0;
  uint64_t *fresh = (uint64_t *)malloc(cap * sizeof(uint64_t));
  if (!fresh) return -1;
  uint8_t blk[2048];
  for (uint64_t b = 0; b < b1; b++) {
    uint64_t f = ~0ull;
    if (nfresh) {
      const uint64_t r = sm_at(seed, pos++);
      if (dup > 0 && r % 100 < dup) f = fresh[sm_at(seed, pos++) % nfresh];
    }
    if (f == ~0ull) {
      if (nfresh == cap) {
        cap *= 2;
        uint64_t *nf = (uint64_t *)realloc(fresh, cap * sizeof(uint64_t));
        if (!nf) { free(fresh); return -1; }
        fresh = nf;
      }
      f = fresh[nfresh++] = pos;
      pos += per_fresh;
    }
    if (b < b0) continue;
    for (int k = 0; k < 256; k++) {
      const uint64_t v = sm_at(seed, f + k);
      memcpy(blk + 8 * k, &v, 8);              /* little-endian host */
    }
    if (magic)
      for (uint64_t k = 0; k < SEG; k++)
        if (sm_at(seed, f + 256 + k) % 100 < magic) blk[k] = 0xF1;
    const uint64_t s = b * SEG, e = s + SEG;
    const uint64_t a = s < lo ? lo : s, z = e > hi ? hi : e;
    memcpy(out + (a - lo), blk + (a - s), z - a);
  }
  free(fresh);
  return 0;
}
