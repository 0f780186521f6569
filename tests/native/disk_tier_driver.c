/* Two XCodecCachePair fronts on one XCodecDisk, driven through the C ABI by a
 * process that never loads PyTorch (a drop-in's process: wanproxy linked
 * against libxcgpu.so).  Test infrastructure for tests/test_gpu_disk.py: the
 * parent test compares what this writes with the oracle's pair.
 *
 *   disk_tier_driver A.bin B.bin OUT.bin limit_bytes disk_bytes disk_flags
 *
 * Streams A and B are cut into 64 KiB chunks; the fronts encode them four
 * chunks per call in alternation (A, B, A, B, ...) with stream semantics.
 * OUT: per call, per chunk: u64 length + bytes; then the two fronts'
 * xcg_pair_stats (4 x u64 each), xcg_disk_stats (4 x u64) and the tier
 * (i64).  Exit status 0, or the failing call's status. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/xcgpu.h"

static uint8_t *slurp(const char *path, uint64_t *len) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *len = (uint64_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *b = (uint8_t *)malloc(*len ? *len : 1);
  if (b && *len && fread(b, 1, *len, f) != *len) {
    free(b);
    b = NULL;
  }
  fclose(f);
  return b;
}

#define CALL(x)                                                       \
  do {                                                                \
    int rc_ = (x);                                                    \
    if (rc_ != XCG_OK) {                                              \
      fprintf(stderr, "%s: %d (%s)\n", #x, rc_, xcg_strerror(rc_));   \
      return rc_ < 0 ? -rc_ : 1;                                      \
    }                                                                 \
  } while (0)

int main(int argc, char **argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s A.bin B.bin OUT.bin limit_bytes disk_bytes disk_flags\n", argv[0]);
    return 2;
  }
  uint64_t la = 0, lb = 0;
  uint8_t *da = slurp(argv[1], &la), *db = slurp(argv[2], &lb);
  FILE *out = fopen(argv[3], "wb");
  if (!da || !db || !out) return 2;
  const uint64_t limit = strtoull(argv[4], NULL, 0), disk_bytes = strtoull(argv[5], NULL, 0);
  const uint32_t dflags = (uint32_t)strtoul(argv[6], NULL, 0);
  xcg_disk *disk = NULL;
  xcg_ctx *ca = NULL, *cb = NULL;
  CALL(xcg_disk_create_ex(disk_bytes, dflags, &disk));
  CALL(xcg_ctx_create_pair_on(0, 0, limit, disk, &ca));
  CALL(xcg_ctx_create_pair_on(0, 0, limit, disk, &cb));
  const uint32_t CH = 65536, PER = 4;
  const uint64_t na = (la + CH - 1) / CH, nb = (lb + CH - 1) / CH;
  uint64_t offs[4], oo[4], ol[4];
  uint32_t lens[4];
  uint8_t *obuf = (uint8_t *)malloc(PER * (2 * (uint64_t)CH + 16));
  for (uint64_t k = 0; k < na || k < nb; k += PER) {
    for (int side = 0; side < 2; ++side) {
      const uint8_t *d = side ? db : da;
      const uint64_t len = side ? lb : la, n = side ? nb : na;
      if (k >= n) continue;
      const uint32_t m = (uint32_t)(n - k < PER ? n - k : PER);
      uint64_t cap = 0;
      for (uint32_t i = 0; i < m; ++i) {
        offs[i] = (k + i) * CH;
        lens[i] = (uint32_t)(len - offs[i] < CH ? len - offs[i] : CH);
        oo[i] = cap;
        cap += xcg_encode_bound(lens[i]);
      }
      CALL(xcg_encode_host(side ? cb : ca, XCG_SEM_STREAM, d, len, offs, lens, m, obuf, cap, oo, ol));
      for (uint32_t i = 0; i < m; ++i) {
        fwrite(&ol[i], 8, 1, out);
        fwrite(obuf + oo[i], 1, ol[i], out);
      }
    }
  }
  uint64_t st[12];
  CALL(xcg_pair_stats(ca, st));
  CALL(xcg_pair_stats(cb, st + 4));
  CALL(xcg_disk_stats(disk, st + 8));
  const int64_t tier = xcg_disk_tier(disk);
  fwrite(st, 8, 12, out);
  fwrite(&tier, 8, 1, out);
  fclose(out);
  xcg_ctx_destroy(ca);
  xcg_ctx_destroy(cb);
  xcg_disk_destroy(disk);
  free(da);
  free(db);
  free(obuf);
  return 0;
}
