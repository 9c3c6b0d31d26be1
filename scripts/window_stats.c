// Window-parse statistics of the LZ4 (SKIP) parse, replayed on the CPU: windows, probes,
// pre-extension rounds, matches, extension lanes.  Diagnostic only; uses the
// oracle library's synthetic input generator (bo_fill).
//   gcc -O2 -o /tmp/window_stats scripts/window_stats.c -L oracle/_build -lbitar_oracle \
//       -Wl,-rpath,$PWD/oracle/_build && /tmp/window_stats 1
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
void bo_fill(int kind, uint64_t seed, uint8_t* out, uint64_t n);
static inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint32_t hsh(uint32_t v) { return (v * 2654435761u) >> 22; }
int main(int argc, char** argv) {
  int kind = atoi(argv[1]);
  uint64_t N = 64ull << 20; uint32_t seg = 65536;
  uint8_t* buf = malloc(N + 64);
  bo_fill(kind, 0, buf, N);
  uint64_t ch16 = 0, ch16w = 0, win = 0, skipw = 0, probes = 0, r2 = 0, withm = 0, matches = 0, extl = 0, ext_chain = 0, lanes16 = 0;
  static uint32_t table[1024];
  for (uint64_t so = 0; so < N; so += seg) {
    const uint8_t* src = buf + so; uint32_t n = seg;
    memset(table, 0, sizeof table);
    uint32_t last_start = n - 12, match_limit = n - 5, pos = 0, g = 0;
    for (uint32_t x = 0; x <= last_start; x += 64) {
      if (pos >= x + 64) { skipw++; continue; }
      if (x >= g + 128) {
        uint32_t s = x >= g + 640 ? 4 : 2; int hit = 0; probes++;
        for (uint32_t l = 0; l < 64 && x + s * l <= last_start; ++l) {
          uint32_t p = x + s * l, c = table[hsh(rd32(src + p))];
          if (c < p && p - c <= 2560 && rd32(src + c) == rd32(src + p)) hit = 1;
        }
        if (!hit) { for (uint32_t l = 0; l < 64 && x + s * l <= last_start; ++l) table[hsh(rd32(src + x + s * l))] = x + s * l; x += (s - 1) * 64; continue; }
        g = x + 64 * (s - 1) - 127u;
      }
      win++;
      uint32_t cnt = last_start - x + 1; if (cnt > 64) cnt = 64;
      uint32_t cand[64], h[64], len[64];
      for (uint32_t l = 0; l < cnt; ++l) { h[l] = hsh(rd32(src + x + l)); cand[l] = table[h[l]]; }
      for (uint32_t l = 0; l < cnt; ++l) table[h[l]] = x + l;
      int any16 = 0;
      for (uint32_t l = 0; l < cnt; ++l) {
        uint32_t p = x + l, c = cand[l]; len[l] = 0;
        if (c < p && p - c <= 2560) { uint32_t k = 0; while (k < 32 && p + k < match_limit && src[c + k] == src[p + k]) ++k; len[l] = k; }
        if (len[l] >= 16) { any16 = 1; lanes16++; }
        if (len[l] >= 32) extl++;
      }
      if (any16) r2++;
      int m = 0, c16w = 0;
      for (;;) {
        uint32_t i = 0, found = 0;
        for (uint32_t l = (pos > x ? pos - x : 0); l < cnt; ++l) if (len[l] >= 4) { i = x + l; found = 1; break; }
        if (!found) break;
        uint32_t c = cand[i - x], L = 4; while (L < match_limit - i && src[c + L] == src[i + L]) ++L;
        if (len[i - x] >= 32) ext_chain++;
        if (len[i - x] >= 16) { ch16++; c16w = 1; }
        matches++; m = 1; pos = i + L;
      }
      if (m) withm++;
      if (c16w) ch16w++;
      if (pos > g) g = pos;
    }
  }
  double W = (double)win;
  printf("kind %d: windows %.0f (per MiB %.0f) skipped %.3f probes %.3f | round2 %.3f  lanes>=16/win %.1f  ext lanes/win %.1f  with match %.3f  matches/win %.2f  ext chain/win %.3f chain16/win %.3f win-with-chain16 %.3f\n",
         kind, W, W / 64, skipw / W, probes / W, r2 / W, lanes16 / W, extl / W, withm / W, matches / W, ext_chain / W, ch16 / W, ch16w / W);
  return 0;
}
