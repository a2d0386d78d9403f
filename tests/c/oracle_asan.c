/* oracle_asan.c -- the C oracle built with -fsanitize=address,undefined (host-only
 * sanitizer run): known-answer checks plus a random add/contains/HLL workout. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t orc_highway_hash64(const uint8_t *, size_t, const uint64_t *);
void orc_redisson_hash128(const uint8_t *, size_t, uint64_t *);
uint64_t orc_murmur64a(const uint8_t *, int, uint64_t);
uint16_t orc_crc16(const uint8_t *, size_t);
int orc_bloom_optimal(int64_t, double, int64_t, int64_t *, int32_t *);
int64_t orc_bloom_add(uint8_t *, uint64_t *, const uint8_t *, const uint64_t *, uint64_t, int, int64_t, uint8_t *);
int64_t orc_bloom_contains(const uint8_t *, uint64_t, const uint8_t *, const uint64_t *, uint64_t, int, int64_t, uint8_t *);
int orc_hll_pfadd(uint8_t *, const uint8_t *, const uint64_t *, uint64_t);
uint64_t orc_hll_count(const uint8_t *);

int main(void) {
    const uint64_t key[4] = {0x0706050403020100ULL, 0x0F0E0D0C0B0A0908ULL, 0x1716151413121110ULL, 0x1F1E1D1C1B1A1918ULL};
    uint8_t d[64];
    for (int i = 0; i < 64; ++i) d[i] = (uint8_t)i;
    if (orc_highway_hash64(d, 0, key) != 0x907A56DE22C26E53ULL) return 1;
    if (orc_highway_hash64(d, 11, key) != 0xC3BBF4615B415C15ULL) return 2;
    if (orc_crc16((const uint8_t *)"123456789", 9) != 0x31C3) return 3;
    int64_t m;
    int32_t k;
    if (orc_bloom_optimal(100, 0.03, 4294967294LL, &m, &k) || m != 729 || k != 5) return 4;
    /* random workout: variable-length keys, every tail shape */
    uint64_t n = 4000, offs[4001];
    uint8_t *buf = malloc(n * 70), *flags = malloc(n);
    uint64_t o = 0, s = 12345;
    for (uint64_t i = 0; i < n; ++i) {
        offs[i] = o;
        uint64_t len = (s = s * 6364136223846793005ULL + 1442695040888963407ULL) >> 58;
        for (uint64_t j = 0; j < len; ++j) buf[o + j] = (uint8_t)((s = s * 6364136223846793005ULL + 1) >> 56);
        o += len;
    }
    offs[n] = o;
    uint8_t *bm = calloc(9585 / 8 + 2, 1);
    uint64_t rl = 0;
    int64_t a = orc_bloom_add(bm, &rl, buf, offs, n, 7, 9585, flags);
    int64_t c = orc_bloom_contains(bm, rl, buf, offs, n, 7, 9585, flags);
    if (a <= 0 || c != (int64_t)n) return 5;
    uint8_t *regs = calloc(16384, 1);
    orc_hll_pfadd(regs, buf, offs, n);
    uint64_t e = orc_hll_count(regs);
    if (e < 3800 || e > 4200) return 6;
    free(buf); free(flags); free(bm); free(regs);
    printf("oracle asan/ubsan: ok\n");
    return 0;
}
