// sb_lz4c.h -- block compressors of the general codecs, host + device.
//
// The writer's Basic codecs (CommonCompression::compress, compression/
// basic.rs:108-152) must produce the same bytes on the device as on the host
// so that a page encoded on the GPU is byte-identical to the host writer's:
//   * LZ4: a restatement of liblz4 1.9.3 LZ4_compress_default (the lz4 crate
//     1.23 wraps that library; basic.rs:115 `compress_to_buffer(.., None,
//     false, ..)` = acceleration 1, no size prefix).  One fresh hash table per
//     block: inputs below LZ4_64Klimit use the 8192-entry u16 table and the
//     4-byte hash, larger inputs the 4096-entry u32 table, the 5-byte hash
//     and the 64 KiB distance check.  Match search with the skip trigger
//     (step grows every 64 misses), backward catch-up, the ip-2 table fill
//     after every match and the immediate re-match test, LASTLITERALS 5 /
//     MFLIMIT 12 end rules.  Verified against the system liblz4 by
//     tests/test_lz4c.py through sb_lz4_compress_host.
//   * Snappy: the engine's own raw-snappy writer (sb_encode.cpp
//     snappy_compress: greedy 14-bit hash matcher, 64-byte copy-2 elements).
// Both are serial: on the device one lane runs them, the hash table in LDS.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SB_HD __host__ __device__
#else
#define SB_HD
#endif

namespace sbc {

constexpr uint32_t kLz4TableBytes = 16384;     // LZ4_MEMORY_USAGE 14
constexpr uint32_t kSnappyTableBytes = 65536;  // 1 << 14 positions of 4 bytes
constexpr uint32_t kLz4_64Klimit = 65536 + 12 - 1;

SB_HD inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
SB_HD inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

SB_HD inline uint32_t lz4_bound(uint32_t n) { return n + n / 255 + 16; }

struct Lz4Table {
  void* t;
  bool u16;
  SB_HD uint32_t get(uint32_t h) const { return u16 ? ((const uint16_t*)t)[h] : ((const uint32_t*)t)[h]; }
  SB_HD void put(uint32_t h, uint32_t idx) const {
    if (u16) ((uint16_t*)t)[h] = (uint16_t)idx;
    else ((uint32_t*)t)[h] = idx;
  }
  // LZ4_hashPosition: hash4 (byU16, log 13) or hash5 of the 8-byte read (byU32, log 12)
  SB_HD uint32_t hash(const uint8_t* p) const {
    if (u16) return (rd32(p) * 2654435761u) >> (32 - 13);
    return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> (64 - 12));
  }
};

// LZ4_compress_default(src, dst, n, LZ4_compressBound(n)); `table` holds
// kLz4TableBytes zeroed bytes.  Returns the compressed size.
SB_HD inline uint32_t lz4_compress(const uint8_t* src, uint32_t n, uint8_t* dst, void* table) {
  const Lz4Table T{table, n < kLz4_64Klimit};
  const uint8_t* ip = src;
  const uint8_t* anchor = src;
  const uint8_t* const iend = src + n;
  const uint8_t* const mflimitPlusOne = iend - 12 + 1;
  const uint8_t* const matchlimit = iend - 5;
  uint8_t* op = dst;
  if (n >= 13) {
    T.put(T.hash(ip), 0);
    ip++;
    uint32_t forwardH = T.hash(ip);
    for (;;) {
      const uint8_t* match;
      uint8_t* token;
      {  // find a match
        const uint8_t* forwardIp = ip;
        uint32_t step = 1, searchMatchNb = 1u << 6;
        for (;;) {
          const uint32_t h = forwardH;
          const uint32_t cur = (uint32_t)(forwardIp - src);
          const uint32_t mi = T.get(h);
          ip = forwardIp;
          forwardIp += step;
          step = searchMatchNb++ >> 6;
          if (forwardIp > mflimitPlusOne) goto last_literals;
          match = src + mi;
          forwardH = T.hash(forwardIp);
          T.put(h, cur);
          if (!T.u16 && mi + 65535 < cur) continue;  // too far
          if (rd32(match) == rd32(ip)) break;
        }
      }
      // catch up
      while (ip > anchor && match > src && ip[-1] == match[-1]) {
        ip--;
        match--;
      }
      {  // literals
        const uint32_t lit = (uint32_t)(ip - anchor);
        token = op++;
        if (lit >= 15) {
          uint32_t len = lit - 15;
          *token = 15 << 4;
          for (; len >= 255; len -= 255) *op++ = 255;
          *op++ = (uint8_t)len;
        } else {
          *token = (uint8_t)(lit << 4);
        }
        for (uint32_t i = 0; i < lit; i++) op[i] = anchor[i];
        op += lit;
      }
      for (;;) {  // _next_match
        const uint32_t off = (uint32_t)(ip - match);
        op[0] = (uint8_t)off;
        op[1] = (uint8_t)(off >> 8);
        op += 2;
        {
          uint32_t ml = 0;  // LZ4_count(ip + 4, match + 4, matchlimit)
          const uint8_t* a = ip + 4;
          const uint8_t* b = match + 4;
          while (a < matchlimit && *a == *b) {
            a++;
            b++;
          }
          ml = (uint32_t)(a - (ip + 4));
          ip += ml + 4;
          if (ml >= 15) {
            *token += 15;
            ml -= 15;
            for (; ml >= 255; ml -= 255) *op++ = 255;
            *op++ = (uint8_t)ml;
          } else {
            *token += (uint8_t)ml;
          }
        }
        anchor = ip;
        if (ip >= mflimitPlusOne) goto last_literals;
        T.put(T.hash(ip - 2), (uint32_t)(ip - 2 - src));
        // test the next position
        const uint32_t h = T.hash(ip);
        const uint32_t cur = (uint32_t)(ip - src);
        const uint32_t mi = T.get(h);
        match = src + mi;
        T.put(h, cur);
        if ((T.u16 || mi + 65535 >= cur) && rd32(match) == rd32(ip)) {
          token = op++;
          *token = 0;
          continue;
        }
        break;
      }
      forwardH = T.hash(++ip);
    }
  }
last_literals : {
  const uint32_t last = (uint32_t)(iend - anchor);
  if (last >= 15) {
    uint32_t acc = last - 15;
    *op++ = 15 << 4;
    for (; acc >= 255; acc -= 255) *op++ = 255;
    *op++ = (uint8_t)acc;
  } else {
    *op++ = (uint8_t)(last << 4);
  }
  for (uint32_t i = 0; i < last; i++) op[i] = anchor[i];
  op += last;
}
  return (uint32_t)(op - dst);
}

// Raw snappy as sb_encode.cpp snappy_compress writes it.  `table` holds
// kSnappyTableBytes bytes (initialised here).  Returns the size.
SB_HD inline uint32_t snappy_literal(uint8_t* o, const uint8_t* p, uint32_t len) {
  uint8_t* o0 = o;
  while (len) {
    const uint32_t c = len < 65536 ? len : 65536, l1 = c - 1;
    if (l1 < 60) {
      *o++ = (uint8_t)(l1 << 2);
    } else if (l1 < 256) {
      *o++ = 60 << 2;
      *o++ = (uint8_t)l1;
    } else {
      *o++ = 61 << 2;
      *o++ = (uint8_t)l1;
      *o++ = (uint8_t)(l1 >> 8);
    }
    for (uint32_t i = 0; i < c; i++) o[i] = p[i];
    o += c;
    p += c;
    len -= c;
  }
  return (uint32_t)(o - o0);
}

SB_HD inline uint32_t snappy_compress(const uint8_t* in, uint32_t n, uint8_t* out, void* table) {
  uint8_t* o = out;
  uint64_t v = n;
  do {
    uint8_t c = v & 0x7F;
    v >>= 7;
    if (v) c |= 0x80;
    *o++ = c;
  } while (v);
  constexpr int HB = 14;
  int32_t* tab = (int32_t*)table;
  for (uint32_t i = 0; i < (1u << HB); i++) tab[i] = -1;
  uint32_t lit = 0, i = 0;
  while (i + 4 <= n) {
    const uint32_t w = rd32(in + i);
    const uint32_t h = (w * 0x1E35A7BDu) >> (32 - HB);
    const int32_t cand = tab[h];
    tab[h] = (int32_t)i;
    if (cand >= 0 && i - (uint32_t)cand <= 65535 && rd32(in + cand) == w) {
      uint32_t len = 4;
      while (i + len < n && in[cand + len] == in[i + len]) len++;
      if (i > lit) o += snappy_literal(o, in + lit, i - lit);
      uint32_t rem = len;
      const uint32_t off = i - (uint32_t)cand;
      while (rem) {
        uint32_t l = rem < 64 ? rem : 64;
        if (rem > 64 && rem - 64 < 4) l = 60;
        *o++ = (uint8_t)(((l - 1) << 2) | 2);
        *o++ = (uint8_t)off;
        *o++ = (uint8_t)(off >> 8);
        rem -= l;
      }
      i += len;
      lit = i;
    } else {
      i++;
    }
  }
  if (n > lit) o += snappy_literal(o, in + lit, n - lit);
  return (uint32_t)(o - out);
}

}  // namespace sbc
