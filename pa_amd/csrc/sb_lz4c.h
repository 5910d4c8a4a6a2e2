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
// On the device LZ4 runs on one wave (lz4_compress_wave), Snappy on one lane;
// their tables in LDS.
//
// The LZ4 compressors restate liblz4's LZ4_compress_generic (lz4.c), whose
// greedy parse they must reproduce byte for byte; that code is
//   LZ4 - Fast LZ compression algorithm
//   Copyright (C) 2011-2020, Yann Collet.
//   BSD 2-Clause License (http://www.opensource.org/licenses/bsd-license.php)
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are
//   met: * Redistributions of source code must retain the above copyright
//   notice, this list of conditions and the following disclaimer.
//   * Redistributions in binary form must reproduce the above copyright
//   notice, this list of conditions and the following disclaimer in the
//   documentation and/or other materials provided with the distribution.
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS
//   IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO,
//   THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR
//   PURPOSE ARE DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT OWNER OR
//   CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL,
//   EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO,
//   PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR
//   PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY THEORY OF
//   LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING
//   NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS
//   SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
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

#if defined(__HIPCC__)
// ---------------------------------------------------------------------------
// Wave-cooperative LZ4_compress_default: the bytes of lz4_compress above,
// produced by the 64 lanes of one wave (all of them call it, uniformly).
// The match search is the serial loop's 64 next iterations at once: lane l
// takes iteration t + l (its position from a scan of the skip steps, step
// (63 + u) >> 6 after iteration u), hashes it, and takes as candidate the
// latest earlier lane with the same hash (those positions are in the table
// by then) or else the table entry from before the batch; the first lane
// whose candidate matches ends the search, and the positions of the lanes up
// to it enter the table (of lanes sharing a hash, the last).  Catch-up,
// literal copies and match extension compare 64 bytes a step.
// ---------------------------------------------------------------------------
__device__ inline uint32_t lz4_ld32(const uint8_t* p) {  // unaligned little-endian dword
  const uintptr_t a = (uintptr_t)p;
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t* q = (const uint32_t*)(a - sh);
  const uint32_t lo = q[0];
  return sh ? __builtin_amdgcn_alignbyte(q[1], lo, sh) : lo;
}

#ifndef SB_LZ4_PREFIX
#define SB_LZ4_PREFIX 0
#endif
constexpr uint32_t kLz4Prefix = SB_LZ4_PREFIX;  // search iterations taken one at a time before the batches

__device__ inline uint32_t lz4_wave_incl_scan(uint32_t v) {  // DPP row shifts + row broadcasts
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
  return v;
}

typedef __attribute__((address_space(3))) uint8_t lz4_lds8;
constexpr uint32_t kLz4WaveLds = 16384 + 8192;  // position table + per-batch hash owners
// The smallest area the compressor runs in: the position table + 1 KiB of
// hash owners indexed by the hash's low bits (k_enc_basic_wave: 17 KiB a
// page-wave, nine a CU instead of six).  An owner slot shared by two hashes
// only sends both lanes through the clash loop, which groups lanes by the
// exact hash, so the parse is the same.
constexpr uint32_t kLz4WaveLdsMin = 16384 + 1024;

// The input of lz4_compress_wave: in HBM (a plain pointer), or staged in LDS
// (every hash, candidate compare and match extension of the parse is a
// dependent read: ~100 cycles from LDS instead of an L2 / HBM round trip).
struct Lz4GSrc {
  const uint8_t* p;
  __device__ __forceinline__ uint32_t u8(uint32_t i) const { return p[i]; }
  __device__ __forceinline__ uint32_t u32(uint32_t i) const { return lz4_ld32(p + i); }
};
struct Lz4LSrc {
  const lz4_lds8* p;  // 4-aligned
  __device__ __forceinline__ uint32_t u8(uint32_t i) const { return p[i]; }
  __device__ __forceinline__ uint32_t u32(uint32_t i) const {
    typedef const __attribute__((address_space(3))) uint32_t l32;
    const l32* q = (const l32*)(p + (i & ~3u));
    const uint32_t sh = i & 3, lo = q[0];
    return sh ? __builtin_amdgcn_alignbyte(q[1], lo, sh) : lo;
  }
};

// `lds`: kLz4WaveLds bytes, the first 16 KiB zeroed (the position table:
// 8192 u16 below LZ4_64Klimit, 4096 u32 above), then 8 KiB of scratch.
template <class Src>
__device__ inline uint32_t lz4_compress_wave(const Src src, uint32_t n, uint8_t* dst, lz4_lds8* lds,
                                             uint32_t own_mask = 8191) {
  const uint32_t lane = threadIdx.x & 63;
  const bool u16 = n < kLz4_64Klimit;
  typedef __attribute__((address_space(3))) uint16_t l16;
  typedef __attribute__((address_space(3))) uint32_t l32;
  l16* t16 = (l16*)lds;
  l32* t32 = (l32*)lds;
  // the lane that last wrote each hash in a batch (volatile: the read must see
  // the other lanes' stores, not be forwarded from this lane's own)
  volatile lz4_lds8* own = lds + 16384;
  auto tget = [&](uint32_t h) -> uint32_t { return u16 ? (uint32_t)t16[h] : t32[h]; };
  auto tput = [&](uint32_t h, uint32_t v) {
    if (u16) t16[h] = (uint16_t)v;
    else t32[h] = v;
  };
  auto hash_at = [&](uint32_t pos) -> uint32_t {
    if (u16) return (src.u32(pos) * 2654435761u) >> (32 - 13);
    const uint64_t v = (uint64_t)src.u32(pos) | ((uint64_t)src.u32(pos + 4) << 32);
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - 12));
  };
  // the run-length bytes of len (all 255 but the last), at dst + at
  auto put_len = [&](uint32_t at, uint32_t len) -> uint32_t {
    const uint32_t nb = len / 255 + 1;
    for (uint32_t i = lane; i < nb; i += 64) dst[at + i] = i + 1 < nb ? 255 : (uint8_t)(len % 255);
    return nb;
  };
  auto copy = [&](uint32_t to, uint32_t from, uint32_t len) {
    for (uint32_t i = lane; i < len; i += 64) dst[to + i] = (uint8_t)src.u8(from + i);
  };
  uint32_t op = 0, anchor = 0;
  if (n >= 13) {
    // (the first T.put(hash(0), 0) stores 0 into a zeroed table: nothing to do)
    const uint32_t mflimitPlusOne = n - 11, matchlimit = n - 5;
    uint32_t ip = 1;
    bool done = false;
    while (!done) {
      // ---- match search from ip ----
      uint32_t c = ip, t = 0, mpos = 0, mmatch = 0;
      bool found = false, ended = false;
      // the first iterations one at a time (uniform: every lane runs them): a
      // match is often this close, and a batch costs more than a few of them
      for (; t < kLz4Prefix; t++) {
        const uint32_t next = c + (t == 0 ? 1u : (63u + t) >> 6);
        if (next > mflimitPlusOne) {
          ended = true;
          break;
        }
        const uint32_t h = hash_at(c), mi = tget(h);
        if (lane == 0) tput(h, c);
        if ((u16 || mi + 65535 >= c) && src.u32(mi) == src.u32(c)) {
          mpos = c;
          mmatch = mi;
          found = true;
          break;
        }
        c = next;
      }
      while (!found && !ended) {  // then 64 iterations a batch
        const uint32_t u = t + lane, step = u == 0 ? 1u : (63u + u) >> 6;
        const uint32_t incl = lz4_wave_incl_scan(step);
        const uint32_t pos = c + incl - step, next = c + incl;
        const bool live = next <= mflimitPlusOne;
        const uint64_t deadm = __ballot(!live);
        const uint32_t E = deadm ? (uint32_t)__builtin_ctzll(deadm) : 64u;
        const uint32_t q = live ? pos : ip;
        const uint32_t h = hash_at(q);
        uint32_t mi = tget(h);
        // lanes sharing a hash: the candidate of each is the latest earlier
        // one, and only the last of them (up to the match) enters the table.
        // A plain byte write per lane finds the clashes, one ballot per
        // clashing hash groups them.
        if (live) own[h & own_mask] = (uint8_t)lane;
        bool todo = live && own[h & own_mask] != lane;
        uint64_t grp = 1ull << lane;
        for (uint64_t lm = __ballot(todo); lm; lm = __ballot(todo)) {
          const uint32_t H = __shfl(h, (uint32_t)__builtin_ctzll(lm), 64);
          const uint64_t same = __ballot(live && h == H);
          const uint64_t below = same & ((1ull << lane) - 1);
          const uint32_t pj = __shfl(pos, below ? 63u - (uint32_t)__builtin_clzll(below) : lane, 64);
          if (live && h == H) {
            if (below) mi = pj;
            grp = same;
            todo = false;
          }
        }
        const bool ok = live && (u16 || mi + 65535 >= pos) && src.u32(mi) == src.u32(q);
        const uint64_t okm = __ballot(ok);
        const uint32_t M = okm ? (uint32_t)__builtin_ctzll(okm) : 64u;
        const uint32_t upto = min(M + 1, E);
        const uint64_t in = upto >= 64 ? ~0ull : (1ull << upto) - 1;
        if (lane < upto && !(grp & in & ~((2ull << lane) - 1))) tput(h, pos);
        if (M < E) {
          mpos = __shfl(pos, M, 64);
          mmatch = __shfl(mi, M, 64);
          found = true;
          break;
        }
        if (E < 64) break;  // forwardIp passed mflimitPlusOne: the last literals
        c = __shfl(next, 63, 64);
        t += 64;
      }
      if (!found) break;
      uint32_t ipp = mpos, mt = mmatch;
      for (;;) {  // catch up
        const uint32_t k = min(min(ipp - anchor, mt), 64u);
        const uint64_t ne = __ballot(lane < k && src.u8(ipp - 1 - lane) != src.u8(mt - 1 - lane));
        const uint32_t j = ne ? (uint32_t)__builtin_ctzll(ne) : k;
        ipp -= j;
        mt -= j;
        if (j < 64) break;
      }
      const uint32_t lit = ipp - anchor;
      uint32_t tpos = op++, token;
      if (lit >= 15) {
        token = 15u << 4;
        op += put_len(op, lit - 15);
      } else {
        token = lit << 4;
      }
      copy(op, anchor, lit);
      op += lit;
      for (;;) {  // _next_match
        const uint32_t off = ipp - mt;
        if (lane == 0) {
          dst[op] = (uint8_t)off;
          dst[op + 1] = (uint8_t)(off >> 8);
        }
        op += 2;
        uint32_t a = ipp + 4, b = mt + 4;
        for (;;) {  // LZ4_count
          const uint32_t k = min(a < matchlimit ? matchlimit - a : 0u, 64u);
          const uint64_t ne = __ballot(lane < k && src.u8(a + lane) != src.u8(b + lane));
          const uint32_t j = ne ? (uint32_t)__builtin_ctzll(ne) : k;
          a += j;
          b += j;
          if (j < 64) break;
        }
        uint32_t ml = a - (ipp + 4);
        ipp += ml + 4;
        if (ml >= 15) {
          token += 15;
          op += put_len(op, ml - 15);
        } else {
          token += ml;
        }
        if (lane == 0) dst[tpos] = (uint8_t)token;
        anchor = ipp;
        if (ipp >= mflimitPlusOne) {
          done = true;
          break;
        }
        const uint32_t h2 = hash_at(ipp - 2);
        if (lane == 0) tput(h2, ipp - 2);
        const uint32_t h = hash_at(ipp);
        const uint32_t mi = tget(h);
        if (lane == 0) tput(h, ipp);
        if ((u16 || mi + 65535 >= ipp) && src.u32(mi) == src.u32(ipp)) {
          mt = mi;
          tpos = op++;
          token = 0;
          continue;
        }
        break;
      }
      ip = ipp + 1;
    }
  }
  const uint32_t last = n - anchor;
  if (last >= 15) {
    if (lane == 0) dst[op] = 15 << 4;
    op++;
    op += put_len(op, last - 15);
  } else {
    if (lane == 0) dst[op] = (uint8_t)(last << 4);
    op++;
  }
  copy(op, anchor, last);
  return op + last;
}
#endif

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
