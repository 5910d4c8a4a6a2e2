// sb_zstdc.h -- Zstandard frame writer of the device encoder (host + device).
//
// The writer's Zstd codec (CommonCompression::compress, compression/
// basic.rs:122-135: zstd::bulk::compress at level 0 -> libzstd level 3) has
// no restatement on the device; the encoder's bar for it is decode
// equivalence: a frame any RFC 8878 decoder (libzstd, the
// engine's sb_zstd.h) turns back into the input bytes.  The frame is built
// from the wave LZ4 compressor's parse (sb_lz4c.h; the same greedy liblz4
// sequences) -- every LZ4 sequence (literals, offset <= 65535, match >= 4)
// is a Zstd sequence:
//   * frame: magic, single-segment header with the content size, no
//     checksum; the input in 128 KiB chunks, each parsed by LZ4 on its own
//     (matches stay inside the chunk);
//   * a chunk's sequences go out in compressed blocks of at most
//     kZSeqPerBlock sequences: the block's literals (zstd_literals: a
//     Huffman-coded 4-stream Compressed_Literals_Block with a directly
//     represented table when that is smaller, an RLE block for one repeated
//     byte, else Raw), then the sequences under the Predefined_Mode FSE
//     tables of literal lengths, match lengths and offsets (RFC 8878
//     §3.1.1.3.2.2), every offset a new one (Offset_Value = offset + 3, no
//     repeat codes), encoded last sequence first as libzstd's
//     ZSTD_encodeSequences does; a block that would not shrink is written
//     Raw instead.
// Decode equivalence is checked against libzstd by tests/test_zstdc.py
// (host build, sb_zstd_compress_host) and tests/test_gpu_encode.py (device).
#pragma once
#include <stdint.h>

#include "sb_lz4c.h"

namespace sbz {

constexpr uint32_t kZChunk = 131072;      // Block_Maximum_Size; one LZ4 parse per chunk
constexpr uint32_t kZSeqPerBlock = 2048;  // sequences of one compressed block (their records: 16 KiB)

SB_HD constexpr uint32_t hbit(uint32_t v) {
  uint32_t r = 0;
  while (v >>= 1) r++;
  return r;
}

// FSE compression table of a normalized distribution (zstd
// FSE_buildCTable_wksp): the state table after the symbol spread the decoder
// uses (step = size/2 + size/8 + 3, -1 symbols at the top), and per symbol
// deltaFindState / deltaNbBits.  FseCTab: the predefined tables (log <= 6);
// FseCTabL: a block's own tables (log <= 9).
template <uint32_t LOGMAX>
struct FseT {
  uint16_t st[1u << LOGMAX];
  int32_t dfs[53];
  uint32_t dnb[53];
};
using FseCTab = FseT<6>;
using FseCTabL = FseT<9>;

// sym: 2^log bytes of work (the spread)
template <class T>
SB_HD constexpr void fse_fill(T& t, const int16_t* norm, uint32_t nsym, uint32_t log, uint8_t* sym) {
  const uint32_t size = 1u << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  uint32_t cumul[54] = {};
  for (uint32_t u = 1; u <= nsym; u++) {
    if (norm[u - 1] == -1) {
      cumul[u] = cumul[u - 1] + 1;
      sym[high--] = (uint8_t)(u - 1);
    } else {
      cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
    }
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s < nsym; s++)
    for (int i = 0; i < norm[s]; i++) {
      sym[pos] = (uint8_t)s;
      pos = (pos + step) & mask;
      while (pos > high) pos = (pos + step) & mask;
    }
  for (uint32_t u = 0; u < size; u++) t.st[cumul[sym[u]]++] = (uint16_t)(size + u);
  int32_t total = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    const int n = norm[s];
    if (n == -1 || n == 1) {
      t.dnb[s] = (log << 16) - size;
      t.dfs[s] = total - 1;
      total++;
    } else if (n > 1) {
      const uint32_t mbo = log - hbit((uint32_t)n - 1), msp = (uint32_t)n << mbo;
      t.dnb[s] = (mbo << 16) - msp;
      t.dfs[s] = total - n;
      total += n;
    }
  }
}

constexpr FseCTab fse_ctab(const int16_t* norm, uint32_t nsym, uint32_t log) {
  FseCTab t{};
  uint8_t sym[64] = {};
  fse_fill(t, norm, nsym, log, sym);
  return t;
}

// RFC 8878 §3.1.1.3.2.2 default distributions
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
constexpr uint32_t kLLLog = 6, kMLLog = 6, kOFLog = 5;

#if defined(__HIPCC__)
#define SBZ_TAB __constant__ const
#else
#define SBZ_TAB static const
#endif
SBZ_TAB FseCTab kLLc = fse_ctab(kLLNorm, 36, kLLLog);  // literal lengths, match lengths, offsets
SBZ_TAB FseCTab kMLc = fse_ctab(kMLNorm, 53, kMLLog);
SBZ_TAB FseCTab kOFc = fse_ctab(kOFNorm, 29, kOFLog);
// literal length codes 16..35 and match length codes 32..52: baselines and extra bits
SBZ_TAB uint32_t kLLBaseT[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                                 20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
SBZ_TAB uint32_t kMLBaseT[53] = {3,   4,   5,   6,   7,    8,    9,    10,   11,   12,    13,    14,    15,   16,
                                 17,  18,  19,  20,  21,   22,   23,   24,   25,   26,    27,    28,    29,   30,
                                 31,  32,  33,  34,  35,   37,   39,   41,   43,   47,    51,    59,    67,   83,
                                 99,  131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
SBZ_TAB uint8_t kLLBitsT[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
SBZ_TAB uint8_t kMLBitsT[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

SB_HD inline uint32_t ll_code(uint32_t ll) {
  if (ll < 16) return ll;
  uint32_t c = 35;
  while (kLLBaseT[c] > ll) c--;
  return c;
}
SB_HD inline uint32_t ml_code(uint32_t ml) {  // ml >= 3
  if (ml < 35) return ml - 3;
  uint32_t c = 52;
  while (kMLBaseT[c] > ml) c--;
  return c;
}
SB_HD inline uint32_t hbit32(uint32_t v) {
  uint32_t r = 0;
  while (v >>= 1) r++;
  return r;
}

// bit writer of the sequences stream (BIT_CStream: LSB first)
struct BitW {
  uint8_t* p;
  uint64_t acc;
  uint32_t n;
  SB_HD inline void add(uint32_t v, uint32_t nb) {
    acc |= (uint64_t)(nb ? (v & (0xFFFFFFFFu >> (32 - nb))) : 0u) << n;
    n += nb;
    while (n >= 8) {
      *p++ = (uint8_t)acc;
      acc >>= 8;
      n -= 8;
    }
  }
  SB_HD inline void close() {  // the end mark, then the last partial byte
    add(1, 1);
    if (n) *p++ = (uint8_t)acc;
  }
};

template <class T>
SB_HD inline uint32_t fse_init(const T& t, uint32_t s) {
  const uint32_t nb = (t.dnb[s] + (1u << 15)) >> 16, v = (nb << 16) - t.dnb[s];
  return t.st[(int32_t)(v >> nb) + t.dfs[s]];
}
template <class T>
SB_HD inline uint32_t fse_encode(const T& t, uint32_t st, uint32_t s, BitW& bw) {
  const uint32_t nb = (st + t.dnb[s]) >> 16;
  bw.add(st, nb);
  return t.st[(int32_t)(st >> nb) + t.dfs[s]];
}

// Bytes the frame of an n-byte input can take: every block but a chunk's last
// covers >= 4 * kZSeqPerBlock bytes, a block is never longer than its bytes + 3
// (Raw fallback), and a compressed block under construction runs at most
// 1/8 byte per sequence + 10 past that before the fallback is decided.
SB_HD inline uint64_t zstd_bound(uint64_t n) { return n + n / 2048 + 3 * (n / kZChunk) + 512; }

// Magic + single-segment frame header with the content size; returns its length.
SB_HD inline uint32_t zstd_frame_header(uint8_t* d, uint32_t n) {
  d[0] = 0x28, d[1] = 0xB5, d[2] = 0x2F, d[3] = 0xFD;
  if (n < 256) {
    d[4] = 0x20;  // single segment, FCS 1 byte
    d[5] = (uint8_t)n;
    return 6;
  }
  if (n < 65536 + 256) {
    d[4] = 0x60;  // FCS 2 bytes: n - 256
    d[5] = (uint8_t)(n - 256), d[6] = (uint8_t)((n - 256) >> 8);
    return 7;
  }
  d[4] = 0xA0;  // FCS 4 bytes
  for (int i = 0; i < 4; i++) d[5 + i] = (uint8_t)(n >> (8 * i));
  return 9;
}

SB_HD inline void put24(uint8_t* d, uint32_t v) { d[0] = (uint8_t)v, d[1] = (uint8_t)(v >> 8), d[2] = (uint8_t)(v >> 16); }

// Scratch of zstd_transcode: the block's sequence records (kZSeqPerBlock
// u64), then 8 KiB of work: the literals' Huffman area (u32: histogram [256],
// lengths / codes [256], tree weights [257], parents [257] + present symbols
// [129]), behind it the Huffman weights' FSE table; once the literals are out,
// the same 8 KiB hold the sequence tables (three FseCTabL, their histograms,
// normalized counts and the spread's work bytes).
constexpr uint32_t kZScratchU64 = kZSeqPerBlock + 1024;  // 24 KiB
constexpr uint32_t kHufMaxBits = 11;

// 16 * log2(x) for x >= 1, integer (identical on host and device): the
// leading bit and a 16-step table of the next four bits.
SB_HD inline uint32_t log2x16(uint32_t x) {
  constexpr uint8_t frac[16] = {0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 15};
  const uint32_t h = hbit32(x);
  const uint32_t f = h >= 4 ? (x >> (h - 4)) & 15 : (x << (4 - h)) & 15;
  return 16 * h + frac[f];
}

// FSE_normalizeCount restated simply: c[0..nsym) (total tot) scaled to 2^log,
// every present symbol >= 1, the largest absorbing the rounding (a symbol
// that would fall below 1 takes from the others still above 1).  Needs
// 2^log >= the present symbols.
SB_HD inline void fse_normalize(const uint32_t* c, uint32_t nsym, uint32_t tot, uint32_t log, int16_t* norm) {
  const uint32_t size = 1u << log;
  int32_t sum = 0;
  uint32_t big = 0, bigc = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    if (!c[s]) {
      norm[s] = 0;
      continue;
    }
    uint32_t v = (uint32_t)(((uint64_t)c[s] * size + tot / 2) / tot);
    if (v < 1) v = 1;
    norm[s] = (int16_t)v;
    sum += (int32_t)v;
    if (c[s] > bigc) {
      bigc = c[s];
      big = s;
    }
  }
  norm[big] = (int16_t)(norm[big] + ((int32_t)size - sum));
  while (norm[big] < 1) {
    uint32_t t = nsym;
    for (uint32_t s = 0; s < nsym; s++)
      if (s != big && norm[s] > 1 && (t == nsym || norm[s] > norm[t])) t = s;
    norm[t]--;
    norm[big]++;
  }
}

// A table log for n symbols drawn from `present` distinct values (zstd
// FSE_optimalTableLog in spirit): small for short inputs, >= 5, room for
// every present value, <= maxlog.
SB_HD inline uint32_t fse_log(uint32_t n, uint32_t present, uint32_t maxlog) {
  uint32_t log = n > 1 ? hbit32(n - 1) + 1 : 1;
  log = log > 2 ? log - 2 : 1;
  if (log > maxlog) log = maxlog;
  while ((1u << log) < present && log < maxlog) log++;
  return log < 5 ? 5 : log;
}

// FSE_writeNCount (RFC 8878 §4.1.1): accuracy log - 5 in 4 bits, then the
// counts + 1 in the variable bit widths the decoder derives from what
// remains, zero runs as 2-bit repeat flags.  Returns the bytes written.
SB_HD inline uint32_t fse_write_ncount(uint8_t* d, const int16_t* norm, uint32_t nsym, uint32_t log) {
  uint8_t* p = d;
  uint64_t acc = (uint64_t)(log - 5);
  uint32_t nb_acc = 4;
  auto flush16 = [&]() {
    while (nb_acc >= 16) {
      *p++ = (uint8_t)acc;
      *p++ = (uint8_t)(acc >> 8);
      acc >>= 16;
      nb_acc -= 16;
    }
  };
  const int32_t size = 1 << log;
  int32_t remaining = size + 1, threshold = size;
  uint32_t nbits = log + 1, sym = 0;
  bool prev0 = false;
  while (sym < nsym && remaining > 1) {
    if (prev0) {
      uint32_t start = sym;
      while (sym < nsym && !norm[sym]) sym++;
      if (sym == nsym) break;
      while (sym >= start + 24) {
        start += 24;
        acc |= (uint64_t)0xFFFFu << nb_acc;
        nb_acc += 16;
        flush16();
      }
      while (sym >= start + 3) {
        start += 3;
        acc |= (uint64_t)3u << nb_acc;
        nb_acc += 2;
      }
      acc |= (uint64_t)(sym - start) << nb_acc;
      nb_acc += 2;
      flush16();
    }
    int32_t count = norm[sym++];
    const int32_t mx = (2 * threshold - 1) - remaining;
    remaining -= count < 0 ? -count : count;
    count++;
    if (count >= threshold) count += mx;
    acc |= (uint64_t)(uint32_t)count << nb_acc;
    nb_acc += nbits;
    nb_acc -= (count < mx) ? 1u : 0u;
    prev0 = count == 1;
    while (remaining < threshold) {
      nbits--;
      threshold >>= 1;
    }
    flush16();
  }
  while (nb_acc > 0) {
    *p++ = (uint8_t)acc;
    acc >>= 8;
    nb_acc = nb_acc > 8 ? nb_acc - 8 : 0;
  }
  return (uint32_t)(p - d);
}

// Code lengths (<= kHufMaxBits) of the symbols counted in h[0..256) into
// len[0..256) (0: absent), a complete prefix code; m >= 2 symbols present.
// Plain Huffman (two smallest active nodes merged, O(m^2): m <= 256), then,
// past kHufMaxBits, lengths clamped and the Kraft sum restored by lengthening
// the longest codes under the limit and shortening where it stays <= 1.
SB_HD inline uint32_t huf_lengths(const uint32_t* h, uint32_t* len, uint32_t* wt, uint32_t* par) {
  uint32_t* sym_of = par + 512;  // [256]
  uint32_t nn = 0;
  for (uint32_t s = 0; s < 256; s++) {
    len[s] = 0;
    if (h[s]) {
      sym_of[nn] = s;
      wt[nn] = h[s];
      nn++;
    }
  }
  const uint32_t m = nn;
  for (uint32_t k = 0; k < m; k++) par[k] = 0x7FFFFFFFu;  // active (not merged), no parent
  for (uint32_t step = 0; step + 1 < m; step++) {
    uint32_t a = 0xFFFFFFFFu, b = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < nn; k++) {
      if (par[k] != 0x7FFFFFFFu) continue;  // merged already
      if (a == 0xFFFFFFFFu || wt[k] < wt[a]) {
        b = a;
        a = k;
      } else if (b == 0xFFFFFFFFu || wt[k] < wt[b]) {
        b = k;
      }
    }
    wt[nn] = wt[a] + wt[b];
    par[nn] = 0x7FFFFFFFu;
    par[a] = nn;
    par[b] = nn;
    nn++;
  }
  uint32_t maxl = 0;
  for (uint32_t k = 0; k < m; k++) {
    uint32_t d = 0;
    for (uint32_t x = k; par[x] != 0x7FFFFFFFu; x = par[x]) d++;
    len[sym_of[k]] = d;
    maxl = d > maxl ? d : maxl;
  }
  if (maxl <= kHufMaxBits) return maxl;
  // limit: clamp, then bring the Kraft sum (in units of 2^-kHufMaxBits) back to 2^kHufMaxBits
  uint32_t K = 0;
  for (uint32_t k = 0; k < m; k++) {
    uint32_t& l = len[sym_of[k]];
    if (l > kHufMaxBits) l = kHufMaxBits;
    K += 1u << (kHufMaxBits - l);
  }
  const uint32_t full = 1u << kHufMaxBits;
  while (K > full) {  // lengthen the longest code below the limit (the rarest among them)
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < m; k++) {
      const uint32_t l = len[sym_of[k]];
      if (l < kHufMaxBits && (best == 0xFFFFFFFFu || l > len[sym_of[best]] ||
                              (l == len[sym_of[best]] && h[sym_of[k]] < h[sym_of[best]])))
        best = k;
    }
    K -= 1u << (kHufMaxBits - len[sym_of[best]] - 1);
    len[sym_of[best]]++;
  }
  while (K < full) {  // shorten the longest code whose shortening keeps the sum <= 1 (the most frequent among them)
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < m; k++) {
      const uint32_t l = len[sym_of[k]];
      if (l > 1 && K + (1u << (kHufMaxBits - l)) <= full &&
          (best == 0xFFFFFFFFu || l > len[sym_of[best]] || (l == len[sym_of[best]] && h[sym_of[k]] > h[sym_of[best]])))
        best = k;
    }
    if (best == 0xFFFFFFFFu) break;
    K += 1u << (kHufMaxBits - len[sym_of[best]]);
    len[sym_of[best]]--;
  }
  maxl = 0;
  for (uint32_t k = 0; k < m; k++) maxl = len[sym_of[k]] > maxl ? len[sym_of[k]] : maxl;
  return maxl;
}

// A block's literals, without staging them: the sequence records give each
// sequence's literal run as the source bytes at its output position, then
// the block's trailing run.  A cursor walks them in either direction.
// Record: literal length (20 bits) | match length (20) << 20 | offset value (24) << 40.
struct LitCur {
  const uint8_t* src;  // the block's first output byte
  const uint64_t* recs;
  uint32_t ns, tail;   // records, trailing literals
  uint32_t k = 0, ls = 0, ps = 0;  // current run: record k (ns = the tail), its first literal, its output position
  SB_HD inline uint32_t rl(uint32_t j) const { return j < ns ? (uint32_t)(recs[j] & 0xFFFFF) : tail; }
  SB_HD inline uint32_t rm(uint32_t j) const { return j < ns ? (uint32_t)((recs[j] >> 20) & 0xFFFFF) : 0u; }
  SB_HD inline uint8_t at(uint32_t i) {
    while (i < ls) {
      k--;
      ls -= rl(k);
      ps -= rl(k) + rm(k);
    }
    while (k < ns && i >= ls + rl(k)) {
      ls += rl(k);
      ps += rl(k) + rm(k);
      k++;
    }
    return src[ps + (i - ls)];
  }
};

// The FSE-compressed Huffman weights of symbols 0..last-1 (RFC 8878 §4.2.1.2:
// a header byte < 128 = the compressed size, an FSE table description of
// accuracy log <= 6, then the weights as two interleaved FSE states, encoded
// last to first as FSE_compress_usingCTable does).  wk: work (u32 [16] counts,
// int16 [16] norms, FseT<6>, 64 spread bytes).  Returns the bytes written at
// d, 0 when they would not fit the header byte's range.
SB_HD inline uint32_t huf_fse_weights(const uint8_t* w, uint32_t nw, uint8_t* d, uint32_t* wk) {
  uint32_t* cnt = wk;
  int16_t* norm = (int16_t*)(wk + 16);
  FseCTab* ct = (FseCTab*)(wk + 32);
  uint8_t* sym = (uint8_t*)(ct + 1);
  uint32_t maxw = 0, present = 0;
  for (uint32_t s = 0; s < 16; s++) cnt[s] = 0;
  for (uint32_t i = 0; i < nw; i++) {
    cnt[w[i]]++;
    maxw = w[i] > maxw ? w[i] : maxw;
  }
  for (uint32_t s = 0; s <= maxw; s++) present += cnt[s] != 0;
  if (present < 2 || nw < 2) return 0;
  const uint32_t log = 6;
  fse_normalize(cnt, maxw + 1, nw, log, norm);
  uint8_t* q = d + 1;
  q += fse_write_ncount(q, norm, maxw + 1, log);
  fse_fill(*ct, norm, maxw + 1, log, sym);
  BitW bw{q, 0, 0};
  uint32_t st[2];
  st[(nw - 1) & 1] = fse_init(*ct, w[nw - 1]);
  st[(nw - 2) & 1] = fse_init(*ct, w[nw - 2]);
  for (int32_t i = (int32_t)nw - 3; i >= 0; i--) st[i & 1] = fse_encode(*ct, st[i & 1], w[i], bw);
  bw.add(st[1], log);  // FSE_flushCState of the second state, then the first: the decoder reads state 1 first
  bw.add(st[0], log);
  bw.close();
  const uint32_t cs = (uint32_t)(bw.p - (d + 1));
  if (cs >= 128) return 0;
  d[0] = (uint8_t)cs;
  return cs + 1;
}

// The block's literals section at d (RFC 8878 §3.1.1.3.1) from the n
// literals of the cursor; returns its length.  Huffman (Literals_Block_Type
// 2, four streams, Size_Format 10 / 11) when it comes out smaller -- the
// weight table directly represented (every literal <= 128) or FSE-compressed,
// whichever is shorter; RLE for one repeated byte; else Raw.  Codes as the
// decoder assigns them (HUF_buildCTable): per length, consecutive values in
// symbol order, longer codes below; each stream is the bit stream of its
// symbols added last to first (HUF_compress1X_usingCTable) with the end mark.
SB_HD inline uint32_t zstd_literals(LitCur& lit, uint32_t n, uint8_t* d, uint32_t* hw) {
  uint32_t* h = hw;
  uint32_t* code = hw + 256;
  uint32_t* wt = hw + 512;
  uint32_t* par = hw + 1024;  // [512] parents, [256] present symbols
  uint32_t* fw = hw + 1792;   // the weights' FSE work
  for (uint32_t s = 0; s < 256; s++) h[s] = 0;
  for (uint32_t i = 0; i < n; i++) h[lit.at(i)]++;
  uint32_t m = 0, last = 0;
  for (uint32_t s = 0; s < 256; s++)
    if (h[s]) {
      m++;
      last = s;
    }
  if (n >= 2 && m == 1) {  // RLE_Literals_Block, Size_Format 11
    put24(d, (n << 4) | 0xDu);
    d[3] = lit.at(0);
    return 4;
  }
  if (n >= 64 && m >= 2) {
    uint32_t* len = code;  // (lengths first, then the codes in place)
    const uint32_t maxb = huf_lengths(h, len, wt, par);
    // the streams' sizes: bits of each quarter + the end mark
    const uint32_t seg = (n + 3) / 4;
    uint32_t sbytes[4], tot = 0;
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t a = k * seg < n ? k * seg : n, b = (k + 1) * seg < n && k < 3 ? (k + 1) * seg : n;
      uint64_t bits = 1;
      for (uint32_t i = a; i < b; i++) bits += len[lit.at(i)];
      sbytes[k] = (uint32_t)((bits + 7) / 8);
      tot += sbytes[k];
    }
    // the weight table: FSE-compressed (written now, behind a 5-byte header
    // slot) or directly represented when every literal is <= 128 and it is shorter
    uint8_t* wts = (uint8_t*)fw + 768;  // weights of symbols 0..last-1 (past the FSE work)
    for (uint32_t s = 0; s < last; s++) wts[s] = len[s] ? (uint8_t)(maxb + 1 - len[s]) : 0u;
    const uint32_t direct = last <= 128 ? 1 + (last + 1) / 2 : 0xFFFFFFFFu;
    const uint32_t fse = huf_fse_weights(wts, last, d + 5, fw);
    const bool use_fse = fse && fse < direct;
    const uint32_t tree = use_fse ? fse : direct;
    if (tree != 0xFFFFFFFFu) {
      const uint32_t csize = tree + 6 + tot, hdr = (n < 16384 && csize < 16384) ? 4 : 5;
      const bool fits = sbytes[0] < 65536 && sbytes[1] < 65536 && sbytes[2] < 65536;
      if (fits && hdr + csize < 3 + n) {
        // codes: nbPerRank / valPerRank (HUF_buildCTable)
        uint32_t per[kHufMaxBits + 2] = {}, val[kHufMaxBits + 2] = {};
        for (uint32_t s = 0; s <= last; s++) per[len[s]]++;
        uint32_t mn = 0;
        for (uint32_t b = maxb; b > 0; b--) {
          val[b] = mn;
          mn += per[b];
          mn >>= 1;
        }
        uint8_t* q = d + hdr;
        if (use_fse) {
          if (hdr == 4)
            for (uint32_t k = 0; k < fse; k++) q[k] = d[5 + k];  // (forward copy: q < the source)
        } else {
          // 127 + (symbols below `last`), 4 bits each, first in the high nibble
          q[0] = (uint8_t)(127 + last);
          for (uint32_t s = 0; s < last; s += 2) {
            const uint32_t w0 = wts[s], w1 = s + 1 < last ? wts[s + 1] : 0u;
            q[1 + s / 2] = (uint8_t)((w0 << 4) | w1);
          }
        }
        if (hdr == 4) {
          const uint32_t v = 2u | (2u << 2) | (n << 4) | (csize << 18);
          for (uint32_t k = 0; k < 4; k++) d[k] = (uint8_t)(v >> (8 * k));
        } else {
          const uint64_t v = 2ull | (3ull << 2) | ((uint64_t)n << 4) | ((uint64_t)csize << 22);
          for (uint32_t k = 0; k < 5; k++) d[k] = (uint8_t)(v >> (8 * k));
        }
        q += tree;
        for (uint32_t s = 0; s <= last; s++) code[s] = len[s] ? (val[len[s]]++ | (len[s] << 16)) : 0u;
        for (uint32_t k = 0; k < 3; k++) {
          q[2 * k] = (uint8_t)sbytes[k];
          q[2 * k + 1] = (uint8_t)(sbytes[k] >> 8);
        }
        q += 6;
        for (uint32_t k = 0; k < 4; k++) {
          const uint32_t a = k * seg < n ? k * seg : n, b = (k + 1) * seg < n && k < 3 ? (k + 1) * seg : n;
          BitW bw{q, 0, 0};
          for (uint32_t i = b; i > a; i--) {
            const uint32_t c = code[lit.at(i - 1)];
            bw.add(c & 0xFFFFu, c >> 16);
          }
          bw.close();
          q = bw.p;
        }
        return (uint32_t)(q - d);
      }
    }
  }
  put24(d, (n << 4) | 0xCu);  // Raw_Literals_Block, Size_Format 11 (20-bit size)
  for (uint32_t i = 0; i < n; i++) d[3 + i] = lit.at(i);
  return 3 + n;
}

// Repeat offsets of a frame (RFC 8878 §3.1.2.5), {1, 4, 8} at its start.
struct ZRep {
  uint32_t r[3];
};

// One sequence table of a block (RFC 8878 §3.1.1.3.2.2): Predefined_Mode,
// RLE_Mode (one code) or FSE_Compressed_Mode with a table of the block's own
// codes, whichever costs fewer bits (codes at 1/16 bit, integer).  Writes the
// description at *q and fills t for the compressed mode; returns the mode.
template <class P>
SB_HD inline uint32_t seq_table(const uint32_t* cnt, uint32_t nsym, uint32_t ns, const int16_t* pnorm, uint32_t plog,
                                uint32_t maxlog, int16_t* norm, FseCTabL& t, uint8_t* sym, uint8_t*& q, uint32_t* rle,
                                const P& pred) {
  uint32_t present = 0, one = 0;
  for (uint32_t s = 0; s < nsym; s++)
    if (cnt[s]) {
      present++;
      one = s;
    }
  if (present == 1 && ns > 2) {  // RLE_Mode: the code, no bits per sequence
    *q++ = (uint8_t)one;
    *rle = one;
    return 1;
  }
  // predefined cost
  uint64_t cp = 0;
  for (uint32_t s = 0; s < nsym; s++)
    if (cnt[s]) {
      const int32_t pn = s < (uint32_t)pred.n ? pnorm[s] : 0;
      if (pn == 0) {
        cp = ~0ull;
        break;
      }
      cp += (uint64_t)cnt[s] * (16 * plog - log2x16(pn < 0 ? 1u : (uint32_t)pn));
    }
  const uint32_t log = fse_log(ns, present, maxlog);
  fse_normalize(cnt, nsym, ns, log, norm);
  uint64_t cc = 0;
  for (uint32_t s = 0; s < nsym; s++)
    if (cnt[s]) cc += (uint64_t)cnt[s] * (16 * log - log2x16((uint32_t)norm[s]));
  uint8_t* d = q;
  const uint32_t hb = fse_write_ncount(d, norm, nsym, log);
  cc += 16 * 8 * (uint64_t)hb;
  if (cc < cp) {
    q += hb;
    fse_fill(t, norm, nsym, log, sym);
    return 2;
  }
  return 0;  // (the description written at q is left behind and overwritten)
}

struct PredN {
  int32_t n;
};

// The Zstd blocks of one chunk (clen input bytes at src, its LZ4 block lz of
// lzlen bytes) at dst; recs = kZScratchU64 words of scratch, rep = the
// frame's repeat offsets.  A block takes up to kZSeqPerBlock LZ4 sequences;
// a match whose Zstd cost (its offset's bits plus the codes, 1/16 bit) is
// more than the literal bits it saves (the block's literal entropy) becomes
// literals; offsets equal to a repeat offset take its code.  The literals
// are read from src through the records; the sequences go out under the
// block's own FSE tables where those are cheaper than the predefined ones.
// A block that would not shrink (an upper bound of its sequences' bits is
// taken before writing them) is written Raw, and its sequences do not move
// the repeat offsets.  The last block carries Last_Block when `last`.
// Returns the bytes written.
SB_HD inline uint32_t zstd_transcode(uint8_t* lz, uint32_t lzlen, const uint8_t* src, uint32_t clen, uint8_t* dst,
                                     uint64_t* recs, bool last, ZRep& rep) {
  uint32_t p = 0, op = 0, out0 = 0;
  bool end = false;
  uint32_t* hw = (uint32_t*)(recs + kZSeqPerBlock);
  (void)clen;
  do {
    uint8_t* bh = dst + op;
    uint32_t ns = 0, dec = 0, tail = 0;
    // 1. the block's LZ4 sequences, and the histogram of their literals
    uint32_t* lh = hw;  // [256]
    for (uint32_t s = 0; s < 256; s++) lh[s] = 0;
    uint32_t nlit = 0;
    while (ns < kZSeqPerBlock) {
      if (p >= lzlen) {
        end = true;
        break;
      }
      const uint32_t tok = lz[p++];
      uint32_t l = tok >> 4;
      if (l == 15) {
        uint32_t b;
        do {
          b = lz[p++];
          l += b;
        } while (b == 255);
      }
      for (uint32_t i = 0; i < l; i++) lh[lz[p + i]]++;
      nlit += l;
      p += l;
      if (p >= lzlen) {  // the block's last literals (no match)
        tail = l;
        dec += l;
        end = true;
        break;
      }
      const uint32_t off = lz[p] | ((uint32_t)lz[p + 1] << 8);
      p += 2;
      uint32_t ml = (tok & 15) + 4;
      if ((tok & 15) == 15) {
        uint32_t b;
        do {
          b = lz[p++];
          ml += b;
        } while (b == 255);
      }
      recs[ns++] = (uint64_t)l | ((uint64_t)ml << 20) | ((uint64_t)off << 40);
      dec += l + ml;
    }
    if (p >= lzlen) end = true;
    // 2. literal entropy (1/16 bit a byte), then the matches kept and their offset values
    uint32_t H16 = 128;
    if (nlit >= 64) {
      uint64_t e = 0;
      const uint32_t ln = log2x16(nlit);
      for (uint32_t s = 0; s < 256; s++)
        if (lh[s]) e += (uint64_t)lh[s] * (ln - log2x16(lh[s]));
      H16 = (uint32_t)(e / nlit);
    }
    const ZRep rep0 = rep;
    uint32_t kept = 0, carry = 0;
    for (uint32_t i = 0; i < ns; i++) {
      const uint64_t r = recs[i];
      const uint32_t l = (uint32_t)(r & 0xFFFFF) + carry, ml = (uint32_t)((r >> 20) & 0xFFFFF),
                     off = (uint32_t)(r >> 40);
      uint32_t ofv = off + 3;
      if (l > 0) {
        if (off == rep.r[0]) ofv = 1;
        else if (off == rep.r[1]) ofv = 2;
        else if (off == rep.r[2]) ofv = 3;
      } else {
        if (off == rep.r[1]) ofv = 1;
        else if (off == rep.r[2]) ofv = 2;
        else if (rep.r[0] > 1 && off == rep.r[0] - 1) ofv = 3;
      }
      const uint32_t cost16 = ofv <= 3 ? 16 * 6 : 16 * (hbit32(ofv) + 10);
      if ((uint64_t)ml * H16 < cost16) {  // cheaper as literals
        carry = l + ml;
        continue;
      }
      carry = 0;
      if (ofv > 3) {
        rep.r[2] = rep.r[1];
        rep.r[1] = rep.r[0];
        rep.r[0] = off;
      } else {
        const uint32_t idx = ofv - 1 + (l == 0 ? 1u : 0u);
        if (idx == 1) {
          const uint32_t t0 = rep.r[0];
          rep.r[0] = rep.r[1];
          rep.r[1] = t0;
        } else if (idx >= 2) {
          const uint32_t nv = idx == 3 ? rep.r[0] - 1 : rep.r[2];
          rep.r[2] = rep.r[1];
          rep.r[1] = rep.r[0];
          rep.r[0] = nv;
        }
      }
      recs[kept++] = (uint64_t)l | ((uint64_t)ml << 20) | ((uint64_t)ofv << 40);
    }
    tail += carry;
    ns = kept;
    uint32_t lits = tail;
    for (uint32_t i = 0; i < ns; i++) lits += (uint32_t)(recs[i] & 0xFFFFF);
    // 3. literals section
    LitCur cur{src + out0, recs, ns, tail};
    uint8_t* q = bh + 3 + zstd_literals(cur, lits, bh + 3, hw);
    // 4. sequences section: header, table modes and descriptions, the bit stream
    if (ns < 128) {
      *q++ = (uint8_t)ns;
    } else {
      *q++ = (uint8_t)((ns >> 8) + 128);
      *q++ = (uint8_t)ns;
    }
    bool raw = false;
    if (ns) {
      uint32_t* cll = hw;        // [36]
      uint32_t* cof = hw + 36;   // [32]
      uint32_t* cml = hw + 68;   // [53]
      int16_t* nll = (int16_t*)(hw + 128);
      int16_t* nof = nll + 36;
      int16_t* nml = nof + 32;
      FseCTabL* tll = (FseCTabL*)(hw + 192);
      FseCTabL* tof = tll + 1;
      FseCTabL* tml = tof + 1;
      uint8_t* sym = (uint8_t*)(tml + 1);
      for (uint32_t s = 0; s < 128; s++) hw[s] = 0;
      uint64_t extra = 0;
      for (uint32_t i = 0; i < ns; i++) {
        const uint64_t r = recs[i];
        const uint32_t ll = (uint32_t)(r & 0xFFFFF), ml = (uint32_t)((r >> 20) & 0xFFFFF), ofv = (uint32_t)(r >> 40);
        const uint32_t llc = ll_code(ll), mlc = ml_code(ml), ofc = hbit32(ofv);
        cll[llc]++;
        cml[mlc]++;
        cof[ofc]++;
        extra += kLLBitsT[llc] + kMLBitsT[mlc] + ofc;
      }
      uint8_t* modes = q++;
      uint32_t rll = 0, rof = 0, rml = 0;
      const uint32_t mll = seq_table(cll, 36, ns, kLLNorm, kLLLog, 9, nll, *tll, sym, q, &rll, PredN{36});
      const uint32_t mof = seq_table(cof, 32, ns, kOFNorm, kOFLog, 8, nof, *tof, sym, q, &rof, PredN{29});
      const uint32_t mml = seq_table(cml, 53, ns, kMLNorm, kMLLog, 9, nml, *tml, sym, q, &rml, PredN{53});
      *modes = (uint8_t)((mll << 6) | (mof << 4) | (mml << 2));
      // an upper bound of the bit stream: every state emission at its table log
      const uint32_t lgll = mll == 2 ? hbit32(tll->st[0]) : mll == 0 ? kLLLog : 0u;
      const uint32_t lgof = mof == 2 ? hbit32(tof->st[0]) : mof == 0 ? kOFLog : 0u;
      const uint32_t lgml = mml == 2 ? hbit32(tml->st[0]) : mml == 0 ? kMLLog : 0u;
      const uint64_t ub = (uint64_t)ns * (lgll + lgof + lgml) + extra + 1;
      const uint32_t pre = (uint32_t)(q - (bh + 3));
      if ((uint64_t)pre + (ub + 7) / 8 >= dec) {
        raw = true;
      } else {
        BitW bw{q, 0, 0};
        uint64_t r = recs[ns - 1];
        uint32_t ll = (uint32_t)(r & 0xFFFFF), ml = (uint32_t)((r >> 20) & 0xFFFFF), ofv = (uint32_t)(r >> 40);
        uint32_t llc = ll_code(ll), mlc = ml_code(ml), ofc = hbit32(ofv);
        auto init = [&](uint32_t m, const FseCTab& pt, const FseCTabL& t, uint32_t s) -> uint32_t {
          return m == 2 ? fse_init(t, s) : m == 0 ? fse_init(pt, s) : 0u;
        };
        auto enc = [&](uint32_t m, const FseCTab& pt, const FseCTabL& t, uint32_t st, uint32_t s) -> uint32_t {
          return m == 2 ? fse_encode(t, st, s, bw) : m == 0 ? fse_encode(pt, st, s, bw) : 0u;
        };
        uint32_t sML = init(mml, kMLc, *tml, mlc), sOF = init(mof, kOFc, *tof, ofc), sLL = init(mll, kLLc, *tll, llc);
        bw.add(ll - kLLBaseT[llc], kLLBitsT[llc]);
        bw.add(ml - kMLBaseT[mlc], kMLBitsT[mlc]);
        bw.add(ofv - (1u << ofc), ofc);
        for (int32_t i = (int32_t)ns - 2; i >= 0; i--) {
          r = recs[i];
          ll = (uint32_t)(r & 0xFFFFF), ml = (uint32_t)((r >> 20) & 0xFFFFF), ofv = (uint32_t)(r >> 40);
          llc = ll_code(ll), mlc = ml_code(ml), ofc = hbit32(ofv);
          sOF = enc(mof, kOFc, *tof, sOF, ofc);
          sML = enc(mml, kMLc, *tml, sML, mlc);
          sLL = enc(mll, kLLc, *tll, sLL, llc);
          bw.add(ll - kLLBaseT[llc], kLLBitsT[llc]);
          bw.add(ml - kMLBaseT[mlc], kMLBitsT[mlc]);
          bw.add(ofv - (1u << ofc), ofc);
        }
        bw.add(sML, lgml);
        bw.add(sOF, lgof);
        bw.add(sLL, lgll);
        bw.close();
        q = bw.p;
      }
    }
    const bool lb = last && end;
    const uint32_t content = (uint32_t)(q - (bh + 3));
    if (raw || content >= dec) {  // Raw_Block: the chunk bytes themselves; the repeat offsets stay
      put24(bh, (dec << 3) | (lb ? 1u : 0u));
      for (uint32_t i = 0; i < dec; i++) bh[3 + i] = src[out0 + i];
      op += 3 + dec;
      rep = rep0;
    } else {
      put24(bh, (content << 3) | (2u << 1) | (lb ? 1u : 0u));
      op += 3 + content;
    }
    out0 += dec;
  } while (!end);
  return op;
}

// The empty input's frame: header + one empty last Raw block.
SB_HD inline uint32_t zstd_empty(uint8_t* d) {
  const uint32_t h = zstd_frame_header(d, 0);
  put24(d + h, 1u);
  return h + 3;
}

}  // namespace sbz
