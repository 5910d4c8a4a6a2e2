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

// FSE compression table of a normalized distribution (zstd
// FSE_buildCTable_wksp): the state table after the symbol spread the decoder
// uses (step = size/2 + size/8 + 3, -1 symbols at the top), and per symbol
// deltaFindState / deltaNbBits.
struct FseCTab {
  uint16_t st[64];
  int32_t dfs[53];
  uint32_t dnb[53];
};

constexpr uint32_t hbit(uint32_t v) {
  uint32_t r = 0;
  while (v >>= 1) r++;
  return r;
}

constexpr FseCTab fse_ctab(const int16_t* norm, uint32_t nsym, uint32_t log) {
  FseCTab t{};
  const uint32_t size = 1u << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  uint8_t sym[64] = {};
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

SB_HD inline uint32_t fse_init(const FseCTab& t, uint32_t s) {
  const uint32_t nb = (t.dnb[s] + (1u << 15)) >> 16, v = (nb << 16) - t.dnb[s];
  return t.st[(int32_t)(v >> nb) + t.dfs[s]];
}
SB_HD inline uint32_t fse_encode(const FseCTab& t, uint32_t st, uint32_t s, BitW& bw) {
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

// Scratch of zstd_transcode: the sequence records, then the literals' Huffman
// work area (u32): histogram [256], codes [256] (value | bits << 16), tree
// node weights [257], parents [257] and the present symbols [129].
constexpr uint32_t kZScratchU64 = kZSeqPerBlock + 1024;  // 24 KiB
constexpr uint32_t kHufMaxBits = 11;

// Code lengths (<= kHufMaxBits) of the symbols counted in h[0..256) into
// len[0..256) (0: absent), a complete prefix code; m >= 2 symbols present.
// Plain Huffman (two smallest active nodes merged, O(m^2): m <= 129), then,
// past kHufMaxBits, lengths clamped and the Kraft sum restored by lengthening
// the longest codes under the limit and shortening where it stays <= 1.
SB_HD inline uint32_t huf_lengths(const uint32_t* h, uint32_t* len, uint32_t* wt, uint32_t* par) {
  uint32_t* sym_of = par + 260;  // [129]
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
  return kHufMaxBits;
}

// The block's literals section at d (RFC 8878 §3.1.1.3.1) from the n staged
// literal bytes at lit; returns its length.  Huffman (Literals_Block_Type 2,
// four streams, Size_Format 10 / 11) when every literal is <= 128 (a directly
// represented weight table: 4 bits a symbol below the largest, whose weight
// is implied) and the section comes out smaller; RLE for one repeated byte;
// else Raw.  Codes as the decoder assigns them (HUF_buildCTable): per length,
// consecutive values in symbol order, longer codes below; each stream is the
// bit stream of its symbols added last to first (HUF_compress1X_usingCTable)
// with the end mark.
SB_HD inline uint32_t zstd_literals(const uint8_t* lit, uint32_t n, uint8_t* d, uint32_t* hw) {
  uint32_t* h = hw;
  uint32_t* code = hw + 256;
  uint32_t* wt = hw + 512;
  uint32_t* par = hw + 800;
  for (uint32_t s = 0; s < 256; s++) h[s] = 0;
  for (uint32_t i = 0; i < n; i++) h[lit[i]]++;
  uint32_t m = 0, last = 0;
  for (uint32_t s = 0; s < 256; s++)
    if (h[s]) {
      m++;
      last = s;
    }
  if (n >= 2 && m == 1) {  // RLE_Literals_Block, Size_Format 11
    put24(d, (n << 4) | 0xDu);
    d[3] = lit[0];
    return 4;
  }
  if (n >= 256 && m >= 2 && last <= 128) {
    uint32_t* len = code;  // (lengths first, then the codes in place)
    const uint32_t maxb = huf_lengths(h, len, wt, par);
    // the streams' sizes: bits of each quarter + the end mark
    const uint32_t seg = (n + 3) / 4;
    uint32_t sbytes[4], tot = 0;
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t a = k * seg < n ? k * seg : n, b = (k + 1) * seg < n && k < 3 ? (k + 1) * seg : n;
      uint64_t bits = 1;
      for (uint32_t i = a; i < b; i++) bits += len[lit[i]];
      sbytes[k] = (uint32_t)((bits + 7) / 8);
      tot += sbytes[k];
    }
    const uint32_t tree = 1 + (last + 1) / 2, csize = tree + 6 + tot, hdr = (n < 16384 && csize < 16384) ? 4 : 5;
    bool fits = sbytes[0] < 65536 && sbytes[1] < 65536 && sbytes[2] < 65536;
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
      // header
      if (hdr == 4) {
        const uint32_t v = 2u | (2u << 2) | (n << 4) | (csize << 18);
        for (uint32_t k = 0; k < 4; k++) d[k] = (uint8_t)(v >> (8 * k));
      } else {
        const uint64_t v = 2ull | (3ull << 2) | ((uint64_t)n << 4) | ((uint64_t)csize << 22);
        for (uint32_t k = 0; k < 5; k++) d[k] = (uint8_t)(v >> (8 * k));
      }
      uint8_t* q = d + hdr;
      // the weight table: 127 + (symbols below `last`), 4 bits each, first in the high nibble
      q[0] = (uint8_t)(127 + last);
      for (uint32_t s = 0; s < last; s += 2) {
        const uint32_t w0 = len[s] ? maxb + 1 - len[s] : 0, w1 = s + 1 < last && len[s + 1] ? maxb + 1 - len[s + 1] : 0;
        q[1 + s / 2] = (uint8_t)((w0 << 4) | w1);
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
          const uint32_t c = code[lit[i - 1]];
          bw.add(c & 0xFFFFu, c >> 16);
        }
        bw.close();
        q = bw.p;
      }
      return (uint32_t)(q - d);
    }
  }
  put24(d, (n << 4) | 0xCu);  // Raw_Literals_Block, Size_Format 11 (20-bit size)
  for (uint32_t i = 0; i < n; i++) d[3 + i] = lit[i];
  return 3 + n;
}

// The Zstd blocks of one chunk (clen input bytes at src, its LZ4 block lz of
// lzlen bytes) at dst; recs = kZScratchU64 words of scratch.  A block's
// literals are staged in lz itself, compacted behind the parse (the write
// index never passes the read index).  The last block carries Last_Block
// when `last`.  Returns the bytes written.
SB_HD inline uint32_t zstd_transcode(uint8_t* lz, uint32_t lzlen, const uint8_t* src, uint32_t clen, uint8_t* dst,
                                     uint64_t* recs, bool last) {
  uint32_t p = 0, op = 0, out0 = 0;
  bool end = false;
  do {
    uint8_t* bh = dst + op;
    uint8_t* lit = lz + p;  // the block's literals, staged
    uint32_t nlit = 0, ns = 0, dec = 0;
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
      for (uint32_t i = 0; i < l; i++) lit[nlit + i] = lz[p + i];
      nlit += l;
      p += l;
      dec += l;
      if (p >= lzlen) {  // the block's last literals (no match)
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
      dec += ml;
    }
    if (p >= lzlen) end = true;
    uint8_t* q = bh + 3 + zstd_literals(lit, nlit, bh + 3, (uint32_t*)(recs + kZSeqPerBlock));
    // Sequences_Section_Header
    if (ns < 128) {
      *q++ = (uint8_t)ns;
    } else {
      *q++ = (uint8_t)((ns >> 8) + 128);
      *q++ = (uint8_t)ns;
    }
    if (ns) {
      *q++ = 0;  // Predefined_Mode for literal lengths, offsets and match lengths
      BitW bw{q, 0, 0};
      uint64_t r = recs[ns - 1];
      uint32_t ll = (uint32_t)(r & 0xFFFFF), ml = (uint32_t)((r >> 20) & 0xFFFFF), ofv = (uint32_t)(r >> 40) + 3;
      uint32_t llc = ll_code(ll), mlc = ml_code(ml), ofc = hbit32(ofv);
      uint32_t sML = fse_init(kMLc, mlc), sOF = fse_init(kOFc, ofc), sLL = fse_init(kLLc, llc);
      bw.add(ll - kLLBaseT[llc], kLLBitsT[llc]);
      bw.add(ml - kMLBaseT[mlc], kMLBitsT[mlc]);
      bw.add(ofv - (1u << ofc), ofc);
      for (int32_t i = (int32_t)ns - 2; i >= 0; i--) {
        r = recs[i];
        ll = (uint32_t)(r & 0xFFFFF), ml = (uint32_t)((r >> 20) & 0xFFFFF), ofv = (uint32_t)(r >> 40) + 3;
        llc = ll_code(ll), mlc = ml_code(ml), ofc = hbit32(ofv);
        sOF = fse_encode(kOFc, sOF, ofc, bw);
        sML = fse_encode(kMLc, sML, mlc, bw);
        sLL = fse_encode(kLLc, sLL, llc, bw);
        bw.add(ll - kLLBaseT[llc], kLLBitsT[llc]);
        bw.add(ml - kMLBaseT[mlc], kMLBitsT[mlc]);
        bw.add(ofv - (1u << ofc), ofc);
      }
      bw.add(sML, kMLLog);
      bw.add(sOF, kOFLog);
      bw.add(sLL, kLLLog);
      bw.close();
      q = bw.p;
    }
    const bool lb = last && end;
    const uint32_t content = (uint32_t)(q - (bh + 3));
    if (content >= dec) {  // Raw_Block: the chunk bytes themselves
      put24(bh, (dec << 3) | (lb ? 1u : 0u));
      for (uint32_t i = 0; i < dec; i++) bh[3 + i] = src[out0 + i];
      op += 3 + dec;
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
