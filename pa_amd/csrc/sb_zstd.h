// sb_zstd.h -- one-wave Zstd frame decoder (RFC 8878) into LDS: the Zstd leg
// of CommonCompression (compression/basic.rs:93-97: the frames whose
// decompressed sizes add up to the page header's usize -- the writer emits
// one; ZSTD_decompress also takes several, skippable frames between them and
// content checksums, verified here with XXH64).  The reference calls
// libzstd 1.4.8 (zstd 0.11 crate); the checks below follow that library's
// acceptance rules so a page the reference rejects is rejected here.
//
// Design (one wavefront per stream, everything in LDS):
//   * the frame / block / section headers are parsed by all 64 lanes in
//     lock-step (the values are wave-uniform);
//   * FSE and Huffman tables are built by lane 0 into an LDS table area;
//   * the (up to 4) Huffman literal streams are decoded by lanes 0..3, the
//     literals landing at the TAIL of the output window (olen - litSize):
//     every sequence writes below the literals it has not read yet, since the
//     frames' output is exactly olen bytes (op + ml <= lp is checked anyway);
//   * sequences are decoded by lane 0 in batches of 64 and executed by the
//     whole wave: literal copies and matches sourced before the batch in
//     parallel (one sequence per lane), the rest in order, 64 bytes a step.
// Included by sb_decode.hip after the LZ4 / Snappy wave decoders (needs
// LdsSrc, lds_u8 and the ST_* codes).
#pragma once

namespace zs {

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) int16_t lds_s16;

constexpr uint32_t kBlockMax = 128 * 1024;  // ZSTD_BLOCKSIZE_MAX
constexpr uint32_t kLitFast = 16, kMatchFast = 32;

// Table area layout (bytes from its 16-aligned base).  FSE cell (u64):
// [15:0] next-state base, [23:16] state bits, [31:24] extra bits, [63:32]
// base value (the symbol itself for the Huffman-weight table).
// The Huffman table comes last: 2048 entries (table log <= 11, what the
// writer's encoder emits) fit the minimum area, a log-12 table needs 4096.
constexpr uint32_t kOffLL = 0;        // 512 cells
constexpr uint32_t kOffML = 4096;     // 512 cells
constexpr uint32_t kOffOF = 8192;     // 256 cells
constexpr uint32_t kOffHWT = 10240;   // 64 cells (Huffman weights, log <= 6)
constexpr uint32_t kOffNorm = 10752;  // 256 x s16 normalized counts
constexpr uint32_t kOffNext = 11264;  // 256 x u16 symbolNext / weight ranks
constexpr uint32_t kOffHW = 11776;    // 256 x u8 Huffman weights
constexpr uint32_t kOffSeq = 12032;   // 5 x 64 x u32 sequence batch
constexpr uint32_t kOffMisc = 13312;  // 64 x u32 lane-0 -> wave results
constexpr uint32_t kOffHUF = 13568;   // u16 entries: symbol | bits << 8
constexpr uint32_t kBytes11 = kOffHUF + 2 * 2048, kBytes12 = kOffHUF + 2 * 4096;
static_assert(kBytes11 <= sb::kZTablesBytes && kBytes12 <= sb::kZTablesMax, "Zstd table area");

// Literals_Length / Match_Length codes (RFC 8878 3.1.1.3.2.1.1)
__constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,   16,    18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,  16,   17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,  34,   35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// predefined distributions (RFC 8878 3.1.1.3.2.2)
__constant__ int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2,  2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,  1,  1,  1,  1,  1,  1,  1,  1,  1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

enum : int { K_RAW = 0, K_LL = 1, K_ML = 2, K_OF = 3 };

struct Tabs {
  lds_u64* ll;
  lds_u64* ml;
  lds_u64* of;
  lds_u64* hwt;
  lds_u16* huf;
  lds_s16* norm;
  lds_u16* next;
  lds_u8* hw;
  lds_u32* seq;
  lds_u32* misc;
  __device__ explicit Tabs(lds_u8* b)
      : ll((lds_u64*)(b + kOffLL)), ml((lds_u64*)(b + kOffML)), of((lds_u64*)(b + kOffOF)),
        hwt((lds_u64*)(b + kOffHWT)), huf((lds_u16*)(b + kOffHUF)), norm((lds_s16*)(b + kOffNorm)),
        next((lds_u16*)(b + kOffNext)), hw(b + kOffHW), seq((lds_u32*)(b + kOffSeq)), misc((lds_u32*)(b + kOffMisc)) {}
};

__device__ __forceinline__ void zsync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t hibit(uint32_t v) { return 31u - __builtin_clz(v); }

// Backward bit stream (RFC 8878 4.1): the highest set bit of the last byte
// marks the end; bits are consumed from there down.  Bits below the stream
// start read as zero and drive pos negative (libzstd's "overflow" state).
template <class Src>
struct RevBits {
  Src in;
  int32_t pos;  // bits not yet consumed
  int32_t wlo;  // stream bit of cont bit 0 (a multiple of 8)
  uint64_t cont;
  __device__ bool init(const Src& src, uint32_t start, uint32_t len) {
    in = src.at(start);
    pos = 0;
    wlo = 0;
    cont = 0;
    if (!len) return false;
    const uint32_t last = in.u8(len - 1);
    if (!last) return false;
    pos = (int32_t)(8 * (len - 1) + hibit(last));
    refill();
    return true;
  }
  // after a refill at least 57 bits sit below pos in cont (or all of them)
  __device__ __forceinline__ void refill() {
    const int32_t b = pos > 64 ? (pos - 57) >> 3 : 0;
    wlo = 8 * b;
    cont = in.u64((uint32_t)b);
  }
  __device__ __forceinline__ uint32_t peek(uint32_t n) const {
    const int32_t lo = pos - (int32_t)n;
    uint64_t v;
    if (lo >= wlo) {
      v = cont >> (lo - wlo);
    } else {
      const int32_t sh = wlo - lo;
      v = sh >= 64 ? 0ull : cont << sh;
    }
    return (uint32_t)v & ((1u << n) - 1);
  }
  __device__ __forceinline__ uint32_t read(uint32_t n) {
    if (!n) return 0;
    if (pos - wlo < (int32_t)n) refill();
    const uint32_t v = peek(n);
    pos -= (int32_t)n;
    return v;
  }
};

__device__ __forceinline__ uint64_t mkcell(int kind, uint32_t s, uint32_t nb, uint32_t nxt) {
  uint32_t add = 0, base = s;
  if (kind == K_LL) {
    add = kLLBits[s];
    base = kLLBase[s];
  } else if (kind == K_ML) {
    add = kMLBits[s];
    base = kMLBase[s];
  } else if (kind == K_OF) {
    add = s;
    base = 1u << s;
  }
  return (uint64_t)(nxt | (nb << 16) | (add << 24)) | ((uint64_t)base << 32);
}

// FSE_readNCount (RFC 8878 4.1.1; libzstd fse_decompress.c): normalized
// counts, forward bits.  Returns the header bytes used, 0 on error.
template <class Src>
__device__ uint32_t read_ncount(const Src& in, uint32_t p, uint32_t avail, lds_s16* norm, uint32_t maxsym,
                                uint32_t maxlog, uint32_t* al_out, uint32_t* nsym_out) {
  if (!avail) return 0;
  uint32_t bp = 0;
  auto bits = [&](uint32_t n) -> uint32_t {
    return (uint32_t)(in.u64(p + (bp >> 3)) >> (bp & 7)) & ((1u << n) - 1);
  };
  const uint32_t al = bits(4) + 5;
  bp = 4;
  if (al > maxlog) return 0;
  const uint32_t lim = 8 * avail + 32;
  int32_t remaining = (1 << al) + 1, threshold = 1 << al;
  uint32_t nb = al + 1, sym = 0;
  bool prev0 = false;
  while (remaining > 1 && sym <= maxsym) {
    if (prev0) {  // 2-bit repeat flags of zero-probability symbols
      uint32_t n0 = sym;
      for (;;) {
        const uint32_t r = bits(2);
        bp += 2;
        n0 += r;
        if (r != 3) break;
        if (bp > lim) return 0;
      }
      if (n0 > maxsym) return 0;
      while (sym < n0) norm[sym++] = 0;
    }
    const int32_t mx = 2 * threshold - 1 - remaining;
    int32_t cnt = (int32_t)bits(nb - 1);
    if (cnt < mx) {
      bp += nb - 1;
    } else {
      cnt = (int32_t)bits(nb);
      if (cnt >= threshold) cnt -= mx;
      bp += nb;
    }
    cnt--;  // -1 = "less than 1"
    remaining -= cnt < 0 ? -cnt : cnt;
    norm[sym++] = (int16_t)cnt;
    prev0 = cnt == 0;
    while (remaining < threshold && threshold > 1) {
      nb--;
      threshold >>= 1;
    }
    if (bp > lim) return 0;
  }
  if (remaining != 1) return 0;
  const uint32_t used = (bp + 7) >> 3;
  if (used > avail) return 0;
  *al_out = al;
  *nsym_out = sym;
  return used;
}

// FSE decoding table from t.norm[0..nsym) (RFC 8878 4.1.1: "-1" symbols at
// the top, the others spread by step (size/2 + size/8 + 3), then states
// numbered in position order).  Lane 0.
__device__ bool build_fse(const Tabs& t, uint32_t nsym, uint32_t al, lds_u64* cells, int kind) {
  const uint32_t size = 1u << al, mask = size - 1;
  int32_t high = (int32_t)size - 1;
  for (uint32_t s = 0; s < nsym; s++) {
    const int32_t c = t.norm[s];
    if (c == -1) {
      if (high < 0) return false;
      cells[high--] = (uint64_t)s << 32;
      t.next[s] = 1;
    } else {
      t.next[s] = (uint16_t)(c > 0 ? c : 0);
    }
  }
  if (high < 0) return false;
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  uint32_t pos = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    const int32_t c = t.norm[s];
    for (int32_t i = 0; i < c; i++) {
      cells[pos] = (uint64_t)s << 32;
      do pos = (pos + step) & mask;
      while ((int32_t)pos > high);
    }
  }
  if (pos != 0) return false;
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t s = (uint32_t)(cells[u] >> 32);
    const uint32_t ns = t.next[s];
    t.next[s] = (uint16_t)(ns + 1);
    const uint32_t nb = al - hibit(ns);
    cells[u] = mkcell(kind, s, nb, (ns << nb) - size);
  }
  return true;
}

// Huffman tree description (RFC 8878 4.2.1) + the single-symbol decoding
// table (libzstd HUF_readStats / HUF_readDTableX1).  Lane 0.
template <class Src>
__device__ uint32_t read_huf(const Src& in, uint32_t p, uint32_t avail, const Tabs& t, bool big, uint32_t* tl_out,
                             uint32_t* used) {
  if (!avail) return ST_CODEC;
  const uint32_t hb = in.u8(p);
  uint32_t nw = 0;
  if (hb >= 128) {  // direct: 4-bit weights, first in the high nibble
    nw = hb - 127;
    const uint32_t nbytes = (nw + 1) >> 1;
    if (nbytes + 1 > avail) return ST_CODEC;
    for (uint32_t i = 0; i < nw; i++) t.hw[i] = (uint8_t)((in.u8(p + 1 + (i >> 1)) >> ((i & 1) ? 0 : 4)) & 15);
    *used = nbytes + 1;
  } else {  // FSE-compressed weights, two interleaved states
    const uint32_t cs = hb;
    if (cs + 1 > avail) return ST_CODEC;
    uint32_t al = 0, nsym = 0;
    const uint32_t nc = read_ncount(in, p + 1, cs, t.norm, 255, 6, &al, &nsym);
    if (!nc || !build_fse(t, nsym, al, t.hwt, K_RAW)) return ST_CODEC;
    RevBits<Src> br;
    if (!br.init(in, p + 1 + nc, cs - nc)) return ST_CODEC;
    uint32_t s1 = br.read(al), s2 = br.read(al);
    for (;;) {
      if (nw > 253) return ST_CODEC;
      uint64_t c = t.hwt[s1];
      t.hw[nw++] = (uint8_t)(c >> 32);
      s1 = (uint32_t)(c & 0xFFFF) + br.read((uint32_t)(c >> 16) & 0xFF);
      if (br.pos < 0) {
        t.hw[nw++] = (uint8_t)(t.hwt[s2] >> 32);
        break;
      }
      if (nw > 253) return ST_CODEC;
      c = t.hwt[s2];
      t.hw[nw++] = (uint8_t)(c >> 32);
      s2 = (uint32_t)(c & 0xFFFF) + br.read((uint32_t)(c >> 16) & 0xFF);
      if (br.pos < 0) {
        t.hw[nw++] = (uint8_t)(t.hwt[s1] >> 32);
        break;
      }
    }
    *used = cs + 1;
  }
  // the last weight is implied: the weights must sum to a power of two
  uint32_t total = 0, rank1 = 0;
  for (uint32_t i = 0; i < nw; i++) {
    const uint32_t w = t.hw[i];
    if (w >= 12) return ST_CODEC;  // HUF_TABLELOG_MAX
    total += (1u << w) >> 1;
    rank1 += w == 1;
  }
  if (!total) return ST_CODEC;
  const uint32_t tl = hibit(total) + 1;
  if (tl > 12) return ST_CODEC;
  const uint32_t rest = (1u << tl) - total, lw = hibit(rest) + 1;
  if ((1u << hibit(rest)) != rest) return ST_CODEC;
  t.hw[nw] = (uint8_t)lw;
  rank1 += lw == 1;
  if (rank1 < 2 || (rank1 & 1)) return ST_CODEC;
  if (tl > 11 && !big) return ST_NYI;  // no room for a 4096-entry table here
  const uint32_t nsym = nw + 1;
  // rank starts: weight 1 (longest codes) first, symbols in order within a weight
  for (uint32_t w = 0; w <= tl; w++) t.next[w] = 0;
  for (uint32_t i = 0; i < nsym; i++) t.next[t.hw[i]]++;
  uint32_t start = 0;
  for (uint32_t w = 1; w <= tl; w++) {
    const uint32_t c = t.next[w];
    t.next[w] = (uint16_t)start;
    start += c << (w - 1);
  }
  for (uint32_t i = 0; i < nsym; i++) {
    const uint32_t w = t.hw[i];
    if (!w) continue;
    const uint32_t len = 1u << (w - 1), st = t.next[w];
    t.next[w] = (uint16_t)(st + len);
    const uint32_t e = i | ((tl + 1 - w) << 8);
    if (len >= 4 && !(st & 3)) {
      const uint64_t e4 = (uint64_t)e * 0x0001000100010001ull;
      lds_u64* d = (lds_u64*)(t.huf + st);
      for (uint32_t k = 0; k < len / 4; k++) d[k] = e4;
    } else {
      for (uint32_t k = 0; k < len; k++) t.huf[st + k] = (uint16_t)e;
    }
  }
  *tl_out = tl;
  return ST_OK;
}

// One sequence table (RFC 8878 3.1.1.3.2.1): Predefined / RLE /
// FSE_Compressed / Repeat.  Lane 0; *q advances past the description.
template <class Src>
__device__ uint32_t seq_table(const Src& in, uint32_t* q, uint32_t bend, uint32_t mode, int kind, const Tabs& t,
                              lds_u64* cells, uint32_t* al, bool* have, bool* pre) {
  const uint32_t maxsym = kind == K_LL ? 35 : kind == K_ML ? 52 : 31;
  const uint32_t maxlog = kind == K_OF ? 8 : 9;
  if (mode == 0) {
    const uint32_t n = kind == K_LL ? 36 : kind == K_ML ? 53 : 29;
    const uint32_t dal = kind == K_OF ? 5 : 6;
    if (!*pre) {
      for (uint32_t s = 0; s < n; s++) t.norm[s] = kind == K_LL ? kLLDef[s] : kind == K_ML ? kMLDef[s] : kOFDef[s];
      if (!build_fse(t, n, dal, cells, kind)) return ST_CODEC;
      *pre = true;
    }
    *al = dal;
    *have = true;
    return ST_OK;
  }
  if (mode == 1) {
    if (*q >= bend) return ST_CODEC;
    const uint32_t s = in.u8((*q)++);
    if (s > maxsym) return ST_CODEC;
    cells[0] = mkcell(kind, s, 0, 0);
    *al = 0;
    *have = true;
    *pre = false;
    return ST_OK;
  }
  if (mode == 2) {
    uint32_t a = 0, ns = 0;
    const uint32_t nc = read_ncount(in, *q, bend - *q, t.norm, maxsym, maxlog, &a, &ns);
    if (!nc || !build_fse(t, ns, a, cells, kind)) return ST_CODEC;
    *q += nc;
    *al = a;
    *have = true;
    *pre = false;
    return ST_OK;
  }
  return *have ? ST_OK : ST_CODEC;  // Repeat needs a table from an earlier block
}

// wave copies (all 64 lanes, wave-uniform arguments)
template <class O>
__device__ __forceinline__ void copy_fwd(O out, uint32_t dst, uint32_t src, uint32_t n) {  // dst <= src
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t c = 0; c < n; c += 64)
    if (lane < n - c) out[dst + c + lane] = out[src + c + lane];
}
template <class O>
__device__ __forceinline__ void copy_match(O out, uint32_t d, uint32_t off, uint32_t ml) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t c = 0; c < ml; c += 64) {
    if (lane < ml - c) {
      const uint32_t x = d + c;
      const uint32_t q = off >= 64 ? x + lane - off : x - off + lane % off;
      out[x + lane] = out[q];
    }
  }
}
template <class O, class Src>
__device__ __forceinline__ void copy_in(O out, uint32_t dst, const Src& in, uint32_t src, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t c = 0; c < n; c += 64)
    if (lane < n - c) out[dst + c + lane] = (uint8_t)in.u8(src + c + lane);
}
template <class O>
__device__ __forceinline__ void fill(O out, uint32_t dst, uint8_t b, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t c = 0; c < n; c += 64)
    if (lane < n - c) out[dst + c + lane] = b;
}

// Execute a decoded batch: t.seq = [ll | ml | off | dst | lit src] x 64.
// op0 / lp0: output and literal positions at the batch start, wend: the
// output position after it.
template <class O>
__device__ void exec_batch(O out, const Tabs& t, uint32_t cnt, uint32_t op0, uint32_t lp0, uint32_t wend) {
  const uint32_t lane = threadIdx.x & 63;
  const bool v = lane < cnt;
  uint32_t ll = 0, ml = 0, off = 1, d = 0, ls = 0;
  if (v) {
    ll = t.seq[lane];
    ml = t.seq[64 + lane];
    off = t.seq[128 + lane];
    d = t.seq[192 + lane];
    ls = t.seq[256 + lane];
  }
  if (wend > lp0) {  // the batch writes over its own literals: strictly in order
    for (uint32_t j = 0; j < cnt; j++) {
      const uint32_t L = __builtin_amdgcn_readlane(ll, j), D = __builtin_amdgcn_readlane(d, j);
      copy_fwd(out, D, __builtin_amdgcn_readlane(ls, j), L);
      copy_match(out, D + L, __builtin_amdgcn_readlane(off, j), __builtin_amdgcn_readlane(ml, j));
    }
    return;
  }
  // 1. literals (every destination lies below every literal source)
  const bool sl = v && ll <= kLitFast;
  for (uint32_t i = 0; __ballot(sl && i < ll); i++)
    if (sl && i < ll) out[d + i] = out[ls + i];
  for (uint64_t m = __ballot(v && ll > kLitFast); m; m &= m - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    copy_fwd(out, __builtin_amdgcn_readlane(d, l), __builtin_amdgcn_readlane(ls, l), __builtin_amdgcn_readlane(ll, l));
  }
  // 2. short matches whose source ends before the batch
  const uint32_t dm = d + ll, src = dm - off;
  const bool haz = v && (src + ml > op0 || ml > kMatchFast);
  const bool fr = v && !haz;
  for (uint32_t i = 0; __ballot(fr && i < ml); i++)
    if (fr && i < ml) out[dm + i] = out[src + i];
  // 3. the others in sequence order
  for (uint64_t m = __ballot(haz); m; m &= m - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    copy_match(out, __builtin_amdgcn_readlane(dm, l), __builtin_amdgcn_readlane(off, l),
               __builtin_amdgcn_readlane(ml, l));
  }
}

// XXH64 (seed 0) of out[s, s + len), low 32 bits: the frame content
// checksum (RFC 8878 3.1.1).  Lanes 0-3 run the four stripe accumulators,
// every lane the (uniform) merge and tail.
constexpr uint64_t kX1 = 11400714785074694791ull, kX2 = 14029467366897019727ull, kX3 = 1609587929392839161ull,
                   kX4 = 9650029242287828579ull, kX5 = 2870177450012600261ull;
__device__ __forceinline__ uint64_t xrotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) { return xrotl(acc + in * kX2, 31) * kX1; }
template <class O>
__device__ uint32_t xxh64_low32(O out, uint32_t s, uint32_t len) {
  const uint32_t lane = threadIdx.x & 63;
  auto rd = [&](uint32_t i, uint32_t nb) {
    uint64_t v = 0;
    for (uint32_t k = 0; k < nb; k++) v |= (uint64_t)(uint8_t)out[s + i + k] << (8 * k);
    return v;
  };
  uint64_t h;
  uint32_t i = 0;
  if (len >= 32) {
    uint64_t v = lane == 0 ? kX1 + kX2 : lane == 1 ? kX2 : lane == 2 ? 0ull : 0ull - kX1;
    const uint32_t stripes = len / 32;
    if (lane < 4)
      for (uint32_t k = 0; k < stripes; k++) v = xround(v, rd(32 * k + 8 * lane, 8));
    __builtin_amdgcn_wave_barrier();
    uint64_t a[4];
#pragma unroll
    for (int l = 0; l < 4; l++) {
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), l, 64);
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, l, 64);
      a[l] = ((uint64_t)hi << 32) | lo;
    }
    h = xrotl(a[0], 1) + xrotl(a[1], 7) + xrotl(a[2], 12) + xrotl(a[3], 18);
#pragma unroll
    for (int l = 0; l < 4; l++) h = (h ^ xround(0, a[l])) * kX1 + kX4;
    i = stripes * 32;
  } else {
    h = kX5;
  }
  h += len;
  for (; i + 8 <= len; i += 8) h = xrotl(h ^ xround(0, rd(i, 8)), 27) * kX1 + kX4;
  if (i + 4 <= len) {
    h = xrotl(h ^ (rd(i, 4) * kX1), 23) * kX2 + kX3;
    i += 4;
  }
  for (; i < len; i++) h = xrotl(h ^ (rd(i, 1) * kX5), 11) * kX1;
  h ^= h >> 33;
  h *= kX2;
  h ^= h >> 29;
  h *= kX3;
  h ^= h >> 32;
  return (uint32_t)h;
}

// Decode the Zstd frames of in[0, csize) into out[0, olen): frames one
// after another (ZSTD_decompress's loop), skippable frames skipped, each
// frame's content size checked against its output, a content checksum
// (XXH64) verified.  Each frame's literals decode into the tail of the
// whole output, which no frame before the last writes.
// All 64 lanes of the wave call it; `tb` is a 16-aligned LDS area of tcap >=
// kZTablesBytes bytes.  Returns a wave-uniform status.
template <class Src, class O>
__device__ __attribute__((noinline)) uint32_t zstd_decode(const Src& in, uint32_t csize, O out, uint32_t olen, lds_u8* tb,
                                uint32_t tcap) {
  const uint32_t lane = threadIdx.x & 63;
  const Tabs t(tb);
  uint32_t p = 0, op = 0;
  bool first = true;
  while (first || p < csize) {
  // skippable frames (RFC 8878 3.1.2): magic 0x184D2A5?, u32 size, payload
  if (csize - p >= 8 && (in.u32(p) & 0xFFFFFFF0u) == 0x184D2A50u) {
    const uint32_t sz = in.u32(p + 4);
    if (sz > csize - p - 8) return ST_CODEC;
    p += 8 + sz;
    first = false;
    continue;
  }
  first = false;
  const uint32_t op0 = op;
  // ---- frame header (RFC 8878 3.1.1.1)
  if (csize - p < 8 || in.u32(p) != 0xFD2FB528u) return ST_CODEC;
  const uint32_t fhd = in.u8(p + 4);
  if (fhd & 8) return ST_CODEC;  // reserved bit
  const uint32_t single = (fhd >> 5) & 1, fcs_flag = fhd >> 6, did_flag = fhd & 3;
  p += 5;
  if (!single) {
    const uint32_t wd = in.u8(p++);
    const uint32_t wlog = 10 + (wd >> 3);
    if (wlog > 27) return ST_CODEC;  // ZSTD_decompress's default window limit
    const uint64_t wsize = (1ull << wlog) + ((1ull << wlog) >> 3) * (wd & 7);
    if (wsize > (1ull << 27) + 1) return ST_CODEC;
  }
  const uint32_t did_len = did_flag == 3 ? 4 : did_flag;
  const uint32_t fcs_len = fcs_flag == 0 ? single : (1u << fcs_flag);
  if (p + did_len + fcs_len > csize) return ST_CODEC;
  uint32_t did = 0;
  for (uint32_t k = 0; k < did_len; k++) did |= in.u8(p + k) << (8 * k);
  p += did_len;
  if (did) return ST_CODEC;  // a dictionary the caller does not have
  uint64_t fcs = ~0ull;
  if (fcs_len) {
    fcs = 0;
    for (uint32_t k = 0; k < fcs_len; k++) fcs |= (uint64_t)in.u8(p + k) << (8 * k);
    if (fcs_len == 2) fcs += 256;
    if (fcs > olen - op0) return ST_CODEC;
    p += fcs_len;
  }
  // ---- blocks
  uint32_t r0 = 1, r1 = 4, r2 = 8;  // repeat offsets (lane 0)
  uint32_t al_ll = 0, al_ml = 0, al_of = 0;
  bool h_ll = false, h_ml = false, h_of = false, p_ll = false, p_ml = false, p_of = false;
  uint32_t htl = 0;  // Huffman table log, 0 = none yet
  for (;;) {
    if (p + 3 > csize) return ST_CODEC;
    const uint32_t bh = in.u8(p) | (in.u8(p + 1) << 8) | (in.u8(p + 2) << 16);
    p += 3;
    const uint32_t last = bh & 1, bt = (bh >> 1) & 3, bs = bh >> 3;
    if (bt == 0) {  // raw
      if (bs > csize - p || bs > olen - op) return ST_CODEC;
      copy_in(out, op, in, p, bs);
      p += bs;
      op += bs;
    } else if (bt == 1) {  // RLE
      if (p >= csize || bs > olen - op) return ST_CODEC;
      fill(out, op, (uint8_t)in.u8(p), bs);
      p += 1;
      op += bs;
    } else if (bt == 2) {  // compressed
      if (bs > csize - p || bs >= kBlockMax || bs == 0) return ST_CODEC;
      const uint32_t bend = p + bs;
      // -- literals section (3.1.1.3.1)
      const uint32_t b0 = in.u8(p), ltype = b0 & 3, sf = (b0 >> 2) & 3;
      uint32_t hl, regen, lcs = 0, ns = 1;
      if (ltype < 2) {
        if (!(sf & 1)) {
          hl = 1;
          regen = b0 >> 3;
        } else if (sf == 1) {
          hl = 2;
          regen = (b0 >> 4) | (in.u8(p + 1) << 4);
        } else {
          hl = 3;
          regen = (b0 >> 4) | (in.u8(p + 1) << 4) | (in.u8(p + 2) << 12);
        }
      } else {
        ns = sf == 0 ? 1 : 4;
        if (sf < 2) {
          hl = 3;
          const uint32_t h = b0 | (in.u8(p + 1) << 8) | (in.u8(p + 2) << 16);
          regen = (h >> 4) & 0x3FF;
          lcs = (h >> 14) & 0x3FF;
        } else if (sf == 2) {
          hl = 4;
          const uint32_t h = in.u32(p);
          regen = (h >> 4) & 0x3FFF;
          lcs = h >> 18;
        } else {
          hl = 5;
          const uint64_t h = (uint64_t)in.u32(p) | ((uint64_t)in.u8(p + 4) << 32);
          regen = (uint32_t)(h >> 4) & 0x3FFFF;
          lcs = (uint32_t)(h >> 22) & 0x3FFFF;
        }
      }
      if (hl > bs || regen > kBlockMax || regen > olen - op) return ST_CODEC;
      const uint32_t lt0 = olen - regen;  // literals live at the tail of the window
      uint32_t q = p + hl;
      if (ltype == 0) {
        if (regen > bend - q) return ST_CODEC;
        copy_in(out, lt0, in, q, regen);
        q += regen;
      } else if (ltype == 1) {
        if (q >= bend) return ST_CODEC;
        fill(out, lt0, (uint8_t)in.u8(q), regen);
        q += 1;
      } else {
        if (lcs > bend - q) return ST_CODEC;
        const uint32_t lend = q + lcs;
        if (ltype == 2) {
          if (lane == 0) {
            uint32_t tl = 0, used = 0;
            t.misc[0] = read_huf(in, q, lcs, t, tcap >= kBytes12, &tl, &used);
            t.misc[1] = tl;
            t.misc[2] = used;
          }
          zsync();
          const uint32_t st = t.misc[0];
          if (st) return st;
          htl = t.misc[1];
          q += t.misc[2];
          zsync();
        } else if (!htl) {
          return ST_CODEC;  // treeless literals without an earlier table
        }
        uint32_t sst = q, sln = lend - q, scnt = regen, sdst = lt0;
        if (ns == 4) {
          if (lend - q < 10) return ST_CODEC;
          const uint32_t j1 = in.u8(q) | (in.u8(q + 1) << 8), j2 = in.u8(q + 2) | (in.u8(q + 3) << 8),
                         j3 = in.u8(q + 4) | (in.u8(q + 5) << 8);
          const uint32_t body = q + 6, tot = lend - body;
          if (j1 + j2 + j3 > tot) return ST_CODEC;
          const uint32_t seg = (regen + 3) >> 2;
          if (3 * seg > regen) return ST_CODEC;
          sst = body;
          sln = j1;
          if (lane >= 1) sst += j1, sln = j2;
          if (lane >= 2) sst += j2, sln = j3;
          if (lane >= 3) sst += j3, sln = tot - j1 - j2 - j3;
          scnt = lane < 3 ? seg : regen - 3 * seg;
          sdst = lt0 + (lane < 4 ? lane : 0) * seg;
        }
        bool bad = false;
        if (lane < ns) {
          RevBits<Src> br;
          if (!br.init(in, sst, sln)) {
            bad = true;
          } else {
            for (uint32_t k = 0; k < scnt; k++) {
              if (br.pos - br.wlo < (int32_t)htl) br.refill();
              const uint32_t e = t.huf[br.peek(htl)];
              out[sdst + k] = (uint8_t)e;
              br.pos -= (int32_t)(e >> 8);
            }
            bad = br.pos != 0;
          }
        }
        if (__ballot(bad)) return ST_CODEC;
        q = lend;
      }
      zsync();
      // -- sequences section (3.1.1.3.2)
      if (q >= bend) return ST_CODEC;
      uint32_t nseq = in.u8(q++);
      if (nseq == 255) {
        if (q + 2 > bend) return ST_CODEC;
        nseq = in.u8(q) + (in.u8(q + 1) << 8) + 0x7F00;
        q += 2;
      } else if (nseq >= 128) {
        if (q >= bend) return ST_CODEC;
        nseq = ((nseq - 128) << 8) + in.u8(q++);
      }
      if (nseq == 0) {
        if (q != bend) return ST_CODEC;
        copy_fwd(out, op, lt0, regen);
        op += regen;
      } else {
        if (q >= bend) return ST_CODEC;
        const uint32_t modes = in.u8(q++);
        if (modes & 3) return ST_CODEC;
        RevBits<Src> br;
        uint32_t sLL = 0, sML = 0, sOF = 0;
        if (lane == 0) {
          uint32_t qq = q;
          uint32_t st = seq_table(in, &qq, bend, modes >> 6, K_LL, t, t.ll, &al_ll, &h_ll, &p_ll);
          if (!st) st = seq_table(in, &qq, bend, (modes >> 4) & 3, K_OF, t, t.of, &al_of, &h_of, &p_of);
          if (!st) st = seq_table(in, &qq, bend, (modes >> 2) & 3, K_ML, t, t.ml, &al_ml, &h_ml, &p_ml);
          if (!st && (qq >= bend || !br.init(in, qq, bend - qq))) st = ST_CODEC;
          if (!st) {
            sLL = br.read(al_ll);
            sOF = br.read(al_of);
            sML = br.read(al_ml);
          }
          t.misc[0] = st;
        }
        zsync();
        if (t.misc[0]) return t.misc[0];
        zsync();
        uint32_t lp = lt0;
        for (uint32_t k0 = 0; k0 < nseq; k0 += 64) {
          const uint32_t cnt = min(64u, nseq - k0);
          if (lane == 0) {
            uint32_t o = op, l = lp, st = ST_OK;
            for (uint32_t j = 0; j < cnt; j++) {
              const uint64_t cl = t.ll[sLL], cm = t.ml[sML], co = t.of[sOF];
              const uint32_t ofv = (uint32_t)(co >> 32) + br.read((uint32_t)(co >> 24) & 0xFF);
              const uint32_t ml = (uint32_t)(cm >> 32) + br.read((uint32_t)(cm >> 24) & 0xFF);
              const uint32_t ll = (uint32_t)(cl >> 32) + br.read((uint32_t)(cl >> 24) & 0xFF);
              uint32_t off;
              if (ofv > 3) {
                off = ofv - 3;
                r2 = r1;
                r1 = r0;
                r0 = off;
              } else {  // repeat offsets (3.1.2.5), libzstd's "offset 0 -> 1" fix-up
                const uint32_t idx = ofv - 1 + (ll == 0);
                if (idx == 0) {
                  off = r0;
                } else {
                  off = idx == 3 ? r0 - 1 : (idx == 1 ? r1 : r2);
                  off += off == 0;
                  if (idx != 1) r2 = r1;
                  r1 = r0;
                  r0 = off;
                }
              }
              // libzstd 1.4.8 updates the states after every sequence (the
              // last update reads past the stream start, which it accepts)
              sLL = (uint32_t)(cl & 0xFFFF) + br.read((uint32_t)(cl >> 16) & 0xFF);
              sML = (uint32_t)(cm & 0xFFFF) + br.read((uint32_t)(cm >> 16) & 0xFF);
              sOF = (uint32_t)(co & 0xFFFF) + br.read((uint32_t)(co >> 16) & 0xFF);
              // a frame's history starts at its own first byte: libzstd 1.4.8
              // resets the prefix per frame (ZSTD_checkContinuity), so an
              // offset reaching into an earlier frame's output is corrupt
              if (ll > olen - l || off > o + ll - op0 || o + ml > l) {
                st = ST_CODEC;
                break;
              }
              t.seq[j] = ll;
              t.seq[64 + j] = ml;
              t.seq[128 + j] = off;
              t.seq[192 + j] = o;
              t.seq[256 + j] = l;
              o += ll + ml;
              l += ll;
            }
            if (!st && k0 + cnt == nseq && br.pos > 0) st = ST_CODEC;  // stream not fully consumed
            t.misc[0] = st;
            t.misc[1] = o;
            t.misc[2] = l;
          }
          zsync();
          if (t.misc[0]) return t.misc[0];
          const uint32_t wend = t.misc[1], lpn = t.misc[2];
          exec_batch(out, t, cnt, op, lp, wend);
          op = wend;
          lp = lpn;
          zsync();
        }
        copy_fwd(out, op, lp, olen - lp);  // the literals after the last match
        op += olen - lp;
      }
      p = bend;
    } else {
      return ST_CODEC;  // reserved block type
    }
    if (last) break;
  }
  if (fcs != ~0ull && op - op0 != fcs) return ST_CODEC;  // the frame's content size
  if (fhd & 4) {  // content checksum: XXH64 of the frame's output, low 32 bits
    if (csize - p < 4) return ST_CODEC;
    zsync();
    if (xxh64_low32(out, op0, op - op0) != in.u32(p)) return ST_CODEC;
    p += 4;
  }
  }  // frames
  if (op != olen) return ST_CODEC;
  zsync();
  return ST_OK;
}

// The LDS-to-LDS form every staged caller uses (one out-of-line copy of the
// decoder: inlined into every kernel that can meet a Zstd stream, it grew
// their code enough to slow the C5 decode by a quarter).
__device__ __attribute__((noinline)) uint32_t zstd_to_lds(const LdsSrc& in, uint32_t csize, lds_u8* out, uint32_t olen, lds_u8* tb,
                                                uint32_t tcap) {
  return zstd_decode(in, csize, out, olen, tb, tcap);
}

}  // namespace zs
