/*
 * sb_oracle.c -- CPU restatement of the strawboat page codec path.
 *
 * TEST INFRASTRUCTURE ONLY (see sb_oracle.h): the parity checker and the
 * "port" CPU baseline.  Every function cites the reference (b41sh/pa @
 * 2025-01-17, /root/reference) file:line it restates.  Third-party pieces
 * (bitpacking 0.8.0 BitPacker4x, roaring 0.10.1, parquet2 0.17 hybrid RLE,
 * liblz4 / libzstd / snap) are restated from their published formats; LZ4 and
 * Zstd call the system liblz4.so.1 / libzstd.so.1 directly.
 */
#include "sb_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---- system codec libraries (runtime .so only; prototypes restated) ---- */
int LZ4_decompress_safe(const char* src, char* dst, int compressedSize, int dstCapacity);
int LZ4_compress_default(const char* src, char* dst, int srcSize, int dstCapacity);
int LZ4_compressBound(int inputSize);
size_t ZSTD_decompress(void* dst, size_t dstCapacity, const void* src, size_t compressedSize);
size_t ZSTD_compress(void* dst, size_t dstCapacity, const void* src, size_t srcSize, int level);
size_t ZSTD_compressBound(size_t srcSize);
unsigned ZSTD_isError(size_t code);

/* ======================================================================= */
/* byte buffer                                                              */
/* ======================================================================= */
void orc_buf_free(orc_buf* b) {
  free(b->data);
  b->data = NULL;
  b->len = b->cap = 0;
}

static int buf_reserve(orc_buf* b, size_t extra) {
  if (b->len + extra <= b->cap) return 0;
  size_t nc = b->cap ? b->cap : 256;
  while (nc < b->len + extra) nc *= 2;
  uint8_t* p = (uint8_t*)realloc(b->data, nc);
  if (!p) return -1;
  b->data = p;
  b->cap = nc;
  return 0;
}

static void buf_put(orc_buf* b, const void* p, size_t n) {
  buf_reserve(b, n);
  if (n) memcpy(b->data + b->len, p, n);
  b->len += n;
}
static void buf_u8(orc_buf* b, uint8_t v) { buf_put(b, &v, 1); }
static void buf_u16(orc_buf* b, uint16_t v) { buf_put(b, &v, 2); }
static void buf_u32(orc_buf* b, uint32_t v) { buf_put(b, &v, 4); }
static void buf_u64(orc_buf* b, uint64_t v) { buf_put(b, &v, 8); }

static uint32_t rd_u32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint16_t rd_u16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
static uint64_t rd_u64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

static int get_bit(const uint8_t* bits, size_t i) { return (bits[i >> 3] >> (i & 7)) & 1; }
static int is_valid(const uint8_t* validity, size_t i) { return validity ? get_bit(validity, i) : 1; }

/* little-endian value of `width` bytes as u64 (widths 1..8) */
static uint64_t ld_w(const uint8_t* p, int width) {
  uint64_t v = 0;
  memcpy(&v, p, (size_t)width);
  return v;
}
/* IntegerType::as_i64 (integer/traits.rs): sign- or zero-extension by type */
static int64_t as_i64(uint64_t raw, int width, int is_signed) {
  if (width == 8) return (int64_t)raw;
  if (!is_signed) return (int64_t)raw;
  int sh = 64 - 8 * width;
  return ((int64_t)(raw << sh)) >> sh;
}
/* ======================================================================= */
/* deterministic sampler standing in for thread_rng (integer/mod.rs:316)    */
/* ======================================================================= */
typedef struct {
  uint64_t s;
} orc_rng;
static uint64_t rng_next(orc_rng* r) { /* splitmix64 */
  uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* ======================================================================= */
/* BitPacker4x (bitpacking 0.8.0): 128 u32 per block, 4 interleaved lanes.  */
/* Value v = 4*i + l lives at bits [i*b, i*b+b) of lane l's bitstream; lane  */
/* bitstream word k is the u32 at byte 16*k + 4*l.  Called from             */
/* integer/bp.rs:45-84 and integer/delta_bp.rs:45-89.                      */
/* ======================================================================= */
uint32_t orc_bp4x_num_bits(const uint32_t* in) {
  uint32_t acc = 0;
  for (int i = 0; i < 128; i++) acc |= in[i];
  uint32_t b = 0;
  while (acc) { b++; acc >>= 1; }
  return b;
}

size_t orc_bp4x_pack(const uint32_t* in, uint32_t b, uint8_t* out) {
  if (b == 0) return 0;
  uint32_t words[4 * 32];
  memset(words, 0, sizeof(words));
  uint64_t mask = (b == 32) ? 0xFFFFFFFFull : ((1ull << b) - 1);
  for (int l = 0; l < 4; l++) {
    for (uint32_t i = 0; i < 32; i++) {
      uint64_t v = in[4 * i + l] & mask;
      uint32_t bit = i * b, k = bit >> 5, s = bit & 31;
      words[4 * k + l] |= (uint32_t)(v << s);
      if (s + b > 32) words[4 * (k + 1) + l] |= (uint32_t)(v >> (32 - s));
    }
  }
  memcpy(out, words, 16 * (size_t)b);
  return 16 * (size_t)b;
}

size_t orc_bp4x_unpack(const uint8_t* in, uint32_t b, uint32_t* out) {
  if (b == 0) { memset(out, 0, 128 * 4); return 0; }
  uint64_t mask = (b == 32) ? 0xFFFFFFFFull : ((1ull << b) - 1);
  for (int l = 0; l < 4; l++) {
    for (uint32_t i = 0; i < 32; i++) {
      uint32_t bit = i * b, k = bit >> 5, s = bit & 31;
      uint64_t lo = rd_u32(in + 16 * k + 4 * l);
      uint64_t hi = (s + b > 32) ? rd_u32(in + 16 * (k + 1) + 4 * l) : 0;
      out[4 * i + l] = (uint32_t)(((hi << 32 | lo) >> s) & mask);
    }
  }
  return 16 * (size_t)b;
}

/* compress_sorted: sequential wrapping deltas from `initial` */
size_t orc_bp4x_pack_sorted(uint32_t initial, const uint32_t* in, uint32_t b, uint8_t* out) {
  uint32_t d[128];
  uint32_t prev = initial;
  for (int i = 0; i < 128; i++) { d[i] = in[i] - prev; prev = in[i]; }
  return orc_bp4x_pack(d, b, out);
}

size_t orc_bp4x_unpack_sorted(uint32_t initial, const uint8_t* in, uint32_t b, uint32_t* out) {
  size_t n = orc_bp4x_unpack(in, b, out);
  uint32_t acc = initial;
  for (int i = 0; i < 128; i++) { acc += out[i]; out[i] = acc; }
  return n;
}

/* ======================================================================= */
/* Patas pack/unpack (double/patas.rs:145-162)                              */
/* ======================================================================= */
uint16_t orc_patas_pack(uint32_t ref_diff, uint32_t sig_bytes, uint32_t tz) {
  return (uint16_t)(((ref_diff & 0xFF) << 9) | ((sig_bytes & 7) << 6) | (tz & 0xFF));
}
void orc_patas_unpack(uint16_t packed, uint32_t* ref_diff, uint32_t* sig_bytes, uint32_t* tz) {
  uint32_t r = (packed >> 9) & 0x7F, sb = (packed >> 6) & 7, t = packed & 0x3F;
  if (t < 63 && sb == 0) sb = 8;
  *ref_diff = r; *sig_bytes = sb; *tz = t;
}

/* ======================================================================= */
/* general codecs: CommonCompression (compression/basic.rs:62-152)          */
/* ======================================================================= */
static int snappy_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_len);
static int snappy_compress(const uint8_t* in, size_t n, orc_buf* out);

int orc_common_decompress(int codec, const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len) {
  switch (codec) {
    case ORC_NONE: /* basic.rs:68-71 copy_from_slice: lengths must match */
      if (in_len != out_len) return ORC_E_OUT_OF_SPEC;
      if (out_len) memcpy(out, in, out_len);
      return ORC_OK;
    case ORC_LZ4: { /* basic.rs:87-91 raw block, no size prefix */
      if (in_len > 0x7FFFFFFF || out_len > 0x7FFFFFFF) return ORC_E_CODEC;
      int r = LZ4_decompress_safe((const char*)in, (char*)out, (int)in_len, (int)out_len);
      if (r < 0 || (size_t)r != out_len) return ORC_E_CODEC;
      return ORC_OK;
    }
    case ORC_ZSTD: { /* basic.rs:93-97 one frame */
      size_t r = ZSTD_decompress(out, out_len, in, in_len);
      if (ZSTD_isError(r) || r != out_len) return ORC_E_CODEC;
      return ORC_OK;
    }
    case ORC_SNAPPY: /* basic.rs:99-106 raw snappy */
      return snappy_decompress(in, in_len, out, out_len);
    default:
      return ORC_E_OUT_OF_SPEC;
  }
}

int orc_common_compress(int codec, const uint8_t* in, size_t in_len, orc_buf* out) {
  switch (codec) {
    case ORC_NONE:
      buf_put(out, in, in_len);
      return ORC_OK;
    case ORC_LZ4: { /* basic.rs:108-120: compress_to_buffer(.., None, false, ..) */
      int bound = LZ4_compressBound((int)in_len);
      buf_reserve(out, (size_t)bound);
      int r = LZ4_compress_default((const char*)in, (char*)out->data + out->len, (int)in_len, bound);
      if (r <= 0 && in_len > 0) return ORC_E_CODEC;
      out->len += (size_t)r;
      return ORC_OK;
    }
    case ORC_ZSTD: { /* basic.rs:122-135: level 0 (= default 3) */
      size_t bound = ZSTD_compressBound(in_len);
      buf_reserve(out, bound);
      size_t r = ZSTD_compress(out->data + out->len, bound, in, in_len, 0);
      if (ZSTD_isError(r)) return ORC_E_CODEC;
      out->len += r;
      return ORC_OK;
    }
    case ORC_SNAPPY:
      return snappy_compress(in, in_len, out);
    default:
      return ORC_E_ARG;
  }
}

/* Snappy raw format (snap 1.1 raw::Decoder / Encoder): varint length, then
 * literal / copy-1 / copy-2 / copy-4 elements. */
static int snappy_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_len) {
  size_t ip = 0, op = 0;
  uint64_t ulen = 0;
  int shift = 0;
  for (;;) {
    if (ip >= n || shift > 35) return ORC_E_CODEC;
    uint8_t c = in[ip++];
    ulen |= (uint64_t)(c & 0x7F) << shift;
    if (!(c & 0x80)) break;
    shift += 7;
  }
  if (ulen != out_len) return ORC_E_CODEC;
  while (ip < n) {
    uint8_t tag = in[ip++];
    uint32_t type = tag & 3;
    if (type == 0) {
      size_t len = (tag >> 2) + 1;
      if (len > 60) {
        size_t nb = len - 60;
        if (ip + nb > n) return ORC_E_CODEC;
        len = 0;
        for (size_t i = 0; i < nb; i++) len |= (size_t)in[ip + i] << (8 * i);
        len += 1;
        ip += nb;
      }
      if (ip + len > n || op + len > out_len) return ORC_E_CODEC;
      memcpy(out + op, in + ip, len);
      ip += len;
      op += len;
    } else {
      size_t len, off;
      if (type == 1) {
        if (ip + 1 > n) return ORC_E_CODEC;
        len = ((tag >> 2) & 7) + 4;
        off = ((size_t)(tag >> 5) << 8) | in[ip];
        ip += 1;
      } else if (type == 2) {
        if (ip + 2 > n) return ORC_E_CODEC;
        len = (tag >> 2) + 1;
        off = rd_u16(in + ip);
        ip += 2;
      } else {
        if (ip + 4 > n) return ORC_E_CODEC;
        len = (tag >> 2) + 1;
        off = rd_u32(in + ip);
        ip += 4;
      }
      if (off == 0 || off > op || op + len > out_len) return ORC_E_CODEC;
      for (size_t i = 0; i < len; i++) out[op + i] = out[op - off + i];
      op += len;
    }
  }
  return op == out_len ? ORC_OK : ORC_E_CODEC;
}

static void snappy_emit_literal(orc_buf* out, const uint8_t* p, size_t len) {
  while (len) {
    size_t chunk = len > 65536 ? 65536 : len;
    size_t l1 = chunk - 1;
    if (l1 < 60) {
      buf_u8(out, (uint8_t)(l1 << 2));
    } else if (l1 < 256) {
      buf_u8(out, 60 << 2);
      buf_u8(out, (uint8_t)l1);
    } else {
      buf_u8(out, 61 << 2);
      buf_u16(out, (uint16_t)l1);
    }
    buf_put(out, p, chunk);
    p += chunk;
    len -= chunk;
  }
}

static void snappy_emit_copy(orc_buf* out, size_t off, size_t len) {
  while (len > 0) {
    size_t l = len > 64 ? 64 : len;
    if (len > 64 && len - 64 < 4) l = 60; /* keep the tail >= 4 */
    buf_u8(out, (uint8_t)(((l - 1) << 2) | 2));
    buf_u16(out, (uint16_t)off);
    len -= l;
  }
}

/* Greedy hash-match compressor producing a valid raw snappy stream (bytes are
 * not identical to snap's encoder; decode-equivalent, which is all the
 * reference's readers rely on). */
static int snappy_compress(const uint8_t* in, size_t n, orc_buf* out) {
  uint64_t v = n;
  do {
    uint8_t c = v & 0x7F;
    v >>= 7;
    if (v) c |= 0x80;
    buf_u8(out, c);
  } while (v);
  enum { HB = 14 };
  int64_t* table = (int64_t*)malloc(sizeof(int64_t) << HB);
  for (size_t i = 0; i < ((size_t)1 << HB); i++) table[i] = -1;
  size_t lit = 0, i = 0;
  while (i + 4 <= n) {
    uint32_t w = rd_u32(in + i);
    uint32_t h = (w * 0x1E35A7BDu) >> (32 - HB);
    int64_t cand = table[h];
    table[h] = (int64_t)i;
    if (cand >= 0 && i - (size_t)cand <= 65535 && rd_u32(in + cand) == w) {
      size_t len = 4;
      while (i + len < n && in[cand + len] == in[i + len]) len++;
      if (i > lit) snappy_emit_literal(out, in + lit, i - lit);
      snappy_emit_copy(out, i - (size_t)cand, len);
      i += len;
      lit = i;
    } else {
      i++;
    }
  }
  if (n > lit) snappy_emit_literal(out, in + lit, n - lit);
  free(table);
  return ORC_OK;
}

/* ======================================================================= */
/* roaring 0.10.1 portable serialization                                     */
/* (integer/freq.rs:74-76, 103-106; binary/freq.rs:86-88, 117-120)          */
/* ======================================================================= */
int orc_roaring_decode(const uint8_t* buf, size_t len, uint32_t* pos_out, size_t cap, size_t* count) {
  size_t p = 0, total = 0;
  if (len < 4) return ORC_E_OUT_OF_SPEC;
  uint32_t cookie = rd_u32(buf);
  uint32_t size;
  const uint8_t* run_flags = NULL;
  int has_offsets;
  if (cookie == 12346) {
    if (len < 8) return ORC_E_OUT_OF_SPEC;
    size = rd_u32(buf + 4);
    p = 8;
    has_offsets = 1;
  } else if ((cookie & 0xFFFF) == 12347) {
    size = (cookie >> 16) + 1;
    p = 4;
    run_flags = buf + p;
    p += (size + 7) / 8;
    has_offsets = size >= 4;
  } else {
    return ORC_E_OUT_OF_SPEC;
  }
  if (size > 65536) return ORC_E_OUT_OF_SPEC;
  size_t desc = p;
  p += 4 * (size_t)size;
  if (has_offsets) p += 4 * (size_t)size;
  if (p > len) return ORC_E_OUT_OF_SPEC;
  for (uint32_t c = 0; c < size; c++) {
    uint32_t key = rd_u16(buf + desc + 4 * c);
    uint32_t card = (uint32_t)rd_u16(buf + desc + 4 * c + 2) + 1;
    int is_run = run_flags ? ((run_flags[c >> 3] >> (c & 7)) & 1) : 0;
    if (is_run) {
      if (p + 2 > len) return ORC_E_OUT_OF_SPEC;
      uint32_t nr = rd_u16(buf + p);
      p += 2;
      if (p + 4 * (size_t)nr > len) return ORC_E_OUT_OF_SPEC;
      for (uint32_t r = 0; r < nr; r++) {
        uint32_t st = rd_u16(buf + p + 4 * r), ln = (uint32_t)rd_u16(buf + p + 4 * r + 2) + 1;
        for (uint32_t x = 0; x < ln; x++) {
          if (pos_out && total < cap) pos_out[total] = (key << 16) | (st + x);
          total++;
        }
      }
      p += 4 * (size_t)nr;
    } else if (card <= 4096) {
      if (p + 2 * (size_t)card > len) return ORC_E_OUT_OF_SPEC;
      for (uint32_t x = 0; x < card; x++) {
        if (pos_out && total < cap) pos_out[total] = (key << 16) | rd_u16(buf + p + 2 * x);
        total++;
      }
      p += 2 * (size_t)card;
    } else {
      if (p + 8192 > len) return ORC_E_OUT_OF_SPEC;
      for (uint32_t w = 0; w < 1024; w++) {
        uint64_t word = rd_u64(buf + p + 8 * w);
        while (word) {
          uint32_t b = (uint32_t)__builtin_ctzll(word);
          if (pos_out && total < cap) pos_out[total] = (key << 16) | (w * 64 + b);
          total++;
          word &= word - 1;
        }
      }
      p += 8192;
    }
  }
  *count = total;
  return ORC_OK;
}

/* serialize_into (roaring 0.10.1): cookie 12346, no run containers. */
int orc_roaring_encode(const uint32_t* pos, size_t count, orc_buf* out) {
  /* containers by high 16 bits; pos ascending */
  size_t nc = 0;
  for (size_t i = 0; i < count; i++)
    if (i == 0 || (pos[i] >> 16) != (pos[i - 1] >> 16)) nc++;
  buf_u32(out, 12346);
  buf_u32(out, (uint32_t)nc);
  size_t* start = (size_t*)malloc((nc + 1) * sizeof(size_t));
  size_t c = 0;
  for (size_t i = 0; i < count; i++)
    if (i == 0 || (pos[i] >> 16) != (pos[i - 1] >> 16)) start[c++] = i;
  start[nc] = count;
  for (size_t k = 0; k < nc; k++) {
    buf_u16(out, (uint16_t)(pos[start[k]] >> 16));
    buf_u16(out, (uint16_t)(start[k + 1] - start[k] - 1));
  }
  uint32_t off = 8 + 8 * (uint32_t)nc;
  for (size_t k = 0; k < nc; k++) {
    buf_u32(out, off);
    size_t card = start[k + 1] - start[k];
    off += card <= 4096 ? (uint32_t)(2 * card) : 8192u;
  }
  for (size_t k = 0; k < nc; k++) {
    size_t card = start[k + 1] - start[k];
    if (card <= 4096) {
      for (size_t i = start[k]; i < start[k + 1]; i++) buf_u16(out, (uint16_t)(pos[i] & 0xFFFF));
    } else {
      uint64_t words[1024];
      memset(words, 0, sizeof(words));
      for (size_t i = start[k]; i < start[k + 1]; i++) {
        uint32_t lo = pos[i] & 0xFFFF;
        words[lo >> 6] |= 1ull << (lo & 63);
      }
      buf_put(out, words, sizeof(words));
    }
  }
  free(start);
  return ORC_OK;
}

/* ======================================================================= */
/* value-stream decoders                                                    */
/* ======================================================================= */

/* read_compress_header (read/read_basic.rs:181-189) */
static int read_header(const uint8_t* buf, size_t len, size_t* pos, int* codec, size_t* csize,
                       size_t* usize) {
  if (*pos + 9 > len) return ORC_E_IO;
  *codec = buf[*pos];
  *csize = rd_u32(buf + *pos + 1);
  *usize = rd_u32(buf + *pos + 5);
  *pos += 9;
  if (*pos + *csize > len) return ORC_E_IO;
  return ORC_OK;
}

/* RLE::decompress_integer (integer/rle.rs:106-134); double/rle.rs:89-119 is
 * the same loop.  Runs of (u32 count, T value); stops once >= length values
 * were produced; a run that overshoots `length` fails the reference's
 * assert_eq!(values.len(), length) (array/integer.rs:81). */
static int rle_decode(const uint8_t* in, size_t n, int width, size_t length, uint8_t* out) {
  size_t p = 0, produced = 0;
  if (length == 0) return ORC_OK;
  while (produced < length) {
    if (p + 4 + (size_t)width > n) return ORC_E_IO;
    uint32_t cnt = rd_u32(in + p);
    const uint8_t* v = in + p + 4;
    p += 4 + (size_t)width;
    if (produced + cnt > length) return ORC_E_OUT_OF_SPEC;
    for (uint32_t i = 0; i < cnt; i++) memcpy(out + (produced + i) * width, v, (size_t)width);
    produced += cnt;
  }
  return ORC_OK;
}

/* OneValue::decode_native (integer/one_value.rs:77-94) */
static int one_value_decode(const uint8_t* in, size_t n, int width, size_t length, uint8_t* out) {
  if (n < (size_t)width) return ORC_E_IO;
  for (size_t i = 0; i < length; i++) memcpy(out + i * width, in, (size_t)width);
  return ORC_OK;
}

/* Bitpacking::decompress (integer/bp.rs:67-86) and DeltaBitpacking
 * (integer/delta_bp.rs:69-92).  T must be 4 bytes; whole 128-blocks. */
static int bp_decode(const uint8_t* in, size_t n, int width, size_t length, uint8_t* out, int delta) {
  if (width != 4) return ORC_E_OUT_OF_SPEC;
  size_t p = 0;
  uint32_t initial = 0, tmp[128];
  size_t nblocks = (length + 127) / 128;
  for (size_t blk = 0; blk < nblocks; blk++) {
    if (p + 1 > n) return ORC_E_IO;
    uint32_t b = in[p++];
    if (b > 32) return ORC_E_OUT_OF_SPEC;
    if (p + 16 * (size_t)b > n) return ORC_E_IO;
    if (delta) {
      p += orc_bp4x_unpack_sorted(initial, in + p, b, tmp);
      initial = tmp[127];
    } else {
      p += orc_bp4x_unpack(in + p, b, tmp);
    }
    size_t take = length - blk * 128 < 128 ? length - blk * 128 : 128;
    memcpy(out + blk * 128 * 4, tmp, take * 4);
  }
  /* bp.rs pushes whole blocks: a length that is not a multiple of 128 leaves
   * values.len() != length and fails array/integer.rs:81 */
  if (length % 128) return ORC_E_OUT_OF_SPEC;
  return ORC_OK;
}

/* Patas::decompress (double/patas.rs:107-132) */
static int patas_decode(const uint8_t* in, size_t n, int width, size_t length, uint8_t* out) {
  if (length == 0) return ORC_E_OUT_OF_SPEC; /* `length - 1` underflows in patas.rs:117 */
  size_t p = 0;
  if (n < (size_t)width) return ORC_E_IO;
  memcpy(out, in, (size_t)width);
  p = (size_t)width;
  for (size_t i = 1; i < length; i++) {
    if (p + 2 > n) return ORC_E_IO;
    uint32_t rd, sb, tz;
    orc_patas_unpack(rd_u16(in + p), &rd, &sb, &tz);
    p += 2;
    /* read_value_custom copies sb bytes into a sizeof(T) buffer (patas.rs:165-189);
     * for f32 a run of repeats makes sb = 8 > 4 (the documented f32 desync) */
    if (sb > (uint32_t)width) return ORC_E_OUT_OF_SPEC;
    if (p + sb > n) return ORC_E_IO;
    uint64_t val = 0;
    memcpy(&val, in + p, sb);
    p += sb;
    if (rd == 0 || rd > i) return ORC_E_OUT_OF_SPEC;
    uint64_t prev = ld_w(out + (i - rd) * width, width);
    uint64_t x;
    if (width == 8) {
      x = (tz >= 64 ? 0 : (val << tz)) ^ prev;
    } else {
      uint32_t v32 = (uint32_t)val;
      x = (uint32_t)((tz >= 32 ? 0u : (v32 << tz)) ^ (uint32_t)prev);
    }
    memcpy(out + i * width, &x, (size_t)width);
  }
  return ORC_OK;
}

static int decompress_stream(const uint8_t* buf, size_t len, size_t* pos, int width, size_t length,
                             uint8_t* out, int is_float);

/* Dict::decompress (integer/dict.rs:75-103; double/dict.rs:80-107) */
static int dict_decode(const uint8_t* in, size_t n, int width, size_t length, uint8_t* out) {
  size_t p = 0;
  uint32_t* idx = (uint32_t*)malloc((length ? length : 1) * 4);
  int rc = decompress_stream(in, n, &p, 4, length, (uint8_t*)idx, 0);
  if (rc) { free(idx); return rc; }
  if (p + 4 > n) { free(idx); return ORC_E_IO; }
  uint32_t k = rd_u32(in + p);
  p += 4;
  if ((size_t)k * width > n - p) { free(idx); return ORC_E_OUT_OF_SPEC; }
  for (size_t i = 0; i < length; i++) {
    if (idx[i] >= k) { free(idx); return ORC_E_OUT_OF_SPEC; } /* data[i] OOB panics */
    memcpy(out + i * width, in + p + (size_t)idx[i] * width, (size_t)width);
  }
  free(idx);
  return ORC_OK;
}

/* Freq::decompress (integer/freq.rs:88-123; double/freq.rs:90-123) */
static int freq_decode(const uint8_t* in, size_t n, int width, size_t length, uint8_t* out,
                       int is_float) {
  size_t p = 0;
  if (n < (size_t)width + 4) return ORC_E_IO;
  for (size_t i = 0; i < length; i++) memcpy(out + i * width, in, (size_t)width);
  p = (size_t)width;
  uint32_t bm = rd_u32(in + p);
  p += 4;
  if (p + bm > n) return ORC_E_IO;
  size_t cnt = 0;
  int rc = orc_roaring_decode(in + p, bm, NULL, 0, &cnt);
  if (rc) return rc;
  uint32_t* pos = (uint32_t*)malloc((cnt ? cnt : 1) * 4);
  orc_roaring_decode(in + p, bm, pos, cnt, &cnt);
  p += bm;
  uint8_t* exc = (uint8_t*)malloc((cnt ? cnt : 1) * (size_t)width);
  rc = decompress_stream(in, n, &p, width, cnt, exc, is_float);
  if (!rc) {
    for (size_t i = 0; i < cnt; i++) {
      if (pos[i] >= length) { rc = ORC_E_OUT_OF_SPEC; break; } /* output[] OOB panics */
      memcpy(out + (size_t)pos[i] * width, exc + i * width, (size_t)width);
    }
  }
  free(pos);
  free(exc);
  return rc;
}

/* decompress_integer (integer/mod.rs:72-117) / decompress_double
 * (double/mod.rs:69-114): header, then the codec body.  The reference hands
 * Extend codecs the rest of the reader buffer; well-formed bodies never read
 * past csize, so the restatement bounds them by csize. */
static int decompress_stream(const uint8_t* buf, size_t len, size_t* pos, int width, size_t length,
                             uint8_t* out, int is_float) {
  int codec;
  size_t csize, usize;
  int rc = read_header(buf, len, pos, &codec, &csize, &usize);
  if (rc) return rc;
  const uint8_t* body = buf + *pos;
  (void)usize;
  switch (codec) {
    case ORC_NONE: case ORC_LZ4: case ORC_ZSTD: case ORC_SNAPPY:
      rc = orc_common_decompress(codec, body, csize, out, length * (size_t)width);
      break;
    case ORC_RLE: rc = rle_decode(body, csize, width, length, out); break;
    case ORC_DICT: rc = dict_decode(body, csize, width, length, out); break;
    case ORC_ONE_VALUE: rc = one_value_decode(body, csize, width, length, out); break;
    case ORC_FREQ: rc = freq_decode(body, csize, width, length, out, is_float); break;
    case ORC_BITPACKING:
      rc = is_float ? ORC_E_OUT_OF_SPEC : bp_decode(body, csize, width, length, out, 0);
      break;
    case ORC_DELTA_BITPACKING:
      rc = is_float ? ORC_E_OUT_OF_SPEC : bp_decode(body, csize, width, length, out, 1);
      break;
    case ORC_PATAS:
      rc = is_float ? patas_decode(body, csize, width, length, out) : ORC_E_OUT_OF_SPEC;
      break;
    default: rc = ORC_E_OUT_OF_SPEC; break;
  }
  if (rc) return rc;
  *pos += csize;
  return ORC_OK;
}

int orc_decompress_integer(const uint8_t* buf, size_t len, size_t* pos, int width, size_t length,
                           uint8_t* out) {
  if (width != 1 && width != 2 && width != 4 && width != 8) return ORC_E_ARG;
  return decompress_stream(buf, len, pos, width, length, out, 0);
}

int orc_decompress_double(const uint8_t* buf, size_t len, size_t* pos, int width, size_t length,
                          uint8_t* out) {
  if (width != 4 && width != 8) return ORC_E_ARG;
  return decompress_stream(buf, len, pos, width, length, out, 1);
}

/* ======================================================================= */
/* hybrid RLE / bit-packed (parquet2 0.17 encoding::hybrid_rle)              */
/* ======================================================================= */
static int uleb(const uint8_t* b, size_t n, size_t* p, uint64_t* v) {
  uint64_t r = 0;
  int sh = 0;
  for (;;) {
    if (*p >= n || sh > 63) return ORC_E_OUT_OF_SPEC;
    uint8_t c = b[(*p)++];
    r |= (uint64_t)(c & 0x7F) << sh;
    if (!(c & 0x80)) break;
    sh += 7;
  }
  *v = r;
  return ORC_OK;
}

int orc_hybrid_decode(const uint8_t* buf, size_t len, uint32_t bw, size_t n, uint32_t* out) {
  size_t p = 0, got = 0;
  if (bw > 32) return ORC_E_ARG;
  /* parquet2 0.17 HybridRleDecoder with num_bits 0 (max level 0: a required
   * nest chain writes no stream, arrow2 write_rep_levels / write_def_levels
   * return early) yields 0 for every level without reading the bytes */
  if (bw == 0) {
    for (size_t i = 0; i < n; i++) out[i] = 0;
    return ORC_OK;
  }
  while (got < n) {
    uint64_t h;
    if (uleb(buf, len, &p, &h)) return ORC_E_OUT_OF_SPEC;
    if (h & 1) {
      uint64_t groups = h >> 1;
      size_t nbytes = (size_t)(groups * bw);
      size_t have = len - p < nbytes ? len - p : nbytes; /* parquet2 clamps to the buffer */
      size_t vals = (size_t)groups * 8;
      if (bw == 0) {
        for (size_t i = 0; i < vals && got < n; i++) out[got++] = 0;
        continue;
      }
      size_t maxv = have * 8 / bw;
      if (vals > maxv) vals = maxv;
      for (size_t i = 0; i < vals && got < n; i++) {
        uint64_t bit = (uint64_t)i * bw, v = 0;
        for (uint32_t k = 0; k < bw; k++) {
          uint64_t q = bit + k;
          v |= (uint64_t)((buf[p + (q >> 3)] >> (q & 7)) & 1) << k;
        }
        out[got++] = (uint32_t)v;
      }
      p += have;
      if (vals == 0) return ORC_E_OUT_OF_SPEC;
    } else {
      uint64_t run = h >> 1;
      size_t vb = (bw + 7) / 8;
      if (p + vb > len) return ORC_E_OUT_OF_SPEC;
      uint32_t v = 0;
      for (size_t k = 0; k < vb; k++) v |= (uint32_t)buf[p + k] << (8 * k);
      p += vb;
      for (uint64_t i = 0; i < run && got < n; i++) out[got++] = v;
    }
  }
  return ORC_OK;
}

/* ======================================================================= */
/* validity: read_validity (read/read_basic.rs:36-63) and write_validity    */
/* (write/serialize.rs:200-215 -> arrow2 write_def_levels V2 -> parquet2    */
/* encode_bool: one bit-packed run, header = ceil(n/8) << 1 | 1)            */
/* ======================================================================= */
int orc_read_validity(const uint8_t* buf, size_t len, size_t* pos, size_t length, uint8_t* out_bits) {
  if (*pos + 4 > len) return ORC_E_IO;
  uint32_t def_len = rd_u32(buf + *pos);
  *pos += 4;
  size_t nbytes = (length + 7) / 8;
  if (def_len == 0) {
    /* nothing pushed: the array's validity length then mismatches (try_new
     * fails) unless the page is empty */
    return length == 0 ? ORC_OK : ORC_E_OUT_OF_SPEC;
  }
  if (*pos + def_len > len) return ORC_E_IO;
  const uint8_t* d = buf + *pos;
  size_t p = 0;
  uint64_t h;
  if (uleb(d, def_len, &p, &h)) return ORC_E_OUT_OF_SPEC;
  if (!(h & 1)) return ORC_E_OUT_OF_SPEC; /* Rle => unreachable!() (read_basic.rs:59) */
  size_t groups = (size_t)(h >> 1);
  size_t avail = def_len - p < groups ? def_len - p : groups;
  if (avail * 8 < length) return ORC_E_OUT_OF_SPEC; /* BitmapIter bound */
  memcpy(out_bits, d + p, nbytes);
  if (length & 7) out_bits[nbytes - 1] &= (uint8_t)((1u << (length & 7)) - 1);
  *pos += def_len;
  return ORC_OK;
}

int orc_write_validity(const uint8_t* validity, size_t length, orc_buf* out) {
  size_t nbytes = (length + 7) / 8;
  uint8_t hdr[10];
  size_t hl = 0;
  uint64_t h = ((uint64_t)nbytes << 1) | 1;
  do {
    uint8_t c = h & 0x7F;
    h >>= 7;
    if (h) c |= 0x80;
    hdr[hl++] = c;
  } while (h);
  buf_u32(out, (uint32_t)(hl + nbytes));
  buf_put(out, hdr, hl);
  size_t at = out->len;
  buf_reserve(out, nbytes);
  for (size_t i = 0; i < nbytes; i++) out->data[at + i] = 0;
  for (size_t i = 0; i < length; i++)
    if (is_valid(validity, i)) out->data[at + (i >> 3)] |= (uint8_t)(1u << (i & 7));
  out->len += nbytes;
  return ORC_OK;
}

/* ======================================================================= */
/* encoders                                                                  */
/* ======================================================================= */
typedef struct {
  const uint8_t* values;
  const uint8_t* validity;
  size_t n;
  int width;
  int is_signed;
  int is_float;
} arr_t;

static uint64_t val_at(const arr_t* a, size_t i) { return ld_w(a->values + i * a->width, a->width); }

/* OrderedFloat ordering for doubles (double/traits.rs): NaN is the greatest
 * and equal to itself; -0.0 == 0.0. Returns a totally ordered u64 key. */
static uint64_t float_order_key(uint64_t bits, int width) {
  if (width == 4) {
    uint32_t b = (uint32_t)bits;
    if ((b & 0x7F800000u) == 0x7F800000u && (b & 0x7FFFFFu)) return 0xFFFFFFFFull; /* NaN */
    if ((b & 0x7FFFFFFFu) == 0) b = 0; /* -0 == 0 */
    return (b & 0x80000000u) ? (uint64_t)(~b) : (uint64_t)(b | 0x80000000u);
  }
  if ((bits & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (bits & 0xFFFFFFFFFFFFFull))
    return 0xFFFFFFFFFFFFFFFFull;
  if ((bits & 0x7FFFFFFFFFFFFFFFull) == 0) bits = 0;
  return (bits & 0x8000000000000000ull) ? ~bits : (bits | 0x8000000000000000ull);
}

/* comparison key: native order for ints, OrderedFloat order for doubles */
static uint64_t ord_key(const arr_t* a, uint64_t raw) {
  if (a->is_float) return float_order_key(raw, a->width);
  if (a->is_signed) {
    int64_t s = as_i64(raw, a->width, 1);
    return (uint64_t)s ^ 0x8000000000000000ull;
  }
  return raw;
}

/* open-addressing hash map u64 key -> (count, first index) */
typedef struct {
  uint64_t* keys;
  uint32_t* counts;
  uint32_t* first;
  uint8_t* used;
  size_t cap;
  size_t size;
} hmap;

static void hm_init(hmap* m, size_t n) {
  size_t cap = 16;
  while (cap < 2 * n + 16) cap <<= 1;
  m->cap = cap;
  m->size = 0;
  m->keys = (uint64_t*)malloc(cap * 8);
  m->counts = (uint32_t*)malloc(cap * 4);
  m->first = (uint32_t*)malloc(cap * 4);
  m->used = (uint8_t*)calloc(cap, 1);
}
static void hm_free(hmap* m) { free(m->keys); free(m->counts); free(m->first); free(m->used); }
static size_t hm_slot(hmap* m, uint64_t k) {
  uint64_t h = k * 0x9E3779B97F4A7C15ull;
  size_t i = (size_t)(h >> 17) & (m->cap - 1);
  while (m->used[i] && m->keys[i] != k) i = (i + 1) & (m->cap - 1);
  return i;
}
/* returns slot; inserts if absent */
static size_t hm_add(hmap* m, uint64_t k, uint32_t idx) {
  size_t i = hm_slot(m, k);
  if (!m->used[i]) {
    m->used[i] = 1;
    m->keys[i] = k;
    m->counts[i] = 0;
    m->first[i] = idx;
    m->size++;
  }
  m->counts[i]++;
  return i;
}

typedef struct {
  size_t tuple_count, total_bytes, null_count, unique_count;
  int is_sorted;
  uint64_t min, max; /* raw bit patterns */
  hmap distinct;     /* keyed by ord_key (OrderedFloat merges for doubles) */
} stats_t;

/* gen_stats (integer/mod.rs:179-229; double/mod.rs:178-229) */
static void gen_stats(const arr_t* a, stats_t* s) {
  s->tuple_count = a->n;
  s->total_bytes = a->n * (size_t)a->width;
  s->null_count = 0;
  for (size_t i = 0; i < a->n; i++)
    if (!is_valid(a->validity, i)) s->null_count++;
  s->is_sorted = 1;
  s->min = s->max = 0;
  hm_init(&s->distinct, a->n);
  uint64_t last = 0; /* T::default() */
  int init = 0;
  for (size_t i = 0; i < a->n; i++) {
    uint64_t v = val_at(a, i);
    uint64_t kv = ord_key(a, v);
    if (is_valid(a->validity, i)) {
      if (kv < ord_key(a, last)) s->is_sorted = 0;
      if (ord_key(a, last) != kv) last = v;
    }
    hm_add(&s->distinct, kv, (uint32_t)i);
    if (!init) { init = 1; s->min = s->max = v; }
    if (kv > ord_key(a, s->max)) s->max = v;
    else if (kv < ord_key(a, s->min)) s->min = v;
  }
  s->unique_count = s->distinct.size;
}

static void stats_free(stats_t* s) { hm_free(&s->distinct); }

static size_t max_count(const stats_t* s, uint64_t* top_key, uint32_t* top_first) {
  /* the reference iterates a HashMap (order unspecified): ties are broken
   * here by first occurrence in row order, a deterministic choice */
  size_t best = 0;
  uint32_t bf = 0xFFFFFFFFu;
  uint64_t bk = 0;
  for (size_t i = 0; i < s->distinct.cap; i++) {
    if (!s->distinct.used[i]) continue;
    size_t c = s->distinct.counts[i];
    if (c > best || (c == best && s->distinct.first[i] < bf)) {
      best = c;
      bf = s->distinct.first[i];
      bk = s->distinct.keys[i];
    }
  }
  if (top_key) *top_key = bk;
  if (top_first) *top_first = bf;
  return best;
}

static int compress_stream(const arr_t* a, const orc_write_options* opt, orc_rng* rng, orc_buf* out);

/* --- codec encoders (Extend) --- */

/* RLE::compress_integer (integer/rle.rs:64-104); double/rle.rs same shape */
static void rle_encode(const arr_t* a, orc_buf* out) {
  uint32_t seen = 0;
  uint64_t last = 0;
  int all_null = 1;
  for (size_t i = 0; i < a->n; i++) {
    uint64_t v = val_at(a, i);
    if (is_valid(a->validity, i)) {
      if (all_null) {
        all_null = 0;
        last = v;
        seen++;
      } else if (ord_key(a, last) != ord_key(a, v)) { /* OrderedFloat eq for doubles (double/rle.rs:81) */
        buf_u32(out, seen);
        buf_put(out, &last, (size_t)a->width);
        last = v;
        seen = 1;
      } else {
        seen++;
      }
    } else {
      seen++;
    }
  }
  if (seen) {
    buf_u32(out, seen);
    buf_put(out, &last, (size_t)a->width);
  }
}

/* OneValue::encode_native (integer/one_value.rs:63-75) */
static void one_value_encode(const arr_t* a, orc_buf* out) {
  uint64_t v = 0;
  for (size_t i = 0; i < a->n; i++)
    if (is_valid(a->validity, i)) { v = val_at(a, i); break; }
  buf_put(out, &v, (size_t)a->width);
}

/* Bitpacking::compress (integer/bp.rs:37-65) / DeltaBitpacking (delta_bp.rs:37-67).
 * Chunks of 128 (caller guarantees n % 128 == 0). */
static void bp_encode(const arr_t* a, orc_buf* out, int delta) {
  uint32_t initial = 0, chunk[128];
  uint8_t tmp[512];
  for (size_t off = 0; off + 128 <= a->n; off += 128) {
    memcpy(chunk, a->values + off * 4, 512);
    uint32_t b = orc_bp4x_num_bits(chunk); /* num_bits of raw values, also for delta (delta_bp.rs:50) */
    buf_u8(out, (uint8_t)b);
    size_t sz = delta ? orc_bp4x_pack_sorted(initial, chunk, b, tmp) : orc_bp4x_pack(chunk, b, tmp);
    if (delta) initial = chunk[127];
    buf_put(out, tmp, sz);
  }
}

/* Dict::compress (integer/dict.rs:34-73; double/dict.rs:38-77): first
 * occurrence ids over the raw bytes; null => last index (or default first). */
static int dict_encode(const arr_t* a, const orc_write_options* opt, orc_rng* rng, orc_buf* out) {
  hmap m;
  hm_init(&m, a->n);
  uint32_t* idx = (uint32_t*)malloc((a->n ? a->n : 1) * 4);
  uint64_t* sets = (uint64_t*)malloc((a->n ? a->n : 1) * 8);
  size_t nsets = 0;
  uint32_t* id_of = (uint32_t*)malloc(m.cap * 4);
  for (size_t i = 0; i < a->n; i++) {
    uint64_t v;
    if (is_valid(a->validity, i)) {
      v = val_at(a, i);
    } else if (i > 0) {
      idx[i] = idx[i - 1];
      continue;
    } else {
      v = 0;
    }
    size_t before = m.size;
    size_t s = hm_add(&m, v, (uint32_t)i);
    if (m.size != before) {
      id_of[s] = (uint32_t)nsets;
      sets[nsets++] = v;
    }
    idx[i] = id_of[s];
  }
  arr_t ia = {(const uint8_t*)idx, NULL, a->n, 4, 0, 0};
  orc_write_options o2 = *opt;
  o2.forbidden_mask |= 1u << ORC_DICT;
  int rc = compress_stream(&ia, &o2, rng, out);
  if (!rc) {
    buf_u32(out, (uint32_t)nsets);
    for (size_t k = 0; k < nsets; k++) buf_put(out, &sets[k], (size_t)a->width);
  }
  free(idx); free(sets); free(id_of);
  hm_free(&m);
  return rc;
}

/* Freq::compress (integer/freq.rs:34-86; double/freq.rs:34-88) */
static int freq_encode(const arr_t* a, const stats_t* st, const orc_write_options* opt, orc_rng* rng,
                       orc_buf* out) {
  int top_is_null = (double)st->null_count / (double)st->tuple_count >= 0.9;
  uint64_t top = 0;
  if (!top_is_null) {
    uint32_t first;
    max_count(st, NULL, &first);
    top = val_at(a, first);
  }
  uint64_t top_key = ord_key(a, top);
  uint32_t* pos = (uint32_t*)malloc((a->n ? a->n : 1) * 4);
  uint8_t* exc = (uint8_t*)malloc((a->n ? a->n : 1) * (size_t)a->width);
  size_t ne = 0;
  for (size_t i = 0; i < a->n; i++) {
    if (!is_valid(a->validity, i)) continue;
    uint64_t v = val_at(a, i);
    if (top_is_null || ord_key(a, v) != top_key) {
      pos[ne] = (uint32_t)i;
      memcpy(exc + ne * a->width, &v, (size_t)a->width);
      ne++;
    }
  }
  buf_put(out, &top, (size_t)a->width);
  orc_buf bm = {0};
  orc_roaring_encode(pos, ne, &bm);
  buf_u32(out, (uint32_t)bm.len);
  buf_put(out, bm.data, bm.len);
  orc_buf_free(&bm);
  arr_t ea = {exc, NULL, ne, a->width, a->is_signed, a->is_float};
  orc_write_options o2 = *opt;
  o2.forbidden_mask |= 1u << ORC_FREQ;
  int rc = compress_stream(&ea, &o2, rng, out);
  free(pos);
  free(exc);
  return rc;
}

/* Patas::compress (double/patas.rs:37-105) */
static void patas_encode(const arr_t* a, orc_buf* out) {
  enum { BLOCK = 128 };
  hmap last; /* value bits -> last index (via first[] updated in place) */
  hm_init(&last, a->n);
  int W = a->width, bits = 8 * W;
  for (size_t i = 0; i < a->n; i++) {
    uint64_t v = val_at(a, i);
    if (i == 0) {
      buf_put(out, &v, (size_t)W);
    } else {
      size_t s = hm_slot(&last, v);
      size_t ref = last.used[s] ? last.first[s] : 0;
      if (ref > i || i - ref >= BLOCK) ref = i - 1;
      size_t diff = i - ref;
      uint64_t refv = val_at(a, i - diff);
      uint64_t x = v ^ refv;
      uint32_t tz, lz;
      if (x == 0) { tz = (uint32_t)bits; lz = (uint32_t)bits; }
      else {
        tz = (uint32_t)__builtin_ctzll(x);
        lz = (uint32_t)__builtin_clzll(x) - (uint32_t)(64 - bits);
      }
      uint32_t is_equal = tz == (uint32_t)bits;
      uint32_t sig_bits = is_equal ? 0 : (uint32_t)bits - tz - lz;
      uint32_t sig_bytes = (sig_bits >> 3) + ((sig_bits & 7) != 0);
      uint32_t sh = tz - is_equal;
      buf_u16(out, orc_patas_pack((uint32_t)diff, sig_bytes, sh));
      uint64_t xs = sh >= 64 ? 0 : x >> sh;
      buf_put(out, &xs, sig_bytes);
    }
    size_t s = hm_slot(&last, v);
    if (!last.used[s]) { last.used[s] = 1; last.keys[s] = v; last.size++; }
    last.first[s] = (uint32_t)i;
  }
  hm_free(&last);
}

/* --- ratios (compress_ratio impls) --- */
static uint32_t bits_needed(uint64_t x) { uint32_t b = 0; while (x) { b++; x >>= 1; } return b; }

static double dict_ratio(const stats_t* s, int width) { /* integer/dict.rs:105-120 */
  if (s->unique_count * 3 >= s->tuple_count) return 0.0;
  size_t after = s->unique_count * (size_t)width + s->tuple_count * (bits_needed(s->unique_count) / 8);
  after += s->tuple_count * 2 / 128;
  return (double)s->total_bytes / (double)after;
}

static double freq_ratio(const arr_t* a, const stats_t* s) { /* integer/freq.rs:129-151 */
  if (s->unique_count <= 1) return 0.0;
  if ((double)s->null_count / (double)s->tuple_count >= 0.9) return (double)(s->tuple_count - 1);
  size_t mc = max_count(s, NULL, NULL);
  if ((double)mc / (double)s->tuple_count >= 0.9) {
    if (a->is_float || as_i64(s->max, a->width, a->is_signed) >= 256) return (double)(s->tuple_count - 1);
  }
  return 0.0;
}

static size_t extend_encode(int codec, const arr_t* a, const stats_t* st, const orc_write_options* opt,
                            orc_rng* rng, orc_buf* out, int* rc);

/* compress_sample_ratio (integer/mod.rs:310-347): 10 windows of 64 rows at
 * seeded offsets (thread_rng in the reference) when n / 10 > 64. */
static double sample_ratio(int codec, const arr_t* a, const stats_t* full, orc_rng* rng) {
  const size_t SC = 10, SS = 64;
  arr_t sa = *a;
  uint8_t* vals = NULL;
  uint8_t* bits = NULL;
  stats_t st;
  int own = 0;
  if (a->n / SC <= SS) {
    st = *full;
  } else {
    size_t sep = a->n / SC, rem = a->n % SC;
    vals = (uint8_t*)malloc(SC * SS * (size_t)a->width);
    bits = a->validity ? (uint8_t*)calloc((SC * SS + 7) / 8, 1) : NULL;
    for (size_t k = 0; k < SC; k++) {
      size_t range_end = (k == SC - 1 ? sep + rem : sep) - SS;
      size_t begin = k * sep + (size_t)(rng_next(rng) % range_end);
      memcpy(vals + k * SS * a->width, a->values + begin * a->width, SS * (size_t)a->width);
      /* the sample is rebuilt by MutablePrimitiveArray::extend_trusted_len
       * (integer/mod.rs:334-336, double/mod.rs:334-336): arrow2 writes
       * T::default() under each None, so null slots read 0 from here on */
      if (bits)
        for (size_t j = 0; j < SS; j++) {
          if (get_bit(a->validity, begin + j)) bits[(k * SS + j) >> 3] |= (uint8_t)(1u << ((k * SS + j) & 7));
          else memset(vals + (k * SS + j) * a->width, 0, (size_t)a->width);
        }
    }
    sa.values = vals;
    sa.validity = bits;
    sa.n = SC * SS;
    gen_stats(&sa, &st);
    own = 1;
  }
  orc_write_options dflt = {0, 0, 0.0, 0, -1, 0};
  orc_buf tmp = {0};
  int rc = 0;
  size_t sz = extend_encode(codec, &sa, &st, &dflt, rng, &tmp, &rc);
  if (rc) sz = st.total_bytes;
  double r = (double)st.total_bytes / (double)sz;
  orc_buf_free(&tmp);
  if (own) { stats_free(&st); free(vals); free(bits); }
  return r;
}

static size_t extend_encode(int codec, const arr_t* a, const stats_t* st, const orc_write_options* opt,
                            orc_rng* rng, orc_buf* out, int* rc) {
  size_t start = out->len;
  *rc = 0;
  switch (codec) {
    case ORC_RLE: rle_encode(a, out); break;
    case ORC_ONE_VALUE: one_value_encode(a, out); break;
    case ORC_BITPACKING: bp_encode(a, out, 0); break;
    case ORC_DELTA_BITPACKING: bp_encode(a, out, 1); break;
    case ORC_DICT: *rc = dict_encode(a, opt, rng, out); break;
    case ORC_FREQ: *rc = freq_encode(a, st, opt, rng, out); break;
    case ORC_PATAS: patas_encode(a, out); break;
    default: *rc = ORC_E_ARG; break;
  }
  return out->len - start;
}

static int bp_eligible(const arr_t* a, const stats_t* s) { /* bp.rs:92-100 */
  return !(as_i64(s->min, a->width, a->is_signed) < 0 || a->width != 4 || a->n % 128 != 0);
}

static double codec_ratio(int codec, const arr_t* a, const stats_t* s, orc_rng* rng) {
  switch (codec) {
    case ORC_ONE_VALUE: return s->unique_count <= 1 ? (double)s->tuple_count : 0.0;
    case ORC_FREQ: return freq_ratio(a, s);
    case ORC_DICT: return dict_ratio(s, a->width);
    case ORC_RLE: return sample_ratio(ORC_RLE, a, s, rng);
    case ORC_PATAS: return sample_ratio(ORC_PATAS, a, s, rng);
    case ORC_BITPACKING:
      return bp_eligible(a, s) ? sample_ratio(ORC_BITPACKING, a, s, rng) : 0.0;
    case ORC_DELTA_BITPACKING: /* delta_bp.rs:97-110 */
      if (!bp_eligible(a, s) || !s->is_sorted || s->null_count > 0) return 0.0;
      return sample_ratio(ORC_BITPACKING, a, s, rng) * 1.5;
    default: return 0.0;
  }
}

/* choose_compressor (integer/mod.rs:231-308; double/mod.rs:231-307) */
static int choose(const arr_t* a, const stats_t* s, const orc_write_options* opt, orc_rng* rng) {
  uint32_t fm = opt->forbidden_mask;
  if (opt->forced_codec >= 0 && !(fm & (1u << opt->forced_codec))) {
    /* DEVIATION 6: forced Bitpacking only for an eligible page */
    int f = opt->forced_codec;
    int ok = a->is_float ? (f == ORC_FREQ || f == ORC_DICT || f == ORC_RLE || f == ORC_PATAS)
                         : (f == ORC_FREQ || f == ORC_DICT || f == ORC_RLE ||
                            (f == ORC_BITPACKING && bp_eligible(a, s)));
    if (ok) return f;
  }
  int result = opt->default_codec;
  if (!opt->has_ratio) return result;
  double maxr = opt->ratio;
  static const int icands[] = {ORC_ONE_VALUE, ORC_FREQ, ORC_DICT, ORC_RLE, ORC_BITPACKING,
                               ORC_DELTA_BITPACKING};
  static const int dcands[] = {ORC_ONE_VALUE, ORC_FREQ, ORC_DICT, ORC_PATAS, ORC_RLE};
  const int* c = a->is_float ? dcands : icands;
  int nc = a->is_float ? 5 : 6;
  for (int k = 0; k < nc; k++) {
    if (fm & (1u << c[k])) continue;
    double r = codec_ratio(c[k], a, s, rng);
    if (r > maxr) {
      maxr = r;
      result = c[k];
      if (r == (double)s->tuple_count) break;
    }
  }
  return result;
}

/* compress_integer (integer/mod.rs:35-70) / compress_double (double/mod.rs:32-67) */
static int compress_stream(const arr_t* a, const orc_write_options* opt, orc_rng* rng, orc_buf* out) {
  stats_t st;
  gen_stats(a, &st);
  int codec = choose(a, &st, opt, rng);
  buf_u8(out, (uint8_t)codec);
  size_t hpos = out->len;
  buf_u64(out, 0);
  size_t before = out->len;
  int rc = 0;
  if (codec <= ORC_SNAPPY) rc = orc_common_compress(codec, a->values, a->n * (size_t)a->width, out);
  else extend_encode(codec, a, &st, opt, rng, out, &rc);
  stats_free(&st);
  if (rc) return rc;
  uint32_t csize = (uint32_t)(out->len - before), usize = (uint32_t)(a->n * (size_t)a->width);
  memcpy(out->data + hpos, &csize, 4);
  memcpy(out->data + hpos + 4, &usize, 4);
  return ORC_OK;
}

int orc_compress_integer(const uint8_t* values, const uint8_t* validity, size_t n, int width, int is_signed,
                         const orc_write_options* opt, orc_buf* out) {
  if (width != 1 && width != 2 && width != 4 && width != 8) return ORC_E_ARG;
  arr_t a = {values, validity, n, width, is_signed, 0};
  orc_rng rng = {opt->seed};
  return compress_stream(&a, opt, &rng, out);
}

int orc_compress_double(const uint8_t* values, const uint8_t* validity, size_t n, int width,
                        const orc_write_options* opt, orc_buf* out) {
  if (width != 4 && width != 8) return ORC_E_ARG;
  arr_t a = {values, validity, n, width, 1, 1};
  orc_rng rng = {opt->seed};
  return compress_stream(&a, opt, &rng, out);
}

/* ======================================================================= */
/* flat pages: [validity?][value stream] (write/serialize.rs:52-132,        */
/* read/array/integer.rs:68-88, read/array/double.rs:68-88)                 */
/* ======================================================================= */
int orc_read_flat_page(const uint8_t* page, size_t page_len, size_t num_values, int kind, int width,
                       int nullable, uint8_t* out_values, uint8_t* out_bits) {
  size_t pos = 0;
  int rc;
  if (nullable) {
    rc = orc_read_validity(page, page_len, &pos, num_values, out_bits);
    if (rc) return rc;
  }
  rc = kind ? orc_decompress_double(page, page_len, &pos, width, num_values, out_values)
            : orc_decompress_integer(page, page_len, &pos, width, num_values, out_values);
  return rc;
}

int orc_write_flat_page(const uint8_t* values, const uint8_t* validity, size_t n, int kind, int width,
                        int is_signed, int nullable, const orc_write_options* opt, orc_buf* out) {
  if (nullable) orc_write_validity(validity, n, out);
  return kind ? orc_compress_double(values, validity, n, width, opt, out)
              : orc_compress_integer(values, validity, n, width, is_signed, opt, out);
}

/* read_integer / read_double (read/array/integer.rs:210-238,
 * read/array/double.rs:210-238): every page of a column chunk appended.
 * metas = n_pages pairs (length, num_values).  Single-threaded, like the
 * reference's batch reader. */
int orc_read_column(const uint8_t* chunk, size_t len, const uint64_t* metas, size_t n_pages, int kind, int width,
                    int nullable, uint8_t* out_values, uint8_t* out_bits) {
  size_t pos = 0, row = 0;
  uint8_t* tmp = NULL;
  size_t tmp_cap = 0;
  for (size_t p = 0; p < n_pages; p++) {
    size_t plen = (size_t)metas[2 * p], nv = (size_t)metas[2 * p + 1];
    if (pos + plen > len) { free(tmp); return ORC_E_IO; }
    uint8_t* bits = NULL;
    if (nullable) {
      size_t need = (nv + 7) / 8 + 1;
      if (need > tmp_cap) { free(tmp); tmp = (uint8_t*)malloc(need); tmp_cap = need; }
      bits = tmp;
    }
    int rc = orc_read_flat_page(chunk + pos, plen, nv, kind, width, nullable, out_values + row * (size_t)width, bits);
    if (rc) { free(tmp); return rc; }
    if (nullable) {
      if ((row & 7) == 0) {
        memcpy(out_bits + row / 8, bits, (nv + 7) / 8);
      } else {
        for (size_t i = 0; i < nv; i++) {
          size_t r = row + i;
          if (get_bit(bits, i)) out_bits[r >> 3] |= (uint8_t)(1u << (r & 7));
          else out_bits[r >> 3] &= (uint8_t)~(1u << (r & 7));
        }
      }
    }
    pos += plen;
    row += nv;
  }
  free(tmp);
  return ORC_OK;
}

/* ======================================================================= */
/* binary / utf8 pages (compression/binary/{mod,dict,freq,one_value}.rs)     */
/* ======================================================================= */

static int bin_push_off(orc_binvec* o, int64_t v) {
  if (o->n_off == o->cap_off) {
    size_t nc = o->cap_off ? 2 * o->cap_off : 1024;
    int64_t* p = (int64_t*)realloc(o->offsets, nc * sizeof(int64_t));
    if (!p) return -1;
    o->offsets = p;
    o->cap_off = nc;
  }
  o->offsets[o->n_off++] = v;
  return 0;
}

static int bin_push_vals(orc_binvec* o, const uint8_t* p, size_t n) {
  if (o->n_val + n > o->cap_val) {
    size_t nc = o->cap_val ? o->cap_val : 4096;
    while (nc < o->n_val + n) nc *= 2;
    uint8_t* q = (uint8_t*)realloc(o->values, nc);
    if (!q) return -1;
    o->values = q;
    o->cap_val = nc;
  }
  if (n) memcpy(o->values + o->n_val, p, n);
  o->n_val += n;
  return 0;
}

void orc_binvec_free(orc_binvec* o) {
  free(o->offsets);
  free(o->values);
  memset(o, 0, sizeof(*o));
}

static int64_t ld_off(const uint8_t* p, int ow) { return ow == 8 ? (int64_t)rd_u64(p) : (int64_t)(int32_t)rd_u32(p); }

/* decompress_binary (binary/mod.rs:95-183): appends `length` rows to `o`
 * exactly as the reference's Vec<O> / Vec<u8> pair grows. */
int orc_decompress_binary(const uint8_t* buf, size_t len, size_t* pos, size_t length, int ow, orc_binvec* o) {
  int codec;
  size_t csize, usize;
  int rc = read_header(buf, len, pos, &codec, &csize, &usize);
  if (rc) return rc;
  const uint8_t* body = buf + *pos;
  if (codec <= ORC_SNAPPY) {
    /* Basic: offsets stream ((length+1) offsets), then values stream decoded
     * with the SAME codec (the second header's codec byte is not read) */
    size_t ob = (length + 1) * (size_t)ow;
    uint8_t* tmp = (uint8_t*)malloc(ob ? ob : 1);
    rc = orc_common_decompress(codec, body, csize, tmp, ob);
    if (rc) { free(tmp); return rc; }
    *pos += csize;
    int had = o->n_off > 0;
    int64_t last = had ? o->offsets[o->n_off - 1] : 0;
    for (size_t i = 0; i <= length; i++) bin_push_off(o, ld_off(tmp + i * ow, ow));
    free(tmp);
    if (had) { /* "fix offset" (mod.rs:136-144): o[i] = last + o[i+1], drop one */
      size_t s = o->n_off - length - 1;
      for (size_t i = s; i + 1 < o->n_off; i++) o->offsets[i] = last + o->offsets[i + 1];
      o->n_off--;
    }
    size_t vcs, vus;
    int vcodec;
    rc = read_header(buf, len, pos, &vcodec, &vcs, &vus);
    if (rc) return rc;
    (void)vcodec;
    uint8_t* vt = (uint8_t*)malloc(vus ? vus : 1);
    rc = orc_common_decompress(codec, buf + *pos, vcs, vt, vus);
    if (!rc) bin_push_vals(o, vt, vus);
    free(vt);
    if (rc) return rc;
    *pos += vcs;
    return ORC_OK;
  }
  size_t p = 0;
  const uint8_t* in = body;
  size_t n = csize;
  if (codec == ORC_ONE_VALUE) { /* one_value.rs:71-99 */
    if (n < 4) return ORC_E_IO;
    uint32_t l = rd_u32(in);
    if (n - 4 < l) return ORC_E_OUT_OF_SPEC;
    if (o->n_off == 0) bin_push_off(o, 0);
    for (size_t i = 0; i < length; i++) {
      bin_push_vals(o, in + 4, l);
      bin_push_off(o, (int64_t)o->n_val);
    }
  } else if (codec == ORC_DICT) { /* dict.rs:95-141 */
    uint32_t* idx = (uint32_t*)malloc((length ? length : 1) * 4);
    rc = decompress_stream(in, n, &p, 4, length, (uint8_t*)idx, 0);
    if (rc) { free(idx); return rc; }
    if (p + 4 > n) { free(idx); return ORC_E_IO; }
    uint32_t k = rd_u32(in + p);
    p += 4;
    size_t* eoff = (size_t*)malloc(((size_t)k + 1) * sizeof(size_t));
    uint64_t* elen = (uint64_t*)malloc(((size_t)k + 1) * sizeof(uint64_t));
    for (uint32_t e = 0; e < k; e++) {
      if (p + 8 > n) { free(idx); free(eoff); free(elen); return ORC_E_IO; }
      uint64_t l = rd_u64(in + p);
      p += 8;
      if (n - p < l) { free(idx); free(eoff); free(elen); return ORC_E_OUT_OF_SPEC; }
      eoff[e] = p;
      elen[e] = l;
      p += (size_t)l;
    }
    int64_t last;
    if (o->n_off == 0) { bin_push_off(o, 0); last = 0; }
    else last = o->offsets[o->n_off - 1];
    for (size_t i = 0; i < length; i++) {
      if (idx[i] >= k) { free(idx); free(eoff); free(elen); return ORC_E_OUT_OF_SPEC; }
      bin_push_vals(o, in + eoff[idx[i]], (size_t)elen[idx[i]]);
      last += (int64_t)elen[idx[i]];
      bin_push_off(o, last);
    }
    free(idx); free(eoff); free(elen);
  } else if (codec == ORC_FREQ) { /* freq.rs:102-145 */
    if (n < 8) return ORC_E_IO;
    uint64_t tl = rd_u64(in);
    p = 8;
    if (n - p < tl) return ORC_E_OUT_OF_SPEC;
    const uint8_t* top = in + p;
    p += (size_t)tl;
    if (p + 4 > n) return ORC_E_IO;
    uint32_t bm = rd_u32(in + p);
    p += 4;
    if (n - p < bm) return ORC_E_IO;
    size_t cnt;
    rc = orc_roaring_decode(in + p, bm, NULL, 0, &cnt);
    if (rc) return rc;
    uint32_t* pos_e = (uint32_t*)malloc((cnt ? cnt : 1) * 4);
    orc_roaring_decode(in + p, bm, pos_e, cnt, &cnt);
    p += bm;
    if (o->n_off == 0) bin_push_off(o, 0);
    size_t e = 0;
    for (size_t i = 0; i < length; i++) {
      while (e < cnt && pos_e[e] < i) e++; /* contains(i) on ascending positions */
      if (e < cnt && pos_e[e] == i) {
        if (p + 8 > n) { free(pos_e); return ORC_E_IO; }
        uint64_t l = rd_u64(in + p);
        p += 8;
        if (n - p < l) { free(pos_e); return ORC_E_OUT_OF_SPEC; }
        bin_push_vals(o, in + p, (size_t)l);
        p += (size_t)l;
      } else {
        bin_push_vals(o, top, (size_t)tl);
      }
      bin_push_off(o, (int64_t)o->n_val);
    }
    free(pos_e);
  } else {
    return ORC_E_OUT_OF_SPEC;
  }
  *pos += csize;
  return ORC_OK;
}

/* ---- binary encoder (compress_binary, binary/mod.rs:26-93) ---- */
typedef struct {
  const uint8_t* values;
  const int64_t* offsets; /* n+1 absolute */
  const uint8_t* validity;
  size_t n;
  int ow;
  uint64_t parent_values_len;
} barr_t;

static uint64_t fnv1a(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

/* string hash set: returns entry id (first occurrence order) */
typedef struct {
  uint64_t* h;
  uint32_t* id;
  uint32_t* cnt;
  uint8_t* used;
  size_t cap;
  size_t* srow; /* representative row of id */
  size_t n_ids;
} smap;

static void smap_init(smap* m, size_t n) {
  size_t cap = 16;
  while (cap < 2 * n + 16) cap <<= 1;
  m->cap = cap;
  m->h = (uint64_t*)malloc(cap * 8);
  m->id = (uint32_t*)malloc(cap * 4);
  m->cnt = (uint32_t*)malloc(cap * 4);
  m->used = (uint8_t*)calloc(cap, 1);
  m->srow = (size_t*)malloc((n + 1) * sizeof(size_t));
  m->n_ids = 0;
}
static void smap_free(smap* m) { free(m->h); free(m->id); free(m->cnt); free(m->used); free(m->srow); }

static const uint8_t* bstr(const barr_t* a, size_t i, size_t* l) {
  *l = (size_t)(a->offsets[i + 1] - a->offsets[i]);
  return a->values + a->offsets[i];
}

/* insert row i's string; returns id; *slot = table slot */
static uint32_t smap_add(smap* m, const barr_t* a, size_t row, size_t* slot) {
  size_t l;
  const uint8_t* s = bstr(a, row, &l);
  uint64_t h = fnv1a(s, l);
  size_t i = (size_t)(h * 0x9E3779B97F4A7C15ull >> 17) & (m->cap - 1);
  for (;;) {
    if (!m->used[i]) {
      m->used[i] = 1;
      m->h[i] = h;
      m->id[i] = (uint32_t)m->n_ids;
      m->cnt[i] = 0;
      m->srow[m->n_ids++] = row;
      break;
    }
    if (m->h[i] == h) {
      size_t l2;
      const uint8_t* s2 = bstr(a, m->srow[m->id[i]], &l2);
      if (l2 == l && !memcmp(s, s2, l)) break;
    }
    i = (i + 1) & (m->cap - 1);
  }
  m->cnt[i]++;
  if (slot) *slot = i;
  return m->id[i];
}

int orc_compress_binary(const uint8_t* values, const int64_t* offsets, const uint8_t* validity, size_t n, int ow,
                        uint64_t parent_values_len, const orc_write_options* opt, orc_buf* out) {
  barr_t a = {values, offsets, validity, n, ow, parent_values_len};
  orc_rng rng = {opt->seed};
  /* gen_stats (binary/mod.rs:265-300): distinct over every slot incl. nulls */
  smap m;
  smap_init(&m, n);
  for (size_t i = 0; i < n; i++) smap_add(&m, &a, i, NULL);
  size_t null_count = 0;
  for (size_t i = 0; i < n; i++) null_count += !is_valid(validity, i);
  size_t unique = m.n_ids, total_unique = 0;
  for (size_t id = 0; id < m.n_ids; id++) { size_t l; bstr(&a, m.srow[id], &l); total_unique += l + 8; }
  size_t total_bytes = (size_t)parent_values_len + (n + 1) * (size_t)ow;
  size_t maxc = 0, top_id = 0;
  { /* top value: highest count, first occurrence on ties */
    for (size_t i = 0; i < m.cap; i++) {
      if (!m.used[i]) continue;
      if (m.cnt[i] > maxc || (m.cnt[i] == maxc && m.id[i] < top_id)) { maxc = m.cnt[i]; top_id = m.id[i]; }
    }
  }
  (void)rng;
  /* choose_compressor (binary/mod.rs:302-348) */
  int codec = opt->default_codec;
  uint32_t fm = opt->forbidden_mask;
  int forced = -1;
  if (opt->forced_codec == ORC_FREQ && !(fm & (1u << ORC_FREQ))) forced = ORC_FREQ;
  else if (opt->forced_codec == ORC_DICT && !(fm & (1u << ORC_DICT))) forced = ORC_DICT;
  if (forced >= 0) {
    codec = forced;
  } else if (opt->has_ratio) {
    double maxr = opt->ratio;
    int cands[3] = {ORC_ONE_VALUE, ORC_FREQ, ORC_DICT};
    for (int k = 0; k < 3; k++) {
      if (fm & (1u << cands[k])) continue;
      double r = 0.0;
      if (cands[k] == ORC_ONE_VALUE) r = unique <= 1 ? (double)n : 0.0;
      else if (cands[k] == ORC_FREQ) {
        if (unique <= 1) r = 0.0;
        else if ((double)null_count / (double)n >= 0.9) r = (double)(n - 1);
        else if ((double)maxc / (double)n >= 0.9) r = (double)(n - 1);
      } else {
        if (unique * 3 < n) {
          size_t after = total_unique + n * (bits_needed(unique) / 8) + n * 2 / 128;
          r = (double)total_bytes / (double)after;
        }
      }
      if (r > maxr) {
        maxr = r;
        codec = cands[k];
        if (r == (double)n) break;
      }
    }
  }
  int rc = ORC_OK;
  buf_u8(out, (uint8_t)codec);
  size_t hpos = out->len;
  buf_u64(out, 0);
  size_t before = out->len;
  if (codec <= ORC_SNAPPY) {
    /* offsets rebased to 0, then values [first, last) */
    size_t ob = (n + 1) * (size_t)ow;
    uint8_t* tmp = (uint8_t*)malloc(ob);
    for (size_t i = 0; i <= n; i++) {
      int64_t v = offsets[i] - offsets[0];
      memcpy(tmp + i * ow, &v, (size_t)ow);
    }
    rc = orc_common_compress(codec, tmp, ob, out);
    free(tmp);
    if (rc) { smap_free(&m); return rc; }
    uint32_t cs = (uint32_t)(out->len - before), us = (uint32_t)ob;
    memcpy(out->data + hpos, &cs, 4);
    memcpy(out->data + hpos + 4, &us, 4);
    buf_u8(out, (uint8_t)codec);
    size_t h2 = out->len;
    buf_u64(out, 0);
    size_t b2 = out->len;
    size_t vl = (size_t)(offsets[n] - offsets[0]);
    rc = orc_common_compress(codec, values + offsets[0], vl, out);
    uint32_t cs2 = (uint32_t)(out->len - b2), us2 = (uint32_t)vl;
    memcpy(out->data + h2, &cs2, 4);
    memcpy(out->data + h2 + 4, &us2, 4);
    smap_free(&m);
    return rc;
  }
  if (codec == ORC_ONE_VALUE) { /* one_value.rs:50-68: first valid value */
    size_t l = 0;
    const uint8_t* s = (const uint8_t*)"";
    for (size_t i = 0; i < n; i++)
      if (is_valid(validity, i)) { s = bstr(&a, i, &l); break; }
    buf_u32(out, (uint32_t)l);
    buf_put(out, s, l);
  } else if (codec == ORC_DICT) { /* dict.rs:55-93 */
    smap d;
    smap_init(&d, n);
    uint32_t* idx = (uint32_t*)malloc((n ? n : 1) * 4);
    for (size_t i = 0; i < n; i++) {
      if (!is_valid(validity, i) && i > 0) idx[i] = idx[i - 1];
      else idx[i] = smap_add(&d, &a, i, NULL);
    }
    arr_t ia = {(const uint8_t*)idx, NULL, n, 4, 0, 0};
    orc_write_options o2 = *opt;
    o2.forbidden_mask |= 1u << ORC_DICT;
    rc = compress_stream(&ia, &o2, &rng, out);
    if (!rc) {
      buf_u32(out, (uint32_t)d.n_ids);
      for (size_t id = 0; id < d.n_ids; id++) {
        size_t l;
        const uint8_t* s = bstr(&a, d.srow[id], &l);
        buf_u64(out, (uint64_t)l);
        buf_put(out, s, l);
      }
    }
    free(idx);
    smap_free(&d);
  } else if (codec == ORC_FREQ) { /* freq.rs:44-100 */
    int top_null = (double)null_count / (double)n >= 0.9;
    size_t tl = 0;
    const uint8_t* ts = (const uint8_t*)"";
    if (!top_null) ts = bstr(&a, m.srow[top_id], &tl);
    uint32_t* pos = (uint32_t*)malloc((n ? n : 1) * 4);
    size_t ne = 0;
    for (size_t i = 0; i < n; i++) {
      if (!is_valid(validity, i)) continue;
      size_t l;
      const uint8_t* s = bstr(&a, i, &l);
      if (top_null || l != tl || memcmp(s, ts, l)) pos[ne++] = (uint32_t)i;
    }
    buf_u64(out, (uint64_t)tl);
    buf_put(out, ts, tl);
    orc_buf bmb = {0};
    orc_roaring_encode(pos, ne, &bmb);
    buf_u32(out, (uint32_t)bmb.len);
    buf_put(out, bmb.data, bmb.len);
    orc_buf_free(&bmb);
    for (size_t e = 0; e < ne; e++) {
      size_t l;
      const uint8_t* s = bstr(&a, pos[e], &l);
      buf_u64(out, (uint64_t)l);
      buf_put(out, s, l);
    }
    free(pos);
  }
  smap_free(&m);
  if (rc) return rc;
  /* Extend header: csize, usize = parent values length (mod.rs:88) */
  uint32_t cs = (uint32_t)(out->len - before), us = (uint32_t)parent_values_len;
  memcpy(out->data + hpos, &cs, 4);
  memcpy(out->data + hpos + 4, &us, 4);
  return ORC_OK;
}

/* one binary page [validity?][binary streams] appended to o (read_binary loop body) */
int orc_read_binary_page(const uint8_t* page, size_t page_len, size_t n, int nullable, int ow, orc_binvec* o,
                         uint8_t* out_bits) {
  size_t pos = 0;
  int rc;
  if (nullable) {
    rc = orc_read_validity(page, page_len, &pos, n, out_bits);
    if (rc) return rc;
  }
  return orc_decompress_binary(page, page_len, &pos, n, ow, o);
}

int orc_write_binary_page(const uint8_t* values, const int64_t* offsets, const uint8_t* validity, size_t n,
                          int ow, int nullable, uint64_t parent_values_len, const orc_write_options* opt,
                          orc_buf* out) {
  if (nullable) orc_write_validity(validity, n, out);
  return orc_compress_binary(values, offsets, validity, n, ow, parent_values_len, opt, out);
}

/* ======================================================================= */
/* nested List<primitive> pages                                              */
/* writer: write_nested_validity (write/serialize.rs:217-232) -> arrow2     */
/*   write_rep_and_def V2 -> parquet2 encode_u32 (one bit-packed run);       */
/* reader: read_validity_nested (read/read_basic.rs:65-173) + create_list    */
/*   (read/array/list.rs:48).  One list level over a primitive leaf.         */
/* ======================================================================= */
static uint32_t bit_width_of(uint32_t max_level) { uint32_t b = 0; while (max_level) { b++; max_level >>= 1; } return b; }

/* parquet2 0.17 hybrid_rle::encode_u32 (one bit-packed run; header groups =
 * ceil(n / 8)) -> bitpacked_encode_u32: 32-value chunks of 4*bw bytes, then
 * the remainder chunk packed from a buffer that still holds the previous
 * chunk's values past the remainder, truncated to ceil(rem * bw / 8) bytes --
 * so the stream is ceil(n * bw / 8) bytes and the last byte's spare bits are
 * stale levels.  Third-party (not in the reference tree): restated from the
 * published crate, parity unpinned beyond round trips. */
static void encode_levels(const uint32_t* lv, size_t n, uint32_t bw, orc_buf* out) {
  size_t groups = (n + 7) / 8;
  uint8_t hdr[10];
  size_t hl = 0;
  uint64_t h = ((uint64_t)groups << 1) | 1;
  do { uint8_t c = h & 0x7F; h >>= 7; if (h) c |= 0x80; hdr[hl++] = c; } while (h);
  buf_put(out, hdr, hl);
  uint32_t buffer[32] = {0};
  size_t chunks = n / 32, rem = n % 32;
  for (size_t c = 0; c <= chunks; c++) {
    size_t take = c < chunks ? 32 : rem;
    if (take == 0) break;
    for (size_t j = 0; j < take; j++) buffer[j] = lv[c * 32 + j];
    uint8_t packed[128];
    memset(packed, 0, sizeof packed);
    for (size_t j = 0; j < 32; j++)
      for (uint32_t k = 0; k < bw; k++)
        if ((buffer[j] >> k) & 1) { size_t q = j * bw + k; packed[q >> 3] |= (uint8_t)(1u << (q & 7)); }
    buf_put(out, packed, (take * bw + 7) / 8);
  }
}

int orc_write_list_page(const int64_t* list_offsets, const uint8_t* list_validity, size_t rows, int list_nullable,
                        const uint8_t* child_values, const uint8_t* child_validity, int item_nullable, int kind,
                        int width, int is_signed, const orc_write_options* opt, orc_buf* out, uint64_t* num_levels) {
  const uint32_t nl = list_nullable ? 1 : 0, ni = item_nullable ? 1 : 0;
  const uint32_t max_def = nl + 1 + ni;
  size_t cap = rows + (size_t)(list_offsets[rows] - list_offsets[0]) + 1;
  uint32_t* rep = (uint32_t*)malloc(cap * 4);
  uint32_t* def = (uint32_t*)malloc(cap * 4);
  size_t L = 0;
  for (size_t r = 0; r < rows; r++) {
    int64_t b = list_offsets[r], e = list_offsets[r + 1];
    if (nl && !is_valid(list_validity, r)) { rep[L] = 0; def[L] = 0; L++; continue; }
    if (e == b) { rep[L] = 0; def[L] = nl; L++; continue; }
    for (int64_t j = b; j < e; j++) {
      rep[L] = j > b;
      def[L] = ni ? (is_valid(child_validity, (size_t)j) ? max_def : max_def - 1) : max_def;
      L++;
    }
  }
  orc_buf lv = {0};
  encode_levels(rep, L, bit_width_of(1), &lv);
  size_t rep_len = lv.len;
  encode_levels(def, L, bit_width_of(max_def), &lv);
  size_t def_len = lv.len - rep_len;
  buf_u32(out, (uint32_t)rows);
  buf_u32(out, (uint32_t)rep_len);
  buf_u32(out, (uint32_t)def_len);
  buf_put(out, lv.data, lv.len);
  orc_buf_free(&lv);
  free(rep);
  free(def);
  /* leaf values of the page's rows (slice_parquet_array), their validity */
  size_t v0 = (size_t)list_offsets[0], nv = (size_t)(list_offsets[rows] - list_offsets[0]);
  uint8_t* vb = NULL;
  if (child_validity) {
    vb = (uint8_t*)calloc((nv + 7) / 8 + 1, 1);
    for (size_t i = 0; i < nv; i++)
      if (get_bit(child_validity, v0 + i)) vb[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  int rc = kind ? orc_compress_double(child_values + v0 * width, vb, nv, width, opt, out)
                : orc_compress_integer(child_values + v0 * width, vb, nv, width, is_signed, opt, out);
  free(vb);
  *num_levels = L;
  return rc;
}

/* One nested page -> this page's ListArray pieces (appended to the column):
 * offsets (rows, page-relative leaf positions; the final offset is the
 * returned leaf count), list validity bits, leaf values and leaf validity. */
int orc_read_list_page(const uint8_t* page, size_t len, size_t num_levels, int list_nullable, int item_nullable,
                       int kind, int width, int64_t* out_offsets, uint8_t* out_list_bits, uint8_t* out_values,
                       uint8_t* out_leaf_bits, size_t* out_rows, size_t* out_leaves) {
  if (len < 12) return ORC_E_IO;
  uint32_t additional = rd_u32(page), rep_len = rd_u32(page + 4), def_len = rd_u32(page + 8);
  size_t pos = 12;
  if (pos + rep_len > len || pos + rep_len + def_len > len) return ORC_E_IO;
  const uint32_t nl = list_nullable ? 1 : 0, ni = item_nullable ? 1 : 0;
  const uint32_t max_def = nl + 1 + ni;
  uint32_t* rep = (uint32_t*)malloc((num_levels + 1) * 4);
  uint32_t* def = (uint32_t*)malloc((num_levels + 1) * 4);
  int rc = orc_hybrid_decode(page + pos, rep_len, bit_width_of(1), num_levels, rep);
  if (!rc) rc = orc_hybrid_decode(page + pos + rep_len, def_len, bit_width_of(max_def), num_levels, def);
  if (rc) { free(rep); free(def); return rc; }
  pos += rep_len + def_len;
  /* A first level that does not start a row would push leaves outside any
   * list; the ListArray built from it fails its offsets check (OutOfSpec).
   * read_basic.rs:107-164 with cum_sum = [0, nl + 1, nl + 1 + ni], cum_rep = [0, 1, 1] */
  if (num_levels > 0 && rep[0] != 0) { free(rep); free(def); return ORC_E_OUT_OF_SPEC; }
  const uint32_t cs1 = nl + 1;
  size_t rows = 0, leaves = 0;
  for (size_t l = 0; l < num_levels; l++) {
    uint32_t r = rep[l], d = def[l];
    if (r == 0) rows++;
    if (r == 0) { /* depth 0: list push(offset = leaf count, valid = nl && def > 0) */
      out_offsets[rows - 1] = (int64_t)leaves;
      if (nl) {
        if (d > 0) out_list_bits[(rows - 1) >> 3] |= (uint8_t)(1u << ((rows - 1) & 7));
        else out_list_bits[(rows - 1) >> 3] &= (uint8_t)~(1u << ((rows - 1) & 7));
      }
    }
    if (r <= 1 && d >= cs1) { /* depth 1: leaf slot */
      if (ni) {
        if (d != cs1) out_leaf_bits[leaves >> 3] |= (uint8_t)(1u << (leaves & 7));
        else out_leaf_bits[leaves >> 3] &= (uint8_t)~(1u << (leaves & 7));
      }
      leaves++;
    }
    uint32_t next_rep = l + 1 < num_levels ? rep[l + 1] : 0;
    if (next_rep == 0 && rows == additional) break;
  }
  free(rep);
  free(def);
  if (rows != additional) return ORC_E_OUT_OF_SPEC; /* create_list would mis-size */
  rc = kind ? orc_decompress_double(page, len, &pos, width, leaves, out_values)
            : orc_decompress_integer(page, len, &pos, width, leaves, out_values);
  *out_rows = rows;
  *out_leaves = leaves;
  return rc;
}

/* Nested page with `depth` nests over a leaf: read_validity_nested
 * (read/read_basic.rs:65-173) in its general form.  nests[0..depth) come
 * from the field's InitNested chain (read/deserialize.rs:140-233): a List /
 * LargeList / Map pushes InitNested::List (arrow2 NestedOptional /
 * NestedValid: repeated, never "required"), a Struct InitNested::Struct
 * (NestedStruct / NestedStructValid: not repeated, is_required() true);
 * bit d of struct_mask marks the struct nests.  nests[depth] is the leaf
 * (NestedPrimitive: not repeated, not required).  cum_sum / cum_rep run over
 * (nullable + repeated) / repeated (:95-105); a nest is pushed when
 * `rep <= cum_rep[d] && def >= cum_sum[d]` or the nest above was pushed as a
 * required nest that was not valid (:118-137 -- so every child of a null
 * struct gets a slot).  A list push appends the child's current length as
 * its offset, every nullable push its validity `def > cum_sum[d]`; the leaf
 * push counts a leaf slot, valid when right && `def != cum_sum[depth]`
 * (:138-149).  Decoding stops after the level whose successor would start
 * row `additional + 1` (:154-163).  Outputs are page-local: out_offsets[d]
 * (list nests only; NULL for structs) holds counts[d] entries (create_list
 * / create_map append the child's length, counts[d + 1]), out_bits[d] the
 * nest validity when nest_nullable[d]; counts[depth] = leaf slots.
 * (arrow2 0.17 nested_utils, not vendored: the is_required rule is restated
 * from its published source, and pinned against pyarrow's levels for
 * struct and map columns, tests/test_pyarrow_nested.py.) */
int orc_read_nest_page(const uint8_t* page, size_t len, size_t num_levels, int depth, const int* nest_nullable,
                       uint32_t struct_mask, int item_nullable, int kind, int width, int64_t** out_offsets,
                       uint8_t** out_bits, uint8_t* out_values, uint8_t* out_leaf_bits, size_t* counts,
                       size_t* out_rows) {
  if (depth < 1 || depth > 4) return ORC_E_NYI;
  if (len < 12) return ORC_E_IO;
  uint32_t additional = rd_u32(page), rep_len = rd_u32(page + 4), def_len = rd_u32(page + 8);
  size_t pos = 12;
  if (pos + rep_len > len || pos + rep_len + def_len > len) return ORC_E_IO;
  const int max_depth = depth + 1;
  int nullable[5], repeated[5], required[5];
  for (int d = 0; d < depth; d++) {
    const int is_struct = (struct_mask >> d) & 1;
    nullable[d] = nest_nullable[d] != 0;
    repeated[d] = !is_struct;
    required[d] = is_struct;
  }
  nullable[depth] = item_nullable != 0; repeated[depth] = 0; required[depth] = 0;
  uint32_t cum_sum[6] = {0}, cum_rep[6] = {0};
  for (int d = 0; d < max_depth; d++) {
    cum_sum[d + 1] = cum_sum[d] + (uint32_t)(nullable[d] + repeated[d]);
    cum_rep[d + 1] = cum_rep[d] + (uint32_t)repeated[d];
  }
  uint32_t* rep = (uint32_t*)malloc((num_levels + 1) * 4);
  uint32_t* def = (uint32_t*)malloc((num_levels + 1) * 4);
  int rc = orc_hybrid_decode(page + pos, rep_len, bit_width_of(cum_rep[max_depth]), num_levels, rep);
  if (!rc) rc = orc_hybrid_decode(page + pos + rep_len, def_len, bit_width_of(cum_sum[max_depth]), num_levels, def);
  if (rc) { free(rep); free(def); return rc; }
  pos += rep_len + def_len;
  if (num_levels > 0 && rep[0] != 0) { free(rep); free(def); return ORC_E_OUT_OF_SPEC; }
  size_t n[5] = {0}, rows = 0;
  for (size_t l = 0; l < num_levels; l++) {
    const uint32_t r = rep[l], dv = def[l];
    if (r == 0) rows++;
    int is_required = 0;
    for (int d = 0; d < max_depth; d++) {
      const int right = r <= cum_rep[d] && dv >= cum_sum[d];
      if (!(is_required || right)) continue;
      const int is_valid = nullable[d] && dv > cum_sum[d];
      if (d < depth) {
        if (repeated[d]) out_offsets[d][n[d]] = (int64_t)n[d + 1];
        if (nullable[d]) {
          if (is_valid) out_bits[d][n[d] >> 3] |= (uint8_t)(1u << (n[d] & 7));
          else out_bits[d][n[d] >> 3] &= (uint8_t)~(1u << (n[d] & 7));
        }
      } else if (nullable[d]) {
        if (right && dv != cum_sum[d]) out_leaf_bits[n[d] >> 3] |= (uint8_t)(1u << (n[d] & 7));
        else out_leaf_bits[n[d] >> 3] &= (uint8_t)~(1u << (n[d] & 7));
      }
      n[d]++;
      is_required = required[d] && !is_valid;
    }
    uint32_t next_rep = l + 1 < num_levels ? rep[l + 1] : 0;
    if (next_rep == 0 && rows == additional) break;
  }
  free(rep);
  free(def);
  if (rows != additional) return ORC_E_OUT_OF_SPEC;
  /* the leaf's values (read_nested_integer / _binary / _boolean): kind 0 / 1 =
   * integer / double stream of `width` bytes, 2 = decompress_binary with
   * offset width `width` into the orc_binvec at out_values, 3 =
   * decompress_boolean into the bitmap at out_values */
  if (kind == 2) rc = orc_decompress_binary(page, len, &pos, n[depth], width, (orc_binvec*)out_values);
  else if (kind == 3) rc = orc_decompress_boolean(page, len, &pos, n[depth], out_values);
  else rc = kind ? orc_decompress_double(page, len, &pos, width, n[depth], out_values)
                 : orc_decompress_integer(page, len, &pos, width, n[depth], out_values);
  for (int d = 0; d <= depth; d++) counts[d] = n[d];
  *out_rows = rows;
  return rc;
}

/* depth list levels over a leaf (no struct nests) */
int orc_read_nested_page(const uint8_t* page, size_t len, size_t num_levels, int depth, const int* list_nullable,
                         int item_nullable, int kind, int width, int64_t** out_offsets, uint8_t** out_bits,
                         uint8_t* out_values, uint8_t* out_leaf_bits, size_t* counts, size_t* out_rows) {
  return orc_read_nest_page(page, len, num_levels, depth, list_nullable, 0u, item_nullable, kind, width,
                            out_offsets, out_bits, out_values, out_leaf_bits, counts, out_rows);
}

/* A nested page from precomputed levels (write_nested, write/serialize.rs:
 * 133-146, with write_nested_validity :217-232): [u32 rows][u32 rep_len]
 * [u32 def_len][rep][def] + the leaf's values stream.  Each level stream is
 * arrow2's write_rep_levels / write_def_levels V2 -- nothing when the max
 * level is 0, else parquet2 encode_u32 at get_bit_width(max level).  The
 * levels themselves (arrow2 to_nested + RepLevelsIter / DefLevelsIter) are
 * made by oracle.nest_levels. */
int orc_write_levels_page(const uint32_t* rep, const uint32_t* def, size_t n_levels, uint32_t max_rep,
                          uint32_t max_def, uint32_t rows, orc_buf* out) {
  orc_buf lv = {0};
  if (max_rep) encode_levels(rep, n_levels, bit_width_of(max_rep), &lv);
  const size_t rep_len = lv.len;
  if (max_def) encode_levels(def, n_levels, bit_width_of(max_def), &lv);
  const size_t def_len = lv.len - rep_len;
  buf_u32(out, rows);
  buf_u32(out, (uint32_t)rep_len);
  buf_u32(out, (uint32_t)def_len);
  if (lv.len) buf_put(out, lv.data, lv.len);
  orc_buf_free(&lv);
  return ORC_OK;
}

/* ======================================================================= */
/* boolean pages (compression/boolean/{mod,rle,one_value}.rs,               */
/* read/array/boolean.rs:59-79, 191-219, write/boolean.rs:24-33)            */
/* ======================================================================= */
typedef struct {
  size_t rows, null_count, false_count, true_count, total_bytes;
} bstats_t;

/* gen_stats (boolean/mod.rs:178-220); total_bytes = values().len() / 8 */
static void bool_stats(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, bstats_t* s) {
  memset(s, 0, sizeof *s);
  s->rows = n;
  s->total_bytes = n / 8;
  for (size_t i = 0; i < n; i++) {
    if (!is_valid(validity, i)) { s->null_count++; continue; }
    if (get_bit(bits, off + i)) s->true_count++; else s->false_count++;
  }
}

/* RLE::compress_integer over the bits as u8 (boolean/rle.rs:31-39 ->
 * integer/rle.rs:64-104): nulls extend the current run. */
static void bool_rle_encode(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, orc_buf* out) {
  uint32_t seen = 0;
  uint8_t last = 0;
  int all_null = 1;
  for (size_t i = 0; i < n; i++) {
    uint8_t v = (uint8_t)get_bit(bits, off + i);
    if (is_valid(validity, i)) {
      if (all_null) { all_null = 0; last = v; seen++; }
      else if (last != v) { buf_u32(out, seen); buf_u8(out, last); last = v; seen = 1; }
      else seen++;
    } else {
      seen++;
    }
  }
  if (seen) { buf_u32(out, seen); buf_u8(out, last); }
}

/* compress_sample_ratio (boolean/mod.rs:282-321) for RLE: 10 windows of 64
 * rows at seeded offsets when n / 10 > 64.  The sample is rebuilt from
 * Option<bool> (MutableBooleanArray), so null slots read false. */
static double bool_rle_ratio(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, orc_rng* rng) {
  const size_t SC = 10, SS = 64;
  orc_buf tmp = {0};
  size_t total_bytes;
  if (n / SC <= SS) {
    total_bytes = n / 8;
    bool_rle_encode(bits, off, validity, n, &tmp);
  } else {
    uint8_t sb[(10 * 64) / 8], sv[(10 * 64) / 8];
    memset(sb, 0, sizeof sb);
    memset(sv, 0, sizeof sv);
    size_t sep = n / SC, rem = n % SC;
    for (size_t k = 0; k < SC; k++) {
      size_t range_end = (k == SC - 1 ? sep + rem : sep) - SS;
      size_t begin = k * sep + (size_t)(rng_next(rng) % range_end);
      for (size_t j = 0; j < SS; j++) {
        size_t q = k * SS + j;
        int valid = is_valid(validity, begin + j);
        if (valid) sv[q >> 3] |= (uint8_t)(1u << (q & 7));
        if (valid && get_bit(bits, off + begin + j)) sb[q >> 3] |= (uint8_t)(1u << (q & 7));
      }
    }
    total_bytes = SC * SS / 8;
    bool_rle_encode(sb, 0, validity ? sv : NULL, SC * SS, &tmp);
  }
  double r = (double)total_bytes / (double)tmp.len;
  orc_buf_free(&tmp);
  return r;
}

/* choose_compressor (boolean/mod.rs:222-280) */
static int bool_choose(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, const bstats_t* s,
                       const orc_write_options* opt, orc_rng* rng) {
  uint32_t fm = opt->forbidden_mask;
  if (opt->forced_codec == ORC_RLE && !(fm & (1u << ORC_RLE))) return ORC_RLE; /* check_rle_env */
  int result = opt->default_codec;
  if (!opt->has_ratio) return result;
  double maxr = opt->ratio;
  static const int cands[] = {ORC_ONE_VALUE, ORC_RLE};
  for (int k = 0; k < 2; k++) {
    if (fm & (1u << cands[k])) continue;
    double r = cands[k] == ORC_ONE_VALUE ? ((s->true_count == 0 || s->false_count == 0) ? (double)s->rows : 0.0)
                                         : bool_rle_ratio(bits, off, validity, n, rng);
    if (r > maxr) {
      maxr = r;
      result = cands[k];
      if (r == (double)s->rows) break;
    }
  }
  return result;
}

/* compress_boolean (boolean/mod.rs:22-61).  bits = the column's values
 * bitmap, off = the page's first row (the page is array.slice(off, n)):
 * Basic compresses bitmap.as_slice() -- the parent's bytes verbatim when
 * off % 8 == 0 (trailing bits of the last byte belong to the next rows),
 * else a rebuilt, zero-padded bitmap.  validity is page-relative. */
int orc_compress_boolean(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n,
                         const orc_write_options* opt, orc_buf* out) {
  bstats_t s;
  orc_rng rng = {opt->seed};
  bool_stats(bits, off, validity, n, &s);
  int codec = bool_choose(bits, off, validity, n, &s, opt, &rng);
  buf_u8(out, (uint8_t)codec);
  size_t hpos = out->len;
  buf_u64(out, 0);
  size_t before = out->len;
  int rc = ORC_OK;
  if (codec <= ORC_SNAPPY) {
    size_t nb = (n + 7) / 8;
    if (off % 8 == 0) {
      rc = orc_common_compress(codec, bits + off / 8, nb, out);
    } else {
      uint8_t* tmp = (uint8_t*)calloc(nb ? nb : 1, 1);
      for (size_t i = 0; i < n; i++)
        if (get_bit(bits, off + i)) tmp[i >> 3] |= (uint8_t)(1u << (i & 7));
      rc = orc_common_compress(codec, tmp, nb, out);
      free(tmp);
    }
  } else if (codec == ORC_RLE) {
    bool_rle_encode(bits, off, validity, n, out);
  } else if (codec == ORC_ONE_VALUE) { /* boolean/one_value.rs:44-52: first valid value, else false */
    uint8_t v = 0;
    for (size_t i = 0; i < n; i++)
      if (is_valid(validity, i)) { v = (uint8_t)get_bit(bits, off + i); break; }
    buf_u8(out, v);
  } else {
    rc = ORC_E_ARG;
  }
  if (rc) return rc;
  uint32_t csize = (uint32_t)(out->len - before), usize = (uint32_t)n;
  memcpy(out->data + hpos, &csize, 4);
  memcpy(out->data + hpos + 4, &usize, 4);
  return ORC_OK;
}

/* decompress_boolean (boolean/mod.rs:63-102) of `length` bits into out_bits
 * (page-relative, LSB first).  Basic: (length+7)/8 bytes through the common
 * codec.  RLE (boolean/rle.rs:41-55) and OneValue (one_value.rs:54-61) are
 * handed the rest of the buffer, not csize bytes.  A run total that passes
 * `length` would push extra bits into the next rows (BooleanArray::try_new
 * then fails): OutOfSpec; input ending before `length` bits: Io. */
int orc_decompress_boolean(const uint8_t* buf, size_t len, size_t* pos, size_t length, uint8_t* out_bits) {
  int codec;
  size_t csize, usize;
  int rc = read_header(buf, len, pos, &codec, &csize, &usize);
  if (rc) return rc;
  const uint8_t* body = buf + *pos;
  const size_t rest = len - *pos;
  (void)usize;
  size_t nb = (length + 7) / 8;
  switch (codec) {
    case ORC_NONE: case ORC_LZ4: case ORC_ZSTD: case ORC_SNAPPY: {
      uint8_t* tmp = (uint8_t*)malloc(nb ? nb : 1);
      rc = orc_common_decompress(codec, body, csize, tmp, nb);
      if (!rc)
        for (size_t i = 0; i < length; i++) {
          if (get_bit(tmp, i)) out_bits[i >> 3] |= (uint8_t)(1u << (i & 7));
          else out_bits[i >> 3] &= (uint8_t)~(1u << (i & 7));
        }
      free(tmp);
      break;
    }
    case ORC_RLE: {
      size_t p = 0, produced = 0;
      while (produced < length) {
        if (p + 5 > rest) { rc = ORC_E_IO; break; }
        uint32_t cnt = rd_u32(body + p);
        int v = body[p + 4] != 0;
        p += 5;
        if (produced + cnt > length) { rc = ORC_E_OUT_OF_SPEC; break; }
        for (uint32_t i = 0; i < cnt; i++) {
          size_t q = produced + i;
          if (v) out_bits[q >> 3] |= (uint8_t)(1u << (q & 7));
          else out_bits[q >> 3] &= (uint8_t)~(1u << (q & 7));
        }
        produced += cnt;
      }
      break;
    }
    case ORC_ONE_VALUE: {
      if (rest < 1) { rc = ORC_E_IO; break; }
      int v = body[0] > 0;
      for (size_t i = 0; i < length; i++) {
        if (v) out_bits[i >> 3] |= (uint8_t)(1u << (i & 7));
        else out_bits[i >> 3] &= (uint8_t)~(1u << (i & 7));
      }
      break;
    }
    default: rc = ORC_E_OUT_OF_SPEC; break;
  }
  if (rc) return rc;
  *pos += csize;
  return ORC_OK;
}

/* one flat boolean page: [validity?][boolean stream] (BooleanIter::deserialize) */
int orc_write_bool_page(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, int nullable,
                        const orc_write_options* opt, orc_buf* out) {
  if (nullable) orc_write_validity(validity, n, out);
  return orc_compress_boolean(bits, off, validity, n, opt, out);
}

int orc_read_bool_page(const uint8_t* page, size_t page_len, size_t n, int nullable, uint8_t* out_bits,
                       uint8_t* out_valid) {
  size_t pos = 0;
  int rc;
  if (nullable) {
    rc = orc_read_validity(page, page_len, &pos, n, out_valid);
    if (rc) return rc;
  }
  return orc_decompress_boolean(page, page_len, &pos, n, out_bits);
}

/* read_boolean (read/array/boolean.rs:191-219): pages appended bitwise. */
int orc_read_bool_column(const uint8_t* chunk, size_t len, const uint64_t* metas, size_t n_pages, int nullable,
                         uint8_t* out_bits, uint8_t* out_valid) {
  size_t pos = 0, row = 0;
  int rc = ORC_OK;
  for (size_t p = 0; p < n_pages && !rc; p++) {
    size_t plen = (size_t)metas[2 * p], nv = (size_t)metas[2 * p + 1];
    if (pos + plen > len) return ORC_E_IO;
    uint8_t* vb = (uint8_t*)calloc((nv + 7) / 8 + 1, 1);
    uint8_t* mb = (uint8_t*)calloc((nv + 7) / 8 + 1, 1);
    rc = orc_read_bool_page(chunk + pos, plen, nv, nullable, vb, mb);
    for (size_t i = 0; !rc && i < nv; i++) {
      size_t r = row + i;
      if (get_bit(vb, i)) out_bits[r >> 3] |= (uint8_t)(1u << (r & 7));
      else out_bits[r >> 3] &= (uint8_t)~(1u << (r & 7));
      if (nullable) {
        if (get_bit(mb, i)) out_valid[r >> 3] |= (uint8_t)(1u << (r & 7));
        else out_valid[r >> 3] &= (uint8_t)~(1u << (r & 7));
      }
    }
    free(vb);
    free(mb);
    pos += plen;
    row += nv;
  }
  return rc;
}
