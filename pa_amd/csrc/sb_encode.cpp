// sb_encode.cpp -- host page encoder of the strawboat format (the writer side
// of the engine; GPU encode kernels are the next step).
//
// Restates the reference writer for flat primitive leaves:
//   NativeWriter::encode_chunk paging         write/common.rs:49-119
//   write_simple / write_validity             write/serialize.rs:52-132, 200-215
//   compress_integer / gen_stats / choose     compression/integer/mod.rs:35-347
//   compress_double                           compression/double/mod.rs:32-347
//   codec encoders                            compression/integer/{bp,delta_bp,rle,dict,freq,one_value}.rs,
//                                             compression/double/patas.rs, compression/basic.rs
// The reference samples trial windows with thread_rng and breaks Freq ties
// by HashMap order; here both are deterministic (seeded splitmix64 sampler,
// first-occurrence tie break), so a page encodes to the same bytes on every
// run.  Pages are independent: a column encodes on all host threads.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/strawboat_gpu.h"
#include "sb_encode.h"

extern "C" {
int LZ4_compress_default(const char* src, char* dst, int srcSize, int dstCapacity);
int LZ4_compressBound(int inputSize);
size_t ZSTD_compress(void* dst, size_t dstCapacity, const void* src, size_t srcSize, int level);
size_t ZSTD_compressBound(size_t srcSize);
unsigned ZSTD_isError(size_t code);
}

namespace sb {
namespace enc {

using Bytes = std::vector<uint8_t>;

enum Codec : int {
  kNone = 0, kLz4 = 1, kZstd = 2, kSnappy = 3, kRle = 10, kDict = 11, kOneValue = 12, kFreq = 13,
  kBitpacking = 14, kDeltaBitpacking = 15, kPatas = 16,
};

struct Rng {
  uint64_t s;
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
};

template <class V>
static void put(Bytes& b, V v, size_t nbytes = sizeof(V)) {
  size_t at = b.size();
  b.resize(at + nbytes);
  std::memcpy(b.data() + at, &v, nbytes);
}

static bool bit(const uint8_t* bm, size_t i) { return bm == nullptr || ((bm[i >> 3] >> (i & 7)) & 1); }

// ---- per-type traits: raw bits, order key (PartialOrd / OrderedFloat), as_i64
template <class T>
struct Tr {
  static constexpr bool kFloat = std::is_floating_point<T>::value;
  using Bits = typename std::conditional<sizeof(T) == 8, uint64_t,
               typename std::conditional<sizeof(T) == 4, uint32_t,
               typename std::conditional<sizeof(T) == 2, uint16_t, uint8_t>::type>::type>::type;
  static uint64_t bits(T v) { Bits b; std::memcpy(&b, &v, sizeof(T)); return (uint64_t)b; }
  // total order key: ints by value, floats by OrderedFloat (NaN largest and
  // equal to itself, -0.0 == 0.0)
  static uint64_t key(T v) {
    if constexpr (kFloat) {
      uint64_t b = bits(v);
      constexpr int nb = 8 * sizeof(T);
      constexpr uint64_t sign = 1ull << (nb - 1);
      constexpr uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1);
      if (std::isnan(v)) return all;
      if ((b & (all >> 1)) == 0) b = 0;
      return (b & sign) ? (~b & all) : (b | sign);
    } else if constexpr (std::is_signed<T>::value) {
      return (uint64_t)(int64_t)v ^ 0x8000000000000000ull;
    } else {
      return (uint64_t)v;
    }
  }
  static int64_t as_i64(T v) {
    if constexpr (kFloat) return 0;
    else return (int64_t)v;  // IntegerType::as_i64: `as i64` (u64 wraps)
  }
};

// ---- open-addressing count table (gen_stats's distinct_values HashMap)
struct CountMap {
  std::vector<uint64_t> keys;
  std::vector<uint32_t> count, first;
  std::vector<uint8_t> used;
  size_t mask = 0, size = 0;
  explicit CountMap(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    keys.resize(cap); count.resize(cap); first.resize(cap); used.assign(cap, 0);
    mask = cap - 1;
  }
  size_t slot(uint64_t k) const {
    size_t i = (size_t)((k * 0x9E3779B97F4A7C15ull) >> 17) & mask;
    while (used[i] && keys[i] != k) i = (i + 1) & mask;
    return i;
  }
  // returns true if inserted
  bool add(uint64_t k, uint32_t idx, size_t* where = nullptr) {
    size_t i = slot(k);
    bool ins = !used[i];
    if (ins) { used[i] = 1; keys[i] = k; count[i] = 0; first[i] = idx; size++; }
    count[i]++;
    if (where) *where = i;
    return ins;
  }
};

template <class T>
struct Stats {
  size_t tuple_count = 0, total_bytes = 0, null_count = 0, unique_count = 0;
  bool is_sorted = true;
  T min{}, max{};
  CountMap distinct;
  explicit Stats(size_t n) : distinct(n) {}
};

template <class T>
struct Arr {
  const T* v;
  const uint8_t* valid;  // LSB bitmap or nullptr
  size_t n;
  bool is_signed;
};

// gen_stats (integer/mod.rs:179-229; double/mod.rs:178-229)
template <class T>
static void gen_stats(const Arr<T>& a, Stats<T>& s) {
  s.tuple_count = a.n;
  s.total_bytes = a.n * sizeof(T);
  for (size_t i = 0; i < a.n; i++) s.null_count += !bit(a.valid, i);
  T last{};
  bool init = false;
  for (size_t i = 0; i < a.n; i++) {
    const T v = a.v[i];
    const uint64_t kv = Tr<T>::key(v);
    if (bit(a.valid, i)) {
      if (kv < Tr<T>::key(last)) s.is_sorted = false;
      if (Tr<T>::key(last) != kv) last = v;
    }
    s.distinct.add(kv, (uint32_t)i);
    if (!init) { init = true; s.min = s.max = v; }
    if (kv > Tr<T>::key(s.max)) s.max = v;
    else if (kv < Tr<T>::key(s.min)) s.min = v;
  }
  s.unique_count = s.distinct.size;
}

template <class T>
static size_t top_count(const Stats<T>& s, uint32_t* first_row) {
  size_t best = 0;
  uint32_t bf = 0xFFFFFFFFu;
  for (size_t i = 0; i <= s.distinct.mask; i++) {
    if (!s.distinct.used[i]) continue;
    const size_t c = s.distinct.count[i];
    if (c > best || (c == best && s.distinct.first[i] < bf)) { best = c; bf = s.distinct.first[i]; }
  }
  if (first_row) *first_row = bf;
  return best;
}

// ---- BitPacker4x (bitpacking 0.8.0) pack
static uint32_t bp_num_bits(const uint32_t* x) {
  uint32_t acc = 0;
  for (int i = 0; i < 128; i++) acc |= x[i];
  return acc ? 32 - (uint32_t)__builtin_clz(acc) : 0;
}

static void bp_pack(const uint32_t* x, uint32_t b, Bytes& out) {
  if (!b) return;
  uint32_t words[128] = {0};
  const uint64_t mask = b == 32 ? 0xFFFFFFFFull : ((1ull << b) - 1);
  for (uint32_t i = 0; i < 32; i++) {
    const uint32_t bitp = i * b, k = bitp >> 5, sft = bitp & 31;
    for (int l = 0; l < 4; l++) {
      const uint64_t v = x[4 * i + l] & mask;
      words[4 * k + l] |= (uint32_t)(v << sft);
      if (sft + b > 32) words[4 * (k + 1) + l] |= (uint32_t)(v >> (32 - sft));
    }
  }
  const size_t at = out.size();
  out.resize(at + 16 * b);
  std::memcpy(out.data() + at, words, 16 * b);
}

// ---- snappy raw (greedy hash matcher; valid stream, snap-decodable)
static void snappy_literal(Bytes& o, const uint8_t* p, size_t len) {
  while (len) {
    const size_t c = std::min<size_t>(len, 65536), l1 = c - 1;
    if (l1 < 60) put<uint8_t>(o, (uint8_t)(l1 << 2));
    else if (l1 < 256) { put<uint8_t>(o, 60 << 2); put<uint8_t>(o, (uint8_t)l1); }
    else { put<uint8_t>(o, 61 << 2); put<uint16_t>(o, (uint16_t)l1); }
    o.insert(o.end(), p, p + c);
    p += c;
    len -= c;
  }
}

static void snappy_compress(const uint8_t* in, size_t n, Bytes& o) {
  uint64_t v = n;
  do { uint8_t c = v & 0x7F; v >>= 7; if (v) c |= 0x80; put<uint8_t>(o, c); } while (v);
  constexpr int HB = 14;
  std::vector<int64_t> table((size_t)1 << HB, -1);
  size_t lit = 0, i = 0;
  while (i + 4 <= n) {
    uint32_t w;
    std::memcpy(&w, in + i, 4);
    const uint32_t h = (w * 0x1E35A7BDu) >> (32 - HB);
    const int64_t cand = table[h];
    table[h] = (int64_t)i;
    uint32_t cw = 0;
    if (cand >= 0) std::memcpy(&cw, in + cand, 4);
    if (cand >= 0 && i - (size_t)cand <= 65535 && cw == w) {
      size_t len = 4;
      while (i + len < n && in[cand + len] == in[i + len]) len++;
      if (i > lit) snappy_literal(o, in + lit, i - lit);
      size_t rem = len;
      while (rem) {
        size_t l = std::min<size_t>(rem, 64);
        if (rem > 64 && rem - 64 < 4) l = 60;
        put<uint8_t>(o, (uint8_t)(((l - 1) << 2) | 2));
        put<uint16_t>(o, (uint16_t)(i - (size_t)cand));
        rem -= l;
      }
      i += len;
      lit = i;
    } else {
      i++;
    }
  }
  if (n > lit) snappy_literal(o, in + lit, n - lit);
}

// CommonCompression::compress (basic.rs:74-152)
static int common_compress(int codec, const uint8_t* in, size_t n, Bytes& o) {
  switch (codec) {
    case kNone: o.insert(o.end(), in, in + n); return 0;
    case kLz4: {
      const int bound = LZ4_compressBound((int)n);
      const size_t at = o.size();
      o.resize(at + (size_t)bound);
      const int r = LZ4_compress_default((const char*)in, (char*)o.data() + at, (int)n, bound);
      if (r <= 0 && n) return SB_E_CODEC;
      o.resize(at + (size_t)r);
      return 0;
    }
    case kZstd: {
      const size_t bound = ZSTD_compressBound(n), at = o.size();
      o.resize(at + bound);
      const size_t r = ZSTD_compress(o.data() + at, bound, in, n, 0);
      if (ZSTD_isError(r)) return SB_E_CODEC;
      o.resize(at + r);
      return 0;
    }
    case kSnappy: snappy_compress(in, n, o); return 0;
  }
  return SB_E_ARG;
}

// roaring 0.10.1 serialize_into: cookie 12346, array (<= 4096) / bitmap containers
static void roaring_serialize(const std::vector<uint32_t>& pos, Bytes& o) {
  std::vector<size_t> start;
  for (size_t i = 0; i < pos.size(); i++)
    if (i == 0 || (pos[i] >> 16) != (pos[i - 1] >> 16)) start.push_back(i);
  const size_t nc = start.size();
  start.push_back(pos.size());
  put<uint32_t>(o, 12346);
  put<uint32_t>(o, (uint32_t)nc);
  for (size_t c = 0; c < nc; c++) {
    put<uint16_t>(o, (uint16_t)(pos[start[c]] >> 16));
    put<uint16_t>(o, (uint16_t)(start[c + 1] - start[c] - 1));
  }
  uint32_t off = 8 + 8 * (uint32_t)nc;
  for (size_t c = 0; c < nc; c++) {
    put<uint32_t>(o, off);
    const size_t card = start[c + 1] - start[c];
    off += card <= 4096 ? (uint32_t)(2 * card) : 8192u;
  }
  for (size_t c = 0; c < nc; c++) {
    const size_t card = start[c + 1] - start[c];
    if (card <= 4096) {
      for (size_t i = start[c]; i < start[c + 1]; i++) put<uint16_t>(o, (uint16_t)(pos[i] & 0xFFFF));
    } else {
      uint64_t words[1024] = {0};
      for (size_t i = start[c]; i < start[c + 1]; i++) words[(pos[i] & 0xFFFF) >> 6] |= 1ull << (pos[i] & 63);
      const size_t at = o.size();
      o.resize(at + sizeof words);
      std::memcpy(o.data() + at, words, sizeof words);
    }
  }
}

template <class T>
static int compress_stream(const Arr<T>& a, const Opts& opt, Rng& rng, Bytes& out);

// ---- Extend codec encoders
template <class T>
static void rle_encode(const Arr<T>& a, Bytes& o) {  // integer/rle.rs:64-104, double/rle.rs
  uint32_t seen = 0;
  T last{};
  bool all_null = true;
  for (size_t i = 0; i < a.n; i++) {
    const T v = a.v[i];
    if (bit(a.valid, i)) {
      if (all_null) { all_null = false; last = v; seen++; }
      else if (Tr<T>::key(last) != Tr<T>::key(v)) { put<uint32_t>(o, seen); put<T>(o, last); last = v; seen = 1; }
      else seen++;
    } else {
      seen++;
    }
  }
  if (seen) { put<uint32_t>(o, seen); put<T>(o, last); }
}

template <class T>
static void one_value_encode(const Arr<T>& a, Bytes& o) {  // one_value.rs:63-75
  T v{};
  for (size_t i = 0; i < a.n; i++)
    if (bit(a.valid, i)) { v = a.v[i]; break; }
  put<T>(o, v);
}

template <class T>
static void bp_encode(const Arr<T>& a, Bytes& o, bool delta) {  // bp.rs:37-65, delta_bp.rs:37-67
  uint32_t initial = 0, chunk[128], d[128];
  for (size_t off = 0; off + 128 <= a.n; off += 128) {
    std::memcpy(chunk, a.v + off, 512);
    const uint32_t b = bp_num_bits(chunk);  // of the raw values, also for delta
    put<uint8_t>(o, (uint8_t)b);
    if (delta) {
      uint32_t prev = initial;
      for (int i = 0; i < 128; i++) { d[i] = chunk[i] - prev; prev = chunk[i]; }
      initial = chunk[127];
      bp_pack(d, b, o);
    } else {
      bp_pack(chunk, b, o);
    }
  }
}

template <class T>
static int dict_encode(const Arr<T>& a, const Opts& opt, Rng& rng, Bytes& o) {  // dict.rs:34-73
  CountMap ids(a.n);
  std::vector<uint32_t> idx(a.n), slot_id(ids.mask + 1);
  std::vector<T> sets;
  for (size_t i = 0; i < a.n; i++) {
    T v;
    if (bit(a.valid, i)) v = a.v[i];
    else if (i > 0) { idx[i] = idx[i - 1]; continue; }
    else v = T{};
    size_t where;
    if (ids.add(Tr<T>::bits(v), (uint32_t)i, &where)) { slot_id[where] = (uint32_t)sets.size(); sets.push_back(v); }
    idx[i] = slot_id[where];
  }
  Opts o2 = opt;
  o2.forbidden |= 1u << kDict;
  Arr<uint32_t> ia{idx.data(), nullptr, a.n, false};
  int rc = compress_stream(ia, o2, rng, o);
  if (rc) return rc;
  put<uint32_t>(o, (uint32_t)sets.size());
  for (const T& v : sets) put<T>(o, v);
  return 0;
}

template <class T>
static int freq_encode(const Arr<T>& a, const Stats<T>& st, const Opts& opt, Rng& rng, Bytes& o) {  // freq.rs:34-86
  const bool top_null = (double)st.null_count / (double)st.tuple_count >= 0.9;
  T top{};
  if (!top_null) {
    uint32_t first;
    top_count(st, &first);
    top = a.v[first];
  }
  const uint64_t tk = Tr<T>::key(top);
  std::vector<uint32_t> pos;
  std::vector<T> exc;
  for (size_t i = 0; i < a.n; i++) {
    if (!bit(a.valid, i)) continue;
    if (top_null || Tr<T>::key(a.v[i]) != tk) { pos.push_back((uint32_t)i); exc.push_back(a.v[i]); }
  }
  put<T>(o, top);
  Bytes bm;
  roaring_serialize(pos, bm);
  put<uint32_t>(o, (uint32_t)bm.size());
  o.insert(o.end(), bm.begin(), bm.end());
  Opts o2 = opt;
  o2.forbidden |= 1u << kFreq;
  Arr<T> ea{exc.data(), nullptr, exc.size(), a.is_signed};
  return compress_stream(ea, o2, rng, o);
}

// Patas::compress (double/patas.rs:37-105).  For f32 a value equal to its
// reference makes the reference write 0 significant bytes that its decoder
// reads as 8 (the documented f32 desync): such a page is reported as not
// encodable with Patas (returns false) instead of being written undecodable.
template <class T>
static bool patas_encode(const Arr<T>& a, Bytes& o) {
  constexpr int nb = 8 * sizeof(T);
  CountMap last(a.n);
  for (size_t i = 0; i < a.n; i++) {
    const uint64_t v = Tr<T>::bits(a.v[i]);
    if (i == 0) {
      put<T>(o, a.v[i]);
    } else {
      size_t s = last.slot(v);
      size_t ref = last.used[s] ? last.first[s] : 0;
      if (ref > i || i - ref >= 128) ref = i - 1;
      const size_t diff = i - ref;
      const uint64_t x = v ^ Tr<T>::bits(a.v[i - diff]);
      uint32_t tz, lz;
      if (x == 0) { tz = nb; lz = nb; }
      else { tz = (uint32_t)__builtin_ctzll(x); lz = (uint32_t)__builtin_clzll(x) - (64 - nb); }
      const uint32_t eq = tz == (uint32_t)nb;
      if (eq && nb == 32) return false;
      const uint32_t sig = eq ? 0 : nb - tz - lz;
      const uint32_t sb = (sig >> 3) + ((sig & 7) != 0);
      const uint32_t sh = tz - eq;
      put<uint16_t>(o, (uint16_t)(((diff & 0xFF) << 9) | ((sb & 7) << 6) | (sh & 0xFF)));
      const uint64_t xs = sh >= 64 ? 0 : x >> sh;
      put<uint64_t>(o, xs, sb);
    }
    size_t s = last.slot(v);
    if (!last.used[s]) { last.used[s] = 1; last.keys[s] = v; last.size++; }
    last.first[s] = (uint32_t)i;
  }
  return true;
}

template <class T>
static int extend_encode(int codec, const Arr<T>& a, const Stats<T>& st, const Opts& opt, Rng& rng, Bytes& o) {
  switch (codec) {
    case kRle: rle_encode(a, o); return 0;
    case kOneValue: one_value_encode(a, o); return 0;
    case kBitpacking: if constexpr (sizeof(T) == 4 && !Tr<T>::kFloat) { bp_encode(a, o, false); return 0; } break;
    case kDeltaBitpacking: if constexpr (sizeof(T) == 4 && !Tr<T>::kFloat) { bp_encode(a, o, true); return 0; } break;
    case kDict: return dict_encode(a, opt, rng, o);
    case kFreq: return freq_encode(a, st, opt, rng, o);
    case kPatas: if constexpr (Tr<T>::kFloat) { return patas_encode(a, o) ? 0 : SB_E_CODEC; } break;
  }
  return SB_E_ARG;
}

static uint32_t bits_needed(uint64_t x) { return x ? 64 - (uint32_t)__builtin_clzll(x) : 0; }

// compress_sample_ratio (integer/mod.rs:310-347)
template <class T>
static double sample_ratio(int codec, const Arr<T>& a, const Stats<T>& full, Rng& rng) {
  constexpr size_t SC = 10, SS = 64;
  if (a.n / SC <= SS) {
    Bytes tmp;
    Opts dflt{};
    dflt.forced = -1;
    const int rc = extend_encode(codec, a, full, dflt, rng, tmp);
    const size_t sz = rc ? full.total_bytes : tmp.size();
    return (double)full.total_bytes / (double)sz;
  }
  const size_t sep = a.n / SC, rem = a.n % SC;
  std::vector<T> vals(SC * SS);
  std::vector<uint8_t> bm(a.valid ? (SC * SS + 7) / 8 : 0, 0);
  for (size_t k = 0; k < SC; k++) {
    const size_t range_end = (k == SC - 1 ? sep + rem : sep) - SS;
    const size_t begin = k * sep + (size_t)(rng.next() % range_end);
    std::memcpy(vals.data() + k * SS, a.v + begin, SS * sizeof(T));
    // extend_trusted_len (integer/mod.rs:334-336) writes T::default() under
    // each null slot of the rebuilt sample
    if (a.valid)
      for (size_t j = 0; j < SS; j++) {
        if (bit(a.valid, begin + j)) bm[(k * SS + j) >> 3] |= (uint8_t)(1u << ((k * SS + j) & 7));
        else vals[k * SS + j] = T{};
      }
  }
  Arr<T> sa{vals.data(), a.valid ? bm.data() : nullptr, SC * SS, a.is_signed};
  Stats<T> st(sa.n);
  gen_stats(sa, st);
  Bytes tmp;
  Opts dflt{};
  dflt.forced = -1;
  const int rc = extend_encode(codec, sa, st, dflt, rng, tmp);
  const size_t sz = rc ? st.total_bytes : tmp.size();
  return (double)st.total_bytes / (double)sz;
}

template <class T>
static bool bp_eligible(const Arr<T>& a, const Stats<T>& s) {  // bp.rs:92-100
  return !Tr<T>::kFloat && sizeof(T) == 4 && Tr<T>::as_i64(s.min) >= 0 && a.n % 128 == 0;
}

template <class T>
static double codec_ratio(int c, const Arr<T>& a, const Stats<T>& s, Rng& rng) {
  switch (c) {
    case kOneValue: return s.unique_count <= 1 ? (double)s.tuple_count : 0.0;
    case kFreq: {  // freq.rs:129-151
      if (s.unique_count <= 1) return 0.0;
      if ((double)s.null_count / (double)s.tuple_count >= 0.9) return (double)(s.tuple_count - 1);
      const size_t mc = top_count(s, nullptr);
      if ((double)mc / (double)s.tuple_count >= 0.9 && (Tr<T>::kFloat || Tr<T>::as_i64(s.max) >= 256))
        return (double)(s.tuple_count - 1);
      return 0.0;
    }
    case kDict: {  // dict.rs:105-120
      if (s.unique_count * 3 >= s.tuple_count) return 0.0;
      size_t after = s.unique_count * sizeof(T) + s.tuple_count * (bits_needed(s.unique_count) / 8);
      after += s.tuple_count * 2 / 128;
      return (double)s.total_bytes / (double)after;
    }
    case kRle: case kPatas: return sample_ratio(c, a, s, rng);
    case kBitpacking: return bp_eligible(a, s) ? sample_ratio(kBitpacking, a, s, rng) : 0.0;
    case kDeltaBitpacking:  // delta_bp.rs:97-110
      if (!bp_eligible(a, s) || !s.is_sorted || s.null_count > 0) return 0.0;
      return sample_ratio(kBitpacking, a, s, rng) * 1.5;
  }
  return 0.0;
}

// choose_compressor (integer/mod.rs:231-308; double/mod.rs:231-307)
template <class T>
static int choose(const Arr<T>& a, const Stats<T>& s, const Opts& opt, Rng& rng) {
  const uint32_t fm = opt.forbidden;
  if (opt.forced >= 0 && !(fm & (1u << opt.forced))) {
    const int f = opt.forced;
    // DEVIATION: the reference's forced Bitpacking
    // (check_bitpack_env, integer/mod.rs:259-265) is unconditional; BitPacker4x
    // needs whole 128-value blocks of non-negative values (bp.rs:46-61 packs a
    // short last chunk the decoder cannot read back), so an ineligible page
    // keeps the default codec here.
    const bool ok = Tr<T>::kFloat ? (f == kFreq || f == kDict || f == kRle || f == kPatas)
                                  : (f == kFreq || f == kDict || f == kRle || (f == kBitpacking && bp_eligible(a, s)));
    if (ok) return f;
  }
  int result = opt.default_codec;
  if (!opt.has_ratio) return result;
  double maxr = opt.ratio;
  static const int ic[] = {kOneValue, kFreq, kDict, kRle, kBitpacking, kDeltaBitpacking};
  static const int dc[] = {kOneValue, kFreq, kDict, kPatas, kRle};
  const int* c = Tr<T>::kFloat ? dc : ic;
  const int nc = Tr<T>::kFloat ? 5 : 6;
  for (int k = 0; k < nc; k++) {
    if (fm & (1u << c[k])) continue;
    const double r = codec_ratio(c[k], a, s, rng);
    if (r > maxr) {
      maxr = r;
      result = c[k];
      if (r == (double)s.tuple_count) break;
    }
  }
  return result;
}

// compress_integer / compress_double: [codec u8][csize u32][usize u32][body]
template <class T>
static int compress_stream(const Arr<T>& a, const Opts& opt, Rng& rng, Bytes& out) {
  Stats<T> st(a.n);
  gen_stats(a, st);
  int codec = choose(a, st, opt, rng);
  const size_t hpos = out.size();
  put<uint8_t>(out, (uint8_t)codec);
  put<uint64_t>(out, 0);
  const size_t before = out.size();
  int rc = codec <= kSnappy ? common_compress(codec, (const uint8_t*)a.v, a.n * sizeof(T), out)
                            : extend_encode(codec, a, st, opt, rng, out);
  if (rc == SB_E_CODEC && codec == kPatas) {  // f32 Patas desync guard: fall back to Basic
    out.resize(before);
    codec = opt.default_codec;
    out[hpos] = (uint8_t)codec;
    rc = common_compress(codec, (const uint8_t*)a.v, a.n * sizeof(T), out);
  }
  if (rc) return rc;
  const uint32_t csize = (uint32_t)(out.size() - before), usize = (uint32_t)(a.n * sizeof(T));
  std::memcpy(out.data() + hpos + 1, &csize, 4);
  std::memcpy(out.data() + hpos + 5, &usize, 4);
  return 0;
}

// write_validity (serialize.rs:200-215): u32 def_len + one bit-packed hybrid run
static void write_validity(const uint8_t* valid, size_t n, Bytes& o) {
  const size_t nbytes = (n + 7) / 8;
  uint8_t hdr[10];
  size_t hl = 0;
  uint64_t h = ((uint64_t)nbytes << 1) | 1;
  do { uint8_t c = h & 0x7F; h >>= 7; if (h) c |= 0x80; hdr[hl++] = c; } while (h);
  put<uint32_t>(o, (uint32_t)(hl + nbytes));
  o.insert(o.end(), hdr, hdr + hl);
  const size_t at = o.size();
  o.resize(at + nbytes, 0);
  for (size_t i = 0; i < n; i++)
    if (bit(valid, i)) o[at + (i >> 3)] |= (uint8_t)(1u << (i & 7));
}

template <class T>
static int encode_page_t(const void* values, const uint8_t* valid, size_t n, bool nullable, bool is_signed,
                         const Opts& opt, uint64_t seed, Bytes& out) {
  Rng rng{seed};
  if (nullable) write_validity(valid, n, out);
  Arr<T> a{(const T*)values, valid, n, is_signed};
  return compress_stream(a, opt, rng, out);
}

int encode_page(int phys, const void* values, const uint8_t* valid, size_t n, bool nullable, const Opts& opt,
                uint64_t seed, Bytes& out) {
  switch (phys) {
    case SB_T_INT8: return encode_page_t<int8_t>(values, valid, n, nullable, true, opt, seed, out);
    case SB_T_INT16: return encode_page_t<int16_t>(values, valid, n, nullable, true, opt, seed, out);
    case SB_T_INT32: return encode_page_t<int32_t>(values, valid, n, nullable, true, opt, seed, out);
    case SB_T_INT64: return encode_page_t<int64_t>(values, valid, n, nullable, true, opt, seed, out);
    case SB_T_UINT8: return encode_page_t<uint8_t>(values, valid, n, nullable, false, opt, seed, out);
    case SB_T_UINT16: return encode_page_t<uint16_t>(values, valid, n, nullable, false, opt, seed, out);
    case SB_T_UINT32: return encode_page_t<uint32_t>(values, valid, n, nullable, false, opt, seed, out);
    case SB_T_UINT64: return encode_page_t<uint64_t>(values, valid, n, nullable, false, opt, seed, out);
    case SB_T_FLOAT32: return encode_page_t<float>(values, valid, n, nullable, false, opt, seed, out);
    case SB_T_FLOAT64: return encode_page_t<double>(values, valid, n, nullable, false, opt, seed, out);
  }
  return SB_E_NYI;
}

// ---- nested List<primitive> pages: write_nested (serialize.rs:133-146) =
// write_nested_validity (:217-232: u32 rows, u32 rep_len, u32 def_len, then
// arrow2 write_rep_and_def V2 -> parquet2 encode_u32 per stream) + the leaf
// values of the page's rows through compress_integer / compress_double.
static void encode_levels_u32(const std::vector<uint32_t>& lv, uint32_t bw, Bytes& o) {
  // one bit-packed hybrid run (groups = ceil(n / 8)); bitpacked_encode_u32
  // packs 32-value chunks and truncates the last to ceil(rem * bw / 8) bytes,
  // its spare bits holding the previous chunk's levels (the reused buffer)
  const size_t n = lv.size();
  uint64_t h = ((uint64_t)((n + 7) / 8) << 1) | 1;
  do { uint8_t c = h & 0x7F; h >>= 7; if (h) c |= 0x80; o.push_back(c); } while (h);
  uint32_t buffer[32] = {0};
  for (size_t c0 = 0; c0 < n; c0 += 32) {
    const size_t take = std::min<size_t>(32, n - c0);
    for (size_t j = 0; j < take; j++) buffer[j] = lv[c0 + j];
    uint8_t packed[128] = {0};
    for (size_t j = 0; j < 32; j++) {
      const uint64_t q = (uint64_t)j * bw;
      const uint64_t v = (uint64_t)buffer[j] << (q & 7);
      for (uint32_t k = 0; k < 3 && (q >> 3) + k < 128; k++) packed[(q >> 3) + k] |= (uint8_t)(v >> (8 * k));
    }
    o.insert(o.end(), packed, packed + (take * bw + 7) / 8);
  }
}

static int compress_values(int phys, const void* v, const uint8_t* valid, size_t n, const Opts& opt, Rng& rng, Bytes& o) {
  switch (phys) {
#define SB_CV(E, T, S) case E: { Arr<T> a{(const T*)v, valid, n, S}; return compress_stream(a, opt, rng, o); }
    SB_CV(SB_T_INT8, int8_t, true) SB_CV(SB_T_INT16, int16_t, true) SB_CV(SB_T_INT32, int32_t, true)
    SB_CV(SB_T_INT64, int64_t, true) SB_CV(SB_T_UINT8, uint8_t, false) SB_CV(SB_T_UINT16, uint16_t, false)
    SB_CV(SB_T_UINT32, uint32_t, false) SB_CV(SB_T_UINT64, uint64_t, false) SB_CV(SB_T_FLOAT32, float, false)
    SB_CV(SB_T_FLOAT64, double, false)
#undef SB_CV
  }
  return SB_E_NYI;
}

int encode_list_page(int phys, const int64_t* offsets, const uint8_t* list_valid, size_t rows, bool list_nullable,
                     const void* child, const uint8_t* child_valid, bool item_nullable, const Opts& opt,
                     uint64_t seed, Bytes& out, uint64_t* num_levels) {
  const int ts = type_size(phys);
  if (!ts) return SB_E_NYI;
  Rng rng{seed};
  const uint32_t nl = list_nullable, ni = item_nullable, max_def = nl + 1 + ni;
  std::vector<uint32_t> rep, def;
  rep.reserve(rows + (size_t)(offsets[rows] - offsets[0]));
  def.reserve(rep.capacity());
  for (size_t r = 0; r < rows; r++) {  // RepLevelsIter / DefLevelsIter of one list level
    const int64_t b = offsets[r], e = offsets[r + 1];
    if (nl && !bit(list_valid, r)) { rep.push_back(0); def.push_back(0); continue; }
    if (e == b) { rep.push_back(0); def.push_back(nl); continue; }
    for (int64_t j = b; j < e; j++) {
      rep.push_back(j > b);
      def.push_back(ni ? (bit(child_valid, (size_t)j) ? max_def : max_def - 1) : max_def);
    }
  }
  Bytes lv;
  encode_levels_u32(rep, 1, lv);
  const size_t rep_len = lv.size();
  encode_levels_u32(def, 32 - (uint32_t)__builtin_clz(max_def), lv);
  put<uint32_t>(out, (uint32_t)rows);
  put<uint32_t>(out, (uint32_t)rep_len);
  put<uint32_t>(out, (uint32_t)(lv.size() - rep_len));
  out.insert(out.end(), lv.begin(), lv.end());
  *num_levels = rep.size();
  // slice_parquet_array: the leaf values of rows [0, rows), validity re-based
  const size_t v0 = (size_t)offsets[0], nv = (size_t)(offsets[rows] - offsets[0]);
  std::vector<uint8_t> vb;
  if (child_valid) {
    vb.assign((nv + 7) / 8 + 1, 0);
    for (size_t i = 0; i < nv; i++)
      if (bit(child_valid, v0 + i)) vb[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
  return compress_values(phys, (const uint8_t*)child + v0 * ts, child_valid ? vb.data() : nullptr, nv, opt, rng, out);
}

// ---- any nest chain over any leaf: encode_chunk's to_nested / to_leaves
// (write/common.rs:60-115) for one leaf path, slice_parquet_array over rows
// [r0, r0 + rows), then write_nested (serialize.rs:135-198) with
// write_nested_validity (:217-232).  The levels are the Dremel encoding
// arrow2's RepLevelsIter / DefLevelsIter produce for one leaf: a null nest
// or an empty list emits one level and stops; a struct passes its slot
// through (its children hold one slot per struct slot, null or not); a list
// slot's children repeat at the list's cumulative repetition level.
namespace {
struct LevelWalk {
  const NestLevel* nests;
  int depth;
  const NestLeaf* leaf;
  uint32_t cum_rep[8];  // d + 1 <= SB_MAX_NEST (masked so the inlined recursion stays in bounds)
  std::vector<uint32_t> rep, def;

  void walk(int d, uint64_t i, uint32_t r, uint32_t dl) {
    if (d == depth) {
      rep.push_back(r);
      def.push_back(dl + (leaf->nullable && bit(leaf->validity, (size_t)i)));
      return;
    }
    const NestLevel& n = nests[d];
    if (n.nullable && !bit(n.validity, (size_t)i)) { rep.push_back(r); def.push_back(dl); return; }
    dl += n.nullable;
    if (n.is_struct) { walk(d + 1, i, r, dl); return; }
    const int64_t b = n.offsets[i], e = n.offsets[i + 1];
    if (b == e) { rep.push_back(r); def.push_back(dl); return; }
    for (int64_t j = b; j < e; j++) walk(d + 1, (uint64_t)j, j == b ? r : cum_rep[(d + 1) & 7], dl + 1);
  }
};

void rebase_bits(const uint8_t* bm, uint64_t at, uint64_t n, std::vector<uint8_t>& out) {
  out.assign((n + 7) / 8 + 1, 0);
  for (uint64_t i = 0; i < n; i++)
    if ((bm[(at + i) >> 3] >> ((at + i) & 7)) & 1) out[i >> 3] |= (uint8_t)(1u << (i & 7));
}
}  // namespace

int nested_max_levels(const NestLevel* nests, int depth, bool leaf_nullable, uint32_t* max_rep, uint32_t* max_def) {
  if (depth < 1 || depth > SB_MAX_NEST) return SB_E_NYI;
  uint32_t mr = 0, md = leaf_nullable;
  for (int d = 0; d < depth; d++) {
    mr += !nests[d].is_struct;
    md += nests[d].nullable + !nests[d].is_struct;
  }
  *max_rep = mr;
  *max_def = md;
  return 0;
}

int encode_nested_page(const NestLevel* nests, int depth, const NestLeaf& leaf, uint64_t r0, uint64_t rows,
                       const Opts& opt, uint64_t seed, Bytes& out, uint64_t* num_levels) {
  uint32_t max_rep, max_def;
  if (int rc = nested_max_levels(nests, depth, leaf.nullable, &max_rep, &max_def)) return rc;
  LevelWalk w{nests, depth, &leaf, {0}, {}, {}};
  for (int d = 0; d < depth; d++) w.cum_rep[d + 1] = w.cum_rep[d] + !nests[d].is_struct;
  for (uint64_t i = r0; i < r0 + rows; i++) w.walk(0, i, 0, 0);
  // write_rep_and_def V2: no stream for a max level of 0
  Bytes lv;
  if (max_rep) encode_levels_u32(w.rep, 32 - (uint32_t)__builtin_clz(max_rep), lv);
  const size_t rep_len = lv.size();
  if (max_def) encode_levels_u32(w.def, 32 - (uint32_t)__builtin_clz(max_def), lv);
  put<uint32_t>(out, (uint32_t)rows);
  put<uint32_t>(out, (uint32_t)rep_len);
  put<uint32_t>(out, (uint32_t)(lv.size() - rep_len));
  out.insert(out.end(), lv.begin(), lv.end());
  *num_levels = w.rep.size();
  // slice_parquet_array: the leaf slots of the page's rows, through each list nest
  uint64_t j0 = r0, j1 = r0 + rows;
  for (int d = 0; d < depth; d++)
    if (!nests[d].is_struct) { j0 = (uint64_t)nests[d].offsets[j0]; j1 = (uint64_t)nests[d].offsets[j1]; }
  const uint64_t m = j1 - j0;
  std::vector<uint8_t> vb;
  if (leaf.validity) rebase_bits(leaf.validity, j0, m, vb);
  const uint8_t* valid = leaf.validity ? vb.data() : nullptr;
  if (leaf.phys == SB_T_BOOLEAN)  // write_bitmap over the sliced leaf: the bitmap at bit offset j0
    return encode_bool_page((const uint8_t*)leaf.values, (size_t)j0, valid, (size_t)m, false, opt, seed, out);
  if (leaf.phys >= SB_T_BINARY && leaf.phys <= SB_T_LARGE_UTF8) {
    const int ow = (leaf.phys == SB_T_BINARY || leaf.phys == SB_T_UTF8) ? 4 : 8;
    return encode_binary_page((const uint8_t*)leaf.values, leaf.offsets + j0, valid, (size_t)m, false, ow,
                              leaf.values_len, opt, seed, out);
  }
  const int ts = type_size(leaf.phys);
  if (!ts) return SB_E_NYI;
  Rng rng{seed};
  return compress_values(leaf.phys, (const uint8_t*)leaf.values + j0 * ts, valid, (size_t)m, opt, rng, out);
}

// ---- boolean pages: compress_boolean (compression/boolean/mod.rs:22-61),
// gen_stats (:178-220), choose_compressor (:222-280), RLE over the bits as u8
// (boolean/rle.rs:31-39), OneValue (boolean/one_value.rs:44-52).
static inline bool getb(const uint8_t* bm, size_t i) { return (bm[i >> 3] >> (i & 7)) & 1; }

static void bool_rle(const uint8_t* bits, size_t off, const uint8_t* valid, size_t n, Bytes& o) {
  uint32_t seen = 0;
  uint8_t last = 0;
  bool all_null = true;
  for (size_t i = 0; i < n; i++) {
    const uint8_t v = getb(bits, off + i);
    if (bit(valid, i)) {
      if (all_null) { all_null = false; last = v; seen++; }
      else if (last != v) { put<uint32_t>(o, seen); put<uint8_t>(o, last); last = v; seen = 1; }
      else seen++;
    } else {
      seen++;
    }
  }
  if (seen) { put<uint32_t>(o, seen); put<uint8_t>(o, last); }
}

// compress_sample_ratio (boolean/mod.rs:282-321): seeded windows stand in for
// thread_rng; the rebuilt sample reads false under null slots.
static double bool_rle_ratio(const uint8_t* bits, size_t off, const uint8_t* valid, size_t n, Rng& rng) {
  constexpr size_t SC = 10, SS = 64;
  Bytes tmp;
  size_t total_bytes;
  if (n / SC <= SS) {
    total_bytes = n / 8;
    bool_rle(bits, off, valid, n, tmp);
  } else {
    uint8_t sb[SC * SS / 8] = {0}, sv[SC * SS / 8] = {0};
    const size_t sep = n / SC, rem = n % SC;
    for (size_t k = 0; k < SC; k++) {
      const size_t range_end = (k == SC - 1 ? sep + rem : sep) - SS;
      const size_t begin = k * sep + (size_t)(rng.next() % range_end);
      for (size_t j = 0; j < SS; j++) {
        const size_t q = k * SS + j;
        const bool v = bit(valid, begin + j);
        if (v) sv[q >> 3] |= (uint8_t)(1u << (q & 7));
        if (v && getb(bits, off + begin + j)) sb[q >> 3] |= (uint8_t)(1u << (q & 7));
      }
    }
    total_bytes = SC * SS / 8;
    bool_rle(sb, 0, valid ? sv : nullptr, SC * SS, tmp);
  }
  return (double)total_bytes / (double)tmp.size();
}

// bits = the column's bitmap, off = the page's first row (array.slice): the
// Basic codec takes bitmap.as_slice() -- the parent's bytes when off % 8 == 0
// (boolean/mod.rs:35-46), a rebuilt zero-padded bitmap otherwise.
int encode_bool_page(const uint8_t* bits, size_t off, const uint8_t* valid, size_t n, bool nullable, const Opts& opt,
                     uint64_t seed, Bytes& out) {
  Rng rng{seed};
  if (nullable) write_validity(valid, n, out);
  size_t t = 0, f = 0;
  for (size_t i = 0; i < n; i++)
    if (bit(valid, i)) (getb(bits, off + i) ? t : f)++;
  int codec = opt.default_codec;
  if (opt.forced == kRle && !(opt.forbidden & (1u << kRle))) {
    codec = kRle;  // check_rle_env
  } else if (opt.has_ratio) {
    double maxr = opt.ratio;
    for (int c : {kOneValue, kRle}) {
      if (opt.forbidden & (1u << c)) continue;
      const double r = c == kOneValue ? ((t == 0 || f == 0) ? (double)n : 0.0) : bool_rle_ratio(bits, off, valid, n, rng);
      if (r > maxr) {
        maxr = r;
        codec = c;
        if (r == (double)n) break;
      }
    }
  }
  const size_t hpos = out.size();
  put<uint8_t>(out, (uint8_t)codec);
  put<uint64_t>(out, 0);
  const size_t before = out.size();
  int rc = 0;
  if (codec <= kSnappy) {
    const size_t nb = (n + 7) / 8;
    if (off % 8 == 0) {
      rc = common_compress(codec, bits + off / 8, nb, out);
    } else {
      std::vector<uint8_t> tmp(nb ? nb : 1, 0);
      for (size_t i = 0; i < n; i++)
        if (getb(bits, off + i)) tmp[i >> 3] |= (uint8_t)(1u << (i & 7));
      rc = common_compress(codec, tmp.data(), nb, out);
    }
  } else if (codec == kRle) {
    bool_rle(bits, off, valid, n, out);
  } else if (codec == kOneValue) {
    uint8_t v = 0;
    for (size_t i = 0; i < n; i++)
      if (bit(valid, i)) { v = getb(bits, off + i); break; }
    put<uint8_t>(out, v);
  } else {
    rc = SB_E_ARG;
  }
  if (rc) return rc;
  const uint32_t csize = (uint32_t)(out.size() - before), usize = (uint32_t)n;
  std::memcpy(out.data() + hpos + 1, &csize, 4);
  std::memcpy(out.data() + hpos + 5, &usize, 4);
  return 0;
}

uint64_t page_seed(uint64_t seed, uint64_t page) {
  Rng r{seed ^ (page * 0xD1B54A32D192ED03ull)};
  return r.next();
}

int type_size(int phys) {
  switch (phys) {
    case SB_T_INT8: case SB_T_UINT8: return 1;
    case SB_T_INT16: case SB_T_UINT16: return 2;
    case SB_T_INT32: case SB_T_UINT32: case SB_T_FLOAT32: return 4;
    case SB_T_INT64: case SB_T_UINT64: case SB_T_FLOAT64: return 8;
  }
  return 0;
}

}  // namespace enc
}  // namespace sb

// ===========================================================================
// Binary / Utf8 pages: compress_binary (compression/binary/mod.rs:26-93),
// gen_stats (:265-300), choose_compressor (:302-348), Dict (dict.rs:55-93),
// Freq (freq.rs:44-100), OneValue (one_value.rs:50-68).
// ===========================================================================
namespace sb {
namespace enc {

namespace {

struct BArr {
  const uint8_t* values;
  const int64_t* offsets;  // n + 1 absolute
  const uint8_t* valid;
  size_t n;
  int ow;
  uint64_t parent_len;
  size_t len(size_t i) const { return (size_t)(offsets[i + 1] - offsets[i]); }
  const uint8_t* str(size_t i) const { return values + offsets[i]; }
};

uint64_t fnv1a(const uint8_t* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

// distinct strings in first-occurrence order
struct StrSet {
  std::vector<uint64_t> h;
  std::vector<uint32_t> id, cnt;
  std::vector<uint8_t> used;
  std::vector<size_t> row;  // representative row per id
  size_t mask;
  explicit StrSet(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    h.resize(cap); id.resize(cap); cnt.resize(cap); used.assign(cap, 0);
    mask = cap - 1;
  }
  uint32_t add(const BArr& a, size_t r, size_t* slot = nullptr) {
    const size_t l = a.len(r);
    const uint8_t* s = a.str(r);
    const uint64_t hh = fnv1a(s, l);
    size_t i = (size_t)((hh * 0x9E3779B97F4A7C15ull) >> 17) & mask;
    for (;;) {
      if (!used[i]) { used[i] = 1; h[i] = hh; id[i] = (uint32_t)row.size(); cnt[i] = 0; row.push_back(r); break; }
      if (h[i] == hh) {
        const size_t r2 = row[id[i]];
        if (a.len(r2) == l && std::memcmp(a.str(r2), s, l) == 0) break;
      }
      i = (i + 1) & mask;
    }
    cnt[i]++;
    if (slot) *slot = i;
    return id[i];
  }
};

}  // namespace

int encode_binary_page(const uint8_t* values, const int64_t* offsets, const uint8_t* valid, size_t n, bool nullable,
                       int ow, uint64_t parent_len, const Opts& opt, uint64_t seed, Bytes& out) {
  Rng rng{seed};
  if (nullable) write_validity(valid, n, out);
  BArr a{values, offsets, valid, n, ow, parent_len};
  StrSet m(n);
  for (size_t i = 0; i < n; i++) m.add(a, i);
  size_t nulls = 0;
  for (size_t i = 0; i < n; i++) nulls += !bit(valid, i);
  const size_t unique = m.row.size();
  size_t total_unique = 0;
  for (size_t r : m.row) total_unique += a.len(r) + 8;
  const size_t total_bytes = (size_t)parent_len + (n + 1) * (size_t)ow;
  size_t maxc = 0;
  uint32_t top_id = 0;
  for (size_t i = 0; i <= m.mask; i++) {
    if (!m.used[i]) continue;
    if (m.cnt[i] > maxc || (m.cnt[i] == maxc && m.id[i] < top_id)) { maxc = m.cnt[i]; top_id = m.id[i]; }
  }
  int codec = opt.default_codec;
  const uint32_t fm = opt.forbidden;
  if (opt.forced == kFreq && !(fm & (1u << kFreq))) codec = kFreq;
  else if (opt.forced == kDict && !(fm & (1u << kDict))) codec = kDict;
  else if (opt.has_ratio) {
    double maxr = opt.ratio;
    for (int c : {kOneValue, kFreq, kDict}) {
      if (fm & (1u << c)) continue;
      double r = 0.0;
      if (c == kOneValue) r = unique <= 1 ? (double)n : 0.0;
      else if (c == kFreq) {
        if (unique > 1) {
          if ((double)nulls / (double)n >= 0.9) r = (double)(n - 1);
          else if ((double)maxc / (double)n >= 0.9) r = (double)(n - 1);
        }
      } else if (unique * 3 < n) {
        const size_t after = total_unique + n * (bits_needed(unique) / 8) + n * 2 / 128;
        r = (double)total_bytes / (double)after;
      }
      if (r > maxr) {
        maxr = r;
        codec = c;
        if (r == (double)n) break;
      }
    }
  }
  const size_t hpos = out.size();
  put<uint8_t>(out, (uint8_t)codec);
  put<uint64_t>(out, 0);
  const size_t before = out.size();
  if (codec <= kSnappy) {
    std::vector<uint8_t> ob((n + 1) * (size_t)ow);
    for (size_t i = 0; i <= n; i++) {
      const int64_t v = offsets[i] - offsets[0];
      std::memcpy(ob.data() + i * ow, &v, (size_t)ow);
    }
    int rc = common_compress(codec, ob.data(), ob.size(), out);
    if (rc) return rc;
    const uint32_t cs = (uint32_t)(out.size() - before), us = (uint32_t)ob.size();
    std::memcpy(out.data() + hpos + 1, &cs, 4);
    std::memcpy(out.data() + hpos + 5, &us, 4);
    const size_t h2 = out.size();
    put<uint8_t>(out, (uint8_t)codec);
    put<uint64_t>(out, 0);
    const size_t b2 = out.size();
    const size_t vl = (size_t)(offsets[n] - offsets[0]);
    rc = common_compress(codec, values + offsets[0], vl, out);
    if (rc) return rc;
    const uint32_t cs2 = (uint32_t)(out.size() - b2), us2 = (uint32_t)vl;
    std::memcpy(out.data() + h2 + 1, &cs2, 4);
    std::memcpy(out.data() + h2 + 5, &us2, 4);
    return 0;
  }
  if (codec == kOneValue) {
    size_t l = 0;
    const uint8_t* s = nullptr;
    for (size_t i = 0; i < n; i++)
      if (bit(valid, i)) { s = a.str(i); l = a.len(i); break; }
    put<uint32_t>(out, (uint32_t)l);
    if (l) out.insert(out.end(), s, s + l);
  } else if (codec == kDict) {
    StrSet d(n);
    std::vector<uint32_t> idx(n);
    for (size_t i = 0; i < n; i++) idx[i] = (!bit(valid, i) && i > 0) ? idx[i - 1] : d.add(a, i);
    Opts o2 = opt;
    o2.forbidden |= 1u << kDict;
    Arr<uint32_t> ia{idx.data(), nullptr, n, false};
    const int rc = compress_stream(ia, o2, rng, out);
    if (rc) return rc;
    put<uint32_t>(out, (uint32_t)d.row.size());
    for (size_t r : d.row) {
      put<uint64_t>(out, (uint64_t)a.len(r));
      out.insert(out.end(), a.str(r), a.str(r) + a.len(r));
    }
  } else {  // Freq
    const bool top_null = (double)nulls / (double)n >= 0.9;
    size_t tl = 0;
    const uint8_t* ts = nullptr;
    if (!top_null) { ts = a.str(m.row[top_id]); tl = a.len(m.row[top_id]); }
    std::vector<uint32_t> pos;
    for (size_t i = 0; i < n; i++) {
      if (!bit(valid, i)) continue;
      if (top_null || a.len(i) != tl || std::memcmp(a.str(i), ts, tl) != 0) pos.push_back((uint32_t)i);
    }
    put<uint64_t>(out, (uint64_t)tl);
    if (tl) out.insert(out.end(), ts, ts + tl);
    Bytes bm;
    roaring_serialize(pos, bm);
    put<uint32_t>(out, (uint32_t)bm.size());
    out.insert(out.end(), bm.begin(), bm.end());
    for (uint32_t r : pos) {
      put<uint64_t>(out, (uint64_t)a.len(r));
      out.insert(out.end(), a.str(r), a.str(r) + a.len(r));
    }
  }
  const uint32_t cs = (uint32_t)(out.size() - before), us = (uint32_t)parent_len;
  std::memcpy(out.data() + hpos + 1, &cs, 4);
  std::memcpy(out.data() + hpos + 5, &us, 4);
  return 0;
}

}  // namespace enc
}  // namespace sb
