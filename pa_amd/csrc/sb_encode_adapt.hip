// sb_encode_adapt.hip -- the writer's adaptive codec cascade on MI355X
// (gfx950): NativeWriter::encode_chunk (write/common.rs:49-119) ->
// write_simple (write/serialize.rs:52-132) -> compress_integer /
// compress_double (compression/integer/mod.rs:35-347,
// compression/double/mod.rs:32-347) for every page of a fixed-width column,
// one 256-thread workgroup per page, byte-identical to the host writer
// (sb_encode.cpp) and the oracle (oracle/sb_oracle.c orc_write_flat_page).
//
// Per value stream (compress_stream below, recursive through Dict / Freq):
//   gen_stats (integer/mod.rs:179-229): null count, min / max and
//     sortedness by the type's total order, distinct count and the most
//     frequent value (first occurrence breaks ties: the seeded, tie-broken
//     selection that replaces the reference's HashMap order) -- an LDS
//     open-addressing table of (count << 16 | first row + 1) words, filled
//     with atomicCAS and lowered to the smallest row;
//   choose_compressor (:231-308) with the seeded splitmix64 trial-window
//     sampler (:310-347, 10 windows x 64 rows) standing in for thread_rng;
//   the codecs: RLE (rle.rs:64-104; runs from a boundary flag scan), Dict
//     (dict.rs:34-73; first-occurrence ids from a flag scan over rows, the
//     index stream cascades), Freq (freq.rs:34-86; exception compaction,
//     roaring 0.10.1 array / bitmap container, the exception stream
//     cascades), OneValue, Bitpacking / DeltaBitpacking (bp.rs:37-65,
//     delta_bp.rs:37-67; BitPacker4x words computed per lane word), Patas
//     (double/patas.rs:37-105; the back reference found by a 127-row window
//     search), and the Basic codecs None / LZ4 (sb_lz4c.h, one wave) /
//     Snappy (one lane) / Zstd (sb_zstdc.h: frames transcoded from the LZ4
//     parse; libzstd level 3's bytes are not reproduced, any Zstd decoder
//     returns the page's bytes).
// Pages are written into per-page slots of a batch, then compacted.
// Integer work; bound by the per-page hash/scan work, not by MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/strawboat_gpu.h"
#include "sb_internal.h"
#include "sb_lz4c.h"
#include "sb_zstdc.h"

namespace sba {

#ifndef SB_ENC_NT
#define SB_ENC_NT 256
#endif
constexpr int NT = SB_ENC_NT, NW = NT / 64;
constexpr uint32_t kMaxRows = 16384;      // pages whose statistics' tables fit the LDS work area
constexpr uint32_t SC = 10, SS = 64, kSample = SC * SS;
// A big Boolean page's HBM work area: the RLE run starts (or the Snappy
// table), then the page's bits one byte a row, then its rebuilt bitmap.
__host__ __device__ constexpr uint64_t bool_work_head(uint64_t P) {
  return (std::max<uint64_t>(4 * (P + 1), sbc::kSnappyTableBytes) + 15) & ~15ull;
}
__host__ __device__ constexpr uint64_t bool_work_bytes(uint64_t P) {
  return bool_work_head(P) + ((P + 15) & ~15ull) + (((P + 7) / 8 + 16 + 15) & ~15ull);
}

enum : int { C_NONE = 0, C_LZ4 = 1, C_ZSTD = 2, C_SNAPPY = 3, C_RLE = 10, C_DICT = 11, C_ONE = 12, C_FREQ = 13, C_BP = 14,
             C_DBP = 15, C_PATAS = 16 };
enum : uint32_t { E_OK = 0, E_SPEC = 1, E_NYI = 2, E_CAP = 6 };

struct Opts {
  int32_t dflt, has_ratio;
  double ratio;
  uint32_t forbidden;
  int32_t forced;
};

// ---------------------------------------------------------------------------
// element traits: raw bits, total-order key (Tr::key in sb_encode.cpp), as_i64
// ---------------------------------------------------------------------------
template <int W> struct UT;
template <> struct UT<1> { using U = uint8_t; };
template <> struct UT<2> { using U = uint16_t; };
template <> struct UT<4> { using U = uint32_t; };
template <> struct UT<8> { using U = uint64_t; };

template <int W>
__device__ __forceinline__ uint64_t ld(const uint8_t* p, uint32_t i) {
  return (uint64_t)((const typename UT<W>::U*)p)[i];
}

template <int W, bool FLT, bool SGN>
__device__ __forceinline__ uint64_t key_of(uint64_t b) {
  if constexpr (FLT) {
    constexpr int nb = 8 * W;
    constexpr uint64_t sign = 1ull << (nb - 1);
    constexpr uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1);
    bool nan;
    if constexpr (W == 8) nan = ((b >> 52) & 0x7FF) == 0x7FF && (b & 0xFFFFFFFFFFFFFull);
    else nan = ((b >> 23) & 0xFF) == 0xFF && (b & 0x7FFFFFull);
    if (nan) return all;  // OrderedFloat: NaN is the largest and equal to itself
    if ((b & (all >> 1)) == 0) b = 0;  // -0.0 == 0.0
    return (b & sign) ? (~b & all) : (b | sign);
  } else if constexpr (SGN) {
    const int64_t s = W == 1 ? (int64_t)(int8_t)b : W == 2 ? (int64_t)(int16_t)b : W == 4 ? (int64_t)(int32_t)b : (int64_t)b;
    return (uint64_t)s ^ 0x8000000000000000ull;
  } else {
    return b;
  }
}
// IntegerType::as_i64 of the value with this key (floats: unused, 0)
template <int W, bool FLT, bool SGN>
__device__ __forceinline__ int64_t key_as_i64(uint64_t k) {
  if constexpr (FLT) return 0;
  else if constexpr (SGN) return (int64_t)(k ^ 0x8000000000000000ull);
  else return (int64_t)k;
}

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  k *= 0xC4CEB9FE1A85EC53ull;
  k ^= k >> 33;
  return k;
}

// ---------------------------------------------------------------------------
// array view: n elements of W bytes + optional LSB validity bitmap
// ---------------------------------------------------------------------------
struct Av {
  const uint8_t* p;
  const uint8_t* vb;  // nullptr = all valid
  uint64_t vbit;      // bit of row 0 in vb
  uint32_t n;
};
__device__ __forceinline__ bool valid_at(const Av& a, uint32_t i) {
  if (!a.vb) return true;
  const uint64_t b = a.vbit + i;
  return (a.vb[b >> 3] >> (b & 7)) & 1;
}

// ---------------------------------------------------------------------------
// per-workgroup state
// ---------------------------------------------------------------------------
struct Sh {
  uint64_t red[NW];
  uint32_t redu[NW];
  uint64_t rng;
  uint32_t win[SC];
  uint32_t err;
  // stats of the current stream
  uint32_t nulls, unique, top_count, top_row;
  uint32_t sorted;
  uint64_t kmin, kmax;
  uint32_t first_valid;
  uint32_t pfail;  // Patas: an f32 value equal to its reference
};

struct Ctx {
  bool wide;        // pages over 65535 rows: 64-bit table words (count << 32 | row + 1), multi-container roaring
  uint32_t* work;   // work area: hash tables, run starts, bitmaps, the Snappy table (LDS, or HBM for big pages)
  uint8_t* lz4;     // LDS: the wave LZ4 compressor's tables (sbc::kLz4WaveLds bytes)
  uint32_t work_bytes;
  uint8_t* samp;    // LDS: kSample * 8 value bytes + kSample / 8 validity bytes
  uint8_t* scratch; // global: 2 levels x nmax x 8 bytes
  uint32_t nmax;
  uint8_t* out;     // global: the page slot
  uint32_t cap;
  Opts o;
};

__device__ __forceinline__ void set_err(Sh& sh, uint32_t e) { atomicMax(&sh.err, e); }

// choose_compressor needs the statistics only with a ratio or an allowed forced codec
__host__ __device__ __forceinline__ bool needs_stats(const Opts& o, uint32_t fm) {
  return o.has_ratio || (o.forced >= 0 && !(fm & (1u << o.forced)));
}

__device__ __forceinline__ uint64_t rng_next(uint64_t& s) {  // splitmix64 (sb_encode.cpp Rng)
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------
// block primitives (all NT threads call them)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_max(uint64_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v = max(v, (uint64_t)__shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v = min(v, (uint64_t)__shfl_xor(v, d, 64));
  return v;
}
__device__ uint64_t bsum(Sh& sh, uint64_t v) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh.red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) t += sh.red[k];
  __syncthreads();
  return t;
}
__device__ uint64_t bmax(Sh& sh, uint64_t v) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh.red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) t = max(t, sh.red[k]);
  __syncthreads();
  return t;
}
__device__ uint64_t bmin(Sh& sh, uint64_t v) {
  v = wave_min(v);
  if ((threadIdx.x & 63) == 0) sh.red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = ~0ull;
#pragma unroll
  for (int k = 0; k < NW; k++) t = min(t, sh.red[k]);
  __syncthreads();
  return t;
}
// exclusive prefix sum over threads; *tot = block total
__device__ uint32_t bscan(Sh& sh, uint32_t v, uint32_t* tot) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) sh.redu[wv] = x;
  __syncthreads();
  uint32_t pre = 0, t = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) {
    pre += (uint32_t)k < wv ? sh.redu[k] : 0u;
    t += sh.redu[k];
  }
  __syncthreads();
  *tot = t;
  return pre + x - v;
}
// exclusive prefix max over threads (0 for thread 0); *tot = block max
__device__ uint32_t bexcl_max(Sh& sh, uint32_t v, uint32_t* tot) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x = max(x, y);
  }
  if (lane == 63) sh.redu[wv] = x;
  __syncthreads();
  uint32_t pre = 0, t = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) {
    if ((uint32_t)k < wv) pre = max(pre, sh.redu[k]);
    t = max(t, sh.redu[k]);
  }
  __syncthreads();
  const uint32_t xl = __shfl_up(x, 1, 64);
  *tot = t;
  return max(pre, lane ? xl : 0u);
}

__device__ __forceinline__ void put8(uint8_t* o, uint64_t v, uint32_t nb) {
  for (uint32_t j = 0; j < nb; j++) o[j] = (uint8_t)(v >> (8 * j));
}
__device__ __forceinline__ bool room(const Ctx& c, Sh& sh, uint64_t end) {
  if (end > c.cap) {
    set_err(sh, E_CAP);
    return false;
  }
  return true;
}

// ---------------------------------------------------------------------------
// Open-addressing hash table, S slots (pow2): word = count << 16 | (first row
// + 1) in LDS, or for pages over 65535 rows (HBM) count << 32 | (row + 1);
// after the ids are assigned, count is replaced by the id.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t tab_slots(uint32_t n) {
  uint32_t s = 64;
  while (s < 2 * n) s <<= 1;
  return s;
}
struct Tab {
  uint32_t* w;
  bool wide;
  __device__ __forceinline__ uint64_t* w64() const { return (uint64_t*)w; }
  __device__ __forceinline__ uint32_t row1(uint32_t h) const {  // first row + 1, 0 = empty
    return wide ? (uint32_t)w64()[h] : (w[h] & 0xFFFFu);
  }
  __device__ __forceinline__ uint32_t hi(uint32_t h) const {  // count, or the id after set()
    return wide ? (uint32_t)(w64()[h] >> 32) : (w[h] >> 16);
  }
  __device__ __forceinline__ void set(uint32_t h, uint32_t hi_v, uint32_t row1_v) const {
    if (wide) w64()[h] = ((uint64_t)hi_v << 32) | row1_v;
    else w[h] = (hi_v << 16) | row1_v;
  }
  __device__ void clear(uint32_t S) const {
    for (uint32_t i = threadIdx.x; i < S; i += blockDim.x) {
      if (wide) w64()[i] = 0;
      else w[i] = 0;
    }
  }
};
template <class Same>
__device__ __forceinline__ uint32_t tab_insert_h(const Tab& t, uint32_t S, uint32_t r, uint64_t hv, Same same) {
  uint32_t h = (uint32_t)(hv >> 32) & (S - 1);
  if (t.wide) {
    uint64_t* tab = t.w64();
    for (;;) {
      uint64_t e = tab[h];
      if (e == 0) {
        const uint64_t prev = atomicCAS((unsigned long long*)&tab[h], 0ull, (1ull << 32) | (r + 1));
        if (prev == 0) return h;
        e = prev;
      }
      const uint32_t o = (uint32_t)e - 1;
      if (same(o)) {
        uint64_t old = atomicAdd((unsigned long long*)&tab[h], 1ull << 32) + (1ull << 32);
        while ((uint32_t)old > r + 1) {  // keep the smallest row
          const uint64_t prev = atomicCAS((unsigned long long*)&tab[h], old, (old & ~0xFFFFFFFFull) | (r + 1));
          if (prev == old) break;
          old = prev;
        }
        return h;
      }
      h = (h + 1) & (S - 1);
    }
  }
  uint32_t* tab = t.w;
  for (;;) {
    uint32_t e = tab[h];
    if (e == 0) {
      const uint32_t prev = atomicCAS(&tab[h], 0u, (1u << 16) | (r + 1));
      if (prev == 0) return h;
      e = prev;
    }
    const uint32_t o = (e & 0xFFFFu) - 1;
    if (same(o)) {
      uint32_t old = atomicAdd(&tab[h], 1u << 16) + (1u << 16);
      while ((old & 0xFFFFu) > r + 1) {  // keep the smallest row
        const uint32_t prev = atomicCAS(&tab[h], old, (old & 0xFFFF0000u) | (r + 1));
        if (prev == old) break;
        old = prev;
      }
      return h;
    }
    h = (h + 1) & (S - 1);
  }
}
template <class KeyF>
__device__ __forceinline__ uint32_t tab_insert(const Tab& t, uint32_t S, uint32_t r, uint64_t k, KeyF key) {
  return tab_insert_h(t, S, r, mix64(k), [&](uint32_t o) { return key(o) == k; });
}

// ---------------------------------------------------------------------------
// gen_stats (integer/mod.rs:179-229, double/mod.rs:178-229)
// ---------------------------------------------------------------------------
template <int W, bool FLT, bool SGN>
__device__ void gen_stats(Ctx& c, Sh& sh, const Av& a) {
  const uint32_t tid = threadIdx.x, n = a.n;
  // sortedness over valid rows against the previous valid value (T::default()
  // before the first), min / max over every slot, null count: thread chunks
  const uint32_t ch = (n + NT - 1) / NT;
  const uint32_t r0 = min(n, tid * ch), r1 = min(n, r0 + ch);
  uint32_t nulls = 0, lastv = 0, firstv = 0;  // rows + 1 (0 = none)
  bool sorted = true;
  uint64_t kmin = ~0ull, kmax = 0, prevk = 0;
  bool have = false;
  for (uint32_t r = r0; r < r1; r++) {
    const uint64_t k = key_of<W, FLT, SGN>(ld<W>(a.p, r));
    kmin = min(kmin, k);
    kmax = max(kmax, k);
    if (valid_at(a, r)) {
      if (have && k < prevk) sorted = false;
      if (!firstv) firstv = r + 1;
      prevk = k;
      have = true;
      lastv = r + 1;
    } else {
      nulls++;
    }
  }
  uint32_t tot;
  const uint32_t prev_row = bexcl_max(sh, lastv, &tot);  // last valid row (+1) before this chunk
  if (firstv) {
    const uint64_t pk = prev_row ? key_of<W, FLT, SGN>(ld<W>(a.p, prev_row - 1)) : key_of<W, FLT, SGN>(0);
    const uint64_t fk = key_of<W, FLT, SGN>(ld<W>(a.p, firstv - 1));
    if (fk < pk) sorted = false;
  }
  const uint64_t s_nulls = bsum(sh, nulls);
  const uint64_t s_unsorted = bsum(sh, sorted ? 0u : 1u);
  const uint64_t s_kmin = bmin(sh, kmin), s_kmax = bmax(sh, kmax);
  const uint64_t s_first = bmin(sh, firstv ? firstv : 0xFFFFFFFFu);
  // distinct values over every slot (nulls included)
  const uint32_t S = tab_slots(n);
  const Tab tab{c.work, c.wide};
  tab.clear(S);
  __syncthreads();
  auto key = [&](uint32_t r) { return key_of<W, FLT, SGN>(ld<W>(a.p, r)); };
  for (uint32_t r = tid; r < n; r += NT) tab_insert(tab, S, r, key(r), key);
  __syncthreads();
  uint32_t uniq = 0;
  uint64_t best = 0;
  for (uint32_t i = tid; i < S; i += NT) {
    const uint32_t r1 = tab.row1(i);
    if (r1) {
      uniq++;
      best = max(best, ((uint64_t)tab.hi(i) << 32) | (0xFFFFFFFFu - (r1 - 1)));
    }
  }
  const uint64_t s_uniq = bsum(sh, uniq);
  const uint64_t s_best = bmax(sh, best);
  if (tid == 0) {
    sh.nulls = (uint32_t)s_nulls;
    sh.sorted = s_unsorted == 0;
    sh.kmin = n ? s_kmin : key_of<W, FLT, SGN>(0);
    sh.kmax = n ? s_kmax : key_of<W, FLT, SGN>(0);
    sh.unique = (uint32_t)s_uniq;
    sh.top_count = (uint32_t)(s_best >> 32);
    sh.top_row = 0xFFFFFFFFu - (uint32_t)s_best;
    sh.first_valid = (uint32_t)s_first;  // row + 1, or ~0u when every row is null
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// size-only and writing codec bodies
// ---------------------------------------------------------------------------
// RLE (rle.rs:64-104): runs start at row 0 and at every valid row whose key
// differs from the previous valid row's; nulls extend the current run.
// WRITE: run records at c.out + pos.  Returns the body size.
template <int W, bool FLT, bool SGN, bool WRITE>
__device__ uint32_t rle_body(Ctx& c, Sh& sh, const Av& a, uint32_t pos) {
  const uint32_t tid = threadIdx.x, n = a.n;
  if (n == 0) return 0;
  uint32_t carry_last = 0, carry_runs = 0;  // last valid row + 1 so far, runs so far
  uint32_t* rs = c.work;                    // run starts (WRITE)
  for (uint32_t t0 = 0; t0 < n; t0 += NT) {
    const uint32_t r = t0 + tid;
    const bool in = r < n;
    const bool v = in && valid_at(a, r);
    uint32_t tmax;
    uint32_t prev = bexcl_max(sh, v ? r + 1 : 0u, &tmax);  // previous valid row (+1) in the tile
    prev = max(prev, carry_last);
    bool start = in && r == 0;
    if (v && prev) {
      const uint64_t k = key_of<W, FLT, SGN>(ld<W>(a.p, r));
      const uint64_t pk = key_of<W, FLT, SGN>(ld<W>(a.p, prev - 1));
      start = k != pk;
    }
    uint32_t tot;
    const uint32_t ex = bscan(sh, start ? 1u : 0u, &tot);
    if (WRITE && start) rs[carry_runs + ex] = r;
    carry_runs += tot;
    carry_last = max(carry_last, tmax);
  }
  const uint32_t R = carry_runs;
  const uint32_t rec = 4 + W;
  if (WRITE) {
    if (!room(c, sh, (uint64_t)pos + (uint64_t)R * rec)) return 0;
    if (tid == 0) rs[R] = n;
    __syncthreads();
    const uint32_t fv = sh.first_valid;
    for (uint32_t j = tid; j < R; j += NT) {
      const uint32_t s = rs[j], e = rs[j + 1];
      uint64_t val;
      if (j == 0) val = fv != 0xFFFFFFFFu ? ld<W>(a.p, fv - 1) : 0;
      else val = ld<W>(a.p, s);
      uint8_t* o = c.out + pos + (uint64_t)j * rec;
      put8(o, e - s, 4);
      put8(o + 4, val, W);
    }
    __syncthreads();
  }
  return R * rec;
}

// first valid row (+1, ~0u if none) of an array (for views whose stats are not current)
__device__ uint32_t first_valid_row(Sh& sh, const Av& a) {
  uint32_t f = 0xFFFFFFFFu;
  for (uint32_t r = threadIdx.x; r < a.n; r += NT)
    if (valid_at(a, r)) {
      f = r + 1;
      break;
    }
  return (uint32_t)bmin(sh, f);
}

// BitPacker4x (bitpacking 0.8.0): value 4i + l of a block at bit i*b of lane
// l's stream, lane word k at byte 16k + 4l; b = bits of the OR of the raw
// values (also for the delta variant, delta_bp.rs:50).
__device__ __forceinline__ uint32_t bp_val(const uint8_t* p, uint32_t base, uint32_t j, bool delta) {
  const uint32_t x = (uint32_t)ld<4>(p, base + j);
  if (!delta) return x;
  const uint32_t prev = (base + j) ? (uint32_t)ld<4>(p, base + j - 1) : 0u;
  return x - prev;
}
template <bool WRITE>
__device__ uint32_t bp_body(Ctx& c, Sh& sh, const Av& a, uint32_t pos, bool delta) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nblk = a.n / 128;
  uint32_t* bw = c.work;                             // [nblk] widths
  uint32_t* boff = c.work + ((nblk + 255) & ~255u);  // [nblk] block offsets
  for (uint32_t k = wv; k < nblk; k += NW) {
    uint32_t acc = (uint32_t)ld<4>(a.p, 128 * k + lane) | (uint32_t)ld<4>(a.p, 128 * k + 64 + lane);
#pragma unroll
    for (int d = 32; d; d >>= 1) acc |= __shfl_xor(acc, d, 64);
    if (lane == 0) bw[k] = acc ? 32 - __builtin_clz(acc) : 0;
  }
  __syncthreads();
  uint32_t tot = 0;
  for (uint32_t k0 = 0; k0 < nblk; k0 += NT) {  // (one tile of blocks per 32768 rows)
    const uint32_t k = k0 + tid;
    uint32_t t;
    const uint32_t ex = bscan(sh, k < nblk ? 1 + 16 * bw[k] : 0u, &t);
    if (WRITE && k < nblk) boff[k] = tot + ex;
    tot += t;
  }
  if (!WRITE) return tot;
  if (!room(c, sh, (uint64_t)pos + tot)) return 0;
  __syncthreads();
  for (uint32_t s = tid; s < nblk * 128; s += NT) {
    const uint32_t k = s >> 7, w = s & 127, b = bw[k];
    uint8_t* o = c.out + pos + boff[k];
    if (w == 0) o[0] = (uint8_t)b;
    if (w < 4 * b) {
      const uint32_t kk = w >> 2, l = w & 3;
      const uint64_t mask = b == 32 ? 0xFFFFFFFFull : ((1ull << b) - 1);
      const uint32_t i0 = (32 * kk) / b, i1 = min(31u, (32 * kk + 31) / b);
      uint32_t word = 0;
      for (uint32_t i = i0; i <= i1; i++) {
        const uint64_t v = bp_val(a.p, 128 * k, 4 * i + l, delta) & mask;
        const int32_t sft = (int32_t)(i * b) - (int32_t)(32 * kk);
        word |= sft >= 0 ? (uint32_t)(v << sft) : (uint32_t)(v >> -sft);
      }
      put8(o + 1 + 4 * w, word, 4);
    }
  }
  __syncthreads();
  return tot;
}

// Patas (double/patas.rs:37-105): reference = the nearest earlier equal value
// within 127 rows, else row i-1 (row 0 while i < 128 and no earlier equal).
// Returns the body size, or ~0u when an f32 value equals its reference (the
// reference writes a page its decoder misreads; the caller falls back).
template <int W, bool WRITE>
__device__ uint32_t patas_body(Ctx& c, Sh& sh, const Av& a, uint32_t pos) {
  const uint32_t tid = threadIdx.x, n = a.n;
  constexpr uint32_t nb = 8 * W;
  if (tid == 0) sh.pfail = 0;
  __syncthreads();
  uint32_t carry = W;
  for (uint32_t t0 = 0; t0 < n; t0 += NT) {
    const uint32_t i = t0 + tid;
    uint32_t sz = 0, packed = 0;
    uint64_t xs = 0;
    if (i < n && i > 0) {
      const uint64_t v = ld<W>(a.p, i);
      uint32_t ref = i < 128 ? 0u : i - 1;
      const uint32_t lo = i >= 127 ? i - 127 : 0u;
      for (uint32_t j = i; j-- > lo;)
        if (ld<W>(a.p, j) == v) {
          ref = j;
          break;
        }
      const uint32_t diff = i - ref;
      const uint64_t x = v ^ ld<W>(a.p, ref);
      uint32_t tz, lz;
      if (x == 0) {
        tz = nb;
        lz = nb;
      } else {
        tz = (uint32_t)__builtin_ctzll(x);
        lz = (uint32_t)__builtin_clzll(x) - (64 - nb);
      }
      const uint32_t eq = tz == nb;
      if (eq && nb == 32) sh.pfail = 1;
      const uint32_t sig = eq ? 0 : nb - tz - lz;
      const uint32_t sb = (sig >> 3) + ((sig & 7) != 0);
      const uint32_t sft = tz - eq;
      packed = ((diff & 0xFF) << 9) | ((sb & 7) << 6) | (sft & 0xFF);
      xs = sft >= 64 ? 0 : x >> sft;
      sz = 2 + sb;
    }
    uint32_t tot;
    const uint32_t ex = bscan(sh, sz, &tot);
    if (WRITE && sz) {
      if ((uint64_t)pos + carry + ex + sz <= c.cap) {
        uint8_t* o = c.out + pos + carry + ex;
        put8(o, packed, 2);
        put8(o + 2, xs, sz - 2);
      } else {
        set_err(sh, E_CAP);
      }
    }
    carry += tot;
  }
  __syncthreads();
  if (sh.pfail) return ~0u;
  if (WRITE && tid == 0 && n) {
    if ((uint64_t)pos + W <= c.cap) put8(c.out + pos, ld<W>(a.p, 0), W);
  }
  __syncthreads();
  return n ? carry : 0u;
}

// the 640-row sample of compress_sample_ratio (integer/mod.rs:310-347) in LDS
template <int W>
__device__ Av take_sample(Ctx& c, Sh& sh, const Av& a) {
  const uint32_t tid = threadIdx.x;
  if (tid == 0) {
    const uint32_t sep = a.n / SC, rem = a.n % SC;
    for (uint32_t k = 0; k < SC; k++) {
      const uint32_t range_end = (k == SC - 1 ? sep + rem : sep) - SS;
      sh.win[k] = k * sep + (uint32_t)(rng_next(sh.rng) % range_end);
    }
  }
  uint8_t* vb = c.samp + kSample * 8;
  for (uint32_t i = tid; i < kSample / 8; i += NT) vb[i] = 0;
  __syncthreads();
  // The reference rebuilds the sample through MutablePrimitiveArray::
  // extend_trusted_len (integer/mod.rs:334-336, double/mod.rs:334-336),
  // which writes T::default() under every null slot: the trial encoders then
  // see zeros there, not the slot's original bits.
  for (uint32_t q = tid; q < kSample; q += NT) {
    const uint32_t src = sh.win[q / SS] + q % SS;
    const bool ok = !a.vb || valid_at(a, src);
    const uint64_t v = ok ? ld<W>(a.p, src) : 0;
    if constexpr (W == 8) ((uint64_t*)c.samp)[q] = v;
    else if constexpr (W == 4) ((uint32_t*)c.samp)[q] = (uint32_t)v;
    else if constexpr (W == 2) ((uint16_t*)c.samp)[q] = (uint16_t)v;
    else c.samp[q] = (uint8_t)v;
    if (a.vb && ok) atomicOr((uint32_t*)vb + (q >> 5), 1u << (q & 31));
  }
  __syncthreads();
  return Av{c.samp, a.vb ? vb : nullptr, 0, kSample};
}

// compress_sample_ratio for RLE / Bitpacking / Patas
template <int W, bool FLT, bool SGN>
__device__ double sample_ratio(Ctx& c, Sh& sh, const Av& a, int codec) {
  Av s = a;
  if (a.n / SC > SS) s = take_sample<W>(c, sh, a);
  const uint64_t total = (uint64_t)s.n * W;
  uint64_t sz;
  if (codec == C_RLE) {
    sz = rle_body<W, FLT, SGN, false>(c, sh, s, 0);
  } else if (codec == C_BP) {
    if constexpr (W == 4 && !FLT) sz = bp_body<false>(c, sh, s, 0, false);
    else sz = total;
  } else {
    const uint32_t r = patas_body<W, false>(c, sh, s, 0);
    sz = r == ~0u ? total : r;
  }
  return (double)total / (double)sz;
}

__device__ __forceinline__ uint32_t bits_needed(uint64_t x) { return x ? 64 - (uint32_t)__clzll(x) : 0; }

// choose_compressor (integer/mod.rs:231-308; double/mod.rs:231-307)
template <int W, bool FLT, bool SGN>
__device__ int choose(Ctx& c, Sh& sh, const Av& a, uint32_t fm) {
  const Opts& o = c.o;
  const uint32_t n = a.n;
  const bool bp_ok = !FLT && W == 4 && key_as_i64<W, FLT, SGN>(sh.kmin) >= 0 && n % 128 == 0;
  if (o.forced >= 0 && !(fm & (1u << o.forced))) {
    const int f = o.forced;
    const bool ok = FLT ? (f == C_FREQ || f == C_DICT || f == C_RLE || f == C_PATAS)
                        : (f == C_FREQ || f == C_DICT || f == C_RLE || (f == C_BP && bp_ok));
    if (ok) return f;
  }
  int result = o.dflt;
  if (!o.has_ratio) return result;
  double maxr = o.ratio;
  const int ic[6] = {C_ONE, C_FREQ, C_DICT, C_RLE, C_BP, C_DBP};
  const int dc[5] = {C_ONE, C_FREQ, C_DICT, C_PATAS, C_RLE};
  const int nc = FLT ? 5 : 6;
  const uint32_t uniq = sh.unique, nulls = sh.nulls;
  for (int k = 0; k < nc; k++) {
    const int cd = FLT ? dc[k] : ic[k];
    if (fm & (1u << cd)) continue;
    double r = 0.0;
    switch (cd) {
      case C_ONE: r = uniq <= 1 ? (double)n : 0.0; break;
      case C_FREQ:  // freq.rs:129-151
        if (uniq > 1) {
          if ((double)nulls / (double)n >= 0.9) r = (double)(n - 1);
          else if ((double)sh.top_count / (double)n >= 0.9 && (FLT || key_as_i64<W, FLT, SGN>(sh.kmax) >= 256))
            r = (double)(n - 1);
        }
        break;
      case C_DICT:  // dict.rs:105-120 (integer division in bits / 8 and 2n / 128)
        if ((uint64_t)uniq * 3 < n) {
          uint64_t after = (uint64_t)uniq * W + (uint64_t)n * (bits_needed(uniq) / 8);
          after += (uint64_t)n * 2 / 128;
          r = (double)((uint64_t)n * W) / (double)after;
        }
        break;
      case C_RLE:
      case C_PATAS: r = sample_ratio<W, FLT, SGN>(c, sh, a, cd); break;
      case C_BP: r = bp_ok ? sample_ratio<W, FLT, SGN>(c, sh, a, C_BP) : 0.0; break;
      case C_DBP:  // delta_bp.rs:97-110
        r = (bp_ok && sh.sorted && nulls == 0) ? sample_ratio<W, FLT, SGN>(c, sh, a, C_BP) * 1.5 : 0.0;
        break;
    }
    if (r > maxr) {
      maxr = r;
      result = cd;
      if (r == (double)n) break;
    }
  }
  return result;
}

// A Zstd frame of src[0, len) at `frame`, one wave: each 128 KiB chunk is
// parsed by the wave LZ4 compressor into `tmp` (the slot past the frame's
// bound), then lane 0 transcodes the parse into the chunk's blocks (sequence
// records in the LZ4 tables' LDS).  Only the ZS kernels hold it: with it
// (inlined, or out of line) the encode kernels grew from 152 to 184-248
// VGPRs (one or two waves a SIMD instead of three).  Returns the frame size.
__device__ __forceinline__ uint32_t zstd_frame_wave(const uint8_t* src, uint32_t len, uint8_t* frame, uint8_t* tmp,
                                                 sbc::lz4_lds8* tab) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t op = 0;
  if (len == 0 && lane == 0) op = sbz::zstd_empty(frame);
  if (len && lane == 0) op = sbz::zstd_frame_header(frame, len);
  sbz::ZRep rep{{1, 4, 8}};  // (lane 0's)
  for (uint32_t off = 0; off < len; off += sbz::kZChunk) {
    const uint32_t cl = min(len - off, sbz::kZChunk);
    for (uint32_t i = lane; i < 4096; i += 64) ((uint32_t*)tab)[i] = 0;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's table stores land before its loads
    __builtin_amdgcn_wave_barrier();
    const uint32_t r = sbc::lz4_compress_wave(sbc::Lz4GSrc{src + off}, cl, tmp, tab);
    __threadfence();  // the parse's stores, visible to lane 0
    if (lane == 0) op += sbz::zstd_transcode(tmp, r, src + off, cl, frame + op, (uint64_t*)tab, off + cl == len, rep);
    __threadfence();
    __builtin_amdgcn_wave_barrier();
  }
  return op;
}

// Basic codecs: the raw bytes of the values, None / LZ4 / Snappy / Zstd
// ZS: the kernel instantiation for a Zstd default codec (only those carry the
// frame writer: the others keep their register budget).
template <bool ZS>
__device__ uint32_t basic_body(Ctx& c, Sh& sh, int codec, const uint8_t* src, uint32_t len, uint32_t pos) {
  const uint32_t tid = threadIdx.x;
  if (codec == C_NONE) {
    if (!room(c, sh, (uint64_t)pos + len)) return 0;
    for (uint32_t j = tid; j < len; j += NT) c.out[pos + j] = src[j];
    __syncthreads();
    return len;
  }
  if (codec == C_LZ4 || codec == C_SNAPPY) {
    const uint64_t bound = codec == C_LZ4 ? sbc::lz4_bound(len) : (uint64_t)len + len / 20 + 32;
    if (!room(c, sh, (uint64_t)pos + bound)) return 0;
    if (codec == C_LZ4)  // the position table (16 KiB)
      for (uint32_t i = tid; i < 4096; i += NT) ((uint32_t*)c.lz4)[i] = 0;
    __syncthreads();
#ifdef SB_LZ4_SERIAL  // A/B: the one-lane compressor
    if (codec == C_LZ4 && tid == 0) {
      sh.redu[0] = sbc::lz4_compress(src, len, c.out + pos, c.lz4);
    }
#else
    if (codec == C_LZ4 && tid < 64) {
      const uint32_t r = sbc::lz4_compress_wave(sbc::Lz4GSrc{src}, len, c.out + pos, (sbc::lz4_lds8*)c.lz4);  // (c.lz4 is LDS)
      if (tid == 0) sh.redu[0] = r;
    }
#endif
    if (codec == C_SNAPPY && tid == 0) {
      sh.redu[0] = sbc::snappy_compress(src, len, c.out + pos, c.work);
    }
    __syncthreads();
    const uint32_t r = sh.redu[0];
    __syncthreads();
    return r;
  }
  if constexpr (!ZS) {
    if (tid == 0) set_err(sh, E_NYI);  // (never: Zstd pages run the ZS instantiation)
    __syncthreads();
    return 0;
  } else {
    // Zstd (sb_zstdc.h): wave 0 writes the frame (zstd_frame_wave)
    const uint32_t cl0 = min(len, sbz::kZChunk);
    const uint64_t zb = sbz::zstd_bound(len);
    if (!room(c, sh, (uint64_t)pos + zb + sbc::lz4_bound(cl0) + 16)) return 0;
    if (tid < 64) {
      const uint32_t r = zstd_frame_wave(src, len, c.out + pos, c.out + pos + zb, (sbc::lz4_lds8*)c.lz4);
      if (tid == 0) sh.redu[0] = r;
    }
    __syncthreads();
    const uint32_t r = sh.redu[0];
    __syncthreads();
    return r;
  }
}

__device__ __forceinline__ void write_hdr(Ctx& c, uint32_t pos, int codec, uint32_t csize, uint32_t usize) {
  if (threadIdx.x == 0) {
    c.out[pos] = (uint8_t)codec;
    put8(c.out + pos + 1, csize, 4);
    put8(c.out + pos + 5, usize, 4);
  }
}

// ---------------------------------------------------------------------------
// compress_integer / compress_double: [codec u8][csize u32][usize u32][body]
// at c.out + pos; returns the position after it.  D = cascade depth.
// ---------------------------------------------------------------------------
template <int W, bool FLT, bool SGN, int D, bool ZS>
__device__ uint32_t enc_stream(Ctx& c, Sh& sh, const Av& a, uint32_t fm, uint32_t pos);

// Dict (dict.rs:34-73): ids by first occurrence over valid rows (a null row
// repeats the previous row's id; a null row 0 is T::default()), the u32
// index stream cascades with Dict forbidden, then u32 k + k raw values.
template <int W, bool FLT, bool SGN, int D, bool ZS>
__device__ uint32_t dict_body(Ctx& c, Sh& sh, const Av& a, uint32_t fm, uint32_t pos) {
  const uint32_t tid = threadIdx.x, n = a.n;
  uint32_t* idx = (uint32_t*)(c.scratch + (uint64_t)D * c.nmax * 8);
  uint32_t* row_of = idx + c.nmax;
  const bool v0 = n && valid_at(a, 0);
  auto dv = [&](uint32_t r) -> uint64_t { return (r == 0 && !v0) ? 0ull : ld<W>(a.p, r); };
  auto ins = [&](uint32_t r) { return r == 0 || valid_at(a, r); };
  const uint32_t S = tab_slots(n);
  const Tab tab{c.work, c.wide};
  tab.clear(S);
  __syncthreads();
  for (uint32_t r = tid; r < n; r += NT)
    if (ins(r)) idx[r] = tab_insert(tab, S, r, dv(r), dv);  // the slot, for now
  __syncthreads();
  // ids: first rows in row order -- one block scan over thread chunks of
  // consecutive rows (a scan per 256 rows cost 32 barriers pairs a page)
  const uint32_t ch = (n + NT - 1) / NT, c0 = min(n, tid * ch), c1 = min(n, c0 + ch);
  auto first = [&](uint32_t r) { return ins(r) && tab.row1(idx[r]) == r + 1; };
  uint32_t nf = 0;
  for (uint32_t r = c0; r < c1; r++) nf += first(r) ? 1u : 0u;
  uint32_t k;
  uint32_t wpos = bscan(sh, nf, &k);
  for (uint32_t r = c0; r < c1; r++)
    if (first(r)) row_of[wpos++] = r;
  __syncthreads();
  for (uint32_t j = tid; j < k; j += NT) {
    const uint32_t r = row_of[j];
    const uint32_t slot = idx[r];
    tab.set(slot, j, r + 1);
  }
  __syncthreads();
  for (uint32_t r = tid; r < n; r += NT)
    if (ins(r)) idx[r] = tab.hi(idx[r]);
  __syncthreads();
  // null rows take the id of the last inserted row before them
  // (same chunks; row 0 is always inserted)
  uint32_t lastc = 0;
  for (uint32_t r = c0; r < c1; r++)
    if (ins(r)) lastc = r + 1;
  uint32_t tmax;
  uint32_t last = bexcl_max(sh, lastc, &tmax);
  for (uint32_t r = c0; r < c1; r++) {
    if (ins(r)) last = r + 1;
    else idx[r] = idx[last - 1];
  }
  __syncthreads();
  const Av ia{(const uint8_t*)idx, nullptr, 0, n};
  const uint32_t p2 = enc_stream<4, false, false, D + 1, ZS>(c, sh, ia, fm | (1u << C_DICT), pos);
  if (sh.err) return pos;
  if (!room(c, sh, (uint64_t)p2 + 4 + (uint64_t)k * W)) return pos;
  if (tid == 0) put8(c.out + p2, k, 4);
  for (uint32_t j = tid; j < k; j += NT) put8(c.out + p2 + 4 + j * W, dv(row_of[j]), W);
  __syncthreads();
  return p2 + 4 + k * W;
}

// roaring 0.10.1 serialize_into (sb_encode.cpp roaring_serialize) of e
// ascending rows (rows[j] < n) for pages over 65536 rows: cookie 12346, the
// containers' (key, card - 1), their offsets, then array (<= 4096) or bitmap
// containers (bitmaps from bm, the rows' n-bit bitmap).  tmp: 4 ceil(n /
// 65536) words of scratch.  All NT threads.  Returns the bytes written at
// c.out + rpos (0 when out of room).
__device__ uint32_t roaring_multi(Ctx& c, Sh& sh, const uint32_t* bm, const uint32_t* rows, uint32_t e, uint32_t n,
                                  uint32_t rpos, uint32_t* tmp) {
  const uint32_t tid = threadIdx.x, nk = (n + 65535) >> 16;
  uint32_t* first = tmp;
  uint32_t* card = tmp + nk;
  uint32_t* doff = tmp + 2 * nk;  // data offset of each present container; tmp[3 nk + k]: its index
  auto lower = [&](uint32_t x) {  // first j with rows[j] >= x
    uint32_t lo = 0, hi = e;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (rows[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  for (uint32_t k = tid; k < nk; k += NT) {
    const uint32_t a = lower(k << 16), b = k + 1 < nk ? lower((k + 1) << 16) : e;
    first[k] = a;
    card[k] = b - a;
  }
  __syncthreads();
  uint32_t nc = 0, dsz = 0;  // present containers and data bytes before the tile
  for (uint32_t k0 = 0; k0 < nk; k0 += NT) {
    const uint32_t k = k0 + tid;
    const uint32_t cd = k < nk ? card[k] : 0u;
    const uint32_t sz = cd == 0 ? 0u : cd <= 4096 ? 2 * cd : 8192u;
    uint32_t tc, ts;
    const uint32_t ic = bscan(sh, cd ? 1u : 0u, &tc), is = bscan(sh, sz, &ts);
    if (k < nk) doff[k] = cd ? dsz + is : 0u;
    if (k < nk && cd) tmp[3 * nk + k] = nc + ic;  // compact index
    nc += tc;
    dsz += ts;
  }
  __syncthreads();
  const uint32_t hdr = 8 + 8 * nc, total = hdr + dsz;
  if (!room(c, sh, (uint64_t)rpos + total)) return 0;
  if (tid == 0) {
    put8(c.out + rpos, 12346, 4);  // SERIAL_COOKIE_NO_RUNCONTAINER
    put8(c.out + rpos + 4, nc, 4);
  }
  for (uint32_t k = tid; k < nk; k += NT) {
    const uint32_t cd = card[k];
    if (!cd) continue;
    const uint32_t i = tmp[3 * nk + k];
    put8(c.out + rpos + 8 + 4 * i, k, 2);
    put8(c.out + rpos + 10 + 4 * i, cd - 1, 2);
    put8(c.out + rpos + 8 + 4 * nc + 4 * i, hdr + doff[k], 4);
  }
  for (uint32_t j = tid; j < e; j += NT) {  // array containers
    const uint32_t r = rows[j], k = r >> 16;
    if (card[k] <= 4096) put8(c.out + rpos + hdr + doff[k] + 2 * (j - first[k]), r & 0xFFFF, 2);
  }
  for (uint32_t k = 0; k < nk; k++) {  // bitmap containers (uniform)
    if (card[k] <= 4096) continue;
    for (uint32_t w = tid; w < 2048; w += NT) {
      const uint32_t g = k * 2048 + w;  // the container's words; none past the page's last row
      put8(c.out + rpos + hdr + doff[k] + 4 * w, g < (n + 31) / 32 ? bm[g] : 0u, 4);
    }
  }
  __syncthreads();
  return total;
}

// Freq (freq.rs:34-86): top value (the most frequent, first occurrence on
// ties; T::default() when >= 90 % nulls), roaring bitmap of the valid rows
// that differ from it, their values as a cascaded stream (Freq forbidden).
template <int W, bool FLT, bool SGN, int D, bool ZS>
__device__ uint32_t freq_body(Ctx& c, Sh& sh, const Av& a, uint32_t fm, uint32_t pos) {
  const uint32_t tid = threadIdx.x, n = a.n;
  const bool top_null = (double)sh.nulls / (double)n >= 0.9;
  const uint64_t top = top_null ? 0ull : ld<W>(a.p, sh.top_row);
  const uint64_t tk = key_of<W, FLT, SGN>(top);
  uint8_t* exc = c.scratch + (uint64_t)D * c.nmax * 8;
  uint32_t* bm = c.work;  // the exceptions' row bitmap (bitmap containers)
  const bool multi = n > 65536;  // (a wide page: several roaring containers)
  uint32_t* rows = (uint32_t*)(c.scratch + (uint64_t)2 * c.nmax * 8);
  const uint32_t bmw = multi ? (n + 31) / 32 : 2048;
  for (uint32_t i = tid; i < bmw; i += NT) bm[i] = 0;
  __syncthreads();
  // exceptions in row order; positions written as an array container after the header
  const uint32_t rpos = pos + W + 4;  // roaring start
  const uint32_t data = rpos + 16;    // container data (one container: n <= 65536)
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += NT) {
    const uint32_t r = t0 + tid;
    bool e = false;
    uint64_t v = 0;
    if (r < n && valid_at(a, r)) {
      v = ld<W>(a.p, r);
      e = top_null || key_of<W, FLT, SGN>(v) != tk;
    }
    uint32_t tot;
    const uint32_t ex = bscan(sh, e ? 1u : 0u, &tot);
    if (e) {
      const uint32_t j = carry + ex;
      if constexpr (W == 8) ((uint64_t*)exc)[j] = v;
      else if constexpr (W == 4) ((uint32_t*)exc)[j] = (uint32_t)v;
      else if constexpr (W == 2) ((uint16_t*)exc)[j] = (uint16_t)v;
      else exc[j] = (uint8_t)v;
      atomicOr(&bm[r >> 5], 1u << (r & 31));
      if (multi) rows[j] = r;
      else if ((uint64_t)data + 2ull * (j + 1) <= c.cap) put8(c.out + data + 2 * j, r & 0xFFFF, 2);
    }
    carry += tot;
  }
  const uint32_t e = carry;
  __syncthreads();
  if (multi) {
    const uint32_t bytes = roaring_multi(c, sh, bm, rows, e, n, rpos, rows + c.nmax);
    if (!bytes) return pos;
    if (tid == 0) {
      put8(c.out + pos, top, W);
      put8(c.out + pos + W, bytes, 4);
    }
    __syncthreads();
    const Av ea{exc, nullptr, 0, e};
    return enc_stream<W, FLT, SGN, D + 1, ZS>(c, sh, ea, fm | (1u << C_FREQ), rpos + bytes);
  }
  const uint32_t bytes = e == 0 ? 8u : (e <= 4096 ? 16 + 2 * e : 16 + 8192u);
  if (!room(c, sh, (uint64_t)rpos + bytes)) return pos;
  if (tid == 0) {
    put8(c.out + pos, top, W);
    put8(c.out + pos + W, bytes, 4);
    put8(c.out + rpos, 12346, 4);  // roaring 0.10.1 SERIAL_COOKIE_NO_RUNCONTAINER
    put8(c.out + rpos + 4, e ? 1u : 0u, 4);
    if (e) {
      put8(c.out + rpos + 8, 0, 2);  // container key (high 16 bits)
      put8(c.out + rpos + 10, e - 1, 2);
      put8(c.out + rpos + 12, 16, 4);  // offset of the data
    }
  }
  if (e > 4096)  // bitmap container: 1024 words
    for (uint32_t i = tid; i < 2048; i += NT) put8(c.out + data + 4 * i, bm[i], 4);
  __syncthreads();
  const Av ea{exc, nullptr, 0, e};
  return enc_stream<W, FLT, SGN, D + 1, ZS>(c, sh, ea, fm | (1u << C_FREQ), rpos + bytes);
}

#ifdef SB_ENC_PHASES  // A/B instrumentation: per workgroup, s_memrealtime at each phase of the top two streams
__device__ uint64_t sb_enc_phase[4096 * 12];
#define SB_EPHASE(k, v) do { if (D < 2 && threadIdx.x == 0 && blockIdx.x < 4096) sb_enc_phase[blockIdx.x * 12 + ((k) == 5 ? 8 + D : 4 * D + (k))] = (v); } while (0)
#else
#define SB_EPHASE(k, v) do { } while (0)
#endif

template <int W, bool FLT, bool SGN, int D, bool ZS>
__device__ uint32_t enc_stream(Ctx& c, Sh& sh, const Av& a, uint32_t fm, uint32_t pos) {
  const uint32_t tid = threadIdx.x, n = a.n;
  SB_EPHASE(0, wall_clock64());
  if (!room(c, sh, (uint64_t)pos + 9)) return pos;
  // the statistics only choose among codecs: with no ratio and no forced
  // codec the page is Basic(default) (integer/mod.rs:267-307)
  if (needs_stats(c.o, fm)) gen_stats<W, FLT, SGN>(c, sh, a);
  SB_EPHASE(1, wall_clock64());
  int codec = choose<W, FLT, SGN>(c, sh, a, fm);
  SB_EPHASE(2, wall_clock64());
  SB_EPHASE(5, (uint64_t)codec);
  const uint32_t body = pos + 9;
  uint32_t end = body;
  switch (codec) {
    case C_NONE:
    case C_LZ4:
    case C_ZSTD:
    case C_SNAPPY: end = body + basic_body<ZS>(c, sh, codec, a.p, n * W, body); break;
    case C_RLE: end = body + rle_body<W, FLT, SGN, true>(c, sh, a, body); break;
    case C_ONE: {  // one_value.rs:63-75: the first valid value, else default
      if (!room(c, sh, (uint64_t)body + W)) break;
      const uint32_t fv = sh.first_valid;
      if (tid == 0) put8(c.out + body, fv != 0xFFFFFFFFu ? ld<W>(a.p, fv - 1) : 0, W);
      __syncthreads();
      end = body + W;
      break;
    }
    case C_BP:
    case C_DBP:
      if constexpr (W == 4 && !FLT) end = body + bp_body<true>(c, sh, a, body, codec == C_DBP);
      break;
    case C_PATAS: {
      const uint32_t r = patas_body<W, true>(c, sh, a, body);
      if (r == ~0u) {  // f32 desync guard (sb_encode.cpp compress_stream): Basic instead
        codec = c.o.dflt;
        end = body + basic_body<ZS>(c, sh, codec, a.p, n * W, body);
      } else {
        end = body + r;
      }
      break;
    }
    case C_DICT:
      if constexpr (D < 2) end = dict_body<W, FLT, SGN, D, ZS>(c, sh, a, fm, body);
      else set_err(sh, E_SPEC);
      break;
    case C_FREQ:
      if constexpr (D < 2) end = freq_body<W, FLT, SGN, D, ZS>(c, sh, a, fm, body);
      else set_err(sh, E_SPEC);
      break;
    default: set_err(sh, E_SPEC);
  }
  __syncthreads();
  SB_EPHASE(3, wall_clock64());
  write_hdr(c, pos, codec, end - body, n * W);
  __syncthreads();
  return end;
}

// ---------------------------------------------------------------------------
// page kernel, scan, compaction
// ---------------------------------------------------------------------------
struct AdArgs {
  const uint8_t* values;
  const uint8_t* validity;  // column bitmap or nullptr
  uint64_t n_rows;
  uint32_t P;
  uint32_t page0;
  uint32_t n_batch;
  int nullable;
  Opts o;
  uint64_t seed;
  uint8_t* slots;
  uint64_t slot_bytes;
  uint8_t* scratch;
  uint64_t scratch_bytes;  // per page
  uint32_t work_bytes;     // LDS work area (0: big pages, whose work area is gwork)
  uint8_t* gwork;          // big pages: per batch page, gwork_bytes of HBM work area
  uint64_t gwork_bytes;
  uint64_t* sizes;         // [n_pages]
  uint32_t* status;        // [n_pages]
  uint64_t* offs;          // [n_pages + 1]: page offsets in the output; [n_pages] running total
  uint8_t* out;
  uint64_t out_cap;
  uint32_t n_pages;
  // Binary / Utf8 columns
  const int64_t* offsets;   // n_rows + 1 absolute positions into values
  uint64_t parent_len;      // the array's whole values length (stats and the Extend header)
  int ow;                   // offset width 4 / 8
  const uint64_t* slot_offs;  // per page of the batch: slot start (variable slots), [n_batch] = end
  // List values (sb_encode_list_column_device): page p holds the child values
  // [rows_at[p], rows_at[p + 1]) and starts with its level header (heads + p *
  // head_slot, head_len[p] bytes) in place of a validity prefix
  const uint64_t* rows_at = nullptr;
  const uint8_t* heads = nullptr;
  uint64_t head_slot = 0;
  const uint32_t* head_len = nullptr;
};

// Page p's rows: [p * P, min((p + 1) * P, n_rows)), or a List page's child values
__device__ __forceinline__ void page_rows(const AdArgs& A, uint32_t p, uint64_t* r0, uint32_t* n) {
  if (A.rows_at) {
    *r0 = A.rows_at[p];
    *n = (uint32_t)(A.rows_at[p + 1] - *r0);
  } else {
    *r0 = (uint64_t)p * A.P;
    *n = (uint32_t)min<uint64_t>(A.P, A.n_rows - *r0);
  }
}

// A List page's level header, copied to the page's start by the threads of
// `nt`; returns its length
__device__ __forceinline__ uint32_t put_head(const AdArgs& A, uint32_t p, uint8_t* out, uint32_t nt) {
  const uint32_t hl = (uint32_t)min<uint64_t>(A.head_len[p], A.head_slot);  // never past the header's slot
  const uint8_t* h = A.heads + (uint64_t)p * A.head_slot;
  for (uint32_t j = threadIdx.x; j < hl; j += nt) out[j] = h[j];
  return hl;
}

__device__ __forceinline__ uint8_t* slot_of(const AdArgs& A, uint32_t b) {
  return A.slot_offs ? A.slots + A.slot_offs[b] : A.slots + (uint64_t)b * A.slot_bytes;
}
__device__ __forceinline__ uint64_t slot_cap(const AdArgs& A, uint32_t b) {
  return A.slot_offs ? A.slot_offs[b + 1] - A.slot_offs[b] : A.slot_bytes;
}

__device__ __forceinline__ uint64_t page_seed(uint64_t seed, uint64_t page) {  // sb_encode.cpp page_seed
  uint64_t s = seed ^ (page * 0xD1B54A32D192ED03ull);
  return rng_next(s);
}

__device__ __forceinline__ uint32_t uleb_len(uint64_t h) {
  uint32_t l = 1;
  while (h >= 0x80) {
    h >>= 7;
    l++;
  }
  return l;
}

// write_validity (serialize.rs:200-215): u32 def_len + ULEB128 bit-packed run
// header + the page's validity bitmap; returns its length (0 when not nullable).
__device__ uint32_t write_prefix(Ctx& c, const AdArgs& A, uint64_t r0, uint32_t n) {
  if (!A.nullable) return 0;
  const uint32_t tid = threadIdx.x;
  const bool has_vb = A.validity != nullptr;
  const uint32_t nb = (n + 7) / 8;
  uint64_t h = ((uint64_t)nb << 1) | 1;
  const uint32_t hl = uleb_len(h);
  if (tid == 0) {
    put8(c.out, hl + nb, 4);
    for (uint32_t j = 0; j < hl; j++, h >>= 7) c.out[4 + j] = (uint8_t)((h & 0x7F) | (j + 1 < hl ? 0x80 : 0));
  }
  for (uint32_t j = tid; j < nb; j += NT) {
    uint32_t v = 0;
    for (uint32_t b = 0; b < 8; b++) {
      const uint32_t i = 8 * j + b;
      const bool ok = i < n && (!has_vb || ((A.validity[(r0 + i) >> 3] >> ((r0 + i) & 7)) & 1));
      v |= (ok ? 1u : 0u) << b;
    }
    c.out[4 + hl + j] = (uint8_t)v;
  }
  return 4 + hl + nb;
}

// The work area: LDS (work_bytes of it), or for a big page its HBM region,
// the LDS then holding the LZ4 tables and the sample.
__device__ __forceinline__ void set_work(Ctx& c, const AdArgs& A, uint32_t* lds) {
  c.lz4 = (uint8_t*)lds;
  c.wide = A.P > 65535;  // (only with an HBM work area)
  if (A.gwork) {
    c.work = (uint32_t*)(A.gwork + (uint64_t)blockIdx.x * A.gwork_bytes);
    c.samp = (uint8_t*)lds + sbc::kLz4WaveLds;
  } else {
    c.work = lds;
    c.samp = (uint8_t*)lds + A.work_bytes;
  }
}

__device__ void ctx_init(Ctx& c, Sh& sh, const AdArgs& A, uint32_t p) {
  c.work = nullptr;
  c.wide = false;
  c.work_bytes = A.work_bytes;
  c.scratch = A.scratch + (uint64_t)blockIdx.x * A.scratch_bytes;
  c.nmax = A.P;
  c.out = slot_of(A, blockIdx.x);
  c.cap = (uint32_t)min<uint64_t>(slot_cap(A, blockIdx.x), 0xFFFFFFFFull);
  c.o = A.o;
  if (threadIdx.x == 0) {
    sh.err = 0;
    sh.rng = page_seed(A.seed, p);
  }
  __syncthreads();
}

// Boolean pages: compress_boolean (compression/boolean/mod.rs:22-61) with
// choose_compressor (:222-280) -- forced RLE, else OneValue / RLE by ratio,
// the RLE ratio from compress_sample_ratio (:282-321: total bytes n / 8, or
// 80 for the 640-row sample) -- RLE over the bits as u8 values
// (boolean/rle.rs:31-39), OneValue (one_value.rs:44-52) or the Basic codecs
// over the page's bitmap bytes (the parent's bytes when the page starts on a
// byte, a rebuilt zero-padded bitmap otherwise).  The page's bits are staged
// one byte per row so the integer RLE and sampler serve unchanged.
template <bool ZS>
__global__ __launch_bounds__(NT) void k_enc_bool(AdArgs A) {
  extern __shared__ uint32_t lds[];
  __shared__ Sh sh;
  const uint32_t tid = threadIdx.x;
  const uint32_t p = A.page0 + blockIdx.x;
  const uint64_t r0 = (uint64_t)p * A.P;
  const uint32_t n = (uint32_t)min<uint64_t>(A.P, A.n_rows - r0);
  Ctx c;
  ctx_init(c, sh, A, p);
  uint8_t* vals;
  if (A.gwork) {  // a big page: run starts / Snappy table, staged bits and rebuilt bitmap in its HBM work area
    c.work = (uint32_t*)(A.gwork + (uint64_t)blockIdx.x * A.gwork_bytes);
    c.lz4 = (uint8_t*)lds;
    c.samp = (uint8_t*)lds + sbc::kLz4WaveLds;
    vals = (uint8_t*)c.work + bool_work_head(A.P);
  } else {
    c.work = lds;
    c.lz4 = (uint8_t*)lds;
    c.samp = (uint8_t*)lds + A.work_bytes;
    vals = c.samp + kSample * 8 + kSample / 8 + 16;
  }
  uint8_t* rebuilt = vals + ((A.P + 15) & ~15u);
  const uint32_t nb = (n + 7) / 8;
  for (uint32_t i = tid; i < n; i += NT) vals[i] = (A.values[(r0 + i) >> 3] >> ((r0 + i) & 7)) & 1;
  __syncthreads();
  if (r0 & 7)
    for (uint32_t j = tid; j < nb; j += NT) {
      uint32_t v = 0;
      for (uint32_t b = 0; b < 8 && 8 * j + b < n; b++) v |= (uint32_t)vals[8 * j + b] << b;
      rebuilt[j] = (uint8_t)v;
    }
  const bool has_vb = A.nullable && A.validity;
  uint32_t pos = write_prefix(c, A, r0, n);
  const Av a{vals, has_vb ? A.validity : nullptr, r0, n};
  uint32_t t = 0, f = 0;
  for (uint32_t i = tid; i < n; i += NT)
    if (valid_at(a, i)) (vals[i] ? t : f)++;
  const uint32_t T = (uint32_t)bsum(sh, t), F = (uint32_t)bsum(sh, f);
  const uint32_t fv = first_valid_row(sh, a);
  if (tid == 0) sh.first_valid = fv;
  __syncthreads();
  int codec = A.o.dflt;
  const uint32_t fm = A.o.forbidden;
  if (A.o.forced == C_RLE && !(fm & (1u << C_RLE))) {
    codec = C_RLE;  // check_rle_env
  } else if (A.o.has_ratio) {
    double maxr = A.o.ratio;
    const int cands[2] = {C_ONE, C_RLE};
    for (int k = 0; k < 2; k++) {
      const int cd = cands[k];
      if (fm & (1u << cd)) continue;
      double r;
      if (cd == C_ONE) {
        r = (T == 0 || F == 0) ? (double)n : 0.0;
      } else if (n / SC <= SS) {
        r = (double)(n / 8) / (double)rle_body<1, false, false, false>(c, sh, a, 0);
      } else {
        const Av smp = take_sample<1>(c, sh, a);
        r = 80.0 / (double)rle_body<1, false, false, false>(c, sh, smp, 0);
      }
      if (r > maxr) {
        maxr = r;
        codec = cd;
        if (r == (double)n) break;
      }
    }
  }
  const uint32_t body = pos + 9;
  uint32_t end = body;
  if (!room(c, sh, (uint64_t)body)) {
  } else if (codec == C_RLE) {
    end = body + rle_body<1, false, false, true>(c, sh, a, body);
  } else if (codec == C_ONE) {
    if (room(c, sh, (uint64_t)body + 1)) {
      if (tid == 0) c.out[body] = fv != 0xFFFFFFFFu ? vals[fv - 1] : 0;
      end = body + 1;
    }
  } else if (codec <= C_SNAPPY) {
    const uint8_t* src = (r0 & 7) ? rebuilt : A.values + r0 / 8;
    end = body + basic_body<ZS>(c, sh, codec, src, nb, body);
  } else {
    set_err(sh, E_SPEC);
  }
  __syncthreads();
  write_hdr(c, pos, codec, end - body, n);
  __syncthreads();
  if (tid == 0) {
    A.sizes[p] = sh.err ? 0 : end;
    A.status[p] = sh.err;
  }
}

template <int W, bool FLT, bool SGN, bool ZS>
__global__ __launch_bounds__(NT) void k_enc_adaptive(AdArgs A) {
  extern __shared__ uint32_t lds[];
  __shared__ Sh sh;
  const uint32_t tid = threadIdx.x;
  const uint32_t p = A.page0 + blockIdx.x;
  uint64_t r0;
  uint32_t n;
  page_rows(A, p, &r0, &n);
  Ctx c;
  ctx_init(c, sh, A, p);
  set_work(c, A, lds);
  const bool has_vb = A.nullable && A.validity;
  uint32_t pos = A.heads ? put_head(A, p, c.out, NT) : write_prefix(c, A, r0, n);
  const Av a{A.values + r0 * W, has_vb ? A.validity : nullptr, r0, n};
  __syncthreads();
  pos = enc_stream<W, FLT, SGN, 0, ZS>(c, sh, a, A.o.forbidden, pos);
  __syncthreads();
  if (tid == 0) {
    A.sizes[p] = sh.err ? 0 : pos;
    A.status[p] = sh.err;
  }
}


// ---------------------------------------------------------------------------
// Basic pages of a default LZ4 / Zstd codec that need no statistics (ratio
// None, no forced codec: choose_compressor returns the default codec,
// integer/mod.rs:267-307, binary/mod.rs:302-348): the page is the validity
// prefix and one headered stream of the raw values (BIN: two -- the offsets
// rebased to the page's first value, then the values), and the whole work is
// the one-wave LZ4 parse.  One 64-lane workgroup a page with only the LZ4
// tables in LDS: six pages a CU, where a 256-thread page workgroup of the
// general kernels holds three idle waves (and the register file for them) --
// C5's four LZ4 columns then overlap the rest of the table.  Bytes identical
// to k_enc_adaptive / k_enc_binary (write_prefix, enc_stream, basic_body).
// W: the value width (fixed-width pages) or the offset width (BIN).
template <int W, bool BIN, bool ZS>
__global__ __launch_bounds__(64) void k_enc_basic_wave(AdArgs A) {
  extern __shared__ uint32_t lds[];
  const uint32_t lane = threadIdx.x;
  const uint32_t p = A.page0 + blockIdx.x;
  uint64_t r0;
  uint32_t n;
  page_rows(A, p, &r0, &n);
  uint8_t* out = slot_of(A, blockIdx.x);
  const uint64_t cap = slot_cap(A, blockIdx.x);
  const int codec = A.o.dflt;
  sbc::lz4_lds8* tab = (sbc::lz4_lds8*)lds;
  uint32_t err = E_OK;
  uint32_t pos = 0;
  if (A.heads) {  // a List page: its level header (no validity prefix)
    pos = put_head(A, p, out, 64);
    __threadfence_block();
  } else if (A.nullable) {  // write_prefix (serialize.rs:200-215), one wave
    const uint32_t nb = (n + 7) / 8;
    uint64_t h = ((uint64_t)nb << 1) | 1;
    const uint32_t hl = uleb_len(h);
    if (4 + hl + nb > cap) {
      err = E_CAP;
    } else {
      if (lane == 0) {
        put8(out, hl + nb, 4);
        for (uint32_t j = 0; j < hl; j++, h >>= 7) out[4 + j] = (uint8_t)((h & 0x7F) | (j + 1 < hl ? 0x80 : 0));
      }
      for (uint32_t j = lane; j < nb; j += 64) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < 8; b++) {
          const uint32_t i = 8 * j + b;
          const bool ok = i < n && (!A.validity || ((A.validity[(r0 + i) >> 3] >> ((r0 + i) & 7)) & 1));
          v |= (ok ? 1u : 0u) << b;
        }
        out[4 + hl + j] = (uint8_t)v;
      }
      pos = 4 + hl + nb;
    }
  }
  // one headered stream of src[0, len) at `at` ([codec][csize][usize][body]); returns its end
  auto stream = [&](const uint8_t* src, uint32_t len, uint32_t at) -> uint32_t {
    const uint32_t body = at + 9;
    uint32_t cs = 0;
    if (codec == C_LZ4) {
      if ((uint64_t)body + sbc::lz4_bound(len) > cap) {
        err = E_CAP;
        return at;
      }
      for (uint32_t i = lane; i < 4096; i += 64) ((__attribute__((address_space(3))) uint32_t*)tab)[i] = 0;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the table's zeroes land before its reads
      __builtin_amdgcn_wave_barrier();
      // (the input stays in HBM: staging a page's 64 KiB in LDS measured 21.3
      // -> 11.9 GB/s on C5's encode -- one wave a CU instead of six)
      cs = sbc::lz4_compress_wave(sbc::Lz4GSrc{src}, len, out + body, tab, 1023);  // (kLz4WaveLdsMin)
    } else if constexpr (ZS) {
      const uint64_t zb = sbz::zstd_bound(len);
      if ((uint64_t)body + zb + sbc::lz4_bound(min(len, sbz::kZChunk)) + 16 > cap) {
        err = E_CAP;
        return at;
      }
      cs = __builtin_amdgcn_readfirstlane(zstd_frame_wave(src, len, out + body, out + body + zb, tab));  // (lane 0's)
    } else {
      err = E_NYI;  // (the host launches the ZS instantiation for a Zstd default codec)
      return at;
    }
    if (lane == 0) {
      out[at] = (uint8_t)codec;
      put8(out + at + 1, cs, 4);
      put8(out + at + 5, len, 4);
    }
    return body + cs;
  };
  if (!err) {
    if constexpr (!BIN) {
      pos = stream(A.values + r0 * W, n * W, pos);
    } else {
      // offsets rebased to the page's first value (the page's scratch), then the values
      const int64_t base = A.offsets[r0];
      uint8_t* obuf = A.scratch + (uint64_t)blockIdx.x * A.scratch_bytes;
      for (uint32_t i = lane; i <= n; i += 64) put8(obuf + i * W, (uint64_t)(A.offsets[r0 + i] - base), W);
      __threadfence_block();  // (the wave's stores before its loads of them)
      __builtin_amdgcn_wave_barrier();
      pos = stream(obuf, (n + 1) * W, pos);
      if (!err) pos = stream(A.values + base, (uint32_t)(A.offsets[r0 + n] - base), pos);
    }
  }
  if (lane == 0) {
    A.sizes[p] = err ? 0 : pos;
    A.status[p] = err;
  }
}

// ---------------------------------------------------------------------------
// Binary / Utf8 pages: compress_binary (compression/binary/mod.rs:26-93) --
// gen_stats (:265-300: distinct strings over every slot, nulls, the bytes of
// the distinct strings + 8 each, the most frequent string), choose_compressor
// (:302-348: forced Freq / Dict, else OneValue / Freq / Dict by ratio), Dict
// (dict.rs:55-93: ids by first occurrence over valid rows, row 0's raw bytes
// when it is null; the u32 index stream cascades), Freq (freq.rs:44-100:
// top string, roaring of the differing valid rows, u64 len + bytes records),
// OneValue (one_value.rs:50-68), Basic (offsets rebased to 0 + values, two
// headered streams).  Strings are compared by a per-row 64-bit hash, then
// by length and bytes.
// ---------------------------------------------------------------------------
struct Strs {
  const uint8_t* v;    // the column's values
  const int64_t* off;  // the page's rows: absolute positions off[0..n]
  const uint64_t* hsh;
  __device__ __forceinline__ uint64_t at(uint32_t r) const { return (uint64_t)off[r]; }
  __device__ __forceinline__ uint32_t len(uint32_t r) const { return (uint32_t)(off[r + 1] - off[r]); }
  __device__ bool eq(uint32_t a, uint32_t b) const {
    if (hsh[a] != hsh[b]) return false;
    const uint32_t l = len(a);
    if (l != len(b)) return false;
    const uint8_t* x = v + at(a);
    const uint8_t* y = v + at(b);
    for (uint32_t i = 0; i < l; i++)
      if (x[i] != y[i]) return false;
    return true;
  }
};

__device__ __forceinline__ uint64_t str_hash(const uint8_t* p, uint32_t n) {  // FNV-1a 64
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < n; i++) {
    h ^= p[i];
    h *= 1099511628211ull;
  }
  return mix64(h ^ n);
}

// records of rows (u64 len + bytes) at out + pos in the given row order;
// returns the bytes written
template <class RowF>
__device__ uint32_t put_records(Ctx& c, Sh& sh, const Strs& S, uint32_t cnt, RowF row, uint32_t pos) {
  const uint32_t tid = threadIdx.x;
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < cnt; t0 += NT) {
    const uint32_t j = t0 + tid;
    const uint32_t r = j < cnt ? row(j) : 0u;
    const uint32_t l = j < cnt ? S.len(r) : 0u;
    uint32_t tot;
    const uint32_t ex = bscan(sh, j < cnt ? 8 + l : 0u, &tot);
    if (j < cnt) {
      if ((uint64_t)pos + carry + ex + 8 + l <= c.cap) {
        uint8_t* o = c.out + pos + carry + ex;
        put8(o, l, 8);
        const uint8_t* x = S.v + S.at(r);
        for (uint32_t i = 0; i < l; i++) o[8 + i] = x[i];
      } else {
        set_err(sh, E_CAP);
      }
    }
    carry += tot;
  }
  __syncthreads();
  return carry;
}

template <int OW, bool ZS>
__global__ __launch_bounds__(NT) void k_enc_binary(AdArgs A) {
  extern __shared__ uint32_t lds[];
  __shared__ Sh sh;
  const uint32_t tid = threadIdx.x;
  const uint32_t p = A.page0 + blockIdx.x;
  const uint64_t r0 = (uint64_t)p * A.P;
  const uint32_t n = (uint32_t)min<uint64_t>(A.P, A.n_rows - r0);
  Ctx c;
  ctx_init(c, sh, A, p);
  set_work(c, A, lds);
  uint32_t* idx = (uint32_t*)c.scratch;  // region 0: ids, then rows of ids
  uint32_t* row_of = idx + A.P;
  uint64_t* hsh = (uint64_t*)(c.scratch + (uint64_t)2 * A.P * 8);
  uint8_t* obuf = c.scratch + (uint64_t)3 * A.P * 8;  // rebased offsets for a compressed Basic page
  const int64_t base = A.offsets[r0];
  auto slen = [&](uint32_t r) { return (uint32_t)(A.offsets[r0 + r + 1] - A.offsets[r0 + r]); };
  auto sptr = [&](uint32_t r) { return A.values + A.offsets[r0 + r]; };
  const bool has_vb = A.nullable && A.validity;
  const Av va{nullptr, has_vb ? A.validity : nullptr, r0, n};
  uint32_t pos = write_prefix(c, A, r0, n);
  auto same = [&](uint32_t a, uint32_t b) {
    if (hsh[a] != hsh[b]) return false;
    const uint32_t l = slen(a);
    if (l != slen(b)) return false;
    const uint8_t* x = sptr(a);
    const uint8_t* y = sptr(b);
    for (uint32_t i = 0; i < l; i++)
      if (x[i] != y[i]) return false;
    return true;
  };
  // stats over every row (nulls included): only to choose among codecs
  // (binary/mod.rs:303-330); a Basic(default) page needs none
  uint32_t NU = 0, U = 0, maxc = 0, top_row = 0;
  uint64_t TU = 0;
  const uint32_t Sl = tab_slots(n);
  const Tab tab{c.work, c.wide};
  if (needs_stats(A.o, A.o.forbidden)) {
    for (uint32_t r = tid; r < n; r += NT) hsh[r] = str_hash(sptr(r), slen(r));
    __syncthreads();
    tab.clear(Sl);
    __syncthreads();
    uint32_t nulls = 0;
    for (uint32_t r = tid; r < n; r += NT) {
      tab_insert_h(tab, Sl, r, hsh[r], [&](uint32_t o) { return same(o, r); });
      nulls += !valid_at(va, r);
    }
    __syncthreads();
    uint32_t uniq = 0;
    uint64_t best = 0, tu = 0;
    for (uint32_t i = tid; i < Sl; i += NT) {
      const uint32_t r1 = tab.row1(i);
      if (r1) {
        uniq++;
        tu += slen(r1 - 1) + 8;
        best = max(best, ((uint64_t)tab.hi(i) << 32) | (0xFFFFFFFFu - (r1 - 1)));
      }
    }
    NU = (uint32_t)bsum(sh, nulls), U = (uint32_t)bsum(sh, uniq);
    TU = bsum(sh, tu);
    const uint64_t BEST = bmax(sh, best);
    maxc = (uint32_t)(BEST >> 32), top_row = 0xFFFFFFFFu - (uint32_t)BEST;
  }
  const uint64_t total_bytes = A.parent_len + (uint64_t)(n + 1) * OW;
  int codec = A.o.dflt;
  const uint32_t fm = A.o.forbidden;
  if (A.o.forced == C_FREQ && !(fm & (1u << C_FREQ))) {
    codec = C_FREQ;
  } else if (A.o.forced == C_DICT && !(fm & (1u << C_DICT))) {
    codec = C_DICT;
  } else if (A.o.has_ratio) {
    double maxr = A.o.ratio;
    const int cands[3] = {C_ONE, C_FREQ, C_DICT};
    for (int k = 0; k < 3; k++) {
      const int cd = cands[k];
      if (fm & (1u << cd)) continue;
      double r = 0.0;
      if (cd == C_ONE) {
        r = U <= 1 ? (double)n : 0.0;
      } else if (cd == C_FREQ) {
        if (U > 1) {
          if ((double)NU / (double)n >= 0.9) r = (double)(n - 1);
          else if ((double)maxc / (double)n >= 0.9) r = (double)(n - 1);
        }
      } else if ((uint64_t)U * 3 < n) {
        const uint64_t after = TU + (uint64_t)n * (bits_needed(U) / 8) + (uint64_t)n * 2 / 128;
        r = (double)total_bytes / (double)after;
      }
      if (r > maxr) {
        maxr = r;
        codec = cd;
        if (r == (double)n) break;
      }
    }
  }
  const uint32_t body = pos + 9;
  uint32_t end = body;
  uint32_t usize = (uint32_t)A.parent_len;
  if (!room(c, sh, (uint64_t)body)) {
  } else if (codec <= C_SNAPPY) {
    // offsets rebased to the page's first value, then the values (two streams)
    const uint32_t ob = (n + 1) * OW;
    uint32_t cs;
    if (codec == C_NONE) {
      if (room(c, sh, (uint64_t)body + ob)) {
        for (uint32_t i = tid; i <= n; i += NT) put8(c.out + body + i * OW, (uint64_t)(A.offsets[r0 + i] - base), OW);
      }
      cs = ob;
    } else {
      for (uint32_t i = tid; i <= n; i += NT) put8(obuf + i * OW, (uint64_t)(A.offsets[r0 + i] - base), OW);
      __syncthreads();
      cs = basic_body<ZS>(c, sh, codec, obuf, ob, body);
    }
    __syncthreads();
    write_hdr(c, pos, codec, cs, ob);
    const uint32_t h2 = body + cs;
    const uint32_t vl = (uint32_t)(A.offsets[r0 + n] - base);
    if (room(c, sh, (uint64_t)h2 + 9)) {
      const uint32_t cs2 = basic_body<ZS>(c, sh, codec, A.values + base, vl, h2 + 9);
      __syncthreads();
      write_hdr(c, h2, codec, cs2, vl);
      end = h2 + 9 + cs2;
    }
    __syncthreads();
    if (tid == 0) {
      A.sizes[p] = sh.err ? 0 : end;
      A.status[p] = sh.err;
    }
    return;
  } else if (codec == C_ONE) {
    const uint32_t fv = first_valid_row(sh, va);
    const uint32_t l = fv != 0xFFFFFFFFu ? slen(fv - 1) : 0u;
    if (room(c, sh, (uint64_t)body + 4 + l)) {
      if (tid == 0) put8(c.out + body, l, 4);
      for (uint32_t i = tid; i < l; i += NT) c.out[body + 4 + i] = sptr(fv - 1)[i];
      end = body + 4 + l;
    }
  } else if (codec == C_DICT) {
    auto ins = [&](uint32_t r) { return r == 0 || valid_at(va, r); };
    tab.clear(Sl);
    __syncthreads();
    for (uint32_t r = tid; r < n; r += NT)
      if (ins(r)) idx[r] = tab_insert_h(tab, Sl, r, hsh[r], [&](uint32_t o) { return same(o, r); });
    __syncthreads();
    // ids over thread chunks of consecutive rows, as dict_body
    const uint32_t ch = (n + NT - 1) / NT, c0 = min(n, tid * ch), c1 = min(n, c0 + ch);
    auto first = [&](uint32_t r) { return ins(r) && tab.row1(idx[r]) == r + 1; };
    uint32_t nf = 0;
    for (uint32_t r = c0; r < c1; r++) nf += first(r) ? 1u : 0u;
    uint32_t k;
    uint32_t wpos = bscan(sh, nf, &k);
    for (uint32_t r = c0; r < c1; r++)
      if (first(r)) row_of[wpos++] = r;
    __syncthreads();
    for (uint32_t j = tid; j < k; j += NT) tab.set(idx[row_of[j]], j, row_of[j] + 1);
    __syncthreads();
    for (uint32_t r = tid; r < n; r += NT)
      if (ins(r)) idx[r] = tab.hi(idx[r]);
    __syncthreads();
    uint32_t lastc = 0;
    for (uint32_t r = c0; r < c1; r++)
      if (ins(r)) lastc = r + 1;
    uint32_t tmax;
    uint32_t last = bexcl_max(sh, lastc, &tmax);
    for (uint32_t r = c0; r < c1; r++) {
      if (ins(r)) last = r + 1;
      else idx[r] = idx[last - 1];
    }
    __syncthreads();
    // the index stream cascades (Dict forbidden) at depth 1 (its scratch: region 1)
    const Av ia{(const uint8_t*)idx, nullptr, 0, n};
    const uint32_t p2 = enc_stream<4, false, false, 1, ZS>(c, sh, ia, fm | (1u << C_DICT), body);
    if (!sh.err && room(c, sh, (uint64_t)p2 + 4)) {
      if (tid == 0) put8(c.out + p2, k, 4);
      const Strs SS2{A.values, A.offsets + r0, hsh};
      end = p2 + 4 + put_records(c, sh, SS2, k, [&](uint32_t j) { return row_of[j]; }, p2 + 4);
    }
  } else if (codec == C_FREQ) {
    const bool top_null = (double)NU / (double)n >= 0.9;
    const uint32_t tl = top_null ? 0u : slen(top_row);
    uint32_t* bm = c.work;
    const bool multi = n > 65536;  // (a wide page: several roaring containers)
    __syncthreads();
    for (uint32_t i = tid; i < (multi ? (n + 31) / 32 : 2048u); i += NT) bm[i] = 0;
    __syncthreads();
    const uint32_t rpos = body + 8 + tl + 4;
    const uint32_t data = rpos + 16;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < n; t0 += NT) {
      const uint32_t r = t0 + tid;
      const bool e = r < n && valid_at(va, r) && (top_null || !same(r, top_row));
      uint32_t tot;
      const uint32_t ex = bscan(sh, e ? 1u : 0u, &tot);
      if (e) {
        const uint32_t j = carry + ex;
        row_of[j] = r;
        atomicOr(&bm[r >> 5], 1u << (r & 31));
        if (!multi && (uint64_t)data + 2ull * (j + 1) <= c.cap) put8(c.out + data + 2 * j, r & 0xFFFF, 2);
      }
      carry += tot;
    }
    const uint32_t e = carry;
    __syncthreads();
    uint32_t bytes = e == 0 ? 8u : (e <= 4096 ? 16 + 2 * e : 16 + 8192u);
    if (multi) bytes = roaring_multi(c, sh, bm, row_of, e, n, rpos, (uint32_t*)(c.scratch + (uint64_t)4 * A.P * 8 + 64));
    if ((!multi || bytes) && room(c, sh, (uint64_t)rpos + bytes)) {
      if (tid == 0) {
        put8(c.out + body, tl, 8);
        put8(c.out + body + 8 + tl, bytes, 4);
        if (!multi) {
          put8(c.out + rpos, 12346, 4);
          put8(c.out + rpos + 4, e ? 1u : 0u, 4);
          if (e) {
            put8(c.out + rpos + 8, 0, 2);
            put8(c.out + rpos + 10, e - 1, 2);
            put8(c.out + rpos + 12, 16, 4);
          }
        }
      }
      for (uint32_t i = tid; i < tl; i += NT) c.out[body + 8 + i] = sptr(top_row)[i];
      if (!multi && e > 4096)
        for (uint32_t i = tid; i < 2048; i += NT) put8(c.out + data + 4 * i, bm[i], 4);
      __syncthreads();
      const Strs SS2{A.values, A.offsets + r0, hsh};
      end = rpos + bytes + put_records(c, sh, SS2, e, [&](uint32_t j) { return row_of[j]; }, rpos + bytes);
    }
  } else {
    set_err(sh, E_SPEC);
  }
  __syncthreads();
  write_hdr(c, pos, codec, end - body, usize);
  __syncthreads();
  if (tid == 0) {
    A.sizes[p] = sh.err ? 0 : end;
    A.status[p] = sh.err;
  }
}

// page offsets of a batch: running total in offs[n_pages]
__global__ __launch_bounds__(NT) void k_enc_offsets(AdArgs A) {
  __shared__ Sh sh;
  uint64_t carry = A.offs[A.n_pages];
  for (uint32_t q0 = 0; q0 < A.n_batch; q0 += NT) {
    const uint32_t q = q0 + threadIdx.x;
    const uint64_t v = q < A.n_batch ? A.sizes[A.page0 + q] : 0;
    // 64-bit exclusive scan
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) sh.red[wv] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int k = 0; k < NW; k++) {
      pre += (uint32_t)k < wv ? sh.red[k] : 0;
      tot += sh.red[k];
    }
    __syncthreads();
    if (q < A.n_batch) A.offs[A.page0 + q] = carry + pre + x - v;
    carry += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) A.offs[A.n_pages] = carry;
}

// slot -> output, one workgroup per page
__global__ __launch_bounds__(NT) void k_enc_compact(AdArgs A) {
  const uint32_t p = A.page0 + blockIdx.x;
  const uint64_t len = A.sizes[p], off = A.offs[p];
  if (off + len > A.out_cap) {
    if (threadIdx.x == 0) A.status[p] = E_CAP;
    return;
  }
  const uint8_t* src = slot_of(A, blockIdx.x);  // 16-byte aligned
  uint8_t* dst = A.out + off;
  const uint32_t head = (uint32_t)min<uint64_t>(len, (16 - ((uintptr_t)dst & 15)) & 15);
  for (uint32_t j = threadIdx.x; j < head; j += NT) dst[j] = src[j];
  // dst + head is 16-aligned; src + head is not in general: assemble from aligned dwords
  const uint64_t body = (len - head) / 16;
  const uint32_t sh4 = (uint32_t)(head & 3);
  const uint32_t* sw = (const uint32_t*)(src + (head & ~3u));
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  for (uint64_t i = threadIdx.x; i < body; i += NT) {
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; k++) w[k] = sw[4 * i + k];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(w[1], w[0], sh4);
    v.y = __builtin_amdgcn_alignbyte(w[2], w[1], sh4);
    v.z = __builtin_amdgcn_alignbyte(w[3], w[2], sh4);
    v.w = __builtin_amdgcn_alignbyte(w[4], w[3], sh4);
    *(u32x4*)(dst + head + 16 * i) = v;
  }
  for (uint64_t j = head + body * 16 + threadIdx.x; j < len; j += NT) dst[j] = src[j];
}

// ---------------------------------------------------------------------------
// List<primitive> pages (write_nested, serialize.rs:133-146; RepLevelsIter /
// DefLevelsIter of one list level, nested/rep.rs, nested/def.rs): one
// workgroup per page of `step` top-level rows writes the page's level header
// -- [rows u32][rep_len u32][def_len u32][rep stream][def stream], each
// stream one bit-packed hybrid run: ULEB128((ceil(L / 8) << 1) | 1), then
// ceil(L * bw / 8) bytes of 32-level chunks.  The writer packs the last,
// partial chunk from its reused 32-value buffer, so the spare bits of its
// last byte hold level i - 32 (zero when there is no earlier chunk): the
// host writer's encode_levels_u32 (sb_encode.cpp), bit for bit.  A row is
// one level (rep 0) when the list is null (def 0) or empty (def nl), else
// one per item (rep 0 for the first, 1 after; def max_def, or max_def - 1
// under a null item).  LDS: the rows' level prefix (dynamic, rows + 1 u32).
// ---------------------------------------------------------------------------
struct ListLv {
  const int64_t* offsets;   // n_rows + 1 absolute child positions
  const uint8_t* lvalid;    // list validity (rows) or nullptr
  const uint8_t* cvalid;    // child validity (child values) or nullptr
  uint64_t n_rows;
  uint32_t step, nl, ni;
  uint8_t* heads;           // page p's header at heads + p * head_slot
  uint64_t head_slot;
  uint32_t* head_len;
  uint64_t* levels;         // [n_pages] level counts (PageMeta.num_values)
};

__device__ __forceinline__ bool bit_at(const uint8_t* bm, uint64_t i) { return (bm[i >> 3] >> (i & 7)) & 1; }

__global__ __launch_bounds__(NT) void k_enc_list_levels(ListLv a) {
  extern __shared__ uint32_t lpre[];  // [m + 1]: the rows' first level
  __shared__ uint32_t s_red[NW];
  const uint32_t p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t r0 = (uint64_t)p * a.step;
  const uint32_t m = (uint32_t)min<uint64_t>(a.step, a.n_rows - r0);
  const uint32_t max_def = a.nl + 1 + a.ni, bwd = 32 - __clz(max_def);
  auto row_levels = [&](uint32_t r) -> uint32_t {
    if (a.nl && a.lvalid && !bit_at(a.lvalid, r0 + r)) return 1u;
    const int64_t len = a.offsets[r0 + r + 1] - a.offsets[r0 + r];
    return len > 0 ? (uint32_t)len : 1u;
  };
  // 1. the level prefix over the rows (chunks of consecutive rows per thread);
  // a decreasing offset pair (a negative list length) fails the page
  __shared__ uint32_t s_bad;
  if (tid == 0) s_bad = 0;
  __syncthreads();
  const uint32_t ch = (m + NT - 1) / NT, b0 = min(m, tid * ch), b1 = min(m, b0 + ch);
  uint32_t sum = 0;
  bool bad = false;
  for (uint32_t r = b0; r < b1; r++) {
    sum += row_levels(r);
    bad |= a.offsets[r0 + r + 1] < a.offsets[r0 + r];
  }
  if (bad) atomicOr(&s_bad, 1u);
  uint32_t x = sum;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_red[wv] = x;
  __syncthreads();
  uint32_t pre = x - sum, L = 0;
  for (uint32_t k = 0; k < NW; k++) {
    pre += k < wv ? s_red[k] : 0u;
    L += s_red[k];
  }
  for (uint32_t r = b0; r < b1; r++) {
    lpre[r] = pre;
    pre += row_levels(r);
  }
  if (tid == 0) lpre[m] = L;
  __syncthreads();
  if (s_bad) {  // every thread sees the flag after the barrier: the page is refused whole
    if (tid == 0) {
      a.head_len[p] = 0;
      a.levels[p] = ~0ull;
    }
    return;
  }
  // level i's (rep, def); the spare bits past L hold level i - 32 (or 0)
  auto level = [&](uint32_t i) -> uint32_t {  // rep | def << 1
    if (i >= L) {
      if (i < 32) return 0u;
      i -= 32;
    }
    uint32_t lo = 0, hi = m;  // the last row with lpre[row] <= i
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (lpre[mid] <= i) lo = mid;
      else hi = mid;
    }
    const uint32_t j = i - lpre[lo];
    if (a.nl && a.lvalid && !bit_at(a.lvalid, r0 + lo)) return 0u;
    const int64_t b = a.offsets[r0 + lo], len = a.offsets[r0 + lo + 1] - b;
    if (len <= 0) return a.nl << 1;
    const uint32_t def = a.ni ? (!a.cvalid || bit_at(a.cvalid, (uint64_t)b + j) ? max_def : max_def - 1) : max_def;
    return (j > 0 ? 1u : 0u) | (def << 1);
  };
  uint64_t h = ((uint64_t)((L + 7) / 8) << 1) | 1;
  uint32_t hl = 1;
  for (uint64_t t = h; t >= 0x80; t >>= 7) hl++;
  const uint32_t rb = (L + 7) / 8, db = (L * bwd + 7) / 8;
  uint8_t* out = a.heads + (uint64_t)p * a.head_slot;
  if (tid == 0) {
    const uint32_t w[3] = {m, hl + rb, hl + db};
    for (uint32_t k = 0; k < 12; k++) out[k] = (uint8_t)(w[k / 4] >> (8 * (k % 4)));
    for (uint32_t k = 0; k < hl; k++) {
      const uint8_t c = (uint8_t)((h >> (7 * k)) & 0x7F) | (k + 1 < hl ? 0x80 : 0);
      out[12 + k] = c;
      out[12 + hl + rb + k] = c;
    }
    a.head_len[p] = 12 + 2 * hl + rb + db;
    a.levels[p] = L;
  }
  for (uint32_t k = tid; k < rb; k += NT) {  // rep: 8 levels a byte
    uint32_t v = 0;
    for (uint32_t b = 0; b < 8; b++) v |= (level(8 * k + b) & 1u) << b;
    out[12 + hl + k] = (uint8_t)v;
  }
  const uint32_t per = 8 / bwd;
  for (uint32_t k = tid; k < db; k += NT) {  // def: 8 / bw levels a byte
    uint32_t v = 0;
    for (uint32_t b = 0; b < per; b++) v |= (level(per * k + b) >> 1) << (b * bwd);
    out[12 + 2 * hl + rb + k] = (uint8_t)v;
  }
}

}  // namespace sba

// ===========================================================================
// host side
// ===========================================================================
namespace sb {

static uint64_t stream_bound(uint64_t n, uint64_t w, int depth) {
  // worst case of one headered stream of n values of w bytes (cascade depth left)
  // (Zstd: the frame's bound + the LZ4 parse of one chunk behind it)
  const uint64_t zstd = sbz::zstd_bound(n * w) + sbc::lz4_bound((uint32_t)std::min<uint64_t>(n * w, sbz::kZChunk)) + 16;
  const uint64_t leaf = 9 + std::max({n * (4 + w), n * w + n * w / 255 + 32, (n / 128) * 513, w + n * (2 + w), zstd});
  if (depth == 0) return leaf;
  const uint64_t dict = 9 + stream_bound(n, 4, depth - 1) + 4 + n * w;
  const uint64_t freq = 9 + w + 4 + 16 + 8 * ((n + 65535) / 65536) + std::max<uint64_t>(2 * n, 8192) +
                        stream_bound(n, w, depth - 1);
  return std::max({leaf, dict, freq});
}

uint64_t adaptive_slot_bytes(uint64_t P, uint32_t w, int nullable) {
  const uint64_t pre = nullable ? 4 + 10 + (P + 7) / 8 : 0;
  return (pre + stream_bound(P, w, 2) + 64 + 15) & ~15ull;
}

// LDS work area of a page's workgroup: the statistics' hash table (two slots
// a row) and the general codecs' tables; a Basic(default) page with no
// statistics needs only its codec's (more workgroups per CU for LZ4 pages)
uint32_t adaptive_work_bytes(uint64_t P, const sba::Opts& o) {
  if (!sba::needs_stats(o, o.forbidden))
    return o.dflt == sba::C_SNAPPY                          ? sbc::kSnappyTableBytes
           : (o.dflt == sba::C_LZ4 || o.dflt == sba::C_ZSTD) ? sbc::kLz4WaveLds
                                                             : 8192;
  uint64_t s = 64;
  while (s < 2 * P) s <<= 1;
  return (uint32_t)std::max<uint64_t>({4 * s, sbc::kSnappyTableBytes, 8192});
}

// A big page's HBM work area (pages over kMaxRows rows): the statistics'
// hash table (rows < 65536: the 16-bit table words hold them), or for a
// Basic page only the Snappy table.
uint64_t big_work_bytes(uint64_t P, bool stats) {
  uint64_t s = 64;
  while (s < 2 * P) s <<= 1;
  const uint64_t word = P > 65535 ? 8 : 4;  // (wide table words)
  return stats ? std::max<uint64_t>(word * s, sbc::kSnappyTableBytes) : sbc::kSnappyTableBytes;
}

// Pages of a batch: at most 2048, and at most ~2 GiB of slots + scratch + work.
static uint32_t batch_pages(uint64_t np, uint64_t per_page) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({np, 2048, (2ull << 30) / std::max<uint64_t>(per_page, 1)}));
}

// A Basic page of a default LZ4 / Zstd codec without statistics: the
// one-wave page kernel (k_enc_basic_wave), LDS = the LZ4 tables.
static bool wave_basic(const sba::Opts& o) {
  return !sba::needs_stats(o, o.forbidden) && (o.dflt == sba::C_LZ4 || o.dflt == sba::C_ZSTD);
}
template <int W, bool BIN>
static void launch_wave_basic(const sba::AdArgs& a, hipStream_t st) {
  constexpr uint32_t lds = sbc::kLz4WaveLds;
  if (a.o.dflt == sba::C_ZSTD) {
    ensure_lds_attr(sba::k_enc_basic_wave<W, BIN, true>, (int)lds);
    hipLaunchKernelGGL((sba::k_enc_basic_wave<W, BIN, true>), dim3(a.n_batch), dim3(64), lds, st, a);
  } else {  // LZ4: the compressor's smallest area (more page-waves a CU)
    ensure_lds_attr(sba::k_enc_basic_wave<W, BIN, false>, (int)sbc::kLz4WaveLdsMin);
    hipLaunchKernelGGL((sba::k_enc_basic_wave<W, BIN, false>), dim3(a.n_batch), dim3(64), sbc::kLz4WaveLdsMin, st, a);
  }
}

template <int W, bool FLT, bool SGN>
static void launch_t(const sba::AdArgs& a, uint32_t lds, hipStream_t st) {
  if (wave_basic(a.o)) {
    launch_wave_basic<W, false>(a, st);
    return;
  }
  if (a.o.dflt == sba::C_ZSTD) {
    ensure_lds_attr(sba::k_enc_adaptive<W, FLT, SGN, true>, (int)lds);
    hipLaunchKernelGGL((sba::k_enc_adaptive<W, FLT, SGN, true>), dim3(a.n_batch), dim3(sba::NT), lds, st, a);
  } else {
    ensure_lds_attr(sba::k_enc_adaptive<W, FLT, SGN, false>, (int)lds);
    hipLaunchKernelGGL((sba::k_enc_adaptive<W, FLT, SGN, false>), dim3(a.n_batch), dim3(sba::NT), lds, st, a);
  }
}
template <int OW>
static void launch_bin(const sba::AdArgs& a, uint32_t lds, hipStream_t st) {
  if (wave_basic(a.o)) {
    launch_wave_basic<OW, true>(a, st);
    return;
  }
  if (a.o.dflt == sba::C_ZSTD) {
    ensure_lds_attr(sba::k_enc_binary<OW, true>, (int)lds);
    hipLaunchKernelGGL((sba::k_enc_binary<OW, true>), dim3(a.n_batch), dim3(sba::NT), lds, st, a);
  } else {
    ensure_lds_attr(sba::k_enc_binary<OW, false>, (int)lds);
    hipLaunchKernelGGL((sba::k_enc_binary<OW, false>), dim3(a.n_batch), dim3(sba::NT), lds, st, a);
  }
}

// Encodes every page of a fixed-width column; returns SB status.
// List pages (encode_list_device): each page's child-value range and level header
struct ListPart {
  const uint64_t* rows_at;  // device [np + 1]
  const uint8_t* heads;
  uint64_t head_slot;
  const uint32_t* head_len;
  const uint64_t* h_levels;  // host [np]: PageMeta.num_values
};

int encode_adaptive(sb_ctx* ctx, int phys, const uint8_t* d_values, const uint8_t* d_validity, uint64_t n_rows,
                    int nullable, const sb_write_options* opts, uint64_t P, uint8_t* d_out, uint64_t out_cap,
                    uint64_t* out_len, sb_page_meta* h_metas, uint64_t np, const ListPart* lp) {
  sba::Opts o{opts->default_codec, opts->has_ratio, opts->ratio, opts->forbidden_mask, opts->forced_codec};
  uint32_t w = 0;
  bool flt = false, sgn = false;
  switch (phys) {
    case SB_T_INT8: w = 1; sgn = true; break;
    case SB_T_INT16: w = 2; sgn = true; break;
    case SB_T_INT32: w = 4; sgn = true; break;
    case SB_T_INT64: w = 8; sgn = true; break;
    case SB_T_UINT8: w = 1; break;
    case SB_T_UINT16: w = 2; break;
    case SB_T_UINT32: w = 4; break;
    case SB_T_UINT64: w = 8; break;
    case SB_T_FLOAT32: w = 4; flt = true; break;
    case SB_T_FLOAT64: w = 8; flt = true; break;
    case SB_T_BOOLEAN: w = 1; break;
    default: return SB_E_NYI;
  }
  const bool is_bool = phys == SB_T_BOOLEAN;
  // Pages over kMaxRows rows keep their work area in HBM (any size; over
  // 65535 rows with 64-bit table words and several roaring containers);
  // Boolean pages stage their bits in LDS up to kMaxRows, in HBM past it
  const bool stats = sba::needs_stats(o, o.forbidden);
  const bool big = P > sba::kMaxRows;
  if (big && (P * w > 0xFFFFFFF0ull || P > 0x7FFFFFFFull)) return SB_E_NYI;
  if (lp && phys == SB_T_BOOLEAN) return SB_E_NYI;
  const uint64_t slot = adaptive_slot_bytes(P, w, lp ? 0 : nullable) + (lp ? lp->head_slot : 0);
  const uint64_t scr = is_bool ? 256 : ((P > 65535 ? 3 : 2) * P * 8 + 255) & ~255ull;  // (wide: roaring rows, level 2)
  const uint64_t gwb = !big ? 0 : is_bool ? sba::bool_work_bytes(P) : big_work_bytes(P, stats);
  const uint32_t batch = batch_pages(np, slot + scr + gwb);
  sba::Opts wo = o;
  if (is_bool) wo.has_ratio = 1;  // (k_enc_bool stages its bits after the full work area)
  const uint32_t work = big ? 0u : adaptive_work_bytes(P, wo);
  uint32_t lds = (big ? sbc::kLz4WaveLds : work) + sba::kSample * 8 + sba::kSample / 8 + 16;
  if (is_bool && !big) lds += (uint32_t)(((P + 15) & ~15ull) + (P + 7) / 8 + 16);  // staged bits + rebuilt bitmap
  uint8_t* slots = (uint8_t*)ctx_scratch(ctx, batch * slot + 256, 0);
  uint8_t* scratch = (uint8_t*)ctx_scratch(ctx, batch * scr, 1);
  uint64_t* meta = (uint64_t*)ctx_scratch(ctx, (2 * np + 2) * 8 + np * 4, 2);
  uint8_t* gwork = big ? (uint8_t*)ctx_scratch(ctx, batch * gwb, 4) : nullptr;
  if (!slots || !scratch || !meta || (big && !gwork)) return ctx_fail(ctx, SB_E_DEVICE, "device encode step 1");
  hipStream_t st = (hipStream_t)sb_ctx_stream(ctx);
  uint64_t* sizes = meta;
  uint64_t* offs = meta + np;  // [np + 1]
  uint32_t* status = (uint32_t*)(meta + 2 * np + 2);
  if (hipMemsetAsync(offs + np, 0, 8, st) != hipSuccess) return ctx_fail(ctx, SB_E_DEVICE, "device encode step 2");
  for (uint64_t b0 = 0; b0 < np; b0 += batch) {
    sba::AdArgs a{d_values, d_validity, n_rows, (uint32_t)P, (uint32_t)b0, (uint32_t)std::min<uint64_t>(batch, np - b0),
                  nullable, o, opts->seed, slots, slot, scratch, scr, work, gwork, gwb, sizes, status, offs, d_out, out_cap,
                  (uint32_t)np, nullptr, 0, 0, nullptr};
    if (lp) {
      a.rows_at = lp->rows_at;
      a.heads = lp->heads;
      a.head_slot = lp->head_slot;
      a.head_len = lp->head_len;
    }
    if (is_bool) {
      if (o.dflt == sba::C_ZSTD) {
        ensure_lds_attr(sba::k_enc_bool<true>, (int)lds);
        hipLaunchKernelGGL(sba::k_enc_bool<true>, dim3(a.n_batch), dim3(sba::NT), lds, st, a);
      } else {
        ensure_lds_attr(sba::k_enc_bool<false>, (int)lds);
        hipLaunchKernelGGL(sba::k_enc_bool<false>, dim3(a.n_batch), dim3(sba::NT), lds, st, a);
      }
    } else if (flt) {
      if (w == 4) launch_t<4, true, false>(a, lds, st);
      else launch_t<8, true, false>(a, lds, st);
    } else if (sgn) {
      if (w == 1) launch_t<1, false, true>(a, lds, st);
      else if (w == 2) launch_t<2, false, true>(a, lds, st);
      else if (w == 4) launch_t<4, false, true>(a, lds, st);
      else launch_t<8, false, true>(a, lds, st);
    } else {
      if (w == 1) launch_t<1, false, false>(a, lds, st);
      else if (w == 2) launch_t<2, false, false>(a, lds, st);
      else if (w == 4) launch_t<4, false, false>(a, lds, st);
      else launch_t<8, false, false>(a, lds, st);
    }
    hipLaunchKernelGGL(sba::k_enc_offsets, dim3(1), dim3(sba::NT), 0, st, a);
    hipLaunchKernelGGL(sba::k_enc_compact, dim3(a.n_batch), dim3(sba::NT), 0, st, a);
    if (const hipError_t e = hipGetLastError(); e != hipSuccess)
      return ctx_fail(ctx, SB_E_DEVICE, "device encode launch (step 3)", (int)e);
  }
  std::vector<uint64_t> sz(np + 1 + np);
  std::vector<uint32_t> stv(np);
  if (hipMemcpyAsync(sz.data(), sizes, (2 * np + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(stv.data(), status, np * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device encode step 4");
  for (uint64_t p = 0; p < np; p++) {
    if (stv[p] == sba::E_NYI) return SB_E_NYI;
    if (stv[p] == sba::E_CAP) return SB_E_ARG;
    if (stv[p]) return SB_E_OUT_OF_SPEC;
  }
  *out_len = sz[np + np];
  for (uint64_t p = 0; p < np; p++)
    h_metas[p] = sb_page_meta{sz[p], lp ? lp->h_levels[p] : std::min<uint64_t>(P, n_rows - p * P)};
  return SB_OK;
}

// encode_chunk of one List<primitive> leaf on the device (write/common.rs:
// 49-119 with slice_parquet_array per page of `step` top-level rows,
// write_nested serialize.rs:133-146): the level headers (k_enc_list_levels),
// then each page's child values through the adaptive page kernels (the
// writer's compress_* over the sliced child array: its validity feeds the
// statistics, no prefix) behind its header.  Byte-identical to
// sb_encode_list_column.
__global__ void k_list_rows_at(const int64_t* offs, uint64_t n_rows, uint64_t step, uint64_t np, uint64_t* out) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= np) out[p] = (uint64_t)offs[std::min<uint64_t>(p * step, n_rows)];
}

int encode_list_device(sb_ctx* ctx, int phys, const int64_t* d_offsets, const uint8_t* d_list_validity,
                       int list_nullable, const void* d_child, const uint8_t* d_child_validity, int item_nullable,
                       uint64_t n_rows, const sb_write_options* opts, uint64_t step, uint8_t* d_out, uint64_t out_cap,
                       uint64_t* out_len, sb_page_meta* h_metas, uint64_t np) {
  hipStream_t st = (hipStream_t)sb_ctx_stream(ctx);
  // rows_at [np + 1] u64 | levels [np] u64 | head_len [np] u32 in one grow-only
  // context slot, the page headers in another (encode_adaptive uses 0..4)
  const size_t meta_bytes = (np + 1) * 8 + np * 8 + np * 4;
  uint8_t* meta = (uint8_t*)ctx_scratch(ctx, meta_bytes, 5);
  if (!meta) return ctx_fail(ctx, SB_E_DEVICE, "device list encode alloc");
  uint64_t* d_rows_at = (uint64_t*)meta;
  uint64_t* d_levels = d_rows_at + np + 1;
  uint32_t* d_hlen = (uint32_t*)(d_levels + np);
  std::vector<uint64_t> rows_at(np + 1), levels(np);
  hipLaunchKernelGGL(k_list_rows_at, dim3((uint32_t)((np + 256) / 256)), dim3(256), 0, st, d_offsets, n_rows, step, np,
                     d_rows_at);
  if (const hipError_t e = hipGetLastError(); e != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device list encode launch (step 1)", (int)e);
  if (hipMemcpyAsync(rows_at.data(), d_rows_at, (np + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device list encode step 1");
  // the host writer's check: offsets must not decrease (else P and the slot sizes wrap)
  for (uint64_t q = 0; q < np; q++)
    if (rows_at[q + 1] < rows_at[q] || (int64_t)rows_at[q] < 0) return ctx_fail(ctx, SB_E_ARG, "decreasing list offsets");
  uint64_t P = 1;
  for (uint64_t q = 0; q < np; q++) P = std::max<uint64_t>(P, rows_at[q + 1] - rows_at[q]);
  // a page's levels: <= rows + values; header: 12 + two ULEB128 runs + the packed levels
  const uint64_t lmax = step + P;
  const uint64_t head_slot = (12 + 2 * 10 + (lmax + 7) / 8 + (2 * lmax + 7) / 8 + 15) & ~15ull;
  uint8_t* d_heads = (uint8_t*)ctx_scratch(ctx, np * head_slot, 6);
  if (!d_heads) return ctx_fail(ctx, SB_E_DEVICE, "device list encode alloc");
  sba::ListLv L{d_offsets, list_nullable ? d_list_validity : nullptr, item_nullable ? d_child_validity : nullptr,
                n_rows, (uint32_t)step, list_nullable ? 1u : 0u, item_nullable ? 1u : 0u, d_heads, head_slot, d_hlen,
                d_levels};
  const uint32_t lds = (uint32_t)((step + 1) * 4);
  ensure_lds_attr(sba::k_enc_list_levels, (int)lds);
  hipLaunchKernelGGL(sba::k_enc_list_levels, dim3((uint32_t)np), dim3(sba::NT), lds, st, L);
  if (const hipError_t e = hipGetLastError(); e != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device list encode launch (step 2)", (int)e);
  if (hipMemcpyAsync(levels.data(), d_levels, np * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device list encode step 2");
  for (uint64_t q = 0; q < np; q++)
    if (levels[q] == ~0ull) return ctx_fail(ctx, SB_E_ARG, "decreasing list offsets");
  const ListPart lp{d_rows_at, d_heads, head_slot, d_hlen, levels.data()};
  return encode_adaptive(ctx, phys, (const uint8_t*)d_child, item_nullable ? d_child_validity : nullptr, rows_at[np],
                         item_nullable, opts, P, d_out, out_cap, out_len, h_metas, np, &lp);
}


__global__ void k_page_offsets(const int64_t* offs, uint64_t n_rows, uint64_t P, uint64_t np, int64_t* out) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= np) out[p] = offs[std::min<uint64_t>(p * P, n_rows)];
}

// per-page slot of a Binary / Utf8 page of n rows and vl value bytes
static uint64_t binary_slot_bytes(uint64_t n, uint64_t vl, int ow, int nullable) {
  const uint64_t pre = nullable ? 4 + 10 + (n + 7) / 8 : 0;
  return (pre + 256 + 2 * (n + 1) * ow + 32 + stream_bound(n, 4, 1) + 10 * n + 8192 + 3 * vl + 15) & ~15ull;
}

uint64_t binary_device_bound(uint64_t n_rows, uint64_t values_len, int ow, int nullable, uint64_t P) {
  if (!P) return 0;
  const uint64_t pages = (n_rows + P - 1) / P;
  return pages * binary_slot_bytes(P, 0, ow, nullable) + 3 * values_len + 64;
}

int encode_binary_adaptive(sb_ctx* ctx, int phys, const uint8_t* d_values, uint64_t values_len,
                           const int64_t* d_offsets, const uint8_t* d_validity, uint64_t n_rows, int nullable,
                           const sb_write_options* opts, uint64_t P, uint8_t* d_out, uint64_t out_cap,
                           uint64_t* out_len, sb_page_meta* h_metas, uint64_t np) {
  const int ow = (phys == SB_T_BINARY || phys == SB_T_UTF8) ? 4 : (phys == SB_T_LARGE_BINARY || phys == SB_T_LARGE_UTF8) ? 8 : 0;
  if (!ow) return SB_E_NYI;
  const sba::Opts o{opts->default_codec, opts->has_ratio, opts->ratio, opts->forbidden_mask, opts->forced_codec};
  const bool stats = sba::needs_stats(o, o.forbidden);
  const bool big = P > sba::kMaxRows;  // (work area in HBM, as encode_adaptive's)
  if (big && P > 0x7FFFFFFFull) return SB_E_NYI;
  // rows / ids (32 P + 64 bytes), then roaring_multi's 4 u32 per container key
  const uint64_t scr = (32 * P + 64 + 16 * ((P + 65535) >> 16) + 255) & ~255ull;
  const uint64_t gwb = big ? big_work_bytes(P, stats) : 0;
  const uint64_t maxpp = batch_pages(np, scr + gwb);
  hipStream_t st = (hipStream_t)sb_ctx_stream(ctx);
  // value bytes of every page from the offsets at the page boundaries
  int64_t* d_po = (int64_t*)ctx_scratch(ctx, (np + 1) * 8, 3);
  if (!d_po) return ctx_fail(ctx, SB_E_DEVICE, "device encode step 5");
  std::vector<int64_t> po(np + 1);
  hipLaunchKernelGGL(k_page_offsets, dim3((uint32_t)((np + 256) / 256)), dim3(256), 0, st, d_offsets, n_rows, P, np, d_po);
  if (hipMemcpyAsync(po.data(), d_po, (np + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device encode step 6");
  // batches of pages whose slots fit ~1 GiB; slot offsets relative to the batch start
  std::vector<uint64_t> soff;
  std::vector<std::pair<uint64_t, uint64_t>> batches;  // (first page, index of its slot_offs)
  uint64_t acc = 0;
  for (uint64_t p = 0; p < np; p++) {
    const uint64_t n = std::min<uint64_t>(P, n_rows - p * P);
    if (po[p + 1] < po[p]) return SB_E_ARG;
    const uint64_t sb = binary_slot_bytes(n, (uint64_t)(po[p + 1] - po[p]), ow, nullable);
    if (batches.empty() || (acc + sb > (1ull << 30) && p > batches.back().first) || p - batches.back().first >= maxpp) {
      if (!batches.empty()) soff.push_back(acc);
      batches.push_back({p, soff.size()});
      acc = 0;
    }
    soff.push_back(acc);
    acc += sb;
  }
  soff.push_back(acc);
  uint64_t max_batch = 0;
  for (size_t b = 0; b < batches.size(); b++) {
    const uint64_t end = b + 1 < batches.size() ? soff[batches[b + 1].second - 1] : soff.back();
    max_batch = std::max(max_batch, end);
  }
  const uint32_t work = big ? 0u : adaptive_work_bytes(P, o);
  const uint32_t lds = (big ? sbc::kLz4WaveLds : work) + sba::kSample * 8 + sba::kSample / 8 + 16;
  uint8_t* slots = (uint8_t*)ctx_scratch(ctx, max_batch + 256, 0);
  const uint32_t maxn = (uint32_t)std::min<uint64_t>(np, maxpp);
  uint8_t* scratch = (uint8_t*)ctx_scratch(ctx, maxn * scr, 1);
  uint64_t* meta = (uint64_t*)ctx_scratch(ctx, (2 * np + 2) * 8 + np * 4 + 8 + soff.size() * 8, 2);
  uint8_t* gwork = big ? (uint8_t*)ctx_scratch(ctx, maxn * gwb, 4) : nullptr;
  if (!slots || !scratch || !meta || (big && !gwork)) return ctx_fail(ctx, SB_E_DEVICE, "device encode step 7");
  uint64_t* sizes = meta;
  uint64_t* offs = meta + np;
  uint32_t* status = (uint32_t*)(meta + 2 * np + 2);
  uint64_t* d_soff = (uint64_t*)((uint8_t*)meta + (2 * np + 2) * 8 + ((np * 4 + 7) & ~7ull));
  if (hipMemcpyAsync(d_soff, soff.data(), soff.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemsetAsync(offs + np, 0, 8, st) != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device encode step 8");
  for (size_t b = 0; b < batches.size(); b++) {
    const uint64_t b0 = batches[b].first;
    const uint64_t b1 = b + 1 < batches.size() ? batches[b + 1].first : np;
    sba::AdArgs a{d_values, d_validity, n_rows, (uint32_t)P, (uint32_t)b0, (uint32_t)(b1 - b0), nullable, o,
                  opts->seed, slots, 0, scratch, scr, work, gwork, gwb, sizes, status, offs, d_out, out_cap, (uint32_t)np,
                  d_offsets, values_len, ow, d_soff + batches[b].second};
    if (ow == 4) launch_bin<4>(a, lds, st);
    else launch_bin<8>(a, lds, st);
    hipLaunchKernelGGL(sba::k_enc_offsets, dim3(1), dim3(sba::NT), 0, st, a);
    hipLaunchKernelGGL(sba::k_enc_compact, dim3(a.n_batch), dim3(sba::NT), 0, st, a);
    if (const hipError_t e = hipGetLastError(); e != hipSuccess)
      return ctx_fail(ctx, SB_E_DEVICE, "device encode launch (step 9)", (int)e);
  }
  std::vector<uint64_t> sz(2 * np + 1);
  std::vector<uint32_t> stv(np);
  if (hipMemcpyAsync(sz.data(), sizes, (2 * np + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(stv.data(), status, np * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ctx_fail(ctx, SB_E_DEVICE, "device encode step 10");
  for (uint64_t p = 0; p < np; p++) {
    if (stv[p] == sba::E_NYI) return SB_E_NYI;
    if (stv[p] == sba::E_CAP) return SB_E_ARG;
    if (stv[p]) return SB_E_OUT_OF_SPEC;
  }
  *out_len = sz[2 * np];
  for (uint64_t p = 0; p < np; p++) h_metas[p] = sb_page_meta{sz[p], std::min<uint64_t>(P, n_rows - p * P)};
  return SB_OK;
}

}  // namespace sb

extern "C" uint64_t sb_encode_binary_device_bound(int32_t physical_type, uint64_t n_rows, uint64_t values_len,
                                                  int32_t nullable, uint64_t max_page_rows) {
  const int ow = (physical_type == SB_T_BINARY || physical_type == SB_T_UTF8) ? 4
                 : (physical_type == SB_T_LARGE_BINARY || physical_type == SB_T_LARGE_UTF8) ? 8 : 0;
  const uint64_t P = max_page_rows ? std::min(max_page_rows, n_rows) : n_rows;
  if (!ow) return 0;
  return sb::binary_device_bound(n_rows, values_len, ow, nullable, P);
}

extern "C" sb_status sb_encode_binary_column_device(sb_ctx* ctx, int32_t physical_type, const uint8_t* d_values,
                                                    uint64_t values_len, const int64_t* d_offsets,
                                                    const uint8_t* d_validity, uint64_t n_rows, int32_t nullable,
                                                    const sb_write_options* opts, uint64_t max_page_rows,
                                                    uint8_t* d_out, uint64_t out_capacity, uint64_t* out_len,
                                                    sb_page_meta* h_metas, uint64_t metas_cap, uint64_t* n_pages) {
  if (!ctx || !opts || !out_len || !n_pages || (n_rows && (!d_offsets || !d_out)) || (nullable && !d_validity))
    return SB_E_ARG;
  const uint64_t P = max_page_rows ? std::min(max_page_rows, n_rows) : n_rows;
  const uint64_t np = n_rows ? (n_rows + P - 1) / P : 0;
  *n_pages = np;
  *out_len = 0;
  if (np > metas_cap || (!h_metas && np)) return SB_E_ARG;
  if (!np) return SB_OK;
  if (hipSetDevice(sb_ctx_device(ctx)) != hipSuccess) return (sb_status)sb::ctx_fail(ctx, SB_E_DEVICE, "hipSetDevice");
  return (sb_status)sb::encode_binary_adaptive(ctx, physical_type, d_values, values_len, d_offsets, d_validity, n_rows,
                                               nullable, opts, P, d_out, out_capacity, out_len, h_metas, np);
}

#ifdef SB_ENC_PHASES
extern "C" int sb_debug_enc_phases(uint64_t* host, uint64_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sba::sb_enc_phase), (n < 4096 * 12 ? n : 4096 * 12) * 8) == hipSuccess ? 0 : -1;
}
#endif
