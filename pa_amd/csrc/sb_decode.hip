// sb_decode.hip -- batched page decode of fixed-width strawboat columns on
// MI355X (gfx950).
//
// One 256-thread workgroup decodes one page: the page bytes are staged into
// LDS with 16-byte loads, the validity prefix and the value stream header are
// parsed from LDS, and the codec body is expanded straight into the Arrow
// buffers in HBM.  Restates, per page:
//   IntegerIter::deserialize / read_integer   read/array/integer.rs:68-88, 210-238
//   DoubleIter::deserialize / read_double     read/array/double.rs:68-88, 210-238
//   read_validity                             read/read_basic.rs:36-63
//   decompress_integer / decompress_double    compression/integer/mod.rs:72-117,
//                                             compression/double/mod.rs:69-114
//   Bitpacking / DeltaBitpacking              compression/integer/bp.rs:67-86,
//                                             compression/integer/delta_bp.rs:69-92
//   RLE                                       compression/integer/rle.rs:106-134
//   OneValue                                  compression/integer/one_value.rs:77-94
//   Dict                                      compression/integer/dict.rs:75-103
//   Freq                                      compression/integer/freq.rs:88-123
// Integer/byte work only: no MFMA.  Bound: HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>

#include "sb_internal.h"

namespace sbk {

using namespace sb;

#ifndef SB_BLOCK
#define SB_BLOCK 256
#endif
#ifndef SB_LOAD_NT
#define SB_LOAD_NT 1
#endif
#ifndef SB_STORE_NT
#define SB_STORE_NT 1
#endif
#ifndef SB_LDS_DMA
#define SB_LDS_DMA 1
#endif
constexpr int NT = SB_BLOCK;
constexpr int NW = NT / 64;
constexpr uint32_t kWinBlocks = 64;  // bitpack blocks per header walk window
constexpr uint32_t kMaxConts = 16;   // roaring containers handled per page
constexpr uint32_t kMaxBitmapConts = 4;  // of which bitmap containers (card > 4096)
constexpr uint32_t kRleFastRows = 8192;  // RLE pages up to this many rows use the run-start bitmap

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int W> struct VT { using T = uint32_t; };
template <> struct VT<8> { using T = uint64_t; };

// ---------------------------------------------------------------------------
// byte sources
// ---------------------------------------------------------------------------
// Page staged in LDS at byte `base` of the dynamic LDS words.  The staging
// buffer carries kStagePad bytes of slack so word-granular over-reads are safe.
struct LdsSrc {
  const uint32_t* w;
  uint32_t base;
  __device__ __forceinline__ uint32_t u8(uint32_t p) const {
    p += base;
    return (w[p >> 2] >> ((p & 3) * 8)) & 0xFFu;
  }
  __device__ __forceinline__ uint32_t u32(uint32_t p) const {
    p += base;
    uint32_t i = p >> 2;
    return __builtin_amdgcn_alignbyte(w[i + 1], w[i], p & 3);
  }
  __device__ __forceinline__ LdsSrc at(uint32_t o) const { return LdsSrc{w, base + o}; }
  __device__ __forceinline__ uint64_t u64(uint32_t p) const {
    p += base;
    uint32_t i = p >> 2, sh = p & 3;
    uint32_t a = w[i], b = w[i + 1], c = w[i + 2];
    return (uint64_t)__builtin_amdgcn_alignbyte(b, a, sh) |
           ((uint64_t)__builtin_amdgcn_alignbyte(c, b, sh) << 32);
  }
  // the 4 lane words at p and (if need_hi) the 4 at p + 16, unaligned
  __device__ __forceinline__ void quad_words(uint32_t p, bool need_hi, uint32_t* d8) const {
    p += base;
    uint32_t i = p >> 2, sh = p & 3;
    uint32_t d[9];
#pragma unroll
    for (int k = 0; k < 9; k++) d[k] = w[i + k];
#pragma unroll
    for (int k = 0; k < 8; k++) d8[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
  }
};

// Page read straight from HBM (pages larger than the LDS stage).  Unaligned
// words are assembled from the aligned dwords that contain them, so no read
// leaves the bytes the page owns.
struct GlbSrc {
  typedef const __attribute__((address_space(1))) uint8_t g8;
  typedef const __attribute__((address_space(1))) uint32_t g32;
  g8* p;  // global address space: global_load, not flat
  __device__ __forceinline__ GlbSrc() : p(nullptr) {}
  __device__ __forceinline__ GlbSrc(const uint8_t* q) : p((g8*)q) {}
  __device__ __forceinline__ GlbSrc(g8* q) : p(q) {}
  __device__ __forceinline__ GlbSrc at(uint32_t o) const { return GlbSrc{p + o}; }
  __device__ __forceinline__ uint32_t u8(uint32_t i) const { return p[i]; }
  __device__ __forceinline__ uint32_t u32(uint32_t i) const {
    const uintptr_t a = (uintptr_t)(p + i);
    g32* q = (g32*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    if (sh == 0) return q[0];
    return __builtin_amdgcn_alignbyte(q[1], q[0], sh);
  }
  __device__ __forceinline__ uint64_t u64(uint32_t i) const {
    return (uint64_t)u32(i) | ((uint64_t)u32(i + 4) << 32);
  }
  __device__ __forceinline__ void quad_words(uint32_t pos, bool need_hi, uint32_t* d8) const {
#pragma unroll
    for (int k = 0; k < 4; k++) d8[k] = u32(pos + 4 * k);
    if (need_hi) {
#pragma unroll
      for (int k = 0; k < 4; k++) d8[4 + k] = u32(pos + 16 + 4 * k);
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) d8[4 + k] = 0;
    }
  }
};

template <int W, class Src>
__device__ __forceinline__ typename VT<W>::T ldv(const Src& s, uint32_t p) {
  if constexpr (W == 8) return s.u64(p);
  else if constexpr (W == 4) return s.u32(p);
  else if constexpr (W == 2) return s.u32(p) & 0xFFFFu;
  else return s.u8(p);
}

// ---------------------------------------------------------------------------
// per-workgroup shared state
// ---------------------------------------------------------------------------
struct Stream {
  uint32_t codec, body, csize, n;
};

struct Shared {
  uint32_t err;
  uint32_t walk_off;
  uint32_t blk_off[kWinBlocks];
  uint32_t blk_bits[kWinBlocks];
  uint64_t wsum[NW];
  uint32_t rle_start[NT + 1];
  uint32_t rle_c;
  uint32_t rle_R;
  uint32_t rle_flags;  // bit0 = a run ends exactly at n, bit1 = a run overshoots n, bit2 = zero-count run
  uint32_t rle_bits[kRleFastRows / 32];  // bit r set <=> a run starts at row r
  uint16_t rle_pref[kRleFastRows / 32];  // set bits before word w
  // page header
  uint32_t has_valid, vb_pos, vb_bytes;
  Stream top;
  Stream sub;  // the leaf stream at the bottom of the cascade
  uint32_t chain;
  uint32_t defer;
  // Dict
  uint32_t dict_k, dict_off;
  // Freq: the roaring bitmap's container tables (roaring_build), in the LDS
  // arrays below when they fit, else in the page's HBM region
  uint64_t freq_top;
  uint32_t n_conts;
  uint32_t roar_r, roar_bm, roar_pending;  // position and size of the portable bitmap; tables still to build
  uint32_t roar_lds, cp_lds;              // tables / checkpoints in the arrays below (else the region)
  uint32_t* rkey;                         // container keys
  uint32_t* rdata;                        // source position of each container's data
  uint32_t* rpre;                         // exceptions before each container (n_conts + 1)
  uint32_t* rbm;                          // bitmap container index into rcp, or ~0u for array containers
  uint16_t* rcp;                          // per bitmap container: set bits before each 16-word group (64)
  uint32_t cont_key[kMaxConts];
  uint32_t cont_data[kMaxConts];
  uint32_t cont_prefix[kMaxConts + 1];
  uint32_t cont_bm[kMaxConts];
  uint16_t cont_cp[kMaxBitmapConts][64];
};

__device__ __forceinline__ void set_err(Shared& sh, uint32_t code) { atomicMax(&sh.err, code); }

// Block-wide exclusive scan (sum) of one value per thread; *total = block sum.
template <class T>
__device__ __forceinline__ T block_excl_scan(T v, Shared& sh, T* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh.wsum[wv] = (uint64_t)x;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NW; k++) {
    T s = (T)sh.wsum[k];
    if (k < wv) pre += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// ---------------------------------------------------------------------------
// output sinks
// ---------------------------------------------------------------------------
template <class V>
__device__ __forceinline__ void st_out(V* p, V v) {
#if SB_STORE_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

template <int W>
struct GSink {
  uint8_t* base;  // page row 0
  bool vec;       // quads store as one 16-byte vector (W >= 4: page row 0 dword-aligned; else 4*W aligned)
  using T = typename VT<W>::T;
  __device__ __forceinline__ void put(uint32_t row, T v) const {
    if constexpr (W == 8) ((uint64_t*)base)[row] = v;
    else if constexpr (W == 4) ((uint32_t*)base)[row] = v;
    else if constexpr (W == 2) ((uint16_t*)base)[row] = (uint16_t)v;
    else base[row] = (uint8_t)v;
  }
  __device__ __forceinline__ void put4(uint32_t row, const T* v, uint32_t nvalid) const {
    if (nvalid == 4 && vec) {
      if constexpr (W == 8) {
        u32x4* p = (u32x4*)(base + (size_t)row * 8);
        st_out(p, u32x4{(uint32_t)v[0], (uint32_t)(v[0] >> 32), (uint32_t)v[1], (uint32_t)(v[1] >> 32)});
        st_out(p + 1, u32x4{(uint32_t)v[2], (uint32_t)(v[2] >> 32), (uint32_t)v[3], (uint32_t)(v[3] >> 32)});
      } else if constexpr (W == 4) {
        st_out((u32x4*)(base + (size_t)row * 4), u32x4{v[0], v[1], v[2], v[3]});
      } else if constexpr (W == 2) {
        *(uint2*)(base + (size_t)row * 2) = make_uint2((v[0] & 0xFFFF) | (v[1] << 16), (v[2] & 0xFFFF) | (v[3] << 16));
      } else {
        *(uint32_t*)(base + row) = (v[0] & 0xFF) | ((v[1] & 0xFF) << 8) | ((v[2] & 0xFF) << 16) | (v[3] << 24);
      }
    } else {
      for (uint32_t l = 0; l < nvalid; l++) put(row + l, v[l]);
    }
  }
};

// ---------------------------------------------------------------------------
// Bitpacking (BitPacker4x layout, bitpacking 0.8.0): header walk
// ---------------------------------------------------------------------------
// Block k of a stream is [u8 b][16*b bytes]; its header offset depends on
// every earlier b.  Wave 0 walks `cnt` headers speculatively: lane j guesses
// block (done + j) sits (j * (1 + 16*b0)) bytes on, i.e. that b stays b0.
// The first lane that reads a different b ends the confirmed prefix (its own
// offset is still right); the next round restarts there.  Constant-width
// pages need one round per 64 blocks; the worst case is one block per round.
template <class Src>
__device__ void bp_walk(const Src& s, Shared& sh, uint32_t end, uint32_t cnt) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t off = sh.walk_off, done = 0;
  while (done < cnt) {
    if (off >= end) { if (lane == 0) set_err(sh, ST_IO); return; }
    uint32_t b0 = s.u8(off);
    if (b0 > 32) { if (lane == 0) set_err(sh, ST_OUT_OF_SPEC); return; }
    uint32_t step = 1 + 16 * b0;
    uint32_t k = done + lane;
    uint32_t g = off + lane * step;
    bool inb = k < cnt;
    uint32_t bj = (inb && g < end) ? s.u8(g) : 0xFFFFFFFFu;
    unsigned long long mism = __ballot(inb && bj != b0);
    uint32_t m = mism ? (uint32_t)__builtin_ctzll(mism) : min(64u, cnt - done);
    if (lane < m) {
      sh.blk_off[k] = g + 1;
      sh.blk_bits[k] = b0;
    }
    done += m;
    off += m * step;
  }
  if (off > end) { if (lane == 0) set_err(sh, ST_IO); return; }
  if (lane == 0) sh.walk_off = off;
}

// 4 values of quad i of a block whose payload starts at P with width b.
template <class Src>
__device__ __forceinline__ void bp_quad(const Src& s, uint32_t P, uint32_t b, uint32_t i, uint32_t* v) {
  if (b == 0) { v[0] = v[1] = v[2] = v[3] = 0; return; }
  uint32_t bit = i * b, w = bit >> 5, sft = bit & 31;
  uint32_t mask = b == 32 ? 0xFFFFFFFFu : ((1u << b) - 1);
  uint32_t d[8];
  s.quad_words(P + 16 * w, sft + b > 32, d);
#pragma unroll
  for (int l = 0; l < 4; l++) v[l] = __builtin_amdgcn_alignbit(d[4 + l], d[l], sft) & mask;
}

// ---------------------------------------------------------------------------
// RLE: runs of (u32 count, T value)
// ---------------------------------------------------------------------------
// Preparation: thread t owns runs [t*c, (t+1)*c); an exclusive scan of the
// per-thread count sums gives each thread chunk's first row.  Validity
// follows rle.rs:115-132: decoding stops at the first run whose end reaches
// n; it must land exactly on n (array/integer.rs:81 assert).
template <int SW, class Src>
__device__ void rle_prepare(const Src& s, Shared& sh, const Stream& st) {
  const uint32_t tid = threadIdx.x;
  const uint32_t runsz = 4 + SW;
  const uint32_t R = st.csize / runsz;
  const uint32_t c = (R + NT - 1) / NT;
  const bool small = st.n <= kRleFastRows;
  if (small)
    for (uint32_t w = tid; w < kRleFastRows / 32; w += NT) sh.rle_bits[w] = 0;
  uint32_t r0 = min(R, tid * c), r1 = min(R, r0 + c);
  uint64_t sum = 0;
  for (uint32_t r = r0; r < r1; r++) sum += s.u32(st.body + r * runsz);
  uint64_t tot;
  uint64_t start = block_excl_scan<uint64_t>(sum, sh, &tot);  // (syncs: the zeroing above is visible)
  uint32_t flags = 0;
  uint64_t acc = start;
  if (start < st.n) {
    for (uint32_t r = r0; r < r1; r++) {
      const uint64_t b = acc;
      const uint32_t cnt = s.u32(st.body + r * runsz);
      acc += cnt;
      if (cnt == 0) flags |= 4;
      if (acc == st.n) flags |= 1;
      if (acc > st.n) flags |= 2;
      if (small) atomicOr(&sh.rle_bits[b >> 5], 1u << (b & 31));
      if (acc >= st.n) break;
    }
  }
  sh.rle_start[tid] = (uint32_t)min<uint64_t>(start, 0xFFFFFFFFull);
  if (tid == 0) {
    sh.rle_start[NT] = (uint32_t)min<uint64_t>(tot, 0xFFFFFFFFull);
    sh.rle_c = c;
    sh.rle_R = R;
    sh.rle_flags = 0;
  }
  __syncthreads();
  if (flags) atomicOr(&sh.rle_flags, flags);
  __syncthreads();
  if (tid == 0 && st.n > 0) {
    const uint32_t f = sh.rle_flags;
    if ((f & 2) || !(f & 1)) set_err(sh, (f & 2) ? ST_OUT_OF_SPEC : ST_IO);
  }
  if (small) {  // prefix popcount of the run-start bitmap (kRleFastRows/32 words)
    constexpr uint32_t kWords = kRleFastRows / 32;
    constexpr uint32_t kPer = kWords >= (uint32_t)NT ? kWords / NT : 1;
    const uint32_t w0 = tid * kPer;
    uint32_t pc[kPer], tsum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      pc[k] = w0 + k < kWords ? __popc(sh.rle_bits[w0 + k]) : 0u;
      tsum += pc[k];
    }
    uint32_t t;
    uint32_t pre = block_excl_scan<uint32_t>(tsum, sh, &t);
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      if (w0 + k < kWords) sh.rle_pref[w0 + k] = (uint16_t)pre;
      pre += pc[k];
    }
  }
  __syncthreads();
}

// Run containing row `row` (row < n): binary search over the thread-chunk
// starts, then a linear walk inside the chunk.  Returns run index and fills
// [rs, re) = its row span.
template <int SW, class Src>
__device__ __forceinline__ uint32_t rle_find(const Src& s, const Shared& sh, const Stream& st, uint32_t row,
                                             uint32_t* rs, uint32_t* re) {
  uint32_t lo = 0, hi = NT;  // largest t with rle_start[t] <= row
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (sh.rle_start[mid] <= row) lo = mid; else hi = mid;
  }
  const uint32_t runsz = 4 + SW;
  uint32_t r = lo * sh.rle_c;
  uint32_t acc = sh.rle_start[lo];
  for (;;) {
    uint32_t cnt = s.u32(st.body + r * runsz);
    if (row < acc + cnt || r + 1 >= sh.rle_R) { *rs = acc; *re = acc + cnt; return r; }
    acc += cnt;
    r++;
  }
}

// ---------------------------------------------------------------------------
// Stream driver: expands one leaf value stream (None, OneValue, RLE,
// Bitpacking, DeltaBitpacking) of n values of width SW and hands every quad
// of consecutive values to fn(first_index, v[4], nvalid).  All threads of the
// workgroup call this uniformly.  Dict and Freq are handled one level up.
// ---------------------------------------------------------------------------
template <int SW, class Src, class Fn>
__device__ __forceinline__ void run_leaf(const Src& s, Shared& sh, const Stream st, Fn&& fn) {
  using T = typename VT<SW>::T;
  const uint32_t tid = threadIdx.x;
  const uint32_t nq = (st.n + 3) >> 2;
  switch (st.codec) {
    case 0: {  // None: raw LE values (basic.rs:68-71 copy_from_slice)
      if (st.csize != st.n * SW) { if (tid == 0) set_err(sh, ST_OUT_OF_SPEC); return; }
      for (uint32_t q = tid; q < nq; q += NT) {
        T v[4];
        uint32_t nv = min(4u, st.n - 4 * q);
#pragma unroll
        for (uint32_t l = 0; l < 4; l++) v[l] = l < nv ? ldv<SW>(s, st.body + (4 * q + l) * SW) : (T)0;
        fn(4 * q, v, nv);
      }
      return;
    }
    case 12: {  // OneValue
      if (st.csize < SW) { if (tid == 0) set_err(sh, ST_IO); return; }
      T x = ldv<SW>(s, st.body);
      for (uint32_t q = tid; q < nq; q += NT) {
        T v[4] = {x, x, x, x};
        fn(4 * q, v, min(4u, st.n - 4 * q));
      }
      return;
    }
    case 10: {  // RLE
      rle_prepare<SW>(s, sh, st);
      if (sh.err) return;
      const uint32_t runsz = 4 + SW;
      if (st.n <= kRleFastRows && !(sh.rle_flags & 4)) {
        // run of row r = (run starts at rows <= r) - 1: one bitmap word and one
        // prefix per quad, no search
        for (uint32_t q = tid; q < nq; q += NT) {
          const uint32_t row = 4 * q, nv = min(4u, st.n - row);
          const uint32_t word = sh.rle_bits[row >> 5], base = sh.rle_pref[row >> 5];
          T v[4];
#pragma unroll
          for (uint32_t l = 0; l < 4; l++) {
            const uint32_t b = (row + l) & 31;
            const uint32_t m = b == 31 ? 0xFFFFFFFFu : ((2u << b) - 1);
            const uint32_t r = base + __popc(word & m) - 1;
            v[l] = ldv<SW>(s, st.body + r * runsz + 4);
          }
          fn(row, v, nv);
        }
        return;
      }
      for (uint32_t q = tid; q < nq; q += NT) {
        uint32_t row = 4 * q, nv = min(4u, st.n - row);
        uint32_t rs, re;
        uint32_t r = rle_find<SW>(s, sh, st, row, &rs, &re);
        T x = ldv<SW>(s, st.body + r * runsz + 4);
        T v[4];
#pragma unroll
        for (uint32_t l = 0; l < 4; l++) {
          if (l < nv && row + l >= re) {
            // advance to the run covering row + l (zero-count runs skipped)
            do {
              r++;
              rs = re;
              re = rs + s.u32(st.body + r * runsz);
            } while (row + l >= re && r + 1 < sh.rle_R);
            x = ldv<SW>(s, st.body + r * runsz + 4);
          }
          v[l] = x;
        }
        fn(row, v, nv);
      }
      return;
    }
    case 14:
    case 15: {  // Bitpacking / DeltaBitpacking (T must be 4 bytes, n % 128 == 0)
      if (SW != 4 || (st.n & 127)) { if (tid == 0) set_err(sh, ST_OUT_OF_SPEC); return; }
      const bool delta = st.codec == 15;
      const uint32_t nblk = st.n >> 7;
      const uint32_t end = st.body + st.csize;
      if (tid == 0) sh.walk_off = st.body;
      __syncthreads();
      uint32_t carry = 0;
      for (uint32_t kb = 0; kb < nblk; kb += kWinBlocks) {
        const uint32_t cnt = min(kWinBlocks, nblk - kb);
        if (tid < 64) bp_walk(s, sh, end, cnt);
        __syncthreads();
        if (sh.err) return;
        const uint32_t nqw = cnt * 32;
        for (uint32_t j = 0; j < (nqw + NT - 1) / NT; j++) {
          const uint32_t q = j * NT + tid;
          uint32_t v[4] = {0, 0, 0, 0};
          const bool act = q < nqw;
          if (act) bp_quad(s, sh.blk_off[q >> 5], sh.blk_bits[q >> 5], q & 31, v);
          if (delta) {
            // wrapping inclusive prefix over the whole page (delta_bp.rs:76-90:
            // each block starts from the previous block's last value)
            v[1] += v[0];
            v[2] += v[1];
            v[3] += v[2];
            uint32_t tot;
            uint32_t pre = block_excl_scan<uint32_t>(act ? v[3] : 0u, sh, &tot) + carry;
#pragma unroll
            for (int l = 0; l < 4; l++) v[l] += pre;
            carry += tot;
          }
          if (act) {
            T tv[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
            fn(kb * 128 + 4 * q, tv, 4u);
          }
        }
        __syncthreads();
      }
      return;
    }
    case 1:
    case 2:
    case 3:   // LZ4 / Zstd / Snappy: expanded first by the deferred / inflate passes, never a leaf here
    case 11:  // Dict / Freq nested below another Dict / Freq
    case 13:
    case 16:  // Patas (float streams)
      if (tid == 0) set_err(sh, ST_NYI);
      return;
    default:
      if (tid == 0) set_err(sh, ST_OUT_OF_SPEC);
      return;
  }
}

// Parse a nested [codec][csize][usize] header at p (bounded by end).
template <class Src>
__device__ __forceinline__ bool parse_stream(const Src& s, uint32_t p, uint32_t end, uint32_t n, Stream* st) {
  if (p + 9 > end) return false;
  st->codec = s.u8(p);
  st->csize = s.u32(p + 1);
  st->body = p + 9;
  st->n = n;
  return st->csize <= end - st->body;
}

// Roaring select: row of exception i.  Array containers index directly;
// bitmap containers find the 16-word group by its checkpoint, then the word by
// popcounts, then the bit.  The container is found by binary search over the
// exception prefix (a 1M-row page has 16 containers, a 100M-row one 1526).
template <class Src>
__device__ __forceinline__ uint32_t roaring_select(const Src& s, const Shared& sh, uint32_t i) {
  typedef const __attribute__((address_space(1))) uint32_t g32;
  typedef const __attribute__((address_space(1))) uint16_t g16;
  uint32_t c = 0, hi = sh.n_conts, j, bmi, key, data;
  if (sh.roar_lds) {  // tables in Shared (ds_ reads)
    while (hi - c > 1) {
      const uint32_t mid = (c + hi) >> 1;
      if (sh.cont_prefix[mid] <= i) c = mid; else hi = mid;
    }
    j = i - sh.cont_prefix[c];
    bmi = sh.cont_bm[c];
    key = sh.cont_key[c];
    data = sh.cont_data[c];
  } else {  // tables in the page's HBM region (global_ reads)
    g32* pre = (g32*)sh.rpre;
    while (hi - c > 1) {
      const uint32_t mid = (c + hi) >> 1;
      if (pre[mid] <= i) c = mid; else hi = mid;
    }
    j = i - pre[c];
    bmi = ((g32*)sh.rbm)[c];
    key = ((g32*)sh.rkey)[c];
    data = ((g32*)sh.rdata)[c];
  }
  if (bmi == ~0u) return (key << 16) | (s.u32(data + 2 * j) & 0xFFFFu);
  uint32_t g = 0;
  if (sh.cp_lds) {
    for (uint32_t step = 32; step; step >>= 1)
      if (g + step < 64 && sh.cont_cp[bmi][g + step] <= j) g += step;
    j -= sh.cont_cp[bmi][g];
  } else {
    g16* cp = (g16*)sh.rcp + 64 * bmi;
    for (uint32_t step = 32; step; step >>= 1)
      if (g + step < 64 && cp[g + step] <= j) g += step;
    j -= cp[g];
  }
  uint32_t w = 16 * g;
  uint64_t word = s.u64(data + 8 * w);
  for (uint32_t pc = __popcll(word); pc <= j && w + 1 < 1024; pc = __popcll(word)) {
    j -= pc;
    word = s.u64(data + 8 * (++w));
  }
  for (uint32_t t = 0; t < j; t++) word &= word - 1;  // drop the j lowest set bits
  return (key << 16) | (w * 64 + (uint32_t)__builtin_ctzll(word));
}

// ---------------------------------------------------------------------------
// validity: copy the page's def-level bitmap to bit offset row_off
// ---------------------------------------------------------------------------
template <class Src>
__device__ __forceinline__ void write_validity(const Src& s, uint32_t vb, uint32_t n, uint64_t row_off, uint32_t* out) {
  if (n == 0) return;
  const uint64_t fw = row_off >> 5, lw = (row_off + n - 1) >> 5;
  for (uint64_t w = fw + threadIdx.x; w <= lw; w += NT) {
    int64_t pb = (int64_t)(w * 32) - (int64_t)row_off;  // page bit of word bit 0
    uint32_t v;
    if (pb >= 0) v = (uint32_t)(s.u64(vb + (uint32_t)(pb >> 3)) >> (pb & 7));
    else v = s.u32(vb) << (uint32_t)(-pb);
    // keep word bits k with 0 <= pb + k < n
    uint32_t lo = pb < 0 ? (uint32_t)(-pb) : 0u;
    int64_t hi_ex = (int64_t)n - pb;  // word bits < hi_ex are inside the page
    uint32_t hi = hi_ex >= 32 ? 32u : (uint32_t)hi_ex;
    uint32_t m = (hi == 32 ? 0xFFFFFFFFu : ((1u << hi) - 1)) & (0xFFFFFFFFu << lo);
    if (m == 0xFFFFFFFFu) out[w] = v;
    else atomicOr(&out[w], v & m);
  }
}

// ---------------------------------------------------------------------------
// the page kernel
// ---------------------------------------------------------------------------
// Parses the header of a roaring portable bitmap of bm bytes at r (roaring
// 0.10.1 serialize_into: cookie 12346, container count, per container
// (key, card - 1), then per container its data offset; array containers of
// u16 values, bitmap containers of 1024 u64 words; cookie 12347 run
// containers are not written by 0.10.1 and report NYI).  Thread 0; *total =
// cardinality.  The container tables are built afterwards by the whole
// workgroup (roaring_build).
template <class Src>
__device__ __forceinline__ bool parse_roaring(const Src& s, Shared& sh, uint32_t r, uint32_t bm, uint32_t* total) {
  if (bm < 8) { set_err(sh, ST_IO); return false; }
  if (s.u32(r) != 12346) { set_err(sh, ST_NYI); return false; }
  const uint32_t nc = s.u32(r + 4);
  if (8 + 8 * (uint64_t)nc > bm) { set_err(sh, ST_OUT_OF_SPEC); return false; }
  uint64_t tot = 0;
  for (uint32_t c = 0; c < nc; c++) tot += (s.u32(r + 8 + 4 * c) >> 16) + 1;
  if (tot > 0xFFFFFFFFull) { set_err(sh, ST_OUT_OF_SPEC); return false; }
  sh.n_conts = nc;
  sh.roar_r = r;
  sh.roar_bm = bm;
  sh.roar_pending = 1;
  *total = (uint32_t)tot;
  return true;
}

// Container tables of the bitmap parse_roaring found (all NT threads, after
// a barrier): keys, data positions, exception prefix and the bitmap
// checkpoints, one wave per bitmap container (lane g popcounts words
// 16g..16g+15, a wave scan turns the counts into checkpoints).  In the LDS
// arrays of Shared when nc <= kMaxConts and at most kMaxBitmapConts bitmap
// containers, else in the page's HBM region (`tabs`, room for `cap`
// containers: roar_area_bytes); NYI when neither holds them.
template <class Src>
__device__ __forceinline__ void roaring_build(const Src& s, Shared& sh, uint8_t* tabs, uint32_t cap) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t nc = sh.n_conts, r = sh.roar_r;
  __syncthreads();
  const bool lds = nc <= kMaxConts;
  if (!lds && (!tabs || nc > cap)) {
    if (tid == 0) { set_err(sh, ST_NYI); sh.roar_pending = 0; }
    __syncthreads();
    return;
  }
  uint32_t* key = lds ? sh.cont_key : (uint32_t*)tabs;
  uint32_t* data = lds ? sh.cont_data : key + cap;
  uint32_t* pre = lds ? sh.cont_prefix : data + cap;
  uint32_t* bmx = lds ? sh.cont_bm : pre + cap + 1;
  uint64_t carry = 0;
  uint32_t bcarry = 0;
  for (uint32_t c0 = 0; c0 < nc; c0 += NT) {
    const uint32_t c = c0 + tid;
    uint32_t card = 0, isbm = 0;
    if (c < nc) {
      const uint32_t kc = s.u32(r + 8 + 4 * c);
      card = (kc >> 16) + 1;
      const uint32_t off = s.u32(r + 8 + 4 * nc + 4 * c);
      const uint32_t dbytes = card > 4096 ? 8192u : 2 * card;  // bitmap : array container
      const uint32_t bm = sh.roar_bm;
      if (off > bm || dbytes > bm - off) set_err(sh, ST_OUT_OF_SPEC);
      key[c] = kc & 0xFFFF;
      data[c] = r + off;
      isbm = card > 4096;
    }
    uint64_t t64;
    const uint64_t p = block_excl_scan<uint64_t>(card, sh, &t64) + carry;
    uint32_t bt;
    const uint32_t bp = block_excl_scan<uint32_t>(isbm, sh, &bt) + bcarry;
    if (c < nc) {
      pre[c] = (uint32_t)p;
      bmx[c] = isbm ? bp : ~0u;
    }
    carry += t64;
    bcarry += bt;
  }
  if (tid == 0) pre[nc] = (uint32_t)carry;
  const uint32_t nbm = bcarry;
  const bool cp_lds = nbm <= kMaxBitmapConts;
  uint16_t* cp = cp_lds ? &sh.cont_cp[0][0] : (tabs ? (uint16_t*)(tabs + align16(4 * (4 * (uint64_t)cap + 1))) : nullptr);
  __syncthreads();  // pre / bmx of every container (and any bounds error) visible
  if (!cp || (!cp_lds && nbm > cap)) {
    if (tid == 0) set_err(sh, ST_NYI);
  } else if (!sh.err) {
    // bitmap containers in container order: wave wv takes containers wv, wv + NW, ...
    for (uint32_t c = wv; c < nc; c += NW) {
      const uint32_t bi = bmx[c];
      if (bi == ~0u) continue;
      uint32_t cnt = 0;
#pragma unroll 4
      for (uint32_t w = 0; w < 16; w++) cnt += __popcll(s.u64(data[c] + 8 * (16 * lane + w)));
      uint32_t x = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
      }
      cp[64 * bi + lane] = (uint16_t)(x - cnt);
      if (lane == 63 && x != pre[c + 1] - pre[c]) set_err(sh, ST_OUT_OF_SPEC);
    }
  }
  if (tid == 0) {
    sh.rkey = key;
    sh.rdata = data;
    sh.rpre = pre;
    sh.rbm = bmx;
    sh.rcp = cp;
    sh.roar_lds = lds;
    sh.cp_lds = cp_lds;
    sh.roar_pending = 0;
  }
  __syncthreads();
}

// Parses a Freq body [T top][u32 bm][roaring][exceptions stream] whose value
// width is `vw` (integer/freq.rs:88-123).  Thread 0 only.
template <class Src>
__device__ __forceinline__ bool parse_freq(const Src& s, Shared& sh, const Stream& st, uint32_t vw, Stream* ex) {
  const uint32_t e = st.body + st.csize;
  if (st.body + vw + 4 > e) { set_err(sh, ST_IO); return false; }
  sh.freq_top = vw == 8 ? s.u64(st.body) : vw == 4 ? s.u32(st.body) : vw == 2 ? (s.u32(st.body) & 0xFFFFu) : s.u8(st.body);
  const uint32_t bm = s.u32(st.body + vw), r = st.body + vw + 4;
  if (bm > e - r) { set_err(sh, ST_IO); return false; }
  uint32_t tot;
  if (!parse_roaring(s, sh, r, bm, &tot)) return false;
  if (!parse_stream(s, r + bm, e, tot, ex)) { set_err(sh, ST_IO); return false; }
  return true;
}

// Parses a Dict body [u32 indices stream][u32 k][k * T] (integer/dict.rs:75-103).
template <class Src>
__device__ __forceinline__ bool parse_dict(const Src& s, Shared& sh, const Stream& st, uint32_t vw, Stream* ix) {
  const uint32_t end = st.body + st.csize;
  if (!parse_stream(s, st.body, end, st.n, ix)) { set_err(sh, ST_IO); return false; }
  const uint32_t e = ix->body + ix->csize;
  if (e + 4 > end) { set_err(sh, ST_IO); return false; }
  const uint32_t k = s.u32(e);
  if ((uint64_t)k * vw > end - (e + 4)) { set_err(sh, ST_OUT_OF_SPEC); return false; }
  sh.dict_k = k;
  sh.dict_off = e + 4;
  return true;
}


// ---------------------------------------------------------------------------
// general codecs: wave-level LZ4 / Snappy block decoder
// ---------------------------------------------------------------------------
// LZ4 raw block (basic.rs:87-91 -> liblz4 LZ4_decompress_safe with the exact
// output size) and Snappy raw (basic.rs:99-106, snap 1.1 raw::Decoder).  The
// format is a serial token stream, so one wave decodes one stream and pages
// run side by side, many waves per CU:
//  * input: a window of four 256-byte register blocks (one dword per lane
//    each) slides over the compressed bytes in HBM, prefetching 768 bytes
//    ahead; tokens are parsed in scalar registers (v_readlane at the uniform
//    position) and literal bytes fetched lane-parallel with ds_bpermute;
//  * output: RING mode keeps the last kRing bytes in a per-wave LDS ring and
//    writes each completed kChunk to HBM; match bytes older than the ring
//    are re-read from HBM at device scope (those chunks were written and
//    waited for at least two chunks earlier).  FULL mode keeps the whole
//    output in LDS (the deferred pass decodes from it).
// A match byte i is out[op - off + i] (off >= 64) or out[op - off + i % off],
// which always lies before op: overlapping copies replicate the period.
typedef __attribute__((address_space(3))) uint8_t lds_u8;

#ifndef SB_INF_WPB
#define SB_INF_WPB 4
#endif
#ifndef SB_INF_FAR128
#define SB_INF_FAR128 1  // free matches' far sources: one 16-byte load for their first four dwords
#endif
#ifdef SB_INF_RING4K  // (before round 6) 4 KiB rings, 1 KiB chunks: 6.5 KiB of LDS a wave, six waves a SIMD
constexpr uint32_t kRing = 4096, kChunk = 1024;
#else  // 2 KiB rings, 512-byte chunks: 4.5 KiB of LDS a wave, eight waves a SIMD
constexpr uint32_t kRing = 2048, kChunk = 512;
#endif
constexpr uint32_t kInfWaves = SB_INF_WPB;  // waves (jobs in flight) per k_inflate workgroup

// Far-history reads re-read bytes this wave stored and waited for (vmcnt(0))
// earlier in the same kernel, so workgroup scope suffices: the CU's L1 and
// its XCD's L2 see their own stores (the gfx942/950 memory model needs no
// invalidate for same-CU store -> load).  sc1 (16, device scope) made every
// such read a fabric request of a whole line (FETCH_SIZE, round 3).
#ifndef SB_FAR_AUX
#define SB_FAR_AUX 0
#endif
typedef const __attribute__((address_space(1))) uint32_t gmem_u32;
typedef const __attribute__((address_space(1))) uint8_t gmem_u8;

// (Stream pointers are global-address-space: a flat load is divergent to the
// compiler even at a uniform address, which would push the parse into VGPRs.)
struct WaveWin {
  gmem_u32* g;        // dword-aligned base of the stream
  uint32_t nd;        // dwords of g holding stream bytes
  uint32_t lo;        // byte position (from g) of w0 lane 0, a multiple of 4
  uint32_t w0, w1, w2, w3;  // blocks [lo, lo + 256), ... [lo + 768, lo + 1024)

  // clamped, not predicated: a select on the loaded value would wait for it
  __device__ __forceinline__ uint32_t ld(uint32_t dw) const { return __builtin_nontemporal_load(g + min(dw, nd - 1)); }
  __device__ void init(const uint8_t* start, uint32_t len) {
    g = (gmem_u32*)((uintptr_t)start & ~(uintptr_t)3);
    nd = (((uint32_t)((uintptr_t)start & 3)) + len + 3) >> 2;
    seek((uint32_t)((uintptr_t)start & 3));
  }
  __device__ void seek(uint32_t pos) {
    const uint32_t lane = threadIdx.x & 63;
    lo = pos & ~3u;
    const uint32_t d = (lo >> 2) + lane;
    w0 = ld(d);
    w1 = ld(d + 64);
    w2 = ld(d + 128);
    w3 = ld(d + 192);
  }
  // after slide(pos): pos - lo < 256.  The shift only waits for the load
  // issued one slide earlier; parsing reads w0 / w1 alone.
  __device__ __forceinline__ void slide(uint32_t pos) {
    if (pos - lo < 256) return;
    if (pos - lo >= 512) { seek(pos); return; }
    w0 = w1;
    w1 = w2;
    w2 = w3;
    lo += 256;
    w3 = ld((lo >> 2) + 192 + (threadIdx.x & 63));
  }
  // uniform byte at pos (the caller bounds pos by the stream end)
  __device__ __forceinline__ uint32_t byte(uint32_t pos) const {
    const uint32_t r = pos - lo;
    uint32_t d;
    if (r < 256) d = __builtin_amdgcn_readlane(w0, r >> 2);
    else if (r < 512) d = __builtin_amdgcn_readlane(w1, (r >> 2) - 64);
    else return ((gmem_u8*)g)[pos];  // past the window (long length runs)
    return (d >> ((r & 3) * 8)) & 0xFFu;
  }
  // uniform dword at pos (any alignment), for pos - lo < 504
  __device__ __forceinline__ uint32_t dw(uint32_t i) const {  // window dword i < 128
    return i < 64 ? __builtin_amdgcn_readlane(w0, i) : __builtin_amdgcn_readlane(w1, i - 64);
  }
  __device__ __forceinline__ uint32_t u32at(uint32_t pos) const {
    const uint32_t r = pos - lo, i = r >> 2;
    return __builtin_amdgcn_alignbyte(dw(i + 1), dw(i), r & 3);
  }
  // byte at pos + lane, for pos - lo < 256
  __device__ __forceinline__ uint32_t lane_byte(uint32_t pos) const {
    const uint32_t r = pos - lo + (threadIdx.x & 63);
    const int addr = (int)(((r >> 2) & 63) << 2);
    const uint32_t a = __builtin_amdgcn_ds_bpermute(addr, (int)w0), b = __builtin_amdgcn_ds_bpermute(addr, (int)w1);
    return ((r < 256 ? a : b) >> ((r & 3) * 8)) & 0xFFu;
  }
};

template <bool RING>
struct WaveOut {
  lds_u8* ring;   // RING: kRing bytes (16-byte aligned); FULL: olen bytes
  uint8_t* dst;   // RING: HBM destination of the whole stream
  __amdgpu_buffer_rsrc_t rs;  // RING: dst, olen bytes (far history reads)
  __amdgpu_buffer_rsrc_t rsa;  // RING: the same bytes from dst rounded down to a dword (dword reads)
  uint32_t dal;                // dst & 3
  uint32_t olen;
  uint32_t op;
  // Rebased offsets stream (RING, dst dword-aligned): every stored word gets
  // xadd; past the column's first page stream word 0 is not stored (the
  // previous page's last offset owns that slot: decompress_binary drops p[0],
  // binary/mod.rs:136-144) but kept in w0; far reads undo both.
  bool xf, skip0;
  uint32_t xadd, w0;
  // RING: some flushed byte has its high bit set (wave-uniform; Utf8 values
  // streams whose bytes are all ASCII skip the UTF-8 scan, k_utf8_pages)
  bool hib = false;

  __device__ __forceinline__ uint32_t slot(uint32_t q) const { return RING ? (q & (kRing - 1)) : q; }
  __device__ __forceinline__ uint32_t far8(uint32_t q) const {  // stream byte q < far_limit(), from HBM
    if (!xf) return __builtin_amdgcn_raw_buffer_load_b8(rs, q, 0, SB_FAR_AUX);
    const uint32_t w = q < 4 ? w0 : __builtin_amdgcn_raw_buffer_load_b32(rsa, q & ~3u, 0, SB_FAR_AUX) - xadd;
    return (w >> (8 * (q & 3))) & 0xFFu;
  }
  __device__ __forceinline__ uint32_t far32(uint32_t a, bool on) const {  // dword at dst-aligned byte a (0 if !on)
    const uint32_t g = __builtin_amdgcn_raw_buffer_load_b32(rsa, on ? a : 0x80000000u, 0, SB_FAR_AUX);
    return !xf ? g : a == 0 ? w0 : g - xadd;
  }
  // four dwords at dst-aligned byte a, one load (0 if !on)
  __device__ __forceinline__ u32x4 far128(uint32_t a, bool on) const {
    u32x4 g = __builtin_amdgcn_raw_buffer_load_b128(rsa, on ? a : 0x80000000u, 0, SB_FAR_AUX);
    if (xf) {
      g -= xadd;
      if (a == 0) g[0] = w0;
    }
    return g;
  }
  // History below this position is read from HBM: writes of up to one chunk
  // past op overwrite the ring slots of chunks k-4 and k-3, and the flushes of
  // chunks <= k-2 have completed (each flush first waits for the previous).
  __device__ __forceinline__ uint32_t far_limit() const {
#ifdef SB_V_NOFAR
    return 0u;
#endif
    const uint32_t k = op / kChunk;
    return k >= 2 ? (k - 2) * kChunk : 0u;
  }
  __device__ __forceinline__ uint32_t room() const {
    return RING ? min(64u, kChunk - (op & (kChunk - 1))) : 64u;
  }
  __device__ void flush(uint32_t c0, uint32_t len) {
    const uint32_t lane = threadIdx.x & 63;
    // the previous chunk's stores must complete before far reads may use them
#ifndef SB_V_NOFLUSHWAIT
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    uint8_t* d = dst + c0;
    if (RING && xf) {  // dst is dword-aligned; len is a multiple of 4
      const __attribute__((address_space(3))) uint32_t* r32 = (const __attribute__((address_space(3))) uint32_t*)ring;
      if (c0 == 0) w0 = r32[0];
      uint32_t* d32 = (uint32_t*)d;
      for (uint32_t w = lane; w < len / 4; w += 64)
        if (!skip0 || (c0 | w)) d32[w] = r32[slot(c0 + 4 * w) >> 2] + xadd;
      return;
    }
    if (len == kChunk) {  // 16 bytes a lane (kChunk / 16 lanes)
      const bool on = 16 * lane < kChunk;
      const u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(ring + slot(c0 + (on ? 16 * lane : 0)));
      hib |= __ballot(on && ((v.x | v.y | v.z | v.w) & 0x80808080u) != 0) != 0;
      const uintptr_t al = (uintptr_t)d;
      if ((al & 3) == 0) {  // one 16-byte store a lane at any dword alignment
        if (on) ((u32x4*)d)[lane] = v;
      } else {
#pragma unroll
        for (uint32_t j = 0; j < kChunk / 64; j++) d[j * 64 + lane] = ring[slot(c0 + j * 64 + lane)];
      }
      return;
    }
    uint32_t hb = 0;
    for (uint32_t j = lane; j < len; j += 64) {
      const uint32_t b = ring[slot(c0 + j)];
      hb |= b;
      d[j] = (uint8_t)b;
    }
    hib |= __ballot((hb & 0x80u) != 0) != 0;
  }
  __device__ __forceinline__ void advance(uint32_t m) {
    op += m;
    if (RING && (op & (kChunk - 1)) == 0) flush(op - kChunk, kChunk);
  }
  __device__ __forceinline__ void lit(const WaveWin& w, uint32_t pos, uint32_t m) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t v = w.lane_byte(pos);
    if (lane < m) ring[slot(op + lane)] = (uint8_t)v;
    advance(m);
  }
  __device__ __forceinline__ void match(uint32_t off, uint32_t m) {
    const uint32_t lane = threadIdx.x & 63;
    if (lane < m) {
      const uint32_t q = op - off + (off >= 64 ? lane : lane % off);
      uint32_t v;
      if (RING && q < far_limit())
        v = far8(q);
      else
        v = ring[slot(q)];
      ring[slot(op + lane)] = (uint8_t)v;
    }
    advance(m);
  }
  __device__ __forceinline__ void finish() {
    if (RING && (op & (kChunk - 1))) flush(op & ~(kChunk - 1), op & (kChunk - 1));
  }
  __device__ __forceinline__ uint32_t hist(uint32_t q) const {
    if (RING && q < far_limit()) return far8(q);
    return ring[slot(q)];
  }
  // n (a multiple of kChunk) stream bytes straight to d: 16 bytes a lane per
  // KiB, two KiB per step, no waits between steps
  __device__ void copy_direct(gmem_u8* src, uint8_t* d, uint32_t n, uint32_t pos) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t sh = (uint32_t)((uintptr_t)src & 3);
    gmem_u32* s32 = (gmem_u32*)((uintptr_t)src - sh);
    const uint32_t dal = (uint32_t)((uintptr_t)d & 15);
    if (xf && pos == 0) w0 = __builtin_amdgcn_alignbyte(s32[1], s32[0], sh);
    constexpr uint32_t B = 1024;  // 16 bytes a lane; n is a multiple of kChunk (<= B)
    for (uint32_t c = 0; c < n; c += 2 * B) {
      uint32_t w[2][5];
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t x = c + h * B + 16 * lane, i = (sh + x) >> 2;
        const bool on = x < n;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) w[h][k] = on ? s32[i + k] : 0u;
        w[h][4] = on && sh ? s32[i + 4] : 0u;  // the dword past byte x + 15 only when x is unaligned
      }
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        if (c + h * B >= n) break;
        const uint32_t x = c + h * B + 16 * lane;
        if (x >= n) continue;
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(w[h][1], w[h][0], sh);
        v.y = __builtin_amdgcn_alignbyte(w[h][2], w[h][1], sh);
        v.z = __builtin_amdgcn_alignbyte(w[h][3], w[h][2], sh);
        v.w = __builtin_amdgcn_alignbyte(w[h][4], w[h][3], sh);
        hib |= __ballot(((v.x | v.y | v.z | v.w) & 0x80808080u) != 0) != 0;
        if (xf) {
          uint32_t* q = (uint32_t*)(d + x);
          if (!skip0 || pos + x) q[0] = v.x + xadd;
          q[1] = v.y + xadd; q[2] = v.z + xadd; q[3] = v.w + xadd;
        } else if ((dal & 3) == 0) {
          *(u32x4*)(d + x) = v;
        } else {
#pragma unroll
          for (uint32_t b = 0; b < 16; b++) d[x + b] = (uint8_t)(v[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
  }
  // len literal bytes from HBM.  Whole chunks more than three chunks before
  // the literal's end go straight to the destination (they are history only
  // far reads reach, and the three ring flushes after them wait for their
  // stores); the rest goes through the ring, a chunk per step.
  __device__ void lit_global(gmem_u8* src, uint32_t len) {
    const uint32_t lane = threadIdx.x & 63;
    if (RING && len > 5 * kChunk) {
      const uint32_t h = (kChunk - (op & (kChunk - 1))) & (kChunk - 1);
      if (h) {
        lit_ring(src, h);
        src += h;
        len -= h;
      }
      const uint32_t direct = (len / kChunk - 3) * kChunk;
      copy_direct(src, dst + op, direct, op);
      op += direct;
      src += direct;
      len -= direct;
    }
    (void)lane;
    lit_ring(src, len);
  }
  // len literal bytes from HBM through the ring, up to a chunk per step (16 loads per lane in flight)
  __device__ void lit_ring(gmem_u8* src, uint32_t len) {
    const uint32_t lane = threadIdx.x & 63;
    while (len) {
      const uint32_t m = min(len, RING ? kChunk - (op & (kChunk - 1)) : kChunk);
      uint32_t b[16];
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) b[j] = src[min(lane + 64 * j, m - 1)];
#pragma unroll
      for (uint32_t j = 0; j < 16; j++)
        if (lane + 64 * j < m) ring[slot(op + lane + 64 * j)] = (uint8_t)b[j];
      src += m;
      len -= m;
      advance(m);
    }
  }
};

template <bool RING>
__device__ uint32_t lz4_wave(WaveWin& w, uint32_t p, uint32_t pend, WaveOut<RING>& o) {
  const uint32_t olen = o.olen;
  if (p == pend) return olen == 0 ? ST_OK : ST_CODEC;
  for (;;) {
    w.slide(p);
    const uint32_t token = w.byte(p++);
    uint32_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (p >= pend) return ST_CODEC;
        b = w.byte(p++);
        lit += b;
      } while (b == 255);
    }
    if (lit > pend - p || lit > olen - o.op) return ST_CODEC;
    while (lit) {
      w.slide(p);
      const uint32_t m = min(lit, o.room());
      o.lit(w, p, m);
      p += m;
      lit -= m;
    }
    if (p == pend) break;  // the last sequence carries literals only
    if (pend - p < 2) return ST_CODEC;
    w.slide(p);
    const uint32_t off = w.byte(p) | (w.byte(p + 1) << 8);
    p += 2;
    if (off == 0 || off > o.op) return ST_CODEC;
    uint32_t ml = (token & 15) + 4;
    if ((token & 15) == 15) {
      uint32_t b;
      do {
        if (p >= pend) return ST_CODEC;
        b = w.byte(p++);
        ml += b;
      } while (b == 255);
    }
    if (ml > olen - o.op) return ST_CODEC;
    while (ml) {
      const uint32_t m = min(ml, o.room());
      o.match(off, m);
      ml -= m;
    }
  }
  if (o.op != olen) return ST_CODEC;
  o.finish();
  return ST_OK;
}

// Snappy raw: varint length, then literal / copy-1 / copy-2 / copy-4 elements.
template <bool RING>
__device__ uint32_t snappy_wave(WaveWin& w, uint32_t p, uint32_t pend, WaveOut<RING>& o) {
  const uint32_t olen = o.olen;
  uint64_t ulen = 0;
  for (uint32_t sft = 0;; sft += 7) {
    if (p >= pend || sft > 35) return ST_CODEC;
    const uint32_t c = w.byte(p++);
    ulen |= (uint64_t)(c & 0x7F) << sft;
    if (!(c & 0x80)) break;
  }
  if (ulen != olen) return ST_CODEC;
  while (p < pend) {
    w.slide(p);
    const uint32_t tag = w.byte(p++);
    const uint32_t type = tag & 3;
    if (type == 0) {
      uint32_t len = (tag >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = len - 60;
        if (pend - p < nb) return ST_CODEC;
        len = 0;
        for (uint32_t i = 0; i < nb; i++) len |= w.byte(p + i) << (8 * i);
        len += 1;
        p += nb;
      }
      if (len > pend - p || len > olen - o.op) return ST_CODEC;
      while (len) {
        w.slide(p);
        const uint32_t m = min(len, o.room());
        o.lit(w, p, m);
        p += m;
        len -= m;
      }
    } else {
      uint32_t len, off;
      if (type == 1) {
        if (pend - p < 1) return ST_CODEC;
        len = ((tag >> 2) & 7) + 4;
        off = ((tag >> 5) << 8) | w.byte(p);
        p += 1;
      } else if (type == 2) {
        if (pend - p < 2) return ST_CODEC;
        len = (tag >> 2) + 1;
        off = w.byte(p) | (w.byte(p + 1) << 8);
        p += 2;
      } else {
        if (pend - p < 4) return ST_CODEC;
        len = (tag >> 2) + 1;
        off = w.byte(p) | (w.byte(p + 1) << 8) | (w.byte(p + 2) << 16) | (w.byte(p + 3) << 24);
        p += 4;
      }
      if (off == 0 || off > o.op || len > olen - o.op) return ST_CODEC;
      while (len) {
        const uint32_t m = min(len, o.room());
        o.match(off, m);
        len -= m;
      }
    }
  }
  if (o.op != olen) return ST_CODEC;
  o.finish();
  return ST_OK;
}


// ---------------------------------------------------------------------------
// Batched LZ4 (k_inflate).  A serial token walk costs ~1000 cycles per
// sequence on one wave, and the pages' streams hold a sequence every ~5
// compressed bytes, so the walk is restated data-parallel per batch:
//  1. every lane parses a sequence at 4 candidate positions p + 4 lane + k
//     (k < 4) and packs the byte distance to its successor (0 = take the
//     serial path: final literal-only sequence, literal > kLitFast, lengths
//     past the staged input, a distance > 255);
//  2. a scalar chase follows successors from p (one v_readlane per sequence)
//     and deals the true sequence starts to lanes;
//  3. lanes decode their sequence, a wave scan places the outputs (at most a
//     chunk per batch), literals are copied lane-parallel, then matches whose
//     source ends before the batch's first match byte are copied
//     lane-parallel and the rest in sequence order, wave-wide.
// The compressed stream is staged into a per-wave kIb ring (LDS-DMA at a
// seek, then half a ring at a time from registers loaded half a ring ahead).
// ---------------------------------------------------------------------------
// Record chains through a window, wave-parallel.  Variable-length records
// whose size follows from their own header (Patas records, LZ4 sequences)
// chain: the next record starts at x + d(x).  Every lane sizes the records
// that WOULD start at 4 positions of a 255-position window (byte k of lane l
// = position 4l + k); successor tables T1 = x -> x + d(x) (0xFF past the
// window or after a record that stops the chain) are doubled by ds_bpermute
// lookups (T2 = T1 o T1, ..., T32), and lane k composes them along the bits
// of k: the k-th record's position.  26 permutes per window instead of a
// scalar chase per record.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t tab_at(uint32_t table, uint32_t x) {  // byte x of the wave-wide table
  const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((x >> 2) << 2), (int)table);
  return x == 0xFF ? 0xFFu : (w >> ((x & 3) * 8)) & 0xFFu;
}
// t1: the packed successor table; returns the k-th record's position in lane k (0xFF: none)
__device__ __forceinline__ uint32_t wave_chain(uint32_t t1) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t T[6];
  T[0] = t1;
#pragma unroll
  for (int j = 1; j < 6; j++) {
    uint32_t nt = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t t = (T[j - 1] >> (8 * k)) & 0xFFu;
      nt |= tab_at(T[j - 1], t) << (8 * k);
    }
    T[j] = nt;
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const uint32_t y = tab_at(T[j], x);
    if ((lane >> j) & 1) x = y;
  }
  return x;
}

// wave_chain through LDS byte tables: T1..T32 at tab + 256 j (T1 bytes 254
// and 255 must be 0xFE and 0xFF, so every table maps both sentinels to
// themselves and no lookup needs a guard); one byte read per lookup instead
// of a permute and a byte extract.
__device__ __forceinline__ uint32_t lds_chain(lds_u8* tab, uint32_t t1) {
  typedef __attribute__((address_space(3))) uint32_t l32;
  const uint32_t lane = threadIdx.x & 63;
  ((l32*)tab)[lane] = t1;
  uint32_t T = t1;
#pragma unroll
  for (int j = 1; j < 6; j++) {
    const lds_u8* prev = tab + 256 * (j - 1);
    uint32_t nt = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) nt |= (uint32_t)prev[(T >> (8 * k)) & 0xFFu] << (8 * k);
    ((l32*)tab)[64 * j + lane] = nt;
    T = nt;
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const uint32_t y = tab[256 * j + x];
    if ((lane >> j) & 1) x = y;
  }
  return x;
}

#ifndef SB_INF_MATCHFAST
#define SB_INF_MATCHFAST 24  // longer matches go the hazard way (C3 3.64 -> 3.59 ms, C5 2.36 -> 2.33 against 32)
#endif
#ifndef SB_INF_LITFAST
#define SB_INF_LITFAST 64
#endif
constexpr uint32_t kIb = 1024, kIbHalf = kIb / 2, kLitFast = SB_INF_LITFAST, kMatchFast = SB_INF_MATCHFAST;
// (a batch's bytes, <= p + 261 + kLitFast, stay inside the staged input window)
static_assert(kIbHalf + 261 + kLitFast + 20 <= kIb, "kLitFast too large for the input ring");
constexpr uint32_t kChainTabs = 6;  // T1..T32: batches of up to 64 sequences
constexpr uint32_t kChainEnd = 0xFE, kChainStop = 0xFF;  // chain sentinels (see cand_steps)

struct InRing {
  gmem_u32* g;   // dword-aligned stream base
  uint32_t nd;   // stream dwords
  lds_u8* ib;    // kIb (1 KiB) bytes: stream byte x at ib[x % kIb]
  lds_u8* ct;    // kChainTabs x 256 bytes: the chain tables T1..T32
  uint32_t base; // [base, base + kIb) staged and complete; base % kIbHalf == 0
  u32x2 pf;      // [base + kIb, base + kIb + kIbHalf), 8 bytes a lane, loaded ahead in registers
  // (a 1 KiB ring and six chain tables keep the wave at 6.5 KiB of LDS: six waves per SIMD)

  __device__ __forceinline__ void dma(uint32_t b) {  // [b, b + kIbHalf) -> ib
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t k = 0; k < kIbHalf / 256; k++) {
      const uint32_t dw = min((b >> 2) + 64 * k + lane, nd - 1);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g + dw),
                                       (__attribute__((address_space(3))) void*)(ib + (b & (kIb - 1)) + 256 * k), 4,
                                       0, 0);
    }
  }
  __device__ __forceinline__ void prefetch(uint32_t b) {  // [b, b + kIbHalf) -> pf
    const uint32_t i = (b >> 2) + 2 * (threadIdx.x & 63);
    pf.x = g[min(i, nd - 1)];
    pf.y = g[min(i + 1, nd - 1)];
  }
  __device__ void seek(uint32_t x) {
    base = x & ~(kIbHalf - 1);
    dma(base);
    dma(base + kIbHalf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    prefetch(base + kIb);
  }
  __device__ __forceinline__ void slide(uint32_t p) {
    if (p - base < kIbHalf) return;
    if (p - base >= kIb) { seek(p); return; }
    // the prefetched half into the slot of base, then the next one
    *(__attribute__((address_space(3))) u32x2*)(ib + (base & (kIb - 1)) + 8 * (threadIdx.x & 63)) = pf;
    base += kIbHalf;
    prefetch(base + kIb);
  }
  __device__ __forceinline__ uint32_t ubyte(uint32_t x) const {  // uniform
    if (x - base < kIb) return ib[x & (kIb - 1)];
    return ((gmem_u8*)g)[x];
  }
};

struct Seq {
  uint32_t lit_pos, lit, off, ml, next;
};

// Lane-parallel parse of the sequence at x from the staged input; false when
// it must take the serial path.  lim: end of the staged, complete input.
__device__ __forceinline__ bool seq_at(const lds_u8* ib, uint32_t x, uint32_t lim, uint32_t pend, Seq& s) {
  if (x >= lim) return false;
  const uint32_t t = ib[x & (kIb - 1)];
  uint32_t y = x + 1, lit = t >> 4;
  if (lit == 15) {
    uint32_t b;
    do {
      if (y >= lim) return false;
      b = ib[y & (kIb - 1)];
      y++;
      lit += b;
    } while (b == 255 && lit <= kLitFast);
  }
  if (lit > kLitFast) return false;
  const uint32_t le = y + lit;
  if (le + 2 > lim || le >= pend) return false;  // (le == pend: the final sequence)
  s.lit_pos = y;
  s.lit = lit;
  s.off = ib[le & (kIb - 1)] | ((uint32_t)ib[(le + 1) & (kIb - 1)] << 8);
  y = le + 2;
  uint32_t ml = (t & 15) + 4;
  if ((t & 15) == 15) {
    uint32_t b;
    do {
      if (y >= lim) return false;
      b = ib[y & (kIb - 1)];
      y++;
      ml += b;
    } while (b == 255);
  }
  s.ml = ml;
  s.next = y;
  return true;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
// *p = (*p & ~clear) | set, one LDS op (lanes sharing a word apply in turn)
__device__ __forceinline__ void lds_mskor(lds_u32* p, uint32_t clear, uint32_t set) {
  asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"((uint32_t)(uintptr_t)p), "v"(clear), "v"(set) : "memory");
}
// Bytes [0, n) of a source whose byte i is byte sh + i of the words w[0..NW)
// (sh + n <= 4 NW), stored at ring position d: one masked store per
// destination word, so lanes writing neighbouring ranges may share edge words.
template <int NW>
__device__ __forceinline__ void ring_put(lds_u8* ring, uint32_t d, uint32_t n, uint32_t sh, const uint32_t* w) {
  lds_u32* r32 = (lds_u32*)ring;
  const uint32_t dsh = d & 3, base = d - dsh, e = (sh - dsh) & 3;
  const bool fwd = sh >= dsh;
#pragma unroll
  for (int t = 0; t <= NW; t++) {
    const int rem = (int)n - (4 * t - (int)dsh);  // source bytes from this word on
    if (!__ballot(rem > 0)) break;
    if (rem > 0) {
      const uint32_t z = t > 0 ? w[t - 1] : 0u, a = t < NW ? w[t] : 0u, b = t + 1 < NW ? w[t + 1] : 0u;
      const uint32_t u = fwd ? __builtin_amdgcn_alignbyte(b, a, e) : __builtin_amdgcn_alignbyte(a, z, e);
      uint32_t m = rem >= 4 ? ~0u : (1u << (8 * rem)) - 1u;
      if (t == 0) m &= ~0u << (8 * dsh);
      lds_mskor(r32 + (((base + 4 * t) & (kRing - 1)) >> 2), m, u & m);
    }
  }
}
// lane % o for lane < 64, 0 < o < 64, without an integer divide
__device__ __forceinline__ uint32_t lane_mod(uint32_t lane, uint32_t o) {
  const uint32_t q = (uint32_t)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)o));
  return lane - q * o;
}

// Successor table of the candidate starts p + r (r = 4 lane + k < 254):
// byte k = r + d for a sequence of d bytes that batch decoding takes (literal
// <= kLitFast, each length with at most one extension byte, not the final
// sequence, staged below lim), kChainEnd when such a sequence's successor
// lies past position 253 (the batch ends after it), else kChainStop (the
// sequence is not taken); entries 254 and 255 are the sentinels themselves.
// A chain position x is a taken sequence iff x < kChainEnd and T1[x] !=
// kChainStop.
__device__ __forceinline__ uint32_t succ_byte(bool ok, uint32_t nr) {
  return !ok ? kChainStop : nr < kChainEnd ? nr : kChainEnd;
}
__device__ __forceinline__ uint32_t cand_steps(const lds_u8* ib, uint32_t p, uint32_t lim, uint32_t pend) {
  typedef __attribute__((address_space(3))) uint32_t l32;
  const l32* ib32 = (const l32*)ib;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t x0 = p + 4 * lane, a0 = x0 & ~3u, sh = x0 & 3;
  const uint32_t w0 = ib32[(a0 & (kIb - 1)) >> 2], w1 = ib32[((a0 + 4) & (kIb - 1)) >> 2],
                 w2 = ib32[((a0 + 8) & (kIb - 1)) >> 2];
  const uint32_t tok = __builtin_amdgcn_alignbyte(w1, w0, sh);   // bytes x0 .. x0 + 3
  const uint32_t nxt = __builtin_amdgcn_alignbyte(w2, w1, sh);   // bytes x0 + 4 .. x0 + 7
  const uint32_t ext = __builtin_amdgcn_alignbyte(nxt, tok, 1);  // bytes x0 + 1 .. x0 + 4
  uint32_t t1 = 0;
  if (lim - p >= 261 + kLitFast) {  // every candidate's bytes (<= p + 260 + kLitFast) are staged: no bounds checks
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t x = x0 + k, t = (tok >> (8 * k)) & 0xFFu, e = (ext >> (8 * k)) & 0xFFu;
      const uint32_t ln = t >> 4, lx = ln == 15;
      const uint32_t lit = lx ? 15 + e : ln;
      const uint32_t y = x + 3 + lx + lit;  // past the offset
      const uint32_t e2 = ib[y & (kIb - 1)], mx = (t & 15) == 15;
      const bool ok = lit <= kLitFast && !(mx && e2 == 255);
      const uint32_t r = 4 * lane + k, nr = r + (y + mx - x);
      t1 |= succ_byte(ok, nr) << (8 * k);
    }
    return lane == 63 ? (t1 & 0xFFFFu) | (kChainEnd << 16) | (kChainStop << 24) : t1;
  }
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint32_t x = x0 + k, t = (tok >> (8 * k)) & 0xFFu, e = (ext >> (8 * k)) & 0xFFu;
    const uint32_t ln = t >> 4;
    const bool lx = ln == 15;
    const uint32_t lit = lx ? 15 + e : ln;
    const uint32_t le = x + 1 + (uint32_t)lx + lit;  // the offset's position
    bool ok = x + 1 + (uint32_t)lx <= lim && lit <= kLitFast && le + 2 <= lim && le < pend;
    uint32_t y = le + 2;
    if (ok && (t & 15) == 15) {
      const uint32_t e2 = y < lim ? (uint32_t)ib[y & (kIb - 1)] : 255u;
      ok = e2 != 255;
      y++;
    }
    const uint32_t r = 4 * lane + k, nr = r + (y - x);
    t1 |= succ_byte(ok, nr) << (8 * k);
  }
  return lane == 63 ? (t1 & 0xFFFFu) | (kChainEnd << 16) | (kChainStop << 24) : t1;
}

// The sequence at x, which cand_steps accepted (no checks left to make).
__device__ __forceinline__ void seq_parse(const lds_u8* ib, uint32_t x, Seq& s) {
  const uint32_t t = ib[x & (kIb - 1)], e = ib[(x + 1) & (kIb - 1)];
  const uint32_t lx = (t >> 4) == 15, lit = lx ? 15 + e : t >> 4;
  const uint32_t le = x + 1 + lx + lit;
  const uint32_t o0 = ib[le & (kIb - 1)], o1 = ib[(le + 1) & (kIb - 1)], e2 = ib[(le + 2) & (kIb - 1)];
  const uint32_t mx = (t & 15) == 15;
  s.lit_pos = x + 1 + lx;
  s.lit = lit;
  s.off = o0 | (o1 << 8);
  s.ml = (t & 15) + 4 + (mx ? e2 : 0u);
  s.next = le + 2 + mx;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {  // DPP: no LDS round trips
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
  return v;
}

// One sequence at *pp, serially (the liblz4 checks of lz4_wave).
__device__ uint32_t lz4_one(InRing& in, uint32_t* pp, uint32_t pend, WaveOut<true>& o, bool* ended) {
  uint32_t p = *pp;
  const uint32_t olen = o.olen;
  const uint32_t token = in.ubyte(p++);
  uint32_t lit = token >> 4;
  if (lit == 15) {
    uint32_t b;
    do {
      if (p >= pend) return ST_CODEC;
      b = in.ubyte(p++);
      lit += b;
    } while (b == 255);
  }
  if (lit > pend - p || lit > olen - o.op) return ST_CODEC;
  o.lit_global((gmem_u8*)in.g + p, lit);
  p += lit;
  if (p == pend) {  // the last sequence carries literals only
    *ended = true;
    *pp = p;
    return ST_OK;
  }
  if (pend - p < 2) return ST_CODEC;
  const uint32_t off = in.ubyte(p) | (in.ubyte(p + 1) << 8);
  p += 2;
  if (off == 0 || off > o.op) return ST_CODEC;
  uint32_t ml = (token & 15) + 4;
  if ((token & 15) == 15) {
    uint32_t b;
    do {
      if (p >= pend) return ST_CODEC;
      b = in.ubyte(p++);
      ml += b;
    } while (b == 255);
  }
  if (ml > olen - o.op) return ST_CODEC;
  while (ml) {
    const uint32_t m = min(ml, o.room());
    o.match(off, m);
    ml -= m;
  }
  *pp = p;
  return ST_OK;
}

#ifdef SB_INF_PHASES  // A/B instrumentation: shader cycles per phase of the batch loop, summed over waves
// [0] slide [1] candidates [2] chain [3] parse + place [4] literals [5] free matches [6] hazards [7] flush
// [8] serial path; counts: [9] batches [10] sequences [11] hazards [12] serial sequences [13] jobs
__device__ unsigned long long sb_dbg_inf[16];
#define INF_T(k)                                                         \
  do {                                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                    \
    ph[k] += t_ - tph;                                                   \
    tph = t_;                                                            \
  } while (0)
#define INF_N(k, v) ph[k] += (v)
#else
#define INF_T(k) do { } while (0)
#define INF_N(k, v) do { } while (0)
#endif

__device__ uint32_t lz4_inflate(InRing& in, uint32_t p, uint32_t pend, WaveOut<true>& o) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t olen = o.olen;
  if (p == pend) return olen == 0 ? ST_OK : ST_CODEC;
  bool ended = false;
#ifdef SB_INF_PHASES
  uint64_t ph[16] = {0};
  uint64_t tph = __builtin_amdgcn_s_memtime();
  INF_N(13, 1);
#endif
  // the chain of the batch at p: found at the loop's top, or (SB_INF_PIPE)
  // by the previous batch while its far loads were in flight
  uint32_t cx = 0, j = 0;
  bool have = false;
  // 1. successor distances of the candidate starts x = p + 4 lane + k, from
  //    the token and at most one extension byte per length: the tokens are
  //    one unaligned dword of the ring, the literal extensions the next
  //    bytes; only a match-length extension needs its own byte read;
  // 2. the chain of sequence starts from p, wave-parallel: a candidate that
  //    needs the serial path ends it
  auto chain_at = [&](uint32_t q) {
    in.slide(q);
    const uint32_t lim = min(in.base + kIb, pend);
    const uint32_t t1 = cand_steps(in.ib, q, lim, pend);
#ifdef SB_INF_BPCHAIN  // the chain by ds_bpermute doubling: no LDS tables
    cx = wave_chain(t1);
    j = (uint32_t)__popcll(__ballot(cx < kChainEnd && tab_at(t1, cx) != kChainStop));
#else
    cx = lds_chain(in.ct, t1);
    j = (uint32_t)__popcll(__ballot(cx < kChainEnd && in.ct[cx] != kChainStop));
#endif
  };
  while (p < pend && !ended) {
    if (!have) chain_at(p);
    have = false;
    INF_T(2);
    const uint32_t starts = p + cx;
    // 3. decode and place
    Seq s{0, 0, 0, 0, 0};
    const bool v0 = lane < j;
    if (v0) seq_parse(in.ib, starts, s);
    const uint32_t len = v0 ? s.lit + s.ml : 0u;
    const uint32_t incl = wave_incl_scan(len), excl = incl - len;
    const uint32_t cap = min(kChunk, olen - o.op);
    const uint32_t dl = o.op + excl, dm = dl + s.lit;  // literal and match destinations
    const bool ok = v0 && incl <= cap && s.off != 0 && s.off <= dm;
    const uint64_t okm = __ballot(ok);
    const uint32_t k = okm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~okm);
    INF_T(3);
    if (k == 0) {  // the serial path takes one sequence (and reports errors)
      const uint32_t st = lz4_one(in, &p, pend, o, &ended);
      if (st) return st;
      INF_T(8);
      INF_N(12, 1);
      continue;
    }
    INF_N(9, 1);
    INF_N(10, k);
    // the batch's end: where the k-th sequence resumes the stream, and the output length
    const uint32_t pnext = __builtin_amdgcn_readlane(s.next, k - 1);
    const uint32_t nop = o.op + __builtin_amdgcn_readlane(incl, k - 1);
#ifdef SB_V_NOCOPY
    const bool v = false;
#else
    const bool v = lane < k;
#endif
    typedef __attribute__((address_space(3))) uint32_t l32;
    const l32* ib32 = (const l32*)in.ib;
    const l32* r32 = (const l32*)o.ring;
#ifdef SB_V_NOLIT
    if (v) s.lit = 0;
#endif
#ifdef SB_INF_EARLYFAR
    // The free matches' sources are final before the batch (below d_first), and
    // those below farlim are in HBM: their first dwords are loaded now, so the
    // loads' latency passes under the literal copies.
    const uint32_t d_first = __builtin_amdgcn_readfirstlane(dm);
    const uint32_t src = dm - s.off;
    const bool hazard = v && (src + s.ml > d_first || s.ml > kMatchFast);
    const bool freel = v && !hazard;
    const uint32_t farlim = o.far_limit();
    const bool mfar = src + s.ml <= farlim, mnear = src >= farlim;
    const bool fw = freel && (mfar || mnear);
    const uint32_t fa = mfar ? src + o.dal : src, fsh = fa & 3, fa0 = fa - fsh, fneed = fw ? fsh + s.ml : 0u;
    constexpr uint32_t kEarly = 3;
    uint32_t pw[kEarly];
#pragma unroll
    for (uint32_t t = 0; t < kEarly; t++) {
      const bool need = fw && mfar && 4 * t < fneed;
      pw[t] = __ballot(need) ? o.far32(fa0 + 4 * t, need) : 0u;
    }
#endif
    // literals, 16 bytes per lane per step: source dwords from the input ring,
    // one masked dword store per destination word
    for (uint32_t c = 0; __ballot(v && c < s.lit); c += 16) {
      if (v && c < s.lit) {
        const uint32_t x = s.lit_pos + c, sh = x & 3, a0 = x - sh, n = min(16u, s.lit - c);
        uint32_t w[5];
#pragma unroll
        for (uint32_t t = 0; t < 5; t++) w[t] = ib32[((a0 + 4 * t) & (kIb - 1)) >> 2];
        ring_put<5>(o.ring, dl + c, n, sh, w);
      }
    }
#ifdef SB_INF_PIPE
    // the next batch's candidates and chain, under the far loads' latency (the
    // literals are in the output ring: the input ring may slide)
    if (pnext < pend) {
      chain_at(pnext);
      have = true;
    }
#endif
    INF_T(4);
#ifndef SB_INF_EARLYFAR
    const uint32_t d_first = __builtin_amdgcn_readfirstlane(dm);
    const uint32_t src = dm - s.off;
#ifdef SB_V_NOHAZ
    const bool hazard = false;
#else
    const bool hazard = v && (src + s.ml > d_first || s.ml > kMatchFast);
#endif
#ifdef SB_V_NOFREE
    const bool freel = false;
#else
    const bool freel = v && !hazard;
#endif
    const uint32_t farlim = o.far_limit();
    // A free match's source is final before the batch: its dwords come from
    // HBM below farlim (an out-of-range buffer offset reads 0 for the other
    // lanes) or from the ring, all loads before the stores; a source
    // straddling farlim goes byte by byte.
    const bool mfar = src + s.ml <= farlim, mnear = src >= farlim;
    const bool fw = freel && (mfar || mnear);
    const uint32_t fa = mfar ? src + o.dal : src, fsh = fa & 3, fa0 = fa - fsh, fneed = fw ? fsh + s.ml : 0u;
#endif
    if (__ballot(fw)) {
      constexpr uint32_t NW = kMatchFast / 4 + 1;
      uint32_t w[NW];
#if SB_INF_FAR128 && !defined(SB_INF_EARLYFAR)
      // the far source's first 16 bytes in one load (C3 3.81 -> 3.65 ms a
      // step: one vector-memory instruction instead of up to four)
      const bool f4 = fw && mfar;
      const u32x4 g4 = __ballot(f4) ? o.far128(fa0, f4) : u32x4{0, 0, 0, 0};
#endif
#pragma unroll
      for (uint32_t t = 0; t < NW; t++) {
        w[t] = 0;
        if (!__ballot(4 * t < fneed)) continue;
#ifdef SB_INF_EARLYFAR
        // ring sources now (this batch's literals are in); far dwords past the
        // early ones loaded here, only when some lane needs them
        const bool nr = !mfar && 4 * t < fneed;
        const uint32_t r = __ballot(nr) ? r32[((fa0 + 4 * t) & (kRing - 1)) >> 2] : 0u;
        uint32_t g;
        if (t < kEarly) {
          g = pw[t < kEarly ? t : 0];
        } else {
          const bool nf = mfar && 4 * t < fneed;
          g = __ballot(nf) ? o.far32(fa0 + 4 * t, nf) : 0u;
        }
#elif SB_INF_FAR128
        const uint32_t g = t < 4 ? g4[t < 4 ? t : 0] : o.far32(fa0 + 4 * t, mfar && 4 * t < fneed);
        const uint32_t r = r32[((fa0 + 4 * t) & (kRing - 1)) >> 2];
#else
        const uint32_t g = o.far32(fa0 + 4 * t, mfar && 4 * t < fneed);
        const uint32_t r = r32[((fa0 + 4 * t) & (kRing - 1)) >> 2];
#endif
        w[t] = mfar ? g : r;
      }
      if (fw) ring_put<NW>(o.ring, dm, s.ml, fsh, w);
    }
    const bool fmix = freel && !mfar && !mnear;
    for (uint32_t i = 0; __ballot(fmix && i < s.ml); i++) {
      if (fmix && i < s.ml) {
        const uint32_t qq = src + i;
        const uint32_t b = qq < farlim ? o.far8(qq) : o.ring[qq & (kRing - 1)];
        o.ring[(dm + i) & (kRing - 1)] = (uint8_t)b;
      }
    }
    INF_T(5);
    INF_N(11, __popcll(__ballot(hazard)));
    // Hazards in sequence order.  The common kind (no self-overlap, source in
    // the ring, <= 64 bytes) is one byte a lane; its ring positions and
    // length are packed per lane beforehand, so each takes one v_readlane.
    const bool hfast = hazard && s.ml <= 64 && s.off >= s.ml && src >= farlim;
#ifdef SB_INF_HAZGROUP
    // Consecutive fast hazards go as one group, one byte a lane: a member joins
    // while the group's bytes fit the wave and its source lies outside the
    // span of the group's destinations (every earlier byte it reads is then
    // final), so a group costs one LDS read and one store instead of a pair
    // per hazard.  Positions are packed relative to op - kRing (13 bits each:
    // sources reach back at most the ring, destinations a chunk ahead).
    const uint32_t rel0 = o.op - kRing;
    const uint32_t hpack = hfast ? ((src - rel0) << 19) | ((dm - rel0) << 6) | (s.ml - 1) : 0u;
    const uint64_t fastm = __ballot(hfast);
    for (uint64_t hm = __ballot(hazard); hm;) {
      const uint32_t l = (uint32_t)__builtin_ctzll(hm);
      if ((fastm >> l) & 1) {
        uint32_t base = 0, gd0 = 0, gend = 0, rs = 0, rd = 0;
        bool act = false;
        while (hm && ((fastm >> __builtin_ctzll(hm)) & 1)) {
          const uint32_t h = __builtin_amdgcn_readlane(hpack, (uint32_t)__builtin_ctzll(hm));
          const uint32_t m = (h & 63u) + 1u, hs = h >> 19, hd = (h >> 6) & 0x1FFFu;
          if (base) {
            if (base + m > 64u || !(hs + m <= gd0 || hs >= gend)) break;
          } else {
            gd0 = hd;
          }
          if (lane >= base && lane < base + m) {
            rs = hs + lane - base;
            rd = hd + lane - base;
            act = true;
          }
          base += m;
          gend = hd + m;
          hm &= hm - 1;
        }
        const uint32_t b = act ? (uint32_t)o.ring[(rs + rel0) & (kRing - 1)] : 0u;
        if (act) o.ring[(rd + rel0) & (kRing - 1)] = (uint8_t)b;
        continue;
      }
      hm &= hm - 1;
#else
    const uint32_t hpack = ((src & (kRing - 1)) << 20) | ((dm & (kRing - 1)) << 8) | (hfast ? s.ml : 0u);
    const uint64_t fastm = __ballot(hfast);
    for (uint64_t hm = __ballot(hazard); hm; hm &= hm - 1) {
      const uint32_t l = (uint32_t)__builtin_ctzll(hm);
      if ((fastm >> l) & 1) {
        const uint32_t h = __builtin_amdgcn_readlane(hpack, l);
        if (lane < (h & 0xFFu))
          o.ring[((h >> 8) + lane) & (kRing - 1)] = o.ring[((h >> 20) + lane) & (kRing - 1)];
        continue;
      }
#endif
      const uint32_t D = __builtin_amdgcn_readlane(dm, l), O = __builtin_amdgcn_readlane(s.off, l),
                     M = __builtin_amdgcn_readlane(s.ml, l);
      for (uint32_t c = 0; c < M; c += 64) {
        if (lane < M - c) {
          const uint32_t x = D + c;
          const uint32_t qq = x - O + (O >= 64 ? lane : lane_mod(lane, O));
          const uint32_t b = qq < farlim ? o.far8(qq) : o.ring[qq & (kRing - 1)];
          o.ring[(x + lane) & (kRing - 1)] = (uint8_t)b;
        }
      }
    }
    INF_T(6);
    p = pnext;
    if ((nop / kChunk) != (o.op / kChunk)) o.flush(o.op & ~(kChunk - 1), kChunk);
    o.op = nop;
    INF_T(7);
  }
#ifdef SB_INF_PHASES
  if (lane < 14) atomicAdd(&sb_dbg_inf[lane], (unsigned long long)ph[lane]);
#endif
  if (!ended || o.op != olen) return ST_CODEC;
  o.finish();
  return ST_OK;
}

// Patas leaf pages of a Float32 / Float64 column (double/patas.rs:107-132),
// one wave per page, decoded straight into the column.  References reach at
// most 127 rows back, so the wave keeps the last 256 values in an LDS ring.
// Per block of 64 rows:
//  1. the rows' record starts come from wave_chain over 255-byte windows
//     (record size = 2 + sig bytes, from the header alone);
//  2. each lane parses its record (v << tz, reference row - ref_diff); a
//     reference before the block reads the ring, references inside it resolve
//     by pointer jumping across lanes (6 rounds of ds_bpermute);
//  3. the block's values go to the ring and, coalesced, to HBM.
// The first bad record decides the status, as in the reference's loop.
// The stream is read through k_inflate's 1 KiB LDS input ring (InRing: the
// next 512 bytes loaded ahead in registers), slid to each window's start:
// a block's headers and records lie within ~650 bytes of it, so they are LDS
// reads; the rare byte past the staged KiB is read from HBM (the same
// clamped dwords).  (Read from HBM directly, a 64-row block cost three
// dependent HBM round trips: 0.37 ms for a C5 Float64 Patas column.)
template <int W>
__device__ uint32_t patas_wave(const uint8_t* src, uint32_t ilen, uint8_t* dst, uint32_t n, lds_u8* ring, lds_u8* ibuf) {
  using T = typename VT<W>::T;
  const uint32_t lane = threadIdx.x & 63;
  if (n == 0) return ST_OUT_OF_SPEC;  // `length - 1` underflows (patas.rs:117)
  if (ilen < W) return ST_IO;
  gmem_u32* g = (gmem_u32*)((uintptr_t)src & ~(uintptr_t)3);
  const uint32_t sb0 = (uint32_t)((uintptr_t)src & 3);
  const uint32_t nd = (sb0 + ilen + 3) >> 2;
  InRing in;
  in.g = g;
  in.nd = nd;
  in.ib = ibuf;
  in.ct = nullptr;
  in.seek(sb0);
  typedef __attribute__((address_space(3))) uint32_t l32;
  const l32* ib32 = (const l32*)ibuf;
  auto dw = [&](uint32_t i) -> uint32_t { return g[min(i, nd - 1)]; };
  auto bytes4 = [&](uint32_t pos) -> uint32_t {  // the 4 stream bytes at pos (clamped at the end)
    const uint32_t a = sb0 + pos, i = a >> 2;
    if (((i + 1) << 2) - in.base < kIb && (i << 2) >= in.base)
      return __builtin_amdgcn_alignbyte(ib32[(i + 1) & (kIb / 4 - 1)], ib32[i & (kIb / 4 - 1)], a & 3);
    return __builtin_amdgcn_alignbyte(dw(i + 1), dw(i), a & 3);
  };
  l32* rlo = (l32*)ring;
  l32* rhi = rlo + 256;
  const uint32_t f_lo = bytes4(0), f_hi = W == 8 ? bytes4(4) : 0u;
  uint32_t q = W;  // the next record's stream position
  for (uint32_t b0 = 0; b0 < n; b0 += 64) {
    const uint32_t r_end = min(b0 + 64, n);
    uint32_t i = b0 ? b0 : 1, start = 0, cerr = 0;
    while (i < r_end && !cerr) {  // record starts of rows [i, r_end), a window at a time
      in.slide(sb0 + q);
      uint32_t t1 = 0, dr = 0, ec = 0;
      {
        const uint32_t w4 = bytes4(q + 4 * lane), w5 = bytes4(q + 4 * lane + 4);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
          const uint32_t r = 4 * lane + k, x = q + r;
          uint32_t d = 0, e = 0;
          if (x + 2 > ilen) {
            e = ST_IO;  // header past the stream
          } else {
            const uint32_t h = __builtin_amdgcn_alignbyte(w5, w4, k) & 0xFFFFu;
            uint32_t sb = (h >> 6) & 7;
            if ((h & 0x3F) < 63 && sb == 0) sb = 8;
            d = 2 + sb;
            if (sb > (uint32_t)W) e = ST_OUT_OF_SPEC;  // the f32 desync (patas.rs:154-160)
            else if (x + d > ilen) e = ST_IO;
          }
          t1 |= ((e || r + d >= 255) ? 0xFFu : r + d) << (8 * k);
          dr |= d << (8 * k);
          ec |= e << (8 * k);
        }
      }
      const uint32_t x = wave_chain(t1);
      const bool valid = x != 0xFF;
      const uint32_t my_d = tab_at(dr, x), my_e = tab_at(ec, x);
      const uint64_t vm = __ballot(valid), em = __ballot(valid && my_e != 0);
      const uint32_t m = (uint32_t)__popcll(vm);
      const uint32_t fe = em ? (uint32_t)__builtin_ctzll(em) : 64u;
      const uint32_t take = min(min(m, fe), r_end - i);
      // record k of the window is row i + k, dealt to lane (i + k) & 63
      const uint32_t k = (lane - i) & 63;
      const uint32_t pos = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(q + x));
      if (k < take) start = pos;
      if (fe < m && fe < r_end - i) cerr = __builtin_amdgcn_readlane(my_e, fe) & 0xFFu;
      if (take) q += __builtin_amdgcn_readlane(x, take - 1) + __builtin_amdgcn_readlane(my_d, take - 1);
      i += take;
    }
    const uint32_t rows_ok = i, row = b0 + lane;
    uint32_t lo = 0, hi = 0, P = 0xFF;  // P: lane of the in-block reference, 0xFF = resolved
    bool bad = false;
    if (row == 0) {
      lo = f_lo;
      hi = f_hi;
    } else if (row < rows_ok) {
      const uint32_t w0 = bytes4(start), w1 = bytes4(start + 4), w2 = bytes4(start + 8);
      const uint32_t h = w0 & 0xFFFFu;
      const uint32_t rd = (h >> 9) & 0x7F, tz = h & 0x3F;
      uint32_t sb = (h >> 6) & 7;
      if (tz < 63 && sb == 0) sb = 8;
      uint64_t v = ((uint64_t)(w0 >> 16) | ((uint64_t)w1 << 16) | ((uint64_t)w2 << 48));
      v = sb >= 8 ? v : (v & ((1ull << (8 * sb)) - 1));
      const uint64_t xv = tz >= 8 * W ? 0ull : (uint64_t)(T)((T)v << tz);
      if (rd == 0 || rd > row) {
        bad = true;
      } else if (row - rd < b0) {
        const uint32_t j = (row - rd) & 255;
        lo = (uint32_t)xv ^ rlo[j];
        hi = (uint32_t)(xv >> 32) ^ rhi[j];
      } else {
        lo = (uint32_t)xv;
        hi = (uint32_t)(xv >> 32);
        P = row - rd - b0;
      }
    }
    if (__ballot(bad)) return ST_OUT_OF_SPEC;  // a reference before row 0 (rows before it are fine)
#pragma unroll
    for (int r = 0; r < 6; r++) {
      const int src_lane = (int)(P == 0xFF ? lane : P) << 2;
      const uint32_t nlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane, (int)lo);
      const uint32_t nhi = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane, (int)hi);
      const uint32_t nP = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane, (int)P);
      if (P != 0xFF) {
        lo ^= nlo;
        hi ^= nhi;
        P = nP;
      }
    }
    if (row < rows_ok) {
      rlo[row & 255] = lo;
      rhi[row & 255] = hi;
      if constexpr (W == 8) ((uint64_t*)dst)[row] = (uint64_t)lo | ((uint64_t)hi << 32);
      else ((uint32_t*)dst)[row] = lo;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (cerr) return cerr;
  }
  return ST_OK;
}


#include "sb_zstd.h"

// One wave expands the general-codec stream [src, src + csize) of `olen`
// bytes into LDS (FULL mode).  Returns a status code.
__device__ uint32_t expand_to_lds(uint32_t codec, const uint8_t* src, uint32_t csize, lds_u8* out, uint32_t olen) {
  WaveWin w;
  w.init(src, csize);
  WaveOut<false> o;
  o.ring = out;
  o.dst = nullptr;
  o.olen = olen;
  o.op = 0;
  const uint32_t p0 = (uint32_t)((uintptr_t)src & 3);
  if (codec == 1) return lz4_wave<false>(w, p0, p0 + csize, o);
  if (codec == 3) return snappy_wave<false>(w, p0, p0 + csize, o);
  return ST_NYI;  // Zstd reads its frame from LDS: zs::zstd_to_lds
}

// Patas (double/patas.rs:107-132): first value raw, then per value a u16
// (ref_diff 7b | sig_bytes 3b | tz 6b; sig 0 => 8 when tz < 63) and sig
// bytes; value = (v << tz) ^ out[i - ref_diff].  All NT threads call it.
//  1. record starts (wave 0): each lane sizes the records that would start at
//     4 of the window's 256 byte positions (2 + sig bytes from the header
//     alone); a scalar chase follows the true chain through the window and
//     deals the starts to lanes, 64 per flush, into the output slots;
//  2. values, 256 rows at a time: each thread parses its row's record, a
//     reference before the block reads the final value, references inside
//     the block resolve by pointer jumping (8 rounds of value ^= value[ref],
//     ref = ref[ref] through LDS).
// Errors keep the reference's order: the first bad record decides the code
// (a short stream is Io, sig bytes > width is the f32 desync OutOfSpec,
// patas.rs:154-160, a reference before row 0 OutOfSpec).
template <int W>
__device__ uint32_t patas_expand(const lds_u8* in, uint32_t ilen, lds_u8* out, uint32_t n, Shared& sh) {
  using T = typename VT<W>::T;
  // the RLE scratch of Shared is idle here (the expanded stream decodes as None):
  // jump values (lo / hi words), jump targets, the first error
  static_assert(kRleFastRows / 32 >= NT, "Patas jump arrays alias the RLE scratch");
  uint32_t* pa_Alo = sh.rle_bits;
  uint32_t* pa_Ahi = sh.rle_start;
  uint16_t* pa_P = sh.rle_pref;
  uint32_t& pa_err = sh.rle_flags;  // (record index << 3) | status of the first bad record, ~0u = none
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  typedef __attribute__((address_space(3))) T lT;
  typedef __attribute__((address_space(3))) uint32_t l32;
  lT* o = (lT*)out;
  if (n == 0) return ST_OUT_OF_SPEC;  // `length - 1` underflows (patas.rs:117)
  if (ilen < W) return ST_IO;
  if (tid == 0) pa_err = 0xFFFFFFFFu;
  uint32_t found = 1;  // records whose start is known: rows [1, found)
  if (tid < 64) {
    uint32_t p = W, i = 1, starts = 0, err = 0;
    while (i < n && !err) {
      uint32_t packed = 0;
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t x = p + 4 * lane + k;
        uint32_t d = 0xFF;  // header past the stream
        if (x + 2 <= ilen) {
          const uint32_t h = in[x] | ((uint32_t)in[x + 1] << 8);
          uint32_t sb = (h >> 6) & 7;
          if ((h & 0x3F) < 63 && sb == 0) sb = 8;
          d = sb > (uint32_t)W ? 0xFE : 2 + sb;
        }
        packed |= d << (8 * k);
      }
      uint32_t q = p;
      while (i < n && q - p < 256) {
        const uint32_t r = q - p;
        const uint32_t d = (__builtin_amdgcn_readlane(packed, r >> 2) >> ((r & 3) * 8)) & 0xFFu;
        if (d == 0xFF || (d != 0xFE && q + d > ilen)) { err = ST_IO; break; }
        if (d == 0xFE) { err = ST_OUT_OF_SPEC; break; }
        starts = lane == (i & 63) ? q : starts;
        if ((i & 63) == 63) ((l32*)(out + (uint64_t)(i - 63) * W))[lane * (W / 4)] = starts;
        q += d;
        i++;
      }
      p = q;
    }
    const uint32_t i0 = i & ~63u;  // the partial group of starts
    if (lane < (i & 63)) ((l32*)(out + (uint64_t)i0 * W))[lane * (W / 4)] = starts;
    if (tid == 0) {
      sh.walk_off = i;
      if (err) pa_err = (i << 3) | err;
    }
  }
  __syncthreads();
  found = sh.walk_off;
  if (tid == 0) {
    T first = 0;
    for (int b = 0; b < W; b++) first |= (T)in[b] << (8 * b);
    o[0] = first;
  }
  __syncthreads();
  const uint32_t nv = found;  // rows with a parsed record (row 0 is the first value)
  for (uint32_t b0 = 0; b0 < nv; b0 += NT) {
    const uint32_t i = b0 + tid;
    uint64_t A = 0;
    uint32_t P = 0xFFFF;  // 0xFFFF: resolved
    if (i < nv && i > 0) {
      const uint32_t q = ((const l32*)(out + (uint64_t)i * W))[0];
      const uint32_t h = in[q] | ((uint32_t)in[q + 1] << 8);
      const uint32_t rd = (h >> 9) & 0x7F, tz = h & 0x3F;
      uint32_t sb = (h >> 6) & 7;
      if (tz < 63 && sb == 0) sb = 8;
      uint64_t v = 0;
      for (uint32_t k = 0; k < sb; k++) v |= (uint64_t)in[q + 2 + k] << (8 * k);
      A = tz >= 8 * W ? 0 : (uint64_t)(T)((T)v << tz);
      if (rd == 0 || rd > i) {
        atomicMin(&pa_err, (i << 3) | ST_OUT_OF_SPEC);
      } else if (i - rd < b0) {
        A ^= (uint64_t)o[i - rd];
      } else {
        P = i - rd - b0;
      }
    } else if (i == 0) {
      A = (uint64_t)o[0];
    }
#pragma unroll 1
    for (uint32_t r = 0; r < 8; r++) {
      pa_Alo[tid] = (uint32_t)A;
      pa_Ahi[tid] = (uint32_t)(A >> 32);
      pa_P[tid] = (uint16_t)P;
      __syncthreads();
      if (P != 0xFFFF) {
        A ^= (uint64_t)pa_Alo[P] | ((uint64_t)pa_Ahi[P] << 32);
        P = pa_P[P];
      }
      __syncthreads();
    }
    if (i < nv) o[i] = (T)A;
    __syncthreads();
  }
  const uint32_t e = pa_err;
  __syncthreads();
  return e == 0xFFFFFFFFu ? ST_OK : (e & 7);
}

// read_validity (read/read_basic.rs:36-63): [def_len u32][ULEB128 h, h&1 =
// bit-packed, h>>1 groups][bitmap].  An RLE run (unreachable!() at :59) or
// fewer than n bits is OutOfSpec; def_len 0 pushes nothing, which only an
// empty page survives.  Thread 0; advances *p past the prefix.
template <class Src>
__device__ __forceinline__ bool parse_validity(const Src& s, Shared& sh, uint32_t len, uint32_t n, uint32_t* pp) {
  uint32_t p = *pp;
  if (p + 4 > len) { set_err(sh, ST_IO); return false; }
  const uint32_t def_len = s.u32(p);
  p += 4;
  if (def_len == 0) {
    if (n) { set_err(sh, ST_OUT_OF_SPEC); return false; }
    *pp = p;
    return true;
  }
  if (def_len > len - p) { set_err(sh, ST_IO); return false; }
  uint32_t q = p, h = 0, sft = 0;
  for (;;) {
    if (q >= p + def_len || sft > 28) { set_err(sh, ST_OUT_OF_SPEC); return false; }
    const uint32_t c = s.u8(q++);
    h |= (c & 0x7Fu) << sft;
    if (!(c & 0x80)) break;
    sft += 7;
  }
  if (!(h & 1)) { set_err(sh, ST_OUT_OF_SPEC); return false; }
  const uint32_t groups = min(h >> 1, p + def_len - q);
  if ((uint64_t)groups * 8 < n) { set_err(sh, ST_OUT_OF_SPEC); return false; }
  sh.has_valid = 1;
  sh.vb_pos = q;
  *pp = p + def_len;
  return true;
}

// Cascade shapes the writer produces (Dict forbids Dict below it, Freq forbids
// Freq: dict.rs:60-62, freq.rs:79-83).
enum : uint32_t { CH_LEAF = 0, CH_DICT = 1, CH_FREQ = 2, CH_DICT_FREQ = 3, CH_FREQ_DICT = 4 };

// A page's HBM region (PageDesc.reserved, planned by sb_api's fixed-width
// plan): the roaring container tables of a Freq page with many containers,
// then the area a spilled leaf stream expands into.
__device__ __forceinline__ uint8_t* region_roar(const LaunchArgs& a, const PageDesc& pd, uint32_t* cap) {
  *cap = 0;
  if (!a.region || !(pd.reserved & kRegionRoar)) return nullptr;
  *cap = (uint32_t)roar_cap(pd.num_values);
  return a.region + (pd.reserved & kRegionOffMask);
}
__device__ __forceinline__ uint8_t* region_spill(const LaunchArgs& a, const PageDesc& pd) {
  if (!a.region || !(pd.reserved & kRegionSpill)) return nullptr;
  return a.region + (pd.reserved & kRegionOffMask) + ((pd.reserved & kRegionRoar) ? roar_area_bytes(pd.num_values) : 0);
}

// Values of a parsed page (sh.chain / sh.sub / Dict / Freq state): the leaf
// stream is read from `ls`, the page's dictionary and roaring bitmap from `s`.
template <int W, class Src, class LSrc>
__device__ __forceinline__ void decode_values(const Src& s, const LSrc& ls, Shared& sh, const PageDesc& pd, const LaunchArgs& a) {
  using T = typename VT<W>::T;
  const uint32_t tid = threadIdx.x;
  const uint32_t n = pd.num_values;
  uint8_t* obase = a.out_values + pd.row_off * W;
  // quads of 4- and 8-byte values leave as one 16-byte store at any dword
  // alignment (global_store_dwordx4 needs 4-byte alignment only; C4's leaf
  // bases are arbitrary rows: 0.175 -> 0.156 ms a step against four dword
  // stores per quad); 1- and 2-byte values need the quad's natural alignment
  GSink<W> out{obase, W >= 4 ? ((uintptr_t)obase & 3) == 0 : ((uintptr_t)obase & (uintptr_t)(4 * W - 1)) == 0};
  const uint32_t chain = sh.chain;
  const Stream leaf = sh.sub;
  const uint32_t k = sh.dict_k, doff = sh.dict_off;

  if (chain == CH_LEAF) {
    run_leaf<W>(ls, sh, leaf, [&](uint32_t row, const T* v, uint32_t nv) { out.put4(row, v, nv); });
    return;
  }
  if (chain == CH_DICT) {
    // Dict: u32 index leaf stream -> gather from the plain dictionary
    run_leaf<4>(ls, sh, leaf, [&](uint32_t row, const uint32_t* idx, uint32_t nv) {
      T v[4];
      bool bad = false;
#pragma unroll
      for (uint32_t l = 0; l < 4; l++) {
        const bool ok = l < nv && idx[l] < k;
        bad |= (l < nv && !ok);
        v[l] = ok ? ldv<W>(s, doff + idx[l] * W) : (T)0;
      }
      if (bad) set_err(sh, ST_OUT_OF_SPEC);  // data[i] out of range panics
      out.put4(row, v, nv);
    });
    return;
  }
  // Freq at the top (CH_FREQ, CH_FREQ_DICT) or under the Dict (CH_DICT_FREQ):
  // fill every row, then scatter the exceptions at their roaring rows.
  if (sh.roar_pending) {
    uint32_t cap;
    uint8_t* tabs = region_roar(a, pd, &cap);
    roaring_build(s, sh, tabs, cap);
    if (sh.err) return;
  }
  T fill;
  if (chain == CH_DICT_FREQ) {
    const uint32_t ti = (uint32_t)sh.freq_top;
    if (ti >= k && leaf.n < n) { if (tid == 0) set_err(sh, ST_OUT_OF_SPEC); return; }
    fill = ti < k ? ldv<W>(s, doff + ti * W) : (T)0;
  } else {
    fill = (T)sh.freq_top;
  }
  for (uint32_t q = tid; q < (n + 3) / 4; q += NT) {
    T v[4] = {fill, fill, fill, fill};
    out.put4(4 * q, v, min(4u, n - 4 * q));
  }
  __syncthreads();  // the scatter below overwrites rows of the fill
  auto scatter = [&](uint32_t i0, const T* x, uint32_t nv) {
    for (uint32_t l = 0; l < nv; l++) {
      const uint32_t row = roaring_select(s, sh, i0 + l);
      if (row < n) out.put(row, x[l]);
      else set_err(sh, ST_OUT_OF_SPEC);  // output[begin + val] out of range panics
    }
  };
  if (chain == CH_FREQ) {
    run_leaf<W>(ls, sh, leaf, scatter);
  } else {
    run_leaf<4>(ls, sh, leaf, [&](uint32_t i0, const uint32_t* idx, uint32_t nv) {
      T v[4];
      bool bad = false;
#pragma unroll
      for (uint32_t l = 0; l < 4; l++) {
        const bool ok = l < nv && idx[l] < k;
        bad |= (l < nv && !ok);
        v[l] = ok ? ldv<W>(s, doff + idx[l] * W) : (T)0;
      }
      if (bad) set_err(sh, ST_OUT_OF_SPEC);
      scatter(i0, v, nv);
    });
  }
}

__device__ __forceinline__ bool general_codec(uint32_t c) { return c == 1 || c == 2 || c == 3 || c == 16; }

// MODE 0: main pass (general-codec / Patas leaves are deferred to a work
// list); MODE 1: deferred pass (the leaf is expanded into LDS at `xpos`,
// xcap bytes available, then decoded as a plain stream; a leaf that does not
// fit -- or any leaf of a page too large to stage (xcap 0) -- is queued for
// k_inflate / k_zinflate to expand into the page's HBM region, sh.defer = 3);
// MODE 2: spilled pass (that expanded leaf, read from `lsrc` as a None stream).
// Z: the instantiation carries the Zstd decoder (sb_zstd.h).  Its out-of-line
// calls make a kernel take the decoder's registers (245 VGPRs, one wave a
// SIMD), so plans without Zstd streams launch Z = false kernels.
template <int W, bool FLT, int MODE, bool Z, class Src>
__device__ __forceinline__ void decode_page(const Src& s, Shared& sh, const PageDesc& pd, const LaunchArgs& a, uint32_t page,
                            uint8_t* xbuf = nullptr, uint32_t xpos = 0, uint32_t xcap = 0,
                            const GlbSrc* lsrc = nullptr) {
  const uint32_t tid = threadIdx.x;
  const uint32_t len = pd.byte_len, n = pd.num_values;

  if (tid == 0) {
    uint32_t p = 0;
    sh.has_valid = 0;
    sh.defer = 0;
    sh.roar_pending = 0;
    do {
      if (a.nullable && !parse_validity(s, sh, len, n, &p)) break;
      Stream st;
      if (!parse_stream(s, p, len, n, &st)) { set_err(sh, ST_IO); break; }
      uint32_t chain = CH_LEAF;
      Stream inner;
      if (st.codec == 11) {
        if (!parse_dict(s, sh, st, W, &inner)) break;
        chain = CH_DICT;
        if (inner.codec == 13) {
          Stream ex;
          if (!parse_freq(s, sh, inner, 4, &ex)) break;
          chain = CH_DICT_FREQ;
          inner = ex;
        }
      } else if (st.codec == 13) {
        if (!parse_freq(s, sh, st, W, &inner)) break;
        chain = CH_FREQ;
        if (inner.codec == 11) {
          Stream ix;
          if (!parse_dict(s, sh, inner, W, &ix)) break;
          chain = CH_FREQ_DICT;
          inner = ix;
        }
      } else {
        inner = st;
      }
      if (inner.codec == 11 || inner.codec == 13) { set_err(sh, ST_OUT_OF_SPEC); break; }
      if (FLT && (inner.codec == 14 || inner.codec == 15) && (chain == CH_LEAF || chain == CH_FREQ)) {
        set_err(sh, ST_OUT_OF_SPEC);  // no Bitpacking in decompress_double
        break;
      }
      sh.top = st;
      sh.sub = inner;
      sh.chain = chain;
      if (general_codec(inner.codec)) {
        if (MODE == 0) {
          if (chain == CH_LEAF && (inner.codec == 1 || inner.codec == 3 || (FLT && inner.codec == 16))) {
            // plain values under LZ4 / Snappy, or a Patas stream: k_inflate
            // writes them straight into the column, one wave per page
            sh.defer = 2;
            const uint32_t slot = atomicAdd(a.job_count + a.parity, 1u);
            a.jobs[slot] = InflateJob{pd.byte_off + inner.body, pd.row_off * W, inner.csize, inner.n * (uint32_t)W,
                                      inner.codec == 16 ? 16u | ((uint32_t)W << 8) : inner.codec, page};
          } else {
            sh.defer = 1;
            const uint32_t slot = atomicAdd(a.defer_count + a.parity, 1u);
            a.defer_list[slot] = page;
          }
        } else if (MODE == 2) {
          // expanded by k_inflate / k_zinflate into the region: a None stream there
          const bool idx_stream = chain == CH_DICT || chain == CH_FREQ_DICT || chain == CH_DICT_FREQ;
          sh.sub = Stream{0u, 0u, inner.n * (idx_stream ? 4u : (uint32_t)W), inner.n};
        }
      } else if (MODE == 2) {
        set_err(sh, ST_OUT_OF_SPEC);  // (the page changed under the plan)
      }
    } while (0);
  }
  __syncthreads();
  if (sh.err) return;
  // validity is written by the main pass, deferred pages included
  if (MODE == 0 && sh.has_valid) write_validity(s, sh.vb_pos, n, pd.row_off, a.out_validity);
  if (sh.defer) return;

  if constexpr (MODE == 1) {
    Stream lf = sh.sub;
    if (general_codec(lf.codec)) {
      const bool idx_stream = sh.chain == CH_DICT || sh.chain == CH_FREQ_DICT || sh.chain == CH_DICT_FREQ;
      const uint32_t sw = idx_stream ? 4u : (uint32_t)W;
      const uint64_t bytes = (uint64_t)lf.n * sw;
      const uint64_t zt = (bytes + 15) & ~15ull;  // Zstd: its tables after the expanded stream
      if ((lf.codec == 2 ? zt + kZTablesBytes : bytes) > xcap) {
        // the expansion does not fit the LDS: spill it into the page's HBM region
        if (tid == 0) {
          uint8_t* sp = region_spill(a, pd);
          if (lf.codec == 16 && (!FLT || idx_stream)) {
            set_err(sh, ST_OUT_OF_SPEC);  // Patas only in decompress_double
          } else if (!sp || bytes > spill_area_bytes(n, W)) {
            set_err(sh, ST_NYI);
          } else {
            const uint32_t slot = atomicAdd(a.spill_count + a.parity, 1u);
            a.spill_jobs[slot] = InflateJob{pd.byte_off + lf.body, kDstScratch | (uint64_t)(sp - a.region), lf.csize,
                                            (uint32_t)bytes, lf.codec == 16 ? 16u | (sw << 8) : lf.codec, page};
            sh.defer = 3;
          }
        }
        __syncthreads();
        return;
      }
      if constexpr (std::is_same<Src, LdsSrc>::value) {
        if (lf.codec == 16) {  // Patas: every thread of the workgroup
          const lds_u8* in = (const lds_u8*)((const uint8_t*)s.w + s.base + lf.body);
          uint32_t st;
          if (!FLT || idx_stream) st = ST_OUT_OF_SPEC;  // Patas only in decompress_double
          else st = patas_expand<W>(in, lf.csize, (lds_u8*)xbuf, lf.n, sh);
          if (st && tid == 0) set_err(sh, st);
        } else if (tid < 64) {
          lds_u8* xo = (lds_u8*)xbuf;
          uint32_t st = ST_OK;
          if (lf.codec == 1 || lf.codec == 3)
            st = expand_to_lds(lf.codec, a.chunk + pd.byte_off + lf.body, lf.csize, xo, (uint32_t)bytes);
          else if constexpr (Z)
            st = zs::zstd_to_lds(LdsSrc{s.w, s.base + lf.body}, lf.csize, xo, (uint32_t)bytes, xo + zt,
                                 (uint32_t)(xcap - zt));
          else
            st = ST_NYI;  // (a plan with Zstd streams launches the Z kernels)
          if (st) set_err(sh, st);
        }
        __syncthreads();
        if (sh.err) return;
        if (tid == 0) sh.sub = Stream{0u, xpos - s.base, (uint32_t)bytes, lf.n};
        __syncthreads();
      }
    }
  }

  if constexpr (MODE == 2) decode_values<W>(s, *lsrc, sh, pd, a);
  else decode_values<W>(s, s, sh, pd, a);
}

// Stage [pg, pg + len) into LDS with aligned 16-byte pieces.
__device__ __forceinline__ uint32_t stage_page(u32x4* stage, const uint8_t* pg, uint32_t len) {
  const uintptr_t a0 = (uintptr_t)pg & ~(uintptr_t)15;
  const uint32_t base = (uint32_t)((uintptr_t)pg & 15);
  const uint32_t nchunks = (base + len + 15) >> 4;
  const u32x4* gsrc = (const u32x4*)a0;
#if SB_LDS_DMA
  {  // LDS-DMA: each wave instruction lands 64 x 16 B contiguously at the wave's LDS base
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t c0 = wv * 64; c0 < nchunks; c0 += NT) {
      if (c0 + lane < nchunks)
        __builtin_amdgcn_global_load_lds((const void*)(gsrc + c0 + lane), (__attribute__((address_space(3))) void*)(stage + c0),
                                         16, 0, SB_LOAD_NT ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#else
  for (uint32_t c = threadIdx.x; c < nchunks; c += NT) {
#if SB_LOAD_NT
    stage[c] = __builtin_nontemporal_load(gsrc + c);
#else
    stage[c] = gsrc[c];
#endif
  }
#endif
  __syncthreads();
  return base;
}

// The validity prefix as parse_validity reads it (one thread, from HBM):
// false for anything but a valid bit-packed prefix of a non-empty page.
__device__ bool light_validity(const GlbSrc& s, uint32_t len, uint32_t n, int nullable, uint32_t* pp, uint32_t* vbpos) {
  uint32_t p = 0;
  *vbpos = 0;
  if (n == 0) return false;
  if (nullable) {
    if (len < 4) return false;
    const uint32_t def_len = s.u32(0);
    p = 4;
    if (def_len == 0 || def_len > len - p) return false;
    uint32_t q = p, h = 0, sft = 0;
    for (;;) {
      if (q >= p + def_len || sft > 28) return false;
      const uint32_t c = s.u8(q++);
      h |= (c & 0x7Fu) << sft;
      if (!(c & 0x80)) break;
      sft += 7;
    }
    if (!(h & 1)) return false;
    if ((uint64_t)min(h >> 1, p + def_len - q) * 8 < n) return false;
    *vbpos = q;  // >= 5: 0 means no bitmap
    p += def_len;
  }
  *pp = p;
  return true;
}

// A slot of `per` entries for each active lane with `want`, from one atomic
// on *ctr per wave (lanes in lane order).
__device__ __forceinline__ uint32_t wave_slot(uint32_t* ctr, bool want, uint32_t per) {
  const uint64_t m = __ballot(want);
  if (!m) return 0;
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  uint32_t base = 0;
  if ((threadIdx.x & 63) == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m) * per);
  base = (uint32_t)__shfl((int)base, (int)leader, 64);
  return base + rank * per;
}

// Header-only fixed-width pages: the leaf is LZ4 / Snappy (or, for Float
// columns, Patas) with no cascade, so the page needs no staging: one thread
// reads the validity prefix and the stream header from HBM (the checks of
// decode_page), appends the k_inflate job and tags the page; the staged /
// global passes then only copy its validity bits.
__global__ __launch_bounds__(NT) void k_fix_light(LaunchArgs a, uint32_t n_pages, uint32_t W, uint32_t flt,
                                                   uint32_t* light) {
  for (uint32_t page = blockIdx.x * NT + threadIdx.x; page < n_pages; page += gridDim.x * NT) {
    const PageDesc pd = a.pages[page];
    const GlbSrc s{a.chunk + pd.byte_off};
    const uint32_t len = pd.byte_len, n = pd.num_values;
    uint32_t p = 0, vb = 0, codec = 0, cs = 0;
    bool lt = light_validity(s, len, n, a.nullable, &p, &vb) && p + 9 <= len;
    if (lt) {
      codec = s.u8(p);
      cs = s.u32(p + 1);
      // Zstd leaves whose page + expansion exceed the deferred pass's LDS
      // expand straight into the column (k_zinflate)
      const bool zbig = codec == 2 && (uint64_t)len + (uint64_t)n * W + kZTablesMax + 1024 > kDeferredLds;
      lt = cs <= len - (p + 9) && (codec == 1 || codec == 3 || (flt && codec == 16) || zbig);
    }
    const uint32_t slot = wave_slot(a.job_count + a.parity, lt, 1);
    if (lt) {
      a.jobs[slot] = InflateJob{pd.byte_off + p + 9, pd.row_off * W, cs, n * W, codec == 16 ? 16u | (W << 8) : codec, page};
      a.status[page] = 0;
    }
    light[page] = lt ? 1 + vb : 0u;
  }
}

// A header-only page in the staged / global passes: its validity bits only.
__device__ __forceinline__ bool light_page(const LaunchArgs& a, const PageDesc& pd, uint32_t page) {
  const uint32_t lt = a.light ? a.light[page] : 0u;
  if (!lt) return false;
  if (lt > 1) write_validity(GlbSrc{a.chunk + pd.byte_off}, lt - 1, pd.num_values, pd.row_off, a.out_validity);
  return true;
}

template <int W, bool FLT>
__global__ __launch_bounds__(NT) void k_decode_staged(LaunchArgs a) {
  extern __shared__ u32x4 stage[];
  __shared__ Shared sh;
  const uint32_t page = a.list ? a.list[blockIdx.x] : blockIdx.x;
  const PageDesc pd = a.pages[page];
  if (threadIdx.x == 0) {
    sh.err = 0;
    if (blockIdx.x == 0) {  // the next decode's work lists
      a.defer_count[a.parity ^ 1] = 0;
      a.job_count[a.parity ^ 1] = 0;
      if (a.spill_count) a.spill_count[a.parity ^ 1] = 0;
    }
  }
  if (light_page(a, pd, page)) return;
  const uint32_t base = stage_page(stage, a.chunk + pd.byte_off, pd.byte_len);
  LdsSrc s{(const uint32_t*)stage, base};
  decode_page<W, FLT, 0, false>(s, sh, pd, a, page);
  __syncthreads();
  if (threadIdx.x == 0 && sh.defer != 1) a.status[page] = sh.err;
}

template <int W, bool FLT>
__global__ __launch_bounds__(NT) void k_decode_global(LaunchArgs a) {
  __shared__ Shared sh;
  const uint32_t page = a.list ? a.list[blockIdx.x] : blockIdx.x;
  const PageDesc pd = a.pages[page];
  if (threadIdx.x == 0) sh.err = 0;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    a.defer_count[a.parity ^ 1] = 0;
    a.job_count[a.parity ^ 1] = 0;
    if (a.spill_count) a.spill_count[a.parity ^ 1] = 0;
  }
  if (light_page(a, pd, page)) return;
  GlbSrc s{a.chunk + pd.byte_off};
  decode_page<W, FLT, 0, false>(s, sh, pd, a, page);
  __syncthreads();
  if (threadIdx.x == 0 && sh.defer != 1) a.status[page] = sh.err;
}

// Deferred pages (general codecs, Patas): one workgroup per listed page, the
// page and its expanded leaf stream both in LDS (a.stage_bytes in total).
template <int W, bool FLT, bool Z>
__global__ __launch_bounds__(NT) void k_decode_deferred(LaunchArgs a) {
  extern __shared__ u32x4 stage[];
  __shared__ Shared sh;
  const uint32_t count = a.defer_count[a.parity];
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    const uint32_t page = a.defer_list[i];
    const PageDesc pd = a.pages[page];
    if (threadIdx.x == 0) sh.err = 0;
    const uint64_t need = align16((uint64_t)pd.byte_len + 15 + kStagePad);
    if (need + 64 > a.stage_bytes) {
      // page too large to stage: parsed from HBM, its leaf spills into the
      // page's region (NYI when the plan reserved none)
      decode_page<W, FLT, 1, Z>(GlbSrc{a.chunk + pd.byte_off}, sh, pd, a, page);
      __syncthreads();
      if (threadIdx.x == 0) a.status[page] = sh.err;
      __syncthreads();
      continue;
    }
    const uint32_t base = stage_page(stage, a.chunk + pd.byte_off, pd.byte_len);
    LdsSrc s{(const uint32_t*)stage, base};
    uint8_t* xbuf = (uint8_t*)stage + need;
    decode_page<W, FLT, 1, Z>(s, sh, pd, a, page, xbuf, (uint32_t)need, a.stage_bytes - (uint32_t)need - kStagePad);
    __syncthreads();
    if (threadIdx.x == 0) a.status[page] = sh.err;
    __syncthreads();
  }
}

// Spilled pages: their leaf was expanded into the page's HBM region by
// k_inflate / k_zinflate (an error there stands); the page is parsed again
// from HBM and decoded with that expansion as a None leaf stream.
template <int W, bool FLT>
__global__ __launch_bounds__(NT) void k_decode_spilled(LaunchArgs a) {
  __shared__ Shared sh;
  const uint32_t count = a.spill_count[a.parity];
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    const InflateJob jb = a.spill_jobs[i];
    const uint32_t page = jb.page;
    if (a.status[page]) continue;
    const PageDesc pd = a.pages[page];
    if (threadIdx.x == 0) sh.err = 0;
    const GlbSrc ls{a.region + (jb.dst & kDstMask)};
    decode_page<W, FLT, 2, false>(GlbSrc{a.chunk + pd.byte_off}, sh, pd, a, page, nullptr, 0, 0, &ls);
    __syncthreads();
    if (threadIdx.x == 0) a.status[page] = sh.err;
    __syncthreads();
  }
}

// Plan-time cascade walk of a fixed-width (or Boolean: W 1, one stream) page
// from HBM, the header walk of decode_page without the tables: bit 0 a Freq
// in the cascade, bit 1 a general-codec / Patas leaf, bit 2 under a Dict /
// Freq, bit 3 some stream of the cascade is Zstd, bit 4 some stream is Patas,
// bit 5 some stream is LZ4 / Snappy.
__device__ uint32_t fix_cascade(const GlbSrc& s, uint32_t len, uint32_t W, int nullable) {
  uint32_t p = 0, bits = 0;
  auto hdr = [&](uint32_t q, uint32_t* codec, uint32_t* body, uint32_t* cs) {
    if (q + 9 > len) return false;
    *codec = s.u8(q);
    *cs = s.u32(q + 1);
    *body = q + 9;
    if (*codec == 2) bits |= 8;
    if (*codec == 16) bits |= 16;
    if (*codec == 1 || *codec == 3) bits |= 32;
    return *cs <= len - *body;
  };
  do {
    if (nullable) {
      if (len < 4) break;
      const uint32_t dl = s.u32(0);
      if (dl > len - 4) break;
      p = 4 + dl;
    }
    uint32_t c0, b0, cs0, c1, b1, cs1;
    if (!hdr(p, &c0, &b0, &cs0)) break;
    uint32_t leaf = c0;
    if (c0 == 11 || c0 == 13) {
      bits |= 4;
      uint32_t q;
      if (c0 == 11) {
        q = b0;  // the index stream
      } else {
        bits |= 1;
        if (b0 + W + 4 > len) break;
        q = b0 + W + 4 + s.u32(b0 + W);  // past top value and bitmap: the exceptions stream
      }
      if (!hdr(q, &c1, &b1, &cs1)) break;
      leaf = c1;
      if (c1 == 11 || c1 == 13) {  // Dict -> Freq or Freq -> Dict
        uint32_t c2, b2, cs2;
        if (c1 == 11) {
          q = b1;
        } else {
          bits |= 1;
          if (b1 + 8 > len) break;
          q = b1 + 8 + s.u32(b1 + 4);  // Freq of u32 indices: u32 top, u32 bitmap size
        }
        if (!hdr(q, &c2, &b2, &cs2)) break;
        leaf = c2;
      }
    }
    if (general_codec(leaf)) bits |= 2;
  } while (0);
  return bits;
}

// The cascade bits of each listed page (fix_cascade), one thread per page.
__global__ __launch_bounds__(NT) void k_fix_probe(const uint8_t* chunk, const PageDesc* pages, const uint32_t* list,
                                                  uint32_t n_list, uint32_t W, int nullable, uint32_t* probe) {
  const uint32_t i = blockIdx.x * NT + threadIdx.x;
  if (i >= n_list) return;
  const PageDesc pd = pages[list[i]];
  probe[i] = fix_cascade(GlbSrc{chunk + pd.byte_off}, pd.byte_len, W, nullable);
}

// Plan time: *flag |= 1 when some page has a Zstd stream (the plan then
// launches the kernels that carry the Zstd decoder), |= 2 when some page has
// a Patas stream (the inflate launches then start with k_patas), |= 4 when
// some page has an LZ4 / Snappy stream.
__global__ __launch_bounds__(NT) void k_zstd_scan(const uint8_t* chunk, const PageDesc* pages, uint32_t n, uint32_t W,
                                                  int nullable, uint32_t* flag) {
  const uint32_t i = blockIdx.x * NT + threadIdx.x;
  uint32_t c = 0;
  if (i < n) {
    const PageDesc pd = pages[i];
    c = fix_cascade(GlbSrc{chunk + pd.byte_off}, pd.byte_len, W, nullable);
  }
  const uint32_t f = (__ballot(c & 8) ? 1u : 0u) | (__ballot(c & 16) ? 2u : 0u) | (__ballot(c & 32) ? 4u : 0u);
  if (f && (threadIdx.x & 63) == 0) atomicOr(flag, f);
}

template <int W, bool FLT>
static int launch(int kind, const LaunchArgs& a, hipStream_t stream) {
  dim3 block(NT);
  if (kind == 3) {
    if (a.n_list == 0) return 0;
    hipLaunchKernelGGL((k_decode_spilled<W, FLT>), dim3(a.n_list), block, 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (kind == 2) {
    if (a.zstd) {
      ensure_lds_attr(k_decode_deferred<W, FLT, true>, (int)kDeferredLds);
      hipLaunchKernelGGL((k_decode_deferred<W, FLT, true>), dim3(a.n_list), block, a.stage_bytes, stream, a);
    } else {
      ensure_lds_attr(k_decode_deferred<W, FLT, false>, (int)kDeferredLds);
      hipLaunchKernelGGL((k_decode_deferred<W, FLT, false>), dim3(a.n_list), block, a.stage_bytes, stream, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (a.n_list == 0) return 0;
  dim3 grid(a.n_list);
  if (kind == 0) {
    hipLaunchKernelGGL((k_decode_staged<W, FLT>), grid, block, a.stage_bytes, stream, a);
  } else {
    hipLaunchKernelGGL((k_decode_global<W, FLT>), grid, block, 0, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// General-codec streams expanded straight into HBM, one wave per stream, each
// wave with its own kRing-byte LDS history ring: 4 waves x 4 KiB per
// workgroup, so 8 waves per SIMD can be resident and the serial token streams
// of many pages overlap.
#ifndef SB_INF_BLOCKS
#ifdef SB_INF_RING4K
#define SB_INF_BLOCKS 6  // 4-wave workgroups: 6 waves per SIMD (6.5 KiB of LDS and <= 80 VGPRs a wave)
#else
#define SB_INF_BLOCKS 8  // 4-wave workgroups: 8 waves per SIMD (4.5 KiB of LDS and <= 64 VGPRs a wave)
#endif
#endif
__global__ __launch_bounds__(64 * kInfWaves, SB_INF_BLOCKS) void k_inflate(InflateLaunch a) {
  __shared__ u32x4 rings[kInfWaves][kRing / 16];
  __shared__ u32x4 ibufs[kInfWaves][kIb / 16];
#ifdef SB_INF_BPCHAIN
  u32x4* const ctabs[kInfWaves] = {};
#else
  __shared__ u32x4 ctabs[kInfWaves][kChainTabs * 256 / 16];
#endif
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n = a.count ? *a.count : a.n_jobs;
  // Jobs are claimed from a counter (a.sched[0]) as waves free up, so the
  // last wave slots do not idle behind a fixed job-to-wave assignment (a
  // static first job per wave measured 2.14 -> 2.55 ms on C3's Utf8 column).
  // Only the first min(waves, n) waves take part; the others leave at once,
  // so a launch with few or no jobs costs no same-address atomics per idle
  // wave (they serialize in L2, ~11 ns each: a full grid of 6144 waves spent
  // 70-140 us on a launch with no jobs).  The last taking-part wave out
  // (a.sched[1] counts them) zeroes both words for the next launch on the
  // stream.  (Reading the counter before each claim, to skip claims once
  // every job is taken, measured 2.14 -> 2.7 ms on that column: the loads
  // queue behind the claims on the one L2 line.)  Without a.sched:
  // grid-strided.
  const uint32_t waves = gridDim.x * kInfWaves, part = min(waves, n);
  uint32_t j = blockIdx.x * kInfWaves + wv;
  if (a.sched_spare && j == 0 && lane < 3) a.sched_spare[lane] = 0;
  // every job k_patas's (it counted the others in a.sched[2]): no claims at all
  if (a.patas_wg && a.sched && __builtin_nontemporal_load(&a.sched[2]) == 0) return;
  if (j >= part) return;
  for (bool first = true;; first = false) {
    if (a.sched) {
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(&a.sched[0], 1u);
      j = __builtin_amdgcn_readfirstlane(c);  // (every lane is active here: lane 0's claim, in an SGPR)
    } else if (!first) {
      j += waves;
    }
    if (j >= n) break;
    const InflateJob jb = a.jobs[j];
    if (jb.codec == 2) continue;  // k_zinflate's
    const uint64_t kind = jb.dst >> 62, off = jb.dst & kDstMask;
#ifdef SB_V_SKIPSCRATCH
    if (kind == 1) continue;
#endif
#ifdef SB_V_SKIPVALS
    if (kind == 2) continue;
#endif
    uint8_t* dst = kind == 1 ? a.scratch + off : kind == 3 ? a.offs + off : a.out + (kind == 2 ? a.bases[off] : off);
    const uint8_t* src = a.chunk + jb.src;
    WaveOut<true> o;
    o.xf = kind == 3;  // Utf8 offsets rebased onto the page's values base
    o.xadd = kind == 3 ? (uint32_t)a.bases[jb.page] : 0u;
    o.skip0 = kind == 3 && jb.page != 0;
    o.w0 = 0;
    o.ring = (lds_u8*)&rings[wv][0];
    o.dst = dst;
    o.rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)jb.usize, 0x00020000);
    o.dal = (uint32_t)((uintptr_t)dst & 3);
    o.rsa = __builtin_amdgcn_make_buffer_rsrc(dst - o.dal, 0, (int)(jb.usize + o.dal), 0x00020000);
    o.olen = jb.usize;
    o.op = 0;
    const uint32_t p0 = (uint32_t)((uintptr_t)src & 3);
    uint32_t st = ST_NYI;
    if (jb.codec == 1) {
      InRing in;
      in.g = (gmem_u32*)((uintptr_t)src & ~(uintptr_t)3);
      in.nd = (p0 + jb.csize + 3) >> 2;
      in.ib = (lds_u8*)&ibufs[wv][0];
      in.ct = (lds_u8*)&ctabs[wv][0];
      in.seek(p0);
      st = lz4_inflate(in, p0, p0 + jb.csize, o);
    }
#ifndef SB_V_LZ4ONLY
    else if (jb.codec == 3) {
      WaveWin w;
      w.init(src, jb.csize);
      st = snappy_wave<true>(w, p0, p0 + jb.csize, o);
    } else if ((jb.codec & 0xFF) == 16) {  // Patas leaf: codec 16 | width << 8
      const uint32_t W = jb.codec >> 8;
      if (a.patas_wg && kind <= 1 && patas_fits(jb.csize, jb.usize / W, W)) continue;  // k_patas's
      st = W == 8 ? patas_wave<8>(src, jb.csize, dst, jb.usize / 8, o.ring, (lds_u8*)&ibufs[wv][0])
                  : patas_wave<4>(src, jb.csize, dst, jb.usize / 4, o.ring, (lds_u8*)&ibufs[wv][0]);
    }
#endif
    if (st && lane == 0) a.status[jb.page] = st;
    if (kind == 2 && a.ascii && lane == 0) a.ascii[jb.page] = (st == ST_OK && !o.hib) ? 1 : 0;
  }
  if (a.sched && lane == 0 && atomicAdd(&a.sched[1], 1u) == part - 1) {
    a.sched[0] = 0;  // every taking part wave has claimed its last job: reset for the next launch
    a.sched[1] = 0;
  }
}

// Zstd frames larger than a workgroup's LDS (a fixed-width leaf stream, or a
// binary Basic page's offsets / values streams, whose expansion does not fit
// the staged passes): one wave per job reads the
// frame from HBM and writes the output straight into the column; only the
// decoder's FSE / Huffman tables and sequence batches live in LDS.  Output
// bytes are stored and re-read (matches, literals at the window's tail) by
// the same wave in program order.
__global__ __launch_bounds__(64) void k_zinflate(InflateLaunch a) {
  __shared__ u32x4 tabs[kZTablesMax / 16];
  const uint32_t n = a.count ? *a.count : a.n_jobs;
  for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
    const InflateJob jb = a.jobs[j];
    if (jb.codec != 2) continue;
    const uint64_t kind = jb.dst >> 62, off = jb.dst & kDstMask;
    if (kind == 3) continue;  // (Zstd offsets streams go through scratch)
    uint8_t* dst = kind == 1 ? a.scratch + off : kind == 2 ? a.out + a.bases[off] : a.out + off;
    const uint32_t st = zs::zstd_decode(GlbSrc{a.chunk + jb.src}, jb.csize, dst, jb.usize, (lds_u8*)&tabs[0], kZTablesMax);
    if (st && (threadIdx.x & 63) == 0) a.status[jb.page] = st;
  }
}

// ===========================================================================
// Binary / Utf8 pages (compression/binary/mod.rs:95-183, dict.rs:95-141,
// freq.rs:102-145, one_value.rs:71-99), assembled as read_binary does
// (read/array/binary.rs:223-265): per-page offsets rebased onto the running
// values length, values appended.  Pass 1 (k_bin_size) sizes each page's
// values; k_bin_scan turns sizes into bases; pass 2 (k_bin_decode) writes
// offsets, values and validity.  A workgroup holds its page, the expanded
// offsets / index stream, the expanded values and the entry table in LDS.
// ===========================================================================
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

struct BinArgs {
  const uint8_t* chunk;
  const PageDesc* pages;
  uint32_t n_pages;
  int nullable;
  uint64_t* sizes;   // pass 1 out: values bytes per page
  uint64_t* bases;   // scan out: first values byte of each page
  uint64_t* total;   // scan out
  uint8_t* out_offsets;
  uint8_t* out_values;
  uint64_t values_cap;
  uint32_t* out_validity;
  uint32_t* status;
  uint32_t lds_bytes;
  InflateJob* jobs;
  uint32_t* job_count;
  uint8_t* scratch;
  uint32_t* lds_need;  // plan time (k_bin_probe): LDS bytes per page
  uint32_t* cls;  // staged list [n] | header-only list [n] | validity bitmap positions [n] | big list [n] | 3 lengths
  uint8_t* region;     // big pages' tables (PageDesc.reserved = region offset + 1)
  uint64_t* rneed;     // plan time (k_bin_probe): region bytes per page
  uint64_t* lb;        // fused pass: look-back state per page, then the page counter (zeroed by the host)
  uint8_t* checked;    // fused pass, Utf8: per page, its rows are whole valid entries (BinLaunch::checked)
};

enum : uint32_t { BIN_BASIC = 0, BIN_ONE = 12, BIN_DICT = 11, BIN_FREQ = 13 };

// Rows per emission tile (bin_emit) and the LDS its row tables take.
constexpr uint32_t kEmitRows = 4 * NT;
constexpr uint32_t kEmitBytes = 8192;  // LDS window of the binary emission (bin_emit)
// Dynamic LDS of the big-page kernels: Zstd tables, one wave's inflate
// buffers (ring, input ring, chain tables), the emission tables.
constexpr uint32_t kBigZt = 0, kBigRing = kZTablesMax, kBigIb = kBigRing + kRing, kBigCt = kBigIb + kIb,
                   kBigEmit = kBigCt + 2048, kBigLds = kBigEmit + kEmitBytes;

struct BinInfo {
  uint32_t codec;      // leading codec byte
  uint32_t ob, ocs;    // Basic: offsets stream body / csize
  uint32_t vb, vcs;    // Basic: values stream body / csize
  uint64_t S;          // values bytes of the page
  uint32_t L, top;     // OneValue / Freq top: length and position
  uint32_t k;          // Dict entries / Freq exceptions consumed (rows < n)
  uint32_t q, end;     // Dict / Freq: first entry record, body end
  uint32_t tot;        // roaring cardinality (a Freq page, or a Dict's Freq index stream)
  uint32_t xcodec;     // a Dict's Freq index stream: its exceptions stream's codec
  uint32_t xoff, yoff; // Basic Zstd: LDS byte offsets of the expanded offsets / values
  uint32_t ztab;       // LDS byte offset of the Zstd decoder's tables
  uint32_t emit;       // LDS byte offset of the emission tables
  uint32_t need;       // LDS bytes the page needs
  // Extend tables (offsets from the tables' base: the LDS after the staged
  // page, or the page's HBM region): Dict indices (u32 per row) or the Freq
  // exception-row bitmap + its prefix (u32 per 32 rows each) at 0, the
  // (position, length) entry table, a Dict's expanded Freq exceptions, the
  // roaring container tables (region only)
  uint32_t tb;         // LDS: byte offset of the tables' base
  uint64_t otab, oxex, oroar;
};

// Typed table pointers: LDS (address space 3) for a staged page, global
// (address space 1) for a big page's region, so every access is a ds_ or a
// global_ instruction rather than a flat one.
template <bool L, class T>
using mptr = typename std::conditional<L, __attribute__((address_space(3))) T*, __attribute__((address_space(1))) T*>::type;
template <class Src>
constexpr bool kLdsSrc = std::is_same<Src, LdsSrc>::value;
template <bool L>
struct TabBase {
  typename std::conditional<L, lds_u8*, __attribute__((address_space(1))) uint8_t*>::type b;
  template <class T>
  __device__ __forceinline__ mptr<L, T> at(uint64_t off) const { return (mptr<L, T>)(b + off); }
};

// Table layout of an Extend page from its header counts (offsets from the
// tables' base; x at 0).  Shared by the plan-time probe and the parse.
struct BinLayout {
  uint64_t tab, xex, roar, end;
};
__device__ __forceinline__ BinLayout bin_layout(uint32_t codec, uint32_t n, uint32_t k, uint32_t tot, bool xex,
                                                bool roar) {
  BinLayout L;
  uint64_t p = codec == BIN_DICT ? align16(4ull * n) : codec == BIN_FREQ ? align16(8ull * ((n + 31) / 32)) : 0;
  L.tab = p;
  const uint64_t ent = codec == BIN_DICT ? k : codec == BIN_FREQ ? min(tot, n) : 0;
  p = align16(p + 8 * ent);
  L.xex = p;
  if (xex) p = align16(p + 4ull * tot);
  L.roar = p;
  if (roar) p += roar_area_bytes(n);
  L.end = p;
  return L;
}

// The Freq header of a u32 index stream [u32 top][u32 bm][roaring][exceptions]
// at body (thread 0): roaring cardinality and the exceptions' codec.
template <class Src>
__device__ bool idx_freq_header(const Src& s, uint32_t body, uint32_t end, uint32_t* tot, uint32_t* xcodec) {
  if (body + 8 > end) return false;
  const uint32_t bm = s.u32(body + 4), r = body + 8;
  if (bm > end - r || bm < 8) return false;
  const uint32_t nc = s.u32(r + 4);
  if (8 + 8 * (uint64_t)nc > bm) return false;
  uint64_t t = 0;
  for (uint32_t c = 0; c < nc; c++) t += (s.u32(r + 8 + 4 * c) >> 16) + 1;
  if (t > 0xFFFFFFFFull || r + bm + 9 > end) return false;
  *tot = (uint32_t)t;
  *xcodec = s.u8(r + bm);
  return true;
}

// Thread 0: validity prefix, binary header, and for Extend pages the counts
// that size the tables and where they go: LDS after the staged page
// (`lds`: stage_end..lds_bytes) or the page's HBM region (lds false).
// Records are not walked here (walk_records).  Returns false on error.
template <int OW, class Src>
__device__ bool bin_parse(const Src& s, Shared& sh, BinInfo& bi, const PageDesc& pd, int nullable, bool lds,
                          uint32_t stage_end, uint32_t lds_bytes, Stream* idx) {
  const uint32_t len = pd.byte_len, n = pd.num_values;
  uint32_t p = 0;
  sh.has_valid = 0;
  sh.roar_pending = 0;
  if (nullable && !parse_validity(s, sh, len, n, &p)) return false;
  if (p + 9 > len) { set_err(sh, ST_IO); return false; }
  bi.codec = s.u8(p);
  const uint32_t cs = s.u32(p + 1), body = p + 9;
  if (cs > len - body) { set_err(sh, ST_IO); return false; }
  const uint32_t end = body + cs;
  bi.xoff = stage_end;
  bi.S = 0;
  bi.k = 0;
  bi.tot = 0;
  bi.xcodec = 0;
  bi.need = stage_end + 64;
  bi.ztab = 0;
  bi.end = end;
  if (bi.codec <= 3) {  // Basic: offsets stream then values stream (same codec)
    bi.ob = body;
    bi.ocs = cs;
    const uint32_t vh = end;
    if (vh + 9 > len) { set_err(sh, ST_IO); return false; }
    bi.vcs = s.u32(vh + 1);
    bi.S = s.u32(vh + 5);
    bi.vb = vh + 9;
    if (bi.vcs > len - bi.vb) { set_err(sh, ST_IO); return false; }
    const uint32_t xb = ((n + 1) * OW + 15) & ~15u;
    bi.yoff = bi.xoff + xb;
    if (bi.codec == 2) {  // Zstd: offsets into X, values into Y, the decoder's tables after Y
      const uint64_t zt = ((uint64_t)bi.yoff + bi.S + 15) & ~15ull;
      bi.need = kDeferredLds;  // (the tables take the rest)
      if (lds && zt + kZTablesBytes + kStagePad > lds_bytes) { set_err(sh, ST_NYI); return false; }
      bi.ztab = (uint32_t)zt;
    }
    return true;
  }
  bool zstd = false, xex = false, roar = false;
  uint32_t k = 0;
  if (bi.codec == BIN_ONE) {
    if (cs < 4) { set_err(sh, ST_IO); return false; }
    bi.L = s.u32(body);
    if (bi.L > cs - 4) { set_err(sh, ST_OUT_OF_SPEC); return false; }
    bi.top = body + 4;
    bi.S = (uint64_t)n * bi.L;
  } else if (bi.codec == BIN_DICT) {
    Stream ix;
    if (!parse_stream(s, body, end, n, &ix)) { set_err(sh, ST_IO); return false; }
    if (ix.codec == 11) { set_err(sh, ST_OUT_OF_SPEC); return false; }
    *idx = ix;
    uint32_t q = ix.body + ix.csize;
    if (q + 4 > end) { set_err(sh, ST_IO); return false; }
    k = s.u32(q);
    bi.q = q + 4;
    zstd = ix.codec == 2;
    if (ix.codec == 13) {
      if (!idx_freq_header(s, ix.body, ix.body + ix.csize, &bi.tot, &bi.xcodec)) { set_err(sh, ST_IO); return false; }
      if (bi.xcodec == 11 || bi.xcodec == 13) { set_err(sh, ST_OUT_OF_SPEC); return false; }
      xex = bi.xcodec == 1 || bi.xcodec == 2 || bi.xcodec == 3;
      zstd = bi.xcodec == 2;
      roar = true;
    }
    bi.k = k;
  } else if (bi.codec == BIN_FREQ) {
    if (cs < 8) { set_err(sh, ST_IO); return false; }
    const uint64_t tl = s.u64(body);
    uint32_t q = body + 8;
    if (tl > end - q) { set_err(sh, ST_OUT_OF_SPEC); return false; }
    bi.L = (uint32_t)tl;
    bi.top = q;
    q += bi.L;
    if (q + 4 > end) { set_err(sh, ST_IO); return false; }
    const uint32_t bm = s.u32(q);
    q += 4;
    if (bm > end - q) { set_err(sh, ST_IO); return false; }
    if (!parse_roaring(s, sh, q, bm, &bi.tot)) return false;
    bi.q = q + bm;
    roar = true;
  } else {
    set_err(sh, ST_OUT_OF_SPEC);
    return false;
  }
  const BinLayout L = bin_layout(bi.codec, n, k, bi.tot, xex, roar && !lds);
  bi.otab = L.tab;
  bi.oxex = L.xex;
  bi.oroar = roar && !lds ? L.roar : ~0ull;
  if (lds) {
    const uint64_t zt = align16(stage_end + L.end);
    const uint64_t em = zt + (zstd ? kZTablesBytes : 0);
#ifdef SB_BIN_EMIT_BLOCK
    const uint64_t need = em + kEmitBytes + kStagePad;
#else
    const uint64_t need = em + kStagePad;  // (staged pages emit through bin_emit_wave: no LDS window)
#endif
    if (need > lds_bytes) { set_err(sh, ST_NYI); return false; }  // (the plan made it a big page)
    bi.ztab = (uint32_t)zt;
    bi.emit = (uint32_t)em;
    bi.need = (uint32_t)need;
    bi.tb = stage_end;
  }
  return true;
}

template <int OW, class Src>
__device__ __forceinline__ uint64_t ldo(const Src& s, uint32_t p) {
  if constexpr (OW == 8) return s.u64(p);
  else return (uint64_t)(int64_t)(int32_t)s.u32(p);
}

__device__ __forceinline__ void bin_put_off(uint8_t* out, uint64_t row, uint64_t v, int ow) {
  if (ow == 8) ((uint64_t*)out)[row] = v;
  else ((uint32_t*)out)[row] = (uint32_t)v;
}

// Copy `len` bytes from LDS byte position `src` to global `dst`, all threads.
__device__ void copy_lds_to_global(const uint8_t* lds, uint32_t src, uint8_t* dst, uint64_t len) {
  const uint32_t tid = threadIdx.x;
  const uint32_t head = (uint32_t)min<uint64_t>(len, (4 - ((uintptr_t)dst & 3)) & 3);
  if (tid < head) dst[tid] = lds[src + tid];
  const uint64_t body = (len - head) >> 2;
  const uint32_t* lw = (const uint32_t*)lds;
  uint32_t* dw = (uint32_t*)(dst + head);
  for (uint64_t w = tid; w < body; w += NT) {
    const uint32_t p = src + head + (uint32_t)w * 4, i = p >> 2;
    dw[w] = __builtin_amdgcn_alignbyte(lw[i + 1], lw[i], p & 3);
  }
  const uint64_t done = head + body * 4;
  if (tid < len - done) dst[done + tid] = lds[src + done + tid];
}

// One wave finds `count` records [u64 len][len bytes] from page position q
// (bounded by end) and writes tab[e] = position of its bytes | length << 32; the
// reference reads them one by one (binary/dict.rs:95-141, freq.rs:127-142).
// A window of 255 byte positions after the current record start: every lane
// sizes the records that would start at 4 of them (successor x + 8 + len,
// 0xFF when it leaves the window or the header is not a record), wave_chain
// composes the successor tables and lane k gets the k-th record's start;
// lanes then check their record and write its entry.  A window yields every
// record it holds (at least one).  Returns the status; *sum = the lengths'
// total.
template <class Src, class TabP>
__device__ uint32_t walk_records(const Src& s, uint32_t q, uint32_t end, uint32_t count, TabP tab, uint64_t* sum) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t part = 0;
  uint32_t st = ST_OK;
  for (uint32_t e = 0, p = q; e < count;) {
    uint32_t t1 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t x = 4 * lane + k, pos = p + x;
      uint32_t d = 0xFF;
      if (x < 255 && pos <= end && end - pos >= 8) {
        const uint32_t lo = s.u32(pos), hi = s.u32(pos + 4);
        if (!hi && lo <= end - pos - 8 && x + 8 + lo < 255) d = x + 8 + lo;
      }
      t1 |= d << (8 * k);
    }
    const uint32_t kx = wave_chain(t1);
    const bool has = kx != 0xFF;
    uint32_t len = 0, bad = ST_OK;
    const uint32_t pos = p + (has ? kx : 0u);
    if (has) {
      if (pos > end || end - pos < 8) {
        bad = ST_IO;
      } else {
        const uint32_t lo = s.u32(pos), hi = s.u32(pos + 4);
        if (hi || lo > end - pos - 8) bad = ST_OUT_OF_SPEC;
        else len = lo;
      }
    }
    const uint32_t m = (uint32_t)__popcll(__ballot(has));
    const uint64_t badm = __ballot(has && bad != ST_OK);
    uint32_t take = min(m, count - e);
    if (badm) {  // only the window's last record can be bad (it stops the chain)
      const uint32_t j = (uint32_t)__builtin_ctzll(badm);
      if (j < take) {
        st = __builtin_amdgcn_readlane(bad, j);
        take = j;
      }
    }
    if (lane < take) {
      tab[e + lane] = (uint64_t)(pos + 8) | ((uint64_t)len << 32);
      part += len;
    }
    if (st) break;
    e += take;
    p = __builtin_amdgcn_readlane(pos + 8 + len, take - 1);
  }
  *sum = wave_sum64(part);
  return st;
}

// One wave expands a general-codec stream (LZ4 / Snappy / Zstd) from HBM
// into HBM, with k_inflate's per-wave LDS (output ring, input ring, chain
// tables) or the Zstd decoder's tables.
template <bool Z>
__device__ uint32_t expand_to_hbm(uint32_t codec, const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t usize,
                                  uint8_t* lds) {
  if (codec == 2) {
    if constexpr (Z) return zs::zstd_decode(GlbSrc{src}, csize, dst, usize, (lds_u8*)(lds + kBigZt), kZTablesMax);
    return ST_NYI;
  }
  WaveOut<true> o;
  o.xf = false;
  o.xadd = 0;
  o.skip0 = false;
  o.w0 = 0;
  o.ring = (lds_u8*)(lds + kBigRing);
  o.dst = dst;
  o.rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)usize, 0x00020000);
  o.dal = (uint32_t)((uintptr_t)dst & 3);
  o.rsa = __builtin_amdgcn_make_buffer_rsrc(dst - o.dal, 0, (int)(usize + o.dal), 0x00020000);
  o.olen = usize;
  o.op = 0;
  const uint32_t p0 = (uint32_t)((uintptr_t)src & 3);
  if (codec == 1) {
    InRing in;
    in.g = (gmem_u32*)((uintptr_t)src & ~(uintptr_t)3);
    in.nd = (p0 + csize + 3) >> 2;
    in.ib = (lds_u8*)(lds + kBigIb);
    in.ct = (lds_u8*)(lds + kBigCt);
    in.seek(p0);
    return lz4_inflate(in, p0, p0 + csize, o);
  }
  if (codec == 3) {
    WaveWin w;
    w.init(src, csize);
    return snappy_wave<true>(w, p0, p0 + csize, o);
  }
  return ST_NYI;
}

// A binary Dict's u32 index stream (n values) into the tables' x: leaf codecs
// via run_leaf; LZ4 / Snappy / Zstd expanded by wave 0 (into LDS for a
// staged page, straight into the region for a big page); Freq: the top index
// filled, then the exceptions (a leaf stream, or a general-codec stream
// expanded into the xex table first) scattered at their roaring rows.  All
// NT threads.
template <bool Z, class Src>
__device__ void materialize_idx(const Src& s, Shared& sh, const BinInfo& bi, TabBase<kLdsSrc<Src>> tb, const Stream ix,
                                const uint8_t* gpage, uint8_t* lds, uint32_t lds_bytes, uint8_t* biglds,
                                uint8_t* region) {
  constexpr bool L = kLdsSrc<Src>;
  const uint32_t tid = threadIdx.x, n = ix.n;
  mptr<L, uint32_t> xi = tb.template at<uint32_t>(0);
  mptr<L, uint32_t> xex = tb.template at<uint32_t>(bi.oxex);
  auto expand = [&](uint32_t codec, uint32_t body, uint32_t csize, uint64_t off, uint32_t bytes) -> uint32_t {
    if constexpr (L) {
      lds_u8* dst = (lds_u8*)(lds + bi.tb + off);
      if (codec == 2) {
        if constexpr (!Z) return ST_NYI;
        else
          return zs::zstd_to_lds(LdsSrc{s.w, s.base + body}, csize, dst, bytes, (lds_u8*)(lds + bi.ztab),
                                 lds_bytes - bi.ztab - kStagePad);
      }
      return expand_to_lds(codec, gpage + body, csize, dst, bytes);
    } else {
      return expand_to_hbm<Z>(codec, gpage + body, csize, region + off, bytes, biglds);
    }
  };
  if (ix.codec == 1 || ix.codec == 2 || ix.codec == 3) {
    if (tid < 64) {
      const uint32_t st = expand(ix.codec, ix.body, ix.csize, 0, 4 * n);
      if (st) set_err(sh, st);
    }
    __syncthreads();
    return;
  }
  if (ix.codec == 13) {
    __shared__ Stream ex;
    if (tid == 0) {
      sh.roar_pending = 0;
      parse_freq(s, sh, ix, 4, &ex);
    }
    __syncthreads();
    if (sh.err) return;
    roaring_build(s, sh, L ? nullptr : region + bi.oroar, L ? 0u : (uint32_t)roar_cap(n));
    if (sh.err) return;
    const uint32_t top = (uint32_t)sh.freq_top;
    for (uint32_t i = tid; i < n; i += NT) xi[i] = top;
    const bool gen = ex.codec == 1 || ex.codec == 2 || ex.codec == 3;
    if (gen && tid < 64) {
      const uint32_t st = expand(ex.codec, ex.body, ex.csize, bi.oxex, 4 * ex.n);
      if (st) set_err(sh, st);
    }
    __syncthreads();
    if (sh.err) return;
    auto scatter = [&](uint32_t i0, const uint32_t* v, uint32_t nv) {
      for (uint32_t l = 0; l < nv; l++) {
        const uint32_t row = roaring_select(s, sh, i0 + l);
        if (row < n) xi[row] = v[l];
        else set_err(sh, ST_OUT_OF_SPEC);
      }
    };
    if (!gen) {
      run_leaf<4>(s, sh, ex, scatter);
    } else {
      for (uint32_t i = tid; i < ex.n; i += NT) {
        const uint32_t v = xex[i];
        scatter(i, &v, 1);
      }
    }
    __syncthreads();
    return;
  }
  run_leaf<4>(s, sh, ix, [&](uint32_t row, const uint32_t* v, uint32_t nv) {
    for (uint32_t l = 0; l < nv; l++) xi[row + l] = v[l];
  });
  __syncthreads();
}

// A binary Freq page's exceptions (all NT threads, after bin_parse): the
// roaring tables, the exceptions at rows < n (freq.rs:127-141 consumes them
// in row order; select is increasing, so a binary search finds the first
// row >= n), and wave 0's walk of their records.  S = (n - ep) * L + sum.
template <class Src>
__device__ void freq_tables(const Src& s, Shared& sh, BinInfo& bi, TabBase<kLdsSrc<Src>> tb, const PageDesc& pd,
                            uint8_t* region) {
  constexpr bool L = kLdsSrc<Src>;
  const uint32_t n = pd.num_values;
  roaring_build(s, sh, L ? nullptr : region + bi.oroar, L ? 0u : (uint32_t)roar_cap(n));
  if (sh.err) return;
  if (threadIdx.x == 0) {
    uint32_t ep = 0, hi_e = bi.tot;
    while (ep < hi_e) {
      const uint32_t mid = (ep + hi_e) / 2;
      if (roaring_select(s, sh, mid) < n) ep = mid + 1;
      else hi_e = mid;
    }
    bi.k = ep;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    uint64_t sum;
    const uint32_t st = walk_records(s, bi.q, bi.end, bi.k, tb.template at<uint64_t>(bi.otab), &sum);
    if (st && threadIdx.x == 0) set_err(sh, st);
    if (threadIdx.x == 0) bi.S = (uint64_t)(n - bi.k) * bi.L + sum;
  }
  __syncthreads();
}

// A binary Dict page's tables (all NT threads, after bin_parse): wave 0
// walks the k entry records, then the index stream is materialized; S = the
// page's values bytes, sum of its rows' entry lengths (an index >= k is
// out of range, dict.rs:131-139 panics).
template <bool Z, class Src>
__device__ void dict_tables(const Src& s, Shared& sh, BinInfo& bi, TabBase<kLdsSrc<Src>> tb, const Stream& ix,
                            const PageDesc& pd, const uint8_t* gpage, uint8_t* lds, uint32_t lds_bytes, uint8_t* biglds,
                            uint8_t* region, bool sized) {
  constexpr bool L = kLdsSrc<Src>;
  if (threadIdx.x < 64) {
    uint64_t sum;
    const uint32_t st = walk_records(s, bi.q, bi.end, bi.k, tb.template at<uint64_t>(bi.otab), &sum);
    if (st && threadIdx.x == 0) set_err(sh, st);
  }
  __syncthreads();
  if (sh.err) return;
  materialize_idx<Z>(s, sh, bi, tb, ix, gpage, lds, lds_bytes, biglds, region);
  if (sh.err || !sized) return;
  const uint32_t k = bi.k;
  mptr<L, uint32_t> xi = tb.template at<uint32_t>(0);
  mptr<L, uint64_t> tab = tb.template at<uint64_t>(bi.otab);
  uint64_t part = 0;
  bool bad = false;
  for (uint32_t i = threadIdx.x; i < pd.num_values; i += NT) {
    const uint32_t x = xi[i];
    if (x < k) part += tab[x] >> 32;
    else bad = true;
  }
  if (bad) set_err(sh, ST_OUT_OF_SPEC);
  uint64_t tot;
  block_excl_scan<uint64_t>(part, sh, &tot);
  if (threadIdx.x == 0) bi.S = tot;
  __syncthreads();
}

// A binary Freq page's exception-row bitmap and its prefix popcounts (at the
// tables' x: ceil(n/32) words, then as many prefixes), after freq_tables; all
// NT threads.  A row's exception rank is then pref[w] + popc(bits[w] & below).
template <class Src>
__device__ void freq_rows(const Src& s, Shared& sh, const BinInfo& bi, TabBase<kLdsSrc<Src>> tb, uint32_t n) {
  constexpr bool L = kLdsSrc<Src>;
  const uint32_t tid = threadIdx.x, nw = (n + 31) / 32;
  mptr<L, uint32_t> bits = tb.template at<uint32_t>(0);
  mptr<L, uint32_t> pref = bits + nw;
  for (uint32_t w = tid; w < nw; w += NT) bits[w] = 0;
  __syncthreads();
  for (uint32_t e = tid; e < bi.k; e += NT) {
    const uint32_t row = roaring_select(s, sh, e);
    atomicOr((uint32_t*)&bits[row >> 5], 1u << (row & 31));
  }
  __syncthreads();
  uint32_t carry = 0;
  for (uint32_t w0 = 0; w0 < nw; w0 += NT) {
    const uint32_t w = w0 + tid;
    const uint32_t pc = w < nw ? __popc(bits[w]) : 0u;
    uint32_t tot;
    const uint32_t pre = block_excl_scan<uint32_t>(pc, sh, &tot);
    if (w < nw) pref[w] = carry + pre;
    carry += tot;
  }
  __syncthreads();
}

// len bytes of `src` from page position sp into the LDS window at byte w:
// byte writes up to a dword boundary, whole dwords (each owned by this row
// alone), byte writes for the tail -- neighbouring rows share only the edge
// dwords, which both fill byte by byte.
template <class Src>
__device__ __forceinline__ void copy_to_win(const Src& src, uint32_t sp, uint32_t len, lds_u8* win, uint32_t w) {
  while (len && (w & 3)) {
    win[w++] = (uint8_t)src.u8(sp++);
    len--;
  }
  for (; len >= 4; len -= 4, w += 4, sp += 4) ((lds_u32*)win)[w >> 2] = src.u32(sp);
  while (len) {
    win[w++] = (uint8_t)src.u8(sp++);
    len--;
  }
}

// Arrow offsets and values bytes of rows [0, n): row i has len_of(i) bytes at
// page position src_of(i) of `src`.  Offsets[R + i + 1] = V + running length
// (read_binary's rebase, binary/mod.rs:136-144).  Rows go NT*4 at a time,
// four consecutive rows a thread; their bytes are gathered into an LDS
// window of kEmitBytes (dword copies, copy_to_win) laid out as the
// destination's 16-byte-aligned span, and each window leaves in 16-byte
// stores (units cut by the page's edges byte by byte).  `ea` is the window.
template <int OW, class Src, class LenF, class SrcF>
__device__ __forceinline__ void bin_emit(Shared& sh, const Src& src, lds_u32* ea, uint32_t n, uint64_t R, uint64_t V,
                                         const BinArgs& a, LenF len_of, SrcF src_of) {
  constexpr uint32_t WB = kEmitBytes & ~15u;
  const uint32_t tid = threadIdx.x;
  lds_u8* win = (lds_u8*)ea;
  uint64_t carry = 0;
  for (uint32_t r0 = 0; r0 < n; r0 += kEmitRows) {
    const uint32_t m = min(kEmitRows, n - r0);
    uint32_t l[4], sp[4], st[4];
    uint32_t tsum = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t i = 4 * tid + j;
      l[j] = i < m ? len_of(r0 + i) : 0u;
      sp[j] = i < m ? src_of(r0 + i) : 0u;
      tsum += l[j];
    }
    uint32_t tot;
    uint32_t pre = block_excl_scan<uint32_t>(tsum, sh, &tot);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t i = 4 * tid + j;
      st[j] = pre;
      if (i < m) {
        pre += l[j];
        bin_put_off(a.out_offsets, R + r0 + i + 1, V + carry + pre, OW);
      }
    }
    uint8_t* d0 = a.out_values + V + carry;
    const uint32_t head = (uint32_t)((uintptr_t)d0 & 15);
    uint8_t* base0 = d0 - head;
    const uint32_t span = head + tot;  // destination bytes from base0 (16-aligned)
    for (uint32_t k0 = 0; k0 < span; k0 += WB) {
      // tile bytes [xlo, xhi) land in this window at window byte x + head - k0
      const int64_t xlo = (int64_t)k0 - head, xhi = xlo + WB;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int64_t lo = max<int64_t>(st[j], xlo), hi = min<int64_t>((int64_t)st[j] + l[j], xhi);
        if (lo < hi)
          copy_to_win(src, sp[j] + (uint32_t)(lo - st[j]), (uint32_t)(hi - lo), win, (uint32_t)(lo - xlo));
      }
      __syncthreads();
      const uint32_t wl = min(WB, span - k0);
      for (uint32_t u = tid; 16 * u < wl; u += NT) {
        const uint32_t q = k0 + 16 * u;  // destination byte (from base0) of the unit
        uint8_t* d = base0 + q;
        const u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(win + 16 * u);
        if (q >= head && q + 16 <= span) {
          *(u32x4*)d = v;
        } else {
          for (uint32_t b = 0; b < 16; b++)
            if (q + b >= head && q + b < span) d[b] = (uint8_t)(v[b >> 2] >> (8 * (b & 3)));
        }
      }
      __syncthreads();
    }
    carry += tot;
  }
}

// Header-only pages: Basic pages under LZ4 / Snappy need no staging.  Their
// two streams are expanded by k_inflate (offsets into scratch, values at the
// page's base), so only the validity prefix and the two stream headers are
// read here, by one thread per page straight from HBM, with the checks of
// parse_validity and bin_parse; any other page (or any check failing) goes to
// the staged passes, which report the error.
struct LightPage {
  uint32_t codec, ob, ocs, vb, vcs, S, vbpos;
};

template <int OW>
__device__ bool bin_light_parse(const GlbSrc& s, uint32_t len, uint32_t n, int nullable, LightPage& lp) {
  uint32_t p;
  if (!light_validity(s, len, n, nullable, &p, &lp.vbpos)) return false;
  if (p + 9 > len) return false;
  lp.codec = s.u8(p);
  if (lp.codec > 3) return false;
  const uint32_t cs = s.u32(p + 1), body = p + 9;
  if (cs > len - body) return false;
  const uint32_t vh = body + cs;
  if (vh + 9 > len) return false;
  lp.vcs = s.u32(vh + 1);
  lp.S = s.u32(vh + 5);
  lp.vb = vh + 9;
  if (lp.vcs > len - lp.vb) return false;
  lp.ob = body;
  lp.ocs = cs;
  // None: both streams are copied as they lie (copy_from_slice lengths, binary/mod.rs:119-160)
  if (lp.codec == 0 && (cs != (n + 1) * (uint32_t)OW || lp.vcs != lp.S)) return false;
  // Zstd: only pages whose streams do not fit the staged pass's LDS (k_zinflate)
  if (lp.codec == 2 && (uint64_t)len + (uint64_t)(n + 1) * OW + lp.S + kZTablesMax + 1024 <= kDeferredLds) return false;
  return true;
}

// Bytes [x, x + 20) of a page from HBM by six aligned dword loads (clamped to
// the dwords that hold page bytes), so a header costs one load round trip,
// not one per byte.  Offsets k <= 16 of the window.
struct HdrWin {
  uint32_t w[6], sh;
  __device__ __forceinline__ void load(const uint8_t* pg, uint32_t x, uint32_t len) {
    const uintptr_t a = (uintptr_t)(pg + x), lastw = (uintptr_t)(pg + (len ? len - 1 : 0)) & ~(uintptr_t)3;
    const uintptr_t a0 = a & ~(uintptr_t)3;
    sh = (uint32_t)(a & 3);
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = *(gmem_u32*)min<uintptr_t>(a0 + 4 * k, lastw);
  }
  __device__ __forceinline__ uint32_t u32(uint32_t k) const {
    const uint32_t b = sh + k, i = b >> 2;
    return __builtin_amdgcn_alignbyte(w[i + 1], w[i], b & 3);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t k) const { return u32(k) & 0xFFu; }
};

// bin_light_parse over HdrWin windows: the validity prefix, the offsets
// stream header and the values stream header, three load round trips.
template <int OW>
__device__ bool bin_light_parse_hbm(const uint8_t* pg, uint32_t len, uint32_t n, int nullable, LightPage& lp) {
  uint32_t p = 0;
  lp.vbpos = 0;
  if (n == 0) return false;
  HdrWin h;
  if (nullable) {  // light_validity
    if (len < 4) return false;
    h.load(pg, 0, len);
    const uint32_t def_len = h.u32(0);
    p = 4;
    if (def_len == 0 || def_len > len - p) return false;
    uint32_t q = p, hv = 0, sft = 0;
    for (;;) {
      if (q >= p + def_len || sft > 28) return false;
      const uint32_t c = h.u8(q++);  // (q <= 8)
      hv |= (c & 0x7Fu) << sft;
      if (!(c & 0x80)) break;
      sft += 7;
    }
    if (!(hv & 1)) return false;
    if ((uint64_t)min(hv >> 1, p + def_len - q) * 8 < n) return false;
    lp.vbpos = q;
    p += def_len;
  }
  if (p + 9 > len) return false;
  h.load(pg, p, len);
  lp.codec = h.u8(0);
  if (lp.codec > 3) return false;
  const uint32_t cs = h.u32(1), body = p + 9;
  if (cs > len - body) return false;
  const uint32_t vh = body + cs;
  if (vh + 9 > len) return false;
  h.load(pg, vh, len);
  lp.vcs = h.u32(1);
  lp.S = h.u32(5);
  lp.vb = vh + 9;
  if (lp.vcs > len - lp.vb) return false;
  lp.ob = body;
  lp.ocs = cs;
  if (lp.codec == 0 && (cs != (n + 1) * (uint32_t)OW || lp.vcs != lp.S)) return false;
  if (lp.codec == 2 && (uint64_t)len + (uint64_t)(n + 1) * OW + lp.S + kZTablesMax + 1024 <= kDeferredLds) return false;
  return true;
}

// Classifies every page (one thread each): header-only pages get their two
// inflate jobs and size here; the rest are listed for k_bin_size.
template <int OW>
__global__ __launch_bounds__(NT) void k_bin_light(BinArgs a) {
  const uint32_t np = a.n_pages;
  uint32_t *staged = a.cls, *light = a.cls + np, *vbpos = a.cls + 2 * np, *cnt = a.cls + 4 * np;
  for (uint32_t page = blockIdx.x * NT + threadIdx.x; page < np; page += gridDim.x * NT) {
    const PageDesc pd = a.pages[page];
    LightPage lp;
    const bool lt = bin_light_parse_hbm<OW>(a.chunk + pd.byte_off, pd.byte_len, pd.num_values, a.nullable, lp);
    // one atomic per wave and counter (12k contended atomics on one address cost ~100 us)
    const bool jobs = lt && lp.codec != 0;  // None pages: copied by k_bin_light_out
    const uint32_t slot = wave_slot(a.job_count, jobs, 2), li = wave_slot(&cnt[1], lt, 1),
                   si = wave_slot(&cnt[0], !lt, 1);
    if (jobs) {
      // Utf8 (32-bit) offsets are expanded straight into the column, rebased
      // (k_inflate xf); LargeUtf8 offsets go through scratch
      a.jobs[slot] = InflateJob{pd.byte_off + lp.ob,
                                OW == 4 && lp.codec != 2 ? kDstBinOffs | (pd.row_off * 4)
                                                         : kDstScratch | ((pd.row_off + page) * OW),
                                lp.ocs, (pd.num_values + 1) * (uint32_t)OW, lp.codec, page};
      a.jobs[slot + 1] = InflateJob{pd.byte_off + lp.vb, kDstBinBase | page, lp.vcs, lp.S, lp.codec, page};
    }
    if (lt) {
      a.sizes[page] = lp.S;
      a.status[page] = 0;
      // bit 31: a None page; bit 30: offsets expanded into scratch (Zstd)
      vbpos[page] = lp.vbpos | (lp.codec == 0 ? 0x80000000u : 0u) | (lp.codec == 2 ? 0x40000000u : 0u);
      light[li] = page;
    } else {
      staged[si] = page;
    }
  }
}

// len bytes from chunk + src to dst, one workgroup: dword loads realigned by
// v_alignbyte, dword stores after the head bytes that align dst.
__device__ void copy_glb(uint64_t src, const uint8_t* chunk, uint8_t* dst, uint64_t len) {
  const uint32_t tid = threadIdx.x;
  const uint32_t head = (uint32_t)min<uint64_t>(len, (4 - ((uintptr_t)dst & 3)) & 3);
  if (tid < head) dst[tid] = chunk[src + tid];
  const uint64_t body = (len - head) >> 2;
  const uint8_t* s0 = chunk + src + head;
  const uint32_t sh = (uint32_t)((uintptr_t)s0 & 3);
  const uint32_t* s32 = (const uint32_t*)((uintptr_t)s0 - sh);
  uint32_t* d32 = (uint32_t*)(dst + head);
  for (uint64_t w = tid; w < body; w += NT)
    d32[w] = sh ? __builtin_amdgcn_alignbyte(s32[w + 1], s32[w], sh) : s32[w];
  const uint64_t done = head + body * 4;
  if (tid < len - done) dst[done + tid] = chunk[src + done + tid];
}

// Header-only pages after k_inflate: offsets rebased from scratch onto the
// page's values base (mod.rs:136-144; p[0] must be 0 and p[n] the values
// length), the validity bitmap copied from the page in HBM.
template <int OW>
__global__ __launch_bounds__(NT) void k_bin_light_out(BinArgs a) {
  __shared__ uint32_t bad;
  const uint32_t np = a.n_pages, nl = a.cls[4 * np + 1], tid = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const uint32_t page = a.cls[np + i];
    const PageDesc pd = a.pages[page];
    const uint32_t n = pd.num_values;
    const uint64_t R = pd.row_off, V = a.bases[page], S = a.sizes[page];
    if (a.status[page]) continue;  // an inflate error stands
    const uint32_t tag = a.cls[2 * np + page], vb = tag & 0x3FFFFFFFu;
    const bool scr = OW == 8 || (tag & 0x40000000u);  // offsets in scratch (else rebased in place by k_inflate)
    const GlbSrc pg{a.chunk + pd.byte_off};
    if (tag & 0x80000000u) {  // a None page: offsets rebased and values copied from the page in HBM
      __shared__ LightPage nl_lp;
      if (tid == 0) {
        bin_light_parse<OW>(pg, pd.byte_len, n, a.nullable, nl_lp);
        bad = (ldo<OW>(pg, nl_lp.ob + n * OW) != S || V + S > a.values_cap) ? ST_OUT_OF_SPEC : 0u;  // DEVIATION 7
      }
      __syncthreads();
      const uint32_t e = bad, ob = nl_lp.ob, vpos = nl_lp.vb;
      __syncthreads();
      if (e) {
        if (tid == 0) a.status[page] = e;
        continue;
      }
      if (page == 0 && tid == 0) bin_put_off(a.out_offsets, 0, ldo<OW>(pg, ob), OW);  // the first page keeps p[0]
      for (uint32_t k = tid + 1; k <= n; k += NT) bin_put_off(a.out_offsets, R + k, V + ldo<OW>(pg, ob + k * OW), OW);
      copy_glb(pd.byte_off + vpos, a.chunk, a.out_values + V, S);
      if (vb) write_validity(pg, vb, n, R, a.out_validity);
      continue;
    }
    const uint8_t* xo = a.scratch + (R + page) * OW;
    auto po = [&](uint32_t k) -> uint64_t {
      if constexpr (OW == 8) return ((const uint64_t*)xo)[k];
      else return (uint64_t)(int64_t)((const int32_t*)xo)[k];
    };
    // p[n] must be the values stream's length (DEVIATION: the reference only
    // fails once the column's last offset passes its values, at try_new)
    if (tid == 0) {
      if (!scr)  // rebased in place by k_inflate
        bad = ((uint32_t)((const uint32_t*)a.out_offsets)[R + n] != (uint32_t)(V + S) || V + S > a.values_cap) ? ST_OUT_OF_SPEC
                                                                                        : 0u;
      else
        bad = (po(n) != S || V + S > a.values_cap) ? ST_OUT_OF_SPEC : 0u;
    }
    __syncthreads();
    const uint32_t e = bad;
    __syncthreads();
    if (e) {
      if (tid == 0) a.status[page] = e;
      continue;
    }
    if (scr) {
      if (page == 0 && tid == 0) bin_put_off(a.out_offsets, 0, po(0), OW);  // the first page keeps its p[0]
      for (uint32_t k = tid + 1; k <= n; k += NT) bin_put_off(a.out_offsets, R + k, V + po(k), OW);
    }
    if (vb) write_validity(pg, vb, n, R, a.out_validity);
  }
}

// Plan time, one thread per page from HBM: the LDS a staged decode of the
// page needs (bin_parse's layout) and the HBM region its tables need when
// that exceeds one workgroup's LDS (an Extend page: OneValue / Dict / Freq).
// Header-only (light) pages need neither.
template <int OW>
__global__ __launch_bounds__(NT) void k_bin_probe(BinArgs a) {
  for (uint32_t page = blockIdx.x * NT + threadIdx.x; page < a.n_pages; page += gridDim.x * NT) {
    const PageDesc pd = a.pages[page];
    const GlbSrc s{a.chunk + pd.byte_off};
    const uint32_t len = pd.byte_len, n = pd.num_values;
    uint32_t need = 0;
    uint64_t rneed = 0;
    bool zpage = false;
    LightPage lp;
    if (!bin_light_parse<OW>(s, len, n, a.nullable, lp)) {
      const uint64_t stage_end = align16((uint64_t)len + 15 + kStagePad);
      uint64_t nd = stage_end + 64;
      uint32_t p = 0;
      bool ok = true;
      if (a.nullable) {
        ok = len >= 4 && s.u32(0) <= len - 4;
        p = ok ? 4 + s.u32(0) : 0;
      }
      ok = ok && p + 9 <= len;
      const uint32_t codec = ok ? s.u8(p) : 0u, cs = ok ? s.u32(p + 1) : 0u, body = p + 9;
      ok = ok && cs <= len - body;
      const uint32_t end = body + cs;
      if (ok && codec == 2) {
        nd = kDeferredLds;
        zpage = true;
      } else if (ok && (codec == BIN_ONE || codec == BIN_DICT || codec == BIN_FREQ)) {
        uint32_t k = 0, tot = 0, xcodec = 0;
        bool zstd = false, xex = false, roar = false;
        if (codec == BIN_DICT && body + 9 <= end) {
          const uint32_t ic = s.u8(body), ics = s.u32(body + 1);
          if (ics <= end - body - 9 && body + 9 + ics + 4 <= end) {
            k = s.u32(body + 9 + ics);
            zstd = ic == 2;
            if (ic == 13 && idx_freq_header(s, body + 9, body + 9 + ics, &tot, &xcodec)) {
              xex = xcodec == 1 || xcodec == 2 || xcodec == 3;
              zstd = xcodec == 2;
              roar = true;
            }
          }
        } else if (codec == BIN_FREQ && body + 8 <= end) {
          const uint64_t tl = s.u64(body);
          if (tl <= end - body - 8 && body + 8 + tl + 4 <= end) {
            const uint32_t r = body + 12 + (uint32_t)tl, bm = s.u32(r - 4);
            if (bm >= 8 && bm <= end - r) {
              const uint32_t nc = s.u32(r + 4);
              uint64_t t = 0;
              if (8 + 8 * (uint64_t)nc <= bm)
                for (uint32_t c = 0; c < nc; c++) t += (s.u32(r + 8 + 4 * c) >> 16) + 1;
              tot = (uint32_t)min<uint64_t>(t, 0xFFFFFFFFull);
              roar = true;
            }
          }
        }
        zpage = zstd;
        const BinLayout L = bin_layout(codec, n, k, tot, xex, false);
#ifdef SB_BIN_EMIT_BLOCK
        nd = align16(stage_end + L.end) + (zstd ? kZTablesBytes : 0) + kEmitBytes + kStagePad;
#else
        // (as bin_parse: staged pages emit through bin_emit_wave, no LDS window --
        // the 8 KiB window held C5's Dict pages at two workgroups a CU)
        nd = align16(stage_end + L.end) + (zstd ? kZTablesBytes : 0) + kStagePad;
#endif
        rneed = max<uint64_t>(bin_layout(codec, n, k, tot, xex, roar).end, 16);
      }
      need = (uint32_t)min<uint64_t>(nd, 0xFFFFFFFFull);
    }
    a.lds_need[page] = need;
    a.rneed[page] = rneed;
    if (zpage && a.total) atomicOr((unsigned long long*)a.total, 1ull);  // (stage 2: the plan's Zstd flag)
  }
}

template <int OW, bool Z>
__global__ __launch_bounds__(NT) void k_bin_size(BinArgs a) {
  extern __shared__ u32x4 stage[];
  __shared__ Shared sh;
  __shared__ BinInfo bi;
  __shared__ Stream idx;
  uint8_t* lds = (uint8_t*)stage;
  const uint32_t np = a.n_pages, n_staged = a.cls[4 * np];
  for (uint32_t i = blockIdx.x; i < n_staged; i += gridDim.x) {
    const uint32_t page = a.cls[i];
    const PageDesc pd = a.pages[page];
    if (pd.reserved) {  // a big page: its tables live in its HBM region (k_bin_big)
      if (threadIdx.x == 0) a.cls[3 * np + atomicAdd(&a.cls[4 * np + 2], 1u)] = page;
      continue;
    }
    if (threadIdx.x == 0) sh.err = 0;
    const uint32_t stage_end = ((pd.byte_len + 15 + kStagePad) + 15) & ~15u;
    if (stage_end + 64 > a.lds_bytes) {  // page larger than the LDS budget
      __syncthreads();
      if (threadIdx.x == 0) { a.status[page] = ST_NYI; a.sizes[page] = 0; }
      __syncthreads();
      continue;
    }
    const uint32_t base = stage_page(stage, a.chunk + pd.byte_off, pd.byte_len);
    LdsSrc s{(const uint32_t*)stage, base};
    if (threadIdx.x == 0) bin_parse<OW>(s, sh, bi, pd, a.nullable, true, stage_end, a.lds_bytes, &idx);
    __syncthreads();
    if (!sh.err) {
      const TabBase<true> tb{(lds_u8*)stage + bi.tb};
      if (bi.codec == 1 || bi.codec == 3) {
        // Basic under LZ4 / Snappy: the offsets stream expands into scratch, the
        // values stream straight into the values buffer at the page's base
        if (threadIdx.x == 0) {
          const uint32_t slot = atomicAdd(a.job_count, 2u);
          a.jobs[slot] = InflateJob{pd.byte_off + bi.ob, kDstScratch | ((pd.row_off + page) * OW), bi.ocs,
                                    (pd.num_values + 1) * (uint32_t)OW, bi.codec, page};
          a.jobs[slot + 1] = InflateJob{pd.byte_off + bi.vb, kDstBinBase | page, bi.vcs, (uint32_t)bi.S, bi.codec, page};
        }
      } else if (bi.codec == BIN_DICT) {
        dict_tables<Z>(s, sh, bi, tb, idx, pd, a.chunk + pd.byte_off, lds, a.lds_bytes, nullptr, nullptr, true);
      } else if (bi.codec == BIN_FREQ) {
        freq_tables(s, sh, bi, tb, pd, nullptr);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      a.status[page] = sh.err;
      a.sizes[page] = sh.err ? 0 : bi.S;
    }
    __syncthreads();
  }
}

// Exclusive scan of the page sizes (one workgroup).
// One workgroup: each thread sums a contiguous run of pages (its loads all
// in flight at once), one block scan, then the run's bases.
__global__ __launch_bounds__(NT) void k_bin_scan(BinArgs a) {
  __shared__ Shared sh;
  const uint32_t n = a.n_pages, c = (n + NT - 1) / NT;
  const uint32_t b = min(n, threadIdx.x * c), e = min(n, b + c);
  uint64_t sum = 0;
#pragma unroll 8
  for (uint32_t p = b; p < e; p++) sum += a.sizes[p];
  uint64_t tot;
  uint64_t ex = block_excl_scan<uint64_t>(sum, sh, &tot);
#pragma unroll 8
  for (uint32_t p = b; p < e; p++) {
    a.bases[p] = ex;
    ex += a.sizes[p];
  }
  if (threadIdx.x == 0) *a.total = tot;
}

// Rows longer than this are copied by the whole wave (bin_emit_wave).
constexpr uint32_t kRowDirect = 64;

// len bytes of a staged page at sp to global dst, one lane: the dwords the
// row covers whole as dword stores, the bytes it shares with its neighbours'
// dwords as byte stores (byte-granular, so no merge is needed).
__device__ __forceinline__ void copy_row(const LdsSrc& src, uint32_t sp, uint32_t len, uint8_t* dst) {
  const uint32_t head = min(len, (uint32_t)((4 - ((uintptr_t)dst & 3)) & 3));
  for (uint32_t i = 0; i < head; i++) dst[i] = (uint8_t)src.u8(sp + i);
  uint32_t k = head;
  for (; k + 4 <= len; k += 4) *(uint32_t*)(dst + k) = src.u32(sp + k);
  for (; k < len; k++) dst[k] = (uint8_t)src.u8(sp + k);
}
// The same for one long row, by the whole wave.
__device__ __forceinline__ void wave_copy_row(const LdsSrc& src, uint32_t sp, uint32_t len, uint8_t* dst) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t head = min(len, (uint32_t)((4 - ((uintptr_t)dst & 3)) & 3));
  if (lane < head) dst[lane] = (uint8_t)src.u8(sp + lane);
  const uint32_t nw = (len - head) / 4;
  for (uint32_t w = lane; w < nw; w += 64) *(uint32_t*)(dst + head + 4 * w) = src.u32(sp + head + 4 * w);
  const uint32_t t0 = head + 4 * nw;
  if (lane < len - t0) dst[t0 + lane] = (uint8_t)src.u8(sp + t0 + lane);
}

// Arrow offsets and values of rows [0, n) of a staged page, wave-parallel
// with one block barrier: wave w takes rows [w q, (w + 1) q), its first byte
// from the other waves' totals; then 64 rows a step, one a lane, placed by a
// DPP scan, offsets as one coalesced store, each lane writing its row
// dword-aligned (copy_row) -- no LDS window, no barrier per tile as in
// bin_emit.  Rows over kRowDirect bytes are copied by the wave.
template <int OW, class LenF, class SrcF>
__device__ void bin_emit_wave(const LdsSrc& src, uint32_t n, uint64_t R, uint64_t V, const BinArgs& a, LenF len_of,
                              SrcF src_of) {
  __shared__ uint64_t qtot[NW];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t q = (n + NW - 1) / NW, r0 = min(n, wv * q), r1 = min(n, r0 + q);
  uint64_t part = 0;
  for (uint32_t r = r0 + lane; r < r1; r += 64) part += len_of(r);
  part = wave_sum64(part);
  if (lane == 0) qtot[wv] = part;
  __syncthreads();
  uint64_t base = V;
  for (uint32_t k = 0; k < wv; k++) base += qtot[k];
  __syncthreads();  // (qtot is the next page's)
  for (uint32_t c0 = r0; c0 < r1; c0 += 64) {
    const uint32_t r = c0 + lane;
    const bool in = r < r1;
    const uint32_t l = in ? len_of(r) : 0u, sp = in ? src_of(r) : 0u;
    const uint32_t incl = wave_incl_scan(l);
    const uint64_t d = base + incl - l;
    if (in) bin_put_off(a.out_offsets, R + r + 1, d + l, OW);
    if (in && l <= kRowDirect) copy_row(src, sp, l, a.out_values + d);
    for (uint64_t big = __ballot(in && l > kRowDirect); big; big &= big - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(big);
      const uint64_t dj = ((uint64_t)__shfl((uint32_t)(d >> 32), j, 64) << 32) | __shfl((uint32_t)d, j, 64);
      wave_copy_row(src, __shfl(sp, j, 64), __shfl(l, j, 64), a.out_values + dj);
    }
    base += __builtin_amdgcn_readlane(incl, 63);
  }
}

// Offsets and values of rows [0, n) through bin_emit_wave (staged pages) or
// bin_emit (pages whose tables live in HBM).
template <int OW, class Src, class LenF, class SrcF>
__device__ __forceinline__ void bin_emit_any(Shared& sh, const Src& src, lds_u32* ea, uint32_t n, uint64_t R, uint64_t V,
                                             const BinArgs& a, LenF len_of, SrcF src_of) {
#ifndef SB_BIN_EMIT_BLOCK
  if constexpr (kLdsSrc<Src>) {
    bin_emit_wave<OW>(src, n, R, V, a, len_of, src_of);
    return;
  }
#endif
  bin_emit<OW>(sh, src, ea, n, R, V, a, len_of, src_of);
}

// The Extend rows of a parsed page (OneValue / Dict / Freq) whose tables are
// built (dict_tables / freq_tables + freq_rows): offsets and values through
// bin_emit_any.  All NT threads.
template <int OW, class Src>
__device__ __forceinline__ void bin_emit_extend(Shared& sh, const Src& s, const BinInfo& bi, TabBase<kLdsSrc<Src>> tb, lds_u32* ea,
                                uint32_t n, uint64_t R, uint64_t V, const BinArgs& a) {
  constexpr bool L = kLdsSrc<Src>;
  if (bi.codec == BIN_ONE) {
    const uint32_t len = bi.L, top = bi.top;
    bin_emit_any<OW>(sh, s, ea, n, R, V, a, [&](uint32_t) { return len; }, [&](uint32_t) { return top; });
  } else if (bi.codec == BIN_DICT) {
    const mptr<L, uint32_t> xi = tb.template at<uint32_t>(0);
    const mptr<L, uint64_t> tab = tb.template at<uint64_t>(bi.otab);
    const uint32_t k = bi.k;
    bin_emit_any<OW>(sh, s, ea, n, R, V, a,
                 [&](uint32_t i) { const uint32_t x = xi[i]; return x < k ? (uint32_t)(tab[x] >> 32) : 0u; },
                 [&](uint32_t i) { const uint32_t x = xi[i]; return x < k ? (uint32_t)tab[x] : 0u; });
  } else {  // Freq: exception rows by the bitmap + prefix popcount rank
    const uint32_t nw = (n + 31) / 32;
    const mptr<L, uint32_t> bits = tb.template at<uint32_t>(0);
    const mptr<L, uint32_t> pref = bits + nw;
    const mptr<L, uint64_t> tab = tb.template at<uint64_t>(bi.otab);
    const uint32_t len = bi.L, top = bi.top;
    auto rank = [&](uint32_t i) { return pref[i >> 5] + __popc(bits[i >> 5] & ((1u << (i & 31)) - 1)); };
    auto exc = [&](uint32_t i) { return (bits[i >> 5] >> (i & 31)) & 1u; };
    bin_emit_any<OW>(sh, s, ea, n, R, V, a, [&](uint32_t i) { return exc(i) ? (uint32_t)(tab[rank(i)] >> 32) : len; },
                 [&](uint32_t i) { return exc(i) ? (uint32_t)tab[rank(i)] : top; });
  }
}

// Look-back state of a page in the fused pass: its values bytes (low 62
// bits) and whether that is the page's own size (AGG) or the inclusive
// prefix through it (INCL).
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 1ull << 63, kLbVal = kLbAgg - 1;

// The values base of `page` from its predecessors' look-back states, wave 0
// (the single-pass chained scan with a wave-wide look-back: 4 x 64
// predecessor states per probe, their loads issued together; the nearest
// INCL ends the walk, AGGs before it add up; a page waits only for lower
// pages, which resident workgroups claimed before it, so every wait ends).
// When every page is resident at once (C5's 1024-page columns) their tables
// finish together and INCL spreads from page 0 one probe at a time, so a
// probe covers 256 pages.  The states are the only data exchanged: relaxed
// agent-scope loads and stores (coherent in L2, no L1 invalidate or L2
// writeback per probe).  Returns the base in every lane.
__device__ uint64_t lookback(uint64_t* lb, uint32_t page, uint64_t S) {
  constexpr uint32_t kProbe = 4;  // windows of 64 states per probe
  const uint32_t lane = threadIdx.x & 63;
  if (page == 0) {
    if (lane == 0) __hip_atomic_store(&lb[0], kLbIncl | S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&lb[page], kLbAgg | S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t acc = 0;
  for (int64_t top = (int64_t)page - 1;;) {
    uint64_t v[kProbe];
#pragma unroll
    for (uint32_t k = 0; k < kProbe; k++) {
      const int64_t j = top - (int64_t)(64 * k + lane);  // window 0 lane 0: the nearest predecessor
      v[k] = j >= 0 ? __hip_atomic_load(&lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
    }
    // the first INCL in walk order (window k, lane l) ends the walk; every state up to it must be published
    uint32_t kk = kProbe, kl = 63;
    bool waiting = false;
#pragma unroll
    for (uint32_t k = 0; k < kProbe; k++) {
      if (kk < kProbe) break;
      const uint64_t incl = __ballot((v[k] & kLbIncl) != 0);
      const uint64_t upto = incl ? ((2ull << __builtin_ctzll(incl)) - 1) : ~0ull;
      if (__ballot(!(v[k] & (kLbAgg | kLbIncl))) & upto) waiting = true;
      if (incl) {
        kk = k;
        kl = (uint32_t)__builtin_ctzll(incl);
      }
    }
    if (waiting) {  // some needed state not published yet
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t part = 0;
#pragma unroll
    for (uint32_t k = 0; k < kProbe; k++)
      if (k < kk || (k == kk && lane <= kl)) part += v[k] & kLbVal;
    acc += wave_sum64(part);
    if (kk < kProbe) break;
    top -= 64 * kProbe;
  }
  if (lane == 0) __hip_atomic_store(&lb[page], kLbIncl | (acc + S), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return acc;
}

// RFC 3629 validity of the bytes [pos, pos + len) of a staged page, one
// thread (simdutf8's rules, as k_utf8_bytes: no overlong forms, no
// surrogates, nothing past U+10FFFF, no truncated sequence).
__device__ bool utf8_span_ok(const LdsSrc& s, uint32_t pos, uint32_t len) {
  auto trail = [](uint32_t b) { return (b & 0xC0u) == 0x80u; };
  for (uint32_t i = 0; i < len;) {
    const uint32_t b = s.u8(pos + i);
    if (b < 0x80u) {
      i++;
      continue;
    }
    const uint32_t L = b < 0xC2u ? 0u : b < 0xE0u ? 2u : b < 0xF0u ? 3u : b < 0xF5u ? 4u : 0u;
    if (L == 0 || L > len - i) return false;
    const uint32_t c1 = s.u8(pos + i + 1);
    if (!trail(c1) || (b == 0xE0u && c1 < 0xA0u) || (b == 0xEDu && c1 >= 0xA0u) || (b == 0xF0u && c1 < 0x90u) ||
        (b == 0xF4u && c1 >= 0x90u))
      return false;
    if (L >= 3 && !trail(s.u8(pos + i + 2))) return false;
    if (L == 4 && !trail(s.u8(pos + i + 3))) return false;
    i += L;
  }
  return true;
}

// Whether every row an Extend page emits is valid UTF-8 by itself: each row
// is a whole dictionary entry, the top value or an exception (OneValue /
// Dict / Freq), so checking those entries once is the whole-buffer check of
// Utf8Array::try_new (read/array/binary.rs:305-306) for the page's bytes --
// a concatenation of valid strings is valid and every row starts a
// character.  A page with an invalid entry (referenced or not) returns false
// and its emitted bytes are checked as they are.  All NT threads.
__device__ bool extend_entries_utf8(const LdsSrc& s, const BinInfo& bi, TabBase<true> tb, uint32_t n) {
  bool ok = true;
  const uint32_t tid = threadIdx.x;
  if (bi.codec == BIN_ONE) {
    if (tid == 0 && n) ok = utf8_span_ok(s, bi.top, bi.L);
  } else {
    const mptr<true, uint64_t> tab = tb.template at<uint64_t>(bi.otab);
    for (uint32_t x = tid; x < bi.k; x += NT) ok &= utf8_span_ok(s, (uint32_t)tab[x], (uint32_t)(tab[x] >> 32));
    if (bi.codec == BIN_FREQ && tid == 0 && bi.k < n) ok &= utf8_span_ok(s, bi.top, bi.L);
  }
  return !__syncthreads_or(!ok);
}

// Pass 2 over the staged pages (FUSED = false: bases from k_bin_size /
// k_bin_scan), or the whole decode in one pass when every page of the plan
// is staged (FUSED = true: pages claimed in order from a counter, each sized
// from its own tables and based by lookback, so k_bin_size / k_bin_scan do
// not run).
#ifdef SB_BIN_PHASES  // A/B instrumentation: per fused page, s_memrealtime at each phase boundary
__device__ uint64_t sb_dbg_phase[4096 * 6];
#define SB_PHASE(k) do { if (FUSED && threadIdx.x == 0 && page < 4096) sb_dbg_phase[page * 6 + (k)] = wall_clock64(); } while (0)
#else
#define SB_PHASE(k) do { } while (0)
#endif

template <int OW, bool FUSED, bool Z>
__device__ __forceinline__ void bin_decode_pages(BinArgs& a) {
  extern __shared__ u32x4 stage[];
  __shared__ Shared sh;
  __shared__ BinInfo bi;
  __shared__ Stream idx;
  __shared__ uint32_t claimed;
  __shared__ uint64_t base_v;
  uint8_t* lds = (uint8_t*)stage;
  const uint32_t tid = threadIdx.x;
  const uint32_t n_staged = FUSED ? a.n_pages : a.cls[4 * a.n_pages];
  for (uint32_t i = blockIdx.x;; i += gridDim.x) {
    if (FUSED) {
      if (tid == 0) claimed = atomicAdd((uint32_t*)(a.lb + a.n_pages), 1u);
      __syncthreads();
      i = claimed;
      __syncthreads();
    }
    if (i >= n_staged) break;
    const uint32_t page = FUSED ? i : a.cls[i];
    const PageDesc pd = a.pages[page];
    if (!FUSED && pd.reserved) continue;  // k_bin_big's
    SB_PHASE(0);
    const uint32_t n = pd.num_values;
    const uint64_t R = pd.row_off;
    const uint32_t stage_end = ((pd.byte_len + 15 + kStagePad) + 15) & ~15u;
    if (tid == 0) {
      sh.err = FUSED ? (pd.reserved || stage_end + 64 > a.lds_bytes ? ST_NYI : ST_OK) : a.status[page];  // sizing errors stand
      if (!FUSED && !sh.err && a.bases[page] + a.sizes[page] > a.values_cap) sh.err = ST_OUT_OF_SPEC;
    }
    __syncthreads();
    if (!FUSED && (sh.err || stage_end + 64 > a.lds_bytes)) {
      __syncthreads();
      if (tid == 0 && sh.err && !a.status[page]) a.status[page] = sh.err;
      continue;
    }
    uint32_t base = 0;
    if (!sh.err) {
      base = stage_page(stage, a.chunk + pd.byte_off, pd.byte_len);
      if (tid == 0) bin_parse<OW>(LdsSrc{(const uint32_t*)stage, base}, sh, bi, pd, a.nullable, true, stage_end,
                                  a.lds_bytes, &idx);
      __syncthreads();
    }
    LdsSrc s{(const uint32_t*)stage, base};
    const TabBase<true> tb{(lds_u8*)stage + bi.tb};
    SB_PHASE(1);
    if (FUSED) {  // tables (and so the size), then the base
      if (!sh.err) {
        if (bi.codec == BIN_DICT) {
          dict_tables<Z>(s, sh, bi, tb, idx, pd, a.chunk + pd.byte_off, lds, a.lds_bytes, nullptr, nullptr, true);
        } else if (bi.codec == BIN_FREQ) {
          freq_tables(s, sh, bi, tb, pd, nullptr);
          if (!sh.err) freq_rows(s, sh, bi, tb, n);
        } else if (bi.codec == 1 || bi.codec == 3) {
          set_err(sh, ST_NYI);  // (a plan with Basic LZ4 / Snappy pages is not fused)
        }
      }
      __syncthreads();
      SB_PHASE(2);
      if (tid < 64) {
        const uint64_t S = sh.err ? 0 : bi.S;
        const uint64_t v = lookback(a.lb, page, S);
        if (tid == 0) {
          base_v = v;
          a.bases[page] = v;
          a.sizes[page] = S;
          if (!sh.err && v + S > a.values_cap) sh.err = ST_OUT_OF_SPEC;
        }
      }
      __syncthreads();
    }
    const uint64_t V = FUSED ? base_v : a.bases[page];
    SB_PHASE(3);
    if (!sh.err) {
      if (sh.has_valid) write_validity(s, sh.vb_pos, n, R, a.out_validity);
      if (page == 0 && tid == 0) bin_put_off(a.out_offsets, 0, 0, OW);  // Extend codecs push 0 first
      if (bi.codec == 2) {  // Zstd: wave 0 decodes both streams into LDS; they then read as a None page
        if constexpr (!Z) {
          if (tid == 0) set_err(sh, ST_NYI);  // (a plan with Zstd streams launches the Z kernels)
        } else if (tid < 64) {
          const uint32_t tcap = a.lds_bytes - bi.ztab - kStagePad;
          uint32_t r = zs::zstd_to_lds(LdsSrc{s.w, s.base + bi.ob}, bi.ocs, (lds_u8*)(lds + bi.xoff), (n + 1) * OW,
                                       (lds_u8*)(lds + bi.ztab), tcap);
          if (!r)
            r = zs::zstd_to_lds(LdsSrc{s.w, s.base + bi.vb}, bi.vcs, (lds_u8*)(lds + bi.yoff), (uint32_t)bi.S,
                                (lds_u8*)(lds + bi.ztab), tcap);
          if (r) set_err(sh, r);
        }
        __syncthreads();
        if (tid == 0) {
          bi.ob = bi.xoff - base;
          bi.ocs = (n + 1) * OW;
          bi.vb = bi.yoff - base;
          bi.vcs = (uint32_t)bi.S;
          bi.codec = 0;
        }
        __syncthreads();
      }
      if (sh.err) {
      } else if (bi.codec <= 3) {
        // offsets: rows 1..n at V + p[i] (mod.rs:136-144 rebase); p[0] must be
        // 0 and p[n] the values length (the writer rebases, mod.rs:45-55)
        if (bi.codec != 0) {
          // expanded by k_inflate: offsets in scratch, values already at V
          const uint8_t* xo = a.scratch + (R + page) * OW;
          auto po = [&](uint32_t i) -> uint64_t {
            if constexpr (OW == 8) return ((const uint64_t*)xo)[i];
            else return (uint64_t)(int64_t)((const int32_t*)xo)[i];
          };
          if (tid == 0 && po(n) != bi.S) set_err(sh, ST_OUT_OF_SPEC);  // DEVIATION, as in k_bin_light_out
          __syncthreads();
          if (!sh.err) {
            if (page == 0 && tid == 0) bin_put_off(a.out_offsets, 0, po(0), OW);  // the first page keeps p[0]
            for (uint32_t i = tid + 1; i <= n; i += NT) bin_put_off(a.out_offsets, R + i, V + po(i), OW);
          }
        } else {
          const uint32_t opos = bi.ob;  // stream position of p[0]
          if (tid == 0 && (bi.ocs != (n + 1) * OW || bi.vcs != bi.S)) set_err(sh, ST_OUT_OF_SPEC);  // copy_from_slice
          __syncthreads();
          if (!sh.err && tid == 0) {
            if (ldo<OW>(s, opos + n * OW) != bi.S) set_err(sh, ST_OUT_OF_SPEC);  // DEVIATION, as above
          }
          __syncthreads();
          if (!sh.err) {
            if (page == 0 && tid == 0) bin_put_off(a.out_offsets, 0, ldo<OW>(s, opos), OW);
            for (uint32_t i = tid + 1; i <= n; i += NT) bin_put_off(a.out_offsets, R + i, V + ldo<OW>(s, opos + i * OW), OW);
            copy_lds_to_global(lds, base + bi.vb, a.out_values + V, bi.S);
          }
        }
      } else {
        if (!FUSED) {
          if (bi.codec == BIN_DICT) {
            dict_tables<Z>(s, sh, bi, tb, idx, pd, a.chunk + pd.byte_off, lds, a.lds_bytes, nullptr, nullptr, false);
          } else if (bi.codec == BIN_FREQ) {
            freq_tables(s, sh, bi, tb, pd, nullptr);
            if (!sh.err) freq_rows(s, sh, bi, tb, n);
          }
        }
        if (!sh.err) bin_emit_extend<OW>(sh, s, bi, tb, (lds_u32*)((lds_u8*)stage + bi.emit), n, R, V, a);
      }
    }
    __syncthreads();
    if (FUSED && a.checked) {  // Utf8: this page's rows need no byte check when its entries are valid
      const bool ext = !sh.err && (bi.codec == BIN_ONE || bi.codec == BIN_DICT || bi.codec == BIN_FREQ);
      const bool ok = ext && extend_entries_utf8(s, bi, tb, n);
      if (tid == 0) a.checked[page] = ok ? 1 : 0;
    }
    SB_PHASE(4);
    if (tid == 0) a.status[page] = sh.err;
    __syncthreads();
  }
}

template <int OW, bool Z>
__global__ __launch_bounds__(NT) void k_bin_decode(BinArgs a) {
  bin_decode_pages<OW, false, Z>(a);
}
template <int OW, bool Z>
__global__ __launch_bounds__(NT) void k_bin_fused(BinArgs a) {
  bin_decode_pages<OW, true, Z>(a);
}

// Big Extend pages (OneValue / Dict / Freq pages whose tables do not fit one
// workgroup's LDS, e.g. a write/common.rs:54-58 one-page column): read from
// HBM, tables in the page's HBM region (PageDesc.reserved - 1).  STAGE 0
// sizes them (entry walk, indices / exception rows into the region); STAGE 1
// emits offsets and values from those tables.
template <int OW, int STAGE>
__global__ __launch_bounds__(NT) void k_bin_big(BinArgs a) {
  extern __shared__ u32x4 dyn[];
  __shared__ Shared sh;
  __shared__ BinInfo bi;
  __shared__ Stream idx;
  uint8_t* lds = (uint8_t*)dyn;
  const uint32_t tid = threadIdx.x, np = a.n_pages, nbig = a.cls[4 * np + 2];
  for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
    const uint32_t page = a.cls[3 * np + i];
    const PageDesc pd = a.pages[page];
    const uint32_t n = pd.num_values;
    const GlbSrc s{a.chunk + pd.byte_off};
    uint8_t* rgn = a.region + (pd.reserved - 1);
    const TabBase<false> tb{(__attribute__((address_space(1))) uint8_t*)rgn};
    const uint64_t R = pd.row_off, V = STAGE ? a.bases[page] : 0;
    if (tid == 0) {
      sh.err = STAGE ? a.status[page] : 0u;
      if (STAGE && !sh.err && V + a.sizes[page] > a.values_cap) sh.err = ST_OUT_OF_SPEC;
    }
    __syncthreads();
    if (sh.err) {
      __syncthreads();
      if (tid == 0 && STAGE && !a.status[page]) a.status[page] = sh.err;
      continue;
    }
    if (tid == 0) {
      bin_parse<OW>(s, sh, bi, pd, a.nullable, false, 0, 0, &idx);
      if (!sh.err && bi.codec <= 3) set_err(sh, ST_NYI);  // (Basic pages are never big)
    }
    __syncthreads();
    if (!sh.err) {
      if (STAGE == 0) {
        if (bi.codec == BIN_DICT) {
          dict_tables<true>(s, sh, bi, tb, idx, pd, a.chunk + pd.byte_off, nullptr, 0, lds, rgn, true);
        } else if (bi.codec == BIN_FREQ) {
          freq_tables(s, sh, bi, tb, pd, rgn);
          if (!sh.err) freq_rows(s, sh, bi, tb, n);
        }
      } else {
        if (sh.has_valid) write_validity(s, sh.vb_pos, n, R, a.out_validity);
        if (page == 0 && tid == 0) bin_put_off(a.out_offsets, 0, 0, OW);
        if (bi.codec == BIN_FREQ) {  // the exceptions consumed (the bitmap and walk are in the region)
          roaring_build(s, sh, rgn + bi.oroar, (uint32_t)roar_cap(n));
          if (tid == 0 && !sh.err) {
            uint32_t ep = 0, hi_e = bi.tot;
            while (ep < hi_e) {
              const uint32_t mid = (ep + hi_e) / 2;
              if (roaring_select(s, sh, mid) < n) ep = mid + 1;
              else hi_e = mid;
            }
            bi.k = ep;
          }
          __syncthreads();
        }
        if (!sh.err) bin_emit_extend<OW>(sh, s, bi, tb, (lds_u32*)((lds_u8*)dyn + kBigEmit), n, R, V, a);
      }
    }
    __syncthreads();
    if (tid == 0) {
      a.status[page] = sh.err;
      if (STAGE == 0) a.sizes[page] = sh.err ? 0 : bi.S;
    }
    __syncthreads();
  }
}

// ===========================================================================
// UTF-8 validation of a decoded Utf8 / LargeUtf8 column.  The reference builds
// the array with Utf8Array::try_new (read/array/binary.rs:305-306), i.e.
// arrow2 0.17 try_check_utf8: the whole values buffer must be UTF-8
// (simdutf8::basic::from_utf8, RFC 3629: no overlong forms, no surrogates,
// nothing above U+10FFFF) and, unless it is all ASCII, every offset up to the
// last one below the values length must start a character (not 0b10xxxxxx).
// k_utf8_bytes: 16 bytes a thread (a lead byte checks its trail bytes, a
// trail byte finds its lead at most 3 bytes back); it raises flags[0] when it
// sees a non-ASCII byte.  k_utf8_bounds: one offset a thread, only then.  A
// failure marks the page that holds the byte / row OutOfSpec.
// ===========================================================================
using Utf8Args = Utf8Launch;

// the last page whose key (values base / first row) is <= x: the non-empty
// page holding x when empty pages share its key
template <class KeyF>
__device__ uint32_t utf8_page(uint32_t n, uint64_t x, KeyF key) {
  uint32_t lo = 0, hi = n;  // key(lo) <= x < key(hi)
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) / 2;
    if (key(m) <= x) lo = m;
    else hi = m;
  }
  return lo;
}

// Bytes [pos, pos + 4) of the buffer as a little-endian word, 0 outside
// [0, len) (a 0 byte is neither a lead nor a trail byte).  pos is a multiple
// of 4 when ALIGNED.
template <bool ALIGNED>
__device__ __forceinline__ uint32_t utf8_word(const uint8_t* v, uint64_t len, int64_t pos) {
  if (pos < 0 || (uint64_t)pos >= len) return 0;
  const uint64_t rem = len - (uint64_t)pos;
  uint32_t w;
  if (ALIGNED) {
    w = *(const uint32_t*)(v + pos);
  } else {
    w = 0;
    for (uint32_t j = 0; j < 4 && j < rem; j++) w |= (uint32_t)v[pos + j] << (8 * j);
  }
  return rem >= 4 ? w : w & ((1u << (8 * rem)) - 1);
}

__device__ __forceinline__ bool utf8_trail(uint32_t b) { return (b & 0xC0u) == 0x80u; }
// sequence length of a lead byte, 0 if the byte cannot start one
__device__ __forceinline__ uint32_t utf8_len(uint32_t b) {
  return b < 0x80u ? 1u : b < 0xC2u ? 0u : b < 0xE0u ? 2u : b < 0xF0u ? 3u : b < 0xF5u ? 4u : 0u;
}

// The 16 bytes of chunk c: a bad byte marks its page OutOfSpec; a non-ASCII
// byte raises flags[0].
template <bool ALIGNED>
__device__ __forceinline__ void utf8_chunk(const Utf8Args& a, uint64_t c) {
  {
    const int64_t p0 = (int64_t)(c * 16);
    uint32_t w[6];  // bytes [p0 - 4, p0 + 20)
    if (ALIGNED && (uint64_t)p0 + 16 <= a.len) {
      const u32x4 m = *(const u32x4*)(a.values + p0);
      w[1] = m.x, w[2] = m.y, w[3] = m.z, w[4] = m.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) w[1 + k] = utf8_word<ALIGNED>(a.values, a.len, p0 + 4 * k);
    }
    const bool ascii = ((w[1] | w[2] | w[3] | w[4]) & 0x80808080u) == 0;
    if (!ascii && *(volatile uint32_t*)a.flags == 0) atomicOr(a.flags, 1u);
    if (ascii) return;  // no trail byte here; a lead just before is checked by its own thread
    w[0] = utf8_word<ALIGNED>(a.values, a.len, p0 - 4);
    w[5] = utf8_word<ALIGNED>(a.values, a.len, p0 + 16);
    auto at = [&](int i) { return (w[(i + 4) >> 2] >> (8 * ((i + 4) & 3))) & 0xFFu; };  // i in [-4, 20)
    bool bad = false;
    int64_t bad_pos = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t b = at(j);
      bool ok = true;
      if (b < 0x80u) {
      } else if (utf8_trail(b)) {  // its lead: the first non-trail byte 1..3 back must start a longer sequence
        const uint32_t b1 = at(j - 1), b2 = at(j - 2), b3 = at(j - 3);
        ok = !utf8_trail(b1) ? utf8_len(b1) > 1 : !utf8_trail(b2) ? utf8_len(b2) > 2 : !utf8_trail(b3) && utf8_len(b3) > 3;
      } else {
        const uint32_t L = utf8_len(b), c1 = at(j + 1);
        ok = L >= 2 && utf8_trail(c1);
        if (L >= 3) ok &= utf8_trail(at(j + 2));
        if (L == 4) ok &= utf8_trail(at(j + 3));
        // second-byte ranges: E0 A0..BF, ED 80..9F (no surrogates), F0 90..BF, F4 80..8F
        if (b == 0xE0u) ok &= c1 >= 0xA0u;
        if (b == 0xEDu) ok &= c1 < 0xA0u;
        if (b == 0xF0u) ok &= c1 >= 0x90u;
        if (b == 0xF4u) ok &= c1 < 0x90u;
      }
      if (!ok && !bad && (uint64_t)(p0 + j) < a.len) bad = true, bad_pos = p0 + j;
    }
    if (bad) {
      const uint32_t pg = utf8_page(a.n_pages, (uint64_t)bad_pos, [&](uint32_t i) { return a.bases[i]; });
      atomicCAS(&a.status[pg], (uint32_t)ST_OK, (uint32_t)ST_OUT_OF_SPEC);  // (a page's earlier failure stands)
    }
  }
}

template <bool ALIGNED>
__global__ __launch_bounds__(NT) void k_utf8_bytes(Utf8Args a) {
  const uint64_t chunks = (a.len + 15) / 16;
  for (uint64_t c = blockIdx.x * (uint64_t)NT + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * NT)
    utf8_chunk<ALIGNED>(a, c);
}

// The same check page by page, skipping the pages whose values k_inflate
// found all ASCII (a.ascii[page]): their bytes are characters by
// themselves, and a lead byte before such a page still checks its trail
// bytes in it.  The chunks a page's values range touches (a chunk on a page
// boundary is checked by both pages).
template <bool ALIGNED>
__global__ __launch_bounds__(NT) void k_utf8_pages(Utf8Args a) {
  for (uint32_t pg = blockIdx.x; pg < a.n_pages; pg += gridDim.x) {
    if (a.ascii[pg]) continue;
    const uint64_t b = a.bases[pg], e = pg + 1 < a.n_pages ? a.bases[pg + 1] : a.len;
    if (b >= e) continue;
    for (uint64_t c = b / 16 + threadIdx.x; c < (e + 15) / 16; c += NT) utf8_chunk<ALIGNED>(a, c);
  }
}

// Offsets j <= last, where last = the last j >= 1 whose offset is below the
// values length (offsets are non-decreasing: j >= 1 is checked iff its offset
// is below it, offset 0 iff offset 1 is).
template <int OW>
__global__ __launch_bounds__(NT) void k_utf8_bounds(Utf8Args a) {
  if (*(volatile uint32_t*)a.flags == 0) return;  // all ASCII: every byte starts a character
  using O = typename VT<OW>::T;
  const O* off = (const O*)a.offsets;
  for (uint64_t j = blockIdx.x * (uint64_t)NT + threadIdx.x; j <= a.n_rows; j += (uint64_t)gridDim.x * NT) {
    const uint64_t o = (uint64_t)off[j];
    const bool in = j == 0 ? (a.n_rows >= 1 && (uint64_t)off[1] < a.len && o < a.len) : o < a.len;
    if (in && utf8_trail(a.values[o])) {
      const uint64_t row = j < a.n_rows ? j : a.n_rows - 1;
      const uint32_t pg = utf8_page(a.n_pages, row, [&](uint32_t i) { return a.pages[i].row_off; });
      atomicCAS(&a.status[pg], (uint32_t)ST_OK, (uint32_t)ST_OUT_OF_SPEC);
    }
  }
}

// ===========================================================================
// Boolean pages (BooleanIter::deserialize / read_boolean,
// read/array/boolean.rs:59-79, 191-219; decompress_boolean,
// compression/boolean/mod.rs:63-102).  One workgroup per page: the page is
// staged in LDS, the values bitmap is produced page-relative (None: the
// staged bytes themselves; RLE / LZ4 / Snappy: expanded into an LDS bitmap)
// and funnel-shifted to the page's first row like the validity.
// ===========================================================================
__device__ void fill_bits(uint32_t n, uint64_t row_off, bool v, uint32_t* out) {
  if (n == 0) return;
  const uint64_t fw = row_off >> 5, lw = (row_off + n - 1) >> 5;
  for (uint64_t w = fw + threadIdx.x; w <= lw; w += NT) {
    const int64_t pb = (int64_t)(w * 32) - (int64_t)row_off;
    const uint32_t lo = pb < 0 ? (uint32_t)(-pb) : 0u;
    const int64_t hi_ex = (int64_t)n - pb;
    const uint32_t hi = hi_ex >= 32 ? 32u : (uint32_t)hi_ex;
    const uint32_t m = (hi == 32 ? 0xFFFFFFFFu : ((1u << hi) - 1)) & (0xFFFFFFFFu << lo);
    if (m == 0xFFFFFFFFu) out[w] = v ? m : 0u;
    else if (v) atomicOr(&out[w], m);
  }
}

// Page-relative bits [b, e) set in a zeroed word bitmap: whole words stored,
// the two edge words OR-ed (a neighbouring run owns their other bits).
__device__ __forceinline__ void set_bit_range(uint32_t* bm, uint64_t b, uint64_t e) {
  if (b >= e) return;
  const uint64_t fw = b >> 5, lw = (e - 1) >> 5;
  for (uint64_t w = fw; w <= lw; w++) {
    const uint32_t lo = w == fw ? (uint32_t)(b & 31) : 0u;
    const uint32_t hi = w == lw ? (uint32_t)((e - 1) & 31) : 31u;
    const uint32_t m = (hi == 31 ? 0xFFFFFFFFu : ((2u << hi) - 1)) & (0xFFFFFFFFu << lo);
    if (m == 0xFFFFFFFFu) bm[w] = m;
    else atomicOr(&bm[w], m);
  }
}

// A Boolean page whose bytes plus expanded bitmap exceed the LDS
// (max_page_size = None writes one page per column chunk,
// write/common.rs:54-58): parsed from HBM; None pages funnel-shift their
// bitmap bytes from the page, OneValue fills; RLE runs (each thread walks its
// own chunk of runs, rle_prepare's starts) and LZ4 / Snappy / Zstd streams
// (wave 0, expand_to_hbm) expand into the page's HBM region, which is then
// funnel-shifted to the page's first row.  `lds` = the dynamic LDS
// (expand_to_hbm's kBig* layout).
template <bool Z>
__device__ void bool_big_page(const LaunchArgs& a, uint32_t page, const PageDesc& pd, Shared& sh, Stream& bs,
                              uint8_t* lds) {
  const uint32_t tid = threadIdx.x, n = pd.num_values, len = pd.byte_len, nb = (n + 7) / 8;
  const GlbSrc s{a.chunk + pd.byte_off};
  uint8_t* rg = a.region + (pd.reserved & kRegionOffMask);
  uint32_t* rw = (uint32_t*)rg;
  if (tid == 0) {
    uint32_t p = 0;
    sh.has_valid = 0;
    do {
      if (a.nullable && !parse_validity(s, sh, len, n, &p)) break;
      if (!parse_stream(s, p, len, n, &bs)) { set_err(sh, ST_IO); break; }
    } while (0);
  }
  __syncthreads();
  if (sh.err) return;
  if (sh.has_valid) write_validity(s, sh.vb_pos, n, pd.row_off, a.out_validity);
  const Stream st = bs;
  switch (st.codec) {
    case 0:  // the page's bitmap bytes (basic.rs:68-71)
      if (st.csize != nb) { if (tid == 0) set_err(sh, ST_OUT_OF_SPEC); }
      else write_validity(s, st.body, n, pd.row_off, (uint32_t*)a.out_values);
      return;
    case 12:  // OneValue (boolean/one_value.rs:54-61)
      if (st.body >= len) { if (tid == 0) set_err(sh, ST_IO); }
      else fill_bits(n, pd.row_off, s.u8(st.body) != 0, (uint32_t*)a.out_values);
      return;
    case 10: {  // RLE (boolean/rle.rs:41-55): (u32 count, u8 value) runs over the rest of the page
      for (uint32_t w = tid; w < (n + 31) / 32; w += NT) rw[w] = 0;
      __threadfence();  // (the zeroes reach L2 before any run's atomics)
      const Stream rs{10u, st.body, len - st.body, n};
      rle_prepare<1>(s, sh, rs);  // run sums, chunk starts, overshoot / short checks (syncs)
      if (sh.err) return;
      const uint32_t R = sh.rle_R, c = sh.rle_c;
      const uint32_t r0 = min(R, tid * c), r1 = min(R, r0 + c);
      uint64_t b = sh.rle_start[tid];
      for (uint32_t r = r0; r < r1 && b < n; r++) {
        const uint32_t cnt = s.u32(rs.body + 5 * r);
        const uint64_t e = min<uint64_t>(b + cnt, n);
        if (s.u8(rs.body + 5 * r + 4) != 0) set_bit_range(rw, b, e);
        b += cnt;
      }
      break;
    }
    case 1:
    case 2:
    case 3:  // LZ4 / Zstd / Snappy over the bitmap bytes
      if (tid < 64) {
        const uint32_t r = expand_to_hbm<Z>(st.codec, a.chunk + pd.byte_off + st.body, st.csize, rg, nb, lds);
        if (r && tid == 0) set_err(sh, r);
      }
      break;
    default:
      if (tid == 0) set_err(sh, ST_OUT_OF_SPEC);  // Compression::from_codec / from_compression
      return;
  }
  __threadfence();  // release the region's bytes ...
  __syncthreads();
  __threadfence();  // ... and drop stale L1 lines before reading them back
  if (!sh.err) write_validity(GlbSrc{rg}, 0, n, pd.row_off, (uint32_t*)a.out_values);
}

template <bool Z>
__global__ __launch_bounds__(NT) void k_bool_decode(LaunchArgs a) {
  extern __shared__ u32x4 stage[];
  __shared__ Shared sh;
  __shared__ Stream bs;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < a.n_list; i += gridDim.x) {
    const uint32_t page = a.list ? a.list[i] : i;
    const PageDesc pd = a.pages[page];
    const uint32_t n = pd.num_values, len = pd.byte_len;
    const uint32_t need = (len + 15 + kStagePad + 15) & ~15u;
    const uint32_t xb = ((n + 7) / 8 + 15) & ~15u;
    if (tid == 0) sh.err = 0;
    if (a.region && pd.reserved) {  // planned as a big page (sb_api plan_bool_regions)
      __syncthreads();
      bool_big_page<Z>(a, page, pd, sh, bs, (uint8_t*)stage);
      __syncthreads();
      if (tid == 0) a.status[page] = sh.err;
      __syncthreads();
      continue;
    }
    if (need + xb + kStagePad > a.stage_bytes) {  // page + bitmap larger than the LDS budget
      __syncthreads();
      if (tid == 0) a.status[page] = ST_NYI;
      continue;
    }
    const uint32_t base = stage_page(stage, a.chunk + pd.byte_off, len);
    LdsSrc s{(const uint32_t*)stage, base};
    if (tid == 0) {
      uint32_t p = 0;
      sh.has_valid = 0;
      do {
        if (a.nullable && !parse_validity(s, sh, len, n, &p)) break;
        if (!parse_stream(s, p, len, n, &bs)) { set_err(sh, ST_IO); break; }
      } while (0);
    }
    __syncthreads();
    if (!sh.err) {
      if (sh.has_valid) write_validity(s, sh.vb_pos, n, pd.row_off, a.out_validity);
      const Stream st = bs;
      uint32_t* xbits = (uint32_t*)((uint8_t*)stage + need);
      const LdsSrc xs{(const uint32_t*)stage, need};
      switch (st.codec) {
        case 0:  // the page's bitmap bytes (basic.rs:68-71: exactly (n + 7) / 8 of them)
          if (st.csize != (n + 7) / 8) { if (tid == 0) set_err(sh, ST_OUT_OF_SPEC); break; }
          write_validity(s, st.body, n, pd.row_off, (uint32_t*)a.out_values);
          break;
        case 12:  // OneValue (boolean/one_value.rs:54-61): the rest of the page, not csize
          if (st.body >= len) { if (tid == 0) set_err(sh, ST_IO); break; }
          fill_bits(n, pd.row_off, s.u8(st.body) != 0, (uint32_t*)a.out_values);
          break;
        case 10: {  // RLE (boolean/rle.rs:41-55): (u32 count, u8 value) runs over the rest of the page
          for (uint32_t w = tid; w < xb / 4; w += NT) xbits[w] = 0;
          __syncthreads();
          const Stream rs{10u, st.body, len - st.body, n};
          run_leaf<1>(s, sh, rs, [&](uint32_t row, const uint32_t* v, uint32_t nv) {
            uint32_t nib = 0;
            for (uint32_t l = 0; l < nv; l++) nib |= (v[l] != 0 ? 1u : 0u) << l;
            if (nib) atomicOr(&xbits[row >> 5], nib << (row & 31));
          });
          __syncthreads();
          if (!sh.err) write_validity(xs, 0, n, pd.row_off, (uint32_t*)a.out_values);
          break;
        }
        case 1:
        case 3: {  // LZ4 / Snappy over the bitmap bytes, expanded into LDS by wave 0
          if (tid < 64) {
            const uint32_t r = expand_to_lds(st.codec, a.chunk + pd.byte_off + st.body, st.csize, (lds_u8*)xbits,
                                             (n + 7) / 8);
            if (r) set_err(sh, r);
          }
          __syncthreads();
          if (!sh.err) write_validity(xs, 0, n, pd.row_off, (uint32_t*)a.out_values);
          break;
        }
        case 2:  // Zstd over the bitmap bytes: wave 0 decodes into LDS, its tables after the bitmap
          if (!Z || need + xb + kZTablesBytes + kStagePad > a.stage_bytes) {
            if (tid == 0) set_err(sh, ST_NYI);  // (Z false: a plan with Zstd pages launches the Z kernel)
            break;
          }
          if constexpr (Z) if (tid < 64) {
            const uint32_t r = zs::zstd_to_lds(LdsSrc{s.w, s.base + st.body}, st.csize, (lds_u8*)xbits, (n + 7) / 8,
                                               (lds_u8*)xbits + xb, a.stage_bytes - need - xb - kStagePad);
            if (r) set_err(sh, r);
          }
          __syncthreads();
          if (!sh.err) write_validity(xs, 0, n, pd.row_off, (uint32_t*)a.out_values);
          break;
        default:
          if (tid == 0) set_err(sh, ST_OUT_OF_SPEC);  // Compression::from_codec / from_compression
      }
    }
    __syncthreads();
    if (tid == 0) a.status[page] = sh.err;
    __syncthreads();
  }
}

// ===========================================================================
// Nested List<primitive> pages: read_validity_nested (read/read_basic.rs:65-173)
// + create_list (read/array/list.rs:48), one list level over a primitive leaf.
// Page = [u32 rows][u32 rep_len][u32 def_len][rep hybrid][def hybrid][values].
// Per level: rep == 0 starts a row (list offset = leaves so far, list valid =
// def > 0); def >= cum_sum[1] = nl + 1 is a leaf (leaf valid = def > nl + 1);
// decoding stops before the level that would start row `rows + 1`
// (:158-162).  k_list_size counts each page's rows and leaves and fills the
// page's values-stream descriptor, k_list_scan turns counts into bases,
// k_list_levels writes offsets and both bitmaps; the values streams then go
// through the flat decode kernels (k_decode_staged / global / deferred /
// k_inflate) at their leaf bases.
// ===========================================================================
constexpr uint32_t kLvK = 32;                   // levels per thread per tile
constexpr uint32_t kMaxRuns = 64;               // hybrid runs per level stream

struct LvRuns {
  uint32_t n;
  uint32_t start[kMaxRuns + 1];  // first level of each run
  uint32_t arg[kMaxRuns];        // bit-packed: 0x80000000 | payload position; RLE: the value
};

struct ListShared {
  uint32_t rows, vpos, bw_def, region, fast;
  LvRuns rep, def;
};

__device__ __forceinline__ void put_err(uint32_t* err, uint32_t code) { *err = max(*err, code); }

// parquet2 HybridRleDecoder (hybrid_rle/decoder.rs) run headers of one level
// stream [p, end) covering L levels, bit width bw.  One lane.
template <class Src>
__device__ bool parse_runs(const Src& s, uint32_t* err, uint32_t p, uint32_t end, uint32_t L, uint32_t bw, LvRuns& R) {
  uint32_t covered = 0, n = 0;
  while (covered < L) {
    uint32_t h = 0, sft = 0;
    for (;;) {  // ULEB128 header
      if (p >= end || sft > 28) { put_err(err, ST_OUT_OF_SPEC); return false; }
      const uint32_t c = s.u8(p++);
      h |= (c & 0x7Fu) << sft;
      if (!(c & 0x80)) break;
      sft += 7;
    }
    if (n == kMaxRuns) { put_err(err, ST_NYI); return false; }
    R.start[n] = covered;
    if (h & 1) {  // bit-packed: h >> 1 groups of 8, clamped to the bytes present
      const uint64_t want = (uint64_t)(h >> 1) * bw;
      const uint32_t have = (uint32_t)min<uint64_t>(want, end - p);
      const uint32_t vals = (uint32_t)min<uint64_t>((uint64_t)(h >> 1) * 8, (uint64_t)have * 8 / bw);
      if (vals == 0) { put_err(err, ST_OUT_OF_SPEC); return false; }
      R.arg[n] = 0x80000000u | p;
      p += have;
      covered += vals;
    } else {  // RLE: h >> 1 repeats of a ceil(bw / 8)-byte value
      const uint32_t vb = (bw + 7) / 8;
      if (p + vb > end) { put_err(err, ST_OUT_OF_SPEC); return false; }
      uint32_t v = 0;
      for (uint32_t k = 0; k < vb; k++) v |= s.u8(p + k) << (8 * k);
      R.arg[n] = v;
      p += vb;
      covered += h >> 1;
    }
    n++;
  }
  R.start[n] = covered;
  R.n = n;
  return true;
}

template <class Src>
__device__ __forceinline__ uint32_t level_at(const Src& s, const LvRuns& R, uint32_t i, uint32_t bw) {
  uint32_t r = 0;
  if (R.n > 1) {  // last run starting at or before i
    uint32_t lo = 0, hi = R.n;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (R.start[mid] <= i) lo = mid; else hi = mid;
    }
    r = lo;
  }
  const uint32_t a = R.arg[r];
  if (!(a & 0x80000000u)) return a;
  const uint32_t bit = (i - R.start[r]) * bw;
  return (s.u32((a & 0x7FFFFFFFu) + (bit >> 3)) >> (bit & 7)) & ((1u << bw) - 1);
}

struct ListArgs {
  const uint8_t* chunk;
  const PageDesc* pages;  // num_values = the page's level count (PageMeta.num_values)
  uint32_t n_pages;
  uint32_t nl, ni, ow;    // list nullable, item nullable, offset width
  uint32_t width;         // leaf value width (the values header's usize / width = leaves)
  uint32_t peek;          // sizes from the page headers (verified at plan time) instead of the levels
  uint64_t* counts;       // [n_pages] rows << 32 | leaves
  uint64_t* local;        // [2 n_pages] row / leaf bases within the page's block of NT pages
  uint64_t* blk;          // [2 ceil(n_pages / NT)] row / leaf totals of each block
  uint64_t* totals;       // [2] rows, leaves
  uint4* lvdesc;          // [2 n_pages] per page: the parse results the levels pass reuses
  PageDesc* vpages;       // values stream of each page, as a flat page at its leaf base
  uint8_t* out_offsets;
  uint32_t* out_list_validity;
  uint32_t* out_leaf_validity;
  uint32_t* status;
  uint32_t epoch;             // k_list_bases: tag of this decode's block totals
};

// Header + run tables (one lane).
template <class Src>
__device__ bool list_parse(const Src& s, uint32_t* err, ListShared& ls, const PageDesc& pd, const ListArgs& a) {
  const uint32_t len = pd.byte_len, L = pd.num_values;
  if (len < 12) { put_err(err, ST_IO); return false; }
  const uint32_t rows = s.u32(0), rl = s.u32(4), dl = s.u32(8);
  if ((uint64_t)12 + rl + dl > len) { put_err(err, ST_IO); return false; }
  const uint32_t max_def = a.nl + 1 + a.ni;
  ls.rows = rows;
  ls.vpos = 12 + rl + dl;
  ls.region = 12 + rl + dl;
  ls.bw_def = 32 - __clz(max_def);
  if (!parse_runs(s, err, 12, 12 + rl, L, 1, ls.rep)) return false;
  if (!parse_runs(s, err, 12 + rl, 12 + rl + dl, L, ls.bw_def, ls.def)) return false;
  if (L > 0 && rows == 0) { put_err(err, ST_OUT_OF_SPEC); return false; }
  // the writer's shape: one bit-packed run per stream, def bit width <= 2
  ls.fast = ls.rep.n == 1 && (ls.rep.arg[0] & 0x80000000u) && ls.def.n == 1 && (ls.def.arg[0] & 0x80000000u) &&
            ls.bw_def <= 2;
  return true;
}

// Gathers the even bits of x (bit 2j -> bit j).
__device__ __forceinline__ uint32_t compact_even(uint64_t x) {
  x &= 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
  return (uint32_t)x;
}

// little-endian bytes [p, p + nb) of the page, nb <= 8, never past `end`
template <class Src>
__device__ __forceinline__ uint64_t ld_bytes(const Src& s, uint32_t p, uint32_t nb, uint32_t end) {
  if (p + 8 <= end) return s.u64(p) & (nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1));
  uint64_t v = 0;
  for (uint32_t k = 0; k < nb && p + k < end; k++) v |= (uint64_t)s.u8(p + k) << (8 * k);
  return v;
}

// Level masks of 32 consecutive levels [i0, i0 + 32): rsm = row starts
// (rep 0), lfm = leaves (def >= nl + 1), lvm = def > 0, fvm = def > nl + 1.
struct LvMasks {
  uint32_t vm, rsm, lfm, lvm, fvm;
};

// Level masks of a page whose level streams are one bit-packed run each (the
// writer's shape): rep payload at rp, def payload at dp (the rep stream ends
// there), def bit width bw <= 2, level streams end at `region`.
template <class Src>
__device__ __forceinline__ LvMasks fast_level_masks(const Src& s, uint32_t rp, uint32_t dp, uint32_t region, uint32_t bw,
                                                    uint32_t i0, uint32_t L, uint32_t cs1) {
  LvMasks m{0, 0, 0, 0, 0};
  if (i0 >= L) return m;
  m.vm = L - i0 >= 32 ? 0xFFFFFFFFu : ((1u << (L - i0)) - 1);
  const uint32_t repw = (uint32_t)ld_bytes(s, rp + i0 / 8, 4, dp);
  m.rsm = ~repw & m.vm;
  const uint64_t dw = ld_bytes(s, dp + i0 * bw / 8, 4 * bw, region);
  auto ge = [&](uint32_t t) -> uint32_t {
    if (t == 0) return 0xFFFFFFFFu;
    if (bw == 1) return t == 1 ? (uint32_t)dw : 0u;
    const uint32_t lo = compact_even(dw), hi = compact_even(dw >> 1);
    return t == 1 ? (lo | hi) : t == 2 ? hi : (hi & lo);
  };
  m.lfm = ge(cs1) & m.vm;
  m.lvm = ge(1) & m.vm;
  m.fvm = ge(cs1 + 1) & m.vm;
  return m;
}

template <class Src>
__device__ __forceinline__ LvMasks level_masks(const Src& s, const ListShared& ls, uint32_t i0, uint32_t L,
                                               uint32_t cs1) {
  if (ls.fast)  // direct bit slices of the single bit-packed runs
    return fast_level_masks(s, ls.rep.arg[0] & 0x7FFFFFFFu, ls.def.arg[0] & 0x7FFFFFFFu, ls.region, ls.bw_def, i0, L, cs1);
  LvMasks m{0, 0, 0, 0, 0};
  if (i0 >= L) return m;
  m.vm = L - i0 >= 32 ? 0xFFFFFFFFu : ((1u << (L - i0)) - 1);
  const uint32_t bw = ls.bw_def;
  for (uint32_t k = 0; k < 32; k++) {
    const uint32_t i = i0 + k;
    if (i >= L) break;
    const uint32_t r = level_at(s, ls.rep, i, 1), d = level_at(s, ls.def, i, bw);
    if (r == 0) m.rsm |= 1u << k;
    if (r <= 1 && d >= cs1) m.lfm |= 1u << k;
    if (d > 0) m.lvm |= 1u << k;
    if (d > cs1) m.fvm |= 1u << k;
  }
  return m;
}

// OR `nbits` (<= 32) bits of v into the LDS bitmap at bit position pos
__device__ __forceinline__ void lds_or_bits(uint32_t* bm, uint32_t pos, uint64_t v, uint32_t nbits) {
  if (!nbits || !v) return;
  const uint32_t w = pos >> 5, sft = pos & 31;
  const uint64_t lo = v << sft;
  atomicOr(&bm[w], (uint32_t)lo);
  if ((uint32_t)(lo >> 32)) atomicOr(&bm[w + 1], (uint32_t)(lo >> 32));
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}


// n bits of an LDS bitmap (bit 0 at word 0, zero past n, one spare zero word
// before it at bm[-1]) to global bit position g0: the shift is uniform over
// the wave, so output word i is a funnel of bm[i - 1] and bm[i]; interior
// words are stored.  An edge word, shared with the neighbouring range, gets
// its own bits cleared (atomicAnd) and then set (atomicOr): the neighbour's
// bits are never touched, so the bitmap needs no zeroing first.
__device__ __forceinline__ void wave_put_bits(const uint32_t* bm, uint32_t n, uint64_t g0, uint32_t* out) {
  if (n == 0) return;
  const uint32_t sh = (uint32_t)(g0 & 31), nw = (sh + n + 31) >> 5, eb = (sh + n) & 31;
  uint32_t* o = out + (g0 >> 5);
  for (uint32_t i = threadIdx.x & 63; i < nw; i += 64) {
    const uint32_t v = sh ? __builtin_amdgcn_alignbit(bm[i], bm[(int)i - 1], 32 - sh) : bm[i];
    const bool lo_edge = i == 0 && sh, hi_edge = i == nw - 1 && eb;
    if (lo_edge || hi_edge) {
      uint32_t m = lo_edge ? ~0u << sh : ~0u;
      if (hi_edge) m &= (1u << eb) - 1;
      atomicAnd(&o[i], ~m);
      if (v) atomicOr(&o[i], v);
    } else {
      o[i] = v;
    }
  }
}

#ifndef SB_LV_STAGE
#define SB_LV_STAGE 4160
#endif
#ifndef SB_LV_STAGE_PAD
#define SB_LV_STAGE_PAD 16  // (>= 3 dwords: LdsSrc::u64 reads two words past the last staged one)
#endif
constexpr uint32_t kLvStage = SB_LV_STAGE;  // page bytes staged per wave (header + level streams)
constexpr uint32_t kLvStep = 64 * kLvK;  // levels per wave step (2048)

#ifndef SB_LV_ACC_BITS
#define SB_LV_ACC_BITS 8192
#endif
// The page's validity bits accumulate over its steps and go out once per
// kLvAccBits (a C4 page: once), as whole words with two edge merges,
// instead of a short partial-line write and two atomics every step.
constexpr uint32_t kLvAccBits = SB_LV_ACC_BITS;
constexpr uint32_t kLvBitsW = kLvAccBits / 32 + 2;

struct ListWave {
  ListShared ls;
  uint32_t err;
  alignas(16) uint16_t obuf[kLvStep + 8];  // step-relative leaf offset of each row start, at row + (g0 & 3)
  uint32_t lbits[kLvBitsW];   // [0] = 0, then the list-validity bits held (rows)
  uint32_t fbits[kLvBitsW];   // [0] = 0, then the leaf-validity bits held (leaves)
};

// Validity bits held in ListWave.lbits / fbits: r / l bits from global bit
// positions g0 / v0 (uniform over the wave).
struct LvAcc {
  uint32_t r, l;
  uint64_t g0, v0;
};

// Page bytes: the staged prefix from LDS, the rest from HBM.
struct StageSrc {
  LdsSrc l;
  GlbSrc g;
  uint32_t lim;  // staged page bytes
  __device__ __forceinline__ uint32_t u8(uint32_t i) const { return i < lim ? l.u8(i) : g.u8(i); }
  __device__ __forceinline__ uint32_t u32(uint32_t i) const { return i + 4 <= lim ? l.u32(i) : g.u32(i); }
  __device__ __forceinline__ uint64_t u64(uint32_t i) const { return i + 8 <= lim ? l.u64(i) : g.u64(i); }
};

// Hacker's Delight 7-4 compress: the bits of x at the set positions of m,
// packed to the low end (a branch-free pext).
__device__ __forceinline__ uint32_t compress32(uint32_t x, uint32_t m) {
  x &= m;
  uint32_t mk = ~m << 1;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    uint32_t mp = mk ^ (mk << 1);
    mp ^= mp << 2;
    mp ^= mp << 4;
    mp ^= mp << 8;
    mp ^= mp << 16;
    const uint32_t mv = mp & m;
    m = (m ^ mv) | (mv >> (1 << i));
    const uint32_t t = x & mv;
    x = (x ^ t) | (t >> (1 << i));
    mk &= ~mp;
  }
  return x;
}

// The held validity bits to the bitmaps; the buffers zeroed again.
__device__ __forceinline__ void lv_flush(ListWave& w, const ListArgs& a, LvAcc& acc) {
  const uint32_t lane = threadIdx.x & 63;
#ifndef SB_V_LV_NOBITS
  if (a.nl) wave_put_bits(w.lbits + 1, acc.r, acc.g0, a.out_list_validity);
  if (a.ni) wave_put_bits(w.fbits + 1, acc.l, acc.v0, a.out_leaf_validity);
#endif
  wave_sync();
  const uint32_t nw = (max(acc.r, acc.l) + 31) / 32 + 2;
  for (uint32_t i = lane; i < nw; i += 64) w.lbits[i] = w.fbits[i] = 0;
  wave_sync();
  acc.g0 += acc.r;
  acc.v0 += acc.l;
  acc.r = acc.l = 0;
}

// One step of kLvStep levels [t0, t0 + kLvStep) of a page, one wave, rows
// and leaves before it = (carry_r, carry_l).  *step_r / *step_l: the step's
// row starts and leaves (all levels); the return value: leaves consumed
// (levels whose inclusive row count stays <= rows, read_basic.rs:158-162).
// WRITE: offsets and bitmaps at (rbase, lbase).
// (m: this lane's masks of levels t0 + 32 lane ..; rows: the page's rows.)
template <bool WRITE, class WV>
__device__ uint32_t lv_step_m(const LvMasks m, WV& w, uint32_t rows, const ListArgs& a, uint32_t t0, uint64_t rbase,
                              uint64_t lbase, uint32_t carry_r, uint32_t carry_l, uint32_t* step_r, uint32_t* step_l,
                              LvAcc& acc) {
  const uint32_t lane = threadIdx.x & 63;
  if (t0 == 0 && lane == 0 && !(m.rsm & 1)) put_err(&w.err, ST_OUT_OF_SPEC);  // level 0 starts no row
  const uint32_t pk = ((uint32_t)__popc(m.rsm) << 16) | (uint32_t)__popc(m.lfm);
  const uint32_t incl = wave_incl_scan(pk), tot = __builtin_amdgcn_readlane(incl, 63), ex = incl - pk;
  const uint32_t rb = carry_r + (ex >> 16), lb = carry_l + (ex & 0xFFFFu);
  uint32_t cm = m.vm;
  if (rb + __popc(m.rsm) > rows) {
    if (rb >= rows + 1) cm = 0;
    else {  // cut at the (rows - rb + 1)-th row start
      uint32_t x = m.rsm;
      for (uint32_t k = rows - rb; k; k--) x &= x - 1;
      cm = (x & (0u - x)) - 1;
    }
  }
  const uint32_t rsm = m.rsm & cm, lfm = m.lfm & cm;
  if constexpr (WRITE) {
    const uint32_t s_r0 = carry_r, s_l0 = carry_l;
    const uint64_t g0 = rbase + s_r0, v0 = lbase + s_l0;
    const uint32_t al = a.ow == 4 ? (uint32_t)(g0 & 3) : (uint32_t)(g0 & 1);  // obuf index of row 0
    if (acc.r + (tot >> 16) > kLvAccBits || acc.l + (tot & 0xFFFFu) > kLvAccBits) lv_flush(w, a, acc);
    const uint32_t pr = acc.r + rb - s_r0, pf = acc.l + lb - s_l0;
    const uint32_t nr = __popc(rsm), nf = __popc(lfm);
    uint16_t* ob = w.obuf + al + (rb - s_r0);
    const uint32_t lrel = lb - s_l0;
    uint32_t j = 0;
#ifndef SB_V_LV_NOOB
    for (uint32_t x = rsm; x; x &= x - 1, j++) ob[j] = (uint16_t)(lrel + __popc(m.lfm & ((x & (0u - x)) - 1)));
#endif
    if (a.nl) lds_or_bits(w.lbits + 1, pr, compress32(m.lvm, rsm), nr);
    if (a.ni) lds_or_bits(w.fbits + 1, pf, compress32(m.fvm, lfm), nf);
    const uint32_t cpk = (nr << 16) | nf;
    const uint32_t ctot = __builtin_amdgcn_readlane(wave_incl_scan(cpk), 63);
    const uint32_t tr = ctot >> 16, tl = ctot & 0xFFFFu;
    wave_sync();
#ifdef SB_V_LV_NOOFF
    constexpr bool wr_off = false;
#else
    constexpr bool wr_off = true;
#endif
    if (!wr_off) {
    } else if (a.ow == 4) {  // quads of rows on 16-byte boundaries: obuf[4q .. 4q + 3] -> o[4q - al ..]
      uint32_t* o = (uint32_t*)a.out_offsets + (g0 - al);
      const uint32_t v32 = (uint32_t)v0, nq = (al + tr + 3) >> 2;
      for (uint32_t q = lane; q < nq; q += 64) {
        const uint32_t* pr = (const uint32_t*)(w.obuf + 4 * q);
        const uint32_t px = pr[0], py = pr[1];
        const uint32_t e0 = v32 + (px & 0xFFFFu), e1 = v32 + (px >> 16), e2 = v32 + (py & 0xFFFFu), e3 = v32 + (py >> 16);
        const uint32_t j0 = 4 * q;
        if (j0 >= al && j0 + 4 <= al + tr) {
          st_out((u32x4*)(o + j0), u32x4{e0, e1, e2, e3});
        } else {
          const uint32_t e[4] = {e0, e1, e2, e3};
#pragma unroll
          for (uint32_t k = 0; k < 4; k++)
            if (j0 + k >= al && j0 + k < al + tr) o[j0 + k] = e[k];
        }
      }
    } else {
      uint64_t* o = (uint64_t*)a.out_offsets + (g0 - al);
      const uint32_t nq = (al + tr + 1) >> 1;
      for (uint32_t q = lane; q < nq; q += 64) {
        const uint32_t j0 = 2 * q;
        const uint64_t x0 = v0 + w.obuf[j0], x1 = v0 + w.obuf[j0 + 1];
        if (j0 >= al && j0 + 2 <= al + tr) {
          st_out((u32x4*)(o + j0), u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)});
        } else {
          if (j0 >= al && j0 < al + tr) o[j0] = x0;
          if (j0 + 1 >= al && j0 + 1 < al + tr) o[j0 + 1] = x1;
        }
      }
    }
    acc.r += tr;
    acc.l += tl;
    wave_sync();
  }
  *step_r = tot >> 16;
  *step_l = tot & 0xFFFFu;
  return __builtin_amdgcn_readlane(wave_incl_scan(__popc(lfm)), 63);  // DPP, not a permute chain
}

template <bool WRITE, class Src>
__device__ __forceinline__ uint32_t lv_step(const Src& s, ListWave& w, const ListShared& ls, const ListArgs& a,
                                            uint32_t t0, uint32_t L, uint64_t rbase, uint64_t lbase, uint32_t carry_r,
                                            uint32_t carry_l, uint32_t* step_r, uint32_t* step_l, LvAcc& acc) {
  const LvMasks m = level_masks(s, ls, t0 + (threadIdx.x & 63) * kLvK, L, a.nl + 1);
  return lv_step_m<WRITE>(m, w, ls.rows, a, t0, rbase, lbase, carry_r, carry_l, step_r, step_l, acc);
}

// One wave walks its page's levels a step at a time (the sizing pass).
template <bool WRITE, class Src>
__device__ void wave_levels(const Src& s, ListWave& w, const ListArgs& a, uint32_t L, uint64_t rbase, uint64_t lbase,
                            uint32_t* rows_c, uint32_t* leaves_c) {
  const uint32_t lane = threadIdx.x & 63, rows = w.ls.rows;
  uint32_t carry_r = 0, carry_l = 0, leaves = 0;
  LvAcc acc{0, 0, rbase, lbase};
  if constexpr (WRITE) {
    for (uint32_t i = lane; i < kLvBitsW; i += 64) w.lbits[i] = w.fbits[i] = 0;
    wave_sync();
  }
  for (uint32_t t0 = 0; t0 < L; t0 += kLvStep) {
    uint32_t sr, sl;
    leaves += lv_step<WRITE>(s, w, w.ls, a, t0, L, rbase, lbase, carry_r, carry_l, &sr, &sl, acc);
    carry_r += sr;
    carry_l += sl;
    if (carry_r > rows) break;  // uniform: every later level is past the last row
  }
  if constexpr (WRITE) lv_flush(w, a, acc);
  const uint32_t rc = min(carry_r, rows);
  if (lane == 0 && rc != rows) put_err(&w.err, ST_OUT_OF_SPEC);  // levels ended before `rows` rows
  *rows_c = rc;
  *leaves_c = leaves;
}

// Row starts and leaves of the step at t0 (all its levels), one wave.
template <class Src>
__device__ __forceinline__ uint32_t lv_count(const Src& s, const ListShared& ls, uint32_t t0, uint32_t L, uint32_t cs1) {
  const LvMasks m = level_masks(s, ls, t0 + (threadIdx.x & 63) * kLvK, L, cs1);
  const uint32_t pk = ((uint32_t)__popc(m.rsm) << 16) | (uint32_t)__popc(m.lfm);
  return __builtin_amdgcn_readlane(wave_incl_scan(pk), 63);  // rows < 2^16 per 2048-level step
}

// Per page setup of one wave: the page's first kLvStage bytes staged in LDS
// in one round of loads (the header and, for the writer's pages, both level
// streams), then the header parse -- or, on the levels pass of a fast page,
// the descriptor the sizing pass left.  *staged: the level streams lie in
// the staged prefix.  Returns false on a parse error.
__device__ bool wave_page_setup(ListWave& w, uint32_t* stage, const ListArgs& a, uint32_t page, const PageDesc& pd, bool reuse,
                                bool* staged, uint32_t* mis_out, uint32_t* lim_out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint8_t* pg = a.chunk + pd.byte_off;
  const uintptr_t a0 = (uintptr_t)pg & ~(uintptr_t)3;
  const uint32_t mis = (uint32_t)((uintptr_t)pg & 3);
  const uint32_t lim = stage ? min(pd.byte_len, kLvStage) : 0u;
  const uint32_t ndw = (mis + lim + 3) >> 2;
  uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
  if (reuse) {
    d0 = a.lvdesc[2 * page];
    d1 = a.lvdesc[2 * page + 1];
  }
  if (stage) {  // every load issued before the first LDS store (one round trip, not one per 64 dwords)
    typedef const __attribute__((address_space(1))) uint32_t g32;
    constexpr uint32_t kIt = (kLvStage / 4 + 2 + 63) / 64;
    uint32_t v[kIt];
#pragma unroll
    for (uint32_t k = 0; k < kIt; k++) {
      const uint32_t d = lane + 64 * k;
      v[k] = d < ndw ? __builtin_nontemporal_load((g32*)a0 + d) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kIt; k++)
      if (lane + 64 * k < ndw) stage[lane + 64 * k] = v[k];
  }
  if (lane == 0) w.err = 0;
  wave_sync();
  *mis_out = mis;
  *lim_out = lim;
  if (reuse && (d0.w & 1)) {  // fast page: one bit-packed run per stream
    if (lane == 0) {
      w.ls.rows = d0.x;
      w.ls.vpos = d0.y;
      w.ls.region = d0.y;
      w.ls.bw_def = d0.w >> 1;
      w.ls.fast = 1;
      w.ls.rep.n = w.ls.def.n = 1;
      w.ls.rep.start[0] = w.ls.def.start[0] = 0;
      w.ls.rep.arg[0] = 0x80000000u | d0.z;
      w.ls.def.arg[0] = 0x80000000u | d1.x;
    }
  } else if (lane == 0) {
    const StageSrc ss{LdsSrc{stage, mis}, GlbSrc{pg}, lim};
    list_parse(ss, &w.err, w.ls, pd, a);
  }
  wave_sync();
  if (w.err) return false;
  *staged = w.ls.region <= lim;
  return true;
}

// Exact sizing pass: one wave per page (4 per workgroup) walks the levels:
// consumed rows / leaves, and the parse results for the levels pass.
__global__ __launch_bounds__(NT) void k_list_size(ListArgs a) {
  __shared__ ListWave waves[NW];
  __shared__ uint32_t stages[NW][kLvStage / 4 + SB_LV_STAGE_PAD];  // the page's first bytes at byte `mis` (+ pad)
  const uint32_t lane = threadIdx.x & 63;
  ListWave& w = waves[threadIdx.x >> 6];
  uint32_t* stage = stages[threadIdx.x >> 6];
  for (uint32_t page = blockIdx.x * NW + (threadIdx.x >> 6); page < a.n_pages; page += gridDim.x * NW) {
    const PageDesc pd = a.pages[page];
    bool staged = false;
    uint32_t mis = 0, lim = 0, rows_c = 0, leaves_c = 0;
    if (wave_page_setup(w, stage, a, page, pd, false, &staged, &mis, &lim)) {
      if (staged) wave_levels<false>(LdsSrc{stage, mis}, w, a, pd.num_values, 0, 0, &rows_c, &leaves_c);
      else wave_levels<false>(GlbSrc{a.chunk + pd.byte_off}, w, a, pd.num_values, 0, 0, &rows_c, &leaves_c);
    }
    wave_sync();
    if (lane == 0) {
      const bool ok = w.err == 0;
      a.counts[page] = ok ? (((uint64_t)rows_c << 32) | leaves_c) : 0;
      const uint32_t fast = ok && w.ls.fast;
      a.lvdesc[2 * page] = make_uint4(w.ls.rows, w.ls.vpos, w.ls.rep.arg[0] & 0x7FFFFFFFu, fast | (w.ls.bw_def << 1));
      a.lvdesc[2 * page + 1] = make_uint4(w.ls.def.arg[0] & 0x7FFFFFFFu, ok, 0, 0);
      a.status[page] = w.err;
    }
    wave_sync();
  }
}

// Block bases: one workgroup per NT pages, one thread per page.  a.peek:
// the page's counts come straight from its headers -- rows from the nested
// header (read_basic.rs:71, `additional`), leaves from the values stream's
// usize = leaves * width (integer/mod.rs:62-63) -- two small reads per page
// instead of a walk over its levels; the plan only takes this path after
// checking it against the exact pass page by page.  Otherwise the counts of
// k_list_size.  Writes each page's bases within its block and the block totals.
__global__ __launch_bounds__(NT) void k_list_bscan(ListArgs a) {
  __shared__ Shared sh;
  const uint32_t p = blockIdx.x * NT + threadIdx.x;
  uint64_t c = 0;
  if (p < a.n_pages) {
    if (a.peek) {
      const PageDesc pd = a.pages[p];
      const GlbSrc g{a.chunk + pd.byte_off};
      if (pd.byte_len >= 12) {
        const uint64_t vpos = 12ull + g.u32(4) + g.u32(8);
        if (vpos + 9 <= pd.byte_len) c = ((uint64_t)g.u32(0) << 32) | (g.u32((uint32_t)vpos + 5) / a.width);
      }
      a.counts[p] = c;
    } else {
      c = a.counts[p];
    }
  }
  uint64_t tr, tl;
  const uint64_t er = block_excl_scan<uint64_t>(c >> 32, sh, &tr);
  const uint64_t el = block_excl_scan<uint64_t>(c & 0xFFFFFFFFull, sh, &tl);
  if (p < a.n_pages) {
    a.local[2 * p] = er;
    a.local[2 * p + 1] = el;
  }
  if (threadIdx.x == 0) {
    a.blk[2 * blockIdx.x] = tr;
    a.blk[2 * blockIdx.x + 1] = tl;
  }
}

// A decode's sizing in one launch: page counts (from the headers with
// a.peek, else the exact pass's), block scans and global bases, and each
// page's values-stream descriptor (a.peek), so the values decode needs
// nothing from k_list_levels.  Block b < nblk scans its NT pages' counts, publishes its
// row / leaf totals as two words of blk tagged with a.epoch (top 16 bits),
// and sums the totals of blocks 0..b-1 -- every predecessor's own total, no
// inclusive prefixes, so no block waits on another's wait: the lower blocks
// were dispatched first (workgroups launch in order on each XCD), each
// publishes as soon as its scan is done.  A stale word (an earlier decode's
// tag, or the plan's zeroed state) reads as not yet published.  The bitmaps
// need no zeroing (k_list_levels clears and sets only the bits it owns), but
// for the bits past the column's last row / leaf: the last page's thread
// zeroes the final word of each bitmap before k_list_levels runs.
__global__ __launch_bounds__(NT) void k_list_bases(ListArgs a) {
  __shared__ Shared sh;
  __shared__ uint64_t red[2][NW];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t p = blockIdx.x * NT + tid;
  uint64_t c = 0;
  uint64_t vpos = ~0ull;
  PageDesc pd{};
  if (p < a.n_pages) {
    if (a.peek) {
      pd = a.pages[p];
      const GlbSrc g{a.chunk + pd.byte_off};
      if (pd.byte_len >= 12) {
        vpos = 12ull + g.u32(4) + g.u32(8);
        if (vpos + 9 <= pd.byte_len) c = ((uint64_t)g.u32(0) << 32) | (g.u32((uint32_t)vpos + 5) / a.width);
      }
      a.counts[p] = c;
    } else {
      c = a.counts[p];
    }
  }
  uint64_t tr, tl;
  const uint64_t er = block_excl_scan<uint64_t>(c >> 32, sh, &tr);
  const uint64_t el = block_excl_scan<uint64_t>(c & 0xFFFFFFFFull, sh, &tl);
  constexpr uint64_t kVal = (1ull << 48) - 1;
  const uint64_t tag = (uint64_t)a.epoch << 48;
  if (tid == 0) {
    __hip_atomic_store(&a.blk[2 * blockIdx.x], tag | tr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.blk[2 * blockIdx.x + 1], tag | tl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (wv == 0) {  // the totals of blocks 0..b-1, 64 blocks a probe
    uint64_t br = 0, bl = 0;
    for (uint32_t b0 = 0; b0 < blockIdx.x; b0 += 64) {
      const uint32_t b = b0 + lane;
      const bool need = b < blockIdx.x;
      uint64_t r = 0, l = 0;
      for (;;) {
        if (need) {
          r = __hip_atomic_load(&a.blk[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          l = __hip_atomic_load(&a.blk[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!__ballot(need && ((r & ~kVal) != tag || (l & ~kVal) != tag))) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (need) {
        br += r & kVal;
        bl += l & kVal;
      }
    }
    br = wave_sum64(br);
    bl = wave_sum64(bl);
    if (lane == 0) {
      red[0][0] = br;
      red[1][0] = bl;
    }
  }
  __syncthreads();
  if (p < a.n_pages) {
    const uint64_t rbase = red[0][0] + er, lbase = red[1][0] + el;
    a.local[2 * p] = rbase;
    a.local[2 * p + 1] = lbase;
    if (p == a.n_pages - 1) {
      const uint64_t tr_all = rbase + (c >> 32), tl_all = lbase + (c & 0xFFFFFFFFull);
      if (a.nl && a.out_list_validity && (tr_all & 31)) a.out_list_validity[tr_all >> 5] = 0;
      if (a.ni && a.out_leaf_validity && (tl_all & 31)) a.out_leaf_validity[tl_all >> 5] = 0;
    }
    if (a.peek) {
      const bool ok = vpos + 9 <= pd.byte_len;
      a.vpages[p] = PageDesc{pd.byte_off + (ok ? vpos : 0), lbase, ok ? pd.byte_len - (uint32_t)vpos : 0,
                             ok ? (uint32_t)c : 0, a.vpages[p].reserved};
    }
  }
}

// Levels pass: one wave per page, at the global bases k_list_bases wrote.
// Writes offsets and both bitmaps, its status, and (unless the values
// descriptors came from the headers) the page's values-stream descriptor;
// the last page also the totals and the final offset.
__global__ __launch_bounds__(NT) void k_list_levels(ListArgs a) {
  __shared__ ListWave waves[NW];
  __shared__ uint32_t stages[NW][kLvStage / 4 + SB_LV_STAGE_PAD];  // the page's first bytes at byte `mis` (+ pad)
  const uint32_t lane = threadIdx.x & 63;
  ListWave& w = waves[threadIdx.x >> 6];
  uint32_t* stage = stages[threadIdx.x >> 6];
  for (uint32_t page = blockIdx.x * NW + (threadIdx.x >> 6); page < a.n_pages; page += gridDim.x * NW) {
    const PageDesc pd = a.pages[page];
    const uint64_t rbase = a.local[2 * page], lbase = a.local[2 * page + 1];
    const uint64_t cnt = a.counts[page];
    bool staged = false;
    uint32_t mis = 0, lim = 0, rows_c = 0, leaves_c = 0;
    const bool sized = a.lvdesc[2 * page + 1].y != 0;  // the exact pass parsed this page
    if (sized && wave_page_setup(w, stage, a, page, pd, true, &staged, &mis, &lim)) {
      if (staged) wave_levels<true>(LdsSrc{stage, mis}, w, a, pd.num_values, rbase, lbase, &rows_c, &leaves_c);
      else wave_levels<true>(GlbSrc{a.chunk + pd.byte_off}, w, a, pd.num_values, rbase, lbase, &rows_c, &leaves_c);
    } else if (lane == 0) {
      w.err = 0;
      if (!sized) {  // re-parse for the status the reference would give
        const StageSrc ss{LdsSrc{nullptr, 0}, GlbSrc{a.chunk + pd.byte_off}, 0};
        list_parse(ss, &w.err, w.ls, pd, a);
        if (!w.err) w.err = ST_OUT_OF_SPEC;
      }
    }
    wave_sync();
    if (lane == 0) {
      uint32_t err = w.err;
      if (!err && (rows_c != (uint32_t)(cnt >> 32) || leaves_c != (uint32_t)cnt)) err = ST_OUT_OF_SPEC;
      const bool ok = err == 0;
      // the page's values stream, decoded as a flat non-nullable page of `leaves` values
      if (!a.peek)
        a.vpages[page] = PageDesc{pd.byte_off + (ok ? w.ls.vpos : 0), lbase, ok ? pd.byte_len - w.ls.vpos : 0,
                                  ok ? leaves_c : 0, a.vpages[page].reserved};
      a.status[page] = err;
      if (page == a.n_pages - 1) {
        const uint64_t tr = rbase + (cnt >> 32), tl = lbase + (uint32_t)cnt;
        a.totals[0] = tr;
        a.totals[1] = tl;
        if (a.out_offsets) bin_put_off(a.out_offsets, tr, tl, a.ow);  // create_list appends values.len()
      }
    }
    wave_sync();
  }
}

// ===========================================================================
// General nesting: a leaf under `depth` nests (List / Map / Struct chains,
// the InitNested chain of read/deserialize.rs:140-233),
// read_validity_nested (read/read_basic.rs:95-164) level by level: nests
// 0..depth-1 are lists (repeated; nullable per level) or, where bit d of
// struct_mask is set, structs (not repeated; arrow2's NestedStruct /
// NestedStructValid are "required"), nest `depth` the primitive; cum_sum /
// cum_rep over (nullable + repeated) / repeated; a nest is pushed when
// rep <= cum_rep[d] && def >= cum_sum[d], or when the nest above is a struct
// that was pushed and is not valid (the is_required chain, :118-137: every
// child of a null struct gets a slot).  One wave per page, one level per
// lane per step: each lane runs the chain over its level, ballots give each
// nest's pushes and ranks; a list push's offset is its child's running
// count; validity bits are compacted to push order and OR-ed into the
// (zeroed) bitmaps.  A zero-width level stream (max level 0: a chain of
// required structs writes none) reads as all zeros, as parquet2's
// HybridRleDecoder does with num_bits 0.
// ===========================================================================
struct NestArgs {
  const uint8_t* chunk;
  const PageDesc* pages;
  uint32_t n_pages, depth, nullable, ow, smask;
  uint64_t* counts;
  const uint64_t* bases;
  const uint64_t* totals;
  PageDesc* vpages;
  uint8_t* out_offsets[kMaxNest];
  uint32_t* out_validity[kMaxNest];
  uint32_t* out_leaf_validity;
  uint32_t* status;
  uint32_t* vpos;
};

// A window of hybrid runs (parquet2 HybridRleDecoder) over the levels of the
// current 64-level step, parsed incrementally by one lane: the run holding
// the step's first level plus every run up to the step's end (each run
// covers >= 1 level, so <= 65 entries), so a stream may hold any number of
// runs (pyarrow's writer mixes many RLE and bit-packed runs).
struct RunWin {
  uint32_t n, p, end, covered, bw;
  uint32_t start[68];
  uint32_t arg[68];  // bit-packed: 0x80000000 | payload position; RLE: the value
};

// lane 0: make the window cover levels [l0, lend)
__device__ bool runwin_advance(const GlbSrc& s, RunWin& R, uint32_t l0, uint32_t lend, uint32_t* err) {
  if (R.bw == 0) {  // no stream: one RLE run of zeros over every level
    R.n = 1;
    R.start[0] = 0;
    R.arg[0] = 0;
    R.covered = 0xFFFFFFFFu;
    R.start[1] = R.covered;
    return true;
  }
  uint32_t k = R.n;
  while (k > 0 && R.start[k - 1] > l0) k--;
  if (k > 1) {  // keep the run holding l0
    for (uint32_t i = k - 1; i < R.n; i++) {
      R.start[i - (k - 1)] = R.start[i];
      R.arg[i - (k - 1)] = R.arg[i];
    }
    R.n -= k - 1;
  }
  while (R.covered < lend) {
    if (R.n >= 66) { put_err(err, ST_NYI); return false; }
    uint32_t h = 0, sft = 0;
    for (;;) {  // ULEB128 header
      if (R.p >= R.end || sft > 28) { put_err(err, ST_OUT_OF_SPEC); return false; }
      const uint32_t c = s.u8(R.p++);
      h |= (c & 0x7Fu) << sft;
      if (!(c & 0x80)) break;
      sft += 7;
    }
    uint32_t cnt, arg;
    if (h & 1) {  // bit-packed: h >> 1 groups of 8, clamped to the bytes present
      const uint64_t want = (uint64_t)(h >> 1) * R.bw;
      const uint32_t have = (uint32_t)min<uint64_t>(want, R.end - R.p);
      cnt = (uint32_t)min<uint64_t>((uint64_t)(h >> 1) * 8, (uint64_t)have * 8 / max(R.bw, 1u));
      arg = 0x80000000u | R.p;
      R.p += have;
    } else {  // RLE: h >> 1 repeats of a ceil(bw / 8)-byte value
      const uint32_t vb = (R.bw + 7) / 8;
      if (R.p + vb > R.end) { put_err(err, ST_OUT_OF_SPEC); return false; }
      arg = 0;
      for (uint32_t b = 0; b < vb; b++) arg |= s.u8(R.p + b) << (8 * b);
      R.p += vb;
      cnt = h >> 1;
    }
    if (cnt == 0) continue;  // an empty run yields no levels
    R.start[R.n] = R.covered;
    R.arg[R.n] = arg;
    R.n++;
    R.covered += cnt;
  }
  R.start[R.n] = R.covered;
  return true;
}

__device__ __forceinline__ uint32_t runwin_at(const GlbSrc& s, const RunWin& R, uint32_t i) {
  uint32_t lo = 0, hi = R.n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (R.start[mid] <= i) lo = mid; else hi = mid;
  }
  const uint32_t a = R.arg[lo];
  if (!(a & 0x80000000u)) return a;
  const uint32_t bit = (i - R.start[lo]) * R.bw;
  return (s.u32((a & 0x7FFFFFFFu) + (bit >> 3)) >> (bit & 7)) & ((1u << R.bw) - 1);
}

struct NestWave {
  RunWin rep, def;
  uint32_t err, rows, vpos;
};

__device__ __forceinline__ uint64_t compress64(uint64_t v, uint64_t m) {
  const uint32_t lo = compress32((uint32_t)v, (uint32_t)m), hi = compress32((uint32_t)(v >> 32), (uint32_t)(m >> 32));
  return (uint64_t)lo | ((uint64_t)hi << __popc((uint32_t)m));
}

// n (<= 64) bits at bit position pos of a zeroed bitmap, OR-ed (lanes 0..2)
__device__ __forceinline__ void put_bits64(uint32_t* bm, uint64_t pos, uint64_t v, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63;
  if (!n || !v || lane > 2) return;
  const uint32_t sh = (uint32_t)(pos & 31);
  const uint64_t w0 = pos >> 5;
  const uint32_t word = lane == 0 ? (uint32_t)(v << sh)
                      : lane == 1 ? (uint32_t)(sh ? (v >> (32 - sh)) : (v >> 32))
                                  : (uint32_t)(sh ? (v >> (64 - sh)) : 0u);
  if (word) atomicOr(&bm[w0 + lane], word);
}

template <bool WRITE>
__global__ __launch_bounds__(NT) void k_nest_walk(NestArgs a) {
  __shared__ NestWave waves[NW];
  const uint32_t lane = threadIdx.x & 63, D = a.depth;
  NestWave& w = waves[threadIdx.x >> 6];
  uint32_t cum_sum[kMaxNest + 2], cum_rep[kMaxNest + 2];
  cum_sum[0] = cum_rep[0] = 0;
  for (uint32_t d = 0; d <= D; d++) {
    const uint32_t nl = (a.nullable >> d) & 1, rp = (d < D && !((a.smask >> d) & 1)) ? 1u : 0u;
    cum_sum[d + 1] = cum_sum[d] + nl + rp;
    cum_rep[d + 1] = cum_rep[d] + rp;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (uint32_t page = blockIdx.x * NW + (threadIdx.x >> 6); page < a.n_pages; page += gridDim.x * NW) {
    const PageDesc pd = a.pages[page];
    const GlbSrc s{a.chunk + pd.byte_off};
    const uint32_t L = pd.num_values;
    if (lane == 0) {
      w.err = 0;
      const uint32_t len = pd.byte_len;
      if (len < 12) {
        w.err = ST_IO;
      } else {
        const uint32_t rows = s.u32(0), rl = s.u32(4), dl = s.u32(8);
        if ((uint64_t)12 + rl + dl > len) {
          w.err = ST_IO;
        } else {
          w.rows = rows;
          w.vpos = 12 + rl + dl;
          w.rep = RunWin{0, 12, 12 + rl, 0, 32u - __clz(cum_rep[D + 1])};
          w.def = RunWin{0, 12 + rl, 12 + rl + dl, 0, 32u - __clz(cum_sum[D + 1])};
          if (L > 0 && rows == 0) w.err = ST_OUT_OF_SPEC;
        }
      }
    }
    wave_sync();
    uint64_t carry[kMaxNest + 1] = {0, 0, 0, 0, 0}, base[kMaxNest + 1] = {0, 0, 0, 0, 0};
    if (WRITE)
      for (uint32_t d = 0; d <= D; d++) base[d] = a.bases[(uint64_t)page * (D + 1) + d];
    uint32_t rows_seen = 0;
    const uint32_t rows = w.rows;
    if (!w.err) {
      for (uint32_t l0 = 0; l0 < L; l0 += 64) {
        if (lane == 0 && runwin_advance(s, w.rep, l0, min(l0 + 64, L), &w.err))
          runwin_advance(s, w.def, l0, min(l0 + 64, L), &w.err);
        wave_sync();
        if (w.err) break;
        const uint32_t l = l0 + lane;
        const bool in = l < L;
        const uint32_t r = in ? runwin_at(s, w.rep, l) : 0u, dv = in ? runwin_at(s, w.def, l) : 0u;
        if (l == 0 && r != 0) w.err = ST_OUT_OF_SPEC;  // the first level starts no row
        const uint64_t rs = __ballot(in && r == 0);
        // consumed: inclusive row count <= rows (read_basic.rs:150-162)
        const bool cons = in && rows_seen + (uint32_t)__popcll(rs & (below | (1ull << lane))) <= rows;
        uint64_t push[kMaxNest + 1];
        bool forced = false;  // the is_required chain: the nest above is a struct pushed invalid
        for (uint32_t d = 0; d <= D; d++) {
          const bool me = cons && (forced || (r <= cum_rep[d] && dv >= cum_sum[d]));
          push[d] = __ballot(me);
          forced = me && ((a.smask >> d) & 1) && !(((a.nullable >> d) & 1) && dv > cum_sum[d]);
        }
        if (WRITE) {
          for (uint32_t d = 0; d <= D; d++) {
            const bool me = (push[d] >> lane) & 1;
            const uint64_t pos = base[d] + carry[d] + (uint32_t)__popcll(push[d] & below);
            if (d < D && me && !((a.smask >> d) & 1)) {  // list offset = the child's count before this level
              const uint64_t v = base[d + 1] + carry[d + 1] + (uint32_t)__popcll(push[d + 1] & below);
              bin_put_off(a.out_offsets[d], pos, v, (int)a.ow);
            }
            if ((a.nullable >> d) & 1) {
              const uint64_t vm = __ballot(me && dv > cum_sum[d]);
              const uint32_t np = (uint32_t)__popcll(push[d]);
              uint32_t* bm = d < D ? a.out_validity[d] : a.out_leaf_validity;
              put_bits64(bm, base[d] + carry[d], compress64(vm, push[d]), np);
            }
            (void)pos;
          }
        }
        for (uint32_t d = 0; d <= D; d++) carry[d] += (uint32_t)__popcll(push[d]);
        rows_seen += (uint32_t)__popcll(rs);
        if (rows_seen > rows) break;  // every later level is past the last row
      }
      if (lane == 0 && min(rows_seen, rows) != rows) w.err = ST_OUT_OF_SPEC;  // levels ended early
    }
    wave_sync();
    if (lane == 0) {
      uint32_t err = w.err;
      if (!WRITE) {
        for (uint32_t d = 0; d <= D; d++) a.counts[(uint64_t)page * (D + 1) + d] = err ? 0 : carry[d];
        a.vpos[page] = err ? 0u : w.vpos;
      } else {
        for (uint32_t d = 0; d <= D; d++)
          if (!err && carry[d] != a.counts[(uint64_t)page * (D + 1) + d]) err = ST_OUT_OF_SPEC;
        const bool ok = err == 0;
        a.vpages[page] = PageDesc{pd.byte_off + (ok ? w.vpos : 0), base[D], ok ? pd.byte_len - w.vpos : 0,
                                  ok ? (uint32_t)carry[D] : 0u, a.vpages[page].reserved};
        if (page == a.n_pages - 1)  // create_list / create_map append each child's length
          for (uint32_t d = 0; d < D; d++)
            if (!((a.smask >> d) & 1)) bin_put_off(a.out_offsets[d], a.totals[d], a.totals[d + 1], (int)a.ow);
      }
      a.status[page] = err;
    }
    wave_sync();
  }
}

}  // namespace sbk

namespace sb {
int launch_fix_light(const LaunchArgs& a, uint32_t n_pages, int width, bool is_float, uint32_t* light, void* stream) {
  if (!n_pages) return 0;
  hipLaunchKernelGGL(sbk::k_fix_light, dim3((n_pages + sbk::NT - 1) / sbk::NT), dim3(sbk::NT), 0, (hipStream_t)stream,
                     a, n_pages, (uint32_t)width, (uint32_t)is_float, light);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_fix_probe(const uint8_t* chunk, const PageDesc* pages, const uint32_t* list, uint32_t n, int width,
                     int nullable, uint32_t* probe, void* stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(sbk::k_fix_probe, dim3((n + sbk::NT - 1) / sbk::NT), dim3(sbk::NT), 0, (hipStream_t)stream, chunk,
                     pages, list, n, (uint32_t)width, nullable, probe);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_zstd_scan(const uint8_t* chunk, const PageDesc* pages, uint32_t n, int width, int nullable, uint32_t* flag,
                     void* stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(sbk::k_zstd_scan, dim3((n + sbk::NT - 1) / sbk::NT), dim3(sbk::NT), 0, (hipStream_t)stream, chunk,
                     pages, n, (uint32_t)width, nullable, flag);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_decode_fixed(int width, bool is_float, int kind, const LaunchArgs& a, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (is_float) {
    if (width == 4) return sbk::launch<4, true>(kind, a, s);
    if (width == 8) return sbk::launch<8, true>(kind, a, s);
    return -2;
  }
  switch (width) {
    case 1: return sbk::launch<1, false>(kind, a, s);
    case 2: return sbk::launch<2, false>(kind, a, s);
    case 4: return sbk::launch<4, false>(kind, a, s);
    case 8: return sbk::launch<8, false>(kind, a, s);
  }
  return -2;
}
}  // namespace sb

namespace sb {
int launch_binary(int stage, int offset_width, const BinLaunch& L, void* stream) {
  const uint32_t lds = L.lds_bytes ? std::min(L.lds_bytes, kDeferredLds) : kDeferredLds;
  sbk::BinArgs a{L.chunk, L.pages, L.n_pages, L.nullable, L.sizes, L.bases, L.total, L.out_offsets, L.out_values,
                 L.values_cap, L.out_validity, L.status, lds, L.jobs, L.job_count, L.scratch, L.lds_need, L.cls,
                 L.region, L.rneed, L.lb, L.checked};
  hipStream_t st = (hipStream_t)stream;
  const dim3 block(sbk::NT);
  // staged passes: one workgroup per listed page (grid-stride), as many
  // resident per CU as the LDS budget allows; header-only pages: one thread
  // each to classify, one workgroup each to write offsets and validity; big
  // pages: one workgroup each (grid-stride) with their tables in HBM
  const dim3 grid(std::max<uint32_t>(1, L.staged_grid));
  const dim3 cgrid((L.n_pages + sbk::NT - 1) / sbk::NT);
  const dim3 lgrid(std::min<uint32_t>(L.n_pages, 65535u));
  const dim3 bgrid(std::max<uint32_t>(1, std::min<uint32_t>(L.n_big, 1024u)));
  ensure_lds_attr(sbk::k_bin_size<4, true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_size<8, true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_decode<4, true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_decode<8, true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_fused<4, true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_fused<8, true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_size<4, false>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_size<8, false>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_decode<4, false>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_decode<8, false>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_fused<4, false>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bin_fused<8, false>, (int)kDeferredLds);
  const bool z = L.zstd != 0;
  if (stage == 2) {  // plan time: per-page LDS / region needs
    if (offset_width == 8) hipLaunchKernelGGL(sbk::k_bin_probe<8>, cgrid, block, 0, st, a);
    else hipLaunchKernelGGL(sbk::k_bin_probe<4>, cgrid, block, 0, st, a);
  } else if (stage == 0) {
    if (hipMemsetAsync(L.cls + 4 * (size_t)L.n_pages, 0, 3 * sizeof(uint32_t), st) != hipSuccess) return -1;
    if (offset_width == 8) {
      hipLaunchKernelGGL(sbk::k_bin_light<8>, cgrid, block, 0, st, a);
      if (z) hipLaunchKernelGGL((sbk::k_bin_size<8, true>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((sbk::k_bin_size<8, false>), grid, block, lds, st, a);
      if (L.n_big) hipLaunchKernelGGL((sbk::k_bin_big<8, 0>), bgrid, block, sbk::kBigLds, st, a);
    } else {
      hipLaunchKernelGGL(sbk::k_bin_light<4>, cgrid, block, 0, st, a);
      if (z) hipLaunchKernelGGL((sbk::k_bin_size<4, true>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((sbk::k_bin_size<4, false>), grid, block, lds, st, a);
      if (L.n_big) hipLaunchKernelGGL((sbk::k_bin_big<4, 0>), bgrid, block, sbk::kBigLds, st, a);
    }
    hipLaunchKernelGGL(sbk::k_bin_scan, dim3(1), block, 0, st, a);
  } else if (stage == 3) {  // every page staged: size, base and decode in one pass
    if (hipMemsetAsync(L.lb, 0, (L.n_pages + 1) * sizeof(uint64_t), st) != hipSuccess) return -1;
    if (offset_width == 8) {
      if (z) hipLaunchKernelGGL((sbk::k_bin_fused<8, true>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((sbk::k_bin_fused<8, false>), grid, block, lds, st, a);
    } else {
      if (z) hipLaunchKernelGGL((sbk::k_bin_fused<4, true>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((sbk::k_bin_fused<4, false>), grid, block, lds, st, a);
    }
  } else {
    if (offset_width == 8) {
      if (z) hipLaunchKernelGGL((sbk::k_bin_decode<8, true>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((sbk::k_bin_decode<8, false>), grid, block, lds, st, a);
      if (L.n_big) hipLaunchKernelGGL((sbk::k_bin_big<8, 1>), bgrid, block, sbk::kBigLds, st, a);
      hipLaunchKernelGGL(sbk::k_bin_light_out<8>, lgrid, block, 0, st, a);
    } else {
      if (z) hipLaunchKernelGGL((sbk::k_bin_decode<4, true>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((sbk::k_bin_decode<4, false>), grid, block, lds, st, a);
      if (L.n_big) hipLaunchKernelGGL((sbk::k_bin_big<4, 1>), bgrid, block, sbk::kBigLds, st, a);
      hipLaunchKernelGGL(sbk::k_bin_light_out<4>, lgrid, block, 0, st, a);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_utf8_check(int offset_width, const Utf8Launch& a, void* stream) {
  if (a.n_rows == 0 || a.n_pages == 0) return 0;  // an empty array: nothing to check (try_check_utf8)
  hipStream_t st = (hipStream_t)stream;
  const uint64_t chunks = (a.len + 15) / 16;
  if (chunks && a.ascii) {  // page by page, skipping the pages k_inflate saw all ASCII
    const dim3 g(std::min<uint32_t>(a.n_pages, 65535u));
    if ((uintptr_t)a.values % 16) hipLaunchKernelGGL(sbk::k_utf8_pages<false>, g, dim3(sbk::NT), 0, st, a);
    else hipLaunchKernelGGL(sbk::k_utf8_pages<true>, g, dim3(sbk::NT), 0, st, a);
  } else if (chunks) {
    const dim3 g((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((chunks + sbk::NT - 1) / sbk::NT, 8192)));
    if ((uintptr_t)a.values % 16) hipLaunchKernelGGL(sbk::k_utf8_bytes<false>, g, dim3(sbk::NT), 0, st, a);
    else hipLaunchKernelGGL(sbk::k_utf8_bytes<true>, g, dim3(sbk::NT), 0, st, a);
  }
  const dim3 g((uint32_t)std::min<uint64_t>((a.n_rows + sbk::NT) / sbk::NT, 8192));
  if (offset_width == 8) hipLaunchKernelGGL(sbk::k_utf8_bounds<8>, g, dim3(sbk::NT), 0, st, a);
  else hipLaunchKernelGGL(sbk::k_utf8_bounds<4>, g, dim3(sbk::NT), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace sb

#ifdef SB_INF_PHASES
extern "C" int sb_debug_inf_phases(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sbk::sb_dbg_inf), 16 * 8) == hipSuccess ? 0 : -1;
}
extern "C" int sb_debug_inf_reset() {
  static const unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(sbk::sb_dbg_inf), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
#ifdef SB_BIN_PHASES
extern "C" int sb_debug_bin_phases(uint64_t* host, uint64_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sbk::sb_dbg_phase), std::min<uint64_t>(n, 4096 * 6) * 8) == hipSuccess ? 0 : -1;
}
#endif

namespace sb {
// Workgroups of k_inflate resident on the whole device at once (one query per device).
static uint32_t inflate_resident() {
  static std::mutex mu;
  static std::map<int, uint32_t> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)sbk::k_inflate, 64 * sbk::kInfWaves, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu <= 0 || cus <= 0)
    per_cu = 0;
  // (the API has reported 8 a CU for this kernel; its launch bounds allow SB_INF_BLOCKS)
  const uint32_t r = per_cu ? (uint32_t)(std::min(per_cu, SB_INF_BLOCKS) * cus) : kInflateGrid;
  cache[dev] = r;
  return r;
}
extern "C" uint32_t sb_debug_inflate_resident() { return inflate_resident(); }
int launch_inflate(const InflateLaunch& a, void* stream) {
  if (a.n_jobs == 0) return 0;
  if (a.patas_wg && launch_patas(a, stream))  // Patas leaf pages that fit a workgroup's LDS: k_patas first,
    return -1;                                // k_inflate skips them
  // A/B switches: SB_INF_STATIC=1 grid-strides the jobs, SB_INF_GRID=n caps the grid
  static const bool stat = getenv("SB_INF_STATIC") != nullptr;
  static const uint32_t gcap = getenv("SB_INF_GRID") ? (uint32_t)atoi(getenv("SB_INF_GRID")) : 0u;
  InflateLaunch b = a;
  if (stat) b.sched = nullptr;
  // claimed jobs: no more workgroups than fit at once (later ones would find none)
  uint32_t cap = b.sched ? std::min<uint32_t>(inflate_resident(), kInflateGrid) : kInflateGrid;
  if (gcap) cap = gcap;
  const uint32_t grid = std::min<uint32_t>((a.n_jobs + sbk::kInfWaves - 1) / sbk::kInfWaves, cap);
  hipLaunchKernelGGL(sbk::k_inflate, dim3(grid), dim3(64 * sbk::kInfWaves), 0, (hipStream_t)stream, b);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_zinflate(const InflateLaunch& a, void* stream) {
  if (a.n_jobs == 0) return 0;
  const uint32_t grid = std::min<uint32_t>(a.n_jobs, 1024u);
  hipLaunchKernelGGL(sbk::k_zinflate, dim3(grid), dim3(64), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace sb

namespace sb {
int launch_bool(const LaunchArgs& a, void* stream) {
  if (a.n_list == 0) return 0;
  ensure_lds_attr(sbk::k_bool_decode<true>, (int)kDeferredLds);
  ensure_lds_attr(sbk::k_bool_decode<false>, (int)kDeferredLds);
  const uint32_t grid = std::min<uint32_t>(a.n_list, 65535u);
  if (a.zstd) hipLaunchKernelGGL(sbk::k_bool_decode<true>, dim3(grid), dim3(sbk::NT), a.stage_bytes, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(sbk::k_bool_decode<false>, dim3(grid), dim3(sbk::NT), a.stage_bytes, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace sb

namespace sb {
int launch_list(int stage, const ListLaunch& L, void* stream) {
  sbk::ListArgs a{L.chunk, L.pages, L.n_pages, L.list_nullable, L.item_nullable, L.offset_width, L.width, L.peek,
                  L.counts, L.local, L.blk, L.totals, (uint4*)L.lvdesc, L.vpages, L.out_offsets, L.out_list_validity,
                  L.out_leaf_validity, L.status, L.epoch};
  if (L.n_pages == 0) return 0;
  const uint32_t grid = std::min<uint32_t>((L.n_pages + sbk::NW - 1) / sbk::NW, kListGrid);
  const uint32_t nblk = (L.n_pages + sbk::NT - 1) / sbk::NT;
  hipStream_t st = (hipStream_t)stream;
  if (stage == 0) {  // exact sizing
    hipLaunchKernelGGL(sbk::k_list_size, dim3(grid), dim3(sbk::NT), 0, st, a);
  } else if (stage == 1) {  // block bases (+ header sizing when peek)
    hipLaunchKernelGGL(sbk::k_list_bscan, dim3(nblk), dim3(sbk::NT), 0, st, a);
  } else if (stage == 4) {  // counts, global bases, values descriptors (peek)
    hipLaunchKernelGGL(sbk::k_list_bases, dim3(nblk), dim3(sbk::NT), 0, st, a);
  } else {
    hipLaunchKernelGGL(sbk::k_list_levels, dim3(grid), dim3(sbk::NT), 0, st, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace sb

namespace sb {
int launch_nest(int stage, const NestLaunch& L, void* stream) {
  if (L.n_pages == 0) return 0;
  sbk::NestArgs a{L.chunk, L.pages, L.n_pages, L.depth, L.nullable, L.offset_width, L.struct_mask, L.counts, L.bases, L.totals,
                  L.vpages, {}, {}, L.out_leaf_validity, L.status, L.vpos};
  for (int d = 0; d < kMaxNest; d++) {
    a.out_offsets[d] = L.out_offsets[d];
    a.out_validity[d] = L.out_validity[d];
  }
  const uint32_t grid = std::min<uint32_t>((L.n_pages + sbk::NW - 1) / sbk::NW, kListGrid);
  if (stage == 0) hipLaunchKernelGGL(sbk::k_nest_walk<false>, dim3(grid), dim3(sbk::NT), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(sbk::k_nest_walk<true>, dim3(grid), dim3(sbk::NT), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace sb
