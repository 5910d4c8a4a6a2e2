// sb_patas.hip -- Patas leaf pages decoded one workgroup a page on MI355X
// (gfx950): k_patas, launched ahead of k_inflate (InflateLaunch::patas_wg),
// which skips the pages it takes (patas_fits, sb_internal.h).
//   Patas records                             compression/double/patas.rs:107-132
// Integer/byte work only: no MFMA.  Bound: LDS (record walks, pointer
// jumping) with the stream read and the rows written once in HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sb_internal.h"

namespace sbk {

using namespace sb;

#ifndef SB_PAT_T
#define SB_PAT_T 512
#endif
#ifndef SB_PAT_SHFL
#define SB_PAT_SHFL 1
#endif
constexpr uint32_t kPatT = SB_PAT_T;  // threads of a k_patas workgroup (and the most segments)
static_assert(kPatMaxRows <= 16 * kPatT, "16 rows a thread");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef const __attribute__((address_space(1))) uint32_t gmem_u32;
template <int W> struct PT { using T = uint32_t; };
template <> struct PT<8> { using T = uint64_t; };

#ifdef SB_PAT_PHASES  // A/B instrumentation: shader cycles per phase, summed over workgroups (thread 0)
// [0] stage [1] segment walks [2] doubling + scan [3] record starts [4] terms [5] pointer jumping
// [6] store; counts: [8] pages [9] jumping rounds
__device__ unsigned long long sb_dbg_pat[16];
#define PAT_T(k)                                             \
  do {                                                       \
    __syncthreads();                                         \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();        \
    if (tid == 0) atomicAdd(&sb_dbg_pat[k], t_ - tph);       \
    tph = t_;                                                \
  } while (0)
#define PAT_N(k, v) \
  if (tid == 0) atomicAdd(&sb_dbg_pat[k], (unsigned long long)(v))
#else
#define PAT_T(k)
#define PAT_N(k, v)
#endif

// ---------------------------------------------------------------------------
// Patas leaf pages, one workgroup a page (k_patas): the same records as
// patas_wave (double/patas.rs:107-132) decoded by the whole workgroup.
//  1. Record starts.  The stream after the first value is cut into S <= 512
//     segments of B >= 16 bytes, one a thread.  A record is 2 + sig bytes
//     (<= 10), sized from its header alone, so the first record of a segment
//     starts at one of its first 10 bytes.  Each thread walks its segment
//     from all 10 of them in lockstep (the ten header reads of a step issued
//     together) and keeps, per entry offset, the records walked, the failing
//     record's code and the entry offset into the next segment.  The last
//     make the segment a map entry -> entry (ten nibbles, 15 = no entry: a
//     failing record before it); a block scan composing those maps gives
//     every segment its true entry, a second scan of the records gives each
//     record its row, and a last walk from the true entry writes each row's
//     record start.
//  2. Values.  Row i = (v << tz) ^ row[i - ref_diff]: every row's own term
//     and reference (held in registers: row c * 512 + tid of the thread),
//     then pointer jumping over the page (log2 of the longest reference
//     chain rounds), the rows' (term, reference) pairs published in LDS.
//  3. The rows go to HBM from the registers, coalesced.
// The status is the reference's: the first failing record's code, unless a
// row before it references a row before row 0 (OutOfSpec).  Pages whose
// stream and rows do not fit the LDS, or with more rows than the registers
// hold (kPatMaxRows: 16 a thread),
// stay with patas_wave (patas_fits).
// ---------------------------------------------------------------------------
constexpr uint64_t kPatIdent = 0xFFFFFF9876543210ull;  // entry e -> e (e < 10); 15 -> 15

// map b after map a: entry e -> b(a(e))
__device__ __forceinline__ uint64_t patas_comp(uint64_t a, uint64_t b) {
  uint64_t r = 0xFFFFFF0000000000ull;
#pragma unroll
  for (uint32_t e = 0; e < kPatE; e++) {
    const uint32_t x = (uint32_t)(a >> (4 * e)) & 15u;
    r |= ((b >> (4 * x)) & 15ull) << (4 * e);
  }
  return r;
}

// The segment [s0, s1) walked from its 10 entry offsets in lockstep.  Per
// entry e: cnt[e] records, er[e] the failing record's code (0: none); the
// returned map sends e to the entry offset into the next segment (15 after
// a failing record).  A record's size comes from its header alone; header or
// body past the stream is Io, more sig bytes than the type has OutOfSpec
// (the f32 desync of patas.rs:154-160).
__device__ __forceinline__ uint64_t patas_walks(const lds_u8* sz, uint32_t ilen, uint32_t s0, uint32_t s1,
                                                uint32_t (&cnt)[kPatE], uint32_t (&er)[kPatE]) {
  constexpr uint32_t kDead = 1u << 24;  // pos >= kDead: the walk met a failing record (pos - kDead: its code)
  uint32_t pos[kPatE];
#pragma unroll
  for (uint32_t e = 0; e < kPatE; e++) {
    pos[e] = s0 + e;
    cnt[e] = 0;
  }
  for (bool more = s0 < s1; more;) {  // a walk is live while pos < s1
    uint32_t d[kPatE];
#pragma unroll
    for (uint32_t e = 0; e < kPatE; e++) d[e] = sz[min(pos[e], ilen)];  // the reads first: one wait a step
    more = false;
#pragma unroll
    for (uint32_t e = 0; e < kPatE; e++) {
      const bool live = pos[e] < s1;
      const uint32_t np = pos[e] + d[e];
      const uint32_t nx = d[e] == 0 ? kDead + ST_OUT_OF_SPEC : np > ilen ? kDead + ST_IO : np;
      cnt[e] += live && nx < kDead ? 1u : 0u;
      pos[e] = live ? nx : pos[e];
      more |= pos[e] < s1;
    }
  }
  uint64_t m = 0xFFFFFF0000000000ull;
#pragma unroll
  for (uint32_t e = 0; e < kPatE; e++) {
    const bool dead = pos[e] >= kDead;
    er[e] = dead ? pos[e] - kDead : 0u;
    m |= (uint64_t)(dead ? 15u : min(pos[e] - s1, 15u)) << (4 * e);
  }
  return m;
}

// sz[p] for p in [0, ilen]: the size of a record whose header is at stream
// position p -- 2 + sig bytes; 0 for more sig bytes than the type has
// (OutOfSpec); 2 when the header itself is past the stream (so p + 2 > ilen:
// Io, which the reference reports first)
template <int W>
__device__ __forceinline__ void patas_sizes(const lds_u8* ib, uint32_t sb0, uint32_t ilen, lds_u8* sz) {
  typedef __attribute__((address_space(3))) uint32_t l32;
  const l32* ib32 = (const l32*)ib;
  l32* sz32 = (l32*)sz;
  for (uint32_t k = threadIdx.x; 4 * k <= ilen; k += kPatT) {
    const uint32_t x = sb0 + 4 * k, a = x >> 2, sh = x & 3;
    const uint32_t d0 = ib32[a], d1 = ib32[a + 1], d2 = ib32[a + 2];
    const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint32_t out = 0;
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) {
      const uint32_t h = (uint32_t)(((((uint64_t)w1 << 32) | w) >> (8 * b)) & 0xFFFFu);
      uint32_t sb = (h >> 6) & 7;
      sb = ((h & 0x3F) < 63 && sb == 0) ? 8u : sb;
      const uint32_t v = 4 * k + b + 2 > ilen ? 2u : sb > (uint32_t)W ? 0u : 2u + sb;
      out |= v << (8 * b);
    }
    sz32[k] = out;
  }
}

template <int W, uint32_t R>
__device__ uint32_t patas_block(const uint8_t* src, uint32_t ilen, uint8_t* dst, uint32_t n, lds_u8* lds) {
  using T = typename PT<W>::T;
  typedef __attribute__((address_space(3))) T lds_t;
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  constexpr uint32_t NW = kPatT / 64;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ uint64_t s_wmap[NW];
  __shared__ uint32_t s_wsum[NW], s_err_row, s_err_code;
  // LDS: the stream (16-byte aligned window) | rows (n + 1: row n is the
  // resolved sentinel; first the record size table) | references (first the
  // rows' record starts, u16: the stream is < 64 KiB)
  const uint32_t sb0 = (uint32_t)((uintptr_t)src & 15);
  const uint32_t nb = (sb0 + ilen + 15) >> 4;           // 16-byte blocks holding the stream
  const uint32_t ib_bytes = ((ilen + 62) + 15) & ~15u;  // >= (nb + 2) * 16
  const uint32_t rows_bytes = (max((n + 1) * W, ilen + 16) + 15) & ~15u;
  lds_u8* ib = lds;
  lds_t* vals = (lds_t*)(lds + ib_bytes);
  lds_u8* sz = (lds_u8*)vals;
  lds_u16* ptr = (lds_u16*)(lds + ib_bytes + rows_bytes);
  lds_u16* starts = ptr;
#ifdef SB_PAT_PHASES
  uint64_t tph = __builtin_amdgcn_s_memtime();
#endif
  {  // stage the stream's 16-byte blocks, four loads in flight a thread (the tail: copies of the last block)
    typedef const __attribute__((address_space(1))) u32x4 g128;
    typedef __attribute__((address_space(3))) u32x4 l128;
    g128* g = (g128*)((uintptr_t)src & ~(uintptr_t)15);
    l128* l = (l128*)ib;
    for (uint32_t i0 = 0; i0 < nb + 2; i0 += 4 * kPatT) {
      u32x4 r[4];
#pragma unroll
      for (uint32_t c = 0; c < 4; c++) r[c] = g[min(i0 + c * kPatT + tid, nb - 1)];
#pragma unroll
      for (uint32_t c = 0; c < 4; c++)
        if (i0 + c * kPatT + tid < nb + 2) l[i0 + c * kPatT + tid] = r[c];
    }
  }
  if (tid == 0) {
    s_err_row = n;
    s_err_code = 0;
  }
  __syncthreads();
  patas_sizes<W>(ib, sb0, ilen, sz);
  __syncthreads();
  PAT_T(0);
  // 1. record starts: segments of B >= 16 bytes after the first value
  const uint32_t q0 = W, body = ilen - q0;
  const uint32_t S = max(1u, min(kPatT, body / 16)), B = (body + S - 1) / S;
  const uint32_t s0 = q0 + min(tid * B, body), s1 = q0 + min((tid + 1) * B, body);
  uint32_t wcnt[kPatE], wer[kPatE];
  uint64_t fm = kPatIdent;
  if (tid < S) fm = patas_walks(sz, ilen, s0, s1, wcnt, wer);
  PAT_T(1);
  // each segment's entry: an exclusive scan of the maps in segment order,
  // evaluated at entry 0 (the first record starts right after the first value)
  uint64_t inc = fm;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc = patas_comp(y, inc);
  }
  uint64_t exc = __shfl_up(inc, 1, 64);
  if (lane == 0) exc = kPatIdent;
  if (lane == 63) s_wmap[wv] = inc;
  __syncthreads();
  uint32_t entry = 0;
  for (uint32_t k = 0; k < wv; k++) entry = (uint32_t)(s_wmap[k] >> (4 * entry)) & 15u;
  entry = (uint32_t)(exc >> (4 * entry)) & 15u;
  uint32_t cnt = 0, err = 0;
  if (tid < S) {
#pragma unroll
    for (uint32_t e = 0; e < kPatE; e++)
      if (entry == e) {
        cnt = wcnt[e];
        err = wer[e];
      }
  }
  // rows of the segments' records: an exclusive scan of the counts
  uint32_t incl = cnt;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wsum[wv] = incl;
  __syncthreads();
  uint32_t base = 1, total = 1;  // row of the segment's first record (row 0 is the first value)
#pragma unroll
  for (uint32_t k = 0; k < NW; k++) {
    base += k < wv ? s_wsum[k] : 0u;
    total += s_wsum[k];
  }
  base += incl - cnt;
  // the failing record (at most one: the walk stops there) in row order
  if (err && base + cnt < n) {
    s_err_row = base + cnt;
    s_err_code = err;
  }
  __syncthreads();
  if (tid == 0 && s_err_row == n && total < n) {  // the stream ends before row n - 1: the next header is past it
    s_err_row = total;
    s_err_code = ST_IO;
  }
  __syncthreads();
  const uint32_t rows_ok = s_err_row;
  PAT_T(2);
  {  // each row's record start
    uint32_t x = s0 + entry;
    const uint32_t m = base < rows_ok ? min(cnt, rows_ok - base) : 0u;
    for (uint32_t k = 0; k < m; k++) {
      starts[base + k] = (uint16_t)x;
      x += sz[x];
    }
  }
  __syncthreads();
  PAT_T(3);
  // 2. the thread's rows c * kPatT + tid: term and reference (kNone: resolved).
  // Rows past n are the sentinel's copies (value 0, reference kNone): every
  // step below runs on all R rows without a branch.
  typedef __attribute__((address_space(3))) uint32_t l32;
  const l32* ib32 = (const l32*)ib;
  const uint32_t kNone = n;  // the sentinel row: value 0, reference itself
  T tv[R];
  uint32_t tp[R];
  bool bad = false;
#pragma unroll
  for (uint32_t c = 0; c < R; c++) {
    const uint32_t i = c * kPatT + tid;
    const bool row = i > 0 && i < rows_ok;
    const uint32_t st = starts[min(i, n - 1)];  // (rows past the failing record hold no start)
    const uint32_t x = sb0 + (row ? st : 0u), a = x >> 2, sh = x & 3;
    const uint32_t d0 = ib32[a], d1 = ib32[a + 1], d2 = ib32[a + 2], d3 = ib32[a + 3];
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh),
                   w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    const uint32_t h = w0 & 0xFFFFu;
    const uint32_t rd = (h >> 9) & 0x7F, tz = h & 0x3F;
    uint32_t sb = (h >> 6) & 7;
    sb = (tz < 63 && sb == 0) ? 8u : sb;
    uint64_t v = ((uint64_t)(w0 >> 16) | ((uint64_t)w1 << 16) | ((uint64_t)w2 << 48));
    v = sb >= 8 ? v : (v & ((1ull << (8 * sb)) - 1));
    const T term = tz >= 8 * W ? (T)0 : (T)((T)v << tz);
    const T first = W == 8 ? (T)((uint64_t)w0 | ((uint64_t)w1 << 32)) : (T)w0;
    tv[c] = i == 0 ? first : row ? term : (T)0;
    bad |= row && (rd == 0 || rd > i);
    tp[c] = row ? i - rd : kNone;
  }
  if (__syncthreads_or(bad)) return ST_OUT_OF_SPEC;  // a reference before row 0, before the first failing record
#if SB_PAT_SHFL
  // references inside the row's wave group (the 64 rows c * kPatT + 64 * wave
  // + lane): pointer jumping through lane shuffles, 6 rounds; afterwards
  // every reference points before its group, so the chains the LDS rounds
  // follow are at most n / 64 groups long
#pragma unroll
  for (uint32_t r = 0; r < 6; r++) {
#pragma unroll
    for (uint32_t c = 0; c < R; c++) {
      const uint32_t g0 = c * kPatT + (tid & ~63u);  // the group's first row
      const bool in = tp[c] != kNone && tp[c] >= g0;
      const int src = (int)(in ? tp[c] - g0 : lane);
      const T ov = __shfl(tv[c], src, 64);
      const uint32_t op = __shfl(tp[c], src, 64);
      tv[c] = in ? (T)(tv[c] ^ ov) : tv[c];
      tp[c] = in ? op : tp[c];
    }
  }
#endif
  bool any = false;
#pragma unroll
  for (uint32_t c = 0; c < R; c++) {
    const uint32_t i = min(c * kPatT + tid, n);
    vals[i] = tv[c];
    ptr[i] = (uint16_t)tp[c];
    any |= tp[c] != kNone;
  }
  if (tid == 0) {  // (also when no row of a thread lies past n)
    vals[n] = 0;
    ptr[n] = (uint16_t)n;
  }
  any = __syncthreads_or(any);
  PAT_T(4);
  // pointer jumping: every row takes its reference's term and reference
  // (read as a pair, written after a barrier, so value(i) = term(i) ^
  // value(ref(i)) holds at every step; a resolved row reads the sentinel)
  for (uint32_t round = 0; any; round++) {
    if (round == 16) return ST_IO;  // (chains are < 8192 rows: 13 rounds; a bound on a broken invariant, never a hang)
    T rv[R];
    uint32_t rp[R];
#pragma unroll
    for (uint32_t c = 0; c < R; c++) {
      rv[c] = vals[tp[c]];
      rp[c] = ptr[tp[c]];
    }
    __syncthreads();
    any = false;
#pragma unroll
    for (uint32_t c = 0; c < R; c++) {
      const uint32_t i = min(c * kPatT + tid, n);
      tv[c] ^= rv[c];
      tp[c] = rp[c];
      vals[i] = tv[c];
      ptr[i] = (uint16_t)tp[c];
      any |= tp[c] != kNone;
    }
    any = __syncthreads_or(any);
    PAT_N(9, 1);
  }
  PAT_T(5);
  // 3. the rows, coalesced from the registers (rows from the failing record
  // on fall outside the buffer's range: the hardware drops them)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(rows_ok * W), 0x00020000);
#pragma unroll
  for (uint32_t c = 0; c < R; c++) {
    const uint32_t i = c * kPatT + tid;
    if constexpr (W == 8)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, (uint64_t)tv[c]), rs, (int)(i * 8), 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)tv[c], rs, (int)(i * 4), 0, 0);
  }
  PAT_T(6);
  PAT_N(8, 1);
  const uint32_t st = s_err_row < n ? s_err_code : ST_OK;
  __syncthreads();
  return st;
}

// Patas leaf jobs whose page fits (patas_fits), one workgroup each; k_inflate
// skips them (InflateLaunch::patas_wg).
// (three waves a SIMD's worth of VGPRs: a CU keeps room for k_inflate waves beside it)
__global__ __launch_bounds__(kPatT) __attribute__((amdgpu_waves_per_eu(3))) void k_patas(InflateLaunch a) {
  extern __shared__ u32x4 pat_dyn[];
  const uint32_t n = a.count ? *a.count : a.n_jobs;
  for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
    const InflateJob jb = a.jobs[j];
    const uint32_t W = jb.codec >> 8;
    const uint64_t kind = jb.dst >> 62, off = jb.dst & kDstMask;
    if ((jb.codec & 0xFF) != 16 || kind > 1 || (W != 4 && W != 8) || !patas_fits(jb.csize, jb.usize / W, W)) {
      if (jb.codec != 2 && a.sched && threadIdx.x == 0) atomicAdd(&a.sched[2], 1u);  // k_inflate's
      continue;
    }
    uint8_t* dst = kind == 1 ? a.scratch + off : a.out + off;
    const uint8_t* src = a.chunk + jb.src;
    const uint32_t rows = jb.usize / W;
    lds_u8* lds = (lds_u8*)pat_dyn;
    uint32_t st;
    if (W == 8)  // (patas_fits: <= 16 rows a thread)
      st = rows <= 4 * kPatT ? patas_block<8, 4>(src, jb.csize, dst, rows, lds)
                             : patas_block<8, 16>(src, jb.csize, dst, rows, lds);
    else
      st = rows <= 4 * kPatT ? patas_block<4, 4>(src, jb.csize, dst, rows, lds)
                             : patas_block<4, 16>(src, jb.csize, dst, rows, lds);
    if (st && threadIdx.x == 0) a.status[jb.page] = st;
  }
}
}  // namespace sbk

namespace sb {
int launch_patas(const InflateLaunch& a, void* stream) {
  ensure_lds_attr(sbk::k_patas, (int)kPatLds);
  // one workgroup a CU (the LDS holds one): each strides over the job list
  // (skipping the jobs that are not its costs a load, not a dispatch)
  static const uint32_t cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? (uint32_t)n : 256u;
  }();
  const uint32_t g = a.n_jobs < cus ? a.n_jobs : cus;
  hipLaunchKernelGGL(sbk::k_patas, dim3(g), dim3(sbk::kPatT), kPatLds, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace sb

#ifdef SB_PAT_PHASES
extern "C" int sb_debug_pat_phases(uint64_t* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(sbk::sb_dbg_pat), 16 * 8) == hipSuccess ? 0 : -1;
}
extern "C" int sb_debug_pat_reset() {
  static const unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(sbk::sb_dbg_pat), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
