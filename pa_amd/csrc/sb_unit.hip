// sb_unit.hip -- page-level unit entry points of the reference's read_basic.rs
// on MI355X (gfx950): the validity prefix of one flat page (read_validity,
// read/read_basic.rs:36-63) and the repetition / definition level streams of
// one nested page (read_validity_nested's decode, :65-86, parquet2's
// HybridRleDecoder).  The column decoders fuse both into their page kernels;
// these are the boundary a caller that walks pages itself binds.  One
// workgroup per call: thread 0 parses the run headers, the workgroup expands
// them.  Byte work; bound by the header walk, not by HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/strawboat_gpu.h"
#include "sb_internal.h"

namespace sbu {
using namespace sb;

constexpr uint32_t NT = 256;
constexpr uint32_t kRuns = 64;  // run headers parsed per round

// byte i of the page, 0 past its end
__device__ __forceinline__ uint32_t pbyte(const uint8_t* p, uint64_t len, uint64_t i) { return i < len ? p[i] : 0u; }
__device__ __forceinline__ uint32_t pu32(const uint8_t* p, uint64_t i) {
  return p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24);
}
__device__ bool uleb(const uint8_t* b, uint64_t n, uint64_t* p, uint64_t* v) {
  uint64_t r = 0;
  for (int sh = 0; sh <= 63; sh += 7) {
    if (*p >= n) return false;
    const uint32_t c = b[(*p)++];
    r |= (uint64_t)(c & 0x7F) << sh;
    if (!(c & 0x80)) {
      *v = r;
      return true;
    }
  }
  return false;
}

struct ValArgs {
  const uint8_t* page;
  uint64_t len, length;
  uint32_t* out;
  uint64_t bit0;
  uint64_t* res;  // [0] status, [1] bytes consumed
};

// The def-level prefix [u32 def_len][ULEB header][bit-packed bits]: one
// bit-packed run (an RLE run is unreachable!(), read_basic.rs:59) whose first
// `length` bits go to out at bit0 (words inside the range whole, edge words
// by mask).
__global__ __launch_bounds__(NT) void k_page_validity(ValArgs a) {
  __shared__ uint64_t src, st;
  if (threadIdx.x == 0) {
    st = ST_OK;
    uint64_t consumed = 0;
    if (a.len < 4) {
      st = ST_IO;
    } else {
      const uint32_t dl = pu32(a.page, 0);
      consumed = 4 + (uint64_t)dl;
      if (dl == 0) {
        if (a.length) st = ST_OUT_OF_SPEC;  // nothing pushed: the validity length mismatches
      } else if (4 + (uint64_t)dl > a.len) {
        st = ST_IO;
      } else {
        uint64_t p = 4, h = 0;
        if (!uleb(a.page, 4 + (uint64_t)dl, &p, &h) || !(h & 1)) {
          st = ST_OUT_OF_SPEC;
        } else {
          const uint64_t avail = min<uint64_t>(4 + (uint64_t)dl - p, h >> 1);
          if (avail * 8 < a.length) st = ST_OUT_OF_SPEC;  // BitmapIter bound
          src = p;
        }
      }
    }
    a.res[0] = st;
    a.res[1] = consumed;
  }
  __syncthreads();
  if (st != ST_OK || a.length == 0) return;
  const uint8_t* d = a.page + src;
  const uint64_t dlen = (a.length + 7) / 8;  // source bytes read
  const uint64_t w0 = a.bit0 >> 5, w1 = (a.bit0 + a.length - 1) >> 5;
  for (uint64_t w = w0 + threadIdx.x; w <= w1; w += NT) {
    const int64_t sb = (int64_t)(w * 32) - (int64_t)a.bit0;  // source bit of the word's bit 0
    uint64_t v;
    if (sb >= 0) {
      const uint64_t B = (uint64_t)sb >> 3;
      v = 0;
      for (uint32_t k = 0; k < 5; k++) v |= (uint64_t)pbyte(d, dlen, B + k) << (8 * k);
      v >>= (sb & 7);
    } else {
      v = 0;
      for (uint32_t k = 0; k < 4; k++) v |= (uint64_t)pbyte(d, dlen, k) << (8 * k);
      v <<= -sb;
    }
    const int64_t lo = max<int64_t>(0, -sb), hi = min<int64_t>(32, (int64_t)a.length - sb);
    const uint32_t m = (hi >= 32 ? 0xFFFFFFFFu : ((1u << hi) - 1)) & (0xFFFFFFFFu << lo);
    const uint32_t bits = (uint32_t)v & m;
    if (m == 0xFFFFFFFFu) {
      a.out[w] = bits;
    } else {
      atomicAnd(&a.out[w], ~m);
      atomicOr(&a.out[w], bits);
    }
  }
}

struct LevArgs {
  const uint8_t* page;
  uint64_t len, n;
  uint32_t bw[2];
  uint16_t* out[2];
  uint64_t* res;  // [0] status, [1] bytes consumed, [2] header row count
};

struct Run {
  uint64_t at;   // first output level
  uint64_t cnt;  // levels
  uint64_t pos;  // bit-packed: byte position of the run's data; RLE: the value
  uint32_t rle;
};

// HybridRleDecoder over [data, data + dlen) with bit width bw -> n levels
// (parquet2: a bit-packed run clamped to the bytes present, an RLE run of
// ceil(bw / 8) value bytes); all threads.
__device__ void hybrid_levels(const uint8_t* data, uint64_t dlen, uint32_t bw, uint64_t n, uint16_t* out,
                              uint64_t* st) {
  __shared__ Run runs[kRuns];
  __shared__ uint32_t nr;
  __shared__ uint64_t p, got;
  if (threadIdx.x == 0) p = 0, got = 0;
  __syncthreads();
  if (bw == 0) {  // no level bits: every level is 0 (nothing read)
    for (uint64_t i = threadIdx.x; i < n; i += NT) out[i] = 0;
    return;
  }
  for (;;) {
    if (threadIdx.x == 0) {
      nr = 0;
      while (got < n && nr < kRuns && *st == ST_OK) {
        uint64_t h;
        if (!uleb(data, dlen, &p, &h)) {
          *st = ST_OUT_OF_SPEC;
          break;
        }
        Run r{got, 0, 0, 0};
        if (h & 1) {
          const uint64_t nbytes = (h >> 1) * bw, have = min<uint64_t>(dlen - p, nbytes);
          const uint64_t vals = min<uint64_t>((h >> 1) * 8, have * 8 / bw);
          if (vals == 0) {
            *st = ST_OUT_OF_SPEC;
            break;
          }
          r.cnt = min<uint64_t>(vals, n - got);
          r.pos = p;
          p += have;
        } else {
          const uint32_t vb = (bw + 7) / 8;
          if (p + vb > dlen) {
            *st = ST_OUT_OF_SPEC;
            break;
          }
          uint32_t v = 0;
          for (uint32_t k = 0; k < vb; k++) v |= (uint32_t)data[p + k] << (8 * k);
          p += vb;
          r.rle = 1;
          r.pos = v;
          r.cnt = min<uint64_t>(h >> 1, n - got);
        }
        runs[nr++] = r;
        got += r.cnt;
      }
    }
    __syncthreads();
    const uint32_t m = nr;
    for (uint32_t k = 0; k < m; k++) {
      const Run r = runs[k];
      for (uint64_t i = threadIdx.x; i < r.cnt; i += NT) {
        uint32_t v;
        if (r.rle) {
          v = (uint32_t)r.pos;
        } else {
          const uint64_t bit = i * bw;
          uint64_t x = 0;
          const uint64_t B = r.pos + (bit >> 3);
          for (uint32_t j = 0; j < 5; j++) x |= (uint64_t)pbyte(data, dlen, B + j) << (8 * j);
          v = (uint32_t)(x >> (bit & 7)) & (bw >= 32 ? 0xFFFFFFFFu : ((1u << bw) - 1));
        }
        out[r.at + i] = (uint16_t)v;
      }
    }
    const bool more = got < n && *st == ST_OK;
    __syncthreads();
    if (!more) return;
  }
}

// [rows u32][rep_len u32][def_len u32][rep levels][def levels] (serialize.rs
// write_nested): both streams to u16 levels.
__global__ __launch_bounds__(NT) void k_page_levels(LevArgs a) {
  __shared__ uint64_t st, rl, dl;
  if (threadIdx.x == 0) {
    st = ST_OK;
    a.res[2] = 0;
    if (a.len < 12) {
      st = ST_IO;
    } else {
      rl = pu32(a.page, 4);
      dl = pu32(a.page, 8);
      if (12 + rl + dl > a.len) st = ST_IO;
      a.res[2] = pu32(a.page, 0);
    }
    a.res[1] = st == ST_OK ? 12 + rl + dl : 0;
  }
  __syncthreads();
  if (st == ST_OK) hybrid_levels(a.page + 12, rl, a.bw[0], a.n, a.out[0], &st);
  __syncthreads();
  if (st == ST_OK) hybrid_levels(a.page + 12 + rl, dl, a.bw[1], a.n, a.out[1], &st);
  __syncthreads();
  if (threadIdx.x == 0) a.res[0] = st;
}

}  // namespace sbu

static uint32_t bit_width(uint32_t max_level) {  // parquet2 get_bit_width
  return max_level ? 32 - (uint32_t)__builtin_clz(max_level) : 0;
}

static sb_status finish(sb_ctx* ctx, uint64_t* d_res, uint64_t* h_res, int n, const char* what) {
  hipStream_t st = (hipStream_t)sb_ctx_stream(ctx);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h_res, d_res, n * sizeof(uint64_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return (sb_status)sb::ctx_fail(ctx, SB_E_DEVICE, what, (int)e);
  if (h_res[0] != sb::ST_OK) return (sb_status)sb::ctx_fail(ctx, (int)h_res[0], what, 0);
  return SB_OK;
}

extern "C" sb_status sb_decode_page_validity(sb_ctx* ctx, const uint8_t* d_page, uint64_t page_len, uint64_t length,
                                             uint32_t* d_validity, uint64_t bit_offset, uint64_t* h_consumed) {
  if (!ctx || !d_page || (length && !d_validity)) return SB_E_ARG;
  if (hipSetDevice(sb_ctx_device(ctx)) != hipSuccess) return SB_E_DEVICE;
  uint64_t* d_res = (uint64_t*)sb::ctx_scratch(ctx, 64, 3);
  if (!d_res) return (sb_status)sb::ctx_fail(ctx, SB_E_DEVICE, "page validity scratch", -1);
  const sbu::ValArgs a{d_page, page_len, length, d_validity, bit_offset, d_res};
  hipLaunchKernelGGL(sbu::k_page_validity, dim3(1), dim3(sbu::NT), 0, (hipStream_t)sb_ctx_stream(ctx), a);
  uint64_t h[2] = {0, 0};
  const sb_status s = finish(ctx, d_res, h, 2, "sb_decode_page_validity");
  if (h_consumed) *h_consumed = h[1];
  return s;
}

extern "C" sb_status sb_decode_page_levels(sb_ctx* ctx, const uint8_t* d_page, uint64_t page_len, uint64_t num_levels,
                                           uint32_t max_rep_level, uint32_t max_def_level, uint16_t* d_rep,
                                           uint16_t* d_def, uint32_t* h_rows, uint64_t* h_consumed) {
  if (!ctx || !d_page || (num_levels && (!d_rep || !d_def)) || max_rep_level > 0xFFFF || max_def_level > 0xFFFF)
    return SB_E_ARG;
  if (hipSetDevice(sb_ctx_device(ctx)) != hipSuccess) return SB_E_DEVICE;
  uint64_t* d_res = (uint64_t*)sb::ctx_scratch(ctx, 64, 3);
  if (!d_res) return (sb_status)sb::ctx_fail(ctx, SB_E_DEVICE, "page levels scratch", -1);
  const sbu::LevArgs a{d_page, page_len, num_levels, {bit_width(max_rep_level), bit_width(max_def_level)},
                       {d_rep, d_def}, d_res};
  hipLaunchKernelGGL(sbu::k_page_levels, dim3(1), dim3(sbu::NT), 0, (hipStream_t)sb_ctx_stream(ctx), a);
  uint64_t h[3] = {0, 0, 0};
  const sb_status s = finish(ctx, d_res, h, 3, "sb_decode_page_levels");
  if (h_rows) *h_rows = (uint32_t)h[2];
  if (h_consumed) *h_consumed = h[1];
  return s;
}
