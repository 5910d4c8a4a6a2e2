// sb_encode_gpu.hip -- page encode on MI355X (gfx950) for the writer options
// whose codec choice needs no sampling: NativeWriter::encode_chunk
// (write/common.rs:49-119) -> write_simple (write/serialize.rs:52-132) with
// default_compress_ratio None, default codec None and optionally the forced
// Bitpacking codec of util/env.rs.  choose_compressor
// (compression/integer/mod.rs:231-308) then picks Bitpacking for a page of
// Int32 / UInt32 whose values are all >= 0 and whose length is a multiple of
// 128 (bp.rs:92-100), and Compression::None otherwise.  Output is byte-identical
// to the host writer (sb_encode.cpp) for those options.
//
// Pass 1 (k_enc_size): one workgroup per page -- per-128-value block bit
// widths (BitPacker4x::num_bits of the raw values, bp.rs:45-51) and the page
// length.  Pass 2 (k_enc_scan): page byte offsets.  Pass 3 (k_enc_write): the
// page is assembled in LDS -- validity prefix (write_validity, serialize.rs:
// 200-215: u32 def_len + ULEB128 bit-packed run header + bitmap), codec header
// [codec u8][csize u32][usize u32], body -- and stored with aligned 16-byte
// writes.  Integer/byte work only: bound by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/strawboat_gpu.h"
#include "sb_internal.h"

namespace sbe {

constexpr int NT = 256;
constexpr uint32_t kMaxPageRows = 16384;
constexpr uint32_t kLds = 140 * 1024;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct EncArgs {
  const uint8_t* values;    // column values, n_rows * W bytes
  const uint8_t* validity;  // LSB bitmap of the column (nullable) or nullptr
  uint64_t n_rows;
  uint32_t page_rows;
  uint32_t n_pages;
  uint32_t width;           // sizeof(T)
  int is_signed;
  int bitpack;              // forced Bitpacking applies to this type
  int nullable;
  uint8_t* bw;              // bit width per block (page p: blocks from p * page_rows / 128)
  uint64_t* sizes;          // page lengths
  uint64_t* offs;           // page offsets (exclusive scan), [n_pages] = total
  uint8_t* out;
};

__device__ __forceinline__ uint32_t page_n(const EncArgs& a, uint32_t p) {
  const uint64_t r0 = (uint64_t)p * a.page_rows;
  return (uint32_t)min<uint64_t>(a.page_rows, a.n_rows - r0);
}
__device__ __forceinline__ uint32_t uleb_len(uint64_t h) {
  uint32_t l = 1;
  while (h >= 0x80) { h >>= 7; l++; }
  return l;
}
// validity prefix bytes: u32 def_len + ULEB128((nbytes << 1) | 1) + nbytes
__device__ __forceinline__ uint32_t prefix_len(const EncArgs& a, uint32_t n) {
  if (!a.nullable) return 0;
  const uint32_t nb = (n + 7) / 8;
  return 4 + uleb_len(((uint64_t)nb << 1) | 1) + nb;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  for (int d = 32; d; d >>= 1) v |= __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ uint32_t val32(const EncArgs& a, uint64_t row) { return ((const uint32_t*)a.values)[row]; }

__global__ __launch_bounds__(NT) void k_enc_size(EncArgs a) {
  __shared__ uint32_t s_sum[NT / 64], s_neg;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (uint32_t p = blockIdx.x; p < a.n_pages; p += gridDim.x) {
    const uint32_t n = page_n(a, p);
    const uint64_t r0 = (uint64_t)p * a.page_rows;
    const uint32_t nblk = n / 128;
    const bool try_bp = a.bitpack && n % 128 == 0;
    if (tid == 0) s_neg = 0;
    __syncthreads();
    uint32_t part = 0;
    if (try_bp) {
      for (uint32_t k = wv; k < nblk; k += NT / 64) {
        const uint64_t b0 = r0 + 128ull * k;
        const uint32_t acc = wave_or(val32(a, b0 + lane) | val32(a, b0 + 64 + lane));
        const uint32_t b = acc ? 32 - __builtin_clz(acc) : 0;
        if (lane == 0) {
          a.bw[(uint64_t)p * (a.page_rows / 128) + k] = (uint8_t)b;
          part += 1 + 16 * b;
          // bp_eligible: min >= 0 over every row, nulls included -- an Int32
          // value is negative exactly when its bit 31 is set
          if (a.is_signed && (acc >> 31)) s_neg = 1;
        }
      }
    }
    if (lane == 0) s_sum[wv] = part;
    __syncthreads();
    if (tid == 0) {
      const bool bp = try_bp && !s_neg;
      uint32_t body = 0;
      for (int w = 0; w < NT / 64; w++) body += s_sum[w];
      if (!bp) body = n * a.width;
      a.sizes[p] = (uint64_t)prefix_len(a, n) + 9 + body;
      if (!bp && a.bitpack) a.bw[(uint64_t)p * (a.page_rows / 128)] = 0xFF;  // marks a None page
    }
    __syncthreads();
  }
}

// exclusive scan of the page lengths, one workgroup
__global__ __launch_bounds__(NT) void k_enc_scan(EncArgs a) {
  __shared__ uint64_t s_w[NT / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint64_t carry = 0;
  for (uint32_t p0 = 0; p0 < a.n_pages; p0 += NT) {
    const uint32_t p = p0 + tid;
    const uint64_t v = p < a.n_pages ? a.sizes[p] : 0;
    uint64_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (uint32_t w = 0; w < NT / 64; w++) {
      pre += w < wv ? s_w[w] : 0;
      tot += s_w[w];
    }
    if (p < a.n_pages) a.offs[p] = carry + pre + x - v;
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) a.offs[a.n_pages] = carry;
}

// BitPacker4x layout (bitpacking 0.8.0): value 4i + l of a block sits at bit
// i*b of lane l's bit stream; lane word k is at byte 16k + 4l.
typedef __attribute__((address_space(3))) uint32_t l32;
__device__ __forceinline__ uint32_t bp_word(const l32* x, uint32_t b, uint32_t w) {  // x: the block's 128 values
  const uint32_t k = w >> 2, l = w & 3;
  const uint64_t mask = b == 32 ? 0xFFFFFFFFull : ((1ull << b) - 1);
  const uint32_t i0 = (32 * k) / b, i1 = min(31u, (32 * k + 31) / b);
  uint32_t word = 0;
  for (uint32_t i = i0; i <= i1; i++) {
    const uint64_t v = x[4 * i + l] & mask;
    const int32_t sft = (int32_t)(i * b) - (int32_t)(32 * k);
    word |= sft >= 0 ? (uint32_t)(v << sft) : (uint32_t)(v >> -sft);
  }
  return word;
}

__global__ __launch_bounds__(NT) void k_enc_write(EncArgs a) {
  extern __shared__ u32x4 lds[];
  __shared__ uint32_t s_boff[kMaxPageRows / 128 + 1];
  typedef __attribute__((address_space(3))) uint8_t l8;
  const uint32_t tid = threadIdx.x;
  for (uint32_t p = blockIdx.x; p < a.n_pages; p += gridDim.x) {
    const uint32_t n = page_n(a, p);
    const uint64_t r0 = (uint64_t)p * a.page_rows;
    uint8_t* dst = a.out + a.offs[p];
    const uint32_t len = (uint32_t)a.sizes[p];
    l8* pg = (l8*)lds + ((uintptr_t)dst & 15);  // the page in LDS, at dst's alignment mod 16
    const uint8_t* bwp = a.bw + (uint64_t)p * (a.page_rows / 128);
    const bool bp = a.bitpack && n % 128 == 0 && bwp[0] != 0xFF;
    uint32_t q = 0;
    if (a.nullable) {  // write_validity
      const uint32_t nb = (n + 7) / 8;
      uint64_t h = ((uint64_t)nb << 1) | 1;
      const uint32_t hl = uleb_len(h);
      if (tid == 0) {
        const uint32_t dl = hl + nb;
        for (int j = 0; j < 4; j++) pg[j] = (uint8_t)(dl >> (8 * j));
        for (uint32_t j = 0; j < hl; j++, h >>= 7) pg[4 + j] = (uint8_t)((h & 0x7F) | (j + 1 < hl ? 0x80 : 0));
      }
      for (uint32_t j = tid; j < nb; j += NT) {
        const uint64_t bit0 = r0 + 8ull * j;
        const uint32_t sh = (uint32_t)(bit0 & 7);
        const uint64_t by = bit0 >> 3;
        uint32_t v = a.validity[by];
        if (sh && bit0 + 8 - sh < a.n_rows) v |= (uint32_t)a.validity[by + 1] << 8;
        v = (v >> sh) & 0xFF;
        const uint32_t left = n - 8 * j;
        if (left < 8) v &= (1u << left) - 1;
        pg[4 + hl + j] = (uint8_t)v;
      }
      q = 4 + hl + nb;
    }
    const uint32_t body = len - q - 9;
    if (tid == 0) {
      pg[q] = bp ? 14 : 0;
      for (int j = 0; j < 4; j++) pg[q + 1 + j] = (uint8_t)(body >> (8 * j));
      const uint32_t us = n * a.width;
      for (int j = 0; j < 4; j++) pg[q + 5 + j] = (uint8_t)(us >> (8 * j));
    }
    q += 9;
    if (bp) {
      const uint32_t nblk = n / 128;
      // the page's values, staged with 16-byte loads after the assembly area
      l32* x = (l32*)((l8*)lds + ((16 + len + 15) & ~15u));
      if (((uintptr_t)a.values & 15) == 0) {
        for (uint32_t i = tid; i < n / 4; i += NT)
          ((__attribute__((address_space(3))) u32x4*)x)[i] = ((const u32x4*)(a.values + r0 * 4))[i];
      } else {
        for (uint32_t i = tid; i < n; i += NT) x[i] = val32(a, r0 + i);
      }
      if (tid == 0) {  // block offsets: [u8 b][16 b bytes] back to back (<= 128 blocks)
        uint32_t o = q;
        for (uint32_t k = 0; k < nblk; k++) {
          s_boff[k] = o;
          o += 1 + 16 * bwp[k];
        }
      }
      __syncthreads();
      for (uint32_t s = tid; s < nblk * 128; s += NT) {
        const uint32_t k = s >> 7, w = s & 127, b = bwp[k];
        const uint32_t o = s_boff[k];
        if (w == 0) pg[o] = (uint8_t)b;
        if (w < 4 * b) {
          const uint32_t word = bp_word(x + 128 * k, b, w);
          for (int j = 0; j < 4; j++) pg[o + 1 + 4 * w + j] = (uint8_t)(word >> (8 * j));
        }
      }
    } else {  // Compression::None: the raw value bytes
      const uint8_t* src = a.values + r0 * a.width;
      for (uint32_t j = tid; j < n * a.width; j += NT) pg[q + j] = src[j];
    }
    __syncthreads();
    // LDS -> HBM: head bytes, aligned 16-byte body, tail bytes
    const uint32_t head = min(len, (16u - (uint32_t)((uintptr_t)dst & 15)) & 15u);
    const uint32_t nq = (len - head) >> 4, tail0 = head + 16 * nq;
    if (tid < head) dst[tid] = pg[tid];
    const __attribute__((address_space(3))) u32x4* lq = (const __attribute__((address_space(3))) u32x4*)(pg + head);
    for (uint32_t i = tid; i < nq; i += NT) ((u32x4*)(dst + head))[i] = lq[i];
    if (tid < len - tail0) dst[tail0 + tid] = pg[tail0 + tid];
    __syncthreads();
  }
}

}  // namespace sbe

static uint32_t type_width(int32_t t) {
  switch (t) {
    case SB_T_INT8: case SB_T_UINT8: return 1;
    case SB_T_INT16: case SB_T_UINT16: return 2;
    case SB_T_INT32: case SB_T_UINT32: case SB_T_FLOAT32: return 4;
    case SB_T_INT64: case SB_T_UINT64: case SB_T_FLOAT64: return 8;
  }
  return 0;
}

namespace sb {
struct ListPart;
uint64_t adaptive_slot_bytes(uint64_t P, uint32_t w, int nullable);
int encode_adaptive(sb_ctx* ctx, int phys, const uint8_t* d_values, const uint8_t* d_validity, uint64_t n_rows,
                    int nullable, const sb_write_options* opts, uint64_t P, uint8_t* d_out, uint64_t out_cap,
                    uint64_t* out_len, sb_page_meta* h_metas, uint64_t np, const ListPart* lp);
int encode_list_device(sb_ctx* ctx, int phys, const int64_t* d_offsets, const uint8_t* d_list_validity,
                       int list_nullable, const void* d_child, const uint8_t* d_child_validity, int item_nullable,
                       uint64_t n_rows, const sb_write_options* opts, uint64_t step, uint8_t* d_out, uint64_t out_cap,
                       uint64_t* out_len, sb_page_meta* h_metas, uint64_t np);
}  // namespace sb

extern "C" uint64_t sb_encode_device_bound(int32_t physical_type, uint64_t n_rows, int32_t nullable,
                                           uint64_t max_page_rows) {
  const uint64_t w = physical_type == SB_T_BOOLEAN ? 1 : type_width(physical_type);
  const uint64_t P = max_page_rows ? std::min(max_page_rows, n_rows) : n_rows;
  if (!w || !P) return 0;
  const uint64_t pages = (n_rows + P - 1) / P;
  // per page: prefix (4 + <= 10 + P/8) + header 9 + max(raw, bitpacked at b = 32)
  const uint64_t fast = (nullable ? 14 + (P + 7) / 8 : 0) + 9 + std::max(P * w, P / 128 * 513) + 16;
  // the adaptive cascade's worst case (forced RLE, Dict / Freq cascades)
  return pages * std::max(fast, sb::adaptive_slot_bytes(P, (uint32_t)w, nullable));
}

extern "C" sb_status sb_encode_column_device(sb_ctx* ctx, int32_t physical_type, const void* d_values,
                                             const uint8_t* d_validity, uint64_t n_rows, int32_t nullable,
                                             const sb_write_options* opts, uint64_t max_page_rows, uint8_t* d_out,
                                             uint64_t out_capacity, uint64_t* out_len, sb_page_meta* h_metas,
                                             uint64_t metas_cap, uint64_t* n_pages) {
  if (!ctx || !opts || !out_len || !n_pages) return SB_E_ARG;
  const bool is_bool = physical_type == SB_T_BOOLEAN;  // d_values = the column's LSB bitmap
  const uint32_t w = is_bool ? 1 : type_width(physical_type);
  // page_size = max_page_size.unwrap_or(len).min(len) (write/common.rs:54-58)
  const uint64_t P = max_page_rows ? std::min(max_page_rows, n_rows) : n_rows;
  if (!w || (nullable && !d_validity) || (n_rows && (!d_values || !d_out))) return SB_E_ARG;
  const uint64_t np = n_rows ? (n_rows + P - 1) / P : 0;
  *n_pages = np;
  if (np > metas_cap || (h_metas == nullptr && np)) return SB_E_ARG;
  *out_len = 0;
  if (!np) return SB_OK;
  if (hipSetDevice(sb_ctx_device(ctx)) != hipSuccess) return SB_E_DEVICE;
  // Options whose codec choice needs no trial compression (ratio None, default
  // None, forced codec none or Bitpacking: choose_compressor,
  // integer/mod.rs:231-240) take the sizing + assembly fast path; every other
  // option runs the adaptive cascade (sb_encode_adapt.hip).
  const bool forced_bp = opts->forced_codec == SB_CODEC_BITPACKING && !(opts->forbidden_mask & (1u << 14));
  const bool forced_other = opts->forced_codec >= 0 && !forced_bp && !(opts->forbidden_mask & (1u << opts->forced_codec));
  if (is_bool || opts->has_ratio || opts->default_codec != SB_CODEC_NONE || forced_other || P > sbe::kMaxPageRows ||
      (P % 128 && P < n_rows) || 2 * P * w + 8192 > sbe::kLds)
    return (sb_status)sb::encode_adaptive(ctx, physical_type, (const uint8_t*)d_values, d_validity, n_rows, nullable,
                                          opts, P, d_out, out_capacity, out_len, h_metas, np, nullptr);
  if (out_capacity < sb_encode_device_bound(physical_type, n_rows, nullable, P)) return SB_E_ARG;
  hipStream_t st = (hipStream_t)sb_ctx_stream(ctx);
  const bool bp = forced_bp && (physical_type == SB_T_INT32 || physical_type == SB_T_UINT32);
  uint8_t* d_bw = nullptr;
  uint64_t* d_sz = nullptr;
  hipError_t e = hipMalloc((void**)&d_bw, np * (P / 128 + 1));
  if (e == hipSuccess) e = hipMalloc((void**)&d_sz, (2 * np + 1) * sizeof(uint64_t));
  if (e != hipSuccess) {
    (void)hipFree(d_bw);
    return SB_E_DEVICE;
  }
  sbe::EncArgs a{(const uint8_t*)d_values, d_validity, n_rows, (uint32_t)P, (uint32_t)np, w,
                 physical_type == SB_T_INT32, bp, nullable, d_bw, d_sz, d_sz + np, d_out};
  sb::ensure_lds_attr(sbe::k_enc_write, (int)sbe::kLds);
  const dim3 grid((uint32_t)std::min<uint64_t>(np, 65535));
  hipLaunchKernelGGL(sbe::k_enc_size, grid, dim3(sbe::NT), 0, st, a);
  hipLaunchKernelGGL(sbe::k_enc_scan, dim3(1), dim3(sbe::NT), 0, st, a);
  // page assembly area (+16 for the alignment shift) and, for Bitpacking, the staged values
  const uint64_t page_max = (nullable ? 14 + (P + 7) / 8 : 0) + 9 + std::max<uint64_t>(P * w, P / 128 * 513);
  const uint32_t lds = (uint32_t)std::min<uint64_t>(sbe::kLds, ((16 + page_max + 15) & ~15ull) + (bp ? 4 * P : 0) + 16);
  hipLaunchKernelGGL(sbe::k_enc_write, grid, dim3(sbe::NT), lds, st, a);
  std::vector<uint64_t> sz(np);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(sz.data(), d_sz, np * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(out_len, d_sz + 2 * np, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d_bw);
  (void)hipFree(d_sz);
  if (e != hipSuccess) return SB_E_DEVICE;
  for (uint64_t p = 0; p < np; p++) h_metas[p] = sb_page_meta{sz[p], std::min<uint64_t>(P, n_rows - p * P)};
  return SB_OK;
}

// encode_chunk for one List<primitive> leaf on the device
// (include/strawboat_gpu.h; byte-identical to sb_encode_list_column).
extern "C" uint64_t sb_encode_list_device_bound(int32_t physical_type, uint64_t n_rows, uint64_t n_child,
                                                int32_t item_nullable, uint64_t max_page_rows) {
  const uint64_t w = type_width(physical_type);
  const uint64_t P = max_page_rows ? std::min(max_page_rows, n_rows) : n_rows;
  if (!w || !P) return 0;
  const uint64_t pages = (n_rows + P - 1) / P;
  // the level headers (<= 12 + 20 + (rows + values) * 3 / 8 + 1 a page) and
  // the child values' pages: adaptive_slot_bytes is affine in the rows, so
  // the pages' slots sum to <= pages x slot(1) + slot(n_child)
  return pages * (48 + 16 + sb::adaptive_slot_bytes(1, (uint32_t)w, 0)) + (n_rows + n_child) * 3 / 8 +
         sb::adaptive_slot_bytes(std::max<uint64_t>(n_child, 1), (uint32_t)w, 0);
}

extern "C" sb_status sb_encode_list_column_device(sb_ctx* ctx, int32_t physical_type, const int64_t* d_offsets,
                                                  const uint8_t* d_list_validity, int32_t list_nullable,
                                                  const void* d_child, const uint8_t* d_child_validity,
                                                  int32_t item_nullable, uint64_t n_rows,
                                                  const sb_write_options* opts, uint64_t max_page_rows, uint8_t* d_out,
                                                  uint64_t out_capacity, uint64_t* out_len, sb_page_meta* h_metas,
                                                  uint64_t metas_cap, uint64_t* n_pages) {
  if (!ctx || !opts || !out_len || !n_pages || !d_offsets) return SB_E_ARG;
  if (!type_width(physical_type)) return SB_E_NYI;
  if ((list_nullable && !d_list_validity) || (item_nullable && !d_child_validity) || (n_rows && !d_out))
    return SB_E_ARG;
  const uint64_t step = max_page_rows ? std::min(max_page_rows, n_rows) : n_rows;
  const uint64_t np = step ? (n_rows + step - 1) / step : 0;
  *n_pages = np;
  if (np > metas_cap || (h_metas == nullptr && np)) return SB_E_ARG;
  *out_len = 0;
  if (!np) return SB_OK;
  if (step > sbe::kMaxPageRows) return SB_E_NYI;  // (the level prefix of a page lives in LDS)
  if (hipSetDevice(sb_ctx_device(ctx)) != hipSuccess) return SB_E_DEVICE;
  return (sb_status)sb::encode_list_device(ctx, physical_type, d_offsets, d_list_validity, list_nullable, d_child,
                                           d_child_validity, item_nullable, n_rows, opts, step, d_out, out_capacity,
                                           out_len, h_metas, np);
}
