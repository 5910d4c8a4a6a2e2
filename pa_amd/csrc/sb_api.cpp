// sb_api.cpp -- host side of the C ABI (include/strawboat_gpu.h).
//
// Plays the role of the reference's NativeReader + read_* drivers
// (read/reader.rs:51-146, read/array/integer.rs:210-238): it turns
// ColumnMeta.pages into a device page table and launches the batched page
// kernels on the context's HIP stream.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/strawboat_gpu.h"
#include "sb_internal.h"

struct sb_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  void* scr[sb::kCtxScratchSlots] = {};  // sb::ctx_scratch
  size_t scr_bytes[sb::kCtxScratchSlots] = {};
};

namespace sb {
void* ctx_scratch(sb_ctx* c, size_t bytes, int slot) {
  if (!c || slot < 0 || slot >= kCtxScratchSlots) return nullptr;
  if (c->scr_bytes[slot] < bytes) {
    if (c->scr[slot]) {
      (void)hipStreamSynchronize(c->stream);  // earlier work on the stream may still use it
      (void)hipFree(c->scr[slot]);
    }
    c->scr[slot] = nullptr;
    c->scr_bytes[slot] = 0;
    if (hipMalloc(&c->scr[slot], bytes) != hipSuccess) return nullptr;
    c->scr_bytes[slot] = bytes;
  }
  return c->scr[slot];
}
int ctx_fail(sb_ctx* c, int st, const char* what, int hip_error) {
  if (c) {
    c->err = what;
    const hipError_t e = hip_error >= 0 ? (hipError_t)hip_error : hipGetLastError();
    if (e != hipSuccess) {
      c->err += ": ";
      c->err += hipGetErrorString(e);
    }
  }
  return st;
}
}  // namespace sb

struct sb_plan {
  sb_column_desc desc{};
  const uint8_t* d_chunk = nullptr;
  uint64_t chunk_len = 0;
  uint64_t n_pages = 0, n_rows = 0;
  int width = 0;
  bool is_float = false;
  sb::PageDesc* d_pages = nullptr;
  uint32_t* d_status = nullptr;
  uint32_t* d_lists = nullptr;  // [staged list | global list]
  uint32_t* d_light = nullptr;  // fixed width: per-page header-only tags (k_fix_light)
  bool has_zstd_big = false;    // some header-only jobs are Zstd frames (k_zinflate)
  uint32_t* d_defer = nullptr;  // [defer count x2 | inflate job count x2 | work list...]
  sb::InflateJob* d_jobs = nullptr;  // fixed: one per page; binary: two per page
  uint8_t* d_scratch = nullptr;      // binary: expanded offsets streams
  uint8_t* d_region = nullptr;       // fixed width: the pages' HBM regions (PageDesc.reserved)
  uint32_t* d_spill = nullptr;       // [2] spilled-leaf job counts (by decode parity)
  uint32_t* d_sched = nullptr;       // [2][3] k_inflate's job claim counters (zero between launches), two triples
  uint32_t sched_flip = 0;           // the pair the next inflate launch claims from
  uint8_t* d_ascii = nullptr;        // binary: per page, its values stream inflated all ASCII (k_inflate)
  sb::InflateJob* d_spill_jobs = nullptr;
  uint32_t n_spill = 0;              // pages with a spill area (bounds the spill launches)
  uint32_t n_big = 0;                // binary: big Extend pages (tables in d_region)
  uint32_t n_bin_jobs = 0;
  uint64_t decodes = 0;
  int deferred_state = -1;  // -1 unknown, 0 no deferred pages, 1 some
  int inflate_state = -1;   // same, for k_inflate jobs
  bool binary = false;
  bool boolean = false;  // SB_T_BOOLEAN: values are a bitmap (k_bool_decode)
  bool list = false;     // List<primitive>: levels kernels + `inner` (the values streams as flat pages)
  bool nested = false;   // general nesting (sb_nested_desc): k_nest_walk + `inner`
  bool list_walk = false;  // a List plan served by the general walk (level streams k_list cannot take)
  sb_nested_desc ndesc{};
  uint64_t* d_nest = nullptr;        // [counts n(D+1) | bases n(D+1) | totals D+1]
  std::vector<uint64_t> nest_totals;  // entries per level
  sb_list_desc ldesc{};
  uint8_t* d_lc = nullptr;  // list state, see list_state_bytes
  bool list_peek = false;   // sizes from the page headers (checked against the levels at plan time)
  uint16_t list_epoch = 0;  // tag of the last decode's block totals (k_list_bases)
  sb_plan* inner = nullptr;
  uint64_t n_leaves = 0;
  int offset_width = 0;
  uint64_t* d_bin = nullptr;  // [sizes n | bases n | total 1 | UTF-8 flags 1] then BinLaunch::cls (u32)
  uint64_t* d_lb = nullptr;   // binary, every page staged: the fused pass's look-back states + counter
  uint32_t bin_grid = 0;      // staged-pass workgroups: the plan pass's staged page count
  uint32_t bin_lds = 0;       // dynamic LDS of the binary kernels (the largest page need, from the plan pass)
  uint32_t zstd = 1;          // some page has a Zstd stream (0: the decode kernels without the Zstd decoder)
  uint32_t patas = 1;         // some page has a Patas stream (0: no k_patas ahead of the inflate launches)
  uint32_t lz4like = 1;       // some page has an LZ4 / Snappy stream (k_inflate jobs beside the Patas ones)
  uint64_t values_bytes = 0;
  uint32_t n_staged = 0, n_global = 0;
  bool staged_identity = false;  // every page staged: no index list
  uint32_t stage_bytes = 0;
  bool validity_needs_zero = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timing = false;  // record HIP events around each decode (sb_plan_enable_timing)
  bool timed = false;
};

// k_inflate claims from one of the plan's two counter pairs and zeroes the
// other at entry; the pairs alternate per launch (see InflateLaunch::sched_spare)
static void sched_pair(sb_plan* p, sb::InflateLaunch& I) {
  if (!p->d_sched || I.n_jobs == 0) return;
  const uint32_t f = p->sched_flip;
  p->sched_flip ^= 1u;
  I.sched = p->d_sched + 3 * f;
  I.sched_spare = p->d_sched + 3 * (f ^ 1u);
}

static sb_status fail(sb_ctx* ctx, sb_status st, const char* fmt, ...) {
  if (ctx) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    ctx->err = buf;
  }
  return st;
}

#define HIP_TRY(ctx, expr)                                                                  \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(ctx, SB_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

static int type_width(int t, bool* is_float) {
  *is_float = false;
  switch (t) {
    case SB_T_INT8: case SB_T_UINT8: return 1;
    case SB_T_INT16: case SB_T_UINT16: return 2;
    case SB_T_INT32: case SB_T_UINT32: return 4;
    case SB_T_INT64: case SB_T_UINT64: return 8;
    case SB_T_FLOAT32: *is_float = true; return 4;
    case SB_T_FLOAT64: *is_float = true; return 8;
  }
  return 0;
}

extern "C" {

const char* sb_status_str(int st) {
  switch (st) {
    case SB_OK: return "ok";
    case SB_E_OUT_OF_SPEC: return "out of spec";
    case SB_E_NYI: return "not yet implemented";
    case SB_E_IO: return "io (short read)";
    case SB_E_CODEC: return "codec error";
    case SB_E_DEVICE: return "device error";
    case SB_E_ARG: return "invalid argument";
  }
  return "unknown";
}

sb_status sb_ctx_create(int device, sb_ctx** out) {
  if (!out) return SB_E_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return SB_E_DEVICE;
  if (device < 0 || device >= n) return SB_E_ARG;
  sb_ctx* c = new sb_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SB_E_DEVICE;
  }
  c->stream = c->own;
  *out = c;
  return SB_OK;
}

void sb_ctx_destroy(sb_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (int i = 0; i < sb::kCtxScratchSlots; i++)
    if (ctx->scr[i]) {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipFree(ctx->scr[i]);
    }
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
}

sb_status sb_ctx_set_stream(sb_ctx* ctx, void* s) {
  if (!ctx) return SB_E_ARG;
  ctx->stream = (hipStream_t)s;  // taken literally: NULL is the legacy default stream
  return SB_OK;
}

void* sb_ctx_stream(sb_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int32_t sb_ctx_device(const sb_ctx* ctx) { return ctx ? ctx->device : -1; }

sb_status sb_sync(sb_ctx* ctx) {
  if (!ctx) return SB_E_ARG;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return SB_OK;
}

const char* sb_last_error(const sb_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void sb_plan_destroy(sb_plan* p) {
  if (!p) return;
  if (p->d_pages) (void)hipFree(p->d_pages);
  if (p->d_status) (void)hipFree(p->d_status);
  if (p->d_lists) (void)hipFree(p->d_lists);
  if (p->d_light) (void)hipFree(p->d_light);
  if (p->d_defer) (void)hipFree(p->d_defer);
  if (p->d_jobs) (void)hipFree(p->d_jobs);
  if (p->d_scratch) (void)hipFree(p->d_scratch);
  if (p->d_region) (void)hipFree(p->d_region);
  if (p->d_spill) (void)hipFree(p->d_spill);
  if (p->d_sched) (void)hipFree(p->d_sched);
  if (p->d_ascii) (void)hipFree(p->d_ascii);
  if (p->d_spill_jobs) (void)hipFree(p->d_spill_jobs);
  if (p->d_bin) (void)hipFree(p->d_bin);
  if (p->d_lb) (void)hipFree(p->d_lb);
  if (p->d_lc) (void)hipFree(p->d_lc);
  if (p->d_nest) (void)hipFree(p->d_nest);
  if (p->inner) sb_plan_destroy(p->inner);
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  delete p;
}

uint64_t sb_plan_num_rows(const sb_plan* p) { return p ? p->n_rows : 0; }
uint64_t sb_plan_num_pages(const sb_plan* p) { return p ? p->n_pages : 0; }

// The page table of a plan: page i at byte pages[i].byte_off of the chunk,
// rows [row_off, row_off + num_values) of the output (sb_plan_column: the
// running sums of the PageMeta; nested leaves: each page's values stream at
// its leaf base).
// Fixed-width page regions (plan_regions): none, sized from a plan-time
// probe of each large page's cascade, or sized conservatively from the page
// table alone (List values streams, whose descriptors the levels pass writes
// at decode time).
enum RegionMode { kRegionsNone = 0, kRegionsProbe = 1, kRegionsBySize = 2 };

static sb_status plan_pages(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                            std::vector<sb::PageDesc> pages, sb_plan** out, int regions = kRegionsProbe);

static sb_status plan_column(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                             const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out, int regions);

sb_status sb_plan_column(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                         const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out) {
  return plan_column(ctx, desc, d_chunk, chunk_len, h_metas, n_pages, out, kRegionsProbe);
}

sb_status sb_plan_column_at(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                            const sb_page_meta* h_metas, uint64_t n_pages, const uint64_t* h_row_offsets,
                            sb_plan** out) {
  if (!ctx || !desc || !out || (n_pages && (!h_metas || !h_row_offsets))) return fail(ctx, SB_E_ARG, "null argument");
  if (n_pages > 0xFFFFFFFFull) return fail(ctx, SB_E_ARG, "too many pages");
  if (desc->physical_type >= SB_T_BINARY && desc->physical_type <= SB_T_LARGE_UTF8)
    return fail(ctx, SB_E_ARG, "binary columns are planned with sb_plan_column");
  std::vector<sb::PageDesc> pages(n_pages);
  uint64_t off = 0, end = 0;
  for (uint64_t i = 0; i < n_pages; i++) {
    const sb_page_meta& m = h_metas[i];
    if (m.length > 0xFFFFFFFFull || m.num_values > 0xFFFFFFFFull)
      return fail(ctx, SB_E_ARG, "page %llu exceeds u32 sizes", (unsigned long long)i);
    if (h_row_offsets[i] < end) return fail(ctx, SB_E_ARG, "page %llu overlaps the rows before it", (unsigned long long)i);
    pages[i] = sb::PageDesc{off, h_row_offsets[i], (uint32_t)m.length, (uint32_t)m.num_values, 0};
    off += m.length;
    end = h_row_offsets[i] + m.num_values;
  }
  return plan_pages(ctx, desc, d_chunk, chunk_len, std::move(pages), out, kRegionsProbe);
}

static sb_status plan_column(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                             const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out, int regions) {
  if (!ctx || !desc || !out || (!h_metas && n_pages)) return fail(ctx, SB_E_ARG, "null argument");
  if (n_pages > 0xFFFFFFFFull) return fail(ctx, SB_E_ARG, "too many pages");
  std::vector<sb::PageDesc> pages(n_pages);
  uint64_t off = 0, rows = 0;
  for (uint64_t i = 0; i < n_pages; i++) {
    const sb_page_meta& m = h_metas[i];
    if (m.length > 0xFFFFFFFFull || m.num_values > 0xFFFFFFFFull)
      return fail(ctx, SB_E_ARG, "page %llu exceeds u32 sizes", (unsigned long long)i);
    pages[i] = sb::PageDesc{off, rows, (uint32_t)m.length, (uint32_t)m.num_values, 0};
    off += m.length;
    rows += m.num_values;
  }
  return plan_pages(ctx, desc, d_chunk, chunk_len, std::move(pages), out, regions);
}

// HBM regions of a fixed-width plan's large pages (PageDesc.reserved): the
// roaring tables of a Freq page that can hold more containers than the LDS
// tables (num_values > 4 bitmap containers' worth), and the area a Dict /
// Freq cascade's general-codec leaf expands into when page + expansion
// exceed the deferred pass's LDS.  Probed pages get only what their cascade
// needs; by-size pages get both.
static hipError_t plan_regions(sb_ctx* ctx, sb_plan* p, std::vector<sb::PageDesc>& pages, int mode) {
  std::vector<uint32_t> cand;
  const uint64_t W = (uint64_t)p->width;
  auto roar_cand = [](const sb::PageDesc& pd) { return pd.num_values > 4u * 4096u; };
  auto spill_cand = [&](const sb::PageDesc& pd) {
    return sb::align16((uint64_t)pd.byte_len + 15 + sb::kStagePad) + sb::spill_area_bytes(pd.num_values, W) +
               sb::kZTablesMax + 64 > sb::kDeferredLds;
  };
  for (uint32_t i = 0; i < (uint32_t)pages.size(); i++)
    if (roar_cand(pages[i]) || spill_cand(pages[i])) cand.push_back(i);
  if (cand.empty()) return hipSuccess;
  std::vector<uint32_t> bits(cand.size(), 7u);
  hipError_t e = hipSuccess;
  if (mode == kRegionsProbe) {
    uint32_t* d = nullptr;
    e = hipMalloc(&d, 2 * cand.size() * sizeof(uint32_t));
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(d, cand.data(), cand.size() * 4, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && sb::launch_fix_probe(p->d_chunk, p->d_pages, d, (uint32_t)cand.size(), p->width,
                                                p->desc.nullable, d + cand.size(), ctx->stream))
      e = hipErrorLaunchFailure;
    if (e == hipSuccess) e = hipMemcpyAsync(bits.data(), d + cand.size(), cand.size() * 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return e;
  }
  uint64_t off = 0;
  uint32_t n_spill = 0;
  for (size_t j = 0; j < cand.size(); j++) {
    sb::PageDesc& pd = pages[cand[j]];
    uint64_t flags = 0, size = 0;
    if (roar_cand(pd) && (bits[j] & 1)) {
      flags |= sb::kRegionRoar;
      size += sb::roar_area_bytes(pd.num_values);
    }
    if (spill_cand(pd) && (bits[j] & 2) && (bits[j] & 4)) {  // (a plain general leaf goes to k_inflate / k_zinflate)
      flags |= sb::kRegionSpill;
      size += sb::spill_area_bytes(pd.num_values, W);
      n_spill++;
    }
    if (flags) {
      pd.reserved = off | flags;
      off += size;
    }
  }
  if (!off) return hipSuccess;
  e = hipMalloc(&p->d_region, off);
  if (e == hipSuccess && n_spill) e = hipMalloc(&p->d_spill, 2 * sizeof(uint32_t));
  if (e == hipSuccess && n_spill) e = hipMemsetAsync(p->d_spill, 0, 2 * sizeof(uint32_t), ctx->stream);
  if (e == hipSuccess && n_spill) e = hipMalloc(&p->d_spill_jobs, n_spill * sizeof(sb::InflateJob));
  if (e == hipSuccess)
    e = hipMemcpyAsync(p->d_pages, pages.data(), pages.size() * sizeof(sb::PageDesc), hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  p->n_spill = n_spill;
  return e;
}

// LDS a staged Boolean page takes in k_bool_decode: the page, its expanded
// bitmap and the Zstd decoder's tables.
static uint64_t bool_lds_need(uint64_t len, uint64_t n, bool zstd = true) {
  return ((len + 15 + sb::kStagePad + 15) & ~15ull) + (((n + 7) / 8 + 15) & ~15ull) + sb::kStagePad +
         (zstd ? sb::kZTablesBytes : 0);
}

// Boolean pages too large for that (max_page_size = None: one page per
// chunk) decode from HBM (k_bool_decode's big-page path) and expand RLE /
// general-codec bitmaps into a region of their own: the page's bitmap words
// plus 16 bytes of over-read slack.
static hipError_t plan_bool_regions(sb_ctx* ctx, sb_plan* p, std::vector<sb::PageDesc>& pages) {
  uint64_t off = 0;
  for (sb::PageDesc& pd : pages) {
    if (bool_lds_need(pd.byte_len, pd.num_values) <= sb::kDeferredLds) continue;
    pd.reserved = off | sb::kRegionSpill;
    off += sb::align16(4 * (((uint64_t)pd.num_values + 31) / 32)) + 16;
  }
  if (!off) return hipSuccess;
  hipError_t e = hipMalloc(&p->d_region, off);
  if (e == hipSuccess)
    e = hipMemcpyAsync(p->d_pages, pages.data(), pages.size() * sizeof(sb::PageDesc), hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  return e;
}

static sb_status plan_pages(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                            std::vector<sb::PageDesc> pages, sb_plan** out, int regions) {
  const uint64_t n_pages = pages.size();
  bool is_float;
  int width = type_width(desc->physical_type, &is_float);
  const int ptype = desc->physical_type;
  const int owidth = (ptype == SB_T_BINARY || ptype == SB_T_UTF8) ? 4
                     : (ptype == SB_T_LARGE_BINARY || ptype == SB_T_LARGE_UTF8) ? 8 : 0;
  const bool is_bool = ptype == SB_T_BOOLEAN;
  if (!width && !owidth && !is_bool) return fail(ctx, SB_E_NYI, "physical type %d not supported", desc->physical_type);
  if (n_pages > 0xFFFFFFFFull) return fail(ctx, SB_E_ARG, "too many pages");
  HIP_TRY(ctx, hipSetDevice(ctx->device));

  std::vector<uint32_t> staged, global;
  uint64_t rows = 0;
  uint32_t max_stage = 0, max_bool = 0, max_bool_noz = 0;
  bool needs_zero = false;
  for (uint64_t i = 0; i < n_pages; i++) {
    const sb::PageDesc& pd = pages[i];
    const sb_page_meta m{pd.byte_len, pd.num_values};
    if (pd.byte_off + m.length > chunk_len)
      return fail(ctx, SB_E_ARG, "page %llu overruns the column chunk", (unsigned long long)i);
    // a 32-bit validity word shared by two pages is merged with atomics
    if ((pd.row_off & 31) || (m.num_values & 31)) needs_zero = true;
    if (is_bool)  // page + its expanded bitmap, as k_bool_decode lays them out in LDS (big pages: all of it)
      max_bool = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(max_bool, bool_lds_need(m.length, m.num_values)),
                                              sb::kDeferredLds);
    if (is_bool)
      max_bool_noz = (uint32_t)std::min<uint64_t>(
          std::max<uint64_t>(max_bool_noz, bool_lds_need(m.length, m.num_values, false)), sb::kDeferredLds);
    if (m.length + 16 <= sb::kStageMaxBytes) {
      staged.push_back((uint32_t)i);
      max_stage = std::max<uint32_t>(max_stage, (uint32_t)m.length);
    } else {
      global.push_back((uint32_t)i);
    }
    rows = std::max<uint64_t>(rows, pd.row_off + m.num_values);
  }

  sb_plan* p = new sb_plan();
  p->desc = *desc;
  p->d_chunk = d_chunk;
  p->chunk_len = chunk_len;
  p->n_pages = n_pages;
  p->n_rows = rows;
  p->width = width;
  p->is_float = is_float;
  p->n_staged = (uint32_t)staged.size();
  p->n_global = (uint32_t)global.size();
  p->staged_identity = global.empty();
  p->stage_bytes = ((max_stage + 16 + 15) & ~15u) + sb::kStagePad;
  p->validity_needs_zero = needs_zero;
  p->binary = owidth != 0;
  p->boolean = is_bool;
  if (is_bool) p->stage_bytes = std::max<uint32_t>(max_bool, 64);
  p->offset_width = owidth;
  size_t np = n_pages ? n_pages : 1;
  hipError_t e = hipMalloc(&p->d_pages, np * sizeof(sb::PageDesc));
  if (e == hipSuccess) e = hipMalloc(&p->d_status, np * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&p->d_lists, np * sizeof(uint32_t));
  if (e == hipSuccess && !owidth && !is_bool) e = hipMalloc(&p->d_light, np * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&p->d_defer, (np + 4) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(p->d_defer, 0, 4 * sizeof(uint32_t), ctx->stream);
  if (e == hipSuccess) e = hipMalloc(&p->d_jobs, (owidth ? 2 : 1) * np * sizeof(sb::InflateJob));
  if (e == hipSuccess) e = hipMalloc(&p->d_sched, 6 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(p->d_sched, 0, 6 * sizeof(uint32_t), ctx->stream);
  if (e == hipSuccess) e = hipEventCreate(&p->ev0);
  if (e == hipSuccess) e = hipEventCreate(&p->ev1);
  if (e == hipSuccess && n_pages) {
    std::vector<uint32_t> lists(staged);
    lists.insert(lists.end(), global.begin(), global.end());
    e = hipMemcpyAsync(p->d_pages, pages.data(), n_pages * sizeof(sb::PageDesc), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(p->d_lists, lists.data(), n_pages * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(p->d_status, 0, n_pages * sizeof(uint32_t), ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);  // host vectors go out of scope
  }
  if (e != hipSuccess) {
    sb_plan_destroy(p);
    return fail(ctx, SB_E_DEVICE, "plan upload: %s", hipGetErrorString(e));
  }
  if (!owidth && n_pages) {  // any Zstd stream?  (binary plans learn it from their probe below)
    uint32_t* d_flag = nullptr;
    uint32_t flag = 1;
    e = hipMalloc(&d_flag, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(d_flag, 0, sizeof(uint32_t), ctx->stream);
    if (e == hipSuccess && sb::launch_zstd_scan(d_chunk, p->d_pages, (uint32_t)n_pages, is_bool ? 1 : width,
                                                desc->nullable, d_flag, ctx->stream))
      e = hipErrorLaunchFailure;
    if (e == hipSuccess) e = hipMemcpyAsync(&flag, d_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (d_flag) (void)hipFree(d_flag);
    if (e != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan zstd scan: %s", hipGetErrorString(e));
    }
    p->zstd = (flag & 1) ? 1 : 0;
    p->patas = (flag & 2) ? 1 : 0;
    p->lz4like = (flag & 4) ? 1 : 0;
    if (is_bool && !p->zstd) p->stage_bytes = std::max<uint32_t>(max_bool_noz, 64);
  }
  if (is_bool && n_pages) {
    e = plan_bool_regions(ctx, p, pages);
    if (e != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "boolean plan regions: %s", hipGetErrorString(e));
    }
  }
  if (regions != kRegionsNone && !owidth && !is_bool && n_pages) {
    e = plan_regions(ctx, p, pages, regions);
    if (e != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan regions: %s", hipGetErrorString(e));
    }
  }
  if (p->d_light && n_pages) {
    // Classify once: the per-decode classify pass (one thread per page) runs
    // only for chunks that hold header-only pages; the staged pass handles
    // every page correctly either way.
    sb::LaunchArgs c{};
    c.chunk = d_chunk;
    c.pages = p->d_pages;
    c.nullable = desc->nullable;
    c.status = p->d_status;
    c.job_count = p->d_defer + 2;
    c.jobs = p->d_jobs;
    uint32_t n_light = 0;
    e = sb::launch_fix_light(c, (uint32_t)n_pages, width, is_float, p->d_light, ctx->stream) ? hipErrorUnknown
                                                                                              : hipSuccess;
    if (e == hipSuccess) e = hipMemcpyAsync(&n_light, p->d_defer + 2, 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(p->d_defer, 0, 4 * sizeof(uint32_t), ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan classify: %s", hipGetErrorString(e));
    }
    if (!n_light) {
      (void)hipFree(p->d_light);
      p->d_light = nullptr;
    } else {  // any Zstd leaves too large for the deferred pass?  (k_zinflate is launched only then)
      std::vector<sb::InflateJob> jobs(n_light);
      if (hipMemcpy(jobs.data(), p->d_jobs, n_light * sizeof(sb::InflateJob), hipMemcpyDeviceToHost) == hipSuccess)
        for (const auto& j : jobs) p->has_zstd_big |= j.codec == 2;
    }
  }
  if (p->binary && n_pages) {  // size every page's values once: they are fixed for the plan
    e = hipMalloc(&p->d_bin, (2 * np + 2) * sizeof(uint64_t) + (4 * np + 3) * sizeof(uint32_t));
    if (e != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan alloc: %s", hipGetErrorString(e));
    }
    uint32_t* cls = (uint32_t*)(p->d_bin + 2 * np + 2);
    // Probe: the LDS each page's staged decode needs; Extend pages that need
    // more than one workgroup's LDS become big pages with an HBM region
    {
      uint32_t* d_need = nullptr;
      uint64_t* d_rneed = nullptr;
      std::vector<uint32_t> need(n_pages);
      std::vector<uint64_t> rneed(n_pages);
      uint64_t zflag = 1;  // the probe ORs bit 0 for a page with a Zstd stream (into the total's slot)
      e = hipMalloc(&d_need, np * sizeof(uint32_t));
      if (e == hipSuccess) e = hipMalloc(&d_rneed, np * sizeof(uint64_t));
      if (e == hipSuccess) e = hipMemsetAsync(p->d_bin + 2 * np, 0, sizeof(uint64_t), ctx->stream);
      if (e == hipSuccess) {
        sb::BinLaunch P{d_chunk, p->d_pages, (uint32_t)n_pages, desc->nullable, nullptr, nullptr, p->d_bin + 2 * np,
                        nullptr, nullptr, 0, nullptr, p->d_status, nullptr, nullptr, nullptr, 0, d_need, cls, 1,
                        nullptr, d_rneed, 0};
        if (sb::launch_binary(2, owidth, P, ctx->stream)) e = hipErrorLaunchFailure;
      }
      if (e == hipSuccess) e = hipMemcpyAsync(need.data(), d_need, n_pages * 4, hipMemcpyDeviceToHost, ctx->stream);
      if (e == hipSuccess) e = hipMemcpyAsync(rneed.data(), d_rneed, n_pages * 8, hipMemcpyDeviceToHost, ctx->stream);
      if (e == hipSuccess) e = hipMemcpyAsync(&zflag, p->d_bin + 2 * np, 8, hipMemcpyDeviceToHost, ctx->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
      p->zstd = (zflag & 1) ? 1 : 0;
      if (d_need) (void)hipFree(d_need);
      if (d_rneed) (void)hipFree(d_rneed);
      uint64_t off = 0;
      uint32_t max_need = 0;
      for (uint64_t i = 0; i < n_pages && e == hipSuccess; i++) {
        if (need[i] > sb::kDeferredLds && rneed[i]) {
          pages[i].reserved = off + 1;
          off += sb::align16(rneed[i]);
          p->n_big++;
        } else {
          max_need = std::max(max_need, need[i]);
        }
      }
      p->bin_lds = std::min<uint32_t>(std::max<uint32_t>((max_need + 1023) & ~1023u, 4096), sb::kDeferredLds);
      if (e == hipSuccess && off) e = hipMalloc(&p->d_region, off);
      if (e == hipSuccess && off)
        e = hipMemcpyAsync(p->d_pages, pages.data(), n_pages * sizeof(sb::PageDesc), hipMemcpyHostToDevice, ctx->stream);
      if (e != hipSuccess) {
        sb_plan_destroy(p);
        return fail(ctx, SB_E_DEVICE, "binary plan probe: %s", hipGetErrorString(e));
      }
    }
    sb::BinLaunch L{d_chunk, p->d_pages, (uint32_t)n_pages, desc->nullable, p->d_bin, p->d_bin + np,
                    p->d_bin + 2 * np, nullptr, nullptr, 0, nullptr, p->d_status, p->d_jobs, p->d_defer + 2, nullptr,
                    p->bin_lds, nullptr, cls, (uint32_t)std::min<size_t>(np, 65535), p->d_region, nullptr, p->n_big};
    L.zstd = p->zstd;
    if (sb::launch_binary(0, owidth, L, ctx->stream) || hipStreamSynchronize(ctx->stream) != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "binary sizing failed: %s", hipGetErrorString(hipGetLastError()));
    }
    std::vector<uint32_t> st(n_pages);
    (void)hipMemcpy(st.data(), p->d_status, n_pages * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&p->values_bytes, p->d_bin + 2 * np, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&p->n_bin_jobs, p->d_defer + 2, 4, hipMemcpyDeviceToHost);
    if (p->n_bin_jobs) {  // streams of big Zstd Basic pages (k_zinflate)
      std::vector<sb::InflateJob> jobs(p->n_bin_jobs);
      if (hipMemcpy(jobs.data(), p->d_jobs, jobs.size() * sizeof(sb::InflateJob), hipMemcpyDeviceToHost) == hipSuccess)
        for (const auto& j : jobs) p->has_zstd_big |= j.codec == 2;
    }
    uint32_t n_staged = 0;
    (void)hipMemcpy(&n_staged, cls + 4 * np, 4, hipMemcpyDeviceToHost);
    p->bin_grid = std::max<uint32_t>(1, std::min<uint32_t>(n_staged, 65535));
    for (uint64_t i = 0; i < n_pages; i++) {
      if (st[i]) {
        sb_plan_destroy(p);
        return fail(ctx, (sb_status)st[i], "page %llu: %s", (unsigned long long)i, sb_status_str((int)st[i]));
      }
    }
    if (p->n_bin_jobs && hipMalloc(&p->d_scratch, (rows + n_pages) * (uint64_t)owidth) != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan alloc: scratch");
    }
    // the pages whose values stream k_inflate expands are the same every
    // decode; it rewrites their flags each time, the rest stay 0 (scanned)
    if (p->n_bin_jobs && (hipMalloc(&p->d_ascii, n_pages) != hipSuccess ||
                          hipMemsetAsync(p->d_ascii, 0, n_pages, ctx->stream) != hipSuccess)) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan alloc: ascii flags");
    }
    // every page staged (no header-only or big pages): one fused pass sizes,
    // bases and decodes them (k_bin_fused)
    if (n_staged == n_pages && !p->n_big && !p->n_bin_jobs && !getenv("SB_NO_BIN_FUSED") &&
        hipMalloc(&p->d_lb, (n_pages + 1) * sizeof(uint64_t)) != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan alloc: look-back");
    }
    // Utf8 through the fused pass: it flags the pages whose emitted rows are
    // whole, valid entries (OneValue / Dict / Freq), and the check skips them
    const bool utf8 = desc->physical_type == SB_T_UTF8 || desc->physical_type == SB_T_LARGE_UTF8;
    if (p->d_lb && utf8 && !getenv("SB_NO_ENTRY_UTF8") &&
        (hipMalloc(&p->d_ascii, n_pages) != hipSuccess || hipMemsetAsync(p->d_ascii, 0, n_pages, ctx->stream) != hipSuccess)) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "plan alloc: entry flags");
    }
  }
  *out = p;
  return SB_OK;
}

uint64_t sb_plan_values_bytes(const sb_plan* p) { return p ? p->values_bytes : 0; }

sb_status sb_decode_binary_planned(sb_ctx* ctx, sb_plan* p, const sb_binary_out* out) {
  if (!ctx || !p || !out) return fail(ctx, SB_E_ARG, "null argument");
  if (!p->binary) return fail(ctx, SB_E_ARG, "not a binary plan");
  if (!out->d_offsets || (p->values_bytes && (!out->d_values || out->values_capacity < p->values_bytes)))
    return fail(ctx, SB_E_ARG, "binary output buffers too small");
  if (p->desc.nullable && p->n_rows && !out->d_validity) return fail(ctx, SB_E_ARG, "validity buffer is null");
  if ((uintptr_t)out->d_offsets % p->offset_width) return fail(ctx, SB_E_ARG, "offsets buffer is not aligned");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (p->desc.nullable && p->validity_needs_zero)
    HIP_TRY(ctx, hipMemsetAsync(out->d_validity, 0, (p->n_rows + 31) / 32 * 4, ctx->stream));
  if (!p->n_pages) return SB_OK;
  if (p->timing) HIP_TRY(ctx, hipEventRecord(p->ev0, ctx->stream));
  const size_t np = p->n_pages;
  if (p->d_lb) {  // every page staged: sizes, bases and rows in one pass
    sb::BinLaunch F{p->d_chunk, p->d_pages, (uint32_t)np, p->desc.nullable, p->d_bin, p->d_bin + np,
                    p->d_bin + 2 * np, (uint8_t*)out->d_offsets, out->d_values, out->values_capacity,
                    (uint32_t*)out->d_validity, p->d_status, p->d_jobs, nullptr, p->d_scratch, p->bin_lds, nullptr,
                    (uint32_t*)(p->d_bin + 2 * np + 2), p->bin_grid, p->d_region, nullptr, p->n_big, p->d_lb};
    F.zstd = p->zstd;
    F.checked = p->d_ascii;
    if (sb::launch_binary(3, p->offset_width, F, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "binary decode launch failed: %s", hipGetErrorString(hipGetLastError()));
  } else {
  // Every decode sizes its pages again (values bytes -> bases, and the list of
  // LZ4 / Snappy streams): the plan-time pass only sized the caller's buffers.
  HIP_TRY(ctx, hipMemsetAsync(p->d_defer + 2, 0, sizeof(uint32_t), ctx->stream));
  sb::BinLaunch S{p->d_chunk, p->d_pages, (uint32_t)np, p->desc.nullable, p->d_bin, p->d_bin + np, p->d_bin + 2 * np,
                  nullptr, nullptr, 0, nullptr, p->d_status, p->d_jobs, p->d_defer + 2, nullptr, p->bin_lds, nullptr,
                  (uint32_t*)(p->d_bin + 2 * np + 2), p->bin_grid, p->d_region, nullptr, p->n_big};
  S.zstd = p->zstd;
  if (sb::launch_binary(0, p->offset_width, S, ctx->stream))
    return fail(ctx, SB_E_DEVICE, "binary sizing launch failed: %s", hipGetErrorString(hipGetLastError()));
  sb::BinLaunch L{p->d_chunk, p->d_pages, (uint32_t)np, p->desc.nullable, p->d_bin, p->d_bin + np, p->d_bin + 2 * np,
                  (uint8_t*)out->d_offsets, out->d_values, out->values_capacity, (uint32_t*)out->d_validity,
                  p->d_status, p->d_jobs, nullptr, p->d_scratch, p->bin_lds, nullptr, (uint32_t*)(p->d_bin + 2 * np + 2),
                  p->bin_grid, p->d_region, nullptr, p->n_big};
  if (p->n_bin_jobs) {  // Basic LZ4 / Snappy pages: streams expanded first, one wave each
    sb::InflateLaunch I{p->d_chunk, p->d_jobs, p->d_defer + 2, p->n_bin_jobs, out->d_values, p->d_scratch,
                        p->d_bin + np, p->d_status, (uint8_t*)out->d_offsets, p->d_sched, p->d_ascii};
    sched_pair(p, I);
    if (sb::launch_inflate(I, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "inflate launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (p->has_zstd_big && sb::launch_zinflate(I, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "zstd inflate launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  L.zstd = p->zstd;
  if (sb::launch_binary(1, p->offset_width, L, ctx->stream))
    return fail(ctx, SB_E_DEVICE, "binary decode launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  if (p->desc.physical_type == SB_T_UTF8 || p->desc.physical_type == SB_T_LARGE_UTF8) {
    // Utf8Array::try_new (read/array/binary.rs:305-306): invalid UTF-8 or an
    // offset inside a character is OutOfSpec for the page that holds it
    uint32_t* flags = (uint32_t*)(p->d_bin + 2 * np + 1);
    HIP_TRY(ctx, hipMemsetAsync(flags, 0, sizeof(uint32_t), ctx->stream));
    sb::Utf8Launch U{out->d_values, p->values_bytes, (const uint8_t*)out->d_offsets, p->n_rows, p->d_pages,
                     (uint32_t)np, p->d_bin + np, p->d_status, flags, p->d_ascii};
    if (sb::launch_utf8_check(p->offset_width, U, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "utf8 check launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  if (p->timing) {
    HIP_TRY(ctx, hipEventRecord(p->ev1, ctx->stream));
    p->timed = true;
  }
  return SB_OK;
}

sb_status sb_decode_planned(sb_ctx* ctx, sb_plan* p, const sb_primitive_out* out) {
  if (!ctx || !p || !out) return fail(ctx, SB_E_ARG, "null argument");
  if (p->binary) return fail(ctx, SB_E_ARG, "binary plan: use sb_decode_binary_planned");
  if (p->n_rows && !out->d_values) return fail(ctx, SB_E_ARG, "values buffer is null");
  if (p->desc.nullable && p->n_rows && !out->d_validity) return fail(ctx, SB_E_ARG, "validity buffer is null");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (p->desc.nullable && p->validity_needs_zero)
    HIP_TRY(ctx, hipMemsetAsync(out->d_validity, 0, (p->n_rows + 31) / 32 * 4, ctx->stream));
  if (p->boolean && p->validity_needs_zero)  // the values bitmap shares words across pages too
    HIP_TRY(ctx, hipMemsetAsync(out->d_values, 0, (p->n_rows + 31) / 32 * 4, ctx->stream));
  if (p->timing) HIP_TRY(ctx, hipEventRecord(p->ev0, ctx->stream));
  sb::LaunchArgs a{};
  a.zstd = p->zstd;
  a.chunk = p->d_chunk;
  a.pages = p->d_pages;
  a.out_values = (uint8_t*)out->d_values;
  a.out_validity = (uint32_t*)out->d_validity;
  a.nullable = p->desc.nullable;
  a.status = p->d_status;
  a.stage_bytes = p->stage_bytes;
  a.defer_count = p->d_defer;
  a.job_count = p->d_defer + 2;
  a.defer_list = p->d_defer + 4;
  a.jobs = p->d_jobs;
  a.region = p->d_region;
  a.spill_count = p->d_spill;
  a.spill_jobs = p->d_spill_jobs;
  a.parity = (uint32_t)(p->decodes & 1);
  p->decodes++;
  if (p->boolean) {
    a.list = nullptr;
    a.n_list = (uint32_t)p->n_pages;
    if (sb::launch_bool(a, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "boolean decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (p->timing) {
      HIP_TRY(ctx, hipEventRecord(p->ev1, ctx->stream));
      p->timed = true;
    }
    return SB_OK;
  }
  if (p->d_light) {  // header-only pages: inflate jobs without staging
    if (sb::launch_fix_light(a, (uint32_t)p->n_pages, p->width, p->is_float, p->d_light, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "page classify launch failed: %s", hipGetErrorString(hipGetLastError()));
    a.light = p->d_light;
  }
  a.list = p->staged_identity ? nullptr : p->d_lists;
  a.n_list = p->n_staged;
  if (sb::launch_decode_fixed(p->width, p->is_float, 0, a, ctx->stream))
    return fail(ctx, SB_E_DEVICE, "staged decode launch failed: %s", hipGetErrorString(hipGetLastError()));
  a.list = p->d_lists + p->n_staged;
  a.n_list = p->n_global;
  if (sb::launch_decode_fixed(p->width, p->is_float, 1, a, ctx->stream))
    return fail(ctx, SB_E_DEVICE, "global decode launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (p->inflate_state != 0 && p->n_pages) {
    // CH_LEAF LZ4 / Snappy pages listed by the pass above: values straight into the column
    sb::InflateLaunch I{p->d_chunk, p->d_jobs, p->d_defer + 2 + a.parity, (uint32_t)p->n_pages,
                        (uint8_t*)out->d_values, nullptr, nullptr, p->d_status, nullptr, p->d_sched};
    sched_pair(p, I);
    static const bool no_patas_wg = getenv("SB_NO_PATAS_WG") != nullptr;  // A/B: the one-wave Patas decoder
    // k_patas when the plan has no LZ4 / Snappy jobs: those are latency-bound
    // one-wave jobs, and one-wave Patas jobs in the same k_inflate launch
    // overlap them for free, where k_patas (a CU a workgroup) ahead of them
    // adds its time, and beside them on a second stream found no CU free
    // (C5's Float64 group with an LZ4 column: 1.39 / 1.38 vs 1.01 ms)
    I.patas_wg = p->is_float && p->patas && !p->lz4like && !no_patas_wg ? 1u : 0u;
    if (sb::launch_inflate(I, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "inflate launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (p->has_zstd_big && sb::launch_zinflate(I, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "zstd inflate launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  if (p->deferred_state != 0 && p->n_pages) {
    // pages whose leaf stream is LZ4 / Zstd / Snappy / Patas, listed by the pass above
    a.list = nullptr;
    a.n_list = (uint32_t)std::min<uint64_t>(p->n_pages, sb::kDeferredGrid);
    a.stage_bytes = sb::kDeferredLds;
    if (sb::launch_decode_fixed(p->width, p->is_float, 2, a, ctx->stream))
      return fail(ctx, SB_E_DEVICE, "deferred decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (p->n_spill) {
      // leaves the deferred pass could not hold in LDS: expanded into the
      // pages' regions (one wave per stream), then the pages decoded from there
      sb::InflateLaunch I{p->d_chunk, p->d_spill_jobs, p->d_spill + a.parity, p->n_spill, nullptr, p->d_region,
                          nullptr, p->d_status, nullptr, p->d_sched};
      sched_pair(p, I);
      if (sb::launch_inflate(I, ctx->stream) || sb::launch_zinflate(I, ctx->stream))
        return fail(ctx, SB_E_DEVICE, "spill inflate launch failed: %s", hipGetErrorString(hipGetLastError()));
      a.n_list = p->n_spill;
      if (sb::launch_decode_fixed(p->width, p->is_float, 3, a, ctx->stream))
        return fail(ctx, SB_E_DEVICE, "spilled decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
  }
  if (p->timing) {
    HIP_TRY(ctx, hipEventRecord(p->ev1, ctx->stream));
    p->timed = true;
  }
  return SB_OK;
}

sb_status sb_plan_status(sb_ctx* ctx, sb_plan* p, int64_t* bad) {
  if (!ctx || !p) return fail(ctx, SB_E_ARG, "null argument");
  if ((p->list || p->nested) && p->inner) {  // levels first, then the values streams
    const bool l = p->list, n = p->nested;
    p->list = p->nested = false;
    sb_status st = sb_plan_status(ctx, p, bad);
    p->list = l;
    p->nested = n;
    if (st) return st;
    return sb_plan_status(ctx, p->inner, bad);
  }
  if (bad) *bad = -1;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (!p->n_pages) return SB_OK;
  std::vector<uint32_t> st(p->n_pages);
  HIP_TRY(ctx, hipMemcpy(st.data(), p->d_status, p->n_pages * 4, hipMemcpyDeviceToHost));
  if (!p->binary && !p->boolean && p->decodes && (p->deferred_state == -1 || p->inflate_state == -1)) {
    // the plan's pages are fixed: learn once which passes they need
    uint32_t cnt[4] = {0, 0, 0, 0};
    HIP_TRY(ctx, hipMemcpy(cnt, p->d_defer, sizeof cnt, hipMemcpyDeviceToHost));
    const uint32_t par = (uint32_t)((p->decodes - 1) & 1);
    p->deferred_state = cnt[par] ? 1 : 0;
    p->inflate_state = cnt[2 + par] ? 1 : 0;
  }
  for (uint64_t i = 0; i < p->n_pages; i++) {
    if (st[i]) {
      if (bad) *bad = (int64_t)i;
      return fail(ctx, (sb_status)st[i], "page %llu: %s", (unsigned long long)i, sb_status_str((int)st[i]));
    }
  }
  return SB_OK;
}

// List state (u64 units): [counts n | block-local bases 2n | block totals
// 2 nblk | totals 2 | level descriptors 4n]
static uint64_t list_nblk(uint64_t n) { return (n + 255) / 256; }
static size_t list_state_bytes(uint64_t n) { return (3 * n + 2 * list_nblk(n) + 2 + 4 * n) * sizeof(uint64_t); }
static uint64_t* list_totals(sb_plan* p) { return (uint64_t*)p->d_lc + 3 * p->n_pages + 2 * list_nblk(p->n_pages); }

static sb_status list_launch(sb_ctx* ctx, sb_plan* p, const sb_list_out* out, int stage, bool peek) {
  const uint64_t n = p->n_pages;
  uint64_t* b = (uint64_t*)p->d_lc;
  uint64_t* tot = list_totals(p);
  sb::ListLaunch L{p->d_chunk, p->d_pages, (uint32_t)n, (uint32_t)p->ldesc.list_nullable,
                   (uint32_t)p->ldesc.item_nullable, (uint32_t)p->ldesc.offset_width, (uint32_t)p->width,
                   peek ? 1u : 0u, b, b + n, b + 3 * n, tot, tot + 2, p->inner->d_pages,
                   out ? (uint8_t*)out->d_offsets : nullptr, out ? (uint32_t*)out->d_list_validity : nullptr,
                   out ? (uint32_t*)out->d_leaf_validity : nullptr, p->d_status};
  L.epoch = p->list_epoch;
  if (sb::launch_list(stage, L, ctx->stream))
    return fail(ctx, SB_E_DEVICE, "list launch failed: %s", hipGetErrorString(hipGetLastError()));
  return SB_OK;
}

sb_status sb_plan_list_column(sb_ctx* ctx, const sb_list_desc* d, const uint8_t* d_chunk, uint64_t chunk_len,
                              const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out) {
  if (!ctx || !d || !out) return fail(ctx, SB_E_ARG, "null argument");
  bool is_float;
  if (!type_width(d->physical_type, &is_float)) return fail(ctx, SB_E_NYI, "list leaf type %d not supported", d->physical_type);
  if (d->offset_width != 4 && d->offset_width != 8) return fail(ctx, SB_E_ARG, "offset width must be 4 or 8");
  sb_column_desc cd{d->physical_type, 0};
  sb_plan* inner = nullptr;
  sb_status st = plan_column(ctx, &cd, d_chunk, chunk_len, h_metas, n_pages, &inner, kRegionsBySize);
  if (st) return st;
  // the inner plan's pages become the values streams only at decode time (its
  // plan-time Zstd scan read the list pages): keep the Zstd kernels
  inner->zstd = 1;
  sb_plan* p = new sb_plan();
  p->desc = cd;
  p->list = true;
  p->ldesc = *d;
  p->inner = inner;
  p->d_chunk = d_chunk;
  p->chunk_len = chunk_len;
  p->n_pages = n_pages;
  p->width = inner->width;
  p->is_float = is_float;
  const size_t np = n_pages ? n_pages : 1;
  hipError_t e = hipMalloc(&p->d_pages, np * sizeof(sb::PageDesc));
  if (e == hipSuccess) e = hipMalloc(&p->d_status, np * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&p->d_lc, list_state_bytes(np));
  if (e == hipSuccess) e = hipEventCreate(&p->ev0);
  if (e == hipSuccess) e = hipEventCreate(&p->ev1);
  if (e == hipSuccess && n_pages)  // the level pages (inner's table becomes the values streams)
    e = hipMemcpyAsync(p->d_pages, inner->d_pages, n_pages * sizeof(sb::PageDesc), hipMemcpyDeviceToDevice, ctx->stream);
  if (e == hipSuccess) e = hipMemsetAsync(p->d_lc, 0, list_state_bytes(np), ctx->stream);
  if (e != hipSuccess) {
    sb_plan_destroy(p);
    return fail(ctx, SB_E_DEVICE, "list plan alloc: %s", hipGetErrorString(e));
  }
  if (n_pages) {  // exact sizing once, so the caller can allocate the outputs
    if (list_launch(ctx, p, nullptr, 0, false) || hipStreamSynchronize(ctx->stream) != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "list sizing failed: %s", hipGetErrorString(hipGetLastError()));
    }
    std::vector<uint32_t> stv(n_pages);
    std::vector<uint64_t> exact(n_pages), peek(n_pages);
    (void)hipMemcpy(stv.data(), p->d_status, n_pages * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(exact.data(), p->d_lc, n_pages * 8, hipMemcpyDeviceToHost);
    if (std::find(stv.begin(), stv.end(), (uint32_t)sb::ST_NYI) != stv.end()) {
      // a level stream with more hybrid runs than k_list's run table holds
      // (writers other than the reference's mix RLE and bit-packed runs
      // freely; parquet2's HybridRleDecoder takes any number): the general
      // level walk (k_nest_walk, depth 1) decodes the same List
      sb_plan_destroy(p);
      sb_nested_desc nd{};
      nd.physical_type = d->physical_type;
      nd.depth = 1;
      nd.list_nullable[0] = d->list_nullable;
      nd.item_nullable = d->item_nullable;
      nd.offset_width = d->offset_width;
      sb_plan* w = nullptr;
      const sb_status wst = sb_plan_nested_column(ctx, &nd, d_chunk, chunk_len, h_metas, n_pages, &w);
      if (wst) return wst;
      w->list_walk = true;
      w->ldesc = *d;
      *out = w;
      return SB_OK;
    }
    for (uint64_t i = 0; i < n_pages; i++) {
      if (stv[i]) {
        sb_plan_destroy(p);
        return fail(ctx, (sb_status)stv[i], "page %llu: %s", (unsigned long long)i, sb_status_str((int)stv[i]));
      }
      p->n_rows += exact[i] >> 32;
      p->n_leaves += exact[i] & 0xFFFFFFFFull;
    }
    // Do the page headers (rows, values usize) give the same counts?  Then
    // decodes size from them instead of walking every level twice.
    if (list_launch(ctx, p, nullptr, 1, true) || hipStreamSynchronize(ctx->stream) != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "list sizing failed: %s", hipGetErrorString(hipGetLastError()));
    }
    (void)hipMemcpy(peek.data(), p->d_lc, n_pages * 8, hipMemcpyDeviceToHost);
    p->list_peek = peek == exact;
    if (!p->list_peek) (void)hipMemcpy(p->d_lc, exact.data(), n_pages * 8, hipMemcpyHostToDevice);
  }
  *out = p;
  return SB_OK;
}

uint64_t sb_plan_num_leaves(const sb_plan* p) { return p ? p->n_leaves : 0; }

sb_status sb_decode_list_planned(sb_ctx* ctx, sb_plan* p, const sb_list_out* out) {
  if (!ctx || !p || !out) return fail(ctx, SB_E_ARG, "null argument");
  if (p->list_walk) {  // planned on the general walk: the same buffers as level 0 + the leaf
    sb_nested_out no{};
    no.d_offsets[0] = out->d_offsets;
    no.d_validity[0] = out->d_list_validity;
    no.d_values = out->d_values;
    no.d_leaf_validity = out->d_leaf_validity;
    return sb_decode_nested_planned(ctx, p, &no);
  }
  if (!p->list) return fail(ctx, SB_E_ARG, "not a list plan");
  if (!out->d_offsets || (p->n_leaves && !out->d_values)) return fail(ctx, SB_E_ARG, "list output buffers are null");
  if (p->ldesc.list_nullable && p->n_rows && !out->d_list_validity) return fail(ctx, SB_E_ARG, "list validity is null");
  if (p->ldesc.item_nullable && p->n_leaves && !out->d_leaf_validity) return fail(ctx, SB_E_ARG, "leaf validity is null");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (p->timing) HIP_TRY(ctx, hipEventRecord(p->ev0, ctx->stream));
  if (!p->n_pages) {
    HIP_TRY(ctx, hipMemsetAsync(out->d_offsets, 0, (size_t)p->ldesc.offset_width, ctx->stream));
  } else {
    // sizes (exact pass, or the headers) and global bases in one launch, the
    // levels walk, then the values streams at their leaf bases.  (Measured
    // on C4 and not kept: the values decode beside the walk on a second
    // stream, 242 vs 214 us, the kernels contend for the same CUs; a walk
    // with one wave per 2048-level step, 113-119 vs 108 us.)
    sb_status lst = p->list_peek ? SB_OK : list_launch(ctx, p, out, 0, false);
    if (!lst) {  // sizes + bases in one launch, this decode's tag on the block totals
      p->list_epoch = (uint16_t)(p->list_epoch + 1) ? (uint16_t)(p->list_epoch + 1) : 1;
      lst = list_launch(ctx, p, out, 4, p->list_peek);
    }
    if (!lst) lst = list_launch(ctx, p, out, 2, p->list_peek);
    if (lst) return lst;
    sb_primitive_out vo{out->d_values ? out->d_values : out->d_offsets, nullptr};  // (no leaves: nothing written)
    sb_status st = sb_decode_planned(ctx, p->inner, &vo);
    if (st) return st;
  }
  if (p->timing) {
    HIP_TRY(ctx, hipEventRecord(p->ev1, ctx->stream));
    p->timed = true;
  }
  return SB_OK;
}

static sb_status nest_launch(sb_ctx* ctx, sb_plan* p, const sb_nested_out* out, int stage) {
  const uint64_t n = p->n_pages, D = (uint64_t)p->ndesc.depth;
  sb::NestLaunch L{};
  L.chunk = p->d_chunk;
  L.pages = p->d_pages;
  L.n_pages = (uint32_t)n;
  L.depth = (uint32_t)D;
  for (uint64_t d = 0; d < D; d++) L.nullable |= (p->ndesc.list_nullable[d] ? 1u : 0u) << d;
  L.nullable |= (p->ndesc.item_nullable ? 1u : 0u) << D;
  L.offset_width = (uint32_t)p->ndesc.offset_width;
  L.struct_mask = (uint32_t)p->ndesc.struct_mask;
  L.counts = p->d_nest;
  L.bases = p->d_nest + n * (D + 1);
  L.totals = p->d_nest + 2 * n * (D + 1);
  L.vpages = p->inner ? p->inner->d_pages : nullptr;
  L.vpos = p->d_nest ? (uint32_t*)(p->d_nest + 2 * n * (D + 1) + D + 1) : nullptr;
  if (out) {
    for (uint64_t d = 0; d < D; d++) {
      L.out_offsets[d] = (uint8_t*)out->d_offsets[d];
      L.out_validity[d] = (uint32_t*)out->d_validity[d];
    }
    L.out_leaf_validity = (uint32_t*)out->d_leaf_validity;
  }
  L.status = p->d_status;
  if (sb::launch_nest(stage, L, ctx->stream))
    return fail(ctx, SB_E_DEVICE, "nested launch failed: %s", hipGetErrorString(hipGetLastError()));
  return SB_OK;
}

sb_status sb_plan_nested_column(sb_ctx* ctx, const sb_nested_desc* d, const uint8_t* d_chunk, uint64_t chunk_len,
                                const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out) {
  if (!ctx || !d || !out || (!h_metas && n_pages)) return fail(ctx, SB_E_ARG, "null argument");
  const int t = d->physical_type;
  bool is_float;
  const bool leaf_bin = t == SB_T_BINARY || t == SB_T_UTF8 || t == SB_T_LARGE_BINARY || t == SB_T_LARGE_UTF8;
  if (!type_width(t, &is_float) && t != SB_T_BOOLEAN && !leaf_bin)
    return fail(ctx, SB_E_NYI, "nested leaf type %d not supported", t);
  if (d->depth < 1 || d->depth > SB_MAX_NEST) return fail(ctx, SB_E_NYI, "nesting depth %d not supported", d->depth);
  if (d->struct_mask < 0 || (d->struct_mask >> d->depth) != 0)
    return fail(ctx, SB_E_ARG, "struct mask 0x%x names nests past depth %d", (unsigned)d->struct_mask, d->depth);
  if (d->offset_width != 4 && d->offset_width != 8) return fail(ctx, SB_E_ARG, "offset width must be 4 or 8");
  if (n_pages > 0xFFFFFFFFull) return fail(ctx, SB_E_ARG, "too many pages");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  std::vector<sb::PageDesc> lpages(n_pages);  // the level pages, back to back
  uint64_t off = 0;
  for (uint64_t i = 0; i < n_pages; i++) {
    if (h_metas[i].length > 0xFFFFFFFFull || h_metas[i].num_values > 0xFFFFFFFFull || off + h_metas[i].length > chunk_len)
      return fail(ctx, SB_E_ARG, "page %llu: bad size", (unsigned long long)i);
    lpages[i] = sb::PageDesc{off, 0, (uint32_t)h_metas[i].length, (uint32_t)h_metas[i].num_values, 0};
    off += h_metas[i].length;
  }
  sb_plan* p = new sb_plan();
  p->desc = sb_column_desc{t, 0};
  p->nested = true;
  p->ndesc = *d;
  p->d_chunk = d_chunk;
  p->chunk_len = chunk_len;
  p->n_pages = n_pages;
  p->is_float = is_float;
  const uint64_t D = (uint64_t)d->depth, np = n_pages ? n_pages : 1;
  hipError_t e = hipMalloc(&p->d_pages, np * sizeof(sb::PageDesc));
  if (e == hipSuccess) e = hipMalloc(&p->d_status, np * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&p->d_nest, (2 * np * (D + 1) + D + 1) * sizeof(uint64_t) + np * sizeof(uint32_t));
  if (e == hipSuccess) e = hipEventCreate(&p->ev0);
  if (e == hipSuccess) e = hipEventCreate(&p->ev1);
  if (e == hipSuccess && n_pages)
    e = hipMemcpy(p->d_pages, lpages.data(), n_pages * sizeof(sb::PageDesc), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    sb_plan_destroy(p);
    return fail(ctx, SB_E_DEVICE, "nested plan alloc: %s", hipGetErrorString(e));
  }
  p->nest_totals.assign(D + 1, 0);
  // count every level once: the caller allocates from the totals, decodes
  // use the bases; the leaf values streams become the pages of `inner`
  std::vector<sb::PageDesc> vpages(n_pages);
  if (n_pages) {
    if (nest_launch(ctx, p, nullptr, 0) || hipStreamSynchronize(ctx->stream) != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "nested counting failed: %s", hipGetErrorString(hipGetLastError()));
    }
    std::vector<uint32_t> stv(n_pages), vpos(n_pages);
    std::vector<uint64_t> cnt(n_pages * (D + 1)), bases(n_pages * (D + 1));
    (void)hipMemcpy(stv.data(), p->d_status, n_pages * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cnt.data(), p->d_nest, cnt.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(vpos.data(), p->d_nest + 2 * n_pages * (D + 1) + D + 1, n_pages * 4, hipMemcpyDeviceToHost);
    for (uint64_t i = 0; i < n_pages; i++) {
      if (stv[i]) {
        sb_plan_destroy(p);
        return fail(ctx, (sb_status)stv[i], "page %llu: %s", (unsigned long long)i, sb_status_str((int)stv[i]));
      }
      for (uint64_t k = 0; k <= D; k++) {
        bases[i * (D + 1) + k] = p->nest_totals[k];
        p->nest_totals[k] += cnt[i * (D + 1) + k];
      }
      vpages[i] = sb::PageDesc{lpages[i].byte_off + vpos[i], bases[i * (D + 1) + D], lpages[i].byte_len - vpos[i],
                               (uint32_t)cnt[i * (D + 1) + D], 0};
    }
    e = hipMemcpy(p->d_nest + n_pages * (D + 1), bases.data(), bases.size() * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_nest + 2 * n_pages * (D + 1), p->nest_totals.data(), (D + 1) * 8,
                                       hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      sb_plan_destroy(p);
      return fail(ctx, SB_E_DEVICE, "nested plan upload: %s", hipGetErrorString(e));
    }
  }
  const sb_column_desc cd{t, 0};
  sb_status st = plan_pages(ctx, &cd, d_chunk, chunk_len, std::move(vpages), &p->inner);
  if (st) {
    sb_plan_destroy(p);
    return st;
  }
  p->width = p->inner->width;
  p->n_rows = p->nest_totals[0];
  p->n_leaves = p->nest_totals[D];
  p->values_bytes = p->inner->values_bytes;
  *out = p;
  return SB_OK;
}

uint64_t sb_plan_nested_count(const sb_plan* p, int32_t level) {
  if (!p || !p->nested || level < 0 || level > p->ndesc.depth) return 0;
  return p->nest_totals[(size_t)level];
}

sb_status sb_decode_nested_planned(sb_ctx* ctx, sb_plan* p, const sb_nested_out* out) {
  if (!ctx || !p || !out) return fail(ctx, SB_E_ARG, "null argument");
  if (!p->nested) return fail(ctx, SB_E_ARG, "not a nested plan");
  const int D = p->ndesc.depth;
  for (int d = 0; d < D; d++) {
    const bool is_list = !((p->ndesc.struct_mask >> d) & 1);
    if (is_list && !out->d_offsets[d]) return fail(ctx, SB_E_ARG, "offsets of level %d are null", d);
    if (p->ndesc.list_nullable[d] && p->nest_totals[d] && !out->d_validity[d])
      return fail(ctx, SB_E_ARG, "validity of level %d is null", d);
  }
  if (p->n_leaves && !out->d_values) return fail(ctx, SB_E_ARG, "values buffer is null");
  if (p->inner && p->inner->binary && !out->d_leaf_offsets) return fail(ctx, SB_E_ARG, "leaf offsets are null");
  if (p->ndesc.item_nullable && p->n_leaves && !out->d_leaf_validity) return fail(ctx, SB_E_ARG, "leaf validity is null");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (p->timing) HIP_TRY(ctx, hipEventRecord(p->ev0, ctx->stream));
  for (int d = 0; d < D; d++)
    if (p->ndesc.list_nullable[d] && p->nest_totals[d])
      HIP_TRY(ctx, hipMemsetAsync(out->d_validity[d], 0, (p->nest_totals[d] + 31) / 32 * 4, ctx->stream));
  if (p->ndesc.item_nullable && p->n_leaves)
    HIP_TRY(ctx, hipMemsetAsync(out->d_leaf_validity, 0, (p->n_leaves + 31) / 32 * 4, ctx->stream));
  if (!p->n_pages) {
    for (int d = 0; d < D; d++)
      if (!((p->ndesc.struct_mask >> d) & 1))
        HIP_TRY(ctx, hipMemsetAsync(out->d_offsets[d], 0, (size_t)p->ndesc.offset_width, ctx->stream));
  } else {
    sb_status lst = nest_launch(ctx, p, out, 1);
    if (lst) return lst;
    sb_status st;
    if (p->inner->binary) {
      sb_binary_out bo{out->d_leaf_offsets, (uint8_t*)out->d_values, out->values_capacity, nullptr};
      st = sb_decode_binary_planned(ctx, p->inner, &bo);
    } else {
      sb_primitive_out vo{out->d_values, nullptr};  // (no leaves: nothing written)
      st = sb_decode_planned(ctx, p->inner, &vo);
    }
    if (st) return st;
  }
  if (p->timing) {
    HIP_TRY(ctx, hipEventRecord(p->ev1, ctx->stream));
    p->timed = true;
  }
  return SB_OK;
}

sb_status sb_plan_enable_timing(sb_plan* p, int32_t on) {
  if (!p) return SB_E_ARG;
  p->timing = on != 0;
  return SB_OK;
}

sb_status sb_plan_last_kernel_ms(sb_ctx* ctx, sb_plan* p, float* ms) {
  if (!ctx || !p || !ms || !p->timed) return fail(ctx, SB_E_ARG, "no timed decode");
  HIP_TRY(ctx, hipEventSynchronize(p->ev1));
  HIP_TRY(ctx, hipEventElapsedTime(ms, p->ev0, p->ev1));
  return SB_OK;
}

sb_status sb_decode_column(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                           const sb_page_meta* h_metas, uint64_t n_pages, const sb_primitive_out* out) {
  sb_plan* p = nullptr;
  sb_status st = sb_plan_column(ctx, desc, d_chunk, chunk_len, h_metas, n_pages, &p);
  if (st) return st;
  st = sb_decode_planned(ctx, p, out);
  if (!st) st = sb_plan_status(ctx, p, nullptr);
  sb_plan_destroy(p);
  return st;
}

sb_status sb_decompress_values(sb_ctx* ctx, int32_t physical_type, const uint8_t* d_stream, uint64_t stream_len,
                               uint64_t length, void* d_out) {
  // one non-nullable page whose bytes are exactly the value stream
  sb_column_desc d{physical_type, 0};
  sb_page_meta m{stream_len, length};
  sb_primitive_out o{d_out, nullptr};
  return sb_decode_column(ctx, &d, d_stream, stream_len, &m, 1, &o);
}

// read_meta (read/reader.rs:148-178): footer = ... meta | u32 schema_size |
// u32 meta_size | FF FF FF FF 00 00 00 00; meta = u64 n_cols, per column
// (u64 offset, u64 n_pages, n_pages * (u64 length, u64 num_values)).
sb_status sb_read_meta(const uint8_t* f, uint64_t flen, uint64_t* col_off, uint64_t* col_start, uint64_t cols_cap,
                       sb_page_meta* pages, uint64_t pages_cap, uint64_t* n_cols, uint64_t* n_pages) {
  if (!f || !n_cols || !n_pages || flen < 16) return SB_E_ARG;
  uint32_t meta_size;
  memcpy(&meta_size, f + flen - 12, 4);
  if ((uint64_t)meta_size + 16 > flen) return SB_E_OUT_OF_SPEC;
  const uint8_t* m = f + flen - 16 - meta_size;
  uint64_t pos = 0;
  auto rd = [&](uint64_t* v) {
    if (pos + 8 > meta_size) return false;
    memcpy(v, m + pos, 8);
    pos += 8;
    return true;
  };
  uint64_t nc;
  if (!rd(&nc)) return SB_E_IO;
  uint64_t total = 0;
  for (uint64_t c = 0; c < nc; c++) {
    uint64_t off, np;
    if (!rd(&off) || !rd(&np)) return SB_E_IO;
    if (c < cols_cap) {
      if (col_off) col_off[c] = off;
      if (col_start) col_start[c] = total;
    }
    for (uint64_t i = 0; i < np; i++) {
      uint64_t len, nv;
      if (!rd(&len) || !rd(&nv)) return SB_E_IO;
      if (pages && total < pages_cap) pages[total] = sb_page_meta{len, nv};
      total++;
    }
  }
  *n_cols = nc;
  *n_pages = total;
  return SB_OK;
}

}  // extern "C"
