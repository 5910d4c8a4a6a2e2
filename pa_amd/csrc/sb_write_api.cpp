// sb_write_api.cpp -- C ABI of the writer side (include/strawboat_gpu.h):
// NativeWriter::encode_chunk paging for one flat leaf (write/common.rs:49-119)
// and the file footer of NativeWriter::finish (write/writer.rs:128-167).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/strawboat_gpu.h"
#include "sb_encode.h"
#include "sb_lz4c.h"
#include "sb_zstdc.h"

using sb::enc::Opts;

static Opts to_opts(const sb_write_options* o) {
  Opts r;
  if (o) {
    r.default_codec = o->default_codec;
    r.has_ratio = o->has_ratio != 0;
    r.ratio = o->ratio;
    r.forbidden = o->forbidden_mask;
    r.forced = o->forced_codec;
  }
  return r;
}

static uint8_t* dup_bytes(const std::vector<uint8_t>& v) {
  uint8_t* p = (uint8_t*)std::malloc(v.size() ? v.size() : 1);
  if (p && !v.empty()) std::memcpy(p, v.data(), v.size());
  return p;
}

extern "C" {

void sb_free(void* p) { std::free(p); }

uint64_t sb_page_seed(uint64_t seed, uint64_t page) { return sb::enc::page_seed(seed, page); }

// The device encoder's block compressors (sb_lz4c.h), run on the host.
uint64_t sb_lz4_compress_host(const uint8_t* src, uint64_t n, uint8_t* dst) {
  std::vector<uint8_t> table(sbc::kLz4TableBytes, 0);
  return sbc::lz4_compress(src, (uint32_t)n, dst, table.data());
}

uint64_t sb_snappy_compress_host(const uint8_t* src, uint64_t n, uint8_t* dst) {
  std::vector<uint8_t> table(sbc::kSnappyTableBytes);
  return sbc::snappy_compress(src, (uint32_t)n, dst, table.data());
}

// The device encoder's Zstd frame writer (sb_zstdc.h): LZ4 parse per 128 KiB
// chunk, transcoded into Predefined_Mode sequence blocks.
uint64_t sb_zstd_compress_host(const uint8_t* src, uint64_t n, uint8_t* dst) {
  if (!n) return sbz::zstd_empty(dst);
  std::vector<uint8_t> table(sbc::kLz4TableBytes), lz(sbc::lz4_bound(sbz::kZChunk));
  std::vector<uint64_t> recs(sbz::kZScratchU64);
  uint64_t op = sbz::zstd_frame_header(dst, (uint32_t)n);
  sbz::ZRep rep{{1, 4, 8}};
  for (uint64_t off = 0; off < n; off += sbz::kZChunk) {
    const uint32_t cl = (uint32_t)std::min<uint64_t>(sbz::kZChunk, n - off);
    std::fill(table.begin(), table.end(), 0);
    const uint32_t ll = sbc::lz4_compress(src + off, cl, lz.data(), table.data());
    op += sbz::zstd_transcode(lz.data(), ll, src + off, cl, dst + op, recs.data(), off + cl == n, rep);
  }
  return op;
}

sb_status sb_encode_page(int32_t phys, const void* h_values, const uint8_t* h_validity, uint64_t n, int32_t nullable,
                         const sb_write_options* opts, uint64_t seed, uint8_t** h_out, uint64_t* out_len) {
  if (!h_out || !out_len || (n && !h_values)) return SB_E_ARG;
  if (!sb::enc::type_size(phys)) return SB_E_NYI;
  std::vector<uint8_t> out;
  int rc = sb::enc::encode_page(phys, h_values, h_validity, n, nullable != 0, to_opts(opts), seed, out);
  if (rc) return (sb_status)rc;
  *h_out = dup_bytes(out);
  *out_len = out.size();
  return SB_OK;
}

sb_status sb_encode_column(int32_t phys, const void* h_values, const uint8_t* h_validity, uint64_t n_rows,
                           int32_t nullable, const sb_write_options* opts, uint64_t max_page_rows, int32_t n_threads,
                           uint8_t** h_out, uint64_t* out_len, sb_page_meta** h_metas, uint64_t* n_pages) {
  if (!h_out || !out_len || !h_metas || !n_pages || (n_rows && !h_values)) return SB_E_ARG;
  const bool is_bool = phys == SB_T_BOOLEAN;  // h_values = the LSB-first values bitmap
  const int ts = sb::enc::type_size(phys);
  if (!ts && !is_bool) return SB_E_NYI;
  // page_size = max_page_size.unwrap_or(len).min(len) (common.rs:54-58)
  const uint64_t step = max_page_rows ? std::min<uint64_t>(max_page_rows, n_rows) : n_rows;
  const uint64_t np = step ? (n_rows + step - 1) / step : 0;
  std::vector<std::vector<uint8_t>> pages(np);
  std::vector<int> rcs(np, 0);
  const Opts o = to_opts(opts);
  const uint64_t seed = opts ? opts->seed : 0;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    std::vector<uint8_t> vb;
    for (;;) {
      const uint64_t p = next.fetch_add(1);
      if (p >= np) return;
      const uint64_t r0 = p * step, m = std::min(step, n_rows - r0);
      const uint8_t* valid = nullptr;
      if (nullable && h_validity) {  // slice_parquet_array: re-base the page's validity bits
        vb.assign((m + 7) / 8, 0);
        for (uint64_t i = 0; i < m; i++)
          if ((h_validity[(r0 + i) >> 3] >> ((r0 + i) & 7)) & 1) vb[i >> 3] |= (uint8_t)(1u << (i & 7));
        valid = vb.data();
      }
      if (is_bool)
        rcs[p] = sb::enc::encode_bool_page((const uint8_t*)h_values, r0, valid, m, nullable != 0, o,
                                           sb::enc::page_seed(seed, p), pages[p]);
      else
        rcs[p] = sb::enc::encode_page(phys, (const uint8_t*)h_values + r0 * ts, valid, m, nullable != 0, o,
                                      sb::enc::page_seed(seed, p), pages[p]);
    }
  };
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<uint64_t>((uint64_t)nt, std::max<uint64_t>(np, 1));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  size_t total = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (rcs[p]) return (sb_status)rcs[p];
    total += pages[p].size();
  }
  uint8_t* buf = (uint8_t*)std::malloc(total ? total : 1);
  sb_page_meta* metas = (sb_page_meta*)std::malloc((np ? np : 1) * sizeof(sb_page_meta));
  if (!buf || !metas) { std::free(buf); std::free(metas); return SB_E_ARG; }
  size_t at = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (!pages[p].empty()) std::memcpy(buf + at, pages[p].data(), pages[p].size());
    at += pages[p].size();
    metas[p] = sb_page_meta{pages[p].size(), std::min(step, n_rows - p * step)};
  }
  *h_out = buf;
  *out_len = total;
  *h_metas = metas;
  *n_pages = np;
  return SB_OK;
}

// encode_chunk for one Binary / Utf8 leaf: h_offsets = n_rows + 1 absolute
// int64 positions into h_values (the array's whole values buffer).
sb_status sb_encode_binary_column(int32_t phys, const uint8_t* h_values, uint64_t values_len, const int64_t* h_offsets,
                                  const uint8_t* h_validity, uint64_t n_rows, int32_t nullable,
                                  const sb_write_options* opts, uint64_t max_page_rows, int32_t n_threads,
                                  uint8_t** h_out, uint64_t* out_len, sb_page_meta** h_metas, uint64_t* n_pages) {
  if (!h_out || !out_len || !h_metas || !n_pages || !h_offsets) return SB_E_ARG;
  const int ow = (phys == SB_T_BINARY || phys == SB_T_UTF8) ? 4 : (phys == SB_T_LARGE_BINARY || phys == SB_T_LARGE_UTF8) ? 8 : 0;
  if (!ow) return SB_E_NYI;
  const uint64_t step = max_page_rows ? std::min<uint64_t>(max_page_rows, n_rows) : n_rows;
  const uint64_t np = step ? (n_rows + step - 1) / step : 0;
  std::vector<std::vector<uint8_t>> pages(np);
  std::vector<int> rcs(np, 0);
  const Opts o = to_opts(opts);
  const uint64_t seed = opts ? opts->seed : 0;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    std::vector<uint8_t> vb;
    for (;;) {
      const uint64_t p = next.fetch_add(1);
      if (p >= np) return;
      const uint64_t r0 = p * step, m = std::min(step, n_rows - r0);
      const uint8_t* valid = nullptr;
      if (nullable && h_validity) {
        vb.assign((m + 7) / 8, 0);
        for (uint64_t i = 0; i < m; i++)
          if ((h_validity[(r0 + i) >> 3] >> ((r0 + i) & 7)) & 1) vb[i >> 3] |= (uint8_t)(1u << (i & 7));
        valid = vb.data();
      }
      rcs[p] = sb::enc::encode_binary_page(h_values, h_offsets + r0, valid, m, nullable != 0, ow, values_len, o,
                                           sb::enc::page_seed(seed, p), pages[p]);
    }
  };
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<uint64_t>((uint64_t)nt, std::max<uint64_t>(np, 1));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  size_t total = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (rcs[p]) return (sb_status)rcs[p];
    total += pages[p].size();
  }
  uint8_t* buf = (uint8_t*)std::malloc(total ? total : 1);
  sb_page_meta* metas = (sb_page_meta*)std::malloc((np ? np : 1) * sizeof(sb_page_meta));
  if (!buf || !metas) { std::free(buf); std::free(metas); return SB_E_ARG; }
  size_t at = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (!pages[p].empty()) std::memcpy(buf + at, pages[p].data(), pages[p].size());
    at += pages[p].size();
    metas[p] = sb_page_meta{pages[p].size(), std::min(step, n_rows - p * step)};
  }
  *h_out = buf;
  *out_len = total;
  *h_metas = metas;
  *n_pages = np;
  return SB_OK;
}

// encode_chunk for one List<primitive> leaf (common.rs:49-119 with
// slice_parquet_array per page of max_page_rows top-level rows; write_nested,
// serialize.rs:133-146).  PageMeta.num_values = the page's level count.
sb_status sb_encode_list_column(int32_t phys, const int64_t* h_offsets, const uint8_t* h_list_validity,
                                int32_t list_nullable, const void* h_child, const uint8_t* h_child_validity,
                                int32_t item_nullable, uint64_t n_rows, const sb_write_options* opts,
                                uint64_t max_page_rows, int32_t n_threads, uint8_t** h_out, uint64_t* out_len,
                                sb_page_meta** h_metas, uint64_t* n_pages) {
  if (!h_out || !out_len || !h_metas || !n_pages || !h_offsets || (n_rows && h_offsets[n_rows] > h_offsets[0] && !h_child))
    return SB_E_ARG;
  if (!sb::enc::type_size(phys)) return SB_E_NYI;
  const uint64_t step = max_page_rows ? std::min<uint64_t>(max_page_rows, n_rows) : n_rows;
  const uint64_t np = step ? (n_rows + step - 1) / step : 0;
  std::vector<std::vector<uint8_t>> pages(np);
  std::vector<uint64_t> levels(np, 0);
  std::vector<int> rcs(np, 0);
  const Opts o = to_opts(opts);
  const uint64_t seed = opts ? opts->seed : 0;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    std::vector<uint8_t> lb;
    for (;;) {
      const uint64_t p = next.fetch_add(1);
      if (p >= np) return;
      const uint64_t r0 = p * step, m = std::min(step, n_rows - r0);
      const uint8_t* lv = nullptr;
      if (list_nullable && h_list_validity) {
        lb.assign((m + 7) / 8, 0);
        for (uint64_t i = 0; i < m; i++)
          if ((h_list_validity[(r0 + i) >> 3] >> ((r0 + i) & 7)) & 1) lb[i >> 3] |= (uint8_t)(1u << (i & 7));
        lv = lb.data();
      }
      rcs[p] = sb::enc::encode_list_page(phys, h_offsets + r0, lv, m, list_nullable != 0, h_child, h_child_validity,
                                         item_nullable != 0, o, sb::enc::page_seed(seed, p), pages[p], &levels[p]);
    }
  };
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<uint64_t>((uint64_t)nt, std::max<uint64_t>(np, 1));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  size_t total = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (rcs[p]) return (sb_status)rcs[p];
    total += pages[p].size();
  }
  uint8_t* buf = (uint8_t*)std::malloc(total ? total : 1);
  sb_page_meta* metas = (sb_page_meta*)std::malloc((np ? np : 1) * sizeof(sb_page_meta));
  if (!buf || !metas) { std::free(buf); std::free(metas); return SB_E_ARG; }
  size_t at = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (!pages[p].empty()) std::memcpy(buf + at, pages[p].data(), pages[p].size());
    at += pages[p].size();
    metas[p] = sb_page_meta{pages[p].size(), levels[p]};
  }
  *h_out = buf;
  *out_len = total;
  *h_metas = metas;
  *n_pages = np;
  return SB_OK;
}

// encode_chunk for one leaf of any nested field (write/common.rs:60-115:
// to_nested + to_leaves, slice_parquet_array per page of max_page_rows
// top-level rows; write_nested serialize.rs:135-198).  The nests' offsets
// must be non-decreasing over the entries the rows reach (SB_E_ARG
// otherwise: slice_parquet_array would read past the child arrays).
sb_status sb_encode_nested_column(const sb_nested_desc* desc, const sb_nest_in* h_nests, const void* h_values,
                                  const int64_t* h_leaf_offsets, uint64_t values_len, const uint8_t* h_leaf_validity,
                                  uint64_t n_rows, const sb_write_options* opts, uint64_t max_page_rows,
                                  int32_t n_threads, uint8_t** h_out, uint64_t* out_len, sb_page_meta** h_metas,
                                  uint64_t* n_pages) {
  if (!desc || !h_nests || !h_out || !out_len || !h_metas || !n_pages) return SB_E_ARG;
  const int depth = desc->depth, phys = desc->physical_type;
  if (depth < 1 || depth > SB_MAX_NEST) return SB_E_NYI;
  const bool binary = phys >= SB_T_BINARY && phys <= SB_T_LARGE_UTF8;
  if (!binary && phys != SB_T_BOOLEAN && !sb::enc::type_size(phys)) return SB_E_NYI;
  sb::enc::NestLevel nests[SB_MAX_NEST];
  uint64_t count = n_rows;  // entries of the current nest
  for (int d = 0; d < depth; d++) {
    const bool is_struct = (desc->struct_mask >> d) & 1;
    nests[d] = sb::enc::NestLevel{h_nests[d].h_offsets, h_nests[d].h_validity, desc->list_nullable[d] != 0, is_struct};
    if (is_struct) continue;
    const int64_t* o = h_nests[d].h_offsets;
    if (!o) return SB_E_ARG;
    for (uint64_t i = 0; i < count; i++)
      if (o[i + 1] < o[i] || o[i] < 0) return SB_E_ARG;
    count = (uint64_t)o[count];
  }
  if (count && !h_values) return SB_E_ARG;
  if (binary) {
    if (!h_leaf_offsets) return SB_E_ARG;
    for (uint64_t i = 0; i < count; i++)
      if (h_leaf_offsets[i + 1] < h_leaf_offsets[i] || h_leaf_offsets[i] < 0) return SB_E_ARG;
    if ((uint64_t)h_leaf_offsets[count] > values_len) return SB_E_ARG;
  }
  const sb::enc::NestLeaf leaf{phys, h_values, h_leaf_offsets, values_len, h_leaf_validity, desc->item_nullable != 0};
  const uint64_t step = max_page_rows ? std::min<uint64_t>(max_page_rows, n_rows) : n_rows;
  const uint64_t np = step ? (n_rows + step - 1) / step : 0;
  std::vector<std::vector<uint8_t>> pages(np);
  std::vector<uint64_t> levels(np, 0);
  std::vector<int> rcs(np, 0);
  const Opts o = to_opts(opts);
  const uint64_t seed = opts ? opts->seed : 0;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    for (;;) {
      const uint64_t p = next.fetch_add(1);
      if (p >= np) return;
      const uint64_t r0 = p * step, m = std::min(step, n_rows - r0);
      rcs[p] = sb::enc::encode_nested_page(nests, depth, leaf, r0, m, o, sb::enc::page_seed(seed, p), pages[p],
                                           &levels[p]);
    }
  };
  int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<uint64_t>((uint64_t)nt, std::max<uint64_t>(np, 1));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  size_t total = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (rcs[p]) return (sb_status)rcs[p];
    total += pages[p].size();
  }
  uint8_t* buf = (uint8_t*)std::malloc(total ? total : 1);
  sb_page_meta* metas = (sb_page_meta*)std::malloc((np ? np : 1) * sizeof(sb_page_meta));
  if (!buf || !metas) { std::free(buf); std::free(metas); return SB_E_ARG; }
  size_t at = 0;
  for (uint64_t p = 0; p < np; p++) {
    if (!pages[p].empty()) std::memcpy(buf + at, pages[p].data(), pages[p].size());
    at += pages[p].size();
    metas[p] = sb_page_meta{pages[p].size(), levels[p]};
  }
  *h_out = buf;
  *out_len = total;
  *h_metas = metas;
  *n_pages = np;
  return SB_OK;
}

// NativeWriter::finish (writer.rs:128-167): schema | meta | u32 schema_size |
// u32 meta_size | FF FF FF FF 00 00 00 00; the body starts with
// b"ARROW2" 00 00 (writer.rs:97-100).  Column chunks are given back to back.
sb_status sb_write_footer(const uint8_t* h_schema, uint64_t schema_len, const uint64_t* h_col_offsets,
                          const uint64_t* h_col_npages, uint64_t n_cols, const sb_page_meta* h_pages,
                          uint8_t** h_out, uint64_t* out_len) {
  if (!h_out || !out_len || (n_cols && (!h_col_offsets || !h_col_npages))) return SB_E_ARG;
  std::vector<uint8_t> f;
  auto u64 = [&](uint64_t v) { const uint8_t* p = (const uint8_t*)&v; f.insert(f.end(), p, p + 8); };
  auto u32 = [&](uint32_t v) { const uint8_t* p = (const uint8_t*)&v; f.insert(f.end(), p, p + 4); };
  if (schema_len) f.insert(f.end(), h_schema, h_schema + schema_len);
  const size_t meta_start = f.size();
  u64(n_cols);
  uint64_t pg = 0;
  for (uint64_t c = 0; c < n_cols; c++) {
    u64(h_col_offsets[c]);
    u64(h_col_npages[c]);
    for (uint64_t i = 0; i < h_col_npages[c]; i++, pg++) {
      u64(h_pages[pg].length);
      u64(h_pages[pg].num_values);
    }
  }
  const size_t meta_size = f.size() - meta_start;
  u32((uint32_t)schema_len);
  u32((uint32_t)meta_size);
  u32(0xFFFFFFFFu);
  u32(0);
  *h_out = dup_bytes(f);
  *out_len = f.size();
  return SB_OK;
}

}  // extern "C"
