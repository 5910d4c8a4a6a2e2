// sb_encode.h -- host page encoder (writer side), see sb_encode.cpp.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace sb {
namespace enc {

// write::WriteOptions (write/common.rs:37-45) + forced codec (util/env.rs)
struct Opts {
  int32_t default_codec = 0;
  bool has_ratio = false;
  double ratio = 0.0;
  uint32_t forbidden = 0;  // bit (1 << codec id)
  int32_t forced = -1;
};

// One flat page of n rows (serialize.rs:52-132) appended to out.
int encode_page(int phys, const void* values, const uint8_t* validity, size_t n, bool nullable, const Opts& opt,
                uint64_t seed, std::vector<uint8_t>& out);
// One Binary / Utf8 page: offsets are n+1 absolute positions into values;
// ow = offset width (4 or 8); parent_len = the array's whole values length.
int encode_binary_page(const uint8_t* values, const int64_t* offsets, const uint8_t* validity, size_t n,
                       bool nullable, int ow, uint64_t parent_len, const Opts& opt, uint64_t seed,
                       std::vector<uint8_t>& out);
// One Boolean page: rows [off, off + n) of the column bitmap `bits`;
// validity is page-relative.
int encode_bool_page(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, bool nullable,
                     const Opts& opt, uint64_t seed, std::vector<uint8_t>& out);
// One List<primitive> page of `rows` top-level rows: offsets are rows + 1
// absolute positions into the child column; list_valid is page-relative,
// child_valid column-level.  *num_levels = the page's PageMeta.num_values.
int encode_list_page(int phys, const int64_t* offsets, const uint8_t* list_valid, size_t rows, bool list_nullable,
                     const void* child, const uint8_t* child_valid, bool item_nullable, const Opts& opt,
                     uint64_t seed, std::vector<uint8_t>& out, uint64_t* num_levels);
// One nest of a leaf path (outermost first): a list / map nest has entries +
// 1 absolute offsets into the next nest's entries (or the leaf's slots); a
// struct nest passes its slots through.  validity is column-level (NULL =
// all valid).
struct NestLevel {
  const int64_t* offsets;
  const uint8_t* validity;
  bool nullable;
  bool is_struct;
};
// The leaf of a nested path: fixed width (values), Boolean (values = the
// LSB-first bitmap), Binary / Utf8 (values + offsets = slots + 1 absolute
// int64 positions; values_len = the whole buffer).  validity column-level.
struct NestLeaf {
  int phys;
  const void* values;
  const int64_t* offsets;
  uint64_t values_len;
  const uint8_t* validity;
  bool nullable;
};
int nested_max_levels(const NestLevel* nests, int depth, bool leaf_nullable, uint32_t* max_rep, uint32_t* max_def);
// One nested page of top-level rows [r0, r0 + rows) of a leaf path;
// *num_levels = the page's PageMeta.num_values.
int encode_nested_page(const NestLevel* nests, int depth, const NestLeaf& leaf, uint64_t r0, uint64_t rows,
                       const Opts& opt, uint64_t seed, std::vector<uint8_t>& out, uint64_t* num_levels);
// Sampler seed of page `page` of a column written with `seed`.
uint64_t page_seed(uint64_t seed, uint64_t page);
int type_size(int phys);

}  // namespace enc
}  // namespace sb
