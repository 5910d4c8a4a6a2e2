/*
 * sb_oracle.h -- CPU restatement of the strawboat (b41sh/pa, crate 0.2.6) page codec path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the CPU
 * baseline ("port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (pa_amd/) never links or calls it.
 *
 * Parity status: the reference is Rust and cannot be built here (no cargo,
 * no crate registry).  The restatement follows the reference sources cited on
 * each function.  Pinned by: the Patas pack/unpack KAT (patas.rs:191-202),
 * hand-derived BitPacker4x KATs (tests/golden), liblz4/libzstd round trips,
 * and pyarrow-generated Parquet hybrid-RLE / LZ4 streams.  BitPacker4x and
 * roaring layouts are third-party (bitpacking 0.8.0, roaring 0.10.1) and are
 * restated from their published designs: "parity unpinned" for those bytes
 * beyond the hand-derived KATs.
 */
#ifndef SB_ORACLE_H
#define SB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (mirror include/strawboat_gpu.h) */
enum {
  ORC_OK = 0,
  ORC_E_OUT_OF_SPEC = 1,
  ORC_E_NYI = 2,
  ORC_E_IO = 3,
  ORC_E_CODEC = 4,
  ORC_E_ARG = 6,
};

/* codec ids: compression/mod.rs:64-82 */
enum {
  ORC_NONE = 0, ORC_LZ4 = 1, ORC_ZSTD = 2, ORC_SNAPPY = 3,
  ORC_RLE = 10, ORC_DICT = 11, ORC_ONE_VALUE = 12, ORC_FREQ = 13,
  ORC_BITPACKING = 14, ORC_DELTA_BITPACKING = 15, ORC_PATAS = 16,
};

typedef struct {
  uint8_t* data;
  size_t len;
  size_t cap;
} orc_buf;

void orc_buf_free(orc_buf* b);

/* write::WriteOptions (write/common.rs:37-45) + the debug-only forced codec of
 * util/env.rs (-1 = none) + the seed of the deterministic sampler that stands
 * in for thread_rng (integer/mod.rs:316). */
typedef struct {
  int32_t default_codec;     /* 0..3 CommonCompression */
  int32_t has_ratio;         /* default_compress_ratio.is_some() */
  double ratio;
  uint32_t forbidden_mask;   /* bit (1u << codec_id) */
  int32_t forced_codec;      /* -1 = none */
  uint64_t seed;
} orc_write_options;

/* ---- BitPacker4x (bitpacking 0.8.0), SIMD-BP128 4-lane vertical layout ---- */
uint32_t orc_bp4x_num_bits(const uint32_t* in128);
size_t orc_bp4x_pack(const uint32_t* in128, uint32_t num_bits, uint8_t* out);
size_t orc_bp4x_unpack(const uint8_t* in, uint32_t num_bits, uint32_t* out128);
size_t orc_bp4x_pack_sorted(uint32_t initial, const uint32_t* in128, uint32_t num_bits, uint8_t* out);
size_t orc_bp4x_unpack_sorted(uint32_t initial, const uint8_t* in, uint32_t num_bits, uint32_t* out128);

/* ---- value streams: [codec u8][csize u32][usize u32][body] ---- */
/* decompress_integer (integer/mod.rs:72-117).  width in {1,2,4,8}.
 * Reads from buf[*pos..len); advances *pos; writes length*width bytes. */
int orc_decompress_integer(const uint8_t* buf, size_t len, size_t* pos, int width,
                           size_t length, uint8_t* out);
/* decompress_double (double/mod.rs:69-114).  width in {4,8}. */
int orc_decompress_double(const uint8_t* buf, size_t len, size_t* pos, int width,
                          size_t length, uint8_t* out);
/* compress_integer (integer/mod.rs:35-70). validity: LSB bitmap or NULL. */
int orc_compress_integer(const uint8_t* values, const uint8_t* validity, size_t n, int width,
                         int is_signed, const orc_write_options* opt, orc_buf* out);
/* compress_double (double/mod.rs:32-67). */
int orc_compress_double(const uint8_t* values, const uint8_t* validity, size_t n, int width,
                        const orc_write_options* opt, orc_buf* out);

/* ---- Patas pack/unpack (patas.rs:145-162) ---- */
uint16_t orc_patas_pack(uint32_t ref_diff, uint32_t sig_bytes, uint32_t tz);
void orc_patas_unpack(uint16_t packed, uint32_t* ref_diff, uint32_t* sig_bytes, uint32_t* tz);

/* ---- validity (read_basic.rs:36-63 / serialize.rs:200-215) ---- */
/* Parses [def_len u32][hybrid-RLE bw=1].  Writes ceil(length/8) bytes of LSB
 * bitmap into out_bits.  *pos advanced. */
int orc_read_validity(const uint8_t* buf, size_t len, size_t* pos, size_t length, uint8_t* out_bits);
int orc_write_validity(const uint8_t* validity, size_t length, orc_buf* out);

/* ---- flat pages (serialize.rs:52-132) ---- */
/* kind: 0 = integer, 1 = float */
int orc_read_flat_page(const uint8_t* page, size_t page_len, size_t num_values, int kind,
                       int width, int nullable, uint8_t* out_values, uint8_t* out_bits);
int orc_write_flat_page(const uint8_t* values, const uint8_t* validity, size_t n, int kind,
                        int width, int is_signed, int nullable, const orc_write_options* opt,
                        orc_buf* out);

/* whole column chunk (read_integer / read_double): metas = (length, num_values) pairs */
int orc_read_column(const uint8_t* chunk, size_t len, const uint64_t* metas, size_t n_pages, int kind, int width,
                    int nullable, uint8_t* out_values, uint8_t* out_bits);

/* ---- binary / utf8 (compression/binary/mod.rs) ---- */
/* The reference's (Vec<O> offsets, Vec<u8> values) pair, grown by appends. */
typedef struct {
  int64_t* offsets;
  size_t n_off, cap_off;
  uint8_t* values;
  size_t n_val, cap_val;
} orc_binvec;
void orc_binvec_free(orc_binvec* o);
/* decompress_binary (binary/mod.rs:95-183); ow = sizeof(O) in {4, 8} */
int orc_decompress_binary(const uint8_t* buf, size_t len, size_t* pos, size_t length, int ow, orc_binvec* o);
/* compress_binary (binary/mod.rs:26-93); offsets are n+1 absolute positions
 * into values; parent_values_len = the array's whole values buffer length
 * (stats total_bytes and the Extend header's usize use it) */
int orc_compress_binary(const uint8_t* values, const int64_t* offsets, const uint8_t* validity, size_t n, int ow,
                        uint64_t parent_values_len, const orc_write_options* opt, orc_buf* out);
int orc_read_binary_page(const uint8_t* page, size_t page_len, size_t n, int nullable, int ow, orc_binvec* o,
                         uint8_t* out_bits);
int orc_write_binary_page(const uint8_t* values, const int64_t* offsets, const uint8_t* validity, size_t n,
                          int ow, int nullable, uint64_t parent_values_len, const orc_write_options* opt,
                          orc_buf* out);

/* ---- nested List<primitive> (read_basic.rs:65-173, serialize.rs:217-232) ---- */
int orc_write_list_page(const int64_t* list_offsets, const uint8_t* list_validity, size_t rows, int list_nullable,
                        const uint8_t* child_values, const uint8_t* child_validity, int item_nullable, int kind,
                        int width, int is_signed, const orc_write_options* opt, orc_buf* out, uint64_t* num_levels);
int orc_read_nested_page(const uint8_t* page, size_t len, size_t num_levels, int depth, const int* list_nullable,
                         int item_nullable, int kind, int width, int64_t** out_offsets, uint8_t** out_bits,
                         uint8_t* out_values, uint8_t* out_leaf_bits, size_t* counts, size_t* out_rows);
int orc_read_nest_page(const uint8_t* page, size_t len, size_t num_levels, int depth, const int* nest_nullable,
                       uint32_t struct_mask, int item_nullable, int kind, int width, int64_t** out_offsets,
                       uint8_t** out_bits, uint8_t* out_values, uint8_t* out_leaf_bits, size_t* counts,
                       size_t* out_rows);
int orc_write_levels_page(const uint32_t* rep, const uint32_t* def, size_t n_levels, uint32_t max_rep,
                          uint32_t max_def, uint32_t rows, orc_buf* out);
int orc_read_list_page(const uint8_t* page, size_t len, size_t num_levels, int list_nullable, int item_nullable,
                       int kind, int width, int64_t* out_offsets, uint8_t* out_list_bits, uint8_t* out_values,
                       uint8_t* out_leaf_bits, size_t* out_rows, size_t* out_leaves);

/* ---- boolean pages (compression/boolean/{mod,rle,one_value}.rs) ---- */
/* bits = the column's values bitmap, off = the page's first row; validity is
 * page-relative.  Bit buffers are LSB-first. */
int orc_compress_boolean(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n,
                         const orc_write_options* opt, orc_buf* out);
int orc_decompress_boolean(const uint8_t* buf, size_t len, size_t* pos, size_t length, uint8_t* out_bits);
int orc_write_bool_page(const uint8_t* bits, size_t off, const uint8_t* validity, size_t n, int nullable,
                        const orc_write_options* opt, orc_buf* out);
int orc_read_bool_page(const uint8_t* page, size_t page_len, size_t n, int nullable, uint8_t* out_bits,
                       uint8_t* out_valid);
int orc_read_bool_column(const uint8_t* chunk, size_t len, const uint64_t* metas, size_t n_pages, int nullable,
                         uint8_t* out_bits, uint8_t* out_valid);

/* ---- roaring portable format (roaring 0.10.1) ---- */
/* Deserializes into ascending positions.  *count set; positions may be NULL to
 * size.  cap = capacity of positions. */
int orc_roaring_decode(const uint8_t* buf, size_t len, uint32_t* positions, size_t cap,
                       size_t* count);
int orc_roaring_encode(const uint32_t* positions, size_t count, orc_buf* out);

/* ---- hybrid RLE / bit-packed (parquet2 0.17), generic bit width ---- */
int orc_hybrid_decode(const uint8_t* buf, size_t len, uint32_t bit_width, size_t n,
                      uint32_t* out);

/* ---- general codecs (basic.rs) ---- */
int orc_common_decompress(int codec, const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len);
int orc_common_compress(int codec, const uint8_t* in, size_t in_len, orc_buf* out);

/* ---- multi-threaded CPU baseline (sb_cpu_mt.c): pages sharded over
 * n_threads contiguous ranges, each decoded by the page readers above ---- */
int orc_mt_read_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int kind, int width, int nullable,
                       uint8_t* out_values, uint8_t* out_bits, int n_threads);
int orc_mt_read_binary_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int nullable, int ow,
                              uint8_t* out_offsets, uint8_t* out_values, uint64_t values_cap, uint8_t* out_bits,
                              int n_threads, uint64_t* values_len);
int orc_mt_read_list_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int list_nullable,
                            int item_nullable, int kind, int width, int64_t* out_offsets, uint8_t* out_list_bits,
                            uint8_t* out_values, uint8_t* out_leaf_bits, int n_threads, uint64_t* rows_out,
                            uint64_t* leaves_out);
int orc_mt_read_bool_column(const uint8_t* chunk, const uint64_t* metas, size_t n_pages, int nullable,
                            uint8_t* out_bits, uint8_t* out_valid, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
