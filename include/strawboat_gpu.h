/*
 * strawboat_gpu.h -- C ABI of the MI355X strawboat page decode/encode engine.
 *
 * This is the drop-in boundary for the reference's codec path (b41sh/pa,
 * crate strawboat 0.2.6).  Every entry point names the reference interface it
 * replaces.  Plain pointers and sizes only; a Rust crate binds it 1:1
 * (INTEGRATION.md shows the extern "C" block).
 *
 * Memory: "d_" pointers are device (HBM) pointers, "h_" pointers host memory.
 * Calls are asynchronous on the context's HIP stream unless stated; sb_sync()
 * waits.  Decode errors are per page (a status word written by the kernel) and
 * are surfaced by sb_plan_status() / sb_decode_column(), never by aborting.
 */
#ifndef STRAWBOAT_GPU_H
#define STRAWBOAT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error convention: arrow2::error::Error variants the reference returns
 * (src/errors.rs:19-31; OutOfSpec for malformed pages e.g.
 * compression/mod.rs:78-80, NotYetImplemented, Io for short reads, External
 * for codec failures basic.rs:115-116).  Reference panics on malformed pages
 * (array/integer.rs:81, read_basic.rs:59) map to SB_E_OUT_OF_SPEC here. */
typedef enum {
  SB_OK = 0,
  SB_E_OUT_OF_SPEC = 1,
  SB_E_NYI = 2,
  SB_E_IO = 3,
  SB_E_CODEC = 4,
  SB_E_DEVICE = 5,
  SB_E_ARG = 6,
} sb_status;

/* Codec ids of the 9-byte value-stream header (compression/mod.rs:64-82). */
typedef enum {
  SB_CODEC_NONE = 0,
  SB_CODEC_LZ4 = 1,
  SB_CODEC_ZSTD = 2,
  SB_CODEC_SNAPPY = 3,
  SB_CODEC_RLE = 10,
  SB_CODEC_DICT = 11,
  SB_CODEC_ONE_VALUE = 12,
  SB_CODEC_FREQ = 13,
  SB_CODEC_BITPACKING = 14,
  SB_CODEC_DELTA_BITPACKING = 15,
  SB_CODEC_PATAS = 16,
} sb_codec;

/* Arrow physical types handled by the page deserializers
 * (read/deserialize.rs:100-135 dispatch). */
typedef enum {
  SB_T_INT8 = 1,
  SB_T_INT16 = 2,
  SB_T_INT32 = 3,
  SB_T_INT64 = 4,
  SB_T_UINT8 = 5,
  SB_T_UINT16 = 6,
  SB_T_UINT32 = 7,
  SB_T_UINT64 = 8,
  SB_T_FLOAT32 = 9,
  SB_T_FLOAT64 = 10,
  SB_T_BINARY = 11,       /* i32 offsets */
  SB_T_LARGE_BINARY = 12, /* i64 offsets */
  SB_T_UTF8 = 13,         /* i32 offsets; values checked as Utf8Array::try_new does (OutOfSpec) */
  SB_T_LARGE_UTF8 = 14,   /* i64 offsets */
  SB_T_BOOLEAN = 15,      /* values are an LSB-first bitmap (read_boolean, read/array/boolean.rs:191-219) */
} sb_physical_type;

/* PageMeta (src/lib.rs:75-80): compressed page length and num_values. */
typedef struct {
  uint64_t length;
  uint64_t num_values;
} sb_page_meta;

/* Leaf column descriptor: the parts of arrow2 Field + parquet2
 * ColumnDescriptor the flat page readers use (array/integer.rs:28-60:
 * is_nullable, data_type). */
typedef struct {
  int32_t physical_type; /* sb_physical_type */
  int32_t nullable;      /* Field::is_nullable */
} sb_column_desc;

/* Output buffers of a primitive column (caller-allocated, device):
 * values: sum(num_values) * sizeof(T) bytes (Boolean: a bitmap laid out like
 * the validity below);
 * validity: 4*ceil(sum(num_values)/32) bytes (LSB-first Arrow bitmap, written
 * as 32-bit words; bits past the last row are zero) or NULL when the column is
 * not nullable.  Both 16-byte aligned for vector stores. */
typedef struct {
  void* d_values;
  uint8_t* d_validity;
} sb_primitive_out;

/* Output buffers of a Binary / Utf8 column (caller-allocated, device):
 * offsets: (sum(num_values) + 1) offsets of 4 (Binary/Utf8) or 8 (Large*)
 * bytes; values: sb_plan_values_bytes() bytes; validity as above. */
typedef struct {
  void* d_offsets;
  uint8_t* d_values;
  uint64_t values_capacity;
  uint8_t* d_validity;
} sb_binary_out;

typedef struct sb_ctx sb_ctx;
typedef struct sb_plan sb_plan;

/* ---- context ---------------------------------------------------------- */
/* One context binds one device and one HIP stream; not thread-safe (the
 * reference's readers are single-consumer iterators, read/reader.rs:51). */
sb_status sb_ctx_create(int device, sb_ctx** out);
void sb_ctx_destroy(sb_ctx* ctx);
/* Launch on an external hipStream_t (e.g. torch.cuda.current_stream()).  The
 * handle is used as given: NULL means the legacy default stream.  A fresh
 * context uses a non-blocking stream of its own. */
sb_status sb_ctx_set_stream(sb_ctx* ctx, void* hip_stream);
void* sb_ctx_stream(sb_ctx* ctx);
/* The device the context binds (-1 for NULL). */
int32_t sb_ctx_device(const sb_ctx* ctx);
sb_status sb_sync(sb_ctx* ctx);
const char* sb_last_error(const sb_ctx* ctx);
const char* sb_status_str(int status);

/* ---- column decode ----------------------------------------------------- */
/* Builds the device page table for one leaf column chunk: the pages are the
 * back-to-back page bytes starting at ColumnMeta.offset (d_chunk, chunk_len
 * bytes, already in HBM), described by h_metas (ColumnMeta.pages).  Replaces
 * the per-page NativeReader::next (read/reader.rs:119-131) walk; the row
 * offsets are the running sum of num_values.  Uploads asynchronously. */
sb_status sb_plan_column(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk,
                         uint64_t chunk_len, const sb_page_meta* h_metas, uint64_t n_pages,
                         sb_plan** out);
/* The same over pages placed at caller-chosen rows: page i decodes into
 * rows [h_row_offsets[i], + num_values) of the outputs (non-decreasing, no
 * overlap; rows in gaps are not written).  Several columns of one type and
 * nullability whose chunks lie back to back in d_chunk (as the columns of a
 * file do) become one plan and one launch sequence, each column at its own
 * row base (a multiple of 32 keeps its validity word-aligned).  Fixed-width
 * and Boolean columns only. */
sb_status sb_plan_column_at(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                            const sb_page_meta* h_metas, uint64_t n_pages, const uint64_t* h_row_offsets,
                            sb_plan** out);
void sb_plan_destroy(sb_plan* plan);
uint64_t sb_plan_num_rows(const sb_plan* plan);
uint64_t sb_plan_num_pages(const sb_plan* plan);

/* Launches the batched page decode of a planned column (asynchronous).
 * Replaces read_integer / read_double (read/array/integer.rs:210-238,
 * read/array/double.rs:210-238) as driven by batch_read_array
 * (read/batch_read.rs:190-209): validity + values of every page, appended. */
sb_status sb_decode_planned(sb_ctx* ctx, sb_plan* plan, const sb_primitive_out* out);

/* Binary / Utf8 columns (read_binary, read/array/binary.rs:223-265; pages via
 * decompress_binary, compression/binary/mod.rs:95-183).  For these types
 * sb_plan_column also sizes every page's values on the device (synchronous)
 * and fails with the first bad page's status. */
uint64_t sb_plan_values_bytes(const sb_plan* plan);
sb_status sb_decode_binary_planned(sb_ctx* ctx, sb_plan* plan, const sb_binary_out* out);

/* List<primitive> columns (one list level over a primitive leaf): the
 * nested page readers (read_nested_integer / read_nested_double,
 * read/array/integer.rs:240-261) over read_validity_nested
 * (read/read_basic.rs:65-173) + create_list (read/array/list.rs:48), pages
 * concatenated as batch_read_array does.  PageMeta.num_values of a nested
 * page is its level count. */
typedef struct {
  int32_t physical_type; /* leaf type (fixed width) */
  int32_t list_nullable; /* the List field is nullable */
  int32_t item_nullable; /* the item field is nullable */
  int32_t offset_width;  /* 4 = List, 8 = LargeList */
} sb_list_desc;

/* offsets: rows + 1 entries of offset_width bytes; list validity over the
 * rows and leaf validity over the leaves (4*ceil(n/32) bytes each, NULL when
 * that level is not nullable); values: leaves * sizeof(T). */
typedef struct {
  void* d_offsets;
  uint8_t* d_list_validity;
  void* d_values;
  uint8_t* d_leaf_validity;
} sb_list_out;

/* Plans a List column and sizes it on the device (synchronous): rows =
 * sb_plan_num_rows, leaves = sb_plan_num_leaves; fails with the first bad
 * page's status. */
sb_status sb_plan_list_column(sb_ctx* ctx, const sb_list_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                              const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out);
uint64_t sb_plan_num_leaves(const sb_plan* plan);
/* Asynchronous decode: sizing pass + bases scan + levels (offsets, bitmaps)
 * + the values streams at their leaf bases. */
sb_status sb_decode_list_planned(sb_ctx* ctx, sb_plan* plan, const sb_list_out* out);

/* One leaf column of a nested field under 1..4 nests: the InitNested chain
 * deserialize_nested builds (read/deserialize.rs:140-233) -- a List /
 * LargeList / FixedSizeList / Map pushes InitNested::List(nullable), a Struct
 * InitNested::Struct(nullable) for each of its children's leaves.  The
 * general read_validity_nested (read/read_basic.rs:95-164): per-nest
 * cum_sum / cum_rep over {nullable, repeated}, lists and the leaf never
 * "required", structs always (arrow2 NestedStruct / NestedStructValid: a
 * null struct pushes a slot into every child); then create_list /
 * create_map per list nest (read/array/list.rs:48, map.rs) with the pages
 * concatenated and each list's offsets moved onto its child's running
 * length.  Nest 0 is the outermost.  PageMeta.num_values is the page's level
 * count.  A Struct / Map field is several leaf columns (to_leaves order),
 * each planned on its own; create_struct takes the struct's validity from
 * its LAST child (read/array/struct_.rs:101-114), and every leaf under a
 * struct nest yields that nest's entries and validity. */
#define SB_MAX_NEST 4
typedef struct {
  int32_t physical_type;                /* leaf type: fixed width, Boolean, Binary / Utf8 (Large too) */
  int32_t depth;                        /* nests, 1..SB_MAX_NEST */
  int32_t list_nullable[SB_MAX_NEST];   /* nest d is nullable (list, map or struct) */
  int32_t item_nullable;                /* the leaf is nullable */
  int32_t offset_width;                 /* 4 = List / Map, 8 = LargeList (every list nest) */
  int32_t struct_mask;                  /* bit d: nest d is a Struct (no offsets), else a List / Map */
} sb_nested_desc;

/* d_offsets[d] (list nests; NULL for struct nests): sb_plan_nested_count(plan,
 * d) + 1 entries; d_validity[d] over nest d's entries (NULL when not
 * nullable); d_leaf_validity over the leaves.  Leaf values: fixed width -- d_values holds
 * sb_plan_nested_count(plan, depth) values; Boolean -- d_values is their
 * bitmap; Binary / Utf8 -- d_leaf_offsets holds leaves + 1 offsets (the
 * physical type's width) and d_values values_capacity >=
 * sb_plan_values_bytes(plan) bytes (read_nested_binary, pages concatenated). */
typedef struct {
  void* d_offsets[SB_MAX_NEST];
  uint8_t* d_validity[SB_MAX_NEST];
  void* d_values;
  uint8_t* d_leaf_validity;
  void* d_leaf_offsets;
  uint64_t values_capacity;
} sb_nested_out;

/* Plans a nested column and counts every level's entries on the device
 * (synchronous); fails with the first bad page's status. */
sb_status sb_plan_nested_column(sb_ctx* ctx, const sb_nested_desc* desc, const uint8_t* d_chunk, uint64_t chunk_len,
                                const sb_page_meta* h_metas, uint64_t n_pages, sb_plan** out);
/* Entries of level d (0 = the top-level rows; depth = the leaves). */
uint64_t sb_plan_nested_count(const sb_plan* plan, int32_t level);
/* Asynchronous decode: the level walk (offsets, bitmaps) + the values
 * streams at their leaf bases; sb_plan_status reports the first bad page. */
sb_status sb_decode_nested_planned(sb_ctx* ctx, sb_plan* plan, const sb_nested_out* out);

/* Waits for the plan's last decode and returns the first failing page's
 * status (SB_OK if every page decoded); *h_bad_page = its index or -1. */
sb_status sb_plan_status(sb_ctx* ctx, sb_plan* plan, int64_t* h_bad_page);

/* ---- page-level unit entry points (synchronous) -------------------------
 * For a caller that walks the pages itself; the column decoders above fuse
 * both steps into their page kernels.
 *
 * read_validity (read/read_basic.rs:36-63) of one flat nullable page at
 * d_page: its [u32 def_len][hybrid RLE / bit-packed def levels] prefix, one
 * bit-packed run (an RLE run is OutOfSpec, :59 unreachable!()), whose first
 * `length` bits are written to the Arrow bitmap d_validity (32-bit words)
 * at bit bit_offset; the bitmap's other bits are kept.  *h_consumed = the
 * prefix bytes (4 + def_len): the values stream starts there.  def_len 0 is
 * OutOfSpec unless length is 0 (nothing pushed, the array would not build). */
sb_status sb_decode_page_validity(sb_ctx* ctx, const uint8_t* d_page, uint64_t page_len, uint64_t length,
                                  uint32_t* d_validity, uint64_t bit_offset, uint64_t* h_consumed);
/* The level streams of read_validity_nested (read/read_basic.rs:65-86) of one
 * nested page: [u32 rows][u32 rep_len][u32 def_len][rep levels][def levels],
 * each decoded by parquet2's HybridRleDecoder with bit width
 * get_bit_width(max level) into num_levels u16 levels (d_rep, d_def).
 * *h_rows = the page's row count, *h_consumed = 12 + rep_len + def_len. */
sb_status sb_decode_page_levels(sb_ctx* ctx, const uint8_t* d_page, uint64_t page_len, uint64_t num_levels,
                                uint32_t max_rep_level, uint32_t max_def_level, uint16_t* d_rep, uint16_t* d_def,
                                uint32_t* h_rows, uint64_t* h_consumed);

/* One-shot: plan + decode + wait + status.  The batch_read_array
 * equivalent for one flat primitive leaf. */
sb_status sb_decode_column(sb_ctx* ctx, const sb_column_desc* desc, const uint8_t* d_chunk,
                           uint64_t chunk_len, const sb_page_meta* h_metas, uint64_t n_pages,
                           const sb_primitive_out* out);

/* Opt-in per-decode timing: when on, sb_decode_planned records HIP events on
 * the launch stream around the decode kernels (off by default: an event
 * record between back-to-back decodes costs a gap on the stream). */
sb_status sb_plan_enable_timing(sb_plan* plan, int32_t on);
/* Device time of the plan's last timed decode, in milliseconds. */
sb_status sb_plan_last_kernel_ms(sb_ctx* ctx, sb_plan* plan, float* ms);

/* ---- value-stream level (unit parity) ---------------------------------- */
/* decompress_integer / decompress_double for ONE page's values, no validity
 * prefix (compression/integer/mod.rs:72-117, double/mod.rs:69-114):
 * d_stream = [codec][csize][usize][body], length values out. Synchronous. */
sb_status sb_decompress_values(sb_ctx* ctx, int32_t physical_type, const uint8_t* d_stream,
                               uint64_t stream_len, uint64_t length, void* d_out);

/* ---- host-side format helpers ------------------------------------------ */
/* read_meta (read/reader.rs:148-178) over the tail of a file held in host
 * memory: fills up to cap column metas.  Returns the number of columns in
 * *n_cols; pages of column i are written to h_pages[page_start[i]..]. */
sb_status sb_read_meta(const uint8_t* h_file, uint64_t file_len, uint64_t* h_col_offsets,
                       uint64_t* h_col_page_start, uint64_t cols_cap, sb_page_meta* h_pages,
                       uint64_t pages_cap, uint64_t* n_cols, uint64_t* n_pages);

/* ---- writer side ------------------------------------------------------- */
/* write::WriteOptions (write/common.rs:37-45) + the debug-build forced codec
 * of util/env.rs (STRAWBOAT_*_COMPRESSION; -1 = none) + the seed of the
 * deterministic trial-window sampler that replaces thread_rng
 * (compression/integer/mod.rs:316). */
typedef struct {
  int32_t default_codec;   /* CommonCompression: SB_CODEC_NONE..SB_CODEC_SNAPPY */
  int32_t has_ratio;       /* default_compress_ratio.is_some() */
  double ratio;            /* default_compress_ratio */
  uint32_t forbidden_mask; /* forbidden_compressions: bit (1u << codec id) */
  int32_t forced_codec;
  uint64_t seed;
} sb_write_options;

/* One flat page (write::write_simple, write/serialize.rs:52-132): optional
 * validity prefix + compress_integer / compress_double value stream.  Host
 * memory in and out; *h_out is freed with sb_free. */
sb_status sb_encode_page(int32_t physical_type, const void* h_values, const uint8_t* h_validity, uint64_t n,
                         int32_t nullable, const sb_write_options* opts, uint64_t seed, uint8_t** h_out,
                         uint64_t* out_len);
/* NativeWriter::encode_chunk (write/common.rs:49-119) for one flat leaf:
 * pages of max_page_rows rows (0 = one page), encoded on n_threads host
 * threads (0 = all).  Page p samples with sb_page_seed(opts->seed, p).
 * Boolean: h_values is the column's LSB-first values bitmap and page p is
 * its slice (compress_boolean, compression/boolean/mod.rs:22-61). */
sb_status sb_encode_column(int32_t physical_type, const void* h_values, const uint8_t* h_validity,
                           uint64_t n_rows, int32_t nullable, const sb_write_options* opts,
                           uint64_t max_page_rows, int32_t n_threads, uint8_t** h_out, uint64_t* out_len,
                           sb_page_meta** h_metas, uint64_t* n_pages);
/* encode_chunk for one Binary / Utf8 leaf (serialize.rs:64-110 ->
 * compress_binary, compression/binary/mod.rs:26-93): h_offsets holds
 * n_rows + 1 absolute positions into h_values (values_len bytes, the
 * array's whole buffer, which the reference's stats and Extend header use). */
sb_status sb_encode_binary_column(int32_t physical_type, const uint8_t* h_values, uint64_t values_len,
                                  const int64_t* h_offsets, const uint8_t* h_validity, uint64_t n_rows,
                                  int32_t nullable, const sb_write_options* opts, uint64_t max_page_rows,
                                  int32_t n_threads, uint8_t** h_out, uint64_t* out_len, sb_page_meta** h_metas,
                                  uint64_t* n_pages);
/* encode_chunk for one List<primitive> leaf (write/common.rs:49-119,
 * write_nested serialize.rs:133-146): pages of max_page_rows top-level rows;
 * h_offsets = n_rows + 1 absolute int64 positions into h_child (the child
 * column's values, sizeof(physical_type) each); h_list_validity is over the
 * rows, h_child_validity over the child values (either may be NULL).
 * PageMeta.num_values of each page is its level count (num_values(nested)). */
sb_status sb_encode_list_column(int32_t physical_type, const int64_t* h_offsets, const uint8_t* h_list_validity,
                                int32_t list_nullable, const void* h_child, const uint8_t* h_child_validity,
                                int32_t item_nullable, uint64_t n_rows, const sb_write_options* opts,
                                uint64_t max_page_rows, int32_t n_threads, uint8_t** h_out, uint64_t* out_len,
                                sb_page_meta** h_metas, uint64_t* n_pages);
/* One nest of a leaf path for the writer (outermost first, as in
 * sb_nested_desc): a List / LargeList / Map nest gives entries + 1 absolute
 * int64 positions into the next nest's entries (or the leaf's slots); a
 * Struct nest gives no offsets (its children hold one slot per struct slot).
 * h_validity: LSB-first bitmap over the nest's entries, NULL = all valid. */
typedef struct {
  const int64_t* h_offsets;
  const uint8_t* h_validity;
} sb_nest_in;
/* encode_chunk for one leaf column of ANY nested field (write/common.rs:
 * 60-115: to_nested + to_leaves, then slice_parquet_array per page of
 * max_page_rows top-level rows; write_nested, serialize.rs:135-198, with the
 * rep / def levels of write_nested_validity :217-232 -- no stream for a max
 * level of 0).  desc is the leaf's InitNested chain (depth, per-nest
 * nullable, struct_mask, item_nullable, physical_type; offset_width is not
 * used: the levels do not depend on it).  The leaf: fixed width -- h_values
 * holds its slots; Boolean -- h_values is the LSB-first bitmap of its slots;
 * Binary / Utf8 (Large too) -- h_leaf_offsets = slots + 1 absolute int64
 * positions into h_values (values_len bytes, the whole buffer the Extend
 * header and stats use).  h_leaf_validity over the slots (NULL = none).  A
 * Struct / Map field is written by one call per leaf, in to_leaves order.
 * PageMeta.num_values = the page's level count.  Page p samples with
 * sb_page_seed(opts->seed, p).  SB_E_ARG for decreasing offsets. */
sb_status sb_encode_nested_column(const sb_nested_desc* desc, const sb_nest_in* h_nests, const void* h_values,
                                  const int64_t* h_leaf_offsets, uint64_t values_len, const uint8_t* h_leaf_validity,
                                  uint64_t n_rows, const sb_write_options* opts, uint64_t max_page_rows,
                                  int32_t n_threads, uint8_t** h_out, uint64_t* out_len, sb_page_meta** h_metas,
                                  uint64_t* n_pages);
uint64_t sb_page_seed(uint64_t seed, uint64_t page);
/* The block compressors the device encoder runs for the Basic codecs
 * (CommonCompression::compress, basic.rs:108-152), built for the host:
 * LZ4 = liblz4 1.9.3 LZ4_compress_default restated (dst holds n + n/255 + 16
 * bytes), Snappy = the engine's raw-snappy writer (dst holds n + n/20 + 16).
 * Return the compressed size. */
uint64_t sb_lz4_compress_host(const uint8_t* src, uint64_t n, uint8_t* dst);
uint64_t sb_snappy_compress_host(const uint8_t* src, uint64_t n, uint8_t* dst);
/* The device encoder's Zstd frame writer (pa_amd/csrc/sb_zstdc.h) on the host:
 * an RFC 8878 frame of n bytes that libzstd decodes to src (the reference's
 * libzstd level-3 bytes are not reproduced; decode equivalence is the bar).
 * dst holds n + n/2048 + 3*(n/131072) + 512 bytes.  Returns the frame size. */
uint64_t sb_zstd_compress_host(const uint8_t* src, uint64_t n, uint8_t* dst);
/* encode_chunk on the device (HIP, gfx950), byte-identical to
 * sb_encode_column with the same options: the adaptive cascade
 * (compress_integer / compress_double / compress_boolean with the seeded
 * trial-window sampler, forced codecs, Dict / Freq cascades, Patas) and the
 * Basic codecs None / LZ4 / Snappy run on the GPU; a Zstd default codec that a
 * page needs reports SB_E_NYI (libzstd's compressor is not restated).
 * Options with ratio None + default None (+ forced Bitpacking) take a
 * dedicated sizing/assembly fast path.  d_values (Boolean: the column's LSB
 * bitmap) / d_validity (column LSB bitmap) / d_out are device memory; d_out
 * holds at least sb_encode_device_bound() bytes; page p is rows
 * [p*P, (p+1)*P), P = min(max_page_rows or n_rows, n_rows) <= 16384.
 * Synchronizes the context's stream. */
uint64_t sb_encode_device_bound(int32_t physical_type, uint64_t n_rows, int32_t nullable, uint64_t max_page_rows);
sb_status sb_encode_column_device(sb_ctx* ctx, int32_t physical_type, const void* d_values, const uint8_t* d_validity,
                                  uint64_t n_rows, int32_t nullable, const sb_write_options* opts,
                                  uint64_t max_page_rows, uint8_t* d_out, uint64_t out_capacity, uint64_t* out_len,
                                  sb_page_meta* h_metas, uint64_t metas_cap, uint64_t* n_pages);
/* encode_chunk for one Binary / Utf8 leaf on the device: d_offsets holds
 * n_rows + 1 absolute int64 positions into d_values (values_len bytes, the
 * array's whole buffer, which the stats and the Extend header use, as
 * sb_encode_binary_column); d_validity the column's LSB bitmap.  The writer's
 * full option set runs on the device (compress_binary, binary/mod.rs:26-93:
 * OneValue / Freq / Dict by ratio or forced, the Dict index stream through the
 * integer cascade, Basic None / LZ4 / Snappy) except a Zstd default codec
 * (SB_E_NYI); byte-identical to sb_encode_binary_column.  d_out holds at
 * least sb_encode_binary_device_bound() bytes.  Synchronizes the stream. */
uint64_t sb_encode_binary_device_bound(int32_t physical_type, uint64_t n_rows, uint64_t values_len, int32_t nullable,
                                       uint64_t max_page_rows);
sb_status sb_encode_binary_column_device(sb_ctx* ctx, int32_t physical_type, const uint8_t* d_values,
                                         uint64_t values_len, const int64_t* d_offsets, const uint8_t* d_validity,
                                         uint64_t n_rows, int32_t nullable, const sb_write_options* opts,
                                         uint64_t max_page_rows, uint8_t* d_out, uint64_t out_capacity,
                                         uint64_t* out_len, sb_page_meta* h_metas, uint64_t metas_cap,
                                         uint64_t* n_pages);
/* encode_chunk for one List<primitive> leaf on the device (write/common.rs:
 * 49-119 with slice_parquet_array per page, write_nested serialize.rs:133-146),
 * byte-identical to sb_encode_list_column with the same options: per page of
 * max_page_rows (<= 16384) top-level rows, the rep / def level streams (one
 * bit-packed hybrid run each) and the sliced child values through the device
 * cascade (sb_encode_column_device's page kernels; the child validity feeds
 * the statistics, no validity prefix).  d_offsets = n_rows + 1 absolute int64
 * positions into d_child; d_list_validity over the rows, d_child_validity over
 * the child values (device LSB bitmaps).  d_out holds at least
 * sb_encode_list_device_bound(.., n_child = d_offsets[n_rows] - d_offsets[0],
 * ..) bytes; PageMeta.num_values = the page's level count.  Synchronizes the
 * context's stream. */
uint64_t sb_encode_list_device_bound(int32_t physical_type, uint64_t n_rows, uint64_t n_child, int32_t item_nullable,
                                     uint64_t max_page_rows);
sb_status sb_encode_list_column_device(sb_ctx* ctx, int32_t physical_type, const int64_t* d_offsets,
                                       const uint8_t* d_list_validity, int32_t list_nullable, const void* d_child,
                                       const uint8_t* d_child_validity, int32_t item_nullable, uint64_t n_rows,
                                       const sb_write_options* opts, uint64_t max_page_rows, uint8_t* d_out,
                                       uint64_t out_capacity, uint64_t* out_len, sb_page_meta* h_metas,
                                       uint64_t metas_cap, uint64_t* n_pages);
/* NativeWriter::finish (write/writer.rs:128-167) footer bytes. */
sb_status sb_write_footer(const uint8_t* h_schema, uint64_t schema_len, const uint64_t* h_col_offsets,
                          const uint64_t* h_col_npages, uint64_t n_cols, const sb_page_meta* h_pages,
                          uint8_t** h_out, uint64_t* out_len);
void sb_free(void* p);

/* ---- file reader: footer, schema, file -> HBM staging ------------------- */
/* One leaf of the schema in arrow2's to_leaves order (write/common.rs:68),
 * i.e. the order of the file's columns: its logical type (the IPC Schema.fbs
 * Type union tag), the reader's physical type (0 when no page path exists,
 * e.g. Decimal, Float16), and the nests above it -- the InitNested chain of
 * deserialize_nested (read/deserialize.rs:202-230): List / LargeList / Map
 * (and FixedSizeList) nests and Struct nests, outermost first, each with a
 * schema-wide id (pre-order) so the leaves of one struct or map can be
 * grouped back into their field (sb_nested_desc takes depth,
 * list_nullable and struct_mask as they are here). */
#define SB_LEAF_STRUCT 1u          /* a Struct lies on the path (a struct nest) */
#define SB_LEAF_MAP 2u             /* a Map lies on the path (a list nest over its entries struct) */
#define SB_LEAF_FIXED_SIZE_LIST 4u /* a FixedSizeList lies on the path (not decoded here) */
#define SB_LEAF_UNION 8u           /* a Union lies on the path (not decoded here) */
#define SB_LEAF_TOO_DEEP 16u       /* more than SB_MAX_NEST nests */
typedef struct {
  char name[64];                      /* the leaf field's name (truncated) */
  int32_t arrow_type;                 /* Schema.fbs Type tag: Int 2, FloatingPoint 3, Binary 4, Utf8 5, Bool 6, ... */
  int32_t physical_type;              /* sb_physical_type, 0 = none */
  int32_t nullable;                   /* the leaf field's nullable flag */
  int32_t depth;                      /* nests above the leaf */
  int32_t list_nullable[SB_MAX_NEST]; /* per nest, outermost first: the nest field is nullable */
  int32_t large_list[SB_MAX_NEST];    /* LargeList (i64 offsets) per nest */
  uint32_t flags;                     /* SB_LEAF_* */
  int32_t top_field;                  /* index of the top-level field it belongs to */
  uint32_t struct_mask;               /* bit d: nest d is a Struct */
  uint32_t map_mask;                  /* bit d: nest d is a Map (its child nest is the entries struct) */
  int32_t nest_id[SB_MAX_NEST];       /* per nest: the nest field's pre-order id in the schema */
} sb_leaf_info;

/* infer_schema (read/reader.rs:227-241) + arrow2 deserialize_schema: the
 * footer's schema bytes (an IPC Message flatbuffer, or an encapsulated
 * message with its FF FF FF FF prefix) -> leaves.  Host only. */
sb_status sb_parse_schema(const uint8_t* h_bytes, uint64_t len, sb_leaf_info* h_leaves, uint64_t cap,
                          uint64_t* n_leaves, uint64_t* n_fields);

typedef struct sb_file sb_file;
/* read_meta / read_meta_async (reader.rs:168-225): opens the file and reads
 * its footer with one 64 KiB pre-read of the tail (DEFAULT_FOOTER_SIZE),
 * reading again only when the footer is larger.  Host only. */
sb_status sb_file_open(const char* path, sb_file** out);
void sb_file_close(sb_file* f);
const char* sb_file_last_error(const sb_file* f);
uint64_t sb_file_num_columns(const sb_file* f);
/* ColumnMeta of leaf column `col`: its offset, chunk bytes, page metas (owned by f). */
sb_status sb_file_column(const sb_file* f, uint64_t col, uint64_t* offset, uint64_t* chunk_len, uint64_t* n_pages,
                         const sb_page_meta** h_pages);
sb_status sb_file_schema(const sb_file* f, const uint8_t** h_bytes, uint64_t* len);
/* The NativeReader page source (reader.rs:60-131) as one staged copy: file
 * bytes [offset, offset + len) -> d_dst through the device's two pinned 16 MiB buffers
 * (parallel pread of chunk k+1 overlaps the DMA of chunk k on the device's
 * copy stream).  The context's stream waits for the copy, so decodes issued
 * on it afterwards read the bytes; the call returns once the last chunk is
 * read and queued, so the next column's upload overlaps this one's decode. */
sb_status sb_file_upload(sb_ctx* ctx, sb_file* f, uint64_t offset, uint64_t len, void* d_dst);

#ifdef __cplusplus
}
#endif
#endif
