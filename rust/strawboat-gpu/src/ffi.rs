//! 1:1 declarations of include/strawboat_gpu.h (the engine's C ABI) and the
//! few HIP runtime calls the safe layer uses.  Kept in sync with the header
//! by tests/test_abi.py (every declared symbol is exported by the library).
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)] pub struct sb_ctx { _p: [u8; 0] }
#[repr(C)] pub struct sb_plan { _p: [u8; 0] }
#[repr(C)] pub struct sb_file { _p: [u8; 0] }

pub const SB_MAX_NEST: usize = 4;

#[repr(C)] #[derive(Clone, Copy)]
pub struct sb_leaf_info {
    pub name: [c_char; 64], pub arrow_type: i32, pub physical_type: i32, pub nullable: i32, pub depth: i32,
    pub list_nullable: [i32; SB_MAX_NEST], pub large_list: [i32; SB_MAX_NEST], pub flags: u32, pub top_field: i32,
    pub struct_mask: u32, pub map_mask: u32, pub nest_id: [i32; SB_MAX_NEST],
}

#[repr(C)] #[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct sb_page_meta { pub length: u64, pub num_values: u64 }   // == crate::PageMeta

#[repr(C)] #[derive(Clone, Copy)]
pub struct sb_column_desc { pub physical_type: i32, pub nullable: i32 }

#[repr(C)]
pub struct sb_primitive_out { pub d_values: *mut c_void, pub d_validity: *mut u8 }

#[repr(C)]
pub struct sb_binary_out { pub d_offsets: *mut c_void, pub d_values: *mut u8,
                          pub values_capacity: u64, pub d_validity: *mut u8 }

#[repr(C)] #[derive(Clone, Copy)]
pub struct sb_list_desc { pub physical_type: i32, pub list_nullable: i32,
                          pub item_nullable: i32, pub offset_width: i32 }

#[repr(C)]
pub struct sb_list_out { pub d_offsets: *mut c_void, pub d_list_validity: *mut u8,
                        pub d_values: *mut c_void, pub d_leaf_validity: *mut u8 }

#[repr(C)] #[derive(Clone, Copy)]
pub struct sb_nested_desc { pub physical_type: i32, pub depth: i32, pub list_nullable: [i32; 4],
                            pub item_nullable: i32, pub offset_width: i32, pub struct_mask: i32 }

#[repr(C)]
pub struct sb_nested_out { pub d_offsets: [*mut c_void; 4], pub d_validity: [*mut u8; 4],
                          pub d_values: *mut c_void, pub d_leaf_validity: *mut u8,
                          pub d_leaf_offsets: *mut c_void, pub values_capacity: u64 }

#[repr(C)] #[derive(Clone, Copy)]
pub struct sb_nest_in { pub h_offsets: *const i64, pub h_validity: *const u8 }

#[repr(C)] #[derive(Clone, Copy)]
pub struct sb_write_options {
    pub default_codec: i32, pub has_ratio: i32, pub ratio: f64,
    pub forbidden_mask: u32, pub forced_codec: i32, pub seed: u64,
}

#[link(name = "strawboat_gpu")]
extern "C" {
    pub fn sb_ctx_create(device: c_int, out: *mut *mut sb_ctx) -> i32;
    pub fn sb_ctx_destroy(ctx: *mut sb_ctx);
    pub fn sb_ctx_set_stream(ctx: *mut sb_ctx, hip_stream: *mut c_void) -> i32;
    pub fn sb_sync(ctx: *mut sb_ctx) -> i32;
    pub fn sb_last_error(ctx: *const sb_ctx) -> *const c_char;
    pub fn sb_plan_column(ctx: *mut sb_ctx, desc: *const sb_column_desc, d_chunk: *const u8,
                          chunk_len: u64, metas: *const sb_page_meta, n_pages: u64,
                          out: *mut *mut sb_plan) -> i32;
    pub fn sb_decode_planned(ctx: *mut sb_ctx, plan: *mut sb_plan, out: *const sb_primitive_out) -> i32;
    pub fn sb_plan_status(ctx: *mut sb_ctx, plan: *mut sb_plan, bad_page: *mut i64) -> i32;
    pub fn sb_plan_column_at(ctx: *mut sb_ctx, desc: *const sb_column_desc, d_chunk: *const u8, chunk_len: u64,
                             metas: *const sb_page_meta, n_pages: u64, row_offsets: *const u64,
                             out: *mut *mut sb_plan) -> i32;
    pub fn sb_plan_destroy(plan: *mut sb_plan);
    pub fn sb_plan_num_rows(plan: *const sb_plan) -> u64;
    pub fn sb_plan_values_bytes(plan: *const sb_plan) -> u64;
    pub fn sb_decode_binary_planned(ctx: *mut sb_ctx, plan: *mut sb_plan, out: *const sb_binary_out) -> i32;
    pub fn sb_plan_list_column(ctx: *mut sb_ctx, desc: *const sb_list_desc, d_chunk: *const u8,
                               chunk_len: u64, metas: *const sb_page_meta, n_pages: u64,
                               out: *mut *mut sb_plan) -> i32;
    pub fn sb_plan_num_leaves(plan: *const sb_plan) -> u64;
    pub fn sb_decode_list_planned(ctx: *mut sb_ctx, plan: *mut sb_plan, out: *const sb_list_out) -> i32;
    pub fn sb_decode_column(ctx: *mut sb_ctx, desc: *const sb_column_desc, d_chunk: *const u8,
                            chunk_len: u64, metas: *const sb_page_meta, n_pages: u64,
                            out: *const sb_primitive_out) -> i32;
    pub fn sb_encode_column(physical_type: i32, values: *const c_void, validity: *const u8,
                            n_rows: u64, nullable: i32, opts: *const sb_write_options,
                            max_page_rows: u64, n_threads: i32, out: *mut *mut u8, out_len: *mut u64,
                            metas: *mut *mut sb_page_meta, n_pages: *mut u64) -> i32;
    pub fn sb_encode_binary_column(physical_type: i32, values: *const u8, values_len: u64,
                                   offsets: *const i64, validity: *const u8, n_rows: u64,
                                   nullable: i32, opts: *const sb_write_options, max_page_rows: u64,
                                   n_threads: i32, out: *mut *mut u8, out_len: *mut u64,
                                   metas: *mut *mut sb_page_meta, n_pages: *mut u64) -> i32;
    pub fn sb_encode_list_column(physical_type: i32, offsets: *const i64, list_validity: *const u8,
                                 list_nullable: i32, child: *const c_void, child_validity: *const u8,
                                 item_nullable: i32, n_rows: u64, opts: *const sb_write_options,
                                 max_page_rows: u64, n_threads: i32, out: *mut *mut u8, out_len: *mut u64,
                                 metas: *mut *mut sb_page_meta, n_pages: *mut u64) -> i32;
    pub fn sb_encode_nested_column(desc: *const sb_nested_desc, nests: *const sb_nest_in, values: *const c_void,
                                   leaf_offsets: *const i64, values_len: u64, leaf_validity: *const u8, n_rows: u64,
                                   opts: *const sb_write_options, max_page_rows: u64, n_threads: i32,
                                   out: *mut *mut u8, out_len: *mut u64, metas: *mut *mut sb_page_meta,
                                   n_pages: *mut u64) -> i32;
    pub fn sb_encode_device_bound(physical_type: i32, n_rows: u64, nullable: i32, max_page_rows: u64) -> u64;
    pub fn sb_encode_column_device(ctx: *mut sb_ctx, physical_type: i32, d_values: *const c_void,
                                   d_validity: *const u8, n_rows: u64, nullable: i32,
                                   opts: *const sb_write_options, max_page_rows: u64, d_out: *mut u8,
                                   out_capacity: u64, out_len: *mut u64, metas: *mut sb_page_meta,
                                   metas_cap: u64, n_pages: *mut u64) -> i32;
    pub fn sb_plan_nested_column(ctx: *mut sb_ctx, desc: *const sb_nested_desc, d_chunk: *const u8,
                                 chunk_len: u64, metas: *const sb_page_meta, n_pages: u64,
                                 out: *mut *mut sb_plan) -> i32;
    pub fn sb_plan_nested_count(plan: *const sb_plan, level: i32) -> u64;
    pub fn sb_decode_nested_planned(ctx: *mut sb_ctx, plan: *mut sb_plan, out: *const sb_nested_out) -> i32;
    pub fn sb_encode_binary_device_bound(physical_type: i32, n_rows: u64, values_len: u64, nullable: i32,
                                         max_page_rows: u64) -> u64;
    pub fn sb_encode_binary_column_device(ctx: *mut sb_ctx, physical_type: i32, d_values: *const u8,
                                          values_len: u64, d_offsets: *const i64, d_validity: *const u8,
                                          n_rows: u64, nullable: i32, opts: *const sb_write_options,
                                          max_page_rows: u64, d_out: *mut u8, out_capacity: u64,
                                          out_len: *mut u64, metas: *mut sb_page_meta, metas_cap: u64,
                                          n_pages: *mut u64) -> i32;
    pub fn sb_encode_list_device_bound(physical_type: i32, n_rows: u64, n_child: u64, item_nullable: i32,
                                       max_page_rows: u64) -> u64;
    pub fn sb_encode_list_column_device(ctx: *mut sb_ctx, physical_type: i32, d_offsets: *const i64,
                                        d_list_validity: *const u8, list_nullable: i32, d_child: *const c_void,
                                        d_child_validity: *const u8, item_nullable: i32, n_rows: u64,
                                        opts: *const sb_write_options, max_page_rows: u64, d_out: *mut u8,
                                        out_capacity: u64, out_len: *mut u64, metas: *mut sb_page_meta,
                                        metas_cap: u64, n_pages: *mut u64) -> i32;
    pub fn sb_encode_page(physical_type: i32, values: *const c_void, validity: *const u8, n: u64,
                          nullable: i32, opts: *const sb_write_options, seed: u64, out: *mut *mut u8,
                          out_len: *mut u64) -> i32;
    pub fn sb_page_seed(seed: u64, page: u64) -> u64;
    pub fn sb_lz4_compress_host(src: *const u8, n: u64, dst: *mut u8) -> u64;
    pub fn sb_snappy_compress_host(src: *const u8, n: u64, dst: *mut u8) -> u64;
    pub fn sb_zstd_compress_host(src: *const u8, n: u64, dst: *mut u8) -> u64;
    pub fn sb_decompress_values(ctx: *mut sb_ctx, physical_type: i32, d_stream: *const u8, stream_len: u64,
                                length: u64, d_out: *mut c_void) -> i32;
    pub fn sb_decode_page_validity(ctx: *mut sb_ctx, d_page: *const u8, page_len: u64, length: u64,
                                   d_validity: *mut u32, bit_offset: u64, consumed: *mut u64) -> i32;
    pub fn sb_decode_page_levels(ctx: *mut sb_ctx, d_page: *const u8, page_len: u64, num_levels: u64,
                                 max_rep_level: u32, max_def_level: u32, d_rep: *mut u16, d_def: *mut u16,
                                 rows: *mut u32, consumed: *mut u64) -> i32;
    pub fn sb_ctx_device(ctx: *const sb_ctx) -> i32;
    pub fn sb_plan_enable_timing(plan: *mut sb_plan, on: i32) -> i32;
    pub fn sb_plan_last_kernel_ms(ctx: *mut sb_ctx, plan: *mut sb_plan, ms: *mut f32) -> i32;
    pub fn sb_write_footer(schema: *const u8, schema_len: u64, col_offsets: *const u64,
                           col_npages: *const u64, n_cols: u64, pages: *const sb_page_meta,
                           out: *mut *mut u8, out_len: *mut u64) -> i32;
    pub fn sb_read_meta(file: *const u8, len: u64, col_offsets: *mut u64, col_page_start: *mut u64,
                        cols_cap: u64, pages: *mut sb_page_meta, pages_cap: u64,
                        n_cols: *mut u64, n_pages: *mut u64) -> i32;
    pub fn sb_free(p: *mut c_void);
    pub fn sb_ctx_stream(ctx: *mut sb_ctx) -> *mut c_void;
    pub fn sb_status_str(status: c_int) -> *const c_char;
    pub fn sb_plan_num_pages(plan: *const sb_plan) -> u64;
    // file reader
    pub fn sb_parse_schema(bytes: *const u8, len: u64, leaves: *mut sb_leaf_info, cap: u64,
                           n_leaves: *mut u64, n_fields: *mut u64) -> i32;
    pub fn sb_file_open(path: *const c_char, out: *mut *mut sb_file) -> i32;
    pub fn sb_file_close(f: *mut sb_file);
    pub fn sb_file_last_error(f: *const sb_file) -> *const c_char;
    pub fn sb_file_num_columns(f: *const sb_file) -> u64;
    pub fn sb_file_column(f: *const sb_file, col: u64, offset: *mut u64, chunk_len: *mut u64, n_pages: *mut u64,
                          pages: *mut *const sb_page_meta) -> i32;
    pub fn sb_file_schema(f: *const sb_file, bytes: *mut *const u8, len: *mut u64) -> i32;
    pub fn sb_file_upload(ctx: *mut sb_ctx, f: *mut sb_file, offset: u64, len: u64, d_dst: *mut c_void) -> i32;
}

// The HIP runtime calls the safe layer needs (libamdhip64).
#[link(name = "amdhip64")]
extern "C" {
    pub fn hipMalloc(ptr: *mut *mut c_void, size: usize) -> c_int;
    pub fn hipFree(ptr: *mut c_void) -> c_int;
    pub fn hipMemcpy(dst: *mut c_void, src: *const c_void, size: usize, kind: c_int) -> c_int;
    pub fn hipMemsetAsync(dst: *mut c_void, value: c_int, size: usize, stream: *mut c_void) -> c_int;
    pub fn hipSetDevice(device: c_int) -> c_int;
    pub fn hipGetDevice(device: *mut c_int) -> c_int;
}
pub const HIP_MEMCPY_HOST_TO_DEVICE: c_int = 1;
pub const HIP_MEMCPY_DEVICE_TO_HOST: c_int = 2;
