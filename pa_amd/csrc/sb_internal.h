// sb_internal.h -- host/device shared layout of the MI355X strawboat engine.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <set>
#include <utility>

struct sb_ctx;

namespace sb {

// Grow-only device scratch owned by a context (slot < kCtxScratchSlots),
// reused across calls on its stream; nullptr if the allocation fails.
constexpr int kCtxScratchSlots = 7;
void* ctx_scratch(sb_ctx* ctx, size_t bytes, int slot);
// Records a failure message on the context (sb_last_error) and returns st.
int ctx_fail(sb_ctx* ctx, int st, const char* what, int hip_error = -1);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device: set it once
// for each (kernel, current device) pair before the first launch there.
template <class F>
inline void ensure_lds_attr(F* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  if (done.insert({(const void*)fn, dev}).second)
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// One entry of the device page table.  Built on the host from
// ColumnMeta.pages (src/lib.rs:40-80): byte_off is the running sum of
// PageMeta.length from the column chunk start, row_off the running sum of
// PageMeta.num_values (the position read_integer appends at,
// read/array/integer.rs:225-231).
struct PageDesc {
  uint64_t byte_off;
  uint64_t row_off;
  uint32_t byte_len;
  uint32_t num_values;
  uint64_t reserved;
};
static_assert(sizeof(PageDesc) == 32, "page table entry is 32 bytes");

// PageDesc.reserved of a fixed-width page: its region in the plan's HBM
// region buffer (sb_api plan_regions), 0 = none.  The region holds the
// roaring container tables of a Freq page with more containers than the LDS
// tables take (kRegionRoar, roar_area_bytes), then the area a leaf stream
// too large for the deferred pass's LDS expands into (kRegionSpill,
// spill_area_bytes).
constexpr uint64_t kRegionRoar = 1ull << 62, kRegionSpill = 1ull << 63, kRegionOffMask = (1ull << 56) - 1;
__host__ __device__ constexpr uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }
// containers of a bitmap whose rows are < n
__host__ __device__ constexpr uint64_t roar_cap(uint64_t n) { return (n + 65535) >> 16; }
// keys, data positions, prefix (cap + 1) and bitmap indices (u32), then 64 u16 checkpoints per container
__host__ __device__ constexpr uint64_t roar_area_bytes(uint64_t n) {
  return align16(4 * (4 * roar_cap(n) + 1)) + align16(128 * roar_cap(n));
}
// an expanded leaf: at most n values of max(W, 4) bytes (Dict indices are u32)
__host__ __device__ constexpr uint64_t spill_area_bytes(uint64_t n, uint64_t w) { return align16(n * (w < 4 ? 4 : w)); }

// Per-page kernel status word (the kernel never traps).
enum : uint32_t {
  ST_OK = 0,
  ST_OUT_OF_SPEC = 1,
  ST_NYI = 2,
  ST_IO = 3,
  ST_CODEC = 4,
};

// Pages whose bytes fit this bound are staged whole into LDS; larger pages
// are decoded straight from HBM by the global-source instantiation.
constexpr uint32_t kStageMaxBytes = 48 * 1024;
constexpr uint32_t kStagePad = 64;  // LDS slack for unaligned over-reads

// A general-codec (LZ4 / Snappy) stream expanded by k_inflate, one wave per
// job.  dst: kind in bits 62-63 -- 0 = out + off, 1 = scratch + off,
// 2 = out + bases[off] (a binary page's values base).
struct InflateJob {
  uint64_t src;  // byte offset of the compressed body in the column chunk
  uint64_t dst;
  uint32_t csize, usize;
  uint32_t codec, page;
};
static_assert(sizeof(InflateJob) == 32, "inflate job is 32 bytes");
constexpr uint64_t kDstScratch = 1ull << 62, kDstBinBase = 2ull << 62, kDstBinOffs = 3ull << 62,
                   kDstMask = (1ull << 62) - 1;

struct InflateLaunch {
  const uint8_t* chunk;
  const InflateJob* jobs;
  const uint32_t* count;  // device job count, or nullptr = n_jobs
  uint32_t n_jobs;        // upper bound of the count (sizes the grid)
  uint8_t* out;
  uint8_t* scratch;
  const uint64_t* bases;
  uint32_t* status;
  uint8_t* offs;  // kDstBinOffs jobs: the column's 32-bit offsets (dword-aligned)
  // k_inflate's job claim counters [3], zero between launches, or nullptr:
  // [0] claims, [1] waves done (the last one out resets both), [2] jobs
  // k_patas left to k_inflate (patas_wg: none -> k_inflate returns at once)
  uint32_t* sched;
  uint8_t* ascii;   // binary values jobs: per page, 1 = every byte written was ASCII (else 0), or nullptr
  // the other counter pair of the plan (the next launch's): zeroed at entry,
  // so a launch that never reached its own reset cannot leave the plan's
  // next launch a stale count (the plan alternates the pairs), or nullptr
  uint32_t* sched_spare = nullptr;
  // 1: Patas leaf jobs whose page fits a workgroup's LDS (patas_fits)
  // decode one workgroup a page (k_patas, launched first on the stream; it
  // counts k_inflate's jobs in sched[2]); k_inflate takes the rest
  uint32_t patas_wg = 0;
};
int launch_inflate(const InflateLaunch& a, void* stream);
// Patas leaf pages, one workgroup a page (k_patas, sb_patas.hip): the stream,
// the rows and the walk tables in dynamic LDS.  Pages that do not fit
// (patas_fits) stay with k_inflate's one-wave decoder.
constexpr uint32_t kPatE = 10;        // entry offsets of a segment (a record is <= 10 bytes)
constexpr uint32_t kPatLds = 128 * 1024;  // (leaves a CU room for other kernels' workgroups beside it)
constexpr uint32_t kPatMaxRows = 8192;  // rows of a page k_patas takes (C5's and the writer's default page)
__host__ __device__ inline uint32_t patas_lds_need(uint32_t ilen, uint32_t n, uint32_t W) {
  const uint32_t ib = ((ilen + 62) + 15) & ~15u;  // the stream's 16-byte blocks (+ two for the tail)
  const uint32_t rows = (n + 1) * W > ilen + 16 ? (n + 1) * W : ilen + 16;  // (first the record size table)
  return ib + ((rows + 15) & ~15u) + (((n + 1) * 2 + 15) & ~15u);
}
__host__ __device__ inline bool patas_fits(uint32_t ilen, uint32_t n, uint32_t W) {
  return n >= 1 && n <= kPatMaxRows && ilen >= W && ilen <= 65535 && patas_lds_need(ilen, n, W) <= kPatLds;
}
int launch_patas(const InflateLaunch& a, void* stream);
// Zstd jobs (codec 2) of the same list: one wave per frame, tables in LDS, output in HBM.
int launch_zinflate(const InflateLaunch& a, void* stream);
constexpr uint32_t kInflateGrid = 2048;  // 4-wave workgroups: 8 waves per SIMD on 256 CUs

// Launch entry points (sb_decode.hip).
struct LaunchArgs {
  const uint8_t* chunk;
  const PageDesc* pages;
  const uint32_t* list;  // page indices for this launch, or nullptr = identity
  uint32_t n_list;
  uint8_t* out_values;
  uint32_t* out_validity;  // 32-bit words of the Arrow bitmap
  int nullable;
  uint32_t* status;
  uint32_t stage_bytes;  // dynamic LDS (staged / deferred launches)
  uint32_t* defer_count;  // [2]: work-list lengths, double-buffered by decode parity
  uint32_t* defer_list;   // page indices deferred to k_decode_deferred
  uint32_t parity;
  uint32_t* job_count;    // [2]: inflate job counts, double-buffered like defer_count
  InflateJob* jobs;       // CH_LEAF LZ4 / Snappy pages, expanded by k_inflate
  const uint32_t* light;  // per page: 0, or 1 + validity bitmap position of a header-only page (k_fix_light)
  uint8_t* region;        // the plan's HBM regions (PageDesc.reserved), or nullptr
  uint32_t* spill_count;  // [2]: spilled leaf jobs, double-buffered like defer_count
  InflateJob* spill_jobs; // leaves expanded into regions by k_inflate / k_zinflate, then k_decode_spilled
  uint32_t zstd = 1;      // 0: no page of the plan has a Zstd stream (kernels without the decoder, whose
                          // out-of-line calls would take 245 VGPRs: one wave a SIMD)
};

// kind: 0 = LDS-staged pages, 1 = pages read from HBM, 2 = deferred work list,
// 3 = spilled work list (a.n_list = its upper bound)
int launch_decode_fixed(int width, bool is_float, int kind, const LaunchArgs& a, void* stream);
// Plan time: per listed page (one thread each, from HBM) the cascade bits
// probe[i] = 1 (a Freq in the cascade) | 2 (a general-codec / Patas leaf) |
// 4 (under a Dict / Freq).
int launch_fix_probe(const uint8_t* chunk, const PageDesc* pages, const uint32_t* list, uint32_t n, int width,
                     int nullable, uint32_t* probe, void* stream);
// Header-only fixed-width pages (LZ4 / Snappy leaf, Float Patas leaf): their
// inflate jobs and light[] tags, one thread per page, before the staged pass.
int launch_fix_light(const LaunchArgs& a, uint32_t n_pages, int width, bool is_float, uint32_t* light, void* stream);
// Plan time: *flag |= 1 when a fixed-width or Boolean page (width 1, one
// stream) has a Zstd stream anywhere in its cascade.
int launch_zstd_scan(const uint8_t* chunk, const PageDesc* pages, uint32_t n, int width, int nullable, uint32_t* flag,
                     void* stream);

// Boolean pages: one workgroup per page (grid-strided), page + expanded
// bitmap in a.stage_bytes of dynamic LDS.
int launch_bool(const LaunchArgs& a, void* stream);

// dynamic LDS of the deferred pass: page + expanded stream
constexpr uint32_t kDeferredLds = 155 * 1024;  // + <= 4 KiB of static LDS = the 160 KiB limit
// LDS table area of the one-wave Zstd decoder (sb_zstd.h), carved after the
// expanded stream: the minimum, and enough for a 12-bit Huffman table
constexpr uint32_t kZTablesBytes = 18 * 1024, kZTablesMax = 22 * 1024;
constexpr uint32_t kDeferredGrid = 1024;

// Binary / Utf8 columns: stage 0 = size pages + scan bases, stage 1 = decode.
struct BinLaunch {
  const uint8_t* chunk;
  const PageDesc* pages;
  uint32_t n_pages;
  int nullable;
  uint64_t* sizes;
  uint64_t* bases;
  uint64_t* total;
  uint8_t* out_offsets;
  uint8_t* out_values;
  uint64_t values_cap;
  uint32_t* out_validity;
  uint32_t* status;
  InflateJob* jobs;       // sizing pass out: Basic LZ4 / Snappy streams (2 per page)
  uint32_t* job_count;
  uint8_t* scratch;       // expanded offsets streams, (row_off + page) * offset width
  uint32_t lds_bytes;     // dynamic LDS per workgroup (0 = kDeferredLds)
  uint32_t* lds_need;     // sizing pass at plan time: max LDS bytes any page needs
  uint32_t* cls;          // [4 n_pages + 3]: staged-page list | header-only page list | validity
                          // bitmap positions | big-page list | the three list lengths (reset by stage 0)
  uint32_t staged_grid;   // workgroups of the staged passes (any >= 1 is correct)
  uint8_t* region;        // big Extend pages' tables (PageDesc.reserved = offset + 1), or nullptr
  uint64_t* rneed;        // stage 2 (plan time) out: region bytes per page; lds_need: LDS bytes per page
  uint32_t n_big;         // big pages of the plan (0: their kernels are not launched)
  uint64_t* lb;           // stage 3: look-back states (n_pages) + page counter
  uint32_t zstd = 1;      // 0: no page has a Zstd stream (the kernels without the decoder, LaunchArgs::zstd);
                          // stage 2 reports it through `total` (bit 0 set by a page with a Zstd stream)
  uint8_t* checked = nullptr;  // stage 3, Utf8 plans: per page, 1 = every row it emitted is a whole
                               // entry that is valid UTF-8 (the check skips its bytes), else 0
};
// stage 2: plan-time probe (lds_need / rneed per page); stage 3: the fused
// single pass when every page is staged (sizes, bases, offsets, values).
int launch_binary(int stage, int offset_width, const BinLaunch& a, void* stream);

// Utf8 / LargeUtf8 columns after the decode: the checks of Utf8Array::try_new
// (read/array/binary.rs:305-306; arrow2 0.17 try_check_utf8).  A failure
// marks its page ST_OUT_OF_SPEC; flags[0] must be zero before the launch.
struct Utf8Launch {
  const uint8_t* values;
  uint64_t len;            // values bytes of the column
  const uint8_t* offsets;  // n_rows + 1 offsets of offset_width bytes
  uint64_t n_rows;
  const PageDesc* pages;
  uint32_t n_pages;
  const uint64_t* bases;   // first values byte of each page
  uint32_t* status;
  uint32_t* flags;         // [0]: a non-ASCII byte was seen
  const uint8_t* ascii;    // per page: values known all ASCII (skip), or nullptr = scan everything
};
int launch_utf8_check(int offset_width, const Utf8Launch& a, void* stream);

// List<primitive> columns: stage 0 = exact sizing pass (one wave per page,
// walks the levels); stage 1 = block bases (peek = 1: counts from the page
// headers instead; the plan's check of the headers); stage 4 = counts +
// global bases + values descriptors (blocks exchange their totals through
// `blk`, tagged with `epoch`); stage 2 = offsets + bitmaps (+ values
// descriptors without peek).
struct ListLaunch {
  const uint8_t* chunk;
  const PageDesc* pages;
  uint32_t n_pages;
  uint32_t list_nullable, item_nullable, offset_width;
  uint32_t width, peek;
  uint64_t* counts;
  uint64_t* local;
  uint64_t* blk;
  uint64_t* totals;
  void* lvdesc;  // 32 B per page
  PageDesc* vpages;
  uint8_t* out_offsets;
  uint32_t* out_list_validity;
  uint32_t* out_leaf_validity;
  uint32_t* status;
  uint32_t epoch;             // stage 4: this decode's tag (1..65535) on the block totals
};
constexpr uint32_t kListGrid = 2048;
int launch_list(int stage, const ListLaunch& a, void* stream);

// A leaf under depth (1..4) list levels, the general level walk
// (read_validity_nested with cum_sum / cum_rep): stage 0 counts each page's
// entries per level, stage 1 writes offsets, bitmaps and the values-stream
// descriptors from host-scanned bases.
constexpr int kMaxNest = 4;
struct NestLaunch {
  const uint8_t* chunk;
  const PageDesc* pages;
  uint32_t n_pages;
  uint32_t depth;
  uint32_t nullable;       // bit d: nest d nullable (d < depth); bit depth: the leaf
  uint32_t offset_width;
  uint32_t struct_mask;    // bit d: nest d is a Struct (InitNested::Struct), else a List / Map
  uint64_t* counts;        // [n_pages][depth + 1] entries per level (stage 0 out)
  const uint64_t* bases;   // [n_pages][depth + 1] first entry of each level (stage 1 in)
  const uint64_t* totals;  // [depth + 1]
  PageDesc* vpages;
  uint8_t* out_offsets[kMaxNest];
  uint32_t* out_validity[kMaxNest];
  uint32_t* out_leaf_validity;
  uint32_t* status;
  uint32_t* vpos;          // stage 0 out: each page's values-stream position
};
int launch_nest(int stage, const NestLaunch& a, void* stream);

}  // namespace sb
