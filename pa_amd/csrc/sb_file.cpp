// sb_file.cpp -- the file side of the reader: footer / meta / IPC schema
// parse and the file -> HBM staging pipeline.
//
// Reference: read/reader.rs:148-262 (deserialize_meta, read_meta,
// read_meta_async with its DEFAULT_FOOTER_SIZE pre-read, infer_schema),
// write/writer.rs:128-167 (the footer layout), lib.rs:34-80 (PageMeta,
// ColumnMeta).  The schema bytes are arrow2's schema_to_bytes (write/
// writer.rs:137): an Arrow IPC `Message` flatbuffer whose header is a
// `Schema`; the leaves follow arrow2's to_leaves order (write/common.rs:68),
// the order the file's columns are written in.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/strawboat_gpu.h"

namespace {

// ---------------------------------------------------------------------------
// A bounds-checked flatbuffer reader (tables, vtables, vectors, strings).
struct Fb {
  const uint8_t* b;
  uint64_t n;
  bool ok = true;

  template <class T>
  T rd(uint64_t p) {
    T v{};
    if (p > n || sizeof(T) > n - p) {
      ok = false;
      return v;
    }
    memcpy(&v, b + p, sizeof(T));
    return v;
  }
  // absolute position of scalar / offset field i of the table at t, 0 if absent
  uint64_t field(uint64_t t, int i) {
    const int64_t vt = (int64_t)t - (int64_t)rd<int32_t>(t);
    if (vt < 0 || (uint64_t)vt >= n) {
      ok = false;
      return 0;
    }
    const uint16_t vsz = rd<uint16_t>((uint64_t)vt);
    if ((uint64_t)(4 + 2 * i) + 2 > vsz) return 0;
    const uint16_t o = rd<uint16_t>((uint64_t)vt + 4 + 2 * i);
    return o ? t + o : 0;
  }
  uint64_t deref(uint64_t p) { return p + rd<uint32_t>(p); }
  uint64_t table(uint64_t t, int i) {
    const uint64_t f = field(t, i);
    return f ? deref(f) : 0;
  }
  template <class T>
  T scalar(uint64_t t, int i, T dflt) {
    const uint64_t f = field(t, i);
    return f ? rd<T>(f) : dflt;
  }
  // vector field: element count and position of element 0 (0 if absent)
  uint64_t vec(uint64_t t, int i, uint32_t* len) {
    const uint64_t f = field(t, i);
    *len = 0;
    if (!f) return 0;
    const uint64_t v = deref(f);
    *len = rd<uint32_t>(v);
    if ((uint64_t)*len * 4 > n) ok = false;
    return v + 4;
  }
  std::string str(uint64_t t, int i) {
    uint32_t len;
    const uint64_t p = vec(t, i, &len);
    if (!p || p > n || len > n - p) return std::string();
    return std::string((const char*)b + p, len);
  }
};

// Schem.fbs union tags of Type.
enum : int {
  kNull = 1, kInt = 2, kFloat = 3, kBinary = 4, kUtf8 = 5, kBool = 6, kDecimal = 7, kDate = 8, kTime = 9,
  kTimestamp = 10, kInterval = 11, kList = 12, kStruct = 13, kUnion = 14, kFixedSizeBinary = 15,
  kFixedSizeList = 16, kMap = 17, kDuration = 18, kLargeBinary = 19, kLargeUtf8 = 20, kLargeList = 21,
};

// The reader's physical type of a leaf's logical type (0: no page path).
int32_t leaf_physical(Fb& fb, int tag, uint64_t ty) {
  switch (tag) {
    case kInt: {
      const int32_t bits = ty ? fb.scalar<int32_t>(ty, 0, 0) : 0;
      const bool sgn = ty ? fb.scalar<uint8_t>(ty, 1, 0) != 0 : false;
      switch (bits) {
        case 8: return sgn ? SB_T_INT8 : SB_T_UINT8;
        case 16: return sgn ? SB_T_INT16 : SB_T_UINT16;
        case 32: return sgn ? SB_T_INT32 : SB_T_UINT32;
        case 64: return sgn ? SB_T_INT64 : SB_T_UINT64;
      }
      return 0;
    }
    case kFloat: {
      const int16_t prec = ty ? fb.scalar<int16_t>(ty, 0, 0) : 0;  // HALF 0, SINGLE 1, DOUBLE 2
      return prec == 1 ? SB_T_FLOAT32 : prec == 2 ? SB_T_FLOAT64 : 0;
    }
    case kBinary: return SB_T_BINARY;
    case kUtf8: return SB_T_UTF8;
    case kLargeBinary: return SB_T_LARGE_BINARY;
    case kLargeUtf8: return SB_T_LARGE_UTF8;
    case kBool: return SB_T_BOOLEAN;
    case kDate: return (ty ? fb.scalar<int16_t>(ty, 0, 1) : 1) == 0 ? SB_T_INT32 : SB_T_INT64;  // DAY: i32, MILLISECOND: i64
    case kTime: return (ty ? fb.scalar<int32_t>(ty, 1, 32) : 32) == 32 ? SB_T_INT32 : SB_T_INT64;
    case kTimestamp: case kDuration: return SB_T_INT64;
  }
  return 0;
}

// Flatbuffer child vectors may alias one table many times (a malicious
// footer can make a nest of Structs with two aliased children each visit
// 2^level fields): the walk is capped by the number of fields it visits.
constexpr uint64_t kMaxSchemaFields = 1u << 16;

struct Walk {
  Fb& fb;
  std::vector<sb_leaf_info>& out;
  int top = 0;
  int32_t next_nest = 0;
  bool fail = false;
  uint64_t visits = 0;

  void field(uint64_t f, sb_leaf_info path, int level) {
    if (!f || level > 64 || !fb.ok || ++visits > kMaxSchemaFields) {
      fail = true;
      return;
    }
    const int tag = fb.scalar<uint8_t>(f, 2, 0);
    const uint64_t ty = fb.table(f, 3);
    const bool nullable = fb.scalar<uint8_t>(f, 1, 0) != 0;
    uint32_t nch = 0;
    const uint64_t ch = fb.vec(f, 5, &nch);
    auto child = [&](uint32_t k) { return fb.deref(ch + 4ull * k); };
    // a nest of deserialize_nested's InitNested chain (read/deserialize.rs:
    // 202-230): List / LargeList / FixedSizeList / Map -> InitNested::List,
    // Struct -> InitNested::Struct; ids number the nest fields in pre-order
    // so leaves under one struct or map share theirs
    auto push_nest = [&](bool is_struct) {
      if (path.depth < SB_MAX_NEST) {
        path.list_nullable[path.depth] = nullable;
        path.large_list[path.depth] = tag == kLargeList;
        path.nest_id[path.depth] = next_nest;
        if (is_struct) path.struct_mask |= 1u << path.depth;
        if (tag == kMap) path.map_mask |= 1u << path.depth;
      }
      next_nest++;
      path.depth++;
    };
    if (tag == kList || tag == kLargeList || tag == kFixedSizeList || tag == kMap) {
      if (nch != 1) {
        fail = true;
        return;
      }
      push_nest(false);
      if (tag == kFixedSizeList) path.flags |= SB_LEAF_FIXED_SIZE_LIST;
      if (tag == kMap) path.flags |= SB_LEAF_MAP;
      field(child(0), path, level + 1);
      return;
    }
    if (tag == kStruct) {
      if (nch == 0) {  // a struct without fields has no leaf column (n_columns 0)
        return;
      }
      push_nest(true);
      path.flags |= SB_LEAF_STRUCT;
      for (uint32_t k = 0; k < nch && !fail; k++) field(child(k), path, level + 1);
      return;
    }
    if (tag == kUnion) {
      path.flags |= SB_LEAF_UNION;
      for (uint32_t k = 0; k < nch && !fail; k++) field(child(k), path, level + 1);
      return;
    }
    sb_leaf_info li = path;
    const std::string nm = fb.str(f, 0);
    memset(li.name, 0, sizeof li.name);
    memcpy(li.name, nm.data(), std::min(nm.size(), sizeof li.name - 1));
    li.arrow_type = tag;
    li.physical_type = leaf_physical(fb, tag, ty);
    li.nullable = nullable;
    li.top_field = top;
    if (path.depth > SB_MAX_NEST) li.flags |= SB_LEAF_TOO_DEEP;
    out.push_back(li);
  }
};

bool parse_schema(const uint8_t* bytes, uint64_t len, std::vector<sb_leaf_info>& out, uint64_t* n_top) {
  // arrow2 schema_to_bytes writes the Message flatbuffer; an encapsulated
  // message (pyarrow Schema.serialize) starts with FF FF FF FF + u32 length
  if (len >= 8 && bytes[0] == 0xFF && bytes[1] == 0xFF && bytes[2] == 0xFF && bytes[3] == 0xFF) {
    bytes += 8;
    len -= 8;
  }
  Fb fb{bytes, len};
  const uint64_t msg = fb.deref(0);
  if (!fb.ok || fb.scalar<uint8_t>(msg, 1, 0) != 1) return false;  // MessageHeader.Schema
  const uint64_t sch = fb.table(msg, 2);
  if (!sch || !fb.ok) return false;
  uint32_t nf = 0;
  const uint64_t fv = fb.vec(sch, 1, &nf);
  Walk w{fb, out};
  for (uint32_t k = 0; k < nf && !w.fail; k++) {
    w.top = (int)k;
    sb_leaf_info root{};
    w.field(fb.deref(fv + 4ull * k), root, 0);
  }
  if (n_top) *n_top = nf;
  return fb.ok && !w.fail;
}

// The column metas of the footer's meta block (deserialize_meta, reader.rs:148-166).
bool parse_meta(const uint8_t* m, uint64_t len, std::vector<uint64_t>& col_off, std::vector<uint64_t>& col_start,
                std::vector<sb_page_meta>& pages) {
  uint64_t pos = 0;
  auto rd = [&](uint64_t* v) {
    if (pos + 8 > len) return false;
    memcpy(v, m + pos, 8);
    pos += 8;
    return true;
  };
  uint64_t nc;
  if (!rd(&nc) || nc > len / 16) return false;
  for (uint64_t c = 0; c < nc; c++) {
    uint64_t off, np;
    if (!rd(&off) || !rd(&np) || np > len / 16) return false;
    col_off.push_back(off);
    col_start.push_back(pages.size());
    for (uint64_t i = 0; i < np; i++) {
      sb_page_meta pm;
      if (!rd(&pm.length) || !rd(&pm.num_values)) return false;
      pages.push_back(pm);
    }
  }
  col_start.push_back(pages.size());
  return true;
}

bool pread_all(int fd, uint8_t* dst, uint64_t len, uint64_t off) {
  while (len) {
    const ssize_t r = ::pread(fd, dst, len, (off_t)off);
    if (r <= 0) return false;
    dst += r;
    len -= (uint64_t)r;
    off += (uint64_t)r;
  }
  return true;
}

}  // namespace

struct sb_file {
  int fd = -1;
  uint64_t size = 0;
  std::vector<uint8_t> schema;
  std::vector<uint64_t> col_off, col_start;
  std::vector<sb_page_meta> pages;
  std::string err;
};

namespace {
constexpr uint64_t kFooterPreRead = 64 * 1024;  // DEFAULT_FOOTER_SIZE (read_meta_async, reader.rs:184-188)
constexpr uint64_t kStageChunk = 16ull << 20;    // bytes per pinned staging buffer
constexpr int kReadThreads = 8;                  // pread workers per staging chunk
constexpr int kMaxDevices = 64;

// The staging of one device, shared by every file (allocated on first use,
// kept for the process): two pinned buffers, a copy stream, their events.
struct Staging {
  std::mutex mu;
  bool ready = false;
  uint8_t* pin[2] = {nullptr, nullptr};
  hipStream_t copy = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipEvent_t done = nullptr;
  hipEvent_t before = nullptr;  // the context stream's work queued before an upload
  bool pending[2] = {false, false};
};
Staging g_staging[kMaxDevices];

bool staging_init(Staging& s) {
  if (s.ready) return true;
  bool ok = hipStreamCreateWithFlags(&s.copy, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&s.before, hipEventDisableTiming) == hipSuccess;
  for (int k = 0; k < 2 && ok; k++)
    ok = hipHostMalloc((void**)&s.pin[k], kStageChunk, hipHostMallocDefault) == hipSuccess &&
         hipEventCreateWithFlags(&s.ev[k], hipEventDisableTiming) == hipSuccess;
  s.ready = ok;  // (a failed init is retried on the next call; what was created is kept)
  return ok;
}

sb_status file_fail(sb_file* f, sb_status st, const std::string& what) {
  if (f) f->err = what;
  return st;
}
}  // namespace

extern "C" {

sb_status sb_parse_schema(const uint8_t* h_bytes, uint64_t len, sb_leaf_info* h_leaves, uint64_t cap,
                          uint64_t* n_leaves, uint64_t* n_fields) {
  if (!h_bytes || !n_leaves) return SB_E_ARG;
  std::vector<sb_leaf_info> v;
  if (!parse_schema(h_bytes, len, v, n_fields)) return SB_E_OUT_OF_SPEC;
  *n_leaves = v.size();
  if (h_leaves) memcpy(h_leaves, v.data(), std::min<uint64_t>(cap, v.size()) * sizeof(sb_leaf_info));
  return SB_OK;
}

sb_status sb_file_open(const char* path, sb_file** out) {
  if (!path || !out) return SB_E_ARG;
  *out = nullptr;
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) return SB_E_IO;
  sb_file* f = new sb_file();
  f->fd = fd;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 16) {
    sb_file_close(f);
    return SB_E_IO;
  }
  f->size = (uint64_t)st.st_size;
  // one pre-read of the file's tail; a footer larger than that is read again
  std::vector<uint8_t> tail(std::min(f->size, kFooterPreRead));
  if (!pread_all(fd, tail.data(), tail.size(), f->size - tail.size())) {
    sb_file_close(f);
    return SB_E_IO;
  }
  uint32_t schema_size, meta_size;
  memcpy(&schema_size, tail.data() + tail.size() - 16, 4);
  memcpy(&meta_size, tail.data() + tail.size() - 12, 4);
  const uint64_t footer = 16ull + meta_size + schema_size;
  if (footer > f->size) {
    sb_file_close(f);
    return SB_E_OUT_OF_SPEC;
  }
  if (footer > tail.size()) {
    tail.resize(footer);
    if (!pread_all(fd, tail.data(), footer, f->size - footer)) {
      sb_file_close(f);
      return SB_E_IO;
    }
  }
  const uint8_t* end = tail.data() + tail.size();
  const uint8_t* meta = end - 16 - meta_size;
  f->schema.assign(meta - schema_size, meta);
  if (!parse_meta(meta, meta_size, f->col_off, f->col_start, f->pages)) {
    sb_file_close(f);
    return SB_E_OUT_OF_SPEC;
  }
  *out = f;
  return SB_OK;
}

void sb_file_close(sb_file* f) {
  if (!f) return;
  if (f->fd >= 0) ::close(f->fd);
  delete f;
}

const char* sb_file_last_error(const sb_file* f) { return f ? f->err.c_str() : "null file"; }

uint64_t sb_file_num_columns(const sb_file* f) { return f ? f->col_off.size() : 0; }

sb_status sb_file_column(const sb_file* f, uint64_t col, uint64_t* offset, uint64_t* chunk_len, uint64_t* n_pages,
                         const sb_page_meta** h_pages) {
  if (!f || col >= f->col_off.size()) return SB_E_ARG;
  const uint64_t a = f->col_start[col], b = f->col_start[col + 1];
  uint64_t len = 0;
  for (uint64_t i = a; i < b; i++) {  // overflow-checked: each page bounded by the file
    if (f->pages[i].length > f->size || len > f->size - f->pages[i].length) return SB_E_OUT_OF_SPEC;
    len += f->pages[i].length;
  }
  if (f->col_off[col] > f->size || len > f->size - f->col_off[col]) return SB_E_OUT_OF_SPEC;
  if (offset) *offset = f->col_off[col];
  if (chunk_len) *chunk_len = len;
  if (n_pages) *n_pages = b - a;
  if (h_pages) *h_pages = f->pages.data() + a;
  return SB_OK;
}

sb_status sb_file_schema(const sb_file* f, const uint8_t** h_bytes, uint64_t* len) {
  if (!f || !h_bytes || !len) return SB_E_ARG;
  *h_bytes = f->schema.data();
  *len = f->schema.size();
  return SB_OK;
}

// File bytes [offset, offset + len) -> d_dst, through the device's two
// pinned buffers: the pread of chunk k+1 (kReadThreads workers) overlaps the
// DMA of chunk k on the staging copy stream; the context's stream waits for the last copy,
// so later decodes on it see the bytes while the caller's thread goes on to
// the next column (its reads and copies overlap the decode).
sb_status sb_file_upload(sb_ctx* ctx, sb_file* f, uint64_t offset, uint64_t len, void* d_dst) {
  if (!ctx || !f || (!d_dst && len)) return SB_E_ARG;
  if (offset > f->size || len > f->size - offset) return file_fail(f, SB_E_IO, "range past the end of the file");
  const int dev = sb_ctx_device(ctx);
  if (dev < 0 || dev >= kMaxDevices || hipSetDevice(dev) != hipSuccess) return file_fail(f, SB_E_DEVICE, "device");
  Staging& sg = g_staging[dev];
  std::lock_guard<std::mutex> lock(sg.mu);
  if (!staging_init(sg)) return file_fail(f, SB_E_DEVICE, "staging buffers");
  uint8_t* dst = (uint8_t*)d_dst;
  // The copies run on the staging stream: they must not overwrite d_dst
  // while work queued earlier on the context's stream (a decode still reading
  // a reused chunk buffer, or the caching allocator's previous user of the
  // block) may touch it.
  if (len && (hipEventRecord(sg.before, (hipStream_t)sb_ctx_stream(ctx)) != hipSuccess ||
              hipStreamWaitEvent(sg.copy, sg.before, 0) != hipSuccess))
    return file_fail(f, SB_E_DEVICE, "stream order");
  for (uint64_t done = 0, k = 0; done < len; k++) {
    const int b = (int)(k & 1);
    const uint64_t n = std::min(kStageChunk, len - done);
    if (sg.pending[b] && hipEventSynchronize(sg.ev[b]) != hipSuccess)  // its previous copy has finished
      return file_fail(f, SB_E_DEVICE, "staging event");
    sg.pending[b] = false;
    const uint64_t part = (n + kReadThreads - 1) / kReadThreads;
    bool ok[kReadThreads];
    std::vector<std::thread> th;
    for (int t = 0; t < kReadThreads; t++) {
      const uint64_t a = std::min(n, t * part), e = std::min(n, a + part);
      ok[t] = true;
      if (e > a) th.emplace_back([&, t, a, e] { ok[t] = pread_all(f->fd, sg.pin[b] + a, e - a, offset + done + a); });
    }
    for (auto& x : th) x.join();
    for (int t = 0; t < kReadThreads; t++)
      if (!ok[t]) return file_fail(f, SB_E_IO, "short read");
    if (hipMemcpyAsync(dst + done, sg.pin[b], n, hipMemcpyHostToDevice, sg.copy) != hipSuccess ||
        hipEventRecord(sg.ev[b], sg.copy) != hipSuccess)
      return file_fail(f, SB_E_DEVICE, "staging copy");
    sg.pending[b] = true;
    done += n;
  }
  if (hipEventRecord(sg.done, sg.copy) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)sb_ctx_stream(ctx), sg.done, 0) != hipSuccess)
    return file_fail(f, SB_E_DEVICE, "stream join");
  return SB_OK;
}

}  // extern "C"
