//! Safe Rust over the MI355X strawboat engine (libstrawboat_gpu, gfx950).
//!
//! This is the shim the `strawboat` crate (b41sh/pa 0.2.6) binds to move its
//! codec path onto the GPU while the host side stays Rust:
//!
//! | reference | here |
//! |---|---|
//! | `read::reader::read_meta` / `infer_schema` (src/read/reader.rs:148-262) | [`File::open`], [`File::columns`], [`File::leaves`] |
//! | `NativeReader` page source (src/read/reader.rs:51-146) | [`File::upload`] (pinned double-buffered file -> HBM) |
//! | `batch_read_array` -> `read_integer` / `read_double` / `read_boolean` (src/read/batch_read.rs:190-209) | [`PrimitiveColumn`] |
//! | `read_binary` (src/read/array/binary.rs:223-265) | [`BinaryColumn`] |
//! | `ListIterator` + `read_validity_nested` + `create_list` (src/read/read_basic.rs:65-173, src/read/array/list.rs:48) | [`ListColumn`], [`NestedColumn`] |
//! | `compress_integer` / `encode_chunk` (src/compression/integer/mod.rs:35-347, src/write/common.rs:49-119) | [`encode_column_device`] |
//! | `NativeWriter::finish` footer (src/write/writer.rs:128-167) | [`write_footer`] |
//!
//! Outputs stay in HBM as [`DeviceBuffer`]s laid out as Arrow buffers
//! (values, LSB-first validity bitmaps, i32 / i64 offsets); the caller wraps
//! them into arrow2 arrays or copies them out with [`DeviceBuffer::to_host`].
//! Errors map onto the reference's `arrow2::error::Error` variants
//! (src/errors.rs:19-31) through [`Error`].
pub mod compat;
pub mod ffi;

use std::ffi::{CStr, CString};
use std::marker::PhantomData;
use std::os::raw::c_void;
use std::ptr;

/// arrow2::error::Error analogue: the engine's status codes.
#[derive(Debug, Clone, PartialEq, Eq)]
pub enum Error {
    /// `Error::OutOfSpec`: a malformed page (the reference panics on some).
    OutOfSpec(String),
    /// `Error::NotYetImplemented`.
    NotYetImplemented(String),
    /// `Error::Io` (short read).
    Io(String),
    /// `Error::External` from a codec.
    Codec(String),
    /// `Error::External`: HIP / device failure.
    Device(String),
    /// `Error::InvalidArgumentError`.
    Argument(String),
}

pub type Result<T> = std::result::Result<T, Error>;

fn status(st: i32, msg: impl FnOnce() -> String) -> Result<()> {
    match st {
        0 => Ok(()),
        1 => Err(Error::OutOfSpec(msg())),
        2 => Err(Error::NotYetImplemented(msg())),
        3 => Err(Error::Io(msg())),
        4 => Err(Error::Codec(msg())),
        5 => Err(Error::Device(msg())),
        _ => Err(Error::Argument(msg())),
    }
}

fn cstr(p: *const std::os::raw::c_char) -> String {
    if p.is_null() {
        String::new()
    } else {
        unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
    }
}

/// `crate::PageMeta` (src/lib.rs:75-80).
pub type PageMeta = ffi::sb_page_meta;

/// `crate::ColumnMeta` (src/lib.rs:40-73).
#[derive(Debug, Clone)]
pub struct ColumnMeta {
    pub offset: u64,
    pub pages: Vec<PageMeta>,
}

impl ColumnMeta {
    /// The chunk's bytes (overflow-checked: page lengths come from the file).
    pub fn total_len(&self) -> Result<u64> {
        self.pages
            .iter()
            .try_fold(0u64, |acc, p| acc.checked_add(p.length))
            .ok_or_else(|| Error::OutOfSpec("column chunk length overflows u64".into()))
    }
}

/// Physical types of the page deserializers (sb_physical_type).
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
#[repr(i32)]
pub enum PhysicalType {
    Int8 = 1, Int16 = 2, Int32 = 3, Int64 = 4, UInt8 = 5, UInt16 = 6, UInt32 = 7, UInt64 = 8,
    Float32 = 9, Float64 = 10, Binary = 11, LargeBinary = 12, Utf8 = 13, LargeUtf8 = 14, Boolean = 15,
}

impl PhysicalType {
    pub fn from_i32(v: i32) -> Option<Self> {
        use PhysicalType::*;
        Some(match v {
            1 => Int8, 2 => Int16, 3 => Int32, 4 => Int64, 5 => UInt8, 6 => UInt16, 7 => UInt32, 8 => UInt64,
            9 => Float32, 10 => Float64, 11 => Binary, 12 => LargeBinary, 13 => Utf8, 14 => LargeUtf8,
            15 => Boolean, _ => return None,
        })
    }
    /// Bytes per value of a fixed-width type (0 for Binary / Utf8 / Boolean).
    pub fn width(self) -> usize {
        use PhysicalType::*;
        match self {
            Int8 | UInt8 => 1, Int16 | UInt16 => 2, Int32 | UInt32 | Float32 => 4, Int64 | UInt64 | Float64 => 8,
            _ => 0,
        }
    }
    pub fn is_binary(self) -> bool {
        matches!(self, PhysicalType::Binary | PhysicalType::LargeBinary | PhysicalType::Utf8 | PhysicalType::LargeUtf8)
    }
    pub fn offset_width(self) -> usize {
        if matches!(self, PhysicalType::LargeBinary | PhysicalType::LargeUtf8) { 8 } else { 4 }
    }
}

/// An HBM allocation (hipMalloc) on one device, freed on drop.
pub struct DeviceBuffer {
    ptr: *mut c_void,
    len: usize,
    device: i32,
}

impl DeviceBuffer {
    /// On the thread's current device (prefer [`Context::alloc`]).
    pub fn new(len: usize) -> Result<Self> {
        let mut dev = 0;
        unsafe { ffi::hipGetDevice(&mut dev) };
        let mut p = ptr::null_mut();
        let e = unsafe { ffi::hipMalloc(&mut p, len.max(16)) };
        if e != 0 {
            return Err(Error::Device(format!("hipMalloc({len}) failed: {e}")));
        }
        Ok(DeviceBuffer { ptr: p, len, device: dev })
    }
    /// A zero-filled buffer on the context's device (zeroed on its stream).
    pub fn zeroed(ctx: &Context, len: usize) -> Result<Self> {
        let b = ctx.alloc(len)?;
        let e = unsafe { ffi::hipMemsetAsync(b.ptr, 0, len.max(16), ffi::sb_ctx_stream(ctx.raw)) };
        if e != 0 {
            return Err(Error::Device(format!("hipMemsetAsync failed: {e}")));
        }
        Ok(b)
    }
    pub fn from_host(bytes: &[u8]) -> Result<Self> {
        let b = Self::new(bytes.len())?;
        let e = unsafe { ffi::hipMemcpy(b.ptr, bytes.as_ptr() as *const c_void, bytes.len(), ffi::HIP_MEMCPY_HOST_TO_DEVICE) };
        if e != 0 {
            return Err(Error::Device(format!("hipMemcpy H2D failed: {e}")));
        }
        Ok(b)
    }
    pub fn to_host(&self) -> Result<Vec<u8>> {
        let mut v = vec![0u8; self.len];
        let e = unsafe { ffi::hipMemcpy(v.as_mut_ptr() as *mut c_void, self.ptr, self.len, ffi::HIP_MEMCPY_DEVICE_TO_HOST) };
        if e != 0 {
            return Err(Error::Device(format!("hipMemcpy D2H failed: {e}")));
        }
        Ok(v)
    }
    /// Bytes [offset, offset + len) of the buffer, one D2H copy (clipped to
    /// the allocation).
    pub fn range_to_host(&self, offset: usize, len: usize) -> Result<Vec<u8>> {
        let off = offset.min(self.len);
        let n = len.min(self.len - off);
        let mut v = vec![0u8; len];
        if n == 0 {
            return Ok(v);
        }
        let e = unsafe {
            ffi::hipMemcpy(v.as_mut_ptr() as *mut c_void, (self.ptr as *const u8).add(off) as *const c_void, n,
                           ffi::HIP_MEMCPY_DEVICE_TO_HOST)
        };
        if e != 0 {
            return Err(Error::Device(format!("hipMemcpy D2H failed: {e}")));
        }
        Ok(v)
    }
    pub fn as_ptr(&self) -> *mut c_void {
        self.ptr
    }
    pub fn len(&self) -> usize {
        self.len
    }
    pub fn is_empty(&self) -> bool {
        self.len == 0
    }
    /// The device the buffer was allocated on.
    pub fn device(&self) -> i32 {
        self.device
    }
}

impl Drop for DeviceBuffer {
    fn drop(&mut self) {
        unsafe { ffi::hipFree(self.ptr) };
    }
}

// A device allocation is a plain handle: any thread may read it through
// `&self` (copies out) or free it (hipFree is not tied to a thread), so
// decoded columns can be shared the way arrow2 shares its buffers.
unsafe impl Send for DeviceBuffer {}
unsafe impl Sync for DeviceBuffer {}

/// One device + one HIP stream (`sb_ctx`); not `Sync`, like the reference's
/// single-consumer readers (src/read/reader.rs:51).
pub struct Context {
    raw: *mut ffi::sb_ctx,
}

impl Context {
    pub fn new(device: i32) -> Result<Self> {
        let mut raw = ptr::null_mut();
        status(unsafe { ffi::sb_ctx_create(device, &mut raw) }, || format!("no usable GPU {device}"))?;
        Ok(Context { raw })
    }
    pub fn device(&self) -> i32 {
        unsafe { ffi::sb_ctx_device(self.raw) }
    }
    /// An HBM buffer on this context's device (whatever the thread's current device).
    pub fn alloc(&self, len: usize) -> Result<DeviceBuffer> {
        let e = unsafe { ffi::hipSetDevice(self.device()) };
        if e != 0 {
            return Err(Error::Device(format!("hipSetDevice({}) failed: {e}", self.device())));
        }
        DeviceBuffer::new(len)
    }
    /// Host bytes into an HBM buffer on this context's device.
    pub fn upload(&self, bytes: &[u8]) -> Result<DeviceBuffer> {
        let b = self.alloc(bytes.len())?;
        let e = unsafe { ffi::hipMemcpy(b.ptr, bytes.as_ptr() as *const c_void, bytes.len(), ffi::HIP_MEMCPY_HOST_TO_DEVICE) };
        if e != 0 {
            return Err(Error::Device(format!("hipMemcpy H2D failed: {e}")));
        }
        Ok(b)
    }
    /// A column chunk must live on this context's device.
    fn check_chunk(&self, chunk: &DeviceBuffer) -> Result<()> {
        if chunk.device != self.device() {
            return Err(Error::Argument(format!("chunk on device {} but the context on {}", chunk.device, self.device())));
        }
        Ok(())
    }
    /// Launch on an external hipStream_t.
    pub fn set_stream(&mut self, stream: *mut c_void) -> Result<()> {
        let raw = self.raw;
        status(unsafe { ffi::sb_ctx_set_stream(raw, stream) }, || self.last_error())
    }
    pub fn sync(&self) -> Result<()> {
        status(unsafe { ffi::sb_sync(self.raw) }, || self.last_error())
    }
    pub fn last_error(&self) -> String {
        cstr(unsafe { ffi::sb_last_error(self.raw) })
    }
    pub fn raw(&self) -> *mut ffi::sb_ctx {
        self.raw
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        unsafe { ffi::sb_ctx_destroy(self.raw) };
    }
}

struct Plan {
    raw: *mut ffi::sb_plan,
}

impl Drop for Plan {
    fn drop(&mut self) {
        unsafe { ffi::sb_plan_destroy(self.raw) };
    }
}

fn bitmap_bytes(n: u64) -> usize {
    (((n + 31) / 32) * 4) as usize
}

/// A flat primitive or Boolean leaf: `read_integer` / `read_double` /
/// `read_boolean` over every page, pages appended.
pub struct PrimitiveColumn<'a> {
    ctx: &'a Context,
    plan: Plan,
    ty: PhysicalType,
    nullable: bool,
    // the plan keeps the chunk's device pointer: the chunk must outlive it
    _chunk: PhantomData<&'a DeviceBuffer>,
}

/// Arrow buffers of a decoded flat column.
pub struct Primitive {
    pub values: DeviceBuffer,
    pub validity: Option<DeviceBuffer>,
    pub len: u64,
}

impl<'a> PrimitiveColumn<'a> {
    pub fn plan(ctx: &'a Context, chunk: &'a DeviceBuffer, pages: &[PageMeta], ty: PhysicalType, nullable: bool) -> Result<Self> {
        ctx.check_chunk(chunk)?;
        let desc = ffi::sb_column_desc { physical_type: ty as i32, nullable: nullable as i32 };
        let mut raw = ptr::null_mut();
        status(unsafe {
            ffi::sb_plan_column(ctx.raw, &desc, chunk.ptr as *const u8, chunk.len as u64, pages.as_ptr(), pages.len() as u64, &mut raw)
        }, || ctx.last_error())?;
        Ok(PrimitiveColumn { ctx, plan: Plan { raw }, ty, nullable, _chunk: PhantomData })
    }
    pub fn num_rows(&self) -> u64 {
        unsafe { ffi::sb_plan_num_rows(self.plan.raw) }
    }
    /// Decodes every page (asynchronous on the context's stream) and waits
    /// for the per-page statuses.
    pub fn decode(&self) -> Result<Primitive> {
        let n = self.num_rows();
        let values = if self.ty == PhysicalType::Boolean {
            self.ctx.alloc(bitmap_bytes(n))?
        } else {
            self.ctx.alloc((n as usize) * self.ty.width())?
        };
        let validity = if self.nullable { Some(self.ctx.alloc(bitmap_bytes(n))?) } else { None };
        let out = ffi::sb_primitive_out {
            d_values: values.ptr,
            d_validity: validity.as_ref().map_or(ptr::null_mut(), |b| b.ptr as *mut u8),
        };
        status(unsafe { ffi::sb_decode_planned(self.ctx.raw, self.plan.raw, &out) }, || self.ctx.last_error())?;
        self.check()?;
        Ok(Primitive { values, validity, len: n })
    }
    fn check(&self) -> Result<()> {
        let mut bad = -1i64;
        status(unsafe { ffi::sb_plan_status(self.ctx.raw, self.plan.raw, &mut bad) }, || {
            format!("page {bad}: {}", self.ctx.last_error())
        })
    }
}

/// A Binary / Utf8 leaf: `read_binary`.
pub struct BinaryColumn<'a> {
    ctx: &'a Context,
    plan: Plan,
    ty: PhysicalType,
    nullable: bool,
    // the plan keeps the chunk's device pointer: the chunk must outlive it
    _chunk: PhantomData<&'a DeviceBuffer>,
}

pub struct Binary {
    pub offsets: DeviceBuffer,
    pub values: DeviceBuffer,
    pub validity: Option<DeviceBuffer>,
    pub len: u64,
}

impl<'a> BinaryColumn<'a> {
    pub fn plan(ctx: &'a Context, chunk: &'a DeviceBuffer, pages: &[PageMeta], ty: PhysicalType, nullable: bool) -> Result<Self> {
        ctx.check_chunk(chunk)?;
        if !ty.is_binary() {
            return Err(Error::Argument(format!("{ty:?} is not a binary type")));
        }
        let desc = ffi::sb_column_desc { physical_type: ty as i32, nullable: nullable as i32 };
        let mut raw = ptr::null_mut();
        status(unsafe {
            ffi::sb_plan_column(ctx.raw, &desc, chunk.ptr as *const u8, chunk.len as u64, pages.as_ptr(), pages.len() as u64, &mut raw)
        }, || ctx.last_error())?;
        Ok(BinaryColumn { ctx, plan: Plan { raw }, ty, nullable, _chunk: PhantomData })
    }
    pub fn decode(&self) -> Result<Binary> {
        let n = unsafe { ffi::sb_plan_num_rows(self.plan.raw) };
        let vb = unsafe { ffi::sb_plan_values_bytes(self.plan.raw) };
        let offsets = self.ctx.alloc((n as usize + 1) * self.ty.offset_width())?;
        let values = self.ctx.alloc(vb as usize)?;
        let validity = if self.nullable { Some(self.ctx.alloc(bitmap_bytes(n))?) } else { None };
        let out = ffi::sb_binary_out {
            d_offsets: offsets.ptr,
            d_values: values.ptr as *mut u8,
            values_capacity: vb,
            d_validity: validity.as_ref().map_or(ptr::null_mut(), |b| b.ptr as *mut u8),
        };
        status(unsafe { ffi::sb_decode_binary_planned(self.ctx.raw, self.plan.raw, &out) }, || self.ctx.last_error())?;
        let mut bad = -1i64;
        status(unsafe { ffi::sb_plan_status(self.ctx.raw, self.plan.raw, &mut bad) }, || format!("page {bad}: {}", self.ctx.last_error()))?;
        Ok(Binary { offsets, values, validity, len: n })
    }
}

/// `List<primitive>`: read_validity_nested + create_list, one list level.
pub struct ListColumn<'a> {
    ctx: &'a Context,
    plan: Plan,
    desc: ffi::sb_list_desc,
    ty: PhysicalType,
    _chunk: PhantomData<&'a DeviceBuffer>,
}

pub struct List {
    pub offsets: DeviceBuffer,
    pub list_validity: Option<DeviceBuffer>,
    pub values: DeviceBuffer,
    pub leaf_validity: Option<DeviceBuffer>,
    pub rows: u64,
    pub leaves: u64,
}

impl<'a> ListColumn<'a> {
    pub fn plan(ctx: &'a Context, chunk: &'a DeviceBuffer, pages: &[PageMeta], ty: PhysicalType, list_nullable: bool,
                item_nullable: bool, large: bool) -> Result<Self> {
        ctx.check_chunk(chunk)?;
        let desc = ffi::sb_list_desc {
            physical_type: ty as i32,
            list_nullable: list_nullable as i32,
            item_nullable: item_nullable as i32,
            offset_width: if large { 8 } else { 4 },
        };
        let mut raw = ptr::null_mut();
        status(unsafe {
            ffi::sb_plan_list_column(ctx.raw, &desc, chunk.ptr as *const u8, chunk.len as u64, pages.as_ptr(), pages.len() as u64, &mut raw)
        }, || ctx.last_error())?;
        Ok(ListColumn { ctx, plan: Plan { raw }, desc, ty, _chunk: PhantomData })
    }
    pub fn decode(&self) -> Result<List> {
        let rows = unsafe { ffi::sb_plan_num_rows(self.plan.raw) };
        let leaves = unsafe { ffi::sb_plan_num_leaves(self.plan.raw) };
        let offsets = self.ctx.alloc((rows as usize + 1) * self.desc.offset_width as usize)?;
        let values = self.ctx.alloc(leaves as usize * self.ty.width())?;
        let list_validity = if self.desc.list_nullable != 0 { Some(self.ctx.alloc(bitmap_bytes(rows))?) } else { None };
        let leaf_validity = if self.desc.item_nullable != 0 { Some(self.ctx.alloc(bitmap_bytes(leaves))?) } else { None };
        let out = ffi::sb_list_out {
            d_offsets: offsets.ptr,
            d_list_validity: list_validity.as_ref().map_or(ptr::null_mut(), |b| b.ptr as *mut u8),
            d_values: values.ptr,
            d_leaf_validity: leaf_validity.as_ref().map_or(ptr::null_mut(), |b| b.ptr as *mut u8),
        };
        status(unsafe { ffi::sb_decode_list_planned(self.ctx.raw, self.plan.raw, &out) }, || self.ctx.last_error())?;
        let mut bad = -1i64;
        status(unsafe { ffi::sb_plan_status(self.ctx.raw, self.plan.raw, &mut bad) }, || format!("page {bad}: {}", self.ctx.last_error()))?;
        Ok(List { offsets, list_validity, values, leaf_validity, rows, leaves })
    }
}

/// A leaf under 1..=4 nests -- List / LargeList / Map and Struct nests, the
/// InitNested chain of read/deserialize.rs:140-233 -- of any kind (fixed
/// width, Boolean, Binary / Utf8).
pub struct NestedColumn<'a> {
    ctx: &'a Context,
    plan: Plan,
    desc: ffi::sb_nested_desc,
    ty: PhysicalType,
    _chunk: PhantomData<&'a DeviceBuffer>,
}

pub struct Nested {
    /// Per nest (outermost first): offsets (list / map nests; None for a
    /// struct nest) and optional validity.
    pub offsets: Vec<Option<DeviceBuffer>>,
    pub validity: Vec<Option<DeviceBuffer>>,
    /// Leaf values (fixed width), the leaf bitmap (Boolean) or value bytes (Binary / Utf8).
    pub values: DeviceBuffer,
    pub leaf_offsets: Option<DeviceBuffer>,
    pub leaf_validity: Option<DeviceBuffer>,
    /// Entries per level: counts[0] = rows ... counts[depth] = leaves.
    pub counts: Vec<u64>,
}

impl<'a> NestedColumn<'a> {
    /// `list_nullable[d]`: nest d is nullable; bit d of `struct_mask`: nest d
    /// is a Struct (else a List / Map).
    pub fn plan(ctx: &'a Context, chunk: &'a DeviceBuffer, pages: &[PageMeta], ty: PhysicalType, list_nullable: &[bool],
                item_nullable: bool, large: bool, struct_mask: u32) -> Result<Self> {
        ctx.check_chunk(chunk)?;
        if list_nullable.is_empty() || list_nullable.len() > ffi::SB_MAX_NEST {
            return Err(Error::NotYetImplemented(format!("nesting depth {}", list_nullable.len())));
        }
        if struct_mask >> list_nullable.len() != 0 {
            return Err(Error::Argument(format!("struct mask {struct_mask:#x} past depth {}", list_nullable.len())));
        }
        let mut ln = [0i32; ffi::SB_MAX_NEST];
        for (d, &x) in list_nullable.iter().enumerate() {
            ln[d] = x as i32;
        }
        let desc = ffi::sb_nested_desc {
            physical_type: ty as i32,
            depth: list_nullable.len() as i32,
            list_nullable: ln,
            item_nullable: item_nullable as i32,
            offset_width: if large { 8 } else { 4 },
            struct_mask: struct_mask as i32,
        };
        let mut raw = ptr::null_mut();
        status(unsafe {
            ffi::sb_plan_nested_column(ctx.raw, &desc, chunk.ptr as *const u8, chunk.len as u64, pages.as_ptr(), pages.len() as u64, &mut raw)
        }, || ctx.last_error())?;
        Ok(NestedColumn { ctx, plan: Plan { raw }, desc, ty, _chunk: PhantomData })
    }
    pub fn decode(&self) -> Result<Nested> {
        let depth = self.desc.depth as usize;
        let ow = self.desc.offset_width as usize;
        let counts: Vec<u64> = (0..=depth).map(|d| unsafe { ffi::sb_plan_nested_count(self.plan.raw, d as i32) }).collect();
        let mut out = ffi::sb_nested_out {
            d_offsets: [ptr::null_mut(); ffi::SB_MAX_NEST],
            d_validity: [ptr::null_mut(); ffi::SB_MAX_NEST],
            d_values: ptr::null_mut(),
            d_leaf_validity: ptr::null_mut(),
            d_leaf_offsets: ptr::null_mut(),
            values_capacity: 0,
        };
        let mut offsets = Vec::new();
        let mut validity = Vec::new();
        for d in 0..depth {
            let o = if (self.desc.struct_mask >> d) & 1 == 0 { Some(self.ctx.alloc((counts[d] as usize + 1) * ow)?) } else { None };
            out.d_offsets[d] = o.as_ref().map_or(ptr::null_mut(), |b| b.ptr);
            offsets.push(o);
            let v = if self.desc.list_nullable[d] != 0 { Some(self.ctx.alloc(bitmap_bytes(counts[d]))?) } else { None };
            out.d_validity[d] = v.as_ref().map_or(ptr::null_mut(), |b| b.ptr as *mut u8);
            validity.push(v);
        }
        let leaves = counts[depth];
        let (values, leaf_offsets) = if self.ty.is_binary() {
            let vb = unsafe { ffi::sb_plan_values_bytes(self.plan.raw) };
            // zeroed: with no pages the C decode writes only the level offsets
            let lo = DeviceBuffer::zeroed(self.ctx, (leaves as usize + 1) * self.ty.offset_width())?;
            out.d_leaf_offsets = lo.ptr;
            out.values_capacity = vb;
            (self.ctx.alloc(vb as usize)?, Some(lo))
        } else if self.ty == PhysicalType::Boolean {
            (self.ctx.alloc(bitmap_bytes(leaves))?, None)
        } else {
            (self.ctx.alloc(leaves as usize * self.ty.width())?, None)
        };
        out.d_values = values.ptr;
        let leaf_validity = if self.desc.item_nullable != 0 { Some(self.ctx.alloc(bitmap_bytes(leaves))?) } else { None };
        out.d_leaf_validity = leaf_validity.as_ref().map_or(ptr::null_mut(), |b| b.ptr as *mut u8);
        status(unsafe { ffi::sb_decode_nested_planned(self.ctx.raw, self.plan.raw, &out) }, || self.ctx.last_error())?;
        let mut bad = -1i64;
        status(unsafe { ffi::sb_plan_status(self.ctx.raw, self.plan.raw, &mut bad) }, || format!("page {bad}: {}", self.ctx.last_error()))?;
        Ok(Nested { offsets, validity, values, leaf_offsets, leaf_validity, counts })
    }
}

/// One schema leaf (`sb_leaf_info`), in to_leaves order.
#[derive(Debug, Clone)]
pub struct Leaf {
    pub name: String,
    pub arrow_type: i32,
    pub physical_type: Option<PhysicalType>,
    pub nullable: bool,
    pub list_nullable: Vec<bool>,
    pub large_list: Vec<bool>,
    pub flags: u32,
    pub top_field: i32,
    /// bit d: nest d is a Struct / a Map; nest d's pre-order id in the schema
    pub struct_mask: u32,
    pub map_mask: u32,
    pub nest_id: Vec<i32>,
}

/// `infer_schema` + arrow2 `deserialize_schema`, flattened to leaves.
pub fn parse_schema(bytes: &[u8]) -> Result<Vec<Leaf>> {
    let (mut n, mut nf) = (0u64, 0u64);
    status(unsafe { ffi::sb_parse_schema(bytes.as_ptr(), bytes.len() as u64, ptr::null_mut(), 0, &mut n, &mut nf) },
           || "schema bytes are not an IPC Schema message".into())?;
    let mut raw: Vec<ffi::sb_leaf_info> = Vec::with_capacity(n as usize);
    status(unsafe { ffi::sb_parse_schema(bytes.as_ptr(), bytes.len() as u64, raw.as_mut_ptr(), n, &mut n, &mut nf) },
           || "schema".into())?;
    unsafe { raw.set_len(n as usize) };
    Ok(raw.iter().map(|l| {
        let depth = (l.depth.max(0) as usize).min(ffi::SB_MAX_NEST);
        Leaf {
            name: cstr(l.name.as_ptr()),
            arrow_type: l.arrow_type,
            physical_type: PhysicalType::from_i32(l.physical_type),
            nullable: l.nullable != 0,
            list_nullable: l.list_nullable[..depth].iter().map(|&x| x != 0).collect(),
            large_list: l.large_list[..depth].iter().map(|&x| x != 0).collect(),
            flags: l.flags,
            top_field: l.top_field,
            struct_mask: l.struct_mask,
            map_mask: l.map_mask,
            nest_id: l.nest_id[..depth].to_vec(),
        }
    }).collect())
}

/// An open strawboat file: `read_meta` with the 64 KiB footer pre-read of
/// `read_meta_async`, the schema's leaves, and staged uploads.
pub struct File {
    raw: *mut ffi::sb_file,
}

impl File {
    pub fn open(path: &str) -> Result<Self> {
        let c = CString::new(path).map_err(|_| Error::Argument("path has a NUL byte".into()))?;
        let mut raw = ptr::null_mut();
        status(unsafe { ffi::sb_file_open(c.as_ptr(), &mut raw) }, || format!("cannot read the footer of {path}"))?;
        Ok(File { raw })
    }
    fn err(&self) -> String {
        cstr(unsafe { ffi::sb_file_last_error(self.raw) })
    }
    pub fn columns(&self) -> Result<Vec<ColumnMeta>> {
        let n = unsafe { ffi::sb_file_num_columns(self.raw) };
        (0..n).map(|c| {
            let (mut off, mut len, mut np) = (0u64, 0u64, 0u64);
            let mut pp: *const ffi::sb_page_meta = ptr::null();
            status(unsafe { ffi::sb_file_column(self.raw, c, &mut off, &mut len, &mut np, &mut pp) }, || self.err())?;
            let pages = if np == 0 { Vec::new() } else { unsafe { std::slice::from_raw_parts(pp, np as usize) }.to_vec() };
            Ok(ColumnMeta { offset: off, pages })
        }).collect()
    }
    pub fn schema_bytes(&self) -> Result<Vec<u8>> {
        let (mut p, mut n): (*const u8, u64) = (ptr::null(), 0);
        status(unsafe { ffi::sb_file_schema(self.raw, &mut p, &mut n) }, || self.err())?;
        Ok(if n == 0 { Vec::new() } else { unsafe { std::slice::from_raw_parts(p, n as usize) }.to_vec() })
    }
    pub fn leaves(&self) -> Result<Vec<Leaf>> {
        parse_schema(&self.schema_bytes()?)
    }
    /// Each schema leaf with its column meta (to_leaves order, one to one);
    /// a schema whose leaf count differs from the footer's columns is OutOfSpec.
    pub fn leaf_columns(&self) -> Result<Vec<(Leaf, ColumnMeta)>> {
        let leaves = self.leaves()?;
        let cols = self.columns()?;
        if leaves.len() != cols.len() {
            return Err(Error::OutOfSpec(format!("schema has {} leaves but the footer {} columns", leaves.len(), cols.len())));
        }
        Ok(leaves.into_iter().zip(cols).collect())
    }
    /// Column chunk `col` into HBM (pinned double-buffered; ordered before
    /// later work on the context's stream).
    pub fn upload(&mut self, ctx: &Context, col: &ColumnMeta) -> Result<DeviceBuffer> {
        let len = col.total_len()?;
        let buf = ctx.alloc(len as usize)?;
        status(unsafe { ffi::sb_file_upload(ctx.raw, self.raw, col.offset, len, buf.ptr) }, || self.err())?;
        Ok(buf)
    }
}

impl Drop for File {
    fn drop(&mut self) {
        unsafe { ffi::sb_file_close(self.raw) };
    }
}

/// `WriteOptions` (src/write/common.rs:37-45) + the deterministic sampler seed.
#[derive(Debug, Clone, Copy)]
pub struct WriteOptions {
    pub default_codec: i32,
    pub default_compress_ratio: Option<f64>,
    pub max_page_size: Option<u64>,
    pub forbidden_mask: u32,
    pub forced_codec: Option<i32>,
    pub seed: u64,
}

impl Default for WriteOptions {
    fn default() -> Self {
        WriteOptions { default_codec: 0, default_compress_ratio: None, max_page_size: None, forbidden_mask: 0, forced_codec: None, seed: 0 }
    }
}

impl WriteOptions {
    fn raw(&self) -> ffi::sb_write_options {
        ffi::sb_write_options {
            default_codec: self.default_codec,
            has_ratio: self.default_compress_ratio.is_some() as i32,
            ratio: self.default_compress_ratio.unwrap_or(0.0),
            forbidden_mask: self.forbidden_mask,
            forced_codec: self.forced_codec.unwrap_or(-1),
            seed: self.seed,
        }
    }
}

/// `encode_chunk` of one flat leaf on the device: values (and the LSB
/// validity bitmap) in HBM -> the column chunk in HBM + its page metas.
pub fn encode_column_device(ctx: &Context, ty: PhysicalType, values: &DeviceBuffer, validity: Option<&DeviceBuffer>,
                            n_rows: u64, nullable: bool, opts: &WriteOptions) -> Result<(DeviceBuffer, Vec<PageMeta>)> {
    let page = opts.max_page_size.unwrap_or(0);
    let cap = unsafe { ffi::sb_encode_device_bound(ty as i32, n_rows, nullable as i32, page) };
    let out = ctx.alloc(cap as usize)?;
    let p = opts.max_page_size.unwrap_or(n_rows).min(n_rows).max(1);
    let mut metas = vec![PageMeta { length: 0, num_values: 0 }; ((n_rows + p - 1) / p).max(1) as usize];
    let (mut len, mut np) = (0u64, 0u64);
    let o = opts.raw();
    status(unsafe {
        ffi::sb_encode_column_device(ctx.raw, ty as i32, values.ptr, validity.map_or(ptr::null(), |b| b.ptr as *const u8),
                                     n_rows, nullable as i32, &o, page, out.ptr as *mut u8, cap, &mut len,
                                     metas.as_mut_ptr(), metas.len() as u64, &mut np)
    }, || ctx.last_error())?;
    metas.truncate(np as usize);
    Ok((out, metas))
}

/// `NativeWriter::finish` footer bytes for the given column metas.
pub fn write_footer(schema: &[u8], columns: &[ColumnMeta]) -> Result<Vec<u8>> {
    let offs: Vec<u64> = columns.iter().map(|c| c.offset).collect();
    let nps: Vec<u64> = columns.iter().map(|c| c.pages.len() as u64).collect();
    let pages: Vec<PageMeta> = columns.iter().flat_map(|c| c.pages.iter().copied()).collect();
    let mut out: *mut u8 = ptr::null_mut();
    let mut len = 0u64;
    status(unsafe {
        ffi::sb_write_footer(schema.as_ptr(), schema.len() as u64, offs.as_ptr(), nps.as_ptr(), columns.len() as u64,
                             pages.as_ptr(), &mut out, &mut len)
    }, || "footer".into())?;
    let v = unsafe { std::slice::from_raw_parts(out, len as usize) }.to_vec();
    unsafe { ffi::sb_free(out as *mut c_void) };
    Ok(v)
}

#[cfg(test)]
mod tests {
    use super::*;

    #[test]
    fn status_maps_onto_arrow2_errors() {
        assert_eq!(status(0, || "x".into()), Ok(()));
        assert!(matches!(status(1, || "x".into()), Err(Error::OutOfSpec(_))));
        assert!(matches!(status(2, || "x".into()), Err(Error::NotYetImplemented(_))));
        assert!(matches!(status(3, || "x".into()), Err(Error::Io(_))));
    }

    #[test]
    fn physical_type_widths() {
        assert_eq!(PhysicalType::Int32.width(), 4);
        assert_eq!(PhysicalType::Float64.width(), 8);
        assert_eq!(PhysicalType::LargeUtf8.offset_width(), 8);
        assert_eq!(PhysicalType::from_i32(15), Some(PhysicalType::Boolean));
    }

    /// Needs a gfx950 GPU: decodes a column the engine itself encoded.
    #[test]
    #[ignore]
    fn gpu_round_trip_int32() {
        let ctx = Context::new(0).unwrap();
        let vals: Vec<i32> = (0..100_000).map(|i| (i * 7919) % 4096).collect();
        let bytes: Vec<u8> = vals.iter().flat_map(|v| v.to_le_bytes()).collect();
        let d = DeviceBuffer::from_host(&bytes).unwrap();
        let opts = WriteOptions { default_compress_ratio: Some(1.2), max_page_size: Some(8192), ..Default::default() };
        let (chunk, pages) = encode_column_device(&ctx, PhysicalType::Int32, &d, None, vals.len() as u64, false, &opts).unwrap();
        let col = PrimitiveColumn::plan(&ctx, &chunk, &pages, PhysicalType::Int32, false).unwrap();
        let out = col.decode().unwrap();
        assert_eq!(out.values.to_host().unwrap(), bytes);
    }
}
