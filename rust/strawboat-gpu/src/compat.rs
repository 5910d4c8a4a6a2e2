//! The reference's own API shapes over the engine, so a
//! `strawboat` (b41sh/pa 0.2.6) caller swaps the codec path without touching
//! its call sites:
//!
//! | reference | here |
//! |---|---|
//! | `read::NativeReadBuf` (src/read/mod.rs:26-53) | [`NativeReadBuf`] |
//! | `read::PageIterator` (src/read/mod.rs:55-57) | [`PageIterator`] |
//! | `read::reader::NativeReader::{new, has_next, current_page, skip_page}` + `Iterator` (src/read/reader.rs:51-146) | [`NativeReader`] |
//! | `read::deserialize::{column_iter_to_arrays, ArrayIter}` (src/read/deserialize.rs:237-253) | [`column_iter_to_arrays`], [`ArrayIter`] |
//! | `read::batch_read::batch_read_array` (src/read/batch_read.rs:190-209) | [`batch_read_array`] |
//! | `write::writer::NativeWriter::{try_new, new, into_inner, start, write, finish, total_size}` (src/write/writer.rs:42-173) | [`NativeWriter`] |
//! | `write::WriteOptions` (src/write/common.rs:37-45) | [`WriteOptions`] |
//! | `compression::{Compression, CommonCompression}` (src/compression/mod.rs:37-108, basic.rs:23-60) | [`Compression`], [`CommonCompression`] |
//!
//! Every entry point keeps the reference's parameters, in the reference's
//! order, with the reference's bounds.  Pages are decoded on the calling
//! thread's default engine context ([`default_context`]: one per thread and
//! HIP device, created on first use, as `pa_amd.default_context` does), so no
//! call site passes one.  arrow2 / parquet2 types are stood in for by the
//! minimal [`Field`], [`DataType`], [`ColumnDescriptor`], [`Schema`],
//! [`Chunk`] and [`Array`] below (this crate has no dependencies).  An
//! [`Array`] is a row range of a decoded column whose Arrow buffers stay in
//! HBM; the per-page arrays of [`column_iter_to_arrays`] share one decode of
//! the whole chunk, as arrow2's sliced arrays share their buffers
//! (INTEGRATION.md shows the arrow2 wrapping).
use std::cell::RefCell;
use std::collections::VecDeque;
use std::io::{BufRead, BufReader, Cursor, Read, Seek, SeekFrom, Write};
use std::os::raw::c_void;
use std::ptr;
use std::rc::Rc;
use std::sync::Arc;

use crate::{
    ffi, status, Binary, BinaryColumn, ColumnMeta, Context, DeviceBuffer, Error, List, ListColumn, Nested,
    NestedColumn, PageMeta, PhysicalType, Primitive, PrimitiveColumn, Result,
};

/// `read::NativeReadBuf` (src/read/mod.rs:26-53): a buffered reader that
/// lets the caller peek at its buffered bytes.
pub trait NativeReadBuf: BufRead {
    fn buffer_bytes(&self) -> &[u8];
}

impl<R: Read> NativeReadBuf for BufReader<R> {
    fn buffer_bytes(&self) -> &[u8] {
        self.buffer()
    }
}

impl NativeReadBuf for &[u8] {
    fn buffer_bytes(&self) -> &[u8] {
        self
    }
}

impl<T: AsRef<[u8]>> NativeReadBuf for Cursor<T> {
    fn buffer_bytes(&self) -> &[u8] {
        let len = self.position().min(self.get_ref().as_ref().len() as u64);
        &self.get_ref().as_ref()[(len as usize)..]
    }
}

impl<B: NativeReadBuf + ?Sized> NativeReadBuf for Box<B> {
    fn buffer_bytes(&self) -> &[u8] {
        (**self).buffer_bytes()
    }
}

/// `read::PageIterator` (src/read/mod.rs:55-57): a page source that hands
/// its read buffer back for reuse.
pub trait PageIterator {
    fn swap_buffer(&mut self, buffer: &mut Vec<u8>);
}

thread_local! {
    static DEFAULT_CONTEXTS: RefCell<Vec<Rc<Context>>> = RefCell::new(Vec::new());
}

/// The calling thread's engine context on its current HIP device
/// (`hipSetDevice` picks the device), created on first use and kept for the
/// thread's lifetime.  An `sb_ctx` is one device + one HIP stream and is not
/// shared between threads.
pub fn default_context() -> Result<Rc<Context>> {
    let mut dev = 0;
    let e = unsafe { ffi::hipGetDevice(&mut dev) };
    if e != 0 {
        return Err(Error::Device(format!("hipGetDevice failed: {e}")));
    }
    DEFAULT_CONTEXTS.with(|c| {
        let mut v = c.borrow_mut();
        if let Some(x) = v.iter().find(|x| x.device() == dev) {
            return Ok(x.clone());
        }
        let ctx = Rc::new(Context::new(dev)?);
        v.push(ctx.clone());
        Ok(ctx)
    })
}

/// `read::reader::NativeReader` (src/read/reader.rs:51-146): the pages of
/// one column chunk, read in order from `page_reader` (positioned at the
/// chunk's first page, `ColumnMeta::offset`).
#[derive(Debug)]
pub struct NativeReader<R: NativeReadBuf> {
    page_reader: R,
    page_metas: Vec<PageMeta>,
    current_page: usize,
    scratch: Vec<u8>,
}

impl<R: NativeReadBuf> NativeReader<R> {
    pub fn new(page_reader: R, page_metas: Vec<PageMeta>, scratch: Vec<u8>) -> Self {
        NativeReader { page_reader, page_metas, current_page: 0, scratch }
    }

    /// true while pages remain (reader.rs:70-72).
    pub fn has_next(&self) -> bool {
        self.current_page < self.page_metas.len()
    }

    pub fn current_page(&self) -> usize {
        self.current_page
    }
}

impl<R: NativeReadBuf + Seek> NativeReader<R> {
    /// Skips the next page (reader.rs:134-145).
    pub fn skip_page(&mut self) -> Result<()> {
        if self.current_page == self.page_metas.len() {
            return Ok(());
        }
        let len = self.page_metas[self.current_page].length;
        self.page_reader.seek(SeekFrom::Current(len as i64)).map_err(io)?;
        self.current_page += 1;
        Ok(())
    }
}

impl<R: NativeReadBuf> PageIterator for NativeReader<R> {
    fn swap_buffer(&mut self, scratch: &mut Vec<u8>) {
        std::mem::swap(&mut self.scratch, scratch)
    }
}

impl<R: NativeReadBuf + Seek> Iterator for NativeReader<R> {
    type Item = Result<(u64, Vec<u8>)>;

    /// The next page: (num_values, page bytes) (reader.rs:119-131).
    fn next(&mut self) -> Option<Self::Item> {
        if self.current_page == self.page_metas.len() {
            return None;
        }
        let mut buffer = std::mem::take(&mut self.scratch);
        let meta = self.page_metas[self.current_page];
        buffer.resize(meta.length as usize, 0);
        if let Err(e) = self.page_reader.read_exact(&mut buffer) {
            return Some(Err(io(e)));
        }
        self.current_page += 1;
        Some(Ok((meta.num_values, buffer)))
    }

    /// Skips n pages, then reads one (reader.rs:90-117).
    fn nth(&mut self, n: usize) -> Option<Self::Item> {
        let mut length = 0u64;
        let mut i = 0;
        while i < n && self.current_page < self.page_metas.len() {
            length += self.page_metas[self.current_page].length;
            self.current_page += 1;
            i += 1;
        }
        if i < n {
            return None;
        }
        if length > 0 {
            if let Err(e) = self.page_reader.seek(SeekFrom::Current(length as i64)) {
                return Some(Err(io(e)));
            }
        }
        self.next()
    }
}

/// The arrow2 `DataType`s the page path carries (Union, FixedSizeList and
/// Dictionary are out of scope).
#[derive(Debug, Clone, PartialEq)]
pub enum DataType {
    Boolean,
    Int8,
    Int16,
    Int32,
    Int64,
    UInt8,
    UInt16,
    UInt32,
    UInt64,
    Float32,
    Float64,
    Binary,
    LargeBinary,
    Utf8,
    LargeUtf8,
    List(Box<Field>),
    LargeList(Box<Field>),
    /// arrow2 `DataType::Struct(Vec<Field>)`
    Struct(Vec<Field>),
    /// arrow2 `DataType::Map(entries, keys_sorted)`: `entries` is a
    /// non-nullable Struct field of the key and value fields
    Map(Box<Field>, bool),
}

/// arrow2 `Field`.
#[derive(Debug, Clone, PartialEq)]
pub struct Field {
    pub name: String,
    pub data_type: DataType,
    pub is_nullable: bool,
}

impl Field {
    pub fn new(name: impl Into<String>, data_type: DataType, is_nullable: bool) -> Self {
        Field { name: name.into(), data_type, is_nullable }
    }
}

/// arrow2 `n_columns` (io/parquet/read): the leaf columns a field is
/// written as (to_leaves, write/common.rs:66-71).
pub fn n_columns(data_type: &DataType) -> usize {
    match data_type {
        DataType::List(c) | DataType::LargeList(c) | DataType::Map(c, _) => n_columns(&c.data_type),
        DataType::Struct(fields) => fields.iter().map(|f| n_columns(&f.data_type)).sum(),
        _ => 1,
    }
}

/// arrow2 `is_primitive`: a field read without levels (is_nested false).
fn is_primitive(data_type: &DataType) -> bool {
    !matches!(data_type, DataType::List(_) | DataType::LargeList(_) | DataType::Struct(_) | DataType::Map(_, _))
}

/// parquet2 `ColumnDescriptor`, reduced to what a leaf reader needs.
#[derive(Debug, Clone, Copy, PartialEq)]
pub struct ColumnDescriptor {
    pub physical_type: PhysicalType,
    pub max_def_level: i16,
    pub max_rep_level: i16,
}

/// The Arrow buffers (in HBM) of one decoded column chunk (or, for a field
/// with Struct / Map nests, of its leaf chunks).
pub enum ColumnData {
    Primitive(Primitive),
    Binary(Binary),
    List(List),
    Nested(Nested),
    Field(FieldNode),
}

impl ColumnData {
    /// Top-level rows.
    pub fn rows(&self) -> u64 {
        match self {
            ColumnData::Primitive(p) => p.len,
            ColumnData::Binary(b) => b.len,
            ColumnData::List(l) => l.rows,
            ColumnData::Nested(n) => n.counts[0],
            ColumnData::Field(f) => f.len,
        }
    }
}

/// A decoded field with Struct / Map nests: a tree of views into the
/// per-leaf decodes.  A node's offsets and validity are those its LAST leaf
/// decoded (create_list / create_map / create_struct pop the last child's
/// NestedState, read/array/struct_.rs:101-114, batch_read.rs:128-180); a
/// leaf node's values are its leaf column's.
pub struct FieldNode {
    pub data_type: DataType,
    /// entries of this node (rows at the top)
    pub len: u64,
    source: Arc<Nested>,
    depth: usize,
    pub children: Vec<FieldNode>,
}

impl FieldNode {
    fn is_leaf(&self) -> bool {
        self.depth == self.source.offsets.len()
    }
    /// The node's validity bitmap (32-bit words, LSB first), None when the
    /// field is not nullable.
    pub fn validity(&self) -> Option<&DeviceBuffer> {
        if self.is_leaf() {
            self.source.leaf_validity.as_ref()
        } else {
            self.source.validity[self.depth].as_ref()
        }
    }
    /// A List / Map node's offsets (len + 1 entries).
    pub fn offsets(&self) -> Option<&DeviceBuffer> {
        if self.is_leaf() {
            None
        } else {
            self.source.offsets[self.depth].as_ref()
        }
    }
    /// A leaf node's values: fixed-width values, a Boolean bitmap, or the
    /// value bytes of a Binary / Utf8 leaf (with [`FieldNode::leaf_offsets`]).
    pub fn values(&self) -> Option<&DeviceBuffer> {
        if self.is_leaf() {
            Some(&self.source.values)
        } else {
            None
        }
    }
    pub fn leaf_offsets(&self) -> Option<&DeviceBuffer> {
        if self.is_leaf() {
            self.source.leaf_offsets.as_ref()
        } else {
            None
        }
    }
}

/// arrow2 `Box<dyn Array>`: rows [offset, offset + len) of a decoded column.
/// Like arrow2's sliced arrays it is a view: the per-page arrays of one
/// column share its buffers; `offset` is the first row's index into them
/// (the bit offset of its validity and Boolean values, the index of its first
/// offset).
#[derive(Clone)]
pub struct Array {
    data_type: DataType,
    data: Arc<ColumnData>,
    offset: u64,
    len: u64,
}

impl Array {
    pub fn data_type(&self) -> &DataType {
        &self.data_type
    }
    pub fn data(&self) -> &ColumnData {
        &self.data
    }
    pub fn offset(&self) -> u64 {
        self.offset
    }
    pub fn len(&self) -> usize {
        self.len as usize
    }
    pub fn is_empty(&self) -> bool {
        self.len == 0
    }
    /// arrow2 `Array::sliced`: rows [offset, offset + length) of this array.
    pub fn sliced(&self, offset: usize, length: usize) -> Array {
        assert!(offset as u64 + length as u64 <= self.len, "the offset of the new array cannot exceed the existing length");
        Array { data_type: self.data_type.clone(), data: self.data.clone(), offset: self.offset + offset as u64, len: length as u64 }
    }

    /// The array's rows as host Arrow buffers, shaped like the reference's
    /// `Box<dyn Array>` (batch_read.rs:190-209 returns host arrays): values,
    /// offsets rebased to start at 0, LSB-first bitmaps at bit 0 -- one D2H
    /// copy per buffer range.  Lists / maps carry only the child slots their
    /// rows reach; a struct's children its rows.
    pub fn to_host(&self) -> Result<HostArray> {
        let (b, e) = (self.offset, self.offset + self.len);
        match self.data.as_ref() {
            ColumnData::Primitive(p) => {
                let ty = leaf_type(&self.data_type);
                let values = if ty == PhysicalType::Boolean {
                    bits_to_host(&p.values, b, self.len)?
                } else {
                    let w = ty.width();
                    p.values.range_to_host(b as usize * w, self.len as usize * w)?
                };
                Ok(HostArray::Primitive { values, validity: opt_bits(&p.validity, b, self.len)?, len: self.len })
            }
            ColumnData::Binary(x) => {
                let ty = leaf_type(&self.data_type);
                binary_to_host(&x.offsets, ty.offset_width(), &x.values, &x.validity, b, e)
            }
            ColumnData::List(l) => {
                let ow = if matches!(self.data_type, DataType::LargeList(_)) { 8 } else { 4 };
                let offs = offsets_to_host(&l.offsets, ow, b, e)?;
                let (c0, c1) = (offs[0] as u64, offs[offs.len() - 1] as u64);
                let DataType::List(item) | DataType::LargeList(item) = &self.data_type else {
                    unreachable!("a List column has a list type")
                };
                let w = leaf_type(&item.data_type).width();
                let child = HostArray::Primitive {
                    values: l.values.range_to_host(c0 as usize * w, (c1 - c0) as usize * w)?,
                    validity: opt_bits(&l.leaf_validity, c0, c1 - c0)?,
                    len: c1 - c0,
                };
                Ok(HostArray::List { offsets: rebase(offs), validity: opt_bits(&l.list_validity, b, self.len)?,
                                     values: Box::new(child), len: self.len })
            }
            ColumnData::Nested(n) => chain_to_host(&self.data_type, n, 0, b, e),
            ColumnData::Field(f) => node_to_host(f, b, e),
        }
    }
}

/// Bits [bit0, bit0 + n) of a device bitmap, re-based to bit 0.
fn bits_to_host(buf: &DeviceBuffer, bit0: u64, n: u64) -> Result<Vec<u8>> {
    let first = (bit0 / 8) as usize;
    let raw = buf.range_to_host(first, ((bit0 % 8 + n + 7) / 8) as usize)?;
    let sh = (bit0 % 8) as u32;
    let mut out = vec![0u8; ((n + 7) / 8) as usize];
    for (i, o) in out.iter_mut().enumerate() {
        let lo = raw[i] >> sh;
        let hi = if sh > 0 && i + 1 < raw.len() { raw[i + 1] << (8 - sh) } else { 0 };
        *o = lo | hi;
    }
    if n % 8 != 0 {
        let last = out.len() - 1;
        out[last] &= (1u8 << (n % 8)) - 1;
    }
    Ok(out)
}

fn opt_bits(buf: &Option<DeviceBuffer>, bit0: u64, n: u64) -> Result<Option<Vec<u8>>> {
    buf.as_ref().map(|b| bits_to_host(b, bit0, n)).transpose()
}

/// Offsets [b, e] (e - b + 1 entries of `width` bytes) as i64.
fn offsets_to_host(buf: &DeviceBuffer, width: usize, b: u64, e: u64) -> Result<Vec<i64>> {
    let raw = buf.range_to_host(b as usize * width, (e - b + 1) as usize * width)?;
    Ok(raw
        .chunks_exact(width)
        .map(|c| if width == 8 { i64::from_le_bytes(c.try_into().unwrap()) } else { i32::from_le_bytes(c.try_into().unwrap()) as i64 })
        .collect())
}

fn rebase(mut offs: Vec<i64>) -> Vec<i64> {
    let o0 = offs[0];
    offs.iter_mut().for_each(|x| *x -= o0);
    offs
}

fn binary_to_host(offsets: &DeviceBuffer, width: usize, values: &DeviceBuffer, validity: &Option<DeviceBuffer>, b: u64,
                  e: u64) -> Result<HostArray> {
    let offs = offsets_to_host(offsets, width, b, e)?;
    let (v0, v1) = (offs[0] as usize, offs[offs.len() - 1] as usize);
    Ok(HostArray::Binary { values: values.range_to_host(v0, v1 - v0)?, offsets: rebase(offs),
                           validity: opt_bits(validity, b, e - b)?, len: e - b })
}

/// A leaf of a nested decode, slots [b, e).
fn leaf_to_host(ty: PhysicalType, n: &Nested, b: u64, e: u64) -> Result<HostArray> {
    if ty.is_binary() {
        let lo = n.leaf_offsets.as_ref().ok_or_else(|| Error::OutOfSpec("binary leaf without offsets".into()))?;
        return binary_to_host(lo, ty.offset_width(), &n.values, &n.leaf_validity, b, e);
    }
    let values = if ty == PhysicalType::Boolean {
        bits_to_host(&n.values, b, e - b)?
    } else {
        n.values.range_to_host(b as usize * ty.width(), (e - b) as usize * ty.width())?
    };
    Ok(HostArray::Primitive { values, validity: opt_bits(&n.leaf_validity, b, e - b)?, len: e - b })
}

/// Nest `depth` of a list-only chain decode, entries [b, e).
fn chain_to_host(dt: &DataType, n: &Nested, depth: usize, b: u64, e: u64) -> Result<HostArray> {
    match dt {
        DataType::List(c) | DataType::LargeList(c) | DataType::Map(c, _) => {
            let buf = n.offsets[depth].as_ref().ok_or_else(|| Error::OutOfSpec("list nest without offsets".into()))?;
            let width = buf.len() / (n.counts[depth] as usize + 1);
            let offs = offsets_to_host(buf, width, b, e)?;
            let (c0, c1) = (offs[0] as u64, offs[offs.len() - 1] as u64);
            let child = Box::new(chain_to_host(&c.data_type, n, depth + 1, c0, c1)?);
            let validity = opt_bits(&n.validity[depth], b, e - b)?;
            Ok(if matches!(dt, DataType::Map(_, _)) {
                HostArray::Map { offsets: rebase(offs), validity, field: child, len: e - b }
            } else {
                HostArray::List { offsets: rebase(offs), validity, values: child, len: e - b }
            })
        }
        DataType::Struct(_) => Err(Error::OutOfSpec("a struct nest in a one-leaf chain".into())),
        leaf => leaf_to_host(leaf_type(leaf), n, b, e),
    }
}

/// A node of a Struct / Map field decode, entries [b, e).
fn node_to_host(node: &FieldNode, b: u64, e: u64) -> Result<HostArray> {
    let validity = || node.validity().map(|v| bits_to_host(v, b, e - b)).transpose();
    match &node.data_type {
        DataType::Struct(_) => {
            let validity = validity()?;
            let values = node.children.iter().map(|c| node_to_host(c, b, e)).collect::<Result<Vec<_>>>()?;
            Ok(HostArray::Struct { values, validity, len: e - b })
        }
        DataType::List(_) | DataType::LargeList(_) | DataType::Map(_, _) => {
            let buf = node.offsets().ok_or_else(|| Error::OutOfSpec("list nest without offsets".into()))?;
            let width = buf.len() / (node.len as usize + 1);
            let offs = offsets_to_host(buf, width, b, e)?;
            let (c0, c1) = (offs[0] as u64, offs[offs.len() - 1] as u64);
            let child = Box::new(node_to_host(&node.children[0], c0, c1)?);
            let validity = validity()?;
            Ok(if matches!(node.data_type, DataType::Map(_, _)) {
                HostArray::Map { offsets: rebase(offs), validity, field: child, len: e - b }
            } else {
                HostArray::List { offsets: rebase(offs), validity, values: child, len: e - b }
            })
        }
        leaf => leaf_to_host(leaf_type(leaf), &node.source, b, e),
    }
}

/// `read::ArrayIter` (src/read/deserialize.rs): the arrays of a column, one
/// per page.
pub type ArrayIter<'a> = Box<dyn Iterator<Item = Result<Array>> + Send + Sync + 'a>;

/// One nest of a leaf's InitNested chain (read/deserialize.rs:202-230): a
/// List / LargeList / Map pushes InitNested::List, a Struct
/// InitNested::Struct, each with the nest field's nullability.
#[derive(Debug, Clone, Copy, PartialEq)]
struct Nest {
    is_struct: bool,
    nullable: bool,
    large: bool,
}

/// One leaf column of a field: its physical type, its nest chain (outermost
/// first) and its own nullability.
#[derive(Debug, Clone, PartialEq)]
struct LeafChain {
    ty: PhysicalType,
    nests: Vec<Nest>,
    nullable: bool,
}

fn leaf_type(dt: &DataType) -> PhysicalType {
    use PhysicalType as P;
    match dt {
        DataType::Boolean => P::Boolean,
        DataType::Int8 => P::Int8,
        DataType::Int16 => P::Int16,
        DataType::Int32 => P::Int32,
        DataType::Int64 => P::Int64,
        DataType::UInt8 => P::UInt8,
        DataType::UInt16 => P::UInt16,
        DataType::UInt32 => P::UInt32,
        DataType::UInt64 => P::UInt64,
        DataType::Float32 => P::Float32,
        DataType::Float64 => P::Float64,
        DataType::Binary => P::Binary,
        DataType::LargeBinary => P::LargeBinary,
        DataType::Utf8 => P::Utf8,
        DataType::LargeUtf8 => P::LargeUtf8,
        DataType::List(_) | DataType::LargeList(_) | DataType::Struct(_) | DataType::Map(_, _) => {
            unreachable!("a nest is not a leaf")
        }
    }
}

/// deserialize_nested's walk (read/deserialize.rs:140-233): the leaves of
/// `field` in to_leaves order, each with its InitNested chain.
fn leaf_chains(field: &Field) -> Vec<LeafChain> {
    fn walk(f: &Field, nests: &mut Vec<Nest>, out: &mut Vec<LeafChain>) {
        match &f.data_type {
            DataType::List(c) | DataType::LargeList(c) | DataType::Map(c, _) => {
                let large = matches!(f.data_type, DataType::LargeList(_));
                nests.push(Nest { is_struct: false, nullable: f.is_nullable, large });
                walk(c, nests, out);
                nests.pop();
            }
            DataType::Struct(fields) => {
                nests.push(Nest { is_struct: true, nullable: f.is_nullable, large: false });
                for c in fields {
                    walk(c, nests, out);
                }
                nests.pop();
            }
            dt => out.push(LeafChain { ty: leaf_type(dt), nests: nests.clone(), nullable: f.is_nullable }),
        }
    }
    let mut out = Vec::new();
    walk(field, &mut Vec::new(), &mut out);
    out
}

/// The one leaf under a field without Struct / Map nests: its physical type,
/// per list level (outermost first) the level's nullability and whether it
/// is a LargeList, and the leaf's own nullability.
fn leaf_path(field: &Field) -> Result<(PhysicalType, Vec<bool>, Vec<bool>, bool)> {
    let mut chains = leaf_chains(field);
    if chains.len() != 1 || chains[0].nests.iter().any(|n| n.is_struct) {
        return Err(Error::NotYetImplemented(format!("{}: a field with Struct / Map nests has no one-leaf path", field.name)));
    }
    let c = chains.pop().unwrap();
    Ok((c.ty, c.nests.iter().map(|n| n.nullable).collect(), c.nests.iter().map(|n| n.large).collect(), c.nullable))
}

/// The read/deserialize.rs dispatch over one column chunk in HBM: flat
/// primitive / Boolean, Binary / Utf8, List<primitive>, or any other list
/// nesting (depth 1..=4, every leaf kind).  Returns once the decode has
/// finished (the per-page statuses are read back).
fn decode_chunk(ctx: &Context, chunk: &DeviceBuffer, pages: &[PageMeta], field: &Field) -> Result<ColumnData> {
    let (ty, lists, large, leaf_nullable) = leaf_path(field)?;
    if lists.is_empty() {
        return if ty.is_binary() {
            Ok(ColumnData::Binary(BinaryColumn::plan(ctx, chunk, pages, ty, leaf_nullable)?.decode()?))
        } else {
            Ok(ColumnData::Primitive(PrimitiveColumn::plan(ctx, chunk, pages, ty, leaf_nullable)?.decode()?))
        };
    }
    if large.iter().any(|&l| l != large[0]) {
        return Err(Error::NotYetImplemented(format!("{}: mixed List / LargeList levels", field.name)));
    }
    if lists.len() == 1 && !ty.is_binary() && ty != PhysicalType::Boolean {
        let c = ListColumn::plan(ctx, chunk, pages, ty, lists[0], leaf_nullable, large[0])?;
        return Ok(ColumnData::List(c.decode()?));
    }
    let c = NestedColumn::plan(ctx, chunk, pages, ty, &lists, leaf_nullable, large[0], 0)?;
    Ok(ColumnData::Nested(c.decode()?))
}

/// A field's leaf chunks in HBM (to_leaves order) decoded: one chunk without
/// Struct / Map nests through [`decode_chunk`]; otherwise each leaf through
/// its InitNested chain (sb_plan_nested_column with a struct mask), then the
/// tree assembled as deserialize_nested does.
fn decode_field(ctx: &Context, chunks: &[DeviceBuffer], pages: &[Vec<PageMeta>], field: &Field) -> Result<ColumnData> {
    let chains = leaf_chains(field);
    if chains.len() != chunks.len() || chunks.len() != pages.len() {
        return Err(Error::Argument(format!("{}: {} leaf columns, {} chunks, {} page lists", field.name, chains.len(),
                                           chunks.len(), pages.len())));
    }
    if chains.len() == 1 && chains[0].nests.iter().all(|n| !n.is_struct) {
        return decode_chunk(ctx, &chunks[0], &pages[0], field);
    }
    let mut decoded = Vec::with_capacity(chains.len());
    for ((c, chunk), p) in chains.iter().zip(chunks).zip(pages) {
        let lists: Vec<bool> = c.nests.iter().filter(|n| !n.is_struct).map(|n| n.large).collect();
        let large = lists.first().copied().unwrap_or(false);
        if lists.iter().any(|&l| l != large) {
            return Err(Error::NotYetImplemented(format!("{}: mixed List / LargeList levels", field.name)));
        }
        let nullable: Vec<bool> = c.nests.iter().map(|n| n.nullable).collect();
        let mask = c.nests.iter().enumerate().filter(|(_, n)| n.is_struct).fold(0u32, |m, (d, _)| m | (1u32 << d));
        let col = NestedColumn::plan(ctx, chunk, p, c.ty, &nullable, c.nullable, large, mask)?;
        decoded.push(Arc::new(col.decode()?));
    }
    Ok(ColumnData::Field(assemble(field, &decoded, 0)?))
}

/// create_struct / create_map / create_list over the leaf decodes under
/// `f` (its nest is at `depth` of their chains): the last leaf's nest, after
/// checking that every leaf under it counted the same entries (StructArray's
/// children must be as long as it is).
fn assemble(f: &Field, leaves: &[Arc<Nested>], depth: usize) -> Result<FieldNode> {
    let last = leaves.last().ok_or_else(|| Error::OutOfSpec(format!("{}: a Struct without fields", f.name)))?;
    let len = last.counts[depth];
    if leaves.iter().any(|l| l.counts[depth] != len) {
        return Err(Error::OutOfSpec(format!("{}: its leaf columns disagree on the entries of a nest", f.name)));
    }
    let children = match &f.data_type {
        DataType::List(c) | DataType::LargeList(c) | DataType::Map(c, _) => vec![assemble(c, leaves, depth + 1)?],
        DataType::Struct(fields) => {
            let mut v = Vec::with_capacity(fields.len());
            let mut k = 0;
            for c in fields {
                let n = n_columns(&c.data_type);
                if k + n > leaves.len() {
                    return Err(Error::OutOfSpec(format!("{}: fewer leaf columns than fields", f.name)));
                }
                v.push(assemble(c, &leaves[k..k + n], depth + 1)?);
                k += n;
            }
            v
        }
        _ => Vec::new(),
    };
    Ok(FieldNode { data_type: f.data_type.clone(), len, source: last.clone(), depth, children })
}

/// A field's leaf chunk bytes into HBM on the thread's default context, decoded.
fn decode_host_chunks(chunks: &[Vec<u8>], pages: &[Vec<PageMeta>], field: &Field) -> Result<ColumnData> {
    let ctx = default_context()?;
    let bufs = chunks.iter().map(|b| ctx.upload(b)).collect::<Result<Vec<_>>>()?;
    decode_field(&ctx, &bufs, pages, field)
}

/// The leaves the caller passes must be the field's (to_leaves order).
fn check_leaves(leaves: &[ColumnDescriptor], field: &Field) -> Result<()> {
    let chains = leaf_chains(field);
    if leaves.len() != chains.len() {
        return Err(Error::OutOfSpec(format!("{}: {} leaves for {} leaf columns", field.name, leaves.len(), chains.len())));
    }
    for (l, c) in leaves.iter().zip(&chains) {
        if l.physical_type != c.ty {
            return Err(Error::OutOfSpec(format!("{}: leaf type {:?} against field {:?}", field.name, l.physical_type, c.ty)));
        }
    }
    Ok(())
}

fn check_nested(is_nested: bool, field: &Field) -> Result<()> {
    if is_nested == is_primitive(&field.data_type) {
        return Err(Error::Argument(format!("{}: is_nested {is_nested} against its data type", field.name)));
    }
    Ok(())
}

/// `batch_read_array` (src/read/batch_read.rs:190-209): every page of the
/// field's leaf columns at once, one array.  Each leaf's pages are read from
/// its reader in one read, staged into HBM with one copy and decoded there.
pub fn batch_read_array<R: NativeReadBuf>(
    mut readers: Vec<R>,
    leaves: Vec<ColumnDescriptor>,
    field: Field,
    is_nested: bool,
    page_metas: Vec<Vec<PageMeta>>,
) -> Result<Array> {
    check_leaves(&leaves, &field)?;
    check_nested(is_nested, &field)?;
    if readers.len() != leaves.len() || page_metas.len() != leaves.len() {
        return Err(Error::Argument(format!("{}: {} readers and {} page lists for {} leaves", field.name, readers.len(),
                                           page_metas.len(), leaves.len())));
    }
    let mut chunks = Vec::with_capacity(readers.len());
    for (reader, metas) in readers.iter_mut().zip(&page_metas) {
        let len = ColumnMeta { offset: 0, pages: metas.clone() }.total_len()?;
        let len = usize::try_from(len).map_err(|_| Error::OutOfSpec("column chunk larger than the address space".into()))?;
        let mut bytes = vec![0u8; len];
        reader.read_exact(&mut bytes).map_err(io)?;
        chunks.push(bytes);
    }
    let data = decode_host_chunks(&chunks, &page_metas, &field)?;
    let len = data.rows();
    Ok(Array { data_type: field.data_type, data: Arc::new(data), offset: 0, len })
}

/// The rows of a nested page: its `u32 rows` header (write_nested_validity,
/// serialize.rs:217-232; read_validity_nested, read_basic.rs:72).
fn nested_page_rows(page: &[u8]) -> Result<u64> {
    if page.len() < 4 {
        return Err(Error::OutOfSpec("nested page shorter than its header".into()));
    }
    Ok(u32::from_le_bytes([page[0], page[1], page[2], page[3]]) as u64)
}

/// Pages decoded per launch by the streaming iterator: enough to fill the
/// chip (one workgroup per page), few enough that memory stays bounded by the
/// range, not the chunk.
const RANGE_PAGES: usize = 64;

/// The iterator `column_iter_to_arrays` returns: page-at-a-time semantics
/// (read/deserialize.rs:237-253 yields one array per page) decoded in ranges
/// of [`RANGE_PAGES`] pages.  Each `next()` that finds no decoded page left
/// reads the next range from every leaf reader (handing each page buffer
/// back through `swap_buffer`), stages it into HBM with one copy per leaf,
/// decodes it in one launch and queues one array per page.  A bad page k of a
/// range is found by decoding the range's pages one by one: the arrays of
/// the pages before it come back first, then its error -- the order the
/// reference's page iterator returns them in.
struct PageArrays<I> {
    readers: Vec<I>,
    field: Field,
    is_nested: bool,
    ready: VecDeque<Result<Array>>,
    done: bool,
}

/// One range of pages of every leaf column: bytes, metas, rows per page.
struct PageRange {
    chunks: Vec<Vec<u8>>,
    metas: Vec<Vec<PageMeta>>,
    rows: Vec<u64>,
}

impl<I> PageArrays<I>
where
    I: Iterator<Item = Result<(u64, Vec<u8>)>> + PageIterator,
{
    /// Up to RANGE_PAGES pages of every reader; the error of a page that
    /// could not be read comes back after the pages before it.
    fn read_range(&mut self) -> (PageRange, Option<Error>) {
        let mut r = PageRange { chunks: Vec::new(), metas: Vec::new(), rows: Vec::new() };
        let mut err = None;
        let mut n_pages = RANGE_PAGES;
        for (k, reader) in self.readers.iter_mut().enumerate() {
            let (mut bytes, mut metas, mut rows) = (Vec::new(), Vec::new(), Vec::new());
            while metas.len() < n_pages {
                let Some(page) = reader.next() else { break };
                let (num_values, mut buf) = match page {
                    Ok(p) => p,
                    Err(e) => {
                        err = Some(e);
                        break;
                    }
                };
                let rows_here = if self.is_nested {
                    match nested_page_rows(&buf) {
                        Ok(x) => x,
                        Err(e) => {
                            err = Some(e);
                            break;
                        }
                    }
                } else {
                    num_values
                };
                rows.push(rows_here);
                metas.push(PageMeta { length: buf.len() as u64, num_values });
                bytes.extend_from_slice(&buf);
                reader.swap_buffer(&mut buf); // the page buffer back to the reader for reuse
            }
            if k == 0 {
                n_pages = metas.len();
                r.rows = rows;
            } else if rows.len() < n_pages && err.is_none() {
                // StructIterator zips page k of every child (struct_.rs:63-85)
                err = Some(Error::OutOfSpec(format!("{}: its leaf columns hold different pages", self.field.name)));
            } else if rows[..n_pages.min(rows.len())] != r.rows[..n_pages.min(rows.len())] {
                err = Some(Error::OutOfSpec(format!("{}: its leaf columns page different rows", self.field.name)));
            }
            if err.is_some() {
                n_pages = n_pages.min(metas.len());
            }
            r.chunks.push(bytes);
            r.metas.push(metas);
        }
        // every leaf keeps the pages all leaves could read
        for (c, m) in r.chunks.iter_mut().zip(r.metas.iter_mut()) {
            m.truncate(n_pages);
            let len: u64 = m.iter().map(|p| p.length).sum();
            c.truncate(len as usize);
        }
        r.rows.truncate(n_pages);
        (r, err)
    }

    /// The arrays of one decoded range, one per page.
    fn queue(&mut self, data: ColumnData, rows: &[u64]) -> Result<()> {
        let total: u64 = rows.iter().sum();
        if total != data.rows() {
            return Err(Error::OutOfSpec(format!("pages hold {total} rows, the decoded range {}", data.rows())));
        }
        let data = Arc::new(data);
        let mut first = 0u64;
        for &r in rows {
            self.ready.push_back(Ok(Array { data_type: self.field.data_type.clone(), data: data.clone(), offset: first, len: r }));
            first += r;
        }
        Ok(())
    }

    fn fill(&mut self) {
        let (r, read_err) = self.read_range();
        let n = r.rows.len();
        if n > 0 {
            let res = decode_host_chunks(&r.chunks, &r.metas, &self.field).and_then(|d| self.queue(d, &r.rows));
            if res.is_err() {
                // find the bad page: the pages before it decode one by one
                for p in 0..n {
                    let one = |x: &Vec<u8>, m: &Vec<PageMeta>| {
                        let start: u64 = m[..p].iter().map(|q| q.length).sum();
                        x[start as usize..(start + m[p].length) as usize].to_vec()
                    };
                    let chunks: Vec<Vec<u8>> = r.chunks.iter().zip(&r.metas).map(|(x, m)| one(x, m)).collect();
                    let metas: Vec<Vec<PageMeta>> = r.metas.iter().map(|m| vec![m[p]]).collect();
                    let page = decode_host_chunks(&chunks, &metas, &self.field).and_then(|d| self.queue(d, &r.rows[p..p + 1]));
                    if let Err(e) = page {
                        self.ready.push_back(Err(e));
                        self.done = true;
                        return;
                    }
                }
            }
        }
        if let Some(e) = read_err {
            self.ready.push_back(Err(e));
            self.done = true;
        } else if n < RANGE_PAGES {
            self.done = true;
        }
    }
}

impl<I> Iterator for PageArrays<I>
where
    I: Iterator<Item = Result<(u64, Vec<u8>)>> + PageIterator,
{
    type Item = Result<Array>;

    fn next(&mut self) -> Option<Self::Item> {
        if self.ready.is_empty() && !self.done {
            self.fill();
        }
        self.ready.pop_front()
    }
}

/// `column_iter_to_arrays` (src/read/deserialize.rs:237-253): one array per
/// page of the field (one reader per leaf column, to_leaves order), decoded
/// lazily in ranges of [`RANGE_PAGES`] pages.
pub fn column_iter_to_arrays<'a, I: 'a>(
    readers: Vec<I>,
    leaves: Vec<ColumnDescriptor>,
    field: Field,
    is_nested: bool,
) -> Result<ArrayIter<'a>>
where
    I: Iterator<Item = Result<(u64, Vec<u8>)>> + PageIterator + Send + Sync,
{
    check_leaves(&leaves, &field)?;
    check_nested(is_nested, &field)?;
    if readers.len() != leaves.len() {
        return Err(Error::Argument(format!("{}: {} readers for {} leaves", field.name, readers.len(), leaves.len())));
    }
    Ok(Box::new(PageArrays { readers, field, is_nested, ready: VecDeque::new(), done: false }))
}

/// `compression::Compression` (src/compression/mod.rs:37-108).
#[derive(Debug, Clone, Copy, PartialEq, Eq, Hash, Default)]
pub enum Compression {
    #[default]
    None,
    Lz4,
    Zstd,
    Snappy,
    Rle,
    Dict,
    OneValue,
    Freq,
    Bitpacking,
    DeltaBitpacking,
    Patas,
}

impl From<Compression> for u8 {
    fn from(value: Compression) -> Self {
        match value {
            Compression::None => 0,
            Compression::Lz4 => 1,
            Compression::Zstd => 2,
            Compression::Snappy => 3,
            Compression::Rle => 10,
            Compression::Dict => 11,
            Compression::OneValue => 12,
            Compression::Freq => 13,
            Compression::Bitpacking => 14,
            Compression::DeltaBitpacking => 15,
            Compression::Patas => 16,
        }
    }
}

/// `compression::basic::CommonCompression` (src/compression/basic.rs:23-60).
#[derive(Debug, Clone, Copy, PartialEq, Eq, Hash, Default)]
pub enum CommonCompression {
    #[default]
    None,
    Lz4,
    Zstd,
    Snappy,
}

impl CommonCompression {
    pub fn to_compression(&self) -> Compression {
        match self {
            Self::None => Compression::None,
            Self::Lz4 => Compression::Lz4,
            Self::Zstd => Compression::Zstd,
            Self::Snappy => Compression::Snappy,
        }
    }
}

/// `write::WriteOptions` (src/write/common.rs:37-45).
#[derive(Debug, Clone, PartialEq, Default)]
pub struct WriteOptions {
    pub default_compression: CommonCompression,
    pub default_compress_ratio: Option<f64>,
    pub max_page_size: Option<usize>,
    pub forbidden_compressions: Vec<Compression>,
}

const FREQ_ENV: (&str, Compression) = ("STRAWBOAT_FREQ_COMPRESSION", Compression::Freq);
const DICT_ENV: (&str, Compression) = ("STRAWBOAT_DICT_COMPRESSION", Compression::Dict);
const RLE_ENV: (&str, Compression) = ("STRAWBOAT_RLE_COMPRESSION", Compression::Rle);
const BITPACK_ENV: (&str, Compression) = ("STRAWBOAT_BITPACK_COMPRESSION", Compression::Bitpacking);
const PATAS_ENV: (&str, Compression) = ("STRAWBOAT_PATAS_COMPRESSION", Compression::Patas);

/// util/env.rs's debug-build codec overrides, as each type's
/// choose_compressor checks them, in its order: integers Freq / Dict / Rle /
/// Bitpacking (compression/integer/mod.rs:236-266), doubles Freq / Dict /
/// Rle / Patas (double/mod.rs:236-268), binary Freq / Dict
/// (binary/mod.rs:298-314), Boolean Rle (boolean/mod.rs:199-207).  The first
/// one set to "1" whose codec is not forbidden becomes the engine's forced
/// codec (one per column; the reference re-checks them in each nested call).
fn forced_from_env(forbidden: &[Compression], ty: PhysicalType) -> Option<i32> {
    if !cfg!(debug_assertions) {
        return None;
    }
    let order: &[(&str, Compression)] = match ty {
        PhysicalType::Boolean => &[RLE_ENV],
        t if t.is_binary() => &[FREQ_ENV, DICT_ENV],
        PhysicalType::Float32 | PhysicalType::Float64 => &[FREQ_ENV, DICT_ENV, RLE_ENV, PATAS_ENV],
        _ => &[FREQ_ENV, DICT_ENV, RLE_ENV, BITPACK_ENV],
    };
    order
        .iter()
        .find(|(var, c)| std::env::var(var).map_or(false, |v| v == "1") && !forbidden.contains(c))
        .map(|(_, c)| u8::from(*c) as i32)
}

impl WriteOptions {
    /// The engine's options for a column of physical type `ty`.
    fn engine(&self, ty: PhysicalType) -> crate::WriteOptions {
        let mut forbidden_mask = 0u32;
        for c in &self.forbidden_compressions {
            forbidden_mask |= 1u32 << u8::from(*c);
        }
        crate::WriteOptions {
            default_codec: u8::from(self.default_compression.to_compression()) as i32,
            default_compress_ratio: self.default_compress_ratio,
            max_page_size: self.max_page_size.map(|p| p as u64),
            forbidden_mask,
            forced_codec: forced_from_env(&self.forbidden_compressions, ty),
            seed: 0,
        }
    }
}

/// arrow2 `Schema` for the writer: the fields and arrow2's
/// `schema_to_bytes` output (the IPC `Message` flatbuffer the footer holds,
/// writer.rs:137).
#[derive(Debug, Clone)]
pub struct Schema {
    pub fields: Vec<Field>,
    pub ipc_bytes: Vec<u8>,
}

/// One array of a [`Chunk`]: host Arrow buffers (LSB-first bitmaps), shaped
/// like arrow2's arrays so a nested field's array is a tree of them.
pub enum HostArray {
    /// `PrimitiveArray<T>`: `len` values of the field's type (a
    /// `BooleanArray`: the LSB-first values bitmap).
    Primitive { values: Vec<u8>, validity: Option<Vec<u8>>, len: u64 },
    /// `BinaryArray<O>` / `Utf8Array<O>`: `len + 1` absolute offsets into
    /// `values` (the whole buffer: the stats and Extend header use its length).
    Binary { values: Vec<u8>, offsets: Vec<i64>, validity: Option<Vec<u8>>, len: u64 },
    /// `ListArray<O>`: `len + 1` absolute offsets into `values`.
    List { offsets: Vec<i64>, validity: Option<Vec<u8>>, values: Box<HostArray>, len: u64 },
    /// `StructArray`: one child per field, each `len` slots long.
    Struct { values: Vec<HostArray>, validity: Option<Vec<u8>>, len: u64 },
    /// `MapArray`: `len + 1` absolute offsets into `field`, the entries struct.
    Map { offsets: Vec<i64>, validity: Option<Vec<u8>>, field: Box<HostArray>, len: u64 },
}

impl HostArray {
    pub fn len(&self) -> u64 {
        match self {
            HostArray::Primitive { len, .. }
            | HostArray::Binary { len, .. }
            | HostArray::List { len, .. }
            | HostArray::Struct { len, .. }
            | HostArray::Map { len, .. } => *len,
        }
    }
    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }
    fn validity(&self) -> &Option<Vec<u8>> {
        match self {
            HostArray::Primitive { validity, .. }
            | HostArray::Binary { validity, .. }
            | HostArray::List { validity, .. }
            | HostArray::Struct { validity, .. }
            | HostArray::Map { validity, .. } => validity,
        }
    }
}

/// arrow2 `Chunk<Box<dyn Array>>`: one array per schema field.
pub struct Chunk {
    pub arrays: Vec<HostArray>,
}

#[derive(Clone, Copy, PartialEq, Eq)]
enum State {
    None,
    Started,
    Written,
    Finished,
    /// a write of the chunk's bytes failed part way: the file is unusable
    Failed,
}

/// `write::writer::NativeWriter` (src/write/writer.rs:42-173): magic, one
/// chunk's columns (encode_chunk through the engine's writer), footer.
pub struct NativeWriter<W: Write> {
    writer: W,
    offset: u64,
    options: WriteOptions,
    schema: Schema,
    pub metas: Vec<ColumnMeta>,
    state: State,
}

fn io(e: std::io::Error) -> Error {
    Error::Io(e.to_string())
}

impl<W: Write> NativeWriter<W> {
    /// Creates a writer and writes the header (writer.rs:60-65).
    pub fn try_new(writer: W, schema: &Schema, options: WriteOptions) -> Result<Self> {
        let mut w = Self::new(writer, schema.clone(), options);
        w.start()?;
        Ok(w)
    }

    pub fn new(writer: W, schema: Schema, options: WriteOptions) -> Self {
        let n = schema.fields.len();
        NativeWriter { writer, offset: 0, options, schema, metas: Vec::with_capacity(n), state: State::None }
    }

    pub fn into_inner(self) -> W {
        self.writer
    }

    fn put(&mut self, b: &[u8]) -> Result<()> {
        if let Err(e) = self.writer.write_all(b) {
            self.state = State::Failed;
            return Err(io(e));
        }
        self.offset += b.len() as u64;
        Ok(())
    }

    fn check_not_failed(&self) -> Result<()> {
        if self.state == State::Failed {
            return Err(Error::Io("an earlier write to the strawboat file failed".into()));
        }
        Ok(())
    }

    /// "ARROW2" + two zero bytes (writer.rs:91-103); once only.
    pub fn start(&mut self) -> Result<()> {
        self.check_not_failed()?;
        if self.state != State::None {
            return Err(Error::OutOfSpec("The strawboat file can only be started once".into()));
        }
        self.put(b"ARROW2\0\0")?;
        self.state = State::Started;
        Ok(())
    }

    /// The chunk's fields, each paged and encoded by the engine's writer leaf
    /// by leaf (write/common.rs:49-119: a Struct / Map / nested List field is
    /// one column per leaf, to_leaves order); one chunk per file
    /// (writer.rs:106-123).
    /// Every column is encoded before any byte is written, so a column that
    /// fails to encode leaves the writer as it was.
    pub fn write(&mut self, chunk: &Chunk) -> Result<()> {
        self.check_not_failed()?;
        if self.state == State::Written {
            return Err(Error::OutOfSpec("The strawboat file can only accept one RowGroup in a single file".into()));
        }
        if self.state != State::Started {
            return Err(Error::OutOfSpec(
                "The strawboat file must be started before it can be written to. Call `start` before `write`".into(),
            ));
        }
        if chunk.arrays.len() != self.schema.fields.len() {
            return Err(Error::Argument("the chunk's arrays differ from the schema's fields".into()));
        }
        let encoded = chunk
            .arrays
            .iter()
            .zip(self.schema.fields.iter())
            .map(|(a, f)| encode_array(a, f, &self.options))
            .collect::<Result<Vec<_>>>()?;
        for (bytes, pages) in encoded.into_iter().flatten() {
            let offset = self.offset;
            self.put(&bytes)?;
            self.metas.push(ColumnMeta { offset, pages });
        }
        self.state = State::Written;
        Ok(())
    }

    /// Footer: schema, column metas, sizes, EOS (writer.rs:128-167).
    pub fn finish(&mut self) -> Result<()> {
        self.check_not_failed()?;
        if self.state != State::Written {
            return Err(Error::OutOfSpec(
                "The strawboat file must be written before it can be finished. Call `start` before `finish`".into(),
            ));
        }
        let footer = crate::write_footer(&self.schema.ipc_bytes, &self.metas)?;
        self.put(&footer)?;
        if let Err(e) = self.writer.flush() {
            self.state = State::Failed;
            return Err(io(e));
        }
        self.state = State::Finished;
        Ok(())
    }

    pub fn total_size(&self) -> usize {
        self.offset as usize
    }
}

fn bitmap_len(n: u64) -> u64 {
    (n + 7) / 8
}

fn arg(msg: String) -> Error {
    Error::Argument(msg)
}

/// An optional LSB bitmap must hold n bits.
fn check_bitmap(b: &Option<Vec<u8>>, n: u64, what: &str) -> Result<()> {
    match b {
        Some(v) if (v.len() as u64) < bitmap_len(n) => {
            Err(arg(format!("{what} bitmap holds {} bytes, {n} rows need {}", v.len(), bitmap_len(n))))
        }
        _ => Ok(()),
    }
}

/// n values of `ty` (Boolean: an n-bit bitmap).
fn check_values(v: &[u8], n: u64, ty: PhysicalType) -> Result<()> {
    let need = if ty == PhysicalType::Boolean {
        bitmap_len(n)
    } else {
        n.checked_mul(ty.width() as u64).ok_or_else(|| arg(format!("{n} rows overflow the values size")))?
    };
    if (v.len() as u64) < need {
        return Err(arg(format!("values hold {} bytes, {n} rows of {ty:?} need {need}", v.len())));
    }
    Ok(())
}

/// n + 1 offsets, non-decreasing from >= 0, the last at most `limit`.
fn check_offsets(offsets: &[i64], n: u64, limit: u64) -> Result<()> {
    let want = n.checked_add(1).ok_or_else(|| arg("row count overflows".into()))?;
    if offsets.len() as u64 != want {
        return Err(arg(format!("{} offsets for {n} rows", offsets.len())));
    }
    if offsets[0] < 0 || offsets.windows(2).any(|w| w[1] < w[0]) {
        return Err(arg("offsets must be non-negative and non-decreasing".into()));
    }
    let last = offsets[offsets.len() - 1] as u64;
    if last > limit {
        return Err(arg(format!("last offset {last} past the {limit} values")));
    }
    Ok(())
}

/// One leaf of a nested array: the arrays on its path (outermost first,
/// each with its nest), the leaf array and its field.
struct LeafArrays<'a> {
    nests: Vec<(&'a HostArray, Nest)>,
    leaf: &'a HostArray,
    field: &'a Field,
}

/// to_leaves / to_nested (write/common.rs:60-71) over a host array: the
/// leaves of `a` in to_leaves order, each with its path.  The array must
/// have the field's shape.
fn leaf_arrays<'a>(f: &'a Field, a: &'a HostArray, nests: &mut Vec<(&'a HostArray, Nest)>,
                   out: &mut Vec<LeafArrays<'a>>) -> Result<()> {
    let shape = || arg(format!("{}: the array does not have the field's shape", f.name));
    match (&f.data_type, a) {
        (DataType::List(c) | DataType::LargeList(c), HostArray::List { values, .. }) => {
            let large = matches!(f.data_type, DataType::LargeList(_));
            nests.push((a, Nest { is_struct: false, nullable: f.is_nullable, large }));
            leaf_arrays(c, values, nests, out)?;
            nests.pop();
        }
        (DataType::Map(c, _), HostArray::Map { field, .. }) => {
            nests.push((a, Nest { is_struct: false, nullable: f.is_nullable, large: false }));
            leaf_arrays(c, field, nests, out)?;
            nests.pop();
        }
        (DataType::Struct(fields), HostArray::Struct { values, .. }) => {
            if fields.len() != values.len() {
                return Err(shape());
            }
            nests.push((a, Nest { is_struct: true, nullable: f.is_nullable, large: false }));
            for (c, v) in fields.iter().zip(values) {
                leaf_arrays(c, v, nests, out)?;
            }
            nests.pop();
        }
        (DataType::List(_) | DataType::LargeList(_) | DataType::Map(_, _) | DataType::Struct(_), _) => {
            return Err(shape())
        }
        (dt, HostArray::Binary { .. }) if leaf_type(dt).is_binary() => {
            out.push(LeafArrays { nests: nests.clone(), leaf: a, field: f })
        }
        (dt, HostArray::Primitive { .. }) if !leaf_type(dt).is_binary() => {
            out.push(LeafArrays { nests: nests.clone(), leaf: a, field: f })
        }
        _ => return Err(shape()),
    }
    Ok(())
}

/// The C encoder's chunk and page metas, freed from the engine's heap.
fn take_encoded(out: *mut u8, len: u64, metas: *mut PageMeta, np: u64) -> (Vec<u8>, Vec<PageMeta>) {
    let bytes = if len == 0 { Vec::new() } else { unsafe { std::slice::from_raw_parts(out, len as usize) }.to_vec() };
    let pages = if np == 0 { Vec::new() } else { unsafe { std::slice::from_raw_parts(metas, np as usize) }.to_vec() };
    unsafe {
        ffi::sb_free(out as *mut c_void);
        ffi::sb_free(metas as *mut c_void);
    }
    (bytes, pages)
}

/// One leaf column of a nested field through sb_encode_nested_column
/// (write_nested, serialize.rs:135-198).  Every buffer on the path is checked
/// against the lengths first: the encoder reads what the offsets promise.
fn encode_nested_leaf(top_len: u64, l: &LeafArrays, o: &WriteOptions) -> Result<(Vec<u8>, Vec<PageMeta>)> {
    let name = &l.field.name;
    if l.nests.len() > ffi::SB_MAX_NEST {
        return Err(Error::NotYetImplemented(format!("{name}: more than {} nests", ffi::SB_MAX_NEST)));
    }
    let ty = leaf_type(&l.field.data_type);
    let mut desc = ffi::sb_nested_desc {
        physical_type: ty as i32,
        depth: l.nests.len() as i32,
        list_nullable: [0; 4],
        item_nullable: l.field.is_nullable as i32,
        offset_width: 4,
        struct_mask: 0,
    };
    let mut nests = [ffi::sb_nest_in { h_offsets: ptr::null(), h_validity: ptr::null() }; ffi::SB_MAX_NEST];
    let mut count = top_len;  // entries of the current nest
    for (d, (a, n)) in l.nests.iter().enumerate() {
        if a.len() != count {
            return Err(arg(format!("{name}: nest {d} holds {} entries, its parent reaches {count}", a.len())));
        }
        check_bitmap(a.validity(), count, "nest validity")?;
        desc.list_nullable[d] = n.nullable as i32;
        nests[d].h_validity = a.validity().as_ref().map_or(ptr::null(), |b| b.as_ptr());
        if n.large {
            desc.offset_width = 8;
        }
        match a {
            HostArray::Struct { .. } => desc.struct_mask |= 1 << d,
            HostArray::List { offsets, values: child, .. } | HostArray::Map { offsets, field: child, .. } => {
                check_offsets(offsets, count, child.len())?;
                nests[d].h_offsets = offsets.as_ptr();
                count = child.len();
            }
            _ => unreachable!("leaf_arrays pushes nests only"),
        }
    }
    if l.leaf.len() != count {
        return Err(arg(format!("{name}: the leaf holds {} slots, its parent reaches {count}", l.leaf.len())));
    }
    check_bitmap(l.leaf.validity(), count, "leaf validity")?;
    let (values, leaf_offsets, values_len) = match l.leaf {
        HostArray::Primitive { values, .. } => {
            check_values(values, count, ty)?;
            (values.as_ptr(), ptr::null(), 0u64)
        }
        HostArray::Binary { values, offsets, .. } => {
            check_offsets(offsets, count, values.len() as u64)?;
            (values.as_ptr(), offsets.as_ptr(), values.len() as u64)
        }
        _ => unreachable!("leaf_arrays pushes leaves only"),
    };
    let eo = o.engine(ty);
    let opts = eo.raw();
    let (mut out, mut len, mut metas, mut np) = (ptr::null_mut(), 0u64, ptr::null_mut(), 0u64);
    let st = unsafe {
        ffi::sb_encode_nested_column(&desc, nests.as_ptr(), values as *const c_void, leaf_offsets, values_len,
                                     l.leaf.validity().as_ref().map_or(ptr::null(), |b| b.as_ptr()), top_len, &opts,
                                     eo.max_page_size.unwrap_or(0), 0, &mut out, &mut len, &mut metas, &mut np)
    };
    status(st, || format!("encoding {name}"))?;
    Ok(take_encoded(out, len, metas as *mut PageMeta, np))
}

/// One field of the chunk: a flat leaf through sb_encode_column /
/// sb_encode_binary_column, a `List<primitive>` through sb_encode_list_column,
/// any other nesting leaf by leaf through sb_encode_nested_column (the host
/// writer, every codec of the cascade).  Returns one (chunk, pages) per leaf
/// column, to_leaves order (encode_chunk, write/common.rs:60-115).  The
/// buffers are checked against `len` first: the C encoder reads exactly what
/// the lengths and offsets promise.
fn encode_array(a: &HostArray, f: &Field, o: &WriteOptions) -> Result<Vec<(Vec<u8>, Vec<PageMeta>)>> {
    if !is_primitive(&f.data_type) {
        if let (Ok((ty, lists, _, leaf_nullable)), HostArray::List { offsets, validity, values: child, len: n }) =
            (leaf_path(f), a)
        {
            if let HostArray::Primitive { values, validity: child_validity, len: nc } = child.as_ref() {
                if lists.len() == 1 && !ty.is_binary() && ty != PhysicalType::Boolean {
                    check_offsets(offsets, *n, *nc)?;
                    check_values(values, *nc, ty)?;
                    check_bitmap(validity, *n, "list validity")?;
                    check_bitmap(child_validity, *nc, "item validity")?;
                    let eo = o.engine(ty);
                    let opts = eo.raw();
                    let bm = |v: &Option<Vec<u8>>| v.as_ref().map_or(ptr::null(), |b| b.as_ptr());
                    let (mut out, mut len, mut metas, mut np) = (ptr::null_mut(), 0u64, ptr::null_mut(), 0u64);
                    let st = unsafe {
                        ffi::sb_encode_list_column(ty as i32, offsets.as_ptr(), bm(validity), lists[0] as i32,
                                                   values.as_ptr() as *const c_void, bm(child_validity),
                                                   leaf_nullable as i32, *n, &opts, eo.max_page_size.unwrap_or(0), 0,
                                                   &mut out, &mut len, &mut metas, &mut np)
                    };
                    status(st, || format!("encoding {}", f.name))?;
                    return Ok(vec![take_encoded(out, len, metas as *mut PageMeta, np)]);
                }
            }
        }
        let mut leaves = Vec::new();
        leaf_arrays(f, a, &mut Vec::new(), &mut leaves)?;
        return leaves.iter().map(|l| encode_nested_leaf(a.len(), l, o)).collect();
    }
    let ty = leaf_type(&f.data_type);
    let eo = o.engine(ty);
    let opts = eo.raw();
    let page = eo.max_page_size.unwrap_or(0);
    let mut out: *mut u8 = ptr::null_mut();
    let mut len = 0u64;
    let mut metas: *mut PageMeta = ptr::null_mut();
    let mut np = 0u64;
    let bm = |v: &Option<Vec<u8>>| v.as_ref().map_or(ptr::null(), |b| b.as_ptr());
    let st = match a {
        HostArray::Primitive { values, validity, len: n } if !ty.is_binary() => {
            check_values(values, *n, ty)?;
            check_bitmap(validity, *n, "validity")?;
            unsafe {
                ffi::sb_encode_column(ty as i32, values.as_ptr() as *const c_void, bm(validity), *n,
                                      f.is_nullable as i32, &opts, page, 0, &mut out, &mut len, &mut metas, &mut np)
            }
        }
        HostArray::Binary { values, offsets, validity, len: n } if ty.is_binary() => {
            check_offsets(offsets, *n, values.len() as u64)?;
            check_bitmap(validity, *n, "validity")?;
            unsafe {
                ffi::sb_encode_binary_column(ty as i32, values.as_ptr(), values.len() as u64, offsets.as_ptr(),
                                             bm(validity), *n, f.is_nullable as i32, &opts, page, 0, &mut out,
                                             &mut len, &mut metas, &mut np)
            }
        }
        _ => return Err(arg(format!("{}: the array does not have the field's shape", f.name))),
    };
    status(st, || format!("encoding {}", f.name))?;
    Ok(vec![take_encoded(out, len, metas, np)])
}

#[cfg(test)]
mod tests {
    use super::*;

    fn metas() -> Vec<PageMeta> {
        vec![PageMeta { length: 3, num_values: 10 }, PageMeta { length: 2, num_values: 7 }, PageMeta { length: 4, num_values: 1 }]
    }

    #[test]
    fn native_reader_pages_and_nth() {
        let mut r = NativeReader::new(Cursor::new(b"aaabbcccc".to_vec()), metas(), Vec::new());
        assert!(r.has_next());
        assert_eq!(r.next().unwrap().unwrap(), (10, b"aaa".to_vec()));
        assert_eq!(r.current_page(), 1);
        let mut r = NativeReader::new(Cursor::new(b"aaabbcccc".to_vec()), metas(), Vec::new());
        assert_eq!(r.nth(2).unwrap().unwrap(), (1, b"cccc".to_vec()));
        assert!(!r.has_next());
        let mut r = NativeReader::new(Cursor::new(b"aaabbcccc".to_vec()), metas(), Vec::new());
        r.skip_page().unwrap();
        assert_eq!(r.next().unwrap().unwrap(), (7, b"bb".to_vec()));
    }

    #[test]
    fn native_read_buf_peeks() {
        let mut c = Cursor::new(b"abcdef".to_vec());
        c.set_position(2);
        assert_eq!(c.buffer_bytes(), b"cdef");
        let s: &[u8] = b"xyz";
        assert_eq!(s.buffer_bytes(), b"xyz");
    }

    #[test]
    fn leaf_paths() {
        let f = Field::new("l", DataType::List(Box::new(Field::new("item", DataType::Int32, true))), false);
        assert_eq!(leaf_path(&f).unwrap(), (PhysicalType::Int32, vec![false], vec![false], true));
    }

    #[test]
    fn struct_and_map_chains() {
        // tests/it/io.rs:294-325 create_map: Map(nullable) of entries {key Int32, value LargeBinary}
        let entries = Field::new("entries", DataType::Struct(vec![Field::new("key", DataType::Int32, false),
                                                                     Field::new("value", DataType::LargeBinary, true)]), false);
        let m = Field::new("m", DataType::Map(Box::new(entries), false), true);
        assert_eq!(n_columns(&m.data_type), 2);
        let c = leaf_chains(&m);
        assert_eq!(c.len(), 2);
        assert_eq!(c[0].ty, PhysicalType::Int32);
        assert_eq!(c[1].ty, PhysicalType::LargeBinary);
        assert_eq!(c[0].nests, vec![Nest { is_struct: false, nullable: true, large: false },
                                    Nest { is_struct: true, nullable: false, large: false }]);
        assert!(!c[0].nullable && c[1].nullable);
        assert!(leaf_path(&m).is_err());
        assert!(check_nested(false, &m).is_err() && check_nested(true, &m).is_ok());
        let leaves = vec![ColumnDescriptor { physical_type: PhysicalType::Int32, max_def_level: 2, max_rep_level: 1 }];
        assert!(check_leaves(&leaves, &m).is_err());
    }

    #[test]
    fn env_overrides_follow_the_column_type() {
        std::env::set_var("STRAWBOAT_PATAS_COMPRESSION", "1");
        assert_eq!(forced_from_env(&[], PhysicalType::Int32), None);
        if cfg!(debug_assertions) {
            assert_eq!(forced_from_env(&[], PhysicalType::Float64), Some(16));
        }
        std::env::remove_var("STRAWBOAT_PATAS_COMPRESSION");
        std::env::set_var("STRAWBOAT_BITPACK_COMPRESSION", "1");
        assert_eq!(forced_from_env(&[], PhysicalType::Utf8), None);
        assert_eq!(forced_from_env(&[], PhysicalType::Boolean), None);
        std::env::remove_var("STRAWBOAT_BITPACK_COMPRESSION");
    }

    #[test]
    fn writer_state_machine() {
        let schema = Schema { fields: vec![], ipc_bytes: vec![] };
        let mut w = NativeWriter::new(Vec::new(), schema, WriteOptions::default());
        assert!(w.finish().is_err());
        w.start().unwrap();
        assert!(w.start().is_err());
        assert_eq!(w.total_size(), 8);
    }

    #[test]
    fn malformed_host_arrays_are_argument_errors() {
        let f = Field::new("x", DataType::Int32, true);
        let o = WriteOptions::default();
        let short = HostArray::Primitive { values: vec![0; 7], validity: None, len: 2 };
        assert!(matches!(encode_array(&short, &f, &o), Err(Error::Argument(_))));
        let bad_bitmap = HostArray::Primitive { values: vec![0; 40], validity: Some(vec![0xFF]), len: 10 };
        assert!(matches!(encode_array(&bad_bitmap, &f, &o), Err(Error::Argument(_))));
        let s = Field::new("s", DataType::Utf8, false);
        let past = HostArray::Binary { values: b"ab".to_vec(), offsets: vec![0, 1, 3], validity: None, len: 2 };
        assert!(matches!(encode_array(&past, &s, &o), Err(Error::Argument(_))));
        let down = HostArray::Binary { values: b"ab".to_vec(), offsets: vec![0, 2, 1], validity: None, len: 2 };
        assert!(matches!(encode_array(&down, &s, &o), Err(Error::Argument(_))));
    }

    #[test]
    fn nested_arrays_follow_the_field() {
        // io.rs:256-278 test_struct_list: Struct { name: LargeBinary, age: List<Int32> }
        let age = Field::new("age", DataType::List(Box::new(Field::new("item", DataType::Int32, true))), true);
        let f = Field::new("s", DataType::Struct(vec![Field::new("name", DataType::LargeBinary, true), age]), false);
        let name = HostArray::Binary { values: b"ab".to_vec(), offsets: vec![0, 1, 2], validity: None, len: 2 };
        let ages = HostArray::List {
            offsets: vec![0, 2, 3],
            validity: Some(vec![0b11]),
            values: Box::new(HostArray::Primitive { values: vec![0; 12], validity: None, len: 3 }),
            len: 2,
        };
        let a = HostArray::Struct { values: vec![name, ages], validity: None, len: 2 };
        let mut leaves = Vec::new();
        leaf_arrays(&f, &a, &mut Vec::new(), &mut leaves).unwrap();
        assert_eq!(leaves.len(), 2);
        assert_eq!(leaves[0].nests.len(), 1);
        assert!(leaves[0].nests[0].1.is_struct);
        assert_eq!(leaves[1].nests.len(), 2);
        assert!(!leaves[1].nests[1].1.is_struct && leaves[1].nests[1].1.nullable);
        // a struct child shorter than the struct, and a field / array mismatch, are argument errors
        let short = HostArray::Struct {
            values: vec![HostArray::Binary { values: b"a".to_vec(), offsets: vec![0, 1], validity: None, len: 1 },
                         HostArray::List { offsets: vec![0, 0, 0], validity: None,
                                           values: Box::new(HostArray::Primitive { values: vec![], validity: None, len: 0 }),
                                           len: 2 }],
            validity: None,
            len: 2,
        };
        assert!(matches!(encode_array(&short, &f, &WriteOptions::default()), Err(Error::Argument(_))));
        let flat = HostArray::Primitive { values: vec![0; 8], validity: None, len: 2 };
        assert!(matches!(encode_array(&flat, &f, &WriteOptions::default()), Err(Error::Argument(_))));
    }

    #[test]
    fn options_map_onto_the_engine() {
        let o = WriteOptions {
            default_compression: CommonCompression::Lz4,
            default_compress_ratio: Some(2.0),
            max_page_size: Some(8192),
            forbidden_compressions: vec![Compression::Dict, Compression::Freq],
        };
        let e = o.engine(PhysicalType::Int32);
        assert_eq!(e.default_codec, 1);
        assert_eq!(e.forbidden_mask, (1 << 11) | (1 << 13));
        assert_eq!(e.max_page_size, Some(8192));
    }

    fn assert_send_sync<T: Send + Sync>() {}

    #[test]
    fn arrays_and_iterators_cross_threads() {
        assert_send_sync::<Array>();
        assert_send_sync::<ArrayIter<'static>>();
    }
}
