//! The reference's own API shapes over the engine, so a
//! `strawboat` (b41sh/pa 0.2.6) maintainer swaps the codec path without
//! rewriting callers:
//!
//! | reference | here |
//! |---|---|
//! | `read::PageIterator` (src/read/mod.rs:55-57) | [`PageIterator`] |
//! | `read::reader::NativeReader::{new, has_next, current_page, skip_page}` + `Iterator` (src/read/reader.rs:51-146) | [`NativeReader`] |
//! | `read::deserialize::column_iter_to_arrays` (src/read/deserialize.rs:237-253) | [`column_iter_to_arrays`] |
//! | `read::batch_read::batch_read_array` (src/read/batch_read.rs:190-209) | [`batch_read_array`] |
//! | `write::writer::NativeWriter::{try_new, new, into_inner, start, write, finish, total_size}` (src/write/writer.rs:42-173) | [`NativeWriter`] |
//!
//! Every function keeps the reference's parameters in the reference's order
//! and adds the engine [`Context`] (one device + one HIP stream) in front:
//! that is where the pages are decoded.  arrow2 / parquet2 types are
//! stood in for by the minimal [`Field`], [`DataType`], [`ColumnDescriptor`],
//! [`Schema`] and [`Chunk`] below (this crate has no dependencies); the
//! decoded [`Array`] holds Arrow buffers in HBM, which the caller wraps into
//! arrow2 arrays.
use std::io::{Read, Seek, SeekFrom, Write};
use std::os::raw::c_void;
use std::ptr;

use crate::{
    ffi, status, Binary, BinaryColumn, ColumnMeta, Context, DeviceBuffer, Error, List, ListColumn, Nested,
    NestedColumn, PageMeta, PhysicalType, Primitive, PrimitiveColumn, Result, WriteOptions,
};

/// `read::PageIterator` (src/read/mod.rs:55-57): a page source that hands
/// its read buffer back for reuse.
pub trait PageIterator {
    fn swap_buffer(&mut self, buffer: &mut Vec<u8>);
}

/// `read::reader::NativeReader` (src/read/reader.rs:51-146): the pages of
/// one column chunk, read in order from `page_reader` (positioned at the
/// chunk's first page, `ColumnMeta::offset`).
#[derive(Debug)]
pub struct NativeReader<R: Read + Seek> {
    page_reader: R,
    page_metas: Vec<PageMeta>,
    current_page: usize,
    scratch: Vec<u8>,
}

impl<R: Read + Seek> NativeReader<R> {
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

    /// Skips the next page (reader.rs:134-145).
    pub fn skip_page(&mut self) -> Result<()> {
        if self.current_page == self.page_metas.len() {
            return Ok(());
        }
        let len = self.page_metas[self.current_page].length;
        self.page_reader.seek(SeekFrom::Current(len as i64)).map_err(|e| Error::Io(e.to_string()))?;
        self.current_page += 1;
        Ok(())
    }

    /// The rest of the chunk's pages in one read (batch_read's read_simple
    /// reads them page by page into one buffer).
    fn read_rest(&mut self) -> Result<(Vec<u8>, Vec<PageMeta>)> {
        let metas = self.page_metas[self.current_page..].to_vec();
        let mut len = 0u64;
        for m in &metas {
            len = len.checked_add(m.length).ok_or_else(|| Error::OutOfSpec("chunk length overflows u64".into()))?;
        }
        let mut buf = std::mem::take(&mut self.scratch);
        buf.resize(len as usize, 0);
        self.page_reader.read_exact(&mut buf).map_err(|e| Error::Io(e.to_string()))?;
        self.current_page = self.page_metas.len();
        Ok((buf, metas))
    }
}

impl<R: Read + Seek> PageIterator for NativeReader<R> {
    fn swap_buffer(&mut self, scratch: &mut Vec<u8>) {
        std::mem::swap(&mut self.scratch, scratch)
    }
}

impl<R: Read + Seek> Iterator for NativeReader<R> {
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
            return Some(Err(Error::Io(e.to_string())));
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
                return Some(Err(Error::Io(e.to_string())));
            }
        }
        self.next()
    }
}

/// The arrow2 `DataType`s the page path carries (Struct / Map / Union are
/// out of scope).
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

/// parquet2 `ColumnDescriptor`, reduced to what a leaf reader needs.
#[derive(Debug, Clone, Copy, PartialEq)]
pub struct ColumnDescriptor {
    pub physical_type: PhysicalType,
    pub max_def_level: i16,
    pub max_rep_level: i16,
}

/// A decoded column (or page): its Arrow buffers in HBM.
pub enum Array {
    Primitive(Primitive),
    Binary(Binary),
    List(List),
    Nested(Nested),
}

/// The leaf under a field: its physical type, per list level (outermost
/// first) the level's nullability and whether it is a LargeList, and the
/// leaf's own nullability (arrow2 to_leaves + InitNested).
fn leaf_path(field: &Field) -> Result<(PhysicalType, Vec<bool>, Vec<bool>, bool)> {
    use PhysicalType as P;
    let (mut lists, mut large) = (Vec::new(), Vec::new());
    let mut f = field;
    loop {
        let ty = match &f.data_type {
            DataType::List(c) | DataType::LargeList(c) => {
                lists.push(f.is_nullable);
                large.push(matches!(f.data_type, DataType::LargeList(_)));
                f = c;
                continue;
            }
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
        };
        return Ok((ty, lists, large, f.is_nullable));
    }
}

/// The read/deserialize.rs dispatch over one column chunk in HBM: flat
/// primitive / Boolean, Binary / Utf8, List<primitive>, or any other list
/// nesting (depth 1..=4, every leaf kind).
fn decode_chunk(ctx: &Context, chunk: &DeviceBuffer, pages: &[PageMeta], field: &Field) -> Result<Array> {
    let (ty, lists, large, leaf_nullable) = leaf_path(field)?;
    if lists.is_empty() {
        return if ty.is_binary() {
            Ok(Array::Binary(BinaryColumn::plan(ctx, chunk, pages, ty, leaf_nullable)?.decode()?))
        } else {
            Ok(Array::Primitive(PrimitiveColumn::plan(ctx, chunk, pages, ty, leaf_nullable)?.decode()?))
        };
    }
    if large.iter().any(|&l| l != large[0]) {
        return Err(Error::NotYetImplemented(format!("{}: mixed List / LargeList levels", field.name)));
    }
    if lists.len() == 1 && !ty.is_binary() && ty != PhysicalType::Boolean {
        let c = ListColumn::plan(ctx, chunk, pages, ty, lists[0], leaf_nullable, large[0])?;
        return Ok(Array::List(c.decode()?));
    }
    let c = NestedColumn::plan(ctx, chunk, pages, ty, &lists, leaf_nullable, large[0])?;
    Ok(Array::Nested(c.decode()?))
}

fn one_leaf(leaves: &[ColumnDescriptor], field: &Field) -> Result<()> {
    if leaves.len() != 1 {
        return Err(Error::NotYetImplemented(format!("{}: {} leaves (Struct / Map nests)", field.name, leaves.len())));
    }
    let (ty, _, _, _) = leaf_path(field)?;
    if leaves[0].physical_type != ty {
        return Err(Error::OutOfSpec(format!("{}: leaf type {:?} against field {:?}", field.name, leaves[0].physical_type, ty)));
    }
    Ok(())
}

/// `batch_read_array` (src/read/batch_read.rs:190-209): every page of the
/// column at once, one array.  The chunk's pages are read from the reader
/// in one read, staged into HBM on the context's device and decoded there.
pub fn batch_read_array<R: Read + Seek>(
    ctx: &Context,
    mut readers: Vec<NativeReader<R>>,
    leaves: Vec<ColumnDescriptor>,
    field: Field,
    is_nested: bool,
    mut page_metas: Vec<Vec<PageMeta>>,
) -> Result<Array> {
    one_leaf(&leaves, &field)?;
    let mut reader = readers.pop().ok_or_else(|| Error::Argument("no reader".into()))?;
    let metas = page_metas.pop().ok_or_else(|| Error::Argument("no page metas".into()))?;
    if is_nested != matches!(field.data_type, DataType::List(_) | DataType::LargeList(_)) {
        return Err(Error::Argument(format!("{}: is_nested {is_nested} against its data type", field.name)));
    }
    if metas.len() != reader.page_metas.len() - reader.current_page {
        return Err(Error::Argument("page metas differ from the reader's".into()));
    }
    let (mut bytes, _) = reader.read_rest()?;
    let out = ctx.upload(&bytes).and_then(|chunk| decode_chunk(ctx, &chunk, &metas, &field));
    reader.swap_buffer(&mut bytes);  // the read buffer back to the reader for reuse
    out
}

/// The iterator `column_iter_to_arrays` returns: one array per page (the
/// reference's streaming read yields one array per page).
pub struct ArrayIter<'a, I> {
    ctx: &'a Context,
    reader: I,
    field: Field,
}

impl<'a, I> Iterator for ArrayIter<'a, I>
where
    I: Iterator<Item = Result<(u64, Vec<u8>)>> + PageIterator,
{
    type Item = Result<Array>;

    fn next(&mut self) -> Option<Self::Item> {
        let (num_values, mut page) = match self.reader.next()? {
            Ok(p) => p,
            Err(e) => return Some(Err(e)),
        };
        let out = (|| {
            let chunk = self.ctx.upload(&page)?;
            let meta = PageMeta { length: page.len() as u64, num_values };
            decode_chunk(self.ctx, &chunk, &[meta], &self.field)
        })();
        self.reader.swap_buffer(&mut page);  // the page buffer back to the reader for reuse
        Some(out)
    }
}

/// `column_iter_to_arrays` (src/read/deserialize.rs:237-253).
pub fn column_iter_to_arrays<'a, I>(
    ctx: &'a Context,
    mut readers: Vec<I>,
    leaves: Vec<ColumnDescriptor>,
    field: Field,
    is_nested: bool,
) -> Result<ArrayIter<'a, I>>
where
    I: Iterator<Item = Result<(u64, Vec<u8>)>> + PageIterator + 'a,
{
    one_leaf(&leaves, &field)?;
    if is_nested != matches!(field.data_type, DataType::List(_) | DataType::LargeList(_)) {
        return Err(Error::Argument(format!("{}: is_nested {is_nested} against its data type", field.name)));
    }
    let reader = readers.pop().ok_or_else(|| Error::Argument("no reader".into()))?;
    Ok(ArrayIter { ctx, reader, field })
}

/// arrow2 `Schema` for the writer: the fields and arrow2's
/// `schema_to_bytes` output (the IPC `Message` flatbuffer the footer holds,
/// writer.rs:137).
#[derive(Debug, Clone)]
pub struct Schema {
    pub fields: Vec<Field>,
    pub ipc_bytes: Vec<u8>,
}

/// One column of a [`Chunk`]: host Arrow buffers (LSB-first bitmaps).
pub enum HostArray {
    Primitive { values: Vec<u8>, validity: Option<Vec<u8>>, len: u64 },
    Binary { values: Vec<u8>, offsets: Vec<i64>, validity: Option<Vec<u8>>, len: u64 },
    List { offsets: Vec<i64>, validity: Option<Vec<u8>>, values: Vec<u8>, child_validity: Option<Vec<u8>>, len: u64 },
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
        self.writer.write_all(b).map_err(io)?;
        self.offset += b.len() as u64;
        Ok(())
    }

    /// "ARROW2" + two zero bytes (writer.rs:91-103); once only.
    pub fn start(&mut self) -> Result<()> {
        if self.state != State::None {
            return Err(Error::OutOfSpec("The strawboat file can only be started once".into()));
        }
        self.put(b"ARROW2\0\0")?;
        self.state = State::Started;
        Ok(())
    }

    /// The chunk's columns, each paged and encoded by the engine's writer
    /// (write/common.rs:49-119); one chunk per file (writer.rs:106-123).
    pub fn write(&mut self, chunk: &Chunk) -> Result<()> {
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
        let fields = self.schema.fields.clone();
        for (a, f) in chunk.arrays.iter().zip(fields.iter()) {
            let (bytes, pages) = encode_array(a, f, &self.options)?;
            let offset = self.offset;
            self.put(&bytes)?;
            self.metas.push(ColumnMeta { offset, pages });
        }
        self.state = State::Written;
        Ok(())
    }

    /// Footer: schema, column metas, sizes, EOS (writer.rs:128-167).
    pub fn finish(&mut self) -> Result<()> {
        if self.state != State::Written {
            return Err(Error::OutOfSpec(
                "The strawboat file must be written before it can be finished. Call `start` before `finish`".into(),
            ));
        }
        let footer = crate::write_footer(&self.schema.ipc_bytes, &self.metas)?;
        self.put(&footer)?;
        self.writer.flush().map_err(io)?;
        self.state = State::Finished;
        Ok(())
    }

    pub fn total_size(&self) -> usize {
        self.offset as usize
    }
}

/// One column through sb_encode_column / sb_encode_binary_column /
/// sb_encode_list_column (the host writer, every codec of the cascade).
fn encode_array(a: &HostArray, f: &Field, o: &WriteOptions) -> Result<(Vec<u8>, Vec<PageMeta>)> {
    let (ty, lists, _, leaf_nullable) = leaf_path(f)?;
    let opts = o.raw();
    let page = o.max_page_size.unwrap_or(0);
    let mut out: *mut u8 = ptr::null_mut();
    let mut len = 0u64;
    let mut metas: *mut PageMeta = ptr::null_mut();
    let mut np = 0u64;
    let bm = |v: &Option<Vec<u8>>| v.as_ref().map_or(ptr::null(), |b| b.as_ptr());
    let st = match a {
        HostArray::Primitive { values, validity, len: n } if lists.is_empty() && !ty.is_binary() => unsafe {
            ffi::sb_encode_column(ty as i32, values.as_ptr() as *const c_void, bm(validity), *n, f.is_nullable as i32,
                                  &opts, page, 0, &mut out, &mut len, &mut metas, &mut np)
        },
        HostArray::Binary { values, offsets, validity, len: n } if lists.is_empty() && ty.is_binary() => unsafe {
            ffi::sb_encode_binary_column(ty as i32, values.as_ptr(), values.len() as u64, offsets.as_ptr(), bm(validity),
                                         *n, f.is_nullable as i32, &opts, page, 0, &mut out, &mut len, &mut metas,
                                         &mut np)
        },
        HostArray::List { offsets, validity, values, child_validity, len: n }
            if lists.len() == 1 && !ty.is_binary() && ty != PhysicalType::Boolean => unsafe {
            ffi::sb_encode_list_column(ty as i32, offsets.as_ptr(), bm(validity), lists[0] as i32,
                                       values.as_ptr() as *const c_void, bm(child_validity), leaf_nullable as i32, *n,
                                       &opts, page, 0, &mut out, &mut len, &mut metas, &mut np)
        },
        _ => return Err(Error::NotYetImplemented(format!("{}: no writer path for this array / field", f.name))),
    };
    status(st, || format!("encoding {}", f.name))?;
    let bytes = unsafe { std::slice::from_raw_parts(out, len as usize) }.to_vec();
    let pages = if np == 0 { Vec::new() } else { unsafe { std::slice::from_raw_parts(metas, np as usize) }.to_vec() };
    unsafe {
        ffi::sb_free(out as *mut c_void);
        ffi::sb_free(metas as *mut c_void);
    }
    Ok((bytes, pages))
}

#[cfg(test)]
mod tests {
    use super::*;
    use std::io::Cursor;

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
    fn leaf_paths() {
        let f = Field::new("l", DataType::List(Box::new(Field::new("item", DataType::Int32, true))), false);
        assert_eq!(leaf_path(&f).unwrap(), (PhysicalType::Int32, vec![false], vec![false], true));
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
}
