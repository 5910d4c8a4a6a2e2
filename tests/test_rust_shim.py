"""The Rust shim crate (rust/strawboat-gpu) cannot be
compiled here (no cargo / rustc in the image); these CPU checks keep its FFI
declarations in step with the C ABI: every function include/strawboat_gpu.h
declares is declared in src/ffi.rs with the same parameter count, and every
one of them is exported by the built library."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "strawboat_gpu.h")
FFI = os.path.join(ROOT, "rust", "strawboat-gpu", "src", "ffi.rs")


def header_functions():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(sb_\w+)\s*\(([^;{]*?)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def rust_functions():
    src = open(FFI).read()
    out = {}
    for m in re.finditer(r"pub fn (sb_\w+)\s*\(([^)]*)\)", src, flags=re.S):
        args = m.group(2).strip().rstrip(",")
        out[m.group(1)] = 0 if not args else args.count(",") + 1
    return out


def test_rust_ffi_declares_the_whole_abi():
    h, r = header_functions(), rust_functions()
    assert h, "no functions parsed from the header"
    assert sorted(set(h) - set(r)) == [], "declared in the header, missing in ffi.rs"
    assert sorted(set(r) - set(h)) == [], "declared in ffi.rs, not in the header"
    assert {k: v for k, v in h.items() if r[k] != v} == {}, "parameter counts differ"


def test_rust_ffi_symbols_exported():
    import ctypes

    lib = ctypes.CDLL(os.path.join(ROOT, "pa_amd", "libstrawboat_gpu.so"))
    for name in rust_functions():
        assert hasattr(lib, name), name


COMPAT = os.path.join(ROOT, "rust", "strawboat-gpu", "src", "compat.rs")

# The reference's signatures (b41sh/pa 0.2.6), parameter names in order:
# the shim keeps them exactly (no engine context argument: the calling
# thread's default context decodes).
REFERENCE_SIGNATURES = {
    # src/read/reader.rs:60
    "new(page_reader": ["page_reader", "page_metas", "scratch"],
    # src/read/deserialize.rs:237-243
    "column_iter_to_arrays": ["readers", "leaves", "field", "is_nested"],
    # src/read/batch_read.rs:190-196
    "batch_read_array": ["readers", "leaves", "field", "is_nested", "page_metas"],
    # src/write/writer.rs:59
    "try_new": ["writer", "schema", "options"],
}
# The generic bounds those functions carry in the reference.
REFERENCE_BOUNDS = [
    "pub fn batch_read_array<R: NativeReadBuf>(",                       # batch_read.rs:190
    "pub fn column_iter_to_arrays<'a, I: 'a>(",                         # deserialize.rs:237
    "I: Iterator<Item = Result<(u64, Vec<u8>)>> + PageIterator + Send + Sync,",  # deserialize.rs:243
    "pub struct NativeReader<R: NativeReadBuf>",                        # reader.rs:51
    "impl<R: NativeReadBuf + Seek> Iterator for NativeReader<R>",       # reader.rs:87
    "pub trait NativeReadBuf: BufRead",                                 # read/mod.rs:26
    "pub type ArrayIter<'a> = Box<dyn Iterator<Item = Result<Array>> + Send + Sync + 'a>;",
]
# src/write/common.rs:37-45
WRITE_OPTIONS_FIELDS = ["default_compression: CommonCompression", "default_compress_ratio: Option<f64>",
                        "max_page_size: Option<usize>", "forbidden_compressions: Vec<Compression>"]
# src/read/reader.rs:69-145, read/mod.rs:26-57, write/writer.rs:66-173
REFERENCE_METHODS = ["has_next", "current_page", "skip_page", "swap_buffer", "buffer_bytes", "next", "nth",
                     "into_inner", "start", "write", "finish", "total_size"]


def _params(src, head):
    i = src.index("pub fn " + head)
    j = src.index("(", i + len("pub fn ") + len(head.split("(")[0]))
    depth, k = 0, j
    while True:
        depth += {"(": 1, ")": -1}.get(src[k], 0)
        if depth == 0:
            break
        k += 1
    args = [a.strip() for a in re.split(r",(?![^<]*>)", src[j + 1:k]) if a.strip()]
    return [a.split(":")[0].replace("mut ", "").strip() for a in args if a not in ("&self", "&mut self", "self")]


def test_rust_compat_keeps_the_reference_signatures():
    src = open(COMPAT).read()
    for head, names in REFERENCE_SIGNATURES.items():
        assert _params(src, head) == names, (head, _params(src, head))
    for b in REFERENCE_BOUNDS:
        assert b in src, b
    for f in WRITE_OPTIONS_FIELDS:
        assert "pub " + f in src, f
    for m in REFERENCE_METHODS:
        assert re.search(r"\bfn %s\b" % m, src), m
    assert "pub struct NativeWriter<W: Write>" in src
    assert "pub trait PageIterator" in src
    # no public entry point of the drop-in surface takes an engine context
    assert not re.search(r"pub fn \w+[^(]*\([^)]*ctx\s*:", src)
    lib = open(os.path.join(ROOT, "rust", "strawboat-gpu", "src", "lib.rs")).read()
    assert "pub mod compat;" in lib


def test_rust_compat_checks_host_buffers_before_ffi():
    """Every unsafe call into the C encoder is preceded (since the previous
    FFI call) by checks of the lengths, bitmaps and offsets it will read
    (ADVICE r03)."""
    src = open(COMPAT).read()
    for call in ("sb_encode_column(", "sb_encode_binary_column(", "sb_encode_list_column(",
                 "sb_encode_nested_column("):
        i = src.index("ffi::" + call)
        prev = src.rfind("ffi::sb_", 0, i)
        assert "check_" in src[prev + 1:i], call


def test_rust_compat_host_array_is_arrow2_shaped():
    """HostArray mirrors arrow2's array tree (PrimitiveArray / BooleanArray,
    BinaryArray / Utf8Array, ListArray, StructArray, MapArray), so
    NativeWriter::write takes the reference's nested chunks (io.rs:167-278);
    a nested field goes leaf by leaf through sb_encode_nested_column."""
    src = open(COMPAT).read()
    enum = src[src.index("pub enum HostArray {"):]
    enum = enum[:enum.index("\n}\n")]
    for v in ("Primitive {", "Binary {", "List { offsets: Vec<i64>, validity: Option<Vec<u8>>, values: Box<HostArray>",
              "Struct { values: Vec<HostArray>", "Map { offsets: Vec<i64>, validity: Option<Vec<u8>>, field: Box<HostArray>"):
        assert v in enum, v
    assert "fn leaf_arrays" in src and "ffi::sb_encode_nested_column(" in src
    assert "encoded.into_iter().flatten()" in src  # one ColumnMeta per leaf column
