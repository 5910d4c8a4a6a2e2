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
