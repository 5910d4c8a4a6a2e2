"""The C ABI library: builds for gfx950, loads without a GPU, and exports
every entry point include/strawboat_gpu.h declares (no compute calls)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "strawboat_gpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(sb_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    import pa_amd

    L = pa_amd.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    from pa_amd import _native

    assert set(_native.EXPORTED) == set(syms)


def test_library_has_gfx950_code_object():
    lib = open(os.path.join(ROOT, "pa_amd", "libstrawboat_gpu.so"), "rb").read()
    assert b"gfx950" in lib


def test_status_strings_and_no_gpu_errors_cleanly():
    import pa_amd

    L = pa_amd.lib()
    assert L.sb_status_str(0) == b"ok"
    assert L.sb_status_str(1) == b"out of spec"
    h = ctypes.c_void_p()
    import torch

    if not torch.cuda.is_available():
        assert L.sb_ctx_create(0, ctypes.byref(h)) == 5  # SB_E_DEVICE, no abort


def test_read_meta_roundtrip_host():
    import numpy as np

    import pa_amd

    w = pa_amd.NativeWriter(pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=2048))
    w.start()
    rng = np.random.default_rng(0)
    cols = [(rng.integers(0, 100, 5000).astype(np.int32), None, False),
            (rng.standard_normal(5000), rng.random(5000) > 0.1, True)]
    w.write(cols)
    f = w.finish()
    assert f[:6] == b"ARROW2" and f[-8:] == b"\xff\xff\xff\xff\x00\x00\x00\x00"
    metas = pa_amd.read_meta(f)
    assert len(metas) == 2 and metas[0].offset == 8
    assert [p.num_values for p in metas[0].pages] == [2048, 2048, 904]
    assert metas[1].offset == metas[0].offset + metas[0].total_len()
    assert metas[0].skip_one_page().offset == 8 + metas[0].pages[0].length
