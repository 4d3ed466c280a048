"""The C-ABI library loads and exports every symbol include/dsybloom.h declares (CPU only; no compute calls)."""
import ctypes
import os
import re

import pytest

from dispersy_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dsybloom.h")


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(dsy_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("dsy_bloom_add", "dsy_bloom_test", "dsy_sync_respond", "dsy_store_upload", "dsy_ctx_create"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.isfile(_native.LIB_PATH):
        pytest.fail("libdsybloom.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    assert sorted(_native.SIGNATURES) == declared_functions()


def test_host_only_entry_points():
    lib = _native.load_library()
    assert lib.dsy_abi_version() == 1
    assert lib.dsy_filter_words(10160) == 318
    k, c = ctypes.c_int32(), ctypes.c_uint32()
    # bloomfilter.py:134-156 table
    for m, kf, kind, chunk in ((10160, 7, 0, 2), (4096, 10, 1, 2), (1 << 20, 7, 2, 4), (1 << 15, 10, 3, 4),
                               (1 << 16, 14, 4, 4), (1 << 31, 7, 4, 8), (1 << 33, 5, 3, 8), (32768, 4, 0, 4)):
        assert lib.dsy_hash_family(m, kf, ctypes.byref(k), ctypes.byref(c)) == 0
        assert (k.value, c.value) == (kind, chunk), (m, kf)
    assert lib.dsy_hash_family(12, 3, ctypes.byref(k), ctypes.byref(c)) == _native.DSY_EINVAL
    assert b"multiple of eight" in lib.dsy_last_error()
    assert lib.dsy_hash_family(1 << 16, 17, ctypes.byref(k), ctypes.byref(c)) == _native.DSY_EINVAL
    assert lib.dsy_hash_family(64, 65, ctypes.byref(k), ctypes.byref(c)) == _native.DSY_EINVAL


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_native.BloomParams) == 8 + 4 * 4 + 256
    assert ctypes.sizeof(_native.Request) == 8 * 2 + 4 * 2 + 8 * 2 + 4 * 4 + 256
    assert ctypes.sizeof(_native.Meta) == 24


def test_constants_match_header():
    text = open(HEADER).read()
    defs = dict(re.findall(r"^#define\s+(DSY_\w+)\s+(\d+)\b", text, flags=re.M))
    assert int(defs["DSY_BLOB_GUARD"]) == _native.BLOB_GUARD
    assert int(defs["DSY_SIM_RESP_MAX"]) == _native.SIM_RESP_MAX


def test_status_codes_match_header():
    defs = dict(re.findall(r"^#define\s+(DSY_E\w+|DSY_OK)\s+(-?\d+)\b", open(HEADER).read(), flags=re.M))
    for name, val in defs.items():
        assert getattr(_native, name) == int(val), name


def test_bytes_gather_addresses_point_at_the_data():
    """SyncStore.append hands bytes packets to dsy_store_append_gather by address (id + the object header): the
    offset found at import reads back every packet's bytes, empty and large ones included (CPU)."""
    import ctypes
    import numpy as np
    from dispersy_amd.store import _BYTES_DATA
    assert _BYTES_DATA == bytes.__basicsize__ - 1
    rng = np.random.Generator(np.random.PCG64(3))
    packets = [b"", b"x"] + [rng.bytes(int(n)) for n in rng.integers(1, 70_000, 50)]
    addrs = np.fromiter(map(id, packets), dtype=np.uint64, count=len(packets)) + np.uint64(_BYTES_DATA)
    for p, a in zip(packets, addrs.tolist()):
        assert ctypes.string_at(a, len(p)) == p
