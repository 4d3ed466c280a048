"""ctypes binding of the C-ABI in include/dsybloom.h (libdsybloom.so, hand-written HIP for gfx950).

There is no CPU fallback: if the shared library is missing or no GPU is visible, using any compute entry point
raises `NativeUnavailable`.  Only the pure host logic of the package (sizing math, serialisation, selection
bookkeeping) runs without it.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSY_LIB", os.path.join(_HERE, "libdsybloom.so"))

DSY_OK, DSY_EINVAL, DSY_EHIP, DSY_ENOMEM, DSY_ECAPACITY, DSY_EUNSORTED, DSY_EEMPTY, DSY_EINTERNAL = 0, -1, -2, -3, -4, -5, -6, -7
DSY_MD5, DSY_SHA1, DSY_SHA256, DSY_SHA384, DSY_SHA512 = range(5)
HASH_KINDS = {"md5": DSY_MD5, "sha1": DSY_SHA1, "sha256": DSY_SHA256, "sha384": DSY_SHA384, "sha512": DSY_SHA512}
DSY_ASC, DSY_DESC, DSY_RANDOM = 0, 1, 2
# dsy_dup_check verdicts (include/dsybloom.h)
DSY_DUP_NEW, DSY_DUP_EXACT, DSY_DUP_KEEP, DSY_DUP_REPLACE, DSY_DUP_TRIPLET = range(5)
DIRECTIONS = {"ASC": DSY_ASC, "DESC": DSY_DESC, "RANDOM": DSY_RANDOM}
BLOB_GUARD = 256
SIM_RESP_MAX = 64  # DSY_SIM_RESP_MAX: packets per simulator response record
SYNC_HEADER = 24  # DSY_SYNC_HEADER: '>QQHHBH' + the 1-byte prefix (conversion.py:727-728)

# the ctx timer classes of dsy_ctx_kernel_time
TIME_PAIR_TEST, TIME_BLOOM, TIME_SELECT, TIME_COMPACT, TIME_SIM_BUILD, TIME_SIM_RESPOND = 0, 1, 2, 3, 4, 5


class NativeUnavailable(RuntimeError):
    """The HIP extension could not be loaded or no MI355X is visible; there is no CPU fallback."""


class DsyError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("dsybloom error %d: %s" % (code, msg))
        self.code = code


class BloomParams(ctypes.Structure):
    _fields_ = [("m_bits", ctypes.c_uint64), ("k", ctypes.c_uint32), ("hash_kind", ctypes.c_int32),
                ("chunk_bytes", ctypes.c_uint32), ("prefix_len", ctypes.c_uint32), ("prefix", ctypes.c_uint8 * 256)]


class Request(ctypes.Structure):
    _fields_ = [("time_low", ctypes.c_uint64), ("time_high", ctypes.c_uint64), ("modulo", ctypes.c_uint32),
                ("offset", ctypes.c_uint32), ("filter_offset", ctypes.c_uint64), ("m_bits", ctypes.c_uint64),
                ("k", ctypes.c_uint32), ("hash_kind", ctypes.c_int32), ("chunk_bytes", ctypes.c_uint32),
                ("prefix_len", ctypes.c_uint32), ("prefix", ctypes.c_uint8 * 256)]


class Meta(ctypes.Structure):
    _fields_ = [("meta_id", ctypes.c_uint32), ("direction", ctypes.c_int32), ("has_pruning", ctypes.c_uint32),
                ("_pad", ctypes.c_uint32), ("inactive_threshold", ctypes.c_uint64)]


_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32
_I32 = ctypes.c_int32
_PU64 = ctypes.POINTER(ctypes.c_uint64)

# name -> (restype, argtypes); exactly the functions declared in include/dsybloom.h
SIGNATURES = {
    "dsy_abi_version": (ctypes.c_int, []),
    "dsy_last_error": (ctypes.c_char_p, []),
    "dsy_filter_words": (_U64, [_U64]),
    "dsy_hash_family": (ctypes.c_int, [_U64, _U32, ctypes.POINTER(_I32), ctypes.POINTER(_U32)]),
    "dsy_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "dsy_ctx_destroy": (ctypes.c_int, [_P]),
    "dsy_ctx_synchronize": (ctypes.c_int, [_P]),
    "dsy_ctx_stream": (_P, [_P]),
    "dsy_ctx_wait_stream": (ctypes.c_int, [_P, _P]),
    "dsy_ctx_signal_stream": (ctypes.c_int, [_P, _P]),
    "dsy_ctx_wait_event": (ctypes.c_int, [_P, _P]),
    "dsy_ctx_set_timing": (ctypes.c_int, [_P, ctypes.c_int]),
    "dsy_ctx_kernel_time": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), _PU64, _PU64, _PU64]),
    "dsy_ctx_reset_timing": (ctypes.c_int, [_P]),
    "dsy_ctx_work": (ctypes.c_int, [_P, ctypes.c_int, _PU64]),
    "dsy_ctx_set_window": (ctypes.c_int, [_P, _U64]),
    "dsy_bloom_add": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _U64, _P, _U64, _P]),
    "dsy_bloom_test": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _U64, _P, _U64, _P, _P]),
    "dsy_bloom_indices": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _U64, _P, _U64, _P]),
    "dsy_bloom_add_dev": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _P, _U64, _P]),
    "dsy_bloom_test_dev": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _P, _U64, _P, _P]),
    "dsy_store_upload": (ctypes.c_int, [_P, _P, _U64, _P, _U64, _P, _P, _P, ctypes.POINTER(_P)]),
    "dsy_store_attach": (ctypes.c_int, [_P, _P, _U64, _P, _U64, _P, _P, _P, ctypes.POINTER(_P)]),
    "dsy_store_free": (ctypes.c_int, [_P]),
    "dsy_store_rows": (_U64, [_P]),
    "dsy_store_append": (ctypes.c_int, [_P, _P, _P, _U64, _P, _U64, _P, _P, _P]),
    "dsy_store_append_gather": (ctypes.c_int, [_P, _P, _P, _P, _U64, _P, _P, _P]),
    "dsy_store_index_stats": (ctypes.c_int, [_P, _P]),
    "dsy_store_index_members": (ctypes.c_int, [_P, _P, _P, _P, _U64]),
    "dsy_store_prune": (ctypes.c_int, [_P, _P, _U32, _U64, _PU64]),
    "dsy_store_delete": (ctypes.c_int, [_P, _P, _P, _U64, _PU64]),
    "dsy_store_set_undone": (ctypes.c_int, [_P, _P, _P, _U64, _P, _P, ctypes.c_int, _PU64]),
    "dsy_dup_check": (ctypes.c_int, [_P, _P, _P, _P, _P, _U64, _P, _U64, _P, _P, _P]),
    "dsy_store_replace": (ctypes.c_int, [_P, _P, _P, _P, _U64, _P, _U64]),
    "dsy_bloom_add_rows": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _P, _U64, _P]),
    "dsy_claim_modulo": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _P, _U32, _U64, _U64, _P, _PU64]),
    "dsy_claim_largest": (ctypes.c_int, [_P, ctypes.POINTER(BloomParams), _P, _P, _U32, _U64, _U64, _U64, _U64, _P, _P]),
    "dsy_sync_respond": (ctypes.c_int, [_P, _P, ctypes.POINTER(Request), _U32, _P, _U64, ctypes.POINTER(Meta), _U32,
                                        _U64, ctypes.c_int, ctypes.c_int64, _U64, _P, _U64, _P]),
    "dsy_sync_respond_refs": (ctypes.c_int, [_P, _P, _P, _P, _U32, ctypes.POINTER(Meta), _U32, _U64, ctypes.c_int,
                                             ctypes.c_int64, _U64, _P, _U64, _P]),
    "dsy_sync_respond_dev": (ctypes.c_int, [_P, _P, ctypes.POINTER(Request), _U32, _P, ctypes.POINTER(Meta), _U32,
                                            _U64, ctypes.c_int, ctypes.c_int64, _U64, ctypes.POINTER(_P),
                                            ctypes.POINTER(_P), _PU64]),
    "dsy_sync_respond_submit": (ctypes.c_int, [_P, _P, ctypes.POINTER(Request), _U32, _P, ctypes.POINTER(Meta), _U32,
                                                _U64, ctypes.c_int, ctypes.c_int64, _U64, _PU64]),
    "dsy_sync_respond_wait": (ctypes.c_int, [_P, _U64, ctypes.POINTER(_P), ctypes.POINTER(_P), _PU64]),
    "dsy_filter_or_reduce": (ctypes.c_int, [_P, _P, _U32, _U64, _P]),
    "dsy_sync_decode": (ctypes.c_int, [_P, _P, _U32, _U64, ctypes.POINTER(Request), _P, _U64, _PU64, _P]),
    "dsy_sync_encode": (ctypes.c_int, [ctypes.POINTER(Request), _U32, _P, _P, _U64, _P]),
    "dsy_sim_setup": (ctypes.c_int, [_P]),
    "dsy_sim_seed": (ctypes.c_int, [_P, _P, _P, _U32]),
    "dsy_sim_claim_counts": (ctypes.c_int, [_P, _P, _U32, _P, _U32]),
    "dsy_sim_claim_matrix": (ctypes.c_int, [_P, _P, _U32, _U32, _P, _U32]),
    "dsy_sim_build_claims": (ctypes.c_int, [_P, _P, _U32, _P, _P, _P, _P, _P, _U32]),
    "dsy_sim_resp_counts": (ctypes.c_int, [_P, _P, _P, _U64, _P, _U32]),
    "dsy_sim_respond": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _U64, _P, _P, _U32, _PU64]),
    "dsy_sim_merge": (ctypes.c_int, [_P, _P, _P, _P, _U64]),
    "dsy_sim_stats": (ctypes.c_int, [_P, _P, _P, _P]),
}

_lib = None
_lib_lock = threading.Lock()


def load_library():
    """Load libdsybloom.so (DSY_LIB_PATH: another build of it, for same-box A/B runs of a kernel change).  torch is imported first (when present) so the library binds to the same HIP runtime
    (libamdhip64.so.7) torch uses and device pointers are shared between them."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("DSY_LIB_PATH") or LIB_PATH
        if not os.path.isfile(path):
            raise NativeUnavailable("%s is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                                    % path)
        try:
            import torch  # noqa: F401  (shares one HIP runtime with the library)
        except ImportError:
            pass
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dsy_abi_version() != 1:
            raise NativeUnavailable("ABI version mismatch")
        _lib = lib
        return lib


def check(rc):
    if rc != DSY_OK:
        msg = _lib.dsy_last_error().decode(errors="replace") if _lib else "?"
        raise DsyError(rc, msg)


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, (bytes, bytearray, memoryview)):
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p).value
    raise TypeError(type(a))


def bloom_params(m, k, hash_kind, chunk, prefix):
    p = BloomParams()
    p.m_bits, p.k, p.hash_kind, p.chunk_bytes = m, k, hash_kind, chunk
    p.prefix_len = len(prefix)
    ctypes.memmove(p.prefix, bytes(prefix), len(prefix))
    return p


class Context(object):
    """One dsy_ctx (a HIP stream + workspace) on one device."""

    handle = None

    def __init__(self, device=0):
        lib = load_library()
        h = ctypes.c_void_p()
        rc = lib.dsy_ctx_create(device, ctypes.byref(h))
        if rc != DSY_OK:
            raise NativeUnavailable("dsy_ctx_create(%d) failed: %s" % (device, lib.dsy_last_error().decode()))
        self.lib, self.handle, self.device = lib, h, device

    def close(self):
        if self.handle:
            self.lib.dsy_ctx_destroy(self.handle)
            self.handle = None

    __del__ = close

    def synchronize(self):
        check(self.lib.dsy_ctx_synchronize(self.handle))

    @staticmethod
    def _torch_stream(device):
        import torch
        return torch.cuda.current_stream(device).cuda_stream

    def wait_torch(self, device=None):
        """The ctx stream waits (on the device) for what is queued on torch's current stream: e.g. tensors torch
        filled, or an RCCL collective's result."""
        check(self.lib.dsy_ctx_wait_stream(self.handle, self._torch_stream(device)))

    def signal_torch(self, device=None):
        """Torch's current stream waits (on the device) for what is queued on the ctx stream."""
        check(self.lib.dsy_ctx_signal_stream(self.handle, self._torch_stream(device)))

    def signal_stream(self, stream):
        """A torch.cuda.Stream waits (on the device) for what is queued on the ctx stream."""
        check(self.lib.dsy_ctx_signal_stream(self.handle, stream.cuda_stream))

    def wait_event(self, event):
        """The ctx stream waits (on the device) for a recorded torch.cuda.Event."""
        check(self.lib.dsy_ctx_wait_event(self.handle, event.cuda_event))

    def set_timing(self, on, only=None):
        """on: bracket kernel launches with HIP events; only: an iterable of TIME_* classes to bracket (default all)."""
        mode = 0
        if on:
            mode = 1 if only is None else 0x100 | sum(1 << int(w) for w in only)
        check(self.lib.dsy_ctx_set_timing(self.handle, mode))

    def reset_timing(self):
        check(self.lib.dsy_ctx_reset_timing(self.handle))

    def kernel_time(self, which):
        ms, n, blocks, nbytes = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        check(self.lib.dsy_ctx_kernel_time(self.handle, which, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(blocks),
                                           ctypes.byref(nbytes)))
        return dict(ms=ms.value, launches=n.value, blocks=blocks.value, bytes=nbytes.value)

    def set_window(self, max_pairs):
        """Cap the responder window (0: default); results are independent of it."""
        check(self.lib.dsy_ctx_set_window(self.handle, max_pairs))

    def work(self, which):
        """Algorithmic work counters of a timer class (dsy_ctx_work)."""
        out = (ctypes.c_uint64 * 4)()
        check(self.lib.dsy_ctx_work(self.handle, which, out))
        return dict(blocks=out[0], bytes=out[1], useful_pairs=out[2], lane_slots=out[3])

    # ---- single filter
    @staticmethod
    def _keys(blob, offsets):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        blob = bytes(blob)
        return blob, offsets, len(offsets) - 1

    def bloom_add(self, params, blob, offsets, filter_bytes):
        blob, offsets, n = self._keys(blob, offsets)
        buf = ctypes.create_string_buffer(bytes(filter_bytes), len(filter_bytes))
        check(self.lib.dsy_bloom_add(self.handle, ctypes.byref(params), blob, len(blob), offsets.ctypes.data, n, buf))
        return buf.raw

    def bloom_test(self, params, blob, offsets, filter_bytes):
        blob, offsets, n = self._keys(blob, offsets)
        out = np.zeros(max(n, 1), dtype=np.uint8)
        check(self.lib.dsy_bloom_test(self.handle, ctypes.byref(params), blob, len(blob), offsets.ctypes.data, n,
                                      bytes(filter_bytes), out.ctypes.data))
        return out[:n]

    def bloom_indices(self, params, blob, offsets):
        blob, offsets, n = self._keys(blob, offsets)
        out = np.zeros(max(n * params.k, 1), dtype=np.uint64)
        check(self.lib.dsy_bloom_indices(self.handle, ctypes.byref(params), blob, len(blob), offsets.ctypes.data, n,
                                         out.ctypes.data))
        return out[:n * params.k].reshape(n, params.k)


_default = {}
_default_lock = threading.Lock()


def default_context(device=0):
    with _default_lock:
        ctx = _default.get(device)
        if ctx is None:
            ctx = _default[device] = Context(device)
        return ctx
