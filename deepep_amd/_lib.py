"""ctypes binding of libdeepep_amd.so (C-ABI in include/deepep_amd.h).

The library is built in-tree by __graft_entry__.build() (hipcc --offload-arch=gfx950).
There is no fallback: if the library is missing or a call fails, the error is raised
(RuntimeError, as the reference's EP_HOST_ASSERT -> EPException does).
"""
import ctypes
import hashlib
import os
import threading
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('DEEPEP_AMD_LIB', os.path.join(_HERE, 'libdeepep_amd.so'))
SOURCES = [os.path.join(_HERE, 'csrc', f) for f in ('combine.hip', 'dispatch.hip', 'symmetric.hip', 'plan.hip', 'fault.h')]
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'deepep_amd.h')
HIPCC_FLAGS = ['--offload-arch=gfx950', '-O3', '-fPIC', '-std=c++17', '-Wall']


def source_build_id() -> Optional[str]:
    """sha256 (16 hex digits) of the library's sources, header and compile flags; None when the
    sources are not next to the package."""
    if not all(os.path.exists(p) for p in SOURCES + [HEADER]):
        return None
    h = hashlib.sha256(' '.join(HIPCC_FLAGS).encode())
    for p in SOURCES + [HEADER]:
        h.update(os.path.basename(p).encode())
        with open(p, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def binary_build_id(path: str) -> Optional[str]:
    """The build id compiled into a library file (read from its bytes, nothing is loaded)."""
    if not os.path.exists(path):
        return None
    with open(path, 'rb') as f:
        data = f.read()
    i = data.find(b'DEEPEP_BUILD_ID=')
    return data[i + 16:i + 32].decode(errors='replace') if i >= 0 else None
ABI_VERSION = 14

MODE_LOCAL, MODE_EPILOGUE, MODE_FUSED = 0, 1, 2

# error record of the window paths (DEEPEP_ERROR_RECORD_INTS, DEEPEP_FLAG_*, DEEPEP_FAULT_*)
ERROR_RECORD_INTS = 8
FLAG_BAD_SLOT, FLAG_TIMEOUT, FLAG_BAD_ADDRESS = 1, 2, 4
FAULT_NAMES = {1: 'scatter row outside every window', 2: 'plan window row past its window',
               3: 'plan unit / received row out of range', 4: 'dispatch row past its destination buffer'}


def describe_error_record(rec) -> str:
    """Human-readable text of an error record (a sequence of DEEPEP_ERROR_RECORD_INTS ints)."""
    rec = [int(v) for v in rec]
    bits = [n for b, n in ((FLAG_BAD_SLOT, 'rejected slot / unit'), (FLAG_TIMEOUT, 'barrier timeout'),
                           (FLAG_BAD_ADDRESS, 'address outside every window')) if rec[0] & b]
    text = f'error flag {rec[0]} ({", ".join(bits) or "none"})'
    if len(rec) > 6 and rec[1]:
        addr = (rec[5] & 0xffffffff) << 32 | (rec[4] & 0xffffffff)
        text += (f'; first fault: {FAULT_NAMES.get(rec[1], rec[1])}, unit/row {rec[2]}, rank/lane {rec[3]}, '
                 f'address {addr:#x}, extent {rec[6]}')
    return text

# deepep_plan_* (include/deepep_amd.h)
PLAN_BLOCK_TOKENS = 64
DISPATCH_BLOCK_ROWS = 128          # DEEPEP_DISPATCH_BLOCK_ROWS: receive-side block of the dispatch
PLAN_EXPANDED, PLAN_SINGLE, PLAN_INTERLEAVE, PLAN_RANK_LAYOUT, PLAN_WINDOW, PLAN_LOCAL_BYPASS = 1, 2, 4, 8, 16, 32

_lib = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64

# Every symbol include/deepep_amd.h declares, with its ctypes signature.
SIGNATURES = {
    'deepep_amd_abi_version': (_I, []),
    'deepep_amd_last_error': (ctypes.c_char_p, []),
    'deepep_amd_build_id': (ctypes.c_char_p, []),
    'deepep_combine_reduce': (_I, [_I, _I,
                                   _P, _I64, _I64,
                                   _P, _I64, _I,
                                   _P,
                                   _P, _P,
                                   _P, _I64,
                                   _I, _I,
                                   _P, _I64,
                                   _P, _P, _I,
                                   _I64, _I,
                                   _I, _P,
                                   _P]),
    'deepep_build_local_plan': (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _P, _P, _P]),
    'deepep_set_launch_config': (_I, [_I, _I]),
    'deepep_combine_buffer_size': (_I64, [_I, _I, _I, _I, _I]),
    'deepep_dispatch_route': (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P]),
    'deepep_dispatch_notify': (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I64, _P]),
    'deepep_dispatch_notify_workspace': (_I64, [_I, _I, _I]),
    'deepep_dispatch_receive': (_I, [_P, _I64, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _P, _P, _P, _I, _I, _P,
                                     _P, _P, _P]),
    'deepep_dispatch_expert_counts': (_I, [_P, _I, _I, _I, _P, _P]),
    'deepep_dispatch_pack': (_I, [_P, _I64, _I, _P, _I64, _I, _P, _P, _I, _I, _I, _P, _P, _I,
                                  _P, _P, _I64, _I64, _I, _I, _I, _I, _P, _P]),
    'deepep_dispatch_count': (_I, [_P, _I64, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _P, _P, _P, _P]),
    'deepep_dispatch_scan': (_I, [_P, _I, _I, _I, _I, _P, _P, _P]),
    'deepep_dispatch_slots': (_I, [_P, _I64, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    'deepep_dispatch_copy': (_I, [_P, _I64, _I, _I, _I, _I, _I, _I, _P, _I, _P, _I64, _P, _I64, _I,
                                  _P, _P, _P, _I64, _P, _P, _P, _I, _P, _P, _P]),
    'deepep_route_block_counts': (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    'deepep_plan_expert': (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _I, _I, _I, _P, _P, _P, _I64, _I64, _P, _P, _I,
                                _P]),
    'deepep_plan_source': (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I64, _I64, _P, _I, _P, _I, _P]),
    'deepep_sym_alloc': (_I, [_I64, ctypes.POINTER(ctypes.c_void_p)]),
    'deepep_sym_free': (_I, [_P]),
    'deepep_sym_export': (_I, [_P, _P]),
    'deepep_sym_import': (_I, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    'deepep_sym_close': (_I, [_P]),
    'deepep_sym_barrier': (_I, [_P, _I, _I, _I64, _I64, _P, _P]),
    'deepep_sym_put': (_I, [_P, _I64, _P, _I, _I64, _I64, _P, _P]),
    'deepep_sym_signal': (_I, [_P, _I, _I, _I, _I64, _P]),
    'deepep_sym_wait': (_I, [_P, _I, _I, _I, _I64, _I64, _P, _P]),
    'deepep_stream_create_cu_budget': (_I, [_I, ctypes.POINTER(ctypes.c_void_p)]),
    'deepep_stream_destroy': (_I, [_P]),
    'deepep_stream_probe_cus': (_I, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    'deepep_combine_reduce_scatter': (_I, [_I, _P, _I64, _I64, _P, _I64, _I, _P, _P, _I, _I, _P, _I64, _P, _I,
                                           _I64, _I, _P, _I, _I64, _P, _P]),
}


class LibraryMissing(RuntimeError):
    pass


def load(path: Optional[str] = None):
    """Load (once) and return the ctypes library; raise LibraryMissing if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise LibraryMissing(f'deepep_amd: HIP library not found at {p}; run __graft_entry__.build()')
        want = source_build_id() if path is None and 'DEEPEP_AMD_LIB' not in os.environ else None
        if want is not None and binary_build_id(p) != want:
            raise RuntimeError(f'deepep_amd: {p} was built from other sources (build id {binary_build_id(p)}, '
                               f'sources {want}); run __graft_entry__.build()')
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        version = lib.deepep_amd_abi_version()
        if version != ABI_VERSION:
            raise RuntimeError(f'deepep_amd: ABI version {version} != expected {ABI_VERSION}')
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().deepep_amd_last_error().decode(errors='replace')
        raise RuntimeError(f'deepep_amd: {what} failed ({rc}): {msg}')


def ptr(t) -> Optional[int]:
    """Raw device address of a tensor (None for None)."""
    return None if t is None else t.data_ptr()
