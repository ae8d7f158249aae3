"""CPU checks of the C-ABI boundary: the in-tree library loads, exports every function
include/deepep_amd.h declares with the ABI version the host layer expects, and rejects
invalid arguments with an error code and message before touching the GPU."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    text = open(os.path.join(ROOT, 'include', 'deepep_amd.h')).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(deepep_\w+)\s*\(', text)))


@pytest.fixture(scope='module')
def lib():
    import __graft_entry__
    __graft_entry__.build()
    from deepep_amd import _lib
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    from deepep_amd import _lib
    declared = _declared_functions()
    assert declared, 'no declarations parsed'
    for name in declared:
        assert hasattr(lib, name), f'{name} not exported'
    assert sorted(_lib.SIGNATURES) == declared


def test_abi_version(lib):
    assert lib.deepep_amd_abi_version() == 14


def test_build_id_matches_sources(lib):
    """The loaded binary was built from the tracked sources (build() rebuilds on any difference and
    the loader refuses a stale binary)."""
    from deepep_amd import _lib
    want = _lib.source_build_id()
    assert want is not None and len(want) == 16
    assert lib.deepep_amd_build_id().decode() == want == _lib.binary_build_id(_lib.LIB_PATH)


def test_invalid_arguments_are_rejected_without_a_gpu(lib):
    # mode out of range
    rc = lib.deepep_combine_reduce(7, 0, None, 0, 8, None, 0, 1, None, None, None, 16, 8, 1, 8,
                                   None, 0, None, None, 0, 0, 0, 0, None, None)
    assert rc == -1 and b'mode' in lib.deepep_amd_last_error()
    # hidden not a multiple of 8 elements
    rc = lib.deepep_combine_reduce(1, 0, 16, 1, 8, None, 0, 1, None, None, None, 16, 8, 1, 6,
                                   None, 0, None, None, 0, 0, 0, 0, None, None)
    assert rc == -1 and b'hidden' in lib.deepep_amd_last_error()
    # misaligned pointers
    rc = lib.deepep_combine_reduce(1, 0, 18, 1, 8, None, 0, 1, None, None, None, 32, 8, 1, 8,
                                   None, 0, None, None, 0, 0, 0, 0, None, None)
    assert rc == -1 and b'aligned' in lib.deepep_amd_last_error()
    # bias in the local phase
    rc = lib.deepep_combine_reduce(0, 0, 16, 1, 8, None, 0, 1, None, 32, None, 48, 8, 1, 8,
                                   None, 0, None, None, 0, 0, 0, 0, None, None)
    assert rc == -1 and b'bias' in lib.deepep_amd_last_error()
    # table width beyond top-32
    rc = lib.deepep_combine_reduce(1, 0, 16, 1, 8, 64, 40, 33, None, None, None, 48, 8, 1, 8,
                                   None, 0, None, None, 0, 0, 0, 0, None, None)
    assert rc == -1
    # zero units: nothing to do, success without a launch
    assert lib.deepep_combine_reduce(1, 0, 16, 1, 8, None, 0, 1, None, None, None, 48, 8, 0, 8,
                                     None, 0, None, None, 0, 0, 0, 0, None, None) == 0
    # launch configuration knobs out of range (vectors per lane 0-2, rows in flight 0 / 2 / 4 / 8)
    assert lib.deepep_set_launch_config(3, 0) == -1 and b'launch configuration' in lib.deepep_amd_last_error()
    assert lib.deepep_set_launch_config(0, 3) == -1
    assert lib.deepep_set_launch_config(-1, 0) == -1
    assert lib.deepep_set_launch_config(2, 8) == 0
    assert lib.deepep_set_launch_config(0, 0) == 0
    # EP > 1 plan builders: rank out of range, too few blocks, wrong table width, single w/o expanded
    assert lib.deepep_plan_expert(16, 4, 8, 8, 8, 64, 16, 16, 1, 1, 1, 16, None, None, 0, 0, None, None,
                                  0, None) == -1
    assert b'plan_expert' in lib.deepep_amd_last_error()
    assert lib.deepep_plan_expert(16, 4, 8, 8, 0, 64, 16, 16, 1, 1, 2, 16, None, None, 0, 0, None, None,
                                  0, None) == -1
    # out_rows need window bases and an extent of at least one row; a negative padded stride
    assert lib.deepep_plan_expert(16, 4, 8, 8, 0, 64, 16, 16, 1, 1, 1, 16, None, 32, 256, 128, 48, None,
                                  0, None) == -1
    assert lib.deepep_plan_expert(16, 4, 8, 8, 0, 64, 16, 16, 1, 1, 1, 16, None, None, 0, 0, None, None,
                                  -1, None) == -1
    # the scatter needs its windows (bases and an extent holding a whole row)
    assert lib.deepep_combine_reduce_scatter(0, 16, 4, 64, None, 0, 1, None, 32, 4, 64, None, 0, None, 0, 0, 0,
                                             None, 1, 4096, None, None) == -1
    assert b'window' in lib.deepep_amd_last_error()
    assert lib.deepep_combine_reduce_scatter(0, 16, 4, 64, None, 0, 1, None, 32, 4, 64, None, 0, None, 0, 0, 0,
                                             48, 1, 64, None, None) == -1
    # dispatch pack: negative destination rows
    assert lib.deepep_plan_source(16, 200, 8, 64, 8, 0, 256, 16, 16, 16, 1, 1, 0, 0, 0, 16, 8, None, 0, None) == -1
    assert lib.deepep_plan_source(16, 64, 8, 64, 8, 0, 256, 16, 16, 16, 1, 1, 0, 0, 0, 16, 7, None, 0, None) == -1
    # rank outside [0, num_ranks)
    assert lib.deepep_plan_source(16, 64, 8, 64, 8, 8, 256, 16, 16, 16, 1, 1, 0, 0, 0, 16, 8, None, 0, None) == -1
    # a padded stride with window rows (the window layout is never padded)
    assert lib.deepep_plan_source(16, 64, 8, 64, 8, 0, 256, 16, 16, 16, 4, 1, 16, 0, 0, 16, 8, None, 64, None) == -1
    assert lib.deepep_dispatch_pack(16, 64, 64, None, 0, 0, 32, None, 4, 2, 0, 48, 64, 2, 80, None, 128, -1,
                                    64, 64, 96, 112, None, None) == -1
    assert lib.deepep_route_block_counts(16, 200, 8, 64, 8, 1, 16, 16, None) == -1
    assert lib.deepep_route_block_counts(None, 0, 8, 64, 8, 0, None, None, None) == 0     # nothing to count
    # a window put must stay inside the destination window: offset + bytes past the extent, or an offset
    # beyond it, is rejected before any launch (16-byte aligned fake pointers: nothing is dereferenced)
    assert lib.deepep_sym_put(16, 64, 32, 2, 65536, 65536 + 48, None, None) == -1
    assert b'outside' in lib.deepep_amd_last_error()
    assert lib.deepep_sym_put(16, 16, 32, 2, 1 << 20, 1 << 19, None, None) == -1
    assert lib.deepep_sym_put(16, 16, 32, 2, 0, -1, None, None) == -1
    assert lib.deepep_sym_put(16, 0, 32, 2, 0, 0, None, None) == 0            # nothing to store
    # a CU budget is whole CUs per XCD; nonsense is rejected
    assert lib.deepep_stream_create_cu_budget(0, None) == -1


def test_buffer_size_matches_reference_formula(lib):
    from deepep_amd.buffer import calculate_buffer_size
    # ElasticBuffer::get_combine_buffer_size, one node: min(R, K) slots x T x (align(2H, 32) + align(8K, 32))
    assert lib.deepep_combine_buffer_size(4096, 7168, 8, 8, 1) == 8 * 4096 * (14336 + 64)
    assert lib.deepep_combine_buffer_size(128, 1024, 2, 8, 1) == 2 * 128 * (2048 + 32)
    assert lib.deepep_combine_buffer_size(128, 1024, 2, 1, 0) == 2 * 128 * (2048 + 32)
    assert lib.deepep_combine_buffer_size(0, 7168, 8, 8, 1) < 0
    size = calculate_buffer_size(8, 4096, 7168, 8, False, True)
    assert size % (2 << 20) == 0 and size >= lib.deepep_combine_buffer_size(4096, 7168, 8, 8, 1)


def test_product_fails_loudly_without_library(tmp_path, monkeypatch):
    from deepep_amd import _lib
    with pytest.raises(_lib.LibraryMissing):
        _lib.load(str(tmp_path / 'missing.so'))


def test_header_is_plain_c():
    """include/deepep_amd.h compiles as strict ISO C (what a cgo / C FFI consumer includes), and the
    C consumer of tests/abi_c builds against it with -Werror."""
    import subprocess
    import __graft_entry__ as g
    src = '#include "deepep_amd.h"\nint main(void) { return deepep_amd_abi_version() == DEEPEP_AMD_ABI_VERSION ? 0 : 1; }\n'
    r = subprocess.run(['gcc', '-std=c99', '-pedantic', '-Wall', '-Wextra', '-Werror', '-fsyntax-only',
                        '-I', os.path.join(ROOT, 'include'), '-x', 'c', '-'], input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(['gcc', '-std=c11', '-Wall', '-Wextra', '-Werror', '-D__HIP_PLATFORM_AMD__',
                        '-I/opt/rocm/include', '-fsyntax-only', g.C_CONSUMER + '.c'], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_reference_version_and_alias():
    """`import deep_ep` reports the reference's API level (deep_ep/__init__.py:97) and its classes are
    this build's; the build's own version stays available beside it."""
    import deep_ep
    import deepep_amd
    assert deep_ep.__version__ == '2.1.0'
    assert deep_ep.ElasticBuffer is deepep_amd.ElasticBuffer
    assert deep_ep.EPHandle is deepep_amd.EPHandle
    assert deepep_amd.__build_version__ != deep_ep.__version__


def test_reference_submodule_import_paths():
    """The reference's own import paths for the combine path's Python surface resolve to this build's
    objects (deep_ep/buffers/elastic.py, deep_ep/utils/event.py, deep_ep/utils/envs.py)."""
    import deepep_amd
    from deep_ep.buffers.elastic import ElasticBuffer, EPHandle
    from deep_ep.utils.envs import check_torch_deterministic, get_logical_domain_size, get_physical_domain_size
    from deep_ep.utils.event import EventHandle, EventOverlap
    assert ElasticBuffer is deepep_amd.ElasticBuffer and EPHandle is deepep_amd.EPHandle
    assert EventOverlap is deepep_amd.EventOverlap and EventHandle is deepep_amd.EventHandle
    assert get_physical_domain_size is deepep_amd.get_physical_domain_size
    assert get_logical_domain_size is deepep_amd.get_logical_domain_size
    assert callable(check_torch_deterministic)
