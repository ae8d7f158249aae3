"""deepep_amd: DeepEP's ElasticBuffer combine path, built for AMD Instinct MI355X (gfx950).

Drop-in surface of `deep_ep` for the combine reduction:
    ElasticBuffer, EPHandle, EventOverlap, EventHandle, topk_idx_t
(deep_ep/__init__.py:90-97 in the reference).  The combine kernels live in
libdeepep_amd.so (hand-written HIP, C-ABI in include/deepep_amd.h).
"""
from .buffer import ElasticBuffer, calculate_buffer_size, topk_idx_t
from .event import EventHandle, EventOverlap
from .handle import EPHandle


def get_physical_domain_size(group=None):
    """(RDMA ranks, xGMI ranks) of a single-node group."""
    import torch.distributed as dist
    n = dist.get_world_size(group)
    return 1, n


def get_logical_domain_size(group=None, allow_hybrid_mode: bool = True):
    """(scale-out ranks, scale-up ranks) of a single-node group."""
    import torch.distributed as dist
    n = dist.get_world_size(group)
    return 1, n


# The API level implemented: the reference's deep_ep.__version__ (deep_ep/__init__.py:97), so caller
# code that gates on it sees the library it was written against.  This build's own version is
# __build_version__; the library's source hash is deepep_amd._lib.source_build_id().
__version__ = '2.1.0'
__build_version__ = '0.6.0'
__all__ = ['ElasticBuffer', 'EPHandle', 'EventOverlap', 'EventHandle', 'topk_idx_t',
           'calculate_buffer_size', 'get_physical_domain_size', 'get_logical_domain_size']
