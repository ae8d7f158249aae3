"""The reference refuses deterministic algorithms together with fill_uninitialized_memory in dispatch and
combine (deep_ep/utils/envs.py:183-189, called at elastic.py:924 and :1083): torch.empty then launches a
fill kernel that may overlap the communication streams.  This build keeps the same guard and
the same exception type (the reference's plain `assert`: AssertionError)."""
import pytest
import torch

from deepep_amd import ElasticBuffer
from deepep_amd.utils import check_torch_deterministic


@pytest.fixture
def deterministic_fill():
    before = (torch.are_deterministic_algorithms_enabled(), torch.utils.deterministic.fill_uninitialized_memory)
    torch.use_deterministic_algorithms(True)
    torch.utils.deterministic.fill_uninitialized_memory = True
    try:
        yield
    finally:
        torch.use_deterministic_algorithms(before[0])
        torch.utils.deterministic.fill_uninitialized_memory = before[1]


def test_guard_passes_by_default():
    check_torch_deterministic()


def test_dispatch_and_combine_refuse_deterministic_fill(deterministic_fill):
    with pytest.raises(AssertionError):
        check_torch_deterministic()
    # the guard is the first thing either call does (nothing about the buffer is touched before it)
    with pytest.raises(AssertionError):
        ElasticBuffer.combine(object(), None, None)
    with pytest.raises(AssertionError):
        ElasticBuffer.dispatch(object(), None)
