"""`deep_ep.utils.envs` import path of the reference (deep_ep/utils/envs.py:116-189): the domain sizes of a
single-node group and the deterministic-mode check the combine runs."""
from deepep_amd import get_logical_domain_size, get_physical_domain_size  # noqa: F401
from deepep_amd.utils import check_torch_deterministic  # noqa: F401
