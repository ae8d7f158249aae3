"""`deep_ep.buffers.elastic` import path of the reference (deep_ep/buffers/elastic.py): the combine path's
ElasticBuffer and EPHandle are this build's (deepep_amd)."""
from deepep_amd.buffer import ElasticBuffer, calculate_buffer_size  # noqa: F401
from deepep_amd.handle import EPHandle  # noqa: F401
