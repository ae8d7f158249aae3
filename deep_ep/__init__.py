"""`import deep_ep` alias for deepep_amd, so code written against the reference's
Python surface runs unchanged on MI355X (combine path: deep_ep.ElasticBuffer)."""
from deepep_amd import *  # noqa: F401,F403
from deepep_amd import ElasticBuffer, EPHandle, EventHandle, EventOverlap, topk_idx_t, __version__  # noqa: F401
