"""`deep_ep.utils.event` import path of the reference (deep_ep/utils/event.py)."""
from deepep_amd.event import EventHandle, EventOverlap  # noqa: F401
