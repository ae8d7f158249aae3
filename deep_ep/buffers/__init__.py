"""`deep_ep.buffers` import path of the reference (deep_ep/buffers/__init__.py); the combine path's buffer."""
