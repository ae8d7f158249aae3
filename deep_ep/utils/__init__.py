"""`deep_ep.utils` import path of the reference (deep_ep/utils/__init__.py), for the modules on the combine path."""
