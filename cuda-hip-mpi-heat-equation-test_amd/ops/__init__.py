"""Native engine binding and raw kernel ops (see _native.py, kernels.py)."""
