"""Slab decomposition, halo-exchange transports and the process launcher."""
