"""Heat-equation models: the distributed FTCS solver, reference-variant presets and the NumPy golden."""
