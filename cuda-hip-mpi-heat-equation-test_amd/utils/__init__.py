"""Config (input.dat), I/O writers, plotting, metrics and checkpointing."""
