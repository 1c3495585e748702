"""Checkpoint / restart (absent in the reference: its only dumps, int.dat /
soln.dat / soln%05d.dat, are never read back — SURVEY.md §5).

Layout of a checkpoint directory:
    meta.json           problem + solver parameters + completed step count
    rank00000.npy ...   each rank's owned rows (plain .npy, loaded with allow_pickle=False)

Restart re-decomposes: a run on P ranks can resume a checkpoint written by Q
ranks (each rank memory-maps the rank files and copies its own row range), so
jobs can move between GPU counts. Restarting is bitwise exact: the state is the
full owned field and FTCS carries no other state.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import numpy as np

FORMAT = "heat2d-checkpoint-v1"


def save(solver, directory: str, step: Optional[int] = None, extra: Optional[dict] = None) -> None:
    """Collective: every rank writes its slab; rank 0 writes meta.json last."""
    os.makedirs(directory, exist_ok=True)
    local = solver.download()
    np.save(os.path.join(directory, f"rank{solver.rank:05d}.npy"), local, allow_pickle=False)
    _barrier(solver)
    if solver.rank == 0:
        p = solver.problem
        meta = {
            "format": FORMAT,
            "step": int(solver.steps_done if step is None else step),
            "nranks": solver.size,
            "dtype": "fp64" if local.dtype == np.float64 else "fp32",
            "n_owned": p.n_owned,
            "n_input": p.n_input,
            "convention": p.convention,
            "sigma": p.sigma, "nu": p.nu, "dom_len": p.dom_len, "r": p.r,
            "rows": [],
        }
        meta.update(extra or {})
        tmp = os.path.join(directory, "meta.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(tmp, os.path.join(directory, "meta.json"))
    _barrier(solver)


def load_meta(directory: str) -> dict:
    with open(os.path.join(directory, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{directory}: not a {FORMAT} checkpoint")
    return meta


def load(solver, directory: str) -> dict:
    """Collective: fill the solver's owned rows from a checkpoint (any writer rank count)."""
    meta = load_meta(directory)
    if meta["n_owned"] != solver.problem.n_owned:
        raise ValueError(f"checkpoint grid {meta['n_owned']} != solver grid {solver.problem.n_owned}")
    if meta["convention"] != solver.problem.convention:
        raise ValueError("checkpoint grid convention differs")
    parts = [np.load(os.path.join(directory, f"rank{r:05d}.npy"), mmap_mode="r", allow_pickle=False)
             for r in range(meta["nranks"])]
    starts = np.cumsum([0] + [p.shape[0] for p in parts])
    r0, r1 = solver.row0, solver.row0 + solver.nrows
    out = np.empty((solver.nrows, solver.ncols), dtype=solver.np_dtype)
    for i, part in enumerate(parts):
        a, b = max(r0, starts[i]), min(r1, starts[i + 1])
        if a < b:
            out[a - r0:b - r0] = part[a - starts[i]:b - starts[i]]
    solver.upload(out)  # + halo exchange (collective)
    return meta


def _barrier(solver) -> None:
    if solver.size > 1:
        import torch.distributed as dist
        dist.barrier()
