"""Checkpoint / restart (absent in the reference: its only dumps, int.dat /
soln.dat / soln%05d.dat, are never read back — SURVEY.md §5).

Layout (v2, shared with the native CLI, csrc/runtime/checkpoint.cpp):
    DIR/step-NNNNNNNNNNNN/rank00000.npy ...  each rank's owned rows (plain .npy, allow_pickle=False)
    DIR/step-NNNNNNNNNNNN/meta.json          problem + solver parameters + completed step count
    DIR/latest                               the newest COMPLETE step directory (atomic commit point)

Every save writes into a FRESH directory (``step-N``, or ``step-N-G`` when step N
was saved before — a restart at its final step, a re-run into the same
directory — so files ``latest`` may point at are never overwritten in place);
rank files and meta.json are fsynced, and only after all of them are there does
rank 0 republish ``latest`` (temp file + fsync + rename + directory fsync) and
prune all but the two newest steps. A crash at any point leaves ``latest`` on a
complete checkpoint — rank files of two different saves are never mixed.
Readers also accept a step directory itself and the v1 flat layout.

Restart re-decomposes: a run on P ranks can resume a checkpoint written by Q
ranks (each rank memory-maps the rank files and copies its own row range), so
jobs can move between GPU counts. Restarting is bitwise exact: the state is the
full owned field and FTCS carries no other state.
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Optional

import numpy as np

from ..ops import _native as N

FORMAT = "heat2d-checkpoint-v2"
FORMATS = (FORMAT, "heat2d-checkpoint-v1")


def step_dir(directory: str, step: int) -> str:
    return os.path.join(directory, f"step-{int(step):012d}")


def step_key(name: str):
    """(step, generation) of a step directory name "step-<12 digits>[-<digits>]"
    (generation 0: the bare name; any all-digit suffix, the legacy -N too), or
    None. Saves are ordered by this key, not by name (csrc twin: checkpoint.cpp
    step_key)."""
    if not name.startswith("step-") or len(name) < 17 or not name[5:17].isdigit():
        return None
    if len(name) == 17:
        return int(name[5:17]), 0
    if name[17] != "-" or not name[18:].isdigit():
        return None
    return int(name[5:17]), int(name[18:])


def fresh_step_dir(directory: str, step: int) -> str:
    """A step directory name no earlier save used, ordered after all of them
    (and before the next step) by step_key: the bare name first, then -000001,
    -000002, ... one past the highest generation present, legacy -N suffixes
    included (a pruned generation's number is never reused; csrc twin:
    checkpoint.cpp step_dir_name)."""
    base = step_dir(directory, step)
    try:
        entries = os.listdir(directory)
    except FileNotFoundError:
        entries = []
    keys = [k for k in map(step_key, entries) if k is not None and k[0] == int(step)]
    if not keys:
        return base
    return f"{base}-{max(g for _, g in keys) + 1:06d}"


def _fsync_dir(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _write_atomic(path: str, text: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    _fsync_dir(os.path.dirname(os.path.abspath(path)))


def save(solver, directory: str, step: Optional[int] = None, extra: Optional[dict] = None) -> None:
    """Collective: every rank writes its slab into the step's directory; rank 0
    then writes meta.json there and atomically republishes ``latest``."""
    step = int(solver.steps_done if step is None else step)
    # every rank names the same fresh directory: rank 0 picks it, the others receive it
    sd = fresh_step_dir(directory, step) if solver.rank == 0 else None
    sd = _broadcast_str(solver, sd)
    os.makedirs(sd, exist_ok=True)
    local = solver.download()
    with open(os.path.join(sd, f"rank{solver.rank:05d}.npy"), "wb") as f:
        np.save(f, local, allow_pickle=False)
        f.flush()
        os.fsync(f.fileno())
    _barrier(solver)
    if solver.rank == 0:
        p = solver.problem
        meta = {
            "format": FORMAT,
            "step": step,
            "nranks": solver.size,
            "dtype": "fp64" if local.dtype == np.float64 else "fp32",
            "n_owned": p.n_owned,
            "n_input": p.n_input,
            "convention": p.convention,
            "sigma": p.sigma, "nu": p.nu, "dom_len": p.dom_len, "r": p.r,
            "edge_shift": int(getattr(solver, "edge_shift", 0)),
        }
        meta.update(extra or {})
        _write_atomic(os.path.join(sd, "meta.json"), json.dumps(meta, indent=1))
        _write_atomic(os.path.join(directory, "latest"), os.path.basename(sd) + "\n")  # the commit point
        steps = sorted((d for d in os.listdir(directory) if step_key(d) is not None), key=step_key)
        for d in steps[:max(0, steps.index(os.path.basename(sd)) - 1)]:  # keep the two newest
            shutil.rmtree(os.path.join(directory, d), ignore_errors=True)
    _barrier(solver)


def resolve(directory: str) -> str:
    """The directory holding the newest complete checkpoint under `directory`."""
    latest = os.path.join(directory, "latest")
    if os.path.exists(latest):
        with open(latest) as f:
            return os.path.join(directory, f.read().strip())
    return directory  # a step directory itself, or the v1 flat layout


def load_meta(directory: str) -> dict:
    sd = resolve(directory)
    with open(os.path.join(sd, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") not in FORMATS:
        raise ValueError(f"{directory}: not a heat2d checkpoint")
    meta["dir"] = sd
    return meta


def load(solver, directory: str) -> dict:
    """Collective: fill the solver's owned rows from a checkpoint (any writer rank count)."""
    meta = load_meta(directory)
    if meta["n_owned"] != solver.problem.n_owned:
        raise ValueError(f"checkpoint grid {meta['n_owned']} != solver grid {solver.problem.n_owned}")
    if meta["convention"] != solver.problem.convention:
        raise ValueError("checkpoint grid convention differs")
    want = "fp64" if solver.np_dtype == np.float64 else "fp32"
    if meta["dtype"] != want:
        raise ValueError(f"checkpoint dtype {meta['dtype']} != solver dtype {want}")
    parts = [np.load(os.path.join(meta["dir"], f"rank{r:05d}.npy"), mmap_mode="r", allow_pickle=False)
             for r in range(meta["nranks"])]
    for r, part in enumerate(parts):
        # the writer's decomposition (common.hpp decompose)
        rows = N.decompose(meta["n_owned"], meta["nranks"], r, int(meta.get("edge_shift", 0)))[1]
        if part.shape != (rows, solver.ncols) or part.dtype != solver.np_dtype:
            raise ValueError(f"rank file {r}: {part.shape} {part.dtype}, expected {(rows, solver.ncols)} {want}")
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


def _broadcast_str(solver, s):
    if solver.size == 1:
        return s
    import torch.distributed as dist
    box = [s]
    dist.broadcast_object_list(box, src=0)
    return box[0]
