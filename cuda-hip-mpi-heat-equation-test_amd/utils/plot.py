"""Visualisation of ``int.dat`` / ``soln.dat`` — the reference's ``make init`` /
``make out`` scripts (fortran/serial/init.py, out.py; fortran/mpi+cuda/out.py,
which saves ``sol.eps``), rebuilt:

    python -m heat2d.utils.plot init            # int.dat   -> surface plot
    python -m heat2d.utils.plot out             # soln.dat (or merged soln%05d.dat)
    python -m heat2d.utils.plot FILE --save sol.eps
    python -m heat2d.utils.plot out --heatmap --save soln.png   # large grids

Differences from the reference scripts: ``fig.gca(projection='3d')`` (removed in
matplotlib >= 3.6) is replaced by ``add_subplot(projection='3d')``; per-rank
files are merged automatically; the grid need not be square; big grids are
decimated to at most --max-points per axis for the surface.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

from .io import merge_rank_files, rank_files, read_xyz


def resolve(what: str, directory: str = ".") -> str:
    if what == "init":
        return os.path.join(directory, "int.dat")
    if what == "out":
        path = os.path.join(directory, "soln.dat")
        if not os.path.exists(path) and rank_files(directory):
            path = merge_rank_files(directory)
        return path
    return what


def plot(path: str, save: str | None = None, heatmap: bool = False, max_points: int = 256,
         zlim=(1.0, 2.5), xlim=(0.0, 2.0), ylim=(0.0, 2.0)):
    import matplotlib
    if save or not os.environ.get("DISPLAY"):
        matplotlib.use("Agg")
    from matplotlib import cm, pyplot

    x, y, T = read_xyz(path)
    sx = max(1, len(x) // max_points)
    sy = max(1, len(y) // max_points)
    x, y, T = x[::sx], y[::sy], T[::sx, ::sy]
    fig = pyplot.figure()
    if heatmap:
        ax = fig.add_subplot()
        im = ax.imshow(T.T, origin="lower", extent=(x[0], x[-1], y[0], y[-1]), cmap=cm.viridis)
        fig.colorbar(im, ax=ax, label="T")
    else:
        ax = fig.add_subplot(projection="3d")
        X, Y = np.meshgrid(x, y, indexing="ij")
        ax.plot_surface(X, Y, T, rstride=1, cstride=1, cmap=cm.viridis, linewidth=0, antialiased=False)
        ax.set_xlim(*xlim)
        ax.set_ylim(*ylim)
        ax.set_zlim(*zlim)
    ax.set_xlabel("$x$")
    ax.set_ylabel("$y$")
    if save:
        fig.savefig(save)
    elif os.environ.get("DISPLAY"):
        pyplot.show()
    return fig


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m heat2d.utils.plot")
    ap.add_argument("what", help="init | out | path to an x y T file")
    ap.add_argument("--dir", default=".")
    ap.add_argument("--save", default=None, help="output image (e.g. sol.eps, soln.png)")
    ap.add_argument("--heatmap", action="store_true")
    ap.add_argument("--max-points", type=int, default=256)
    a = ap.parse_args(argv)
    path = resolve(a.what, a.dir)
    save = a.save
    if save is None and not os.environ.get("DISPLAY"):
        save = os.path.splitext(os.path.basename(path))[0] + (".png" if a.heatmap else ".eps")
    plot(path, save=save, heatmap=a.heatmap, max_points=a.max_points)
    if save:
        print(f"wrote {save}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
