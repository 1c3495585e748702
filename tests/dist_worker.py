"""Worker for multi-process tests: one rank of a distributed heat2d run over
torch.distributed (gloo) with the native solver + TorchDistTransport.

Launched as `python tests/dist_worker.py RANK WORLD PORT OUTDIR JSON_ARGS`.
Rank 0 gathers the field and writes OUTDIR/result.npy.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def random_field(prob, dtype):
    """Frame-inclusive field: the problem's frame, seeded uniform noise inside."""
    import numpy as np
    from heat2d.models import reference as R
    dt = np.float64 if dtype == "fp64" else np.float32
    T0 = R.initial_field(prob, dt)
    T0[1:-1, 1:-1] = np.random.default_rng(1234).random(T0[1:-1, 1:-1].shape).astype(dt)
    return T0


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    args = json.loads(sys.argv[5])
    import numpy as np
    import torch
    import torch.distributed as dist

    import heat2d
    from heat2d.models.heat2d import HeatSolver
    from heat2d.parallel.transport import IpcTransport, TorchDistTransport

    from datetime import timedelta
    timeout = float(os.environ.get("HEAT2D_COMM_TIMEOUT", "600"))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=timedelta(seconds=timeout))
    inp = heat2d.InputDat(n=args["n"], sigma=0.25, nu=0.05, dom_len=args.get("dom", 1.0), ntime=args["steps"])
    prob = heat2d.make_problem(inp, args.get("conv", "ghost"), args.get("ic", "uniform"))
    backend = args.get("backend", "cpu")
    if backend == "hip":
        torch.cuda.set_device(0)
    # ipc: process-per-GPU transport (all ranks on GPU 0), host collectives over this gloo group
    tr = IpcTransport(0) if args.get("transport") == "ipc" else TorchDistTransport()
    tb = args.get("tb_rank", {}).get(str(rank), args.get("tb", 8))  # per-rank override: a deliberate mismatch
    s = HeatSolver(prob, dtype=args.get("dtype", "fp64"), backend=backend, tb=tb,
                   overlap=args.get("overlap", True), transport=tr, device=0 if backend == "hip" else None,
                   graph=args.get("graph", False))
    if args.get("random"):  # non-trivial data everywhere: a stale halo cannot hide
        from heat2d.models import reference as R
        T0 = random_field(prob, args.get("dtype", "fp64"))
        lay = s.layout
        s.upload(R.owned(T0)[lay.row0:lay.row0 + lay.nrows])
    # split the stepping to exercise restarts of the cycle schedule
    first = args["steps"] // 3
    if args.get("prepare"):  # collective: the ranks agree on step(first)'s cycles / exchange depths
        try:
            s.prepare(first)
        except Exception as e:  # noqa: BLE001 - the test inspects the message
            with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
                f.write(str(e))
            s.close()
            dist.barrier()
            dist.destroy_process_group()
            return
    s.halo_rows_exchanged(reset=True)
    seqs = [s.step_cycles(first)]
    s.step(first)
    if args.get("die_rank") == rank:  # failure injection: this rank dies mid-run (tests/test_watchdog.py)
        s.step(args.get("die_after", 0))
        sys.stdout.flush()
        os._exit(3)
    # the rest with the global statistics + one-step residual of the final field
    seqs.append(s.step_cycles(args["steps"] - first))
    ghost_before = s.ghost_rows
    if args.get("plain_step"):  # step() itself (step_stats on the CPU twin runs n-1 + 1 steps)
        s.step(args["steps"] - first)
        st = s.stats()
    else:
        st = s.step_stats(args["steps"] - first)
    halo = s.halo_rows_exchanged()
    full = s.gather()
    if rank == 0:
        np.save(os.path.join(outdir, "result.npy"), full)
        with open(os.path.join(outdir, "stats.json"), "w") as f:
            json.dump({"stats": st, "info": {k: v for k, v in s.info().items() if k != "layout"}, "seqs": seqs,
                       "halo_rows": halo, "ghost_before": ghost_before, "ghost_after": s.ghost_rows}, f)
    s.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
