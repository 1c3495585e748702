"""Worker for tests/test_select.py: one gloo rank running the collective
transport selection (parallel/select.py) with fake candidates.

`python tests/select_worker.py RANK WORLD PORT OUTDIR SCENARIO` writes
OUTDIR/rank<R>.json = {"chosen": ..., "report": ..., "verify": ...}.
Scenarios:
  fail_rccl_on_1   rank 1's "rccl" build raises; "ipc" works everywhere
  slow_rank        every candidate works; "rccl" is fast on rank 0 but slow on rank 1
  verify           verify_decomposition over the CPU twin + gloo (bitwise)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, outdir, scenario = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                                           sys.argv[5])
    import torch
    import torch.distributed as dist
    from datetime import timedelta
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=timedelta(seconds=120))
    import heat2d  # noqa: F401
    from heat2d.parallel import select

    def reduce(v, op):
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())

    amin = lambda v: reduce(v, dist.ReduceOp.MIN)  # noqa: E731
    amax = lambda v: reduce(v, dist.ReduceOp.MAX)  # noqa: E731
    out = {}
    if scenario == "fail_rccl_on_1":
        built = []

        def trial(kind):
            def make():
                if kind == "rccl" and rank == 1:
                    raise RuntimeError("ncclCommInitRank: invalid usage (duplicate GPU)")
                built.append(kind)
                return kind
            obj, why = select.try_collective(make, amin, cleanup=lambda k: built.append("cleanup-" + k))
            if why is not None:
                raise select.Skip(why)
            return {"rccl": 1.0, "ipc": 2.0}[kind]

        out["chosen"], out["report"] = select.choose_transport(["rccl", "ipc"], trial, amin, amax)
        out["built"] = built
    elif scenario == "slow_rank":
        def trial(kind):
            return {"rccl": 1.0 if rank == 0 else 5.0, "ipc": 3.0}[kind]
        out["chosen"], out["report"] = select.choose_transport(["rccl", "ipc"], trial, amin, amax)
    elif scenario == "verify":
        from heat2d.parallel.transport import TorchDistTransport
        out["verify"] = select.verify_decomposition(TorchDistTransport, rank=rank, world=world, dtype="fp64",
                                                    arith="jacobi", backend="cpu", n=3 * 37 + 2, steps=29)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
