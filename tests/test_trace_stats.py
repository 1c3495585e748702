"""tools/trace_stats.py on a synthetic rocprofv3 SQLite database (the two views
it reads, `top_kernels` and `kernels`, with the columns ROCm 7 writes)."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TB = "void heat2d::kern::tbimpl::tb_kernel<double, 1, 20, 6, true, 2, 0>(double const*, double*, TbArgs, double)"
JIT = "heat2d_jit_step(double const*, double*)"


def make_db(path):
    con = sqlite3.connect(path)
    con.execute("create table top_kernels (name text, total_calls int, total_duration real, average real, "
                "percentage real)")
    con.execute("create table kernels (name text, start int, end int, grid_x int, workgroup_x int)")
    con.execute("insert into top_kernels values (?, 3, 12000.0, 4000.0, 97.5)", (TB,))
    con.execute("insert into top_kernels values (?, 1, 300.0, 300.0, 2.5)", (JIT,))
    rows = [(TB, 0, 4_000_000), (TB, 4_010_000, 8_010_000), (TB, 8_020_000, 12_020_000), (JIT, 12_030_000, 12_330_000)]
    for name, s, e in rows:
        con.execute("insert into kernels values (?, ?, ?, ?, 256)", (name, s, e, 2048 * 64))
    con.commit()
    con.close()


def test_trace_stats_tables(tmp_path):
    db = tmp_path / "t_results.db"
    make_db(str(db))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_stats.py"), str(db), "--last", "tb_kernel",
                        "2", "--before", "jit"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    out = p.stdout.splitlines()
    top = [l for l in out if l.startswith("tb_kernel<double, 1, 20, 6, true, 2, 0>")]
    # totals in ms and averages in us (the views hold microseconds)
    assert top and "12.000" in top[0] and "4000.00" in top[0]
    last = out[out.index(next(l for l in out if l.startswith("last 2 dispatches"))) + 2:]
    assert len(last) == 2
    # the last two tb dispatches before the first JIT kernel (the 2nd and 3rd), starts relative to
    # the first of them: 0 and 4010 us, 4000 us each, a 10 us gap, 2048 waves
    assert last[0].split()[-3:] == ["0.00", "4000.00", "2048"]
    assert last[1].split()[-4:] == ["4010.00", "4000.00", "10.00", "2048"]
