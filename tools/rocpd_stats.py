#!/usr/bin/env python3
"""Per-kernel summary (calls, average / total microseconds, grid) of a rocprofv3
SQLite result (`run_results.db`, the default output format on this image).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top 40]
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"^_ZN9srpc_impl12_GLOBAL__N_1\d+", "", name)
    return name[:100]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), avg(duration)/1000.0, sum(duration)/1000.0, max(grid_x) "
                     "from kernels group by name order by 4 desc").fetchall()
    print(f"{'calls':>6} {'avg_us':>10} {'total_us':>12} {'grid_x':>10}  kernel")
    for name, n, avg, tot, gx in rows[:a.top]:
        print(f"{n:6d} {avg:10.2f} {tot:12.1f} {gx:10d}  {short(name)}")


if __name__ == "__main__":
    main()
