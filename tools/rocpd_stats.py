#!/usr/bin/env python3
"""Per-kernel summary (calls, average / total microseconds, grid) of a rocprofv3
SQLite result (`run_results.db`, the default output format on this image).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--top 40]
    python tools/rocpd_stats.py DB --split k_sx_spec   # per call, calls told apart
                                                        # by that kernel's grid
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
    ap.add_argument("--split", default=None,
                    help="a kernel name pattern: each of its launches starts a call, labelled by its grid")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    if a.split:
        by = {}
        label = None
        for name, dur, gx in c.execute("select name, duration, grid_x from kernels order by start"):
            if re.search(a.split, name):
                label = gx
            if label is None:
                continue
            by.setdefault((label, short(name)), []).append(dur / 1000.0)
        print(f"{'grid':>10} {'calls':>6} {'avg_us':>10} {'max_us':>10}  kernel")
        for (gx, name), v in sorted(by.items(), key=lambda kv: (kv[0][0], -max(kv[1]))):
            print(f"{gx:10d} {len(v):6d} {sum(v) / len(v):10.2f} {max(v):10.2f}  {name}")
        return
    rows = c.execute("select name, count(*), avg(duration)/1000.0, sum(duration)/1000.0, max(grid_x) "
                     "from kernels group by name order by 4 desc").fetchall()
    print(f"{'calls':>6} {'avg_us':>10} {'total_us':>12} {'grid_x':>10}  kernel")
    for name, n, avg, tot, gx in rows[:a.top]:
        print(f"{n:6d} {avg:10.2f} {tot:12.1f} {gx:10d}  {short(name)}")


if __name__ == "__main__":
    main()
