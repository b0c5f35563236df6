"""Per-kernel summary (calls, average and total ms) of a rocprofv3 --kernel-trace
results database, for runs written without the CSV stats files.

    python tools/prof_summary.py gpurun_out/prof/x_results.db [limit]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(end - start) / 1e6, sum(end - start) / 1e6 "
                     "from kernels group by name order by 4 desc limit ?", (limit,)).fetchall()
    print(f"{'kernel':70s} {'calls':>6s} {'avg_ms':>9s} {'total_ms':>9s}")
    for name, cnt, avg, tot in rows:
        print(f"{name[:70]:70s} {cnt:6d} {avg:9.3f} {tot:9.3f}")


if __name__ == "__main__":
    main()
