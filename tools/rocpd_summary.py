"""Summarise kernel dispatches of a rocprofv3 rocpd SQLite database (kernel-trace) as CSV:
name, calls, total_ns, avg_ns, min_ns, max_ns, pct. Usage: python tools/rocpd_summary.py run_results.db"""
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                       "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print("name,calls,total_ns,avg_ns,min_ns,max_ns,pct")
    for n, c, t, a, mi, ma in rows:
        print(f"\"{n}\",{c},{t},{a:.0f},{mi},{ma},{100.0 * t / total:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
