"""Kernel statistics of a rocprofv3 run written in its default rocpd (SQLite) format, as the CSV
`--stats --output-format csv` writes (Name, Calls, TotalDurationNs, AverageNs, Percentage).
Usage: python3 tools/rocpd_stats.py RUN_results.db OUT.csv"""
import csv
import sqlite3
import sys


def main(db, out):
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels order by total_duration desc").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, calls, tot_us, avg_us, pct in rows:  # (rocpd's view is in microseconds)
            short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            w.writerow([short, calls, round(tot_us * 1e3), round(avg_us * 1e3, 3), pct])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
