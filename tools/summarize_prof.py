"""Summarise rocprofv3 outputs of tools/profile.sh into profiles/<tag>_*.{csv,json}."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
out = os.path.join(ROOT, "gpurun_out")
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)


def find(pattern):
    hits = sorted(glob.glob(os.path.join(out, pattern), recursive=True))
    return hits[0] if hits else None


summary = {"tag": tag}
stats = find("prof_%s/**/*kernel_stats.csv" % tag)
if stats:
    shutil.copyfile(stats, os.path.join(prof, "%s_kernel_stats.csv" % tag))
    with open(stats) as f:
        rows = list(csv.DictReader(f))
    summary["kernel_stats"] = [{k: r[k] for k in r if k in ("Name", "Calls", "TotalDurationNs",
                                                           "AverageNs", "Percentage", "MinNs",
                                                           "MaxNs")} for r in rows[:12]]
bench = os.path.join(out, "prof_%s_bench.log" % tag)
if os.path.exists(bench):
    lines = [l for l in open(bench) if l.startswith("{")]
    if lines:
        summary["bench_line_under_profiler"] = json.loads(lines[-1])


def pmc(kind, counter):
    path = find("pmc_%s_%s/**/*counter_collection.csv" % (kind, tag))
    if not path:
        return None
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: {"dispatches": len(v), "mean_per_dispatch": sum(v) / len(v)} for k, v in vals.items()}


fetch = pmc("fetch", "FETCH_SIZE")
write = pmc("write", "WRITE_SIZE")
summary["FETCH_SIZE_kib"] = fetch
summary["WRITE_SIZE_kib"] = write
# HBM-side bytes per epoch-kernel launch, corrected as MI355X_MICROARCH.md (HBM) prescribes:
# FETCH_SIZE tallies 128-B read requests at 64 B on gfx950 -> x2; WRITE_SIZE is exact.
# Calibrated on our own access pattern: log_reduce_kernel reads a known 404 B/rating from
# 448-B-strided rows (4 x 128-B lines each), and 2 x FETCH_SIZE matches that line count.
bench_line = summary.get("bench_line_under_profiler")
if fetch and write and bench_line and "mf_epoch_kernel" in fetch and "mf_epoch_kernel" in write:
    fb = 2 * fetch["mf_epoch_kernel"]["mean_per_dispatch"] * 1024
    wb = write["mf_epoch_kernel"]["mean_per_dispatch"] * 1024
    cfg = bench_line["config"]
    n_up = bench_line["roofline"]["updates_per_launch"]
    traffic = {"kernel": "mf_epoch_kernel", "bytes_per_launch": fb + wb, "read_bytes": fb,
               "write_bytes": wb, "bytes_per_update": (fb + wb) / n_up,
               "algorithmic_bytes_per_update": bench_line["roofline"]["algorithmic_bytes_per_update"],
               "source": "profiles/%s_summary.json (2 x FETCH_SIZE + WRITE_SIZE, separate passes)" % tag,
               "workload": cfg["workload"]}
    summary["traffic"] = traffic
    with open(os.path.join(prof, "traffic_%s_k%d.json" % (cfg["algo"], cfg["n_factors"])), "w") as f:
        json.dump(traffic, f, indent=1)
with open(os.path.join(prof, "%s_summary.json" % tag), "w") as f:
    json.dump(summary, f, indent=1)
print(json.dumps(summary, indent=1)[:4000])
