"""Summarise rocprofv3 outputs of tools/profile.sh into profiles/<tag>_*.{csv,json} and
profiles/traffic_<algo>_k<K>_<shape>.json (HBM bytes of ONE step, every kernel of the step)."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
tag = sys.argv[1]
PMC_STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 11  # warmup + timed + phase steps of a --pmc run
# one-off setup kernels, not in a step (torch's sort / scan / reduce: the engine's duplicate-item
# check at construction)
SETUP = ("elementwise", "rocclr", "user_sq_kernel", "fill", "mergepath", "radix_sort",
         "lookback", "scan_state", "onesweep")
SETUP_EXACT = ("compute_cuda_kernel", "reduce_kernel")
out = os.path.join(ROOT, "gpurun_out")
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
EPOCH = "mf_epoch_kernel"


def find(pattern):
    hits = sorted(glob.glob(os.path.join(out, pattern), recursive=True))
    return hits[0] if hits else None


def short(name):
    """kernel name without template arguments / parameter list"""
    n = name.split("(")[0]
    n = n.split("<")[0]
    return n.replace("void ", "").split("::")[-1].strip()


summary = {"tag": tag}
stats = find("prof_%s/**/*kernel_stats.csv" % tag)
if stats:
    shutil.copyfile(stats, os.path.join(prof, "%s_kernel_stats.csv" % tag))
    with open(stats) as f:
        rows = list(csv.DictReader(f))
    summary["kernel_stats"] = [{k: r[k] for k in r if k in ("Name", "Calls", "TotalDurationNs",
                                                           "AverageNs", "Percentage", "MinNs",
                                                           "MaxNs")} for r in rows[:16]]
bench = os.path.join(out, "prof_%s_bench.log" % tag)
if os.path.exists(bench):
    lines = [l for l in open(bench) if l.startswith("{")]
    if lines:
        summary["bench_line_under_profiler"] = json.loads(lines[-1])
        # (the stdout line is the compact one since round 5: the full dictionary is its detail file,
        # which every pass of tools/profile.sh rewrites with the same configuration)
        line = summary["bench_line_under_profiler"]
        det = line.get("detail")
        if det and os.path.exists(os.path.join(ROOT, det)):
            with open(os.path.join(ROOT, det)) as f:
                full = json.load(f)
            # (a detail file another profile's pass rewrote: keep the compact line)
            if full.get("config", {}).get("workload") == line["config"]["workload"]:
                summary["bench_line_under_profiler"] = full


def pmc(kind, counter):
    path = find("pmc_%s_%s/**/*counter_collection.csv" % (kind, tag))
    if not path:
        return None
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            vals.setdefault(short(r.get("Kernel_Name", "")), []).append(float(r["Counter_Value"]))
    return {k: {"dispatches": len(v), "mean_per_dispatch": sum(v) / len(v)} for k, v in vals.items()}


fetch = pmc("fetch", "FETCH_SIZE")
write = pmc("write", "WRITE_SIZE")
summary["FETCH_SIZE_kib"] = fetch
summary["WRITE_SIZE_kib"] = write
# HBM-side bytes, corrected as MI355X_MICROARCH.md (HBM) prescribes: FETCH_SIZE tallies 128-B read
# requests at 64 B on gfx950 -> x2; WRITE_SIZE is exact.  One step = every dispatch of the PMC run
# (PMC_STEPS epochs, nothing else) / PMC_STEPS, setup kernels listed apart.
bench_line = summary.get("bench_line_under_profiler")
if fetch and write and bench_line:
    per, setup = {}, {}
    for k in sorted(set(fetch) & set(write)):
        d = fetch[k]["dispatches"] / PMC_STEPS  # dispatches per step
        fb = 2 * fetch[k]["mean_per_dispatch"] * 1024 * d
        wb = write[k]["mean_per_dispatch"] * 1024 * d
        row = {"dispatches_per_step": d, "read_bytes": fb, "write_bytes": wb,
               "bytes_per_step": fb + wb}
        (setup if any(x in k for x in SETUP) or k in SETUP_EXACT else per)[k] = row
    total = sum(v["bytes_per_step"] for v in per.values())
    cfg = bench_line["config"]
    rl = bench_line["roofline"]
    n_up = cfg["train_ratings_rank0"]  # one epoch per step: every training rating once
    import bench
    ex = rl.get("step", {}).get("executed_bytes")
    traffic = {"bytes_per_step": total, "bytes_per_update": total / n_up,
               "algorithmic_bytes_per_update": (rl["survey_8d"]["bytes_per_update"]
                                                if "survey_8d" in rl else
                                                bench.algorithmic_bytes_per_update(
                                                    cfg["algo"], cfg["n_factors"],
                                                    bench.ELEM_BYTES[cfg.get("dtype", "f32")])),
               "executed_bytes_per_update": ex / n_up if ex else None,
               "per_kernel": per, "setup_kernels_excluded": setup,
               "source": "profiles/%s_summary.json (2 x FETCH_SIZE + WRITE_SIZE, separate --pmc "
                         "passes of %d epochs, every kernel of the step)" % (tag, PMC_STEPS),
               "workload": cfg["workload"]}
    summary["traffic"] = traffic
    dt = cfg.get("dtype", "f32")
    U_FULL = {"c4": 2_000_000, "c5": 10_000_000}
    shp = cfg.get("shape", "ml-1m")
    users = cfg.get("users_total", 0)
    key = bench.shape_key(shp, users if users and users < U_FULL.get(shp, 0) else 0)
    name = "traffic_%s_k%d_%s%s%s.json" % (cfg["algo"], cfg["n_factors"], key,
                                           "" if dt == "f32" else "_" + dt,
                                           "_qlog" if "+qlog" in cfg["workload"] else "")
    with open(os.path.join(prof, name), "w") as f:
        json.dump(traffic, f, indent=1)
hit, miss = pmc("l2", "TCC_HIT_sum"), pmc("l2", "TCC_MISS_sum")
if hit and miss:
    summary["l2_hit_rate"] = {k: hit[k]["mean_per_dispatch"] / max(1.0, hit[k]["mean_per_dispatch"] +
                                                                    miss[k]["mean_per_dispatch"])
                              for k in sorted(set(hit) & set(miss))}
with open(os.path.join(prof, "%s_summary.json" % tag), "w") as f:
    json.dump(summary, f, indent=1)
print(json.dumps(summary, indent=1)[:4000])
