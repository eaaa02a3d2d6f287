"""Summarize a tools/profile_round.sh output directory into profiles/.

  python tools/summarize_prof.py gpurun_out/<tag> <round-tag> [kernel]

Writes profiles/<round-tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats
summary, verbatim), profiles/<round-tag>_pmc.json (per-launch counters of `kernel`,
default k_rollout) and merges HBM bytes + VALU instructions per launch of that kernel
into profiles/traffic_latest.json ("kernels": {name: ...}), which bench.py reads.
HBM bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE (KB) doubled on gfx950,
WRITE_SIZE (KB) as is.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_rollout"


def per_launch(path, kernel):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].split("(")[0] == kernel:
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    by = collections.defaultdict(list)
    for (_d, c), v in sorted(agg.items(), key=lambda kv: int(kv[0][0])):
        by[c].append(v)
    # drop the warm-up launch (first dispatch of the kernel) unless the profiled run had
    # no warm-up step (KEEP_FIRST=1: e.g. config5, whose 8 launches are one search)
    k = 0 if os.environ.get("KEEP_FIRST") == "1" else 1
    return {c: sum(v[k:]) / len(v[k:]) if len(v) > k else v[0] for c, v in by.items()}


def main(src, tag, kernel=KERNEL):
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    pmc = {}
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(f):
            pmc.update(per_launch(f, kernel))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
            if r["Kernel_Name"].split("(")[0] == kernel]
    pmc["trace_avg_ms_excl_first"] = sum(durs[1:]) / max(len(durs) - 1, 1) / 1e6
    json.dump(pmc, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        t = {"kernel": kernel, "source": f"profiles/{tag}_pmc.json",
             "fetch_kb": pmc["FETCH_SIZE"], "write_kb": pmc["WRITE_SIZE"],
             "bytes_per_launch": (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0,
             "valu_insts_per_launch": pmc.get("SQ_INSTS_VALU")}
        path = os.path.join(prof, "traffic_latest.json")
        try:
            cur = json.load(open(path))
        except (OSError, ValueError):
            cur = {}
        kernels = cur.get("kernels", {})
        if "kernel" in cur and cur["kernel"] not in kernels:  # round-1 single-kernel layout
            kernels[cur["kernel"]] = {k: v for k, v in cur.items() if k != "kernels"}
        kernels[kernel] = t
        out = dict(kernels.get("k_rollout", t))
        out["kernels"] = kernels
        json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(pmc, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:4])
