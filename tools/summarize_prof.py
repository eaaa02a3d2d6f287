"""Summarize a tools/profile_round.sh output directory into profiles/.

  python tools/summarize_prof.py gpurun_out/<tag> <profile-name> <kernel> --units N --unit NAME

Writes profiles/<profile-name>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary,
verbatim) and profiles/<profile-name>_pmc.json (per-launch counters of `kernel`), and
merges the kernel's HBM bytes and VALU instructions into profiles/traffic_latest.json
("kernels": {name: ...}), which bench.py reads.

Counters are stored PER UNIT of work -- a playout (k_rollout*), a board-player
(k_movegen*), a simulation (k_mcts*: iterations x searches in the launch) -- together
with the units one profiled launch processed, so a bench line whose launches hold a
different amount of work (config 5's --chunk, config 4's per-round searches) scales them
by its own units per launch instead of pairing another launch size's counts with its
time.  HBM bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE (KB) doubled on
gfx950, WRITE_SIZE (KB) as is.
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel, keep_first):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].split("(")[0] == kernel:
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    by = collections.defaultdict(list)
    for (_d, c), v in sorted(agg.items(), key=lambda kv: int(kv[0][0])):
        by[c].append(v)
    # drop the warm-up launch (first dispatch of the kernel) unless the profiled run had
    # no warm-up step of the same size (--keep-first: e.g. config 5's chunked launches)
    k = 0 if keep_first else 1
    return {c: sum(v[k:]) / len(v[k:]) if len(v) > k else v[0] for c, v in by.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("name")
    ap.add_argument("kernel")
    ap.add_argument("--units", type=float, required=True, help="units of work per profiled launch")
    ap.add_argument("--unit", required=True, help="playout | board-player | simulation")
    ap.add_argument("--keep-first", action="store_true")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(os.path.dirname(os.path.join(prof, a.name)), exist_ok=True)
    shutil.copy(os.path.join(a.src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{a.name}_kernel_stats.csv"))
    pmc = {}
    for d in sorted(os.listdir(a.src)):
        f = os.path.join(a.src, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(f):
            pmc.update(per_launch(f, a.kernel, a.keep_first))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(os.path.join(a.src, "trace", "run_kernel_trace.csv")))
            if r["Kernel_Name"].split("(")[0] == a.kernel]
    k = 0 if a.keep_first else 1
    pmc["trace_avg_ms"] = sum(durs[k:]) / max(len(durs) - k, 1) / 1e6
    pmc["units_per_launch"], pmc["unit"] = a.units, a.unit
    json.dump(pmc, open(os.path.join(prof, f"{a.name}_pmc.json"), "w"), indent=1, sort_keys=True)
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        b = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0
        v = pmc.get("SQ_INSTS_VALU")
        t = {"kernel": a.kernel, "source": f"profiles/{a.name}_pmc.json",
             "stats": f"profiles/{a.name}_kernel_stats.csv", "unit": a.unit, "units_per_launch": a.units,
             "bytes_per_launch": b, "valu_insts_per_launch": v, "bytes_per_unit": b / a.units,
             "valu_insts_per_unit": v / a.units if v is not None else None, "trace_avg_ms": pmc["trace_avg_ms"]}
        path = os.path.join(prof, "traffic_latest.json")
        try:
            cur = json.load(open(path))
        except (OSError, ValueError):
            cur = {}
        kernels = cur.get("kernels", {})
        kernels[a.kernel] = t
        json.dump({"note": "per-unit PMC HBM bytes and VALU instructions per kernel (tools/summarize_prof.py); "
                           "bench.py scales them by its own launch's units", "kernels": kernels},
                  open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(pmc, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
