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


def totals(path, kernel):
    """Counters summed over every launch of `kernel` in one PMC run, plus the launch count."""
    agg = collections.defaultdict(float)
    ids = set()
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].split("(")[0] == kernel:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            ids.add(r["Dispatch_Id"])
    return agg, len(ids)


def wave_concurrency(pmc_dir, kernel):
    """Time-weighted waves of `kernel` resident while any of its launches runs (launches on
    several streams overlap): sum(SQ_WAVES x duration) / time covered by >= 1 launch."""
    waves = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(pmc_dir, "run_counter_collection.csv"))):
        if r["Kernel_Name"].split("(")[0] == kernel and r["Counter_Name"] == "SQ_WAVES":
            waves[r["Dispatch_Id"]] += float(r["Counter_Value"])
    tr = {r["Dispatch_Id"]: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in csv.DictReader(open(os.path.join(pmc_dir, "run_kernel_trace.csv")))
          if r["Kernel_Name"].split("(")[0] == kernel}
    ids = [i for i in waves if i in tr]
    if not ids:
        return None
    ev = sorted([(tr[i][0], 1) for i in ids] + [(tr[i][1], -1) for i in ids])
    cov, c, last = 0, 0, 0
    for t, d in ev:
        if c > 0:
            cov += t - last
        c += d
        last = t
    busy = sum(waves[i] * (tr[i][1] - tr[i][0]) for i in ids)
    return {"launches": len(ids), "waves_per_launch_mean": sum(waves[i] for i in ids) / len(ids),
            "waves_per_launch_max": max(waves[i] for i in ids), "covered_ms": cov / 1e6,
            "mean_concurrent_waves": busy / cov if cov else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("name")
    ap.add_argument("kernel")
    ap.add_argument("--units", type=float, default=None, help="units of work per profiled launch")
    ap.add_argument("--total-units", type=float, default=None,
                    help="units of work over ALL launches of the kernel in one run (launch sizes vary, e.g. "
                         "config 4's pipelined searches): counters are summed over every launch of each PMC "
                         "run and divided by this")
    ap.add_argument("--unit", required=True, help="playout | board-player | simulation")
    ap.add_argument("--keep-first", action="store_true")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(os.path.dirname(os.path.join(prof, a.name)), exist_ok=True)
    shutil.copy(os.path.join(a.src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{a.name}_kernel_stats.csv"))
    if (a.units is None) == (a.total_units is None):
        raise SystemExit("give exactly one of --units / --total-units")
    pmc = {}
    for d in sorted(os.listdir(a.src)):
        f = os.path.join(a.src, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(f):
            if a.total_units is None:
                pmc.update(per_launch(f, a.kernel, a.keep_first))
            else:  # per unit first, scaled to the trace run's mean launch below
                agg, _n = totals(f, a.kernel)
                pmc.update({c: v / a.total_units for c, v in agg.items()})
                conc = wave_concurrency(os.path.join(a.src, d), a.kernel)
                if conc:
                    pmc["wave_concurrency"] = conc
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for r in csv.DictReader(open(os.path.join(a.src, "trace", "run_kernel_trace.csv")))
            if r["Kernel_Name"].split("(")[0] == a.kernel]
    k = 0 if a.keep_first or a.total_units is not None else 1
    pmc["trace_avg_ms"] = sum(durs[k:]) / max(len(durs) - k, 1) / 1e6
    if a.total_units is not None:
        a.units = a.total_units / len(durs)  # the trace run's mean launch
        for c in list(pmc):
            if c.isupper():
                pmc[c] *= a.units
        pmc["total_units"], pmc["trace_launches"] = a.total_units, len(durs)
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
