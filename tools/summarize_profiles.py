"""Summarise a tools/collect_profiles.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/.

Writes kernel_stats.csv (rocprofv3 --stats, unchanged), kernel_trace_search.csv
(search-kernel rows of the trace), bench_under_trace.json (the traced bench's own
JSON line) and pmc_search.json (PMC values of the search
kernel per launch, HBM bytes with the MI355X_MICROARCH.md gfx950 correction),
and refreshes profiles/pmc_search.json, which bench.py reads for roofline.traffic.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag="r01", roots=None, iterations=None):
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    with open(os.path.join(src, "trace", "run_kernel_trace.csv")) as fh:
        rows = [r for r in csv.DictReader(fh) if "search_kernel" in r["Kernel_Name"]]
    # the dominant launch shape only: (kernel, grid) with the largest total time -- a step's
    # fallback pass (small grid, drains at once) and the small-batch leg are other shapes
    tot = {}
    for r in rows:
        key = (r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size")))
        tot[key] = tot.get(key, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    dom = None
    if tot:
        dom = max(tot, key=tot.get)
        rows = [r for r in rows if (r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size"))) == dom]
    with open(os.path.join(dst, "kernel_trace_search.csv"), "w", newline="") as fh:
        keep = ["Kernel_Name", "Grid_Size_X", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                "SGPR_Count", "Start_Timestamp", "End_Timestamp"]
        w = csv.DictWriter(fh, fieldnames=keep + ["Duration_ns"])
        w.writeheader()
        for r in rows:
            d = {k: r.get(k, "") for k in keep}
            d["Duration_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            w.writerow(d)
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    # the bench line printed by the traced run itself: its HIP-event search time is the
    # one the trace durations must agree with (box-to-box clocks differ by several %)
    traced_bench = None
    with open(os.path.join(src, "trace.log")) as fh:
        for line in fh:
            if line.startswith("{"):
                traced_bench = json.loads(line)
    if traced_bench is not None:
        with open(os.path.join(dst, "bench_under_trace.json"), "w") as fh:
            json.dump(traced_bench, fh, indent=1)
    # the launch size the PMC passes ran (bench.py defaults: the traced run's config)
    if roots is None:
        roots = traced_bench["config"]["roots_per_gpu"] if traced_bench else None
    if iterations is None:
        iterations = traced_bench["config"]["iterations"] if traced_bench else None
    pmc = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "p_counter_collection.csv"))):
        per = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "search_kernel" not in r["Kernel_Name"]:
                    continue
                # the trace's dominant launch shape only (the small-batch leg and the fallback
                # pass are other kernels / grids)
                if dom is not None and (r["Kernel_Name"], r.get("Grid_Size")) != dom:
                    continue
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        # main launches only (the fallback pass of a step drains at once: tiny counter totals)
        wt = {}
        for (disp, name), v in per.items():
            wt[disp] = wt.get(disp, 0.0) + v
        top = max(wt.values()) if wt else 0.0
        for (disp, name), v in per.items():
            if wt[disp] >= 0.05 * top:
                pmc.setdefault(name, []).append(v)
    vals = {k: sum(v) / len(v) for k, v in pmc.items()}
    fetch_kb = vals.get("FETCH_SIZE")
    write_kb = vals.get("WRITE_SIZE")
    out = {
        "kernel": "search_kernel<dk::FdoE>",
        "roots": roots,
        "iterations": iterations,
        "trace_avg_ns": sum(durs) / len(durs) if durs else None,
        "trace_launches": len(durs),
        "bench_search_kernel_ms_same_run": traced_bench.get("search_kernel_ms") if traced_bench else None,
        "pmc_per_launch": vals,
        "fetch_bytes_raw": fetch_kb * 1024 if fetch_kb is not None else None,
        "write_bytes": write_kb * 1024 if write_kb is not None else None,
        "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half the bytes of wide reads; "
                      "uncalibrated for this 16-B-per-lane random pattern, so this is an upper reading)",
    }
    if fetch_kb is not None and write_kb is not None:
        out["hbm_bytes_per_launch"] = 2 * fetch_kb * 1024 + write_kb * 1024
    with open(os.path.join(dst, "pmc_search.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    shutil.copy(os.path.join(dst, "pmc_search.json"), os.path.join(ROOT, "profiles", "pmc_search.json"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["r01"]))
