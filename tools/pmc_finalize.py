"""Turn tools/pmc_passes.sh output into the committed PMC summaries.

  calib:  python tools/pmc_finalize.py calib <pmc_dir> <calib.jsonl>        -> profiles/r03/pmc_calib.json
  search: python tools/pmc_finalize.py search <pmc_dir> <kernel> <roots> <iterations> <out.json> [calib.json] [main|max]

Calibration (tools/pmc_calib.hip, known work per launch) fixes how the gfx950 counters read:
  * DRAM read bytes = 32 x TCC_EA0_RDREQ_32B + 64 x TCC_EA0_RDREQ_64B + 128 x TCC_EA0_RDREQ_128B
    (FETCH_SIZE = 64 x TCC_EA0_RDREQ: half the bytes of 128-B requests, which is what a
    random 8-B or 16-B load costs: a whole 128-B line);
  * DRAM write bytes = WRITE_SIZE (32-B and 64-B write requests read exactly: a random 8-B
    store moves 32 B, a 64-B record store 64 B);
  * a wave64 integer VALU instruction holds its SIMD 4 cycles at 1, 2, 3 and 8 waves per
    SIMD (SQ_INSTS_VALU x 4 / SIMD cycles = 0.93-0.99 on a saturated pipe), so VALU busy =
    SQ_INSTS_VALU x 4 / (SIMDs x GRBM_GUI_ACTIVE / XCDs).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_report import collect  # noqa: E402

SIMDS, XCDS = 1024, 8


def dram_read(c):
    return 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) + \
        128 * c.get("TCC_EA0_RDREQ_128B_sum", 0)


def derived(c, ms=None):
    cyc = c["GRBM_GUI_ACTIVE"] / XCDS
    d = {
        "dram_read_bytes": dram_read(c),
        "dram_write_bytes": c["WRITE_SIZE"] * 1024.0,
        "fetch_size_bytes": c["FETCH_SIZE"] * 1024.0,
        "read_requests_128B_frac": c.get("TCC_EA0_RDREQ_128B_sum", 0) / max(1.0, c.get("TCC_EA0_RDREQ_sum", 0)),
        "valu_busy": c["SQ_INSTS_VALU"] * 4.0 / SIMDS / cyc,
        "valu_cycles_per_inst_per_simd": cyc * SIMDS / max(1.0, c["SQ_INSTS_VALU"]),
        "valu_dual_issue_frac": c.get("SQ_ACTIVE_INST_VALU2", 0) / max(1.0, c.get("SQ_ACTIVE_INST_VALU", 1)),
        "mem_wait_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
        "issue_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"],
        "l2_hit": c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
        "shader_clock_ghz_counter": None,
    }
    d["dram_bytes"] = d["dram_read_bytes"] + d["dram_write_bytes"]
    if ms:
        d["shader_clock_ghz_counter"] = cyc / (ms * 1e-3) / 1e9
        d["dram_gbs"] = d["dram_bytes"] / (ms * 1e-3) / 1e9
    return d


def calib(pmc_dir, jsonl):
    runs = [json.loads(l) for l in open(jsonl) if l.startswith("{")]
    pmc = collect(pmc_dir, [r["kernel"] for r in runs], "last")
    out = {"source": "tools/pmc_calib.hip (16 GiB buffer, 1 M lanes x 64 accesses; VALU: 8 integer chains per wave)",
           "tests": {}}
    for r in runs:
        c = pmc[r["kernel"]]
        d = derived(c, r["ms"])
        e = dict(r)
        e.update({k: d[k] for k in ("dram_read_bytes", "dram_write_bytes", "fetch_size_bytes", "read_requests_128B_frac",
                                    "valu_busy", "valu_cycles_per_inst_per_simd", "valu_dual_issue_frac", "dram_gbs")})
        if r.get("alg_bytes"):
            e["dram_bytes_per_access"] = d["dram_bytes"] / r["accesses"] if r.get("accesses") else None
            e["dram_over_alg"] = d["dram_bytes"] / r["alg_bytes"]
            e["fetch_size_over_alg"] = d["fetch_size_bytes"] / r["alg_bytes"]
        e["counters"] = {k: v for k, v in c.items() if not k.startswith("_")}
        out["tests"][r["test"]] = e
    return out


def search(pmc_dir, kernel, roots, iters, calib_path=None, mode="main"):
    c = collect(pmc_dir, [kernel], mode)[kernel]
    trace_ns = []
    import csv
    import glob
    for f in glob.glob(os.path.join(pmc_dir, "p*", "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel in r["Kernel_Name"]:
                    trace_ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if mode == "max":
        main = [t for t in trace_ns if t >= 0.95 * max(trace_ns)] if trace_ns else []
    else:
        main = [t for t in trace_ns if t >= 0.05 * max(trace_ns)] if trace_ns else []
    ms = sum(main) / len(main) / 1e6 if main else None
    d = derived(c, ms)
    sims = roots * iters
    out = {"kernel": kernel, "roots": roots, "iterations": iters, "pmc_trace_avg_ms": ms,
           "pmc_per_launch": {k: v for k, v in c.items() if not k.startswith("_")},
           "derived": d,
           "dram_bytes_per_sim": d["dram_bytes"] / sims,
           "dram_read_lines_per_sim": c.get("TCC_EA0_RDREQ_128B_sum", 0) / sims,
           "dram_write_requests_per_sim": c.get("TCC_EA0_WRREQ_sum", 0) / sims,
           "valu_insts_per_sim_per_wave64": c["SQ_INSTS_VALU"] * 64.0 / sims,
           # kept for bench.py: calibrated HBM (DRAM-side) bytes per launch
           "hbm_bytes_per_launch": d["dram_bytes"],
           "correction": "calibrated (tools/pmc_calib.hip): reads = 128 B per TCC_EA0_RDREQ_128B request (+64/32 B for "
                         "the 64-/32-B ones), writes = WRITE_SIZE (exact for 32-B and 64-B write requests)"}
    if calib_path and os.path.exists(calib_path):
        cal = json.load(open(calib_path))["tests"]
        rd = cal.get("rd16x1", {})
        out["random_line_read_peak_gbs_measured"] = rd.get("dram_gbs")
        if ms and rd.get("dram_gbs"):
            out["dram_frac_of_random_line_peak"] = d["dram_gbs"] / rd["dram_gbs"]
        out["calibration"] = os.path.relpath(calib_path)
    return out


def main():
    mode = sys.argv[1]
    if mode == "calib":
        res = calib(sys.argv[2], sys.argv[3])
        path = sys.argv[4] if len(sys.argv) > 4 else "profiles/r03/pmc_calib.json"
    else:
        res = search(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]),
                     sys.argv[7] if len(sys.argv) > 7 else None, sys.argv[8] if len(sys.argv) > 8 else "main")
        path = sys.argv[6]
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("tests", "pmc_per_launch")}, indent=1)[:3000])


if __name__ == "__main__":
    main()
