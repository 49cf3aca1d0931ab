"""Phase table of the C3 search kernel from the doubling measurements (tools/gpu/doubling.sh):
per measurement build, the extra instructions (PMC) and the extra kernel time (in-process A/B
against the product build) that doing one phase a second time costs = that phase's share.

usage: python tools/doubling_report.py <gpurun_out dir> [--out profiles/r06/valu_by_phase.json]
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_report import collect  # noqa: E402

ROOTS, ITERS = 36864 * 64, 1000
WAVE_SIMS = ROOTS * ITERS / 64          # wave-simulations per launch (64 roots per wave)
VARIANTS = {
    "roll2": "rollout (card phase + reservation / announcement collapse + scoring), second copy",
    "exp2": "expansion: unpack, action set, transition, pack (second copy)",
    "pick2": "UCT pick of every branching selection trip (second copy)",
    "trick16": "fast-path rollout tricks whose wave has <= 16 active lanes (second copy)",
    "trick64": "every fast-path rollout trick (second copy)",
}


def ab_ratio(path):
    with open(path) as fh:
        txt = fh.read()
    m = re.search(r"\| B/A time ([0-9.]+) \(median ([0-9.]+)\)", txt)
    a = re.search(r"A \S+ mean ([0-9.]+) median ([0-9.]+)", txt)
    return (float(m.group(1)), float(m.group(2)), float(a.group(2))) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    base = collect(os.path.join(a.dir, "pmc_base"), ["search_kernel"], "max")["search_kernel"]
    res = {"workload": "C3, 36,864 infostates x 64 samples x 1000 simulations (bench.py default), search_kernel<FdoE, false, NodeHot8>",
           "method": "each measurement build runs one phase a second time on copies with the result discarded and kept "
                     "alive (results unchanged, checked); PMC: SQ_INSTS_* of the search launch (rocprofv3, one pass per "
                     "build); time: in-process A/B against the product build (tools/ab_inproc.py, 3 rounds, both orders)",
           "base": {"valu_per_wave_sim": base["SQ_INSTS_VALU"] / WAVE_SIMS, "salu_per_wave_sim": base["SQ_INSTS_SALU"] / WAVE_SIMS,
                    "counters": {k: v for k, v in base.items() if not k.startswith("_")}},
           "phases": {}}
    for v, desc in VARIANTS.items():
        d = os.path.join(a.dir, "pmc_" + v)
        if not os.path.isdir(d):
            continue
        c = collect(d, ["search_kernel"], "max")["search_kernel"]
        ab = ab_ratio(os.path.join(a.dir, "ab_%s.log" % v))
        dv = (c["SQ_INSTS_VALU"] - base["SQ_INSTS_VALU"]) / WAVE_SIMS
        ds = (c["SQ_INSTS_SALU"] - base["SQ_INSTS_SALU"]) / WAVE_SIMS
        res["phases"][v] = {"what": desc, "valu_per_wave_sim": dv, "salu_per_wave_sim": ds,
                            "valu_share": dv / res["base"]["valu_per_wave_sim"],
                            "time_ratio_mean": ab[0] if ab else None, "time_ratio_median": ab[1] if ab else None,
                            "time_share": (ab[1] - 1.0) if ab else None, "base_ms_median": ab[2] if ab else None}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
