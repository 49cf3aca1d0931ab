"""Sum the PMC values of one kernel (by name substring) per launch from tools/pmc.sh passes.
usage: python tools/pmc_sum.py [kernel_substring] [pmc_dir]  -> JSON on stdout"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(kname="search_kernel", d="gpurun_out/pmc"):
    """Per-launch averages over the kernel's MAIN launches: a search step also launches the
    fallback pass, which drains at once when no root overflowed; dispatches whose counter
    total is under 5 % of the largest are those and are left out."""
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kname not in r["Kernel_Name"]:
                    continue
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        if not per:
            continue
        weight = {k: sum(v.values()) for k, v in per.items()}
        top = max(weight.values())
        main_launches = [k for k in per if weight[k] >= 0.05 * top]
        for name in per[main_launches[0]]:
            out[name] = sum(per[k].get(name, 0.0) for k in main_launches) / len(main_launches)
        out.setdefault("_launches", {})[os.path.basename(os.path.dirname(f))] = len(main_launches)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
