"""Sum the PMC values of one kernel (by name substring) per launch from tools/pmc.sh passes.
usage: python tools/pmc_sum.py [kernel_substring] [pmc_dir]  -> JSON on stdout"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(kname="search_kernel", d="gpurun_out/pmc"):
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        launches = set()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kname not in r["Kernel_Name"]:
                    continue
                launches.add(r["Dispatch_Id"])
                per[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in per.items():
            out[k] = v / max(1, len(launches))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
