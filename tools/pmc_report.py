"""Per-dispatch PMC values of named kernels from tools/pmc_passes.sh output.

usage: python tools/pmc_report.py <pmc_dir> <kernel substring> [...] [--last | --main]
  --last : the kernel's last dispatch in each pass (pmc_calib: warm-up, then the timed launch)
  --main : the average over the kernel's main dispatches (counter total >= 5 % of the largest;
           the search's fallback pass drains at once and is left out)
Prints {substring: {counter: value}} as JSON."""
import csv
import glob
import json
import os
import sys
from collections import OrderedDict, defaultdict


def collect(d, subs, mode):
    out = {s: {} for s in subs}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = {s: OrderedDict() for s in subs}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                for s in subs:
                    if s in r["Kernel_Name"]:
                        per[s].setdefault(int(r["Dispatch_Id"]), defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
        for s in subs:
            if not per[s]:
                continue
            ids = sorted(per[s])
            if mode == "last":
                pick = [ids[-1]]
            elif mode == "max":   # the single heaviest dispatch (the headline launch of a bench run)
                w = {k: sum(per[s][k].values()) for k in ids}
                pick = [max(ids, key=lambda k: w[k])]
            else:
                w = {k: sum(per[s][k].values()) for k in ids}
                top = max(w.values())
                pick = [k for k in ids if w[k] >= 0.05 * top]
            for name in per[s][pick[0]]:
                out[s][name] = sum(per[s][k].get(name, 0.0) for k in pick) / len(pick)
            out[s].setdefault("_dispatches", {})[os.path.basename(os.path.dirname(f)) or f] = len(pick)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    mode = "last" if "--last" in sys.argv else "main"
    print(json.dumps(collect(args[0], args[1:], mode), indent=1))


if __name__ == "__main__":
    main()
