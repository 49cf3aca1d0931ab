"""Check PMC pass definitions before a GPU run: every counter exists for gfx950 and no pass
exceeds the per-block limits (MI355X: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM; _sum etc. of one
counter count once).  usage: python tools/pmc_check.py "C1 C2 ..." "C3 ..." """
import sys

import yaml

LIMIT = {"SQ": 8, "TCC": 4, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2, "SQC": 4}


def names():
    d = yaml.safe_load(open("/opt/rocm/share/rocprofiler-sdk/counter_defs.yaml"))
    lst = d if isinstance(d, list) else d.get("rocprofiler-sdk", {}).get("counters", d)
    if isinstance(lst, dict):
        lst = next(v for v in lst.values() if isinstance(v, list))
    return {c["name"] for c in lst for df in c.get("definitions", []) if "gfx950" in df.get("architectures", [])}


def main(passes):
    have = names()
    ok = True
    for p in passes:
        used = {}
        for c in p.split():
            if c not in have and c not in ("FETCH_SIZE", "WRITE_SIZE"):
                print("unknown counter", c)
                ok = False
            base = c
            for suf in ("_sum", "_avr", "_min", "_max"):
                if base.endswith(suf):
                    base = base[: -len(suf)]
            blk = base.split("_")[0]
            used.setdefault(blk, set()).add(base)
        for blk, s in used.items():
            if blk in LIMIT and len(s) > LIMIT[blk]:
                print("pass exceeds", blk, len(s), p)
                ok = False
    print("ok" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
