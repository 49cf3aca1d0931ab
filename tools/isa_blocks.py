"""Per-basic-block instruction counts of one kernel in a line-table assembly listing, with the
source lines each block's instructions come from (the attribution behind
profiles/r06/valu_by_phase.json).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
        -gline-tables-only -o doko_g.s master_doko_reinforcement_learning_amd/csrc/doko_amd.hip
    python tools/isa_blocks.py doko_g.s 'search_kernelIN2dk4FdoEELb0ENS1_8NodeHot8E' [--json out.json]

A block is the code between two labels (`.LBB*` / `; %bb.*`).  Instructions are classed as VALU
(v_*, not v_readlane/writelane... which are counted as VALU too, as the SQ counts them), SALU
(s_* minus the memory, branch and wait ones), SMEM, VMEM (global_/buffer_/flat_), LDS (ds_),
branch, waitcnt.  Each instruction carries the last `.loc` before it (file, line)."""
import argparse
import collections
import json
import re
import sys


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_store", "s_dcache")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_sched", "s_endpgm", "s_setprio")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return None


def parse(path, kernel):
    files = {}
    blocks = []
    cur = None
    loc = (None, 0)
    inside = False
    with open(path) as fh:
        for line in fh:
            m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', line)
            if m:
                files[int(m.group(1))] = m.group(2).split("/")[-1]
                continue
            if not inside:
                if line.startswith("_Z") and kernel in line.split(":")[0] and line.split(":")[0].endswith("_") is not None \
                        and re.match(r"^_Z\S*:", line):
                    inside = True
                    cur = {"label": "entry", "ins": [], "succ": []}
                    blocks.append(cur)
                continue
            if re.match(r"^\s*\.Lfunc_end", line) or line.startswith("\t.size"):
                break
            m = re.match(r"^(\.LBB\w+):", line) or re.match(r"^; %(bb\.\d+):", line)
            if m:
                if cur["ins"] and not cur["ins"][-1][0].startswith(("s_branch", "s_setpc")):
                    cur["succ"].append(m.group(1))   # fall through
                cur = {"label": m.group(1), "ins": [], "succ": []}
                blocks.append(cur)
                continue
            m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
            if m:
                loc = (int(m.group(1)), int(m.group(2)))
                continue
            m = re.match(r"^\s+([a-z_][a-z0-9_]*)\b(.*)", line)
            if m and not line.lstrip().startswith("."):
                op = m.group(1)
                k = classify(op)
                if k is None:
                    continue
                cur["ins"].append((op, k, loc))
                if k == "branch":
                    t = re.search(r"(\.LBB\w+)", m.group(2))
                    if t:
                        cur["succ"].append(t.group(1))
    return files, blocks


def summarize(files, blocks):
    out = []
    index = {b["label"]: i for i, b in enumerate(blocks)}
    for i, b in enumerate(blocks):
        cnt = collections.Counter(k for _, k, _ in b["ins"])
        src = collections.Counter("%s:%d" % (files.get(f, "?"), l) for _, _, (f, l) in b["ins"] if f is not None and l)
        back = [s for s in b["succ"] if s in index and index[s] <= i]
        out.append({"i": i, "label": b["label"], "n": len(b["ins"]), **{k: cnt.get(k, 0) for k in
                    ("valu", "salu", "smem", "vmem", "lds", "branch", "wait")},
                    "src": src.most_common(4), "succ": b["succ"], "back_edges": back})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--json")
    a = ap.parse_args()
    files, blocks = parse(a.asm, a.kernel)
    s = summarize(files, blocks)
    for b in s:
        print("%4d %-12s n=%4d valu=%4d salu=%3d vmem=%2d lds=%2d br=%2d  %s%s" % (
            b["i"], b["label"], b["n"], b["valu"], b["salu"], b["vmem"], b["lds"], b["branch"],
            " ".join("%s(%d)" % x for x in b["src"]), ("  BACK->" + ",".join(b["back_edges"])) if b["back_edges"] else ""))
    tot = collections.Counter()
    for b in s:
        for k in ("valu", "salu", "vmem", "lds"):
            tot[k] += b[k]
    print("total", dict(tot), "blocks", len(s), file=sys.stderr)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(s, fh, indent=0)


if __name__ == "__main__":
    main()
