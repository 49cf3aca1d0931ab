"""Algorithmic bytes per simulation for the roofline.

B_sim = 128 (packed root state) + 16 * sum_B (sibling stats read in selection)
        + 32 * (d + 1) (path stats read-modify-write in backup) + 32 (new node)
with sum_B (children scanned per simulation) and d + 1 (path nodes per
simulation) measured by the ORACLE's counters on roots of the bench workload.
Writes profiles/alg_bytes_<workload>.json (read by bench.py).
usage: python tools/alg_bytes.py [c3|c2|c2d]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def root_of(workload, k, infostates=512, samples=64):
    """Root k of the bench workload (bench.make_workload's seeds) and its search seed."""
    import oracle_lib as ol
    if workload == "c2":
        i = (k * 997) % 32768
        st = ol.DoState.new_game(0xD0C00000 + i)
        for _ in range(4):
            st.play(24)
        return st, (i * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF
    j, s = (k * 37) % infostates, (k * 11) % samples   # spread over the workload's infostates / samples
    if workload == "c2d":
        st = ol.DoState.new_game(0xC3000000 + j)
        for _ in range(4):
            st.play(24)
        st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4])
        return st.sample_assignment_full(ol.rng_seed(0xC3200000 + j * samples + s)), 0xC3300000 + j * samples + s
    st = ol.FdoState.new_game(0xC3000000 + j)
    for _ in range(4):
        st.play(24)
    st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4], True)
    return st.card_matching(ol.rng_seed(0xC3200000 + j * samples + s)), 0xC3300000 + j * samples + s


def main(workload="c3", n_roots=256, iters=1000):
    import oracle_lib as ol
    scanned = path = sims = 0
    for k in range(n_roots):
        root, seed = root_of(workload, k)
        _, _, _, ctr = root.search(ol.rng_seed(seed), iters, 2.5)
        sims += ctr[0]
        scanned += ctr[1]
        path += ctr[2]
    cs, pn = scanned / sims, path / sims
    out = {"workload": workload, "roots_sampled": n_roots, "iterations": iters, "children_scanned_per_sim": cs,
           "path_nodes_per_sim": pn, "b_sim": 128 + 16 * cs + 32 * pn + 32,
           "formula": "128 + 16*children_scanned + 32*path_nodes + 32 (SURVEY.md 8(d))"}
    with open(os.path.join(ROOT, "profiles", "alg_bytes_%s.json" % workload), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:2])
