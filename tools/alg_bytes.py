"""Algorithmic bytes per simulation for the roofline.

B_sim = 128 (packed root state) + 16 * sum_B (sibling stats read in selection)
        + 32 * (d + 1) (path stats read-modify-write in backup) + 32 (new node)
with sum_B (children scanned per simulation) and d + 1 (path nodes per
simulation) measured by the ORACLE's counters on roots of the bench workload.
Writes profiles/alg_bytes_<workload>.json (read by bench.py).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(n_roots=256, iters=1000, infostates=512, samples=64):
    import oracle_lib as ol
    scanned = path = sims = 0
    for k in range(n_roots):
        j, s = (k * 37) % infostates, (k * 11) % samples   # spread over the workload's infostates / samples
        st = ol.FdoState.new_game(0xC3000000 + j)
        for _ in range(4):
            st.play(24)
        st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4], True)
        smp = st.card_matching(ol.rng_seed(0xC3200000 + j * samples + s))
        _, _, _, ctr = smp.search(ol.rng_seed(0xC3300000 + j * samples + s), iters, 2.5)
        sims += ctr[0]
        scanned += ctr[1]
        path += ctr[2]
    cs, pn = scanned / sims, path / sims
    out = {"workload": "c3", "roots_sampled": n_roots, "iterations": iters, "children_scanned_per_sim": cs,
           "path_nodes_per_sim": pn, "b_sim": 128 + 16 * cs + 32 * pn + 32,
           "formula": "128 + 16*children_scanned + 32*path_nodes + 32 (SURVEY.md 8(d))"}
    with open(os.path.join(ROOT, "profiles", "alg_bytes_c3.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
