"""Regression fixtures made by the ORACLE (SURVEY.md §8(c) "fixtures to commit"), after it
passes the reference's own KATs (tests/test_oracle_golden.py):

  oracle_rollouts.json   1000 seeded random rollouts (rs-full-doko, C3 infostates)
                         -> player_points and the final SmallRng state (which fixes the
                         whole sequence of draws, i.e. of actions)
  oracle_searches.json   100 seeded 1000-simulation UCT searches -> visits[39], values[39]
                         (f64 bit patterns), best action, final SmallRng state
  oracle_cap.json        100 seeded CAP samples -> the packed sample and is_consistent

Inputs follow bench.py's C3 construction: infostate j = new_game(0xC3000000 + j), 4 x
Healthy, k_j in {0, 8, 20, 32} random plies without announcements (ply RNG
seed 0xC3100000 + j).  GPU tests compare the device against these files directly.
Run from the repository root: python tests/golden/make_oracle_fixtures.py
"""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def infostate(j):
    s = ol.FdoState.new_game(0xC3000000 + j)
    for _ in range(4):
        s.play(24)
    s.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4], True)
    return s


def rollouts(n=1000):
    out = []
    for i in range(n):
        s = infostate(i % 64)
        rng = ol.rng_seed(0x5EED0000 + i)
        pts = s.rollout(rng)
        out.append({"info": i % 64, "seed": 0x5EED0000 + i, "points": [int(p) for p in pts],
                    "rng_end": ["%016x" % x for x in rng]})
    return out


def searches(n=100, iters=1000, c=2.5):
    out = []
    for i in range(n):
        s = infostate(i)
        smp = s.card_matching(ol.rng_seed(0xC3200000 + i))
        rng = ol.rng_seed(0xC3300000 + i)
        best, visits, values, _ = smp.search(rng, iters, c)
        out.append({"info": i, "sample_seed": 0xC3200000 + i, "search_seed": 0xC3300000 + i, "iterations": iters, "c": c,
                    "root": smp.pack().hex(), "best": best, "visits": visits,
                    "values": ["%016x" % struct.unpack("<Q", struct.pack("<d", v))[0] for v in values],
                    "rng_end": ["%016x" % x for x in rng]})
    return out


def cap(n=100):
    out = []
    for i in range(n):
        s = infostate(i)
        smp = s.card_matching(ol.rng_seed(0xCA900000 + i))
        out.append({"info": i, "seed": 0xCA900000 + i, "infostate": s.pack().hex(), "sample": smp.pack().hex(),
                    "consistent": s.consistent_sample(smp)})
    return out


def main():
    for name, fn in (("oracle_rollouts.json", rollouts), ("oracle_searches.json", searches), ("oracle_cap.json", cap)):
        with open(os.path.join(OUT, name), "w") as fh:
            json.dump(fn(), fh, indent=None, separators=(",", ":"))
    print("wrote oracle fixtures to", OUT)


if __name__ == "__main__":
    main()
