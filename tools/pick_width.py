"""Design data for the search kernel's pick width (oracle-side, CPU).

A 64-lane wave runs the 64 CAP samples of one C3 infostate in lockstep, one simulation
at a time; selection trip t of simulation k is the t-th branching pick of every lane
still selecting.  The device unrolls every pick over SCAN_REG = 12 children; a
wave-uniform dispatch on the largest child count among the lanes picking in a trip
could run a narrower unrolled pick.  Prints, per bucket width, the share of trips and
the relative pick cost against the fixed 12-wide pick."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def traces_for_infostate(ol, j, S=64, iters=1000):
    st = ol.FdoState.new_game(0xC3000000 + j)
    for _ in range(4):
        st.play(24)
    st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4], True)
    lanes = []
    buf = (ctypes.c_uint8 * 200000)()
    for s in range(S):
        smp = st.card_matching(ol.rng_seed(0xC3200000 + j * S + s))
        n = ol.lib().or_fdo_search_trace(smp.h, ol.rng_seed(0xC3300000 + j * S + s), iters, ctypes.c_double(2.5), buf, 200000)
        seq = list(buf[:n])
        sims, cur = [], []
        for x in seq:
            if x == 0:
                sims.append(cur)
                cur = []
            else:
                cur.append(x)
        lanes.append(sims)
    return lanes


def main(n_info=24, buckets=(2, 3, 4, 6, 8, 12)):
    import oracle_lib as ol
    lib = ol.lib()
    lib.or_fdo_search_trace.restype = ctypes.c_int
    lib.or_fdo_search_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_double,
                                        ctypes.c_void_p, ctypes.c_int]
    hist = {b: 0 for b in buckets}
    big = 0
    trips = 0
    lane_picks = 0
    for j in range(n_info):
        lanes = traces_for_infostate(ol, j * 7 + 1)
        iters = len(lanes[0])
        for k in range(iters):
            per = [ln[k] for ln in lanes]
            T = max(len(p) for p in per)
            for t in range(T):
                ns = [p[t] for p in per if len(p) > t]
                lane_picks += len(ns)
                m = max(ns)
                trips += 1
                for b in buckets:
                    if m <= b:
                        hist[b] += 1
                        break
                else:
                    big += 1
    print("trips %d, lane-picks per trip %.1f of 64, >12 children: %d" % (trips, lane_picks / trips, big))
    cost = 0.0
    for b in buckets:
        print("wave max n <= %2d: %5.1f %% of trips" % (b, 100.0 * hist[b] / trips))
        cost += hist[b] * b
    cost += big * 12
    print("bucketed pick cost / 12-wide pick cost: %.2f" % (cost / (12.0 * trips)))


if __name__ == "__main__":
    main()
