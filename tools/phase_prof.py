"""Phase breakdown of the search kernel (profiling build, -DDK_PHASE_PROF).

Runs the bench workload once with libdoko_amd_prof.so and prints, per phase,
the mean wave-clock cycles per simulation (select / expand / rollout / backup)
plus the mean select depth.  Usage (GPU box):
    DK_LIB=master_doko_reinforcement_learning_amd/libdoko_amd_prof.so python tools/phase_prof.py [bench args]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = _native.lib()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng, step, n_roots, bufs = bench.make_workload(args, dk, L, dev, stream.cuda_stream, 0, 1, 0)
    prof = getattr(L, "dk_phase_profile", None)
    if prof is not None:
        prof.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        out = np.zeros((n_roots, 40), dtype=np.uint64)
        prof(eng.ctx, out.ctypes.data, n_roots)  # clear
    step()
    torch.cuda.synchronize(dev)
    ms = eng.last_search_ms()
    res = {"roots": n_roots, "iterations": args.iterations, "search_ms": ms,
           "rpw": os.environ.get("DK_ROOTS_PER_WAVE", "64"), "layout": os.environ.get("DK_LAYOUT", "0")}
    if prof is not None:
        prof(eng.ctx, out.ctypes.data, n_roots)
        sims = n_roots * args.iterations
        tot = out[:, :4].astype(np.float64).sum(axis=0) / sims
        res.update({"cyc_per_sim": {"select": tot[0], "expand": tot[1], "rollout": tot[2], "backup": tot[3]},
                    "mean_depth": float(out[:, 4].astype(np.float64).sum() / sims),
                    "forced_levels": float(out[:, 5].astype(np.float64).sum() / sims),
                    "branch_levels": float(out[:, 6].astype(np.float64).sum() / sims),
                    "wave_max_depth": float(out[:, 7].astype(np.float64).sum() / sims),
                    "select_load_cyc": float(out[:, 8].astype(np.float64).sum() / sims),
                    "select_pick_cyc": float(out[:, 9].astype(np.float64).sum() / sims),
                    "rollout_plies": float(out[:, 10].astype(np.float64).sum() / sims),
                    "rollout_plies_wave_max": float(out[:, 11].astype(np.float64).sum() / sims),
                    "expand_step_cyc": float(out[:, 12].astype(np.float64).sum() / sims),
                    "expand_allowed_cyc": float(out[:, 13].astype(np.float64).sum() / sims),
                    "expand_load_cyc": float(out[:, 14].astype(np.float64).sum() / sims),
                    "expand_unpack_cyc": float(out[:, 15].astype(np.float64).sum() / sims),
                    "expand_first_allowed_cyc": float(out[:, 16].astype(np.float64).sum() / sims),
                    "expand_first_fraction": float(out[:, 17].astype(np.float64).sum() / sims),
                    "expand_pack_store_cyc": float(out[:, 18].astype(np.float64).sum() / sims),
                    "select_forced_cyc": float(out[:, 19].astype(np.float64).sum() / sims),
                    "select_forced_loads_wave_max": float(out[:, 20].astype(np.float64).sum() / sims)})
        # wave-level branching trips (counted once per wave): per wave-simulation, the histogram of
        # their active lanes and the mean active lanes of a trip
        # roots per wave of the launch (DK_PROF_RPW: 64 for C3, 32 for single-wave launches like C2)
        res["rpw_eff"] = int(os.environ.get("DK_PROF_RPW", "64"))
        wsims = sims / float(res["rpw_eff"])
        trips = float(out[:, 21].astype(np.float64).sum())
        res["select_trips_per_wave_sim"] = trips / wsims
        res["select_trip_active_hist_per_wave_sim"] = {
            b: float(out[:, 22 + i].astype(np.float64).sum()) / wsims for i, b in enumerate(["<=8", "<=16", "<=32", "<=48", "<=64"])}
        res["select_trip_mean_active_lanes"] = float(out[:, 27].astype(np.float64).sum()) / max(trips, 1.0)
        tot = out[:, :4].astype(np.float64).sum(axis=1)   # per-root wave-clock cycles over the whole search
        if args.workload == "c3":
            k = np.array([[0, 8, 20, 32][(r // args.samples) % 4] for r in range(n_roots)])
            res["wave_cycles_by_k"] = {int(kk): [float(tot[k == kk].min()), float(tot[k == kk].mean()), float(tot[k == kk].max())]
                                       for kk in (0, 8, 20, 32)}
        res["wave_cycles_min_mean_max"] = [float(tot.min()), float(tot.mean()), float(tot.max())]
    print(json.dumps(res))
    eng.close()


if __name__ == "__main__":
    main()
