"""C3 search time against context-creation settings, alternated in one process.

Each variant is a set of environment variables read by dk_create (DK_POOL_CONTIG,
DK_SLOT_CAPACITY, ...).  Contexts are created in the order A B B A A B ..., each runs the
C3 search `reps` times (the first warms up), so allocation-to-allocation spread and clock
drift show up per variant.  Results must be identical across variants (checked).

A variant may name its own build with LIB=<file in the package dir> (libraries loaded side by
side, as tools/ab_inproc.py does).

usage: python tools/env_sweep.py "A=DK_POOL_CONTIG=0" "B=DK_POOL_CONTIG=1,LIB=libdoko_amd_x.so" [--contexts 4]
       [--infostates 18432] [--samples 64] [--reps 3]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--contexts", type=int, default=4)
    ap.add_argument("--infostates", type=int, default=18432)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--samples", type=int, default=64, help="samples per infostate (8 = one rank's share at N = 8)")
    ap.add_argument("--no-check", action="store_true", help="speed-of-light variants: results may differ")
    ap.add_argument("--workload", choices=["c3", "c2"], default="c3",
                    help="c2: bench.py's C2 roots (rs-doko deals after 4x Healthy), --roots of them")
    ap.add_argument("--roots", type=int, default=32768)
    a = ap.parse_args()
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    from cap_sweep import c3_roots
    from ab_inproc import load
    L = _native.lib()
    variants = []
    for v in a.variants:
        name, _, rest = v.partition("=")
        env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
        lib = env.pop("LIB", None)
        variants.append((name, env, load(os.path.join(ROOT, "master_doko_reinforcement_learning_amd", lib)) if lib else L))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    I, S, iters = a.infostates, a.samples, 1000
    game = 0
    if a.workload == "c2":
        n, game = a.roots, 1
        gen = dk.Engine(device=0, max_roots=n, max_iterations=1, slot_capacity=64)
        gidx = np.arange(n, dtype=np.uint64)
        d_rs = torch.tensor((gidx + np.uint64(0xD0C00000)).view(np.int64), device=dev)
        roots = torch.zeros((n, 128), dtype=torch.uint8, device=dev)
        assert L.dk_new_game_batch_async(gen.ctx, 1, d_rs.data_ptr(), n, roots.data_ptr(), sp) == 0
        h = torch.full((n,), 1 << 24, dtype=torch.int64, device=dev)
        for _ in range(4):
            assert L.dk_env_step_batch_async(gen.ctx, roots.data_ptr(), h.data_ptr(), n, sp) == 0
        assert L.dk_sync(gen.ctx, sp) == 0
        gen.close()
        d_srch = torch.tensor((gidx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)).view(np.int64), device=dev)
    else:
        n = I * S
        roots, d_srch = c3_roots(dk, L, dev, sp, I, S)
    v = torch.zeros((n, 39), dtype=torch.int32, device=dev)
    q = torch.zeros((n, 39), dtype=torch.float64, device=dev)
    bst = torch.zeros(n, dtype=torch.uint8, device=dev)
    times = {name: [] for name, _, _ in variants}
    ref = None
    order = list(range(len(variants)))
    for c in range(a.contexts):
        for k in order:
            name, env, Lk = variants[k]
            saved = {key: os.environ.get(key) for key in env}
            os.environ.update(env)
            cfg = _native.dk_config(0, n, iters, 0)
            ctx = Lk.dk_create(ctypes.byref(cfg))
            assert ctx
            for key, val in saved.items():
                if val is None:
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = val
            got = []
            for r in range(a.reps):
                assert Lk.dk_search_batch_async(ctx, game, roots.data_ptr(), d_srch.data_ptr(), n, iters, 2.5,
                                                v.data_ptr(), q.data_ptr(), bst.data_ptr(), sp) == 0
                assert Lk.dk_sync(ctx, sp) == 0
                ms = ctypes.c_float()
                Lk.dk_last_search_ms(ctx, ctypes.byref(ms))
                if r > 0:
                    got.append(ms.value)
            Lk.dk_destroy(ctx)
            if ref is None:
                ref = v.clone()
            assert a.no_check or torch.equal(ref, v), "variant changed the results"
            times[name].extend(got)
            print("ctx %d %-10s %s ms" % (c, name, " ".join("%.1f" % t for t in got)), flush=True)
        order = order[::-1]
    for name, _, _ in variants:
        t = np.array(times[name])
        print("%-10s median %.1f mean %.1f min %.1f max %.1f ms" % (name, np.median(t), t.mean(), t.min(), t.max()))


if __name__ == "__main__":
    main()
