"""Phase clocks of mlp_ln_f32x3_kernel (a -DDK_NET_PROF build): mean shader cycles per workgroup of
its wave 0 in each phase (drained stamps).
usage (GPU box): DK_LIB=.../libdoko_amd_nprof.so python tools/mlp_f32_prof.py [rows]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["prologue_stage0", "gemm1", "gelu_split", "gemm2", "wait_barrier", "epilogue"]


def main(rows=8192 * 62, reps=10, d=160):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    rows = int(rows)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    n = 4 * d
    h = torch.randn(rows, d, device=dev)
    x = torch.randn(rows, d, device=dev)
    w = [torch.randn(n, d, device=dev) / d ** 0.5, torch.randn(d, n, device=dev) / n ** 0.5]
    from master_doko_reinforcement_learning_amd.az_network import mlp_split_bf16x3
    sp = mlp_split_bf16x3(*w)
    b1, b2 = torch.randn(n, device=dev) * 0.1, torch.randn(d, device=dev) * 0.1
    g, be = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    out = torch.empty(rows, d, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    f = lambda: L.dk_net_mlp_ln_f32x3_async(h.data_ptr(), x.data_ptr(), sp[0].data_ptr(), sp[1].data_ptr(), b1.data_ptr(),
                                            sp[2].data_ptr(), sp[3].data_ptr(), b2.data_ptr(), rows, d, n, g.data_ptr(),
                                            be.data_ptr(), 1e-5, out.data_ptr(), st)
    rd = L.dk_net_mlp_prof_read
    import ctypes
    rd.argtypes = [ctypes.c_void_p]
    acc = np.zeros(16, dtype=np.uint64)
    assert f() == 0
    torch.cuda.synchronize()
    rd(acc.ctypes.data)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        assert f() == 0
    e1.record()
    torch.cuda.synchronize()
    rd(acc.ctypes.data)
    wpg = 4
    wgs = (rows + 32 * wpg - 1) // (32 * wpg)
    per = acc.astype(np.float64) / (wgs * reps)
    print(json.dumps({"rows": rows, "ms": e0.elapsed_time(e1) / reps, "waves_per_wg": wpg,
                      "wave0_cycles_per_wg": {k: round(float(v)) for k, v in zip(PHASES, per[:6])}}))


if __name__ == "__main__":
    main(*sys.argv[1:2])
