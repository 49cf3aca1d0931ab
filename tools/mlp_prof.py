"""Phase clocks of mlp_ln_kernel (a -DDK_NET_PROF build): mean shader cycles per workgroup in
each phase, for wave 0 (the early group of the skewed chunk loop) and wave 4 (the late group).
usage (GPU box): DK_LIB=.../libdoko_amd_nprof.so python tools/mlp_prof.py [rows]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["prologue", "gelu_gemm2", "store_chunk", "barrier", "gemm1", "epilogue"]


def main(rows=8192 * 62, reps=10, d=160):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    rows = int(rows)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    n = 4 * d
    h = torch.randn(rows, d, device=dev).bfloat16()
    x = (torch.randn(rows, d, device=dev) * 2).bfloat16()
    w1 = (torch.randn(n, d, device=dev) / d ** 0.5).bfloat16()
    b1 = (torch.randn(n, device=dev) * 0.1).bfloat16()
    w2 = (torch.randn(d, n, device=dev) / n ** 0.5).bfloat16()
    b2 = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = torch.ones(d, device=dev).bfloat16()
    be = torch.zeros(d, device=dev).bfloat16()
    out = torch.empty(rows, d, device=dev).bfloat16()
    st = torch.cuda.current_stream(dev).cuda_stream
    f = lambda: L.dk_net_mlp_ln_bf16_async(h.data_ptr(), x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                           b2.data_ptr(), rows, d, n, g.data_ptr(), be.data_ptr(), 1e-5,
                                           out.data_ptr(), st)
    rd = L.dk_net_mlp_prof_read
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
    wgs = (rows + 255) // 256
    per = acc.astype(np.float64) / (wgs * reps)
    print(json.dumps({"rows": rows, "ms": e0.elapsed_time(e1) / reps,
                      "wave0_early": {k: round(float(v)) for k, v in zip(PHASES, per[:6])},
                      "wave4_late": {k: round(float(v)) for k, v in zip(PHASES, per[8:14])}}))


if __name__ == "__main__":
    main(*sys.argv[1:2])
