"""Phase clocks of qkv_attn_ln_kernel (a -DDK_NET_PROF build, e.g. tools/build_variant.sh nprof
-DDK_NET_PROF): mean shader cycles per workgroup (its wave 0) in each phase at the C5 shape.
usage (GPU box): DK_LIB=.../libdoko_amd_nprof.so python tools/attn_prof.py [d] [samples]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["h_stage", "v_proj", "k_proj", "q_proj", "attn_core", "y_barrier", "proj_res_ln"]


def main(d=160, B=8192, reps=10):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    d, B = int(d), int(B)
    dev = torch.device("cuda", 0)
    torch.manual_seed(2)
    h = torch.randn(B * 62, d, device=dev).bfloat16()
    x = (torch.randn(B * 62, d, device=dev) * 2).bfloat16()
    wq = (torch.randn(3 * d, d, device=dev) / d ** 0.5).bfloat16()
    bq = (torch.randn(3 * d, device=dev) * 0.1).bfloat16()
    w = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
    b = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = torch.ones(d, device=dev).bfloat16()
    be = torch.zeros(d, device=dev).bfloat16()
    out = torch.empty_like(h)
    st = torch.cuda.current_stream(dev).cuda_stream
    f = lambda: L.dk_net_qkv_attn_ln_bf16_async(h.data_ptr(), x.data_ptr(), wq.data_ptr(), bq.data_ptr(), w.data_ptr(),
                                                b.data_ptr(), B, 4, d // 4, g.data_ptr(), be.data_ptr(), 1e-5,
                                                out.data_ptr(), st)
    rd = L.dk_net_prof_read
    rd.argtypes = [ctypes.c_void_p]
    acc = np.zeros(8, dtype=np.uint64)
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
    per = acc[:len(PHASES)].astype(np.float64) / (B * reps)
    print(json.dumps({"d": d, "samples": B, "ms": e0.elapsed_time(e1) / reps,
                      "cycles_per_workgroup": {k: round(float(v)) for k, v in zip(PHASES, per)},
                      "total": round(float(per.sum()))}))


if __name__ == "__main__":
    main(*sys.argv[1:3])
