"""The MLP half of a DokoAzNet block at the C5 batch (8192 x 62 rows, d 160, hidden 640):
unfused (fc_gelu_kernel -> hipBLASLt proj -> add_ln_kernel) against the fused
mlp_ln_kernel, event-timed on the same inputs; prints ms, TFLOP/s and the max difference.
usage (GPU box): python tools/mlp_bench.py [rows] [reps] [d]"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(rows=8192 * 62, reps=20, d=160):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    rows, reps, d = int(rows), int(reps), int(d)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    n = 4 * d
    h = torch.randn(rows, d, device=dev).bfloat16()
    x0 = (torch.randn(rows, d, device=dev) * 2).bfloat16()
    w1 = (torch.randn(n, d, device=dev) / d ** 0.5).bfloat16()
    b1 = (torch.randn(n, device=dev) * 0.1).bfloat16()
    w2 = (torch.randn(d, n, device=dev) / n ** 0.5).bfloat16()
    b2 = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = torch.ones(d, device=dev).bfloat16()
    be = torch.zeros(d, device=dev).bfloat16()
    st = torch.cuda.current_stream(dev).cuda_stream
    a = torch.empty(rows, n, device=dev).bfloat16()
    out = torch.empty(rows, d, device=dev).bfloat16()

    def unfused(x):
        assert L.dk_net_fc_gelu_bf16_async(h.data_ptr(), w1.data_ptr(), b1.data_ptr(), rows, d, n, a.data_ptr(), st) == 0
        delta = F.linear(a, w2, b2)
        assert L.dk_net_add_ln_bf16_async(x.data_ptr(), delta.data_ptr(), rows, d, g.data_ptr(), be.data_ptr(), 1e-5,
                                          out.data_ptr(), st) == 0

    def fused(x):
        assert L.dk_net_mlp_ln_bf16_async(h.data_ptr(), x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                          b2.data_ptr(), rows, d, n, g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(),
                                          st) == 0

    res = {}
    outs = {}
    for name, fn in (("unfused", unfused), ("fused", fused), ("unfused2", unfused), ("fused2", fused)):
        x = x0.clone()
        fn(x)
        torch.cuda.synchronize()
        outs[name] = (x.clone(), out.clone())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        xs = [x0.clone() for _ in range(reps)]
        torch.cuda.synchronize()
        e0.record()
        for i in range(reps):
            fn(xs[i])
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res[name] = {"ms": ms, "tflops": 4.0 * rows * d * n / (ms * 1e-3) / 1e12}
    res["max_abs_diff_x"] = (outs["fused"][0].float() - outs["unfused"][0].float()).abs().max().item()
    res["max_abs_diff_h"] = (outs["fused"][1].float() - outs["unfused"][1].float()).abs().max().item()
    res["rows"] = rows
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
