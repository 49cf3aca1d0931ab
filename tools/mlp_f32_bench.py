"""The f32 MLP half of a block: mlp_ln_f32x3_kernel (one pass, bf16x3 products) against the
unfused f32 path FusedTrunkF32 took until round 5 (hipBLASLt F.linear at matmul precision
"medium" without bias + gelu_bias_f32 + F.linear + add_bias_ln_f32), alternated, HIP events.
usage: python tools/mlp_f32_bench.py [rows] [d] [reps]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(rows=507904, d=160, reps=20):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    n = 4 * d
    h = torch.randn(rows, d, device=dev)
    x0 = torch.randn(rows, d, device=dev)
    w1, b1 = torch.randn(n, d, device=dev) / d ** 0.5, torch.randn(n, device=dev) * 0.1
    w2, b2 = torch.randn(d, n, device=dev) / n ** 0.5, torch.randn(d, device=dev) * 0.1
    g, be = 1 + 0.1 * torch.randn(d, device=dev), 0.1 * torch.randn(d, device=dev)
    from master_doko_reinforcement_learning_amd.az_network import mlp_split_bf16x3
    split = mlp_split_bf16x3(w1, w2)
    st = torch.cuda.current_stream(dev).cuda_stream
    torch.set_float32_matmul_precision("medium")
    x = x0.clone()
    out = torch.empty_like(x)

    def fused():
        assert L.dk_net_mlp_ln_f32x3_async(h.data_ptr(), x.data_ptr(), split[0].data_ptr(), split[1].data_ptr(),
                                           b1.data_ptr(), split[2].data_ptr(), split[3].data_ptr(), b2.data_ptr(), rows,
                                           d, n, g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(), st) == 0

    def unfused():
        a = F.linear(h, w1)
        assert L.dk_net_gelu_bias_f32_async(a.data_ptr(), b1.data_ptr(), a.numel(), n, st) == 0
        dl = F.linear(a, w2)
        assert L.dk_net_add_bias_ln_f32_async(x.data_ptr(), dl.data_ptr(), b2.data_ptr(), rows, d, g.data_ptr(),
                                              be.data_ptr(), 1e-5, out.data_ptr(), st) == 0

    res = {"fused": [], "unfused": []}
    for name, fn in (("fused", fused), ("unfused", unfused)):
        fn()
    torch.cuda.synchronize()
    for r in range(reps):
        for name, fn in ((("fused", fused), ("unfused", unfused)) if r % 2 == 0 else (("unfused", unfused), ("fused", fused))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
    flop = 2.0 * rows * d * n * 2
    for name, v in res.items():
        v = sorted(v)
        med = v[len(v) // 2]
        print("%-8s rows %d d %d: median %.3f ms min %.3f ms  %.0f TFLOP/s (f32 GEMM FLOPs)" % (
            name, rows, d, med, v[0], flop / med / 1e9))


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a)
