"""The attention half of a block after the qkv GEMM: unfused (attn62_kernel -> hipBLASLt
folded proj -> add_ln_kernel) against the fused attn_ln_kernel, event-timed on the same
inputs for several (d, samples); prints ms and the max difference per case.
usage (GPU box): python tools/attn_bench.py [reps] [d:samples ...]   (default 160:8192 160:740
256:740 256:2048 256:8192)"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def case(L, d, B, reps):
    dev = torch.device("cuda", 0)
    torch.manual_seed(2)
    hd, rows = d // 4, B * 62
    qkv = (torch.randn(B, 62, 3 * d, device=dev) * 1.5).bfloat16()
    x0 = (torch.randn(B, 62, d, device=dev) * 2).bfloat16()
    w = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
    b = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = torch.ones(d, device=dev).bfloat16()
    be = torch.zeros(d, device=dev).bfloat16()
    st = torch.cuda.current_stream(dev).cuda_stream
    y = torch.empty(B, 62, d, device=dev).bfloat16()
    out = torch.empty(B, 62, d, device=dev).bfloat16()

    def unfused(x):
        assert L.dk_net_attn62_bf16_async(qkv.data_ptr(), y.data_ptr(), B, 4, hd, st) == 0
        delta = F.linear(y, w, b)
        assert L.dk_net_add_ln_bf16_async(x.data_ptr(), delta.data_ptr(), rows, d, g.data_ptr(), be.data_ptr(), 1e-5,
                                          out.data_ptr(), st) == 0

    def fused(x):
        assert L.dk_net_attn_ln_bf16_async(qkv.data_ptr(), x.data_ptr(), w.data_ptr(), b.data_ptr(), B, 4, hd,
                                           g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(), st) == 0

    # with the qkv projection: hipBLASLt qkv GEMM + attn_ln_kernel against qkv_attn_ln_kernel
    h = torch.randn(B, 62, d, device=dev).bfloat16()
    wq = (torch.randn(3 * d, d, device=dev) / d ** 0.5).bfloat16()
    bq = (torch.randn(3 * d, device=dev) * 0.1).bfloat16()

    def gemm_fused(x):
        q = F.linear(h, wq, bq)
        assert L.dk_net_attn_ln_bf16_async(q.data_ptr(), x.data_ptr(), w.data_ptr(), b.data_ptr(), B, 4, hd,
                                           g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(), st) == 0

    def all_fused(x):
        assert L.dk_net_qkv_attn_ln_bf16_async(h.data_ptr(), x.data_ptr(), wq.data_ptr(), bq.data_ptr(), w.data_ptr(),
                                               b.data_ptr(), B, 4, hd, g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(),
                                               st) == 0

    res = {"d": d, "samples": B}
    outs = {}
    for name, fn in (("unfused", unfused), ("fused", fused), ("unfused2", unfused), ("fused2", fused),
                     ("qkv_gemm+fused", gemm_fused), ("qkv_fused", all_fused), ("qkv_gemm+fused2", gemm_fused),
                     ("qkv_fused2", all_fused)):
        x = x0.clone()
        fn(x)
        torch.cuda.synchronize()
        outs[name] = (x.clone(), out.clone())
        xs = [x0.clone() for _ in range(reps)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for i in range(reps):
            fn(xs[i])
        e1.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = round(e0.elapsed_time(e1) / reps, 4)
    res["max_abs_diff_x"] = (outs["fused"][0].float() - outs["unfused"][0].float()).abs().max().item()
    res["max_abs_diff_h"] = (outs["fused"][1].float() - outs["unfused"][1].float()).abs().max().item()
    res["qkv_max_abs_diff_x"] = (outs["qkv_fused"][0].float() - outs["qkv_gemm+fused"][0].float()).abs().max().item()
    res["qkv_max_abs_diff_h"] = (outs["qkv_fused"][1].float() - outs["qkv_gemm+fused"][1].float()).abs().max().item()
    return res


def main(argv):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    reps = int(argv[0]) if argv else 20
    cases = argv[1:] or ["160:8192", "160:740", "256:740", "256:2048", "256:8192"]
    for c in cases:
        d, B = (int(v) for v in c.split(":"))
        print(json.dumps(case(L, d, B, reps)), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
