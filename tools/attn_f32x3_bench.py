"""The f32 attention half of a block: qkv_attn_ln_f32x3_kernel (one pass per sample, bf16x3
products) against the unfused f32 path (hipBLASLt qkv F.linear at matmul precision "medium" +
attn62_bias_f32 (f32 MFMA) + F.linear of the folded projection + add_bias_ln_f32), alternated.
usage: python tools/attn_f32x3_bench.py [samples] [reps] [d]  (d = 160 or 256, four heads)"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(B=8192, reps=20, d=160):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H = 4
    hd = d // H
    h = torch.randn(B, 62, d, device=dev)
    x = torch.randn(B, 62, d, device=dev)
    wq, bq = torch.randn(3 * d, d, device=dev) / d ** 0.5, torch.randn(3 * d, device=dev) * 0.1
    wp, bp = torch.randn(d, d, device=dev) / d ** 0.5, torch.randn(d, device=dev) * 0.1
    g, be = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    sp = []
    for w in (wq, wp):
        hi = w.bfloat16().contiguous()
        sp += [hi, (w - hi.float()).bfloat16().contiguous()]
    st = torch.cuda.current_stream(dev).cuda_stream
    torch.set_float32_matmul_precision("medium")
    out = torch.empty_like(x)

    def fused():
        assert L.dk_net_qkv_attn_ln_f32x3_async(h.data_ptr(), x.data_ptr(), sp[0].data_ptr(), sp[1].data_ptr(), bq.data_ptr(),
                                                sp[2].data_ptr(), sp[3].data_ptr(), bp.data_ptr(), B, H, hd, g.data_ptr(),
                                                be.data_ptr(), 1e-5, out.data_ptr(), st) == 0

    def unfused():
        qkv = F.linear(h, wq)
        y = torch.empty_like(h)
        assert L.dk_net_attn62_bias_f32_async(qkv.data_ptr(), bq.data_ptr(), y.data_ptr(), B, H, hd, st) == 0
        dl = F.linear(y, wp)
        assert L.dk_net_add_bias_ln_f32_async(x.data_ptr(), dl.data_ptr(), bp.data_ptr(), B * 62, d, g.data_ptr(),
                                              be.data_ptr(), 1e-5, out.data_ptr(), st) == 0

    res = {"fused": [], "unfused": []}
    fused(); unfused()
    torch.cuda.synchronize()
    for r in range(reps):
        for name, fn in ((("fused", fused), ("unfused", unfused)) if r % 2 == 0 else (("unfused", unfused), ("fused", fused))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
    for name, v in res.items():
        v = sorted(v)
        print("%-8s samples %d: median %.3f ms min %.3f ms" % (name, B, v[len(v) // 2], v[0]))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
