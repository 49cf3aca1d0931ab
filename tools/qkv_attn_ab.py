"""A/B of the attention half (dk_net_qkv_attn_ln_bf16_async, or with f32 as the sixth argument
dk_net_qkv_attn_ln_f32x3_async) between two builds of the library loaded into one process,
alternated launch by launch on the same inputs (HIP events); prints medians and the max output
difference between the builds.
usage (GPU box): python tools/qkv_attn_ab.py libA.so libB.so [d] [samples] [reps] [bf16|f32]"""
import ctypes
import sys

import torch


def main(lib_a, lib_b, d=160, B=8192, reps=30, prec="bf16"):
    d, B, reps = int(d), int(B), int(reps)
    if prec == "f32":
        return main_f32(lib_a, lib_b, d, B, reps)
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    libs = []
    for p in (lib_a, lib_b):
        L = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        f = L.dk_net_qkv_attn_ln_bf16_async
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        f.argtypes = [vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp, ctypes.c_float, vp, vp]
        f.restype = ctypes.c_int
        libs.append(f)
    torch.manual_seed(3)
    h = torch.randn(B, 62, d, device=dev).bfloat16()
    x0 = (torch.randn(B, 62, d, device=dev) * 2).bfloat16()
    wq = (torch.randn(3 * d, d, device=dev) / d ** 0.5).bfloat16()
    bq = (torch.randn(3 * d, device=dev) * 0.1).bfloat16()
    wp = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
    bp = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = torch.ones(d, device=dev).bfloat16()
    be = torch.zeros(d, device=dev).bfloat16()
    st = torch.cuda.current_stream(dev).cuda_stream
    xs = [x0.clone(), x0.clone()]
    outs = [torch.empty_like(x0), torch.empty_like(x0)]

    def run(i):
        xs[i].copy_(x0)
        assert libs[i](h.data_ptr(), xs[i].data_ptr(), wq.data_ptr(), bq.data_ptr(), wp.data_ptr(), bp.data_ptr(), B, 4,
                       d // 4, g.data_ptr(), be.data_ptr(), 1e-5, outs[i].data_ptr(), st) == 0

    run(0); run(1)
    torch.cuda.synchronize()
    dx = (xs[0].float() - xs[1].float()).abs().max().item()
    dh = (outs[0].float() - outs[1].float()).abs().max().item()
    times = [[], []]
    for r in range(reps):
        for i in ((0, 1) if r % 2 == 0 else (1, 0)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            xs[i].copy_(x0)
            e0.record()
            assert libs[i](h.data_ptr(), xs[i].data_ptr(), wq.data_ptr(), bq.data_ptr(), wp.data_ptr(), bp.data_ptr(), B, 4,
                           d // 4, g.data_ptr(), be.data_ptr(), 1e-5, outs[i].data_ptr(), st) == 0
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1))
    for i, name in enumerate(("A", "B")):
        v = sorted(times[i])
        print("%s %s: median %.4f ms min %.4f ms" % (name, (lib_a, lib_b)[i].split("/")[-1], v[len(v) // 2], v[0]))
    print("max |x_A - x_B| %.3g, max |h_A - h_B| %.3g" % (dx, dh))


def main_f32(lib_a, lib_b, d, B, reps):
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    libs = []
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    for p in (lib_a, lib_b):
        f = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL).dk_net_qkv_attn_ln_f32x3_async
        f.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp, ctypes.c_float, vp, vp]
        f.restype = ctypes.c_int
        libs.append(f)
    torch.manual_seed(3)
    h = torch.randn(B, 62, d, device=dev)
    x0 = torch.randn(B, 62, d, device=dev) * 2
    wq, bq = torch.randn(3 * d, d, device=dev) / d ** 0.5, torch.randn(3 * d, device=dev) * 0.1
    wp, bp = torch.randn(d, d, device=dev) / d ** 0.5, torch.randn(d, device=dev) * 0.1
    sp = []
    for w in (wq, wp):
        hi = w.bfloat16().contiguous()
        sp += [hi, (w - hi.float()).bfloat16().contiguous()]
    g, be = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    xs = [x0.clone(), x0.clone()]
    outs = [torch.empty_like(x0), torch.empty_like(x0)]

    def run(i):
        xs[i].copy_(x0)
        assert libs[i](h.data_ptr(), xs[i].data_ptr(), sp[0].data_ptr(), sp[1].data_ptr(), bq.data_ptr(), sp[2].data_ptr(),
                       sp[3].data_ptr(), bp.data_ptr(), B, 4, d // 4, g.data_ptr(), be.data_ptr(), 1e-5,
                       outs[i].data_ptr(), st) == 0

    run(0); run(1)
    torch.cuda.synchronize()
    dh = (outs[0] - outs[1]).abs().max().item()
    times = [[], []]
    for r in range(reps):
        for i in ((0, 1) if r % 2 == 0 else (1, 0)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(i)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1))
    for i, name in enumerate(("A", "B")):
        v = sorted(times[i])
        print("%s %s f32 d %d: median %.4f ms min %.4f ms (incl. the x reset copy)" % (name, (lib_a, lib_b)[i].split("/")[-1], d, v[len(v) // 2], v[0]))
    print("max |h_A - h_B| %.3g" % dh)


if __name__ == "__main__":
    main(*sys.argv[1:])
