"""What an f32 GEMM costs and computes on this box under each torch matmul precision.

The reference network runs f32 activations with torch.set_float32_matmul_precision("medium")
and allow_tf32 (az_doko.py:539-541, main.py:402/508): TF32-class products on CUDA.  gfx950 has
no xf32 MFMA; this probe times the networks' GEMM shapes at "highest" / "high" / "medium" and
measures the error against f64, so DESIGN.md can say which compute type hipBLASLt picked.
"""
import json
import sys

import torch


def main():
    dev = torch.device("cuda", 0)
    shapes = [(507904, 160, 640), (507904, 640, 160), (507904, 160, 480), (196608, 256, 1024), (196608, 1024, 256)]
    out = []
    g = torch.Generator(device=dev).manual_seed(0)
    for m, k, n in shapes:
        a = torch.randn((m, k), device=dev, generator=g)
        b = torch.randn((n, k), device=dev, generator=g) / k ** 0.5
        ref = (a[:4096].double() @ b.double().t())
        for prec in ("highest", "high", "medium"):
            torch.set_float32_matmul_precision(prec)
            y = a @ b.t()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                y = a @ b.t()
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / 10
            err = ((y[:4096].double() - ref).abs().max() / ref.abs().max()).item()
            out.append({"m": m, "k": k, "n": n, "precision": prec, "ms": ms, "tflops": 2 * m * k * n / ms / 1e9,
                        "max_rel_err_vs_f64": err})
            print(json.dumps(out[-1]), flush=True)
        for dt in (torch.bfloat16,):
            ab, bb = a.to(dt), b.to(dt)
            y = ab @ bb.t()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                y = ab @ bb.t()
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / 10
            err = ((y[:4096].double() - ref).abs().max() / ref.abs().max()).item()
            out.append({"m": m, "k": k, "n": n, "precision": "bf16", "ms": ms, "tflops": 2 * m * k * n / ms / 1e9,
                        "max_rel_err_vs_f64": err})
            print(json.dumps(out[-1]), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
