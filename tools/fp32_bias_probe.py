"""hipBLASLt f32 GEMMs of the networks at matmul precision "medium": F.linear with the bias in the
GEMM epilogue against the GEMM alone (the bias then added by the next f32 row kernel).
usage (GPU box): python tools/fp32_bias_probe.py"""
import json

import torch
import torch.nn.functional as F


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    torch.set_float32_matmul_precision("medium")
    torch.backends.cuda.matmul.allow_tf32 = True
    out = []
    for m, k, n in ((507904, 160, 480), (507904, 160, 160), (507904, 160, 640), (507904, 640, 160),
                    (196608, 256, 768), (196608, 256, 1024), (196608, 1024, 256)):
        x = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) / k ** 0.5
        b = torch.randn(n, device=dev)
        r = {"m": m, "k": k, "n": n,
             "linear_bias_ms": t(lambda: F.linear(x, w, b)),
             "linear_nobias_ms": t(lambda: F.linear(x, w)),
             "matmul_ms": t(lambda: x @ w.t())}
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
