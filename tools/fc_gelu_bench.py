"""Time dk_net_fc_gelu_bf16_async against hipBLASLt F.linear + F.gelu on the networks' MLP shapes."""
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from master_doko_reinforcement_learning_amd import _native


def main():
    dev = torch.device("cuda", 0)
    L = _native.lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    for rows, k, n in ((8192 * 62, 160, 640), (24576 * 62, 256, 1024)):
        x = torch.randn(rows, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / k ** 0.5).bfloat16()
        b = torch.zeros(n, device=dev).bfloat16()
        y = torch.empty(rows, n, device=dev).bfloat16()

        def fused():
            assert L.dk_net_fc_gelu_bf16_async(x.data_ptr(), w.data_ptr(), b.data_ptr(), rows, k, n, y.data_ptr(), st) == 0

        def unfused():
            return F.gelu(F.linear(x, w, b))

        for name, fn in (("torch", unfused), ("fused", fused), ("torch", unfused), ("fused", fused)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 20 * 1e3
            print("rows %d k %d n %d %s %.3f ms (%.0f TFLOP/s, %.2f TB/s out)" % (
                rows, k, n, name, ms, 2.0 * rows * k * n / ms / 1e9, rows * n * 2 / ms / 1e9), flush=True)
        ref = F.gelu(F.linear(x.float(), w.float(), b.float()))
        fused()
        torch.cuda.synchronize()
        print("max abs err %.4f" % (y.float() - ref).abs().max().item())


if __name__ == "__main__":
    main()
