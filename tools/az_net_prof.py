"""Per-op GPU time of one DokoAzNet forward (bf16) at the C5 batch, via torch.profiler.
Usage (GPU box): python tools/az_net_prof.py [batch]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from master_doko_reinforcement_learning_amd.az_network import VOCAB, DokoAzNet  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    dev = torch.device("cuda", 0)
    net = DokoAzNet().to(dev).eval().to(torch.bfloat16)
    tok = torch.cat([torch.randint(0, v, (B, 62 if i < 5 else 1), device=dev) for i, v in enumerate(VOCAB)], 1).int()
    with torch.inference_mode():
        for _ in range(3):
            net(tok)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            net(tok)
        torch.cuda.synchronize()
        print("forward ms", (time.perf_counter() - t0) / 5 * 1e3, "batch", B)
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            net(tok)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))


if __name__ == "__main__":
    main()
