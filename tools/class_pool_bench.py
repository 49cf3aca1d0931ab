"""class_pool_ln_kernel at the C5 shapes (8,192 samples, d 160; 39 policy and 4 value classes):
event-timed launches and a hash of the output bytes (variants must agree bit for bit).
usage (GPU box): [DK_LIB=...] python tools/class_pool_bench.py"""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(reps=20):
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    dev = torch.device("cuda", 0)
    res = {}
    for d, B, C in ((160, 8192, 39), (160, 8192, 4), (256, 2048, 33)):
        torch.manual_seed(7)
        x = (torch.randn(B, 62, d, device=dev) * 2).bfloat16()
        q = torch.randn(C, d, device=dev).bfloat16()
        w = (1 + 0.1 * torch.randn(C, d, device=dev)).bfloat16()
        b = (0.1 * torch.randn(C, d, device=dev)).bfloat16()
        out = torch.empty(C, B, d, device=dev).bfloat16()
        st = torch.cuda.current_stream(dev).cuda_stream
        f = lambda: L.dk_net_class_pool_ln_bf16_async(x.data_ptr(), B, d, q.data_ptr(), C, d ** -0.5, w.data_ptr(),
                                                       b.data_ptr(), 1e-5, out.data_ptr(), st)
        assert f() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        h = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
        res["d%d_B%d_C%d" % (d, B, C)] = {"ms": e0.elapsed_time(e1) / reps, "sha1": h}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
