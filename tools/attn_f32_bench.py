"""The f32 attention core (dk_net_attn62_f32_async) at the C5 / IMPI shapes: event-timed launches
and the max difference against torch at full f32.  usage (GPU box): python tools/attn_f32_bench.py"""
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
    out = {}
    for hd, B in ((40, 8192), (64, 740), (64, 8192)):
        torch.manual_seed(5)
        d = 4 * hd
        qkv = torch.randn(B, 62, 3 * d, device=dev) * 1.5
        y = torch.empty(B, 62, d, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        f = lambda: L.dk_net_attn62_f32_async(qkv.data_ptr(), y.data_ptr(), B, 4, hd, st)
        assert f() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        q, k, v = qkv[:64].double().view(64, 62, 3, 4, hd).permute(2, 0, 3, 1, 4)
        ref = (torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1) @ v).transpose(1, 2).reshape(64, 62, d)
        err = (y[:64].double() - ref).abs().max().item()
        flop = 4.0 * B * 4 * 62 * 62 * hd
        out["hd%d_B%d" % (hd, B)] = {"ms": ms, "tflops": flop / ms / 1e9, "max_abs_err": err}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
