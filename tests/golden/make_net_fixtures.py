"""Golden vectors of the reference's transformer block (TEST INFRASTRUCTURE; run in the build
container, where /root/reference exists -- the GPU box and the tests never read it).

Imports the reference's own modules, rs-doko-py-bridge/python/TransformerBlock.py:5-27 and
SelfAttention.py:4-36 (they import only torch), builds TransformerBlock(config) for the two
network widths this repository runs -- d = 160 (AlphaZero, az_doko.py:62-75: n_embd 160, n_head 4)
and d = 256 (IMPI, create_ar.py: n_embd 256, n_head 4) -- with seeded weights, puts it in eval()
mode (the reference's dropout 0.1 is inactive at inference) and evaluates it in float32 on the CPU
at matmul precision "highest".

Weights and inputs are small integers times powers of two (int8 x 2^-e, exact in f32), so the
fixture stores them as int8 with their exponent; the outputs are stored as float32:
    tests/golden/net_block_d{160,256}.npz
        w/<state_dict name>  int8,   e/<state_dict name>  exponent (value = w * 2^-e; LayerNorm
                                     weights are 1 + w * 2^-e)
        x                    int8 [B, 62, d] (x = x_int * 2^-5)
        y_attn               float32: x + attn(ln_1(x))          (the block's first residual)
        y                    float32: the block's output
Usage:  python tests/golden/make_net_fixtures.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/rs-doko-py-bridge/python"
SEQ, B = 62, 3


class Config:   # the fields TransformerBlock / SelfAttention read (az_doko.py:62-75)
    def __init__(self, d):
        self.n_embd, self.n_head, self.attn_pdrop, self.resid_pdrop = d, 4, 0.1, 0.1


def quantised(shape, fan_in, g, ln=False):
    """int8 values and exponent e with value = w * 2^-e (~ the default uniform init's scale)."""
    e = int(round(np.log2(127 * np.sqrt(fan_in)))) if not ln else 9
    w = g.integers(-127, 128, size=shape, dtype=np.int64).astype(np.int8)
    return w, e


def main():
    sys.path.insert(0, REF)
    from TransformerBlock import TransformerBlock   # the reference's own code
    torch.set_float32_matmul_precision("highest")
    for d in (160, 256):
        g = np.random.default_rng(1600 + d)
        blk = TransformerBlock(Config(d)).eval()
        out = {}
        sd = {}
        for name, p in blk.state_dict().items():
            is_ln = name.startswith("ln_")
            fan_in = p.shape[-1] if p.dim() == 2 else d
            w, e = quantised(tuple(p.shape), fan_in, g, ln=is_ln)
            if name.endswith("bias"):
                e = 10
            val = w.astype(np.float64) * 2.0 ** -e
            if is_ln and name.endswith("weight"):
                val = 1.0 + val
            sd[name] = torch.from_numpy(val.astype(np.float32))
            out["w/" + name] = w
            out["e/" + name] = np.int32(e)
        blk.load_state_dict(sd)
        xi = np.clip(np.round(g.standard_normal((B, SEQ, d)) * 32), -127, 127).astype(np.int8)
        x = torch.from_numpy(xi.astype(np.float32) * 2.0 ** -5)
        with torch.no_grad():
            y_attn = x + blk.attn(blk.ln_1(x))
            y = blk(x)
        out["x"] = xi
        out["y_attn"] = y_attn.numpy().astype(np.float32)
        out["y"] = y.numpy().astype(np.float32)
        path = os.path.join(HERE, "net_block_d%d.npz" % d)
        np.savez_compressed(path, **out)
        print("wrote", path, "params", sum(v.size for k, v in out.items() if k.startswith("w/")))


if __name__ == "__main__":
    main()
