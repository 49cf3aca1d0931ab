"""Loader of the reference transformer-block fixtures (tests/golden/net_block_d*.npz, written by
tests/golden/make_net_fixtures.py from the reference's own TransformerBlock.py / SelfAttention.py),
and RefStructBlock: the reference block's structure and state_dict names as a plain torch module,
which tests/test_net_fixtures.py pins to those fixtures (the whole-network structure tests build
their reference-structured networks from it).  Test infrastructure only."""
import os

import numpy as np
import torch
from torch import nn

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(d):
    """(state_dict of float32 tensors, x, y_attn, y) of the d-wide fixture block."""
    z = np.load(os.path.join(GOLD, "net_block_d%d.npz" % d))   # allow_pickle stays False
    sd = {}
    for k in z.files:
        if not k.startswith("w/"):
            continue
        name = k[2:]
        v = z[k].astype(np.float64) * 2.0 ** -int(z["e/" + name])
        if name.startswith("ln_") and name.endswith("weight"):
            v = 1.0 + v
        sd[name] = torch.from_numpy(v.astype(np.float32))
    x = torch.from_numpy(z["x"].astype(np.float32) * 2.0 ** -5)
    return sd, x, torch.from_numpy(z["y_attn"]), torch.from_numpy(z["y"])


class _Cfg:
    def __init__(self, d, heads=4):
        self.n_embd, self.n_head = d, heads


class _SelfAttention(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.attn = nn.MultiheadAttention(c.n_embd, c.n_head, dropout=0.0, batch_first=True)
        self.c_proj = nn.Linear(c.n_embd, c.n_embd)

    def forward(self, x):
        return self.c_proj(self.attn(x, x, x)[0])


class RefStructBlock(nn.Module):
    """TransformerBlock.py:5-27's structure at inference (dropout inactive)."""

    def __init__(self, d, heads=4):
        super().__init__()
        c = _Cfg(d, heads)
        self.ln_1 = nn.LayerNorm(d)
        self.attn = _SelfAttention(c)
        self.ln_2 = nn.LayerNorm(d)
        self.mlp = nn.ModuleDict(dict(c_fc=nn.Linear(d, 4 * d), c_proj=nn.Linear(4 * d, d)))

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp.c_proj(nn.functional.gelu(self.mlp.c_fc(self.ln_2(x))))
