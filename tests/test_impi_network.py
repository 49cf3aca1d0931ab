"""IMPI network (impi_network.DokoImpiNet) against a plain-PyTorch fp32 module with the
reference's structure and state_dict names (rs-doko-py-bridge/python/main.py:25-138,
TransformerBlock.py, SelfAttention.py): identical logits after load_reference_state_dict.
CPU only."""
import torch
from torch import nn

from master_doko_reinforcement_learning_amd.impi_network import VOCAB_IPI, DokoImpiNet
from test_az_network import _Block, _Head


class _Cfg:
    n_embd, n_head, attn_pdrop, resid_pdrop = 32, 4, 0.0, 0.0


class _RefImpiNet(nn.Module):
    def __init__(self, c, layers=2):
        super().__init__()
        d = c.n_embd
        names = ["game_object_e", "position_e", "player_played_e", "subposition_e", "team_e", "player_guess_e"]
        mods = {n: nn.Embedding(v, d) for n, v in zip(names, VOCAB_IPI)}
        mods.update(h=nn.ModuleList([_Block(c) for _ in range(layers)]), ln_f=nn.LayerNorm(d))
        self.transformer = nn.ModuleDict(mods)
        self.lm_head = _Head(d, 33)

    def forward(self, x):
        t = self.transformer
        h = (t.game_object_e(x[:, 0:62]) + t.position_e(x[:, 62:124]) + t.player_played_e(x[:, 124:186]) +
             t.subposition_e(x[:, 186:248]) + t.team_e(x[:, 248:310]) + t.player_guess_e(x[:, 310:311]).expand(-1, 62, -1))
        for b in t.h:
            h = b(h)
        return self.lm_head(t.ln_f(h))


def _tokens(n, seed):
    g = torch.Generator().manual_seed(seed)
    parts = [torch.randint(0, v, (n, 62 if i < 5 else 1), generator=g) for i, v in enumerate(VOCAB_IPI)]
    return torch.cat(parts, dim=1)


def test_impi_network_matches_reference_structure():
    torch.manual_seed(0)
    ref = _RefImpiNet(_Cfg()).eval()
    net = DokoImpiNet(d=32, heads=4, layers=2).eval()
    net.load_reference_state_dict(ref.state_dict())
    x = _tokens(8, 3)
    with torch.no_grad():
        l0 = ref(x)
        l1 = net(x.int())
    assert l1.shape == (8, 33)
    torch.testing.assert_close(l1, l0, rtol=1e-4, atol=1e-5)


def test_default_impi_network_shapes():
    """create_ar.py:12-18: n_embd 256, 4 layers, 4 heads."""
    net = DokoImpiNet().eval()
    n_params = sum(p.numel() for p in net.parameters())
    assert 3.0e6 < n_params < 8.0e6
    with torch.no_grad():
        p = net(_tokens(3, 4))
    assert p.shape == (3, 33) and torch.isfinite(p).all()
