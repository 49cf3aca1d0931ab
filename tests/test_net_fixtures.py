"""The networks' transformer block against the reference's own code: tests/golden/net_block_d*.npz
hold seeded weights, inputs and float32 outputs of rs-doko-py-bridge/python/TransformerBlock.py
(with SelfAttention.py) at d = 160 (AlphaZero) and d = 256 (IMPI), 4 heads, made by importing those
modules (tests/golden/make_net_fixtures.py).  CPU, float32 at matmul precision "highest".
The per-class attention heads (az_doko.py:28-55 / main.py:25-55) sit in modules that cannot be
imported here (tensorboardX, jaxtyping, the PyO3 bridge): they stay parity unpinned."""
import pytest
import torch

import net_fixtures as nf
from master_doko_reinforcement_learning_amd.az_network import Block


def _close(got, ref, base, tol):
    return (got - ref).abs().max().item() / (ref - base).abs().max().item() < tol


@pytest.mark.parametrize("d", [160, 256])
def test_block_matches_reference_fixture(d):
    """az_network.Block (load_reference: the reference state_dict names) reproduces the reference
    block's outputs: the first residual and the block output within 1e-5 of the residual scale."""
    sd, x, y_attn, y = nf.load(d)
    blk = Block(d, 4).eval()
    blk.load_reference(sd)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        with torch.no_grad():
            ya = x + blk.attn_delta(blk.ln_1(x))
            yo = blk(x)
    finally:
        torch.set_float32_matmul_precision(prev)
    assert _close(ya, y_attn, x, 1e-5) and _close(yo, y, y_attn, 1e-5)


@pytest.mark.parametrize("d", [160, 256])
def test_reference_structured_block_pinned(d):
    """RefStructBlock -- the block the whole-network structure tests (test_az_network.py,
    test_impi_network.py) build their reference networks from -- loads the reference state_dict
    strictly and reproduces the reference's outputs."""
    sd, x, y_attn, y = nf.load(d)
    blk = nf.RefStructBlock(d).eval()
    blk.load_state_dict(sd, strict=True)
    with torch.no_grad():
        yo = blk(x)
    assert _close(yo, y, y_attn, 1e-5)


def test_fixture_shapes():
    for d in (160, 256):
        sd, x, y_attn, y = nf.load(d)
        assert x.shape == y.shape == y_attn.shape == (3, 62, d)
        assert sd["attn.attn.in_proj_weight"].shape == (3 * d, d) and sd["mlp.c_fc.weight"].shape == (4 * d, d)
        assert torch.isfinite(y).all() and (y - y_attn).abs().max() > 0.05
