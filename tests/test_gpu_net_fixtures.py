"""The networks' fused block kernels against the reference's own transformer block: the fixtures
of tests/golden/net_block_d*.npz (seeded weights / inputs and float32 outputs of
rs-doko-py-bridge/python/TransformerBlock.py + SelfAttention.py, tests/golden/make_net_fixtures.py)
run through the product's trunk methods -- FusedTrunkF32 (qkv_attn_ln_f32x3 + mlp_ln_f32x3 /
mlp16_ln_f32x3, bf16x3 products) and FusedTrunk (the bf16 pair qkv_attn_ln + mlp_ln).
Bounds: f32 within 2e-5 of each half's residual-delta scale (the kernels' stated bound against
exact f32); bf16 within 2 % of the output scale (bf16 activations and weights)."""
import pytest
import torch
import torch.nn.functional as F

import net_fixtures as nf

pytestmark = pytest.mark.gpu


def _trunk(cls, rows, d, dev):
    from master_doko_reinforcement_learning_amd import _native
    f = cls.__new__(cls)
    f.L, f.st, f.rows, f.d = _native.lib(), torch.cuda.current_stream(dev).cuda_stream, rows, d
    return f


@pytest.mark.parametrize("d", [160, 256])
def test_f32_block_kernels_match_reference_fixture(d):
    from master_doko_reinforcement_learning_amd.az_network import Block, FusedTrunkF32
    dev = torch.device("cuda", 0)
    sd, x, y_attn, y = nf.load(d)
    blk = Block(d, 4).eval()
    blk.load_reference(sd)
    blk = blk.to(dev)
    x, y_attn, y = x.to(dev), y_attn.to(dev), y.to(dev)
    f = _trunk(FusedTrunkF32, x.shape[0] * x.shape[1], d, dev)
    with torch.no_grad():
        h = F.layer_norm(x, (d,), blk.ln_1.weight, blk.ln_1.bias, blk.ln_1.eps)
        xo = x.clone()
        h2 = f.attn_ln(xo, blk, h, blk.ln_2)                      # x += attn(ln_1 x); h2 = ln_2(x)
        torch.cuda.synchronize()
        ea = (xo - y_attn).abs().max().item() / (y_attn - x).abs().max().item()
        eh = (h2 - F.layer_norm(y_attn, (d,), blk.ln_2.weight, blk.ln_2.bias, 1e-5)).abs().max().item()
        h3 = f.mlp_ln(xo, blk, h2, blk.ln_1)                      # x += mlp(ln_2 x); h3 = ln_1(x)
        torch.cuda.synchronize()
    em = (xo - y).abs().max().item() / (y - y_attn).abs().max().item()
    assert torch.isfinite(h3).all()
    assert ea < 2e-5 and em < 2e-5 and eh < 1e-4, (ea, em, eh)


@pytest.mark.parametrize("d", [160, 256])
def test_bf16_block_kernels_match_reference_fixture(d):
    from master_doko_reinforcement_learning_amd.az_network import Block, FusedTrunk
    dev = torch.device("cuda", 0)
    sd, x, y_attn, y = nf.load(d)
    blk = Block(d, 4).eval()
    blk.load_reference(sd)
    blk = blk.to(dev).bfloat16()
    xb = x.to(dev).bfloat16()
    f = _trunk(FusedTrunk, x.shape[0] * x.shape[1], d, dev)
    with torch.no_grad():
        h = F.layer_norm(xb.float(), (d,), blk.ln_1.weight.float(), blk.ln_1.bias.float(), 1e-5).bfloat16()
        xo = xb.clone()
        h2 = f.attn_ln(xo, blk, h, blk.ln_2)
        f.mlp_ln(xo, blk, h2, blk.ln_1)
        torch.cuda.synchronize()
    e = (xo.float().cpu() - y).abs().max().item() / y.abs().max().item()
    assert e < 0.02, e
