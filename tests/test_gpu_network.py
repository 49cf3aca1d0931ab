"""GPU numerics of the AlphaZero network's fused row kernels (csrc/az_net_kernels.h)
against plain PyTorch fp32 references of the same ops."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from master_doko_reinforcement_learning_amd import _native
    return _native.lib()


@pytest.mark.parametrize("d", [160, 64, 256])
def test_add_ln_matches_torch(d):
    dev = torch.device("cuda", 0)
    torch.manual_seed(d)
    rows = 62 * 129
    x = (torch.randn(rows, d, device=dev) * 3 + 0.5).bfloat16()
    delta = torch.randn(rows, d, device=dev).bfloat16()
    g = (1 + 0.1 * torch.randn(d, device=dev)).bfloat16()
    b = (0.1 * torch.randn(d, device=dev)).bfloat16()
    x_ref = (x.float() + delta.float()).bfloat16()
    h_ref = F.layer_norm(x_ref.float(), (d,), g.float(), b.float(), 1e-5)
    h = torch.empty_like(x)
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = _lib().dk_net_add_ln_bf16_async(x.data_ptr(), delta.data_ptr(), rows, d, g.data_ptr(), b.data_ptr(), 1e-5,
                                         h.data_ptr(), st)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(x, x_ref)                                  # the residual add rounds like torch's bf16 add
    torch.testing.assert_close(h.float(), h_ref, rtol=1e-2, atol=2e-2)   # bf16 output of an f32 LayerNorm


@pytest.mark.parametrize("d,n", [(160, 640), (256, 1024)])
def test_mlp_ln_f32x3_matches_torch(d, n):
    """The f32 MLP half with bf16x3 products (mlp_ln_f32x3_kernel): x += proj(GELU(fc(h))) + b,
    h' = LN'(x), against exact f32 torch (matmul precision "highest") on f32 inputs: within 2e-5
    of the output scale (bf16x3 products carry ~16 bits; hipBLASLt at "medium" measured ~5e-6
    relative per GEMM, profiles/r04/fp32_gemm_probe.json)."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(11)
    rows = 62 * 41 + 3                                   # not a multiple of the 128-row workgroup tile
    h = torch.randn(rows, d, device=dev)
    x = torch.randn(rows, d, device=dev) * 2
    w1 = torch.randn(n, d, device=dev) / d ** 0.5
    b1 = torch.randn(n, device=dev) * 0.1
    w2 = torch.randn(d, n, device=dev) / n ** 0.5
    b2 = torch.randn(d, device=dev) * 0.1
    g = 1 + 0.1 * torch.randn(d, device=dev)
    be = 0.1 * torch.randn(d, device=dev)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        delta_ref = F.linear(F.gelu(F.linear(h, w1, b1)), w2, b2)
    finally:
        torch.set_float32_matmul_precision(prev)
    x_ref = x + delta_ref
    h_ref = F.layer_norm(x_ref, (d,), g, be, 1e-5)
    from master_doko_reinforcement_learning_amd.az_network import mlp_split_bf16x3
    split = mlp_split_bf16x3(w1, w2)
    xo = x.clone()
    out = torch.full((rows, d), float("nan"), device=dev)
    rc = _lib().dk_net_mlp_ln_f32x3_async(h.data_ptr(), xo.data_ptr(), split[0].data_ptr(), split[1].data_ptr(),
                                          b1.data_ptr(), split[2].data_ptr(), split[3].data_ptr(), b2.data_ptr(), rows,
                                          d, n, g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(),
                                          torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out).all() and torch.isfinite(xo).all()
    ex = (xo - x_ref).abs().max().item() / delta_ref.abs().max().item()
    eh = (out - h_ref).abs().max().item() / h_ref.abs().max().item()
    assert ex < 2e-5 and eh < 2e-5, (ex, eh)


@pytest.mark.parametrize("d", [256, 160])
@pytest.mark.parametrize("write_h", [False, True])
def test_ex_halves_normalise_x_input(write_h, d):
    """The halves with the LayerNorm in the consumer (dk_net_*_f32x3_ex_async, h_in NULL; d = 256:
    round 5, d = 160: round 6): each against exact f32 torch on LN_in(x) (matmul precision
    "highest"): x' within 2e-5 of the delta scale; h_out NULL leaves its buffer untouched, otherwise
    h' = LN(x') within 2e-5."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(17 + d)
    n, B, H = 4 * d, 29, 4
    hd = d // H
    x = torch.randn(B, 62, d, device=dev) * 2 + 0.5
    gi, bi = 1 + 0.1 * torch.randn(d, device=dev), 0.1 * torch.randn(d, device=dev)
    g, be = 1 + 0.1 * torch.randn(d, device=dev), 0.1 * torch.randn(d, device=dev)
    wq, bq = torch.randn(3 * d, d, device=dev) / d ** 0.5, torch.randn(3 * d, device=dev) * 0.1
    wp, bp = torch.randn(d, d, device=dev) / d ** 0.5, torch.randn(d, device=dev) * 0.1
    w1, b1 = torch.randn(n, d, device=dev) / d ** 0.5, torch.randn(n, device=dev) * 0.1
    w2, b2 = torch.randn(d, n, device=dev) / n ** 0.5, torch.randn(d, device=dev) * 0.1
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        h = F.layer_norm(x, (d,), gi, bi, 1e-5)
        qkv = F.linear(h, wq, bq)
        q, k, v = (qkv[..., i * d:(i + 1) * d].reshape(B, 62, H, hd).transpose(1, 2) for i in range(3))
        p = torch.softmax((q @ k.transpose(-1, -2)) / hd ** 0.5, dim=-1)
        da = F.linear((p @ v).transpose(1, 2).reshape(B, 62, d), wp, bp)
        xa = x + da
        dm = F.linear(F.gelu(F.linear(F.layer_norm(xa, (d,), gi, bi, 1e-5), w1, b1)), w2, b2)
        xm = xa + dm
    finally:
        torch.set_float32_matmul_precision(prev)
    sp = []
    for w in (wq, wp):
        hi = w.bfloat16().contiguous()
        sp += [hi, (w - hi.float()).bfloat16().contiguous()]
    from master_doko_reinforcement_learning_amd.az_network import mlp_split_bf16x3
    sm = mlp_split_bf16x3(w1, w2)
    st = torch.cuda.current_stream(dev).cuda_stream
    xo = x.clone()
    ha = torch.full_like(x, float("nan"))
    hm = torch.full_like(x, float("nan"))
    L = _lib()
    # d = 160: the attention half hands the MLP half the new rows' LayerNorm statistics
    stats = torch.full((B * 62, 2), float("nan"), device=dev) if d == 160 else None
    sptr = stats.data_ptr() if stats is not None else None
    assert L.dk_net_qkv_attn_ln_f32x3_ex_async(None, xo.data_ptr(), gi.data_ptr(), bi.data_ptr(), 1e-5, sp[0].data_ptr(),
                                               sp[1].data_ptr(), bq.data_ptr(), sp[2].data_ptr(), sp[3].data_ptr(),
                                               bp.data_ptr(), B, H, hd, g.data_ptr() if write_h else None,
                                               be.data_ptr() if write_h else None, 1e-5,
                                               ha.data_ptr() if write_h else None, None, sptr, None, st) == 0
    torch.cuda.synchronize()
    xa_got = xo.clone()
    # x_out: the same half from the same x into another buffer, x left as it was
    xsrc, xdst = x.clone(), torch.full_like(x, float("nan"))
    assert L.dk_net_qkv_attn_ln_f32x3_ex_async(None, xsrc.data_ptr(), gi.data_ptr(), bi.data_ptr(), 1e-5, sp[0].data_ptr(),
                                               sp[1].data_ptr(), bq.data_ptr(), sp[2].data_ptr(), sp[3].data_ptr(),
                                               bp.data_ptr(), B, H, hd, None, None, 1e-5, None, None, None,
                                               xdst.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(xsrc, x) and torch.equal(xdst, xa_got)
    assert L.dk_net_mlp_ln_f32x3_ex_async(None, xo.data_ptr(), gi.data_ptr(), bi.data_ptr(), 1e-5, sm[0].data_ptr(),
                                          sm[1].data_ptr(), b1.data_ptr(), sm[2].data_ptr(), sm[3].data_ptr(), b2.data_ptr(),
                                          B * 62, d, n, g.data_ptr() if write_h else None,
                                          be.data_ptr() if write_h else None, 1e-5, hm.data_ptr() if write_h else None,
                                          sptr, None, st) == 0
    torch.cuda.synchronize()
    ea = (xa_got - xa).abs().max().item() / da.abs().max().item()
    em = (xo - xm).abs().max().item() / dm.abs().max().item()
    assert ea < 2e-5 and em < 2e-5, (ea, em)
    if stats is not None:   # the statistics the attention half wrote: those of x' = xa
        mu = xa.reshape(-1, d).mean(-1)
        rs = torch.rsqrt(xa.reshape(-1, d).var(-1, unbiased=False) + 1e-5)
        assert torch.allclose(stats[:, 0], mu, rtol=1e-5, atol=1e-5) and torch.allclose(stats[:, 1], rs, rtol=1e-5)
    if write_h:
        for got, xr in ((ha, xa), (hm, xm)):
            ref = F.layer_norm(xr, (d,), g, be, 1e-5)
            assert (got - ref).abs().max().item() / ref.abs().max().item() < 2e-5
    else:
        assert torch.isnan(ha).all() and torch.isnan(hm).all()
    # the invalid forms: neither h_in nor ln_in; h_out aliasing x; d = 160 with h given (its halves
    # exist only in the x-input form); a width without kernels
    assert L.dk_net_mlp_ln_f32x3_ex_async(None, xo.data_ptr(), None, None, 1e-5, sm[0].data_ptr(), sm[1].data_ptr(),
                                          b1.data_ptr(), sm[2].data_ptr(), sm[3].data_ptr(), b2.data_ptr(), B * 62, d, n,
                                          None, None, 1e-5, None, sptr, None, st) != 0
    assert L.dk_net_qkv_attn_ln_f32x3_ex_async(None, xo.data_ptr(), gi.data_ptr(), bi.data_ptr(), 1e-5, sp[0].data_ptr(),
                                               sp[1].data_ptr(), bq.data_ptr(), sp[2].data_ptr(), sp[3].data_ptr(),
                                               bp.data_ptr(), B, H, hd, g.data_ptr(), be.data_ptr(), 1e-5, xo.data_ptr(),
                                               None, None, None, st) != 0
    hdummy = torch.zeros_like(x)
    assert L.dk_net_mlp_ln_f32x3_ex_async(hdummy.data_ptr(), xo.data_ptr(), None, None, 1e-5, sm[0].data_ptr(),
                                          sm[1].data_ptr(), b1.data_ptr(), sm[2].data_ptr(), sm[3].data_ptr(), b2.data_ptr(),
                                          B * 62, 160, 640, None, None, 1e-5, None, sptr, None, st) != 0
    assert L.dk_net_mlp_ln_f32x3_ex_async(None, xo.data_ptr(), gi.data_ptr(), bi.data_ptr(), 1e-5, sm[0].data_ptr(),
                                          sm[1].data_ptr(), b1.data_ptr(), sm[2].data_ptr(), sm[3].data_ptr(), b2.data_ptr(),
                                          B * 62, 192, 768, None, None, 1e-5, None, None, None, st) != 0
    # the MLP half at d = 160 needs the statistics; at d = 256 none are accepted
    assert L.dk_net_mlp_ln_f32x3_ex_async(None, xo.data_ptr(), gi.data_ptr(), bi.data_ptr(), 1e-5, sm[0].data_ptr(),
                                          sm[1].data_ptr(), b1.data_ptr(), sm[2].data_ptr(), sm[3].data_ptr(), b2.data_ptr(),
                                          B * 62, d, n, None, None, 1e-5, None, None if d == 160 else xo.data_ptr(), None,
                                          st) != 0


@pytest.mark.parametrize("d", [160, 256])
def test_qkv_attn_ln_f32x3_matches_torch(d):
    """The f32 attention half with bf16x3 products (qkv_attn_ln_f32x3_kernel, d = 160 / 256, 4 heads of 40 / 64):
    x += (softmax(q k^T / sqrt(40)) v) Wp^T + bp, h' = LN(x), against exact f32 torch (matmul
    precision "highest"): within 2e-5 of the output scale."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(13)
    B, H = 37, 4
    hd = d // H
    h = torch.randn(B, 62, d, device=dev)
    x = torch.randn(B, 62, d, device=dev) * 2
    wq, bq = torch.randn(3 * d, d, device=dev) / d ** 0.5, torch.randn(3 * d, device=dev) * 0.1
    wp, bp = torch.randn(d, d, device=dev) / d ** 0.5, torch.randn(d, device=dev) * 0.1
    g, be = 1 + 0.1 * torch.randn(d, device=dev), 0.1 * torch.randn(d, device=dev)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        qkv = F.linear(h, wq, bq)
        q, k, v = (qkv[..., i * d:(i + 1) * d].reshape(B, 62, H, hd).transpose(1, 2) for i in range(3))
        p = torch.softmax((q @ k.transpose(-1, -2)) / hd ** 0.5, dim=-1)
        y = (p @ v).transpose(1, 2).reshape(B, 62, d)
        delta = F.linear(y, wp, bp)
    finally:
        torch.set_float32_matmul_precision(prev)
    x_ref = x + delta
    h_ref = F.layer_norm(x_ref, (d,), g, be, 1e-5)
    sp = []
    for w in (wq, wp):
        hi = w.bfloat16().contiguous()
        sp += [hi, (w - hi.float()).bfloat16().contiguous()]
    xo = x.clone()
    out = torch.full_like(x, float("nan"))
    rc = _lib().dk_net_qkv_attn_ln_f32x3_async(h.data_ptr(), xo.data_ptr(), sp[0].data_ptr(), sp[1].data_ptr(), bq.data_ptr(),
                                               sp[2].data_ptr(), sp[3].data_ptr(), bp.data_ptr(), B, H, hd, g.data_ptr(),
                                               be.data_ptr(), 1e-5, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out).all() and torch.isfinite(xo).all()
    ex = (xo - x_ref).abs().max().item() / delta.abs().max().item()
    eh = (out - h_ref).abs().max().item() / h_ref.abs().max().item()
    assert ex < 2e-5 and eh < 2e-5, (ex, eh)


@pytest.mark.parametrize("hd", [40, 64])
def test_attn62_matches_torch(hd):
    """MFMA attention core (62 tokens, 4 heads x hd) against fp32 softmax(q k^T / sqrt(hd)) v."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    B, d = 77, 4 * hd
    qkv = (torch.randn(B, 62, 3 * d, device=dev) * 1.5).bfloat16()
    y = torch.full((B, 62, d), float("nan"), device=dev).bfloat16()
    rc = _lib().dk_net_attn62_bf16_async(qkv.data_ptr(), y.data_ptr(), B, 4, hd, torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    q, k, v = qkv.float().view(B, 62, 3, 4, hd).permute(2, 0, 3, 1, 4)
    ref = torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1) @ v          # [B, 4, 62, hd]
    ref = ref.transpose(1, 2).reshape(B, 62, d)
    assert torch.isfinite(y.float()).all()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


def _tokens(dev, n, vocab):
    return torch.cat([torch.randint(0, v, (n, 62 if i < 5 else 1), device=dev) for i, v in enumerate(vocab)], 1).int()


def _argmax_where_decided(p, p32, bound):
    """Rows whose fp32 top-two gap exceeds 2 x `bound` (so an output within `bound` of the
    fp32 one cannot change the argmax): the argmax must be the fp32 argmax there."""
    top2 = p32.topk(2, dim=1).values
    decided = (top2[:, 0] - top2[:, 1]) > 2 * bound
    agree = p.float().argmax(1) == p32.argmax(1)
    return int(decided.sum().item()), bool(agree[decided].all().item())


# Bounds of the networks' outputs against full f32, relative to the output scale (random
# weights and tokens); the measured errors are printed (profiles/r04/net_precision.log).
BF16_REL = 0.03
F32_REL = 2e-4


def test_fused_network_matches_fp32_module():
    """DokoAzNet's fused bf16 forward (embedding+LN, fused attention and MLP halves, class
    pooling) against the same weights run as the fp32 module at full f32 precision: every
    output within BF16_REL of the output scale, and the policy argmax exact wherever the fp32
    top-two gap exceeds twice that bound."""
    from master_doko_reinforcement_learning_amd.az_network import VOCAB, DokoAzNet
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    torch.set_float32_matmul_precision("highest")
    net32 = DokoAzNet().to(dev).eval()
    net16 = DokoAzNet().to(dev).eval()
    net16.load_state_dict(net32.state_dict())
    net16 = net16.bfloat16()
    tok = _tokens(dev, 1024, VOCAB)
    with torch.inference_mode():
        v32, p32 = net32(tok)
        v16, p16 = net16(tok)
    scale_v, scale_p = v32.abs().max().item(), p32.abs().max().item()
    ev = (v16.float() - v32).abs().max().item() / scale_v
    ep = (p16.float() - p32).abs().max().item() / scale_p
    print("bf16 network: value err %.4f, policy err %.4f of the output scale" % (ev, ep))
    assert ev < BF16_REL and ep < BF16_REL
    n, ok = _argmax_where_decided(p16, p32, BF16_REL * scale_p)
    print("policy rows decided beyond the bound: %d of %d" % (n, tok.shape[0]))
    assert ok and n > tok.shape[0] // 4


@pytest.mark.parametrize("net_name", ["az", "impi"])
@pytest.mark.parametrize("batch", [1, 3])
def test_f32_network_tiny_batch(net_name, batch):
    """The f32 network's HIP kernels on 1 and 3 samples (a single, partial row block of the MLP,
    one workgroup of the attention and head kernels) against the f32 module at full precision."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(7)
    if net_name == "az":
        from master_doko_reinforcement_learning_amd.az_network import VOCAB, DokoAzNet
        net = DokoAzNet().to(dev).eval()
    else:
        from master_doko_reinforcement_learning_amd.impi_network import VOCAB_IPI as VOCAB, DokoImpiNet
        net = DokoImpiNet().to(dev).eval()
    tok = _tokens(dev, batch, VOCAB)
    try:
        torch.set_float32_matmul_precision("highest")
        with torch.inference_mode():
            ref = net.forward_torch(tok)
            got = net(tok)
    finally:
        torch.set_float32_matmul_precision("highest")
    ref = ref if isinstance(ref, tuple) else (ref,)
    got = got if isinstance(got, tuple) else (got,)
    for r, g in zip(ref, got):
        assert g.shape == r.shape and torch.isfinite(g).all()
        assert (g - r).abs().max().item() < F32_REL * r.abs().max().item()


@pytest.mark.parametrize("net_name", ["az", "impi"])
def test_f32_network_reference_precision(net_name):
    """The f32 network path (FusedTrunkF32: f32 embedding + LayerNorm, add + LayerNorm,
    attention-core and GELU kernels, GEMMs at the reference's matmul precision "medium",
    az_doko.py:539-541, main.py:508) against the plain f32 module at full f32 precision: within
    F32_REL of the output scale, argmax exact wherever the top-two gap exceeds twice that."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    if net_name == "az":
        from master_doko_reinforcement_learning_amd.az_network import VOCAB, DokoAzNet
        net = DokoAzNet().to(dev).eval()
    else:
        from master_doko_reinforcement_learning_amd.impi_network import VOCAB_IPI as VOCAB, DokoImpiNet
        net = DokoImpiNet().to(dev).eval()
    tok = _tokens(dev, 512, VOCAB)
    try:
        torch.set_float32_matmul_precision("highest")
        with torch.inference_mode():
            ref = net.forward_torch(tok)            # the plain f32 module, exact f32 GEMMs
        torch.set_float32_matmul_precision("medium")
        torch.backends.cuda.matmul.allow_tf32 = True
        with torch.inference_mode():
            got = net(tok)                          # FusedTrunkF32: f32 HIP row kernels + "medium" GEMMs
    finally:
        torch.set_float32_matmul_precision("highest")
        torch.backends.cuda.matmul.allow_tf32 = False
    ref = ref if isinstance(ref, tuple) else (ref,)
    got = got if isinstance(got, tuple) else (got,)
    for r, g in zip(ref, got):
        assert g.dtype == torch.float32
        scale = r.abs().max().item()
        e = (g - r).abs().max().item() / scale
        print("%s f32 ('medium') network: err %.2e of the output scale" % (net_name, e))
        assert e < F32_REL
        n, ok = _argmax_where_decided(g, r, F32_REL * scale)
        assert ok and n > r.shape[0] // 2


@pytest.mark.parametrize("k,n", [(160, 640), (256, 1024)])
def test_fc_gelu_matches_torch(k, n):
    """Fused MLP first layer: GELU(x W^T + b) (exact erf GELU) against fp32 torch."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    rows = 62 * 37 + 5                                   # not a multiple of the 256-row tile
    x = torch.randn(rows, k, device=dev).bfloat16()
    w = (torch.randn(n, k, device=dev) / k ** 0.5).bfloat16()
    b = (torch.randn(n, device=dev) * 0.1).bfloat16()
    y = torch.full((rows, n), float("nan"), device=dev).bfloat16()
    rc = _lib().dk_net_fc_gelu_bf16_async(x.data_ptr(), w.data_ptr(), b.data_ptr(), rows, k, n, y.data_ptr(),
                                          torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    ref = F.gelu(F.linear(x.float(), w.float(), b.float()))
    assert torch.isfinite(y.float()).all()
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("d,n", [(160, 640), (256, 1024)])
def test_mlp_ln_matches_torch(d, n):
    """The fused MLP half of a block (d = 160 AlphaZero, 256 IMPI): x += proj(GELU(fc(h))) and
    h' = LN'(x), against fp32 torch on the same bf16 inputs (the delta rounded to bf16 like the
    unfused proj GEMM)."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(7)
    rows = 62 * 41 + 3                                   # not a multiple of the 128-row workgroup tile
    h = torch.randn(rows, d, device=dev).bfloat16()
    x = (torch.randn(rows, d, device=dev) * 2).bfloat16()
    w1 = (torch.randn(n, d, device=dev) / d ** 0.5).bfloat16()
    b1 = (torch.randn(n, device=dev) * 0.1).bfloat16()
    w2 = (torch.randn(d, n, device=dev) / n ** 0.5).bfloat16()
    b2 = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = (1 + 0.1 * torch.randn(d, device=dev)).bfloat16()
    be = (0.1 * torch.randn(d, device=dev)).bfloat16()
    delta_ref = F.linear(F.gelu(F.linear(h.float(), w1.float(), b1.float())), w2.float(), b2.float())
    x_ref = x.float() + delta_ref.bfloat16().float()
    h_ref = F.layer_norm(x_ref.bfloat16().float(), (d,), g.float(), be.float(), 1e-5)
    xo = x.clone()
    out = torch.full((rows, d), float("nan"), device=dev).bfloat16()
    rc = _lib().dk_net_mlp_ln_bf16_async(h.data_ptr(), xo.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                         b2.data_ptr(), rows, d, n, g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(),
                                         torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all() and torch.isfinite(xo.float()).all()
    torch.testing.assert_close(xo.float(), x_ref, rtol=1e-2, atol=3e-2)
    torch.testing.assert_close(out.float(), h_ref, rtol=1e-2, atol=3e-2)


@pytest.mark.parametrize("hd", [40, 64])
def test_attn_ln_matches_torch(hd):
    """The fused attention half of a block (4 heads x hd, 62 tokens): x += proj(MHA(qkv)) and
    h = LN(x), against fp32 torch on the same bf16 inputs (attention output and delta rounded
    to bf16 like the unfused kernels)."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(11)
    B, d = 53, 4 * hd
    qkv = (torch.randn(B, 62, 3 * d, device=dev) * 1.5).bfloat16()
    x = (torch.randn(B, 62, d, device=dev) * 2).bfloat16()
    w = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
    b = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = (1 + 0.1 * torch.randn(d, device=dev)).bfloat16()
    be = (0.1 * torch.randn(d, device=dev)).bfloat16()
    q, k, v = qkv.float().view(B, 62, 3, 4, hd).permute(2, 0, 3, 1, 4)
    y = (torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1) @ v).transpose(1, 2).reshape(B, 62, d)
    delta = F.linear(y.bfloat16().float(), w.float(), b.float()).bfloat16().float()
    x_ref = (x.float() + delta).bfloat16().float()
    h_ref = F.layer_norm(x_ref, (d,), g.float(), be.float(), 1e-5)
    xo = x.clone()
    out = torch.full((B, 62, d), float("nan"), device=dev).bfloat16()
    rc = _lib().dk_net_attn_ln_bf16_async(qkv.data_ptr(), xo.data_ptr(), w.data_ptr(), b.data_ptr(), B, 4, hd,
                                          g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(),
                                          torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all() and torch.isfinite(xo.float()).all()
    torch.testing.assert_close(xo.float(), x_ref, rtol=1e-2, atol=3e-2)
    torch.testing.assert_close(out.float(), h_ref, rtol=2e-2, atol=4e-2)


@pytest.mark.parametrize("hd", [40, 64])
def test_qkv_attn_ln_matches_torch(hd):
    """The whole attention half from h = ln_1(x) (qkv projection inside the kernel) against fp32
    torch: qkv = h Wqkv^T + b rounded to bf16 like the unfused GEMM, then as test_attn_ln."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(13)
    B, d = 45, 4 * hd
    h = torch.randn(B, 62, d, device=dev).bfloat16()
    wq = (torch.randn(3 * d, d, device=dev) / d ** 0.5).bfloat16()
    bq = (torch.randn(3 * d, device=dev) * 0.1).bfloat16()
    x = (torch.randn(B, 62, d, device=dev) * 2).bfloat16()
    w = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
    b = (torch.randn(d, device=dev) * 0.1).bfloat16()
    g = (1 + 0.1 * torch.randn(d, device=dev)).bfloat16()
    be = (0.1 * torch.randn(d, device=dev)).bfloat16()
    qkv = F.linear(h.float(), wq.float(), bq.float()).bfloat16().float()
    q, k, v = qkv.view(B, 62, 3, 4, hd).permute(2, 0, 3, 1, 4)
    y = (torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1) @ v).transpose(1, 2).reshape(B, 62, d)
    delta = F.linear(y.bfloat16().float(), w.float(), b.float()).bfloat16().float()
    x_ref = (x.float() + delta).bfloat16().float()
    h_ref = F.layer_norm(x_ref, (d,), g.float(), be.float(), 1e-5)
    xo = x.clone()
    out = torch.full((B, 62, d), float("nan"), device=dev).bfloat16()
    L = _lib()
    assert L.dk_net_qkv_attn_ln_bf16_async(h.data_ptr(), xo.data_ptr(), wq.data_ptr(), bq.data_ptr(), w.data_ptr(),
                                           b.data_ptr(), B, 4, hd, g.data_ptr(), be.data_ptr(), 1e-5, h.data_ptr(),
                                           None) != 0            # h_out aliasing h is refused
    rc = L.dk_net_qkv_attn_ln_bf16_async(h.data_ptr(), xo.data_ptr(), wq.data_ptr(), bq.data_ptr(), w.data_ptr(),
                                         b.data_ptr(), B, 4, hd, g.data_ptr(), be.data_ptr(), 1e-5, out.data_ptr(),
                                         torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all() and torch.isfinite(xo.float()).all()
    torch.testing.assert_close(xo.float(), x_ref, rtol=1e-2, atol=3e-2)
    torch.testing.assert_close(out.float(), h_ref, rtol=2e-2, atol=4e-2)


@pytest.mark.parametrize("d,C", [(160, 39), (160, 4), (256, 33)])
def test_class_pool_ln_matches_torch(d, C):
    """PerClassAttentionMLPHead's pooling + per-class LayerNorm (policy 39 / value 4 classes at
    d 160, IMPI 33 at d 256) against fp32 torch with the bf16 path's roundings (scores, scaled
    scores, softmax weights and the pooled rows rounded to bf16)."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(17)
    B = 37
    x = (torch.randn(B, 62, d, device=dev) * 1.5).bfloat16()
    q = torch.randn(C, d, device=dev).bfloat16()
    lw = (1 + 0.1 * torch.randn(C, d, device=dev)).bfloat16()
    lb = (0.1 * torch.randn(C, d, device=dev)).bfloat16()
    scale = d ** -0.5
    bf = lambda t: t.bfloat16().float()   # noqa: E731
    sc = bf(bf(torch.einsum("cd,bsd->bcs", q.float(), x.float())) * scale)
    w = bf(torch.softmax(sc, dim=-1))
    a = bf(torch.einsum("bcs,bsd->bcd", w, x.float()))
    ref = (F.layer_norm(a, (d,)) * lw.float() + lb.float()).transpose(0, 1)      # [C, B, d]
    out = torch.full((C, B, d), float("nan"), device=dev).bfloat16()
    rc = _lib().dk_net_class_pool_ln_bf16_async(x.data_ptr(), B, d, q.data_ptr(), C, scale, lw.data_ptr(), lb.data_ptr(),
                                                1e-5, out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=4e-2)


@pytest.mark.parametrize("d,C", [(160, 39), (256, 33)])
def test_class_mlp_bf16_matches_fp32(d, C):
    """The bf16 class MLPs (class_mlp_bf16_kernel) on the bf16 pooled operand against the same
    MLPs in fp32 on the same bf16 operands: only the final bf16 rounding apart (B = 300: a
    partial row block); the whole bf16 head against its torch bf16 form within bf16 noise."""
    import torch.nn.functional as F
    from master_doko_reinforcement_learning_amd.az_network import ClassHead
    dev = torch.device("cuda", 0)
    torch.manual_seed(6)
    head = ClassHead(d, C).to(dev).to(torch.bfloat16).eval()
    x = torch.randn(300, 62, d, device=dev).to(torch.bfloat16)
    with torch.inference_mode():
        assert head.bf16_fused_ok(x)
        got = head(x)
        tor = head(x, fused=False)
        ac = head.pooled(x).float()
        h = F.gelu(torch.bmm(ac, head.w1.float().transpose(1, 2)) + head.b1.float()[:, None, :])
        ref = ((h * head.w2.float()[:, None, :]).sum(-1) + head.b2.float()[:, None]).transpose(0, 1)
    assert got.dtype == torch.bfloat16 and got.shape == ref.shape == (300, C)
    scale = ref.abs().max().item()
    e = (got.float() - ref).abs().max().item() / scale
    assert e < 8e-3, e
    e2 = (got.float() - tor.float()).abs().max().item() / scale
    assert e2 < 5e-2, e2


@pytest.mark.parametrize("d,C", [(160, 39), (160, 4), (256, 33), (256, 4), (160, 8), (160, 9)])
def test_class_head_f32_matches_torch(d, C):
    """The f32 heads (class_pool_ln_f32x3_kernel -- C <= 8: class_pool_small_ln_f32_kernel, f32
    FMAs -- + class_mlp_f32x3_kernel, bf16x3 products) against ClassHead's torch forward at matmul
    precision "highest": within 2e-5 of the output scale (B = 300: a partial row block of the class
    MLP grid)."""
    from master_doko_reinforcement_learning_amd.az_network import ClassHead
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    head = ClassHead(d, C).to(dev).eval()
    with torch.no_grad():
        head.ln_w.add_(0.1 * torch.randn_like(head.ln_w))
        head.ln_b.add_(0.1 * torch.randn_like(head.ln_b))
    x = torch.randn(300, 62, d, device=dev)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        with torch.inference_mode():
            assert head.f32_fused_ok(x)
            ref = head(x, fused=False)
            got = head(x)
    finally:
        torch.set_float32_matmul_precision(prev)
    assert got.shape == ref.shape == (300, C) and torch.isfinite(got).all()
    e = (got - ref).abs().max().item() / ref.abs().max().item()
    assert e < 2e-5, e


@pytest.mark.parametrize("hd", [40, 64])
def test_attn62_f32_matches_torch(hd):
    """f32 attention core (one wave per sample and head on the f32 matrix cores; -DDK_ATTN_F32_MFMA=0:
    the VALU kernel with an online softmax over chunks of 8 keys)
    against torch f32 softmax(q k^T / sqrt(hd)) v at full f32 precision."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(13)
    B, d = 53, 4 * hd
    qkv = torch.randn(B, 62, 3 * d, device=dev) * 1.5
    y = torch.full((B, 62, d), float("nan"), device=dev)
    rc = _lib().dk_net_attn62_f32_async(qkv.data_ptr(), y.data_ptr(), B, 4, hd, torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    torch.set_float32_matmul_precision("highest")
    q, k, v = qkv.double().view(B, 62, 3, 4, hd).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1) @ v).transpose(1, 2).reshape(B, 62, d)
    torch.testing.assert_close(y.double(), ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("d", [160, 256])
def test_f32_row_kernels_match_torch(d):
    """embed + LayerNorm, add + LayerNorm and GELU in f32 against torch f32."""
    from master_doko_reinforcement_learning_amd.az_network import VOCAB
    dev = torch.device("cuda", 0)
    torch.manual_seed(d + 1)
    B = 37
    tables = [torch.randn(v, d, device=dev) for v in VOCAB]
    tok = _tokens(dev, B, VOCAB)
    g, b = 1 + 0.1 * torch.randn(d, device=dev), 0.1 * torch.randn(d, device=dev)
    x = torch.empty(B, 62, d, device=dev)
    h = torch.empty_like(x)
    st = torch.cuda.current_stream(dev).cuda_stream
    tp = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in tables])
    assert _lib().dk_net_embed_ln_f32_async(tok.data_ptr(), B, tp, d, g.data_ptr(), b.data_ptr(), 1e-5, x.data_ptr(),
                                           h.data_ptr(), st) == 0
    t = tok.long()
    xr = tables[0][t[:, 0:62]]
    for i in range(1, 5):
        xr = xr + tables[i][t[:, 62 * i:62 * (i + 1)]]
    xr = xr + tables[5][t[:, 310:311]]
    torch.cuda.synchronize()
    assert torch.equal(x, xr)                               # the same left-to-right f32 sum
    torch.testing.assert_close(h, F.layer_norm(xr, (d,), g, b, 1e-5), rtol=1e-5, atol=1e-5)
    x1 = torch.full_like(x, float("nan"))                   # x only (h_out NULL): embed_f32_kernel
    assert _lib().dk_net_embed_ln_f32_async(tok.data_ptr(), B, tp, d, None, None, 1e-5, x1.data_ptr(), None, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(x1, xr)
    delta = torch.randn_like(x)
    x2 = x.clone()
    assert _lib().dk_net_add_ln_f32_async(x2.data_ptr(), delta.data_ptr(), B * 62, d, g.data_ptr(), b.data_ptr(), 1e-5,
                                         h.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(x2, x + delta)
    torch.testing.assert_close(h, F.layer_norm(x + delta, (d,), g, b, 1e-5), rtol=1e-5, atol=1e-5)
    a = torch.randn(B * 62, 4 * d, device=dev) * 3
    a2 = a.clone()
    assert _lib().dk_net_gelu_f32_async(a2.data_ptr(), a2.numel(), st) == 0
    torch.cuda.synchronize()
    torch.testing.assert_close(a2, F.gelu(a), rtol=2e-6, atol=2e-6)


@pytest.mark.parametrize("d", [160, 256])
def test_f32_bias_kernels_match_torch(d):
    """The f32 kernels that take the producing GEMM's bias (the GEMMs then run without their
    bias epilogue): GELU(y + b) and x += (delta + b), h = LN(x), and the attention core with the
    qkv bias added as q / k / v load -- against torch f32 in the epilogue's order."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(d + 7)
    B = 29
    st = torch.cuda.current_stream(dev).cuda_stream
    n = 4 * d
    y = torch.randn(B * 62, n, device=dev)
    b = torch.randn(n, device=dev)
    ref = F.gelu(y + b)
    assert _lib().dk_net_gelu_bias_f32_async(y.data_ptr(), b.data_ptr(), y.numel(), n, st) == 0
    torch.cuda.synchronize()
    torch.testing.assert_close(y, ref, rtol=1e-6, atol=1e-6)
    x = torch.randn(B * 62, d, device=dev)
    delta = torch.randn(B * 62, d, device=dev)
    bd = torch.randn(d, device=dev)
    g, be = 1 + 0.1 * torch.randn(d, device=dev), 0.1 * torch.randn(d, device=dev)
    x_ref = x + (delta + bd)
    h_ref = F.layer_norm(x_ref, (d,), g, be, 1e-5)
    h = torch.empty_like(x)
    assert _lib().dk_net_add_bias_ln_f32_async(x.data_ptr(), delta.data_ptr(), bd.data_ptr(), B * 62, d, g.data_ptr(),
                                               be.data_ptr(), 1e-5, h.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(x, x_ref)
    torch.testing.assert_close(h, h_ref, rtol=1e-5, atol=1e-5)
    hd = d // 4
    qkv = torch.randn(B, 62, 3 * d, device=dev) * 1.5
    bq = torch.randn(3 * d, device=dev)
    out = torch.empty(B, 62, d, device=dev)
    assert _lib().dk_net_attn62_bias_f32_async(qkv.data_ptr(), bq.data_ptr(), out.data_ptr(), B, 4, hd, st) == 0
    torch.cuda.synchronize()
    q, k, v = (qkv + bq).double().view(B, 62, 3, 4, hd).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1) @ v).transpose(1, 2).reshape(B, 62, d)
    torch.testing.assert_close(out.double(), ref, rtol=2e-5, atol=2e-5)
