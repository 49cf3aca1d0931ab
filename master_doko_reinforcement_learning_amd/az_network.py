"""The AlphaZero policy/value network for full Doppelkopf, inference side.

Architecture of rs-doko-py-bridge/python/az_doko.py:28-138 (AlphaZeroTicTacToeNetwork
with TransformerBlock.py / SelfAttention.py), default config n_embd 160, 4 heads,
4 shared blocks + 1 policy block + 1 value block:

    tokens [B, 311] = 5 x 62 token rows + phase (encode_state_pi, see az_encode)
    x = E_obj[t0] + E_pos[t1] + E_player[t2] + E_subpos[t3] + E_team[t4] + E_phase[t5]   [B, 62, d]
    blocks: x += c_proj(MHA(LN1 x));  x += W2 GELU(W1 LN2 x)
    heads : per-class attention pooling (learned class queries over the 62 positions),
            then a per-class LN -> Linear(d, d) -> GELU -> Linear(d, 1)
    value [B, 4], policy logits [B, 39]

Re-expressed for MI355X rather than translated (forward_fused):
  * bf16 inference runs on hand-written gfx950 kernels (csrc/az_net_kernels.h): the
    embedding sum + first LayerNorm, the whole attention half of a block (qkv projection,
    MFMA attention core, folded out/c projection, residual add + LayerNorm) in
    qkv_attn_ln_kernel, the whole MLP half (GEMM + GELU + GEMM + residual + LayerNorm) in
    mlp_ln_kernel, and the heads' class pooling + LayerNorm in class_pool_ln_kernel;
  * the reference's f32 precision (FusedTrunkF32, csrc/az_net_f32_kernels.h) for
    `--net-precision f32`;
  * the 4 + 39 per-class MLPs of the heads run in ONE kernel launch (class_mlp_bf16_kernel /
    class_mlp_f32x3_kernel over class-stacked weights [C, d, d]) instead of 43 small module calls;
  * the tokens come straight from the device encoder, no host round trip.
  forward_torch keeps the reference structure (the qkv projection has the
  nn.MultiheadAttention in_proj [q; k; v] layout, see load_reference_state_dict).
Weights are random-initialised here (no checkpoint ships with the reference);
load_reference_state_dict maps a reference state_dict onto this module.
"""
import ctypes
import math
import os

import torch
import torch.nn.functional as F
from torch import nn

ctypes_vp = ctypes.c_void_p
VOCAB = (43, 57, 5, 13, 3, 3)   # object, position, player, subposition, team, phase (az_doko.py:85-90)
SEQ = 62


class Block(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.heads = heads
        self.ln_1 = nn.LayerNorm(d)
        self.qkv = nn.Linear(d, 3 * d)          # MultiheadAttention.in_proj
        self.out = nn.Linear(d, d)              # MultiheadAttention.out_proj
        self.c_proj = nn.Linear(d, d)           # SelfAttention.c_proj
        self.ln_2 = nn.LayerNorm(d)
        self.fc = nn.Linear(d, 4 * d)
        self.proj = nn.Linear(4 * d, d)

    def attn_delta(self, h):                     # h = ln_1(x)
        b, s, d = h.shape
        q, k, v = self.qkv(h).view(b, s, 3, self.heads, d // self.heads).permute(2, 0, 3, 1, 4)
        y = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, s, d)
        return self.c_proj(self.out(y))

    def folded_proj(self):
        """c_proj(out(y)) = (Wc Wo) y + (Wc bo + bc): the two back-to-back projections of
        the reference's SelfAttention (MultiheadAttention.out_proj, then c_proj) folded
        into one GEMM for inference (products in f64 on the host, cached until the weights change)."""
        key = tuple((p.data_ptr(), p._version) for p in (self.out.weight, self.out.bias, self.c_proj.weight,
                                                          self.c_proj.bias)) + (self.out.weight.dtype,)
        if getattr(self, "_fold_key", None) != key:
            # (in f64 on the host, once per weight version: exact to the storage dtype's rounding,
            # and no BLAS kernel on the device)
            wo, bo = self.out.weight.detach().double().cpu(), self.out.bias.detach().double().cpu()
            wc, bc = self.c_proj.weight.detach().double().cpu(), self.c_proj.bias.detach().double().cpu()
            dt, dev = self.out.weight.dtype, self.out.weight.device
            self._fold = ((wc @ wo).to(dev, dt), (wc @ bo + bc).to(dev, dt))
            self._fold_key = key
        return self._fold

    def mlp_delta(self, h):                      # h = ln_2(x)
        return self.proj(F.gelu(self.fc(h)))

    def forward(self, x):
        x = x + self.attn_delta(self.ln_1(x))
        return x + self.mlp_delta(self.ln_2(x))

    # state_dict names of the reference's TransformerBlock (TransformerBlock.py:5-27, SelfAttention.py:4-36)
    REF_NAMES = (("ln_1.weight", "ln_1.weight"), ("ln_1.bias", "ln_1.bias"),
                 ("qkv.weight", "attn.attn.in_proj_weight"), ("qkv.bias", "attn.attn.in_proj_bias"),
                 ("out.weight", "attn.attn.out_proj.weight"), ("out.bias", "attn.attn.out_proj.bias"),
                 ("c_proj.weight", "attn.c_proj.weight"), ("c_proj.bias", "attn.c_proj.bias"),
                 ("ln_2.weight", "ln_2.weight"), ("ln_2.bias", "ln_2.bias"),
                 ("fc.weight", "mlp.c_fc.weight"), ("fc.bias", "mlp.c_fc.bias"),
                 ("proj.weight", "mlp.c_proj.weight"), ("proj.bias", "mlp.c_proj.bias"))

    @torch.no_grad()
    def load_reference(self, sd, prefix=""):
        """Copy a reference TransformerBlock's parameters (state_dict entries `prefix + name`)."""
        own = self.state_dict()
        for mine, ref in self.REF_NAMES:
            own[mine].copy_(sd[prefix + ref])


class ClassHead(nn.Module):
    """PerClassAttentionMLPHead (az_doko.py:28-56) with class-stacked MLP weights."""

    def __init__(self, d, classes):
        super().__init__()
        self.queries = nn.Parameter(torch.randn(classes, d))
        self.scale = d ** -0.5
        self.ln_w = nn.Parameter(torch.ones(classes, d))
        self.ln_b = nn.Parameter(torch.zeros(classes, d))
        self.w1 = nn.Parameter(torch.empty(classes, d, d))
        self.b1 = nn.Parameter(torch.empty(classes, d))
        self.w2 = nn.Parameter(torch.empty(classes, d))
        self.b2 = nn.Parameter(torch.empty(classes))
        bound = 1.0 / math.sqrt(d)
        for p in (self.w1, self.b1, self.w2, self.b2):
            nn.init.uniform_(p, -bound, bound)

    def pooled(self, x):
        """The attention pooling and each class's LayerNorm, class-major [C, B, d]."""
        B, S, d = x.shape
        C = self.queries.shape[0]
        # the HIP kernel has no backward: inference only, and only on bf16 contiguous operands
        if (x.is_cuda and x.dtype == torch.bfloat16 and S == SEQ and d in (160, 256) and C <= 64
                and not torch.is_grad_enabled()
                and all(p.dtype == torch.bfloat16 and p.is_contiguous() for p in (self.queries, self.ln_w, self.ln_b))):
            from . import _native
            x = x.contiguous()
            ac = torch.empty((C, B, d), dtype=x.dtype, device=x.device)
            rc = _native.lib().dk_net_class_pool_ln_bf16_async(
                x.data_ptr(), B, d, self.queries.data_ptr(), C, self.scale, self.ln_w.data_ptr(), self.ln_b.data_ptr(),
                1e-5, ac.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)
            if rc != 0:
                raise RuntimeError("doko_amd class pooling kernel error %d" % rc)
            return ac
        w = torch.softmax(torch.einsum("cd,bsd->bcs", self.queries, x) * self.scale, dim=-1)
        a = torch.einsum("bcs,bsd->bcd", w, x)                  # [B, C, d]
        a = F.layer_norm(a, a.shape[-1:]) * self.ln_w + self.ln_b
        # per-class MLP as one batched GEMM over the classes on a contiguous [C, B, d]
        # operand: einsum("bci,coi->bco") hands the GEMM a class-batched view whose batch
        # stride (d) is smaller than its row stride (C d), and a PyTorch TunableOp candidate
        # faulted on that layout
        return a.transpose(0, 1).contiguous()                    # [C, B, d]

    def f32_fused_ok(self, x):
        B, S, d = x.shape
        return (x.is_cuda and x.dtype == torch.float32 and S == SEQ and d in (160, 256) and self.queries.shape[0] <= 64
                and not torch.is_grad_enabled() and not autocast_on(x.device.type)
                and all(p.dtype == torch.float32 and p.is_contiguous() for p in self.parameters()))

    def forward_f32(self, x):
        """The f32 forward on two HIP kernels (bf16x3 products): the pooling + class LayerNorms
        (class_pool_ln_f32x3_kernel) and every class's MLP (class_mlp_f32x3_kernel) -> [B, C]."""
        from . import _native
        L = _native.lib()
        B, S, d = x.shape
        C = self.queries.shape[0]
        x = x.contiguous()
        st = torch.cuda.current_stream(x.device).cuda_stream
        key = (self.w1.data_ptr(), self.w1._version)
        if getattr(self, "_w1_split", (None,))[0] != key:
            hi = self.w1.detach().bfloat16().contiguous()
            self._w1_split = (key, hi, (self.w1.detach() - hi.float()).bfloat16().contiguous())
        _, w1h, w1l = self._w1_split
        ac = torch.empty((C, B, d), dtype=torch.float32, device=x.device)
        out = torch.empty((B, C), dtype=torch.float32, device=x.device)
        for rc in (L.dk_net_class_pool_ln_f32_async(x.data_ptr(), B, d, self.queries.data_ptr(), C, self.scale,
                                                    self.ln_w.data_ptr(), self.ln_b.data_ptr(), 1e-5, ac.data_ptr(), st),
                   L.dk_net_class_mlp_f32x3_async(ac.data_ptr(), B, d, C, w1h.data_ptr(), w1l.data_ptr(), self.b1.data_ptr(),
                                                  self.w2.data_ptr(), self.b2.data_ptr(), out.data_ptr(), st)):
            if rc != 0:
                raise RuntimeError("doko_amd f32 head kernel error %d" % rc)
        return out

    def bf16_fused_ok(self, x):
        B, S, d = x.shape
        return (x.is_cuda and x.dtype == torch.bfloat16 and S == SEQ and d in (160, 256) and self.queries.shape[0] <= 64
                and not torch.is_grad_enabled()
                and all(p.dtype == torch.bfloat16 and p.is_contiguous() for p in self.parameters()))

    def forward(self, x, fused=True):                            # x [B, S, d]
        if fused and self.f32_fused_ok(x):
            return self.forward_f32(x)
        if fused and self.bf16_fused_ok(x):
            # pooling + class LayerNorms, then every class's MLP in one launch (class_mlp_bf16_kernel)
            from . import _native
            ac = self.pooled(x)
            B, C = x.shape[0], self.queries.shape[0]
            out = torch.empty((B, C), dtype=torch.bfloat16, device=x.device)
            rc = _native.lib().dk_net_class_mlp_bf16_async(ac.data_ptr(), B, x.shape[2], C, self.w1.data_ptr(),
                                                           self.b1.data_ptr(), self.w2.data_ptr(), self.b2.data_ptr(),
                                                           out.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)
            if rc != 0:
                raise RuntimeError("doko_amd class MLP kernel error %d" % rc)
            return out
        ac = self.pooled(x)
        h = F.gelu(torch.bmm(ac, self.w1.transpose(1, 2)) + self.b1[:, None, :])   # [C, B, d]
        return ((h * self.w2[:, None, :]).sum(-1) + self.b2[:, None]).transpose(0, 1)   # [B, C]


class FusedTrunk:
    """The bf16 GPU forward of a token trunk (shared by DokoAzNet and DokoImpiNet): HIP
    kernels (csrc/az_net_kernels.h) for the embedding sum + first LayerNorm, every
    residual add fused with the LayerNorm that follows it, (4 heads of 40 or 64) the whole
    attention half (qkv projection + attention core + folded projection + residual +
    LayerNorm in one kernel), and (d = 160 or 256) the whole MLP half; the heads run
    class_pool_ln_kernel and class_mlp_bf16_kernel (ClassHead).  Other shapes fall back to torch
    GEMMs (hipBLASLt).  `x` is the residual stream, `h` the current LayerNorm output."""

    def __init__(self, tokens, emb, ln0):
        from . import _native
        self.L = _native.lib()
        self.st = torch.cuda.current_stream(tokens.device).cuda_stream
        tok = tokens.int().contiguous()
        B, d = tok.shape[0], emb[0].weight.shape[1]
        self.rows, self.d = B * SEQ, d
        self.x = torch.empty((B, SEQ, d), dtype=torch.bfloat16, device=tok.device)
        self.h = torch.empty_like(self.x)
        tables = (ctypes_vp * 6)(*[e.weight.data_ptr() for e in emb])
        self.ck(self.L.dk_net_embed_ln_bf16_async(tok.data_ptr(), B, tables, d, ln0.weight.data_ptr(), ln0.bias.data_ptr(),
                                                  ln0.eps, self.x.data_ptr(), self.h.data_ptr(), self.st))

    @staticmethod
    def ck(rc):
        if rc != 0:
            raise RuntimeError("doko_amd network kernel error %d" % rc)

    def add_ln(self, x, delta, ln):
        h = torch.empty_like(x)
        self.ck(self.L.dk_net_add_ln_bf16_async(x.data_ptr(), delta.data_ptr() if delta is not None else None, self.rows,
                                                self.d, ln.weight.data_ptr(), ln.bias.data_ptr(), ln.eps, h.data_ptr(), self.st))
        return h

    def attn_delta(self, blk, h):
        if not (blk.heads == 4 and self.d // 4 in (40, 64) and self.d % 4 == 0):
            return blk.attn_delta(h)
        qkv = blk.qkv(h)                                     # [B, 62, 3d]: q | k | v, heads contiguous
        y = torch.empty_like(h)
        self.ck(self.L.dk_net_attn62_bf16_async(qkv.data_ptr(), y.data_ptr(), h.shape[0], 4, self.d // 4, self.st))
        w, b = blk.folded_proj()
        return F.linear(y, w, b)

    def mlp_delta(self, blk, h):
        """proj(GELU(fc(h))): the first layer and its exact GELU in one kernel (the 4d-wide
        activation is written once), the second layer on hipBLASLt."""
        n = blk.fc.weight.shape[0]
        if self.d not in (160, 256) or n % 64:
            return blk.mlp_delta(h)
        a = torch.empty(h.shape[:-1] + (n,), dtype=h.dtype, device=h.device)
        self.ck(self.L.dk_net_fc_gelu_bf16_async(h.data_ptr(), blk.fc.weight.data_ptr(), blk.fc.bias.data_ptr(),
                                                 self.rows, self.d, n, a.data_ptr(), self.st))
        return blk.proj(a)

    def attn_ln(self, x, blk, h, ln):
        """x += c_proj(out(MHA(qkv(h)))); returns LN(x): the qkv projection, the attention core,
        the folded projection, the residual add and the LayerNorm in one kernel per sample."""
        if not (blk.heads == 4 and self.d // 4 in (40, 64) and self.d % 4 == 0):
            return self.add_ln(x, self.attn_delta(blk, h), ln)
        w, b = blk.folded_proj()
        out = torch.empty_like(x)
        wq, bq = blk.qkv.weight, blk.qkv.bias
        assert wq.dtype == torch.bfloat16 and wq.is_contiguous() and bq is not None and bq.is_contiguous()
        self.ck(self.L.dk_net_qkv_attn_ln_bf16_async(h.data_ptr(), x.data_ptr(), wq.data_ptr(), bq.data_ptr(), w.data_ptr(),
                                                     b.data_ptr(), h.shape[0], 4, self.d // 4, ln.weight.data_ptr(),
                                                     ln.bias.data_ptr(), ln.eps, out.data_ptr(), self.st))
        return out

    def mlp_ln(self, x, blk, h, ln):
        """x += proj(GELU(fc(h))); returns LN(x): the whole MLP half of the block and the
        LayerNorm after it in one kernel (d = 160 or 256: the hidden activation never leaves the CU)."""
        n = blk.fc.weight.shape[0]
        if self.d not in (160, 256) or n % (64 if self.d == 160 else 32):
            return self.add_ln(x, self.mlp_delta(blk, h), ln)
        out = torch.empty_like(x)
        self.ck(self.L.dk_net_mlp_ln_bf16_async(h.data_ptr(), x.data_ptr(), blk.fc.weight.data_ptr(),
                                                blk.fc.bias.data_ptr(), blk.proj.weight.data_ptr(), blk.proj.bias.data_ptr(),
                                                self.rows, self.d, n, ln.weight.data_ptr(), ln.bias.data_ptr(), ln.eps,
                                                out.data_ptr(), self.st))
        return out

    def run(self, h, blocks, final_ln, x=None):
        x = self.x if x is None else x
        for i, blk in enumerate(blocks):
            h = self.attn_ln(x, blk, h, blk.ln_2)
            nxt = blocks[i + 1].ln_1 if i + 1 < len(blocks) else final_ln
            h = self.mlp_ln(x, blk, h, nxt)
        return h


def autocast_on(dev_type="cuda"):
    """True when torch autocast would change F.linear's output dtype on `dev_type`."""
    try:
        return torch.is_autocast_enabled(dev_type)
    except TypeError:   # (older torch: no per-device query)
        return torch.is_autocast_enabled()


def f32_fused_ok(tokens, weight):
    """The f32 fused forward reads every GEMM output through raw pointers as float32: take it
    only for f32 weights on the GPU, without autograd, and with autocast off (under autocast
    F.linear returns bf16 / f16 buffers half the size)."""
    return (tokens.is_cuda and weight.dtype == torch.float32 and not torch.is_grad_enabled()
            and not autocast_on(tokens.device.type))


def _f32c(t):
    """A GEMM output handed to an f32 kernel: float32 and contiguous, or raise (never reinterpret)."""
    if t.dtype != torch.float32:
        raise RuntimeError("f32 fused trunk: expected a float32 activation, got %s (autocast?)" % t.dtype)
    return t.contiguous()


def mlp_split_bf16x3(w1, w2):
    """The MLP weights in the f32 MLP kernels' split layout: bf16 hi / lo pairs (w = hi + lo to
    ~16 bits) of W1 [n, d] and of W2 [d, n] with W2's columns permuted so that a lane's GEMM2
    fragment is one 16-B piece in GEMM1's accumulator order:
      d = 160 (mlp_ln_f32x3_kernel, 32 x 32 tiles): within every group of 16 hidden units,
        units 4-7 and 8-11 swapped;
      d = 256 (mlp16_ln_f32x3_kernel, 16 x 16 tiles): within every group of 32, slot q holds unit
        4 (q >> 3) + (q & 7) if (q & 7) < 4, else 16 + 4 (q >> 3) + (q & 7) - 4."""
    w2 = w2.float()
    d, n = w2.shape
    if d == 256:
        q = torch.arange(32)
        kg, j = q // 8, q % 8
        src = torch.where(j < 4, 4 * kg + j, 16 + 4 * kg + j - 4)
        w2 = w2.reshape(d, n // 32, 32)[:, :, src.to(w2.device)].reshape(d, n)
    else:
        w2 = w2.reshape(-1, n // 16, 4, 4)[:, :, [0, 2, 1, 3], :].reshape(-1, n)
    parts = []
    for w in (w1.float(), w2):
        hi = w.bfloat16().contiguous()
        parts += [hi, (w - hi.float()).bfloat16().contiguous()]
    return tuple(parts)


def split_bf16x3(blk):
    """A block's MLP weights in the split layout (mlp_split_bf16x3), cached on the block and
    rebuilt when a weight changes (version counter)."""
    key = (blk.fc.weight.data_ptr(), blk.fc.weight._version, blk.proj.weight.data_ptr(), blk.proj.weight._version)
    c = getattr(blk, "_bf16x3", None)
    if c is None or c[0] != key:
        c = (key, mlp_split_bf16x3(blk.fc.weight.detach(), blk.proj.weight.detach()))
        blk._bf16x3 = c
    return c[1]


def split_attn_bf16x3(blk):
    """The attention half's weights as bf16 hi / lo pairs: Wqkv and the folded projection
    (Block.folded_proj, f32), cached on the block until a weight changes; with the folded f32 bias."""
    key = tuple((p.data_ptr(), p._version) for p in (blk.qkv.weight, blk.out.weight, blk.out.bias, blk.c_proj.weight,
                                                     blk.c_proj.bias))
    c = getattr(blk, "_attn_bf16x3", None)
    if c is None or c[0] != key:
        wp, bp = blk.folded_proj()
        parts = []
        for w in (blk.qkv.weight.detach(), wp.detach()):
            hi = w.float().bfloat16().contiguous()
            parts += [hi, (w.float() - hi.float()).bfloat16().contiguous()]
        c = (key, tuple(parts) + (bp.detach().float().contiguous(),))
        blk._attn_bf16x3 = c
    return c[1]


class FusedTrunkF32(FusedTrunk):
    """The f32 GPU forward of a token trunk: the reference's precision (f32 activations; GEMM
    products at least as fine as the reference's matmul precision "medium", az_doko.py:539-541)
    with HIP kernels (csrc/az_net_f32_kernels.h): the embedding sum + first LayerNorm; at d = 160
    each block as two kernels with bf16x3 products (round 5; d = 160 or 256, 4 heads): the whole
    attention half (qkv_attn_ln_f32x3_kernel) and the whole MLP half (mlp_ln_f32x3_kernel);
    other shapes keep the attention core (f32 MFMA), residual adds fused with the LayerNorm after
    them and the GEMMs on hipBLASLt at "medium", the attention half's out_proj and c_proj folded
    into one GEMM (Block.folded_proj, f32).  The heads: ClassHead.forward_f32."""

    def __init__(self, tokens, emb, ln0, need_h=True):
        from . import _native
        self.L = _native.lib()
        self.st = torch.cuda.current_stream(tokens.device).cuda_stream
        tok = tokens.int().contiguous()
        B, d = tok.shape[0], emb[0].weight.shape[1]
        self.rows, self.d = B * SEQ, d
        self.x = torch.empty((B, SEQ, d), dtype=torch.float32, device=tok.device)
        # (need_h False: the embedding sum only; the x-only chain normalises x in its first half)
        self.h = torch.empty_like(self.x) if need_h else None
        tables = (ctypes_vp * 6)(*[e.weight.data_ptr() for e in emb])
        self.ck(self.L.dk_net_embed_ln_f32_async(tok.data_ptr(), B, tables, d, ln0.weight.data_ptr(), ln0.bias.data_ptr(),
                                                 ln0.eps, self.x.data_ptr(), self.h.data_ptr() if need_h else None,
                                                 self.st))

    # The GEMMs run without their bias (hipBLASLt's f32 GEMMs at "medium" take about twice as long
    # with the bias epilogue, profiles/r04/fp32_bias_probe.log); each bias is added, in the
    # epilogue's order (GEMM output + bias, then the next op), by the f32 kernel that reads the
    # GEMM's output.
    def add_ln(self, x, delta, ln, bias=None):
        h = torch.empty_like(x)
        self.ck(self.L.dk_net_add_bias_ln_f32_async(x.data_ptr(), delta.data_ptr() if delta is not None else None,
                                                    bias.data_ptr() if bias is not None else None, self.rows, self.d,
                                                    ln.weight.data_ptr(), ln.bias.data_ptr(), ln.eps, h.data_ptr(),
                                                    self.st))
        return h

    def attn_ln(self, x, blk, h, ln):
        if not (self.d % blk.heads == 0 and self.d // blk.heads in (40, 64)):
            return self.add_ln(x, _f32c(blk.attn_delta(h)), ln)
        if self.d in (160, 256) and blk.heads == 4 and blk.qkv.bias is not None:
            # the whole attention half in one kernel per sample, bf16x3 products (qkv_attn_ln_f32x3_kernel)
            wqh, wql, wph, wpl, bpf = split_attn_bf16x3(blk)
            ho = torch.empty_like(x)
            self.ck(self.L.dk_net_qkv_attn_ln_f32x3_async(h.data_ptr(), x.data_ptr(), wqh.data_ptr(), wql.data_ptr(),
                                                          blk.qkv.bias.data_ptr(), wph.data_ptr(), wpl.data_ptr(),
                                                          bpf.data_ptr(), h.shape[0], 4, self.d // 4, ln.weight.data_ptr(),
                                                          ln.bias.data_ptr(), ln.eps, ho.data_ptr(), self.st))
            return ho
        qkv = _f32c(F.linear(h, blk.qkv.weight))                         # [B, 62, 3d]: q | k | v, heads contiguous
        y = torch.empty_like(h)
        bq = blk.qkv.bias.contiguous() if blk.qkv.bias is not None else None
        self.ck(self.L.dk_net_attn62_bias_f32_async(qkv.data_ptr(), bq.data_ptr() if bq is not None else None,
                                                    y.data_ptr(), h.shape[0], blk.heads, self.d // blk.heads, self.st))
        w, b = blk.folded_proj()
        return self.add_ln(x, _f32c(F.linear(y, w)), ln, b)

    @classmethod
    def chain_ok(cls, d, blocks):
        """True when `run` takes the x-only chain over these blocks of width d (DK_F32_XCHAIN=0: the
        h-in / h-out chain, a measurement switch)."""
        return (d in (160, 256) and len(blocks) > 0 and all(cls.ex_ok(blk) for blk in blocks)
                and os.environ.get("DK_F32_XCHAIN", "1") != "0")

    def chain(self, blocks):
        return self.chain_ok(self.d, blocks)

    def run(self, h, blocks, final_ln, x=None, x_out=None):
        """x_out (x-only chain): the first half reads x and writes the new x to x_out, the rest
        continue in place on x_out -- a branch from a shared trunk's x without copying it."""
        if not self.chain(blocks):
            if x_out is not None:
                x_out.copy_(self.x if x is None else x)
                x = x_out
            return super().run(h, blocks, final_ln, x)
        # d = 256 (round 5) and d = 160 (round 6): every half reads the residual stream x and applies
        # the LayerNorm its producer used to write out as h (the *_ex kernels; at d = 160 also the
        # first half, from x and ln_1); only the last half writes h (the final LayerNorm, for the
        # heads).  Per half, x in and out instead of h in, x in and out, h out.
        x = self.x if x is None else x
        # d = 160: the halves pass each other the new x rows' LayerNorm statistics (mean, 1/std), so
        # that the consumer does not reduce over the row (8 B per row; one buffer, used in place)
        st = torch.empty((x.shape[0] * SEQ, 2), dtype=torch.float32, device=x.device) if self.d == 160 else None
        stp = st.data_ptr() if st is not None else None
        ho = None
        for i, blk in enumerate(blocks):
            wqh, wql, wph, wpl, bpf = split_attn_bf16x3(blk)
            lin = None if (i == 0 and self.d == 256 and h is not None) else blk.ln_1   # (h None: x only)
            self.ck(self.L.dk_net_qkv_attn_ln_f32x3_ex_async(
                h.data_ptr() if lin is None else None, x.data_ptr(), lin.weight.data_ptr() if lin else None,
                lin.bias.data_ptr() if lin else None, lin.eps if lin else 0.0, wqh.data_ptr(), wql.data_ptr(),
                blk.qkv.bias.data_ptr(), wph.data_ptr(), wpl.data_ptr(), bpf.data_ptr(), x.shape[0], 4, self.d // 4, None,
                None, blk.ln_2.eps, None, stp if i > 0 else None, stp,
                x_out.data_ptr() if (i == 0 and x_out is not None) else None, self.st))
            if i == 0 and x_out is not None:
                x = x_out
            last = i + 1 == len(blocks)
            w1h, w1l, w2h, w2l = split_bf16x3(blk)
            wh = last and final_ln is not None   # (final_ln None: no h at all)
            ho = torch.empty_like(x) if wh else None
            nxt_eps = blocks[i + 1].ln_1.eps if not last else (final_ln.eps if final_ln is not None else 1e-5)
            self.ck(self.L.dk_net_mlp_ln_f32x3_ex_async(
                None, x.data_ptr(), blk.ln_2.weight.data_ptr(), blk.ln_2.bias.data_ptr(), blk.ln_2.eps, w1h.data_ptr(),
                w1l.data_ptr(), blk.fc.bias.data_ptr(), w2h.data_ptr(), w2l.data_ptr(), blk.proj.bias.data_ptr(), self.rows,
                self.d, blk.fc.weight.shape[0], final_ln.weight.data_ptr() if wh else None,
                final_ln.bias.data_ptr() if wh else None, final_ln.eps if wh else nxt_eps,
                ho.data_ptr() if wh else None, stp, stp if not last else None, self.st))
        return ho

    @staticmethod
    def ex_ok(blk):
        n = blk.fc.weight.shape[0]
        return (blk.heads == 4 and blk.qkv.bias is not None and n % 64 == 0 and n <= 1024 and blk.fc.bias is not None
                and blk.proj.bias is not None and blk.ln_1.weight is not None and blk.ln_2.weight is not None)

    def mlp_ln(self, x, blk, h, ln):
        n = blk.fc.weight.shape[0]
        if self.d in (160, 256) and n % (64 if self.d == 256 else 32) == 0 and n <= 1024 and blk.fc.bias is not None and blk.proj.bias is not None:
            # the whole MLP half in one kernel, bf16x3 products (mlp_ln_f32x3_kernel)
            w1h, w1l, w2h, w2l = split_bf16x3(blk)
            ho = torch.empty_like(x)
            self.ck(self.L.dk_net_mlp_ln_f32x3_async(h.data_ptr(), x.data_ptr(), w1h.data_ptr(), w1l.data_ptr(),
                                                     blk.fc.bias.data_ptr(), w2h.data_ptr(), w2l.data_ptr(),
                                                     blk.proj.bias.data_ptr(), self.rows, self.d, n, ln.weight.data_ptr(),
                                                     ln.bias.data_ptr(), ln.eps, ho.data_ptr(), self.st))
            return ho
        a = _f32c(F.linear(h, blk.fc.weight))
        b1 = blk.fc.bias.contiguous() if blk.fc.bias is not None else None
        self.ck(self.L.dk_net_gelu_bias_f32_async(a.data_ptr(), b1.data_ptr() if b1 is not None else None, a.numel(),
                                                  a.shape[-1], self.st))
        return self.add_ln(x, _f32c(F.linear(a, blk.proj.weight)), ln, blk.proj.bias)


class DokoAzNet(nn.Module):
    def __init__(self, d=160, heads=4, layers=4, policy_layers=1, value_layers=1):
        super().__init__()
        self.emb = nn.ModuleList([nn.Embedding(v, d) for v in VOCAB])
        self.blocks = nn.ModuleList([Block(d, heads) for _ in range(layers)])
        self.p_blocks = nn.ModuleList([Block(d, heads) for _ in range(policy_layers)])
        self.v_blocks = nn.ModuleList([Block(d, heads) for _ in range(value_layers)])
        self.p_ln = nn.LayerNorm(d)
        self.v_ln = nn.LayerNorm(d)
        self.value_head = ClassHead(d, 4)
        self.policy_head = ClassHead(d, 39)

    def forward(self, tokens):                                   # int32/int64 [B, 311]
        if tokens.is_cuda and self.emb[0].weight.dtype == torch.bfloat16:
            return self.forward_fused(tokens)
        if f32_fused_ok(tokens, self.emb[0].weight):
            return self.forward_fused(tokens, FusedTrunkF32)
        return self.forward_torch(tokens)

    def forward_torch(self, tokens):
        """The plain module forward (reference structure; any device and dtype, autograd)."""
        t = tokens.long()
        x = sum(self.emb[i](t[:, SEQ * i:SEQ * (i + 1)]) for i in range(5)) + self.emb[5](t[:, 310:311])
        for blk in self.blocks:
            x = blk(x)
        xp, xv = x, x
        for blk in self.p_blocks:
            xp = blk(xp)
        for blk in self.v_blocks:
            xv = blk(xv)
        return self.value_head(self.v_ln(xv), fused=False), self.policy_head(self.p_ln(xp), fused=False)

    def forward_fused(self, tokens, trunk=None):
        """bf16 forward on the GPU with HIP kernels (csrc/az_net_kernels.h): the embedding
        sum + first LayerNorm, each block as two kernels (the attention half from the qkv
        projection to the next LayerNorm, the MLP half likewise: FusedTrunk), and the heads'
        attention pooling + per-class LayerNorm (ClassHead.pooled).  trunk=FusedTrunkF32: the
        f32 forward (reference precision)."""
        if not (self.blocks and self.p_blocks and self.v_blocks):
            raise ValueError("the fused forward needs shared, policy and value blocks")
        # (f32 at d = 160: every half normalises x itself, so neither the embedding nor the branch
        # inputs need an h)
        d = self.emb[0].weight.shape[1]
        x_only = trunk is FusedTrunkF32 and d == 160 and all(FusedTrunkF32.chain_ok(d, b) for b in
                                                             (self.blocks, self.p_blocks, self.v_blocks))
        f = trunk(tokens, self.emb, self.blocks[0].ln_1, need_h=False) if x_only else \
            (trunk or FusedTrunk)(tokens, self.emb, self.blocks[0].ln_1)
        hp = f.run(f.h, self.blocks, None if x_only else self.p_blocks[0].ln_1)   # f.x: the shared trunk's output
        if x_only:
            # the value branch first, its first half writing a new x (the trunk's x stays for the
            # policy branch, no copy); then the policy branch in place on the trunk's x
            hv = f.run(None, self.v_blocks, self.v_ln, x_out=torch.empty_like(f.x))
            hp = f.run(hp, self.p_blocks, self.p_ln)
            return self.value_head(hv), self.policy_head(hp)
        xv = f.x.clone()
        hv = f.add_ln(xv, None, self.v_blocks[0].ln_1)
        hp = f.run(hp, self.p_blocks, self.p_ln)
        hv = f.run(hv, self.v_blocks, self.v_ln, x=xv)
        return self.value_head(hv), self.policy_head(hp)

    @torch.no_grad()
    def load_reference_state_dict(self, sd):
        """Map a state_dict of the reference AlphaZeroTicTacToeNetwork onto this module
        (load it with torch.load(path, weights_only=True))."""
        names = ["game_object_e", "position_e", "player_played_e", "subposition_e", "team_e", "phase_e"]
        for i, n in enumerate(names):
            self.emb[i].weight.copy_(sd["transformer.%s.weight" % n])

        for group, mods in (("h", self.blocks), ("p_h", self.p_blocks), ("v_h", self.v_blocks)):
            for i, m in enumerate(mods):
                m.load_reference(sd, "transformer.%s.%d." % (group, i))
        for ln, n in ((self.p_ln, "p_ln_f"), (self.v_ln, "v_ln_f")):
            ln.weight.copy_(sd["transformer.%s.weight" % n]); ln.bias.copy_(sd["transformer.%s.bias" % n])
        for head, n in ((self.value_head, "value_head"), (self.policy_head, "policy_head")):
            head.queries.copy_(sd[n + ".card_queries"])
            for c in range(head.queries.shape[0]):
                pre = "%s.mlps.%d." % (n, c)
                head.ln_w[c].copy_(sd[pre + "0.weight"]); head.ln_b[c].copy_(sd[pre + "0.bias"])
                head.w1[c].copy_(sd[pre + "1.weight"]); head.b1[c].copy_(sd[pre + "1.bias"])
                head.w2[c].copy_(sd[pre + "3.weight"][0]); head.b2[c].copy_(sd[pre + "3.bias"][0])


class AzEvaluator:
    """The network as AlphaZeroSearch's `network` callable: dk_az_state records ->
    device encoder (az_encode) -> DokoAzNet -> (value f32 [n, 4], logits f32 [n, 39]).  dtype
    float32 (default) is the reference's precision (az_doko.py:379-400, 539-541: f32 activations,
    matmul precision "medium"); torch.bfloat16 runs the narrower bf16 kernels."""

    def __init__(self, engine, net, dtype=torch.float32):
        self.engine = engine
        self.net = net.eval().to(dtype)
        self.dtype = dtype
        self._tok = None

    @torch.inference_mode()
    def __call__(self, records):
        from .api import az_encode
        n = records.shape[0]
        if self._tok is None or self._tok.shape[0] < n:
            self._tok = torch.empty((n, 311), dtype=torch.int32, device=records.device)
        tok = az_encode(self.engine, records, self._tok[:n])
        v, p = self.net(tok)
        return v.float(), p.float()
