"""The IMPI (autoregressive determinization) network, inference side.

Architecture of ImperfectInformationNetwork (rs-doko-py-bridge/python/main.py:99-138, with
TransformerBlock.py / SelfAttention.py; PerClassAttentionMLPHead :25-55).  The configuration
the comparison runs load is create_ar.py:12-18: n_embd 256, 4 layers, 4 heads.

    tokens [B, 311] = 5 x 62 token rows + the player to guess for (encode_state_ipi)
    x = E_obj[t0] + E_pos[t1] + E_player[t2] + E_subpos[t3] + E_team[t4] + E_guess[t5]   [B, 62, d]
    blocks: x += c_proj(MHA(LN1 x));  x += W2 GELU(W1 LN2 x)
    ln_f, then the per-class attention head over 33 classes
    logits [B, 33] (ImperfectInformationOutput: 9 reservations, then the 24 cards)

The bf16 GPU forward reuses the AlphaZero network's fused trunk (az_network.FusedTrunk):
the embedding sum and every residual add run fused with their LayerNorm in HIP kernels.
Weights are random-initialised (no checkpoint ships with the reference);
load_reference_state_dict maps a reference state_dict onto this module.
"""
import torch
from torch import nn

from .az_network import SEQ, Block, ClassHead, FusedTrunk, FusedTrunkF32, f32_fused_ok

VOCAB_IPI = (43, 57, 5, 13, 3, 5)   # object, position, player, subposition, team, player to guess (main.py:91-96)
IPI_CLASSES = 33


class DokoImpiNet(nn.Module):
    def __init__(self, d=256, heads=4, layers=4):
        super().__init__()
        self.emb = nn.ModuleList([nn.Embedding(v, d) for v in VOCAB_IPI])
        self.blocks = nn.ModuleList([Block(d, heads) for _ in range(layers)])
        self.ln_f = nn.LayerNorm(d)
        self.head = ClassHead(d, IPI_CLASSES)

    def forward(self, tokens):                                   # int32/int64 [B, 311] -> [B, 33]
        if tokens.is_cuda and self.emb[0].weight.dtype == torch.bfloat16:
            return self.forward_fused(tokens)
        if f32_fused_ok(tokens, self.emb[0].weight):
            return self.forward_fused(tokens, FusedTrunkF32)
        return self.forward_torch(tokens)

    def forward_torch(self, tokens):
        t = tokens.long()
        x = sum(self.emb[i](t[:, SEQ * i:SEQ * (i + 1)]) for i in range(5)) + self.emb[5](t[:, 310:311])
        for blk in self.blocks:
            x = blk(x)
        return self.head(self.ln_f(x), fused=False)

    def forward_fused(self, tokens, trunk=None):
        d = self.emb[0].weight.shape[1]
        if trunk is FusedTrunkF32 and FusedTrunkF32.chain_ok(d, self.blocks):
            # x-only chain: the embedding writes x alone and the first half normalises it itself
            f = trunk(tokens, self.emb, self.blocks[0].ln_1, need_h=False)
            return self.head(f.run(None, self.blocks, self.ln_f))
        f = (trunk or FusedTrunk)(tokens, self.emb, self.blocks[0].ln_1)
        return self.head(f.run(f.h, self.blocks, self.ln_f))

    @torch.no_grad()
    def load_reference_state_dict(self, sd):
        """Map a state_dict of the reference ImperfectInformationNetwork onto this module
        (load it with torch.load(path, weights_only=True))."""
        names = ["game_object_e", "position_e", "player_played_e", "subposition_e", "team_e", "player_guess_e"]
        for i, n in enumerate(names):
            self.emb[i].weight.copy_(sd["transformer.%s.weight" % n])
        for i, m in enumerate(self.blocks):
            m.load_reference(sd, "transformer.h.%d." % i)
        self.ln_f.weight.copy_(sd["transformer.ln_f.weight"]); self.ln_f.bias.copy_(sd["transformer.ln_f.bias"])
        self.head.queries.copy_(sd["lm_head.card_queries"])
        for c in range(IPI_CLASSES):
            pre = "lm_head.mlps.%d." % c
            self.head.ln_w[c].copy_(sd[pre + "0.weight"]); self.head.ln_b[c].copy_(sd[pre + "0.bias"])
            self.head.w1[c].copy_(sd[pre + "1.weight"]); self.head.b1[c].copy_(sd[pre + "1.bias"])
            self.head.w2[c].copy_(sd[pre + "3.weight"][0]); self.head.b2[c].copy_(sd[pre + "3.bias"][0])
