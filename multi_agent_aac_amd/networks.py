"""Actor / critic of the ``one_model_att`` MADDPG on PyTorch-ROCm + HIP attention.

ActorNetwork_ATT_TwoPortion  ATT/nets:177-213, same layer names and init order, so its
                             ``reference_state_dict()`` is a drop-in ``.pth`` for the reference
                             actor (ATT/maddpg:131-139).  k and v are stored fused as one
                             (128, 64) weight (one GEMM instead of two) and split on export.
CriticCombine                the canonical N-agent form of critic_combine_ignore_radar
                             (ATT/nets:672-724, hard-wired to 8 agents there; contract R3): one
                             encoder Linear(D0+2, 128) per agent index -> concat -> 256 -> 1,
                             radar ignored.  The N encoders are one stacked batched GEMM.

All parameters of a network live in one flat fp32 buffer (``FlatParams``) with a matching flat
gradient buffer, so Adam, Polyak and the RCCL gradient all-reduce are single launches.
"""
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import IDENTITY, RELU, TANH, GradSlot, fused_linear, stacked_linear_relu
from .ops import masked_attention


class FlatParams:
    """Re-point every parameter of ``module`` (already on its device) into one flat buffer.

    ``grad`` is a flat buffer too and each ``param.grad`` is a view into it, so autograd
    accumulates in place and ``grad.zero_()`` is the whole ``zero_grad``.
    """

    def __init__(self, module):
        params = list(module.parameters())
        n = sum(p.numel() for p in params)
        dev = params[0].device
        self.data = torch.zeros(n, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n, device=dev, dtype=torch.float32)
        self.slices = []
        off = 0
        for p in params:
            k = p.numel()
            self.data[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.data[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            self.slices.append((p, off, k))
            off += k
        self.numel = n

    def zero_grad(self):
        self.grad.zero_()


def _rows(x, tail):
    return x.reshape(-1, *tail)


class ActorNetwork_ATT_TwoPortion(nn.Module):
    """Attention actor; inputs [own (.., D0), radar (.., 18), nei (.., K, 6)] -> tanh(2)."""

    def __init__(self, actor_dim, n_actions):
        super().__init__()
        self.actor_dim = list(actor_dim)
        self.own_fc = nn.Sequential(nn.Linear(actor_dim[0], 64), nn.ReLU())
        self.own_grid = nn.Sequential(nn.Linear(actor_dim[1], 64), nn.ReLU())
        self.neigh_fc = nn.Sequential(nn.Linear(actor_dim[2], 64), nn.ReLU())
        self.merge_feature = nn.Sequential(nn.Linear(64 + 64 + 64, 256), nn.ReLU())
        self.act_out = nn.Sequential(nn.Linear(256, n_actions), nn.Tanh())
        k = nn.Linear(64, 64, bias=False)     # init order k, q, v as ATT/nets:187-189
        self.q = nn.Linear(64, 64, bias=False)
        v = nn.Linear(64, 64, bias=False)
        self.kv_weight = nn.Parameter(torch.cat([k.weight.data, v.weight.data], 0))
        self.slot = GradSlot()

    def forward(self, cur_state):
        own, grid, nei = cur_state[0], cur_state[1], cur_state[2]
        lead = own.shape[:-1]
        K = nei.shape[-2]
        own = _rows(own, (own.shape[-1],))
        grid = _rows(grid, (grid.shape[-1],))
        nei = _rows(nei, (K, nei.shape[-1]))
        s = self.slot
        R = own.shape[0]
        e_o = fused_linear(own, self.own_fc[0].weight, self.own_fc[0].bias, RELU, s)
        e_g = fused_linear(grid, self.own_grid[0].weight, self.own_grid[0].bias, RELU, s)
        x = fused_linear(nei.reshape(R * K, -1), self.neigh_fc[0].weight, self.neigh_fc[0].bias, RELU, s)
        q = fused_linear(e_o, self.q.weight, None, IDENTITY, s)
        kv = fused_linear(x, self.kv_weight, None, IDENTITY, s).view(R, K, 128)
        v_att = masked_attention(q, kv, nei)
        h = fused_linear(torch.cat((e_o, e_g, v_att), dim=1), self.merge_feature[0].weight,
                         self.merge_feature[0].bias, RELU, s)
        out = fused_linear(h, self.act_out[0].weight, self.act_out[0].bias, TANH, s)
        return out.reshape(*lead, out.shape[-1])

    # .pth compatibility with the reference actor (keys of ATT/nets:180-189)
    def reference_state_dict(self):
        sd = OrderedDict()
        for name in ("own_fc", "own_grid", "neigh_fc", "merge_feature", "act_out"):
            lin = getattr(self, name)[0]
            sd[f"{name}.0.weight"] = lin.weight.detach().cpu().clone()
            sd[f"{name}.0.bias"] = lin.bias.detach().cpu().clone()
        sd["k.weight"] = self.kv_weight[:64].detach().cpu().clone()
        sd["q.weight"] = self.q.weight.detach().cpu().clone()
        sd["v.weight"] = self.kv_weight[64:].detach().cpu().clone()
        return sd

    @torch.no_grad()
    def load_reference_state_dict(self, sd):
        for name in ("own_fc", "own_grid", "neigh_fc", "merge_feature", "act_out"):
            lin = getattr(self, name)[0]
            lin.weight.copy_(sd[f"{name}.0.weight"])
            lin.bias.copy_(sd[f"{name}.0.bias"])
        self.kv_weight[:64].copy_(sd["k.weight"])
        self.q.weight.copy_(sd["q.weight"])
        self.kv_weight[64:].copy_(sd["v.weight"])


class CriticCombine(nn.Module):
    """Centralised critic over N agents: per-agent encoders on [own_i, a_i] (radar ignored)."""

    def __init__(self, critic_obs, n_agents, n_actions, hidden=128):
        super().__init__()
        self.n_agents = n_agents
        encs = [nn.Linear(critic_obs[0] + n_actions, hidden) for _ in range(n_agents)]
        self.enc_w = nn.Parameter(torch.stack([e.weight.data for e in encs]))   # (N, 128, D0+2)
        self.enc_b = nn.Parameter(torch.stack([e.bias.data for e in encs]))     # (N, 128)
        self.combine_agents_fea = nn.Sequential(nn.Linear(hidden * n_agents, 256), nn.ReLU())
        self.out_feature_q = nn.Sequential(nn.Linear(256, 1))
        self.slot = GradSlot()

    def forward(self, combine_state, combine_action):
        own = combine_state[0]                       # (B, N, D0)
        if isinstance(combine_action, (list, tuple)):
            combine_action = torch.stack(list(combine_action), 1)
        x = torch.cat((own, combine_action), dim=-1)            # (B, N, D0+2)
        s = self.slot
        f = stacked_linear_relu(x, self.enc_w, self.enc_b, s)   # (B, N*128), agent-major features
        h = fused_linear(f, self.combine_agents_fea[0].weight, self.combine_agents_fea[0].bias, RELU, s)
        return fused_linear(h, self.out_feature_q[0].weight, self.out_feature_q[0].bias, IDENTITY, s)

    def reference_state_dict(self):
        sd = OrderedDict()
        for i in range(self.n_agents):
            sd[f"o{i + 1}a{i + 1}.0.weight"] = self.enc_w[i].detach().cpu().clone()
            sd[f"o{i + 1}a{i + 1}.0.bias"] = self.enc_b[i].detach().cpu().clone()
        for name in ("combine_agents_fea", "out_feature_q"):
            lin = getattr(self, name)[0]
            sd[f"{name}.0.weight"] = lin.weight.detach().cpu().clone()
            sd[f"{name}.0.bias"] = lin.bias.detach().cpu().clone()
        return sd

    @torch.no_grad()
    def load_reference_state_dict(self, sd):
        for i in range(self.n_agents):
            self.enc_w[i].copy_(sd[f"o{i + 1}a{i + 1}.0.weight"])
            self.enc_b[i].copy_(sd[f"o{i + 1}a{i + 1}.0.bias"])
        for name in ("combine_agents_fea", "out_feature_q"):
            lin = getattr(self, name)[0]
            lin.weight.copy_(sd[f"{name}.0.weight"])
            lin.bias.copy_(sd[f"{name}.0.bias"])
