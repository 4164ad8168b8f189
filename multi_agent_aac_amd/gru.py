"""GRU-actor MADDPG on the device: SURVEY.md section 8(f) row f2 (config 4, ``randomOD_gru_radar``).

Reference: MADDPG_ownENV_randomOD_Wgru_radar (``WGRU/`` below):
  GRUCELL_actor_TwoPortion           WGRU/Nnetworks_randomOD_Wgru_radar.py:181-198
  critic_single_obs_wGRU_TwoPortion  WGRU/Nnetworks_randomOD_Wgru_radar.py:428-446
  MADDPG (one actor and one critic per agent, per-agent Adam)      WGRU/maddpg_agent_*.py:31-92
  update_myown                       WGRU/maddpg_agent_*.py:211-326
  choose_action (hidden carried per agent)                         WGRU/maddpg_agent_*.py:336-428
  save_model / load_model            WGRU/maddpg_agent_*.py:94-131
  replay rows with cur_hidden / next_hidden                        WGRU/ma_main_*.py:601-647

MI355X layout.  The N agents' networks of one kind live in one flat fp32 buffer, agent-major
(``AgentStack`` + ``FlatParams``), so Adam, Polyak and the RCCL all-reduce stay single launches.
Every batch tensor is sample-major ``[rows][N][width]``: agent i's operand of a per-agent product is
the same tensor at column offset i*width with leading dimension N*width, so the N agents' products
of one layer are ONE grouped-GEMM launch (``aac_gemm_batch``) and the GRU cells of all agents are
ONE ``aac_gru_cell`` launch (row r = b*N + i).  The reference's loop over agents touches disjoint
networks with a read-only batch, so one step of all agents at once is the same update.

update_myown as a launch list (one HIP graph; ``GruUpdate``):
  sample + gather                                   replay kernels
  target actor  enc | gates | GRU fwd + pack [own'|a']     grouped GEMM x2 + aac_gru_cell
  target critic enc | gates | GRU TD target        grouped GEMM x2 + aac_gru_cell
  critic step   pack [own|a] | enc | gates | GRU (q, 2(q-y)/B, gate backward) |
                dW_out, dW_ih, dW_hh, d cat | dW_sa, dW_grid | Adam
  actor step    enc | gates | GRU fwd + pack [own|pi] | critic enc | gates |
                GRU (-1/B, gate backward) | d SA | d a | GRU actor backward |
                dW_out, dW_ih, dW_hh, d cat | dW_own, dW_grid | Adam
  Polyak (both targets)
"""
import ctypes
import os
from copy import deepcopy

import numpy as np
import torch
import torch.nn as nn

from . import fused, ops, parallel, trace
from .fused import RELU, TANH, Collective, gemm_launches, prob, ptr
from .memory import DeviceReplay, Experience, ReplayMemory
from .networks import FlatParams

H = 64
vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
FWD, TD, CRITIC, ACTLOSS, ACTBWD = 0, 1, 2, 3, 4


class GruArgs(ctypes.Structure):
    """aac_gru_args (include/aac_gru.h)."""
    _fields_ = [("gi", vp), ("gh", vp), ("ldg", i32), ("h", vp), ("ldh", i32), ("wout", vp), ("bout", vp),
                ("wstride", i32), ("bstride", i32), ("O", i32), ("act", i32), ("R", i32), ("N", i32), ("mode", i32),
                ("hout", vp), ("ldho", i32), ("y", vp), ("ldy", i32), ("pack_src", vp), ("ld_pack_src", i32),
                ("npack", i32), ("pack_dst", vp), ("ld_pack_dst", i32), ("target", vp), ("rew", vp), ("done", vp),
                ("gamma", f32), ("inv_m", f32), ("yout", vp), ("da", vp), ("ldda", i32), ("dq", vp), ("dgi", vp),
                ("dgh", vp), ("ldd", i32), ("dsa", vp), ("lddsa", i32), ("wsa", vp), ("wsa_stride", i32),
                ("ldwsa", i32), ("wsa_col", i32)]


class GruActorArgs(ctypes.Structure):
    """aac_gru_actor_args (include/aac_gru.h)."""
    _fields_ = [("own", vp), ("ld_own", i32), ("d_own", i32), ("radar", vp), ("ld_radar", i32), ("h", vp),
                ("ldh", i32)] + [(k, vp) for k in ("Wo", "bo", "Wg", "bg", "Wih", "bih", "Whh", "bhh", "Wout", "bout")] + \
               [("pstride", i32), ("E", i32), ("N", i32), ("hout", vp), ("ldho", i32), ("y", vp), ("ldy", i32),
                ("cat", vp), ("gi", vp), ("gh", vp), ("ldc", i32), ("ldg", i32),
                ("noisy", i32), ("episode", vp), ("eps_end", i32), ("noise_start", f32), ("noise_end", f32),
                ("seed", ctypes.c_uint64), ("counter", vp), ("noise_out", vp)]


# weights-stationary aac_gru_actor_fwd: the act path as one launch instead of the encoder and gate
# GEMM launches + aac_gru_cell, and in update_myown each network evaluation's encoder + gate GEMM
# launches as one launch (projection mode); AAC_GRU_WS=0 keeps the grouped-GEMM launches
ACT_WS = os.environ.get("AAC_GRU_WS", "1") == "1"
# the projection mode in update_myown (one launch per network evaluation instead of the encoder and
# gate GEMM launches): config 4 0.463 -> 0.402 ms per step; AAC_GRU_WS_PROJ=0 keeps the GEMM launches
WS_PROJ = ACT_WS and os.environ.get("AAC_GRU_WS_PROJ", "1") == "1"
# the three projections that read only the batch (target actor on s', critic on (s, a), actor on s)
# in one aac_gru_actor_proj_multi launch; AAC_GRU_MULTI_PROJ=0: three launches
MULTI_PROJ = os.environ.get("AAC_GRU_MULTI_PROJ", "1") == "1"
# the actor step's d a (critic input layer backward, 64 -> 2 per row) inside the ACTBWD cell launch;
# AAC_GRU_CELL_DA=0: a grouped-GEMM launch of N products
CELL_DA = os.environ.get("AAC_GRU_CELL_DA", "1") == "1"
# the two forward cells (target actor, actor) in one launch, and the TD cell with the critic's mse cell
# chained per row (aac_gru_cell2); AAC_GRU_CELL_PAIRS=0: four launches
CELL_PAIRS = os.environ.get("AAC_GRU_CELL_PAIRS", "1") == "1"
_WS_NAMES = ("Wo", "bo", "Wg", "bg", "Wih", "bih", "Whh", "bhh", "Wout", "bout")


def _agent_stride(P, stride):
    """The agent stacks are agent-major flat buffers: agent i's parameters at agent 0's + i * stride."""
    for i in range(len(P)):
        assert all(P[i][k] == P[0][k] + 4 * i * stride for k in _WS_NAMES)
    return stride


class WsProj:
    """enc2_probs + gate_probs of one network evaluation (cat, gi, gh of M samples x N agents) as one
    aac_gru_actor_fwd launch in projection mode."""

    def __init__(self, P, stride, X1, w1, k1, radar, h, cat, gi, gh, M, N):
        self.args = GruActorArgs(X1, w1, k1, radar, 18, h, H, *[P[0][k] for k in _WS_NAMES],
                                 _agent_stride(P, stride), M, N, None, 0, None, 0, cat, gi, gh, 128, 192)
        self.flops = 2 * M * N * (64 * k1 + 64 * 18 + 192 * 128 + 192 * H)     # 2 M N K of the four products

    def __call__(self):
        _chk(glib().aac_gru_actor_fwd(ctypes.byref(self.args), fused._stream()), "aac_gru_actor_fwd")


class WsProjMulti:
    """Up to three independent WsProj evaluations in one aac_gru_actor_proj_multi launch."""

    def __init__(self, projs):
        self.projs = projs
        self.arr = (GruActorArgs * len(projs))(*[q.args for q in projs])
        self.flops = sum(q.flops for q in projs)

    def __call__(self):
        _chk(glib().aac_gru_actor_proj_multi(self.arr, len(self.projs), fused._stream()), "aac_gru_actor_proj_multi")

_GL = None


def glib():
    global _GL
    if _GL is None:
        L = fused.lib()
        L.aac_gru_last_error.restype = ctypes.c_char_p
        L.aac_gru_cell.argtypes = [ctypes.POINTER(GruArgs), vp]
        L.aac_pack_rows.argtypes = [vp, i32, vp, i32, i32, vp, i32, i32, i32, vp]
        L.aac_gru_reset_hidden.argtypes = [vp, i32, i32, vp, vp]
        L.aac_gru_actor_fwd.argtypes = [ctypes.POINTER(GruActorArgs), vp]
        L.aac_gru_actor_proj_multi.argtypes = [ctypes.POINTER(GruActorArgs), i32, vp]
        L.aac_gru_cell2.argtypes = [ctypes.POINTER(GruArgs), ctypes.POINTER(GruArgs), i32, vp]
        _GL = L
    return _GL


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {glib().aac_gru_last_error().decode(errors='replace')}")


class GruCell:
    """One aac_gru_cell launch with fixed arguments (graph-capturable)."""

    def __init__(self, **kw):
        self.args = GruArgs(**kw)

    def __call__(self):
        _chk(glib().aac_gru_cell(ctypes.byref(self.args), fused._stream()), "aac_gru_cell")


class GruCell2:
    """Two GruCell argument sets in one aac_gru_cell2 launch (independent, or TD -> CRITIC chained)."""

    def __init__(self, c0, c1, chain):
        self.c = (c0, c1)
        self.chain = int(chain)

    def __call__(self):
        _chk(glib().aac_gru_cell2(ctypes.byref(self.c[0].args), ctypes.byref(self.c[1].args), self.chain,
                                  fused._stream()), "aac_gru_cell2")


def pack_rows(dst, ldd, a, lda, n0, b, ldb, n1, R):
    _chk(glib().aac_pack_rows(vp(dst), ldd, vp(a), lda, n0, vp(b), ldb, n1, R, fused._stream()), "aac_pack_rows")


def reset_hidden(h, env_done):
    """Zero the hidden states of the envs whose episode ended (h: (E, N, H), env_done: (E,) u8)."""
    E = h.shape[0]
    _chk(glib().aac_gru_reset_hidden(vp(h.data_ptr()), E, h[0].numel(), vp(env_done.data_ptr()), fused._stream()),
         "aac_gru_reset_hidden")


# =============================================================================== networks
class GRUCELL_actor_TwoPortion(nn.Module):
    """WGRU/Nnetworks:181-198 (same layer names, so ``state_dict`` is the reference's .pth)."""

    def __init__(self, actor_dim, n_actions, actor_hidden_state_size=H):
        super().__init__()
        assert actor_hidden_state_size == H, "the GRU row kernel is built for 64 hidden units"
        self.own_fc = nn.Sequential(nn.Linear(actor_dim[0], 64), nn.ReLU())
        self.own_grid = nn.Sequential(nn.Linear(actor_dim[1], 64), nn.ReLU())
        self.rnn_hidden_dim = actor_hidden_state_size
        self.gru_cell = nn.GRUCell(64 + 64, actor_hidden_state_size)
        self.outlay = nn.Sequential(nn.Linear(64, n_actions), nn.Tanh())

    @torch.no_grad()
    def forward(self, cur_state, history_hidden_state):
        """(action, h') for rows of [own, grid] on the device path (inference; no autograd)."""
        own, grid = cur_state[0].contiguous(), cur_state[1].contiguous()
        h = history_hidden_state.reshape(-1, H).contiguous()
        R = own.shape[0]
        dev = own.device
        cat, gi, gh = (torch.empty(R, w, device=dev) for w in (128, 192, 192))
        a, hn = torch.empty(R, 2, device=dev), torch.empty(R, H, device=dev)
        P = [param_addrs(self, ACTOR_PARAMS)]
        for L in gemm_launches(enc2_probs(P, "Wo", "bo", "Wg", "bg", ptr(own), own.shape[1], own.shape[1],
                                          ptr(grid), grid.shape[1], grid.shape[1], ptr(cat), R, 1)):
            L()
        for L in gemm_launches(gate_probs(P, ptr(cat), ptr(h), ptr(gi), ptr(gh), R, 1)):
            L()
        gru_cell(P, "Wout", "bout", 0, 2, TANH, ptr(gi), ptr(gh), ptr(h), R, 1, FWD, hout=ptr(hn), y=ptr(a), ldy=2)()
        return a, hn


class critic_single_obs_wGRU_TwoPortion(nn.Module):
    """WGRU/Nnetworks:428-446 (same layer names)."""

    def __init__(self, critic_obs, n_agents, n_actions, single_history=None, hidden_state_size=H):
        super().__init__()
        assert hidden_state_size == H, "the GRU row kernel is built for 64 hidden units"
        self.SA_fc = nn.Sequential(nn.Linear(critic_obs[0] + n_actions, 64), nn.ReLU())
        self.SA_grid = nn.Sequential(nn.Linear(critic_obs[1], 64), nn.ReLU())
        self.rnn_hidden_dim = hidden_state_size
        self.gru_cell = nn.GRUCell(64 + 64, hidden_state_size)
        self.own_fc_outlay = nn.Linear(64, 1)


ACTOR_PARAMS = {"Wo": "own_fc.0.weight", "bo": "own_fc.0.bias", "Wg": "own_grid.0.weight", "bg": "own_grid.0.bias",
                "Wih": "gru_cell.weight_ih", "Whh": "gru_cell.weight_hh", "bih": "gru_cell.bias_ih",
                "bhh": "gru_cell.bias_hh", "Wout": "outlay.0.weight", "bout": "outlay.0.bias"}
CRITIC_PARAMS = {"Wo": "SA_fc.0.weight", "bo": "SA_fc.0.bias", "Wg": "SA_grid.0.weight", "bg": "SA_grid.0.bias",
                 "Wih": "gru_cell.weight_ih", "Whh": "gru_cell.weight_hh", "bih": "gru_cell.bias_ih",
                 "bhh": "gru_cell.bias_hh", "Wout": "own_fc_outlay.weight", "bout": "own_fc_outlay.bias"}


def param_addrs(module, names, flat=None, base=None):
    """{short name: device address} of ``module``'s parameters, or of the same offsets inside
    another buffer of ``flat``'s layout when ``base`` (e.g. the flat gradient) is given."""
    p = dict(module.named_parameters())
    if base is None:
        return {k: p[v].data_ptr() for k, v in names.items()}
    d0 = flat.data.data_ptr()
    return {k: base + (p[v].data_ptr() - d0) for k, v in names.items()}


class AgentStack(nn.Module):
    """N networks of one class in one flat buffer (agent-major, ``FlatParams``)."""

    def __init__(self, nets):
        super().__init__()
        self.nets = nn.ModuleList(nets)

    def __getitem__(self, i):
        return self.nets[i]

    def __len__(self):
        return len(self.nets)


def stack_addrs(stack, names, flat, grad=False):
    base = flat.grad.data_ptr() if grad else None
    return [param_addrs(n, names, flat, base) for n in stack.nets]


# =============================================================================== launch builders
# rows are sample-major [M][N][w]: agent i's operand = base + 4*i*w with leading dimension N*w
def enc2_probs(P, W1, b1, W2, b2, X1, w1, k1, X2, w2, k2, cat, M, N):
    """cat[:, i, 0:64] = relu(X1_i W1_i^T + b1_i), cat[:, i, 64:128] = relu(X2_i W2_i^T + b2_i)."""
    out = []
    for i in range(N):
        out.append(prob(X1 + 4 * i * w1, P[i][W1], cat + 4 * i * 128, M, 64, k1, N * w1, k1, N * 128, tb=1,
                        bias=P[i][b1], act=RELU))
        out.append(prob(X2 + 4 * i * w2, P[i][W2], cat + 4 * i * 128 + 4 * 64, M, 64, k2, N * w2, k2, N * 128, tb=1,
                        bias=P[i][b2], act=RELU))
    return out


def gate_probs(P, cat, h, gi, gh, M, N):
    """gi = cat W_ih^T + b_ih, gh = h W_hh^T + b_hh (both [M][N][192])."""
    out = []
    for i in range(N):
        out.append(prob(cat + 4 * i * 128, P[i]["Wih"], gi + 4 * i * 192, M, 192, 128, N * 128, 128, N * 192, tb=1,
                        bias=P[i]["bih"]))
        out.append(prob(h + 4 * i * H, P[i]["Whh"], gh + 4 * i * 192, M, 192, H, N * H, H, N * 192, tb=1,
                        bias=P[i]["bhh"]))
    return out


def gru_cell(P, Wout, bout, stride, O, act, gi, gh, h, M, N, mode, **kw):
    """aac_gru_cell over R = M*N rows; agent i's output layer at P[0][Wout] + i*stride floats."""
    for k, v in (("ldho", H), ("ldy", O), ("ldd", 192), ("ldda", O)):
        kw.setdefault(k, v)
    return GruCell(gi=gi, gh=gh, ldg=192, h=h, ldh=H, wout=P[0][Wout], bout=P[0][bout], wstride=stride,
                   bstride=stride, O=O, act=act, R=M * N, N=N, mode=mode, **kw)


def wgrad_probs(G, g_off, gw, X, x_off, xw, k, Pg, Wn, bn, M, rows, N):
    """dW_i | db_i = G_i^T X_i over ``rows`` samples: G [rows][N][gw] (cols g_off..g_off+M),
    X [rows][N][xw] (cols x_off..x_off+k)."""
    return [prob(G + 4 * (i * gw + g_off), X + 4 * (i * xw + x_off), Pg[i][Wn], M, k, rows, N * gw, N * xw, k, ta=1,
                 ones=1, cextra=Pg[i][bn]) for i in range(N)]


# The learner's grouped-GEMM launches hold 8 or 16 equal per-agent products each.  With the XCD-aware
# workgroup order (aac_gemm_batch_ordered, AAC_GRU_XCD=1) each XCD takes whole products, which read
# their operands from HBM about once (traffic 3.06x -> 1.19x the algorithmic bytes), but config 4 is
# ~1 % slower (0.371 -> 0.375 ms per step, profiles/r03_ab_gru_xcd_order.txt: a product's tiles then
# share one XCD's CUs).  Throughput is the metric, so the round-robin order is the default.
XCD_ORDER = os.environ.get("AAC_GRU_XCD", "0") == "1"


def _glaunch(probs, heads=()):
    return gemm_launches(probs, heads, xcd=XCD_ORDER and not heads)


# =============================================================================== update
class GruUpdate:
    """One update_myown (WGRU/maddpg:211-326) as a fixed launch list (graph-capturable)."""

    def __init__(self, model, replay, B):
        self.m, self.rep, self.B = model, replay, B
        # own rows are as wide as the replay stores them (D0 of the ATT env, or d_own for the
        # reference's two-portion states); the networks read their first d_own columns
        N, D0, d = model.n_agents, replay.D0, model.d_own
        if replay.N != N or replay.H != H or replay.R != 18 or D0 < d:
            raise ValueError(f"replay layout (N={replay.N}, D0={D0}, R={replay.R}, H={replay.H}) does not fit "
                             f"the GRU learner (N={N}, d_own={d}, R=18, H={H})")
        self.D0 = D0
        dev = model.device
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)   # noqa: E731
        self.bidx, self.batch, _ = replay.batch_buffers(B)
        self.Xsa, self.Xsa_t, self.Xsa2 = z(B, N, d + 2), z(B, N, d + 2), z(B, N, d + 2)
        self.cat_a, self.cat_c = z(B, N, 128), z(B, N, 128)
        self.gi_a, self.gh_a, self.gi_c, self.gh_c = z(B, N, 192), z(B, N, 192), z(B, N, 192), z(B, N, 192)
        # the target networks' projections get their own rows (they run beside the critic's and the
        # actor's in one launch, MULTI_PROJ)
        self.cat_at, self.cat_ct = z(B, N, 128), z(B, N, 128)
        self.gi_at, self.gh_at, self.gi_ct, self.gh_ct = z(B, N, 192), z(B, N, 192), z(B, N, 192), z(B, N, 192)
        self.y, self.q_c, self.q_a, self.dq = z(B, N), z(B, N), z(B, N), z(B, N)
        self.hc, self.ha = z(B, N, H), z(B, N, H)
        self.dgi_c, self.dgh_c, self.dgi_a, self.dgh_a = z(B, N, 192), z(B, N, 192), z(B, N, 192), z(B, N, 192)
        self.dcat_c, self.dcat_a, self.dsa = z(B, N, 128), z(B, N, 128), z(B, N, 64)
        self.da, self.dout = z(B, N, 2), z(B, N, 2)
        self._build()

    def _proj(self, P, stride, X1, w1, k1, radar, h, cat, gi, gh):
        """The encoders + input projections of one network evaluation over the batch: one
        weights-stationary launch (WsProj) or the two grouped-GEMM launches."""
        B, N = self.B, self.m.n_agents
        if WS_PROJ and k1 <= 8:
            return [WsProj(P, stride, X1, w1, k1, radar, h, cat, gi, gh, B, N)]
        return (_glaunch(enc2_probs(P, "Wo", "bo", "Wg", "bg", X1, w1, k1, radar, 18, 18, cat, B, N))
                + _glaunch(gate_probs(P, cat, h, gi, gh, B, N)))

    def _adam(self, opt, flat):
        m = self.m
        L = []
        if m.world > 1:     # SUM over the ranks; the Adam launch applies the 1 / world
            L.append(Collective(lambda: m._allreduce(flat)))
        L.append(lambda: fused.adam_at(opt, 1, 1.0 / m.world))
        return L

    def _build(self):
        m, B, N, D0, d = self.m, self.B, self.m.n_agents, self.D0, self.m.d_own
        rep, b = self.rep, self.batch
        A, At = stack_addrs(m.actors, ACTOR_PARAMS, m.fa), stack_addrs(m.actors_target, ACTOR_PARAMS, m.fa_t)
        C, Ct = stack_addrs(m.critics, CRITIC_PARAMS, m.fc), stack_addrs(m.critics_target, CRITIC_PARAMS, m.fc_t)
        gA, gC = stack_addrs(m.actors, ACTOR_PARAMS, m.fa, grad=True), stack_addrs(m.critics, CRITIC_PARAMS, m.fc,
                                                                                 grad=True)
        sa, sc = m.fa.numel // N, m.fc.numel // N          # floats per agent network
        own, radar, act = ptr(b["s_own"]), ptr(b["s_radar"]), ptr(b["act"])
        nown, nradar = ptr(b["n_own"]), ptr(b["n_radar"])
        hcur, hnext = ptr(b["h_cur"]), ptr(b["h_next"])
        P = ptr
        Dsa = d + 2
        L = [lambda: ops.replay_sample(rep.meta, B, rep.seed, rep.counter, self.bidx),
             lambda: ops.replay_gather(rep.ring, self.bidx, [b[k] for k in rep.fields], rep.widths)]
        # the projections that read only the batch and weights fixed until their step's Adam: the target
        # actor on s', the critic on (s, a) and the actor on s -- one launch (MULTI_PROJ) or three
        L.append(lambda: pack_rows(P(self.Xsa), Dsa, own, D0, d, act, 2, 2, B * N))
        early = [(At, sa, nown, D0, d, nradar, hnext, P(self.cat_at), P(self.gi_at), P(self.gh_at)),
                 (C, sc, P(self.Xsa), Dsa, Dsa, radar, hcur, P(self.cat_c), P(self.gi_c), P(self.gh_c)),
                 (A, sa, own, D0, d, radar, hcur, P(self.cat_a), P(self.gi_a), P(self.gh_a))]
        multi = MULTI_PROJ and WS_PROJ and max(e[4] for e in early) <= 8
        if multi:
            L.append(WsProjMulti([WsProj(*e, B, N) for e in early]))
        else:
            for e in early:
                L += self._proj(*e)
        # ---------------- TD target (WGRU/maddpg:265, :280-282), target networks
        fwd_t = gru_cell(At, "Wout", "bout", sa, 2, TANH, P(self.gi_at), P(self.gh_at), hnext, B, N, FWD,
                         pack_src=nown, ld_pack_src=D0, npack=d, pack_dst=P(self.Xsa_t), ld_pack_dst=Dsa)
        # the actor step's forward cell (actor weights fixed until its Adam) beside the target actor's
        fwd_a = gru_cell(A, "Wout", "bout", sa, 2, TANH, P(self.gi_a), P(self.gh_a), hcur, B, N, FWD,
                         hout=P(self.ha), ldho=H, pack_src=own, ld_pack_src=D0, npack=d, pack_dst=P(self.Xsa2),
                         ld_pack_dst=Dsa)
        pair = multi and CELL_PAIRS
        L.append(GruCell2(fwd_t, fwd_a, 0) if pair else fwd_t)
        L += self._proj(Ct, sc, P(self.Xsa_t), Dsa, Dsa, nradar, hnext, P(self.cat_ct), P(self.gi_ct), P(self.gh_ct))
        td = gru_cell(Ct, "Wout", "bout", sc, 1, 0, P(self.gi_ct), P(self.gh_ct), hnext, B, N, TD,
                      rew=ptr(b["rew"]), done=ptr(b["done"]), gamma=m.GAMMA, yout=P(self.y))
        # ---------------- critic step (WGRU/maddpg:272, :284-291); its mse head chained on the TD rows
        crit = gru_cell(C, "Wout", "bout", sc, 1, 0, P(self.gi_c), P(self.gh_c), hcur, B, N, CRITIC,
                        target=P(self.y), y=P(self.q_c), dq=P(self.dq), hout=P(self.hc), ldho=H, inv_m=1.0 / B,
                        dgi=P(self.dgi_c), dgh=P(self.dgh_c), ldd=192)
        L += [GruCell2(td, crit, 1)] if pair else [td, crit]
        L += _glaunch(
            wgrad_probs(P(self.dq), 0, 1, P(self.hc), 0, H, H, gC, "Wout", "bout", 1, B, N)
            + wgrad_probs(P(self.dgi_c), 0, 192, P(self.cat_c), 0, 128, 128, gC, "Wih", "bih", 192, B, N)
            + wgrad_probs(P(self.dgh_c), 0, 192, hcur, 0, H, H, gC, "Whh", "bhh", 192, B, N)
            + [prob(P(self.dgi_c) + 4 * i * 192, C[i]["Wih"], P(self.dcat_c) + 4 * i * 128, B, 128, 192, N * 192,
                    128, N * 128, mask=P(self.cat_c) + 4 * i * 128, ldmask=N * 128, mact=RELU) for i in range(N)])
        L += _glaunch(
            wgrad_probs(P(self.dcat_c), 0, 128, P(self.Xsa), 0, Dsa, Dsa, gC, "Wo", "bo", 64, B, N)
            + wgrad_probs(P(self.dcat_c), 64, 128, radar, 0, 18, 18, gC, "Wg", "bg", 64, B, N))
        L += self._adam(m.critic_optimizer, m.fc)
        # ---------------- actor step (WGRU/maddpg:293-310): 3 - mean Q(s, pi(s, h), h); its projection (and
        # with CELL_PAIRS its forward cell) ran above
        if not pair:
            L.append(fwd_a)
        L += self._proj(C, sc, P(self.Xsa2), Dsa, Dsa, radar, hcur, P(self.cat_c), P(self.gi_c), P(self.gh_c))
        L.append(gru_cell(C, "Wout", "bout", sc, 1, 0, P(self.gi_c), P(self.gh_c), hcur, B, N, ACTLOSS,
                          y=P(self.q_a), inv_m=1.0 / B, dgi=P(self.dgi_c), ldd=192))
        # d SA = (dgi W_ih[:, :64]) * (SA > 0); d a = d SA . W_sa[:, d:d+2]
        L += _glaunch([prob(P(self.dgi_c) + 4 * i * 192, C[i]["Wih"], P(self.dsa) + 4 * i * 64, B, 64, 192,
                                 N * 192, 128, N * 64, mask=P(self.cat_c) + 4 * i * 128, ldmask=N * 128, mact=RELU)
                            for i in range(N)])
        if CELL_DA:      # d a = d SA . W_sa[:, d:d+2] inside the backward cell (no product launch)
            L.append(gru_cell(A, "Wout", "bout", sa, 2, TANH, P(self.gi_a), P(self.gh_a), hcur, B, N, ACTBWD,
                              dsa=P(self.dsa), lddsa=64, wsa=C[0]["Wo"], wsa_stride=_agent_stride(C, sc), ldwsa=Dsa, wsa_col=d,
                              dq=P(self.dout), dgi=P(self.dgi_a), dgh=P(self.dgh_a), ldd=192))
        else:
            L += _glaunch([prob(P(self.dsa) + 4 * i * 64, C[i]["Wo"] + 4 * d, P(self.da) + 4 * i * 2, B, 2, 64,
                                N * 64, Dsa, N * 2) for i in range(N)])
            L.append(gru_cell(A, "Wout", "bout", sa, 2, TANH, P(self.gi_a), P(self.gh_a), hcur, B, N, ACTBWD,
                              da=P(self.da), ldda=2, dq=P(self.dout), dgi=P(self.dgi_a), dgh=P(self.dgh_a), ldd=192))
        L += _glaunch(
            wgrad_probs(P(self.dout), 0, 2, P(self.ha), 0, H, H, gA, "Wout", "bout", 2, B, N)
            + wgrad_probs(P(self.dgi_a), 0, 192, P(self.cat_a), 0, 128, 128, gA, "Wih", "bih", 192, B, N)
            + wgrad_probs(P(self.dgh_a), 0, 192, hcur, 0, H, H, gA, "Whh", "bhh", 192, B, N)
            + [prob(P(self.dgi_a) + 4 * i * 192, A[i]["Wih"], P(self.dcat_a) + 4 * i * 128, B, 128, 192, N * 192,
                    128, N * 128, mask=P(self.cat_a) + 4 * i * 128, ldmask=N * 128, mact=RELU) for i in range(N)])
        L += _glaunch(
            wgrad_probs(P(self.dcat_a), 0, 128, own, 0, D0, d, gA, "Wo", "bo", 64, B, N)
            + wgrad_probs(P(self.dcat_a), 64, 128, radar, 0, 18, 18, gA, "Wg", "bg", 64, B, N))
        L += self._adam(m.actor_optimizer, m.fa)
        # ---------------- soft update of every target (WGRU/maddpg:318-322)
        # (the Polyak launches also advance the optimisers' step counters)
        L += [lambda: ops.polyak_flat2(m.fc_t.data, m.fc.data, m.critic_optimizer.step_t, m.fa_t.data, m.fa.data,
                                       m.actor_optimizer.step_t, m.tau, 1)]
        self.L = L
        # i_episode % UPDATE_EVERY != 0 (WGRU/maddpg:320): the same launch with tau = 0 keeps the targets
        # bit-exactly (1 * t + 0 * s) and still advances the step counters
        self.hold = lambda: ops.polyak_flat2(m.fc_t.data, m.fc.data, m.critic_optimizer.step_t, m.fa_t.data,  # noqa
                                             m.fa.data, m.actor_optimizer.step_t, 0.0, 1)

    def ops(self):
        return self.L

    def run(self, idx=None, soft=True):
        """One eager update; ``soft=False`` skips the soft update (the step counters still advance)."""
        self.rep.check_sample(self.B)
        if idx is None:
            self.L[0]()
        else:
            self.bidx.copy_(idx.reshape(-1))
        for op in self.L[1:-1]:
            op()
        (self.L[-1] if soft else self.hold)()

    def segments(self):
        """The launch list cut at the collectives (kept inline when RCCL can be captured)."""
        if parallel.capturable(self.m.pg):
            return [list(self.L)], []
        segs, colls, cur = [], [], []
        for op in self.L:
            if isinstance(op, Collective):
                segs.append(cur)
                colls.append(op)
                cur = []
            else:
                cur.append(op)
        segs.append(cur)
        return segs, colls

    def stats(self):
        """[(loss_q, loss_a, q, target)] per agent, as the reference's c_loss / a_loss lists."""
        out = []
        for i in range(self.m.n_agents):
            q, y = self.q_c[:, i].unsqueeze(1), self.y[:, i]
            out.append((((q - y.unsqueeze(1)) ** 2).mean(), 3 - self.q_a[:, i].mean(), q, y))
        return out


def _p_or_none(t):
    return None if t is None else ptr(t)


class _ActPlan:
    """Batched choose_action for E envs: enc | gates | GRU fwd (actions, next hidden).  Built for
    fixed input / output buffers (no copies): own, radar, h as given, the next hidden into h_out (a
    plan-owned buffer when None)."""

    def __init__(self, m, own, radar, h, h_out=None):
        N, dev = m.n_agents, m.device
        E = own.shape[0]
        self.E = E
        for t in (own, radar, h):
            assert t.is_contiguous() and t.device == dev and t.dtype == torch.float32 and t.shape[0] == E
        self.inputs = (own, radar, h)            # kept alive with the plan
        D0 = own.shape[-1]
        self.a = torch.empty(E, N, 2, device=dev)
        self.hn = h_out if h_out is not None else torch.empty(E, N, H, device=dev)
        assert self.hn.is_contiguous() and self.hn.shape == (E, N, H)
        A = stack_addrs(m.actors, ACTOR_PARAMS, m.fa)
        self.ws = ACT_WS and m.d_own <= 8
        if self.ws:
            self.args = GruActorArgs(ptr(own), D0, m.d_own, ptr(radar), 18, ptr(h), H, *[A[0][k] for k in _WS_NAMES],
                                     _agent_stride(A, m.fa.numel // N), E, N, ptr(self.hn), H, ptr(self.a), 2)
            self.L = [lambda: _chk(glib().aac_gru_actor_fwd(ctypes.byref(self.args), fused._stream()),
                                   "aac_gru_actor_fwd")]
            return
        # the launch path's intermediate rows (the weights-stationary launch keeps them on chip)
        self.cat, self.gi, self.gh = (torch.empty(E, N, w, device=dev) for w in (128, 192, 192))
        self.L = gemm_launches(enc2_probs(A, "Wo", "bo", "Wg", "bg", ptr(own), D0, m.d_own, ptr(radar), 18, 18,
                                          ptr(self.cat), E, N))
        self.L += gemm_launches(gate_probs(A, ptr(self.cat), ptr(h), ptr(self.gi), ptr(self.gh), E, N))
        self.L.append(gru_cell(A, "Wout", "bout", m.fa.numel // N, 2, TANH, ptr(self.gi), ptr(self.gh), ptr(h),
                               E, N, FWD, hout=ptr(self.hn), ldho=H, y=ptr(self.a), ldy=2))

    def __call__(self, noise=None):
        """noise = (episode, eps_end, noise_start, noise_end, seed, counter, noise_out): the weights-
        stationary launch adds the exploration noise itself; returns whether it did."""
        if self.ws:
            a = self.args
            a.noisy = 0 if noise is None else 1
            if noise is not None:
                ep, eps_end, n0, n1, seed, ctr, nout = noise
                a.episode, a.eps_end, a.noise_start, a.noise_end = _p_or_none(ep), int(eps_end), float(n0), float(n1)
                a.seed, a.counter, a.noise_out = seed & 0xFFFFFFFFFFFFFFFF, ptr(ctr), _p_or_none(nout)
        for op in self.L:
            op()
        return self.a, self.hn, self.ws and noise is not None


# =============================================================================== MADDPG
class MADDPG:
    """GRU-actor MADDPG with the reference's surface (WGRU/maddpg:31-92, :211, :336, :94-131).

    Batched API: ``act(own, radar, h)`` -> (actions, next hidden) for E envs; ``attach_replay`` (rows
    carry h_cur / h_next); ``update(B)`` = one update_myown replayed from a captured HIP graph."""

    def __init__(self, actor_dim, critic_dim, dim_act, actor_hidden_state_size=H, gru_history_length=10, n_agents=8,
                 args=None, cr_lr=1e-3, ac_lr=1e-3, gamma=0.95, tau=0.01, device=None, seed=None, memory_length=None,
                 batch_size=None, process_group=None, own_width=None):
        """own_width: the env's own-observation row width the act / replay rows use: 6 for the WGRU
        env variant (``BatchedEnv(variant="wgru")``, WGRU/env:990), default 6 + 4 (N - 1) (the ATT
        env's rows, of which the networks read the first actor_dim[0])."""
        from .maddpg import _Adam
        self.args = args
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.n_agents = N = int(n_agents)
        self.n_actions = int(dim_act)
        assert self.n_actions == 2, "the tanh output layer of the row kernel is 2 actions wide (WGRU/nets:187)"
        self.d_own = int(actor_dim[0])                 # own-state columns the networks read (6 in WGRU/main:380)
        self.D0 = max(self.d_own, int(own_width) if own_width else 6 + 4 * (N - 1))   # env own-row width
        self.n_actor_dim, self.n_critic_dim = list(actor_dim), list(critic_dim)
        if seed is not None:
            torch.manual_seed(seed)
        mk_a = lambda: GRUCELL_actor_TwoPortion(actor_dim, dim_act, actor_hidden_state_size)  # noqa: E731
        mk_c = lambda: critic_single_obs_wGRU_TwoPortion(critic_dim, N, dim_act, gru_history_length,  # noqa: E731
                                                         actor_hidden_state_size)
        self.actors = AgentStack([mk_a() for _ in range(N)]).to(self.device)
        self.critics = AgentStack([mk_c() for _ in range(N)]).to(self.device)
        self.actors_target = deepcopy(self.actors)
        self.critics_target = deepcopy(self.critics)
        self.fa, self.fc = FlatParams(self.actors), FlatParams(self.critics)
        self.fa_t, self.fc_t = FlatParams(self.actors_target), FlatParams(self.critics_target)
        for p in list(self.actors_target.parameters()) + list(self.critics_target.parameters()):
            p.requires_grad_(False)
        self.GAMMA, self.tau = float(gamma), float(tau)
        # one Adam per agent network in the reference = one elementwise Adam over the flat buffer
        self.actor_optimizer = _Adam(self.fa, ac_lr)
        self.critic_optimizer = _Adam(self.fc, cr_lr)
        mem_len = memory_length or (getattr(args, "memory_length", None) or int(1e5))
        self.batch_size = batch_size or (getattr(args, "batch_size", None) or 512)
        self.memory = ReplayMemory(mem_len, device=self.device, hidden=H)
        self.replay = None
        self.var = [1.0 for _ in range(N)]
        self.noise_seed = int(seed or 0) * 7919 + 3
        self.noise_counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self._plans, self._acts = {}, {}
        self._graph = None
        self._graph_B = None
        self._last_src = None
        self.steps_done = 0

    # ------------------------------------------------------------------ batched API
    def attach_replay(self, capacity, seed=0):
        self.replay = DeviceReplay(capacity, self.n_agents, self.D0, 18, self.device, seed=seed, hidden=H)
        return self.replay

    @torch.no_grad()
    def act(self, own, radar, h, episode=None, noisy=True, eps_end=8000, noise_start=1.0, noise_end=0.03,
            noise_out=None, h_out=None):
        """Batched choose_action (WGRU/maddpg:336-428): (tanh actions + noise, clamped; next hidden).
        own (E, N, >= d_own), radar (E, N, 18), h (E, N, 64) contiguous on the device.  The next hidden
        goes to ``h_out`` when given (e.g. the other half of a ping-pong pair), else to a buffer of
        the plan; the actions are a plan buffer (valid until the next call on the same inputs).  One
        plan per input / output buffer set, so no copies."""
        own, radar, h = own.contiguous(), radar.contiguous(), h.contiguous()
        key = (own.data_ptr(), radar.data_ptr(), h.data_ptr(), None if h_out is None else h_out.data_ptr(),
               tuple(own.shape))
        plan = self._acts.get(key)
        if plan is None:
            if len(self._acts) >= 8:      # callers with fresh tensors every step: evict the oldest plan only
                self._acts.pop(next(iter(self._acts)))
            plan = self._acts[key] = _ActPlan(self, own, radar, h, h_out)
        else:
            self._acts[key] = self._acts.pop(key)      # most recently used last (dicts keep insertion order)
        noise = (episode, eps_end, noise_start, noise_end, self.noise_seed, self.noise_counter, noise_out)
        a, hn, fused_noise = plan(noise if noisy else None)
        if noisy and not fused_noise:
            ops.noise_clamp(a, episode, eps_end, noise_start, self.noise_seed, self.noise_counter, noise_out,
                            noise_end=noise_end)
        return a, hn

    def _allreduce(self, flat):
        """SUM over the ranks of one flat gradient (the plan's Adam launch applies the 1 / world)."""
        if self.world > 1:
            parallel.allreduce_sum_(flat.grad, self.pg)

    def _plan(self, B, rep=None):
        if rep is None:
            rep = self.replay if self.replay is not None else self.memory.dev
        key = (B, id(rep))
        if key not in self._plans:
            self._plans[key] = GruUpdate(self, rep, B)
        return self._plans[key]

    def _snapshot(self):
        rep = self.replay if self.replay is not None else self.memory.dev
        ts = [self.fa.data, self.fc.data, self.fa_t.data, self.fc_t.data, rep.counter]
        ts += self.actor_optimizer.state() + self.critic_optimizer.state()
        return ts, [t.clone() for t in ts]

    def capture(self, B, warmup=2):
        """Capture one update into HIP graphs (one graph, or one per segment between the gradient
        all-reduces when world > 1); the model state is restored afterwards."""
        ts, saved = self._snapshot()
        plan = self._plan(B)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                plan.run()
        torch.cuda.current_stream().wait_stream(s)
        segs, colls = plan.segments()
        graphs = []
        for seg in segs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for op in seg:
                    op()
            graphs.append(g)
        self._graph = (graphs, colls)
        for t, v in zip(ts, saved):
            t.copy_(v)
        self._graph_B = B
        return self._graph

    def invalidate_graphs(self):
        """Drop the captured update graph (a checkpoint load changed a seed the graph bakes in)."""
        self._graph = None

    def has_graph(self):
        return self._graph is not None

    def _replay(self):
        graphs, colls = self._graph
        for k, g in enumerate(graphs):
            with trace.range(f"update.seg{k}"):
                g.replay()
            if k < len(colls):
                with trace.range("allreduce"):
                    colls[k]()

    def update(self, B=None, use_graph=True, idx=None, want_stats=True, replay=None, soft_update=True):
        """One update_myown on the device replay (no host synchronisation); ``replay`` defaults to
        the attached batched replay, else the reference-API memory.  ``soft_update=False`` keeps the
        targets (UPDATE_EVERY > 1, WGRU/maddpg:320) and runs eagerly."""
        B = B or self.batch_size
        plan = self._plan(B, replay)
        if idx is None and use_graph and replay is None and soft_update:
            plan.rep.check_sample(B)
            if self._graph is None or self._graph_B != B:
                self.capture(B)
            self._replay()
        else:
            plan.run(idx, soft=soft_update)
        self._last_src = plan
        return plan.stats() if want_stats else None

    # ------------------------------------------------------------------ reference API
    def choose_action(self, state, cur_total_step, cur_episode, step, total_training_steps, noise_start_level,
                      actor_hiddens, noisy=True):
        """WGRU/maddpg:336 signature and returns (actions (N, 2), noise, cur hidden, next hidden)."""
        N = self.n_agents
        own = torch.as_tensor(np.stack([np.asarray(x, dtype=np.float32).reshape(-1) for x in state[0]]))
        grid = torch.as_tensor(np.stack([np.asarray(x, dtype=np.float32).reshape(-1) for x in state[1]]))
        hin = torch.as_tensor(np.asarray(actor_hiddens, dtype=np.float32)).reshape(N, H)
        own_p = torch.zeros(1, N, self.D0)
        own_p[0, :, :own.shape[1]] = own
        for i in range(N):
            self.var[i] = _scale(cur_episode, total_training_steps, noise_start_level)
        a, hn = self.act(own_p.to(self.device), grid.reshape(1, N, -1).to(self.device),
                         hin.reshape(1, N, H).to(self.device), noisy=False)
        act = a[0].clone()
        noise_value = np.zeros(2)
        if noisy:
            for i in range(N):
                noise_value = np.random.randn(2) * self.var[i]
                act[i] = torch.clamp(act[i] + torch.from_numpy(noise_value).float().to(self.device), -1.0, 1.0)
        self.steps_done += 1
        return act.cpu().numpy(), noise_value, hin.clone(), hn[0].cpu().clone()

    def update_myown(self, i_episode, total_step_count, UPDATE_EVERY, wandb=None):
        """WGRU/maddpg:211 signature and returns (c_loss list, a_loss list)."""
        if len(self.memory) <= self.batch_size:
            return None, None
        soft = i_episode % UPDATE_EVERY == 0      # WGRU/maddpg:320
        stats = self.update(self.batch_size, use_graph=False, replay=self.memory.dev, soft_update=soft)
        return [s[0] for s in stats], [s[1] for s in stats]

    def save_model(self, episode, file_path):
        """WGRU/maddpg:119-131: one actor state_dict per agent."""
        os.makedirs(file_path, exist_ok=True)
        for i in range(self.n_agents):
            sd = {k: v.detach().cpu().clone() for k, v in self.actors[i].state_dict().items()}
            torch.save(sd, os.path.join(file_path, f"episode_{episode}_agent_{i}actor_net.pth"))

    def load_model(self, filePath):
        """WGRU/maddpg:94-117 (weights_only load); targets re-copied as the reference's deepcopy."""
        for i, path in enumerate(filePath):
            self.actors[i].load_state_dict(torch.load(path, weights_only=True, map_location="cpu"))
        self.fa_t.data.copy_(self.fa.data)
        self.fc_t.data.copy_(self.fc.data)


def _scale(episode, eps_end, start_scale=1, end_scale=0.03):
    """get_custom_linear_scaling_factor (WGRU/maddpg:432-439)."""
    if episode <= eps_end:
        return start_scale + (end_scale - start_scale) / (eps_end - 1) * (episode - 1)
    return end_scale
