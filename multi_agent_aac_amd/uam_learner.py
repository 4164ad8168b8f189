"""The UAM variant's learner on the device, in float64.

UAM/ = MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM.  With the default flags of
UAM/main:60-100 (full_observable_critic_flag = use_GRU_flag = use_*_wRadar = False) the learner is
ONE shared ``ActorNetwork_TwoPortion`` and ONE shared ``critic_single_TwoPortion`` (UAM/maddpg:45-104),
both converted to float64 (UAM/maddpg:148-180), trained on per-aircraft transitions
(UAM/main:582-603): each ``update_myown`` (UAM/maddpg:304-595) is ONE gradient iteration
(var_iteration = 1) -- sample B transitions, TD target ``r + 0.95 Q'(s', pi'(s')) (1 - done)`` with the
aircraft's own done, MSE critic Adam step, ``-mean Q(s, pi(s))`` actor Adam step (lr 1e-4 both,
UAM/main:245-246) -- then the Polyak update (tau 0.01).

Canonical contract: the two networks read [own (7), radar (18)]
(UAM/maddpg:445-554), so their second encoder is 18 wide; the reference declares
``actor_dim[1] = (N-1)*5`` for it, which cannot run (R1).

Batched API: ``act`` (choose_action for E x N aircraft + noise), ``UamReplay.push_batch`` (E x N
transitions per env step into a device fp64 ring), ``update`` (one update_myown, replayed from a
captured HIP graph).  Reference API (drop-in for UAM/main, E = 1): ``choose_action``,
``update_myown``, ``memory.push/sample/len``, ``save_model``, ``load_model``.

Compute: ``act`` is one HIP launch (``aac_uam_actor``: the three wide layers on the fp64 matrix
cores, output layer, tanh, noise and clamp fused); the update is torch fp64 GEMMs on the matrix
cores and fused elementwise kernels, captured as one HIP graph; the sampler is the replay kernel
of aac_learn.hip (``aac_replay_sample``).  Nothing runs on the CPU.
"""
import copy
import ctypes
import os
from collections import namedtuple

import numpy as np
import torch
import torch.nn as nn

from . import ops, parallel, trace, uam

F64 = torch.float64
ROW = 7 + 18 + 2 + 1 + 1 + 7 + 18           # [own | radar | a | r | done | own' | radar']
SLICES = {"own": (0, 7), "radar": (7, 25), "act": (25, 27), "rew": (27, 28), "done": (28, 29),
          "n_own": (29, 36), "n_radar": (36, 54)}
Experience = namedtuple("Experience", ("states_obs", "states_nei", "states_grid", "actions", "next_states_obs",
                                       "next_states_nei", "next_states_grid", "rewards", "dones", "history_info",
                                       "cur_hidden", "next_hidden"))


class ActorNetwork_TwoPortion(nn.Module):
    """UAM/nets:167-190: relu(own_fc(own)) | relu(own_grid(radar)) -> relu(merge) -> tanh(act_out)."""

    def __init__(self, actor_dim, n_actions):
        super().__init__()
        self.own_fc = nn.Sequential(nn.Linear(actor_dim[0], 64), nn.ReLU())
        self.own_grid = nn.Sequential(nn.Linear(actor_dim[2], 64), nn.ReLU())   # radar width (R1)
        self.merge_feature = nn.Sequential(nn.Linear(64 + 64, 128), nn.ReLU())
        self.act_out = nn.Sequential(nn.Linear(128, n_actions), nn.Tanh())

    def forward(self, cur_state):
        x = torch.cat((self.own_fc(cur_state[0]), self.own_grid(cur_state[1])), dim=1)
        return self.act_out(self.merge_feature(x))


class critic_single_TwoPortion(nn.Module):
    """UAM/nets:692-720: relu(SA_fc([own, a])) | relu(SA_grid(radar)) -> relu(256) -> q."""

    def __init__(self, critic_obs, n_agents, n_actions, single_history=None, hidden_state_size=None):
        super().__init__()
        self.SA_fc = nn.Sequential(nn.Linear(critic_obs[0] + n_actions, 64), nn.ReLU())
        self.SA_grid = nn.Sequential(nn.Linear(critic_obs[2], 64), nn.ReLU())    # radar width (R1)
        self.merge_fc_grid = nn.Sequential(nn.Linear(64 + 64, 256), nn.ReLU())
        self.out_feature_q = nn.Sequential(nn.Linear(256, 1))

    def forward(self, single_state, single_action):
        x = torch.cat((self.SA_fc(torch.cat((single_state[0], single_action), dim=1)), self.SA_grid(single_state[1])),
                      dim=1)
        return self.out_feature_q(self.merge_fc_grid(x))


def noise_scale(episode, eps_end, start_scale=1, end_scale=0):
    """get_custom_linear_scaling_factor (UAM/maddpg:1399-1406), elementwise on a device tensor."""
    slope = (end_scale - start_scale) / (eps_end - 1)
    ep = episode.to(F64)
    return torch.where(ep <= eps_end, start_scale + slope * (ep - 1), torch.full_like(ep, float(end_scale)))


class UamReplay:
    """Device ring of fp64 transition rows [own | radar | a | r | done | own' | radar'] (54 doubles).
    The reference stores one Experience per aircraft (UAM/main:582-603) and the learner reads only
    these fields (the neighbour rows, history and hidden states are unused with the default
    flags).  ``meta`` = [next position, size] lives on the device for the sampler kernel."""

    def __init__(self, capacity, device="cuda", seed=0):
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.ring = torch.zeros(self.capacity, ROW, dtype=F64, device=self.device)
        self.meta = torch.zeros(2, dtype=torch.int64, device=self.device)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.seed = int(seed)
        self.pos = 0
        self.size = 0

    def __len__(self):
        return self.size

    def push_batch(self, own, radar, act, rew, done, n_own, n_radar, pos_io=None):
        """E x N transitions (leading dims flattened): one aac_uam_push launch for contiguous device
        float64 inputs (done uint8 or float64), else a row-assembly launch per ring segment.
        ``pos_io`` = (pos_in, pos_out) int64 device words (graph replays, aac_uam_push_io): the kernel
        reads the position from pos_in and advances it into pos_out and meta; the host mirror
        advances as usual."""
        M = own.numel() // 7
        if M > self.capacity:
            raise ValueError("one push larger than the replay capacity")
        if pos_io is not None and self.device.type != "cuda":
            raise ValueError("pos_io needs the device ring")
        ts = (own, radar, act, rew, n_own, n_radar)
        if (self.device.type == "cuda" and all(t.is_cuda and t.dtype == F64 and t.is_contiguous() for t in ts)
                and done.is_cuda and done.is_contiguous() and done.dtype in (torch.uint8, F64)
                and rew.numel() == M and done.numel() == M):
            from . import fused
            p = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
            if pos_io is not None:
                pin, pout = pos_io
                assert pin.dtype == torch.int64 and pout.dtype == torch.int64 and pin.data_ptr() != pout.data_ptr()
                _ok(_learn_lib().aac_uam_push_io(p(self.ring), self.capacity, M, p(own), p(radar), p(act), p(rew),
                                                 p(done), int(done.dtype == torch.uint8), p(n_own), p(n_radar),
                                                 p(self.meta), p(pin), p(pout), fused._stream()), "aac_uam_push_io")
                self._advance(M, meta=False)
                return
            _ok(_learn_lib().aac_uam_push(p(self.ring), self.capacity, self.pos, M, p(own), p(radar), p(act), p(rew),
                                          p(done), int(done.dtype == torch.uint8), p(n_own), p(n_radar),
                                          p(self.meta), self.size, fused._stream()), "aac_uam_push")
            self._advance(M, meta=False)       # the kernel wrote meta
            return
        if pos_io is not None:
            raise ValueError("pos_io needs contiguous device float64 sources (the aac_uam_push_io launch)")
        cols = [own.reshape(-1, 7), radar.reshape(-1, 18), act.reshape(-1, 2), rew.reshape(-1, 1),
                done.reshape(-1, 1), n_own.reshape(-1, 7), n_radar.reshape(-1, 18)]
        cols = [c if c.dtype == F64 else c.to(F64) for c in cols]
        p = self.pos
        first = min(M, self.capacity - p)
        torch.cat([c[:first] for c in cols], dim=1, out=self.ring[p:p + first])
        if first < M:
            torch.cat([c[first:] for c in cols], dim=1, out=self.ring[:M - first])
        self._advance(M)

    def _advance(self, M, meta=True):
        self.pos = (self.pos + M) % self.capacity
        self.size = min(self.size + M, self.capacity)
        if meta:
            self.meta[0] = self.pos          # device-side copies of the host counters (no sync)
            self.meta[1] = self.size

    def fields(self, rows):
        return {k: rows[:, a:b] for k, (a, b) in SLICES.items()}


class UamReplayMemory:
    """ReplayMemory surface of UAM/memory:8-23: ``push(*12 fields)`` per aircraft, ``sample``, ``len``."""

    def __init__(self, capacity, device="cuda", seed=0):
        self.dev = UamReplay(capacity, device, seed)
        self.memory = self
        self.position = 0

    def push(self, states_obs, states_nei, states_grid, actions, next_states_obs, next_states_nei, next_states_grid,
             rewards, dones, history_info=None, cur_hidden=None, next_hidden=None):
        d = self.dev.device
        t = lambda x, n: torch.as_tensor(np.asarray(x.cpu() if torch.is_tensor(x) else x, dtype=np.float64)  # noqa: E731
                                         ).reshape(1, n).to(d)
        self.dev.push_batch(t(states_obs, 7), t(states_grid, 18), t(actions, 2), t(rewards, 1), t(dones, 1),
                            t(next_states_obs, 7), t(next_states_grid, 18))
        self.position = self.dev.pos

    def sample(self, batch_size):
        idx = torch.empty(batch_size, dtype=torch.int32, device=self.dev.device)
        ops.replay_sample(self.dev.meta, batch_size, self.dev.seed, self.dev.counter, idx)
        f = self.dev.fields(self.dev.ring.index_select(0, idx.long()))
        return [Experience(f["own"][i], None, f["radar"][i], f["act"][i], f["n_own"][i], None, f["n_radar"][i],
                           f["rew"][i, 0], f["done"][i, 0], None, None, None) for i in range(batch_size)]

    def __len__(self):
        return len(self.dev)


def _init_adam_state(opt):
    """Device-side Adam state before the first step, so a graph can be captured from step 1.  The
    fused kernel keeps a float32 step counter (integers are exact in it) and computes the bias
    corrections 1 - beta^t in float64 for float64 parameters (the non-fused capturable path would
    round them to float32: 7 digits)."""
    for group in opt.param_groups:
        for p in group["params"]:
            opt.state[p] = {"step": torch.zeros((), dtype=torch.float32, device=p.device),
                            "exp_avg": torch.zeros_like(p, memory_format=torch.preserve_format),
                            "exp_avg_sq": torch.zeros_like(p, memory_format=torch.preserve_format)}


_LL = None


def _learn_lib():
    """The fused-learner entry points of libaac_env.so (include/aac_uam_learn.h)."""
    global _LL
    if _LL is None:
        from . import fused
        L = uam.lib()
        vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        L.aac_uam_learn_last_error.restype = ctypes.c_char_p
        L.aac_gemm64_batch.argtypes = [ctypes.POINTER(Gemm64Prob), i32, vp]
        L.aac_uam_gather.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
        L.aac_uam_head.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp, i32, dbl, vp, vp, vp, vp]
        L.aac_uam_td_mse_head.argtypes = [vp, vp, vp, vp, vp, i32, dbl, vp, vp, vp, vp, i32, vp, vp, vp, vp]
        L.aac_adam64_sum.argtypes = [vp, vp, i32, vp, vp, i64, dbl, dbl, dbl, dbl, vp, i32, vp]
        L.aac_adam64_sum_scaled.argtypes = [vp, vp, i32, vp, vp, i64, dbl, dbl, dbl, dbl, vp, i32, dbl, vp]
        L.aac_uam_polyak.argtypes = [vp, vp, i64, dbl, vp, vp, vp, i32, vp, vp]
        L.aac_uam_push.argtypes = [vp, i64, i64, i64, vp, vp, vp, vp, vp, i32, vp, vp, vp, i64, vp]
        L.aac_uam_push_io.argtypes = [vp, i64, i64, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp]
        L.aac_sum64_partials.argtypes = [vp, vp, i32, i64, vp]
        _LL = L
    return _LL


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {_learn_lib().aac_uam_learn_last_error().decode()}")


def p64(t, off=0):
    """Device address of float64 element ``off`` of tensor ``t``."""
    return None if t is None else t.data_ptr() + 8 * off


class Gemm64Prob(ctypes.Structure):
    """aac_gemm64_prob (include/aac_uam_learn.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("A", "B", "C", "bias", "addend", "mask", "cextra")] + \
        [("split_stride", ctypes.c_int64)] + \
        [(n, ctypes.c_int32) for n in ("M", "N", "K", "lda", "ldb", "ldc", "ldadd", "ldmask", "ta", "tb", "act", "mact",
                                       "ones", "ksplit")] + \
        [("dvec", ctypes.c_void_p), ("C2", ctypes.c_void_p), ("dscale", ctypes.c_double)]


def prob64(A, B, C, M, N, K, lda, ldb, ldc, ta=0, tb=0, bias=None, act=0, mask=None, ldmask=0, mact=0, ones=0,
           cextra=None, ksplit=1, split_stride=0, dvec=None, C2=None, dscale=0.0):
    """One float64 product C[M][N] = mact(act(op(A) op(B) + bias)) (aac_gemm64_prob; addresses as ints);
    with C2 also C2 = (C > 0) dscale dvec[n] (the actor-loss head's dh)."""
    return Gemm64Prob(A, B, C, bias, None, mask, cextra, split_stride, M, N + ones, K, lda, ldb, ldc, 0, ldmask,
                      ta, tb, act, mact, ones, ksplit, dvec, C2, dscale)


def _rebind(params, flat):
    """Copy the parameters into ``flat`` (in order) and make each ``param.data`` a view of it."""
    o = 0
    for p in params:
        n = p.numel()
        flat[o:o + n].copy_(p.data.reshape(-1))
        p.data = flat[o:o + n].view_as(p.data)
        o += n
    return o


class FusedUamUpdate:
    """update_myown of UAM/maddpg:304-595 on the device as ~20 launches (include/aac_uam_learn.h):
    grouped float64 products on the fp64 matrix cores with fused bias / ReLU / tanh epilogues and
    relu' / tanh' backward masks, weight gradients as KS partial copies over the B sampled rows
    (bias gradients from a virtual ones column), the critic head with the TD target / mse / -mean Q
    gradients, fused Adam on the partial sums, and one soft-update kernel for both targets.

    Parameters of the four networks live in two flat float64 buffers ([critic | actor] and the
    targets), which the torch modules view, so ``save_model`` / ``load_model`` / the torch path see
    the same weights.  The Adam moments are flat buffers too (``m1`` / ``m2``, one int32 step
    counter), owned by the MADDPG object (``MADDPG._flat_state``) so every plan -- any B, any
    replay -- and the torch-autograd path continue from the same optimiser state."""
    # split-K partial copies of the weight gradients: 4 beat 8 by 0.5 % at config 5 with the reset
    # overlapped (profiles/r05_uam_ks_ab.txt; 2 and 16 no better); AAC_UAM_KS overrides
    KS = int(os.environ.get("AAC_UAM_KS", "4"))

    def __init__(self, m, B, rep):
        self.m, self.B, self.rep = m, int(B), rep
        dev = m.device
        z = lambda *s: torch.zeros(*s, dtype=F64, device=dev)   # noqa: E731
        fs = m._flat_state()
        self.nC, self.nA = nC, nA = fs["nC"], fs["nA"]
        self.flat, self.tflat, self.m1, self.m2, self.step = fs["flat"], fs["tflat"], fs["m1"], fs["m2"], fs["step"]
        self.lr_c = m.critic_optimizer.param_groups[0]["lr"]
        self.lr_a = m.actor_optimizer.param_groups[0]["lr"]
        self.betas = m.critic_optimizer.param_groups[0]["betas"]
        self.eps = m.critic_optimizer.param_groups[0]["eps"]
        self.gc, self.ga = z(self.KS, nC), z(self.KS, nA)
        # world > 1: the summed gradient [critic | actor] that the ranks average before each Adam step
        self.gflat = z(nC + nA) if m.world > 1 else None
        B = self.B
        self.idx = torch.zeros(B, dtype=torch.int32, device=dev)
        self.rows, self.xc, self.xt, self.xp = z(B, ROW), z(B, 9), z(B, 9), z(B, 9)
        self.ha1t, self.ha2t, self.hc1t, self.hc2t = z(B, 128), z(B, 128), z(B, 128), z(B, 256)
        self.hc1, self.hc2, self.dh1, self.dh2 = z(B, 128), z(B, 256), z(B, 128), z(B, 256)
        self.ha1, self.ha2, self.hp1, self.hp2 = z(B, 128), z(B, 128), z(B, 128), z(B, 256)
        self.dp1, self.dp2, self.dout, self.dha1, self.dha2 = z(B, 64), z(B, 256), z(B, 2), z(B, 128), z(B, 128)
        self.y, self.dq, self.lq, self.la, self.loss = z(B), z(B), z(B), z(B), z(2)
        self._launches = self._build()

    def _offsets(self, module, base):
        out, o = {}, base
        for name, p in module.named_parameters():
            out[name] = o
            o += p.numel()
        return out

    def _build(self):
        m, B, KS, L = self.m, self.B, self.KS, _learn_lib()
        from . import fused
        nC, nA = self.nC, self.nA
        oc = self._offsets(m.critics, 0)
        oa = self._offsets(m.actors, nC)
        F, T = self.flat, self.tflat
        c = {k: p64(F, v) for k, v in oc.items()}
        a = {k: p64(F, v) for k, v in oa.items()}
        ct = {k: p64(T, v) for k, v in oc.items()}
        at = {k: p64(T, v) for k, v in oa.items()}
        gc = {k: p64(self.gc, v) for k, v in oc.items()}
        ga = {k: p64(self.ga, v - nC) for k, v in oa.items()}
        R, P = self.rows, p64
        own, g, g2 = P(R), P(R, 7), P(R, 36)
        xc, xt, xp = P(self.xc), P(self.xt), P(self.xp)
        RELU, TANH = 1, 2
        Wc = lambda d, k: d[k + ".0.weight"]      # noqa: E731
        Bc = lambda d, k: d[k + ".0.bias"]        # noqa: E731

        def lin(A, lda, W, bias, C, ldc, K, N, act, M=B):
            return prob64(A, W, C, M, N, K, lda, K, ldc, tb=1, bias=bias, act=act)

        def wgrad(dY, lddy, X, ldx, M, N, Cw, Cb, stride):
            # dW[M][N] = dY^T X over the B rows (K split into KS copies), bias gradient from the ones column
            return prob64(dY, X, Cw, M, N, B, lddy, ldx, N, ta=1, ones=1, cextra=Cb, ksplit=KS, split_stride=stride)

        def gemm(probs):
            arr = (Gemm64Prob * len(probs))(*probs)
            n = len(probs)
            return lambda: _ok(L.aac_gemm64_batch(arr, n, fused._stream()), "aac_gemm64_batch")

        st = self
        launches = [
            # replay sample + gather (UAM/maddpg:330-345)
            lambda: ops.replay_sample(st.rep.meta, B, st.rep.seed, st.rep.counter, st.idx),
            lambda: _ok(L.aac_uam_gather(P(st.rep.ring), st.idx.data_ptr(), B, P(R), xc, xt, xp, fused._stream()),
                        "aac_uam_gather"),
            # first layers of the target actor, the critic (both inputs), the target critic's radar
            # encoder and the actor (actor weights are unchanged until the actor step)
            gemm([lin(xt, 9, Wc(at, "own_fc"), Bc(at, "own_fc"), P(st.ha1t), 128, 7, 64, RELU),
                  lin(g2, ROW, Wc(at, "own_grid"), Bc(at, "own_grid"), P(st.ha1t, 64), 128, 18, 64, RELU),
                  lin(g2, ROW, Wc(ct, "SA_grid"), Bc(ct, "SA_grid"), P(st.hc1t, 64), 128, 18, 64, RELU),
                  lin(xc, 9, Wc(c, "SA_fc"), Bc(c, "SA_fc"), P(st.hc1), 128, 9, 64, RELU),
                  lin(g, ROW, Wc(c, "SA_grid"), Bc(c, "SA_grid"), P(st.hc1, 64), 128, 18, 64, RELU),
                  lin(own, ROW, Wc(a, "own_fc"), Bc(a, "own_fc"), P(st.ha1), 128, 7, 64, RELU),
                  lin(g, ROW, Wc(a, "own_grid"), Bc(a, "own_grid"), P(st.ha1, 64), 128, 18, 64, RELU)]),
            gemm([lin(P(st.ha1t), 128, Wc(at, "merge_feature"), Bc(at, "merge_feature"), P(st.ha2t), 128, 128, 128,
                      RELU),
                  lin(P(st.hc1), 128, Wc(c, "merge_fc_grid"), Bc(c, "merge_fc_grid"), P(st.hc2), 256, 128, 256, RELU),
                  lin(P(st.ha1), 128, Wc(a, "merge_feature"), Bc(a, "merge_feature"), P(st.ha2), 128, 128, 128,
                      RELU)]),
            # tanh action layers: target actions into xt[:, 7:9], policy actions into xp[:, 7:9]
            gemm([lin(P(st.ha2t), 128, Wc(at, "act_out"), Bc(at, "act_out"), P(st.xt, 7), 9, 128, 2, TANH),
                  lin(P(st.ha2), 128, Wc(a, "act_out"), Bc(a, "act_out"), P(st.xp, 7), 9, 128, 2, TANH)]),
            gemm([lin(xt, 9, Wc(ct, "SA_fc"), Bc(ct, "SA_fc"), P(st.hc1t), 128, 9, 64, RELU)]),
            gemm([lin(P(st.hc1t), 128, Wc(ct, "merge_fc_grid"), Bc(ct, "merge_fc_grid"), P(st.hc2t), 256, 128, 256,
                      RELU)]),
            # TD target r + gamma Q'(s', a')(1 - done) and the mse gradient (UAM/maddpg:346-380), one
            # launch: the critic's head chained on each row's just-computed target
            lambda: _ok(L.aac_uam_td_mse_head(P(st.hc2t), Wc(ct, "out_feature_q"), Bc(ct, "out_feature_q"), P(R, 27),
                                              P(R, 28), ROW, float(m.GAMMA), P(st.y), P(st.hc2),
                                              Wc(c, "out_feature_q"), Bc(c, "out_feature_q"), B, P(st.dq), P(st.dh2),
                                              P(st.lq), fused._stream()), "aac_uam_td_mse_head"),
            # critic weight gradients and the backward into the merge layer's input
            gemm([wgrad(P(st.dq), 1, P(st.hc2), 256, 1, 256, gc["out_feature_q.0.weight"], gc["out_feature_q.0.bias"],
                        nC),
                  wgrad(P(st.dh2), 256, P(st.hc1), 128, 256, 128, gc["merge_fc_grid.0.weight"],
                        gc["merge_fc_grid.0.bias"], nC),
                  prob64(P(st.dh2), Wc(c, "merge_fc_grid"), P(st.dh1), B, 128, 256, 256, 128, 128,
                         mask=P(st.hc1), ldmask=128, mact=RELU)]),
            gemm([wgrad(P(st.dh1), 128, xc, 9, 64, 9, gc["SA_fc.0.weight"], gc["SA_fc.0.bias"], nC),
                  wgrad(P(st.dh1, 64), 128, g, ROW, 64, 18, gc["SA_grid.0.weight"], gc["SA_grid.0.bias"], nC)]),
            *self._adam_launches(0, nC, st.gc, st.lr_c),
            # actor step: -mean Q(s, pi(s)) through the updated critic (UAM/maddpg:389-512)
            gemm([lin(xp, 9, Wc(c, "SA_fc"), Bc(c, "SA_fc"), P(st.hp1), 128, 9, 64, RELU),
                  lin(g, ROW, Wc(c, "SA_grid"), Bc(c, "SA_grid"), P(st.hp1, 64), 128, 18, 64, RELU)]),
            # -mean Q has the constant gradient dq = -1/B (UAM/maddpg:512): the head's dh is a second
            # output of the merge layer's epilogue, and Q itself (the actor loss) an N = 1 product
            # beside the backward into the merge layer's input -- no head launch on this chain
            gemm([prob64(P(st.hp1), Wc(c, "merge_fc_grid"), P(st.hp2), B, 256, 128, 128, 128, 256, tb=1,
                         bias=Bc(c, "merge_fc_grid"), act=RELU, dvec=Wc(c, "out_feature_q"), C2=P(st.dp2),
                         dscale=-1.0 / B)]),
            # d/d(own-encoder input) of the critic, first 64 features only (the action columns)
            gemm([prob64(P(st.dp2), Wc(c, "merge_fc_grid"), P(st.dp1), B, 64, 256, 256, 128, 64,
                         mask=P(st.hp1), ldmask=128, mact=RELU),
                  lin(P(st.hp2), 256, Wc(c, "out_feature_q"), Bc(c, "out_feature_q"), P(st.la), 1, 256, 1, 0)]),
            # da = dx V1[:, 7:9], times tanh' of the policy action
            gemm([prob64(P(st.dp1), Wc(c, "SA_fc") + 8 * 7, P(st.dout), B, 2, 64, 64, 9, 2,
                         mask=P(st.xp, 7), ldmask=9, mact=TANH)]),
            gemm([prob64(P(st.dout), Wc(a, "act_out"), P(st.dha2), B, 128, 2, 2, 128, 128,
                         mask=P(st.ha2), ldmask=128, mact=RELU),
                  wgrad(P(st.dout), 2, P(st.ha2), 128, 2, 128, ga["act_out.0.weight"], ga["act_out.0.bias"], nA)]),
            gemm([prob64(P(st.dha2), Wc(a, "merge_feature"), P(st.dha1), B, 128, 128, 128, 128, 128,
                         mask=P(st.ha1), ldmask=128, mact=RELU),
                  wgrad(P(st.dha2), 128, P(st.ha1), 128, 128, 128, ga["merge_feature.0.weight"],
                        ga["merge_feature.0.bias"], nA)]),
            gemm([wgrad(P(st.dha1), 128, own, ROW, 64, 7, ga["own_fc.0.weight"], ga["own_fc.0.bias"], nA),
                  wgrad(P(st.dha1, 64), 128, g, ROW, 64, 18, ga["own_grid.0.weight"], ga["own_grid.0.bias"], nA)]),
            *self._adam_launches(nC, nA, st.ga, st.lr_a),
            # soft update of both targets (UAM/maddpg:21-25), the shared step counter and the losses
            lambda: _ok(L.aac_uam_polyak(P(T), P(F), nC + nA, float(m.tau), st.step.data_ptr(), P(st.lq), P(st.la),
                                         B, P(st.loss), fused._stream()), "aac_uam_polyak"),
        ]
        return launches

    def _adam_launches(self, off, n, gpart, lr):
        """The Adam step of the network at [off, off + n) of the flat buffers.  world == 1: Adam sums
        the KS partial copies itself.  world > 1: sum them, average over the ranks (one collective,
        between graph segments), Adam on the average.  The collective SUMs and Adam multiplies by
        1 / world, which equals the mean exactly only for power-of-two worlds: there the update is
        bit-identical to one rank when every rank holds the same data; for other world sizes it is
        within one rounding of the mean per gradient element."""
        from . import fused
        L, st, KS, P = _learn_lib(), self, self.KS, p64

        gs = 1.0 / self.m.world     # world > 1: the collective SUMs, the Adam launch applies 1 / world

        def adam(src, ns):
            return lambda: _ok(L.aac_adam64_sum_scaled(P(st.flat, off), src, ns, P(st.m1, off), P(st.m2, off), n, lr,
                                                       st.betas[0], st.betas[1], st.eps, st.step.data_ptr(), 1, gs,
                                                       fused._stream()), "aac_adam64_sum")
        if self.m.world == 1:
            return [adam(P(gpart), KS)]
        g = self.gflat[off:off + n]
        m = self.m
        return [lambda: _ok(L.aac_sum64_partials(P(g), P(gpart), KS, n, fused._stream()), "aac_sum64_partials"),
                fused.Collective(lambda: m._allreduce_flat(g)),
                adam(P(g), 1)]

    def segments(self):
        """The launch list cut at the collectives: ([segment launches], [collective]); kept inline
        (one segment) when RCCL can capture them (parallel.capturable)."""
        from . import fused
        if parallel.capturable(self.m.pg):
            return [list(self._launches)], []
        segs, colls, cur = [], [], []
        for f in self._launches:
            if isinstance(f, fused.Collective):
                segs.append(cur)
                colls.append(f)
                cur = []
            else:
                cur.append(f)
        segs.append(cur)
        return segs, colls

    def run(self, idx=None):
        """One update from the replay (or the given sampled indices); returns (loss_q, loss_a)."""
        if idx is None:
            for f in self._launches:
                f()
        else:
            self.idx.copy_(idx.reshape(-1).to(torch.int32))
            for f in self._launches[1:]:
                f()
        return self.loss[0], self.loss[1]

    def capture(self):
        """One update as HIP graphs (raw launches only: nothing to warm up, no state to restore): one
        graph, or one per segment between the gradient all-reduces when world > 1."""
        segs, colls = self.segments()
        graphs = []
        for seg in segs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for f in seg:
                    f()
            graphs.append(g)
        self.graphs, self.colls = graphs, colls
        self.graph = graphs[0] if len(graphs) == 1 else None
        return graphs

    def replay(self):
        for k, g in enumerate(self.graphs):
            with trace.range(f"update.seg{k}"):
                g.replay()
            if k < len(self.colls):
                with trace.range("allreduce"):
                    self.colls[k]()


class MADDPG:
    """UAM/maddpg:35-181 with the default flags (shared actor + shared single critic, float64)."""

    def __init__(self, actor_dim, critic_dim, dim_act, actor_hidden_state_size=64, gru_history_length=10,
                 n_agents=5, args=None, cr_lr=1e-4, ac_lr=1e-4, gamma=0.95, tau=0.01,
                 full_observable_critic_flag=False, use_GRU_flag=False, use_single_portion_selfATT=False,
                 use_selfATT_with_radar=False, use_allNeigh_wRadar=False, own_obs_only=False, normalizer=None,
                 use_nearestN_neigh_wRadar=False, device=None, seed=None, memory_length=None, batch_size=None,
                 process_group=None):
        if full_observable_critic_flag or use_GRU_flag or use_single_portion_selfATT or use_selfATT_with_radar \
                or use_allNeigh_wRadar or use_nearestN_neigh_wRadar:
            raise NotImplementedError("UAM learner: the default flags of UAM/main:60-100 only")
        self.args = args
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if seed is not None:
            torch.manual_seed(seed)
        self.n_agents, self.n_actions = int(n_agents), int(dim_act)
        self.n_actor_dim, self.n_critic_dim = list(actor_dim), list(critic_dim)
        self.actors = ActorNetwork_TwoPortion(actor_dim, dim_act).to(self.device, F64)
        self.critics = critic_single_TwoPortion(critic_dim, n_agents, dim_act).to(self.device, F64)
        self.actors_target = copy.deepcopy(self.actors)
        self.critics_target = copy.deepcopy(self.critics)
        for p in list(self.actors_target.parameters()) + list(self.critics_target.parameters()):
            p.requires_grad_(False)
        self.GAMMA, self.tau = float(gamma), float(tau)
        cap = self.device.type == "cuda"
        # fused Adam: one kernel per optimizer step (capturable on the device)
        kw = dict(capturable=True, fused=True) if cap else dict(foreach=False)
        self.critic_optimizer = torch.optim.Adam(self.critics.parameters(), lr=cr_lr, **kw)
        self.actor_optimizer = torch.optim.Adam(self.actors.parameters(), lr=ac_lr, **kw)
        if cap:
            for opt in (self.critic_optimizer, self.actor_optimizer):
                _init_adam_state(opt)
        mem_len = memory_length or (getattr(args, "memory_length", None) or int(1e5))
        self.batch_size = batch_size or (getattr(args, "batch_size", None) or 512)
        self.memory = UamReplayMemory(mem_len, self.device, seed=int(seed or 0))
        self.replay = None
        self.var = [1.0 for _ in range(self.n_agents)]
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.steps_done = 0
        self._graph = None
        self._graph_B = None
        self._static = {}
        self.noise_seed = int(seed or 0) * 7919 + 1
        self.noise_counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        # update() path on one GPU: the fused float64 learner (FusedUamUpdate), else torch autograd
        self.fused_learner = self.device.type == "cuda" and os.environ.get("AAC_UAM_FUSED", "1") != "0"
        self._fu = None
        self._fstate = None         # shared flat parameter / Adam state (``_flat_state``)
        self._opt_steps = []

    # ------------------------------------------------------------------ batched API
    def attach_replay(self, capacity, seed=0):
        self.replay = UamReplay(capacity, self.device, seed)
        return self.replay

    @torch.no_grad()
    def act(self, own, radar, episode, noisy=True, eps_end=10000, noise_start=1.0):
        """choose_action (UAM/maddpg:597-676) for every aircraft: tanh actor + N(0, var^2) noise with
        var from each env's own episode counter, clamped to [-1, 1].  own (E, N, 7), radar (E, N, 18)
        float64; one ``aac_uam_actor`` launch (fp64 matrix cores, noise fused)."""
        E, N = own.shape[0], own.shape[1]
        for t, w in ((own, 7), (radar, 18)):
            assert t.is_contiguous() and t.dtype == F64 and t.device == self.device and t.shape[-1] == w
        if episode is not None:
            assert episode.dtype == torch.int32 and episode.numel() == E
        out = torch.empty(E, N, 2, dtype=F64, device=self.device)
        a = self.actors
        ws = [a.own_fc[0].weight, a.own_fc[0].bias, a.own_grid[0].weight, a.own_grid[0].bias,
              a.merge_feature[0].weight, a.merge_feature[0].bias, a.act_out[0].weight, a.act_out[0].bias]
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
        rc = uam.lib().aac_uam_actor(p(own), p(radar), E * N, *[p(w) for w in ws], p(out), N, p(episode),
                                     int(eps_end), float(noise_start), 0.0, ctypes.c_uint64(self.noise_seed),
                                     p(self.noise_counter), int(bool(noisy)),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(f"aac_uam_actor failed: {uam.lib().aac_uam_actor_last_error().decode()}")
        return out

    def _soft_update(self):
        """soft_update (UAM/maddpg:21-25): target <- target (1 - tau) + source tau, one foreach
        kernel per network (lerp: target + tau (source - target), the same value to rounding)."""
        for tgt, src in ((self.critics_target, self.critics), (self.actors_target, self.actors)):
            torch._foreach_lerp_(list(tgt.parameters()), [p.detach() for p in src.parameters()], self.tau)

    def _allreduce_flat(self, t):
        """SUM over the ranks of one flat float64 gradient (the fused learner's collective; its Adam
        launch applies the 1 / world)."""
        from . import parallel
        parallel.allreduce_sum_(t, self.pg)

    def _allreduce_grads(self, module):
        if self.world > 1:
            from . import parallel
            grads = [p.grad for p in module.parameters()]
            flat = torch.cat([g.reshape(-1) for g in grads])
            parallel.allreduce_mean_(flat, self.pg)
            torch._foreach_copy_(grads, [t.view_as(g) for t, g in zip(flat.split([g.numel() for g in grads]), grads)])

    def _core(self, rows):
        """One update_myown gradient iteration on sampled rows (UAM/maddpg:330-512) + soft update."""
        f = {k: rows[:, a:b] for k, (a, b) in SLICES.items()}
        s, s2 = [f["own"], f["radar"]], [f["n_own"], f["n_radar"]]
        with torch.no_grad():
            na = self.actors_target(s2)
            q_next = self.critics_target(s2, na).squeeze()
            target = (f["rew"][:, 0] + self.GAMMA * q_next * (1 - f["done"][:, 0])).unsqueeze(1)
        if self._fstate is not None:
            # the fused plans count Adam steps in one int32 counter: mirror it into the torch
            # optimisers' per-parameter step tensors, and advance it after the two steps below
            torch._foreach_copy_(self._opt_steps, [self._fstate["step"].to(torch.float32).reshape(())]
                                 * len(self._opt_steps))
        q = self.critics(s, f["act"])
        loss_q = nn.MSELoss()(q, target.detach())
        torch._foreach_zero_(self._cgrads)
        loss_q.backward()
        self._allreduce_grads(self.critics)
        self.critic_optimizer.step()
        # the actor loss back-propagates through the critic only for d/da: the reference also
        # accumulates critic weight gradients there, which the next critic zero_grad discards
        for p in self.critics.parameters():
            p.requires_grad_(False)
        try:
            loss_a = -self.critics(s, self.actors(s)).mean()
            torch._foreach_zero_(self._agrads)
            loss_a.backward()
        finally:
            for p in self.critics.parameters():
                p.requires_grad_(True)
        self._allreduce_grads(self.actors)
        self.actor_optimizer.step()
        if self._fstate is not None:
            self._fstate["step"].add_(1)
        self._soft_update()
        return loss_q.detach(), loss_a.detach()

    def _buffers(self, rep, B):
        key = (id(rep), B)
        if key not in self._static:
            self._static[key] = (torch.empty(B, dtype=torch.int32, device=self.device),
                                 torch.empty(B, ROW, dtype=F64, device=self.device))
        return self._static[key]

    def _sampled_core(self, rep, B, idx=None):
        self._init_grads()
        bidx, rows = self._buffers(rep, B)
        if idx is None:
            ops.replay_sample(rep.meta, B, rep.seed, rep.counter, bidx)
        else:
            bidx.copy_(idx.reshape(-1))
        torch.index_select(rep.ring, 0, bidx.long(), out=rows)
        return self._core(rows)

    def _init_grads(self):
        for m in (self.actors, self.critics):
            for p in m.parameters():
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
        self._agrads = [p.grad for p in self.actors.parameters()]
        self._cgrads = [p.grad for p in self.critics.parameters()]

    def capture(self, B, rep):
        """Capture one update (sample -> gather -> critic step -> actor step -> soft update) into a HIP
        graph; the state is restored afterwards so capture has no side effect."""
        self._init_grads()
        snap = [t.clone() for t in self._state_tensors(rep)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._sampled_core(rep, B)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._graph_out = self._sampled_core(rep, B)
        for t, v in zip(self._state_tensors(rep), snap):
            t.copy_(v)
        self._graph, self._graph_B, self._graph_rep = g, B, id(rep)
        return g

    def _state_tensors(self, rep):
        ts = [p.data for m in (self.actors, self.critics, self.actors_target, self.critics_target)
              for p in m.parameters()]
        for opt in (self.actor_optimizer, self.critic_optimizer):
            for st in opt.state.values():
                ts += [v for v in st.values() if torch.is_tensor(v)]
        return ts + [rep.counter]

    def update(self, B=None, use_graph=True, idx=None, replay=None):
        """One update_myown-equivalent; returns (loss_q, loss_a) device scalars."""
        B = B or self.batch_size
        rep = replay if replay is not None else (self.replay if self.replay is not None else self.memory.dev)
        if len(rep) < B:
            raise ValueError(f"replay holds {len(rep)} transitions, cannot sample {B} distinct rows")
        if self.device.type == "cuda" and self.fused_learner and (self.world > 1 or (idx is None and use_graph)):
            # the fused learner: one graph (world == 1) or one per segment between the gradient
            # all-reduces (world > 1, also for eager calls: the torch path would all-reduce per module)
            fu = self.fused(B, rep)
            if idx is not None or not use_graph:
                return fu.run(idx)
            if getattr(fu, "graphs", None) is None:
                fu.capture()
            fu.replay()
            return fu.loss[0], fu.loss[1]
        if idx is None and use_graph and self.device.type == "cuda" and self.world == 1:
            if self._graph is None or self._graph_B != B or self._graph_rep != id(rep):
                self.capture(B, rep)
            self._graph.replay()
            return self._graph_out
        return self._sampled_core(rep, B, idx)

    def _flat_state(self):
        """Flat float64 parameter / target / Adam-moment buffers and the shared int32 Adam step
        counter, built once.  The modules' parameters and the torch optimisers' ``exp_avg`` /
        ``exp_avg_sq`` become views of them (moments the torch path already accumulated carry over),
        so the fused plans and the torch-autograd path share one optimiser state; the torch path
        copies the counter into its per-parameter ``step`` tensors before stepping (``_core``)."""
        if self._fstate is not None:
            return self._fstate
        dev = self.device
        cp, ap = list(self.critics.parameters()), list(self.actors.parameters())
        nC, nA = sum(p.numel() for p in cp), sum(p.numel() for p in ap)
        z = lambda n: torch.zeros(n, dtype=F64, device=dev)   # noqa: E731
        flat, tflat, m1, m2 = z(nC + nA), z(nC + nA), z(nC + nA), z(nC + nA)
        _rebind(cp + ap, flat)
        _rebind(list(self.critics_target.parameters()) + list(self.actors_target.parameters()), tflat)
        step = torch.zeros(1, dtype=torch.int32, device=dev)
        o, steps = 0, []
        for opt, ps in ((self.critic_optimizer, cp), (self.actor_optimizer, ap)):
            for p in ps:
                n = p.numel()
                st = opt.state.setdefault(p, {})
                if "exp_avg" in st:
                    m1[o:o + n].copy_(st["exp_avg"].reshape(-1))
                    m2[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                    steps.append(int(st["step"].item()))
                st["exp_avg"] = m1[o:o + n].view_as(p)
                st["exp_avg_sq"] = m2[o:o + n].view_as(p)
                if "step" not in st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
                o += n
        if steps:
            step.fill_(steps[0])
        self._graph = None          # a torch-path graph captured before holds the old storages
        self._fstate = dict(nC=nC, nA=nA, flat=flat, tflat=tflat, m1=m1, m2=m2, step=step)
        self._opt_steps = [st["step"] for opt in (self.critic_optimizer, self.actor_optimizer)
                           for st in opt.state.values()]
        return self._fstate

    def invalidate_graphs(self):
        """Drop every captured update graph (a checkpoint load changed a seed the graphs bake in)."""
        self._graph = None
        if self._fu is not None:
            self._fu.graphs = None

    def has_graph(self):
        return self._graph is not None or getattr(self._fu, "graphs", None) is not None

    def fused(self, B, rep):
        """The FusedUamUpdate of (B, replay), built on first use.  Building it moves the parameters
        into flat buffers (the modules keep views), so a torch-path graph captured before is dropped."""
        if self._fu is None or self._fu.B != B or self._fu.rep is not rep:
            self._graph = None
            self._fu = FusedUamUpdate(self, B, rep)
        return self._fu

    # ------------------------------------------------------------------ reference API
    def choose_action(self, state, cur_total_step, cur_episode, step, mini_noise_eps, noise_start_level,
                      actor_hiddens=None, use_allNeigh_wRadar=False, use_selfATT_with_radar=False, own_obs_only=False,
                      use_nearestN_neigh_wRadar=False, noisy=True, use_GRU_flag=False):
        """UAM/maddpg:597-676 (E = 1): returns (actions (N, 2) float64, noise, hiddens, act_hn)."""
        N = self.n_agents
        own = torch.as_tensor(np.stack(state[0]), dtype=F64, device=self.device).view(1, N, 7)
        radar = torch.as_tensor(np.stack(state[2]), dtype=F64, device=self.device).view(1, N, 18)
        for i in range(N):
            self.var[i] = float(noise_scale(torch.tensor([cur_episode]), mini_noise_eps, noise_start_level)[0])
        ep = torch.full((1,), int(cur_episode), dtype=torch.int32, device=self.device)
        a = self.act(own, radar, ep, noisy=noisy, eps_end=mini_noise_eps, noise_start=noise_start_level)
        self.steps_done += 1
        return a[0].cpu().numpy(), np.zeros(2), actor_hiddens, torch.zeros(N, self.n_actions)

    def update_myown(self, i_episode, total_step_count, UPDATE_EVERY, single_eps_critic_cal_record,
                     transfer_learning=False, use_allNeigh_wRadar=False, use_selfATT_with_radar=False,
                     use_nearestN_neigh_wRadar=False, wandb=None, full_observable_critic_flag=False,
                     use_GRU_flag=False):
        """UAM/maddpg:304-595: guard len(memory) <= batch_size, one gradient iteration, soft update."""
        if len(self.memory) <= self.batch_size:
            return None, None, single_eps_critic_cal_record
        lq, la = self.update(self.batch_size, use_graph=False, replay=self.memory.dev)
        return [lq], [la], single_eps_critic_cal_record

    def save_model(self, episode, file_path):
        os.makedirs(file_path, exist_ok=True)
        sd = {k: v.detach().cpu() for k, v in self.actors.state_dict().items()}
        torch.save(sd, os.path.join(file_path, "episode_" + str(episode) + "_actor_net.pth"))

    def load_model(self, filePath, full_observable_critic_flag=False):
        for path in filePath:
            sd = torch.load(path, map_location="cpu", weights_only=True)
            self.actors.load_state_dict({k: v.to(F64) for k, v in sd.items()})
        self.actors_target.load_state_dict(self.actors.state_dict())
        self.critics_target.load_state_dict(self.critics.state_dict())
        self._graph = None
