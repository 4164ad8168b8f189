"""MADDPG learner of ``one_model_att`` on the device (ATT/maddpg:31-570).

Batched API (what the bench and the vectorised loop use):
    act(own, radar, nei, episode)        choose_action for all E envs (actor + noise kernel)
    push(...)                            replay push of E transitions (one HIP launch)
    update(B)                            one ``update_myown``-equivalent: N gradient iterations
                                         (sample B -> critic Adam step -> actor Adam step) then the
                                         Polyak update, replayed from a captured HIP graph.
Reference API (drop-in for ma_main, E = 1): ``choose_action``, ``update_myown``, ``memory``,
``save_model``, ``load_model`` with the reference's signatures and return values.

Canonical contract: D0 = 6 + 4(N-1) (R1), neighbour tensor (K, 6) (R2),
N-agent critic (R3), the actor always gets [own, radar, nei] (R4).
"""
import math
import os
import warnings

import numpy as np
import torch
import torch.nn.functional as F

from . import fused, ops, parallel, trace
from .memory import DeviceReplay, ReplayMemory
from .networks import ActorNetwork_ATT_TwoPortion, CriticCombine, FlatParams


class _Adam:
    """torch.optim.Adam (defaults, lr from the reference) on a FlatParams buffer."""

    def __init__(self, flat, lr, betas=(0.9, 0.999), eps=1e-8):
        self.flat, self.lr, self.betas, self.eps = flat, lr, betas, eps
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=flat.data.device)

    def zero_grad(self):
        self.flat.zero_grad()

    def step(self):
        self.step_t.add_(1)
        ops.adam_flat(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, self.step_t, self.lr,
                      self.betas[0], self.betas[1], self.eps)

    def state(self):
        return [self.exp_avg, self.exp_avg_sq, self.step_t]


def _noise_scale(episode, eps_end, start_scale=1, end_scale=0):
    """get_custom_linear_scaling_factor (ATT/maddpg:563-570)."""
    if episode <= eps_end:
        slope = (end_scale - start_scale) / (eps_end - 1)
        return start_scale + slope * (episode - 1)
    return end_scale


class MADDPG:
    def __init__(self, actor_dim, critic_dim, dim_act, actor_hidden_state_size=64, gru_history_length=10,
                 n_agents=5, args=None, cr_lr=1e-3, ac_lr=1e-3, gamma=0.95, tau=0.01,
                 full_observable_critic_flag=True, device=None, seed=None, memory_length=None, batch_size=None,
                 process_group=None, blas="cublas", fused=True):
        self.args = args
        self.fused = bool(fused)     # fused HIP learner (fused.py); False = autograd over layers.py
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.n_agents = N = int(n_agents)
        self.n_actions = int(dim_act)
        self.D0 = 6 + 4 * (N - 1)
        if actor_dim[0] != self.D0:
            warnings.warn(f"actor_dim[0]={actor_dim[0]} != 6+4(N-1)={self.D0}; using the env's width (contract R1)")
        self.n_actor_dim = [self.D0, actor_dim[1], actor_dim[2]]
        self.n_critic_dim = [self.D0, critic_dim[1], critic_dim[2]]
        if not full_observable_critic_flag:
            raise NotImplementedError("one_model_att runs with full_observable_critic_flag=True (ATT/main:77)")
        if seed is not None:
            torch.manual_seed(seed)
        # rocBLAS picks split-K kernels for the reduction-heavy weight-gradient GEMMs
        # (dW = G^T X over 5k-20k rows); hipBLASLt ran them on 1-6 workgroups (a round-2 microbenchmark, in the git history)
        torch.backends.cuda.preferred_blas_library(blas)
        self.actors = ActorNetwork_ATT_TwoPortion(self.n_actor_dim, dim_act).to(self.device)
        self.critics = CriticCombine(self.n_critic_dim, N, dim_act).to(self.device)
        self.actors_target = ActorNetwork_ATT_TwoPortion(self.n_actor_dim, dim_act).to(self.device)
        self.critics_target = CriticCombine(self.n_critic_dim, N, dim_act).to(self.device)
        self.fa, self.fc = FlatParams(self.actors), FlatParams(self.critics)
        self.fa_t, self.fc_t = FlatParams(self.actors_target), FlatParams(self.critics_target)
        self.fa_t.data.copy_(self.fa.data)
        self.fc_t.data.copy_(self.fc.data)
        for p in list(self.actors_target.parameters()) + list(self.critics_target.parameters()):
            p.requires_grad_(False)
        self.GAMMA, self.tau = float(gamma), float(tau)
        self.actor_optimizer = _Adam(self.fa, ac_lr)
        self.critic_optimizer = _Adam(self.fc, cr_lr)
        mem_len = memory_length or (getattr(args, "memory_length", None) or int(1e5))
        self.batch_size = batch_size or (getattr(args, "batch_size", None) or 512)
        self.memory = ReplayMemory(mem_len, device=self.device)
        self.replay = None
        self.var = [1.0 for _ in range(N)]
        self.noise_seed = int(seed or 0) * 7919 + 1
        self.noise_counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.grads = None
        if self.world > 1:
            self._share_grads()
        self._graph = None
        self._graph_B = None
        self.steps_done = 0
        self._last_src = None
        self._fplans = {}
        self._infer = None

    # ------------------------------------------------------------------ batched API
    def attach_replay(self, capacity, seed=0):
        self.replay = DeviceReplay(capacity, self.n_agents, self.D0, 18, self.device, seed=seed)
        return self.replay

    @torch.no_grad()
    def act(self, own, radar, nei, episode=None, noisy=True, eps_end=8000, noise_start=1.0, noise_out=None):
        """Batched choose_action (ATT/maddpg:455-550): tanh actor + N(0, var^2) noise, clamp."""
        if self.fused:
            if self._infer is None:
                self._infer = fused.ActorInfer(self.actors, self.n_agents, self.D0, self.device)
            # noisy: the output layer, noise and clamp in one launch (aac_actor_out_noise)
            nz = (episode, eps_end, noise_start, 0.0, self.noise_seed, self.noise_counter, noise_out) if noisy else None
            return self._infer(own, radar, nei, noise=nz).view(*own.shape[:-1], 2)
        a = self.actors([own, radar, nei]).contiguous()
        if noisy:
            ops.noise_clamp(a, episode, eps_end, noise_start, self.noise_seed, self.noise_counter, noise_out)
        return a

    def _allreduce(self, flat):
        if self.world > 1:
            parallel.allreduce_mean_(flat.grad, self.pg)

    def _share_grads(self):
        """world > 1: the critic's and the actor's flat gradients become the two halves of one
        buffer [critic | actor], so the fused learner averages both with one collective."""
        nc, na = self.fc.numel, self.fa.numel
        self.grads = torch.zeros(nc + na, dtype=torch.float32, device=self.device)
        for flat, g in ((self.fc, self.grads[:nc]), (self.fa, self.grads[nc:])):
            flat.grad = g
            for p, off, k in flat.slices:
                p.grad = g[off:off + k].view_as(p)

    def _allreduce_grads(self, critic, actor):
        """SUM over the ranks of the critic and / or actor gradient (one collective; the fused plan's
        Adam launches apply the 1 / world)."""
        nc = self.fc.numel
        t = self.grads if (critic and actor) else (self.grads[:nc] if critic else self.grads[nc:])
        parallel.allreduce_sum_(t, self.pg)

    def _targets(self, b, B):
        """y for all N iterations at once.  The target networks only change in the Polyak step
        after the N iterations (ATT/maddpg:436-438), so evaluating them for the N independently
        sampled batches in one batched forward is exactly the reference's per-iteration value."""
        N = self.n_agents
        with torch.no_grad():
            na = self.actors_target([b["n_own"], b["n_radar"], b["n_nei"]])
            q_next = self.critics_target([b["n_own"], b["n_radar"]], na).squeeze(-1)      # (N*B,)
            done_any = (b["done"] == 1).any(dim=1).to(torch.float32)
            rew = b["rew"].reshape(N, B, N).diagonal(dim1=0, dim2=2).transpose(0, 1)      # r[:, i] of batch i
            # ATT/maddpg:357: tar_Q_before_rew = GAMMA * Q' * (1 - done), kept for the records
            self._last_pre = self.GAMMA * q_next * (1 - done_any)
            return rew.reshape(-1) + self._last_pre

    def _iteration(self, b, target, agent, freeze_actor=False):
        q = self.critics([b["s_own"], b["s_radar"]], b["act"])
        loss_q = F.mse_loss(q, target.unsqueeze(1))
        self.critic_optimizer.zero_grad()
        loss_q.backward()            # fused layers write the critic's grads into its flat buffer
        self._allreduce(self.fc)
        self.critic_optimizer.step()
        if freeze_actor:
            # transfer learning, i_episode <= 10000 (ATT/maddpg:411-416): the actor loss is computed
            # and returned, but no actor backward and no actor Adam step (moments and count untouched)
            with torch.no_grad():
                a_pi = self.actors([b["s_own"], b["s_radar"], b["s_nei"]])
                loss_a = -self.critics([b["s_own"], b["s_radar"]], a_pi).mean()
            return loss_q.detach(), loss_a.detach(), q.detach(), target
        a_pi = self.actors([b["s_own"], b["s_radar"], b["s_nei"]])
        loss_a = -self.critics([b["s_own"], b["s_radar"]], a_pi).mean()
        self.actor_optimizer.zero_grad()
        self.critics.slot.enabled = False    # only d/da flows through the critic here (ATT/maddpg:421-425)
        try:
            loss_a.backward()
        finally:
            self.critics.slot.enabled = True
        self._allreduce(self.fa)
        self.actor_optimizer.step()
        return loss_q.detach(), loss_a.detach(), q.detach(), target

    def _fused_plan(self, B, rep=None):
        if rep is None:
            rep = self.replay if self.replay is not None else self.memory.dev
        key = (B, id(rep))
        if key not in self._fplans:
            self._fplans[key] = fused.FusedUpdate(self, rep, B)
        return self._fplans[key]

    def _update_core(self, B, idx_list=None, rep=None, soft=True, freeze_actor=False):
        if rep is None:
            rep = self.replay if self.replay is not None else self.memory.dev
        N = self.n_agents
        idx = None if idx_list is None else torch.cat([i.reshape(-1) for i in idx_list])
        if self.fused and not freeze_actor:     # the frozen-actor phase runs on the autograd path
            rep.check_sample(B)
            fu = self._fused_plan(B, rep)
            fu.run(idx, soft=soft)
            return fu
        ball = rep.sample_batch(B, idx, nb=N)           # N independent batches, one launch each
        target = self._targets(ball, B)
        stats = []
        for agent in range(N):
            b = {k: v[agent * B:(agent + 1) * B] for k, v in ball.items()}
            stats.append(self._iteration(b, target[agent * B:(agent + 1) * B], agent, freeze_actor))
        self._last_rew = ball["rew"].reshape(N, B, N)
        if soft:        # ATT/maddpg:436-438: soft update when i_episode % UPDATE_EVERY == 0
            ops.polyak_flat(self.fc_t.data, self.fc.data, self.tau)
            ops.polyak_flat(self.fa_t.data, self.fa.data, self.tau)
        return stats

    def _snapshot(self):
        rep = self.replay if self.replay is not None else self.memory.dev
        ts = [self.fa.data, self.fc.data, self.fa_t.data, self.fc_t.data, rep.counter]
        ts += self.actor_optimizer.state() + self.critic_optimizer.state()
        return ts, [t.clone() for t in ts]

    def capture(self, B, warmup=2):
        """Capture one update_myown-equivalent into HIP graphs (state restored afterwards).

        world == 1: one graph.  world > 1 (fused learner) over RCCL: one graph with the gradient
        all-reduces captured in it (parallel.capturable).  Otherwise (gloo, AAC_GRAPH_COLL=0): one
        graph per segment between the all-reduces, the collectives issued between the replays (RCCL
        enqueues them on its own stream, ordered against the current stream)."""
        if self.world > 1 and not self.fused:
            self._graph = None
            return None
        ts, saved = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._update_core(B)
        torch.cuda.current_stream().wait_stream(s)
        if self.world > 1:
            fu = self._fused_plan(B)
            segs, colls = fu.segments()
            graphs = []
            for seg in segs:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for op in seg:
                        op()
                graphs.append(g)
            self._graph = (graphs, colls)
            self._graph_stats = fu
        elif self.fused:
            # one graph; the fused plan's overlapped segments put branch B on a second stream
            fu = self._fused_plan(B)
            side = torch.cuda.Stream()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fu.run_streams(side)
            self._graph_stats = fu
            self._graph = g
            self._side = side
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._graph_stats = self._update_core(B)
            self._graph = g
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
        if isinstance(self._graph, tuple):
            graphs, colls = self._graph
            for k, g in enumerate(graphs):
                with trace.range(f"update.seg{k}"):
                    g.replay()
                if k < len(colls):
                    with trace.range("allreduce"):
                        colls[k]()
        else:
            with trace.range("update.graph"):
                self._graph.replay()

    def update(self, B=None, use_graph=True, idx_list=None, want_stats=True, replay=None, soft_update=True,
               freeze_actor=False):
        """One update_myown-equivalent on the device replay (no host synchronisation).  Returns
        [(loss_q, loss_a, q, target)] per iteration (computed on demand: ``want_stats=False``
        launches nothing beyond the update itself).  ``replay`` defaults to the attached batched
        replay, else the reference-API memory.  ``soft_update=False`` (UPDATE_EVERY > 1 between soft
        updates, ATT/maddpg:436-438) keeps the targets and runs eagerly.  ``freeze_actor`` (the
        transfer-learning phase of ATT/maddpg:411-416) runs the critic steps only, eagerly."""
        B = B or self.batch_size
        if replay is not None or not soft_update or freeze_actor:
            self._last_src = self._update_core(B, idx_list, replay, soft=soft_update, freeze_actor=freeze_actor)
            return self.last_stats if want_stats else None
        if idx_list is None and use_graph and (self.world == 1 or self.fused):
            (self.replay if self.replay is not None else self.memory.dev).check_sample(B)
            if self._graph is None or self._graph_B != B:
                self.capture(B)
            self._replay()
            self._last_src = self._graph_stats
        else:
            self._last_src = self._update_core(B, idx_list)
        return self.last_stats if want_stats else None

    @property
    def last_stats(self):
        src = self._last_src
        return src.stats() if isinstance(src, fused.FusedUpdate) else src

    # ------------------------------------------------------------------ reference API
    def choose_action(self, state, cur_total_step, cur_episode, step, mini_noise_eps, noise_start_level,
                      actor_hiddens=None, noisy=True):
        """ATT/maddpg:455 signature; state = norm_state lists (E = 1)."""
        N = self.n_agents
        own = torch.from_numpy(np.stack(state[0])).float().to(self.device).reshape(1, N, -1)
        grid = torch.from_numpy(np.stack(state[1])).float().to(self.device).reshape(1, N, -1)
        nei = torch.stack([torch.from_numpy(np.stack(x)).float().reshape(N - 1, 6) for x in state[2]])
        nei = nei.to(self.device).reshape(1, N, N - 1, 6)
        for i in range(N):
            self.var[i] = _noise_scale(cur_episode, mini_noise_eps, noise_start_level)
        with torch.no_grad():
            act = self.actors([own, grid, nei])[0]
        noise_value = np.zeros(2)
        if noisy:
            acts = []
            for i in range(N):
                noise_value = np.random.randn(2) * self.var[i]
                a = act[i] + torch.from_numpy(noise_value).float().to(self.device)
                acts.append(torch.clamp(a, -1.0, 1.0))
            act = torch.stack(acts)
        self.steps_done += 1
        hid = torch.zeros(N, self.n_actions)
        if actor_hiddens is not None:
            hid_in = torch.as_tensor(np.asarray(actor_hiddens), dtype=torch.float32)
        else:
            hid_in = torch.zeros(N, 64)
        return act.cpu().numpy(), noise_value, hid_in, hid

    def update_myown(self, i_episode, total_step_count, UPDATE_EVERY, single_eps_critic_cal_record,
                     transfer_learning=False, wandb=None, full_observable_critic_flag=True):
        """ATT/maddpg:219 signature and returns; the work is ``update`` on the device ring.

        The soft update runs when ``i_episode % UPDATE_EVERY == 0`` (ATT/maddpg:436-438).  Each
        gradient iteration appends the reference's 8-field record (ATT/maddpg:372-379)."""
        if len(self.memory) <= self.batch_size:
            return None, None, single_eps_critic_cal_record
        if transfer_learning and i_episode > 10000:
            # ATT/maddpg:411-416: after episode 10000 a transfer run indexes the one-model actor
            # optimiser as a list (self.actor_optimizer[agent]), which raises in the reference
            raise NotImplementedError("transfer_learning past episode 10000: the reference's branch indexes its "
                                      "single actor optimiser as a list (ATT/maddpg:413-416) and fails")
        soft = i_episode % UPDATE_EVERY == 0
        # transfer learning up to episode 10000: the actor is frozen (critic steps only)
        stats = self.update(self.batch_size, use_graph=False, replay=self.memory.dev, soft_update=soft,
                            freeze_actor=bool(transfer_learning))
        c_loss = [s[0] for s in stats]
        a_loss = [s[1] for s in stats]
        single_eps_critic_cal_record.extend(self.critic_records(stats))
        return c_loss, a_loss, single_eps_critic_cal_record

    def critic_records(self, stats=None):
        """The 8-field ``single_eps_critic_cal_record`` entry of each gradient iteration of the last
        update (ATT/maddpg:372-379): [target Q before the reward (B,), the batch rewards (B, N), the
        target Q (B, 1), the critic loss, and the (min, max) of each].  The target before the reward
        is gamma Q' (1 - done) as the TD head computed it (not re-derived as y - r, which rounds)."""
        stats = self.last_stats if stats is None else stats
        src = self._last_src
        out = []
        for i, (loss_q, _, _, y) in enumerate(stats):
            if isinstance(src, fused.FusedUpdate):
                rew, pre = src.batch_rewards(i), src.pre_reward_target(i)
            else:
                B = y.numel()
                rew, pre = self._last_rew[i], self._last_pre[i * B:(i + 1) * B]
            r = rew.detach().cpu().numpy()
            after = y.detach().cpu().numpy().reshape(-1, 1)
            before = pre.detach().cpu().numpy().reshape(-1)
            loss = loss_q.detach().cpu().numpy()
            out.append([before, r, after, loss, (before.min(), before.max()), (r.min(), r.max()),
                        (after.min(), after.max()), (loss.min(), loss.max())])
        return out

    def save_model(self, episode, file_path):
        """ATT/maddpg:131-139: actor state_dict only, reference key names."""
        os.makedirs(file_path, exist_ok=True)
        torch.save(self.actors.reference_state_dict(), os.path.join(file_path, f"episode_{episode}_actor_net.pth"))

    def load_model(self, filePath):
        """ATT/maddpg:106-129 (weights_only load)."""
        for path in filePath:
            self.actors.load_reference_state_dict(torch.load(path, weights_only=True, map_location="cpu"))
        self.fa_t.data.copy_(self.fa.data)
        self.fc_t.data.copy_(self.fc.data)

