"""Vectorised ``ma_main`` training loops on one GPU (the drop-in for the E > 1 use of the hot path).

``ATT/main:248-668`` runs, per env step: ``choose_action`` -> ``env.step`` + ``ss_reward`` ->
``memory.push`` -> ``update_myown`` -> termination / ``reset_world``.  ``Trainer`` runs the same
iteration over E envs at once:

  act            actor forward + exploration noise for E x N agents (``ATT/maddpg:455-570``)
  step_tail      env step + ss_reward + termination, the replay push of the E transitions and the
                 OD-bank auto-reset of the finished envs in one launch (``aac_env_step_tail``)
  update         one ``update_myown`` (N gradient iterations + Polyak, ``ATT/maddpg:219-440``) as
                 one HIP-graph replay

``model="gru"`` is the ``MADDPG_ownENV_randomOD_Wgru_radar`` loop (GRU actor, hidden states carried
per agent and zeroed at episode start, ``WGRU/ma_main:476-647``); ``UamTrainer`` is the UAM loop
(``UAM/main:361-640``).  ``bench.py`` times these loops; the checkpoint tests resume them.

Module flags (environment variables read at import):
  AAC_FUSED_TAIL   0 / 1 forces the separate / fused env tail (default fused)
  AAC_STEP_GRAPH   0: the ATT training step launched from the host (default: graph replays, two
                   steps per replay in bench.py; config 3 0.818 -> 0.812 ms per step)
  AAC_STEP_GRAPH_GRU 0: the GRU training step launched from the host (default: one graph replay;
                   config 4 0.3331 -> 0.3310 ms per step)
  AAC_OVERLAP_RESET 1: separate-launch auto-reset on a side stream (measured slower, off)
  AAC_UAM_OVERLAP_RESET 0: the UAM loop's packed auto-reset before the update instead of on a side
                   stream beside it (default on: config 5 0.543 -> 0.519 ms per step)
  AAC_UAM_STEP_GRAPH 1: the UAM training step as graph replays (measured slower, off)
"""
import os

import torch

from . import trace

NO_GRAPH = False
OVERLAP_RESET = os.environ.get("AAC_OVERLAP_RESET", "0") == "1"   # measured slower: 1.241 vs 1.164 ms
# replay push, GRU hidden-row zeroing and auto-reset fused into the env step launch (aac_env_step_tail):
# config 3 env part 0.084 -> 0.070 ms per step (tools/tail_probe.py); config 4 (one round of 1024
# workgroups since the 4-env workgroups) 0.378 -> 0.371 ms per step.  AAC_FUSED_TAIL=0 / 1 forces it.
_FT = os.environ.get("AAC_FUSED_TAIL")
FUSED_TAIL = None if _FT is None else _FT == "1"
# config 3: the timed steps (act + fused env tail + update) replay captured HIP graphs, two steps per
# replay in bench.py (both buffer parities in one graph).  One step per replay measured neutral in
# rounds 3-5 (0.8173 vs 0.8178 ms); two per replay halve the ~6-9 us GPU idle at each graph-launch
# boundary: 0.8102-0.8119 vs 0.8167-0.8184 ms interleaved (profiles/r06_step_graph_ab.txt).
# AAC_STEP_GRAPH=0 launches the steps from the host
STEP_GRAPH = os.environ.get("AAC_STEP_GRAPH", "1") == "1"
# the GRU training step (config 4) as one graph replay: its host-side launch sequence left the GPU idle
# ~5 % of a step (act, env tail and update launched from Python); AAC_STEP_GRAPH_GRU=0 keeps it eager
STEP_GRAPH_GRU = os.environ.get("AAC_STEP_GRAPH_GRU", "1") == "1"
# config 5: the UAM env step and the replay push as one launch was built (bit-exact) and measured
# slower -- the step launch grew 188 -> 234 us against the 23-us push launch it replaced (226-231 vs
# 238-240 M agent-env-steps/s; profiles/r05_uam_tail_ab.txt) -- and removed in round 6
# config 5: the packed auto-reset (UAM/env:551-771) on a side stream beside the update, whose small
# float64 launches leave most CUs idle: 0.543 -> 0.519 ms per step, interleaved
# (profiles/r05_uam_overlap_reset_ab.txt); AAC_UAM_OVERLAP_RESET=0 runs it before the update
UAM_OVERLAP_RESET = os.environ.get("AAC_UAM_OVERLAP_RESET", "1") == "1"
# config 5: the whole UAM training step (act, env step, replay push with the ring position in device
# words, auto-reset beside the update) as graph replays, two steps per replay in bench.py
# (AAC_UAM_STEP_GRAPH=1; bit-identical, test_uam_whole_step_graph_equals_eager).  Measured slower than
# the host-launched step (0.5167 / 0.5189 vs 0.5115 / 0.5144 ms interleaved, profiles/r06_uam_step_graph_ab.txt),
# so off by default
UAM_STEP_GRAPH = os.environ.get("AAC_UAM_STEP_GRAPH", "0") == "1"


class CheckpointMixin:
    """Full-state checkpoint of the training loop (multi_agent_aac_amd/checkpoint.py): learner,
    replay, env state + episode counters, and the loop's current observation rows (+ GRU hidden
    states).  A run resumed from it continues bit-identically (tests/test_checkpoint_gpu.py)."""

    def checkpoint_parts(self):
        extra = {f"cur.{k}": v for k, v in vars(self.cur).items() if torch.is_tensor(v)}
        if getattr(self, "gru", False):
            extra["h"] = self.h
        return dict(learner=self.model, replay=self.replay, env=self.env, extra=extra)

    def save_checkpoint(self, path):
        from . import checkpoint
        return checkpoint.save(path, **self.checkpoint_parts())

    def load_checkpoint(self, path):
        from . import checkpoint
        try:
            return checkpoint.load(path, **self.checkpoint_parts())
        finally:
            # whole-step graphs bake the noise seed and the ring position word: re-capture / re-seed
            # them whatever the load did (a refused file changes nothing, but re-capturing is cheap)
            if hasattr(self, "_sg"):
                self._sg, self._sg2 = {}, {}
            self._pos_dirty = True


class Trainer(CheckpointMixin):
    """Vectorised ATT/main loop (configs 2-3) or WGRU/ma_main loop (``model="gru"``, config 4) on one
    GPU: E envs x N agents, B-row updates from a device replay of ``memory`` rows."""

    def __init__(self, E, N, B, memory, radar, seed, pg=None, model="att", maps=1):
        from . import world
        from .env import BatchedEnv
        from .maddpg import MADDPG
        self.E, self.N, self.B = E, N, B
        self.gru = model == "gru"
        # config 4 runs the randomOD_Wgru_radar env (obstacle radar, per-agent WGRU reward, 6-wide own
        # rows, max_spd 10, episodes of 150 steps); configs 2-3 the one_model_att env
        variant = "wgru" if self.gru else "att"
        if maps > 1:      # the 8-map stack, seeds 2026..2033; one OD bank per map
            self.occ = world.map_stack(range(2026, 2026 + maps))
            self.bank = world.MapBanks(self.occ, n_pairs=max(8192, 65536 // maps), seed=2026 + seed, max_wp=32)
        else:
            self.occ = world.synthetic_map(2026)
            self.bank = world.ODBank(self.occ, n_pairs=65536, seed=2026 + seed, max_wp=32)
        self.env = BatchedEnv(E, N, self.occ, radar_mode=None if self.gru else radar, max_wp=32, variant=variant)
        self.env.set_od_bank(self.bank, seed=1234 + seed)
        D0 = 6 + 4 * (N - 1)
        if self.gru:
            from . import gru
            # WGRU/ma_main:380-389: actor_dim = critic_dim = [6, 18, 6], 64 hidden units
            self.model = gru.MADDPG([6, 18, 6], [6, 18, 6], 2, 64, 10, n_agents=N, seed=777, batch_size=B,
                                    memory_length=memory, process_group=pg, own_width=self.env.D0)
            # hidden states as a ping-pong pair: act reads h[k] and writes the next hidden into h[1 - k]
            # (one act plan per buffer set, no copies)
            self.hp = [torch.zeros(E, N, 64, device="cuda"), torch.zeros(E, N, 64, device="cuda")]
            self.h = self.hp[0]
        else:
            self.model = MADDPG([D0, 18, 6], [D0, 18, 6], 2, n_agents=N, seed=777, batch_size=B,
                                memory_length=memory, process_group=pg)
        self.model.noise_seed = 99 + seed
        self.replay = self.model.attach_replay(memory, seed=seed)
        self.cur = self.env.alloc_buffers()
        self.nxt = self.env.alloc_buffers()
        self.episode = self.env_episode_view()
        self.env.auto_reset(None, out=self.cur)      # all envs: first OD draw + initial obs
        self.env_events = []
        self.fused_tail = True if FUSED_TAIL is None else FUSED_TAIL
        self.bufs = [self.cur, self.nxt]
        self._sg = {}                                 # parity -> captured whole-step graph
        self.pos_dev = torch.zeros(2, dtype=torch.int64, device="cuda")   # ring position ping-pong
        self._pos_dirty = True       # the host mirror moved outside step_graph: re-seed pos_dev
        # debug surface: callables run around each eager step --
        # pre(trainer) before the act launch, post(trainer, act, cur, nxt) after the env step (before
        # the auto-reset of an unfused tail and before the update).  A step with hooks runs eagerly
        # (no whole-step graph).  tests/oracle_diff.py hooks the C oracle in this way.
        self.pre_step_hooks, self.post_step_hooks = [], []

    def graph_ok(self):
        """Whole-step graphs: the fused env tail, one rank, the fused learner (ATT: AAC_STEP_GRAPH; the
        GRU step: AAC_STEP_GRAPH_GRU)."""
        if self.gru:
            return (STEP_GRAPH_GRU and self.fused_tail and self.model.world == 1 and not NO_GRAPH
                    and len(self.replay) > self.B and not self.hooked())
        return (STEP_GRAPH and self.fused_tail and self.model.world == 1 and self.model.fused
                and not NO_GRAPH and len(self.replay) > self.B and not self.hooked())

    def hooked(self):
        return bool(self.pre_step_hooks or self.post_step_hooks)

    def _step_body(self, p, side=None):
        """The launches of one training step whose current buffers are bufs[p] (act + env step tail +
        update_myown), for capture: the ring position is read from / advanced in pos_dev[p] /
        pos_dev[1 - p]."""
        c, n = self.bufs[p], self.bufs[1 - p]
        if self.gru:
            # the hidden-state pair flips with the buffer pair: parity p reads hp[p ^ hoff]
            hin, hout = self.hp[p ^ self._hoff], self.hp[1 - (p ^ self._hoff)]
            act, hn = self.model.act(c.own, c.radar, hin, self.episode, noisy=True, h_out=hout)
            srcs = [c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei, hin, hn]
            self.env.step_tail(act, out=n, replay=self.replay, srcs=srcs, zero_rows=hn,
                               pos_io=(self.pos_dev[p], self.pos_dev[1 - p]))
            self.model._plan(self.B).run()
            return
        act = self.model.act(c.own, c.radar, c.nei, self.episode, noisy=True)
        srcs = [c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei]
        self.env.step_tail(act, out=n, replay=self.replay, srcs=srcs, pos_io=(self.pos_dev[p], self.pos_dev[1 - p]))
        self.model._fused_plan(self.B).run_streams(side)

    def _capture_step(self, p, steps=1):
        """``steps`` consecutive training steps from parity p (act + env step tail + update_myown
        each, parities alternating), captured as one HIP graph.  Nothing runs during the capture; the
        replay's host mirror is restored."""
        saved = (self.replay.pos, self.replay.size)
        side = None if self.gru else torch.cuda.Stream()
        if not self.gru:
            self.model._fused_plan(self.B)        # built outside the capture
        else:
            self.model._plan(self.B)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(steps):
                self._step_body(p ^ (k & 1), side)
        self.replay.pos, self.replay.size = saved
        return g, side

    def _graphs_current(self):
        gen = getattr(self.env, "bank_generation", 0)
        if (self._sg or getattr(self, "_sg2", None)) and getattr(self, "_sg_bank_gen", gen) != gen:
            self._sg, self._sg2 = {}, {}      # the env's OD bank / seed changed under the captured graphs
        self._sg_bank_gen = gen
        if self.gru and not self._sg and not getattr(self, "_sg2", None):
            # (re)capture: the hidden-state pair's offset against the buffer parity, as of now
            p = 0 if self.cur is self.bufs[0] else 1
            self._hoff = (0 if self.h is self.hp[0] else 1) ^ p

    def _advance_mirror(self, steps):
        if self._pos_dirty:
            # eager steps / a checkpoint load moved the host mirror: the graph reads pos_dev[p]
            p = 0 if self.cur is self.bufs[0] else 1
            self.pos_dev[p].fill_(self.replay.pos)
            self._pos_dirty = False
        rep = self.replay
        for _ in range(steps):
            rep.pos = (rep.pos + self.E) % rep.capacity
            rep.size = min(rep.size + self.E, rep.capacity)
            p = 0 if self.cur is self.bufs[0] else 1
            self.cur, self.nxt = self.nxt, self.cur
            if self.gru:
                self.h = self.hp[1 - (p ^ self._hoff)]

    def step_graph(self):
        """One training step as one graph replay (the same launches as ``step(update=True)``; the
        ring position lives in device words, the host keeps its mirror)."""
        p = 0 if self.cur is self.bufs[0] else 1
        self._graphs_current()
        if not self._sg:
            for q in (0, 1):
                self._sg[q] = self._capture_step(q)
        self._advance_mirror(0)
        with trace.range("step_graph"):
            self._sg[p][0].replay()
        self._advance_mirror(1)

    def step_graph_pair(self, steps=2):
        """``steps`` (even) training steps as ONE graph replay (the buffer parities in sequence): the
        GPU idles at each graph launch boundary (~6-9 us between the end of one replay and the first
        kernel of the next), so k steps per replay cut those gaps k-fold.  The same launches and
        results as ``steps`` ``step_graph`` calls."""
        assert steps >= 2 and steps % 2 == 0
        p = 0 if self.cur is self.bufs[0] else 1
        self._graphs_current()
        if not getattr(self, "_sg2", None):
            self._sg2 = {}
        if (p, steps) not in self._sg2:
            self._sg2[(p, steps)] = self._capture_step(p, steps=steps)
        self._advance_mirror(0)
        with trace.range("step_graph_pair"):
            self._sg2[(p, steps)][0].replay()
        self._advance_mirror(steps)

    def env_episode_view(self):
        # the env's own per-env episode counter (advanced by each auto-reset; 1 after the first)
        # drives the noise schedule (env e's own episode index, ATT/maddpg:476-477)
        return self.env.use_episode_buffer(torch.zeros(self.E, dtype=torch.int32, device="cuda"))

    def step(self, update=True, time_env=False):
        self._pos_dirty = True
        c, n = self.cur, self.nxt
        for f in self.pre_step_hooks:
            f(self)
        with trace.range("act"):
            if self.gru:
                hn_buf = self.hp[1] if self.h is self.hp[0] else self.hp[0]
                act, hn = self.model.act(c.own, c.radar, self.h, self.episode, noisy=True, h_out=hn_buf)
            else:
                act = self.model.act(c.own, c.radar, c.nei, self.episode, noisy=True)
        if time_env:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        if self.fused_tail:
            # step + replay push + zeroed next hidden rows (GRU) + auto-reset in the step launch
            # (aac_env_step_tail): the same results as the separate launches below
            with trace.range("env_step"):
                if self.gru:
                    srcs = [c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei, self.h, hn]
                    self.env.step_tail(act, out=n, replay=self.replay, srcs=srcs, zero_rows=hn)
                    self.h = hn
                else:
                    srcs = [c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei]
                    self.env.step_tail(act, out=n, replay=self.replay, srcs=srcs)
            if time_env:
                ev1.record()
                self.env_events.append((ev0, ev1))
            for f in self.post_step_hooks:
                f(self, act, c, n)
            self.cur, self.nxt = n, c
            if update and len(self.replay) > self.B:
                with trace.range("update"):
                    self.model.update(self.B, use_graph=not NO_GRAPH, want_stats=False)
            return
        with trace.range("env_step"):
            self.env.step(act, out=n)
        if time_env:
            ev1.record()
            self.env_events.append((ev0, ev1))
        for f in self.post_step_hooks:
            f(self, act, c, n)
        with trace.range("replay_push"):
            if self.gru:     # rows keep (cur_hidden, next_hidden) as WGRU/ma_main:636
                self.replay.push_batch(c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei, self.h,
                                       hn)
                self.h = hn
                from . import gru
                gru.reset_hidden(self.h, n.env_done)     # a new episode starts from zeros (WGRU/ma_main:476-478)
            else:
                self.replay.push_batch(c.own, c.radar, c.nei, act, n.reward, n.done, n.own, n.radar, n.nei)
        self.cur, self.nxt = n, c
        run_update = update and len(self.replay) > self.B
        # the auto-reset writes env state and the next observation rows, which the update never reads:
        # it may run on a side stream beside the update (the next act waits for both)
        with side_stream(self, run_update), trace.range("auto_reset"):
            self.env.auto_reset(n.env_done, out=n)
        if run_update:
            with trace.range("update"):
                self.model.update(self.B, use_graph=not NO_GRAPH, want_stats=False)
        join_side(self)


class side_stream:
    """Run the block on the trainer's side stream, ordered after the main stream's work so far (a
    no-op context when off)."""

    def __init__(self, tr, on, flag=None):
        self.tr, self.on = tr, on and (OVERLAP_RESET if flag is None else flag)

    def __enter__(self):
        if not self.on:
            return
        if getattr(self.tr, "_side", None) is None:
            self.tr._side = torch.cuda.Stream()
        self.tr._side.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.stream(self.tr._side)
        self._ctx.__enter__()
        self.tr._side_used = True

    def __exit__(self, *a):
        if self.on:
            self._ctx.__exit__(*a)


def join_side(tr):
    if getattr(tr, "_side_used", False):
        torch.cuda.current_stream().wait_stream(tr._side)
        tr._side_used = False


class UamTrainer(CheckpointMixin):
    """Vectorised UAM/main:361-640 loop on one GPU: actor + noise, env step, one replay row per
    aircraft, GPU auto-reset from the episode bank, one update_myown (one gradient iteration)."""

    def __init__(self, E, N, B, memory, seed, pg=None):
        from . import uam, uam_learner
        self.E, self.N, self.B = E, N, B
        self.gru = False
        # tdCPA outputs live (tcpa / dcpa per neighbour, conflict counts)
        self.env = uam.BatchedUAM(E, N, neighbours=True, tdcpa=True)
        self.env.set_bank(uam.build_bank(16384, N, seed=2026 + seed), seed=1234 + seed)
        # UAM/main:159-165: actor_dim = critic_dim = [7, (N-1)*5, 18, 6]
        dims = [7, (N - 1) * 5, 18, 6]
        self.model = uam_learner.MADDPG(dims, dims, 2, n_agents=N, seed=777, batch_size=B, memory_length=memory,
                                        process_group=pg)
        self.replay = self.model.attach_replay(memory, seed=seed)
        self.cur = self.env.alloc_buffers()
        self.nxt = self.env.alloc_buffers()
        self.episode = self.env.use_episode_buffer(torch.zeros(E, dtype=torch.int32, device="cuda"))
        self.env.auto_reset(None, out=self.cur)      # episode counters -> 1
        self.env_events = []
        self.pre_step_hooks, self.post_step_hooks = [], []      # as Trainer's
        self.bufs = [self.cur, self.nxt]
        self._sg, self._sg2 = {}, {}                  # parity -> captured whole-step graph (1 / 2 steps)
        self.pos_dev = torch.zeros(2, dtype=torch.int64, device="cuda")   # ring position ping-pong
        self._pos_dirty = True

    def graph_ok(self):
        """Whole-step graphs: one rank, the fused learner, the replay past one batch, no hooks."""
        m = self.model
        return (UAM_STEP_GRAPH and m.world == 1 and m.fused_learner and not NO_GRAPH
                and len(self.replay) > self.B and not self.hooked())

    def hooked(self):
        return bool(self.pre_step_hooks or self.post_step_hooks)

    def _step_body(self, p, side):
        """The launches of ``step(update=True)`` from buffer parity p, for capture: the push reads /
        advances the ring position in pos_dev[p] / pos_dev[1 - p] (aac_uam_push_io); the update is the
        fused learner's raw launches."""
        c, n = self.bufs[p], self.bufs[1 - p]
        act = self.model.act(c.own, c.radar, self.episode, noisy=True)
        self.env.step(act, out=n)
        self.replay.push_batch(c.own, c.radar, act, n.reward, n.done, n.own, n.radar,
                               pos_io=(self.pos_dev[p], self.pos_dev[1 - p]))
        fu = self.model.fused(self.B, self.replay)
        if side is not None:
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.env.auto_reset(n.env_done, out=n)
            fu.run()
            main.wait_stream(side)
        else:
            self.env.auto_reset(n.env_done, out=n)
            fu.run()

    def _capture_step(self, p, steps=1):
        saved = (self.replay.pos, self.replay.size)
        side = torch.cuda.Stream() if UAM_OVERLAP_RESET else None
        self.model.fused(self.B, self.replay)        # built outside the capture
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(steps):
                self._step_body(p ^ (k & 1), side)
        self.replay.pos, self.replay.size = saved
        return g, side

    def _advance_mirror(self, steps):
        if self._pos_dirty:
            p = 0 if self.cur is self.bufs[0] else 1
            self.pos_dev[p].fill_(self.replay.pos)
            self._pos_dirty = False
        rep, M = self.replay, self.E * self.N
        for _ in range(steps):
            rep.pos = (rep.pos + M) % rep.capacity
            rep.size = min(rep.size + M, rep.capacity)
            self.cur, self.nxt = self.nxt, self.cur

    def _graphs_current(self):
        gen = getattr(self.env, "bank_generation", 0)
        if (self._sg or self._sg2) and (getattr(self, "_sg_bank_gen", gen) != gen
                                        or getattr(self, "_sg_fu", None) is not self.model._fu):
            # the episode bank / seed changed, or the fused learner was rebuilt (new buffers), under
            # the captured graphs
            self._sg, self._sg2 = {}, {}
        self._sg_bank_gen = gen
        self._sg_fu = self.model.fused(self.B, self.replay)

    def step_graph(self):
        """One training step (``step(update=True)``'s launches) as one graph replay."""
        p = 0 if self.cur is self.bufs[0] else 1
        self._graphs_current()
        if p not in self._sg:
            self._sg[p] = self._capture_step(p)
        self._advance_mirror(0)
        with trace.range("step_graph"):
            self._sg[p][0].replay()
        self._advance_mirror(1)

    def step_graph_pair(self, steps=2):
        """``steps`` (even) training steps as one graph replay (the buffer parities in sequence)."""
        assert steps >= 2 and steps % 2 == 0
        p = 0 if self.cur is self.bufs[0] else 1
        self._graphs_current()
        if (p, steps) not in self._sg2:
            self._sg2[(p, steps)] = self._capture_step(p, steps=steps)
        self._advance_mirror(0)
        with trace.range("step_graph_pair"):
            self._sg2[(p, steps)][0].replay()
        self._advance_mirror(steps)

    def step(self, update=True, time_env=False):
        self._pos_dirty = True
        c, n = self.cur, self.nxt
        for f in self.pre_step_hooks:
            f(self)
        with trace.range("act"):
            act = self.model.act(c.own, c.radar, self.episode, noisy=True)
        if time_env:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        with trace.range("env_step"):
            self.env.step(act, out=n)
        if time_env:
            ev1.record()
            self.env_events.append((ev0, ev1))
        for f in self.post_step_hooks:
            f(self, act, c, n)
        with trace.range("replay_push"):
            self.replay.push_batch(c.own, c.radar, act, n.reward, n.done, n.own, n.radar)
        self.cur, self.nxt = n, c
        run_update = update and len(self.replay) > self.B
        with side_stream(self, run_update, UAM_OVERLAP_RESET), trace.range("auto_reset"):
            self.env.auto_reset(n.env_done, out=n)
        if run_update:
            with trace.range("update"):
                self.model.update(self.B, use_graph=not NO_GRAPH)
        join_side(self)
