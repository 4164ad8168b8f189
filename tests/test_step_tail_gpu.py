"""The fused env step tail (aac_env_step_tail: step + replay push + zeroed rows + auto-reset in the
step launch) against the separate launches it replaces (aac_env_step, aac_replay_push_at, the row
zeroing, aac_env_auto_reset): bit-identical outputs, env state, episode counters, replay ring and
ring position over many steps with short episodes (most steps reset some envs), ragged last
workgroups and a ring that wraps.  The separate launches are themselves oracle-checked
(test_env_gpu, test_wgru_gpu, test_learner_gpu)."""
import numpy as np
import pytest
import torch

from tests.helpers import W_DEFAULT

pytestmark = pytest.mark.gpu


def _pair(E, N, occ, variant, radar, maps, ep_len):
    from multi_agent_aac_amd import world
    from multi_agent_aac_amd.env import BatchedEnv
    if maps > 1:
        occ = world.map_stack(range(2026, 2026 + maps))
        bank = world.MapBanks(occ, n_pairs=2048, seed=7, max_wp=W_DEFAULT)
    else:
        bank = world.ODBank(occ, n_pairs=4096, seed=5, max_wp=W_DEFAULT)
    envs = []
    for _ in range(2):
        env = BatchedEnv(E, N, occ, radar_mode=radar, max_wp=W_DEFAULT, variant=variant, episode_length=ep_len)
        env.set_od_bank(bank, seed=4321)
        envs.append(env)
    return envs


@pytest.mark.parametrize("variant,N,E,radar,maps,ep_len", [
    ("att", 5, 1001, "combined", 1, 6),        # config-3 shape, ragged last workgroup (epb 4)
    ("att", 3, 517, "drones", 2, 5),           # multi-map draw inside the tail
    ("wgru", 8, 763, None, 1, 7),              # config-4 shape: 11 fields, hidden rows zeroed
])
def test_step_tail_equals_separate_launches(native_lib, occ, variant, N, E, radar, maps, ep_len):
    from multi_agent_aac_amd.memory import DeviceReplay
    ea, eb = _pair(E, N, occ, variant, radar, maps, ep_len)
    H = 64 if variant == "wgru" else 0
    cap = int(2.5 * E)        # wraps on the third push
    ra = DeviceReplay(cap, N, ea.D0, hidden=H, seed=1)
    rb = DeviceReplay(cap, N, eb.D0, hidden=H, seed=1)
    bufs = [[e.alloc_buffers(), e.alloc_buffers()] for e in (ea, eb)]
    ea.auto_reset(None, out=bufs[0][0])
    eb.auto_reset(None, out=bufs[1][0])
    g = torch.Generator(device="cuda").manual_seed(3)
    hid = [torch.rand(E, N, H or 1, device="cuda", generator=g) for _ in range(2)]
    ha = [h.clone() for h in hid]
    hb = [h.clone() for h in hid]
    rng = np.random.default_rng(11)
    resets = 0
    for t in range(14):
        act = torch.from_numpy(rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)).cuda()
        k = t % 2
        ca, na = bufs[0][k], bufs[0][1 - k]
        cb, nb = bufs[1][k], bufs[1][1 - k]
        # separate launches (bench.py AAC_FUSED_TAIL=0 order)
        ea.step(act, out=na)
        extra = [ha[k], ha[1 - k]] if H else []
        ra.push_batch(ca.own, ca.radar, ca.nei, act, na.reward, na.done, na.own, na.radar, na.nei, *extra)
        if H:
            ha[1 - k].mul_((na.env_done == 0).to(torch.float32)[:, None, None])
        ea.auto_reset(na.env_done, out=na)
        # fused
        srcs = [cb.own, cb.radar, cb.nei, act, nb.reward, nb.done, nb.own, nb.radar, nb.nei]
        if H:
            srcs += [hb[k], hb[1 - k]]
        eb.step_tail(act, out=nb, replay=rb, srcs=srcs, zero_rows=hb[1 - k] if H else None)
        torch.cuda.synchronize()
        resets += int(na.env_done.sum())
        for f in ("own", "radar", "nei", "reward", "done", "mask", "env_done", "bbc"):
            assert torch.equal(getattr(na, f), getattr(nb, f)), (t, f)
        sa, sb = ea.get_state(), eb.get_state()
        for key in sa:
            assert torch.equal(sa[key], sb[key]), (t, key)
        assert torch.equal(ra.meta, rb.meta), t
        assert (ra.pos, ra.size) == (rb.pos, rb.size)
        assert torch.equal(ra.ring, rb.ring), t
        if H:
            assert torch.equal(ha[1 - k], hb[1 - k]), t
    assert resets > E // 2, resets      # the tail's reset path ran on many envs
    assert ra.size == cap and ra.pos == (14 * E) % cap


def test_step_tail_without_push_or_reset(native_lib, occ):
    """Each part is optional: no ring and no reset is the plain step; reset without a push is step +
    auto-reset."""
    E, N = 300, 5
    ea, eb = _pair(E, N, occ, "att", "combined", 1, 4)
    for e in (ea, eb):
        e.auto_reset(None)
    rng = np.random.default_rng(2)
    for t in range(8):
        act = torch.from_numpy(rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)).cuda()
        ea.step(act)
        if t % 2:
            ea.auto_reset(ea.bufs.env_done)
        eb.step_tail(act, auto_reset=bool(t % 2))
        torch.cuda.synchronize()
        for f in ("own", "radar", "nei", "reward", "mask", "env_done"):
            assert torch.equal(getattr(ea.bufs, f), getattr(eb.bufs, f)), (t, f)
        sa, sb = ea.get_state(), eb.get_state()
        assert all(torch.equal(sa[k], sb[k]) for k in sa), t


def test_step_tail_rejects_bad_fields(native_lib, occ):
    from multi_agent_aac_amd import _native
    from multi_agent_aac_amd.env import BatchedEnv
    import ctypes
    E, N = 16, 3
    env = BatchedEnv(E, N, occ, max_wp=W_DEFAULT)
    ring = torch.zeros(64, 10, device="cuda")
    meta = torch.zeros(2, dtype=torch.int64, device="cuda")
    src = torch.zeros(E, 4, device="cuda")
    t = _native.StepTail()
    t.ring, t.row_width, t.capacity, t.pos, t.size, t.meta = ring.data_ptr(), 10, 64, 0, 0, meta.data_ptr()
    t.n_fields = 2
    t.srcs = (ctypes.c_void_p * 2)(src.data_ptr(), src.data_ptr())
    t.widths = (ctypes.c_int32 * 2)(8, 4)          # 12 > row_width
    act = torch.zeros(E, N, 2, device="cuda")
    o = env.bufs.c_struct()
    rc = _native.lib().aac_env_step_tail(env._h, ctypes.c_void_p(act.data_ptr()), ctypes.byref(o), ctypes.byref(t),
                                         None)
    assert rc != 0 and b"row_width" in _native.lib().aac_last_error()
    t.widths = (ctypes.c_int32 * 2)(4, 6)            # (a row stride past the fields' sum: padding, allowed)
    t.capacity = 8                                  # < E
    rc = _native.lib().aac_env_step_tail(env._h, ctypes.c_void_p(act.data_ptr()), ctypes.byref(o), ctypes.byref(t),
                                         None)
    assert rc != 0 and b"capacity" in _native.lib().aac_last_error()
    t.capacity = 64
    t.ring = None
    t.auto_reset = 1                                # no OD bank installed
    rc = _native.lib().aac_env_step_tail(env._h, ctypes.c_void_p(act.data_ptr()), ctypes.byref(o), ctypes.byref(t),
                                         None)
    assert rc != 0 and b"OD bank" in _native.lib().aac_last_error()


@pytest.mark.parametrize("E,N,B,mem,steps,model", [(256, 5, 64, 2000, 7, "att"), (4096, 5, 1024, 20000, 5, "att"),
                                                   (512, 8, 128, 3000, 7, "gru"), (4096, 8, 512, 20000, 5, "gru")])
def test_whole_step_graph_equals_eager(native_lib, monkeypatch, E, N, B, mem, steps, model):
    """trainer.Trainer.step_graph (act + fused env tail + update_myown replayed from one captured HIP
    graph per buffer parity, the ring position in device words) against the same steps launched
    eagerly: bit-identical networks, optimiser state, replay ring and env state.  The second case is
    config 3 (4096 envs x 5 agents, B = 1024); the GRU step (config 4: 4096 x 8, B = 512) carries the
    hidden-state pair through the replays.  An eager step between graph replays re-seeds the device
    ring-position word.  Then two and four steps per replay (step_graph_pair, the parities
    in sequence in one graph: the bench's timed forms) from either starting parity."""
    from multi_agent_aac_amd import trainer
    monkeypatch.setattr(trainer, "STEP_GRAPH", True)
    tr = [trainer.Trainer(E, N, B, mem, "combined", seed=0, model=model) for _ in range(2)]
    for t in tr:
        while len(t.replay) <= 3 * B:
            t.step(update=False)
        for _ in range(2):
            t.step(update=True)
    assert tr[1].graph_ok()
    for k in range(steps):                  # odd: both parities, and the host mirror across the wrap
        tr[0].step(update=True)
        if k == steps // 2:
            tr[1].step(update=True)         # eager step between replays: pos_dev re-seeded
        else:
            tr[1].step_graph()
    # two steps per replay (the bench's form), from either parity, after the single-step replays
    for _ in range(2):
        tr[0].step(update=True)
        tr[0].step(update=True)
        tr[1].step_graph_pair()
    tr[0].step(update=True)
    tr[1].step_graph()
    for _ in range(2):
        tr[0].step(update=True)
        tr[0].step(update=True)
        tr[1].step_graph_pair()
    # four steps per replay (the bench's form when the step count allows it)
    for _ in range(4):
        tr[0].step(update=True)
    tr[1].step_graph_pair(4)
    torch.cuda.synchronize()
    a, b = tr[0], tr[1]
    for x, y in ((a.model.fa.data, b.model.fa.data), (a.model.fc.data, b.model.fc.data),
                 (a.model.fa_t.data, b.model.fa_t.data), (a.model.fc_t.data, b.model.fc_t.data),
                 (a.replay.ring, b.replay.ring), (a.replay.meta, b.replay.meta), (a.replay.counter, b.replay.counter),
                 (a.model.noise_counter, b.model.noise_counter), (a.episode, b.episode)):
        assert torch.equal(x, y)
    assert (a.replay.pos, a.replay.size) == (b.replay.pos, b.replay.size)
    sa, sb = a.env.get_state(), b.env.get_state()
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    for f in ("own", "radar", "nei", "reward", "env_done"):
        assert torch.equal(getattr(a.cur, f), getattr(b.cur, f)), f
    if model == "gru":
        assert torch.equal(a.h, b.h)
