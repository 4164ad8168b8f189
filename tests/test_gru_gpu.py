"""GPU tests of the GRU-actor MADDPG (include/aac_gru.h, gru.py):
the GRU-cell row kernel in every mode against fp64 torch autograd of nn.GRUCell, and the device
choose_action / update_myown against the torch-CPU restatement of
MADDPG_ownENV_randomOD_Wgru_radar (oracle/gru_ref.py) on identical weights and batches."""
import numpy as np
import pytest
import torch

from oracle import gru_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
H = 64


@pytest.mark.parametrize("mode", ["fwd", "td", "critic", "actloss", "actbwd"])
def test_gru_cell_modes(native_lib, mode):
    from multi_agent_aac_amd import gru
    from multi_agent_aac_amd.fused import ptr
    N, M = 3, 37
    R = M * N
    O = 2 if mode in ("fwd", "actbwd") else 1
    act = gru.TANH if O == 2 else 0
    torch.manual_seed(5)
    cells = [torch.nn.GRUCell(128, H).double() for _ in range(N)]
    outs = [torch.nn.Linear(H, O).double() for _ in range(N)]
    x = torch.randn(M, N, 128, dtype=torch.float64)
    h = torch.tanh(torch.randn(M, N, H, dtype=torch.float64))
    # reference (fp64 autograd), per agent
    gi = torch.stack([x[:, i] @ cells[i].weight_ih.t() + cells[i].bias_ih for i in range(N)], 1).detach()
    gh = torch.stack([h[:, i] @ cells[i].weight_hh.t() + cells[i].bias_hh for i in range(N)], 1).detach()
    gi_r, gh_r = gi.clone().requires_grad_(True), gh.clone().requires_grad_(True)
    rr = torch.sigmoid(gi_r[..., :H] + gh_r[..., :H])
    zz = torch.sigmoid(gi_r[..., H:2 * H] + gh_r[..., H:2 * H])
    nn_ = torch.tanh(gi_r[..., 2 * H:] + rr * gh_r[..., 2 * H:])
    hp = (h - nn_) * zz + nn_
    W = torch.stack([o.weight.detach() for o in outs])          # (N, O, H)
    b = torch.stack([o.bias.detach() for o in outs])            # (N, O)
    y = torch.einsum("mnh,noh->mno", hp, W) + b
    if act:
        y = torch.tanh(y)
    tgt = torch.randn(M, N, dtype=torch.float64)
    rew, done = torch.randn(M, N, dtype=torch.float64), (torch.rand(M, N) < 0.3).double()
    da = torch.randn(M, N, O, dtype=torch.float64)
    if mode == "critic":
        loss = ((y[..., 0] - tgt) ** 2).mean(0).sum()           # per-agent MSE mean over M rows
    elif mode == "actloss":
        loss = (3 - y[..., 0].mean(0)).sum()
    elif mode == "actbwd":
        loss = (y * da).sum()
    if mode in ("critic", "actloss", "actbwd"):
        loss.backward()
    # device
    f = lambda t: t.float().to(DEV).contiguous()                # noqa: E731
    gi_d, gh_d, h_d = f(gi), f(gh), f(h)
    rew_d, done_d, tgt_d, da_d = f(rew), f(done), f(tgt), f(da)       # kept alive: kernels read them
    wpack = torch.zeros(N, 200, device=DEV)                     # agent stride 200 floats
    for i in range(N):
        wpack[i, :O * H] = f(W[i]).reshape(-1)
        wpack[i, O * H:O * H + O] = f(b[i])
    P = [{"W": ptr(wpack), "b": ptr(wpack, O * H)}]
    hout, yout = torch.zeros(M, N, H, device=DEV), torch.zeros(M, N, O, device=DEV)
    dgi, dgh = torch.zeros(M, N, 192, device=DEV), torch.zeros(M, N, 192, device=DEV)
    dq, q = torch.zeros(M, N, O, device=DEV), torch.zeros(M, N, device=DEV)
    kw = dict(hout=ptr(hout))
    if mode == "fwd":
        src = torch.randn(M, N, 10, device=DEV)
        pk = torch.zeros(M, N, 8, device=DEV)
        kw.update(y=ptr(yout), pack_src=ptr(src), ld_pack_src=10, npack=6, pack_dst=ptr(pk), ld_pack_dst=8)
        gru.gru_cell(P, "W", "b", 200, O, act, ptr(gi_d), ptr(gh_d), ptr(h_d), M, N, gru.FWD, **kw)()
        np.testing.assert_allclose(yout.cpu().double(), y.detach(), atol=2e-6)
        np.testing.assert_allclose(pk[..., :6].cpu(), src[..., :6].cpu())
        np.testing.assert_allclose(pk[..., 6:].cpu(), yout.cpu())
    elif mode == "td":
        yo = torch.zeros(M, N, device=DEV)
        gru.gru_cell(P, "W", "b", 200, O, act, ptr(gi_d), ptr(gh_d), ptr(h_d), M, N, gru.TD, rew=ptr(rew_d),
                     done=ptr(done_d), gamma=0.95, yout=ptr(yo), **kw)()
        want = rew + 0.95 * y[..., 0].detach() * (1 - done)
        np.testing.assert_allclose(yo.cpu().double(), want, atol=5e-6)
    else:
        m = {"critic": gru.CRITIC, "actloss": gru.ACTLOSS, "actbwd": gru.ACTBWD}[mode]
        extra = dict(target=ptr(tgt_d), y=ptr(q)) if mode == "critic" else \
            (dict(y=ptr(q)) if mode == "actloss" else dict(da=ptr(da_d), ldda=O))
        gru.gru_cell(P, "W", "b", 200, O, act, ptr(gi_d), ptr(gh_d), ptr(h_d), M, N, m, inv_m=1.0 / M, dq=ptr(dq),
                     dgi=ptr(dgi), dgh=ptr(dgh), **kw, **extra)()
        np.testing.assert_allclose(dgi.cpu().double(), gi_r.grad, atol=2e-6, rtol=1e-4)
        np.testing.assert_allclose(dgh.cpu().double(), gh_r.grad, atol=2e-6, rtol=1e-4)
        if mode == "critic":
            np.testing.assert_allclose(q.cpu().double(), y[..., 0].detach(), atol=2e-6)
    np.testing.assert_allclose(hout.cpu().double(), hp.detach(), atol=2e-6)


def _model(N, B, E, seed=0, d_own=6, own_width=None):
    from multi_agent_aac_amd.gru import MADDPG
    m = MADDPG([d_own, 18, 6], [d_own, 18, 6], 2, 64, 10, n_agents=N, device=DEV, seed=seed, batch_size=B,
               own_width=own_width)
    rep = m.attach_replay(4 * E, seed=seed + 3)
    return m, rep


def _ref_nets(m):
    N, d = m.n_agents, m.d_own
    actors = [gru_ref.RefGRUActor([d, 18, 6], 2) for _ in range(N)]
    critics = [gru_ref.RefGRUCritic([d, 18, 6], 2) for _ in range(N)]
    for i in range(N):
        actors[i].load_state_dict({k: v.cpu() for k, v in m.actors[i].state_dict().items()})
        critics[i].load_state_dict({k: v.cpu() for k, v in m.critics[i].state_dict().items()})
    import copy
    return actors, critics, copy.deepcopy(actors), copy.deepcopy(critics)


KEYS = ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei", "h_cur", "h_next")


@pytest.mark.parametrize("N,B,own_width,every", [(3, 64, None, 1), (8, 256, None, 1), (8, 256, 6, 1),
                                                  (3, 64, None, 2)])
def test_gru_update_matches_cpu_restatement(native_lib, N, B, own_width, every):
    """own_width 6: the replay rows of the WGRU env variant (config 4, 6-wide own observation).
    every 2: UPDATE_EVERY = 2, the soft update only on even i_episode (WGRU/maddpg:320)."""
    E = 96
    m, rep = _model(N, B, E, seed=N, own_width=own_width)
    assert m.D0 == (own_width or 6 + 4 * (N - 1))
    actors, critics, actors_t, critics_t = _ref_nets(m)
    host = {k: [] for k in KEYS}
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 10 * N + p, D0=own_width)
        rep.push_batch(*[tr[k].to(DEV).contiguous() for k in KEYS])
        for k in KEYS:
            host[k].append(tr[k])
    host = {k: torch.cat(v) for k, v in host.items()}
    gen = np.random.default_rng(N)
    # Adam's first steps are +-lr wherever |grad| << eps, so a last-bit difference in a near-zero
    # gradient moves a weight by up to 2 lr; with eps = 1e-3 on both sides the step is ~lr g / eps
    # there, and the weights after the updates compare the gradients themselves (tight tolerance)
    eps = 1e-3
    m.actor_optimizer.eps = m.critic_optimizer.eps = eps
    opts = ([torch.optim.Adam(a.parameters(), lr=1e-3, eps=eps) for a in actors],
            [torch.optim.Adam(c.parameters(), lr=1e-3, eps=eps) for c in critics])
    for it in range(3):
        idx = torch.from_numpy(gen.choice(len(rep), size=B, replace=False).astype(np.int32))
        soft = (it + 1) % every == 0
        stats = m.update(B, use_graph=False, idx=idx.to(DEV), soft_update=soft)
        b = {k: v[idx.long()].clone() for k, v in host.items()}
        b["done"] = b["done"].float()
        rstats, opts = gru_ref.ref_gru_update(actors, critics, actors_t, critics_t, b, m.d_own, opts=opts, soft=soft)
        for ag, ((lq, la, q, tg), (rlq, rla, rq, rtg)) in enumerate(zip(stats, rstats)):
            dt, dqv = float((tg.cpu() - rtg).abs().max()), float((q.cpu() - rq).abs().max())
            assert dt < 2e-5 * max(1.0, float(rtg.abs().max())), ("target", it, ag, dt)
            assert dqv < 2e-5 * max(1.0, float(rq.abs().max())), ("q", it, ag, dqv)
            assert abs(float(lq) - rlq) <= 1e-4 * max(1.0, abs(rlq)), ("loss_q", it, ag, float(lq), rlq)
            assert abs(float(la) - rla) <= 1e-4 * max(1.0, abs(rla)), ("loss_a", it, ag, float(la), rla)
    for i in range(N):
        for mine, ref in ((m.actors[i], actors[i]), (m.critics[i], critics[i]),
                          (m.actors_target[i], actors_t[i]), (m.critics_target[i], critics_t[i])):
            for (k, v), (_, rv) in zip(mine.state_dict().items(), ref.state_dict().items()):
                d = float((v.cpu() - rv).abs().max())
                assert d < 2e-5, (i, k, d)
    assert int(m.actor_optimizer.step_t) == int(m.critic_optimizer.step_t) == 3      # one Adam step per update


def test_gru_graph_equals_eager(native_lib):
    N, B, E = 4, 128, 64
    ma, repa = _model(N, B, E, seed=1)
    mb, repb = _model(N, B, E, seed=1)
    for p in range(3):
        tr = gru_ref.random_gru_transitions(E, N, 100 + p)
        for rep in (repa, repb):
            rep.push_batch(*[tr[k].to(DEV).contiguous() for k in KEYS])
    for _ in range(3):
        ma.update(B, use_graph=True, want_stats=False)
        mb.update(B, use_graph=False, want_stats=False)
    torch.cuda.synchronize()
    for x, y in ((ma.fa.data, mb.fa.data), (ma.fc.data, mb.fc.data), (ma.fa_t.data, mb.fa_t.data)):
        assert torch.equal(x, y)


def test_gru_act_matches_reference(native_lib):
    N, E = 8, 300
    m, _ = _model(N, 64, E, seed=2)
    actors, _, _, _ = _ref_nets(m)
    tr = gru_ref.random_gru_transitions(E, N, 7)
    a, hn = m.act(tr["s_own"].to(DEV), tr["s_radar"].to(DEV), tr["h_cur"].to(DEV), noisy=False)
    ra, rh = gru_ref.ref_gru_act(actors, tr["s_own"], tr["s_radar"], tr["h_cur"], m.d_own)
    np.testing.assert_allclose(a.cpu(), ra, atol=2e-5)
    np.testing.assert_allclose(hn.cpu(), rh, atol=2e-5)
    # module forward (device path) of one agent = the same rows
    a0, h0 = m.actors[3]([tr["s_own"][:, 3, :6].to(DEV), tr["s_radar"][:, 3].to(DEV)], tr["h_cur"][:, 3].to(DEV))
    np.testing.assert_allclose(a0.cpu(), ra[:, 3], atol=2e-5)
    np.testing.assert_allclose(h0.cpu(), rh[:, 3], atol=2e-5)
    # noise: clamp to [-1, 1], schedule end 0.03 after eps_end
    ep = torch.full((E,), 9000, dtype=torch.int32, device=DEV)
    noise = torch.zeros(E, N, 2, device=DEV)
    a2, _ = m.act(tr["s_own"].to(DEV), tr["s_radar"].to(DEV), tr["h_cur"].to(DEV), episode=ep, noise_out=noise)
    assert float(a2.abs().max()) <= 1.0
    z = noise.cpu().double() / 0.03
    assert abs(float(z.std()) - 1) < 0.1


@pytest.mark.parametrize("E,own_width", [(4096, 6), (301, 34), (17, 6)])
def test_gru_act_weights_stationary_matches_launch_path(native_lib, monkeypatch, E, own_width):
    """aac_gru_actor_fwd (the act path in one weights-stationary launch) against the encoder + gate
    GEMM launches + aac_gru_cell it replaces, and against the fp64 reference actor (config-4 shape
    E = 4096 x 8; ragged blocks; own rows wider than d_own)."""
    from multi_agent_aac_amd import gru
    N = 8
    m, _ = _model(N, 64, E, seed=5)
    actors, _, _, _ = _ref_nets(m)
    tr = gru_ref.random_gru_transitions(E, N, 9)
    own = torch.zeros(E, N, own_width)
    own[:, :, :6] = tr["s_own"][:, :, :6]
    own, radar, h = own.to(DEV), tr["s_radar"].to(DEV), tr["h_cur"].to(DEV)
    outs = {}
    for ws in (True, False):
        monkeypatch.setattr(gru, "ACT_WS", ws)
        m._acts.clear()
        a, hn = m.act(own, radar, h, noisy=False)
        outs[ws] = (a.clone(), hn.clone())
    torch.testing.assert_close(outs[True][0], outs[False][0], atol=2e-6, rtol=1e-5)
    torch.testing.assert_close(outs[True][1], outs[False][1], atol=2e-6, rtol=1e-5)
    ra, rh = gru_ref.ref_gru_act(actors, tr["s_own"], tr["s_radar"], tr["h_cur"], m.d_own)
    np.testing.assert_allclose(outs[True][0].cpu(), ra, atol=2e-5)
    np.testing.assert_allclose(outs[True][1].cpu(), rh, atol=2e-5)


def test_gru_act_fused_noise_matches_noise_launch(native_lib, monkeypatch):
    """The weights-stationary act launch with the exploration noise inside (noisy=True) against the
    launch path + aac_noise_clamp: the same noise bit for bit (per-row hash of the same counter epoch),
    the same clamped actions, and the counter advanced once per call either way."""
    from multi_agent_aac_amd import gru
    E, N = 1000, 8
    m, _ = _model(N, 64, E, seed=6)
    tr = gru_ref.random_gru_transitions(E, N, 4)
    own, radar, h = tr["s_own"].to(DEV), tr["s_radar"].to(DEV), tr["h_cur"].to(DEV)
    episode = torch.randint(1, 9000, (E,), dtype=torch.int32, device=DEV)
    outs = {}
    for ws in (True, False):
        monkeypatch.setattr(gru, "ACT_WS", ws)
        m._acts.clear()
        m.noise_counter.zero_()
        res = []
        for _ in range(2):
            nz = torch.empty(E, N, 2, device=DEV)
            a, _ = m.act(own, radar, h, episode=episode, noisy=True, noise_out=nz)
            res.append((a.clone(), nz))
        outs[ws] = (res, int(m.noise_counter.item()))
    assert outs[True][1] == outs[False][1] == 2
    for (a1, n1), (a0, n0) in zip(outs[True][0], outs[False][0]):
        assert torch.equal(n1, n0)
        torch.testing.assert_close(a1, a0, atol=2e-6, rtol=1e-5)
        assert float(a1.abs().max()) <= 1.0
    assert not torch.equal(outs[True][0][0][1], outs[True][0][1][1])      # a new epoch per call


def test_gru_act_plan_cache_is_lru(native_lib):
    """Act plans are keyed on the caller's buffers: fresh tensors every call evict only the oldest
    plan (at most 8 kept), and a buffer set in steady use keeps its plan (no rebuild)."""
    E, N = 64, 3
    m, _ = _model(N, 4, E, seed=2)
    own, radar, h = (torch.zeros(E, N, w, device=DEV) for w in (6, 18, H))
    m.act(own, radar, h, noisy=False)
    steady = next(iter(m._acts.values()))
    for _ in range(12):
        m.act(own.clone(), radar.clone(), h.clone(), noisy=False)
        m.act(own, radar, h, noisy=False)           # the steady set, used every step
    assert len(m._acts) <= 8
    assert any(p is steady for p in m._acts.values())


def test_gru_reset_hidden_and_reference_api(native_lib, tmp_path):
    from multi_agent_aac_amd import gru
    N = 3
    h = torch.ones(5, N, H, device=DEV)
    done = torch.tensor([0, 1, 0, 0, 1], dtype=torch.uint8, device=DEV)
    gru.reset_hidden(h, done)
    assert torch.equal(h.sum((1, 2)).cpu(), torch.tensor([192., 0., 192., 192., 0.]))
    m, _ = _model(N, 4, 8, seed=3)
    state = [[np.random.randn(6).astype(np.float32) for _ in range(N)],
             [np.random.rand(18).astype(np.float32) * 15 for _ in range(N)]]
    hid = [np.zeros(H) for _ in range(N)]
    acts, noise, cur, nxt = m.choose_action(state, 0, 1, 0, 8000, 1.0, hid, noisy=False)
    assert acts.shape == (N, 2) and cur.shape == (N, H) and nxt.shape == (N, H)
    for t in range(6):        # reference ma_main push path (two-portion states, hidden states)
        m.memory.push(state, acts, state, np.random.randn(N), np.zeros(N), None, cur, nxt)
    c, a = m.update_myown(1, 0, 1)
    assert len(c) == N and len(a) == N
    m.save_model(7, str(tmp_path))
    files = [str(tmp_path / f"episode_7_agent_{i}actor_net.pth") for i in range(N)]
    sd = torch.load(files[1], weights_only=True)
    assert set(sd) == set(gru_ref.RefGRUActor([6, 18, 6], 2).state_dict())
    m2, _ = _model(N, 4, 8, seed=9)
    m2.load_model(files)
    for i in range(N):
        for k, v in m.actors[i].state_dict().items():
            assert torch.equal(v, m2.actors[i].state_dict()[k])
