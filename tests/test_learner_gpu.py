"""GPU tests of the learner kernels (attention, replay, Adam, Polyak, noise) and of the full
device update_myown against the torch-CPU restatement (oracle/learner_ref.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import learner_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_attention(q, k, v, nei):
    mask = nei.mean(axis=2, keepdim=True).bool()
    score = torch.bmm(k, q.unsqueeze(2))
    sm = score.clone()
    sm[~mask] = float("-inf")
    alpha = F.softmax(sm / np.sqrt(64), dim=1)
    am = alpha.clone()
    am[~mask] = 0
    return torch.sum(v * am, axis=1)


@pytest.mark.parametrize("K", [1, 2, 4, 7, 15])
def test_attention_fwd_bwd(native_lib, K):
    from multi_agent_aac_amd import ops
    torch.manual_seed(K)
    R = 1000
    q = torch.randn(R, 64, dtype=torch.float64)
    kv = torch.randn(R, K, 128, dtype=torch.float64)
    nei = torch.randn(R, K, 6, dtype=torch.float64)
    nei[torch.rand(R, K) < 0.3] = 0.0
    nei[:5] = 0.0                                     # all-masked rows
    dout = torch.randn(R, 64, dtype=torch.float64)
    qr, kvr = q.clone().requires_grad_(), kv.clone().requires_grad_()
    ref = _ref_attention(qr, kvr[..., :64], kvr[..., 64:], nei)
    ref.backward(dout)
    qg = q.float().to(DEV).requires_grad_()
    kvg = kv.float().to(DEV).requires_grad_()
    out = ops.masked_attention(qg, kvg, nei.float().to(DEV))
    out.backward(dout.float().to(DEV))
    assert torch.isfinite(out).all() and torch.isfinite(qg.grad).all() and torch.isfinite(kvg.grad).all()
    np.testing.assert_allclose(out.detach().cpu().double(), ref.detach(), atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(qg.grad.cpu().double(), qr.grad, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(kvg.grad.cpu().double(), kvr.grad, atol=2e-5, rtol=1e-5)
    assert out[:5].abs().max() == 0 and qg.grad[:5].abs().max() == 0


def test_replay_push_gather_sample(native_lib):
    from multi_agent_aac_amd.memory import DeviceReplay
    N, D0, E, cap = 5, 22, 300, 1000
    rep = DeviceReplay(cap, N, D0, device=DEV, seed=3)
    host = []
    for p in range(5):                      # wraps around the ring (1500 > 1000)
        tr = learner_ref.random_transitions(E, N, p)
        rep.push_batch(*[tr[k].to(DEV).contiguous() for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done",
                                                               "n_own", "n_radar", "n_nei")])
        host.append(tr)
    assert len(rep) == cap and int(rep.meta[0]) == 1500 % cap and int(rep.meta[1]) == cap
    # ring row r holds transition (r - (1500 % cap)) mod cap of the last 1000 pushed
    allh = {k: torch.cat([h[k] for h in host])[-cap:] for k in host[0]}
    start = 1500 % cap
    idx = torch.arange(0, cap, 7, dtype=torch.int32)
    b = rep.sample_batch(len(idx), idx.to(DEV))
    src = (idx.long() - start) % cap
    for k, v in b.items():
        assert torch.equal(v.cpu(), allh[k][src].to(torch.float32)), k
    # sampler: distinct, in range, deterministic in (seed, counter), ~uniform
    counts = np.zeros(cap)
    c0 = int(rep.counter)
    for t in range(200):
        b = rep.sample_batch(512)
        ids = rep.batch_buffers(512)[0].cpu().numpy()
        assert len(np.unique(ids)) == 512 and ids.min() >= 0 and ids.max() < cap
        counts[ids] += 1
    assert int(rep.counter) == c0 + 200
    expected = 200 * 512 / cap
    chi2 = ((counts - expected) ** 2 / expected).sum()
    assert chi2 < cap + 6 * np.sqrt(2 * cap), chi2
    rep.counter.fill_(c0)
    rep.sample_batch(512)
    first = rep.batch_buffers(512)[0].clone()
    rep.counter.fill_(c0)
    rep.sample_batch(512)
    assert torch.equal(first, rep.batch_buffers(512)[0])


def _mix64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _draw_rounds(seed, ctr, block, B, size):
    """The redraw sampler of aac_replay_sample (size >= 2B) restated: B draws of hash(seed, epoch,
    workgroup, index, attempt) mod size; every round the least index holding a value keeps it and
    the others draw again with the next attempt, until the B values are distinct."""
    idx = np.arange(B, dtype=np.uint64)
    att = np.zeros(B, dtype=np.uint64)
    base = _mix64(_mix64(np.uint64(seed)) ^ np.uint64(ctr))

    def draw(i, a):
        key = (np.uint64(block) << np.uint64(44)) | (i << np.uint64(20)) | a
        return (_mix64(base ^ key) % np.uint64(size)).astype(np.int64)

    val = draw(idx, att)
    for _ in range(64):
        order = np.lexsort((np.arange(B), val))          # by value, then index
        first = np.ones(B, dtype=bool)
        first[1:] = val[order][1:] != val[order][:-1]
        lose = np.zeros(B, dtype=bool)
        lose[order[~first]] = True
        if not lose.any():
            break
        att[lose] += np.uint64(1)
        val[lose] = draw(idx[lose], att[lose])
    return val


@pytest.mark.parametrize("B,size,nb", [(1024, 2048, 1), (1024, 3000, 1), (1024, 200000, 2), (512, 1000000, 1),
                                       (4096, 8192, 1), (100, 250, 3)])
def test_sampler_rows_match_restatement(native_lib, B, size, nb):
    """aac_replay_sample's rows against the numpy restatement of its draw, bit for bit, over several
    epochs (the counter advancing once per launch) and batches (one workgroup each); ring sizes from
    2B (many redraw rounds) up."""
    from multi_agent_aac_amd import ops
    meta = torch.tensor([0, size], dtype=torch.int64, device=DEV)
    counter = torch.zeros(1, dtype=torch.int64, device=DEV)
    idx = torch.zeros(nb * B, dtype=torch.int32, device=DEV)
    with np.errstate(over="ignore"):
        for ctr in range(3):
            ops.replay_sample(meta, B, 12345, counter, idx)
            got = idx.cpu().numpy().reshape(nb, B)
            assert int(counter.item()) == ctr + 1
            for blk in range(nb):
                want = _draw_rounds(12345, ctr, blk, B, size)
                assert np.array_equal(got[blk], want), (ctr, blk)
                assert len(np.unique(got[blk])) == B


@pytest.mark.parametrize("extra", [0, 1, 7, 1023, 1024])
def test_sampler_distinct_on_small_ring(native_lib, extra):
    """size = B + extra rows (the first updates after the len(memory) > B guard): every batch holds
    B distinct in-range rows (size < 2B takes the exact partial Fisher-Yates path; 1024 = 2B the
    redraw path), and each row is drawn about equally often."""
    from multi_agent_aac_amd.memory import DeviceReplay
    N, D0, B = 3, 14, 1024
    rep = DeviceReplay(4096, N, D0, device=DEV, seed=5)
    tr = learner_ref.random_transitions(B + extra, N, 1)
    rep.push_batch(*[tr[k].to(DEV).contiguous() for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done",
                                                           "n_own", "n_radar", "n_nei")])
    size = B + extra
    counts = np.zeros(size)
    for _ in range(40):
        rep.sample_batch(B)
        ids = rep.batch_buffers(B)[0].cpu().numpy()
        assert len(np.unique(ids)) == B and ids.min() >= 0 and ids.max() < size
        counts[ids] += 1
    if extra >= 7:
        expected = 40 * B / size
        chi2 = ((counts - expected) ** 2 / expected).sum()
        assert chi2 < size + 6 * np.sqrt(2 * size), chi2


def test_adam_polyak_flat(native_lib):
    from multi_agent_aac_amd import ops
    torch.manual_seed(0)
    n = 100003
    p = torch.randn(n)
    ref = p.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=1e-3)
    pd = p.to(DEV)
    m, v = torch.zeros_like(pd), torch.zeros_like(pd)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    for t in range(5):
        g = torch.randn(n)
        ref.grad = g.clone()
        opt.step()
        step.add_(1)
        ops.adam_flat(pd, g.to(DEV), m, v, step, 1e-3)
    np.testing.assert_allclose(pd.cpu(), ref.detach(), atol=1e-6, rtol=1e-6)
    tgt, src = torch.randn(n), torch.randn(n)
    want = (1 - 0.01) * tgt + 0.01 * src
    td = tgt.to(DEV)
    ops.polyak_flat(td, src.to(DEV), 0.01)
    np.testing.assert_allclose(td.cpu(), want, atol=1e-7, rtol=1e-6)
    # the counter-advancing form: same soft update, step += 5 in the same launch
    td2 = tgt.to(DEV)
    ops.polyak_flat(td2, src.to(DEV), 0.01, step, 5)
    assert torch.equal(td2, td) and int(step.item()) == 10
    # both networks in one launch: bit-equal to two single-network launches, both counters advanced
    t1, s1, t2, s2 = (torch.randn(k, device=DEV) for k in (n, n, 3 * n + 7, 3 * n + 7))
    w1, w2 = t1.clone(), t2.clone()
    st1, st2 = torch.zeros(1, dtype=torch.int32, device=DEV), torch.full((1,), 3, dtype=torch.int32, device=DEV)
    ops.polyak_flat(w1, s1, 0.01)
    ops.polyak_flat(w2, s2, 0.01)
    ops.polyak_flat2(t1, s1, st1, t2, s2, st2, 0.01, 5)
    assert torch.equal(t1, w1) and torch.equal(t2, w2) and int(st1.item()) == 5 and int(st2.item()) == 8


def test_noise_clamp_schedule(native_lib):
    from multi_agent_aac_amd import ops
    E, N = 20000, 5
    act = torch.zeros(E, N, 2, device=DEV)
    ep = torch.full((E,), 4001, dtype=torch.int32, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    noise = torch.empty(E, N, 2, device=DEV)
    ops.noise_clamp(act, ep, 8000, 1.0, 7, ctr, noise)
    var = 1 + (-1 / 7999) * 4000
    z = noise.cpu().double() / var
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1) < 0.02
    assert torch.equal(act.cpu(), noise.cpu().clamp(-1, 1))
    assert int(ctr) == 1
    ep.fill_(8001)
    act.zero_()
    ops.noise_clamp(act, ep, 8000, 1.0, 7, ctr, noise)
    assert act.abs().max() == 0


def test_noise_rows_match_restatement(native_lib):
    """aac_noise_clamp's per-row noise (choose_action's N(0, var^2), ATT/maddpg:476-500) against the
    numpy restatement of aacn::row_noise: the Box-Muller pair of hash(seed, epoch, row) in float64,
    var from each env's episode on the linear schedule, rounded to float32; every row of 3 launches
    with ragged episodes (both sides of eps_end), 1 float32 ulp."""
    from multi_agent_aac_amd import ops
    E, N, eps_end, seed = 3001, 5, 8000, 99
    g = torch.Generator(device=DEV).manual_seed(4)
    ep = torch.randint(1, 9000, (E,), dtype=torch.int32, device=DEV, generator=g)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    noise = torch.empty(E, N, 2, device=DEV)
    rows = np.arange(E * N, dtype=np.uint64)
    epn = ep.cpu().numpy()[(rows // N).astype(np.int64)].astype(np.float64)
    ns, ne = float(np.float32(1.0)), float(np.float32(0.05))
    var = np.where(epn <= eps_end, ns + (ne - ns) / (eps_end - 1) * (epn - 1), ne)
    with np.errstate(over="ignore"):
        for k in range(3):
            act = torch.rand(E, N, 2, device=DEV, generator=g) * 2 - 1
            a0 = act.cpu().numpy().reshape(-1, 2)
            ops.noise_clamp(act, ep, eps_end, 1.0, seed, ctr, noise, noise_end=0.05)
            assert int(ctr.item()) == k + 1
            h1 = _mix64(_mix64(_mix64(np.uint64(seed)) ^ np.uint64(k)) ^ (np.uint64(2) * rows))
            h2 = _mix64(h1 ^ np.uint64(0xD1B54A32D192ED03))
            u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
            u2 = (h2 >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
            rr = np.sqrt(-2.0 * np.log(u1))
            want = np.stack([rr * np.cos(6.283185307179586 * u2) * var,
                             rr * np.sin(6.283185307179586 * u2) * var], 1).astype(np.float32)
            got = noise.cpu().numpy().reshape(-1, 2)
            np.testing.assert_array_max_ulp(got, want, maxulp=1)
            np.testing.assert_array_equal(act.cpu().numpy().reshape(-1, 2), np.clip(a0 + got, -1, 1))


@pytest.mark.parametrize("N,B", [(3, 64), (5, 256)])
def test_update_matches_cpu_restatement(native_lib, N, B):
    from multi_agent_aac_amd.maddpg import MADDPG
    assert learner_ref.check_one_update(MADDPG, device=DEV, N=N, B=B, E=128, tol=1e-5, iters=2)


def test_update_launch_forms_match_cpu_restatement(native_lib, monkeypatch):
    """The non-default launch form of the fused update (AAC_DAOB=0: the critic data gradient and actor
    output backward as two launches) against the same restatement."""
    from multi_agent_aac_amd import fused
    from multi_agent_aac_amd.maddpg import MADDPG
    monkeypatch.setattr(fused.FusedUpdate, "DAOB", False)
    assert learner_ref.check_one_update(MADDPG, device=DEV, N=5, B=256, E=128, tol=1e-5, iters=2)


@pytest.mark.parametrize("fused", [True, False])
def test_update_every_and_critic_records(native_lib, fused):
    """UPDATE_EVERY = 2 (ATT/maddpg:436-438: the soft update only when i_episode % 2 == 0; the Adam
    steps still count) and the 8-field single_eps_critic_cal_record entries (ATT/maddpg:372-379)
    against the restatement, for the fused and the autograd learner."""
    from multi_agent_aac_amd.maddpg import MADDPG

    def cls(*a, **k):
        return MADDPG(*a, fused=fused, **k)
    assert learner_ref.check_one_update(cls, device=DEV, N=3, B=64, E=128, tol=1e-5, iters=3, update_every=2,
                                        check_records=True)


def test_update_myown_reference_api_update_every(native_lib):
    """The reference surface: update_myown(i_episode, total, UPDATE_EVERY, record) keeps the targets
    on odd episodes with UPDATE_EVERY = 2 and appends N 8-field records per call."""
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B = 3, 32
    m = MADDPG([14, 18, 6], [14, 18, 6], 2, n_agents=N, device=DEV, seed=4, batch_size=B, memory_length=256)
    tr = learner_ref.random_transitions(64, N, 1)
    for e in range(64):
        st = [tr["s_own"][e].numpy(), tr["s_radar"][e].numpy(), [list(x.numpy()) for x in tr["s_nei"][e]]]
        nx = [tr["n_own"][e].numpy(), tr["n_radar"][e].numpy(), [list(x.numpy()) for x in tr["n_nei"][e]]]
        m.memory.push(st, tr["act"][e].numpy(), nx, tr["rew"][e].numpy(), tr["done"][e].numpy())
    t0 = (m.fa_t.data.clone(), m.fc_t.data.clone())
    rec = []
    c, a, rec = m.update_myown(1, 1, 2, rec)
    assert len(c) == N and len(rec) == N and all(len(r) == 8 for r in rec)
    assert rec[0][1].shape == (B, N) and rec[0][2].shape == (B, 1) and rec[0][0].shape == (B,)
    assert torch.equal(m.fa_t.data, t0[0]) and torch.equal(m.fc_t.data, t0[1])       # odd episode: no soft update
    c, a, rec = m.update_myown(2, 2, 2, rec)
    assert len(rec) == 2 * N and not torch.equal(m.fa_t.data, t0[0])
    assert int(m.actor_optimizer.step_t) == 2 * N


def test_graph_replay_equals_eager(native_lib):
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B, E = 5, 128, 256
    ms = []
    for _ in range(2):
        m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=N, device=DEV, seed=1, batch_size=B)
        rep = m.attach_replay(4 * E, seed=9)
        for p in range(3):
            tr = learner_ref.random_transitions(E, N, p)
            rep.push_batch(*[tr[k].to(DEV).contiguous() for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done",
                                                                   "n_own", "n_radar", "n_nei")])
        ms.append(m)
    for _ in range(3):
        ms[0].update(B, use_graph=True)
        ms[1].update(B, use_graph=False)
    torch.cuda.synchronize()
    for a, b in ((ms[0].fa.data, ms[1].fa.data), (ms[0].fc.data, ms[1].fc.data), (ms[0].fc_t.data, ms[1].fc_t.data)):
        np.testing.assert_allclose(a.cpu(), b.cpu(), atol=1e-6, rtol=1e-5)


def test_actor_pth_roundtrip(native_lib, tmp_path):
    from multi_agent_aac_amd.maddpg import MADDPG
    m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=5, device=DEV, seed=2)
    m.save_model(7, str(tmp_path))
    sd = torch.load(tmp_path / "episode_7_actor_net.pth", weights_only=True)
    ref = learner_ref.RefActor([22, 18, 6], 2)
    ref.load_state_dict(sd)                      # reference key names and shapes
    own, grid = torch.randn(40, 22), torch.rand(40, 18) * 15
    nei = torch.randn(40, 4, 6)
    want = ref([own, grid, nei])
    got = m.actors([own.to(DEV), grid.to(DEV), nei.to(DEV)]).cpu()
    np.testing.assert_allclose(got.detach(), want.detach(), atol=1e-5)
    m2 = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=5, device=DEV, seed=3)
    m2.load_model([str(tmp_path / "episode_7_actor_net.pth")])
    assert torch.equal(m2.fa.data, m.fa.data)


def test_transfer_learning_freezes_actor(native_lib):
    """ATT/maddpg:411-416: with transfer_learning the actor is frozen up to episode 10000 (critic
    steps only: the actor's parameters, Adam moments and step count stay; its target still moves
    by the soft update), and the reference's branch fails past it (NotImplementedError here).  The
    critic trajectory is the normal update's (the critic steps never read the online actor)."""
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B = 3, 32
    ms = []
    for _ in range(2):
        m = MADDPG([14, 18, 6], [14, 18, 6], 2, n_agents=N, device=DEV, seed=4, batch_size=B, memory_length=256)
        tr = learner_ref.random_transitions(64, N, 1)
        for e in range(64):
            st = [tr["s_own"][e].numpy(), tr["s_radar"][e].numpy(), [list(x.numpy()) for x in tr["s_nei"][e]]]
            nx = [tr["n_own"][e].numpy(), tr["n_radar"][e].numpy(), [list(x.numpy()) for x in tr["n_nei"][e]]]
            m.memory.push(st, tr["act"][e].numpy(), nx, tr["rew"][e].numpy(), tr["done"][e].numpy())
        ms.append(m)
    frozen, normal = ms
    fa0 = frozen.fa.data.clone()
    mom0 = [t.clone() for t in frozen.actor_optimizer.state()]
    fat0 = frozen.fa_t.data.clone()
    c, a, rec = frozen.update_myown(5, 5, 1, [], transfer_learning=True)
    normal.update_myown(5, 5, 1, [], transfer_learning=False)
    torch.cuda.synchronize()
    assert len(c) == N and len(a) == N and len(rec) == N and all(torch.isfinite(x) for x in a)
    assert torch.equal(frozen.fa.data, fa0)
    assert all(torch.equal(x, y) for x, y in zip(frozen.actor_optimizer.state(), mom0))
    assert not torch.equal(frozen.fa_t.data, fat0)                  # the soft update still runs
    np.testing.assert_allclose(frozen.fc.data.cpu(), normal.fc.data.cpu(), atol=1e-4, rtol=1e-5)
    assert not torch.equal(normal.fa.data, fa0)
    with pytest.raises(NotImplementedError):
        frozen.update_myown(10001, 10001, 1, [], transfer_learning=True)
