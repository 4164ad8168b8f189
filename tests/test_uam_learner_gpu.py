"""GPU tests of the UAM learner (multi_agent_aac_amd/uam_learner.py)
against the CPU float64 restatement oracle/uam_learner_ref.py: identical weights and sampled rows,
parameters after two update_myown calls within 1e-10; graph replay equal to eager; the batched
act / replay; the reference method surface."""
import copy

import numpy as np
import pytest
import torch

from oracle import uam_learner_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed=1, B=64):
    from multi_agent_aac_amd import uam_learner as L
    m = L.MADDPG([7, 20, 18, 6], [7, 20, 18, 6], 2, n_agents=5, device=DEV, seed=seed, batch_size=B,
                 memory_length=4096)
    rep = m.attach_replay(4096, seed=3)
    g = torch.Generator().manual_seed(seed)
    E, N = 64, 5
    for _ in range(4):
        rnd = lambda *s: torch.rand(*s, generator=g, dtype=torch.float64) * 2 - 1   # noqa: E731
        rep.push_batch(rnd(E, N, 7).to(DEV), rnd(E, N, 18).abs().mul(5).to(DEV), rnd(E, N, 2).to(DEV),
                       rnd(E, N).mul(50).to(DEV), (rnd(E, N) > 0.8).double().to(DEV), rnd(E, N, 7).to(DEV),
                       rnd(E, N, 18).abs().mul(5).to(DEV))
    return m, rep


def _ref_from(m):
    a, c = R.RefActor().double(), R.RefCritic().double()
    a.load_state_dict({k: v.cpu() for k, v in m.actors.state_dict().items()})
    c.load_state_dict({k: v.cpu() for k, v in m.critics.state_dict().items()})
    return a, c, copy.deepcopy(a), copy.deepcopy(c)


def test_update_matches_cpu_restatement(native_lib):
    from multi_agent_aac_amd import uam_learner as L
    m, rep = _model()
    a, c, at, ct = _ref_from(m)
    oa = torch.optim.Adam(a.parameters(), lr=1e-4)
    oc = torch.optim.Adam(c.parameters(), lr=1e-4)
    rng = np.random.default_rng(0)
    for it in range(2):
        idx = torch.as_tensor(rng.choice(len(rep), 64, replace=False), dtype=torch.int32, device=DEV)
        lq, la = m.update(64, idx=idx)
        rows = rep.ring[idx.long()].cpu()
        b = {k: rows[:, s:e] for k, (s, e) in L.SLICES.items()}
        b["rew"], b["done"] = b["rew"][:, 0], b["done"][:, 0]
        rq, ra = R.ref_update(a, c, at, ct, oa, oc, b)
        assert abs(float(lq) - rq) < 1e-10 and abs(float(la) - ra) < 1e-10
    for mine, ref in ((m.actors, a), (m.critics, c), (m.actors_target, at), (m.critics_target, ct)):
        for (k, p), (_, q) in zip(mine.state_dict().items(), ref.state_dict().items()):
            np.testing.assert_allclose(p.cpu().numpy(), q.numpy(), rtol=0, atol=1e-10, err_msg=k)


def test_graph_replay_equals_eager(native_lib):
    """The torch-autograd path: captured graph == eager, three updates."""
    m1, rep1 = _model(seed=4)
    m2, rep2 = _model(seed=4)
    m1.fused_learner = False
    for _ in range(3):
        m1.update(64, use_graph=True)
        m2.update(64, use_graph=False)
    torch.cuda.synchronize()
    for p, q in zip(list(m1.actors.parameters()) + list(m1.critics_target.parameters()),
                    list(m2.actors.parameters()) + list(m2.critics_target.parameters())):
        np.testing.assert_allclose(p.detach().cpu().numpy(), q.detach().cpu().numpy(), rtol=0, atol=1e-14)


def test_fused_update_matches_cpu_restatement(native_lib):
    """The fused float64 learner (FusedUamUpdate, include/aac_uam_learn.h) against the CPU
    restatement: two updates on the same sampled rows, losses and all four networks within 1e-10."""
    from multi_agent_aac_amd import uam_learner as L
    m, rep = _model(seed=6)
    a, c, at, ct = _ref_from(m)
    oa = torch.optim.Adam(a.parameters(), lr=1e-4)
    oc = torch.optim.Adam(c.parameters(), lr=1e-4)
    fu = m.fused(64, rep)
    rng = np.random.default_rng(1)
    for it in range(2):
        idx = torch.as_tensor(rng.choice(len(rep), 64, replace=False), dtype=torch.int32, device=DEV)
        lq, la = fu.run(idx)
        rows = rep.ring[idx.long()].cpu()
        b = {k: rows[:, s:e] for k, (s, e) in L.SLICES.items()}
        b["rew"], b["done"] = b["rew"][:, 0], b["done"][:, 0]
        rq, ra = R.ref_update(a, c, at, ct, oa, oc, b)
        assert abs(float(lq) - rq) < 1e-10 and abs(float(la) - ra) < 1e-10, (float(lq), rq, float(la), ra)
    for mine, ref in ((m.actors, a), (m.critics, c), (m.actors_target, at), (m.critics_target, ct)):
        for (k, p), (_, q) in zip(mine.state_dict().items(), ref.state_dict().items()):
            np.testing.assert_allclose(p.cpu().numpy(), q.numpy(), rtol=0, atol=1e-10, err_msg=k)


def test_fused_graph_equals_eager_and_torch_path(native_lib):
    """update() replays the fused learner's graph: bit-equal to its eager launches, and within
    1e-12 of the torch-autograd path on the same sampled rows (same replay sampler stream)."""
    m1, rep1 = _model(seed=5)
    m2, rep2 = _model(seed=5)
    m3, rep3 = _model(seed=5)
    m3.fused_learner = False
    f2 = m2.fused(64, rep2)
    for _ in range(3):
        m1.update(64, use_graph=True)
        f2.run()
        m3.update(64, use_graph=False)
    torch.cuda.synchronize()
    ps = lambda m: list(m.actors.parameters()) + list(m.critics.parameters()) + list(m.critics_target.parameters())  # noqa
    for p, q, t in zip(ps(m1), ps(m2), ps(m3)):
        assert torch.equal(p, q)
        np.testing.assert_allclose(p.detach().cpu().numpy(), t.detach().cpu().numpy(), rtol=0, atol=1e-12)


@pytest.mark.parametrize("case", range(6))
def test_gemm64_products(native_lib, case):
    """aac_gemm64_batch against float64 torch: transposes, ragged tiles, epilogues, the ones column
    and split-K partial copies, several products in one launch."""
    from multi_agent_aac_amd import fused
    from multi_agent_aac_amd import uam_learner as L
    g = torch.Generator(device=DEV).manual_seed(case)
    rnd = lambda *s: torch.randn(*s, dtype=torch.float64, device=DEV, generator=g)   # noqa: E731
    specs = [  # (M, N, K, ta, tb, act, mact, ones, ks)
        [(512, 64, 7, 0, 1, 1, 0, 0, 1), (512, 256, 128, 0, 1, 1, 0, 0, 1), (37, 19, 5, 0, 0, 2, 0, 0, 1)],
        [(256, 128, 512, 1, 0, 0, 0, 1, 8), (1, 256, 512, 1, 0, 0, 0, 1, 8)],
        [(512, 128, 256, 0, 0, 0, 1, 0, 1), (512, 2, 64, 0, 0, 0, 2, 0, 1)],
        [(64, 9, 512, 1, 0, 0, 0, 1, 8), (64, 18, 513, 1, 0, 0, 0, 1, 3)],
        [(17, 33, 65, 1, 1, 2, 1, 0, 1), (100, 3, 1, 0, 0, 1, 0, 0, 1)],
        [(512, 128, 2, 0, 0, 0, 1, 0, 1), (2, 128, 512, 1, 0, 0, 0, 1, 8)],
    ][case]
    probs, checks, keep = [], [], []
    for M, N, K, ta, tb, act, mact, ones, ks in specs:
        A = rnd(K, M) if ta else rnd(M, K)
        Bm = rnd(N, K) if tb else rnd(K, N)
        opA, opB = (A.t() if ta else A), (Bm.t() if tb else Bm)
        bias = rnd(N) if (act and ks == 1) else None
        mask = rnd(M, N) if mact else None
        stride = M * N + M
        C = torch.full((ks * stride,), 7.0, dtype=torch.float64, device=DEV)
        cx = C[M * N:] if ones else None
        probs.append(L.prob64(L.p64(A), L.p64(Bm), L.p64(C), M, N, K, M if ta else K, K if tb else N, N, ta=ta,
                              tb=tb, bias=L.p64(bias), act=act, mask=L.p64(mask), ldmask=N, mact=mact, ones=ones,
                              cextra=L.p64(cx), ksplit=ks, split_stride=stride if ks > 1 else 0))
        keep += [A, Bm, C, bias, mask]
        want = opA @ opB
        if bias is not None:
            want = want + bias
        want = torch.relu(want) if act == 1 else (torch.tanh(want) if act == 2 else want)
        if mact == 1:
            want = want * (mask > 0)
        elif mact == 2:
            want = want * (1 - mask * mask)
        checks.append((C, M, N, ks, stride, ones, want, opA.sum(1)))
    arr = (L.Gemm64Prob * len(probs))(*probs)
    L._ok(L._learn_lib().aac_gemm64_batch(arr, len(probs), fused._stream()), "gemm64")
    torch.cuda.synchronize()
    for C, M, N, ks, stride, ones, want, rowsum in checks:
        parts = C.view(ks, stride) if ks > 1 else C[:stride].view(1, stride)
        got = parts[:, :M * N].sum(0).view(M, N)
        torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)
        if ones:
            torch.testing.assert_close(parts[:, M * N:].sum(0), rowsum, rtol=1e-12, atol=1e-12)


def test_act_and_noise_schedule(native_lib):
    m, _ = _model()
    own = torch.rand(32, 5, 7, dtype=torch.float64, device=DEV)
    radar = torch.rand(32, 5, 18, dtype=torch.float64, device=DEV) * 5
    ep = torch.ones(32, dtype=torch.int32, device=DEV)
    a0 = m.act(own, radar, ep, noisy=False)
    ref = m.actors([own.view(-1, 7), radar.view(-1, 18)]).view(32, 5, 2)
    # aac_uam_actor (fp64 MFMA) vs the torch module: same float64 forward, summation order aside
    torch.testing.assert_close(a0, ref, rtol=0, atol=1e-13)
    assert a0.dtype == torch.float64
    ep[:] = 20000       # past eps_end = 10000: var = 0, no noise (UAM/maddpg:1399-1406)
    torch.testing.assert_close(m.act(own, radar, ep, noisy=True), torch.clamp(a0, -1, 1), rtol=0, atol=0)
    ep[:] = 1
    an = m.act(own, radar, ep, noisy=True)
    assert an.abs().max() <= 1 and not torch.equal(an, a0)
    # the launch advances the noise epoch itself (one per noisy call, arrivals field back at 0)
    assert int(m.noise_counter.item()) == 2
    assert not torch.equal(m.act(own, radar, ep, noisy=True), an)
    assert int(m.noise_counter.item()) == 3


def _mix64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def test_actor_noise_epoch_per_launch(native_lib):
    """The config-5 act launch (8192 envs x 16 aircraft: 256 workgroups) over several noisy calls:
    every row's noise is the Box-Muller pair of hash(seed, epoch, row) with the launch's epoch (one
    per call, whichever workgroup reads it), the counter advances by exactly one per launch with the
    arrival field back at 0 -- restated here in numpy for a sample of rows, 1e-12."""
    m, _ = _model()
    E, N = 8192, 16
    g = torch.Generator(device=DEV).manual_seed(5)
    own = torch.rand(E, N, 7, dtype=torch.float64, device=DEV, generator=g) * 2 - 1
    radar = torch.rand(E, N, 18, dtype=torch.float64, device=DEV, generator=g) * 5
    ep = torch.randint(1, 12000, (E,), dtype=torch.int32, device=DEV, generator=g)
    plain = m.act(own, radar, ep, noisy=False).view(-1, 2).cpu().numpy()
    rows = np.unique(np.concatenate([np.arange(0, E * N, 61), np.arange(E * N - 64, E * N)])).astype(np.uint64)
    epn = ep.cpu().numpy()[(rows // N).astype(np.int64)].astype(np.float64)
    var = np.where(epn <= 10000, 1.0 + (0.0 - 1.0) / 9999.0 * (epn - 1), 0.0)
    with np.errstate(over="ignore"):
        for k in range(4):
            out = m.act(own, radar, ep, noisy=True).view(-1, 2).cpu().numpy()
            assert int(m.noise_counter.item()) == k + 1
            h1 = _mix64(_mix64(_mix64(np.uint64(m.noise_seed)) ^ np.uint64(k)) ^ (np.uint64(2) * rows))
            h2 = _mix64(h1 ^ np.uint64(0xD1B54A32D192ED03))
            u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
            u2 = (h2 >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
            rr = np.sqrt(-2.0 * np.log(u1))
            want = np.stack([rr * np.cos(6.283185307179586 * u2) * var, rr * np.sin(6.283185307179586 * u2) * var], 1)
            want = np.clip(plain[rows.astype(np.int64)] + want, -1.0, 1.0)
            np.testing.assert_allclose(out[rows.astype(np.int64)], want, rtol=0, atol=1e-12)


@pytest.mark.parametrize("R", [1, 15, 16, 17, 1000, 131072])
def test_actor_kernel_rows(native_lib, R):
    """aac_uam_actor over ragged row counts (partial 16-row blocks, one row, the config-5 size)
    against the float64 torch module."""
    m, _ = _model()
    g = torch.Generator(device=DEV).manual_seed(R)
    own = torch.rand(R, 1, 7, dtype=torch.float64, device=DEV, generator=g) * 2 - 1
    radar = torch.rand(R, 1, 18, dtype=torch.float64, device=DEV, generator=g) * 5
    a = m.act(own, radar, None, noisy=False)
    ref = m.actors([own.view(-1, 7), radar.view(-1, 18)]).view(R, 1, 2)
    torch.testing.assert_close(a, ref, rtol=0, atol=1e-13)


def test_actor_tiles_bit_identical(native_lib):
    """aac_uam_actor with 1, 2 and 4 sixteen-row tiles per block (aac_uam_actor_set_tiles): the same
    per-row arithmetic, so identical outputs to the bit, with and without the exploration noise."""
    import ctypes
    from multi_agent_aac_amd import uam
    m, _ = _model()
    L = uam.lib()
    L.aac_uam_actor_set_tiles.argtypes = [ctypes.c_int32]
    R = 4099                       # ragged: partial 64-row blocks
    g = torch.Generator(device=DEV).manual_seed(9)
    own = torch.rand(R, 1, 7, dtype=torch.float64, device=DEV, generator=g) * 2 - 1
    radar = torch.rand(R, 1, 18, dtype=torch.float64, device=DEV, generator=g) * 5
    ep = torch.randint(1, 12000, (R,), dtype=torch.int32, device=DEV, generator=g)
    outs = []
    try:
        for nt in (1, 2, 4):
            assert L.aac_uam_actor_set_tiles(nt) == 0
            m.noise_counter.zero_()
            outs.append((m.act(own, radar, None, noisy=False), m.act(own, radar, ep, noisy=True)))
    finally:
        L.aac_uam_actor_set_tiles(4)
    for a, b in outs[1:]:
        assert torch.equal(a, outs[0][0]) and torch.equal(b, outs[0][1])
    assert L.aac_uam_actor_set_tiles(3) != 0


def test_reference_surface(native_lib, tmp_path):
    from multi_agent_aac_amd import uam_learner as L
    m = L.MADDPG([7, 20, 18, 6], [7, 20, 18, 6], 2, n_agents=3, device=DEV, seed=2, batch_size=8, memory_length=64)
    st = [[np.random.rand(7) for _ in range(3)], [np.random.rand(20) for _ in range(3)],
          [np.random.rand(18) for _ in range(3)]]
    act, noise, _, _ = m.choose_action(st, 1, 1, 1, 10000, 1, None)
    assert act.shape == (3, 2) and act.dtype == np.float64
    assert m.update_myown(1, 1, 1, []) == (None, None, [])
    for _ in range(4):
        for i in range(3):
            m.memory.push(st[0][i], st[1][i], st[2][i], act[i], st[0][i], st[1][i], st[2][i], 1.0, 0, None, None, None)
    assert len(m.memory) == 12
    cl, al, rec = m.update_myown(1, 1, 1, [])
    assert len(cl) == 1 and np.isfinite(float(cl[0]))
    assert len(m.memory.sample(8)) == 8
    m.save_model(3, str(tmp_path))
    m2 = L.MADDPG([7, 20, 18, 6], [7, 20, 18, 6], 2, n_agents=3, device=DEV, seed=9)
    m2.load_model([str(tmp_path / "episode_3_actor_net.pth")])
    for p, q in zip(m.actors.parameters(), m2.actors.parameters()):
        assert torch.equal(p, q)


@pytest.mark.parametrize("done_u8", [True, False])
def test_replay_push_kernel(native_lib, done_u8):
    """aac_uam_push (one launch, ring wrap-around in the kernel) writes the same rows as the
    torch.cat row assembly, bit for bit."""
    from multi_agent_aac_amd import uam_learner as L
    cap, M = 100, 40
    rep = L.UamReplay(cap, DEV, seed=1)
    want = torch.zeros(cap, L.ROW, dtype=torch.float64)
    g = torch.Generator(device=DEV).manual_seed(3)
    pos = 0
    for it in range(4):           # 160 rows through a 100-row ring: two wraps
        f = lambda *s: torch.randn(*s, dtype=torch.float64, device=DEV, generator=g)   # noqa: E731
        own, radar, act, rew, nown, nradar = f(8, 5, 7), f(8, 5, 18), f(8, 5, 2), f(8, 5), f(8, 5, 7), f(8, 5, 18)
        done = (torch.rand(8, 5, device=DEV, generator=g) > 0.5)
        done = done.to(torch.uint8) if done_u8 else done.double()
        rep.push_batch(own, radar, act, rew, done, nown, nradar)
        rows = torch.cat([own.reshape(-1, 7), radar.reshape(-1, 18), act.reshape(-1, 2), rew.reshape(-1, 1),
                          done.reshape(-1, 1).double(), nown.reshape(-1, 7), nradar.reshape(-1, 18)], 1).cpu()
        for i in range(M):
            want[(pos + i) % cap] = rows[i]
        pos = (pos + M) % cap
    assert rep.pos == pos and len(rep) == cap
    assert torch.equal(rep.ring.cpu(), want)
    assert rep.meta.tolist() == [pos, cap]


def test_adam_state_shared_across_plans_and_torch_path(native_lib):
    """The fused plans of different B and the torch-autograd path continue from one optimiser state
    (MADDPG._flat_state): update(B=64) and update(B=128) (graph-replayed fused plans, indices from
    the device sampler) then a torch-path update, all against the CPU restatement with one pair of
    torch.optim.Adam (a rebuilt plan used to restart from the stale torch moments)."""
    from multi_agent_aac_amd import uam_learner as L
    m, rep = _model(seed=8)
    a, c, at, ct = _ref_from(m)
    oa = torch.optim.Adam(a.parameters(), lr=1e-4)
    oc = torch.optim.Adam(c.parameters(), lr=1e-4)

    def ref_step(idx):
        rows = rep.ring[idx.long()].cpu()
        b = {k: rows[:, s:e] for k, (s, e) in L.SLICES.items()}
        b["rew"], b["done"] = b["rew"][:, 0], b["done"][:, 0]
        return R.ref_update(a, c, at, ct, oa, oc, b)

    for B in (64, 128, 64):
        lq, la = m.update(B, use_graph=True)
        idx = m.fused(B, rep).idx.clone()
        rq, ra = ref_step(idx)
        assert abs(float(lq) - rq) < 1e-10 * max(1, abs(rq)) and abs(float(la) - ra) < 1e-10 * max(1, abs(ra))
    idx = torch.as_tensor(np.random.default_rng(2).choice(len(rep), 96, replace=False), dtype=torch.int32,
                          device=DEV)
    lq, la = m.update(96, use_graph=False, idx=idx)           # torch-autograd path
    rq, ra = ref_step(idx)
    assert abs(float(lq) - rq) < 1e-10 * max(1, abs(rq)) and abs(float(la) - ra) < 1e-10 * max(1, abs(ra))
    lq, la = m.update(128, use_graph=True)                    # and back to a fused plan
    rq, ra = ref_step(m.fused(128, rep).idx.clone())
    assert abs(float(lq) - rq) < 1e-10 * max(1, abs(rq)) and abs(float(la) - ra) < 1e-10 * max(1, abs(ra))
    for mine, ref in ((m.actors, a), (m.critics, c), (m.actors_target, at), (m.critics_target, ct)):
        for (k, p), (_, q) in zip(mine.state_dict().items(), ref.state_dict().items()):
            np.testing.assert_allclose(p.cpu().numpy(), q.numpy(), rtol=0, atol=1e-10, err_msg=k)


def test_td_mse_head_equals_two_heads(native_lib):
    """aac_uam_td_mse_head (the TD target and the critic's mse head chained per row) equals the two
    aac_uam_head launches (mode 2, then mode 0) bit for bit."""
    from multi_agent_aac_amd import fused
    from multi_agent_aac_amd import uam_learner as L
    g = torch.Generator(device="cuda").manual_seed(4)
    B, ldr = 300, 5
    r = lambda *s: torch.rand(*s, device="cuda", dtype=torch.float64, generator=g) * 2 - 1   # noqa: E731
    ht, h = torch.relu(r(B, 256)), torch.relu(r(B, 256))
    wt, bt, w, b = r(256), r(1), r(256), r(1)
    rows = r(B, ldr)
    rows[:, 1] = (rows[:, 1] > 0.6).double()              # done flags
    rew, done = rows[:, 0:], rows[:, 1:]
    P = lambda t: t.data_ptr()                            # noqa: E731
    outs = [[torch.full((B,), 7.0, device="cuda", dtype=torch.float64) for _ in range(3)] +
            [torch.full((B, 256), 7.0, device="cuda", dtype=torch.float64)] for _ in range(2)]
    lib = L._learn_lib()
    y, dq, lq, dh = outs[0]
    L._ok(lib.aac_uam_head(P(ht), B, P(wt), P(bt), 2, P(y), P(rew), P(done), ldr, 0.95, None, None, None,
                           fused._stream()), "head2")
    L._ok(lib.aac_uam_head(P(h), B, P(w), P(b), 0, P(y), None, None, 0, 0.0, P(dq), P(dh), P(lq), fused._stream()),
          "head0")
    y, dq, lq, dh = outs[1]
    L._ok(lib.aac_uam_td_mse_head(P(ht), P(wt), P(bt), P(rew), P(done), ldr, 0.95, P(y), P(h), P(w), P(b), B, P(dq),
                                  P(dh), P(lq), fused._stream()), "td_mse")
    torch.cuda.synchronize()
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
