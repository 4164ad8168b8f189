"""GPU tests of the fused learner building blocks (include/aac_fused.h) against plain PyTorch
fp64 references, and of the fused update against the autograd learner and the CPU restatement."""
import functools

import numpy as np
import pytest
import torch

from oracle import learner_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _op(x, t):
    return x.t() if t else x


CASES = [  # M, N, K, ta, tb, ones, act, mact, addend
    (5, 3, 7, 0, 0, 0, 0, 0, False),
    (130, 70, 300, 0, 1, 0, 1, 0, False),
    (64, 64, 16, 1, 0, 0, 2, 0, True),
    (1, 256, 1024, 1, 0, 1, 0, 0, False),
    (256, 193, 5120, 1, 0, 1, 0, 0, False),
    (1024, 640, 256, 0, 0, 0, 0, 1, False),
    (5120, 2, 256, 0, 1, 0, 2, 0, False),
    (5120, 64, 64, 0, 0, 0, 0, 1, True),
    (97, 129, 33, 1, 1, 0, 0, 2, False),
    (25600, 256, 192, 0, 1, 0, 1, 0, True),      # >= 2048 tiles: one tile per wave (wide), 16-B epilogue
    (20480, 130, 64, 0, 1, 0, 2, 1, False),      # wide, unaligned rows: element-wise epilogue
    (20480, 100, 64, 0, 1, 0, 1, 0, True),       # wide, 16-B rows with a ragged last column group
    # LDS-staged workgroup tiles, every operand layout, ragged edges, the ones column
    (256, 640, 1024, 1, 0, 1, 0, 0, False),      # weight gradient: A and B row-contiguous, ones column
    (96, 100, 100, 1, 1, 0, 1, 0, True),         # A row-contiguous, B K-contiguous, ragged K chunk
    (200, 132, 68, 1, 0, 0, 2, 2, True),
    (1000, 36, 260, 0, 0, 0, 1, 1, True),        # ragged rows
    (256, 300, 64, 0, 1, 0, 0, 0, False),
    (192, 64, 96, 1, 1, 0, 1, 0, True),
    (32, 200, 128, 0, 0, 0, 0, 1, False),
    (5120, 256, 640, 0, 1, 0, 1, 0, True),
]
LDS_CASES = {(1024, 640, 256), (5120, 64, 64), (25600, 256, 192), (20480, 130, 64), (20480, 100, 64), (256, 640, 1024),
             (96, 100, 100), (200, 132, 68), (1000, 36, 260), (5120, 256, 640), (130, 70, 300),
             (256, 300, 64), (192, 64, 96), (32, 200, 128)}

@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["t64x64", "t64x32", "t32x64", "t32x32", "registers"])
def lds_everywhere(request):
    """Every eligible product on the given LDS workgroup tile, whatever its size; or ("registers")
    none, so every product takes the register path."""
    from multi_agent_aac_amd import fused
    fused.set_lds_policy(-1 - request.param if request.param < 4 else 1 << 30)
    yield request.param
    fused.set_lds_policy()


@pytest.mark.parametrize("case", CASES)
def test_gemm_batch_epilogues(native_lib, lds_everywhere, case):
    from multi_agent_aac_amd import fused
    M, N, K, ta, tb, ones, act, mact, add = case
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N)
    r = lambda *s: torch.rand(*s, device=DEV, generator=g) * 2 - 1   # noqa: E731
    A = r(K, M) if ta else r(M, K)
    B = r(N, K) if tb else r(K, N)
    bias = r(N) if not ones else None
    addend = r(M, N) if add else None
    mask = r(M, N) if mact else None
    C = torch.full((M, N), 7.0, device=DEV)
    cextra = torch.zeros(M, device=DEV) if ones else None
    p = fused.prob(fused.ptr(A), fused.ptr(B), fused.ptr(C), M, N, K, A.shape[1], B.shape[1], N, ta=ta, tb=tb,
                   bias=fused.ptr(bias), act=act, addend=fused.ptr(addend), ldadd=N, mask=fused.ptr(mask), ldmask=N,
                   mact=mact, ones=ones, cextra=fused.ptr(cextra))
    launch = fused.GemmLaunch([p])
    cfg = launch.plan()[0][0]
    if lds_everywhere < 4:
        assert (cfg > 0) == ((M, N, K) in LDS_CASES), launch.plan()
        assert cfg == 0 or (cfg - 1) >> 2 == lds_everywhere
    else:
        assert cfg == 0
    launch()
    prod = _op(A.double(), ta) @ _op(B.double(), tb)
    want = prod.clone()
    if add:
        want += addend.double()
    if bias is not None:
        want += bias.double()
    if act == 1:
        want = want.clamp_min(0)
    elif act == 2:
        want = torch.tanh(want)
    if mact == 1:
        want = want * (mask > 0)
    elif mact == 2:
        want = want * (1 - mask.double() ** 2)
    tol = 2e-6 * np.sqrt(K) + 1e-6
    np.testing.assert_allclose(C.cpu().double(), want.cpu(), atol=tol, rtol=1e-5)
    if ones:
        np.testing.assert_allclose(cextra.cpu().double(), _op(A.double(), ta).sum(1).cpu(), atol=tol, rtol=1e-5)
    C2 = torch.zeros_like(C)
    p2 = fused.prob(fused.ptr(A), fused.ptr(B), fused.ptr(C2), M, N, K, A.shape[1], B.shape[1], N, ta=ta, tb=tb,
                    bias=fused.ptr(bias), act=act, addend=fused.ptr(addend), ldadd=N, mask=fused.ptr(mask),
                    ldmask=N, mact=mact, ones=ones, cextra=fused.ptr(cextra))
    fused.GemmLaunch([p2])()
    assert torch.equal(C, C2)                    # deterministic


def test_gemm_batch_grouped(native_lib):
    """Several products of different shapes in one launch land where they should."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(0)
    shapes = [(100, 64, 22), (300, 128, 64), (2, 256, 5000), (64, 6, 9000)]
    As = [torch.randn(M, K, device=DEV) for M, N, K in shapes]
    Bs = [torch.randn(K, N, device=DEV) for M, N, K in shapes]
    Cs = [torch.empty(M, N, device=DEV) for M, N, K in shapes]
    probs = [fused.prob(fused.ptr(a), fused.ptr(b), fused.ptr(c), M, N, K, K, N, N)
             for (M, N, K), a, b, c in zip(shapes, As, Bs, Cs)]
    fused.GemmLaunch(probs)()
    for (M, N, K), a, b, c in zip(shapes, As, Bs, Cs):
        np.testing.assert_allclose(c.cpu().double(), (a.double() @ b.double()).cpu(), atol=3e-6 * np.sqrt(K) * 3,
                                   rtol=1e-5)


def test_gemm_xcd_order_bit_identical(native_lib):
    """aac_gemm_batch_ordered (XCD-aware workgroup order, the GRU learner's launches) only remaps
    workgroups to tiles: bit-identical to the round-robin order, on the learner's per-agent weight-
    gradient shapes (192 x 129 over K = 512 with the ones column) and ragged ones."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(5)
    shapes = [(192, 128, 512)] * 8 + [(64, 18, 512)] * 5 + [(37, 70, 333)] * 3
    Gs = [torch.randn(K, M, device=DEV) for M, N, K in shapes]
    Xs = [torch.randn(K, N, device=DEV) for M, N, K in shapes]
    out = []
    for xcd in (False, True):
        Cs = [torch.full((M * (N + 1),), 7.0, device=DEV) for M, N, K in shapes]
        probs = [fused.prob(fused.ptr(g), fused.ptr(x), fused.ptr(c), M, N, K, M, N, N, ta=1, ones=1,
                            cextra=fused.ptr(c, M * N)) for (M, N, K), g, x, c in zip(shapes, Gs, Xs, Cs)]
        fused.GemmLaunch(probs, xcd=xcd)()
        out.append(Cs)
    torch.cuda.synchronize()
    for a, b in zip(*out):
        assert torch.equal(a, b)
    for (M, N, K), g, x, c in zip(shapes, Gs, Xs, out[1]):
        np.testing.assert_allclose(c[:M * N].reshape(M, N).cpu().double(), (g.double().t() @ x.double()).cpu(),
                                   atol=3e-6 * np.sqrt(K) * 3, rtol=1e-5)


@pytest.mark.parametrize("N", [23, 64])
def test_gemm_split_copies(native_lib, lds_everywhere, N):
    """ksplit > 1 writes per-split partial products that sum to the full product (N = 64: the LDS
    workgroup tile, whose B image carries the ones column)."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(1)
    M, K, S = 64, 5120, 16
    G = torch.randn(K, M, device=DEV)          # stored rows x outputs, op(A) = G^T
    X = torch.randn(K, N, device=DEV)
    stride = M * N + M + 7
    part = torch.full((S, stride), 3.0, device=DEV)
    launch = fused.GemmLaunch([fused.prob(fused.ptr(G), fused.ptr(X), fused.ptr(part), M, N, K, M, N, N, ta=1, ones=1,
                                          cextra=fused.ptr(part, M * N), ksplit=S, split_stride=stride)])
    assert (launch.plan()[0][0] > 0) == (N % 4 == 0 and lds_everywhere < 4)
    launch()
    tot = part.double().sum(0)
    np.testing.assert_allclose(tot[:M * N].reshape(M, N).cpu(), (G.double().t() @ X.double()).cpu(), atol=2e-4)
    np.testing.assert_allclose(tot[M * N:M * N + M].cpu(), G.double().sum(0).cpu(), atol=2e-4)
    out = torch.empty(stride, device=DEV)
    fused.sum_partials(out, part, S)
    np.testing.assert_allclose(out.cpu().double(), tot.cpu(), atol=1e-4)


def test_gemm_rejects_bad_plans(native_lib):
    from multi_agent_aac_amd import fused
    for p, msg in ((fused.prob(1, 1, 1, 0, 4, 4, 4, 4, 4), "empty"),
                   (fused.prob(1, 1, 1, 4, 4, 4, 4, 4, 4, ones=1), "cextra"),
                   (fused.prob(1, 1, 1, 4, 4, 4, 4, 4, 4, bias=1, ksplit=2, split_stride=64), "plain")):
        with pytest.raises(RuntimeError, match=msg):
            fused.GemmLaunch([p])()


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_critic_head(native_lib, mode):
    from multi_agent_aac_amd import fused
    torch.manual_seed(mode)
    M, B, N = 3 * 128, 128, 3
    h = torch.relu(torch.randn(M, 256, device=DEV))
    w, b = torch.randn(256, device=DEV), torch.randn(1, device=DEV)
    y = torch.randn(M, device=DEV)
    rew = torch.randn(M, N, device=DEV)
    done = (torch.rand(M, N, device=DEV) < 0.2).float()
    q, dq, dh, yout = (torch.empty(M, device=DEV), torch.empty(M, device=DEV), torch.empty(M, 256, device=DEV),
                       torch.empty(M, device=DEV))
    P = fused.ptr
    fused.critic_head(P(h), M, P(w), P(b), mode, y=P(y), rew=P(rew), done=P(done), B=B, N=N, gamma=0.95, q=P(q),
                      dq=P(dq), dh=P(dh), yout=P(yout))
    qr = h.double() @ w.double() + b.double()
    np.testing.assert_allclose(q.cpu(), qr.cpu(), atol=1e-4, rtol=1e-5)
    if mode == 2:
        it = torch.arange(M, device=DEV) // B
        r = rew[torch.arange(M, device=DEV), it]
        want = r + 0.95 * q * (1 - (done == 1).any(1).float())
        np.testing.assert_allclose(yout.cpu(), want.cpu(), atol=1e-5, rtol=1e-5)
        return
    g = (2.0 / M) * (q - y) if mode == 0 else torch.full_like(q, -1.0 / M)
    np.testing.assert_allclose(dq.cpu(), g.cpu(), atol=1e-6, rtol=1e-6)
    np.testing.assert_allclose(dh.cpu(), (g[:, None] * w[None] * (h > 0)).cpu(), atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("with_product", [False, True])
def test_head_job_in_gemm_launch(native_lib, mode, with_product):
    """A critic-head job riding along in a grouped GEMM launch (aac_gemm_batch_heads) computes
    exactly what the standalone aac_critic_head launch computes (same device code), and the
    products of the launch are unaffected."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(10 + mode)
    M, B, N = 2 * 512 + 3, 512, 2
    P = fused.ptr
    h = torch.relu(torch.randn(M, 256, device=DEV))
    w, b = torch.randn(256, device=DEV), torch.randn(1, device=DEV)
    y, rew = torch.randn(M, device=DEV), torch.randn(M, N, device=DEV)
    done = (torch.rand(M, N, device=DEV) < 0.2).float()
    outs = [[torch.full((M,), 7.0, device=DEV), torch.full((M,), 7.0, device=DEV),
             torch.full((M, 256), 7.0, device=DEV), torch.full((M,), 7.0, device=DEV)] for _ in range(2)]
    kw = dict(y=P(y), rew=P(rew), done=P(done), B=B, N=N, gamma=0.95)
    q, dq, dh, yout = outs[0]
    fused.critic_head(P(h), M, P(w), P(b), mode, q=P(q), dq=P(dq), dh=P(dh), yout=P(yout), **kw)
    q, dq, dh, yout = outs[1]
    job = fused.head_job(P(h), M, P(w), P(b), mode, q=P(q), dq=P(dq), dh=P(dh), yout=P(yout), **kw)
    A, W = torch.randn(300, 40, device=DEV), torch.randn(72, 40, device=DEV)
    C = torch.zeros(300, 72, device=DEV)
    probs = [fused.prob(P(A), P(W), P(C), 300, 72, 40, 40, 40, 72, tb=1, act=fused.RELU)] if with_product else []
    fused.GemmLaunch(probs, heads=[job])()
    torch.cuda.synchronize()
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    if with_product:
        torch.testing.assert_close(C, torch.relu(A @ W.T), rtol=1e-5, atol=1e-5)


def test_chained_td_and_mse_head(native_lib):
    """A mode-2 head job with a chained mse head (critic step 0's loss on the first B rows of the TD
    targets it has just computed; aac_critic_head_job) equals the two standalone aac_critic_head
    launches bit for bit."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(21)
    B, nb, N = 300, 3, 4
    Bt = nb * B
    P = fused.ptr
    ht, h = torch.relu(torch.randn(Bt, 256, device=DEV)), torch.relu(torch.randn(B, 256, device=DEV))
    wt, bt, w, b = (torch.randn(256, device=DEV), torch.randn(1, device=DEV), torch.randn(256, device=DEV),
                    torch.randn(1, device=DEV))
    rew = torch.randn(Bt, N, device=DEV)
    done = (torch.rand(Bt, N, device=DEV) < 0.2).float()
    outs = [[torch.full((Bt,), 7.0, device=DEV), torch.full((B,), 7.0, device=DEV), torch.full((B,), 7.0, device=DEV),
             torch.full((B, 256), 7.0, device=DEV)] for _ in range(2)]
    y, q, dq, dh = outs[0]
    fused.critic_head(P(ht), Bt, P(wt), P(bt), 2, rew=P(rew), done=P(done), B=B, N=N, gamma=0.95, yout=P(y))
    fused.critic_head(P(h), B, P(w), P(b), 0, y=P(y), q=P(q), dq=P(dq), dh=P(dh))
    y, q, dq, dh = outs[1]
    job = fused.head_job(P(ht), Bt, P(wt), P(bt), 2, rew=P(rew), done=P(done), B=B, N=N, gamma=0.95, yout=P(y),
                         chain=(P(h), P(w), P(b), P(q), P(dq), P(dh), B))
    fused.critic_head_job(job)
    torch.cuda.synchronize()
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    with pytest.raises(RuntimeError, match="chained"):
        fused.GemmLaunch([], heads=[job])()


def test_dual_output_is_actor_loss_head(native_lib):
    """The combine layer's dual output C2 = (C > 0) dscale w equals aac_critic_head mode 1's dh
    (dq = -1/B) bit for bit, on the register path with ragged tiles."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(3)
    B, K = 1000, 640
    P = fused.ptr
    f = torch.relu(torch.randn(B, K, device=DEV))
    Wc, bc = torch.randn(256, K, device=DEV) * 0.05, torch.randn(256, device=DEV) * 0.1
    wq, bq = torch.randn(256, device=DEV), torch.randn(1, device=DEV)
    h, dh = torch.empty(B, 256, device=DEV), torch.empty(B, 256, device=DEV)
    scale = -float(np.float32(1.0) / np.float32(B))
    fused.GemmLaunch([fused.prob(P(f), P(Wc), P(h), B, 256, K, K, K, 256, tb=1, bias=P(bc), act=fused.RELU,
                                 dvec=P(wq), C2=P(dh), dscale=scale)])()
    dh_ref = torch.empty(B, 256, device=DEV)
    fused.critic_head(P(h), B, P(wq), P(bq), 1, dh=P(dh_ref))
    torch.cuda.synchronize()
    assert torch.equal(dh, dh_ref)
    torch.testing.assert_close(h, torch.relu(f @ Wc.T + bc), rtol=1e-4, atol=1e-4)


def test_gather_strided(native_lib):
    from multi_agent_aac_amd import fused
    rw, B = 50, 33
    ring = torch.arange(200 * rw, dtype=torch.float32, device=DEV).reshape(200, rw)
    idx = torch.randperm(200, device=DEV)[:B].to(torch.int32)
    X = torch.full((B, 3, 6), -1.0, device=DEV)
    X2 = torch.full((B, 3, 6), -2.0, device=DEV)
    rest = torch.empty(B, 50 - 18, device=DEV)
    fused.gather_strided(ring, idx, [fused.ptr(X), fused.ptr(X, 4), fused.ptr(rest)], [12, 6, 32], [4, 2, 32],
                         [6, 6, 32], dsts2=[fused.ptr(X2), None, None])
    src = ring[idx.long()].cpu()
    Xc = X.cpu()
    assert torch.equal(X2.cpu()[:, :, :4], src[:, :12].reshape(B, 3, 4))
    assert (X2.cpu()[:, :, 4:] == -2.0).all()
    assert torch.equal(Xc[:, :, :4], src[:, :12].reshape(B, 3, 4))
    assert torch.equal(Xc[:, :, 4:], src[:, 12:18].reshape(B, 3, 2))
    assert torch.equal(rest.cpu(), src[:, 18:])


@pytest.mark.parametrize("N,B", [(3, 64), (5, 256)])
def test_autograd_learner_matches_cpu_restatement(native_lib, N, B):
    """The layer-by-layer autograd learner (fused=False) stays a second, independent GPU path."""
    from multi_agent_aac_amd.maddpg import MADDPG
    cls = functools.partial(MADDPG, fused=False)
    assert learner_ref.check_one_update(cls, device=DEV, N=N, B=B, E=128, tol=1e-5, iters=2)


def test_fused_equals_autograd_learner(native_lib):
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B, E = 5, 256, 512
    ms = []
    for fz in (True, False):
        m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=N, device=DEV, seed=4, batch_size=B, fused=fz)
        rep = m.attach_replay(4 * E, seed=2)
        for p in range(3):
            tr = learner_ref.random_transitions(E, N, 10 + p)
            rep.push_batch(*[tr[k].to(DEV).contiguous() for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done",
                                                                   "n_own", "n_radar", "n_nei")])
        ms.append(m)
    for _ in range(3):
        sa = ms[0].update(B, use_graph=False)
        sb = ms[1].update(B, use_graph=False)
        for (la, aa, qa, ta), (lb, ab, qb, tb) in zip(sa, sb):
            np.testing.assert_allclose(qa.cpu(), qb.cpu(), atol=1e-5, rtol=1e-5)
            np.testing.assert_allclose(ta.cpu(), tb.cpu(), atol=1e-5, rtol=1e-5)
            np.testing.assert_allclose(float(aa), float(ab), atol=1e-5, rtol=1e-5)
    # 15 Adam steps: a parameter whose gradient sits near zero moves by ~lr * sign(m / sqrt(v)), so
    # fp32 summation-order differences between the two learners can show at ~1e-5 there
    for a, b in ((ms[0].fa.data, ms[1].fa.data), (ms[0].fc.data, ms[1].fc.data), (ms[0].fa_t.data, ms[1].fa_t.data)):
        np.testing.assert_allclose(a.cpu(), b.cpu(), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("K", [1, 4, 7, 15])
def test_attn_block_matches_reference_attention(native_lib, K):
    """Fused inference attention (x_j on the fly, Wqk = Wk^T Wq, v_att = Wv sum a_j x_j) against
    the reference's k / v projections and masked softmax (ATT/nets:186-210), fp64."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(K)
    R = 777
    eo = torch.relu(torch.randn(R, 64, device=DEV))
    nei = torch.randn(R, K, 6, device=DEV)
    nei[::5, 0] = 0.0                          # masked neighbours
    nei[3] = 0.0                               # an all-masked row
    Wn, bn = torch.randn(64, 6, device=DEV) * 0.4, torch.randn(64, device=DEV) * 0.1
    Wq, Wk, Wv = (torch.randn(64, 64, device=DEV) * 0.125 for _ in range(3))
    kv = torch.cat([Wk, Wv], 0).contiguous()
    wqk = (Wk.t() @ Wq).contiguous()
    out = torch.full((R, 64), 9.0, device=DEV)
    P = fused.ptr
    fused.attn_block(P(eo), 64, P(nei), P(Wn), P(bn), P(wqk), P(kv, 64 * 64), P(out), 64, R, K)
    d = lambda t: t.double().cpu()   # noqa: E731
    x = torch.relu(d(nei) @ d(Wn).t() + d(bn))
    q = d(eo) @ d(Wq).t()
    k, v = x @ d(Wk).t(), x @ d(Wv).t()
    score = torch.einsum("rkc,rc->rk", k, q) / 8.0
    mask = d(nei).mean(-1) != 0
    score[~mask] = float("-inf")
    a = torch.softmax(score, dim=1)
    a[~mask] = 0.0
    a = torch.nan_to_num(a)
    want = torch.einsum("rk,rkc->rc", a, v)
    np.testing.assert_allclose(out.cpu().double(), want, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("ws,E", [(True, 1024), (True, 77), (False, 1024)])
def test_fused_act_matches_ref_actor(native_lib, monkeypatch, ws, E):
    """The fused HIP choose_action forward (encoders + attention in one launch, then merge + tanh: the
    weights-stationary aac_actor_head_ws when ``ws``, else a grouped-GEMM launch + aac_actor_out_noise)
    at config 2's size (E = 1024 envs x N = 5 agents; E = 77: a ragged last row block) against
    oracle/learner_ref.RefActor, the CPU restatement of ActorNetwork_ATT_TwoPortion (ATT/nets:177-213),
    loaded with the same reference state_dict."""
    from multi_agent_aac_amd import fused
    from multi_agent_aac_amd.maddpg import MADDPG
    monkeypatch.setattr(fused, "ACT_HEAD_WS", ws)
    m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=5, device=DEV, seed=3)
    ref = learner_ref.RefActor([22, 18, 6], 2)
    ref.load_state_dict({k: v.cpu() for k, v in m.actors.reference_state_dict().items()})
    g = torch.Generator().manual_seed(5)
    N = 5
    own, radar = torch.randn(E, N, 22, generator=g), torch.rand(E, N, 18, generator=g) * 15
    nei = torch.randn(E, N, 4, 6, generator=g)
    nei[::7, :, 1] = 0.0                         # masked neighbours
    nei[5, 2] = 0.0                              # an all-masked attention row
    got = m.act(own.to(DEV), radar.to(DEV), nei.to(DEV), noisy=False).clone()
    with torch.no_grad():
        want = learner_ref.actor_rows(ref, own, radar, nei)
    np.testing.assert_allclose(got.cpu(), want, atol=1e-5, rtol=1e-5)
    # noisy: the output layer + noise + clamp launch (aac_actor_out_noise) = clamp(tanh + noise), with
    # the noise of the standalone noise kernel (same draw from the same counter epoch)
    from multi_agent_aac_amd import ops
    ep = torch.randint(1, 9000, (E,), dtype=torch.int32, device=DEV)
    noise = torch.empty(E, N, 2, device=DEV)
    c0 = m.noise_counter.clone()
    noisy = m.act(own.to(DEV), radar.to(DEV), nei.to(DEV), episode=ep, noise_out=noise).clone()
    assert int(m.noise_counter) == int(c0) + 1
    np.testing.assert_allclose(noisy.cpu(), torch.clamp(torch.as_tensor(want) + noise.cpu(), -1, 1), atol=1e-5,
                               rtol=1e-5)
    a2, n2 = got.clone(), torch.empty_like(noise)
    ops.noise_clamp(a2, ep, 8000, 1.0, m.noise_seed, c0, n2)
    assert torch.equal(n2, noise)
    assert float(noise.abs().max()) > 0.1


@pytest.mark.parametrize("K", [1, 4, 7, 12])       # K <= 8: MFMA kernels; 12: per-row kernels
def test_attn_train_fwd_bwd_matches_autograd(native_lib, K):
    """Training attention kernels (in-kernel q / k / v projections) against fp64 autograd of the
    reference form (ATT/nets:186-210): v_att, and the gradients into x_j, q and e_o."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(10 + K)
    R = 600
    eo = torch.relu(torch.randn(R, 64, device=DEV))
    x = torch.relu(torch.randn(R, K, 64, device=DEV))
    nei = torch.randn(R, K, 6, device=DEV)
    nei[::4, 0] = 0.0
    nei[7] = 0.0
    Wq, Wk, Wv = (torch.randn(64, 64, device=DEV) * 0.125 for _ in range(3))
    kv = torch.cat([Wk, Wv], 0).contiguous()
    cat = torch.zeros(R, 192, device=DEV)
    cat[:, :64] = eo
    z = lambda *s: torch.empty(*s, device=DEV)   # noqa: E731
    q, qk, alpha, xb = z(R, 64), z(R, 64), z(R, K), z(R, 64)
    P = fused.ptr
    fused.attn_train_fwd(P(cat), 192, P(x), P(nei), P(Wq), P(kv), P(kv, 64 * 64), P(q), P(qk), P(alpha), P(xb),
                         P(cat, 128), 192, R, K)
    dv, dcat_o = torch.randn(R, 64, device=DEV), torch.randn(R, 64, device=DEV)
    dxn, dqk, dq, deo = z(R * K, 64), z(R, 64), z(R, 64), z(R, 64)
    fused.attn_train_bwd(P(dv), 64, P(x), P(alpha), P(qk), P(cat), 192, P(dcat_o), 64, P(Wq), P(kv), P(kv, 64 * 64),
                         P(dxn), P(dqk), P(dq), P(deo), R, K)
    d = lambda t: t.double().cpu()   # noqa: E731
    eo_r = d(eo).requires_grad_()
    x_r = d(x).requires_grad_()
    q_r = eo_r @ d(Wq).t()
    q_r.retain_grad()
    k_r, v_r = x_r @ d(Wk).t(), x_r @ d(Wv).t()
    score = torch.einsum("rkc,rc->rk", k_r, q_r) / 8.0
    mask = d(nei).mean(-1) != 0
    score = score.masked_fill(~mask, float("-inf"))
    a = torch.nan_to_num(torch.softmax(score, dim=1)).masked_fill(~mask, 0.0)
    v_att = torch.einsum("rk,rkc->rc", a, v_r)
    ((v_att * d(dv)).sum() + (eo_r * d(dcat_o)).sum()).backward()
    np.testing.assert_allclose(cat[:, 128:].cpu().double(), v_att.detach(), atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(alpha.cpu().double(), a.detach(), atol=1e-6)
    np.testing.assert_allclose(q.cpu().double(), q_r.detach(), atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(dxn.cpu().double().reshape(R, K, 64), x_r.grad * (d(x) > 0), atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(dq.cpu().double(), q_r.grad, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(deo.cpu().double(), eo_r.grad * (d(eo) > 0), atol=2e-5, rtol=1e-5)
    if K <= 8:
        # the same backward with the neighbour encoder's weight-gradient partials instead of the dx_j
        # rows: the rows sum to dWn | dbn = sum dx_j^T [nei_j | 1]; dqk, dq, deo bit-identical
        npart = fused.attn_bwd_partials(R)
        pwn = torch.full((npart, 448), 7.0, device=DEV)
        dqk2, dq2, deo2 = z(R, 64), z(R, 64), z(R, 64)
        fused.attn_train_bwd_wn(P(dv), 64, P(x), P(alpha), P(qk), P(cat), 192, P(dcat_o), 64, P(Wq), P(kv),
                                P(kv, 64 * 64), P(dqk2), P(dq2), P(deo2), R, K, P(nei), P(pwn))
        torch.cuda.synchronize()
        assert torch.equal(dqk2, dqk) and torch.equal(dq2, dq) and torch.equal(deo2, deo)
        g = d(dxn).reshape(R * K, 64)
        want_w = g.t() @ d(nei).reshape(R * K, 6)
        tot = d(pwn).sum(0)
        np.testing.assert_allclose(tot[:384].reshape(64, 6), want_w, atol=2e-4, rtol=1e-5)
        np.testing.assert_allclose(tot[384:], g.sum(0), atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("K", [1, 4, 7])
def test_attn_enc_fwd_matches_reference(native_lib, K):
    """aac_attn_enc_fwd: the actor's encoders (e_o, e_g, x_j) computed inside the attention launch
    (ATT/nets:194-210) against fp64 torch -- training (q, qk, alpha, xb, x_j kept) and inference --
    plus the riding critic-encoder job (ATT/nets:697-701); a two-set launch gives the same bits as
    the sets launched alone."""
    from types import SimpleNamespace

    from multi_agent_aac_amd import fused
    torch.manual_seed(20 + K)
    R, D0, Nc, Din, rows = 611, 6 + 4 * K, 5, 24, 203
    d = lambda t: t.double().cpu()   # noqa: E731
    r = lambda *s, sc=1.0: (torch.randn(*s, device=DEV) * sc).contiguous()   # noqa: E731
    own = r(R, D0 + 2)                            # row stride D0 + 2 (the critic-input rows)
    radar = torch.rand(R, 18, device=DEV) * 15
    nei = r(R, K, 6)
    nei[::4, 0] = 0.0
    nei[9] = 0.0                                  # an all-masked row
    W = {k: r(*s, sc=sc) for k, s, sc in (("Wo", (64, D0), 0.3), ("bo", (64,), 0.1), ("Wg", (64, 18), 0.1),
                                             ("bg", (64,), 0.1), ("Wn", (64, 6), 0.4), ("bn", (64,), 0.1),
                                             ("Wq", (64, 64), 0.125))}
    kv = r(128, 64, sc=0.125)
    P = fused.ptr
    ap = SimpleNamespace(**{k: P(v) for k, v in W.items()}, Wkv=P(kv))
    cx = r(rows, Nc, Din)
    cw, cb = r(Nc, 128, Din, sc=0.2), r(Nc, 128, sc=0.1)
    cp = SimpleNamespace(enc_w=[P(cw, n * 128 * Din) for n in range(Nc)], enc_b=[P(cb, n * 128) for n in range(Nc)])
    acts = fused.ActorActs(R, K, DEV)
    cat_t = torch.full((R, 192), 7.0, device=DEV)
    cat_i = torch.full((R, 192), 7.0, device=DEV)
    f1 = torch.full((rows, Nc * 128), 7.0, device=DEV)
    tr = fused.attn_set(ap, P(own), D0 + 2, D0, P(radar), P(nei), R, K, P(cat_t), acts=acts,
                        ride=fused.critic_enc_ride(cp, P(cx), rows, Nc, Din, f1))
    inf = fused.attn_set(ap, P(own), D0 + 2, D0, P(radar), P(nei), R, K, P(cat_i))
    fused.AttnEnc(tr, inf)()
    torch.cuda.synchronize()
    # reference (fp64)
    eo = torch.relu(d(own)[:, :D0] @ d(W["Wo"]).t() + d(W["bo"]))
    eg = torch.relu(d(radar) @ d(W["Wg"]).t() + d(W["bg"]))
    x = torch.relu(d(nei) @ d(W["Wn"]).t() + d(W["bn"]))
    q = eo @ d(W["Wq"]).t()
    k, v = x @ d(kv[:64]).t(), x @ d(kv[64:]).t()
    score = torch.einsum("rkc,rc->rk", k, q) / 8.0
    mask = d(nei).mean(-1) != 0
    a = torch.nan_to_num(torch.softmax(score.masked_fill(~mask, float("-inf")), dim=1)).masked_fill(~mask, 0.0)
    want = torch.cat([eo, eg, torch.einsum("rk,rkc->rc", a, v)], 1)
    for cat in (cat_t, cat_i):
        np.testing.assert_allclose(cat.cpu().double(), want, atol=3e-5, rtol=1e-5)
    np.testing.assert_allclose(acts.xn.cpu().double().reshape(R, K, 64), x, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(acts.qa.cpu().double(), q, atol=2e-5, rtol=1e-5)
    np.testing.assert_allclose(acts.qk.cpu().double(), q @ d(kv[:64]), atol=3e-5, rtol=1e-5)
    np.testing.assert_allclose(acts.alpha.cpu().double(), a, atol=1e-6)
    np.testing.assert_allclose(acts.xb.cpu().double(), torch.einsum("rk,rkc->rc", a, x), atol=2e-5, rtol=1e-5)
    fw = torch.relu(torch.einsum("bnd,ncd->bnc", d(cx), d(cw)) + d(cb)).reshape(rows, Nc * 128)
    np.testing.assert_allclose(f1.cpu().double(), fw, atol=2e-5, rtol=1e-5)
    # the sets alone, and the riding job alone: the same bits
    cat2, cat3, f2 = torch.zeros_like(cat_t), torch.zeros_like(cat_i), torch.zeros_like(f1)
    acts2 = fused.ActorActs(R, K, DEV)
    fused.AttnEnc(fused.attn_set(ap, P(own), D0 + 2, D0, P(radar), P(nei), R, K, P(cat2), acts=acts2))()
    fused.AttnEnc(fused.attn_set(ap, P(own), D0 + 2, D0, P(radar), P(nei), R, K, P(cat3)))()
    fused.AttnEnc(fused.ride_only(fused.critic_enc_ride(cp, P(cx), rows, Nc, Din, f2)))()
    torch.cuda.synchronize()
    assert torch.equal(cat2, cat_t) and torch.equal(cat3, cat_i) and torch.equal(f2, f1)
    for n in ("xn", "qa", "qk", "alpha", "xb"):
        assert torch.equal(getattr(acts2, n), getattr(acts, n)), n


@pytest.mark.parametrize("rows", [1024, 203])
def test_out_layer_folded_into_critic_encoder_job(native_lib, rows):
    """The actor's tanh output layer folded into the critic-encoder riding job (o_h: ATT/nets:213 on
    the actor rows ha[b*N + n]): the actions written into the critic-input rows match fp64 torch,
    the encoders use them, and a critic-head job riding in the same launch (aac_attn_enc_fwd_head)
    gives the bits of the standalone aac_critic_head."""
    from types import SimpleNamespace

    from multi_agent_aac_amd import fused
    torch.manual_seed(31 + rows)
    Nc, D0 = 5, 22
    Din = D0 + 2
    d = lambda t: t.double().cpu()   # noqa: E731
    P = fused.ptr
    X = torch.randn(rows, Nc, Din, device=DEV)
    X[:, :, D0:] = 99.0                                   # stale actions: must be overwritten
    ha = torch.relu(torch.randn(rows * Nc, 256, device=DEV))
    wa, ba = torch.randn(2, 256, device=DEV) * 0.1, torch.randn(2, device=DEV) * 0.1
    cw, cb = torch.randn(Nc, 128, Din, device=DEV) * 0.2, torch.randn(Nc, 128, device=DEV) * 0.1
    cp = SimpleNamespace(enc_w=[P(cw, n * 128 * Din) for n in range(Nc)], enc_b=[P(cb, n * 128) for n in range(Nc)])
    ap = SimpleNamespace(Wa=P(wa), ba=P(ba))
    f = torch.full((rows, Nc * 128), 7.0, device=DEV)
    # a head job beside it (mode 0 on unrelated rows)
    M = 517
    h = torch.relu(torch.randn(M, 256, device=DEV))
    w, b, y = torch.randn(256, device=DEV), torch.randn(1, device=DEV), torch.randn(M, device=DEV)
    outs = [[torch.full((M,), 7.0, device=DEV), torch.full((M,), 7.0, device=DEV),
             torch.full((M, 256), 7.0, device=DEV)] for _ in range(2)]
    q, dq, dh = outs[0]
    fused.critic_head(P(h), M, P(w), P(b), 0, y=P(y), q=P(q), dq=P(dq), dh=P(dh))
    q, dq, dh = outs[1]
    job = fused.head_job(P(h), M, P(w), P(b), 0, y=P(y), q=P(q), dq=P(dq), dh=P(dh))
    ride = fused.critic_enc_ride(cp, P(X), rows, Nc, Din, f, fold=(P(ha), ap, D0))
    fused.AttnEnc(fused.ride_only(ride), head=job)()
    torch.cuda.synchronize()
    a_ref = torch.tanh(d(ha) @ d(wa).t() + d(ba)).reshape(rows, Nc, 2)
    np.testing.assert_allclose(d(X[:, :, D0:]), a_ref, atol=2e-6, rtol=1e-5)
    xin = d(X).clone()
    fw = torch.relu(torch.einsum("bnd,ncd->bnc", xin, d(cw)) + d(cb)).reshape(rows, Nc * 128)
    np.testing.assert_allclose(d(f), fw, atol=2e-5, rtol=1e-5)
    for a_, c_ in zip(outs[0], outs[1]):
        assert torch.equal(a_, c_)


@pytest.mark.parametrize("n,ns,pad", [(65536, 32, 0), (180228, 8, 0), (4100, 40, 0), (1001, 8, 0), (1001, 8, 1),
                                      (4098, 16, 1), (4096, 3, 0), (256, 1, 0)])
def test_adam_sum_matches_torch(native_lib, n, ns, pad):
    """aac_adam_flat_sum (the copy-parallel kernel when the copy stride % 4 == 0, else the element
    kernel): the summed split-K gradient and torch.optim.Adam's arithmetic, two steps,
    deterministic; copies padded to a multiple of 4 floats as the learners lay them out
    (``pad``); aac_sum_partials gives the same bits as the Adam kernel's sum (the world > 1 path)."""
    from types import SimpleNamespace

    from multi_agent_aac_amd import fused
    g = torch.Generator(device=DEV).manual_seed(n + ns)
    p0 = torch.randn(n, device=DEV, generator=g)
    w = fused.padded(n) if pad else n
    parts = [torch.randn(ns, w, device=DEV, generator=g) * 1e-3 for _ in range(2)]
    runs = []
    for _ in range(2):
        flat = SimpleNamespace(data=p0.clone())
        opt = SimpleNamespace(flat=flat, exp_avg=torch.zeros(n, device=DEV), exp_avg_sq=torch.zeros(n, device=DEV),
                              lr=1e-3, betas=(0.9, 0.999), eps=1e-3, step_t=torch.zeros(1, dtype=torch.int32, device=DEV))
        gout = torch.empty(n, device=DEV)
        for k in range(2):
            fused.adam_sum(opt, parts[k], ns, k + 1, grad_out=gout)
        torch.cuda.synchronize()
        runs.append((flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), gout.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)                     # deterministic
    ref = p0.double().clone().requires_grad_(False)
    m = torch.zeros(n, dtype=torch.float64, device=DEV)
    v = torch.zeros(n, dtype=torch.float64, device=DEV)
    for k in range(2):
        gk = parts[k][:, :n].double().sum(0)
        t = k + 1
        m = 0.9 * m + 0.1 * gk
        v = 0.999 * v + 0.001 * gk * gk
        # eps 1e-3: the step is continuous in the gradient (at 1e-8 a summed gradient at rounding level
        # moves a weight by +-lr whatever its size, so fp32 vs fp64 summation could flip it)
        ref = ref - 1e-3 / (1 - 0.9 ** t) * m / (v.sqrt() / np.sqrt(1 - 0.999 ** t) + 1e-3)
    p, mm, vv, gg = runs[0]
    summed = torch.empty(n, device=DEV)
    fused.sum_partials(summed, parts[1], ns)
    torch.cuda.synchronize()
    assert torch.equal(summed, gg)
    np.testing.assert_allclose(gg.cpu().double(), parts[1][:, :n].double().sum(0).cpu(), rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(mm.cpu().double(), m.cpu(), rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(p.cpu().double(), ref.cpu(), rtol=0, atol=1e-6)


def test_merged_schedule_equals_serial(native_lib, monkeypatch):
    """world == 1: the merged schedule (critic step i+1 zipped with the actor step i into shared
    launches, both Adam steps in one launch) is bit-identical to the serial update order, with
    fewer launches."""
    from multi_agent_aac_amd import fused
    from multi_agent_aac_amd.maddpg import MADDPG
    N, B, E = 5, 256, 512
    ms, nl = [], []
    for merged in (True, False):
        monkeypatch.setattr(fused.FusedUpdate, "MERGED", merged)
        m = MADDPG([22, 18, 6], [22, 18, 6], 2, n_agents=N, device=DEV, seed=4, batch_size=B)
        rep = m.attach_replay(4 * E, seed=2)
        for p in range(3):
            tr = learner_ref.random_transitions(E, N, 10 + p)
            rep.push_batch(*[tr[k].to(DEV).contiguous() for k in ("s_own", "s_radar", "s_nei", "act", "rew", "done",
                                                                   "n_own", "n_radar", "n_nei")])
        for _ in range(2):
            m.update(B, use_graph=False)
        m.update(B, use_graph=True)
        nl.append(m._fused_plan(B).n_launches)
        ms.append(m)
    torch.cuda.synchronize()
    for name in ("fa", "fc", "fa_t", "fc_t"):
        assert torch.equal(getattr(ms[0], name).data, getattr(ms[1], name).data), name
    assert torch.equal(ms[0].actor_optimizer.exp_avg_sq, ms[1].actor_optimizer.exp_avg_sq)
    assert nl[0] < nl[1], nl


@pytest.mark.parametrize("N,B,with_head", [(5, 1024, False), (3, 200, True), (8, 64, False)])
def test_dcomb_out_bwd_matches_reference(native_lib, N, B, with_head):
    """aac_actor_dcomb_out_bwd (the actor step's critic data gradient df = (dh Wc) * (f > 0) reduced
    straight into the actor output backward, ATT/maddpg:421-425) against fp64 torch, and against the
    two launches it replaces (grouped-GEMM df + aac_actor_out_bwd) at fp32 rounding; a riding head job
    equals the standalone aac_critic_head bit for bit.  B = 200: a ragged last sample block."""
    from multi_agent_aac_amd import fused
    torch.manual_seed(N * 100 + B)
    P = fused.ptr
    D0 = 6 + 4 * (N - 1)
    Din = D0 + 2
    R = B * N
    dh = torch.randn(B, 256, device=DEV) * 0.1
    Wc = torch.randn(256, 128 * N, device=DEV) * 0.05
    f = torch.relu(torch.randn(B, 128 * N, device=DEV))
    wenc = torch.randn(N, 128, Din, device=DEV) * 0.1
    X = torch.rand(B, N, Din, device=DEV) * 2 - 1
    wa = torch.randn(2, 256, device=DEV) * 0.1
    ha = torch.relu(torch.randn(R, 256, device=DEV))
    dout, dha = torch.full((R, 2), 7.0, device=DEV), torch.full((R, 256), 7.0, device=DEV)
    head, houts = None, None
    if with_head:
        M = 3 * 64 + 5
        hh = torch.relu(torch.randn(M, 256, device=DEV))
        hw, hb, hy = torch.randn(256, device=DEV), torch.randn(1, device=DEV), torch.randn(M, device=DEV)
        houts = [[torch.full((M,), 7.0, device=DEV), torch.full((M,), 7.0, device=DEV),
                  torch.full((M, 256), 7.0, device=DEV)] for _ in range(2)]
        q, dq, dhh = houts[0]
        fused.critic_head(P(hh), M, P(hw), P(hb), 0, y=P(hy), q=P(q), dq=P(dq), dh=P(dhh))
        q, dq, dhh = houts[1]
        head = fused.head_job(P(hh), M, P(hw), P(hb), 0, y=P(hy), q=P(q), dq=P(dq), dh=P(dhh))
    a = fused.DaobArgs(P(dh), P(Wc), P(f), P(wenc), P(X), P(wa), P(ha), P(dout), P(dha), 128 * N, Din, D0, N, B)
    fused.DcombAob(a, head)()
    # the two-launch path
    df = torch.empty(B, 128 * N, device=DEV)
    fused.GemmLaunch([fused.prob(P(dh), P(Wc), P(df), B, 128 * N, 256, 256, 128 * N, 128 * N, mask=P(f),
                                 ldmask=128 * N, mact=fused.RELU)])()
    dout2, dha2 = torch.empty(R, 2, device=DEV), torch.empty(R, 256, device=DEV)
    fused.actor_out_bwd(P(df), 128 * N, P(wenc), Din, D0, P(X), P(wa), P(ha), N, R, P(dout2), P(dha2))
    torch.cuda.synchronize()
    # fp64 reference
    d = dh.double() @ Wc.double() * (f > 0)
    da = torch.einsum("bnc,ncj->bnj", d.view(B, N, 128), wenc.double()[:, :, D0:D0 + 2]).reshape(R, 2)
    a_ = X.double()[:, :, D0:D0 + 2].reshape(R, 2)
    o = da * (1 - a_ * a_)
    dh_ref = (o @ wa.double()) * (ha > 0)
    np.testing.assert_allclose(dout.cpu().double(), o.cpu(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dha.cpu().double(), dh_ref.cpu(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dout.cpu(), dout2.cpu(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dha.cpu(), dha2.cpu(), rtol=1e-4, atol=1e-6)
    if with_head:
        for x, y in zip(*houts):
            assert torch.equal(x, y)
