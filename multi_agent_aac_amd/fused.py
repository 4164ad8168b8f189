"""Fused MADDPG learner: ``update_myown`` (ATT/maddpg:219-440) as ~25 HIP launches per gradient
iteration instead of ~90 autograd kernels.

Every product of the actor / critic forward and backward is an ``aac_gemm_batch`` launch (grouped
fp32 MFMA GEMM with the activation, activation-derivative, bias-gradient and add epilogues fused,
include/aac_fused.h); independent products of the same depth share one launch.  The backward is
written out by hand (no autograd):

critic step (batch i, ATT/maddpg:375-387)        actor step (ATT/maddpg:389-425)
  f_n = relu(enc_n [own_n, a_n])   (N products)    e_o, e_g, x = relu(...)          (3 products)
  h   = relu(Wc f)                                 attention: q, Wk^T q, softmax, Wv sum a x (kernel)
  q, dq = 2(q - y)/B, dh = dq Wo * (h > 0)         h_a = relu(Wm [e_o e_g v_att]); a = tanh(Wa h_a)
  dWo|dbo, dWc|dbc, df = dh Wc * (f > 0)  (3)      critic forward on a (2 + head), dh (dq = -1/B)
  dW_enc_n | db_enc_n                     (N)      df; dout = (df W_enc[:, a]) (1 - a^2), dh_a (kernel)
  Adam                                             dWa|dba, dWm|dbm, d e_o', d e_g, d v_att  (5)
                                                   attention backward -> dx, dqk, dq, d e_o (kernel)
                                                   dWv, dWk, dWq, dW_nei|db, dW_own|db, dW_grid|db (6)
                                                   Adam
The TD targets of all N iterations are one batched forward of the target networks (they only
change in the Polyak step after the loop, ATT/maddpg:436-438), and the N batches are sampled and
gathered in one launch each.  Weight gradients are written (never accumulated) straight into the
networks' flat gradient buffers, so there is no zero_grad.
"""
import ctypes
import os

import numpy as np
import torch

from . import _native, ops, parallel

vp = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f32 = ctypes.c_float

NONE, RELU, TANH = 0, 1, 2


class GemmProb(ctypes.Structure):
    _fields_ = [("A", vp), ("B", vp), ("C", vp), ("bias", vp), ("addend", vp), ("mask", vp), ("cextra", vp),
                ("split_stride", i64), ("M", i32), ("N", i32), ("K", i32), ("lda", i32), ("ldb", i32), ("ldc", i32), ("ldadd", i32),
                ("ldmask", i32), ("ta", i32), ("tb", i32), ("act", i32), ("mact", i32), ("ones", i32),
                ("ksplit", i32), ("dvec", vp), ("C2", vp), ("dscale", f32)]


class HeadJob(ctypes.Structure):
    """aac_head_job: a critic-head row job riding along in a grouped GEMM launch."""
    _fields_ = [("h", vp), ("ldh", i32), ("M", i32), ("w", vp), ("b", vp), ("mode", i32), ("y", vp), ("rew", vp),
                ("done", vp), ("B", i32), ("N", i32), ("gamma", f32), ("q", vp), ("dq", vp), ("dh", vp), ("yout", vp),
                ("h2", vp), ("w2", vp), ("b2", vp), ("q2", vp), ("dq2", vp), ("dh2", vp), ("M2", i32)]


class AttnEncArgs(ctypes.Structure):
    """aac_attn_enc_args (include/aac_fused.h): the actor's encoders + neighbour attention of R rows,
    plus an optional riding job (the critic's per-agent encoders of c_rows samples)."""
    _fields_ = [("own", vp), ("ld_own", i32), ("d_own", i32), ("radar", vp), ("ld_radar", i32), ("nei", vp),
                ("Wo", vp), ("bo", vp), ("Wg", vp), ("bg", vp), ("Wn", vp), ("bn", vp), ("Wq", vp), ("Wk", vp),
                ("Wv", vp), ("cat", vp), ("ld_cat", i32), ("xn", vp), ("q", vp), ("qk", vp), ("alpha", vp),
                ("xb", vp), ("R", i32), ("K", i32), ("cx", vp), ("cx_ld", i32), ("c_din", i32), ("cW", vp),
                ("cb", vp), ("cf", vp), ("c_rows", i32), ("c_n", i32), ("o_h", vp), ("o_w", vp), ("o_b", vp),
                ("o_x", vp), ("o_d0", i32)]


class DaobArgs(ctypes.Structure):
    """aac_dcomb_aob_args (include/aac_fused.h): the actor step's critic data gradient + actor output
    backward in one launch."""
    _fields_ = [("dh", vp), ("Wc", vp), ("f", vp), ("wenc", vp), ("X", vp), ("wa", vp), ("ha", vp), ("dout", vp),
                ("dha", vp), ("ldw", i32), ("din", i32), ("d0", i32), ("N", i32), ("B", i32)]


GEMM_MAX = 16
HEAD_MAX = 1
_L = None


def lib():
    global _L
    if _L is None:
        L = _native.lib()
        L.aac_fused_last_error.restype = ctypes.c_char_p
        L.aac_gemm_batch.argtypes = [ctypes.POINTER(GemmProb), i32, vp]
        L.aac_gemm_batch_ordered.argtypes = [ctypes.POINTER(GemmProb), i32, i32, vp]
        L.aac_gemm_batch_heads.argtypes = [ctypes.POINTER(GemmProb), i32, ctypes.POINTER(HeadJob), i32, vp]
        L.aac_critic_head_job.argtypes = [ctypes.POINTER(HeadJob), vp]
        L.aac_gemm_plan.argtypes = [ctypes.POINTER(GemmProb), i32, vp, vp]
        L.aac_gemm_set_lds_policy.argtypes = [i32, i32]
        L.aac_adam_flat_sum.argtypes = [vp, vp, i32, vp, vp, vp, i64, f32, f32, f32, f32, vp, i32, vp]
        L.aac_sum_partials.argtypes = [vp, vp, i32, i64, vp]
        L.aac_sum_partials_strided.argtypes = [vp, vp, i32, i64, i64, vp]
        L.aac_adam_flat_sum_pair.argtypes = [ctypes.POINTER(AdamJob), ctypes.POINTER(AdamJob), vp]
        L.aac_adam_flat_sum_strided.argtypes = [vp, vp, i32, i64, vp, vp, vp, i64, f32, f32, f32, f32, vp, i32, vp]
        L.aac_critic_head.argtypes = [vp, i32, i32, vp, vp, i32, vp, vp, vp, i32, i32, f32, vp, vp, vp, vp, vp]
        L.aac_replay_gather_strided.argtypes = [vp, i32, vp, i32, i32, vp, vp, vp, vp, vp, vp]
        L.aac_attn_block.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp]
        L.aac_actor_out_bwd.argtypes = [vp, i32, vp, i32, i32, vp, vp, vp, i32, i32, vp, vp, vp]
        L.aac_actor_dcomb_out_bwd.argtypes = [ctypes.POINTER(DaobArgs), ctypes.POINTER(HeadJob), vp]
        L.aac_attn_train_fwd.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp]
        L.aac_attn_train_bwd.argtypes = [vp, i32, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, i32, i32,
                                         vp]
        L.aac_attn_enc_fwd.argtypes = [ctypes.POINTER(AttnEncArgs), i32, vp]
        L.aac_attn_enc_fwd_head.argtypes = [ctypes.POINTER(AttnEncArgs), i32, ctypes.POINTER(HeadJob), vp]
        L.aac_attn_train_bwd_wn.argtypes = [vp, i32, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, i32,
                                            i32, vp, vp, vp]
        L.aac_attn_train_bwd_partials.argtypes = [i32]
        L.aac_attn_train_bwd_partials.restype = i32
        L.aac_adam_flat_at.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, f32, vp, i32, vp]
        L.aac_adam_flat_at_scaled.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, f32, vp, i32, f32, vp]
        _L = L
    return _L


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().aac_fused_last_error().decode(errors='replace')}")


def _stream():
    return vp(torch.cuda.current_stream().cuda_stream)


def ptr(t, off=0):
    """Device address of element ``off`` of tensor ``t`` (fp32 / int32 elements)."""
    return None if t is None else t.data_ptr() + 4 * off


def prob(A, B, C, M, N, K, lda, ldb, ldc, ta=0, tb=0, bias=None, act=NONE, addend=None, ldadd=0, mask=None,
         ldmask=0, mact=NONE, ones=0, cextra=None, ksplit=1, split_stride=0, dvec=None, C2=None, dscale=0.0):
    """C[M][N] = mact(act(op(A) op(B) + addend + bias)); pointers are ints (see ``ptr``).  With C2:
    also C2[m][n] = C[m][n] > 0 ? dscale * dvec[n] : 0 (the actor-loss critic head's dh)."""
    return GemmProb(A, B, C, bias, addend, mask, cextra, split_stride, M, N + ones, K, lda, ldb, ldc, ldadd, ldmask,
                    ta, tb, act, mact, ones, ksplit, dvec, C2, dscale)


# weight gradients whose real output width fills whole tiles take their bias gradient (the virtual
# ones column, which would cost a tile column of its own for one real column) as a separate M x 1
# product against a ones vector: dWm 4 -> 3 column tiles, dWc 11 -> 10, dWa / dWq 9 -> 8 (round 6);
# AAC_BIAS_SPLIT=0 keeps the ones column
BIAS_SPLIT = os.environ.get("AAC_BIAS_SPLIT", "1") == "1"


def split_bias(p, ones_vec):
    """[p] or, for a weight-gradient product with a ones column whose real width is a multiple of 32
    (BIAS_SPLIT), [p without it, the bias gradient op(A) . ones as an M x 1 product into cextra] --
    the same sums, the bias's in another order."""
    nreal = p.N - p.ones
    if not (BIAS_SPLIT and p.ones and nreal % 32 == 0 and ones_vec is not None):
        return [p]
    w = GemmProb.from_buffer_copy(p)
    w.N, w.ones, w.cextra = nreal, 0, None
    b = GemmProb(p.A, ones_vec, p.cextra, None, None, None, None, p.split_stride, p.M, 1, p.K, p.lda, 1, 1, 0, 0,
                 p.ta, 0, NONE, NONE, 0, p.ksplit, None, None, 0.0)
    return [w, b]


def head_job(h, M, w, b, mode, y=None, rew=None, done=None, B=0, N=0, gamma=0.0, q=None, dq=None, dh=None,
             yout=None, chain=None):
    """aac_critic_head's arguments as a job for a grouped GEMM launch (``GemmLaunch(heads=...)``).
    chain (mode 2): (h2, w2, b2, q2, dq2, dh2, M2), the mse head of rows r < M2 of h2 on the TD target
    just computed for row r."""
    c = chain if chain is not None else (None, None, None, None, None, None, 0)
    return HeadJob(h, 256, M, w, b, mode, y, rew, done, B, N, gamma, q, dq, dh, yout, *c)


class Collective:
    """A cross-rank exchange in a launch list (the gradient all-reduce): the graph is cut there."""

    def __init__(self, fn):
        self.fn = fn

    def __call__(self):
        self.fn()


class GemmLaunch:
    """One aac_gemm_batch launch with a fixed problem list (validated when built), plus up to
    HEAD_MAX critic-head jobs that do not depend on the products (aac_gemm_batch_heads)."""

    def __init__(self, probs, heads=(), xcd=False):
        assert 0 <= len(probs) <= GEMM_MAX and len(heads) <= HEAD_MAX and len(probs) + len(heads) >= 1
        assert not (xcd and heads)
        self.n = len(probs)
        self.xcd = bool(xcd)        # XCD-aware workgroup order (aac_gemm_batch_ordered)
        self.arr = (GemmProb * max(self.n, 1))(*probs)
        self.nh = len(heads)
        self.heads = (HeadJob * self.nh)(*heads) if heads else None
        # algorithmic FLOPs (2 M N K per product; the virtual ones column is the bias gradient; a head
        # job's 256-wide dot per row)
        self.flops = sum(2.0 * p.M * p.N * p.K for p in probs) + sum(2.0 * 256 * (h.M + h.M2) for h in heads)
        # algorithmic HBM bytes: every operand read once, every output (each split-K copy) written once
        self.bytes = sum(4.0 * (p.M * p.K + p.K * (p.N - p.ones) + max(1, p.ksplit) * p.M * p.N
                                + (p.M * p.N if p.addend else 0) + (p.M * (p.N - p.ones) if p.mask else 0)
                                + (p.N if p.bias else 0) + (p.M * p.N if p.C2 else 0)) for p in probs)
        # head job: h read, dh written (modes 0 / 1)
        self.bytes += sum(4.0 * 256 * (h.M * (1 if h.mode == 2 else 2) + 2 * h.M2) for h in heads)

    def __call__(self):
        if self.nh:
            _chk(lib().aac_gemm_batch_heads(self.arr, self.n, self.heads, self.nh, _stream()), "aac_gemm_batch_heads")
        elif self.xcd:
            _chk(lib().aac_gemm_batch_ordered(self.arr, self.n, 1, _stream()), "aac_gemm_batch_ordered")
        else:
            _chk(lib().aac_gemm_batch(self.arr, self.n, _stream()), "aac_gemm_batch")

    def plan(self):
        """(per-product tile mode: 0 register fragments / 1 + cfg LDS workgroup tile, grid size)."""
        if self.n == 0:
            return [], 0
        cfg = (ctypes.c_int32 * self.n)()
        wg = ctypes.c_int32()
        _chk(lib().aac_gemm_plan(self.arr, self.n, cfg, ctypes.byref(wg)), "aac_gemm_plan")
        return list(cfg), wg.value


class AttnEnc:
    """One aac_attn_enc_fwd launch over one or two independent argument sets (AttnEncArgs), with an
    optional critic-head job (HeadJob, no chained head) as extra workgroups (aac_attn_enc_fwd_head)."""

    def __init__(self, *sets, head=None):
        assert 1 <= len(sets) <= 2
        self.n = len(sets)
        self.arr = (AttnEncArgs * self.n)(*sets)
        self.head = head
        self.flops, self.bytes = 0.0, 0.0
        for a in sets:
            f, b = attn_enc_cost(a)
            self.flops += f
            self.bytes += b
        if head is not None:
            self.flops += 2.0 * 256 * head.M
            self.bytes += 4.0 * 256 * head.M * (1 if head.mode == 2 else 2)

    def __call__(self):
        h = ctypes.byref(self.head) if self.head is not None else None
        _chk(lib().aac_attn_enc_fwd_head(self.arr, self.n, h, _stream()), "aac_attn_enc_fwd_head")


_RIDE = ("cx", "cx_ld", "c_din", "cW", "cb", "cf", "c_rows", "c_n", "o_h", "o_w", "o_b", "o_x", "o_d0")


def attn_enc_cost(a):
    """Algorithmic (FLOPs, HBM bytes) of one aac_attn_enc_fwd argument set (ActorNetwork_ATT_TwoPortion
    forward, ATT/nets:194-210, over R rows; riding critic encoders ATT/nets:697-701).  Per attention
    row: the encoders 2*64*(d_own + 18 + 6K), q, Wk^T q and Wv xb 3 * 2*64*64, scores and the alpha
    sum 2 * 2*64*K; bytes: own / radar / nei rows read, cat row written (training: x_j, q, qk, xb,
    alpha kept).  Per riding row (sample, agent): 2*128*c_din (+ the folded 256 -> 2 output layer,
    2*2*256, reading the 256-wide actor row)."""
    R, K = int(a.R), int(a.K)
    f = R * (2.0 * 64 * (a.d_own + 18 + 6 * K) + 3 * 2.0 * 64 * 64 + 2 * 2.0 * 64 * K)
    b = 4.0 * R * (a.d_own + 18 + 6 * K + 192)
    if a.xn:
        b += 4.0 * R * (64 * K + 3 * 64 + K)
    rows = int(a.c_rows) * int(a.c_n)
    if rows:
        f += rows * 2.0 * 128 * a.c_din
        b += 4.0 * rows * (a.c_din + 128)
        if a.o_h:
            f += rows * 2.0 * 2 * 256
            b += 4.0 * rows * 256
    return f, b


class AttnBwd:
    """One attention-backward launch (aac_attn_train_bwd[_wn]) of the actor step, with its algorithmic
    cost.  Per row (ATT/nets:194-210 backward): dxb = Wv^T dv, dq = Wk dqk and Wq^T dq 3 * 2*64*64;
    the softmax backward and dqk 8*64*K; the neighbour encoder's dWn partials 2*7*64*K.  Bytes: dv, qk,
    e_o, dcat_o, x_j, alpha, nei read; dqk, dq, de_o written (+ the partial dWn rows)."""

    def __init__(self, fn, R, K, partial_rows=0):
        self.fn, self.R, self.K = fn, R, K
        self.flops = R * (3 * 2.0 * 64 * 64 + 8.0 * 64 * K + 14.0 * 64 * K)
        self.bytes = 4.0 * R * (4 * 64 + 64 * K + K + 6 * K + 3 * 64) + 4.0 * 448 * partial_rows

    def __call__(self):
        self.fn()


def attn_set(ap, own, ld_own, d_own, radar, nei, R, K, cat, acts=None, ride=None):
    """Argument set of the actor's encoders + attention over R rows (ATT/nets:194-210): e_o, e_g and
    v_att land in cat[r][0:192]; with ``acts`` (ActorActs) the backward's x_j, q, qk, alpha, xb are
    kept.  ``ride``: the critic-encoder job (``critic_enc_ride``) sharing the launch."""
    a = AttnEncArgs()
    a.own, a.ld_own, a.d_own, a.radar, a.ld_radar, a.nei = own, ld_own, d_own, radar, 18, nei
    a.Wo, a.bo, a.Wg, a.bg, a.Wn, a.bn = ap.Wo, ap.bo, ap.Wg, ap.bg, ap.Wn, ap.bn
    a.Wq, a.Wk, a.Wv = ap.Wq, ap.Wkv, ap.Wkv + 4 * 64 * 64
    a.cat, a.ld_cat, a.R, a.K = cat, 192, R, K
    if acts is not None:
        a.xn, a.q, a.qk, a.alpha, a.xb = ptr(acts.xn), ptr(acts.qa), ptr(acts.qk), ptr(acts.alpha), ptr(acts.xb)
    return with_ride(a, ride)


def with_ride(a, ride):
    """A copy of argument set ``a`` carrying the riding critic-encoder job ``ride`` (or none)."""
    b = AttnEncArgs.from_buffer_copy(a)
    for k in _RIDE:
        setattr(b, k, 0 if ride is None else ride[k])
    return b


def critic_enc_ride(cp, X, rows, N, Din, f, fold=None):
    """The critic's per-agent encoders f[b][n*128:(n+1)*128] = relu(enc_n X[b][n]) (ATT/nets:697-701,
    R3) as a riding job of an aac_attn_enc_fwd launch (the per-agent weights are consecutive).
    ``fold`` = (ha, ap, d0): the actor's tanh output layer (ATT/nets:213) over the actor rows
    ha[b*N + n] is computed inside the job and its actions land in X[b][n][d0:d0+2] (no launch of
    its own)."""
    r = {"cx": X, "cx_ld": N * Din, "c_din": Din, "cW": cp.enc_w[0], "cb": cp.enc_b[0], "cf": ptr(f),
         "c_rows": rows, "c_n": N, "o_h": 0, "o_w": 0, "o_b": 0, "o_x": 0, "o_d0": 0}
    if fold is not None:
        ha, ap, d0 = fold
        r.update(o_h=ha, o_w=ap.Wa, o_b=ap.ba, o_x=X, o_d0=d0)
    return r


def ride_only(ride):
    """An argument set with no attention rows that runs only the riding critic-encoder job."""
    return with_ride(AttnEncArgs(), ride)


def set_lds_policy(min_workgroups=256, small_tiles=False):
    """Tile policy of the plans built from now on (include/aac_fused.h aac_gemm_set_lds_policy)."""
    lib().aac_gemm_set_lds_policy(int(min_workgroups), int(bool(small_tiles)))


def gemm_launches(probs, heads=(), xcd=False):
    """Split a product list into launches of at most GEMM_MAX (head jobs ride in the first)."""
    if not probs:
        return [GemmLaunch([], heads)] if heads else []
    return [GemmLaunch(probs[i:i + GEMM_MAX], heads if i == 0 else (), xcd=xcd) for i in range(0, len(probs), GEMM_MAX)]


def critic_head(h, M, w, b, mode, y=None, rew=None, done=None, B=0, N=0, gamma=0.0, q=None, dq=None, dh=None,
                yout=None):
    _chk(lib().aac_critic_head(vp(h), 256, M, vp(w), vp(b), mode, vp(y) if y else None, vp(rew) if rew else None,
                               vp(done) if done else None, B, N, gamma, vp(q) if q else None,
                               vp(dq) if dq else None, vp(dh) if dh else None, vp(yout) if yout else None,
                               _stream()), "aac_critic_head")


def critic_head_job(job):
    """One HeadJob as its own launch (aac_critic_head_job; the chained TD + mse head)."""
    _chk(lib().aac_critic_head_job(ctypes.byref(job), _stream()), "aac_critic_head_job")


def gather_strided(ring, idx, dsts, widths, chunks, dstrides, dsts2=None):
    n = len(dsts)
    arr = (vp * n)(*dsts)
    arr2 = (vp * n)(*dsts2) if dsts2 is not None else None
    w = (i32 * n)(*widths)
    c = (i32 * n)(*chunks)
    d = (i32 * n)(*dstrides)
    _chk(lib().aac_replay_gather_strided(vp(ring.data_ptr()), ring.shape[1], vp(idx.data_ptr()), idx.numel(), n,
                                         arr, arr2, w, c, d, _stream()), "aac_replay_gather_strided")


def adam_sum(opt, gpart, nsplit, step_add, grad_out=None):
    """Adam step whose gradient is the sum of ``nsplit`` partial copies in ``gpart`` ([nsplit][stride],
    stride >= the parameter count)."""
    _chk(lib().aac_adam_flat_sum_strided(vp(opt.flat.data.data_ptr()), vp(gpart.data_ptr()), nsplit, gpart.shape[-1],
                                         vp(grad_out.data_ptr()) if grad_out is not None else None,
                                         vp(opt.exp_avg.data_ptr()), vp(opt.exp_avg_sq.data_ptr()),
                                         opt.flat.data.numel(), opt.lr, opt.betas[0], opt.betas[1], opt.eps,
                                         vp(opt.step_t.data_ptr()), step_add, _stream()), "aac_adam_flat_sum")


class AdamJob(ctypes.Structure):
    _fields_ = [("param", vp), ("gpart", vp), ("nsplit", i32), ("gstride", i64), ("grad_out", vp), ("exp_avg", vp),
                ("exp_avg_sq", vp), ("n", i64), ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32),
                ("step", vp), ("step_add", i32)]


def _adam_job(opt, gpart, nsplit, step_add, grad_out):
    return AdamJob(vp(opt.flat.data.data_ptr()), vp(gpart.data_ptr()), nsplit, gpart.shape[-1],
                   vp(grad_out.data_ptr()) if grad_out is not None else None, vp(opt.exp_avg.data_ptr()),
                   vp(opt.exp_avg_sq.data_ptr()), opt.flat.data.numel(), opt.lr, opt.betas[0], opt.betas[1], opt.eps,
                   vp(opt.step_t.data_ptr()), step_add)


def adam_pair_ok(*gparts):
    """aac_adam_flat_sum_pair's conditions: the copy-parallel Adam (AAC_ADAM4) over >= 2 copies at
    a 16-B aligned stride."""
    return os.environ.get("AAC_ADAM4", "1") != "0" and all(
        g.shape[0] >= 2 and g.shape[-1] % 4 == 0 and g.data_ptr() % 16 == 0 for g in gparts)


def adam_sum_pair(a, b):
    """Two networks' adam_sum steps in one launch; a, b = (opt, gpart, nsplit, step_add, grad_out)."""
    ja, jb = _adam_job(*a), _adam_job(*b)
    _chk(lib().aac_adam_flat_sum_pair(ctypes.byref(ja), ctypes.byref(jb), _stream()), "aac_adam_flat_sum_pair")


def sum_partials(out, gpart, nsplit):
    _chk(lib().aac_sum_partials_strided(vp(out.data_ptr()), vp(gpart.data_ptr()), nsplit, gpart.shape[-1],
                                        out.numel(), _stream()), "aac_sum_partials")


def padded(n, q=4):
    """The copy stride of split-K partial gradients: a multiple of 4 floats (16-B aligned copies)."""
    return (n + q - 1) // q * q


def adam_at(opt, step_add, gscale=1.0):
    """Adam step ``step_t + step_add`` on ``gscale`` x the flat gradient (1 / world after a SUM
    all-reduce)."""
    _chk(lib().aac_adam_flat_at_scaled(vp(opt.flat.data.data_ptr()), vp(opt.flat.grad.data_ptr()),
                                       vp(opt.exp_avg.data_ptr()), vp(opt.exp_avg_sq.data_ptr()),
                                       opt.flat.data.numel(), opt.lr, opt.betas[0], opt.betas[1], opt.eps,
                                       vp(opt.step_t.data_ptr()), step_add, gscale, _stream()),
         "aac_adam_flat_at_scaled")


class DcombAob:
    """One aac_actor_dcomb_out_bwd launch: the actor step's critic data gradient df = (dh Wc) * (f > 0)
    reduced straight into the actor's output-layer backward (dout, dha), plus an optional critic-head
    job riding along.  Algorithmic cost: 2 B (128 N) 256 FLOPs for df, 2*2*128 per actor row for da and
    2*2*256 for dha; bytes: dh, Wc, f, the encoder action columns, ha read; dout, dha written."""

    def __init__(self, a, head=None):
        self.a = a
        self.head = head
        B, N = int(a.B), int(a.N)
        self.flops = 2.0 * B * 128 * N * 256 + B * N * (4.0 * 128 + 4.0 * 256)
        self.bytes = 4.0 * (B * 256 + 256 * 128 * N + B * 128 * N + 2 * 128 * N + B * N * (2 + 256 + 2 + 256))
        if head is not None:
            self.flops += 2.0 * 256 * head.M
            self.bytes += 4.0 * 256 * head.M * (1 if head.mode == 2 else 2)

    def __call__(self):
        h = ctypes.byref(self.head) if self.head is not None else None
        _chk(lib().aac_actor_dcomb_out_bwd(ctypes.byref(self.a), h, _stream()), "aac_actor_dcomb_out_bwd")


def actor_out_bwd(df, ldf, wenc, din, d0, X, wa, ha, N, R, dout, dha):
    _chk(lib().aac_actor_out_bwd(vp(df), ldf, vp(wenc), din, d0, vp(X), vp(wa), vp(ha), N, R, vp(dout), vp(dha),
                                 _stream()), "aac_actor_out_bwd")


def attn_train_fwd(eo, lde, xn, nei, Wq, Wk, Wv, q, qk, alpha, xb, vout, ldv, R, K):
    _chk(lib().aac_attn_train_fwd(vp(eo), lde, vp(xn), vp(nei), vp(Wq), vp(Wk), vp(Wv), vp(q), vp(qk), vp(alpha),
                                  vp(xb), vp(vout), ldv, R, K, _stream()), "aac_attn_train_fwd")


def attn_train_bwd(dv, lddv, xn, alpha, qk, eo, lde, dcat_o, ldd, Wq, Wk, Wv, dxn, dqk, dq, deo, R, K):
    _chk(lib().aac_attn_train_bwd(vp(dv), lddv, vp(xn), vp(alpha), vp(qk), vp(eo), lde, vp(dcat_o), ldd, vp(Wq),
                                  vp(Wk), vp(Wv), vp(dxn), vp(dqk), vp(dq), vp(deo), R, K, _stream()),
         "aac_attn_train_bwd")


def attn_train_bwd_wn(dv, lddv, xn, alpha, qk, eo, lde, dcat_o, ldd, Wq, Wk, Wv, dqk, dq, deo, R, K, nei, pwn):
    """aac_attn_train_bwd_wn: the attention backward with the neighbour encoder's weight-gradient
    partials (pwn rows) instead of the d x_j rows."""
    _chk(lib().aac_attn_train_bwd_wn(vp(dv), lddv, vp(xn), vp(alpha), vp(qk), vp(eo), lde, vp(dcat_o), ldd, vp(Wq),
                                     vp(Wk), vp(Wv), None, vp(dqk), vp(dq), vp(deo), R, K, vp(nei), vp(pwn),
                                     _stream()), "aac_attn_train_bwd_wn")


def attn_bwd_partials(R):
    return int(lib().aac_attn_train_bwd_partials(R))


def attn_block(eo, lde, nei, Wn, bn, Wqk, Wv, out, ldo, R, K):
    _chk(lib().aac_attn_block(vp(eo), lde, vp(nei), vp(Wn), vp(bn), vp(Wqk), vp(Wv), vp(out), ldo, R, K, _stream()),
         "aac_attn_block")


# =============================================================================== networks
def _addr(flat, gbase):
    """Parameter -> address: its own storage, or the same offset inside another flat buffer."""
    if gbase is None:
        return lambda p, o=0: ptr(p, o)
    base = flat.data.data_ptr()
    return lambda p, o=0: gbase + (p.data_ptr() - base) + 4 * o


class ActorParams:
    """Device addresses of ActorNetwork_ATT_TwoPortion's weights (or of the same offsets in a
    gradient-partial buffer when ``gbase`` is given)."""

    def __init__(self, a, flat=None, gbase=None):
        g = _addr(flat, gbase)
        self.Wo, self.bo = g(a.own_fc[0].weight), g(a.own_fc[0].bias)
        self.Wg, self.bg = g(a.own_grid[0].weight), g(a.own_grid[0].bias)
        self.Wn, self.bn = g(a.neigh_fc[0].weight), g(a.neigh_fc[0].bias)
        self.Wm, self.bm = g(a.merge_feature[0].weight), g(a.merge_feature[0].bias)
        self.Wa, self.ba = g(a.act_out[0].weight), g(a.act_out[0].bias)
        self.Wq, self.Wkv = g(a.q.weight), g(a.kv_weight)


class CriticParams:
    def __init__(self, c, flat=None, gbase=None):
        g = _addr(flat, gbase)
        N, H, Din = c.enc_w.shape
        self.enc_w = [g(c.enc_w, n * H * Din) for n in range(N)]
        self.enc_b = [g(c.enc_b, n * H) for n in range(N)]
        self.Wc, self.bc = g(c.combine_agents_fea[0].weight), g(c.combine_agents_fea[0].bias)
        self.Wq, self.bq = g(c.out_feature_q[0].weight), g(c.out_feature_q[0].bias)


class ActorActs:
    """Activations of one actor forward over R rows (kept for the backward)."""

    def __init__(self, R, K, dev):
        z = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)   # noqa: E731
        self.R, self.K = R, K
        self.cat = z(R, 192)          # [e_o | e_g | v_att]
        self.xn = z(R * K, 64)        # neighbour features x_j
        self.qa = z(R, 64)            # q = Wq e_o
        self.qk = z(R, 64)            # Wk^T q
        self.xb = z(R, 64)            # sum_j alpha_j x_j
        self.alpha = z(R, max(K, 1))
        self.ha = z(R, 256)


def actor_forward_stages(ap, acts, own, ld_own, radar, nei, R, K, D0, out, ld_out):
    """ActorNetwork_ATT_TwoPortion.forward (ATT/nets:194-213) over R rows as dependent stages
    [encoders + attention (AttnEncArgs set of aac_attn_enc_fwd: e_o, e_g, x_j, q, Wk^T q, masked
    softmax, Wv sum a x), merge, out]; GEMM stages are product lists and the attention set can carry
    a riding job, so they share launches with independent work.  The tanh actions land at ``out``
    (row stride ``ld_out``, e.g. the critic-input rows)."""
    c = acts
    attn = attn_set(ap, own, ld_own, D0, radar, nei, R, K, ptr(c.cat), acts=c)
    merge = [prob(ptr(c.cat), ap.Wm, ptr(c.ha), R, 256, 192, 192, 192, 256, tb=1, bias=ap.bm, act=RELU)]
    outp = [prob(ptr(c.ha), ap.Wa, out, R, 2, 256, 256, 256, ld_out, tb=1, bias=ap.ba, act=TANH)]
    return attn, merge, outp


def actor_forward(ap, acts, own, ld_own, radar, nei, R, K, D0, out, ld_out):
    """Launch list of the training actor forward (activations kept for the backward)."""
    attn, merge, outp = actor_forward_stages(ap, acts, own, ld_own, radar, nei, R, K, D0, out, ld_out)
    return [AttnEnc(attn)] + gemm_launches(merge) + gemm_launches(outp)


class ActorInferActs:
    """Buffers of the inference (no-backward) actor forward over R rows."""

    def __init__(self, R, dev):
        self.R = R
        self.cat = torch.empty(R, 192, dtype=torch.float32, device=dev)
        self.ha = torch.empty(R, 256, dtype=torch.float32, device=dev)


def actor_infer_stages(ap, acts, own, ld_own, radar, nei, R, K, D0, out, ld_out):
    """ActorNetwork_ATT_TwoPortion.forward for inference as dependent stages [encoders + attention
    (AttnEncArgs set, nothing kept for a backward), merge, out]; GEMM stages are product lists so
    that independent work can share their launches."""
    c = acts
    attn = attn_set(ap, own, ld_own, D0, radar, nei, R, K, ptr(c.cat))
    merge = [prob(ptr(c.cat), ap.Wm, ptr(c.ha), R, 256, 192, 192, 192, 256, tb=1, bias=ap.bm, act=RELU)]
    outp = [prob(ptr(c.ha), ap.Wa, out, R, 2, 256, 256, 256, ld_out, tb=1, bias=ap.ba, act=TANH)]
    return attn, merge, outp


def actor_forward_infer(ap, acts, own, ld_own, radar, nei, R, K, D0, out, ld_out):
    """Inference launch list of ActorNetwork_ATT_TwoPortion.forward: encoders + attention in one
    aac_attn_enc_fwd launch, merge, out."""
    attn, merge, outp = actor_infer_stages(ap, acts, own, ld_own, radar, nei, R, K, D0, out, ld_out)
    return [AttnEnc(attn)] + gemm_launches(merge) + gemm_launches(outp)


def critic_forward_stages(cp, X, rows, N, Din, f, h):
    """Encoders + combine of CriticCombine (ATT/nets:672-724, R3) over ``rows`` samples whose
    inputs are the rows X[b][n][:Din] = [own_n | a_n], as two product lists."""
    enc = [prob(X + 4 * n * Din, cp.enc_w[n], ptr(f, n * 128), rows, 128, Din, N * Din, Din, 128 * N, tb=1,
                bias=cp.enc_b[n], act=RELU) for n in range(N)]
    comb = [prob(ptr(f), cp.Wc, ptr(h), rows, 256, 128 * N, 128 * N, 128 * N, 256, tb=1, bias=cp.bc, act=RELU)]
    return enc, comb


def critic_forward(cp, X, rows, N, Din, f, h):
    enc, comb = critic_forward_stages(cp, X, rows, N, Din, f, h)
    return gemm_launches(enc) + gemm_launches(comb)


# the act path's merge + output layer (+ noise) as one weights-stationary launch (aac_actor_head_ws)
# instead of a grouped-GEMM launch + aac_actor_out_noise (config 3: 32.6 us against 26.2 + 10.2 us);
# AAC_ACT_HEAD_WS=0 keeps the two launches
ACT_HEAD_WS = os.environ.get("AAC_ACT_HEAD_WS", "1") == "1"


class ActorInfer:
    """Batched choose_action forward (ATT/maddpg:455-550) of one actor over E*N rows, as a cached
    launch list per input buffer set."""

    def __init__(self, actor, N, D0, dev):
        self.ap = ActorParams(actor)
        self.N, self.D0, self.K, self.dev = N, D0, N - 1, dev
        self.plans = {}

    def __call__(self, own, radar, nei, noise=None):
        """tanh actions [R][2]; with ``noise`` = (episode, eps_end, noise_start, noise_end, seed,
        counter, noise_out) the output layer, the exploration noise and the clamp run as one
        aac_actor_out_noise launch instead of a grouped-GEMM launch + aac_noise_clamp."""
        R = own.numel() // self.D0
        key = (own.data_ptr(), radar.data_ptr(), nei.data_ptr(), R)
        if key not in self.plans:
            for t in (own, radar, nei):
                assert t.is_contiguous() and t.device == self.dev and t.dtype == torch.float32
            acts = ActorInferActs(R, self.dev)
            out = torch.empty(R, 2, dtype=torch.float32, device=self.dev)
            attn, merge, outp = actor_infer_stages(self.ap, acts, ptr(own), self.D0, ptr(radar), ptr(nei), R,
                                                   self.K, self.D0, ptr(out), 2)
            L = [AttnEnc(attn)] + ([] if ACT_HEAD_WS else gemm_launches(merge))
            self.plans[key] = (L, gemm_launches(outp), acts, out, (own, radar, nei))
        L, Lout, acts, out, _ = self.plans[key]
        for op in L:
            op()
        ap = self.ap
        if ACT_HEAD_WS:
            # merge + output layer (+ noise) in one weights-stationary launch (aac_actor_head_ws)
            if noise is None:
                ops.actor_head_ws(acts.cat, ap.Wm, ap.bm, ap.Wa, ap.ba, out, self.N, noisy=False)
            else:
                episode, eps_end, noise_start, noise_end, seed, counter, noise_out = noise
                ops.actor_head_ws(acts.cat, ap.Wm, ap.bm, ap.Wa, ap.ba, out, self.N, episode, eps_end, noise_start,
                                  noise_end, seed, counter, noise_out)
        elif noise is None:
            for op in Lout:
                op()
        else:
            episode, eps_end, noise_start, noise_end, seed, counter, noise_out = noise
            ops.actor_out_noise(acts.ha, self.ap.Wa, self.ap.ba, out, self.N, episode, eps_end, noise_start,
                                noise_end, seed, counter, noise_out)
        return out


class FusedUpdate:
    """One update_myown-equivalent on a DeviceReplay as a fixed launch list (graph-capturable)."""

    # K splits of the weight gradients (partial copies summed by the Adam kernel); actor K = B*N
    # or B*N*K rows, critic K = B rows.  AAC_SPLIT_ACTOR / AAC_SPLIT_CRITIC override (tuning).
    SPLIT_ACTOR = int(os.environ.get("AAC_SPLIT_ACTOR", "20"))
    SPLIT_CRITIC = int(os.environ.get("AAC_SPLIT_CRITIC", "4"))
    # the merge layer's weight gradient dWm | dbm (256 x 192 + 1 over K = B N) takes fewer split copies
    # than the actor's others: its LDS tiles then fill one round of the launch (the copies past it stay
    # zero); tools/mb_split.py, round 6
    SPLIT_DWM = int(os.environ.get("AAC_SPLIT_DWM", "10"))
    # world == 1: run the critic step of iteration i+1 beside the actor step of iteration i on a
    # second stream of the captured graph (AAC_OVERLAP=1; measured slower, off: DESIGN section 4)
    OVERLAP = os.environ.get("AAC_OVERLAP", "0") == "1"
    # world == 1: the same independence used to merge launches instead -- the critic step of
    # iteration i+1 zipped stage by stage with the actor forward + step of iteration i in shared
    # grouped-GEMM launches, both Adam steps in one launch (AAC_MERGED=0: the serial order)
    MERGED = os.environ.get("AAC_MERGED", "1") == "1"
    # the actor step's critic data gradient + actor output backward as one launch (DcombAob) instead of
    # a grouped-GEMM product and actor_out_bwd; AAC_DAOB=0 restores the two launches
    DAOB = os.environ.get("AAC_DAOB", "1") == "1"
    def __init__(self, model, replay, B):
        self.m, self.rep, self.B = model, replay, B
        N, D0, K = model.n_agents, model.D0, model.n_agents - 1
        self.N, self.D0, self.K, self.Din = N, D0, K, D0 + 2
        dev = model.device
        self.dev = dev
        nb = N
        self.nb = nb
        z = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)   # noqa: E731
        Bt = nb * B
        # gathered batches (all N iterations), critic-input rows [own | a] and [own' | a']
        self.idx = torch.empty(Bt, dtype=torch.int32, device=dev)
        self.X = z(Bt, N, self.Din)      # [own | replay action]   (critic step)
        self.X2 = z(Bt, N, self.Din)     # [own | policy action]   (actor step)
        self.Xt = z(Bt, N, self.Din)     # [own' | target action]  (TD target)
        self.radar, self.nei = z(Bt, N, 18), z(Bt, N, K, 6)
        self.nradar, self.nnei = z(Bt, N, 18), z(Bt, N, K, 6)
        self.rew, self.done = z(Bt, N), z(Bt, N)
        self.y = z(Bt)
        self.qn = z(Bt)                              # target critic Q' of every TD row (records)
        self.q_c, self.q_a = z(Bt), z(Bt)            # per-iteration Q (stats)
        # activations / gradients
        self.acts_t = ActorInferActs(Bt * N, dev)    # target actor over all batches
        self.acts = ActorActs(B * N, K, dev)
        self.f_t, self.h_t = z(Bt, 128 * N), z(Bt, 256)
        self.f, self.h = z(B, 128 * N), z(B, 256)
        self.dq, self.dh, self.df = z(B), z(B, 256), z(B, 128 * N)
        # critic-step activation sets [f, h, dq, dh, df]: [0] is shared with the actor step; world > 1
        # runs the critic step of iteration i+1 beside the actor step of i, in set [1]
        self.cbuf = [(self.f, self.h, self.dq, self.dh, self.df)]
        if model.world > 1 or self.OVERLAP or self.MERGED:
            self.cbuf.append((z(B, 128 * N), z(B, 256), z(B), z(B, 256), z(B, 128 * N)))
        R = B * N
        self.dout, self.dha = z(R, 2), z(R, 256)
        self.dcat_o, self.dcat_g, self.dv = z(R, 64), z(R, 64), z(R, 64)
        self.dqa, self.dqk, self.deo, self.dxn = z(R, 64), z(R, 64), z(R, 64), z(R * K, 64)
        # K <= 8: the attention backward accumulates dWn | dbn per workgroup (pwn rows, zero rows up to
        # the split count); a [1 x P] x [P x 448] product sums them into the split copies
        self.wn_part = K <= 8 and os.environ.get("AAC_ATTN_WN", "1") == "1"
        if self.wn_part:
            P = max(attn_bwd_partials(R), self.SPLIT_ACTOR)
            self.pwn = torch.zeros(P, 448, device=dev)
            self.ones_p = torch.ones(P, device=dev)
        # the bias gradients' ones vector (split_bias; K <= B N rows)
        self.ones_k = torch.ones(max(B * N, B), device=dev)
        # weight-gradient partial copies (summed by the Adam kernel)
        self.ga = torch.zeros(self.SPLIT_ACTOR, padded(model.fa.numel), device=dev)
        self.gc = torch.zeros(self.SPLIT_CRITIC, padded(model.fc.numel), device=dev)
        self._build()

    # ------------------------------------------------------------------ plan
    def _build(self):
        m, B, N, D0, K, Din, nb = self.m, self.B, self.N, self.D0, self.K, self.Din, self.nb
        A, At = ActorParams(m.actors), ActorParams(m.actors_target)
        C, Ct = CriticParams(m.critics), CriticParams(m.critics_target)
        rep = self.rep
        self.pre = []      # sample + gather + targets
        self.pre.append(lambda: ops.replay_sample(rep.meta, B, rep.seed, rep.counter, self.idx))
        w = rep.widths
        dsts = [ptr(self.X), ptr(self.radar), ptr(self.nei), ptr(self.X, D0), ptr(self.rew), ptr(self.done),
                ptr(self.Xt), ptr(self.nradar), ptr(self.nnei)]
        chunks = [D0, w[1], w[2], 2, w[4], w[5], D0, w[7], w[8]]
        strides = [Din, w[1], w[2], Din, w[4], w[5], Din, w[7], w[8]]
        dsts2 = [ptr(self.X2)] + [None] * 8
        self.pre.append(lambda: gather_strided(rep.ring, self.idx, dsts, w, chunks, strides, dsts2=dsts2))
        Bt = nb * B
        # the target actor's output layer is folded into the target critic's encoder job (its actions
        # land in Xt's action columns there)
        t_attn, t_merge, _ = actor_infer_stages(At, self.acts_t, ptr(self.Xt), Din, ptr(self.nradar),
                                                ptr(self.nnei), Bt * N, K, D0, ptr(self.Xt, D0), Din)
        _, t_comb = critic_forward_stages(Ct, ptr(self.Xt), Bt, N, Din, self.f_t, self.h_t)
        t_cenc = critic_enc_ride(Ct, ptr(self.Xt), Bt, N, Din, self.f_t, fold=(ptr(self.acts_t.ha), At, D0))
        t_head = lambda: critic_head(ptr(self.h_t), Bt, Ct.Wq, Ct.bq, 2, rew=ptr(self.rew),  # noqa: E731
                                     done=ptr(self.done), B=B, N=N, gamma=m.GAMMA, q=ptr(self.qn), yout=ptr(self.y))
        self.segs = None
        zip0 = not self.OVERLAP and self.MERGED
        if zip0:
            # the TD-target chain reads only the target networks and the gathered batches: the critic
            # step 0's forward and the actor forward 0 (current weights, their own buffers) share its
            # launches up to the point where the critic step needs the targets y
            cs0 = self._critic_stages(0, C, self.cbuf[1])
            a0_attn, a0_merge = self._actor_fwd_stages(0, A)
            self.pre += [AttnEnc(with_ride(t_attn, cs0["enc"]), a0_attn)]
            self.pre += gemm_launches(t_merge + cs0["comb"] + a0_merge)
            # the TD target of all batches with critic step 0's mse head chained on batch 0's rows
            f0, h0, dq0, dh0, _ = self.cbuf[1]
            tjob = head_job(ptr(self.h_t), Bt, Ct.Wq, Ct.bq, 2, rew=ptr(self.rew), done=ptr(self.done), B=B, N=N,
                            gamma=m.GAMMA, q=ptr(self.qn), yout=ptr(self.y),
                            chain=(ptr(h0), C.Wq, C.bq, ptr(self.q_c), ptr(dq0), ptr(dh0), B))
            self.pre += [AttnEnc(ride_only(t_cenc))] + gemm_launches(t_comb) + [lambda: critic_head_job(tjob)]
        else:
            self.pre += [AttnEnc(t_attn)] + gemm_launches(t_merge)
            self.pre += [AttnEnc(ride_only(t_cenc))] + gemm_launches(t_comb) + [t_head]
        if m.world > 1 and not zip0:
            self.iters = self._pipelined(A, C)
        elif self.OVERLAP:
            self.segs = self._overlapped(A, C)
            self.iters = [a + b + j for a, b, j in self.segs]
        elif self.MERGED:
            self.iters = self._merged(A, C, cs0)
        else:
            self.iters = [self._critic_step(i, A, C, self.cbuf[0], fuse_actor_fwd=True)
                          + self._adam(m.critic_optimizer, m.fc, self.gc, self.SPLIT_CRITIC, i + 1)
                          + self._actor_step(i, A, C)
                          + self._adam(m.actor_optimizer, m.fa, self.ga, self.SPLIT_ACTOR, i + 1)
                          for i in range(N)]
        # the Polyak launches also advance the optimisers' step counters (no separate add kernels)
        self.post = [lambda: ops.polyak_flat2(m.fc_t.data, m.fc.data, m.critic_optimizer.step_t, m.fa_t.data,
                                              m.fa.data, m.actor_optimizer.step_t, m.tau, N)]
        # an update without the soft update (i_episode % UPDATE_EVERY != 0, ATT/maddpg:436-438): the same
        # launch with tau = 0 (targets kept bit-exactly: 1 * t + 0 * s) still advances the step counters
        self.post_hold = [lambda: ops.polyak_flat2(m.fc_t.data, m.fc.data, m.critic_optimizer.step_t, m.fa_t.data,
                                                   m.fa.data, m.actor_optimizer.step_t, 0.0, N)]
        self.n_launches = len(self.pre) + sum(len(it) for it in self.iters) + len(self.post)

    def _adam(self, opt, flat, gpart, ns, step_add):
        """world == 1: the Adam step sums the split-K partial copies itself.  world > 1: the partial
        copies are summed into the shared gradient buffer, all-reduced (SUM) and the Adam launch
        applies the 1 / world."""
        m = self.m
        if m.world == 1:
            return [lambda: adam_sum(opt, gpart, ns, step_add, grad_out=flat.grad)]
        critic = opt is m.critic_optimizer
        return [lambda: sum_partials(flat.grad, gpart, ns),
                Collective(lambda: m._allreduce_grads(critic=critic, actor=not critic)),
                lambda: adam_at(opt, step_add, 1.0 / m.world)]

    def _adam_pair(self, i_critic, i_actor):
        """Critic Adam step i_critic + 1 and actor Adam step i_actor + 1 as one launch (or two); at
        world > 1 behind ONE all-reduce of both gradients (contiguous in MADDPG._share_grads)."""
        m = self.m
        ca = (m.critic_optimizer, self.gc, self.SPLIT_CRITIC, i_critic + 1, m.fc.grad)
        aa = (m.actor_optimizer, self.ga, self.SPLIT_ACTOR, i_actor + 1, m.fa.grad)
        if m.world > 1:
            gs = 1.0 / m.world
            return [lambda: sum_partials(m.fa.grad, self.ga, self.SPLIT_ACTOR),
                    lambda: sum_partials(m.fc.grad, self.gc, self.SPLIT_CRITIC),
                    Collective(lambda: m._allreduce_grads(critic=True, actor=True)),
                    lambda: adam_at(ca[0], ca[3], gs), lambda: adam_at(aa[0], aa[3], gs)]
        if adam_pair_ok(self.gc, self.ga):
            return [lambda: adam_sum_pair(ca, aa)]
        return [lambda: adam_sum(*ca[:4], grad_out=ca[4]), lambda: adam_sum(*aa[:4], grad_out=aa[4])]

    def _merged(self, A, C, cs0):
        """Fewer, fuller launches.  The critic step of iteration i+1 reads the critic
        weights after critic Adam step i (and the fixed targets) -- exactly what the actor step of
        iteration i reads -- and neither reads the other's result (as in ``_pipelined``).  So
        segment i+1 zips the actor forward + actor step of iteration i with the critic step of
        iteration i+1 (activation set 1) stage by stage into shared grouped-GEMM launches (the
        critic head riding along as a head job) and ends with both Adam steps in one launch.  The
        forward half of critic step 0 and the actor forward 0 ran inside the TD-target launches
        (``pre``).  Every product's arithmetic is unchanged, so the update is bit-identical to the
        serial order (tests/test_fused_gpu.py).  At world > 1 each Adam boundary becomes partial sums +
        ONE all-reduce + the Adam launches (``_adam`` / ``_adam_pair``): the same N + 1 collectives as
        ``_pipelined`` with the merged launches between them (tests/test_parallel_gpu.py)."""
        m, N = self.m, self.N
        segs = [gemm_launches(cs0["grad"]) + gemm_launches(cs0["encw"])      # its head ran chained in pre
                + self._adam(m.critic_optimizer, m.fc, self.gc, self.SPLIT_CRITIC, 1)]
        for i in range(N):
            cs = self._critic_stages(i + 1, C, self.cbuf[1]) if i + 1 < N else None
            ac = self._actor_stages(i, A, C)
            L = []
            if i == 0 and cs is not None:
                # iteration 0's actor forward ran in pre: critic step 1 rides on the actor step's stages
                L += [AttnEnc(ride_only(ac["cenc"]), ride_only(cs["enc"]))] + gemm_launches(ac["ccomb"] + cs["comb"])
                if self.DAOB:
                    L.append(ac["daob"](cs["head_job"]))
                else:
                    L += gemm_launches(ac["dcomb"], heads=[cs["head_job"]])
                    L.append(ac["aob"])
                L += gemm_launches(ac["wgrad1"] + cs["grad"])
                L.append(ac["attn_bwd"])
                L += gemm_launches(ac["wgrad2"] + cs["encw"] + ac.get("qstat", []))
                L += self._adam_pair(i + 1, i)
                segs.append(L)
                continue
            if i > 0:
                a_attn, a_merge = self._actor_fwd_stages(i, A)
                if cs is None:
                    L += [AttnEnc(a_attn)] + gemm_launches(a_merge)
                else:
                    L += [AttnEnc(with_ride(a_attn, cs["enc"]))] + gemm_launches(a_merge + cs["comb"])
            # the actor's output layer runs inside the critic-encoder job on its actions; critic step
            # i+1's head rides along (it needs only that step's combine, done in the launch before)
            L.append(AttnEnc(ride_only(ac["cenc"]), head=cs["head_job"] if (cs is not None and i > 0) else None))
            if self.DAOB:
                # critic step i+1's encoder weight gradients and the Q statistics ride with the actor's
                # weight gradients (both only need to finish before the Adam launch)
                L += gemm_launches(ac["ccomb"] + (cs["grad"] if cs is not None else [])) + [ac["daob"]()]
                L += gemm_launches(ac["wgrad1"])
                L.append(ac["attn_bwd"])
                L += gemm_launches(ac["wgrad2"] + (cs["encw"] if cs is not None else []) + ac["qstat"])
            else:
                if cs is None:
                    L += gemm_launches(ac["ccomb"]) + gemm_launches(ac["dcomb"])
                else:
                    L += gemm_launches(ac["ccomb"] + cs["grad"]) + gemm_launches(ac["dcomb"] + cs["encw"])
                L.append(ac["aob"])
                L += gemm_launches(ac["wgrad1"])
                L.append(ac["attn_bwd"])
                L += gemm_launches(ac["wgrad2"])
            if cs is not None:
                L += self._adam_pair(i + 1, i)
            else:
                L += self._adam(m.actor_optimizer, m.fa, self.ga, self.SPLIT_ACTOR, i + 1)
            segs.append(L)
        return segs

    def _overlapped(self, A, C):
        """world == 1: the update as segments (branch A, branch B, join).  The critic step of
        iteration i+1 reads the critic weights after critic Adam step i (and the fixed targets),
        exactly what the actor step of iteration i reads, and neither reads the other's result, so
        branch B (critic step i+1, activation set 1) runs beside branch A (actor forward + actor step
        of iteration i, set 0) on a second stream of the captured graph; the join runs both Adam
        steps.  Every product's arithmetic is unchanged: bit-identical to the serial order."""
        m, N = self.m, self.N
        SA, SC = self.SPLIT_ACTOR, self.SPLIT_CRITIC
        copt, aopt = m.critic_optimizer, m.actor_optimizer
        segs = [([], self._critic_step(0, A, C, self.cbuf[1], fuse_actor_fwd=False),
                 self._adam(copt, m.fc, self.gc, SC, 1))]
        for i in range(N):
            a = self._actor_fwd_launches(i, A) + self._actor_step(i, A, C)
            b, j = [], []
            if i + 1 < N:
                b = self._critic_step(i + 1, A, C, self.cbuf[1], fuse_actor_fwd=False)
                j = self._adam(copt, m.fc, self.gc, SC, i + 2)
            j = j + self._adam(aopt, m.fa, self.ga, SA, i + 1)
            segs.append((a, b, j))
        return segs

    def run_streams(self, side):
        """The update with branch B of every segment on ``side`` (fork / join by stream waits):
        what the world == 1 graph captures.  Without segments: the serial launch list."""
        cur = torch.cuda.current_stream()
        if self.segs is None:
            for op in self.ops():
                op()
            return
        for op in self.pre:
            op()
        for a, b, j in self.segs:
            if b:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    for op in b:
                        op()
            for op in a:
                op()
            if b:
                cur.wait_stream(side)
            for op in j:
                op()
        for op in self.post:
            op()

    def _pipelined(self, A, C):
        """world > 1 with AAC_MERGED=0 (the merged schedules are the default at every world size):
        one gradient all-reduce per ``update_myown`` iteration boundary instead of two.

        The critic step of iteration i+1 reads the critic weights after critic Adam step i (and
        the fixed targets), exactly what the actor step of iteration i reads, and neither reads
        the other's result: so the two are computed in the same segment (separate activation
        buffers) and their gradients -- contiguous in the shared gradient buffer
        (MADDPG._share_grads) -- are averaged by ONE collective.  N + 1 all-reduces per update
        (6 at N = 5) instead of 2N; the arithmetic of every product is unchanged, so the result
        is bit-identical to the per-step order (tests/test_parallel_gpu.py)."""
        m, N = self.m, self.N
        SA, SC = self.SPLIT_ACTOR, self.SPLIT_CRITIC
        copt, aopt = m.critic_optimizer, m.actor_optimizer
        gs = 1.0 / m.world          # the collectives SUM; each Adam launch applies the 1 / world
        red_c = lambda: sum_partials(m.fc.grad, self.gc, SC)      # noqa: E731
        red_a = lambda: sum_partials(m.fa.grad, self.ga, SA)      # noqa: E731
        L = self._critic_step(0, A, C, self.cbuf[0], fuse_actor_fwd=False)
        L += [red_c, Collective(lambda: m._allreduce_grads(critic=True, actor=False)), lambda: adam_at(copt, 1, gs)]
        segs = [L]
        for i in range(N):
            L = self._actor_fwd_launches(i, A) + self._actor_step(i, A, C)
            if i + 1 < N:
                L += self._critic_step(i + 1, A, C, self.cbuf[1], fuse_actor_fwd=False)
                L += [red_a, red_c, Collective(lambda: m._allreduce_grads(critic=True, actor=True)),
                      lambda i=i: adam_at(copt, i + 2, gs), lambda i=i: adam_at(aopt, i + 1, gs)]
            else:
                L += [red_a, Collective(lambda: m._allreduce_grads(critic=False, actor=True)),
                      lambda i=i: adam_at(aopt, i + 1, gs)]
            segs.append(L)
        return segs

    def _batch_ptrs(self, i):
        B, N, D0, K, Din = self.B, self.N, self.D0, self.K, self.Din
        return (ptr(self.X, i * B * N * Din), ptr(self.X2, i * B * N * Din), ptr(self.radar, i * B * N * 18),
                ptr(self.nei, i * B * N * K * 6), ptr(self.y, i * B))

    def _actor_fwd_stages(self, i, A):
        """The actor forward of iteration i up to the merge layer: [attention set, merge products]; its
        tanh output layer runs inside the actor step's critic-encoder job (``_actor_stages`` cenc)."""
        B, N, D0, K, Din = self.B, self.N, self.D0, self.K, self.Din
        _, X2, radar, nei, _ = self._batch_ptrs(i)
        attn, merge, _ = actor_forward_stages(A, self.acts, X2, Din, radar, nei, B * N, K, D0, X2 + 4 * D0, Din)
        return attn, merge

    def _actor_fwd_launches(self, i, A):
        a_attn, a_merge = self._actor_fwd_stages(i, A)
        return [AttnEnc(a_attn)] + gemm_launches(a_merge)

    def _critic_step(self, i, A, C, cb, fuse_actor_fwd):
        """Critic step of iteration i (ATT/maddpg:375-387) up to its weight-gradient partials.
        With ``fuse_actor_fwd`` the actor forward of the same iteration (ATT/maddpg:389-392) --
        which depends only on the actor weights, changed after the critic step -- shares the
        critic step's launches; the policy actions land in X2 (own columns gathered there too)."""
        cs = self._critic_stages(i, C, cb)
        if fuse_actor_fwd:
            a_attn, a_merge = self._actor_fwd_stages(i, A)
            L = [AttnEnc(with_ride(a_attn, cs["enc"]))]
        else:
            a_merge = []
            L = [AttnEnc(ride_only(cs["enc"]))]
        L += gemm_launches(cs["comb"])
        L.append(cs["head"])
        L += gemm_launches(cs["grad"] + a_merge)
        L += gemm_launches(cs["encw"])
        return L

    def _critic_stages(self, i, C, cb):
        """The critic step of iteration i as dependent stages: enc (the encoders as a riding job of an
        aac_attn_enc_fwd launch), product lists comb, grad (weight gradients of the head and combine,
        data gradient of the combine), encw (encoder weight gradients) and the head callable (mse
        gradient) between comb and grad."""
        m, B, N, Din = self.m, self.B, self.N, self.Din
        SC, nC = self.SPLIT_CRITIC, self.gc.shape[1]     # copy stride
        gC = CriticParams(m.critics, m.fc, self.gc.data_ptr())
        X, _, _, _, y = self._batch_ptrs(i)
        f, h, dq, dh, df = cb
        _, c_comb = critic_forward_stages(C, X, B, N, Din, f, h)
        c_enc = critic_enc_ride(C, X, B, N, Din, f)
        hj = head_job(ptr(h), B, C.Wq, C.bq, 0, y=y, q=ptr(self.q_c, i * B), dq=ptr(dq), dh=ptr(dh))
        head = lambda: critic_head(ptr(h), B, C.Wq, C.bq, 0, y=y, q=ptr(self.q_c, i * B), dq=ptr(dq),  # noqa: E731
                                   dh=ptr(dh))
        ov = ptr(self.ones_k)
        grad = split_bias(
            prob(ptr(dq), ptr(h), gC.Wq, 1, 256, B, 1, 256, 256, ta=1, ones=1, cextra=gC.bq, ksplit=SC,
                 split_stride=nC), ov) + split_bias(
            prob(ptr(dh), ptr(f), gC.Wc, 256, 128 * N, B, 256, 128 * N, 128 * N, ta=1, ones=1, cextra=gC.bc,
                 ksplit=SC, split_stride=nC), ov) + [
            prob(ptr(dh), C.Wc, ptr(df), B, 128 * N, 256, 256, 128 * N, 128 * N, mask=ptr(f), ldmask=128 * N,
                 mact=RELU)]
        encw = [prob(ptr(df, n * 128), X + 4 * n * Din, gC.enc_w[n], 128, Din, B, 128 * N, N * Din, Din, ta=1, ones=1,
                     cextra=gC.enc_b[n], ksplit=SC, split_stride=nC) for n in range(N)]
        return {"enc": c_enc, "comb": c_comb, "head": head, "head_job": hj, "grad": grad, "encw": encw}

    def _actor_step(self, i, A, C):
        """Actor step of iteration i (ATT/maddpg:389-425) after its forward, up to the weight-
        gradient partials: critic on the policy actions, backward into the actor."""
        st = self._actor_stages(i, A, C)
        L = [AttnEnc(ride_only(st["cenc"]))] + gemm_launches(st["ccomb"])
        if self.DAOB:
            L.append(st["daob"]())
        else:
            L += gemm_launches(st["dcomb"])
            L.append(st["aob"])
        L += gemm_launches(st["wgrad1"])
        L.append(st["attn_bwd"])
        L += gemm_launches(st["wgrad2"] + st.get("qstat", []))
        return L

    def _actor_stages(self, i, A, C):
        """The actor step of iteration i after its forward, as dependent stages: cenc (riding job), ccomb
        (critic on the policy actions), head (-mean Q gradient), dcomb, aob (actor output
        backward), wgrad1, attn_bwd, wgrad2."""
        m, B, N, D0, K, Din = self.m, self.B, self.N, self.D0, self.K, self.Din
        R = B * N
        SA, nA = self.SPLIT_ACTOR, self.ga.shape[1]
        gA = ActorParams(m.actors, m.fa, self.ga.data_ptr())
        _, X, radar, nei, _ = self._batch_ptrs(i)
        f, h, dq, dh, df = self.cbuf[0]
        c = self.acts
        st = {}
        st["cenc"] = critic_enc_ride(C, X, B, N, Din, f, fold=(ptr(c.ha), A, D0))
        # the actor loss -mean Q has the constant gradient dq = -1/B (ATT/maddpg:424), so the head's
        # dh = dq Wo (h > 0) is a second output of the combine layer's epilogue, and Q itself (stats
        # only) is an N = 1 product beside the combine's data gradient: no head launch on this chain
        st["ccomb"] = [prob(ptr(f), C.Wc, ptr(h), B, 256, 128 * N, 128 * N, 128 * N, 256, tb=1, bias=C.bc, act=RELU,
                            dvec=C.Wq, C2=ptr(dh), dscale=-float(np.float32(1.0) / np.float32(B)))]
        st["dcomb"] = [prob(ptr(dh), C.Wc, ptr(df), B, 128 * N, 256, 256, 128 * N, 128 * N, mask=ptr(f),
                            ldmask=128 * N, mact=RELU),
                       prob(ptr(h), C.Wq, ptr(self.q_a, i * B), B, 1, 256, 256, 256, 1, tb=1, bias=C.bq)]
        # da_n = df_n . W_enc_n[:, D0:D0+2]; dout = da * (1 - a^2); dh_a = (dout Wa) * (h_a > 0)
        st["aob"] = lambda: actor_out_bwd(ptr(df), 128 * N, C.enc_w[0], Din, D0, X, A.Wa, ptr(c.ha), N, R,  # noqa: E731
                                          ptr(self.dout), ptr(self.dha))
        if self.DAOB:
            # df never reaches memory: one launch computes it per (16 samples, agent) tile and reduces it
            # into da; the Q statistics product moves to the weight-gradient launch (h is read only there)
            da = DaobArgs(ptr(dh), C.Wc, ptr(f), C.enc_w[0], X, A.Wa, ptr(c.ha), ptr(self.dout), ptr(self.dha),
                          128 * N, Din, D0, N, B)
            st["daob"] = lambda head=None: DcombAob(da, head)
            st["qstat"] = [st["dcomb"][1]]
        ov = ptr(self.ones_k)
        wout = split_bias(
            prob(ptr(self.dout), ptr(c.ha), gA.Wa, 2, 256, R, 2, 256, 256, ta=1, ones=1, cextra=gA.ba, ksplit=SA,
                 split_stride=nA), ov) + split_bias(
            prob(ptr(self.dha), ptr(c.cat), gA.Wm, 256, 192, R, 256, 192, 192, ta=1, ones=1, cextra=gA.bm,
                 ksplit=min(self.SPLIT_DWM, SA), split_stride=nA), ov)
        st["wgrad1"] = wout + [
            prob(ptr(self.dha), A.Wm, ptr(self.dcat_o), R, 64, 256, 256, 192, 64),
            prob(ptr(self.dha), A.Wm + 4 * 64, ptr(self.dcat_g), R, 64, 256, 256, 192, 64, mask=ptr(c.cat, 64),
                 ldmask=192, mact=RELU),
            prob(ptr(self.dha), A.Wm + 4 * 128, ptr(self.dv), R, 64, 256, 256, 192, 64)]
        if self.wn_part:
            st["attn_bwd"] = AttnBwd(lambda: attn_train_bwd_wn(
                ptr(self.dv), 64, ptr(c.xn), ptr(c.alpha), ptr(c.qk), ptr(c.cat), 192, ptr(self.dcat_o), 64, A.Wq,
                A.Wkv, A.Wkv + 4 * 64 * 64, ptr(self.dqk), ptr(self.dqa), ptr(self.deo), R, K, nei, ptr(self.pwn)),
                R, K, attn_bwd_partials(R))
            # dWn | dbn (adjacent in the flat gradient) = the sum of the partial rows
            assert gA.bn == gA.Wn + 4 * 64 * 6
            P = self.pwn.shape[0]
            dwn = prob(ptr(self.ones_p), ptr(self.pwn), gA.Wn, 1, 448, P, P, 448, 448, ksplit=SA, split_stride=nA)
        else:
            st["attn_bwd"] = AttnBwd(lambda: attn_train_bwd(
                ptr(self.dv), 64, ptr(c.xn), ptr(c.alpha), ptr(c.qk), ptr(c.cat), 192, ptr(self.dcat_o), 64, A.Wq,
                A.Wkv, A.Wkv + 4 * 64 * 64, ptr(self.dxn), ptr(self.dqk), ptr(self.dqa), ptr(self.deo), R, K), R, K)
            dwn = prob(ptr(self.dxn), nei, gA.Wn, 64, 6, R * K, 64, 6, 6, ta=1, ones=1, cextra=gA.bn, ksplit=SA,
                       split_stride=nA)
        st["wgrad2"] = [
            prob(ptr(self.dv), ptr(c.xb), gA.Wkv + 4 * 64 * 64, 64, 64, R, 64, 64, 64, ta=1, ksplit=SA,
                 split_stride=nA),                                                         # dWv
            prob(ptr(c.qa), ptr(self.dqk), gA.Wkv, 64, 64, R, 64, 64, 64, ta=1, ksplit=SA, split_stride=nA),  # dWk
            prob(ptr(self.dqa), ptr(c.cat), gA.Wq, 64, 64, R, 64, 192, 64, ta=1, ksplit=SA, split_stride=nA),
            dwn,
            prob(ptr(self.deo), X, gA.Wo, 64, D0, R, 64, Din, D0, ta=1, ones=1, cextra=gA.bo, ksplit=SA,
                 split_stride=nA),
            prob(ptr(self.dcat_g), radar, gA.Wg, 64, 18, R, 64, 18, 18, ta=1, ones=1, cextra=gA.bg, ksplit=SA,
                 split_stride=nA)]
        return st

    # ------------------------------------------------------------------ run
    def ops(self):
        return self.pre + [op for it in self.iters for op in it] + self.post

    def run(self, idx=None, soft=True):
        """One eager update; ``soft=False`` skips the Polyak step (the Adam counters still advance)."""
        if idx is None:
            self.pre[0]()
        else:
            self.idx.copy_(idx.reshape(-1))
        for op in self.pre[1:]:
            op()
        for it in self.iters:
            for op in it:
                op()
        for op in (self.post if soft else self.post_hold):
            op()

    def segments(self):
        """The launch list cut at the collectives: ([segment ops], [collective]) with
        len(segments) == len(collectives) + 1.  Collectives a HIP graph can hold (RCCL,
        parallel.capturable) stay inline: one segment, no cut."""
        if parallel.capturable(self.m.pg):
            return [self.ops()], []
        segs, colls, cur = [], [], []
        for op in self.ops():
            if isinstance(op, Collective):
                segs.append(cur)
                colls.append(op)
                cur = []
            else:
                cur.append(op)
        segs.append(cur)
        return segs, colls

    def run_timed(self):
        """One eager update with a HIP event pair around every GEMM launch (on the launching
        stream); returns [(algorithmic FLOPs, event pair)] for the grouped-GEMM roofline."""
        rec = []
        for op in self.ops():
            if isinstance(op, GemmLaunch):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                op()
                e1.record()
                rec.append((op.flops, e0, e1))
            else:
                op()
        return rec

    def batch_rewards(self, i):
        """The reward rows [B][N] of iteration i's sampled batch."""
        return self.rew[i * self.B:(i + 1) * self.B]

    def pre_reward_target(self, i):
        """gamma Q' (1 - any done) of iteration i's batch -- the reference's ``tar_Q_before_rew``
        (ATT/maddpg:357) -- in the TD head's own fp32 operation order, from the Q' it stored."""
        B = self.B
        qn = self.qn[i * B:(i + 1) * B]
        done_any = (self.done[i * B:(i + 1) * B] == 1.0).any(dim=1).to(torch.float32)
        g = torch.tensor(self.m.GAMMA, dtype=torch.float32, device=qn.device)
        return (g * qn) * (1.0 - done_any)

    def stats(self):
        """[(loss_q, loss_a, q, target)] per iteration, like MADDPG._iteration."""
        B = self.B
        out = []
        for i in range(self.N):
            q = self.q_c[i * B:(i + 1) * B].unsqueeze(1)
            y = self.y[i * B:(i + 1) * B]
            out.append((((q - y.unsqueeze(1)) ** 2).mean(), -self.q_a[i * B:(i + 1) * B].mean(), q, y))
        return out
