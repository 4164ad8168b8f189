"""torch bindings of the learner kernels in libaac_env.so (C ABI: include/aac_learn.h).

Every op launches on torch's current stream (so it can be captured in a HIP graph) and raises
if the native library is missing -- there is no eager-PyTorch fallback.
"""
import ctypes

import torch

from . import _native

vp = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f32 = ctypes.c_float
u64 = ctypes.c_uint64

_L = None


def lib():
    global _L
    if _L is None:
        L = _native.lib()
        L.aac_learn_last_error.restype = ctypes.c_char_p
        L.aac_attn_fwd.argtypes = [vp, vp, vp, i32, vp, vp, i32, vp, i32, i32, vp]
        L.aac_attn_bwd.argtypes = [vp, vp, vp, i32, vp, vp, i32, vp, vp, vp, i32, i32, vp]
        L.aac_replay_push.argtypes = [vp, i32, i64, vp, i32, vp, vp, vp, i32, vp]
        L.aac_actor_out_noise.argtypes = [vp, i64, vp, vp, vp, i32, vp, i32, f32, f32, u64, vp, i32, vp, vp]
        L.aac_actor_head_ws.argtypes = [vp, i32, i64, vp, vp, vp, vp, vp, i32, vp, i32, f32, f32, u64, vp, i32, vp, vp]
        L.aac_replay_push_at.argtypes = [vp, i32, i64, vp, i64, i64, i32, vp, vp, vp, i32, vp]
        L.aac_replay_sample.argtypes = [vp, i32, i32, u64, vp, vp, vp]
        L.aac_replay_gather.argtypes = [vp, i32, vp, i32, i32, vp, vp, vp]
        L.aac_adam_flat.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, f32, vp, vp]
        L.aac_polyak_flat.argtypes = [vp, vp, i64, f32, vp]
        L.aac_polyak_flat_step.argtypes = [vp, vp, i64, f32, vp, i32, vp]
        L.aac_polyak_flat2.argtypes = [vp, vp, i64, vp, vp, vp, i64, vp, f32, i32, vp]
        L.aac_noise_clamp.argtypes = [vp, i32, i32, vp, i32, f32, f32, u64, vp, vp, vp]
        L.aac_act_bgrad.argtypes = [vp, i32, vp, i32, vp, i32, vp, i32, i32, i32, vp, vp, vp]
        L.aac_bias_act.argtypes = [vp, vp, i64, i32, i32, vp]
        _L = L
    return _L


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().aac_learn_last_error().decode(errors='replace')}")


def _s():
    return vp(torch.cuda.current_stream().cuda_stream)


def _p(t, byte_offset=0):
    return vp(t.data_ptr() + byte_offset) if t is not None else None


# ----------------------------------------------------------------------------- attention
class _MaskedAttention(torch.autograd.Function):
    """ATT/nets:194-210 on (R rows, K neighbours, 64 dims); kv = [k | v] rows of 128."""

    @staticmethod
    def forward(ctx, q, kv, nei):
        R, K = kv.shape[0], kv.shape[1]
        q = q.contiguous()
        kv = kv.contiguous()
        nei = nei.contiguous()
        out = torch.empty(R, 64, device=q.device, dtype=torch.float32)
        alpha = torch.empty(R, K, device=q.device, dtype=torch.float32)
        _chk(lib().aac_attn_fwd(_p(q), _p(kv), _p(kv, 256), 128, _p(nei), _p(out), 64, _p(alpha), R, K, _s()),
             "aac_attn_fwd")
        ctx.save_for_backward(q, kv, alpha)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kv, alpha = ctx.saved_tensors
        R, K = kv.shape[0], kv.shape[1]
        dout = dout.contiguous()
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        _chk(lib().aac_attn_bwd(_p(q), _p(kv), _p(kv, 256), 128, _p(alpha), _p(dout), 64, _p(dq), _p(dkv),
                                _p(dkv, 256), R, K, _s()), "aac_attn_bwd")
        return dq, dkv, None


def masked_attention(q, kv, nei):
    """q (R, 64), kv (R, K, 128) = [k | v], nei (R, K, 6) mask source -> v_att (R, 64)."""
    return _MaskedAttention.apply(q, kv, nei)


# ----------------------------------------------------------------------------- layers
_tickets = {}


def _ticket_buf(dev):
    t = _tickets.get(dev)
    if t is None:
        t = _tickets[dev] = torch.zeros(64, dtype=torch.int32, device=dev)   # kernel keeps it zeroed
    return t


def act_bgrad(gy, y, gm, db, act):
    """gm = gy * act'(y); db = column sums of gm, deterministic (see aac_act_bgrad)."""
    M, O = gy.shape
    ws = tk = None
    if db is not None:
        ws = torch.empty(((M + 31) // 32) * O, dtype=torch.float32, device=gy.device)
        tk = _ticket_buf(gy.device)
    _chk(lib().aac_act_bgrad(_p(gy), gy.stride(0), _p(y), y.stride(0) if y is not None else 0, _p(gm),
                             gm.stride(0) if gm is not None else 0, _p(db), M, O, act, _p(ws), _p(tk), _s()),
         "aac_act_bgrad")


def bias_act(y, b, act):
    """y = act(y + b) in place; y (M, O) contiguous, b (O,)."""
    M, O = y.shape
    _chk(lib().aac_bias_act(_p(y), _p(b), M, O, act, _s()), "aac_bias_act")


# ----------------------------------------------------------------------------- optimiser
def adam_flat(param, grad, exp_avg, exp_avg_sq, step, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    _chk(lib().aac_adam_flat(_p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(), lr, beta1, beta2,
                             eps, _p(step), _s()), "aac_adam_flat")


def polyak_flat2(t1, s1, step1, t2, s2, step2, tau, step_add):
    """Both networks' soft updates and step counters in one launch (aac_polyak_flat2)."""
    _chk(lib().aac_polyak_flat2(_p(t1), _p(s1), t1.numel(), _p(step1), _p(t2), _p(s2), t2.numel(), _p(step2), tau,
                                step_add, _s()), "aac_polyak_flat2")


def polyak_flat(target, source, tau, step=None, step_add=0):
    """soft_update (ATT/maddpg:18-22); with ``step`` (device int32) also ``step += step_add``."""
    if step is None:
        _chk(lib().aac_polyak_flat(_p(target), _p(source), target.numel(), tau, _s()), "aac_polyak_flat")
    else:
        _chk(lib().aac_polyak_flat_step(_p(target), _p(source), target.numel(), tau, _p(step), step_add, _s()),
             "aac_polyak_flat_step")


def actor_out_noise(ha, wa, ba, act, N, episode, eps_end, noise_start, noise_end, seed, counter, noise_out=None,
                    noisy=True):
    """act[R][2] = clamp(tanh(wa ha + ba) + noise) (aac_actor_out_noise; wa / ba device addresses)."""
    R = ha.shape[0]
    _chk(lib().aac_actor_out_noise(_p(ha), R, vp(wa), vp(ba), _p(act), N, _p(episode), eps_end, noise_start, noise_end,
                                   u64(seed), _p(counter), int(noisy), _p(noise_out), _s()), "aac_actor_out_noise")


def actor_head_ws(cat, wm, bm, wa, ba, act, N, episode=None, eps_end=1, noise_start=0.0, noise_end=0.0, seed=0,
                  counter=None, noise_out=None, noisy=True):
    """act[R][2] = clamp(tanh(wa relu(wm cat + bm) + ba) + noise) over the rows of cat [R][192]
    (aac_actor_head_ws: merge + output layer + noise in one weights-stationary launch; wm, bm, wa, ba
    device addresses)."""
    R = cat.shape[0]
    _chk(lib().aac_actor_head_ws(_p(cat), cat.stride(0), R, vp(wm), vp(bm), vp(wa), vp(ba), _p(act), N, _p(episode),
                                 eps_end, noise_start, noise_end, u64(seed), _p(counter), int(noisy), _p(noise_out),
                                 _s()), "aac_actor_head_ws")


def noise_clamp(act, episode, eps_end, noise_start, seed, counter, noise_out=None, noise_end=0.0):
    E, N = act.shape[0], act.shape[1]
    _chk(lib().aac_noise_clamp(_p(act), E, N, _p(episode), eps_end, noise_start, noise_end, u64(seed), _p(counter),
                               _p(noise_out), _s()), "aac_noise_clamp")


# ----------------------------------------------------------------------------- replay
def replay_push(ring, meta, srcs, widths, dtypes, E):
    n = len(srcs)
    arr = (vp * n)(*[s.data_ptr() for s in srcs])
    w = (i32 * n)(*widths)
    d = (i32 * n)(*dtypes)
    _chk(lib().aac_replay_push(_p(ring), ring.shape[1], ring.shape[0], _p(meta), n, arr, w, d, E, _s()),
         "aac_replay_push")


def replay_push_at(ring, meta, pos, size, srcs, widths, dtypes, E):
    """replay_push with the host's [pos, size] mirror (aac_replay_push_at: one launch)."""
    n = len(srcs)
    arr = (vp * n)(*[s.data_ptr() for s in srcs])
    w = (i32 * n)(*widths)
    d = (i32 * n)(*dtypes)
    _chk(lib().aac_replay_push_at(_p(ring), ring.shape[1], ring.shape[0], _p(meta), pos, size, n, arr, w, d, E, _s()),
         "aac_replay_push_at")


def replay_sample(meta, B, seed, counter, idx_out):
    """idx_out (n_batches * B,) int32: n_batches independent draws of B distinct rows."""
    nb = idx_out.numel() // B
    _chk(lib().aac_replay_sample(_p(meta), B, nb, u64(seed), _p(counter), _p(idx_out), _s()), "aac_replay_sample")


def replay_gather(ring, idx, dsts, widths):
    n = len(dsts)
    arr = (vp * n)(*[t.data_ptr() for t in dsts])
    w = (i32 * n)(*widths)
    _chk(lib().aac_replay_gather(_p(ring), ring.shape[1], _p(idx), idx.shape[0], n, arr, w, _s()),
         "aac_replay_gather")
