"""Full-state checkpoint / resume of the vectorised training loop ("next").

The reference saves the actor ``state_dict`` only (ATT/maddpg:131-139, kept as
``MADDPG.save_model``).  Resuming a run bit-identically needs everything the next steps read:

  learner   online + target parameters, Adam moments and step counters, the exploration-noise RNG
            counter (ATT / GRU: the flat fp32 buffers of ``FlatParams`` and ``_Adam``; UAM: the
            float64 flat state of ``uam_learner.MADDPG._flat_state``)
  replay    the stored rows, ring position and size, the sampler's RNG counter
  env       the device state (``get_state``) and the per-env episode counters that drive the
            OD-bank draws and the noise schedule
  extra     whatever else the loop carries (current observation rows, GRU hidden states)

Every part is a named set of device tensors that ``load`` overwrites IN PLACE (``copy_``), so the
HIP graphs a running learner already captured stay valid.  The file is a ``torch.save`` of a dict of
CPU tensors and plain values, read back with ``weights_only=True``.  RNG counters are 32-bit epochs
(aac_learn.hip ``take_epoch``): values >= 2^32 are rejected on load.
"""
import torch

FORMAT = "aac-checkpoint-v1"
_EPOCH_LIMIT = 1 << 32


# --------------------------------------------------------------------------- per-object state
def learner_tensors(m):
    """Live device tensors of a learner (maddpg.MADDPG, gru.MADDPG or uam_learner.MADDPG)."""
    if hasattr(m, "fa") and hasattr(m, "fc"):            # ATT / GRU: FlatParams + _Adam
        t = {"fa": m.fa.data, "fc": m.fc.data, "fa_t": m.fa_t.data, "fc_t": m.fc_t.data}
        for tag, opt in (("adam_a", m.actor_optimizer), ("adam_c", m.critic_optimizer)):
            t[f"{tag}.m1"], t[f"{tag}.m2"], t[f"{tag}.step"] = opt.exp_avg, opt.exp_avg_sq, opt.step_t
    elif hasattr(m, "_flat_state"):                      # UAM: flat float64 parameters / targets / moments
        st = m._flat_state()
        t = {k: st[k] for k in ("flat", "tflat", "m1", "m2", "step")}
    else:
        raise TypeError(f"not a learner: {type(m).__name__}")
    t["noise_counter"] = m.noise_counter
    return t


def learner_meta(m):
    return {"class": f"{type(m).__module__}.{type(m).__name__}", "n_agents": int(m.n_agents),
            "noise_seed": int(m.noise_seed)}


def replay_tensors(rep):
    return {"ring": rep.ring, "meta": rep.meta, "counter": rep.counter}


def replay_meta(rep):
    return {"seed": int(rep.seed), "pos": int(rep.pos), "size": int(rep.size), "capacity": int(rep.capacity),
            "row_width": int(rep.ring.shape[1])}


def env_tensors(env):
    """The env's state as a dict of fresh device tensors (get_state); with its episode buffer."""
    t = dict(env.get_state())
    ep = getattr(env, "_episode_buf", None)
    if ep is not None:
        t["episode"] = ep
    return t


# --------------------------------------------------------------------------- save / load
def _cpu(t):
    return t.detach().to("cpu", copy=True)


def save(path, learner=None, replay=None, env=None, extra=None):
    """Write one checkpoint file.  The replay ring is stored up to its size (a full ring entirely)."""
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    ck = {"format": FORMAT, "parts": {}}
    if learner is not None:
        ck["parts"]["learner"] = {"meta": learner_meta(learner),
                                  "tensors": {k: _cpu(v) for k, v in learner_tensors(learner).items()}}
    if replay is not None:
        t = replay_tensors(replay)
        ring = t.pop("ring")
        tens = {k: _cpu(v) for k, v in t.items()}
        tens["ring"] = _cpu(ring[:replay.size])
        ck["parts"]["replay"] = {"meta": replay_meta(replay), "tensors": tens}
    if env is not None:
        ck["parts"]["env"] = {"meta": {"E": int(env.E), "N": int(env.N)},
                              "tensors": {k: _cpu(v) for k, v in env_tensors(env).items()}}
    if extra:
        ck["parts"]["extra"] = {"meta": {}, "tensors": {k: _cpu(v) for k, v in extra.items()}}
    torch.save(ck, path)
    return path


def _copy_into(dst, src, name):
    if dst.shape != src.shape or dst.dtype != src.dtype:
        raise ValueError(f"checkpoint tensor {name}: {tuple(src.shape)} {src.dtype} does not fit "
                         f"{tuple(dst.shape)} {dst.dtype}")
    dst.copy_(src.to(dst.device))


def _check_counter(name, t):
    v = int(t.reshape(-1)[0])
    if v < 0 or v >= _EPOCH_LIMIT:
        raise ValueError(f"{name} = {v}: RNG epochs are 32-bit (0 <= value < 2^32)")


def load(path, learner=None, replay=None, env=None, extra=None):
    """Restore the parts given (each must have been saved) into the live objects, in place."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(ck, dict) or ck.get("format") != FORMAT:
        raise ValueError(f"{path}: not an {FORMAT} file")
    parts = ck["parts"]
    for want, obj in (("learner", learner), ("replay", replay), ("env", env), ("extra", extra)):
        if obj is not None and want not in parts:
            raise KeyError(f"{path} holds no {want} state")
    if learner is not None:
        p = parts["learner"]
        meta = learner_meta(learner)
        if p["meta"]["class"] != meta["class"] or p["meta"]["n_agents"] != meta["n_agents"]:
            raise ValueError(f"checkpoint learner {p['meta']} does not match {meta}")
        _check_counter("learner.noise_counter", p["tensors"]["noise_counter"])
        live = learner_tensors(learner)
        if set(live) != set(p["tensors"]):
            raise ValueError(f"checkpoint learner tensors {sorted(p['tensors'])} != {sorted(live)}")
        for k, v in live.items():
            _copy_into(v, p["tensors"][k], "learner." + k)
        learner.noise_seed = p["meta"]["noise_seed"]
    if replay is not None:
        p = parts["replay"]
        m = p["meta"]
        if m["capacity"] != replay.capacity or m["row_width"] != replay.ring.shape[1]:
            raise ValueError(f"checkpoint replay {m} does not fit capacity {replay.capacity} x {replay.ring.shape[1]}")
        _check_counter("replay.counter", p["tensors"]["counter"])
        live = replay_tensors(replay)
        _copy_into(live["ring"][:m["size"]], p["tensors"]["ring"], "replay.ring")
        _copy_into(live["meta"], p["tensors"]["meta"], "replay.meta")
        _copy_into(live["counter"], p["tensors"]["counter"], "replay.counter")
        replay.seed, replay.pos, replay.size = m["seed"], m["pos"], m["size"]
    if env is not None:
        p = parts["env"]
        if p["meta"] != {"E": int(env.E), "N": int(env.N)}:
            raise ValueError(f"checkpoint env {p['meta']} does not match E={env.E} N={env.N}")
        t = dict(p["tensors"])
        ep = t.pop("episode", None)
        env.set_state(**t)
        if ep is not None:
            buf = getattr(env, "_episode_buf", None)
            if buf is None:
                raise ValueError("checkpoint carries episode counters but the env has no episode buffer")
            _copy_into(buf, ep, "env.episode")
    if extra is not None:
        p = parts["extra"]["tensors"]
        for k, v in extra.items():
            _copy_into(v, p[k], "extra." + k)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return ck
