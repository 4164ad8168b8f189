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
HIP graphs a running learner already captured keep pointing at the restored storage.  Host scalars
baked into captured graphs -- the replay sampler's seed and the exploration-noise seed -- are the
exception: when a load changes either, the learner's captured update graph is dropped (re-captured
on the next update), and ``trainer.CheckpointMixin`` drops its whole-step graphs.

The env part also records what the auto-reset's future OD draws depend on but ``get_state`` does not
export: the env configuration (variant, radar mode, episode length, waypoint slots), the OD bank's
fingerprint and its draw seed.  A bank or configuration mismatch is refused on load; a draw seed that
differs from the live env's is restored (the bank is re-installed with the saved seed).

The file is a ``torch.save`` of a dict of CPU tensors and plain values, read back with
``weights_only=True``.  RNG counters are 32-bit epochs (aac_learn.hip ``take_epoch``): values >= 2^32
are rejected on load.
"""
import hashlib

import numpy as np
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


def bank_fingerprint(bank):
    """sha1 over the bank's arrays (OD starts / waypoints / counts, or UAM starts / goals / clouds),
    cached on the bank object."""
    fp = getattr(bank, "_fingerprint", None)
    if fp is None:
        h = hashlib.sha1()
        for name in ("start", "wps", "cnt", "counts", "goal", "clouds"):
            a = getattr(bank, name, None)
            if a is not None:
                h.update(name.encode())
                h.update(np.ascontiguousarray(a).tobytes())
        fp = h.hexdigest()
        try:
            bank._fingerprint = fp
        except AttributeError:
            pass
    return fp


def env_meta(env):
    """What the env's future steps and auto-reset draws depend on beyond its device state."""
    m = {"E": int(env.E), "N": int(env.N), "class": type(env).__name__}
    for k in ("variant", "radar_mode", "W", "D0", "tdcpa", "neighbours", "p3"):
        if hasattr(env, k):
            v = getattr(env, k)
            m[k] = v if isinstance(v, (bool, str)) or v is None else int(v)
    cfg = getattr(env, "cfg", None)
    if cfg is not None and hasattr(cfg, "episode_length"):
        m["episode_length"] = int(cfg.episode_length)
    occ = getattr(env, "occ", None)
    if occ is not None:
        m["maps"] = hashlib.sha1(np.ascontiguousarray(np.asarray(occ, dtype=np.uint8)).tobytes()).hexdigest()
    bank = getattr(env, "bank", None)
    if bank is not None:
        m["bank"] = bank_fingerprint(bank)
        m["bank_seed"] = int(getattr(env, "bank_seed", 0))
    return m


def env_tensors(env):
    """The env's state as a dict of fresh device tensors (get_state); with its episode buffer."""
    t = dict(env.get_state())
    ep = getattr(env, "_episode_buf", None)
    if ep is not None:
        t["episode"] = ep
    return t


# --------------------------------------------------------------------------- save / load
def drop_graphs(learner):
    """Forget the learner's captured update graph (re-captured by the next ``update``)."""
    if learner is not None:
        learner.invalidate_graphs()


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
        ck["parts"]["env"] = {"meta": env_meta(env),
                              "tensors": {k: _cpu(v) for k, v in env_tensors(env).items()}}
    if extra:
        ck["parts"]["extra"] = {"meta": {}, "tensors": {k: _cpu(v) for k, v in extra.items()}}
    torch.save(ck, path)
    return path


def _check_counter(name, t):
    v = int(t.reshape(-1)[0])
    if v < 0 or v >= _EPOCH_LIMIT:
        raise ValueError(f"{name} = {v}: RNG epochs are 32-bit (0 <= value < 2^32)")


def _check_fit(dst, src, name):
    if tuple(dst.shape) != tuple(src.shape) or dst.dtype != src.dtype:
        raise ValueError(f"checkpoint tensor {name}: {tuple(src.shape)} {src.dtype} does not fit "
                         f"{tuple(dst.shape)} {dst.dtype}")


def _plan(ck, path, learner, replay, env, extra):
    """Validate every requested part against the live objects WITHOUT touching them.  Returns the
    list of (dst, src, name) copies and the scalar updates to apply; raises on any mismatch, so a
    refused file leaves the running loop exactly as it was (a half-restored loop replayed
    stale graphs against a moved ring position)."""
    parts = ck["parts"]
    for want, obj in (("learner", learner), ("replay", replay), ("env", env), ("extra", extra)):
        if obj is not None and want not in parts:
            raise KeyError(f"{path} holds no {want} state")
    copies, todo = [], {}
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
            _check_fit(v, p["tensors"][k], "learner." + k)
            copies.append((v, p["tensors"][k], "learner." + k))
        todo["noise_seed"] = p["meta"]["noise_seed"]
    if replay is not None:
        p = parts["replay"]
        m = p["meta"]
        if m["capacity"] != replay.capacity or m["row_width"] != replay.ring.shape[1]:
            raise ValueError(f"checkpoint replay {m} does not fit capacity {replay.capacity} x {replay.ring.shape[1]}")
        if not 0 <= m["size"] <= m["capacity"] or not 0 <= m["pos"] < max(1, m["capacity"]):
            raise ValueError(f"checkpoint replay position {m['pos']} / size {m['size']} out of range")
        _check_counter("replay.counter", p["tensors"]["counter"])
        if replay.seed != m["seed"] and learner is None:
            raise ValueError("the checkpoint's replay seed differs from the live replay's: load the learner "
                             "with it, so that its captured update graph (which bakes the seed) is dropped")
        live = replay_tensors(replay)
        for k, dst in (("ring", live["ring"][:m["size"]]), ("meta", live["meta"]), ("counter", live["counter"])):
            _check_fit(dst, p["tensors"][k], "replay." + k)
            copies.append((dst, p["tensors"][k], "replay." + k))
        todo["replay"] = (m["seed"], m["pos"], m["size"])
    if env is not None:
        p = parts["env"]
        saved, live = dict(p["meta"]), env_meta(env)
        seed = saved.pop("bank_seed", None)
        live_seed = live.pop("bank_seed", None)
        bad = {k: (saved[k], live.get(k)) for k in saved if saved[k] != live.get(k)}
        if bad:
            raise ValueError(f"checkpoint env does not match the live env (saved, live): {bad}")
        t = dict(p["tensors"])
        ep = t.pop("episode", None)
        cur = env_tensors(env)
        cur.pop("episode", None)
        if set(t) != set(cur):
            raise ValueError(f"checkpoint env tensors {sorted(t)} != {sorted(cur)}")
        for k, v in cur.items():
            _check_fit(v, t[k], "env." + k)
        if ep is not None:
            buf = getattr(env, "_episode_buf", None)
            if buf is None:
                raise ValueError("checkpoint carries episode counters but the env has no episode buffer")
            _check_fit(buf, ep, "env.episode")
        todo["env"] = (t, ep, seed if seed is not None and seed != live_seed else None)
    if extra is not None:
        p = parts["extra"]["tensors"]
        for k, v in extra.items():
            if k not in p:
                raise KeyError(f"{path} holds no extra tensor {k}")
            _check_fit(v, p[k], "extra." + k)
            copies.append((v, p[k], "extra." + k))
    return copies, todo


def load(path, learner=None, replay=None, env=None, extra=None):
    """Restore the parts given (each must have been saved) into the live objects, in place.  Every
    part is checked first; nothing is written unless the whole file fits."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(ck, dict) or ck.get("format") != FORMAT:
        raise ValueError(f"{path}: not an {FORMAT} file")
    copies, todo = _plan(ck, path, learner, replay, env, extra)
    for dst, src, _ in copies:
        dst.copy_(src.to(dst.device))
    reseeded = False
    if "noise_seed" in todo:
        reseeded |= learner.noise_seed != todo["noise_seed"]
        learner.noise_seed = todo["noise_seed"]
    if "replay" in todo:
        seed, pos, size = todo["replay"]
        reseeded |= replay.seed != seed
        replay.seed, replay.pos, replay.size = seed, pos, size
    if reseeded:
        drop_graphs(learner)
    if "env" in todo:
        t, ep, seed = todo["env"]
        if seed is not None:
            # same bank, other draw seed: restore the saved one (future episodes draw as in the saved
            # run).  The env's bank generation advances, so graphs captured around its step tail or
            # auto-reset (which bake the bank pointers and seed) are re-captured by their owner.
            if hasattr(env, "set_od_bank"):
                env.set_od_bank(env.bank, seed=seed)
            else:
                env.set_bank(env.bank, seed=seed)
        env.set_state(**t)
        if ep is not None:
            env._episode_buf.copy_(ep.to(env._episode_buf.device))
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return ck
