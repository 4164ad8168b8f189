"""Full-state checkpoint / resume (multi_agent_aac_amd/checkpoint.py): a
training loop interrupted after a checkpoint and resumed in a fresh process state (new env, learner,
replay, captured graphs) continues bit-identically to the uninterrupted run -- parameters, targets,
Adam moments and steps, replay rows / position / sampler counter, env state and episode counters,
observation rows.  ATT (config 3 shape, small), GRU (config 4 learner + WGRU env), UAM (config 5)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _trainer(model, seed=1):
    from multi_agent_aac_amd import trainer
    if model == "uam":
        return trainer.UamTrainer(256, 6, 128, 8192, seed=seed)
    return trainer.Trainer(256, 5 if model == "att" else 4, 128, 4096, "combined", seed=seed, model=model)


def _snapshot(tr):
    from multi_agent_aac_amd import checkpoint
    torch.cuda.synchronize()
    out = {"L." + k: v.clone() for k, v in checkpoint.learner_tensors(tr.model).items()}
    out.update({"R." + k: v.clone() for k, v in checkpoint.replay_tensors(tr.replay).items()})
    out.update({"E." + k: v.clone() for k, v in checkpoint.env_tensors(tr.env).items()})
    out.update({"X." + k: v.clone() for k, v in tr.checkpoint_parts()["extra"].items()})
    return out


@pytest.mark.parametrize("model", ["att", "gru", "uam"])
def test_resume_is_bit_identical(native_lib, model, tmp_path):
    a = _trainer(model)
    while len(a.replay) <= a.B:
        a.step(update=False)
    for _ in range(3):
        a.step(update=True)
    path = str(tmp_path / f"{model}.ckpt")
    a.save_checkpoint(path)
    for _ in range(4):
        a.step(update=True)
    want = _snapshot(a)
    b = _trainer(model)                  # fresh loop: its own first OD draws, random init, empty replay
    b.load_checkpoint(path)
    for _ in range(4):
        b.step(update=True)
    got = _snapshot(b)
    assert set(want) == set(got)
    bad = [k for k in want if not torch.equal(want[k], got[k])]
    assert not bad, bad
    assert len(a.replay) == len(b.replay) and a.replay.pos == b.replay.pos


def test_uam_overlapped_reset_matches_serial(native_lib, monkeypatch):
    """UamTrainer's packed auto-reset on the side stream beside the update (trainer.UAM_OVERLAP_RESET,
    the default) leaves every learner, replay and env tensor bit-identical to the serial order."""
    from multi_agent_aac_amd import trainer
    snaps = []
    for flag in (True, False):
        monkeypatch.setattr(trainer, "UAM_OVERLAP_RESET", flag)
        t = _trainer("uam")
        while len(t.replay) <= t.B:
            t.step(update=False)
        for _ in range(6):
            t.step(update=True)
        snaps.append(_snapshot(t))
    a, b = snaps
    assert set(a) == set(b)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, bad


@pytest.mark.parametrize("overlap", [True, False])
def test_uam_whole_step_graph_equals_eager(native_lib, monkeypatch, overlap):
    """UamTrainer.step_graph / step_graph_pair (act + env step + replay push with the ring position in
    device words (aac_uam_push_io) + auto-reset beside the update, replayed from captured graphs)
    against the same steps launched eagerly: every learner, replay and env tensor bit-identical, the
    host mirror of the ring position too, across ring wraps (8192 rows, 1536 per push), an eager step
    between replays (the device word re-seeded) and both starting parities."""
    from multi_agent_aac_amd import trainer
    monkeypatch.setattr(trainer, "UAM_OVERLAP_RESET", overlap)
    monkeypatch.setattr(trainer, "UAM_STEP_GRAPH", True)     # off by default in the bench (measured slower)
    tr = [_trainer("uam") for _ in range(2)]
    for t in tr:
        while len(t.replay) <= t.B:
            t.step(update=False)
        t.step(update=True)
    assert tr[1].graph_ok()
    for k in range(5):
        tr[0].step(update=True)
        if k == 2:
            tr[1].step(update=True)
        else:
            tr[1].step_graph()
    for _ in range(3):
        tr[0].step(update=True)
        tr[0].step(update=True)
        tr[1].step_graph_pair()
    tr[0].step(update=True)
    tr[1].step(update=True)
    for _ in range(2):
        tr[0].step(update=True)
        tr[0].step(update=True)
        tr[1].step_graph_pair()
    a, b = _snapshot(tr[0]), _snapshot(tr[1])
    assert set(a) == set(b)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, bad
    assert (tr[0].replay.pos, tr[0].replay.size) == (tr[1].replay.pos, tr[1].replay.size)
    assert torch.equal(tr[0].episode, tr[1].episode)


def test_checkpoint_refuses_mismatch(native_lib, tmp_path):
    from multi_agent_aac_amd import checkpoint
    a = _trainer("att")
    path = str(tmp_path / "att.ckpt")
    checkpoint.save(path, learner=a.model, replay=a.replay)
    g = _trainer("gru")
    with pytest.raises(ValueError):
        checkpoint.load(path, learner=g.model)
    with pytest.raises(KeyError):
        checkpoint.load(path, learner=a.model, env=a.env)
    ck = torch.load(path, weights_only=True)
    ck["parts"]["replay"]["tensors"]["counter"].fill_(1 << 32)     # 32-bit RNG epochs only
    torch.save(ck, path)
    with pytest.raises(ValueError):
        checkpoint.load(path, replay=a.replay)


@pytest.mark.parametrize("model", ["att", "uam"])
def test_resume_into_running_loop_with_other_seeds(native_lib, model, tmp_path, monkeypatch):
    """a load into a loop that already captured its update graph (and, for ATT, its
    whole-step graphs) with other replay / noise seeds -- host scalars baked into those graphs --
    still resumes bit-identically: the load drops the stale graphs and re-seeds the ring word."""
    from multi_agent_aac_amd import trainer
    monkeypatch.setattr(trainer, "STEP_GRAPH", True)
    a = _trainer(model)
    while len(a.replay) <= a.B:
        a.step(update=False)
    for _ in range(2):
        a.step(update=True)
    path = str(tmp_path / f"{model}.ckpt")
    a.save_checkpoint(path)
    for _ in range(4):
        a.step(update=True)
    want = _snapshot(a)
    b = _trainer(model)
    b.model.noise_seed += 17                 # other host-side seeds, baked into b's graphs below
    b.replay.seed += 5
    while len(b.replay) <= b.B:
        b.step(update=False)
    for _ in range(2):
        b.step(update=True)
    b.step_graph()
    assert b._sg
    assert b.model.has_graph()
    b.load_checkpoint(path)
    for k in range(4):
        if k % 2:
            b.step_graph()
        else:
            b.step(update=True)
    got = _snapshot(b)
    bad = [k for k in want if not torch.equal(want[k], got[k])]
    assert not bad, bad


def test_checkpoint_refuses_other_env_bank(native_lib, tmp_path):
    """the auto-reset's OD bank and draw seed are part of the env's checkpoint: a bank
    that differs is refused, a draw seed that differs is restored."""
    a = _trainer("att", seed=1)
    while len(a.replay) <= a.B:
        a.step(update=False)
    a.step(update=True)
    path = str(tmp_path / "att.ckpt")
    a.save_checkpoint(path)
    other = _trainer("att", seed=2)          # other OD bank (seed 2028) and draw seed
    for _ in range(3):
        other.step(update=False)
    before = _snapshot(other)
    pos, size, seed = other.replay.pos, other.replay.size, other.replay.seed
    with pytest.raises(ValueError, match="bank"):
        other.load_checkpoint(path)
    # a refused file changes nothing -- learner, replay rows / position, env, extra
    after = _snapshot(other)
    bad = [k for k in before if not torch.equal(before[k], after[k])]
    assert not bad, bad
    assert (other.replay.pos, other.replay.size, other.replay.seed) == (pos, size, seed)
    same = _trainer("att", seed=1)
    same.env.set_od_bank(same.bank, seed=999)
    gen = same.env.bank_generation
    same.load_checkpoint(path)
    assert same.env.bank_seed == a.env.bank_seed
    assert same.env.bank_generation == gen + 1      # captured step graphs are re-captured


def test_step_graph_recaptures_after_bank_change(native_lib, monkeypatch):
    """a whole-step graph bakes the OD bank's device pointers and draw seed; re-installing
    the bank (set_od_bank re-allocates it) must not leave the trainer replaying the old graph."""
    from multi_agent_aac_amd import trainer
    monkeypatch.setattr(trainer, "STEP_GRAPH", True)
    a = _trainer("att", seed=1)
    while len(a.replay) <= a.B:
        a.step(update=False)
    a.step_graph()
    g0 = a._sg[0][0]
    a.env.set_od_bank(a.bank, seed=4321)
    a.step_graph()
    assert a._sg and a._sg[0][0] is not g0
