"""The runtime CPU-oracle diff mode (tests/oracle_diff.py) on live training: a Trainer stepping with
updates (ATT config-3 env, WGRU config-4 env), every 3rd step a sampled subset of envs re-run on the
C oracle from the GPU's pre-step state -- no mismatch over the run; and a corrupted step (the GPU
env moved after the snapshot) is caught."""
import pytest
import torch

from tests.oracle_diff import OracleDiff, OracleMismatch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,N", [("att", 5), ("gru", 8)])
def test_training_steps_match_oracle_subset(native_lib, model, N):
    from multi_agent_aac_amd import trainer
    tr = trainer.Trainer(256, N, 64, 4096, "combined", seed=3, model=model)
    diff = OracleDiff(tr, every=3, n_envs=64, seed=1)
    assert not tr.graph_ok()          # a hooked trainer steps eagerly
    for _ in range(36):
        tr.step(update=True)
    torch.cuda.synchronize()
    assert diff.checked == 12
    diff.detach()
    assert not tr.hooked()


def test_corrupted_step_is_caught(native_lib):
    from multi_agent_aac_amd import trainer
    tr = trainer.Trainer(256, 5, 64, 4096, "combined", seed=4)
    OracleDiff(tr, every=1, n_envs=32, seed=2)

    def corrupt(t):           # runs after the snapshot: the GPU steps from other positions
        s = t.env.get_state()
        t.env.set_state(pos=s["pos"] + 0.25)
    tr.pre_step_hooks.append(corrupt)
    with pytest.raises(OracleMismatch):
        tr.step(update=False)
