"""multi_agent_aac_amd -- MI355X-native (gfx950) implementation of the Multi_agent_AAC
``one_model_att`` hot path: the vectorised multi-agent env.step + ss_reward (HIP kernels in
``csrc/aac_env.hip`` behind the C ABI ``include/aac_env.h``) and the MADDPG update
(PyTorch-ROCm + HIP attention/replay kernels in ``csrc/aac_learn.hip``).

Modules are imported lazily; nothing here falls back to a CPU path: if the in-tree native
library is missing, the first call raises.
"""
__all__ = ["env", "world", "maddpg", "networks", "memory", "parallel", "build"]
