"""Replay memory on the device (ATT/mem:6-23 ``ReplayMemory``).

``DeviceReplay`` stores one transition per fixed-width fp32 row
    [s_own (N*D0) | s_radar (N*18) | s_nei (N*K*6) | a (N*2) | r (N) | done (N) | s'_own | s'_radar | s'_nei]
(660 floats = 2 640 B at N = 5, padded to 672 = 21 whole 128-B lines) in a ring of ``capacity`` rows; with ``hidden = H`` (the GRU-actor
learner) the row also carries the actor hidden states before and after
the step, ``| h_cur (N*H) | h_next (N*H)`` (the ``cur_hidden`` / ``next_hidden`` fields of
MADDPG_ownENV_randomOD_Wgru_radar/ma_main_randomOD_Wgru_radar.py:636).  Push is one HIP launch for all E
transitions of a step; sampling draws B distinct rows uniformly (``random.sample`` semantics) and
gathers them into field-contiguous batch tensors, all on the device (graph-capturable: the ring
position / size and the RNG counter live in device memory).

``ReplayMemory`` keeps the reference's ``push(*8 fields)`` / ``sample(B)`` / ``len`` surface for
an unchanged ``ma_main`` (E = 1); its rows land in the same device ring.
"""
import ctypes
import os
from collections import namedtuple

import numpy as np
import torch

from . import ops

Experience = namedtuple("Experience", ("states", "actions", "next_states", "rewards", "dones", "history_info",
                                       "cur_hidden", "next_hidden"))

FIELDS = ("s_own", "s_radar", "s_nei", "act", "rew", "done", "n_own", "n_radar", "n_nei")
# ring rows padded to a multiple of this many bytes (0: unpadded); AAC_RING_PAD overrides
ROW_PAD = int(os.environ.get("AAC_RING_PAD", "128"))
HIDDEN_FIELDS = ("h_cur", "h_next")


class DeviceReplay:
    def __init__(self, capacity, N, D0, R=18, device="cuda", seed=0, hidden=0):
        self.N, self.D0, self.R, self.K, self.H = N, D0, R, N - 1, int(hidden)
        K = self.K
        self.shapes = [(N, D0), (N, R), (N, K, 6), (N, 2), (N,), (N,), (N, D0), (N, R), (N, K, 6)]
        self.dtypes = [0, 0, 0, 0, 0, 1, 0, 0, 0]
        self.fields = FIELDS
        if self.H:
            self.shapes += [(N, self.H), (N, self.H)]
            self.dtypes += [0, 0]
            self.fields = FIELDS + HIDDEN_FIELDS
        self.widths = [int(torch.Size(s).numel()) for s in self.shapes]
        self.row_width = sum(self.widths)          # data floats per transition
        # the ring's row stride: rounded up to whole 128-B lines (ROW_PAD), so that no line holds the
        # end of one transition and the start of the next (the fused env tail writes each row's fields
        # from one workgroup); the pad columns stay zero
        q = ROW_PAD // 4 if ROW_PAD else 1
        self.stride = (self.row_width + q - 1) // q * q
        self.capacity = int(capacity)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.ring = torch.zeros(self.capacity, self.stride, dtype=torch.float32, device=self.device)
        self.meta = torch.zeros(2, dtype=torch.int64, device=self.device)       # [next pos, size]
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)    # sampler RNG counter
        self.seed = int(seed)
        self.size = 0          # host mirror of meta[1] (pushes are host-initiated, so no sync needed)
        self.pos = 0           # host mirror of meta[0]
        self._batch = {}

    def __len__(self):
        return self.size

    def push_batch(self, s_own, s_radar, s_nei, act, rew, done, n_own, n_radar, n_nei, h_cur=None, h_next=None):
        srcs = [s_own, s_radar, s_nei, act, rew, done, n_own, n_radar, n_nei]
        if self.H:
            assert h_cur is not None and h_next is not None, "this replay stores hidden states"
            srcs += [h_cur, h_next]
        E = s_own.shape[0]
        for t in srcs:
            assert t.is_contiguous() and t.device == self.device and t.shape[0] == E
        ops.replay_push_at(self.ring, self.meta, self.pos, self.size, srcs, self.widths, self.dtypes, E)
        self.pos = (self.pos + E) % self.capacity
        self.size = min(self.size + E, self.capacity)

    def tail_push(self, srcs, E):
        """The push of ``push_batch(*srcs)`` as the replay part of a fused env step tail
        (``BatchedEnv.step_tail``, aac_env_step_tail): returns the aac_step_tail fields and advances
        the host mirror of the ring position (the launch advances ``meta``)."""
        if self.H:
            assert len(srcs) == 11, "this replay stores hidden states"
        else:
            assert len(srcs) == 9
        for t in srcs:
            assert t.is_contiguous() and t.device == self.device and t.shape[0] == E
        n = len(srcs)
        d = dict(ring=self.ring.data_ptr(), row_width=self.stride, capacity=self.capacity, pos=self.pos,
                 size=self.size, meta=self.meta.data_ptr(), n_fields=n,
                 srcs=(ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs]),
                 widths=(ctypes.c_int32 * n)(*self.widths[:n]), dtypes=(ctypes.c_int32 * n)(*self.dtypes[:n]))
        self.pos = (self.pos + E) % self.capacity
        self.size = min(self.size + E, self.capacity)
        return d

    def check_sample(self, B):
        """random.sample semantics need at least B stored rows (the reference guards with
        len(memory) > batch_size, ATT/maddpg:223)."""
        if self.size < B:
            raise ValueError(f"replay holds {self.size} transitions, cannot sample {B} distinct rows")

    def batch_buffers(self, B, nb=1):
        key = (B, nb)
        if key not in self._batch:
            bufs = [torch.empty((nb * B,) + s, dtype=torch.float32, device=self.device) for s in self.shapes]
            idx = torch.empty(nb * B, dtype=torch.int32, device=self.device)
            self._batch[key] = (idx, dict(zip(self.fields, bufs)), bufs)
        return self._batch[key]

    def sample_batch(self, B, idx=None, nb=1):
        """Draw ``nb`` independent batches of B distinct rows (or use the given device indices,
        shape (nb * B,)) into static field-contiguous tensors of leading size nb * B."""
        bidx, named, bufs = self.batch_buffers(B, nb)
        self.check_sample(B)
        if idx is None:
            ops.replay_sample(self.meta, B, self.seed, self.counter, bidx)
        else:
            bidx.copy_(idx.reshape(-1))
        ops.replay_gather(self.ring, bidx, bufs, self.widths)
        return named


class ReplayMemory:
    """Reference surface (ATT/mem:6-23) over ``DeviceReplay``; states are the reference's
    ``[own (N, D0), radar (N, 18), [nei_i (K, 1, 6) or (K, 6)] * N]`` lists."""

    def __init__(self, capacity, device="cuda", hidden=0):
        self.capacity = int(capacity)
        self.device = device
        self.hidden = int(hidden)      # GRU-actor rows also keep cur_hidden / next_hidden
        self.dev = None
        self.memory = self       # reference code reads ``len(model.memory)``
        self.position = 0

    @staticmethod
    def _mat(x):
        """(N, D) tensor from a tensor / array or a list of per-agent rows (ATT/main:363-390)."""
        if isinstance(x, (list, tuple)):
            x = np.stack([np.asarray(v.cpu() if torch.is_tensor(v) else v, dtype=np.float32) for v in x])
        return torch.as_tensor(x, dtype=torch.float32)

    def _ensure(self, states):
        if self.dev is None:
            N, D0 = self._mat(states[0]).shape
            self.dev = DeviceReplay(self.capacity, N, D0, self._mat(states[1]).shape[1], self.device,
                                    hidden=self.hidden)

    def _obs(self, states):
        own = self._mat(states[0]).reshape(1, self.dev.N, self.dev.D0)
        radar = self._mat(states[1]).reshape(1, self.dev.N, self.dev.R)
        if len(states) > 2:
            nei = torch.stack([self._mat([np.asarray(v.cpu() if torch.is_tensor(v) else v).reshape(6) for v in x])
                               for x in states[2]])
        else:       # two-portion states [own, grid] (WGRU/ma_main:601-636): no neighbour rows
            nei = torch.zeros(self.dev.N, self.dev.K, 6)
        return [t.to(self.dev.device).contiguous() for t in (own, radar, nei.reshape(1, self.dev.N, self.dev.K, 6))]

    def push(self, states, actions, next_states, rewards, dones, history_info=None, cur_hidden=None,
             next_hidden=None):
        self._ensure(states)
        s = self._obs(states)
        n = self._obs(next_states)
        d = self.dev.device
        a = torch.as_tensor(actions, dtype=torch.float32).reshape(1, self.dev.N, 2).to(d).contiguous()
        r = torch.as_tensor(rewards, dtype=torch.float32).reshape(1, self.dev.N).to(d).contiguous()
        dn = (torch.as_tensor(dones).reshape(1, self.dev.N) != 0).to(torch.uint8).to(d).contiguous()
        hid = []
        if self.hidden:
            hid = [self._mat(h).reshape(1, self.dev.N, self.hidden).to(d).contiguous() for h in (cur_hidden, next_hidden)]
        self.dev.push_batch(s[0], s[1], s[2], a, r, dn, n[0], n[1], n[2], *hid)
        self.position = (self.position + 1) % self.capacity

    def sample(self, batch_size):
        b = self.dev.sample_batch(batch_size)
        out = []
        for i in range(batch_size):
            st = [b["s_own"][i], b["s_radar"][i], [b["s_nei"][i, k] for k in range(self.dev.N)]]
            nx = [b["n_own"][i], b["n_radar"][i], [b["n_nei"][i, k] for k in range(self.dev.N)]]
            hc = b["h_cur"][i] if self.hidden else None
            hn = b["h_next"][i] if self.hidden else None
            out.append(Experience(st, b["act"][i], nx, b["rew"][i], b["done"][i], None, hc, hn))
        return out

    def __len__(self):
        return 0 if self.dev is None else len(self.dev)
