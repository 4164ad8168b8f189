"""Synthetic replay transitions for the tools' microbenchmarks (random rows of the replay's field
shapes; the tools never touch oracle/, which is test infrastructure)."""
import torch


def transitions(E, N, seed, D0=None, H=0):
    """Fields of one push: (s_own, s_radar, s_nei, act, rew, done, n_own, n_radar, n_nei[, h_cur, h_next])
    on the GPU; ~10 % of the neighbour slots zero (masked attention entries)."""
    g = torch.Generator().manual_seed(seed)
    D0, K = D0 or 6 + 4 * (N - 1), N - 1
    r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    nei = [r(E, N, K, 6) * 0.5, r(E, N, K, 6) * 0.5]
    z = torch.rand(E, N, K, generator=g) < 0.1
    for x in nei:
        x[z] = 0.0
    out = [r(E, N, D0), torch.rand(E, N, 18, generator=g) * 15, nei[0], torch.rand(E, N, 2, generator=g) * 2 - 1,
           r(E, 1).repeat(1, N) * 5, (torch.rand(E, N, generator=g) < 0.1).to(torch.uint8), r(E, N, D0),
           torch.rand(E, N, 18, generator=g) * 15, nei[1]]
    if H:
        out += [torch.tanh(r(E, N, H)), torch.tanh(r(E, N, H))]
    return [t.cuda().contiguous() for t in out]
