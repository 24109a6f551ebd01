"""Which association torch.prod(x, dim=1) uses for [N, M] float32 rows on this GPU (M = 3, 4): counts the rows where
each candidate order differs from torch's result."""
import itertools

import torch


def trees(idx):
    if len(idx) == 1:
        yield idx[0]
        return
    for i in range(1, len(idx)):
        for a in trees(idx[:i]):
            for b in trees(idx[i:]):
                yield (a, b)


def ev(t, x):
    if isinstance(t, int):
        return x[:, t]
    return ev(t[0], x) * ev(t[1], x)


dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
for M in (3, 4):
    x = torch.exp(torch.randn((200_000, M), generator=g) * 4).to(dev)
    ref = torch.prod(x, dim=1)
    res = []
    for perm in itertools.permutations(range(M)):
        for t in trees(list(perm)):
            res.append((int((ev(t, x) != ref).sum()), str(t)))
    res.sort()
    print(M, res[:6])
