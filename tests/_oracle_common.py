"""Shared deterministic test case for the reference-oracle comparison."""
import torch
import torch.nn as nn


class SmallNet(nn.Module):
    """Conv (stride/pad/bias variety) + Linear with and without bias."""

    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(3, 8, 3, stride=1, padding=1, bias=True)
        self.c2 = nn.Conv2d(8, 12, 3, stride=2, padding=1, bias=False)
        self.c3 = nn.Conv2d(12, 16, 1, stride=1, padding=0, bias=True)
        self.fc1 = nn.Linear(16 * 4 * 4, 32)
        self.fc2 = nn.Linear(32, 10, bias=False)

    def forward(self, x):
        x = torch.relu(self.c1(x))
        x = torch.relu(self.c2(x))
        x = torch.relu(self.c3(x))
        x = x.flatten(1)
        return self.fc2(torch.relu(self.fc1(x)))


def build_case(cfg):
    torch.manual_seed(cfg.get('seed', 0))
    model = SmallNet()
    g = torch.Generator().manual_seed(1)
    data = [(torch.randn(cfg['batch'], 3, 8, 8, generator=g),
             torch.randint(0, 10, (cfg['batch'],), generator=g)) for _ in range(cfg['steps'])]
    return model, data


def run_steps(model, pre, data, steps, lr=0.05):
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    grads = []
    for i in range(steps):
        x, y = data[i]
        opt.zero_grad()
        loss = nn.functional.cross_entropy(model(x), y)
        loss.backward()
        pre.step()
        grads.append([p.grad.detach().clone() for p in model.parameters()])
        opt.step()
    if hasattr(pre, 'join_factor_comm'):
        pre.join_factor_comm()    # a deferred factor all-reduce may still be in flight
    factors = [(l.state['A'].clone(), l.state['G'].clone()) for l in pre.layers]
    return grads, factors
