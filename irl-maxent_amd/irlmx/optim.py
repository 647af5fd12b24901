"""Batched optimisers of the IRL outer loop (reference src/optimizer.py) on device tensors.

``BatchedMaxEnt`` updates the theta rows of all active instances at once with
one of these; each mirrors a reference class step for step:

    Sga(lr)                    theta += lr_k * grad                 optimizer.py:61-108
    ExpSga(lr, normalize)      theta *= exp(lr_k * grad)
                               (normalize: theta /= sum(theta))     optimizer.py:110-167
    NormalizeGrad(opt, ord)    opt with grad / ||grad||_ord         optimizer.py:170-214

``lr`` is a float or a callable of the step index k -- the schedules below, or
the reference's own ``linear_decay`` / ``power_decay`` / ``exponential_decay``
closures.  The step size is evaluated on the host with numpy exactly as the
reference does (one float64 per step, shared by every instance: all instances
start together, so their step indices agree); the update itself runs on the
device for the whole batch.
"""

import numpy as np
import torch


def linear_decay(lr0=0.2, decay_rate=1.0, decay_steps=1):
    """lr0 / (1 + decay_rate * floor(k / decay_steps)) (optimizer.py:217-240)."""
    return lambda k: lr0 / (1.0 + decay_rate * np.floor(k / decay_steps))


def power_decay(lr0=0.2, decay_rate=1.0, decay_steps=1, power=2):
    """lr0 / (decay_rate * floor(k / decay_steps) + 1) ** power (optimizer.py:243-267)."""
    return lambda k: lr0 / (decay_rate * np.floor(k / decay_steps) + 1.0) ** power


def exponential_decay(lr0=0.2, decay_rate=0.5, decay_steps=1):
    """lr0 * exp(-decay_rate * floor(k / decay_steps)) (optimizer.py:270-293)."""
    return lambda k: lr0 * np.exp(-decay_rate * np.floor(k / decay_steps))


def _lr(lr, k):
    return float(lr(k) if callable(lr) else lr)


class Sga:
    """theta + lr_k * grad (optimizer.py:61-108)."""

    def __init__(self, lr):
        self.lr = lr

    def apply(self, theta, grad, k):
        return theta + _lr(self.lr, k) * grad


class ExpSga:
    """theta * exp(lr_k * grad), then theta / sum(theta) if ``normalize`` (optimizer.py:110-167)."""

    def __init__(self, lr, normalize=False):
        self.lr, self.normalize = lr, normalize

    def apply(self, theta, grad, k):
        new = theta * torch.exp(_lr(self.lr, k) * grad)
        if self.normalize:
            new = new / new.sum(dim=1, keepdim=True)
        return new


class NormalizeGrad:
    """Steps ``opt`` with grad / np.linalg.norm(grad, ord) per instance (optimizer.py:170-214)."""

    def __init__(self, opt, ord=None):
        self.opt, self.ord = opt, ord

    def apply(self, theta, grad, k):
        o = 2 if self.ord is None else self.ord
        norm = torch.linalg.vector_norm(grad, ord=o, dim=1, keepdim=True)
        return self.opt.apply(theta, grad / norm, k)
