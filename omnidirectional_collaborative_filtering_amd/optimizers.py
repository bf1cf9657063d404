"""Keras 2.0.4 optimizer surface (train.py:12,50-51; train_jester.py:61).

Only the hyper-parameters live here; the update itself runs on the GPU inside the weight-gradient
GEMM epilogue (``OCF_EPI_OPTIM``) or ``ocf_opt_step``.  ``step_params()`` turns the Keras
schedule (decay, Adam bias correction) into the per-step scalars the kernels take.
"""
from __future__ import annotations

import math

from . import _lib


class Optimizer:
    kind = _lib.OPT_SGD
    n_slots = 0

    def __init__(self, lr=0.01, decay=0.0, **kw):
        self.lr = float(lr)
        self.decay = float(decay)
        self.iterations = 0
        self.extra = kw

    def _lr(self):
        lr = self.lr
        if self.decay > 0:
            lr = lr * (1.0 / (1.0 + self.decay * self.iterations))
        return lr

    def step_params(self, gscale=1.0, l2=0.0):
        o = _lib.OcfOptParams()
        o.kind = self.kind
        o.lr = self._lr()
        o.eps = getattr(self, "epsilon", 1e-8)
        o.rho = 0.0
        o.beta2 = 0.0
        o.l2 = float(l2 or 0.0)
        o.gscale = float(gscale)
        return o

    def get_config(self):
        return {"lr": self.lr, "decay": self.decay}


class SGD(Optimizer):
    kind = _lib.OPT_SGD


class Adagrad(Optimizer):
    """a += g^2; p -= lr*g/(sqrt(a)+eps)   (Keras 2.0.4 Adagrad.get_updates)."""
    kind = _lib.OPT_ADAGRAD
    n_slots = 1

    def __init__(self, lr=0.01, epsilon=1e-8, decay=0.0):
        super().__init__(lr, decay)
        self.epsilon = float(epsilon)


class RMSprop(Optimizer):
    """a = rho*a + (1-rho)*g^2; p -= lr*g/(sqrt(a)+eps)."""
    kind = _lib.OPT_RMSPROP
    n_slots = 1

    def __init__(self, lr=0.001, rho=0.9, epsilon=1e-8, decay=0.0):
        super().__init__(lr, decay)
        self.rho = float(rho)
        self.epsilon = float(epsilon)

    def step_params(self, gscale=1.0, l2=0.0):
        o = super().step_params(gscale, l2)
        o.rho = self.rho
        return o


class Adam(Optimizer):
    """lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m,v EMAs; p -= lr_t*m/(sqrt(v)+eps)."""
    kind = _lib.OPT_ADAM
    n_slots = 2

    def __init__(self, lr=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-8, decay=0.0):
        super().__init__(lr, decay)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)

    def step_params(self, gscale=1.0, l2=0.0):
        o = super().step_params(gscale, l2)
        t = self.iterations + 1
        o.lr = self._lr() * (math.sqrt(1.0 - self.beta_2 ** t) / (1.0 - self.beta_1 ** t))
        o.rho = self.beta_1
        o.beta2 = self.beta_2
        return o


def get(identifier):
    """Keras string identifiers ('adagrad', 'rmsprop', 'adam', 'sgd') or an instance."""
    if isinstance(identifier, Optimizer):
        return identifier
    table = {"sgd": SGD, "adagrad": Adagrad, "rmsprop": RMSprop, "adam": Adam}
    key = str(identifier).lower()
    if key not in table:
        raise ValueError("unknown optimizer %r" % (identifier,))
    return table[key]()
