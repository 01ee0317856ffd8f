"""NumPy neural networks with explicit backprop (``DL_Basics/ANN_Basics.ipynb``, sections
"基于NumPy的神经网络构建与训练": y=wx+b, y=Xw+b, two-layer / two-hidden-layer nets, multi-epoch
loop, mini-batches, regularisation; and the optimiser comparison of "优化器 / 自适应学习率").

Everything is float64 NumPy so gradients can be checked against ``torch.autograd`` exactly.
Parameters live in a flat ``dict[str, ndarray]`` (``W0, b0, W1, b1, …``); optimisers update that
dict in place from a same-keyed gradient dict.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------- activations


def _act(name: str, z: np.ndarray) -> np.ndarray:
    if name == "relu":
        return np.maximum(z, 0.0)
    if name == "sigmoid":
        return 1.0 / (1.0 + np.exp(-z))
    if name == "tanh":
        return np.tanh(z)
    if name in ("identity", "linear", None):
        return z
    raise ValueError(f"unknown activation {name!r}")


def _act_grad(name: str, z: np.ndarray, a: np.ndarray) -> np.ndarray:
    """d act / d z given pre-activation ``z`` and output ``a``."""
    if name == "relu":
        return (z > 0).astype(z.dtype)
    if name == "sigmoid":
        return a * (1.0 - a)
    if name == "tanh":
        return 1.0 - a * a
    return np.ones_like(z)

# ----------------------------------------------------------------------------- losses


def mse_loss(pred: np.ndarray, y: np.ndarray) -> tuple[float, np.ndarray]:
    d = pred - y
    return float(np.mean(d * d)), 2.0 * d / d.size


def softmax(z: np.ndarray) -> np.ndarray:
    e = np.exp(z - z.max(axis=-1, keepdims=True))
    return e / e.sum(axis=-1, keepdims=True)


def cross_entropy_loss(logits: np.ndarray, labels: np.ndarray) -> tuple[float, np.ndarray]:
    """Mean softmax cross entropy over rows; ``labels`` are class indices (nn.CrossEntropyLoss)."""
    n = logits.shape[0]
    p = softmax(logits)
    loss = -np.mean(np.log(p[np.arange(n), labels] + 1e-300))
    g = p.copy()
    g[np.arange(n), labels] -= 1.0
    return float(loss), g / n


def bce_with_logits_loss(logits: np.ndarray, y: np.ndarray) -> tuple[float, np.ndarray]:
    """Numerically stable nn.BCEWithLogitsLoss (mean)."""
    loss = np.maximum(logits, 0) - logits * y + np.log1p(np.exp(-np.abs(logits)))
    return float(loss.mean()), (1.0 / (1.0 + np.exp(-logits)) - y) / y.size


def huber_loss(pred: np.ndarray, y: np.ndarray, delta: float = 1.0) -> tuple[float, np.ndarray]:
    d = pred - y
    a = np.abs(d)
    loss = np.where(a <= delta, 0.5 * d * d, delta * (a - 0.5 * delta))
    return float(loss.mean()), np.where(a <= delta, d, delta * np.sign(d)) / d.size


LOSSES = {"mse": mse_loss, "ce": cross_entropy_loss, "bce": bce_with_logits_loss, "huber": huber_loss}

# ----------------------------------------------------------------------------- model


class MLP:
    """Fully connected net ``sizes[0] → … → sizes[-1]``; ``act`` between layers, linear output.

    ``forward`` caches (z, a) per layer; ``backward(dout)`` returns the gradient dict and adds the
    L2 term ``l2 · W`` (weights only — the notebook's "正则化机制").
    """

    def __init__(self, sizes: list[int], act: str = "relu", init: str = "he", seed: int = 0,
                 l2: float = 0.0):
        rng = np.random.default_rng(seed)
        self.sizes, self.act, self.l2 = list(sizes), act, l2
        self.params: dict[str, np.ndarray] = {}
        for i, (fi, fo) in enumerate(zip(sizes[:-1], sizes[1:])):
            std = np.sqrt(2.0 / fi) if init == "he" else np.sqrt(2.0 / (fi + fo))   # He / Xavier normal
            self.params[f"W{i}"] = rng.normal(0.0, std, (fi, fo))
            self.params[f"b{i}"] = np.zeros(fo)
        self._cache: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []

    @property
    def n_layers(self) -> int:
        return len(self.sizes) - 1

    def forward(self, x: np.ndarray) -> np.ndarray:
        self._cache = []
        a = x
        for i in range(self.n_layers):
            z = a @ self.params[f"W{i}"] + self.params[f"b{i}"]
            out = z if i == self.n_layers - 1 else _act(self.act, z)
            self._cache.append((a, z, out))
            a = out
        return a

    __call__ = forward

    def backward(self, dout: np.ndarray) -> dict[str, np.ndarray]:
        grads: dict[str, np.ndarray] = {}
        g = dout
        for i in reversed(range(self.n_layers)):
            a_in, z, out = self._cache[i]
            if i != self.n_layers - 1:
                g = g * _act_grad(self.act, z, out)
            grads[f"W{i}"] = a_in.T @ g + self.l2 * self.params[f"W{i}"]
            grads[f"b{i}"] = g.sum(axis=0)
            g = g @ self.params[f"W{i}"].T
        self.dx = g
        return grads

    def l2_penalty(self) -> float:
        return 0.5 * self.l2 * sum(float(np.sum(self.params[f"W{i}"] ** 2)) for i in range(self.n_layers))

# ----------------------------------------------------------------------------- optimisers


class SGD:
    def __init__(self, params: dict, lr: float = 0.01):
        self.params, self.lr = params, lr

    def step(self, grads: dict) -> None:
        for k, g in grads.items():
            self.params[k] -= self.lr * g


class Momentum(SGD):
    """torch.optim.SGD(momentum=μ): v = μ v + g; p -= lr v."""

    def __init__(self, params: dict, lr: float = 0.01, momentum: float = 0.9):
        super().__init__(params, lr)
        self.mu, self.v = momentum, {k: np.zeros_like(p) for k, p in params.items()}

    def step(self, grads: dict) -> None:
        for k, g in grads.items():
            self.v[k] = self.mu * self.v[k] + g
            self.params[k] -= self.lr * self.v[k]


class AdaGrad(SGD):
    def __init__(self, params: dict, lr: float = 0.01, eps: float = 1e-10):
        super().__init__(params, lr)
        self.eps, self.s = eps, {k: np.zeros_like(p) for k, p in params.items()}

    def step(self, grads: dict) -> None:
        for k, g in grads.items():
            self.s[k] += g * g
            self.params[k] -= self.lr * g / (np.sqrt(self.s[k]) + self.eps)


class RMSProp(SGD):
    def __init__(self, params: dict, lr: float = 0.01, alpha: float = 0.99, eps: float = 1e-8):
        super().__init__(params, lr)
        self.alpha, self.eps, self.s = alpha, eps, {k: np.zeros_like(p) for k, p in params.items()}

    def step(self, grads: dict) -> None:
        for k, g in grads.items():
            self.s[k] = self.alpha * self.s[k] + (1 - self.alpha) * g * g
            self.params[k] -= self.lr * g / (np.sqrt(self.s[k]) + self.eps)


class Adam(SGD):
    """torch.optim.Adam semantics (bias-corrected moments, eps outside the sqrt)."""

    def __init__(self, params: dict, lr: float = 1e-3, betas: tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8):
        super().__init__(params, lr)
        self.b1, self.b2, self.eps, self.t = betas[0], betas[1], eps, 0
        self.m = {k: np.zeros_like(p) for k, p in params.items()}
        self.v = {k: np.zeros_like(p) for k, p in params.items()}

    def step(self, grads: dict) -> None:
        self.t += 1
        c1, c2 = 1 - self.b1 ** self.t, 1 - self.b2 ** self.t
        for k, g in grads.items():
            self.m[k] = self.b1 * self.m[k] + (1 - self.b1) * g
            self.v[k] = self.b2 * self.v[k] + (1 - self.b2) * g * g
            self.params[k] -= self.lr * (self.m[k] / c1) / (np.sqrt(self.v[k] / c2) + self.eps)


OPTIMIZERS = {"sgd": SGD, "momentum": Momentum, "adagrad": AdaGrad, "rmsprop": RMSProp, "adam": Adam}

# ----------------------------------------------------------------------------- training loop


def train_mlp(model: MLP, x: np.ndarray, y: np.ndarray, *, loss: str = "mse", optimizer: str = "adam",
              lr: float = 1e-2, epochs: int = 100, batch_size: int | None = None, seed: int = 0,
              patience: int | None = None, x_val: np.ndarray | None = None,
              y_val: np.ndarray | None = None) -> dict[str, list[float]]:
    """Multi-epoch mini-batch training (``batch_size=None`` → full batch) with optional early
    stopping on a validation set (the notebook's "早停法"). Returns ``{"train": [...], "val": [...]}``."""
    rng = np.random.default_rng(seed)
    loss_fn = LOSSES[loss]
    opt = OPTIMIZERS[optimizer](model.params, lr=lr)
    hist: dict[str, list[float]] = {"train": [], "val": []}
    n = x.shape[0]
    bs = batch_size or n
    best, best_params, bad = np.inf, None, 0
    for _ in range(epochs):
        perm = rng.permutation(n)
        tot = 0.0
        for s in range(0, n, bs):
            idx = perm[s:s + bs]
            val, dout = loss_fn(model.forward(x[idx]), y[idx])
            opt.step(model.backward(dout))
            tot += (val + model.l2_penalty()) * idx.size
        hist["train"].append(tot / n)
        if x_val is not None:
            v, _ = loss_fn(model.forward(x_val), y_val)
            hist["val"].append(v)
            if patience is not None:
                if v < best - 1e-12:
                    best, bad = v, 0
                    best_params = {k: p.copy() for k, p in model.params.items()}
                else:
                    bad += 1
                    if bad >= patience:
                        model.params.update(best_params)
                        break
    return hist


def fit_linear(x: np.ndarray, y: np.ndarray, lr: float = 0.1, epochs: int = 200) -> tuple[np.ndarray, np.ndarray]:
    """Notebook examples 1-2: gradient descent on ``y = Xw + b`` with MSE; returns (w, b)."""
    x2 = x.reshape(len(x), -1)
    y2 = y.reshape(len(y), -1)
    w = np.zeros((x2.shape[1], y2.shape[1]))
    b = np.zeros(y2.shape[1])
    for _ in range(epochs):
        _, d = mse_loss(x2 @ w + b, y2)
        w -= lr * x2.T @ d
        b -= lr * d.sum(axis=0)
    return w, b
