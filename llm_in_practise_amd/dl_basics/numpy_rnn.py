"""Manual recurrent nets with BPTT (``DL_Basics/CNN_and_RNN.ipynb``: "RNN的前向传播 / 基于NumPy的RNN
示例 / 带前向传播和反向传播的示例 / RNN BPTT示例", "多时间步+batch_size=3的LSTM手动前向传播",
"手动实现GRU前向传播 / 多时间步，支持batch的GRU前向传播").

Layout is time-major ``x: (T, B, D)`` and the weights use PyTorch's packing so a
``torch.nn.RNN/LSTM/GRU`` state dict drops straight in (:func:`params_from_torch`):

* RNN  ``h' = tanh(W_ih x + b_ih + W_hh h + b_hh)``
* LSTM gates ``[i, f, g, o]`` stacked along rows of ``W_ih (4H, D)`` / ``W_hh (4H, H)``
* GRU  gates ``[r, z, n]``, ``n = tanh(W_in x + b_in + r ⊙ (W_hn h + b_hn))``, ``h' = (1-z) n + z h``

Each ``*_forward`` returns ``(H_all (T,B,H), cache)``; ``*_backward(dH_all, cache)`` runs
backpropagation through time and returns ``(dx, grads)`` with grads keyed like the params.
"""
from __future__ import annotations

import numpy as np


def _sig(z):
    return 1.0 / (1.0 + np.exp(-z))


def init_params(kind: str, d_in: int, hidden: int, seed: int = 0) -> dict[str, np.ndarray]:
    """U(-1/√H, 1/√H) like torch.nn.RNNBase.reset_parameters."""
    g = {"rnn": 1, "lstm": 4, "gru": 3}[kind]
    rng = np.random.default_rng(seed)
    k = 1.0 / np.sqrt(hidden)
    return {"W_ih": rng.uniform(-k, k, (g * hidden, d_in)), "W_hh": rng.uniform(-k, k, (g * hidden, hidden)),
            "b_ih": rng.uniform(-k, k, g * hidden), "b_hh": rng.uniform(-k, k, g * hidden)}


def params_from_torch(module, layer: int = 0) -> dict[str, np.ndarray]:
    sd = module.state_dict()
    return {k: sd[f"{k.replace('W_', 'weight_').replace('b_', 'bias_')}_l{layer}"].detach().double().numpy()
            for k in ("W_ih", "W_hh", "b_ih", "b_hh")}

# ----------------------------------------------------------------------------- vanilla RNN


def rnn_forward(x, p, h0=None):
    T, B, _ = x.shape
    H = p["W_hh"].shape[1]
    h = np.zeros((B, H)) if h0 is None else h0
    hs = [h]
    for t in range(T):
        h = np.tanh(x[t] @ p["W_ih"].T + p["b_ih"] + h @ p["W_hh"].T + p["b_hh"])
        hs.append(h)
    return np.stack(hs[1:]), (x, p, hs)


def rnn_backward(dH, cache):
    x, p, hs = cache
    grads = {k: np.zeros_like(v) for k, v in p.items()}
    dx = np.zeros_like(x)
    dh_next = np.zeros_like(hs[0])
    for t in reversed(range(x.shape[0])):
        da = (dH[t] + dh_next) * (1.0 - hs[t + 1] ** 2)
        grads["W_ih"] += da.T @ x[t]
        grads["W_hh"] += da.T @ hs[t]
        grads["b_ih"] += da.sum(0)
        grads["b_hh"] += da.sum(0)
        dx[t] = da @ p["W_ih"]
        dh_next = da @ p["W_hh"]
    return dx, grads, dh_next

# ----------------------------------------------------------------------------- LSTM


def lstm_forward(x, p, h0=None, c0=None):
    T, B, _ = x.shape
    H = p["W_hh"].shape[1]
    h = np.zeros((B, H)) if h0 is None else h0
    c = np.zeros((B, H)) if c0 is None else c0
    steps, out = [], []
    for t in range(T):
        a = x[t] @ p["W_ih"].T + p["b_ih"] + h @ p["W_hh"].T + p["b_hh"]
        i, f, g, o = _sig(a[:, :H]), _sig(a[:, H:2 * H]), np.tanh(a[:, 2 * H:3 * H]), _sig(a[:, 3 * H:])
        c_new = f * c + i * g
        tc = np.tanh(c_new)
        h_new = o * tc
        steps.append((h, c, i, f, g, o, tc))
        h, c = h_new, c_new
        out.append(h)
    return np.stack(out), (x, p, steps, c)


def lstm_backward(dH, cache, dc_last=None):
    x, p, steps, _ = cache
    grads = {k: np.zeros_like(v) for k, v in p.items()}
    dx = np.zeros_like(x)
    dh_next = np.zeros_like(steps[0][0])
    dc_next = np.zeros_like(dh_next) if dc_last is None else dc_last
    for t in reversed(range(x.shape[0])):
        h_prev, c_prev, i, f, g, o, tc = steps[t]
        dh = dH[t] + dh_next
        dc = dc_next + dh * o * (1.0 - tc * tc)
        da = np.concatenate([dc * g * i * (1 - i), dc * c_prev * f * (1 - f), dc * i * (1 - g * g),
                             dh * tc * o * (1 - o)], axis=1)
        grads["W_ih"] += da.T @ x[t]
        grads["W_hh"] += da.T @ h_prev
        grads["b_ih"] += da.sum(0)
        grads["b_hh"] += da.sum(0)
        dx[t] = da @ p["W_ih"]
        dh_next = da @ p["W_hh"]
        dc_next = dc * f
    return dx, grads, (dh_next, dc_next)

# ----------------------------------------------------------------------------- GRU


def gru_forward(x, p, h0=None):
    T, B, _ = x.shape
    H = p["W_hh"].shape[1]
    h = np.zeros((B, H)) if h0 is None else h0
    steps, out = [], []
    for t in range(T):
        gi = x[t] @ p["W_ih"].T + p["b_ih"]
        gh = h @ p["W_hh"].T + p["b_hh"]
        r = _sig(gi[:, :H] + gh[:, :H])
        z = _sig(gi[:, H:2 * H] + gh[:, H:2 * H])
        n = np.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
        steps.append((h, r, z, n, gh[:, 2 * H:]))
        h = (1.0 - z) * n + z * h
        out.append(h)
    return np.stack(out), (x, p, steps)


def gru_backward(dH, cache):
    x, p, steps = cache
    grads = {k: np.zeros_like(v) for k, v in p.items()}
    dx = np.zeros_like(x)
    dh_next = np.zeros_like(steps[0][0])
    for t in reversed(range(x.shape[0])):
        h_prev, r, z, n, ghn = steps[t]
        dh = dH[t] + dh_next
        dan = dh * (1.0 - z) * (1.0 - n * n)
        daz = dh * (h_prev - n) * z * (1.0 - z)
        dar = dan * ghn * r * (1.0 - r)
        dgi = np.concatenate([dar, daz, dan], axis=1)
        dgh = np.concatenate([dar, daz, dan * r], axis=1)
        grads["W_ih"] += dgi.T @ x[t]
        grads["W_hh"] += dgh.T @ h_prev
        grads["b_ih"] += dgi.sum(0)
        grads["b_hh"] += dgh.sum(0)
        dx[t] = dgi @ p["W_ih"]
        dh_next = dh * z + dgh @ p["W_hh"]
    return dx, grads, dh_next


FORWARD = {"rnn": rnn_forward, "lstm": lstm_forward, "gru": gru_forward}
BACKWARD = {"rnn": rnn_backward, "lstm": lstm_backward, "gru": gru_backward}


def train_sequence_regressor(kind: str = "lstm", T: int = 12, B: int = 16, hidden: int = 16, steps: int = 300,
                             lr: float = 0.05, seed: int = 0) -> list[float]:
    """BPTT demo: predict the (normalised) sum of a noisy scalar sequence from the last hidden state
    through a linear head; plain SGD with global-norm clipping 1.0.  Returns per-step losses."""
    rng = np.random.default_rng(seed)
    p = init_params(kind, 1, hidden, seed)
    w = rng.normal(0, 0.1, (hidden, 1))
    b = np.zeros(1)
    losses = []
    for _ in range(steps):
        x = rng.normal(0, 1, (T, B, 1))
        y = x.sum(axis=0) / np.sqrt(T)            # unit-variance target that needs every step
        Hs, cache = FORWARD[kind](x, p)
        pred = Hs[-1] @ w + b
        d = pred - y
        losses.append(float(np.mean(d * d)))
        dpred = 2 * d / d.size
        dH = np.zeros_like(Hs)
        dH[-1] = dpred @ w.T
        _, g, _ = BACKWARD[kind](dH, cache)
        g["w"], g["b"] = Hs[-1].T @ dpred, dpred.sum(0)
        norm = np.sqrt(sum(float(np.sum(v * v)) for v in g.values()))
        s = min(1.0, 1.0 / (norm + 1e-6))
        for k in p:
            p[k] -= lr * s * g[k]
        w -= lr * s * g["w"]
        b -= lr * s * g["b"]
    return losses
