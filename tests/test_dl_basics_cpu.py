"""DL basics track: NumPy backprop / BPTT / conv checked against torch autograd."""
import numpy as np
import pytest
import torch

from llm_in_practise_amd.dl_basics import numpy_cnn as C
from llm_in_practise_amd.dl_basics import numpy_nn as N
from llm_in_practise_amd.dl_basics import numpy_rnn as R
from llm_in_practise_amd.dl_basics import seq2seq as S


@pytest.mark.parametrize("act", ["relu", "sigmoid", "tanh"])
@pytest.mark.parametrize("loss", ["mse", "ce", "huber"])
def test_mlp_backprop_matches_autograd(act, loss):
    rng = np.random.default_rng(0)
    m = N.MLP([5, 7, 6, 3], act=act, l2=0.01, seed=1)
    x = rng.normal(size=(8, 5))
    y = rng.integers(0, 3, 8) if loss == "ce" else rng.normal(size=(8, 3))
    val, d = N.LOSSES[loss](m.forward(x), y)
    g = m.backward(d)

    tp = {k: torch.tensor(v, requires_grad=True) for k, v in m.params.items()}
    a = torch.tensor(x, requires_grad=True)
    for i in range(m.n_layers):
        a = a @ tp[f"W{i}"] + tp[f"b{i}"]
        if i < m.n_layers - 1:
            a = getattr(torch, act)(a)
    ty = torch.tensor(y)
    tl = {"mse": lambda: torch.nn.functional.mse_loss(a, ty), "ce": lambda: torch.nn.functional.cross_entropy(a, ty),
          "huber": lambda: torch.nn.functional.huber_loss(a, ty)}[loss]()
    (tl + 0.5 * 0.01 * sum((tp[f"W{i}"] ** 2).sum() for i in range(3))).backward()
    assert abs(val - tl.item()) < 1e-10
    for k in tp:
        np.testing.assert_allclose(g[k], tp[k].grad.numpy(), rtol=1e-7, atol=1e-10)


def test_bce_with_logits_matches_torch():
    rng = np.random.default_rng(0)
    z, y = rng.normal(size=(6, 2)) * 4, rng.integers(0, 2, (6, 2)).astype(float)
    val, g = N.bce_with_logits_loss(z, y)
    tz = torch.tensor(z, requires_grad=True)
    tl = torch.nn.functional.binary_cross_entropy_with_logits(tz, torch.tensor(y))
    tl.backward()
    assert abs(val - tl.item()) < 1e-12
    np.testing.assert_allclose(g, tz.grad.numpy(), rtol=1e-9)


@pytest.mark.parametrize("name,kw,tcls", [("sgd", {}, torch.optim.SGD), ("momentum", {"momentum": 0.9}, torch.optim.SGD),
                                         ("adagrad", {}, torch.optim.Adagrad), ("rmsprop", {}, torch.optim.RMSprop),
                                         ("adam", {}, torch.optim.Adam)])
def test_optimizers_match_torch(name, kw, tcls):
    rng = np.random.default_rng(0)
    p = {"w": rng.normal(size=(4, 3))}
    tw = torch.tensor(p["w"].copy(), requires_grad=True)
    opt = N.OPTIMIZERS[name](p, lr=0.05, **kw)
    topt = tcls([tw], lr=0.05, **kw)
    for _ in range(5):
        g = rng.normal(size=(4, 3))
        opt.step({"w": g})
        tw.grad = torch.tensor(g)
        topt.step()
    np.testing.assert_allclose(p["w"], tw.detach().numpy(), rtol=1e-6, atol=1e-8)


def test_mlp_learns_xor_minibatch_and_linear_fit():
    x = np.array([[0, 0], [0, 1], [1, 0], [1, 1]], float).repeat(8, 0)
    y = (x[:, 0] != x[:, 1]).astype(int)
    m = N.MLP([2, 16, 2], act="tanh", init="xavier", seed=0)
    hist = N.train_mlp(m, x, y, loss="ce", optimizer="adam", lr=0.05, epochs=200, batch_size=8)
    assert hist["train"][-1] < 0.05
    assert (m.forward(x).argmax(1) == y).all()
    xs = np.linspace(-1, 1, 50)
    w, b = N.fit_linear(xs, 3 * xs + 0.5, lr=0.5, epochs=300)
    assert abs(w.item() - 3) < 1e-3 and abs(b.item() - 0.5) < 1e-3


def test_early_stopping_restores_best():
    rng = np.random.default_rng(0)
    x, y = rng.normal(size=(20, 3)), rng.normal(size=(20, 1))
    m = N.MLP([3, 64, 1], seed=0)
    hist = N.train_mlp(m, x, y, lr=0.05, epochs=500, patience=5, x_val=rng.normal(size=(20, 3)),
                       y_val=rng.normal(size=(20, 1)))
    assert len(hist["val"]) < 500


@pytest.mark.parametrize("kind", ["rnn", "lstm", "gru"])
def test_manual_rnn_forward_bptt_match_torch(kind):
    torch.manual_seed(0)
    T, B, D, H = 5, 3, 4, 6
    mod = {"rnn": torch.nn.RNN, "lstm": torch.nn.LSTM, "gru": torch.nn.GRU}[kind](D, H).double()
    p = R.params_from_torch(mod)
    x = np.random.default_rng(1).normal(size=(T, B, D))
    Hs, cache = R.FORWARD[kind](x, p)
    tx = torch.tensor(x, requires_grad=True)
    th, _ = mod(tx)
    np.testing.assert_allclose(Hs, th.detach().numpy(), rtol=1e-10, atol=1e-12)
    dH = np.random.default_rng(2).normal(size=Hs.shape)
    dx, g, _ = R.BACKWARD[kind](dH, cache)
    th.backward(torch.tensor(dH))
    np.testing.assert_allclose(dx, tx.grad.numpy(), rtol=1e-8, atol=1e-10)
    names = {"W_ih": "weight_ih_l0", "W_hh": "weight_hh_l0", "b_ih": "bias_ih_l0", "b_hh": "bias_hh_l0"}
    for k, tn in names.items():
        np.testing.assert_allclose(g[k], getattr(mod, tn).grad.numpy(), rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("kind", ["rnn", "lstm", "gru"])
def test_bptt_training_reduces_loss(kind):
    losses = R.train_sequence_regressor(kind, steps=200)
    assert np.mean(losses[-20:]) < 0.5 * np.mean(losses[:20])


@pytest.mark.parametrize("stride,pad", [(1, 0), (1, 2), (2, 1)])
def test_conv2d_forward_backward_match_torch(stride, pad):
    rng = np.random.default_rng(0)
    x, w, b = rng.normal(size=(2, 3, 9, 8)), rng.normal(size=(4, 3, 3, 3)), rng.normal(size=4)
    out, cache = C.conv2d_forward(x, w, b, stride, pad)
    tx, tw, tb = (torch.tensor(a, requires_grad=True) for a in (x, w, b))
    to = torch.nn.functional.conv2d(tx, tw, tb, stride=stride, padding=pad)
    np.testing.assert_allclose(out, to.detach().numpy(), rtol=1e-10, atol=1e-10)
    d = rng.normal(size=out.shape)
    dx, dw, db = C.conv2d_backward(d, cache)
    to.backward(torch.tensor(d))
    for mine, ref in ((dx, tx), (dw, tw), (db, tb)):
        np.testing.assert_allclose(mine, ref.grad.numpy(), rtol=1e-9, atol=1e-10)


def test_maxpool_forward_backward_match_torch():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(2, 3, 8, 6))
    out, cache = C.maxpool2d_forward(x, 2)
    tx = torch.tensor(x, requires_grad=True)
    to = torch.nn.functional.max_pool2d(tx, 2)
    np.testing.assert_allclose(out, to.detach().numpy())
    d = rng.normal(size=out.shape)
    to.backward(torch.tensor(d))
    np.testing.assert_allclose(C.maxpool2d_backward(d, cache), tx.grad.numpy())


def test_lenet5_shapes_and_step():
    net = C.LeNet5()
    x = torch.randn(4, 1, 28, 28)
    out = net(x)
    assert out.shape == (4, 10)
    torch.nn.functional.cross_entropy(out, torch.tensor([0, 1, 2, 3])).backward()
    assert all(p.grad is not None for p in net.parameters())


def test_seq2seq_bahdanau_learns_reversal():
    rng = np.random.default_rng(0)
    words = ["".join(rng.choice(list("abcdef"), rng.integers(3, 7))) for _ in range(400)]
    pairs = [(w, w[::-1]) for w in words]
    model, sv, tv, losses = S.train_seq2seq(pairs, epochs=25, batch_size=32, seed=0)
    assert losses[-1] < 0.25 * losses[0]
    test = [w for w, _ in pairs[:50]]
    acc = np.mean([o == w[::-1] for o, w in zip(S.translate(model, sv, tv, test), test)])
    assert acc > 0.7, acc
    src, lens, _ = S.pad_collate([(sv.encode("abc"), [S.EOS])])
    _, attn = model.greedy_decode(src, lens, 4)
    assert torch.allclose(attn.sum(-1), torch.ones(1, 4)) and attn.shape == (1, 4, src.shape[1])


@pytest.mark.parametrize("demo", ["mlp", "optimizers", "rnn", "cnn"])
def test_cli_dl_basics(demo, capsys):
    from llm_in_practise_amd.cli.main import main
    main(["dl-basics", demo, "--epochs", "3"])
    assert '"demo"' in capsys.readouterr().out


def test_glove_embedding(tmp_path):
    from llm_in_practise_amd.dl_basics.embeddings import build_embedding
    p = tmp_path / "glove.txt"
    p.write_text("the 0.1 0.2 0.3\ncat -1 0.5 2\nbad 1 2\nzebra 9 9 9\n")
    vocab = {"<pad>": 0, "the": 1, "cat": 2, "dog": 3}
    emb, n = build_embedding(vocab, 3, str(p), freeze=True)
    assert n == 2 and emb.weight.shape == (4, 3) and not emb.weight.requires_grad
    assert torch.allclose(emb.weight[2], torch.tensor([-1.0, 0.5, 2.0]))
    assert torch.all(emb.weight[0] == 0) and emb.weight[3].abs().sum() > 0
