"""Transformer_Basics notebook models (cells 20-41): enc-dec Transformer, decoder-only, MiniBert
IMDb-style classifier, notebook GPT (WikiText / Chinese CLUECorpusSmall drivers) on CPU."""
import random

import torch

from llm_in_practise_amd.models.teaching import (DecoderOnlyTransformer, MiniBert, NotebookGPT, NotebookGPTConfig,
                                                 Seq2SeqTransformer)
from llm_in_practise_amd.train.data import CharTokenizer
from llm_in_practise_amd.train.teaching import (MiniBertConfig, train_minibert_classifier, train_notebook_gpt,
                                                train_seq2seq)


def test_forward_shapes_match_notebook_cells():
    torch.manual_seed(0)
    t = Seq2SeqTransformer(10000, 8000, d_model=64, num_heads=4, d_ff=256, num_layers=2)     # cell 22 demo
    src, tgt = torch.randint(1, 10000, (2, 10)), torch.randint(1, 8000, (2, 7))
    assert t(src, tgt).shape == (2, 7, 8000)
    d = DecoderOnlyTransformer(10000, 64, 4, 256, 2)                                        # cell 24 demo
    assert d(torch.randint(0, 10000, (2, 9))).shape == (2, 9, 10000)
    b = MiniBert(200, hidden_size=64, num_heads=4, num_layers=2, ffn_size=128, max_len=50, num_classes=2)
    assert b(torch.randint(0, 200, (3, 20)), torch.ones(3, 20, dtype=torch.long)).shape == (3, 2)
    g = NotebookGPT(NotebookGPTConfig(vocab_size=21128, n_layer=2, max_seq_len=32))        # cell 41 vocab
    out = g.generate(torch.zeros(1, 4, dtype=torch.long), 5, generator=torch.Generator().manual_seed(0))
    assert out.shape == (1, 9)


def test_decoder_causality():
    """position i's output must not depend on later tokens (triu mask)"""
    torch.manual_seed(0)
    d = DecoderOnlyTransformer(50, 32, 4, 64, 2).eval()
    x = torch.randint(0, 50, (1, 8))
    y = x.clone()
    y[0, 5:] = (y[0, 5:] + 7) % 50
    assert torch.allclose(d(x)[0, :5], d(y)[0, :5], atol=1e-5)


def test_seq2seq_learns_reversal():
    _, losses, acc = train_seq2seq(steps=400, vocab=10, length=5, d_model=64, num_layers=2, device=torch.device("cpu"))
    assert losses[-1] < 0.5 * losses[0] and acc > 0.5


def test_minibert_learns_sentiment_rule():
    rng = random.Random(0)
    pos_w, neg_w, filler = ["great", "good", "fun"], ["bad", "awful", "boring"], ["the", "movie", "was", "plot", "a"]

    def rec():
        lab = rng.random() < 0.5
        words = [rng.choice(filler) for _ in range(rng.randint(3, 10))]
        words.insert(rng.randrange(len(words) + 1), rng.choice(pos_w if lab else neg_w))
        return {"text": " ".join(words), "label": int(lab)}
    train, test = [rec() for _ in range(400)], [rec() for _ in range(100)]
    tok = CharTokenizer("".join(r["text"] for r in train + test))
    cfg = MiniBertConfig(hidden_size=64, num_layers=2, ffn_size=128, max_len=64, epochs=6, dropout=0.0)
    h = train_minibert_classifier(train, test, tok, cfg, device=torch.device("cpu"), pad_id=0)
    assert h["test_acc"][-1] > 0.85, h["test_acc"]


def test_chinese_notebook_gpt_trains_and_generates():
    text = ["马哥教育AI小助手正在学习大语言模型的训练与推理。"] * 60
    tok = CharTokenizer("".join(text))
    out = train_notebook_gpt(text, tok, NotebookGPTConfig(vocab_size=tok.vocab_size, n_embd=64, n_head=4, n_layer=2,
                                                          max_seq_len=16, dropout=0.0),
                             epochs=8, batch_size=8, lr=3e-3, prompt="马哥", gen_tokens=8, device=torch.device("cpu"))
    assert out["losses"][-1] < 0.3 * out["losses"][0]
    assert out["sample"].startswith("马哥") and len(out["sample"]) == 10
