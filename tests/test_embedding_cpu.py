"""ops.Embedding is a drop-in nn.Embedding (same parameter / state-dict key, same CPU numerics)."""
import torch

from llm_in_practise_amd.ops.embedding import Embedding


def test_embedding_is_drop_in_on_cpu():
    torch.manual_seed(0)
    ref = torch.nn.Embedding(20, 16, padding_idx=2)
    ours = Embedding(20, 16, padding_idx=2)
    ours.load_state_dict(ref.state_dict())
    assert list(ours.state_dict()) == ["weight"] and isinstance(ours, torch.nn.Embedding)
    ids = torch.tensor([[1, 2, 3, 1], [2, 5, 19, 0]])
    y0, y1 = ref(ids), ours(ids)
    assert torch.equal(y0, y1)
    g = torch.randn_like(y0)
    y0.backward(g)
    y1.backward(g)
    assert torch.equal(ref.weight.grad, ours.weight.grad)


def test_models_use_native_embedding():
    from llm_in_practise_amd.models.gptlike import GPTLike
    m = GPTLike(vocab_size=50, d_model=32, n_head=4, n_layer=1, block_size=16)
    assert isinstance(m.tok_emb, Embedding)
