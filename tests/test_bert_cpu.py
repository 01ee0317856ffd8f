"""BERT classification (G5): HF-named encoder, Trainer eval/accuracy/best-model, dynamic padding."""
import torch

from llm_in_practise_amd.models.bert import BertConfig, BertForSequenceClassification, accuracy_metric
from llm_in_practise_amd.train.data import DataCollatorWithPadding
from llm_in_practise_amd.train.trainer import Trainer, TrainingArguments


class _Toy(torch.utils.data.Dataset):
    """Label = whether token 7 occurs — learnable by a tiny encoder."""

    def __init__(self, n, seed):
        g = torch.Generator().manual_seed(seed)
        self.rows = []
        for _ in range(n):
            L = int(torch.randint(6, 16, (1,), generator=g))
            ids = torch.randint(8, 60, (L,), generator=g)
            lab = int(torch.rand(1, generator=g) < 0.5)
            if lab:
                ids[int(torch.randint(1, L, (1,), generator=g))] = 7
            self.rows.append({"input_ids": [1] + ids.tolist(), "label": lab})

    def __len__(self):
        return len(self.rows)

    def __getitem__(self, i):
        return self.rows[i]


def test_bert_names_and_padding_invariance():
    c = BertConfig(vocab_size=64, hidden_size=32, num_hidden_layers=2, num_attention_heads=4, intermediate_size=64)
    m = BertForSequenceClassification(c).eval()
    names = set(m.state_dict())
    assert "bert.encoder.layer.1.attention.self.query.weight" in names and "classifier.weight" in names
    assert "bert.embeddings.LayerNorm.weight" in names and "bert.pooler.dense.bias" in names
    ids = torch.randint(2, 64, (1, 9))
    a = m(ids, torch.ones_like(ids)).logits
    padded = torch.cat([ids, torch.zeros(1, 5, dtype=torch.long)], 1)
    b = m(padded, torch.cat([torch.ones(1, 9), torch.zeros(1, 5)], 1).long()).logits
    assert torch.allclose(a, b, atol=1e-5)


def test_bert_trainer_learns_with_eval_and_best_model(tmp_path):
    torch.manual_seed(0)
    c = BertConfig(vocab_size=64, hidden_size=32, num_hidden_layers=2, num_attention_heads=4, intermediate_size=64,
                   hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForSequenceClassification(c)
    args = TrainingArguments(output_dir=str(tmp_path), per_device_train_batch_size=16, per_device_eval_batch_size=32,
                             num_train_epochs=6, learning_rate=3e-3, eval_strategy="epoch", save_strategy="epoch",
                             load_best_model_at_end=True, metric_for_best_model="accuracy", save_total_limit=1,
                             logging_steps=100, optim="adamw_torch")
    tr = Trainer(m, args, train_dataset=_Toy(256, 0), eval_dataset=_Toy(128, 1),
                 data_collator=DataCollatorWithPadding(pad_token_id=0), compute_metrics=accuracy_metric)
    tr.train()
    acc = tr.evaluate()["eval_accuracy"]
    assert acc > 0.8 and tr.state.best_metric >= acc - 1e-6
    assert tr.state.best_model_checkpoint is not None
