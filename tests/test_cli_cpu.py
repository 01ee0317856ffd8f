"""CLI smoke tests (CPU): every track's entry point runs end to end on tiny configs."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from llm_in_practise_amd.cli.main import main


def test_minigpt_train_and_generate(tmp_path, capsys):
    ck = str(tmp_path / "mg.pth")
    main(["minigpt-train", "--epochs", "30", "--out", ck])
    first = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert first["final_loss"] < 1.0
    ckd = torch.load(ck, weights_only=True)
    assert set(ckd) == {"model_state", "char2idx", "config"}
    main(["minigpt-generate", "--checkpoint", ck, "--max_new", "10"])
    assert capsys.readouterr().out.startswith("马哥")


def test_minigpt2_train_and_test(tmp_path, capsys):
    ck = str(tmp_path / "m2.pth")
    main(["minigpt2-train", "--epochs", "2", "--out", ck])
    capsys.readouterr()
    main(["minigpt2-test", "--checkpoint", ck, "--max_new", "5"])
    assert len(capsys.readouterr().out.strip()) >= 2


@pytest.mark.parametrize("model", ["gptlike", "deepseek", "simple"])
def test_lm_train(tmp_path, capsys, model):
    main(["lm-train", "--model", model, "--tokenizer", "byte", "--block_size", "32", "--n_layer", "1",
          "--d_model", "64", "--n_head", "4", "--batch_size", "4", "--epochs", "1", "--max_steps", "3",
          "--save_dir", str(tmp_path / "ck"), "--scheduler", "step", "--step_per_batch"])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["train_loss"][0] > 0
    ck = torch.load(tmp_path / "ck" / "model_epoch_1.pth", weights_only=True)
    assert {"epoch", "model_state_dict", "optimizer_state_dict", "vocab_size", "block_size"} <= set(ck)


def test_lm_train_val_best_earlystop_resume(tmp_path, capsys, monkeypatch):
    """C6 (temp/ddp_gpt_bpe_tokenizer_02.py): seeded validation split, best_model.pt, early stopping
    on validation loss, and resume from latest_checkpoint.pt reproducing the uninterrupted run."""
    base = ["lm-train", "--model", "gptlike", "--tokenizer", "byte", "--block_size", "32", "--n_layer", "1",
            "--d_model", "64", "--n_head", "4", "--batch_size", "4", "--val_fraction", "0.2",
            "--scheduler", "cosine", "--dropout", "0.0"]
    full = tmp_path / "full"
    main(base + ["--epochs", "3", "--save_dir", str(full), "--best_model", str(full / "best_model.pt")])
    ref = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert len(ref["eval_loss"]) == 3 and (full / "best_model.pt").exists()
    part = tmp_path / "part"
    per_epoch = ref["global_step"] // 3
    monkeypatch.setenv("FAULT_INJECT", f"*:{2 * per_epoch + 1}:raise")   # crash in epoch 3
    from llm_in_practise_amd.utils.faults import InjectedFault
    with pytest.raises(InjectedFault):
        main(base + ["--epochs", "3", "--save_dir", str(part)])
    monkeypatch.delenv("FAULT_INJECT")
    capsys.readouterr()
    main(base + ["--epochs", "3", "--save_dir", str(part), "--resume"])
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["train_loss"] == pytest.approx(ref["train_loss"], rel=1e-5)
    assert res["eval_loss"] == pytest.approx(ref["eval_loss"], rel=1e-5)
    main(base + ["--epochs", "6", "--lr", "0", "--patience", "1", "--save_dir", str(tmp_path / "es")])
    es = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert len(es["train_loss"]) == 2      # lr 0: no val improvement after epoch 1 → stop after epoch 2


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pretrain_worker(rank, world, port, strategy, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    main(["pretrain", "--strategy", strategy, "--tokenizer", "byte", "--block_size", "32", "--n_layer", "2",
          "--d_model", "64", "--n_head", "4", "--batch_size", "2", "--epochs", "1", "--max_steps", "2",
          "--save_dir", d, "--final_model", os.path.join(d, "final_model.pth")])


@pytest.mark.parametrize("strategy", ["ddp", "zero2", "fsdp"])
def test_pretrain_strategies_world2(tmp_path, strategy):
    d = str(tmp_path / strategy)
    mp.spawn(_pretrain_worker, args=(2, _port(), strategy, d), nprocs=2, join=True)
    assert os.path.exists(os.path.join(d, "final_model.pth"))
    if strategy != "ddp":
        assert os.path.exists(os.path.join(d, "latest"))


def test_finetune_random_init_qlora(tmp_path):
    out = str(tmp_path / "ft")
    main(["finetune", "--preset", "qwen3-8b-qlora-dist", "--random-init", "qwen3-tiny", "--max-steps", "2",
          "--output-dir", out, "--synthetic-samples", "8", "--no-grad-ckpt"])
    assert os.path.exists(os.path.join(out, "adapter_model.safetensors"))
    assert os.path.exists(os.path.join(out, "train_results.json"))


def test_quantize_and_eval_cli(tmp_path, capsys):
    out = str(tmp_path / "q")
    main(["quantize", "--method", "awq", "--model", "random:qwen3-tiny", "--out", out, "--n_calib", "2",
          "--calib_len", "32"])
    assert json.load(open(os.path.join(out, "config.json")))["quantization_config"]["quant_method"] == \
        "compressed-tensors"
    capsys.readouterr()
    main(["eval-quant", "--model", out, "--start", "0", "--end", "2", "--max_new", "6"])
    r = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert r["self_ppl"] > 1


def test_convert_alpaca(tmp_path):
    src = tmp_path / "sc.jsonl"
    src.write_text(json.dumps({"query": "你是谁?", "response": "我是{{NAME}}，由{{AUTHOR}}开发。"}, ensure_ascii=False))
    out = tmp_path / "a.json"
    main(["convert-alpaca", "--input", str(src), "--out", str(out)])
    d = json.load(open(out))
    assert d[0]["instruction"] == "你是谁?" and "马哥教育AI小助手" in d[0]["output"]


def test_hf_classify_and_env(tmp_path, capsys):
    main(["hf-classify", "--epochs", "2", "--lr", "1e-3", "--output-dir", str(tmp_path / "r"), "--batch-size", "32"])
    assert os.path.exists(tmp_path / "r" / "eval_results.json")
    main(["env"])
    assert "torch" in capsys.readouterr().out


@pytest.mark.parametrize("par", [["-pp", "2"], ["-tp", "2"]])
def test_infer_tp_pp_under_torchrun(par, capsys):
    """`torchrun --nproc-per-node 2 lipa infer -pp 2 | -tp 2` prints the single-process greedy text."""
    import subprocess
    import sys
    args = ["infer", "--model", "random:qwen3-tiny", "--tokenizer", "bytes", "--prompt", "pipeline",
            "--temperature", "0", "--max_new", "8"]
    main(args)
    single = capsys.readouterr().out
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m",
                        "llm_in_practise_amd.cli.main", *args, *par],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.rstrip("\n").splitlines()[-1] == single.rstrip("\n")   # (gloo logs its connects first)


def test_teaching_notebook_commands(tmp_path):
    """lipa seq2seq-demo / nb-gpt (Chinese corpus directory) / minibert-imdb (JSONL) run end to end."""
    import json as _json
    import subprocess as _sp
    import sys as _sys
    d = tmp_path / "clue"
    d.mkdir()
    (d / "part0.txt").write_text("学习大模型训练与推理。\n马哥教育AI小助手。\n" * 4, encoding="utf-8")
    recs = tmp_path / "imdb.jsonl"
    recs.write_text("\n".join(_json.dumps({"text": ("great fun " if i % 2 else "awful boring ") * 3, "label": i % 2})
                              for i in range(40)))
    cmds = [["seq2seq-demo", "--steps", "20"],
            ["nb-gpt", "--data", str(d), "--n-layer", "1", "--n-embd", "32", "--n-head", "2", "--max-seq-len", "8",
             "--batch-size", "2", "--prompt", "马哥", "--gen-tokens", "3", "--save", str(tmp_path / "g.pt")],
            ["minibert-imdb", "--data", str(recs), "--epochs", "1", "--max-len", "32", "--hidden-size", "32",
             "--save", str(tmp_path / "b.pt")]]
    for c in cmds:
        r = _sp.run([_sys.executable, "-m", "llm_in_practise_amd.cli.main", *c], capture_output=True, text=True,
                    timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        out = _json.loads(r.stdout.strip().splitlines()[-1])
        assert out
    assert (tmp_path / "g.pt").exists() and (tmp_path / "b.pt").exists()
