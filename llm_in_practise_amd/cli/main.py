"""``lipa`` — one entry point for every executable of the reference.

    lipa minigpt-train | minigpt-generate | minigpt2-train | minigpt2-test      (A1-A5)
    lipa lm-train --model {simple,gptlike,deepseek,deepseek-dense} ...           (B1-B6, single device)
    lipa pretrain --strategy {ddp,fsdp,fsdp2,zero1,zero2,zero3,zero-offload}     (C1-C6, D0-D6; torchrun)
    lipa finetune --preset qwen3-8b-qlora-dist ...                              (E1-E7, E11)
    lipa chat --base DIR [--adapter DIR]                                        (E8, G1, G2)
    lipa merge --base DIR --adapter DIR --out DIR                               (E10 export, E11 02/04, K19)
    lipa quantize --method {gptq,awq,rtn} --model DIR --out DIR [--format ...]  (F1-F4)
    lipa eval-quant --model DIR                                                  (F2b)
    lipa infer --model DIR --prompt TEXT                                        (F1b, F2c, G1)
    lipa serve --model DIR [--adapter DIR] [--port 8000]                        (G4, H1)
               [--enable-lora --lora-modules n1=dir1 n2=dir2] [--kv-host-cache-blocks N]
    lipa guard --backend URL [--port 8099]                                      (H3)
    lipa router --config deploy/litellm/config.yaml [--port 4000]               (H2 LiteLLM router)
    lipa convert-alpaca --input self_cognition.jsonl --out alpaca.json           (E10 converter)
    lipa hf-classify [--model-path bert-dir] [--data imdb.jsonl]                 (G5 Trainer demo)
    lipa dl-basics {mlp,optimizers,rnn,cnn,seq2seq}                            (B9 DL_Basics notebooks)
    lipa env                                                                     (G5 env_test)
    lipa bench ...                                                               (bench.py)

Datasets / checkpoints are LOCAL paths (no hub access); ``--random-init`` builds the named
architecture with random weights for smoke runs.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys

import torch


def _device(arg: str | None = None):
    if arg:
        return torch.device(arg)
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0))) if torch.cuda.is_available() else \
        torch.device("cpu")


# ============================================================================ track A
DEMO_TEXT = "马哥教育创立于2009年，是一家专注于云计算、SRE、DevOps、网络安全、Go开发和云原生课程培训的高端IT教育机构。"


def cmd_minigpt_train(a):
    from ..models.minigpt import MiniGPT
    from ..train.data import CharTokenizer, CharWindowDataset
    from ..train.loops import LoopConfig, train_lm
    text = open(a.text).read() if a.text else DEMO_TEXT
    tok = CharTokenizer(text)
    ds = CharWindowDataset(text, tok.stoi, a.seq_len, a.repeat)
    m = MiniGPT(tok.vocab_size, a.embed_dim, a.n_heads, a.n_layers, 0.1, a.seq_len,
                reference_layout=not a.causal, causal=a.causal).to(_device(a.device))
    hist = train_lm(m, ds, LoopConfig(epochs=a.epochs, batch_size=a.batch_size, lr=a.lr, weight_decay=0.01,
                                      clip_grad_norm=1.0, log_every=0, seed=a.seed))
    torch.save({"model_state": m.state_dict(), "char2idx": tok.stoi,
                "config": {"embed_dim": a.embed_dim, "seq_len": a.seq_len, "n_heads": a.n_heads,
                           "n_layers": a.n_layers, "causal": a.causal}}, a.out)
    print(json.dumps({"final_loss": hist["train_loss"][-1], "checkpoint": a.out}))


def cmd_minigpt_generate(a):
    from ..infer.generate import generate_simple
    from ..models.minigpt import MiniGPT
    ck = torch.load(a.checkpoint, map_location="cpu", weights_only=True)
    stoi = ck["char2idx"]
    itos = {i: c for c, i in stoi.items()}
    c = ck["config"]
    m = MiniGPT(len(stoi), c["embed_dim"], c.get("n_heads", 2), c.get("n_layers", 2), 0.1, c["seq_len"],
                reference_layout=not c.get("causal", False), causal=c.get("causal", False))
    m.load_state_dict(ck["model_state"])
    idx = torch.tensor([[stoi[ch] for ch in a.prompt if ch in stoi]])
    out = generate_simple(m, idx, a.max_new, c["seq_len"], temperature=a.temperature)
    print("".join(itos[int(i)] for i in out[0]))


def cmd_minigpt2_train(a):
    from ..models.minigpt import MiniGPT2, MiniGPT2Config
    from ..train.data import CharTokenizer, CharWindowDataset
    from ..train.loops import LoopConfig, train_lm
    text = open(a.text).read() if a.text else DEMO_TEXT
    tok = CharTokenizer(text)
    cfg = MiniGPT2Config(vocab_size=tok.vocab_size, seq_len=min(a.seq_len, max(2, len(text) - 1)))
    # the reference's dataset is empty when text < seq_len (minigpt2/model.py:111, ZeroDivisionError);
    # here the window shrinks to the text length instead
    ds = CharWindowDataset(text, tok.stoi, cfg.seq_len, 1)
    m = MiniGPT2(cfg).to(_device(a.device))
    hist = train_lm(m, ds, LoopConfig(epochs=a.epochs, batch_size=min(cfg.batch_size, len(ds)), lr=cfg.lr,
                                      weight_decay=cfg.weight_decay, log_every=0))
    torch.save({"model_state": m.state_dict(), "stoi": tok.stoi, "itos": {i: c for c, i in tok.stoi.items()},
                "config": cfg.__dict__}, a.out)
    print(json.dumps({"final_loss": hist["train_loss"][-1], "checkpoint": a.out}))


def cmd_minigpt2_test(a):
    from ..infer.generate import generate_simple
    from ..models.minigpt import MiniGPT2, MiniGPT2Config
    ck = torch.load(a.checkpoint, map_location="cpu", weights_only=True)
    cfg = MiniGPT2Config(**{k: v for k, v in ck["config"].items() if k in MiniGPT2Config.__dataclass_fields__})
    m = MiniGPT2(cfg)
    m.load_state_dict(ck["model_state"])
    stoi, itos = ck["stoi"], {int(k): v for k, v in ck["itos"].items()}
    x = torch.tensor([[stoi.get(ch, 0) for ch in a.prompt]])
    logits = m(torch.nn.functional.pad(x, (cfg.seq_len - x.shape[1], 0))[:, -cfg.seq_len:])
    assert logits.shape == (1, cfg.seq_len, cfg.vocab_size), "output shape test"
    out = generate_simple(m, x, a.max_new, cfg.seq_len, temperature=0.8, pad_left_to=cfg.seq_len)
    print("".join(itos.get(int(i), "?") for i in out[0]))


# ============================================================================ tracks B-D
def _lm_corpus(a):
    from ..train.data import (ByteBlocksDataset, ByteTokenizer, TokenBlockDataset, load_text_corpus,
                              train_bpe_tokenizer)
    texts = load_text_corpus(a.data) if a.data else [DEMO_TEXT * 40]
    if a.tokenizer == "byte":
        tok = ByteTokenizer()
        return ByteBlocksDataset(texts, a.block_size), tok
    if a.tokenizer.startswith("hf:"):
        from ..train.data import load_tokenizer
        tok = load_tokenizer(a.tokenizer[3:])
    else:
        tok = train_bpe_tokenizer(texts, a.vocab_size, "bytelevel" if a.tokenizer == "bpe-bytelevel" else "whitespace",
                                  save_path=os.path.join(a.save_dir or ".", "tokenizer.json"))
    ids = []
    for t in texts:
        ids.extend(tok.encode(t))
    return TokenBlockDataset(ids, a.block_size), tok


def _build_lm(a, vocab):
    from ..models.deepseeklike import DeepSeekLike
    from ..models.gptlike import GPTLike, SimpleTransformer
    if a.model == "simple":
        return SimpleTransformer(vocab, a.d_model, a.n_head, a.n_layer, a.block_size, a.dropout)
    if a.model.startswith("deepseek"):
        return DeepSeekLike(vocab, a.block_size, a.n_layer, a.n_head, a.d_model, a.dropout, a.latent_dim,
                            a.num_experts, a.top_k, a.num_shared, a.rope_theta,
                            moe_dispatch="dense" if a.model == "deepseek-dense" else "sparse")
    return GPTLike(vocab, a.block_size, a.n_layer, a.n_head, a.d_model, a.dropout,
                   pos="learned" if a.pe == "learned" else "sinusoidal")


def cmd_lm_train(a, strategy="single"):
    from ..parallel import dist as D
    from ..train.loops import LoopConfig, train_lm
    if strategy != "single":
        D.init_distributed(timeout_s=a.timeout)
    ds, tok = _lm_corpus(a)
    vocab = getattr(tok, "vocab_size", 256)
    torch.manual_seed(a.seed)
    m = _build_lm(a, vocab).to(_device())
    cfg = LoopConfig(epochs=a.epochs, batch_size=a.batch_size, lr=a.lr, weight_decay=a.weight_decay,
                     clip_grad_norm=a.clip_grad_norm, strategy=strategy, ds_config=a.ds_config,
                     precision=a.precision, scheduler=a.scheduler, step_per_batch=a.step_per_batch,
                     save_dir=a.save_dir, keep_last=a.keep_last, final_model=a.final_model, seed=a.seed,
                     max_steps=a.max_steps, grad_accum=a.grad_accum, patience=a.patience, best_model=a.best_model,
                     resume=a.resume, eval_every_epoch=a.val_fraction > 0,
                     no_decay_groups=getattr(a, "no_decay_groups", False))
    eval_ds = None
    if a.val_fraction > 0:       # temp/ddp_gpt_bpe_tokenizer_02.py:262-300: seeded random_split
        n_val = max(1, int(len(ds) * a.val_fraction))
        ds, eval_ds = torch.utils.data.random_split(ds, [len(ds) - n_val, n_val],
                                                    generator=torch.Generator().manual_seed(a.seed))
    hist = train_lm(m, ds, cfg, eval_ds=eval_ds, meta={"vocab_size": vocab, "block_size": a.block_size})
    if D.is_main():
        print(json.dumps({"train_loss": hist["train_loss"], "eval_loss": hist["eval_loss"],
                          "global_step": hist.get("global_step"), "strategy": strategy}))
    if strategy != "single":
        D.destroy()


# ============================================================================ track E
def _load_base(a, preset, device):
    from ..models.qwen3 import BitsAndBytesConfig, Qwen3ForCausalLM, qwen3_config
    qc = BitsAndBytesConfig(load_in_4bit=True, bnb_4bit_quant_type="nf4", bnb_4bit_use_double_quant=True,
                            bnb_4bit_compute_dtype=torch.bfloat16) if preset.quant == "nf4" else None
    if a.random_init or not a.model_path:
        m = Qwen3ForCausalLM.from_config(qwen3_config(a.random_init or preset.model), dtype=torch.bfloat16,
                                         device=device)
        if qc is not None:
            from ..peft.lora import quantize_model_nf4
            quantize_model_nf4(m)
        return m
    return Qwen3ForCausalLM.from_pretrained(a.model_path, dtype=torch.bfloat16, device=device, quantization_config=qc,
                                            rope_scaling=None if preset.rope_scaling == "none" else "keep")


def cmd_finetune(a):
    from ..cli.recipes import PRESETS
    from ..parallel import dist as D
    from ..peft.lora import LoraConfig, get_peft_model, prepare_model_for_kbit_training
    from ..train.data import (ByteTokenizer, DataCollatorForLanguageModeling, SFTDataset, SyntheticLMDataset,
                              load_records, load_tokenizer, synthetic_self_cognition)
    from ..train.trainer import Trainer, TrainingArguments
    p = PRESETS[a.preset]
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        D.init_distributed(timeout_s=1800)
    dev = _device()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    model = _load_base(a, p, dev)
    if p.quant:
        model = prepare_model_for_kbit_training(model, use_gradient_checkpointing=p.grad_ckpt and not a.no_grad_ckpt)
    elif p.grad_ckpt and not a.no_grad_ckpt:
        model.gradient_checkpointing_enable()
    model = get_peft_model(model, LoraConfig(r=p.lora_r, lora_alpha=p.lora_alpha, lora_dropout=p.lora_dropout,
                                             target_modules=list(p.targets), task_type="CAUSAL_LM"))
    if D.is_main():
        model.print_trainable_parameters()
    if not (p.grad_ckpt and not a.no_grad_ckpt):
        model.fuse_projections()
    tok = load_tokenizer(a.tokenizer or a.model_path, pad_to_eos=p.pad_to_eos) if (a.tokenizer or a.model_path) \
        else None
    if tok is not None:
        recs = load_records(a.data) if a.data else synthetic_self_cognition()
        train_ds = SFTDataset(recs, tok, p.max_length, p.padding, label_mode=a.label_mode, system=p.system,
                              space_before_end=p.space_before_end)
        collator = DataCollatorForLanguageModeling(tok, mlm=False) if a.label_mode == "reference" else None
    else:                                        # no tokenizer available offline: synthetic ids at the preset shape
        vocab = model.config.vocab_size
        train_ds = SyntheticLMDataset(vocab, p.max_length, a.synthetic_samples)
        collator = None
    ds = p.deepspeed if not a.no_deepspeed else None
    if ds and not os.path.exists(ds):            # bundled configs/ next to the package
        ds = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), ds)
    args = TrainingArguments(
        output_dir=a.output_dir or p.output_dir, per_device_train_batch_size=p.per_device_batch,
        gradient_accumulation_steps=p.grad_accum, num_train_epochs=a.epochs or p.epochs, max_steps=a.max_steps,
        learning_rate=p.lr, weight_decay=p.weight_decay, logging_steps=p.logging_steps, save_steps=p.save_steps,
        save_total_limit=p.save_total_limit, bf16=True, optim=p.optim, report_to=[], remove_unused_columns=False,
        deepspeed=ds, ddp_timeout=1800,
        gradient_checkpointing=p.grad_ckpt and not a.no_grad_ckpt, metrics_jsonl=a.metrics_jsonl)
    tr = Trainer(model, args, train_dataset=train_ds, data_collator=collator, tokenizer=tok)
    try:
        out = tr.train(resume_from_checkpoint=a.resume)
    except Exception:
        d = tr.save_interrupted()                # reference: qwen3-8b-lora.py:190-204
        print(f"training interrupted; adapter saved to {d}", file=sys.stderr)
        raise
    tr.save_model(args.output_dir)
    tr.log_metrics("train", out.metrics)
    tr.save_metrics("train", out.metrics)
    tr.save_state()


# ============================================================================ inference / quant
def _parallel(a=None):
    """torchrun with WORLD_SIZE > 1 on an inference command: ``world = tp × pp`` ranks
    (vLLM ``--tensor-parallel-size`` / ``--pipeline-parallel-size``; default
    all tensor parallel).  Returns ``(spmd_group, tp_group, pp_group)`` — every rank of the
    world replays the same engine iterations."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None, None, None
    from ..parallel import dist as D
    D.init_distributed()
    import torch.distributed as dist
    from ..parallel.pipeline_parallel import make_tp_pp_groups
    world = dist.get_world_size()
    pp = int(getattr(a, "pp", None) or 1)
    tp = int(getattr(a, "tp", None) or world // pp)
    tp_group, pp_group = make_tp_pp_groups(tp, pp)
    return dist.group.WORLD, tp_group, pp_group


def _load_for_inference(path, adapter=None, device=None, quant=None, fuse=True, tp_group=None, pp_group=None):
    from ..models.qwen3 import BitsAndBytesConfig, Qwen3ForCausalLM, qwen3_config
    dev = device or _device()
    if tp_group is not None or pp_group is not None:   # shard the bf16 weights (+ adapter), THEN quantise
        from ..parallel.pipeline_parallel import apply_pipeline_parallel
        from ..parallel.tensor_parallel import apply_tensor_parallel
        from ..peft.lora import quantize_model_nf4
        m = _load_for_inference(path, adapter, dev, None, fuse=False)
        if pp_group is not None:
            apply_pipeline_parallel(m, pp_group)
        if tp_group is not None:
            apply_tensor_parallel(m, tp_group)
        if quant == "nf4":
            quantize_model_nf4(m)
        lm = m
        while not hasattr(lm, "fuse_projections") and hasattr(lm, "model"):
            lm = lm.model
        if fuse and hasattr(lm, "fuse_projections"):
            lm.fuse_projections()
        return m.eval()
    if path.startswith("random:"):
        m = Qwen3ForCausalLM.from_config(qwen3_config(path[7:]), dtype=torch.bfloat16, device=dev)
    else:
        with open(os.path.join(path, "config.json")) as f:
            qc = json.load(f).get("quantization_config")
        if qc and qc.get("quant_method") in ("compressed-tensors", "gptq", "awq"):
            from ..quant.io import load_quantized
            m = load_quantized(path, dev)
        else:
            bnb = BitsAndBytesConfig(load_in_4bit=True) if quant == "nf4" else None
            m = Qwen3ForCausalLM.from_pretrained(path, dtype=torch.bfloat16, device=dev, quantization_config=bnb)
    if adapter:
        from ..peft.lora import PeftModel
        m = PeftModel.from_pretrained(m, adapter)
    m.requires_grad_(False)
    lm = m
    while not hasattr(lm, "fuse_projections") and hasattr(lm, "model"):
        lm = lm.model
    if fuse and hasattr(lm, "fuse_projections"):
        lm.fuse_projections()          # q|k|v and gate|up as single GEMMs (frozen weights)
    return m.eval()


def _add_parallel_args(p):
    p.add_argument("--tensor-parallel-size", "-tp", dest="tp", type=int, default=None,
                   help="under torchrun: TP degree (default WORLD_SIZE / pp)")
    p.add_argument("--pipeline-parallel-size", "-pp", dest="pp", type=int, default=1,
                   help="under torchrun: pipeline stages (layers split across ranks)")


def cmd_chat(a):
    from ..infer.engine import SamplingParams, ServingEngine
    from ..train.data import load_tokenizer
    m = _load_for_inference(a.base, a.adapter, quant=a.quant)
    tok = load_tokenizer(a.tokenizer or a.base)
    eng = ServingEngine(m, tok, system_prompt=a.system, space_before_end=True)
    history = []                                  # multi-turn (inferences.py:77-83, 04-*-multisession*.py)
    params = SamplingParams(max_tokens=a.max_new, temperature=a.temperature, top_p=a.top_p)
    while True:
        try:
            q = input("user> ").strip()
        except EOFError:
            break
        if q in ("exit", "quit"):
            break
        if q == "clear":
            history = []
            continue
        history.append({"role": "user", "content": q})
        prompt = eng.build_chat_prompt(history)
        print("assistant> ", end="", flush=True)
        text = ""
        for delta, final in eng.stream(prompt, params):
            print(delta, end="", flush=True)
            text += delta
        print()
        history.append({"role": "assistant", "content": text})


def cmd_infer(a):
    from ..infer.generate import generate
    from ..train.data import load_tokenizer, render_chatml
    tp, tpg, ppg = _parallel(a)      # torchrun → TP / PP; every rank decodes in lockstep
    m = _load_for_inference(a.model, a.adapter, quant=a.quant, tp_group=tpg, pp_group=ppg)
    tok = load_tokenizer(a.tokenizer or a.model)
    text = render_chatml([{"role": "user", "content": a.prompt}], add_generation_prompt=True) if a.chat else a.prompt
    ids = torch.tensor([tok.encode(text, add_special_tokens=False)], device=_device())
    out = generate(m, ids, max_new_tokens=a.max_new, do_sample=a.temperature > 0, temperature=a.temperature,
                   top_p=a.top_p, repetition_penalty=a.repetition_penalty, eos_token_id=tok.eos_token_id,
                   seed=1234 if tp is not None else None)
    if tp is None or torch.distributed.get_rank() == 0:
        print(tok.decode(out[0, ids.shape[1]:].tolist(), skip_special_tokens=True))


def cmd_merge(a):
    from ..peft.lora import PeftModel
    from ..models.qwen3 import Qwen3ForCausalLM
    base = Qwen3ForCausalLM.from_pretrained(a.base, dtype=torch.bfloat16, device=_device(a.device))
    merged = PeftModel.from_pretrained(base, a.adapter).merge_and_unload()
    merged.save_pretrained(a.out)
    if a.tokenizer or os.path.exists(os.path.join(a.base, "tokenizer.json")):
        from ..train.data import load_tokenizer
        load_tokenizer(a.tokenizer or a.base).save_pretrained(a.out)
    print(json.dumps({"merged": a.out}))


def _calib_ids(a, tok, vocab, device):
    if a.calib and tok is not None:
        from ..train.data import load_text_corpus
        texts = load_text_corpus(a.calib)[:a.n_calib]
        return [torch.tensor([tok.encode(t)[:a.calib_len]], device=device) for t in texts if t.strip()]
    g = torch.Generator().manual_seed(0)
    return [torch.randint(0, vocab, (1, a.calib_len), generator=g).to(device) for _ in range(a.n_calib)]


def cmd_quantize(a):  # calibration hooks need the unfused Linear modules
    from ..quant.awq import awq_quantize_model
    from ..quant.gptq import gptq_quantize_model, replace_with_int4
    from ..quant.int4 import quantize_rtn
    from ..quant.io import save_quantized
    dev = _device(a.device)
    m = _load_for_inference(a.model, device=dev, fuse=False)
    tok = None
    if not a.model.startswith("random:"):
        try:
            from ..train.data import load_tokenizer
            tok = load_tokenizer(a.tokenizer or a.model)
        except Exception:
            tok = None
    calib = _calib_ids(a, tok, m.config.vocab_size, dev)
    if a.method == "gptq":
        gptq_quantize_model(m, calib, a.group_size, a.sym)
    elif a.method == "awq":
        awq_quantize_model(m, calib, a.group_size)
    else:
        ws = {}
        for n, mod in m.named_modules():
            if isinstance(mod, torch.nn.Linear) and n.startswith("model.layers"):
                ws[n] = quantize_rtn(mod.weight.detach(), a.group_size, a.sym)
        replace_with_int4(m, ws)
    save_quantized(m, a.out, a.format, tok)
    print(json.dumps({"quantized": a.out, "method": a.method, "format": a.format}))


def cmd_eval_quant(a):
    from ..quant.eval import PASS_THRESHOLD, self_ppl
    from ..train.data import load_text_corpus, load_tokenizer
    dev = _device()
    m = _load_for_inference(a.model, device=dev, fuse=False)
    tok = load_tokenizer(a.tokenizer or a.model) if not a.model.startswith("random:") else None
    if a.prompts and tok is not None:
        prompts = [torch.tensor(tok.encode(t)[:256], device=dev) for t in load_text_corpus(a.prompts)[a.start:a.end]]
    else:
        prompts = [torch.randint(0, m.config.vocab_size, (32,), device=dev) for _ in range(a.end - a.start)]
    ppl = self_ppl(m, prompts, a.max_new, getattr(tok, "eos_token_id", None))
    print(json.dumps({"self_ppl": ppl, "pass": ppl < PASS_THRESHOLD, "threshold": PASS_THRESHOLD}))


_VLLM_QUANT = {"awq": ("awq", "compressed-tensors"), "awq_marlin": ("awq", "compressed-tensors"),
               "gptq": ("gptq", "compressed-tensors"), "gptq_marlin": ("gptq", "compressed-tensors"),
               "compressed-tensors": ("compressed-tensors", "awq", "gptq")}


def _vllm_compat(a):
    """Map vLLM's ``vllm serve`` flags onto ``lipa serve`` so the reference's manifests apply unchanged
    (``LLM_on_Kubernetes/Inference_Platfrom/01-Base/vLLM/vllm-deployment.yaml:97-114``, the litellm-proxy compose
    files, ``07-L1-Cache/LMCache/vllm-statefulset-lmcache.yaml``):

    * positional ``MODEL`` (the vllm-openai image's first arg) = ``--model``;
    * ``--max-num-seqs`` = ``--max-batch``; ``--gpu-memory-utilization`` sizes the KV pool (``kv_slots_for_budget``);
    * ``--dtype auto|bfloat16`` run bf16 (the kernels' compute dtype); ``half``/``float16`` are served in bf16
      with a notice (no fp16 kernel path on this stack);
    * ``--quantization awq|gptq|compressed-tensors`` check the checkpoint's ``quantization_config`` (the int4
      W4A16 path loads it either way); ``bitsandbytes`` = in-flight NF4 (``--quant nf4``);
    * ``--kv-transfer-config`` with an LMCache connector = the prefix cache with the host tier
      (``LMCACHE_MAX_LOCAL_CPU_SIZE`` GB) and, from ``LMCACHE_REMOTE_URL`` (lm://host:port), the shared
      ``lipa kv-server`` at http://host:port; ``LMCACHE_CHUNK_SIZE`` = the prefix block;
    * ``--enforce-eager`` = no decode hipGraphs; ``--trust-remote-code``, ``--disable-log-requests``,
      ``--disable-usage-stats`` are accepted (nothing to switch).
    Returns ``a`` (mutated)."""
    import sys
    if getattr(a, "model_tag", None):
        if a.model and a.model != a.model_tag:
            raise SystemExit(f"model given twice: positional {a.model_tag!r} and --model {a.model!r}")
        a.model = a.model_tag
    if not getattr(a, "model", None):
        raise SystemExit("lipa serve: a model is required (--model DIR or positional DIR)")
    dt = getattr(a, "dtype", "auto")
    if dt in ("half", "float16"):
        print(f"[lipa serve] --dtype {dt}: this stack computes in bfloat16 (MFMA bf16 kernels); serving bf16",
              file=sys.stderr)
    elif dt == "float32":
        raise SystemExit("--dtype float32: not supported (bf16 kernels)")
    vq = getattr(a, "vllm_quant", None)
    if vq == "bitsandbytes":
        a.quant = "nf4"
    elif vq is not None:
        cfgp = os.path.join(a.model, "config.json")
        qc = None
        if os.path.exists(cfgp):
            with open(cfgp) as f:
                qc = (json.load(f).get("quantization_config") or {}).get("quant_method")
        if qc is None:
            raise SystemExit(f"--quantization {vq}: {cfgp} declares no quantization_config")
        if qc not in _VLLM_QUANT[vq]:
            raise SystemExit(f"--quantization {vq}: the checkpoint is quantized with {qc!r}")
    kvt = getattr(a, "kv_transfer_config", None)
    if kvt:
        spec = json.loads(kvt)
        if str(spec.get("kv_connector", "")).startswith("LMCache"):
            a.prefix_caching = True
            if os.environ.get("LMCACHE_LOCAL_CPU", "True").lower() in ("1", "true") and not a.host_blocks:
                gb = float(os.environ.get("LMCACHE_MAX_LOCAL_CPU_SIZE", "5"))
                a.prefix_block = int(os.environ.get("LMCACHE_CHUNK_SIZE", a.prefix_block))
                a.host_blocks = -int(gb * 2 ** 30)     # bytes: converted to blocks once the model is known
            url = os.environ.get("LMCACHE_REMOTE_URL")
            if url and not a.kv_remote_url:
                a.kv_remote_url = "http://" + url.split("://", 1)[-1] if url.startswith("lm://") else url
        else:
            raise SystemExit(f"--kv-transfer-config: connector {spec.get('kv_connector')!r} not supported")
    return a


def _serving_engine_from_args(a, tp=None, tpg=None, ppg=None):
    """Build the ServingEngine ``lipa serve`` describes (runs in the engine process by default)."""
    from ..infer.engine import ServingEngine
    from ..train.data import load_tokenizer
    g = lambda k, d=None: getattr(a, k, d)      # noqa: E731  (namespaces built by other commands)
    m = _load_for_inference(a.model, g("adapter"), quant=g("quant"), tp_group=tpg, pp_group=ppg)
    tok = load_tokenizer(g("tokenizer") or a.model)
    if g("chat_template"):                        # vLLM --chat-template: a jinja file (or the template itself)
        path = g("chat_template")
        text = open(path).read() if os.path.exists(path) else path
        if hasattr(tok, "chat_template"):
            tok.chat_template = text
    loras = dict(spec.split("=", 1) for spec in g("lora_modules")) if g("lora_modules") else None
    host_blocks = g("host_blocks", 0)
    block = g("prefix_block", 64)
    if host_blocks < 0:                           # a byte budget (LMCache LMCACHE_MAX_LOCAL_CPU_SIZE): in blocks
        cfg = m.config
        per = 2 * cfg.num_hidden_layers * block * cfg.num_key_value_heads * cfg.head_dim * 2
        host_blocks = max(1, -host_blocks // per)
    return ServingEngine(m, tok, model_name=g("served_model_name") or os.path.basename(a.model.rstrip("/")),
                         max_batch=g("max_batch", 32), system_prompt=g("system"), tp_group=tp,
                         max_model_len=g("max_model_len"),
                         prefix_cache_blocks=g("prefix_blocks", 1024) if g("prefix_caching") else 0,
                         prefix_block=block,
                         chunked_prefill=g("max_batched_tokens", 2048) if g("chunked_prefill") else 0,
                         lora_modules=loras, host_cache_blocks=host_blocks,
                         kv_remote_url=g("kv_remote_url"), gpu_memory_utilization=g("gpu_memory_utilization"),
                         use_graphs=False if g("enforce_eager") else None)


def cmd_serve(a):
    """OpenAI server.  Single-GPU serving runs the engine core in its own process (the HTTP
    process only formats and streams — ``infer/mp_engine.py``); TP/PP groups and
    ``--no-engine-process`` keep the engine in-process."""
    from ..infer.server import serve
    _vllm_compat(a)
    if getattr(a, "lora_modules", None) and not a.enable_lora:
        raise SystemExit("--lora-modules needs --enable-lora (vLLM semantics)")
    moderation = None
    if a.guard_url:
        from ..infer.guard import GuardClient
        moderation = GuardClient(a.guard_url).moderate_sync
    tp, tpg, ppg = _parallel(a)
    if tp is None and getattr(a, "engine_process", True):
        from ..infer.mp_engine import EngineClient, PromptFormatter
        from ..train.data import load_tokenizer
        fmt = PromptFormatter(load_tokenizer(a.tokenizer or a.model), a.system)
        args = argparse.Namespace(**{k: v for k, v in vars(a).items() if k != "fn"})   # picklable
        eng = EngineClient(_serving_engine_from_args, (args,), fmt)
    else:
        eng = _serving_engine_from_args(a, tp, tpg, ppg)
        if tp is not None and eng.tp_rank != 0:
            eng.follower_loop()              # TP / PP followers replay rank 0's iterations
            return
    serve(eng, a.host, a.port, api_key=a.api_key, moderation=moderation,
          log_level=getattr(a, "uvicorn_log_level", "info"))


def cmd_serve_deploy(a):
    """``serve deploy <config.yaml>`` with Ray Serve LLM-app semantics: replicas of
    ``lipa serve`` on the given GPUs behind an autoscaling proxy (``infer/serve_app.py``)."""
    import uvicorn
    from ..infer.serve_app import ServeController, create_serve_proxy, load_serve_config, process_replica_factory
    gpus = [int(g) for g in a.gpus.split(",")] if a.gpus else None
    ctl = ServeController(load_serve_config(a.config), process_replica_factory(), gpus=gpus,
                          control_interval=a.control_interval)
    ctl.start()
    try:
        uvicorn.run(create_serve_proxy(ctl), host=a.host, port=a.port)
    finally:
        ctl.shutdown()


def cmd_kv_server(a):
    """LMCache-server role: the remote prefix-KV chunk store shared by serving replicas."""
    import uvicorn
    from ..infer.kv_server import create_kv_server
    uvicorn.run(create_kv_server(int(a.max_gib * (1 << 30))), host=a.host, port=a.port)


def cmd_guard(a):
    import uvicorn
    from ..infer.guard import GuardClient, create_guard_app
    uvicorn.run(create_guard_app(GuardClient(a.backend, a.model), a.api_key), host=a.host, port=a.port)


def cmd_cache_gateway(a):
    import uvicorn
    from ..infer.cache_gateway import create_cache_gateway, http_backend, make_store
    app = create_cache_gateway(http_backend(a.backend, a.api_key), make_store(a.redis), a.exact_ttl, a.semantic_ttl)
    uvicorn.run(app, host=a.host, port=a.port)


def cmd_router(a):
    """H2 LiteLLM proxy equivalent: model groups, routing strategy, retries, cooldown, fallbacks, guard."""
    import uvicorn
    from ..infer.router import Router, create_router_app
    uvicorn.run(create_router_app(Router(a.config)), host=a.host, port=a.port)


def cmd_lf(a):
    """``llamafactory-cli train|export|webchat <yaml>``."""
    from .llamafactory import lf_export, lf_train, load_lf_yaml
    cfg = load_lf_yaml(a.config)
    cfg.update({k: v for k, v in (kv.split("=", 1) for kv in a.overrides)})   # key=value CLI overrides
    for k in ("learning_rate", "num_train_epochs", "warmup_ratio", "lora_dropout"):
        if isinstance(cfg.get(k), str):
            cfg[k] = float(cfg[k])
    for k in ("max_steps", "save_steps", "logging_steps", "lora_rank", "cutoff_len", "max_samples"):
        if isinstance(cfg.get(k), str):
            cfg[k] = int(cfg[k])
    if a.action == "train":
        lf_train(cfg, a.tokenizer)
    elif a.action == "export":
        print(json.dumps({"exported": lf_export(cfg, a.tokenizer)}))
    else:  # webchat / api: the OpenAI server + browser UI at /ui
        ns = argparse.Namespace(model=str(cfg["model_name_or_path"]), adapter=cfg.get("adapter_name_or_path"),
                                tokenizer=a.tokenizer, quant="nf4" if int(cfg.get("quantization_bit") or 0) == 4
                                else None, host="0.0.0.0", port=int(cfg.get("port", 7860)), max_batch=16,
                                served_model_name=None, api_key=None, guard_url=None, system=None,
                                prefix_caching=True, prefix_blocks=512, max_model_len=None,
                                engine_process=False)
        cmd_serve(ns)


def cmd_cluster_check(a):
    """torchrun-launched collective health probe (H4 ray_cluster_healthcheck.py role)."""
    from ..parallel import dist as D
    from ..parallel.healthcheck import cluster_check
    D.init_distributed(timeout_s=a.timeout)
    if not D.is_dist():
        print(json.dumps({"error": "run under torchrun with WORLD_SIZE >= 2"}))
        return
    rep = cluster_check(a.allreduce_mib, a.iters)
    if rep is not None:
        print(json.dumps(rep, indent=1))
    D.destroy()


def cmd_convert_alpaca(a):
    from ..train.data import load_records, replace_placeholders
    recs = [replace_placeholders(r, a.name, a.author) for r in load_records(a.input)]
    out = [{"instruction": r["query"], "input": "", "output": r["response"]} for r in recs]
    with open(a.out, "w") as f:
        json.dump(out, f, ensure_ascii=False, indent=2)
    print(json.dumps({"records": len(out), "out": a.out}))


def _nb_tokenizer(spec: str, texts: list[str]):
    from ..train.data import ByteTokenizer, CharTokenizer, load_tokenizer
    if spec == "char":
        return CharTokenizer("".join(texts))
    if spec == "bytes":
        return ByteTokenizer()
    return load_tokenizer(spec[3:] if spec.startswith("hf:") else spec, pad_to_eos=False)


def cmd_minibert_imdb(a):
    """Transformer_Basics cell 34: MiniBert sentiment classifier (IMDb in the notebook; any local
    JSONL/JSON of {text, label} here, or a synthetic sentiment set without --data)."""
    import random
    from ..train.data import load_records
    from ..train.teaching import MiniBertConfig, train_minibert_classifier
    if a.data:
        recs = load_records(a.data)
        recs = [{"text": r[a.text_field], "label": int(r[a.label_field])} for r in recs]
    else:
        rng = random.Random(0)
        recs = [{"text": " ".join(rng.choice(["the", "movie", "plot", "was", "acting"]) for _ in range(8)) +
                 (" great fun" if i % 2 else " awful boring"), "label": i % 2} for i in range(600)]
    test = load_records(a.test) if a.test else None
    if test is None:
        n = max(1, len(recs) // 10)
        recs, test = recs[n:], recs[:n]
    else:
        test = [{"text": r[a.text_field], "label": int(r[a.label_field])} for r in test]
    tok = _nb_tokenizer(a.tokenizer, [r["text"] for r in recs + test])
    cfg = MiniBertConfig(hidden_size=a.hidden_size, num_layers=a.num_layers, max_len=a.max_len, epochs=a.epochs,
                         batch_size=a.batch_size, lr=a.lr)
    h = train_minibert_classifier(recs, test, tok, cfg, pad_id=getattr(tok, "pad_token_id", None) or 0)
    if a.save:
        torch.save({"model_state": h["model"].state_dict(), "config": dataclasses.asdict(cfg)}, a.save)
    print(json.dumps({k: v for k, v in h.items() if k != "model"}))


def cmd_nb_gpt(a):
    """Transformer_Basics cells 39 / 41: notebook GPT on WikiText-2 (GPT-2 vocab) or the Chinese
    CLUECorpusSmall (bert-base-chinese vocab) — any local corpus (file or directory of .txt)."""
    from ..models.teaching import NotebookGPTConfig
    from ..train.data import load_text_corpus
    from ..train.teaching import train_notebook_gpt
    if os.path.isdir(a.data):                    # CLUECorpusSmall layout: a directory of text files
        texts = []
        for fn in sorted(os.listdir(a.data)):
            if fn.endswith((".txt", ".jsonl", ".json")):
                texts += load_text_corpus(os.path.join(a.data, fn))
    else:
        texts = load_text_corpus(a.data)
    tok = _nb_tokenizer(a.tokenizer, texts)
    cfg = NotebookGPTConfig(vocab_size=int(getattr(tok, "vocab_size", 256) or len(tok)), n_embd=a.n_embd,
                            n_head=a.n_head, n_layer=a.n_layer, max_seq_len=a.max_seq_len)
    out = train_notebook_gpt(texts, tok, cfg, epochs=a.epochs, batch_size=a.batch_size, lr=a.lr,
                             max_steps=a.max_steps, prompt=a.prompt, gen_tokens=a.gen_tokens)
    if a.save:
        torch.save({"model_state": out["model"].state_dict(), "config": dataclasses.asdict(cfg)}, a.save)
    print(json.dumps({"final_loss": out["losses"][-1], "steps": out["steps"], "sample": out.get("sample")},
                     ensure_ascii=False))


def cmd_seq2seq_demo(a):
    """Transformer_Basics cells 20-22: the encoder-decoder Transformer learns sequence reversal."""
    from ..train.teaching import train_seq2seq
    _, losses, acc = train_seq2seq(steps=a.steps, vocab=a.vocab, length=a.length, num_layers=a.num_layers)
    print(json.dumps({"first_loss": losses[0], "final_loss": losses[-1], "exact_match": acc}))


def cmd_hf_classify(a):
    """G5 ``HF_Basics/trainer_demo.py``: BERT sequence classification with the Trainer (eval and
    save per epoch, best model by accuracy)."""
    from ..models.bert import BertConfig, BertForSequenceClassification, accuracy_metric
    from ..train.data import DataCollatorWithPadding, load_records, load_tokenizer
    from ..train.trainer import Trainer, TrainingArguments
    dev = _device()
    if a.model_path:
        m = BertForSequenceClassification.from_pretrained(a.model_path, a.num_labels, dev)
        tok = load_tokenizer(a.model_path, pad_to_eos=False)
        enc = lambda t: tok(t, truncation=True, max_length=a.max_length)["input_ids"]  # noqa: E731
    else:                                  # offline smoke: byte tokens on a tiny encoder
        m = BertForSequenceClassification(BertConfig(vocab_size=260, hidden_size=128, num_hidden_layers=2,
                                                     num_attention_heads=4, intermediate_size=256,
                                                     num_labels=a.num_labels)).to(dev)
        enc = lambda t: [257] + list(t.encode("utf-8"))[:a.max_length - 1]  # noqa: E731
    recs = load_records(a.data) if a.data else \
        [{"text": ("great film " if i % 2 else "awful film ") * (1 + i % 3), "label": i % 2} for i in range(200)]
    rows = [{"input_ids": enc(r[a.text_field]), "label": int(r[a.label_field])} for r in recs]
    n_eval = max(1, int(len(rows) * a.eval_fraction))
    args = TrainingArguments(output_dir=a.output_dir, per_device_train_batch_size=a.batch_size,
                             per_device_eval_batch_size=a.batch_size, num_train_epochs=a.epochs,
                             learning_rate=a.lr, weight_decay=0.01, eval_strategy="epoch", save_strategy="epoch",
                             load_best_model_at_end=True, metric_for_best_model="accuracy", save_total_limit=2,
                             logging_steps=50)
    tr = Trainer(m, args, train_dataset=rows[n_eval:], eval_dataset=rows[:n_eval],
                 data_collator=DataCollatorWithPadding(pad_token_id=0), compute_metrics=accuracy_metric)
    tr.train()
    res = tr.evaluate()
    tr.log_metrics("eval", res)
    tr.save_metrics("eval", res)


def cmd_dl_basics(a):
    """B9 ``DL_Basics/*.ipynb`` demos as runnable commands; prints one JSON line per result."""
    import numpy as np

    from ..dl_basics import numpy_cnn, numpy_nn, numpy_rnn, seq2seq
    rng = np.random.default_rng(a.seed)
    if a.demo == "mlp":                    # two-hidden-layer net on a noisy sine, mini-batches + L2
        x = rng.uniform(-3, 3, (512, 1))
        y = np.sin(x) + rng.normal(0, 0.05, x.shape)
        m = numpy_nn.MLP([1, 32, 32, 1], act="tanh", l2=1e-4, seed=a.seed)
        h = numpy_nn.train_mlp(m, x, y, optimizer="adam", lr=1e-2, epochs=a.epochs, batch_size=64, seed=a.seed)
        print(json.dumps({"demo": "mlp", "first_loss": h["train"][0], "final_loss": h["train"][-1]}))
    elif a.demo == "optimizers":           # the notebook's optimiser comparison on the same problem
        x = rng.normal(size=(256, 4))
        y = x @ rng.normal(size=(4, 1)) + 0.1 * rng.normal(size=(256, 1))
        for name in numpy_nn.OPTIMIZERS:
            m = numpy_nn.MLP([4, 16, 1], seed=a.seed)
            h = numpy_nn.train_mlp(m, x, y, optimizer=name, lr=1e-2, epochs=a.epochs, batch_size=32, seed=a.seed)
            print(json.dumps({"demo": "optimizers", "optimizer": name, "final_loss": h["train"][-1]}))
    elif a.demo == "rnn":
        for kind in ("rnn", "lstm", "gru"):
            ls = numpy_rnn.train_sequence_regressor(kind, steps=10 * a.epochs, seed=a.seed)
            print(json.dumps({"demo": "bptt", "cell": kind, "first_loss": ls[0], "final_loss": float(np.mean(ls[-20:]))}))
    elif a.demo == "cnn":                  # LeNet-5 on synthetic 28x28 "digits" (class = bright quadrant)
        net = numpy_cnn.LeNet5(num_classes=4)
        opt = torch.optim.Adam(net.parameters(), lr=1e-3)
        for step in range(a.epochs):
            lab = torch.randint(0, 4, (64,))
            img = torch.randn(64, 1, 28, 28) * 0.3
            for i, c in enumerate(lab.tolist()):
                img[i, 0, (c // 2) * 14:(c // 2) * 14 + 14, (c % 2) * 14:(c % 2) * 14 + 14] += 1.0
            loss = torch.nn.functional.cross_entropy(net(img), lab)
            opt.zero_grad()
            loss.backward()
            opt.step()
        print(json.dumps({"demo": "lenet5", "final_loss": loss.item()}))
    else:                                  # seq2seq: string reversal with Bahdanau attention
        words = ["".join(rng.choice(list("abcdefgh"), rng.integers(3, 8))) for _ in range(600)]
        model, sv, tv, ls = seq2seq.train_seq2seq([(w, w[::-1]) for w in words], epochs=a.epochs, seed=a.seed)
        test = words[:5]
        print(json.dumps({"demo": "seq2seq", "final_loss": ls[-1],
                          "samples": dict(zip(test, seq2seq.translate(model, sv, tv, test)))}, ensure_ascii=False))


def cmd_env(a):
    """G5 ``env_test.py``: device / runtime versions."""
    info = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
            "gpu_available": torch.cuda.is_available(), "device_count": torch.cuda.device_count()}
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        info.update(name=p.name, arch=getattr(p, "gcnArchName", ""), hbm_gib=round(p.total_memory / 2 ** 30, 1),
                    cus=p.multi_processor_count)
    print(json.dumps(info, indent=2))


def cmd_bench(a):
    import subprocess
    here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.exit(subprocess.call([sys.executable, os.path.join(here, "bench.py")] + a.rest))


# ============================================================================ parser
def _lm_args(p):
    p.add_argument("--model", default="gptlike", choices=["simple", "gptlike", "deepseek", "deepseek-dense"])
    p.add_argument("--pe", default="fixed", choices=["fixed", "learned"])
    p.add_argument("--data", help="local text corpus (.txt/.jsonl/.parquet); default: built-in demo text")
    p.add_argument("--tokenizer", default="bpe-whitespace",
                   help="bpe-whitespace | bpe-bytelevel | byte | hf:<local dir> (e.g. a bert-base-uncased dir)")
    p.add_argument("--vocab_size", type=int, default=3000)
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--batch_size", type=int, default=16)
    p.add_argument("--block_size", type=int, default=256)
    p.add_argument("--lr", type=float, default=3e-4)
    p.add_argument("--weight_decay", type=float, default=0.01)
    p.add_argument("--no_decay_groups", action="store_true",
                   help="AdamW decay / no-decay param groups (biases, LayerNorm) as temp/ddp_gpt_wikitext2.py:337-344")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--n_layer", type=int, default=6)
    p.add_argument("--n_head", type=int, default=8)
    p.add_argument("--d_model", type=int, default=768)
    p.add_argument("--dropout", type=float, default=0.1)
    p.add_argument("--clip_grad_norm", type=float, default=1.0)
    p.add_argument("--save_dir", default=None)
    p.add_argument("--keep_last", type=int, default=5)
    p.add_argument("--final_model", default=None)
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "fp16"])
    p.add_argument("--scheduler", default="none", choices=["none", "step", "cosine"])
    p.add_argument("--step_per_batch", action="store_true", help="reproduce the per-batch StepLR of B2/B4/B6")
    p.add_argument("--max_steps", type=int, default=-1)
    p.add_argument("--grad_accum", type=int, default=1)
    p.add_argument("--val_fraction", type=float, default=0.0, help="seeded random_split validation set (C6)")
    p.add_argument("--patience", type=int, default=0, help="early stopping on validation loss (C6)")
    p.add_argument("--best_model", default=None, help="path for the best-validation checkpoint (C6)")
    p.add_argument("--resume", action="store_true", help="continue from <save_dir>/latest_checkpoint.pt (C6)")
    p.add_argument("--latent_dim", type=int, default=None)
    p.add_argument("--num_experts", type=int, default=8)
    p.add_argument("--top_k", type=int, default=2)
    p.add_argument("--num_shared", type=int, default=2)
    p.add_argument("--rope_theta", type=float, default=10000.0)
    p.add_argument("--ds_config", default=None)
    p.add_argument("--timeout", type=int, default=1800)
    p.add_argument("--local_rank", type=int, default=None)


class _Parser(argparse.ArgumentParser):
    """vLLM's parser accepts ``--flag_name`` for ``--flag-name``; ``lipa serve`` does too (the reference's
    compose files pass ``--trust_remote_code``).  Other subcommands keep their own underscore flags."""

    def parse_known_args(self, args=None, namespace=None):
        args = list(sys.argv[1:] if args is None else args)
        if args and args[0] == "serve":
            args = [("--" + a[2:].split("=", 1)[0].replace("_", "-") + ("=" + a.split("=", 1)[1] if "=" in a else ""))
                    if a.startswith("--") else a for a in args]
        return super().parse_known_args(args, namespace)


def build_parser() -> argparse.ArgumentParser:
    ap = _Parser(prog="lipa", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    p = sub.add_parser("minigpt-train")
    p.add_argument("--text")
    p.add_argument("--epochs", type=int, default=200)
    p.add_argument("--batch_size", type=int, default=4)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--seq_len", type=int, default=16)
    p.add_argument("--repeat", type=int, default=10)
    p.add_argument("--embed_dim", type=int, default=64)
    p.add_argument("--n_heads", type=int, default=2)
    p.add_argument("--n_layers", type=int, default=2)
    p.add_argument("--causal", action="store_true", help="fix the reference's missing causal mask")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--load-format", dest="load_format", default="auto", choices=["auto", "safetensors", "pt"],
                   help="vLLM flag: checkpoint files are read by their extension (safetensors first)")
    p.add_argument("--device", default="cpu")
    p.add_argument("--out", default="mg_edu_gpt.pth")
    p.set_defaults(fn=cmd_minigpt_train)
    p = sub.add_parser("minigpt-generate")
    p.add_argument("--checkpoint", default="mg_edu_gpt.pth")
    p.add_argument("--prompt", default="马哥")
    p.add_argument("--max_new", type=int, default=50)
    p.add_argument("--temperature", type=float, default=0.0)
    p.set_defaults(fn=cmd_minigpt_generate)
    p = sub.add_parser("minigpt2-train")
    p.add_argument("--text")
    p.add_argument("--epochs", type=int, default=200)
    p.add_argument("--seq_len", type=int, default=256)
    p.add_argument("--device", default="cpu")
    p.add_argument("--out", default="minigpt_model.pth")
    p.set_defaults(fn=cmd_minigpt2_train)
    p = sub.add_parser("minigpt2-test")
    p.add_argument("--checkpoint", default="minigpt_model.pth")
    p.add_argument("--prompt", default="马哥")
    p.add_argument("--max_new", type=int, default=50)
    p.set_defaults(fn=cmd_minigpt2_test)

    p = sub.add_parser("lm-train")
    _lm_args(p)
    p.set_defaults(fn=lambda a: cmd_lm_train(a, "single"))
    p = sub.add_parser("pretrain")
    _lm_args(p)
    p.add_argument("--strategy", default="ddp",
                   choices=["ddp", "fsdp", "fsdp2", "zero1", "zero2", "zero3", "zero-offload"])
    p.set_defaults(fn=lambda a: cmd_lm_train(a, a.strategy))

    from .recipes import PRESETS
    p = sub.add_parser("finetune")
    p.add_argument("--preset", required=True, choices=sorted(PRESETS))
    p.add_argument("--model-path", dest="model_path")
    p.add_argument("--tokenizer")
    p.add_argument("--data", help="self-cognition JSONL (query/response with {{NAME}}/{{AUTHOR}})")
    p.add_argument("--random-init", dest="random_init", help="Qwen3 preset name: random weights, no checkpoint")
    p.add_argument("--output-dir", dest="output_dir")
    p.add_argument("--epochs", type=float, default=None)
    p.add_argument("--max-steps", dest="max_steps", type=int, default=-1)
    p.add_argument("--label-mode", dest="label_mode", default="reference", choices=["reference", "assistant", "none"])
    p.add_argument("--no-grad-ckpt", dest="no_grad_ckpt", action="store_true")
    p.add_argument("--no-deepspeed", dest="no_deepspeed", action="store_true")
    p.add_argument("--resume", default=None)
    p.add_argument("--metrics-jsonl", dest="metrics_jsonl")
    p.add_argument("--synthetic-samples", dest="synthetic_samples", type=int, default=108)
    p.set_defaults(fn=cmd_finetune)

    for name, fn in (("chat", cmd_chat), ("infer", cmd_infer)):
        p = sub.add_parser(name)
        p.add_argument("--base" if name == "chat" else "--model", required=True)
        p.add_argument("--adapter")
        p.add_argument("--tokenizer")
        p.add_argument("--quant", choices=["nf4"])
        p.add_argument("--max_new", type=int, default=256)
        p.add_argument("--temperature", type=float, default=0.7)
        p.add_argument("--top_p", type=float, default=0.9)
        if name == "chat":
            p.add_argument("--system", default=None)
        else:
            p.add_argument("--prompt", required=True)
            p.add_argument("--chat", action="store_true")
            p.add_argument("--repetition_penalty", type=float, default=1.0)
            _add_parallel_args(p)
        p.set_defaults(fn=fn)

    p = sub.add_parser("merge")
    p.add_argument("--base", required=True)
    p.add_argument("--adapter", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--tokenizer")
    p.add_argument("--device", default=None)
    p.set_defaults(fn=cmd_merge)

    p = sub.add_parser("quantize")
    p.add_argument("--method", default="awq", choices=["awq", "gptq", "rtn"])
    p.add_argument("--model", required=True, help="HF dir or random:<qwen3 preset>")
    p.add_argument("--out", required=True)
    p.add_argument("--format", default="compressed-tensors", choices=["compressed-tensors", "gptq", "awq"])
    p.add_argument("--group_size", type=int, default=128)
    p.add_argument("--sym", action="store_true")
    p.add_argument("--calib", help="local calibration corpus (Alpaca-style texts)")
    p.add_argument("--n_calib", type=int, default=128)
    p.add_argument("--calib_len", type=int, default=2048)
    p.add_argument("--tokenizer")
    p.add_argument("--device", default=None)
    p.set_defaults(fn=cmd_quantize)

    p = sub.add_parser("eval-quant")
    p.add_argument("--model", required=True)
    p.add_argument("--tokenizer")
    p.add_argument("--prompts")
    p.add_argument("--start", type=int, default=128)
    p.add_argument("--end", type=int, default=256)
    p.add_argument("--max_new", type=int, default=256)
    p.set_defaults(fn=cmd_eval_quant)

    p = sub.add_parser("serve", help="OpenAI-compatible server; also takes vLLM's `vllm serve` flags (_vllm_compat)")
    p.add_argument("model_tag", nargs="?", default=None, metavar="MODEL", help="model dir (vLLM positional form)")
    p.add_argument("--model", default=None)
    p.add_argument("--adapter")
    p.add_argument("--tokenizer")
    p.add_argument("--quant", choices=["nf4"])
    p.add_argument("--quantization", dest="vllm_quant", default=None,
                   choices=["awq", "awq_marlin", "gptq", "gptq_marlin", "compressed-tensors", "bitsandbytes"],
                   help="vLLM flag: int4 checkpoints load by their quantization_config; bitsandbytes = NF4")
    p.add_argument("--dtype", default="auto", choices=["auto", "bfloat16", "bf16", "half", "float16", "float32"])
    p.add_argument("--gpu-memory-utilization", dest="gpu_memory_utilization", type=float, default=None,
                   help="vLLM flag: fraction of device memory for weights + KV; sizes the KV slot pool")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--max-batch", "--max-num-seqs", dest="max_batch", type=int, default=32,
                   help="concurrent sequences (vLLM --max-num-seqs)")
    p.add_argument("--uvicorn-log-level", dest="uvicorn_log_level", default="info",
                   choices=["critical", "error", "warning", "info", "debug", "trace"])
    p.add_argument("--chat-template", dest="chat_template", default=None, help="jinja chat template file")
    p.add_argument("--kv-transfer-config", dest="kv_transfer_config", default=None,
                   help="vLLM KV connector JSON; LMCache connectors map onto the prefix cache tiers")
    p.add_argument("--prefix-block", dest="prefix_block", type=int, default=64, help="prefix-cache chunk tokens")
    p.add_argument("--enforce-eager", dest="enforce_eager", action="store_true", help="no decode hipGraphs")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--load-format", dest="load_format", default="auto", choices=["auto", "safetensors", "pt"],
                   help="vLLM flag: checkpoint files are read by their extension (safetensors first)")
    for flag in ("--trust-remote-code", "--disable-log-requests", "--disable-usage-stats"):
        p.add_argument(flag, action="store_true", help="accepted for vLLM compatibility (no effect)")
    p.add_argument("--served-model-name", dest="served_model_name")
    p.add_argument("--api-key", dest="api_key")
    p.add_argument("--guard-url", dest="guard_url")
    p.add_argument("--system", default=None)
    p.add_argument("--enable-prefix-caching", dest="prefix_caching", action="store_true",
                   help="reuse the KV of cached prompt chunks (vLLM --enable-prefix-caching)")
    p.add_argument("--prefix-cache-blocks", dest="prefix_blocks", type=int, default=1024,
                   help="HBM pool size in 64-token chunks")
    p.add_argument("--max-model-len", dest="max_model_len", type=int, default=None)
    p.add_argument("--enable-chunked-prefill", dest="chunked_prefill", action="store_true",
                   help="prefill long prompts in chunks interleaved with decode (vLLM flag)")
    p.add_argument("--max-num-batched-tokens", dest="max_batched_tokens", type=int, default=2048,
                   help="chunk size for --enable-chunked-prefill")
    p.add_argument("--enable-lora", dest="enable_lora", action="store_true",
                   help="serve LoRA adapters next to the base (vLLM flag; Fine-Tuning/README.md:346-351)")
    p.add_argument("--lora-modules", dest="lora_modules", nargs="+", default=None, metavar="NAME=DIR",
                   help="adapters selectable per request by `model` name")
    p.add_argument("--kv-host-cache-blocks", dest="host_blocks", type=int, default=0,
                   help="prefix-cache host tier (LMCache local-CPU role): 64-token chunks spilled to pinned RAM")
    p.add_argument("--kv-remote-url", dest="kv_remote_url", default=None,
                   help="shared remote KV-chunk store (LMCache server role; `lipa kv-server`)")
    p.add_argument("--no-engine-process", dest="engine_process", action="store_false",
                   help="run the engine core in the HTTP process (default: its own process)")
    _add_parallel_args(p)
    p.set_defaults(fn=cmd_serve)

    p = sub.add_parser("serve-deploy", help="Ray Serve-style autoscaling replicas from a serve config (H4)")
    p.add_argument("config")
    p.add_argument("--gpus", default=None, help="GPU pool, e.g. 0,1,2,3 (default: no GPU pinning)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--control-interval", dest="control_interval", type=float, default=1.0)
    p.set_defaults(fn=cmd_serve_deploy)

    p = sub.add_parser("kv-server", help="remote KV-chunk store shared by replicas (LMCache server role)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8100)
    p.add_argument("--max-gib", dest="max_gib", type=float, default=64.0)
    p.set_defaults(fn=cmd_kv_server)

    p = sub.add_parser("guard")
    p.add_argument("--backend", required=True, help="guard model completions URL")
    p.add_argument("--model", default="llama-guard-3")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8099)
    p.add_argument("--api-key", dest="api_key", default=None)
    p.set_defaults(fn=cmd_guard)

    p = sub.add_parser("router", help="LiteLLM-config model router: strategies, retries, cooldown, fallbacks (H2)")
    p.add_argument("--config", required=True, help="LiteLLM proxy YAML (model_list / router_settings / guardrails)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=4000)
    p.set_defaults(fn=cmd_router)
    p = sub.add_parser("cache-gateway", help="exact + semantic response cache in front of a server (H6)")
    p.add_argument("--backend", required=True, help="upstream OpenAI-compatible base URL")
    p.add_argument("--api-key", dest="api_key", default=None)
    p.add_argument("--redis", default=None, help="redis://host:port/db (default: in-process store)")
    p.add_argument("--exact-ttl", dest="exact_ttl", type=int, default=300)
    p.add_argument("--semantic-ttl", dest="semantic_ttl", type=int, default=600)
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8088)
    p.set_defaults(fn=cmd_cache_gateway)

    p = sub.add_parser("lf", help="llamafactory-cli train|export|webchat <yaml> equivalents (E10)")
    p.add_argument("action", choices=["train", "export", "webchat", "api"])
    p.add_argument("config")
    p.add_argument("overrides", nargs="*", help="key=value overrides of the YAML")
    p.add_argument("--tokenizer", default=None)
    p.set_defaults(fn=cmd_lf)

    p = sub.add_parser("cluster-check", help="per-rank inventory + broadcast / all-reduce probe (torchrun)")
    p.add_argument("--allreduce-mib", dest="allreduce_mib", type=int, default=64)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--timeout", type=int, default=300)
    p.set_defaults(fn=cmd_cluster_check)

    p = sub.add_parser("convert-alpaca")
    p.add_argument("--input", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--name", default="马哥教育AI小助手")
    p.add_argument("--author", default="马哥教育AI团队")
    p.set_defaults(fn=cmd_convert_alpaca)

    p = sub.add_parser("minibert-imdb", help="Transformer_Basics cell 34: MiniBert sentiment classifier")
    p.add_argument("--data", default=None, help="JSONL/JSON with text + label (IMDb export); synthetic if omitted")
    p.add_argument("--test", default=None)
    p.add_argument("--text-field", dest="text_field", default="text")
    p.add_argument("--label-field", dest="label_field", default="label")
    p.add_argument("--tokenizer", default="bytes", help="bytes | char | hf:<local bert-base-uncased dir>")
    p.add_argument("--hidden-size", dest="hidden_size", type=int, default=128)
    p.add_argument("--num-layers", dest="num_layers", type=int, default=2)
    p.add_argument("--max-len", dest="max_len", type=int, default=256)
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--batch-size", dest="batch_size", type=int, default=16)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--save", default=None)
    p.set_defaults(fn=cmd_minibert_imdb)

    p = sub.add_parser("nb-gpt", help="Transformer_Basics cells 39/41: notebook GPT (WikiText / Chinese GPT)")
    p.add_argument("--data", required=True, help="text file or a directory of .txt files (CLUECorpusSmall)")
    p.add_argument("--tokenizer", default="char", help="char | bytes | hf:<local gpt2 or bert-base-chinese dir>")
    p.add_argument("--n-embd", dest="n_embd", type=int, default=256)
    p.add_argument("--n-head", dest="n_head", type=int, default=8)
    p.add_argument("--n-layer", dest="n_layer", type=int, default=6)
    p.add_argument("--max-seq-len", dest="max_seq_len", type=int, default=128)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--batch-size", dest="batch_size", type=int, default=16)
    p.add_argument("--lr", type=float, default=3e-4)
    p.add_argument("--max-steps", dest="max_steps", type=int, default=-1)
    p.add_argument("--prompt", default=None)
    p.add_argument("--gen-tokens", dest="gen_tokens", type=int, default=50)
    p.add_argument("--save", default=None)
    p.set_defaults(fn=cmd_nb_gpt)

    p = sub.add_parser("seq2seq-demo", help="Transformer_Basics cells 20-22: encoder-decoder on sequence reversal")
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--vocab", type=int, default=12)
    p.add_argument("--length", type=int, default=6)
    p.add_argument("--num-layers", dest="num_layers", type=int, default=2)
    p.set_defaults(fn=cmd_seq2seq_demo)

    p = sub.add_parser("hf-classify")
    p.add_argument("--model-path", dest="model_path", help="local bert-base-uncased style dir")
    p.add_argument("--data", help="local jsonl/json/csv with text + label")
    p.add_argument("--text-field", dest="text_field", default="text")
    p.add_argument("--label-field", dest="label_field", default="label")
    p.add_argument("--num-labels", dest="num_labels", type=int, default=2)
    p.add_argument("--max-length", dest="max_length", type=int, default=256)
    p.add_argument("--eval-fraction", dest="eval_fraction", type=float, default=0.1)
    p.add_argument("--epochs", type=float, default=3)
    p.add_argument("--batch-size", dest="batch_size", type=int, default=16)
    p.add_argument("--lr", type=float, default=2e-5)
    p.add_argument("--output-dir", dest="output_dir", default="./results")
    p.set_defaults(fn=cmd_hf_classify)
    p = sub.add_parser("dl-basics", help="DL_Basics notebook demos (numpy backprop, BPTT, LeNet-5, seq2seq)")
    p.add_argument("demo", choices=["mlp", "optimizers", "rnn", "cnn", "seq2seq"])
    p.add_argument("--epochs", type=int, default=30)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--load-format", dest="load_format", default="auto", choices=["auto", "safetensors", "pt"],
                   help="vLLM flag: checkpoint files are read by their extension (safetensors first)")
    p.set_defaults(fn=cmd_dl_basics)
    p = sub.add_parser("env")
    p.set_defaults(fn=cmd_env)

    p = sub.add_parser("bench")
    p.add_argument("rest", nargs=argparse.REMAINDER)
    p.set_defaults(fn=cmd_bench)
    return ap


def main(argv=None):
    a = build_parser().parse_args(argv)
    a.fn(a)


if __name__ == "__main__":
    main()
