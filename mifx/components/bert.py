"""BERT fine-tune pipeline components (BASELINE config 4: "BERT-base fine-tune Trainer component, TP=8").

* `TextExampleGen`: tokenised sequence-classification examples -> Examples artifact (train / eval splits of
  `input_ids` int32 [N, S], `token_type_ids` / `attention_mask` int8 [N, S], `labels` int64 [N], npy files).
  Input: a JSONL file of {"input_ids": [...], "label": k} (ids already tokenised: there is no network for a
  vocabulary) or a synthetic GLUE-shaped set whose label is a learnable function of the tokens.
* `BertTrainer`: fine-tunes `mifx.models.bert.BertForSequenceClassification` (bf16 autocast, fp32 master AdamW,
  fused HIP LayerNorm / GELU / attention kernels, whole step in one hipGraph at TP=1) on the examples and
  exports the TP=1 state as a ModelExportPath artifact. `custom_config={"tp": N}` runs Megatron-style tensor
  parallelism over N ranks (one per GPU, RCCL over xGMI; gloo processes on a CPU host; `"sequence_parallel": true`:
  token-sharded LayerNorms / dropouts between the TP regions) launched by the component itself
  (mifx.trainer.distributed); rank 0 gathers the full state and exports.

Contract mirrored from the TFX Trainer of the reference (`airflow-dags/taxi_pipeline.py:92-99`: examples in,
ModelExportPath out, lineage in MLMD; train_args / eval_args num_steps)."""
from __future__ import annotations

import json
import os
import time

import numpy as np

from ..orchestration import artifact as A
from ..orchestration.component import BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec, ExecutionParameter
from . import proto

_ARRAYS = ("input_ids", "token_type_ids", "attention_mask", "labels")


class _KwComponent(BaseComponent):
    def __init__(self, name: str | None = None, **kwargs):
        super().__init__(self.SPEC_CLASS(**kwargs), name=name)


def synthetic_text_examples(n: int, seq_len: int, vocab_size: int, num_labels: int = 2, seed: int = 0) -> dict:
    """GLUE-shaped pairs: [CLS] a [SEP] b [SEP] with random lengths and padding; label = bucket of the first
    token of segment a (a function the model can learn)."""
    rng = np.random.default_rng(seed)
    ids = np.zeros((n, seq_len), np.int32)
    tt = np.zeros((n, seq_len), np.int8)
    am = np.zeros((n, seq_len), np.int8)
    lab = np.zeros(n, np.int64)
    lo = min(1000, vocab_size // 4)
    for i in range(n):
        L = int(rng.integers(seq_len // 2, seq_len + 1))
        a = max(2, (L - 3) // 2)
        b = max(1, L - 3 - a)
        toks = rng.integers(lo, vocab_size, size=a + b)
        seq = [101] + list(toks[:a]) + [102] + list(toks[a:]) + [102]
        seq = seq[:seq_len]
        ids[i, :len(seq)] = seq
        tt[i, a + 2:len(seq)] = 1
        am[i, :len(seq)] = 1
        lab[i] = int((toks[0] - lo) * num_labels // (vocab_size - lo))
    return {"input_ids": ids, "token_type_ids": tt, "attention_mask": am, "labels": lab}


def _split(n: int):
    h = (np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(61)
    ev = (h % np.uint64(3)) == 0
    return np.nonzero(~ev)[0], np.nonzero(ev)[0]


def _read_jsonl(path: str, seq_len: int) -> dict:
    rows = [json.loads(line) for line in open(path) if line.strip()]
    n = len(rows)
    out = {"input_ids": np.zeros((n, seq_len), np.int32), "token_type_ids": np.zeros((n, seq_len), np.int8),
           "attention_mask": np.zeros((n, seq_len), np.int8), "labels": np.zeros(n, np.int64)}
    for i, r in enumerate(rows):
        ids = list(r["input_ids"])[:seq_len]
        out["input_ids"][i, :len(ids)] = ids
        tt = list(r.get("token_type_ids", [0] * len(ids)))[:seq_len]
        out["token_type_ids"][i, :len(tt)] = tt
        out["attention_mask"][i, :len(ids)] = 1
        out["labels"][i] = int(r["label"])
    return out


def load_split(uri: str) -> dict:
    return {k: np.load(os.path.join(uri, f"{k}.npy"), allow_pickle=False) for k in _ARRAYS}


# ------------------------------------------------------------------------------------------ TextExampleGen
class TextExampleGenSpec(ComponentSpec):
    PARAMETERS = {"num_synthetic": ExecutionParameter(optional=True, default=0),
                  "seq_len": ExecutionParameter(optional=True, default=128),
                  "vocab_size": ExecutionParameter(optional=True, default=30522),
                  "num_labels": ExecutionParameter(optional=True, default=2),
                  "seed": ExecutionParameter(optional=True, default=0)}
    INPUTS = {"input_base": ChannelParameter(A.EXTERNAL, optional=True)}
    OUTPUTS = {"examples": ChannelParameter(A.EXAMPLES)}


class TextExampleGenExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        S = int(exec_properties["seq_len"])
        if input_dict.get("input_base"):
            base = input_dict["input_base"][0].uri
            files = sorted(f for f in os.listdir(base) if f.endswith(".jsonl"))
            parts = [_read_jsonl(os.path.join(base, f), S) for f in files]
            data = {k: np.concatenate([p[k] for p in parts]) for k in _ARRAYS}
        else:
            data = synthetic_text_examples(int(exec_properties["num_synthetic"]), S,
                                           int(exec_properties["vocab_size"]), int(exec_properties["num_labels"]),
                                           int(exec_properties["seed"]))
        tr, ev = _split(len(data["labels"]))
        for art in output_dict["examples"]:
            sel = tr if art.split == "train" else ev
            os.makedirs(art.uri, exist_ok=True)
            for k in _ARRAYS:
                np.save(os.path.join(art.uri, f"{k}.npy"), np.ascontiguousarray(data[k][sel]))
            art.custom_properties["num_examples"] = int(len(sel))
            art.custom_properties["seq_len"] = S


class TextExampleGen(_KwComponent):
    SPEC_CLASS = TextExampleGenSpec
    EXECUTOR_CLASS = TextExampleGenExecutor
    EXECUTION_TYPE = "examples_gen"
    OUTPUT_SPLITS = {"examples": ["train", "eval"]}


# ------------------------------------------------------------------------------------------ BertTrainer
_CFG_KEYS = ("vocab_size", "hidden", "layers", "heads", "intermediate", "max_position", "dropout", "num_labels",
             "sequence_parallel")


def run_bert_rank(spec: dict) -> dict:
    """One rank (or the only process) of a BertTrainer run: train, evaluate, rank 0 exports the TP=1 state."""
    import torch
    import torch.distributed as dist
    from safetensors.torch import save_file

    from ..models.bert import BertConfig, gather_full_state
    from ..parallel.tensor_parallel import TPGroup
    from ..trainer.bert_trainer import BertTrainer, load_gemm_table

    cc = spec["custom_config"]
    dev_s = spec.get("device")
    if dev_s in (None, "cuda") and torch.cuda.is_available():
        shared = os.environ.get("MIFX_SHARED_GPU") == "1"
        dev = torch.device("cuda", 0 if shared else int(os.environ.get("LOCAL_RANK", 0)))
        torch.cuda.set_device(dev)
        if cc.get("gemm_table", True):
            load_gemm_table()
    else:
        dev = torch.device(dev_s or "cpu")
    tp = TPGroup(dist.group.WORLD if dist.is_initialized() and dist.get_world_size() > 1 else None)
    cfg = BertConfig(**{k: cc[k] for k in _CFG_KEYS if k in cc})
    tr_data, ev_data = load_split(spec["train_uri"]), load_split(spec["eval_uri"])
    B = int(cc.get("batch_size", 32))
    S = tr_data["input_ids"].shape[1]
    torch.manual_seed(int(cc.get("seed", 0)))
    tr = BertTrainer(cfg, B, S, dev, tp, lr=float(cc.get("learning_rate", 2e-5)),
                     graph=cc.get("graph"))
    T = {k: torch.from_numpy(v.astype(np.int64) if k != "attention_mask" else v.astype(np.float32))
         for k, v in tr_data.items()}
    n = len(T["labels"])
    steps = int(spec["train_steps"])
    losses = []
    t0 = time.time()
    for i in range(steps):
        idx = (torch.arange(B) + i * B) % n
        tr.set_batch(T["input_ids"][idx], T["token_type_ids"][idx], T["attention_mask"][idx], T["labels"][idx])
        loss = tr.step()
        if i % max(1, steps // 20) == 0 or i == steps - 1:
            losses.append(float(loss))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    secs = time.time() - t0
    E = {k: torch.from_numpy(v.astype(np.int64) if k != "attention_mask" else v.astype(np.float32))
         for k, v in ev_data.items()}
    ne = len(E["labels"]) if not spec.get("eval_steps") else min(len(E["labels"]), int(spec["eval_steps"]) * B)
    correct = 0
    for s0 in range(0, ne, B):
        sl = slice(s0, min(ne, s0 + B))
        logits = tr.predict(E["input_ids"][sl], E["token_type_ids"][sl], E["attention_mask"][sl])
        correct += int((logits.argmax(-1).cpu() == E["labels"][sl]).sum())
    full = gather_full_state(tr.model)  # collective
    res = {"eval": {"accuracy": correct / max(1, ne), "num_eval_examples": ne}, "losses": losses,
           "train_sequences_per_sec": steps * B / max(secs, 1e-9), "tp": tp.size, "steps": steps}
    if tp.rank == 0:
        exp = os.path.join(spec["out_dir"], "serving_model_dir", "export", "bert", str(int(time.time() * 1000)))
        os.makedirs(exp, exist_ok=True)
        save_file({k: v.detach().float().cpu().contiguous() for k, v in full.items()},
                  os.path.join(exp, "variables.safetensors"))
        with open(os.path.join(exp, "config.json"), "w") as f:
            json.dump({k: getattr(cfg, k) for k in _CFG_KEYS} | {"seq_len": S, "model": "bert_seq_cls"}, f)
        res["export"] = exp
    return res


class BertTrainerSpec(ComponentSpec):
    PARAMETERS = {"train_args": ExecutionParameter(), "eval_args": ExecutionParameter(),
                  "custom_config": ExecutionParameter(optional=True)}
    INPUTS = {"examples": ChannelParameter(A.EXAMPLES), "schema": ChannelParameter(A.SCHEMA, optional=True)}
    OUTPUTS = {"output": ChannelParameter(A.MODEL)}


class BertTrainerExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        ex = {a.split: a.uri for a in input_dict["examples"]}
        out = output_dict["output"][0]
        targs = proto.from_dict(proto.TrainArgs, exec_properties["train_args"])
        eargs = proto.from_dict(proto.EvalArgs, exec_properties["eval_args"])
        cc = dict(exec_properties.get("custom_config") or {})
        spec = {"train_uri": ex["train"], "eval_uri": ex.get("eval", ex["train"]), "out_dir": out.uri,
                "train_steps": int(targs.num_steps), "eval_steps": int(eargs.num_steps or 0), "custom_config": cc,
                "device": self.context.device, "hparams": {"device": self.context.device}}
        n = int(cc.get("tp", 1) or 1)
        if n > 1:
            from ..trainer import distributed

            work = os.path.join(out.uri, "tp_run")
            res = distributed.launch(dict(spec, target="mifx.components.bert:run_bert_rank", work_dir=work), n, work,
                                     timeout=cc.get("timeout_s"))
        else:
            res = run_bert_rank(spec)
        with open(os.path.join(out.uri, "metrics.json"), "w") as f:
            json.dump(res, f, default=float)
        out.custom_properties.update(eval_accuracy=float(res["eval"]["accuracy"]), tp=int(res["tp"]),
                                     train_steps=int(targs.num_steps),
                                     train_sequences_per_sec=float(res["train_sequences_per_sec"]))


class BertTrainer(BaseComponent):
    SPEC_CLASS = BertTrainerSpec
    EXECUTOR_CLASS = BertTrainerExecutor
    EXECUTION_TYPE = "trainer"

    def __init__(self, examples, train_args, eval_args, schema=None, custom_config: dict | None = None,
                 name: str | None = None, output=None):
        super().__init__(BertTrainerSpec(examples=examples, schema=schema,
                                         train_args=train_args.to_dict() if hasattr(train_args, "to_dict")
                                         else train_args,
                                         eval_args=eval_args.to_dict() if hasattr(eval_args, "to_dict") else eval_args,
                                         custom_config=custom_config, output=output), name=name)


def load_bert_export(path: str, device="cpu"):
    """Export dir -> (BertForSequenceClassification at TP=1, seq_len)."""
    from safetensors.torch import load_file

    from ..models.bert import BertConfig, BertForSequenceClassification

    with open(os.path.join(path, "config.json")) as f:
        c = json.load(f)
    cfg = BertConfig(**{k: c[k] for k in _CFG_KEYS if k in c})
    m = BertForSequenceClassification(cfg, None, seed=None)
    m.load_full(load_file(os.path.join(path, "variables.safetensors")))
    return m.to(device).eval(), int(c["seq_len"])
