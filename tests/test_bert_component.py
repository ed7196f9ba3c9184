"""BERT fine-tune as a pipeline Trainer component (BASELINE config 4): TextExampleGen -> BertTrainer through
LocalDagRunner with MLMD lineage; tensor parallelism (custom_config tp) launched by the component must match
TP=1 (CPU: gloo ranks)."""
import json
import os

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from mifx.components import EvalArgs, TrainArgs
from mifx.components.bert import BertTrainer, TextExampleGen, load_bert_export
from mifx.metadata.lineage import TFXArtifactTypes, TFXExecutionTypes, TFXReadonlyMetadataStore
from mifx.orchestration import LocalDagRunner, Pipeline

TINY = dict(vocab_size=1000, hidden=64, layers=2, heads=4, intermediate=128, max_position=64, dropout=0.0)


def _pipe(root, name, tp, steps=40, device="cpu", **extra):
    eg = TextExampleGen(num_synthetic=480, seq_len=32, vocab_size=1000, num_labels=2, seed=3)
    tr = BertTrainer(examples=eg.outputs.examples, train_args=TrainArgs(num_steps=steps),
                     eval_args=EvalArgs(num_steps=5),
                     custom_config=dict(TINY, tp=tp, batch_size=16, learning_rate=1e-3, graph=False, **extra))
    p = Pipeline(pipeline_name=name, pipeline_root=str(root / name), components=[eg, tr],
                 metadata_db_root=str(root / f"md_{name}"))
    res = LocalDagRunner(device=device).run(p)
    assert res.succeeded
    return res, res.components["BertTrainer"].outputs["output"][0]


def _export(model_art):
    m = json.load(open(os.path.join(model_art.uri, "metrics.json")))
    return m, load_file(os.path.join(m["export"], "variables.safetensors"))


def test_bert_trainer_component_lineage_and_export(tmp_path):
    res, art = _pipe(tmp_path, "bert1", 1, steps=60)
    m, sd = _export(art)
    assert art.custom_properties["tp"] == 1 and m["steps"] == 60
    assert m["losses"][-1] < m["losses"][0]
    md = TFXReadonlyMetadataStore.from_sqlite_db(str(tmp_path / "md_bert1" / "bert1" / "metadata.db"))
    model = md.store.get_artifacts_by_type(TFXArtifactTypes.MODEL)[0]
    ex = md.get_source_artifact_of_type(model.id, TFXArtifactTypes.EXAMPLES)
    assert ex is not None and "TextExampleGen" in ex.uri
    assert md.get_execution_for_output_artifact(model.id, TFXExecutionTypes.TRAINER) is not None
    model_t, S = load_bert_export(m["export"])
    ids = torch.randint(0, 1000, (3, S))
    assert model_t(ids, torch.zeros_like(ids), torch.ones(3, S)).shape == (3, 2)


def test_bert_trainer_component_tp2_matches_tp1(tmp_path):
    _, a1 = _pipe(tmp_path, "tp1", 1, steps=20)
    _, a2 = _pipe(tmp_path, "tp2", 2, steps=20)
    m1, s1 = _export(a1)
    m2, s2 = _export(a2)
    assert a2.custom_properties["tp"] == 2
    assert set(s1) == set(s2)
    for k in s1:
        np.testing.assert_allclose(s2[k].numpy(), s1[k].numpy(), rtol=1e-3, atol=2e-5, err_msg=k)
    np.testing.assert_allclose(m2["losses"], m1["losses"], rtol=1e-4)


def test_bert_trainer_component_tp2_sequence_parallel_matches_tp1(tmp_path):
    """custom_config sequence_parallel: the token-sharded TP=2 trainer (gloo ranks) exports the TP=1 model."""
    _, a1 = _pipe(tmp_path, "sp1", 1, steps=15)
    _, a2 = _pipe(tmp_path, "sp2", 2, steps=15, sequence_parallel=True)
    m1, s1 = _export(a1)
    m2, s2 = _export(a2)
    assert json.load(open(os.path.join(m2["export"], "config.json")))["sequence_parallel"] is True
    for k in s1:
        np.testing.assert_allclose(s2[k].numpy(), s1[k].numpy(), rtol=1e-3, atol=2e-5, err_msg=k)
    np.testing.assert_allclose(m2["losses"], m1["losses"], rtol=1e-4)


@pytest.mark.gpu
def test_bert_trainer_component_tp2_gpu_shared_rehearsal(tmp_path, monkeypatch):
    """TP=2 through the component with both ranks on cuda:0 (gloo collectives): the multi-GPU flow rehearsed on a
    1-GPU box, against TP=1 on the GPU (bf16 autocast: loose tolerance)."""
    monkeypatch.setenv("MIFX_SHARED_GPU", "1")
    monkeypatch.setenv("MIFX_DIST_BACKEND", "gloo")
    _, a1 = _pipe(tmp_path, "g1", 1, steps=20, device="cuda")
    _, a2 = _pipe(tmp_path, "g2", 2, steps=20, device="cuda")
    m1, s1 = _export(a1)
    m2, s2 = _export(a2)
    assert a2.custom_properties["tp"] == 2
    np.testing.assert_allclose(m2["losses"], m1["losses"], rtol=2e-2, atol=2e-2)
    for k in s1:  # (TP = 1 runs the fused embedding LayerNorm in bf16, TP = 2 the fp32 library one)
        np.testing.assert_allclose(s2[k].numpy(), s1[k].numpy(), rtol=5e-2, atol=1e-2, err_msg=k)
