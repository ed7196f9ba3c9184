"""Image pipeline components (BASELINE config 5: ImageNet-shaped ExampleGen -> Transform -> Trainer).

* `ImageExampleGen`: ingests `.npy` shards (uint8 [N, H, W, 3] images + int64 labels; files this
  framework or the user wrote, loaded with allow_pickle=False) or synthesises an ImageNet-shaped
  set; deterministic hash split train:eval = 2:1; writes `images.npy` / `labels.npy` per split.
* `ImageTransform`: full-pass per-channel mean / std analyzer over the training split (fp64 on the
  GPU via the HIP column-moments kernel when available) -> transform artifact (JSON), applied by the
  trainer's fused crop/flip/normalize kernel.
* `ImageTrainer`: ResNet-50 v2 on the fused input kernel, bf16 channels_last, optional
  data-parallel (RCCL) inside the component; exports a servable model (`save_module`)."""
from __future__ import annotations

import json
import os

import numpy as np

from ..orchestration import artifact as A
from ..orchestration.component import (BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec,
                                       ExecutionParameter)


class _KwComponent(BaseComponent):
    """Component whose constructor forwards keyword arguments to its spec."""

    def __init__(self, name: str | None = None, **kwargs):
        super().__init__(self.SPEC_CLASS(**kwargs), name=name)


def _split_ids(n: int, eval_buckets: int = 1, total: int = 3):
    h = (np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(61)
    is_eval = (h % np.uint64(total)) < np.uint64(eval_buckets)
    return np.nonzero(~is_eval)[0], np.nonzero(is_eval)[0]


class ImageExampleGenSpec(ComponentSpec):
    PARAMETERS = {"num_synthetic": ExecutionParameter(optional=True, default=0),
                  "image_size": ExecutionParameter(optional=True, default=256),
                  "num_classes": ExecutionParameter(optional=True, default=1000),
                  "seed": ExecutionParameter(optional=True, default=0)}
    INPUTS = {"input_base": ChannelParameter(A.EXTERNAL, optional=True)}
    OUTPUTS = {"examples": ChannelParameter(A.EXAMPLES)}


class ImageExampleGenExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        if input_dict.get("input_base"):
            base = input_dict["input_base"][0].uri
            imgs = np.load(os.path.join(base, "images.npy"), allow_pickle=False)
            labels = np.load(os.path.join(base, "labels.npy"), allow_pickle=False)
        else:
            from ..trainer.resnet_trainer import synthetic_imagenet

            t_imgs, t_labels = synthetic_imagenet(int(exec_properties["num_synthetic"]),
                                                  int(exec_properties["image_size"]),
                                                  int(exec_properties["num_classes"]), int(exec_properties["seed"]))
            imgs, labels = t_imgs.numpy(), t_labels.numpy()
        tr, ev = _split_ids(len(labels))
        for art in output_dict["examples"]:
            sel = tr if art.split == "train" else ev
            os.makedirs(art.uri, exist_ok=True)
            np.save(os.path.join(art.uri, "images.npy"), np.ascontiguousarray(imgs[sel]))
            np.save(os.path.join(art.uri, "labels.npy"), labels[sel].astype(np.int64))
            art.custom_properties["num_examples"] = int(len(sel))


class ImageExampleGen(_KwComponent):
    SPEC_CLASS = ImageExampleGenSpec
    EXECUTOR_CLASS = ImageExampleGenExecutor
    EXECUTION_TYPE = "examples_gen"
    OUTPUT_SPLITS = {"examples": ["train", "eval"]}


class ImageTransformSpec(ComponentSpec):
    INPUTS = {"input_data": ChannelParameter(A.EXAMPLES)}
    OUTPUTS = {"transform_output": ChannelParameter(A.TRANSFORM)}
    PARAMETERS = {"crop": ExecutionParameter(optional=True, default=224)}


class ImageTransformExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        train = next(a for a in input_dict["input_data"] if a.split == "train")
        imgs = np.load(os.path.join(train.uri, "images.npy"), mmap_mode="r", allow_pickle=False)
        mean, std = _channel_stats(imgs)
        out = output_dict["transform_output"][0]
        os.makedirs(out.uri, exist_ok=True)
        with open(os.path.join(out.uri, "image_transform.json"), "w") as f:
            json.dump({"mean": mean, "std": std, "crop": int(exec_properties.get("crop") or 224)}, f)


def _channel_stats(imgs: np.ndarray):
    """Per-channel mean / std of pixel/255 over the whole split (fp64; HIP moments kernel on GPU)."""
    from ..ops import analyzers

    dev = None
    try:
        import torch

        dev = "cuda" if torch.cuda.is_available() else None
    except ImportError:
        pass
    C = imgs.shape[-1]
    mean, std = [], []
    for c in range(C):
        col = np.asarray(imgs[..., c], dtype=np.float64).reshape(-1) / 255.0
        m = analyzers.column_moments(col, device=dev)
        mean.append(float(m["mean"]))
        std.append(float(m["std"]))
    return mean, std


class ImageTransform(_KwComponent):
    SPEC_CLASS = ImageTransformSpec
    EXECUTOR_CLASS = ImageTransformExecutor
    EXECUTION_TYPE = "transform"


class ImageTrainerSpec(ComponentSpec):
    INPUTS = {"examples": ChannelParameter(A.EXAMPLES), "transform_output": ChannelParameter(A.TRANSFORM)}
    OUTPUTS = {"output": ChannelParameter(A.MODEL)}
    PARAMETERS = {"train_steps": ExecutionParameter(optional=True, default=100),
                  "batch_size": ExecutionParameter(optional=True, default=64),
                  "learning_rate": ExecutionParameter(optional=True, default=0.1),
                  "num_classes": ExecutionParameter(optional=True, default=1000)}


class ImageTrainerExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        import torch

        from ..serving.saved_model import save_module
        from ..trainer.resnet_trainer import ResNetTrainer

        ex = {a.split: a.uri for a in input_dict["examples"]}
        with open(os.path.join(input_dict["transform_output"][0].uri, "image_transform.json")) as f:
            tf = json.load(f)
        imgs = torch.from_numpy(np.load(os.path.join(ex["train"], "images.npy"), allow_pickle=False))
        labels = torch.from_numpy(np.load(os.path.join(ex["train"], "labels.npy"), allow_pickle=False))
        dev = self.context.extra.get("device") or ("cuda" if torch.cuda.is_available() else "cpu")
        tr = ResNetTrainer(int(exec_properties["batch_size"]), dev, imgs, labels,
                           num_classes=int(exec_properties["num_classes"]), lr=float(exec_properties["learning_rate"]),
                           warmup_steps=max(1, int(exec_properties["train_steps"]) // 10), mean=tuple(tf["mean"]),
                           std=tuple(tf["std"]), crop=int(tf["crop"]))
        for _ in range(int(exec_properties["train_steps"])):
            loss = tr.step()
        ev_imgs = torch.from_numpy(np.load(os.path.join(ex["eval"], "images.npy"), allow_pickle=False))
        ev_labels = torch.from_numpy(np.load(os.path.join(ex["eval"], "labels.npy"), allow_pickle=False))
        acc = tr.evaluate(ev_imgs, ev_labels)
        out = output_dict["output"][0]
        save_module(os.path.join(out.uri, "serving_model_dir", "export", "1"), tr.model.cpu().float(),
                    "mifx.models.resnet:ResNetV2", {"num_classes": int(exec_properties["num_classes"])},
                    [3, tf["crop"], tf["crop"]])
        out.custom_properties.update({"eval_accuracy": acc, "final_loss": float(loss)})
        self.context.logger.info("ImageTrainer: loss %.4f eval accuracy %.4f", float(loss), acc)


class ImageTrainer(_KwComponent):
    SPEC_CLASS = ImageTrainerSpec
    EXECUTOR_CLASS = ImageTrainerExecutor
    EXECUTION_TYPE = "trainer"
