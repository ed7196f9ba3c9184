"""ResNet-50 image pipeline (BASELINE config 5): ImageExampleGen -> ImageTransform -> ImageTrainer -> Pusher-ready
export, on LocalDagRunner with MLMD lineage. Synthetic ImageNet-shaped data (no downloads)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.components.image import ImageExampleGen, ImageTrainer, ImageTransform  # noqa: E402
from mifx.orchestration import LocalDagRunner, Pipeline  # noqa: E402


def create_pipeline(root: str, num_images: int, image_size: int, crop: int, classes: int, steps: int, batch: int,
                    num_gpus: int = 1, checkpoint_every: int = 0, accum_steps: int = 1, name: str = "resnet_image_pipeline"):
    """num_gpus > 1: the Trainer component runs data-parallel, one rank per GPU (BASELINE config 5: DP=8);
    batch is per replica."""
    gen = ImageExampleGen(num_synthetic=num_images, image_size=image_size, num_classes=classes)
    tfm = ImageTransform(input_data=gen.outputs["examples"], crop=crop)
    trainer = ImageTrainer(examples=gen.outputs["examples"], transform_output=tfm.outputs["transform_output"],
                           train_steps=steps, batch_size=batch, num_classes=classes,
                           custom_config={"num_gpus": num_gpus, "checkpoint_every": checkpoint_every,
                                          "accum_steps": accum_steps})
    return Pipeline(name, os.path.join(root, "pipeline"), [gen, tfm, trainer], enable_cache=True,
                    metadata_db_root=os.path.join(root, "metadata.db"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/tmp/mifx_image_pipeline")
    ap.add_argument("--num-images", type=int, default=1024)
    ap.add_argument("--image-size", type=int, default=256)
    ap.add_argument("--crop", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--device", default=None)
    ap.add_argument("--num-gpus", type=int, default=1, help="data-parallel Trainer ranks (one per GPU)")
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--accum-steps", type=int, default=1)
    a = ap.parse_args(argv)
    p = create_pipeline(a.root, a.num_images, a.image_size, a.crop, a.classes, a.steps, a.batch, a.num_gpus,
                        a.checkpoint_every, a.accum_steps)
    return LocalDagRunner(device=a.device).run(p)


if __name__ == "__main__":
    print(main())
