"""Which aten ops (outside the hand-written kernels) an eager BERT-base B=32 S=128 step launches: one profiled step
after warmup, torch.profiler; prints each aten op's count with its input shapes and its CUDA time, largest first."""
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mifx.models.bert import BertConfig  # noqa: E402
from mifx.parallel.tensor_parallel import TPGroup  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer, load_gemm_table  # noqa: E402


def main():
    dev = torch.device("cuda")
    load_gemm_table()
    tr = BertTrainer(BertConfig(layers=12, dropout=0.1), 32, 128, dev, TPGroup(None), graph=False)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                                record_shapes=True) as prof:
        tr.step()
        torch.cuda.synchronize()
    rows = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.key_averages(group_by_input_shape=True):
        if ev.key.startswith("aten::") and ev.device_time_total > 0:
            r = rows[(ev.key, str(ev.input_shapes)[:120])]
            r[0] += ev.count
            r[1] += ev.self_device_time_total
    for (k, shp), (n, us) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{us:9.1f} us  {n:4d}x  {k:32s} {shp}")


if __name__ == "__main__":
    main()
