"""Is the sequence-parallel EAGER BERT step run-to-run reproducible with W ranks sharing one GPU? Each rank trains
two identically seeded trainers (eager, peer-memory collectives) for 9 steps and reports whether their loss
trajectories and parameters are bit-identical (diagnostic for the tests/test_tp_ipc.py SP comparison)."""
import os
import socket
import sys
from pathlib import Path

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _worker(rank, world, port, sp, graph):
    from mifx.models.bert import BertConfig
    from mifx.parallel.tensor_parallel import TPGroup
    from mifx.trainer.bert_trainer import BertTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    runs = []
    for _ in range(2):
        tp = TPGroup()
        torch.manual_seed(0)
        tr = BertTrainer(BertConfig(layers=2, dropout=0.1, sequence_parallel=sp), 4, 128, dev, tp, graph=graph,
                         tp_ipc=True)
        losses = [float(tr.step()) for _ in range(9)]
        torch.cuda.synchronize(dev)
        tp.check()
        runs.append((losses, {n: p.detach().float().cpu() for n, p in tr.model.named_parameters()}))
        dist.barrier()
        tp.disable_ipc()
    (l0, p0), (l1, p1) = runs
    bad = [n for n in p0 if not torch.equal(p0[n], p1[n])]
    print(f"[sp={sp} graph={graph} rank {rank}] losses identical: {l0 == l1}; params differing: {len(bad)} "
          f"{bad[:4]}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    for sp, graph in ((True, False), (False, False), (True, True)):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.start_processes(_worker, args=(world, port, sp, graph), nprocs=world, start_method="spawn")
