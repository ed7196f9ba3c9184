#!/bin/bash
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/prof_run.sh bert 600 -- python3 -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 5 --warmup 2 &&
bash tools/prof_run.sh resnet 600 -- python3 -m mifx.trainer.resnet_trainer --batch 256 --images 1024 --steps 5 --warmup 2
