"""BERT-base fine-tune step benchmark entry (mifx.trainer.bert_trainer's CLI as a script, for rocprofv3 runs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.trainer import bert_trainer  # noqa: E402

if __name__ == "__main__":
    raise SystemExit(bert_trainer.main())
