"""`kfp`-style command line: `python -m mifx.kfp [--endpoint E] run {list,submit,get}`."""
