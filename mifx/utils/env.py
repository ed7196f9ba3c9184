"""Environment report (reference `notebooks/00_Explore_Environment.ipynb`: framework/Python versions
and the accelerator resolver): Python, torch, HIP/ROCm, RCCL, gfx architecture, CU count, HBM size
per device, the mifx native libraries that are built, and the torchrun-style rank variables.

    python -m mifx.utils.env [--json]"""
import json
import os
import platform
import sys


def report() -> dict:
    import torch

    out = {"python": sys.version.split()[0], "platform": platform.platform(), "torch": torch.__version__,
           "hip": getattr(torch.version, "hip", None), "gpus": []}
    try:
        out["rccl"] = ".".join(map(str, torch.cuda.nccl.version())) if torch.cuda.is_available() else None
    except Exception:  # noqa: BLE001 - RCCL query unsupported in this build
        out["rccl"] = None
    if torch.cuda.is_available():
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            out["gpus"].append({"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", ""),
                                "compute_units": p.multi_processor_count,
                                "hbm_gib": round(p.total_memory / 2 ** 30, 1)})
    from ..ops.build import LIBDIR

    out["native_libs"] = sorted(f for f in os.listdir(LIBDIR) if f.endswith(".so")) if os.path.isdir(LIBDIR) else []
    out["dist_env"] = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                       "MASTER_PORT") if os.environ.get(k)}
    return out


def main(argv=None) -> dict:
    argv = sys.argv[1:] if argv is None else argv
    r = report()
    if "--json" in argv:
        print(json.dumps(r))
    else:
        for k, v in r.items():
            if k == "gpus":
                for g in v:
                    print(f"gpu {g['index']}: {g['name']} {g['arch']} {g['compute_units']} CUs {g['hbm_gib']} GiB")
                if not v:
                    print("gpus: none visible")
            else:
                print(f"{k}: {v}")
    return r


if __name__ == "__main__":
    main()
