"""Graph-capturable tensor-parallel all-reduce over xGMI peer memory (csrc/tp_allreduce.hip).

Every rank of the TP group allocates three IPC-exportable buffers -- its partial-sum buffer and its reduced-slice
buffer ([2][npad] bf16 each, double-buffered by epoch parity) and an uncached flag array -- and opens its peers'
(handles all-gathered over the process group once, as mifx.parallel.xgmi does for the W&D gradient). An all-reduce
is then three kernels on the current stream (publish, reduce-scatter, all-gather) synchronised by device-side
epoch flags: no host collective, so a TP step captures into a hipGraph like a single-GPU step, and the result lands
in a fresh tensor (no defensive `.clone()` of the input). The reduction is a rank-order fp32 sum rounded once to
bf16: every rank gets the same bits. A peer that never arrives sets a sticky error flag after a bounded wait;
`check()` raises. Used by mifx.parallel.tensor_parallel when `TPGroup.enable_ipc()` was called, and -- with
dtype=torch.float32 (rank-order fp32 sum, scaled once by the average) -- by mifx.parallel.ddp's exchange="ipc" for
data-parallel gradient buckets inside the captured backward."""
from __future__ import annotations

import ctypes
import functools

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops._lib import F32, I32, I64, VP, check, ptr, sig, stream_handle
from .xgmi import MAX_WORLD, _fns as _xg_fns


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("tp_allreduce")
    return {"chunk": sig(lib, "mifx_tpar_chunk", []),
            "ar": sig(lib, "mifx_tpar_allreduce", [VP, VP, I64, VP, VP, VP, I32, I32, I64, VP, VP, VP, VP]),
            "ar32": sig(lib, "mifx_tpar_allreduce_f32", [VP, VP, I64, VP, VP, VP, I32, I32, I64, VP, VP, VP, F32, VP]),
            "ar2": sig(lib, "mifx_tpar_allreduce2", [VP, VP, I64, VP, VP, VP, I32, I32, I64, VP, VP, VP, I32, F32, I32,
                                                    VP]),
            "rs": sig(lib, "mifx_tpar_reduce_scatter", [VP, VP, I64, VP, VP, I32, I32, I64, VP, VP, VP, I32, VP]),
            "ag": sig(lib, "mifx_tpar_all_gather", [VP, VP, I64, VP, VP, I32, I32, I64, VP, VP, VP, I32, VP])}


def _device_key(device) -> str:
    """Identity of the physical GPU behind `device`, comparable across processes."""
    props = torch.cuda.get_device_properties(device)
    u = getattr(props, "uuid", None)
    return str(u) if u is not None else f"{getattr(props, 'pci_bus_id', '?')}:{getattr(props, 'pci_device_id', '?')}"


class IpcAllReduce:
    """All-reduce (sum) of bf16 (or fp32) tensors of up to `max_elems` elements over the ranks of `pg`, one GPU each
    (or ranks sharing one GPU in rehearsals: the IPC path is the same)."""

    def __init__(self, pg, device, max_elems: int, dtype: torch.dtype = torch.bfloat16, waiters: bool | None = None):
        """waiters: split waits (csrc/tp_allreduce.hip header) -- no data-moving workgroup spins, a one-wave kernel
        waits between them. Needed whenever the exchange can run concurrently with a kernel that needs whole CUs: the
        data-parallel exchange on a side stream next to the backward (pass True), or ranks sharing one GPU (rehearsals).
        None: split when any two ranks of the group share a device, else the three-kernel form (tensor parallelism on
        the compute stream, one GPU per rank: nothing runs beside it)."""
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("IPC all-reduce: bf16 or fp32")
        self.dtype = dtype
        if dtype == torch.float32:
            max_elems = 2 * int(max_elems)  # the buffers are sized in bf16-element units
        self.pg, self.device = pg, torch.device(device)
        self.rank, self.world = dist.get_rank(pg), dist.get_world_size(pg)
        if not 1 <= self.world <= MAX_WORLD:
            raise ValueError(f"IPC all-reduce supports 1..{MAX_WORLD} ranks")
        chunk = _fns()["chunk"]()
        self.chunk = int(chunk)
        self.npad = -(-int(max_elems) // chunk) * chunk
        self.nchunks = self.npad // chunk
        xf = _xg_fns()
        self._own, self._opened = [], []
        mine, err = None, ""
        bufs = [VP(), VP(), VP()]
        try:
            with torch.cuda.device(self.device):
                sizes = (2 * self.npad * 2, 2 * self.npad * 2, 2 * self.nchunks * MAX_WORLD * 4)
                for b, nbytes, unc in zip(bufs, sizes, (0, 0, 1)):
                    check(xf["malloc"](nbytes, unc, ctypes.byref(b)), "tp ipc malloc")
                    self._own.append(b)
                hs = xf["hsize"]()
                hdl = []
                for b in bufs:
                    h = (ctypes.c_char * hs)()
                    check(xf["export"](b, h), "hipIpcGetMemHandle")
                    hdl.append(bytes(h))
                mine = tuple(hdl)
        except Exception as e:  # noqa: BLE001 -- agreed on below
            err = f"rank {self.rank}: {e}"
        try:
            dkey = _device_key(self.device)
        except Exception:  # noqa: BLE001 -- unknown identity: treat as its own device
            dkey = f"rank{self.rank}"
        handles = [None] * self.world
        dist.all_gather_object(handles, (mine, err, dkey), group=pg)
        self._agree([h[1] for h in handles])
        self.shared_device = len({h[2] for h in handles}) < self.world
        self.waiters = bool(self.shared_device if waiters is None else waiters)
        handles = [(h[0], h[1]) for h in handles]
        cols = [[], [], []]
        try:
            with torch.cuda.device(self.device):
                for p, (hs_, _) in enumerate(handles):
                    for k in range(3):
                        if p == self.rank:
                            cols[k].append(bufs[k].value)
                            continue
                        q = VP()
                        check(xf["open"](hs_[k], ctypes.byref(q)), f"hipIpcOpenMemHandle (rank {p})")
                        self._opened.append(q)
                        cols[k].append(q.value)
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=pg)
        self._agree(errs)
        self.bufs, self.reds, self.flags = ((VP * self.world)(*c) for c in cols)
        self.ep = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.done = torch.zeros(3, dtype=torch.int32, device=self.device)  # gather / publish / reduce arrivals
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        dist.barrier(group=pg)  # every rank's buffers exist (zeroed) before any flag can be stored

    def _agree(self, errs) -> None:
        bad = [e for e in errs if e]
        if bad:
            self.close()
            raise RuntimeError("TP IPC all-reduce setup failed: " + "; ".join(bad))

    def close(self) -> None:
        xf = _xg_fns()
        for p in self._opened:
            xf["close"](p)
        self._opened = []
        for p in self._own:
            xf["free"](p)
        self._own = []

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None, scale: float = 1.0) -> torch.Tensor:
        """Sum of `x` over the ranks (the group's dtype, any shape; bf16: numel % 4 == 0, fp32: even numel; <=
        max_elems) into `out` (default: a new tensor; `out=x` reduces in place), times `scale` (fp32 only).
        Stream-ordered and graph-capturable."""
        if x.dtype != self.dtype or x.device != self.device:
            raise ValueError(f"IPC all-reduce takes {self.dtype} tensors on the group's device")
        x = x.contiguous()
        n = x.numel()
        y = torch.empty_like(x) if out is None else out
        f32 = self.dtype == torch.float32
        if f32:
            if n % 2 or 2 * n > self.npad:
                raise ValueError(f"{n} fp32 elements: need an even count <= {self.npad // 2}")
        else:
            if scale != 1.0:
                raise ValueError("scale is for the fp32 path")
            if n % 4 or n > self.npad:
                raise ValueError(f"{n} elements: need a multiple of 4 and <= {self.npad}")
        check(_fns()["ar2"](ptr(x), ptr(y), n, self.bufs, self.reds, self.flags, self.world, self.rank, self.npad,
                            ptr(self.ep), ptr(self.done), ptr(self.err), int(f32), float(scale), int(self.waiters),
                            stream_handle(self.device)), "mifx_tpar_allreduce2")
        return y

    # ---- sequence parallelism: token-major [T, H] bf16 activations, rank r owns tokens [r T / W, (r + 1) T / W)
    def shard_ok(self, n: int) -> bool:
        """n elements split into `world` contiguous shards of whole chunks (the reduce-scatter / all-gather layout)."""
        return self.dtype == torch.bfloat16 and n % (self.world * self.chunk) == 0 and n <= self.npad

    def reduce_scatter(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """This rank's shard (the n / world elements starting at rank * n / world, flattened) of the rank-order sum
        of the ranks' bf16 x, rounded once to bf16. Stream-ordered, graph-capturable."""
        x = x.contiguous()
        n = x.numel()
        if x.dtype != torch.bfloat16 or not self.shard_ok(n):
            raise ValueError(f"reduce_scatter: bf16 with numel % (world x {self.chunk}) == 0 and <= {self.npad}")
        y = torch.empty(n // self.world, dtype=x.dtype, device=x.device) if out is None else out
        check(_fns()["rs"](ptr(x), ptr(y), n, self.bufs, self.flags, self.world, self.rank, self.npad, ptr(self.ep),
                           ptr(self.done), ptr(self.err), int(self.waiters), stream_handle(self.device)),
              "mifx_tpar_reduce_scatter")
        return y

    def all_gather(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """The ranks' shards concatenated in rank order (flattened, world x numel(x) elements)."""
        x = x.contiguous()
        n = x.numel() * self.world
        if x.dtype != torch.bfloat16 or not self.shard_ok(n):
            raise ValueError(f"all_gather: bf16 shards of whole chunks, total <= {self.npad}")
        y = torch.empty(n, dtype=x.dtype, device=x.device) if out is None else out
        check(_fns()["ag"](ptr(x), ptr(y), n, self.bufs, self.flags, self.world, self.rank, self.npad, ptr(self.ep),
                           ptr(self.done), ptr(self.err), int(self.waiters), stream_handle(self.device)),
              "mifx_tpar_all_gather")
        return y

    def check(self) -> None:
        if int(self.err.item()) != 0:
            raise RuntimeError("TP IPC all-reduce: a peer never published (wait timed out); results since are invalid")
