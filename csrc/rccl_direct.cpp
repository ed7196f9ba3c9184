// Direct RCCL collectives for the data-parallel trainers' hot path (host-only; dlopen'ed RCCL).
//
// torch.distributed's ProcessGroupNCCL (RCCL on ROCm) wraps every collective in its own stream, events and
// work bookkeeping; for the W&D step's single 82 KB gradient bucket that wrapper, not the wire, is the cost
// (tools/dp_step_overhead.py). Here the SAME communicator (ProcessGroupNCCL._comm_ptr()) is driven directly:
// ncclAllReduce is enqueued on the caller's compute stream, in order with the step's kernels, with no extra
// stream hop. The RCCL library is the one torch already loaded (its path is passed in), so there is one RCCL
// instance in the process. All ranks must issue the same collectives in the same order on the communicator,
// interleaved identically with torch's own collectives on it (the trainers' code paths are rank-symmetric).
#include <dlfcn.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>

namespace {

typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, void*, void*);
typedef const char* (*ErrStrFn)(int);

void* g_lib = nullptr;
AllReduceFn g_allreduce = nullptr;
ErrStrFn g_errstr = nullptr;
char g_err[256] = {0};

constexpr int kNcclFloat32 = 7;  // ncclDataType_t ncclFloat32 / ncclFloat
constexpr int kNcclBfloat16 = 9;  // ncclBfloat16
constexpr int kNcclSum = 0;       // ncclRedOp_t ncclSum

}  // namespace

extern "C" {

// path: the RCCL shared library torch loaded (torch/lib/librccl.so). Returns 0 on success.
int mifx_rccl_load(const char* path) {
  if (g_allreduce != nullptr) return 0;
  g_lib = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (g_lib == nullptr) {
    std::snprintf(g_err, sizeof(g_err), "dlopen(%s) failed: %s", path, dlerror());
    return -1;
  }
  g_allreduce = (AllReduceFn)dlsym(g_lib, "ncclAllReduce");
  g_errstr = (ErrStrFn)dlsym(g_lib, "ncclGetErrorString");
  if (g_allreduce == nullptr) {
    std::snprintf(g_err, sizeof(g_err), "ncclAllReduce not found in %s", path);
    return -2;
  }
  return 0;
}

const char* mifx_rccl_last_error(void) { return g_err; }

// in-place sum all-reduce of n elements (dtype 0 fp32, 1 bf16) on `stream` over `comm` (an ncclComm_t)
int mifx_rccl_allreduce_sum(void* comm, void* buf, size_t n, int dtype, void* stream) {
  if (g_allreduce == nullptr || comm == nullptr || buf == nullptr) return -1;
  const int rc = g_allreduce(buf, buf, n, dtype ? kNcclBfloat16 : kNcclFloat32, kNcclSum, comm, stream);
  if (rc != 0 && g_errstr != nullptr) std::snprintf(g_err, sizeof(g_err), "ncclAllReduce: %s", g_errstr(rc));
  return rc;
}

}  // extern "C"
