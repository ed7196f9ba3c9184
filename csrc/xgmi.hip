// Peer memory for one-shot cross-GPU exchanges over xGMI (host side).
//
// One process per GPU: each rank allocates its exchange buffers here, exports them as IPC handles (64-byte
// opaque blobs the Python side all-gathers over torch.distributed), and opens the peers' handles, which maps
// their HBM into this process so kernels can load from it directly over xGMI. Flag arrays are allocated
// uncached (hipDeviceMallocUncached) so the epoch flags peers store into them are seen by spinning waves
// without cache maintenance. Used by the W&D data-parallel step (csrc/wide_deep.hip wd_reduce_xgmi_opt,
// mifx/parallel/xgmi.py).
#include <hip/hip_runtime.h>
#include <string.h>

extern "C" {

int mifx_xgmi_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// zero-filled device allocation; uncached != 0: fine-grained uncached memory (flags)
int mifx_xgmi_malloc(size_t bytes, int uncached, void** out) {
  *out = nullptr;
  hipError_t e = uncached ? hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached) : hipMalloc(out, bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}

int mifx_xgmi_free(void* p) { return (int)hipFree(p); }

int mifx_xgmi_export(void* p, void* handle_out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e == hipSuccess) memcpy(handle_out, &h, sizeof(h));
  return (int)e;
}

int mifx_xgmi_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  *out = nullptr;
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int mifx_xgmi_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

}  // extern "C"
